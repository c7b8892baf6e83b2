"""Per-wave cycle breakdown of the pipelined recursions (dev tool, GPU; needs
`make stamps`). For one workgroup (LT_STAMP_BLOCK, default 0 = alpha of
utterance 0) every wave's lane 0 records s_memtime at the start of a step,
after its wait (tag / slot-free) and at the end. Reports medians over steps."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

nat.LIB_PATH = os.path.join(ROOT, 'build', 'stamps', 'liblt_lattice_stamps.so')
NW = 8


def report(st, T):
  st = st.reshape(NW, T, 4).astype(np.int64)
  names = ['den', 'num'] + [f'helper{k}' for k in range(NW - 2)]
  for w in range(NW):
    s = st[w]
    idx = np.nonzero(s[:, 0])[0]
    if len(idx) < 20:
      continue
    idx = idx[5:-5]
    s = s[idx]
    wait = s[:, 1] - s[:, 0]
    work = s[:, 2] - s[:, 1]
    step = np.diff(s[:, 0])
    print(f'  {names[w]:8s} steps {len(idx):4d}  period {np.median(step):7.0f}  wait {np.median(wait):6.0f}'
          f' (p90 {np.percentile(wait, 90):6.0f})  work {np.median(work):6.0f}'
          f' (p90 {np.percentile(work, 90):6.0f})', flush=True)


def main():
  B = int(os.environ.get('B', 64))
  T, U, V, n = 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn(B, T, C, V + 1, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  st = torch.zeros(NW * T * 4, dtype=torch.int64, device='cuda')
  os.environ['LT_STAMPS_PTR'] = str(st.data_ptr())
  for blk in os.environ.get('BLOCKS', f'0,{B}').split(','):
    os.environ['LT_STAMP_BLOCK'] = blk
    fn = lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
    fn()
    st.zero_()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    print(f'== block {blk}: {e0.elapsed_time(e1):.3f} ms (stamped build)')
    report(st.cpu().numpy(), T)


if __name__ == '__main__':
  main()
