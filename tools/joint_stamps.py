"""Per-wave cycle breakdown of the fused joint loss's forward recursions (dev
tool, GPU; needs `make stamps`). Workgroup LT_STAMP_BLOCK of pipe_kernel's
producer mode: den / num waves record (start, after wait, end); producer
helpers record (start, after ring + slot waits, after the W tiles, end).
Reports medians over steps in s_memtime ticks."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402
from tools.joint_fused_bench import inputs  # noqa: E402

nat.LIB_PATH = os.path.join(ROOT, 'build', 'liblt_lattice_stamps.so')  # copied out of build/stamps (gpurun-ignored)
NW = 8


def report(st, T):
  st = st.reshape(NW, T, 4).astype(np.int64)
  names = ['den', 'num'] + [f'helper{k}' for k in range(NW - 2)]
  for w in range(NW):
    s = st[w]
    idx = np.nonzero(s[:, 0])[0]
    if len(idx) < 20:
      continue
    s = s[idx[5:-5]]
    step = np.median(np.diff(s[:, 0]))
    parts = [np.median(s[:, k + 1] - s[:, k]) if (s[:, k + 1] > 0).all() else float('nan')
             for k in range(3)]
    print(f'  {names[w]:8s} steps {len(s):4d} period {step:7.0f}  phases ' +
          ' '.join(f'{p:7.0f}' for p in parts), flush=True)


def report_marg(st, nblk):
  """jf_marg_kernel: per-block stamps [start, staged, loop end, end, wave 0's
  W tile / marginals / barrier / backward cycles summed over the state tiles]."""
  st = st.reshape(-1, 8).astype(np.int64)
  live = st[:, 3] > 0
  s = st[live]
  dur = s[:, 3] - s[:, 0]
  span = s[:, 3].max() - s[s[:, 0] > 0, 0].min()
  print(f'  jf_marg blocks {len(s)} span {span} busy-sum/span {dur.sum() / span:.1f} (blocks in flight)')
  for name, v in (('block', dur), ('staging', s[:, 1] - s[:, 0]), ('tiles', s[:, 2] - s[:, 1]),
                  ('outputs', s[:, 3] - s[:, 2]), ('w0 W tile', s[:, 4]), ('w0 margs', s[:, 5]),
                  ('w0 barrier', s[:, 6]), ('w0 bwd', s[:, 7])):
    print(f'    {name:10s} median {np.median(v):9.0f} p10 {np.percentile(v, 10):9.0f}'
          f' p90 {np.percentile(v, 90):9.0f}', flush=True)


def main():
  B, T, U, V = int(os.environ.get('B', 64)), 1000, 100, 32
  for H in (32, 128):
    pc, pf, wo, bias, nf, lab, nl = inputs(B, T, U, H, V, 'cuda')
    st = torch.zeros(NW * T * 4, dtype=torch.int64, device='cuda')
    os.environ['LT_STAMPS_PTR'] = str(st.data_ptr())
    for blk in os.environ.get('BLOCKS', '0').split(','):
      os.environ['LT_STAMP_BLOCK'] = blk
      fn = lambda: nat.joint_loss_forward(pc, pf, wo, bias, nf, lab, nl)
      fn()
      torch.cuda.synchronize()
      st.zero_()
      e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
      e0.record()
      fn()
      e1.record()
      torch.cuda.synchronize()
      print(f'== H {H} block {blk}: {e0.elapsed_time(e1):.3f} ms (stamped build)')
      report(st.cpu().numpy(), T)
    loss, lz, num, state = nat.joint_loss_forward(pc, pf, wo, bias, nf, lab, nl)
    nblk = (T + 31) // 32
    js = torch.zeros(B * nblk * 8, dtype=torch.int64, device='cuda')
    os.environ['LT_JSTAMPS_PTR'] = str(js.data_ptr())
    nat.joint_loss_backward(pc, pf, wo, bias, nf, lab, state)
    torch.cuda.synchronize()
    js.zero_()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    nat.joint_loss_backward(pc, pf, wo, bias, nf, lab, state)
    e1.record()
    torch.cuda.synchronize()
    print(f'== H {H} backward {e0.elapsed_time(e1):.3f} ms (stamped build)')
    report_marg(js.cpu().numpy(), nblk)
    del os.environ['LT_JSTAMPS_PTR']


if __name__ == '__main__':
  main()
