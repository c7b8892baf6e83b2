"""Per-frame phases of the quad trigram recursions (dev tool, GPU; needs
`make stamps`): quad 0 (utterance 0's alpha) and quad B (its beta), every
member's waves: [poll start, inputs taken, after the barrier, step end],
medians over the frames in s_memtime ticks."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

nat.LIB_PATH = os.path.join(ROOT, 'build', 'liblt_lattice_stamps.so')  # copied out of build/stamps
W8 = 13
NAMES = ['st%d' % w for w in range(8)] + ['aux', 'ld0', 'ld1', 'num', 'wr']


def main():
  B, T, U, V, n = 32, 1000, 100, 32, 2
  C = nat.num_context_states(V, n)
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  st = torch.zeros(4 * W8 * T * 4, dtype=torch.int64, device='cuda')
  os.environ['LT_T4_STAMPS'] = str(st.data_ptr())
  fn = lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
  fn()
  torch.cuda.synchronize()
  st.zero_()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  fn()
  e1.record()
  torch.cuda.synchronize()
  print(f'loss_forward {e0.elapsed_time(e1):.3f} ms (stamped build; quad 0 = alpha of utterance 0)')
  s = st.cpu().numpy().reshape(4, W8, T, 4).astype(np.int64)
  for k in range(4):
    for w in range(W8):
      x = s[k, w]
      ok = (x[:, 0] > 0) & (x[:, 3] > 0)
      if ok.sum() < 20:
        continue
      x = x[ok][5:-5]
      per = np.median(np.diff(x[:, 0]))
      ph = [np.median(x[:, j + 1] - x[:, j]) for j in range(3)]
      print(f'  member {k} {NAMES[w]}: period {per:6.0f}  poll {ph[0]:6.0f}  barrier {ph[1]:6.0f}'
            f'  compute {ph[2]:6.0f}', flush=True)


if __name__ == '__main__':
  main()
