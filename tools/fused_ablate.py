"""Dev tool (GPU): marginal roles of the fused loss+grad alone (LT_PIPE_DBG
128: the recursion roles publish at once), with parts switched off; prints
the kernel time and the per-tile work time. Results are garbage here."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402
from fused_check import timeit  # noqa: E402


def main():
  B, T, U, V, n = 64, 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([1 << 30], dtype=torch.uint8, device='cuda')
  FT = int(os.environ.get('LT_FUSED_FW', 4)) * 6
  NB = (T + FT - 1) // FT
  tr = torch.zeros([4 * B + 4 * NB * B], dtype=torch.int64, device='cuda')
  for dbg in [128, 128 | 256, 128 | 1024, 128 | 2048, 128 | 4096, 128 | 1024 | 2048 | 4096]:
    os.environ['LT_PIPE_DBG'] = str(dbg)
    ms = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws))
    os.environ['LT_FUSED_TRACE'] = str(tr.data_ptr())
    nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
    torch.cuda.synchronize()
    del os.environ['LT_FUSED_TRACE']
    t = tr.cpu().numpy()[4 * B:].reshape(-1, 4)
    work = (t[:, 2] - t[:, 1]) / 100.0
    print(f'dbg={dbg:5d}: {ms:.3f} ms  tile work mean {work.mean():.1f} us', flush=True)


if __name__ == '__main__':
  main()
