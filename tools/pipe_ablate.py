"""Timing ablations of the pipelined recursions (dev tool, GPU): loss_forward
(checkpoints) with parts of the work switched off through LT_PIPE_DBG
(results are garbage in the ablated runs; only the time is reported)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def main():
  B, T, U, V, n = int(os.environ.get('B', 64)), 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn(B, T, C, V + 1, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  fn = lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
  for helpers in os.environ.get('HELPERS', '3').split(','):
    os.environ['LT_PIPE_HELPERS'] = helpers
    for dbg in [0, 1, 2, 3, 4, 8, 12, 15]:
      os.environ['LT_PIPE_DBG'] = str(dbg)
      fn()
      torch.cuda.synchronize()
      e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
      e0.record()
      for _ in range(10):
        fn()
      e1.record()
      torch.cuda.synchronize()
      print(f'helpers={helpers} dbg={dbg:2d}: {e0.elapsed_time(e1) / 10:.3f} ms', flush=True)


if __name__ == '__main__':
  main()
