"""Dev tool (GPU): the pipelined bigram recursions alone (lt_loss_forward
with checkpoints) at B (default 256) over helper-wave counts, ring slots and
LDS caps, in one process. SWEEP = "helpers:slots:lds,..." (empty = default)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from last_torch_amd import _native as nat  # noqa: E402
from fused_check import timeit  # noqa: E402


def main():
  B, T, U, V, n = int(os.environ.get('B', 256)), 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  os.environ['LT_VERBOSE'] = '1'
  for cfg in os.environ.get('SWEEP', '::,4:16:,3:16:,2:16:,4:8:,4:32:,4:16:65536').split(','):
    h, s, l = (cfg.split(':') + ['', '', ''])[:3]
    os.environ['LT_PIPE_HELPERS'], os.environ['LT_PIPE_SLOTS'], os.environ['LT_PIPE_LDS'] = h, s, l
    t = timeit(lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True))
    print(f'helpers={h or "default"} slots={s or "default"} lds={l or "default"}: {t:.3f} ms',
          flush=True)


if __name__ == '__main__':
  main()
