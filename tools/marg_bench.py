"""Times the checkpointing marginal pass for a few tile sizes (dev tool, GPU)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def main():
  T, U, V, n = 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  for B in [int(x) for x in os.environ.get('BS', '64,256').split(',')]:
    for bf16 in (False, True):
      W = torch.randn(B, T, C, V + 1, device='cuda')
      if bf16:
        W = W.bfloat16()
      nf = torch.full([B], T, dtype=torch.int32, device='cuda')
      lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
      nl = torch.full([B], U, dtype=torch.int32, device='cuda')
      out = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
      es = 2 if bf16 else 4
      byt = B * T * (2 * C * (V + 1) * es + 8 * C + 8 * (U + 1))
      for units in os.environ.get('UNITS', '1,2,3,4,5').split(','):
        os.environ['LT_MARG_UNITS'] = units
        f = lambda: nat.loss_backward(W, nf, lab, nl, *out[1:5], None, V, n, False, ck=out[5])
        for _ in range(3):
          f()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(10):
          f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f'B={B} bf16={bf16} units={units}: {ms:.3f} ms  {byt / ms / 1e9:.2f} TB/s',
              flush=True)


main()
