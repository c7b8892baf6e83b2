"""Diagnostic: lt_loss_grad per-call time (HIP events around N calls, best
of 3 rounds) for the library LT_LIB_PATH names, at BS batch sizes of the
bench shape. Prints one line per batch size, prefixed by TAG."""
import os
import sys

import torch

ROOT = os.environ.get('LT_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

T, U, V = 1000, 100, 32
N = int(os.environ.get('N', 20))
tag = os.environ.get('TAG', os.path.basename(os.environ.get('LT_LIB_PATH', 'product')))
DESIGN = {'auto': -1, 'chunk': 0, 'fused': 1, 'checkpoints': 2, 'recursion': 3}[
    os.environ.get('DESIGN', 'auto')]
for B in [int(x) for x in os.environ.get('BS', '64').split(',')]:
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False, DESIGN)],
                   dtype=torch.uint8, device='cuda')
  best = 1e9
  for _ in range(3):
    for _ in range(3):
      out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws, design=DESIGN)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(N):
      out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws, design=DESIGN)
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / N)
  print(f'{tag:24s} {os.environ.get("DESIGN", "auto"):11s} B={B}: {best:.3f} ms  loss[0] {out[0][0].item():.6f}', flush=True)
