"""Diagnostic: lt_loss_grad call time with phase B's walks ablated
(diagnostic build, LT_CK_DBG: 1 den walks off, 2 numerator walks off, 3
both), so the A+B launch's time beyond A's own shows. Results are wrong
under the ablations; only the times mean anything."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
from last_torch_amd import _native  # noqa: E402

T, U, V = 1000, 100, 32
for B in [int(x) for x in os.environ.get('BS', '64').split(',')]:
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False, 0)], dtype=torch.uint8,
                   device='cuda')
  for dbg in [x for x in os.environ.get('DBGS', '0,1,2,3,16,12').split(',')]:
    os.environ['LT_CK_DBG'] = dbg
    best = 1e9
    for _ in range(3):
      for _ in range(2):
        _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws, design=0)
      e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
      e0.record()
      for _ in range(10):
        _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws, design=0)
      e1.record()
      torch.cuda.synchronize()
      best = min(best, e0.elapsed_time(e1) / 10)
    print(f'B={B} LT_CK_DBG={dbg:4s} {best:.3f} ms', flush=True)
  os.environ['LT_CK_DBG'] = '0'
