"""Diagnostic: time lt_loss_grad on the chunked path with role ablations
(LT_CK_DBG bitmask, honoured only by the diagnostic build: make diag;
LT_LIB_PATH=build/diag/liblt_lattice_diag.so). Results are wrong under
ablation; only the times mean anything."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
from last_torch_amd import _native  # noqa: E402

B, T, U, V = int(os.environ.get('B', 64)), 1000, 100, 32
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False)], dtype=torch.uint8,
                 device='cuda')
names = {0: 'all', 1: 'B: no den', 2: 'B: no num', 3: 'B: nothing', 4: 'C: no den rec',
         8: 'C: no num rec', 16: 'C: no marginals', 28: 'C: DMA + tables only', 31: 'A only (+B/C shells)'}
if os.environ.get('DBGS'):
  names = {int(x): f'dbg {x}' for x in os.environ['DBGS'].split(',')}
for dbg, name in names.items():
  os.environ['LT_CK_DBG'] = str(dbg)
  for _ in range(3):
    _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(10):
    _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
  e1.record()
  torch.cuda.synchronize()
  print(f'dbg={dbg:2d} {name:24s} {e0.elapsed_time(e1) / 10:.3f} ms', flush=True)
