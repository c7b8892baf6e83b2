"""Diagnostic: 20 lt_loss_grad calls at the bench shape (for rocprofv3)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
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
for _ in range(int(os.environ.get('N', 20))):
  _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
torch.cuda.synchronize()
