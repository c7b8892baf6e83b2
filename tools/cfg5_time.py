"""Diagnostic: cfg5 (trigram bf16 loss + dW, B=32 T=1000 U=100 V=32 n=2)
lt_loss_grad time under the current environment (LT_CHECKPOINTS etc.)."""
import os
import sys

import torch

ROOT = os.environ.get('LT_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

B, T, U, V, n = 32, 1000, 100, 32, 2
C = nat.num_context_states(V, n)
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
lab = torch.randint(1, V + 1, (B, U), generator=g, device='cuda', dtype=torch.int32)
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
ws = torch.empty([nat.loss_grad_workspace_bytes(W, V, n, U, False)], dtype=torch.uint8, device='cuda')
WARM, N = int(os.environ.get('WARM', 2)), int(os.environ.get('N', 5))
for _ in range(WARM):
  out = nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
e0.record()
for _ in range(N):
  out = nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
e1.record()
torch.cuda.synchronize()
print(f"lib={os.environ.get('LT_LIB_PATH', 'prod')} mid={os.environ.get('LT_TRI_MID', 'default')}: {e0.elapsed_time(e1) / N:.2f} ms, "
      f"loss[0]={out[0][0].item():.4f}", flush=True)
