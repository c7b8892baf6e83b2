"""Diagnostic: which dW elements of the overlap's frames differ from the
frame-serial design (LT_TRI_MIX=0), grouped by the marginal wave's unit
loop: unit u = (e - h0) / 8 of lane u % 64, trip u // 320, round (u // 64) % 5."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

B, T, U, V, n = 8, 1000, 100, 32, 2
C = nat.num_context_states(V, n)
FR = C * (V + 1)
g = torch.Generator(device='cuda')
g.manual_seed(5)
W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
os.environ['LT_TRI_MIX'] = '0'
ref = nat.loss_grad(W, nf, lab, nl, V, n, False)[3].float().reshape(B, T, FR)
os.environ['LT_TRI_MIX'] = '1'
dW = torch.full_like(W, float('nan'))
out = nat.loss_grad(W, nf, lab, nl, V, n, False)[3].float().reshape(B, T, FR)
wrong = ((out - ref).abs() > 1e-2) | ~torch.isfinite(out)
nw = wrong.sum(-1)
print('frames with wrong elements', int((nw > 0).sum()), 'of', B * T)
frames = (nw > 0).nonzero().tolist()
for bb, tt in frames[:3] + frames[len(frames) // 2:len(frames) // 2 + 2]:
  base = (bb * T + tt) * FR
  h0 = ((16 - (2 * base) % 16) % 16) // 2
  nunits = (FR - h0) // 8
  idx = wrong[bb, tt].nonzero().flatten().cpu()
  tail = idx[(idx < h0) | (idx >= h0 + nunits * 8)]
  u = (idx[(idx >= h0) & (idx < h0 + nunits * 8)] - h0) // 8
  lanes = torch.unique(u % 64)
  trips = torch.unique(u // 320)
  rounds = torch.unique((u // 64) % 5)
  print(f'b={bb} t={tt} h0={h0}: wrong {idx.numel()} (tail {tail.numel()}), units {torch.unique(u).numel()} '
        f'of {nunits}; lanes {lanes.numel()} {lanes[:12].tolist()}; trips {trips.tolist()[:12]}; rounds {rounds.tolist()}; '
        f'values {out[bb, tt, idx[:3]].tolist()} vs {ref[bb, tt, idx[:3]].tolist()}', flush=True)
