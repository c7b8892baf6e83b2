"""Diagnostic (a build with -DLT_MIX_DUMPLZ): the log-Z norm each marginal
wave used per frame, read back from the done flags, per utterance."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

B, T, U, V, n = 8, 1000, 100, 32, 2
C = nat.num_context_states(V, n)
g = torch.Generator(device='cuda')
g.manual_seed(5)
W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
nb = nat.loss_grad_workspace_bytes(W, V, n, U, False)
ws = torch.zeros([nb], dtype=torch.uint8, device='cuda')
off = nb - ((4 * (8 * B + 256 + B * T) + 255) & ~255)
loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
torch.cuda.synchronize()
mw = ws[off:off + 4 * (8 * B + 256 + B * T)].view(torch.int32)
ts = mw[4 * B + 256 + B * T:4 * B + 256 + B * T + 8].tolist()
print('row mismatches alpha / beta / alpha_num / beta_num, frames checked:', ts[:5], '; table mismatches, jobs:', ts[5:7])
bad = ~torch.isfinite(dW.float().reshape(B, T, -1)).all(-1)
print('non-finite frames', int(bad.sum()))
print('num from the recursions', num.tolist())
done = mw[4 * B + 256:4 * B + 256 + B * T].reshape(B, T).view(torch.float32).cpu()
for b in range(B):
  vals, counts = torch.unique(done[b], return_counts=True)
  order = counts.argsort(descending=True)
  print(f'utt {b}: {vals.numel()} distinct; top', [(float(vals[i]), int(counts[i])) for i in order[:4]])
