"""Diagnostic: the trigram overlap's timeline at cfg5 (B=32 T=1000 U=100
bf16) in the diagnostic build (LT_TRI_MIX_DBG=16): when each recursion
workgroup started and ended and when each frame's marginals were done, in
microseconds from the first recursion start (s_memrealtime, 100 MHz)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
os.environ['LT_TRI_MIX_DBG'] = str(16 | int(os.environ.get('DBG', '0')))
from last_torch_amd import _native as nat  # noqa: E402

B, T, U, V, n = 32, 1000, 100, 32, 2
B = int(os.environ.get('B', B))
C = nat.num_context_states(V, n)
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
lab = torch.randint(1, V + 1, (B, U), generator=g, device='cuda', dtype=torch.int32)
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
nb = nat.loss_grad_workspace_bytes(W, V, n, U, False)
ws = torch.zeros([nb], dtype=torch.uint8, device='cuda')
off = nb - ((4 * (8 * B + 256 + B * T) + 255) & ~255)
for _ in range(3):
  nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
torch.cuda.synchronize()
mw = ws[off:off + 4 * (8 * B + 256 + B * T)].view(torch.int32).cpu().long()
done = mw[4 * B + 256:4 * B + 256 + B * T].reshape(B, T)
ts = mw[4 * B + 256 + B * T:]
t0 = int(ts[:2 * B].min())
rs = (ts[:2 * B] - t0).float() / 100.0
re = (ts[2 * B:4 * B] - t0).float() / 100.0
print(f'recursion starts (us): max {float(rs.max()):.1f}; ends: min {float(re.min()):.1f} '
      f'median {float(re.median()):.1f} max {float(re.max()):.1f}', flush=True)
mixed = done != 0
tc = ((done & 0x3fffffff) - t0).float() / 100.0
tc[~mixed] = float('nan')
v = tc[mixed]
print(f'frames done by the marginal waves: {int(mixed.sum())} of {B * T}; completion (us): '
      f'first {float(v.min()):.1f} median {float(v.median()):.1f} last {float(v.max()):.1f}; '
      f'after the last recursion end: {int((v > float(re.max())).sum())}', flush=True)
edges = list(range(0, int(float(v.max())) + 100, 100))
hist = [int(((v >= a) & (v < a + 100)).sum()) for a in edges]
print('frames done per 100 us: ' + ' '.join(f'{a}:{h}' for a, h in zip(edges, hist)), flush=True)
mid = T // 2
for dist in (0, 100, 200, 300, 400, 450, 490, 499):
  print(f'  |t - mid| = {dist}: completion median {float(tc[:, mid + dist if mid + dist < T else T - 1].nanmedian()):.1f} us',
        flush=True)
