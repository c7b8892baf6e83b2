"""Diagnostic: the chunked path's boundary state (den alpha / beta at every
chunk start) vs a float64 recursion, on a tiny bigram problem."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

B, T, U, V = 2, 8, 4, int(os.environ.get('DIAG_V', 5))
L = int(os.environ.get('LT_CHUNK_LEN', 1))
rng = np.random.default_rng(0)
C = V + 1
W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
nf = np.full(B, T, np.int32)
lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
nl = np.full(B, U, np.int32)
dev = torch.device('cuda')
a = [torch.from_numpy(x).to(dev) for x in (W, nf, lab, nl)]
nb = _native.loss_grad_workspace_bytes(a[0], V, 1, U, False)
ws = torch.zeros([nb], dtype=torch.uint8, device=dev)
_native.loss_grad(a[0], a[1], a[2], a[3], V, 1, False, workspace=ws)
torch.cuda.synchronize()
K = (T + L - 1) // L
CP = (C + 3) & ~3
up = lambda x: (x + 255) & ~255
off = 3 * up(4 * B)
st = ws.cpu().numpy()
abd = st[off:off + 4 * B * (K + 1) * CP].view(np.float32).reshape(B, K + 1, CP)[:, :, :C]
off += up(4 * B * (K + 1) * CP)
bbd = st[off:off + 4 * B * (K + 1) * CP].view(np.float32).reshape(B, K + 1, CP)[:, :, :C]
print('uflag', st[:8].view(np.int32))
for b in range(B):
  Wb = W[b].astype(np.float64)
  al = np.full(C, -np.inf); al[0] = 0
  alist = [al.copy()]
  for f in range(T):
    w = Wb[f]
    new = np.full(C, -np.inf)
    for q in range(1, C):
      terms = [al[p] + w[p, q] for p in range(C)] + [al[q] + w[q, 0]]
      new[q] = np.logaddexp.reduce(terms)
    new[0] = al[0] + w[0, 0]
    al = new
    alist.append(al.copy())
  be = np.zeros(C); blist = [None] * (T + 1); blist[T] = be.copy()
  for f in range(T - 1, -1, -1):
    w = Wb[f]
    new = np.zeros(C)
    for p in range(C):
      terms = [w[p, y] + be[y] for y in range(1, C)] + [w[p, 0] + be[p]]
      new[p] = np.logaddexp.reduce(terms)
    be = new
    blist[f] = be.copy()
  for k in range(K + 1):
    t = min(k * L, T)
    print(f'b={b} k={k} t={t} alpha err {np.abs(abd[b, k] - alist[t]).max():.2e}  '
          f'beta err {np.abs(bbd[b, k] - blist[t]).max():.2e}  beta0 got {bbd[b, k, 0]:.5f} '
          f'ref {blist[t][0]:.5f} core-err {np.abs(bbd[b, k, 1:] - blist[t][1:]).max():.2e}')
