"""Diagnostic: phase C's timeline at the bench shape from s_memtime marks
(diagnostic build: make diag). The walks' phase-2 workgroups (blocks [0, B))
against the chunk workgroups (block B + j B + b: level j of utterance b, the
levels middle-out): when each starts and ends, relative to its XCD's first
start (s_memtime is per XCD, so blocks are compared within block % 8), and
how long a chunk's poll for its walk boundaries took."""
import os
import sys

import numpy as np
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
K = -(-T // 6)
st = torch.zeros([(B + B * K) * 8], dtype=torch.int64, device='cuda')
for _ in range(30):
  _native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
os.environ['LT_CK_STAMPS'] = hex(st.data_ptr())
_native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
del os.environ['LT_CK_STAMPS']
s = st.cpu().numpy().reshape(-1, 8).astype(np.int64)
blk = np.arange(len(s))
xcd = blk % 8
t0 = np.zeros(8, np.int64)
for x in range(8):
  m = (xcd == x) & (s[:, 0] > 0)
  t0[x] = s[m, 0].min()
rel = s - t0[xcd][:, None]
walk = slice(0, B)
print(f'walk blocks: start median {np.median(rel[walk, 0]):.0f} max {rel[walk, 0].max()}; '
      f'end median {np.median(rel[walk, 4]):.0f} max {rel[walk, 4].max()} cycles')
ch = rel[B:B + B * K]
live = s[B:B + B * K, 0] > 0
lev = (np.arange(B * K) // B)
print(f'chunk blocks live {live.sum()}; last end {ch[live, 4].max()} cycles')
for lo in range(0, K, 12):
  m = live & (lev >= lo) & (lev < lo + 12)
  if not m.any():
    continue
  pw = np.where(s[B:B + B * K, 6][m] > 0, ch[m, 6] - ch[m, 0], 0)
  print(f'levels {lo:3d}-{lo + 11:3d}: start {np.median(ch[m, 0]):8.0f}  end {np.median(ch[m, 4]):8.0f}  '
        f'life {np.median(ch[m, 4] - ch[m, 0]):6.0f}  poll {np.median(pw):6.0f} p90 {np.percentile(pw, 90):6.0f}')
