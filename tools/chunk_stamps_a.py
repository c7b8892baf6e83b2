"""Diagnostic: s_memtime marks per phase-A chunk wave (diagnostic build:
make diag; LT_LIB_PATH=build/diag/liblt_lattice_diag.so): prologue (labels,
string offsets), the frame loop, the record / band stores; the spread of
start times (dispatch rounds). LT_CHUNK_FUSE as set by the caller."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
from last_torch_amd import _native  # noqa: E402

B, T, U, V = int(os.environ.get('B', 64)), 1000, 100, 32
K = -(-T // 6)
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
st = torch.zeros([B * K * 12 + 64], dtype=torch.int64, device='cuda')
for _ in range(3):
  _native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
os.environ['LT_CK_DBG'] = '256'
os.environ['LT_CK_STAMPS'] = hex(st.data_ptr())
_native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
del os.environ['LT_CK_STAMPS'], os.environ['LT_CK_DBG']
s = st.cpu().numpy()[B * K * 8:B * K * 12].reshape(-1, 4)
s = s[s[:, 0] > 0]
for nm, i, j in [('prologue', 0, 1), ('frames', 1, 2), ('stores', 2, 3), ('total', 0, 3)]:
  d = s[:, j] - s[:, i]
  print(f'{nm:10s} median {np.median(d):8.0f}  p10 {np.percentile(d, 10):8.0f}  '
        f'p90 {np.percentile(d, 90):8.0f} cycles (s_memtime)')
t0 = s[:, 0].min()
span = s[:, 3].max() - t0
print(f'waves {len(s)}, span {span} cycles; start-time deciles:',
      np.percentile(s[:, 0] - t0, np.arange(0, 101, 10)).astype(int))
