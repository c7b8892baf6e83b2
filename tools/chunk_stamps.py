"""Diagnostic: s_memtime marks per phase-C workgroup (diagnostic build:
make diag; LT_LIB_PATH=build/diag/liblt_lattice_diag.so). Prints the median
and 90th percentile of each segment in cycles, and the spread of start
times."""
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
st = torch.zeros([B * 200 * 8], dtype=torch.int64, device='cuda')
for _ in range(3):
  _native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
os.environ['LT_CK_STAMPS'] = hex(st.data_ptr())
_native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
del os.environ['LT_CK_STAMPS']
if os.environ.get('LT_CK_LDS_PAD'):
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(10):
    _native.loss_grad(W, nf, lab, nl, V, 1, False)
  e1.record()
  torch.cuda.synchronize()
  print(f'LDS pad {os.environ["LT_CK_LDS_PAD"]}: {e0.elapsed_time(e1) / 10:.3f} ms per call')
s = st.cpu().numpy().reshape(-1, 8)[:B * (-(-T // 6))]
s = s[s[:, 0] > 0]
segs = [('DMA+tables', 0, 1), ('nw + E', 1, 5), ('recursions', 5, 2), ('marginals', 2, 3),
        ('dW stream', 3, 4)]
for nm, i, j in segs:
  if not s[:, j].any():
    continue
  d = s[:, j] - s[:, i]
  print(f'{nm:12s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f} cycles')
tot = s[:, 4] - s[:, 0]
print(f'{"total":12s} median {np.median(tot):8.0f}  p90 {np.percentile(tot, 90):8.0f}; '
      f'workgroups {len(s)}, span {s[:, 4].max() - s[:, 0].min()} cycles')
