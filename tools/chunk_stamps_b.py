"""Diagnostic: per-wave start/end s_memtime marks of phase B (diagnostic
build, LT_CK_DBG=64). Waves: 0 den alpha, 1 den beta, 2 num alpha, 3 num beta."""
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
st = torch.zeros([B * 8 * 8], dtype=torch.int64, device='cuda')
for _ in range(3):
  _native.loss_grad(W, nf, lab, nl, V, 1, False)
torch.cuda.synchronize()
for extra, what in ((0, 'all waves'), (1 | 128, 'num beta alone'), (2, 'den alone'),
                    (2 | 512, 'den alone, no record loads')):
  st.zero_()
  os.environ['LT_CK_DBG'] = str(64 | extra)
  os.environ['LT_CK_STAMPS'] = hex(st.data_ptr())
  _native.loss_grad(W, nf, lab, nl, V, 1, False)
  torch.cuda.synchronize()
  s = st.cpu().numpy().reshape(-1, 8)[:B]
  print(what)
  for w, nm in enumerate(['den alpha', 'den beta', 'num alpha', 'num beta']):
    d = s[:, 2 * w + 1] - s[:, 2 * w]
    print(f'  {nm:10s} median {np.median(d):9.0f} cycles  max {d.max():9.0f}')
