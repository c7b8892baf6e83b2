"""Diagnostic: s_memtime segments of the Viterbi chain wave (block 0, the
first 128 frames) in the diagnostic build: frame wait + LDS reads, compute +
alpha write + publish, slack check + ring issue, loop back. Median cycles."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
from last_torch_amd import _native as nat  # noqa: E402

B, T, V = 64, 2000, 32
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
st = torch.zeros([128 * 4], dtype=torch.int64, device='cuda')
nat.viterbi(W, nf, V, 1, nat.LABELS_REFERENCE)
torch.cuda.synchronize()
os.environ['LT_VIT_STAMPS'] = hex(st.data_ptr())
nat.viterbi(W, nf, V, 1, nat.LABELS_REFERENCE)
torch.cuda.synchronize()
s = st.cpu().numpy().reshape(128, 4)[8:127].astype(np.float64)
nxt = st.cpu().numpy().reshape(128, 4)[9:128, 0].astype(np.float64)
for nm, d in [('wait + LDS reads', s[:, 1] - s[:, 0]), ('compute + write + publish', s[:, 2] - s[:, 1]),
              ('slack check + issue', s[:, 3] - s[:, 2]), ('loop back', nxt - s[:, 3]),
              ('step', nxt - s[:, 0])]:
  print(f'{nm:28s} median {np.median(d):7.0f}  p90 {np.percentile(d, 90):7.0f}')
