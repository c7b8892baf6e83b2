"""Diagnostic: den-only / num-only split of the chunked path's dW on a tiny
bigram problem, per frame, vs the C oracle (tools/ only; not a test)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402
from oracle import oracle as orc  # noqa: E402

B, T, U, V = 2, 8, 4, int(os.environ.get('DIAG_V', 5))
rng = np.random.default_rng(0)
C = V + 1
W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
nf = np.full(B, T, np.int32)
lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
nl = np.full(B, U, np.int32)
dev = torch.device('cuda')
args = [torch.from_numpy(x).to(dev) for x in (W, nf, lab, nl)]
_, _, _, dg = _native.loss_grad(args[0], args[1], args[2], args[3], V, 1, False)
_, _, _, dl = _native.loss_grad(args[0], args[1], args[2], args[3], V, 1, True)
dg, dl = dg.cpu().numpy(), dl.cpu().numpy()
_, ref_den = orc.den_grad(W, nf, V, 1)
_, _, _, ref_loc = orc.loss_grad(W, nf, lab, nl, V, 1, local_norm=True)
print('L =', os.environ.get('LT_CHUNK_LEN', 'auto'), 'V =', V)
print('num-only (local) err per frame:', np.abs(dl - ref_loc).max(axis=(0, 2, 3)))
print('den err per frame:', np.abs((dg - dl) - ref_den).max(axis=(0, 2, 3)))
