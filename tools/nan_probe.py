"""Diagnostic: where lt_loss_grad's dW goes NaN on the mixed fallback batch
of tests/test_gpu_full_size.py (per design), and which utterances took the
frame-serial fallback."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

V, n, T, U = 32, 1, 300, 40
rng = np.random.default_rng(21)
W = rng.standard_normal((6, T, V + 1, V + 1)).astype(np.float32)
W[1] *= 30.0
W[3, 17, 5, 7] = -np.inf
W[4, 250] *= 40.0
nf = np.array([300, 300, 123, 300, 280, 1], np.int32)
lab = rng.integers(1, V + 1, (6, U)).astype(np.int32)
nl = np.array([40, 35, 20, 40, 40, 0], np.int32)
dev = torch.device('cuda')
Wd = torch.tensor(W, device=dev)
nfd, labd, nld = (torch.tensor(x, device=dev) for x in (nf, lab, nl))
for name, d in (('auto', nat.DESIGN_AUTO), ('recursion', nat.DESIGN_RECURSION),
                ('checkpoints', nat.DESIGN_CHECKPOINTS), ('fused', nat.DESIGN_FUSED_PIPE)):
  for local in (False, True):
    nb = nat.loss_grad_workspace_bytes(Wd, V, n, U, local, d)
    ws = torch.zeros([max(nb, 1)], dtype=torch.uint8, device=dev)
    loss, lz, num, dW = nat.loss_grad(Wd, nfd, labd, nld, V, n, local, workspace=ws, design=d)
    torch.cuda.synchronize()
    bad = ~torch.isfinite(dW)
    per_b = bad.reshape(6, -1).sum(1).tolist()
    frames = {b: sorted(set(torch.nonzero(bad[b].reshape(T, -1).any(1)).flatten().tolist()))[:8]
              for b in range(6) if per_b[b]}
    fb = ws[:24].view(torch.int32).tolist() if d in (nat.DESIGN_AUTO, nat.DESIGN_CHUNK) else None
    print(name, 'local' if local else 'global', 'nonfinite dW per utt', per_b, 'frames', frames,
          'uflag', fb, 'loss', loss.tolist(), flush=True)
