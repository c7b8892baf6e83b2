"""Diagnostic: host issue time of lt_loss_grad at the bench shape against its
GPU time -- per call, the Python + ctypes + launch time measured without a
sync (N calls enqueued back to back), then the whole batch's GPU time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

B, T, U, V = int(os.environ.get('B', 64)), 1000, 100, 32
N = int(os.environ.get('N', 50))
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
nl = torch.full([B], U, dtype=torch.int32, device='cuda')
ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False)], dtype=torch.uint8,
                 device='cuda')
for _ in range(5):
  _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
torch.cuda.synchronize()
for rnd in range(3):
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  t0 = time.perf_counter()
  e0.record()
  host = []
  for _ in range(N):
    h0 = time.perf_counter()
    _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
    host.append(time.perf_counter() - h0)
  e1.record()
  t_issue = time.perf_counter() - t0
  torch.cuda.synchronize()
  t_all = time.perf_counter() - t0
  host.sort()
  print(f'round {rnd}: host per call median {host[N // 2] * 1e6:.1f} us, max {host[-1] * 1e6:.1f} us; '
        f'issue of {N} calls {t_issue * 1e3:.2f} ms; GPU {e0.elapsed_time(e1) / N:.4f} ms/call; '
        f'wall {t_all / N * 1e3:.4f} ms/call', flush=True)
