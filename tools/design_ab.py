"""Diagnostic: lt_loss_grad per-call time of the chunked scan against the
frame-serial designs (LT_CHUNK=0: checkpointing pipe + marginal pass, or the
fused pipe launch) at the same shape, interleaved in rounds on one box (HIP
events around N calls). BS = batch sizes, default 64,128,192,256."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

T, U, V = 1000, 100, 32
N = int(os.environ.get('N', 20))
designs = {'chunk': {'LT_CHUNK': '1'}, 'serial': {'LT_CHUNK': '0'},
           'fused': {'LT_CHUNK': '0', 'LT_MID': '1'}}
for B in [int(x) for x in os.environ.get('BS', '64,128,192,256').split(',')]:
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  res = {k: [] for k in designs}
  losses = {}
  for rnd in range(3):
    for name, env in designs.items():
      for k in ('LT_CHUNK', 'LT_MID'):
        os.environ.pop(k, None)
      os.environ.update(env)
      ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False)], dtype=torch.uint8,
                       device='cuda')
      for _ in range(3):
        out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record()
      for _ in range(N):
        out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
      e1.record()
      torch.cuda.synchronize()
      res[name].append(e0.elapsed_time(e1) / N)
      losses[name] = out[0].double().cpu()
      del ws
  os.environ.pop('LT_CHUNK', None)
  os.environ.pop('LT_MID', None)
  dl = (losses['chunk'] - losses['serial']).abs().max().item()
  gb = 15756.0 * B * T / 1e9
  line = ' '.join(f'{k} {min(v):.3f} ms ({100 * gb / min(v) / 8:.1f} %)' for k, v in res.items())
  print(f'B={B}: {line}  max|dloss| {dl:.2e}', flush=True)
