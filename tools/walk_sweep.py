"""Diagnostic: lt_loss_grad time at the bench shape vs the fused launch's walk
position (LT_CHUNK_WALK_AT, percent of phase A's workgroups) and unfused
(LT_CHUNK_FUSE=0), for several batch sizes. HIP events around 20 calls."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

T, U, V = 1000, 100, 32
for B in [int(x) for x in os.environ.get('BS', '32,64,128,256').split(',')]:
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False)], dtype=torch.uint8,
                   device='cuda')
  ref = None
  for at in ['nofuse', 'default', '0', '25', '50', '65', '75', '85', '92', '100']:
    os.environ.pop('LT_CHUNK_WALK_AT', None)
    os.environ['LT_CHUNK_FUSE'] = '0' if at == 'nofuse' else '1'
    if at not in ('nofuse', 'default'):
      os.environ['LT_CHUNK_WALK_AT'] = at
    for _ in range(3):
      out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
      out = _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    loss = out[0].cpu()
    if ref is None:
      ref = loss
    same = bool(torch.equal(loss, ref))
    print(f'B={B} walk_at={at}: {ms * 1e3:.1f} us per call, loss identical={same}', flush=True)
  del W, ws
  torch.cuda.empty_cache()
