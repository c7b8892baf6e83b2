"""Diagnostic: the trigram overlap (lt_tri.hip) on several shapes: which
frames of dW come out non-finite or differ from the frame-serial design's
dW (LT_TRI_MIX=0 in the diagnostic build), per utterance, and how many
frames the overlap's marginal waves did (the done flags at the workspace's
end, LT_TRI_MIX_DBG=8: each flag the XCD id + 1 of the wave that did it)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('LT_LIB_PATH', os.path.join(ROOT, 'build/diag/liblt_lattice_diag.so'))
from last_torch_amd import _native as nat  # noqa: E402

V, n = 32, 2
C = nat.num_context_states(V, n)
print('CUs', torch.cuda.get_device_properties(0).multi_processor_count, flush=True)


def up(x):
  return (x + 255) & ~255


REPS = int(os.environ.get('REPS', '3'))
QUICK = os.environ.get('QUICK') == '1'
for (B, T, U) in ([(8, 1000, 100)] if QUICK else [(8, 160, 12), (8, 1000, 100), (32, 1000, 100)]):
  g = torch.Generator(device='cuda')
  g.manual_seed(5)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(torch.bfloat16)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  nb = nat.loss_grad_workspace_bytes(W, V, n, U, False)
  ws = torch.zeros([nb], dtype=torch.uint8, device='cuda')
  mix_off = nb - up(4 * (8 * B + 8 * 32 + B * T))
  os.environ['LT_TRI_MIX'] = '0'
  ref = nat.loss_grad(W, nf, lab, nl, V, n, False)[3].float().reshape(B, T, -1)
  for mode in (['8'] if QUICK else ['8'] * REPS + ['1', '2', '4']):
    os.environ['LT_TRI_MIX'] = '1'
    os.environ['LT_TRI_MIX_DBG'] = mode
    ws.fill_(0x7f)
    loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
    torch.cuda.synchronize()
    mw = ws[mix_off:mix_off + 4 * (4 * B + 256 + B * T)].view(torch.int32)
    prog, xcc, done = mw[:2 * B], mw[2 * B:4 * B], mw[4 * B + 256:].reshape(B, T)
    d = dW.float().reshape(B, T, -1)
    bad = ~torch.isfinite(d).all(-1)
    err = (d - ref).abs().nan_to_num(1e30).amax(-1)
    wrong = err > 1e-2
    print(f'B={B} T={T} dbg={mode}: bad {int(bad.sum())} wrong {int(wrong.sum())} of {B * T}; '
          f'done by mix {int((done != 0).sum())}; wrong & done {int((wrong & (done != 0)).sum())}; '
          f'prog {prog[:4].tolist()} xcc {xcc.tolist()[:16]}', flush=True)
    if mode == '8':
      own = done[done != 0]
      xr = xcc[:B].repeat_interleave(T).reshape(B, T)
      print(f'   done flag values {torch.unique(own).tolist()}; frames done off their recursion XCD '
            f'{int(((done != 0) & (done != xr)).sum())}', flush=True)
    if int(wrong.sum()):
      bb, tt = wrong.nonzero()[0].tolist()
      x, y = d[bb, tt], ref[bb, tt]
      idx = (((x - y).abs() > 1e-2) | ~torch.isfinite(x)).nonzero().flatten()
      print(f'   b={bb} t={tt} done={int(done[bb, tt])}: wrong elements {idx.numel()}, first '
            f'{idx[:6].tolist()}; mix {x[idx[:4]].tolist()} serial {y[idx[:4]].tolist()}', flush=True)
  del W, ws, ref
