"""Dev tool (GPU): timeline of one fused loss+grad launch (LT_FUSED_TRACE):
recursion workgroup spans and marginal tile grab/ready/done times."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def main():
  B, T, U, V, n = int(os.environ.get('B', 64)), 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([1 << 30], dtype=torch.uint8, device='cuda')
  FT = int(os.environ.get('LT_FUSED_FW', 4)) * 6
  NB = (T + FT - 1) // FT
  grid = int(os.environ.get('GRID', 512))
  tr = torch.zeros([2 * 2 * B + 4 * NB * B + 2 * grid], dtype=torch.int64, device='cuda')
  for _ in range(3):
    nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
  torch.cuda.synchronize()
  os.environ['LT_FUSED_TRACE'] = str(tr.data_ptr())
  nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
  torch.cuda.synchronize()
  del os.environ['LT_FUSED_TRACE']
  t = tr.cpu().numpy()
  rec = t[:4 * B].reshape(2 * B, 2)
  tiles = t[4 * B:4 * B + 4 * NB * B].reshape(NB * B, 4)
  wg = t[4 * B + 4 * NB * B:].reshape(grid, 2)
  hw = wg[:, 1]
  xcc = (hw >> 32) & 0xff
  hwid = hw & 0xffffffff
  cu = (hwid >> 8) & 0xf
  sh = (hwid >> 12) & 1
  se = (hwid >> 13) & 0x7
  key = xcc * 1000 + se * 100 + sh * 20 + cu
  uniq, cnt = np.unique(key, return_counts=True)
  print(f'workgroups started: {int((wg[:,0] > 0).sum())}, distinct CUs: {uniq.size}, '
        f'per-CU counts: {np.bincount(cnt).tolist()}')
  st = (wg[:, 0] - rec[:, 0].min()) / 100.0
  print('start times (us) quantiles:', np.quantile(st, [0, 0.25, 0.5, 0.75, 0.9, 1.0]).round(1).tolist())
  t0 = rec[:, 0].min()
  us = lambda x: (x - t0) / 100.0  # s_memrealtime: 100 MHz
  print(f'recursion start: {us(rec[:,0]).min():.1f}..{us(rec[:,0]).max():.1f} us, '
        f'end: {us(rec[:,1]).min():.1f}..{us(rec[:,1]).max():.1f} us')
  print(f'alpha dur mean {np.mean((rec[:B,1]-rec[:B,0])/100):.1f} us, '
        f'beta dur mean {np.mean((rec[B:,1]-rec[B:,0])/100):.1f} us')
  g, r, d = us(tiles[:, 0]), us(tiles[:, 1]), us(tiles[:, 2])
  print(f'tiles: grab {g.min():.1f}..{g.max():.1f}, done {d.min():.1f}..{d.max():.1f} us')
  work = d - np.maximum(r, g)
  print(f'tile work (done - ready) mean {np.mean(work):.1f} us p50 {np.median(work):.1f} '
        f'p90 {np.percentile(work, 90):.1f} max {work.max():.1f}')
  wait = r - g
  print(f'tile wait (ready - grab) mean {np.mean(wait):.1f} us max {wait.max():.1f}')
  for q in (0.25, 0.5, 0.75, 0.9, 1.0):
    print(f'  {int(q*100)}% of tiles done by {np.quantile(d, q):.1f} us')
  hist = np.histogram(d, bins=20)
  print('done histogram:', list(zip(hist[1][:-1].round(0).tolist(), hist[0].tolist())))
  roles = np.unique(tiles[:, 3]).size
  print(f'marginal workgroups used: {roles}')


if __name__ == '__main__':
  main()
