"""Rounding budget of the general table kernels (lt_table.hip) at T=1000:
FrameLabelDependent(K) bigram (tests/test_gpu_table.py::
test_fld_k2_bigram_full_length's problem) -- log_z, num and every dW element
of the global and the locally normalised loss against the table oracle,
as ratios to golden_cases.marginal_scale, with the worst element's den and
num marginals. A round-4 diagnostic.

  python tools/fld_precision.py [K]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from last_torch_amd import _native as nat  # noqa: E402
from golden_cases import grad_error_ratio, table_den_marginals  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (the checker)


def main():
  K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
  cuda = torch.device('cuda', 0)
  V, n, B, T, U = 32, 1, 8, 1000, 100
  rng = np.random.default_rng(1000)
  tab = orc.full_ngram_table(V, n)
  W = rng.standard_normal((B, T, V + 1, V + 1)).astype(np.float32)
  nf = rng.integers(T // 2, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(U // 2, U + 1, B).astype(np.int32)
  g = nat.TableGraph(tab, K, cuda)
  Wd = torch.tensor(W, device=cuda)
  nfd, labd, nld = (torch.tensor(x, device=cuda) for x in (nf, lab, nl))
  den = table_den_marginals(orc, tab, W, nf, lab, nl, K)
  for local in (False, True):
    loss, lz, num, dW = nat.table_loss_grad(g, Wd, nfd, labd, nld, local)
    rl, rlz, rnum, rdW = orc.tab_loss_grad(tab, W, nf, lab, nl, K, local_norm=local)
    mag = np.maximum(1.0, np.maximum(np.abs(rlz), np.abs(rnum)))
    u = 2.0 ** -24 * mag
    print(f'local={local}')
    print('  log_z err / u:', np.round(np.abs(lz.cpu().numpy() - rlz) / u, 2))
    print('  num   err / u:', np.round(np.abs(num.cpu().numpy() - rnum) / u, 2))
    r = grad_error_ratio(dW.cpu().numpy(), rdW, None if local else den, rlz, rnum)
    for b in range(B):
      i = np.unravel_index(np.argmax(r[b]), r[b].shape)
      d = 0.0 if local else den[b][i]
      nm = max(d - rdW[b][i], 0.0)
      print(f'  utt {b}: max ratio {r[b].max():.3f} at {list(i)} den {d:.3e} num {nm:.3e} '
            f'(> 1: {(r[b] > 1).sum()})')
  # the den alone: lt_table_den_backward against the oracle
  dist, alpha = nat.table_forward(g, Wd, nfd, nat.SEMIRING_LOG)
  dd = nat.table_den_backward(g, Wd, nfd, nat.SEMIRING_LOG, dist, alpha)
  rlz = orc.tab_den_forward(tab, W, nf, K, orc.LOG)
  r = grad_error_ratio(dd.cpu().numpy(), den, den, rlz, None)
  print('den only: max ratio per utt', np.round(r.reshape(B, -1).max(-1), 3))
  print('  log_z err / u', np.round(np.abs(dist.cpu().numpy() - rlz) / (2.0 ** -24 * np.abs(rlz)), 2))


if __name__ == '__main__':
  main()
