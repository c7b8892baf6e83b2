"""Quick GPU check of the chunked bigram path (lt_loss_grad -> lt_chunk_*)
against the C oracle on assorted shapes; prints one line per case and the
worst errors. Diagnostic tool (the tests live in tests/test_gpu_chunk.py)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def case(name, B, T, U, V, seed=0, scale=1.0, local=False, var=False, bf16=False, eps=0.0):
  rng = np.random.default_rng(seed)
  C = V + 1
  W = (rng.standard_normal((B, T, C, V + 1)) * scale).astype(np.float32)
  if local:
    W = W - np.log(np.exp(W).sum(-1, keepdims=True))
  if bf16:
    W = torch.from_numpy(W).bfloat16().float().numpy()
  nf = (rng.integers(T // 2, T + 1, B) if var else np.full(B, T)).astype(np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  if eps:
    lab[rng.random((B, U)) < eps] = 0
  nl = (rng.integers(0, U + 1, B) if var else np.full(B, U)).astype(np.int32)
  dev = torch.device('cuda')
  Wt = torch.from_numpy(W).to(dev)
  if bf16:
    Wt = Wt.bfloat16()
  t0 = time.time()
  loss, lz, num, dW = _native.loss_grad(Wt, torch.from_numpy(nf).to(dev), torch.from_numpy(lab).to(dev),
                                        torch.from_numpy(nl).to(dev), V, 1, local)
  torch.cuda.synchronize()
  dt = time.time() - t0
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, 1, local_norm=local)
  got = loss.cpu().numpy()
  fin = np.isfinite(rl)
  ok_fin = np.array_equal(fin, np.isfinite(got))
  le = np.max(np.abs(got[fin] - rl[fin]) / np.maximum(1, np.abs(rl[fin]))) if fin.any() else 0
  d = dW.float().cpu().numpy()
  de = np.max(np.abs(d - rdW))
  tol = 1e-5 + 1e-6 * max(1.0, float(np.max(np.abs(rlz)))) + (8e-3 if bf16 else 0)
  status = 'OK' if (ok_fin and le <= 1e-4 and de <= tol) else 'FAIL'
  if status == 'FAIL' or os.environ.get('CK_VERBOSE'):
    idx = np.unravel_index(np.argmax(np.abs(d - rdW)), d.shape)
    print(f'   worst at (b,t,p,y)={idx}: got {d[idx]:.6g} ref {rdW[idx]:.6g}; '
          f'frame sums got {d[idx[0], idx[1]].sum():.4g} ref {rdW[idx[0], idx[1]].sum():.4g}')
    err = np.abs(d - rdW).max(axis=(0, 3))
    print('   max err per (t, p) row p=0..3:', np.array2string(err[:, :4].T, precision=2))
    print('   lz', lz.cpu().numpy()[:3], rlz[:3], 'num', num.cpu().numpy()[:3], rnum[:3])
  print(f'{status} {name}: B={B} T={T} U={U} V={V} loss_rel={le:.2e} dW_abs={de:.2e} '
        f'(tol {tol:.1e}) fin={ok_fin} {dt*1e3:.1f} ms', flush=True)
  return status == 'OK'


def main():
  ok = True
  ok &= case('tiny', 2, 8, 4, 5)
  ok &= case('one-chunk', 3, 10, 3, 32)
  ok &= case('multi-chunk', 4, 100, 20, 32, seed=1)
  ok &= case('varlen', 6, 77, 9, 32, seed=2, var=True)
  ok &= case('small-V', 4, 60, 7, 3, seed=3, var=True)
  ok &= case('V=17', 3, 45, 11, 17, seed=4)
  ok &= case('local', 4, 50, 8, 32, seed=5, local=True)
  ok &= case('eps-labels', 4, 40, 10, 32, seed=6, eps=0.3)
  ok &= case('peaked-fallback', 3, 30, 5, 32, seed=7, scale=30.0)
  ok &= case('bf16', 3, 64, 10, 32, seed=8, bf16=True)
  ok &= case('U=0', 2, 20, 0, 32, seed=9)
  ok &= case('bench-slice', 4, 1000, 100, 32, seed=10)
  print('ALL OK' if ok else 'SOME FAILED')
  return 0 if ok else 1


if __name__ == '__main__':
  sys.exit(main())
