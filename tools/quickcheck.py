"""Quick GPU parity sweep (dev tool): HIP vs oracle on random problems."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from last_torch_amd import _native as nat
from oracle import oracle as orc

def run(B, T, U, V, n, dtype=torch.float32, seed=0):
  rng = np.random.default_rng(seed)
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  if dtype == torch.bfloat16:
    W = torch.tensor(W).bfloat16().float().numpy()
  nf = rng.integers(0, T + 1, B).astype(np.int32); nf[0] = T
  labels = rng.integers(0, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(0, U + 1, B).astype(np.int32)
  Wd = torch.tensor(W).to(dtype).cuda(); nfd = torch.tensor(nf).cuda()
  ld = torch.tensor(labels).cuda(); nld = torch.tensor(nl).cuda()
  out = {}
  for s in (0, 1, 2):
    d, a = nat.den_forward(Wd, nfd, V, n, s)
    rd, ra = orc.den_forward(W, nf, V, n, s)
    ok = np.allclose(d.cpu().numpy(), rd, rtol=1e-4, atol=1e-4, equal_nan=True) if s != 1 else np.array_equal(d.cpu().numpy(), rd)
    oka = np.allclose(a.cpu().numpy(), ra, rtol=1e-4, atol=1e-4) if s != 1 else np.array_equal(a.cpu().numpy(), ra)
    out[f'den{s}'] = (ok, oka)
    nm, an = nat.num_forward(Wd, nfd, ld, nld, V, n, s)
    rn, ran = orc.num_forward(W, nf, labels, nl, V, n, s)
    out[f'num{s}'] = (np.allclose(nm.cpu().numpy(), rn, rtol=1e-4, atol=1e-4), np.allclose(an.cpu().numpy(), ran, rtol=1e-4, atol=1e-4))
  for local in (False, True):
    loss, lz, num, al, an = nat.loss_forward(Wd, nfd, ld, nld, V, n, local)
    dW = nat.loss_backward(Wd, nfd, ld, nld, lz, num, al, an, None, V, n, local)
    rl, rlz, rnum, rdW = orc.loss_grad(W, nf, labels, nl, V, n, local)
    l = loss.cpu().numpy(); fin = np.isfinite(rl)
    out[f'loss{int(local)}'] = (np.array_equal(fin, np.isfinite(l)) and np.allclose(l[fin], rl[fin], rtol=1e-4, atol=1e-4),
                               float(np.abs(dW.float().cpu().numpy() - rdW).max()))
  lz, al = nat.den_forward(Wd, nfd, V, n, 0)
  dWd = nat.den_backward(Wd, nfd, lz, al, None, V, n)
  _, rdWd = orc.den_grad(W, nf, V, n)
  out['den_grad'] = float(np.abs(dWd.float().cpu().numpy() - rdWd).max())
  for conv in (0, 1):
    lab, w, arcs = nat.viterbi(Wd, nfd, V, n, conv, want_arcs=True)
    rlab, rw, rarcs = orc.viterbi(W, nf, V, n, conv, want_arcs=True)
    out[f'vit{conv}'] = (np.array_equal(lab.cpu().numpy(), rlab), np.array_equal(w.cpu().numpy(), rw), np.array_equal(arcs.float().cpu().numpy(), rarcs))
  print(f'B={B} T={T} U={U} V={V} n={n} {dtype}:', out, flush=True)

if __name__ == '__main__':
  for args in [(3, 7, 4, 2, 0), (3, 7, 4, 3, 1), (4, 9, 5, 5, 1), (3, 6, 4, 3, 2), (2, 5, 3, 2, 2), (4, 50, 10, 32, 1), (2, 20, 6, 8, 2)]:
    run(*args)
  run(4, 50, 10, 32, 1, torch.bfloat16)
  run(2, 8, 5, 32, 2, torch.bfloat16)
