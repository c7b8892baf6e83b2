"""Times the lattice kernels under LT_DBG ablations (dev tool, GPU)."""
import os, sys, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from last_torch_amd import _native as nat

def timeit(fn, reps=10):
  fn(); torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps): fn()
  e.record(); torch.cuda.synchronize()
  return s.elapsed_time(e) / reps

def main():
  B = int(os.environ.get('B', 64)); T, U, V, n = 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn(B, T, C, V + 1, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  loss, lz, num, al, an = nat.loss_forward(W, nf, lab, nl, V, n, False)
  g = torch.ones(B, device='cuda')
  res = {}
  for dbg in [0, 1, 2, 3, 4, 7, 8, 15]:
    os.environ['LT_DBG'] = str(dbg)
    f = timeit(lambda: nat.loss_forward(W, nf, lab, nl, V, n, False))
    bwd = timeit(lambda: nat.loss_backward(W, nf, lab, nl, lz, num, al, an, g, V, n, False))
    den = timeit(lambda: nat.den_forward(W, nf, V, n, 0, want_alpha=False))
    vit = timeit(lambda: nat.den_forward(W, nf, V, n, 1, want_alpha=False))
    res[dbg] = dict(fwd=round(f, 4), bwd=round(bwd, 4), den_only=round(den, 4), max_only=round(vit, 4))
    print(dbg, res[dbg], flush=True)
  for L in [2, 4, 8, 16]:
    os.environ['LT_DBG'] = '0'; os.environ['LT_DEN_LANES'] = str(L)
    try:
      f = timeit(lambda: nat.loss_forward(W, nf, lab, nl, V, n, False))
      bwd = timeit(lambda: nat.loss_backward(W, nf, lab, nl, lz, num, al, an, g, V, n, False))
      print('L', L, round(f, 4), round(bwd, 4), flush=True)
    except Exception as ex:
      print('L', L, 'fail', ex)
  os.environ.pop('LT_DEN_LANES')

main()
