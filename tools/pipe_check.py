"""Dev tool (GPU): the pipelined bigram recursions (lt_pipe.hip) against the
frame-barrier kernels (LT_NO_PIPE=1) on the BASELINE shape -- checkpoints,
loss, dW -- and their timings."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def run(W, nf, lab, nl, V, n, ck):
  out = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=ck)
  dW = nat.loss_backward(W, nf, lab, nl, *out[1:5], None, V, n, False,
                         ck=out[5] if ck else None)
  torch.cuda.synchronize()
  return out, dW


def timeit(fn, reps=20):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def main():
  B = int(os.environ.get('B', 64))
  T, U, V, n = int(os.environ.get('T', 1000)), 100, 32, 1
  C = nat.num_context_states(V, n)
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda')
  nf = torch.randint(T // 2, T + 1, [B], generator=g, device='cuda', dtype=torch.int32)
  nf[0] = T
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  for ck in (True, False):
    os.environ['LT_NO_PIPE'] = '1'
    ref, rdW = run(W, nf, lab, nl, V, n, ck)
    os.environ['LT_NO_PIPE'] = '0'
    got, dW = run(W, nf, lab, nl, V, n, ck)
    names = ['loss', 'log_z', 'num', 'alpha', 'alpha_num']
    for k, nm in enumerate(names):
      d = (got[k] - ref[k]).abs()
      fin = torch.isfinite(ref[k])
      same_inf = bool((torch.isfinite(got[k]) == fin).all())
      print(f'ck={ck} {nm:9s} max|d| {float(d[fin].max()):.3e}  max|ref| '
            f'{float(ref[k][fin].abs().max()):.3e}  inf-pattern-equal {same_inf}', flush=True)
    if ck:
      for k, nm in enumerate(['beta', 'beta_num']):
        r, q = ref[5][k], got[5][k]
        live = torch.isfinite(r)
        d = (q - r).abs()
        print(f'ck={ck} {nm:9s} max|d| {float(d[live].max()):.3e}', flush=True)
    print(f'ck={ck} dW max|d| {float((dW - rdW).abs().max()):.3e}', flush=True)
  for ck in (True, False):
    for pipe in ('0', '1'):
      os.environ['LT_NO_PIPE'] = '1' if pipe == '0' else '0'
      tf = timeit(lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=ck))
      print(f'loss_forward ck={ck} pipe={pipe}: {tf:.3f} ms', flush=True)


if __name__ == '__main__':
  main()
