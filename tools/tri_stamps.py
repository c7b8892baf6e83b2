"""Per-wave, per-frame cycle breakdown from the diagnostic (-DLT_STAMPS)
(trigram bf16 variant: V=32, n=2, env B default 32, CASES default fwd,ck_beta)
library (dev tool, GPU; build it with `make stamps`).

For workgroup 0 of each launch every wave's lane 0 records s_memtime at the
loop top, after the frame barrier and at the end of its frame work. Reports
medians over frames 10..T-10 per wave: step, wait (+barrier) and work.
Env: B (batch), CASES (comma list of fwd,bwd,ck_beta,ck_alpha), plus any
LT_* planner knobs.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

nat.LIB_PATH = os.path.join(ROOT, 'build', 'stamps', 'liblt_lattice_stamps.so')
NW = 16


def report(name, st, T):
  st = st.reshape(NW, T, 4).astype(np.int64)
  print(f'== {name}')
  v = slice(10, T - 10)
  for w in range(NW):
    s = st[w]
    if not s[:, 0].any():
      continue
    step = np.diff(s[:, 0])[10:T - 11]
    wait = s[v, 1] - s[v, 0]
    work = s[v, 2] - s[v, 1]
    print(f'  wave {w:2d}: step {np.median(step):6.0f}  wait {np.median(wait):6.0f}  '
          f'work {np.median(work):6.0f}  work p90 {np.percentile(work, 90):6.0f}', flush=True)


def main():
  B = int(os.environ.get('B', 32))
  T, U, V, n = 1000, 100, 32, int(os.environ.get('N', 2))
  C = nat.num_context_states(V, n)
  W = torch.randn(B, T, C, V + 1, device='cuda').to(torch.bfloat16)
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  st = torch.zeros(NW * T * 4, dtype=torch.int64, device='cuda')
  os.environ['LT_STAMPS_PTR'] = str(st.data_ptr())
  out = nat.loss_forward(W, nf, lab, nl, V, n, False)
  g = torch.ones(B, device='cuda')
  cases = {
      'fwd': lambda: nat.loss_forward(W, nf, lab, nl, V, n, False),
      'bwd': lambda: nat.loss_backward(W, nf, lab, nl, *out[1:5], g, V, n, False),
      'ck_beta': lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True),
  }
  for name in os.environ.get('CASES', 'fwd,ck_beta').split(','):
    if name == 'ck_beta':
      os.environ['LT_CK_SOLO'] = '1'
    fn = cases[name]
    st.zero_()
    fn()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    report(f'{name}: {e0.elapsed_time(e1):.3f} ms (stamped build)', st.cpu().numpy(), T)
    os.environ.pop('LT_CK_SOLO', None)


if __name__ == '__main__':
  main()
