"""Dev tool (GPU): the north-star shape (B=256, T=1000, U=100, bigram V=32)
under each loss + gradient design, in one process (box-to-box variance is
larger than the differences): recursion (LT_CHECKPOINTS=0), two-call
checkpointing (LT_FUSED=0) and the fused launch forced on (LT_FUSED=1) with
a sweep of marginal workgroup counts. Checks the forced fused result against
the two-call one first."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from last_torch_amd import _native as nat  # noqa: E402
from fused_check import check, timeit  # noqa: E402


def step(W, nf, lab, nl, V, n, g1, ws):
  return nat.scale_grad(nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)[3], g1, V, n)


def main():
  B = int(os.environ.get('B', 256))
  T, U, V, n = 1000, 100, 32, 1
  os.environ['LT_CHECKPOINTS'] = '1'
  os.environ['LT_FUSED'] = '1'
  if os.environ.get('CHECK', '1') == '1':
    ok = check(B, T, U, V, varlen=True) and check(B, T, U, V, bf16=True, seed=1)
    print('forced fused', 'OK' if ok else 'FAILED', flush=True)
    if not ok:
      sys.exit(1)
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  g1 = torch.ones([B], device='cuda')
  ws = torch.empty([nat.loss_grad_workspace_bytes(W, V, n, U, False)], dtype=torch.uint8,
                   device='cuda')
  cells = B * T * C * (V + 1)
  runs = [('recursion', {'LT_CHECKPOINTS': '0', 'LT_FUSED': '0'})]
  for u in os.environ.get('UNITS', '5').split(','):
    runs.append((f'two-call checkpoints units={u}',
                 {'LT_CHECKPOINTS': '1', 'LT_FUSED': '0', 'LT_MARG_UNITS': u}))
  for m in [m for m in os.environ.get('MARG', '0,64,128,256,512').split(',') if m]:
    runs.append((f'fused marg={m}', {'LT_CHECKPOINTS': '1', 'LT_FUSED': '1', 'LT_MARG_UNITS': '',
                                     'LT_FUSED_MARG': '' if m == '0' else m}))
  for name, env in runs:
    os.environ.update(env)
    t = timeit(lambda: step(W, nf, lab, nl, V, n, g1, ws))
    bw = 15756 * B * T / (t * 1e-3) / 1e12  # SURVEY 8d step bytes (bench hbm_frac_step)
    print(f'{name}: {t:.3f} ms  {cells / (t * 1e-3):.3e} cells/s  {bw:.2f} TB/s '
          f'({bw / 8 * 100:.1f} % of 8 TB/s)', flush=True)


if __name__ == '__main__':
  main()
