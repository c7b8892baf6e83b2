"""Per-frame cycle breakdown from the diagnostic (-DLT_STAMPS) library (dev tool, GPU)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat
nat.LIB_PATH = os.path.join(ROOT, 'build', 'stamps', 'liblt_lattice_stamps.so')

def report(name, st, T):
  st = st.reshape(3, T, 4).astype(np.int64)
  for r, rn in enumerate(['den', 'aux', 'load']):
    s = st[r]
    if not s[:, 0].any():
      continue
    v = slice(10, T - 10)
    wait = (s[v, 1] - s[v, 0])
    work = (s[v, 2] - s[v, 1])
    step = np.diff(s[:, 0])[10:T - 11]
    extra = ''
    if s[v, 3].any():
      extra = f'  store part med {np.median(s[v, 3] - s[v, 1]):7.0f}'
    print(f'{name:12s} {rn:5s} step med {np.median(step):7.0f}  wait+barrier med {np.median(wait):7.0f}  '
          f'work med {np.median(work):7.0f}{extra}  (cycles)', flush=True)

def main():
  B = int(os.environ.get('B', 64)); T, U, V, n = 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn(B, T, C, V + 1, device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  st = torch.zeros(3 * T * 4, dtype=torch.int64, device='cuda')
  os.environ['LT_STAMPS_PTR'] = str(st.data_ptr())
  loss, lz, num, al, an = nat.loss_forward(W, nf, lab, nl, V, n, False)
  g = torch.ones(B, device='cuda')
  for dbg, lanes, aux, mx in [(0, None, '0', '5')]:
    os.environ['LT_BWD_AUX'] = aux; os.environ['LT_MAX_DEN_WAVES'] = mx
    os.environ['LT_DBG'] = str(dbg)
    if lanes: os.environ['LT_DEN_LANES'] = lanes
    else: os.environ.pop('LT_DEN_LANES', None)
    for name, fn in [('loss_fwd', lambda: nat.loss_forward(W, nf, lab, nl, V, n, False)),
                     ('loss_bwd', lambda: nat.loss_backward(W, nf, lab, nl, lz, num, al, an, g, V, n, False))]:
      st.zero_(); fn(); fn(); torch.cuda.synchronize()
      report(f'{name} d{dbg} L{lanes} aux{aux} mx{mx}', st.cpu().numpy(), T)
  os.environ.pop('LT_DEN_LANES', None)
  # clock estimate: s_memtime vs wall for one kernel
  os.environ['LT_DBG'] = '0'
  st.zero_(); torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record(); nat.den_forward(W, nf, V, n, 0, want_alpha=True); e1.record(); torch.cuda.synchronize()
  s = st.cpu().numpy().reshape(3, T, 4)
  cyc = s[0, T - 1, 0] - s[0, 0, 0]
  print('clock est GHz', cyc / (e0.elapsed_time(e1) * 1e-3) / 1e9, 'kernel ms', e0.elapsed_time(e1))

if __name__ == "__main__":
  main()
