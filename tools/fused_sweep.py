"""Dev tool (GPU): timing sweep of the fused loss+grad (marginal workgroup
count, frames per wave) and of its parts (pipe alone at the fused LDS cap)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402
from fused_check import ref, timeit  # noqa: E402


def main():
  B, T, U, V, n = int(os.environ.get('B', 64)), 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  ws = torch.empty([1 << 30], dtype=torch.uint8, device='cuda')
  print(f'separate fwd+bwd: {timeit(lambda: ref(W, nf, lab, nl, V, n, False)):.3f} ms', flush=True)
  for lds in ('', '81920'):
    os.environ['LT_PIPE_LDS'] = lds
    t = timeit(lambda: nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True))
    print(f'pipe alone LDS={lds or "default"}: {t:.3f} ms', flush=True)
  os.environ['LT_PIPE_LDS'] = ''
  for fl in os.environ.get('FLDS', '').split(','):
    os.environ['LT_FUSED_LDS'] = fl
    for marg in os.environ.get('MARG1', '128').split(','):
      os.environ['LT_FUSED_MARG'] = marg
      t = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws))
      print(f'fused LDS={fl or "default"} marg={marg}: {t:.3f} ms', flush=True)
  os.environ['LT_FUSED_LDS'] = ''
  for dbg in os.environ.get('DBGS', '0').split(','):
    os.environ['LT_PIPE_DBG'] = dbg
    t = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws))
    print(f'fused dbg={dbg}: {t:.3f} ms', flush=True)
  os.environ['LT_PIPE_DBG'] = '0'
  for fw in os.environ.get('FWS', '4').split(','):
    os.environ['LT_FUSED_FW'] = fw
    for marg in os.environ.get('MARG', '64,128,256,384').split(','):
      os.environ['LT_FUSED_MARG'] = marg
      t = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws))
      print(f'fused FW={fw} marg={marg}: {t:.3f} ms', flush=True)


if __name__ == '__main__':
  main()
