"""Child of tests/test_gpu_diag.py: the quad trigram recursions (lt_tri4.hip,
diagnostic build, LT_TRI4=1) against the oracle -- V = 32 trigram, bf16 and
fp32, utterances of 0, 1, 2, T-1 and T frames, loss and dW under the
per-element marginal bound. Prints 'ok' on success."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from last_torch_amd import _native as nat  # noqa: E402
from golden_cases import assert_loss_close, assert_grad_marginal_close  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (test infrastructure only)


def main():
  assert os.environ.get('LT_TRI4') == '1'
  dev = torch.device('cuda', 0)
  B, T, U, V, n = 5, 24, 6, 32, 2
  rng = np.random.default_rng(4242)
  C = nat.num_context_states(V, n)
  for bf16 in (True, False):
    W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
    lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
    nf = np.array([T, 0, 1, 2, T - 1], dtype=np.int32)
    nl = np.array([U, 0, 1, 2, U - 1], dtype=np.int32)
    if bf16:
      W = torch.tensor(W).bfloat16().float().numpy()
    Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(dev)
    nfd, labd, nld = (torch.tensor(x).to(dev) for x in (nf, lab, nl))
    out = nat.loss_forward(Wd, nfd, labd, nld, V, n, False, checkpoints=True)
    dW = nat.loss_backward(Wd, nfd, labd, nld, *out[1:5], None, V, n, False, ck=out[5])
    rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
    assert_loss_close(out[0].cpu().numpy(), rl)
    assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, orc.den_grad(W, nf, V, n)[1], rlz,
                               rnum, bf16)
  print('ok')


if __name__ == '__main__':
  main()
