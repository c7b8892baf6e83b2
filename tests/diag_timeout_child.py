"""Child process of tests/test_gpu_diag.py (run with LT_LIB_PATH = the
diagnostic build and LT_CK_DBG=512): one chunked lt_loss_grad call whose
utterance 0 takes the hand-off timeout route. Checks that the route was taken
(the utterance's fallback word is set) and that every utterance's loss and
every dW element match the oracle. Prints 'ok'."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from golden_cases import assert_grad_marginal_close, assert_loss_close  # noqa: E402
from last_torch_amd import _native as nat  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (test infrastructure only)


def main():
  V, n, T, U, B = 32, 1, 240, 30, 4
  rng = np.random.default_rng(5)
  W = rng.standard_normal((B, T, V + 1, V + 1)).astype(np.float32)
  nf = np.array([240, 200, 240, 97], np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = np.array([30, 25, 30, 12], np.int32)
  dev = torch.device('cuda')
  Wd = torch.tensor(W, device=dev)
  nfd, labd, nld = (torch.tensor(x, device=dev) for x in (nf, lab, nl))
  assert nat.chunk_path(B, T, U, V, n)
  ws = torch.empty([nat.loss_grad_workspace_bytes(Wd, V, n, U, False)], dtype=torch.uint8,
                   device=dev)
  loss, lz, num, dW = nat.loss_grad(Wd, nfd, labd, nld, V, n, False, workspace=ws)
  torch.cuda.synchronize()
  fell = nat.chunk_fallback_count(ws, B)
  assert fell >= 1, 'the withheld chunk did not send utterance 0 to the frame-serial kernels'
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n, local_norm=False)
  den = orc.den_grad(W, nf, V, n)[1]
  assert_loss_close(loss.cpu().numpy(), rl)
  assert_loss_close(lz.cpu().numpy(), rlz)
  assert_loss_close(num.cpu().numpy(), rnum)
  assert_grad_marginal_close(dW.cpu().numpy(), rdW, den, rlz, rnum)
  print(f'ok: {fell} utterance(s) through the timeout route')


if __name__ == '__main__':
  main()
