"""The RecognitionLattice API surface on the HIP kernels (the CPU twin is
tests/test_lattice_api.py): the ``_backward`` callback, gradients through
``_forward``, and the autograd contract of ``forward`` (dW from the
forward's lt_loss_grad, scaled by the incoming gradient; a second backward
with retain_graph)."""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat
from golden_cases import assert_grad_marginal_close, assert_loss_close, load
from test_lattice_api import (CASES, check_backward_callback, check_backward_vjp,
                              check_forward_gradients)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('case', CASES)
def test_backward_callback_gpu(cuda, case):
  check_backward_callback(load(case), cuda)


def test_backward_weight_vjp_gpu(cuda):
  check_backward_vjp(cuda)


@pytest.mark.parametrize('case', CASES)
def test_forward_gradients_gpu(cuda, case):
  check_forward_gradients(load(case), cuda)


@pytest.mark.parametrize('V,n', [(32, 1), (3, 2)])
def test_loss_autograd_contract(cuda, V, n):
  """forward is one lt_loss_grad call (loss and dW together, the design the
  shape picks); the backward scales dW by the incoming gradient; a second
  backward (retain_graph) recomputes it and gives the same gradient."""
  from oracle import oracle as orc  # test infrastructure only
  rng = np.random.default_rng(3)
  B, T, U = 5, 40, 6
  C = nat.num_context_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = np.array([40, 33, 17, 40, 1], np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = np.array([6, 4, 2, 6, 0], np.int32)
  table = torch.tensor(W, device=cuda, requires_grad=True)
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.arange(T, dtype=torch.float32, device=cuda)[None, :, None].expand(B, T, 1)
  loss = lat(frames, torch.tensor(nf), torch.tensor(lab), torch.tensor(nl))
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  assert_loss_close(loss.detach().cpu().numpy(), rl)
  w = torch.linspace(-1.0, 2.0, B, device=cuda)
  (w * loss).sum().backward(retain_graph=True)
  g1 = table.grad.clone()
  den = orc.den_grad(W, nf, V, n)[1]
  assert_grad_marginal_close(g1.cpu().numpy(), rdW, den, rlz, rnum, weights=w.cpu().numpy())
  table.grad = None
  (w * loss).sum().backward()
  assert torch.equal(table.grad, g1)
