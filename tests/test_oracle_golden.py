"""Pins the C oracle (oracle/lattice_oracle.c) to the reference.

Every fixture under tests/golden/ was produced by the reference itself
(tests/golden/make_golden.py); the oracle must reproduce all of it before
any GPU parity claim built on the oracle means anything. CPU only.
"""
import numpy as np
import pytest

from golden_cases import (LATTICE_CASES, SEMIRINGS, assert_loss_close, assert_values_close,
                          load)
from oracle import oracle as orc

SEMIRING_ID = {'Log': orc.LOG, 'MaxTropical': orc.MAX, 'Real': orc.REAL}


def _real_tol(ref):
  return dict(rtol=2e-5, atol=1e-5 * max(1.0, float(np.abs(ref[np.isfinite(ref)]).max(initial=0))))


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('semiring', SEMIRINGS)
def test_den_forward(case, semiring):
  c = load(case)
  dist, alpha = orc.den_forward(c['W'], c['num_frames'], c['V'], c['n'], SEMIRING_ID[semiring])
  ref_d, ref_a = c[f'den_{semiring}'], c[f'alpha_{semiring}']
  if semiring == 'MaxTropical':  # exact: max and + in the reference's operand order
    np.testing.assert_array_equal(dist, ref_d)
    np.testing.assert_array_equal(alpha, ref_a)
  elif semiring == 'Real':
    assert_values_close(dist, ref_d, **_real_tol(ref_d))
    assert_values_close(alpha, ref_a, **_real_tol(ref_a))
  else:
    assert_values_close(dist, ref_d)
    assert_values_close(alpha, ref_a)


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('semiring', SEMIRINGS)
def test_num_forward(case, semiring):
  c = load(case)
  num, _ = orc.num_forward(c['W'], c['num_frames'], c['labels'], c['num_labels'], c['V'], c['n'],
                           SEMIRING_ID[semiring])
  ref = c[f'num_{semiring}']
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(num, ref)
  elif semiring == 'Real':
    assert_values_close(num, ref, **_real_tol(ref))
  else:
    assert_values_close(num, ref)


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('local', [False, True])
def test_loss_and_grad(case, local):
  c = load(case)
  W = c['W_local'] if local else c['W']
  loss, _, _, dW = orc.loss_grad(W, c['num_frames'], c['labels'], c['num_labels'], c['V'],
                                 c['n'], local_norm=local)
  assert_loss_close(loss, c['loss_local' if local else 'loss'])
  np.testing.assert_allclose(dW, c['loss_local_grad' if local else 'loss_grad'], atol=2e-6,
                             rtol=1e-5)


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_den_grad(case):
  c = load(case)
  _, dW = orc.den_grad(c['W'], c['num_frames'], c['V'], c['n'])
  np.testing.assert_allclose(dW, c['den_grad'], atol=2e-6, rtol=1e-5)


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('convention', ['reference', 'true'])
def test_viterbi_bit_exact(case, convention):
  c = load(case)
  labels, weights, _ = orc.viterbi(c['W'], c['num_frames'], c['V'], c['n'],
                                   convention=1 if convention == 'reference' else 0)
  np.testing.assert_array_equal(labels, c[f'vit_labels_{convention}'])
  np.testing.assert_array_equal(weights, c['vit_weights'])


def test_kat_closed_forms():
  """The literal expectations of tests/lattices_test.py:209-288."""
  c = load('kat')
  lse = lambda xs: float(np.log(np.sum(np.exp(np.asarray(xs, np.float64)))))
  W, nf, V, n = c['W'], c['num_frames'], c['V'], c['n']
  np.testing.assert_array_equal(orc.den_forward(W, nf, V, n, orc.MAX)[0], [-3 + 18, 21, 0])
  np.testing.assert_allclose(
      orc.den_forward(W, nf, V, n, orc.REAL)[0],
      [-(10 + 11 + 12) - 2 * (13 + 14 + 15) - 3 * (16 + 17 + 18), 19 + 20 + 21, 1])
  log9 = lse([-1 + 10, -1 + 11, -1 + 12, -2 + 13, -2 + 14, -2 + 15, -3 + 16, -3 + 17, -3 + 18])
  np.testing.assert_allclose(orc.den_forward(W, nf, V, n, orc.LOG)[0],
                             [log9, lse([19, 20, 21]), 0], rtol=1e-6)
  labels, weights, _ = orc.viterbi(W, nf, V, n, convention=1)
  # lattices_test.py:238-242 pins [[1, 1], [0, 0], [0, 0]]: row 1 there is the
  # batched vjp's cross-utterance mask aliasing. Decoded one
  # utterance at a time the reference itself gives [1, 0] (fixture 'kat').
  np.testing.assert_array_equal(labels, [[1, 1], [1, 0], [0, 0]])
  np.testing.assert_array_equal(labels, c['vit_labels_reference'])
  np.testing.assert_array_equal(weights, [-3 + 18, 21, 0])
  lab, nl = c['labels'], c['num_labels']
  np.testing.assert_array_equal(orc.num_forward(W, nf, lab, nl, V, n, orc.MAX)[0],
                                [-2 + 13, 21, 0])
  np.testing.assert_allclose(orc.num_forward(W, nf, lab, nl, V, n, orc.REAL)[0],
                             [-11 - 2 * 13, 21, 1])
  num = lse([-1 + 11, -2 + 13])
  np.testing.assert_allclose(orc.num_forward(W, nf, lab, nl, V, n, orc.LOG)[0], [num, 21, 0],
                             rtol=1e-6)
  for s in (orc.LOG, orc.MAX):  # non-reachable num_labels -> semiring zero
    r = orc.num_forward(W, nf, lab, np.array([3, 2, 1], np.int32), V, n, s)[0]
    np.testing.assert_array_equal(r, [-np.inf] * 3)
  assert (orc.num_forward(W, nf, lab, np.array([3, 2, 1], np.int32), V, n, orc.REAL)[0] == 0).all()
  loss = orc.loss_grad(W, nf, lab, nl, V, n)[0]
  np.testing.assert_allclose(loss, [log9 - num, lse([19, 20, 21]) - 21, 0], rtol=1e-6)


def test_marginals_sum_to_one_per_frame():
  """Size-independent property of d log_z / dW: each live frame's arc
  marginals sum to 1, padding frames to 0."""
  rng = np.random.default_rng(5)
  V, n, B, T = 4, 2, 3, 9
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = np.array([9, 4, 0], np.int32)
  _, dW = orc.den_grad(W, nf, V, n)
  s = dW.reshape(B, T, -1).sum(-1)
  expect = (np.arange(T)[None, :] < nf[:, None]).astype(np.float64)
  np.testing.assert_allclose(s, expect, atol=1e-5)


def test_marginal_bound_negative_control():
  """The per-element dW bound (golden_cases.marginal_scale) at the bench
  shape: the oracle's own float32 dW of one B=1, T=1000, U=100 bigram
  utterance passes it; the same dW with every element below 4e-3 in
  magnitude zeroed (what round 2's absolute slack of ~1e-6 |log_z| let
  through) fails it, and so does a single low-probability arc off by 1e-6."""
  from golden_cases import assert_grad_marginal_close, grad_error_ratio, marginal_scale
  rng = np.random.default_rng(40)
  T, U, V, n = 1000, 100, 32, 1
  W = rng.standard_normal((1, T, V + 1, V + 1)).astype(np.float32)
  nf = np.array([T], np.int32)
  lab = rng.integers(1, V + 1, (1, U)).astype(np.int32)
  nl = np.array([U], np.int32)
  _, lz, num, dW = orc.loss_grad(W, nf, lab, nl, V, n)
  _, den = orc.den_grad(W, nf, V, n)
  assert abs(float(lz[0])) > 1000  # the regime where the absolute slack was ~4e-3
  assert_grad_marginal_close(dW, dW, den, lz, num)
  zeroed = np.where(np.abs(dW) < 4e-3, 0.0, dW).astype(np.float32)
  assert (zeroed != dW).mean() > 0.5
  with pytest.raises(AssertionError):
    assert_grad_marginal_close(zeroed, dW, den, lz, num)
  # one arc of tiny marginal perturbed by 1e-6
  scale = marginal_scale(dW, den, lz, num)
  i = np.unravel_index(np.argmin(scale), scale.shape)
  bumped = dW.copy()
  bumped[i] += 1e-6
  assert grad_error_ratio(bumped, dW, den, lz, num).max() > 1
  with pytest.raises(AssertionError):
    assert_grad_marginal_close(bumped, dW, den, lz, num)
  # the frame sums of the round-2 style absolute bound would not see it
  assert 1e-6 < 1e-5 + 1e-6 * abs(float(lz[0]))
