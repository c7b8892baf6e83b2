"""Pins the table oracle (oracle/table_oracle.c: any next-state table,
FrameDependent or FrameLabelDependent(K)) to the reference. CPU only.

* FrameLabelDependent(K): fixtures made by the reference itself
  (tests/golden/make_golden_fld.py).
* Next-state tables: FullNGram.next_state_table() (contexts.py:258-263) run
  through the table oracle must reproduce every FullNGram fixture, and it
  is bit-identical to the pinned FullNGram oracle. (The reference's
  NextStateTable.forward_reduce is defective, D8, so other tables have no
  reference output: their results are checked for the equivalence below
  and, on the GPU, against this oracle.)
"""
import numpy as np
import pytest

from golden_cases import (FLD_CASES, LATTICE_CASES, SEMIRINGS, assert_grad_close,
                          assert_grad_marginal_close, assert_loss_close, assert_values_close, load,
                          load_fld)
from oracle import oracle as orc

SID = {'Log': orc.LOG, 'MaxTropical': orc.MAX, 'Real': orc.REAL}


def _real_tol(ref):
  return dict(rtol=2e-5, atol=1e-5 * max(1.0, float(np.abs(ref[np.isfinite(ref)]).max(initial=0))))


@pytest.mark.parametrize('case', FLD_CASES)
@pytest.mark.parametrize('semiring', SEMIRINGS)
def test_fld_den_forward(case, semiring):
  c = load_fld(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  d, a = orc.tab_den_forward(tab, c['W'], c['num_frames'], c['K'], SID[semiring],
                             want_alpha=True)
  ref_d, ref_a = c[f'den_{semiring}'], c[f'alpha_{semiring}']
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(d, ref_d)
    np.testing.assert_array_equal(a, ref_a)
  elif semiring == 'Real':
    assert_values_close(d, ref_d, **_real_tol(ref_d))
  else:
    assert_values_close(d, ref_d)
    assert_values_close(a, ref_a)


@pytest.mark.parametrize('case', FLD_CASES)
@pytest.mark.parametrize('semiring', SEMIRINGS)
def test_fld_num_forward(case, semiring):
  c = load_fld(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  num = orc.tab_num_forward(tab, c['W'], c['num_frames'], c['labels'], c['num_labels'], c['K'],
                            SID[semiring])
  ref = c[f'num_{semiring}']
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(num, ref)
  elif semiring == 'Real':
    assert_values_close(num, ref, **_real_tol(ref))
  else:
    assert_loss_close(num, ref)


@pytest.mark.parametrize('case', FLD_CASES)
def test_fld_loss_and_grad(case):
  c = load_fld(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  loss, lz, _, dW = orc.tab_loss_grad(tab, c['W'], c['num_frames'], c['labels'],
                                      c['num_labels'], c['K'])
  assert_loss_close(loss, c['loss'])
  assert_loss_close(lz, c['den_Log'])
  assert_grad_close(dW, c['loss_grad'], c['den_Log'])


@pytest.mark.parametrize('case', FLD_CASES)
def test_fld_den_grad(case):
  """tab_den_grad (d log_z / dW alone) against the reference's den_grad
  (its FrameLabelDependent.backward composed in reverse frame order), every
  element within its marginal bound."""
  c = load_fld(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  lz, d = orc.tab_den_grad(tab, c['W'], c['num_frames'], c['K'])
  assert_loss_close(lz, c['den_Log'])
  assert_grad_marginal_close(d, c['den_grad'], c['den_grad'], c['den_Log'], None)


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_full_ngram_den_grad_through_table(case):
  c = load(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  W = c['W'].astype(np.float32)
  lz, d = orc.tab_den_grad(tab, W, c['num_frames'], 0)
  assert_loss_close(lz, c['den_Log'])
  assert_grad_marginal_close(d, c['den_grad'], c['den_grad'], c['den_Log'], None)


@pytest.mark.parametrize('case', FLD_CASES)
def test_fld_viterbi(case):
  """Path weight = the reference's MaxTropical distance; labels keep the
  reference test's invariants (tests/lattices_test.py:145-176): A = K+1
  slots per frame, the last slot always blank, labels in [0, V], padding
  frames blank; and re-summing the decoded path's arcs gives the weight."""
  c = load_fld(case)
  V, K = c['V'], c['K']
  tab = orc.full_ngram_table(V, c['n'])
  W, nf = c['W'], c['num_frames']
  for conv in (0, 1):
    labels, w = orc.tab_viterbi(tab, W, nf, K, conv)
    np.testing.assert_array_equal(w, c['den_MaxTropical'])
    B, T = W.shape[:2]
    lab = labels.reshape(B, T, K + 1)
    assert (lab[..., K] == 0).all()
    assert (lab >= 0).all() and (lab <= V).all()
    for b in range(B):
      assert (lab[b, nf[b]:] == 0).all()
  # re-sum the path (true labels): start state 0, per frame the expansions
  # then the blank, in the reference's float32 operand order
  labels, w = orc.tab_viterbi(tab, W, nf, K, 0)
  lab = labels.reshape(W.shape[0], W.shape[1], K + 1)
  for b in range(W.shape[0]):
    q, s = 0, np.float32(0)
    for t in range(nf[b]):
      for y in lab[b, t, :K]:
        if y == 0:
          break
        s = np.float32(s + W[b, t, q, y])
        q = tab[q, y - 1]
      s = np.float32(s + W[b, t, q, 0])
    assert s == w[b], (b, s, w[b])


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_table_reproduces_full_ngram(case):
  """K = 0 with FullNGram.next_state_table(): the FullNGram fixtures."""
  c = load(case)
  tab = orc.full_ngram_table(c['V'], c['n'])
  for s in SEMIRINGS:
    d = orc.tab_den_forward(tab, c['W'], c['num_frames'], 0, SID[s])
    num = orc.tab_num_forward(tab, c['W'], c['num_frames'], c['labels'], c['num_labels'], 0,
                              SID[s])
    if s == 'MaxTropical':
      np.testing.assert_array_equal(d, c['den_MaxTropical'])
      np.testing.assert_array_equal(num, c['num_MaxTropical'])
    elif s == 'Log':
      assert_loss_close(d, c['den_Log'])
      assert_loss_close(num, c['num_Log'])
  loss, lz, _, dW = orc.tab_loss_grad(tab, c['W'], c['num_frames'], c['labels'],
                                      c['num_labels'], 0)
  assert_loss_close(loss, c['loss'])
  assert_grad_close(dW, c['loss_grad'], c['den_Log'], c['bf16'])
  labels, w = orc.tab_viterbi(tab, c['W'], c['num_frames'], 0, 1)
  np.testing.assert_array_equal(labels, c['vit_labels_reference'])
  np.testing.assert_array_equal(w, c['vit_weights'])


def test_table_matches_full_ngram_oracle_bitwise():
  rng = np.random.default_rng(0)
  for V, n in [(5, 1), (3, 2), (4, 0)]:
    C = orc.num_states(V, n)
    tab = orc.full_ngram_table(V, n)
    W = rng.standard_normal((3, 9, C, V + 1)).astype(np.float32)
    nf = np.array([9, 4, 0], np.int32)
    lab = rng.integers(0, V + 1, (3, 5)).astype(np.int32)
    nl = np.array([5, 2, 0], np.int32)
    r = orc.loss_grad(W, nf, lab, nl, V, n)
    t = orc.tab_loss_grad(tab, W, nf, lab, nl, 0)
    for x, y in zip(r, t):
      np.testing.assert_array_equal(x, y)


def test_random_table_properties():
  """An arbitrary DFA (next-state table with merges): loss >= 0,
  Real(exp W) == exp(Log W), and the denominator gradient equals a finite
  difference of log_z."""
  rng = np.random.default_rng(1)
  C, V, B, T, U = 7, 4, 3, 8, 4
  tab = rng.integers(0, C, (C, V)).astype(np.int32)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = np.array([8, 5, 1], np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = np.array([4, 2, 1], np.int32)
  for K in (0, 1, 2):
    loss, lz, num, dW = orc.tab_loss_grad(tab, W, nf, lab, nl, K)
    fin = np.isfinite(loss)
    assert (loss[fin] > -1e-4).all()
    dr = orc.tab_den_forward(tab, np.exp(W), nf, K, orc.REAL)  # Real on exp(W) = exp(Log)
    np.testing.assert_allclose(np.log(dr), lz, rtol=1e-5, atol=1e-5)
    eps = 1e-2
    Wp = W.copy()
    Wp[0, 2, 1, 2] += eps
    Wm = W.copy()
    Wm[0, 2, 1, 2] -= eps
    fd = (orc.tab_den_forward(tab, Wp, nf, K)[0] - orc.tab_den_forward(tab, Wm, nf, K)[0]) / (2 * eps)
    _, _, _, dd = orc.tab_loss_grad(tab, W, nf, lab, nl, K, local_norm=False)
    _, _, _, dn = orc.tab_loss_grad(tab, W, nf, lab, nl, K, local_norm=True)
    den_g = dd - dn  # (den - num) - (-num)
    np.testing.assert_allclose(den_g[0, 2, 1, 2], fd, rtol=2e-3, atol=2e-4)
