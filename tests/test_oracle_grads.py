"""The C oracle's MaxTropical and Real distance gradients (table_oracle.c
tab_dist_grad) against the reference's own autograd (tests/golden/grads_*.npz,
made by make_golden_grads.py from the reference): _forward (den) and
_string_forward (num), FrameDependent and FrameLabelDependent(K), on the
inputs of every lattice / FLD fixture.

MaxTropical gradients are one-hot path indicators with the reference's tie
rules (semirings.py:354-401): exact. Real gradients (alpha * beta',
semirings.py:143-173): the reference computes them in fp32 and the oracle
in double, compared at rtol 1e-4 plus 1e-5 of the utterance's largest
element (randn Real weights cancel).
"""
import os

import numpy as np
import pytest

from golden_cases import GOLDEN

CASES = sorted(f[len('grads_'):-4] for f in os.listdir(GOLDEN) if f.startswith('grads_'))


def _orc():
  from oracle import oracle as orc
  return orc


def _load(name):
  with np.load(os.path.join(GOLDEN, name + '.npz')) as z:
    d = {k: z[k] for k in z.files}
  with np.load(os.path.join(GOLDEN, 'grads_' + name + '.npz')) as z:
    d.update({k: z[k] for k in z.files})
  d['K'] = int(d['K']) if 'K' in d else 0
  return d


def assert_real_grad_close(got, ref):
  """rtol 1e-4 plus 1e-5 of each utterance's largest |element|."""
  got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
  assert np.isfinite(ref).all() and np.isfinite(got).all()
  scale = np.abs(ref).reshape(ref.shape[0], -1).max(-1)
  tol = 1e-4 * np.abs(ref) + 1e-5 * scale.reshape(-1, *([1] * (ref.ndim - 1))) + 1e-30
  bad = np.abs(got - ref) > tol
  assert not bad.any(), (int(bad.sum()), float((np.abs(got - ref) / tol).max()))


def test_cases_present():
  assert len(CASES) >= 20


@pytest.mark.parametrize('name', CASES)
@pytest.mark.parametrize('which', ['den', 'num'])
def test_oracle_semiring_grads_match_reference(name, which):
  d = _load(name)
  orc = _orc()
  V, n, K = int(d['vocab_size']), int(d['context_size']), d['K']
  table = orc.full_ngram_table(V, n)
  kw = dict(labels=d['labels'], num_labels=d['num_labels']) if which == 'num' else {}
  for sname, sr in (('MaxTropical', orc.MAX), ('Real', orc.REAL)):
    dist, g = orc.tab_dist_grad(table, d['W'], d['num_frames'], K, sr, **kw)
    ref = d[f'{which}_grad_{sname}']
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(dist, d[f'{which}_MaxTropical'])
      np.testing.assert_array_equal(g, ref)
    else:
      np.testing.assert_allclose(dist, d[f'{which}_Real'], rtol=1e-4,
                                 atol=1e-5 * max(1.0, float(np.abs(d[f'{which}_Real']).max())))
      assert_real_grad_close(g, ref)


def test_oracle_grads_scale_with_incoming_gradient():
  d = _load('lattice_bigram_v5')
  orc = _orc()
  table = orc.full_ngram_table(5, 1)
  g = np.array([2.0, -0.5], np.float32)
  for sr in (orc.MAX, orc.REAL, orc.LOG):
    _, a = orc.tab_dist_grad(table, d['W'], d['num_frames'], 0, sr, d['labels'], d['num_labels'])
    _, b = orc.tab_dist_grad(table, d['W'], d['num_frames'], 0, sr, d['labels'], d['num_labels'],
                             grad=g)
    np.testing.assert_allclose(b, a * g[:, None, None, None], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('name', ['lattice_bigram_v5', 'lattice_epsilon_labels', 'fld_k2_epsilon'])
def test_oracle_log_grads_match_fixture_marginals(name):
  """tab_dist_grad in Log: the den marginals (den_grad) and, for the string,
  the num marginals the loss fixtures imply (den_grad - loss_grad)."""
  d = _load(name)
  orc = _orc()
  V, n, K = int(d['vocab_size']), int(d['context_size']), d['K']
  table = orc.full_ngram_table(V, n)
  _, g = orc.tab_dist_grad(table, d['W'], d['num_frames'], K, orc.LOG)
  np.testing.assert_allclose(g, d['den_grad'], rtol=1e-4, atol=1e-6)
  _, gn = orc.tab_dist_grad(table, d['W'], d['num_frames'], K, orc.LOG, d['labels'],
                            d['num_labels'])
  reach = np.isfinite(d['loss'])[:, None, None, None]
  np.testing.assert_allclose(np.where(reach, gn, 0), np.where(reach, d['den_grad'] - d['loss_grad'], 0),
                             rtol=1e-4, atol=1e-5)
