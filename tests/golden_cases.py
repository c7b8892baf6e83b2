"""Loader for the golden fixtures written by tests/golden/make_golden.py."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
LATTICE_CASES = sorted(
    os.path.basename(p)[len('lattice_'):-len('.npz')]
    for p in glob.glob(os.path.join(GOLDEN, 'lattice_*.npz')))
SEMIRINGS = ('Log', 'MaxTropical', 'Real')
FLD_CASES = sorted(
    os.path.basename(p)[len('fld_'):-len('.npz')]
    for p in glob.glob(os.path.join(GOLDEN, 'fld_*.npz')))


def load(name):
  with np.load(os.path.join(GOLDEN, f'lattice_{name}.npz')) as d:
    c = {k: d[k] for k in d.files}
  c['V'] = int(c.pop('vocab_size'))
  c['n'] = int(c.pop('context_size'))
  c['bf16'] = bool(c['bf16'])
  return c


def load_fld(name):
  """FrameLabelDependent(K) fixtures (tests/golden/make_golden_fld.py)."""
  with np.load(os.path.join(GOLDEN, f'fld_{name}.npz')) as d:
    c = {k: d[k] for k in d.files}
  c['V'] = int(c.pop('vocab_size'))
  c['n'] = int(c.pop('context_size'))
  c['K'] = int(c['K'])
  return c


def load_npz(stem):
  with np.load(os.path.join(GOLDEN, f'{stem}.npz')) as d:
    return {k: d[k] for k in d.files}


def loss_tol(ref):
  """|got - ref| <= 1e-4 * max(1, |ref|) (BASELINE north_star tolerance)."""
  return 1e-4 * np.maximum(1.0, np.abs(ref))


def assert_loss_close(got, ref):
  got = np.asarray(got, np.float64)
  ref = np.asarray(ref, np.float64)
  fin = np.isfinite(ref)
  np.testing.assert_array_equal(np.isfinite(got), fin)
  np.testing.assert_array_equal(got[~fin], ref[~fin])
  err = np.abs(got[fin] - ref[fin])
  assert (err <= loss_tol(ref[fin])).all(), (got, ref, err)


def assert_values_close(got, ref, rtol=1e-5, atol=1e-5):
  got = np.asarray(got, np.float64)
  ref = np.asarray(ref, np.float64)
  np.testing.assert_array_equal(np.isneginf(got), np.isneginf(ref))
  np.testing.assert_array_equal(np.isposinf(got), np.isposinf(ref))
  fin = np.isfinite(ref)
  np.testing.assert_allclose(got[fin], ref[fin], rtol=rtol, atol=atol)


def marginal_scale(ref, den, log_z, num, bf16=False):
  """Per-element tolerance of a loss gradient dW = g (den - num) against a
  float64 reference: 1e-8 + (1e-4 + 4 * 2^-24 * max(1, |log_z_b|, |num_b|))
  * (den + num), den / num the arc's denominator / numerator marginals
  (alignments.py:300-318: exp(alpha + w + beta - log_z)). Each marginal is an
  exponential of an fp32 log-space sum of terms of magnitude ~|log_z| (or
  |num|), so its rounding is relative to the marginal itself, not absolute:
  an arc whose marginals are 1e-6 is checked to ~1e-9. `den` None: a locally
  normalised loss (no denominator; num = -ref). bf16 dW adds its own
  rounding, 2^-8 (den + num)."""
  ref = np.asarray(ref, np.float64)
  if den is None:
    den = np.zeros_like(ref)
    nm = -ref
  else:
    den = np.asarray(den, np.float64)
    nm = den - ref
  nm = np.maximum(nm, 0.0)
  mag = np.maximum(1.0, np.abs(np.where(np.isfinite(log_z), log_z, 0.0)))
  if num is not None:
    mag = np.maximum(mag, np.abs(np.where(np.isfinite(num), num, 0.0)))
  rel = 1e-4 + 4 * 2.0 ** -24 * mag.astype(np.float64) + (2.0 ** -8 if bf16 else 0.0)
  return 1e-8 + rel.reshape([-1] + [1] * (ref.ndim - 1)) * (den + nm)


def grad_error_ratio(got, ref, den, log_z, num, bf16=False, weights=None):
  """|got - ref| / marginal_scale: <= 1 everywhere passes. `weights` [B]:
  got is the gradient of sum_b weights_b * loss_b, so ref and the bound are
  both scaled by weights_b (a zero weight demands an exact zero)."""
  got = np.asarray(got, np.float64)
  ref = np.asarray(ref, np.float64)
  scale = marginal_scale(ref, den, log_z, num, bf16)
  if weights is not None:
    w = np.asarray(weights, np.float64).reshape([-1] + [1] * (ref.ndim - 1))
    ref = ref * w
    scale = scale * np.abs(w) + np.where(w == 0, 0.0, 1e-12)
    with np.errstate(divide='ignore', invalid='ignore'):
      r = np.abs(got - ref) / scale
    return np.where((w == 0) & (got == 0), 0.0, np.where(w == 0, np.inf, r))
  return np.abs(got - ref) / scale


def assert_grad_marginal_close(got, ref, den, log_z, num, bf16=False, weights=None):
  """Every dW element within marginal_scale (relative to its own marginals),
  plus the absolute check of assert_grad_close as a secondary bound. `den`
  the arc's denominator marginals (the oracle's den_grad; None for a locally
  normalised loss); for a denominator-only gradient (d log_z / dW) pass
  ref = den and num = None. `weights`: see grad_error_ratio."""
  r = grad_error_ratio(got, ref, den, log_z, num, bf16, weights)
  bad = ~(r <= 1.0)
  assert not bad.any(), (f'{int(bad.sum())} of {bad.size} dW elements beyond the marginal bound; '
                         f'worst ratio {float(np.nanmax(r)):.3g} at '
                         f'{np.argwhere(bad)[0].tolist()}')
  if weights is None:
    assert_grad_close(got, ref, log_z, bf16=bf16, num=num)
  else:
    w = np.asarray(weights, np.float64)
    assert_grad_close(got, np.asarray(ref, np.float64) * w.reshape([-1] + [1] * (np.ndim(ref) - 1)),
                      np.asarray(log_z, np.float64) * np.maximum(np.abs(w), 1e-30), bf16=bf16,
                      num=None if num is None else np.asarray(num, np.float64) * np.abs(w))


def table_den_marginals(orc, table, W, nf, lab, nl, K):
  """Denominator arc marginals d log_z / dW of a table lattice from the
  pinned table oracle (tab_den_grad; the string arguments are not used).
  Test infrastructure."""
  del lab, nl
  return orc.tab_den_grad(table, W, nf, K)[1].astype(np.float64)


def assert_grad_close(got, ref, log_z, bf16=False, num=None):
  """Arc-marginal gradients: per utterance b,
  |got - ref| <= 1e-5 + 1e-6 * max(1, |log_z_b|, |num_b|) (+ 8e-3 relative
  for bf16 dW). The fp32 log-space arguments alpha + w + beta - log_z (and
  the numerator's alpha_num + w + beta_num - num) are sums of terms of
  magnitude ~|log_z| (~|num|), each rounded at that magnitude * 2^-24, so a
  marginal near 1 carries an absolute error proportional to it (the
  reference, which runs in fp32, carries the same); the float64 fixtures are
  exact. With locally normalised weights log_z is ~0 while |num| is not."""
  got = np.asarray(got, np.float64)
  ref = np.asarray(ref, np.float64)
  lz = np.abs(np.where(np.isfinite(log_z), log_z, 0.0)).astype(np.float64)
  if num is not None:
    lz = np.maximum(lz, np.abs(np.where(np.isfinite(num), num, 0.0)).astype(np.float64))
  atol = 1e-5 + 1e-6 * np.maximum(1.0, lz)
  tol = atol.reshape([-1] + [1] * (ref.ndim - 1)) + (8e-3 if bf16 else 1e-4) * np.abs(ref)
  err = np.abs(got - ref)
  bad = err > tol
  assert not bad.any(), (f'{int(bad.sum())} of {bad.size} beyond tolerance; '
                         f'max err {float(err.max()):.3g} at {np.argwhere(bad)[0].tolist()}')
