"""GPU gradients of the string distance (RecognitionLattice._string_forward
under autograd, lattices.py:250-377) and of the denominator distance
(_forward, :379-496) in MaxTropical and Real, against:

* the reference's own autograd (tests/golden/grads_*.npz, make_golden_grads.py)
  on the inputs of every FrameDependent and FrameLabelDependent fixture --
  MaxTropical bit-exact (one-hot paths with the tie rules of
  semirings.py:354-401), Real at rtol 1e-4 plus 1e-5 of the utterance's
  largest element (the reference computes Real in fp32);
* the pinned C oracle (table_oracle.c tab_dist_grad, itself checked against
  those fixtures by tests/test_oracle_grads.py) on random problems beyond the
  fixtures' sizes: bigram V=32 at T=300, random next-state tables,
  FrameLabelDependent(K), bf16 arc weights, epsilon labels, unreachable
  strings, num_labels = 0, zero-length utterances.

The kernels: lt_table_num_backward (strings, any next-state table; FullNGram
through its next_state_table()), lt_viterbi arcs (FullNGram den MaxTropical),
lt_table_den_backward (den Real, and MaxTropical on tables).
"""
import os
import zlib

import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat
from golden_cases import GOLDEN

pytestmark = pytest.mark.gpu

CASES = sorted(f[len('grads_'):-4] for f in os.listdir(GOLDEN) if f.startswith('grads_'))


def _orc():
  from oracle import oracle as orc  # test infrastructure only
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


def _lattice(context, K, table):
  align = lt.alignments.FrameDependent() if K == 0 else lt.alignments.FrameLabelDependent(K)
  return lt.RecognitionLattice(
      context=context, alignment=align,
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))


def _frames(B, T, device):
  return torch.arange(T, dtype=torch.float32, device=device)[None, :, None].expand(B, T, 1)


def _grad(lat, which, semiring, B, T, nf, lab, nl, device, table, weights=None):
  table.grad = None
  frames = _frames(B, T, device)
  if which == 'den':
    d, _ = lat._forward(None, frames, nf, semiring)
  else:
    d = lat._string_forward(None, frames, nf, lab, nl, semiring)
  w = torch.ones_like(d) if weights is None else weights
  (w * d).sum().backward()
  return d.detach().cpu().numpy(), table.grad.float().cpu().numpy()


@pytest.mark.parametrize('name', CASES)
@pytest.mark.parametrize('which', ['den', 'num'])
def test_semiring_grads_match_reference_autograd(cuda, name, which):
  """_forward / _string_forward gradients in MaxTropical and Real on ROCm
  tensors = the reference's own autograd on the same fixture."""
  d = _load(name)
  V, n, K = int(d['vocab_size']), int(d['context_size']), d['K']
  B, T = d['W'].shape[:2]
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  table = torch.tensor(d['W'], device=cuda, requires_grad=True)
  lat = _lattice(ctx, K, table)
  nf = torch.tensor(d['num_frames'])
  lab, nl = torch.tensor(d['labels']), torch.tensor(d['num_labels'])
  for sname in ('MaxTropical', 'Real'):
    s = getattr(lt.semirings, sname)
    dist, g = _grad(lat, which, s, B, T, nf, lab, nl, cuda, table)
    ref = d[f'{which}_grad_{sname}']
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(dist, d[f'{which}_MaxTropical'])
      np.testing.assert_array_equal(g, ref)
    else:
      assert_real_grad_close(g, ref)


def _random_problem(rng, B, T, U, C, V, table=None, scale=1.0, epsilon=False):
  W = (scale * rng.standard_normal((B, T, C, V + 1))).astype(np.float32)
  nf = rng.integers(0, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(0 if epsilon else 1, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(0, U + 1, B).astype(np.int32)
  nl[0] = U
  return W, nf, lab, nl


RANDOM = [
    # name, V, n (FullNGram) or None (random table with C states), C, K, B, T, U, dtype, scale
    ('bigram_v32_t300', 32, 1, None, 0, 4, 300, 40, 'f32', 1.0),
    ('bigram_v32_bf16', 32, 1, None, 0, 3, 120, 25, 'bf16', 1.0),
    ('trigram_v4', 4, 2, None, 0, 3, 60, 12, 'f32', 1.0),
    ('dfa_c23_k0', 9, None, 23, 0, 3, 50, 10, 'f32', 1.0),
    ('dfa_c23_k3', 9, None, 23, 3, 3, 40, 10, 'f32', 1.0),
    ('fld_k2_bigram_v5_bf16', 5, 1, None, 2, 3, 30, 12, 'bf16', 1.0),
    ('unigram_v6_k1', 6, 0, None, 1, 2, 25, 9, 'f32', 1.0),
]


@pytest.mark.parametrize('case', RANDOM, ids=[c[0] for c in RANDOM])
@pytest.mark.parametrize('epsilon', [False, True])
def test_semiring_grads_random_against_oracle(cuda, case, epsilon):
  """Random problems past the fixtures' sizes against the pinned oracle:
  MaxTropical bit-exact (distance and one-hot arcs, scaled by an incoming
  gradient), Real within the Real bound (weights scaled so that alpha stays
  inside fp32 over the utterance)."""
  name, V, n, C, K, B, T, U, dt, _ = case
  orc = _orc()
  rng = np.random.default_rng(zlib.crc32(f'{name}-{epsilon}'.encode()))
  if n is not None:
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    tab = orc.full_ngram_table(V, n)
    C = tab.shape[0]
  else:
    tab = rng.integers(0, C, (C, V)).astype(np.int32)
    ctx = lt.contexts.NextStateTable(torch.tensor(tab))
  W, nf, lab, nl = _random_problem(rng, B, T, U, C, V, epsilon=epsilon)
  if dt == 'bf16':
    W = torch.tensor(W).bfloat16().float().numpy()
  tdtype = torch.bfloat16 if dt == 'bf16' else torch.float32
  gin = np.linspace(0.5, 2.0, B).astype(np.float32)
  for which in ('num', 'den'):
    kw = dict(labels=lab, num_labels=nl) if which == 'num' else {}
    # MaxTropical
    table = torch.tensor(W, device=cuda, dtype=tdtype, requires_grad=True)
    lat = _lattice(ctx, K, table)
    dist, g = _grad(lat, which, lt.semirings.MaxTropical, B, T, torch.tensor(nf), torch.tensor(lab),
                    torch.tensor(nl), cuda, table, torch.tensor(gin, device=cuda))
    rd, rg = orc.tab_dist_grad(tab, W, nf, K, orc.MAX, grad=gin, **kw)
    np.testing.assert_array_equal(dist, rd)
    np.testing.assert_array_equal(g, rg)
    # Real: products of weights over the utterance, so only a short stretch
    # stays inside fp32 (the reference's Real semiring is plain fp32
    # arithmetic too): 12 frames of weights near 1 / (arcs per state)
    Tr = min(T, 12)
    nfr = np.minimum(nf, Tr).astype(np.int32)
    Wr = (np.exp(W[:, :Tr] - np.log(V + 1.0)) * 1.3).astype(np.float32)
    if dt == 'bf16':
      Wr = torch.tensor(Wr).bfloat16().float().numpy()
    table = torch.tensor(Wr, device=cuda, dtype=tdtype, requires_grad=True)
    lat = _lattice(ctx, K, table)
    dist, g = _grad(lat, which, lt.semirings.Real, B, Tr, torch.tensor(nfr), torch.tensor(lab),
                    torch.tensor(nl), cuda, table, torch.tensor(gin, device=cuda))
    rd, rg = orc.tab_dist_grad(tab, Wr, nfr, K, orc.REAL, grad=gin, **kw)
    assert np.isfinite(rd).all() and np.isfinite(rg).all()
    np.testing.assert_allclose(dist, rd, rtol=1e-4, atol=1e-30)
    if dt == 'bf16':  # dW rounded to bf16: 2^-8 relative
      np.testing.assert_allclose(g, rg, rtol=2 ** -8 + 1e-4, atol=1e-30)
    else:
      assert_real_grad_close(g, rg)


def test_string_grad_edge_cases(cuda):
  """num_labels = 0 (a gradient along the all-blank path of position 0),
  unreachable strings (num_labels beyond what the frames allow: no
  gradient in MaxTropical, zero in Real), num_labels > U, zero-length
  utterances, a fully masked utterance, all against the oracle."""
  orc = _orc()
  V, n, T, U, B = 4, 1, 6, 5, 6
  rng = np.random.default_rng(5)
  tab = orc.full_ngram_table(V, n)
  C = tab.shape[0]
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  W[4] = -np.inf
  nf = np.array([6, 3, 0, 6, 6, 2], np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = np.array([0, 5, 0, 7, 2, 0], np.int32)  # 1: 5 labels in 3 frames; 3: beyond U
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  for sname, sr in (('MaxTropical', orc.MAX), ('Real', orc.REAL)):
    Wx = W if sname == 'MaxTropical' else np.nan_to_num(np.exp(W), neginf=0.0).astype(np.float32)
    table = torch.tensor(Wx, device=cuda, requires_grad=True)
    lat = _lattice(ctx, 0, table)
    dist, g = _grad(lat, 'num', getattr(lt.semirings, sname), B, T, torch.tensor(nf),
                    torch.tensor(lab), torch.tensor(nl), cuda, table)
    rd, rg = orc.tab_dist_grad(tab, Wx, nf, 0, sr, lab, nl)
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(dist, rd)
      np.testing.assert_array_equal(g, rg)
      assert g[1].sum() == 0 and g[3].sum() == 0   # unreachable / beyond U
      assert g[0].sum() == nf[0] and g[5].sum() == nf[5]  # position 0's blanks
    else:
      np.testing.assert_allclose(dist, rd, rtol=1e-5)
      assert_real_grad_close(g, rg)


def test_den_max_fully_masked_utterance_follows_reference_ties(cuda):
  """An utterance of -inf MaxTropical distance (every arc masked) still
  gets the first maximum's path -- the all-blank path from state 0, as the
  reference's argmax backward gives it -- on the tuned FullNGram path
  (lt_viterbi arcs) and the table path (lt_table_den_backward) alike."""
  orc = _orc()
  V, n, T, B = 3, 1, 5, 2
  rng = np.random.default_rng(9)
  tab = orc.full_ngram_table(V, n)
  W = rng.standard_normal((B, T, tab.shape[0], V + 1)).astype(np.float32)
  W[1] = -np.inf
  nf = np.array([5, 4], np.int32)
  _, rg = orc.tab_dist_grad(tab, W, nf, 0, orc.MAX)
  assert rg[1, :4, 0, 0].sum() == 4 and rg[1].sum() == 4
  for ctx in (lt.contexts.FullNGram(vocab_size=V, context_size=n),
              lt.contexts.NextStateTable(torch.tensor(tab))):
    table = torch.tensor(W, device=cuda, requires_grad=True)
    _, g = _grad(_lattice(ctx, 0, table), 'den', lt.semirings.MaxTropical, B, T,
                 torch.tensor(nf), None, None, cuda, table)
    np.testing.assert_array_equal(g, rg)
