"""GPU gradients of the general lattices and of the Real semiring
(lt_table_den_backward, through RecognitionLattice on ROCm tensors):

* ``_forward`` under autograd on FrameLabelDependent(K) and NextStateTable
  lattices: Log -> the arc marginals (the reference's FrameLabelDependent
  fixtures' den_grad, or golden_cases.table_den_marginals from the pinned
  table oracle), element by element within golden_cases.marginal_scale;
  MaxTropical -> the best path's arcs, element by element against the
  pinned oracle (table_oracle.c tab_dist_grad) plus properties (labels = the
  table Viterbi's, weights re-sum to the distance); Real -> alpha * beta'
  against the pinned oracle (both pinned to the reference's own autograd,
  tests/golden/grads_*.npz, tests/test_oracle_grads.py).
* ``_string_forward`` (Log) on the table path: d num / dW against the table
  oracle's string-only loss gradient.
* ``_backward`` with a callback on a FrameLabelDependent lattice
  (lattices.py:686-799, ``self.alignment.backward`` at :764): per-frame
  marginals summed over alignment states = den_grad.
* Real gradients of the tuned FullNGram x FrameDependent path (_DenFn).
"""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat
from golden_cases import (FLD_CASES, LATTICE_CASES, assert_grad_marginal_close, assert_loss_close,
                          load, load_fld, table_den_marginals)

pytestmark = pytest.mark.gpu


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _lattice(context, alignment, table):
  return lt.RecognitionLattice(
      context=context, alignment=alignment,
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))


def _frames(B, T, device):
  return torch.arange(T, dtype=torch.float32, device=device)[None, :, None].expand(B, T, 1)


def _fld(c):
  return (lt.contexts.FullNGram(vocab_size=c['V'], context_size=c['n']),
          lt.alignments.FrameLabelDependent(max_expansions=c['K']))


def _real_ref(W, nf, V, n, K):
  """(dist, d dist / dW) of the Real distance from the pinned oracle
  (table_oracle.c tab_dist_grad, double; checked against the reference's
  own Real autograd by tests/test_oracle_grads.py)."""
  orc = _orc()
  return orc.tab_dist_grad(orc.full_ngram_table(V, n), W, nf, K, orc.REAL)


def _assert_real_grad(got, ref):
  scale = max(1.0, float(np.abs(ref).max()))
  np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize('case', FLD_CASES)
def test_fld_forward_gradients(cuda, case):
  """_forward's Log / MaxTropical / Real gradients on the reference's
  FrameLabelDependent fixtures."""
  c = load_fld(case)
  B, T = c['W'].shape[:2]
  ctx, align = _fld(c)
  nf = torch.tensor(c['num_frames'])
  frames = _frames(B, T, cuda)
  # Log: the arc marginals (den_grad), relative to each arc's own marginal
  table = torch.tensor(c['W'], device=cuda, requires_grad=True)
  lat = _lattice(ctx, align, table)
  d, _ = lat._forward(None, frames, nf, lt.semirings.Log)
  assert_loss_close(d.detach().cpu().numpy(), c['den_Log'])
  d.sum().backward()
  assert_grad_marginal_close(table.grad.cpu().numpy(), c['den_grad'], c['den_grad'], c['den_Log'],
                             None)
  # MaxTropical: the best path's arcs
  table.grad = None
  d, _ = lat._forward(None, frames, nf, lt.semirings.MaxTropical)
  np.testing.assert_array_equal(d.detach().cpu().numpy(), c['den_MaxTropical'])
  w = torch.linspace(0.5, 2.0, B, device=cuda)
  (w * d).sum().backward()
  g = table.grad.cpu().numpy()
  # the path's arcs re-sum to its weight (each arc's weight once per use)
  resum = (g.astype(np.float64) * c['W']).sum(axis=(1, 2, 3)) / w.cpu().numpy()
  np.testing.assert_allclose(resum, c['den_MaxTropical'], rtol=1e-5, atol=1e-4)
  # every live frame takes one blank and up to K lexical arcs; labels agree
  # with the table Viterbi decode
  K = c['K']
  live = np.arange(T)[None, :] < c['num_frames'][:, None]
  blanks = g[..., 0].sum(-1) / w.cpu().numpy()[:, None]
  np.testing.assert_allclose(blanks, live.astype(np.float64), atol=1e-6)
  labels, _ = nat.table_viterbi(nat.TableGraph(_orc().full_ngram_table(c['V'], c['n']), K, cuda),
                                table.detach(), nf.to(cuda), 0)
  labels = labels.cpu().numpy().reshape(B, T, K + 1)
  nlex = (labels > 0).sum(-1)
  lexsum = g[..., 1:].sum((-2, -1)) / w.cpu().numpy()[:, None]
  np.testing.assert_allclose(lexsum, nlex * live, atol=1e-6)
  # and element by element: the oracle's first-maximum path, scaled by w
  orc = _orc()
  _, rg = orc.tab_dist_grad(orc.full_ngram_table(c['V'], c['n']), c['W'], c['num_frames'], K,
                            orc.MAX, grad=w.cpu().numpy())
  np.testing.assert_array_equal(g, rg)
  # Real: alpha * beta' against the pinned oracle
  table.grad = None
  d, _ = lat._forward(None, frames, nf, lt.semirings.Real)
  rd, rg = _real_ref(c['W'], c['num_frames'], c['V'], c['n'], K)
  np.testing.assert_allclose(d.detach().cpu().numpy(), rd,
                             rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(rd).max())))
  d.sum().backward()
  _assert_real_grad(table.grad.cpu().numpy(), rg)


@pytest.mark.parametrize('case', [k for k in LATTICE_CASES if not k.startswith('bf16')])
def test_real_semiring_gradient_full_ngram(cuda, case):
  """Real-semiring _forward gradient on the tuned FullNGram x
  FrameDependent path (_DenFn -> lt_table_den_backward)."""
  c = load(case)
  B, T = c['W'].shape[:2]
  ctx = lt.contexts.FullNGram(vocab_size=c['V'], context_size=c['n'])
  align = lt.alignments.FrameDependent()
  table = torch.tensor(c['W'], device=cuda, requires_grad=True)
  lat = _lattice(ctx, align, table)
  nf = torch.tensor(c['num_frames'])
  d, _ = lat._forward(None, _frames(B, T, cuda), nf, lt.semirings.Real)
  rd, rg = _real_ref(c['W'], c['num_frames'], c['V'], c['n'], 0)
  np.testing.assert_allclose(d.detach().cpu().numpy(), rd,
                             rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(rd).max())))
  g = torch.linspace(-1.0, 1.5, B, device=cuda)
  (g * d).sum().backward()
  _assert_real_grad(table.grad.cpu().numpy(), rg * g.cpu().numpy()[:, None, None, None])


RANDOM_DFA = [
    # C, V, K, B, T, U, dtype
    (7, 4, 0, 4, 30, 6, 'f32'),
    (7, 4, 2, 4, 30, 6, 'bf16'),
    (23, 9, 3, 3, 25, 8, 'f32'),
    (40, 16, 1, 2, 40, 12, 'f32'),
]


@pytest.mark.parametrize('C,V,K,B,T,U,dt', RANDOM_DFA)
def test_next_state_table_gradients(cuda, C, V, K, B, T, U, dt):
  """A NextStateTable context (FrameDependent or FrameLabelDependent(K)):
  _forward's Log gradient against the table oracle's den marginals,
  _string_forward's Log gradient against its string-only gradient, the
  MaxTropical gradient against the Viterbi path weight, and _backward's
  callback marginals."""
  orc = _orc()
  rng = np.random.default_rng(C * 7 + V + K)
  tab = rng.integers(0, C, (C, V)).astype(np.int32)
  bf16 = dt == 'bf16'
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  nf = rng.integers(1, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(0, U + 1, B).astype(np.int32)
  ctx = lt.contexts.NextStateTable(torch.tensor(tab))
  align = (lt.alignments.FrameDependent() if K == 0
           else lt.alignments.FrameLabelDependent(max_expansions=K))
  table = torch.tensor(W, device=cuda, requires_grad=True)
  lat = _lattice(ctx, align, table)
  frames = _frames(B, T, cuda)
  den = table_den_marginals(orc, tab, W, nf, lab, nl, K)
  rlz = orc.tab_den_forward(tab, W, nf, K, orc.LOG)
  # _forward, Log
  d, alpha = lat._forward(None, frames, torch.tensor(nf), lt.semirings.Log)
  assert_loss_close(d.detach().cpu().numpy(), rlz)
  d.sum().backward()
  assert_grad_marginal_close(table.grad.cpu().numpy(), den, den, rlz, None)
  # _string_forward, Log: d num / dW = -(the string-only loss gradient)
  table.grad = None
  s = lat._string_forward(None, frames, torch.tensor(nf), torch.tensor(lab), torch.tensor(nl),
                          lt.semirings.Log)
  rl, _, rnum, rdl = orc.tab_loss_grad(tab, W, nf, lab, nl, K, local_norm=True)
  assert_loss_close(s.detach().cpu().numpy(), rnum)
  fin = torch.isfinite(s.detach())
  s.masked_fill(~fin, 0).sum().backward()
  assert_grad_marginal_close(-table.grad.cpu().numpy(), rdl, None, np.zeros_like(rnum), rnum,
                             weights=fin.float().cpu().numpy())
  # _forward, MaxTropical: the arcs re-sum to the path weight
  table.grad = None
  dm, _ = lat._forward(None, frames, torch.tensor(nf), lt.semirings.MaxTropical)
  np.testing.assert_array_equal(dm.detach().cpu().numpy(), orc.tab_den_forward(tab, W, nf, K, orc.MAX))
  dm.sum().backward()
  resum = (table.grad.cpu().numpy().astype(np.float64) * W).sum(axis=(1, 2, 3))
  np.testing.assert_allclose(resum, dm.detach().cpu().numpy(), rtol=1e-5, atol=1e-4)
  # _backward: the callback's marginals (summed over alignment states)
  seen = []

  def callback(weight_vjp_fn, carry, blank_marginal, lexical_marginals):
    seen.append(torch.cat([blank_marginal[..., None], lexical_marginals], dim=-1).cpu().numpy())
    return carry + 1, blank_marginal.sum(-1)

  carry, _ = lat._backward(None, frames, torch.tensor(nf), d.detach(), alpha.detach(), 0, callback)
  assert carry == T
  marg = np.stack(seen[::-1], axis=1)
  assert_grad_marginal_close(marg, den, den, rlz, None)


def test_entropy_frame_label_dependent(cuda):
  """RecognitionLattice.entropy on a FrameLabelDependent lattice (the HIP
  marginals through lt_table_den_backward) against the CPU path."""
  c = load_fld('k2_unigram_v5')
  B, T = c['W'].shape[:2]
  ctx, align = _fld(c)
  nf = torch.tensor(c['num_frames'])
  got = _lattice(ctx, align, torch.tensor(c['W'], device=cuda)).entropy(_frames(B, T, cuda), nf)
  ref = _lattice(ctx, align, torch.tensor(c['W'])).entropy(_frames(B, T, 'cpu'), nf)
  np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
