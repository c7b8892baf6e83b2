"""The remaining RecognitionLattice API surface on CPU tensors (the CPU path;
tests/test_gpu_api.py runs the same checks on the HIP kernels):

* ``_backward`` with a callback (reference intent lattices.py:686-799 with
  the frame order fixed, D4; BackwardStepCallback :644-684): frames visited
  T-1 .. 0, blank / lexical marginals equal to the den_grad fixtures, outputs
  stacked in time order, and weight_vjp_fn(marginals) summed over frames
  equal to autograd's d log_z / d frames;
* the gradient through ``_forward``: Log -> the arc marginals (den_grad),
  MaxTropical -> the one-hot best-path arcs (the Viterbi labels).
"""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from golden_cases import LATTICE_CASES, assert_grad_marginal_close, assert_loss_close, load

CASES = [c for c in LATTICE_CASES if c in ('kat', 'bigram_v3', 'trigram_v2', 'cfg1', 'peaked',
                                            'unigram_v3')]


def _table_lattice(c, table):
  return lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=c['V'], context_size=c['n']),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))


def _frames(B, T, device='cpu'):
  return torch.arange(T, dtype=torch.float32, device=device)[None, :, None].expand(B, T, 1)


def check_backward_callback(c, device):
  B, T = c['W'].shape[:2]
  table = torch.tensor(c['W'], device=device)
  lat = _table_lattice(c, table)
  frames = _frames(B, T, device)
  nf = torch.tensor(c['num_frames'])
  log_z, alpha = lat._forward(None, frames, nf, lt.semirings.Log)
  seen = []

  def callback(weight_vjp_fn, carry, blank_marginal, lexical_marginals):
    seen.append((blank_marginal.detach().cpu().numpy(), lexical_marginals.detach().cpu().numpy()))
    return carry + 1, blank_marginal.sum(-1)

  carry, outs = lat._backward(None, frames, nf, log_z, alpha, 0, callback)
  assert carry == T and len(seen) == T
  seen.reverse()  # visited T-1 .. 0
  marg = np.stack([np.concatenate([b[..., None], l], axis=-1) for b, l in seen], axis=1)
  # every element relative to its own marginal (den-only: ref = den, no num)
  assert_grad_marginal_close(marg, c['den_grad'], c['den_grad'], c['den_Log'], None)
  # outputs stacked in time order along the frame axis
  np.testing.assert_allclose(outs.cpu().numpy(), marg[..., 0].sum(-1), rtol=1e-6, atol=1e-6)


def check_backward_vjp(device):
  """weight_vjp_fn: sum_t vjp_t(marginals_t) = d log_z / d frames."""
  torch.manual_seed(0)
  B, T, F, V = 2, 6, 5, 3
  cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=4,
                                         device=device)
  wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=8, device=device)
  lat = lt.RecognitionLattice(context=lt.contexts.FullNGram(vocab_size=V, context_size=1),
                              alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: cacher,
                              weight_fn_factory=lambda _: wfn)
  frames = torch.randn([B, T, F], device=device, requires_grad=True)
  nf = torch.tensor([T, T - 2])
  cache = lat.build_cache()
  log_z, alpha = lat._forward(cache, frames, nf, lt.semirings.Log)
  (want,) = torch.autograd.grad(log_z.sum(), frames)

  def callback(weight_vjp_fn, carry, blank_marginal, lexical_marginals):
    _, d_frame = weight_vjp_fn((blank_marginal, lexical_marginals))
    return carry, d_frame

  _, got = lat._backward(cache, frames.detach(), nf, log_z.detach(), alpha.detach(), None,
                         callback)
  np.testing.assert_allclose(got.detach().cpu().numpy(), want.cpu().numpy(), rtol=1e-4, atol=1e-5)


def check_forward_gradients(c, device):
  B, T = c['W'].shape[:2]
  nf = torch.tensor(c['num_frames'])
  # Log: the arc marginals
  table = torch.tensor(c['W'], device=device, requires_grad=True)
  dist, _ = _table_lattice(c, table)._forward(None, _frames(B, T, device), nf, lt.semirings.Log)
  assert_loss_close(dist.detach().cpu().numpy(), c['den_Log'])
  dist.sum().backward()
  assert_grad_marginal_close(table.grad.cpu().numpy(), c['den_grad'], c['den_grad'], c['den_Log'],
                             None)
  # MaxTropical: one arc per live frame, its label the Viterbi label
  table = torch.tensor(c['W'], device=device, requires_grad=True)
  dist, _ = _table_lattice(c, table)._forward(None, _frames(B, T, device), nf,
                                              lt.semirings.MaxTropical)
  assert_loss_close(dist.detach().cpu().numpy(), c['den_MaxTropical'])
  dist.sum().backward()
  g = table.grad.cpu().numpy()
  live = np.arange(T)[None, :] < c['num_frames'][:, None]
  np.testing.assert_array_equal(g.reshape(B, T, -1).sum(-1), live.astype(np.float32))
  lab = np.where(live, g.sum(2).argmax(-1), 0)  # summed over source states: the label taken
  np.testing.assert_array_equal(lab, c['vit_labels_true'])


@pytest.mark.parametrize('case', CASES)
def test_backward_callback_cpu(case):
  check_backward_callback(load(case), 'cpu')


def test_backward_weight_vjp_cpu():
  check_backward_vjp('cpu')


@pytest.mark.parametrize('case', CASES)
def test_forward_gradients_cpu(case):
  check_forward_gradients(load(case), 'cpu')
