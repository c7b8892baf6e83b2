"""The PyTorch CPU path (last_torch_amd/cpu.py, RecognitionLattice on CPU
tensors) against every lattice fixture of tests/golden (made from the
reference, tests/golden/make_golden.py), cfg1 (B=2, T=8, U=4, V=5, n=0)
included: distances, alphas, numerators, losses, loss gradients, Viterbi
labels and weights. Tolerances as the GPU parity tests (golden_cases)."""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import cpu
from golden_cases import LATTICE_CASES, assert_grad_close, assert_loss_close, load


def _setup(case):
  d = load(case)
  V, n = d['V'], d['n']
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  return d, ctx, lt.alignments.FrameDependent()


def _t(x, dtype=None):
  return torch.tensor(np.asarray(x), dtype=dtype)


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_cpu_distances(case):
  d, ctx, al = _setup(case)
  W, nf = _t(d['W']), _t(d['num_frames']).long()
  for sname in ('Log', 'MaxTropical'):
    sr = getattr(lt.semirings, sname)
    dist, alpha = cpu.den_forward(W, nf, ctx, al, sr)
    assert_loss_close(dist.numpy(), d[f'den_{sname}'])
    np.testing.assert_allclose(alpha.numpy(), d[f'alpha_{sname}'], rtol=1e-5, atol=1e-4)
    num = cpu.num_forward(W, nf, _t(d['labels']), _t(d['num_labels']).long(), ctx, al, sr)
    assert_loss_close(num.numpy(), d[f'num_{sname}'])


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_cpu_loss_and_grad(case):
  d, ctx, al = _setup(case)
  nf, lab, nl = _t(d['num_frames']).long(), _t(d['labels']), _t(d['num_labels']).long()
  for local, key in ((False, 'W'), (True, 'W_local')):
    W = _t(d[key]).requires_grad_(True)
    loss = cpu.loss(W, nf, lab, nl, ctx, al, local)
    assert_loss_close(loss.detach().numpy(), d['loss_local' if local else 'loss'])
    loss.sum().backward()
    ref = d['loss_local_grad' if local else 'loss_grad']
    lz = d['den_Log'] if not local else np.zeros_like(d['den_Log'])
    assert_grad_close(W.grad.numpy(), ref, lz, num=d['num_Log'], bf16=bool(d['bf16']))


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_cpu_viterbi(case):
  d, ctx, al = _setup(case)
  W, nf = _t(d['W']), _t(d['num_frames']).long()
  for conv, key in (('reference', 'vit_labels_reference'), ('true', 'vit_labels_true')):
    labels, weights = cpu.viterbi(W, nf, ctx, al, conv)
    np.testing.assert_array_equal(labels.numpy(), d[key])
    assert_loss_close(weights.numpy(), d['vit_weights'])


def test_lattice_on_cpu_tensors_cfg1():
  """RecognitionLattice with CPU tensors at cfg1's exact shape runs the CPU
  path (no GPU needed): loss, its gradient, shortest_path, _forward,
  _string_forward all against the fixture."""
  d = load('cfg1')
  V, n = d['V'], d['n']
  B, T = d['W'].shape[:2]
  table = torch.tensor(d['W'], requires_grad=True)  # frame t's weights are row t
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.arange(T, dtype=torch.float32)[None, :, None].expand(B, T, 1)
  nf, lab, nl = (torch.tensor(d[k]) for k in ('num_frames', 'labels', 'num_labels'))
  loss = lat(frames, nf, lab, nl)
  assert loss.device.type == 'cpu'
  assert_loss_close(loss.detach().numpy(), d['loss'])
  loss.sum().backward()
  assert_grad_close(table.grad.numpy(), d['loss_grad'], d['den_Log'], num=d['num_Log'])
  labels, nlab, weights = lat.shortest_path(frames, nf)
  np.testing.assert_array_equal(labels.numpy(), d['vit_labels_reference'])
  assert_loss_close(weights.numpy(), d['vit_weights'])
  dist, alpha = lat._forward(None, frames, nf, lt.semirings.Log)
  assert_loss_close(dist.detach().numpy(), d['den_Log'])
  num = lat._string_forward(None, frames, nf, lab, nl, lt.semirings.Log)
  assert_loss_close(num.detach().numpy(), d['num_Log'])
