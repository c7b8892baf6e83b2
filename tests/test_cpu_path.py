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
from golden_cases import (FLD_CASES, LATTICE_CASES, assert_grad_close, assert_grad_marginal_close,
                          assert_loss_close, load, load_fld)


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


def _fld_setup(case):
  d = load_fld(case)
  ctx = lt.contexts.FullNGram(vocab_size=d['V'], context_size=d['n'])
  return d, ctx, lt.alignments.FrameLabelDependent(max_expansions=d['K'])


@pytest.mark.parametrize('case', FLD_CASES)
def test_cpu_frame_label_dependent_fixtures(case):
  """FrameLabelDependent(K) on the CPU path against the reference's own FLD
  fixtures (tests/golden/make_golden_fld.py): Log / MaxTropical / Real
  distances and alphas, numerators, the loss and every gradient element
  relative to its marginals; Viterbi labels and weights bit-exact against
  the pinned table oracle (the reference's FLD labels are aliased, D6)."""
  from oracle import oracle as orc  # the checker
  d, ctx, al = _fld_setup(case)
  W, nf = _t(d['W']), _t(d['num_frames']).long()
  lab, nl = _t(d['labels']), _t(d['num_labels']).long()
  for sname in ('Log', 'MaxTropical', 'Real'):
    sr = getattr(lt.semirings, sname)
    dist, alpha = cpu.den_forward(W, nf, ctx, al, sr)
    num = cpu.num_forward(W, nf, lab, nl, ctx, al, sr)
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(dist.numpy(), d['den_MaxTropical'])
      np.testing.assert_array_equal(alpha.numpy(), d['alpha_MaxTropical'])
      np.testing.assert_array_equal(num.numpy(), d['num_MaxTropical'])
    else:
      tol = 1e-4 * max(1.0, float(np.abs(d[f'den_{sname}'][np.isfinite(d[f'den_{sname}'])]).max(
          initial=0)))
      np.testing.assert_allclose(dist.numpy(), d[f'den_{sname}'], rtol=1e-4, atol=tol)
      np.testing.assert_allclose(num.numpy(), d[f'num_{sname}'], rtol=1e-4, atol=tol)
      np.testing.assert_allclose(alpha.numpy(), d[f'alpha_{sname}'], rtol=1e-4, atol=1e-4)
  Wg = W.clone().requires_grad_(True)
  loss = cpu.loss(Wg, nf, lab, nl, ctx, al, False)
  assert_loss_close(loss.detach().numpy(), d['loss'])
  fin = torch.isfinite(loss.detach())
  loss.masked_fill(~fin, 0).sum().backward()
  assert_grad_marginal_close(Wg.grad.numpy(), d['loss_grad'], d['den_grad'], d['den_Log'],
                             d['num_Log'])
  table = orc.full_ngram_table(d['V'], d['n'])
  for conv in ('reference', 'true'):
    labels, weights = cpu.viterbi(W, nf, ctx, al, conv)
    rl, rw = orc.tab_viterbi(table, d['W'], d['num_frames'], d['K'],
                             1 if conv == 'reference' else 0)
    np.testing.assert_array_equal(labels.numpy(), rl)
    np.testing.assert_array_equal(weights.numpy(), rw)


def test_cpu_frame_label_dependent_lattice_api():
  """tests/lattices_test.py:129-176 (the reference's FrameLabelDependent
  test) through RecognitionLattice on CPU tensors: the loss finiteness
  pattern, the gradient against the table oracle, the alignment-label
  padding and last-slot invariants, path weight = MaxTropical distance."""
  from oracle import oracle as orc
  V, n, K, B, T = 2, 1, 2, 4, 6
  rng = np.random.default_rng(3)
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  table = torch.tensor(W, requires_grad=True)
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
      alignment=lt.alignments.FrameLabelDependent(max_expansions=K),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.arange(T, dtype=torch.float32)[None, :, None].expand(B, T, 1)
  num_frames = torch.tensor([6, 3, 2, 1])
  labels = torch.tensor([[1, 1, 1, 1], [2, 2, 2, 2], [1, 2, 1, 2], [2, 1, 2, 1]])
  num_labels = torch.tensor([4, 3, 4, 3])
  loss = lat(frames, num_frames, labels, num_labels)
  assert loss.device.type == 'cpu'
  np.testing.assert_array_equal(torch.isfinite(loss).numpy(), [True, True, True, False])
  fin = torch.isfinite(loss.detach())
  loss.masked_fill(~fin, 0).sum().backward()
  tab = orc.full_ngram_table(V, n)
  rl, rlz, _, rdW = orc.tab_loss_grad(tab, W, num_frames.numpy().astype(np.int32),
                                      labels.numpy().astype(np.int32),
                                      num_labels.numpy().astype(np.int32), K)
  assert_loss_close(loss.detach().numpy(), rl)
  assert_grad_close(table.grad.numpy(), rdW, rlz)
  al, nal, pw = lat.shortest_path(frames, num_frames)
  np.testing.assert_array_equal(nal.numpy(), 3 * num_frames.numpy())
  np.testing.assert_array_equal(al.reshape(4, 6, 3)[..., -1].numpy(), np.zeros([4, 6]))
  assert ((al >= 0) & (al <= V)).all()
  d, _ = lat._forward(None, frames, num_frames, lt.semirings.MaxTropical)
  np.testing.assert_array_equal(pw.numpy(), d.detach().numpy())
  rlab, rw = orc.tab_viterbi(tab, W, num_frames.numpy().astype(np.int32), K, 1)
  np.testing.assert_array_equal(al.numpy(), rlab)


@pytest.mark.parametrize('K', [0, 1, 2])
def test_cpu_next_state_table_contexts(K):
  """A random NextStateTable DFA with FrameDependent (K = 0) or
  FrameLabelDependent(K) on CPU tensors against the table oracle: Log and
  MaxTropical distances, the loss and its gradient, Viterbi."""
  from oracle import oracle as orc
  rng = np.random.default_rng(90 + K)
  C, V, B, T, U = 6, 3, 3, 12, 4
  tab = rng.integers(0, C, (C, V)).astype(np.int32)
  ctx = lt.contexts.NextStateTable(torch.tensor(tab))
  al = lt.alignments.FrameDependent() if K == 0 else \
      lt.alignments.FrameLabelDependent(max_expansions=K)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = np.array([12, 7, 3], np.int32)
  lab = rng.integers(0, V + 1, (B, U)).astype(np.int32)
  nl = np.array([4, 2, 1], np.int32)
  Wt, nft, labt, nlt = _t(W), _t(nf).long(), _t(lab), _t(nl).long()
  d, _ = cpu.den_forward(Wt, nft, ctx, al, lt.semirings.Log)
  assert_loss_close(d.numpy(), orc.tab_den_forward(tab, W, nf, K, orc.LOG))
  dm, _ = cpu.den_forward(Wt, nft, ctx, al, lt.semirings.MaxTropical)
  np.testing.assert_array_equal(dm.numpy(), orc.tab_den_forward(tab, W, nf, K, orc.MAX))
  s = cpu.num_forward(Wt, nft, labt, nlt, ctx, al, lt.semirings.MaxTropical)
  np.testing.assert_array_equal(s.numpy(), orc.tab_num_forward(tab, W, nf, lab, nl, K, orc.MAX))
  Wg = Wt.clone().requires_grad_(True)
  loss = cpu.loss(Wg, nft, labt, nlt, ctx, al, False)
  fin = torch.isfinite(loss.detach())
  loss.masked_fill(~fin, 0).sum().backward()
  rl, rlz, _, rdW = orc.tab_loss_grad(tab, W, nf, lab, nl, K)
  assert_loss_close(loss.detach().numpy(), rl)
  assert_grad_close(Wg.grad.numpy(), rdW, rlz)
  labels, w = cpu.viterbi(Wt, nft, ctx, al, 'true')
  rlab, rw = orc.tab_viterbi(tab, W, nf, K, 0)
  np.testing.assert_array_equal(labels.numpy(), rlab)
  np.testing.assert_array_equal(w.numpy(), rw)
