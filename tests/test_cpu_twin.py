"""The host twin (liblt_lattice_cpu.so, include/lt_lattice_cpu.h) against the
reference's golden fixtures and the pinned C oracle -- the same checks and
tolerances the GPU parity tests apply to the HIP kernels
(tests/test_gpu_parity.py):

  * Log loss / log_z / numerator: |got - ref| <= 1e-4 * max(1, |ref|);
  * dW: every element within golden_cases.marginal_scale (relative to its own
    den + num marginals, alignments.py:300-318);
  * MaxTropical distances, alpha and Viterbi labels / weights: bit-exact.

CPU only: runs in the default `-m "not gpu"` suite.
"""
import ctypes

import numpy as np
import pytest
import torch

from last_torch_amd import _native_cpu as cpu
from golden_cases import (LATTICE_CASES, assert_grad_close, assert_grad_marginal_close,
                          assert_loss_close, assert_values_close, load)

LOG, MAX, REAL = 0, 1, 2
SID = {'Log': LOG, 'MaxTropical': MAX, 'Real': REAL}


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _host(c, key='W'):
  W = torch.tensor(c[key])
  if c['bf16']:
    W = W.to(torch.bfloat16)
  return W, torch.tensor(c['num_frames']), torch.tensor(c['labels']), torch.tensor(c['num_labels'])


def test_exports():
  """Every symbol include/lt_lattice_cpu.h declares is exported."""
  l = ctypes.CDLL(cpu.LIB_PATH)
  for name in cpu.EXPORTED:
    assert hasattr(l, name), name
  with open(cpu.LIB_PATH.replace('last_torch_amd/liblt_lattice_cpu.so',
                                 'include/lt_lattice_cpu.h')) as f:
    hdr = f.read()
  for name in cpu.EXPORTED:
    assert name + '(' in hdr, name


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('semiring', ['Log', 'MaxTropical', 'Real'])
def test_golden_den_forward(case, semiring):
  c = load(case)
  W, nf, _, _ = _host(c)
  d, a = cpu.den_forward(W, nf, c['V'], c['n'], SID[semiring])
  d, a = d.numpy(), a.numpy()
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(d, c['den_MaxTropical'])
    np.testing.assert_array_equal(a, c['alpha_MaxTropical'])
  elif semiring == 'Log':
    assert_loss_close(d, c['den_Log'])
    assert_values_close(a, c['alpha_Log'], rtol=1e-4, atol=1e-4)
  else:
    ref = c['den_Real']
    scale = max(1.0, float(np.abs(ref).max()))
    assert_values_close(d, ref, rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('semiring', ['Log', 'MaxTropical', 'Real'])
def test_golden_num_forward(case, semiring):
  c = load(case)
  W, nf, lab, nl = _host(c)
  num, _ = cpu.num_forward(W, nf, lab, nl, c['V'], c['n'], SID[semiring])
  num = num.numpy()
  ref = c[f'num_{semiring}']
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(num, ref)
  elif semiring == 'Log':
    assert_loss_close(num, ref)
  else:
    scale = max(1.0, float(np.abs(ref).max()))
    assert_values_close(num, ref, rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('local', [False, True])
def test_golden_loss_and_grad(case, local):
  c = load(case)
  W, nf, lab, nl = _host(c, 'W_local' if local else 'W')
  loss, lz, num, dW = cpu.loss_grad(W, nf, lab, nl, c['V'], c['n'], local)
  assert_loss_close(loss.numpy(), c['loss_local' if local else 'loss'])
  if not local:
    assert_loss_close(lz.numpy(), c['den_Log'])
  ref = c['loss_local_grad' if local else 'loss_grad']
  assert_grad_marginal_close(dW.float().numpy(), ref, None if local else c['den_grad'],
                             c['den_Log'], c['num_Log'], c['bf16'])


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_golden_den_grad(case):
  c = load(case)
  W, nf, _, _ = _host(c)
  lz, al = cpu.den_forward(W, nf, c['V'], c['n'], LOG)
  dW = cpu.den_backward(W, nf, lz, al, c['V'], c['n'])
  assert_grad_close(dW.float().numpy(), c['den_grad'], c['den_Log'], c['bf16'])


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('convention', ['reference', 'true'])
def test_golden_viterbi_bit_exact(case, convention):
  c = load(case)
  W, nf, _, _ = _host(c)
  labels, weights, _ = cpu.viterbi(W, nf, c['V'], c['n'], 1 if convention == 'reference' else 0)
  np.testing.assert_array_equal(labels.numpy(), c[f'vit_labels_{convention}'])
  np.testing.assert_array_equal(weights.numpy(), c['vit_weights'])


def _random(B, T, U, V, n, seed, dtype=torch.float32):
  g = torch.Generator().manual_seed(seed)
  C = sum(V ** i for i in range(n + 1))
  W = torch.randn([B, T, C, V + 1], generator=g).to(dtype)
  nf = torch.randint(0, T + 1, [B], generator=g).to(torch.int32)
  nf[0] = T
  lab = torch.randint(0, V + 1, [B, U], generator=g).to(torch.int32)
  nl = torch.randint(0, U + 1, [B], generator=g).to(torch.int32)
  return W, nf, lab, nl


@pytest.mark.parametrize('V,n,dtype', [(4, 0, torch.float32), (6, 1, torch.float32),
                                       (5, 2, torch.float32), (3, 3, torch.float32),
                                       (6, 1, torch.bfloat16), (4, 2, torch.bfloat16)])
def test_random_against_oracle(V, n, dtype):
  """Random problems (ragged lengths, epsilon labels, padding) against the C
  oracle: loss, dW (per-element bound), Viterbi bit-exact, arcs one-hot."""
  orc = _orc()
  B, T, U = 5, 37, 6
  W, nf, lab, nl = _random(B, T, U, V, n, 100 + V * 10 + n, dtype)
  Wf = W.float().numpy()
  loss, lz, num, dW = cpu.loss_grad(W, nf, lab, nl, V, n)
  rl, rlz, rnum, rdW = orc.loss_grad(Wf, nf.numpy(), lab.numpy(), nl.numpy(), V, n)
  assert_loss_close(loss.numpy(), rl)
  den = orc.den_grad(Wf, nf.numpy(), V, n)[1]
  assert_grad_marginal_close(dW.float().numpy(), rdW, den, rlz, rnum, dtype == torch.bfloat16)
  for conv in (0, 1):
    labels, wts, arcs = cpu.viterbi(W, nf, V, n, conv, with_arcs=True)
    rlab, rw, rarcs = orc.viterbi(Wf, nf.numpy(), V, n, convention=conv, want_arcs=True)
    np.testing.assert_array_equal(labels.numpy(), rlab)
    np.testing.assert_array_equal(wts.numpy(), rw)
    np.testing.assert_array_equal(arcs.float().numpy(), rarcs)


def test_grad_scaling_and_unreachable():
  """dW scales with the incoming gradient; an unreachable string gives
  loss = +inf and dW = 0 (lattices_test.py:57); T = 0 gives loss 0."""
  V, n = 3, 1
  W, nf, lab, nl = _random(4, 9, 3, V, n, 7)
  g = torch.tensor([1.0, -2.0, 0.5, 3.0])
  _, _, _, d1 = cpu.loss_grad(W, nf, lab, nl, V, n)
  _, _, _, dg = cpu.loss_grad(W, nf, lab, nl, V, n, grad=g)
  np.testing.assert_allclose(dg.numpy(), d1.numpy() * g.numpy()[:, None, None, None], rtol=1e-6,
                             atol=1e-7)
  # 3 labels in 1 frame cannot be emitted
  nf2 = torch.tensor([1, 0, 9, 9], dtype=torch.int32)
  nl2 = torch.tensor([3, 0, 3, 0], dtype=torch.int32)
  loss, _, _, dW = cpu.loss_grad(W, nf2, lab, nl2, V, n)
  assert np.isposinf(loss[0].item()) and float(dW[0].abs().sum()) == 0.0
  assert loss[1].item() == 0.0 and float(dW[1].abs().sum()) == 0.0


def test_threads_do_not_change_results():
  V, n = 4, 2
  W, nf, lab, nl = _random(7, 20, 5, V, n, 11)
  cpu.set_num_threads(1)
  try:
    a = cpu.loss_grad(W, nf, lab, nl, V, n)
  finally:
    cpu.set_num_threads(0)
  b = cpu.loss_grad(W, nf, lab, nl, V, n)
  for x, y in zip(a, b):
    np.testing.assert_array_equal(x.numpy(), y.numpy())


def test_errors():
  W = torch.zeros([1, 2, 3, 3])
  with pytest.raises(Exception, match='vocab_size'):
    cpu.den_forward(W, torch.tensor([2]), 0, 1, LOG)
  with pytest.raises(Exception, match='semiring'):
    cpu.den_forward(W, torch.tensor([2]), 2, 1, 7)


def test_twin_double_backward_matches_cpu_autograd():
  """create_graph through RecognitionLattice.forward on host tensors: the
  twin's constant dW cannot carry a second derivative, so its backward goes
  through cpu.py's autograd; the gradient of |dL/dW|^2 matches cpu.py's own
  double backward."""
  import last_torch_amd as lt
  from last_torch_amd import cpu as cpu_path
  rng = np.random.default_rng(8)
  B, T, U, V, n = 3, 7, 3, 3, 1
  W = rng.standard_normal((B, T, V + 1, V + 1)).astype(np.float32)
  nf = torch.tensor([7, 5, 3])
  lab = torch.tensor(rng.integers(1, V + 1, (B, U)))
  nl = torch.tensor([3, 2, 1])
  table = torch.tensor(W, requires_grad=True)
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.arange(T, dtype=torch.float32)[None, :, None].expand(B, T, 1)
  loss = lat(frames, nf, lab, nl)
  (g,) = torch.autograd.grad(loss.sum(), table, create_graph=True)
  (h,) = torch.autograd.grad((g * g).sum(), table)
  Wr = torch.tensor(W, requires_grad=True)
  ref = cpu_path.loss(Wr, nf, lab, nl, lt.contexts.FullNGram(vocab_size=V, context_size=n),
                      lt.alignments.FrameDependent(), False)
  (gr,) = torch.autograd.grad(ref.sum(), Wr, create_graph=True)
  (hr,) = torch.autograd.grad((gr * gr).sum(), Wr)
  np.testing.assert_allclose(g.detach().numpy(), gr.detach().numpy(), atol=1e-5)
  np.testing.assert_allclose(h.numpy(), hr.numpy(), atol=1e-4)
  assert h.abs().sum() > 0


def test_worker_count_follows_affinity():
  """The default pool is the process's affinity mask, not the machine."""
  import os
  cpu.set_num_threads(0)
  assert cpu.num_threads() == len(os.sched_getaffinity(0))
