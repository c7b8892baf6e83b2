"""Host-side plugin surface (contexts / semirings / alignments / lattice
validation) against the reference's golden tables. CPU only: these are the
PyTorch-level mirrors of contexts.py, semirings.py and alignments.py that the
HIP path plugs in behind; none of them touch the GPU."""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from golden_cases import load_npz

CTX_CONFIGS = [(3, 0), (3, 1), (3, 2), (2, 3), (5, 1), (4, 2)]
SEMIRING_NAMES = ('Log', 'MaxTropical', 'Real')


@pytest.fixture(scope='module')
def ctx_tables():
  return load_npz('contexts')


@pytest.fixture(scope='module')
def sr_tables():
  return load_npz('semirings')


@pytest.mark.parametrize('V,n', CTX_CONFIGS)
def test_fullngram_next_state(ctx_tables, V, n):
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  C, vocab = ctx.shape()
  assert vocab == V and C == ctx_tables[f'next_{V}_{n}'].shape[0]
  st = torch.arange(C)[:, None].expand(C, V + 1)
  y = torch.arange(V + 1)[None, :].expand(C, V + 1)
  np.testing.assert_array_equal(ctx.next_state(st, y).numpy(), ctx_tables[f'next_{V}_{n}'])
  # the dense table the kernels' arithmetic restates
  np.testing.assert_array_equal(ctx.next_state_table().numpy(), ctx_tables[f'next_{V}_{n}'][:, 1:])


@pytest.mark.parametrize('V,n', CTX_CONFIGS)
@pytest.mark.parametrize('semiring', SEMIRING_NAMES)
def test_fullngram_forward_reduce(ctx_tables, V, n, semiring):
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  x = torch.tensor(ctx_tables[f'reduce_in_{V}_{n}'])
  got = ctx.forward_reduce(x, getattr(lt.semirings, semiring)).numpy()
  ref = ctx_tables[f'reduce_{semiring}_{V}_{n}']
  if semiring == 'MaxTropical':
    np.testing.assert_array_equal(got, ref)
  else:
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('V,n', CTX_CONFIGS)
def test_fullngram_backward_broadcast_and_walk(ctx_tables, V, n):
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  b = torch.tensor(ctx_tables[f'bcast_in_{V}_{n}'])
  np.testing.assert_array_equal(ctx.backward_broadcast(b).numpy(), ctx_tables[f'bcast_{V}_{n}'])
  labs = torch.tensor(ctx_tables[f'walk_in_{V}_{n}']).long()
  np.testing.assert_array_equal(ctx.walk_states(labs).numpy(), ctx_tables[f'walk_{V}_{n}'])


@pytest.mark.parametrize('semiring', SEMIRING_NAMES)
def test_semiring_ops(sr_tables, semiring):
  s = getattr(lt.semirings, semiring)
  x, y = torch.tensor(sr_tables['x']), torch.tensor(sr_tables['y'])
  for op, got in [('plus', s.plus(x, y)), ('times', s.times(x, y)), ('sum', s.sum(x, dim=-1)),
                  ('prod', s.prod(x, dim=-1)), ('zeros', s.zeros([2])), ('ones', s.ones([2]))]:
    np.testing.assert_allclose(got.numpy(), sr_tables[f'{op}_{semiring}'], rtol=1e-6,
                               err_msg=f'{semiring}.{op}')


def test_log_semiring_autograd_is_sound():
  """The build's Log.plus/sum carry working gradients (reference D1/D2)."""
  x = torch.tensor([1., 2., 3.], requires_grad=True)
  lt.semirings.Log.sum(x, dim=-1).backward()
  np.testing.assert_allclose(x.grad.numpy(), torch.softmax(x.detach(), -1).numpy(), rtol=1e-6)
  a = torch.tensor([0.5, -np.inf], requires_grad=True)
  b = torch.tensor([1.5, -np.inf], requires_grad=True)
  lt.semirings.Log.plus(a, b).sum().backward()
  assert torch.isfinite(a.grad).all() and torch.isfinite(b.grad).all()
  np.testing.assert_allclose((a.grad + b.grad)[0].item(), 1.0, rtol=1e-6)


def test_max_tropical_tie_rules():
  """Maximum picks `a` on ties (semirings.py:363); Max the first argmax (:382)."""
  a = torch.tensor([1., 2.], requires_grad=True)
  b = torch.tensor([1., 3.], requires_grad=True)
  lt.semirings.MaxTropical.plus(a, b).sum().backward()
  np.testing.assert_array_equal(a.grad.numpy(), [1., 0.])
  np.testing.assert_array_equal(b.grad.numpy(), [0., 1.])
  x = torch.tensor([2., 5., 5., 1.], requires_grad=True)
  lt.semirings.MaxTropical.sum(x, dim=-1).backward()
  np.testing.assert_array_equal(x.grad.numpy(), [0., 1., 0., 0.])


def test_frame_dependent_closed_forms():
  """FrameDependent topology and step functions (alignments.py:250-329;
  tests/alignments_test.py:49-207 closed forms)."""
  fd = lt.alignments.FrameDependent()
  assert fd.num_states() == 1 and fd.start() == 0
  assert fd.blank_next(0) == 0 and fd.lexical_next(0) == 0
  assert fd.topological_visit() == [0]
  ctx = lt.contexts.FullNGram(vocab_size=2, context_size=1)
  alpha = torch.tensor([0., 1., 2.])
  blank = torch.tensor([3., 4., 5.])
  lexical = torch.tensor([[6., 7.], [8., 9.], [10., 11.]])
  r = fd.forward(alpha, [blank], [lexical], ctx, lt.semirings.Real)
  # dest 0 only blank; dest y gathers all sources' label-y arcs
  np.testing.assert_allclose(r.numpy(), [0 * 3, 1 * 4 + (0 * 6 + 1 * 8 + 2 * 10),
                                         2 * 5 + (0 * 7 + 1 * 9 + 2 * 11)])
  sf = fd.string_forward(torch.tensor([1., 2., 3.]), [torch.tensor([4., 5., 6.])],
                         [torch.tensor([7., 8., 9.])], lt.semirings.Real)
  np.testing.assert_allclose(sf.numpy(), [4., 2 * 5 + 7, 3 * 6 + 2 * 8])
  with pytest.raises(ValueError):
    fd.forward(alpha, [blank, blank], [lexical], ctx, lt.semirings.Real)


@pytest.mark.parametrize('align', ['fd', 'fld1', 'fld3'])
def test_alignment_backward_is_forward_vjp(align):
  """One frame's backward (alignments.py:300-318, :379-419) against autograd
  of its forward: with log_z the frame's total into beta, the marginals are
  d log_z / d weights and beta_t satisfies log_z = (+) alpha + beta_t."""
  torch.manual_seed(0)
  al = (lt.alignments.FrameDependent() if align == 'fd' else
        lt.alignments.FrameLabelDependent(max_expansions=int(align[3:])))
  ctx = lt.contexts.FullNGram(vocab_size=3, context_size=2)
  C, V, k = ctx.num_states(), 3, al.num_states()
  Log = lt.semirings.Log
  alpha, beta = torch.randn(2, C, dtype=torch.float64), torch.randn(2, C, dtype=torch.float64)
  blank = [torch.randn(2, C, dtype=torch.float64, requires_grad=True) for _ in range(k)]
  lexical = [torch.randn(2, C, V, dtype=torch.float64, requires_grad=True) for _ in range(k)]
  log_z = Log.sum(al.forward(alpha, blank, lexical, ctx, Log) + beta, dim=-1)
  grads = torch.autograd.grad(log_z.sum(), blank + lexical, allow_unused=True)
  nb, bm, lm = al.backward(alpha, [b.detach() for b in blank], [w.detach() for w in lexical],
                           beta, log_z.detach(), ctx)
  np.testing.assert_allclose(Log.sum(alpha + nb, dim=-1).numpy(), log_z.detach().numpy(),
                             rtol=1e-12)
  for got, want, ref in zip(bm + lm, grads, blank + lexical):
    want = torch.zeros_like(ref) if want is None else want
    np.testing.assert_allclose(got.detach().numpy(), want.numpy(), rtol=1e-10, atol=1e-12)


def test_lattice_validates_batch_dims():
  """RecognitionLattice.forward's shape checks (lattices.py:157-166) fire
  before any device work, with the reference's messages."""
  table = torch.zeros([4, 6, 3, 3])
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=2, context_size=1),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.zeros([4, 6, 1])
  nf = torch.tensor([6, 3, 2, 1])
  labels = torch.ones([4, 4])
  nl = torch.tensor([4, 3, 1, 2])
  with pytest.raises(ValueError, match='frames and num_frames have different batch_dims'):
    lat(frames[:1], nf, labels, nl)
  with pytest.raises(ValueError, match='labels and num_frames have different batch_dims'):
    lat(frames, nf, labels[:1], nl)
  with pytest.raises(ValueError, match='num_labels and num_frames have different batch_dims'):
    lat(frames, nf, labels, nl[:1])
  with pytest.raises(ValueError, match='frames and num_frames have different batch_dims'):
    lat.shortest_path(frames[:1], nf)


def test_lattice_device_dispatch():
  """The device of the arc weights picks the implementation: CPU tensors run
  the PyTorch restatement (cpu.py) with no GPU involved; the HIP path is
  taken only for ROCm tensors, and a ROCm tensor with the library missing
  raises (tests/test_abi_and_sharding.py checks the loader)."""
  table = torch.randn([2, 3, 3, 3])
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=2, context_size=1),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  frames = torch.arange(3.)[None, :, None].expand(2, 3, 1)
  loss = lat(frames, torch.tensor([3, 2]), torch.ones([2, 2]), torch.tensor([1, 1]))
  assert loss.device.type == 'cpu' and torch.isfinite(loss).all()
  labels, _, weights = lat.shortest_path(frames, torch.tensor([3, 2]))
  assert labels.shape == (2, 3) and weights.device.type == 'cpu'
  fsa = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=2, context_size=1),
      alignment=lt.alignments.FrameLabelDependent(max_expansions=2),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  # FrameLabelDependent runs on the CPU path too (round 3)
  loss = fsa(frames, torch.tensor([3, 2]), torch.ones([2, 2]), torch.tensor([1, 1]))
  assert loss.device.type == 'cpu' and torch.isfinite(loss).all()
  labels, nal, _ = fsa.shortest_path(frames, torch.tensor([3, 2]))
  assert labels.shape == (2, 9) and nal.tolist() == [9, 6]

  class NotAnAlignment:
    def num_states(self):
      return 1

  odd = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=2, context_size=1), alignment=NotAnAlignment(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  with pytest.raises(NotImplementedError, match='FrameDependent'):
    odd(frames, torch.tensor([3, 2]), torch.ones([2, 2]), torch.tensor([1, 1]))


# ---------------------------------------------------------------------------
# NextStateTable / FrameLabelDependent host classes
# ---------------------------------------------------------------------------
def test_next_state_table_validation_and_full_ngram():
  """contexts_test.py:175-200: invalid tables raise; a FullNGram table gives
  the same maps as FullNGram."""
  import last_torch_amd as lt
  with pytest.raises(ValueError, match='non-zero size'):
    lt.contexts.NextStateTable(torch.zeros([1, 0], dtype=torch.int32))
  with pytest.raises(ValueError, match='non-zero size'):
    lt.contexts.NextStateTable(torch.zeros([0, 1], dtype=torch.int32))
  with pytest.raises(ValueError, match='should have shape'):
    lt.contexts.NextStateTable(torch.zeros([1], dtype=torch.int32))
  with pytest.raises(ValueError, match='int32'):
    lt.contexts.NextStateTable(torch.zeros([2, 3]))
  full = lt.contexts.FullNGram(vocab_size=3, context_size=2)
  table = full.next_state_table().to(torch.int32)
  assert tuple(table.shape) == (13, 3)
  ctx = lt.contexts.NextStateTable(table)
  assert ctx.shape() == (13, 3) and ctx.start() == 0
  states = torch.arange(13)[:, None]
  for y in range(4):
    np.testing.assert_array_equal(ctx.next_state(states, torch.full_like(states, y)).numpy(),
                                  full.next_state(states, torch.full_like(states, y)).numpy())
  w = torch.randn(2, 13, 3, dtype=torch.float64)
  for sr in (lt.semirings.Log, lt.semirings.MaxTropical, lt.semirings.Real):
    np.testing.assert_allclose(ctx.forward_reduce(w, sr).numpy(),
                               full.forward_reduce(w, sr).numpy(), rtol=1e-12, atol=1e-12)
  b = torch.randn(2, 13, dtype=torch.float64)
  np.testing.assert_array_equal(ctx.backward_broadcast(b).numpy(),
                                full.backward_broadcast(b).numpy())
  labels = torch.tensor([2, 0, 0, 3, 1])
  np.testing.assert_array_equal(ctx.walk_states(labels).numpy(), full.walk_states(labels).numpy())


def test_frame_label_dependent_host_matches_reference_fixtures():
  """The host FrameLabelDependent (the plugin surface) composed over frames
  reproduces the reference's FLD fixtures (den Log / MaxTropical, and the
  loss gradient through its backward)."""
  import last_torch_amd as lt
  from golden_cases import FLD_CASES, load_fld
  for case in FLD_CASES:
    c = load_fld(case)
    V, n, K = c['V'], c['n'], c['K']
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    align = lt.alignments.FrameLabelDependent(max_expansions=K)
    assert align.num_states() == K + 1 and align.lexical_next(K) is None
    W = torch.tensor(c['W'], dtype=torch.float64)
    nf = torch.tensor(c['num_frames'])
    B, T, C, _ = W.shape
    for sname in ('Log', 'MaxTropical'):
      sr = getattr(lt.semirings, sname)
      alpha = sr.ones([B, C], dtype=torch.float64)
      alpha = torch.where(torch.arange(C) == 0, alpha, sr.zeros([B, C], dtype=torch.float64))
      for t in range(T):
        nxt = align.forward(alpha, [W[:, t, :, 0]] * (K + 1), [W[:, t, :, 1:]] * (K + 1), ctx, sr)
        alpha = torch.where((t < nf)[:, None], nxt, alpha)
      d = sr.sum(alpha, dim=-1).numpy()
      np.testing.assert_allclose(d, c[f'den_{sname}'], rtol=1e-5, atol=1e-5)


# ---- tuple semirings (semirings.py:404-533), the reference's own checks
# (tests/semirings_test.py:256-385) restated
def _tree_equal(a, b):
  assert len(a) == len(b)
  for x, y in zip(a, b):
    np.testing.assert_array_equal(x.float().numpy(), y.float().numpy())


def test_expectation_basics():
  E = lt.semirings.LogLogExpectation
  one, zero = E.ones([]), E.zeros([])
  for wx in [E.weighted(torch.tensor([1.]), torch.tensor([2.])), one, zero]:
    _tree_equal(E.times(wx, one), wx)
    _tree_equal(E.times(one, wx), wx)
    _tree_equal(E.plus(wx, zero), wx)
    _tree_equal(E.plus(zero, wx), wx)


def test_expectation_shape_dtypes():
  E = lt.semirings.LogLogExpectation
  one = E.ones([1, 2], (torch.float32, torch.bfloat16))
  assert lt.semirings.value_shape(one) == (1, 2)
  assert lt.semirings.value_dtype(one) == (torch.float32, torch.bfloat16)
  zero = E.zeros([], (torch.bfloat16, torch.float32))
  assert lt.semirings.value_shape(zero) == ()
  assert lt.semirings.value_dtype(zero) == (torch.bfloat16, torch.float32)


def test_expectation_weighted_and_safety():
  E = lt.semirings.LogLogExpectation
  w, x = E.weighted(torch.log(torch.tensor([0., 1., 2.])), torch.log(torch.tensor([3., 4., 5.])))
  np.testing.assert_allclose(torch.exp(w), [0, 1, 2], rtol=1e-6)
  np.testing.assert_allclose(torch.exp(x), [0 * 3, 1 * 4, 2 * 5], rtol=1e-6)
  w, x = E.weighted(torch.tensor([-np.inf]), torch.tensor([np.inf]))
  assert w.item() == -np.inf and x.item() == -np.inf


def test_expectation_sum_and_entropy():
  E = lt.semirings.LogLogExpectation
  w, x = E.sum(E.weighted(torch.log(torch.tensor([[0., 1.], [2., 3.]])),
                          torch.log(torch.tensor([[4., 5.], [6., 7.]]))), axis=1)
  np.testing.assert_allclose(torch.exp(w), [1, 5], rtol=1e-6)
  np.testing.assert_allclose(torch.exp(x), [5, 33], rtol=1e-6)
  probs = torch.tensor([0.25, 0.25, 0.5])
  lp = torch.log(probs)
  wx = E.weighted(lp, torch.log(-lp))
  log_z, log_sum = E.sum(wx, axis=0)
  np.testing.assert_allclose(log_z, 0, atol=1e-7)
  np.testing.assert_allclose(torch.exp(log_sum), -torch.sum(probs * lp), rtol=1e-6)
  probs2 = torch.tensor([0.25, 0.5, 0.25])
  lp2 = torch.log(probs2)
  log_z, log_sum = E.sum(E.times(wx, E.weighted(lp2, torch.log(-lp2))), axis=0)
  np.testing.assert_allclose(torch.exp(log_z), torch.sum(probs * probs2), rtol=1e-6)
  entropy = log_z + torch.exp(log_sum - log_z)
  np.testing.assert_allclose(
      entropy, -torch.sum(probs * probs2 * torch.exp(-log_z) * (lp + lp2 - log_z)), rtol=0.2)


def test_cartesian():
  S = lt.semirings.Cartesian(lt.semirings.Real, lt.semirings.MaxTropical)
  one, zero = S.ones([]), S.zeros([])
  for wx in [(torch.tensor(1.0), torch.tensor(2.0)), one, zero]:
    _tree_equal(S.times(wx, one), wx)
    _tree_equal(S.times(one, wx), wx)
    _tree_equal(S.plus(wx, zero), wx)
    _tree_equal(S.plus(zero, wx), wx)
  one = S.ones([1, 2], (torch.float32, torch.bfloat16))
  assert lt.semirings.value_shape(one) == (1, 2)
  assert lt.semirings.value_dtype(one) == (torch.float32, torch.bfloat16)
  a, b = (torch.tensor(2.0), torch.tensor(1.0)), (torch.tensor(3.0), torch.tensor(4.0))
  c = (torch.tensor([1.0, 2.0]), torch.tensor([3.0, 4.0]))
  assert [v.item() for v in S.times(a, b)] == [6.0, 5.0]
  assert [v.item() for v in S.plus(a, b)] == [5.0, 4.0]
  assert [v.item() for v in S.sum(c, axis=0)] == [3.0, 4.0]
  assert [v.item() for v in S.prod(c, axis=0)] == [2.0, 7.0]


def test_cartesian_rejected_by_lattice():
  """Cartesian has no lattice path (the lattice's weights are single
  tensors); LogLogExpectation has one (tests/test_entropy.py)."""
  ctx = lt.contexts.FullNGram(vocab_size=2, context_size=1)
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
                              weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(
                                  torch.zeros([1, 3, 3])))
  with pytest.raises(NotImplementedError):
    lat._forward(None, torch.zeros([1, 1, 1]), torch.ones([1]),
                 lt.semirings.Cartesian(lt.semirings.Real, lt.semirings.MaxTropical))


def test_joint_weight_fn_host_paths():
  """On the CPU JointWeightFn takes the PyTorch path: forward_joint is the
  [..., C, V+1] concatenation of forward's (blank, lexical), and a per-state
  call (state given) picks the same rows (weight_fns.py:174-227)."""
  torch.manual_seed(0)
  V, H, C = 5, 16, 6
  wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=H)
  ctx = torch.randn([C, 8])
  frames = torch.randn([2, 7, 10])
  blank, lexical = wfn(ctx, frames)
  W = wfn.forward_joint(ctx, frames)
  assert W.shape == (2, 7, C, V + 1)
  assert torch.equal(W[..., 0], blank) and torch.equal(W[..., 1:], lexical)
  state = torch.tensor([[3] * 7, [1] * 7])
  b1, l1 = wfn(ctx, frames, state)
  torch.testing.assert_close(b1, torch.stack([blank[0, :, 3], blank[1, :, 1]]))
  torch.testing.assert_close(l1[1], lexical[1, :, 1])


@pytest.mark.parametrize('C,H,R,rows,ok', [
    (33, 512, 33, 64000, True),     # the bench head
    (33, 48, 33, 10, False),        # hidden % 32
    (33, 320, 33, 10, True),        # 10 column blocks of 2-wave workgroups
    (1057, 512, 33, 10, False),     # trigram: d_ctx_proj block exceeds LDS
    (33, 512, 65, 10, False),       # V + 1 > 64
    (33, 512, 33, 2 ** 26, False),  # rows * H >= 2^31
])
def test_joint_weights_backward_supported(C, H, R, rows, ok):
  from last_torch_amd import _native
  assert _native.joint_weights_backward_supported(C, H, R, rows) is ok
