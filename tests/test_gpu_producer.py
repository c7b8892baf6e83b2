"""GPU tests of the joint weight function's matrix-core producer
(lt_joint_weights / lt_joint_weights_ex, lt_producer.hip; SURVEY.md 8(f)
rank 1).

Numerics reference: a plain PyTorch fp32 restatement of JointWeightFn
(weight_fns.py:174-227): W = bias + tanh(pc[c] + pf[f]) @ wo^T.
* precision 'bf16' feeds the tanh values and wo to the matrix cores as bf16
  (8 significant bits) and sums in fp32, so each logit may differ from fp32
  by the bf16 rounding of its products: |dW| <= 2^-7 * (|tanh| @ |wo|^T) +
  1e-5 (`_tol`). Against a bf16-emulating reference (the same roundings,
  fp32 sums) the difference is summation order plus the rare bf16 rounding
  flip of a tanh value: checked on the mean.
* precision 'fp32' (the default, LT_JOINT_SPLIT) splits both into bf16
  hi + lo and sums hi*hi + hi*lo + lo*hi: each product carries ~2^-17
  relative error, so |dW| <= 2^-14 * (|tanh| @ |wo|^T) + 1e-5 (`_tol32`),
  i.e. fp32 autograd parity at 1e-4 of the logits' scale.
The backward is fp32 (recomputed tanh): against torch autograd of the fp32
formula, 1e-4 relative.
"""
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat

pytestmark = pytest.mark.gpu


def _ref(pc, pf, wo, bias, bf16=False):
  hid = torch.tanh(pc[None] + pf.reshape(-1, pf.shape[-1])[:, None, :])
  w = wo
  if bf16:
    hid = hid.bfloat16().float()
    w = wo.bfloat16().float()
  W = torch.matmul(hid, w.t()) + bias
  return W.reshape(*pf.shape[:-1], pc.shape[0], wo.shape[0]), hid


def _tol(pc, pf, wo):
  hid = torch.tanh(pc[None] + pf.reshape(-1, pf.shape[-1])[:, None, :]).abs()
  return 2.0 ** -7 * torch.matmul(hid, wo.abs().t()).reshape(
      *pf.shape[:-1], pc.shape[0], wo.shape[0]) + 1e-5


def _tol32(pc, pf, wo):
  return _tol(pc, pf, wo) * 2.0 ** -7 + 1e-5


def _inputs(cuda, lead, C, H, R, scale=1.0, seed=0):
  g = torch.Generator(device=cuda)
  g.manual_seed(seed)
  pc = scale * torch.randn([C, H], generator=g, device=cuda)
  pf = scale * torch.randn([*lead, H], generator=g, device=cuda)
  wo = torch.randn([R, H], generator=g, device=cuda) / H ** 0.5
  bias = torch.randn([R], generator=g, device=cuda)
  return pc, pf, wo, bias


@pytest.mark.parametrize('lead,C,H,R', [
    ((4, 7), 33, 64, 33),     # bigram V=32 (two column tiles, the second with 1 column)
    ((3, 5), 1, 16, 6),       # n = 0, V = 5
    ((2, 9), 17, 48, 17),     # one column tile
    ((1, 1), 33, 16, 64),     # full two tiles
    ((5, 13), 21, 512, 33),   # H = 512 (the bench hidden size), ragged rows
    ((37,), 33, 32, 33),      # rows * C not a multiple of 32
    ((2, 3), 5, 848, 33),     # frame block exceeds LDS: the row-tile kernel
])
def test_forward_vs_torch(cuda, lead, C, H, R):
  pc, pf, wo, bias = _inputs(cuda, lead, C, H, R)
  W = nat.joint_weights(pc, pf, wo, bias, precision='bf16')
  torch.cuda.synchronize()
  ref, _ = _ref(pc, pf, wo, bias)
  assert W.shape == ref.shape
  assert bool(((W - ref).abs() <= _tol(pc, pf, wo)).all())
  emu, _ = _ref(pc, pf, wo, bias, bf16=True)
  assert float((W - emu).abs().mean()) < 1e-4 * max(1.0, float(emu.abs().mean()))


@pytest.mark.parametrize('lead,C,H,R', [
    ((4, 7), 33, 64, 33),     # bigram V=32 (two column tiles)
    ((3, 5), 1, 16, 6),       # n = 0, V = 5
    ((1, 1), 33, 16, 64),     # full two tiles
    ((5, 13), 21, 512, 33),   # H = 512 (the bench hidden size), ragged rows
    ((37,), 33, 32, 33),      # rows * C not a multiple of 32
    ((2, 3), 5, 848, 33),     # frame block exceeds LDS: the row-tile kernel
])
@pytest.mark.parametrize('scale', [1.0, 30.0])  # split e^{2a} e^{2b} / direct e^{2(a+b)}
def test_forward_fp32_faithful(cuda, lead, C, H, R, scale):
  """precision 'fp32' (split-bf16 products): fp32 parity at 2^-14 of the
  logits' product scale, ~128x tighter than the bf16 bound."""
  pc, pf, wo, bias = _inputs(cuda, lead, C, H, R, scale=scale)
  W = nat.joint_weights(pc, pf, wo, bias, precision='fp32')
  torch.cuda.synchronize()
  ref, _ = _ref(pc, pf, wo, bias)
  assert W.shape == ref.shape
  err = (W - ref).abs()
  assert bool((err <= _tol32(pc, pf, wo)).all()), float((err / _tol32(pc, pf, wo)).max())
  Wb = nat.joint_weights(pc, pf, wo, bias, precision='bf16')
  assert float(err.mean()) * 16 < float((Wb - ref).abs().mean()) + 1e-7


@pytest.mark.parametrize('scale', [8.0, 30.0])  # split path (|x| <= 40) / direct path
def test_forward_bf16_output_and_saturation(cuda, scale):
  pc, pf, wo, bias = _inputs(cuda, (3, 11), 33, 64, 33, scale=scale)  # tanh saturates
  W = nat.joint_weights(pc, pf, wo, bias, dtype=torch.bfloat16, precision='bf16')
  ref, _ = _ref(pc, pf, wo, bias)
  assert W.dtype == torch.bfloat16
  assert bool(torch.isfinite(W.float()).all())
  tol = _tol(pc, pf, wo) + 2.0 ** -8 * ref.abs()
  assert bool(((W.float() - ref).abs() <= tol).all())


def test_split_and_direct_paths_agree(cuda):
  """One projection above 40 switches the whole call to the direct path; the
  other rows must come out as on the split path up to bf16 rounding of tanh."""
  pc, pf, wo, bias = _inputs(cuda, (2, 9), 33, 64, 33, scale=3.0)
  W = nat.joint_weights(pc, pf, wo, bias, precision='bf16')
  pf2 = pf.clone()
  pf2[1, 8, 0] = 50.0
  W2 = nat.joint_weights(pc, pf2, wo, bias, precision='bf16')
  torch.cuda.synchronize()
  assert bool(((W[:1] - W2[:1]).abs() <= _tol(pc, pf[:1], wo)).all())
  ref, _ = _ref(pc, pf2, wo, bias)
  assert bool(((W2 - ref).abs() <= _tol(pc, pf2, wo)).all())
  pf3 = pf.clone()
  pf3[0, 0, 0] = float('nan')
  W3 = nat.joint_weights(pc, pf3, wo, bias, precision='bf16')
  torch.cuda.synchronize()
  assert bool(torch.isnan(W3[0, 0]).all()) and bool(torch.isfinite(W3[1]).all())


def test_empty_and_errors(cuda):
  pc, pf, wo, bias = _inputs(cuda, (0, 5), 33, 16, 33)
  assert nat.joint_weights(pc, pf, wo, bias).shape == (0, 5, 33, 33)
  pc, pf, wo, bias = _inputs(cuda, (2, 3), 33, 20, 33)   # hidden not a multiple of 16
  with pytest.raises(nat.LatticeLibraryError):
    nat.joint_weights(pc, pf, wo, bias)
  pc, pf, wo, bias = _inputs(cuda, (2, 3), 33, 16, 65)   # V + 1 > 64
  with pytest.raises(nat.LatticeLibraryError):
    nat.joint_weights(pc, pf, wo, bias)


@pytest.mark.parametrize('lead,C,H,R', [
    ((3, 50), 33, 64, 33),    # bigram V=32: second column block holds one row
    ((2, 7), 1, 32, 6),       # n = 0, V = 5: 32 frames per tile
    ((5, 9), 17, 96, 17),     # three waves, one K block pair
    ((4, 3), 5, 32, 64),      # two full column blocks
    ((2, 40), 33, 512, 33),   # bench hidden size: two workgroups per tile column
    ((37,), 3, 288 - 32, 16), # hidden 256 exactly, rows * C not a multiple of 32
    ((3, 11), 9, 320, 40),    # 2-wave workgroups over 5 column blocks, R in (32, 48]
    ((3, 20), 33, 128, 33),   # 4-wave workgroups (g split in each wave)
])
@pytest.mark.parametrize('path', ['kernel', 'torch'])
def test_backward_vs_torch(cuda, lead, C, H, R, path):
  """lt_joint_weights_backward (split-bf16 products) and the chunked PyTorch
  fallback both match fp32 autograd of the reference formula within 1e-4 of
  each gradient's scale."""
  pc, pf, wo, bias = _inputs(cuda, lead, C, H, R)
  g = torch.randn([*lead, C, R], device=cuda)
  leaves = [t.clone().requires_grad_(True) for t in (pc, pf, wo, bias)]
  if path == 'kernel':
    assert nat.joint_weights_backward_supported(C, H, R)
    W = lt.weight_fns._JointWeightsFn.apply(*leaves, 37, 'fp32')
    (W * g).sum().backward()
  else:
    grads = _torch_backward(pc, pf, wo, g, chunk=37)
    for t, gr in zip(leaves, grads):
      t.grad = gr
  ref_leaves = [t.clone().requires_grad_(True) for t in (pc, pf, wo, bias)]
  ref, _ = _ref(*ref_leaves)
  (ref * g).sum().backward()
  for name, a, b in zip(('pc', 'pf', 'wo', 'bias'), leaves, ref_leaves):
    scale = float(b.grad.abs().max())
    err = float((a.grad - b.grad).abs().max())
    assert err <= 1e-4 * max(1.0, scale), (name, err, scale)


def _torch_backward(pc, pf, wo, g, chunk):
  """The fallback branch of _JointWeightsFn.backward, forced."""
  class Ctx:
    pass
  ctx = Ctx()
  ctx.saved_tensors = (pc, pf, wo)
  ctx.chunk = chunk
  orig = nat.joint_weights_backward_supported
  nat.joint_weights_backward_supported = lambda *a, **k: False
  try:
    return lt.weight_fns._JointWeightsFn.backward(ctx, g)[:4]
  finally:
    nat.joint_weights_backward_supported = orig


def test_backward_errors_and_empty(cuda):
  pc, pf, wo, bias = _inputs(cuda, (0, 4), 33, 64, 33)
  dpc, dpf, dwo, db = nat.joint_weights_backward(pc, pf, wo, torch.zeros([0, 4, 33, 33], device=cuda))
  assert dpf.shape == (0, 4, 64) and float(dpc.abs().sum()) == 0 and float(dwo.abs().sum()) == 0
  assert db.shape == (33,) and float(db.abs().sum()) == 0
  assert not nat.joint_weights_backward_supported(33, 48, 33)     # hidden % 32
  assert nat.joint_weights_backward_supported(33, 320, 33)        # 10 column blocks: 5 x 2 waves
  assert not nat.joint_weights_backward_supported(1057, 512, 33)  # d_ctx_proj exceeds LDS
  pc, pf, wo, bias = _inputs(cuda, (2, 3), 33, 48, 33)
  with pytest.raises(nat.LatticeLibraryError):
    nat.joint_weights_backward(pc, pf, wo, torch.zeros([2, 3, 33, 33], device=cuda))


@pytest.mark.parametrize('precision,rtol', [('fp32', 1e-4), ('bf16', 2e-2)])
def test_joint_weight_fn_in_lattice(cuda, precision, rtol):
  """RecognitionLattice with SharedEmbCacher + JointWeightFn: the fused
  producer and the PyTorch fp32 path give the same loss (1e-4 relative with
  the default fp32-faithful products, the bf16 product tolerance with
  precision='bf16'), and gradients reach every parameter."""
  torch.manual_seed(0)
  V, n, H, B, T, U = 8, 1, 32, 3, 12, 4
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=16,
                                         device=cuda)
  fused = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=H, device=cuda,
                                      precision=precision)
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: cacher,
                              weight_fn_factory=lambda _: fused)
  frames = torch.randn([B, T, 10], device=cuda)
  nf = torch.tensor([T, T - 3, 5], device=cuda)
  labels = torch.randint(1, V + 1, [B, U], device=cuda)
  nl = torch.tensor([U, 2, 3], device=cuda)
  loss = lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl)
  loss.sum().backward()
  fused.fused = False
  grads = {k: p.grad.clone() for k, p in fused.named_parameters()}
  for p in fused.parameters():
    p.grad = None
  loss_ref = lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl)
  loss_ref.sum().backward()
  assert torch.allclose(loss, loss_ref, rtol=rtol, atol=rtol), (loss, loss_ref)
  for k, p in fused.named_parameters():
    assert torch.isfinite(grads[k]).all() and grads[k].abs().sum() > 0, k
    gt = 10 * rtol if precision == 'fp32' else 5e-2
    assert torch.allclose(grads[k], p.grad, rtol=gt, atol=gt * float(p.grad.abs().max())), k
