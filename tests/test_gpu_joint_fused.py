"""The joint weight function fused into the lattice loss (lt_loss_grad_joint,
lt_joint.hip): JointWeightFn's arc weights
(weight_fns.py:174-227) formed on the matrix cores inside the recursions'
helper waves and the marginal pass, the parameter gradients formed from the
marginals in LDS -- W and dW never in HBM.

* Against the separate launches on the materialised W: lt_joint_weights_ex
  (the same precision) -> lt_loss_grad (the checkpointing design, whose
  kernels the fused path shares) -> lt_joint_weights_backward. The fused W is
  the producer's bit for bit, so loss, log_z and num must be bit-identical;
  d_frame_proj agrees to fp32 rounding (the compiler may contract the
  marginals' arithmetic differently in the two kernels: a few ulp);
  d_ctx_proj / d_out_weight / d_out_bias are sums over the blocks in another
  grouping (fp32 rounding only).
* Against the oracle on the materialised W (the loss, 1e-4 as north_star).
* Against fp32 PyTorch autograd of the reference formulation (hidden tensor
  in fp32, the lattice gradient from the checkpointing kernels on that W):
  loss 1e-4, parameter gradients 1e-3 of their scale (the producer's bounds,
  tests/test_gpu_producer.py).
"""
import math

import numpy as np
import pytest
import torch

from last_torch_amd import _native as nat
from golden_cases import assert_loss_close

pytestmark = pytest.mark.gpu


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _problem(B, T, U, H, device, seed, V=32, varlen=True, scale=0.5):
  g = torch.Generator(device=device)
  g.manual_seed(seed)
  C = R = V + 1
  pc = torch.randn([C, H], generator=g, device=device) * scale
  pf = torch.randn([B, T, H], generator=g, device=device) * scale
  wo = torch.randn([R, H], generator=g, device=device) * (2.0 / math.sqrt(H))
  bias = torch.randn([R], generator=g, device=device) * 0.1
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=device, dtype=torch.int32)
  if varlen:
    nf = torch.randint(T // 2, T + 1, [B], generator=g, device=device, dtype=torch.int32)
    nl = torch.randint(U // 2, U + 1, [B], generator=g, device=device, dtype=torch.int32)
    nf[0], nl[0] = T, U
  else:
    nf = torch.full([B], T, dtype=torch.int32, device=device)
    nl = torch.full([B], U, dtype=torch.int32, device=device)
  return pc, pf, wo, bias, nf, lab, nl


def _separate(pc, pf, wo, bias, nf, lab, nl, gin, precision):
  """The separate launches: producer -> lattice (checkpointing) -> producer backward."""
  W = nat.joint_weights(pc, pf, wo, bias, precision=precision)
  # the checkpointing pair with the incoming gradient inside the marginal
  # pass (pipe_kernel, then marg_kernel: the kernels the fused path shares)
  loss, lz, num, alpha, an, ck = nat.loss_forward(W, nf, lab, nl, 32, 1, False, checkpoints=True)
  dW = nat.loss_backward(W, nf, lab, nl, lz, num, alpha, an, gin.float().contiguous(), 32, 1, False,
                         ck=ck)
  dpc, dpf, dwo, dbias = nat.joint_weights_backward(pc, pf, wo, dW)
  return W, loss, lz, num, dpc, dpf, dwo, dbias


def _close(got, ref, rtol):
  scale = float(ref.abs().max()) + 1e-30
  err = float((got - ref).abs().max())
  assert err <= rtol * scale, (err, scale)


@pytest.mark.parametrize('H', [32, 64, 128])
@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_fused_matches_separate_launches(cuda, H, precision):
  B, T, U = 12, 233, 37  # T not a multiple of 32: blocks end inside an utterance
  pc, pf, wo, bias, nf, lab, nl = _problem(B, T, U, H, cuda, seed=H)
  gin = torch.linspace(0.5, 2.0, B, device=cuda)
  out = nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl, grad=gin, precision=precision)
  loss, lz, num, dpc, dpf, dwo, dbias = out
  W, rl, rlz, rnum, rdpc, rdpf, rdwo, rdbias = _separate(pc, pf, wo, bias, nf, lab, nl, gin,
                                                         precision)
  torch.cuda.synchronize()
  assert torch.equal(loss, rl), float((loss - rl).abs().max())
  assert torch.equal(lz, rlz) and torch.equal(num, rnum)
  _close(dpf, rdpf, 1e-5)
  for got, ref in ((dpc, rdpc), (dwo, rdwo), (dbias, rdbias)):
    _close(got, ref, 1e-5)
  # the loss against the oracle on the materialised W
  orc = _orc()
  rl2, _, _, _ = orc.loss_grad(W.cpu().numpy(), nf.cpu().numpy(), lab.cpu().numpy(),
                               nl.cpu().numpy(), 32, 1, want_grad=False)
  assert_loss_close(loss.cpu().numpy(), rl2)


@pytest.mark.parametrize('H', [32, 128])
def test_fused_matches_fp32_autograd(cuda, H):
  """Against the reference formulation in fp32: W from PyTorch's hidden
  tensor, the lattice gradient (the checkpointing kernels on that W) pulled
  back through PyTorch autograd to the parameters."""
  B, T, U = 6, 160, 30
  pc, pf, wo, bias, nf, lab, nl = _problem(B, T, U, H, cuda, seed=7 + H)
  loss, _, _, dpc, dpf, dwo, dbias = nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl)
  ps = [x.clone().requires_grad_(True) for x in (pc, pf, wo, bias)]
  hid = torch.tanh(ps[0][None, None] + ps[1][:, :, None, :])  # [B, T, C, H] fp32
  W = hid @ ps[2].t() + ps[3]
  rl, _, _, dW = nat.loss_grad(W.detach().contiguous(), nf, lab, nl, 32, 1, False,
                               design=nat.DESIGN_CHECKPOINTS)
  (W * dW).sum().backward()
  torch.cuda.synchronize()
  np.testing.assert_allclose(loss.cpu().numpy(), rl.cpu().numpy(), rtol=1e-4, atol=1e-3)
  for got, p in zip((dpc, dpf, dwo, dbias), ps):
    _close(got, p.grad, 1e-3)


def test_fused_forward_backward_split_and_edge_cases(cuda):
  """lt_loss_joint_forward then lt_loss_joint_backward (what the autograd
  Function calls) equal the one-call form; an unreachable string (num_labels
  beyond what its frames can emit) and a zero-length utterance give zero
  gradient rows and finite sums; the backward reruns from the same state."""
  B, T, U, H = 5, 64, 20, 32
  pc, pf, wo, bias, nf, lab, nl = _problem(B, T, U, H, cuda, seed=3, varlen=False)
  nf[2] = 5    # 20 labels in 5 frames: unreachable, loss = +inf
  nf[3] = 0
  nl[3] = 0
  gin = torch.tensor([1.0, -0.5, 2.0, 1.0, 0.25], device=cuda)
  one = nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl, grad=gin)
  loss, lz, num, state = nat.joint_loss_forward(pc, pf, wo, bias, nf, lab, nl)
  g1 = nat.joint_loss_backward(pc, pf, wo, bias, nf, lab, state, grad=gin)
  g2 = nat.joint_loss_backward(pc, pf, wo, bias, nf, lab, state, grad=gin)
  torch.cuda.synchronize()
  assert torch.equal(loss, one[0])
  assert torch.isinf(loss[2]) and loss[3] == 0
  for a, b2, c in zip(g1, g2, one[3:]):
    assert torch.equal(a, b2) and torch.equal(a, c)
  dpf = g1[1]
  assert (dpf[2] == 0).all() and (dpf[3] == 0).all()
  assert all(torch.isfinite(x).all() for x in g1)
  W, rl, _, _, rdpc, rdpf, rdwo, rdbias = _separate(pc, pf, wo, bias, nf, lab, nl, gin, 'fp32')
  _close(dpf, rdpf, 1e-5)
  for got, ref in zip((g1[0], g1[2], g1[3]), (rdpc, rdwo, rdbias)):
    _close(got, ref, 1e-5)


@pytest.mark.parametrize('H', [32, 64])
def test_recognition_lattice_with_fused_joint_weight_fn(cuda, H):
  """RecognitionLattice(SharedEmbCacher + JointWeightFn(lattice_fusion='on'))
  -- the drop-in API, weight_fns.py:174-242 -- forward and backward through
  the fused kernels against lattice_fusion='off' (W materialised by the
  matrix-core producer, the lattice's own design, the producer's backward):
  the loss and every parameter's gradient (the projections' weights through
  PyTorch autograd from d_ctx_proj / d_frame_proj)."""
  import last_torch_amd as lt
  torch.manual_seed(0)
  V, B, T, U, F = 32, 4, 120, 20, 48
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=1)
  cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=24, device=cuda)
  wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=H, device=cuda)
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: cacher,
                              weight_fn_factory=lambda _: wfn)
  frames = torch.randn([B, T, F], device=cuda)
  nf = torch.tensor([T, T - 7, 60, 1], device=cuda)
  labels = torch.randint(1, V + 1, [B, U], device=cuda)
  nl = torch.tensor([U, 15, 11, 0], device=cuda)
  w = torch.tensor([1.0, 0.5, -1.0, 2.0], device=cuda)
  lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl)  # materialise the lazy layers
  params = [p for p in list(cacher.parameters()) + list(wfn.parameters())]
  out = {}
  for mode in ('on', 'off'):
    wfn.lattice_fusion = mode
    for p in params:
      p.grad = None
    loss = lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl)
    (w * loss).sum().backward()
    out[mode] = (loss.detach().clone(), [p.grad.clone() for p in params])
  torch.cuda.synchronize()
  np.testing.assert_allclose(out['on'][0].cpu().numpy(), out['off'][0].cpu().numpy(), rtol=1e-5,
                             atol=1e-3)
  for a, b in zip(out['on'][1], out['off'][1]):
    _close(a, b, 1e-4)


@pytest.mark.parametrize('H', [32, 128])
def test_fused_at_bench_shape_against_oracle(cuda, H):
  """The shapes r05_joint_step.jsonl times (B=64, T=1000, U=100): the fused
  loss against the oracle on the materialised W (the producer's W in the same
  precision, bit-identical to the fused one), and the parameter gradients
  against PyTorch fp32 autograd of the reference formulation pulled back from
  the ORACLE's dW (orc.loss_grad), not the product's; plus the separate
  launches at this shape."""
  B, T, U = 64, 1000, 100
  pc, pf, wo, bias, nf, lab, nl = _problem(B, T, U, H, cuda, seed=100 + H, varlen=False)
  out = nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl)
  loss, lz, num, dpc, dpf, dwo, dbias = out
  W = nat.joint_weights(pc, pf, wo, bias, precision='fp32')
  torch.cuda.synchronize()
  orc = _orc()
  rl, rlz, rnum, rdW = orc.loss_grad(W.cpu().numpy(), nf.cpu().numpy(), lab.cpu().numpy(),
                                     nl.cpu().numpy(), 32, 1)
  assert_loss_close(loss.cpu().numpy(), rl)
  assert_loss_close(lz.cpu().numpy(), rlz)
  assert_loss_close(num.cpu().numpy(), rnum)
  ps = [x.clone().requires_grad_(True) for x in (pc, pf, wo, bias)]
  hid = torch.tanh(ps[0][None, None] + ps[1][:, :, None, :])  # [B, T, C, H] fp32
  Wr = hid @ ps[2].t() + ps[3]
  (Wr * torch.from_numpy(rdW).to(cuda)).sum().backward()
  del hid, Wr
  for got, p in zip((dpc, dpf, dwo, dbias), ps):
    _close(got, p.grad, 1e-3)
  _, sl, _, _, sdpc, sdpf, sdwo, sdbias = _separate(pc, pf, wo, bias, nf, lab, nl,
                                                    torch.ones([B], device=cuda), 'fp32')
  assert torch.equal(loss, sl)
  for got, ref in ((dpc, sdpc), (dpf, sdpf), (dwo, sdwo), (dbias, sdbias)):
    _close(got, ref, 1e-5)


def test_fused_largest_hidden_and_unsupported_fallback(cuda):
  """joint_loss_supported asks the library (its LDS rule): at
  U = 100 the split-product marginal pass fits up to H = 192 and not at 224 /
  256. H = 192 (six backward waves) runs against the separate launches; an
  H = 256 JointWeightFn with lattice_fusion='on' falls back to the separate
  launches instead of raising."""
  import last_torch_amd as lt
  U = 100
  assert nat.joint_loss_supported(4, 64, U, 32, 1, 192)
  assert not nat.joint_loss_supported(4, 64, U, 32, 1, 224)
  assert not nat.joint_loss_supported(4, 64, U, 32, 1, 256)
  assert nat.joint_loss_supported(4, 64, U, 32, 1, 224, precision='bf16')
  B, T, H = 4, 300, 192
  pc, pf, wo, bias, nf, lab, nl = _problem(B, T, U, H, cuda, seed=192)
  gin = torch.tensor([1.0, 0.5, -1.0, 2.0], device=cuda)
  loss, lz, num, dpc, dpf, dwo, dbias = nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl,
                                                            grad=gin)
  _, rl, rlz, rnum, rdpc, rdpf, rdwo, rdbias = _separate(pc, pf, wo, bias, nf, lab, nl, gin, 'fp32')
  torch.cuda.synchronize()
  assert torch.equal(loss, rl) and torch.equal(lz, rlz) and torch.equal(num, rnum)
  for got, ref in ((dpc, rdpc), (dpf, rdpf), (dwo, rdwo), (dbias, rdbias)):
    _close(got, ref, 1e-5)
  # the drop-in API at H = 256: 'on' cannot fuse here, so the separate launches run
  V, F = 32, 16
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=1)
  cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=8, device=cuda)
  wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=256, device=cuda,
                                    lattice_fusion='on')
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: cacher,
                              weight_fn_factory=lambda _: wfn)
  frames = torch.randn([2, 40, F], device=cuda)
  nf2 = torch.tensor([40, 31], device=cuda)
  lab2 = torch.randint(1, V + 1, [2, U], device=cuda)
  nl2 = torch.tensor([12, 9], device=cuda)
  l_on = lat(frames=frames, num_frames=nf2, labels=lab2, num_labels=nl2)
  wfn.lattice_fusion = 'off'
  l_off = lat(frames=frames, num_frames=nf2, labels=lab2, num_labels=nl2)
  torch.cuda.synchronize()
  assert torch.equal(l_on, l_off)
