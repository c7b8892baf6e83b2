"""Lattice entropy through the LogLogExpectation semiring (semirings.py:
405-484; the entropy use of tests/semirings_test.py:305-324):
``RecognitionLattice.entropy`` and ``_forward(..., LogLogExpectation)``.

Oracle: brute force over every alignment path of small bigram lattices
(each frame takes label y in 0..V from state p: y = 0 keeps p, y >= 1 moves
to y; frames past num_frames take none; every state is final), H = -sum p
log p with p = softmax of the path weights. The GPU path (the den backward
kernel's marginals) is checked against the same brute force and against the
CPU path at larger sizes."""
import itertools

import numpy as np
import pytest
import torch

import last_torch_amd as lt


def _lattice(W, V):
  return lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=1),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(W))


def _frames(B, T, device):
  return torch.arange(T, dtype=torch.float32, device=device)[None, :, None].expand(B, T, 1)


def _brute(W, nf, V):
  """(entropy, log_z) per utterance by enumerating every path."""
  W = W.double().cpu().numpy()
  out = []
  for b in range(W.shape[0]):
    ws = []
    for ys in itertools.product(range(V + 1), repeat=int(nf[b])):
      p, w = 0, 0.0
      for t, y in enumerate(ys):
        w += W[b, t, p, y]
        p = p if y == 0 else y
      ws.append(w)
    ws = np.array(ws)
    lz = np.log(np.exp(ws - ws.max()).sum()) + ws.max()
    pr = np.exp(ws - lz)
    out.append((-(pr * np.log(pr)).sum(), lz))
  return np.array(out)


def _case(seed=0, B=3, T=5, V=2, log_probs=False):
  g = torch.Generator().manual_seed(seed)
  W = torch.randn([B, T, V + 1, V + 1], generator=g)
  if log_probs:
    W = torch.log_softmax(W, dim=-1)
  nf = torch.tensor([T, T - 2, 1][:B])
  return W, nf


def check_entropy(device):
  for seed, log_probs in ((0, False), (1, True)):
    W, nf = _case(seed, log_probs=log_probs)
    V = W.shape[-1] - 1
    ref = _brute(W, nf, V)
    lat = _lattice(W.to(device), V)
    H = lat.entropy(_frames(W.shape[0], W.shape[1], device), nf)
    np.testing.assert_allclose(H.cpu().numpy(), ref[:, 0], rtol=1e-5, atol=1e-5)
    (log_z, log_sum), alpha = lat._forward(None, _frames(W.shape[0], W.shape[1], device), nf,
                                           lt.semirings.LogLogExpectation)
    assert alpha is None
    np.testing.assert_allclose(log_z.cpu().numpy(), ref[:, 1], rtol=1e-5, atol=1e-5)
    if log_probs:  # v = -w >= 0: the pair is finite and entropy = log_z + exp(log_sum - log_z)
      Hx = (log_z + torch.exp(log_sum - log_z)).cpu().numpy()
      np.testing.assert_allclose(Hx, ref[:, 0], rtol=1e-5, atol=1e-5)


def test_entropy_cpu():
  check_entropy('cpu')


@pytest.mark.gpu
def test_entropy_gpu(cuda):
  check_entropy(cuda)


@pytest.mark.gpu
def test_entropy_gpu_matches_cpu_path(cuda):
  """B=4, T=60, V=32 bigram: the HIP marginals' entropy against the CPU path's."""
  g = torch.Generator().manual_seed(7)
  W = torch.randn([4, 60, 33, 33], generator=g)
  nf = torch.tensor([60, 41, 7, 60])
  H_cpu = _lattice(W, 32).entropy(_frames(4, 60, 'cpu'), nf)
  H_gpu = _lattice(W.to(cuda), 32).entropy(_frames(4, 60, cuda), nf)
  np.testing.assert_allclose(H_gpu.cpu().numpy(), H_cpu.numpy(), rtol=1e-4, atol=1e-4)
