"""lt_loss_grad captured into a HIP graph and replayed with new arc weights.

The chunked scan's and the fused pipe's inter-workgroup hand-off words carry
a per-call tag chosen on the host. A captured graph replays the tag it was
captured with, so the library zeroes those words by a memset node whenever
the caller's stream is capturing. Each replay here runs on different W and
must give the same bits as an eager call on that W (every design is
deterministic), so a replay that read the previous replay's hand-off words
(stale records, a stale boundary state) fails.
"""
import ctypes

import pytest
import torch

from last_torch_amd import _native as nat

pytestmark = pytest.mark.gpu


def _inputs(B, T, U, V, device, seed):
  g = torch.Generator(device=device)
  g.manual_seed(seed)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device=device)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=device, dtype=torch.int32)
  nf = torch.randint(T // 2, T + 1, [B], generator=g, device=device, dtype=torch.int32)
  nl = torch.randint(U // 2, U + 1, [B], generator=g, device=device, dtype=torch.int32)
  return W, nf, lab, nl


@pytest.mark.parametrize('design,B', [('chunk', 48), ('fused', 48), ('checkpoints', 48),
                                      ('auto', 256)])
def test_loss_grad_graph_replays_match_eager(cuda, design, B):
  V, n, T, U = 32, 1, 400, 60
  d = {'auto': nat.DESIGN_AUTO, 'chunk': nat.DESIGN_CHUNK, 'fused': nat.DESIGN_FUSED_PIPE,
       'checkpoints': nat.DESIGN_CHECKPOINTS}[design]
  W, nf, lab, nl = _inputs(B, T, U, V, cuda, seed=1)
  pb = nat._problem(W, V, n, U)
  nbytes = nat.loss_grad_workspace_bytes(W, V, n, U, False, d)
  ws = torch.empty([max(nbytes, 1)], dtype=torch.uint8, device=cuda)
  loss, lz, num = (torch.empty([B], device=cuda) for _ in range(3))
  dW = torch.empty_like(W)

  def call():
    nat._check(nat.lib().lt_loss_grad_ex(
        ctypes.byref(pb), 0, d, nat._ptr(W), nat._ptr(nf), nat._ptr(lab), nat._ptr(nl),
        nat._ptr(loss), nat._ptr(lz), nat._ptr(num), nat._ptr(dW), nat._ptr(ws), ws.numel(),
        nat._stream()), 'lt_loss_grad_ex')

  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    call()  # eager on the side stream first, as torch's capture recipe does
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    call()
  for seed in (2, 3, 4):
    W2 = _inputs(B, T, U, V, cuda, seed=seed)[0]
    W.copy_(W2)
    g.replay()
    torch.cuda.synchronize()
    rl, rlz, rnum, rdW = nat.loss_grad(W2, nf, lab, nl, V, n, False, design=d)
    torch.cuda.synchronize()
    assert torch.equal(loss, rl), (seed, float((loss - rl).abs().max()))
    assert torch.equal(lz, rlz) and torch.equal(num, rnum)
    assert torch.equal(dW, rdW), (seed, float((dW - rdW).abs().max()))
  # and the replays did see the new weights (a graph that ignored W would
  # match eager only on the captured W)
  assert not torch.equal(rl, nat.loss_grad(_inputs(B, T, U, V, cuda, seed=1)[0], nf, lab, nl,
                                           V, n, False, design=d)[0])
