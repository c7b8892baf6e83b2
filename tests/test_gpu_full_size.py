"""GPU parity of the exact launches bench.py times, at the BASELINE sizes.

* cfg2 (configs[1]): lt_loss_grad at B=64, T=1000, U=100, V=32 bigram fp32 --
  the bench step's launch (the chunked two-level scan, lt_chunk.hip) -- every
  utterance against the C oracle, plus size-independent properties
  (per-frame marginal sums, determinism, linearity in the incoming gradient).
* the same shape with realistic weights: log_softmax(sigma * randn) rows
  (weight_fns.py:120-136) and masked (-inf) arcs (lattices.py:450-453).
* north star: B=256 of the same shape (64 utterances + properties), in
  the design lt_loss_grad picks there and in the chunked scan forced.
* cfg4: MaxTropical Viterbi at B=64, T=2000: labels and path weights
  bit-exact on every utterance.
* cfg5: trigram (C = 1057) bf16 at B=32, T=1000, U=100: loss and every dW
  element on sixteen utterances, frame sums on all 32.
* the chunked path's fallback: utterances whose frames leave its fast path
  (NaN-free but wide or masked frames; a frame spanning 200) mixed into a batch.

dW is checked element by element relative to its own arc marginals
(golden_cases.marginal_scale): |got - ref| <= 1e-8 + (1e-4 + 4 * 2^-24 *
max(1, |log_z|, |num|)) * (den + num), so a wrong low-probability arc fails
(tests/test_oracle_golden.py has the negative control).
"""
import numpy as np
import pytest
import torch

from last_torch_amd import _native as nat
from golden_cases import assert_grad_marginal_close, assert_loss_close

pytestmark = pytest.mark.gpu


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _bench_inputs(B, T, U, V, n, device, seed, dtype=torch.float32, varlen=False):
  """bench.make_inputs: randn arc weights, uniform labels."""
  g = torch.Generator(device=device)
  g.manual_seed(seed)
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], generator=g, device=device, dtype=torch.float32).to(dtype)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=device, dtype=torch.int32)
  if varlen:
    nf = torch.randint(T // 2, T + 1, [B], generator=g, device=device, dtype=torch.int32)
    nl = torch.randint(U // 2, U + 1, [B], generator=g, device=device, dtype=torch.int32)
  else:
    nf = torch.full([B], T, dtype=torch.int32, device=device)
    nl = torch.full([B], U, dtype=torch.int32, device=device)
  return W, nf, lab, nl


def _np(*xs):
  return [x.float().cpu().numpy() if x.is_floating_point() else x.cpu().numpy() for x in xs]


def _frame_sums(dW):
  """Per (b, t): sum of dW over the frame's arcs (den marginals sum to 1,
  num marginals to 1, so live frames give 0)."""
  return dW.double().reshape(dW.shape[0], dW.shape[1], -1).sum(-1)


def _frame_sum_tol(lz, num=None, bf16=False):
  """The frame sum's bound from marginal_scale: the den and num marginals
  of a frame each sum to 1, so sum |err| <= 2 * rel + 1e-8 * arcs."""
  mag = lz.abs().double().nan_to_num(posinf=0.0, neginf=0.0).clamp(min=1.0)
  if num is not None:
    mag = torch.maximum(mag, num.abs().double().nan_to_num(posinf=0.0, neginf=0.0))
  rel = 1e-4 + 4 * 2.0 ** -24 * mag + (2.0 ** -8 if bf16 else 0.0)
  return (2 * rel + 1e-8 * 34881)[:, None]


def _check_loss_grad(W, nf, lab, nl, V, n, local=False, idx=None, bf16=False,
                     design=nat.DESIGN_AUTO):
  """lt_loss_grad on the batch, the utterances `idx` (all: None) against the
  oracle: loss, log_z, num and every dW element relative to its marginals."""
  loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, local, design=design)
  torch.cuda.synchronize()
  sel = slice(None) if idx is None else idx
  Wc, nfc, labc, nlc = _np(W[sel], nf[sel], lab[sel], nl[sel])
  orc = _orc()
  rl, rlz, rnum, rdW = orc.loss_grad(Wc, nfc, labc, nlc, V, n, local_norm=local)
  den = None if local else orc.den_grad(Wc, nfc, V, n)[1]
  assert_loss_close(loss[sel].cpu().numpy(), rl)
  if not local:
    assert_loss_close(lz[sel].cpu().numpy(), rlz)
  assert_loss_close(num[sel].cpu().numpy(), rnum)
  assert_grad_marginal_close(dW[sel].float().cpu().numpy(), rdW, den, rlz, rnum, bf16=bf16)
  return loss, lz, num, dW


@pytest.fixture(scope='module')
def cfg2(cuda):
  return _bench_inputs(64, 1000, 100, 32, 1, cuda, seed=1234)


def test_cfg2_bench_launch_every_utterance(cfg2):
  """The bench step (lt_loss_grad, B=64 T=1000 U=100 V=32 fp32): every
  utterance's loss and every dW element against the oracle."""
  W, nf, lab, nl = cfg2
  assert nat.chunk_path(W.shape[0], W.shape[1], lab.shape[1], 32, 1)
  _check_loss_grad(W, nf, lab, nl, 32, 1)


def test_cfg2_properties(cfg2):
  W, nf, lab, nl = cfg2
  V, n = 32, 1
  loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, False)
  loss2, _, _, dW2 = nat.loss_grad(W, nf, lab, nl, V, n, False)
  # deterministic: the same bits on a second call
  assert torch.equal(loss, loss2) and torch.equal(dW, dW2)
  assert torch.isfinite(loss).all() and (loss > -1e-3).all()  # log_z >= numerator
  # each live frame: den marginals and num marginals both sum to 1
  s = _frame_sums(dW)
  tol = _frame_sum_tol(lz, num)
  assert (s.abs() <= tol).all(), float((s.abs() / tol).max())
  # forward / backward split with an incoming gradient: linear in it
  g = torch.linspace(-1.0, 2.0, W.shape[0], device=W.device)
  l3, _, _, state = nat.chunk_forward(W, nf, lab, nl, V, n, False)
  assert torch.equal(l3, loss)
  dWg = nat.chunk_backward(W, nf, lab, nl, V, n, False, state, grad=g)
  assert torch.allclose(dWg, dW * g[:, None, None, None], atol=1e-7, rtol=1e-6)
  # the state serves a second backward (retain_graph semantics)
  assert torch.equal(nat.chunk_backward(W, nf, lab, nl, V, n, False, state, grad=g), dWg)


def test_cfg2_varlen_local_norm(cuda):
  """Variable lengths and the locally normalised loss (numerator only) at
  the bench shape: every utterance against the oracle."""
  V, n = 32, 1
  W, nf, lab, nl = _bench_inputs(16, 1000, 100, V, n, cuda, seed=7, varlen=True)
  W = torch.log_softmax(W, dim=-1)
  for local in (False, True):
    _, _, _, dW = _check_loss_grad(W, nf, lab, nl, V, n, local=local)
    pad = torch.arange(W.shape[1], device=cuda)[None, :] >= nf[:, None].long()
    assert (dW[pad] == 0).all()


def _realistic(kind, B, T, V, device, seed):
  """Arc weights a trained model produces: log_softmax(sigma * randn) rows
  (weight_fns.py:120-136; sigma 10 spans ~60 nats per frame, up to 90), or
  randn with masked arcs (lattices.py:450-453): one -inf arc per utterance,
  or one label masked in every state of one frame."""
  g = torch.Generator(device=device)
  g.manual_seed(seed)
  C = V + 1
  W = torch.randn([B, T, C, V + 1], generator=g, device=device)
  if kind.startswith('logsoftmax'):
    W = torch.log_softmax(float(kind[len('logsoftmax'):]) * W, dim=-1)
  elif kind == 'neginf_arc':
    t = torch.randint(0, T, [B], generator=g, device=device)
    p = torch.randint(0, C, [B], generator=g, device=device)
    y = torch.randint(0, V + 1, [B], generator=g, device=device)
    W[torch.arange(B, device=device), t, p, y] = -float('inf')
  elif kind == 'neginf_label':
    t = torch.randint(0, T, [B], generator=g, device=device)
    W[torch.arange(B, device=device), t, :, 5] = -float('inf')
  return W.contiguous()


@pytest.mark.parametrize('kind', ['logsoftmax5', 'logsoftmax10', 'logsoftmax20', 'neginf_arc',
                                  'neginf_label'])
def test_cfg2_realistic_weights(cuda, kind):
  """The bench shape with a trained model's kind of weights: every
  utterance of a B=16 batch (B=64 for log_softmax sigma=10) against the
  oracle, element by element."""
  V, n, T, U = 32, 1, 1000, 100
  B = 64 if kind == 'logsoftmax10' else 16
  W = _realistic(kind, B, T, V, cuda, seed=11)
  _, nf, lab, nl = _bench_inputs(B, T, U, V, n, cuda, seed=12)
  _check_loss_grad(W, nf, lab, nl, V, n)
  _check_loss_grad(W, nf, lab, nl, V, n, local=True)


@pytest.mark.parametrize('design', ['auto', 'chunk', 'fused'])
def test_north_star_b256(cuda, design):
  """B=256 (the north-star shape): 64 utterances spread over the batch
  (every residue mod 8, both ends) against the oracle, every dW element, and
  the per-frame marginal sums of all 256 -- the design lt_loss_grad picks
  there (what bench.py times), the chunked scan and the one-launch fused pipe
  (lt_loss_grad_ex; its 2B recursion workgroups co-resident on 256 CUs)."""
  V, n = 32, 1
  d = {'auto': nat.DESIGN_AUTO, 'chunk': nat.DESIGN_CHUNK, 'fused': nat.DESIGN_FUSED_PIPE}[design]
  W, nf, lab, nl = _bench_inputs(256, 1000, 100, V, n, cuda, seed=99)
  # 64 of the 256 utterances (a quarter): every fourth, shifted by one per
  # block of 64 so each residue mod 8 (the XCD groups) and both ends are in
  idx = sorted({4 * i + (i // 16) for i in range(64)} | {255})[:64]
  loss, lz, num, dW = _check_loss_grad(W, nf, lab, nl, V, n, idx=idx, design=d)
  s = _frame_sums(dW)
  assert (s.abs() <= _frame_sum_tol(lz, num)).all()


def test_chunk_fallback_mixed_batch(cuda):
  """Utterances that leave the chunked path's fast range (a frame spanning
  more than 60, a -inf weight, a +-30 peaked utterance, a NaN-free frame
  spanning ~200) next to ordinary ones, in one call: every utterance and
  every dW element against the oracle."""
  V, n, T, U = 32, 1, 300, 40
  rng = np.random.default_rng(21)
  W = rng.standard_normal((6, T, V + 1, V + 1)).astype(np.float32)
  W[1] *= 30.0                        # peaked: range ~ 200
  W[3, 17, 5, 7] = -np.inf            # a masked arc
  W[4, 250] *= 40.0                   # one wide frame late in the utterance
  nf = np.array([300, 300, 123, 300, 280, 1], np.int32)
  lab = rng.integers(1, V + 1, (6, U)).astype(np.int32)
  nl = np.array([40, 35, 20, 40, 40, 0], np.int32)
  Wd = torch.tensor(W, device=cuda)
  nfd, labd, nld = (torch.tensor(x, device=cuda) for x in (nf, lab, nl))
  assert nat.chunk_path(6, T, U, V, n)
  for local in (False, True):
    _check_loss_grad(Wd, nfd, labd, nld, V, n, local=local)


def test_cfg4_viterbi_t2000_every_utterance(cuda):
  """cfg4: MaxTropical shortest path at B=64, T=2000 (U=200 is unused by the
  decode): labels and path weights bit-exact on every utterance, both label
  conventions (reference y-1, D5; true y)."""
  V, n = 32, 1
  W, nf, _, _ = _bench_inputs(64, 2000, 200, V, n, cuda, seed=4)
  Wc, nfc = _np(W, nf)
  for conv in (nat.LABELS_REFERENCE, nat.LABELS_TRUE):
    labels, weights, _ = nat.viterbi(W, nf, V, n, conv)
    rlab, rw, _ = _orc().viterbi(Wc, nfc, V, n, convention=conv)
    np.testing.assert_array_equal(labels.cpu().numpy(), rlab)
    np.testing.assert_array_equal(weights.cpu().numpy(), rw)


@pytest.mark.parametrize('T', [2400, 4500])
def test_viterbi_long_utterances_backtrace_routes(cuda, T):
  """Viterbi past the length whose backpointers fit the forward's LDS (T <=
  2,300 at V = 32: the backtrace in the same launch): T = 2400 runs the
  separate segmented backtrace launch, T = 4500 (beyond its 144 KB) the
  generic one. Labels, path weights and the one-hot arcs (the gradient of
  the distance) bit-exact against the oracle, varied lengths, both
  conventions."""
  V, n, B = 32, 1, 4
  W, nf, _, _ = _bench_inputs(B, T, 10, V, n, cuda, seed=T)
  nf = torch.tensor([T, T - 1, T // 2, 1], dtype=torch.int32, device=cuda)
  Wc, nfc = _np(W, nf)
  for conv in (nat.LABELS_REFERENCE, nat.LABELS_TRUE):
    labels, weights, arcs = nat.viterbi(W, nf, V, n, conv, want_arcs=True)
    rlab, rw, rarcs = _orc().viterbi(Wc, nfc, V, n, convention=conv, want_arcs=True)
    np.testing.assert_array_equal(labels.cpu().numpy(), rlab)
    np.testing.assert_array_equal(weights.cpu().numpy(), rw)
    np.testing.assert_array_equal(arcs.cpu().numpy(), rarcs)


def test_cfg5_trigram_bf16(cuda):
  """cfg5: trigram (|ctx| = 1057) bf16 arc weights at B=32, T=1000, U=100
  (lt_loss_grad's trigram overlap: the one-workgroup recursions of lt_tri.hip
  with marginal waves on the idle CUs, tri_mix_kernel, then marg_kernel on the
  frames left; the quad design, lt_tri4.hip, is diagnostic-only and covered by
  test_gpu_diag.py): losses and every dW element of sixteen utterances spread
  over the batch against the oracle on the bf16-rounded weights; per-frame
  marginal sums of the whole batch."""
  V, n = 32, 2
  W, nf, lab, nl = _bench_inputs(32, 1000, 100, V, n, cuda, seed=5, dtype=torch.bfloat16)
  loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, False)
  s = _frame_sums(dW.float())
  # bf16 dW: each element carries 2^-9 relative rounding (in the sum: 2^-8 * 2)
  assert (s.abs() <= _frame_sum_tol(lz, num, bf16=True)).all()
  orc = _orc()
  idx = [0, 1, 3, 5, 7, 9, 12, 14, 17, 19, 22, 24, 26, 27, 30, 31]  # 16 of 32
  Wc, nfc, labc, nlc = _np(W[idx], nf[idx], lab[idx], nl[idx])
  rl, rlz, rnum, rdW = orc.loss_grad(Wc, nfc, labc, nlc, V, n)
  _, den = orc.den_grad(Wc, nfc, V, n)
  assert_loss_close(loss[idx].cpu().numpy(), rl)
  assert_grad_marginal_close(dW[idx].float().cpu().numpy(), rdW, den, rlz, rnum, bf16=True)


def test_trigram_overlap_b8_t1000_every_utterance(cuda):
  """The trigram overlap with one utterance per XCD, so that each marginal
  wave takes many frames of its utterance (B = 8, T = 1000: cus - 2B marginal
  workgroups for 8000 frames): every dW element of every utterance against the
  oracle. A build that computed only each wave's first frame right (DESIGN.md
  3d, the open item) fails here."""
  V, n = 32, 2
  W, nf, lab, nl = _bench_inputs(8, 1000, 100, V, n, cuda, seed=11, dtype=torch.bfloat16)
  assert nat.loss_grad_design(8, 1000, 100, V, n) == nat.DESIGN_CHECKPOINTS
  loss, lz, num, dW = nat.loss_grad(W, nf, lab, nl, V, n, False)
  orc = _orc()
  Wc, nfc, labc, nlc = _np(W, nf, lab, nl)
  rl, rlz, rnum, rdW = orc.loss_grad(Wc, nfc, labc, nlc, V, n)
  _, den = orc.den_grad(Wc, nfc, V, n)
  assert_loss_close(loss.cpu().numpy(), rl)
  assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, den, rlz, rnum, bf16=True)


@pytest.mark.parametrize('B', [8, 64, 120, 160, 176, 177, 192, 256, 512])
def test_design_query_matches_python_mirrors(cuda, B):
  """lt_loss_grad_design (the C dispatch) and the Python mirrors the autograd
  path and bench.py use agree at the bench shape for every batch size."""
  T, U, V, n = 1000, 100, 32, 1
  d = nat.loss_grad_design(B, T, U, V, n)
  assert (d == nat.DESIGN_CHUNK) == nat.chunk_path(B, T, U, V, n)
  assert (d == nat.DESIGN_FUSED_PIPE) == nat.fused_path(B, T, U, V, n)
  if B == 64:
    assert d == nat.DESIGN_CHUNK
  if B == 256:  # the checkpointing pair (the fused pipe measured level with it)
    assert d == nat.DESIGN_CHECKPOINTS

