"""GPU parity: the HIP kernels (through the C ABI and through the
RecognitionLattice plugin API) against the reference's golden fixtures and
the pinned C oracle.

Tolerances (BASELINE.json north_star):
  * Log loss / log_z / numerator: |got - ref| <= 1e-4 * max(1, |ref|);
    alpha histories rtol 1e-4, atol 1e-4.
  * dW, every element relative to its own arc marginals
    (golden_cases.marginal_scale, alignments.py:300-318):
    |got - ref| <= 1e-8 + (1e-4 + 4 * 2^-24 * max(1, |log_z|, |num|)) *
    (den + num), den / num the arc's denominator / numerator marginals (the
    oracle's den_grad and den - dW); bf16 dW adds 2^-8 (den + num). The
    denominator-only gradient (lt_den_backward, d log_z / dW) is held to the
    same bound with num = 0. The round-2 absolute bound
    (golden_cases.assert_grad_close) stays as a secondary assert.
  * MaxTropical distances, alpha histories and Viterbi labels/path weights:
    bit-exact (same fp32 adds, same tie rules).
"""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat
from golden_cases import (LATTICE_CASES, assert_grad_marginal_close, assert_loss_close,
                          assert_values_close, load)

pytestmark = pytest.mark.gpu

SID = {'Log': nat.SEMIRING_LOG, 'MaxTropical': nat.SEMIRING_MAX, 'Real': nat.SEMIRING_REAL}


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _dev(c, cuda, key='W'):
  dt = torch.bfloat16 if c['bf16'] else torch.float32
  W = torch.tensor(c[key]).to(dt).to(cuda)
  nf = torch.tensor(c['num_frames']).to(cuda)
  lab = torch.tensor(c['labels']).to(cuda)
  nl = torch.tensor(c['num_labels']).to(cuda)
  return W, nf, lab, nl


# ---------------------------------------------------------------------------
# golden fixtures (reference outputs) through the C ABI
# ---------------------------------------------------------------------------
@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('semiring', ['Log', 'MaxTropical', 'Real'])
def test_golden_den_forward(cuda, case, semiring):
  c = load(case)
  W, nf, _, _ = _dev(c, cuda)
  d, a = nat.den_forward(W, nf, c['V'], c['n'], SID[semiring])
  d, a = d.cpu().numpy(), a.cpu().numpy()
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
def test_golden_num_forward(cuda, case, semiring):
  c = load(case)
  W, nf, lab, nl = _dev(c, cuda)
  num, _ = nat.num_forward(W, nf, lab, nl, c['V'], c['n'], SID[semiring])
  num = num.cpu().numpy()
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
@pytest.mark.parametrize('ckpt', [False, True])
def test_golden_loss_and_grad(cuda, case, local, ckpt):
  c = load(case)
  W, nf, lab, nl = _dev(c, cuda, 'W_local' if local else 'W')
  out = nat.loss_forward(W, nf, lab, nl, c['V'], c['n'], local, checkpoints=ckpt)
  loss, lz, num, al, an = out[:5]
  dW = nat.loss_backward(W, nf, lab, nl, lz, num, al, an, None, c['V'], c['n'], local,
                         ck=out[5] if ckpt else None)
  torch.cuda.synchronize()
  assert_loss_close(loss.cpu().numpy(), c['loss_local' if local else 'loss'])
  if not local:
    assert_loss_close(lz.cpu().numpy(), c['den_Log'])
  ref = c['loss_local_grad' if local else 'loss_grad']
  assert_grad_marginal_close(dW.float().cpu().numpy(), ref, None if local else c['den_grad'],
                             c['den_Log'], c['num_Log'], c['bf16'])


@pytest.mark.parametrize('case', LATTICE_CASES)
def test_golden_den_grad(cuda, case):
  c = load(case)
  W, nf, _, _ = _dev(c, cuda)
  lz, al = nat.den_forward(W, nf, c['V'], c['n'], nat.SEMIRING_LOG)
  dW = nat.den_backward(W, nf, lz, al, None, c['V'], c['n'])
  assert_grad_marginal_close(dW.float().cpu().numpy(), c['den_grad'], c['den_grad'], c['den_Log'],
                             None, c['bf16'])


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('convention', ['reference', 'true'])
def test_golden_viterbi_bit_exact(cuda, case, convention):
  c = load(case)
  W, nf, _, _ = _dev(c, cuda)
  conv = nat.LABELS_REFERENCE if convention == 'reference' else nat.LABELS_TRUE
  labels, weights, _ = nat.viterbi(W, nf, c['V'], c['n'], conv)
  np.testing.assert_array_equal(labels.cpu().numpy(), c[f'vit_labels_{convention}'])
  np.testing.assert_array_equal(weights.cpu().numpy(), c['vit_weights'])


# ---------------------------------------------------------------------------
# golden fixtures through the plugin API (RecognitionLattice + TableWeightFn)
# ---------------------------------------------------------------------------
def _table_lattice(c, table):
  return lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=c['V'], context_size=c['n']),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))


def _frames(B, T):
  return torch.arange(T, dtype=torch.float32)[None, :, None].expand(B, T, 1).contiguous()


@pytest.mark.parametrize('case', [k for k in LATTICE_CASES if not k.startswith('bf16')])
def test_golden_recognition_lattice_api(cuda, case):
  c = load(case)
  B, T = c['W'].shape[:2]
  table = torch.tensor(c['W'], device=cuda, requires_grad=True)
  lat = _table_lattice(c, table)
  frames = _frames(B, T).to(cuda)
  nf = torch.tensor(c['num_frames'], dtype=torch.float32)  # float lengths, as the reference tests
  labels = torch.tensor(c['labels'], dtype=torch.float32)
  nl = torch.tensor(c['num_labels'], dtype=torch.float32)
  loss = lat(frames, nf, labels, nl)
  assert_loss_close(loss.detach().cpu().numpy(), c['loss'])
  fin = torch.isfinite(loss)
  loss.masked_fill(~fin, 0).sum().backward()
  assert_grad_marginal_close(table.grad.cpu().numpy(), c['loss_grad'], c['den_grad'], c['den_Log'],
                             c['num_Log'])
  for sname in ('Log', 'MaxTropical'):
    d, a = lat._forward(None, frames, nf, getattr(lt.semirings, sname))
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(d.detach().cpu().numpy(), c['den_MaxTropical'])
      np.testing.assert_array_equal(a.detach().cpu().numpy(), c['alpha_MaxTropical'])
    else:
      assert_loss_close(d.detach().cpu().numpy(), c['den_Log'])
    s = lat._string_forward(None, frames, nf, labels, nl, getattr(lt.semirings, sname))
    if sname == 'MaxTropical':
      np.testing.assert_array_equal(s.detach().cpu().numpy(), c['num_MaxTropical'])
    else:
      assert_loss_close(s.detach().cpu().numpy(), c['num_Log'])
  for conv in ('reference', 'true'):
    al, nal, pw = lat.shortest_path(frames, nf, label_convention=conv)
    np.testing.assert_array_equal(al.cpu().numpy(), c[f'vit_labels_{conv}'])
    np.testing.assert_array_equal(pw.cpu().numpy(), c['vit_weights'])
    np.testing.assert_array_equal(nal.cpu().numpy(), c['num_frames'])


def test_locally_normalised_weight_fn_api(cuda):
  """LocallyNormalizedWeightFn(hat_normalize) switches the loss to -numerator
  (lattices.py:178-179); its gradient flows back through the normaliser."""
  c = load('locally_normalised')
  B, T = c['W'].shape[:2]
  table = torch.tensor(c['W'], device=cuda, requires_grad=True)
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=c['V'], context_size=c['n']),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.LocallyNormalizedWeightFn(
          lt.weight_fns.TableWeightFn(table)))
  frames = _frames(B, T).to(cuda)
  loss = lat(frames, torch.tensor(c['num_frames']), torch.tensor(c['labels']),
             torch.tensor(c['num_labels']))
  assert_loss_close(loss.detach().cpu().numpy(), c['loss_local'])
  loss.sum().backward()
  # chain rule through hat_normalize, in float64 on the CPU
  Wl = torch.tensor(c['W'], dtype=torch.float64, requires_grad=True)
  hb, hl = lt.weight_fns.hat_normalize(Wl[..., 0], Wl[..., 1:])
  Wn = torch.cat([hb[..., None], hl], dim=-1)
  (Wn * torch.tensor(c['loss_local_grad'], dtype=torch.float64)).sum().backward()
  np.testing.assert_allclose(table.grad.cpu().numpy(), Wl.grad.numpy(), atol=1e-5, rtol=1e-4)


# ---------------------------------------------------------------------------
# random problems against the oracle (sizes the oracle finishes in seconds)
# ---------------------------------------------------------------------------
RANDOM = [
    # B, T, U, V, n, dtype
    (8, 200, 30, 32, 1, 'f32'),
    (8, 200, 30, 32, 1, 'bf16'),
    (4, 64, 12, 8, 2, 'f32'),
    (3, 40, 10, 16, 2, 'bf16'),
    (2, 30, 8, 32, 2, 'bf16'),   # cfg5 shape class: trigram V=32 (C=1057), bf16
    (2, 30, 8, 32, 2, 'f32'),    # trigram fp32: the wide-frame direct path
    (6, 120, 20, 32, 0, 'f32'),
    (4, 100, 20, 64, 1, 'f32'),
    (5, 90, 15, 3, 3, 'f32'),
    (1, 1, 1, 5, 1, 'f32'),
]


def _random_problem(B, T, U, V, n, seed):
  orc = _orc()
  rng = np.random.default_rng(seed)
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = rng.integers(0, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(0, V + 1, (B, U)).astype(np.int32)  # includes epsilon (0) labels
  nl = rng.integers(0, U + 1, B).astype(np.int32)
  nl[0] = min(U, T)
  return W, nf, lab, nl


@pytest.mark.parametrize('B,T,U,V,n,dt', RANDOM)
def test_random_checkpointing_vs_oracle(cuda, B, T, U, V, n, dt):
  """Checkpointing loss path: concurrent beta pass + streaming marginal pass."""
  orc = _orc()
  W, nf, lab, nl = _random_problem(B, T, U, V, n, seed=B * 1000 + T + V + n + 7)
  bf16 = dt == 'bf16'
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  for local in (False, True):
    out = nat.loss_forward(Wd, nfd, labd, nld, V, n, local, checkpoints=True)
    dW = nat.loss_backward(Wd, nfd, labd, nld, *out[1:5], None, V, n, local, ck=out[5])
    rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n, local_norm=local)
    den = None if local else orc.den_grad(W, nf, V, n)[1]
    assert_loss_close(out[0].cpu().numpy(), rl)
    assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, den, rlz, rnum, bf16)


def test_trigram_v32_short_and_empty_utterances(cuda):
  """The trigram den roles at V = 32 (lt_tri.hip; the backward's padded beta
  rows, den_bwd_tri32) on utterances of 0, 1, 2, T-1 and T frames, bf16,
  against the oracle: loss, and dW under the per-element marginal bound."""
  orc = _orc()
  B, T, U, V, n = 5, 24, 6, 32, 2
  W, _, lab, _ = _random_problem(B, T, U, V, n, seed=4242)
  nf = np.array([T, 0, 1, 2, T - 1], dtype=np.int32)
  nl = np.array([U, 0, 1, 2, U - 1], dtype=np.int32)
  W = torch.tensor(W).bfloat16().float().numpy()
  Wd = torch.tensor(W).to(torch.bfloat16).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  out = nat.loss_forward(Wd, nfd, labd, nld, V, n, False, checkpoints=True)
  dW = nat.loss_backward(Wd, nfd, labd, nld, *out[1:5], None, V, n, False, ck=out[5])
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  assert_loss_close(out[0].cpu().numpy(), rl)
  assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, orc.den_grad(W, nf, V, n)[1], rlz,
                             rnum, True)


@pytest.mark.parametrize('dt', ['bf16', 'f32'])
def test_trigram_overlap_loss_grad_vs_oracle(cuda, dt):
  """lt_loss_grad's trigram V = 32 route (lt_tri.hip, tri_mix_kernel): the
  recursions with marginal workgroups on the CUs they leave idle, each taking
  frames as both recursions pass them, then marg_kernel on the frames they
  did not take. B = 8 (the route needs a multiple of 8), T = 160 (progress
  published every 16 frames), lengths 0, 1, 2, 3, T - 1 and T, epsilon labels,
  an unreachable string: loss and every dW element against the oracle, and a
  second call bit-identical (which kernel takes a frame does not change it)."""
  orc = _orc()
  B, T, U, V, n = 8, 160, 12, 32, 2
  W, _, lab, _ = _random_problem(B, T, U, V, n, seed=777)
  nf = np.array([T, 0, 1, 2, T - 1, 150, 3, T], dtype=np.int32)
  nl = np.array([U, 0, 1, 2, U - 1, U, 5, U], dtype=np.int32)  # utterance 6 unreachable
  bf16 = dt == 'bf16'
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  assert nat.loss_grad_design(B, T, U, V, n) == nat.DESIGN_CHECKPOINTS
  loss, lz, num, dW = nat.loss_grad(Wd, nfd, labd, nld, V, n, False)
  loss2, _, _, dW2 = nat.loss_grad(Wd, nfd, labd, nld, V, n, False)
  torch.cuda.synchronize()
  assert torch.equal(loss, loss2) and torch.equal(dW, dW2)
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  assert_loss_close(loss.cpu().numpy(), rl)
  assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, orc.den_grad(W, nf, V, n)[1], rlz,
                             rnum, bf16)


@pytest.mark.parametrize('B,T,U,V,n,dt', RANDOM)
def test_random_vs_oracle(cuda, B, T, U, V, n, dt):
  orc = _orc()
  W, nf, lab, nl = _random_problem(B, T, U, V, n, seed=B * 1000 + T + V + n)
  bf16 = dt == 'bf16'
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  loss, lz, num, al, an = nat.loss_forward(Wd, nfd, labd, nld, V, n, False)
  dW = nat.loss_backward(Wd, nfd, labd, nld, lz, num, al, an, None, V, n, False)
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  assert_loss_close(loss.cpu().numpy(), rl)
  assert_loss_close(lz.cpu().numpy(), rlz)
  den = orc.den_grad(W, nf, V, n)[1]
  assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, den, rlz, rnum, bf16)
  # the den-only backward (lt_den_backward: _backward, _forward_backward)
  dd = nat.den_backward(Wd, nfd, lz, al, None, V, n)
  assert_grad_marginal_close(dd.float().cpu().numpy(), den, den, rlz, None, bf16)
  for conv in (nat.LABELS_REFERENCE, nat.LABELS_TRUE):
    labels, weights, arcs = nat.viterbi(Wd, nfd, V, n, conv, want_arcs=True)
    rlab, rw, rarcs = orc.viterbi(W, nf, V, n, convention=conv, want_arcs=True)
    np.testing.assert_array_equal(labels.cpu().numpy(), rlab)
    np.testing.assert_array_equal(weights.cpu().numpy(), rw)
    np.testing.assert_array_equal(arcs.float().cpu().numpy(), rarcs)
  d, a = nat.den_forward(Wd, nfd, V, n, nat.SEMIRING_MAX)
  rd, ra = orc.den_forward(W, nf, V, n, orc.MAX)
  np.testing.assert_array_equal(d.cpu().numpy(), rd)
  np.testing.assert_array_equal(a.cpu().numpy(), ra)


def _poisoned_ws(W, V, n, U, local, design=nat.DESIGN_AUTO):
  # NaN bytes: a stale hand-off read of a checkpoint row would show in dW
  nb = nat.loss_grad_workspace_bytes(W, V, n, U, local, design)
  return torch.full([max(nb, 1)], 0xFF, dtype=torch.uint8, device=W.device)


# lt_loss_grad's designs (lt_loss_grad_ex): the chunked two-level scan
# (bigram default), the fused pipe launch, the checkpointing pair and the
# recursion pair
LOSS_GRAD_PATHS = {'chunk': nat.DESIGN_CHUNK, 'fused': nat.DESIGN_FUSED_PIPE,
                   'two-call': nat.DESIGN_CHECKPOINTS, 'recursion': nat.DESIGN_RECURSION}


def _design_or_skip(path, B, T, U, V, n, device, bf16=False):
  d = LOSS_GRAD_PATHS[path]
  if d == nat.DESIGN_CHUNK and not (n == 1 and 1 <= V <= 32 and U + 1 <= 128 and T >= 1):
    pytest.skip('shape outside the chunked design (bigram, V <= 32, U < 128)')
  if d == nat.DESIGN_FUSED_PIPE and not (nat.pipe_path(B, T, U, V, n, bf16) and U + 1 <= 128):
    pytest.skip('shape outside the fused pipe design (bigram, U < 128)')
  return d


@pytest.mark.parametrize('case', LATTICE_CASES)
@pytest.mark.parametrize('local', [False, True])
@pytest.mark.parametrize('path', list(LOSS_GRAD_PATHS))
def test_golden_loss_grad(cuda, case, local, path):
  """lt_loss_grad against the reference's fixtures, on each design."""
  c = load(case)
  W, nf, lab, nl = _dev(c, cuda, 'W_local' if local else 'W')
  U = lab.shape[-1]
  d = _design_or_skip(path, W.shape[0], W.shape[1], U, c['V'], c['n'], cuda,
                      W.dtype == torch.bfloat16)
  ws = _poisoned_ws(W, c['V'], c['n'], U, local, d)
  loss, lz, _, dW = nat.loss_grad(W, nf, lab, nl, c['V'], c['n'], local, workspace=ws, design=d)
  torch.cuda.synchronize()
  assert_loss_close(loss.cpu().numpy(), c['loss_local' if local else 'loss'])
  if not local:
    assert_loss_close(lz.cpu().numpy(), c['den_Log'])
  ref = c['loss_local_grad' if local else 'loss_grad']
  assert_grad_marginal_close(dW.float().cpu().numpy(), ref, None if local else c['den_grad'],
                             c['den_Log'], c['num_Log'], c['bf16'])
  if d == nat.DESIGN_FUSED_PIPE:
    assert nat.grad_workspace_errors(ws, W, c['V'], c['n'], U, local) == 0


FUSED_RANDOM = [
    # B, T, U, V, dtype: bigram shapes of the fused launch (V <= 32, U < 128)
    (8, 200, 30, 32, 'f32'),
    (8, 200, 30, 32, 'bf16'),
    (6, 150, 70, 32, 'f32'),    # 2 numerator values per lane
    (4, 90, 120, 16, 'f32'),    # 2 numerator values per lane, V = 16
    (12, 80, 10, 8, 'f32'),
    (9, 50, 6, 3, 'f32'),
    (5, 33, 4, 1, 'bf16'),
    (1, 1, 1, 5, 'f32'),
]


@pytest.mark.parametrize('B,T,U,V,dt', FUSED_RANDOM)
@pytest.mark.parametrize('path', ['chunk', 'fused'])
def test_random_loss_grad_vs_oracle(cuda, B, T, U, V, dt, path):
  orc = _orc()
  n = 1
  W, nf, lab, nl = _random_problem(B, T, U, V, n, seed=B * 100 + T + U + V)
  bf16 = dt == 'bf16'
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  d = _design_or_skip(path, B, T, U, V, n, cuda, bf16)
  for local in (False, True):
    ws = _poisoned_ws(Wd, V, n, U, local, d)
    loss, lz, _, dW = nat.loss_grad(Wd, nfd, labd, nld, V, n, local, workspace=ws, design=d)
    rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n, local_norm=local)
    den = None if local else orc.den_grad(W, nf, V, n)[1]
    assert_loss_close(loss.cpu().numpy(), rl)
    assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, den, rlz, rnum, bf16)
    if path == 'fused':
      assert nat.grad_workspace_errors(ws, Wd, V, n, U, local) == 0
    # deterministic: a second call gives the same bits
    loss2, _, _, dW2 = nat.loss_grad(Wd, nfd, labd, nld, V, n, local, design=d)
    assert torch.equal(loss, loss2) and torch.equal(dW, dW2)


def test_scale_grad(cuda):
  """lt_scale_grad: dW[b] *= g[b]; utterances with g == 1 are untouched."""
  V, n = 5, 1
  g = torch.Generator(device=cuda)
  g.manual_seed(3)
  for dt in (torch.float32, torch.bfloat16):
    dW = torch.randn([5, 7, 6, 6], generator=g, device=cuda).to(dt)
    ref = dW.clone()
    gr = torch.tensor([1.0, 0.5, -2.0, 1.0, 0.0], device=cuda)
    nat.scale_grad(dW, gr, V, n)
    exp = (ref.float() * gr[:, None, None, None]).to(dt)
    assert torch.equal(dW, exp)
    assert torch.equal(dW[0], ref[0]) and torch.equal(dW[3], ref[3])


def test_loss_grad_autograd_scaling(cuda):
  """RecognitionLattice.forward -> (w * loss).sum().backward(): the fused
  gradient times the incoming per-utterance weights, against the oracle."""
  orc = _orc()
  B, T, U, V, n = 6, 40, 8, 7, 1
  W, nf, lab, nl = _random_problem(B, T, U, V, n, seed=5)
  table = torch.tensor(W, device=cuda, requires_grad=True)
  lat = lt.RecognitionLattice(
      context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
      alignment=lt.alignments.FrameDependent(),
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))
  loss = lat(_frames(B, T).to(cuda), torch.tensor(nf), torch.tensor(lab), torch.tensor(nl))
  w = torch.tensor([0.5, 1.0, 2.0, -1.0, 3.0, 1.0], device=cuda)
  fin = torch.isfinite(loss.detach())
  (w * loss.masked_fill(~fin, 0)).sum().backward()
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  assert_loss_close(loss.detach().cpu().numpy(), rl)
  den = orc.den_grad(W, nf, V, n)[1]
  assert_grad_marginal_close(table.grad.cpu().numpy(), rdW, den, rlz, rnum,
                             weights=(w * fin).cpu().numpy())
  # dW is formed in the backward: a second backward (retain_graph) repeats it
  table.grad = None
  loss2 = lat(_frames(B, T).to(cuda), torch.tensor(nf), torch.tensor(lab), torch.tensor(nl))
  s2 = loss2.masked_fill(~fin, 0).sum()
  s2.backward(retain_graph=True)
  g1 = table.grad.clone()
  s2.backward()
  assert torch.equal(table.grad, 2 * g1)


def test_edge_cases(cuda):
  """Empty utterances, T=0 and U=0, unreachable label strings (+inf loss,
  zero gradient), lengths beyond max (clamped), labels all epsilon."""
  orc = _orc()
  V, n, T, U = 4, 1, 6, 5
  C = orc.num_states(V, n)
  rng = np.random.default_rng(11)
  W = rng.standard_normal((6, T, C, V + 1)).astype(np.float32)
  nf = np.array([0, 6, 2, 6, 9, 3], np.int32)           # 9 > T is clamped
  nl = np.array([0, 5, 4, 0, 2, 3], np.int32)           # utt 2: 4 labels in 2 frames
  lab = rng.integers(1, V + 1, (6, U)).astype(np.int32)
  lab[5] = 0                                              # all-epsilon string
  Wd = torch.tensor(W, device=cuda)
  nfd, labd, nld = (torch.tensor(x, device=cuda) for x in (nf, lab, nl))
  loss, lz, num, al, an = nat.loss_forward(Wd, nfd, labd, nld, V, n, False)
  dW = nat.loss_backward(Wd, nfd, labd, nld, lz, num, al, an, None, V, n, False)
  rl, rlz, rnum, rdW = orc.loss_grad(W, nf, lab, nl, V, n)
  den = orc.den_grad(W, nf, V, n)[1]
  l = loss.cpu().numpy()
  assert l[0] == 0.0                                      # T=0, U=0 -> 0 (lattices_test.py:286)
  assert np.isposinf(l[2]) and np.isposinf(rl[2])        # unreachable -> +inf
  assert (dW[2] == 0).all()
  assert_loss_close(l, rl)
  assert_grad_marginal_close(dW.cpu().numpy(), rdW, den, rlz, rnum)
  # T = 0 for the whole batch
  W0 = torch.zeros([3, 0, C, V + 1], device=cuda)
  z = torch.zeros([3], dtype=torch.int32, device=cuda)
  d0, _ = nat.den_forward(W0, z, V, n, nat.SEMIRING_LOG)
  np.testing.assert_array_equal(d0.cpu().numpy(), [0., 0., 0.])
  lab0, w0, _ = nat.viterbi(W0, z, V, n, nat.LABELS_TRUE)
  assert lab0.shape == (3, 0) and (w0.cpu().numpy() == 0).all()


# ---------------------------------------------------------------------------
# BASELINE sizes: size-independent properties + an oracle spot check
# ---------------------------------------------------------------------------
@pytest.fixture(scope='module')
def full_size(cuda):
  B, T, U, V, n = 64, 1000, 100, 32, 1
  g = torch.Generator(device=cuda)
  g.manual_seed(0)
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], generator=g, device=cuda)
  nf = torch.randint(T // 2, T + 1, [B], generator=g, device=cuda, dtype=torch.int32)
  nf[0] = T
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=cuda, dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device=cuda)
  return W, nf, lab, nl, V, n


def test_full_size_marginals_sum_to_one(full_size):
  W, nf, _, _, V, n = full_size
  lz, al = nat.den_forward(W, nf, V, n, nat.SEMIRING_LOG)
  dW = nat.den_backward(W, nf, lz, al, None, V, n)
  s = dW.double().reshape(W.shape[0], W.shape[1], -1).sum(-1)
  live = (torch.arange(W.shape[1], device=W.device)[None, :] < nf[:, None].long()).double()
  # fp32 log-space rounding scales with |log_z| (~4e3 here); see assert_grad_close
  tol = 1e-5 + 1e-6 * lz.abs().double().clamp(min=1.0)[:, None]
  assert ((s - live).abs() <= tol).all(), float(((s - live).abs() / tol).max())


def test_full_size_loss_properties_and_determinism(full_size):
  W, nf, lab, nl, V, n = full_size
  out1 = nat.loss_forward(W, nf, lab, nl, V, n, False)
  dW1 = nat.loss_backward(W, nf, lab, nl, *out1[1:], None, V, n, False)
  out2 = nat.loss_forward(W, nf, lab, nl, V, n, False)
  dW2 = nat.loss_backward(W, nf, lab, nl, *out2[1:], None, V, n, False)
  assert torch.equal(out1[0], out2[0])  # the loss is bitwise reproducible
  # dW (recursion backward): numerator marginals of positions sharing an arc
  # meet in LDS float atomics, so their summation order may vary run to run
  assert torch.allclose(dW1, dW2, atol=1e-6, rtol=0)
  # checkpointing path: fixed summation order -> bitwise reproducible, and
  # equal to the recursion path within rounding (for the bigram it runs the
  # scaled linear-space recursions of lt_pipe.hip, a different rounding)
  c1 = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
  d1 = nat.loss_backward(W, nf, lab, nl, *c1[1:5], None, V, n, False, ck=c1[5])
  c2 = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
  d2 = nat.loss_backward(W, nf, lab, nl, *c2[1:5], None, V, n, False, ck=c2[5])
  assert torch.equal(c1[0], c2[0]) and torch.equal(d1, d2)
  assert ((c1[0] - out1[0]).abs() <= 1e-5 + 1e-6 * out1[0].abs()).all()
  tol = 1e-5 + 2e-6 * out1[1].abs().clamp(min=1.0)[:, None, None, None]
  assert ((d1 - dW1).abs() <= tol).all()
  loss = out1[0]
  assert torch.isfinite(loss).all() and (loss > -1e-3).all()    # log_z >= numerator
  # linearity in the incoming gradient
  g = torch.linspace(0.5, 2.0, W.shape[0], device=W.device)
  dWg = nat.loss_backward(W, nf, lab, nl, *out1[1:], g, V, n, False)
  assert torch.allclose(dWg, dW1 * g[:, None, None, None], atol=1e-6, rtol=1e-5)
  # each live frame: den marginals sum to 1 and num marginals sum to 1
  s = dW1.double().reshape(W.shape[0], W.shape[1], -1).sum(-1)
  tol = 1e-5 + 2e-6 * out1[1].abs().double().clamp(min=1.0)[:, None]
  assert (s.abs() <= tol).all(), float((s.abs() / tol).max())


def test_full_size_den_backward_every_utterance(full_size):
  """lt_den_backward (the kernel behind _backward, _forward_backward, the
  _forward Log autograd and entropy) at the BASELINE shape: every utterance,
  every element of d log_z / dW against the oracle's den_grad under the
  per-element marginal bound (den-only: num = 0)."""
  orc = _orc()
  W, nf, _, _, V, n = full_size
  lz, al = nat.den_forward(W, nf, V, n, nat.SEMIRING_LOG)
  dW = nat.den_backward(W, nf, lz, al, None, V, n)
  rlz, den = orc.den_grad(W.cpu().numpy(), nf.cpu().numpy(), V, n)
  assert_loss_close(lz.cpu().numpy(), rlz)
  assert_grad_marginal_close(dW.cpu().numpy(), den, den, rlz, None)


@pytest.mark.parametrize('ckpt', [False, True])
def test_full_size_recursion_backward_vs_oracle(full_size, ckpt):
  """The recursion backward (lt_loss_forward + lt_loss_backward, the _NumFn
  string-gradient path and the non-chunked loss designs) and the
  checkpointing pair at T=1000 on 8 full utterances: loss and every dW
  element under the per-element marginal bound, plus the string-only
  gradient (local normalisation: -num marginals)."""
  orc = _orc()
  W, nf, lab, nl, V, n = full_size
  idx = [0, 5, 7, 13, 21, 34, 55, 63]
  Wc = W[idx].cpu().numpy()
  nfc, labc, nlc = (x[idx].cpu().numpy() for x in (nf, lab, nl))
  _, den = orc.den_grad(Wc, nfc, V, n)
  for local in (False, True):
    out = nat.loss_forward(W, nf, lab, nl, V, n, local, checkpoints=ckpt)
    dW = nat.loss_backward(W, nf, lab, nl, *out[1:5], None, V, n, local,
                           ck=out[5] if ckpt else None)
    rl, rlz, rnum, rdW = orc.loss_grad(Wc, nfc, labc, nlc, V, n, local_norm=local)
    assert_loss_close(out[0][idx].cpu().numpy(), rl)
    assert_grad_marginal_close(dW[idx].cpu().numpy(), rdW, None if local else den, rlz, rnum)


def test_full_size_viterbi_properties(full_size):
  """cfg4-class decode: the path weight is the MaxTropical distance, the
  one-hot arcs re-sum to it, and labels match the oracle on a sample."""
  orc = _orc()
  W, nf, _, _, V, n = full_size
  labels, weights, arcs = nat.viterbi(W, nf, V, n, nat.LABELS_TRUE, want_arcs=True)
  d, _ = nat.den_forward(W, nf, V, n, nat.SEMIRING_MAX, want_alpha=False)
  assert torch.equal(weights, d)
  resum = (arcs.double() * W.double()).sum(dim=(1, 2, 3))
  assert torch.allclose(resum, weights.double(), atol=1e-3, rtol=1e-6)
  per_frame = arcs.reshape(W.shape[0], W.shape[1], -1).sum(-1)
  live = (torch.arange(W.shape[1], device=W.device)[None, :] < nf[:, None].long()).float()
  assert torch.equal(per_frame.float(), live)
  idx = [0, 5]
  rlab, rw, _ = orc.viterbi(W[idx].cpu().numpy(), nf[idx].cpu().numpy(), V, n, convention=0)
  np.testing.assert_array_equal(labels[idx].cpu().numpy(), rlab)
  np.testing.assert_array_equal(weights[idx].cpu().numpy(), rw)
