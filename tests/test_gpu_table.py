"""GPU parity of the general lattice kernels (lt_table.hip): any next-state
table, FrameDependent (K = 0) or FrameLabelDependent(K), through the C ABI
and through RecognitionLattice.

Oracles: the reference's own FrameLabelDependent fixtures
(tests/golden/make_golden_fld.py), every FullNGram fixture (via
FullNGram.next_state_table()), and the pinned table oracle
(oracle/table_oracle.c) for random DFAs. Tolerances as test_gpu_parity.py:
Log values 1e-4 * max(1, |ref|); MaxTropical values and Viterbi labels
bit-exact; dW element by element within golden_cases.marginal_scale
(relative to the arc's own den + num marginals; the den marginals from the
fixture's den_grad or, for random tables, golden_cases.table_den_marginals).
"""
import numpy as np
import pytest
import torch

import last_torch_amd as lt
from last_torch_amd import _native as nat
from golden_cases import (FLD_CASES, LATTICE_CASES, assert_grad_marginal_close, assert_loss_close,
                          assert_values_close, load, load_fld, table_den_marginals)

pytestmark = pytest.mark.gpu

SID = {'Log': nat.SEMIRING_LOG, 'MaxTropical': nat.SEMIRING_MAX, 'Real': nat.SEMIRING_REAL}


def _orc():
  from oracle import oracle as orc  # test infrastructure only
  return orc


def _real_tol(ref):
  return dict(rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(ref[np.isfinite(ref)]).max(initial=0))))


def _check_case(c, K, cuda, bf16=False):
  orc = _orc()
  V, n = c['V'], c['n']
  table = orc.full_ngram_table(V, n)
  g = nat.TableGraph(table, K, cuda)
  W = torch.tensor(c['W']).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nf = torch.tensor(c['num_frames']).to(cuda)
  lab = torch.tensor(c['labels']).to(cuda)
  nl = torch.tensor(c['num_labels']).to(cuda)
  for s in ('Log', 'MaxTropical', 'Real'):
    d, a = nat.table_forward(g, W, nf, SID[s])
    num = nat.table_num_forward(g, W, nf, lab, nl, SID[s])
    d, a, num = d.cpu().numpy(), a.cpu().numpy(), num.cpu().numpy()
    if s == 'MaxTropical':
      np.testing.assert_array_equal(d, c['den_MaxTropical'])
      np.testing.assert_array_equal(a, c['alpha_MaxTropical'])
      np.testing.assert_array_equal(num, c['num_MaxTropical'])
    elif s == 'Log':
      assert_loss_close(d, c['den_Log'])
      assert_values_close(a, c['alpha_Log'], rtol=1e-4, atol=1e-4)
      assert_loss_close(num, c['num_Log'])
    else:
      assert_values_close(d, c['den_Real'], **_real_tol(c['den_Real']))
  loss, lz, _, dW = nat.table_loss_grad(g, W, nf, lab, nl, False)
  assert_loss_close(loss.cpu().numpy(), c['loss'])
  assert_grad_marginal_close(dW.float().cpu().numpy(), c['loss_grad'], c['den_grad'], c['den_Log'],
                             c['num_Log'], bf16)
  for conv in (0, 1):
    labels, w = nat.table_viterbi(g, W, nf, conv)
    rl, rw = orc.tab_viterbi(table, c['W'], c['num_frames'], K, conv)
    np.testing.assert_array_equal(w.cpu().numpy(), c['den_MaxTropical'])
    np.testing.assert_array_equal(labels.cpu().numpy(), rl)


@pytest.mark.parametrize('case', FLD_CASES)
def test_fld_fixtures(cuda, case):
  c = load_fld(case)
  _check_case(c, c['K'], cuda)


@pytest.mark.parametrize('case', [k for k in LATTICE_CASES if not k.startswith('bf16')])
def test_full_ngram_fixtures_through_table(cuda, case):
  """K = 0 with FullNGram.next_state_table() reproduces the FullNGram
  fixtures (and the tuned kernels' Viterbi labels)."""
  c = load(case)
  _check_case(c, 0, cuda)
  np.testing.assert_array_equal(
      nat.table_viterbi(nat.TableGraph(_orc().full_ngram_table(c['V'], c['n']), 0, cuda),
                        torch.tensor(c['W']).to(cuda), torch.tensor(c['num_frames']).to(cuda),
                        1)[0].cpu().numpy(), c['vit_labels_reference'])


RANDOM_DFA = [
    # C, V, K, B, T, U, dtype
    (7, 4, 0, 4, 30, 6, 'f32'),
    (7, 4, 1, 4, 30, 6, 'f32'),
    (7, 4, 2, 4, 30, 6, 'bf16'),
    (23, 9, 3, 3, 25, 8, 'f32'),
    (1, 6, 2, 3, 20, 5, 'f32'),
    (40, 16, 2, 2, 40, 12, 'f32'),
]


@pytest.mark.parametrize('C,V,K,B,T,U,dt', RANDOM_DFA)
def test_random_dfa_vs_oracle(cuda, C, V, K, B, T, U, dt):
  orc = _orc()
  rng = np.random.default_rng(C * 100 + V * 10 + K)
  table = rng.integers(0, C, (C, V)).astype(np.int32)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  bf16 = dt == 'bf16'
  if bf16:
    W = torch.tensor(W).bfloat16().float().numpy()
  nf = rng.integers(0, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(0, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(0, U + 1, B).astype(np.int32)
  g = nat.TableGraph(table, K, cuda)
  Wd = torch.tensor(W).to(torch.bfloat16 if bf16 else torch.float32).to(cuda)
  nfd, labd, nld = (torch.tensor(x).to(cuda) for x in (nf, lab, nl))
  for s, sid in (('Log', orc.LOG), ('MaxTropical', orc.MAX)):
    d, _ = nat.table_forward(g, Wd, nfd, SID[s], want_alpha=False)
    rd = orc.tab_den_forward(table, W, nf, K, sid)
    num = nat.table_num_forward(g, Wd, nfd, labd, nld, SID[s])
    rn = orc.tab_num_forward(table, W, nf, lab, nl, K, sid)
    if s == 'MaxTropical':
      np.testing.assert_array_equal(d.cpu().numpy(), rd)
      np.testing.assert_array_equal(num.cpu().numpy(), rn)
    else:
      assert_loss_close(d.cpu().numpy(), rd)
      assert_loss_close(num.cpu().numpy(), rn)
  den = table_den_marginals(orc, table, W, nf, lab, nl, K)
  for local in (False, True):
    loss, lz, _, dW = nat.table_loss_grad(g, Wd, nfd, labd, nld, local)
    rl, rlz, rnum, rdW = orc.tab_loss_grad(table, W, nf, lab, nl, K, local_norm=local)
    assert_loss_close(loss.cpu().numpy(), rl)
    assert_grad_marginal_close(dW.float().cpu().numpy(), rdW, None if local else den, rlz, rnum,
                               bf16)
  labels, w = nat.table_viterbi(g, Wd, nfd, 0)
  rlab, rw = orc.tab_viterbi(table, W, nf, K, 0)
  np.testing.assert_array_equal(w.cpu().numpy(), rw)
  np.testing.assert_array_equal(labels.cpu().numpy(), rlab)


def _table_lattice(context, alignment, table):
  return lt.RecognitionLattice(
      context=context, alignment=alignment,
      weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
      weight_fn_factory=lambda _: lt.weight_fns.TableWeightFn(table))


def test_frame_label_dependent_api(cuda):
  """tests/lattices_test.py:129-176 (the reference's FrameLabelDependent
  test) on the kernels, with its invariants, plus the loss gradient against
  the oracle."""
  orc = _orc()
  V, n, K = 2, 1, 2
  B, T = 4, 6
  rng = np.random.default_rng(3)
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  table = torch.tensor(W, device=cuda, requires_grad=True)
  lat = _table_lattice(lt.contexts.FullNGram(vocab_size=V, context_size=n),
                       lt.alignments.FrameLabelDependent(max_expansions=K), table)
  frames = torch.arange(T, dtype=torch.float32, device=cuda)[None, :, None].expand(B, T, 1).contiguous()
  num_frames = torch.tensor([6, 3, 2, 1])
  labels = torch.tensor([[1, 1, 1, 1], [2, 2, 2, 2], [1, 2, 1, 2], [2, 1, 2, 1]])
  num_labels = torch.tensor([4, 3, 4, 3])
  loss = lat(frames, num_frames, labels, num_labels)
  np.testing.assert_array_equal(torch.isfinite(loss).cpu().numpy(), [True, True, True, False])
  fin = torch.isfinite(loss.detach())
  loss.masked_fill(~fin, 0).sum().backward()
  tab = orc.full_ngram_table(V, n)
  args = (num_frames.numpy().astype(np.int32), labels.numpy().astype(np.int32),
          num_labels.numpy().astype(np.int32), K)
  rl, rlz, rnum, rdW = orc.tab_loss_grad(tab, W, *args)
  assert_loss_close(loss.detach().cpu().numpy(), rl)
  assert_grad_marginal_close(table.grad.cpu().numpy(), rdW, table_den_marginals(orc, tab, W, *args),
                             rlz, rnum, weights=fin.float().cpu().numpy())
  al, nal, pw = lat.shortest_path(frames, num_frames)
  np.testing.assert_array_equal(nal.numpy(), 3 * num_frames.numpy())
  is_padding = torch.arange(18) >= nal[:, None]
  np.testing.assert_array_equal(is_padding.int().numpy(),
                                [[0] * 18, [0] * 9 + [1] * 9, [0] * 6 + [1] * 12,
                                 [0] * 3 + [1] * 15])
  al = al.cpu()
  np.testing.assert_array_equal(al.reshape(4, 6, 3)[..., -1].numpy(), np.zeros([4, 6]))
  assert ((al >= 0) & (al <= V)).all()
  assert torch.isfinite(pw).all()
  d, _ = lat._forward(None, frames, num_frames, lt.semirings.MaxTropical)
  np.testing.assert_array_equal(pw.cpu().numpy(), d.detach().cpu().numpy())


def test_next_state_table_api(cuda):
  """A NextStateTable context through RecognitionLattice: loss, gradient,
  distances and Viterbi against the table oracle."""
  orc = _orc()
  rng = np.random.default_rng(9)
  C, V, B, T, U = 6, 3, 3, 12, 4
  tab = rng.integers(0, C, (C, V)).astype(np.int32)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  table = torch.tensor(W, device=cuda, requires_grad=True)
  ctx = lt.contexts.NextStateTable(torch.tensor(tab))
  for K, align in ((0, lt.alignments.FrameDependent()),
                   (1, lt.alignments.FrameLabelDependent(max_expansions=1))):
    lat = _table_lattice(ctx, align, table)
    frames = torch.arange(T, dtype=torch.float32, device=cuda)[None, :, None].expand(B, T, 1).contiguous()
    nf = np.array([12, 7, 3], np.int32)
    lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
    nl = np.array([4, 2, 1], np.int32)
    table.grad = None
    loss = lat(frames, torch.tensor(nf), torch.tensor(lab), torch.tensor(nl))
    fin = torch.isfinite(loss.detach())
    loss.masked_fill(~fin, 0).sum().backward()
    rl, rlz, rnum, rdW = orc.tab_loss_grad(tab, W, nf, lab, nl, K)
    assert_loss_close(loss.detach().cpu().numpy(), rl)
    assert_grad_marginal_close(table.grad.cpu().numpy(), rdW,
                               table_den_marginals(orc, tab, W, nf, lab, nl, K), rlz, rnum,
                               weights=fin.float().cpu().numpy())
    d, _ = lat._forward(None, frames, torch.tensor(nf), lt.semirings.Log)
    assert_loss_close(d.detach().cpu().numpy(), orc.tab_den_forward(tab, W, nf, K, orc.LOG))
    s = lat._string_forward(None, frames, torch.tensor(nf), torch.tensor(lab), torch.tensor(nl),
                            lt.semirings.MaxTropical)
    np.testing.assert_array_equal(s.detach().cpu().numpy(),
                                  orc.tab_num_forward(tab, W, nf, lab, nl, K, orc.MAX))
    al, nal, pw = lat.shortest_path(frames, torch.tensor(nf), label_convention='true')
    rlab, rw = orc.tab_viterbi(tab, W, nf, K, 0)
    np.testing.assert_array_equal(al.cpu().numpy(), rlab)
    np.testing.assert_array_equal(pw.cpu().numpy(), rw)


def test_fld_k2_bigram_full_length(cuda):
  """FrameLabelDependent(K=2) bigram at B=8, T=1000, U=100, V=32 (the
  general table kernels at the BASELINE frame count): loss, log_z and every
  dW element against the table oracle under the per-element marginal bound,
  the string-only gradient (local normalisation) too."""
  orc = _orc()
  V, n, K, B, T, U = 32, 1, 2, 8, 1000, 100
  rng = np.random.default_rng(1000)
  tab = orc.full_ngram_table(V, n)
  W = rng.standard_normal((B, T, V + 1, V + 1)).astype(np.float32)
  nf = rng.integers(T // 2, T + 1, B).astype(np.int32)
  nf[0] = T
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = rng.integers(U // 2, U + 1, B).astype(np.int32)
  g = nat.TableGraph(tab, K, cuda)
  Wd = torch.tensor(W, device=cuda)
  nfd, labd, nld = (torch.tensor(x, device=cuda) for x in (nf, lab, nl))
  den = table_den_marginals(orc, tab, W, nf, lab, nl, K)
  for local in (False, True):
    loss, lz, _, dW = nat.table_loss_grad(g, Wd, nfd, labd, nld, local)
    rl, rlz, rnum, rdW = orc.tab_loss_grad(tab, W, nf, lab, nl, K, local_norm=local)
    assert_loss_close(loss.cpu().numpy(), rl)
    if not local:
      assert_loss_close(lz.cpu().numpy(), rlz)
    assert_grad_marginal_close(dW.cpu().numpy(), rdW, None if local else den, rlz, rnum)
