"""Generates tests/golden/fld_*.npz: FrameLabelDependent(K) lattices computed
by the reference itself (alignments.py:331-432 driven by lattices.py).

Run in the development container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fld.py /root/reference

Every expected value comes from the reference's own code:

  den_*     RecognitionLattice._forward with alignment=FrameLabelDependent(K)
            (Log / MaxTropical / Real)                       lattices.py:379-496
  num_*     RecognitionLattice._string_forward (same alignment) lattices.py:250-377
  loss      RecognitionLattice.forward                       lattices.py:131-183
  den_grad  FrameLabelDependent.backward (alignments.py:379-419) composed in
            reverse frame order, float64; with alignment-state-invariant
            weights the K+1 blank and K lexical marginals of a frame add up
  num_grad  d num / dW, num = log of the Real-semiring
            FrameLabelDependent.string_forward (alignments.py:421-432) on
            exp(W), float64 autograd (Real's autograd is sound)
  loss_grad den_grad - num_grad; 0 for unreachable strings (the build's rule)

The reference's shortest_path is not used for K > 0: its lexical mask is
aliased across the batch and alignment states (scan_step_forward,
lattices.py:868-876), so only the path weight (= den_MaxTropical)
is pinned; the alignment labels are checked against the C oracle and the
reference test's invariants (tests/lattices_test.py:145-176).
"""
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def main(ref_path):
  os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
  sys.dont_write_bytecode = True
  sys.path.insert(0, ref_path)
  import last_torch as lt
  torch.set_default_dtype(torch.float32)

  class Table64(lt.weight_fns.TableWeightFn):
    """TableWeightFn without the float32 cast (weight_fns.py:333)."""

    def forward(self, cache, frame, state=None):
      del cache
      *batch, _, c, _ = self.table.shape
      row = frame[..., 0].long()
      idx = row[..., None, None, None].expand(*batch, 1, c, self.table.shape[-1])
      w = torch.take_along_dim(self.table, idx, dim=-3)[..., 0, :, :]
      if state is not None:
        st = torch.broadcast_to(torch.as_tensor(state), tuple(batch)).long()
        w = torch.take_along_dim(w, st[..., None, None].expand(*batch, 1, w.shape[-1]),
                                 dim=-2)[..., 0, :]
      return w[..., 0], w[..., 1:]

  def lattice_for(W, V, n, K, f64=False, local=False):
    table = torch.as_tensor(W)
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    base = (lambda _: Table64(table)) if f64 else (lambda _: lt.weight_fns.TableWeightFn(table))
    fn = (lambda c: lt.weight_fns.LocallyNormalizedWeightFn(base(c))) if local else base
    return lt.RecognitionLattice(
        context=ctx, alignment=lt.alignments.FrameLabelDependent(max_expansions=K),
        weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
        weight_fn_factory=fn), ctx

  def frames_for(B, T):
    return torch.broadcast_to(torch.arange(T)[None, :, None], [B, T, 1]).float()

  def den(W, nf, V, n, K, semiring):
    lat, _ = lattice_for(W, V, n, K)
    B, T = W.shape[:2]
    with torch.no_grad():
      d, a = lat._forward(cache=None, frames=frames_for(B, T),
                          num_frames=torch.as_tensor(nf).float(), semiring=semiring)
    return d.numpy().astype(np.float32), a.numpy().astype(np.float32)

  def num(W, nf, lab, nl, V, n, K, semiring):
    lat, _ = lattice_for(W, V, n, K)
    B, T = W.shape[:2]
    with torch.no_grad():
      r = lat._string_forward(cache=None, frames=frames_for(B, T),
                              num_frames=torch.as_tensor(nf).float(),
                              labels=torch.as_tensor(lab).float(),
                              num_labels=torch.as_tensor(nl).float(), semiring=semiring)
    return r.numpy().astype(np.float32)

  def loss(W, nf, lab, nl, V, n, K):
    lat, _ = lattice_for(W, V, n, K)
    B, T = W.shape[:2]
    with torch.no_grad():
      r = lat(frames=frames_for(B, T), num_frames=torch.as_tensor(nf).float(),
              labels=torch.as_tensor(lab).float(), num_labels=torch.as_tensor(nl).float())
    return r.numpy().astype(np.float32)

  def den_grad(W, nf, V, n, K):
    B, T, C, _ = W.shape
    W64 = W.astype(np.float64)
    lat, ctx = lattice_for(W64, V, n, K, f64=True)
    with torch.no_grad():
      log_z, alpha = lat._forward(cache=None, frames=frames_for(B, T),
                                  num_frames=torch.as_tensor(nf).double(),
                                  semiring=lt.semirings.Log)
    Wt = torch.as_tensor(W64)
    beta = torch.zeros([B, C], dtype=torch.float64)
    g = torch.zeros([B, T, C, V + 1], dtype=torch.float64)
    align = lt.alignments.FrameLabelDependent(max_expansions=K)
    for t in reversed(range(T)):
      blank = [Wt[:, t, :, 0]] * (K + 1)
      lex = [Wt[:, t, :, 1:]] * (K + 1)
      nb, bm, lm = align.backward(alpha[:, t], blank, lex, beta, log_z, ctx)
      live = torch.as_tensor(t < nf)[:, None]
      beta = torch.where(live, nb, beta)
      g[:, t, :, 0] = torch.where(live, sum(bm), 0.)
      g[:, t, :, 1:] = torch.where(live[..., None], sum(lm), 0.)
    return log_z.numpy(), g.numpy()

  def num_grad(W, nf, lab, nl, V, n, K):
    """Composed from the reference's pieces in float64: walk_states
    (contexts.py:109-146), next-label padding / epsilon class 1
    (lattices.py:314-315, 336-338), FrameLabelDependent.string_forward under
    Real with the padding carry and final-position sum of lattices.py:353-377."""
    B, T, C, _ = W.shape
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    align = lt.alignments.FrameLabelDependent(max_expansions=K)
    real = lt.semirings.Real
    labels = torch.as_tensor(lab).long()
    U = labels.shape[-1]
    states = ctx.walk_states(labels).long()
    nxt = torch.cat([labels, torch.ones_like(labels[..., :1])], dim=-1)
    nxt = torch.where(nxt - 1 < 0, 1, nxt)
    E = torch.tensor(np.exp(W.astype(np.float64)), requires_grad=True)
    bi = torch.arange(B)[:, None]
    alpha = torch.zeros([B, U + 1], dtype=torch.float64)
    alpha[:, 0] = 1.
    nf_t = torch.as_tensor(nf)
    for t in range(T):
      blank = E[bi, t, states, 0]
      lexw = E[bi, t, states, nxt]
      nxt_alpha = align.string_forward(alpha=alpha, blank=[blank] * (K + 1),
                                       lexical=[lexw] * (K + 1), semiring=real)
      alpha = torch.where((t >= nf_t)[:, None], alpha, nxt_alpha)
    is_final = torch.as_tensor(nl)[:, None] == torch.arange(U + 1)
    r = real.sum(torch.where(is_final, alpha, 0.), dim=-1)
    (gE,) = torch.autograd.grad(r.sum(), E, allow_unused=True)
    if gE is None:
      gE = torch.zeros_like(E)
    with torch.no_grad():
      ok = (r > 0)[:, None, None, None]
      g = torch.where(ok, gE * E / torch.where(r > 0, r, 1.)[:, None, None, None], 0.)
    return g.numpy()

  def case(name, B, T, U, V, n, K, seed, nf=None, nl=None, lab=None, scale=1.0):
    rng = np.random.default_rng(seed)
    C = lt.contexts.FullNGram(vocab_size=V, context_size=n).num_states()
    W = (scale * rng.standard_normal((B, T, C, V + 1))).astype(np.float32)
    nf = np.asarray(nf if nf is not None else rng.integers(0, T + 1, B), np.int32)
    nf[0] = T
    lab = np.asarray(lab if lab is not None else rng.integers(1, V + 1, (B, U)), np.int32)
    nl = np.asarray(nl if nl is not None else rng.integers(0, U + 1, B), np.int32)
    d = {'W': W, 'num_frames': nf, 'labels': lab, 'num_labels': nl,
         'vocab_size': np.int32(V), 'context_size': np.int32(n), 'K': np.int32(K)}
    for s in ('Log', 'MaxTropical', 'Real'):
      sr = getattr(lt.semirings, s)
      d[f'den_{s}'], d[f'alpha_{s}'] = den(W, nf, V, n, K, sr)
      d[f'num_{s}'] = num(W, nf, lab, nl, V, n, K, sr)
    d['loss'] = loss(W, nf, lab, nl, V, n, K)
    lz, dg = den_grad(W, nf, V, n, K)
    ng = num_grad(W, nf, lab, nl, V, n, K)
    reach = np.isfinite(d['loss'])[:, None, None, None]
    d['den_grad'] = dg.astype(np.float32)
    d['loss_grad'] = np.where(reach, dg - ng, 0.).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, f'fld_{name}.npz'), **d)
    print(name, 'loss', d['loss'], 'den', d['den_Log'])

  # the reference test's shape (tests/lattices_test.py:129-176): V=2 bigram, K=2
  case('test_shape', 4, 6, 4, 2, 1, 2, seed=1, nf=[6, 3, 2, 1], nl=[4, 3, 4, 3],
       lab=[[1, 1, 1, 1], [2, 2, 2, 2], [1, 2, 1, 2], [2, 1, 2, 1]])
  case('k1_bigram_v3', 3, 7, 5, 3, 1, 1, seed=2)
  case('k3_bigram_v4', 3, 6, 6, 4, 1, 3, seed=3)
  case('k2_unigram_v5', 3, 5, 4, 5, 0, 2, seed=4)
  case('k2_trigram_v2', 2, 5, 4, 2, 2, 2, seed=5)
  case('k2_epsilon', 3, 6, 5, 3, 1, 2, seed=6,
       lab=[[0, 1, 0, 2, 3], [3, 0, 0, 1, 0], [0, 0, 0, 0, 0]], nl=[5, 4, 2])
  case('k2_peaked', 2, 6, 3, 3, 1, 2, seed=7, scale=30.0)


if __name__ == '__main__':
  main(sys.argv[1] if len(sys.argv) > 1 else '/root/reference')
