"""Generates the golden fixtures in tests/golden/*.npz from the reference.

Run in the development container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference

The reference package is imported read-only from the given path; only the
numeric inputs and outputs are written (npz, no pickles). Every expected
value comes from the reference's own code:

  den_*      RecognitionLattice._forward            lattices.py:379-496
  num_*      RecognitionLattice._string_forward     lattices.py:250-377
  loss       RecognitionLattice.forward             lattices.py:131-183
  vit_*      RecognitionLattice.shortest_path       lattices.py:185-247 (B=1 per
             utterance); true-label mode from the same vjp mask
  den_grad   FrameDependent.backward composed in the correct reverse order
             (alignments.py:300-318, padding per lattices.py:775-779), float64
  num_grad   d/dW log(_string_forward under Real on exp(W)), float64 autograd
             (the Real semiring's autograd is sound; Log's is not)
  ctx_*      FullNGram next_state / forward_reduce / backward_broadcast /
             walk_states                            contexts.py:181-256, 109-146

Reference defects are handled as SURVEY.md 8c/Appendix A states: loss
gradients are den_grad - num_grad; unreachable numerators (loss = +inf) get
a zero gradient (the build's defined behaviour, the reference has none).
"""
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference(path):
  os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
  sys.dont_write_bytecode = True
  sys.path.insert(0, path)
  import last_torch  # noqa: F401
  return last_torch


def main(ref_path):
  lt = _import_reference(ref_path)
  torch.set_default_dtype(torch.float32)

  class Table64(lt.weight_fns.TableWeightFn):
    """TableWeightFn without the float32 cast (weight_fns.py:333), so that
    float64 fixtures stay float64 through the reference recursions."""

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

  def lattice_for(W, V, n, f64=False):
    table = torch.as_tensor(W)
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    fn = (lambda _: Table64(table)) if f64 else (lambda _: lt.weight_fns.TableWeightFn(table))
    return lt.RecognitionLattice(
        context=ctx, alignment=lt.alignments.FrameDependent(),
        weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
        weight_fn_factory=fn), ctx

  def frames_for(B, T):
    return torch.broadcast_to(torch.arange(T)[None, :, None], [B, T, 1]).float()

  def den(W, nf, V, n, semiring):
    lat, _ = lattice_for(W, V, n)
    B, T = W.shape[:2]
    with torch.no_grad():
      d, a = lat._forward(cache=None, frames=frames_for(B, T),
                          num_frames=torch.as_tensor(nf).float(), semiring=semiring)
    return d.numpy().astype(np.float32), a.numpy().astype(np.float32)

  def num(W, nf, lab, nl, V, n, semiring):
    lat, _ = lattice_for(W, V, n)
    B, T = W.shape[:2]
    with torch.no_grad():
      r = lat._string_forward(cache=None, frames=frames_for(B, T),
                              num_frames=torch.as_tensor(nf).float(),
                              labels=torch.as_tensor(lab).float(),
                              num_labels=torch.as_tensor(nl).float(), semiring=semiring)
    return r.numpy().astype(np.float32)

  def loss(W, nf, lab, nl, V, n, local):
    table = torch.as_tensor(W)
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    base = lambda _: lt.weight_fns.TableWeightFn(table)
    fn = (lambda c: lt.weight_fns.LocallyNormalizedWeightFn(base(c))) if local else base
    lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                                weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
                                weight_fn_factory=fn)
    B, T = W.shape[:2]
    with torch.no_grad():
      r = lat(frames=frames_for(B, T), num_frames=torch.as_tensor(nf).float(),
              labels=torch.as_tensor(lab).float(), num_labels=torch.as_tensor(nl).float())
    return r.numpy().astype(np.float32)

  def viterbi(W, nf, V, n):
    """Per-utterance shortest_path (D6) plus the true-label variant taken
    from the same vjp mask the reference differentiates (lattices.py:219-241)."""
    B, T = W.shape[:2]
    ref_labels = np.zeros([B, T], np.int64)
    true_labels = np.zeros([B, T], np.int64)
    weights = np.zeros([B], np.float32)
    for b in range(B):
      lat, _ = lattice_for(W[b:b + 1], V, n)
      fr = frames_for(1, T)
      nfb = torch.as_tensor(nf[b:b + 1]).float()
      labels, num_al, pw = lat.shortest_path(fr, nfb)
      ref_labels[b] = labels.numpy()[0]
      weights[b] = pw.detach().numpy()[0]
      assert num_al.numpy()[0] == nf[b]

      def helper(mask):
        d, _ = lat._forward(cache=None, frames=fr, num_frames=nfb,
                            semiring=lt.semirings.MaxTropical,
                            lexical_mask=[mask[..., 0, None, :]])
        return d
      mask = torch.zeros([1, T, 1, V])
      _, vjp = torch.func.vjp(helper, mask)
      m = vjp(torch.ones([1]))[0][0, :, 0, :]
      is_blank = torch.all(m == 0, dim=-1)
      true_labels[b] = torch.where(is_blank, 0, torch.argmax(m, dim=-1) + 1).numpy()
    return ref_labels, true_labels, weights

  def den_grad(W, nf, V, n):
    """d log_z / dW: FrameDependent.backward in reverse frame order, float64."""
    B, T, C, _ = W.shape
    W64 = W.astype(np.float64)
    lat, ctx = lattice_for(W64, V, n, f64=True)
    with torch.no_grad():
      log_z, alpha = lat._forward(cache=None, frames=frames_for(B, T),
                                  num_frames=torch.as_tensor(nf).double(),
                                  semiring=lt.semirings.Log)
    Wt = torch.as_tensor(W64)
    beta = torch.zeros([B, C], dtype=torch.float64)
    g = torch.zeros([B, T, C, V + 1], dtype=torch.float64)
    align = lt.alignments.FrameDependent()
    for t in reversed(range(T)):
      nb, bm, lm = align.backward(alpha[:, t], [Wt[:, t, :, 0]], [Wt[:, t, :, 1:]], beta,
                                  log_z, ctx)
      live = torch.as_tensor(t < nf)[:, None]
      beta = torch.where(live, nb, beta)
      g[:, t, :, 0] = torch.where(live, bm[0], 0.)
      g[:, t, :, 1:] = torch.where(live[..., None], lm[0], 0.)
    return log_z.numpy(), g.numpy()

  def num_grad(W, nf, lab, nl, V, n):
    """d num / dW with num = log of the Real-semiring string forward on exp(W),
    float64 autograd. The reference's own _string_forward casts its gather mask
    to float32 (lattices.py:324), so the float64 recursion is composed here from
    the same pieces: walk_states (contexts.py:109-146), the next-label padding
    and epsilon mapping (lattices.py:314-315, 336-338) and
    FrameDependent.string_forward (alignments.py:320-329) with the padding carry
    and final-position sum of lattices.py:353-377."""
    B, T, C, _ = W.shape
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    align = lt.alignments.FrameDependent()
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
      nxt_alpha = align.string_forward(alpha=alpha, blank=[blank], lexical=[lexw],
                                       semiring=real)
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

  def lattice_case(name, W, nf, lab, nl, V, n, bf16=False):
    W = np.ascontiguousarray(W, np.float32)
    if bf16:
      W = torch.tensor(W).bfloat16().float().numpy()
    nf = np.asarray(nf, np.int32)
    lab = np.asarray(lab, np.int32)
    nl = np.asarray(nl, np.int32)
    d = dict(W=W, num_frames=nf, labels=lab, num_labels=nl, vocab_size=np.int32(V),
             context_size=np.int32(n), bf16=np.int32(bf16))
    for sname in ('Log', 'MaxTropical', 'Real'):
      s = getattr(lt.semirings, sname)
      d[f'den_{sname}'], d[f'alpha_{sname}'] = den(W, nf, V, n, s)
      d[f'num_{sname}'] = num(W, nf, lab, nl, V, n, s)
    d['loss'] = loss(W, nf, lab, nl, V, n, local=False)
    d['loss_local'] = loss(W, nf, lab, nl, V, n, local=True)
    d['vit_labels_reference'], d['vit_labels_true'], d['vit_weights'] = viterbi(W, nf, V, n)
    lz64, dg = den_grad(W, nf, V, n)
    ng = num_grad(W, nf, lab, nl, V, n)
    reach = np.isfinite(d['num_Log'])[:, None, None, None]
    d['den_grad'] = dg.astype(np.float32)
    d['num_grad'] = ng.astype(np.float32)
    d['loss_grad'] = np.where(reach, dg - ng, 0.).astype(np.float32)
    # Locally normalised model: the lattice sees hat_normalize(W)
    # (weight_fns.py:99-117, the LocallyNormalizedWeightFn default) and the
    # loss is -numerator (lattices.py:178-179); its gradient is w.r.t. W_local.
    with torch.no_grad():
      Wt = torch.tensor(W)
      hb, hl = lt.weight_fns.hat_normalize(Wt[..., 0], Wt[..., 1:])
    W_local = torch.cat([hb[..., None], hl], dim=-1).numpy().astype(np.float32)
    if bf16:  # the bf16 kernels see W_local rounded to bf16: -numerator of that
      W_local = torch.tensor(W_local).bfloat16().float().numpy()
      d['loss_local'] = -num(W_local, nf, lab, nl, V, n, lt.semirings.Log)
    d['W_local'] = W_local
    ngl = num_grad(W_local, nf, lab, nl, V, n)
    reach_l = np.isfinite(num(W_local, nf, lab, nl, V, n, lt.semirings.Log))[:, None, None, None]
    d['loss_local_grad'] = np.where(reach_l, -ngl, 0.).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, f'lattice_{name}.npz'), **d)
    print('wrote', name, {k: v.shape for k, v in d.items() if v.ndim})

  # --- 1. the reference's own test_frame_dependent KAT (lattices_test.py:181-288)
  B, T, V, n, C = 3, 2, 2, 1, 3
  W = 1 + np.arange(B * T * C * (V + 1), dtype=np.float32).reshape(B, T, C, V + 1)
  W *= np.array([[-1, 1], [1, -1], [1, 1]], np.float32)[:, :, None, None]
  lattice_case('kat', W, [2, 1, 0], [[1, 2, 0], [2, 1, 0], [1, 2, 0]], [1, 1, 0], V, n)

  rng = np.random.default_rng(20250328)

  def rand_case(name, B, T, U, V, n, nf=None, nl=None, lab=None, kind='randn', bf16=False):
    C = (V ** (n + 1) - 1) // (V - 1) if V > 1 else n + 1
    if kind == 'randn':
      W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
    elif kind == 'ints':  # small integers: frequent exact ties in MaxTropical
      W = rng.integers(-2, 3, (B, T, C, V + 1)).astype(np.float32)
    elif kind == 'zeros':
      W = np.zeros((B, T, C, V + 1), np.float32)
    elif kind == 'peaked':  # large dynamic range: exercises the safe-max paths
      W = (rng.standard_normal((B, T, C, V + 1)) * 30).astype(np.float32)
    elif kind == 'lognorm':  # log_softmax over V+1 (SURVEY 8d locally normalised)
      x = rng.standard_normal((B, T, C, V + 1))
      W = (x - np.log(np.exp(x).sum(-1, keepdims=True))).astype(np.float32)
    nf = rng.integers(0, T + 1, B) if nf is None else nf
    lab = rng.integers(1, V + 1, (B, U)) if lab is None else lab
    nl = rng.integers(0, U + 1, B) if nl is None else nl
    lattice_case(name, W, nf, lab, nl, V, n, bf16=bf16)

  rand_case('unigram_v3', 3, 7, 3, 3, 0, nf=[7, 4, 0], nl=[3, 2, 0])
  rand_case('bigram_v3', 4, 9, 4, 3, 1, nf=[9, 5, 2, 0], nl=[4, 2, 3, 0])
  rand_case('bigram_v5', 2, 16, 6, 5, 1, nf=[16, 11], nl=[6, 5])
  rand_case('trigram_v2', 3, 11, 5, 2, 2, nf=[11, 8, 3], nl=[5, 3, 1])
  rand_case('trigram_v4', 2, 8, 3, 4, 2, nf=[8, 6], nl=[3, 2])
  rand_case('fourgram_v2', 2, 10, 4, 2, 3, nf=[10, 7], nl=[4, 2])
  rand_case('epsilon_labels', 3, 8, 5, 3, 1, nf=[8, 8, 6],
            lab=[[1, 0, 2, 0, 3], [0, 0, 1, 2, 0], [3, 3, 0, 1, 1]], nl=[5, 4, 3])
  rand_case('epsilon_trigram', 2, 9, 4, 3, 2, nf=[9, 7], lab=[[2, 0, 1, 3], [0, 2, 2, 0]],
            nl=[4, 4])
  rand_case('ties_ints', 4, 12, 4, 3, 1, nf=[12, 9, 4, 1], kind='ints')
  rand_case('ties_ints_trigram', 2, 10, 3, 2, 2, nf=[10, 6], kind='ints')
  rand_case('all_zero', 2, 6, 3, 3, 1, nf=[6, 3], nl=[3, 1], kind='zeros')
  rand_case('peaked', 3, 12, 4, 4, 1, nf=[12, 10, 7], nl=[4, 3, 2], kind='peaked')
  rand_case('locally_normalised', 2, 10, 4, 5, 1, nf=[10, 7], nl=[4, 3], kind='lognorm')
  rand_case('unreachable', 3, 5, 6, 3, 1, nf=[5, 2, 0], nl=[6, 3, 1])
  rand_case('bf16_bigram', 2, 10, 4, 5, 1, nf=[10, 9], nl=[4, 3], bf16=True)
  rand_case('v1_bigram', 2, 6, 3, 1, 1, nf=[6, 4], nl=[3, 2])
  # BASELINE.json configs[0] at its exact shape: B=2, T=8, U=4, vocab 5,
  # FullNGram order 0 (its own generator: the fixtures above stay as they were)
  rng_cfg1 = np.random.default_rng(1)
  lattice_case('cfg1', rng_cfg1.standard_normal((2, 8, 1, 6)).astype(np.float32), [8, 8],
               rng_cfg1.integers(1, 6, (2, 4)), [4, 4], 5, 0)

  # --- 2. FullNGram closed forms (contexts.py:181-256, 109-146)
  d = {}
  for V, n in [(3, 0), (3, 1), (3, 2), (2, 3), (5, 1), (4, 2)]:
    ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
    C, _ = ctx.shape()
    st = torch.arange(C)[:, None].expand(C, V + 1)
    y = torch.arange(V + 1)[None, :].expand(C, V + 1)
    d[f'next_{V}_{n}'] = ctx.next_state(st, y).numpy().astype(np.int32)
    x = torch.tensor(rng.standard_normal((2, C, V)).astype(np.float32))
    d[f'reduce_in_{V}_{n}'] = x.numpy()
    for sname in ('Log', 'MaxTropical', 'Real'):
      d[f'reduce_{sname}_{V}_{n}'] = ctx.forward_reduce(
          x, getattr(lt.semirings, sname)).numpy()
    b = torch.tensor(rng.standard_normal((2, C)).astype(np.float32))
    d[f'bcast_in_{V}_{n}'] = b.numpy()
    d[f'bcast_{V}_{n}'] = ctx.backward_broadcast(b).numpy()
    labs = torch.tensor(rng.integers(0, V + 1, (3, 6)))
    d[f'walk_in_{V}_{n}'] = labs.numpy().astype(np.int32)
    d[f'walk_{V}_{n}'] = ctx.walk_states(labs).numpy().astype(np.int32)
  np.savez_compressed(os.path.join(OUT, 'contexts.npz'), **d)
  print('wrote contexts', len(d))

  # --- 3. semiring reductions incl. -inf edge cases (semirings.py:184-401)
  d = {}
  x = np.array([[0., -np.inf, 2.], [-np.inf, -np.inf, -np.inf], [1., 1., 1.],
                [np.inf, 0., 1.], [-1e30, 3., -2.]], np.float32)
  y = np.array([[1., -np.inf, -np.inf], [-np.inf, 0., 5.], [1., 2., 0.],
                [0., 0., 0.], [3., -1e30, 7.]], np.float32)
  d['x'], d['y'] = x, y
  for sname in ('Log', 'MaxTropical', 'Real'):
    s = getattr(lt.semirings, sname)
    xt, yt = torch.tensor(x), torch.tensor(y)
    d[f'plus_{sname}'] = s.plus(xt, yt).numpy()
    d[f'times_{sname}'] = s.times(xt, yt).numpy()
    d[f'sum_{sname}'] = s.sum(xt, dim=-1).numpy()
    d[f'prod_{sname}'] = s.prod(xt, dim=-1).numpy()
    d[f'zeros_{sname}'] = s.zeros([2]).numpy()
    d[f'ones_{sname}'] = s.ones([2]).numpy()
  np.savez_compressed(os.path.join(OUT, 'semirings.npz'), **d)
  print('wrote semirings', len(d))


if __name__ == '__main__':
  main(sys.argv[1] if len(sys.argv) > 1 else '/root/reference')
