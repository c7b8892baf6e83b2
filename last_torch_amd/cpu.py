"""PyTorch CPU restatement of the lattice algorithms, for CPU tensors.

``RecognitionLattice`` runs here when its arc weights live on the CPU and on
the HIP kernels (liblt_lattice.so) when they live on a ROCm device: the
device of the tensors picks the implementation, as in the reference, and
there is no fallback from one to the other (a ROCm tensor never runs here;
a missing HIP library raises).

The formulation is the reference's own: a loop over frames vectorised over
the batch and the states, built from the plugin classes' per-frame methods
(``alignment.forward`` / ``string_forward``, ``context.forward_reduce``), with
gradients by torch autograd through the semirings' sound derivatives
(semirings.py). FrameDependent alignments (the north-star path).

  den_forward   lattices.py:379-496   shortest distance + alpha_0..T-1
  num_forward   lattices.py:250-377   string (numerator) distance
  loss          lattices.py:131-183   log_z - num (or -num, locally normalised)
  viterbi       lattices.py:185-247   max-tropical distance, labels from its
                                      derivative w.r.t. a lexical mask
"""
import torch

from last_torch_amd import alignments
from last_torch_amd import contexts
from last_torch_amd import semirings


def _check_alignment(alignment):
  if not isinstance(alignment, alignments.FrameDependent):
    raise NotImplementedError('the CPU lattice path implements FrameDependent alignments; '
                              f'got {type(alignment).__name__} (run it on a ROCm device)')


def _live(nf: torch.Tensor, t: int) -> torch.Tensor:
  return (t < nf)[:, None]


def den_forward(W: torch.Tensor, nf: torch.Tensor, context: contexts.ContextDependency,
                alignment, semiring) -> tuple[torch.Tensor, torch.Tensor]:
  """(dist [B], alpha_0..T-1 [B, T, C]) over W [B, T, C, V+1]: alpha_0 = one
  at the start state; frames t >= num_frames[b] leave alpha unchanged; dist =
  (+) of the final alphas (every state is final, lattices.py:496)."""
  _check_alignment(alignment)
  B, T, C, _ = W.shape
  one = semiring.ones([], W.dtype)
  zero = semiring.zeros([], W.dtype)
  alpha = torch.where(torch.arange(C) == context.start(), one, zero).expand(B, C)
  alphas = []
  for t in range(T):
    alphas.append(alpha)
    nxt = alignment.forward(alpha, [W[:, t, :, 0]], [W[:, t, :, 1:]], context, semiring)
    alpha = torch.where(_live(nf, t), nxt, alpha)
  alpha_all = torch.stack(alphas, dim=1) if alphas else W.new_zeros([B, 0, C])
  return semiring.sum(alpha, dim=-1), alpha_all


def string_weights(W: torch.Tensor, labels: torch.Tensor, context: contexts.ContextDependency):
  """Per frame the string lattice's arc weights [B, T, U+1]: blank[u] =
  W[ctx_u, 0] and lexical[u] = W[ctx_u, y_{u+1}] (the arc u -> u+1; none
  from u = U), ctx_u the context after the first u labels (walk_states,
  contexts.py:109-146). Labels outside 1..V read label 1's weight
  (make_safe_classes) and keep the context (epsilon)."""
  B, T, C, R = W.shape
  V = R - 1
  U = labels.shape[-1]
  lab = labels.long()
  ctx = context.walk_states(lab)                      # [B, U+1]
  safe = torch.where((lab >= 1) & (lab <= V), lab, torch.ones_like(lab))
  Wc = torch.gather(W, 2, ctx[:, None, :, None].expand(B, T, U + 1, R))  # [B, T, U+1, R]
  blank = Wc[..., 0]
  lex = torch.gather(Wc[:, :, :U, :], 3, safe[:, None, :, None].expand(B, T, U, 1))[..., 0]
  return blank, lex


def num_forward(W: torch.Tensor, nf: torch.Tensor, labels: torch.Tensor, nl: torch.Tensor,
                context: contexts.ContextDependency, alignment, semiring) -> torch.Tensor:
  """Shortest distance of the lattice intersected with the label string
  (lattices.py:250-377): alpha over string positions 0..U, read at nl."""
  _check_alignment(alignment)
  B, T = W.shape[:2]
  U = labels.shape[-1]
  blank, lex = string_weights(W, labels, context)
  zero = semiring.zeros([B, 1], W.dtype)
  one = semiring.ones([], W.dtype)
  alpha = torch.where(torch.arange(U + 1) == 0, one, semiring.zeros([], W.dtype)).expand(B, U + 1)
  for t in range(T):
    lex_t = torch.cat([lex[:, t], zero], dim=-1)   # no arc out of position U
    nxt = alignment.string_forward(alpha, [blank[:, t]], [lex_t], semiring)
    alpha = torch.where(_live(nf, t), nxt, alpha)
  ok = (nl >= 0) & (nl <= U)
  num = torch.gather(alpha, 1, nl.clamp(0, U).long()[:, None])[:, 0]
  return torch.where(ok, num, semiring.zeros([], W.dtype))


def loss(W: torch.Tensor, nf: torch.Tensor, labels: torch.Tensor, nl: torch.Tensor,
         context: contexts.ContextDependency, alignment, local_norm: bool) -> torch.Tensor:
  """-log P(labels | frames) = log_z - num, or -num for a locally
  normalised weight function (lattices.py:131-183)."""
  num = num_forward(W, nf, labels, nl, context, alignment, semirings.Log)
  if local_norm:
    out = -num
  else:
    log_z, _ = den_forward(W, nf, context, alignment, semirings.Log)
    out = log_z - num
  # an unreachable string (num = -inf, loss = +inf) contributes no gradient
  return torch.where(torch.isfinite(num), out, out.detach())


def viterbi(W: torch.Tensor, nf: torch.Tensor, context: contexts.ContextDependency, alignment,
            label_convention: str) -> tuple[torch.Tensor, torch.Tensor]:
  """Best path by differentiating the max-tropical distance w.r.t. a zero
  lexical mask (lattices.py:185-247): per frame the one-hot mask derivative
  names the lexical label taken, all-zero means blank. 'reference' emits
  label y as y - 1, 'true' emits y. Every utterance is decoded
  on its own (its distance depends on its own mask only)."""
  _check_alignment(alignment)
  B, T, C, R = W.shape
  with torch.enable_grad():
    mask = torch.zeros([B, T, 1, R - 1], dtype=W.dtype, requires_grad=True)
    Wm = torch.cat([W.detach()[..., :1], W.detach()[..., 1:] + mask], dim=-1)
    dist, _ = den_forward(Wm, nf, context, alignment, semirings.MaxTropical)
    (g,) = torch.autograd.grad(dist.sum(), mask, allow_unused=True)
  if g is None:
    g = torch.zeros_like(mask)
  g = g[:, :, 0, :]
  blank = torch.all(g == 0, dim=-1)
  idx = torch.argmax(g, dim=-1)
  lexical = idx if label_convention == 'reference' else idx + 1
  return torch.where(blank, torch.zeros_like(idx), lexical), dist.detach()
