"""Alignment lattices (mirrors last_torch/alignments.py).

``FrameDependent`` and ``FrameLabelDependent(K)`` are both run by HIP
kernels: FrameDependent x FullNGram by the tuned kernels (lt_lattice.hip,
lt_pipe.hip), everything else by the general table kernels (lt_table.hip).
The per-frame methods below are the plugin surface (alignments.py:54-230),
evaluated with torch ops on any device; ``RecognitionLattice`` does not
call them on its hot path.
"""
import abc
from collections.abc import Sequence
from typing import Optional

import torch

from last_torch_amd import contexts
from last_torch_amd import semirings


class TimeSyncAlignmentLattice(abc.ABC):
  """A frame-local alignment automaton repeated once per frame
  (alignments.py:26-230)."""

  @abc.abstractmethod
  def num_states(self) -> int:
    """Number of non-final frame-local alignment states."""

  @abc.abstractmethod
  def start(self) -> int:
    """Start state of the frame-local alignment lattice."""

  @abc.abstractmethod
  def blank_next(self, state: int) -> Optional[int]:
    """Next state after a blank arc (None if there is none)."""

  @abc.abstractmethod
  def lexical_next(self, state: int) -> Optional[int]:
    """Next state after a lexical arc (None if there is none)."""

  @abc.abstractmethod
  def topological_visit(self) -> list[int]:
    """Non-final states in topological order."""

  @abc.abstractmethod
  def forward(self, alpha: torch.Tensor, blank: Sequence[torch.Tensor],
              lexical: Sequence[torch.Tensor], context: contexts.ContextDependency,
              semiring: semirings.Semiring) -> torch.Tensor:
    """One frame of the forward algorithm: alpha_t -> alpha_{t+1}."""

  @abc.abstractmethod
  def backward(self, alpha: torch.Tensor, blank: Sequence[torch.Tensor],
               lexical: Sequence[torch.Tensor], beta: torch.Tensor, log_z: torch.Tensor,
               context: contexts.ContextDependency):
    """One frame of the backward algorithm: (beta_t, blank marginals,
    lexical marginals) from beta_{t+1} (Log semiring)."""

  @abc.abstractmethod
  def string_forward(self, alpha: torch.Tensor, blank: Sequence[torch.Tensor],
                     lexical: Sequence[torch.Tensor],
                     semiring: semirings.Semiring) -> torch.Tensor:
    """One frame of the forward algorithm on the label-string acceptor."""


def shift_down(x: torch.Tensor, semiring: semirings.Semiring) -> torch.Tensor:
  """out[..., i+1] = x[..., i]; out[..., 0] = semiring zero (alignments.py:233-248)."""
  pad = semiring.zeros((*x.shape[:-1], 1), x.dtype, x.device)
  return torch.cat([pad, x[..., :-1]], dim=-1)


def check_num_weights(alignment: TimeSyncAlignmentLattice, blank: Sequence[torch.Tensor],
                      lexical: Sequence[torch.Tensor]) -> None:
  """Exactly one blank / lexical array per alignment state (alignments.py:251-263)."""
  k = alignment.num_states()
  if len(blank) != k:
    raise ValueError(f'blank should be a length {k} sequence of ndarrays, '
                     f'but got length {len(blank)}')
  if len(lexical) != k:
    raise ValueError(f'lexical should be a length {k} sequence of ndarrays, '
                     f'but got length {len(lexical)}')


def _reach(alpha, lexical, step):
  """[alpha, L alpha, L^2 alpha, ...]: the context vectors of the frame-local
  states reached after 0, 1, ... lexical arcs, one per weight array in
  ``lexical`` (``step(v, w)`` takes one arc)."""
  reached = [alpha]
  for w in lexical:
    reached.append(step(reached[-1], w))
  return reached


def _context_step(context, semiring):
  return lambda v, w: context.forward_reduce(semiring.times(v[..., None], w), semiring)


def _string_step(semiring):
  return lambda v, w: shift_down(semiring.times(v, w), semiring)


def _completions(blank, lex_to, beta):
  """Log-space completion weights of one frame, last alignment state first.

  ``done[i]`` is the total weight from alignment state i to the end of the
  lattice through this frame's blank (which closes the frame onto beta) or a
  lexical arc to ``lex_to(i)``; returns ``done`` and the per-arc lexical
  totals ``lex[i] = lexical_i + beta_of(lex_to(i))`` the marginals share.
  """
  k = len(blank)
  done, lex = [None] * k, [None] * k
  for i in range(k - 1, -1, -1):
    closed = blank[i] + beta
    target = lex_to(i, done)
    if target is None:
      done[i] = closed
      continue
    lex[i] = target
    done[i] = semirings.Log.plus(closed, semirings.Log.sum(target, dim=-1))
  return done, lex


class FrameDependent(TimeSyncAlignmentLattice):
  """Each frame emits exactly one blank or one lexical label
  (alignments.py:266-329)."""

  def num_states(self) -> int:
    return 1

  def start(self) -> int:
    return 0

  def blank_next(self, state: int) -> Optional[int]:
    return 0

  def lexical_next(self, state: int) -> Optional[int]:
    return 0

  def topological_visit(self) -> list[int]:
    return [0]

  def forward(self, alpha, blank, lexical, context, semiring):
    """alignments.py:286-298: alpha (x) blank (+) the label arcs' reduce."""
    check_num_weights(self, blank, lexical)
    emitted = _context_step(context, semiring)(alpha, lexical[0])
    return semiring.plus(semiring.times(alpha, blank[0]), emitted)

  def backward(self, alpha, blank, lexical, beta, log_z, context):
    """alignments.py:300-318: both arcs leave the frame, so the lexical arcs
    land on beta_{t+1} itself."""
    check_num_weights(self, blank, lexical)
    done, lex = _completions(blank, lambda i, _: lexical[0] + context.backward_broadcast(beta),
                             beta)
    rel = alpha - log_z[..., None]
    return done[0], [torch.exp(rel + blank[0] + beta)], [torch.exp(rel[..., None] + lex[0])]

  def string_forward(self, alpha, blank, lexical, semiring):
    """alignments.py:320-329 on the string acceptor (shift_down)."""
    check_num_weights(self, blank, lexical)
    return semiring.plus(semiring.times(alpha, blank[0]),
                         _string_step(semiring)(alpha, lexical[0]))


class FrameLabelDependent(TimeSyncAlignmentLattice):
  """Each frame emits up to ``max_expansions`` lexical labels followed by one
  blank (alignments.py:331-432). Alignment state i counts the lexical labels
  emitted so far in the frame."""

  def __init__(self, max_expansions: int) -> None:
    super().__init__()
    self.max_expansions = max_expansions

  def num_states(self) -> int:
    return self.max_expansions + 1

  def start(self) -> int:
    return 0

  def blank_next(self, state: int) -> Optional[int]:
    return 0

  def lexical_next(self, state: int) -> Optional[int]:
    nxt = state + 1
    return nxt if nxt <= self.max_expansions else None

  def topological_visit(self) -> list[int]:
    return list(range(self.max_expansions + 1))

  def _closed(self, reached, blank, semiring):
    return semiring.sum(torch.stack([semiring.times(v, w) for v, w in zip(reached, blank)]), dim=0)

  def forward(self, alpha, blank, lexical, context, semiring):
    """alignments.py:363-377: (+)_i (L^i alpha) (x) blank[i]."""
    check_num_weights(self, blank, lexical)
    reached = _reach(alpha, lexical[:self.max_expansions], _context_step(context, semiring))
    return self._closed(reached, blank, semiring)

  def backward(self, alpha, blank, lexical, beta, log_z, context):
    """alignments.py:379-419: (beta_t, blank marginals [K+1], lexical
    marginals [K+1], the last all zero) of one frame, Log semiring. State i's
    lexical arcs lead to state i + 1 of the same frame; state K has none."""
    check_num_weights(self, blank, lexical)
    K = self.max_expansions
    reached = _reach(alpha, lexical[:K], _context_step(context, semirings.Log))
    done, lex = _completions(
        blank,
        lambda i, d: None if i == K else lexical[i] + context.backward_broadcast(d[i + 1]),
        beta)
    rel = [v - log_z[..., None] for v in reached]
    blank_m = [torch.exp(r + w + beta) for r, w in zip(rel, blank)]
    lex_m = [torch.exp(rel[i][..., None] + lex[i]) for i in range(K)]
    return done[0], blank_m, lex_m + [torch.zeros_like(lexical[K])]

  def string_forward(self, alpha, blank, lexical, semiring):
    """alignments.py:421-432 on the string acceptor (shift_down)."""
    check_num_weights(self, blank, lexical)
    reached = _reach(alpha, lexical[:self.max_expansions], _string_step(semiring))
    return self._closed(reached, blank, semiring)
