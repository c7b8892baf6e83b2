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
    check_num_weights(self, blank, lexical)
    stay = semiring.times(alpha, blank[0])
    move = context.forward_reduce(semiring.times(alpha[..., None], lexical[0]), semiring)
    return semiring.plus(stay, move)

  def backward(self, alpha, blank, lexical, beta, log_z, context):
    check_num_weights(self, blank, lexical)
    blank_beta = blank[0] + beta
    lexical_beta = lexical[0] + context.backward_broadcast(beta)
    scale = alpha - log_z[..., None]
    blank_marginal = torch.exp(blank_beta + scale)
    lexical_marginal = torch.exp(lexical_beta + scale[..., None])
    next_beta = semirings.Log.plus(blank_beta, semirings.Log.sum(lexical_beta, dim=-1))
    return next_beta, [blank_marginal], [lexical_marginal]

  def string_forward(self, alpha, blank, lexical, semiring):
    check_num_weights(self, blank, lexical)
    return semiring.plus(semiring.times(alpha, blank[0]),
                         shift_down(semiring.times(alpha, lexical[0]), semiring))


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

  def forward(self, alpha, blank, lexical, context, semiring):
    """alignments.py:363-377: sum_i (L^i alpha) (x) blank[i]."""
    check_num_weights(self, blank, lexical)
    terminated = [semiring.times(alpha, blank[0])]
    last = alpha
    for i in range(self.max_expansions):
      last = context.forward_reduce(semiring.times(last[..., None], lexical[i]), semiring)
      terminated.append(semiring.times(last, blank[i + 1]))
    return semiring.sum(torch.stack(terminated), dim=0)

  def backward(self, alpha, blank, lexical, beta, log_z, context):
    """alignments.py:379-419: (beta_t, blank marginals [K+1], lexical
    marginals [K+1], the last all zero) of one frame, Log semiring."""
    check_num_weights(self, blank, lexical)
    K = self.max_expansions
    la = [alpha]
    last = alpha
    for i in range(K):
      last = context.forward_reduce(last[..., None] + lexical[i], semirings.Log)
      la.append(last)
    scale = beta - log_z[..., None]
    blank_marginals = [torch.exp(la[i] + blank[i] + scale) for i in range(K + 1)]
    next_beta = blank[K] + beta
    lexical_marginals = []
    for i in range(K):
      j = K - 1 - i
      lexical_beta = lexical[j] + context.backward_broadcast(next_beta)
      lexical_marginals.append(torch.exp(lexical_beta + (la[j] - log_z[..., None])[..., None]))
      next_beta = semirings.Log.plus(blank[j] + beta, semirings.Log.sum(lexical_beta, dim=-1))
    lexical_marginals.reverse()
    lexical_marginals.append(torch.zeros_like(lexical[K]))
    return next_beta, blank_marginals, lexical_marginals

  def string_forward(self, alpha, blank, lexical, semiring):
    """alignments.py:421-432 on the string acceptor (shift_down)."""
    check_num_weights(self, blank, lexical)
    terminated = [semiring.times(alpha, blank[0])]
    last = alpha
    for i in range(self.max_expansions):
      last = shift_down(semiring.times(last, lexical[i]), semiring)
      terminated.append(semiring.times(last, blank[i + 1]))
    return semiring.sum(torch.stack(terminated), dim=0)
