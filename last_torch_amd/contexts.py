"""Context dependencies (mirrors last_torch/contexts.py).

``FullNGram`` is the context DFA the tuned HIP kernels implement natively
(its index maps are evaluated in-kernel: DESIGN.md). ``NextStateTable`` (any
DFA as a transition table) runs on the general table kernels
(lt_table.hip), which take any context through ``next_state_table()``. The
tensor methods below are the per-frame plugin surface (contexts.py:43-146);
``RecognitionLattice`` does not call them on its hot path.
"""
import abc
import dataclasses

import torch

from last_torch_amd import semirings


def _in_arcs(table: torch.Tensor, device) -> torch.Tensor:
  """[C, D] flat arc indices p * V + (y - 1) into each destination state,
  ascending, padded with C * V (one past the last arc) where the in-degree
  is below the maximum D."""
  C, V = table.shape
  dst = table.reshape(-1).long().cpu()
  order = torch.argsort(dst * (C * V) + torch.arange(C * V), stable=True)
  counts = torch.bincount(dst, minlength=C)
  D = max(int(counts.max()), 1)
  idx = torch.full((C, D), C * V, dtype=torch.int64)
  start = torch.cumsum(counts, 0) - counts
  for q in range(C):
    idx[q, :counts[q]] = order[start[q]:start[q] + counts[q]]
  return idx.to(device)


def _cached(ctx, key, make):
  """A per-instance cache (the dataclasses are frozen): the in-arc index and
  the next-state table are built once per context and device, not on every
  per-frame forward_reduce call."""
  cache = ctx.__dict__.get('_cache')
  if cache is None:
    cache = {}
    object.__setattr__(ctx, '_cache', cache)
  if key not in cache:
    cache[key] = make()
  return cache[key]


def _reduce_by_table(weights: torch.Tensor, ctx, table_fn, semiring) -> torch.Tensor:
  """result[..., q] = (+)_{p -y-> q} weights[..., p, y-1]: one gather of
  every state's in-arcs (ascending, so the semiring's own tie rules see the
  arcs in the order a per-state loop would) and one semiring sum."""
  C, V = ctx.shape()
  idx = _cached(ctx, ('in_arcs', str(weights.device)), lambda: _in_arcs(table_fn(), weights.device))
  flat = weights.reshape(*weights.shape[:-2], C * V)
  pad = semiring.zeros((*flat.shape[:-1], 1), flat.dtype, flat.device)
  return semiring.sum(torch.cat([flat, pad], dim=-1)[..., idx], dim=-1)


class ContextDependency(abc.ABC):
  """A DFA over the lexical vocabulary whose states encode output history
  (contexts.py:25-146). All states are final; label 0 is epsilon."""

  @abc.abstractmethod
  def shape(self) -> tuple[int, int]:
    """(num_states, vocab_size)."""

  @abc.abstractmethod
  def start(self) -> int:
    """Start state id."""

  @abc.abstractmethod
  def next_state(self, state: torch.Tensor, label: torch.Tensor) -> torch.Tensor:
    """Transition; label 0 keeps the state (contexts.py:64-77)."""

  @abc.abstractmethod
  def forward_reduce(self, weights: torch.Tensor,
                     semiring: semirings.Semiring) -> torch.Tensor:
    """result[..., q] = (+)_{p -y-> q} weights[..., p, y-1] (contexts.py:79-94)."""

  @abc.abstractmethod
  def backward_broadcast(self, weights: torch.Tensor) -> torch.Tensor:
    """result[..., p, y-1] = weights[..., next(p, y)] (contexts.py:96-107)."""

  def walk_states(self, labels: torch.Tensor) -> torch.Tensor:
    """States after each label prefix: [..., U] -> [..., U+1]
    (contexts.py:109-146). states[..., 0] is the start state."""
    labels = torch.as_tensor(labels)
    states = [torch.full(labels.shape[:-1], self.start(), dtype=torch.int64,
                         device=labels.device)]
    for u in range(labels.shape[-1]):
      states.append(self.next_state(states[-1], labels[..., u].to(torch.int64)))
    return torch.stack(states, dim=-1)


@dataclasses.dataclass(frozen=True)
class FullNGram(ContextDependency):
  """Every n-gram of length 0..context_size is a state, numbered in
  lexicographic order; appending a label keeps the last context_size labels
  (contexts.py:150-263, GNAT section 4.1)."""

  vocab_size: int
  context_size: int

  def __post_init__(self):
    if self.vocab_size <= 0:
      raise ValueError(f'vocab_size should be > 0, but got vocab_size={self.vocab_size}')
    if self.context_size < 0:
      raise ValueError('context_size should be >= 0, but got '
                       f'context_size={self.context_size}')

  # sum_{i < k} V^i
  def _geo(self, k: int) -> int:
    return sum(self.vocab_size**i for i in range(max(k, 0)))

  def num_states(self) -> int:
    return self._geo(self.context_size + 1)

  def shape(self) -> tuple[int, int]:
    return self.num_states(), self.vocab_size

  def start(self) -> int:
    return 0

  def next_state(self, state, label):
    state = torch.as_tensor(state)
    label = torch.as_tensor(label)
    V, n = self.vocab_size, self.context_size
    ascending = self._geo(n)  # histories shorter than n
    grow = state * V + label
    if n == 0:
      full = torch.zeros_like(grow)
    else:
      full = torch.remainder(state - ascending, V**(n - 1)) * V + ascending + label - 1
    nxt = torch.where(state < ascending, grow, full)
    return torch.where(label == 0, state, nxt)

  def next_state_table(self) -> torch.Tensor:
    """[num_states, vocab_size]: table[p, y-1] = next_state(p, y) (contexts.py:258-263)."""
    C, V = self.shape()
    return self.next_state(torch.arange(C)[:, None], torch.arange(1, V + 1)[None, :])

  def _arc_index(self, device):
    # destination of arc (p, y) flattened as p*V + (y-1)
    return _cached(self, ('dst', str(device)),
                   lambda: self.next_state_table().reshape(-1).to(device))

  def forward_reduce(self, weights, semiring):
    if tuple(weights.shape[-2:]) != self.shape():
      raise ValueError(f'weights.shape[-2:] should be {self.shape()} but got'
                       f' {tuple(weights.shape[-2:])}')
    # every destination has the same in-degree except the start (none) and
    # the ascending states (one)
    return _reduce_by_table(weights, self, self.next_state_table, semiring)

  def backward_broadcast(self, weights):
    C, V = self.shape()
    if weights.shape[-1] != C:
      raise ValueError(f'weights.shape[-1] should be {C} but got {weights.shape[-1]}')
    dst = self._arc_index(weights.device)
    return weights[..., dst].reshape(*weights.shape[:-1], C, V)


@dataclasses.dataclass(frozen=True)
class NextStateTable(ContextDependency):
  """Context dependency described as a transition table (contexts.py:266-320).

  next_state_table: [num_states, vocab_size] int32; entry [p, y-1] is the
  state reached from p with label y.
  """
  next_state_table: torch.Tensor

  def __post_init__(self):
    t = self.next_state_table
    if t.ndim != 2:
      raise ValueError('next_state_table should have shape [num_states, vocab_size], but'
                       f'got shape {t.shape}')
    if 0 in t.size():
      raise ValueError('next_state_table should have a non-zero size, but '
                       f'got shape {t.shape}')
    if t.dtype != torch.int32:
      raise ValueError('next_state_table should be an int32 ndarray, but '
                       f'got dtype {t.dtype}')

  def shape(self) -> tuple[int, int]:
    return tuple(self.next_state_table.shape)

  def start(self) -> int:
    return 0

  def next_state(self, state, label):
    """contexts.py:291-298: epsilon (0) stays."""
    state = torch.as_tensor(state)
    label = torch.as_tensor(label)
    is_eps = label == 0
    zb = torch.where(is_eps, 0, label - 1)
    nxt = self.next_state_table[state.long(), zb.long()]
    return torch.where(is_eps, state.to(nxt.dtype), nxt)

  def forward_reduce(self, weights, semiring):
    """(+) of weights[..., p, y-1] over the arcs into each state. The
    reference scatters with 'sum' and then takes a max (contexts.py:300-313,
    SURVEY D8), which is no semiring sum; this is the intended reduction."""
    C, V = self.shape()
    if tuple(weights.shape[-2:]) != (C, V):
      raise ValueError(f'weights.shape[-2:] should be {(C, V)} but got {tuple(weights.shape[-2:])}')
    return _reduce_by_table(weights, self, lambda: self.next_state_table, semiring)

  def backward_broadcast(self, weights):
    """contexts.py:315-320: [..., C] -> [..., C, V] = weights[next_state]."""
    if weights.shape[-1] != self.shape()[0]:
      raise ValueError(f'weights.shape[-1] should be {self.shape()[0]} but '
                       f'got {weights.shape[-1]}')
    return weights[..., self.next_state_table.to(weights.device).long()]
