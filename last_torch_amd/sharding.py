"""Utterance sharding for data-parallel lattice losses.

Utterances are independent lattices, so the path shards with no data-path
collective: each rank runs the HIP kernels on its own utterances, and dW
stays utterance-local. The only exchange is one all-reduce(SUM) per step of
a flat fp32 bucket [sum of losses || weight-fn parameter grads], which on
ROCm is RCCL over xGMI (torch.distributed backend "nccl") and gloo on CPU.

Partitioning is longest-processing-time (LPT) with equal utterance counts:
utterances are visited longest first and each goes to the least-loaded rank
that still has room, so every rank gets B/N (+-1) utterances and the
frame totals are balanced against length stragglers.
"""
from typing import Iterable, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard_utterances(num_frames: Sequence[int], world_size: int) -> list[np.ndarray]:
  """Returns, per rank, the ascending utterance indices it owns."""
  nf = np.asarray(num_frames, dtype=np.int64).reshape(-1)
  if world_size < 1:
    raise ValueError(f'world_size must be >= 1, got {world_size}')
  B = nf.shape[0]
  cap = [B // world_size + (1 if r < B % world_size else 0) for r in range(world_size)]
  load = np.zeros(world_size, np.int64)
  owned: list[list[int]] = [[] for _ in range(world_size)]
  for i in np.argsort(-nf, kind='stable'):
    open_ranks = [r for r in range(world_size) if len(owned[r]) < cap[r]]
    r = min(open_ranks, key=lambda k: (load[k], len(owned[k]), k))
    owned[r].append(int(i))
    load[r] += nf[i]
  return [np.asarray(sorted(o), dtype=np.int64) for o in owned]


def local_shard(num_frames, rank: int, world_size: int) -> np.ndarray:
  """Indices of the utterances `rank` owns (see shard_utterances)."""
  nf = num_frames.detach().cpu().numpy() if torch.is_tensor(num_frames) else num_frames
  return shard_utterances(nf, world_size)[rank]


def all_reduce_step(loss: torch.Tensor, params: Iterable[torch.nn.Parameter] = (),
                    group: Optional[dist.ProcessGroup] = None,
                    skip_unused: bool = False) -> torch.Tensor:
  """The step's single collective: all-reduce(SUM) of [loss.sum() || grads].

  Parameter gradients are summed in place (callers that want the mean
  divide by the global utterance count). Returns the global loss sum.
  Without an initialised process group this is the identity.

  A parameter without a gradient on this rank (unused here, or an empty
  shard) contributes zeros, so every rank all-reduces the same layout. The
  same all-reduce carries one "used" count per parameter: a parameter some
  rank produced a gradient for gets the summed gradient on every rank (a
  fresh .grad where it had none), so the replicas' optimizer updates stay
  identical; a parameter no rank used keeps .grad None everywhere, so
  optimizers with weight decay or momentum skip it as they would without
  the collective. ``skip_unused=True`` leaves a None .grad None on this rank
  even when other ranks used the parameter (the replicas may then drift
  apart; only for callers that re-synchronise parameters themselves)."""
  total = loss.detach().sum().reshape(1).to(torch.float32)
  if not (dist.is_available() and dist.is_initialized()):
    return total[0]
  params = list(params)
  parts = [total]
  for p in params:
    parts.append(torch.zeros([p.numel()], dtype=torch.float32, device=total.device)
                 if p.grad is None else p.grad.reshape(-1).to(torch.float32))
  parts.append(torch.tensor([0.0 if p.grad is None else 1.0 for p in params],
                            dtype=torch.float32, device=total.device))
  flat = torch.cat(parts)
  dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
  used = flat[flat.numel() - len(params):].tolist()
  off = 1
  for p, u in zip(params, used):
    k = p.numel()
    red = flat[off:off + k].view(p.shape)
    if p.grad is not None:
      p.grad.copy_(red.to(p.grad.dtype))
    elif u > 0 and not skip_unused:
      p.grad = red.to(p.dtype).clone()
    off += k
  return flat[0]


class GradBucket:
  """The step's collective with no packing: one flat fp32 buffer [loss sum ||
  grads], the parameters' .grad set to views of it (as DDP's buckets do), so
  a step is the loss sum written into slot 0 and ONE all-reduce -- no
  concatenate before it and no copy back after it. Parameters must be fp32.
  Backward accumulates into the views in place; ``zero_grad()`` (instead of
  the optimizer's, whose default set_to_none would detach .grad from the
  bucket) clears them for the next step, and ``all_reduce_step`` re-binds any
  .grad that was replaced or dropped (copying a replaced gradient's values
  into the bucket first), so the reduced buffer is always the one the
  optimizer steps on."""

  def __init__(self, params: Iterable[torch.nn.Parameter], device=None):
    self.params = list(params)
    n = sum(p.numel() for p in self.params)
    dev = device if device is not None else (self.params[0].device if self.params else 'cpu')
    self.flat = torch.zeros([1 + n], dtype=torch.float32, device=dev)
    self.views = []
    self.calls = 0  # all-reduces issued (one per step)
    off = 1
    for p in self.params:
      if p.dtype != torch.float32:
        raise TypeError(f'GradBucket: parameters must be float32, got {p.dtype}')
      k = p.numel()
      v = self.flat[off:off + k].view_as(p)
      self.views.append(v)
      p.grad = v
      off += k

  def zero_grad(self) -> None:
    """Zeros every gradient (and the loss slot) in place, keeping the views."""
    self.flat.zero_()
    self._bind()

  def _bind(self) -> None:
    for p, v in zip(self.params, self.views):
      g = p.grad
      if g is None:
        v.zero_()
      elif g.data_ptr() != v.data_ptr():
        # optimizer.zero_grad(set_to_none) then backward made a fresh tensor
        v.copy_(g)
      else:
        continue
      p.grad = v

  def all_reduce_step(self, loss: torch.Tensor, group: Optional[dist.ProcessGroup] = None
                      ) -> torch.Tensor:
    """all-reduce(SUM) of [loss.sum() || grads] in place; returns the global
    loss sum (the identity without an initialised process group)."""
    self._bind()
    torch.sum(loss.detach().reshape(-1).to(torch.float32), dim=0, keepdim=True,
              out=self.flat[:1])
    if dist.is_available() and dist.is_initialized():
      dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
      self.calls += 1
    return self.flat[0]
