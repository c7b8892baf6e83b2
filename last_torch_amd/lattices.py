"""Recognition lattice (mirrors last_torch/lattices.py).

``RecognitionLattice`` keeps the reference's constructor and methods
(lattices.py:103-247, 250-799). Each method materialises the frame's arc
weights once through the ``WeightFn`` plugin as a contiguous
[B, T, C, V+1] tensor and hands it to the HIP kernels in
``liblt_lattice.so`` through ``_native`` (C ABI: include/lt_lattice.h):

  forward         -> lt_loss_grad (loss + dW, the design per shape);
                     lt_scale_grad in the backward; lt_loss_forward without grad
  _forward        -> lt_den_forward (Log, MaxTropical, Real);
                     autograd: lt_den_backward (Log) / lt_viterbi arcs (Max) /
                     lt_table_den_backward (Real)
  _forward_backward -> lt_den_forward + lt_den_backward
  _backward       -> lt_den_backward marginals, streamed to the callback
  _string_forward -> lt_num_forward; autograd: lt_loss_backward (Log) /
                     lt_table_num_backward (MaxTropical, Real)
  shortest_path   -> lt_viterbi

The device of the arc weights picks the implementation, as in the
reference: ROCm tensors run the HIP kernels (FrameDependent and
FrameLabelDependent alignments, FullNGram or any next-state table), CPU
tensors the C++ host twin (``liblt_lattice_cpu.so``, include/lt_lattice_cpu.h:
``forward`` and ``shortest_path`` of FullNGram x FrameDependent) or the
PyTorch restatement in ``cpu.py`` (every other method and lattice). There is no
fallback between the two: a ROCm tensor never runs on the CPU, and a missing
HIP library raises. Arbitrary batch dims are flattened (the reference's
``_string_forward`` supports only one, D13).
"""
from collections.abc import Callable, Sequence
from typing import Any, Generic, Optional, Protocol, TypeVar

import torch
import torch.nn as nn

from last_torch_amd import _native
from last_torch_amd import _native_cpu
from last_torch_amd import alignments
from last_torch_amd import cpu
from last_torch_amd import contexts
from last_torch_amd import semirings
from last_torch_amd import weight_fns

T = TypeVar('T')

_SEMIRING_IDS = {'Log': _native.SEMIRING_LOG, 'MaxTropical': _native.SEMIRING_MAX,
                 'Real': _native.SEMIRING_REAL}


def _semiring_id(semiring) -> int:
  name = getattr(semiring, 'name', None)
  if name not in _SEMIRING_IDS:
    raise NotImplementedError(f'lattice kernels support Log, MaxTropical and Real, got {semiring!r}')
  return _SEMIRING_IDS[name]


def _compute_device(W, *tensors) -> torch.device:
  """The arc weights' device (a ROCm device if any input is on one): ROCm
  -> HIP kernels, CPU -> cpu.py."""
  for t in (W, *tensors):
    if isinstance(t, torch.Tensor) and t.is_cuda:
      return t.device
  return torch.device('cpu')


def _lengths(x, batch_numel, device) -> torch.Tensor:
  return torch.as_tensor(x).reshape(batch_numel).to(device=device, dtype=torch.int32)


def _kernel_weights(W: torch.Tensor) -> torch.Tensor:
  if W.dtype not in (torch.float32, torch.bfloat16):
    W = W.float()
  W = W.contiguous()
  if W.data_ptr() % 16:
    W = W.clone()
  return W


class _LossFn(torch.autograd.Function):
  """loss = log_z - num (or -num), lattices.py:131-183, on the HIP kernels.

  With a gradient wanted, the forward is ONE lt_loss_grad call -- the loss
  and d(sum loss)/dW together, in whichever design lt_loss_grad_design picks
  for the shape (the chunked scan at the bench's B=64, the checkpointing
  pipe + marginal pass at B=256, the trigram's checkpointing pair): exactly
  what bench.py times, with the chunked path's per-frame certificate deciding
  which utterances the frame-serial kernels redo. The backward scales that
  dW by the incoming per-utterance gradient in place (lt_scale_grad: no work
  where it is 1); a second backward (retain_graph) recomputes it. Without a
  gradient only the loss is computed (lt_loss_forward)."""

  @staticmethod
  def forward(ctx, W, nf, labels, nl, V, n, local):
    ctx.cfg = (V, n, local)
    if not ctx.needs_input_grad[0]:
      return _native.loss_forward(W, nf, labels, nl, V, n, local, want_alpha=False)[0]
    loss, _, _, dW = _native.loss_grad(W, nf, labels, nl, V, n, local)
    ctx.dW = dW
    ctx.save_for_backward(W, nf, labels, nl)
    return loss

  @staticmethod
  def backward(ctx, g):
    V, n, local = ctx.cfg
    dW = ctx.dW
    ctx.dW = None
    if dW is None:  # a second backward through the same graph
      W, nf, labels, nl = ctx.saved_tensors
      dW = _native.loss_grad(W, nf, labels, nl, V, n, local)[3]
    _native.scale_grad(dW, g.float().contiguous(), V, n)
    return dW, None, None, None, None, None, None


class _CpuLossFn(torch.autograd.Function):
  """The same loss on host tensors through the C++ twin (lt_cpu_loss_grad,
  include/lt_lattice_cpu.h): FullNGram x FrameDependent, loss and
  d(sum loss)/dW in one call on the host thread pool; the backward scales
  it by the incoming gradient."""

  @staticmethod
  def forward(ctx, W, nf, labels, nl, V, n, local):
    want = ctx.needs_input_grad[0]
    loss, _, _, dW = _native_cpu.loss_grad(W, nf, labels, nl, V, n, local, with_grad=want)
    ctx.dW = dW
    if want:
      ctx.save_for_backward(W, nf, labels, nl)
    ctx.cfg = (V, n, local)
    return loss

  @staticmethod
  def backward(ctx, g):
    if torch.is_grad_enabled():
      # create_graph (higher-order gradients): the twin's dW is a constant,
      # so the differentiable backward goes through cpu.py's autograd
      W, nf, labels, nl = ctx.saved_tensors
      V, n, local = ctx.cfg
      loss = cpu.loss(W, nf.long(), labels, nl.long(),
                      contexts.FullNGram(vocab_size=V, context_size=n),
                      alignments.FrameDependent(), local)
      fin = torch.isfinite(loss)
      (dW,) = torch.autograd.grad(loss, W, torch.where(fin, g, torch.zeros_like(g)),
                                  create_graph=True)
      return dW, None, None, None, None, None, None
    dW = ctx.dW
    ctx.dW = None
    if dW is None:  # a second backward through the same graph
      W, nf, labels, nl = ctx.saved_tensors
      dW = _native_cpu.loss_grad(W, nf, labels, nl, *ctx.cfg)[3]
    return (dW * g.to(dW.dtype)[:, None, None, None], None, None, None, None, None, None)


class _TableLossFn(torch.autograd.Function):
  """loss for the general lattices (lt_table_loss_grad): any next-state
  table, FrameDependent or FrameLabelDependent(K). The gradient of
  sum(loss) comes with the forward; the backward scales it."""

  @staticmethod
  def forward(ctx, W, nf, labels, nl, graph, local):
    want = ctx.needs_input_grad[0]
    loss, _, _, dW = _native.table_loss_grad(graph, W, nf, labels, nl, local, want_grad=want)
    ctx.dW = dW
    return loss

  @staticmethod
  def backward(ctx, g):
    dW = ctx.dW
    if dW is None:
      raise RuntimeError('the lattice loss gradient was already consumed: backward through '
                         'RecognitionLattice.forward twice is not supported (call it again)')
    ctx.dW = None
    return (dW * g.to(dW.dtype)[:, None, None, None], None, None, None, None, None)


class _DenFn(torch.autograd.Function):
  """Denominator shortest distance; gradient = arc marginals (Log) or the
  best-path indicator (MaxTropical)."""

  @staticmethod
  def forward(ctx, W, nf, V, n, sid, graph=None):
    dist, alpha = _native.den_forward(W, nf, V, n, sid, want_alpha=True)
    ctx.save_for_backward(W, nf, dist, alpha)
    ctx.cfg = (V, n, sid)
    ctx.graph = graph
    ctx.mark_non_differentiable(alpha)
    return dist, alpha

  @staticmethod
  def backward(ctx, g, g_alpha):
    del g_alpha  # alpha_0..T-1 is a checkpoint, not differentiated
    W, nf, dist, alpha = ctx.saved_tensors
    V, n, sid = ctx.cfg
    g = g.float().contiguous()
    if sid == _native.SEMIRING_LOG:
      dW = _native.den_backward(W, nf, dist, alpha, g, V, n)
    elif sid == _native.SEMIRING_MAX:
      _, _, dW = _native.viterbi(W, nf, V, n, _native.LABELS_TRUE, grad=g, want_arcs=True)
    else:
      # Real (semirings.py:143-173, plain-arithmetic autograd in the
      # reference): d dist / dW = alpha * beta' from the general table
      # kernels on FullNGram.next_state_table() (the same state numbering)
      if ctx.graph is None:
        raise NotImplementedError('Real-semiring gradients need the lattice graph')
      dW = _native.table_den_backward(ctx.graph, W, nf, sid, dist, alpha, g)
    return dW, None, None, None, None, None


class _TableDenFn(torch.autograd.Function):
  """_forward's distance on the general table kernels (any next-state table,
  FrameDependent or FrameLabelDependent); gradient lt_table_den_backward: the
  arc marginals (Log), alpha * beta' (Real), the best path's arcs
  (MaxTropical)."""

  @staticmethod
  def forward(ctx, W, nf, graph, sid):
    dist, alpha = _native.table_forward(graph, W, nf, sid, want_alpha=True)
    ctx.save_for_backward(W, nf, dist, alpha)
    ctx.graph, ctx.sid = graph, sid
    ctx.mark_non_differentiable(alpha)
    return dist, alpha

  @staticmethod
  def backward(ctx, g, g_alpha):
    del g_alpha
    W, nf, dist, alpha = ctx.saved_tensors
    dW = _native.table_den_backward(ctx.graph, W, nf, ctx.sid, dist, alpha, g.float())
    return dW, None, None, None


class _TableNumFn(torch.autograd.Function):
  """_string_forward on the general table kernels; Log gradient = the string
  marginals (lt_table_loss_grad with local normalisation gives -d num / dW)."""

  @staticmethod
  def forward(ctx, W, nf, labels, nl, graph, sid):
    num = _native.table_num_forward(graph, W, nf, labels, nl, sid)
    ctx.save_for_backward(W, nf, labels, nl)
    ctx.graph, ctx.sid = graph, sid
    return num

  @staticmethod
  def backward(ctx, g):
    W, nf, labels, nl = ctx.saved_tensors
    if ctx.sid != _native.SEMIRING_LOG:
      # MaxTropical: the best string-aligned path's arcs; Real: alpha * beta'
      # (lt_table_num_backward, the reference's autograd through
      # semirings.py:143-173 / 354-401)
      _, dW = _native.table_num_backward(ctx.graph, W, nf, labels, nl, ctx.sid, g.float())
      return dW, None, None, None, None, None
    _, _, _, dW = _native.table_loss_grad(ctx.graph, W, nf, labels, nl, True)
    # an unreachable string has num = -inf and dW = 0 already
    return dW * (-g).to(dW.dtype)[:, None, None, None], None, None, None, None, None


class _NumFn(torch.autograd.Function):
  """Numerator (string) shortest distance; gradient = the string marginals
  (Log), the best string-aligned path's arcs (MaxTropical) or alpha * beta'
  (Real)."""

  @staticmethod
  def forward(ctx, W, nf, labels, nl, V, n, sid, graph=None):
    num, an = _native.num_forward(W, nf, labels, nl, V, n, sid,
                                  want_alpha=sid == _native.SEMIRING_LOG)
    ctx.save_for_backward(W, nf, labels, nl, num, an)
    ctx.cfg = (V, n, sid)
    ctx.graph = graph
    return num

  @staticmethod
  def backward(ctx, g):
    W, nf, labels, nl, num, an = ctx.saved_tensors
    V, n, sid = ctx.cfg
    if sid != _native.SEMIRING_LOG:
      # the general string-gradient kernel on FullNGram.next_state_table()
      # (the same state numbering): lt_table_num_backward
      if ctx.graph is None:
        raise NotImplementedError('MaxTropical / Real string gradients need the lattice graph')
      _, dW = _native.table_num_backward(ctx.graph, W, nf, labels, nl, sid, g.float())
      return dW, None, None, None, None, None, None, None
    # local-norm loss backward gives -grad * num marginals; feed -g.
    dW = _native.loss_backward(W, nf, labels, nl, None, num, None, an,
                               (-g).float().contiguous(), V, n, True)
    return dW, None, None, None, None, None, None, None


class RecognitionLattice(nn.Module, Generic[T]):
  """GNAT recognition lattice = context dependency x alignment lattice, with
  arc weights from a weight function (lattices.py:35-116)."""

  def __init__(self, context: contexts.ContextDependency,
               alignment: alignments.TimeSyncAlignmentLattice,
               weight_fn_cacher_factory: Callable[[contexts.ContextDependency],
                                                  weight_fns.WeightFnCacher[T]],
               weight_fn_factory: Callable[[contexts.ContextDependency], weight_fns.WeightFn[T]]):
    super().__init__()
    self.context = context
    self.alignment = alignment
    self.weight_fn_cacher_factory = weight_fn_cacher_factory
    self.weight_fn_factory = weight_fn_factory
    self.weight_fn_cacher = weight_fn_cacher_factory(context)
    self.weight_fn = weight_fn_factory(context)

  # -- helpers -------------------------------------------------------------
  def _table_path(self) -> bool:
    """False: FullNGram x FrameDependent, the tuned kernels (lt_lattice.hip,
    lt_pipe.hip). True: any other context (through its next-state table)
    with FrameDependent or FrameLabelDependent -- the general table kernels
    (lt_table.hip)."""
    if not isinstance(self.alignment, (alignments.FrameDependent,
                                       alignments.FrameLabelDependent)):
      raise NotImplementedError(f'lattice kernels implement FrameDependent and '
                                f'FrameLabelDependent alignments, got '
                                f'{type(self.alignment).__name__}')
    return not (isinstance(self.context, contexts.FullNGram) and
                isinstance(self.alignment, alignments.FrameDependent))

  def _graph(self, device) -> '_native.TableGraph':
    cache = self.__dict__.setdefault('_graphs', {})
    key = str(device)
    if key not in cache:
      if isinstance(self.context, contexts.NextStateTable):
        table = self.context.next_state_table
      elif hasattr(self.context, 'next_state_table'):
        table = self.context.next_state_table()
      else:
        raise NotImplementedError(f'{type(self.context).__name__} has no next-state table')
      K = (self.alignment.max_expansions
           if isinstance(self.alignment, alignments.FrameLabelDependent) else 0)
      cache[key] = _native.TableGraph(table, K, device)
    return cache[key]

  def _ngram(self) -> tuple[int, int]:
    if not isinstance(self.context, contexts.FullNGram):
      raise NotImplementedError(f'lattice kernels implement FullNGram contexts, got '
                                f'{type(self.context).__name__}')
    if not isinstance(self.alignment, alignments.FrameDependent):
      raise NotImplementedError(f'lattice kernels implement FrameDependent alignments, got '
                                f'{type(self.alignment).__name__}')
    return self.context.vocab_size, self.context.context_size

  def build_cache(self) -> T:
    """Builds the weight function cache (lattices.py:118-129)."""
    return self.weight_fn_cacher()

  def arc_weights(self, cache: T, frames: torch.Tensor) -> torch.Tensor:
    """All arc weights [batch..., T, C, V+1]: [..., 0] blank, [..., y] label y.

    Calls ``weight_fn(cache, frame)`` vectorised over time (the reference
    vmaps weight_fn the same way, lattices.py:308-313), falling back to one
    call per frame for weight functions vmap cannot trace.
    """
    tdim = frames.ndim - 2
    if getattr(self.weight_fn, 'time_batched', False):
      # the weight function takes any leading dims (JointWeightFn's
      # matrix-core producer: one launch for every frame)
      if hasattr(self.weight_fn, 'forward_joint'):
        return self.weight_fn.forward_joint(cache, frames)
      blank, lexical = self.weight_fn(cache, frames)
      return torch.cat([blank[..., None], lexical], dim=-1)

    def frame_weights(frame):
      blank, lexical = self.weight_fn(cache, frame)
      return torch.cat([blank[..., None], lexical], dim=-1)

    try:
      return torch.vmap(frame_weights, in_dims=tdim, out_dims=tdim, randomness='same')(frames)
    except Exception:  # pylint: disable=broad-except
      return torch.stack([frame_weights(frames[..., t, :]) for t in range(frames.shape[-2])],
                         dim=tdim)

  def _prepare(self, cache, frames, num_frames):
    batch_dims = tuple(num_frames.shape)
    if tuple(frames.shape[:-2]) != batch_dims:
      raise ValueError('frames and num_frames have different batch_dims: '
                       f'{tuple(frames.shape[:-2])} vs {batch_dims}')
    V, n = self._ngram() if not self._table_path() else (None, None)
    if cache is None:
      cache = self.weight_fn_cacher()
    W = self.arc_weights(cache, frames)
    B = 1
    for d in batch_dims:
      B *= d
    dev = _compute_device(W, frames, num_frames)
    W = W.to(dev).reshape(B, *W.shape[-3:])
    W = _kernel_weights(W) if dev.type == 'cuda' else W.float()
    nf = _lengths(num_frames, B, dev)
    if dev.type != 'cuda':
      nf = nf.long()
    return W, nf, batch_dims, B, V, n, cache

  @staticmethod
  def _home(x, like):
    return x.to(like.device) if isinstance(like, torch.Tensor) else x

  # -- public API ------------------------------------------------------------
  def forward(self, frames: torch.Tensor, num_frames: torch.Tensor, labels: torch.Tensor,
              num_labels: torch.Tensor, cache: Optional[T] = None) -> torch.Tensor:
    """Negative sequence log-probability -log P(labels | frames)
    (lattices.py:131-183); differentiable w.r.t. the weight function."""
    batch_dims = tuple(num_frames.shape)
    if tuple(frames.shape[:-2]) != batch_dims:
      raise ValueError('frames and num_frames have different batch_dims: '
                       f'{tuple(frames.shape[:-2])} vs {batch_dims}')
    if tuple(labels.shape[:-1]) != batch_dims:
      raise ValueError('labels and num_frames have different batch_dims: '
                       f'{tuple(labels.shape[:-1])} vs {batch_dims}')
    if tuple(num_labels.shape) != batch_dims:
      raise ValueError('num_labels and num_frames have different batch_dims: '
                       f'{tuple(num_labels.shape)} vs {batch_dims}')
    fused = self._fused_joint_loss(cache, frames, num_frames, labels, num_labels)
    if fused is not None:
      return self._home(fused.reshape(batch_dims), frames)
    W, nf, batch_dims, B, V, n, cache = self._prepare(cache, frames, num_frames)
    lab = torch.as_tensor(labels).reshape(B, -1).to(device=W.device, dtype=torch.int32)
    nl = _lengths(num_labels, B, W.device)
    local = isinstance(self.weight_fn, weight_fns.LocallyNormalizedWeightFn)
    if W.device.type == 'cpu':
      if not self._table_path() and _native_cpu.available():
        loss = _CpuLossFn.apply(W, nf, lab.contiguous(), nl, V, n, local)
      else:
        loss = cpu.loss(W, nf, lab, nl.long(), self.context, self.alignment, local)
    elif self._table_path():
      loss = _TableLossFn.apply(W, nf, lab.contiguous(), nl, self._graph(W.device), local)
    else:
      loss = _LossFn.apply(W, nf, lab.contiguous(), nl, V, n, local)
    return self._home(loss.reshape(batch_dims), frames)

  def _fused_joint_loss(self, cache, frames, num_frames, labels, num_labels):
    """The loss through the fused joint weight function + lattice kernels
    (JointWeightFn.fused_lattice_loss, lt_loss_joint_forward / _backward) when
    the weight function takes that path: FullNGram x FrameDependent on a ROCm
    device, one batch dim; else None."""
    fn = getattr(self.weight_fn, 'fused_lattice_loss', None)
    if fn is None or self._table_path() or frames.ndim != 3 or not frames.is_cuda:
      return None
    if cache is None:
      cache = self.weight_fn_cacher()
    dev = frames.device
    B = frames.shape[0]
    nf = _lengths(num_frames, B, dev)
    lab = torch.as_tensor(labels).reshape(B, -1).to(device=dev, dtype=torch.int32).contiguous()
    nl = _lengths(num_labels, B, dev)
    return fn(cache, frames, nf, lab, nl, self.context.vocab_size, self.context.context_size)

  def shortest_path(self, frames: torch.Tensor, num_frames: torch.Tensor,
                    cache: Optional[T] = None, label_convention: str = 'reference'):
    """Best alignment path (lattices.py:185-247).

    Returns (alignment_labels [batch..., T], num_alignment_labels, path_weights).
    ``label_convention='reference'`` (default) emits lexical label y as y-1
    exactly like the reference (lattices.py:242-244);
    ``'true'`` emits y. Unlike the reference, every utterance of a batch is
    decoded independently (D6).
    """
    conv = {'reference': _native.LABELS_REFERENCE, 'true': _native.LABELS_TRUE}[label_convention]
    W, nf, batch_dims, B, V, n, _ = self._prepare(cache, frames, num_frames)
    with torch.no_grad():
      if W.device.type == 'cpu' and not self._table_path() and _native_cpu.available():
        labels, weights, _ = _native_cpu.viterbi(W.detach(), nf, V, n, conv)
      elif W.device.type == 'cpu':
        labels, weights = cpu.viterbi(W, nf, self.context, self.alignment, label_convention)
      elif self._table_path():
        # A labels per frame: slot i = the (i+1)-th lexical label of the frame
        labels, weights = _native.table_viterbi(self._graph(W.device), W.detach(), nf, conv)
      else:
        labels, weights, _ = _native.viterbi(W.detach(), nf, V, n, conv)
    labels = self._home(labels.reshape(*batch_dims, -1), frames)
    num_alignment_labels = self.alignment.num_states() * num_frames
    return labels, num_alignment_labels, self._home(weights.reshape(batch_dims), frames)

  def _string_forward(self, cache: T, frames: torch.Tensor, num_frames: torch.Tensor,
                      labels: torch.Tensor, num_labels: torch.Tensor,
                      semiring: semirings.Semiring) -> torch.Tensor:
    """Shortest distance on the lattice intersected with the label string
    (lattices.py:250-377)."""
    batch_dims = tuple(num_frames.shape)
    if tuple(frames.shape[:-2]) != batch_dims:
      raise ValueError('frames and num_frames have different batch_dims: '
                       f'{tuple(frames.shape[:-2])} vs {batch_dims}')
    if tuple(labels.shape[:-1]) != batch_dims:
      raise ValueError('labels and num_frames have different batch_dims: '
                       f'{tuple(labels.shape[:-1])} vs {batch_dims}')
    if tuple(num_labels.shape) != batch_dims:
      raise ValueError('num_labels and num_frames have different batch_dims: '
                       f'{tuple(num_labels.shape)} vs {batch_dims}')
    sid = _semiring_id(semiring)
    W, nf, batch_dims, B, V, n, _ = self._prepare(cache, frames, num_frames)
    lab = torch.as_tensor(labels).reshape(B, -1).to(device=W.device, dtype=torch.int32)
    nl = _lengths(num_labels, B, W.device)
    if W.device.type == 'cpu':
      num = cpu.num_forward(W, nf, lab, nl.long(), self.context, self.alignment, semiring)
    elif self._table_path():
      num = _TableNumFn.apply(W, nf, lab.contiguous(), nl, self._graph(W.device), sid)
    else:
      # MaxTropical / Real gradients run on the general string-gradient kernel
      # over FullNGram.next_state_table(): its graph is built only when a
      # gradient can be asked for, and its LDS rule is checked here, before
      # the forward, rather than mid-backward
      graph = None
      if sid != _native.SEMIRING_LOG and torch.is_grad_enabled() and W.requires_grad:
        graph = self._graph(W.device)
        _native.table_num_backward_check(graph, W, lab, sid)
      num = _NumFn.apply(W, nf, lab.contiguous(), nl, V, n, sid, graph)
    return self._home(num.reshape(batch_dims), frames)

  def _forward(self, cache: T, frames: torch.Tensor, num_frames: torch.Tensor,
               semiring: semirings.Semiring,
               blank_mask: Optional[Sequence[torch.Tensor]] = None,
               lexical_mask: Optional[Sequence[torch.Tensor]] = None):
    """Shortest distance and alpha_0..T-1 (lattices.py:379-496).

    Masks are added to the arc weights (lattices.py:450-453), so their
    gradients are the arc marginals (Log) or the best-path indicator
    (MaxTropical) -- per utterance, without the batch aliasing of D6.
    """
    if semiring is semirings.LogLogExpectation and blank_mask is None and lexical_mask is None:
      return self._forward_expectation(cache, frames, num_frames)
    for name, mask in (('blank_mask', blank_mask), ('lexical_mask', lexical_mask)):
      if mask is not None and len(mask) != self.alignment.num_states():
        raise ValueError(f'The length of {name} should be equal to '
                         f'{self.alignment.num_states()} (the number of alignment states), '
                         f'but is {len(mask)}')
    sid = _semiring_id(semiring)
    batch_dims = tuple(num_frames.shape)
    if tuple(frames.shape[:-2]) != batch_dims:
      raise ValueError('frames and num_frames have different batch_dims: '
                       f'{tuple(frames.shape[:-2])} vs {batch_dims}')
    table = self._table_path()
    V, n = self._ngram() if not table else (None, None)
    if table:
      # alignment-state-invariant weights (lattices.py:444-447): one mask
      # for every alignment state
      for mask in (blank_mask, lexical_mask):
        if mask is not None and any(m is not mask[0] and not torch.equal(m, mask[0])
                                    for m in mask[1:]):
          raise NotImplementedError('per-alignment-state masks differ: the kernels use '
                                    'alignment-state-invariant weights')
    if cache is None:
      cache = self.weight_fn_cacher()
    W = self.arc_weights(cache, frames)
    if blank_mask is not None:
      W = torch.cat([W[..., :1] + blank_mask[0].to(W.device)[..., None], W[..., 1:]], dim=-1)
    if lexical_mask is not None:
      W = torch.cat([W[..., :1], W[..., 1:] + lexical_mask[0].to(W.device)], dim=-1)
    B = 1
    for d in batch_dims:
      B *= d
    dev = _compute_device(W, frames, num_frames)
    nf = _lengths(num_frames, B, dev)
    if dev.type == 'cpu':
      dist, alpha = cpu.den_forward(W.reshape(B, *W.shape[-3:]).float(), nf.long(), self.context,
                                    self.alignment, semiring)
      C = alpha.shape[-1]
      return (dist.reshape(batch_dims),
              alpha.reshape(*batch_dims, frames.shape[-2], C))
    Wk = _kernel_weights(W.to(dev).reshape(B, *W.shape[-3:]))
    if table:
      dist, alpha = _TableDenFn.apply(Wk, nf, self._graph(Wk.device), sid)
    else:
      graph = self._graph(Wk.device) if sid == _native.SEMIRING_REAL else None
      dist, alpha = _DenFn.apply(Wk, nf, V, n, sid, graph)
    C = alpha.shape[-1]
    return (self._home(dist.reshape(batch_dims), frames),
            self._home(alpha.reshape(*batch_dims, frames.shape[-2], C), frames))

  def _expectation(self, cache, frames, num_frames):
    """(log Z, sum over arcs of m(arc) * w(arc)) per utterance, m the arc
    marginals (the gradient of log Z: the den backward kernel on a ROCm
    device, autograd through cpu.py on the CPU). FullNGram x FrameDependent."""
    W, nf, batch_dims, B, V, n, _ = self._prepare(cache, frames, num_frames)
    with torch.enable_grad():
      Wd = W.detach().requires_grad_(True)
      if Wd.device.type == 'cpu':
        log_z, _ = cpu.den_forward(Wd, nf, self.context, self.alignment, semirings.Log)
      elif self._table_path():
        log_z, _ = _TableDenFn.apply(Wd, nf, self._graph(Wd.device), _native.SEMIRING_LOG)
      else:
        log_z, _ = _DenFn.apply(Wd, nf, V, n, _semiring_id(semirings.Log))
      (m,) = torch.autograd.grad(log_z.sum(), Wd)
    # arcs of zero weight (w = -inf) carry m = 0 and contribute nothing
    mw = torch.where(m > 0, m * Wd.detach().float(), torch.zeros_like(m)).sum(dim=(-3, -2, -1))
    return log_z.detach(), mw, batch_dims

  def _forward_expectation(self, cache, frames, num_frames):
    """_forward under semirings.LogLogExpectation (semirings.py:405-484).
    The lattice's arc weights are single tensors, so every arc carries the
    expectation pair weighted(w, -w): the value -w, the convention of the
    reference's entropy test (tests/semirings_test.py:305-312). The shortest
    distance is then (log Z, log Z + log E_p[-w_path]) by the forward-backward
    identity (the x component sums Z m(arc) v(arc) over arcs). Returns
    ((log_z, log_sum), None): there is no per-frame alpha of a pair."""
    log_z, mw, batch_dims = self._expectation(cache, frames, num_frames)
    log_sum = log_z + torch.log(-mw)
    return ((self._home(log_z.reshape(batch_dims), frames),
             self._home(log_sum.reshape(batch_dims), frames)), None)

  def entropy(self, frames: torch.Tensor, num_frames: torch.Tensor,
              cache: Optional[T] = None) -> torch.Tensor:
    """Entropy (nats) of the alignment-path distribution p(path) = exp(w_path)
    / Z of every utterance: H = log Z - E_p[w_path], the lattice entropy the
    LogLogExpectation semiring computes (tests/semirings_test.py:305-312:
    entropy = log_z + exp(log_sum - log_z)), here for weights of any sign.
    Values only (no gradient)."""
    log_z, mw, batch_dims = self._expectation(cache, frames, num_frames)
    return self._home((log_z - mw).reshape(batch_dims), frames)

  def _forward_backward(self, cache: T, frames: torch.Tensor, num_frames: torch.Tensor):
    """log_z with gradients from the backward algorithm (lattices.py:498-642;
    the reference's backward raises, D3). Returns (log_z, alpha_0..T-1)."""
    return self._forward(cache, frames, num_frames, semirings.Log)

  class BackwardStepCallback(Protocol):
    """Callback of the backward algorithm loop (lattices.py:644-684)."""

    def __call__(self, weight_vjp_fn, carry, blank_marginal: torch.Tensor,
                 lexical_marginals: torch.Tensor) -> tuple[Any, Any]:
      raise NotImplementedError

  def _backward(self, cache: T, frames: torch.Tensor, num_frames: torch.Tensor,
                log_z: torch.Tensor, alpha_0_to_T_minus_1: torch.Tensor,
                init_callback_carry: Any, callback: BackwardStepCallback):
    """Arc marginals by the backward algorithm (lattices.py:686-799).

    The marginals of every frame come from one ``lt_den_backward`` launch;
    the callback then runs frame by frame from T-1 down to 0 (the reference
    iterates in the wrong direction, D4) with ``weight_vjp_fn`` for that
    frame. Outputs are stacked in time order along the frame axis.
    """
    batch_dims = tuple(num_frames.shape)
    if tuple(frames.shape[:-2]) != batch_dims:
      raise ValueError('frames and num_frames have different batch_dims: '
                       f'{tuple(frames.shape[:-2])} vs {batch_dims}')
    if tuple(log_z.shape) != batch_dims:
      raise ValueError('log_z and num_frames have different batch_dims: '
                       f'{tuple(log_z.shape)} vs {batch_dims}')
    if tuple(alpha_0_to_T_minus_1.shape[:-2]) != batch_dims:
      raise ValueError('alpha_0_to_T_minus_1 and num_frames have different '
                       f'batch_dims: {tuple(alpha_0_to_T_minus_1.shape[:-2])} vs {batch_dims}')
    with torch.no_grad():
      W = self.arc_weights(cache, frames)
      B = 1
      for d in batch_dims:
        B *= d
      dev = _compute_device(W, frames, num_frames)
      nf = _lengths(num_frames, B, dev)
    if dev.type == 'cpu':
      # arc marginals = d log_z / dW (the reference's backward algorithm
      # computes the same quantities frame by frame)
      with torch.enable_grad():
        Wd = W.detach().reshape(B, *W.shape[-3:]).float().requires_grad_(True)
        dist, _ = cpu.den_forward(Wd, nf.long(), self.context, self.alignment, semirings.Log)
        (marg,) = torch.autograd.grad(dist.sum(), Wd)
      marg = marg.reshape(*batch_dims, *marg.shape[1:])
    else:
      with torch.no_grad():
        Wk = _kernel_weights(W.to(dev).reshape(B, *W.shape[-3:]))
        lz = log_z.detach().reshape(B).to(dev, torch.float32).contiguous()
        al = alpha_0_to_T_minus_1.detach().reshape(B, Wk.shape[1], -1).to(dev, torch.float32)
        if self._table_path():
          # any next-state table, FrameDependent or FrameLabelDependent
          # (self.alignment.backward, lattices.py:764)
          marg = _native.table_den_backward(self._graph(dev), Wk, nf, _native.SEMIRING_LOG, lz,
                                            al.contiguous()).float()
        else:
          V, n = self._ngram()
          marg = _native.den_backward(Wk, nf, lz, al.contiguous(), None, V, n).float()
        marg = self._home(marg.reshape(*batch_dims, *marg.shape[1:]), frames)
    tdim = len(batch_dims)
    carry, outs = init_callback_carry, []
    # weight_vjp_fn(cotangent) -> (d cache, d frame); a cache that is not a
    # tree of tensors (NullCacher: None) is held fixed and gets None
    leaves = torch.utils._pytree.tree_leaves(cache)
    cache_is_tensor = cache is not None and all(isinstance(x, torch.Tensor) for x in leaves)

    def frame_vjp(frame):
      if cache_is_tensor:
        return torch.func.vjp(lambda c, f: self.weight_fn(c, f), cache, frame)[1]
      fn = torch.func.vjp(lambda f: self.weight_fn(cache, f), frame)[1]
      return lambda ct: (None, *fn(ct))

    for t in reversed(range(frames.shape[-2])):
      frame = frames.select(tdim, t)
      vjp_fn = frame_vjp(frame)
      m = marg.select(tdim, t)
      carry, out = callback(weight_vjp_fn=vjp_fn, carry=carry, blank_marginal=m[..., 0],
                            lexical_marginals=m[..., 1:])
      outs.append(out)
    outs.reverse()
    stacked = torch.utils._pytree.tree_map(lambda *xs: torch.stack(xs, dim=tdim), *outs) \
        if outs else None
    return carry, stacked
