"""Weight functions (mirrors last_torch/weight_fns.py).

A ``WeightFn`` produces the arc weights of one frame; it is the producer side
of the lattice boundary (weight_fns.py:42-83). ``RecognitionLattice``
materialises them once per call as one contiguous [B, T, C, V+1] tensor that
the HIP kernels stream from HBM.

Differences from the reference, all bug fixes:
  * ``JointWeightFn`` owns its projections (created once, trainable,
    deterministic) instead of building fresh random ``nn.Linear`` layers on
    every call.
  * ``SharedEmbCacher`` returns the embedding table tensor, not the module.
  * ``SharedRNNCacher`` creates its default ``LSTMCell`` once.

``JointWeightFn`` on a ROCm device (all context states at once) runs the
``lt_joint_weights`` matrix-core kernel (lt_producer.hip): the [..., C, H]
hidden tensor is formed tile by tile in registers instead of in HBM; the
tanh values and the output projection enter the products as bf16, the sums
are fp32. Its backward (``lt_joint_weights_backward``) recomputes the hidden
tiles in fp32 and forms every gradient on the matrix cores with split-bf16
products; shapes it cannot take fall back to PyTorch in frame chunks.
"""
import abc
from typing import Callable, Generic, Optional, TypeVar

import einops
import torch
from torch import nn
from torch.nn import functional as F

T = TypeVar('T')


class WeightFn(nn.Module, Generic[T], abc.ABC):
  """Computes (blank, lexical) arc weights for a frame (weight_fns.py:42-83).

  state=None: blank [batch..., C], lexical [batch..., C, V].
  state given: blank [batch...], lexical [batch..., V] for that state.
  """

  @abc.abstractmethod
  def forward(self, cache: T, frame: torch.Tensor,
              state: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
    raise NotImplementedError


class WeightFnCacher(nn.Module, Generic[T], abc.ABC):
  """Builds the static data a WeightFn reuses across frames (weight_fns.py:86-96)."""

  @abc.abstractmethod
  def forward(self) -> T:
    """Builds the cached data."""


def hat_normalize(blank: torch.Tensor, lexical: torch.Tensor):
  """HAT local normalisation: sigmoid(blank) is P(blank), the lexical weights
  are a log-softmax scaled by P(not blank) (weight_fns.py:99-117)."""
  z = F.softplus(blank)  # log(1 + exp(blank)); log P(not blank) = -z
  return blank - z, F.log_softmax(lexical, dim=-1) - z[..., None]


def log_softmax_normalize(blank: torch.Tensor, lexical: torch.Tensor):
  """Joint log-softmax over [blank, lexical] (weight_fns.py:120-136)."""
  z = torch.logsumexp(torch.cat([blank[..., None], lexical], dim=-1), dim=-1)
  return blank - z, lexical - z[..., None]


class LocallyNormalizedWeightFn(WeightFn[T]):
  """Wraps a WeightFn with a local normaliser. ``RecognitionLattice`` skips
  the denominator for this type (lattices.py:178-179)."""

  def __init__(self, weight_fn: WeightFn[T],
               normalize: Callable[[torch.Tensor, torch.Tensor],
                                   tuple[torch.Tensor, torch.Tensor]] = hat_normalize):
    super().__init__()
    self.weight_fn = weight_fn
    self.normalize = normalize

  @property
  def time_batched(self):
    return getattr(self.weight_fn, 'time_batched', False)

  def forward(self, cache, frame, state=None):
    return self.normalize(*self.weight_fn(cache, frame, state))


class _JointWeightsFn(torch.autograd.Function):
  """W[..., c, :] = bias + tanh(pc[c] + pf[...]) @ wo^T via lt_joint_weights;
  the backward is lt_joint_weights_backward where its LDS holds d_ctx_proj,
  else PyTorch recomputing tanh in fp32, `chunk` frame rows at a time."""

  # forward / setup_context split: torch.func transforms (the per-frame
  # weight_vjp_fn of RecognitionLattice._backward) accept only this form
  @staticmethod
  def forward(pc, pf, wo, bias, chunk, precision):
    from last_torch_amd import _native
    return _native.joint_weights(pc, pf, wo, bias, precision=precision)

  @staticmethod
  def setup_context(ctx, inputs, output):
    pc, pf, wo, _, chunk, _ = inputs
    ctx.save_for_backward(pc, pf, wo)
    ctx.chunk = chunk

  @staticmethod
  def backward(ctx, gW):
    from last_torch_amd import _native
    pc, pf, wo = ctx.saved_tensors
    C, H = pc.shape
    R = wo.shape[0]
    if _native.joint_weights_backward_supported(C, H, R, pf.numel() // H):
      dpc, dpf, dwo, dbias = _native.joint_weights_backward(pc, pf, wo, gW)
      return dpc, dpf, dwo, dbias, None, None
    pf2 = pf.reshape(-1, H)
    g2 = gW.reshape(-1, C, R).float()
    dpc = torch.zeros_like(pc)
    dpf = torch.empty_like(pf2)
    dwo = torch.zeros_like(wo)
    for s in range(0, pf2.shape[0], ctx.chunk):
      hid = torch.tanh(pc[None] + pf2[s:s + ctx.chunk, None, :])  # [n, C, H]
      g = g2[s:s + ctx.chunk]                                     # [n, C, R]
      dwo += torch.einsum('ncr,nch->rh', g, hid)
      dh = torch.matmul(g, wo) * (1.0 - hid * hid)
      dpc += dh.sum(0)
      dpf[s:s + ctx.chunk] = dh.sum(1)
    return dpc, dpf.reshape(pf.shape), dwo, g2.sum((0, 1)), None, None


class _JointLossFn(torch.autograd.Function):
  """RecognitionLattice.forward's loss with JointWeightFn's arc weights fused
  into the lattice kernels (lt_loss_joint_forward / _backward, lt_joint.hip):
  W and d loss / dW are never materialised; the backward gives the
  projections' and the output layer's gradients directly."""

  @staticmethod
  def forward(ctx, pc, pf, wo, bias, nf, labels, nl, precision):
    from last_torch_amd import _native
    loss, _, _, state = _native.joint_loss_forward(pc, pf, wo, bias, nf, labels, nl, precision)
    ctx.save_for_backward(pc, pf, wo, bias, nf, labels, state)
    ctx.precision = precision
    return loss

  @staticmethod
  def backward(ctx, g):
    from last_torch_amd import _native
    pc, pf, wo, bias, nf, labels, state = ctx.saved_tensors
    dpc, dpf, dwo, dbias = _native.joint_loss_backward(pc, pf, wo, bias, nf, labels, state,
                                                       grad=g, precision=ctx.precision)
    return dpc, dpf.reshape(pf.shape), dwo, dbias, None, None, None, None


class JointWeightFn(WeightFn[torch.Tensor]):
  """tanh(P_c ctx_emb[c] + P_f frame) -> (blank, V lexical) logits: the
  shared-emb / shared-rnn weight function (weight_fns.py:174-227).

  ``fused`` (default): on a ROCm device, with all context states at once,
  the logits come from the lt_joint_weights matrix-core kernel (fp32 sums;
  hidden_size a multiple of 16, vocab_size < 64). ``precision`` 'fp32'
  (default, faithful to the reference's fp32 layers): split-bf16 products,
  about 16 mantissa bits each, as the backward; 'bf16': one bf16 product
  (faster, ~2^-8 relative per product).

  ``lattice_fusion``: whether ``RecognitionLattice.forward`` hands this
  weight function's projections to the fused joint lattice loss
  (lt_loss_grad_joint: W and dW never in HBM) instead of materialising W.
  'auto' takes it where it measured faster than the separate launches
  (``fused_lattice_preferred``), 'on' whenever the shape allows it, 'off'
  never."""

  def __init__(self, vocab_size: int, hidden_size: int, device=None, fused: bool = True,
               backward_chunk: int = 16384, precision: str = 'fp32',
               lattice_fusion: str = 'auto'):
    super().__init__()
    if precision not in ('fp32', 'bf16'):
      raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
    if lattice_fusion not in ('auto', 'on', 'off'):
      raise ValueError(f"lattice_fusion must be 'auto', 'on' or 'off', got {lattice_fusion!r}")
    self.lattice_fusion = lattice_fusion
    self.vocab_size = vocab_size
    self.hidden_size = hidden_size
    self.fused = fused
    self.precision = precision
    self.backward_chunk = backward_chunk
    self.context_projection = nn.LazyLinear(hidden_size, bias=False, device=device)
    self.frame_projection = nn.LazyLinear(hidden_size, bias=False, device=device)
    self.to_blank = nn.Linear(hidden_size, 1, device=device)
    self.to_vocab = nn.Linear(hidden_size, vocab_size, device=device)

  # forward() takes frames with any leading dims (RecognitionLattice calls it
  # once for [batch..., T, F] instead of vmapping over T)
  time_batched = True

  def _use_kernel(self, frame):
    return (self.fused and frame.is_cuda and frame.dtype == torch.float32 and
            self.hidden_size % 16 == 0 and self.vocab_size + 1 <= 64)

  def forward_joint(self, cache, frame):
    """All context states' arc weights as ONE tensor [..., C, V+1] (blank at
    [..., 0]), the layout RecognitionLattice hands to the lattice kernels:
    with the matrix-core producer no split / concatenate round trip."""
    if self._use_kernel(frame):
      pc = self.context_projection(cache)
      pf = self.frame_projection(frame)
      wo = torch.cat([self.to_blank.weight, self.to_vocab.weight], 0)
      bias = torch.cat([self.to_blank.bias, self.to_vocab.bias], 0)
      return _JointWeightsFn.apply(pc, pf, wo, bias, self.backward_chunk, self.precision)
    blank, lexical = self.forward(cache, frame)
    return torch.cat([blank[..., None], lexical], dim=-1)

  def fused_lattice_loss(self, cache, frames, num_frames, labels, num_labels, vocab_size,
                         context_size):
    """The lattice loss with the arc weights formed inside the lattice kernels
    (lt_loss_joint_forward / _backward), or None where this weight function
    does not take that path (lattice_fusion, device, shape)."""
    from last_torch_amd import _native
    if self.lattice_fusion == 'off' or not self._use_kernel(frames) or frames.ndim != 3:
      return None
    B, T = frames.shape[:2]
    U = labels.shape[-1]
    if not _native.joint_loss_supported(B, T, U, vocab_size, context_size, self.hidden_size,
                                        self.precision):
      return None
    if self.lattice_fusion == 'auto' and not fused_lattice_preferred(B, T, U, self.hidden_size):
      return None
    pc = self.context_projection(cache)
    pf = self.frame_projection(frames)
    wo = torch.cat([self.to_blank.weight, self.to_vocab.weight], 0)
    bias = torch.cat([self.to_blank.bias, self.to_vocab.bias], 0)
    return _JointLossFn.apply(pc, pf, wo, bias, num_frames, labels, num_labels, self.precision)

  def forward(self, cache, frame, state=None):
    ctx = cache
    if state is None and self._use_kernel(frame):
      W = self.forward_joint(cache, frame)
      return W[..., 0], W[..., 1:]
    if state is None:
      joint = self.context_projection(ctx) + self.frame_projection(frame)[..., None, :]
    else:
      ctx = torch.index_select(ctx, 0, state.reshape(-1).long()).reshape(
          *state.shape, ctx.shape[-1])
      joint = self.context_projection(ctx) + self.frame_projection(frame)
    joint = torch.tanh(joint)
    return self.to_blank(joint)[..., 0], self.to_vocab(joint)


def fused_lattice_preferred(batch, frames, labels, hidden):
  """Where the fused joint lattice loss (lt_loss_grad_joint) measured faster
  than the separate launches (lt_joint_weights -> lt_loss_grad ->
  lt_joint_weights_backward) on MI355X: profiles/r05_joint_step.jsonl. At
  the bench shape (T = 1000, U = 100, V = 32, B = 64 and 256, H = 32..128)
  it measured slower everywhere -- the producer is issue-bound, so forming W
  inside the latency-bound recursions and again in the marginal pass costs
  more than W's HBM round trip saves -- so 'auto' keeps the
  separate launches."""
  del batch, frames, labels, hidden
  return False


class SharedEmbCacher(WeightFnCacher[torch.Tensor]):
  """An independent trainable [num_context_states, embedding_size] table
  (weight_fns.py:230-242)."""

  def __init__(self, num_context_states: int, embedding_size: int, device=None):
    super().__init__()
    self.num_context_states = num_context_states
    self.embedding_size = embedding_size
    self.embedding = nn.Embedding(num_context_states, embedding_size, device=device)

  def forward(self):
    return self.embedding.weight


class SharedRNNCacher(WeightFnCacher[torch.Tensor]):
  """Context embeddings from an RNN run over every n-gram history, in
  FullNGram state order (weight_fns.py:245-294). LSTM cells contribute their
  cell state, other cells their output."""

  def __init__(self, vocab_size: int, context_size: int, rnn_size: int,
               rnn_embedding_size: int, rnn_cell: Optional[nn.RNNCellBase] = None):
    super().__init__()
    self.vocab_size = vocab_size
    self.context_size = context_size
    self.rnn_size = rnn_size
    self.rnn_embedding_size = rnn_embedding_size
    self.embedding = nn.Embedding(vocab_size + 1, rnn_embedding_size)
    self.rnn_cell = rnn_cell if rnn_cell is not None else nn.LSTMCell(
        rnn_embedding_size, rnn_size)

  def _step(self, inputs, state):
    out = self.rnn_cell(inputs, state) if state is not None else self.rnn_cell(inputs)
    if isinstance(out, tuple):  # LSTMCell: (h, c); the embedding is c
      return out, out[1]
    return out, out

  def forward(self):
    dev = self.embedding.weight.device
    state, emb = self._step(self.embedding(torch.zeros([1], dtype=torch.long, device=dev)), None)
    parts = [emb]
    labels = self.embedding(torch.arange(1, self.vocab_size + 1, device=dev))
    inputs = None
    for order in range(self.context_size):
      # histories of length order+1: prefix state (n) x appended label (v)
      inputs = labels if order == 0 else einops.repeat(inputs, 'n ... -> (v n) ...',
                                                       v=self.vocab_size)
      tile = lambda x: einops.repeat(x, 'n ... -> (n v) ...', v=self.vocab_size)
      state = tuple(tile(s) for s in state) if isinstance(state, tuple) else tile(state)
      state, emb = self._step(inputs, state)
      parts.append(emb)
    return torch.cat(parts, dim=0)


class NullCacher(WeightFnCacher[type(None)]):
  """Returns None; pairs with TableWeightFn (weight_fns.py:297-304)."""

  def forward(self):
    return None


class TableWeightFn(WeightFn[type(None)]):
  """Looks arc weights up in a fixed table (weight_fns.py:307-342).

  table: [batch..., input_vocab, C, 1+V]; frame[..., 0] is the integer row.
  Weights are returned in float32 like the reference (weight_fns.py:333).
  """

  def __init__(self, table: torch.Tensor):
    super().__init__()
    self.table = table

  def forward(self, cache, frame, state=None):
    del cache
    *batch, x, c, _ = self.table.shape
    if tuple(frame.shape[:-1]) != tuple(batch):
      raise ValueError(f'frame should have batch_dims={tuple(batch)} but '
                       f'got ({tuple(frame.shape[:-1])})')
    table = self.table.to(frame.device).float()
    row = frame[..., 0].long()[..., None, None, None]
    w = torch.take_along_dim(table, row.expand(*batch, 1, c, table.shape[-1]), dim=-3)[..., 0, :, :]
    if state is not None:
      st = torch.broadcast_to(torch.as_tensor(state, device=w.device), tuple(batch)).long()
      w = torch.take_along_dim(w, st[..., None, None].expand(*batch, 1, w.shape[-1]),
                               dim=-2)[..., 0, :]
    return w[..., 0], w[..., 1:]
