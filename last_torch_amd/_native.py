"""ctypes binding of the HIP lattice library (liblt_lattice.so, include/lt_lattice.h).

Every call is issued on ``torch.cuda.current_stream()`` and works on device
tensors owned by the PyTorch caching allocator; the library never allocates.
There is no CPU fallback: if the library is missing or no ROCm device is
present, calls raise.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# LT_LIB_PATH: a diagnostic build of the same library (make diag); never set
# in normal use
LIB_PATH = os.environ.get('LT_LIB_PATH') or os.path.join(_HERE, 'liblt_lattice.so')

LT_DTYPE_F32, LT_DTYPE_BF16 = 0, 1
SEMIRING_LOG, SEMIRING_MAX, SEMIRING_REAL = 0, 1, 2
LABELS_TRUE, LABELS_REFERENCE = 0, 1

_lock = threading.Lock()
_lib = None


class LatticeLibraryError(RuntimeError):
  """Raised when the HIP library is unavailable or a call fails."""


class Problem(ctypes.Structure):
  _fields_ = [('batch', ctypes.c_int32), ('max_frames', ctypes.c_int32),
              ('vocab_size', ctypes.c_int32), ('context_size', ctypes.c_int32),
              ('max_labels', ctypes.c_int32), ('weight_dtype', ctypes.c_int32)]


class Graph(ctypes.Structure):
  """lt_graph: a next-state table and its in-arc CSR (device pointers)."""
  _fields_ = [('num_states', ctypes.c_int32), ('vocab_size', ctypes.c_int32),
              ('expansions', ctypes.c_int32), ('next_state', ctypes.c_void_p),
              ('in_offsets', ctypes.c_void_p), ('in_arcs', ctypes.c_void_p)]


class TableProblem(ctypes.Structure):
  _fields_ = [('batch', ctypes.c_int32), ('max_frames', ctypes.c_int32),
              ('max_labels', ctypes.c_int32), ('weight_dtype', ctypes.c_int32)]


class JointParams(ctypes.Structure):
  """lt_joint_params: the joint weight function's operands (device pointers)."""
  _fields_ = [('hidden', ctypes.c_int32), ('precision', ctypes.c_int32),
              ('ctx_proj', ctypes.c_void_p), ('frame_proj', ctypes.c_void_p),
              ('out_weight', ctypes.c_void_p), ('out_bias', ctypes.c_void_p)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_G = ctypes.POINTER(Graph)
_TP = ctypes.POINTER(TableProblem)
_SIG = {
    'lt_num_context_states': [_I32, _I32, ctypes.POINTER(ctypes.c_int64)],
    'lt_den_forward': [ctypes.POINTER(Problem), _I32, _P, _P, _P, _P, _P],
    'lt_den_backward': [ctypes.POINTER(Problem), _P, _P, _P, _P, _P, _P, _P],
    'lt_num_forward': [ctypes.POINTER(Problem), _I32, _P, _P, _P, _P, _P, _P, _P],
    'lt_loss_forward': [ctypes.POINTER(Problem), _I32] + [_P] * 13,
    'lt_loss_backward_workspace_bytes': [ctypes.POINTER(Problem), _I32,
                                         ctypes.POINTER(ctypes.c_size_t)],
    'lt_loss_backward': [ctypes.POINTER(Problem), _I32] + [_P] * 14 + [ctypes.c_size_t, _P],
    'lt_loss_grad_design': [ctypes.POINTER(Problem), ctypes.POINTER(ctypes.c_int32)],
    'lt_loss_grad_workspace_bytes': [ctypes.POINTER(Problem), _I32,
                                     ctypes.POINTER(ctypes.c_size_t)],
    'lt_loss_grad': [ctypes.POINTER(Problem), _I32] + [_P] * 9 + [ctypes.c_size_t, _P],
    'lt_loss_grad_workspace_bytes_ex': [ctypes.POINTER(Problem), _I32, _I32,
                                        ctypes.POINTER(ctypes.c_size_t)],
    'lt_loss_grad_ex': [ctypes.POINTER(Problem), _I32, _I32] + [_P] * 9 + [ctypes.c_size_t, _P],
    'lt_scale_grad': [ctypes.POINTER(Problem), _P, _P, _P],
    'lt_chunk_workspace_bytes': [ctypes.POINTER(Problem), _I32, ctypes.POINTER(ctypes.c_size_t),
                                 ctypes.POINTER(ctypes.c_size_t)],
    'lt_chunk_forward': [ctypes.POINTER(Problem), _I32] + [_P] * 8 + [ctypes.c_size_t, _P,
                                                                    ctypes.c_size_t, _P],
    'lt_chunk_backward': [ctypes.POINTER(Problem), _I32] + [_P] * 7 + [ctypes.c_size_t, _P,
                                                                     ctypes.c_size_t, _P],
    'lt_graph_in_arcs': [_I32, _I32, _P, _P, _P],
    'lt_table_forward': [_G, _TP, _I32, _P, _P, _P, _P, _P],
    'lt_table_num_forward': [_G, _TP, _I32, _P, _P, _P, _P, _P, _P],
    'lt_table_loss_grad_workspace_bytes': [_G, _TP, ctypes.POINTER(ctypes.c_size_t)],
    'lt_table_loss_grad': [_G, _TP, _I32] + [_P] * 9 + [ctypes.c_size_t, _P],
    'lt_table_den_backward_workspace_bytes': [_G, _TP, _I32, ctypes.POINTER(ctypes.c_size_t)],
    'lt_table_den_backward': [_G, _TP, _I32] + [_P] * 7 + [ctypes.c_size_t, _P],
    'lt_table_num_backward_workspace_bytes': [_G, _TP, _I32, ctypes.POINTER(ctypes.c_size_t)],
    'lt_table_num_backward': [_G, _TP, _I32] + [_P] * 8 + [ctypes.c_size_t, _P],
    'lt_table_viterbi_workspace_bytes': [_G, _TP, ctypes.POINTER(ctypes.c_size_t)],
    'lt_table_viterbi': [_G, _TP, _P, _P, _I32, _P, _P, _P, ctypes.c_size_t, _P],
    'lt_joint_weights_workspace_bytes': [ctypes.c_int64, _I32, _I32,
                                         ctypes.POINTER(ctypes.c_size_t)],
    'lt_joint_weights': [ctypes.c_int64, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _P,
                         ctypes.c_size_t, _P],
    'lt_joint_weights_ex': [ctypes.c_int64, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _I32,
                            _P, ctypes.c_size_t, _P],
    'lt_joint_weights_backward_workspace_bytes': [ctypes.c_int64, _I32, _I32, _I32,
                                                  ctypes.POINTER(ctypes.c_size_t)],
    'lt_joint_weights_backward': [ctypes.c_int64, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P,
                                  _P, _P, ctypes.c_size_t, _P],
    'lt_loss_joint_workspace_bytes': [ctypes.POINTER(Problem), ctypes.POINTER(JointParams),
                                      ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_size_t)],
    'lt_loss_joint_forward': [ctypes.POINTER(Problem), ctypes.POINTER(JointParams)] + [_P] * 7 +
                             [ctypes.c_size_t, _P],
    'lt_loss_joint_backward': [ctypes.POINTER(Problem), ctypes.POINTER(JointParams)] + [_P] * 7 +
                              [ctypes.c_size_t, _P, ctypes.c_size_t, _P],
    'lt_loss_grad_joint': [ctypes.POINTER(Problem), ctypes.POINTER(JointParams)] + [_P] * 12 +
                          [ctypes.c_size_t, _P],
    'lt_viterbi_workspace_bytes': [ctypes.POINTER(Problem), ctypes.POINTER(ctypes.c_size_t)],
    'lt_viterbi': [ctypes.POINTER(Problem), _P, _P, _I32, _P, _P, _P, _P, _P, ctypes.c_size_t,
                   _P],
}
EXPORTED = tuple(_SIG) + ('lt_last_error', 'lt_version')


def lib():
  """Loads liblt_lattice.so (built in-tree by __graft_entry__.build())."""
  global _lib
  with _lock:
    if _lib is None:
      if not os.path.exists(LIB_PATH):
        raise LatticeLibraryError(
            f'{LIB_PATH} is missing: build it with `python -c "import __graft_entry__ as g; '
            'g.build()"` (hipcc --offload-arch=gfx950)')
      l = ctypes.CDLL(LIB_PATH)
      for name, argtypes in _SIG.items():
        fn = getattr(l, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
      l.lt_last_error.restype = ctypes.c_char_p
      l.lt_last_error.argtypes = []
      l.lt_version.restype = ctypes.c_char_p
      l.lt_version.argtypes = []
      _lib = l
  return _lib


def version():
  return lib().lt_version().decode()


def _check(rc, what):
  if rc != 0:
    raise LatticeLibraryError(f'{what} failed ({rc}): {lib().lt_last_error().decode()}')


def _ptr(t):
  return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
  return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _problem(W, vocab_size, context_size, max_labels=0):
  if W.dtype not in (torch.float32, torch.bfloat16):
    raise TypeError(f'arc weights must be float32 or bfloat16, got {W.dtype}')
  if not W.is_cuda:
    raise LatticeLibraryError('lattice kernels need the arc weights on a ROCm device')
  if not W.is_contiguous() or W.data_ptr() % 16:
    raise ValueError('arc weights must be contiguous and 16-byte aligned')
  B, T, C, R = W.shape
  if R != vocab_size + 1:
    raise ValueError(f'arc weights last dim {R} != vocab_size + 1 = {vocab_size + 1}')
  return Problem(B, T, vocab_size, context_size, max_labels,
                 LT_DTYPE_BF16 if W.dtype == torch.bfloat16 else LT_DTYPE_F32)


def num_context_states(vocab_size, context_size):
  out = ctypes.c_int64()
  _check(lib().lt_num_context_states(vocab_size, context_size, ctypes.byref(out)),
         'lt_num_context_states')
  return out.value


def _f32(shape, like):
  return torch.empty(shape, dtype=torch.float32, device=like.device)


def den_forward(W, num_frames, vocab_size, context_size, semiring, want_alpha=True):
  """lt_den_forward: (dist [B], alpha [B,T,C] or None)."""
  pb = _problem(W, vocab_size, context_size)
  B, T, C, _ = W.shape
  dist = _f32([B], W)
  alpha = _f32([B, T, C], W) if want_alpha else None
  _check(lib().lt_den_forward(ctypes.byref(pb), semiring, _ptr(W), _ptr(num_frames), _ptr(dist),
                              _ptr(alpha), _stream()), 'lt_den_forward')
  return dist, alpha


def den_backward(W, num_frames, log_z, alpha, grad, vocab_size, context_size):
  """lt_den_backward: grad-scaled arc marginals, W's dtype/shape."""
  pb = _problem(W, vocab_size, context_size)
  dW = torch.empty_like(W)
  _check(lib().lt_den_backward(ctypes.byref(pb), _ptr(W), _ptr(num_frames), _ptr(log_z),
                               _ptr(alpha), _ptr(grad), _ptr(dW), _stream()), 'lt_den_backward')
  return dW


def num_forward(W, num_frames, labels, num_labels, vocab_size, context_size, semiring,
                want_alpha=True):
  """lt_num_forward: (num [B], alpha_num [B,T,U+1] or None)."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  B, T = W.shape[:2]
  num = _f32([B], W)
  an = _f32([B, T, U + 1], W) if want_alpha else None
  _check(lib().lt_num_forward(ctypes.byref(pb), semiring, _ptr(W), _ptr(num_frames),
                              _ptr(labels), _ptr(num_labels), _ptr(num), _ptr(an), _stream()),
         'lt_num_forward')
  return num, an


def prefer_checkpoints(batch, device=None, shape=None):
  """Whether the checkpointing loss path is the faster one for `batch`
  utterances: it runs the alpha and beta recursions as separate workgroups
  (2 per utterance) and adds a streaming marginal pass, which pays off while
  2*batch workgroups still find idle CUs -- and, for shapes on the pipelined
  bigram recursions (`shape` = (frames, labels, vocab_size, context_size,
  bf16)), up to 1.5 CUs of utterances; beyond that the single-workgroup
  recursion backward (marginals fused into the beta recursion) is faster.
  Mirrors lt_loss_grad_design."""
  cus = torch.cuda.get_device_properties(device or torch.cuda.current_device()).multi_processor_count
  if 2 * batch <= cus:
    return True
  return shape is not None and 2 * batch <= 3 * cus and pipe_path(batch, *shape)


def pipe_path(batch, frames, labels, vocab_size, context_size, bf16=False):
  """Whether lt_loss_forward with checkpoints runs the pipelined bigram
  recursions (lt_pipe.hip, kernel ``pipe_kernel``) for this shape; mirrors
  lt_impl::pipe_eligible."""
  if context_size != 1 or not 1 <= vocab_size <= 32 or labels + 1 > 256:
    return False
  C = vocab_size + 1
  return batch * frames * C * C * (2 if bf16 else 4) < 0xFFFFFFF0


def loss_forward(W, num_frames, labels, num_labels, vocab_size, context_size, local_norm,
                 want_alpha=True, checkpoints=False):
  """lt_loss_forward: (loss, log_z, num, alpha, alpha_num), plus a 6th element
  ``ck = (beta, beta_num, arcs)`` with ``checkpoints=True`` -- the backward
  recursion then runs concurrently with the forward and loss_backward(ck=ck)
  is one streaming pass."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  B, T, C, _ = W.shape
  loss, log_z, num = _f32([B], W), _f32([B], W), _f32([B], W)
  want_alpha = want_alpha or checkpoints
  alpha = _f32([B, T, C], W) if (want_alpha and not local_norm) else None
  an = _f32([B, T, U + 1], W) if want_alpha else None
  beta = _f32([B, T, C], W) if (checkpoints and not local_norm) else None
  beta_num = _f32([B, T, U + 1], W) if checkpoints else None
  arcs = (torch.empty([B, 4 * (U + 1)], dtype=torch.int32, device=W.device)
          if checkpoints else None)
  if local_norm:
    log_z.zero_()
  _check(lib().lt_loss_forward(ctypes.byref(pb), int(bool(local_norm)), _ptr(W),
                               _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(loss),
                               None if local_norm else _ptr(log_z), _ptr(num), _ptr(alpha),
                               _ptr(an), _ptr(beta), _ptr(beta_num), _ptr(arcs), _stream()),
         'lt_loss_forward')
  if checkpoints:
    return loss, log_z, num, alpha, an, (beta, beta_num, arcs)
  return loss, log_z, num, alpha, an


def loss_backward(W, num_frames, labels, num_labels, log_z, num, alpha, alpha_num, grad,
                  vocab_size, context_size, local_norm, ck=None):
  """lt_loss_backward: d loss / dW (scaled by grad), W's dtype/shape. With
  ``ck`` from loss_forward(checkpoints=True) the marginal pass runs."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  beta, beta_num, arcs = ck if ck is not None else (None, None, None)
  ws_bytes = ctypes.c_size_t(0)
  if ck is None:
    _check(lib().lt_loss_backward_workspace_bytes(ctypes.byref(pb), int(bool(local_norm)),
                                                  ctypes.byref(ws_bytes)),
           'lt_loss_backward_workspace_bytes')
  ws = (torch.empty([ws_bytes.value], dtype=torch.uint8, device=W.device)
        if ws_bytes.value else None)
  dW = torch.empty_like(W)
  _check(lib().lt_loss_backward(ctypes.byref(pb), int(bool(local_norm)), _ptr(W),
                                _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(log_z),
                                _ptr(num), _ptr(alpha), _ptr(alpha_num), _ptr(beta),
                                _ptr(beta_num), _ptr(arcs), _ptr(grad), _ptr(dW), _ptr(ws),
                                ws_bytes.value, _stream()), 'lt_loss_backward')
  return dW


def chunk_path(batch, frames, labels, vocab_size, context_size, device=None):
  """Whether lt_loss_grad runs the chunked two-level scan (lt_chunk.hip) for
  this shape; mirrors lt_impl::chunk_preferred: an eligible shape and
  16 * batch <= 11 * CUs (beyond that the frame-serial checkpointing design is
  faster, profiles/r04_design_crossover.txt)."""
  if context_size != 1 or not 1 <= vocab_size <= 32 or labels + 1 > 128 or frames < 1:
    return False
  C = vocab_size + 1
  if batch * frames * C * C >= 2 ** 31:
    return False
  if not torch.cuda.is_available():
    return True
  cus = torch.cuda.get_device_properties(device or torch.cuda.current_device()).multi_processor_count
  return 16 * batch <= 11 * cus


def fused_path(batch, frames, labels, vocab_size, context_size, device=None, bf16=False):
  """Whether lt_loss_grad runs as ONE fused pipe launch for this shape: the
  bigram past the chunked scan's range while the launch's recursion grid is
  co-resident (an occupancy query: lt_loss_grad_design answers it)."""
  if chunk_path(batch, frames, labels, vocab_size, context_size, device):
    return False
  if not pipe_path(batch, frames, labels, vocab_size, context_size, bf16):
    return False
  return loss_grad_design(batch, frames, labels, vocab_size, context_size, bf16) == DESIGN_FUSED_PIPE


DESIGN_AUTO, DESIGN_CHUNK, DESIGN_FUSED_PIPE, DESIGN_CHECKPOINTS, DESIGN_RECURSION = -1, 0, 1, 2, 3
DESIGN_NAMES = {DESIGN_CHUNK: 'chunk', DESIGN_FUSED_PIPE: 'fused_pipe',
                DESIGN_CHECKPOINTS: 'checkpoints', DESIGN_RECURSION: 'recursion'}


def loss_grad_design(batch, frames, labels, vocab_size, context_size, bf16=False):
  """lt_loss_grad_design: the design lt_loss_grad runs for this shape on the
  current device (DESIGN_* above)."""
  pb = Problem(batch, frames, vocab_size, context_size, labels,
               LT_DTYPE_BF16 if bf16 else LT_DTYPE_F32)
  out = ctypes.c_int32(-1)
  _check(lib().lt_loss_grad_design(ctypes.byref(pb), ctypes.byref(out)), 'lt_loss_grad_design')
  return out.value


def loss_grad_workspace_bytes(W, vocab_size, context_size, max_labels, local_norm,
                              design=DESIGN_AUTO):
  pb = _problem(W, vocab_size, context_size, max_labels)
  out = ctypes.c_size_t(0)
  _check(lib().lt_loss_grad_workspace_bytes_ex(ctypes.byref(pb), int(bool(local_norm)),
                                               int(design), ctypes.byref(out)),
         'lt_loss_grad_workspace_bytes_ex')
  return out.value


def loss_grad(W, num_frames, labels, num_labels, vocab_size, context_size, local_norm,
              workspace=None, design=DESIGN_AUTO):
  """lt_loss_grad(_ex): (loss, log_z, num, dW) with dW = d(sum loss)/dW in one
  call, in `design` (DESIGN_AUTO: the call's own choice for the shape).
  ``workspace`` (uint8 device tensor of loss_grad_workspace_bytes) is
  allocated when not given."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  B = W.shape[0]
  nbytes = loss_grad_workspace_bytes(W, vocab_size, context_size, U, local_norm, design)
  if workspace is None or workspace.numel() < nbytes:
    workspace = torch.empty([max(nbytes, 1)], dtype=torch.uint8, device=W.device)
  loss, log_z, num = _f32([B], W), _f32([B], W), _f32([B], W)
  dW = torch.empty_like(W)
  _check(lib().lt_loss_grad_ex(ctypes.byref(pb), int(bool(local_norm)), int(design), _ptr(W),
                               _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(loss),
                               _ptr(log_z), _ptr(num), _ptr(dW), _ptr(workspace),
                               workspace.numel(), _stream()), 'lt_loss_grad_ex')
  return loss, log_z, num, dW


def chunk_workspace_bytes(W, vocab_size, context_size, max_labels, local_norm):
  """(state_bytes, scratch_bytes) of lt_chunk_forward / lt_chunk_backward."""
  pb = _problem(W, vocab_size, context_size, max_labels)
  st, sc = ctypes.c_size_t(0), ctypes.c_size_t(0)
  _check(lib().lt_chunk_workspace_bytes(ctypes.byref(pb), int(bool(local_norm)), ctypes.byref(st),
                                        ctypes.byref(sc)), 'lt_chunk_workspace_bytes')
  return st.value, sc.value


def chunk_forward(W, num_frames, labels, num_labels, vocab_size, context_size, local_norm):
  """lt_chunk_forward: (loss, log_z, num, state); `state` (uint8 device
  tensor) carries the chunk-boundary values to chunk_backward. The scratch
  buffer lives only for the call."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  B = W.shape[0]
  st, sc = chunk_workspace_bytes(W, vocab_size, context_size, U, local_norm)
  state = torch.empty([max(st, 16)], dtype=torch.uint8, device=W.device)
  scratch = torch.empty([max(sc, 16)], dtype=torch.uint8, device=W.device)
  loss, log_z, num = _f32([B], W), _f32([B], W), _f32([B], W)
  _check(lib().lt_chunk_forward(ctypes.byref(pb), int(bool(local_norm)), _ptr(W), _ptr(num_frames),
                                _ptr(labels), _ptr(num_labels), _ptr(loss), _ptr(log_z), _ptr(num),
                                _ptr(state), st, _ptr(scratch), sc, _stream()), 'lt_chunk_forward')
  return loss, log_z, num, state


def chunk_backward(W, num_frames, labels, num_labels, vocab_size, context_size, local_norm, state,
                   grad=None):
  """lt_chunk_backward: dW = grad[b] * d loss_b / dW (grad None = ones) from
  the forward's `state`."""
  U = labels.shape[-1]
  pb = _problem(W, vocab_size, context_size, U)
  st, sc = chunk_workspace_bytes(W, vocab_size, context_size, U, local_norm)
  scratch = torch.empty([max(sc, 16)], dtype=torch.uint8, device=W.device)
  dW = torch.empty_like(W)
  g = None if grad is None else grad.float().contiguous()
  _check(lib().lt_chunk_backward(ctypes.byref(pb), int(bool(local_norm)), _ptr(W),
                                 _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(g),
                                 _ptr(dW), _ptr(state), st, _ptr(scratch), sc, _stream()),
         'lt_chunk_backward')
  return dW


def grad_workspace_errors(workspace, W, vocab_size, context_size, max_labels, local_norm):
  """The hand-off error word of a fused-pipe lt_loss_grad workspace (0 = no
  timed-out wait): after the granule rows (alpha, beta [B,T,C]; alpha^n,
  beta^n [B,T,U+1]; 8 bytes each) and the band flags [2][B] of
  pipe_mid_workspace_bytes; test / diagnostic use, synchronises."""
  del local_norm
  C = num_context_states(vocab_size, context_size)
  B, T = W.shape[:2]
  NP = max_labels + 1
  off = 8 * (2 * B * T * C + 2 * B * T * NP + 2 * B)
  return int(workspace[off:off + 4].view(torch.int32).item())


def chunk_fallback_count(workspace, batch):
  """Utterances the last chunked lt_loss_grad call on `workspace` sent to the
  frame-serial kernels (the state's per-utterance fallback words, at its
  start); diagnostic use, synchronises."""
  return int(workspace[:4 * batch].view(torch.int32).ne(0).sum().item())


def scale_grad(dW, grad, vocab_size, context_size):
  """lt_scale_grad: dW[b] *= grad[b] in place (no work where grad[b] == 1)."""
  pb = _problem(dW, vocab_size, context_size)
  _check(lib().lt_scale_grad(ctypes.byref(pb), _ptr(grad.float().contiguous()), _ptr(dW),
                             _stream()), 'lt_scale_grad')
  return dW


def viterbi(W, num_frames, vocab_size, context_size, label_convention, grad=None,
            want_arcs=False):
  """lt_viterbi: (labels int64 [B,T], path_weight [B], arcs or None)."""
  pb = _problem(W, vocab_size, context_size)
  B, T = W.shape[:2]
  ws_bytes = ctypes.c_size_t()
  _check(lib().lt_viterbi_workspace_bytes(ctypes.byref(pb), ctypes.byref(ws_bytes)),
         'lt_viterbi_workspace_bytes')
  ws = torch.empty([max(ws_bytes.value, 1)], dtype=torch.uint8, device=W.device)
  labels = torch.empty([B, T], dtype=torch.int64, device=W.device)
  weight = _f32([B], W)
  arcs = torch.empty_like(W) if want_arcs else None
  _check(lib().lt_viterbi(ctypes.byref(pb), _ptr(W), _ptr(num_frames), label_convention,
                          _ptr(labels), _ptr(weight), _ptr(grad), _ptr(arcs), _ptr(ws),
                          ws_bytes.value, _stream()), 'lt_viterbi')
  return labels, weight, arcs


# ---------------------------------------------------------------------------
# General lattices (lt_table.hip): any next-state table, FrameDependent (K=0)
# or FrameLabelDependent(K)
# ---------------------------------------------------------------------------
class TableGraph:
  """Device copy of a next-state table [C, V] (entry [p, y-1] = next state)
  with its in-arc CSR, for alignment expansions K (0 = FrameDependent)."""

  def __init__(self, next_state_table, expansions, device):
    import numpy as np
    tab = torch.as_tensor(next_state_table).to(torch.int32).cpu().contiguous()
    if tab.ndim != 2 or 0 in tab.shape:
      raise ValueError(f'next_state_table must be a non-empty [C, V] table, got {tuple(tab.shape)}')
    C, V = tab.shape
    tab_np = tab.numpy()
    in_off = np.zeros([C + 1], np.int32)
    in_arc = np.zeros([C * V], np.int32)
    _check(lib().lt_graph_in_arcs(C, V, tab_np.ctypes.data_as(_P), in_off.ctypes.data_as(_P),
                                  in_arc.ctypes.data_as(_P)), 'lt_graph_in_arcs')
    self.C, self.V, self.K = int(C), int(V), int(expansions)
    self.table = tab.to(device)
    self.in_off = torch.from_numpy(in_off).to(device)
    self.in_arc = torch.from_numpy(in_arc).to(device)
    self.g = Graph(self.C, self.V, self.K, self.table.data_ptr(), self.in_off.data_ptr(),
                   self.in_arc.data_ptr())

  def num_alignment_states(self):
    return 1 if self.K == 0 else self.K + 1


def _tproblem(graph, W, max_labels=0):
  if W.dtype not in (torch.float32, torch.bfloat16):
    raise TypeError(f'arc weights must be float32 or bfloat16, got {W.dtype}')
  if not W.is_cuda:
    raise LatticeLibraryError('lattice kernels need the arc weights on a ROCm device')
  if not W.is_contiguous():
    raise ValueError('arc weights must be contiguous')
  B, T, C, R = W.shape
  if C != graph.C or R != graph.V + 1:
    raise ValueError(f'arc weights {tuple(W.shape)} do not match the graph (C={graph.C}, '
                     f'V+1={graph.V + 1})')
  return TableProblem(B, T, max_labels, LT_DTYPE_BF16 if W.dtype == torch.bfloat16 else LT_DTYPE_F32)


def table_forward(graph, W, num_frames, semiring, want_alpha=True):
  """lt_table_forward: (dist [B], alpha [B,T,C] or None)."""
  pb = _tproblem(graph, W)
  B, T = W.shape[:2]
  dist = _f32([B], W)
  alpha = _f32([B, T, graph.C], W) if want_alpha else None
  _check(lib().lt_table_forward(ctypes.byref(graph.g), ctypes.byref(pb), semiring, _ptr(W),
                                _ptr(num_frames), _ptr(dist), _ptr(alpha), _stream()),
         'lt_table_forward')
  return dist, alpha


def table_num_forward(graph, W, num_frames, labels, num_labels, semiring):
  pb = _tproblem(graph, W, labels.shape[-1])
  num = _f32([W.shape[0]], W)
  _check(lib().lt_table_num_forward(ctypes.byref(graph.g), ctypes.byref(pb), semiring, _ptr(W),
                                    _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(num),
                                    _stream()), 'lt_table_num_forward')
  return num


def table_loss_grad(graph, W, num_frames, labels, num_labels, local_norm, want_grad=True):
  """lt_table_loss_grad: (loss, log_z, num, dW = d(sum loss)/dW or None)."""
  pb = _tproblem(graph, W, labels.shape[-1])
  B = W.shape[0]
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_table_loss_grad_workspace_bytes(ctypes.byref(graph.g), ctypes.byref(pb),
                                                  ctypes.byref(nbytes)),
         'lt_table_loss_grad_workspace_bytes')
  ws = (torch.empty([max(nbytes.value, 1)], dtype=torch.uint8, device=W.device)
        if want_grad else None)
  loss, log_z, num = _f32([B], W), _f32([B], W), _f32([B], W)
  dW = torch.empty_like(W) if want_grad else None
  _check(lib().lt_table_loss_grad(ctypes.byref(graph.g), ctypes.byref(pb), int(bool(local_norm)),
                                  _ptr(W), _ptr(num_frames), _ptr(labels), _ptr(num_labels),
                                  _ptr(loss), _ptr(log_z), _ptr(num), _ptr(dW), _ptr(ws),
                                  nbytes.value if want_grad else 0, _stream()),
         'lt_table_loss_grad')
  return loss, log_z, num, dW


def table_den_backward(graph, W, num_frames, semiring, dist=None, alpha=None, grad=None):
  """lt_table_den_backward: dW [B,T,C,V+1] (W's dtype) = grad_b * the gradient
  of the semiring's distance (Log: the arc marginals, from lt_table_forward's
  log_z and alpha; Real: alpha * beta'; MaxTropical: the best path's arcs)."""
  pb = _tproblem(graph, W)
  B = W.shape[0]
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_table_den_backward_workspace_bytes(ctypes.byref(graph.g), ctypes.byref(pb),
                                                     semiring, ctypes.byref(nbytes)),
         'lt_table_den_backward_workspace_bytes')
  ws = torch.empty([max(nbytes.value, 1)], dtype=torch.uint8, device=W.device)
  dW = torch.empty_like(W)
  if dist is not None:
    dist = dist.to(torch.float32).contiguous()
  if alpha is not None:
    alpha = alpha.to(torch.float32).contiguous()
  if grad is not None:
    grad = grad.to(device=W.device, dtype=torch.float32).reshape(B).contiguous()
  _check(lib().lt_table_den_backward(ctypes.byref(graph.g), ctypes.byref(pb), semiring, _ptr(W),
                                     _ptr(num_frames), _ptr(dist), _ptr(alpha), _ptr(grad),
                                     _ptr(dW), _ptr(ws), nbytes.value, _stream()),
         'lt_table_den_backward')
  return dW


def table_num_backward_check(graph, W, labels, semiring):
  """Raises LatticeLibraryError now if lt_table_num_backward would refuse
  this problem (its string-gradient LDS rule, the semiring): a host-only
  query, no launch."""
  pb = _tproblem(graph, W, labels.shape[-1])
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_table_num_backward_workspace_bytes(ctypes.byref(graph.g), ctypes.byref(pb),
                                                     semiring, ctypes.byref(nbytes)),
         'lt_table_num_backward_workspace_bytes')


def table_num_backward(graph, W, num_frames, labels, num_labels, semiring, grad=None):
  """lt_table_num_backward: (num [B], dW [B,T,C,V+1] in W's dtype) = the
  string distance and grad_b * its gradient in MaxTropical (the best
  string-aligned path's arcs) or Real (alpha * beta' on the string
  acceptor)."""
  pb = _tproblem(graph, W, labels.shape[-1])
  B = W.shape[0]
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_table_num_backward_workspace_bytes(ctypes.byref(graph.g), ctypes.byref(pb),
                                                     semiring, ctypes.byref(nbytes)),
         'lt_table_num_backward_workspace_bytes')
  ws = torch.empty([max(nbytes.value, 1)], dtype=torch.uint8, device=W.device)
  num = _f32([B], W)
  dW = torch.empty_like(W)
  if grad is not None:
    grad = grad.to(device=W.device, dtype=torch.float32).reshape(B).contiguous()
  _check(lib().lt_table_num_backward(ctypes.byref(graph.g), ctypes.byref(pb), semiring, _ptr(W),
                                     _ptr(num_frames), _ptr(labels), _ptr(num_labels), _ptr(grad),
                                     _ptr(num), _ptr(dW), _ptr(ws), nbytes.value, _stream()),
         'lt_table_num_backward')
  return num, dW


def table_viterbi(graph, W, num_frames, label_convention):
  """lt_table_viterbi: (labels int64 [B, T*A], path weights [B])."""
  pb = _tproblem(graph, W)
  B, T = W.shape[:2]
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_table_viterbi_workspace_bytes(ctypes.byref(graph.g), ctypes.byref(pb),
                                                ctypes.byref(nbytes)),
         'lt_table_viterbi_workspace_bytes')
  ws = torch.empty([max(nbytes.value, 1)], dtype=torch.uint8, device=W.device)
  labels = torch.empty([B, T * graph.num_alignment_states()], dtype=torch.int64, device=W.device)
  weight = _f32([B], W)
  _check(lib().lt_table_viterbi(ctypes.byref(graph.g), ctypes.byref(pb), _ptr(W),
                                _ptr(num_frames), label_convention, _ptr(labels), _ptr(weight),
                                _ptr(ws), nbytes.value, _stream()), 'lt_table_viterbi')
  return labels, weight


JOINT_BF16, JOINT_SPLIT = 0, 1  # lt_joint_weights_ex precisions (include/lt_lattice.h)


def joint_weights(ctx_proj, frame_proj, out_weight, out_bias, dtype=torch.float32,
                  precision='fp32'):
  """lt_joint_weights_ex: W [..., C, R] = out_bias + tanh(ctx_proj[c] + frame_proj[...]) @
  out_weight^T on the matrix cores, fp32 sums; frame_proj [..., H], ctx_proj
  [C, H], out_weight [R, H], out_bias [R] (fp32). precision 'fp32': split-bf16
  products (LT_JOINT_SPLIT, fp32-faithful); 'bf16': one bf16 product."""
  if precision not in ('fp32', 'bf16'):
    raise ValueError(f"lt_joint_weights: precision must be 'fp32' or 'bf16', got {precision!r}")
  for name, t in (('ctx_proj', ctx_proj), ('frame_proj', frame_proj),
                  ('out_weight', out_weight), ('out_bias', out_bias)):
    if not t.is_cuda:
      raise LatticeLibraryError(f'lt_joint_weights: {name} must be on a ROCm device')
    if t.dtype != torch.float32:
      raise TypeError(f'lt_joint_weights: {name} must be float32, got {t.dtype}')
  C, H = ctx_proj.shape
  R = out_weight.shape[0]
  pc = ctx_proj.contiguous()
  pf = frame_proj.reshape(-1, H).contiguous()
  wo, bo = out_weight.contiguous(), out_bias.contiguous()
  W = torch.empty([*frame_proj.shape[:-1], C, R], dtype=dtype, device=frame_proj.device)
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_joint_weights_workspace_bytes(pf.shape[0], C, H, ctypes.byref(nbytes)),
         'lt_joint_weights_workspace_bytes')
  ws = torch.empty([(nbytes.value + 15) // 16 * 4], dtype=torch.float32, device=pf.device)
  _check(lib().lt_joint_weights_ex(pf.shape[0], C, H, R, _ptr(pc), _ptr(pf), _ptr(wo), _ptr(bo),
                                   _ptr(W), LT_DTYPE_BF16 if dtype == torch.bfloat16 else LT_DTYPE_F32,
                                   JOINT_SPLIT if precision == 'fp32' else JOINT_BF16,
                                   _ptr(ws), ws.numel() * 4, _stream()), 'lt_joint_weights_ex')
  return W


def joint_weights_backward_supported(C, H, R, rows=0):
  """Shapes lt_joint_weights_backward takes (its LDS holds a d_ctx_proj block)."""
  if H % 32 or R > 64 or rows * max(C, H) >= 2 ** 31:
    return False
  n = H // 32
  waves = 8 if n % 8 == 0 else 4 if n % 4 == 0 else 2 if n % 2 == 0 else 1
  KB = (R + 15) // 16
  RB = 64 if R > 32 else 32
  # the bf16 hi/lo tiles only for 8-wave workgroups (lt_producer.hip bwd_lds)
  bufb = 4 * 32 * (16 * KB + 4) + (4 * 32 * (16 * KB + 8) + 4 * RB * 36 if waves == 8 else 0)
  return 2 * bufb + 4 * C * 32 * waves <= 160 * 1024


def joint_weights_backward(ctx_proj, frame_proj, out_weight, grad_W):
  """lt_joint_weights_backward: (d_ctx_proj [C, H], d_frame_proj [..., H],
  d_out_weight [R, H], d_out_bias [R]) for grad_W = dL/dW [..., C, R] (fp32,
  split-bf16 products on the matrix cores)."""
  C, H = ctx_proj.shape
  R = out_weight.shape[0]
  pc = ctx_proj.contiguous()
  pf = frame_proj.reshape(-1, H).contiguous()
  wo = out_weight.contiguous()
  g = grad_W.reshape(-1, C, R).float().contiguous()
  rows = pf.shape[0]
  dpc = torch.empty_like(pc)
  dpf = torch.empty_like(pf)
  dwo = torch.empty_like(wo)
  dbias = torch.empty([R], dtype=torch.float32, device=pc.device)
  nbytes = ctypes.c_size_t(0)
  _check(lib().lt_joint_weights_backward_workspace_bytes(rows, C, H, R, ctypes.byref(nbytes)),
         'lt_joint_weights_backward_workspace_bytes')
  ws = torch.empty([max(1, nbytes.value // 4)], dtype=torch.float32, device=pc.device)
  _check(lib().lt_joint_weights_backward(rows, C, H, R, _ptr(pc), _ptr(pf), _ptr(wo), _ptr(g),
                                         _ptr(dpc), _ptr(dpf), _ptr(dwo), _ptr(dbias), _ptr(ws),
                                         ws.numel() * 4, _stream()), 'lt_joint_weights_backward')
  return dpc, dpf.reshape(frame_proj.shape), dwo, dbias


# ---------------------------------------------------------------------------
# The joint weight function fused into the lattice loss (lt_joint.hip)
# ---------------------------------------------------------------------------
def _joint(ctx_proj, frame_proj, out_weight, out_bias, precision):
  for name, t in (('ctx_proj', ctx_proj), ('frame_proj', frame_proj),
                  ('out_weight', out_weight), ('out_bias', out_bias)):
    if not t.is_cuda:
      raise LatticeLibraryError(f'joint loss: {name} must be on a ROCm device')
    if t.dtype != torch.float32:
      raise TypeError(f'joint loss: {name} must be float32, got {t.dtype}')
  C, H = ctx_proj.shape
  ops = tuple(x.contiguous() for x in (ctx_proj, frame_proj.reshape(-1, H), out_weight, out_bias))
  jp = JointParams(H, JOINT_SPLIT if precision == 'fp32' else JOINT_BF16,
                   *(x.data_ptr() for x in ops))
  return jp, ops


def joint_problem(batch, frames, labels, vocab_size):
  return Problem(batch, frames, vocab_size, 1, labels, LT_DTYPE_F32)


def joint_loss_supported(batch, frames, labels, vocab_size, context_size, hidden,
                         precision='fp32'):
  """Shapes lt_loss_grad_joint takes, as the library itself decides
  (lt_loss_joint_workspace_bytes returns LT_EUNSUPPORTED otherwise): FullNGram
  n = 1, 16 < V <= 32, U < 128, hidden a multiple of 32 up to 256 whose
  marginal-pass LDS image (jf_lds: Wo rows, the checkpoint rows, the per-state
  d_Pc and e^{2Pc} rows) fits the CU's 160 KB -- e.g. H = 256 at U = 100 does
  not (about 193 KB), H = 160 does."""
  if context_size != 1:
    return False
  if batch * frames * (vocab_size + 1) ** 2 * 4 >= 0xFFFFFFF0:
    return False
  pb = joint_problem(batch, frames, labels, vocab_size)
  jp = JointParams(hidden, JOINT_SPLIT if precision == 'fp32' else JOINT_BF16, None, None, None,
                   None)
  st, sc = ctypes.c_size_t(0), ctypes.c_size_t(0)
  return lib().lt_loss_joint_workspace_bytes(ctypes.byref(pb), ctypes.byref(jp), ctypes.byref(st),
                                             ctypes.byref(sc)) == 0  # LT_OK


def joint_loss_workspace_bytes(batch, frames, labels, vocab_size, hidden, precision='fp32'):
  """(state_bytes, scratch_bytes) of lt_loss_joint_forward / _backward."""
  pb = joint_problem(batch, frames, labels, vocab_size)
  jp = JointParams(hidden, JOINT_SPLIT if precision == 'fp32' else JOINT_BF16, None, None, None,
                   None)
  st, sc = ctypes.c_size_t(0), ctypes.c_size_t(0)
  _check(lib().lt_loss_joint_workspace_bytes(ctypes.byref(pb), ctypes.byref(jp), ctypes.byref(st),
                                             ctypes.byref(sc)), 'lt_loss_joint_workspace_bytes')
  return st.value, sc.value


def joint_loss_forward(ctx_proj, frame_proj, out_weight, out_bias, num_frames, labels, num_labels,
                       precision='fp32'):
  """lt_loss_joint_forward: (loss [B], log_z, num, state) with W formed on the
  matrix cores where the recursions use it; frame_proj [B, T, H]."""
  B, T, H = frame_proj.shape
  V = out_weight.shape[0] - 1
  U = labels.shape[-1]
  jp, ops = _joint(ctx_proj, frame_proj, out_weight, out_bias, precision)
  pb = joint_problem(B, T, U, V)
  st, _ = joint_loss_workspace_bytes(B, T, U, V, H, precision)
  state = torch.empty([max(st, 16)], dtype=torch.uint8, device=frame_proj.device)
  loss, log_z, num = (_f32([B], frame_proj) for _ in range(3))
  _check(lib().lt_loss_joint_forward(ctypes.byref(pb), ctypes.byref(jp), _ptr(num_frames),
                                     _ptr(labels), _ptr(num_labels), _ptr(loss), _ptr(log_z),
                                     _ptr(num), _ptr(state), state.numel(), _stream()),
         'lt_loss_joint_forward')
  del ops  # the launch is queued on the stream; the caching allocator orders reuse
  return loss, log_z, num, state


def joint_loss_backward(ctx_proj, frame_proj, out_weight, out_bias, num_frames, labels, state,
                        grad=None, precision='fp32'):
  """lt_loss_joint_backward: (d_ctx_proj, d_frame_proj [B, T, H], d_out_weight,
  d_out_bias) of sum_b grad[b] loss_b from the forward's `state`."""
  B, T, H = frame_proj.shape
  V = out_weight.shape[0] - 1
  U = labels.shape[-1]
  jp, ops = _joint(ctx_proj, frame_proj, out_weight, out_bias, precision)
  pb = joint_problem(B, T, U, V)
  st, sc = joint_loss_workspace_bytes(B, T, U, V, H, precision)
  scratch = torch.empty([max(sc, 16)], dtype=torch.uint8, device=frame_proj.device)
  dpc = torch.empty_like(ops[0])
  dpf = torch.empty_like(ops[1])
  dwo = torch.empty_like(ops[2])
  dbias = torch.empty_like(ops[3])
  g = None if grad is None else grad.to(torch.float32).reshape(B).contiguous()
  _check(lib().lt_loss_joint_backward(ctypes.byref(pb), ctypes.byref(jp), _ptr(num_frames), _ptr(g),
                                      _ptr(dpc), _ptr(dpf), _ptr(dwo), _ptr(dbias), _ptr(state),
                                      state.numel(), _ptr(scratch), scratch.numel(), _stream()),
         'lt_loss_joint_backward')
  return dpc, dpf.reshape(B, T, H), dwo, dbias


def loss_grad_joint(ctx_proj, frame_proj, out_weight, out_bias, num_frames, labels, num_labels,
                    grad=None, precision='fp32', workspace=None):
  """lt_loss_grad_joint: (loss, log_z, num, d_ctx_proj, d_frame_proj, d_out_weight,
  d_out_bias) in one call; `workspace` (uint8, state + scratch bytes) reused
  when given."""
  B, T, H = frame_proj.shape
  V = out_weight.shape[0] - 1
  U = labels.shape[-1]
  jp, ops = _joint(ctx_proj, frame_proj, out_weight, out_bias, precision)
  pb = joint_problem(B, T, U, V)
  st, sc = joint_loss_workspace_bytes(B, T, U, V, H, precision)
  if workspace is None or workspace.numel() < st + sc:
    workspace = torch.empty([st + sc], dtype=torch.uint8, device=frame_proj.device)
  loss, log_z, num = (_f32([B], frame_proj) for _ in range(3))
  dpc = torch.empty_like(ops[0])
  dpf = torch.empty_like(ops[1])
  dwo = torch.empty_like(ops[2])
  dbias = torch.empty_like(ops[3])
  g = None if grad is None else grad.to(torch.float32).reshape(B).contiguous()
  _check(lib().lt_loss_grad_joint(ctypes.byref(pb), ctypes.byref(jp), _ptr(num_frames),
                                  _ptr(labels), _ptr(num_labels), _ptr(g), _ptr(loss), _ptr(log_z),
                                  _ptr(num), _ptr(dpc), _ptr(dpf), _ptr(dwo), _ptr(dbias),
                                  _ptr(workspace), workspace.numel(), _stream()),
         'lt_loss_grad_joint')
  return loss, log_z, num, dpc, dpf.reshape(B, T, H), dwo, dbias
