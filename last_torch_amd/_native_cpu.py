"""ctypes binding of the host twin (liblt_lattice_cpu.so, include/lt_lattice_cpu.h).

The same lattice computations as ``_native`` for host (CPU) tensors, built
with g++ alone, so the drop-in binds a native implementation on a GPU-less
host too. Calls are synchronous; utterances run on a pool of host threads
(``set_num_threads``).
"""
import ctypes
import os
import threading

import torch

from ._native import Problem, LatticeLibraryError, LT_DTYPE_BF16, LT_DTYPE_F32

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'liblt_lattice_cpu.so')

_lock = threading.Lock()
_lib = None
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_PB = ctypes.POINTER(Problem)
_SIG = {
    'lt_cpu_set_num_threads': [_I32],
    'lt_cpu_num_threads': [],
    'lt_cpu_den_forward': [_PB, _I32, _P, _P, _P, _P],
    'lt_cpu_num_forward': [_PB, _I32, _P, _P, _P, _P, _P, _P],
    'lt_cpu_den_backward': [_PB, _P, _P, _P, _P, _P, _P],
    'lt_cpu_loss_grad': [_PB, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    'lt_cpu_viterbi': [_PB, _P, _P, _I32, _P, _P, _P, _P],
}
EXPORTED = tuple(_SIG) + ('lt_cpu_last_error',)


def lib():
  """Loads liblt_lattice_cpu.so (built in-tree by __graft_entry__.build())."""
  global _lib
  with _lock:
    if _lib is None:
      if not os.path.exists(LIB_PATH):
        raise LatticeLibraryError(f'{LIB_PATH} is missing: build it with `make` (g++)')
      l = ctypes.CDLL(LIB_PATH)
      for name, argtypes in _SIG.items():
        fn = getattr(l, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
      l.lt_cpu_last_error.restype = ctypes.c_char_p
      l.lt_cpu_last_error.argtypes = []
      _lib = l
  return _lib


def _cpu_supported():
  """The twin is built for x86-64-v3 (AVX2, FMA; Makefile CPUFLAGS): on a
  host without them it would die of SIGILL, so it is not offered there."""
  try:
    with open('/proc/cpuinfo') as f:
      for line in f:
        if line.startswith('flags'):
          flags = set(line.split(':', 1)[1].split())
          return {'avx2', 'fma', 'bmi2'} <= flags
  except OSError:
    pass
  return False


_SUPPORTED = None


def available():
  """The library exists and this host can run its code."""
  global _SUPPORTED
  if _SUPPORTED is None:
    _SUPPORTED = _cpu_supported()
  return _SUPPORTED and os.path.exists(LIB_PATH)


def _check(rc):
  if rc != 0:
    raise LatticeLibraryError(f'lt_cpu error {rc}: {lib().lt_cpu_last_error().decode()}')


def _ptr(t):
  return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def _weights(W):
  if W.device.type != 'cpu':
    raise LatticeLibraryError('the host twin takes CPU tensors')
  if W.dtype not in (torch.float32, torch.bfloat16):
    W = W.float()
  return W.contiguous()


def _i32(x, B):
  return torch.as_tensor(x).to(torch.int32).reshape(B).contiguous()


def _problem(W, V, n, U):
  B, T = W.shape[0], W.shape[1]
  return Problem(B, T, V, n, U, LT_DTYPE_BF16 if W.dtype == torch.bfloat16 else LT_DTYPE_F32)


def set_num_threads(n):
  _check(lib().lt_cpu_set_num_threads(int(n)))


def num_threads():
  return lib().lt_cpu_num_threads()


def den_forward(W, num_frames, V, n, semiring, with_alpha=True):
  """lt_cpu_den_forward: (dist [B], alpha [B,T,C] or None)."""
  W = _weights(W)
  B, T, C = W.shape[0], W.shape[1], W.shape[2]
  dist = torch.empty([B], dtype=torch.float32)
  alpha = torch.empty([B, T, C], dtype=torch.float32) if with_alpha else None
  pb = _problem(W, V, n, 0)
  nf = _i32(num_frames, B)  # converted arguments stay referenced through the call
  _check(lib().lt_cpu_den_forward(ctypes.byref(pb), semiring, _ptr(W), _ptr(nf), _ptr(dist),
                                  _ptr(alpha)))
  return dist, alpha


def num_forward(W, num_frames, labels, num_labels, V, n, semiring, with_alpha=True):
  """lt_cpu_num_forward: (num [B], alpha_num [B,T,U+1] or None)."""
  W = _weights(W)
  B, T = W.shape[0], W.shape[1]
  labels = torch.as_tensor(labels).to(torch.int32).reshape(B, -1).contiguous()
  U = labels.shape[1]
  num = torch.empty([B], dtype=torch.float32)
  an = torch.empty([B, T, U + 1], dtype=torch.float32) if with_alpha else None
  pb = _problem(W, V, n, U)
  nf, nl = _i32(num_frames, B), _i32(num_labels, B)
  _check(lib().lt_cpu_num_forward(ctypes.byref(pb), semiring, _ptr(W), _ptr(nf), _ptr(labels),
                                  _ptr(nl), _ptr(num), _ptr(an)))
  return num, an


def den_backward(W, num_frames, log_z, alpha, V, n, grad=None):
  """lt_cpu_den_backward: dW [B,T,C,V+1] (W's dtype) = grad * den marginals."""
  W = _weights(W)
  B = W.shape[0]
  dW = torch.empty_like(W)
  pb = _problem(W, V, n, 0)
  g = None if grad is None else torch.as_tensor(grad, dtype=torch.float32).reshape(B).contiguous()
  nf = _i32(num_frames, B)
  lz, al = log_z.float().contiguous(), alpha.float().contiguous()
  _check(lib().lt_cpu_den_backward(ctypes.byref(pb), _ptr(W), _ptr(nf), _ptr(lz), _ptr(al),
                                   _ptr(g), _ptr(dW)))
  return dW


def loss_grad(W, num_frames, labels, num_labels, V, n, local_norm=False, grad=None,
              with_grad=True):
  """lt_cpu_loss_grad: (loss, log_z, num, dW or None); dW = grad * d loss / dW."""
  W = _weights(W)
  B = W.shape[0]
  labels = torch.as_tensor(labels).to(torch.int32).reshape(B, -1).contiguous()
  U = labels.shape[1]
  loss = torch.empty([B], dtype=torch.float32)
  log_z = torch.empty([B], dtype=torch.float32)
  num = torch.empty([B], dtype=torch.float32)
  dW = torch.empty_like(W) if with_grad else None
  g = None if grad is None else torch.as_tensor(grad, dtype=torch.float32).reshape(B).contiguous()
  pb = _problem(W, V, n, U)
  nf, nl = _i32(num_frames, B), _i32(num_labels, B)
  _check(lib().lt_cpu_loss_grad(ctypes.byref(pb), 1 if local_norm else 0, _ptr(W), _ptr(nf),
                                _ptr(labels), _ptr(nl), _ptr(g), _ptr(loss), _ptr(log_z),
                                _ptr(num), _ptr(dW)))
  return loss, log_z, num, dW


def viterbi(W, num_frames, V, n, label_convention, grad=None, with_arcs=False):
  """lt_cpu_viterbi: (labels [B,T] int64, path_weight [B], arcs or None)."""
  W = _weights(W)
  B, T = W.shape[0], W.shape[1]
  labels = torch.empty([B, T], dtype=torch.int64)
  weight = torch.empty([B], dtype=torch.float32)
  arcs = torch.empty_like(W) if with_arcs else None
  g = None if grad is None else torch.as_tensor(grad, dtype=torch.float32).reshape(B).contiguous()
  pb = _problem(W, V, n, 0)
  nf = _i32(num_frames, B)
  _check(lib().lt_cpu_viterbi(ctypes.byref(pb), _ptr(W), _ptr(nf),
                              int(label_convention), _ptr(labels), _ptr(weight), _ptr(g),
                              _ptr(arcs)))
  return labels, weight, arcs
