"""ctypes front end of the C oracle (lattice_oracle.c) -- TEST INFRASTRUCTURE.

Every function takes and returns numpy arrays. Arc weights W are float32
[B, T, C, V+1] (blank at [..., 0], label y at [..., y]); lengths and labels
are int32. See lattice_oracle.c for the reference file:line each step
restates. Not used by the product path (last_torch_amd).
"""
import ctypes
import os
import subprocess

import numpy as np

LOG, MAX, REAL = 0, 1, 2
_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, 'build', 'liblt_oracle.so')
_lib = None

_F = np.ctypeslib.ndpointer(dtype=np.float32, flags='C_CONTIGUOUS')
_I = np.ctypeslib.ndpointer(dtype=np.int32, flags='C_CONTIGUOUS')
_L = np.ctypeslib.ndpointer(dtype=np.int64, flags='C_CONTIGUOUS')
_c_int = ctypes.c_int


def build():
  """Compiles the oracle with make (gcc)."""
  subprocess.run(['make', '-s', '-C', _HERE], check=True)


def lib():
  global _lib
  if _lib is None:
    if not os.path.exists(_LIB_PATH):
      build()
    l = ctypes.CDLL(_LIB_PATH)
    l.orc_num_states.argtypes = [_c_int, _c_int]
    l.orc_num_states.restype = _c_int
    l.orc_next_state.argtypes = [_c_int] * 4
    l.orc_next_state.restype = _c_int
    l.orc_den_forward.argtypes = [_c_int] * 4 + [_F, _I, _c_int, _F, ctypes.c_void_p]
    l.orc_num_forward.argtypes = [_c_int] * 5 + [_F, _I, _I, _I, _c_int, _F, ctypes.c_void_p]
    l.orc_viterbi.argtypes = [_c_int] * 4 + [_F, _I, _c_int, _L, _F, ctypes.c_void_p]
    l.orc_den_grad.argtypes = [_c_int] * 4 + [_F, _I, ctypes.c_void_p, _F, _F]
    l.orc_loss_grad.argtypes = ([_c_int] * 5 + [_F, _I, _I, _I, _c_int, ctypes.c_void_p, _F,
                                                 _F, _F, ctypes.c_void_p])
    for f in ('orc_den_forward', 'orc_num_forward', 'orc_viterbi', 'orc_den_grad',
              'orc_loss_grad'):
      getattr(l, f).restype = None
    # table_oracle.c: any next-state table, FrameDependent (K=0) or
    # FrameLabelDependent(K)
    l.tab_den_forward.argtypes = [_c_int] * 5 + [_I, _F, _I, _c_int, _F, ctypes.c_void_p]
    l.tab_num_forward.argtypes = [_c_int] * 6 + [_I, _F, _I, _I, _I, _c_int, _F]
    l.tab_loss_grad.argtypes = ([_c_int] * 6 + [_I, _F, _I, _I, _I, _c_int, ctypes.c_void_p,
                                                 _F, _F, _F, ctypes.c_void_p])
    l.tab_viterbi.argtypes = [_c_int] * 5 + [_I, _F, _I, _c_int, _L, _F]
    l.tab_den_grad.argtypes = [_c_int] * 5 + [_I, _F, _I, _F, _F]
    l.tab_dist_grad.argtypes = ([_c_int] * 6 + [_I, _F, _I, ctypes.c_void_p, ctypes.c_void_p,
                                                 _c_int, _c_int, ctypes.c_void_p, _F, _F])
    for f in ('tab_den_forward', 'tab_num_forward', 'tab_loss_grad', 'tab_viterbi',
              'tab_den_grad', 'tab_dist_grad'):
      getattr(l, f).restype = None
    _lib = l
  return _lib


def _f32(x):
  return np.ascontiguousarray(x, dtype=np.float32)


def _i32(x):
  return np.ascontiguousarray(x, dtype=np.int32)


def _ptr(x):
  return None if x is None else x.ctypes.data_as(ctypes.c_void_p)


def num_states(V, n):
  return lib().orc_num_states(V, n)


def next_state(V, n, state, label):
  return lib().orc_next_state(V, n, state, label)


def _dims(W, V):
  W = _f32(W)
  B, T, C, R = W.shape
  assert R == V + 1, (W.shape, V)
  return W, B, T, C


def den_forward(W, num_frames, V, n, semiring=LOG, want_alpha=True):
  """_forward (lattices.py:379-496): returns (dist [B], alpha [B,T,C])."""
  W, B, T, C = _dims(W, V)
  assert C == num_states(V, n)
  nf = _i32(num_frames)
  dist = np.zeros([B], np.float32)
  alpha = np.zeros([B, T, C], np.float32) if want_alpha else None
  lib().orc_den_forward(B, T, V, n, W, nf, semiring, dist, _ptr(alpha))
  return dist, alpha


def num_forward(W, num_frames, labels, num_labels, V, n, semiring=LOG, want_alpha=True):
  """_string_forward (lattices.py:250-377): returns (num [B], alpha [B,T,U+1])."""
  W, B, T, C = _dims(W, V)
  labels = _i32(labels).reshape(B, -1)
  U = labels.shape[1]
  num = np.zeros([B], np.float32)
  an = np.zeros([B, T, U + 1], np.float32) if want_alpha else None
  lib().orc_num_forward(B, T, U, V, n, W, _i32(num_frames), labels, _i32(num_labels),
                        semiring, num, _ptr(an))
  return num, an


def viterbi(W, num_frames, V, n, convention=1, want_arcs=False):
  """shortest_path (lattices.py:185-247) per utterance: (labels, weights, arcs)."""
  W, B, T, C = _dims(W, V)
  labels = np.zeros([B, T], np.int64)
  weight = np.zeros([B], np.float32)
  arcs = np.zeros(W.shape, np.float32) if want_arcs else None
  lib().orc_viterbi(B, T, V, n, W, _i32(num_frames), convention, labels, weight, _ptr(arcs))
  return labels, weight, arcs


def den_grad(W, num_frames, V, n, grad=None):
  """(log_z [B], d log_z / dW [B,T,C,V+1]) via correct-order FrameDependent.backward."""
  W, B, T, C = _dims(W, V)
  log_z = np.zeros([B], np.float32)
  dW = np.zeros(W.shape, np.float32)
  g = None if grad is None else _f32(grad)
  lib().orc_den_grad(B, T, V, n, W, _i32(num_frames), _ptr(g), log_z, dW)
  return log_z, dW


def loss_grad(W, num_frames, labels, num_labels, V, n, local_norm=False, grad=None,
              want_grad=True):
  """RecognitionLattice.forward loss and d loss / dW: (loss, log_z, num, dW)."""
  W, B, T, C = _dims(W, V)
  labels = _i32(labels).reshape(B, -1)
  U = labels.shape[1]
  loss = np.zeros([B], np.float32)
  log_z = np.zeros([B], np.float32)
  num = np.zeros([B], np.float32)
  dW = np.zeros(W.shape, np.float32) if want_grad else None
  g = None if grad is None else _f32(grad)
  lib().orc_loss_grad(B, T, U, V, n, W, _i32(num_frames), labels, _i32(num_labels),
                      int(bool(local_norm)), _ptr(g), loss, log_z, num, _ptr(dW))
  return loss, log_z, num, dW


# ---------------------------------------------------------------------------
# table_oracle.c: arbitrary next-state tables and FrameLabelDependent(K)
# ---------------------------------------------------------------------------
def full_ngram_table(V, n):
  """FullNGram.next_state_table() (contexts.py:258-263): [C, V] int32,
  entry [p, y-1] = next_state(p, y)."""
  C = num_states(V, n)
  return np.array([[next_state(V, n, p, y) for y in range(1, V + 1)] for p in range(C)],
                  np.int32)


def _tab(table, W):
  table = _i32(table)
  W = _f32(W)
  C, V = table.shape
  B, T = W.shape[:2]
  assert W.shape[2:] == (C, V + 1), (W.shape, table.shape)
  return table, W, B, T, C, V


def tab_den_forward(table, W, num_frames, K, semiring=LOG, want_alpha=False):
  table, W, B, T, C, V = _tab(table, W)
  dist = np.zeros([B], np.float32)
  alpha = np.zeros([B, T, C], np.float32) if want_alpha else None
  lib().tab_den_forward(B, T, C, V, K, table, W, _i32(num_frames), semiring, dist, _ptr(alpha))
  return (dist, alpha) if want_alpha else dist


def tab_num_forward(table, W, num_frames, labels, num_labels, K, semiring=LOG):
  table, W, B, T, C, V = _tab(table, W)
  labels = _i32(labels)
  U = labels.shape[1]
  num = np.zeros([B], np.float32)
  lib().tab_num_forward(B, T, U, C, V, K, table, W, _i32(num_frames), labels, _i32(num_labels),
                        semiring, num)
  return num


def tab_loss_grad(table, W, num_frames, labels, num_labels, K, local_norm=False, grad=None):
  """(loss, log_z, num, dW) for any next-state table and alignment K."""
  table, W, B, T, C, V = _tab(table, W)
  labels = _i32(labels)
  U = labels.shape[1]
  loss, lz, num = (np.zeros([B], np.float32) for _ in range(3))
  dW = np.zeros_like(W)
  g = None if grad is None else _f32(grad)
  lib().tab_loss_grad(B, T, U, C, V, K, table, W, _i32(num_frames), labels, _i32(num_labels),
                      int(bool(local_norm)), _ptr(g), loss, lz, num, _ptr(dW))
  return loss, lz, num, dW


def tab_den_grad(table, W, num_frames, K):
  """(log_z [B], d log_z / dW [B,T,C,V+1]): the denominator's arc marginals
  for any next-state table and alignment K."""
  table, W, B, T, C, V = _tab(table, W)
  lz = np.zeros([B], np.float32)
  dW = np.zeros_like(W)
  lib().tab_den_grad(B, T, C, V, K, table, W, _i32(num_frames), lz, dW)
  return lz, dW


def tab_viterbi(table, W, num_frames, K, convention=1):
  """(labels int64 [B, T*A], path weights [B]); A = 1 (K = 0) or K + 1."""
  table, W, B, T, C, V = _tab(table, W)
  A = 1 if K == 0 else K + 1
  labels = np.zeros([B, T * A], np.int64)
  weight = np.zeros([B], np.float32)
  lib().tab_viterbi(B, T, C, V, K, table, W, _i32(num_frames), convention, labels, weight)
  return labels, weight


def tab_dist_grad(table, W, num_frames, K, semiring, labels=None, num_labels=None, grad=None):
  """(dist [B], d dist / dW [B,T,C,V+1]) under `semiring` for any next-state
  table and alignment K: the denominator (_forward, lattices.py:379-496) when
  `labels` is None, else the numerator (_string_forward, lattices.py:250-377).
  Log: the arc marginals; MaxTropical: `grad` on the first-maximum path's
  arcs (semirings.py:354-401); Real: alpha * beta' (semirings.py:143-173)."""
  table, W, B, T, C, V = _tab(table, W)
  string = labels is not None
  lab = _i32(labels) if string else None
  U = lab.shape[1] if string else 0
  nl = _i32(num_labels) if string else None
  dist = np.zeros([B], np.float32)
  dW = np.zeros_like(W)
  g = None if grad is None else _f32(grad)
  lib().tab_dist_grad(B, T, U, C, V, K, table, W, _i32(num_frames), _ptr(lab), _ptr(nl),
                      semiring, int(string), _ptr(g), dist, dW)
  return dist, dW
