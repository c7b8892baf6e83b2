"""CPU checks of the C-ABI boundary and of the utterance-sharded N>1 path.

* liblt_lattice.so loads (no GPU needed) and exports every function
  include/lt_lattice.h declares; argument validation runs on the host and
  returns the documented error codes before any device work.
* world_size-2 gloo: each rank owns an LPT shard of the utterances; per-shard
  losses and dW reassemble exactly to the full batch, and the one
  all-reduce of the step gives the global loss sum.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from last_torch_amd import _native
from last_torch_amd import sharding

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'lt_lattice.h')


def _declared_functions():
  src = open(HEADER).read()
  src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
  return sorted(set(re.findall(r'\b(lt_[a-z_]+)\s*\(', src)))


def _header_define(name):
  m = re.search(rf'#define\s+{name}\s+\(?(-?\d+)\)?', open(HEADER).read())
  return int(m.group(1))


def test_library_exports_every_declared_symbol():
  declared = _declared_functions()
  assert len(declared) == 30, declared
  lib = _native.lib()
  for name in declared:
    assert hasattr(lib, name), f'{name} declared in lt_lattice.h but not exported'
  assert set(declared) == set(_native.EXPORTED)


def test_version_and_context_states():
  assert _native.version().startswith('last_torch_amd-lattice')
  lib = _native.lib()
  out = ctypes.c_int64(0)
  for V, n, C in [(32, 1, 33), (32, 2, 1057), (5, 0, 1), (2, 3, 15), (1, 4, 5)]:
    assert lib.lt_num_context_states(V, n, ctypes.byref(out)) == 0
    assert out.value == C
  assert lib.lt_num_context_states(0, 1, ctypes.byref(out)) == _header_define('LT_EINVAL')
  assert lib.lt_num_context_states(4, -1, ctypes.byref(out)) == _header_define('LT_EINVAL')
  assert lib.lt_num_context_states(1024, 3, ctypes.byref(out)) == \
      _header_define('LT_EUNSUPPORTED')


def test_host_validation_error_codes():
  lib = _native.lib()
  EINVAL = _header_define('LT_EINVAL')
  P = _native.Problem
  null = ctypes.c_void_p(0)
  assert lib.lt_den_forward(None, 0, null, null, null, null, null) == EINVAL
  assert b'null problem' in lib.lt_last_error()
  bad = P(batch=-1, max_frames=4, vocab_size=3, context_size=1, max_labels=0, weight_dtype=0)
  assert lib.lt_den_forward(ctypes.byref(bad), 0, null, null, null, null, null) == EINVAL
  assert b'negative' in lib.lt_last_error()
  bad = P(batch=2, max_frames=4, vocab_size=3, context_size=1, max_labels=0, weight_dtype=7)
  assert lib.lt_den_forward(ctypes.byref(bad), 0, null, null, null, null, null) == EINVAL
  ok = P(batch=2, max_frames=4, vocab_size=3, context_size=1, max_labels=2, weight_dtype=0)
  assert lib.lt_den_forward(ctypes.byref(ok), 9, null, null, null, null, null) == EINVAL
  assert lib.lt_den_forward(ctypes.byref(ok), 0, null, null, null, null, null) == EINVAL
  assert b'null pointer' in lib.lt_last_error()
  # an empty batch is a no-op that succeeds without touching a device
  empty = P(batch=0, max_frames=4, vocab_size=3, context_size=1, max_labels=2, weight_dtype=0)
  assert lib.lt_den_forward(ctypes.byref(empty), 0, null, null, null, null, null) == 0
  nbytes = ctypes.c_size_t(0)
  assert lib.lt_viterbi_workspace_bytes(ctypes.byref(ok), ctypes.byref(nbytes)) == 0
  assert nbytes.value >= 2 * 4 * 4


def test_lpt_shards_are_balanced_and_disjoint():
  rng = np.random.default_rng(0)
  nf = rng.integers(100, 1000, 64)
  for world in (1, 2, 3, 8):
    shards = sharding.shard_utterances(nf, world)
    allidx = np.concatenate(shards)
    assert sorted(allidx.tolist()) == list(range(64))
    sizes = [len(s) for s in shards]
    assert max(sizes) - min(sizes) <= 1
    loads = [int(nf[s].sum()) for s in shards]
    assert max(loads) - min(loads) <= nf.max(), loads


def _gloo_worker(rank, world, port, payload, out_q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from oracle import oracle as orc  # test infrastructure: the per-shard compute
    W, nf, lab, nl, V, n = payload
    idx = sharding.local_shard(torch.tensor(nf), rank, world)
    loss, _, _, dW = orc.loss_grad(W[idx], nf[idx], lab[idx], nl[idx], V, n)
    # a stand-in weight-fn parameter whose grad is exercised by the bucket
    p = torch.nn.Parameter(torch.zeros(5))
    p.grad = torch.full([5], float(rank + 1))
    total = sharding.all_reduce_step(torch.tensor(loss), [p])
    # the same exchange through a persistent bucket (grads are views of it)
    q = torch.nn.Parameter(torch.zeros(2, 3))
    bucket = sharding.GradBucket([q])
    q.grad.fill_(float(rank + 1))
    total2 = bucket.all_reduce_step(torch.tensor(loss))
    assert q.grad.data_ptr() == bucket.flat[1:].data_ptr()
    out_q.put((rank, idx, loss, dW, float(total), p.grad.numpy().copy(), float(total2),
               q.grad.numpy().copy()))
  finally:
    dist.destroy_process_group()


def test_gloo_world2_sharded_loss_matches_full_batch():
  from oracle import oracle as orc
  rng = np.random.default_rng(3)
  B, T, U, V, n = 6, 9, 3, 3, 1
  C = orc.num_states(V, n)
  W = rng.standard_normal((B, T, C, V + 1)).astype(np.float32)
  nf = np.array([9, 3, 7, 5, 8, 2], np.int32)
  lab = rng.integers(1, V + 1, (B, U)).astype(np.int32)
  nl = np.array([3, 1, 2, 2, 3, 0], np.int32)
  full_loss, _, _, full_dW = orc.loss_grad(W, nf, lab, nl, V, n)

  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = 29500 + (os.getpid() % 2000)
  procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, (W, nf, lab, nl, V, n), q))
           for r in range(2)]
  for p in procs:
    p.start()
  res = [q.get(timeout=120) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  loss = np.zeros(B, np.float32)
  dW = np.zeros_like(full_dW)
  for rank, idx, l, g, total, pgrad, total2, qgrad in res:
    loss[idx] = l
    dW[idx] = g
    np.testing.assert_allclose(total, full_loss.sum(), rtol=1e-6)
    np.testing.assert_array_equal(pgrad, np.full(5, 3.0))  # 1 + 2
    np.testing.assert_allclose(total2, full_loss.sum(), rtol=1e-6)
    np.testing.assert_array_equal(qgrad, np.full((2, 3), 3.0))
  np.testing.assert_array_equal(loss, full_loss)
  np.testing.assert_array_equal(dW, full_dW)
