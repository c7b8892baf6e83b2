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
  assert len(declared) == 40, declared
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
  """One rank: its LPT shard through the product's CPU path
  (RecognitionLattice on host tensors -> cpu.py) with the arc weights as a
  trainable table, loss.sum().backward() into a GradBucket, then the step's
  one all-reduce; a second step after bucket.zero_grad()."""
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    import last_torch_amd as lt
    W, nf, lab, nl, V, n = payload
    idx = sharding.local_shard(torch.tensor(nf), rank, world)
    table = torch.nn.Parameter(torch.tensor(W[idx]))
    head = torch.nn.Parameter(torch.zeros(W.shape[-2:]))  # shared by every rank
    bucket = sharding.GradBucket([head])
    wfn = lt.weight_fns.TableWeightFn(table.detach())  # a plain tensor attribute
    lat = lt.RecognitionLattice(context=lt.contexts.FullNGram(vocab_size=V, context_size=n),
                                alignment=lt.alignments.FrameDependent(),
                                weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
                                weight_fn_factory=lambda _: wfn)
    T = W.shape[1]
    frames = torch.arange(T, dtype=torch.float32)[None, :, None].expand(len(idx), T, 1)
    totals, head_grads = [], []
    for _ in range(2):
      bucket.zero_grad()
      table.grad = None
      wfn.table = table + head
      loss = lat(frames, torch.tensor(nf[idx]), torch.tensor(lab[idx]), torch.tensor(nl[idx]))
      loss.sum().backward()
      assert head.grad.data_ptr() == bucket.flat[1:].data_ptr()
      totals.append(float(bucket.all_reduce_step(loss)))
      head_grads.append(head.grad.numpy().copy())
    # the functional form: a parameter used on rank 1 only gets the same
    # reduced .grad on both ranks (identical replica updates); with
    # skip_unused its .grad stays None on the rank that did not use it
    p = torch.nn.Parameter(torch.zeros(5))
    partial = torch.nn.Parameter(torch.zeros(3))
    p.grad = torch.full([5], float(rank + 1))
    if rank == 1:
      partial.grad = torch.tensor([1.0, 2.0, 3.0])
    total3 = float(sharding.all_reduce_step(loss, [p, partial]))
    skipped = torch.nn.Parameter(torch.zeros(2))
    if rank == 1:
      skipped.grad = torch.ones(2)
    sharding.all_reduce_step(loss, [skipped], skip_unused=True)
    skip_ok = (skipped.grad is None) if rank != 1 else bool((skipped.grad == 1).all())
    # a parameter no rank used keeps .grad None on every rank (weight decay /
    # momentum must not see a zero gradient for it)
    idle = torch.nn.Parameter(torch.zeros(4))
    sharding.all_reduce_step(loss, [idle])
    skip_ok = skip_ok and idle.grad is None
    out_q.put((rank, idx, loss.detach().numpy(), table.grad.numpy().copy(), totals, head_grads,
               p.grad.numpy().copy(), partial.grad.numpy().copy(), skip_ok, total3,
               bucket.calls))
  finally:
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_gloo_world2_sharded_loss_matches_full_batch(world):
  """world_size-2 (and 4) gloo: each rank's shard through the product's CPU
  path; per-shard losses and dW reassemble to the oracle's full batch, and the
  one all-reduce per step gives the global loss sum and the summed head
  gradient on every rank, on two consecutive steps (zero_grad between)."""
  from oracle import oracle as orc  # the checker
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
  port = 29500 + (os.getpid() % 2000) + 2100 * (world // 4)
  procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, (W, nf, lab, nl, V, n), q))
           for r in range(world)]
  for p in procs:
    p.start()
  res = [q.get(timeout=120) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  loss = np.zeros(B, np.float32)
  dW = np.zeros_like(full_dW)
  for rank, idx, l, g, totals, head_grads, pgrad, partial_grad, skip_ok, total3, calls in res:
    loss[idx] = l
    dW[idx] = g
    for total in totals + [total3]:
      np.testing.assert_allclose(total, full_loss.sum(), rtol=1e-5)
    # the head's gradient is the sum of every utterance's dW, on both steps
    for hg in head_grads:
      np.testing.assert_allclose(hg, full_dW.sum(axis=(0, 1)), atol=1e-5)
    np.testing.assert_array_equal(pgrad, np.full(5, world * (world + 1) / 2))  # 1 + ... + world
    np.testing.assert_array_equal(partial_grad, [1.0, 2.0, 3.0])  # same on both ranks
    assert skip_ok
    assert calls == 2  # one all-reduce per step
  np.testing.assert_allclose(loss, full_loss, rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(dW, full_dW, atol=1e-5)


def test_bench_launcher_n2_cpu():
  """bench.py --gpus 2 without a torch.distributed environment starts its
  own two ranks (torch.distributed.run as a child), every rank sees world
  size 2, the global batch is LPT-sharded, one all-reduce per step, one
  JSON line whose global loss sum is the oracle's."""
  import json
  import subprocess
  import sys
  from oracle import oracle as orc
  import bench
  env = dict(os.environ)
  env.pop('WORLD_SIZE', None)
  B, T, U, V = 3, 8, 3, 3
  out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--device', 'cpu', '--batch', str(B), '--frames', str(T), '--labels',
                        str(U), '--vocab', str(V), '--steps', '2', '--warmup', '1',
                        '--varlen'], capture_output=True, text=True, timeout=240, env=env,
                       cwd='/tmp')
  assert out.returncode == 0, out.stderr[-2000:]
  line = [x for x in out.stdout.splitlines() if x.startswith('{')]
  assert len(line) == 1, out.stdout
  r = json.loads(line[0])
  assert r['ranks'] == 2 and r['gloo_world_size'] == 2
  assert r['collectives_per_step'] == 1.0
  assert r['shard_sizes'] == [3, 3]
  nf, lab, nl = bench.global_batch(2 * B, T, U, V, 1234, True)
  W = bench.shard_weights(range(2 * B), T, V + 1, V, 'cpu', 1234).numpy()
  ref, _, _, _ = orc.loss_grad(W, nf.numpy(), lab.numpy(), nl.numpy(), V, 1, want_grad=False)
  np.testing.assert_allclose(r['global_loss_sum'], ref.sum(), rtol=1e-5)
  # a mismatched world is refused
  env2 = dict(env, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
  bad = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--device', 'cpu'], capture_output=True, text=True, timeout=120, env=env2,
                       cwd='/tmp')
  assert bad.returncode != 0 and 'WORLD_SIZE=1' in bad.stderr
