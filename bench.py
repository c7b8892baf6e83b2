"""Benchmark: Log-semiring lattice forward-backward (loss + dW) on MI355X.

One step = one pass of the hot path over one batch of synthetic arc weights
already resident in HBM: lt_loss_grad, i.e. the loss and dW = d(sum
loss)/dW (what loss.sum().backward() needs). For the bigram it is the
chunked two-level scan (lt_chunk.hip: ck_ab_kernel -- the chunk transfers
with the boundary walks in the same launch -- then ck_marg_kernel, plus the frame-serial pair whose workgroups exit at once
unless an utterance is out of the fast path's range). For N > 1 the step
adds the single RCCL all-reduce of the summed loss.
--design checkpoints / recursion time the older two-call designs
(lt_loss_forward + lt_loss_backward).

Workload (BASELINE.json configs[1], weak-scaled per GPU as configs[2]):
B=64 utterances per GPU, T=1000 frames, U=100 labels, V=32, bigram FullNGram
(C=33 context states), fp32. Metric: nominal lattice cells/s = B*T*U*C / s.

Run: python bench.py [--gpus N --steps K --warmup W]
     python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from last_torch_amd import _native  # noqa: E402
from last_torch_amd import sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = 'lattice cells/s (B·T·U·|ctx|) at T=1000,U=100; 1/2/4/8-GPU scaling'


def algorithmic_bytes(T, U, V, C, es=4, checkpoints=True):
  """Per-frame HBM bytes each kernel must move.

  SURVEY.md 8d's design-independent step figure is
  F_fb = A_w(2 s_w + s_g) + 8C + (U+1)(4 s_w + 8) = 15,756 B/frame (bigram
  fp32, U=100); it is what hbm_frac_step is priced on.

  checkpointing design (default):
    loss_forward : alpha pass and beta pass each stream W (2 A_w s_w) and
                   write their checkpoints alpha, beta (8C) and alpha_num,
                   beta_num (8(U+1)); numerator gathers come from the LDS copy.
    loss_backward: marginal pass reads W, writes dW (2 A_w s_w) and reads the
                   four checkpoints (8C + 8(U+1)).
  recursion design (--no-checkpoints):
    loss_forward : A_w s_w + 4C + (U+1)(2 s_w + 4)
    loss_backward: 2 A_w s_w + 4C + (U+1)(2 s_w + 4)
  """
  Aw = C * (V + 1)
  if checkpoints:
    fwd = 2 * Aw * es + 8 * C + 8 * (U + 1)
    bwd = 2 * Aw * es + 8 * C + 8 * (U + 1)
  else:
    fwd = Aw * es + 4 * C + (U + 1) * (2 * es + 4)
    bwd = 2 * Aw * es + 4 * C + (U + 1) * (2 * es + 4)
  survey = Aw * 3 * es + 8 * C + (U + 1) * (4 * es + 8)
  return fwd, bwd, survey


def make_inputs(B, T, U, V, C, device, seed, dtype=torch.float32):
  g = torch.Generator(device=device)
  g.manual_seed(seed)
  W = torch.randn([B, T, C, V + 1], generator=g, device=device, dtype=torch.float32).to(dtype)
  labels = torch.randint(1, V + 1, [B, U], generator=g, device=device, dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device=device)
  nl = torch.full([B], U, dtype=torch.int32, device=device)
  return W, nf, labels, nl


def run_steps(W, nf, labels, nl, V, n, steps, warmup, dist_on, events=True, checkpoints=True,
              fused=False, settle_s=0.0, info=None):
  """Returns (wall seconds over `steps`, fwd ms list, bwd ms list, all-reduces
  issued). settle_s: untimed steps for that long before the `warmup` steps,
  while the GPU's clock settles under the load (info['settle_calls'] counts
  them); fused:
  lt_loss_grad in one C-ABI call (fwd list; bwd list empty), else
  lt_loss_forward (fwd list) + lt_loss_backward (bwd list)."""
  grad = torch.ones([W.shape[0]], dtype=torch.float32, device=W.device)
  ws = None
  if fused:
    nbytes = _native.loss_grad_workspace_bytes(W, V, n, labels.shape[-1], False)
    ws = torch.empty([max(nbytes, 1)], dtype=torch.uint8, device=W.device)
  # stand-in weight-fn projection head (512 x 33 fp32) so the
  # step's one collective carries [loss sum || parameter grads]
  head = torch.nn.Parameter(torch.zeros([512, 33], device=W.device))
  bucket = sharding.GradBucket([head], device=W.device)  # head.grad is a view of the bucket

  def step(ev=None):
    if ev is not None:
      ev[0].record()
    if fused:
      loss, _, _, dW = _native.loss_grad(W, nf, labels, nl, V, n, False, workspace=ws)
      if ev is not None:
        ev[1].record()
    else:
      out = _native.loss_forward(W, nf, labels, nl, V, n, False, checkpoints=checkpoints)
      loss, log_z, num, alpha, an = out[:5]
      if ev is not None:
        ev[1].record()
      dW = _native.loss_backward(W, nf, labels, nl, log_z, num, alpha, an, grad, V, n, False,
                                 ck=out[5] if checkpoints else None)
    if ev is not None:
      ev[2].record()
    if dist_on:
      bucket.all_reduce_step(loss)
    return dW

  # the shader clock under this load rises from ~2.2 to ~2.39 GHz over the
  # first 25-50 calls after an idle GPU (a probe beside the calls,
  # profiles/r05_warmup_probe.jsonl): the timed steps measure the sustained
  # rate, so the load runs until the clock has settled first
  settle_calls = 0
  t_settle = time.perf_counter()
  while time.perf_counter() - t_settle < settle_s:
    step()
    settle_calls += 1
    if settle_calls % 8 == 0:
      torch.cuda.synchronize()
  if info is not None:
    info['settle_calls'] = settle_calls
  for _ in range(warmup):
    step()
  torch.cuda.synchronize()
  if dist_on:
    torch.distributed.barrier()
  torch.cuda.synchronize()
  # one C-ABI call per step with no collective (N = 1): two HIP events around
  # the whole timed loop give the call's average (event records between the
  # calls cost the stream a few microseconds each); otherwise a pair per step
  # separates the call from the step's collective
  whole = events and fused and not dist_on
  evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)] \
      if events and not whole else [None] * steps
  ew = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if whole else None
  t0 = time.perf_counter()
  if whole:
    ew[0].record()
  for i in range(steps):
    step(evs[i])
  if whole:
    ew[1].record()
  torch.cuda.synchronize()
  if dist_on:
    torch.distributed.barrier()
  torch.cuda.synchronize()
  wall = time.perf_counter() - t0
  if whole:
    fwd_ms = [ew[0].elapsed_time(ew[1]) / steps] * steps
  else:
    fwd_ms = [e[0].elapsed_time(e[1]) for e in evs] if events else []
  bwd_ms = [e[1].elapsed_time(e[2]) for e in evs] if (events and not fused) else []
  return wall, fwd_ms, bwd_ms, bucket.calls


def weights_leg(B, T, U, V, n, C, device, reps=10):
  """The bench step on a trained model's kind of arc weights:
  log_softmax(sigma * randn) rows (weight_fns.py:120-136) for sigma 5 and
  10, and randn with one masked (-inf) arc per utterance
  (lattices.py:450-453): ms per lt_loss_grad call and the utterances that
  left the chunked fast path (its fallback flag words)."""
  out = {}
  g = torch.Generator(device=device)
  lab = torch.randint(1, V + 1, [B, U], generator=g.manual_seed(5), device=device,
                      dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device=device)
  nl = torch.full([B], U, dtype=torch.int32, device=device)
  for name in ('randn', 'logsoftmax_s5', 'logsoftmax_s10', 'neginf_arc'):
    W = torch.randn([B, T, C, V + 1], generator=g.manual_seed(6), device=device)
    if name.startswith('logsoftmax'):
      W = torch.log_softmax(float(name.split('_s')[1]) * W, dim=-1)
    elif name == 'neginf_arc':
      ar = torch.arange(B, device=device)
      W[ar, torch.randint(0, T, [B], generator=g, device=device),
        torch.randint(0, C, [B], generator=g, device=device),
        torch.randint(0, V + 1, [B], generator=g, device=device)] = -float('inf')
    ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, n, U, False)], dtype=torch.uint8,
                     device=device)
    for _ in range(2):
      _native.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
      _native.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    rec = {'ms_per_call': e0.elapsed_time(e1) / reps}
    if _native.loss_grad_design(B, T, U, V, n) == _native.DESIGN_CHUNK:
      rec['fallback_utterances'] = _native.chunk_fallback_count(ws, B)
    out[name] = rec
    del W, ws
  out['slowdown_logsoftmax_s10_vs_randn'] = (out['logsoftmax_s10']['ms_per_call'] /
                                             out['randn']['ms_per_call'])
  return out


def cold_w_leg(B, T, U, V, n, C, device, nbuf=3, reps=12):
  """lt_loss_grad with `nbuf` W buffers used in rotation:
  3 x 279 MB at B=64 cannot sit in the 256 MiB Infinity Cache, so each call
  reads its W from HBM. Reported beside the same call on one W (hot)."""
  lab = torch.randint(1, V + 1, [B, U], generator=torch.Generator(device=device).manual_seed(7),
                      device=device, dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device=device)
  nl = torch.full([B], U, dtype=torch.int32, device=device)
  Ws = [make_inputs(B, T, U, V, C, device, seed=300 + i)[0] for i in range(nbuf)]
  ws = torch.empty([_native.loss_grad_workspace_bytes(Ws[0], V, n, U, False)], dtype=torch.uint8,
                   device=device)
  out = {'buffers': nbuf, 'w_bytes_each': Ws[0].numel() * 4}
  for name, order in (('hot', [0] * reps), ('cold', [i % nbuf for i in range(reps)])):
    for i in range(nbuf):
      _native.loss_grad(Ws[i], nf, lab, nl, V, n, False, workspace=ws)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(True), torch.cuda.Event(True)) for _ in order]
    for (e0, e1), i in zip(evs, order):
      e0.record()
      _native.loss_grad(Ws[i], nf, lab, nl, V, n, False, workspace=ws)
      e1.record()
    torch.cuda.synchronize()
    out[f'{name}_ms_per_call'] = float(np.mean([a.elapsed_time(b) for a, b in evs]))
  out['cold_over_hot'] = out['cold_ms_per_call'] / out['hot_ms_per_call']
  del Ws, ws
  torch.cuda.empty_cache()
  return out


def joint_step_leg(T, U, V, n, device, B=64, F=256, H=512, reps=5):
  """a whole training step of RecognitionLattice driven
  by SharedEmbCacher + JointWeightFn (weight_fns.py:174-242) at the bench
  lattice shape, with the matrix-core producer (lt_joint_weights / _backward)
  and with the PyTorch hidden tensor; the lattice kernels are the same in
  both (tools/joint_step_bench.py has the H sweep)."""
  import last_torch_amd as lt
  torch.manual_seed(0)
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  cacher = lt.weight_fns.SharedEmbCacher(num_context_states=V + 1, embedding_size=128,
                                         device=device)
  wfn = lt.weight_fns.JointWeightFn(vocab_size=V, hidden_size=H, device=device)
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: cacher,
                              weight_fn_factory=lambda _: wfn)
  frames = torch.randn([B, T, F], device=device)
  nf = torch.full([B], T, device=device)
  labels = torch.randint(1, V + 1, [B, U], device=device)
  nl = torch.full([B], U, device=device)
  out = {'batch': B, 'frames': T, 'labels': U, 'features': F, 'hidden': H,
         'producer_precision': 'fp32-faithful split-bf16 products (JointWeightFn default)'}
  for name, fused, prec in (('producer', True, 'fp32'), ('producer_bf16', True, 'bf16'),
                            ('pytorch_hidden', False, 'fp32')):
    wfn.fused = fused
    wfn.precision = prec
    for _ in range(3):
      lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl).sum().backward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
      lat(frames=frames, num_frames=nf, labels=labels, num_labels=nl).sum().backward()
    e1.record()
    torch.cuda.synchronize()
    out[f'{name}_ms_per_step'] = e0.elapsed_time(e1) / reps
  out['speedup'] = out['pytorch_hidden_ms_per_step'] / out['producer_ms_per_step']
  return out


def cpu_ref(T, U, V, n, sample_utts):
  """SURVEY 8(d) cpu_ref: the reference's own CPU formulation -- PyTorch on
  the host, the per-frame recursion vectorised over the batch and the
  states, dW by autograd (last_torch_amd/cpu.py, the drop-in's CPU path) --
  at full thread count, on a bounded sample of the same workload."""
  import last_torch_amd as lt
  from last_torch_amd import cpu
  g = torch.Generator().manual_seed(0)
  W = torch.randn([sample_utts, T, V + 1, V + 1], generator=g).requires_grad_(True)
  nf = torch.full([sample_utts], T)
  lab = torch.randint(1, V + 1, (sample_utts, U), generator=g)
  nl = torch.full([sample_utts], U)
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  t0 = time.perf_counter()
  loss = cpu.loss(W, nf, lab, nl, ctx, lt.alignments.FrameDependent(), False)
  loss.sum().backward()
  dt = time.perf_counter() - t0
  C = V + 1
  return {
      'value': sample_utts * T * U * C / dt,
      'unit': 'cells/s',
      'cores': torch.get_num_threads(),
      'kind': 'port',
      'affinity_cores': len(os.sched_getaffinity(0)),
      'torch_threads': torch.get_num_threads(),
      'sample': (f'PyTorch CPU (last_torch_amd/cpu.py, the reference per-frame algorithm, '
                 f'fp32, autograd dW) loss+dW on {sample_utts} utterances of T={T} U={U} V={V} '
                 f'n={n}: {dt:.2f} s on {torch.get_num_threads()} threads'),
  }


def cpu_twin(T, U, V, n, C, sample_utts, min_seconds=10.0):
  """The C++ host twin of the library (liblt_lattice_cpu.so,
  include/lt_lattice_cpu.h: the same lattice, loss + dW, fp32, utterances
  over a host thread pool) on the same workload shape, timed on this box's
  host cores (at most 16 threads: the GPU box's CPU share)."""
  from last_torch_amd import _native_cpu
  threads = max(1, min(16, len(os.sched_getaffinity(0))))
  _native_cpu.set_num_threads(threads)
  g = torch.Generator().manual_seed(0)
  W = torch.randn([sample_utts, T, C, V + 1], generator=g)
  nf = torch.full([sample_utts], T, dtype=torch.int32)
  lab = torch.randint(1, V + 1, (sample_utts, U), generator=g, dtype=torch.int32)
  nl = torch.full([sample_utts], U, dtype=torch.int32)
  _native_cpu.loss_grad(W[:threads], nf[:threads], lab[:threads], nl[:threads], V, n)  # warm
  # passes over the sample until about 10 s of host work (16 threads x 10 s)
  passes, dt = 0, 0.0
  t0 = time.perf_counter()
  while passes < 1 or (dt < min_seconds and passes < 1000):
    _native_cpu.loss_grad(W, nf, lab, nl, V, n)
    passes += 1
    dt = time.perf_counter() - t0
  return {
      'value': passes * sample_utts * T * U * C / dt,
      'unit': 'cells/s',
      'cores': threads,
      'kind': 'port',
      'affinity_cores': len(os.sched_getaffinity(0)),
      'sample': (f'C++ host twin (last_torch_amd/liblt_lattice_cpu.so, lt_cpu_loss_grad: loss + '
                 f'dW, fp32) on {sample_utts} utterances of T={T} U={U} V={V} n={n}, '
                 f'{passes} passes: {dt:.2f} s on {threads} threads'),
  }


def cpu_baseline(T, U, V, n, C, sample_utts):
  """The C oracle (single-threaded restatement of the reference) on a
  bounded sample of the same workload: loss + dW for `sample_utts`
  utterances of shape (T, U, V, n)."""
  from oracle import oracle as orc
  rng = np.random.default_rng(0)
  W = rng.standard_normal((sample_utts, T, C, V + 1)).astype(np.float32)
  nf = np.full([sample_utts], T, np.int32)
  lab = rng.integers(1, V + 1, (sample_utts, U)).astype(np.int32)
  nl = np.full([sample_utts], U, np.int32)
  t0 = time.perf_counter()
  orc.loss_grad(W, nf, lab, nl, V, n)
  dt = time.perf_counter() - t0
  return {
      'value': sample_utts * T * U * C / dt,
      'unit': 'cells/s',
      'cores': 1,
      'kind': 'port',
      'sample': (f'oracle/lattice_oracle.c loss+dW (double precision, 1 thread) on '
                 f'{sample_utts} utterances of T={T} U={U} V={V} n={n}: {dt:.2f} s'),
  }


def read_traffic(profile_json, kernels, B, T):
  """HBM bytes per call summed over `kernels` (the launches one C-ABI call
  makes) from a committed PMC summary (profiles/*pmc*.json written by
  tools/pmc_summary.py), or None."""
  try:
    with open(profile_json) as f:
      d = json.load(f)
    total = 0.0
    for kernel in kernels:
      k = d['kernels'][kernel]
      if k.get('batch') != B or k.get('frames') != T or k['hbm_bytes_per_launch'] is None:
        return None
      total += k['hbm_bytes_per_launch']
    return total
  except (OSError, KeyError, ValueError, TypeError):
    return None


def chunk_design_bytes(T, U, V, L, es=4):
  """Per-frame HBM bytes the chunked design moves:
  W read by ck_ab_kernel and again by ck_marg_kernel, dW written once;
  per chunk of L frames a 1248-float record and the numerator group bands
  (NPG x 8 floats per 7-frame group) written by A and read by B; the
  boundary vectors written by B and read by C; the frame offsets c_t."""
  Aw = (V + 1) * (V + 1)
  NPG = (U + 2) & ~1
  CP = (V + 4) & ~3
  groups = -(-L // 7)
  rec = 1248 * 4 * 2 / L
  bands = ((groups * 8 * NPG + 31) & ~31) * 4 * 2 / L
  bound = 2 * (CP + NPG) * 4 * 2 / L
  return Aw * es * 3 + rec + bands + bound + 4 * 2


def chunk_len(B, T, U, V):
  """The chunk length lt_chunk.hip picks (its LDS budget, mirrored)."""
  FB = (V + 1) * (V + 1) * 4
  NPG = (U + 2) & ~1
  CP = (V + 4) & ~3
  al16 = lambda x: (x + 15) & ~15
  budget = 40 * 1024
  L = 32
  while True:
    n16 = (L * FB + 30) // 16
    b = ((n16 + 63) // 64) * 1024 + 2 * al16(4 * L * CP) + 2 * al16(4 * L * NPG) + \
        al16(8 * L * NPG) + al16(32 * L) + al16(8 * NPG + 4 * U) + al16(4 * L) + 1024 + al16(4 * (2 * L + 3))
    if L <= 4 or b <= budget:
      return L
    L -= 1


def loss_grad_design(B, T, U, V, n, C, device):
  """(kernel names, description, design bytes per frame) of the design
  lt_loss_grad dispatches to for this shape (lt_loss_grad_design)."""
  d = _native.loss_grad_design(B, T, U, V, n)
  if d == _native.DESIGN_CHUNK:
    L = chunk_len(B, T, U, V)
    fuse_ab = B <= torch.cuda.get_device_properties(device).multi_processor_count
    knames = ['ck_ab_kernel'] + ([] if fuse_ab else ['ck_combine_kernel']) + ['ck_marg_kernel']
    design = (f'chunked two-level scan, L={L} frames per chunk (lt_chunk.hip: '
              f"{' -> '.join(knames)})")
    return knames, design, chunk_design_bytes(T, U, V, L)
  ck_b = sum(algorithmic_bytes(T, U, V, C, checkpoints=True)[:2])
  if d == _native.DESIGN_FUSED_PIPE:
    return ['pipe_kernel'], 'lt_loss_grad (fused pipe)', ck_b
  if d == _native.DESIGN_CHECKPOINTS:
    knames = ['pipe_kernel' if _native.pipe_path(B, T, U, V, n) else 'fwdbwd_kernel',
              'marg_kernel']
    return knames, ('checkpointing: alpha || beta recursions with checkpoints, then the '
                    f"marginal pass ({' -> '.join(knames)})"), ck_b
  return ['fwd_kernel', 'bwd_kernel'], 'recursion backward', sum(
      algorithmic_bytes(T, U, V, C, checkpoints=False)[:2])


def launch_ranks(argv, n):
  """`--gpus N > 1` without a torch.distributed environment: start N ranks
  with torch.distributed.run as a CHILD process (one process per GPU, RCCL
  rendezvous on 127.0.0.1) and exit with its status. The parent never
  touches the GPU (no HIP call before or after), so nothing is exec'ed over
  an initialised device."""
  import socket
  import subprocess
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
         '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + argv
  return subprocess.call(cmd)


def global_batch(B_global, T, U, V, seed, varlen):
  """The step's global batch, the same on every rank: num_frames (T, or
  U[T/2, T] with --varlen), labels and num_labels, host tensors. Each rank
  keeps the LPT shard sharding.shard_utterances gives it."""
  g = torch.Generator().manual_seed(seed)
  if varlen:
    nf = torch.randint(T // 2, T + 1, [B_global], generator=g, dtype=torch.int32)
  else:
    nf = torch.full([B_global], T, dtype=torch.int32)
  labels = torch.randint(1, V + 1, [B_global, U], generator=g, dtype=torch.int32)
  nl = torch.full([B_global], U, dtype=torch.int32)
  return nf, labels, nl


def shard_weights(idx, T, C, V, device, seed):
  """Arc weights of the utterances `idx` of the global batch: utterance i
  from its own seeded stream (seed + i), so a rank materialises only its
  shard and every rank agrees on every utterance."""
  W = torch.empty([len(idx), T, C, V + 1], dtype=torch.float32, device=device)
  g = torch.Generator(device=device)
  for j, i in enumerate(idx):
    g.manual_seed(seed + int(i))
    W[j] = torch.randn([T, C, V + 1], generator=g, device=device)
  return W


def cpu_dist_step(args, world, rank):
  """--device cpu: the N > 1 control flow on host tensors with gloo (the
  CPU test of the launcher): each rank's LPT shard through the product's
  CPU path (RecognitionLattice on CPU tensors -> cpu.py), the loss into
  the GradBucket, one all-reduce per step; prints the same JSON line."""
  import last_torch_amd as lt
  B, T, U, V, n = args.batch, args.frames, args.labels, args.vocab, args.context
  C = lt.contexts.FullNGram(vocab_size=V, context_size=n).num_states()
  nf, lab, nl = global_batch(B * world, T, U, V, 1234, args.varlen)
  idx = sharding.local_shard(nf, rank, world)
  head = torch.nn.Parameter(torch.zeros([C, V + 1]))
  bucket = sharding.GradBucket([head])
  ctx = lt.contexts.FullNGram(vocab_size=V, context_size=n)
  W = shard_weights(idx, T, C, V, 'cpu', 1234)
  wfn = lt.weight_fns.TableWeightFn(W)
  lat = lt.RecognitionLattice(context=ctx, alignment=lt.alignments.FrameDependent(),
                              weight_fn_cacher_factory=lambda _: lt.weight_fns.NullCacher(),
                              weight_fn_factory=lambda _: wfn)
  frames = torch.arange(T, dtype=torch.float32)[None, :, None].expand(len(idx), T, 1)

  def step():
    bucket.zero_grad()
    wfn.table = W + head  # a stand-in trainable head on the arc weights
    loss = lat(frames, nf[idx], lab[idx], nl[idx])
    loss.sum().backward()
    return bucket.all_reduce_step(loss)

  for _ in range(args.warmup):
    step()
  torch.distributed.barrier()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    total = step()
  torch.distributed.barrier()
  wall = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
  torch.distributed.all_reduce(wall, op=torch.distributed.ReduceOp.MAX)
  cells = int(nf.sum()) * U * C
  if rank == 0:
    print(json.dumps({
        'metric': METRIC, 'value': cells * args.steps / float(wall), 'unit': 'cells/s',
        'n_gpus': 0, 'ranks': world, 'rccl_world_size': None,
        'gloo_world_size': torch.distributed.get_world_size(), 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': float(wall) / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'device': 'cpu',
        'collectives_per_step': bucket.calls / (args.steps + args.warmup),
        'global_loss_sum': float(total), 'shard_sizes': [len(s) for s in
                                                         sharding.shard_utterances(nf, world)],
        'head_grad_sum': float(head.grad.sum()),
    }), flush=True)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  # the defaults time the sustained rate (--settle-ms below: the clock under
  # load settles over the first 25-50 calls); 120 calls take < 0.1 s
  ap.add_argument('--steps', type=int, default=100)
  ap.add_argument('--warmup', type=int, default=20)
  ap.add_argument('--batch', type=int, default=64, help='utterances per GPU')
  ap.add_argument('--frames', type=int, default=1000)
  ap.add_argument('--labels', type=int, default=100)
  ap.add_argument('--vocab', type=int, default=32)
  ap.add_argument('--context', type=int, default=1)
  ap.add_argument('--varlen', action='store_true',
                  help='num_frames ~ U[T/2, T] over the global batch (LPT-sharded)')
  ap.add_argument('--device', choices=['cuda', 'cpu'], default='cuda',
                  help='cpu: the N > 1 control flow on host tensors with gloo (tests)')
  ap.add_argument('--cpu-utts', type=int, default=int(os.environ.get('LT_BENCH_CPU_UTTS', 128)),
                  help='utterances of the C-oracle baseline (0: skip)')
  ap.add_argument('--cpu-twin-utts', type=int,
                  default=int(os.environ.get('LT_BENCH_CPU_TWIN_UTTS', 64)),
                  help='utterances of the C++ host twin baseline (cpu_baseline; 0: skip)')
  ap.add_argument('--cpu-ref-utts', type=int,
                  default=int(os.environ.get('LT_BENCH_CPU_REF_UTTS', 8)),
                  help='utterances of the PyTorch-CPU cpu_ref baseline (0: skip)')
  ap.add_argument('--no-north-star', action='store_true')
  ap.add_argument('--no-joint', action='store_true')
  ap.add_argument('--no-weights', action='store_true',
                  help='skip the realistic-weights leg (log_softmax / masked arcs)')
  ap.add_argument('--design', choices=['auto', 'checkpoints', 'recursion'], default='auto',
                  help='auto: lt_loss_grad (the chunked scan for the bigram); checkpoints / '
                       'recursion: the two-call lt_loss_forward + lt_loss_backward designs')
  ap.add_argument('--settle-ms', type=float, default=60.0,
                  help='untimed calls for this long before the warmup steps, while the GPU clock '
                       'settles under the load (reported as settle_ms / settle_calls; 0: none)')
  ap.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'r05_pmc_summary.json'),
                  help='PMC summary (tools/pmc_summary.py) the traffic figure is read from')
  args = ap.parse_args()

  if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
    sys.exit(launch_ranks(sys.argv[1:], args.gpus))
  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local_rank = int(os.environ.get('LOCAL_RANK', '0'))
  if world != args.gpus:
    raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
  if args.device == 'cpu':
    torch.distributed.init_process_group('gloo')
    try:
      cpu_dist_step(args, world, rank)
    finally:
      torch.distributed.destroy_process_group()
    return
  # LT_BENCH_DIST=1: the N > 1 code path (RCCL init, barriers, the per-step
  # all-reduce, max-over-ranks timing) even with one rank, to exercise it on
  # a one-GPU box
  dist_on = world > 1 or os.environ.get('LT_BENCH_DIST', '0') == '1'
  torch.cuda.set_device(local_rank)
  device = torch.device('cuda', local_rank)
  rccl_world = None
  if dist_on:
    # RCCL logging: its version banner (NCCL_DEBUG=VERSION) is printed to
    # stdout, so the level is WARN and the log file stderr -- stdout carries
    # only the one JSON line the driver parses
    os.environ['NCCL_DEBUG'] = 'WARN'
    os.environ['NCCL_DEBUG_FILE'] = '/dev/stderr'
    torch.distributed.init_process_group('nccl', device_id=device)
    # the rank count RCCL itself sees: an all-reduce of ones
    ones = torch.ones([1], device=device)
    torch.distributed.all_reduce(ones)
    rccl_world = int(ones.item())
    if rccl_world != args.gpus or torch.distributed.get_world_size() != args.gpus:
      raise SystemExit(f'bench.py: RCCL sees {rccl_world} ranks, --gpus {args.gpus}')

  B, T, U, V, n = args.batch, args.frames, args.labels, args.vocab, args.context
  C = _native.num_context_states(V, n)
  # the global batch of B * N utterances, LPT-sharded; each rank
  # materialises its shard's arc weights only
  nf_g, lab_g, nl_g = global_batch(B * world, T, U, V, 1234, args.varlen)
  idx = sharding.local_shard(nf_g, rank, world)
  W = shard_weights(idx, T, C, V, device, 1234)
  nf, labels, nl = (x[idx].to(device) for x in (nf_g, lab_g, nl_g))
  fused = args.design == 'auto'
  ckpt = args.design == 'checkpoints'
  settle = {}
  wall, fwd_ms, bwd_ms, calls = run_steps(W, nf, labels, nl, V, n, args.steps, args.warmup,
                                          dist_on, checkpoints=ckpt, fused=fused,
                                          settle_s=args.settle_ms * 1e-3, info=settle)

  t = torch.tensor([wall], dtype=torch.float64, device=device)
  if dist_on:
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
  wall = float(t.item())
  # the units all ranks processed: every utterance's live frames
  cells_per_step = int(nf_g.sum()) * U * C
  value = cells_per_step * args.steps / wall

  fwd_b, bwd_b, survey_b = algorithmic_bytes(T, U, V, C, checkpoints=ckpt)
  if fused:
    call_s = float(np.mean(fwd_ms)) * 1e-3
    knames, design, design_b = loss_grad_design(len(idx), T, U, V, n, C, device)
    kernel = f"lt_loss_grad ({' + '.join(knames)})"
    kernels_ms = {'loss_grad': call_s * 1e3}
  else:
    fwd_avg = float(np.mean(fwd_ms)) * 1e-3
    bwd_avg = float(np.mean(bwd_ms)) * 1e-3
    call_s = fwd_avg + bwd_avg
    knames = ['fwd_kernel', 'bwd_kernel_ck' if ckpt else 'bwd_kernel', 'marg_kernel']
    design = 'checkpointing (alpha || beta, then marginal pass)' if ckpt else 'recursion backward'
    design_b = fwd_b + bwd_b
    kernel = 'lt_loss_forward + lt_loss_backward'
    kernels_ms = {'loss_forward': fwd_avg * 1e3, 'loss_backward': bwd_avg * 1e3}
  # roofline: SURVEY 8(d)'s design-independent bytes per frame for every
  # design (the design's own bytes are reported beside it), over the C-ABI
  # call's own duration (HIP events on the stream the kernels run on)
  frames_local = int(nf.sum())
  achieved = survey_b * frames_local / call_s / 1e9
  traffic = read_traffic(args.pmc, knames, len(idx), T)

  result = None
  if rank == 0:
    result = {
        'metric': METRIC,
        'value': value,
        'unit': 'cells/s',
        'n_gpus': world,
        'rccl_world_size': rccl_world,
        'steps': args.steps,
        'warmup': args.warmup,
        'settle_ms': args.settle_ms,
        'settle_calls': settle.get('settle_calls', 0),
        'ms_per_step': wall / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': ('synthetic (randn arc weights, uniform labels, '
                 f"{'U[T/2,T] lengths' if args.varlen else 'full-length utterances'}, "
                 'global batch LPT-sharded over the ranks)'),
        'config': {
            'workload': (f'Log-semiring forward-backward (loss + dW), B={B}/GPU, T={T}, '
                         f'U={U}, V={V}, FullNGram n={n} (C={C}), fp32 (BASELINE configs[1]; '
                         f'configs[2] at 8 GPUs)'),
            'batch_per_gpu': B, 'global_batch': B * world, 'frames': T, 'labels': U,
            'vocab': V, 'context_size': n, 'context_states': C,
            'parallelism': f'utterance-sharded x{world} (LPT), one RCCL all-reduce per step',
        },
        'collectives_per_step': (calls / (args.steps + args.warmup)) if dist_on else 0,
        'design': design,
        'kernels_ms': kernels_ms,
        'roofline': {
            'bound': 'hbm',
            'kernel': kernel,
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'traffic': traffic,
            'survey_bytes_per_frame': survey_b,
            'design_bytes_per_frame': design_b,
            'traffic_bytes_per_frame': traffic / frames_local if traffic else None,
        },
    }
    result['step_gbs'] = survey_b * int(nf_g.sum()) / (wall / args.steps) / 1e9
    result['hbm_frac_step'] = result['step_gbs'] / HBM_PEAK_GBS

  # north-star shape (B=256 on one GPU), measured in the same run at N=1
  if not dist_on and not args.no_north_star and B != 256:
    del W
    torch.cuda.empty_cache()
    W2, nf2, lab2, nl2 = make_inputs(256, T, U, V, C, device, seed=99)
    steps2 = max(5, args.steps // 2)
    # warmup calls: the freshly allocated 1.1 GB W's first passes run slower
    wall2, f2, b2, _ = run_steps(W2, nf2, lab2, nl2, V, n, steps2, max(5, args.warmup), False,
                                 checkpoints=ckpt, fused=fused, settle_s=args.settle_ms * 1e-3)
    ms2 = wall2 / steps2 * 1e3
    call2 = float(np.mean(f2)) + (float(np.mean(b2)) if b2 else 0.0)
    result['north_star_b256'] = {
        'value': 256 * T * U * C * steps2 / wall2,
        'ms_per_step': ms2,
        'ms_per_call': call2,
        'hbm_frac_step': survey_b * 256 * T / (ms2 * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'frac_call': survey_b * 256 * T / (call2 * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'design': (loss_grad_design(256, T, U, V, n, C, device)[1] if fused else
                   ('checkpoints' if ckpt else 'recursion')),
    }
    del W2
    torch.cuda.empty_cache()
    if not args.no_weights and fused:
      result['realistic_weights'] = weights_leg(B, T, U, V, n, C, device)
      result['cold_w'] = cold_w_leg(B, T, U, V, n, C, device)
    if not args.no_joint:
      result['joint_weight_fn_step'] = joint_step_leg(T, U, V, n, device)

  if rank == 0 and args.cpu_twin_utts > 0:
    # the C++ host twin beside every line, N > 1 included (rank 0, after the
    # timed steps, so the other ranks only wait at the final barrier): at
    # N > 1 a shorter sample (about 5 s), the same cells/s measure
    result['cpu_baseline'] = cpu_twin(T, U, V, n, C, args.cpu_twin_utts,
                                      min_seconds=10.0 if not dist_on else 5.0)
  if rank == 0 and not dist_on:
    if args.cpu_ref_utts > 0:
      result['cpu_baseline_torch'] = cpu_ref(T, U, V, n, args.cpu_ref_utts)
    if args.cpu_utts > 0:
      result['cpu_baseline_oracle'] = cpu_baseline(T, U, V, n, C, args.cpu_utts)
  if rank == 0:
    print(json.dumps(result), flush=True)
  if dist_on:
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
  main()
