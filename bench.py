"""Benchmark: Log-semiring lattice forward-backward (loss + dW) on MI355X.

One step = one pass of the hot path over one batch of synthetic arc weights
already resident in HBM: lt_loss_grad (loss and dW = d(sum loss)/dW; for the
bigram at B=64 ONE launch in which the alpha and beta recursions run while
other workgroups turn every frame both have passed into arc marginals), then
lt_scale_grad with the incoming gradient (ones), plus, for N > 1, the single
RCCL all-reduce of the summed loss. --design checkpoints /
recursion time the two-call designs (lt_loss_forward + lt_loss_backward).

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
              fused=False):
  """Returns (wall seconds over `steps`, fwd kernel ms list, bwd kernel ms list);
  fused: lt_loss_grad (fwd list) + lt_scale_grad (bwd list)."""
  grad = torch.ones([W.shape[0]], dtype=torch.float32, device=W.device)
  ws = None
  if fused:
    nbytes = _native.loss_grad_workspace_bytes(W, V, n, labels.shape[-1], False)
    ws = torch.empty([max(nbytes, 1)], dtype=torch.uint8, device=W.device)
  # stand-in weight-fn projection head (512 x 33 fp32) so the
  # step's one collective carries [loss sum || parameter grads]
  head = torch.nn.Parameter(torch.zeros([512, 33], device=W.device))
  head.grad = torch.zeros_like(head)

  def step(ev=None):
    if ev is not None:
      ev[0].record()
    if fused:
      loss, _, _, dW = _native.loss_grad(W, nf, labels, nl, V, n, False, workspace=ws)
      if ev is not None:
        ev[1].record()
      _native.scale_grad(dW, grad, V, n)
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
      sharding.all_reduce_step(loss, [head])
    return dW

  for _ in range(warmup):
    step()
  torch.cuda.synchronize()
  if dist_on:
    torch.distributed.barrier()
  torch.cuda.synchronize()
  evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)] \
      if events else [None] * steps
  t0 = time.perf_counter()
  for i in range(steps):
    step(evs[i])
  torch.cuda.synchronize()
  if dist_on:
    torch.distributed.barrier()
  torch.cuda.synchronize()
  wall = time.perf_counter() - t0
  fwd_ms = [e[0].elapsed_time(e[1]) for e in evs] if events else []
  bwd_ms = [e[1].elapsed_time(e[2]) for e in evs] if events else []
  return wall, fwd_ms, bwd_ms


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
  out = {'batch': B, 'frames': T, 'labels': U, 'features': F, 'hidden': H}
  for name, fused in (('producer', True), ('pytorch_hidden', False)):
    wfn.fused = fused
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


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=20)
  ap.add_argument('--warmup', type=int, default=3)
  ap.add_argument('--batch', type=int, default=64, help='utterances per GPU')
  ap.add_argument('--frames', type=int, default=1000)
  ap.add_argument('--labels', type=int, default=100)
  ap.add_argument('--vocab', type=int, default=32)
  ap.add_argument('--context', type=int, default=1)
  ap.add_argument('--cpu-utts', type=int, default=int(os.environ.get('LT_BENCH_CPU_UTTS', 512)))
  ap.add_argument('--no-north-star', action='store_true')
  ap.add_argument('--design', choices=['auto', 'checkpoints', 'recursion'], default='auto',
                  help='auto: lt_loss_grad (one fused launch where eligible, else the '
                       'library policy below); checkpoints: lt_loss_forward with the '
                       'concurrent beta pass + lt_loss_backward marginal pass; recursion: '
                       'lt_loss_forward + beta recursion with fused marginals')
  ap.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'r01_pmc_summary.json'),
                  help='PMC summary of the checkpointing design; *_fused.json / '
                       '*_recursion.json for the others')
  args = ap.parse_args()

  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local_rank = int(os.environ.get('LOCAL_RANK', '0'))
  dist_on = world > 1
  torch.cuda.set_device(local_rank)
  device = torch.device('cuda', local_rank)
  if dist_on:
    torch.distributed.init_process_group('nccl', device_id=device)

  B, T, U, V, n = args.batch, args.frames, args.labels, args.vocab, args.context
  C = _native.num_context_states(V, n)
  W, nf, labels, nl = make_inputs(B, T, U, V, C, device, seed=1234 + rank)
  ckpt = (_native.prefer_checkpoints(B, device, (T, U, V, n, False)) if args.design == 'auto'
          else args.design == 'checkpoints')
  fused = args.design == 'auto' and _native.fused_path(B, T, U, V, n, device)
  wall, fwd_ms, bwd_ms = run_steps(W, nf, labels, nl, V, n, args.steps, args.warmup, dist_on,
                                   checkpoints=ckpt, fused=fused)

  t = torch.tensor([wall], dtype=torch.float64, device=device)
  if dist_on:
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
  wall = float(t.item())
  cells_per_step = world * B * T * U * C
  value = cells_per_step * args.steps / wall

  fwd_b, bwd_b, survey_b = algorithmic_bytes(T, U, V, C, checkpoints=ckpt)
  fwd_avg = float(np.mean(fwd_ms)) * 1e-3
  bwd_avg = float(np.mean(bwd_ms)) * 1e-3
  if fused:  # one launch does both passes' work (fwd list = lt_loss_grad)
    fwd_b, bwd_b = fwd_b + bwd_b, 0
  dominant, dom_bytes, dom_s = ('loss_backward', bwd_b * B * T, bwd_avg) \
      if bwd_avg >= fwd_avg else ('loss_forward', fwd_b * B * T, fwd_avg)
  achieved = dom_bytes / dom_s / 1e9
  if fused:
    dominant = 'loss_grad'
    knames = ['pipe_kernel']
  elif ckpt:
    fk = (['pipe_kernel'] if _native.pipe_path(B, T, U, V, n)
          else ['fwd_kernel', 'bwd_kernel_ck'])
    knames = ['marg_kernel'] if dominant == 'loss_backward' else fk
  else:
    knames = ['bwd_kernel'] if dominant == 'loss_backward' else ['fwd_kernel']
  pmc = (args.pmc.replace('.json', '_fused.json') if fused else
         args.pmc if ckpt else args.pmc.replace('.json', '_recursion.json'))
  traffic = read_traffic(pmc, knames, B, T)

  result = None
  if rank == 0:
    result = {
        'metric': METRIC,
        'value': value,
        'unit': 'cells/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': wall / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic (randn arc weights, uniform labels, full-length utterances)',
        'config': {
            'workload': (f'Log-semiring forward-backward (loss + dW), B={B}/GPU, T={T}, '
                         f'U={U}, V={V}, FullNGram n={n} (C={C}), fp32 (BASELINE configs[1]; '
                         f'configs[2] at 8 GPUs)'),
            'batch_per_gpu': B, 'global_batch': B * world, 'frames': T, 'labels': U,
            'vocab': V, 'context_size': n, 'context_states': C,
            'parallelism': f'utterance-sharded x{world}, RCCL all-reduce of summed loss',
        },
        'kernels_ms': ({'loss_grad': fwd_avg * 1e3, 'scale_grad': bwd_avg * 1e3} if fused else
                       {'loss_forward': fwd_avg * 1e3, 'loss_backward': bwd_avg * 1e3}),
        'roofline': {
            'bound': 'hbm',
            'kernel': f"{dominant} ({' || '.join(knames)})",
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'traffic': traffic,
            'algorithmic_bytes_per_frame': {'loss_forward': fwd_b, 'loss_backward': bwd_b,
                                            'survey_step': survey_b},
        },
        'design': ('fused (alpha || beta recursions with concurrent marginal workgroups, '
                   'one launch)' if fused else
                   'checkpointing (alpha || beta, then marginal pass)' if ckpt
                   else 'recursion backward'),
    }
    result['step_gbs'] = survey_b * B * T * world / (wall / args.steps) / 1e9
    result['hbm_frac_step'] = result['step_gbs'] / HBM_PEAK_GBS

  # north-star shape (B=256 on one GPU), measured in the same run at N=1
  if not dist_on and not args.no_north_star and B != 256:
    del W
    torch.cuda.empty_cache()
    W2, nf2, lab2, nl2 = make_inputs(256, T, U, V, C, device, seed=99)
    steps2 = max(5, args.steps // 2)
    ck2 = (_native.prefer_checkpoints(256, device, (T, U, V, n, False)) if args.design == 'auto'
           else args.design == 'checkpoints')
    wall2, f2, b2 = run_steps(W2, nf2, lab2, nl2, V, n, steps2, 2, False, checkpoints=ck2)
    fb2, bb2, _ = algorithmic_bytes(T, U, V, C, checkpoints=ck2)
    ms2 = wall2 / steps2 * 1e3
    result['north_star_b256'] = {
        'value': 256 * T * U * C * steps2 / wall2,
        'ms_per_step': ms2,
        'hbm_frac_step': survey_b * 256 * T / (ms2 * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'kernels_ms': {'loss_forward': float(np.mean(f2)), 'loss_backward': float(np.mean(b2))},
        'frac_loss_backward': bb2 * 256 * T / (float(np.mean(b2)) * 1e-3) / 1e9 / HBM_PEAK_GBS,
        'design': 'checkpoints' if ck2 else 'recursion',
    }
    del W2
    torch.cuda.empty_cache()
    result['joint_weight_fn_step'] = joint_step_leg(T, U, V, n, device)

  if rank == 0 and not dist_on and args.cpu_utts > 0:
    result['cpu_baseline'] = cpu_baseline(T, U, V, n, C, args.cpu_utts)
  if rank == 0:
    print(json.dumps(result), flush=True)
  if dist_on:
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
  main()
