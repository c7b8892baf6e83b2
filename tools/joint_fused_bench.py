"""The JointWeightFn training step's kernels, fused against separate launches
(SURVEY.md 8(f) rank 1), at the bench lattice shape (T=1000, U=100, V=32):

  separate  lt_joint_weights_ex -> lt_loss_grad (its own design for B) ->
            lt_joint_weights_backward (W and dW through HBM)
  fused     lt_loss_grad_joint (W and dW never in HBM)

Both give the loss and d_ctx_proj / d_frame_proj / d_out_weight / d_out_bias
of sum(loss). One JSON line per (B, H, precision): ms per step (HIP events
over `reps` steps after warm-up), and the loss difference between the two.

    python tools/joint_fused_bench.py [--batches 64 256] [--hidden 32 64 128]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from last_torch_amd import _native as nat  # noqa: E402


def inputs(B, T, U, H, V, device, seed=0):
  g = torch.Generator(device=device).manual_seed(seed)
  C = R = V + 1
  pc = torch.randn([C, H], generator=g, device=device) * 0.5
  pf = torch.randn([B, T, H], generator=g, device=device) * 0.5
  wo = torch.randn([R, H], generator=g, device=device) * (2.0 / math.sqrt(H))
  bias = torch.randn([R], generator=g, device=device) * 0.1
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=device, dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device=device)
  nl = torch.full([B], U, dtype=torch.int32, device=device)
  return pc, pf, wo, bias, nf, lab, nl


def time_it(fn, reps, warmup):
  for _ in range(warmup):
    fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    out = fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps, out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--batches', type=int, nargs='+', default=[64, 256])
  ap.add_argument('--hidden', type=int, nargs='+', default=[32, 64, 128])
  ap.add_argument('--precision', nargs='+', default=['fp32'])
  ap.add_argument('--frames', type=int, default=1000)
  ap.add_argument('--labels', type=int, default=100)
  ap.add_argument('--reps', type=int, default=10)
  ap.add_argument('--warmup', type=int, default=3)
  args = ap.parse_args()
  dev = torch.device('cuda', 0)
  T, U, V = args.frames, args.labels, 32
  for B in args.batches:
    for H in args.hidden:
      for prec in args.precision:
        pc, pf, wo, bias, nf, lab, nl = inputs(B, T, U, H, V, dev)
        ws = torch.empty([sum(nat.joint_loss_workspace_bytes(B, T, U, V, H, prec))],
                         dtype=torch.uint8, device=dev)

        def fused():
          return nat.loss_grad_joint(pc, pf, wo, bias, nf, lab, nl, precision=prec, workspace=ws)

        lws = [None]

        def separate():
          W = nat.joint_weights(pc, pf, wo, bias, precision=prec)
          if lws[0] is None:
            lws[0] = torch.empty([nat.loss_grad_workspace_bytes(W, V, 1, U, False)],
                                 dtype=torch.uint8, device=dev)
          loss, _, _, dW = nat.loss_grad(W, nf, lab, nl, V, 1, False, workspace=lws[0])
          return (loss,) + nat.joint_weights_backward(pc, pf, wo, dW)

        ms_f, of = time_it(fused, args.reps, args.warmup)
        ms_s, os_ = time_it(separate, args.reps, args.warmup)
        rec = {'batch': B, 'frames': T, 'labels': U, 'vocab': V, 'hidden': H, 'precision': prec,
               'separate_ms': ms_s, 'fused_ms': ms_f, 'fused_over_separate': ms_f / ms_s,
               'separate_lattice_design': nat.DESIGN_NAMES[nat.loss_grad_design(B, T, U, V, 1)],
               'max_abs_loss_diff': float((of[0] - os_[0]).abs().max()),
               'max_rel_dwo_diff': float((of[5] - os_[3]).abs().max() / os_[3].abs().max())}
        print(json.dumps(rec), flush=True)
        del pc, pf, wo, bias, ws, lws
        torch.cuda.empty_cache()


if __name__ == '__main__':
  main()
