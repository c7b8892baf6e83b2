"""Realistic arc weights on lt_loss_grad: time the bench
shape (B=64, T=1000, U=100, V=32 bigram fp32) with randn weights, with
log_softmax(sigma * randn) for several sigma, and with one -inf arc per
utterance; per variant the ms per call, the share of utterances that left
the chunked fast path (its uflag word) and, optionally, the per-element dW
error against the oracle relative to the arc marginals.

  python tools/weights_sweep.py [--err] [--batch 64] > gpurun_out/ws.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from last_torch_amd import _native as nat  # noqa: E402


def variant_weights(name, B, T, C, R, dev, seed):
  g = torch.Generator(device=dev)
  g.manual_seed(seed)
  W = torch.randn([B, T, C, R], generator=g, device=dev)
  if name.startswith('logsoftmax'):
    sigma = float(name.split('_s')[1])
    W = torch.log_softmax(sigma * W, dim=-1)
  elif name == 'neginf':
    t = torch.randint(0, T, [B], generator=g, device=dev)
    p = torch.randint(0, C, [B], generator=g, device=dev)
    y = torch.randint(0, R, [B], generator=g, device=dev)
    W[torch.arange(B, device=dev), t, p, y] = -float('inf')
  elif name == 'neginf_row':  # a whole label masked in one frame of every utterance
    t = torch.randint(0, T, [B], generator=g, device=dev)
    W[torch.arange(B, device=dev), t, :, 5] = -float('inf')
  return W.contiguous()


def time_call(W, nf, lab, nl, V, reps=20):
  ws = torch.empty([nat.loss_grad_workspace_bytes(W, V, 1, lab.shape[1], False)],
                   dtype=torch.uint8, device=W.device)
  for _ in range(3):
    out = nat.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    out = nat.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
  e1.record()
  torch.cuda.synchronize()
  fb = None
  if nat.loss_grad_design(W.shape[0], W.shape[1], lab.shape[1], V, 1) == nat.DESIGN_CHUNK:
    fb = int(ws[:4 * W.shape[0]].view(torch.int32).sum().item())
  return e0.elapsed_time(e1) / reps, fb, out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--batch', type=int, default=64)
  ap.add_argument('--frames', type=int, default=1000)
  ap.add_argument('--err', action='store_true', help='per-element dW error vs the oracle')
  ap.add_argument('--variants', default='randn,logsoftmax_s1,logsoftmax_s5,logsoftmax_s10,'
                                        'logsoftmax_s20,neginf,neginf_row')
  args = ap.parse_args()
  dev = torch.device('cuda', 0)
  B, T, U, V = args.batch, args.frames, 100, 32
  C = R = V + 1
  g = torch.Generator(device=dev)
  g.manual_seed(1)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=dev, dtype=torch.int32)
  nf = torch.full([B], T, dtype=torch.int32, device=dev)
  nl = torch.full([B], U, dtype=torch.int32, device=dev)
  for name in args.variants.split(','):
    W = variant_weights(name, B, T, C, R, dev, seed=1234)
    ms, fb, (loss, lz, num, dW) = time_call(W, nf, lab, nl, V)
    rec = {'variant': name, 'batch': B, 'frames': T, 'ms_per_call': ms, 'fallback_utts': fb,
           'design': nat.DESIGN_NAMES[nat.loss_grad_design(B, T, U, V, 1)],
           'range_mean': float((W.amax((-1, -2)) - W.amin((-1, -2))).clamp(max=1e9).mean())}
    if args.err:
      from golden_cases import grad_error_ratio
      from oracle import oracle as orc
      idx = list(range(0, B, max(1, B // 8)))
      Wc = W[idx].cpu().numpy()
      rl, rlz, rnum, rdW = orc.loss_grad(Wc, nf[idx].cpu().numpy(), lab[idx].cpu().numpy(),
                                         nl[idx].cpu().numpy(), V, 1)
      _, den = orc.den_grad(Wc, nf[idx].cpu().numpy(), V, 1)
      r = grad_error_ratio(dW[idx].cpu().numpy(), rdW, den, rlz, rnum)
      rec['err_ratio_max'] = float(r.max())
      rec['err_ratio_p999'] = float(np.quantile(r, 0.999))
      rec['loss_err_max'] = float(np.max(np.abs(loss[idx].cpu().numpy() - rl) /
                                         np.maximum(1, np.abs(rl))))
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
  main()
