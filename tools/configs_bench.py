"""Times the SURVEY.md 8(d) configurations that are not bench.py's line, one
JSON line each (HIP events around the C-ABI call; inputs resident in HBM):

  cfg4  MaxTropical Viterbi (lt_viterbi), B=64 T=2000 V=32 bigram, fp32;
        algorithmic bytes A_w*s_w + C + 5 = 4,394 B/frame (8d)
  cfg5  trigram bf16 loss + dW (lt_loss_grad), B=32 T=1000 U=100 V=32 n=2;
        219,358 B/frame (8d)
  cfg2  the bench line's shape, for reference (lt_loss_grad, fused)
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

PEAK = 8000.0  # GB/s


def timeit(fn, reps=10):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def inputs(B, T, U, V, n, dtype, seed=0):
  C = nat.num_context_states(V, n)
  g = torch.Generator(device='cuda')
  g.manual_seed(seed)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(dtype)
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, max(U, 1)), generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  return C, W, nf, lab[:, :U].contiguous(), nl


def report(name, B, T, U, C, ms, bytes_per_frame, dtype, call):
  gbs = bytes_per_frame * B * T / (ms * 1e-3) / 1e9
  print(json.dumps({'config': name, 'call': call, 'B': B, 'T': T, 'U': U, 'C': C,
                    'dtype': dtype, 'ms': ms, 'cells_per_s': B * T * max(U, 1) * C / (ms * 1e-3),
                    'algorithmic_bytes_per_frame': bytes_per_frame, 'achieved_GBps': gbs,
                    'frac_of_8TBps': gbs / PEAK}), flush=True)


def main():
  # cfg4: Viterbi, bit-exact labels (tests/test_gpu_parity.py)
  B, T, V, n = 64, 2000, 32, 1
  C, W, nf, _, _ = inputs(B, T, 0, V, n, torch.float32)
  ms = timeit(lambda: nat.viterbi(W, nf, V, n, nat.LABELS_REFERENCE))
  report('cfg4 Viterbi', B, T, 0, C, ms, C * (V + 1) * 4 + C + 5, 'f32', 'lt_viterbi')
  del W
  # cfg5: trigram bf16 loss + dW
  B, T, U, V, n = 32, 1000, 100, 32, 2
  C, W, nf, lab, nl = inputs(B, T, U, V, n, torch.bfloat16)
  ws = torch.empty([nat.loss_grad_workspace_bytes(W, V, n, U, False)], dtype=torch.uint8,
                   device='cuda')
  ms = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws), reps=5)
  Aw = C * (V + 1)
  report('cfg5 trigram bf16', B, T, U, C, ms, Aw * (2 * 2 + 2) + 8 * C + (U + 1) * (4 * 2 + 8),
         'bf16', 'lt_loss_grad')
  del W, ws
  # cfg2 (bench.py's line), same call
  B, T, U, V, n = 64, 1000, 100, 32, 1
  C, W, nf, lab, nl = inputs(B, T, U, V, n, torch.float32)
  ws = torch.empty([nat.loss_grad_workspace_bytes(W, V, n, U, False)], dtype=torch.uint8,
                   device='cuda')
  ms = timeit(lambda: nat.loss_grad(W, nf, lab, nl, V, n, False, workspace=ws))
  Aw = C * (V + 1)
  report('cfg2 bigram fp32', B, T, U, C, ms, Aw * 12 + 8 * C + (U + 1) * 24, 'f32', 'lt_loss_grad')


if __name__ == '__main__':
  main()
