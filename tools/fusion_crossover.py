"""Measures the crossover SURVEY.md §8(f) rank 1 asks about: where a producer
fused into the lattice kernels (W never written to HBM) would beat the
separate MFMA producer launch, at the bench shape (B=64, T=1000, bigram
V=32: C=33, R=33) for hidden sizes H.

The separate design writes W once and the chunked scan reads it twice (phase
A and phase C); a fused design recomputes W inside both consumers instead.
Per H this prints, all measured on this GPU:
  producer_fwd_ms     lt_joint_weights (fp32-faithful split-bf16 and bf16)
  w_write_ms          a 279 MB fill of W (the producer's write floor)
  w_read_ms           one read pass of W (torch.sum, f32 accumulation)
  w_roundtrip_ms      w_write + 2 x w_read: what the forward fusion saves
  fused_fwd_extra_ms  the fused forward's extra cost = producer compute (fwd
                      minus its write floor) paid twice instead of once,
                      minus the round trip it saves; < 0 means fusion wins
  producer_bwd_ms     lt_joint_weights_backward (dW read once)
  dw_roundtrip_ms     phase C's dW write + the backward's dW read, what a
                      backward fused into phase C saves
  lattice_ms          lt_loss_grad on the same W (chunked scan)
  step_ms             the whole separate-launch training step (producer
                      fwd + lattice + producer bwd), no autograd overhead
One JSON line per H."""
import json
import os
import sys

import torch

ROOT = os.environ.get('LT_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def timeit(fn, reps=10):
  for _ in range(2):
    fn()
  torch.cuda.synchronize()
  best = 1e9
  for _ in range(3):
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
      fn()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / reps)
  return best


def main():
  B, T, U, V = 64, 1000, 100, 32
  C = R = V + 1
  dev = torch.device('cuda')
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  nf = torch.full([B], T, dtype=torch.int32, device=dev)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=dev, dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device=dev)
  # the W traffic floors, measured once (they do not depend on H)
  Wbuf = torch.empty([B, T, C, R], device=dev)
  w_write = timeit(lambda: Wbuf.fill_(1.0))
  Wbuf.normal_()
  w_read = timeit(lambda: torch.sum(Wbuf))
  ws = torch.empty([nat.loss_grad_workspace_bytes(Wbuf, V, 1, U, False)], dtype=torch.uint8,
                   device=dev)
  lattice = timeit(lambda: nat.loss_grad(Wbuf, nf, lab, nl, V, 1, False, workspace=ws))
  del Wbuf
  rt = w_write + 2 * w_read
  for H in [int(h) for h in os.environ.get('HS', '32,64,128,256,512').split(',')]:
    pc = torch.randn([C, H], generator=g, device=dev)
    pf = torch.randn([B, T, H], generator=g, device=dev)
    wo = torch.randn([R, H], generator=g, device=dev) / H ** 0.5
    bias = torch.randn([R], generator=g, device=dev)
    fwd = timeit(lambda: nat.joint_weights(pc, pf, wo, bias, precision='fp32'))
    fwd16 = timeit(lambda: nat.joint_weights(pc, pf, wo, bias, precision='bf16'))
    W = nat.joint_weights(pc, pf, wo, bias, precision='fp32')
    out = nat.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
    dW = out[3]
    bwd = timeit(lambda: nat.joint_weights_backward(pc, pf, wo, dW), reps=5)

    def step():
      Wx = nat.joint_weights(pc, pf, wo, bias, precision='fp32')
      o = nat.loss_grad(Wx, nf, lab, nl, V, 1, False, workspace=ws)
      nat.joint_weights_backward(pc, pf, wo, o[3])

    st = timeit(step, reps=5)
    row = {'H': H, 'B': B, 'T': T, 'C': C, 'R': R,
           'producer_fwd_ms': round(fwd, 4), 'producer_fwd_bf16_ms': round(fwd16, 4),
           'w_write_ms': round(w_write, 4), 'w_read_ms': round(w_read, 4),
           'w_roundtrip_ms': round(rt, 4),
           'fused_fwd_extra_ms': round(2 * (fwd - w_write) - ((fwd - w_write) + rt), 4),
           'fused_fwd_extra_bf16_ms': round(2 * (fwd16 - w_write) - ((fwd16 - w_write) + rt), 4),
           'producer_bwd_ms': round(bwd, 4), 'dw_roundtrip_ms': round(w_write + w_read, 4),
           'lattice_ms': round(lattice, 4), 'step_ms': round(st, 4)}
    row['fusion_wins_fwd'] = row['fused_fwd_extra_ms'] < 0
    print(json.dumps(row), flush=True)
    del pc, pf, wo, bias, W, out, dW


if __name__ == '__main__':
  main()
