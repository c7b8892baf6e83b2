"""Times the joint weight function's arc weights at the bench shape (B=64,
T=1000, bigram V=32: C=33, R=33) for hidden sizes H: the matrix-core
producer (lt_joint_weights) against the PyTorch formula (the [B,T,C,H]
hidden tensor materialised, as JointWeightFn without the kernel), forward
and forward+backward. One JSON line per H."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402
from last_torch_amd import weight_fns  # noqa: E402


def timeit(fn, reps=5):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def main():
  B, T, C, R = 64, 1000, 33, 33
  for H in [int(h) for h in os.environ.get('HS', '128,512').split(',')]:
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    pc = torch.randn([C, H], generator=g, device='cuda')
    pf = torch.randn([B, T, H], generator=g, device='cuda')
    wo = torch.randn([R, H], generator=g, device='cuda') / H ** 0.5
    bias = torch.randn([R], generator=g, device='cuda')

    def torch_fwd():
      return torch.matmul(torch.tanh(pc[None, None] + pf[:, :, None, :]), wo.t()) + bias

    kern = timeit(lambda: nat.joint_weights(pc, pf, wo, bias, precision='fp32'))
    kern_bf16 = timeit(lambda: nat.joint_weights(pc, pf, wo, bias, precision='bf16'))
    # some |ctx projection| > 40: every block takes the direct e^{2(a+b)} path
    pc_big = pc.clone()
    pc_big.view(-1)[0] = 100.0
    kern_direct = timeit(lambda: nat.joint_weights(pc_big, pf, wo, bias))
    del pc_big
    ref = timeit(torch_fwd)
    leaves = [t.clone().requires_grad_(True) for t in (pc, pf, wo, bias)]
    gW = torch.randn([B, T, C, R], device='cuda')

    def kern_fb():
      W = weight_fns._JointWeightsFn.apply(*leaves, int(os.environ.get("CHUNK", 16384)), 'fp32')
      torch.autograd.backward(W, gW)

    def torch_fb():
      W = torch.matmul(torch.tanh(leaves[0][None, None] + leaves[1][:, :, None, :]),
                       leaves[2].t()) + leaves[3]
      torch.autograd.backward(W, gW)

    kbwd = timeit(lambda: nat.joint_weights_backward(pc, pf, wo, gW), reps=3)
    kfb = timeit(kern_fb, reps=3)
    rfb = timeit(torch_fb, reps=3)
    flops = 2.0 * B * T * C * R * H
    print(json.dumps({'H': H, 'B': B, 'T': T, 'C': C, 'R': R,
                      'producer_fwd_ms': kern, 'producer_fwd_bf16_ms': kern_bf16,
                      'producer_fwd_direct_ms': kern_direct,
                      'torch_fwd_ms': ref,
                      'producer_bwd_kernel_ms': kbwd, 'producer_fwd_bwd_ms': kfb, 'torch_fwd_bwd_ms': rfb,
                      'producer_fwd_TFLOPs': flops / (kern * 1e-3) / 1e12,
                      'producer_bwd_TFLOPs': 2 * flops / (kbwd * 1e-3) / 1e12,
                      'W_write_GBps': B * T * C * R * 4 / (kern * 1e-3) / 1e9}), flush=True)
    del leaves, gW


if __name__ == '__main__':
  main()
