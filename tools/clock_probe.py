"""The GPU shader clock across a process's first lt_loss_grad calls (dev
tool, GPU; needs `make probe`). Before every call of the bench workload
(configs[1]: B=64, T=1000, U=100, V=32) a one-wave kernel measures the shader
clock against the 100 MHz constant clock (tools/probe/clock_probe.hip); the
call itself is timed with HIP events, and so is a 512 MB device-to-device
copy beside it (HBM-bound: the memory side's rate). Then the same after a
2 s idle gap. Prints the median clock, call time and copy rate per range of
call indices."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native  # noqa: E402

T, U, V, B = 1000, 100, 32, 64


def main():
  probe = ctypes.CDLL(os.path.join(ROOT, 'build', 'libclock_probe.so'))
  probe.clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                               ctypes.c_void_p]
  dev = torch.device('cuda', 0)
  g = torch.Generator(device=dev)
  g.manual_seed(0)
  W = torch.randn([B, T, V + 1, V + 1], generator=g, device=dev)
  nf = torch.full([B], T, dtype=torch.int32, device=dev)
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=dev, dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device=dev)
  ws = torch.empty([_native.loss_grad_workspace_bytes(W, V, 1, U, False)], dtype=torch.uint8,
                   device=dev)
  n = int(os.environ.get('N', 200))
  clk = torch.zeros([n, 4], dtype=torch.int64, device=dev)
  # a random cyclic chain over 1 MB (stride > a cache line between hops)
  perm = torch.randperm(4096, generator=torch.Generator().manual_seed(1))
  nxt = torch.empty(4096, dtype=torch.int64)
  nxt[perm] = torch.roll(perm, -1)
  chain = (nxt * 64).to(torch.int32).repeat_interleave(64).to(dev)
  stream = torch.cuda.current_stream().cuda_stream
  ev = [(torch.cuda.Event(True), torch.cuda.Event(True)) for _ in range(n)]
  cev = [(torch.cuda.Event(True), torch.cuda.Event(True)) for _ in range(n)]
  src = torch.empty([128 << 20], dtype=torch.float32, device=dev)
  dst = torch.empty_like(src)
  src.fill_(1.0)

  def run(tag):
    torch.cuda.synchronize()
    for i in range(n):
      probe.clock_probe(ctypes.c_void_p(clk[i].data_ptr()), 48000, ctypes.c_void_p(chain.data_ptr()),
                        ctypes.c_void_p(stream))
      ev[i][0].record()
      _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
      ev[i][1].record()
      cev[i][0].record()
      dst.copy_(src)
      cev[i][1].record()
    torch.cuda.synchronize()
    c = clk.cpu().numpy()
    mhz = c[:, 0] / np.maximum(c[:, 1], 1) * 100.0
    lat_ns = c[:, 2] * 10.0 / 256
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    gbs = np.array([2 * src.numel() * 4 / (a.elapsed_time(b) * 1e6) for a, b in cev])
    for lo, hi in ((0, 5), (5, 25), (25, 50), (50, 100), (100, 200)):
      if hi <= n:
        print(json.dumps({'phase': tag, 'calls': f'{lo}-{hi - 1}',
                          'shader_clock_mhz_median': round(float(np.median(mhz[lo:hi])), 1),
                          'call_ms_median': round(float(np.median(ms[lo:hi])), 4),
                          'call_ms_mean': round(float(np.mean(ms[lo:hi])), 4),
                          'copy_gb_s_median': round(float(np.median(gbs[lo:hi])), 1),
                          'uncached_load_ns_median': round(float(np.median(lat_ns[lo:hi])), 1)}),
              flush=True)

  run('first calls of the process')
  time.sleep(2.0)
  run('after 2 s idle')
  # the clock DURING the calls: the probe on a second stream, launched right
  # behind each call and spinning about as long as the call (one wave on one
  # CU beside the call's workgroups)
  side = torch.cuda.Stream()
  time.sleep(2.0)
  torch.cuda.synchronize()
  for i in range(n):
    ev[i][0].record()
    _native.loss_grad(W, nf, lab, nl, V, 1, False, workspace=ws)
    ev[i][1].record()
    with torch.cuda.stream(side):
      probe.clock_probe(ctypes.c_void_p(clk[i].data_ptr()), 600000, ctypes.c_void_p(chain.data_ptr()),
                        ctypes.c_void_p(side.cuda_stream))
    torch.cuda.current_stream().wait_stream(side)
  torch.cuda.synchronize()
  c = clk.cpu().numpy()
  mhz = c[:, 0] / np.maximum(c[:, 1], 1) * 100.0
  ms = np.array([a.elapsed_time(b) for a, b in ev])
  for lo, hi in ((0, 5), (5, 25), (25, 50), (50, 100), (100, 200)):
    if hi <= n:
      print(json.dumps({'phase': 'clock during the calls (side stream), after 2 s idle',
                        'calls': f'{lo}-{hi - 1}',
                        'shader_clock_mhz_median': round(float(np.median(mhz[lo:hi])), 1),
                        'call_ms_median': round(float(np.median(ms[lo:hi])), 4)}), flush=True)


if __name__ == '__main__':
  main()
