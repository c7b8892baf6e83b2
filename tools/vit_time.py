"""Diagnostic: lt_viterbi at cfg4 (B=64, T=2000, V=32 bigram, fp32), HIP events
over 10 calls; LT_LIB_PATH / LT_VIT_DBG as set by the caller."""
import os
import sys

import torch

ROOT = os.environ.get('LT_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402

B, T, V = int(os.environ.get('B', 64)), int(os.environ.get('T', 2000)), 32
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, V + 1, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
WARM, N = int(os.environ.get('WARM', 2)), int(os.environ.get('N', 10))
for _ in range(WARM):
  nat.viterbi(W, nf, V, 1, nat.LABELS_REFERENCE)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
e0.record()
for _ in range(N):
  nat.viterbi(W, nf, V, 1, nat.LABELS_REFERENCE)
e1.record()
torch.cuda.synchronize()
print(f"{os.environ.get('TAG', '')} lt_viterbi B={B} T={T}: {e0.elapsed_time(e1) / N:.3f} ms "
      f"({WARM} warmup, {N} timed calls)", flush=True)
