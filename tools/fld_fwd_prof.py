"""Diagnostic: FrameLabelDependent(2) x FullNGram bigram (B=64, T=1000, V=32)
denominator forward (lt_table_forward, Log) and backward alone, for PMC passes."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402
from last_torch_amd import contexts  # noqa: E402

B, T, V, K = int(os.environ.get('B', 64)), 1000, 32, int(os.environ.get('K', 2))
table = contexts.FullNGram(vocab_size=V, context_size=1).next_state_table().to(torch.int32)
C = table.shape[0]
g = torch.Generator(device='cuda')
g.manual_seed(0)
W = torch.randn([B, T, C, V + 1], generator=g, device='cuda')
nf = torch.full([B], T, dtype=torch.int32, device='cuda')
graph = nat.TableGraph(table, K, 'cuda')
for _ in range(int(os.environ.get('N', 3))):
  d, a = nat.table_forward(graph, W, nf, nat.SEMIRING_LOG)
  if os.environ.get('BWD', '1') == '1':
    nat.table_den_backward(graph, W, nf, nat.SEMIRING_LOG, d, a)
torch.cuda.synchronize()
print('ok', float(d[0]))
