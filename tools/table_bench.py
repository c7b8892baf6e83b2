"""Measures the general lattice kernels (lt_table.hip) on BASELINE-sized
lattices: loss + gradient (lt_table_loss_grad) and Viterbi, for
FrameLabelDependent(K) x FullNGram bigram, a random NextStateTable DFA, and
FrameDependent x FullNGram (also run by the tuned kernels, for reference).
Prints one JSON line per workload (ms, lattice cells/s = B*T*U*C*(K+1)/s,
algorithmic GB/s of W read twice + dW written)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


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


def full_ngram_table(V, n):
  from last_torch_amd import contexts
  return contexts.FullNGram(vocab_size=V, context_size=n).next_state_table().to(torch.int32)


def run(name, table, K, B, T, U, dtype=torch.float32):
  C, V = table.shape
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda').to(dtype)
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  graph = nat.TableGraph(table, K, 'cuda')
  ms = timeit(lambda: nat.table_loss_grad(graph, W, nf, lab, nl, False))
  mv = timeit(lambda: nat.table_viterbi(graph, W, nf, 1))
  if os.environ.get('BREAK') == '1':  # the four passes of the loss + gradient apart (Log)
    d, a = nat.table_forward(graph, W, nf, nat.SEMIRING_LOG)
    parts = {
        'den_forward_ms': timeit(lambda: nat.table_forward(graph, W, nf, nat.SEMIRING_LOG)),
        'num_forward_ms': timeit(lambda: nat.table_num_forward(graph, W, nf, lab, nl, nat.SEMIRING_LOG)),
        'den_backward_ms': timeit(lambda: nat.table_den_backward(graph, W, nf, nat.SEMIRING_LOG, d, a)),
    }
    print(json.dumps({'workload': name, 'parts': parts}), flush=True)
  es = 2 if dtype == torch.bfloat16 else 4
  byts = B * T * C * (V + 1) * (3 * es)
  print(json.dumps({'workload': name, 'B': B, 'T': T, 'U': U, 'C': int(C), 'V': int(V), 'K': K,
                    'dtype': str(dtype).split('.')[-1], 'loss_grad_ms': ms,
                    'cells_per_s': B * T * U * C * (K + 1) / (ms * 1e-3),
                    'algorithmic_GBps': byts / (ms * 1e-3) / 1e9, 'viterbi_ms': mv}), flush=True)


def main():
  # ONLY=fld2 (or fld1, dfa, fd): one workload (profiling runs)
  B, T, U = int(os.environ.get('B', 64)), 1000, 100
  only = os.environ.get('ONLY')
  if only in (None, 'fld2'):
    run('FrameLabelDependent(2) x FullNGram bigram V=32', full_ngram_table(32, 1), 2, B, T, U)
  if only in (None, 'fld1'):
    run('FrameLabelDependent(1) x FullNGram bigram V=32', full_ngram_table(32, 1), 1, B, T, U)
  if only in (None, 'dfa'):
    g = torch.Generator().manual_seed(1)
    dfa = torch.randint(0, 64, (64, 32), generator=g, dtype=torch.int32)
    run('FrameDependent x NextStateTable (random DFA, C=64, V=32)', dfa, 0, B, T, U)
  if only in (None, 'fd'):
    run('FrameDependent x FullNGram bigram V=32 (table path)', full_ngram_table(32, 1), 0, B, T, U)


if __name__ == '__main__':
  main()
