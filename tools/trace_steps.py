"""Runs a few loss+grad steps for a kernel trace (dev tool).

  rocprofv3 --kernel-trace -d gpurun_out/tr -o tr --output-format csv -- \
      python3 tools/trace_steps.py --batch 64 --steps 3
  python tools/trace_steps.py --summarize gpurun_out/tr
"""
import argparse
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
  import torch
  from last_torch_amd import _native as nat
  V, n, T, U = args.vocab, args.context, args.frames, args.labels
  C = nat.num_context_states(V, n)
  g = torch.Generator(device='cuda')
  g.manual_seed(0)
  dt = torch.bfloat16 if args.bf16 else torch.float32
  W = torch.randn([args.batch, T, C, V + 1], generator=g, device='cuda').to(dt)
  nf = torch.full([args.batch], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, [args.batch, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([args.batch], U, dtype=torch.int32, device='cuda')
  for _ in range(args.steps):
    out = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=not args.rec)
    nat.loss_backward(W, nf, lab, nl, *out[1:5], None, V, n, False,
                      ck=None if args.rec else out[5])
  torch.cuda.synchronize()


def summarize(path):
  files = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
  rows = []
  for f in files:
    with open(f) as fh:
      rows += list(csv.DictReader(fh))
  rows.sort(key=lambda r: int(r['Start_Timestamp']))
  t0 = int(rows[0]['Start_Timestamp']) if rows else 0
  for r in rows:
    name = r['Kernel_Name']
    if 'kernel' not in name:
      continue
    short = name.split('(')[0].split('::')[-1][:60]
    s, e = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
    print(f"{short:60s} start {s / 1e3:10.1f} us  end {e / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f} us"
          f"  grid {r.get('Grid_Size', '?')} wg {r.get('Workgroup_Size', '?')} lds {r.get('LDS_Block_Size', '?')}"
          f" vgpr {r.get('VGPR_Count', '?')} q {r.get('Queue_Id', '?')}")


if __name__ == '__main__':
  ap = argparse.ArgumentParser()
  ap.add_argument('--batch', type=int, default=64)
  ap.add_argument('--frames', type=int, default=1000)
  ap.add_argument('--labels', type=int, default=100)
  ap.add_argument('--vocab', type=int, default=32)
  ap.add_argument('--context', type=int, default=1)
  ap.add_argument('--steps', type=int, default=3)
  ap.add_argument('--bf16', action='store_true')
  ap.add_argument('--rec', action='store_true')
  ap.add_argument('--summarize')
  a = ap.parse_args()
  if a.summarize:
    summarize(a.summarize)
  else:
    run(a)
