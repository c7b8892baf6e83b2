"""Per-kernel times of the chunked scan's role ablations (diagnostic build):
reads a rocprofv3 --kernel-trace CSV of `tools/chunk_ablate.py` (DBGS list,
3 warm-up + 10 timed calls per value) and prints the median ck_ab_kernel /
ck_marg_kernel duration per ablation value, in the order they ran.

  python tools/ck_abl_trace.py <kernel_trace.csv> <dbg,dbg,...>
"""
import csv
import statistics
import sys

path, dbgs = sys.argv[1], sys.argv[2].split(',')
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
seq = {'ab': [], 'marg': []}
for r in rows:
  n = r['Kernel_Name']
  d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
  if 'ck_ab_kernel' in n:
    seq['ab'].append(d)
  elif 'ck_marg_kernel' in n:
    seq['marg'].append(d)
per = 13
for i, dbg in enumerate(dbgs):
  ab = seq['ab'][i * per + 3:(i + 1) * per]
  mg = seq['marg'][i * per + 3:(i + 1) * per]
  if not ab:
    break
  print(f'dbg={dbg:>5s}  ck_ab {statistics.median(ab):7.1f} us  ck_marg {statistics.median(mg):7.1f} us')
