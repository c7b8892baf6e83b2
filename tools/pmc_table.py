"""Per-kernel averages of every PMC counter in rocprofv3 databases:
  python tools/pmc_table.py DIR [DIR ...] [--match SUBSTR]"""
import collections
import glob
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith('--')]
match = next((a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--match=')), '')
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
  for db in glob.glob(f'{d}/**/*.db', recursive=True):
    c = sqlite3.connect(db)
    for name, ctr, val, disp in c.execute(
        'select kernel_name, counter_name, value, dispatch_id from counters_collection'):
      short = name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:60]
      if match in short:
        acc[short][ctr].append(val)
for k, ctrs in acc.items():
  print(k)
  for ctr, v in sorted(ctrs.items()):
    print(f'  {ctr:28s} {sum(v) / len(v):16.1f}  (n={len(v)})')
