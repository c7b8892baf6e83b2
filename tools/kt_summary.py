"""Median kernel durations (us) per kernel name in rocprofv3 databases:
  python tools/kt_summary.py DIR [DIR ...]"""
import collections
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
  acc = collections.defaultdict(list)
  for db in glob.glob(f'{d}/**/*.db', recursive=True):
    c = sqlite3.connect(db)
    for name, s, e in c.execute('select name, start, end from kernels'):
      short = name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:40]
      acc[short].append((e - s) / 1e3)
  print(d)
  for k, v in sorted(acc.items(), key=lambda x: -sum(x[1])):
    v = sorted(v)
    print(f'  {k:40s} n={len(v):4d} median {v[len(v) // 2]:9.1f} us')
