"""Per-kernel duration stats from a rocprofv3 run: the *_kernel_stats.csv if
present, else the rocpd sqlite database (-o run -> run_results.db)."""
import glob
import sqlite3
import sys
from collections import defaultdict


def stats_from_db(path):
  c = sqlite3.connect(path)
  q = ('select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d '
       'join rocpd_info_kernel_symbol s on d.kernel_id = s.id')
  acc = defaultdict(list)
  for name, dur in c.execute(q):
    acc[name].append(dur)
  return acc


def main():
  root = sys.argv[1]
  dbs = glob.glob(f'{root}/**/*.db', recursive=True)
  acc = defaultdict(list)
  for db in dbs:
    for k, v in stats_from_db(db).items():
      acc[k] += v
  rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
  print('name,calls,total_ns,avg_ns,min_ns,max_ns')
  for name, d in rows:
    short = name.split('(')[0][:90]
    print(f'"{short}",{len(d)},{sum(d)},{sum(d) / len(d):.1f},{min(d)},{max(d)}')


if __name__ == '__main__':
  main()
