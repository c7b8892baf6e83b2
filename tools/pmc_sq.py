"""Per-kernel PMC counter averages (per dispatch) from rocprofv3 --pmc runs
written as rocpd databases (-o run -> run_results.db).

Usage: python tools/pmc_sq.py KERNEL_SUBSTRING DIR [DIR ...]
Prints one line per counter: the mean over the kernel's dispatches of the
counter's value summed over the dispatch's records (SE / XCD instances).
"""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
  key, dirs = sys.argv[1], sys.argv[2:]
  per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
  meta = {}
  for d in dirs:
    for db in glob.glob(f'{d}/**/*.db', recursive=True):
      c = sqlite3.connect(db)
      q = ('select dispatch_id, kernel_name, counter_name, value, vgpr_count, accum_vgpr_count, '
           'sgpr_count, lds_block_size, grid_size, workgroup_size from counters_collection')
      for disp, name, cn, v, vg, ag, sg, lds, grid, wg in c.execute(q):
        if key not in name:
          continue
        per[cn][(db, disp)] += v
        meta = {'vgpr': vg, 'agpr': ag, 'sgpr': sg, 'lds': lds, 'grid': grid, 'wg': wg}
  print(f'kernel ~ {key}: {meta}')
  for cn in sorted(per):
    vals = list(per[cn].values())
    print(f'{cn:28s} {sum(vals) / len(vals):16.1f}  (dispatches {len(vals)})')


if __name__ == '__main__':
  main()
