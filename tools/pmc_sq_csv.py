"""Per-kernel PMC counter averages (per dispatch) from rocprofv3 --pmc runs
written as CSV (--output-format csv: *_counter_collection.csv).

Usage: python tools/pmc_sq_csv.py KERNEL_SUBSTRING DIR [DIR ...]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
  key, dirs = sys.argv[1], sys.argv[2:]
  per = defaultdict(lambda: defaultdict(float))
  meta = {}
  for d in dirs:
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
      for r in csv.DictReader(open(f)):
        if key not in r['Kernel_Name']:
          continue
        per[r['Counter_Name']][(f, r['Dispatch_Id'])] += float(r['Counter_Value'])
        meta = {'vgpr': r['VGPR_Count'], 'agpr': r['Accum_VGPR_Count'], 'sgpr': r['SGPR_Count'],
                'lds': r['LDS_Block_Size'], 'grid': r['Grid_Size'], 'wg': r['Workgroup_Size']}
  print(f'kernel ~ {key}: {meta}')
  for cn in sorted(per):
    vals = list(per[cn].values())
    print(f'{cn:32s} {sum(vals) / len(vals):16.1f}  (dispatches {len(vals)})')


if __name__ == '__main__':
  main()
