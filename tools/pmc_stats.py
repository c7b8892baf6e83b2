"""Per-kernel PMC counter sums from a rocprofv3 --pmc run (CSV output):
python tools/pmc_stats.py <dir> [kernel-substring]."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
  root = sys.argv[1]
  want = sys.argv[2] if len(sys.argv) > 2 else ''
  acc = defaultdict(lambda: defaultdict(float))
  calls = defaultdict(set)
  for path in glob.glob(f'{root}/**/*counter_collection.csv', recursive=True):
    with open(path) as f:
      for row in csv.DictReader(f):
        name = row.get('Kernel_Name', '')
        if want not in name:
          continue
        m = re.search(r'(\w+_kernel)', name)
        short = m.group(1) if m else name[:60]
        acc[short][row['Counter_Name']] += float(row['Counter_Value'])
        calls[short].add(row.get('Dispatch_Id', ''))
  for k, d in acc.items():
    n = max(1, len(calls[k]))
    print(k, f'({n} dispatches)')
    for c, v in sorted(d.items()):
      print(f'  {c:28s} {v / n:16.0f} per dispatch')


if __name__ == '__main__':
  main()
