"""Summarises rocprofv3 PMC passes into per-launch HBM bytes per kernel.

Usage (after two separate passes, one counter each -- FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC
slots"):

  python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
      --batch 64 --frames 1000 --out profiles/r01_pmc_summary.json

Corrections (MI355X_MICROARCH.md "HBM [CDNA4]"):
  * FETCH_SIZE is in KiB and, on gfx950, reports exactly half of the bytes
    of a wide (16 B/lane) coalesced streaming read -- both global_load and
    buffer/global_load ... lds. The arc-weight and alpha streams of these
    kernels are 16 B/lane LDS-DMA reads, so FETCH_SIZE is doubled.
  * WRITE_SIZE (KiB) is exact for 16 B/lane streaming stores and dword
    float stores; it is taken as is.
  * The chunked path's transfer kernel (ck_ab_kernel, with the walks) reads W with
    dword loads, a width the guide leaves uncalibrated; it reads every frame
    exactly once (B*T*FR*4 bytes), so its doubled FETCH_SIZE against that
    count is the calibration, printed as ``fetch_vs_w``.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _rows(path):
  files = glob.glob(os.path.join(path, '**', '*counter_collection.csv'), recursive=True)
  if not files:
    raise SystemExit(f'no *counter_collection.csv under {path}')
  for f in files:
    with open(f) as fh:
      yield from csv.DictReader(fh)


def _kernel_key(name):
  """Kernel family: fwd_kernel, bwd_kernel (beta + marginals), bwd_kernel_ck
  (checkpointing beta pass: last template argument true), marg_kernel, ..."""
  if 'bwd_kernel' in name:
    args = name.split('bwd_kernel<', 1)[-1].split('>', 1)[0].split(',')
    return 'bwd_kernel_ck' if len(args) >= 6 and args[5].strip() == 'true' else 'bwd_kernel'
  if 'tab_' in name:  # the general table kernels (lt_table.hip): their own names
    import re
    m = re.search(r'(tab_\w+)', name)
    return m.group(1) if m else None
  for k in ('ck_ab_kernel', 'ck_combine_kernel', 'ck_marg_kernel',
            'fwd_kernel', 'marg_kernel', 'backtrace_kernel', 'num_scatter_kernel', 'pipe_kernel',
            'joint_weights_fb_kernel', 'joint_weights_kernel', 'joint_backward_kernel',
            'joint_exp_kernel', 'joint_reduce_kernel'):
    if k in name:
      return k
  return None


def collect(path, counter):
  per = defaultdict(list)
  for r in _rows(path):
    if r.get('Counter_Name') != counter:
      continue
    k = _kernel_key(r.get('Kernel_Name', ''))
    if k:
      per[(k, r.get('Dispatch_Id'))].append(float(r['Counter_Value']))
  out = defaultdict(list)
  for (k, _), vals in per.items():
    out[k].append(sum(vals))  # sum over XCD/instance rows of one dispatch
  return out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--fetch', required=True)
  ap.add_argument('--write', required=True)
  ap.add_argument('--batch', type=int, required=True)
  ap.add_argument('--frames', type=int, required=True)
  ap.add_argument('--out', required=True)
  ap.add_argument('--w-bytes', type=float, default=None,
                  help='bytes of W per launch (B*T*C*(V+1)*4): fetch_vs_w calibration')
  args = ap.parse_args()
  fetch = collect(args.fetch, 'FETCH_SIZE')
  write = collect(args.write, 'WRITE_SIZE')
  kernels = {}
  for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k, [])
    w = write.get(k, [])
    fb = 2 * 1024 * (sum(f) / len(f)) if f else None
    wb = 1024 * (sum(w) / len(w)) if w else None
    kernels[k] = {
        'batch': args.batch, 'frames': args.frames,
        'dispatches': {'fetch_pass': len(f), 'write_pass': len(w)},
        'fetch_bytes_per_launch': fb, 'write_bytes_per_launch': wb,
        'fetch_bytes_per_launch_uncorrected': fb / 2 if fb is not None else None,
        'hbm_bytes_per_launch': (fb or 0) + (wb or 0) if (fb is not None and wb is not None)
        else None,
    }
    if args.w_bytes and fb is not None:
      kernels[k]['fetch_vs_w'] = fb / args.w_bytes
  res = {'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)',
         'corrections': 'FETCH_SIZE KiB x1024 x2 (gfx950 wide-read half count); '
                        'WRITE_SIZE KiB x1024',
         'kernels': kernels}
  os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
  with open(args.out, 'w') as f:
    json.dump(res, f, indent=1)
  print(json.dumps(res, indent=1))


if __name__ == '__main__':
  main()
