"""Per-kernel register / occupancy / spill summary of one HIP source for
gfx950 (hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel.

  python tools/kres.py last_torch_amd/csrc/lt_chunk.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
extra = [x for x in sys.argv[3:]]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
out = subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950',
                      '-c', src, '-o', '/tmp/kres.o', '-Rpass-analysis=kernel-resource-usage',
                      '--offload-device-only'] + extra, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
  m = re.search(r'remark: +(Function Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|'
                r'VGPRs Spill|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\S+)', line)
  if not m:
    continue
  k, v = m.groups()
  if k == 'Function Name':
    cur = v
    rows[cur] = {}
  elif cur:
    rows[cur][k.split(' [')[0]] = v
for name, r in rows.items():
  if flt in name:
    print(f"{name[:70]:70s} V={r.get('VGPRs')} A={r.get('AGPRs')} occ={r.get('Occupancy')} "
          f"sspill={r.get('SGPRs Spill')} vspill={r.get('VGPRs Spill')} scratch={r.get('ScratchSize')} "
          f"lds={r.get('LDS Size')}")
