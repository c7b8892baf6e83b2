"""Diagnostic: lt_loss_grad time across phase-C LDS budgets (chunk lengths)."""
import os
import subprocess
import sys

for lds in os.environ.get('BUDGETS', '40960 49152 57344 81920').split():
  env = dict(os.environ, LT_CHUNK_LDS=lds)
  out = subprocess.run([sys.executable, '-u', 'tools/chunk_ablate.py'], env=env, capture_output=True,
                       text=True, timeout=180)
  lines = [l for l in out.stdout.splitlines() if l.startswith('dbg')]
  print(lds, ' | '.join(lines[:1] + lines[3:4] + lines[5:6]) if lines else out.stderr[-500:],
        flush=True)
