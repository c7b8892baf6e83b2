"""The chunked scan's hand-off timeout route (lt_chunk.hip, ChunkReady::timeout).

A walk whose chunk record is never published gives up after a bounded spin,
and its utterance goes to the frame-serial kernels in the same call. Only
the diagnostic build (make diag: build/diag/liblt_lattice_diag.so) can force
that route: LT_CK_DBG=512 withholds utterance 0's chunk-1 ready flag. A child
process (tests/diag_timeout_child.py) makes one call against it: the
utterance's fallback word must be set, and every utterance and every dW
element must still match the oracle.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(ROOT, 'build', 'diag', 'liblt_lattice_diag.so')


def test_chunk_handoff_timeout_route(cuda):
  if not os.path.exists(DIAG):
    pytest.skip('diagnostic build absent (make diag)')
  env = dict(os.environ, LT_LIB_PATH=DIAG, LT_CK_DBG='512')
  r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'diag_timeout_child.py')],
                     cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
  assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
  assert r.stdout.startswith('ok'), r.stdout[-2000:]


def test_quad_trigram_recursions(cuda):
  """The quad trigram recursions (lt_tri4.hip; diagnostic build only, they
  measured slower than the one-workgroup kernel) still match the oracle."""
  if not os.path.exists(DIAG):
    pytest.skip('diagnostic build absent (make diag)')
  env = dict(os.environ, LT_LIB_PATH=DIAG, LT_TRI4='1')
  r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'diag_tri4_child.py')],
                     cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
  assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
  assert r.stdout.startswith('ok'), r.stdout[-2000:]
