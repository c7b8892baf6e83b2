"""last_torch_amd: MI355X-native lattice hot path of theadamsabra/last_torch.

Mirrors the reference's public API (last_torch/__init__.py:18-22):
``alignments``, ``contexts``, ``semirings``, ``weight_fns`` and
``RecognitionLattice``. The lattice algorithms run as HIP kernels for gfx950
(``liblt_lattice.so``, C ABI in include/lt_lattice.h).
"""
from last_torch_amd import alignments
from last_torch_amd import contexts
from last_torch_amd import semirings
from last_torch_amd import weight_fns
from last_torch_amd.lattices import RecognitionLattice

__version__ = '0.1.0'
