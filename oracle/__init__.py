"""CPU oracle for the lattice hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, as the checker or the timed
CPU baseline. ``last_torch_amd`` never imports it.
"""
