"""CPU oracle for the NeRF render hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU (numpy float32 arithmetic, float64 running
products/sums where the reference's CPU torch kernels accumulate in double),
the reference renderer's algorithm so the HIP product path can be checked
against it. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker or
the timed CPU baseline. The product path (``nerf-rep_for_test_amd/``) never
imports it and fails loudly when the HIP library is missing.

Parity pinning: ``tests/golden/*.npz`` are captured from the reference Python
renderer itself (``tests/golden/make_golden.py``, run in the survey container
where ``/root/reference`` is importable); ``tests/test_oracle_golden.py`` checks
this restatement against every one of them.
"""
