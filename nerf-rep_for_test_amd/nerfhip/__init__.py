"""MI355X-native NeRF render path (gfx950 HIP kernels behind a C ABI).

Submodules: ``_lib`` (ctypes binding of lib/libnerfhip.so), ``pack`` (MLP weight
packing), ``render`` (device pipeline), ``synthetic`` (deterministic weights and
occupancy grids), ``dist`` (tile sharding + RCCL gather).
"""
