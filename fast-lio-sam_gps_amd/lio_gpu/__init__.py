"""lio_gpu — MI355X-native (gfx950) scan-matching hot path of FAST-LIO-SAM.

Host-side mirror of the reference interfaces over the C-ABI in
``include/lio_gpu.h`` (liblio_gpu.so, hand-written HIP kernels):

* :mod:`lio_gpu.frontend` — ikd-Tree map, ``h_share_model``, IESKF update
* :mod:`lio_gpu.loop_closure` — ``LoopClosure::icpAlignment``
* :mod:`lio_gpu.dist` — one-process-per-GPU sharding of the loop ICP
* :mod:`lio_gpu.synth` — seeded synthetic scans/maps for tests and bench
"""
from ._capi import LioError, lib  # noqa: F401

__all__ = ["LioError", "lib"]
