"""pico_amd -- libbine's reduce-family collectives (allreduce / reduce_scatter /
reduce) re-built for AMD MI355X: host-side Bine schedule planner, CDNA4 HIP
reduction kernels, RCCL point-to-point over xGMI.

The native library lives in pico_amd/lib/ (built in-tree by
``__graft_entry__.build()``); this package is a thin ctypes mirror of its C ABI
(include/bine_amd.h) with the reference's function names.
"""
from ._lib import ALGOS, DTYPES, OPS, BineError, lib  # noqa: F401
from .api import *  # noqa: F401,F403
from .api import __all__ as _api_all

__all__ = ["ALGOS", "DTYPES", "OPS", "lib"] + _api_all
