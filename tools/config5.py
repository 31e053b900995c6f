"""BASELINE config 5's synthetic unstructured domains through
tools/lib/libconfig5.so (tools/config5_gen.cpp holds the definition). Input generation for
bench.py and the tests, not product code."""
from __future__ import annotations

import ctypes
import os

import numpy as np

SEED = 20260715
CELLS = 10_000_000
HALO_FRACTION = 0.05  # outer cells per owned cell
_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libconfig5.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise ImportError(f"{_LIB} missing: build with `make -C tools lib/libconfig5.so`")
        L = ctypes.CDLL(_LIB)
        P = ctypes.POINTER(ctypes.c_int64)
        L.config5_generate.restype = ctypes.c_int
        L.config5_generate.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_uint64, P, P]
        _lib = L
    return _lib


def halo_cells(cells: int = CELLS) -> int:
    return int(round(cells * HALO_FRACTION))


def generate(rank: int, world: int, cells: int = CELLS, halo: int | None = None,
             seed: int = SEED):
    """(gids, outer_lids) of `rank`'s domain: its `cells` owned cells (gid rank*10^7 + i) and
    `halo` outer cells drawn from the other ranks' cells, in a permuted storage order."""
    halo = halo_cells(cells) if halo is None else halo
    gids = np.empty(cells + halo, dtype=np.int64)
    outer = np.empty(max(1, halo), dtype=np.int64)
    P = ctypes.POINTER(ctypes.c_int64)
    rc = _load().config5_generate(rank, world, cells, halo, seed, gids.ctypes.data_as(P),
                                  outer.ctypes.data_as(P))
    if rc:
        raise ValueError(f"config5_generate({rank}, {world}, {cells}, {halo}) refused")
    return gids, outer[:halo]


def value(gids, levels: int = 1):
    """The cell values (unstructured_test_case.hpp:345-359 encoding): gid*100 + level, shape
    (cells, levels) levels-first."""
    return (gids.astype(np.float64)[:, None] * 100.0 +
            np.arange(levels, dtype=np.float64)[None, :])
