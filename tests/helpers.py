"""Shared test geometry, restating the reference tests' setups (data + checks only)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as orc


# ---------------------------------------------------------------------------------------------
# test/structured/regular/test_regular_domain.cpp:33-121, 660-800
# 4 ranks x 2 domains (4 x Y x 1 decomposition), local extent (4,3,2), offset 3, periodic,
# pattern 1 halos {0,0,1,0,1,2}, pattern 2 halos {2,2,2,2,2,2}; 3 fields per domain with
# value type array<T,3> = the global coordinate of the cell.
# ---------------------------------------------------------------------------------------------
LOCAL_EXT = (4, 3, 2)
OFFSET = (3, 3, 3)
HALOS_1 = (0, 0, 1, 0, 1, 2)
HALOS_2 = (2, 2, 2, 2, 2, 2)


def regular_test_domains(n_ranks=4):
    g_last = (LOCAL_EXT[0] * 4 - 1, ((n_ranks - 1) // 2 + 1) * LOCAL_EXT[1] - 1, LOCAL_EXT[2] - 1)
    ranks = []
    for r in range(n_ranks):
        doms = []
        for k in range(2):
            f = (((r % 2) * 2 + k) * LOCAL_EXT[0], (r // 2) * LOCAL_EXT[1], 0)
            l = (((r % 2) * 2 + k + 1) * LOCAL_EXT[0] - 1, (r // 2 + 1) * LOCAL_EXT[1] - 1,
                 LOCAL_EXT[2] - 1)
            doms.append(orc.RegularDomain(r * 2 + k, f, l))
        ranks.append(doms)
    return ranks, (0, 0, 0), g_last


def coord_field(dom, dtype):
    """fill_values (test_regular_domain.cpp:711-724): interior cell = its global coordinate,
    stored as array<T,3>; x fastest (layout_map<2,1,0>). Halo cells start at -1 sentinel."""
    ext = tuple(LOCAL_EXT[d] + 2 * OFFSET[d] for d in range(3))
    a = np.full((ext[2], ext[1], ext[0], 3), -1, dtype=dtype)
    for z in range(LOCAL_EXT[2]):
        for y in range(LOCAL_EXT[1]):
            for x in range(LOCAL_EXT[0]):
                a[z + OFFSET[2], y + OFFSET[1], x + OFFSET[0]] = (
                    x + dom.first[0], y + dom.first[1], z + dom.first[2])
    return a


def coord_fieldspec(arr):
    ext = (arr.shape[2], arr.shape[1], arr.shape[0])
    return orc.FieldSpec(arr, arr.itemsize * 3, (2, 1, 0), OFFSET, ext)


def check_coord_field(arr, dom, halos, g_first, g_last, periodic=(True, True, True)):
    """check_values (test_regular_domain.cpp:739-800) for the periodic case: every cell of the
    halo box (owned + halos) holds the periodic-wrapped global coordinate. Returns #bad cells."""
    bad = 0
    ext_g = [g_last[d] - g_first[d] + 1 for d in range(3)]
    for zl in range(-halos[4], LOCAL_EXT[2] + halos[5]):
        for yl in range(-halos[2], LOCAL_EXT[1] + halos[3]):
            for xl in range(-halos[0], LOCAL_EXT[0] + halos[1]):
                g = [xl + dom.first[0], yl + dom.first[1], zl + dom.first[2]]
                w = [((g[d] - g_first[d]) + ext_g[d]) % ext_g[d] + g_first[d] for d in range(3)]
                v = arr[zl + OFFSET[2], yl + OFFSET[1], xl + OFFSET[0]]
                if not (v[0] == w[0] and v[1] == w[1] and v[2] == w[2]):
                    bad += 1
    return bad


# ---------------------------------------------------------------------------------------------
# generic cube geometry (bench configs scaled down): N^3 per rank, halo H, periodic,
# decomposition parts=(px,py,pz); rank r <-> (r%px, r//px%py, r//(px*py)); x fastest.
# ---------------------------------------------------------------------------------------------
def cube_domains(N, parts):
    px, py, pz = parts
    ranks = []
    for r in range(px * py * pz):
        c = (r % px, (r // px) % py, r // (px * py))
        f = tuple(c[d] * N for d in range(3))
        l = tuple((c[d] + 1) * N - 1 for d in range(3))
        ranks.append([orc.RegularDomain(r, f, l)])
    g_last = (px * N - 1, py * N - 1, pz * N - 1)
    return ranks, (0, 0, 0), g_last


def linear_index_field(dom, N, H, g_last, dtype=np.float64, layout=(2, 1, 0), seed=None, add=0):
    """Cube field of extent (N+2H)^3, owned cells = global linear index (exact in fp64 < 2^53),
    halos pre-filled with -1 (SURVEY §8(d) synthetic inputs). Returns (array, FieldSpec).

    layout is the gridtools layout_map of (x,y,z); the numpy array is allocated so that the
    memory order matches it (the dim with layout value 2 is contiguous)."""
    E = N + 2 * H
    order = sorted(range(3), key=lambda d: layout[d])  # slowest ... fastest dim
    shape = tuple(E for _ in order)
    a = np.full(shape, -1).astype(dtype)  # -1 sentinel (wraps for unsigned types)
    gx, gy, gz = g_last[0] + 1, g_last[1] + 1, g_last[2] + 1
    idx = np.meshgrid(*[np.arange(N) for _ in range(3)], indexing="ij")  # idx[k] over memory axes
    coords = [None, None, None]
    for ax, d in enumerate(order):
        coords[d] = idx[ax] + dom.first[d]
    val = coords[0] + gx * (coords[1] + gy * coords[2])
    if seed is not None:
        val = (val * 2654435761 + seed) % (1 << 40)
    if add:  # per-field offset (BASELINE config 4: field number), rounded once from f64
        val = (val + add).astype(np.float64)
    a[tuple(slice(H, H + N) for _ in order)] = val.astype(dtype)
    spec = orc.FieldSpec(a, a.itemsize, tuple(layout), (H, H, H), (E, E, E))
    return a, spec


def expected_linear_halo(a, dom, N, H, g_last, layout=(2, 1, 0)):
    """Expected field after a periodic exchange: every cell of the (N+2H)^3 box = the wrapped
    global linear index (the reference tests' own halo property)."""
    E = N + 2 * H
    order = sorted(range(3), key=lambda d: layout[d])
    G = [g_last[d] + 1 for d in range(3)]
    idx = np.meshgrid(*[np.arange(E) for _ in range(3)], indexing="ij")
    coords = [None, None, None]
    for ax, d in enumerate(order):
        coords[d] = (idx[ax] - H + dom.first[d]) % G[d]
    return (coords[0] + G[0] * (coords[1] + G[1] * coords[2])).astype(a.dtype)
