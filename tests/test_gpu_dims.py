"""GPU parity for 1-D and 2-D structured exchanges (the reference's halo generator and pattern are
dimension-generic: halo_generator.hpp:93-160 recurses over D; the 2-D case is what
test/structured/regular/test_simple_regular_domain.cpp:99-138 exchanges).

Several domains on one rank, uneven splits, asymmetric halos (0 on a side included), periodic and
non-periodic dimensions, both layout maps in 2-D, 2/4/8-byte elements; fused (all-self) and
two-launch exchanges. Bit-exact against the oracle: every packed message and every field byte.
"""
import itertools

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()  # must load: no fallback


def _splits(G, parts):
    """Uneven cuts of [0, G) into `parts` pieces (the last ones one cell longer)."""
    base, extra = divmod(G, parts)
    out, f = [], 0
    for p in range(parts):
        n = base + (1 if p >= parts - extra else 0)
        out.append((f, f + n - 1))
        f += n
    return out


def _domains(G, parts):
    per_dim = [_splits(G[d], parts[d]) for d in range(len(G))]
    doms = []
    for i, cut in enumerate(itertools.product(*reversed(per_dim))):
        cut = tuple(reversed(cut))  # dim 0 fastest in the domain numbering
        doms.append(orc.RegularDomain(i, tuple(c[0] for c in cut), tuple(c[1] for c in cut)))
    return doms


def _field(dom, G, halos, layout, dtype, seed):
    """Memory-order array (slowest dim first): owned cell = global linear index + 1 + seed
    (< 2^15 here, exact in every tested dtype), halo = -1, which no owned cell holds."""
    D = len(G)
    n = [dom.last[d] - dom.first[d] + 1 for d in range(D)]
    E = [n[d] + halos[2 * d] + halos[2 * d + 1] for d in range(D)]
    logical = np.full(E, -1, dtype=np.float64)
    idx = np.meshgrid(*[np.arange(n[d]) + dom.first[d] for d in range(D)], indexing="ij")
    lin = np.zeros(n, dtype=np.float64)
    mul = 1
    for d in range(D):
        lin += idx[d] * mul
        mul *= G[d]
    sl = tuple(slice(halos[2 * d], halos[2 * d] + n[d]) for d in range(D))
    logical[sl] = lin + 1 + seed
    order = sorted(range(D), key=lambda d: layout[d])  # memory axis -> logical dim
    mem = np.ascontiguousarray(logical.transpose(order)).astype(dtype)
    offs = tuple(halos[2 * d] for d in range(D))
    return mem, offs, tuple(E)


CASES = [
    # (G, parts, halos (d0-, d0+, d1-, d1+), periodic)
    ((64,), (1,), (1, 1), (True,)),
    ((64,), (3,), (2, 3), (True,)),
    ((61,), (4,), (0, 2), (False,)),
    ((24, 17), (1, 1), (1, 1, 1, 1), (True, True)),
    ((24, 17), (2, 3), (2, 1, 0, 3), (True, False)),
    ((24, 17), (3, 2), (3, 3, 3, 3), (True, True)),
    ((30, 11), (2, 1), (1, 2, 2, 1), (False, True)),
]


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int16])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_low_dim_exchange(case, dtype, fused):
    import torch
    import ghex_amd
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    G, parts, halos, periodic = CASES[case]
    D = len(G)
    gf, gl = (0,) * D, tuple(g - 1 for g in G)
    layouts = [(0,)] if D == 1 else [(1, 0), (0, 1)]
    for layout in layouts:
        doms = _domains(G, parts)
        mems = [_field(d, G, halos, layout, dtype, 3 * k) for k, d in enumerate(doms)]
        elem = np.dtype(dtype).itemsize
        specs = [orc.FieldSpec(m.copy(), elem, layout, offs, E) for m, offs, E in mems]
        pats = orc.regular_make_pattern([doms], gf, gl, halos, periodic)
        obufs = orc.regular_exchange([[(s, d.id, i, 0) for i, (s, d) in
                                       enumerate(zip(specs, doms))]], {0: pats}, 1)

        ctx = ghex_amd.make_context()
        dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in doms]
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, halos, periodic), dds)
        bases, fds = [], []
        for dd, (m, offs, E) in zip(dds, mems):
            base, logical = device_field(m, layout)
            bases.append(base)
            fds.append(R.make_field_descriptor(dd, logical, offs, E))
        co = R.make_communication_object(ctx, fuse_self=fused)
        bis = [pc(fd) for fd in fds]
        co.exchange(bis).wait()
        torch.cuda.synchronize()
        for base, spec in zip(bases, specs):
            np.testing.assert_array_equal(base.cpu().numpy(), spec.data)
        plan = co.plan(bis)
        send, _ = co.buffers(plan, bases[0].device)
        assert len(plan.send) == len(obufs)
        for b, t in zip(plan.send, send):
            ob = obufs[(0, tuple(b["pair"]))]
            assert b["size"] == ob.size
            np.testing.assert_array_equal(t[:ob.size].cpu().numpy(), ob)
