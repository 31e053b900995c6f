"""ghex_amd.unstructured — mirror of ghex.unstructured (bindings/python/src/ghex/unstructured.py)
on the MI355X-native path: index-list gather/scatter halos."""
from __future__ import annotations

import ctypes
from typing import Sequence

from . import _ghx
from .communication_object import CommunicationObject
from .pattern import PatternContainer


def make_communication_object(context, **options) -> CommunicationObject:
    return CommunicationObject(context, **options)


class DomainDescriptor:
    """unstructured::domain_descriptor(id, gids, outer_lids)
    (include/ghex/unstructured/user_concepts.hpp:143-175): all global ids in storage order and
    the local ids of the outer (halo) cells. The gid -> lid maps live in libghx (ghx_udomain,
    flat hash tables built once); gids and outer lids are kept here as int64 numpy arrays."""

    def __init__(self, index: int, indices, halo_indices):
        import numpy as np
        self._id = int(index)
        self.gids = np.ascontiguousarray(indices, dtype=np.int64).reshape(-1)
        self.outer_lids = np.ascontiguousarray(halo_indices, dtype=np.int64).reshape(-1)
        h = ctypes.c_void_p()
        _ghx.call("ghx_udomain_create", self._id, _ghx.i64_ptr(self.gids), self.gids.size,
                  _ghx.i64_ptr(self.outer_lids), self.outer_lids.size, ctypes.byref(h))
        self._h = h
        inner = ctypes.c_int64()
        _ghx.call("ghx_udomain_info", h, None, None, ctypes.byref(inner), None)
        self._inner_size = inner.value

    def __del__(self):
        h = self.__dict__.get("_h")
        if h is not None and h.value and _ghx is not None and _ghx._lib is not None:
            _ghx._lib.ghx_udomain_destroy(h)
            self._h = None

    def domain_id(self) -> int:
        return self._id

    def size(self) -> int:
        return int(self.gids.size)

    def inner_size(self) -> int:
        return self._inner_size

    def halo_gids(self, halo_gen: "HaloGenerator"):
        """The reduced halo: gids of halo_gen(domain)'s local indices (pattern.hpp:247-254)."""
        import numpy as np
        g = halo_gen.gids
        cap = self.outer_lids.size if g is None else g.size
        out = np.empty(max(1, cap), dtype=np.int64)
        n = ctypes.c_int64()
        _ghx.call("ghx_udomain_halo", self._h, None if g is None else _ghx.i64_ptr(g),
                  -1 if g is None else g.size, _ghx.i64_ptr(out), cap, ctypes.byref(n))
        return out[:n.value]


class HaloGenerator:
    """unstructured::halo_generator (user_concepts.hpp:234-253): all outer gids (default) or
    an explicit halo gid list."""

    def __init__(self, gids=None):
        import numpy as np
        self.gids = None if gids is None else np.ascontiguousarray(gids, dtype=np.int64).reshape(-1)

    @classmethod
    def from_gids(cls, gids):
        return cls(gids)


def _agree(context, err, stage):
    """Every rank learns whether any rank failed at this setup stage (one all_gather of a short
    string): all raise together instead of the healthy ranks blocking in the next collective
    (ADVICE r05). A failing rank re-raises its own error; the others name the first failure."""
    why = context.all_gather_object(None if err is None else f"{type(err).__name__}: {err}")
    if err is not None:
        raise err
    bad = [(r, w) for r, w in enumerate(why) if w]
    if bad:
        raise RuntimeError(f"make_pattern<unstructured> ({stage}): rank {bad[0][0]} failed: "
                           f"{bad[0][1]}")


def make_pattern(context, halo_gen: HaloGenerator, domain_range: Sequence[DomainDescriptor]):
    """make_pattern<unstructured::grid> (include/ghex/unstructured/pattern.hpp:187-370), the
    reference's reduced-halo algorithm: this rank passes only its own domains; the ranks
    exchange their domains' halo gids (never their full gid lists), each rank resolves every
    halo against its own inner gids (its send halos) and ships the gids it found back to the
    halo's owner, which turns them into outer local ids (its receive halos). Collectives:
    `context.all_gather_object` (ids, record metadata), `context.ring_arrays` (reduced halos,
    the reference's distributed_for_each ring), `context.exchange_arrays` (gid lists, point to
    point)."""
    import numpy as np
    doms = list(domain_range)
    if not doms:
        raise ValueError("make_pattern needs at least one local domain")
    me = context.rank()
    ids = [d.domain_id() for d in doms]
    # tags from the global max domain id and max domains per rank (:218-233)
    meta = context.all_gather_object((max(ids), len(ids)))
    max_id = max(m[0] for m in meta)
    max_n = max(m[1] for m in meta)
    handles = (ctypes.c_void_p * len(doms))(*[d._h.value for d in doms])
    b = ctypes.c_void_p()
    err = None
    try:
        _ghx.call("ghx_upattern_create", handles, len(doms), me, max_n, max_id, ctypes.byref(b))
        # reduced halos of my domains: [n, ids..., sizes..., gids...] (:243-254)
        halos = [d.halo_gids(halo_gen) for d in doms]
        payload = np.concatenate([np.array([len(doms)], np.int64), np.array(ids, np.int64),
                                  np.array([h.size for h in halos], np.int64)] + halos)
    except Exception as e:  # every rank learns of it below, none is left in the ring
        err, payload = e, np.zeros(1, np.int64)
    _agree(context, err, "setup")
    p = ctypes.c_void_p()
    try:
        n_rec = ctypes.c_int64()
        # every rank's reduced halos, around the ring, against my inner gids -> send halos
        # (:284-330; at most two ranks' halos held at a time). A rank that fails on one step
        # keeps passing the arrays on, so its peers finish the ring and all raise together.
        for r, arr in context.ring_arrays(payload):
            if err is not None:
                continue
            try:
                k = int(arr[0])
                rid = np.ascontiguousarray(arr[1:1 + k], dtype=np.int32)
                sizes = np.ascontiguousarray(arr[1 + k:1 + 2 * k])
                gids = np.ascontiguousarray(arr[1 + 2 * k:])
                _ghx.call("ghx_upattern_add_halos", b, r, k,
                          rid.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          _ghx.i64_ptr(sizes), _ghx.i64_ptr(gids), ctypes.byref(n_rec))
            except Exception as e:
                err = e
        _agree(context, err, "send halos")
        recs, sends = [], []
        f = [ctypes.c_int32() for _ in range(4)]
        n = ctypes.c_int64()
        gp = ctypes.POINTER(ctypes.c_int64)()
        for k in range(n_rec.value):
            _ghx.call("ghx_upattern_record", b, k, *[ctypes.byref(x) for x in f],
                      ctypes.byref(n), ctypes.byref(gp))
            src_id, dst_id, dst_rank, tag = (x.value for x in f)
            recs.append((src_id, dst_id, dst_rank, tag, n.value))
            sends.append((dst_rank, np.ctypeslib.as_array(gp, shape=(n.value,)).copy()))
        # the records addressed to me, then the gid lists point to point (:337-365)
        every = context.all_gather_object(recs)
        mine = [(src, rec) for src, rs in enumerate(every) for rec in rs if rec[2] == me]
        got = context.exchange_arrays(sends, [(src, rec[4]) for src, rec in mine])
        try:
            for (src, (src_id, dst_id, _, tag, cnt)), g in zip(mine, got):
                g = np.ascontiguousarray(g, dtype=np.int64)
                _ghx.call("ghx_upattern_add_recv", b, src, src_id, dst_id, tag, _ghx.i64_ptr(g),
                          cnt)
            _ghx.call("ghx_upattern_finish", b, ctypes.byref(p))
        except Exception as e:
            err = e
        try:
            _agree(context, err, "receive halos")
        except Exception:
            if p.value:
                _ghx.lib().ghx_pattern_destroy(p)
            raise
    finally:
        if b.value:
            _ghx.lib().ghx_upattern_destroy(b)
    return PatternContainer(p.value, context, doms, "unstructured", 1)


class DataDescriptor:
    """unstructured::data_descriptor<gpu> (user_concepts.hpp:526-577) over a device tensor of
    shape (domain size,) or (domain size, levels); levels_first / outer stride derived from the
    strides exactly as bindings/python/src/_pyghex/unstructured/field_descriptor.cpp:66-131."""

    kind = 1

    def __init__(self, domain: DomainDescriptor, field):
        from .util import as_device_tensor
        field = as_device_tensor(field)
        if field.device.type != "cuda":
            raise TypeError("field must be a torch.Tensor in device memory")
        if field.dim() > 2:
            raise TypeError(f"Field has too many dimensions. Expected at most 2, but got {field.dim()}")
        if field.shape[0] != domain.size():
            raise TypeError(f"Field's first dimension ({field.shape[0]}) must match the size of "
                            f"the domain ({domain.size()})")
        T = field.element_size()
        s0 = field.stride(0) * T
        s1 = field.stride(1) * T if field.dim() == 2 else 0
        levels_first, outer = True, 0
        if field.dim() == 2 and s1 != T:
            levels_first = False
            if s0 != T:
                raise TypeError(f"Field's strides are not compatible with GHEX. Expected that the "
                                f"(byte) stride of dimension 0 is {T} but got {s0}.")
            if s1 % T:
                raise TypeError("Field's strides are not compatible with GHEX (dimension 1).")
            outer = s1 // T
        elif field.dim() == 2:
            if s0 % T:
                raise TypeError("Field's strides are not compatible with GHEX (dimension 0).")
            outer = s0 // T
        elif s0 != T:
            raise TypeError(f"Field's strides are not compatible with GHEX. With one dimension "
                            f"expected the stride to be {T} but got {s0}.")
        levels = 1 if field.dim() == 1 else int(field.shape[1])
        self.domain = domain
        self.tensor = field
        self.levels = levels
        self.levels_first = levels_first
        # data_descriptor ctor (user_concepts.hpp:556-566)
        self.index_stride = (outer if outer else levels) if levels_first else 1
        self.level_stride = 1 if levels_first else (outer if outer else domain.size())
        u = _ghx.UDataDesc()
        u.elem_size, u.levels, u.levels_first = T, levels, 1 if levels_first else 0
        u.index_stride, u.level_stride = self.index_stride, self.level_stride
        self.desc = u
        self.align = T

    def domain_id(self) -> int:
        return self.domain.domain_id()

    def num_components(self) -> int:
        return self.levels

    def data_ptr(self) -> int:
        return self.tensor.data_ptr()

    @property
    def device(self):
        return self.tensor.device


def make_field_descriptor(domain_desc: DomainDescriptor, field, *, arch=None):
    from .util import check_arch
    check_arch(arch)
    return DataDescriptor(domain_desc, field)


def wrap_field(*args, **kw):
    return make_field_descriptor(*args, **kw)
