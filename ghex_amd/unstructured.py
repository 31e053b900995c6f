"""ghex_amd.unstructured — mirror of ghex.unstructured (bindings/python/src/ghex/unstructured.py)
on the MI355X-native path: index-list gather/scatter halos."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

from . import _ghx
from .communication_object import CommunicationObject
from .pattern import PatternContainer


def make_communication_object(context, **options) -> CommunicationObject:
    return CommunicationObject(context, **options)


class DomainDescriptor:
    """unstructured::domain_descriptor(id, gids, outer_lids)
    (include/ghex/unstructured/user_concepts.hpp:143-175): all global ids in storage order and
    the local ids of the outer (halo) cells."""

    def __init__(self, index: int, indices: Sequence[int], halo_indices: Sequence[int]):
        self._id = int(index)
        self.gids = [int(g) for g in indices]
        self.outer_lids = [int(l) for l in halo_indices]
        if len(set(self.outer_lids)) != len(self.outer_lids):
            raise RuntimeError("repeated outer (local) index")
        outer = set(self.outer_lids)
        inner = {}
        for lid, gid in enumerate(self.gids):
            if lid in outer:
                continue
            if gid in inner:
                raise RuntimeError("repeated inner (global) index")
            inner[gid] = lid
        self._inner = inner

    def domain_id(self) -> int:
        return self._id

    def size(self) -> int:
        return len(self.gids)

    def inner_size(self) -> int:
        return len(self._inner)


class HaloGenerator:
    """unstructured::halo_generator (user_concepts.hpp:234-253): all outer gids (default) or
    an explicit halo gid list."""

    def __init__(self, gids: Optional[Sequence[int]] = None):
        self.gids = None if gids is None else [int(g) for g in gids]

    @classmethod
    def from_gids(cls, gids):
        return cls(gids)


def make_pattern(context, halo_gen: HaloGenerator, domain_range: Sequence[DomainDescriptor]):
    """make_pattern<unstructured::grid> (include/ghex/unstructured/pattern.hpp:187-370)."""
    mine = [(d.domain_id(), d.gids, d.outer_lids, halo_gen.gids) for d in domain_range]
    gathered = context.all_gather_object(mine)
    ids, ranks, gids, gc, outer, oc, hg, hc = [], [], [], [], [], [], [], []
    for r, lst in enumerate(gathered):
        for (i, g, o, h) in lst:
            ids.append(i)
            ranks.append(r)
            gids += g
            gc.append(len(g))
            outer += o
            oc.append(len(o))
            if h is None:
                hc.append(-1)
            else:
                hg += h
                hc.append(len(h))
    p = ctypes.c_void_p()
    _ghx.call("ghx_unstructured_pattern_create", len(ids), _ghx.i32_array(ids),
              _ghx.i32_array(ranks), _ghx.i64_array(gids), _ghx.i64_array(gc),
              _ghx.i64_array(outer), _ghx.i64_array(oc), _ghx.i64_array(hg),
              _ghx.i64_array(hc), context.rank(), ctypes.byref(p))
    return PatternContainer(p.value, context, domain_range, "unstructured", 1)


class DataDescriptor:
    """unstructured::data_descriptor<gpu> (user_concepts.hpp:526-577) over a device tensor of
    shape (domain size,) or (domain size, levels); levels_first / outer stride derived from the
    strides exactly as bindings/python/src/_pyghex/unstructured/field_descriptor.cpp:66-131."""

    kind = 1

    def __init__(self, domain: DomainDescriptor, field):
        import torch
        if not isinstance(field, torch.Tensor) or field.device.type != "cuda":
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
