"""ghex_amd.structured.regular — mirror of ghex.structured.regular
(bindings/python/src/ghex/structured/regular.py) on the MI355X-native path.

Structured regular grids: domain descriptors, the halo generator, make_pattern, field
descriptors over device tensors, and the communication object."""
from __future__ import annotations

import ctypes
from typing import Sequence

from .. import _ghx
from ..communication_object import CommunicationObject
from ..pattern import PatternContainer
from .cartesian_sets import IndexSpace, ProductSet, UnitRange, union  # noqa: F401 (re-exported)


def make_communication_object(context, **options) -> CommunicationObject:
    return CommunicationObject(context, **options)


def _corners(index_set):
    """(first, last) of a box given as the reference binding's index sets do it
    (bindings/python/src/ghex/structured/regular.py:31-38, 111-135): any object with `ndim` and
    corner indexing, set[(0,)*ndim] = first cell, set[(-1,)*ndim] = last cell (e.g. a
    cartesian_sets.ProductSet or ghex_amd.structured.cartesian_sets.ProductSet)."""
    nd = int(index_set.ndim)
    return (tuple(int(x) for x in index_set[(0,) * nd]),
            tuple(int(x) for x in index_set[(-1,) * nd]))


class DomainDescriptor:
    """structured::regular::domain_descriptor (include/ghex/structured/regular/domain_descriptor.hpp):
    an id and the inclusive global first/last coordinates of the owned box — given as
    (id, first, last), or as the reference binding does, (id, sub_domain_indices) with an index
    set (bindings/python/src/ghex/structured/regular.py:31-38)."""

    def __init__(self, id_: int, first, last: Sequence[int] = None):
        if last is None:
            first, last = _corners(first)
        self._id = int(id_)
        self._first = tuple(int(x) for x in first)
        self._last = tuple(int(x) for x in last)
        if len(self._first) != len(self._last) or not 1 <= len(self._first) <= 3:
            raise ValueError("first/last must have the same length 1..3")

    def domain_id(self) -> int:
        return self._id

    def first(self):
        return self._first

    def last(self):
        return self._last

    @property
    def ndim(self):
        return len(self._first)

    def __repr__(self):
        return f"DomainDescriptor({self._id}, {self._first}, {self._last})"


class HaloGenerator:
    """structured::regular::halo_generator (halo_generator.hpp:61-88).

    halos: per dimension an int or an (minus, plus) pair (the Python binding's canonical form,
    bindings/python/src/ghex/structured/regular.py:137-139), or the flat C++ list
    (dim0-, dim0+, dim1-, dim1+, ...)."""

    def __init__(self, global_first, global_last, halos, periodicity: Sequence[bool] = None):
        if periodicity is None:
            # the reference binding's form: (glob_domain_indices, halos, periodicity)
            # (bindings/python/src/ghex/structured/regular.py:111-135)
            global_first, global_last, halos, periodicity = (*_corners(global_first), global_last,
                                                             halos)
        self.global_first = tuple(int(x) for x in global_first)
        self.global_last = tuple(int(x) for x in global_last)
        D = len(self.global_first)
        if len(halos) == 2 * D and all(isinstance(h, int) for h in halos):
            flat = tuple(int(h) for h in halos)
        else:
            if len(halos) != D:
                raise ValueError("need one halo spec per dimension")
            flat = tuple(x for h in halos for x in ((h, h) if isinstance(h, int) else h))
        self.halos = flat
        self.periodic = tuple(bool(p) for p in periodicity)
        if len(self.periodic) != D:
            raise ValueError("need one periodicity flag per dimension")

    @property
    def ndim(self):
        return len(self.global_first)

    def __call__(self, domain: DomainDescriptor):
        """The receive boxes of `domain`: [(local_first, local_last, global_first, global_last)]."""
        D = self.ndim
        arr = _ghx.i32_array
        n = ctypes.c_int32()
        args = (D, arr(self.global_first), arr(self.global_last), arr(self.halos),
                arr([int(p) for p in self.periodic]), arr(domain.first()), arr(domain.last()))
        _ghx.call("ghx_regular_halo_boxes", *args, None, None, 0, ctypes.byref(n))
        loc = (_ghx.Box * max(1, n.value))()
        glo = (_ghx.Box * max(1, n.value))()
        _ghx.call("ghx_regular_halo_boxes", *args, loc, glo, n.value, ctypes.byref(n))
        boxes = HaloBoxes((tuple(loc[i].first[:D]), tuple(loc[i].last[:D]),
                           tuple(glo[i].first[:D]), tuple(glo[i].last[:D])) for i in range(n.value))
        boxes.ndim = D
        return boxes


class HaloBoxes(list):
    """The receive boxes of a domain, [(local_first, local_last, global_first, global_last)] in
    generation order; `.local` / `.global_` are the two halves of the reference binding's
    HaloContainer (bindings/python/src/ghex/structured/regular.py:105-154): each the union of
    the boxes as one index set (cartesian_sets.union, simplified like the reference's)."""

    ndim = 3

    def _set(self, lo, hi):
        if not self:
            return ProductSet(*([UnitRange(0, 0)] * self.ndim))
        return union(*(ProductSet.from_coords(b[lo], b[hi]) for b in self))

    @property
    def local(self):
        return self._set(0, 1)

    @property
    def global_(self):
        return self._set(2, 3)


def make_pattern(context, halo_gen: HaloGenerator, domain_range: Sequence[DomainDescriptor]):
    """make_pattern<structured::grid>(context, halo_gen, domains)
    (include/ghex/pattern_container.hpp:112-120; structured/pattern.hpp:214-571).

    The domains of all ranks are all-gathered once (setup), then this rank's send/recv maps are
    derived locally in libghx."""
    D = halo_gen.ndim
    mine = [(d.domain_id(), d.first(), d.last()) for d in domain_range]
    gathered = context.all_gather_object(mine)
    doms = []
    for r, lst in enumerate(gathered):
        for (i, f, l) in lst:
            rd = _ghx.RegularDomain()
            rd.id, rd.rank = i, r
            for k in range(D):
                rd.first[k], rd.last[k] = f[k], l[k]
            doms.append(rd)
    darr = (_ghx.RegularDomain * len(doms))(*doms)
    h = ctypes.c_void_p()
    arr = _ghx.i32_array
    _ghx.call("ghx_regular_pattern_create", D, darr, len(doms), arr(halo_gen.global_first),
              arr(halo_gen.global_last), arr(halo_gen.halos),
              arr([int(p) for p in halo_gen.periodic]), context.rank(), ctypes.byref(h))
    return PatternContainer(h.value, context, domain_range, "structured", D)


def make_staged_pattern(context, domain_range: Sequence[DomainDescriptor], domain_lookup,
                        global_first, global_last, halos, periodicity):
    """make_staged_pattern(ctx, domains, d_lu, g_first, g_last, halos, periodic)
    (include/ghex/structured/regular/make_pattern.hpp:47-250): one pattern container per
    dimension; exchanging them in order (stage 0, then 1, ...) fills the whole halo including
    edges and corners, stage i moving the dimension-i slabs over the box already extended by the
    halos of the earlier stages.

    domain_lookup(domain_id, offset) -> the neighbour at `offset` (a tuple with one -1/+1 entry):
    an object with id() (and rank()), an (id, rank) pair, or an id. halos as for HaloGenerator
    (per dimension an int or a (minus, plus) pair, or the flat list). Each rank evaluates the
    look-up for its own domains; the tables are all-gathered once (the reference exchanges tag
    lists over MPI instead, make_pattern.hpp:218-227)."""
    hg = HaloGenerator(global_first, global_last, halos, periodicity)
    D = hg.ndim

    def nid(x):
        if x is None:
            return -1
        if hasattr(x, "id"):
            return int(x.id() if callable(x.id) else x.id)
        if isinstance(x, (tuple, list)):
            return int(x[0])
        return int(x)

    mine = []
    for d in domain_range:
        if d.ndim != D:
            raise ValueError("domain and halo dimensions differ")
        nb = []
        for i in range(D):
            for side in (-1, 1):
                off = [0] * D
                off[i] = side
                h = hg.halos[2 * i + (0 if side < 0 else 1)]
                nb.append(nid(domain_lookup(d.domain_id(), tuple(off))) if h > 0 else -1)
        mine.append((d.domain_id(), d.first(), d.last(), nb))
    gathered = context.all_gather_object(mine)
    doms, nbrs = [], []
    for r, lst in enumerate(gathered):
        for (i, f, l, nb) in lst:
            rd = _ghx.RegularDomain()
            rd.id, rd.rank = i, r
            for k in range(D):
                rd.first[k], rd.last[k] = f[k], l[k]
            doms.append(rd)
            nbrs.extend(nb)
    darr = (_ghx.RegularDomain * len(doms))(*doms)
    hs = (ctypes.c_void_p * D)()
    arr = _ghx.i32_array
    _ghx.call("ghx_staged_pattern_create", D, darr, len(doms), arr(nbrs), arr(hg.global_first),
              arr(hg.global_last), arr(hg.halos), arr([int(p) for p in hg.periodic]),
              context.rank(), hs)
    return [PatternContainer(hs[i], context, domain_range, "structured", D) for i in range(D)]


def _layout_order(strides) -> tuple:
    """Layout map from strides (bindings/python/src/ghex/structured/regular.py:41-63): the
    largest stride gets 0, the smallest gets dim-1; ties broken to keep values unique."""
    ordered = list(reversed(sorted(strides)))
    layout = [ordered.index(s) for s in strides]
    for i, v in enumerate(layout):
        if v in layout[:i]:
            layout[i] = max(layout) + 1
    return tuple(layout)


class FieldDescriptor:
    """structured::regular::field_descriptor over a device tensor
    (include/ghex/structured/field_descriptor.hpp:21-269, regular/field_descriptor.hpp).

    `pack(buffer, spaces, stream)` / `unpack(...)` are the field-descriptor concept's member
    functions (doc_src/scope/scope.rst:356-359), executed by libghx on the device."""

    kind = 0

    def __init__(self, domain: DomainDescriptor, field, offsets, extents, num_components=None):
        from ..util import as_device_tensor
        field = as_device_tensor(field)
        if field.device.type != "cuda":
            raise TypeError("ghex_amd fields live in device memory (torch device 'cuda')")
        D = domain.ndim
        nd = field.dim()
        if nd not in (D, D + 1):
            raise ValueError(f"field has {nd} dims, domain has {D}")
        self.domain = domain
        self.tensor = field
        self.has_components = nd == D + 1
        self.num_components = int(field.shape[-1]) if self.has_components else 1
        if num_components is not None and num_components != self.num_components:
            raise ValueError("num_components does not match the field's last dimension")
        itemsize = field.element_size()
        strides = tuple(int(s) * itemsize for s in field.stride())
        self.layout = _layout_order(strides)
        offs = list(offsets) + ([0] if self.has_components else [])
        exts = list(extents) + ([self.num_components] if self.has_components else [])
        if len(offs) != nd or len(exts) != nd:
            raise ValueError("offsets/extents must have one entry per spatial dimension")
        for d in range(nd):
            if int(field.shape[d]) < exts[d]:
                raise ValueError("field smaller than its declared extents")
        fd = _ghx.FieldDesc()
        fd.dim, fd.elem_size = nd, itemsize
        for d in range(nd):
            fd.layout[d] = self.layout[d]
            fd.byte_strides[d] = strides[d]
            fd.offsets[d] = int(offs[d])
            fd.extents[d] = int(exts[d])
        fd.num_components = self.num_components
        fd.has_components = 1 if self.has_components else 0
        self.desc = fd
        self.align = itemsize  # alignof(T) of the scalar element types the bindings register
        self.offsets = tuple(offs)
        self.extents = tuple(exts)

    def domain_id(self) -> int:
        return self.domain.domain_id()

    def data_ptr(self) -> int:
        return self.tensor.data_ptr()

    @property
    def device(self):
        return self.tensor.device

    def _boxes(self, spaces):
        arr = (_ghx.Box * max(1, len(spaces)))()
        for i, sp in enumerate(spaces):
            lf, ll = sp[0], sp[1]
            for d in range(len(lf)):
                arr[i].first[d], arr[i].last[d] = lf[d], ll[d]
        return arr

    def pack(self, buffer, spaces, stream=None):
        """field.pack(buffer, index_container, stream): spaces back to back into `buffer`
        (a device tensor or pointer), enqueued on `stream` (torch stream; None = current)."""
        import torch
        s = (stream or torch.cuda.current_stream()).cuda_stream
        bp = buffer.data_ptr() if hasattr(buffer, "data_ptr") else int(buffer)
        _ghx.call("ghx_structured_pack", ctypes.byref(self.desc), self.data_ptr(), bp,
                  self._boxes(spaces), len(spaces), s)

    def unpack(self, buffer, spaces, stream=None):
        import torch
        s = (stream or torch.cuda.current_stream()).cuda_stream
        bp = buffer.data_ptr() if hasattr(buffer, "data_ptr") else int(buffer)
        _ghx.call("ghx_structured_unpack", ctypes.byref(self.desc), self.data_ptr(), bp,
                  self._boxes(spaces), len(spaces), s)


def make_field_descriptor(domain_desc: DomainDescriptor, field, offsets, extents, *, arch=None):
    """make_field_descriptor(domain, field, offsets, extents)
    (bindings/python/src/ghex/structured/regular.py:66-107): the layout map is derived from the
    tensor's strides. Only device (GPU) fields: this package is the device hot path."""
    from ..util import check_arch
    check_arch(arch)
    return FieldDescriptor(domain_desc, field, offsets, extents)


def wrap_field(*args, **kw):
    return make_field_descriptor(*args, **kw)
