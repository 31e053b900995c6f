"""Pattern containers (include/ghex/pattern_container.hpp) over ghx_pattern handles."""
from __future__ import annotations

import ctypes

from . import _ghx


class PatternContainer:
    """pattern_container<grid, domain_id>: one pattern per local domain of this rank.

    Calling it on a field returns the buffer_info the communication object exchanges
    (pattern_container::operator(), include/ghex/pattern_container.hpp:88-95)."""

    grid_type = None  # "structured" | "unstructured"
    domain_id_type = "int"  # domain ids are int (the bindings' only instantiation)

    def __init__(self, handle: int, context, domains, kind: str, dim: int):
        self._h = ctypes.c_void_p(handle)
        self.context = context
        self.domains = list(domains)
        self.kind = kind
        self.grid_type = kind
        self.dim = dim
        n = ctypes.c_int32()
        _ghx.call("ghx_pattern_num_domains", self._h, ctypes.byref(n))
        self._n = n.value
        mt = ctypes.c_int32()
        _ghx.call("ghx_pattern_max_tag", self._h, ctypes.byref(mt))
        self._max_tag = mt.value

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if self._h:
                _ghx.lib().ghx_pattern_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def __len__(self):
        return self._n

    def max_tag(self) -> int:
        return self._max_tag

    def local_index(self, domain_id: int) -> int:
        for i in range(self._n):
            d = ctypes.c_int32()
            _ghx.call("ghx_pattern_domain_id", self._h, i, ctypes.byref(d))
            if d.value == domain_id:
                return i
        raise KeyError(f"domain {domain_id} is not a local domain of this pattern container")

    def _keys(self, local_index: int, direction: int):
        n = ctypes.c_int32()
        _ghx.call("ghx_pattern_num_keys", self._h, local_index, direction, ctypes.byref(n))
        out = []
        for k in range(n.value):
            rid, rr, tag, ns = (ctypes.c_int32() for _ in range(4))
            ne = ctypes.c_int64()
            _ghx.call("ghx_pattern_key", self._h, local_index, direction, k, ctypes.byref(rid),
                      ctypes.byref(rr), ctypes.byref(tag), ctypes.byref(ns), ctypes.byref(ne))
            out.append((k, rid.value, rr.value, tag.value, ns.value, ne.value))
        return out

    def halos(self, local_index: int, direction: int):
        """send (direction 0) / recv (1) halos of a local domain, in the reference's map order:
        [(remote_id, remote_rank, tag, spaces)], spaces = [(local_first, local_last,
        global_first, global_last)] (structured) or the lid list (unstructured)."""
        out = []
        for k, rid, rr, tag, ns, ne in self._keys(local_index, direction):
            if self.kind == "structured":
                loc = (_ghx.Box * max(1, ns))()
                glo = (_ghx.Box * max(1, ns))()
                _ghx.call("ghx_pattern_key_boxes", self._h, local_index, direction, k, loc, glo,
                          ns)
                sp = [(tuple(loc[i].first[:self.dim]), tuple(loc[i].last[:self.dim]),
                       tuple(glo[i].first[:self.dim]), tuple(glo[i].last[:self.dim]))
                      for i in range(ns)]
            else:
                arr = (ctypes.c_int64 * max(1, ne))()
                _ghx.call("ghx_pattern_key_lids", self._h, local_index, direction, k, arr, ne)
                sp = list(arr[:ne])
            out.append((rid, rr, tag, sp))
        return out

    def lid_arrays(self, local_index: int, direction: int):
        """Unstructured: halos(local_index, direction) with each lid list as an int64 numpy
        array (no Python list of ints)."""
        import numpy as np
        if self.kind == "structured":
            raise TypeError("lid_arrays is for unstructured patterns")
        out = []
        for k, rid, rr, tag, ns, ne in self._keys(local_index, direction):
            arr = np.empty(max(1, ne), dtype=np.int64)
            _ghx.call("ghx_pattern_key_lids", self._h, local_index, direction, k,
                      _ghx.i64_ptr(arr), ne)
            out.append((rid, rr, tag, arr[:ne]))
        return out

    def send_halos(self, local_index: int = 0):
        return self.halos(local_index, 0)

    def recv_halos(self, local_index: int = 0):
        return self.halos(local_index, 1)

    def __call__(self, field):
        return BufferInfo(self, field)

    def filtered(self, ranks, keep: bool) -> "PatternContainer":
        """The same pattern with only the halos to/from `ranks` (keep=True) or to/from every
        other rank (keep=False): the reference bulk object's local / remote pattern maps
        (include/ghex/bulk_communication_object.hpp:330-383)."""
        rs = [int(r) for r in ranks]
        h = ctypes.c_void_p()
        _ghx.call("ghx_pattern_filter", self._h, _ghx.i32_array(rs), len(rs), 1 if keep else 0,
                  ctypes.byref(h))
        return type(self)(h.value, self.context, self.domains, self.kind, self.dim)


class BufferInfo:
    """buffer_info<pattern, arch, field> (include/ghex/buffer_info.hpp)."""

    def __init__(self, pattern: PatternContainer, field):
        self.pattern_container = pattern
        self.field = field
        self.local_index = pattern.local_index(field.domain_id())

    def get_pattern_container(self):
        return self.pattern_container

    def get_field(self):
        return self.field
