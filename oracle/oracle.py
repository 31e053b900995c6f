"""oracle.py — TEST INFRASTRUCTURE ONLY: the CPU parity oracle for the halo pack/unpack path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module. The product (``ghex_amd``/``libghx.so``) never imports, links or calls it and has
no CPU fallback.

Two halves:
  * byte movement (pack/unpack) is plain C in ``ghex_oracle.c``, loaded here with ctypes from
    ``oracle/build/libghex_oracle.so`` (built by ``oracle/Makefile``);
  * the setup-time logic that fixes the buffer byte layout — the regular halo generator, the
    structured ``make_pattern`` intersection / tag / send-box order, the communication object's
    buffer planning and the unstructured pattern — is restated below in pure Python (small
    integer loops over ≤ 3^D boxes x domains). Each function cites the reference lines it follows.

Pinning (see oracle/README.md): ``regular_halo_boxes`` and ``intersect`` are checked against the
reference's own ``halo_generator`` compiled from /root/reference (oracle/ref_halo_boxes.cpp ->
tests/golden/ref_halo_boxes.json). The unstructured pattern is checked against the known-answer
tables of test/unstructured/unstructured_test_case.hpp:217-343 (tests/golden/unstructured_case.json).
Byte-level buffer contents have no reference golden file (the reference tests are
self-validating); the structured exchange is pinned by the reference tests' own property —
every halo cell equals the periodic-wrapped global coordinate after an exchange
(test/structured/regular/test_regular_domain.cpp:739-800).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field as dc_field
from typing import Dict, List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libghex_oracle.so")
_lib = None


def lib():
    """Load the compiled C oracle (build it with ``make -C oracle``)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle library missing: {_LIB_PATH} (run make -C oracle)")
        L = ctypes.CDLL(_LIB_PATH)
        i64, i32p, i64p, vp = ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), \
            ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p
        for name in ("orc_structured_pack", "orc_structured_unpack"):
            fn = getattr(L, name)
            fn.restype = i64
            fn.argtypes = [vp, vp, ctypes.c_int, i64, i32p, i64p, i32p, i32p, ctypes.c_int,
                           ctypes.c_int]
        for name in ("orc_unstructured_get", "orc_unstructured_set"):
            fn = getattr(L, name)
            fn.restype = i64
            fn.argtypes = [vp, vp, i64, i64p, i64, i64, ctypes.c_int, i64, i64]
        L.orc_fnv1a64.restype = ctypes.c_uint64
        L.orc_fnv1a64.argtypes = [vp, i64, ctypes.c_uint64]
        _lib = L
    return _lib


def _i32(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int32))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _i64(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int64))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


# --------------------------------------------------------------------------------------------
# structured, regular: halo generator (include/ghex/structured/regular/halo_generator.hpp)
# --------------------------------------------------------------------------------------------
Box = Tuple[Tuple[int, ...], Tuple[int, ...]]  # (first, last), inclusive


@dataclass
class Box2:
    """halo_generator::box2 (halo_generator.hpp:51-59): local and global boxes."""
    lf: Tuple[int, ...]
    ll: Tuple[int, ...]
    gf: Tuple[int, ...]
    gl: Tuple[int, ...]

    @property
    def size(self) -> int:
        s = 1
        for a, b in zip(self.lf, self.ll):
            s *= b - a + 1
        return s


def _cmod(a: int, b: int) -> int:
    """C/C++ integer remainder (truncating division): the sign follows the dividend."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def regular_halo_boxes(gfirst, glast, halos, periodic, dfirst, dlast) -> List[Box2]:
    """halo_generator::operator() (halo_generator.hpp:93-148).

    Three 1-D spaces per dimension {left, middle, right}; boxes enumerated by compute_spaces
    (:163-197) with dimension 0 outermost; the centre box (index 3^D/2) and empty boxes
    (any local last < first) dropped (:124-131); then periodic wrap of the global coordinates
    (:133-145). Halos are (dim0-, dim0+, dim1-, dim1+, ...)."""
    D = len(dfirst)
    left, mid, right = [], [], []
    for d in range(D):
        lf = -halos[2 * d]
        left.append((lf, -1, lf + dfirst[d], dfirst[d] - 1))
        mid.append((0, dlast[d] - dfirst[d], dfirst[d], dlast[d]))
        rf = dlast[d] - dfirst[d] + 1
        right.append((rf, dlast[d] - dfirst[d] + halos[2 * d + 1], dlast[d] + 1,
                      dlast[d] + halos[2 * d + 1]))
    spaces = (left, mid, right)
    out = []
    centre = 3 ** D // 2
    for j in range(3 ** D):
        if j == centre:
            continue
        digits = []
        r = j
        for _ in range(D):
            digits.append(r % 3)
            r //= 3
        digits = digits[::-1]  # digit for dim 0 is the most significant
        lf = tuple(spaces[digits[d]][d][0] for d in range(D))
        ll = tuple(spaces[digits[d]][d][1] for d in range(D))
        gf = tuple(spaces[digits[d]][d][2] for d in range(D))
        gl = tuple(spaces[digits[d]][d][3] for d in range(D))
        if all(ll[d] >= lf[d] for d in range(D)):
            out.append(Box2(lf, ll, gf, gl))
    for b in out:
        gf, gl = list(b.gf), list(b.gl)
        for d in range(D):
            if not periodic[d]:
                continue
            ext_h = gl[d] - gf[d]
            ext = glast[d] + 1 - gfirst[d]
            off = gf[d] - gfirst[d]
            # C++ `%` truncates toward zero: a box starting more than one period before the
            # domain keeps a negative offset (halo_generator.hpp:139-141), unlike Python's `%`
            gf[d] = _cmod(off + ext, ext) + gfirst[d]
            gl[d] = gf[d] + ext_h
        b.gf, b.gl = tuple(gf), tuple(gl)
    return out


def intersect(lf_a, gf_a, gl_a, gf_b, gl_b) -> Box2:
    """halo_generator::intersect (halo_generator.hpp:150-160)."""
    gf = tuple(max(a, b) for a, b in zip(gf_a, gf_b))
    gl = tuple(min(a, b) for a, b in zip(gl_a, gl_b))
    lf = tuple(l + (g - ga) for l, g, ga in zip(lf_a, gf, gf_a))
    ll = tuple(l + (g - ga) for l, g, ga in zip(lf_a, gl, gf_a))
    return Box2(lf, ll, gf, gl)


# --------------------------------------------------------------------------------------------
# structured make_pattern over all ranks (include/ghex/structured/pattern.hpp:214-571)
# --------------------------------------------------------------------------------------------
@dataclass
class RegularDomain:
    id: int
    first: Tuple[int, ...]
    last: Tuple[int, ...]


@dataclass
class ISPair:
    """pattern::iteration_space_pair (pattern.hpp:95-120)."""
    lf: Tuple[int, ...]
    ll: Tuple[int, ...]
    gf: Tuple[int, ...]
    gl: Tuple[int, ...]

    def size(self) -> int:
        s = 1
        for a, b in zip(self.lf, self.ll):
            s *= b - a + 1
        return s


@dataclass
class RegularPattern:
    """pattern<structured grid> for one local domain: maps keyed by (id, tag) -> (rank, [ISPair]).

    Key ordering follows extended_domain_id_type::operator< (pattern.hpp:133-136): (id, tag)."""
    domain_id: int
    rank: int
    recv: Dict[Tuple[int, int], Tuple[int, List[ISPair]]] = dc_field(default_factory=dict)
    send: Dict[Tuple[int, int], Tuple[int, List[ISPair]]] = dc_field(default_factory=dict)
    max_tag: int = 0

    def recv_items(self):
        return sorted(self.recv.items())

    def send_items(self):
        return sorted(self.send.items())


def regular_make_pattern(ranks_domains: Sequence[Sequence[RegularDomain]], gfirst, glast, halos,
                         periodic) -> List[List[RegularPattern]]:
    """All-ranks restatement of make_pattern_impl<structured grid>::apply.

    ranks_domains[r] = rank r's domains in its d_range order. Returns patterns[r][i]."""
    world = len(ranks_domains)
    pats = [[RegularPattern(d.id, r) for d in doms] for r, doms in enumerate(ranks_domains)]
    # recv halos: per my domain, per generated box, per rank j, per domain k (pattern.hpp:293-329)
    for r, doms in enumerate(ranks_domains):
        for i, d in enumerate(doms):
            boxes = regular_halo_boxes(gfirst, glast, halos, periodic, d.first, d.last)
            recv: Dict[int, Tuple[int, List[ISPair]]] = {}
            for b in boxes:
                for j in range(world):
                    for od in ranks_domains[j]:
                        x = intersect(b.lf, b.gf, b.gl, od.first, od.last)
                        if all(f <= l for f, l in zip(x.gf, x.gl)):
                            ent = recv.setdefault(od.id, (j, []))
                            ent[1].append(ISPair(x.lf, x.ll, x.gf, x.gl))
            # keys are (id, tag=0) during insertion: std::map order by id
            pats[r][i].recv = {(k, 0): v for k, v in sorted(recv.items())}
    # tags: per (receiver rank, remote rank), 0, 1, ... in map order over my patterns
    # (pattern.hpp:331-367)
    max_tag = 0
    for r in range(world):
        tag_map: Dict[int, int] = {}
        for p in pats[r]:
            new = {}
            for (rid, _), (rrank, lst) in sorted(p.recv.items()):
                if rrank not in tag_map:
                    tag_map[rrank] = 0
                    tag = 0
                else:
                    tag_map[rrank] += 1
                    tag = tag_map[rrank]
                    max_tag = max(max_tag, tag)
                new[(rid, tag)] = (rrank, lst)
            p.recv = new
    # send halos: receiver's lists translated to the sender's local coords (pattern.hpp:369-567)
    for r in range(world):
        for p in pats[r]:
            for (rid, tag), (rrank, lst) in sorted(p.recv.items()):
                k = [d.id for d in ranks_domains[rrank]].index(rid)
                od = ranks_domains[rrank][k]
                sp = pats[rrank][k]
                key = (p.domain_id, tag)
                ent = sp.send.setdefault(key, (r, []))
                for isp in lst:
                    lf = tuple(g - f for g, f in zip(isp.gf, od.first))
                    ll = tuple(g - f for g, f in zip(isp.gl, od.first))
                    ent[1].append(ISPair(lf, ll, isp.gf, isp.gl))
    for r in range(world):
        for p in pats[r]:
            p.max_tag = max_tag
    return pats


def staged_make_pattern(ranks_domains: Sequence[Sequence[RegularDomain]], lookup, gfirst, glast,
                        halos, periodic) -> List[List[List[RegularPattern]]]:
    """All-ranks restatement of structured::regular::make_staged_pattern
    (include/ghex/structured/regular/make_pattern.hpp:47-250). lookup(id, offset) -> neighbour id.
    Returns stages[i][r][k]: stage i exchanges the dimension-i slabs over the domain box extended
    by the halos of stages < i (:90-181); tags per receiving rank and remote rank in pattern and
    key order (:199-214); senders take the receiver's tag for (sender id, receiver id)
    (:229-243); max_tag is the rank's own (:201, 227)."""
    D = len(gfirst)
    rank_of = {d.id: r for r, doms in enumerate(ranks_domains) for d in doms}
    stages = [[[RegularPattern(d.id, r) for d in doms] for r, doms in enumerate(ranks_domains)]
              for _ in range(D)]
    raw = {}  # (stage, id) -> (recv {neighbour id: [ISPair]}, send {neighbour id: [ISPair]})
    for doms in ranks_domains:
        for d in doms:
            lf = [0] * D
            ll = [d.last[c] - d.first[c] for c in range(D)]
            gf, gl = list(d.first), list(d.last)
            for i in range(D):
                hl, hr = halos[2 * i], halos[2 * i + 1]
                has_left = hl > 0 and (periodic[i] or gf[i] - hl >= gfirst[i])
                has_right = hr > 0 and (periodic[i] or gl[i] + hr <= glast[i])
                recv, send = {}, {}

                def box(a, b, c, e, dim=i):
                    x = [list(lf), list(ll), list(gf), list(gl)]
                    x[0][dim], x[1][dim], x[2][dim], x[3][dim] = a, b, c, e
                    return ISPair(*(tuple(t) for t in x))
                off_l = tuple(-1 if c == i else 0 for c in range(D))
                off_r = tuple(1 if c == i else 0 for c in range(D))
                if has_left:
                    left = lookup(d.id, off_l)
                    recv.setdefault(left, []).append(
                        box(lf[i] - hl, lf[i] - 1, gf[i] - hl, gf[i] - 1))
                if has_right:
                    right = lookup(d.id, off_r)
                    if hl > 0:  # hl = 0: empty, never received (the reference keys it and
                        # its tag hand-off, make_pattern.hpp:219-243, then waits forever)
                        send.setdefault(right, []).append(
                            box(ll[i] + 1 - hl, ll[i], gl[i] + 1 - hl, gl[i]))
                    recv.setdefault(right, []).append(
                        box(ll[i] + 1, ll[i] + hr, gl[i] + 1, gl[i] + hr))
                if has_left:
                    if hr > 0:  # (hr = 0: as send_right above)
                        send.setdefault(left, []).append(
                            box(lf[i], lf[i] - 1 + hr, gf[i], gf[i] - 1 + hr))
                    lf[i] -= hl
                    gf[i] -= hl
                if has_right:
                    ll[i] += hr
                    gl[i] += hr
                raw[(i, d.id)] = (recv, send)
    for i in range(D):
        tag_of = {}
        for r, doms in enumerate(ranks_domains):
            last, mt = {}, 0
            for d in doms:
                for nid in sorted(raw[(i, d.id)][0]):
                    rr = rank_of[nid]
                    last[rr] = last[rr] + 1 if rr in last else 0
                    tag_of[(nid, d.id)] = last[rr]
                    mt = max(mt, last[rr])
            for p in stages[i][r]:
                p.max_tag = mt
        for r, doms in enumerate(ranks_domains):
            for k, d in enumerate(doms):
                recv, send = raw[(i, d.id)]
                p = stages[i][r][k]
                p.recv = {(nid, tag_of[(nid, d.id)]): (rank_of[nid], recv[nid])
                          for nid in sorted(recv)}
                p.send = {(nid, tag_of[(d.id, nid)]): (rank_of[nid], send[nid])
                          for nid in sorted(send)}
    return stages


# --------------------------------------------------------------------------------------------
# buffer planning: communication_object::allocate (communication_object.hpp:1003-1067)
# --------------------------------------------------------------------------------------------
@dataclass
class PlannedField:
    field_index: int          # position in the exchange() argument list
    offset: int               # byte offset in the message (alignment-padded)
    boxes: List[ISPair]       # the iteration spaces (pattern order)


@dataclass
class PlannedBuffer:
    pair: Tuple[int, int]     # domain_id_pair (first, second)
    rank: int
    tag: int
    size: int = 0
    fields: List[PlannedField] = dc_field(default_factory=list)


def plan_buffers(items, receive: bool):
    """items: [(field_index, my_dom_id, pattern, elem_size, align, num_components, tag_offset)].

    Returns {domain_id_pair: PlannedBuffer} in std::map order (pair ordering :165-174)."""
    mem: Dict[Tuple[int, int], PlannedBuffer] = {}
    for fi, my_id, pat, elem, align, nc, tag_off in items:
        halos = pat.recv_items() if receive else pat.send_items()
        for (rid, tag), (rrank, lst) in halos:
            n = sum(isp.size() for isp in lst) * nc
            if n < 1:
                continue
            pair = (my_id, rid) if receive else (rid, my_id)
            b = mem.get(pair)
            if b is None:
                b = mem[pair] = PlannedBuffer(pair, rrank, tag + tag_off)
            elif b.size == 0:
                b.rank, b.tag, b.fields = rrank, tag + tag_off, []
            prev = b.size
            pad = ((prev + align - 1) // align) * align - prev
            b.fields.append(PlannedField(fi, prev + pad, lst))
            b.size += pad + n * elem
    return dict(sorted(mem.items()))


# --------------------------------------------------------------------------------------------
# field description + pack/unpack through the C oracle
# --------------------------------------------------------------------------------------------
@dataclass
class FieldSpec:
    """A wrapped field (structured::field_descriptor, field_descriptor.hpp:152-197)."""
    data: np.ndarray          # the raw storage (any dtype; bytes are what matter)
    elem: int                 # sizeof(T)
    layout: Tuple[int, ...]   # layout_map values per dim (incl. component dim)
    offsets: Tuple[int, ...]
    extents: Tuple[int, ...]
    byte_strides: Tuple[int, ...] = None
    num_components: int = 1
    has_components: bool = False

    def __post_init__(self):
        if self.byte_strides is None:
            self.byte_strides = default_byte_strides(self.layout, self.extents, self.elem)

    @property
    def D(self):
        return len(self.layout)


def default_byte_strides(layout, extents, elem):
    """compute_strides<D>::apply<layout,T>(extents, strides, 0) (field_utils.hpp:96-112)."""
    D = len(layout)
    find = {v: d for d, v in enumerate(layout)}
    bs = [0] * D
    bs[find[D - 1]] = elem
    for k in range(D - 1, 0, -1):
        bs[find[k - 1]] = bs[find[k]] * extents[find[k]]
    return tuple(bs)


def expand_boxes(f: FieldSpec, boxes: Sequence[ISPair]) -> np.ndarray:
    """make_is (regular/field_descriptor.hpp:131-150): add the component axis [0, nc-1]."""
    rows = []
    for b in boxes:
        lf, ll = list(b.lf), list(b.ll)
        if f.has_components:
            lf.append(0)
            ll.append(f.num_components - 1)
        rows.append(lf + ll)
    return np.array(rows, dtype=np.int32).reshape(-1)


def structured_pack(f: FieldSpec, buffer: np.ndarray, boxes: Sequence[ISPair], byte_offset=0,
                    elementwise=False) -> int:
    L = lib()
    lay, lay_p = _i32(f.layout)
    bs, bs_p = _i64(f.byte_strides)
    off, off_p = _i32(f.offsets)
    bx, bx_p = _i32(expand_boxes(f, boxes))
    assert buffer.flags.c_contiguous  # the field may be any strided view: byte_strides rule
    return L.orc_structured_pack(f.data.ctypes.data, buffer.ctypes.data + byte_offset, f.D, f.elem,
                                 lay_p, bs_p, off_p, bx_p, len(boxes), 1 if elementwise else 0)


def structured_unpack(f: FieldSpec, buffer: np.ndarray, boxes: Sequence[ISPair], byte_offset=0,
                      elementwise=False) -> int:
    L = lib()
    lay, lay_p = _i32(f.layout)
    bs, bs_p = _i64(f.byte_strides)
    off, off_p = _i32(f.offsets)
    bx, bx_p = _i32(expand_boxes(f, boxes))
    return L.orc_structured_unpack(f.data.ctypes.data, buffer.ctypes.data + byte_offset, f.D,
                                   f.elem, lay_p, bs_p, off_p, bx_p, len(boxes),
                                   1 if elementwise else 0)


def fnv1a64(arr: np.ndarray, h: int = 0) -> int:
    a = np.ascontiguousarray(arr)
    return int(lib().orc_fnv1a64(a.ctypes.data, a.nbytes, h))


def regular_exchange(ranks_fields, patterns, n_ranks):
    """Full-exchange oracle for a structured exchange() over all ranks in one process.

    ranks_fields[r] = [(FieldSpec, my_domain_id, local_domain_index, pattern_container_id)]
    in exchange() argument order; patterns[pc][r][i] = RegularPattern.
    Packs every send buffer (communication_object::pack, :568-597), routes each message by
    (sender domain pair, tag), unpacks (packer<cpu>::unpack). Returns the send buffers so that
    byte-level parity can be checked: {(rank, pair): bytes}."""
    # tag offsets per pattern container (prepare_exchange_buffers :540-549)
    send_bufs, recv_plans = {}, {}
    for r in range(n_ranks):
        tag_off, pc_off, mt = {}, 0, 0
        for (_, _, _, pc) in ranks_fields[r]:
            if pc not in tag_off:
                tag_off[pc] = pc_off
                pc_off += patterns[pc][r][0].max_tag + 1
        send_items, recv_items = [], []
        for k, (f, dom_id, li, pc) in enumerate(ranks_fields[r]):
            p = patterns[pc][r][li]
            align = f.data.dtype.alignment
            send_items.append((k, dom_id, p, f.elem, align, f.num_components, tag_off[pc]))
            recv_items.append((k, dom_id, p, f.elem, align, f.num_components, tag_off[pc]))
        sp = plan_buffers(send_items, receive=False)
        rp = plan_buffers(recv_items, receive=True)
        for pair, b in sp.items():
            buf = np.zeros(b.size, dtype=np.uint8)
            for pf in b.fields:
                structured_pack(ranks_fields[r][pf.field_index][0], buf, pf.boxes, pf.offset)
            send_bufs[(r, pair)] = (b, buf)
        recv_plans[r] = rp
    for r in range(n_ranks):
        for pair, b in recv_plans[r].items():
            # the sender's send key is {remote(=me), my(=sender)} == my recv pair (:1032-1043)
            sb, buf = send_bufs[(b.rank, pair)]
            assert sb.size == b.size and sb.tag == b.tag, (sb, b)
            for pf in b.fields:
                structured_unpack(ranks_fields[r][pf.field_index][0], buf, pf.boxes, pf.offset)
    return {k: v[1] for k, v in send_bufs.items()}


# --------------------------------------------------------------------------------------------
# unstructured (include/ghex/unstructured/user_concepts.hpp, pattern.hpp)
# --------------------------------------------------------------------------------------------
class UnstructuredDomain:
    """unstructured::domain_descriptor (user_concepts.hpp:37-176)."""

    def __init__(self, id_, gids, outer_lids):
        self.id = id_
        self.gids = list(gids)
        outer = set()
        for l in outer_lids:
            if l in outer:
                raise RuntimeError("repeated outer (local) index")
            outer.add(l)
        self.inner: Dict[int, int] = {}
        # unordered_multimap: libstdc++ inserts an equal key in FRONT of its equal range,
        # so equal_range yields reverse insertion order (_M_insert_multi_node)
        self.outer: Dict[int, List[int]] = {}
        self.outer_gids = []
        for lid, gid in enumerate(self.gids):
            if lid in outer:
                self.outer.setdefault(gid, []).insert(0, lid)
                self.outer_gids.append(gid)
            else:
                if gid in self.inner:
                    raise RuntimeError("repeated inner (global) index")
                self.inner[gid] = lid

    def size(self):
        return len(self.gids)

    def make_outer_lids(self, gids):
        """domain_descriptor::make_outer_lids (user_concepts.hpp:88-113)."""
        lids, count = [], {}
        for gid in gids:
            rng = self.outer.get(gid)
            if rng is None:
                continue
            if gid in count:
                count[gid] += 1
                if count[gid] >= len(rng):
                    raise RuntimeError("halo gid does not have an associated lid in the domain")
                lids.append(rng[count[gid]])
            else:
                count[gid] = 0
                lids.append(rng[0])
        for gid, c in count.items():
            if c + 1 != len(self.outer[gid]):
                raise RuntimeError("halo gid occurs not often enough")
        return lids


def _num_bits(n):
    return 1 if n == 0 else 1 + _num_bits(n >> 1)


def unstructured_make_pattern(ranks_domains, ranks_halo_gids=None):
    """All-ranks restatement of make_pattern_impl<unstructured grid>::apply (no hints)
    (unstructured/pattern.hpp:187-370). ranks_halo_gids[r][i] = explicit halo gids of the
    halo_generator (None = all outer gids, user_concepts.hpp:244-252).

    Returns pats[r][i] = {"send": {(rank, tag): (id, lids)}, "recv": {(rank, tag): (id, lids)}}
    with keys ordered by (mpi_rank, tag) (pattern.hpp:105-110)."""
    world = len(ranks_domains)
    max_num_domains = max(len(ds) for ds in ranks_domains)
    shift = _num_bits(max_num_domains)

    def make_tag(src_local_idx, tgt_id):
        return (src_local_idx << shift) | tgt_id

    pats = [[{"id": d.id, "send": {}, "recv": {}} for d in ds] for ds in ranks_domains]
    # reduced halos: per rank, per domain the halo gids in halo order
    halos = []
    for r, ds in enumerate(ranks_domains):
        hs = []
        for i, d in enumerate(ds):
            g = d.outer_gids if ranks_halo_gids is None else ranks_halo_gids[r][i]
            lids = d.make_outer_lids(g)
            hs.append([d.gids[l] for l in lids])
        halos.append(hs)
    recv_data = [[] for _ in range(world)]  # per rank: records it created
    # distributed_for_each visits every rank's data (own included) in ring order; the resulting
    # maps are std::map keyed by (rank, tag) so the visit order does not change the result.
    for me in range(world):
        for other in range(world):
            for od_idx, od in enumerate(ranks_domains[other]):
                hgids = halos[other][od_idx]
                for i, d in enumerate(ranks_domains[me]):
                    tag = make_tag(i, od.id)
                    lids = [d.inner[g] for g in hgids if g in d.inner]
                    if not lids:
                        continue
                    recv_data[me].append((d.id, od.id, other, tag, [d.gids[l] for l in lids]))
                    pats[me][i]["send"][(other, tag)] = (od.id, lids)
    for me in range(world):
        for src in range(world):
            for (did, other_id, recv_rank, tag, gids) in recv_data[src]:
                if recv_rank != me:
                    continue
                for i, d in enumerate(ranks_domains[me]):
                    if d.id == other_id:
                        pats[me][i]["recv"][(src, tag)] = (did, d.make_outer_lids(gids))
                        break
    for r in range(world):
        for p in pats[r]:
            p["send"] = dict(sorted(p["send"].items()))
            p["recv"] = dict(sorted(p["recv"].items()))
    return pats


def unstructured_get(values: np.ndarray, buffer: np.ndarray, elem, lids, levels, levels_first,
                     index_stride, level_stride, byte_offset=0):
    lid_a, lid_p = _i64(lids)
    return lib().orc_unstructured_get(values.ctypes.data, buffer.ctypes.data + byte_offset, elem,
                                      lid_p, len(lid_a), levels, 1 if levels_first else 0,
                                      index_stride, level_stride)


def unstructured_set(values: np.ndarray, buffer: np.ndarray, elem, lids, levels, levels_first,
                     index_stride, level_stride, byte_offset=0):
    lid_a, lid_p = _i64(lids)
    return lib().orc_unstructured_set(values.ctypes.data, buffer.ctypes.data + byte_offset, elem,
                                      lid_p, len(lid_a), levels, 1 if levels_first else 0,
                                      index_stride, level_stride)
