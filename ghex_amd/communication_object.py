"""communication_object — the exchange of the halo path
(include/ghex/communication_object.hpp:271-285, 483-828) on MI355X.

exchange(buffer_infos):
  1. plan (cached per field set): buffers per domain pair, fields in argument order with
     alignof padding, tags = pattern tag + per-container offset (communication_object::allocate,
     :1003-1067) — done in libghx (ghx_exchange_create);
  2. ONE fused pack launch for all send buffers on the current stream;
  3. transport: self-messages are not sent — the unpack reads the send buffer directly
     (SURVEY §8(e)); peer messages go through torch.distributed point-to-point (backend
     "nccl" = RCCL over xGMI), posted as one group (batch_isend_irecv), stream-ordered like the
     reference's stream-aware branch (:703-714, 751-765);
  4. ONE fused unpack launch for all recv buffers.

staging="host" (the NIC-side path; arch_traits.hpp:51-75 keeps device buffers
through oomph): after the pack, each peer send buffer is copied to a pinned host buffer (D2H on
the exchange stream, one event per buffer so each host send starts as soon as its copy lands),
messages travel over a gloo group between host buffers, and each received buffer is copied back
(H2D) as soon as its message has arrived; the unpack launch is queued behind the copies.
Self messages stay on the device exactly as in the default mode.

pipelined=True (the reference's per-buffer streams + send-as-packed,
include/ghex/device/cuda/stream.hpp:25-73, communication_object.hpp:568-637, 703-767): each peer
rank rides one of `max_streams` greatest-priority streams (dealt in round order; the device has
few hardware queues) on which its send buffers are packed (one launch per buffer), its messages
exchanged and its recv buffers unpacked, so a message leaves as soon as its
own pack is done and is unpacked as soon as it lands. Device buffers: the native pipeline
(ghx_pipeline_*) with one 2-rank RCCL communicator per peer pair (one shared communicator would
serialise the per-peer groups); host staging: per-peer D2H after the pack, host sends as the
copies land, H2D + unpack per message as it arrives. Peers are issued in one global round-robin
order on every rank (round_of), which keeps streams that share a hardware queue deadlock-free.

direct=True (node-local peers, device buffers): no transport step at all. Every rank exports its
peer receive buffers (IPC) at the first exchange of a plan and imports the buffers its peers
receive into; the ONE pack launch then writes each peer message straight into the receiver's
buffer (lane-linear 16-B stores: dense writes over xGMI between GPUs, where the bulk object's
field-to-field puts scatter the x-normal faces' 16-B rows), and the receiver unpacks it locally.
Ordering is stream-ordered device epochs (libghx ghx_epochs_*; the reference's access guards,
include/ghex/rma/access_guard.hpp:35-140) in ONE launch per exchange: each peer receive buffer
exists twice and exchange e uses the copy of parity e&1 (chosen on the device from the epoch
counter, so graph replays alternate), so the copy a source writes at e+1 was last read by this
rank's unpack of e-1 — done before this rank's close of e, which says so to its sources. Per
exchange: pack (into copy e&1 of the receivers' buffers) — k_epoch_close1 (this rank's writes
visible on every XCD, peers signalled, every source's writes and every target's previous unpack
awaited) — unpack (copy e&1). No host synchronisation; graph-capturable; structured and
unstructured fields alike.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

from . import _ghx


class _ExchangePlan:
    def __init__(self, items: List[_ghx.ExchangeItem]):
        arr = (_ghx.ExchangeItem * len(items))(*items)
        h = ctypes.c_void_p()
        _ghx.call("ghx_exchange_create", arr, len(items), ctypes.byref(h))
        self.h = h
        self.send = self._buffers(0)
        self.recv = self._buffers(1)

    def _buffers(self, direction):
        n = ctypes.c_int32()
        _ghx.call("ghx_exchange_num_buffers", self.h, direction, ctypes.byref(n))
        out = []
        for i in range(n.value):
            a, b, r, t = (ctypes.c_int32() for _ in range(4))
            s = ctypes.c_uint64()
            _ghx.call("ghx_exchange_buffer", self.h, direction, i, ctypes.byref(a),
                      ctypes.byref(b), ctypes.byref(r), ctypes.byref(t), ctypes.byref(s))
            out.append(dict(pair=(a.value, b.value), rank=r.value, tag=t.value, size=s.value))
        return out

    def __del__(self):
        try:
            if self.h:
                _ghx.lib().ghx_exchange_destroy(self.h)
                self.h = None
        except Exception:
            pass


def as_stream(stream, device=None):
    """The stream argument of schedule_exchange / schedule_wait as a torch stream, accepted in
    the forms the reference binding accepts (bindings/python/src/_pyghex/unstructured/
    communication_object.cpp:39-85): None (the current stream), a torch stream, any object with
    the CUDA stream protocol (`__cuda_stream__()` -> (0, address)) or a `.ptr` (CuPy-style);
    anything else raises TypeError."""
    import torch
    if stream is None:
        return torch.cuda.current_stream(device)
    if isinstance(stream, torch.cuda.Stream):
        return stream
    if hasattr(stream, "__cuda_stream__"):
        proto = stream.__cuda_stream__()
        if not isinstance(proto, tuple) or len(proto) != 2:
            raise TypeError("Expected a tuple of length 2 from `__cuda_stream__`, got "
                            f"{proto!r}")
        if proto[0] != 0:
            raise TypeError(f"Expected `__cuda_stream__` protocol version 0, but got {proto[0]}")
        return torch.cuda.ExternalStream(int(proto[1]), device=device)
    if hasattr(stream, "ptr"):
        return torch.cuda.ExternalStream(int(stream.ptr), device=device)
    raise TypeError("Failed to convert the stream object into a CUDA stream.")


def _dbl(size):
    """Offset of the odd-parity copy of a double-buffered receive buffer (256-B aligned)."""
    return max(256, (int(size) + 255) // 256 * 256)


def route(context, sends, recvs, group=None):
    """Post one group of point-to-point messages. sends/recvs: [(peer_rank, tag, tensor)].

    Messages between one pair of ranks are matched in (tag) order on both sides (NCCL/RCCL
    matches by issue order; gloo by tag) — the tag of a send buffer equals the tag of the
    matching recv buffer by construction of the pattern. Returns the list of works: the recvs
    first, in (peer, tag) order, then the sends."""
    dist = context.distributed
    group = context.group if group is None else group
    ops = []
    for peer, tag, t in sorted(recvs, key=lambda x: (x[0], x[1])):
        ops.append(dist.P2POp(dist.irecv, t, context.global_rank(peer), group, tag))
    for peer, tag, t in sorted(sends, key=lambda x: (x[0], x[1])):
        ops.append(dist.P2POp(dist.isend, t, context.global_rank(peer), group, tag))
    if not ops:
        return []
    return dist.batch_isend_irecv(ops)


def direct_matches(me, send, recv_of):
    """The direct exchange's message matching: for each of this rank's peer send buffers
    (`send`: the plan's send dicts) the receiver's published entry (src, tag, size, ...) from
    `recv_of[peer]`. Messages of one rank pair match k-th to k-th in tag order on both sides, as
    route() matches them (stable sorts keep the plan order among equal tags); counts, tags and
    sizes must agree. Returns [(send index, entry)]."""
    by_peer = {}
    for i, x in enumerate(send):
        if x["rank"] != me:
            by_peer.setdefault(x["rank"], []).append(i)
    out = []
    for p, idx in sorted(by_peer.items()):
        theirs = sorted((e for e in recv_of[p] if e[0] == me), key=lambda e: e[1])
        ours = sorted(idx, key=lambda i: send[i]["tag"])
        if len(theirs) != len(ours):
            raise RuntimeError(f"direct exchange: rank {p} expects {len(theirs)} messages "
                               f"from rank {me}, which sends {len(ours)}")
        for i, e in zip(ours, theirs):
            if e[1] != send[i]["tag"] or e[2] != send[i]["size"]:
                raise RuntimeError(f"direct exchange: message mismatch with rank {p} (tag "
                                   f"{send[i]['tag']}/{e[1]}, {send[i]['size']}/{e[2]} B)")
            out.append((i, e))
    return out


def round_of(a: int, b: int, world: int) -> int:
    """Round of the pair (a, b) in a round-robin tournament over `world` ranks (circle method):
    every rank meets every other rank exactly once, each rank in at most one pair per round.
    With m = world rounded up to even and q = m - 1: pairs with b = m - 1 play in round a, the
    others in the round r with a + b = 2r (mod q)."""
    m = world + (world % 2)
    q = m - 1
    a, b = min(a, b), max(a, b)
    if q <= 0:
        return 0
    if b == q:
        return a
    return ((a + b) * (m // 2)) % q


def peer_order(me: int, peers, world: int):
    """Peers of `me` in global round order (the issue order every rank uses)."""
    return sorted(peers, key=lambda p: (round_of(me, p, world), p))


class _Pipeline:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            if self.h:
                _ghx.lib().ghx_pipeline_destroy(self.h)
                self.h = None
        except Exception:
            pass


class CommunicationHandle:
    """communication_handle (communication_object.hpp:78-130): wait / is_ready / progress /
    schedule_wait."""

    def __init__(self, co, stream, event):
        self._co = co
        self._stream = stream
        self._event = event

    def wait(self):
        co, self._co = self._co, None
        if co is not None and co.has_scheduled_exchange():
            co.complete_schedule_exchange()  # (:810-819) syncs the schedule_wait stream
        elif self._event is not None:
            self._event.synchronize()
        if co is not None:
            co._valid = False
            if co.direct:
                co.check_epochs()

    def is_ready(self) -> bool:
        if self._co is not None and self._co.has_scheduled_exchange():
            if not self._co._scheduled_event.query():
                return False
            self.wait()
            return True
        if self._event is None or self._event.query():
            co, self._co = self._co, None
            if co is not None:
                co._valid = False
                if co.direct:
                    co.check_epochs()  # a poller learns of an epoch failure as wait() would
            return True
        return False

    def progress(self):
        self.is_ready()

    def schedule_wait(self, stream=None):
        """Make `stream` (None = the current stream) wait for the exchange without blocking the
        host (communication_handle::schedule_wait, communication_object.hpp:832-856, 918-945).
        Afterwards co.has_scheduled_exchange() is True until wait() or the next exchange."""
        import torch
        if self._event is None or self._co is None:
            return
        stream = as_stream(stream, self._stream.device)
        stream.wait_event(self._event)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._co._scheduled_event = ev
        self._co._valid = False  # a new exchange may start; it completes this one first


class CommunicationObject:
    """communication_object<grid, domain_id> (make_communication_object, :1105-1112)."""

    def __init__(self, context, fuse_self: bool = True, staging=None, pipelined: bool = False,
                 rccl_self: bool = False, max_streams: int = 4, copy_engine: str = "probe",
                 direct: bool = False, epoch_timeout: float = 30.0):
        if staging not in (None, "host"):
            raise ValueError("staging must be None (device buffers) or 'host'")
        if direct and (staging is not None or pipelined or rccl_self):
            raise ValueError("direct packs into the peers' device buffers: no staging, no "
                             "pipeline, no rccl_self")
        # direct: pack straight into node-local peers' receive buffers (module docstring)
        self.direct = bool(direct)
        self.epoch_timeout = float(epoch_timeout)
        self._direct = {}
        if copy_engine not in ("probe", "runtime"):
            raise ValueError("copy_engine must be 'probe' (measured SDMA engines) or 'runtime'")
        # host staging: "probe" = D2H / H2D on the SDMA engines ghex_amd.staging measured,
        # "runtime" = hipMemcpyAsync (the HIP runtime picks the engines)
        self.copy_engine = copy_engine
        if rccl_self and staging == "host":
            # the host-staged pipeline keeps self messages on the device (recv aliases send);
            # routing them through RCCL is a device-buffer-only test mode
            raise ValueError("rccl_self applies to device buffers only (staging=None)")
        self.context = context
        self.fuse_self = fuse_self
        self.staging = staging
        self.pipelined = pipelined
        # tests: route the self messages through RCCL too (a 1-rank communicator), so the
        # pipeline's RCCL path runs on a one-GPU box
        self.rccl_self = rccl_self
        # pipelined: peers dealt over this many streams in round order (hardware queues are few)
        self.max_streams = max(1, int(max_streams))
        self._streams = {}
        self._plans = {}
        self._bufs = {}
        self._host = {}
        self._valid = False
        self._scheduled_event = None
        self._host_group = None
        if staging == "host" and context.distributed is not None and context.size() > 1:
            dist = context.distributed
            if dist.get_backend(context.group) == "gloo":
                self._host_group = context.group
            else:  # a host-transport group over the same ranks (collective: every rank builds it)
                ranks = None if context.group is None else dist.get_process_group_ranks(context.group)
                self._host_group = dist.new_group(ranks=ranks, backend="gloo")

    def all_self(self, plan) -> bool:
        """Every message is a self message and libghx can fuse pack+unpack (ghx_exchange_self)."""
        if getattr(plan, "_all_self", None) is None:
            me = self.context.rank()
            f = ctypes.c_int32()
            _ghx.call("ghx_exchange_self_fusable", plan.h, ctypes.byref(f))
            plan._all_self = bool(f.value) and all(b["rank"] == me for b in plan.send + plan.recv)
        return plan._all_self

    def mixed(self, plan) -> bool:
        """Self AND peer messages: the pack launch also completes the self messages
        (ghx_exchange_pack_self) and the unpack launch covers the peers only."""
        if getattr(plan, "_mixed", None) is None:
            f = ctypes.c_int32()
            _ghx.call("ghx_exchange_mixed", plan.h, ctypes.byref(f))
            plan._mixed = bool(f.value)
        return plan._mixed

    # -- planning -----------------------------------------------------------------------------
    def _key(self, bis):
        k = []
        for bi in bis:
            f = bi.field
            k.append((id(bi.pattern_container), bi.local_index, f.kind, bytes(f.desc), f.align))
        return tuple(k)

    def plan(self, bis):
        key = self._key(bis)
        p = self._plans.get(key)
        if p is None:
            # tag offsets per distinct pattern container (prepare_exchange_buffers :540-549)
            offsets, acc = {}, 0
            for bi in bis:
                pc = bi.pattern_container
                if id(pc) not in offsets:
                    offsets[id(pc)] = acc
                    acc += pc.max_tag() + 1
            items = []
            for bi in bis:
                it = _ghx.ExchangeItem()
                it.pattern = bi.pattern_container.handle
                it.local_index = bi.local_index
                it.kind = bi.field.kind
                if bi.field.kind == 0:
                    it.field = bi.field.desc
                else:
                    it.udata = bi.field.desc
                it.align = bi.field.align
                it.tag_offset = offsets[id(bi.pattern_container)]
                items.append(it)
            p = _ExchangePlan(items)
            self._plans[key] = (p, [bi.pattern_container for bi in bis])
        else:
            p = p[0]
        return p

    def buffers(self, plan, device):
        """Device buffers, reused across exchanges while sizes are unchanged (:581-589)."""
        import torch
        key = (id(plan), str(device))
        b = self._bufs.get(key)
        if b is None:
            send = [torch.empty(max(1, x["size"]), dtype=torch.uint8, device=device)
                    for x in plan.send]
            recv = []
            me = self.context.rank()
            # (rccl_self routes self messages through RCCL: distinct recv buffers then)
            alias = not (self.pipelined and self.rccl_self)
            for x in plan.recv:
                # self-message: unpack straight from the matching send buffer
                j = next((i for i, s in enumerate(plan.send)
                          if s["pair"] == x["pair"] and x["rank"] == me and alias), None)
                if j is not None:
                    recv.append(send[j])
                elif self.direct and x["rank"] != me:
                    # direct: a peer's receive buffer exists twice, the copy of each exchange's
                    # epoch parity (one-launch epochs, _direct_of); the odd copy _dbl bytes on
                    recv.append(torch.empty(2 * _dbl(x["size"]), dtype=torch.uint8, device=device))
                else:
                    recv.append(torch.empty(max(1, x["size"]), dtype=torch.uint8, device=device))
            b = (send, recv)
            self._bufs[key] = b
        return b

    # -- exchange ------------------------------------------------------------------------------
    def has_scheduled_exchange(self) -> bool:
        """A schedule_wait()-ed exchange whose completion has not been awaited on the host."""
        return self._scheduled_event is not None

    def complete_schedule_exchange(self):
        """communication_object::complete_schedule_exchange (:950-968)."""
        ev, self._scheduled_event = self._scheduled_event, None
        if ev is not None:
            ev.synchronize()
            self._valid = False

    @staticmethod
    def _as_list(buffer_infos):
        if len(buffer_infos) == 1 and isinstance(buffer_infos[0], (list, tuple)):
            return list(buffer_infos[0])
        return list(buffer_infos)

    def exchange(self, *buffer_infos) -> CommunicationHandle:
        """Non-blocking exchange on the current stream (communication_object::exchange,
        :271-285): pack, transport, unpack are stream-ordered; wait() blocks the host."""
        import torch
        bis = self._as_list(buffer_infos)
        stream = torch.cuda.current_stream(bis[0].field.device.index) if bis else None
        return self._start(bis, stream)

    def schedule_exchange(self, stream, *buffer_infos) -> CommunicationHandle:
        """communication_object::schedule_exchange (:287-330): the exchange starts after all
        work submitted to `stream` (None = the current stream) so far, without blocking the
        host; call schedule_wait(stream) on the handle to order later work after the unpack."""
        bis = self._as_list(buffer_infos)
        if bis:
            stream = as_stream(stream, bis[0].field.device)
        return self._start(bis, stream)

    def _done_event(self, stream):
        """The completion event of the exchange being started, recorded on `stream`. One event per
        object suffices: an exchange cannot start before the previous one completed."""
        import torch
        ev = self.__dict__.get("_ev")
        if ev is None:
            ev = self._ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def _start(self, bis, stream) -> CommunicationHandle:
        import torch
        self.complete_schedule_exchange()
        if self._valid:
            raise RuntimeError("earlier exchange operation was not finished")
        if not bis:
            return CommunicationHandle(None, None, None)
        device = bis[0].field.device
        plan = self.plan(bis)
        send, recv = self.buffers(plan, device)
        # pointer arrays cached per (plan, field pointers): repeated exchanges of the same fields
        # (the common case) rebuild nothing on the host
        fkey = tuple(bi.field.data_ptr() for bi in bis)
        cache = plan.__dict__.setdefault("_ptr_cache", {})
        arrs = cache.get(fkey)
        if arrs is None:
            if len(cache) > 64:
                cache.clear()
            arrs = cache[fkey] = (_ghx.ptr_array(list(fkey)),
                                  _ghx.ptr_array([t.data_ptr() for t in send]),
                                  _ghx.ptr_array([t.data_ptr() for t in recv]))
        fptrs, sptrs, rptrs = arrs
        # an exchange is "in flight" (exchange() again before wait() raises) only once it has
        # been enqueued: a failure while posting it leaves the object usable
        h = self._enqueue(bis, plan, send, recv, fptrs, sptrs, rptrs, stream)
        self._valid = True
        return h

    def _enqueue(self, bis, plan, send, recv, fptrs, sptrs, rptrs, stream):
        import torch
        device = bis[0].field.device
        if self.direct:
            d = self._direct_of(plan, send, recv)  # collective at a plan's first exchange
            if not (self.fuse_self and self.all_self(plan)):
                return self._exchange_direct(plan, d, fptrs, len(bis), rptrs, len(recv), stream)
        if self.pipelined:
            if self.staging == "host":
                self._exchange_host_pipelined(plan, send, recv, fptrs, sptrs, rptrs, len(bis),
                                              stream)
            else:
                pl = self._pipeline_of(plan, device)
                _ghx.call("ghx_pipeline_run", pl.h, fptrs, len(bis), sptrs, len(send), rptrs,
                          len(recv), stream.cuda_stream)
            return CommunicationHandle(self, stream, self._done_event(stream))
        if self.fuse_self and self.all_self(plan):
            # every message stays on this device: pack + unpack in one launch (the launch and
            # the event go to `stream` explicitly: no current-stream switch needed)
            rc = _ghx.lib().ghx_exchange_self(plan.h, fptrs, len(bis), sptrs, len(send),
                                              stream.cuda_stream)
            if rc:
                _ghx.check(rc, "ghx_exchange_self")
            return CommunicationHandle(self, stream, self._done_event(stream))
        with torch.cuda.stream(stream):
            mixed = self.fuse_self and self.mixed(plan)
            _ghx.call("ghx_exchange_pack_self" if mixed else "ghx_exchange_pack", plan.h,
                      fptrs, len(bis), sptrs, len(send), stream.cuda_stream)
            me = self.context.rank()
            sends = [(x["rank"], x["tag"], send[i][:x["size"]])
                     for i, x in enumerate(plan.send) if x["rank"] != me]
            recvs = [(x["rank"], x["tag"], recv[i][:x["size"]])
                     for i, x in enumerate(plan.recv) if x["rank"] != me]
            if self.staging == "host":
                self._exchange_host_staged(plan, sends, recvs, stream)
            else:
                for w in route(self.context, sends, recvs):
                    w.wait()  # NCCL: the stream waits for the recvs, the host does not
            _ghx.call("ghx_exchange_unpack_peers" if mixed else "ghx_exchange_unpack",
                      plan.h, fptrs, len(bis), rptrs, len(recv), stream.cuda_stream)
            ev = self._done_event(stream)
        return CommunicationHandle(self, stream, ev)

    def _host_buffers(self, plan, sends, recvs):
        import torch
        key = id(plan)
        h = self._host.get(key)
        if h is None:
            h = ([torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True) for _, _, t in sends],
                 [torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True) for _, _, t in recvs])
            self._host[key] = h
        return h

    def _exchange_host_staged(self, plan, sends, recvs, stream):
        """pack (queued) -> D2H per buffer -> host sends as copies land; host recvs -> H2D per
        buffer as messages land; the caller queues the unpack afterwards. copy_engine="probe":
        copies on the measured SDMA engines (the host waits for the pack, the copy engines run
        D2H and H2D concurrently; the unpack is queued behind an L2 acquire); "runtime": the
        copies are hipMemcpyAsync on the exchange stream."""
        import torch
        hs, hr = self._host_buffers(plan, sends, recvs)
        dist = self.context.distributed
        group = self._host_group
        gr = self.context.global_rank
        if self.copy_engine == "probe":
            from .staging import Copier
            cp = Copier.for_device(stream.device)
            packed = torch.cuda.Event()
            packed.record(stream)
            rops = [(dist.irecv(h, gr(peer), group, tag), h, peer, tag)
                    for (peer, tag, _), h in sorted(zip(recvs, hr), key=lambda x: (x[0][0], x[0][1]))]
            packed.synchronize()  # the send buffers are complete
            tks = [cp.d2h(h.data_ptr(), t.data_ptr(), t.numel()) for (_, _, t), h in zip(sends, hs)]
            sops = []
            for ((peer, tag, _), h), tk in sorted(zip(zip(sends, hs), tks),
                                                  key=lambda x: (x[0][0][0], x[0][0][1])):
                cp.wait(tk)
                sops.append(dist.isend(h, gr(peer), group, tag))
            dev_of = {(p, g): t for p, g, t in recvs}
            h2d = []
            for w, h, peer, tag in rops:
                w.wait()
                t = dev_of[(peer, tag)]
                h2d.append(cp.h2d(t.data_ptr(), h.data_ptr(), t.numel()))
            for tk in h2d:
                cp.wait(tk)
            if h2d:
                cp.acquire(stream)
            for w in sops:
                w.wait()
            return
        evs = []
        with torch.cuda.stream(stream):
            for (_, _, t), h in zip(sends, hs):
                h.copy_(t, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                evs.append(ev)
        rops = []
        for (peer, tag, _), h in sorted(zip(recvs, hr), key=lambda x: (x[0][0], x[0][1])):
            rops.append((dist.irecv(h, gr(peer), group, tag), h, peer, tag))
        sops = []
        for ((peer, tag, _), h), ev in sorted(zip(zip(sends, hs), evs),
                                              key=lambda x: (x[0][0][0], x[0][0][1])):
            ev.synchronize()
            sops.append(dist.isend(h, gr(peer), group, tag))
        dev_of = {(p, g): t for p, g, t in recvs}
        with torch.cuda.stream(stream):
            for w, h, peer, tag in rops:
                w.wait()
                dev_of[(peer, tag)].copy_(h, non_blocking=True)
        for w in sops:
            w.wait()

    # -- pipelined exchange ---------------------------------------------------------------------
    def _peer_stream(self, lane, device):
        import torch
        key = (lane, str(device))
        s = self._streams.get(key)
        if s is None:
            s = self._streams[key] = torch.cuda.Stream(device, priority=-1)
        return s

    def _split(self, plan):
        if not getattr(plan, "_split", False):
            _ghx.call("ghx_exchange_split", plan.h)
            plan._split = True

    def _rccl_comms(self, peers):
        """The context's pair communicators (Context.pair_communicators), created in round
        order at the first pipelined exchange that needs them, reused afterwards."""
        me, world = self.context.rank(), self.context.size()
        return self.context.pair_communicators(peers, lambda ps: peer_order(me, ps, world))

    def _pipeline_of(self, plan, device):
        pl = getattr(plan, "_pipeline", None)
        if pl is None:
            self._split(plan)
            me, world = self.context.rank(), self.context.size()
            ranks = {x["rank"] for x in plan.send + plan.recv}
            peers = peer_order(me, [r for r in ranks if r != me or self.rccl_self], world)
            comms = self._rccl_comms(peers)
            h = ctypes.c_void_p()
            _ghx.call("ghx_pipeline_create", plan.h, me, len(peers), _ghx.i32_array(peers),
                      _ghx.ptr_array([c.value for c, _ in comms]),
                      _ghx.i32_array([r for _, r in comms]), self.max_streams, ctypes.byref(h))
            pl = plan._pipeline = _Pipeline(h)
        return pl

    def _exchange_host_pipelined(self, plan, send, recv, fptrs, sptrs, rptrs, nf, stream):
        """Host staging with per-peer overlap (reference non-stream-aware branch,
        communication_object.hpp:611-637, 715-729): per peer stream pack -> D2H; each host send
        is posted when its own copy has landed; each arrived message is copied back (H2D) and
        unpacked on its peer's stream while the others are still in flight."""
        import torch
        self._split(plan)
        me, world = self.context.rank(), self.context.size()
        L = _ghx.lib()
        device = stream.device
        sends_of, recvs_of = {}, {}
        for i, x in enumerate(plan.send):
            sends_of.setdefault(x["rank"], []).append(i)
        for j, x in enumerate(plan.recv):
            recvs_of.setdefault(x["rank"], []).append(j)
        peers = peer_order(me, [r for r in set(sends_of) | set(recvs_of) if r != me], world)
        key = ("hostpipe", id(plan))
        h = self._host.get(key)
        if h is None:
            h = self._host[key] = (
                [torch.empty(max(1, x["size"]), dtype=torch.uint8, pin_memory=True) for x in plan.send],
                [torch.empty(max(1, x["size"]), dtype=torch.uint8, pin_memory=True) for x in plan.recv])
        hs, hr = h
        start = torch.cuda.Event()
        start.record(stream)
        landed = {}
        probe = self.copy_engine == "probe"
        if probe:
            from .staging import Copier
            cp = Copier.for_device(device)
        lane_of = {p: k % self.max_streams for k, p in enumerate(peers)}
        for p in peers:
            sp = self._peer_stream(lane_of[p], device)
            sp.wait_event(start)
            for i in sends_of.get(p, []):
                _ghx.check(L.ghx_exchange_pack_buffer(plan.h, i, fptrs, nf, sptrs, len(send),
                                                      sp.cuda_stream), "pack_buffer")
                if not probe:
                    with torch.cuda.stream(sp):
                        hs[i][:plan.send[i]["size"]].copy_(send[i][:plan.send[i]["size"]],
                                                           non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(sp)
            landed[p] = ev
        # self messages: packed and unpacked on the caller's stream (recv aliases send)
        for i, x in enumerate(plan.send):
            if x["rank"] == me:
                _ghx.check(L.ghx_exchange_pack_buffer(plan.h, i, fptrs, nf, sptrs, len(send),
                                                      stream.cuda_stream), "pack_buffer")
        for j, x in enumerate(plan.recv):
            if x["rank"] == me:
                _ghx.check(L.ghx_exchange_unpack_buffer(plan.h, j, fptrs, nf, rptrs, len(recv),
                                                        stream.cuda_stream), "unpack_buffer")
        dist = self.context.distributed
        group = self._host_group
        rops = []
        for p in peers:
            for j in sorted(recvs_of.get(p, []), key=lambda j: (plan.recv[j]["tag"], plan.recv[j]["pair"])):
                x = plan.recv[j]
                rops.append([dist.irecv(hr[j][:x["size"]], self.context.global_rank(p), group,
                                        x["tag"]), j, p])
        sops = []
        for p in peers:
            landed[p].synchronize()  # this peer's packs (and, with "runtime" copies, its D2H)
            order = sorted(sends_of.get(p, []), key=lambda i: (plan.send[i]["tag"], plan.send[i]["pair"]))
            if probe:
                tks = {i: cp.d2h(hs[i].data_ptr(), send[i].data_ptr(), plan.send[i]["size"])
                       for i in order if plan.send[i]["size"]}
            for i in order:
                x = plan.send[i]
                if probe and i in tks:
                    cp.wait(tks[i])
                sops.append(dist.isend(hs[i][:x["size"]], self.context.global_rank(p), group,
                                       x["tag"]))
        # every send is posted before the first blocking receive wait, so the in-order waits
        # below cannot deadlock; each message's H2D + unpack is queued as soon as it is in (gloo
        # receive works complete only inside wait(): no polling)
        for w, j, p in rops:
            w.wait()
            sp = self._peer_stream(lane_of[p], device)
            n = plan.recv[j]["size"]
            if probe:
                if n:
                    cp.wait(cp.h2d(recv[j].data_ptr(), hr[j].data_ptr(), n))
                    cp.acquire(sp)
            else:
                with torch.cuda.stream(sp):
                    recv[j][:n].copy_(hr[j][:n], non_blocking=True)
            _ghx.check(L.ghx_exchange_unpack_buffer(plan.h, j, fptrs, nf, rptrs, len(recv),
                                                    sp.cuda_stream), "unpack_buffer")
        for w in sops:
            w.wait()
        for lane in set(lane_of.values()):
            stream.wait_stream(self._peer_stream(lane, device))

    # -- direct: pack into the peers' receive buffers ----------------------------------------
    def _direct_of(self, plan, send, recv):
        """Set up a plan's direct exchange (collective: every rank, at the plan's first exchange).
        Returns {"sptrs": send pointer array with every peer message's entry replaced by the
        receiver's buffer, "ep": epochs handle or None, "imports": IPC bases}."""
        d = self._direct.get(id(plan))
        if d is not None:
            return d
        import torch
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("direct exchange: a plan's first exchange sets up IPC handles and "
                               "flag blocks collectively and cannot run inside a stream capture; "
                               "run one exchange of these fields before capturing")
        from .bulk_communication_object import hostname
        me, world = self.context.rank(), self.context.size()
        host = hostname()
        by_peer = {}
        for i, x in enumerate(plan.send):
            if x["rank"] != me:
                by_peer.setdefault(x["rank"], []).append(i)
        mine = []
        for j, x in enumerate(plan.recv):
            if x["rank"] == me:
                continue
            h = (ctypes.c_ubyte * 64)()
            off = ctypes.c_uint64()
            _ghx.call("ghx_ipc_export", ctypes.c_void_p(recv[j].data_ptr()), h, ctypes.byref(off))
            mine.append((x["rank"], x["tag"], x["size"], bytes(h), off.value, _dbl(x["size"])))
        allr = self.context.all_gather_object({"host": host, "recv": mine,
                                               "targets": sorted(by_peer)})
        # every rank checks every pair, so all raise together (none is left in a collective)
        far = [(r, p) for r, a in enumerate(allr) for p in a["targets"]
               if allr[p]["host"] != a["host"]]
        if far:
            r, p = far[0]
            raise RuntimeError(f"direct exchange needs node-local peers: rank {r} (host "
                               f"{allr[r]['host']!r}) sends to rank {p} (host "
                               f"{allr[p]['host']!r}); use the buffered exchange across hosts")
        ptrs = [t.data_ptr() for t in send]
        imports = []
        d = {"sptrs": None, "ep": None, "imports": imports}
        self._direct[id(plan)] = d  # before anything can raise: __del__ closes what was opened
        send_dbl = [0] * len(plan.send)
        for i, (_, tag, size, hb, off, dbl) in direct_matches(
                me, plan.send, {r: a["recv"] for r, a in enumerate(allr)}):
            base, ptr = ctypes.c_void_p(), ctypes.c_void_p()
            _ghx.call("ghx_ipc_import", (ctypes.c_ubyte * 64).from_buffer_copy(hb), off,
                      ctypes.byref(base), ctypes.byref(ptr))
            imports.append(base.value)
            ptrs[i] = ptr.value
            send_dbl[i] = dbl
        if world > 1:
            # one node-shared flag block per plan and host: the host's lowest rank creates it,
            # the host's other ranks attach (node-local indices); ranks of other hosts take part
            # in the collective setup only
            from .bulk_communication_object import attach_epochs
            d["hosts"] = [a["host"] for a in allr]
            srcs = sorted({x["rank"] for x in plan.recv if x["rank"] != me})
            d["ep"] = attach_epochs(self.context, d["hosts"], self.epoch_timeout, srcs,
                                    sorted(by_peer), prefix="dx")
        if d["ep"] is not None:
            # one launch of epochs per exchange (ghx_epochs phase 2): the peers' receive buffers
            # are double-buffered by epoch parity, read on the device from the epoch counter
            word = ctypes.c_void_p()
            _ghx.call("ghx_epochs_counter", d["ep"], ctypes.byref(word))
            recv_dbl = [_dbl(x["size"]) if x["rank"] != me else 0 for x in plan.recv]
            for direction, add, offs in ((0, 1, send_dbl), (1, 0, recv_dbl)):
                _ghx.call("ghx_exchange_set_parity", plan.h, direction, word, add,
                          (ctypes.c_int64 * max(1, len(offs)))(*offs), len(offs))
        d["sptrs"] = _ghx.ptr_array(ptrs)
        return d

    def _exchange_direct(self, plan, d, fptrs, nf, rptrs, nr, stream):
        s = stream.cuda_stream
        mixed = self.fuse_self and self.mixed(plan)
        # pack into copy e&1 of the receivers' buffers -> one-launch close (release, signal,
        # wait, acquire) -> unpack copy e&1 of this rank's
        _ghx.call("ghx_exchange_pack_self" if mixed else "ghx_exchange_pack", plan.h, fptrs, nf,
                  d["sptrs"], len(plan.send), s)
        if d["ep"] is not None:
            _ghx.call("ghx_epochs_enqueue", d["ep"], 2, s)
        _ghx.call("ghx_exchange_unpack_peers" if mixed else "ghx_exchange_unpack", plan.h, fptrs,
                  nf, rptrs, nr, s)
        import torch
        if torch.cuda.is_current_stream_capturing():
            return CommunicationHandle(self, stream, None)  # completion is the graph replay's
        return CommunicationHandle(self, stream, self._done_event(stream))

    def check_epochs(self):
        """Raise if a direct exchange's epochs recorded a failure (a wait timed out: a peer
        never reached it; or a source failed an epoch wait)."""
        from .bulk_communication_object import epochs_error
        for d in self._direct.values():
            if d["ep"] is None:
                continue
            why = epochs_error(d["ep"], d.get("hosts"), self.context.rank())
            if why:
                raise RuntimeError(f"direct exchange failed (epoch timeout "
                                   f"{self.epoch_timeout:.0f} s): {why}")

    def __del__(self):
        try:
            for d in self.__dict__.get("_direct", {}).values():
                for b in d["imports"]:
                    _ghx.lib().ghx_ipc_close(ctypes.c_void_p(b))
                if d["ep"] is not None:
                    _ghx.lib().ghx_epochs_destroy(d["ep"])
        except Exception:
            pass
        self._direct = {}

    # low-level access for benchmarks / tests (no transport)
    def _plain_plan(self, bis):
        """The plan of `bis` for the single-buffered low-level helpers below. A direct object's
        plan, once its first exchange has set the epoch parity (ghx_exchange_set_parity), packs
        into and unpacks from the copy of the exchange's parity: with this object's single-size
        local send buffers that would write past their end, so it is refused."""
        plan = self.plan(bis)
        d = self.__dict__.get("_direct", {}).get(id(plan))
        if d is not None and d.get("ep") is not None:
            raise RuntimeError("pack_only / unpack_only and their mixed forms are not available "
                               "on a direct exchange's plan (its launches are double-buffered "
                               "by epoch parity); use exchange()")
        return plan

    def pack_only(self, bis, stream=None):
        import torch
        plan = self._plain_plan(bis)
        send, recv = self.buffers(plan, bis[0].field.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _ghx.call("ghx_exchange_pack", plan.h, _ghx.ptr_array([b.field.data_ptr() for b in bis]),
                  len(bis), _ghx.ptr_array([t.data_ptr() for t in send]), len(send), s)
        return plan, send, recv

    def pack_self_only(self, bis, stream=None):
        """Mixed exchanges: pack every send buffer and complete the self messages."""
        import torch
        plan = self._plain_plan(bis)
        send, recv = self.buffers(plan, bis[0].field.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _ghx.call("ghx_exchange_pack_self", plan.h,
                  _ghx.ptr_array([b.field.data_ptr() for b in bis]), len(bis),
                  _ghx.ptr_array([t.data_ptr() for t in send]), len(send), s)
        return plan, send, recv

    def unpack_peers_only(self, bis, stream=None):
        """Mixed exchanges: unpack the peer messages only."""
        import torch
        plan = self._plain_plan(bis)
        send, recv = self.buffers(plan, bis[0].field.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _ghx.call("ghx_exchange_unpack_peers", plan.h,
                  _ghx.ptr_array([b.field.data_ptr() for b in bis]), len(bis),
                  _ghx.ptr_array([t.data_ptr() for t in recv]), len(recv), s)
        return plan, send, recv

    def unpack_only(self, bis, stream=None):
        import torch
        plan = self._plain_plan(bis)
        send, recv = self.buffers(plan, bis[0].field.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _ghx.call("ghx_exchange_unpack", plan.h,
                  _ghx.ptr_array([b.field.data_ptr() for b in bis]), len(bis),
                  _ghx.ptr_array([t.data_ptr() for t in recv]), len(recv), s)
        return plan, send, recv
