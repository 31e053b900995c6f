"""bulk_communication_object — zero-copy halo exchange between node-local GPUs
(include/ghex/bulk_communication_object.hpp:206-704; RMA put include/ghex/structured/rma_put.hpp;
CUDA IPC handles include/ghex/rma/cuda/handle.hpp). SURVEY §8(f) #2.

Instead of pack -> send -> recv -> unpack, every rank copies its send regions straight into the
receiving rank's halo cells in peer memory (xGMI on a multi-GPU node), one launch per group of
up to 64 messages (libghx ghx_put_*: the pack plan of the source side and the unpack plan of the
target side address the same message positions, so a lane moves element p register-to-register). Self messages are
the same copy inside one field.

Usage mirrors the reference:
    bco = make_bulk_communication_object(ctx)
    bco.add_field(pattern(field)); ...            # same order on every rank
    bco.init()                                    # exchanges IPC handles (collective)
    bco.exchange().wait()                         # collective

Epochs (the reference's access guards, rma/access_guard.hpp:35-140, and the bulk object's
open / put-when-writable / wait sequence, bulk_communication_object.hpp:621-694), stream-ordered
(epochs="device", the default): exchange() enqueues on the caller's stream
  k_epoch(open)  -> this rank's halos are open to its sources (its earlier kernels are done with
                    them); wait until each of its targets has opened its halos
  puts           -> one k_put launch per group of <= 64 messages
  k_epoch(close) -> signal each target that this epoch's puts are in; wait until each source's are
with flags in each receiver's fine-grained device memory (its "inbox", IPC-mapped into its
node-local peers and polled locally; a node-shared host block carries the inbox handles and each
rank's epoch and error for the host: libghx ghx_epochs_*). Nothing blocks the host;
only the ranks a rank exchanges with synchronise with it; wait() reports a peer that never
arrived (bounded waits, `timeout` seconds). epochs="host" keeps the round-2 form: drain the
stream, barrier, puts, drain, barrier. Puts go to node-local peers (ranks whose hostnames
match); the halos of ranks on other hosts travel through a CommunicationObject over the
pattern's remote part (`remote_options`), started in the same exchange() and awaited by the same
wait() — the reference's local / remote pattern maps and its m_co
(bulk_communication_object.hpp:330-383, 674-694).
"""
from __future__ import annotations

import ctypes
import os
import secrets
import socket

from . import _ghx

MAX_SLOTS = 64


def hostname() -> str:
    """This rank's host as the bulk exchange groups ranks (GHX_HOSTNAME overrides it: tests emulate
    several hosts on one machine)."""
    return os.environ.get("GHX_HOSTNAME") or socket.gethostname()


def node_local_group(hosts, me):
    """The epochs' node-local group of rank `me`: (ranks on its host in ascending order, its
    index among them). hosts: every rank's host name, by global rank. Flag blocks are per host
    and indexed by this position, so their size follows the ranks per host, not the world size
    (ghx_epochs_create takes at most 64 ranks per host, any number of hosts)."""
    local = [r for r, h in enumerate(hosts) if h == hosts[me]]
    return local, local.index(me)


def attach_epochs(context, hosts, timeout, sources, targets, prefix="ep"):
    """Create (the host's lowest rank) or attach (the others) this host's flag block and set the
    peers. Collective over the context: every rank calls it, including ranks that end up with
    no block. sources / targets: global ranks, all on this host. Returns the ghx_epochs handle,
    or None when this host holds only this rank."""
    me = context.rank()
    local, idx = node_local_group(hosts, me)
    lead = local[0] == me
    name = f"/ghx_{prefix}_{os.getpid()}_{secrets.token_hex(6)}" if lead and len(local) > 1 else None
    h = None
    if name is not None:  # created (and sized) before anyone learns its name
        h = ctypes.c_void_p()
        _ghx.call("ghx_epochs_create", name.encode(), 1, len(local), idx, float(timeout),
                  ctypes.byref(h))
    names = context.all_gather_object(name)
    try:
        if len(local) > 1 and not lead:
            h = ctypes.c_void_p()
            _ghx.call("ghx_epochs_create", names[local[0]].encode(), 0, len(local), idx,
                      float(timeout), ctypes.byref(h))
    finally:
        context.all_gather_object(None)  # every rank of every host has attached (or failed)
        if name is not None:
            _ghx.call("ghx_epochs_unlink", name.encode())
    if h is None:
        return None
    pos = {r: i for i, r in enumerate(local)}
    for r in list(sources) + list(targets):
        if r not in pos:
            raise RuntimeError(f"epochs: rank {r} is not on this host ({hosts[me]!r})")
    srcs = [pos[r] for r in sorted(set(sources))]
    tgts = [pos[r] for r in sorted(set(targets))]
    _ghx.call("ghx_epochs_peers", h, _ghx.i32_array(srcs), len(srcs), _ghx.i32_array(tgts),
              len(tgts))
    return h


def epochs_error(ep, hosts=None, me=None):
    """None, or a description of the epochs' recorded failure (ghx_epochs_status codes)."""
    err = ctypes.c_int32()
    _ghx.call("ghx_epochs_status", ep, ctypes.byref(err), None)
    v = err.value
    if not v:
        return None
    if v == 1:
        return "a wait of the open phase timed out (a target never opened its memory)"
    if v == 2:
        return "a wait of the close phase timed out (a source never completed its writes)"
    if v == 3:
        return "the close kernel did not reach every XCD in time (fence placement)"
    if v & 0xff == 4:
        s = v >> 8
        who = f"node-local rank {s}"
        if hosts is not None and me is not None:
            who = f"rank {node_local_group(hosts, me)[0][s]}"
        return (f"{who} failed an epoch wait: its later writes may have overlapped this rank's "
                f"reads")
    return f"epoch error code {v}"


def put_messages(bis, groups, allr, local):
    """The node-local messages of this rank's fields, as (source field index k, send spaces,
    target (rank, field index), target spaces): each send halo of field k (domain d, its j-th
    field) paired with the receive halo of (my domain d, tag) on the target rank's j-th field of
    the receiving domain (the reference's put ranges, bulk_communication_object.hpp:384-455).
    bis[k] needs .pattern_container / .local_index; allr[r] = rank r's gathered setup record;
    groups = _field_groups(); local = the ranks on this host."""
    target = {}
    for r, info in enumerate(allr):
        for i, f in enumerate(info["fields"]):
            target[(r, f["domain"], f["j"])] = (r, i)
    msgs = []
    for k, (bi, (d, j)) in enumerate(zip(bis, groups)):
        for rid, rr, tag, spaces in bi.pattern_container.send_halos(bi.local_index):
            if rr not in local:
                continue  # a remote rank: the buffered exchange carries it
            key = (rr, rid, j)
            if key not in target:
                raise RuntimeError(f"rank {rr} registered no field #{j} for domain {rid}")
            tr, ti = target[key]
            tf = allr[tr]["fields"][ti]
            tsp = next((sp for (sid, stag, sp) in tf["recv"] if sid == d and stag == tag), None)
            if tsp is None:
                raise RuntimeError(f"no receive halo on rank {tr} for domain {d}, tag {tag}")
            msgs.append((k, [(sp[0], sp[1]) for sp in spaces], (tr, ti), tsp))
    return msgs


def put_chunks(msgs):
    """Messages grouped into put plans (one launch each) of <= 64 messages, <= 64 source and
    <= 64 target fields: [(chunk, source field indices, target (rank, index) list)]."""
    out, chunk, srcs, dsts = [], [], [], []
    for m in msgs + [None]:
        if (m is None or len(chunk) == MAX_SLOTS or
                (m[0] not in srcs and len(srcs) == MAX_SLOTS) or
                (m[2] not in dsts and len(dsts) == MAX_SLOTS)):
            if chunk:
                out.append((chunk, srcs, dsts))
            chunk, srcs, dsts = [], [], []
            if m is None:
                break
        if m[0] not in srcs:
            srcs.append(m[0])
        if m[2] not in dsts:
            dsts.append(m[2])
        chunk.append(m)
    return out


def put_entries(chunk, srcs, dsts, src_descs, allr):
    """ghx_put_create's two entry arrays for one chunk: message b is virtual buffer b on both
    sides; the source side names this rank's fields (src_descs[k]), the target side the
    target ranks' field descriptors as gathered. Returns (src, dst, keep-alive list)."""
    n = len(chunk)
    src = (_ghx.PackEntry * n)()
    dst = (_ghx.PackEntry * n)()
    keep = [src, dst]
    for b, (k, sps, tgt, tsps) in enumerate(chunk):
        tdesc = _ghx.FieldDesc.from_buffer_copy(allr[tgt[0]]["fields"][tgt[1]]["desc"])
        for e, desc, slot, spaces in ((src[b], src_descs[k], srcs.index(k), sps),
                                      (dst[b], tdesc, dsts.index(tgt), tsps)):
            arr = (_ghx.Box * max(1, len(spaces)))()
            for i, (lf, ll) in enumerate(spaces):
                for d in range(len(lf)):
                    arr[i].first[d], arr[i].last[d] = lf[d], ll[d]
            keep.append(arr)
            e.field = desc
            e.field_slot = slot
            e.buffer_slot = b
            e.buffer_offset = 0
            e.boxes = ctypes.cast(arr, ctypes.POINTER(_ghx.Box))
            e.n_boxes = len(spaces)
    return src, dst, keep


class BulkHandle:
    """Handle of a bulk exchange: wait() blocks until this rank's halos are written (and raises
    if a peer never reached the exchange); is_ready() polls."""

    def __init__(self, bco=None, event=None, remote=None):
        self._bco, self._event, self._remote = bco, event, remote

    def wait(self):
        if self._remote is not None:
            self._remote.wait()
            self._remote = None
        if self._event is not None:
            self._event.synchronize()
            self._check()

    def is_ready(self) -> bool:
        if self._remote is not None:
            if not self._remote.is_ready():
                return False
            self._remote = None
        if self._event is None:
            return True
        if not self._event.query():
            return False
        self._check()
        return True

    def progress(self):
        self.is_ready()

    def _check(self):
        bco, self._bco = self._bco, None
        if bco is not None:
            bco.check_epochs()


class BulkCommunicationObject:
    def __init__(self, context, epochs: str = "device", timeout: float = 30.0,
                 remote_options=None):
        if epochs not in ("device", "host"):
            raise ValueError("epochs must be 'device' (stream-ordered flags) or 'host' (barriers)")
        self.context = context
        self.epochs = epochs
        self.timeout = float(timeout)
        # options of the buffered CommunicationObject that carries halos to/from other hosts
        self.remote_options = dict(remote_options or {})
        self._co, self._remote_bis = None, []
        self._bis = []
        self._initialized = False
        self._puts = []       # [(handle, src_ptr_array, n_src, dst_ptr_array, n_dst)]
        self._imports = []    # IPC bases to close
        self._keep = []
        self._ep = None       # ghx_epochs handle (epochs="device", node-local peers)
        self._hosts = None    # every rank's host (the epochs' node-local groups)

    # -- setup -------------------------------------------------------------------------------
    def add_field(self, bi):
        if self._initialized:
            raise RuntimeError("error: this bulk communication object has been initialized already")
        if bi.field.kind != 0:
            raise TypeError("bulk (zero-copy) exchange is implemented for structured fields")
        self._bis.append(bi)

    def add_fields(self, *bis):
        for bi in bis:
            self.add_field(bi)

    def initialized(self) -> bool:
        return self._initialized

    def _field_groups(self):
        """j-th field of each domain on this rank: (domain_id, j) -> field index."""
        seen, out = {}, []
        for bi in self._bis:
            d = bi.field.domain_id()
            j = seen.get(d, 0)
            seen[d] = j + 1
            out.append((d, j))
        return out

    def init(self):
        if self._initialized:
            return
        me = self.context.rank()
        world = self.context.size()
        groups = self._field_groups()
        host = hostname()
        mine = {"host": host, "fields": []}
        for bi, (d, j) in zip(self._bis, groups):
            h = (ctypes.c_ubyte * 64)()
            off = ctypes.c_uint64()
            _ghx.call("ghx_ipc_export", ctypes.c_void_p(bi.field.data_ptr()), h, ctypes.byref(off))
            recv = [(rid, tag, [(sp[0], sp[1]) for sp in spaces])
                    for rid, rr, tag, spaces in bi.pattern_container.recv_halos(bi.local_index)]
            mine["fields"].append({"domain": d, "j": j, "desc": bytes(bi.field.desc),
                                   "ipc": bytes(h), "offset": off.value, "recv": recv})
        allr = self.context.all_gather_object(mine)
        local = sorted(r for r, info in enumerate(allr) if info["host"] == host)
        remote = [r for r in range(world) if r not in local]
        if remote:
            # ranks on other hosts: their halos travel through a buffered exchange of the
            # pattern's remote part (the reference's remote pattern map + m_co,
            # bulk_communication_object.hpp:330-383, 674-694); node-local ones are put
            from .communication_object import CommunicationObject
            part = {}
            for bi in self._bis:
                pc = bi.pattern_container
                if id(pc) not in part:
                    part[id(pc)] = pc.filtered(remote, keep=True)
            self._remote_bis = [part[id(bi.pattern_container)](bi.field) for bi in self._bis]
            self._co = CommunicationObject(self.context, **self.remote_options)
        if self.epochs == "device" and world > 1:
            # one node-shared flag block per host (created by the host's lowest rank, attached
            # by the others, indexed by node-local position); sources: node-local ranks whose
            # puts land in my halos; targets: those mine land in
            srcs = sorted({rr for bi in self._bis
                           for _, rr, _, _ in bi.pattern_container.recv_halos(bi.local_index)
                           if rr != me and rr in local})
            tgts = sorted({rr for bi in self._bis
                           for _, rr, _, _ in bi.pattern_container.send_halos(bi.local_index)
                           if rr != me and rr in local})
            self._hosts = [info["host"] for info in allr]
            self._ep = attach_epochs(self.context, self._hosts, self.timeout, srcs, tgts)
            self._ep_peers = (srcs, tgts)
        msgs = put_messages(self._bis, groups, allr, local)
        # import peer allocations once per target field
        ptr_of = {}
        for (tr, ti) in sorted({m[2] for m in msgs}):
            if tr == me:
                ptr_of[(tr, ti)] = self._bis[ti].field.data_ptr()
                continue
            f = allr[tr]["fields"][ti]
            h = (ctypes.c_ubyte * 64).from_buffer_copy(f["ipc"])
            base, ptr = ctypes.c_void_p(), ctypes.c_void_p()
            _ghx.call("ghx_ipc_import", h, f["offset"], ctypes.byref(base), ctypes.byref(ptr))
            self._imports.append(base.value)
            ptr_of[(tr, ti)] = ptr.value
        for chunk, srcs, dsts in put_chunks(msgs):
            self._make_put(chunk, srcs, dsts, allr, ptr_of)
        self._initialized = True

    def _make_put(self, chunk, srcs, dsts, allr, ptr_of):
        src, dst, keep = put_entries(chunk, srcs, dsts, [bi.field.desc for bi in self._bis], allr)
        n = len(chunk)
        h = ctypes.c_void_p()
        _ghx.call("ghx_put_create", src, n, dst, n, ctypes.byref(h))
        sp = _ghx.ptr_array([self._bis[k].field.data_ptr() for k in srcs])
        dp = _ghx.ptr_array([ptr_of[t] for t in dsts])
        self._keep.append(keep)
        self._puts.append((h, sp, len(srcs), dp, len(dsts)))

    def check_epochs(self):
        """Raise if this rank's epochs recorded a failure (a wait timed out: a peer never reached
        the exchange; or a source failed an epoch wait)."""
        if self._ep is None:
            return
        why = epochs_error(self._ep, self._hosts, self.context.rank())
        if why:
            raise RuntimeError(f"bulk exchange failed (epoch timeout {self.timeout:.0f} s): {why}")

    # -- exchange ----------------------------------------------------------------------------
    def _barrier(self):
        dist = self.context.distributed
        if dist is not None and self.context.size() > 1:
            dist.barrier(group=self.context.group)

    def exchange(self) -> BulkHandle:
        import torch
        if not self._initialized:
            self.init()
        if not self._bis:
            return BulkHandle()
        stream = torch.cuda.current_stream(self._bis[0].field.device)
        remote = self._co.exchange(self._remote_bis) if self._co is not None else None
        if self.epochs == "host":
            stream.synchronize()  # this rank's kernels no longer read its halos: targets open
            self._barrier()
            for h, sp, ns, dp, nd in self._puts:
                _ghx.call("ghx_put_execute", h, sp, ns, dp, nd, stream.cuda_stream)
            stream.synchronize()  # this rank's puts have landed in peer memory
            self._barrier()       # ... and every other rank's in ours
            return BulkHandle(remote=remote)
        s = stream.cuda_stream
        if self._ep is not None:
            _ghx.call("ghx_epochs_enqueue", self._ep, 0, s)
        for h, sp, ns, dp, nd in self._puts:
            _ghx.call("ghx_put_execute", h, sp, ns, dp, nd, s)
        if self._ep is not None:
            _ghx.call("ghx_epochs_enqueue", self._ep, 1, s)
        if torch.cuda.is_current_stream_capturing():
            return BulkHandle(self, None)  # captured into a graph: completion is the replay's
        ev = self.__dict__.get("_event")
        if ev is None:
            ev = self._event = torch.cuda.Event()
        ev.record(stream)
        return BulkHandle(self, ev, remote)

    def bytes_per_exchange(self) -> int:
        tot = 0
        for h, *_ in self._puts:
            b = ctypes.c_uint64()
            _ghx.call("ghx_put_info", h, ctypes.byref(b), None)
            tot += b.value
        return tot

    def __del__(self):
        try:
            for h, *_ in self._puts:
                _ghx.lib().ghx_put_destroy(h)
            for b in self._imports:
                _ghx.lib().ghx_ipc_close(ctypes.c_void_p(b))
            if self._ep is not None:
                _ghx.lib().ghx_epochs_destroy(self._ep)
        except Exception:
            pass
        self._puts, self._imports, self._ep = [], [], None


def make_bulk_communication_object(context, epochs: str = "device", timeout: float = 30.0,
                                   remote_options=None) -> BulkCommunicationObject:
    """epochs="device": stream-ordered per-pair epochs (no host synchronisation); "host": the
    drain + barrier form. timeout: seconds an epoch wait may take before wait() raises.
    remote_options: CommunicationObject options for the halos of ranks on other hosts (e.g.
    staging="host"); node-local ranks always get puts."""
    return BulkCommunicationObject(context, epochs=epochs, timeout=timeout,
                                   remote_options=remote_options)
