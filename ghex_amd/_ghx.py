"""ctypes binding of libghx.so (include/ghx.h). Fails loudly when the library is missing:
there is no CPU fallback anywhere in ghex_amd."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libghx.so")

MAX_DIM = 4
MAX_SLOTS = 64

c_i32, c_i64, c_u64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p


class FieldDesc(ctypes.Structure):
    _fields_ = [("dim", c_i32), ("elem_size", c_i32), ("layout", c_i32 * MAX_DIM),
                ("byte_strides", c_i64 * MAX_DIM), ("offsets", c_i32 * MAX_DIM),
                ("extents", c_i32 * MAX_DIM), ("num_components", c_i32),
                ("has_components", c_i32)]


class Box(ctypes.Structure):
    _fields_ = [("first", c_i32 * MAX_DIM), ("last", c_i32 * MAX_DIM)]


class PackEntry(ctypes.Structure):
    _fields_ = [("field", FieldDesc), ("field_slot", c_i32), ("buffer_slot", c_i32),
                ("buffer_offset", c_u64), ("boxes", ctypes.POINTER(Box)), ("n_boxes", c_i32)]


class UDataDesc(ctypes.Structure):
    _fields_ = [("elem_size", c_i32), ("levels", c_i32), ("levels_first", c_i32),
                ("index_stride", c_i64), ("level_stride", c_i64)]


class UPackEntry(ctypes.Structure):
    _fields_ = [("data", UDataDesc), ("field_slot", c_i32), ("buffer_slot", c_i32),
                ("buffer_offset", c_u64), ("lids", ctypes.POINTER(c_i64)), ("n_lids", c_i64)]


class RegularDomain(ctypes.Structure):
    _fields_ = [("id", c_i32), ("rank", c_i32), ("first", c_i32 * 3), ("last", c_i32 * 3)]


class ExchangeItem(ctypes.Structure):
    _fields_ = [("pattern", c_vp), ("local_index", c_i32), ("kind", c_i32), ("field", FieldDesc),
                ("udata", UDataDesc), ("align", c_i32), ("tag_offset", c_i32)]


P = ctypes.POINTER
_SIGS = {
    "ghx_tune": (c_i32, [ctypes.c_char_p, c_i32]),
    "ghx_launch_timing": (c_i32, [c_i32]),
    "ghx_launch_timing_read": (c_i32, [ctypes.POINTER(ctypes.c_float), c_i32,
                                       ctypes.POINTER(c_i32)]),
    "ghx_last_error": (ctypes.c_char_p, []),
    "ghx_version": (ctypes.c_char_p, []),
    "ghx_plan_create": (c_i32, [P(PackEntry), c_i32, c_i32, P(c_vp)]),
    "ghx_plan_execute": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_plan_destroy": (c_i32, [c_vp]),
    "ghx_plan_info": (c_i32, [c_vp, P(c_u64), P(c_i32), P(c_i32)]),
    "ghx_structured_pack": (c_i32, [P(FieldDesc), c_vp, c_vp, P(Box), c_i32, c_vp]),
    "ghx_structured_unpack": (c_i32, [P(FieldDesc), c_vp, c_vp, P(Box), c_i32, c_vp]),
    "ghx_uplan_create": (c_i32, [P(UPackEntry), c_i32, c_i32, P(c_vp)]),
    "ghx_uplan_execute": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_uplan_destroy": (c_i32, [c_vp]),
    "ghx_uplan_info": (c_i32, [c_vp, P(c_u64), P(c_i32), P(c_i32)]),
    "ghx_regular_halo_boxes": (c_i32, [c_i32, P(c_i32), P(c_i32), P(c_i32), P(c_i32), P(c_i32),
                                       P(c_i32), P(Box), P(Box), c_i32, P(c_i32)]),
    "ghx_regular_pattern_create": (c_i32, [c_i32, P(RegularDomain), c_i32, P(c_i32), P(c_i32),
                                           P(c_i32), P(c_i32), c_i32, P(c_vp)]),
    "ghx_staged_pattern_create": (c_i32, [c_i32, P(RegularDomain), c_i32, P(c_i32), P(c_i32),
                                          P(c_i32), P(c_i32), P(c_i32), c_i32, P(c_vp)]),
    "ghx_udomain_create": (c_i32, [c_i32, P(c_i64), c_i64, P(c_i64), c_i64, P(c_vp)]),
    "ghx_udomain_destroy": (c_i32, [c_vp]),
    "ghx_udomain_info": (c_i32, [c_vp, P(c_i32), P(c_i64), P(c_i64), P(c_i64)]),
    "ghx_udomain_halo": (c_i32, [c_vp, P(c_i64), c_i64, P(c_i64), c_i64, P(c_i64)]),
    "ghx_upattern_create": (c_i32, [P(c_vp), c_i32, c_i32, c_i32, c_i32, P(c_vp)]),
    "ghx_upattern_add_halos": (c_i32, [c_vp, c_i32, c_i32, P(c_i32), P(c_i64), P(c_i64),
                                       P(c_i64)]),
    "ghx_upattern_record": (c_i32, [c_vp, c_i64, P(c_i32), P(c_i32), P(c_i32), P(c_i32),
                                    P(c_i64), P(P(c_i64))]),
    "ghx_upattern_add_recv": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, P(c_i64), c_i64]),
    "ghx_upattern_finish": (c_i32, [c_vp, P(c_vp)]),
    "ghx_upattern_destroy": (c_i32, [c_vp]),
    "ghx_pattern_destroy": (c_i32, [c_vp]),
    "ghx_pattern_filter": (c_i32, [c_vp, P(c_i32), c_i32, c_i32, P(c_vp)]),
    "ghx_pattern_num_domains": (c_i32, [c_vp, P(c_i32)]),
    "ghx_pattern_max_tag": (c_i32, [c_vp, P(c_i32)]),
    "ghx_pattern_domain_id": (c_i32, [c_vp, c_i32, P(c_i32)]),
    "ghx_pattern_num_keys": (c_i32, [c_vp, c_i32, c_i32, P(c_i32)]),
    "ghx_pattern_key": (c_i32, [c_vp, c_i32, c_i32, c_i32, P(c_i32), P(c_i32), P(c_i32),
                                P(c_i32), P(c_i64)]),
    "ghx_pattern_key_boxes": (c_i32, [c_vp, c_i32, c_i32, c_i32, P(Box), P(Box), c_i32]),
    "ghx_pattern_key_lids": (c_i32, [c_vp, c_i32, c_i32, c_i32, P(c_i64), c_i64]),
    "ghx_exchange_create": (c_i32, [P(ExchangeItem), c_i32, P(c_vp)]),
    "ghx_exchange_destroy": (c_i32, [c_vp]),
    "ghx_exchange_num_buffers": (c_i32, [c_vp, c_i32, P(c_i32)]),
    "ghx_exchange_buffer": (c_i32, [c_vp, c_i32, c_i32, P(c_i32), P(c_i32), P(c_i32), P(c_i32),
                                    P(c_u64)]),
    "ghx_exchange_pack": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_unpack": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_self_fusable": (c_i32, [c_vp, P(c_i32)]),
    "ghx_exchange_self": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_mixed": (c_i32, [c_vp, P(c_i32)]),
    "ghx_exchange_pack_self": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_unpack_peers": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_split": (c_i32, [c_vp]),
    "ghx_exchange_pack_buffer": (c_i32, [c_vp, c_i32, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_exchange_unpack_buffer": (c_i32, [c_vp, c_i32, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_rccl_open": (c_i32, [ctypes.c_char_p]),
    "ghx_rccl_unique_id": (c_i32, [P(ctypes.c_ubyte)]),
    "ghx_rccl_comm_init": (c_i32, [P(ctypes.c_ubyte), c_i32, c_i32, P(c_vp)]),
    "ghx_rccl_comm_destroy": (c_i32, [c_vp]),
    "ghx_rccl_comm_check": (c_i32, [c_vp]),
    "ghx_pipeline_create": (c_i32, [c_vp, c_i32, c_i32, P(c_i32), P(c_vp), P(c_i32), c_i32,
                                    P(c_vp)]),
    "ghx_pipeline_run": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_pipeline_destroy": (c_i32, [c_vp]),
    "ghx_unstructured_pack": (c_i32, [P(UDataDesc), c_vp, c_vp, c_vp, c_i32, ctypes.c_int64, c_vp]),
    "ghx_unstructured_unpack": (c_i32, [P(UDataDesc), c_vp, c_vp, c_vp, c_i32, ctypes.c_int64, c_vp]),
    "ghx_ipc_export": (c_i32, [c_vp, P(ctypes.c_ubyte), P(ctypes.c_uint64)]),
    "ghx_ipc_import": (c_i32, [P(ctypes.c_ubyte), ctypes.c_uint64, P(c_vp), P(c_vp)]),
    "ghx_ipc_close": (c_i32, [c_vp]),
    "ghx_put_create": (c_i32, [P(PackEntry), c_i32, P(PackEntry), c_i32, P(c_vp)]),
    "ghx_put_execute": (c_i32, [c_vp, P(c_vp), c_i32, P(c_vp), c_i32, c_vp]),
    "ghx_put_info": (c_i32, [c_vp, P(ctypes.c_uint64), P(c_i32)]),
    "ghx_put_destroy": (c_i32, [c_vp]),
    "ghx_epochs_create": (c_i32, [ctypes.c_char_p, c_i32, c_i32, c_i32, ctypes.c_double, P(c_vp)]),
    "ghx_epochs_unlink": (c_i32, [ctypes.c_char_p]),
    "ghx_epochs_peers": (c_i32, [c_vp, P(c_i32), c_i32, P(c_i32), c_i32]),
    "ghx_epochs_enqueue": (c_i32, [c_vp, c_i32, c_vp]),
    "ghx_epochs_status": (c_i32, [c_vp, P(c_i32), P(ctypes.c_uint64)]),
    "ghx_epochs_info": (c_i32, [c_vp, P(c_i32), P(c_i32)]),
    "ghx_epochs_counter": (c_i32, [c_vp, P(c_vp)]),
    "ghx_exchange_set_parity": (c_i32, [c_vp, c_i32, c_vp, ctypes.c_uint32, P(ctypes.c_int64), c_i32]),
    "ghx_epochs_destroy": (c_i32, [c_vp]),
    "ghx_copier_create": (c_i32, [ctypes.c_uint64, ctypes.c_double, P(c_vp)]),
    "ghx_copier_info": (c_i32, [c_vp, P(c_i32), P(c_i32), P(ctypes.c_float), P(ctypes.c_float),
                                P(ctypes.c_float)]),
    "ghx_copier_submit": (c_i32, [c_vp, c_vp, c_vp, ctypes.c_uint64, c_i32, ctypes.c_int64,
                                  P(ctypes.c_uint64)]),
    "ghx_copier_wait": (c_i32, [c_vp, ctypes.c_uint64]),
    "ghx_copier_acquire": (c_i32, [c_vp, c_vp]),
    "ghx_copier_destroy": (c_i32, [c_vp]),
}
EXPORTED = tuple(_SIGS)

_lib = None


class GhxError(RuntimeError):
    """A failed ghx_* call (the reference raises std::runtime_error)."""


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"ghex_amd native library missing: {LIB_PATH}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
                "There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().ghx_last_error().decode()
        raise GhxError(f"{what} failed ({rc}): {msg}")


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def ptr_array(ptrs):
    arr = (c_vp * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def i32_array(vals):
    return (c_i32 * max(1, len(vals)))(*vals)


def i64_array(vals):
    return (c_i64 * max(1, len(vals)))(*vals)


def i64_ptr(a):
    """ctypes int64* into a C-contiguous numpy int64 array (kept alive by the caller)."""
    return a.ctypes.data_as(ctypes.POINTER(c_i64))
