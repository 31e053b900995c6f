"""ghex.util's Architecture (bindings/python/src/ghex/util.py:22-24), so that reference-style
calls make_field_descriptor(..., arch=Architecture.GPU) work unchanged. This package is the
device path: Architecture.CPU is refused (no CPU fallback)."""
from enum import Enum


class Architecture(Enum):
    CPU = "cpu"
    GPU = "gpu"


def check_arch(arch) -> None:
    """None (derive from the field) and GPU are accepted; CPU raises."""
    if arch is None:
        return
    value = arch.value if isinstance(arch, Architecture) else str(arch).lower()
    if value != "gpu":
        raise ValueError("ghex_amd is the device path: fields must live in GPU memory "
                         f"(arch={arch!r} is not supported)")


class _CAI:
    """Re-exposes a __hip_array_interface__ under the name torch reads."""

    def __init__(self, obj):
        self._obj = obj  # keeps the producer alive as long as the view
        self.__cuda_array_interface__ = obj.__hip_array_interface__


def as_device_tensor(field):
    """The field as a torch device tensor, sharing its memory: a torch tensor as is, or any
    object exposing __cuda_array_interface__ / __hip_array_interface__ (the GPU forms the
    reference binding accepts, bindings/python/src/ghex/structured/regular.py:66-98) viewed
    zero-copy. Host arrays (__array_interface__) are refused: this package is the device path."""
    import torch
    if isinstance(field, torch.Tensor):
        return field
    src = None
    if hasattr(field, "__cuda_array_interface__"):
        src = field
    elif hasattr(field, "__hip_array_interface__"):
        src = _CAI(field)
    if src is None:
        raise TypeError("ghex_amd fields live in device memory: pass a torch tensor on the GPU "
                        "or an object with __cuda_array_interface__ / __hip_array_interface__"
                        + (" (a host array was given)" if hasattr(field, "__array_interface__")
                           else ""))
    cai = src.__cuda_array_interface__
    t = torch.as_tensor(src, device="cuda")
    ptr = cai["data"][0] if isinstance(cai.get("data"), (tuple, list)) else None
    if ptr is not None and t.numel() and t.data_ptr() != ptr:
        raise RuntimeError("the array interface was copied, not viewed; pass a torch tensor")
    return t
