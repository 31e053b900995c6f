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
