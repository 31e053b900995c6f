"""ghex_amd — MI355X-native halo pack/unpack path for GHEX (drop-in for the field-descriptor
pack/unpack concept, the pattern and the communication object of that path).

Python mirror of the reference's Python API (bindings/python/src/ghex/...) over the C ABI of
libghx.so (include/ghx.h). Device memory and streams come from PyTorch-ROCm, transport from
torch.distributed (backend "nccl" = RCCL over xGMI). The native library is required: importing
any compute entry point without it raises ImportError — there is no CPU fallback.
"""
from ._ghx import GhxError, LIB_PATH  # noqa: F401
from .context import Context, make_context  # noqa: F401
from .bulk_communication_object import (BulkCommunicationObject,  # noqa: F401
                                        make_bulk_communication_object)

__version__ = "0.1.0"

# the build configuration, as the reference's ghex.__config__ / config() / print_config()
# (bindings/python/src/_pyghex/config.cpp): the exchange's transport is torch.distributed
# ("nccl" = RCCL between GPUs, gloo for host staging), the kernels are gfx950 HIP.
__config__ = {"transport": "RCCL", "gpu": True, "gpu_mode": "hip", "xpmem": False,
              "version": __version__, "arch": "gfx950"}


def config() -> dict:
    return dict(__config__)


def print_config(d: dict = None) -> None:
    d = config() if d is None else d
    print("GHEX's configuration:\n" + "".join(f"     {k:<16}: {str(v):>10}\n" for k, v in d.items()),
          end="")


def native_library():
    """Load (and return) libghx.so; raises ImportError if it has not been built."""
    from ._ghx import lib
    return lib()
