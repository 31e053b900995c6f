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


def native_library():
    """Load (and return) libghx.so; raises ImportError if it has not been built."""
    from ._ghx import lib
    return lib()
