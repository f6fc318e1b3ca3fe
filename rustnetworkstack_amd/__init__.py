"""MI355X-native batched Internet checksum — the hot path of jbush001/RustNetworkStack
(src/stack/util.rs:86-119, 180-207), as hand-written gfx950 HIP kernels behind a C ABI
(include/rns_checksum.h).

* ``util``      — the reference's `netstack::util` checksum surface, same names and errors;
* ``batch``     — device-resident / host-resident batch API (torch tensors, numpy arrays);
* ``workloads`` — the synthetic packet batches BASELINE.json's configs name.
"""
from . import _lib, util  # noqa: F401
from ._lib import ChecksumError, ChecksumLibraryMissing  # noqa: F401

__all__ = ["util", "batch", "workloads", "ChecksumError", "ChecksumLibraryMissing"]


def __getattr__(name):
    if name in ("batch", "workloads"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
