"""The C-ABI library loads, exports exactly what include/rns_checksum.h declares,
and its batch entry points fail loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from rustnetworkstack_amd import _lib

HEADER = os.path.join(ROOT, "include", "rns_checksum.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(rns_[a-z0-9_]+)\s*\(", text))


def test_header_matches_binding_list():
    assert header_functions() == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = header_functions() - exported
    assert not missing, f"declared but not exported: {missing}"


def test_loads_and_versions():
    lib = _lib.load()
    assert lib.rns_abi_version() == 1
    assert b"gfx950" in lib.rns_build_info()
    assert lib.rns_strerror(_lib.RNS_E_EMPTY).startswith(b"empty slice")


def test_library_contains_gfx950_code_object():
    out = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH], text=True)
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob and b"csum_batch_kernel" in blob


def test_header_compiles_as_c():
    src = '#include "rns_checksum.h"\nint main(void){ return rns_abi_version() == RNS_ABI_VERSION ? 0 : 1; }\n'
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-x", "c", "-",
                    "-fsyntax-only"], input=src, text=True, check=True)


@pytest.mark.skipif(_lib.load().rns_device_count() > 0, reason="checks the GPU-less behaviour")
def test_batch_calls_fail_loudly_without_gpu():
    lib = _lib.load()
    out = ctypes.c_uint16()
    fake = ctypes.c_void_p(4096)
    st = lib.rns_csum_batch_dev(fake, 16, fake, fake, None, ctypes.addressof(out), 1, 0, 0, None, None)
    assert st == _lib.RNS_E_NODEVICE
    st = lib.rns_csum_batch_dev_off32(fake, 16, fake, fake, None, ctypes.addressof(out), 1, 0, 0, None, None)
    assert st == _lib.RNS_E_NODEVICE
    p = ctypes.c_void_p()
    assert lib.rns_host_ctx_create(0, 1 << 20, 2, ctypes.byref(p)) == _lib.RNS_E_NODEVICE
    assert lib.rns_fill_splitmix64_dev(fake, 64, 1, None) == _lib.RNS_E_NODEVICE
    assert lib.rns_csum_fill_dev(fake, 64, fake, fake, None, None, 0, None, 1, 0, None, None) == _lib.RNS_E_NODEVICE
    assert lib.rns_csum_fill_packed_dev(fake, 64, fake, fake, 4, None, None, 16, None, 1, 0, 0, None,
                                        None) == _lib.RNS_E_NODEVICE
    assert lib.rns_rx_verify_dev(fake, 64, fake, fake, 1, fake, fake, fake, None, None) == _lib.RNS_E_NODEVICE
    assert lib.rns_tx_fill_dev(fake, 64, fake, fake, 1, None, None) == _lib.RNS_E_NODEVICE
    assert lib.rns_tx_fill_packed_dev(fake, 64, fake, fake, 4, 1, None, 0, None) == _lib.RNS_E_NODEVICE
    assert lib.rns_rx_verify_strided_dev(fake, 64, 0, 64, fake, 1, fake, fake, fake, None,
                                         None) == _lib.RNS_E_NODEVICE
    assert lib.rns_tx_fill_chain_dev(fake, 64, fake, fake, 1, fake, 1, None, None) == _lib.RNS_E_NODEVICE


def test_argument_errors_before_the_device():
    """Bad arguments are reported as RNS_E_INVALID before any device call (no GPU needed):
    strided offsets that would wrap 64 bits, a packed finalize below 16-byte alignment, a
    packed receive into an MRU of more than 65535 bytes."""
    lib = _lib.load()
    fake = ctypes.c_void_p(4096)
    out = ctypes.c_uint16()
    big = (1 << 63) + 16
    assert lib.rns_csum_batch_strided_dev(fake, 64, 0, big, 64, None, ctypes.addressof(out), 3, 0, None,
                                          None) == _lib.RNS_E_INVALID
    assert lib.rns_csum_batch_strided_dev(fake, 64, (1 << 64) - 8, 16, 64, None, ctypes.addressof(out), 1, 0, None,
                                          None) == _lib.RNS_E_INVALID
    assert lib.rns_rx_verify_strided_dev(fake, 64, 0, big, fake, 3, fake, fake, fake, None,
                                         None) == _lib.RNS_E_INVALID
    assert lib.rns_tx_fill_packed_dev(fake, 64, fake, fake, 3, 1, None, 0, None) == _lib.RNS_E_INVALID
    assert lib.rns_tx_fill_chain_dev(fake, 64, fake, fake, 1, None, 1, None, None) == _lib.RNS_E_INVALID
    assert lib.rns_tx_fill_chain_dev(fake, 64, fake, fake, 1, fake, _lib.RNS_CHAIN_MAX_PACKETS + 1, None,
                                     None) == _lib.RNS_E_INVALID
    end = ctypes.c_uint64()
    assert lib.rns_io_recv_batch_packed(0, fake, 4096, 70000, 4, fake, fake, ctypes.byref(end), 0) == \
        _lib.RNS_E_INVALID


def test_python_batch_api_refuses_cpu_tensors():
    import torch

    from rustnetworkstack_amd.batch import csum_batch
    with pytest.raises(ValueError, match="no CPU fallback"):
        csum_batch(torch.zeros(16, dtype=torch.uint8), torch.zeros(1, dtype=torch.int64),
                   torch.ones(1, dtype=torch.int32))


def test_missing_library_is_loud(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.ChecksumLibraryMissing):
        _lib.load()
