"""A plain C program calls the batch C ABI the way a Rust / cgo / FFI binding would
(no torch, no Python in the process): tests/c/test_batch_abi.c.  It checks the
host-resident and device-resident batch entries against the oracle and that errors
come back as status codes.  `make` builds it in-tree (tests/c/test_batch_abi)."""
import os
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "c", "test_batch_abi.c")
EXE = os.path.join(ROOT, "tests", "c", "test_batch_abi")
PKG = os.path.join(ROOT, "rustnetworkstack_amd")


def _compile(out: str) -> None:
    subprocess.check_call(["gcc", "-std=gnu11", "-O1", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", SRC,
                           os.path.join(ROOT, "oracle", "csum_oracle.c"), "-L", PKG, "-lrns_checksum",
                           f"-Wl,-rpath,{PKG}", "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib",
                           "-lpthread", "-o", out])


def test_c_caller_builds_and_fails_loudly_without_gpu(tmp_path):
    from rustnetworkstack_amd import _lib
    if _lib.load().rns_device_count() > 0:
        pytest.skip("checks the GPU-less behaviour")
    exe = str(tmp_path / "test_batch_abi")
    _compile(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "rns_host_alloc failed" in r.stderr


@pytest.mark.gpu
def test_c_caller_on_gpu(tmp_path):
    exe = EXE
    if not os.path.exists(exe):  # `make` builds it in-tree; a tree without it gets a private copy
        exe = str(tmp_path / "test_batch_abi")
        _compile(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "all checks passed" in r.stdout
