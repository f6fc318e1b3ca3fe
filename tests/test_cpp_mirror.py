"""Builds and runs the C++ netstack::util mirror's tests (tests/cpp), which follow
the reference's util.rs test module function by function."""
import os
import subprocess

from conftest import ROOT


def test_cpp_mirror(tmp_path):
    exe = tmp_path / "test_netstack_util"
    pkg = os.path.join(ROOT, "rustnetworkstack_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_netstack_util.cpp"), "-L", pkg, "-lrns_checksum",
                           f"-Wl,-rpath,{pkg}", "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout
