"""The C++ host mirror (orb_slam2-chinese-annotation_amd/host/orb_amd.hpp):
compiles with plain g++ against the C ABI (CPU test) and, on the GPU, extracts
and matches bit-exactly vs the oracle (GPU test)."""
import subprocess

import pytest

from conftest import PKG_DIR, ROOT

SRC = ROOT / "tests" / "cpp" / "test_host.cpp"


def _build(out):
    cmd = ["g++", "-std=c++17", "-O2", str(SRC), "-o", str(out),
           f"-L{PKG_DIR / 'lib'}", "-lorb_amd", f"-L{ROOT / 'oracle'}", "-lorb_oracle",
           f"-Wl,-rpath,{PKG_DIR / 'lib'}", f"-Wl,-rpath,{ROOT / 'oracle'}",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


def test_host_header_compiles_with_gxx(tmp_path, orb, oracle):
    orb.lib()
    _build(tmp_path / "test_host")
    assert (tmp_path / "test_host").exists()


@pytest.mark.gpu
def test_host_mirror_on_gpu(gpu, oracle, tmp_path):
    exe = tmp_path / "test_host"
    _build(exe)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")
