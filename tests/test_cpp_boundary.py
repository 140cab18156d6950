"""The C++ boundary compiles for a reference-style Decoder subclass (tests/cpp/subclass_decoder.cpp):
build it with g++ against include/ and libpolarcode_amd.so, run it (CPU only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "antpolarcodes_amd", "lib")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_reference_style_subclass_compiles_and_runs(tmp_path):
    exe = str(tmp_path / "subclass_decoder")
    src = os.path.join(ROOT, "tests", "cpp", "subclass_decoder.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                    "-L", LIB, "-lpolarcode_amd", "-lpcg", f"-Wl,-rpath,{LIB}"], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "subclass_decoder ok" in r.stdout
