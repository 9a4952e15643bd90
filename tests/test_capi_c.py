"""The ABI from C and C++ without Python: tests/c/capi_min.c (plain C, gcc) builds against
include/mtg_boss.h and links libmtg_boss.so; the INTEGRATION.md adapter (C++) compiles against
declaration-only stand-ins of the reference headers (boss_chunk_construct.hpp:18-34).  The GPU
test runs capi_min on device 0 against the oracle-written fixture."""
import os
import re
import subprocess

import pytest

from conftest import GOLDEN, ROOT

boss = __import__("importlib").import_module("projects2014-metagenome_amd.boss")

C_DIR = os.path.join(ROOT, "tests", "c")


def _build_capi_min(out):
    libdir = os.path.dirname(boss.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(C_DIR, "capi_min.c"),
                    "-L", libdir, "-l:" + os.path.basename(boss.LIB_PATH),
                    "-Wl,-rpath," + libdir, "-o", out], check=True, capture_output=True, text=True)


def test_capi_min_compiles_and_links(tmp_path):
    exe = str(tmp_path / "capi_min")
    _build_capi_min(exe)
    assert os.access(exe, os.X_OK)


def test_integration_adapter_compiles(tmp_path):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. C++ adapter"):text.index("## 3.")]
    code = re.search(r"```cpp\n(.*?)```", sec, re.S).group(1)
    src = tmp_path / "adapter.cpp"
    src.write_text(code + "\nint main() { return 0; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra",
                        "-I", os.path.join(C_DIR, "stubs"), "-I", os.path.join(ROOT, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_capi_min_build_matches_fixture(tmp_path):
    exe = str(tmp_path / "capi_min")
    _build_capi_min(exe)
    r = subprocess.run([exe, os.path.join(GOLDEN, "capi_reads.fa"), "19", "1", "8",
                        os.path.join(GOLDEN, "capi_k20_fixture.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "identical to the fixture" in r.stdout
