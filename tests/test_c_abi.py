"""The C ABI from C: tests/c_client/abi_client.c includes include/concrete_hip.h, is compiled
by gcc as C99 (and the header alone as C++17), links libconcrete_hip.so and runs its
device-free calls — the boundary a cgo / JNI / N-API binding would use."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "concrete_amd")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_c_client_compiles_links_and_runs(tmp_path):
    assert os.path.exists(os.path.join(LIBDIR, "libconcrete_hip.so")), "build the library first"
    exe = tmp_path / "abi_client"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_client", "abi_client.c"), "-L", LIBDIR, "-lconcrete_hip",
                    f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=120)
    assert "abi_client ok" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_header_is_valid_cpp(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text('#include "concrete_hip.h"\nint main() { return concrete_hip_abi_version() == 5 ? 0 : 1; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                    str(src)], check=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_sdfg_client_compiles_and_links(tmp_path):
    """The stream-emulator replay client (run by tests/test_gpu_sdfg.py on the GPU) is plain C99
    against include/concrete_hip.h Part 5; here it must compile warning-free and link."""
    exe = tmp_path / "sdfg_client"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_client", "sdfg_client.c"), "-L", LIBDIR, "-lconcrete_hip",
                    f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    # bad usage is refused before any device call
    assert subprocess.run([str(exe)], capture_output=True, timeout=60).returncode == 2
