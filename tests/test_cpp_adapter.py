"""The C++ KVVector adapter (parameter_server_amd/csrc/kv_vector.h) built
with plain g++ against libpsg.so -- the way a reference server would link
it.  The host mode checks slice / shard bounds; the GPU
mode runs the merge path and compares with the oracle bit-for-bit."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "parameter_server_amd")
ORC = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libpsg.so")):
        pytest.fail("libpsg.so not built (run __graft_entry__.build())")
    exe = str(tmp_path_factory.mktemp("cpp") / "test_kv_vector")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
           os.path.join(ROOT, "tests", "cpp", "test_kv_vector.cc"),
           "-o", exe, f"-L{LIB}", "-lpsg", f"-L{ORC}", "-lorc",
           f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,{ORC}"]
    subprocess.run(cmd, check=True)
    return exe


def test_cpp_adapter_host(driver):
    r = subprocess.run([driver, "host"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_adapter_gpu(driver):
    r = subprocess.run([driver, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
