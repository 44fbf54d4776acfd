"""The C++ limiter mirror (distributedratelimiting.redis_amd/host) through its own test
program, tests/host/host_test.cpp.  CPU: option validation, value types, registration.
GPU: decisions through libtbe.so checked against the C oracle and hand-derived cases."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributedratelimiting.redis_amd")
SRC = os.path.join(ROOT, "tests", "host", "host_test.cpp")
BIN = os.path.join(ROOT, "tests", "host", "host_test")


def build_host_test() -> str:
    """Compile the test program against libtbe_host.so, libtbe.so and the oracle
    library (checker).  Relative rpaths so the built binary also runs on the GPU box."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_tbe_build", os.path.join(PKG, "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build_host()
    from oracle.build import build_oracle
    oracle_lib = build_oracle()
    deps = [SRC, mod.HOST_LIB, oracle_lib, os.path.join(PKG, "host", "rate_limiting.hpp")]
    if os.path.exists(BIN) and all(os.path.getmtime(d) <= os.path.getmtime(BIN) for d in deps):
        return BIN
    cmd = ["g++", "-O1", "-std=c++17", "-Wall", "-pthread", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(PKG, "host"), "-o", BIN + ".tmp", SRC,
           "-L", PKG, "-ltbe_host", "-ltbe", "-L", os.path.dirname(oracle_lib), "-ltbref",
           "-L", "/opt/rocm/lib",
           "-Wl,-rpath,$ORIGIN/../../distributedratelimiting.redis_amd",
           "-Wl,-rpath,$ORIGIN/../../oracle/lib"]
    subprocess.run(cmd, check=True)
    os.replace(BIN + ".tmp", BIN)
    return BIN


def run(mode: str):
    exe = build_host_test() if mode == "cpu" else BIN
    if not os.path.exists(exe):
        pytest.fail("tests/host/host_test is not built (run __graft_entry__.build())")
    p = subprocess.run([exe, mode], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_host_cpp_cpu(oracle_lib):
    out = run("cpu")
    assert "0 failed" in out


@pytest.mark.gpu
def test_host_cpp_gpu(gpu):
    out = run("gpu")
    assert "0 failed" in out
