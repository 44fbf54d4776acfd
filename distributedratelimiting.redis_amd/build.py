"""Build the HIP engine in-tree: ``libtbe.so`` next to this file (gfx950 only).

Flags that matter for parity: ``-ffp-contract=off`` (the reference script's
``v + dt*rate`` is two roundings; an FMA would differ in ~3% of refills)
and no fast-math (f64 division must stay the IEEE-correct sequence).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.realpath(__file__))   # also when imported through the distributedratelimiting/ symlink
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", n) for n in ("tbe_engine.hip", "tbe_tools.hip", "tbe_cluster.hip", "tbe_strdir.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", n) for n in ("tbe_device.hpp", "tbe_numfmt.hpp", "tbe_hash.hpp")] + \
    [os.path.join(ROOT, "include", n) for n in ("tbe.h", "tbe_tools.h", "tbe_cluster.h", "tbe_strdir.h")]
LIB = os.path.join(HERE, "libtbe.so")
ARCH = "gfx950"
HIPCC_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-result", f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError("hipcc not found")


def _digest(deps, flags) -> str:
    import hashlib
    h = hashlib.sha256(" ".join(flags).encode())
    for d in deps:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()


def up_to_date(target: str, deps, flags=()) -> bool:
    """The library was built from exactly these sources and flags: a SHA-256 of both is
    stored beside it (target + ".sha256"), so copying the tree (file times change, e.g.
    on the GPU box) neither forces a rebuild nor hides a stale one."""
    stamp = target + ".sha256"
    if not (os.path.exists(target) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == _digest(deps, flags)


def _stamp(target: str, deps, flags=()) -> None:
    with open(target + ".sha256", "w") as f:
        f.write(_digest(deps, flags) + "\n")


def build_engine(force: bool = False, verbose: bool = False, defines=(), out: str = LIB) -> str:
    """Build libtbe.so (or, for ablation experiments, a variant with extra -D defines
    written to `out`)."""
    flags = HIPCC_FLAGS + [f"-D{d}" for d in defines]
    if not force and up_to_date(out, DEPS, flags):
        if verbose:
            print(f"build: {os.path.basename(out)} up to date (sources sha256 {_digest(DEPS, flags)[:12]})",
                  file=sys.stderr)
        return out
    cmd = [hipcc()] + flags + ["-I", os.path.join(ROOT, "include"), "-o", out + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    _stamp(out, DEPS, flags)
    return out


HOST_SRC = os.path.join(HERE, "host", "rate_limiting.cpp")
HOST_DEPS = [HOST_SRC, os.path.join(HERE, "host", "rate_limiting.hpp"), os.path.join(ROOT, "include", "tbe.h")]
HOST_LIB = os.path.join(HERE, "libtbe_host.so")
CXX_FLAGS = ["-O2", "-std=c++17", "-Wall", "-Wextra", "-Wno-unused-parameter", "-pthread"]


def build_host(force: bool = False, verbose: bool = False) -> str:
    """libtbe_host.so: the C++ limiter classes (host/) over libtbe.so."""
    build_engine(verbose=verbose)
    if not force and up_to_date(HOST_LIB, HOST_DEPS + [LIB], CXX_FLAGS):
        return HOST_LIB
    cmd = ["g++"] + CXX_FLAGS + ["-fPIC", "-shared", "-I", os.path.join(ROOT, "include"),
                                 "-o", HOST_LIB + ".tmp", HOST_SRC, "-L", HERE, "-ltbe",
                                 "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(HOST_LIB + ".tmp", HOST_LIB)
    _stamp(HOST_LIB, HOST_DEPS + [LIB], CXX_FLAGS)
    return HOST_LIB


if __name__ == "__main__":
    print(build_engine(force="--force" in sys.argv, verbose=True))
    print(build_host(force="--force" in sys.argv, verbose=True))
