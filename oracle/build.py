"""Build the C restatement ``oracle/tb_ref.c`` into ``oracle/lib/libtbref.so``.

TEST INFRASTRUCTURE.  The reference itself (C# + Lua inside Redis) cannot be built in
this image (no .NET, no Redis, no Lua VM: SURVEY.md §8c), so there is no
``oracle/_ref`` build; see DESIGN.md "Parity".
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "tb_ref.c")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libtbref.so")
CFLAGS = ["-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-pthread",
          "-Wall"]


def build_oracle(force: bool = False) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    subprocess.run(["gcc"] + CFLAGS + ["-o", LIB + ".tmp", SRC, "-lm"], check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_oracle(force="--force" in sys.argv))
