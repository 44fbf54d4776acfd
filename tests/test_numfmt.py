"""Device helper round_trip_14g (csrc/tbe_numfmt.hpp) == C# double.Parse(Lua "%.14g" % x),
i.e. Python float("%.14g" % x), checked on CPU (the header is host/device code)."""
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "distributedratelimiting.redis_amd", "csrc", "tbe_numfmt.hpp")

DRIVER = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "tbe_numfmt.hpp"
int main(void) {
    uint64_t bits;
    while (fread(&bits, 8, 1, stdin) == 1) {
        double x; memcpy(&x, &bits, 8);
        double r = tbe::round_trip_14g(x);
        fwrite(&r, 8, 1, stdout);
    }
    return 0;
}
"""


def values():
    rng = np.random.default_rng(14)
    v = [0.2, 0.1, 1.0, 0.125, 1 / 3, 2 / 3, 0.3, 1e-9, 9.99999999999995e-9, 1e22, 9.99999999999995e22,
         0.19999999999999998, 0.20000000000000004, 12345.678901234567, 5e-5, 123456789012345.6,
         0.8 ** 40, 99999999999999.5, 9999999999999.95, 0.15, 0.25, 1.0000000000000002]
    v += list(10.0 ** rng.uniform(-9, 23, 300_000))
    v += list(rng.uniform(0, 2, 200_000))
    # values near 14-digit ties: d.ddddddddddddd5 * 10^k
    mant = rng.integers(10 ** 13, 10 ** 14, 100_000)
    ex = rng.integers(-22, 9, 100_000)
    v += [float(f"{m}5e{k - 1}") for m, k in zip(mant, ex) if 1e-9 <= float(f"{m}5e{k - 1}") < 1e23]
    # one ulp either side of exact 14-digit ties (the fast path's sign-of-error decisions)
    mant = rng.integers(10 ** 13, 10 ** 14, 60_000)
    ex = rng.integers(-22, 1, 60_000)
    for m, k in zip(mant, ex):
        t = float(f"{m}5e{k - 1}")
        v += [t, np.nextafter(t, 0.0), np.nextafter(t, np.inf)]
    # EWMA periods like the sync script produces
    p = 0.0
    for dt in rng.uniform(0, 3, 20_000):
        p = p * 0.8 + dt * 0.2
        v.append(p)
    return [x for x in v if 1e-9 <= x < 1e23]


def test_round_trip_14g_matches_python(tmp_path):
    src = tmp_path / "drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.dirname(HDR),
                    "-o", str(exe), str(src)], check=True)
    xs = values()
    inp = b"".join(struct.pack("<d", x) for x in xs)
    out = subprocess.run([str(exe)], input=inp, capture_output=True, check=True).stdout
    got = struct.unpack(f"<{len(xs)}d", out)
    bad = [(x, g, float("%.14g" % x)) for x, g in zip(xs, got) if g != float("%.14g" % x)]
    assert not bad, bad[:5]
    assert len(xs) > 500_000
