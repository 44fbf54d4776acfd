"""The engine replaces `usec / 1e6` (TB:203) by a reciprocal multiply with one FMA
correction and splits ts into (sec, usec) via an f64 estimate plus one integer
correction (csrc/tbe_device.hpp new_t_fast / split_ts).  Both are checked here
EXHAUSTIVELY for the usec domain [0, 1e6) with the same IEEE operations (C fma() is the
correctly rounded fused multiply-add, as gfx950's v_fma_f64), so the device result is
the IEEE quotient bit for bit."""
import subprocess

import numpy as np

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
int main(void) {
    const double d = 1000000.0, rcp = 1.0 / 1000000.0;
    long bad = 0;
    for (int64_t u = 0; u < 1000000; ++u) {
        double x = (double)u, q0 = x * rcp, r = fma(-q0, d, x), q = fma(r, rcp, q0);
        if (q != x / d) ++bad;
    }
    long bad2 = 0;
    for (int64_t k = 0; k < 5000000; ++k) {
        int64_t ts = (k % 3 == 0) ? k * 1000003LL : 1760000000000000LL + k * 7919LL + (k % 13) * 1000003LL;
        int64_t sec = (int64_t)((double)ts * 1e-6), rem = ts - sec * 1000000;
        if (rem < 0) { sec -= 1; rem += 1000000; } else if (rem >= 1000000) { sec += 1; rem -= 1000000; }
        if (sec != ts / 1000000 || rem != ts % 1000000) ++bad2;
    }
    printf("%ld %ld\n", bad, bad2);
    return 0;
}
"""


def test_fast_division_is_exact(tmp_path):
    c = tmp_path / "fd.c"
    c.write_text(SRC)
    exe = tmp_path / "fd"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["0", "0"]


def test_relative_time_split_matches_direct():
    """req_time_rel (csrc/tbe_device.hpp): (sec, usec) and the millisecond expiry bound of a
    timestamp ts = tbase + d, formed from tbase's own split plus 32-bit arithmetic on d,
    equal the direct split of ts, so new_t and exp_lt are those of req_time."""
    rng = np.random.default_rng(7)
    k_rel_max = 0xFFFFFFFF - 1_000_000
    ttl_ms = 31_536_000_000
    for tbase in [0, 999_999, 1_000_000, 1_760_000_000_000_000 - (1 << 31), 123_456_789_012_345]:
        sec0, usec0, r0 = tbase // 1_000_000, tbase % 1_000_000, tbase % 1000
        e0 = (tbase // 1000 - ttl_ms) * 1000
        ds = np.concatenate([rng.integers(0, k_rel_max + 1, 20000, dtype=np.int64),
                             np.array([0, 1, 999_999, 1_000_000, k_rel_max], dtype=np.int64)])
        for d in ds.tolist():
            ts = tbase + d
            u = (usec0 + d) & 0xFFFFFFFF
            assert u == usec0 + d                       # no u32 wrap inside the window
            assert (sec0 + u // 1_000_000, u % 1_000_000) == (ts // 1_000_000, ts % 1_000_000)
            assert e0 + ((r0 + d) // 1000) * 1000 == (ts // 1000 - ttl_ms) * 1000
