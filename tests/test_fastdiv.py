"""The engine replaces `usec / 1e6` (TB:203) by a reciprocal multiply with one FMA
correction and splits ts into (sec, usec) via an f64 estimate plus one integer
correction (csrc/tbe_device.hpp new_t_fast / split_ts).  Both are checked here
EXHAUSTIVELY for the usec domain [0, 1e6) with the same IEEE operations (C fma() is the
correctly rounded fused multiply-add, as gfx950's v_fma_f64), so the device result is
the IEEE quotient bit for bit."""
import subprocess

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
