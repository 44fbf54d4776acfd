// tbe_numfmt.hpp -- exact emulation of the approximate limiter's reply round trip
//     Lua  tostring(new_p)            "%.14g"  (A:270, LUA_NUMBER_FMT)
//     C#   (double)RedisValue          double.Parse (A:442)
// i.e. round a double to 14 significant decimal digits (ties to even on the exact
// binary value, as glibc printf does) and read the decimal back correctly rounded.
// Host/device header without HIP includes, so tests/test_numfmt.py compiles it with g++
// and checks it against Python's "%.14g" / float() on millions of values.
//
// Exact domain: 1e-9 <= x < 1e23 (the EWMA of seconds between syncs lives far inside
// it), x == 0, and non-finite x.  Outside, the result is the nearest-double
// approximation `x` itself (documented in DESIGN.md §2c as unpinned).
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TBE_HD __host__ __device__
#else
#define TBE_HD
#endif

namespace tbe {

typedef unsigned __int128 u128;

TBE_HD inline u128 pow10_u128(int k) {
    u128 r = 1;
    for (int i = 0; i < k; ++i) r *= 10;
    return r;
}

TBE_HD inline double pow10_exact(int k) {  // 10^k for 0 <= k <= 22 is exact in binary64
    double r = 1.0;
    for (int i = 0; i < k; ++i) r *= 10.0;
    return r;
}

// round-half-even of num / den (den > 0, 2*den < 2^128)
TBE_HD inline u128 div_round_even(u128 num, u128 den) {
    const u128 q = num / den;
    const u128 rem = num - q * den;
    const u128 twice = rem * 2;
    if (twice > den || (twice == den && (q & 1))) return q + 1;
    return q;
}

// a * 10^s = num / den exactly, with a = m * 2^e (see round_trip_14g for the bit budget)
TBE_HD inline void scaled_fraction(uint64_t m, int e, int s, u128 &num, u128 &den) {
    num = m;
    den = 1;
    if (s >= 0) num *= pow10_u128(s); else den *= pow10_u128(-s);
    if (e >= 0) num <<= e; else den <<= -e;
}

// x rounded to 14 significant digits and parsed back (see file header).
// Bit budget on the exact domain 1e-9 <= |x| < 1e23, a = m*2^e, s = 13 - E:
//   E >= -9  -> s <= 22: num <= 2^53 * 10^22 < 2^127; e >= -83: den <= 2^83
//   E <= 22  -> -s <= 9: den <= 10^9 * 2^6; e <= 24: num <= 2^77
// Fast path for 1e-9 <= a < 1e14 (every realistic EWMA period): there s = 13 - E lies in
// [0, 22], so 10^s is an exact double P, and y = fl(a*P) with err = fma(a, P, -y) is the
// exact product y + err (the rounding error of a product is representable).  On
// [1e13, 1e14] y is a multiple of its ulp (2^-9 .. 2^-6) and |err| <= ulp/2, so
//   d = (y - floor(y)) - 0.5  (exact)  and  sign(d + err) = d != 0 ? sign(d) : sign(err)
// decide the half-even rounding of the exact value without any 128-bit division.  Same
// result as the exact path (tests/test_numfmt.py checks both against "%.14g" + float()).
TBE_HD inline bool round_trip_14g_fast(double a, int be, double &out) {
    const double kP[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    int E = (int)((double)(be - 1023) * 0.30102999566398120) - ((be - 1023) < 0 ? 1 : 0);
    E = E < -9 ? -9 : (E > 13 ? 13 : E);
    double y = 0.0, err = 0.0;
    for (int it = 0; it < 4; ++it) {
        const double P = kP[13 - E];
        y = a * P;
        err = __builtin_fma(a, P, -y);
        const bool below = y < 1e13 || (y == 1e13 && err < 0);    // exact product < 10^13
        const bool above = y > 1e14 || (y == 1e14 && err >= 0);   // exact product >= 10^14
        if (below && E > -9) { --E; continue; }
        if (above && E < 13) { ++E; continue; }
        if (below || above) return false;
        break;
    }
    const double fl = __builtin_floor(y);
    const double d = (y - fl) - 0.5;
    bool up;
    if (d != 0.0) up = d > 0.0;
    else if (err != 0.0) up = err > 0.0;
    else up = __builtin_fmod(fl, 2.0) != 0.0;                     // exact tie: to even
    const double dm = up ? fl + 1.0 : fl;                          // <= 10^14 < 2^53, exact
    const int k = E - 13;                                          // -22 <= k <= 0
    out = (k == 0) ? dm : dm / kP[-k];                             // one rounding
    return true;
}

TBE_HD inline double round_trip_14g(double x) {
    if (!(x == x) || x == 0.0) return x;                     // NaN, +-0
    const bool neg = x < 0;
    const double a = neg ? -x : x;
    if (!(a >= 1e-9 && a < 1e23)) return x;                  // inf / outside the exact domain
    uint64_t bits;
    memcpy(&bits, &a, sizeof bits);
    const int be = (int)((bits >> 52) & 0x7FF);
    if (a < 1e14) {
        double r;
        if (round_trip_14g_fast(a, be, r)) return neg ? -r : r;
    }
    const uint64_t m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    const int e = be - 1075;                                  // a = m * 2^e
    // E = floor(log10(a)): estimate from the binary exponent, fix with exact compares.
    // On the domain E is in [-9, 22]; clamping keeps every probe inside the bit budget.
    int E = (int)((double)(be - 1023) * 0.30102999566398120) - ((be - 1023) < 0 ? 1 : 0);
    E = E < -9 ? -9 : (E > 22 ? 22 : E);
    u128 num, den;
    for (int it = 0; it < 4; ++it) {
        scaled_fraction(m, e, 13 - E, num, den);              // a * 10^(13-E)
        const u128 fl = num / den;
        if (fl < (u128)10000000000000ull && E > -9) { --E; continue; }     // a < 10^E
        if (fl >= (u128)100000000000000ull && E < 22) { ++E; continue; }   // a >= 10^(E+1)
        break;
    }
    scaled_fraction(m, e, 13 - E, num, den);
    const u128 M = div_round_even(num, den);                 // 14 digits (or 10^14)
    const double dm = (double)(uint64_t)M;                    // exact: M <= 10^14 < 2^53
    const int k = E - 13;                                     // -22 <= k <= 9
    const double r = (k >= 0) ? dm * pow10_exact(k) : dm / pow10_exact(-k);   // one rounding
    return neg ? -r : r;
}

}  // namespace tbe
