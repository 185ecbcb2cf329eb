/* Empirical check of the reciprocal-based division used on the device
   (rt_device.h div_rcp): q0 = x*r, two FMA-residual corrections with
   r = RN(1/y) must equal RN(x/y) whenever both exponents are in the guarded
   range.  Build: gcc -O2 -march=native -ffp-contract=off tools/fastdiv_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint64_t s = 0x243F6A8885A308D3ull;
static uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double bits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static uint64_t ubits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }
static int ok_exp(double v) { uint32_t e = (uint32_t)(ubits(v) >> 52) & 0x7ff; return e - 573u < 901u; /* |v| in [2^-450, 2^451): quotient and residuals stay normal */ }
static double div_rcp(double x, double y, double r) {
    double q0 = x * r;
    double e0 = fma(-q0, y, x);
    double q1 = fma(e0, r, q0);
    double e1 = fma(-q1, y, x);
    return fma(e1, r, q1);
}
int main(void) {
    long bad = 0, n = 0;
    for (long i = 0; i < 200000000L; ++i) {
        uint64_t mx = nxt() & 0xFFFFFFFFFFFFFull, my = nxt() & 0xFFFFFFFFFFFFFull;
        int mode = (int)(nxt() % 8);
        if (mode == 1) my = 0xFFFFFFFFFFFFFull - (nxt() % 64);           /* y mantissa near all ones */
        if (mode == 2) my = nxt() % 64;                                   /* y near a power of two */
        if (mode == 3) mx = 0xFFFFFFFFFFFFFull - (nxt() % 64);
        uint64_t ex = 1023 + (int)(nxt() % 1200) - 600, ey = 1023 + (int)(nxt() % 1200) - 600;
        double x = bits((ex << 52) | mx), y = bits((ey << 52) | my);
        if (nxt() & 1) x = -x;
        if (nxt() & 1) y = -y;
        if (mode == 4) { double k = (double)(nxt() % 1000000) + 1; x = y * k; x = bits(ubits(x) + (nxt() % 5) - 2); }
        if (mode == 5) { x = y * bits(ubits(1.0) + (nxt() % 9) - 4); }
        if (!ok_exp(x) || !ok_exp(y)) continue;
        double r = 1.0 / y;
        double a = div_rcp(x, y, r), b = x / y;
        ++n;
        if (ubits(a) != ubits(b)) { if (bad < 10) printf("MISMATCH x=%a y=%a fast=%a true=%a\n", x, y, a, b); ++bad; }
    }
    printf("checked %ld, mismatches %ld\n", n, bad);
    return bad != 0;
}
