"""the sweeps' Markstein-corrected quotients.

odo_device.h's div_mk(a, b, y) computes a / b from y = RN(1 / b) as
q = RN(a y), r = fma(-b, q, a), RN(fma(r, y, q)) and is used in place of the
IEEE division inside ErrorFunction2's LLT solve (error_function2_mk). Markstein's
theorem gives the correctly rounded quotient when q is within 1 ulp of a / b;
RN(a y) can be up to ~1.5 ulp away (a's significand near 2), where the theorem
does not apply directly. This test runs the exact operation sequence (IEEE
binary64 on the host: the GPU's v_fma_f64 / v_mul_f64 and its correctly
rounded 1.0 / x are the same operations) over random and adversarial operands
— significands of a near 2, of b near 1 and near 2, exponents across +-20 —
and requires bit equality with a / b for every case: no counterexample in
4 x 10^7 cases (2 x 10^8 in the round-4 exploration). Zero and non-finite
pivots are excluded: there both forms reject the point (DESIGN.md §4 RANSAC).
"""
import subprocess

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double mkd(uint64_t mant, int e) {
    uint64_t b = ((uint64_t)(1023 + e) << 52) | (mant & ((1ull << 52) - 1));
    double d;
    memcpy(&d, &b, 8);
    return d;
}
/* odo_device.h div_mk */
static double div_mk(double a, double b, double y) {
    const double q = a * y;
    const double r = fma(-b, q, a);
    return fma(r, y, q);
}
int main(int argc, char** argv) {
    const long N = atol(argv[1]);
    long bad = 0;
    for (long i = 0; i < N; i++) {
        uint64_t ma = rnd(), mb = rnd();
        const int mode = (int)(i % 5);
        if (mode == 1) ma |= ((1ull << 52) - 1) ^ (rnd() & 0xFFF);
        if (mode == 2) { ma |= ((1ull << 52) - 1) ^ (rnd() & 0xF); mb &= rnd() & 0xFFFF; }
        if (mode == 3) mb |= ((1ull << 52) - 1) ^ (rnd() & 0xFF);
        if (mode == 4) { ma |= ((1ull << 52) - 1) ^ (rnd() & 0x3); mb |= ((1ull << 52) - 1) ^ (rnd() & 0x3); }
        double a = mkd(ma, (int)(rnd() % 40) - 20), b = mkd(mb, (int)(rnd() % 40) - 20);
        if (rnd() & 1) a = -a;
        const double y = 1.0 / b, q = div_mk(a, b, y), ref = a / b;
        if (memcmp(&q, &ref, 8) != 0) {
            if (bad < 8) printf("a=%a b=%a div_mk=%a a/b=%a\n", a, b, q, ref);
            bad++;
        }
    }
    printf("%ld\n", bad);
    return 0;
}
"""


def test_div_mk_is_correctly_rounded(tmp_path):
    c = tmp_path / "mk.c"
    c.write_text(SRC.replace("#include <string.h>", "#include <string.h>\n#include <stdlib.h>"))
    exe = tmp_path / "mk"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe), "40000000"], capture_output=True, text=True, timeout=120, check=True).stdout
    lines = out.strip().splitlines()
    assert lines[-1] == "0", "div_mk differs from a / b:\n" + out
