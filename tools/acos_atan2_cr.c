/* tools/acos_atan2_cr.c -- how often glibc's acos / atan2 (the reference's libm, restated in csrc/glibc_trig.h) differ
 * from the correctly rounded values, measured with MPFR at 200 bits over uniform unit vectors (the acos(-y),
 * atan2(-z, x) arguments of get_sphere_uv, sphere.h:24-37).  This is why the device restates glibc's code instead of
 * computing correctly rounded values: DESIGN.md §3.  The image ships libmpfr.so.6 without its header, so the few entry
 * points used are declared here (MPFR 4 ABI: mpfr_t = {long prec; int sign; long exp; void* limbs}).
 *   gcc -O2 tools/acos_atan2_cr.c -o /tmp/acos_atan2_cr -lm -l:libmpfr.so.6 && /tmp/acos_atan2_cr 1000000 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { long prec; int sign; long exp; void* d; } mpfr_struct;
typedef mpfr_struct mpfr_t[1];
enum { MPFR_RNDN = 0 };
void mpfr_init2(mpfr_t x, long prec);
void mpfr_clear(mpfr_t x);
int mpfr_set_d(mpfr_t rop, double op, int rnd);
double mpfr_get_d(const mpfr_t op, int rnd);
int mpfr_acos(mpfr_t rop, const mpfr_t op, int rnd);
int mpfr_atan2(mpfr_t rop, const mpfr_t y, const mpfr_t x, int rnd);

static uint64_t sm(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t* s) { return (double)(sm(s) >> 11) * 0x1p-53; }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    mpfr_t a, b, r;
    mpfr_init2(a, 200);
    mpfr_init2(b, 200);
    mpfr_init2(r, 200);
    uint64_t s = 12345;
    long acos_bad = 0, atan2_bad = 0;
    for (long k = 0; k < n; ++k) {
        const double zc = 2.0 * u01(&s) - 1.0, ang = 2.0 * 3.1415926535897932385 * u01(&s), rr = sqrt(fmax(0.0, 1.0 - zc * zc));
        const double x = rr * cos(ang), y = zc, z = rr * sin(ang);
        mpfr_set_d(a, -y, MPFR_RNDN);
        mpfr_acos(r, a, MPFR_RNDN);
        const double ca = mpfr_get_d(r, MPFR_RNDN), ga = acos(-y);
        acos_bad += memcmp(&ca, &ga, 8) != 0;
        mpfr_set_d(a, -z, MPFR_RNDN);
        mpfr_set_d(b, x, MPFR_RNDN);
        mpfr_atan2(r, a, b, MPFR_RNDN);
        const double ct = mpfr_get_d(r, MPFR_RNDN), gt = atan2(-z, x);
        atan2_bad += memcmp(&ct, &gt, 8) != 0;
    }
    printf("{\"unit_vectors\": %ld, \"acos_not_correctly_rounded\": %ld, \"atan2_not_correctly_rounded\": %ld, "
           "\"acos_share\": %.5f, \"atan2_share\": %.5f}\n", n, acos_bad, atan2_bad, (double)acos_bad / n, (double)atan2_bad / n);
    mpfr_clear(a);
    mpfr_clear(b);
    mpfr_clear(r);
    return 0;
}
