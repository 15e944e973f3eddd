/* Host restatement of exp_neg_tab (custom_envs_amd/csrc/optimize_kernels.h)
 * over the generated table (exp2_table.h): prints the largest error in ulp
 * against expl over random arguments in [-700, 750] and near 0, and whether
 * e^0 is exactly 1.  Built and run by tests/test_exp_table.py. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "exp2_table.h"

static const double kTab[CE_EXP2_TAB_SIZE] = CE_EXP2_TAB;
static const double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10,
                    kLog2e = 1.44269504088896338700e+00;

static double exp_neg_tab(double a) {
    const double kShift = 0x1.8p52, kC = kLog2e * CE_EXP2_TAB_SIZE,
                 kH = kLn2Hi / CE_EXP2_TAB_SIZE, kL = kLn2Lo / CE_EXP2_TAB_SIZE;
    const double big = fma(a, -kC, kShift);
    const double m = big - kShift;
    const double r = fma(m, -kL, fma(m, -kH, -a));
    int64_t bits;
    memcpy(&bits, &big, 8);
    const int lo = (int)(uint32_t)bits;
    const double t = kTab[lo & (CE_EXP2_TAB_SIZE - 1)];
    double p = fma(r, 1.0 / 6.0, 0.5);
    p = fma(p, r, 1.0);
    p *= r;
    return ldexp(fma(t, p, t), lo >> 11);   /* CE_EXP2_TAB_SIZE = 2^11 */
}

int main(void) {
    double worst = 0.0;
    srand(1);
    for (long i = 0; i < 4000000; ++i) {
        double x = -700.0 + 1450.0 * ((double)rand() / RAND_MAX);
        if (i % 4 == 0) x = (((double)rand() / RAND_MAX) - 0.5) * 20;
        if (i % 4 == 1) x = (((double)rand() / RAND_MAX) - 0.5) * 1e-3;
        const long double ref = expl(-(long double)x);
        if (ref < 2.2250738585072014e-308L) continue;
        const double ulp = nextafter((double)ref, INFINITY) - (double)ref;
        const double e = (double)(fabsl((long double)exp_neg_tab(x) - ref) / ulp);
        if (e > worst) worst = e;
    }
    printf("%.4f %d\n", worst, exp_neg_tab(0.0) == 1.0);
    return 0;
}
