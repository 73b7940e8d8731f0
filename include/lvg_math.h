/*
 * lvg_math.h — the elementary functions of the LVG path, written once so the
 * CPU (oracle, host code) and the GPU (HIP kernels) evaluate them bit for bit
 * identically. Only IEEE-754 basic operations (+ - * /), which are correctly
 * rounded on both sides, plus the exact helpers rint/ldexp/frexp are used; the
 * including translation unit must be compiled WITHOUT floating-point
 * contraction (-ffp-contract=off) so no multiply-add is fused.
 *
 * Where the reference uses them: exp in the detailed-balance up rate
 * (coll_rates.cpp:194, :214; coll_rates_ch3oh.cpp:531; coll_rates_h2o.cpp:545;
 * coll_rates_oh.cpp:344, :404) and log10 of the dust parameter in the
 * line-overlap table (lvg_method_functions.cpp:329). The reference links its
 * platform libm; results differ from any libm by at most ~1 ulp (the tests
 * check the bound), which is below what the reference itself pins.
 *
 * Algorithms: the classic fdlibm reductions (e_exp.c, e_log.c) with their
 * published minimax coefficients.
 */
#ifndef LVG_MATH_H
#define LVG_MATH_H

#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define LVG_HD __host__ __device__ __forceinline__
#else
#define LVG_HD static inline
#endif

/* exp(x), |error| < 1 ulp */
LVG_HD double lvg_exp(double x)
{
    const double o_threshold = 7.09782712893383973096e+02;
    const double u_threshold = -7.45133219101941108420e+02;
    const double ln2hi = 6.93147180369123816490e-01;   /* 0x3fe62e42 fee00000 */
    const double ln2lo = 1.90821492927058770002e-10;   /* 0x3dea39ef 35793c76 */
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > o_threshold) return HUGE_VAL;
    if (x < u_threshold) return 0.0;
    double kd = rint(x * invln2);
    double hi = x - kd * ln2hi;          /* exact: ln2hi has 32 trailing zero bits */
    double lo = kd * ln2lo;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return ldexp(y, (int)kd);
}

/* natural log for finite x > 0 (fdlibm e_log.c), |error| < 1 ulp */
LVG_HD double lvg_log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01;
    const double Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01;
    const double Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01;
    const double Lg7 = 1.479819860511658591e-01;
    if (x != x || x < 0.0) return 0.0 / 0.0;
    if (x == 0.0) return -HUGE_VAL;
    if (x == HUGE_VAL) return x;
    int e;
    double m = frexp(x, &e);                 /* x = m 2^e, m in [0.5, 1) */
    if (m < 0.70710678118654752440) { m = m * 2.0; e = e - 1; }
    double f = m - 1.0;                      /* exact (Sterbenz) */
    double k = (double)e;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + k * ln2_lo)) - f);
}

/* log10(x) = log(x) / ln(10), a few ulp */
LVG_HD double lvg_log10(double x)
{
    const double ivln10 = 4.34294481903251816668e-01;
    return lvg_log(x) * ivln10;
}

#endif /* LVG_MATH_H */
