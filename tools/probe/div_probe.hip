// Probe (diagnostic, not product): the fp64 division with the denominator-only part (v_rcp_f64
// and its two Newton steps) computed once per denominator and shared, against the compiler's
// own a / b sequence (v_div_scale, v_rcp, 2 x Newton, v_div_scale, mul, fma, v_div_fmas,
// v_div_fixup), bit for bit. The shared part assumes v_div_scale leaves the denominator
// unscaled; each quotient checks that (div_scale(num, den, false) == den bitwise) and falls
// back to a / b otherwise. usage: ./div_probe  -> mismatches per input class
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>

struct DivDen { double den, r; };
__device__ __forceinline__ DivDen div_prep(double den) {
    double r = __builtin_amdgcn_rcp(den);
    double e = fma(-den, r, 1.0);
    r = fma(r, e, r);
    e = fma(-den, r, 1.0);
    r = fma(r, e, r);
    return DivDen{den, r};
}
__device__ __forceinline__ double div_shared(double num, const DivDen &D) {
    bool f0, vcc;
    const double d0 = __builtin_amdgcn_div_scale(num, D.den, false, &f0);
    if (__double_as_longlong(d0) == __double_as_longlong(D.den)) {
        const double s1 = __builtin_amdgcn_div_scale(num, D.den, true, &vcc);
        const double m = s1 * D.r;
        const double f = fma(-D.den, m, s1);
        const double q = __builtin_amdgcn_div_fmas(f, D.r, m, vcc);
        return __builtin_amdgcn_div_fixup(q, D.den, num);
    }
    return num / D.den;
}

__global__ void kcheck(const double *a, const double *b, unsigned long long *bad, int n, double *first) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b[i];
    const double q0 = x / y;
    const double q1 = div_shared(x, div_prep(y));
    if (__double_as_longlong(q0) != __double_as_longlong(q1)) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k == 0) { first[0] = x; first[1] = y; first[2] = q0; first[3] = q1; }
    }
}

static uint64_t rs = 88172645463325252ull;
static uint64_t xr() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

int main() {
    const int n = 1 << 24;
    double *ha = (double *)malloc(n * 8), *hb = (double *)malloc(n * 8);
    double *da, *db, *dfirst; unsigned long long *dbad;
    hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dbad, 8); hipMalloc(&dfirst, 32);
    const char *names[] = {"random bit patterns", "exponents within 2^+-64", "near-equal", "denormal / huge mix",
                           "populations-like 1e-40..1e2"};
    int total_bad = 0;
    for (int cls = 0; cls < 5; cls++) {
        for (int i = 0; i < n; i++) {
            uint64_t u = xr(), v = xr();
            double x, y;
            if (cls == 0) { x = bits(u); y = bits(v); }
            else if (cls == 1) { x = ldexp((double)(u >> 11) / 9007199254740992.0 + 0.5, (int)(u % 129) - 64) * ((v & 1) ? -1 : 1);
                                 y = ldexp((double)(v >> 11) / 9007199254740992.0 + 0.5, (int)(v % 129) - 64); }
            else if (cls == 2) { y = ldexp((double)(v >> 11) / 9007199254740992.0 + 0.5, (int)(v % 41) - 20);
                                 x = y * (1. + ((double)(u >> 11) / 9007199254740992.0 - 0.5) * 1e-12); }
            else if (cls == 3) { x = bits((u & 0x800fffffffffffffull) | ((u >> 52 & 1) ? 0x7fe0000000000000ull : 0ull));
                                 y = bits((v & 0x800fffffffffffffull) | ((v >> 52 & 1) ? 0x0010000000000000ull : 0x7fd0000000000000ull)); }
            else { x = pow(10., -40. + 42. * ((double)(u >> 11) / 9007199254740992.0)) * ((u & 1) ? -1 : 1);
                   y = pow(10., -40. + 42. * ((double)(v >> 11) / 9007199254740992.0)); }
            ha[i] = x; hb[i] = y;
        }
        hipMemcpy(da, ha, n * 8, hipMemcpyHostToDevice);
        hipMemcpy(db, hb, n * 8, hipMemcpyHostToDevice);
        hipMemset(dbad, 0, 8);
        kcheck<<<n / 256, 256>>>(da, db, dbad, n, dfirst);
        unsigned long long bad = 0; double first[4] = {0, 0, 0, 0};
        hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(first, dfirst, 32, hipMemcpyDeviceToHost);
        printf("%-30s %d pairs, mismatches %llu", names[cls], n, bad);
        if (bad) printf("  first: %a / %a -> %a vs %a", first[0], first[1], first[2], first[3]);
        printf("\n");
        total_bad += bad != 0;
    }
    // specials
    const double sp[] = {0., -0., INFINITY, -INFINITY, NAN, 1., -1., 4.9e-324, 2.2250738585072014e-308, 1.7976931348623157e308};
    const int ns = sizeof(sp) / 8;
    int m = 0;
    for (int i = 0; i < ns; i++) for (int j = 0; j < ns; j++) { ha[m] = sp[i]; hb[m] = sp[j]; m++; }
    hipMemcpy(da, ha, m * 8, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, m * 8, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 8);
    kcheck<<<1, 256>>>(da, db, dbad, m, dfirst);
    unsigned long long bad = 0;
    hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost);
    hipDeviceSynchronize();
    printf("%-30s %d pairs, mismatches %llu\n", "specials (0, inf, nan, denormal)", m, bad);
    total_bad += bad != 0;
    printf(total_bad ? "DIFFER\n" : "IDENTICAL\n");
    return 0;
}
