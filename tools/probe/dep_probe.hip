// Probe: latency of dependent VALU chains on one wave alone on a CU (fp64 add / fma, fp32 add,
// a DPP max step, v_readlane -> SGPR -> VALU), cycles per link by s_memtime. Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int IT = 4096;
template <int MODE>
__global__ void chain(double *out, long long *cyc, double a0, double b0) {
    double a = a0 + threadIdx.x * 1e-9, b = b0;
    float af = (float)a, bf = (float)b;
    unsigned u = threadIdx.x;
    long long t0 = clock64();
    for (int i = 0; i < IT; i++) {
        if (MODE == 0) { a = a - b; asm volatile("" : "+v"(a)); }
        if (MODE == 1) { a = __builtin_fma(a, b, 1e-30); asm volatile("" : "+v"(a)); }
        if (MODE == 2) { af = af - bf; asm volatile("" : "+v"(af)); }
        if (MODE == 3) { u = max(u, (unsigned)__builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, true)); asm volatile("" : "+v"(u)); }
        if (MODE == 4) { int s = __builtin_amdgcn_readlane((int)u, 5); u = u + (unsigned)s; asm volatile("" : "+v"(u)); }
        if (MODE == 5) { a = a / b; asm volatile("" : "+v"(a)); }
    }
    long long t1 = clock64();
    out[threadIdx.x] = a + af + u;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double *out; long long *cyc, h;
    hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
    const char *names[] = {"v_add_f64 (a - b)", "v_fma_f64", "v_sub_f32", "v_max_u32 dpp row_shr:1", "v_readlane -> s -> v_add_u32", "fp64 division (x / y)"};
#define RUN(M) for (int r = 0; r < 2; r++) { hipLaunchKernelGGL(chain<M>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0, 1e-20); hipDeviceSynchronize(); } \
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost); printf("%-32s %6.1f cycles per dependent link\n", names[M], (double)h / IT);
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5)
    return 0;
}
