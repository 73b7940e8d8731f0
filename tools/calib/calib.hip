// Calibration microbenchmark (diagnostic only): s_memtime rate and dependent
// fp64 FMA / LDS round-trip / DPP latencies on one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_fma(double *out, unsigned long long *t, int n) {
    double a = out[threadIdx.x], b = 1.0000001, c = 1e-9;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) a = fma(a, b, c);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = r1 - r0; }
}
__global__ void k_lds(double *out, unsigned long long *t, int n) {
    __shared__ double s[64];
    s[threadIdx.x] = out[threadIdx.x];
    __syncthreads();
    int idx = threadIdx.x;
    double a = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        a += s[idx];
        idx = ((int)a & 0) + ((idx + 1) & 63);   // dependent address
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) t[2] = t1 - t0;
}
__global__ void k_bar(double *out, unsigned long long *t, int n) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) t[3] = t1 - t0;
}
__global__ void k_glob(double *buf, unsigned long long *t, int n) {
    // dependent global loads (pointer chase within 1 MB)
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    long long idx = threadIdx.x;
    double a = 0;
    for (int i = 0; i < n; i++) {
        double v = buf[idx];
        a += v;
        idx = (idx + 4099 + (long long)(v * 0)) & ((1 << 17) - 1);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    buf[threadIdx.x] += a * 0;
    if (threadIdx.x == 0) t[4] = t1 - t0;
}
int main() {
    double *d; unsigned long long *t;
    hipMalloc(&d, (1 << 17) * sizeof(double));
    hipMemset(d, 0, (1 << 17) * sizeof(double));
    hipMalloc(&t, 8 * sizeof(unsigned long long));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int n = 100000;
    hipLaunchKernelGGL(k_fma, 1, 64, 0, 0, d, t, 10); hipDeviceSynchronize();
    hipEventRecord(e0); hipLaunchKernelGGL(k_fma, 1, 64, 0, 0, d, t, n); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[8]; hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost);
    double fmas = 16.0 * n;
    printf("fma chain: %.0f dep fmas, event %.3f ms, memtime %llu, realtime %llu (100MHz?)\n", fmas, ms, h[0], h[1]);
    printf("  memtime rate = %.3f GHz (vs event), realtime rate = %.3f MHz\n", h[0] / (ms * 1e6), h[1] / (ms * 1e3));
    printf("  memtime ticks per dependent fma = %.2f; ns per fma = %.3f\n", h[0] / fmas, ms * 1e6 / fmas);
    hipLaunchKernelGGL(k_lds, 1, 64, 0, 0, d, t, n); hipLaunchKernelGGL(k_bar, 1, 256, 0, 0, d, t, n);
    hipLaunchKernelGGL(k_glob, 1, 64, 0, 0, d, t, 20000); hipDeviceSynchronize();
    hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost);
    double tick_ns = ms * 1e6 / h[0];
    printf("lds dependent load+add: %.1f ticks (%.1f ns)\n", (double)h[2] / n, h[2] * tick_ns / n);
    printf("barrier (4 waves): %.1f ticks (%.1f ns)\n", (double)h[3] / n, h[3] * tick_ns / n);
    printf("global dependent load (1 MB, idle GPU): %.1f ticks (%.1f ns)\n", (double)h[4] / 20000, h[4] * tick_ns / 20000);
    return 0;
}
