// Throughput probe on one CU: v_mfma_f64_16x16x4_f64 vs v_fma_f64, alone and co-issued.
// mode 0: all 8 waves MFMA; mode 1: all 8 waves VALU fma; mode 2: waves 0-3 MFMA, 4-7 VALU.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int ITERS = 2048;

__global__ void __launch_bounds__(512) rate(double *out, long long *cyc, int mode) {
    const int w = threadIdx.x >> 6;
    const bool mf = (mode == 0) || (mode == 2 && w < 4);
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
    long long t0 = clock64();
    if (mf) {
        v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
        for (int i = 0; i < ITERS; i++) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
            c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4, 0, 0, 0);
            c5 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c5, 0, 0, 0);
            c6 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c6, 0, 0, 0);
            c7 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c7, 0, 0, 0);
        }
        v4d s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
        out[threadIdx.x] = s[0] + s[1] + s[2] + s[3];
    } else {
        double x[16];
        for (int j = 0; j < 16; j++) x[j] = a + j;
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int r = 0; r < 8; r++)
#pragma unroll
                for (int j = 0; j < 16; j++) x[j] = __builtin_fma(x[j], b, a);
        }
        double s = 0;
        for (int j = 0; j < 16; j++) s += x[j];
        out[threadIdx.x] = s;
    }
    long long t1 = clock64();
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

int main() {
    double *out; long long *cyc;
    hipMalloc(&out, 512 * 8); hipMalloc(&cyc, 8 * 8);
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(rate, dim3(1), dim3(512), 0, 0, out, cyc, mode);
            hipDeviceSynchronize();
        }
        long long c[8];
        hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
        printf("mode %d cycles per wave:", mode);
        for (int w = 0; w < 8; w++) printf(" %lld", c[w]);
        printf("\n");
        // per wave: MFMA 8*ITERS instr (1024 FMA each); VALU 128*ITERS wave-fma (64 FMA each)
        for (int w = 0; w < 8; w++) {
            bool mf = mode == 0 || (mode == 2 && w < 4);
            double fma = mf ? 8.0 * ITERS * 1024 : 128.0 * ITERS * 64;
            printf("  wave %d %s: %.2f FMA/clk (SIMD holds 2 waves)\n", w, mf ? "mfma" : "valu", fma / c[w]);
        }
    }
    return 0;
}
