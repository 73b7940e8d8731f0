// Latency probe: dependent v_mfma_f64_16x16x4_f64 chains (1, 2, 4, 8 accumulators), one wave,
// then the cost of reading a result (v_mov of the accumulator) right after the chain.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int IT = 256;

template <int NA>
__global__ void chain(double *out, long long *cyc) {
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
    v4d c[NA];
    for (int j = 0; j < NA; j++) c[j] = v4d{0, 0, 0, 0};
    long long t0 = clock64();
    for (int i = 0; i < IT; i++)
#pragma unroll
        for (int j = 0; j < NA; j++) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
    double s = 0;
    for (int j = 0; j < NA; j++) s += c[j][0];     // forces completion
    long long t1 = clock64();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// issue cost seen by the wave: NA independent MFMAs then an unrelated VALU chain
__global__ void issue8(double *out, long long *cyc) {
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
    v4d c[8];
    for (int j = 0; j < 8; j++) c[j] = v4d{0, 0, 0, 0};
    long long t0 = clock64();
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
    long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; j++) s += c[j][0];
    long long t2 = clock64();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
}

int main() {
    double *out; long long *cyc, h[2];
    hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 16);
#define RUN(NA) for (int r = 0; r < 2; r++) { hipLaunchKernelGGL(chain<NA>, dim3(1), dim3(64), 0, 0, out, cyc); hipDeviceSynchronize(); } \
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost); printf("chains %d: %.1f cycles per MFMA\n", NA, (double)h[0] / (IT * NA));
    RUN(1) RUN(2) RUN(4) RUN(8)
    for (int r = 0; r < 2; r++) { hipLaunchKernelGGL(issue8, dim3(1), dim3(64), 0, 0, out, cyc); hipDeviceSynchronize(); }
    hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
    printf("8 independent MFMAs: issue %lld cycles, drain %lld cycles\n", h[0], h[1]);
    return 0;
}
