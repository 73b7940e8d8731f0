// Probe: does a 16-byte LDS-DMA (global_load_lds_dwordx4) from an 8-byte aligned global address
// deliver the right 16 bytes? (The LU stages L rows of odd-N matrices, whose row segments are
// only 8-byte aligned.) Prints the number of mismatching doubles; exit status 0 when none.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k(const double *g, double *out, int stride) {
    __shared__ double buf[128];
    const int l = threadIdx.x;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(g + 1 + (size_t)stride * l),
                                     (__attribute__((address_space(3))) void *)buf, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    out[2 * l] = buf[2 * l];
    out[2 * l + 1] = buf[2 * l + 1];
}

int main() {
    const int stride = 257;   // odd row length, as an odd-N matrix
    std::vector<double> h(64 * stride + 8);
    for (size_t i = 0; i < h.size(); i++) h[i] = 1.0 + i;
    double *dg, *dout;
    if (hipMalloc(&dg, h.size() * 8) != hipSuccess || hipMalloc(&dout, 128 * 8) != hipSuccess) return 2;
    hipMemcpy(dg, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout, stride);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
    std::vector<double> o(128);
    hipMemcpy(o.data(), dout, 128 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 2; j++)
            if (o[2 * l + j] != h[1 + (size_t)stride * l + j]) bad++;
    printf("glds16 from 8-byte aligned addresses: %d of 128 doubles wrong\n", bad);
    return bad ? 1 : 0;
}
