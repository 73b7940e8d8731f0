// Probe: does v_mfma_f64_16x16x4_f64 equal a chain of fp64 fma in k order?
// Writes A[16x4], B[4x16], C[16x16], D[16x16] for several random trials to a binary file;
// tools/probe/mfma_f64_check.py compares D with candidate evaluation orders (exact rationals).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void probe(const double *A, const double *B, const double *C, double *D, int trials) {
    const int l = threadIdx.x;
    for (int t = 0; t < trials; t++) {
        const double *a = A + t * 64, *b = B + t * 64, *c = C + t * 256;
        // A: lane l holds A[row=l&15][k=l>>4]; B: lane l holds B[k=l>>4][col=l&15]
        double av = a[(l & 15) * 4 + (l >> 4)];
        double bv = b[(l >> 4) * 16 + (l & 15)];
        v4d acc;
        for (int r = 0; r < 4; r++) acc[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        for (int r = 0; r < 4; r++) D[t * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
    }
}

static double rnd(unsigned long long *s, int mode) {
    *s = *s * 6364136223846793005ULL + 1442695040888963407ULL;
    double u = (double)(*s >> 11) * (1.0 / 9007199254740992.0);
    if (mode == 0) return 2 * u - 1;
    // wide dynamic range with signs: exercises cancellation and rounding
    *s = *s * 6364136223846793005ULL + 1442695040888963407ULL;
    double e = (double)((*s >> 40) % 60) - 30;
    return (u - 0.5) * pow(2.0, e);
}

int main(int argc, char **argv) {
    const int trials = 400;
    size_t nA = trials * 64, nC = trials * 256;
    double *A = (double *)malloc(nA * 8), *B = (double *)malloc(nA * 8), *C = (double *)malloc(nC * 8),
           *D = (double *)malloc(nC * 8);
    unsigned long long s = 12345;
    for (int t = 0; t < trials; t++) {
        int mode = t % 2;
        for (int i = 0; i < 64; i++) { A[t * 64 + i] = rnd(&s, mode); B[t * 64 + i] = rnd(&s, mode); }
        for (int i = 0; i < 256; i++) C[t * 256 + i] = rnd(&s, mode);
    }
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, nA * 8); hipMalloc(&dB, nA * 8); hipMalloc(&dC, nC * 8); hipMalloc(&dD, nC * 8);
    hipMemcpy(dA, A, nA * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, nA * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, nC * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, trials);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
    hipMemcpy(D, dD, nC * 8, hipMemcpyDeviceToHost);
    FILE *f = fopen(argc > 1 ? argv[1] : "mfma_f64_probe.bin", "wb");
    int tr = trials;
    fwrite(&tr, 4, 1, f);
    fwrite(A, 8, nA, f); fwrite(B, 8, nA, f); fwrite(C, 8, nC, f); fwrite(D, 8, nC, f);
    fclose(f);
    printf("wrote %d trials\n", trials);
    return 0;
}
