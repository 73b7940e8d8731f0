// lvg_sched.hip — layer scheduling order for the persistent solve kernel.
//
// The kernel's work queue hands out layers in this order. Layers are independent and
// computed identically in any order, so the order only affects load balance: the
// number of iterations per layer has a long tail (CH3OH-A 4096 layers: 2..20, mean
// 3.6), and an expensive layer picked up last stretches the launch. The LVG column
// density per velocity N_mol/|dv/dz| sets the line optical depths and predicts the
// iteration count well (Spearman 0.69 on synth_v1); layers go in decreasing order of
// it (longest-processing-time first).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

namespace {
__global__ void sched_keys(const double *__restrict__ soa, int ld, int n, double *__restrict__ keys,
                           int *__restrict__ idx) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    keys[l] = soa[7 * (int64_t)ld + l] / fabs(soa[9 * (int64_t)ld + l]);   // mol_conc / |vel_grad|
    idx[l] = l;
}
__global__ void row_keys(const double *__restrict__ soa, int ld, int n, int row, double *__restrict__ keys,
                         int *__restrict__ idx) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    keys[l] = soa[(int64_t)row * ld + l];
    idx[l] = l;
}
}  // namespace

// Layers in decreasing order of one SoA row (row 0: gas temperature) -- the order
// coll_kernel builds collision operators in, so the layers resident on one XCD at a time
// interpolate between the same temperature rows of the tables (L2 hits). Same scratch
// contract as lvg_sched_order.
extern "C" hipError_t lvg_row_order(const double *soa, int ld, int n, int row, double *keys, double *keys_sorted,
                                    int *idx, int *order, void *temp, size_t *temp_bytes, hipStream_t s) {
    if (!temp)
        return hipcub::DeviceRadixSort::SortPairsDescending(nullptr, *temp_bytes, keys, keys_sorted, idx, order, n, 0,
                                                            64, s);
    hipLaunchKernelGGL(row_keys, dim3((n + 255) / 256), dim3(256), 0, s, soa, ld, n, row, keys, idx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, *temp_bytes, keys, keys_sorted, idx, order, n, 0, 64, s);
}

// temp == nullptr: *temp_bytes receives the scratch size needed for n layers.
extern "C" hipError_t lvg_sched_order(const double *soa, int ld, int n, double *keys, double *keys_sorted, int *idx,
                                      int *order, void *temp, size_t *temp_bytes, hipStream_t s) {
    if (!temp)
        return hipcub::DeviceRadixSort::SortPairsDescending(nullptr, *temp_bytes, keys, keys_sorted, idx, order, n, 0,
                                                            64, s);
    hipLaunchKernelGGL(sched_keys, dim3((n + 255) / 256), dim3(256), 0, s, soa, ld, n, keys, idx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, *temp_bytes, keys, keys_sorted, idx, order, n, 0, 64, s);
}
