// lvg_kernels_wide.hip — the 512-thread instantiation of lvg_kernels.hip for N <= 256:
// eight waves per workgroup, one workgroup per CU, block columns of 128 in the LU
// (lvg_lu256.h). Chosen for launches with at most two independent layers or one warm
// chain per CU (the per-GPU share of a strongly scaled cloud, chains): there one layer's
// latency is the step, and eight waves halve each wave's share of the updates and give
// every SIMD a second wave to cover LDS latency. Same code, same operation order, same
// results; entry points carry the suffix _wide.
#define LVG_WIDE 1
#include "lvg_kernels.hip"
