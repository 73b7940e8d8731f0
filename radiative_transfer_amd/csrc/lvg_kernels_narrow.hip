// lvg_kernels_narrow.hip — the one-wave instantiation of lvg_kernels.hip for N <= 256:
// 64 threads per workgroup, eight workgroups (one wave each) per CU, each wave a layer of
// its own. Chosen for launches with many independent layers (at least eight per CU): the
// layer's whole pipeline runs on one wave with no barrier to any other, its LU the
// chunk-pipelined one of lvg_lu3.h with every chunk owned by the one wave, so a CU works on
// eight layers at once and every SIMD switches between two of them. Same code, same
// operation order, same results; entry points carry the suffix _narrow.
#define LVG_NARROW 1
#include "lvg_kernels.hip"
