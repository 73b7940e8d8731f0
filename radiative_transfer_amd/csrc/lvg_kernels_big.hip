// lvg_kernels_big.hip — the second instantiation of lvg_kernels.hip for 256 < N <= 768
// (the reference's CH3OH level count, radiative_transfer.cpp:647, :773): 768 threads per
// workgroup, one panel row per thread, one workgroup per CU with the whole LDS
// (P[768][17] panel buffer), line terms in the slot workspace. Same code, same
// operation order, same results; entry points carry the suffix _big.
#define LVG_BIG 1
#include "lvg_kernels.hip"
