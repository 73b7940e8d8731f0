// lvg_kernels.hip — MI355X (gfx950) block kernels of the LVG level-population solver.
//
// One workgroup owns one cloud layer at a time and runs the whole reference per-layer
// pipeline on the device (radiative_transfer.cpp:236-288): layer parameters
// (iteration_lvg.cpp:59-85), collision operator (coll_rates*.cpp get_rate_*),
// boundary_layer_populations (iteration_control.cpp:52-91), the iteration_control
// fixed-point loop with Ng acceleration (iteration_control.h:84-242), and per iteration
// the rate-matrix assembly, residual and LU solve of calc_new_pop (iteration_lvg.cpp:87-161).
//
// The grid is persistent: blocks pull layers from an atomic work queue, so layers with
// very different iteration counts balance across CUs, and each block's scratch
// (collision operator K, working matrix A, Ng history) lives in a per-slot HBM workspace.
//
// fp64 throughout, no MFMA. Bit-exact with the CPU oracle by construction: this file is
// compiled with -ffp-contract=off, every operation follows the oracle's order, and the
// only fused multiply-adds are the explicit fma() of the LU, whose per-element update
// sequence (k ascending) the blocked factorization preserves.
//
// Instantiation. The product library compiles this file three times: as is (namespace
// lvg, 256 threads, N <= 256, 2 workgroups per CU), through lvg_kernels_wide.hip
// (LVG_WIDE: namespace lvg_wide, 512 threads, N <= 256, one workgroup per CU — for
// launches with at most two layers or one chain per CU, where one layer's latency is the
// step) and through lvg_kernels_big.hip (LVG_BIG: namespace lvg_big, 768 threads,
// N <= 768 — the reference's CH3OH callers, radiative_transfer.cpp:647, :773 — one
// workgroup per CU, the whole LDS). The algorithm, the operation order and hence the
// results are the same; every extern "C" entry of the other copies carries the suffix
// _wide / _big. The wave-per-layer kernel for N <= 64 is lvg_wave.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "lvg_device.h"
#include "../../include/lvg_amd.h"
#include "../../include/lvg_math.h"

#ifndef LVG_BIG
#define LVG_BIG 0
#endif
#ifndef LVG_WIDE
#define LVG_WIDE 0
#endif
#if LVG_BIG
#define LVG_NS lvg_big
#define LVG_SYM(name) name##_big
#elif LVG_WIDE
#define LVG_NS lvg_wide
#define LVG_SYM(name) name##_wide
#else
#define LVG_NS lvg
#define LVG_SYM(name) name
#endif

namespace LVG_NS {

#include "lvg_common.h"

#if defined(LVG_PHASE_TIMERS) && !LVG_BIG
// timer build of the 256-thread kernel: lane 0 of every wave accumulates (LDS atomics), so
// the phases of waves that work while wave 0 waits are counted too (sums over 4 waves)
#undef TACC
#define TACC(ph, v0) do { if ((lvg_tid() & 63) == 0) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    atomicAdd(&lvg_ph_lds[(ph) + lvg_ph_shift], t_ - (v0)); } } while (0)
#endif

constexpr int BT   = LVG_BIG ? 768 : LVG_WIDE ? 512 : 256;   // threads per workgroup
constexpr int NMAX = LVG_BIG ? 768 : 256;   // max levels of this kernel
#ifndef LVG_OCC
#define LVG_OCC (LVG_BIG || LVG_WIDE ? 1 : 2)
#endif
// the second __launch_bounds__ argument: waves per SIMD the register allocation is built for
// (amdgpu-waves-per-eu; 2 -> 256 registers a wave: two 4-wave workgroups per CU for the
// 256-thread kernel; the 512- and 768-thread kernels are bounded by their workgroup size)
constexpr int OCC  = LVG_OCC;
constexpr int LU_CW = 16;                   // N <= 256 LU: columns per chunk (lvg_lu256.h)
constexpr int NW   = BT / 64;
constexpr int NB   = 16;                    // LU panel width (chunk)
static_assert(NMAX <= BT && BT % 64 == 0 && NMAX % 32 == 0, "at least one row per thread, whole waves");
constexpr int YCAP = LVG_BIG ? 1 : 2048;    // line terms kept in LDS when 2*nb_lines <= YCAP
constexpr int TC = 4;                       // columns per thread in the LU register tile (TR rows x TC)
constexpr int TR = NMAX * 8 / BT;           // tile rows per thread: the BT/8 row groups cover NMAX
static_assert(TR * (BT / 8) >= NMAX && TR % 2 == 0, "the register tiles cover every row");
[[maybe_unused]] constexpr int WB = 8 * TC;  // LU block-column width (768-thread kernel)
#ifndef LVG_COLL_PU
#define LVG_COLL_PU 4
#endif
constexpr int COLL_PU = LVG_COLL_PU;        // 16x16 pair tiles per batch of the in-kernel collision build
#ifndef LVG_COLLP_PU
#define LVG_COLLP_PU 2     // ... and per batch of the pipelined build (two batches in flight)
#endif

constexpr int EGRID_CAP = 256;   // escape grids copied to LDS (esc_nd + esc_ng doubles)
#if LVG_BIG
struct Smem {
    double pold[NMAX], bvec[NMAX];
    union { double pnew[NMAX]; double blog[NMAX]; };   // pnew only ever copies blog
    double diag[NMAX];          // assembled diagonal of the rate matrix (fused assembly)
    double ylds[YCAP];          // line terms y of the current iteration (if they fit)
    int    tmap[NMAX];          // physical row of each tile row at the current block load
    int    perm[NMAX];          // LU row permutation: logical position -> physical row
    int    pos[NMAX];           // its inverse: physical row -> logical position
    double red[NW];
    int    ired[2 * NW];
    unsigned long long pkey[2 * NW];   // panel: per-wave pivot keys (|v| bits, active flag), double buffered
    alignas(16) double cand[2][NW][NB + 2]; // panel: each wave's pivot candidate row and its b, double buffered
    double L11[NB][NB + 1];
    alignas(16) double Ub[2][NB][WB + 2];   // U rows of one chunk across the block column (by chunk parity)
    union alignas(16) {
        double P[NMAX][NB + 1]; // panel, physical rows
        double LT[NB][NMAX];    // L of one chunk, transposed, physical rows
        double hist_acc[32];    // accel_step sums (used outside the LU only)
    } pu;
#else
struct Smem {
    double pold[NMAX], bvec[NMAX];
    union { double pnew[NMAX]; double blog[NMAX]; };   // pnew only ever copies blog
    double diag[NMAX];          // assembled diagonal of the rate matrix (fused assembly)
    double resid[NMAX];         // residual rows (physical), handed from wave to wave in column order
    double ylds[YCAP];          // line terms y of the current iteration (if they fit)
    int    perm[NMAX];          // LU row permutation: logical position -> physical row
    int    pos[NMAX];           // its inverse: physical row -> logical position
    double red[NW];
    alignas(16) double L11[NB][NB + 1];    // unit-lower diagonal block of the current chunk
    alignas(16) double Ub[NW][LU_CW][LU_CW];   // per wave: the chunk's pivot rows in its columns, then U
    int seq;                    // LU chunk sequence: 2 x chunks published (odd while one is published)
    int rdone;                  // chunks whose columns the residual has taken
    union alignas(16) {
        double L11c[NMAX / LU_CW][LU_CW][LU_CW + 1];   // unit-lower diagonal block of every chunk
        double hist_acc[32];    // accel_step sums (used outside the LU only)
    } pu;
#endif
    // the escape-probability grids (esc_delta, esc_gamma) when they fit: the bisections of
    // every line's escape probability step through LDS instead of L2 (esc_in_lds; +1.2%,
    // profiles/r5/variants.txt item 25)
    double egrid[EGRID_CAP];
    int esc_in_lds;
    // per-layer scalars
    double T, Te, vw, vgrad, nmol, ne;
    double cc[LVG_MAX_COMBOS];
    double teff[LVG_MAX_TABLES];
    int    lo[LVG_MAX_TABLES];
    const double *tcol[LVG_MAX_TABLES];   // coefficients at T index lo (T-major row)
    const double *tder[LVG_MAX_TABLES];   // their slopes over [lo, lo+1]
    int64_t timax[LVG_MAX_TABLES];        // pairs per T row
    double tdt[LVG_MAX_TABLES];           // tgrid[lo+1] - tgrid[lo]
    double tx[LVG_MAX_TABLES];            // min(T, tmax) - tgrid[lo]
    int8_t ttab[LVG_MAX_CLASSES][LVG_MAX_TERMS], tcombo[LVG_MAX_CLASSES][LVG_MAX_TERMS];
    int8_t tet[LVG_MAX_CLASSES], tgrp[LVG_MAX_CLASSES];
    double dust[LVG_MAX_DUST];
    int    layer, pidx;
};

// OCC workgroups per CU must fit the CU's LDS (gfx950: 160 KB; the layout above, the L11 of
// every chunk in particular, is sized for it): a smaller-LDS target fails here instead of
// silently running fewer workgroups per CU
constexpr size_t LDS_PER_CU = 160 * 1024;
static_assert(sizeof(Smem) * OCC <= LDS_PER_CU, "Smem x workgroups per CU exceeds the CU's LDS");

__device__ __forceinline__ double block_max(double v, Smem &sm) {
    const int t = lvg_tid(), w = t >> 6;
    v = wave_max(v);
    __syncthreads();
    if ((t & 63) == 0) sm.red[w] = v;
    __syncthreads();
    double r = sm.red[0];
#pragma unroll
    for (int i = 1; i < NW; i++) r = fmax(r, sm.red[i]);
    return r;
}

__device__ __forceinline__ void layer_setup(const LvgDevProblem &P, const LvgLaunch &Lc, int l, Smem &sm) {
    if (lvg_tid() == 0) layer_scalars<Smem, true>(P, Lc, l, sm);
    __syncthreads();
}

// the layer's collision operator K (and the boundary matrix B) in the slot, pair classes
// staged in the panel buffer, which is free between factorizations, when they fit
__device__ __forceinline__ void layer_collisions(const LvgDevProblem &P, Smem &sm, double *K, double *B,
                                                 bool electrons = true) {
    const int M = P.N * (P.N - 1) / 2;
    uint8_t *cls = M <= (int)sizeof(sm.pu) ? reinterpret_cast<uint8_t *>(&sm.pu) : nullptr;
    // no boundary matrix to write and at most three neutral terms per pair (CH3OH, OH, p-H2O
    // below 3 tables): the pipelined build, two batches in flight (+1.8%, profiles/r6/variants.txt
    // item 2; not in the 768-thread kernel, whose register allocation it wrecks); otherwise
    // build_collision_operators
#if !LVG_BIG
    if (!B && cls && P.terms.nt_max <= 3) {
        TSTAMP(tq0);
        {
            const int n16 = M >> 4;
            const uint4 *src4 = reinterpret_cast<const uint4 *>(P.pair_class);
            for (int e = lvg_tid(); e < n16; e += BT) reinterpret_cast<uint4 *>(cls)[e] = src4[e];
            for (int e = (n16 << 4) + lvg_tid(); e < M; e += BT) cls[e] = P.pair_class[e];
            __syncthreads();
        }
        if (electrons && P.terms.any_e) build_collision_pipe<BT, LVG_COLLP_PU, 3, true>(P, sm, K, cls, true);
        else build_collision_pipe<BT, LVG_COLLP_PU, 3, false>(P, sm, K, cls, false);
        __syncthreads();
        TACC(PH_PAIRS, tq0);
        return;
    }
#endif
    build_collision_operators<BT, COLL_PU>(P, sm, K, B, cls, electrons);
}

// Diagonal of the boundary-layer matrix B formed from K (no electron tables: B = K + A/2 above
// the diagonal, K below it; iteration_control.cpp:69-85): minus the column sum of B for r
// ascending, the operations build_collision_operators applies to B itself (and coll_kernel to
// form B_all's diagonal), into dg[N]
__device__ __forceinline__ void boundary_diagonal(const LvgDevProblem &P, const double *K, double *dg) {
    const int N = P.N;
    for (int d = lvg_tid(); d < N; d += BT) {
        double a = 0.;
        for (int r0 = 0; r0 < N; r0 += 16) {
            double kv[16], ev[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int r = r0 + u < N ? r0 + u : 0;
                kv[u] = K[(int64_t)r * N + d];
                ev[u] = P.einst_t[(int64_t)r * N + d];     // einst[d][r], coalesced over d
            }
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int r = r0 + u;
                if (r < N && r != d) {
                    const double bb = (r < d) ? 0.5 * ev[u] + kv[u] : kv[u];
                    a = a - bb;
                }
            }
        }
        dg[d] = a;
    }
    __syncthreads();
}

// the escape grids into LDS once per launch (compute_line_terms reads them from there)
__device__ __forceinline__ void load_esc_grids(const LvgDevProblem &P, Smem &sm) {
    const int nd = P.esc_nd, ng = P.esc_ng;
    const bool fit = nd + ng <= EGRID_CAP;
    if (fit)
        for (int e = lvg_tid(); e < nd + ng; e += BT) sm.egrid[e] = e < nd ? P.esc_delta[e] : P.esc_gamma[e - nd];
    if (lvg_tid() == 0) sm.esc_in_lds = fit;
    __syncthreads();
}

// y[2n] = A_ul(1+I), y[2n+1] = A_lu*I for every line of the scheme
__device__ __forceinline__ void line_terms_with(const LvgDevProblem &P, const EscGrids &G, const LvgModeLines &M,
                                                const Smem &sm, const double *pop, double *y) {
    for (int q = lvg_tid(); q < M.nb_units; q += BT) {
        int n1 = M.unit_l0[q], n2 = M.unit_l1[q];
        if (n2 < 0) {
            double I = intensity_single(P, G, M, sm, n1, pop);
            y[2 * n1] = M.line_aul[n1] * (1. + I);
            y[2 * n1 + 1] = M.line_alu[n1] * I;
        } else {
            double i1, i2;
            intensity_pair(P, G, M, sm, n1, n2, pop, i1, i2);
            y[2 * n1] = M.line_aul[n1] * (1. + i1);
            y[2 * n1 + 1] = M.line_alu[n1] * i1;
            y[2 * n2] = M.line_aul[n2] * (1. + i2);
            y[2 * n2 + 1] = M.line_alu[n2] * i2;
        }
    }
}
__device__ __forceinline__ void compute_line_terms(const LvgDevProblem &P, const LvgModeLines &M, const Smem &sm,
                                                   const double *pop, double *y) {
    EscGrids G = global_grids(P);
    if (sm.esc_in_lds) {
        G.ed = sm.egrid;
        G.eg = sm.egrid + P.esc_nd;
        line_terms_with(P, G, M, sm, pop, y);
    } else {
        line_terms_with(P, G, M, sm, pop, y);
    }
}

// Diagonal of the rate matrix (iteration_lvg.cpp:117-151): thread d folds column
// d of K in the reference's order: for partner levels r ascending, -rate(d->r)
// then, if a line joins d and r, -y (plain scheme); or all collision terms first
// and the lines after, in line order (overlap scheme). The off-diagonal entries
// are formed where the LU loads them (block_lu_solve, fused).
__device__ __forceinline__ void column_diagonals(const LvgDevProblem &P, const LvgModeLines &M,
                                                 const double *K, const double *y, Smem &sm) {
    const int N = P.N, t = lvg_tid();
    for (int d = t; d < N; d += BT) {
        double a = 0.;
        for (int r0 = 0; r0 < N; r0 += 16) {
            double kv[16];
            int lv[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const bool ok = r0 + u < N;
                kv[u] = ok ? K[(r0 + u) * N + d] : 0.;
                lv[u] = ok ? M.line_idx[(r0 + u) * N + d] : -1;
            }
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int r = r0 + u;
                if (r < N && r != d) {
                    a = a - kv[u];
                    if (M.diag_interleaved && lv[u] >= 0) a = a - y[lv[u]];
                }
            }
        }
        if (!M.diag_interleaved)
            for (int q = M.diag_ptr[d]; q < M.diag_ptr[d + 1]; q++) a = a - y[M.diag_ent[q]];
        sm.diag[d] = a;
    }
    __syncthreads();
}

// Source of the matrix the LU factors: the assembled A already in the slot
// (boundary layer), or fused: K + line terms + sm.diag, row 0 <- 1, formed while
// each block column is loaded, with the residual df = e0 - A n accumulated on the
// way (row by row in ascending column order, as iteration_lvg.cpp:153-160).
struct LuSrc {
    const double *K = nullptr, *y = nullptr;
    const int *li = nullptr;
    const double *pop = nullptr;   // LDS populations for the residual
    double *df = nullptr;          // [N] residual out
    double *dump = nullptr;        // optional [N*N] copy of the assembled matrix (debug)
    const double *B = nullptr;     // unfused: read the matrix from here, factor into A (NULL: A in place)
    // unfused, boundary matrix formed from the layer's K (no electron rates): row 0 = 1,
    // diagonal BD, above it 0.5 A_{d,r} + K_{r,d} (BE = einst), below it K_{r,d}
    const double *BK = nullptr, *BE = nullptr, *BD = nullptr;
    const double *BET = nullptr;   // einst transposed (einst_t): einst[d][r] at BET[r * N + d]
};

// ---- back substitution U x = y in logical order, blocked by NB from the bottom:
//      wave 0 solves the diagonal block in registers, then all threads update the
//      rows above; every entry receives its updates for k descending (oracle order).
//      b: LDS [N] by physical row; on return sm.blog holds x (logical = level order).
__device__ __forceinline__ void back_substitute(const double *A, int N, const double *b, Smem &sm) {
    const int t = lvg_tid();
    TSTAMP(tb0);
    for (int i = t; i < N; i += BT) sm.blog[i] = b[sm.perm[i]];
    __syncthreads();
    const int nblk = (N + NB - 1) / NB;
    // operands of block kb, loaded one block ahead so their latency hides behind the
    // diagonal solve: the 16x16 diagonal block (one entry per thread) and the U
    // segment U[perm[t]][k0..k0+nb) of this thread's row (rows above the block)
    auto load_blk = [&](int kb, double &dv, double (&u)[NB]) {
        const int k0 = kb * NB, nb = min(NB, N - k0);
        const int r = t / NB, c = t - r * NB;
        dv = (r < nb && c < nb) ? A[(int64_t)sm.perm[k0 + r] * N + k0 + c] : 0.;
        const double *row = A + (int64_t)sm.perm[t < k0 ? t : 0] * N + k0;
        if ((N & 1) == 0 && nb == NB) {
            const double2 *r2 = reinterpret_cast<const double2 *>(row);
#pragma unroll
            for (int m = 0; m < NB / 2; m++) {
                const double2 v = (t < k0) ? r2[m] : make_double2(0., 0.);
                u[2 * m] = v.x;
                u[2 * m + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int m = 0; m < NB; m++) u[m] = (t < k0 && m < nb) ? row[m] : 0.;
        }
    };
    double dcur, ucur[NB], dnxt = 0., unxt[NB];
    load_blk(nblk - 1, dcur, ucur);
    for (int kb = nblk - 1; kb >= 0; kb--) {
        const int k0 = kb * NB, nb = min(NB, N - k0);
        {
            const int r = t / NB, c = t - r * NB;
            if (r < nb && c < nb) sm.L11[r][c] = dcur;
        }
        __syncthreads();
        if (kb > 0) load_blk(kb - 1, dnxt, unxt);
        TSTAMP(td0);
        if (t < 64) {
            // diagonal block by wave 0 in registers: lane r < nb holds b_r and row r of the
            // block; x_m (lane m's b_m / U_mm once final) is broadcast by DPP row_newbcast:m
            const int r = t & 15;
            double bt = (t < nb) ? sm.blog[k0 + t] : 0., ur[NB];
#pragma unroll
            for (int m = 0; m < NB; m++) ur[m] = (t < nb) ? sm.L11[r][m] : 1.;
#define LVG_BSUB_STEP(M_)                                                                  \
            if ((M_) < nb) {                                                               \
                const double xm = dpp_d<0x150 + (M_), 0xf, 0xf>(bt / ur[M_]);              \
                if (r < (M_)) bt = fma(-ur[M_], xm, bt);                                   \
                else if (r == (M_)) bt = xm;                                               \
            }
            LVG_BSUB_STEP(15) LVG_BSUB_STEP(14) LVG_BSUB_STEP(13) LVG_BSUB_STEP(12)
            LVG_BSUB_STEP(11) LVG_BSUB_STEP(10) LVG_BSUB_STEP(9) LVG_BSUB_STEP(8)
            LVG_BSUB_STEP(7) LVG_BSUB_STEP(6) LVG_BSUB_STEP(5) LVG_BSUB_STEP(4)
            LVG_BSUB_STEP(3) LVG_BSUB_STEP(2) LVG_BSUB_STEP(1) LVG_BSUB_STEP(0)
#undef LVG_BSUB_STEP
            if (t < nb) sm.blog[k0 + t] = bt;
        }
        __syncthreads();
        TACC(PH_BS_DIAG, td0);
        TSTAMP(tu0);
        if (t < k0) {
            double s = sm.blog[t];
#pragma unroll
            for (int m = NB - 1; m >= 0; m--)
                if (m < nb) s = fma(-ucur[m], sm.blog[k0 + m], s);
            sm.blog[t] = s;
        }
        __syncthreads();
        TACC(PH_BS_UPD, tu0);
        dcur = dnxt;
#pragma unroll
        for (int m = 0; m < NB; m++) ucur[m] = unxt[m];
    }
    TACC(PH_BACKSUB, tb0);
}

#if LVG_BIG
// ------------------------------------------------------------------------------
// Left-looking blocked LU with partial pivoting, b eliminated alongside.
//
// A: N x N row-major (physical rows) in the slot workspace, read once per block
// column and overwritten in place by the factors (L below the pivots, U in the
// pivot rows), never row-swapped: pivoting is virtual (perm/pos in LDS).
// Block columns of WB = 32 columns live in registers, an 8x4 fp64 tile per thread
// (tile rows 8*rg.., cols 4*cg..; tile row r = physical row perm[r] at the block load).
// For each 16-wide chunk kk to the left (earlier block columns, then the block's own
// chunks once factored): the chunk's pivot rows are solved against L11 (TRSM -> U rows,
// stored to A), then every row below is updated with the chunk's L (staged transposed
// in LDS) and those U rows. Chunks are factored by all four waves, one row per thread
// in registers, or by one wave when every active row lies in one or two waves' tile rows.
//
// Every element receives fma(-l_ik, u_kj, a_ij) for k ascending and the pivots are
// chosen from identical values, so the result equals the unblocked, physically
// pivoting oracle (oracle_lu_solve) bit for bit. On return sm.blog holds x.
// b: LDS [N] indexed by physical row.
// ------------------------------------------------------------------------------
__device__ __forceinline__ void panel_factor(double *A, int N, int kk, int nb, double *b, Smem &sm) {
    // chunk columns kk..kk+nb-1 are in sm.pu.P[p][0..nb) for every physical row p;
    // rows with pos[p] >= kk take part. One row per thread (N <= NMAX = BT), the row's
    // right-hand side b[p] in a register; the pivot candidate of each wave publishes
    // its row and its b through LDS.
    const int t = lvg_tid(), w = t >> 6;
    double rw[NB];
    const bool valid = t < N;
    const int p = valid ? t : 0;
    const bool part = valid && sm.pos[p] >= kk;
    bool act = part;
    int lp = act ? sm.pos[p] - kk : 0x7fffffff;
    double rb = b[p];
#pragma unroll
    for (int j = 0; j < NB; j++) rw[j] = sm.pu.P[p][j];
#pragma clang loop unroll(full)
    for (int c = 0; c < NB; c++) {
        if (c < nb) {
            const int buf = c & 1;
            // argmax |v| (ties: smallest logical position) as u32 max reductions
            unsigned hi, lo;
            pivot_key(rw[c], act, lp == c, hi, lo);
            TSTAMP(tpr);
            const unsigned H = wave_max_u32(hi);
            unsigned Lw;
            int wmin;
            const unsigned long long tie = __ballot(hi == H);
            if (__popcll(tie) == 1) {
                // one lane holds the wave's maximum upper word: it is the candidate
                const int ln = __ffsll((long long)tie) - 1;
                Lw = (unsigned)__builtin_amdgcn_readlane((int)lo, ln);
                wmin = __builtin_amdgcn_readlane(lp, ln);
            } else {
                Lw = wave_max_u32(hi == H ? lo : 0u);
                const unsigned X = wave_max_u32((hi == H && lo == Lw && act) ? ~(unsigned)lp : 0u);
                wmin = (int)~X;
            }
            if ((t & 63) == 0) {
                sm.pkey[NW * buf + w] = ((unsigned long long)H << 32) | Lw;
                sm.ired[NW * buf + w] = wmin;
            }
            if (act && lp == wmin) {               // this wave's candidate publishes its row
#pragma unroll
                for (int j = 0; j < NB; j += 2)         // 16-byte stores from column c & ~1
                    if (j + 1 >= c) *reinterpret_cast<double2 *>(&sm.cand[buf][w][j]) = make_double2(rw[j], rw[j + 1]);
                sm.cand[buf][w][NB] = rb;
            }
            __syncthreads();                       // one barrier per column
            TACC(PH_P_RED, tpr);
            TSTAMP(tpp);
            // the candidates at once, winner picked without branches
            unsigned long long ok[NW];
            int oi[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) { ok[i] = sm.pkey[NW * buf + i]; oi[i] = sm.ired[NW * buf + i]; }
            unsigned long long kmax = ok[0];
            int lmin = oi[0], ww = 0;
#pragma unroll
            for (int i = 1; i < NW; i++) {
                const bool better = ok[i] > kmax || (ok[i] == kmax && (unsigned)oi[i] < (unsigned)lmin);
                kmax = better ? ok[i] : kmax;
                lmin = better ? oi[i] : lmin;
                ww = better ? i : ww;
            }
            const bool owner = act && lp == lmin;
            const double *prow0 = sm.cand[buf][ww];
            double prow[NB];
#pragma unroll
            for (int j = 0; j < NB; j += 2)             // 16-byte reads from column c & ~1
                if (j + 1 >= c) {
                    const double2 v = *reinterpret_cast<const double2 *>(prow0 + j);
                    prow[j] = v.x;
                    prow[j + 1] = v.y;
                }
            const double piv = prow[c];
            const double bc = prow0[NB];
            if (owner) { act = false; lp = c; }
            else if (lp == c) lp = lmin;
            if (act) {
                const double l = rw[c] / piv;
                rw[c] = l;
#pragma unroll
                for (int j = 0; j < NB; j++) if (j > c) rw[j] = fma(-l, prow[j], rw[j]);
                rb = fma(-l, bc, rb);
            }
            TACC(PH_P_POST, tpp);
        }
    }
    TSTAMP(tpw);
    __syncthreads();
    if (part) {
        // rows of this chunk and below: factors back to A (physical row p)
        if ((N & 1) == 0 && nb == NB) {
            double2 *d2 = reinterpret_cast<double2 *>(A + (int64_t)p * N + kk);
#pragma unroll
            for (int j = 0; j < NB / 2; j++) d2[j] = make_double2(rw[2 * j], rw[2 * j + 1]);
        } else {
#pragma unroll
            for (int j = 0; j < NB; j++) if (j < nb) A[(int64_t)p * N + kk + j] = rw[j];
        }
        sm.perm[kk + lp] = p;
        sm.pos[p] = kk + lp;
        b[p] = rb;
#pragma unroll
        for (int j = 0; j < NB; j++) sm.pu.P[p][j] = rw[j];
    }
    __syncthreads();
    TACC(PH_P_WB, tpw);
}

// One-wave panel: when every row still active in the chunk lies in one or two waves'
// tile rows (block columns c0 >= 128 at N = 256), wave w0 factors the chunk alone, R
// rows per lane in registers. Per column: a compare over the lane's rows, one DPP wave
// reduction (+ ballot) for the pivot and a v_readlane broadcast of the pivot row; no
// workgroup barrier and no LDS round trip. Same pivots (largest |v|, ties to the
// smallest logical position) and the same fma sequence as panel_factor, so the factors
// are identical. The other waves go straight to the closing barrier and leave their
// SIMDs to the co-resident workgroup.
template <int R>
__device__ __forceinline__ void panel_factor_wave(double *A, int N, int kk, int nb, double *b, Smem &sm, int w0,
                                                  const int (&rows)[R]) {
    if ((__builtin_amdgcn_readfirstlane(lvg_tid()) >> 6) == w0) {
        const int ln = lvg_tid() & 63;
        double rw[R][NB], rb[R];
        bool act[R], part[R];
        int lp[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            const int p = rows[i];
            const int pp = p >= 0 ? p : 0;
            const int ps = sm.pos[pp];
            part[i] = p >= 0 && ps >= kk;
            act[i] = part[i];
            lp[i] = part[i] ? ps - kk : 0x7fffffff;
            rb[i] = b[pp];
#pragma unroll
            for (int j = 0; j < NB; j++) rw[i][j] = sm.pu.P[pp][j];
        }
#pragma clang loop unroll(full)
        for (int c = 0; c < NB; c++) {
            if (c < nb) {
                // the lane's best row: largest key, ties to the smallest logical position
                unsigned bh = 0u, bl = 0u;
                int bp = 0x7fffffff, bs = 0;
#pragma unroll
                for (int i = 0; i < R; i++) {
                    unsigned hi, lo;
                    pivot_key(rw[i][c], act[i], lp[i] == c, hi, lo);
                    const bool better = hi > bh || (hi == bh && (lo > bl || (lo == bl && (unsigned)lp[i] < (unsigned)bp)));
                    bh = better ? hi : bh;
                    bl = better ? lo : bl;
                    bp = better ? lp[i] : bp;
                    bs = better ? i : bs;
                }
                const unsigned H = wave_max_u32(bh);
                const unsigned long long tie = __ballot(bh == H);
                int pl;
                if (__popcll(tie) == 1) {
                    pl = __ffsll((long long)tie) - 1;
                } else {
                    const unsigned Lw = wave_max_u32(bh == H ? bl : 0u);
                    const unsigned X = wave_max_u32((bh == H && bl == Lw) ? ~(unsigned)bp : 0u);
                    pl = __ffsll((long long)__ballot(bh == H && bl == Lw && bp == (int)~X)) - 1;
                }
                pl = __builtin_amdgcn_readfirstlane(pl);
                const int s = __builtin_amdgcn_readlane(bs, pl);
                const int plp = __builtin_amdgcn_readlane(bp, pl);
                double prow[NB], bc;
                auto bcast = [&](const double (&r)[NB], double rbv) {
#pragma unroll
                    for (int j = 0; j < NB; j++) if (j >= c) prow[j] = readlane_d(r[j], pl);
                    bc = readlane_d(rbv, pl);
                };
                if (R == 1 || s == 0) bcast(rw[0], rb[0]);
                else bcast(rw[R > 1 ? 1 : 0], rb[R > 1 ? 1 : 0]);
                const double piv = prow[c];
#pragma unroll
                for (int i = 0; i < R; i++) {
                    if (ln == pl && s == i) { act[i] = false; lp[i] = c; }
                    else if (lp[i] == c) lp[i] = plp;
                    if (act[i]) {
                        const double l = rw[i][c] / piv;
                        rw[i][c] = l;
#pragma unroll
                        for (int j = 0; j < NB; j++) if (j > c) rw[i][j] = fma(-l, prow[j], rw[i][j]);
                        rb[i] = fma(-l, bc, rb[i]);
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < R; i++) {
            if (part[i]) {
                const int p = rows[i];
                if ((N & 1) == 0 && nb == NB) {
                    double2 *d2 = reinterpret_cast<double2 *>(A + (int64_t)p * N + kk);
#pragma unroll
                    for (int j = 0; j < NB / 2; j++) d2[j] = make_double2(rw[i][2 * j], rw[i][2 * j + 1]);
                } else {
#pragma unroll
                    for (int j = 0; j < NB; j++) if (j < nb) A[(int64_t)p * N + kk + j] = rw[i][j];
                }
                sm.perm[kk + lp[i]] = p;
                sm.pos[p] = kk + lp[i];
                b[p] = rb[i];
#pragma unroll
                for (int j = 0; j < NB; j++) sm.pu.P[p][j] = rw[i][j];
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ double block_lu_solve(double *A, int N, double *b, Smem &sm, const LuSrc &src, const bool FUSED) {
    const int t = lvg_tid();
    const int rg = t >> 3, cg = t & 7;   // tile rows TR*rg.., columns TC*cg..
    double s_acc = (t == 0) ? 1. : 0.;             // residual row t (FUSED)
    for (int i = t; i < N; i += BT) { sm.perm[i] = i; sm.pos[i] = i; }
    __syncthreads();
    for (int c0 = 0; c0 < N; c0 += WB) {
        TSTAMP(tp0);
        const int wJ = min(WB, N - c0);
        double acc[TR][TC];
        // The block column is held in LOGICAL row order as of this load: tile row r is
        // physical row perm[r]. Rows below an earlier block's chunk kk are then the
        // contiguous tile rows >= kk + 16, so whole threads and waves drop out of the
        // updates as kk grows (virtual pivoting alone scatters them).
        int prow[TR];
#pragma unroll
        for (int i = 0; i < TR; i++) prow[i] = (TR * rg + i < N) ? sm.perm[TR * rg + i] : 0;
        const int trow = (t < N) ? sm.perm[t] : 0;   // physical row of tile row t (L staging)
        if (t < N) sm.tmap[t] = trow;
        // ---- block column c0..c0+wJ-1 into registers (physical rows, coalesced)
        if (!FUSED && src.BK) {
#pragma unroll
            for (int i = 0; i < TR; i++)
#pragma unroll
                for (int j = 0; j < TC; j++) {
                    const int col = TC * cg + j, pr = prow[i], d = c0 + col;
                    const bool ok = TR * rg + i < N && col < wJ;
                    const double k = ok ? src.BK[(int64_t)pr * N + d] : 0.;
                    const double e = (ok && pr < d) ? src.BE[(int64_t)d * N + pr] : 0.;
                    const double dg = (ok && pr == d) ? src.BD[d] : 0.;
                    double v = (pr < d) ? 0.5 * e + k : k;   // build_collision_operators: 0.5 * af + dn
                    if (pr == d) v = dg;
                    if (pr == 0) v = 1.;
                    acc[i][j] = ok ? v : 0.;
                }
        } else if (!FUSED) {
#pragma unroll
            for (int i = 0; i < TR; i++)
#pragma unroll
                for (int j = 0; j < TC; j++) {
                    const int col = TC * cg + j;
                    acc[i][j] = (TR * rg + i < N && col < wJ) ? (src.B ? src.B : A)[(int64_t)prow[i] * N + c0 + col] : 0.;
                }
        } else {
            int li[TR][TC];
            if ((N & 3) == 0 && TC * cg + TC <= wJ) {
                // whole TC-column segments, aligned: 16-byte K loads, one li load
#pragma unroll
                for (int i = 0; i < TR; i++) {
                    const bool ok = TR * rg + i < N;
                    const int64_t o = (int64_t)(ok ? prow[i] : 0) * N + c0 + TC * cg;
                    const double2 k0 = ok ? reinterpret_cast<const double2 *>(src.K + o)[0] : make_double2(0., 0.);
                    const double2 k1 = ok ? reinterpret_cast<const double2 *>(src.K + o)[1] : make_double2(0., 0.);
                    const int4 l4 = ok ? *reinterpret_cast<const int4 *>(src.li + o) : make_int4(-1, -1, -1, -1);
                    acc[i][0] = k0.x; acc[i][1] = k0.y; acc[i][2] = k1.x; acc[i][3] = k1.y;
                    li[i][0] = l4.x; li[i][1] = l4.y; li[i][2] = l4.z; li[i][3] = l4.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < TR; i++)
#pragma unroll
                    for (int j = 0; j < TC; j++) {
                        const int col = TC * cg + j;
                        const bool ok = TR * rg + i < N && col < wJ;
                        const int64_t o = (int64_t)prow[i] * N + c0 + col;
                        acc[i][j] = ok ? src.K[o] : 0.;
                        li[i][j] = ok ? src.li[o] : -1;
                    }
            }
#pragma unroll
            for (int i = 0; i < TR; i++)
#pragma unroll
                for (int j = 0; j < TC; j++) {
                    const int pr = prow[i], d = c0 + TC * cg + j;
                    double v = acc[i][j];
                    if (li[i][j] >= 0) v = v + src.y[li[i][j]];
                    if (pr == d) v = sm.diag[d < NMAX ? d : 0];
                    if (pr == 0) v = 1.;
                    acc[i][j] = v;
                    if (src.dump && TR * rg + i < N && TC * cg + j < wJ) src.dump[(int64_t)pr * N + d] = v;
                }
            // residual rows: 16 columns at a time through LDS, each thread its own row
            for (int h = 0; h < wJ; h += NB) {
                const int g = cg - h / TC;
                if (g >= 0 && g < NB / TC) {
#pragma unroll
                    for (int i = 0; i < TR; i++)
#pragma unroll
                        for (int j = 0; j < TC; j++) sm.pu.P[prow[i]][TC * g + j] = acc[i][j];
                }
                __syncthreads();
                const int nc = min(NB, wJ - h);
                if (t < N)
                    for (int c = 0; c < nc; c++) s_acc = s_acc - sm.pu.P[t][c] * src.pop[c0 + h + c];
                __syncthreads();
            }
        }
        TACC(PH_BLOAD, tp0);
        for (int kk = 0; kk < c0 + wJ; kk += NB) {
            const int nb = min(NB, N - kk);
            const int ub = (kk >> 4) & 1;              // Ub buffer of this chunk
            int jlo;                                   // first block-local column to update
            if (kk >= c0) {
                // ---- a chunk of this block column: all updates from k < kk are in; factor it
                TSTAMP(tp1);
                const int g = cg - (kk - c0) / TC;     // this thread's column group within the chunk
#pragma unroll
                for (int i = 0; i < TR; i++) {
                    if (TR * rg + i < N && g >= 0 && g < NB / TC) {
#pragma unroll
                        for (int j = 0; j < TC; j++) sm.pu.P[prow[i]][TC * g + j] = acc[i][j];
                    }
                }
                __syncthreads();
                if ((c0 >> 6) != ((N - 1) >> 6) && (c0 >> 7) == ((N - 1) >> 7)) {
                    // active rows within two waves' tile rows: one wave takes both (2 rows per lane)
                    const int base = (c0 >> 7) << 7, l = t & 63;
                    const int r2[2] = {base + l < N ? sm.tmap[base + l] : -1, base + 64 + l < N ? sm.tmap[base + 64 + l] : -1};
                    panel_factor_wave<2>(A, N, kk, nb, b, sm, base >> 6, r2);
                } else if ((c0 >> 6) == ((N - 1) >> 6)) {
                    // every active row is a tile row >= c0, all in wave c0 / 64: no barriers
                    const int r1[1] = {t < N ? trow : -1};
                    panel_factor_wave<1>(A, N, kk, nb, b, sm, c0 >> 6, r1);
                } else {
                    panel_factor(A, N, kk, nb, b, sm);
                }
                for (int e = t; e < NB * NB; e += BT) {
                    const int r = e / NB, m = e - r * NB;
                    sm.L11[r][m] = (r < nb && m < r) ? sm.pu.P[sm.perm[kk + r]][m] : 0.;
                }
                __syncthreads();
                TACC(PH_PANEL, tp1);
                jlo = kk - c0 + nb;
                if (jlo >= wJ) break;                  // last chunk of the block column
            } else {
                jlo = 0;
            }
            // L rows of chunk kk (rows below it) and, for an earlier block's chunk, its
            // L11 entries: from A for an earlier block's chunk; for a chunk of this block,
            // from the panel output still in LDS (P). They land in LDS (LT, which aliases
            // P) after the barrier below.
            static_assert(NB * NB <= BT, "one L11 entry per thread");
            double l11v = 0., lrow[NB];
            TSTAMP(tp2);
            if (kk < c0) {
                // tile row t is logical row t here (earlier pivots were final at the block
                // load), so rows t >= kk + nb are below the chunk
                const bool la = t < N && t >= kk + nb;
                const double *src_l = A + (int64_t)(la ? trow : 0) * N + kk;
                if ((N & 1) == 0 && nb == NB) {
                    // 16-byte aligned row segment (N even, kk a multiple of 16): 8 vector loads
                    const double2 *s2 = reinterpret_cast<const double2 *>(src_l);
#pragma unroll
                    for (int m = 0; m < NB / 2; m++) {
                        const double2 v = la ? s2[m] : make_double2(0., 0.);
                        lrow[2 * m] = v.x;
                        lrow[2 * m + 1] = v.y;
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < NB; m++) lrow[m] = (la && m < nb) ? src_l[m] : 0.;
                }
                const int r = t / NB, m = t - r * NB;
                l11v = (t < NB * NB && r < nb && m < r) ? A[(int64_t)sm.perm[kk + r] * N + kk + m] : 0.;
            } else {
                const bool la = t < N && sm.pos[trow] >= kk + nb;
#pragma unroll
                for (int m = 0; m < NB; m++) lrow[m] = (la && m < nb) ? sm.pu.P[la ? trow : 0][m] : 0.;
            }
            // ---- pivot rows of chunk kk (logical kk..kk+nb-1): their current values
            //      in this block column -> Ub (owners write from registers). For an
            //      earlier block's chunk they are tile rows kk.. (logical order as of
            //      the block load, when those pivots were already final).
#pragma unroll
            for (int i = 0; i < TR; i++) {
                if (TR * rg + i < N) {
                    const int q = (kk < c0 ? TR * rg + i : sm.pos[prow[i]]) - kk;
                    if (q >= 0 && q < nb) {
#pragma unroll
                        for (int j = 0; j < TC; j++) sm.Ub[ub][q][TC * cg + j] = acc[i][j];
                    }
                }
            }
            if (kk < c0 && t < NB * NB) sm.L11[t / NB][t % NB] = l11v;
            __syncthreads();
            TACC(PH_T_FETCH, tp2);
            TSTAMP(tp2s);
            // ---- TRSM U = L11^-1 Ub: wave w owns columns [WB/4*w, WB/4*(w+1)), lane l row
            //      l&15 of TC/2 of them; x_r takes its updates for m ascending (oracle
            //      order), x_m broadcast within the 16-lane row by DPP. U rows to A for back
            //      substitution.
            {
                const int l = t & 63, w = t >> 6, r = l & 15;
                double x[TC / 2];
#pragma unroll
                for (int q = 0; q < TC / 2; q++) {
                    const int c = (WB / 4) * w + (l >> 4) + 4 * q;
                    x[q] = (r < nb && c < wJ) ? sm.Ub[ub][r][c] : 0.;
                }
                double lrw[NB];
#pragma unroll
                for (int m = 0; m < NB; m++) lrw[m] = sm.L11[r][m];
                // x_m from lane m of each 16-lane row: DPP row_share:m (0x150 + m)
#define LVG_TRSM_STEP(M_)                                                                  \
                if ((M_) < nb - 1) {                                                       \
                    _Pragma("unroll") for (int q = 0; q < TC / 2; q++) {                   \
                        const double y = dpp_d<0x150 + (M_), 0xf, 0xf>(x[q]);              \
                        if (r > (M_)) x[q] = fma(-lrw[M_], y, x[q]);                       \
                    }                                                                      \
                }
                LVG_TRSM_STEP(0) LVG_TRSM_STEP(1) LVG_TRSM_STEP(2) LVG_TRSM_STEP(3)
                LVG_TRSM_STEP(4) LVG_TRSM_STEP(5) LVG_TRSM_STEP(6) LVG_TRSM_STEP(7)
                LVG_TRSM_STEP(8) LVG_TRSM_STEP(9) LVG_TRSM_STEP(10) LVG_TRSM_STEP(11)
                LVG_TRSM_STEP(12) LVG_TRSM_STEP(13) LVG_TRSM_STEP(14)
#undef LVG_TRSM_STEP
                if (r < nb) {
                    const int64_t prw = (int64_t)sm.perm[kk + r] * N + c0;
#pragma unroll
                    for (int q = 0; q < TC / 2; q++) {
                        const int c = (WB / 4) * w + (l >> 4) + 4 * q;
                        if (c >= jlo && c < wJ) {
                            sm.Ub[ub][r][c] = x[q];
                            A[prw + c] = x[q];
                        }
                    }
                }
            }
            TACC(PH_T_SOLVE, tp2s);
            TSTAMP(tp2t);
            // ---- staged L, transposed (thread per row: conflict-free LDS writes)
            if (t < NMAX) {
#pragma unroll
                for (int m = 0; m < NB; m++) sm.pu.LT[m][t] = lrow[m];
            }
            __syncthreads();
            TACC(PH_T_STAGE, tp2t);
            TACC(PH_TRSM, tp2);
            TSTAMP(tp3);
            // ---- rank-nb update of the rows below (8 x TC register tiles). No masks:
            //      rows that are not below the chunk get l = 0 from the staging, and
            //      both they and the columns left of jlo are final (stored) already,
            //      so whatever lands in their registers is never read again.
            bool any = false;
            if (kk < c0) {
                any = TR * rg + TR - 1 >= kk + nb && TR * rg < N;   // contiguous suffix of tile rows
            } else {
#pragma unroll
                for (int i = 0; i < TR; i++) any = any || (TR * rg + i < N && sm.pos[prow[i]] >= kk + nb);
            }
            if (any && TC * cg + TC - 1 >= jlo) {
                for (int m = 0; m < nb; m++) {
                    // 16-byte LDS reads (ds_read_b128: half the LDS cycles of ds_read2_b64)
                    double a[TR], u[TC];
                    const double2 *ap = reinterpret_cast<const double2 *>(&sm.pu.LT[m][TR * rg]);
                    const double2 *up = reinterpret_cast<const double2 *>(&sm.Ub[ub][m][TC * cg]);
#pragma unroll
                    for (int i = 0; i < TR / 2; i++) { const double2 v = ap[i]; a[2 * i] = v.x; a[2 * i + 1] = v.y; }
#pragma unroll
                    for (int j = 0; j < TC / 2; j++) { const double2 v = up[j]; u[2 * j] = v.x; u[2 * j + 1] = v.y; }
#pragma unroll
                    for (int i = 0; i < TR; i++)
#pragma unroll
                        for (int j = 0; j < TC; j++) acc[i][j] = fma(-a[i], u[j], acc[i][j]);
                }
            }
            // between two earlier chunks the next step's opening barrier suffices: its Ub goes
            // to the other buffer, L11 and LT are only rewritten after every wave has left
            // this step's TRSM / passed that barrier
            if (kk + NB >= c0) __syncthreads();
            TACC(PH_GEMM, tp3);
        }
    }
    back_substitute(A, N, b, sm);
    double emax = 0.;
    if (FUSED && t < N) { src.df[t] = s_acc; emax = fabs(s_acc); }
    return FUSED ? block_max(emax, sm) : 0.;
}

#else
#include "lvg_lu256.h"
#endif

// ------------------------------------------------------------------------------
// iteration_control (iteration_control.h:84-242)
// ------------------------------------------------------------------------------
// accel_step (iteration_control.h:139-193). Each of the nb_param*nb_param + nb_param
// sums runs in one thread in the reference's k order; the small system is solved
// by thread 0 exactly as oracle_lu_solve does.
__device__ __forceinline__ void accel_step(Ctl &C, Slot &S, int N, Smem &sm) {
    const int t = lvg_tid();
    const int np = C.nb_prev - 1;
    const double *r0 = ring(S.res, C.hr, 0, N);
    const double *p0 = ring(S.prev, C.hp, 0, N);
    const int nsum = np * np + np;
    if (t < nsum) {
        int i, j;
        if (t < np * np) { i = t / np; j = t - i * np; } else { i = t - np * np; j = -1; }
        const double *ri = ring(S.res, C.hr, i + 1, N);
        const double *rj = (j >= 0) ? ring(S.res, C.hr, j + 1, N) : nullptr;
        double a = 0.;
        for (int k = 0; k < N; k++) {
            double w = p0[k] + 1.e-99;
            double num = (j >= 0) ? (r0[k] - ri[k]) * (r0[k] - rj[k]) : (r0[k] - ri[k]) * r0[k];
            a = a + num / (w * w);
        }
        sm.pu.hist_acc[t] = a;
    }
    __syncthreads();
    if (t == 0) accel_solve_small(sm.pu.hist_acc, np);
    __syncthreads();
    const double sum = sm.pu.hist_acc[31];
    for (int k = t; k < N; k += BT) {
        double a = (1. - sum) * p0[k];
        for (int i = 0; i < np; i++) a = a + sm.pu.hist_acc[16 + i] * ring(S.prev, C.hp, i + 1, N)[k];
        sm.pold[k] = a;
    }
    __syncthreads();
}

// iteration_control::next_step (iteration_control.h:84-137), split around the
// calc_new_pop solve so that the layer driver has a single LU call site.
__device__ __forceinline__ void next_step_pre(Ctl &C, const LvgDevProblem &P, Slot &S, Smem &sm) {
    const int N = P.N, t = lvg_tid();
    // prev_level_pop.push_front(pop_old)
    C.hp = (C.hp + NHIST - 1) & (NHIST - 1);
    C.np++;
    double *pf = ring(S.prev, C.hp, 0, N);
    for (int i = t; i < N; i += BT) pf[i] = sm.pold[i];
    __syncthreads();
    if (C.acceleration && (C.iter_nb == C.accel_start || C.nb_after_accel == C.accel_period)) {
        accel_step(C, S, N, sm);
        C.nb_after_accel = 0;
    }
}

__device__ __forceinline__ void next_step_post(Ctl &C, const LvgDevProblem &P, Slot &S, Smem &sm, double eq) {
    const int N = P.N, t = lvg_tid();
    C.eq_error = eq;
    if (C.acceleration && C.iter_nb >= C.accel_start) C.nb_after_accel++;
    const bool better = C.eq_error < C.best_eq;
    if (better) C.best_eq = C.eq_error;
    // residual_list.push_front(pop_new - pop_old)
    C.hr = (C.hr + NHIST - 1) & (NHIST - 1);
    C.nr++;
    double *rf = ring(S.res, C.hr, 0, N);
    double pe = 0., re = 0.;
    for (int i = t; i < N; i += BT) {
        double r = sm.pnew[i] - sm.pold[i];
        rf[i] = r;
        pe = fmax(pe, fabs(r));
        re = fmax(re, fabs(r / (sm.pold[i] + 1.e-99)));
        if (better) S.opt[i] = sm.pold[i];
    }
    C.pop_error = block_max(pe, sm);
    C.rel_error = block_max(re, sm);
    if (C.nr > C.nb_prev + 1) C.nr = C.nb_prev + 1;
    if (C.np > C.nb_prev + 1) C.np = C.nb_prev + 1;
    __syncthreads();
    if (C.iter_nb < C.max_iter - 1) {
        for (int i = t; i < N; i += BT) sm.pold[i] = sm.pnew[i];
    } else {
        for (int i = t; i < N; i += BT) sm.pold[i] = S.opt[i];
        C.eq_error = C.best_eq;
    }
    C.iter_nb++;
    __syncthreads();
}

// iteration_control::calculate_populations (iteration_control.h:196-242): state reset
// of one pass; its iteration loop is the driver loop of solve_layer.
__device__ __forceinline__ void start_pass(Ctl &C, const LvgDevProblem &P, Slot &S, const LvgLaunch &Lc,
                                           int max_nb, int accel) {
    const int N = P.N;
    C.acceleration = accel;
    C.accel_start = Lc.accel_start;
    C.accel_period = Lc.accel_period;
    C.nb_prev = Lc.accel_nb;
    C.max_iter = max_nb;
    C.iter_nb = C.nb_after_accel = 0;
    C.best_eq = 1.;
    C.eq_error = C.pop_error = C.rel_error = 0.;
    C.hp = C.hr = 0;
    C.np = C.nr = 0;
    for (int i = lvg_tid(); i < N; i += BT) S.opt[i] = 0.;
    __syncthreads();
}

// One layer of calc_molecular_populations (radiative_transfer.cpp:236-288). from_prev:
// warm chain and the previous layer of the chain converged (:247-249). Returns is_found.
__device__ __forceinline__ bool solve_layer(const LvgDevProblem &P, const LvgLaunch &Lc, int l, Slot &S, Smem &sm,
                                            bool from_prev) {
    const int N = P.N, t = lvg_tid();
    const LvgModeLines &M = Lc.line_overlap ? P.overlap : P.plain;
    TSTAMP(ts0);
    RSTAMP(rs0);
    layer_setup(P, Lc, l, sm);
    TACC(PH_LSETUP, ts0);
    double *pops = Lc.pops + (int64_t)l * N;
    lvg_layer_status *st = reinterpret_cast<lvg_layer_status *>(Lc.status) + l;
    const bool need_boundary = (Lc.init != LVG_INIT_GIVEN);
    // collision operator K and boundary matrix B: built here, or read from the batch
    // built ahead by coll_kernel (K in place, B copied into the slot the LU factors in)
    const double *Kl = S.K, *Bsrc = nullptr, *Bdg = nullptr;
    if (Lc.kall) {
        Kl = Lc.kall + (int64_t)l * N * N;
        if (need_boundary && !from_prev) {
            if (Lc.ball) Bsrc = Lc.ball + (int64_t)l * N * N;   // the boundary LU loads B from here
            else Bdg = Lc.bdiag + (int64_t)l * N;               // ... or forms it from K
        }
    } else if (need_boundary && !from_prev && P.nb_tables == P.nb_neutral) {
        // no electron tables: the boundary LU forms B from K in its chunk load (as from coll_kernel's
        // K), so B is never written to the slot and read back; only its diagonal is kept, in LDS
        layer_collisions(P, sm, S.K, nullptr);
        TSTAMP(tbd0);
        boundary_diagonal(P, S.K, sm.diag);
        TACC(PH_BDIAG, tbd0);
        Bdg = sm.diag;
    } else {
        layer_collisions(P, sm, S.K, (need_boundary && !from_prev) ? S.A : nullptr);
    }
    TACC(PH_SETUP, ts0);

    // initial guess (radiative_transfer.cpp:247-252); the previous layer's populations
    // were written by this same thread (same level index), so they are visible here
    if (Lc.init == LVG_INIT_GIVEN) {
        for (int i = t; i < N; i += BT) { sm.pold[i] = pops[i]; S.given[i] = pops[i]; }
        __syncthreads();
    } else if (from_prev) {
        for (int i = t; i < N; i += BT) { sm.pold[i] = pops[i - N]; S.given[i] = pops[i - N]; }
        __syncthreads();
    }
    // Driver: the boundary-layer solve (iteration_control.cpp:52-91), then the passes of
    // calculate_populations (accelerated, then the plain retry of radiative_transfer.cpp:
    // 258-276), all through ONE block_lu_solve call site (one copy of the LU code).
    Ctl C;
    const int accel = Lc.acceleration;
    const double *yp = (2 * M.nb_lines <= YCAP) ? sm.ylds : S.y;   // line terms in LDS when they fit
    bool boundary = need_boundary && !from_prev;
    bool found = false;
    int iters = 0, retry = 0;
    if (!boundary) start_pass(C, P, S, Lc, accel ? Lc.max_iter_acc : Lc.max_iter_plain, accel);
    for (;;) {
        TSTAMP(tb0);
        LuSrc src;
        if (!boundary) {
            next_step_pre(C, P, S, sm);
            TSTAMP(tl0);
            compute_line_terms(P, M, sm, sm.pold, const_cast<double *>(yp));
            __syncthreads();
            TACC(PH_LINES, tl0);
            TSTAMP(ta0);
            column_diagonals(P, M, Kl, yp, sm);
            TACC(PH_ASSEMBLE, ta0);
            src.K = Kl; src.y = yp; src.li = M.line_idx; src.pop = sm.pold; src.df = S.df;
        } else {
            src.B = Bsrc;
            if (Bdg) { src.BK = Kl; src.BE = P.einst; src.BET = P.einst_t; src.BD = Bdg; }
        }
        for (int i = t; i < N; i += BT) sm.bvec[i] = (i == 0) ? 1. : 0.;
        PH_SHIFT(boundary ? 32 : 0);
        __syncthreads();
        TSTAMP(tlu0);
        const double eq = block_lu_solve(S.A, N, sm.bvec, sm, src, !boundary);
        PH_SHIFT(0);
        if (!boundary) TACC(PH_ITERLU, tlu0);
        if (boundary) {
            TACC(PH_BOUNDARY, tb0);
            for (int i = t; i < N; i += BT) { sm.pold[i] = sm.blog[i]; S.given[i] = sm.blog[i]; }
            __syncthreads();
            if (Lc.dbg_mode == 2) {
                for (int i = t; i < N; i += BT) pops[i] = sm.pold[i];
                return false;
            }
            boundary = false;
            start_pass(C, P, S, Lc, accel ? Lc.max_iter_acc : Lc.max_iter_plain, accel);
            continue;
        }
        for (int i = t; i < N; i += BT) sm.pnew[i] = sm.blog[i];
        __syncthreads();
        next_step_post(C, P, S, sm, eq);
        TACC(PH_ITER, tb0);
        found = C.rel_error < Lc.min_error;
        if (C.iter_nb < C.max_iter && !found) continue;
        iters += C.iter_nb;
        if (!retry && !found && accel && Lc.allow_plain_retry) {
            retry = 1;
            for (int i = t; i < N; i += BT) sm.pold[i] = S.given[i];
            __syncthreads();
            start_pass(C, P, S, Lc, Lc.max_iter_plain, 0);
            continue;
        }
        break;
    }
    for (int i = t; i < N; i += BT) pops[i] = sm.pold[i];
    if (t == 0) {
        st->converged = found ? 1 : 0;
        st->iterations = iters;
        st->used_plain_retry = retry;
        st->reserved = 0;
        st->eq_error = C.eq_error;
        st->rel_error = C.rel_error;
        st->pop_error = C.pop_error;
    }
    TACC(PH_CLK_MEMTIME, ts0);
    RACC(PH_CLK_REALTIME, rs0);
    __syncthreads();
    return found;
}

// Persistent: workgroups pull queue items (layers, or whole warm chains) from an atomic
// counter; `order` maps queue positions to items (longest expected first).
__global__ void __launch_bounds__(BT, OCC) solve_kernel(const LvgDevProblem *__restrict__ Pp,
                                                        const LvgLaunch *__restrict__ Lp) {
    __shared__ Smem sm;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    PH_INIT();
    load_rule_table<BT>(P, sm);
    load_esc_grids(P, sm);
    Slot S = make_slot(P, Lc, blockIdx.x);
    const int nq = Lc.chain_off ? Lc.nb_chain : Lc.nb_lay;
#if !LVG_BIG
    // one solve_layer call site (one copy of the LU code): an independent layer is a chain
    // of one layer; k runs over the current queue item's layers [k, hi)
    int k = 0, hi = 0;
    bool prev = false;
    for (;;) {
        if (k >= hi) {
            if (lvg_tid() == 0) {
                const int q = atomicAdd(Lc.counter, 1);
                sm.layer = (q < nq && Lc.order) ? Lc.order[q] : q;
                sm.pidx = q;
            }
            __syncthreads();
            const int item = uni(sm.layer), q = uni(sm.pidx);
            __syncthreads();
            if (q >= nq) break;
            // warm chain: layers in order, each from its predecessor if that converged
            k = Lc.chain_off ? Lc.chain_off[item] : item;
            hi = Lc.chain_off ? Lc.chain_off[item + 1] : item + 1;
            prev = false;
            continue;
        }
        prev = solve_layer(P, Lc, k, S, sm, prev);
        k++;
    }
#else
    // 768-thread kernel: two call sites allocate better at its 168-register budget (725 vs
    // 3.7 K VGPRs spilled with the single call site)
    for (;;) {
        if (lvg_tid() == 0) {
            const int q = atomicAdd(Lc.counter, 1);
            sm.layer = (q < nq && Lc.order) ? Lc.order[q] : q;
            sm.pidx = q;
        }
        __syncthreads();
        const int l = uni(sm.layer), q = uni(sm.pidx);
        __syncthreads();
        if (q >= nq) break;
        if (!Lc.chain_off) {
            solve_layer(P, Lc, l, S, sm, false);
        } else {
            // warm chain l: layers in order, each from its predecessor if that converged
            const int lo = Lc.chain_off[l], hi = Lc.chain_off[l + 1];
            bool prev = false;
            for (int k = lo; k < hi; k++) prev = solve_layer(P, Lc, k, S, sm, k > lo && prev);
        }
    }
#endif
    PH_FLUSH();
}

// lvg_debug_calc_new_pop: one calc_new_pop for one layer (block 0 only)
__global__ void __launch_bounds__(BT, OCC) debug_kernel(const LvgDevProblem *__restrict__ Pp,
                                                        const LvgLaunch *__restrict__ Lp) {
    __shared__ Smem sm;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    load_rule_table<BT>(P, sm);
    load_esc_grids(P, sm);
    Slot S = make_slot(P, Lc, 0);
    const int N = P.N, t = lvg_tid();
    const LvgModeLines &M = Lc.line_overlap ? P.overlap : P.plain;
    layer_setup(P, Lc, 0, sm);
    layer_collisions(P, sm, S.K, nullptr);
    for (int i = t; i < N; i += BT) sm.pold[i] = Lc.dbg_pop_in[i];
    __syncthreads();
    double *yp = (2 * M.nb_lines <= YCAP) ? sm.ylds : S.y;   // line terms in LDS when they fit
    compute_line_terms(P, M, sm, sm.pold, yp);
    __syncthreads();
    column_diagonals(P, M, S.K, yp, sm);
    for (int i = t; i < N; i += BT) sm.bvec[i] = (i == 0) ? 1. : 0.;
    __syncthreads();
    LuSrc src;
    src.K = S.K; src.y = yp; src.li = M.line_idx; src.pop = sm.pold; src.df = S.df; src.dump = Lc.dbg_matrix;
    const double eq = block_lu_solve(S.A, N, sm.bvec, sm, src, true);
    for (int i = t; i < N; i += BT) { Lc.pops[i] = sm.blog[i]; Lc.dbg_df[i] = S.df[i]; }
    if (t == 0) Lc.dbg_df[N] = eq;
}

// lim_luminosity_lvg (maser_luminosity.cpp:7-106): one workgroup per layer (persistent
// queue), one thread per (transition, level of it). Loss rate of level j: radiative
// terms A_ji (1 + I) / A_ji I over the partners i without inversion (intensity_calc
// with the first layer's populations, as the reference, or the layer's own), then the
// neutral collision rates j -> i for every i (coll_rates.cpp:225-240) in level order,
// read from the neutral-only collision operator K_n (rate j -> i = K_n[i][j]).
__global__ void __launch_bounds__(BT, OCC) lum_kernel(const LvgDevProblem *__restrict__ Pp,
                                                      const LvgLaunch *__restrict__ Lp,
                                                      const LvgLumArgs *__restrict__ Ap) {
    __shared__ Smem sm;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    const LvgLumArgs &A = *Ap;
    load_rule_table<BT>(P, sm);
    Slot S = make_slot(P, Lc, blockIdx.x);
    const LvgModeLines &M = P.plain;
    const int N = P.N, t = lvg_tid(), T = A.nb_trans, nl = Lc.nb_lay;
    const int64_t ld = Lc.soa_ld;
    for (;;) {
        if (t == 0) sm.layer = atomicAdd(Lc.counter, 1);
        __syncthreads();
        const int l = uni(sm.layer);
        __syncthreads();
        if (l >= nl) break;
        layer_setup(P, Lc, l, sm);
        layer_collisions(P, sm, S.K, nullptr, false);
        const double *pl = Lc.pops + (int64_t)l * N;
        const double *ip = A.layer_pops ? pl : Lc.pops;
        for (int w = t; w < 2 * T; w += BT) {
            const int tr = w >> 1, lo = A.low[tr], hi = A.up[tr], j = (w & 1) ? hi : lo;
            double loss = 0.;
            for (int i = 0; i < N; i++) {
                const double aij = P.einst[i * N + j];
                if (aij != 0. && i != lo && i != hi) {
                    const double aji = P.einst[j * N + i];
                    if (i < j && pl[i] * aij > pl[j] * aji) {
                        const double I = intensity_single(P, global_grids(P), M, sm, M.line_idx[i * N + j] >> 1, ip);
                        loss += aji * (1. + I);
                    } else if (i > j && pl[i] * aij < pl[j] * aji) {
                        const double I = intensity_single(P, global_grids(P), M, sm, M.line_idx[j * N + i] >> 1, ip);
                        loss += aji * I;
                    }
                }
            }
            for (int i = 0; i < N; i++)
                if (i != j) loss += S.K[i * N + j];
            S.A[w] = loss;                   // slot scratch: [2T] loss rates (low, up)
        }
        __syncthreads();
        const double *s_ = Lc.soa + l;
        const double ph2 = s_[4 * ld], oh2 = s_[5 * ld], mol = s_[7 * ld], velg = s_[9 * ld];
        for (int tr = t; tr < T; tr += BT) {
            const int lo = A.low[tr], hi = A.up[tr];
            const double low_loss = S.A[2 * tr], up_loss = S.A[2 * tr + 1];
            const double gu = P.g[hi], gl = P.g[lo];
            const int64_t o = (int64_t)tr * nl + l;
            A.emiss[o] = (ph2 + oh2) * mol / velg;
            const double inversion = pl[hi] / gu - pl[lo] / gl;
            if (inversion > 0.) {
                A.lum_arr[o] = inversion / (1. / (up_loss * gu) + 1. / (low_loss * gl)) * mol;
                A.pump_eff[o] = inversion / (pl[hi] / gu + pl[lo] / gl);
            } else {
                A.lum_arr[o] = A.pump_eff[o] = 1.e-99;
            }
            A.loss_rate[o] = (up_loss * gu + low_loss * gl) / (gu + gl);
            A.pump_rate[o] = 0.5 * (pl[hi] * up_loss + pl[lo] * low_loss) / (ph2 + oh2);
        }
        __syncthreads();
    }
}

// cloud average of the luminosity, summed in layer order (one thread per transition)
__global__ void __launch_bounds__(64) lum_reduce_kernel(const LvgLumArgs *__restrict__ Ap, int nl) {
    const LvgLumArgs &A = *Ap;
    const int tr = blockIdx.x * blockDim.x + lvg_tid();
    if (tr >= A.nb_trans) return;
    double s = 0.;
    for (int l = 0; l < nl; l++) s += A.lum_arr[(int64_t)tr * nl + l] * A.dz[l];
    A.lum[tr] = s / A.height;
}

#if !LVG_BIG && !LVG_WIDE
// ---- collision operators of a whole batch of layers, ahead of the solve ----------------
// build_collision_operators for every layer of the launch into K_all / B_all (HBM), with
// a small LDS footprint (layer scalars and the rule table only) so that many workgroups
// per CU overlap the table-fetch latency that one LU-sized workgroup per layer exposes.
// Same function, same arithmetic: the solve reads bit-identical K and B. Any N (the
// 16x16 pair tiles and the column sums loop over N).
struct CollSmem {
    double T, Te, vw, vgrad, nmol, ne;
    double cc[LVG_MAX_COMBOS];
    double teff[LVG_MAX_TABLES];
    int    lo[LVG_MAX_TABLES];
    const double *tcol[LVG_MAX_TABLES];
    const double *tder[LVG_MAX_TABLES];
    int64_t timax[LVG_MAX_TABLES];
    double tdt[LVG_MAX_TABLES];
    double tx[LVG_MAX_TABLES];
    int8_t ttab[LVG_MAX_CLASSES][LVG_MAX_TERMS], tcombo[LVG_MAX_CLASSES][LVG_MAX_TERMS];
    int8_t tet[LVG_MAX_CLASSES], tgrp[LVG_MAX_CLASSES];
    double dust[LVG_MAX_DUST];
};

constexpr int COLL_K_PU = 2;    // pair tiles per batch in coll_kernel (1 and 8 WG/CU variants spill)
constexpr int COLL_K_OCC = 4;   // workgroups per CU coll_kernel is built for (register budget)
__global__ void __launch_bounds__(BT, COLL_K_OCC) coll_kernel(const LvgDevProblem *__restrict__ Pp,
                                                              const LvgLaunch *__restrict__ Lp) {
    __shared__ CollSmem sm;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    PH_INIT();
    load_rule_table<BT>(P, sm);
    const int64_t NN = (int64_t)P.N * P.N;
    // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so workgroup b
    // takes position chunk (b % 8) of the temperature-ordered list: each XCD's resident
    // layers span a narrow temperature range and share table rows in its L2
    const int G = gridDim.x, b = blockIdx.x;
    const int rb = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
    for (int pos = rb; pos < Lc.nb_lay; pos += G) {
        const int l = Lc.coll_order ? Lc.coll_order[pos] : pos;
        if (lvg_tid() == 0) layer_scalars(P, Lc, l, sm);
        __syncthreads();
        double *Kl = const_cast<double *>(Lc.kall) + l * NN;
        build_collision_operators<BT, COLL_K_PU>(P, sm, Kl, Lc.ball ? const_cast<double *>(Lc.ball) + l * NN : nullptr,
                                                 nullptr);
        if (Lc.bdiag) {
            // B's diagonal only (no electron rates: B = K + A/2 above the diagonal, K below):
            // minus the ascending column sum, as build_collision_operators forms it
            const int N = P.N;
            for (int d = lvg_tid(); d < N; d += BT) {
                double a = 0.;
                for (int r = 0; r < N; r++) {
                    if (r == d) continue;
                    const double k = Kl[(int64_t)r * N + d];
                    const double bb = (r < d) ? 0.5 * P.einst[(int64_t)d * N + r] + k : k;
                    a = a - bb;
                }
                const_cast<double *>(Lc.bdiag)[(int64_t)l * N + d] = a;
            }
        }
        __syncthreads();
    }
    PH_FLUSH();
}
#endif

}  // namespace LVG_NS

extern "C" hipError_t LVG_SYM(lvg_launch_lum)(const LvgDevProblem *P, const LvgLaunch *L, const LvgLumArgs *A, int grid,
                                              int nb_trans, int nb_lay, hipStream_t s) {
    hipLaunchKernelGGL(LVG_NS::lum_kernel, dim3(grid), dim3(LVG_NS::BT), 0, s, P, L, A);
    hipLaunchKernelGGL(LVG_NS::lum_reduce_kernel, dim3((nb_trans + 63) / 64), dim3(64), 0, s, A, nb_lay);
    return hipGetLastError();
}

// P and L are DEVICE pointers to the parameter blocks
extern "C" hipError_t LVG_SYM(lvg_launch_solve)(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s) {
    hipLaunchKernelGGL(LVG_NS::solve_kernel, dim3(grid), dim3(LVG_NS::BT), 0, s, P, L);
    return hipGetLastError();
}

#if !LVG_BIG && !LVG_WIDE
extern "C" hipError_t lvg_launch_coll(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s) {
    hipLaunchKernelGGL(lvg::coll_kernel, dim3(grid), dim3(lvg::BT), 0, s, P, L);
    return hipGetLastError();
}
#endif

extern "C" hipError_t LVG_SYM(lvg_launch_debug)(const LvgDevProblem *P, const LvgLaunch *L, hipStream_t s) {
    hipLaunchKernelGGL(LVG_NS::debug_kernel, dim3(1), dim3(LVG_NS::BT), 0, s, P, L);
    return hipGetLastError();
}

extern "C" int LVG_SYM(lvg_kernel_max_levels)(void) { return LVG_NS::NMAX; }
extern "C" int LVG_SYM(lvg_kernel_block_threads)(void) { return LVG_NS::BT; }
extern "C" hipError_t LVG_SYM(lvg_kernel_occupancy)(int *blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, LVG_NS::solve_kernel, LVG_NS::BT, 0);
}

#ifdef LVG_PHASE_TIMERS
extern "C" int LVG_SYM(lvg_debug_phase_cycles)(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(LVG_NS::lvg_phase_cycles), sizeof(unsigned long long) * LVG_NS::PH_SLOTS) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[LVG_NS::PH_SLOTS] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(LVG_NS::lvg_phase_cycles), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
