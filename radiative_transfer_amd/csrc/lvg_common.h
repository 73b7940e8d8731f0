// lvg_common.h — device helpers shared by the block kernels (lvg_kernels.hip, compiled
// as namespace lvg and lvg_big) and the wave kernel (lvg_wave.hip, namespace lvg).
// Included INSIDE the including translation unit's namespace: every function is an
// inline device function, so each kernel family gets its own copy.
//
// Contents: physical constants, DPP wave reductions, the escape-probability lookups
// (lvg_method_functions.cpp:74-110, :324-392), the layer scalars of set_parameters /
// set_gas_param (iteration_lvg.cpp:59-85, coll_rates.cpp:152-174), the collision-operator
// build (coll_rates*.cpp get_rate_*, iteration_lvg.cpp:118-131, iteration_control.cpp:
// 69-85), the line-term helpers of intensity_calc (iteration_lvg.cpp:163-185, :428-501)
// and the iteration-control state of iteration_control.h:84-242.
#pragma once

// Diagnostic build only (-DLVG_PHASE_TIMERS): per-phase s_memtime cycle sums, kept in
// LDS by thread 0 of a workgroup (lane 0 of every wave in the wave kernel), flushed to
// lvg_phase_cycles[] once per workgroup. Never in the product library.
#ifdef LVG_PHASE_TIMERS
enum { PH_SETUP, PH_BOUNDARY, PH_LINES, PH_ASSEMBLE, PH_PANEL, PH_TRSM, PH_GEMM, PH_BACKSUB, PH_CTL,
       PH_LSETUP, PH_PAIRS, PH_BDIAG, PH_BLOAD, PH_CLK_MEMTIME, PH_CLK_REALTIME, PH_RSV,
       PH_T_FETCH, PH_T_SOLVE, PH_T_STAGE, PH_P_RED, PH_P_POST, PH_P_WB, PH_BS_DIAG, PH_BS_UPD, PH_BS_WAIT,
       PH_ITERLU, PH_ITER, PH_N };
// 64 counters: [0, 32) as named above; in the 256/512-thread block kernels the phases timed
// inside a boundary-layer LU land at +32 (lvg_ph_shift), so the LU sub-phases of the boundary
// and of the iteration LUs are told apart (tools/phase_timers.py)
constexpr int PH_SLOTS = 64;
__device__ unsigned long long lvg_phase_cycles[PH_SLOTS];
#define TSTAMP(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define RSTAMP(v) unsigned long long v = __builtin_amdgcn_s_memrealtime()
// sums kept in LDS (no global atomics inside the timed code: queued atomics would hold
// up the vmcnt waits of later loads), flushed once per block
__shared__ unsigned long long lvg_ph_lds[PH_SLOTS];
__shared__ int lvg_ph_shift;
#define RACC(ph, v0) do { if (lvg_tid() == 0) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); \
    lvg_ph_lds[ph] += t_ - (v0); } } while (0)
#define TACC(ph, v0) do { if (lvg_tid() == 0) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    lvg_ph_lds[ph] += t_ - (v0); } } while (0)
#define PH_INIT() do { if (lvg_tid() < PH_SLOTS) lvg_ph_lds[lvg_tid()] = 0; if (lvg_tid() == 0) lvg_ph_shift = 0; \
    __syncthreads(); } while (0)
#define PH_SHIFT(v) do { if (lvg_tid() == 0) lvg_ph_shift = (v); } while (0)
#define PH_FLUSH() do { __syncthreads(); if (lvg_tid() < PH_SLOTS && lvg_ph_lds[lvg_tid()]) \
    atomicAdd(&lvg_phase_cycles[lvg_tid()], lvg_ph_lds[lvg_tid()]); } while (0)
#else
#define TSTAMP(v) do {} while (0)
#define TACC(ph, v0) do {} while (0)
#define RSTAMP(v) do {} while (0)
#define RACC(ph, v0) do {} while (0)
#define PH_INIT() do {} while (0)
#define PH_SHIFT(v) do {} while (0)
#define PH_FLUSH() do {} while (0)
#endif

constexpr int NHIST = LVG_HIST_SLOTS;

// The thread index behind an empty asm, so that nothing derived from it (per-thread row
// addresses of the slot arrays, LDS offsets, lane masks) is hoisted out of the persistent
// loops and kept live across the LU: in the block kernels those hoisted values were what
// pushed solve_kernel into scratch (128 VGPRs spilled, 280 B/lane, round 4). Recomputing
// them where they are used costs a few integer instructions per use.
__device__ __forceinline__ int lvg_tid() {
    int v = threadIdx.x;
    __asm__ volatile("" : "+v"(v));
    return v;
}

// Global-memory pointers (address space 1). The slot, table and layer pointers reach the kernels
// through structs in device memory, so the compiler cannot infer their address space and emits
// FLAT accesses: those complete out of order with LDS operations, so every use of a loaded value
// waits for ALL of the wave's outstanding memory and LDS operations (s_waitcnt vmcnt(0)
// lgkmcnt(0)). Through a gp<T> pointer it emits global loads with counted vmcnt waits.
template <class T> using gp = __attribute__((address_space(1))) T *;
//
// RULE: glb() only on pointers that always name HBM (A, K, li, BK / BE / B, line_idx, the tables).
// Never on y / diag / pop / b: those are LDS arrays on some paths (the y-cache when the lines fit
// YCAP), and a global load of an LDS offset reads an unmapped address (the round-5 fault of probes
// vgB / vgC, profiles/r5/variants.txt item 13). The checked build (-DLVG_CHECKED_GLB, used by the
// timer / variant builds and tools/build_checked.sh) traps on a shared or private pointer.
#ifdef LVG_CHECKED_GLB
template <class T> __device__ __forceinline__ gp<T> glb(T *p) {
#if __HIP_DEVICE_COMPILE__
    if (__builtin_amdgcn_is_shared((const void *)p) || __builtin_amdgcn_is_private((const void *)p)) __builtin_trap();
#endif
    return (gp<T>)p;
}
#else
template <class T> __device__ __forceinline__ gp<T> glb(T *p) { return (gp<T>)p; }
#endif
// 16-byte vectors for loads and stores through gp pointers (builtin vector types: HIP's double2 /
// int4 classes cannot be copied from an address-space-qualified object)
typedef double vd2 __attribute__((ext_vector_type(2)));
typedef double vd2u __attribute__((ext_vector_type(2), aligned(8)));
typedef int vi4 __attribute__((ext_vector_type(4)));

constexpr double BOLTZMANN_CONSTANT    = 1.380649e-16;
constexpr double CM_INVERSE_TO_KELVINS = 1.438776877;
constexpr double EIGHT_PI              = 25.132741228718345;
constexpr double SPEED_OF_LIGHT        = 2.99792458e+10;
constexpr double MIN_COLLISION_RATE    = 1.e-99;
constexpr double INV_TRANS_FACTOR      = -0.1;
constexpr double MIN_LINE_OPACITY      = 1.e-99;

// ------------------------------------------------------------------------------
// wave reductions and broadcasts
// ------------------------------------------------------------------------------
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// DPP wave reductions (gfx9 row_shr / row_bcast sequence; the result lands in lane 63
// and is broadcast with readlane). old == src makes lanes without a DPP source keep
// their own value, the identity of max/min.
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ double dpp_d(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    // every caller broadcasts within full rows (row_newbcast, all rows and banks): no lane keeps
    // an old value, so the DPP move writes a fresh register instead of a copy of x
    static_assert(ROW == 0xf && BANK == 0xf, "mov_dpp leaves disabled lanes undefined");
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, ROW, BANK, false);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, ROW, BANK, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ unsigned dpp_u0(unsigned x) {   // out-of-row lanes read 0 (bound_ctrl)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW, BANK, true);
}
// wave-wide unsigned max; each step folds into one v_max_u32_dpp
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, dpp_u0<0x111, 0xf, 0xf>(v));   // row_shr:1
    v = max(v, dpp_u0<0x112, 0xf, 0xf>(v));   // row_shr:2
    v = max(v, dpp_u0<0x113, 0xf, 0xf>(v));   // row_shr:3
    v = max(v, dpp_u0<0x114, 0xf, 0xe>(v));   // row_shr:4
    v = max(v, dpp_u0<0x118, 0xf, 0xc>(v));   // row_shr:8
    v = max(v, dpp_u0<0x142, 0xa, 0xf>(v));   // row_bcast:15
    v = max(v, dpp_u0<0x143, 0xc, 0xf>(v));   // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ double readlane_d(double x, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
    return __hiloint2double(hi, lo);
}

// Pivot key of oracle_lu_solve's rule (largest |v|, first maximum wins; amax seeded with
// |a_kk| and replaced on a strict '>', so a NaN below never wins and a NaN on the
// diagonal always does): |v| >= 0 orders like its bit pattern; rows still taking part
// carry the top bit. Returns the upper word in hi, the lower in lo.
__device__ __forceinline__ void pivot_key(double v, bool act, bool on_diag, unsigned &hi, unsigned &lo) {
    const double av = fabs(v);
    const unsigned long long bits = (act && av == av) ? (unsigned long long)__double_as_longlong(av) : 0ull;
    const bool dnan = act && on_diag && av != av;
    hi = dnan ? 0xffffffffu : act ? ((unsigned)(bits >> 32) | 0x80000000u) : 0u;
    lo = dnan ? 0xffffffffu : (unsigned)bits;
}

// ------------------------------------------------------------------------------
// escape probabilities
// ------------------------------------------------------------------------------
// locate_index restatement: -1 below, n-1 above, else a[j] <= x < a[j+1]
__device__ __forceinline__ int locate_index(const double *a, int n, double x) {
    if (x < a[0]) return -1;
    if (x > a[n - 1]) return n - 1;
    int l = 0, r = n - 1;
    while (r - l > 1) {
        int m = l + ((r - l) >> 1);
        if (a[m] <= x) l = m; else r = m;
    }
    return l;
}

// Grids the escape-probability lookups bisect: the problem's global copies (block
// kernel) or LDS copies (wave kernel); the tables stay in HBM/L2.
struct EscGrids {
    const double *ed, *eg;                 // esc_delta, esc_gamma
    const double *old, *odx, *ogr, *og;    // ov_ld, ov_dx, ov_gr, ov_g
};
__device__ __forceinline__ EscGrids global_grids(const LvgDevProblem &P) {
    return EscGrids{P.esc_delta, P.esc_gamma, P.ov_ld, P.ov_dx, P.ov_gr, P.ov_g};
}

// lvg_method_data::get_esc_func (lvg_method_functions.cpp:74-110)
__device__ __forceinline__ double esc_func(const LvgDevProblem &P, const EscGrids &G, double gamma, double delta) {
    const int nd = P.esc_nd, ng = P.esc_ng;
    int k = locate_index(G.ed, nd, delta);
    int l = locate_index(G.eg, ng, gamma);
    double t, u;
    if (k < 0) { t = 0.; k = 0; }
    else if (k > nd - 2) { t = 1.; k = nd - 2; }
    else t = (delta - G.ed[k]) / (G.ed[k + 1] - G.ed[k]);
    if (l < 0) { l = 0; u = 0.; }
    else if (l > ng - 2) { l = ng - 2; u = 1.; }
    else u = (gamma - G.eg[l]) / (G.eg[l + 1] - G.eg[l]);
    const double *p = P.esc_p;
    double e = p[k * ng + l] * (1. - t) * (1. - u) + p[(k + 1) * ng + l] * t * (1. - u)
             + p[k * ng + l + 1] * (1. - t) * u + p[(k + 1) * ng + l + 1] * u * t;
    return e > 1. ? 1. : (e < 0. ? 0. : e);
}

// lvg_line_overlap_data::get_esc_func (lvg_method_functions.cpp:324-392); the
// 16 terms in the reference's order, each weighted (u, t, p, y) left to right
__device__ __forceinline__ double overlap_esc_func(const LvgDevProblem &P, const EscGrids &G, const double *tab,
                                                   double gamma, double delta, double gratio, double dxv) {
    delta = lvg_log10(delta);
    int m = locate_index(G.old, P.ov_nd, delta);
    int l = locate_index(G.og, P.ov_ng, gamma);
    int k = locate_index(G.ogr, P.ov_ngr, gratio);
    int n = locate_index(G.odx, P.ov_ndx, dxv);
    double y = 0., u = 0., t = 0., p = 0.;
    if (m < 0) m = 0;
    else if (m > P.ov_nd - 2) { m = P.ov_nd - 2; y = 1.; }
    else y = (delta - G.old[m]) / (G.old[m + 1] - G.old[m]);
    if (n < 0) n = 0;
    else if (n > P.ov_ndx - 2) { p = 1.; n = P.ov_ndx - 2; }
    else p = (dxv - G.odx[n]) / (G.odx[n + 1] - G.odx[n]);
    if (l < 0) l = 0;
    else if (l > P.ov_ng - 2) { l = P.ov_ng - 2; u = 1.; }
    else u = (gamma - G.og[l]) / (G.og[l + 1] - G.og[l]);
    if (k < 0) k = 0;
    else if (k > P.ov_ngr - 2) { t = 1.; k = P.ov_ngr - 2; }
    else t = (gratio - G.ogr[k]) / (G.ogr[k + 1] - G.ogr[k]);
    const int W = P.ov_ngr * P.ov_ng, ndx = P.ov_ndx, ng = P.ov_ng;
    double e = 0.;
#pragma unroll
    for (int dm = 0; dm < 2; dm++)
#pragma unroll
        for (int dn = 0; dn < 2; dn++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++)
#pragma unroll
                for (int dl = 0; dl < 2; dl++)
                    e += tab[(int64_t)((m + dm) * ndx + n + dn) * W + (k + dk) * ng + l + dl]
                         * (dl ? u : 1. - u) * (dk ? t : 1. - t) * (dn ? p : 1. - p) * (dm ? y : 1. - y);
    return e > 1. ? 1. : (e < 0. ? 0. : e);
}

// ------------------------------------------------------------------------------
// layer setup: iteration_scheme_lvg::set_parameters / set_gas_param
// ------------------------------------------------------------------------------
// the layer's scalars into sm (one thread; SM: the block kernels' Smem / CollSmem or the
// wave kernel's WaveLayer)
// collision table tb's temperature interval at the layer's T (neutral) or Te (electrons)
template <class SM>
__device__ __forceinline__ void layer_table(const LvgDevProblem &P, int tb, double T, double Te, SM &sm) {
    const double *tg = P.tab_tgrid + P.tab_tg_off[tb];
    int jm = P.tab_jmax[tb];
    double temp = (tb < P.nb_neutral) ? T : Te;
    int lo = 0, hi = jm - 1;                  // collision_data::locate, strict '<'
    while (hi - lo > 1) {
        int j = lo + ((hi - lo) >> 1);
        if (tg[j] < temp) lo = j; else hi = j;
    }
    sm.lo[tb] = lo;
    double tmax = tg[jm - 1];
    sm.teff[tb] = temp < tmax ? temp : tmax;
    const int64_t imax = (int64_t)P.tab_nb_lev[tb] * (P.tab_nb_lev[tb] - 1) / 2;
    sm.timax[tb] = imax;
    sm.tcol[tb] = P.tab_coeff + P.tab_c_off[tb] + (int64_t)lo * imax;
    sm.tder[tb] = P.tab_deriv + P.tab_c_off[tb] + (int64_t)lo * imax;
    sm.tdt[tb] = tg[lo + 1] - tg[lo];
    sm.tx[tb] = sm.teff[tb] - tg[lo];
}

// SPLIT: the table intervals through layer_table (the block kernels: same operations, a register
// allocation with 116 fewer SGPR spills in solve_kernel at equal speed, profiles/r6/variants.txt
// item 8's build); the wave kernel keeps the loop inline (its NM = 48 allocation spills more otherwise)
template <class SM, bool SPLIT = false>
__device__ __forceinline__ void layer_scalars(const LvgDevProblem &P, const LvgLaunch &Lc, int l, SM &sm) {
    const int64_t ld = Lc.soa_ld;
    const double *s = Lc.soa + Lc.lay_offset + l;
    double T = s[0 * ld], Te = s[1 * ld];
    double ne = s[2 * ld], nh = s[3 * ld], nph2 = s[4 * ld], noh2 = s[5 * ld], nhe = s[6 * ld];
    double vt = s[8 * ld];
    sm.T = T; sm.Te = Te;
    sm.nmol = s[7 * ld];
    sm.ne = ne;
    sm.vgrad = s[9 * ld];
    sm.vw = sqrt(2. * BOLTZMANN_CONSTANT * T / P.mass + vt * vt);   // iteration_lvg.cpp:65
    for (int c = 0; c < P.nb_comp; c++) sm.dust[c] = s[(10 + c) * ld];
    const double n5[5] = {nhe, nph2, noh2, nh, ne};
    for (int k = 0; k < P.terms.nb_combos; k++) {
        double a = 0.;
        bool first = true;
        for (int q = 0; q < 5; q++) {
            double w = P.terms.combo_w[k][q];
            if (w == 0.) continue;
            double term = (w == 1.) ? n5[q] : w * n5[q];
            a = first ? term : a + term;
            first = false;
        }
        sm.cc[k] = a;
    }
    if (SPLIT) {
        for (int tb = 0; tb < P.nb_tables; tb++) layer_table(P, tb, T, Te, sm);
        return;
    }
    for (int tb = 0; tb < P.nb_tables; tb++) {
        const double *tg = P.tab_tgrid + P.tab_tg_off[tb];
        int jm = P.tab_jmax[tb];
        double temp = (tb < P.nb_neutral) ? T : Te;
        int lo = 0, hi = jm - 1;                  // collision_data::locate, strict '<'
        while (hi - lo > 1) {
            int j = lo + ((hi - lo) >> 1);
            if (tg[j] < temp) lo = j; else hi = j;
        }
        sm.lo[tb] = lo;
        double tmax = tg[jm - 1];
        sm.teff[tb] = temp < tmax ? temp : tmax;
        const int64_t imax = (int64_t)P.tab_nb_lev[tb] * (P.tab_nb_lev[tb] - 1) / 2;
        sm.timax[tb] = imax;
        sm.tcol[tb] = P.tab_coeff + P.tab_c_off[tb] + (int64_t)lo * imax;
        sm.tder[tb] = P.tab_deriv + P.tab_c_off[tb] + (int64_t)lo * imax;
        sm.tdt[tb] = tg[lo + 1] - tg[lo];
        sm.tx[tb] = sm.teff[tb] - tg[lo];
    }
}

// the compiled molecule rule, copied to LDS once per launch (BTH threads)
template <int BTH, class SM>
__device__ __forceinline__ void load_rule_table(const LvgDevProblem &P, SM &sm) {
    for (int e = lvg_tid(); e < LVG_MAX_CLASSES * LVG_MAX_TERMS; e += BTH) {
        (&sm.ttab[0][0])[e] = (&P.terms.table[0][0])[e];
        (&sm.tcombo[0][0])[e] = (&P.terms.combo[0][0])[e];
    }
    for (int e = lvg_tid(); e < LVG_MAX_CLASSES; e += BTH) {
        sm.tet[e] = P.terms.etable[e];
        sm.tgrp[e] = P.terms.group[e];
    }
    __syncthreads();
}

// Collision operator K (neutral + electron rates; iteration_lvg.cpp:121-131) and
// the boundary-layer matrix B (neutrals + A/2; iteration_control.cpp:69-85),
// row-major M[final][initial]. K keeps off-diagonals only (its diagonal is
// rebuilt every iteration in the reference's order); B gets its diagonal as the
// ascending column sum, row 0 <- 1. Level pairs (f > s) are walked in 16x16 tiles
// of the lower triangle, one pair per thread: table reads and the K[f][s] writes
// are 128-byte row segments, every lane is busy. The pair classes are staged in LDS
// (cls, when the caller has room: one wide coalesced copy instead of a dependent global
// load in front of every batch's coefficient loads). A batch of PU tiles issues its
// index and coefficient loads first; its K/B stores go out behind the next batch's
// loads (vmcnt counts loads and stores in order, so a load issued after a store
// would wait for it).
template <int BTH, int PU, class SM>
__device__ __forceinline__ void build_collision_operators(const LvgDevProblem &P, SM &sm, double *K, double *B,
                                                          uint8_t *cls_lds, bool electrons = true) {
    const int N = P.N, t = lvg_tid();
    const double T = sm.T, Te = sm.Te;
    const int nt = (N + 15) >> 4, ntiles = nt * (nt + 1) / 2;
    const int fl = (t >> 4) & 15, sl = t & 15;
    TSTAMP(tq0);
    const int M = N * (N - 1) / 2;
    if (cls_lds) {
        const int n16 = M >> 4;
        const uint4 *src4 = reinterpret_cast<const uint4 *>(P.pair_class);
        for (int e = t; e < n16; e += BTH) reinterpret_cast<uint4 *>(cls_lds)[e] = src4[e];
        for (int e = (n16 << 4) + t; e < M; e += BTH) cls_lds[e] = P.pair_class[e];
        __syncthreads();
    }
    constexpr int TG = BTH / 256;                    // TG groups of 256 threads, PU tiles each
    const int tg = t >> 8;
    double wk0[PU], wk1[PU], wb0[PU], wb1[PU];
    int wf[PU], ws[PU];
#pragma unroll
    for (int u = 0; u < PU; u++) wf[u] = -1;
    auto flush = [&]() {
#pragma unroll
        for (int u = 0; u < PU; u++) {
            if (wf[u] >= 0) {
                const int f = wf[u], s2 = ws[u];
                K[s2 * N + f] = wk0[u];
                K[f * N + s2] = wk1[u];
                if (B) {
                    B[s2 * N + f] = wb0[u];
                    B[f * N + s2] = wb1[u];
                }
            }
        }
    };
    for (int q0 = 0; q0 < ntiles; q0 += PU * TG) {
        int pc[PU], fc[PU], sc[PU], cls[PU];
#pragma unroll
        for (int u = 0; u < PU; u++) {
            // tile q = (F, S), S <= F, in row order of the lower triangle of tiles
            const int q = q0 + tg * PU + u;
            int F = (int)((sqrt(8. * q + 1.) - 1.) * 0.5);
            while (F * (F + 1) / 2 > q) F--;
            while ((F + 1) * (F + 2) / 2 <= q) F++;
            const int S = q - F * (F + 1) / 2;
            fc[u] = 16 * F + fl; sc[u] = 16 * S + sl;
            pc[u] = (q < ntiles && fc[u] < N && sc[u] < fc[u]) ? fc[u] * (fc[u] - 1) / 2 + sc[u] : -1;
        }
#pragma unroll
        for (int u = 0; u < PU; u++) cls[u] = pc[u] < 0 ? 0 : cls_lds ? cls_lds[pc[u]] : P.pair_class[pc[u]];
        // level data of the batch, loaded before any store of it
        double ef[PU], es[PU], gf[PU], gs[PU], af[PU];
#pragma unroll
        for (int u = 0; u < PU; u++) {
            const bool ok = pc[u] >= 0;
            const int f = ok ? fc[u] : 1, s = ok ? sc[u] : 0;
            ef[u] = P.energy[f]; es[u] = P.energy[s];
            gf[u] = P.g[f]; gs[u] = P.g[s];
            af[u] = B ? P.einst[f * N + s] : 0.;
        }
        double c0[PU][LVG_MAX_TERMS + 1], c1[PU][LVG_MAX_TERMS + 1];
#pragma unroll
        for (int u = 0; u < PU; u++) {
            bool alive = pc[u] >= 0;
#pragma unroll
            for (int k = 0; k <= LVG_MAX_TERMS; k++) {
                const int tb = (k < LVG_MAX_TERMS) ? sm.ttab[cls[u]][k] : sm.tet[cls[u]];
                if (k < LVG_MAX_TERMS) alive = alive && tb >= 0;
                const bool ld = (k < LVG_MAX_TERMS) ? alive : (pc[u] >= 0 && tb >= 0);
                c0[u][k] = 0.; c1[u][k] = 0.;
                if (ld) {
                    c0[u][k] = sm.tcol[tb][pc[u]];
                    c1[u][k] = sm.tder[tb][pc[u]];          // slope (calc_coeff_deriv)
                }
            }
        }
        flush();                                // the previous batch's stores, behind this batch's loads
#pragma unroll
        for (int u = 0; u < PU; u++) {
            wf[u] = -1;
            if (pc[u] < 0) continue;
            const int cl = cls[u], f = fc[u], s = sc[u];
            const int grp = sm.tgrp[cl];
            double dn = 0., gsum = 0.;
            int ng = 0;
#pragma unroll
            for (int k = 0; k < LVG_MAX_TERMS; k++) {
                const int tb = sm.ttab[cl][k];
                if (tb < 0) break;
                const double r = (c0[u][k] + c1[u][k] * sm.tx[tb]) * sm.cc[sm.tcombo[cl][k]];   // get_rate
                if (k < grp) dn = (k == 0) ? r : dn + r;
                else { gsum = (ng == 0) ? r : gsum + r; ng++; }
            }
            if (ng) dn = dn + gsum;
            const double de = es[u] - ef[u];
            double un = 0.;
            if (dn > MIN_COLLISION_RATE) un = dn * lvg_exp(de * CM_INVERSE_TO_KELVINS / T) * gf[u] / gs[u];
            else dn = 0.;
            double dE = 0., uE = 0.;
            const int et = sm.tet[cl];
            if (et >= 0 && electrons) {
                dE = (c0[u][LVG_MAX_TERMS] + c1[u][LVG_MAX_TERMS] * sm.tx[et]) * sm.ne;
                if (dE > MIN_COLLISION_RATE) uE = dE * lvg_exp(de * CM_INVERSE_TO_KELVINS / Te) * gf[u] / gs[u];
                else dE = 0.;
            }
            wk0[u] = dn + dE;
            wk1[u] = un + uE;
            wb0[u] = 0.5 * af[u] + dn;
            wb1[u] = un;
            wf[u] = f;
            ws[u] = s;
        }
    }
    flush();
    __syncthreads();
    TACC(PH_PAIRS, tq0);
    TSTAMP(tq1);
    if (B) {
        for (int d = t; d < N; d += BTH) {
            double a = 0.;
            for (int r0 = 0; r0 < N; r0 += 32) {
                double bv[32];
#pragma unroll
                for (int u = 0; u < 32; u++) bv[u] = (r0 + u < N) ? B[(r0 + u) * N + d] : 0.;
#pragma unroll
                for (int u = 0; u < 32; u++) {
                    const int r = r0 + u;
                    if (r < N && r != d) a = a - bv[u];
                }
            }
            B[d * N + d] = a;
        }
        __syncthreads();
        for (int j = t; j < N; j += BTH) B[j] = 1.;   // row 0 <- 1 (iteration_control.cpp:82-84)
        __syncthreads();
    }
    TACC(PH_BDIAG, tq1);
}

// build_collision_operators with two batches in flight (the block kernels, no B: the boundary
// matrix is formed from K in the LU's chunk load). NT neutral term slots and, when HE, the
// electron slot are loaded for every pair, UNCONDITIONALLY (a missing term reads a clamped address
// of table 0 and is never used), and the K stores are unconditional too (an idle lane writes
// K[0], a diagonal entry nothing reads), so the number of memory operations between a batch's
// loads and their use is fixed and the waits are counted: batch b + 1's loads are issued
// before batch b is evaluated. Same operations per pair as build_collision_operators.
template <int BTH, int PU, int NT, bool HE, class SM>
__device__ __forceinline__ void build_collision_pipe(const LvgDevProblem &P, SM &sm, double *K, const uint8_t *cls_gen,
                                                     bool electrons) {
    typedef __attribute__((address_space(3))) const uint8_t *lds_u8;
    const lds_u8 cls_lds = (lds_u8)cls_gen;          // the pair classes staged in LDS (required)
    const int N = P.N, t = lvg_tid();
    const double T = sm.T, Te = sm.Te;
    const int nt = (N + 15) >> 4, ntiles = nt * (nt + 1) / 2;
    const int fl = (t >> 4) & 15, sl = t & 15;
    constexpr int TG = BTH / 256;
    constexpr int NS = NT + (HE ? 1 : 0);
    const int tg = t >> 8;
    gp<double> Kg = glb(K);
    struct Stage {
        int pc[PU], fc[PU], sc[PU], cls[PU];
        double ef[PU], es[PU], gf[PU], gs[PU];
        double c0[PU][NS], c1[PU][NS];
    };
    auto issue = [&](Stage &S, int q0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < PU; u++) {
            const int q = q0 + tg * PU + u;
            int F = (int)((sqrt(8. * q + 1.) - 1.) * 0.5);
            while (F * (F + 1) / 2 > q) F--;
            while ((F + 1) * (F + 2) / 2 <= q) F++;
            const int S2 = q - F * (F + 1) / 2;
            S.fc[u] = 16 * F + fl; S.sc[u] = 16 * S2 + sl;
            S.pc[u] = (q < ntiles && S.fc[u] < N && S.sc[u] < S.fc[u]) ? S.fc[u] * (S.fc[u] - 1) / 2 + S.sc[u] : -1;
        }
#pragma unroll
        for (int u = 0; u < PU; u++) S.cls[u] = cls_lds[S.pc[u] < 0 ? 0 : S.pc[u]];
#pragma unroll
        for (int u = 0; u < PU; u++) {
            const bool ok = S.pc[u] >= 0;
            const int f = ok ? S.fc[u] : 1, s = ok ? S.sc[u] : 0;
            S.ef[u] = glb(P.energy)[f]; S.es[u] = glb(P.energy)[s];
            S.gf[u] = glb(P.g)[f]; S.gs[u] = glb(P.g)[s];
#pragma unroll
            for (int k = 0; k < NS; k++) {
                int tb = (k < NT) ? sm.ttab[S.cls[u]][k] : sm.tet[S.cls[u]];
                tb = tb < 0 ? 0 : tb;
                const int64_t pcc = S.pc[u] < 0 ? 0 : S.pc[u] < sm.timax[tb] ? S.pc[u] : sm.timax[tb] - 1;
                S.c0[u][k] = glb(sm.tcol[tb])[pcc];
                S.c1[u][k] = glb(sm.tder[tb])[pcc];      // slope (calc_coeff_deriv)
            }
        }
    };
    auto eval_store = [&](const Stage &S) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < PU; u++) {
            const int cl = S.cls[u], f = S.fc[u], s = S.sc[u];
            const int grp = sm.tgrp[cl];
            double dn = 0., gsum = 0.;
            int ng = 0;
#pragma unroll
            for (int k = 0; k < NT; k++) {
                const int tb = sm.ttab[cl][k];
                if (tb < 0) break;
                const double r = (S.c0[u][k] + S.c1[u][k] * sm.tx[tb]) * sm.cc[sm.tcombo[cl][k]];   // get_rate
                if (k < grp) dn = (k == 0) ? r : dn + r;
                else { gsum = (ng == 0) ? r : gsum + r; ng++; }
            }
            if (ng) dn = dn + gsum;
            const double de = S.es[u] - S.ef[u];
            double un = 0.;
            if (dn > MIN_COLLISION_RATE) un = dn * lvg_exp(de * CM_INVERSE_TO_KELVINS / T) * S.gf[u] / S.gs[u];
            else dn = 0.;
            double dE = 0., uE = 0.;
            if (HE) {
                const int et = sm.tet[cl];
                if (et >= 0 && electrons) {
                    dE = (S.c0[u][NS - 1] + S.c1[u][NS - 1] * sm.tx[et]) * sm.ne;
                    if (dE > MIN_COLLISION_RATE) uE = dE * lvg_exp(de * CM_INVERSE_TO_KELVINS / Te) * S.gf[u] / S.gs[u];
                    else dE = 0.;
                }
            }
            const bool ok = S.pc[u] >= 0;
            Kg[ok ? (int64_t)s * N + f : 0] = dn + dE;
            Kg[ok ? (int64_t)f * N + s : 0] = un + uE;
        }
    };
    Stage A, B;
    constexpr int STEP = PU * TG;
    issue(A, 0);
    for (int q0 = 0; q0 < ntiles; q0 += 2 * STEP) {
        issue(B, q0 + STEP);
        eval_store(A);
        if (q0 + 2 * STEP < ntiles) issue(A, q0 + 2 * STEP);
        if (q0 + STEP < ntiles) eval_store(B);
    }
}

// ------------------------------------------------------------------------------
// radiative terms: intensity_calc (iteration_lvg.cpp:163-185, :428-501)
// ------------------------------------------------------------------------------
template <class SM>
__device__ __forceinline__ double dust_opacity(const LvgDevProblem &P, const LvgModeLines &M, const SM &sm, int n) {
    double a = 0.;
    for (int c = 0; c < P.nb_comp; c++) a += M.line_sigma[(int64_t)c * M.nb_lines + n] * sm.dust[c];
    return a;
}

template <class SM>
__device__ __forceinline__ double intensity_single(const LvgDevProblem &P, const EscGrids &G, const LvgModeLines &M,
                                                   const SM &sm, int n, const double *pop) {
    const int u = M.line_u[n], l = M.line_l[n];
    const double energy = M.line_e[n];
    const double c = sm.nmol / (EIGHT_PI * sm.vw * energy * energy * energy);
    const double emiss = c * M.line_aul[n] * pop[u];
    double opac = c * M.line_alu[n] * pop[l] - emiss + MIN_LINE_OPACITY;
    if (opac < 0.) opac *= INV_TRANS_FACTOR;
    const double dop = dust_opacity(P, M, sm, n);
    const double gamma = fabs(sm.vgrad) / (sm.vw * opac);
    const double delta = fabs(sm.vgrad) / (sm.vw * dop);
    return emiss / opac * esc_func(P, G, gamma, delta);
}

template <class SM>
__device__ __forceinline__ void intensity_pair(const LvgDevProblem &P, const EscGrids &G, const LvgModeLines &M,
                                               const SM &sm, int n1, int n2, const double *pop, double &i1, double &i2) {
    const double max_dx = 4.;
    const int u1 = M.line_u[n1], l1 = M.line_l[n1], u2 = M.line_u[n2], l2 = M.line_l[n2];
    const double energy = M.line_e[n1];
    double c = sm.nmol / (EIGHT_PI * sm.vw * energy * energy * energy);
    const double em1 = c * M.line_aul[n1] * pop[u1];
    double op1 = c * (M.line_alu[n1] * pop[l1] - M.line_aul[n1] * pop[u1]) + MIN_LINE_OPACITY;
    const double em2 = c * M.line_aul[n2] * pop[u2];
    double op2 = c * (M.line_alu[n2] * pop[l2] - M.line_aul[n2] * pop[u2]) + MIN_LINE_OPACITY;
    if (op1 < 0.) op1 *= INV_TRANS_FACTOR;
    if (op2 < 0.) op2 *= INV_TRANS_FACTOR;
    const double g1 = fabs(sm.vgrad) / (sm.vw * op1), g2 = fabs(sm.vgrad) / (sm.vw * op2);
    const double delta = fabs(sm.vgrad) / (sm.vw * dust_opacity(P, M, sm, n1));
    double dx = (P.energy[u1] - P.energy[l1] - P.energy[u2] + P.energy[l2]) * SPEED_OF_LIGHT / (energy * sm.vw);
    if (sm.vgrad < 0.) dx *= -1.;
    double ep1 = 0., ep2 = 0., ep01 = 0., ep02 = 0.;
    if (fabs(dx) < max_dx) {
        ep1 = overlap_esc_func(P, G, P.ov_p1, g1, delta, g2 / g1, dx);
        ep2 = overlap_esc_func(P, G, P.ov_p1, g2, delta, g1 / g2, -dx);
    }
    if (fabs(dx) > max_dx - 0.5) {
        ep01 = esc_func(P, G, g1, delta);
        ep02 = esc_func(P, G, g2, delta);
    }
    if (fabs(dx) > max_dx) { ep1 = ep01; ep2 = ep02; }
    else if (fabs(dx) > max_dx - 0.5) {
        c = 2. * (max_dx - fabs(dx));
        ep1 = ep01 * (1. - c) + ep1 * c;
        ep2 = ep02 * (1. - c) + ep2 * c;
    }
    i1 = em1 / op1 * ep1;
    i2 = em2 / op2 * ep2;
    if (fabs(dx) < max_dx) {
        ep1 = overlap_esc_func(P, G, P.ov_p2, g1, delta, g2 / g1, dx);
        ep2 = overlap_esc_func(P, G, P.ov_p2, g2, delta, g1 / g2, -dx);
        if (fabs(dx) > max_dx - 0.5) {
            c = 2. * (max_dx - fabs(dx));
            ep1 *= c; ep2 *= c;
        }
        i1 += em2 / op2 * ep1;
        i2 += em1 / op1 * ep2;
    }
}

// ------------------------------------------------------------------------------
// iteration_control state (iteration_control.h:84-242) and the slot workspace
// ------------------------------------------------------------------------------
struct Ctl {
    int acceleration, accel_start, accel_period, nb_prev, max_iter;
    int iter_nb, nb_after_accel;
    double best_eq, eq_error, pop_error, rel_error;
    int hp, np, hr, nr;   // ring heads and sizes: prev_level_pop / residual_list
};

struct Slot {
    double *K, *A, *prev, *res, *opt, *y, *given, *df;
};

// A value every lane holds alike, read back from LDS: as a scalar (v_readfirstlane), so that
// the compiler keeps it in SGPRs and branches on it stay uniform (an LDS load is a VGPR, which
// the compiler must treat as divergent).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double uni(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}

__device__ __forceinline__ double *ring(double *base, int head, int i, int N) {
    return base + (int64_t)((head + i) & (NHIST - 1)) * N;
}

__device__ __forceinline__ Slot make_slot(const LvgDevProblem &P, const LvgLaunch &Lc, int slot) {
    const int N = P.N;
    double *w = Lc.ws + (int64_t)slot * Lc.ws_stride;
    Slot S;
    S.K = w; w += (int64_t)N * N;
    S.A = w; w += (int64_t)N * N;
    S.prev = w; w += (int64_t)NHIST * N;
    S.res = w; w += (int64_t)NHIST * N;
    S.opt = w; w += N;
    S.given = w; w += N;
    S.df = w; w += N;
    S.y = w;
    return S;
}

// the 4x4 (np x np) system of accel_step solved by one thread exactly as
// oracle_lu_solve does (iteration_control.h:176): hist_acc[0..np*np) = A, [np*np..) = b;
// the solution goes to hist_acc[16 + i], its sum to hist_acc[31]
__device__ __forceinline__ void accel_solve_small(double *hist_acc, int np) {
    // registers with compile-time indices only (np <= 4): no stack array, no scratch; the
    // row swap is a select over the candidate rows, the arithmetic that of the loops over np
    double Am[4][4], bv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j < 4; j++) Am[i][j] = (i < np && j < np) ? hist_acc[i * np + j] : 0.;
        bv[i] = (i < np) ? hist_acc[np * np + i] : 0.;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < np) {
            int p = k;
            double amax = fabs(Am[k][k]);
#pragma unroll
            for (int i = k + 1; i < 4; i++)
                if (i < np && fabs(Am[i][k]) > amax) { amax = fabs(Am[i][k]); p = i; }
#pragma unroll
            for (int i = k + 1; i < 4; i++) {
                if (i == p) {
#pragma unroll
                    for (int j = 0; j < 4; j++) { double x = Am[k][j]; Am[k][j] = Am[i][j]; Am[i][j] = x; }
                    double x = bv[k]; bv[k] = bv[i]; bv[i] = x;
                }
            }
            double piv = Am[k][k];
#pragma unroll
            for (int i = k + 1; i < 4; i++) {
                if (i < np) {
                    double l = Am[i][k] / piv;
                    Am[i][k] = l;
#pragma unroll
                    for (int j = k + 1; j < 4; j++) if (j < np) Am[i][j] = fma(-l, Am[k][j], Am[i][j]);
                    bv[i] = fma(-l, bv[k], bv[i]);
                }
            }
        }
    }
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        if (k < np) {
            bv[k] /= Am[k][k];
            double x = bv[k];
#pragma unroll
            for (int i = 0; i < k; i++) bv[i] = fma(-Am[i][k], x, bv[i]);
        }
    }
    double sum = 0.;
#pragma unroll
    for (int i = 0; i < 4; i++) if (i < np) { sum = sum + bv[i]; hist_acc[16 + i] = bv[i]; }
    hist_acc[31] = sum;
}
