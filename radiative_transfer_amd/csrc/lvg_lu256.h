// lvg_lu256.h — the LU of calc_new_pop / boundary_layer_populations for N <= 256 (the
// 256-thread solve_kernel), included by lvg_kernels.hip inside namespace lvg.
//
// lu_matrix_solve (absent library; call sites iteration_lvg.cpp:100, iteration_control.cpp:87)
// as a left-looking blocked LU with partial pivoting, b eliminated alongside, in which
// every wave OWNS COLUMNS:
//  * Block columns of 64; wave w holds columns c0 + 16w .. c0 + 16w + 15 of every row in
//    registers: lane l keeps tile rows 64 s + l (s < 4, logical order as of the block
//    load), acc[s][0..16) — 128 fp64 registers.
//  * An earlier chunk kk (16 columns of L, final) is staged once per workgroup into LDS
//    by tile row (Lst[m][row]); each wave then solves the chunk's 16 pivot rows in ITS
//    columns (TRSM against L11 in a 4 x 16-lane layout, DPP row broadcasts) and updates
//    its rows below with L (LDS) and U (its own LDS rows, broadcast reads). The waves do
//    identical work, so the two barriers of a step cost little; rows above the chunk
//    drop out in whole 64-row slots, for every wave alike.
//  * The block's own chunks are factored by the wave that owns them, alone in its
//    registers (pivot by DPP max over 4 rows per lane + ballot, pivot row by readlane):
//    no barrier per column. Its L is published through the same LDS stage, and the
//    waves to its right apply it (TRSM + update) while the next owner factors.
//  * The residual df = e0 - A n of the fused assembly runs row by row in column order,
//    handed from wave to wave through LDS (one barrier per wave per block column).
// Every element receives fma(-l_ik, u_kj, a_ij) for k ascending and the pivots are chosen
// from identical values with the oracle's rule (largest |v|, first maximum in logical
// order, NaN diagonal kept), so the factors, the solution and the residual equal the
// unblocked, physically pivoting oracle_lu_solve bit for bit. On return sm.blog holds x.
// b: LDS [N] indexed by physical row.

constexpr int S4 = NMAX / 64;   // row slots per lane: tile row 64 s + lane
constexpr int CW = LU_CW;       // columns per wave = chunk (panel) width: 16 or 8
constexpr int BW = 4 * CW;      // block-column width
constexpr int CL = CW / 4;      // TRSM columns per lane (4 x 16-lane rows)
static_assert(CW == 16 || CW == 8, "chunk width");
#ifndef LU2_PREFETCH
#define LU2_PREFETCH 0          // 1: next earlier chunk's L loaded into registers during this one (slower)
#endif
#ifndef LU2_UHALF
#define LU2_UHALF 0             // the rank-CW update in two column halves (fewer live U registers)
#endif
#ifndef LU2_PANEL
#define LU2_PANEL 1             // 1: masked rows, register select + v_readlane; 2: unmasked, pivot rows saved to LDS
#endif
#ifndef LU2_LIGHTBAR
#define LU2_LIGHTBAR 0          // 1: LU barriers wait for LDS only (lgkmcnt), not for global accesses (measured slower)
#endif
#ifndef LU2_BSUB_WAVE
#define LU2_BSUB_WAVE 0         // 1: back substitution by one wave without barriers (measured slower)
#endif
#ifndef LU2_PRIO
#define LU2_PRIO 0               // 1: panels (the critical path) at raised wave priority (measured slower)
#endif
#ifndef LU2_SLOT_FENCE
#define LU2_SLOT_FENCE 0        // block load: one 64-row slot's loads in flight at a time
#endif

// LDS stores of one lane visible to the other lanes of its wave: a wave's LDS instructions
// execute in issue order, so only compiler motion has to be stopped (wavefront-scope
// fences emit no wait; a workgroup-scope fence would also wait for the wave's global
// stores and prefetch loads, vmcnt(0))
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs only: lgkmcnt(0) + s_barrier. __syncthreads() also
// waits for every outstanding global access of the wave (vmcnt(0)), which would drain the
// next chunk's L prefetch and the U / L stores at every step. Global data written inside
// the LU is read by another wave only after that wave's own waits and a full barrier
// (next block's L fetch, back substitution).
__device__ __forceinline__ void lds_barrier() {
    if (!LU2_LIGHTBAR) { __syncthreads(); return; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0); vmcnt, expcnt untouched
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One chunk applied to this wave's columns: the chunk's pivot rows (tile rows kk.. for an
// earlier chunk, the rows whose logical position is kk.. for one of this block) published
// by their owner lanes to Ub[w], solved against L11 (x_r takes its updates for m ascending,
// x_m broadcast within the 16-lane row by DPP row_share), written back as U rows and
// stored to A; then the rows of slots >= s_lo updated with Lst (0 where a row takes no
// update) and those U rows, m ascending.
__device__ __forceinline__ void lu2_apply(double (&acc)[S4][CW], const int (&prow)[S4], bool earlier, int kk, int nb,
                                          int s_lo, int cw0, int nw, double *A, int N, Smem &sm, bool critical = false) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    double (*Ub)[CW] = sm.Ub[w];
    if (LU2_PRIO && critical) __builtin_amdgcn_s_setprio(2);
    TSTAMP(ta0);
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + l;
        if (r < N) {
            const int q = (earlier ? r : sm.pos[prow[s]]) - kk;
            if (q >= 0 && q < nb) {
                double2 *d = reinterpret_cast<double2 *>(&Ub[q][0]);
#pragma unroll
                for (int j = 0; j < CW / 2; j++) d[j] = make_double2(acc[s][2 * j], acc[s][2 * j + 1]);
            }
        }
    }
    wave_lds_sync();
    {
        const int q4 = l >> 4, r = l & 15;        // lane: row r of the chunk, columns CL*q4..
        double x[CL];
        if (r < CW) {
#pragma unroll
            for (int i = 0; i < CL; i++) x[i] = Ub[r][CL * q4 + i];
        }
        const double *lrw = sm.L11[r < CW ? r : 0];
#define LVG_TRSM_STEP(M_)                                                                  \
        if ((M_) < nb - 1) {                                                               \
            const double lm = lrw[M_];                                                     \
            _Pragma("unroll") for (int i = 0; i < CL; i++) {                               \
                const double y = dpp_d<0x150 + (M_), 0xf, 0xf>(x[i]);                      \
                if (r > (M_)) x[i] = fma(-lm, y, x[i]);                                    \
            }                                                                              \
        }
        LVG_TRSM_STEP(0) LVG_TRSM_STEP(1) LVG_TRSM_STEP(2) LVG_TRSM_STEP(3)
        LVG_TRSM_STEP(4) LVG_TRSM_STEP(5) LVG_TRSM_STEP(6)
        if (CW == 16) {
            LVG_TRSM_STEP(7) LVG_TRSM_STEP(8) LVG_TRSM_STEP(9) LVG_TRSM_STEP(10)
            LVG_TRSM_STEP(11) LVG_TRSM_STEP(12) LVG_TRSM_STEP(13) LVG_TRSM_STEP(14)
        }
#undef LVG_TRSM_STEP
        if (r < nb) {
#pragma unroll
            for (int i = 0; i < CL; i++) Ub[r][CL * q4 + i] = x[i];
            double *urow = A + (int64_t)sm.perm[kk + r] * N + cw0 + CL * q4;
#pragma unroll
            for (int i = 0; i < CL; i++) if (CL * q4 + i < nw) urow[i] = x[i];
        }
    }
    wave_lds_sync();
    TACC(PH_T_SOLVE, ta0);
    TSTAMP(tg0);
    constexpr int UH = LU2_UHALF ? CW / 2 : CW;          // U columns per pass
    for (int m = 0; m < nb; m++) {
#pragma unroll
        for (int h = 0; h < CW; h += UH) {
            double u[UH];
            const double2 *up = reinterpret_cast<const double2 *>(&Ub[m][h]);
#pragma unroll
            for (int j = 0; j < UH / 2; j++) { const double2 v = up[j]; u[2 * j] = v.x; u[2 * j + 1] = v.y; }
#pragma unroll
            for (int s = 0; s < S4; s++) {
                if (s >= s_lo) {
                    const double a = sm.pu.Lst[m][64 * s + l];
#pragma unroll
                    for (int c = 0; c < UH; c++) acc[s][h + c] = fma(-a, u[c], acc[s][h + c]);
                }
            }
        }
    }
    if (LU2_PRIO && critical) __builtin_amdgcn_s_setprio(0);
    TACC(PH_GEMM, tg0);
}

// The chunk kk (this wave's CW columns) factored by this wave alone: rows of slots >= s_lo
// whose logical position is >= kk take part, 4 rows per lane. Per column: the lane's best
// key over its rows, one DPP wave max (+ ballot; lower word and position only on a tie)
// for the pivot, the pivot row through the wave's LDS row (written by the pivot lane, read
// back by all), one division and the row update per active row, b eliminated alongside
// (b[p], LDS by physical row). Look-ahead: column c+1 is updated first and its key
// reduction issued before the rest of column c's update, so the two overlap. The wave
// runs at raised priority: it is the critical path while the co-resident workgroup
// streams its updates.
template <int NS>
__device__ __forceinline__ void lu2_best_key(const double (&acc)[S4][CW], const bool (&act)[S4], const int (&lp)[S4],
                                             int c, unsigned &bh, unsigned &bl, int &bp, int &bs) {
    bh = 0u; bl = 0u; bp = 0x7fffffff; bs = 0;
#pragma unroll
    for (int s = S4 - NS; s < S4; s++) {
        unsigned hi, lo;
        pivot_key(acc[s][c], act[s], lp[s] == c, hi, lo);
        const bool better = hi > bh || (hi == bh && (lo > bl || (lo == bl && (unsigned)lp[s] < (unsigned)bp)));
        bh = better ? hi : bh;
        bl = better ? lo : bl;
        bp = better ? lp[s] : bp;
        bs = better ? s : bs;
    }
}

// NS = active slots (the top NS slots: tile rows >= c0 = 64 (4 - NS)). Each pivot row is
// final when chosen (its multipliers left of c, its U values from c on, its b): the pivot
// lane saves it to Prow[c] (LDS), every lane reads the row back as the broadcast, and the
// publish takes the chunk's pivot rows from there. So the row updates need no mask: rows
// no longer active get the multiplier 0 and whatever lands in their registers is never
// read again (their values were saved, or are final U values already stored).
template <int NS>
__device__ __forceinline__ void lu2_panel_ns(double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb, int N,
                                             const double *b, bool (&part)[S4], int (&lp)[S4], double (&rb)[S4],
                                             Smem &sm) {
    const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
    double (*Prow)[CW] = sm.Ub[w];
    double *Pb = sm.Pb[w];
    bool act[S4];
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + ln;
        const bool valid = s >= S4 - NS && r < N;
        const int p = valid ? prow[s] : 0;
        const int ps = sm.pos[p];
        part[s] = valid && ps >= kk;
        act[s] = part[s];
        lp[s] = part[s] ? ps - kk : 0x7fffffff;
        rb[s] = b[p];
    }
    unsigned bh, bl, H;
    int bp, bs;
    lu2_best_key<NS>(acc, act, lp, 0, bh, bl, bp, bs);
    H = wave_max_u32(bh);
#pragma clang loop unroll(full)
    for (int c = 0; c < CW; c++) {
        if (c < nb) {
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
            const int ss = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bs, pl));
            const int plp = __builtin_amdgcn_readlane(bp, pl);
            // the pivot row (final: multipliers, U values, b) saved by its lane to Prow[c]
            if (ln == pl) {
                // one branch per slot, each with an opaque barrier: otherwise the compiler
                // folds the chain into acc[ss][j] and moves acc to scratch memory
#pragma unroll
                for (int s = S4 - NS; s < S4; s++) {
                    if (ss == s) {
                        asm volatile("" ::: "memory");
#pragma unroll
                        for (int j = 0; j < CW; j++) Prow[c][j] = acc[s][j];
                        Pb[c] = rb[s];
                    }
                }
            }
            wave_lds_sync();
            double pr[CW];
#pragma unroll
            for (int j = 0; j < CW; j++) if (j >= c) pr[j] = Prow[c][j];
            const double bc = Pb[c];
            const double piv = pr[c];
            double lv[S4];
#pragma unroll
            for (int s = S4 - NS; s < S4; s++) {
                const bool me = ln == pl && s == ss;
                act[s] = act[s] && !me;
                lp[s] = me ? c : (lp[s] == c ? plp : lp[s]);
                const double q = acc[s][c] / piv;
                lv[s] = act[s] ? q : 0.;
                if (c + 1 < CW) acc[s][c + 1] = fma(-lv[s], pr[c + 1], acc[s][c + 1]);
            }
            if (c + 1 < nb) {                      // look-ahead: the next column's pivot reduction
                lu2_best_key<NS>(acc, act, lp, c + 1, bh, bl, bp, bs);
                H = wave_max_u32(bh);
            }
#pragma unroll
            for (int s = S4 - NS; s < S4; s++) {
                acc[s][c] = lv[s];
#pragma unroll
                for (int j = 0; j < CW; j++) if (j > c + 1) acc[s][j] = fma(-lv[s], pr[j], acc[s][j]);
                rb[s] = fma(-lv[s], bc, rb[s]);
            }
        }
    }
}

// LU2_PANEL 1: rows under exec masks (if act), the pivot row selected from the lane's slots
// in registers and broadcast by v_readlane; b and the pivot rows stay in the registers.
__device__ __forceinline__ void lu2_panel_v1(double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb, int s_lo,
                                             int N, const double *b, bool (&part)[S4], int (&lp)[S4],
                                             double (&rb)[S4], Smem &sm) {
    const int ln = threadIdx.x & 63;
    bool act[S4];
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + ln;
        const bool valid = s >= s_lo && r < N;
        const int p = valid ? prow[s] : 0;
        const int ps = sm.pos[p];
        part[s] = valid && ps >= kk;
        act[s] = part[s];
        lp[s] = part[s] ? ps - kk : 0x7fffffff;
        rb[s] = b[p];
    }
#pragma clang loop unroll(full)
    for (int c = 0; c < CW; c++) {
        if (c < nb) {
            unsigned bh = 0u, bl = 0u;
            int bp = 0x7fffffff, bs = 0;
#pragma unroll
            for (int s = 0; s < S4; s++) {
                if (s >= s_lo) {
                    unsigned hi, lo;
                    pivot_key(acc[s][c], act[s], lp[s] == c, hi, lo);
                    const bool better = hi > bh || (hi == bh && (lo > bl || (lo == bl && (unsigned)lp[s] < (unsigned)bp)));
                    bh = better ? hi : bh;
                    bl = better ? lo : bl;
                    bp = better ? lp[s] : bp;
                    bs = better ? s : bs;
                }
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
            const int ss = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bs, pl));
            const int plp = __builtin_amdgcn_readlane(bp, pl);
            double pr[CW], bc;
            {
                double sv[CW], sb = rb[0];
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) sv[j] = acc[0][j];
#pragma unroll
                for (int s = 1; s < S4; s++) {
                    const bool pick = ss == s;
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j >= c) sv[j] = pick ? acc[s][j] : sv[j];
                    sb = pick ? rb[s] : sb;
                }
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) pr[j] = readlane_d(sv[j], pl);
                bc = readlane_d(sb, pl);
            }
            const double piv = pr[c];
#pragma unroll
            for (int s = 0; s < S4; s++) {
                if (s >= s_lo) {
                    if (ln == pl && s == ss) { act[s] = false; lp[s] = c; }
                    else if (lp[s] == c) lp[s] = plp;
                    if (act[s]) {
                        const double lv = acc[s][c] / piv;
                        acc[s][c] = lv;
#pragma unroll
                        for (int j = 0; j < CW; j++) if (j > c) acc[s][j] = fma(-lv, pr[j], acc[s][j]);
                        rb[s] = fma(-lv, bc, rb[s]);
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ void lu2_panel(double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb, int s_lo,
                                          int N, const double *b, bool (&part)[S4], int (&lp)[S4],
                                          double (&rb)[S4], Smem &sm) {
    if (LU2_PRIO) __builtin_amdgcn_s_setprio(2);
    if (LU2_PANEL == 1) lu2_panel_v1(acc, prow, kk, nb, s_lo, N, b, part, lp, rb, sm);
    else lu2_panel_ns<S4>(acc, prow, kk, nb, N, b, part, lp, rb, sm);
    if (LU2_PRIO) __builtin_amdgcn_s_setprio(0);
}

// The factored chunk's rows (logical position >= kk) to A (L below the pivots; the pivot
// rows, saved at pivot time, with L11 and U), perm/pos/b, L11 (strictly lower) and the
// stage Lst (L of the rows below the chunk, 0 for the others) for the waves to its right.
__device__ __forceinline__ void lu2_publish(const double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb,
                                            int s_lo, double *A, int N, double *b, const bool (&part)[S4],
                                            const int (&lp)[S4], const double (&rb)[S4], Smem &sm) {
    const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double (*Prow)[CW] = sm.Ub[w];
    const double *Pb = sm.Pb[w];
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + ln;
        if (s < s_lo || r >= N) continue;
        if (part[s]) {
            const int p = prow[s], q = lp[s];
            const bool piv = q < nb;
            const bool saved = LU2_PANEL != 1 && piv;     // panel 2 saved its pivot rows at pivot time
            double v[CW];
#pragma unroll
            for (int j = 0; j < CW; j++) v[j] = saved ? Prow[q < nb ? q : 0][j] : acc[s][j];
            if ((N & 1) == 0 && nb == CW) {
                double2 *d2 = reinterpret_cast<double2 *>(A + (int64_t)p * N + kk);
#pragma unroll
                for (int j = 0; j < CW / 2; j++) d2[j] = make_double2(v[2 * j], v[2 * j + 1]);
            } else {
#pragma unroll
                for (int j = 0; j < CW; j++) if (j < nb) A[(int64_t)p * N + kk + j] = v[j];
            }
            sm.perm[kk + q] = p;
            sm.pos[p] = kk + q;
            b[p] = saved ? Pb[q < nb ? q : 0] : rb[s];
            if (piv) {
#pragma unroll
                for (int m = 0; m < CW; m++) { sm.L11[q][m] = m < q ? v[m] : 0.; sm.pu.Lst[m][r] = 0.; }
            } else {
#pragma unroll
                for (int m = 0; m < CW; m++) sm.pu.Lst[m][r] = m < nb ? v[m] : 0.;
            }
        } else {
#pragma unroll
            for (int m = 0; m < CW; m++) sm.pu.Lst[m][r] = 0.;
        }
    }
}

// L of earlier chunk kk for tile row t (= logical row t: the pivots of earlier blocks are
// final at this block's load): the row's 16 values from A when t >= kk, else zeros
__device__ __forceinline__ void lu2_fetch_l(const double *A, int N, int kk, int trow, double (&pf)[CW]) {
    const int t = threadIdx.x;
    const bool need = t < N && t >= kk;
    const double *src = A + (int64_t)(need ? trow : 0) * N + kk;
    if ((N & 1) == 0) {
        const double2 *s2 = reinterpret_cast<const double2 *>(src);
#pragma unroll
        for (int j = 0; j < CW / 2; j++) {
            const double2 v = need ? s2[j] : make_double2(0., 0.);
            pf[2 * j] = v.x;
            pf[2 * j + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < CW; j++) pf[j] = need ? src[j] : 0.;
    }
}

// ... into the stage: rows below the chunk keep their 16 values; the chunk's own rows go
// to L11 (strictly lower part) and stage zeros, as do the rows above
__device__ __forceinline__ void lu2_stage_l(int N, int kk, const double (&pf)[CW], Smem &sm) {
    const int t = threadIdx.x;
    if (t >= N) return;
    if (t >= kk + CW) {
#pragma unroll
        for (int m = 0; m < CW; m++) sm.pu.Lst[m][t] = pf[m];
    } else {
        if (t >= kk) {
            const int q = t - kk;
#pragma unroll
            for (int m = 0; m < CW; m++) sm.L11[q][m] = m < q ? pf[m] : 0.;
        }
#pragma unroll
        for (int m = 0; m < CW; m++) sm.pu.Lst[m][t] = 0.;
    }
}

// Back substitution U x = y (y_k = b[perm[k]]) by wave 0 alone, no barrier: lane l keeps
// the right-hand sides of logical rows 64 s + l. Blocks of 16 from the bottom: the block's
// 16 rows (one 16-lane DPP row of slot k0/64) solve their triangle (x_M = b_M / U_MM,
// broadcast by DPP row_share, b_r = fma(-U_rM, x_M, b_r) for M descending), then every row
// above takes fma(-U_im, x_m, b_i) for m descending, x_m from v_readlane. The same
// operations in the same order as back_substitute (k descending per entry). On return
// (after the caller's barrier) sm.blog holds x.
__device__ __forceinline__ void back_substitute_wave(const double *A, int N, const double *b, Smem &sm) {
    if ((__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) != 0) return;
    TSTAMP(tb0);
    const int l = threadIdx.x & 63, r = l & 15;
    double bv[S4];
    int prw[S4];
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int i = 64 * s + l;
        prw[s] = i < N ? sm.perm[i] : 0;
        bv[s] = i < N ? b[prw[s]] : 0.;
    }
    const int nblk = (N + NB - 1) / NB;
    for (int kb = nblk - 1; kb >= 0; kb--) {
        const int k0 = kb * NB, nb = min(NB, N - k0), sd = k0 >> 6, rl = k0 & 63;
        // U row segments [k0, k0 + 16) of this lane's rows at or above the block
        double u[S4][NB];
#pragma unroll
        for (int s = 0; s < S4; s++) {
            if (s <= sd) {
                const int i = 64 * s + l;
                const bool ok = i < k0 + nb;
                const double *row = A + (int64_t)(ok ? prw[s] : 0) * N + k0;
                if ((N & 1) == 0 && nb == NB) {
                    const double2 *r2 = reinterpret_cast<const double2 *>(row);
#pragma unroll
                    for (int m = 0; m < NB / 2; m++) {
                        const double2 v = ok ? r2[m] : make_double2(0., 0.);
                        u[s][2 * m] = v.x;
                        u[s][2 * m + 1] = v.y;
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < NB; m++) u[s][m] = (ok && m < nb) ? row[m] : 0.;
                }
            }
        }
        // the block's triangle: its rows are lanes rl..rl+nb-1 of slot sd
        double bt = bv[0], ur[NB];
#pragma unroll
        for (int m = 0; m < NB; m++) ur[m] = u[0][m];
#pragma unroll
        for (int s = 1; s < S4; s++) {
            if (sd == s) {
                bt = bv[s];
#pragma unroll
                for (int m = 0; m < NB; m++) ur[m] = u[s][m];
            }
        }
        const bool inblk = l >= rl && l < rl + nb;
        if (!inblk) {
#pragma unroll
            for (int m = 0; m < NB; m++) ur[m] = 1.;
        }
#define LVG_BSUB_STEP(M_)                                                                  \
        if ((M_) < nb) {                                                                   \
            const double xm = dpp_d<0x150 + (M_), 0xf, 0xf>(bt / ur[M_]);                  \
            if (r < (M_)) bt = fma(-ur[M_], xm, bt);                                       \
            else if (r == (M_)) bt = xm;                                                   \
        }
        LVG_BSUB_STEP(15) LVG_BSUB_STEP(14) LVG_BSUB_STEP(13) LVG_BSUB_STEP(12)
        LVG_BSUB_STEP(11) LVG_BSUB_STEP(10) LVG_BSUB_STEP(9) LVG_BSUB_STEP(8)
        LVG_BSUB_STEP(7) LVG_BSUB_STEP(6) LVG_BSUB_STEP(5) LVG_BSUB_STEP(4)
        LVG_BSUB_STEP(3) LVG_BSUB_STEP(2) LVG_BSUB_STEP(1) LVG_BSUB_STEP(0)
#undef LVG_BSUB_STEP
#pragma unroll
        for (int s = 0; s < S4; s++) if (sd == s && inblk) bv[s] = bt;
        // rows above the block
        double xk[NB];
#pragma unroll
        for (int m = 0; m < NB; m++) xk[m] = readlane_d(bt, rl + m);
#pragma unroll
        for (int s = 0; s < S4; s++) {
            if (s <= sd) {
                const int i = 64 * s + l;
                if (i < k0) {
#pragma unroll
                    for (int m = NB - 1; m >= 0; m--)
                        if (m < nb) bv[s] = fma(-u[s][m], xk[m], bv[s]);
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int i = 64 * s + l;
        if (i < N) sm.blog[i] = bv[s];
    }
    TACC(PH_BACKSUB, tb0);
}

__device__ __forceinline__ double block_lu_solve(double *A, int N, double *b, Smem &sm, const LuSrc &src, const bool FUSED) {
    const int t = threadIdx.x;
    for (int i = t; i < N; i += BT) {
        sm.perm[i] = i;
        sm.pos[i] = i;
        if (FUSED) sm.resid[i] = (i == 0) ? 1. : 0.;
    }
    __syncthreads();
    const int l = t & 63, w = t >> 6;
    for (int c0 = 0; c0 < N; c0 += BW) {
        const int SLO = c0 >> 6;                  // slots above this block's rows hold earlier pivots
        TSTAMP(tp0);
        const int wJ = min(BW, N - c0);
        const int cw0 = c0 + CW * w;                  // this wave's first column
        const int nw = max(0, min(CW, wJ - CW * w));  // ... and how many it has
        int prow[S4];                                 // physical row of tile row 64 s + l
#pragma unroll
        for (int s = 0; s < S4; s++) prow[s] = (64 * s + l < N) ? sm.perm[64 * s + l] : 0;
        const int trow = (t < N) ? sm.perm[t] : 0;    // physical row of tile row t (L fetch)
        double acc[S4][CW];
        // ---- this wave's columns of the block into registers (fused: assembled from K,
        //      the line terms and the diagonal, row 0 <- 1)
#pragma unroll
        for (int s = 0; s < S4; s++) {
            const int r = 64 * s + l, pr = prow[s];
            const bool okr = r < N && nw > 0;
            if (!FUSED) {
#pragma unroll
                for (int j = 0; j < CW; j++) {
                    const int d = cw0 + j;
                    const bool ok = okr && j < nw;
                    double v;
                    if (src.BK) {
                        const double k = ok ? src.BK[(int64_t)pr * N + d] : 0.;
                        const double e = (ok && pr < d) ? src.BE[(int64_t)d * N + pr] : 0.;
                        const double dg = (ok && pr == d) ? src.BD[d] : 0.;
                        v = (pr < d) ? 0.5 * e + k : k;   // build_collision_operators: 0.5 * af + dn
                        if (pr == d) v = dg;
                        if (pr == 0) v = 1.;
                    } else {
                        v = ok ? (src.B ? src.B : A)[(int64_t)pr * N + d] : 0.;
                    }
                    acc[s][j] = ok ? v : 0.;
                }
            } else {
                int li[CW];
                const int64_t o = (int64_t)(okr ? pr : 0) * N + cw0;
                if ((N & 3) == 0 && nw == CW) {
                    const double2 *k2 = reinterpret_cast<const double2 *>(src.K + o);
                    const int4 *l4 = reinterpret_cast<const int4 *>(src.li + o);
#pragma unroll
                    for (int j = 0; j < CW / 2; j++) {
                        const double2 v = okr ? k2[j] : make_double2(0., 0.);
                        acc[s][2 * j] = v.x; acc[s][2 * j + 1] = v.y;
                    }
#pragma unroll
                    for (int j = 0; j < CW / 4; j++) {
                        const int4 v = okr ? l4[j] : make_int4(-1, -1, -1, -1);
                        li[4 * j] = v.x; li[4 * j + 1] = v.y; li[4 * j + 2] = v.z; li[4 * j + 3] = v.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < CW; j++) {
                        const bool ok = okr && j < nw;
                        acc[s][j] = ok ? src.K[o + j] : 0.;
                        li[j] = ok ? src.li[o + j] : -1;
                    }
                }
#pragma unroll
                for (int j = 0; j < CW; j++) {
                    const int d = cw0 + j;
                    double v = acc[s][j];
                    if (li[j] >= 0) v = v + src.y[li[j]];
                    if (pr == d) v = sm.diag[d < NMAX ? d : 0];
                    if (pr == 0) v = 1.;
                    acc[s][j] = (okr && j < nw) ? v : 0.;
                    if (src.dump && okr && j < nw) src.dump[(int64_t)pr * N + d] = v;
                }
            }
            if (LU2_SLOT_FENCE) __builtin_amdgcn_sched_barrier(0);   // one slot's loads in flight at a time
        }
        TACC(PH_BLOAD, tp0);
        TSTAMP(tr0);
        // ---- residual rows (physical), columns ascending: wave 0's columns, then wave 1's, ...
        if (FUSED) {
#pragma unroll
            for (int wq = 0; wq < NW; wq++) {
                if (w == wq && nw > 0) {
#pragma unroll
                    for (int s = 0; s < S4; s++) {
                        const int r = 64 * s + l;
                        if (r < N) {
                            double sr = sm.resid[prow[s]];
#pragma unroll
                            for (int j = 0; j < CW; j++) if (j < nw) sr = sr - acc[s][j] * src.pop[cw0 + j];
                            sm.resid[prow[s]] = sr;
                        }
                    }
                }
                lds_barrier();
            }
        } else {
            lds_barrier();
        }
        TACC(PH_RSV, tr0);
        // ---- earlier chunks: L staged by tile row (the next chunk's rows prefetched into
        //      registers during this one), two barriers a step
        if (c0 > 0) {
            double pf[CW];
            if (LU2_PREFETCH) lu2_fetch_l(A, N, 0, trow, pf);
            for (int kk = 0; kk < c0; kk += CW) {
                TSTAMP(tf0);
                if (!LU2_PREFETCH) lu2_fetch_l(A, N, kk, trow, pf);
                lu2_stage_l(N, kk, pf, sm);
                lds_barrier();
                TACC(PH_T_FETCH, tf0);
                if (LU2_PREFETCH && kk + CW < c0) lu2_fetch_l(A, N, kk + CW, trow, pf);
                if (nw > 0) lu2_apply(acc, prow, true, kk, CW, (kk + CW) >> 6, cw0, nw, A, N, sm);
                TSTAMP(tb0);
                lds_barrier();
                TACC(PH_TRSM, tb0);
            }
        }
        // ---- this block's chunks: owner factors, waves to its right apply
        bool part[S4];
        int lp[S4];
        double rb[S4];
        for (int wq = 0; wq < NW; wq++) {
            const int kk = c0 + CW * wq;
            if (kk >= N) break;
            const int nb = min(CW, N - kk);
            TSTAMP(tp1);
            if (w == wq) lu2_panel(acc, prow, kk, nb, SLO, N, b, part, lp, rb, sm);
            TACC(PH_PANEL, tp1);
            TSTAMP(tw0);
            lds_barrier();                       // the applies of the previous chunk are done
            if (w == wq) lu2_publish(acc, prow, kk, nb, SLO, A, N, b, part, lp, rb, sm);
            lds_barrier();
            TACC(PH_P_WB, tw0);
            if (w > wq && nw > 0) lu2_apply(acc, prow, false, kk, nb, SLO, cw0, nw, A, N, sm, w == wq + 1);
        }
    }
    __syncthreads();
    if (LU2_BSUB_WAVE) {
        back_substitute_wave(A, N, b, sm);
        __syncthreads();
    } else {
        back_substitute(A, N, b, sm);
    }
    double emax = 0.;
    if (FUSED && t < N) { const double r = sm.resid[t]; src.df[t] = r; emax = fabs(r); }
    return FUSED ? block_max(emax, sm) : 0.;
}
