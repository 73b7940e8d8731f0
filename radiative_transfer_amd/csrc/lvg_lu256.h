// lvg_lu256.h — the LU of calc_new_pop / boundary_layer_populations for N <= 256 (the
// 256-thread solve_kernel), included by lvg_kernels.hip inside namespace lvg.
//
// lu_matrix_solve (absent library; call sites iteration_lvg.cpp:100, iteration_control.cpp:87)
// as a left-looking blocked LU with partial pivoting, b eliminated alongside, in which
// every wave OWNS COLUMNS:
//  * Block columns of 16 x (waves): 64 for the 256-thread kernel, 128 for the 512-thread
//    one (LVG_WIDE); wave w holds columns c0 + 16w .. c0 + 16w + 15 of every row in
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
constexpr int BW = NW * CW;     // block-column width: 64 (4 waves) or 128 (8 waves, LVG_WIDE)
constexpr int CL = CW / 4;      // TRSM columns per lane (4 x 16-lane rows)
static_assert(CW == 16 || CW == 8, "chunk width: the TRSM lays 16 rows over 16-lane groups");

// LDS stores of one lane visible to the other lanes of its wave: a wave's LDS instructions
// execute in issue order, so only compiler motion has to be stopped (wavefront-scope
// fences emit no wait; a workgroup-scope fence would also wait for the wave's global
// stores and prefetch loads, vmcnt(0))
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#if !LVG_LU3
// One chunk applied to this wave's columns: the chunk's pivot rows (tile rows kk.. for an
// earlier chunk, the rows whose logical position is kk.. for one of this block) published
// by their owner lanes to Ub[w], solved against L11 (x_r takes its updates for m ascending,
// x_m broadcast within the 16-lane row by DPP row_share), written back as U rows and
// stored to A; then the rows of slots >= s_lo updated with Lst (0 where a row takes no
// update) and those U rows, m ascending.
__device__ __forceinline__ void lu2_apply(double (&acc)[S4][CW], const int (&prow)[S4], bool earlier, int kk, int nb,
                                          int s_lo, int cw0, int nw, double *A, int N, Smem &sm) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    double (*Ub)[CW] = sm.Ub[w];
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
        LVG_TRSM_STEP(4) LVG_TRSM_STEP(5) LVG_TRSM_STEP(6) LVG_TRSM_STEP(7)
        LVG_TRSM_STEP(8) LVG_TRSM_STEP(9) LVG_TRSM_STEP(10) LVG_TRSM_STEP(11)
        LVG_TRSM_STEP(12) LVG_TRSM_STEP(13) LVG_TRSM_STEP(14)
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
    for (int m = 0; m < nb; m++) {
        double u[CW];
        const double2 *up = reinterpret_cast<const double2 *>(&Ub[m][0]);
#pragma unroll
        for (int j = 0; j < CW / 2; j++) { const double2 v = up[j]; u[2 * j] = v.x; u[2 * j + 1] = v.y; }
        // every slot's L read with the U row (one LDS wait per m, not one per slot): the
        // asm use keeps the reads from being sunk into the slot branches
        double a[S4];
#pragma unroll
        for (int s = 0; s < S4; s++) a[s] = sm.pu.Lst[m][64 * s + l];
        static_assert(S4 == 4, "four row slots");
        asm volatile("" :: "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
#pragma unroll
        for (int s = 0; s < S4; s++) {
            if (s >= s_lo) {
#pragma unroll
                for (int c = 0; c < CW; c++) acc[s][c] = fma(-a[s], u[c], acc[s][c]);
            }
        }
    }
    TACC(PH_GEMM, tg0);
}

#endif

// The chunk kk (this wave's CW columns) factored by this wave alone: rows of slots >= s_lo
// whose logical position is >= kk take part (exec-masked), 4 rows per lane. Per column:
// the lane's best key over its rows, one DPP wave max + ballot (lower word and position
// only on a tie) for the pivot, the pivot row selected from the lane's slots in registers
// and broadcast by v_readlane, one division and the row update per active row, b
// eliminated alongside (b[p], LDS by physical row; kept in registers until the publish).
// The row select is a v_cndmask chain: written as branches on the (uniform) slot, or
// through LDS, the compiler folds it into a dynamic acc[ss] index and moves acc to
// scratch memory (measured: 352 -> 800 B/lane).
__device__ __forceinline__ void lu2_panel(double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb, int s_lo,
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
            // fast path: upper words only (|v|'s sign bit replaced by the active flag), the
            // lane's best of its slots, one wave max, one ballot per slot. It decides when
            // exactly one row carries the maximum upper word and that word is finite (an inf
            // or NaN among the active rows puts it at 0xfff00000 or above); a tie in the
            // upper word, an inf or a NaN takes the full key (lower word, then the first
            // logical position, NaN diagonal), so the pivot is the oracle's in every case.
            unsigned kh[S4];
#pragma unroll
            for (int s = 0; s < S4; s++)
                kh[s] = (s >= s_lo && act[s]) ? ((unsigned)__double2hiint(acc[s][c]) | 0x80000000u) : 0u;
            const unsigned H0 = wave_max_u32(max(max(kh[0], kh[1]), max(kh[2], kh[3])));
            unsigned long long mk[S4];
            int cnt = 0;
#pragma unroll
            for (int s = 0; s < S4; s++) { mk[s] = __ballot(kh[s] == H0); cnt += __popcll(mk[s]); }
            int pl, ss, plp;
            if (H0 < 0xfff00000u && cnt == 1) {
                ss = mk[0] ? 0 : mk[1] ? 1 : mk[2] ? 2 : 3;
                pl = __builtin_amdgcn_readfirstlane(__ffsll((long long)(mk[0] | mk[1] | mk[2] | mk[3])) - 1);
                int lps = lp[0];
#pragma unroll
                for (int s = 1; s < S4; s++) lps = ss == s ? lp[s] : lps;
                plp = __builtin_amdgcn_readlane(lps, pl);
            } else {
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
                if (__popcll(tie) == 1) {
                    pl = __ffsll((long long)tie) - 1;
                } else {
                    const unsigned Lw = wave_max_u32(bh == H ? bl : 0u);
                    const unsigned X = wave_max_u32((bh == H && bl == Lw) ? ~(unsigned)bp : 0u);
                    pl = __ffsll((long long)__ballot(bh == H && bl == Lw && bp == (int)~X)) - 1;
                }
                pl = __builtin_amdgcn_readfirstlane(pl);
                ss = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bs, pl));
                plp = __builtin_amdgcn_readlane(bp, pl);
            }
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

#if !LVG_LU3
// The factored chunk's rows (logical position >= kk) to A (L below the pivots; the pivot
// rows with L11 and U), perm/pos/b, L11 (strictly lower) and the
// stage Lst (L of the rows below the chunk, 0 for the others) for the waves to its right.
__device__ __forceinline__ void lu2_publish(const double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb,
                                            int s_lo, double *A, int N, double *b, const bool (&part)[S4],
                                            const int (&lp)[S4], const double (&rb)[S4], Smem &sm) {
    const int ln = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + ln;
        if (s < s_lo || r >= N) continue;
        if (part[s]) {
            const int p = prow[s], q = lp[s];
            const bool piv = q < nb;
            const double (&v)[CW] = acc[s];
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
            b[p] = rb[s];
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
                __syncthreads();
            }
        } else {
            __syncthreads();
        }
        TACC(PH_RSV, tr0);
        // ---- earlier chunks: L staged by tile row, two barriers a step (prefetching the next
        //      chunk's rows into registers during this one measured slower)
        if (c0 > 0) {
            double pf[CW];
            for (int kk = 0; kk < c0; kk += CW) {
                TSTAMP(tf0);
                lu2_fetch_l(A, N, kk, trow, pf);
                lu2_stage_l(N, kk, pf, sm);
                __syncthreads();
                TACC(PH_T_FETCH, tf0);
                if (nw > 0) lu2_apply(acc, prow, true, kk, CW, (kk + CW) >> 6, cw0, nw, A, N, sm);
                TSTAMP(tb0);
                __syncthreads();
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
            __syncthreads();                       // the applies of the previous chunk are done
            if (w == wq) lu2_publish(acc, prow, kk, nb, SLO, A, N, b, part, lp, rb, sm);
            __syncthreads();
            TACC(PH_P_WB, tw0);
            if (w > wq && nw > 0) lu2_apply(acc, prow, false, kk, nb, SLO, cw0, nw, A, N, sm);
        }
    }
    TSTAMP(tw0);
    __syncthreads();
    TACC(PH_BS_WAIT, tw0);
    back_substitute(A, N, b, sm);
    double emax = 0.;
    if (FUSED && t < N) { const double r = sm.resid[t]; src.df[t] = r; emax = fabs(r); }
    return FUSED ? block_max(emax, sm) : 0.;
}
#else
#include "lvg_lu3.h"
#endif
