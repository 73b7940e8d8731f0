// lvg_lu256.h — the LU of calc_new_pop / boundary_layer_populations for N <= 256 (the
// 256- and 512-thread solve_kernel), included by lvg_kernels.hip inside its namespace.
//
// lu_matrix_solve (absent library; call sites iteration_lvg.cpp:100, iteration_control.cpp:87)
// as a left-looking LU over chunks of CW = 16 columns, chunk j owned by wave j mod NW, with
// no workgroup barrier between chunks:
//  * A wave takes its next chunk as soon as it has published the previous one: it loads the
//    chunk's columns (assembled from K, the line terms and the diagonal when fused) for the
//    tile rows of a consistent snapshot of the row permutation (seqlock on sm.seq: positions
//    of published chunks are final, so their rows sit at their own tile rows), adds the
//    chunk's columns to the residual in column order (chunks in turn, sm.rdone), then
//    applies chunks 0 .. j-1 in order, waiting only for those not yet published, and factors
//    the chunk (lu_panel) and publishes it.
//  * Applying chunk i: the chunk's pivot rows in this wave's columns are solved against
//    L11 of chunk i (kept in LDS for every chunk, sm.pu.L11c) and stored as U rows; the rows
//    below take the rank-16 update with L read straight from the factors in A (4 columns of
//    L at a time), U broadcast from the wave's LDS rows.
//  * Publishing chunk j: L and the pivot rows to A, perm / pos / b, L11 of the chunk, then
//    sm.seq = 2 (j + 1) behind a workgroup release fence.
// So while the owner of chunk j factors it, the other waves already apply the published
// chunks to their next chunks instead of waiting at a barrier; the chain is panel j ->
// apply of j to chunk j+1 -> panel j+1.
// Every element still receives fma(-l_ik, u_kj, a_ij) for k ascending and the pivots are
// those of lu_panel (the oracle's rule), so the results are the unblocked oracle's bit for
// bit. On return sm.blog holds x.

// Rows: lane l of every wave keeps tile rows 64 s + l (s < 4) of its chunk, acc[s][0..16)
// (128 fp64 registers); b: LDS [N] indexed by physical row.

constexpr int S4 = NMAX / 64;   // row slots per lane: tile row 64 s + lane
constexpr int CW = LU_CW;       // chunk (panel) width
constexpr int CL = CW / 4;      // TRSM columns per lane (4 x 16-lane rows)
static_assert(CW == 16, "chunk width: the TRSM lays the 16 rows of a chunk over 16-lane groups");

// LDS stores of one lane visible to the other lanes of its wave: a wave's LDS instructions
// execute in issue order, so only compiler motion has to be stopped (wavefront-scope
// fences emit no wait; a workgroup-scope fence would also wait for the wave's global
// stores and prefetch loads, vmcnt(0))
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The chunk kk (this wave's CW columns) factored by this wave alone: rows of slots >= s_lo
// whose logical position is >= kk take part (exec-masked), 4 rows per lane. Per column:
// the lane's best key over its rows, one DPP wave max + ballot (lower word and position
// only on a tie) for the pivot, the pivot row selected from the lane's slots in registers
// and broadcast by v_readlane, one division and the row update per active row, b
// eliminated alongside (b[p], LDS by physical row; kept in registers until the publish).
// The row select is a v_cndmask chain: written as branches on the (uniform) slot, or
// through LDS, the compiler folds it into a dynamic acc[ss] index and moves acc to
// scratch memory (measured: 352 -> 800 B/lane).
__device__ __forceinline__ void lu_panel(double (&acc)[S4][CW], const int (&prow)[S4], int kk, int nb, int s_lo,
                                         int N, const double *b, bool (&part)[S4], int (&lp)[S4],
                                         double (&rb)[S4], Smem &sm) {
    const int ln = lvg_tid() & 63;
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

__device__ __forceinline__ int lu_ld(const int &x) {
    return __hip_atomic_load(&x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lu_st(int &x, int v) {
    __hip_atomic_store(&x, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the wave waits (sleeping between polls) until the sequence word reaches v
__device__ __forceinline__ void lu_wait(const int &x, int v) {
    while (lu_ld(x) < v) __builtin_amdgcn_s_sleep(1);
}

// L source of the rows that take no update in lu_apply (and of the slots below s_up): every
// lane of every slot loads, from its row or from these zeros. Exec-masked loads behind
// s_cbranch_execz left the number of loads in flight path-dependent, so the waitcnt pass
// drained the queue (vmcnt(0)) at every slot block of the FMA stream; unconditional loads
// through global (not flat) pointers measured +6% (profiles/r5/variants.txt item 14).
__device__ __attribute__((aligned(16))) double lu_zero_row[CW] = {0.};

// Chunk ci (columns kk.., nb of them, published) applied to this wave's columns cw0.. (nw).
// earlier: ci was published before this chunk's load, so its pivot rows sit at tile rows
// kk..kk+15 and the rows taking its update at tile rows >= kk + 16. s_up: first row slot
// that can hold a row taking an update (tile rows below 16 x the chunks final at the load
// are pivots of earlier chunks).
__device__ __forceinline__ void lu_apply(double (&acc)[S4][CW], const int (&prow)[S4], bool earlier, int ci, int nb,
                                         int s_up, int cw0, int nw, double *A, int N, Smem &sm) {
    const int l = lvg_tid() & 63, w = lvg_tid() >> 6, kk = ci * CW;
    double (*Ub)[CW] = sm.Ub[w];
    TSTAMP(ta0);
    // the chunk's pivot rows in this wave's columns to Ub (their owner lanes)
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + l;
        if (s >= (earlier ? kk >> 6 : s_up) && r < N) {
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
        const double *lrw = sm.pu.L11c[ci][r < CW ? r : 0];
        // the lane's L11 row read once, ahead of the steps (one LDS wait instead of one per step)
        double lmv[CW - 1];
#pragma unroll
        for (int m = 0; m < CW - 1; m++) lmv[m] = lrw[m];
#define LVG_TRSM_STEP(M_)                                                                  \
        if ((M_) < nb - 1) {                                                               \
            const double lm = lmv[M_];                                                     \
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
            gp<double> urow = glb(A) + (int64_t)sm.perm[kk + r] * N + cw0 + CL * q4;
#pragma unroll
            for (int i = 0; i < CL; i++) if (CL * q4 + i < nw) urow[i] = x[i];
        }
    }
    wave_lds_sync();
    TACC(PH_T_SOLVE, ta0);
    TSTAMP(tg0);
    // rows taking the update: below the chunk's pivots (logical position >= kk + nb)
    bool take[S4];
    gp<const double> lsrc[S4];
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + l;
        take[s] = s >= s_up && r < N && (earlier ? r : sm.pos[prow[s]]) >= kk + nb;
        lsrc[s] = take[s] ? glb((const double *)A) + (int64_t)prow[s] * N + kk : glb((const double *)lu_zero_row);
    }
    // slots with no row taking the update skip their FMAs (uniform: one ballot per slot)
    bool upd[S4];
#pragma unroll
    for (int s = 0; s < S4; s++) upd[s] = s >= s_up && __ballot(take[s]) != 0;
    constexpr int MG = 4;                         // columns of L per load group
    auto load = [&](double (&a)[S4][MG], int g) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < S4; s++) {
            // 16-byte loads at 8-byte alignment (odd N): global memory takes them unaligned
            gp<const vd2u> p2 = reinterpret_cast<gp<const vd2u>>(lsrc[s] + g);
#pragma unroll
            for (int h = 0; h < MG / 2; h++) { const vd2u v = p2[h]; a[s][2 * h] = v.x; a[s][2 * h + 1] = v.y; }
        }
    };
    auto update = [&](const double (&a)[S4][MG], int g) __attribute__((always_inline)) {
#pragma unroll
        for (int mm = 0; mm < MG; mm++) {
            const int m = g + mm;
            if (m < nb) {
                double u[CW];
                const double2 *up = reinterpret_cast<const double2 *>(&Ub[m][0]);
#pragma unroll
                for (int j = 0; j < CW / 2; j++) { const double2 v = up[j]; u[2 * j] = v.x; u[2 * j + 1] = v.y; }
#pragma unroll
                for (int s = 0; s < S4; s++) {
                    if (upd[s]) {
#pragma unroll
                        for (int c = 0; c < CW; c++) acc[s][c] = fma(-a[s][mm], u[c], acc[s][c]);
                    }
                }
            }
        }
    };
    double a[S4][MG];
#pragma unroll
    for (int g = 0; g < CW; g += MG) {
        if (g < nb) {
            load(a, g);
            update(a, g);
        }
    }
    TACC(PH_GEMM, tg0);
}

// The factored chunk ci's participating rows to A (L below the pivots; the pivot rows with
// L11 and U), perm / pos / b, and L11 of the chunk (strictly lower) to sm.pu.L11c[ci].
__device__ __forceinline__ void lu_publish(const double (&acc)[S4][CW], const int (&prow)[S4], int ci, int nb,
                                            int s_lo, double *A, int N, double *b, const bool (&part)[S4],
                                            const int (&lp)[S4], const double (&rb)[S4], Smem &sm) {
    const int ln = lvg_tid() & 63, kk = ci * CW;
#pragma unroll
    for (int s = 0; s < S4; s++) {
        const int r = 64 * s + ln;
        if (s < s_lo || r >= N || !part[s]) continue;
        const int p = prow[s], q = lp[s];
        const double (&v)[CW] = acc[s];
        gp<double> Ap = glb(A) + (int64_t)p * N + kk;
        if ((N & 1) == 0 && nb == CW) {
            gp<vd2> d2 = reinterpret_cast<gp<vd2>>(Ap);
#pragma unroll
            for (int j = 0; j < CW / 2; j++) { const vd2 x = {v[2 * j], v[2 * j + 1]}; d2[j] = x; }
        } else {
#pragma unroll
            for (int j = 0; j < CW; j++) if (j < nb) Ap[j] = v[j];
        }
        sm.perm[kk + q] = p;
        sm.pos[p] = kk + q;
        b[p] = rb[s];
        if (q < nb) {
#pragma unroll
            for (int m = 0; m < CW; m++) sm.pu.L11c[ci][q][m] = m < q ? v[m] : 0.;
        }
    }
}

__device__ __forceinline__ double block_lu_solve(double *A, int N, double *b, Smem &sm, const LuSrc &src, const bool FUSED) {
    const int t = lvg_tid();
    for (int i = t; i < N; i += BT) {
        sm.perm[i] = i;
        sm.pos[i] = i;
        if (FUSED) sm.resid[i] = (i == 0) ? 1. : 0.;
    }
    if (t == 0) { sm.seq = 0; sm.rdone = 0; }
    __syncthreads();
    const int l = t & 63, w = t >> 6;
    const int nch = (N + CW - 1) / CW;
    for (int j = w; j < nch; j += NW) {
        const int c0 = j * CW;
        const int nw = min(CW, N - c0);
        TSTAMP(tp0);
        // ---- a consistent snapshot of the tile -> physical row map: kp chunks are final
        //      (seqlock reader: an even sequence word read before and after the perm reads
        //      means no publish overlapped them, given the writer's in-order LDS stores, see
        //      the writer below)
        int prow[S4], kp;
        for (;;) {
            const int s1 = lu_ld(sm.seq);
            if (s1 & 1) { __builtin_amdgcn_s_sleep(1); continue; }
#pragma unroll
            for (int s = 0; s < S4; s++) prow[s] = (64 * s + l < N) ? sm.perm[64 * s + l] : 0;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (lu_ld(sm.seq) == s1) { kp = s1 >> 1; break; }
        }
        const int SLO = (CW * kp) >> 6;             // slots below hold pivots of final chunks only
        double acc[S4][CW];
        // ---- this wave's chunk into registers (fused: assembled from K, the line terms and the
        //      diagonal, row 0 <- 1)
#pragma unroll
        for (int s = 0; s < S4; s++) {
            const int r = 64 * s + l, pr = prow[s];
            const bool okr = r < N;
            if (!FUSED) {
                // every load unconditional (rows past N read row 0 or the zero row, columns past N
                // column N - 1), the values selected after: no exec-masked loads (lu_zero_row)
                double kv[CW];
                gp<const double> rsrc = glb(src.BK ? src.BK : (src.B ? src.B : A));
                if (nw == CW) {
                    gp<const vd2u> k2 = reinterpret_cast<gp<const vd2u>>(
                        okr ? rsrc + (int64_t)pr * N + c0 : glb((const double *)lu_zero_row));
#pragma unroll
                    for (int jj = 0; jj < CW / 2; jj++) { const vd2u x = k2[jj]; kv[2 * jj] = x.x; kv[2 * jj + 1] = x.y; }
                } else {
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) kv[jj] = rsrc[(int64_t)pr * N + min(c0 + jj, N - 1)];
                }
                if (src.BK) {
                    // einst[d][pr] for the chunk's columns d: row pr of the transposed copy, as the K row
                    double ev[CW];
                    if (nw == CW) {
                        gp<const vd2u> e2 = reinterpret_cast<gp<const vd2u>>(
                            okr ? glb(src.BET) + (int64_t)pr * N + c0 : glb((const double *)lu_zero_row));
#pragma unroll
                        for (int jj = 0; jj < CW / 2; jj++) { const vd2u x = e2[jj]; ev[2 * jj] = x.x; ev[2 * jj + 1] = x.y; }
                    } else {
#pragma unroll
                        for (int jj = 0; jj < CW; jj++) ev[jj] = glb(src.BET)[(int64_t)pr * N + min(c0 + jj, N - 1)];
                    }
                    double bd[CW];
                    if (src.BD == sm.diag) {     // B's diagonal in LDS (formed in-kernel) or HBM (coll_kernel)
                        typedef __attribute__((address_space(3))) const double *lds_d;
#pragma unroll
                        for (int jj = 0; jj < CW; jj++) bd[jj] = ((lds_d)src.BD)[min(c0 + jj, N - 1)];
                    } else {
#pragma unroll
                        for (int jj = 0; jj < CW; jj++) bd[jj] = glb(src.BD)[min(c0 + jj, N - 1)];
                    }
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) {
                        const int d = c0 + jj;
                        const double e = ev[jj];
                        const double dg = bd[jj];
                        double v = (pr < d) ? 0.5 * e + kv[jj] : kv[jj];   // build_collision_operators: 0.5 * af + dn
                        if (pr == d) v = dg;
                        if (pr == 0) v = 1.;
                        kv[jj] = v;
                    }
                }
#pragma unroll
                for (int jj = 0; jj < CW; jj++) acc[s][jj] = (okr && jj < nw) ? kv[jj] : 0.;
            } else {
                // every load unconditional through global (K, line index) or LDS-typed (y-cache)
                // pointers, rows past N reading row 0 and columns past N column N - 1, the line
                // terms gathered at clamped indices: the values are selected after
                int li[CW];
                double kv[CW], yv[CW];
                const int64_t o = (int64_t)(okr ? pr : 0) * N + c0;
                const gp<const double> Kg = glb(src.K) + o;
                const gp<const int> Lg = glb(src.li) + o;
                if ((N & 3) == 0 && nw == CW) {
                    const gp<const vd2> k2 = reinterpret_cast<gp<const vd2>>(Kg);
                    const gp<const vi4> l4 = reinterpret_cast<gp<const vi4>>(Lg);
#pragma unroll
                    for (int jj = 0; jj < CW / 2; jj++) { const vd2 x = k2[jj]; kv[2 * jj] = x.x; kv[2 * jj + 1] = x.y; }
#pragma unroll
                    for (int jj = 0; jj < CW / 4; jj++) {
                        const vi4 x = l4[jj];
                        li[4 * jj] = x.x; li[4 * jj + 1] = x.y; li[4 * jj + 2] = x.z; li[4 * jj + 3] = x.w;
                    }
                } else {
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) {
                        const int cj = min(jj, N - 1 - c0);
                        kv[jj] = Kg[cj];
                        li[jj] = Lg[cj];
                    }
                }
                if (src.y == sm.ylds) {
                    typedef __attribute__((address_space(3))) const double *lds_y;
                    const lds_y Yl = (lds_y)src.y;
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) yv[jj] = Yl[li[jj] >= 0 ? li[jj] : 0];
                } else {
                    const gp<const double> Yg = glb(src.y);
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) yv[jj] = Yg[li[jj] >= 0 ? li[jj] : 0];
                }
#pragma unroll
                for (int jj = 0; jj < CW; jj++) {
                    const int d = c0 + jj;
                    double v = kv[jj];
                    v = (okr && li[jj] >= 0) ? v + yv[jj] : v;
                    if (pr == d) v = sm.diag[d < NMAX ? d : 0];
                    if (pr == 0) v = 1.;
                    acc[s][jj] = (okr && jj < nw) ? v : 0.;
                    if (src.dump && okr && jj < nw) src.dump[(int64_t)pr * N + d] = v;
                }
            }
        }
        TACC(PH_BLOAD, tp0);
        // ---- residual rows (physical), this chunk's columns in ascending order, chunks in turn
        if (FUSED) {
            TSTAMP(tr0);
            lu_wait(sm.rdone, j);
#pragma unroll
            for (int s = 0; s < S4; s++) {
                const int r = 64 * s + l;
                if (r < N) {
                    double sr = sm.resid[prow[s]];
#pragma unroll
                    for (int jj = 0; jj < CW; jj++) if (jj < nw) sr = sr - acc[s][jj] * src.pop[c0 + jj];
                    sm.resid[prow[s]] = sr;
                }
            }
            wave_lds_sync();
            if (l == 0) lu_st(sm.rdone, j + 1);
            TACC(PH_RSV, tr0);
        }
        // ---- the chunks before this one, in order, each once it is published
        for (int ci = 0; ci < j; ci++) {
            TSTAMP(tf0);
            if (ci >= kp) lu_wait(sm.seq, 2 * (ci + 1));
            TACC(PH_T_FETCH, tf0);
            const bool earlier = ci < kp;
            lu_apply(acc, prow, earlier, ci, CW, earlier ? (CW * (ci + 1)) >> 6 : SLO, c0, nw, A, N, sm);
        }
        // ---- this chunk: factor, publish
        const int nb = nw;
        bool part[S4];
        int lp[S4];
        double rb[S4];
        TSTAMP(tp1);
        lu_panel(acc, prow, c0, nb, SLO, N, b, part, lp, rb, sm);
        TACC(PH_PANEL, tp1);
        TSTAMP(tw0);
        // Seqlock writer. The odd marker must be visible before any perm / pos write of
        // lu_publish, which are plain LDS stores: a release fence orders earlier accesses
        // before LATER ATOMIC stores only, so this order rests on the hardware: a wave's LDS
        // instructions execute in issue order on gfx9 (the fence keeps the compiler from
        // moving the stores above the marker). If perm / pos ever move out of LDS (global
        // memory is not in order), write them with relaxed workgroup-scope atomic stores.
        if (l == 0) __hip_atomic_store(&sm.seq, 2 * j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        lu_publish(acc, prow, j, nb, SLO, A, N, b, part, lp, rb, sm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wave_lds_sync();
        if (l == 0) lu_st(sm.seq, 2 * j + 2);
        TACC(PH_P_WB, tw0);
    }
    TSTAMP(tw1);
    __syncthreads();
    TACC(PH_BS_WAIT, tw1);
    back_substitute(A, N, b, sm);
    double emax = 0.;
    if (FUSED && t < N) { const double r = sm.resid[t]; src.df[t] = r; emax = fabs(r); }
    return FUSED ? block_max(emax, sm) : 0.;
}
