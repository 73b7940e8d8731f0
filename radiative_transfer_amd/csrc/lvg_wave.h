// lvg_wave.h — wave-per-layer solver for small molecules (N <= 64), included by
// lvg_kernels.hip inside namespace lvg (it reuses the block kernel's layer scalars,
// line-term and iteration-control helpers).
//
// Why a second kernel: for N <= 64 the 256-thread block of solve_kernel keeps at most
// N threads busy and pays a workgroup barrier per LU column (ph2o45: ≈2 K cycles a
// column, 95 K per LU in the panel alone). Here ONE wavefront owns a layer:
//  * lane i holds row i of the N x N rate matrix in registers (double a[NM]), so the
//    LU needs no barrier and no LDS round trip: the pivot is a DPP u32 max (+ ballot),
//    the pivot row is broadcast with v_readlane into SGPRs, every lane updates its own
//    row with fma(-l, u_kj, a_ij) for k ascending (the oracle's order, bit for bit);
//  * the collision operator K of the layer lives in LDS (row stride N|1, conflict-light),
//    with the line-index map shared by the block's waves and the escape-table grids
//    copied to LDS, so the per-iteration assembly, diagonal fold, residual and the
//    escape-probability bisections never touch HBM;
//  * four waves per block (fewer if K does not fit) work independent layers from the
//    same atomic queue as solve_kernel.
// The arithmetic of every step is the block kernel's (and the oracle's), in the same
// order; results are bit-identical, which tests/test_gpu_parity.py checks.
#pragma once

#ifndef LVG_WAVE_CLAMP
#define LVG_WAVE_CLAMP 1              // assembly operands read unconditionally (clamped indices)
#endif
#ifndef LVG_WAVE_OPAQUE_N
#define LVG_WAVE_OPAQUE_N 1
#endif
#ifndef LVG_WAVE_LINE_INV
#define LVG_WAVE_LINE_INV 1           // line terms from per-layer invariant records (wave_line_invariants)
#endif
#ifndef LVG_WAVE_KROW
#define LVG_WAVE_KROW 1               // 1: the lane's K / line-index row held in registers for the layer
#endif
#ifndef LVG_WAVE_ACCEL_BATCH
#define LVG_WAVE_ACCEL_BATCH 1        // Ng sums: ring reads of 8 levels per round trip
#endif
constexpr int WYCAP = 512;        // line terms y per wave kept in LDS (host checks 2*nb_lines <= WYCAP)
constexpr int WGRID_CAP = 1024;   // escape + overlap grid doubles copied to LDS (host checks)
constexpr int WNMAX = 64;

struct WaveLayer {                // per-wave LDS
    double pold[WNMAX], pnew[WNMAX], diag[WNMAX];
    alignas(16) double prow[WNMAX + 2];   // LU: the pivot row of the current column, then its b
    double y[WYCAP];
    double hist_acc[32];
    double T, Te, vw, vgrad, nmol, ne;
    double cc[LVG_MAX_COMBOS];
    double teff[LVG_MAX_TABLES];
    int    lo[LVG_MAX_TABLES];
    const double *tcol[LVG_MAX_TABLES];
    const double *tder[LVG_MAX_TABLES];
    int64_t timax[LVG_MAX_TABLES];
    double tdt[LVG_MAX_TABLES];
    double tx[LVG_MAX_TABLES];
    double dust[LVG_MAX_DUST];
};

#ifdef LVG_PHASE_TIMERS
// timer build: every wave's lane 0 accumulates (LDS atomics), not just thread 0 of the block
#undef TACC
#define TACC(ph, v0) do { if ((threadIdx.x & 63) == 0) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    atomicAdd(&lvg_ph_lds[ph], t_ - (v0)); } } while (0)
#endif

struct WaveShared {               // per-block LDS (static part)
    int8_t ttab[LVG_MAX_CLASSES][LVG_MAX_TERMS], tcombo[LVG_MAX_CLASSES][LVG_MAX_TERMS];
    int8_t tet[LVG_MAX_CLASSES], tgrp[LVG_MAX_CLASSES];
    double grids[WGRID_CAP];
    WaveLayer w[4];
};

// dynamic LDS: line index map [N][N|1] (int), then K [wpb][N][N|1] (double)
extern __shared__ double lvg_wave_dyn[];

// LDS stores of one lane become visible to the other lanes of its wave (workgroup-scope
// fences: lgkmcnt(0); no wait for outstanding global stores, which a lane only reads
// back itself, in program order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// ... and global stores too (s_waitcnt 0: the wave's own stores have completed), before a
// lane reads global data another lane wrote: the Ng history rings (accel_step) and the
// boundary-layer matrix B
__device__ __forceinline__ void wave_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Collision operator of the layer (build_collision_operators, one pair per lane):
// K[s][f] = down + electrons, K[f][s] = up + electrons (LDS, stride ldk); the
// boundary matrix B (neutrals + A/2, global, stride N) when B != nullptr.
__device__ __forceinline__ void wave_collisions(const LvgDevProblem &P, const WaveShared &sh, const WaveLayer &sm,
                                                double *K, int ldk, double *B) {
    const int N = P.N, M2 = N * (N - 1) / 2;
    const double T = sm.T, Te = sm.Te;
    for (int p = lane_id(); p < M2; p += 64) {
        int f = (int)((1. + sqrt(1. + 8. * (double)p)) * 0.5);
        while (f * (f - 1) / 2 > p) f--;
        while (f * (f + 1) / 2 <= p) f++;
        const int s = p - f * (f - 1) / 2;
        const int cl = P.pair_class[p];
        const int grp = sh.tgrp[cl];
        double dn = 0., gsum = 0.;
        int ng = 0;
#pragma unroll
        for (int k = 0; k < LVG_MAX_TERMS; k++) {
            const int tb = sh.ttab[cl][k];
            if (tb < 0) break;
            const double r = (sm.tcol[tb][p] + sm.tder[tb][p] * sm.tx[tb]) * sm.cc[sh.tcombo[cl][k]];   // get_rate
            if (k < grp) dn = (k == 0) ? r : dn + r;
            else { gsum = (ng == 0) ? r : gsum + r; ng++; }
        }
        if (ng) dn = dn + gsum;
        const double ef = P.energy[f], es = P.energy[s], gf = P.g[f], gs = P.g[s];
        const double de = es - ef;
        double un = 0.;
        if (dn > MIN_COLLISION_RATE) un = dn * lvg_exp(de * CM_INVERSE_TO_KELVINS / T) * gf / gs;
        else dn = 0.;
        double dE = 0., uE = 0.;
        const int et = sh.tet[cl];
        if (et >= 0) {
            dE = (sm.tcol[et][p] + sm.tder[et][p] * sm.tx[et]) * sm.ne;
            if (dE > MIN_COLLISION_RATE) uE = dE * lvg_exp(de * CM_INVERSE_TO_KELVINS / Te) * gf / gs;
            else dE = 0.;
        }
        K[s * ldk + f] = dn + dE;
        K[f * ldk + s] = un + uE;
        if (B) {
            B[s * N + f] = 0.5 * P.einst[f * N + s] + dn;
            B[f * N + s] = un;
        }
    }
}

// ---- line terms with the table lookups batched -------------------------------------
// Same arithmetic as esc_func / overlap_esc_func / intensity_single / intensity_pair
// (lvg_kernels.hip), reorganised so that a lane's independent table reads are issued
// together: the bisections run in LDS first, then every table value the lane needs
// is loaded in one round trip. Overlap: the p1 and p2 tables share the interpolation
// indices (same gamma, delta, gratio, dx), so each direction is located once.
struct OvIdx {
    int m, n, k, l;
    double y, p, u, t;
};
__device__ __forceinline__ OvIdx ov_index(const LvgDevProblem &P, const EscGrids &G, double gamma, double ldelta,
                                          double gratio, double dxv) {
    OvIdx o;
    o.m = locate_index(G.old, P.ov_nd, ldelta);
    o.l = locate_index(G.og, P.ov_ng, gamma);
    o.k = locate_index(G.ogr, P.ov_ngr, gratio);
    o.n = locate_index(G.odx, P.ov_ndx, dxv);
    o.y = 0.; o.u = 0.; o.t = 0.; o.p = 0.;
    if (o.m < 0) o.m = 0;
    else if (o.m > P.ov_nd - 2) { o.m = P.ov_nd - 2; o.y = 1.; }
    else o.y = (ldelta - G.old[o.m]) / (G.old[o.m + 1] - G.old[o.m]);
    if (o.n < 0) o.n = 0;
    else if (o.n > P.ov_ndx - 2) { o.p = 1.; o.n = P.ov_ndx - 2; }
    else o.p = (dxv - G.odx[o.n]) / (G.odx[o.n + 1] - G.odx[o.n]);
    if (o.l < 0) o.l = 0;
    else if (o.l > P.ov_ng - 2) { o.l = P.ov_ng - 2; o.u = 1.; }
    else o.u = (gamma - G.og[o.l]) / (G.og[o.l + 1] - G.og[o.l]);
    if (o.k < 0) o.k = 0;
    else if (o.k > P.ov_ngr - 2) { o.t = 1.; o.k = P.ov_ngr - 2; }
    else o.t = (gratio - G.ogr[o.k]) / (G.ogr[o.k + 1] - G.ogr[o.k]);
    return o;
}
__device__ __forceinline__ void ov_load(const LvgDevProblem &P, const double *tab, const OvIdx &o, double (&v)[16]) {
    const int W = P.ov_ngr * P.ov_ng, ndx = P.ov_ndx, ng = P.ov_ng;
#pragma unroll
    for (int dm = 0; dm < 2; dm++)
#pragma unroll
        for (int dn = 0; dn < 2; dn++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++)
#pragma unroll
                for (int dl = 0; dl < 2; dl++)
                    v[8 * dm + 4 * dn + 2 * dk + dl] =
                        tab[(int64_t)((o.m + dm) * ndx + o.n + dn) * W + (o.k + dk) * ng + o.l + dl];
}
__device__ __forceinline__ double ov_sum(const OvIdx &o, const double (&v)[16]) {
    double e = 0.;
#pragma unroll
    for (int dm = 0; dm < 2; dm++)
#pragma unroll
        for (int dn = 0; dn < 2; dn++)
#pragma unroll
            for (int dk = 0; dk < 2; dk++)
#pragma unroll
                for (int dl = 0; dl < 2; dl++)
                    e += v[8 * dm + 4 * dn + 2 * dk + dl] * (dl ? o.u : 1. - o.u) * (dk ? o.t : 1. - o.t) *
                         (dn ? o.p : 1. - o.p) * (dm ? o.y : 1. - o.y);
    return e > 1. ? 1. : (e < 0. ? 0. : e);
}

struct EscIdx {
    int k, l;
    double t, u;
};
__device__ __forceinline__ EscIdx esc_index(const LvgDevProblem &P, const EscGrids &G, double gamma, double delta) {
    const int nd = P.esc_nd, ng = P.esc_ng;
    EscIdx o;
    o.k = locate_index(G.ed, nd, delta);
    o.l = locate_index(G.eg, ng, gamma);
    if (o.k < 0) { o.t = 0.; o.k = 0; }
    else if (o.k > nd - 2) { o.t = 1.; o.k = nd - 2; }
    else o.t = (delta - G.ed[o.k]) / (G.ed[o.k + 1] - G.ed[o.k]);
    if (o.l < 0) { o.l = 0; o.u = 0.; }
    else if (o.l > ng - 2) { o.l = ng - 2; o.u = 1.; }
    else o.u = (gamma - G.eg[o.l]) / (G.eg[o.l + 1] - G.eg[o.l]);
    return o;
}
__device__ __forceinline__ void esc_load(const LvgDevProblem &P, const EscIdx &o, double (&v)[4]) {
    const int ng = P.esc_ng;
    const double *p = P.esc_p;
    v[0] = p[o.k * ng + o.l]; v[1] = p[(o.k + 1) * ng + o.l]; v[2] = p[o.k * ng + o.l + 1];
    v[3] = p[(o.k + 1) * ng + o.l + 1];
}
__device__ __forceinline__ double esc_sum(const EscIdx &o, const double (&v)[4]) {
    const double t = o.t, u = o.u;
    double e = v[0] * (1. - t) * (1. - u) + v[1] * t * (1. - u) + v[2] * (1. - t) * u + v[3] * u * t;
    return e > 1. ? 1. : (e < 0. ? 0. : e);
}

// ---- per-layer line invariants -----------------------------------------------------
// Everything in intensity_single / intensity_pair that does not depend on the
// populations is fixed for the whole layer: the unit's line indices and Einstein
// coefficients, c = n_mol / (8 pi v_w E^3), the dust opacity and from it delta, its
// escape-grid interval (k, t) and log10(delta)'s overlap-grid interval (m, y), and for a
// pair the frequency offset dx with its overlap-grid intervals for +dx and -dx. They are
// computed once per layer (same expressions, same results) into the wave's slot as
// structure-of-arrays records (field f of unit q at inv[f * cap + q]), so an iteration
// reads one coalesced record per unit: one global round trip instead of the dependent
// unit -> line data -> level energies chain, and no dust sum, log10 or delta / dx
// bisection per iteration.
enum { WI_N1, WI_U1, WI_L1, WI_A1, WI_B1, WI_C, WI_EK, WI_ET, WI_PLAIN,
       WI_N2 = WI_PLAIN, WI_U2, WI_L2, WI_A2, WI_B2, WI_DX, WI_OM, WI_OY, WI_AN, WI_AP, WI_BN, WI_BP, WI_ALL };
static_assert(WI_ALL == LVG_WAVE_INV_FIELDS, "host reserves LVG_WAVE_INV_FIELDS doubles per line");

__device__ __forceinline__ void ov_interval(const double *g, int n, double x, int &j, double &w) {
    j = locate_index(g, n, x);
    if (j < 0) { j = 0; w = 0.; }
    else if (j > n - 2) { j = n - 2; w = 1.; }
    else w = (x - g[j]) / (g[j + 1] - g[j]);
}

__device__ __forceinline__ void wave_line_invariants(const LvgDevProblem &P, const EscGrids &G, const LvgModeLines &M,
                                                     const WaveLayer &sm, bool ov, double *inv, int cap) {
    for (int q = lane_id(); q < M.nb_units; q += 64) {
        const int n1 = M.unit_l0[q];
        const double energy = M.line_e[n1];
        const double c = sm.nmol / (EIGHT_PI * sm.vw * energy * energy * energy);
        const double delta = fabs(sm.vgrad) / (sm.vw * dust_opacity(P, M, sm, n1));
        const int u1 = M.line_u[n1], l1 = M.line_l[n1];
        int k;
        double t;
        ov_interval(G.ed, P.esc_nd, delta, k, t);   // esc_index's delta part
        inv[WI_N1 * cap + q] = n1;
        inv[WI_U1 * cap + q] = u1;
        inv[WI_L1 * cap + q] = l1;
        inv[WI_A1 * cap + q] = M.line_aul[n1];
        inv[WI_B1 * cap + q] = M.line_alu[n1];
        inv[WI_C * cap + q] = c;
        inv[WI_EK * cap + q] = k;
        inv[WI_ET * cap + q] = t;
        if (!ov) continue;
        const int n2 = M.unit_l1[q];
        inv[WI_N2 * cap + q] = n2;
        if (n2 < 0) continue;
        const int u2 = M.line_u[n2], l2 = M.line_l[n2];
        double dx = (P.energy[u1] - P.energy[l1] - P.energy[u2] + P.energy[l2]) * SPEED_OF_LIGHT / (energy * sm.vw);
        if (sm.vgrad < 0.) dx *= -1.;
        int m, an, bn;
        double y, ap, bp;
        ov_interval(G.old, P.ov_nd, lvg_log10(delta), m, y);
        ov_interval(G.odx, P.ov_ndx, dx, an, ap);
        ov_interval(G.odx, P.ov_ndx, -dx, bn, bp);
        inv[WI_U2 * cap + q] = u2;
        inv[WI_L2 * cap + q] = l2;
        inv[WI_A2 * cap + q] = M.line_aul[n2];
        inv[WI_B2 * cap + q] = M.line_alu[n2];
        inv[WI_DX * cap + q] = dx;
        inv[WI_OM * cap + q] = m;
        inv[WI_OY * cap + q] = y;
        inv[WI_AN * cap + q] = an;
        inv[WI_AP * cap + q] = ap;
        inv[WI_BN * cap + q] = bn;
        inv[WI_BP * cap + q] = bp;
    }
}

// plain scheme from the invariants: WUB units per lane per pass, stores last
__device__ __forceinline__ void wave_line_terms_plain_inv(const LvgDevProblem &P, const EscGrids &G,
                                                          const LvgModeLines &M, WaveLayer &sm, const double *inv,
                                                          int cap) {
    const int t = lane_id(), U = M.nb_units;
    constexpr int B = 4;
    for (int q0 = t; q0 < U; q0 += 64 * B) {
        double f[B][WI_PLAIN];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int q = (q0 + 64 * b < U) ? q0 + 64 * b : q0;
#pragma unroll
            for (int i = 0; i < WI_PLAIN; i++) f[b][i] = inv[i * cap + q];
        }
        EscIdx ix[B];
        double em[B], op[B], tv[B][4];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const double c = f[b][WI_C];
            em[b] = c * f[b][WI_A1] * sm.pold[(int)f[b][WI_U1]];
            op[b] = c * f[b][WI_B1] * sm.pold[(int)f[b][WI_L1]] - em[b] + MIN_LINE_OPACITY;
            if (op[b] < 0.) op[b] *= INV_TRANS_FACTOR;
            const double gamma = fabs(sm.vgrad) / (sm.vw * op[b]);
            ix[b].k = (int)f[b][WI_EK];
            ix[b].t = f[b][WI_ET];
            ov_interval(G.eg, P.esc_ng, gamma, ix[b].l, ix[b].u);   // esc_index's gamma part
        }
#pragma unroll
        for (int b = 0; b < B; b++) esc_load(P, ix[b], tv[b]);
#pragma unroll
        for (int b = 0; b < B; b++) {
            if (q0 + 64 * b < U) {
                const double I = em[b] / op[b] * esc_sum(ix[b], tv[b]);
                const int n = (int)f[b][WI_N1];
                sm.y[2 * n] = f[b][WI_A1] * (1. + I);
                sm.y[2 * n + 1] = f[b][WI_B1] * I;
            }
        }
    }
}

// overlap scheme from the invariants (intensity_single / intensity_pair sequences)
__device__ __forceinline__ void wave_line_terms_overlap_inv(const LvgDevProblem &P, const EscGrids &G,
                                                            const LvgModeLines &M, WaveLayer &sm, const double *inv,
                                                            int cap) {
    const double max_dx = 4.;
    const double *pop = sm.pold;
    for (int q = lane_id(); q < M.nb_units; q += 64) {
        double f[WI_ALL];
#pragma unroll
        for (int i = 0; i < WI_ALL; i++) f[i] = inv[i * cap + q];
        const int n1 = (int)f[WI_N1], n2 = (int)f[WI_N2];
        const double c0 = f[WI_C], a1 = f[WI_A1], b1 = f[WI_B1];
        if (n2 < 0) {
            const double emiss = c0 * a1 * pop[(int)f[WI_U1]];
            double opac = c0 * b1 * pop[(int)f[WI_L1]] - emiss + MIN_LINE_OPACITY;
            if (opac < 0.) opac *= INV_TRANS_FACTOR;
            const double gamma = fabs(sm.vgrad) / (sm.vw * opac);
            EscIdx ix;
            ix.k = (int)f[WI_EK];
            ix.t = f[WI_ET];
            ov_interval(G.eg, P.esc_ng, gamma, ix.l, ix.u);
            double tv[4];
            esc_load(P, ix, tv);
            const double I = emiss / opac * esc_sum(ix, tv);
            sm.y[2 * n1] = a1 * (1. + I);
            sm.y[2 * n1 + 1] = b1 * I;
            continue;
        }
        const int u1 = (int)f[WI_U1], l1 = (int)f[WI_L1], u2 = (int)f[WI_U2], l2 = (int)f[WI_L2];
        const double a2 = f[WI_A2], b2 = f[WI_B2], dx = f[WI_DX];
        const double em1 = c0 * a1 * pop[u1];
        double op1 = c0 * (b1 * pop[l1] - a1 * pop[u1]) + MIN_LINE_OPACITY;
        const double em2 = c0 * a2 * pop[u2];
        double op2 = c0 * (b2 * pop[l2] - a2 * pop[u2]) + MIN_LINE_OPACITY;
        if (op1 < 0.) op1 *= INV_TRANS_FACTOR;
        if (op2 < 0.) op2 *= INV_TRANS_FACTOR;
        const double g1 = fabs(sm.vgrad) / (sm.vw * op1), g2 = fabs(sm.vgrad) / (sm.vw * op2);
        const bool near = fabs(dx) < max_dx, far = fabs(dx) > max_dx - 0.5;
        double ep1 = 0., ep2 = 0., ep01 = 0., ep02 = 0., q1 = 0., q2 = 0.;
        if (near) {
            OvIdx A, B;
            A.m = B.m = (int)f[WI_OM];
            A.y = B.y = f[WI_OY];
            A.n = (int)f[WI_AN]; A.p = f[WI_AP];
            B.n = (int)f[WI_BN]; B.p = f[WI_BP];
            ov_interval(G.og, P.ov_ng, g1, A.l, A.u);
            ov_interval(G.ogr, P.ov_ngr, g2 / g1, A.k, A.t);
            ov_interval(G.og, P.ov_ng, g2, B.l, B.u);
            ov_interval(G.ogr, P.ov_ngr, g1 / g2, B.k, B.t);
            double v1[16], v2[16], w1[16], w2[16];
            ov_load(P, P.ov_p1, A, v1);
            ov_load(P, P.ov_p1, B, v2);
            ov_load(P, P.ov_p2, A, w1);
            ov_load(P, P.ov_p2, B, w2);
            ep1 = ov_sum(A, v1);
            ep2 = ov_sum(B, v2);
            q1 = ov_sum(A, w1);
            q2 = ov_sum(B, w2);
        }
        if (far) {
            EscIdx A, B;
            A.k = B.k = (int)f[WI_EK];
            A.t = B.t = f[WI_ET];
            ov_interval(G.eg, P.esc_ng, g1, A.l, A.u);
            ov_interval(G.eg, P.esc_ng, g2, B.l, B.u);
            double v1[4], v2[4];
            esc_load(P, A, v1);
            esc_load(P, B, v2);
            ep01 = esc_sum(A, v1);
            ep02 = esc_sum(B, v2);
        }
        double c = c0;
        if (fabs(dx) > max_dx) { ep1 = ep01; ep2 = ep02; }
        else if (far) {
            c = 2. * (max_dx - fabs(dx));
            ep1 = ep01 * (1. - c) + ep1 * c;
            ep2 = ep02 * (1. - c) + ep2 * c;
        }
        double i1 = em1 / op1 * ep1;
        double i2 = em2 / op2 * ep2;
        if (near) {
            ep1 = q1;
            ep2 = q2;
            if (far) {
                c = 2. * (max_dx - fabs(dx));
                ep1 *= c; ep2 *= c;
            }
            i1 += em2 / op2 * ep1;
            i2 += em1 / op1 * ep2;
        }
        sm.y[2 * n1] = a1 * (1. + i1);
        sm.y[2 * n1 + 1] = b1 * i1;
        sm.y[2 * n2] = a2 * (1. + i2);
        sm.y[2 * n2 + 1] = b2 * i2;
    }
}

// plain scheme: WUB single-line units per lane per pass (intensity_single), stores last
constexpr int WUB = 4;
__device__ __forceinline__ void wave_line_terms_plain(const LvgDevProblem &P, const EscGrids &G, const LvgModeLines &M,
                                                      WaveLayer &sm) {
    const int t = lane_id();
    for (int q0 = t; q0 < M.nb_units; q0 += 64 * WUB) {
        int n[WUB];
        double I[WUB], aul[WUB], alu[WUB];
        EscIdx ix[WUB];
        double em[WUB], op[WUB], tv[WUB][4];
#pragma unroll
        for (int b = 0; b < WUB; b++) {
            const int q = q0 + 64 * b;
            n[b] = (q < M.nb_units) ? M.unit_l0[q] : M.unit_l0[t];
        }
#pragma unroll
        for (int b = 0; b < WUB; b++) {
            const int nn = n[b];
            const int u = M.line_u[nn], l = M.line_l[nn];
            const double energy = M.line_e[nn];
            aul[b] = M.line_aul[nn];
            alu[b] = M.line_alu[nn];
            const double c = sm.nmol / (EIGHT_PI * sm.vw * energy * energy * energy);
            em[b] = c * aul[b] * sm.pold[u];
            op[b] = c * alu[b] * sm.pold[l] - em[b] + MIN_LINE_OPACITY;
            if (op[b] < 0.) op[b] *= INV_TRANS_FACTOR;
            const double dop = dust_opacity(P, M, sm, nn);
            const double gamma = fabs(sm.vgrad) / (sm.vw * op[b]);
            const double delta = fabs(sm.vgrad) / (sm.vw * dop);
            ix[b] = esc_index(P, G, gamma, delta);
        }
#pragma unroll
        for (int b = 0; b < WUB; b++) esc_load(P, ix[b], tv[b]);
#pragma unroll
        for (int b = 0; b < WUB; b++) I[b] = em[b] / op[b] * esc_sum(ix[b], tv[b]);
#pragma unroll
        for (int b = 0; b < WUB; b++) {
            if (q0 + 64 * b < M.nb_units) {
                sm.y[2 * n[b]] = aul[b] * (1. + I[b]);
                sm.y[2 * n[b] + 1] = alu[b] * I[b];
            }
        }
    }
}

// overlap scheme: one unit per lane per pass; pairs through intensity_pair's sequence
__device__ __forceinline__ void wave_line_terms_overlap(const LvgDevProblem &P, const EscGrids &G,
                                                        const LvgModeLines &M, WaveLayer &sm) {
    const double max_dx = 4.;
    for (int q = lane_id(); q < M.nb_units; q += 64) {
        const int n1 = M.unit_l0[q], n2 = M.unit_l1[q];
        if (n2 < 0) {
            const double I = intensity_single(P, G, M, sm, n1, sm.pold);
            sm.y[2 * n1] = M.line_aul[n1] * (1. + I);
            sm.y[2 * n1 + 1] = M.line_alu[n1] * I;
            continue;
        }
        const double *pop = sm.pold;
        const int u1 = M.line_u[n1], l1 = M.line_l[n1], u2 = M.line_u[n2], l2 = M.line_l[n2];
        const double energy = M.line_e[n1];
        double c = sm.nmol / (EIGHT_PI * sm.vw * energy * energy * energy);
        const double a1 = M.line_aul[n1], b1 = M.line_alu[n1], a2 = M.line_aul[n2], b2 = M.line_alu[n2];
        const double em1 = c * a1 * pop[u1];
        double op1 = c * (b1 * pop[l1] - a1 * pop[u1]) + MIN_LINE_OPACITY;
        const double em2 = c * a2 * pop[u2];
        double op2 = c * (b2 * pop[l2] - a2 * pop[u2]) + MIN_LINE_OPACITY;
        if (op1 < 0.) op1 *= INV_TRANS_FACTOR;
        if (op2 < 0.) op2 *= INV_TRANS_FACTOR;
        const double g1 = fabs(sm.vgrad) / (sm.vw * op1), g2 = fabs(sm.vgrad) / (sm.vw * op2);
        const double delta = fabs(sm.vgrad) / (sm.vw * dust_opacity(P, M, sm, n1));
        double dx = (P.energy[u1] - P.energy[l1] - P.energy[u2] + P.energy[l2]) * SPEED_OF_LIGHT / (energy * sm.vw);
        if (sm.vgrad < 0.) dx *= -1.;
        const bool near = fabs(dx) < max_dx, far = fabs(dx) > max_dx - 0.5;
        double ep1 = 0., ep2 = 0., ep01 = 0., ep02 = 0., q1 = 0., q2 = 0.;
        if (near) {
            const double ld = lvg_log10(delta);
            const OvIdx A = ov_index(P, G, g1, ld, g2 / g1, dx), B = ov_index(P, G, g2, ld, g1 / g2, -dx);
            double v1[16], v2[16], w1[16], w2[16];
            ov_load(P, P.ov_p1, A, v1);
            ov_load(P, P.ov_p1, B, v2);
            ov_load(P, P.ov_p2, A, w1);
            ov_load(P, P.ov_p2, B, w2);
            ep1 = ov_sum(A, v1);
            ep2 = ov_sum(B, v2);
            q1 = ov_sum(A, w1);
            q2 = ov_sum(B, w2);
        }
        if (far) {
            const EscIdx A = esc_index(P, G, g1, delta), B = esc_index(P, G, g2, delta);
            double v1[4], v2[4];
            esc_load(P, A, v1);
            esc_load(P, B, v2);
            ep01 = esc_sum(A, v1);
            ep02 = esc_sum(B, v2);
        }
        if (fabs(dx) > max_dx) { ep1 = ep01; ep2 = ep02; }
        else if (far) {
            c = 2. * (max_dx - fabs(dx));
            ep1 = ep01 * (1. - c) + ep1 * c;
            ep2 = ep02 * (1. - c) + ep2 * c;
        }
        double i1 = em1 / op1 * ep1;
        double i2 = em2 / op2 * ep2;
        if (near) {
            ep1 = q1;
            ep2 = q2;
            if (far) {
                c = 2. * (max_dx - fabs(dx));
                ep1 *= c; ep2 *= c;
            }
            i1 += em2 / op2 * ep1;
            i2 += em1 / op1 * ep2;
        }
        sm.y[2 * n1] = a1 * (1. + i1);
        sm.y[2 * n1 + 1] = b1 * i1;
        sm.y[2 * n2] = a2 * (1. + i2);
        sm.y[2 * n2 + 1] = b2 * i2;
    }
}

// LU with partial pivoting of the register rows a (lane = physical row) and the
// right-hand side rb, then back substitution; x[k] (LDS) receives solution k.
// Same operation sequence as oracle_lu_solve: pivot = first maximum |a_ik| in the
// oracle's (physically swapped) row order, tracked here as each row's logical
// position lp; every a_ij receives fma(-l_ik, u_kj, a_ij) for k ascending; x_k =
// b_k / u_kk and b_i = fma(-u_ik, x_k, b_i) for k descending.
#ifndef LVG_WAVE_LOOKAHEAD
#define LVG_WAVE_LOOKAHEAD 1          // next column's pivot reduction overlapped with this column's update
#endif
#ifndef LVG_WAVE_LDS_BCAST
#define LVG_WAVE_LDS_BCAST 0          // 1: pivot row broadcast through LDS (measured slower than v_readlane)
#endif
template <int NM>
__device__ __forceinline__ void wave_lu_solve(double (&a)[NM], double rb, int N, double *x, double *pb) {
    const int ln = lane_id();
    TSTAMP(tf0);
    bool act = ln < N;
    int lp = ln;
#if LVG_WAVE_LOOKAHEAD
    // Look-ahead pivot search: column c+1 is updated first and its max-key reduction (a
    // dependent DPP chain) is issued before the rest of column c's row update, so the two
    // overlap. Same pivots and the same fma per element as the plain loop below.
    unsigned khi, klo, H;
    auto col_key = [&](int c, double v) {
        const double av = fabs(v);
        const unsigned long long bits = (act && av == av) ? (unsigned long long)__double_as_longlong(av) : 0ull;
        const bool dnan = act && lp == c && av != av;
        khi = dnan ? 0xffffffffu : act ? ((unsigned)(bits >> 32) | 0x80000000u) : 0u;
        klo = dnan ? 0xffffffffu : (unsigned)bits;
    };
    col_key(0, a[0]);
    H = wave_max_u32(khi);
#pragma unroll
    for (int c = 0; c < NM; c++) {
        if (c < N) {
            const unsigned long long tie = __ballot(khi == H);
            int pl;
            if (__popcll(tie) == 1) {
                pl = __ffsll((long long)tie) - 1;
            } else {
                const unsigned Lw = wave_max_u32(khi == H ? klo : 0u);
                const unsigned X = wave_max_u32((khi == H && klo == Lw && act) ? ~(unsigned)lp : 0u);
                const int wmin = (int)~X;
                pl = __ffsll((long long)__ballot(act && khi == H && klo == Lw && lp == wmin)) - 1;
            }
            pl = __builtin_amdgcn_readfirstlane(pl);
            const int plp = __builtin_amdgcn_readlane(lp, pl);
            const double piv = readlane_d(a[c], pl);
            const double bc = readlane_d(rb, pl);
            if (ln == pl) { act = false; lp = c; }
            else if (lp == c) lp = plp;
            const double l = a[c] / piv;
            if (c + 1 < NM) {
                const double u = readlane_d(a[c + 1], pl);
                a[c + 1] = act ? fma(-l, u, a[c + 1]) : a[c + 1];
                col_key(c + 1, a[c + 1]);
                H = wave_max_u32(khi);
            }
#pragma unroll
            for (int j = c + 2; j < NM; j++) {
                const double u = readlane_d(a[j], pl);
                a[j] = act ? fma(-l, u, a[j]) : a[j];
            }
            if (act) { a[c] = l; rb = fma(-l, bc, rb); }
        }
    }
#else
#pragma unroll
    for (int c = 0; c < NM; c++) {
        if (c < N) {
            const double av = fabs(a[c]);
            const unsigned long long bits = (act && av == av) ? (unsigned long long)__double_as_longlong(av) : 0ull;
            // oracle_lu_solve: amax seeded with |a_kk|, replaced on a strict '>' -> a NaN below
            // never wins, a NaN on the diagonal (logical position c) always does
            const bool dnan = act && lp == c && av != av;
            const unsigned hi = dnan ? 0xffffffffu : act ? ((unsigned)(bits >> 32) | 0x80000000u) : 0u;
            const unsigned lo = dnan ? 0xffffffffu : (unsigned)bits;
            const unsigned H = wave_max_u32(hi);
            const unsigned long long tie = __ballot(hi == H);
            int pl;
            if (__popcll(tie) == 1) {
                pl = __ffsll((long long)tie) - 1;
            } else {
                const unsigned Lw = wave_max_u32(hi == H ? lo : 0u);
                const unsigned X = wave_max_u32((hi == H && lo == Lw && act) ? ~(unsigned)lp : 0u);
                const int wmin = (int)~X;
                pl = __ffsll((long long)__ballot(act && hi == H && lo == Lw && lp == wmin)) - 1;
            }
            pl = __builtin_amdgcn_readfirstlane(pl);
            const int plp = __builtin_amdgcn_readlane(lp, pl);
            double piv, bc;
            if (LVG_WAVE_LDS_BCAST) {
                // the pivot lane stores its row from column c (16-byte pairs from c & ~1) and
                // its b; every lane reads them back (LDS is in order within a wave)
                const int c2 = c & ~1;
                if (ln == pl) {
#pragma unroll
                    for (int j = c2; j < NM; j += 2)
                        *reinterpret_cast<double2 *>(pb + j) = make_double2(a[j], j + 1 < NM ? a[j + 1] : 0.);
                    pb[NM + (NM & 1)] = rb;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double u[NM];
#pragma unroll
                for (int j = c2; j < NM; j += 2) {
                    const double2 v = *reinterpret_cast<const double2 *>(pb + j);
                    u[j] = v.x;
                    if (j + 1 < NM) u[j + 1] = v.y;
                }
                piv = u[c];
                bc = pb[NM + (NM & 1)];
                if (ln == pl) { act = false; lp = c; }
                else if (lp == c) lp = plp;
                const double l = a[c] / piv;
#pragma unroll
                for (int j = c + 1; j < NM; j++)
                    if (act) a[j] = fma(-l, u[j], a[j]);
                if (act) { a[c] = l; rb = fma(-l, bc, rb); }
                __builtin_amdgcn_wave_barrier();    // reads of pb done before the next column's stores
            } else {
                piv = readlane_d(a[c], pl);
                bc = readlane_d(rb, pl);
                if (ln == pl) { act = false; lp = c; }
                else if (lp == c) lp = plp;
                const double l = a[c] / piv;
#pragma unroll
                for (int j = c + 1; j < NM; j++) {
                    const double u = readlane_d(a[j], pl);
                    if (act) a[j] = fma(-l, u, a[j]);
                }
                if (act) { a[c] = l; rb = fma(-l, bc, rb); }
            }
        }
    }
#endif
    TACC(PH_PANEL, tf0);
    TSTAMP(tb0);
#pragma unroll
    for (int k = NM - 1; k >= 0; k--) {
        if (k < N) {
            const int ow = __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(ln < N && lp == k)) - 1);
            const double xk = readlane_d(rb / a[k], ow);
            if (ln == ow) rb = xk;
            else if (lp < k) rb = fma(-a[k], xk, rb);
        }
    }
    if (ln < N) x[lp] = rb;
    TACC(PH_BACKSUB, tb0);
}

// Rows of the boundary-layer matrix B (iteration_control.cpp:52-91) into registers:
// diagonal = minus the ascending column sum, row 0 <- 1.
template <int NM>
__device__ __forceinline__ void wave_boundary_rows(const double *B, int N, double (&a)[NM]) {
    const int ln = lane_id(), i = ln < N ? ln : 0;
    double d = 0.;
    for (int r = 0; r < N; r++)
        if (r != i) d = d - B[r * N + i];
#pragma unroll
    for (int j = 0; j < NM; j++) {
        double v = (j < N) ? B[i * N + j] : 0.;
        if (j == i) v = d;
        if (i == 0) v = 1.;
        a[j] = v;
    }
}

// iteration_control (iteration_control.h:84-242) per wave: as the block versions in
// lvg_kernels.hip, with lanes for threads and wave_sync for barriers.
__device__ __forceinline__ void wave_accel_step(Ctl &C, Slot &S, int N, WaveLayer &sm) {
    const int t = lane_id();
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
#if LVG_WAVE_ACCEL_BATCH
        // the ring reads of 8 levels issued together (one round trip per block), the sum
        // still taken for k ascending
        const double *rjj = (j >= 0) ? rj : ri;
        for (int k0 = 0; k0 < N; k0 += 8) {
            double pv[8], r0v[8], riv[8], rjv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int k = (k0 + u < N) ? k0 + u : k0;
                pv[u] = p0[k]; r0v[u] = r0[k]; riv[u] = ri[k]; rjv[u] = rjj[k];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (k0 + u < N) {
                    double w = pv[u] + 1.e-99;
                    double num = (j >= 0) ? (r0v[u] - riv[u]) * (r0v[u] - rjv[u]) : (r0v[u] - riv[u]) * r0v[u];
                    a = a + num / (w * w);
                }
            }
        }
#else
        for (int k = 0; k < N; k++) {
            double w = p0[k] + 1.e-99;
            double num = (j >= 0) ? (r0[k] - ri[k]) * (r0[k] - rj[k]) : (r0[k] - ri[k]) * r0[k];
            a = a + num / (w * w);
        }
#endif
        sm.hist_acc[t] = a;
    }
    wave_sync();
    if (t == 0) {
        double Am[4][4], bv[4];
        for (int i = 0; i < np; i++) {
            for (int j = 0; j < np; j++) Am[i][j] = sm.hist_acc[i * np + j];
            bv[i] = sm.hist_acc[np * np + i];
        }
        for (int k = 0; k < np; k++) {
            int p = k;
            double amax = fabs(Am[k][k]);
            for (int i = k + 1; i < np; i++) if (fabs(Am[i][k]) > amax) { amax = fabs(Am[i][k]); p = i; }
            if (p != k) {
                for (int j = 0; j < np; j++) { double x = Am[k][j]; Am[k][j] = Am[p][j]; Am[p][j] = x; }
                double x = bv[k]; bv[k] = bv[p]; bv[p] = x;
            }
            double piv = Am[k][k];
            for (int i = k + 1; i < np; i++) {
                double l = Am[i][k] / piv;
                Am[i][k] = l;
                for (int j = k + 1; j < np; j++) Am[i][j] = fma(-l, Am[k][j], Am[i][j]);
                bv[i] = fma(-l, bv[k], bv[i]);
            }
        }
        for (int k = np - 1; k >= 0; k--) {
            bv[k] /= Am[k][k];
            double x = bv[k];
            for (int i = 0; i < k; i++) bv[i] = fma(-Am[i][k], x, bv[i]);
        }
        double sum = 0.;
        for (int i = 0; i < np; i++) { sum = sum + bv[i]; sm.hist_acc[16 + i] = bv[i]; }
        sm.hist_acc[31] = sum;
    }
    wave_sync();
    const double sum = sm.hist_acc[31];
    for (int k = t; k < N; k += 64) {
        double a = (1. - sum) * p0[k];
#if LVG_WAVE_ACCEL_BATCH
        double pv[4];                   // np <= 4 (accel_nb <= 5, checked by the host)
#pragma unroll
        for (int i = 0; i < 4; i++) pv[i] = (i < np) ? ring(S.prev, C.hp, i + 1, N)[k] : 0.;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (i < np) a = a + sm.hist_acc[16 + i] * pv[i];
#else
        for (int i = 0; i < np; i++) a = a + sm.hist_acc[16 + i] * ring(S.prev, C.hp, i + 1, N)[k];
#endif
        sm.pold[k] = a;
    }
    wave_sync();
}

__device__ __forceinline__ void wave_start_pass(Ctl &C, Slot &S, const LvgLaunch &Lc, int N, int max_nb, int accel) {
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
    if (lane_id() < N) S.opt[lane_id()] = 0.;
    wave_sync();
}

__device__ __forceinline__ void wave_next_step_pre(Ctl &C, Slot &S, int N, WaveLayer &sm) {
    const int t = lane_id();
    C.hp = (C.hp + NHIST - 1) & (NHIST - 1);
    C.np++;
    if (t < N) ring(S.prev, C.hp, 0, N)[t] = sm.pold[t];
    wave_sync();
    if (C.acceleration && (C.iter_nb == C.accel_start || C.nb_after_accel == C.accel_period)) {
        wave_sync_global();             // the rings are read across lanes
        wave_accel_step(C, S, N, sm);
        C.nb_after_accel = 0;
    }
}

__device__ __forceinline__ void wave_next_step_post(Ctl &C, Slot &S, int N, WaveLayer &sm, double eq) {
    const int t = lane_id();
    C.eq_error = eq;
    if (C.acceleration && C.iter_nb >= C.accel_start) C.nb_after_accel++;
    const bool better = C.eq_error < C.best_eq;
    if (better) C.best_eq = C.eq_error;
    C.hr = (C.hr + NHIST - 1) & (NHIST - 1);
    C.nr++;
    double pe = 0., re = 0.;
    if (t < N) {
        const double r = sm.pnew[t] - sm.pold[t];
        ring(S.res, C.hr, 0, N)[t] = r;
        pe = fmax(pe, fabs(r));
        re = fmax(re, fabs(r / (sm.pold[t] + 1.e-99)));
        if (better) S.opt[t] = sm.pold[t];
    }
    C.pop_error = wave_max(pe);
    C.rel_error = wave_max(re);
    if (C.nr > C.nb_prev + 1) C.nr = C.nb_prev + 1;
    if (C.np > C.nb_prev + 1) C.np = C.nb_prev + 1;
    wave_sync();
    if (t < N) {
        if (C.iter_nb < C.max_iter - 1) sm.pold[t] = sm.pnew[t];
        else sm.pold[t] = S.opt[t];
    }
    if (C.iter_nb >= C.max_iter - 1) C.eq_error = C.best_eq;
    C.iter_nb++;
    wave_sync();
}

// One layer of calc_molecular_populations (radiative_transfer.cpp:236-288), one wave.
// from_prev: warm chain and the chain's previous layer converged (:247-249). Returns is_found.
template <int NM>
__device__ __forceinline__ bool wave_solve_layer(const LvgDevProblem &P, const LvgLaunch &Lc, const WaveShared &sh,
                                                 WaveLayer &sm, const EscGrids &G, const int *li, int ldk, double *K,
                                                 Slot &S, int l, bool from_prev) {
    const int N = P.N, t = lane_id();
    const LvgModeLines &M = Lc.line_overlap ? P.overlap : P.plain;
    TSTAMP(ts0);
    if (t == 0) layer_scalars(P, Lc, l, sm);
    wave_sync();
    double *pops = Lc.pops + (int64_t)l * N;
    lvg_layer_status *st = reinterpret_cast<lvg_layer_status *>(Lc.status) + l;
    const bool need_boundary = (Lc.init != LVG_INIT_GIVEN);
    wave_collisions(P, sh, sm, K, ldk, (need_boundary && !from_prev) ? S.A : nullptr);
    // line invariants after the y region of the slot (host: ensure_workspace)
    const int inv_cap = P.plain.nb_lines > P.overlap.nb_lines ? P.plain.nb_lines : P.overlap.nb_lines;
    double *inv = S.y + 2 * inv_cap + 64;
    if (LVG_WAVE_LINE_INV) wave_line_invariants(P, G, M, sm, Lc.line_overlap != 0, inv, inv_cap);
    if (LVG_WAVE_LINE_INV || (need_boundary && !from_prev)) wave_sync_global();   // B is read across lanes
    else wave_sync();
    TACC(PH_SETUP, ts0);
    if (!need_boundary) {
        if (t < N) { sm.pold[t] = pops[t]; S.given[t] = pops[t]; }
        wave_sync();
    } else if (from_prev) {
        // the previous layer's populations were stored by this same lane
        if (t < N) { sm.pold[t] = pops[t - N]; S.given[t] = pops[t - N]; }
        wave_sync();
    }
    Ctl C;
    const int accel = Lc.acceleration;
    bool boundary = need_boundary && !from_prev, found = false;
    int iters = 0, retry = 0;
    const int row = t < N ? t : 0;
#if LVG_WAVE_KROW
    // the lane's row of K and of the line-index map, fixed for the layer, in registers
    double krow[NM];
    int lrow[NM];
#pragma unroll
    for (int j = 0; j < NM; j++) {
        const int jj = (j < N) ? j : 0;
        krow[j] = K[row * ldk + jj];
        lrow[j] = (j < N) ? li[row * ldk + jj] : -1;
    }
#endif
    if (!boundary) wave_start_pass(C, S, Lc, N, accel ? Lc.max_iter_acc : Lc.max_iter_plain, accel);
    for (;;) {
        double a[NM];
        double eq = 0.;
        // N through an opaque SGPR copy each pass: otherwise the compiler hoists every
        // N-derived lane mask and K address of the unrolled loops out of the layer loop and
        // spills them (v_writelane / v_readlane + s_nop on every use)
        int N = P.N;
        if (LVG_WAVE_OPAQUE_N && NM <= 32) asm volatile("" : "+s"(N));   // measured: helps NM=24, hurts NM=48
        if (boundary) {
            TSTAMP(tbd);
            wave_boundary_rows<NM>(S.A, N, a);
            TACC(PH_BOUNDARY, tbd);
        } else {
            TSTAMP(tc0);
            wave_next_step_pre(C, S, N, sm);
            TACC(PH_CTL, tc0);
            TSTAMP(tl0);
            // line terms y (compute_line_terms)
            if (LVG_WAVE_LINE_INV) {
                if (Lc.line_overlap) wave_line_terms_overlap_inv(P, G, M, sm, inv, inv_cap);
                else wave_line_terms_plain_inv(P, G, M, sm, inv, inv_cap);
            } else if (Lc.line_overlap) wave_line_terms_overlap(P, G, M, sm);
            else wave_line_terms_plain(P, G, M, sm);
            wave_sync();
            TACC(PH_LINES, tl0);
            TSTAMP(ta0);
            // diagonal (column_diagonals): lane d folds column d of K in the reference order.
            // Operands come in blocks of 8 (all LDS loads of a block issued before use) and
            // the data-dependent terms are selects, not branches: same operations, same order.
            double dg = 0.;
            {
                const int d = row;
                const bool il = M.diag_interleaved != 0;
#pragma unroll
                for (int r0 = 0; r0 < NM; r0 += 8) {
                    double kc[8], yc[8];
                    int lc[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int r = r0 + u;
                        if (LVG_WAVE_CLAMP) {   // unconditional LDS reads (row 0 stands in past N)
                            const int rr = (r < N) ? r : 0;
                            kc[u] = K[rr * ldk + d];
                            const int lv = li[rr * ldk + d];
                            lc[u] = (il && r < N) ? lv : -1;
                        } else {
                            kc[u] = (r < N) ? K[r * ldk + d] : 0.;
                            lc[u] = (il && r < N) ? li[r * ldk + d] : -1;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++) yc[u] = sm.y[lc[u] >= 0 ? lc[u] : 0];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int r = r0 + u;
                        if (r < N) {
                            double x = dg - kc[u];
                            x = (lc[u] >= 0) ? x - yc[u] : x;
                            dg = (r != d) ? x : dg;
                        }
                    }
                }
                if (!M.diag_interleaved)
                    for (int q = M.diag_ptr[d]; q < M.diag_ptr[d + 1]; q++) dg = dg - sm.y[M.diag_ent[q]];
            }
            // row `row` of A = K + line terms, diagonal, row 0 <- 1; residual e0 - A n
            double s = (t == 0) ? 1. : 0.;
#pragma unroll
            for (int j0 = 0; j0 < NM; j0 += 8) {
                double kc[8], yc[8], pc[8];
                int lc[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + u;
                    if (LVG_WAVE_KROW) {
#if LVG_WAVE_KROW
                        kc[u] = krow[j];
                        lc[u] = lrow[j];
                        pc[u] = sm.pold[j];
#endif
                    } else if (LVG_WAVE_CLAMP) {
                        const int jj = (j < N) ? j : 0;
                        kc[u] = K[row * ldk + jj];
                        const int lv = li[row * ldk + jj];
                        lc[u] = (j < N) ? lv : -1;
                        pc[u] = sm.pold[j];        // j < NM <= WNMAX
                    } else {
                        kc[u] = (j < N) ? K[row * ldk + j] : 0.;
                        lc[u] = (j < N) ? li[row * ldk + j] : -1;
                        pc[u] = (j < N) ? sm.pold[j] : 0.;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; u++) yc[u] = sm.y[lc[u] >= 0 ? lc[u] : 0];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + u;
                    if (j < N) {
                        double v = kc[u];
                        v = (lc[u] >= 0) ? v + yc[u] : v;
                        v = (j == row) ? dg : v;
                        v = (row == 0) ? 1. : v;
                        a[j] = v;
                        s = s - v * pc[u];
                    } else {
                        a[j] = 0.;
                    }
                }
            }
            eq = wave_max(t < N ? fabs(s) : 0.);
            TACC(PH_ASSEMBLE, ta0);
        }
        wave_lu_solve<NM>(a, t == 0 ? 1. : 0., N, sm.pnew, sm.prow);
        wave_sync();
        if (boundary) {
            if (t < N) { sm.pold[t] = sm.pnew[t]; S.given[t] = sm.pnew[t]; }
            wave_sync();
            if (Lc.dbg_mode == 2) {
                if (t < N) pops[t] = sm.pold[t];
                return false;
            }
            boundary = false;
            wave_start_pass(C, S, Lc, N, accel ? Lc.max_iter_acc : Lc.max_iter_plain, accel);
            continue;
        }
        TSTAMP(tc1);
        wave_next_step_post(C, S, N, sm, eq);
        TACC(PH_CTL, tc1);
        found = C.rel_error < Lc.min_error;
        if (C.iter_nb < C.max_iter && !found) continue;
        iters += C.iter_nb;
        if (!retry && !found && accel && Lc.allow_plain_retry) {
            retry = 1;
            if (t < N) sm.pold[t] = S.given[t];
            wave_sync();
            wave_start_pass(C, S, Lc, N, Lc.max_iter_plain, 0);
            continue;
        }
        break;
    }
    if (t < N) pops[t] = sm.pold[t];
    if (t == 0) {
        st->converged = found ? 1 : 0;
        st->iterations = iters;
        st->used_plain_retry = retry;
        st->reserved = 0;
        st->eq_error = C.eq_error;
        st->rel_error = C.rel_error;
        st->pop_error = C.pop_error;
    }
    wave_sync();
    return found;
}

template <int NM>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) solve_wave_kernel(const LvgDevProblem *__restrict__ Pp,
                                                            const LvgLaunch *__restrict__ Lp) {
    __shared__ WaveShared sh;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    const int N = P.N, ldk = N | 1, wpb = blockDim.x >> 6, w = threadIdx.x >> 6, tid = threadIdx.x;
    PH_INIT();
    const LvgModeLines &M = Lc.line_overlap ? P.overlap : P.plain;
    int *li = reinterpret_cast<int *>(lvg_wave_dyn);
    const int li_dbl = (N * ldk + 1) / 2;
    double *K = lvg_wave_dyn + li_dbl + (int64_t)w * N * ldk;
    // block-wide tables: molecule rule, escape/overlap grids, line index map
    for (int e = tid; e < LVG_MAX_CLASSES * LVG_MAX_TERMS; e += blockDim.x) {
        (&sh.ttab[0][0])[e] = (&P.terms.table[0][0])[e];
        (&sh.tcombo[0][0])[e] = (&P.terms.combo[0][0])[e];
    }
    for (int e = tid; e < LVG_MAX_CLASSES; e += blockDim.x) {
        sh.tet[e] = P.terms.etable[e];
        sh.tgrp[e] = P.terms.group[e];
    }
    const int o1 = P.esc_nd, o2 = o1 + P.esc_ng;
    const bool ov = Lc.line_overlap != 0;
    const int o3 = o2 + (ov ? P.ov_nd : 0), o4 = o3 + (ov ? P.ov_ndx : 0), o5 = o4 + (ov ? P.ov_ngr : 0),
              o6 = o5 + (ov ? P.ov_ng : 0);
    for (int e = tid; e < o6; e += blockDim.x) {
        double v;
        if (e < o1) v = P.esc_delta[e];
        else if (e < o2) v = P.esc_gamma[e - o1];
        else if (e < o3) v = P.ov_ld[e - o2];
        else if (e < o4) v = P.ov_dx[e - o3];
        else if (e < o5) v = P.ov_gr[e - o4];
        else v = P.ov_g[e - o5];
        sh.grids[e] = v;
    }
    for (int e = tid; e < N * N; e += blockDim.x) {
        const int r = e / N, d = e - r * N;
        li[r * ldk + d] = M.line_idx[e];
    }
    __syncthreads();
    const EscGrids G{sh.grids, sh.grids + o1, sh.grids + o2, sh.grids + o3, sh.grids + o4, sh.grids + o5};
    WaveLayer &sm = sh.w[w];
    Slot S = make_slot(P, Lc, blockIdx.x * wpb + w);
    const int nq = Lc.chain_off ? Lc.nb_chain : Lc.nb_lay;
    for (;;) {
        int q = 0;
        if (lane_id() == 0) q = atomicAdd(Lc.counter, 1);
        q = __builtin_amdgcn_readfirstlane(q);
        if (q >= nq) break;
        const int l = Lc.order ? Lc.order[q] : q;
        if (!Lc.chain_off) {
            wave_solve_layer<NM>(P, Lc, sh, sm, G, li, ldk, K, S, l, false);
        } else {
            // warm chain l, in layer order (one wave per chain)
            const int lo = Lc.chain_off[l], hi = Lc.chain_off[l + 1];
            bool prev = false;
            for (int k = lo; k < hi; k++) prev = wave_solve_layer<NM>(P, Lc, sh, sm, G, li, ldk, K, S, k, k > lo && prev);
        }
    }
    PH_FLUSH();
}

// host-side plan: waves per block and dynamic LDS bytes for N, or 0 if the wave
// kernel does not apply (N > 64, too many line terms or grid points for LDS)
inline size_t wave_dyn_bytes(int N, int wpb) {
    const int ldk = N | 1;
    return sizeof(double) * ((size_t)(N * ldk + 1) / 2 + (size_t)wpb * N * ldk);
}
