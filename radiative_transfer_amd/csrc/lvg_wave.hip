// lvg_wave.hip — wave-per-layer solver for small molecules (N <= 64).
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
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "lvg_device.h"
#include "../../include/lvg_amd.h"
#include "../../include/lvg_math.h"

namespace lvg {

#include "lvg_common.h"

#ifdef LVG_PHASE_TIMERS
// timer build: every wave's lane 0 accumulates (LDS atomics), not just thread 0 of the block
#undef TACC
#define TACC(ph, v0) do { if ((threadIdx.x & 63) == 0) { unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    atomicAdd(&lvg_ph_lds[ph], t_ - (v0)); } } while (0)
#endif

constexpr int WYCAP = 512;        // line terms y per wave kept in LDS (host checks 2*nb_lines <= WYCAP)
constexpr int WGRID_CAP = 1024;   // escape + overlap grid doubles copied to LDS (host checks)
constexpr int WNMAX = LVG_WAVE_NMAX;

struct WaveLayer {                // per-wave LDS
    double pold[WNMAX], pnew[WNMAX], diag[WNMAX];
    int ivh[6][64];                     // grid interval hints, per lane (ov_interval_hint)
    double y[WYCAP + 1];             // y[WYCAP] = +0: the line term of a pair with no line
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

struct WaveShared {               // per-block LDS (static part)
    int8_t ttab[LVG_MAX_CLASSES][LVG_MAX_TERMS], tcombo[LVG_MAX_CLASSES][LVG_MAX_TERMS];
    int8_t tet[LVG_MAX_CLASSES], tgrp[LVG_MAX_CLASSES];
    double grids[WGRID_CAP];
    WaveLayer w[4];
};

// dynamic LDS: line index map [NM][NM|1] (int), then K [wpb][NM][NM|1] (double); rows N..NM-1 unused
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

// the plain thread index: through the opaque one (lvg_tid) solve_wave_kernel<48> spills no VGPRs
// (55 otherwise, 200 B/lane) but runs 1-2% slower (profiles/r5/variants.txt item 9)
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Collision operator of the layer (build_collision_operators, one pair per lane):
// K[s][f] = down + electrons, K[f][s] = up + electrons (LDS, stride ldk = NM | 1); the
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
// (lvg_common.h), reorganised so that a lane's independent table reads are issued
// together: the bisections run in LDS first, then every table value the lane needs
// is loaded in one round trip. Overlap: the p1 and p2 tables share the interpolation
// indices (same gamma, delta, gratio, dx), so each direction is located once.
struct OvIdx {
    int m, n, k, l;
    double y, p, u, t;
};
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

// locate_index + clamp to the interpolation interval (esc_func / overlap_esc_func)
__device__ __forceinline__ void ov_interval(const double *g, int n, double x, int &j, double &w) {
    j = locate_index(g, n, x);
    if (j < 0) { j = 0; w = 0.; }
    else if (j > n - 2) { j = n - 2; w = 1.; }
    else w = (x - g[j]) / (g[j + 1] - g[j]);
}

// the same with the lane's previous result h for this lookup (-1: none). On a non-decreasing
// grid at most one l has g[l] <= x < g[l+1] (or l = n-2 with x = g[n-1]), and locate_index's
// bisection returns that l, so when h still brackets x it IS the bisection's answer and the
// bisection is skipped. Converging populations move gamma less and less, so late iterations
// mostly hit. mono: the grids were checked non-decreasing (solve_wave_kernel) and h is this
// lane's own record (its first unit); otherwise the plain bisection, h untouched.
__device__ __forceinline__ void ov_interval_hint(const double *g, int n, double x, int &j, double &w, int &h,
                                                 bool mono) {
    const int p = h;
    const bool hit = mono && p >= 0 && p <= n - 2 && g[p] <= x && (x < g[p + 1] || (p == n - 2 && x == g[n - 1]));
    j = hit ? p : locate_index(g, n, x);
    if (mono) h = j;
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
        ov_interval(G.ed, P.esc_nd, delta, k, t);   // esc_func's delta part
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

// plain scheme from the invariants: B units per lane per pass, stores last
__device__ __forceinline__ void wave_line_terms_plain(const LvgDevProblem &P, const EscGrids &G,
                                                      const LvgModeLines &M, WaveLayer &sm, const double *inv,
                                                      int cap, bool mono) {
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
            // esc_func's gamma part; the lane's first B units keep their intervals as hints
            ov_interval_hint(G.eg, P.esc_ng, gamma, ix[b].l, ix[b].u, sm.ivh[b][t], mono && q0 < 64);
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

// overlap scheme from the invariants (intensity_single / intensity_pair sequences).
// One wave holds every unit at once at the BASELINE sizes, so the lane-divergent paths (single
// lines, near pairs, far pairs) would run one after the other with their latency chains
// (record -> grid bisections in LDS -> table fetch) exposed in turn. Instead every lane runs all
// of them with clamped indices and the results are selected: a single line is a far-only pair
// with no second line (its own opacity expression, intensity_single), near / far / mixed pairs
// take the same operations in the same order as intensity_pair. Same values bit for bit; the
// bisections and table fetches of all paths are in flight together.
__device__ __forceinline__ void wave_line_terms_overlap(const LvgDevProblem &P, const EscGrids &G,
                                                        const LvgModeLines &M, WaveLayer &sm, const double *inv,
                                                        int cap, bool mono) {
    const double max_dx = 4.;
    const double *pop = sm.pold;
    for (int q = lane_id(); q < M.nb_units; q += 64) {
        TSTAMP(lt0);
        double f[WI_ALL];
#pragma unroll
        for (int i = 0; i < WI_ALL; i++) f[i] = inv[i * cap + q];
        const int n1 = (int)f[WI_N1], n2 = (int)f[WI_N2];
        const bool pair = n2 >= 0;
        // a single line's pair fields are not written (wave_line_invariants): indices clamped
        const int u1 = (int)f[WI_U1], l1 = (int)f[WI_L1];
        const int u2 = pair ? (int)f[WI_U2] : 0, l2 = pair ? (int)f[WI_L2] : 0;
        const double c0 = f[WI_C], a1 = f[WI_A1], b1 = f[WI_B1];
        const double a2 = pair ? f[WI_A2] : 0., b2 = pair ? f[WI_B2] : 0.;
        const double adx = pair ? fabs(f[WI_DX]) : 2. * max_dx;
        const double em1 = c0 * a1 * pop[u1];
        double op1 = pair ? c0 * (b1 * pop[l1] - a1 * pop[u1]) + MIN_LINE_OPACITY
                          : c0 * b1 * pop[l1] - em1 + MIN_LINE_OPACITY;
        const double em2 = c0 * a2 * pop[u2];
        double op2 = c0 * (b2 * pop[l2] - a2 * pop[u2]) + MIN_LINE_OPACITY;
        if (op1 < 0.) op1 *= INV_TRANS_FACTOR;
        if (op2 < 0.) op2 *= INV_TRANS_FACTOR;
        const double g1 = fabs(sm.vgrad) / (sm.vw * op1), g2 = fabs(sm.vgrad) / (sm.vw * op2);
        const bool near = adx < max_dx, far = adx > max_dx - 0.5;
        TACC(PH_T_FETCH, lt0);      // timer build: record, populations, opacities, gammas
        TSTAMP(lt1);
        // near: the 4-D overlap tables in both directions
        OvIdx A, B;
        A.m = B.m = near ? (int)f[WI_OM] : 0;
        A.y = B.y = f[WI_OY];
        A.n = near ? (int)f[WI_AN] : 0; A.p = f[WI_AP];
        B.n = near ? (int)f[WI_BN] : 0; B.p = f[WI_BP];
        // the lane's first unit keeps its intervals of the previous iteration as hints
        const bool hm = mono && q < 64;
        int (&hint)[6][64] = sm.ivh;
        const int ln = q & 63;
        ov_interval_hint(G.og, P.ov_ng, g1, A.l, A.u, hint[0][ln], hm);
        ov_interval_hint(G.ogr, P.ov_ngr, g2 / g1, A.k, A.t, hint[1][ln], hm);
        ov_interval_hint(G.og, P.ov_ng, g2, B.l, B.u, hint[2][ln], hm);
        ov_interval_hint(G.ogr, P.ov_ngr, g1 / g2, B.k, B.t, hint[3][ln], hm);
        // far (and single): the escape table in both directions
        EscIdx FA, FB;
        FA.k = FB.k = (int)f[WI_EK];
        FA.t = FB.t = f[WI_ET];
        ov_interval_hint(G.eg, P.esc_ng, g1, FA.l, FA.u, hint[4][ln], hm);
        ov_interval_hint(G.eg, P.esc_ng, g2, FB.l, FB.u, hint[5][ln], hm);
        TACC(PH_T_SOLVE, lt1);      // grid intervals
        TSTAMP(lt2);
        double v1[16], v2[16], w1[16], w2[16], e1[4], e2[4];
        ov_load(P, P.ov_p1, A, v1);
        ov_load(P, P.ov_p1, B, v2);
        ov_load(P, P.ov_p2, A, w1);
        ov_load(P, P.ov_p2, B, w2);
        esc_load(P, FA, e1);
        esc_load(P, FB, e2);
        double ep1 = near ? ov_sum(A, v1) : 0., ep2 = near ? ov_sum(B, v2) : 0.;
        const double q1 = near ? ov_sum(A, w1) : 0., q2 = near ? ov_sum(B, w2) : 0.;
        const double ep01 = far ? esc_sum(FA, e1) : 0., ep02 = far ? esc_sum(FB, e2) : 0.;
        TACC(PH_T_STAGE, lt2);      // table fetch and interpolation sums
        TSTAMP(lt3);
        const double cm = 2. * (max_dx - adx);
        if (adx > max_dx) { ep1 = ep01; ep2 = ep02; }
        else if (far) {
            ep1 = ep01 * (1. - cm) + ep1 * cm;
            ep2 = ep02 * (1. - cm) + ep2 * cm;
        }
        double i1 = em1 / op1 * ep1;
        double i2 = em2 / op2 * ep2;
        if (near) {
            double r1 = q1, r2 = q2;
            if (far) { r1 *= cm; r2 *= cm; }
            i1 += em2 / op2 * r1;
            i2 += em1 / op1 * r2;
        }
        sm.y[2 * n1] = a1 * (1. + i1);
        sm.y[2 * n1 + 1] = b1 * i1;
        if (pair) {
            sm.y[2 * n2] = a2 * (1. + i2);
            sm.y[2 * n2 + 1] = b2 * i2;
        }
        TACC(PH_P_RED, lt3);        // intensities and stores
    }
}

// LU with partial pivoting of the register rows a (lane = physical row) and the
// right-hand side rb, then back substitution; x[k] (LDS) receives solution k.
// Same operation sequence as oracle_lu_solve: pivot = first maximum |a_ik| in the
// oracle's (physically swapped) row order, tracked here as each row's logical
// position lp; every a_ij receives fma(-l_ik, u_kj, a_ij) for k ascending; x_k =
// b_k / u_kk and b_i = fma(-u_ik, x_k, b_i) for k descending.
// Look-ahead pivot search: column c+1 is updated first and its max-key reduction (a
// dependent DPP chain) is issued before the rest of column c's row update, so the two
// overlap.
template <int NM>
__device__ __forceinline__ void wave_lu_solve(double (&a)[NM], double rb, int N, double *x) {
    const int ln = lane_id();
    TSTAMP(tf0);
    bool act = ln < N;
    int lp = ln;
    unsigned khi, klo, H;
    pivot_key(a[0], act, lp == 0, khi, klo);
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
                pivot_key(a[c + 1], act, lp == c + 1, khi, klo);
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
        const double *rj = (j >= 0) ? ring(S.res, C.hr, j + 1, N) : ri;
        double a = 0.;
        // the ring reads of 8 levels issued together (one round trip per block), the sum
        // still taken for k ascending
        for (int k0 = 0; k0 < N; k0 += 8) {
            double pv[8], r0v[8], riv[8], rjv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int k = (k0 + u < N) ? k0 + u : k0;
                pv[u] = p0[k]; r0v[u] = r0[k]; riv[u] = ri[k]; rjv[u] = rj[k];
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
        sm.hist_acc[t] = a;
    }
    wave_sync();
    if (t == 0) accel_solve_small(sm.hist_acc, np);
    wave_sync();
    const double sum = sm.hist_acc[31];
    for (int k = t; k < N; k += 64) {
        double a = (1. - sum) * p0[k];
        double pv[4];                   // np <= 4 (accel_nb <= 5, checked by the host)
#pragma unroll
        for (int i = 0; i < 4; i++) pv[i] = (i < np) ? ring(S.prev, C.hp, i + 1, N)[k] : 0.;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (i < np) a = a + sm.hist_acc[16 + i] * pv[i];
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
                                                 Slot &S, int l, bool from_prev, bool mono) {
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
    wave_line_invariants(P, G, M, sm, Lc.line_overlap != 0, inv, inv_cap);
    wave_sync_global();             // B and the invariants are read across lanes
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
    // the lane's row of K and of the line-index map, fixed for the layer, in registers
    double krow[NM];
    int lrow[NM];
#pragma unroll
    for (int j = 0; j < NM; j++) {
        krow[j] = K[row * ldk + j];          // +0 / -1 past N
        lrow[j] = li[row * ldk + j];
    }
    if (!boundary) wave_start_pass(C, S, Lc, N, accel ? Lc.max_iter_acc : Lc.max_iter_plain, accel);
#pragma unroll
    for (int k = 0; k < 6; k++) sm.ivh[k][t] = -1;   // no interval hints yet for this layer
    for (;;) {
        double a[NM];
        double eq = 0.;
        // N through an opaque SGPR copy each pass: otherwise the compiler hoists every
        // N-derived lane mask and K address of the unrolled loops out of the layer loop and
        // spills them (v_writelane / v_readlane + s_nop on every use). Round 5 measured it to help
        // NM = 24 and hurt NM = 48; with the padded LDS map of round 6 it also helps NM = 48
        // (SGPR spills 1058 -> 607, p-H2O -2%, profiles/r6/variants.txt item 14)
        int N = P.N;
        asm volatile("" : "+s"(N));
        int rowo = row;                  // the lane's row, recomputed masks instead of hoisted spilled ones
        asm volatile("" : "+v"(rowo));
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
            if (Lc.line_overlap) wave_line_terms_overlap(P, G, M, sm, inv, inv_cap, mono);
            else wave_line_terms_plain(P, G, M, sm, inv, inv_cap, mono);
            wave_sync();
            TACC(PH_LINES, tl0);
            TSTAMP(ta0);
            // diagonal (column_diagonals): lane d folds column d of K in the reference order.
            // Operands come in blocks of 8 (all LDS loads of a block issued before use, row 0
            // standing in past N) and the data-dependent terms are selects, not branches:
            // same operations, same order.
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
                        // rows N..NM-1 exist (allocated, unused): fixed offsets, no clamp on N
                        const int r = r0 + u;
                        kc[u] = K[r * ldk + d];
                        const int lv = li[r * ldk + d];
                        lc[u] = il ? lv : -1;
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++) yc[u] = sm.y[lc[u] >= 0 ? lc[u] : WYCAP];
                    // the skipped terms become subtractions of +0, which leave dg unchanged
                    // bit for bit, so the dependent chain is the subtractions alone
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        // K[d][d] and the rows past N are +0, their line index -1
                        dg = dg - kc[u];
                        dg = dg - yc[u];                  // +0 where no line
                    }
                }
                if (!M.diag_interleaved) {
                    // the line terms of level d in line order, entries and y read 8 at a time
                    const int q0 = M.diag_ptr[d], q1 = M.diag_ptr[d + 1];
                    for (int qb = q0; qb < q1; qb += 8) {
                        int e[8];
                        double ye[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) e[u] = (qb + u < q1) ? M.diag_ent[qb + u] : -1;
#pragma unroll
                        for (int u = 0; u < 8; u++) ye[u] = sm.y[e[u] >= 0 ? e[u] : WYCAP];
#pragma unroll
                        for (int u = 0; u < 8; u++) dg = dg - ye[u];
                    }
                }
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
                    kc[u] = krow[j];
                    lc[u] = lrow[j];
                    pc[u] = sm.pold[j];        // j < NM <= WNMAX
                }
#pragma unroll
                for (int u = 0; u < 8; u++) yc[u] = sm.y[lc[u] >= 0 ? lc[u] : WYCAP];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int j = j0 + u;
                    double v = kc[u];
                    v = v + yc[u];                        // K is never -0: K + (+0) == K
                    v = (j == rowo) ? dg : v;
                    v = (rowo == 0) ? 1. : v;
                    // columns past N: K and the populations there are +0, so v * pc is +0 (the
                    // subtraction leaves s unchanged bit for bit); a[j] past N is never read back
                    // into a column below N (pivots, updates and the back substitution stop at N)
                    a[j] = v;
                    s = s - v * pc[u];
                }
            }
            eq = wave_max(t < N ? fabs(s) : 0.);
            TACC(PH_ASSEMBLE, ta0);
        }
        wave_lu_solve<NM>(a, t == 0 ? 1. : 0., N, sm.pnew);
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
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
solve_wave_kernel(const LvgDevProblem *__restrict__ Pp, const LvgLaunch *__restrict__ Lp) {
    __shared__ WaveShared sh;
    const LvgDevProblem &P = *Pp;
    const LvgLaunch &Lc = *Lp;
    // K / line-index row stride fixed per instantiation: the per-row LDS offsets of the
    // unrolled row loops (diagonal fold) become instruction immediates instead of address
    // registers hoisted out of the layer loop (at NM = 48 those spilled, a scratch reload
    // per LDS read)
    constexpr int ldk = NM | 1;
    const int N = P.N, wpb = blockDim.x >> 6, w = threadIdx.x >> 6, tid = threadIdx.x;
    PH_INIT();
    const LvgModeLines &M = Lc.line_overlap ? P.overlap : P.plain;
    int *li = reinterpret_cast<int *>(lvg_wave_dyn);
    const int li_dbl = (NM * ldk + 1) / 2;
    double *K = lvg_wave_dyn + li_dbl + (int64_t)w * NM * ldk;
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
    // the whole NM x ldk map: rows / columns past N hold -1 (no line), so the diagonal fold and the
    // row assembly need no N masks; with K's diagonal and padding at +0 (below) and the populations
    // past N at 0, every skipped term is a subtraction of +0
    for (int e = tid; e < NM * ldk; e += blockDim.x) {
        const int r = e / ldk, d = e - r * ldk;
        li[e] = (r < N && d < N) ? M.line_idx[r * N + d] : -1;
    }
    for (int e = lane_id(); e < NM * ldk; e += 64) K[e] = 0.;     // this wave's K: diagonal and padding stay +0
    for (int e = lane_id(); e < WNMAX; e += 64) sh.w[w].pold[e] = 0.;
    if (lane_id() == 0) sh.w[w].y[WYCAP] = 0.;
    __syncthreads();
    // the gamma / gamma-ratio grids non-decreasing (a NaN fails the test): the precondition of
    // the interval hints (ov_interval_hint)
    int bad = 0;
    for (int e = tid; e < o6; e += blockDim.x) {
        const bool seg = (e >= o1 && e + 1 < o2) || (ov && ((e >= o4 && e + 1 < o5) || (e >= o5 && e + 1 < o6)));
        if (seg && !(sh.grids[e] <= sh.grids[e + 1])) bad = 1;
    }
    const bool mono = __syncthreads_or(bad) == 0;
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
            wave_solve_layer<NM>(P, Lc, sh, sm, G, li, ldk, K, S, l, false, mono);
        } else {
            // warm chain l, in layer order (one wave per chain)
            const int lo = Lc.chain_off[l], hi = Lc.chain_off[l + 1];
            bool prev = false;
            for (int k = lo; k < hi; k++)
                prev = wave_solve_layer<NM>(P, Lc, sh, sm, G, li, ldk, K, S, k, k > lo && prev, mono);
        }
    }
    PH_FLUSH();
}

// host-side plan: dynamic LDS bytes of wpb waves for N levels
inline size_t wave_dyn_bytes(int N, int wpb) {
    // solve_wave_kernel<NM>'s layout: NM rows of stride NM | 1 for the line-index map and
    // for each wave's K
    const int nm = N <= 16 ? 16 : ((N + 7) / 8) * 8, ldk = nm | 1;
    return sizeof(double) * ((size_t)(nm * ldk + 1) / 2 + (size_t)wpb * nm * ldk);
}

}  // namespace lvg

// 1 and the waves per block / dynamic LDS bytes if the wave kernel applies to N levels
// with nb_y line terms and grid_doubles escape-grid points; 0 if not.
extern "C" int lvg_wave_plan(int N, int nb_y, int grid_doubles, size_t lds_cap, int *wpb, size_t *dyn) {
    if (N < 2 || N > lvg::WNMAX || nb_y > lvg::WYCAP || grid_doubles > lvg::WGRID_CAP) return 0;
    for (int w = 4; w >= 1; w >>= 1) {
        const size_t d = lvg::wave_dyn_bytes(N, w);
        if (sizeof(lvg::WaveShared) + d <= lds_cap) { *wpb = w; *dyn = d; return 1; }
    }
    return 0;
}

// instantiations every 8 levels from 24 up (the unrolled row loops run to NM): OH-HF 24
// and p-H2O 45 run NM = 24 and 48, the reference's OH-HF 56 runs NM = 56
#define LVG_WAVE_NMS(X) X(16) X(24) X(32) X(40) X(48) X(56) X(64)
static int wave_nm(int N) { return N <= 16 ? 16 : ((N + 7) / 8) * 8; }
static const void *wave_kernel(int N) {
#define LVG_WK(NM_) if (wave_nm(N) == NM_) return reinterpret_cast<const void *>(&lvg::solve_wave_kernel<NM_>);
    LVG_WAVE_NMS(LVG_WK)
#undef LVG_WK
    return nullptr;
}

extern "C" hipError_t lvg_wave_occupancy(int N, int wpb, size_t dyn, int *blocks_per_cu) {
    const void *k = wave_kernel(N);
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * wpb, dyn);
}

extern "C" hipError_t lvg_launch_solve_wave(const LvgDevProblem *P, const LvgLaunch *L, int N, int grid, int wpb,
                                            size_t dyn, hipStream_t s) {
    const dim3 g(grid), b(64 * wpb);
#define LVG_WL(NM_) if (wave_nm(N) == NM_) hipLaunchKernelGGL(lvg::solve_wave_kernel<NM_>, g, b, dyn, s, P, L);
    LVG_WAVE_NMS(LVG_WL)
#undef LVG_WL
    return hipGetLastError();
}
extern "C" size_t lvg_wave_static_lds(void) { return sizeof(lvg::WaveShared); }

#ifdef LVG_PHASE_TIMERS
extern "C" int lvg_debug_wave_phase_cycles(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lvg::lvg_phase_cycles), sizeof(unsigned long long) * lvg::PH_SLOTS) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[lvg::PH_SLOTS] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(lvg::lvg_phase_cycles), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
