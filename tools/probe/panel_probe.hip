// Probe: latency of one 256 x 16 LU panel (partial pivoting, largest |v| / first row on
// ties, fma row updates) on a CU, factored
//   mode 0: by one wave holding 4 rows per lane (the product's owner-wave panel: upper-word
//           key fast path, slot select by v_cndmask, pivot row by v_readlane);
//   mode 1: by four waves holding 1 row per lane each: per column a DPP max per wave, the
//           wave's candidate (key, row, values) to LDS, one workgroup barrier, the winner's
//           row read back from LDS by every wave;
//   mode 2: as mode 1 with two waves of 2 rows per lane.
// Scenarios: one workgroup per CU, two per CU (both factoring), two per CU where the odd
// workgroups run an fp64 FMA stream (the co-resident LU's rank-16 updates).
// Every mode's factors are compared bit for bit with mode 0 and with a host restatement.
// Diagnostic only (make -C tools/probe; run on the GPU box).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <vector>

constexpr int NR = 256, CW = 16, REP = 16;

template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ unsigned dppu(unsigned x) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW, BANK, true);
}
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, dppu<0x111, 0xf, 0xf>(v));
    v = max(v, dppu<0x112, 0xf, 0xf>(v));
    v = max(v, dppu<0x113, 0xf, 0xf>(v));
    v = max(v, dppu<0x114, 0xf, 0xe>(v));
    v = max(v, dppu<0x118, 0xf, 0xc>(v));
    v = max(v, dppu<0x142, 0xa, 0xf>(v));
    v = max(v, dppu<0x143, 0xc, 0xf>(v));
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ double readlane_d(double x, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ unsigned khi(double v, bool act) {
    return act ? ((unsigned)__double2hiint(fabs(v)) | 0x80000000u) : 0u;
}
__device__ __forceinline__ unsigned klo(double v, bool act) {
    return act ? (unsigned)__double2loint(fabs(v)) : 0u;
}

struct Out { double *F; int *piv; unsigned long long *cyc, *rt; };

// ---- mode 0: one wave, 4 rows per lane -------------------------------------------------
// ablation flags (modes 3..): 1 = multiply instead of divide, 2 = no pivot search (row c),
// 4 = no slot select (pivot row read from slot 0), 8 = update column c+1 only
template <int F>
__device__ void panel_owner(const double *M, Out o, int wg) {
    const int ln = threadIdx.x & 63;
    double acc[4][CW];
    bool act[4];
    unsigned long long tsum = 0;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < REP; rep++) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const double2 *p = reinterpret_cast<const double2 *>(M + (size_t)(64 * s + ln) * CW);
#pragma unroll
            for (int j = 0; j < CW / 2; j++) { double2 v = p[j]; acc[s][2 * j] = v.x; acc[s][2 * j + 1] = v.y; }
            act[s] = true;
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma clang loop unroll(full)
        for (int c = 0; c < CW; c++) {
            int pl, ss;
            if (F & 2) { ss = 0; pl = c; goto have_pivot; }
            {
            unsigned kh[4];
#pragma unroll
            for (int s = 0; s < 4; s++) kh[s] = khi(acc[s][c], act[s]);
            const unsigned H0 = wave_max_u32(max(max(kh[0], kh[1]), max(kh[2], kh[3])));
            unsigned long long mk[4];
            int cnt = 0;
#pragma unroll
            for (int s = 0; s < 4; s++) { mk[s] = __ballot(kh[s] == H0); cnt += __popcll(mk[s]); }
            if (cnt == 1) {
                ss = mk[0] ? 0 : mk[1] ? 1 : mk[2] ? 2 : 3;
                pl = __builtin_amdgcn_readfirstlane(__ffsll((long long)(mk[0] | mk[1] | mk[2] | mk[3])) - 1);
            } else {
                // full key: lower word, then the first row (slot-major row order 64 s + lane)
                unsigned bl = 0u; int br = 0x7fffffff;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const unsigned lo = klo(acc[s][c], act[s]);
                    const bool better = kh[s] == H0 && (lo > bl || (lo == bl && 64 * s + ln < br));
                    bl = better ? lo : bl; br = better ? 64 * s + ln : br;
                }
                const unsigned Lw = wave_max_u32(bl);
                const unsigned R = wave_max_u32(bl == Lw ? ~(unsigned)br : 0u);
                const int row = (int)~R;
                ss = row >> 6; pl = row & 63;
                ss = __builtin_amdgcn_readfirstlane(ss); pl = __builtin_amdgcn_readfirstlane(pl);
            }
            }
          have_pivot:
            double pr[CW];
            {
                double sv[CW];
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) sv[j] = acc[0][j];
#pragma unroll
                for (int s = 1; s < 4; s++) {
                    if (F & 4) break;
                    const bool pick = ss == s;
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j >= c) sv[j] = pick ? acc[s][j] : sv[j];
                }
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) pr[j] = readlane_d(sv[j], pl);
            }
            const double piv = pr[c];
#pragma unroll
            for (int s = 0; s < 4; s++) {
                if (ln == pl && s == ss) act[s] = false;
                else if (act[s]) {
                    const double lv = (F & 1) ? acc[s][c] * piv : acc[s][c] / piv;
                    acc[s][c] = lv;
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j > c && (!(F & 8) || j == c + 1)) acc[s][j] = fma(-lv, pr[j], acc[s][j]);
                }
            }
            if (ln == 0 && rep == 0) o.piv[wg * CW + c] = 64 * ss + pl;
        }
        tsum += __builtin_amdgcn_s_memtime() - t0;
    }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int j = 0; j < CW; j++) o.F[((size_t)wg * NR + 64 * s + ln) * CW + j] = acc[s][j];
    if (ln == 0) { o.cyc[wg] = tsum / REP; o.rt[wg] = __builtin_amdgcn_s_memrealtime() - r0; }
}


// mode 11: as mode 0 with the rows stored per column as 4-slot vectors and the pivot row read
// by a dynamic (wave-uniform) slot index, which the compiler may lower to VGPR indexing
typedef double d8 __attribute__((ext_vector_type(8)));
#define AV(j, s) avp[(j) >> 1][2 * (s) + ((j) & 1)]
__device__ void panel_owner_idx(const double *M, Out o, int wg) {
    const int ln = threadIdx.x & 63;
    d8 avp[CW / 2];
    bool act[4];
    unsigned long long tsum = 0;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < REP; rep++) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const double2 *p = reinterpret_cast<const double2 *>(M + (size_t)(64 * s + ln) * CW);
#pragma unroll
            for (int j = 0; j < CW / 2; j++) { double2 v = p[j]; AV(2 * j, s) = v.x; AV(2 * j + 1, s) = v.y; }
            act[s] = true;
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma clang loop unroll(full)
        for (int c = 0; c < CW; c++) {
            unsigned kh[4];
#pragma unroll
            for (int s = 0; s < 4; s++) kh[s] = khi(AV(c, s), act[s]);
            const unsigned H0 = wave_max_u32(max(max(kh[0], kh[1]), max(kh[2], kh[3])));
            unsigned long long mk[4];
            int cnt = 0;
#pragma unroll
            for (int s = 0; s < 4; s++) { mk[s] = __ballot(kh[s] == H0); cnt += __popcll(mk[s]); }
            int pl, ss;
            if (cnt == 1) {
                ss = mk[0] ? 0 : mk[1] ? 1 : mk[2] ? 2 : 3;
                pl = __builtin_amdgcn_readfirstlane(__ffsll((long long)(mk[0] | mk[1] | mk[2] | mk[3])) - 1);
            } else {
                unsigned bl = 0u; int br = 0x7fffffff;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const unsigned lo = klo(AV(c, s), act[s]);
                    const bool better = kh[s] == H0 && (lo > bl || (lo == bl && 64 * s + ln < br));
                    bl = better ? lo : bl; br = better ? 64 * s + ln : br;
                }
                const unsigned Lw = wave_max_u32(bl);
                const unsigned R = wave_max_u32(bl == Lw ? ~(unsigned)br : 0u);
                const int row = (int)~R;
                ss = row >> 6; pl = row & 63;
            }
            ss = __builtin_amdgcn_readfirstlane(ss); pl = __builtin_amdgcn_readfirstlane(pl);
            double pr[CW];
#pragma unroll
            for (int j = 0; j < CW; j++) if (j >= c) pr[j] = readlane_d(AV(j, ss), pl);
            const double piv = pr[c];
#pragma unroll
            for (int s = 0; s < 4; s++) {
                if (ln == pl && s == ss) act[s] = false;
                else if (act[s]) {
                    const double lv = AV(c, s) / piv;
                    AV(c, s) = lv;
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j > c) AV(j, s) = fma(-lv, pr[j], AV(j, s));
                }
            }
            if (ln == 0 && rep == 0) o.piv[wg * CW + c] = 64 * ss + pl;
        }
        tsum += __builtin_amdgcn_s_memtime() - t0;
    }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int j = 0; j < CW; j++) o.F[((size_t)wg * NR + 64 * s + ln) * CW + j] = AV(j, s);
    if (ln == 0) { o.cyc[wg] = tsum / REP; o.rt[wg] = __builtin_amdgcn_s_memrealtime() - r0; }
}

// ---- modes 1 / 2: NWV waves, SL rows per lane each (rows 64 (SL w + s) + lane) ----------
struct Cand { unsigned hi, lo; int row, pad; double v[CW]; };
template <int NWV>
__device__ void panel_dist(const double *M, Out o, int wg, Cand (*cd)[4]) {
    constexpr int SL = 4 / NWV;
    const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w >= NWV) { for (int rep = 0; rep < REP; rep++) for (int c = 0; c < CW; c++) __syncthreads(); return; }
    double a[SL][CW];
    bool act[SL];
    unsigned long long tsum = 0;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < REP; rep++) {
#pragma unroll
        for (int s = 0; s < SL; s++) {
            const double2 *p = reinterpret_cast<const double2 *>(M + (size_t)(64 * (SL * w + s) + ln) * CW);
#pragma unroll
            for (int j = 0; j < CW / 2; j++) { double2 v = p[j]; a[s][2 * j] = v.x; a[s][2 * j + 1] = v.y; }
            act[s] = true;
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma clang loop unroll(full)
        for (int c = 0; c < CW; c++) {
            // the wave's candidate: upper word, then lower word, then the first row
            unsigned kh[SL];
#pragma unroll
            for (int s = 0; s < SL; s++) kh[s] = khi(a[s][c], act[s]);
            unsigned hm = kh[0];
#pragma unroll
            for (int s = 1; s < SL; s++) hm = max(hm, kh[s]);
            const unsigned H = wave_max_u32(hm);
            unsigned long long mk[SL];
            int cnt = 0;
#pragma unroll
            for (int s = 0; s < SL; s++) { mk[s] = __ballot(kh[s] == H); cnt += __popcll(mk[s]); }
            int pl, ss;
            unsigned Lw;
            if (cnt == 1) {
                ss = 0;
#pragma unroll
                for (int s = SL - 1; s > 0; s--) if (mk[s]) ss = s;
                unsigned long long m = 0;
#pragma unroll
                for (int s = 0; s < SL; s++) m |= mk[s];
                pl = __builtin_amdgcn_readfirstlane(__ffsll((long long)m) - 1);
                double pv = a[0][c];
#pragma unroll
                for (int s = 1; s < SL; s++) pv = ss == s ? a[s][c] : pv;
                Lw = (unsigned)__builtin_amdgcn_readlane((int)klo(pv, true), pl);
            } else {
                unsigned bl = 0u; int br = 0x7fffffff;
#pragma unroll
                for (int s = 0; s < SL; s++) {
                    const unsigned lo = klo(a[s][c], act[s]);
                    const int r = 64 * (SL * w + s) + ln;
                    const bool better = kh[s] == H && (lo > bl || (lo == bl && r < br));
                    bl = better ? lo : bl; br = better ? r : br;
                }
                Lw = wave_max_u32(bl);
                const unsigned R = wave_max_u32(bl == Lw ? ~(unsigned)br : 0u);
                const int row = (int)~R - 64 * SL * w;
                ss = __builtin_amdgcn_readfirstlane(row >> 6); pl = __builtin_amdgcn_readfirstlane(row & 63);
            }
            Cand *my = &cd[c & 1][w];
            if (ln == pl) {
                double sv[CW];
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) sv[j] = a[0][j];
#pragma unroll
                for (int s = 1; s < SL; s++)
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j >= c) sv[j] = ss == s ? a[s][j] : sv[j];
                my->hi = H; my->lo = Lw; my->row = 64 * (SL * w + ss) + pl;
#pragma unroll
                for (int j = 0; j < CW; j++) if (j >= c) my->v[j] = sv[j];
            }
            __syncthreads();
            // the winner: largest (hi, lo), first row on a tie (waves hold ascending rows)
            unsigned bh = cd[c & 1][0].hi, bl2 = cd[c & 1][0].lo; int bw = 0;
#pragma unroll
            for (int q = 1; q < NWV; q++) {
                const unsigned h = cd[c & 1][q].hi, l = cd[c & 1][q].lo;
                const bool better = h > bh || (h == bh && l > bl2);
                bh = better ? h : bh; bl2 = better ? l : bl2; bw = better ? q : bw;
            }
            bw = __builtin_amdgcn_readfirstlane(bw);
            const Cand *wc = &cd[c & 1][bw];
            const int prow = __builtin_amdgcn_readfirstlane(wc->row);
            double pr[CW];
#pragma unroll
            for (int j = 0; j < CW; j++) if (j >= c) pr[j] = wc->v[j];
            const double piv = pr[c];
#pragma unroll
            for (int s = 0; s < SL; s++) {
                const int r = 64 * (SL * w + s) + ln;
                if (r == prow) act[s] = false;
                else if (act[s]) {
                    const double lv = a[s][c] / piv;
                    a[s][c] = lv;
#pragma unroll
                    for (int j = 0; j < CW; j++) if (j > c) a[s][j] = fma(-lv, pr[j], a[s][j]);
                }
            }
            if (threadIdx.x == 0 && rep == 0) o.piv[wg * CW + c] = prow;
        }
        tsum += __builtin_amdgcn_s_memtime() - t0;
    }
#pragma unroll
    for (int s = 0; s < SL; s++)
#pragma unroll
        for (int j = 0; j < CW; j++) o.F[((size_t)wg * NR + 64 * (SL * w + s) + ln) * CW + j] = a[s][j];
    if (threadIdx.x == 0) { o.cyc[wg] = tsum / REP; o.rt[wg] = __builtin_amdgcn_s_memrealtime() - r0; }
}

// the co-resident LU's rank-16 updates: 4 waves of back-to-back fp64 FMAs
__device__ void filler(Out o, int wg, int iters) {
    double x[16];
    for (int j = 0; j < 16; j++) x[j] = 1.0 + threadIdx.x * 1e-9 + j;
    const double b = 0.9999999, cc = 1e-9;
    for (int i = 0; i < iters; i++)
#pragma unroll
        for (int j = 0; j < 16; j++) x[j] = fma(x[j], b, cc);
    double s = 0;
    for (int j = 0; j < 16; j++) s += x[j];
    if (s == 12345.) o.F[0] = s;
    if (threadIdx.x == 0) o.cyc[wg] = 0;
}

__global__ void __launch_bounds__(256, 2) probe(const double *M, Out o, int mode, int fill_odd, int fill_iters) {
    extern __shared__ char lds_raw[];
    Cand (*cd)[4] = reinterpret_cast<Cand (*)[4]>(lds_raw);
    const int wg = blockIdx.x;
    if (fill_odd && (wg & 1)) { filler(o, wg, fill_iters); return; }
    const double *Mw = M + (size_t)wg * NR * CW;
    if (mode == 1) panel_dist<4>(Mw, o, wg, cd);
    else if (mode == 2) panel_dist<2>(Mw, o, wg, cd);
    else if (threadIdx.x < 64) {
        switch (mode) {
        case 0: panel_owner<0>(Mw, o, wg); break;
        case 3: panel_owner<1>(Mw, o, wg); break;
        case 4: panel_owner<2>(Mw, o, wg); break;
        case 5: panel_owner<4>(Mw, o, wg); break;
        case 6: panel_owner<8>(Mw, o, wg); break;
        case 7: panel_owner<1 | 2 | 4>(Mw, o, wg); break;
        case 8: panel_owner<1 | 2 | 4 | 8>(Mw, o, wg); break;
        case 9: panel_owner<2 | 4 | 8>(Mw, o, wg); break;
        case 10: panel_owner<1 | 8>(Mw, o, wg); break;
        case 11: panel_owner_idx(Mw, o, wg); break;
        }
    }
}

// host restatement: unblocked partial pivoting on the 256 x 16 panel, physical rows kept
static void host_panel(const double *M, double *F, int *piv) {
    memcpy(F, M, sizeof(double) * NR * CW);
    bool act[NR];
    for (int r = 0; r < NR; r++) act[r] = true;
    for (int c = 0; c < CW; c++) {
        int p = -1; unsigned long long best = 0;
        for (int r = 0; r < NR; r++) {
            if (!act[r]) continue;
            double av = fabs(F[r * CW + c]); unsigned long long k; memcpy(&k, &av, 8);
            if (p < 0 || k > best) { best = k; p = r; }
        }
        piv[c] = p; act[p] = false;
        for (int r = 0; r < NR; r++) {
            if (!act[r]) continue;
            const double l = F[r * CW + c] / F[p * CW + c];
            F[r * CW + c] = l;
            for (int j = c + 1; j < CW; j++) F[r * CW + j] = fma(-l, F[p * CW + j], F[r * CW + j]);
        }
    }
}

int main(int argc, char **argv) {
    const int NWG = 1024;
    std::vector<double> M((size_t)NWG * NR * CW);
    srand(12345);
    for (auto &v : M) v = (rand() / (double)RAND_MAX - 0.5) * pow(10., (rand() % 7) - 3);
    // ties in the upper word on a few workgroups (exercise the full-key path)
    for (int g = 0; g < NWG; g += 7) for (int r = 0; r < NR; r += 3) M[((size_t)g * NR + r) * CW] = 1.0 + r * 1e-14;
    double *dM, *dF; int *dP; unsigned long long *dC, *dR;
    hipMalloc(&dM, M.size() * 8); hipMalloc(&dF, M.size() * 8); hipMalloc(&dP, NWG * CW * 4); hipMalloc(&dC, NWG * 8); hipMalloc(&dR, NWG * 8);
    hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice);
    std::vector<double> F0(M.size()), F(M.size()), Fh(NR * CW);
    std::vector<int> P(NWG * CW), Ph(CW);
    std::vector<unsigned long long> C(NWG), R(NWG);
    const size_t LDS = 72 * 1024;     // the product's per-workgroup LDS: two workgroups per CU
    hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    int bad_host = 0;
    struct Sc { const char *name; int nwg, fill; } sc[] = {{"1 WG/CU", 256, 0}, {"2 WG/CU both panels", 512, 0},
                                                         {"2 WG/CU, other WG fp64 FMA", 512, 1}};
    for (int mode = 0; mode < 12; mode++) {
        for (auto &s : sc) {
            if (mode >= 3 && mode < 11 && s.nwg != 256) continue;
            Out o{dF, dP, dC, dR};
            for (int warm = 0; warm < 2; warm++) {
                hipLaunchKernelGGL(probe, dim3(s.nwg), dim3(256), LDS, 0, dM, o, mode, s.fill, 200000);
                hipDeviceSynchronize();
            }
            hipMemcpy(C.data(), dC, NWG * 8, hipMemcpyDeviceToHost); hipMemcpy(R.data(), dR, NWG * 8, hipMemcpyDeviceToHost);
            hipMemcpy(F.data(), dF, M.size() * 8, hipMemcpyDeviceToHost);
            hipMemcpy(P.data(), dP, NWG * CW * 4, hipMemcpyDeviceToHost);
            double sum = 0, rsum = 0; int n = 0;
            for (int g = 0; g < s.nwg; g++) if (!(s.fill && (g & 1))) { sum += C[g]; rsum += R[g]; n++; }
            int mism = 0;
            for (int g = 0; g < s.nwg; g++) {
                if (s.fill && (g & 1)) continue;
                if (mode == 0 && s.nwg == 256 && !s.fill) {
                    host_panel(&M[(size_t)g * NR * CW], Fh.data(), Ph.data());
                    if (memcmp(Fh.data(), &F[(size_t)g * NR * CW], NR * CW * 8) || memcmp(Ph.data(), &P[g * CW], CW * 4))
                        bad_host++;
                }
            }
            if (mode == 0 && s.nwg == 256 && !s.fill) F0 = F;
            for (int g = 0; g < 256; g++)
                if (!(s.fill && (g & 1)) && memcmp(&F0[(size_t)g * NR * CW], &F[(size_t)g * NR * CW], NR * CW * 8)) mism++;
            const double ns = rsum / n * 10. / REP;      // s_memrealtime: 100 MHz
            printf("mode %d  %-28s  %8.0f memtime ticks per panel (%5.0f per column), %7.0f ns per panel"
                   " (%4.0f ns per column)  factors != mode 0: %d\n", mode, s.name, sum / n, sum / n / CW, ns, ns / CW, mism);
        }
    }
    printf("mode 0 vs host restatement: %d of 256 panels differ\n", bad_host);
    // s_memtime tick rate against s_memrealtime (100 MHz) for the conversion to cycles
    return 0;
}
