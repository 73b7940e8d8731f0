// lvg_abi.cpp — host side of the C ABI (include/lvg_amd.h): validation, the
// packer that turns an lvg_problem into the device layout of lvg_device.h,
// device memory, launches and HIP-event timing.
//
// The packer replaces the reference's object construction before the layer
// loop (radiative_transfer.cpp:614-670 for CH3OH): the molecule rule of each
// collisional_transitions subclass is compiled to per-pair term classes, the
// line list of iteration_scheme_lvg::operator() (A > 0, iteration_lvg.cpp:134)
// and the hfs_lines grouping of iteration_scheme_line_overlap::init_molecule_data
// (iteration_lvg.cpp:317-346) are flattened, and the dust cross section at each
// line energy (dust_model.cpp:473-490) is tabulated once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>
#include <cstdlib>

#include "../../include/lvg_amd.h"
#include "lvg_device.h"

extern "C" hipError_t lvg_launch_solve(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s);
extern "C" hipError_t lvg_launch_coll(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s);
extern "C" hipError_t lvg_row_order(const double *soa, int ld, int n, int row, double *keys, double *keys_sorted,
                                    int *idx, int *order, void *temp, size_t *temp_bytes, hipStream_t s);
extern "C" int lvg_wave_plan(int N, int nb_y, int grid_doubles, size_t lds_cap, int *wpb, size_t *dyn);
extern "C" hipError_t lvg_wave_occupancy(int N, int wpb, size_t dyn, int *blocks_per_cu);
extern "C" hipError_t lvg_launch_solve_wave(const LvgDevProblem *P, const LvgLaunch *L, int N, int grid, int wpb,
                                            size_t dyn, hipStream_t s);
extern "C" hipError_t lvg_launch_debug(const LvgDevProblem *P, const LvgLaunch *L, hipStream_t s);
extern "C" int lvg_kernel_max_levels(void);
extern "C" hipError_t lvg_kernel_occupancy(int *blocks_per_cu);
extern "C" hipError_t lvg_launch_lum(const LvgDevProblem *P, const LvgLaunch *L, const LvgLumArgs *A, int grid,
                                     int nb_trans, int nb_lay, hipStream_t s);
// the 512-thread instantiation for underfilled launches at N <= 256 (lvg_kernels_wide.hip)
extern "C" hipError_t lvg_launch_solve_wide(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s);
extern "C" hipError_t lvg_kernel_occupancy_wide(int *blocks_per_cu);
// the 768-thread instantiation for 256 < N <= 768 (lvg_kernels_big.hip)
extern "C" hipError_t lvg_launch_solve_big(const LvgDevProblem *P, const LvgLaunch *L, int grid, hipStream_t s);
extern "C" hipError_t lvg_launch_debug_big(const LvgDevProblem *P, const LvgLaunch *L, hipStream_t s);
extern "C" int lvg_kernel_max_levels_big(void);
extern "C" hipError_t lvg_kernel_occupancy_big(int *blocks_per_cu);
extern "C" hipError_t lvg_launch_lum_big(const LvgDevProblem *P, const LvgLaunch *L, const LvgLumArgs *A, int grid,
                                         int nb_trans, int nb_lay, hipStream_t s);
extern "C" hipError_t lvg_sched_order(const double *soa, int ld, int n, double *keys, double *keys_sorted, int *idx,
                                      int *order, void *temp, size_t *temp_bytes, hipStream_t s);
extern "C" hipError_t lvg_tr_launch(int stage, const void *args_dev, int nb_lines, int nb_lay, int nb_sel, hipStream_t s);

namespace {

thread_local std::string g_create_error;

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
};

struct ModeHost {
    std::vector<int> u, l, unit0, unit1, dptr, dent, cptr, cr, cy, li;
    std::vector<double> aul, alu, e, sigma;
    int interleaved = 1;
};

}  // namespace

// Tuning and diagnostics (not results: every setting gives bit-identical populations and
// status). Defaults, then the LVG_TUNING environment variable once at lvg_create (a spec
// that does not parse is ignored with a message on stderr: it never stops a handle from
// being created), then lvg_set_tuning, whose keys are MERGED into the current settings
// (keys it does not name keep their value; an empty spec resets to the defaults). The
// format is "key=value,key=value" with the keys below.
struct LvgTuning {
    int block_kernel = 0;      // block_kernel=1: the block kernel also for N <= 64
    int queue_order = 1;       // queue_order=0: work queue in layer order, not longest-expected-first
    int coll_ahead = 0;        // coll_ahead=1: coll_kernel builds the batch's collision operators ahead
    double coll_mem = 0.5;     // coll_mem=f: ... when they fit this fraction of the free device memory
    int coll_order = 1;        // coll_order=0: coll_kernel in layer order, not temperature order
    int blocks_per_cu = 0;     // blocks_per_cu=k: resident block-kernel workgroups per CU (0: automatic)
    int wide = 1;              // wide=0: never the 512-thread kernel; 1: when underfilled; 2: always (N <= 256)
};

struct lvg_handle {
    int device = 0;
    int N = 0;
    int nb_comp = 0;
    int has_overlap = 0;
    int cus = 0, blocks_per_cu = 1;
    int wide_bpc = 0;              // resident 512-thread workgroups per CU (0: not available)
    int big = 0;                   // N > 256: the 768-thread block kernel (lvg_kernels_big.hip)
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evc = nullptr;   // evc: end of coll_kernel
    LvgDevProblem P{};
    std::vector<DevBuf> bufs;
    // workspace
    double *ws = nullptr;
    size_t ws_bytes = 0;
    int64_t ws_stride = 0;
    int *counter = nullptr;
    size_t lds_cap = 0;            // LDS bytes per workgroup (wave kernel plan)
    int last_kernel = -1;          // lvg_last_kernel_kind: -1 none (no launch yet, or an empty batch),
                                   // 0 block, 1 wave, 2 512-thread, 3 768-thread kernel
    // scratch for host-buffer solves
    double *d_soa = nullptr, *d_pops = nullptr;
    void *d_status = nullptr;
    size_t soa_cap = 0, pops_cap = 0, status_cap = 0;
    // layer scheduling order (lvg_sched.hip)
    void *d_sched = nullptr, *d_sched_tmp = nullptr;
    size_t sched_cap = 0, sched_tmp_cap = 0;
    void *d_coll = nullptr;            // K_all, B_all of the last coll_kernel batch
    size_t coll_cap = 0;
    void *d_corder = nullptr;          // coll_kernel temperature order + its sort scratch
    size_t corder_cap = 0;
    // warm chains: offsets [nb_chain + 1] then queue order [nb_chain] (device + host staging)
    int *d_chain = nullptr;
    size_t chain_cap = 0;
    std::vector<int> chain_host;
    double last_ms = 0., last_coll_ms = 0.;
    int last_coll = 0;
    int last_launches = 0;
    // an asynchronous lvg_solve_layers_device (caller's stream) may still be running:
    // its kernel reads the launch block, the queue counter and the workspace slots, so
    // any later call on this handle is ordered after it (settle) and nothing it uses is
    // freed before it ends (drain). ev1 marks its end.
    int pending = 0;
    hipStream_t pending_stream = nullptr;
    // device-resident parameter blocks (kernels take pointers: no kernarg copies)
    LvgDevProblem *d_prob = nullptr;
    LvgLaunch *d_launch = nullptr;
    int n_launch_slots = 0;
    LvgTuning tune;
    std::string err;
    // lvg_create_devices / lvg_create_multi: the handles of the further devices (this handle is
    // the first device); lvg_solve_layers / lvg_solve_chains / lvg_boundary_layer_populations
    // split their layers over all of them, one host thread and one stream per device
    std::vector<lvg_handle *> peers;
};

namespace {

int fail(lvg_handle *h, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf; else g_create_error = buf;
    return code;
}

// "key=value,key=value" onto t (keys of LvgTuning); LVG_E_ARG on anything else
int parse_tuning(lvg_handle *h, const char *spec, LvgTuning &t) {
    if (!spec) return LVG_OK;
    std::string s(spec);
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        const std::string item = s.substr(i, j - i);
        i = j + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) return fail(h, LVG_E_ARG, "tuning item '%s' is not key=value", item.c_str());
        const std::string k = item.substr(0, eq), v = item.substr(eq + 1);
        char *end = nullptr;
        const double x = std::strtod(v.c_str(), &end);
        if (v.empty() || *end) return fail(h, LVG_E_ARG, "tuning value '%s' is not a number", v.c_str());
        if (k == "block_kernel") t.block_kernel = x != 0.;
        else if (k == "queue_order") t.queue_order = x != 0.;
        else if (k == "coll_ahead") t.coll_ahead = x != 0.;
        else if (k == "coll_mem" && x >= 0. && x <= 1.) t.coll_mem = x;
        else if (k == "coll_order") t.coll_order = x != 0.;
        else if (k == "blocks_per_cu" && x >= 0. && x <= 8.) t.blocks_per_cu = (int)x;
        else if (k == "wide" && (x == 0. || x == 1. || x == 2.)) t.wide = (int)x;
        else return fail(h, LVG_E_ARG, "unknown tuning key or bad value '%s'", item.c_str());
    }
    return LVG_OK;
}

#define HIPCHECK(h, x)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) return fail(h, LVG_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

template <class T>
int upload(lvg_handle *h, const T *src, size_t n, const T **dst) {
    DevBuf b;
    b.n = std::max<size_t>(1, n) * sizeof(T);
    if (hipMalloc(&b.p, b.n) != hipSuccess) return fail(h, LVG_E_NOMEM, "hipMalloc(%zu) failed", b.n);
    h->bufs.push_back(b);
    if (n && hipMemcpy(b.p, src, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return fail(h, LVG_E_DEVICE, "hipMemcpy H2D failed");
    *dst = static_cast<const T *>(b.p);
    return LVG_OK;
}

// dust_component::absorption (dust_model.cpp:473-490)
double dust_sigma(const lvg_dust_component &c, double energy) {
    const int n = c.nb_en;
    if (energy < c.energy[0]) return c.abs_coeff[0] * std::pow(c.energy[0] / energy, c.wvl_exp);
    if (energy > c.energy[n - 1]) return c.abs_coeff[n - 1];
    int l = 0, r = n - 1;
    while (r - l > 1) {
        int i = l + ((r - l) >> 1);
        if (c.energy[i] < energy) l = i; else r = i;
    }
    double deriv = (c.abs_coeff[l + 1] - c.abs_coeff[l]) / (c.energy[l + 1] - c.energy[l]);
    return c.abs_coeff[l] + deriv * (energy - c.energy[l]);
}

// ---- rule compiler ----------------------------------------------------------
struct TermList {
    int nt = 0;
    int table[LVG_MAX_TERMS];
    int combo[LVG_MAX_TERMS];
    int etable = -1;
    int group = LVG_MAX_TERMS;
    bool operator<(const TermList &o) const {
        if (nt != o.nt) return nt < o.nt;
        if (group != o.group) return group < o.group;
        for (int i = 0; i < nt; i++) {
            if (table[i] != o.table[i]) return table[i] < o.table[i];
            if (combo[i] != o.combo[i]) return combo[i] < o.combo[i];
        }
        return etable < o.etable;
    }
};

struct Combos {
    std::vector<std::vector<double>> w;
    int get(std::vector<double> v) {
        for (size_t i = 0; i < w.size(); i++) if (w[i] == v) return (int)i;
        w.push_back(v);
        return (int)w.size() - 1;
    }
};

enum { HE = 0, PH2 = 1, OH2 = 2, HH = 3, EE = 4 };
std::vector<double> sp(int s) { std::vector<double> v(5, 0.); v[s] = 1.; return v; }

int compile_rule(lvg_handle *h, const lvg_problem *prob, std::vector<uint8_t> &pair_class, LvgTermTable &tt) {
    const lvg_molecule &M = *prob->mol;
    const lvg_collisions &C = *prob->coll;
    const int N = M.nb_lev, nb1 = C.nb_neutral, nb2 = C.nb_neutral + C.nb_electron;
    auto covers = [&](int t, int f) { return f < C.tables[t].nb_lev; };
    Combos cb;
    // fixed combo ids first so the common ones are stable
    std::map<TermList, int> classes;
    pair_class.assign((size_t)N * (N - 1) / 2, 0);
    auto need = [&](int t, int f) -> bool {
        if (t >= nb1) return false;
        return covers(t, f);
    };
    for (int f = 1; f < N; f++) {
        for (int s = 0; s < f; s++) {
            TermList tl;
            auto add = [&](int t, std::vector<double> w) {
                tl.table[tl.nt] = t;
                tl.combo[tl.nt] = cb.get(w);
                tl.nt++;
            };
            switch (C.rule) {
            case LVG_COLL_CH3OH: {                        // coll_rates_ch3oh.cpp:484-533
                if (nb1 < 3) return fail(h, LVG_E_ARG, "CH3OH rule needs 3 neutral tables");
                for (int t = 0; t < 3; t++)
                    if (!covers(t, f)) return fail(h, LVG_E_ARG, "CH3OH table %d covers %d levels < %d", t, C.tables[t].nb_lev, N);
                if (!M.v || !M.j) return fail(h, LVG_E_ARG, "CH3OH rule needs level v and J");
                if (M.v[f] == M.v[s]) {
                    if (M.v[f] == 0 && M.j[f] <= 9 && M.j[s] <= 9) { add(1, sp(PH2)); add(2, sp(OH2)); }
                    else { std::vector<double> w(5, 0.); w[PH2] = 1.; w[OH2] = 1.; add(1, w); }
                    add(0, sp(HE));
                } else {
                    std::vector<double> w(5, 0.); w[HE] = 1.; w[PH2] = 1.; w[OH2] = 3.;
                    add(0, w);
                }
                break;
            }
            case LVG_COLL_H2O: {                          // coll_rates_h2o.cpp:530-548
                if (nb1 < 6) return fail(h, LVG_E_ARG, "H2O rule needs 6 neutral tables");
                if (f < 45) {
                    const int ts[4] = {0, 2, 3, 5};
                    const int ss[4] = {HE, PH2, OH2, HH};
                    for (int q = 0; q < 4; q++) {
                        if (!covers(ts[q], f)) return fail(h, LVG_E_ARG, "H2O table %d does not cover level %d", ts[q], f);
                        add(ts[q], sp(ss[q]));
                    }
                } else {
                    if (!covers(1, f) || !covers(4, f)) return fail(h, LVG_E_ARG, "H2O rovib tables do not cover level %d", f);
                    std::vector<double> w1(5, 0.); w1[HE] = 1.; w1[HH] = 0.2;
                    std::vector<double> w4(5, 0.); w4[PH2] = 1.; w4[OH2] = 1.;
                    add(1, w1);
                    add(4, w4);
                }
                break;
            }
            case LVG_COLL_OH:                             // coll_rates_oh.cpp:334-347
            case LVG_COLL_OH_HF: {                        // coll_rates_oh.cpp:392-407
                if (nb1 < 3) return fail(h, LVG_E_ARG, "OH rules need 3 neutral tables");
                if (C.rule == LVG_COLL_OH && !covers(0, f))
                    return fail(h, LVG_E_ARG, "OH He table must cover all levels (read unchecked, coll_rates_oh.cpp:336)");
                if (covers(0, f)) add(0, sp(HE));
                if (covers(1, f)) { tl.group = tl.nt; add(1, sp(PH2)); add(2, sp(OH2)); }
                break;
            }
            case LVG_COLL_GENERIC: {                      // coll_rates.cpp:181-197
                for (int t = 0; t < nb1; t++) {
                    if (tl.nt >= LVG_MAX_TERMS) return fail(h, LVG_E_UNSUPPORTED, "more than %d neutral tables", LVG_MAX_TERMS);
                    int spc = C.tables[t].species;
                    if (spc < 0 || spc >= LVG_NB_SPECIES) return fail(h, LVG_E_ARG, "table %d: bad species", t);
                    if (need(t, f)) add(t, sp(spc));
                }
                break;
            }
            default:
                return fail(h, LVG_E_ARG, "unknown collision rule %d", C.rule);
            }
            for (int t = nb1; t < nb2; t++)                // coll_rates.cpp:204-211
                if (covers(t, f)) { tl.etable = t; break; }
            auto it = classes.find(tl);
            int id;
            if (it == classes.end()) {
                id = (int)classes.size();
                if (id >= LVG_MAX_CLASSES) return fail(h, LVG_E_UNSUPPORTED, "too many collision term classes");
                classes[tl] = id;
            } else id = it->second;
            pair_class[(size_t)f * (f - 1) / 2 + s] = (uint8_t)id;
        }
    }
    if ((int)cb.w.size() > LVG_MAX_COMBOS) return fail(h, LVG_E_UNSUPPORTED, "too many concentration combinations");
    memset(&tt, 0, sizeof tt);
    for (int c = 0; c < LVG_MAX_CLASSES; c++) {
        for (int k = 0; k < LVG_MAX_TERMS; k++) { tt.table[c][k] = -1; tt.combo[c][k] = 0; }
        tt.etable[c] = -1;
        tt.group[c] = LVG_MAX_TERMS;
    }
    for (auto &kv : classes) {
        const TermList &tl = kv.first;
        for (int k = 0; k < tl.nt; k++) { tt.table[kv.second][k] = (int8_t)tl.table[k]; tt.combo[kv.second][k] = (int8_t)tl.combo[k]; }
        tt.etable[kv.second] = (int8_t)tl.etable;
        tt.group[kv.second] = (int8_t)tl.group;
        tt.nt_max = std::max(tt.nt_max, tl.nt);
        if (tl.etable >= 0) tt.any_e = 1;
    }
    tt.nb_combos = (int)cb.w.size();
    for (size_t i = 0; i < cb.w.size(); i++)
        for (int q = 0; q < 5; q++) tt.combo_w[i][q] = cb.w[i][q];
    return LVG_OK;
}

// ---- line lists ------------------------------------------------------------------
void add_line(ModeHost &m, const lvg_problem *prob, int u, int l) {
    const lvg_molecule &M = *prob->mol;
    const int N = M.nb_lev;
    m.u.push_back(u);
    m.l.push_back(l);
    m.aul.push_back(M.einst[(size_t)u * N + l]);
    m.alu.push_back(M.einst[(size_t)l * N + u]);
    m.e.push_back(M.energy[u] - M.energy[l]);
}

void finish_mode(ModeHost &m, const lvg_problem *prob) {
    const int N = prob->mol->nb_lev, nl = (int)m.u.size();
    const int nc = prob->dust ? prob->dust->nb_comp : 0;
    m.sigma.assign((size_t)std::max(1, nc) * std::max(1, nl), 0.);
    for (int c = 0; c < nc; c++)
        for (int n = 0; n < nl; n++) m.sigma[(size_t)c * nl + n] = dust_sigma(prob->dust->comp[c], m.e[n]);
    std::vector<std::vector<int>> per(N);                 // line order
    std::vector<std::vector<std::pair<int, int>>> col(N); // (partner level, y index)
    for (int n = 0; n < nl; n++) {
        per[m.u[n]].push_back(2 * n);
        per[m.l[n]].push_back(2 * n + 1);
        col[m.u[n]].push_back({m.l[n], 2 * n});
        col[m.l[n]].push_back({m.u[n], 2 * n + 1});
    }
    m.dptr.assign(N + 1, 0);
    m.cptr.assign(N + 1, 0);
    for (int i = 0; i < N; i++) {
        m.dptr[i] = (int)m.dent.size();
        for (int e : per[i]) m.dent.push_back(e);
        std::sort(col[i].begin(), col[i].end());
        m.cptr[i] = (int)m.cr.size();
        for (auto &pr : col[i]) { m.cr.push_back(pr.first); m.cy.push_back(pr.second); }
    }
    m.dptr[N] = (int)m.dent.size();
    m.cptr[N] = (int)m.cr.size();
    // dense map for the fused assembly: li[r*N + d] = y index of the line joining
    // levels r and d (its term lands at row r of column d), -1 if none
    m.li.assign((size_t)N * N, -1);
    for (int d = 0; d < N; d++)
        for (int e = m.cptr[d]; e < m.cptr[d + 1]; e++) m.li[(size_t)m.cr[e] * N + d] = m.cy[e];
}

// hfs_lines::sort / split (iteration_lvg.cpp:259-302), stale minimum kept (quirk q6)
struct Hfs {
    int nb = 0, up[4], lo[4];
    double en[4];
    void swap_lines(int i, int j) { std::swap(up[i], up[j]); std::swap(lo[i], lo[j]); std::swap(en[i], en[j]); }
    void sort() {
        if (nb <= 2) return;
        for (int i = 0; i < nb; i++)
            for (int j = i + 1; j < nb; j++)
                if (en[j] < en[i]) swap_lines(i, j);
        int jj = 0;
        double e = en[1] - en[0];
        for (int i = 1; i < nb - 1; i++)
            if (en[i + 1] - en[i] < e) jj = i;
        e = en[jj];
        for (int i = 0; i < nb; i++)
            for (int j = i + 1; j < nb; j++)
                if (std::fabs(en[j] - e) < std::fabs(en[i] - e)) swap_lines(i, j);
    }
};

void build_overlap_mode(ModeHost &m, const lvg_problem *prob) {
    const lvg_molecule &M = *prob->mol;
    const int N = M.nb_lev;
    m.interleaved = 0;
    auto group = [&](const Hfs &h, int start, int cnt) {
        int n0 = (int)m.u.size();
        add_line(m, prob, h.up[start], h.lo[start]);
        int n1 = -1;
        if (cnt == 2) { n1 = n0 + 1; add_line(m, prob, h.up[start + 1], h.lo[start + 1]); }
        m.unit0.push_back(n0);
        m.unit1.push_back(n1);
    };
    for (int i = 2; i < N; i += 2)
        for (int j = 0; j < i; j += 2) {
            Hfs h;
            for (int a = 0; a < 2; a++)
                for (int b = 0; b < 2; b++)
                    if (M.einst[(size_t)(i + a) * N + j + b] > 1.e-99) {
                        h.up[h.nb] = i + a; h.lo[h.nb] = j + b;
                        h.en[h.nb] = M.energy[i + a] - M.energy[j + b];
                        h.nb++;
                    }
            h.sort();
            int start = 0;
            if (h.nb >= 3) { group(h, 0, 2); start = 2; }
            if (h.nb - start > 0) group(h, start, h.nb - start);
        }
    finish_mode(m, prob);
}

void build_plain_mode(ModeHost &m, const lvg_problem *prob) {
    const lvg_molecule &M = *prob->mol;
    const int N = M.nb_lev;
    for (int i = 1; i < N; i++)
        for (int j = 0; j < i; j++)
            if (M.einst[(size_t)i * N + j] > 0.) {      // iteration_lvg.cpp:134
                m.unit0.push_back((int)m.u.size());
                m.unit1.push_back(-1);
                add_line(m, prob, i, j);
            }
    finish_mode(m, prob);
}

int upload_mode(lvg_handle *h, const ModeHost &m, LvgModeLines &d) {
    int rc;
    d.nb_lines = (int)m.u.size();
    d.nb_units = (int)m.unit0.size();
    if ((rc = upload(h, m.u.data(), m.u.size(), &d.line_u))) return rc;
    if ((rc = upload(h, m.l.data(), m.l.size(), &d.line_l))) return rc;
    if ((rc = upload(h, m.aul.data(), m.aul.size(), &d.line_aul))) return rc;
    if ((rc = upload(h, m.alu.data(), m.alu.size(), &d.line_alu))) return rc;
    if ((rc = upload(h, m.e.data(), m.e.size(), &d.line_e))) return rc;
    if ((rc = upload(h, m.sigma.data(), m.sigma.size(), &d.line_sigma))) return rc;
    if ((rc = upload(h, m.unit0.data(), m.unit0.size(), &d.unit_l0))) return rc;
    if ((rc = upload(h, m.unit1.data(), m.unit1.size(), &d.unit_l1))) return rc;
    if ((rc = upload(h, m.dptr.data(), m.dptr.size(), &d.diag_ptr))) return rc;
    if ((rc = upload(h, m.dent.data(), m.dent.size(), &d.diag_ent))) return rc;
    if ((rc = upload(h, m.cptr.data(), m.cptr.size(), &d.col_ptr))) return rc;
    if ((rc = upload(h, m.cr.data(), m.cr.size(), &d.col_r))) return rc;
    if ((rc = upload(h, m.cy.data(), m.cy.size(), &d.col_y))) return rc;
    if ((rc = upload(h, m.li.data(), m.li.size(), &d.line_idx))) return rc;
    d.diag_interleaved = m.interleaved;
    return LVG_OK;
}

bool ascending(const double *a, int n, bool strict) {
    for (int i = 1; i < n; i++)
        if (strict ? !(a[i] > a[i - 1]) : !(a[i] >= a[i - 1])) return false;
    return true;
}

int validate(lvg_handle *h, const lvg_problem *p) {
    if (!p || !p->mol || !p->coll || !p->esc) return fail(h, LVG_E_ARG, "problem, molecule, collisions and escape table are required");
    const lvg_molecule &M = *p->mol;
    if (M.nb_lev < 2) return fail(h, LVG_E_ARG, "nb_lev must be >= 2");
    if (M.nb_lev > lvg_kernel_max_levels_big())
        return fail(h, LVG_E_UNSUPPORTED, "nb_lev %d exceeds this build's %d", M.nb_lev, lvg_kernel_max_levels_big());
    if (!M.energy || !M.g || !M.einst || !(M.mass > 0.)) return fail(h, LVG_E_ARG, "molecule arrays / mass missing");
    if (!ascending(M.energy, M.nb_lev, false)) return fail(h, LVG_E_ARG, "level energies must be ascending");
    for (int i = 0; i < M.nb_lev; i++) if (M.g[i] <= 0) return fail(h, LVG_E_ARG, "g[%d] must be positive", i);
    for (int i = 1; i < M.nb_lev; i++)
        for (int j = 0; j < i; j++)
            if (M.einst[(size_t)i * M.nb_lev + j] > 0. && !(M.energy[i] > M.energy[j]))
                return fail(h, LVG_E_ARG, "line %d->%d has non-positive energy", i, j);
    const lvg_collisions &C = *p->coll;
    const int nt = C.nb_neutral + C.nb_electron;
    if (C.nb_neutral < 0 || C.nb_electron < 0 || nt > LVG_MAX_TABLES || (nt && !C.tables))
        return fail(h, LVG_E_ARG, "bad collision table counts");
    for (int t = 0; t < nt; t++) {
        const lvg_coll_table &T = C.tables[t];
        if (T.jmax < 2 || T.nb_lev < 2 || !T.tgrid || !T.coeff) return fail(h, LVG_E_ARG, "collision table %d malformed", t);
        if (!ascending(T.tgrid, T.jmax, true)) return fail(h, LVG_E_ARG, "collision table %d: tgrid not ascending", t);
        if (T.nb_lev > M.nb_lev) {
            // tables may cover more levels than the molecule uses; pairs beyond N are never read
        }
    }
    const int nc = p->dust ? p->dust->nb_comp : 0;
    if (nc > LVG_MAX_DUST) return fail(h, LVG_E_UNSUPPORTED, "more than %d dust components", LVG_MAX_DUST);
    if (nc > 0 && !p->dust->comp) return fail(h, LVG_E_ARG, "dust components missing");
    for (int c = 0; c < nc; c++) {
        const lvg_dust_component &d = p->dust->comp[c];
        if (d.nb_en < 2 || !d.energy || !d.abs_coeff || !ascending(d.energy, d.nb_en, true))
            return fail(h, LVG_E_ARG, "dust component %d malformed", c);
    }
    if (!p->esc->delta || !p->esc->gamma || !p->esc->p) return fail(h, LVG_E_ARG, "escape table arrays missing");
    if (p->esc->nb_d < 2 || p->esc->nb_g < 2 || !ascending(p->esc->delta, p->esc->nb_d, true) ||
        !ascending(p->esc->gamma, p->esc->nb_g, true))
        return fail(h, LVG_E_ARG, "escape table malformed");
    if ((p->overlap1 == nullptr) != (p->overlap2 == nullptr)) return fail(h, LVG_E_ARG, "give both overlap tables or neither");
    if (p->overlap1) {
        const lvg_overlap_table *o[2] = {p->overlap1, p->overlap2};
        for (auto t : o)
            if (!t->log10_delta || !t->dx || !t->gratio || !t->gamma || !t->p)
                return fail(h, LVG_E_ARG, "overlap table arrays missing");
        for (auto t : o)
            if (t->nb_d != o[0]->nb_d || t->nb_dx != o[0]->nb_dx || t->nb_gr != o[0]->nb_gr || t->nb_g != o[0]->nb_g ||
                t->nb_d < 2 || t->nb_dx < 2 || t->nb_gr < 2 || t->nb_g < 2)
                return fail(h, LVG_E_ARG, "overlap tables must share grids");
        // The device keeps one copy of the grids (overlap1's) for both tables. The reference's two
        // lvg_line_overlap_data objects (lvg_method_functions.h:55-70) each carry their own grids;
        // its two files share them, and this build requires that (DESIGN.md §8 restrictions)
        auto same = [](const double *x, const double *y, int n) { return memcmp(x, y, sizeof(double) * n) == 0; };
        if (!same(o[0]->log10_delta, o[1]->log10_delta, o[0]->nb_d) || !same(o[0]->dx, o[1]->dx, o[0]->nb_dx) ||
            !same(o[0]->gratio, o[1]->gratio, o[0]->nb_gr) || !same(o[0]->gamma, o[1]->gamma, o[0]->nb_g))
            return fail(h, LVG_E_ARG, "overlap tables must share grids");
        if (M.nb_lev % 2) return fail(h, LVG_E_ARG, "line overlap needs an even number of levels (hyperfine doublets)");
    }
    return LVG_OK;
}

int build(lvg_handle *h, const lvg_problem *p) {
    const lvg_molecule &M = *p->mol;
    const int N = M.nb_lev;
    LvgDevProblem &D = h->P;
    memset(&D, 0, sizeof D);
    D.N = N;
    D.mass = M.mass;
    D.nb_comp = p->dust ? p->dust->nb_comp : 0;
    D.nb_neutral = p->coll->nb_neutral;
    D.nb_electron = p->coll->nb_electron;
    D.nb_tables = D.nb_neutral + D.nb_electron;
    int rc;
    std::vector<double> g(N);
    for (int i = 0; i < N; i++) g[i] = (double)M.g[i];
    if ((rc = upload(h, M.energy, N, &D.energy))) return rc;
    if ((rc = upload(h, g.data(), N, &D.g))) return rc;
    if ((rc = upload(h, M.einst, (size_t)N * N, &D.einst))) return rc;
    {
        // transposed copy: the block kernels' boundary-matrix diagonal reads it by columns (coalesced)
        std::vector<double> et((size_t)N * N);
        for (int i = 0; i < N; i++)
            for (int j = 0; j < N; j++) et[(size_t)j * N + i] = M.einst[(size_t)i * N + j];
        if ((rc = upload(h, et.data(), (size_t)N * N, &D.einst_t))) return rc;
    }
    // collision tables, T-major, restricted to the levels the molecule uses
    std::vector<int> jmax, nbl;
    std::vector<int64_t> tgo, co;
    std::vector<double> tg, cf, cd;
    for (int t = 0; t < D.nb_tables; t++) {
        const lvg_coll_table &T = p->coll->tables[t];
        const int nl = std::min(T.nb_lev, N);
        const int64_t imax_src = (int64_t)T.nb_lev * (T.nb_lev - 1) / 2;
        const int64_t imax = (int64_t)nl * (nl - 1) / 2;
        (void)imax_src;
        jmax.push_back(T.jmax);
        nbl.push_back(nl);
        tgo.push_back((int64_t)tg.size());
        co.push_back((int64_t)cf.size());
        tg.insert(tg.end(), T.tgrid, T.tgrid + T.jmax);
        size_t base = cf.size();
        cf.resize(base + (size_t)imax * T.jmax);
        for (int64_t i = 0; i < imax; i++)
            for (int j = 0; j < T.jmax; j++) cf[base + (size_t)j * imax + i] = T.coeff[(size_t)i * T.jmax + j];
        // collision_data::calc_coeff_deriv (coll_rates.cpp): slope of each T interval,
        // the same expression get_rate evaluates, so the values are identical
        cd.resize(cf.size(), 0.);
        for (int j = 0; j + 1 < T.jmax; j++) {
            const double dt = T.tgrid[j + 1] - T.tgrid[j];
            for (int64_t i = 0; i < imax; i++)
                cd[base + (size_t)j * imax + i] = (T.coeff[(size_t)i * T.jmax + j + 1] - T.coeff[(size_t)i * T.jmax + j]) / dt;
        }
    }
    if ((rc = upload(h, jmax.data(), jmax.size(), &D.tab_jmax))) return rc;
    if ((rc = upload(h, nbl.data(), nbl.size(), &D.tab_nb_lev))) return rc;
    if ((rc = upload(h, tgo.data(), tgo.size(), &D.tab_tg_off))) return rc;
    if ((rc = upload(h, co.data(), co.size(), &D.tab_c_off))) return rc;
    if ((rc = upload(h, tg.data(), tg.size(), &D.tab_tgrid))) return rc;
    if ((rc = upload(h, cf.data(), cf.size(), &D.tab_coeff))) return rc;
    if ((rc = upload(h, cd.data(), cd.size(), &D.tab_deriv))) return rc;
    std::vector<uint8_t> pc;
    if ((rc = compile_rule(h, p, pc, D.terms))) return rc;
    if ((rc = upload(h, pc.data(), pc.size(), &D.pair_class))) return rc;
    // escape tables
    D.esc_nd = p->esc->nb_d;
    D.esc_ng = p->esc->nb_g;
    if ((rc = upload(h, p->esc->delta, D.esc_nd, &D.esc_delta))) return rc;
    if ((rc = upload(h, p->esc->gamma, D.esc_ng, &D.esc_gamma))) return rc;
    if ((rc = upload(h, p->esc->p, (size_t)D.esc_nd * D.esc_ng, &D.esc_p))) return rc;
    if (p->overlap1) {
        const lvg_overlap_table &o = *p->overlap1;
        D.ov_nd = o.nb_d; D.ov_ndx = o.nb_dx; D.ov_ngr = o.nb_gr; D.ov_ng = o.nb_g;
        size_t n = (size_t)o.nb_d * o.nb_dx * o.nb_gr * o.nb_g;
        if ((rc = upload(h, o.log10_delta, o.nb_d, &D.ov_ld))) return rc;
        if ((rc = upload(h, o.dx, o.nb_dx, &D.ov_dx))) return rc;
        if ((rc = upload(h, o.gratio, o.nb_gr, &D.ov_gr))) return rc;
        if ((rc = upload(h, o.gamma, o.nb_g, &D.ov_g))) return rc;
        if ((rc = upload(h, o.p, n, &D.ov_p1))) return rc;
        if ((rc = upload(h, p->overlap2->p, n, &D.ov_p2))) return rc;
        h->has_overlap = 1;
        ModeHost mo;
        build_overlap_mode(mo, p);
        if ((rc = upload_mode(h, mo, D.overlap))) return rc;
    }
    ModeHost mp;
    build_plain_mode(mp, p);
    if ((rc = upload_mode(h, mp, D.plain))) return rc;
    return LVG_OK;
}

// block the host until the last asynchronous solve on this handle has finished
void drain(lvg_handle *h) {
    if (h->pending) {
        (void)hipEventSynchronize(h->ev1);
        h->pending = 0;
    }
}

// order a call that works on stream s after the last asynchronous solve: same stream ->
// stream order suffices; another stream -> wait for it
void settle(lvg_handle *h, hipStream_t s) {
    if (h->pending && s != h->pending_stream) drain(h);
}

int ensure_workspace(lvg_handle *h, int slots) {
    const int N = h->N;
    const int lines = std::max(h->P.plain.nb_lines, h->P.overlap.nb_lines);
    int64_t stride = 2LL * N * N + 2LL * LVG_HIST_SLOTS * N + 3LL * N + 2LL * lines + 64;
    // wave kernel: per-layer line invariants after the y region (wave_line_invariants)
    if (N <= LVG_WAVE_NMAX) stride += (int64_t)LVG_WAVE_INV_FIELDS * lines;
    stride = (stride + 31) & ~31LL;
    size_t bytes = (size_t)stride * slots * sizeof(double);
    if (bytes > h->ws_bytes) {
        drain(h);
        if (h->ws) (void)hipFree(h->ws);
        h->ws = nullptr;
        h->ws_bytes = 0;
        if (hipMalloc(&h->ws, bytes) != hipSuccess) return fail(h, LVG_E_NOMEM, "workspace hipMalloc(%zu) failed", bytes);
        h->ws_bytes = bytes;
    }
    h->ws_stride = stride;
    return LVG_OK;
}

int check_opts(lvg_handle *h, const lvg_solve_opts *o) {
    if (!o) return fail(h, LVG_E_ARG, "opts is NULL");
    if (!(o->min_error > 0.) || o->max_iter_acc < 1 || o->max_iter_plain < 1)
        return fail(h, LVG_E_ARG, "min_error / iteration caps invalid");
    if (o->accel_nb < 2 || o->accel_nb > 5 || o->accel_period < 1 || (o->acceleration && o->accel_start < o->accel_nb))
        return fail(h, LVG_E_ARG, "acceleration parameters invalid (accel_nb in [2,5], accel_start >= accel_nb)");
    if (o->init < LVG_INIT_BOUNDARY_LAYER || o->init > LVG_INIT_WARM_CHAIN) return fail(h, LVG_E_ARG, "bad init mode");
    if (o->line_overlap && !h->has_overlap) return fail(h, LVG_E_ARG, "line_overlap requested but no overlap tables");
    return LVG_OK;
}

void fill_launch(lvg_handle *h, LvgLaunch &L, const lvg_solve_opts *o) {
    memset(&L, 0, sizeof L);
    L.min_error = o->min_error;
    L.max_iter_acc = o->max_iter_acc;
    L.max_iter_plain = o->max_iter_plain;
    L.accel_start = o->accel_start;
    L.accel_period = o->accel_period;
    L.accel_nb = o->accel_nb;
    L.acceleration = o->acceleration;
    L.allow_plain_retry = o->allow_plain_retry;
    L.init = o->init;
    L.line_overlap = o->line_overlap;
    L.ws = h->ws;
    L.ws_stride = h->ws_stride;
    L.counter = h->counter;
}

// copy launch parameter block `slot` to the device (stream-ordered)
int push_launch(lvg_handle *h, const LvgLaunch &L, int slot, hipStream_t s, const LvgLaunch **dptr) {
    if (slot >= h->n_launch_slots) {
        int n = std::max(slot + 1, 2 * h->n_launch_slots);
        LvgLaunch *p = nullptr;
        drain(h);
        if (h->d_launch) { (void)hipStreamSynchronize(s); (void)hipFree(h->d_launch); }
        if (hipMalloc(&p, sizeof(LvgLaunch) * n) != hipSuccess) return fail(h, LVG_E_NOMEM, "launch block alloc failed");
        h->d_launch = p;
        h->n_launch_slots = n;
    }
    HIPCHECK(h, hipMemcpyAsync(h->d_launch + slot, &L, sizeof L, hipMemcpyHostToDevice, s));
    *dptr = h->d_launch + slot;
    return LVG_OK;
}

int grow(lvg_handle *h, void **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return LVG_OK;
    drain(h);
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) return fail(h, LVG_E_NOMEM, "hipMalloc(%zu) failed", bytes);
    *cap = bytes;
    return LVG_OK;
}

// grow() without an error: false (and the buffer released) if the allocation fails
bool try_grow(lvg_handle *h, void **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return true;
    drain(h);
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) {
        (void)hipGetLastError();     // clear the sticky allocation error
        *p = nullptr;
        return false;
    }
    *cap = bytes;
    return true;
}

}  // namespace

extern "C" {

int lvg_abi_version(void) { return LVG_ABI_VERSION; }

int lvg_set_tuning(lvg_handle *h, const char *spec) {
    if (!h) return LVG_E_STATE;
    // merged into the current settings (the environment's included); "" resets them
    LvgTuning t = (spec && *spec) ? h->tune : LvgTuning();
    const int rc = parse_tuning(h, spec, t);
    if (rc == LVG_OK) {
        h->tune = t;
        for (lvg_handle *q : h->peers) q->tune = t;
    }
    return rc;
}

void lvg_solve_opts_default(lvg_solve_opts *o) {
    if (!o) return;
    o->min_error = 1.e-5;       // rel_population_error, radiative_transfer.cpp:45
    o->max_iter_acc = 150;      // MAX_NB_ITER_ACC, :27
    o->max_iter_plain = 15000;  // MAX_NB_ITER_EXT, :26
    o->accel_start = 40;        // iteration_control.h:71
    o->accel_period = 5;
    o->accel_nb = 5;
    o->acceleration = 1;
    o->allow_plain_retry = 1;
    o->init = LVG_INIT_BOUNDARY_LAYER;
    o->line_overlap = 0;
}

const char *lvg_last_error(const lvg_handle *h) { return h ? h->err.c_str() : g_create_error.c_str(); }

int lvg_nb_lev(const lvg_handle *h) { return h ? h->N : 0; }

int lvg_layer_soa_rows(const lvg_handle *h) { return h ? 10 + h->nb_comp : 0; }

void lvg_destroy(lvg_handle *h) {
    if (!h) return;
    for (lvg_handle *q : h->peers) lvg_destroy(q);
    h->peers.clear();
    (void)hipSetDevice(h->device);
    drain(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto &b : h->bufs) (void)hipFree(b.p);
    if (h->ws) (void)hipFree(h->ws);
    if (h->counter) (void)hipFree(h->counter);
    if (h->d_soa) (void)hipFree(h->d_soa);
    if (h->d_pops) (void)hipFree(h->d_pops);
    if (h->d_status) (void)hipFree(h->d_status);
    if (h->d_prob) (void)hipFree(h->d_prob);
    if (h->d_launch) (void)hipFree(h->d_launch);
    if (h->d_sched) (void)hipFree(h->d_sched);
    if (h->d_sched_tmp) (void)hipFree(h->d_sched_tmp);
    if (h->d_coll) (void)hipFree(h->d_coll);
    if (h->d_corder) (void)hipFree(h->d_corder);
    if (h->d_chain) (void)hipFree(h->d_chain);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->evc) (void)hipEventDestroy(h->evc);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int lvg_create(const lvg_problem *prob, int device, lvg_handle **out) {
    g_create_error.clear();
    if (!out) return fail(nullptr, LVG_E_ARG, "out is NULL");
    *out = nullptr;
    lvg_handle *h = new (std::nothrow) lvg_handle();
    if (!h) return fail(nullptr, LVG_E_NOMEM, "out of host memory");
    int rc = validate(h, prob);
    if (rc == LVG_OK) {
        // diagnostics only: a bad LVG_TUNING is reported and ignored, never fatal
        LvgTuning t;
        if (parse_tuning(h, std::getenv("LVG_TUNING"), t) == LVG_OK) h->tune = t;
        else std::fprintf(stderr, "liblvg_amd: LVG_TUNING ignored (%s)\n", h->err.c_str());
        h->err.clear();
    }
    if (rc == LVG_OK) {
        h->device = device;
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) rc = fail(h, LVG_E_DEVICE, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    }
    if (rc == LVG_OK) {
        h->N = prob->mol->nb_lev;
        h->nb_comp = prob->dust ? prob->dust->nb_comp : 0;
        rc = build(h, prob);
    }
    if (rc == LVG_OK) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
            hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
            hipEventCreate(&h->evc) != hipSuccess ||
            hipMalloc(&h->counter, sizeof(int)) != hipSuccess)
            rc = fail(h, LVG_E_DEVICE, "device setup failed");
        else {
            h->cus = prop.multiProcessorCount;
            h->lds_cap = prop.sharedMemPerBlock;
            if (hipMalloc(&h->d_prob, sizeof(LvgDevProblem)) != hipSuccess ||
                hipMemcpy(h->d_prob, &h->P, sizeof(LvgDevProblem), hipMemcpyHostToDevice) != hipSuccess)
                rc = fail(h, LVG_E_DEVICE, "problem block upload failed");
            int b = 1;
            h->big = h->N > lvg_kernel_max_levels();
            if ((h->big ? lvg_kernel_occupancy_big(&b) : lvg_kernel_occupancy(&b)) != hipSuccess || b < 1) b = 1;
            h->blocks_per_cu = b;
            int bw = 0;
            if (!h->big && lvg_kernel_occupancy_wide(&bw) == hipSuccess) h->wide_bpc = std::min(bw, 1);
        }
    }
    if (rc != LVG_OK) {
        g_create_error = h->err;
        lvg_destroy(h);
        return rc;
    }
    *out = h;
    return LVG_OK;
}

int lvg_shard_range(int n, int nb_dev, int r, int *lo, int *hi) {
    if (n < 0 || nb_dev < 1 || r < 0 || r >= nb_dev || !lo || !hi) return LVG_E_ARG;
    *lo = (int)(((int64_t)n * r) / nb_dev);
    *hi = (int)(((int64_t)n * (r + 1)) / nb_dev);
    return LVG_OK;
}

int lvg_chain_shard(int nb_chain, const int *chain_off, int nb_dev, int r, int *c_lo, int *c_hi) {
    if (nb_chain < 0 || !chain_off || !c_lo || !c_hi) return LVG_E_ARG;
    int lo, hi;
    const int rc = lvg_shard_range(chain_off[nb_chain], nb_dev, r, &lo, &hi);
    if (rc) return rc;
    // first chain starting at or after lo / hi (chain starts are non-decreasing)
    const int *b = chain_off, *e = chain_off + nb_chain;
    *c_lo = (int)(std::lower_bound(b, e, lo) - b);
    *c_hi = (r == nb_dev - 1) ? nb_chain : (int)(std::lower_bound(b, e, hi) - b);
    return LVG_OK;
}

int lvg_create_devices(const lvg_problem *prob, int nb_devices, const int *devices, lvg_handle **out) {
    g_create_error.clear();
    if (!out) return fail(nullptr, LVG_E_ARG, "out is NULL");
    *out = nullptr;
    if (nb_devices < 1 || nb_devices > 64 || !devices) return fail(nullptr, LVG_E_ARG, "need 1..64 device ordinals");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    for (int i = 0; i < nb_devices; i++)
        if (devices[i] < 0 || devices[i] >= ndev)
            return fail(nullptr, LVG_E_DEVICE, "device %d not present (%d visible)", devices[i], ndev);
    lvg_handle *h = nullptr;
    int rc = lvg_create(prob, devices[0], &h);
    if (rc) return rc;
    for (int i = 1; i < nb_devices; i++) {
        lvg_handle *q = nullptr;
        rc = lvg_create(prob, devices[i], &q);
        if (rc) {
            const std::string e = g_create_error;
            lvg_destroy(h);
            return fail(nullptr, rc, "device %d: %s", devices[i], e.c_str());
        }
        q->tune = h->tune;
        h->peers.push_back(q);
    }
    *out = h;
    return LVG_OK;
}

int lvg_create_multi(const lvg_problem *prob, unsigned device_mask, lvg_handle **out) {
    g_create_error.clear();
    std::vector<int> devs;
    for (int d = 0; d < 32; d++)
        if (device_mask & (1u << d)) devs.push_back(d);
    if (devs.empty()) {
        if (out) *out = nullptr;
        return fail(nullptr, LVG_E_ARG, "device_mask is empty");
    }
    return lvg_create_devices(prob, (int)devs.size(), devs.data(), out);
}

int lvg_nb_devices(const lvg_handle *h) { return h ? 1 + (int)h->peers.size() : 0; }

}  // extern "C"

namespace {

// chain_off: host [nb_chain + 1] (warm chains) or NULL (independent layers)
int check_chains(lvg_handle *h, int nb_lay, int nb_chain, const int *chain_off) {
    if (nb_lay == 0 && nb_chain == 0) return LVG_OK;     // an empty batch (e.g. a rank with no clouds)
    if (nb_chain < 1 || !chain_off) return fail(h, LVG_E_ARG, "warm chains need nb_chain >= 1 and chain_off");
    if (chain_off[0] != 0 || chain_off[nb_chain] != nb_lay)
        return fail(h, LVG_E_ARG, "chain_off must start at 0 and end at nb_lay");
    for (int c = 0; c < nb_chain; c++)
        if (chain_off[c + 1] < chain_off[c]) return fail(h, LVG_E_ARG, "chain_off must be non-decreasing");
    return LVG_OK;
}

// One persistent launch over device-resident buffers (caller has validated arguments).
int launch_solve(lvg_handle *h, int nb_lay, const double *d_soa, double *d_pops, const lvg_solve_opts *o,
                 lvg_layer_status *d_status, void *stream, int nb_chain, const int *chain_off) {
    int rc;
    h->last_ms = 0.;
    h->last_launches = 0;
    h->last_kernel = -1;            // an empty batch launches nothing
    if (nb_lay == 0) return LVG_OK;
    HIPCHECK(h, hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    settle(h, s);
    const int nq = chain_off ? nb_chain : nb_lay;   // queue items
    int per_cu = h->blocks_per_cu;
    // at most two independent layers per CU (e.g. 4096 layers strong-scaled over 8 GPUs):
    // one workgroup per CU with the CU to itself finishes the longest layers sooner (512
    // CH3OH-A layers: 9.2 vs 9.8 ms; at 1024 layers two per CU win, 12.2 vs 13.4 ms). Not
    // for warm chains, whose items are long and even: 512 chains of 8 layers take 57.7 ms
    // at one workgroup per CU against 39.8 ms at two.
    if (!chain_off && nq <= 2 * h->cus) per_cu = 1;
    if (h->tune.blocks_per_cu >= 1 && h->tune.blocks_per_cu <= h->blocks_per_cu) per_cu = h->tune.blocks_per_cu;
    // kernel choice: one wave per layer for N <= 64 (lvg_wave.hip), else one block per layer.
    // Both give bit-identical results; tuning block_kernel=1 forces the block kernel.
    int wpb = 0, wave_bpc = 0;
    size_t wdyn = 0;
    {
        const LvgModeLines &mh = o->line_overlap ? h->P.overlap : h->P.plain;
        const int grid_dbl = h->P.esc_nd + h->P.esc_ng +
                             (o->line_overlap ? h->P.ov_nd + h->P.ov_ndx + h->P.ov_ngr + h->P.ov_ng : 0);
        if (!h->tune.block_kernel && lvg_wave_plan(h->N, 2 * mh.nb_lines, grid_dbl, h->lds_cap, &wpb, &wdyn) &&
            lvg_wave_occupancy(h->N, wpb, wdyn, &wave_bpc) == hipSuccess && wave_bpc >= 1) {
        } else {
            wpb = 0;
        }
    }
    const bool wave = wpb > 0;
    // the 512-thread kernel (lvg_kernels_wide.hip, N <= 256) when the launch leaves CUs to
    // spare: at most two independent layers or one warm chain per CU. There one layer's
    // latency is the step, and eight waves per layer give every SIMD two waves to switch
    // between and halve each wave's update work. Bit-identical results.
    const bool wide = !wave && !h->big && h->wide_bpc >= 1 &&
                      (h->tune.wide == 2 || (h->tune.wide == 1 && nq <= (chain_off ? 1 : 2) * h->cus));
    const int grid = wave ? std::max(1, std::min((nq + wpb - 1) / wpb, h->cus * wave_bpc))
                   : wide ? std::max(1, std::min(nq, h->cus * h->wide_bpc))
                          : std::max(1, std::min(nq, h->cus * per_cu));
    const int slots = wave ? grid * wpb : grid;
    h->last_kernel = wave ? 1 : wide ? 2 : h->big ? 3 : 0;
    if ((rc = ensure_workspace(h, slots))) return rc;
    LvgLaunch L;
    fill_launch(h, L, o);
    L.nb_lay = nb_lay;
    L.lay_offset = 0;
    L.soa_ld = nb_lay;
    L.soa = d_soa;
    L.pops = d_pops;
    L.status = d_status;
    if (chain_off) {
        // chains: offsets, then the queue in decreasing chain length (stable; results do
        // not depend on the order, each chain is computed on its own)
        auto &hc = h->chain_host;
        drain(h);   // the staging vector may still feed an earlier asynchronous copy
        hc.assign(chain_off, chain_off + nb_chain + 1);
        std::vector<int> ord(nb_chain);
        for (int c = 0; c < nb_chain; c++) ord[c] = c;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
            return chain_off[a + 1] - chain_off[a] > chain_off[b + 1] - chain_off[b];
        });
        hc.insert(hc.end(), ord.begin(), ord.end());
        if ((rc = grow(h, (void **)&h->d_chain, &h->chain_cap, sizeof(int) * hc.size()))) return rc;
        HIPCHECK(h, hipMemcpyAsync(h->d_chain, hc.data(), sizeof(int) * hc.size(), hipMemcpyHostToDevice, s));
        L.chain_off = h->d_chain;
        L.nb_chain = nb_chain;
        L.order = h->d_chain + nb_chain + 1;
    } else if (nb_lay > slots && h->tune.queue_order) {
        // longest-expected-first order of the work queue (lvg_sched.hip); results do not
        // depend on it. Scratch: keys, sorted keys (double), indices, order (int).
        size_t tmp = 0;
        HIPCHECK(h, lvg_sched_order(nullptr, nb_lay, nb_lay, nullptr, nullptr, nullptr, nullptr, nullptr, &tmp, s));
        if ((rc = grow(h, &h->d_sched, &h->sched_cap, (size_t)nb_lay * (2 * sizeof(double) + 2 * sizeof(int))))) return rc;
        if ((rc = grow(h, &h->d_sched_tmp, &h->sched_tmp_cap, std::max<size_t>(tmp, 1)))) return rc;
        double *keys = static_cast<double *>(h->d_sched), *keys2 = keys + nb_lay;
        int *idx = reinterpret_cast<int *>(keys2 + nb_lay), *order = idx + nb_lay;
        HIPCHECK(h, lvg_sched_order(d_soa, nb_lay, nb_lay, keys, keys2, idx, order, h->d_sched_tmp, &tmp, s));
        L.order = order;
    }
    // independent layers on the block kernels: collision operators of the whole batch
    // built ahead by coll_kernel into HBM (K, and B for the boundary-layer start) when the
    // tuning asks for it and they fit coll_mem of the free device memory; if the buffer
    // cannot be had, every layer builds its own in the solve kernel (same results)
    bool coll_ahead = false;
    if (!wave && !chain_off && h->tune.coll_ahead) {
        const bool need_b = o->init != LVG_INIT_GIVEN;
        const bool b_from_k = h->P.nb_tables == h->P.nb_neutral;   // no electron tables: B = f(K)
        const size_t nn = (size_t)nb_lay * h->N * h->N * sizeof(double);
        const size_t nd = (size_t)nb_lay * h->N * sizeof(double);
        const size_t bytes = nn + (need_b ? (b_from_k ? nd : nn) : 0);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        if ((double)bytes <= h->tune.coll_mem * (double)(free_b + h->coll_cap) && try_grow(h, &h->d_coll, &h->coll_cap, bytes)) {
            L.kall = static_cast<const double *>(h->d_coll);
            const double *tail = static_cast<const double *>(h->d_coll) + nn / sizeof(double);
            L.ball = (need_b && !b_from_k) ? tail : nullptr;
            L.bdiag = (need_b && b_from_k) ? tail : nullptr;
            coll_ahead = true;
            if (h->tune.coll_order) {
                // temperature order for coll_kernel (lvg_sched.hip); its own scratch, since
                // the solve queue's order may live in d_sched
                size_t tmp = 0;
                HIPCHECK(h, lvg_row_order(nullptr, nb_lay, nb_lay, 0, nullptr, nullptr, nullptr, nullptr, nullptr, &tmp, s));
                if ((rc = grow(h, &h->d_corder, &h->corder_cap,
                               (size_t)nb_lay * (2 * sizeof(double) + 2 * sizeof(int)) + tmp + 256))) return rc;
                double *keys = static_cast<double *>(h->d_corder), *keys2 = keys + nb_lay;
                int *idx = reinterpret_cast<int *>(keys2 + nb_lay), *ord = idx + nb_lay;
                char *scratch = reinterpret_cast<char *>(ord + nb_lay);
                scratch += (256 - (reinterpret_cast<uintptr_t>(scratch) & 255)) & 255;
                HIPCHECK(h, lvg_row_order(d_soa, nb_lay, nb_lay, 0, keys, keys2, idx, ord, scratch, &tmp, s));
                L.coll_order = ord;
            }
        }
    }
    if (!coll_ahead && h->d_coll) {
        // the batch buffer of an earlier call is not held across calls that do not use it
        drain(h);
        (void)hipFree(h->d_coll);
        h->d_coll = nullptr;
        h->coll_cap = 0;
    }
    const LvgLaunch *dL = nullptr;
    if ((rc = push_launch(h, L, 0, s, &dL))) return rc;
    HIPCHECK(h, hipMemsetAsync(h->counter, 0, sizeof(int), s));
    HIPCHECK(h, hipEventRecord(h->ev0, s));
    h->last_coll = coll_ahead ? 1 : 0;
    h->last_coll_ms = 0.;
    if (coll_ahead) {
        HIPCHECK(h, lvg_launch_coll(h->d_prob, dL, std::min(nb_lay, 8 * h->cus), s));
        HIPCHECK(h, hipEventRecord(h->evc, s));
    }
    if (wave) HIPCHECK(h, lvg_launch_solve_wave(h->d_prob, dL, h->N, grid, wpb, wdyn, s));
    else if (wide) HIPCHECK(h, lvg_launch_solve_wide(h->d_prob, dL, grid, s));
    else HIPCHECK(h, h->big ? lvg_launch_solve_big(h->d_prob, dL, grid, s) : lvg_launch_solve(h->d_prob, dL, grid, s));
    HIPCHECK(h, hipEventRecord(h->ev1, s));
    h->last_launches = 1;
    if (!stream) {
        HIPCHECK(h, hipStreamSynchronize(s));
        float ms = 0.f;
        if (h->last_coll) {
            float mc = 0.f;
            (void)hipEventElapsedTime(&mc, h->ev0, h->evc);
            (void)hipEventElapsedTime(&ms, h->evc, h->ev1);
            h->last_coll_ms = mc;
        } else {
            (void)hipEventElapsedTime(&ms, h->ev0, h->ev1);
        }
        h->last_ms = ms;
        h->pending = 0;
    } else {
        h->pending = 1;
        h->pending_stream = s;
    }
    return LVG_OK;
}

}  // namespace

extern "C" {

int lvg_solve_layers_device(lvg_handle *h, int nb_lay, const double *d_soa, double *d_pops,
                            const lvg_solve_opts *o, lvg_layer_status *d_status, void *stream) {
    if (!h) return LVG_E_STATE;
    int rc = check_opts(h, o);
    if (rc) return rc;
    if (nb_lay < 0 || (nb_lay > 0 && (!d_soa || !d_pops || !d_status))) return fail(h, LVG_E_ARG, "bad device buffers");
    if (o->init == LVG_INIT_WARM_CHAIN) {   // one chain over all layers
        const int off[2] = {0, nb_lay};
        return launch_solve(h, nb_lay, d_soa, d_pops, o, d_status, stream, 1, nb_lay ? off : nullptr);
    }
    return launch_solve(h, nb_lay, d_soa, d_pops, o, d_status, stream, 0, nullptr);
}

int lvg_solve_chains_device(lvg_handle *h, int nb_lay, const double *d_soa, int nb_chain, const int *chain_off,
                            double *d_pops, const lvg_solve_opts *o, lvg_layer_status *d_status, void *stream) {
    if (!h) return LVG_E_STATE;
    int rc = check_opts(h, o);
    if (rc) return rc;
    if (o->init != LVG_INIT_WARM_CHAIN) return fail(h, LVG_E_ARG, "lvg_solve_chains needs init = LVG_INIT_WARM_CHAIN");
    if (nb_lay < 0 || (nb_lay > 0 && (!d_soa || !d_pops || !d_status))) return fail(h, LVG_E_ARG, "bad device buffers");
    if ((rc = check_chains(h, nb_lay, nb_chain, chain_off))) return rc;
    return launch_solve(h, nb_lay, d_soa, d_pops, o, d_status, stream, nb_chain, chain_off);
}

int lvg_last_kernel_time(const lvg_handle *h, double *ms, int *nb) {
    if (!h) return LVG_E_STATE;
    lvg_handle *hh = const_cast<lvg_handle *>(h);
    if (hh->last_launches && hh->last_ms == 0.) {
        float f = 0.f;
        float fc = 0.f;
        if (hipEventSynchronize(hh->ev1) == hipSuccess &&
            hipEventElapsedTime(&f, hh->last_coll ? hh->evc : hh->ev0, hh->ev1) == hipSuccess)
            hh->last_ms = f;
        if (hh->last_coll && hipEventElapsedTime(&fc, hh->ev0, hh->evc) == hipSuccess) hh->last_coll_ms = fc;
    }
    if (ms) *ms = hh->last_ms;
    if (nb) *nb = hh->last_launches;
    return LVG_OK;
}

int lvg_last_coll_time(const lvg_handle *h, double *ms) {
    if (!h) return LVG_E_STATE;
    double k = 0.;
    int rc = lvg_last_kernel_time(h, &k, nullptr);   // settles both timings
    if (rc) return rc;
    if (ms) *ms = h->last_coll ? h->last_coll_ms : 0.;
    return LVG_OK;
}

int lvg_last_kernel_kind(const lvg_handle *h, int *kind) {
    if (!h) return LVG_E_STATE;
    if (!kind) return LVG_E_ARG;
    *kind = h->last_kernel;
    return LVG_OK;
}

static int upload_layers(lvg_handle *h, const lvg_layers *L) {
    const int nl = L->nb_lay, rows = 10 + h->nb_comp;
    std::vector<double> soa((size_t)rows * nl);
    const double *f[10] = {L->temp_n, L->temp_el, L->el_conc, L->h_conc, L->ph2_conc,
                           L->oh2_conc, L->he_conc, L->mol_conc, L->vel_turb, L->vel_grad};
    for (int r = 0; r < 10; r++) {
        if (!f[r]) return fail(h, LVG_E_ARG, "layer field %d is NULL", r);
        memcpy(&soa[(size_t)r * nl], f[r], sizeof(double) * nl);
    }
    if (h->nb_comp && !L->dust_conc) return fail(h, LVG_E_ARG, "dust_conc is NULL");
    for (int c = 0; c < h->nb_comp; c++)
        for (int l = 0; l < nl; l++) soa[(size_t)(10 + c) * nl + l] = L->dust_conc[(size_t)l * h->nb_comp + c];
    int rc = grow(h, (void **)&h->d_soa, &h->soa_cap, soa.size() * sizeof(double));
    if (rc) return rc;
    HIPCHECK(h, hipMemcpyAsync(h->d_soa, soa.data(), soa.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HIPCHECK(h, hipStreamSynchronize(h->stream));
    return LVG_OK;
}

}  // extern "C"

namespace {

// host-buffer solve: upload the layer SoA (and given populations), one launch, copy back
int solve_host(lvg_handle *h, const lvg_layers *layers, double *pops, const lvg_solve_opts *o,
               lvg_layer_status *status, int nb_chain, const int *chain_off) {
    const int nl = layers->nb_lay, N = h->N;
    int rc;
    if (nl == 0) return LVG_OK;
    HIPCHECK(h, hipSetDevice(h->device));
    settle(h, h->stream);
    if ((rc = upload_layers(h, layers))) return rc;
    if ((rc = grow(h, (void **)&h->d_pops, &h->pops_cap, sizeof(double) * (size_t)nl * N))) return rc;
    if ((rc = grow(h, &h->d_status, &h->status_cap, sizeof(lvg_layer_status) * (size_t)nl))) return rc;
    if (o->init == LVG_INIT_GIVEN)
        HIPCHECK(h, hipMemcpyAsync(h->d_pops, pops, sizeof(double) * (size_t)nl * N, hipMemcpyHostToDevice, h->stream));
    rc = launch_solve(h, nl, h->d_soa, h->d_pops, o, (lvg_layer_status *)h->d_status, nullptr, nb_chain, chain_off);
    if (rc) return rc;
    HIPCHECK(h, hipMemcpy(pops, h->d_pops, sizeof(double) * (size_t)nl * N, hipMemcpyDeviceToHost));
    if (status) HIPCHECK(h, hipMemcpy(status, h->d_status, sizeof(lvg_layer_status) * (size_t)nl, hipMemcpyDeviceToHost));
    return LVG_OK;
}

}  // namespace

namespace {

// the layers [lo, hi) of `L` as a view (no copy)
lvg_layers layer_block(const lvg_layers &L, int nb_comp, int lo, int hi) {
    lvg_layers v = L;
    v.nb_lay = hi - lo;
    const double **f[10] = {&v.temp_n, &v.temp_el, &v.el_conc, &v.h_conc, &v.ph2_conc,
                            &v.oh2_conc, &v.he_conc, &v.mol_conc, &v.vel_turb, &v.vel_grad};
    for (auto p : f) if (*p) *p += lo;
    if (v.dust_conc) v.dust_conc += (size_t)lo * nb_comp;
    return v;
}

// Multi-device handle: part d of the batch on device d (this handle, then its peers), one host
// thread per device (each handle is used by exactly one thread: the one-handle-per-thread rule
// holds), each on its own stream. part(handle, d) returns an LVG code. Kernel time: the slowest
// device's (the step of a strongly split batch); launches summed.
template <class F>
int run_split(lvg_handle *h, F part) {
    const int G = 1 + (int)h->peers.size();
    std::vector<lvg_handle *> hs(G);
    hs[0] = h;
    for (int d = 1; d < G; d++) hs[d] = h->peers[d - 1];
    std::vector<int> rc(G, LVG_OK);
    std::vector<std::thread> th;
    for (int d = 1; d < G; d++) th.emplace_back([&, d] { rc[d] = part(hs[d], d); });
    rc[0] = part(hs[0], 0);
    for (auto &t : th) t.join();
    double ms = 0.;
    int launches = 0, kind = -1;
    for (int d = 0; d < G; d++) {
        if (rc[d]) {
            if (d) fail(h, rc[d], "device %d: %s", hs[d]->device, hs[d]->err.c_str());
            return rc[d];
        }
        double m = 0.;
        int n = 0;
        (void)lvg_last_kernel_time(hs[d], &m, &n);
        ms = std::max(ms, m);
        launches += n;
        if (kind < 0 && n) kind = hs[d]->last_kernel;
    }
    h->last_ms = ms;
    h->last_launches = launches;
    h->last_kernel = kind;
    h->last_coll = 0;
    return LVG_OK;
}

}  // namespace

extern "C" {

int lvg_solve_layers(lvg_handle *h, const lvg_layers *layers, double *pops, const lvg_solve_opts *o,
                     lvg_layer_status *status) {
    if (!h) return LVG_E_STATE;
    if (!layers || (layers->nb_lay > 0 && !pops)) return fail(h, LVG_E_ARG, "layers / pops missing");
    int rc = check_opts(h, o);
    if (rc) return rc;
    const int nl = layers->nb_lay;
    if (o->init == LVG_INIT_WARM_CHAIN) {
        // the reference default (radiative_transfer.cpp:247-252): one chain over the cloud,
        // sequential by construction (the first device of a multi-device handle)
        const int off[2] = {0, nl};
        return solve_host(h, layers, pops, o, status, 1, off);
    }
    if (!h->peers.empty() && nl > 0) {
        // independent layers: contiguous blocks, layer l on device floor(l G / nl) (lvg_shard_range),
        // no exchange between devices
        const int G = 1 + (int)h->peers.size(), N = h->N;
        return run_split(h, [&](lvg_handle *q, int d) {
            int lo, hi;
            lvg_shard_range(nl, G, d, &lo, &hi);
            q->last_ms = 0.; q->last_launches = 0; q->last_kernel = -1;
            if (hi == lo) return LVG_OK;
            const lvg_layers v = layer_block(*layers, h->nb_comp, lo, hi);
            return solve_host(q, &v, pops + (size_t)lo * N, o, status ? status + lo : nullptr, 0, nullptr);
        });
    }
    return solve_host(h, layers, pops, o, status, 0, nullptr);
}

int lvg_solve_chains(lvg_handle *h, const lvg_layers *layers, int nb_chain, const int *chain_off, double *pops,
                     const lvg_solve_opts *o, lvg_layer_status *status) {
    if (!h) return LVG_E_STATE;
    if (!layers || (layers->nb_lay > 0 && !pops)) return fail(h, LVG_E_ARG, "layers / pops missing");
    int rc = check_opts(h, o);
    if (rc) return rc;
    if (o->init != LVG_INIT_WARM_CHAIN) return fail(h, LVG_E_ARG, "lvg_solve_chains needs init = LVG_INIT_WARM_CHAIN");
    if ((rc = check_chains(h, layers->nb_lay, nb_chain, chain_off))) return rc;
    if (!h->peers.empty() && layers->nb_lay > 0) {
        // whole clouds per device, contiguous and balanced by layer count (lvg_chain_shard)
        const int G = 1 + (int)h->peers.size(), N = h->N;
        return run_split(h, [&](lvg_handle *q, int d) {
            int c_lo, c_hi;
            lvg_chain_shard(nb_chain, chain_off, G, d, &c_lo, &c_hi);
            q->last_ms = 0.; q->last_launches = 0; q->last_kernel = -1;
            const int lo = chain_off[c_lo], hi = chain_off[c_hi];
            if (hi == lo) return LVG_OK;
            std::vector<int> off(chain_off + c_lo, chain_off + c_hi + 1);
            for (int &x : off) x -= lo;
            const lvg_layers v = layer_block(*layers, h->nb_comp, lo, hi);
            return solve_host(q, &v, pops + (size_t)lo * N, o, status ? status + lo : nullptr, c_hi - c_lo, off.data());
        });
    }
    return solve_host(h, layers, pops, o, status, nb_chain, chain_off);
}

int lvg_debug_calc_new_pop(lvg_handle *h, const lvg_layers *layers, int layer, const double *pop_in, int line_overlap,
                           double *matrix_out, double *df_out, double *pop_out, double *eq_error) {
    if (!h) return LVG_E_STATE;
    if (!layers || layer < 0 || layer >= layers->nb_lay || !pop_in || !pop_out)
        return fail(h, LVG_E_ARG, "bad debug arguments");
    if (line_overlap && !h->has_overlap) return fail(h, LVG_E_ARG, "no overlap tables");
    const int N = h->N;
    HIPCHECK(h, hipSetDevice(h->device));
    settle(h, h->stream);
    int rc = upload_layers(h, layers);
    if (rc) return rc;
    if ((rc = ensure_workspace(h, 1))) return rc;
    double *dbg = nullptr;
    HIPCHECK(h, hipMalloc(&dbg, sizeof(double) * ((size_t)N * N + 3 * N + 1)));
    lvg_solve_opts o;
    lvg_solve_opts_default(&o);
    o.line_overlap = line_overlap;
    LvgLaunch L;
    fill_launch(h, L, &o);
    L.soa = h->d_soa;
    L.soa_ld = layers->nb_lay;
    L.lay_offset = layer;
    L.nb_lay = 1;
    L.dbg_matrix = dbg;
    L.dbg_df = dbg + (size_t)N * N;            // N + 1 (eq_error at [N])
    L.dbg_pop_in = L.dbg_df + N + 1;
    L.pops = L.dbg_pop_in + N;
    const LvgLaunch *dL = nullptr;
    if ((rc = push_launch(h, L, 0, h->stream, &dL))) { (void)hipFree(dbg); return rc; }
    hipError_t e = hipMemcpy(L.dbg_pop_in, pop_in, sizeof(double) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = h->big ? lvg_launch_debug_big(h->d_prob, dL, h->stream) : lvg_launch_debug(h->d_prob, dL, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    std::vector<double> host((size_t)N * N + 3 * N + 1);
    if (e == hipSuccess) e = hipMemcpy(host.data(), dbg, sizeof(double) * host.size(), hipMemcpyDeviceToHost);
    (void)hipFree(dbg);
    if (e != hipSuccess) return fail(h, LVG_E_DEVICE, "debug kernel: %s", hipGetErrorString(e));
    if (matrix_out) memcpy(matrix_out, host.data(), sizeof(double) * N * N);
    if (df_out) memcpy(df_out, host.data() + (size_t)N * N, sizeof(double) * N);
    if (eq_error) *eq_error = host[(size_t)N * N + N];
    memcpy(pop_out, host.data() + (size_t)N * N + 2 * N + 1, sizeof(double) * N);
    return LVG_OK;
}

int lvg_boundary_layer_populations(lvg_handle *h, const lvg_layers *layers, double *pops_out) {
    if (!h) return LVG_E_STATE;
    if (!layers || !pops_out) return fail(h, LVG_E_ARG, "bad arguments");
    const int nl = layers->nb_lay, N = h->N;
    if (nl == 0) return LVG_OK;
    if (!h->peers.empty()) {
        const int G = 1 + (int)h->peers.size();
        std::vector<lvg_handle *> peers;
        peers.swap(h->peers);          // each block runs on its device's handle alone
        std::vector<lvg_handle *> hs(1, h);
        hs.insert(hs.end(), peers.begin(), peers.end());
        std::vector<int> rc(G, LVG_OK);
        std::vector<std::thread> th;
        auto part = [&](int d) {
            int lo, hi;
            lvg_shard_range(nl, G, d, &lo, &hi);
            if (hi == lo) return;
            const lvg_layers v = layer_block(*layers, h->nb_comp, lo, hi);
            rc[d] = lvg_boundary_layer_populations(hs[d], &v, pops_out + (size_t)lo * N);
        };
        for (int d = 1; d < G; d++) th.emplace_back(part, d);
        part(0);
        for (auto &t : th) t.join();
        h->peers.swap(peers);
        for (int d = 0; d < G; d++)
            if (rc[d]) return d ? fail(h, rc[d], "device %d: %s", hs[d]->device, hs[d]->err.c_str()) : rc[d];
        return LVG_OK;
    }
    HIPCHECK(h, hipSetDevice(h->device));
    settle(h, h->stream);
    int rc = upload_layers(h, layers);
    if (rc) return rc;
    if ((rc = grow(h, (void **)&h->d_pops, &h->pops_cap, sizeof(double) * (size_t)nl * N))) return rc;
    if ((rc = grow(h, &h->d_status, &h->status_cap, sizeof(lvg_layer_status) * (size_t)nl))) return rc;
    const int grid = std::max(1, std::min(nl, h->cus * h->blocks_per_cu));
    if ((rc = ensure_workspace(h, grid))) return rc;
    lvg_solve_opts o;
    lvg_solve_opts_default(&o);
    LvgLaunch L;
    fill_launch(h, L, &o);
    L.soa = h->d_soa;
    L.soa_ld = nl;
    L.nb_lay = nl;
    L.pops = h->d_pops;
    L.status = h->d_status;
    L.dbg_mode = 2;
    const LvgLaunch *dL = nullptr;
    if ((rc = push_launch(h, L, 0, h->stream, &dL))) return rc;
    HIPCHECK(h, hipMemsetAsync(h->counter, 0, sizeof(int), h->stream));
    HIPCHECK(h, h->big ? lvg_launch_solve_big(h->d_prob, dL, grid, h->stream) : lvg_launch_solve(h->d_prob, dL, grid, h->stream));
    HIPCHECK(h, hipStreamSynchronize(h->stream));
    HIPCHECK(h, hipMemcpy(pops_out, h->d_pops, sizeof(double) * (size_t)nl * N, hipMemcpyDeviceToHost));
    return LVG_OK;
}

}  // extern "C"

// ---- post-processing: transition_data_container::find --------------------------------
namespace {
struct TmpDev {   // call-scoped device buffers
    std::vector<void *> ptrs;
    ~TmpDev() { for (void *p : ptrs) (void)hipFree(p); }
    template <class T> T *alloc(size_t n) {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return static_cast<T *>(p);
    }
};
}  // namespace

void lvg_find_opts_default(lvg_find_opts *o) {
    if (!o) return;
    o->rel_error = 1.e-5;
    o->min_optical_depth = 0.01;    // transition_data.cpp:182
    o->velocity_shift = 5.e+5;      // :190
    o->delta_aspect_ratio = 0.25;   // :18
    o->h2o22_up = o->h2o22_low = -1;
}

int lvg_find_transitions(lvg_handle *h, const lvg_layers *layers, const lvg_cloud_geometry *geo, const double *pops,
                         const lvg_find_opts *opts, int max_out, int *nb_out, lvg_transition *out, double *inv_arr,
                         double *gain_arr, double *exc_temp_arr) {
    if (!h) return LVG_E_STATE;
    if (!layers || !geo || !opts || !nb_out || max_out < 0 || (max_out > 0 && !out))
        return fail(h, LVG_E_ARG, "lvg_find_transitions: missing argument");
    *nb_out = 0;
    const int nl = layers->nb_lay, N = h->N, nlines = h->P.plain.nb_lines;
    if (nl == 0 || nlines == 0) return LVG_OK;
    if (!pops || !geo->dz || !geo->vel_n) return fail(h, LVG_E_ARG, "lvg_find_transitions: pops / dz / vel_n missing");
    HIPCHECK(h, hipSetDevice(h->device));
    settle(h, h->stream);
    int rc = upload_layers(h, layers);
    if (rc) return rc;
    TmpDev T;
    const size_t nll = (size_t)nlines * nl;
    double *d_pops = T.alloc<double>((size_t)nl * N), *d_dz = T.alloc<double>(nl), *d_vel = T.alloc<double>(nl);
    double *d_inv = T.alloc<double>(nll), *d_gain = T.alloc<double>(nll), *d_exc = T.alloc<double>(nll);
    double *d_lop = T.alloc<double>(nll), *d_dop = T.alloc<double>(nll), *d_vw = T.alloc<double>(nl);
    double *d_sum = T.alloc<double>(4 * (size_t)nlines);
    int *d_inverted = T.alloc<int>(nlines);
    lvgtr::TrArgs *d_args = T.alloc<lvgtr::TrArgs>(1);
    if (!d_pops || !d_dz || !d_vel || !d_inv || !d_gain || !d_exc || !d_lop || !d_dop || !d_vw || !d_sum ||
        !d_inverted || !d_args)
        return fail(h, LVG_E_NOMEM, "lvg_find_transitions: device allocation failed");
    HIPCHECK(h, hipMemcpy(d_pops, pops, sizeof(double) * (size_t)nl * N, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMemcpy(d_dz, geo->dz, sizeof(double) * nl, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMemcpy(d_vel, geo->vel_n, sizeof(double) * nl, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMemset(d_inverted, 0, sizeof(int) * nlines));
    const LvgModeLines &M = h->P.plain;
    lvgtr::TrArgs a{};
    a.N = N; a.nb_lines = nlines; a.nb_lay = nl; a.nb_comp = h->nb_comp; a.soa_ld = nl;
    a.line_u = M.line_u; a.line_l = M.line_l; a.line_aul = M.line_aul; a.line_e = M.line_e; a.line_sigma = M.line_sigma;
    a.g = h->P.g; a.mass = h->P.mass;
    a.soa = h->d_soa; a.pops = d_pops; a.dz = d_dz; a.vel_n = d_vel;
    a.height = geo->height; a.rel_error = opts->rel_error; a.velocity_shift = opts->velocity_shift;
    a.delta_aspect = opts->delta_aspect_ratio; a.h2o22_up = opts->h2o22_up; a.h2o22_low = opts->h2o22_low;
    a.inv = d_inv; a.gain = d_gain; a.exc = d_exc; a.lop = d_lop; a.dop = d_dop; a.vw = d_vw;
    a.inverted = d_inverted; a.line_sum = d_sum;
    HIPCHECK(h, hipMemcpy(d_args, &a, sizeof a, hipMemcpyHostToDevice));
    HIPCHECK(h, lvg_tr_launch(0, d_args, nlines, nl, 0, h->stream));
    std::vector<int> inverted(nlines), lu(nlines), ll(nlines);
    std::vector<double> sums(4 * (size_t)nlines), le(nlines);
    HIPCHECK(h, hipStreamSynchronize(h->stream));
    HIPCHECK(h, hipMemcpy(inverted.data(), d_inverted, sizeof(int) * nlines, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(sums.data(), d_sum, sizeof(double) * sums.size(), hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(lu.data(), M.line_u, sizeof(int) * nlines, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(ll.data(), M.line_l, sizeof(int) * nlines, hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(le.data(), M.line_e, sizeof(double) * nlines, hipMemcpyDeviceToHost));
    std::vector<int> sel;
    for (int n = 0; n < nlines; n++)
        if (inverted[n]) sel.push_back(n);
    const int nsel = (int)sel.size();
    if (nsel == 0) return LVG_OK;
    int *d_sel = T.alloc<int>(nsel);
    double *d_od = T.alloc<double>((size_t)nsel * LVG_NB_FREQ * LVG_NB_ASPECT);
    double *d_asp = T.alloc<double>((size_t)nsel * LVG_NB_ASPECT), *d_freq = T.alloc<double>((size_t)nsel * LVG_NB_FREQ);
    if (!d_sel || !d_od || !d_asp || !d_freq) return fail(h, LVG_E_NOMEM, "lvg_find_transitions: device allocation failed");
    HIPCHECK(h, hipMemcpy(d_sel, sel.data(), sizeof(int) * nsel, hipMemcpyHostToDevice));
    a.sel = d_sel; a.nb_sel = nsel; a.od = d_od; a.tau_asp = d_asp; a.tau_freq = d_freq;
    HIPCHECK(h, hipMemcpy(d_args, &a, sizeof a, hipMemcpyHostToDevice));
    HIPCHECK(h, lvg_tr_launch(1, d_args, nlines, nl, nsel, h->stream));
    HIPCHECK(h, hipStreamSynchronize(h->stream));
    std::vector<double> asp((size_t)nsel * LVG_NB_ASPECT), freq((size_t)nsel * LVG_NB_FREQ);
    HIPCHECK(h, hipMemcpy(asp.data(), d_asp, sizeof(double) * asp.size(), hipMemcpyDeviceToHost));
    HIPCHECK(h, hipMemcpy(freq.data(), d_freq, sizeof(double) * freq.size(), hipMemcpyDeviceToHost));
    std::vector<int> kept;   // indices into sel, in line order (tau_max >= min_optical_depth)
    for (int k = 0; k < nsel; k++)
        if (asp[(size_t)k * LVG_NB_ASPECT] >= opts->min_optical_depth) kept.push_back(k);
    const int cnt = (int)kept.size();
    *nb_out = cnt;
    for (int j = 0; j < cnt && j < max_out; j++) {
        const int k = kept[cnt - 1 - j], n = sel[k];   // the reference's list is push_front
        lvg_transition &r = out[j];
        r.up = lu[n]; r.low = ll[n];
        r.lay_nb_hg = (int)sums[4 * (size_t)n + 3];
        r.reserved = 0;
        r.energy = le[n];
        r.inv = sums[4 * (size_t)n + 0];
        r.gain = sums[4 * (size_t)n + 1];
        r.tau_eff = sums[4 * (size_t)n + 2];
        r.tau_max = asp[(size_t)k * LVG_NB_ASPECT];
        memcpy(r.tau_vs_aspect_ratio, &asp[(size_t)k * LVG_NB_ASPECT], sizeof r.tau_vs_aspect_ratio);
        memcpy(r.tau_vs_frequency, &freq[(size_t)k * LVG_NB_FREQ], sizeof r.tau_vs_frequency);
        const size_t off = (size_t)n * nl;
        if (inv_arr) HIPCHECK(h, hipMemcpy(inv_arr + (size_t)j * nl, d_inv + off, sizeof(double) * nl, hipMemcpyDeviceToHost));
        if (gain_arr) HIPCHECK(h, hipMemcpy(gain_arr + (size_t)j * nl, d_gain + off, sizeof(double) * nl, hipMemcpyDeviceToHost));
        if (exc_temp_arr) HIPCHECK(h, hipMemcpy(exc_temp_arr + (size_t)j * nl, d_exc + off, sizeof(double) * nl, hipMemcpyDeviceToHost));
    }
    return LVG_OK;
}

int lvg_lim_luminosity(lvg_handle *h, const lvg_layers *layers, const lvg_cloud_geometry *geo, const double *pops,
                       int nb_trans, const int *up, const int *low, int layer_pops, double *lum, double *lum_arr,
                       double *emiss_coeff_arr, double *pump_rate_arr, double *pump_eff_arr, double *loss_rate_arr) {
    if (!h) return LVG_E_STATE;
    if (!layers || !geo || nb_trans < 0 || (nb_trans > 0 && (!up || !low)))
        return fail(h, LVG_E_ARG, "lvg_lim_luminosity: missing argument");
    const int nl = layers->nb_lay, N = h->N;
    if (nl == 0 || nb_trans == 0) return LVG_OK;
    if (!pops || !geo->dz) return fail(h, LVG_E_ARG, "lvg_lim_luminosity: pops / dz missing");
    for (int t = 0; t < nb_trans; t++)
        if (up[t] <= low[t] || low[t] < 0 || up[t] >= N) return fail(h, LVG_E_ARG, "transition %d: need N > up > low >= 0", t);
    if (2 * nb_trans > N * N) return fail(h, LVG_E_UNSUPPORTED, "too many transitions for the slot scratch");
    HIPCHECK(h, hipSetDevice(h->device));
    settle(h, h->stream);
    int rc = upload_layers(h, layers);
    if (rc) return rc;
    if ((rc = grow(h, (void **)&h->d_pops, &h->pops_cap, sizeof(double) * (size_t)nl * N))) return rc;
    HIPCHECK(h, hipMemcpy(h->d_pops, pops, sizeof(double) * (size_t)nl * N, hipMemcpyHostToDevice));
    const int grid = std::max(1, std::min(nl, h->cus * h->blocks_per_cu));
    if ((rc = ensure_workspace(h, grid))) return rc;
    TmpDev T;
    const size_t ntl = (size_t)nb_trans * nl;
    int *d_up = T.alloc<int>(nb_trans), *d_low = T.alloc<int>(nb_trans);
    double *d_dz = T.alloc<double>(nl), *d_lum = T.alloc<double>(nb_trans);
    double *d_arr[5];
    for (auto &p : d_arr) p = T.alloc<double>(ntl);
    LvgLumArgs *d_args = T.alloc<LvgLumArgs>(1);
    if (!d_up || !d_low || !d_dz || !d_lum || !d_arr[0] || !d_arr[1] || !d_arr[2] || !d_arr[3] || !d_arr[4] || !d_args)
        return fail(h, LVG_E_NOMEM, "lvg_lim_luminosity: device allocation failed");
    HIPCHECK(h, hipMemcpy(d_up, up, sizeof(int) * nb_trans, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMemcpy(d_low, low, sizeof(int) * nb_trans, hipMemcpyHostToDevice));
    HIPCHECK(h, hipMemcpy(d_dz, geo->dz, sizeof(double) * nl, hipMemcpyHostToDevice));
    LvgLumArgs a{};
    a.nb_trans = nb_trans; a.layer_pops = layer_pops ? 1 : 0; a.up = d_up; a.low = d_low; a.dz = d_dz; a.height = geo->height;
    a.lum = d_lum; a.lum_arr = d_arr[0]; a.emiss = d_arr[1]; a.pump_rate = d_arr[2]; a.pump_eff = d_arr[3]; a.loss_rate = d_arr[4];
    HIPCHECK(h, hipMemcpy(d_args, &a, sizeof a, hipMemcpyHostToDevice));
    lvg_solve_opts o;
    lvg_solve_opts_default(&o);
    LvgLaunch L;
    fill_launch(h, L, &o);
    L.nb_lay = nl; L.lay_offset = 0; L.soa_ld = nl; L.soa = h->d_soa; L.pops = h->d_pops;
    const LvgLaunch *dL = nullptr;
    if ((rc = push_launch(h, L, 0, h->stream, &dL))) return rc;
    HIPCHECK(h, hipMemsetAsync(h->counter, 0, sizeof(int), h->stream));
    HIPCHECK(h, h->big ? lvg_launch_lum_big(h->d_prob, dL, d_args, grid, nb_trans, nl, h->stream)
                       : lvg_launch_lum(h->d_prob, dL, d_args, grid, nb_trans, nl, h->stream));
    HIPCHECK(h, hipStreamSynchronize(h->stream));
    if (lum) HIPCHECK(h, hipMemcpy(lum, d_lum, sizeof(double) * nb_trans, hipMemcpyDeviceToHost));
    double *outs[5] = {lum_arr, emiss_coeff_arr, pump_rate_arr, pump_eff_arr, loss_rate_arr};
    for (int k = 0; k < 5; k++)
        if (outs[k]) HIPCHECK(h, hipMemcpy(outs[k], d_arr[k], sizeof(double) * ntl, hipMemcpyDeviceToHost));
    return LVG_OK;
}

