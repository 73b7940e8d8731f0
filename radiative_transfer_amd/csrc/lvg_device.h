// lvg_device.h — packed, device-resident form of an lvg_problem (built once in
// lvg_create) and the per-launch parameter block of the solve kernels.
//
// Layout choices (HBM, all fp64 unless noted):
//  * collision tables are stored T-major, coeff[t][pair] (pair = f(f-1)/2 + s), so a
//    wavefront that walks consecutive level pairs at one temperature index reads
//    contiguous bytes (coll_rates.cpp:54-59 reads coeff[pair][t]);
//  * the molecule rule (coll_rates_{ch3oh,h2o,oh}.cpp get_rate_neutrals) is compiled
//    on the host into a per-pair class byte plus a small class table of
//    (table, concentration-combination) terms, so the device evaluates
//    sum_k k_table(T) * n_combo with no molecule branches;
//  * radiative lines are a flat list (u, l, A_ul, A_lu, E, sigma_dust[c]) plus
//    "units" (1 line, or 2 overlapping lines of iteration_scheme_line_overlap) and a
//    per-level CSR of (line, role) used to form the diagonal deterministically.
#pragma once
#include <stdint.h>

#define LVG_MAX_TABLES   16
#define LVG_MAX_TERMS    6
#define LVG_MAX_CLASSES  32
#define LVG_MAX_COMBOS   16
#define LVG_MAX_DUST     4
#define LVG_HIST_SLOTS   8      // ring slots for prev_level_pop / residual_list
#define LVG_WAVE_INV_FIELDS 20  // wave kernel: per-layer line-invariant doubles per unit (slot tail)
#define LVG_WAVE_NMAX    64     // wave kernel level cap (slots carry the invariant records up to here)

struct LvgTermTable {
    int8_t table[LVG_MAX_CLASSES][LVG_MAX_TERMS];  // neutral terms, -1 = none
    int8_t combo[LVG_MAX_CLASSES][LVG_MAX_TERMS];
    int8_t etable[LVG_MAX_CLASSES];                // first applicable electron table, -1 = none
    int8_t group[LVG_MAX_CLASSES];                 // terms [group, nt) are summed first, then added
                                                   // (coll_rates_oh.cpp:341: d += k1*c1 + k2*c2)
    double combo_w[LVG_MAX_COMBOS][5];             // combo = sum_s w[s] * n[s] (he, ph2, oh2, h, e)
    int    nb_combos;
    int    nt_max;                                 // most neutral terms of any class
    int    any_e;                                  // some class has an electron table
};

struct LvgModeLines {          // one radiative scheme (plain LVG or line overlap)
    int nb_lines, nb_units;
    const int    *line_u, *line_l;
    const double *line_aul, *line_alu, *line_e;
    const double *line_sigma;  // [nb_comp][nb_lines] dust cross section at the line energy
    const int    *unit_l0, *unit_l1;   // unit -> line index (l1 = -1 for a single line)
    // per level d, radiative partners r sorted ascending: column d of the rate matrix
    // gets +y at row r and the diagonal gets -y (y index = line*2 + role,
    // role 0: d is the upper level -> y1 = A_ul(1+I); role 1: lower -> y2 = A_lu I)
    const int    *col_ptr;     // [N+1]
    const int    *col_r;
    const int    *col_y;
    const int    *line_idx;    // [N*N] y index of the term at (row r, column d), -1 if none
    // diagonal order: interleaved with the collision terms (plain scheme,
    // iteration_lvg.cpp:118-147) or after all of them in line order (overlap
    // scheme, iteration_lvg.cpp:354-412)
    int           diag_interleaved;
    const int    *diag_ptr;    // [N+1], line order (overlap scheme)
    const int    *diag_ent;
};

struct LvgDevProblem {
    int N, nb_comp, nb_tables, nb_neutral, nb_electron;
    double mass;
    const double *energy;      // [N]
    const double *g;           // [N]
    const double *einst;       // [N*N]
    const double *einst_t;     // [N*N] transposed: einst_t[r*N + d] = einst[d*N + r]
    // collision tables
    const int     *tab_jmax, *tab_nb_lev;
    const int64_t *tab_tg_off, *tab_c_off;
    const double  *tab_tgrid, *tab_coeff;          // T-major coeff[t][pair]
    const double  *tab_deriv;                      // T-major slope of interval t, [t][pair]
    const uint8_t *pair_class;                     // [N(N-1)/2]
    LvgTermTable   terms;
    // LVG escape table (lvg_method_functions.cpp:74-110)
    int esc_nd, esc_ng;
    const double *esc_delta, *esc_gamma, *esc_p;
    // line-overlap tables (lvg_method_functions.cpp:324-392)
    int ov_nd, ov_ndx, ov_ngr, ov_ng;
    const double *ov_ld, *ov_dx, *ov_gr, *ov_g, *ov_p1, *ov_p2;
    LvgModeLines plain, overlap;
};

// Per-launch options / buffers.
struct LvgLaunch {
    int nb_lay, lay_offset, soa_ld;   // layer SoA row stride (= total layers of the SoA)
    const double *soa;                // [10 + nb_comp][soa_ld]
    double       *pops;               // [nb_lay][N] (layer index relative to lay_offset)
    void         *status;             // lvg_layer_status[nb_lay]
    double        min_error;
    int max_iter_acc, max_iter_plain, accel_start, accel_period, accel_nb;
    int acceleration, allow_plain_retry, init, line_overlap;
    // warm chains (LVG_INIT_WARM_CHAIN): queue items are chains, chain c is layers
    // [chain_off[c], chain_off[c+1]) solved in order by one workgroup / wave, each layer
    // starting from its predecessor when that converged (radiative_transfer.cpp:247-252)
    const int *chain_off;             // [nb_chain + 1], NULL: queue items are layers
    int nb_chain;
    // workspace (per resident block slot)
    double   *ws;                     // [nb_slots][ws_stride]
    int64_t   ws_stride;
    int      *counter;                // work queue head
    const int *order;                 // queue position -> layer (NULL: index order)
    // collision operators built ahead by coll_kernel (NULL: each layer builds its own):
    // K [nb_lay][N][N] and the boundary matrix B [nb_lay][N][N] (B NULL when not needed)
    const double *kall, *ball;
    // without electron tables B is K + A/2 above the diagonal and K below it: then only
    // its diagonal is stored, bdiag [nb_lay][N], and the boundary LU forms B from K
    const double *bdiag;
    const int *coll_order;            // coll_kernel: position -> layer (temperature order), NULL: index order
    // debug probe outputs (lvg_debug_calc_new_pop)
    double   *dbg_matrix, *dbg_df, *dbg_pop_in;
    int       dbg_mode;               // 0 solve, 1 debug calc_new_pop, 2 boundary pops only
};

// lim_luminosity_lvg parameters (lum_kernel in lvg_kernels.hip)
struct LvgLumArgs {
    int nb_trans, layer_pops;          // layer_pops: 0 = intensity_calc sees layer 0 (reference)
    const int *up, *low;               // [nb_trans]
    const double *dz;                  // [nb_lay]
    double height;
    double *lum, *lum_arr, *emiss, *pump_rate, *pump_eff, *loss_rate;   // [nb_trans], [nb_trans][nb_lay]
};

// Parameter block of the post-processing kernels (lvg_transitions.hip).
namespace lvgtr {
struct TrArgs {
    int N, nb_lines, nb_lay, nb_comp, soa_ld;
    const int *line_u, *line_l;
    const double *line_aul, *line_e, *line_sigma;   // sigma: [comp][line]
    const double *g;                                // [N]
    double mass;
    const double *soa;                              // [10 + nb_comp][soa_ld] layer SoA
    const double *pops;                             // [nb_lay][N]
    const double *dz, *vel_n;                       // [nb_lay]
    double height, rel_error, velocity_shift, delta_aspect;
    int h2o22_up, h2o22_low;
    // per (line, layer) outputs, [nb_lines][nb_lay]
    double *inv, *gain, *exc, *lop, *dop;
    double *vw;                                     // [nb_lay] thermal + turbulent width
    int *inverted;                                  // [nb_lines]
    double *line_sum;                               // [nb_lines][4]: inv, gain, tau_eff, lay_nb_hg
    // profile stage
    const int *sel;                                 // [nb_sel] line indices (inverted lines)
    int nb_sel;
    double *od;                                     // [nb_sel][NB_FREQ][NB_ASPECT]
    double *tau_asp, *tau_freq;                     // [nb_sel][37], [nb_sel][300]
};
}  // namespace lvgtr
