/*
 * lvg_oracle.c — CPU ORACLE (test infrastructure only; never shipped, never on
 * the product path). A plain-C restatement of the reference's LVG level-
 * population path, used by tests/ as the parity checker and by bench.py as the
 * cpu_baseline ("port") leg.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or data for this path
 * and cannot be compiled here (every hot-path file includes headers of its
 * absent numerics library: utils.h, linear_algebra.h, interpolation.h,
 * integration.h, special_functions.h, constants.h — radiative_transfer.vcxproj:93,
 * :156-159). This file therefore restates the reference sources function by
 * function (citations below), and restates the three pieces of the absent
 * library it needs with explicit, documented choices:
 *   - lu_matrix_solve: in-place LU with partial pivoting (first maximum of |a_ik|
 *     wins), right-looking kij order, forward substitution fused into the
 *     elimination, column-ordered back substitution;
 *   - locate_index: -1 below the grid, n-1 above it, else a[j] <= x < a[j+1]
 *     (value-equivalent under the clamped interpolation that uses it);
 *   - constants.h: CODATA-2018 CGS values.
 * Arithmetic follows the reference's expression order; build with
 * -ffp-contract=off (no FMA contraction) so it is a faithful scalar restatement.
 * Three deliberate, documented choices make the oracle and the GPU path agree
 * bit for bit (DESIGN.md "Parity"): the LU updates use an explicit fused
 * multiply-add (fma) — the absent library's rounding is unknown anyway; exp and
 * log10 come from include/lvg_math.h (< 1-2 ulp from libm, identical on host and
 * device); the thermal width uses sqrt(x) for the reference's pow(x, 0.5).
 *
 * ORACLE_REF_ARITH (second build, oracle/_build/liblvg_oracle_ref.so): the same
 * restatement with the reference's own arithmetic instead of those three choices —
 * glibc exp/log10/log (coll_rates.cpp:194, coll_rates_ch3oh.cpp:531,
 * transition_data.cpp:348, lvg_method_functions.cpp:330), pow(x, 0.5) and pow(x, 2.)
 * (iteration_lvg.cpp:65, transition_data.cpp:256-262), and an LU whose updates are
 * a - l*b with two roundings (no FMA; lu_matrix_solve call site iteration_lvg.cpp:100).
 * tests/test_oracle_refarith_cpu.py measures how far the bit-exact build sits from
 * it against SURVEY.md 8(c)'s tolerances.
 */
#include "lvg_oracle.h"
#include "../include/lvg_math.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* The three choices can be undone one at a time (tests/test_oracle_refarith_cpu.py
 * attributes the Ng-layer gap to one of them): ORACLE_REF_EXP glibc exp/log10/log,
 * ORACLE_REF_LU the LU without fma, ORACLE_REF_POW pow(x, 0.5) / pow(x, 2.).
 * ORACLE_REF_ARITH sets all three. */
#ifdef ORACLE_REF_ARITH
#define ORACLE_REF_EXP 1
#define ORACLE_REF_LU  1
#define ORACLE_REF_POW 1
#endif
#ifdef ORACLE_REF_EXP
#define O_EXP(x)         exp(x)
#define O_LOG10(x)       log10(x)
#define O_LOG(x)         log(x)
#else
#define O_EXP(x)         lvg_exp(x)
#define O_LOG10(x)       lvg_log10(x)
#define O_LOG(x)         lvg_log(x)
#endif
#ifdef ORACLE_REF_LU
#define O_FMSUB(l, b, a) ((a) - (l) * (b))      /* a -= l*b: product and difference rounded */
#else
#define O_FMSUB(l, b, a) fma(-(l), (b), (a))
#endif
#ifdef ORACLE_REF_POW
#define O_SQRT(x)        pow((x), 0.5)
#define O_SQR(x)         pow((x), 2.)
#else
#define O_SQRT(x)        sqrt(x)
#define O_SQR(x)         ((x) * (x))
#endif
/* which choices this build undoes: 1 exp/log10/log, 2 LU without fma, 4 pow */
int oracle_ref_arith(void)
{
    int m = 0;
#ifdef ORACLE_REF_EXP
    m |= 1;
#endif
#ifdef ORACLE_REF_LU
    m |= 2;
#endif
#ifdef ORACLE_REF_POW
    m |= 4;
#endif
    return m;
}

/* constants.h (absent; CODATA 2018, CGS) — used at iteration_lvg.cpp:65, :168,
 * :455, coll_rates.cpp:194 */
#define BOLTZMANN_CONSTANT    1.380649e-16
#define CM_INVERSE_TO_KELVINS 1.438776877
#define EIGHT_PI              25.132741228718345
#define SPEED_OF_LIGHT        2.99792458e+10

#define MIN_COLLISION_RATE 1.e-99   /* coll_rates.h:9 */
#define INV_TRANS_FACTOR   -0.1     /* iteration_lvg.cpp:23 */
#define MIN_LINE_OPACITY   1.e-99   /* iteration_lvg.cpp:24 */
#define MAX_TABLES 16
#define MAX_HIST   16

/* ------------------------------------------------------------------------ */
/* absent numerics library                                                   */
/* ------------------------------------------------------------------------ */

/* locate_index(arr, n, x, j) — used at lvg_method_functions.cpp:79-80, :330-333 */
static int locate_index(const double *a, int n, double x)
{
    if (x < a[0]) return -1;
    if (x > a[n - 1]) return n - 1;
    int l = 0, r = n - 1;
    while (r - l > 1) {
        int m = l + ((r - l) >> 1);
        if (a[m] <= x) l = m; else r = m;
    }
    return l;
}

/* lu_matrix_solve(double **a, double *b, int n) — call sites
 * iteration_lvg.cpp:100, iteration_control.cpp:87, iteration_control.h:176. */
int oracle_lu_solve(double *a, double *b, int n)
{
    int sing = 0;
    for (int k = 0; k < n; k++) {
        int p = k;
        double amax = fabs(a[k * n + k]);
        for (int i = k + 1; i < n; i++) {
            double v = fabs(a[i * n + k]);
            if (v > amax) { amax = v; p = i; }
        }
        if (p != k) {
            for (int j = 0; j < n; j++) {
                double t = a[k * n + j]; a[k * n + j] = a[p * n + j]; a[p * n + j] = t;
            }
            double t = b[k]; b[k] = b[p]; b[p] = t;
        }
        double piv = a[k * n + k];
        if (piv == 0.) sing = 1;
        for (int i = k + 1; i < n; i++) {
            double l = a[i * n + k] / piv;
            a[i * n + k] = l;
            for (int j = k + 1; j < n; j++)
                a[i * n + j] = O_FMSUB(l, a[k * n + j], a[i * n + j]);
            b[i] = O_FMSUB(l, b[k], b[i]);
        }
    }
    for (int k = n - 1; k >= 0; k--) {
        b[k] /= a[k * n + k];
        double x = b[k];
        for (int i = 0; i < k; i++)
            b[i] = O_FMSUB(a[i * n + k], x, b[i]);
    }
    return sing ? -1 : 0;
}

/* ------------------------------------------------------------------------ */
/* tables                                                                    */
/* ------------------------------------------------------------------------ */

/* collision_data::locate (coll_rates.cpp:71-82): strict '<' (quirk q8) */
static int coll_locate(const lvg_coll_table *t, double temp)
{
    int j, l = 0, r = t->jmax - 1;
    while (r - l > 1) {
        j = l + ((r - l) >> 1);
        if (t->tgrid[j] < temp) l = j; else r = j;
    }
    return l;
}

/* collision_data::get_rate (coll_rates.cpp:54-59) + calc_coeff_deriv (:61-69) */
static double coll_get_rate(const lvg_coll_table *t, int f, int s, int lo, double temp)
{
    int i = f * (f - 1) / 2 + s;
    const double *c = t->coeff + (size_t)i * t->jmax;
    double deriv = (c[lo + 1] - c[lo]) / (t->tgrid[lo + 1] - t->tgrid[lo]);
    return c[lo] + deriv * (temp - t->tgrid[lo]);
}

static double max_temp(const lvg_coll_table *t) { return t->tgrid[t->jmax - 1]; }

/* lvg_method_data::get_esc_func (lvg_method_functions.cpp:74-110) */
double oracle_esc_func(const lvg_esc_table *T, double gamma, double delta)
{
    int k = locate_index(T->delta, T->nb_d, delta);
    int l = locate_index(T->gamma, T->nb_g, gamma);
    double t, u, escf;
    if (k < 0) { t = 0.; k = 0; }
    else if (k > T->nb_d - 2) { t = 1.; k = T->nb_d - 2; }
    else t = (delta - T->delta[k]) / (T->delta[k + 1] - T->delta[k]);
    if (l < 0) { l = 0; u = 0.; }
    else if (l > T->nb_g - 2) { l = T->nb_g - 2; u = 1.; }
    else u = (gamma - T->gamma[l]) / (T->gamma[l + 1] - T->gamma[l]);
    const double *p = T->p;
    int ng = T->nb_g;
    escf = p[k * ng + l] * (1. - t) * (1. - u) + p[(k + 1) * ng + l] * t * (1. - u)
         + p[k * ng + l + 1] * (1. - t) * u + p[(k + 1) * ng + l + 1] * u * t;
    if (escf > 1.) escf = 1.;
    else if (escf < 0.) escf = 0.;
    return escf;
}

/* lvg_line_overlap_data::get_esc_func (lvg_method_functions.cpp:324-392) */
double oracle_overlap_esc_func(const lvg_overlap_table *T, double gamma, double delta,
                               double gamma_ratio, double delta_x)
{
    int l, k, n, m;
    double u, t, p, y, escf;
    delta = O_LOG10(delta);
    m = locate_index(T->log10_delta, T->nb_d, delta);
    l = locate_index(T->gamma, T->nb_g, gamma);
    k = locate_index(T->gratio, T->nb_gr, gamma_ratio);
    n = locate_index(T->dx, T->nb_dx, delta_x);
    y = u = t = p = 0.;
    if (m < 0) m = 0;
    else if (m > T->nb_d - 2) { m = T->nb_d - 2; y = 1.; }
    else y = (delta - T->log10_delta[m]) / (T->log10_delta[m + 1] - T->log10_delta[m]);
    if (n < 0) n = 0;
    else if (n > T->nb_dx - 2) { p = 1.; n = T->nb_dx - 2; }
    else p = (delta_x - T->dx[n]) / (T->dx[n + 1] - T->dx[n]);
    if (l < 0) l = 0;
    else if (l > T->nb_g - 2) { l = T->nb_g - 2; u = 1.; }
    else u = (gamma - T->gamma[l]) / (T->gamma[l + 1] - T->gamma[l]);
    if (k < 0) k = 0;
    else if (k > T->nb_gr - 2) { t = 1.; k = T->nb_gr - 2; }
    else t = (gamma_ratio - T->gratio[k]) / (T->gratio[k + 1] - T->gratio[k]);

    const int W = T->nb_gr * T->nb_g, ndx = T->nb_dx, ng = T->nb_g;
#define PA(r, c) T->p[(size_t)(r) * W + (c)]
    escf = PA(m * ndx + n, k * ng + l) * (1. - u) * (1. - t) * (1. - p) * (1. - y)
        + PA(m * ndx + n, k * ng + l + 1) * u * (1. - t) * (1. - p) * (1. - y)
        + PA(m * ndx + n, (k + 1) * ng + l) * (1. - u) * t * (1. - p) * (1. - y)
        + PA(m * ndx + n, (k + 1) * ng + l + 1) * u * t * (1. - p) * (1. - y)
        + PA(m * ndx + n + 1, k * ng + l) * (1. - u) * (1. - t) * p * (1. - y)
        + PA(m * ndx + n + 1, k * ng + l + 1) * u * (1. - t) * p * (1. - y)
        + PA(m * ndx + n + 1, (k + 1) * ng + l) * (1. - u) * t * p * (1. - y)
        + PA(m * ndx + n + 1, (k + 1) * ng + l + 1) * u * t * p * (1. - y)
        + PA((m + 1) * ndx + n, k * ng + l) * (1. - u) * (1. - t) * (1. - p) * y
        + PA((m + 1) * ndx + n, k * ng + l + 1) * u * (1. - t) * (1. - p) * y
        + PA((m + 1) * ndx + n, (k + 1) * ng + l) * (1. - u) * t * (1. - p) * y
        + PA((m + 1) * ndx + n, (k + 1) * ng + l + 1) * u * t * (1. - p) * y
        + PA((m + 1) * ndx + n + 1, k * ng + l) * (1. - u) * (1. - t) * p * y
        + PA((m + 1) * ndx + n + 1, k * ng + l + 1) * u * (1. - t) * p * y
        + PA((m + 1) * ndx + n + 1, (k + 1) * ng + l) * (1. - u) * t * p * y
        + PA((m + 1) * ndx + n + 1, (k + 1) * ng + l + 1) * u * t * p * y;
#undef PA
    if (escf > 1.) escf = 1.;
    else if (escf < 0.) escf = 0.;
    return escf;
}

/* dust_component::absorption (dust_model.cpp:473-490) and
 * dust_model::absorption(E, conc) (dust_model.cpp:834-841) */
static double dust_comp_absorption(const lvg_dust_component *c, double energy)
{
    int n = c->nb_en;
    if (energy < c->energy[0])
        return c->abs_coeff[0] * pow(c->energy[0] / energy, c->wvl_exp);
    if (energy > c->energy[n - 1])
        return c->abs_coeff[n - 1];
    int i, l = 0, r = n - 1;
    while (r - l > 1) {
        i = l + ((r - l) >> 1);
        if (c->energy[i] < energy) l = i; else r = i;
    }
    double deriv = (c->abs_coeff[l + 1] - c->abs_coeff[l]) / (c->energy[l + 1] - c->energy[l]);
    return c->abs_coeff[l] + deriv * (energy - c->energy[l]);
}

double oracle_dust_absorption(const lvg_dust *d, double energy, const double *conc)
{
    double a = 0.;
    if (!d) return a;
    for (int i = 0; i < d->nb_comp; i++)
        a += dust_comp_absorption(&d->comp[i], energy) * conc[i];
    return a;
}

/* ------------------------------------------------------------------------ */
/* collisional_transitions and the molecule overrides                        */
/* ------------------------------------------------------------------------ */

typedef struct {
    const lvg_problem *P;
    int N;
    /* iteration_scheme_lvg state (iteration_lvg.h:20-33) */
    double temp_n, temp_el, mol_conc, vel_width, vel_grad;
    const double *dgrain_conc;
    int indices[MAX_TABLES];
    double conc[MAX_TABLES];
    double *matrix;           /* N*N */
    /* line_list of iteration_scheme_line_overlap (iteration_lvg.h:92) */
    int nb_groups;
    int *groups;              /* [nb_groups*5]: nb, u0, l0, u1, l1 */
} scheme_t;

/* collisional_transitions::set_gas_param (coll_rates.cpp:152-174) and the
 * overrides ch3oh (coll_rates_ch3oh.cpp:472-481), h2o (coll_rates_h2o.cpp:515-527),
 * oh (coll_rates_oh.cpp:323-332), oh_hf (coll_rates_oh.cpp:380-389). */
static void set_gas_param(scheme_t *S, double tn, double te, double he, double ph2, double oh2,
                          double h, double e)
{
    const lvg_collisions *C = S->P->coll;
    int nb1 = C->nb_neutral, nb2 = C->nb_neutral + C->nb_electron;
    for (int i = 0; i < nb1; i++) S->indices[i] = coll_locate(&C->tables[i], tn);
    for (int i = nb1; i < nb2; i++) { S->conc[i] = e; S->indices[i] = coll_locate(&C->tables[i], te); }
    switch (C->rule) {
    case LVG_COLL_CH3OH:
    case LVG_COLL_OH_HF:
        S->conc[0] = he; S->conc[1] = ph2; S->conc[2] = oh2; break;
    case LVG_COLL_OH:
        S->conc[0] = he; S->conc[1] = ph2; S->conc[2] = oh2; break;
    case LVG_COLL_H2O:
        S->conc[0] = he; S->conc[1] = he + 0.2 * h; S->conc[2] = ph2; S->conc[3] = oh2;
        S->conc[4] = ph2 + oh2; S->conc[5] = h; break;
    default: {
        double sp[LVG_NB_SPECIES] = {he, ph2, oh2, h, e};
        for (int i = 0; i < nb1; i++) S->conc[i] = sp[C->tables[i].species];
    } }
}

#define KRATE(t, T) coll_get_rate(&tab[t], up, low, S->indices[t], ((T) < max_temp(&tab[t])) ? (T) : max_temp(&tab[t]))

/* get_rate_neutrals: base coll_rates.cpp:181-197; ch3oh coll_rates_ch3oh.cpp:484-533;
 * h2o coll_rates_h2o.cpp:530-548; oh coll_rates_oh.cpp:334-347; oh_hf coll_rates_oh.cpp:392-407 */
static void get_rate_neutrals(const scheme_t *S, int up, int low, double *down_rate, double *up_rate)
{
    const lvg_molecule *M = S->P->mol;
    const lvg_collisions *C = S->P->coll;
    const lvg_coll_table *tab = C->tables;
    const double *c = S->conc;
    double tn = S->temp_n, d = 0.;
    int rule = C->rule;
    if (rule == LVG_COLL_CH3OH) {
        if (M->v[up] == M->v[low]) {
            if (M->v[up] == 0 && M->j[up] <= 9 && M->j[low] <= 9)
                d = KRATE(1, tn) * c[1] + KRATE(2, tn) * c[2];
            else
                d = KRATE(1, tn) * (c[1] + c[2]);
            d += KRATE(0, tn) * c[0];
        } else {
            d = KRATE(0, tn) * (c[0] + c[1] + 3. * c[2]);
        }
        if (d > MIN_COLLISION_RATE)
            *up_rate = d * O_EXP((M->energy[low] - M->energy[up]) * CM_INVERSE_TO_KELVINS / tn) * M->g[up] / ((double)M->g[low]);
        else *up_rate = d = 0.;
        *down_rate = d;
        return;
    }
    if (rule == LVG_COLL_H2O) {
        if (up < 45)
            d = KRATE(0, tn) * c[0] + KRATE(2, tn) * c[2] + KRATE(3, tn) * c[3] + KRATE(5, tn) * c[5];
        else
            d = KRATE(1, tn) * c[1] + KRATE(4, tn) * c[4];
        if (d > MIN_COLLISION_RATE)
            *up_rate = d * O_EXP((M->energy[low] - M->energy[up]) * CM_INVERSE_TO_KELVINS / tn) * M->g[up] / ((double)M->g[low]);
        else *up_rate = d = 0.;
        *down_rate = d;
        return;
    }
    if (rule == LVG_COLL_OH || rule == LVG_COLL_OH_HF) {
        double u = 0.;
        if (rule == LVG_COLL_OH) {
            d = KRATE(0, tn) * c[0];                  /* no bound check: quirk q10 */
        } else if (up < tab[0].nb_lev) {
            d = KRATE(0, tn) * c[0];
        }
        if (up < tab[1].nb_lev)
            d += KRATE(1, tn) * c[1] + KRATE(2, tn) * c[2];
        if (d > MIN_COLLISION_RATE)
            u = d * O_EXP((M->energy[low] - M->energy[up]) * CM_INVERSE_TO_KELVINS / tn) * M->g[up] / ((double)M->g[low]);
        else d = 0.;
        *down_rate = d; *up_rate = u;
        return;
    }
    /* base class */
    for (int i = 0; i < C->nb_neutral; i++)
        if (up < tab[i].nb_lev) d += KRATE(i, tn) * c[i];
    if (d > MIN_COLLISION_RATE)
        *up_rate = d * O_EXP((M->energy[low] - M->energy[up]) * CM_INVERSE_TO_KELVINS / tn) * M->g[up] / ((double)M->g[low]);
    else *up_rate = d = 0.;
    *down_rate = d;
}

/* collisional_transitions::get_rate_electrons (coll_rates.cpp:199-217): only the
 * first applicable set (quirk q5) */
static void get_rate_electrons(const scheme_t *S, int up, int low, double *down_rate, double *up_rate)
{
    const lvg_molecule *M = S->P->mol;
    const lvg_collisions *C = S->P->coll;
    const lvg_coll_table *tab = C->tables;
    double te = S->temp_el, d = 0.;
    for (int i = C->nb_neutral; i < C->nb_neutral + C->nb_electron; i++) {
        if (up < tab[i].nb_lev) { d = KRATE(i, te) * S->conc[i]; break; }
    }
    if (d > MIN_COLLISION_RATE)
        *up_rate = d * O_EXP((M->energy[low] - M->energy[up]) * CM_INVERSE_TO_KELVINS / te) * M->g[up] / ((double)M->g[low]);
    else *up_rate = d = 0.;
    *down_rate = d;
}
#undef KRATE

/* ------------------------------------------------------------------------ */
/* iteration_scheme_lvg                                                      */
/* ------------------------------------------------------------------------ */

#define LAYER(f) (L->f[l])

/* set_vel_grad (iteration_lvg.h:44), set_dust_parameters (iteration_lvg.cpp:70-85),
 * set_parameters (iteration_lvg.cpp:59-68) */
static void scheme_set_layer(scheme_t *S, const lvg_layers *L, int l)
{
    int nc = S->P->dust ? S->P->dust->nb_comp : 0;
    S->vel_grad = LAYER(vel_grad);
    S->dgrain_conc = L->dust_conc ? L->dust_conc + (size_t)l * nc : NULL;
    S->temp_n = LAYER(temp_n);
    S->temp_el = LAYER(temp_el);
    S->mol_conc = LAYER(mol_conc);
    S->vel_width = O_SQRT(2. * BOLTZMANN_CONSTANT * S->temp_n / S->P->mol->mass + LAYER(vel_turb) * LAYER(vel_turb));
    set_gas_param(S, LAYER(temp_n), LAYER(temp_el), LAYER(he_conc), LAYER(ph2_conc), LAYER(oh2_conc),
                  LAYER(h_conc), LAYER(el_conc));
}

/* iteration_scheme_lvg::intensity_calc (iteration_lvg.cpp:163-185) */
static double intensity_single(const scheme_t *S, int up, int low, const double *level_pop)
{
    const lvg_molecule *M = S->P->mol;
    int N = S->N;
    double c, energy, dust_opacity, line_emiss, line_opacity, gamma, delta, ep1;
    energy = M->energy[up] - M->energy[low];
    c = S->mol_conc / (EIGHT_PI * S->vel_width * energy * energy * energy);
    line_emiss = c * M->einst[up * N + low] * level_pop[up];
    line_opacity = c * M->einst[low * N + up] * level_pop[low] - line_emiss + MIN_LINE_OPACITY;
    if (line_opacity < 0.) line_opacity *= INV_TRANS_FACTOR;      /* quirk q1, q2 */
    dust_opacity = oracle_dust_absorption(S->P->dust, energy, S->dgrain_conc);
    gamma = fabs(S->vel_grad) / (S->vel_width * line_opacity);
    delta = fabs(S->vel_grad) / (S->vel_width * dust_opacity);
    ep1 = oracle_esc_func(S->P->esc, gamma, delta);
    return line_emiss / line_opacity * ep1;
}

/* iteration_scheme_line_overlap::intensity_calc(u1,l1,u2,l2) (iteration_lvg.cpp:428-501) */
static void intensity_pair(const scheme_t *S, int u1, int l1, int u2, int l2, const double *level_pop,
                           double *intens1, double *intens2)
{
    const lvg_molecule *M = S->P->mol;
    const double *E = M->energy, *A = M->einst;
    const double max_dx = 4.;                      /* iteration_lvg.cpp:307 */
    int N = S->N;
    double c, energy, line_emiss1, line_opacity1, line_emiss2, line_opacity2, gamma1, gamma2, gratio, dx,
           ep1, ep2, ep01, ep02, dust_opacity, delta;

    energy = E[u1] - E[l1];
    c = S->mol_conc / (EIGHT_PI * S->vel_width * energy * energy * energy);
    line_emiss1 = c * A[u1 * N + l1] * level_pop[u1];
    line_opacity1 = c * (A[l1 * N + u1] * level_pop[l1] - A[u1 * N + l1] * level_pop[u1]) + MIN_LINE_OPACITY;
    line_emiss2 = c * A[u2 * N + l2] * level_pop[u2];
    line_opacity2 = c * (A[l2 * N + u2] * level_pop[l2] - A[u2 * N + l2] * level_pop[u2]) + MIN_LINE_OPACITY;
    if (line_opacity1 < 0.) line_opacity1 *= INV_TRANS_FACTOR;
    if (line_opacity2 < 0.) line_opacity2 *= INV_TRANS_FACTOR;
    gamma1 = fabs(S->vel_grad) / (S->vel_width * line_opacity1);
    gamma2 = fabs(S->vel_grad) / (S->vel_width * line_opacity2);
    dust_opacity = oracle_dust_absorption(S->P->dust, energy, S->dgrain_conc);
    delta = fabs(S->vel_grad) / (S->vel_width * dust_opacity);
    dx = (E[u1] - E[l1] - E[u2] + E[l2]) * SPEED_OF_LIGHT / (energy * S->vel_width);
    if (S->vel_grad < 0.) dx *= -1.;

    ep1 = ep2 = ep01 = ep02 = 0.;
    if (fabs(dx) < max_dx) {
        gratio = gamma2 / gamma1;
        ep1 = oracle_overlap_esc_func(S->P->overlap1, gamma1, delta, gratio, dx);
        gratio = gamma1 / gamma2;
        ep2 = oracle_overlap_esc_func(S->P->overlap1, gamma2, delta, gratio, -dx);
    }
    if (fabs(dx) > max_dx - 0.5) {
        ep01 = oracle_esc_func(S->P->esc, gamma1, delta);
        ep02 = oracle_esc_func(S->P->esc, gamma2, delta);
    }
    if (fabs(dx) > max_dx) {
        ep1 = ep01; ep2 = ep02;
    } else if (fabs(dx) > max_dx - 0.5) {
        c = 2. * (max_dx - fabs(dx));
        ep1 = ep01 * (1. - c) + ep1 * c;
        ep2 = ep02 * (1. - c) + ep2 * c;
    }
    *intens1 = line_emiss1 / line_opacity1 * ep1;
    *intens2 = line_emiss2 / line_opacity2 * ep2;
    if (fabs(dx) < max_dx) {
        gratio = gamma2 / gamma1;
        ep1 = oracle_overlap_esc_func(S->P->overlap2, gamma1, delta, gratio, dx);
        gratio = gamma1 / gamma2;
        ep2 = oracle_overlap_esc_func(S->P->overlap2, gamma2, delta, gratio, -dx);
        if (fabs(dx) > max_dx - 0.5) {
            c = 2. * (max_dx - fabs(dx));
            ep1 *= c; ep2 *= c;
        }
        *intens1 += line_emiss2 / line_opacity2 * ep1;
        *intens2 += line_emiss1 / line_opacity1 * ep2;
    }
}

/* iteration_scheme_lvg::operator() (iteration_lvg.cpp:112-161) and
 * iteration_scheme_line_overlap::operator() (iteration_lvg.cpp:348-426) */
static void scheme_assemble(scheme_t *S, const double *level_pop, double *df, int overlap)
{
    const lvg_molecule *M = S->P->mol;
    const double *A = M->einst;
    int N = S->N;
    double *m = S->matrix;
    double a, b, y, down_rate, up_rate, intensity;
    memset(m, 0, sizeof(double) * N * N);
    for (int i = 1; i < N; i++) {
        for (int j = 0; j < i; j++) {
            get_rate_neutrals(S, i, j, &down_rate, &up_rate);
            get_rate_electrons(S, i, j, &a, &b);
            down_rate += a;
            up_rate += b;
            m[i * N + i] -= down_rate;
            m[j * N + i] += down_rate;
            m[i * N + j] += up_rate;
            m[j * N + j] -= up_rate;
            if (!overlap && A[i * N + j] > 0.) {
                intensity = intensity_single(S, i, j, level_pop);
                y = A[i * N + j] * (1. + intensity);
                m[i * N + i] -= y;
                m[j * N + i] += y;
                y = A[j * N + i] * intensity;
                m[i * N + j] += y;
                m[j * N + j] -= y;
            }
        }
    }
    if (overlap) {
        for (int g = 0; g < S->nb_groups; g++) {
            const int *G = S->groups + 5 * g;
            int mu = G[1], l = G[2];
            double intens1, intens2;
            if (G[0] == 1) {
                intens1 = intensity_single(S, mu, l, level_pop);
                y = A[mu * N + l] * (1. + intens1);
                m[mu * N + mu] -= y; m[l * N + mu] += y;
                y = A[l * N + mu] * intens1;
                m[mu * N + l] += y; m[l * N + l] -= y;
            } else if (G[0] == 2) {
                int mm = G[3], ll = G[4];
                intensity_pair(S, mu, l, mm, ll, level_pop, &intens1, &intens2);
                y = A[mu * N + l] * (1. + intens1);
                m[mu * N + mu] -= y; m[l * N + mu] += y;
                y = A[l * N + mu] * intens1;
                m[mu * N + l] += y; m[l * N + l] -= y;
                y = A[mm * N + ll] * (1. + intens2);
                m[mm * N + mm] -= y; m[ll * N + mm] += y;
                y = A[ll * N + mm] * intens2;
                m[mm * N + ll] += y; m[ll * N + ll] -= y;
            }
        }
    }
    for (int j = 0; j < N; j++) m[j] = 1.;
    memset(df, 0, sizeof(double) * N);
    df[0] = 1.;
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++)
            df[i] -= m[i * N + j] * level_pop[j];
}

/* iteration_scheme_lvg::calc_new_pop (iteration_lvg.cpp:87-110) */
static void scheme_calc_new_pop(scheme_t *S, const double *old_pop, double *new_pop, double *eq_error,
                                double *f_vector, int overlap)
{
    int N = S->N;
    scheme_assemble(S, old_pop, f_vector, overlap);
    memset(new_pop, 0, sizeof(double) * N);
    new_pop[0] = 1.;
    oracle_lu_solve(S->matrix, new_pop, N);
    *eq_error = 0.;
    for (int i = 0; i < N; i++)
        if (*eq_error < fabs(f_vector[i])) *eq_error = fabs(f_vector[i]);
}

/* hfs_lines::sort / split (iteration_lvg.cpp:259-302), including the stale
 * running minimum of :276-280 (quirk q6). */
typedef struct { int nb; int upl[4], lowl[4]; double en[4]; } hfs_t;

static void hfs_swap(hfs_t *h, int i, int j)
{
    int t = h->upl[i]; h->upl[i] = h->upl[j]; h->upl[j] = t;
    t = h->lowl[i]; h->lowl[i] = h->lowl[j]; h->lowl[j] = t;
    double e = h->en[i]; h->en[i] = h->en[j]; h->en[j] = e;
}

static void hfs_sort(hfs_t *h)
{
    if (h->nb <= 2) return;
    int i, j;
    double e;
    for (i = 0; i < h->nb; i++)
        for (j = i + 1; j < h->nb; j++)
            if (h->en[j] < h->en[i]) hfs_swap(h, i, j);
    j = 0;
    e = h->en[1] - h->en[0];
    for (i = 1; i < h->nb - 1; i++)
        if (h->en[i + 1] - h->en[i] < e) j = i;
    e = h->en[j];
    for (i = 0; i < h->nb; i++)
        for (j = i + 1; j < h->nb; j++)
            if (fabs(h->en[j] - e) < fabs(h->en[i] - e)) hfs_swap(h, i, j);
}

/* iteration_scheme_line_overlap::init_molecule_data (iteration_lvg.cpp:317-346) */
int oracle_line_groups(const lvg_problem *P, int *groups, int max_groups)
{
    const lvg_molecule *M = P->mol;
    int N = M->nb_lev, ng = 0;
    if (N % 2) return -1;
    for (int i = 2; i < N; i += 2) {
        for (int j = 0; j < i; j += 2) {
            hfs_t h; h.nb = 0;
            for (int m = 0; m < 2; m++)
                for (int l = 0; l < 2; l++)
                    if (M->einst[(i + m) * N + j + l] > 1.e-99) {
                        h.upl[h.nb] = i + m; h.lowl[h.nb] = j + l;
                        h.en[h.nb] = M->energy[i + m] - M->energy[j + l];
                        h.nb++;
                    }
            hfs_sort(&h);
            int start = 0;
            if (h.nb >= 3) {       /* split(): the first two become their own group */
                if (ng >= max_groups) return -2;
                int *G = groups + 5 * ng++;
                G[0] = 2; G[1] = h.upl[0]; G[2] = h.lowl[0]; G[3] = h.upl[1]; G[4] = h.lowl[1];
                start = 2;
            }
            int rem = h.nb - start;
            if (rem > 0) {
                if (ng >= max_groups) return -2;
                int *G = groups + 5 * ng++;
                G[0] = rem; G[1] = h.upl[start]; G[2] = h.lowl[start];
                G[3] = rem > 1 ? h.upl[start + 1] : -1; G[4] = rem > 1 ? h.lowl[start + 1] : -1;
            }
        }
    }
    return ng;
}

/* ------------------------------------------------------------------------ */
/* boundary_layer_populations (iteration_control.cpp:52-91)                  */
/* ------------------------------------------------------------------------ */
static void boundary_layer_pops(scheme_t *S, double *arr)
{
    const lvg_molecule *M = S->P->mol;
    int N = S->N;
    double *m = S->matrix, down, up;
    memset(m, 0, sizeof(double) * N * N);
    memset(arr, 0, sizeof(double) * N);
    for (int i = 1; i < N; i++) {
        for (int j = 0; j < i; j++) {
            get_rate_neutrals(S, i, j, &down, &up);           /* no electrons: quirk q7 */
            m[j * N + i] = 0.5 * M->einst[i * N + j] + down;
            m[i * N + i] -= 0.5 * M->einst[i * N + j] + down;
            m[i * N + j] = up;
            m[j * N + j] -= up;
        }
    }
    for (int i = 0; i < N; i++) m[i] = 1.;
    arr[0] = 1.;
    oracle_lu_solve(m, arr, N);
}

/* ------------------------------------------------------------------------ */
/* iteration_control<T> (iteration_control.h:34-242)                         */
/* ------------------------------------------------------------------------ */
typedef struct {
    int N;
    int acceleration, nb_prev_steps, accel_start, accel_period, iter_nb, nb_after_accel, max_iter_nb;
    double best_eq_error, eq_error, pop_error, rel_error;
    double *opt_level_pop;
    double *prev[MAX_HIST]; int nprev;       /* prev_level_pop, front = [0] */
    double *res[MAX_HIST];  int nres;        /* residual_list, front = [0]  */
    double *pool[2 * MAX_HIST + 2]; int npool;
    double *pop_new, *f_vector;
} ictl_t;

static double *pool_get(ictl_t *C) { return C->pool[--C->npool]; }
static void pool_put(ictl_t *C, double *p) { C->pool[C->npool++] = p; }

static void list_push_front(double **lst, int *n, double *v)
{
    for (int i = *n; i > 0; i--) lst[i] = lst[i - 1];
    lst[0] = v; (*n)++;
}

/* iteration_control::accel_step (iteration_control.h:139-193) */
static void accel_step(ictl_t *C, double *accel_pop)
{
    int N = C->N, nb_param = C->nb_prev_steps - 1;
    double A[MAX_HIST * MAX_HIST], b[MAX_HIST], w, sum;
    memset(A, 0, sizeof A); memset(b, 0, sizeof b);
    const double *r0 = C->res[0], *p0 = C->prev[0];
    for (int i = 0; i < nb_param; i++) {
        const double *ri = C->res[i + 1];
        for (int j = 0; j < nb_param; j++) {
            const double *rj = C->res[j + 1];
            for (int k = 0; k < N; k++) {
                w = p0[k] + 1.e-99;
                A[i * nb_param + j] += (r0[k] - ri[k]) * (r0[k] - rj[k]) / (w * w);
            }
        }
        for (int k = 0; k < N; k++) {
            w = p0[k] + 1.e-99;
            b[i] += (r0[k] - ri[k]) * r0[k] / (w * w);
        }
    }
    oracle_lu_solve(A, b, nb_param);
    sum = 0.;
    for (int i = 0; i < nb_param; i++) sum += b[i];
    for (int k = 0; k < N; k++) {
        accel_pop[k] = (1. - sum) * p0[k];
        for (int i = 0; i < nb_param; i++) accel_pop[k] += b[i] * C->prev[i + 1][k];
    }
}

/* iteration_control::next_step (iteration_control.h:84-137) */
static void next_step(ictl_t *C, scheme_t *S, double *pop_old, int overlap)
{
    int N = C->N;
    double a;
    double *copy = pool_get(C);
    memcpy(copy, pop_old, sizeof(double) * N);
    list_push_front(C->prev, &C->nprev, copy);
    if (C->acceleration && (C->iter_nb == C->accel_start || C->nb_after_accel == C->accel_period)) {
        accel_step(C, pop_old);
        C->nb_after_accel = 0;
    }
    scheme_calc_new_pop(S, pop_old, C->pop_new, &C->eq_error, C->f_vector, overlap);
    if (C->acceleration && C->iter_nb >= C->accel_start) C->nb_after_accel++;
    if (C->eq_error < C->best_eq_error) {
        C->best_eq_error = C->eq_error;
        memcpy(C->opt_level_pop, pop_old, sizeof(double) * N);
    }
    double *residual = pool_get(C);
    C->pop_error = C->rel_error = 0.;
    for (int i = 0; i < N; i++) {
        residual[i] = C->pop_new[i] - pop_old[i];
        if ((a = fabs(residual[i])) > C->pop_error) C->pop_error = a;
        if ((a = fabs(residual[i] / (pop_old[i] + 1.e-99))) > C->rel_error) C->rel_error = a;
    }
    list_push_front(C->res, &C->nres, residual);
    if (C->nres > C->nb_prev_steps + 1) pool_put(C, C->res[--C->nres]);
    if (C->nprev > C->nb_prev_steps + 1) pool_put(C, C->prev[--C->nprev]);
    if (C->iter_nb < C->max_iter_nb - 1) {
        memcpy(pop_old, C->pop_new, sizeof(double) * N);
    } else {
        memcpy(pop_old, C->opt_level_pop, sizeof(double) * N);   /* quirk q3 */
        C->eq_error = C->best_eq_error;
    }
    C->iter_nb++;
}

static int ictl_init(ictl_t *C, int N, int nb_prev)
{
    memset(C, 0, sizeof *C);
    C->N = N;
    C->nb_prev_steps = nb_prev;
    C->npool = 2 * (nb_prev + 2) + 2;
    if (C->npool > 2 * MAX_HIST + 2) return -1;
    for (int i = 0; i < C->npool; i++) C->pool[i] = (double *)malloc(sizeof(double) * N);
    C->opt_level_pop = (double *)malloc(sizeof(double) * N);
    C->pop_new = (double *)malloc(sizeof(double) * N);
    C->f_vector = (double *)malloc(sizeof(double) * N);
    return 0;
}

static void ictl_free(ictl_t *C)
{
    for (int i = 0; i < C->nprev; i++) pool_put(C, C->prev[i]);
    for (int i = 0; i < C->nres; i++) pool_put(C, C->res[i]);
    for (int i = 0; i < C->npool; i++) free(C->pool[i]);
    free(C->opt_level_pop); free(C->pop_new); free(C->f_vector);
}

/* iteration_control::calculate_populations (iteration_control.h:196-242) */
static int calculate_populations(ictl_t *C, scheme_t *S, const lvg_solve_opts *o, double *pop_arr,
                                 int max_nb, int accel, int overlap)
{
    int is_found;
    C->acceleration = accel;
    C->accel_start = o->accel_start;
    C->accel_period = o->accel_period;
    C->max_iter_nb = max_nb;
    C->iter_nb = C->nb_after_accel = 0;
    C->best_eq_error = 1.;
    C->eq_error = C->pop_error = C->rel_error = 0.;
    memset(C->opt_level_pop, 0, sizeof(double) * C->N);
    for (int i = 0; i < C->nprev; i++) pool_put(C, C->prev[i]);
    for (int i = 0; i < C->nres; i++) pool_put(C, C->res[i]);
    C->nprev = C->nres = 0;
    do {
        next_step(C, S, pop_arr, overlap);
        is_found = (C->rel_error < o->min_error);
    } while (C->iter_nb < C->max_iter_nb && !is_found);
    return is_found;
}

/* ------------------------------------------------------------------------ */
/* public entry points                                                       */
/* ------------------------------------------------------------------------ */

static int scheme_init(scheme_t *S, const lvg_problem *P, int overlap)
{
    memset(S, 0, sizeof *S);
    S->P = P;
    S->N = P->mol->nb_lev;
    S->matrix = (double *)malloc(sizeof(double) * S->N * S->N);
    if (overlap) {
        int maxg = S->N * S->N;
        S->groups = (int *)malloc(sizeof(int) * 5 * maxg);
        S->nb_groups = oracle_line_groups(P, S->groups, maxg);
        if (S->nb_groups < 0) return -1;
    }
    return 0;
}

static void scheme_free(scheme_t *S) { free(S->matrix); free(S->groups); }

void oracle_opts_default(lvg_solve_opts *o)
{
    o->min_error = 1.e-5;
    o->max_iter_acc = 150;
    o->max_iter_plain = 15000;
    o->accel_start = 40;
    o->accel_period = 5;
    o->accel_nb = 5;
    o->acceleration = 1;
    o->allow_plain_retry = 1;
    o->init = LVG_INIT_BOUNDARY_LAYER;
    o->line_overlap = 0;
}

/* One layer of calc_molecular_populations (radiative_transfer.cpp:236-288). */
static void solve_one_layer(scheme_t *S, ictl_t *C, const lvg_layers *L, int l, double *pops,
                            const double *given, int prev_found, const lvg_solve_opts *o,
                            lvg_layer_status *st)
{
    int N = S->N;
    double *pop = pops + (size_t)l * N;
    scheme_set_layer(S, L, l);
    int accel = o->acceleration;
    int max_it = accel ? o->max_iter_acc : o->max_iter_plain;
#define INIT_GUESS()                                                                  \
    do {                                                                              \
        if (o->init == LVG_INIT_GIVEN) memcpy(pop, given, sizeof(double) * N);        \
        else if (o->init == LVG_INIT_WARM_CHAIN && l > 0 && prev_found)               \
            memcpy(pop, pops + (size_t)(l - 1) * N, sizeof(double) * N);              \
        else boundary_layer_pops(S, pop);                                             \
    } while (0)
    INIT_GUESS();
    int found = calculate_populations(C, S, o, pop, max_it, accel, o->line_overlap);
    int iters = C->iter_nb, retry = 0;
    if (!found && accel && o->allow_plain_retry) {
        INIT_GUESS();
        found = calculate_populations(C, S, o, pop, o->max_iter_plain, 0, o->line_overlap);
        iters += C->iter_nb;
        retry = 1;
    }
#undef INIT_GUESS
    if (st) {
        st->converged = found;
        st->iterations = iters;
        st->used_plain_retry = retry;
        st->reserved = 0;
        st->eq_error = C->eq_error;
        st->rel_error = C->rel_error;
        st->pop_error = C->pop_error;
    }
}

int oracle_solve_layers(const lvg_problem *P, const lvg_layers *L, double *pops,
                        const lvg_solve_opts *o, lvg_layer_status *status, int nthreads)
{
    int N = P->mol->nb_lev, nl = L->nb_lay;
    if (o->line_overlap && (!P->overlap1 || !P->overlap2)) return LVG_E_ARG;
    if (o->accel_nb < 2 || o->accel_nb + 2 > MAX_HIST || (o->acceleration && o->accel_start < o->accel_nb))
        return LVG_E_ARG;
    double *given = NULL;
    if (o->init == LVG_INIT_GIVEN) {
        given = (double *)malloc(sizeof(double) * (size_t)nl * N);
        memcpy(given, pops, sizeof(double) * (size_t)nl * N);
    }
    int err = 0;
    if (o->init == LVG_INIT_WARM_CHAIN) {
        scheme_t S; ictl_t C;
        if (scheme_init(&S, P, o->line_overlap) || ictl_init(&C, N, o->accel_nb)) return LVG_E_ARG;
        int prev_found = 0;
        for (int l = 0; l < nl; l++) {
            lvg_layer_status st;
            solve_one_layer(&S, &C, L, l, pops, NULL, prev_found, o, &st);
            prev_found = st.converged;
            if (status) status[l] = st;
        }
        ictl_free(&C); scheme_free(&S);
    } else {
#ifdef _OPENMP
        if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : err)
#endif
        {
            scheme_t S; ictl_t C;
            if (scheme_init(&S, P, o->line_overlap) || ictl_init(&C, N, o->accel_nb)) err = 1;
            else {
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
                for (int l = 0; l < nl; l++)
                    solve_one_layer(&S, &C, L, l, pops, given ? given + (size_t)l * N : NULL, 0, o,
                                    status ? status + l : NULL);
                ictl_free(&C);
            }
            scheme_free(&S);
        }
    }
    free(given);
    return err ? LVG_E_ARG : LVG_OK;
}

/* Independent clouds, each a warm chain (radiative_transfer.cpp:219-289 with the
 * default start rule :247-252): chain c is layers [chain_off[c], chain_off[c+1]),
 * solved in order; chains run in parallel, one per OpenMP thread, as the reference
 * runs one shock model per thread (radiative_transfer.cpp:152-216). */
int oracle_solve_chains(const lvg_problem *P, const lvg_layers *L, int nb_chain, const int *chain_off,
                        double *pops, const lvg_solve_opts *o, lvg_layer_status *status, int nthreads)
{
    int N = P->mol->nb_lev;
    if (o->init != LVG_INIT_WARM_CHAIN || nb_chain < 1 || chain_off[0] != 0 || chain_off[nb_chain] != L->nb_lay)
        return LVG_E_ARG;
    if (o->line_overlap && (!P->overlap1 || !P->overlap2)) return LVG_E_ARG;
    if (o->accel_nb < 2 || o->accel_nb + 2 > MAX_HIST || (o->acceleration && o->accel_start < o->accel_nb))
        return LVG_E_ARG;
    int err = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : err)
#endif
    {
        scheme_t S; ictl_t C;
        if (scheme_init(&S, P, o->line_overlap) || ictl_init(&C, N, o->accel_nb)) err = 1;
        else {
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
            for (int c = 0; c < nb_chain; c++) {
                int prev_found = 0;
                for (int l = chain_off[c]; l < chain_off[c + 1]; l++) {
                    lvg_layer_status st;
                    solve_one_layer(&S, &C, L, l, pops, NULL, l > chain_off[c] && prev_found, o, &st);
                    prev_found = st.converged;
                    if (status) status[l] = st;
                }
            }
            ictl_free(&C);
        }
        scheme_free(&S);
    }
    (void)N;
    return err ? LVG_E_ARG : LVG_OK;
}

int oracle_calc_new_pop(const lvg_problem *P, const lvg_layers *L, int layer, const double *pop_in,
                        int overlap, double *matrix_out, double *df_out, double *pop_out, double *eq_error)
{
    scheme_t S;
    int N = P->mol->nb_lev;
    if (scheme_init(&S, P, overlap)) return LVG_E_ARG;
    scheme_set_layer(&S, L, layer);
    double *f = (double *)malloc(sizeof(double) * N);
    scheme_assemble(&S, pop_in, f, overlap);
    if (matrix_out) memcpy(matrix_out, S.matrix, sizeof(double) * N * N);
    if (df_out) memcpy(df_out, f, sizeof(double) * N);
    double e = 0.;
    for (int i = 0; i < N; i++) if (e < fabs(f[i])) e = fabs(f[i]);
    memset(pop_out, 0, sizeof(double) * N);
    pop_out[0] = 1.;
    oracle_lu_solve(S.matrix, pop_out, N);
    if (eq_error) *eq_error = e;
    free(f);
    scheme_free(&S);
    return LVG_OK;
}

int oracle_boundary_layer_populations(const lvg_problem *P, const lvg_layers *L, double *pops_out)
{
    int N = P->mol->nb_lev;
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        scheme_t S;
        scheme_init(&S, P, 0);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int l = 0; l < L->nb_lay; l++) {
            scheme_set_layer(&S, L, l);
            boundary_layer_pops(&S, pops_out + (size_t)l * N);
        }
        scheme_free(&S);
    }
    return LVG_OK;
}

int oracle_coll_rates(const lvg_problem *P, const lvg_layers *L, int layer, double *down_n, double *up_n,
                      double *down_e, double *up_e)
{
    scheme_t S;
    int N = P->mol->nb_lev;
    if (scheme_init(&S, P, 0)) return LVG_E_ARG;
    scheme_set_layer(&S, L, layer);
    for (int i = 1; i < N; i++)
        for (int j = 0; j < i; j++) {
            get_rate_neutrals(&S, i, j, down_n + i * N + j, up_n + i * N + j);
            get_rate_electrons(&S, i, j, down_e + i * N + j, up_e + i * N + j);
        }
    scheme_free(&S);
    return LVG_OK;
}

/* get_nb_overlap_lines (iteration_lvg.cpp:528-583) */
int oracle_nb_overlap_lines(const lvg_problem *P, double vel_width, int *nb_double, int *nb_triple)
{
    const lvg_molecule *M = P->mol;
    const double dx_lim = 4.;
    const double *E = M->energy;
    int N = M->nb_lev;
    *nb_double = *nb_triple = 0;
    for (int i = 2; i < N; i += 2) {
        for (int j = 0; j < i; j += 2) {
            hfs_t h; h.nb = 0;
            for (int m = 0; m < 2; m++)
                for (int l = 0; l < 2; l++)
                    if (M->einst[(i + m) * N + j + l] > 1.e-99) {
                        h.upl[h.nb] = i + m; h.lowl[h.nb] = j + l;
                        h.en[h.nb] = E[i + m] - E[j + l]; h.nb++;
                    }
            hfs_sort(&h);
            double en = E[i] - E[j], dx;
            if (h.nb > 1) {
                dx = (E[h.upl[0]] - E[h.lowl[0]] - E[h.upl[1]] + E[h.lowl[1]]) * SPEED_OF_LIGHT / (en * vel_width);
                if (fabs(dx) < dx_lim) (*nb_double)++;
            }
            if (h.nb > 2) {
                dx = (E[h.upl[1]] - E[h.lowl[1]] - E[h.upl[2]] + E[h.lowl[2]]) * SPEED_OF_LIGHT / (en * vel_width);
                if (fabs(dx) < dx_lim) (*nb_triple)++;
            }
            if (h.nb == 4) {
                /* split() removes the first two lines */
                dx = (E[h.upl[2]] - E[h.lowl[2]] - E[h.upl[3]] + E[h.lowl[3]]) * SPEED_OF_LIGHT / (en * vel_width);
                if (fabs(dx) < dx_lim) (*nb_double)++;
            }
        }
    }
    return LVG_OK;
}

/* probes of the shared elementary functions (tests compare them with libm) */
/* ------------------------------------------------------------------------ */
/* transition_data_container (transition_data.cpp:181-417): post-processing   */
/* ------------------------------------------------------------------------ */
#define ONEDIVBY_SQRT_PI 0.56418958354775628  /* constants.h (absent): 1/sqrt(pi) */

void oracle_find_opts_default(lvg_find_opts *o)
{
    o->rel_error = 1.e-5;
    o->min_optical_depth = 0.01;      /* transition_data.cpp:182 */
    o->velocity_shift = 5.e+5;        /* :190 */
    o->delta_aspect_ratio = 0.25;     /* :18 */
    o->h2o22_up = o->h2o22_low = -1;
}

typedef struct {
    int up, low;
    double energy, inv, gain, tau_eff, tau_max;
    int lay_nb_hg;
    double *inv_arr, *gain_arr, *exc_temp_arr, tau_asp[LVG_NB_ASPECT], tau_freq[LVG_NB_FREQ];
} otrans_t;

/* calc_inv (:210-223) */
static void o_calc_inv(otrans_t *t, const lvg_problem *P, const lvg_cloud_geometry *G, int nlay, const double *pop)
{
    const int N = P->mol->nb_lev;
    t->inv = 0.;
    for (int lay = 0; lay < nlay; lay++) {
        double low_pop = pop[lay * N + t->low], up_pop = pop[lay * N + t->up];
        t->inv_arr[lay] = up_pop / P->mol->g[t->up] - low_pop / P->mol->g[t->low];
        t->inv += t->inv_arr[lay] * G->dz[lay];
    }
    t->inv /= G->height;
}

/* calc_exc_temp (:225-238), log from lvg_math.h */
static void o_calc_exc_temp(otrans_t *t, const lvg_problem *P, int nlay, const double *pop)
{
    const int N = P->mol->nb_lev;
    for (int lay = 0; lay < nlay; lay++) {
        double low_pop = pop[lay * N + t->low], up_pop = pop[lay * N + t->up];
        t->exc_temp_arr[lay] = CM_INVERSE_TO_KELVINS * t->energy
            / O_LOG((low_pop * P->mol->g[t->up]) / (up_pop * P->mol->g[t->low]));
    }
}

/* calc_gain (:240-294); pow(x, 0.5) -> sqrt, pow(x, 2.) -> x*x (DESIGN.md "Parity") */
static void o_calc_gain(otrans_t *t, const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G,
                        const lvg_find_opts *o)
{
    const int N = P->mol->nb_lev, nlay = L->nb_lay, nc = P->dust ? P->dust->nb_comp : 0;
    const int h2o22 = (t->up == o->h2o22_up && t->low == o->h2o22_low);
    const double energy = t->energy, energy_th = energy * energy * energy;
    const double aul = P->mol->einst[t->up * N + t->low];
    for (int lay = 0; lay < nlay; lay++) {
        double vel, vt = L->vel_turb[lay];
        if (h2o22) {
            double a = O_SQRT(2. * BOLTZMANN_CONSTANT * L->temp_n[lay] / P->mol->mass) + 5.e+4;
            vel = O_SQRT(a * a + vt * vt);
        } else {
            vel = O_SQRT(2. * BOLTZMANN_CONSTANT * L->temp_n[lay] / P->mol->mass + vt * vt);
        }
        double line_gain = t->inv_arr[lay] * P->mol->g[t->up] * aul * ONEDIVBY_SQRT_PI * L->mol_conc[lay]
            / (energy_th * EIGHT_PI * vel);
        double d_abs = nc ? oracle_dust_absorption(P->dust, energy, L->dust_conc + (size_t)lay * nc) : 0.;
        t->gain_arr[lay] = line_gain - d_abs;
    }
    double g = 0.;
    t->gain = t->tau_eff = 0.;
    t->lay_nb_hg = 0;
    for (int lay = 0; lay < nlay; lay++) {
        t->gain += t->gain_arr[lay] * G->dz[lay];
        if (t->gain_arr[lay] > 0.) t->tau_eff += t->gain_arr[lay] * G->dz[lay];
        if (t->gain_arr[lay] > g) { g = t->gain_arr[lay]; t->lay_nb_hg = lay; }
    }
    t->gain /= G->height;
    if (g < 1.e-99) t->lay_nb_hg = 0;
}

/* calc_line_profile (:296-378), exp from lvg_math.h */
static void o_calc_line_profile(otrans_t *t, const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G,
                                const lvg_find_opts *o)
{
    const int N = P->mol->nb_lev, nlay = L->nb_lay, nc = P->dust ? P->dust->nb_comp : 0;
    const double energy = t->energy, energy_th = energy * energy * energy;
    const double aul = P->mol->einst[t->up * N + t->low];
    const double vmax = G->vel_n[0] + o->velocity_shift, vmin = G->vel_n[nlay - 1] - o->velocity_shift;
    const double dv = (vmax - vmin) / (LVG_NB_FREQ - 1.);
    double *lo = (double *)malloc(sizeof(double) * nlay * 3), *vw = lo + nlay, *dop = vw + nlay;
    double *od = (double *)malloc(sizeof(double) * LVG_NB_FREQ * LVG_NB_ASPECT);
    for (int lay = 0; lay < nlay; lay++) {
        double vt = L->vel_turb[lay];
        vw[lay] = O_SQRT(2. * BOLTZMANN_CONSTANT * L->temp_n[lay] / P->mol->mass + vt * vt);
        lo[lay] = t->inv_arr[lay] * P->mol->g[t->up] * aul * L->mol_conc[lay] * ONEDIVBY_SQRT_PI
            / (energy_th * EIGHT_PI * vw[lay]);
        dop[lay] = nc ? oracle_dust_absorption(P->dust, energy, L->dust_conc + (size_t)lay * nc) : 0.;
    }
    for (int i = 0; i < LVG_NB_ASPECT; i++) {
        double aspect_ratio = 1. + o->delta_aspect_ratio * i;
        double vel = vmin;
        for (int n = 0; n < LVG_NB_FREQ; vel += dv, n++) {
            double acc = 0.;
            for (int lay = 0; lay < nlay; lay++) {
                double x = (vel - G->vel_n[lay] / aspect_ratio) / vw[lay];
                double profile = O_EXP(-x * x);
                if (lo[lay] * profile - dop[lay] > 0.)
                    acc += (lo[lay] * profile - dop[lay]) * G->dz[lay] * aspect_ratio;
            }
            od[n * LVG_NB_ASPECT + i] = acc;
        }
    }
    for (int i = 0; i < LVG_NB_ASPECT; i++) {
        double x = 0.;
        for (int n = 0; n < LVG_NB_FREQ; n++)
            if (x < od[n * LVG_NB_ASPECT + i]) x = od[n * LVG_NB_ASPECT + i];
        t->tau_asp[i] = x;
    }
    t->tau_max = t->tau_asp[0];
    for (int n = 0; n < LVG_NB_FREQ; n++) t->tau_freq[n] = od[n * LVG_NB_ASPECT];
    free(od);
    free(lo);
}

/* find (:380-417). Output in the reference's list order (push_front). */
int oracle_find_transitions(const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G,
                            const double *pops, const lvg_find_opts *o, int max_out, int *nb_out,
                            lvg_transition *out, double *inv_arr, double *gain_arr, double *exc_temp_arr)
{
    const int N = P->mol->nb_lev, nlay = L->nb_lay;
    if (nlay < 1) { *nb_out = 0; return 0; }
    int cap = 16, nf = 0;
    otrans_t *found = (otrans_t *)malloc(sizeof(otrans_t) * cap);
    otrans_t t;
    t.inv_arr = (double *)malloc(sizeof(double) * nlay * 3);
    t.gain_arr = t.inv_arr + nlay;
    t.exc_temp_arr = t.gain_arr + nlay;
    for (int i = 1; i < N; i++)
        for (int j = 0; j < i; j++) {
            if (P->mol->einst[i * N + j] == 0.) continue;
            t.up = i; t.low = j;
            t.energy = P->mol->energy[i] - P->mol->energy[j];
            o_calc_inv(&t, P, G, nlay, pops);
            int inverted = 0;
            for (int lay = 0; lay < nlay; lay++) {
                inverted = (t.inv_arr[lay] * P->mol->g[i] > o->rel_error * pops[i]);   /* level_pop[i]: layer 0 (:398) */
                if (inverted) break;
            }
            if (!inverted) continue;
            o_calc_gain(&t, P, L, G, o);
            o_calc_line_profile(&t, P, L, G, o);
            if (t.tau_max >= o->min_optical_depth) {
                o_calc_exc_temp(&t, P, nlay, pops);
                if (nf == cap) { cap *= 2; found = (otrans_t *)realloc(found, sizeof(otrans_t) * cap); }
                found[nf] = t;
                found[nf].inv_arr = (double *)malloc(sizeof(double) * nlay * 3);
                memcpy(found[nf].inv_arr, t.inv_arr, sizeof(double) * nlay * 3);
                found[nf].gain_arr = found[nf].inv_arr + nlay;
                found[nf].exc_temp_arr = found[nf].gain_arr + nlay;
                nf++;
            }
        }
    *nb_out = nf;
    for (int k = 0; k < nf && k < max_out; k++) {
        const otrans_t *f = &found[nf - 1 - k];
        lvg_transition *r = &out[k];
        r->up = f->up; r->low = f->low; r->lay_nb_hg = f->lay_nb_hg; r->reserved = 0;
        r->energy = f->energy; r->inv = f->inv; r->gain = f->gain; r->tau_eff = f->tau_eff; r->tau_max = f->tau_max;
        memcpy(r->tau_vs_aspect_ratio, f->tau_asp, sizeof f->tau_asp);
        memcpy(r->tau_vs_frequency, f->tau_freq, sizeof f->tau_freq);
        if (inv_arr) memcpy(inv_arr + (size_t)k * nlay, f->inv_arr, sizeof(double) * nlay);
        if (gain_arr) memcpy(gain_arr + (size_t)k * nlay, f->gain_arr, sizeof(double) * nlay);
        if (exc_temp_arr) memcpy(exc_temp_arr + (size_t)k * nlay, f->exc_temp_arr, sizeof(double) * nlay);
    }
    for (int k = 0; k < nf; k++) free(found[k].inv_arr);
    free(found);
    free(t.inv_arr);
    return 0;
}

/* lim_luminosity_lvg (maser_luminosity.cpp:7-106). intensity_calc gets the FIRST
 * layer's populations (level_pop, :54, :58) unless layer_pops != 0. */
int oracle_lim_luminosity(const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G, const double *pops,
                          int nb_trans, const int *up, const int *low, int layer_pops, double *lum, double *lum_arr,
                          double *emiss_coeff_arr, double *pump_rate_arr, double *pump_eff_arr, double *loss_rate_arr)
{
    const int N = P->mol->nb_lev, nlay = L->nb_lay;
    const double *A = P->mol->einst;
    const int *g = P->mol->g;
    scheme_t S;
    if (scheme_init(&S, P, 0)) return -1;
    double *up_loss = (double *)calloc((size_t)nlay * 2, sizeof(double)), *low_loss = up_loss + nlay;
    for (int t = 0; t < nb_trans; t++) {
        const int lo = low[t], hi = up[t];
        double lsum = 0.;
        for (int lay = 0; lay < nlay; lay++) {
            const int shift = N * lay;
            const double *ipop = layer_pops ? pops + shift : pops;
            scheme_set_layer(&S, L, lay);
            for (int k = 0; k <= 1; k++) {
                const int j = k == 0 ? lo : hi;
                double loss_rate = 0.;
                for (int i = 0; i < N; i++) {
                    if (A[i * N + j] != 0 && i != lo && i != hi) {
                        if (i < j && pops[shift + i] * A[i * N + j] > pops[shift + j] * A[j * N + i]) {
                            double intensity = intensity_single(&S, j, i, ipop);
                            loss_rate += A[j * N + i] * (1. + intensity);
                        } else if (i > j && pops[shift + i] * A[i * N + j] < pops[shift + j] * A[j * N + i]) {
                            double intensity = intensity_single(&S, i, j, ipop);
                            loss_rate += A[j * N + i] * intensity;
                        }
                    }
                }
                if (k == 0) low_loss[lay] = loss_rate; else up_loss[lay] = loss_rate;
            }
            /* collisional_transitions::get_rate_neutrals(init, fin) (coll_rates.cpp:225-240) */
            for (int i = 0; i < N; i++) {
                double d, u;
                if (i != lo) {
                    if (lo > i) { get_rate_neutrals(&S, lo, i, &d, &u); low_loss[lay] += d; }
                    else        { get_rate_neutrals(&S, i, lo, &d, &u); low_loss[lay] += u; }
                }
                if (i != hi) {
                    if (hi > i) { get_rate_neutrals(&S, hi, i, &d, &u); up_loss[lay] += d; }
                    else        { get_rate_neutrals(&S, i, hi, &d, &u); up_loss[lay] += u; }
                }
            }
            const size_t o = (size_t)t * nlay + lay;
            const double ph2 = L->ph2_conc[lay], oh2 = L->oh2_conc[lay], mol = L->mol_conc[lay];
            if (emiss_coeff_arr) emiss_coeff_arr[o] = (ph2 + oh2) * mol / L->vel_grad[lay];
            const double inversion = pops[shift + hi] / g[hi] - pops[shift + lo] / g[lo];
            double la, pe;
            if (inversion > 0.) {
                la = inversion / (1. / (up_loss[lay] * g[hi]) + 1. / (low_loss[lay] * g[lo])) * mol;
                pe = inversion / (pops[shift + hi] / g[hi] + pops[shift + lo] / g[lo]);
            } else {
                la = pe = 1.e-99;
            }
            if (lum_arr) lum_arr[o] = la;
            if (pump_eff_arr) pump_eff_arr[o] = pe;
            lsum += la * G->dz[lay];
            if (loss_rate_arr) loss_rate_arr[o] = (up_loss[lay] * g[hi] + low_loss[lay] * g[lo]) / ((double)g[hi] + g[lo]);
            if (pump_rate_arr)
                pump_rate_arr[o] = 0.5 * (pops[shift + hi] * up_loss[lay] + pops[shift + lo] * low_loss[lay]) / (ph2 + oh2);
        }
        if (lum) lum[t] = lsum / G->height;
    }
    free(up_loss);
    scheme_free(&S);
    return 0;
}

double oracle_exp(double x) { return lvg_exp(x); }
double oracle_log10(double x) { return lvg_log10(x); }
