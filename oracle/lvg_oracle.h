/*
 * lvg_oracle.h — CPU oracle (TEST INFRASTRUCTURE ONLY; parity unpinned, see
 * lvg_oracle.c). Consumes the same description structs as the product ABI
 * (include/lvg_amd.h) so tests can run both on identical inputs.
 */
#ifndef LVG_ORACLE_H
#define LVG_ORACLE_H
#include "../include/lvg_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
void   oracle_opts_default(lvg_solve_opts *o);
int    oracle_solve_layers(const lvg_problem *P, const lvg_layers *L, double *pops,
                           const lvg_solve_opts *o, lvg_layer_status *status, int nthreads);
int    oracle_solve_chains(const lvg_problem *P, const lvg_layers *L, int nb_chain, const int *chain_off,
                           double *pops, const lvg_solve_opts *o, lvg_layer_status *status, int nthreads);
int    oracle_calc_new_pop(const lvg_problem *P, const lvg_layers *L, int layer, const double *pop_in,
                           int overlap, double *matrix_out, double *df_out, double *pop_out,
                           double *eq_error);
int    oracle_boundary_layer_populations(const lvg_problem *P, const lvg_layers *L, double *pops_out);
int    oracle_coll_rates(const lvg_problem *P, const lvg_layers *L, int layer, double *down_n,
                         double *up_n, double *down_e, double *up_e);
int    oracle_line_groups(const lvg_problem *P, int *groups, int max_groups);
int    oracle_nb_overlap_lines(const lvg_problem *P, double vel_width, int *nb_double, int *nb_triple);
double oracle_esc_func(const lvg_esc_table *T, double gamma, double delta);
double oracle_overlap_esc_func(const lvg_overlap_table *T, double gamma, double delta,
                               double gamma_ratio, double delta_x);
double oracle_dust_absorption(const lvg_dust *d, double energy, const double *conc);
int    oracle_lu_solve(double *a, double *b, int n);
void   oracle_find_opts_default(lvg_find_opts *o);
int    oracle_find_transitions(const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G,
                               const double *pops, const lvg_find_opts *o, int max_out, int *nb_out,
                               lvg_transition *out, double *inv_arr, double *gain_arr, double *exc_temp_arr);
int    oracle_lim_luminosity(const lvg_problem *P, const lvg_layers *L, const lvg_cloud_geometry *G, const double *pops,
                             int nb_trans, const int *up, const int *low, int layer_pops, double *lum, double *lum_arr,
                             double *emiss_coeff_arr, double *pump_rate_arr, double *pump_eff_arr, double *loss_rate_arr);
double oracle_exp(double x);
double oracle_log10(double x);
#ifdef __cplusplus
}
#endif
#endif
