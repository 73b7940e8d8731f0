/* Sanitizer driver of the CPU oracle (test infrastructure; tests/test_sanitizers_cpu.py).
 * Built together with oracle/lvg_oracle.c under -fsanitize=address,undefined. Reads a
 * problem + layers dump (manifest.txt + <name>.bin, written by the test from synth_v1),
 * runs every oracle entry point, writes the results as raw binaries into <out>, and
 * exits 0; any sanitizer report aborts with a non-zero status.
 *   oracle_driver <in_dir> <out_dir> */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/lvg_oracle.h"

typedef struct { char name[80]; char dt[8]; long n; void *data; } arr_t;
static arr_t A[1024];
static int nA;

static void load(const char *dir) {
    char p[4096];
    snprintf(p, sizeof p, "%s/manifest.txt", dir);
    FILE *m = fopen(p, "r");
    if (!m) { fprintf(stderr, "no manifest in %s\n", dir); exit(2); }
    while (nA < 1024 && fscanf(m, "%79s %7s %ld", A[nA].name, A[nA].dt, &A[nA].n) == 3) {
        size_t es = strcmp(A[nA].dt, "f8") == 0 ? 8 : 4;
        A[nA].data = malloc(es * (size_t)(A[nA].n > 0 ? A[nA].n : 1));
        snprintf(p, sizeof p, "%s/%s.bin", dir, A[nA].name);
        FILE *f = fopen(p, "rb");
        if (!f || fread(A[nA].data, es, (size_t)A[nA].n, f) != (size_t)A[nA].n) { fprintf(stderr, "bad %s\n", p); exit(2); }
        fclose(f);
        nA++;
    }
    fclose(m);
}

static arr_t *find(const char *name) {
    for (int i = 0; i < nA; i++)
        if (strcmp(A[i].name, name) == 0) return &A[i];
    return NULL;
}
static const double *D(const char *name) { arr_t *a = find(name); return a ? (const double *)a->data : NULL; }
static const int *I(const char *name) { arr_t *a = find(name); return a ? (const int *)a->data : NULL; }
static long len(const char *name) { arr_t *a = find(name); return a ? a->n : 0; }

static void dump(const char *dir, const char *name, const void *p, size_t bytes) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s.bin", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(p, 1, bytes, f) != bytes) { fprintf(stderr, "cannot write %s\n", path); exit(2); }
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    load(argv[1]);
    const char *out = argv[2];
    char k[128];
    /* molecule */
    lvg_molecule mol = {(int)len("mol_energy"), D("mol_mass")[0], D("mol_energy"), I("mol_g"), I("mol_v"), D("mol_j"),
                        D("mol_einst")};
    const int N = mol.nb_lev;
    /* collisions */
    const int *cm = I("coll_meta");
    const int nt = cm[1] + cm[2];
    lvg_coll_table *tabs = calloc((size_t)nt, sizeof *tabs);
    for (int t = 0; t < nt; t++) {
        snprintf(k, sizeof k, "coll_t%d_meta", t);
        const int *tm = I(k);
        tabs[t].nb_lev = tm[0]; tabs[t].jmax = tm[1]; tabs[t].species = tm[2];
        snprintf(k, sizeof k, "coll_t%d_tgrid", t);
        tabs[t].tgrid = D(k);
        snprintf(k, sizeof k, "coll_t%d_coeff", t);
        tabs[t].coeff = D(k);
    }
    lvg_collisions coll = {cm[0], cm[1], cm[2], tabs};
    /* dust */
    const int nc = I("dust_meta")[0];
    lvg_dust_component *comp = calloc((size_t)(nc > 0 ? nc : 1), sizeof *comp);
    for (int c = 0; c < nc; c++) {
        snprintf(k, sizeof k, "dust_c%d_energy", c);
        comp[c].nb_en = (int)len(k);
        comp[c].energy = D(k);
        snprintf(k, sizeof k, "dust_c%d_abs", c);
        comp[c].abs_coeff = D(k);
        snprintf(k, sizeof k, "dust_c%d_wvl_exp", c);
        comp[c].wvl_exp = D(k)[0];
    }
    lvg_dust dust = {nc, comp};
    lvg_esc_table esc = {(int)len("esc_delta"), (int)len("esc_gamma"), D("esc_delta"), D("esc_gamma"), D("esc_p")};
    lvg_overlap_table ov[2];
    const int has_ov = find("ov1_p") != NULL;
    for (int q = 0; q < 2 && has_ov; q++) {
        char b[5][32];
        const char *f[5] = {"ld", "dx", "gr", "g", "p"};
        for (int i = 0; i < 5; i++) snprintf(b[i], sizeof b[i], "ov%d_%s", q + 1, f[i]);
        ov[q].nb_d = (int)len(b[0]); ov[q].nb_dx = (int)len(b[1]); ov[q].nb_gr = (int)len(b[2]); ov[q].nb_g = (int)len(b[3]);
        ov[q].log10_delta = D(b[0]); ov[q].dx = D(b[1]); ov[q].gratio = D(b[2]); ov[q].gamma = D(b[3]); ov[q].p = D(b[4]);
    }
    lvg_problem P = {&mol, &coll, &dust, &esc, has_ov ? &ov[0] : NULL, has_ov ? &ov[1] : NULL};
    /* layers */
    const int nl = (int)len("lay_temp_n");
    lvg_layers L = {nl, D("lay_temp_n"), D("lay_temp_el"), D("lay_el_conc"), D("lay_h_conc"), D("lay_ph2_conc"),
                    D("lay_oh2_conc"), D("lay_he_conc"), D("lay_mol_conc"), D("lay_vel_turb"), D("lay_vel_grad"),
                    D("lay_dust_conc")};
    const int *opt_i = I("opts_i");   /* acceleration, allow_plain_retry, max_iter_acc, max_iter_plain */
    lvg_solve_opts o;
    oracle_opts_default(&o);
    o.acceleration = opt_i[0];
    o.allow_plain_retry = opt_i[1];
    o.max_iter_acc = opt_i[2];
    o.max_iter_plain = opt_i[3];
    const size_t pb = sizeof(double) * (size_t)nl * N, sb = sizeof(lvg_layer_status) * (size_t)nl;
    double *pops = calloc((size_t)nl * N, sizeof(double));
    lvg_layer_status *st = calloc((size_t)nl, sizeof *st);
    int rc = 0;
    rc |= oracle_solve_layers(&P, &L, pops, &o, st, 2);
    dump(out, "solve_b_pops", pops, pb);
    dump(out, "solve_b_status", st, sb);
    o.init = LVG_INIT_WARM_CHAIN;
    rc |= oracle_solve_layers(&P, &L, pops, &o, st, 2);
    dump(out, "solve_w_pops", pops, pb);
    dump(out, "solve_w_status", st, sb);
    const int off[3] = {0, nl / 2, nl};
    rc |= oracle_solve_chains(&P, &L, 2, off, pops, &o, st, 2);
    dump(out, "chains_pops", pops, pb);
    dump(out, "chains_status", st, sb);
    o.init = LVG_INIT_BOUNDARY_LAYER;
    if (has_ov) {
        o.line_overlap = 1;
        rc |= oracle_solve_layers(&P, &L, pops, &o, st, 2);
        dump(out, "solve_ov_pops", pops, pb);
        dump(out, "solve_ov_status", st, sb);
        o.line_overlap = 0;
    }
    double *bnd = calloc((size_t)nl * N, sizeof(double));
    rc |= oracle_boundary_layer_populations(&P, &L, bnd);
    dump(out, "bnd", bnd, pb);
    double *M = calloc((size_t)N * N, sizeof(double)), *df = calloc((size_t)N, sizeof(double));
    double *pn = calloc((size_t)N, sizeof(double)), eq = 0.;
    rc |= oracle_calc_new_pop(&P, &L, nl - 1, bnd + (size_t)(nl - 1) * N, has_ov, M, df, pn, &eq);
    dump(out, "cnp_matrix", M, sizeof(double) * (size_t)N * N);
    dump(out, "cnp_df", df, sizeof(double) * (size_t)N);
    dump(out, "cnp_pop", pn, sizeof(double) * (size_t)N);
    /* post-processing of the boundary-init solution */
    rc |= oracle_solve_layers(&P, &L, pops, &o, st, 2);
    lvg_cloud_geometry geo = {D("geo_dz"), D("geo_vel_n"), D("geo_height")[0]};
    lvg_find_opts fo;
    oracle_find_opts_default(&fo);
    fo.rel_error = 1e-12;
    int nf = 0;
    const int maxo = 64;
    lvg_transition *tr = calloc((size_t)maxo, sizeof *tr);
    double *inv = calloc((size_t)maxo * nl, sizeof(double)), *gain = calloc((size_t)maxo * nl, sizeof(double)),
           *exc = calloc((size_t)maxo * nl, sizeof(double));
    rc |= oracle_find_transitions(&P, &L, &geo, pops, &fo, maxo, &nf, tr, inv, gain, exc);
    const int kf = nf < maxo ? nf : maxo;
    dump(out, "find_n", &nf, sizeof nf);
    dump(out, "find_tr", tr, sizeof *tr * (size_t)kf);
    dump(out, "find_inv", inv, sizeof(double) * (size_t)kf * nl);
    int up[3] = {1, 2, 3}, low[3] = {0, 0, 1};
    double lum[3], *la = calloc((size_t)3 * nl * 5, sizeof(double));
    rc |= oracle_lim_luminosity(&P, &L, &geo, pops, 3, up, low, 0, lum, la, la + 3 * nl, la + 6 * nl, la + 9 * nl,
                                la + 12 * nl);
    dump(out, "lum", lum, sizeof lum);
    dump(out, "lum_arr", la, sizeof(double) * (size_t)15 * nl);
    free(la); free(inv); free(gain); free(exc); free(tr); free(M); free(df); free(pn); free(bnd); free(pops); free(st);
    free(comp); free(tabs);
    for (int i = 0; i < nA; i++) free(A[i].data);
    printf("ORACLE DRIVER rc=%d\n", rc);
    return rc ? 1 : 0;
}
