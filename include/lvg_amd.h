/*
 * lvg_amd.h — C ABI of the MI355X-native LVG level-population solver.
 *
 * This is the drop-in boundary for the reference's `calc_molecular_populations`
 * layer loop (/root/reference/radiative_transfer/radiative_transfer.cpp:219-289)
 * and the per-layer solve it drives:
 *   iteration_control<iteration_scheme_lvg>::calculate_populations
 *       (/root/reference/radiative_transfer/iteration_control.h:196-242)
 *   iteration_scheme_lvg::calc_new_pop / operator() / intensity_calc
 *       (/root/reference/radiative_transfer/iteration_lvg.cpp:87-185)
 *   iteration_scheme_line_overlap::operator() / intensity_calc(u1,l1,u2,l2)
 *       (/root/reference/radiative_transfer/iteration_lvg.cpp:348-501)
 *   boundary_layer_populations (/root/reference/radiative_transfer/iteration_control.cpp:52-91)
 *
 * Plain C: no torch or HIP types cross this boundary. Every pointer in the
 * description structs is a HOST pointer that is read during the call only
 * (lvg_create copies all tables to the device; no pointer is retained).
 * The exceptions are lvg_solve_layers_device() and lvg_solve_chains_device(),
 * whose layer/population/status buffers are device pointers (inputs already
 * resident in HBM).
 *
 * Units are the reference's CGS units: energies in cm^-1, masses in g,
 * concentrations in cm^-3, velocities in cm/s, velocity gradients in s^-1,
 * collision coefficients in cm^3 s^-1, dust cross sections in cm^2 per grain.
 *
 * Errors: every entry returns 0 on success and a negative LVG_E_* code
 * otherwise; the text is available from lvg_last_error(). The library never
 * exits. Non-convergence of a layer is NOT an error: it is reported per layer
 * in lvg_layer_status (the reference's `bad_layers`, radiative_transfer.cpp:278-288).
 *
 * Threading: one handle per host thread. Every call on a handle is synchronous
 * except lvg_solve_layers_device / lvg_solve_chains_device with a non-NULL stream, which returns once its
 * kernel is queued; later calls on the same handle are ordered after it (same
 * stream: stream order; any other stream, including the handle's own: the call
 * first waits for it), and the handle frees nothing that kernel uses before it ends.
 */
#ifndef LVG_AMD_H
#define LVG_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define LVG_ABI_VERSION 1

/* ---- error codes ------------------------------------------------------- */
#define LVG_OK            0
#define LVG_E_ARG        -1   /* invalid argument / inconsistent description  */
#define LVG_E_DEVICE     -2   /* HIP runtime error                             */
#define LVG_E_NOMEM      -3   /* host or device allocation failed              */
#define LVG_E_UNSUPPORTED -4  /* valid request this build does not implement   */
#define LVG_E_STATE      -5   /* wrong call order / null handle                */

/* ---- collision-partner species (concentration slots) ------------------- */
/* The order of the arguments of collisional_transitions::set_gas_param
 * (coll_rates.h:66-67): he, ph2, oh2, h, e. */
enum lvg_species {
    LVG_SP_HE  = 0,
    LVG_SP_PH2 = 1,   /* for OH (non-HF) this slot carries n(H2, J=0) */
    LVG_SP_OH2 = 2,   /* for OH (non-HF) this slot carries n(H2, J>=1) */
    LVG_SP_H   = 3,
    LVG_SP_E   = 4,
    LVG_NB_SPECIES = 5
};

/* ---- molecule-specific collision rules ---------------------------------- */
/* Each value selects the get_rate_neutrals/set_gas_param override of one
 * reference collisional_transitions subclass. */
enum lvg_coll_rule {
    /* collisional_transitions base (coll_rates.cpp:181-197): every neutral table t
     * with up < table.nb_lev contributes k_t * n[table.species]. */
    LVG_COLL_GENERIC = 0,
    /* ch3oh_collisions (coll_rates_ch3oh.cpp:472-533): tables {He, pH2, oH2}. */
    LVG_COLL_CH3OH   = 1,
    /* h2o_collisions (coll_rates_h2o.cpp:515-548): tables {He, He-rovib, pH2,
     * oH2, H2-rovib, H} + electron tables. */
    LVG_COLL_H2O     = 2,
    /* oh_collisions (coll_rates_oh.cpp:323-347): tables {He, H2(J=0), H2(J>=1)}. */
    LVG_COLL_OH      = 3,
    /* oh_hf_collisions (coll_rates_oh.cpp:380-407): tables {He, pH2, oH2}. */
    LVG_COLL_OH_HF   = 4
};

/* ---- initial-guess policy ---------------------------------------------- */
enum lvg_init {
    /* boundary_layer_populations for every layer: layers independent, sharded
     * across CUs and GPUs (the reference's branch radiative_transfer.cpp:251-252). */
    LVG_INIT_BOUNDARY_LAYER = 0,
    /* pops_inout holds the initial guess of every layer. */
    LVG_INIT_GIVEN          = 1,
    /* the reference default (radiative_transfer.cpp:247-252): layer l starts from
     * layer l-1's result when l-1 converged, else from boundary_layer_populations.
     * Sequential across the layers of one cloud by construction: one workgroup
     * (one wave for N <= 64) walks the chain. lvg_solve_chains runs many clouds'
     * chains in one launch (the reference's OpenMP axis, radiative_transfer.cpp:152-216). */
    LVG_INIT_WARM_CHAIN     = 2
};

/* energy_level / energy_diagram / einstein_coeff (spectroscopy.h:46-87, :179-190) */
typedef struct lvg_molecule {
    int           nb_lev;   /* N                                                 */
    double        mass;     /* molecule mass, g (molecule::mass)                */
    const double *energy;   /* [N] level energies, cm^-1, strictly ascending     */
    const int    *g;        /* [N] statistical weights                           */
    const int    *v;        /* [N] vibrational/torsional number (CH3OH rule)     */
    const double *j;        /* [N] angular momentum J (CH3OH rule)               */
    const double *einst;    /* [N*N] einstein_coeff::arr row-major: einst[i*N+j] is
                               the rate i->j; A_ul for i>j, g_u/g_l*A_ul for i<j */
} lvg_molecule;

/* collision_data (coll_rates.h:12-41): packed lower triangle, linear in T. */
typedef struct lvg_coll_table {
    int           nb_lev;   /* levels covered; imax = nb_lev*(nb_lev-1)/2        */
    int           jmax;     /* number of temperature grid points                 */
    const double *tgrid;    /* [jmax] K, ascending                               */
    const double *coeff;    /* [imax*jmax] coeff[i*jmax+t], i = f*(f-1)/2 + s, f>s */
    int           species;  /* LVG_COLL_GENERIC only: concentration slot (lvg_species) */
} lvg_coll_table;

typedef struct lvg_collisions {
    int                   rule;        /* enum lvg_coll_rule                     */
    int                   nb_neutral;  /* nb1 (coll_rates.h:59)                  */
    int                   nb_electron; /* nb2 - nb1                              */
    const lvg_coll_table *tables;      /* [nb_neutral + nb_electron], coll_data order */
} lvg_collisions;

/* dust_component::absorption (dust_model.cpp:473-490) */
typedef struct lvg_dust_component {
    int           nb_en;
    double        wvl_exp;    /* long-wavelength exponent                         */
    const double *energy;     /* [nb_en] cm^-1, ascending                         */
    const double *abs_coeff;  /* [nb_en] absorption cross section per grain, cm^2 */
} lvg_dust_component;

typedef struct lvg_dust {
    int                        nb_comp;
    const lvg_dust_component  *comp;   /* [nb_comp] */
} lvg_dust;

/* lvg_method_data (lvg_method_functions.h:23-39): p(delta, gamma) */
typedef struct lvg_esc_table {
    int           nb_d, nb_g;
    const double *delta;    /* [nb_d] ascending (raw, bilinear in raw values)     */
    const double *gamma;    /* [nb_g] ascending                                   */
    const double *p;        /* [nb_d*nb_g] p[k*nb_g + l]                          */
} lvg_esc_table;

/* lvg_line_overlap_data (lvg_method_functions.h:55-70) */
typedef struct lvg_overlap_table {
    int           nb_d, nb_dx, nb_gr, nb_g;
    const double *log10_delta; /* [nb_d] log10(delta) grid (the file stores delta) */
    const double *dx;          /* [nb_dx]                                          */
    const double *gratio;      /* [nb_gr]                                          */
    const double *gamma;       /* [nb_g]                                           */
    const double *p;           /* [(nb_d*nb_dx)*(nb_gr*nb_g)]
                                  p[(m*nb_dx+n)*(nb_gr*nb_g) + k*nb_g + l]         */
} lvg_overlap_table;

typedef struct lvg_problem {
    const lvg_molecule      *mol;
    const lvg_collisions    *coll;
    const lvg_dust          *dust;
    const lvg_esc_table     *esc;        /* lvg/lvg_loss_func.txt                 */
    const lvg_overlap_table *overlap1;   /* line_overlap_func_p1 (NULL: no overlap) */
    const lvg_overlap_table *overlap2;   /* line_overlap_func_p2                  */
} lvg_problem;

/* cloud_layer fields read by the solver (cloud_data.h:27-33), SoA [nb_lay]. */
typedef struct lvg_layers {
    int           nb_lay;
    const double *temp_n, *temp_el;
    const double *el_conc, *h_conc, *ph2_conc, *oh2_conc, *he_conc;
    const double *mol_conc, *vel_turb, *vel_grad;
    const double *dust_conc;   /* [nb_lay*nb_comp] grain concentrations          */
} lvg_layers;

/* Defaults (lvg_solve_opts_default): the reference's constants
 * MAX_NB_ITER_ACC/EXT (radiative_transfer.cpp:26-27), rel_population_error
 * (:45), accel start/period/nb (iteration_control.h:71). */
typedef struct lvg_solve_opts {
    double min_error;         /* 1e-5                                            */
    int    max_iter_acc;      /* 150                                             */
    int    max_iter_plain;    /* 15000                                           */
    int    accel_start;       /* 40                                              */
    int    accel_period;      /* 5                                               */
    int    accel_nb;          /* 5 (nb_prev_steps)                               */
    int    acceleration;      /* 1: Ng-type acceleration on                      */
    int    allow_plain_retry; /* 1; 0 for CH3OHa/CH3OHe (radiative_transfer.cpp:259) */
    int    init;              /* enum lvg_init                                   */
    int    line_overlap;      /* 1: iteration_scheme_line_overlap (needs overlap tables) */
} lvg_solve_opts;

/* Per-layer outcome. */
typedef struct lvg_layer_status {
    int    converged;         /* is_found of the last calculate_populations call */
    int    iterations;        /* calc_new_pop calls, all passes of this layer    */
    int    used_plain_retry;  /* the non-accelerated retry pass ran              */
    int    reserved;
    double eq_error;          /* iteration_control::eq_error at exit             */
    double rel_error;         /* iteration_control::rel_error at exit            */
    double pop_error;         /* iteration_control::pop_error at exit            */
} lvg_layer_status;

typedef struct lvg_handle lvg_handle;

/* ---- entry points -------------------------------------------------------- */
int         lvg_abi_version(void);
void        lvg_solve_opts_default(lvg_solve_opts *opts);

/* Validate the description, build the packed device tables on `device`
 * (HIP ordinal of this process). Replaces the object graph the reference
 * builds before the layer loop: energy_diagram, einstein_coeff,
 * collisional_transitions, dust_model, iteration_scheme_lvg(::init_molecule_data). */
int         lvg_create(const lvg_problem *prob, int device, lvg_handle **out);
void        lvg_destroy(lvg_handle *h);

/* ---- several GPUs in one process (lvg_create(..., device_mask, ...)) ----------
 * One handle over the devices of `device_mask` (bit d = HIP ordinal d of this process): the
 * tables are replicated on every device, and lvg_solve_layers (independent layers),
 * lvg_solve_chains and lvg_boundary_layer_populations split their batch into contiguous
 * blocks, layer l on the (l*G/nb_lay)-th device (lvg_shard_range), whole clouds per device for
 * chains (lvg_chain_shard), one host thread and one stream per device, no exchange between
 * devices (the layers are independent). This replaces the reference's serial layer loop
 * (radiative_transfer.cpp:236-256) across GPUs without MPI / RCCL; a caller that runs one
 * process per GPU uses lvg_create per rank instead. A warm chain over the
 * whole cloud (lvg_solve_layers with LVG_INIT_WARM_CHAIN) is sequential and runs on the first
 * device; every other entry point works on the first device. lvg_last_kernel_time reports
 * the slowest device's kernel time and the launches of all devices. Results are bit-identical
 * to one device's. lvg_create_devices takes an explicit list (repeats allowed: several blocks
 * on one GPU, each with its own stream). */
int         lvg_create_multi(const lvg_problem *prob, unsigned device_mask, lvg_handle **out);
int         lvg_create_devices(const lvg_problem *prob, int nb_devices, const int *devices, lvg_handle **out);
int         lvg_nb_devices(const lvg_handle *h);
/* the partition rules (pure functions, no device): block [lo, hi) of device r of nb_dev over n
 * layers; the chains [c_lo, c_hi) of device r (chain c = layers [chain_off[c], chain_off[c+1])) */
int         lvg_shard_range(int n, int nb_dev, int r, int *lo, int *hi);
int         lvg_chain_shard(int nb_chain, const int *chain_off, int nb_dev, int r, int *c_lo, int *c_hi);
const char *lvg_last_error(const lvg_handle *h);   /* h may be NULL: last create error */
int         lvg_nb_lev(const lvg_handle *h);

/* Batched replacement of calc_molecular_populations' layer loop.
 * pops_inout: host [nb_lay*N] layer-major (pop[l*N+i]); read when
 * opts->init == LVG_INIT_GIVEN, always written. status: host [nb_lay] or NULL. */
int         lvg_solve_layers(lvg_handle *h, const lvg_layers *layers, double *pops_inout,
                             const lvg_solve_opts *opts, lvg_layer_status *status);

/* Device-resident variant (all buffers already in HBM, stream = hipStream_t
 * or NULL for the handle's stream). d_layer_soa is [10 + nb_comp][nb_lay] fp64
 * in the field order of lvg_layers (temp_n, temp_el, el_conc, h_conc, ph2_conc,
 * oh2_conc, he_conc, mol_conc, vel_turb, vel_grad, then dust_conc[c]) — see
 * lvg_layer_soa_rows(). d_status: [nb_lay] lvg_layer_status. Asynchronous on
 * a non-NULL `stream` (see Threading above); synchronous with NULL.
 * LVG_INIT_WARM_CHAIN treats the nb_lay layers as one cloud (one chain). */
int         lvg_layer_soa_rows(const lvg_handle *h);
int         lvg_solve_layers_device(lvg_handle *h, int nb_lay, const double *d_layer_soa,
                                    double *d_pops_inout, const lvg_solve_opts *opts,
                                    lvg_layer_status *d_status, void *stream);

/* Batched warm chains: nb_chain independent clouds in ONE launch. The reference
 * runs calc_molecular_populations (radiative_transfer.cpp:219-289, default start
 * rule :247-252) once per cloud, one cloud per OpenMP thread (:152-216); here chain
 * c is layers [chain_off[c], chain_off[c+1]) of `layers`, walked in layer order by
 * one workgroup (one wave for N <= 64), all chains in parallel (longest first).
 * Results per chain equal lvg_solve_layers(LVG_INIT_WARM_CHAIN) on that chain alone.
 * chain_off: HOST [nb_chain + 1], chain_off[0] = 0, non-decreasing,
 * chain_off[nb_chain] = nb_lay. opts->init must be LVG_INIT_WARM_CHAIN.
 * pops_out: host [nb_lay*N]; status: host [nb_lay] or NULL. */
int         lvg_solve_chains(lvg_handle *h, const lvg_layers *layers, int nb_chain, const int *chain_off,
                             double *pops_out, const lvg_solve_opts *opts, lvg_layer_status *status);
/* Device-resident variant: d_layer_soa / d_pops_out / d_status as in
 * lvg_solve_layers_device; chain_off stays a HOST array (copied on `stream`). */
int         lvg_solve_chains_device(lvg_handle *h, int nb_lay, const double *d_layer_soa, int nb_chain,
                                    const int *chain_off, double *d_pops_out, const lvg_solve_opts *opts,
                                    lvg_layer_status *d_status, void *stream);

/* One calc_new_pop (iteration_lvg.cpp:87-110) for layer `layer` on the device:
 * returns the assembled rate matrix before LU (matrix_out [N*N] row-major,
 * M[final][initial], row 0 = ones; may be NULL), the residual df (df_out [N],
 * may be NULL), the new populations and eq_error. A debugging / parity probe. */
int         lvg_debug_calc_new_pop(lvg_handle *h, const lvg_layers *layers, int layer,
                                   const double *pop_in, int line_overlap,
                                   double *matrix_out, double *df_out,
                                   double *pop_out, double *eq_error);

/* boundary_layer_populations (iteration_control.cpp:52-91) for every layer,
 * on the device: pops_out host [nb_lay*N]. */
int         lvg_boundary_layer_populations(lvg_handle *h, const lvg_layers *layers,
                                           double *pops_out);

/* ---- post-processing of the populations ------------------------------------
 * transition_data_container::find (transition_data.cpp:380-417) with calc_inv,
 * calc_gain, calc_line_profile and calc_exc_temp (:210-377), on the device.
 * Lines are the (u > l) pairs with A_ul != 0 in (u, l) ascending order; a line is
 * kept when some layer has inv * g_u > rel_error * pops[u] (the reference compares
 * with the FIRST layer's population of u, level_pop[i], :398 — reproduced) and then
 * tau_max >= min_optical_depth. Results come in the order of the reference's list
 * (push_front: last found first). */
#define LVG_NB_ASPECT 37    /* transition_data::nb_aspect_ratio (transition_data.cpp:18) */
#define LVG_NB_FREQ   300   /* transition_data::nb_freq                                  */

typedef struct lvg_cloud_geometry {
    const double *dz;      /* [nb_lay] cloud_layer::dz, cm                           */
    const double *vel_n;   /* [nb_lay] cloud_layer::vel_n, cm/s                      */
    double height;         /* cloud_data::get_height() = zu(last) - zl(first) (cloud_data.cpp:106) */
} lvg_cloud_geometry;

typedef struct lvg_find_opts {
    double rel_error;           /* find(level_pop, rel_error)                         */
    double min_optical_depth;   /* 0.01 (transition_data.cpp:182)                     */
    double velocity_shift;      /* 5e5 cm/s (:190)                                    */
    double delta_aspect_ratio;  /* 0.25 (:18)                                         */
    int    h2o22_up, h2o22_low; /* levels of the o-H2O 6_16-5_23 22 GHz line, whose gain
                                   width includes the hyperfine spread (:251-263); -1: none */
} lvg_find_opts;

typedef struct lvg_transition {
    int    up, low;             /* level indices                                     */
    int    lay_nb_hg;           /* layer of the highest gain (0 if none positive)    */
    int    reserved;
    double energy;              /* E_up - E_low, cm^-1                               */
    double inv, gain;           /* dz-weighted averages over the cloud               */
    double tau_eff, tau_max;
    double tau_vs_aspect_ratio[LVG_NB_ASPECT];
    double tau_vs_frequency[LVG_NB_FREQ];
} lvg_transition;

void        lvg_find_opts_default(lvg_find_opts *o);
/* pops: host [nb_lay*N]. out: [max_out]; inv_arr, gain_arr, exc_temp_arr: host
 * [max_out*nb_lay] (row k belongs to out[k]) or NULL. *nb_out receives the number of
 * transitions found even when it exceeds max_out (then only max_out are written). */
int         lvg_find_transitions(lvg_handle *h, const lvg_layers *layers, const lvg_cloud_geometry *geo,
                                 const double *pops, const lvg_find_opts *opts, int max_out, int *nb_out,
                                 lvg_transition *out, double *inv_arr, double *gain_arr, double *exc_temp_arr);

/* lim_luminosity_lvg (maser_luminosity.cpp:7-106) for the transitions (up[t], low[t])
 * (e.g. those lvg_find_transitions kept), on the device. Per transition and layer:
 * the loss rates of both levels (radiative terms through intensity_calc, then the
 * neutral collision rates to every other level, in level order), the limiting
 * luminosity, pump efficiency, loss rate, pump rate and emission measure; lum[t] is
 * the dz-weighted cloud average. The reference passes the FIRST layer's populations
 * to intensity_calc (level_pop, :54, :58); layer_pops_in_intensity = 0 reproduces
 * that, 1 uses each layer's own populations. Per-layer outputs: host
 * [nb_trans*nb_lay] or NULL. */
int         lvg_lim_luminosity(lvg_handle *h, const lvg_layers *layers, const lvg_cloud_geometry *geo,
                               const double *pops, int nb_trans, const int *up, const int *low,
                               int layer_pops_in_intensity, double *lum, double *lum_arr,
                               double *emiss_coeff_arr, double *pump_rate_arr, double *pump_eff_arr,
                               double *loss_rate_arr);

/* Kernel timing of the last lvg_solve_layers* call on this handle, measured
 * with HIP events on the stream the kernels ran on: total milliseconds of the
 * solve kernel(s) and their count. */
int         lvg_last_kernel_time(const lvg_handle *h, double *ms, int *nb_launches);

/* Milliseconds of the collision-operator kernel (coll_kernel) that ran ahead of
 * the solve kernel in the last lvg_solve_layers* call, 0 if it did not run
 * (the default; wave kernel, warm chains, or the batch over its memory budget). The
 * reference builds these operators inside set_gas_param per layer
 * (coll_rates.cpp:152-174, iteration_lvg.cpp:121-131); no reference counterpart. */
int         lvg_last_coll_time(const lvg_handle *h, double *ms);

/* Which solve kernel ran the last lvg_solve_* call on this handle (diagnostic; every
 * kernel gives bit-identical results): 0 the 256-thread block kernel (N <= 256), 1 the
 * wave kernel (N <= 64), 2 the 512-thread block kernel (N <= 256, launches with at most
 * two independent layers or one warm chain per CU), 3 the 768-thread block kernel
 * (N > 256); -1 when nothing was launched (no solve yet, or an empty batch). No
 * reference counterpart. */
int         lvg_last_kernel_kind(const lvg_handle *h, int *kind);

/* Tuning and diagnostics of this handle: "key=value,key=value", MERGED into the
 * current settings (keys not named keep their value; NULL or "" resets to the defaults);
 * the environment variable LVG_TUNING supplies the initial value at lvg_create (a value
 * that does not parse is reported on stderr and ignored; it never fails lvg_create).
 * No setting changes a result (populations and status stay bit-identical).
 * Keys: block_kernel (1: the block kernel also for N <= 64), queue_order (0: layer
 * order instead of longest-expected-first), coll_ahead (1: collision operators of the
 * batch built ahead by a separate kernel), coll_mem (fraction of free device memory
 * that batch may take, default 0.5), coll_order (0: that kernel in layer order),
 * blocks_per_cu (resident block-kernel workgroups per CU, 0 = automatic), wide (0: never
 * the 512-thread kernel, 1: when the launch leaves CUs to spare, 2: always for N <= 256).
 * LVG_E_ARG on an unknown key or value (the tuning is then unchanged). No reference
 * counterpart (the reference has no device). */
int         lvg_set_tuning(lvg_handle *h, const char *spec);

#ifdef __cplusplus
}
#endif
#endif /* LVG_AMD_H */
