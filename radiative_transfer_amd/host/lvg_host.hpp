// lvg_host.hpp — C++ host surface of the MI355X LVG solver.
//
// Keeps the class shapes a user of nesterenok/radiative_transfer programs
// against on this path — energy_diagram / einstein_coeff (spectroscopy.h:46-87,
// :179-190), collision_data / collisional_transitions (coll_rates.h:12-78),
// dust_model (dust_model.h:201-230), lvg_method_data / lvg_line_overlap_data
// (lvg_method_functions.h:23-70), cloud_layer / cloud_data (cloud_data.h:23-60),
// iteration_scheme_lvg / iteration_scheme_line_overlap (iteration_lvg.h:17-102),
// iteration_control<T> (iteration_control.h:34-242), boundary_layer_populations
// (iteration_control.cpp:52-91) and calc_molecular_populations
// (radiative_transfer.cpp:82-84, :219-289) — and runs every computation through
// the C ABI of include/lvg_amd.h on the GPU. The classes here are data holders and
// drivers; there is no host implementation of the physics.
//
// Differences from the reference, all deliberate:
//  * errors throw lvg_error instead of exit(1);
//  * the scheme owns a device handle built in init_molecule_data();
//  * calc_molecular_populations takes an init policy: the reference's warm chain
//    (default, sequential across layers) or independent boundary-layer starts
//    (all layers in one batched launch).
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/lvg_amd.h"

namespace lvgamd {

struct lvg_error : std::runtime_error {
    int code;
    lvg_error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// ---- spectroscopy (spectroscopy.h:46-87, :179-190) ------------------------------
struct energy_level {
    int nb = 0, g = 1, v = 0, syminv = 0;
    double j = 0., k1 = 0., k2 = 0., spin = 0., hf = 0., energy = 0.;   // energy in cm^-1
    std::string name;
    // spectroscopy.h:57-64: equal if all quantum numbers coincide; ordered by energy
    bool operator==(const energy_level &o) const;
    bool operator<(const energy_level &o) const { return energy < o.energy && !(*this == o); }
};

class energy_diagram {
public:
    int nb_lev = 0;
    std::string mol_name;          // molecule::name, e.g. "CH3OHa" (drives the retry rule)
    double mol_mass = 0.;          // g
    double mol_spin = 0.;          // molecule::spin (selects the spin isomer in the file readers)
    int isotop = 1;                // molecule::isotop
    std::vector<energy_level> lev_array;
    energy_diagram(const std::string &name, double mass) : mol_name(name), mol_mass(mass) {}
    virtual ~energy_diagram() = default;
    void add_level(const energy_level &l) { lev_array.push_back(l); nb_lev = (int)lev_array.size(); }
    // level lookups of the molecule subclasses (spectroscopy.h:79-83); -1: not found
    virtual int get_nb(int /*v*/, double /*j*/, double /*k*/) const { return -1; }
    virtual int get_nb(int /*syminv*/, int /*v*/, double /*j*/, double /*k*/, double /*hf*/) const { return -1; }
};

// arr[i][j]: rate i->j, arr[u][l] = A_ul, arr[l][u] = g_u/g_l A_ul (spectroscopy.cpp:918-921)
class einstein_coeff {
public:
    int nb_lev = 0;
    double **arr = nullptr;
    explicit einstein_coeff(const energy_diagram *di);
    einstein_coeff(const einstein_coeff &) = delete;
    einstein_coeff &operator=(const einstein_coeff &) = delete;
    // A_ul for u > l, the l->u entry set from detailed balance as the reference does
    void set_line(int u, int l, double a_ul, const energy_diagram *di);
    const double *data() const { return storage.data(); }
private:
    std::vector<double> storage;
    std::vector<double *> rows;
};

// ---- collisions (coll_rates.h:12-78) --------------------------------------------
class collision_data {
public:
    int imax = 0, jmax = 0, nb_lev = 0;
    std::vector<double> tgrid;     // [jmax]
    double **coeff = nullptr;      // coeff[i][t], i = f(f-1)/2 + s (f > s): 1->0, 2->0, 2->1, ...
    int species = LVG_SP_HE;       // concentration slot used by the generic rule
    collision_data(int nb_lev, const std::vector<double> &tgrid);
    virtual ~collision_data() = default;
    collision_data(const collision_data &) = delete;
    collision_data &operator=(const collision_data &) = delete;
    double get_max_temp() const { return tgrid.back(); }
    const double *data() const { return storage.data(); }
protected:
    collision_data() = default;
    void allocate(int nb_lev, int jmax);   // zeroed coeff[imax][jmax], tgrid[jmax]
private:
    std::vector<double> storage;
    std::vector<double *> rows;
};

// The molecule rule of get_rate_neutrals / set_gas_param is the subclass, as in the
// reference; the device evaluates it (lvg_coll_rule). coll_data: neutral tables
// first (nb1 of them), then electron tables; the object owns them.
class collisional_transitions {
public:
    int nb_lev = 0, nb1 = 0, nb2 = 0;
    std::vector<collision_data *> coll_data;
    virtual int rule() const { return LVG_COLL_GENERIC; }
    void add_neutral(collision_data *d);
    void add_electron(collision_data *d);
    virtual ~collisional_transitions();
};
// The path constructors read the reference's data files (lvg_ingest.cpp):
// coll_rates_ch3oh.cpp:444-470, coll_rates_h2o.cpp:486-513, coll_rates_oh.cpp:350-378.
struct ch3oh_collisions : collisional_transitions {
    ch3oh_collisions() = default;
    // file_levels*: levels listed in the vt files / the rovibrational He file / the oH2
    // file (the reference's fixed 256 / 150 / 100, coll_rates_ch3oh.cpp:47, :148, :373)
    ch3oh_collisions(const std::string &path, const energy_diagram *levels, int verbosity = 0, int file_levels = 256,
                     int file_levels_rovibr = 150, int file_levels_oh2 = 100);
    int rule() const override { return LVG_COLL_CH3OH; }
};
struct h2o_collisions : collisional_transitions {
    h2o_collisions() = default;
    h2o_collisions(const std::string &path, const energy_diagram *levels, bool he_is_scaled, int verbosity = 0);
    int rule() const override { return LVG_COLL_H2O; }
};
struct oh_collisions : collisional_transitions { int rule() const override { return LVG_COLL_OH; } };
struct oh_hf_collisions : collisional_transitions {
    oh_hf_collisions() = default;
    oh_hf_collisions(const std::string &path, const energy_diagram *levels, int verbosity = 0);
    int rule() const override { return LVG_COLL_OH_HF; }
};

// ---- dust (dust_model.cpp:473-490, :834-841) ------------------------------------
class dust_component {
public:
    int nb_ph_en = 0;
    double wvl_exp = 2.;
    std::vector<double> ph_en_arr, abs_coeff;   // cm^-1, cm^2 per grain
    dust_component(std::vector<double> en, std::vector<double> abs, double wexp)
        : nb_ph_en((int)en.size()), wvl_exp(wexp), ph_en_arr(std::move(en)), abs_coeff(std::move(abs)) {}
};

class dust_model {
public:
    int nb_of_comp = 0;
    std::vector<dust_component *> components;
    void add_component(dust_component *c) { components.push_back(c); nb_of_comp = (int)components.size(); }
    ~dust_model();
};

// ---- escape-probability tables (lvg_method_functions.cpp:21-64, :264-313) -------
class lvg_method_data {
public:
    int nb_g = 0, nb_d = 0;
    std::vector<double> delta_arr, gamma_arr, p;   // p[k*nb_g + l]
    lvg_method_data(const std::string &path, const std::string &name, int verbosity = 0);
    lvg_method_data(std::vector<double> delta, std::vector<double> gamma, std::vector<double> p);
    // writes the reference's file format (3 comment lines, "nb_d nb_g", gamma, rows)
    void save(const std::string &path, const std::string &name) const;
};

class lvg_line_overlap_data {
public:
    int nb_d = 0, nb_dx = 0, nb_gr = 0, nb_g = 0;
    std::vector<double> log10_delta, dx_arr, gratio_arr, gamma_arr, p;
    lvg_line_overlap_data(const std::string &path, const std::string &name, int verbosity = 0);
    lvg_line_overlap_data(std::vector<double> log10_delta, std::vector<double> dx, std::vector<double> gratio,
                          std::vector<double> gamma, std::vector<double> p);
};

// ---- cloud (cloud_data.h:23-60) ------------------------------------------------
class cloud_layer {
public:
    double zl = 0., zu = 0., dz = 0., zm = 0.;   // layer coordinates, cm
    double temp_n = 0., temp_el = 0., av_temp_d = 0., vel_n = 0., tot_h_conc = 0., h2_opr = 0.,
           el_conc = 0., h_conc = 0., ph2_conc = 0., oh2_conc = 0., he_conc = 0., mol_conc = 0.,
           vel_turb = 0., velg_n = 0.;
    std::vector<double> dust_grain_conc, dust_grain_temp;
};

class cloud_data {
public:
    int nb_lay = 0;
    std::vector<cloud_layer> lay_array;
    void add_layer(const cloud_layer &l) { lay_array.push_back(l); nb_lay = (int)lay_array.size(); }
    void remove_layer(int i) { lay_array.erase(lay_array.begin() + i); nb_lay = (int)lay_array.size(); }
    void delete_layers() { lay_array.clear(); nb_lay = 0; }
    void set_vel_turb(double vt) { for (auto &l : lay_array) l.vel_turb = vt; }
    double get_height() const { return lay_array.back().zu - lay_array.front().zl; }   // cloud_data.cpp:106
};

// Packed SoA view of a cloud (the ABI's lvg_layers); keeps its buffers alive.
struct layer_pack {
    std::vector<double> f[10], dust;
    lvg_layers view{};
    layer_pack(const cloud_data &c, int nb_comp);
    explicit layer_pack(const std::vector<cloud_layer> &lays, int nb_comp);
};

// ---- iteration scheme (iteration_lvg.h:17-102) -----------------------------------
class iteration_scheme_lvg {
public:
    iteration_scheme_lvg(const dust_model *dust, const lvg_method_data *loss_func, int verbosity = 0,
                         int device = 0);
    virtual ~iteration_scheme_lvg();
    iteration_scheme_lvg(const iteration_scheme_lvg &) = delete;
    iteration_scheme_lvg &operator=(const iteration_scheme_lvg &) = delete;

    // builds the device tables (lvg_create); must be called again if the molecule changes
    virtual void init_molecule_data(const energy_diagram *, const einstein_coeff *, const collisional_transitions *);
    // several GPUs of this process for the next init_molecule_data (lvg_create_devices / the
    // device_mask of SURVEY 8b): calc_molecular_populations with independent (boundary-layer)
    // starts then splits the cloud's layers over them, one block per device. Empty: `device` only.
    void set_devices(const std::vector<int> &devs) { devices = devs; }
    void set_device_mask(unsigned mask) {
        devices.clear();
        for (int d = 0; d < 32; d++) if (mask & (1u << d)) devices.push_back(d);
    }
    int nb_devices() const { return h ? lvg_nb_devices(h) : 0; }
    int get_vector_dim() const { return nb_mol_lev; }

    void set_parameters(double temp_n, double temp_e, double el_conc, double h_conc, double ph2_conc,
                        double oh2_conc, double he_conc, double mol_conc, double vel_turb);
    void set_dust_parameters(const std::vector<double> &conc, const std::vector<double> &temp);
    void set_vel_grad(double vg) { cur.velg_n = vg; }

    // one calc_new_pop (iteration_lvg.cpp:87-110) for the current layer, on the device
    void calc_new_pop(double *old_pop, double *new_pop, double &eq_error);
    // the assembled rate matrix and residual of the same step (debug probe)
    void rate_matrix(const double *pop, double *matrix, double *df);

    lvg_handle *handle() const { return h; }
    bool line_overlap() const { return overlap; }
    const cloud_layer &current_layer() const { return cur; }
    const energy_diagram *diagram() const { return diag; }
    // the packed description handed to lvg_create (valid after init_molecule_data)
    const lvg_problem &problem() const { return prob; }

protected:
    int nb_mol_lev = 0, verbosity = 0, device = 0;
    std::vector<int> devices;     // set_devices: more than one -> lvg_create_devices
    bool overlap = false;
    const dust_model *dust;
    const lvg_method_data *loss_func;
    const lvg_line_overlap_data *ov1 = nullptr, *ov2 = nullptr;
    const energy_diagram *diag = nullptr;
    cloud_layer cur;
    lvg_handle *h = nullptr;
    // packed views (lvg_create copies them; kept for problem())
    std::vector<double> en, jj;
    std::vector<int> g, v;
    std::vector<lvg_coll_table> tabs;
    std::vector<lvg_dust_component> dc;
    lvg_molecule mol{};
    lvg_collisions coll{};
    lvg_dust du{};
    lvg_esc_table et{};
    lvg_overlap_table o1{}, o2{};
    lvg_problem prob{};
};

// iteration_scheme_line_overlap (iteration_lvg.h:96-102): the hfs line groups of
// iteration_lvg.cpp:259-346 are formed by lvg_create from the level structure.
class iteration_scheme_line_overlap : public iteration_scheme_lvg {
public:
    iteration_scheme_line_overlap(const dust_model *dust, const lvg_method_data *loss_func,
                                  const lvg_line_overlap_data *p1, const lvg_line_overlap_data *p2,
                                  int verbosity = 0, int device = 0);
};

// ---- iteration_control<T> (iteration_control.h:34-242) -----------------------------
// calculate_populations runs the whole accelerated fixed-point iteration of the
// scheme's current layer on the device (one lvg_solve_layers call, init = given).
template <class T>
class iteration_control {
public:
    int iter_nb = 0, accel_start = 40, accel_period = 5, nb_prev_steps = 5;
    double eq_error = 0., pop_error = 0., rel_error = 0.;
    explicit iteration_control(T *s) : scheme(s) {}
    bool calculate_populations(double *pop, int max_nb_iter, double min_error, bool acceleration, int verbosity = 0);
private:
    T *scheme;
};

// ---- drivers ----------------------------------------------------------------------
enum class init_policy { warm_chain, boundary_layer };

// boundary_layer_populations (iteration_control.cpp:52-91) of the scheme's molecule for
// the given layer conditions; pop: [nb_lev]
void boundary_layer_populations(iteration_scheme_lvg *scheme, double *pop, double temp_neutrals,
                                double temp_el, double el_conc, double h_conc, double ph2_conc,
                                double oh2_conc, double he_conc);

// calc_molecular_populations (radiative_transfer.cpp:219-289). mol_popul: [nb_lay*nb_lev]
// layer-major. Returns the layers without a solution (the reference's bad_layers).
std::vector<int> calc_molecular_populations(cloud_data *cloud, iteration_scheme_lvg *it_scheme_lvg,
                                            energy_diagram *mol_levels, einstein_coeff *mol_einst,
                                            collisional_transitions *mol_coll, double *mol_popul, int nb_lev,
                                            bool acceleration, int verbosity,
                                            init_policy init = init_policy::warm_chain,
                                            std::vector<lvg_layer_status> *status = nullptr);

// ---- populations on disk (spectroscopy.cpp:1294-1368) -------------------------------
// save_populations: "<output_path><mol_name>_populations<id>.txt", N rows x nb_lay columns
// (scientific, 6 digits), divided by g when `normalized`; unlike the reference's setw(12)
// fields, a space follows every value (12-character values would otherwise run
// together and not read back). read_populations: the same
// layout back into arr[l*N + i]; throws on a size mismatch (the reference prints).
std::string save_populations(const std::string &output_path, const energy_diagram *diagram, const double *arr,
                             int nb_cloud_lay, int nb_mol_lev, bool normalized, const std::string &id);
void read_populations(const std::string &file_name, double *arr, int nb_cloud_lay, int nb_mol_lev);

// ---- post-processing (transition_data.h:11-80, maser_luminosity.cpp:7-106) ----------
struct cloud_geometry {
    std::vector<double> dz, vel_n;   // cloud_layer::dz, ::vel_n
    double height = 0.;              // cloud_data::get_height()
};

struct transition_data {
    int up = 0, low = 0, lay_nb_hg = 0;
    double energy = 0., inv = 0., gain = 0., lum = 0., tau_eff = 0., tau_max = 0.;
    std::vector<double> inv_arr, gain_arr, exc_temp_arr;
    std::vector<double> lum_arr, emiss_coeff_arr, pump_rate_arr, pump_eff_arr, loss_rate_arr;
    std::vector<double> tau_vs_aspect_ratio, tau_vs_frequency;
};

class transition_data_container {
public:
    double min_optical_depth = 0.01, velocity_shift = 5.e+5;
    int h2o22_up = -1, h2o22_low = -1;    // the o-H2O 22 GHz line, if any
    std::vector<transition_data> data;    // the reference's list order
    transition_data_container(const cloud_data *cl, const cloud_geometry *geo, iteration_scheme_lvg *scheme)
        : cloud(cl), geo(geo), scheme(scheme) {}
    // find(level_pop, rel_error) (transition_data.cpp:380-417) on the device
    void find(const double *level_pop, double rel_error);
private:
    const cloud_data *cloud;
    const cloud_geometry *geo;
    iteration_scheme_lvg *scheme;
    friend void lim_luminosity_lvg(iteration_scheme_lvg *, transition_data_container *, const cloud_data *,
                                   const double *, bool);
};

// lim_luminosity_lvg for every transition of the container, on the device. The
// reference passes the first layer's populations to intensity_calc; keep that with
// first_layer_pops_in_intensity = true (default).
void lim_luminosity_lvg(iteration_scheme_lvg *calc_scheme, transition_data_container *container,
                        const cloud_data *cloud, const double *level_pop, bool first_layer_pops_in_intensity = true);

}  // namespace lvgamd
