// lvg_ingest.hpp — readers of the reference's on-disk input formats (SURVEY.md §8f
// rows 3-4): molecular levels, radiative rates and collision tables for the three
// molecules of the BASELINE configurations (CH3OH A/E, ortho/para-H2O, OH with
// hyperfine splitting), and the C-shock cloud profile files.
//
// Each reader restates one reference constructor or function and keeps its file
// layout, index conventions and in-place corrections (detailed-balance
// symmetrisation, unit conversion, level matching by quantum numbers). The
// differences are deliberate and few:
//  * errors throw lvg_error (LVG_E_ARG) instead of printing and calling exit(1);
//  * the CH3OH collision readers take the number of levels listed in each file as an
//    argument (default: the reference's fixed 256 / 150 / 100), so that test files
//    can be small;
//  * the readers never print unless verbosity > 0.
// All physics stays on the device; these are host-side, once-per-run parsers.
#pragma once

#include "lvg_host.hpp"

namespace lvgamd {

constexpr int NB_VIBR_EXCIT_H2O = 4;              // spectroscopy.h:8
constexpr int NB_VIBR_EXCIT_CH3OH_MEKHTIEV = 2;   // spectroscopy.h:11
constexpr int NB_ANG_MOM_CH3OH = 22;              // spectroscopy.h:13
constexpr int NB_VIBR_EXCIT_CH3OH_RABLI = 2;      // coll_rates_ch3oh.h:7
constexpr bool USE_TEMPER_EXTRAP_CH3OH = false;   // coll_rates_ch3oh.h:8
constexpr bool USE_EXTENDED_OH_HF_H2_DATA = true; // coll_rates_oh.h:4
constexpr double MIN_VELOCITY_GRADIENT = 3.e-14;  // cloud_data.cpp:13

// CGS constants of the absent constants.h (CODATA 2018; as oracle/lvg_oracle.c)
constexpr double CM_INVERSE_TO_KELVINS = 1.438776877;
constexpr double PLANCK_CONSTANT = 6.62607015e-27;
constexpr double DEBYE = 1.e-18;

// utils.h rounding(): nearest integer, halves up
int rounding(double x);

// ---- energy diagrams (spectroscopy.cpp) ---------------------------------------------
// <path>spectroscopy/levels_ch3oh.txt; A (spin 3/2) or E (spin 1/2) species; levels with
// vt <= nb_vibr and J <= ang_mom_max, energies relative to the J=0 K=0 vt=0 level,
// sorted by energy and cut to n_l (n_l receives the count). spectroscopy.cpp:295-385
class ch3oh_diagram : public energy_diagram {
public:
    ch3oh_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int &n_l,
                  int nb_vibr = NB_VIBR_EXCIT_CH3OH_MEKHTIEV, int ang_mom_max = NB_ANG_MOM_CH3OH, int verbosity = 0);
    int get_nb(int v, double j, double k) const override;   // spectroscopy.cpp:387-394
};

// <path>spectroscopy/levels_h2o16.txt (isotop 1) or levels_h2o18.txt; ortho (spin 1) or
// para (spin 0) by (ka + kc + v3) parity. spectroscopy.cpp:218-273
class h2o_diagram : public energy_diagram {
public:
    h2o_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int isotop, int &n_l,
                int nb_vibr = NB_VIBR_EXCIT_H2O, int verbosity = 0);
    int get_nb(int v, double j, double tau) const override;  // tau = ka - kc; spectroscopy.cpp:275-282
    int get_vibr_nb(int v1, int v2, int v3) const;            // spectroscopy.cpp:284-293
};

// <path>spectroscopy/levels_oh_hf.txt, g = 2F + 1. spectroscopy.cpp:560-608
class oh_hf_diagram : public energy_diagram {
public:
    oh_hf_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int &n_l,
                  int verbosity = 0);
    int get_nb(int parity, int v, double j, double omega, double hf) const override;   // :610-619
};

// ---- radiative rates ----------------------------------------------------------------
// radiative_ch3oh_a.txt / _e.txt: A_ul from the line strength,
// 64 S DEBYE^2 pi (pi dE)^3 / (3 h (2 J_u + 1)). spectroscopy.cpp:865-927
class ch3oh_einstein_coeff : public einstein_coeff {
public:
    ch3oh_einstein_coeff(const std::string &path, const energy_diagram *ch3oh_di, int verbosity = 0);
};
// radiative_h2o16.txt / _h2o18.txt. spectroscopy.cpp:816-863
class h2o_einstein_coeff : public einstein_coeff {
public:
    h2o_einstein_coeff(const std::string &path, const h2o_diagram *h2o_di, int verbosity = 0);
};
// radiative_oh_hf.txt. spectroscopy.cpp:1090-1131
class oh_hf_einstein_coeff : public einstein_coeff {
public:
    oh_hf_einstein_coeff(const std::string &path, const energy_diagram *di, int verbosity = 0);
};

// ---- collision tables -------------------------------------------------------------------
// CH3OH (coll_rates_ch3oh.cpp:27-441): per-vt files with a full rate matrix per
// temperature, symmetrised 0.5 (k_down + k_up g_l/g_u e^{dE/kT}).
class ch3oh_he_coll_data : public collision_data {
public:
    ch3oh_he_coll_data(const std::string &path, const energy_diagram *levels, int verbosity = 0,
                       int file_levels = 256, int file_levels_rovibr = 150);
};
class ch3oh_ph2_coll_data : public collision_data {
public:
    ch3oh_ph2_coll_data(const std::string &path, const energy_diagram *levels, int verbosity = 0, int file_levels = 256);
};
class ch3oh_oh2_coll_data : public collision_data {
public:
    ch3oh_oh2_coll_data(const std::string &path, const energy_diagram *levels, int verbosity = 0, int file_levels = 100);
};
// H2O (coll_rates_h2o.cpp:28-484)
class h2o_oh2_coll_data : public collision_data {       // 45 levels, packed lines
public:
    h2o_oh2_coll_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
class h2o_ph2_coll_data : public collision_data {
public:
    h2o_ph2_coll_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
class h2o_h2_coll_rovibr_data : public collision_data { // lines labelled by quantum numbers
public:
    h2o_h2_coll_rovibr_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
class h2o_he_coll_data : public collision_data {        // both directions, symmetrised
public:
    h2o_he_coll_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
class h2o_he_coll_rovibr_data : public collision_data {
public:
    h2o_he_coll_rovibr_data(const std::string &path, const energy_diagram *di, bool is_scaled, int verbosity = 0);
};
class h2o_e_coll_rovibr_data : public collision_data {
public:
    h2o_e_coll_rovibr_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
class h2o_h_coll_data : public collision_data {
public:
    h2o_h_coll_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};
// OH hyperfine (coll_rates_oh.cpp:129-293)
class oh_hf_h2_coll_data : public collision_data {      // Offer et al. 1994 layout
public:
    oh_hf_h2_coll_data(const std::string &path, const energy_diagram *di, bool coll_partner_is_ortho, int verbosity = 0);
};
class oh_hf_h2_ext_coll_data : public collision_data {  // Cragg et al. 2002 layout (the default)
public:
    oh_hf_h2_ext_coll_data(const std::string &path, const energy_diagram *di, bool coll_partner_is_ortho,
                           int verbosity = 0);
};
class oh_hf_he_coll_data : public collision_data {
public:
    oh_hf_he_coll_data(const std::string &path, const energy_diagram *di, int verbosity = 0);
};

// ---- cloud profiles (cloud_data.cpp:143-472) ----------------------------------------------
// Reads sim_phys_param.txt, sim_data_h2_chemistry.txt, sim_specimen_abund.txt and
// sim_dust_data.txt of one shock model; layer values are the averages of adjacent
// points; |velg_n| is raised to MIN_VELOCITY_GRADIENT. Returns false if a file is missing.
bool set_physical_parameters(const std::string &data_path, cloud_data *cloud);
// Column-averaged concentration of the named species over each layer, times f.
bool set_molecular_conc(const std::string &data_path, const std::string &mol_name, cloud_data *cloud, double f = 1.);
// Merges every nb consecutive layers, dz-weighted; drops the remainder.
void join_layers(cloud_data *cloud, int nb);
// the geometry the post-processing needs (cloud_layer::dz, ::vel_n; get_height())
cloud_geometry geometry_of(const cloud_data &cloud);

}  // namespace lvgamd
