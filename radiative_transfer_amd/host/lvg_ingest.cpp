// lvg_ingest.cpp — readers of the reference's input files (see lvg_ingest.hpp).
// Every function cites the reference code it restates; the parsing steps (stream
// extraction order, skipped lines, quirks) follow it token for token.
#include "lvg_ingest.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <fstream>
#include <iostream>
#include <sstream>

namespace lvgamd {

int rounding(double x) { return (int)std::floor(x + 0.5); }

namespace {
void skip(std::istream &in, int n) {
    std::string s;
    for (int i = 0; i < n; i++) std::getline(in, s);
}

std::ifstream open_or_throw(const std::string &fname, const char *who) {
    std::ifstream in(fname);
    if (!in) throw lvg_error(LVG_E_ARG, std::string(who) + ": can't open " + fname);
    return in;
}

void check_stream(const std::istream &in, const std::string &fname, const char *who) {
    if (in.bad() || (in.fail() && !in.eof())) throw lvg_error(LVG_E_ARG, std::string(who) + ": malformed " + fname);
}

void report(int verbosity, const std::string &what, const std::string &fname) {
    if (verbosity) std::cout << "  " << what << " read from " << fname << std::endl;
}

// the CH3OH files write some rates as "a.b-dfg" without the E: the mantissa is read,
// the exponent is the next token and the rate is dropped (coll_rates_ch3oh.cpp:103-110)
double ch3oh_rate(std::istream &in) {
    double rate, a;
    in >> rate;
    if (std::fabs(rate) >= 1. - DBL_EPSILON) {
        in >> a;
        rate = 0.;
    } else if (rate < 0.) {
        rate = 0.;
    }
    return rate;
}

// symmetrised contribution of one file entry (initial k -> final i) to the packed
// down-rate table at temperature index j (coll_rates_ch3oh.cpp:115-127)
void ch3oh_accumulate(collision_data &c, const energy_diagram *lev, int i1, int i2, int j, double rate,
                      bool reset_same_v) {
    if (i1 == -1 || i2 == -1) return;
    if (i1 > i2) {
        const int l = i1 * (i1 - 1) / 2 + i2;
        if (reset_same_v && lev->lev_array[i1].v == lev->lev_array[i2].v) c.coeff[l][j] = 0.;
        c.coeff[l][j] += 0.5 * rate;
    } else if (i1 < i2) {
        const int l = i2 * (i2 - 1) / 2 + i1;
        if (reset_same_v && lev->lev_array[i1].v == lev->lev_array[i2].v) c.coeff[l][j] = 0.;
        c.coeff[l][j] += 0.5 * rate * lev->lev_array[i1].g / ((double)lev->lev_array[i2].g) *
                         std::exp((lev->lev_array[i2].energy - lev->lev_array[i1].energy) * CM_INVERSE_TO_KELVINS /
                                  c.tgrid[j]);
    }
}

char ch3oh_species(const energy_diagram *lev) { return rounding(2. * lev->mol_spin) == 3 ? 'a' : 'e'; }

// the level table at the head of a CH3OH collision file -> level indices
// (coll_rates_ch3oh.cpp:84-92; with_vt: the rovibrational file lists vt per level, :168-176)
void ch3oh_level_table(std::istream &in, const energy_diagram *lev, int nb_of_levels, int vt_fixed, bool with_vt,
                       std::vector<int> &nb_arr) {
    const bool a_type = rounding(2. * lev->mol_spin) == 3;
    nb_arr.assign(nb_of_levels, 0);
    for (int i = 0; i < nb_of_levels; i++) {
        int l, vt = vt_fixed, j, k;
        char ch;
        double energy;
        in >> l;
        if (with_vt) in >> vt;
        in >> ch;
        if (a_type) in >> ch;
        in >> j >> k >> energy;
        if (ch == '-') k = -k;
        nb_arr[i] = lev->get_nb(vt, j, k);
    }
    skip(in, 4);   // the end of the last level line and three header lines
}

// one rate block per temperature: "T", then per final level "idx rate[initial]..."
void ch3oh_rate_blocks(std::istream &in, collision_data &c, const energy_diagram *lev, int j_end,
                       const std::vector<int> &nb_arr, bool reset_same_v) {
    const int n = (int)nb_arr.size();
    for (int j = 1; j < j_end; j++) {
        in >> c.tgrid[j];
        for (int i = 0; i < n; i++) {     // row: index of the final level
            int l;
            in >> l;
            for (int k = 0; k < n; k++) { // column: index of the initial level
                const double rate = ch3oh_rate(in);
                ch3oh_accumulate(c, lev, nb_arr[k], nb_arr[i], j, rate, reset_same_v && k > i);
            }
        }
    }
}
}  // namespace

// ---- energy diagrams ------------------------------------------------------------------
ch3oh_diagram::ch3oh_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int &n_l,
                             int nb_vibr, int ang_mom_max, int verbosity)
    : energy_diagram(name, mass) {
    mol_spin = spin;
    const std::string fname = data_path + "spectroscopy/levels_ch3oh.txt";
    std::ifstream input = open_or_throw(fname, "ch3oh_diagram");
    if (nb_vibr > NB_VIBR_EXCIT_CH3OH_MEKHTIEV) nb_vibr = NB_VIBR_EXCIT_CH3OH_MEKHTIEV;
    skip(input, 2);
    const int vt_max = 8;   // torsional states listed per row
    double energy_min = 0.;
    int j, k1;
    // the block counter is the J read from the file, as in spectroscopy.cpp:321-361
    for (j = 0; j <= NB_ANG_MOM_CH3OH; j++) {
        skip(input, 4);
        for (int l = 0; l < 2 * (2 * j + 1); l++) {
            char ch1, ch2;
            input >> ch1;
            if (l < 2 * j + 1) input >> ch2;
            else ch2 = ' ';
            input >> j >> k1;
            for (int vt = 0; vt <= vt_max; vt++) {
                double energy;
                input >> energy;
                if (j == 0 && k1 == 0 && vt == 0 && l == 0) energy_min = energy;
                if (vt <= nb_vibr && j <= ang_mom_max &&
                    ((rounding(2. * spin) == 3 && ch1 == 'A') || (rounding(2. * spin) == 1 && ch1 == 'E'))) {
                    energy_level level;
                    level.v = vt;
                    level.j = j;
                    level.k1 = (ch2 == '-') ? -k1 : k1;   // A species: the sign tells the pair apart
                    level.spin = spin;
                    level.energy = energy - energy_min;
                    level.g = rounding(2. * spin + 1.) * (2 * j + 1);
                    lev_array.push_back(level);
                }
            }
        }
        skip(input, 1);
    }
    check_stream(input, fname, "ch3oh_diagram");
    std::sort(lev_array.begin(), lev_array.end());
    if ((int)lev_array.size() > n_l) lev_array.resize(n_l);
    nb_lev = n_l = (int)lev_array.size();
    for (int i = 0; i < nb_lev; i++) lev_array[i].nb = i;
    report(verbosity, "CH3OH levels", fname);
}

int ch3oh_diagram::get_nb(int v, double j, double k) const {
    for (int i = 0; i < nb_lev; i++)
        if (lev_array[i].v == v && rounding(lev_array[i].j) == rounding(j) && rounding(lev_array[i].k1) == rounding(k))
            return i;
    return -1;
}

h2o_diagram::h2o_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int iso,
                         int &n_l, int nb_vibr, int verbosity)
    : energy_diagram(name, mass) {
    mol_spin = spin;
    isotop = iso;
    if (nb_vibr > NB_VIBR_EXCIT_H2O) nb_vibr = NB_VIBR_EXCIT_H2O;
    const std::string fname = data_path + (iso == 1 ? "spectroscopy/levels_h2o16.txt" : "spectroscopy/levels_h2o18.txt");
    std::ifstream input = open_or_throw(fname, "h2o_diagram");
    skip(input, 2);
    int i_max;
    input >> i_max;
    int nb = 0, i = 0;
    while (nb < n_l && i < i_max) {   // spectroscopy.cpp:247-270
        int v1, v2, v3, j, ka, kc;
        double energy;
        input >> v1 >> v2 >> v3 >> j >> ka >> kc >> energy;
        const int v = get_vibr_nb(v1, v2, v3);
        if (std::abs(ka + kc + v3) % 2 == rounding(spin) && v <= nb_vibr) {
            energy_level level;
            level.v = v;
            level.j = j;
            level.k1 = ka;
            level.k2 = kc;
            level.energy = energy;
            level.spin = spin;
            level.g = rounding(2. * spin + 1.) * (2 * j + 1);
            level.nb = nb;
            lev_array.push_back(level);
            nb++;
        }
        i++;
    }
    check_stream(input, fname, "h2o_diagram");
    nb_lev = n_l = (int)lev_array.size();
    report(verbosity, "H2O levels", fname);
}

int h2o_diagram::get_nb(int v, double j, double tau) const {
    for (int i = 0; i < nb_lev; i++)
        if (lev_array[i].v == v && rounding(lev_array[i].j) == rounding(j) &&
            rounding(lev_array[i].k1 - lev_array[i].k2) == rounding(tau))
            return i;
    return -1;
}

int h2o_diagram::get_vibr_nb(int v1, int v2, int v3) const {
    if (v1 == 0 && v2 == 0 && v3 == 0) return 0;
    if (v1 == 0 && v2 == 1 && v3 == 0) return 1;
    if (v1 == 0 && v2 == 2 && v3 == 0) return 2;
    if (v1 == 1 && v2 == 0 && v3 == 0) return 3;
    if (v1 == 0 && v2 == 0 && v3 == 1) return 4;
    return 5;
}

oh_hf_diagram::oh_hf_diagram(const std::string &data_path, const std::string &name, double mass, double spin, int &n_l,
                             int verbosity)
    : energy_diagram(name, mass) {
    mol_spin = spin;
    const std::string fname = data_path + "spectroscopy/levels_oh_hf.txt";
    std::ifstream input = open_or_throw(fname, "oh_hf_diagram");
    skip(input, 3);
    int i_max;
    input >> i_max;
    int nb = 0;
    while (nb < n_l && nb < i_max) {   // spectroscopy.cpp:580-598
        int v, parity, hf;
        double j, omega, energy;
        input >> v >> j >> omega >> parity >> hf >> energy;
        energy_level level;
        level.v = v;
        level.j = j;
        level.k1 = omega;
        level.syminv = parity;
        level.hf = hf;
        level.energy = energy;
        level.spin = spin;
        level.g = 2 * hf + 1;
        level.nb = nb;
        lev_array.push_back(level);
        nb++;
    }
    check_stream(input, fname, "oh_hf_diagram");
    nb_lev = n_l = (int)lev_array.size();
    report(verbosity, "OH (hyperfine) levels", fname);
}

int oh_hf_diagram::get_nb(int parity, int v, double j, double omega, double hf) const {
    for (int i = 0; i < nb_lev; i++)
        if (lev_array[i].v == v && rounding(2. * lev_array[i].j) == rounding(2. * j) &&
            rounding(2. * lev_array[i].k1) == rounding(2. * omega) && rounding(2. * lev_array[i].hf) == rounding(2. * hf) &&
            lev_array[i].syminv == parity)
            return i;
    return -1;
}

// ---- radiative rates ------------------------------------------------------------------
ch3oh_einstein_coeff::ch3oh_einstein_coeff(const std::string &path, const energy_diagram *di, int verbosity)
    : einstein_coeff(di) {
    const std::string fname =
        path + (rounding(2. * di->mol_spin) == 3 ? "spectroscopy/radiative_ch3oh_a.txt" : "spectroscopy/radiative_ch3oh_e.txt");
    std::ifstream input = open_or_throw(fname, "ch3oh_einstein_coeff");
    skip(input, 4);
    int i_max;
    input >> i_max;
    for (int i = 0; i < i_max; i++) {   // spectroscopy.cpp:893-923
        char ch;
        int v, j, k;
        double a, energy, line_strength;
        input.get(ch);   // the end of the previous line
        input.get(ch);
        input >> v >> j >> k;
        input.get(ch);   // '+' / '-' for A species, ' ' for E
        if (ch == '-') k = -k;
        const int up = di->get_nb(v, j, k);
        input >> v >> j >> k;
        input.get(ch);
        if (ch == '-') k = -k;
        const int low = di->get_nb(v, j, k);
        input >> energy >> a >> line_strength;
        for (int l = 0; l < 6; l++) input >> a;
        if (low != -1 && up != -1) {
            energy = di->lev_array[up].energy - di->lev_array[low].energy;
            arr[up][low] = 64. * line_strength * DEBYE * DEBYE * M_PI * std::pow(M_PI * energy, 3.) /
                           (3. * PLANCK_CONSTANT * (2. * di->lev_array[up].j + 1.));
            arr[low][up] = di->lev_array[up].g * arr[up][low] / ((double)di->lev_array[low].g);
        }
    }
    check_stream(input, fname, "ch3oh_einstein_coeff");
    report(verbosity, "CH3OH radiative rates", fname);
}

h2o_einstein_coeff::h2o_einstein_coeff(const std::string &path, const h2o_diagram *di, int verbosity)
    : einstein_coeff(di) {
    const std::string fname =
        path + (di->isotop == 1 ? "spectroscopy/radiative_h2o16.txt" : "spectroscopy/radiative_h2o18.txt");
    std::ifstream input = open_or_throw(fname, "h2o_einstein_coeff");
    skip(input, 2);
    int i_max;
    input >> i_max;
    for (int i = 0; i < i_max; i++) {   // spectroscopy.cpp:840-858
        int v1, v2, v3, j, ka, kc;
        double coeff, energy;
        input >> v1 >> v2 >> v3 >> j >> ka >> kc;
        const int up = di->get_nb(di->get_vibr_nb(v1, v2, v3), j, ka - kc);
        input >> v1 >> v2 >> v3 >> j >> ka >> kc;
        const int low = di->get_nb(di->get_vibr_nb(v1, v2, v3), j, ka - kc);
        input >> coeff >> energy;
        if (low != -1 && up != -1) {
            arr[up][low] = coeff;
            arr[low][up] = di->lev_array[up].g * coeff / ((double)di->lev_array[low].g);
        }
    }
    check_stream(input, fname, "h2o_einstein_coeff");
    report(verbosity, "H2O radiative rates", fname);
}

oh_hf_einstein_coeff::oh_hf_einstein_coeff(const std::string &path, const energy_diagram *di, int verbosity)
    : einstein_coeff(di) {
    const std::string fname = path + "spectroscopy/radiative_oh_hf.txt";
    std::ifstream input = open_or_throw(fname, "oh_hf_einstein_coeff");
    skip(input, 2);
    int i_max;
    input >> i_max;
    for (int i = 0; i < i_max; i++) {   // spectroscopy.cpp:1111-1126
        int v, parity;
        double j, omega, hf, coeff, energy;
        input >> v >> j >> omega >> parity >> hf;
        const int up = di->get_nb(parity, v, j, omega, hf);
        input >> v >> j >> omega >> parity >> hf;
        const int low = di->get_nb(parity, v, j, omega, hf);
        input >> coeff >> energy;
        if (low != -1 && up != -1) {
            arr[up][low] = coeff;
            arr[low][up] = di->lev_array[up].g * coeff / ((double)di->lev_array[low].g);
        }
    }
    check_stream(input, fname, "oh_hf_einstein_coeff");
    report(verbosity, "OH (hyperfine) radiative rates", fname);
}

// ---- CH3OH collision tables -------------------------------------------------------------
ch3oh_he_coll_data::ch3oh_he_coll_data(const std::string &path, const energy_diagram *lev, int verbosity,
                                       int file_levels, int file_levels_rovibr) {
    allocate(lev->nb_lev, 41);   // 40 temperatures + T = 0 K (coll_rates_ch3oh.cpp:40)
    for (int i = 0; i < jmax; i++) tgrid[i] = i * 10.;
    species = LVG_SP_HE;
    const char sp = ch3oh_species(lev);
    std::vector<int> nb_arr;
    for (int vt = 0; vt <= NB_VIBR_EXCIT_CH3OH_RABLI; vt++) {   // :55-136
        const std::string fname = path + "coll_ch3oh/coll_ch3oh_" + sp + std::to_string(vt) + "_he.txt";
        std::ifstream input = open_or_throw(fname, "ch3oh_he_coll_data");
        skip(input, 4);
        ch3oh_level_table(input, lev, file_levels, vt, false, nb_arr);
        ch3oh_rate_blocks(input, *this, lev, 21, nb_arr, false);
        check_stream(input, fname, "ch3oh_he_coll_data");
        report(verbosity, "CH3OH-He rates", fname);
    }
    // above 200 K: the 200 K value (USE_TEMPER_EXTRAP_CH3OH off; :138-145)
    for (int i = 0; i < imax; i++)
        for (int j = 21; j < jmax; j++)
            coeff[i][j] = USE_TEMPER_EXTRAP_CH3OH ? coeff[i][20] * std::sqrt(tgrid[j] / tgrid[20]) : coeff[i][20];
    // rovibrational data over the full grid; same-vt entries with initial > final in
    // the file replace the earlier data (:147-222)
    const std::string fname = path + "coll_ch3oh/coll_ch3oh_" + sp + "_he_rovibr.txt";
    std::ifstream input = open_or_throw(fname, "ch3oh_he_coll_data");
    skip(input, 4);
    ch3oh_level_table(input, lev, file_levels_rovibr, 0, true, nb_arr);
    ch3oh_rate_blocks(input, *this, lev, jmax, nb_arr, true);
    check_stream(input, fname, "ch3oh_he_coll_data");
    report(verbosity, "CH3OH-He rovibrational rates", fname);
}

ch3oh_ph2_coll_data::ch3oh_ph2_coll_data(const std::string &path, const energy_diagram *lev, int verbosity,
                                         int file_levels) {
    allocate(lev->nb_lev, 21);   // coll_rates_ch3oh.cpp:242
    species = LVG_SP_PH2;
    const char sp = ch3oh_species(lev);
    std::vector<int> nb_arr;
    for (int vt = 0; vt <= NB_VIBR_EXCIT_CH3OH_RABLI; vt++) {   // :256-330
        const std::string fname = path + "coll_ch3oh/coll_ch3oh_" + sp + std::to_string(vt) + "_ph2.txt";
        std::ifstream input = open_or_throw(fname, "ch3oh_ph2_coll_data");
        skip(input, 4);
        ch3oh_level_table(input, lev, file_levels, vt, false, nb_arr);
        ch3oh_rate_blocks(input, *this, lev, jmax, nb_arr, false);
        check_stream(input, fname, "ch3oh_ph2_coll_data");
        report(verbosity, "CH3OH-pH2 rates", fname);
    }
}

ch3oh_oh2_coll_data::ch3oh_oh2_coll_data(const std::string &path, const energy_diagram *lev, int verbosity,
                                         int file_levels) {
    allocate(lev->nb_lev, 21);   // coll_rates_ch3oh.cpp:352
    species = LVG_SP_OH2;
    const std::string fname = path + "coll_ch3oh/coll_ch3oh_" + ch3oh_species(lev) + "0_oh2.txt";
    std::ifstream input = open_or_throw(fname, "ch3oh_oh2_coll_data");
    skip(input, 4);
    std::vector<int> nb_arr;
    ch3oh_level_table(input, lev, file_levels, 0, false, nb_arr);   // vt = 0 only (:389)
    ch3oh_rate_blocks(input, *this, lev, jmax, nb_arr, false);
    check_stream(input, fname, "ch3oh_oh2_coll_data");
    report(verbosity, "CH3OH-oH2 rates", fname);
}

ch3oh_collisions::ch3oh_collisions(const std::string &path, const energy_diagram *lev, int verbosity, int file_levels,
                                   int file_levels_rovibr, int file_levels_oh2) {
    add_neutral(new ch3oh_he_coll_data(path, lev, verbosity, file_levels, file_levels_rovibr));   // :452-455
    add_neutral(new ch3oh_ph2_coll_data(path, lev, verbosity, file_levels));
    add_neutral(new ch3oh_oh2_coll_data(path, lev, verbosity, file_levels_oh2));
    nb_lev = lev->nb_lev;
}

// ---- H2O collision tables ----------------------------------------------------------------
namespace {
const char *h2o_spin(const energy_diagram *di) { return rounding(di->mol_spin) == 0 ? "ph2o" : "oh2o"; }

// 45-level tables, one line per packed pair: "l li lf" (or "li lf x x") then the rates
// (coll_rates_h2o.cpp:58-69, :458-467)
void h2o_packed(collision_data &c, std::istream &in, int nb_lines, bool four_labels) {
    for (int i = 0; i < nb_lines && i < c.imax; i++) {
        int a, b, d;
        in >> a >> b >> d;
        if (four_labels) in >> d;
        for (int j = 1; j < c.jmax; j++) in >> c.coeff[i][j];
    }
}

// lines labelled by (v J tau) of both levels; unknown levels are skipped (:160-180)
void h2o_labelled(collision_data &c, std::istream &in, int nb_lines, const energy_diagram *di) {
    for (int line = 0; line < nb_lines; line++) {
        int v1, j1, tau1, v2, j2, tau2;
        in >> v1 >> j1 >> tau1 >> v2 >> j2 >> tau2;
        const int up = di->get_nb(v1, j1, tau1), low = di->get_nb(v2, j2, tau2);
        double val;
        if (low != -1 && up != -1) {
            const int i = up * (up - 1) / 2 + low;
            for (int j = 1; j < c.jmax; j++) in >> c.coeff[i][j];
        } else {
            for (int j = 1; j < c.jmax; j++) in >> val;
        }
    }
}
}  // namespace

h2o_oh2_coll_data::h2o_oh2_coll_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(45, 9);   // coll_rates_h2o.cpp:35-37
    species = LVG_SP_OH2;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_oh2.txt";
    std::ifstream in = open_or_throw(fname, "h2o_oh2_coll_data");
    skip(in, 1);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_packed(*this, in, nb_lines, false);
    check_stream(in, fname, "h2o_oh2_coll_data");
    report(verbosity, "H2O-oH2 rates", fname);
}

h2o_ph2_coll_data::h2o_ph2_coll_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(45, 9);   // coll_rates_h2o.cpp:87-89
    species = LVG_SP_PH2;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_ph2.txt";
    std::ifstream in = open_or_throw(fname, "h2o_ph2_coll_data");
    skip(in, 1);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_packed(*this, in, nb_lines, false);
    check_stream(in, fname, "h2o_ph2_coll_data");
    report(verbosity, "H2O-pH2 rates", fname);
}

h2o_h2_coll_rovibr_data::h2o_h2_coll_rovibr_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(di->nb_lev, 12);   // coll_rates_h2o.cpp:141-145
    species = LVG_SP_PH2;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_h2_rovibr.txt";
    std::ifstream in = open_or_throw(fname, "h2o_h2_coll_rovibr_data");
    skip(in, 2);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_labelled(*this, in, nb_lines, di);
    check_stream(in, fname, "h2o_h2_coll_rovibr_data");
    report(verbosity, "H2O-H2 rovibrational rates", fname);
}

h2o_he_coll_data::h2o_he_coll_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(45, 11);   // coll_rates_h2o.cpp:212-215
    species = LVG_SP_HE;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_he.txt";
    std::ifstream in = open_or_throw(fname, "h2o_he_coll_data");
    skip(in, 1);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    // both directions of every pair: row li*(nb_lev-1) + lf' (lf' skips li itself)
    std::vector<double> temp((size_t)2 * imax * jmax, 0.);
    for (int i = 0; i < nb_lines && i < 2 * imax; i++) {
        int li, lf, f;
        in >> li >> lf >> f >> f;
        for (int j = 1; j < jmax; j++) in >> temp[(size_t)i * jmax + j];
    }
    for (int li = 1; li < nb_lev; li++)   // :247-262
        for (int lf = 0; lf < li; lf++) {
            const int i = li * (nb_lev - 1) + lf, f = lf * (nb_lev - 1) + li - 1, nb = li * (li - 1) / 2 + lf;
            if (li < di->nb_lev)
                for (int j = 1; j < jmax; j++)
                    coeff[nb][j] = 0.5 * (temp[(size_t)i * jmax + j] +
                                          temp[(size_t)f * jmax + j] * di->lev_array[lf].g / ((double)di->lev_array[li].g) *
                                              std::exp((di->lev_array[li].energy - di->lev_array[lf].energy) *
                                                       CM_INVERSE_TO_KELVINS / tgrid[j]));
        }
    check_stream(in, fname, "h2o_he_coll_data");
    report(verbosity, "H2O-He rates", fname);
}

h2o_he_coll_rovibr_data::h2o_he_coll_rovibr_data(const std::string &path, const energy_diagram *di, bool is_scaled,
                                                 int verbosity) {
    const std::string fname =
        path + "coll_h2o/coll_" + h2o_spin(di) + (is_scaled ? "_he_rovibr_scaled.txt" : "_he_rovibr.txt");
    std::ifstream in = open_or_throw(fname, "h2o_he_coll_rovibr_data");
    skip(in, 1);
    int nb_lines, jm;
    in >> nb_lines >> jm;   // coll_rates_h2o.cpp:309-311
    if (!in || jm < 1) throw lvg_error(LVG_E_ARG, "h2o_he_coll_rovibr_data: bad header in " + fname);
    allocate(di->nb_lev, jm + 1);
    species = LVG_SP_HE;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_labelled(*this, in, nb_lines, di);
    check_stream(in, fname, "h2o_he_coll_rovibr_data");
    report(verbosity, "H2O-He rovibrational rates", fname);
}

h2o_e_coll_rovibr_data::h2o_e_coll_rovibr_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(di->nb_lev, 12);   // coll_rates_h2o.cpp:366-370
    species = LVG_SP_E;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_e_rovibr.txt";
    std::ifstream in = open_or_throw(fname, "h2o_e_coll_rovibr_data");
    skip(in, 2);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_labelled(*this, in, nb_lines, di);
    check_stream(in, fname, "h2o_e_coll_rovibr_data");
    report(verbosity, "H2O-e rovibrational rates", fname);
}

h2o_h_coll_data::h2o_h_coll_data(const std::string &path, const energy_diagram *di, int verbosity) {
    allocate(45, 15);   // coll_rates_h2o.cpp:436-438
    species = LVG_SP_H;
    const std::string fname = path + "coll_h2o/coll_" + h2o_spin(di) + "_h.txt";
    std::ifstream in = open_or_throw(fname, "h2o_h_coll_data");
    skip(in, 2);
    int nb_lines;
    in >> nb_lines;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    h2o_packed(*this, in, nb_lines, true);
    check_stream(in, fname, "h2o_h_coll_data");
    report(verbosity, "H2O-H rates", fname);
}

h2o_collisions::h2o_collisions(const std::string &path, const energy_diagram *di, bool he_is_scaled, int verbosity) {
    // coll_rates_h2o.cpp:494-503: order fixes the rule's table slots
    add_neutral(new h2o_he_coll_data(path, di, verbosity));
    add_neutral(new h2o_he_coll_rovibr_data(path, di, he_is_scaled, verbosity));
    add_neutral(new h2o_ph2_coll_data(path, di, verbosity));
    add_neutral(new h2o_oh2_coll_data(path, di, verbosity));
    add_neutral(new h2o_h2_coll_rovibr_data(path, di, verbosity));
    add_neutral(new h2o_h_coll_data(path, di, verbosity));
    add_electron(new h2o_e_coll_rovibr_data(path, di, verbosity));
    nb_lev = di->nb_lev;
}

// ---- OH hyperfine collision tables -----------------------------------------------------------
oh_hf_h2_coll_data::oh_hf_h2_coll_data(const std::string &path, const energy_diagram *, bool ortho, int verbosity) {
    const std::string fname = path + (ortho ? "coll_oh/coll_oh_hf_oh2.txt" : "coll_oh/coll_oh_hf_ph2.txt");
    std::ifstream in = open_or_throw(fname, "oh_hf_h2_coll_data");
    skip(in, 3);
    int nb, jm;
    in >> nb >> jm;   // coll_rates_oh.cpp:148-150
    if (!in || nb < 2 || jm < 1) throw lvg_error(LVG_E_ARG, "oh_hf_h2_coll_data: bad header in " + fname);
    allocate(nb, jm + 1);
    species = ortho ? LVG_SP_OH2 : LVG_SP_PH2;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    for (int i = 0; i < imax; i++) {
        int j, li, lf;
        in >> j >> li >> lf;
        const int n = (li - 2) * (li - 1) / 2 + lf - 1;   // levels numbered from 1 in the file
        if (n < 0 || n >= imax) throw lvg_error(LVG_E_ARG, "oh_hf_h2_coll_data: bad level pair in " + fname);
        for (j = 1; j < jmax; j++) in >> coeff[n][j];
    }
    check_stream(in, fname, "oh_hf_h2_coll_data");
    report(verbosity, "OH-H2 (hyperfine) rates", fname);
}

oh_hf_h2_ext_coll_data::oh_hf_h2_ext_coll_data(const std::string &path, const energy_diagram *, bool ortho,
                                               int verbosity) {
    const std::string fname = path + (ortho ? "coll_oh/coll_oh_hf_oh2_ext.txt" : "coll_oh/coll_oh_hf_ph2_ext.txt");
    std::ifstream in = open_or_throw(fname, "oh_hf_h2_ext_coll_data");
    skip(in, 3);
    int nb, jm;
    in >> nb >> jm;   // coll_rates_oh.cpp:202-204
    if (!in || nb < 2 || jm < 1) throw lvg_error(LVG_E_ARG, "oh_hf_h2_ext_coll_data: bad header in " + fname);
    allocate(nb, jm + 1);
    species = ortho ? LVG_SP_OH2 : LVG_SP_PH2;
    for (int j = 1; j < jmax; j++) {   // one block per temperature, every ordered pair listed (:215-226)
        in >> tgrid[j];
        for (int i = 0; i < imax + nb_lev; i++) {
            int li, lf;
            double a;
            in >> li >> lf;
            if (li > lf) {
                const int n = (li - 2) * (li - 1) / 2 + lf - 1;
                if (n < 0 || n >= imax) throw lvg_error(LVG_E_ARG, "oh_hf_h2_ext_coll_data: bad level pair in " + fname);
                in >> coeff[n][j];
            } else {
                in >> a;
            }
        }
    }
    check_stream(in, fname, "oh_hf_h2_ext_coll_data");
    report(verbosity, "OH-H2 (hyperfine, extended) rates", fname);
}

oh_hf_he_coll_data::oh_hf_he_coll_data(const std::string &path, const energy_diagram *, int verbosity) {
    const std::string fname = path + "coll_oh/coll_oh_hf_he.txt";
    std::ifstream in = open_or_throw(fname, "oh_hf_he_coll_data");
    skip(in, 3);
    int nb, jm;
    in >> nb >> jm;   // coll_rates_oh.cpp:256-258
    if (!in || nb < 2 || jm < 1) throw lvg_error(LVG_E_ARG, "oh_hf_he_coll_data: bad header in " + fname);
    allocate(nb, jm + 1);
    species = LVG_SP_HE;
    for (int j = 1; j < jmax; j++) in >> tgrid[j];
    for (int i = 0; i < imax; i++) {
        int li, lf, j;
        in >> li >> lf >> j >> j;
        const int n = (li - 2) * (li - 1) / 2 + lf - 1;
        if (n < 0 || n >= imax) throw lvg_error(LVG_E_ARG, "oh_hf_he_coll_data: bad level pair in " + fname);
        for (j = 1; j < jmax; j++) in >> coeff[n][j];
    }
    check_stream(in, fname, "oh_hf_he_coll_data");
    report(verbosity, "OH-He (hyperfine) rates", fname);
}

oh_hf_collisions::oh_hf_collisions(const std::string &path, const energy_diagram *di, int verbosity) {
    add_neutral(new oh_hf_he_coll_data(path, di, verbosity));   // coll_rates_oh.cpp:358-366
    if (USE_EXTENDED_OH_HF_H2_DATA) {
        add_neutral(new oh_hf_h2_ext_coll_data(path, di, false, verbosity));
        add_neutral(new oh_hf_h2_ext_coll_data(path, di, true, verbosity));
    } else {
        add_neutral(new oh_hf_h2_coll_data(path, di, false, verbosity));
        add_neutral(new oh_hf_h2_coll_data(path, di, true, verbosity));
    }
    nb_lev = di->nb_lev;
}

// ---- cloud profiles ------------------------------------------------------------------------
namespace {
// next line that is not a comment ('!' or '#'); false at the end (an empty line)
bool data_line(std::istream &in, std::string &s) {
    do {
        if (!std::getline(in, s)) { s.clear(); break; }
    } while (!s.empty() && (s[0] == '!' || s[0] == '#'));
    return !s.empty();
}
}  // namespace

bool set_physical_parameters(const std::string &data_path, cloud_data *cloud) {
    cloud->delete_layers();
    std::ifstream in1(data_path + "sim_phys_param.txt"), in2(data_path + "sim_data_h2_chemistry.txt"),
        in3(data_path + "sim_specimen_abund.txt"), in4(data_path + "sim_dust_data.txt");
    if (!in1 || !in2 || !in3 || !in4) return false;
    std::string s;
    std::istringstream ss;
    while (!in1.eof() && !in2.eof() && !in3.eof() && !in4.eof()) {   // cloud_data.cpp:269-345
        cloud_layer c;
        double a, z, h2, td, abund;
        if (!data_line(in1, s)) break;
        ss.clear();
        ss.str(s);
        // the second of the two velocity gradients (instantaneous, from the MHD equations)
        ss >> c.zl >> a >> c.temp_n >> a >> c.temp_el >> c.vel_n >> a >> c.tot_h_conc >> a >> c.el_conc >> a >> a >>
            c.velg_n;
        c.el_conc *= c.tot_h_conc;
        if (!data_line(in2, s)) break;
        ss.clear();
        ss.str(s);
        ss >> z >> c.h2_opr;
        if (!data_line(in3, s)) break;
        ss.clear();
        ss.str(s);
        ss >> z >> c.h_conc >> h2 >> c.he_conc;
        h2 *= c.tot_h_conc;
        c.ph2_conc = h2 / (1. + c.h2_opr);
        c.oh2_conc = h2 - c.ph2_conc;
        c.he_conc *= c.tot_h_conc;
        c.h_conc *= c.tot_h_conc;
        if (!data_line(in4, s)) break;
        ss.clear();
        ss.str(s);
        ss >> z;
        while (!ss.eof()) {   // per component: temperature, abundance, 14 more columns
            ss >> td >> abund;
            for (int j = 0; j < 14; j++) ss >> a;
            c.dust_grain_temp.push_back(td);
            c.dust_grain_conc.push_back(abund * c.tot_h_conc);
        }
        if (c.dust_grain_temp.empty()) return false;
        c.av_temp_d = c.dust_grain_temp.back();   // the last group is the average / total
        c.dust_grain_temp.pop_back();
        c.dust_grain_conc.pop_back();
        cloud->add_layer(c);
    }
    if (cloud->nb_lay < 2) return false;
    // layer values: averages of the adjacent points (cloud_data.cpp:352-380)
    for (int i = 0; i < cloud->nb_lay - 1; i++) {
        cloud_layer &c = cloud->lay_array[i];
        const cloud_layer &n = cloud->lay_array[i + 1];
        c.zu = n.zl;
        c.dz = c.zu - c.zl;
        c.zm = c.zl + 0.5 * c.dz;
        c.temp_n = 0.5 * (c.temp_n + n.temp_n);
        c.temp_el = 0.5 * (c.temp_el + n.temp_el);
        c.av_temp_d = 0.5 * (c.av_temp_d + n.av_temp_d);
        c.vel_n = 0.5 * (c.vel_n + n.vel_n);
        c.velg_n = 0.5 * (c.velg_n + n.velg_n);
        c.tot_h_conc = 0.5 * (c.tot_h_conc + n.tot_h_conc);
        c.he_conc = 0.5 * (c.he_conc + n.he_conc);
        c.h_conc = 0.5 * (c.h_conc + n.h_conc);
        c.oh2_conc = 0.5 * (c.oh2_conc + n.oh2_conc);
        c.ph2_conc = 0.5 * (c.ph2_conc + n.ph2_conc);
        c.el_conc = 0.5 * (c.el_conc + n.el_conc);
        c.mol_conc = 0.5 * (c.mol_conc + n.mol_conc);
        c.h2_opr = 0.5 * (c.h2_opr + n.h2_opr);
        c.vel_turb = 0.5 * (c.vel_turb + n.vel_turb);
        for (size_t j = 0; j < c.dust_grain_temp.size(); j++)
            c.dust_grain_temp[j] = 0.5 * (c.dust_grain_temp[j] + n.dust_grain_temp[j]);
        for (size_t j = 0; j < c.dust_grain_conc.size(); j++)
            c.dust_grain_conc[j] = 0.5 * (c.dust_grain_conc[j] + n.dust_grain_conc[j]);
    }
    cloud->remove_layer(cloud->nb_lay - 1);
    for (auto &c : cloud->lay_array)   // :385-392
        if (std::fabs(c.velg_n) < MIN_VELOCITY_GRADIENT) c.velg_n = c.velg_n > 0. ? MIN_VELOCITY_GRADIENT : -MIN_VELOCITY_GRADIENT;
    return true;
}

bool set_molecular_conc(const std::string &data_path, const std::string &mol_name, cloud_data *cloud, double f) {
    std::ifstream in1(data_path + "sim_specimen_abund.txt"), in2(data_path + "sim_phys_param.txt");
    if (!in1 || !in2) return false;
    std::string s, str;
    std::istringstream ss;
    std::vector<double> z_vect, conc_vect;
    std::getline(in1, s);
    std::getline(in1, s);
    ss.str(s);       // the line with the species names (cloud_data.cpp:419-427)
    ss >> str;       // the first word labels the depth column
    int mol_nb = 1;
    while (ss >> str) {
        if (str == mol_name) break;
        mol_nb++;
    }
    while (!in1.eof() && !in2.eof()) {   // :429-454
        double a;
        if (!std::getline(in1, s) || s.empty()) break;
        ss.clear();
        ss.str(s);
        ss >> a;
        z_vect.push_back(a);
        for (int j = 0; j < mol_nb; j++) ss >> a;
        conc_vect.push_back(a);
        if (!data_line(in2, s)) break;
        ss.clear();
        ss.str(s);
        for (int j = 0; j < 8; j++) ss >> a;
        conc_vect.back() *= a;   // times the H nuclei concentration
    }
    if (z_vect.size() < 2) return false;
    const int nz = (int)z_vect.size();
    for (auto &c : cloud->lay_array) {   // column density over [zl, zu] (:458-476)
        int j, k;
        for (j = 0; j < nz - 1 && z_vect[j] < c.zl; j++) {}
        for (k = j; k < nz - 1 && z_vect[k] < c.zu; k++) {}
        c.mol_conc = 0.;
        if (j > 0 && z_vect[j] > c.zl)
            c.mol_conc += 0.5 * (z_vect[j] - c.zl) *
                          (conc_vect[j] + conc_vect[j - 1] +
                           (conc_vect[j] - conc_vect[j - 1]) * (c.zl - z_vect[j - 1]) / (z_vect[j] - z_vect[j - 1]));
        for (; j < k; j++) c.mol_conc += 0.5 * (z_vect[j + 1] - z_vect[j]) * (conc_vect[j] + conc_vect[j + 1]);
        if (k > 0 && z_vect[k] > c.zu)
            c.mol_conc -= 0.5 * (z_vect[k] - c.zu) *
                          (conc_vect[k] + conc_vect[k - 1] +
                           (conc_vect[k] - conc_vect[k - 1]) * (c.zu - z_vect[k - 1]) / (z_vect[k] - z_vect[k - 1]));
        c.mol_conc *= f / (c.zu - c.zl);
    }
    return true;
}

void join_layers(cloud_data *cloud, int nb) {   // cloud_data.cpp:143-222
    if (nb < 1) throw lvg_error(LVG_E_ARG, "join_layers: nb must be >= 1");
    std::vector<double> x(nb);
    auto &L = cloud->lay_array;
    for (int i = 0; i < nb * (cloud->nb_lay / nb); i += nb) {
        double a = 0.;
        for (int j = 0; j < nb; j++) {
            x[j] = L[i + j].dz;
            a += x[j];
        }
        for (int j = 0; j < nb; j++) x[j] /= a;
        cloud_layer &c = L[i];
        c.zu = L[i + nb - 1].zu;
        c.dz = c.zu - c.zl;
        c.zm = c.zl + 0.5 * c.dz;
        double *fields[] = {&c.temp_n, &c.temp_el, &c.av_temp_d, &c.vel_n, &c.velg_n, &c.tot_h_conc, &c.he_conc,
                            &c.h_conc, &c.oh2_conc, &c.ph2_conc, &c.el_conc, &c.mol_conc, &c.h2_opr, &c.vel_turb};
        for (double *p : fields) *p *= x[0];
        for (auto &v : c.dust_grain_temp) v *= x[0];
        for (auto &v : c.dust_grain_conc) v *= x[0];
        for (int j = 1; j < nb; j++) {
            const cloud_layer &o = L[i + j];
            const double *ofields[] = {&o.temp_n, &o.temp_el, &o.av_temp_d, &o.vel_n, &o.velg_n, &o.tot_h_conc,
                                       &o.he_conc, &o.h_conc, &o.oh2_conc, &o.ph2_conc, &o.el_conc, &o.mol_conc,
                                       &o.h2_opr, &o.vel_turb};
            for (int f = 0; f < 14; f++) *fields[f] += *ofields[f] * x[j];
            for (size_t l = 0; l < c.dust_grain_temp.size(); l++) c.dust_grain_temp[l] += o.dust_grain_temp[l] * x[j];
            for (size_t l = 0; l < c.dust_grain_conc.size(); l++) c.dust_grain_conc[l] += o.dust_grain_conc[l] * x[j];
        }
    }
    const int l = cloud->nb_lay / nb;
    for (int i = 0; i < l; i++)
        for (int j = 1; j < nb; j++) cloud->remove_layer(i + 1);
    while (cloud->nb_lay > l) cloud->remove_layer(l);
}

cloud_geometry geometry_of(const cloud_data &cloud) {
    cloud_geometry g;
    for (const auto &c : cloud.lay_array) {
        g.dz.push_back(c.dz);
        g.vel_n.push_back(c.vel_n);
    }
    g.height = cloud.nb_lay ? cloud.get_height() : 0.;
    return g;
}

}  // namespace lvgamd
