// C++ host-facade test (tests/ infrastructure): drives the reference-shaped class
// surface of radiative_transfer_amd/host/lvg_host.hpp on the GPU and checks every
// result bit for bit against the CPU oracle fed the identical lvg_problem.
// Exit codes: 0 all equal, 1 mismatch, 3 no usable device (lvg_create failed).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../oracle/lvg_oracle.h"
#include "../../radiative_transfer_amd/host/lvg_host.hpp"

using namespace lvgamd;

static int failures = 0;
static void expect_equal(const char *what, const double *a, const double *b, size_t n) {
    size_t bad = 0;
    for (size_t i = 0; i < n; i++)
        if (std::memcmp(&a[i], &b[i], sizeof(double)) != 0) bad++;
    std::printf("%-44s %s (%zu/%zu differ)\n", what, bad ? "MISMATCH" : "equal", bad, n);
    if (bad) failures++;
}

// deterministic pseudo-random in [0,1)
static double urand(unsigned &s) { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0 / 16777216.0); }

int main(int argc, char **argv) {
    const std::string tmp = argc > 1 ? argv[1] : "/tmp/";
    const int N = 20;
    unsigned seed = 12345;
    // ---- molecule: a rotational ladder (synthetic)
    energy_diagram di("TESTMOL", 17. * 1.66053906660e-24);
    for (int i = 0; i < N; i++) {
        energy_level l;
        l.nb = i; l.j = i; l.g = 2 * i + 1; l.v = 0;
        l.energy = 0.9 * i * (i + 1) + 0.05 * i;
        di.add_level(l);
    }
    einstein_coeff ei(&di);
    for (int u = 1; u < N; u++)
        for (int l = 0; l < u; l++)
            if (u - l <= 2) {
                const double de = di.lev_array[u].energy - di.lev_array[l].energy;
                ei.set_line(u, l, 3e-7 * de * de * de * (0.1 + 0.9 * urand(seed)) * 1e-3, &di);
            }
    // ---- collisions: two neutral tables (He, pH2) and one electron table
    collisional_transitions co;
    const std::vector<double> tg = {0., 10., 20., 50., 100., 200., 500., 1000.};
    auto table = [&](int species, double scale) {
        auto *d = new collision_data(N, tg);
        d->species = species;
        for (int f = 1; f < N; f++)
            for (int s = 0; s < f; s++) {
                const double de = di.lev_array[f].energy - di.lev_array[s].energy;
                for (int t = 0; t < d->jmax; t++)
                    d->coeff[f * (f - 1) / 2 + s][t] =
                        (t == 0) ? 0. : scale * std::sqrt(1. + tg[t] / 100.) * std::exp(-de / 100.) * (0.5 + urand(seed));
            }
        return d;
    };
    co.add_neutral(table(LVG_SP_HE, 1e-11));
    co.add_neutral(table(LVG_SP_PH2, 2e-11));
    co.add_electron(table(LVG_SP_E, 1e-7));
    // ---- dust: one component
    dust_model dust;
    {
        std::vector<double> en, ab;
        for (int k = 0; k < 40; k++) { en.push_back(std::pow(10., -1. + 0.1 * k)); ab.push_back(1e-10 * std::pow(en.back(), 1.5)); }
        dust.add_component(new dust_component(en, ab, 2.));
    }
    // ---- LVG table: build, save in the reference format, load back (loader test)
    std::vector<double> gam, del, p;
    for (int i = 0; i < 41; i++) gam.push_back(std::pow(10., -6. + 0.3 * i));
    for (int k = 0; k < 25; k++) del.push_back(std::pow(10., -4. + 0.5 * k));
    for (int k = 0; k < 25; k++)
        for (int i = 0; i < 41; i++) {
            const double tau = 1. / gam[i];
            p.push_back((1. - (1. - std::exp(-tau)) / tau) * del[k] / (1. + del[k]));
        }
    lvg_method_data mem(del, gam, p);
    mem.save(tmp, "lvg_test_table.txt");
    lvg_method_data esc(tmp, "lvg_test_table.txt");
    expect_equal("lvg_method_data save/load round trip (gamma)", esc.gamma_arr.data(), mem.gamma_arr.data(), gam.size());
    expect_equal("lvg_method_data save/load round trip (p)", esc.p.data(), mem.p.data(), p.size());
    // ---- cloud
    cloud_data cloud;
    for (int l = 0; l < 6; l++) {
        cloud_layer c;
        c.temp_n = c.temp_el = 30. + 60. * l;
        const double nh2 = std::pow(10., 4. + 0.7 * l);
        c.oh2_conc = 0.75 * nh2; c.ph2_conc = 0.25 * nh2; c.he_conc = 0.18 * nh2; c.h_conc = 1e-3 * nh2;
        c.el_conc = 1e-7 * nh2; c.mol_conc = 1e-7 * nh2; c.vel_turb = 3e4; c.velg_n = (l % 2 ? -1. : 1.) * 1e-9;
        c.dust_grain_conc = {2.46e-11 * nh2};
        c.dust_grain_temp = {20.};
        cloud.add_layer(c);
    }
    // ---- scheme on the device
    iteration_scheme_lvg scheme(&dust, &esc);
    try {
        scheme.init_molecule_data(&di, &ei, &co);
    } catch (const lvg_error &e) {
        std::printf("NO_DEVICE: %s\n", e.what());
        return e.code == LVG_E_DEVICE ? 3 : 1;
    }
    const lvg_problem &P = scheme.problem();
    layer_pack lp(cloud, 1);
    // 1. calc_molecular_populations, warm chain (the reference default) and independent starts
    for (int mode = 0; mode < 2; mode++) {
        std::vector<double> pg((size_t)cloud.nb_lay * N, 0.), po((size_t)cloud.nb_lay * N, 0.);
        std::vector<lvg_layer_status> sg, so(cloud.nb_lay);
        calc_molecular_populations(&cloud, &scheme, &di, &ei, &co, pg.data(), N, true, 0,
                                   mode ? init_policy::boundary_layer : init_policy::warm_chain, &sg);
        lvg_solve_opts o;
        lvg_solve_opts_default(&o);
        o.init = mode ? LVG_INIT_BOUNDARY_LAYER : LVG_INIT_WARM_CHAIN;
        oracle_solve_layers(&P, &lp.view, po.data(), &o, so.data(), 1);
        expect_equal(mode ? "calc_molecular_populations (boundary starts)" : "calc_molecular_populations (warm chain)",
                     pg.data(), po.data(), pg.size());
        int it_bad = 0;
        for (int l = 0; l < cloud.nb_lay; l++) it_bad += sg[l].iterations != so[l].iterations;
        std::printf("%-44s %s\n", "  iteration counts", it_bad ? "MISMATCH" : "equal");
        failures += it_bad != 0;
    }
    // 2. boundary_layer_populations, calc_new_pop and iteration_control on layer 3
    const cloud_layer &c3 = cloud.lay_array[3];
    scheme.set_vel_grad(c3.velg_n);
    scheme.set_dust_parameters(c3.dust_grain_conc, c3.dust_grain_temp);
    scheme.set_parameters(c3.temp_n, c3.temp_el, c3.el_conc, c3.h_conc, c3.ph2_conc, c3.oh2_conc, c3.he_conc,
                          c3.mol_conc, c3.vel_turb);
    std::vector<double> b0(N), bo((size_t)cloud.nb_lay * N);
    boundary_layer_populations(&scheme, b0.data(), c3.temp_n, c3.temp_el, c3.el_conc, c3.h_conc, c3.ph2_conc,
                               c3.oh2_conc, c3.he_conc);
    oracle_boundary_layer_populations(&P, &lp.view, bo.data());
    expect_equal("boundary_layer_populations", b0.data(), bo.data() + 3 * N, N);
    std::vector<double> n1(N), n1o(N);
    double e1, e1o;
    scheme.calc_new_pop(b0.data(), n1.data(), e1);
    oracle_calc_new_pop(&P, &lp.view, 3, b0.data(), 0, nullptr, nullptr, n1o.data(), &e1o);
    expect_equal("iteration_scheme_lvg::calc_new_pop", n1.data(), n1o.data(), N);
    expect_equal("  eq_error", &e1, &e1o, 1);
    iteration_control<iteration_scheme_lvg> ctl(&scheme);
    std::vector<double> pc(b0), pco(b0);
    const bool found = ctl.calculate_populations(pc.data(), 150, 1e-5, true);
    lvg_solve_opts o;
    lvg_solve_opts_default(&o);
    o.init = LVG_INIT_GIVEN;
    o.allow_plain_retry = 0;
    lvg_layer_status so{};
    std::vector<cloud_layer> one{c3};
    layer_pack l1(one, 1);
    oracle_solve_layers(&P, &l1.view, pco.data(), &o, &so, 1);
    expect_equal("iteration_control::calculate_populations", pc.data(), pco.data(), N);
    std::printf("%-44s %s (found %d, iterations %d/%d)\n", "  status", (found == (so.converged != 0) &&
                ctl.iter_nb == so.iterations) ? "equal" : "MISMATCH", (int)found, ctl.iter_nb, so.iterations);
    failures += !(found == (so.converged != 0) && ctl.iter_nb == so.iterations);
    // 3. populations on disk (spectroscopy.cpp:1294-1368): 6 significant digits
    {
        std::vector<double> pg((size_t)cloud.nb_lay * N, 0.), back((size_t)cloud.nb_lay * N, 0.);
        calc_molecular_populations(&cloud, &scheme, &di, &ei, &co, pg.data(), N, true, 0, init_policy::boundary_layer);
        const std::string f = save_populations(tmp, &di, pg.data(), cloud.nb_lay, N, false, "_test");
        read_populations(f, back.data(), cloud.nb_lay, N);
        double worst = 0.;
        for (size_t i = 0; i < pg.size(); i++) worst = std::max(worst, std::fabs(back[i] - pg[i]) / std::fabs(pg[i]));
        std::printf("%-44s %s (max rel %.1e)\n", "save_populations / read_populations", worst < 5e-6 ? "equal" : "MISMATCH", worst);
        failures += !(worst < 5e-6);
        // 4. transition_data_container::find and lim_luminosity_lvg vs the oracle
        cloud_geometry geo;
        for (int l = 0; l < cloud.nb_lay; l++) { geo.dz.push_back(3e16); geo.vel_n.push_back(2e6 * (1. - l / 6.)); }
        geo.height = 3e16 * cloud.nb_lay;
        transition_data_container tc(&cloud, &geo, &scheme);
        tc.min_optical_depth = 0.;
        tc.find(pg.data(), 0.);
        lim_luminosity_lvg(&scheme, &tc, &cloud, pg.data());
        lvg_cloud_geometry g{geo.dz.data(), geo.vel_n.data(), geo.height};
        lvg_find_opts fo;
        oracle_find_opts_default(&fo);
        fo.rel_error = 0.; fo.min_optical_depth = 0.;
        std::vector<lvg_transition> ro(256);
        int nro = 0;
        oracle_find_transitions(&P, &lp.view, &g, pg.data(), &fo, 256, &nro, ro.data(), nullptr, nullptr, nullptr);
        int bad = nro != (int)tc.data.size();
        std::vector<int> up, low;
        for (int k = 0; !bad && k < nro; k++) {
            bad += ro[k].up != tc.data[k].up || ro[k].low != tc.data[k].low ||
                   std::memcmp(&ro[k].tau_max, &tc.data[k].tau_max, sizeof(double)) != 0;
            up.push_back(ro[k].up); low.push_back(ro[k].low);
        }
        std::printf("%-44s %s (%d transitions)\n", "transition_data_container::find", bad ? "MISMATCH" : "equal", nro);
        failures += bad != 0;
        if (!bad && nro > 0) {
            std::vector<double> lum(nro);
            oracle_lim_luminosity(&P, &lp.view, &g, pg.data(), nro, up.data(), low.data(), 0, lum.data(), nullptr,
                                  nullptr, nullptr, nullptr, nullptr);
            std::vector<double> lg(nro);
            for (int k = 0; k < nro; k++) lg[k] = tc.data[k].lum;
            expect_equal("lim_luminosity_lvg (lum)", lg.data(), lum.data(), nro);
        }
    }
    // 5. the same cloud over several devices behind one scheme (set_devices: lvg_create_devices;
    //    on a one-GPU box the device list repeats device 0, each block with its own stream)
    {
        iteration_scheme_lvg multi(&dust, &esc);
        multi.set_devices({0, 0, 0});
        multi.init_molecule_data(&di, &ei, &co);
        std::vector<double> pm((size_t)cloud.nb_lay * N, 0.), po((size_t)cloud.nb_lay * N, 0.);
        std::vector<lvg_layer_status> so(cloud.nb_lay);
        const std::vector<int> bad = calc_molecular_populations(&cloud, &multi, &di, &ei, &co, pm.data(), N, true, 0,
                                                                init_policy::boundary_layer);
        lvg_solve_opts o;
        lvg_solve_opts_default(&o);
        oracle_solve_layers(&P, &lp.view, po.data(), &o, so.data(), 1);
        std::printf("%-44s %d devices\n", "set_devices({0, 0, 0})", multi.nb_devices());
        failures += multi.nb_devices() != 3;
        expect_equal("calc_molecular_populations (3 devices)", pm.data(), po.data(), pm.size());
    }
    std::printf(failures ? "FAILED\n" : "ALL EQUAL\n");
    return failures ? 1 : 0;
}
