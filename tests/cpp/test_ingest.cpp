// Ingest dump (tests/ infrastructure): reads a directory written in the reference's
// input formats with the readers of radiative_transfer_amd/host/lvg_ingest.hpp and
// dumps every resulting array as raw little-endian binary plus a manifest line
// "name dtype count" per array, for tests/test_ingest_cpu.py to compare. No GPU.
// usage: test_ingest <data_dir/> <out_dir/> <ch3oh_n_l> <ch3oh_ang_mom_max> <file_lev> <file_lev_rovibr> <file_lev_oh2>
//                    <h2o_n_l> <oh_n_l> <join_nb>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "../../radiative_transfer_amd/host/lvg_ingest.hpp"

using namespace lvgamd;

static std::string out_dir;
static std::ofstream manifest;

static void dump(const std::string &name, const double *p, size_t n) {
    std::ofstream f(out_dir + name + ".bin", std::ios::binary);
    f.write(reinterpret_cast<const char *>(p), n * sizeof(double));
    manifest << name << " f8 " << n << "\n";
}
static void dump(const std::string &name, const std::vector<double> &v) { dump(name, v.data(), v.size()); }
static void dump_i(const std::string &name, const std::vector<int> &v) {
    std::ofstream f(out_dir + name + ".bin", std::ios::binary);
    f.write(reinterpret_cast<const char *>(v.data()), v.size() * sizeof(int));
    manifest << name << " i4 " << v.size() << "\n";
}

static void dump_diagram(const std::string &p, const energy_diagram &d) {
    std::vector<double> e, j, k1, k2, hf;
    std::vector<int> g, v, sy;
    for (const auto &l : d.lev_array) {
        e.push_back(l.energy); j.push_back(l.j); k1.push_back(l.k1); k2.push_back(l.k2); hf.push_back(l.hf);
        g.push_back(l.g); v.push_back(l.v); sy.push_back(l.syminv);
    }
    dump(p + "_energy", e); dump(p + "_j", j); dump(p + "_k1", k1); dump(p + "_k2", k2); dump(p + "_hf", hf);
    dump_i(p + "_g", g); dump_i(p + "_v", v); dump_i(p + "_syminv", sy);
}

static void dump_coll(const std::string &p, const collisional_transitions &c) {
    std::vector<int> meta = {c.nb1, c.nb2, (int)c.coll_data.size()};
    dump_i(p + "_meta", meta);
    for (size_t t = 0; t < c.coll_data.size(); t++) {
        const collision_data *d = c.coll_data[t];
        const std::string q = p + "_t" + std::to_string(t);
        dump(q + "_tgrid", d->tgrid);
        dump(q + "_coeff", d->data(), (size_t)d->imax * d->jmax);
        dump_i(q + "_shape", std::vector<int>{d->nb_lev, d->imax, d->jmax, d->species});
    }
}

int main(int argc, char **argv) {
    if (argc < 11) { std::fprintf(stderr, "usage: see source\n"); return 2; }
    const std::string dir = argv[1];
    out_dir = argv[2];
    manifest.open(out_dir + "manifest.txt");
    try {
        int n_l = std::atoi(argv[3]);
        ch3oh_diagram ch(dir, "CH3OHa", 32. * 1.66053906660e-24, 1.5, n_l, 2, std::atoi(argv[4]));
        dump_diagram("ch3oh", ch);
        ch3oh_einstein_coeff che(dir, &ch);
        dump("ch3oh_einst", che.data(), (size_t)ch.nb_lev * ch.nb_lev);
        ch3oh_collisions chc(dir, &ch, 0, std::atoi(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]));
        dump_coll("ch3oh", chc);

        int n_w = std::atoi(argv[8]);
        h2o_diagram hw(dir, "pH2O", 18. * 1.66053906660e-24, 0., 1, n_w);
        dump_diagram("h2o", hw);
        h2o_einstein_coeff hwe(dir, &hw);
        dump("h2o_einst", hwe.data(), (size_t)hw.nb_lev * hw.nb_lev);
        h2o_collisions hwc(dir, &hw, false);
        dump_coll("h2o", hwc);

        int n_o = std::atoi(argv[9]);
        oh_hf_diagram oh(dir, "OH", 17. * 1.66053906660e-24, 0.5, n_o);
        dump_diagram("oh", oh);
        oh_hf_einstein_coeff ohe(dir, &oh);
        dump("oh_einst", ohe.data(), (size_t)oh.nb_lev * oh.nb_lev);
        oh_hf_collisions ohc(dir, &oh);
        dump_coll("oh", ohc);

        cloud_data cl;
        if (!set_physical_parameters(dir, &cl)) { std::printf("set_physical_parameters failed\n"); return 1; }
        if (!set_molecular_conc(dir, "CH3OH", &cl, 0.5)) { std::printf("set_molecular_conc failed\n"); return 1; }
        auto dump_cloud = [&](const std::string &p, const cloud_data &c) {
            std::vector<double> f[20];
            std::vector<double> dt, dc;
            for (const auto &l : c.lay_array) {
                const double vals[20] = {l.zl, l.zu, l.dz, l.zm, l.temp_n, l.temp_el, l.av_temp_d, l.vel_n, l.velg_n,
                                         l.tot_h_conc, l.he_conc, l.h_conc, l.oh2_conc, l.ph2_conc, l.el_conc,
                                         l.mol_conc, l.h2_opr, l.vel_turb, (double)l.dust_grain_temp.size(),
                                         (double)l.dust_grain_conc.size()};
                for (int i = 0; i < 20; i++) f[i].push_back(vals[i]);
                dt.insert(dt.end(), l.dust_grain_temp.begin(), l.dust_grain_temp.end());
                dc.insert(dc.end(), l.dust_grain_conc.begin(), l.dust_grain_conc.end());
            }
            std::vector<double> all;
            for (auto &v : f) all.insert(all.end(), v.begin(), v.end());
            dump(p + "_fields", all);
            dump(p + "_dust_temp", dt);
            dump(p + "_dust_conc", dc);
            const cloud_geometry g = geometry_of(c);
            dump(p + "_height", &g.height, 1);
        };
        dump_cloud("cloud", cl);
        join_layers(&cl, std::atoi(argv[10]));
        dump_cloud("joined", cl);
    } catch (const lvg_error &e) {
        std::printf("lvg_error %d: %s\n", e.code, e.what());
        return 1;
    }
    manifest.close();
    std::printf("INGEST OK\n");
    return 0;
}
