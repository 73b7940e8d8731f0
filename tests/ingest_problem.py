"""A seeded data directory in the reference's input formats, read by the C++ readers
(host/lvg_ingest.cpp via tests/cpp/test_ingest), turned into solver inputs
(test infrastructure: tests/test_ingest_cpu.py checks the arrays, tests/test_gpu_ingest.py
solves the ingested molecules on the GPU against the oracle)."""
import os
import subprocess

import numpy as np

import ingest_files as W
from oracle import ingest as O
from radiative_transfer_amd import abi, synth

CH3OH_NL, ANG_MAX = 60, 8
FILE_LEV, FILE_LEV_ROVIBR, FILE_LEV_OH2 = 40, 30, 25
H2O_NL, OH_NL, JOIN_NB = 45, 20, 3
AMU = 1.66053906660e-24


def _load(out):
    arrs = {}
    with open(os.path.join(out, "manifest.txt")) as f:
        for line in f:
            name, dt, n = line.split()
            a = np.fromfile(os.path.join(out, name + ".bin"), dtype=np.float64 if dt == "f8" else np.int32)
            assert a.size == int(n), name
            arrs[name] = a
    return arrs


def write_and_ingest(d, out, exe):
    """Write the data set into d, run the reader dump into out; return the arrays and truths."""
    rng = np.random.default_rng(2024)
    truth = {}
    # CH3OH-A
    blocks = W.ch3oh_levels_truth(rng)
    W.write_ch3oh_levels(d, blocks)
    ch = O.ch3oh_diagram(blocks, 1.5, CH3OH_NL, 2, ANG_MAX)
    alev = W.a_levels(blocks, nb_vibr=2, ang_mom_max=10)        # a pool wider than the diagram
    pool = [(v, J, K) for v, J, K, _ in alev]
    inside = [(l["v"], int(l["j"]), int(l["k1"])) for l in ch.lev]
    lines = []
    for q in range(300):
        src = inside if q % 4 else pool          # mostly levels of the diagram, some absent
        a, b = rng.choice(len(src), 2, replace=False)
        lines.append(src[a] + src[b] + (float(rng.uniform(0.1, 5.0)),))
    W.write_ch3oh_radiative(d, lines)
    truth["ch3oh_coll"] = W.write_ch3oh_coll(d, rng, pool, FILE_LEV, FILE_LEV_ROVIBR, FILE_LEV_OH2)
    # p-H2O
    rows = W.h2o_levels_truth(rng)
    W.write_h2o_levels(d, rows)
    hw = O.h2o_diagram(rows, 0., H2O_NL)
    hlines = []
    for _ in range(200):
        a, b = rng.choice(len(rows), 2, replace=False)
        hlines.append((rows[a][:6], rows[b][:6], float(rng.uniform(1e-6, 1e-2))))
    W.write_h2o_radiative(d, hlines)
    truth["h2o_coll"] = W.write_h2o_coll(d, rng, [O.h2o_label(hw, i) for i in range(hw.n)])
    # OH hyperfine
    orows = W.oh_levels_truth(rng, 24)
    W.write_oh_levels(d, orows)
    oh = O.oh_diagram(orows, OH_NL)
    olines = []
    for _ in range(60):
        a, b = rng.choice(len(orows), 2, replace=False)
        olines.append((orows[a][:5], orows[b][:5], float(rng.uniform(1e-11, 1e-9))))
    W.write_oh_radiative(d, olines)
    truth["oh_coll"] = W.write_oh_coll(d, rng, 24)
    # cloud
    truth["cloud"] = W.write_cloud(d, rng)
    r = subprocess.run([exe, d, out, str(CH3OH_NL), str(ANG_MAX), str(FILE_LEV), str(FILE_LEV_ROVIBR),
                        str(FILE_LEV_OH2), str(H2O_NL), str(OH_NL), str(JOIN_NB)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "INGEST OK" in r.stdout, (r.stdout, r.stderr)
    return dict(got=_load(out), truth=truth, ch=ch, ch_lines=lines, hw=hw, h_lines=hlines, oh=oh, o_lines=olines)




def molecule(got, prefix, name, mass_amu, spin):
    n = got[prefix + "_energy"].size
    return abi.Molecule(name=name, mass=mass_amu * AMU, energy=got[prefix + "_energy"].copy(),
                        g=got[prefix + "_g"].astype(np.int32), einst=got[prefix + "_einst"].reshape(n, n).copy(),
                        v=got[prefix + "_v"].astype(np.int32), j=got[prefix + "_j"].copy(), spin=spin)


def collisions(got, prefix, rule, floor=None):
    """The ingested tables; with `floor`, zero rates at T > 0 (pairs the files do not
    list, or whose entries the readers dropped) become `floor` cm^3/s, so that no level
    is isolated — an isolated level makes the rate matrix singular (NaN on both sides)."""
    nb1, nb2, nt = (int(x) for x in got[prefix + "_meta"])
    tabs = []
    for t in range(nt):
        q = f"{prefix}_t{t}"
        nb_lev, imax, jmax, species = (int(x) for x in got[q + "_shape"])
        coeff = got[q + "_coeff"].reshape(imax, jmax).copy()
        if floor is not None:
            coeff[:, 1:] = np.where(coeff[:, 1:] == 0., floor, coeff[:, 1:])
        tabs.append(abi.CollTable(nb_lev=nb_lev, tgrid=got[q + "_tgrid"].copy(), coeff=coeff, species=species))
    return abi.Collisions(rule=rule, neutral=tabs[:nb1], electron=tabs[nb1:nb1 + nb2])


def layers(got, prefix="cloud"):
    """The ingested cloud (set_physical_parameters + set_molecular_conc) as solver layers;
    the dust concentrations per layer are the cloud's dust components."""
    F = O.FIELDS
    nl = got[prefix + "_fields"].size // (len(F) + 2)
    f = got[prefix + "_fields"].reshape(len(F) + 2, nl)
    col = lambda name: f[F.index(name)].copy()
    ndc = f[len(F) + 1].astype(int)
    assert np.all(ndc == ndc[0])
    dc = got[prefix + "_dust_conc"].reshape(nl, ndc[0]).copy()
    return abi.Layers(temp_n=col("temp_n"), temp_el=col("temp_el"), el_conc=col("el_conc"), h_conc=col("h_conc"),
                      ph2_conc=col("ph2_conc"), oh2_conc=col("oh2_conc"), he_conc=col("he_conc"),
                      mol_conc=col("mol_conc"), vel_turb=col("vel_turb"), vel_grad=col("velg_n"), dust_conc=dc)


def problem(got, prefix, rule, name, mass_amu, spin, nb_comp, overlap=False, floor=None):
    dust = synth.dust_components()
    dust = [dust[c % len(dust)] for c in range(nb_comp)]
    ov1 = ov2 = None
    if overlap:
        ov1, ov2 = synth.overlap_tables()
    return abi.Problem(mol=molecule(got, prefix, name, mass_amu, spin), coll=collisions(got, prefix, rule, floor),
                       dust=dust, esc=synth.esc_table(), overlap1=ov1, overlap2=ov2)
