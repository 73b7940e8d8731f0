"""Input-file readers (radiative_transfer_amd/host/lvg_ingest.cpp):
molecular levels, radiative rates and collision tables of CH3OH-A, p-H2O and OH
(hyperfine), and the C-shock cloud profile files with set_molecular_conc and
join_layers.

A seeded synthetic data directory is written in the reference's formats
(tests/ingest_files.py), read by the C++ readers (tests/cpp/test_ingest.cpp dumps every
array), and compared bit for bit with oracle/ingest.py, which derives the same arrays
from the values written. The files exercise the readers' quirks: CH3OH rates written
as "a.b-dfg" (dropped) or negative (clipped), levels listed in a file but absent from
the diagram, the rovibrational CH3OH-He data overriding same-vt entries, H2O-He rates
given in both directions, OH tables in shuffled pair order, comment lines, velocity
gradients below MIN_VELOCITY_GRADIENT. Parity unpinned: the reference ships no data
files, so the formats are read off its parsing code.
"""
import os
import subprocess

import numpy as np
import pytest

import ingest_files as W
import ingest_problem as IP
from oracle import ingest as O
from ingest_problem import (CH3OH_NL, ANG_MAX, FILE_LEV, FILE_LEV_ROVIBR, FILE_LEV_OH2, H2O_NL, OH_NL,
                            JOIN_NB)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "test_ingest")



def _build():
    from radiative_transfer_amd import build
    build.build_host()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])


@pytest.fixture(scope="module")
def ingest(tmp_path_factory):
    _build()
    d = str(tmp_path_factory.mktemp("data")) + "/"
    out = str(tmp_path_factory.mktemp("out")) + "/"
    return IP.write_and_ingest(d, out, EXE)


def _check_diagram(got, prefix, di):
    exp = di.arrays()
    for k, v in exp.items():
        np.testing.assert_array_equal(got[f"{prefix}_{k}"], v, err_msg=f"{prefix}_{k}")


def _check_coll(got, prefix, exp):
    nb1, nb2, nt = got[f"{prefix}_meta"]
    assert (nb1, nb2, nt) == (exp["nb1"], exp["nb2"], len(exp["tables"]))
    for t, (tg, c, sp, nlev) in enumerate(exp["tables"]):
        q = f"{prefix}_t{t}"
        nb_lev, imax, jmax, species = got[q + "_shape"]
        assert (nb_lev, imax, jmax, species) == (nlev, c.shape[0], c.shape[1], sp), q
        np.testing.assert_array_equal(got[q + "_tgrid"], tg, err_msg=q)
        np.testing.assert_array_equal(got[q + "_coeff"].reshape(imax, jmax), c, err_msg=q)


def test_ch3oh_levels(ingest):
    di = ingest["ch"]
    assert di.n == CH3OH_NL
    _check_diagram(ingest["got"], "ch3oh", di)
    # sorted by energy, J cut, A species g = 4 (2J + 1)
    assert np.all(np.diff(di.e) > 0) and max(l["j"] for l in di.lev) <= ANG_MAX


def test_ch3oh_einstein(ingest):
    di = ingest["ch"]
    exp = O.ch3oh_einstein(di, ingest["ch_lines"])
    assert np.count_nonzero(exp) > 10
    np.testing.assert_array_equal(ingest["got"]["ch3oh_einst"].reshape(di.n, di.n), exp)


def test_ch3oh_collisions(ingest):
    exp = O.ch3oh_collisions(ingest["ch"], ingest["truth"]["ch3oh_coll"])
    assert all(np.count_nonzero(c) > 0 for _, c, _, _ in exp["tables"])
    _check_coll(ingest["got"], "ch3oh", exp)


def test_h2o(ingest):
    di = ingest["hw"]
    _check_diagram(ingest["got"], "h2o", di)
    np.testing.assert_array_equal(ingest["got"]["h2o_einst"].reshape(di.n, di.n), O.h2o_einstein(di, ingest["h_lines"]))
    _check_coll(ingest["got"], "h2o", O.h2o_collisions(di, ingest["truth"]["h2o_coll"]))


def test_oh_hyperfine(ingest):
    di = ingest["oh"]
    _check_diagram(ingest["got"], "oh", di)
    exp = O.oh_einstein(di, ingest["o_lines"])
    assert np.count_nonzero(exp) > 0
    np.testing.assert_array_equal(ingest["got"]["oh_einst"].reshape(di.n, di.n), exp)
    _check_coll(ingest["got"], "oh", O.oh_collisions(24, ingest["truth"]["oh_coll"]))


def test_cloud_profiles(ingest):
    t = ingest["truth"]["cloud"]
    lays = O.set_molecular_conc(O.set_physical_parameters(t), t, "CH3OH", 0.5)
    got = ingest["got"]
    for prefix, L in (("cloud", lays), ("joined", O.join_layers(lays, JOIN_NB))):
        fields, dt, dc, height = O.cloud_arrays(L)
        np.testing.assert_array_equal(got[prefix + "_fields"], fields, err_msg=prefix)
        np.testing.assert_array_equal(got[prefix + "_dust_temp"], dt, err_msg=prefix)
        np.testing.assert_array_equal(got[prefix + "_dust_conc"], dc, err_msg=prefix)
        assert got[prefix + "_height"][0] == height
    # the clamp of small velocity gradients (cloud_data.cpp:385-392)
    assert np.all(np.abs([c["velg_n"] for c in lays]) >= O.MIN_VELOCITY_GRADIENT)
    assert len(O.join_layers(lays, JOIN_NB)) == len(lays) // JOIN_NB


def test_missing_file_is_an_error(tmp_path):
    """A missing file raises lvg_error (the reference prints and exits)."""
    _build()
    out = str(tmp_path) + "/"
    r = subprocess.run([EXE, str(tmp_path) + "/nowhere/", out, "10", "5", "4", "4", "4", "10", "10", "2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "lvg_error" in r.stdout, (r.stdout, r.stderr)
