"""End to end: files in the reference's input formats -> the C++
readers (host/lvg_ingest.cpp, through tests/cpp/test_ingest) -> lvg_create -> a GPU solve
of the ingested C-shock cloud -> bit-exact against the oracle on the same arrays.
CH3OH-A (60 levels, 3 tables), p-H2O (45 levels, 6 tables + e-), OH hyperfine (20
levels, plain and line-overlap scheme). Rates the files do not list get a floor of
1e-13 cm^3/s (ingest_problem.collisions) so that no level is isolated: an isolated
level makes the rate matrix singular and both sides would agree on NaN only. The
molecular concentrations are also scaled up 1e3 so that the lines matter (more
iterations). Parity unpinned as the readers are: the reference ships no data files."""
import os

import numpy as np
import pytest

import ingest_problem as IP
from oracle import oracle
from parity_helpers import assert_same
from radiative_transfer_amd import abi
from radiative_transfer_amd.native import LvgSolver

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "test_ingest")


@pytest.fixture(scope="module")
def ingested(tmp_path_factory):
    assert os.path.exists(EXE), "tests/cpp/_build/test_ingest missing: run __graft_entry__.build() first"
    d = str(tmp_path_factory.mktemp("data")) + "/"
    out = str(tmp_path_factory.mktemp("out")) + "/"
    return IP.write_and_ingest(d, out, EXE)["got"]


MOLS = [("ch3oh", abi.LVG_COLL_CH3OH, "CH3OHa", 32.0, 1.5, {"allow_plain_retry": 0}),
        ("h2o", abi.LVG_COLL_H2O, "pH2O", 18.0, 0.0, {}),
        ("oh", abi.LVG_COLL_OH_HF, "OH", 17.0, 0.5, {"acceleration": 0}),
        ("oh", abi.LVG_COLL_OH_HF, "OH", 17.0, 0.5, {"acceleration": 0, "line_overlap": 1})]


@pytest.mark.parametrize("prefix,rule,name,mass,spin,kw", MOLS, ids=["ch3oh", "h2o", "oh", "oh_overlap"])
@pytest.mark.parametrize("scale", [1.0, 1e3])
def test_ingested_cloud_solve(ingested, prefix, rule, name, mass, spin, kw, scale):
    for cloud in ("cloud", "joined"):
        L = IP.layers(ingested, cloud)
        L.mol_conc *= scale
        P = IP.problem(ingested, prefix, rule, name, mass, spin, L.dust_conc.shape[1],
                       overlap=kw.get("line_overlap", 0), floor=1e-13)
        opts = abi.default_opts(**kw)
        s = LvgSolver(P)
        pg, sg = s.solve_layers(L, opts)
        po, so = oracle.solve_layers(P, L, opts)
        assert np.all(np.isfinite(po))         # (one CH3OH layer at 1e3 hits the 150-iteration cap: q3)
        assert_same(pg, sg, po, so)
        s.close()
