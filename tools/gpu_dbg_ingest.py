"""Debug: ingested CH3OH (N=60) GPU vs oracle, wave vs block kernel."""
import os, sys, tempfile
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np
import ingest_problem as IP
from oracle import oracle
from radiative_transfer_amd import abi
from radiative_transfer_amd.native import LvgSolver
d = tempfile.mkdtemp() + "/"; out = tempfile.mkdtemp() + "/"
got = IP.write_and_ingest(d, out, "/root/repo/tests/cpp/_build/test_ingest")["got"]
L = IP.layers(got)
P = IP.problem(got, "ch3oh", abi.LVG_COLL_CH3OH, "CH3OHa", 32.0, 1.5, L.dust_conc.shape[1])
opts = abi.default_opts(allow_plain_retry=0)
po, so = oracle.solve_layers(P, L, opts)
for force in (None, "1"):
    if force: os.environ["LVG_BLOCK_KERNEL"] = force
    s = LvgSolver(P)
    pg, sg = s.solve_layers(L, opts)
    print("force_block", force, "iters", sg["iterations"], so["iterations"])
    print("  gpu", pg[0, :6], "\n  ora", po[0, :6], "\n  sum", pg[0].sum(), po[0].sum())
    bg = s.boundary_layer_populations(L); bo = oracle.boundary_layer_populations(P, L)
    print("  boundary equal", np.array_equal(bg, bo), "gpu", bg[0, :4], "ora", bo[0, :4])
    Mg, dfg, pgn, eg = s.debug_calc_new_pop(L, 0, bo[0], 0)
    Mo, dfo, pon, eo = oracle.calc_new_pop(P, L, 0, bo[0], 0)
    print("  M equal", np.array_equal(Mg, Mo), "df equal", np.array_equal(dfg, dfo), "p equal", np.array_equal(pgn, pon))
    if not np.array_equal(Mg, Mo):
        bad = np.argwhere(Mg != Mo); print("  M diffs", len(bad), bad[:5].tolist(), Mg[tuple(bad[0])], Mo[tuple(bad[0])])
    s.close()
print("v", P.mol.v[:10], "j", P.mol.j[:10], "g", P.mol.g[:10])
