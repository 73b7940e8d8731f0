"""Diagnostic behind DESIGN.md §5's per-choice table: each reference-arithmetic choice of the
oracle undone alone (oracle.solve_layers(..., ref="exp" | "lu" | "pow" | "all")) and a control
with no arithmetic change (n_mol x (1 + 2^-52)), on the refarith.SAMPLES subset of a config.
usage: python tools/refarith_per_choice.py [config]   (tests/test_oracle_refarith_cpu.py asserts it)"""
import os, json, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle, refarith
from radiative_transfer_amd import abi, synth
name = sys.argv[1] if len(sys.argv) > 1 else "ph2o45_1024"
prob, L, o = synth.make_problem(name)
nb = refarith.SAMPLES[name]
idx = np.unique(np.linspace(0, L.nb_lay - 1, min(nb, L.nb_lay)).round().astype(int))
L = L.subset(idx)
opts = abi.default_opts(**o)
pe, se = oracle.solve_layers(prob, L, opts)
for ref in ["exp", "lu", "pow", "all"]:
    t = time.time()
    pr, sr = oracle.solve_layers(prob, L, opts, ref=ref)
    acc = (se["iterations"] >= opts.accel_start) | (sr["iterations"] >= opts.accel_start)
    d = refarith.rel_dev(pe, pr).max(axis=1)
    same = se["iterations"] == sr["iterations"]
    print(name, ref, json.dumps(dict(layers=int(L.nb_lay), ng_layers=int(acc.sum()), iter_diff=int((~same).sum()),
          max_plain=float(d[~acc].max()) if (~acc).any() else 0., max_ng=float(d[acc].max()) if acc.any() else 0.,
          max_pm1=float(d[~same].max()) if (~same).any() else 0., max_same=float(d[same].max()) if same.any() else 0.,
          bitident_layers=int((d == 0).sum()), over_2e5=int((d > 2e-5).sum()), secs=round(time.time()-t,1))))
# control: no arithmetic change, the molecule density moved by one ulp (1 + 2^-52)
import copy
L2 = L.subset(np.arange(L.nb_lay)); L2.mol_conc = L2.mol_conc * (1 + 2.0**-52)
pp, sp = oracle.solve_layers(prob, L2, opts)
d = refarith.rel_dev(pe, pp).max(axis=1)
acc = (se["iterations"] >= opts.accel_start) | (sp["iterations"] >= opts.accel_start)
print(name, "ulp", json.dumps(dict(iter_diff=int((se["iterations"]!=sp["iterations"]).sum()), max_plain=float(d[~acc].max()) if (~acc).any() else 0., max_ng=float(d[acc].max()) if acc.any() else 0., over_2e5=int((d>2e-5).sum()))))
print("accel_start", opts.accel_start, "iters max", se["iterations"].max())
