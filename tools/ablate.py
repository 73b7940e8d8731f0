"""Timing ablations (diagnostic): per-LU kernel time of library variants built with
-DLVG_ABL=k on CH3OH-A 256 x 4096 layers with exactly 4 iterations per layer
(min_error = 1e-300, max_iter_acc = 4), so every variant factors the same number of matrices."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, ROOT)
    from radiative_transfer_amd import abi, synth
    from radiative_transfer_amd.native import LvgSolver
    P, L, o = synth.make_problem("ch3oha256_4096")
    s = LvgSolver(P)
    opts = abi.default_opts(**{**o, "min_error": 1e-300, "max_iter_acc": 4, "allow_plain_retry": 0})
    s.solve_layers(L, opts)
    best = 1e30
    for _ in range(3):
        _, st = s.solve_layers(L, opts)
        ms, _ = s.last_kernel_time()
        best = min(best, ms)
    lus = int(st["iterations"].sum()) + L.nb_lay
    print(json.dumps({"lib": os.environ.get("LVG_LIB_PATH"), "kernel_ms": best, "lus": lus,
                      "us_per_lu_per_slot": best * 1e3 / lus * 512}))
    sys.exit(0)
for v in sys.argv[1:] or ["0", "1", "2", "3", "4"]:
    env = dict(os.environ, LVG_LIB_PATH=os.path.join(ROOT, "radiative_transfer_amd", "_lib", f"liblvg_amd_v{v}.so"))
    r = subprocess.run([sys.executable, __file__, "--one"], env=env, capture_output=True, text=True, timeout=600)
    print(f"v{v}", r.stdout.strip() or r.stderr[-500:], flush=True)
