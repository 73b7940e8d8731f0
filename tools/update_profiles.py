"""Copy a tools/profile.sh run (gpurun_out/prof_<tag>_<workload>/) into
profiles/<tag>/<workload>/ and refresh profiles/pmc_traffic.json (HBM bytes per launch of
the solve kernel — lvg::solve_kernel, or lvg::solve_wave_kernel<NM> for N <= 64 — for bench.py).
FETCH_SIZE is doubled on gfx950 (MI355X_MICROARCH.md §HBM); WRITE_SIZE is taken as is."""
import csv, glob, json, os, shutil, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
workload = sys.argv[2] if len(sys.argv) > 2 else "ch3oha256_4096"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{workload}")
dst = os.path.join(ROOT, "profiles", tag, workload)
KERNELS = ("lvg::solve_kernel", "lvg_wide::solve_kernel", "lvg_big::solve_kernel", "solve_wave_kernel")
os.makedirs(dst, exist_ok=True)


def one(pattern):
    f = glob.glob(os.path.join(src, pattern), recursive=True)
    if not f:
        sys.exit(f"missing {pattern} under {src}")
    return f[0]


shutil.copy(one("trace/**/*kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
per = {}
for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    f = one(f"{kind}/**/*counter_collection.csv")
    rows = [r for r in csv.DictReader(open(f)) if any(k in r["Kernel_Name"] for k in KERNELS)]
    with open(os.path.join(dst, f"pmc_{kind}_solve_kernel.csv"), "w", newline="") as fo:
        w = csv.DictWriter(fo, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    by = {}
    for r in rows:
        by[r["Dispatch_Id"]] = by.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    per[counter] = sum(by.values()) / len(by)
    per[counter + "_launches"] = len(by)
bj = json.load(open(os.path.join(src, "bench_trace.json")))
shutil.copy(os.path.join(src, "bench_trace.json"), os.path.join(dst, "bench_trace.json"))
shutil.copy(os.path.join(ROOT, "tools", "profile.sh"), os.path.join(dst, "profile_command.sh"))
hbm = (2.0 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0
p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
data = json.load(open(p)) if os.path.exists(p) else {}
data[workload] = {
    "round": tag, "kernel": bj["roofline"]["kernel"], "launches_measured": per["FETCH_SIZE_launches"],
    "FETCH_SIZE_kB_per_launch": per["FETCH_SIZE"], "WRITE_SIZE_kB_per_launch": per["WRITE_SIZE"],
    "hbm_bytes_per_launch": hbm,
    "correction": "MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 1/2 of the bytes of wide coalesced reads on gfx950 -> doubled; WRITE_SIZE taken as is; bytes = kB*1024",
    "units_per_launch": bj["config"]["layer_iterations_per_step"],
    "source": f"profiles/{tag}/{workload}/pmc_fetch_solve_kernel.csv, pmc_write_solve_kernel.csv (rocprofv3 --pmc, separate passes)",
    "commit": open(os.path.join(ROOT, ".commit")).read().strip() if os.path.exists(os.path.join(ROOT, ".commit")) else "?",
}
json.dump(data, open(p, "w"), indent=1)
print(json.dumps(data[workload], indent=1))
