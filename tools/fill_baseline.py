"""Fill BASELINE.md §4's results row from the committed benchmark outputs (run after a
bench/profile round; the table is not edited by hand): profiles/<TAG>/<workload>/bench_line.json,
profiles/pmc_traffic.json, profiles/<TAG>/refarith.json and, when present, the newest
SCALE_rNN.json with driver-measured values."""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


TAG = "r3"


def main():
    b = json.load(open(os.path.join(ROOT, "profiles", TAG, "ch3oha256_4096", "bench_line.json")))
    ra = {r["config"]: r for r in json.load(open(os.path.join(ROOT, "profiles", TAG, "refarith.json")))}
    cb = b["cpu_baseline"]
    roof = b["roofline"]
    scale = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "SCALE_r*.json"))):   # the newest file with values wins
        got = {}
        try:
            for line in json.load(open(f)).get("runs", []):
                p = line.get("parsed") or {}
                if p.get("n_gpus"):
                    got[int(p["n_gpus"])] = p["value"]
        except Exception:
            pass
        if got:
            scale = got
    gbs = roof["traffic"] / (roof["kernel_ms"] * 1e-3) / 1e9 if roof.get("traffic") else None
    k = lambda v: f"{v / 1e3:.1f} K" if v is not None else "—"
    r = ra["ch3oha256_4096"]
    row = (f"| CH3OH-A-256 × 4096 | {k(cb['one_thread']['value'])} | {k(cb['value'])} (n={cb['cores']} of "
           f"{cb['host']['nproc']}) | {k(b['value'])} | {k(scale.get(2))} | {k(scale.get(4))} | {k(scale.get(8))} | "
           f"{roof['achieved']:.2f} TFLOP/s = {roof['frac']:.3f} of FP64 | "
           f"{gbs:.0f} (PMC) | 0 vs oracle (bit-exact); oracle vs reference arithmetic "
           f"{max(r['rel_max_lockstep'], r['rel_max_same_iters']):.1e} (p-H2O Ng layers: within 2x their "
           f"fixed-point distance, as under a one-ulp input change; DESIGN §5) |")
    p = os.path.join(ROOT, "BASELINE.md")
    s = open(p).read()
    s = re.sub(r"^\| CH3OH-A-256 × 4096 \|.*$", row, s, flags=re.M)
    open(p, "w").write(s)
    print(row)


if __name__ == "__main__":
    main()
