#!/usr/bin/env python3
"""Turns one profiles/collect.sh run (gpurun_out/prof_<tag>/) into the committed
summaries: profiles/<tag>/kernel_stats.csv (rocprofv3 --stats), pmc_fsm.csv
(per-dispatch FETCH_SIZE / WRITE_SIZE of the FSM kernel) and
profiles/traffic.json (HBM bytes per launch, read by bench.py's roofline).

Counter handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes, values are KB
(x1024), and FETCH_SIZE is doubled on gfx950 (it tallies 128-B reads at 64 B).

    python profiles/summarize.py <tag> [--kernel 'fsm_solve_kernel<float, 2, true>']
"""
import argparse
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_rev():
    with open(os.path.join(ROOT, "bench.py")) as f:
        return re.search(r'KERNEL_REV = "([^"]+)"', f.read()).group(1)


def per_dispatch(path, kernel):
    """Sum of a counter over the agents/instances of each dispatch of `kernel`."""
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                d = int(row["Dispatch_Id"])
                acc[d] = acc.get(d, 0.0) + float(row["Counter_Value"])
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="fsm_solve_kernel<float, 2, true, 2>")
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--chains", type=int, default=1024)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench_under_trace.log"), os.path.join(dst, "bench_under_trace.log"))
    fetch = per_dispatch(os.path.join(src, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), a.kernel)
    write = per_dispatch(os.path.join(src, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), a.kernel)
    if not fetch or not write:
        sys.exit(f"no dispatches of {a.kernel!r} in the PMC passes")
    with open(os.path.join(dst, "pmc_fsm.csv"), "w") as f:
        f.write("counter,dispatch,value_kb\n")
        for name, d in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write)):
            for k in sorted(d):
                f.write(f"{name},{k},{d[k]}\n")
    fb = sum(fetch.values()) / len(fetch) * 1024.0
    wb = sum(write.values()) / len(write) * 1024.0
    tj = {
        "round": int((re.match(r"r(\d+)", a.tag) or re.match("()", "0")).group(1) or 0),
        "workload": a.workload,
        "chains_per_gpu": a.chains,
        "kernel": a.kernel,
        "kernel_rev": kernel_rev(),
        "dispatches": [len(fetch), len(write)],
        "fetch_size_bytes_raw": fb,
        "write_size_bytes": wb,
        "hbm_bytes_per_launch": 2.0 * fb + wb,
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM: gfx950 reports 1/2 of 16-B/lane reads); "
                      "WRITE_SIZE exact; KB x 1024",
        "source": a.source or f"profiles/collect.sh {a.tag} (separate --pmc passes)",
    }
    with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as f:
        json.dump(tj, f, indent=1)
    print(json.dumps(tj, indent=1))


if __name__ == "__main__":
    main()
