#!/usr/bin/env python3
"""profiles/traffic.json from a tools/measure_r04.sh output directory: HBM
bytes per one-pipe launch of the sampler's FSM kernels (FETCH_SIZE x2 +
WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction, KB x 1024), the SQ
instruction counters and the VALU per wave macro step -- the fp32 record at
the top level (bench.py's headline) and the fp64 record under "f64" (the
line's f64 record).
usage: tools/traffic_json.py <dir> <kernel_rev> [round] [f64_dir] [f64_kernel_rev] > profiles/traffic.json
(the fp32 record from <dir>; the fp64 record from f64_dir, default <dir>)"""
import csv
import collections
import glob
import json
import os
import sys

KERNELS = {32: ("fsm16_solve_kernel", "fsm16_solve_kernel<2, 1>"),
           64: ("fsm_solve_kernel<double, 2, true", "fsm_solve_kernel<double, 2, true, 2, 1, 4>")}


def pmc(d, name):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) for k in tot}, {k: len(v) for k, v in disp.items()}


def record(d, prec, rev, rnd):
    match, kname = KERNELS[prec]
    f1, n1 = pmc(os.path.join(d, f"f{prec}_pmc1"), match)
    f2, n2 = pmc(os.path.join(d, f"f{prec}_pmc2"), match)
    sq, _ = pmc(os.path.join(d, f"f{prec}_pmc3"), match)
    iss, clk = {}, None
    if os.path.isdir(os.path.join(d, f"f{prec}_pmc4")):
        iss, _ = pmc(os.path.join(d, f"f{prec}_pmc4"), match)
        l4 = [x for x in open(os.path.join(d, f"bench_f{prec}_pmc4.log")) if x.startswith("{")][-1]
        ms4 = json.loads(l4)["roofline"]["avg_launch_ms"]
        if "GRBM_GUI_ACTIVE" in iss:
            clk = round(iss.pop("GRBM_GUI_ACTIVE") / 8.0 / (ms4 * 1e-3) / 1e9, 3)
        iss.pop("GRBM_COUNT", None)
    line = json.loads(open(os.path.join(d, f"bench_f{prec}_pipes1_raw.log")).read().strip().splitlines()[-1])
    ws = line["roofline"]["wave_steps_per_step"]
    fetch = f1["FETCH_SIZE"] * 1024.0
    write = f2["WRITE_SIZE"] * 1024.0
    alg = line["roofline"]["alg_bytes_per_step"]
    return {
        "round": rnd,
        "workload": "C3",
        "chains_per_gpu": line["config"]["chains_per_gpu"],
        "kernel": kname,
        "kernel_rev": rev,
        "dispatches": [n1["FETCH_SIZE"], n2["WRITE_SIZE"]],
        "fetch_size_bytes_raw": fetch,
        "write_size_bytes": write,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "alg_bytes_per_launch": alg,
        "hbm_over_alg": round((2.0 * fetch + write) / alg, 4),
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM: gfx950 reports 1/2 of 16-B/lane reads); "
                      "WRITE_SIZE exact; KB x 1024",
        "source": f"tools/measure_r04.sh ({d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ passes over bench.py "
                  f"--steps 1 --warmup 1 --pipes 1 --precision {prec}, {match} dispatches averaged)",
        "sq_per_launch": {k: v for k, v in sorted(sq.items())},
        "sq_issue_per_launch": {k: v for k, v in sorted(iss.items())} or None,
        "effective_clock_ghz": clk,
        "wave_steps_per_launch": int(ws),
        "valu_per_wave_step": round(sq["SQ_INSTS_VALU"] / ws, 1) if "SQ_INSTS_VALU" in sq else None,
        "z_per_wave_step": 16 if prec == 32 else 8,
    }


def main():
    d, rev = sys.argv[1], sys.argv[2]
    rnd = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    d64 = sys.argv[4] if len(sys.argv) > 4 else d
    rev64 = sys.argv[5] if len(sys.argv) > 5 else rev
    out = record(d, 32, rev, rnd)
    if os.path.isdir(os.path.join(d64, "f64_pmc1")):
        out["f64"] = record(d64, 64, rev64, rnd)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
