#!/usr/bin/env python3
"""profiles/traffic.json from a tools/measure_r03.sh output directory: HBM
bytes per one-pipe launch of the sampler's FSM kernel (FETCH_SIZE x2 +
WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction, KB x 1024), the SQ
instruction counters and the VALU per wave macro step.
usage: tools/traffic_json.py <dir> <kernel_rev> [round] > profiles/traffic.json"""
import csv
import collections
import glob
import json
import os
import re
import sys


def pmc(d, name="fsm16_solve_kernel"):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) for k in tot}, {k: len(v) for k, v in disp.items()}


def main():
    d, rev = sys.argv[1], sys.argv[2]
    rnd = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    f1, n1 = pmc(os.path.join(d, "pmc1"))
    f2, n2 = pmc(os.path.join(d, "pmc2"))
    sq, _ = pmc(os.path.join(d, "pmc3"))
    line = json.loads(open(os.path.join(d, "bench_pipes1_raw.log")).read().strip().splitlines()[-1])
    ws = line["roofline"]["wave_steps_per_step"]
    fetch = f1["FETCH_SIZE"] * 1024.0
    write = f2["WRITE_SIZE"] * 1024.0
    out = {
        "round": rnd,
        "workload": "C3",
        "chains_per_gpu": line["config"]["chains_per_gpu"],
        "kernel": "fsm16_solve_kernel<2, 1>",
        "kernel_rev": rev,
        "dispatches": [n1["FETCH_SIZE"], n2["WRITE_SIZE"]],
        "fetch_size_bytes_raw": fetch,
        "write_size_bytes": write,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM: gfx950 reports 1/2 of 16-B/lane reads); "
                      "WRITE_SIZE exact; KB x 1024",
        "source": f"tools/measure_r03.sh ({d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py "
                  "--steps 1 --warmup 1 --pipes 1, fsm16_solve_kernel dispatches averaged)",
        "sq_per_launch": {k: v for k, v in sorted(sq.items())},
        "wave_steps_per_launch": int(ws),
        "valu_per_wave_step": round(sq["SQ_INSTS_VALU"] / ws, 1) if "SQ_INSTS_VALU" in sq else None,
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
