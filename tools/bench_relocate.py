#!/usr/bin/env python3
"""Relocation grid search (SURVEY s.8f row 2, mceik_relocate) at a C3-sized
catalogue: 32 station tables on the 128^3 grid (fp32), 32 events x 32 P
picks.  Times the single-pass LDS kernel and the two-pass kernel with HIP
events on the launch stream and prints one JSON line with the HBM roofline of
each (algorithmic bytes: every table value read once + the outputs written;
the two-pass kernel re-reads each observed row twice per event).

    python tools/bench_relocate.py [--iters 20] [--t0]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--stations", type=int, default=32)
    ap.add_argument("--events", type=int, default=32)
    ap.add_argument("--t0", action="store_true", help="also write the origin-time grids")
    args = ap.parse_args()
    import torch
    from mceik_amd.eikonal import relocate
    dev = torch.device("cuda", 0)
    ngrd = args.n ** 3
    tables = torch.rand((args.stations, ngrd), device=dev) * 4.0
    rng = np.random.default_rng(1)
    events = [dict(rows=np.arange(args.stations), tobs=rng.uniform(1, 5, args.stations).astype(np.float32),
                   varobs=rng.uniform(0.5, 2, args.stations).astype(np.float32)) for _ in range(args.events)]
    stream = torch.cuda.current_stream(dev)
    out = {"workload": f"relocate: {args.stations} tables x {args.n}^3 grid, {args.events} events x "
                       f"{args.stations} picks, fp32", "peak_GBs": 8000.0}
    for single in (True, False):
        for _ in range(2):
            relocate(tables, events, single_pass=single, want_t0=args.t0, stream=stream.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            relocate(tables, events, single_pass=single, want_t0=args.t0, stream=stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.iters      # includes the host-side packing of the small obs arrays
        alg = 4.0 * ngrd * (args.stations + args.events * (2 if args.t0 else 1))
        key = "single_pass" if single else "two_pass"
        out[key] = {"ms_per_call": round(ms, 4), "alg_GBs": round(alg / ms / 1e6, 1),
                    "frac": round(alg / ms / 1e6 / 8000.0, 4), "alg_bytes": alg}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
