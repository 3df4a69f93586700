#!/usr/bin/env python3
"""Per-step FSM time from a rocprofv3 kernel trace when the sampler runs two
pipes: the half launches of consecutive steps overlap, so
the time the GPU spends in FSM work is the UNION of their [start, end]
intervals, not the sum of their durations.

    tools/trace_union.py <kernel_trace.csv> [--skip N] [--steps K]

--skip: FSM launches to drop first (the sampler's full-size init forward and
the warm-up steps' halves); --steps: timed steps (2 launches each)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--kernel", default="fsm16_solve_kernel")
    a = ap.parse_args()
    with open(a.trace) as f:
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)
                    if a.kernel in r["Kernel_Name"])
    seg = iv[a.skip:a.skip + 2 * a.steps]
    union, cov = 0, 0
    for s, e in seg:
        s = max(s, cov)
        if e > s:
            union += e - s
        cov = max(cov, e)
    dur = [(e - s) / 1e6 for s, e in seg]
    print(f"{len(seg)} launches: durations {', '.join(f'{d:.1f}' for d in dur)} ms (mean {sum(dur) / len(dur):.1f}); "
          f"union {union / 1e6:.1f} ms = {union / 1e6 / a.steps:.1f} ms per step; sum {sum(dur):.1f} ms")


if __name__ == "__main__":
    main()
