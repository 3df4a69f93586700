#!/usr/bin/env python3
"""Probe: does running the C3 chains as two halves on two HIP streams (each
half's next FSM launch queued behind its own accept) hide the per-step
work-queue tail (waves 96.6% busy)?  Prints proposals/s of
one 1024-chain sampler and of two 512-chain samplers on two streams, same
box, same models, and whether the two paths end in the same chain states."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mceik_amd import mcmc  # noqa: E402


def main():
    import torch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    p = mcmc.make_problem("C3", picks="analytic")
    n = 1024
    v0 = mcmc.initial_models(p, range(0, n))
    tt = mcmc.picks_from_forward(0)(p)
    torch.cuda.empty_cache()
    rng = np.random.default_rng(p.seed + 1)
    p.tobs = tt.T.ravel().astype(np.float64) + rng.normal(0.0, 5e-4, p.nevents * p.nstat)
    p.var[:] = 5e-4 ** 2
    dev = torch.device("cuda", 0)

    def timed(samplers, streams):
        for s, st in zip(samplers, streams):
            s.set_stream(st.cuda_stream)
            s.run(1)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            for s in samplers:
                s.run(1)
        torch.cuda.synchronize(dev)
        return n * steps / (time.perf_counter() - t)

    one = mcmc.Sampler(p, nchains=n, chain_offset=0, v0=v0, device=0)
    r1 = timed([one], [torch.cuda.Stream(dev)])
    v1, l1, a1, _ = one.state()
    one.close()
    torch.cuda.empty_cache()
    halves = [mcmc.Sampler(p, nchains=n // 2, chain_offset=k * n // 2, v0=v0[k * n // 2:(k + 1) * n // 2], device=0)
              for k in range(2)]
    r2 = timed(halves, [torch.cuda.Stream(dev), torch.cuda.Stream(dev)])
    st = [h.state() for h in halves]
    same = bool(np.array_equal(np.concatenate([s[0] for s in st]), v1) and
                np.array_equal(np.concatenate([s[1] for s in st]), l1))
    for h in halves:
        h.close()
    print(f"pipe_probe C3 {steps} steps: one sampler {r1:.1f} proposals/s, two halves on two streams {r2:.1f} "
          f"({r2 / r1:.4f}x); states equal: {same}", flush=True)


if __name__ == "__main__":
    main()
