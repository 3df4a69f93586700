#!/usr/bin/env python3
"""Diagnostic (GPU): where multi-step sampler launches first differ from the
step-by-step launches.  For N = 1 .. NMAX: a fresh multi-step sampler runs N
steps in one launch; its state is compared with the step-by-step sampler's
after N steps.  Also a multi-step sampler driven one step per launch.
usage: tools/ms_diag.py [phases] [nchains] [nmax]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    phases = sys.argv[1] if len(sys.argv) > 1 else "PS"
    nch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    nmax = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", nstat=8, nev=8, seed=77, phases=phases, picks=mcmc.picks_from_forward(0))
    p.dvmax = 300
    p.var[:] = 1e-5

    def sampler(multi):
        os.environ["MCEIK_PERSIST"] = "1" if multi else "0"
        os.environ["MCEIK_PIPES"] = "1"
        return mcmc.Sampler(p, nchains=nch, chain_offset=11)

    ref = sampler(False)
    states = []
    phs = []
    for n in range(nmax):
        ref.run(1)
        v, lg, na, _ = ref.state()
        states.append((v.copy(), lg.copy()))
        phs.append(ref.last_phase().copy() if phases == "PS" else np.zeros(nch, int))
    ref.close()
    one = sampler(True)
    for n in range(nmax):
        one.run(1)
        v, lg, _, _ = one.state()
        bad = np.flatnonzero((v.reshape(nch, -1) != states[n][0].reshape(nch, -1)).any(1) |
                             (lg.view(np.uint64) != states[n][1].view(np.uint64)))
        if len(bad):
            print(f"one-step launches: step {n + 1} differs in chains {bad[:10]} (proposal phases {phs[n][bad[:10]]})")
            break
    else:
        print(f"one-step launches: equal for {nmax} steps")
    one.close()
    for n in range(1, nmax + 1):
        s = sampler(True)
        s.run(n)
        v, lg, _, _ = s.state()
        s.close()
        bad = np.flatnonzero((v.reshape(nch, -1) != states[n - 1][0].reshape(nch, -1)).any(1) |
                             (lg.view(np.uint64) != states[n - 1][1].view(np.uint64)))
        if len(bad):
            print(f"{n} steps in one launch: chains {bad[:10]} differ; their phases by step: "
                  f"{[list(phs[k][bad[:4]]) for k in range(n)]}")
            break
        print(f"{n} steps in one launch: equal")


if __name__ == "__main__":
    main()
