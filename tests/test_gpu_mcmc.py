"""GPU MCMC step (propose -> FSM -> misfit -> Metropolis) vs the CPU restatement.

The accept sequence, chain models and logL must be BIT-IDENTICAL to
oracle_mcmc_run (oracle/mceik_oracle.c) under the same Philox seed.  The
reference defines no MCMC, so this parity is against the build's own
restatement (parity unpinned by the reference for this row).
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _problem(n=24, nstat=4, nev=6, seed=7):
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", n=n, nstat=nstat, nev=nev, seed=seed, picks=mcmc.picks_from_forward(0))
    p.dvmax = 400                       # large steps: both accepts and rejects in a few steps
    p.var[:] = 1e-4                     # sharp likelihood so that some proposals are rejected
    return p


def test_initial_loglik_matches_oracle():
    _dev()
    from mceik_amd import mcmc
    p = _problem()
    s = mcmc.Sampler(p, nchains=3, chain_offset=5)
    v, logl, nacc, step = s.state()
    P = O.make_problem(p)
    for c in range(3):
        tt, _ = O.forward_f32(P, v[c])
        assert logl[c] == O.loglik(P, tt)
    s.close()


def test_accept_sequence_bit_identical():
    _dev()
    from mceik_amd import mcmc
    p = _problem()
    nch, nsteps, off = 4, 6, 11
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off)
    v0, logl0, _, _ = s.state()
    gpu_acc = []
    gpu_logl = []
    for _ in range(nsteps):
        s.run(1)
        _, _, a = s.last()
        _, lg, _, _ = s.state()
        gpu_acc.append(a.copy())
        gpu_logl.append(lg.copy())
    v, logl, nacc, step = s.state()
    s.close()
    P = O.make_problem(p)
    vo, lo, acc, trace = O.mcmc_run(P, v0, logl0, off, 0, nsteps)
    assert np.array_equal(np.array(gpu_acc), acc)
    assert np.array_equal(np.array(gpu_logl).view(np.uint64), trace.view(np.uint64))
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert step == nsteps and nacc.sum() == acc.sum()
    assert 0 < acc.sum() < acc.size            # the test exercises both branches


def test_sharding_independent_chains():
    """Chains are keyed by global id: 2 shards of 2 == 1 shard of 4."""
    _dev()
    from mceik_amd import mcmc
    p = _problem(seed=3)
    full = mcmc.Sampler(p, nchains=4, chain_offset=0)
    full.run(3)
    vf, lf, af, _ = full.state()
    full.close()
    parts = []
    for r in range(2):
        lo, hi = mcmc.shard(4, r, 2)
        sp = mcmc.Sampler(p, nchains=hi - lo, chain_offset=lo)
        sp.run(3)
        parts.append(sp.state())
        sp.close()
    assert np.array_equal(np.concatenate([q[0] for q in parts]), vf)
    assert np.array_equal(np.concatenate([q[1] for q in parts]).view(np.uint64), lf.view(np.uint64))


def test_kept_samples():
    _dev()
    from mceik_amd import mcmc
    p = _problem(seed=5)
    p.nburn, p.keepk = 2, 2
    s = mcmc.Sampler(p, nchains=2, max_samples=8)
    states = []
    for st in range(7):
        s.run(1)
        v, lg, _, _ = s.state()
        if st >= 2 and (st - 2) % 2 == 0:
            states.append((v.copy(), lg.copy()))
    kv, kl = s.samples()
    s.close()
    assert len(kv) == len(states) == 3
    for k, (v, lg) in enumerate(states):
        assert np.array_equal(kv[k], v)
        assert np.array_equal(kl[k], lg)
