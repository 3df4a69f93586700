"""Multi-step sampler launches: one FSM launch runs many
MCMC steps, the wave that completes a chain's solves of a step runs the
chain's accept, kept state and next proposal inside the kernel, and the
chains' groups are owned by XCDs.  The results must be those of the
step-by-step launches (propose / FSM / accept kernels) bit for bit, and those
of oracle_mcmc_run.
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _problem(phases, nstat=8, nev=8):
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", nstat=nstat, nev=nev, seed=77, phases=phases, picks=mcmc.picks_from_forward(0))
    p.dvmax = 300
    p.var[:] = 1e-5
    p.nburn, p.keepk = 5, 3
    return p


def _run(p, nchains, nsteps, multi, monkeypatch, max_samples=8):
    from mceik_amd import mcmc
    monkeypatch.setenv("MCEIK_PERSIST", "1" if multi else "0")
    monkeypatch.setenv("MCEIK_PIPES", "1")
    s = mcmc.Sampler(p, nchains=nchains, chain_offset=11, max_samples=max_samples)
    info = s.info()
    s.run(nsteps)
    v, logl, nacc, step = s.state()
    kv, kl = s.samples()
    tt, _, acc = s.last()
    _, nl, _, _ = s.fsm_stats()
    s.close()
    return info, (v, logl, nacc, step, kv, kl, tt, acc), nl


@pytest.mark.parametrize("phases", ["P", "PS"])
def test_multi_step_launches_equal_step_by_step(phases, monkeypatch):
    """70 steps of 64 chains (two launches: 64 + 6 steps), kept states every
    3rd step after 5 burn-in steps into an 8-slot ring (it wraps): models,
    logL, accept counts, kept models and logL, the last step's tables and
    accept flags equal the per-step launches' bit for bit."""
    _dev()
    p = _problem(phases)
    ia, a, nla = _run(p, 64, 70, True, monkeypatch)
    ib, b, nlb = _run(p, 64, 70, False, monkeypatch)
    assert ia["multi_step"] and not ib["multi_step"] and ia["step_z"] == 16
    assert nla == 2 and nlb == 70
    names = ("v", "logl", "naccept", "step", "kept v", "kept logl", "tables", "accept")
    for n, x, y in zip(names, a, b):
        if isinstance(x, np.ndarray):
            assert x.shape == y.shape and x.tobytes() == y.tobytes(), n
        else:
            assert x == y, n
    assert a[3] == 70 and len(a[4]) == 8
    assert 0 < a[2].sum() < 64 * 70


def test_multi_step_few_chains_vs_oracle(monkeypatch):
    """3 chains (5 of the 8 chain groups empty), 5 steps in one launch:
    models and logL == oracle_mcmc_run."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("P", nstat=5, nev=6)
    monkeypatch.setenv("MCEIK_PERSIST", "1")
    s = mcmc.Sampler(p, nchains=3, chain_offset=4)
    assert s.info()["multi_step"]
    v0, logl0, _, _ = s.state()
    s.run(5)
    v, logl, _, step = s.state()
    s.close()
    vo, lo, acco, _ = O.mcmc_run(O.make_problem(p), v0, logl0, 4, 0, 5)
    assert step == 5
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert 0 < acco.sum()


def test_multi_step_broken_queue_is_reported(monkeypatch):
    """A multi-step wave that gives up waiting for a chain's previous step
    (the ~30-s safety net; MCEIK_MC_SPIN_LIMIT=0 makes every wait give up at
    once) leaves the launch without solving from unready state, and the
    sampler reports the failure at the next synchronisation instead of
    returning corrupt chains."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("P")
    monkeypatch.setenv("MCEIK_PERSIST", "1")
    monkeypatch.setenv("MCEIK_PIPES", "1")
    monkeypatch.setenv("MCEIK_MC_SPIN_LIMIT", "0")
    s = mcmc.Sampler(p, nchains=64, max_samples=8)
    assert s.info()["multi_step"]
    ck = s.checkpoint()
    s.run(8)
    with pytest.raises(RuntimeError):
        s.sync()
    with pytest.raises(RuntimeError):
        s.state()
    with pytest.raises(RuntimeError):
        s.fsm_stats()
    with pytest.raises(RuntimeError):
        s.fsm_solves()
    # the checkpoint gather refuses the broken state too (single-rank RCCL communicator)
    comm = mcmc.Comm(0, 1, 0)
    with pytest.raises(RuntimeError):
        comm.gather(s, 64, which=0)
    # restoring a checkpoint replaces the state and clears the flag
    s.restore(ck)
    v, logl, nacc, step = s.state()
    assert step == ck["step"] and np.array_equal(v, ck["v"])
    assert np.array_equal(logl.view(np.uint64), ck["logl"].view(np.uint64))
    vg, lg = comm.gather(s, 64, which=0)
    assert np.array_equal(vg, ck["v"])
    comm.close()
    s.close()
