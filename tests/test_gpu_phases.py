"""Joint P/S sampling on the GPU (include/mceik.h nphase = 2) against the oracle.

The reference's data model and flows are joint P/S: pickType P = 1 / S = 2
(mceik_struct.h:4-8), homog.c makes a P and an S pick per station and event
and separate vp / vs models (homog.c:203-258), the locator stacks both phases
(locate.f90:399,442) and h5io writes both tables (h5io.c:662-697).  The
sampler holds a P and an S model per chain; a proposal changes one cell of one
of them and only that model's tables are re-solved (the other model's tables
are kept from the last accepted state).  The oracle (oracle_mcmc_run)
re-solves every model of the chain for every proposal, so bitwise agreement
also shows the kept tables are exact.  The MCMC definition itself is unpinned
by the reference (mceik.h:1-14 is empty), as for the P-only sampler.
"""
import os

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _ps_problem(n=28, nstat=5, nev=6, seed=31):
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", n=n, nstat=nstat, nev=nev, seed=seed, phases="PS",
                          picks=mcmc.picks_from_forward(0))
    p.dvmax = 300
    p.var[:] = 1e-5
    p.scorr = np.linspace(-0.01, 0.02, nstat)      # S statics take part (mceik_struct.h:42-44)
    p.pcorr = np.linspace(0.005, -0.005, nstat)
    return p


def test_ps_catalog_layout_follows_homog():
    """make_problem(phases='PS'): per event, per station a P then an S pick
    (homog.c:203-229), S model = round(vp / sqrt(3)) (homog.c:53-54)."""
    p = _ps_problem()
    assert p.nphase == 2
    assert list(p.pick_type[:4]) == [1, 2, 1, 2] and list(p.obs_stat[:4]) == [0, 0, 1, 1]
    assert np.array_equal(p.vs_true, np.rint(p.v_true / np.sqrt(3.0)).astype(np.int32))
    assert p.obs_phase.sum() == p.nevents * p.nstat


def test_ps_init_tables_and_loglik_bitwise():
    """Init forward of 3 chains: P and S tables, iteration counts and logL of
    every chain == the fp32 twin / oracle_loglik over both phases."""
    _dev()
    from mceik_amd import mcmc
    p = _ps_problem()
    s = mcmc.Sampler(p, nchains=3, chain_offset=7)
    assert s.info()["nphase"] == 2
    v0, logl0, _, _ = s.state()
    assert v0.shape == (3, 2, p.ncell)
    tt, niter, _, ierr = s.last(with_ierr=True)
    s.close()
    assert tt.shape == (3, 2, p.nstat, p.nevents) and not ierr.any()
    P = O.make_problem(p)
    for c in range(3):
        to = O.forward_all_f32(P, v0[c])
        assert np.array_equal(tt[c].view(np.uint32), to.view(np.uint32)), c
        for ph in range(2):
            _, it = O.forward_f32(P, v0[c, ph])
            assert np.array_equal(niter[c, ph], it), (c, ph)
        assert logl0[c] == O.loglik(P, to)


@pytest.mark.parametrize("mode", ["multi", "pipes1", "pipes2"])
def test_ps_mcmc_steps_bitwise(mode, monkeypatch):
    """8 steps of 4 chains: accept sequence, logL trace and both models ==
    oracle_mcmc_run (which re-solves both models every proposal); proposals
    hit both models; multi-step launches, one pipe and two pipes alike."""
    _dev()
    monkeypatch.setenv("MCEIK_PERSIST", "1" if mode == "multi" else "0")
    monkeypatch.setenv("MCEIK_PIPES", "2" if mode == "pipes2" else "1")
    from mceik_amd import mcmc
    p = _ps_problem()
    nch, off, nsteps = 4, 3, 8
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off)
    assert s.info()["npipe"] == (2 if mode == "pipes2" else 1)
    assert s.info()["multi_step"] == (mode == "multi")
    v0, logl0, _, _ = s.state()
    acc, trace, phases = [], [], []
    for _ in range(nsteps):
        s.run(1)
        _, _, a = s.last()
        _, lg, _, _ = s.state()
        acc.append(a.copy())
        trace.append(lg.copy())
        phases.append(s.last_phase())
    v, logl, nacc, step = s.state()
    s.close()
    vo, lo, acco, traceo = O.mcmc_run(O.make_problem(p), v0, logl0, off, 0, nsteps)
    ph = np.array(phases)
    assert (ph == 0).any() and (ph == 1).any()
    assert np.array_equal(np.array(acc), acco)
    assert np.array_equal(np.array(trace).view(np.uint64), traceo.view(np.uint64))
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert 0 < acco.sum() < acco.size


def test_ps_step_tables_are_the_changed_model():
    """After a step the tables are the proposed phase's solve of the proposed
    model (in or out of the prior, every step costs one solve per station)."""
    _dev()
    from mceik_amd import mcmc
    p = _ps_problem(nev=4)
    s = mcmc.Sampler(p, nchains=2)
    v0, _, _, _ = s.state()
    s.run(1)
    tt, _, _ = s.last()
    ph = s.last_phase()
    s.close()
    P = O.make_problem(p)
    for c in range(2):
        cell, vn, inp, _ = O.propose(P, c, 0, v0[c].ravel())
        vp = v0[c].copy().reshape(-1)
        if inp:
            vp[cell] = vn
        assert ph[c] == (cell >= p.ncell)
        to = O.forward_all_f32(P, vp)
        assert np.array_equal(tt[c].view(np.uint32), to[ph[c]].view(np.uint32)), c


def test_p_only_sampler_refuses_s_picks_unless_masked():
    """A P-only sampler (nphase 1) given a catalog with S picks fails init
    (no observation disappears silently); with mask_s it fits the P picks
    only, exactly like the same catalog without its S picks."""
    _dev()
    from mceik_amd import mcmc
    p = _ps_problem(nev=4)
    v0 = mcmc.initial_models(p, range(2))
    p.nphase = 1
    with pytest.raises(RuntimeError, match=r"\(1\)"):
        mcmc.Sampler(p, nchains=2, v0=v0[:, 0])
    p.mask_s = 1
    s = mcmc.Sampler(p, nchains=2, v0=v0[:, 0])
    assert s.info()["masked_s"] == p.nevents * p.nstat
    s.run(3)
    v, logl, _, _ = s.state()
    s.close()
    keep = p.pick_type == mcmc.P_PRIMARY_PICK
    q = mcmc.Problem(**{k: getattr(p, k) for k in ("nx", "ny", "nz", "h", "nref", "maxit", "tol", "vmin", "vmax",
                                                     "dvmax", "seed")})
    q.sx, q.sy, q.sz, q.pcorr, q.scorr = p.sx, p.sy, p.sz, p.pcorr, p.scorr
    q.ex, q.ey, q.ez, q.v_true = p.ex, p.ey, p.ez, p.v_true
    q.obs_ptr = (np.arange(p.nevents + 1) * p.nstat).astype(np.int32)
    q.obs_stat, q.pick_type = p.obs_stat[keep], p.pick_type[keep]
    q.luse, q.tobs, q.var = p.luse[keep], p.tobs[keep], p.var[keep]
    s2 = mcmc.Sampler(q, nchains=2, v0=v0[:, 0])
    s2.run(3)
    v2, logl2, _, _ = s2.state()
    s2.close()
    assert np.array_equal(v, v2) and np.array_equal(logl.view(np.uint64), logl2.view(np.uint64))


def test_ps_checkpoint_restore_bitwise():
    """6 steps == 3 steps + checkpoint + restore (logL recomputed by one forward
    of both models) + 3 steps, with two models per chain."""
    _dev()
    from mceik_amd import mcmc
    p = _ps_problem(nev=4)
    a = mcmc.Sampler(p, nchains=3)
    a.run(6)
    va, la, na, _ = a.state()
    a.close()
    b = mcmc.Sampler(p, nchains=3)
    b.run(3)
    ck = b.checkpoint()
    b.close()
    c = mcmc.Sampler(p, nchains=3)
    c.restore(ck, recompute_logl=True)
    c.run(3)
    vc, lc, nc, step = c.state()
    c.close()
    assert step == 6
    assert np.array_equal(va, vc) and np.array_equal(la.view(np.uint64), lc.view(np.uint64))
    assert np.array_equal(na, nc)


def test_ps_posterior_writes_s_tables(tmp_path):
    """write_posterior with P and S models: PTravelTimes and STravelTimes of
    every model x station (h5io.c:662-697) == the fp32 twin's fields."""
    _dev()
    from mceik_amd import h5io, mcmc
    p = _ps_problem(n=20, nstat=3, nev=2)
    models = mcmc.initial_models(p, range(2))            # [2, 2, ncell]
    ttn, _ = h5io.write_posterior(p, models, str(tmp_path), "ps", relocate_events=False)
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    cell = ((k // p.nrz) * p.ncy + j // p.nry) * p.ncx + i // p.nrx
    with h5io.H5File.open(ttn) as f:
        for m in range(2):
            for ph in range(2):
                slow = (1.0 / models[m, ph].astype(np.float32)).astype(np.float32)
                for st in range(p.nstat):
                    got = f.read_ttimes(st + 1, m + 1, iphase=ph + 1)
                    ref, _, _ = O.eikonal_solve(p.nx, p.ny, p.nz, slow[cell].ravel(), p.h,
                                                np.array([[0.0, p.sx[st], p.sy[st], p.sz[st]]]), maxit=p.maxit,
                                                tol=p.tol, dtype=np.float32)
                    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (m, ph, st)


@pytest.mark.parametrize("mode", ["pipes2", "multi", "f64_pipes2"])
def test_station_flags_skip_solves_bitwise(mode, monkeypatch):
    """Half the stations have no S picks (lhasS = 0, homog.c:313-335 makes no
    table for them): their S solves are skipped (table FLT_MAX, niter 0), the
    P tables of every station and the S tables of the others are the twin's,
    logL, accept sequence and both models after 6 steps == oracle_mcmc_run
    (with the same skip rule), and mceik_mcmc_fsm_solves counts only the
    solves that ran.  f64_pipes2: the fp64 sampler (fsm_solve_kernel<double>,
    the skip path of fsm_kernel.hip) against the fp64 oracle forward
    (oracle_mcmc_problem.prec = 64)."""
    _dev()
    prec = 64 if mode.startswith("f64") else 32
    monkeypatch.setenv("MCEIK_PERSIST", "1" if mode == "multi" else "0")
    monkeypatch.setenv("MCEIK_PIPES", "1" if mode == "multi" else "2")
    from mceik_amd import mcmc
    p = _ps_problem(nstat=6)
    nos = np.arange(p.nstat) % 2 == 1                     # stations 1, 3, 5: no S picks
    p.luse[(p.pick_type == mcmc.S_PRIMARY_PICK) & nos[p.obs_stat]] = 0
    hp, hs = p.station_flags()
    assert hp.all() and np.array_equal(hs, (~nos).astype(np.int32))
    nch, off, nsteps = 4, 3, 6
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off, precision=prec)
    assert s.info()["multi_step"] == (mode == "multi")
    assert s.info()["kernel"].startswith("fsm_solve_kernel<double" if prec == 64 else "fsm16_solve_kernel")
    v0, logl0, _, _ = s.state()
    tt, niter, _, ierr = s.last(with_ierr=True)
    assert not ierr.any()
    assert (tt[:, 1, nos] == np.float32(np.finfo(np.float32).max)).all() and (niter[:, 1, nos] == 0).all()
    P = O.make_problem(p, precision=prec)
    for c in range(nch):
        to = O.forward_all_f32(P, v0[c])
        assert np.array_equal(tt[c].view(np.uint32), to.view(np.uint32)), c
        for ph in range(2):
            _, it = O.forward_f32(P, v0[c, ph], phase=ph)
            assert np.array_equal(niter[c, ph], it), (c, ph)
        assert logl0[c] == O.loglik(P, to)
    assert s.fsm_solves() == 0                            # init's forward is not counted
    acc, trace, phases = [], [], []
    for _ in range(nsteps):
        s.run(1)
        _, _, a = s.last()
        _, lg, _, _ = s.state()
        acc.append(a.copy())
        trace.append(lg.copy())
        phases.append(s.last_phase())
    v, logl, _, _ = s.state()
    solves = s.fsm_solves()
    s.close()
    ph = np.array(phases)
    assert (ph == 1).any()
    assert solves == int((ph == 0).sum()) * p.nstat + int((ph == 1).sum()) * int((~nos).sum())
    vo, lo, acco, traceo = O.mcmc_run(P, v0, logl0, off, 0, nsteps)
    assert np.array_equal(np.array(acc), acco)
    assert np.array_equal(np.array(trace).view(np.uint64), traceo.view(np.uint64))
    assert np.array_equal(v, vo) and np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
