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


@pytest.mark.parametrize("n", [24, 40], ids=["n24_kb3", "n40_kb4"])
def test_accept_sequence_bit_identical(n):
    """n = 40 runs 4-brick z-blocks: the compile-time-kb kernel of the 128^3 bench."""
    _dev()
    from mceik_amd import mcmc
    p = _problem(n=n)
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


def test_posterior_h5io_files(tmp_path):
    """Kept samples -> the reference's HDF5 posterior (h5io.c layout): the
    stored P tables are the GPU forward of each kept model bitwise (fp32
    twin), and each event's logJPDF is the relocation grid search over those
    tables; noise-free picks of the true model put its maximum on the event
    node."""
    _dev()
    from mceik_amd import h5io, mcmc
    p = _problem(n=20, nstat=4, nev=3)
    s = mcmc.Sampler(p, nchains=2, chain_offset=0, max_samples=2)
    s.run(2)
    kept, _ = s.samples()
    s.close()
    models = np.concatenate([kept.reshape(-1, p.ncell)[:2], p.v_true[None]], 0)
    tt_true = mcmc.picks_from_forward(0, precision=32)(p)          # [nstat, nev] at the event nodes
    p.tobs = np.array([tt_true[p.obs_stat[k], e] for e in range(p.nevents)
                       for k in range(p.obs_ptr[e], p.obs_ptr[e + 1])], dtype=np.float64)
    ttn, locn = h5io.write_posterior(p, models, str(tmp_path), "post")
    assert ttn.endswith("post_ttimes.h5") and locn.endswith("post_locations.h5")
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    cell = ((k // p.nrz) * p.ncy + j // p.nry) * p.ncx + i // p.nrx
    with h5io.H5File.open(ttn) as f:
        assert f.dims() == (p.nx, p.ny, p.nz)
        for m in range(models.shape[0]):
            slow = (1.0 / models[m].astype(np.float32)).astype(np.float32)
            for st in range(p.nstat):
                got = f.read_ttimes(st + 1, m + 1)
                ref, _, _ = O.eikonal_solve(p.nx, p.ny, p.nz, slow[cell].ravel(), p.h,
                                            np.array([[0.0, p.sx[st], p.sy[st], p.sz[st]]]), maxit=p.maxit,
                                            tol=p.tol, dtype=np.float32)
                assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (m, st)
    with h5io.H5File.open(locn) as f:
        for e in range(p.nevents):
            lp = f.read_logjpdf(models.shape[0], e + 1)                # the true model
            assert int(np.argmax(lp)) == int(p.ev_node[e])
            assert lp.max() <= 0.0


def test_checkpoint_restore_bitwise():
    """6 steps == 3 steps + checkpoint + restore into a fresh sampler + 3 steps
    (Philox is keyed by (global chain, step): the checkpoint is the complete
    state), with the stored logL and with logL recomputed by one forward."""
    _dev()
    from mceik_amd import mcmc
    p = _problem(seed=9)
    p.nburn, p.keepk = 0, 1
    full = mcmc.Sampler(p, nchains=3, chain_offset=7, max_samples=8)
    full.run(6)
    vf, lf, af, sf = full.state()
    kf, klf = full.samples()
    full.close()
    a = mcmc.Sampler(p, nchains=3, chain_offset=7, max_samples=8)
    a.run(3)
    ck = a.checkpoint()
    a.close()
    assert ck["step"] == 3 and ck["nkept"] == 3
    for recompute in (False, True):
        b = mcmc.Sampler(p, nchains=3, chain_offset=7, max_samples=8)
        b.restore(ck, recompute_logl=recompute)
        b.run(3)
        vb, lb, ab, sb = b.state()
        kb, klb = b.samples()
        b.close()
        assert sb == sf == 6
        assert np.array_equal(vb, vf) and np.array_equal(lb.view(np.uint64), lf.view(np.uint64))
        assert np.array_equal(ab, af)
        # the restored sampler kept only steps 3..5 (its ring slots 3..5)
        assert len(kb) == 3 and np.array_equal(kb, kf[3:6]) and np.array_equal(klb, klf[3:6])


def test_run_to_niter_and_sample_ring_order():
    """run(-1) runs the remaining mcparms.niter proposals; once the sample ring
    wraps, get_samples returns the most recent states oldest first."""
    _dev()
    from mceik_amd import mcmc
    p = _problem(seed=13)
    p.nburn, p.keepk, p.niter = 0, 1, 5
    s = mcmc.Sampler(p, nchains=2, max_samples=2)
    states = []
    s.run(2)
    states += [s.state()[0]]
    s.run(-1)                                       # steps 2, 3, 4
    v, _, _, step = s.state()
    assert step == 5
    kv, _ = s.samples()
    s.run(-1)                                       # nothing left
    assert s.state()[3] == 5
    s.close()
    ref = mcmc.Sampler(p, nchains=2)
    seq = []
    for _ in range(5):
        ref.run(1)
        seq.append(ref.state()[0])
    ref.close()
    assert np.array_equal(v, seq[4])
    assert len(kv) == 2 and np.array_equal(kv[0], seq[3]) and np.array_equal(kv[1], seq[4])


def test_station_on_first_node_fails_init():
    """A station exactly on the grid's first x node triggers the reference's
    SETBCS quirk (ierr = 1, fsm3d.f90:736-745): init fails instead of running
    chains on u_nan tables."""
    _dev()
    from mceik_amd import mcmc
    p = _problem(n=20, seed=17)
    p.sx = p.sx.copy()
    p.sx[1] = p.x0
    with pytest.raises(RuntimeError):
        mcmc.Sampler(p, nchains=1)



@pytest.mark.parametrize("nch,pipes", [(5, "2"), (8, "2"), (5, "1"), (7, "3"), (5, "multi"), (9, "multi")],
                         ids=["odd_halves", "even_halves", "one_pipe", "three_pipes", "multi_step", "multi_step_9"])
def test_pipes_bitwise(nch, pipes, monkeypatch):
    """Two pipes (halves of the chains on two streams), one
    pipe (MCEIK_PIPES=1), three, and multi-step launches (MCEIK_PERSIST=1: the
    accept, kept state and next proposal inside the FSM kernel): models, logL,
    accept counts and kept samples bit-identical to oracle_mcmc_run, with
    run() split over calls (kept-state slots carried across launches)."""
    _dev()
    from mceik_amd import mcmc
    monkeypatch.setenv("MCEIK_PERSIST", "1" if pipes == "multi" else "0")
    monkeypatch.setenv("MCEIK_PIPES", "1" if pipes == "multi" else pipes)
    p = _problem(n=64 if pipes == "multi" else 40, seed=9)     # (64^3: the 16-z kernel, which runs multi-step)
    p.nburn, p.keepk = 1, 2                   # kept after steps 2, 4, 6
    off = 3
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off, max_samples=8)
    info = s.info()
    assert info["multi_step"] == (pipes == "multi")
    assert info["npipe"] == (1 if pipes == "multi" else int(pipes))
    v0, logl0, _, _ = s.state()
    s.run(2)
    s.run(1)
    s.run(3)
    _, _, last_acc = s.last()
    v, logl, nacc, step = s.state()
    kv, kl = s.samples()
    s.close()
    P = O.make_problem(p)
    vo, lo, acc, trace = O.mcmc_run(P, v0, logl0, off, 0, 6)
    assert step == 6
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert np.array_equal(last_acc, acc[-1])
    assert nacc.sum() == acc.sum() and 0 < acc.sum() < acc.size
    assert len(kv) == 3
    for k, n in enumerate((2, 4, 6)):
        vk, lk, _, _ = O.mcmc_run(P, v0, logl0, off, 0, n)
        assert np.array_equal(kv[k], vk)
        assert np.array_equal(kl[k].view(np.uint64), lk.view(np.uint64))
