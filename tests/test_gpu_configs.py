"""Parity at the BASELINE.json configurations (SURVEY s.8 table), on the GPU.

Every test runs the kernel instance the bench or the sampler actually runs at
that geometry and compares with the oracle (oracle/fsm_impl.inc fp32 twin,
oracle_mcmc_run) bit for bit:

* C1  1 chain, 32^3 homogeneous, 4 stations, 100 proposals (the plumbing case)
* C2  256 chains x 16 stations at 64^3: 4096 solves on at most 2048 waves,
      so waves run several solves in their reused scratch field
* C3  128^3, 32 stations, 32 events: the bench's own production launch --
      1024 chains in two pipes, fsm16_solve_kernel<2, 1> (16-z steps, the
      fixed LDS layout, cell cache, short sqrt) on 2 x 2048 resident waves in
      two workspaces -- with chains on both sides of the pipe split checked
      after init and one step; plus 4 chains on 16 waves (8 solves per wave in
      reused scratch) and two MCMC steps
* C5  256^3, 64 stations: the sampler's own launch (fsm16_solve_kernel<0, 4>,
      32-brick z-blocks, scratch-budget-capped waves, several solves per
      wave) checked on one chain; and two full fields
C4 is C3's geometry sharded over 8 GPUs (the driver's scaling run).
The CPU side uses the oracle's OpenMP (one solve per thread).
"""
import concurrent.futures as cf

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _problem(config, **kw):
    from mceik_amd import mcmc
    return mcmc.make_problem(config, picks=mcmc.picks_from_forward(0), **kw)


def test_c3_sampler_forward_bitwise_reused_scratch():
    """C3 geometry through the sampler's own launch (the bench instance): the
    initial forward's travel-time tables and iteration counts of 4 chains x
    32 stations equal the fp32 twin bit for bit.  max_waves = 16 puts 8 solves
    on every wave, one after another in the wave's reused u / u0 scratch."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C3")
    assert (p.nx, p.nstat, p.nevents) == (128, 32, 32)
    s = mcmc.Sampler(p, nchains=4, chain_offset=100, max_waves=16)
    v0, logl0, _, _ = s.state()
    ttab, niter, _, ierr = s.last(with_ierr=True)
    s.close()
    assert not ierr.any()
    P = O.make_problem(p)
    for c in range(4):
        tt, it = O.forward_f32(P, v0[c])
        assert np.array_equal(ttab[c].view(np.uint32), tt.view(np.uint32)), c
        assert np.array_equal(niter[c], it), c
        assert logl0[c] == O.loglik(P, tt)


@pytest.mark.timeout(900)
def test_c3_bench_production_launch_bitwise():
    """The bench's exact C3 launch: Sampler(C3) with 1024 chains and the
    library defaults (two pipes, occupancy-many waves, two workspaces).
    Chains {0, 1, 511, 512, 1022, 1023} straddle the pipe split: their init
    tables, iteration counts and logL == the fp32 twin, and their models,
    logL and accept counts after three steps == oracle_mcmc_run."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C3")
    p.dvmax = 400
    p.var[:] = 1e-6
    nsteps = 3
    s = mcmc.Sampler(p, nchains=1024)
    info = s.info()
    assert info["npipe"] == 2 and info["chains"] == [512, 512]
    assert info["step_z"] == 16 and info["fixed_layout"] and not info["multi_step"]
    assert info["kernel"] == "fsm16_solve_kernel<2, 1>"
    assert min(info["waves"]) >= 1024, info           # the full-occupancy launch (2048 on a 256-CU MI355X)
    v0, logl0, _, _ = s.state()
    ttab, niter, _, ierr = s.last(with_ierr=True)
    assert not ierr.any()
    s.run(nsteps)
    v1, logl1, nacc1, step = s.state()
    _, nl, _, _ = s.fsm_stats()
    s.close()
    assert step == nsteps and nl == 2 * nsteps        # one timed half launch per pipe and step
    P = O.make_problem(p)
    for c in (0, 1, 511, 512, 1022, 1023):
        tt, it = O.forward_f32(P, v0[c])
        assert np.array_equal(ttab[c].view(np.uint32), tt.view(np.uint32)), c
        assert np.array_equal(niter[c], it), c
        assert logl0[c] == O.loglik(P, tt), c
    for c in (0, 511, 1022):                          # pairs of consecutive global ids
        sl = slice(c, c + 2)
        vo, lo, acc, _ = O.mcmc_run(P, v0[sl], logl0[sl], c, 0, nsteps)
        assert np.array_equal(v1[sl], vo), c
        assert np.array_equal(logl1[sl].view(np.uint64), lo.view(np.uint64)), c
        assert np.array_equal(nacc1[sl], acc.sum(0)), c


@pytest.mark.timeout(600)
def test_c3_fp64_sampler_tables_bitwise():
    """The bench line's f64 record: Sampler(C3, precision=64) launches the fp64
    instance with the short sqrt (fsm_solve_kernel<double, 2, true, 2, 1, 4>).
    Chain 0's initial tables of stations 0..5 == the fp64 oracle (bitwise the
    reference on the goldens) on the expanded fp32 cell slowness, cast to
    fp32; iteration counts equal."""
    dev = _dev()
    from mceik_amd import mcmc
    p = _problem("C3")
    s = mcmc.Sampler(p, nchains=1, precision=64)
    assert s.info()["kernel"].startswith("fsm_solve_kernel<double, 2, true, 2, 1, 4>"), s.info()["kernel"]
    v0, _, _, _ = s.state()
    ttab, niter, _, ierr = s.last(with_ierr=True)
    s.close()
    assert not ierr.any()
    scell = (1.0 / v0[0].astype(np.float32)).reshape(p.ncz, p.ncy, p.ncx)
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    sfield = scell[k // p.nrz, j // p.nry, i // p.nrx].ravel().astype(np.float64)
    stations = range(6)
    with cf.ThreadPoolExecutor(6) as ex:
        res = list(ex.map(lambda st: O.eikonal_solve(p.nx, p.ny, p.nz, sfield, p.h,
                                                     [(0.0, p.sx[st], p.sy[st], p.sz[st])], p.maxit, p.tol,
                                                     p.x0, p.y0, p.z0), stations))
    for st, (u, e, it) in zip(stations, res):
        assert e == 0
        assert np.array_equal(ttab[0, st].view(np.uint32), u[p.ev_node].astype(np.float32).view(np.uint32)), st
        assert int(niter[0, st]) == it, st


@pytest.mark.timeout(600)
def test_c2_fp64_sampler_mcmc_bitwise():
    """The fp64 sampler's MCMC path (bench.py's f64 record: the short-sqrt
    fp64 instance, compact LDS, whole-line loads): C2 geometry, chains 3 and
    4 -- init tables, iterations and logL, then models, logL and accept
    counts after three steps == oracle_mcmc_run with the fp64 forward
    (oracle_mcmc_problem.prec = 64: the literal fp64 solve on the per-cell
    fp32 slowness, tables (float)u)."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C2")
    p.dvmax = 400
    p.var[:] = 1e-6
    nsteps = 3
    s = mcmc.Sampler(p, nchains=2, chain_offset=3, precision=64)
    assert s.info()["kernel"] == "fsm_solve_kernel<double, 2, true, 2, 1, 4>", s.info()["kernel"]
    v0, logl0, _, _ = s.state()
    ttab, niter, _, ierr = s.last(with_ierr=True)
    assert not ierr.any()
    s.run(nsteps)
    v1, logl1, nacc1, step = s.state()
    s.close()
    assert step == nsteps
    P = O.make_problem(p, precision=64)
    for c in range(2):
        tt, it = O.forward_f32(P, v0[c])
        assert np.array_equal(ttab[c].view(np.uint32), tt.view(np.uint32)), c
        assert np.array_equal(niter[c], it), c
        assert logl0[c] == O.loglik(P, tt), c
    vo, lo, acc, _ = O.mcmc_run(P, v0, logl0, 3, 0, nsteps)
    assert np.array_equal(v1, vo)
    assert np.array_equal(logl1.view(np.uint64), lo.view(np.uint64))
    assert np.array_equal(nacc1, acc.sum(0))


@pytest.mark.timeout(600)
def test_c5_sampler_launch_bitwise():
    """C5 through the sampler: 256^3, 64 stations, 32 chains = 2048 solves per
    step on scratch-budget-capped waves (the runtime-kb fsm16 instance with
    32-brick z-blocks, each wave running several solves in its reused 128-MiB
    u / u0 fields).  Chain 0's init tables of 8 stations == the fp32 twin."""
    dev = _dev()
    torch.cuda.empty_cache()
    from mceik_amd import mcmc
    p = mcmc.make_problem("C5", picks="analytic")
    assert (p.nx, p.nstat, p.nevents) == (256, 64, 64)
    s = mcmc.Sampler(p, nchains=32)
    info = s.info()
    v0, _, _, _ = s.state()
    ttab, niter, _, ierr = s.last(with_ierr=True)
    s.run(1)                                          # a step of the same launch runs too
    s.close()
    assert info["step_z"] == 16 and info["kernel"] == "fsm16_solve_kernel<0, 4>", info
    assert sum(info["waves"]) < 32 * 64, info        # fewer resident waves than solves
    assert not ierr.any()
    P = O.make_problem(p)
    P.nstat = 8                                       # the first 8 stations (same arrays)
    tt, it = O.forward_f32(P, v0[0])
    assert np.array_equal(ttab[0, :8].view(np.uint32), tt.view(np.uint32))
    assert np.array_equal(niter[0, :8], it)


@pytest.mark.timeout(900)
def test_c5_bench_load_launch_bitwise():
    """C5 at the bench's per-GPU load: 256 chains x 64 stations at 256^3 =
    16384 solves per step on scratch-budget-capped waves in ONE pipe (the
    library refuses to split capped waves), several solves per wave.  Chains 0
    and 255, 8 stations each: the init tables and the first step's tables of
    the proposed models == the fp32 twin."""
    _dev()
    torch.cuda.empty_cache()
    from mceik_amd import mcmc
    p = mcmc.make_problem("C5", picks="analytic")
    s = mcmc.Sampler(p, nchains=256)
    info = s.info()
    assert info["npipe"] == 1 and info["kernel"] == "fsm16_solve_kernel<0, 4>", info
    assert sum(info["waves"]) < 256 * 64 / 4, info   # budget-capped: several solves per wave
    v0, _, _, _ = s.state()
    ttab0, niter0, _, ierr = s.last(with_ierr=True)
    assert not ierr.any()
    s.run(1)
    ttab1, niter1, _ = s.last()
    s.close()
    P = O.make_problem(p)
    P.nstat = 8                                       # the first 8 stations (same arrays)
    for c in (0, 255):
        tt, it = O.forward_f32(P, v0[c])
        assert np.array_equal(ttab0[c, :8].view(np.uint32), tt.view(np.uint32)), c
        assert np.array_equal(niter0[c, :8], it), c
        cell, vn, inp, _ = O.propose(P, c, 0, v0[c])
        vp = v0[c].copy()
        vp[cell] = vn                                 # the step forwards the proposed model
        tt, it = O.forward_f32(P, vp)
        assert np.array_equal(ttab1[c, :8].view(np.uint32), tt.view(np.uint32)), c
        assert np.array_equal(niter1[c, :8], it), c


def test_c3_mcmc_two_steps_bitwise():
    """Two MCMC steps of 2 chains at C3 geometry: accept sequence, logL trace
    and chain models bitwise = oracle_mcmc_run."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C3")
    p.dvmax = 400
    p.var[:] = 1e-6
    off, nch, nsteps = 517, 2, 2
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off)
    v0, logl0, _, _ = s.state()
    acc, trace = [], []
    for _ in range(nsteps):
        s.run(1)
        _, _, a = s.last()
        _, lg, _, _ = s.state()
        acc.append(a.copy())
        trace.append(lg.copy())
    v, logl, nacc, step = s.state()
    s.close()
    vo, lo, acco, traceo = O.mcmc_run(O.make_problem(p), v0, logl0, off, 0, nsteps)
    assert np.array_equal(np.array(acc), acco)
    assert np.array_equal(np.array(trace).view(np.uint64), traceo.view(np.uint64))
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert step == nsteps and nacc.sum() == acco.sum()


def test_c2_workload_sampled_chains():
    """C2: 256 chains x 16 stations at 64^3 in one sampler (4096 solves per
    step, more than the resident waves); chains 0-3 and 252-255 after two
    steps equal oracle_mcmc_run bitwise."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C2")
    assert (p.nx, p.nstat, p.nevents) == (64, 16, 16)
    p.dvmax = 400
    p.var[:] = 1e-6
    s = mcmc.Sampler(p, nchains=256)
    v0, logl0, _, _ = s.state()
    s.run(2)
    v, logl, _, _ = s.state()
    s.close()
    P = O.make_problem(p)
    for lo in (0, 252):
        sl = slice(lo, lo + 4)
        tt, _ = O.forward_f32(P, v0[lo])
        assert logl0[lo] == O.loglik(P, tt)
        vo, lgo, _, _ = O.mcmc_run(P, v0[sl], logl0[sl], lo, 0, 2)
        assert np.array_equal(v[sl], vo), lo
        assert np.array_equal(logl[sl].view(np.uint64), lgo.view(np.uint64)), lo


def test_c1_plumbing_100_proposals():
    """C1: 1 chain, 32^3 homogeneous (2000 m/s, h = 1000 m), 4 stations,
    4 events, 100 proposals through the sampler == oracle_mcmc_run."""
    _dev()
    from mceik_amd import mcmc
    p = _problem("C1")
    assert (p.nx, p.nstat, p.nevents, p.h) == (32, 4, 4, 1000.0)
    assert (p.v_true == 2000).all()
    p.dvmax = 400
    p.var[:] = 1e-4
    s = mcmc.Sampler(p, nchains=1)
    v0, logl0, _, _ = s.state()
    s.run(100)
    v, logl, nacc, step = s.state()
    s.close()
    vo, lo, acc, _ = O.mcmc_run(O.make_problem(p), v0, logl0, 0, 0, 100)
    assert step == 100
    assert np.array_equal(v, vo)
    assert np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    assert nacc[0] == acc.sum() and 0 < acc.sum() < 100


def _cells_field(nx, ny, nz, nref, seed):
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), nref)]
    v = np.random.default_rng(seed).integers(2500, 6500, (ncz, ncy, ncx)).astype(np.int32)
    scell = (1.0 / v.astype(np.float32)).astype(np.float32)
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return scell, scell[k // nref[2], j // nref[1], i // nref[0]].ravel()


def test_c5_256cube_fields_bitwise():
    """C5 geometry: two stations on a 256^3 cell model (runtime-kb kernel,
    32-brick z-blocks), both full fields and iteration counts == twin."""
    dev = _dev()
    n, h, nref = 256, 100.0, (4, 4, 4)
    scell, sfield = _cells_field(n, n, n, nref, 21)
    src = np.array([[[0.0, 12345.6, 6543.2, (n - 1) * h]], [[0.0, 3000.0, 22000.0, (n - 1) * h]]])
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(n, n, n, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(1, -1), device=dev), want_fields=True)
    u = out["u"].cpu().numpy().reshape(2, -1)
    niter = out["niter"].cpu().numpy()
    del out
    with cf.ThreadPoolExecutor(2) as ex:       # ctypes releases the GIL: 2 solves in parallel
        res = list(ex.map(lambda s: O.eikonal_solve(n, n, n, sfield, h, src[s], dtype=np.float32), range(2)))
    for s, (t, ierr, it) in enumerate(res):
        assert ierr == 0
        assert np.array_equal(u[s].view(np.uint32), t.view(np.uint32)), s
        assert int(niter[s]) == it


def test_cells_fast_many_solves_per_wave():
    """Production path at a moderate size: 16 models x 8 stations (40^3, cells,
    short sqrt, kb = 4) on 8 waves -- 16 solves per wave in its reused scratch
    (slot = wave, u0 guarded by the per-block epochs only); every table and
    iteration count == twin."""
    dev = _dev()
    n, h, nref, nmodel, nstat = 40, 100.0, (4, 4, 4), 16, 8
    rng = np.random.default_rng(4)
    cells, fields = zip(*[_cells_field(n, n, n, nref, 100 + m) for m in range(nmodel)])
    src = np.stack([np.array([[0.0, rng.uniform(250, 3650), rng.uniform(250, 3650), (n - 1) * h]])
                    for _ in range(nstat)])
    ev = rng.integers(0, n ** 3, 24).astype(np.int32)
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(n, n, n, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
    out = bs.solve(torch.tensor(src), torch.tensor(np.stack(cells).reshape(nmodel, -1), device=dev),
                   ev_node=torch.tensor(ev), max_waves=8)
    tt = out["ttab"].cpu().numpy().reshape(nmodel, nstat, -1)
    niter = out["niter"].cpu().numpy().reshape(nmodel, nstat)

    def twin(ms):
        m, s = ms
        return O.eikonal_solve(n, n, n, fields[m], h, src[s], dtype=np.float32)
    with cf.ThreadPoolExecutor(8) as ex:
        res = list(ex.map(twin, [(m, s) for m in range(nmodel) for s in range(nstat)]))
    for k, (t, _, it) in enumerate(res):
        m, s = divmod(k, nstat)
        assert np.array_equal(tt[m, s].view(np.uint32), t[ev].view(np.uint32)), (m, s)
        assert niter[m, s] == it, (m, s)
