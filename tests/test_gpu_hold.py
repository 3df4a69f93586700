"""Held-stream stress: the sampler instances of both sweep
kernels -- fsm16_kernel.hip (fp32, 16-z steps) and the compact-layout fp64
instance of fsm_kernel.hip -- visit a z-block only when a settled change
reached it.  That is exact only if every sweep leaves the field the full
sweep would have left, so these tests stop the solve after EVERY sweep budget
(max_sweeps = 1, 2, ...) and compare the partial field with the oracle's
full-sweep twin after the same number of sweeps (fsm3d.f90:28-99: the eight
sweeps of an iteration, each over every node), bitwise.

The models are high-contrast (per 4^3 cell: slow inclusions of 700 m/s in
a 6500 m/s medium, or fast 9000 m/s channels in a 1500 m/s one): fronts bend
around them, so changes travel back upwind for many sweeps and blocks are
held, released and revisited in every sweep direction.  Several solves share one wave (max_waves 1): the held
stream's LDS state must be reset between solves.  maxit 2 / 3 cut the solve
before convergence (iterations and ierr compared too).
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

NREF = (4, 4, 4)
H = 100.0


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _inclusions(nmodel, ncz, ncy, ncx, seed):
    """Per-cell velocities: even models 6500 m/s with ~12% of the cells at
    700 m/s (slow inclusions), odd models 1500 m/s with ~30% at 9000 m/s
    (fast channels: head waves run back upwind, 6 iterations)."""
    rng = np.random.default_rng(seed)
    v = np.empty((nmodel, ncz, ncy, ncx), np.int32)
    for m in range(nmodel):
        base, inc, frac = (6500, 700, 0.12) if m % 2 == 0 else (1500, 9000, 0.30)
        v[m] = base
        v[m][rng.random(v[m].shape) < frac] = inc
    return v


def _expand(scell_m, nx, ny, nz):
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return scell_m[k // NREF[2], j // NREF[1], i // NREF[0]].ravel()


def _problem(nx, ny, nz, nmodel, seed):
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), NREF)]
    v = _inclusions(nmodel, ncz, ncy, ncx, seed)
    scell = (1.0 / v.astype(np.float32)).astype(np.float32)
    src = np.array([[[0.0, 0.37 * (nx - 1) * H, 0.61 * (ny - 1) * H, (nz - 1) * H]],
                    [[0.2, 0.83 * (nx - 1) * H, 0.12 * (ny - 1) * H, 0.45 * (nz - 1) * H]]])
    return scell, src


def _batch(nx, ny, nz, precision, maxit):
    from mceik_amd.eikonal import BatchSolver
    return BatchSolver(nx, ny, nz, H, 0.0, 0.0, 0.0, maxit, 1e-8, precision, nref=NREF, fast_sqrt=True)


def _check(out, scell, src, nx, ny, nz, precision, maxit, max_sweeps=-1):
    ut = np.uint32 if precision == 32 else np.uint64
    dt = np.float32 if precision == 32 else np.float64
    nmodel, nstat = scell.shape[0], len(src)
    u = out["u"].cpu().numpy().reshape(nmodel * nstat, -1)
    for m in range(nmodel):
        sfield = _expand(scell[m], nx, ny, nz).astype(dt)
        for s in range(nstat):
            t, ierr, it = O.eikonal_solve(nx, ny, nz, sfield, H, src[s], maxit=maxit, tol=1e-8, dtype=dt,
                                          max_sweeps=max_sweeps)
            q = m * nstat + s
            bad = np.flatnonzero(u[q].view(ut) != t.view(ut))
            assert bad.size == 0, (f"sweeps {max_sweeps}, model {m}, station {s}: {bad.size} nodes differ, "
                                   f"first {bad[0]} gpu {u[q][bad[0]]!r} twin {t[bad[0]]!r}")
            if max_sweeps < 0:
                assert int(out["niter"][q]) == it and int(out["ierr"][q]) == ierr, (m, s)
    return out


# (precision, grid, the kernel the sampler runs at that precision)
CASES = [(32, (30, 26, 67), 16), (64, (30, 26, 67), 8)]


@pytest.mark.parametrize("precision,grid,step_z", CASES, ids=["fp32_fsm16", "fp64_compact"])
def test_held_stream_every_sweep_budget(precision, grid, step_z):
    """Partial fields after every sweep budget up to convergence, bitwise =
    the full-sweep twin (fp32: the stable-update twin; fp64: the reference's
    arithmetic)."""
    dev = _dev()
    nx, ny, nz = grid
    scell, src = _problem(nx, ny, nz, 2, 31)
    bs = _batch(nx, ny, nz, precision, 50)
    sl = torch.tensor(scell.reshape(2, -1), device=dev)
    full = bs.solve(torch.tensor(src), sl, want_fields=True, max_waves=1)
    assert full["step_z"] == step_z
    _check(full, scell, src, nx, ny, nz, precision, 50)
    niter = int(full["niter"].max())
    assert niter >= 4, niter          # the inclusions make the fronts travel back upwind
    for ms in range(1, 8 * niter + 1):
        out = bs.solve(torch.tensor(src), sl, want_fields=True, max_waves=1, max_sweeps=ms)
        _check(out, scell, src, nx, ny, nz, precision, 50, max_sweeps=ms)


@pytest.mark.parametrize("precision", [32, 64], ids=["fp32_fsm16", "fp64_compact"])
@pytest.mark.parametrize("maxit", [2, 3])
def test_held_stream_maxit_cut(precision, maxit):
    """maxit below the iterations the model needs: the held stream stops at
    the same iteration as the reference, same field, niter and ierr."""
    dev = _dev()
    nx, ny, nz = 34, 29, 34
    scell, src = _problem(nx, ny, nz, 2, 47)
    bs = _batch(nx, ny, nz, precision, maxit)
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(2, -1), device=dev), want_fields=True)
    assert out["step_z"] == (16 if precision == 32 else 8)
    _check(out, scell, src, nx, ny, nz, precision, maxit)
    assert int(out["niter"].max()) == maxit


def test_held_stream_runtime_kb_budgets():
    """The runtime-kb instance of the 16-z kernel (C5's: 136 x 136 x 128 has
    more z-blocks of 32 z than the LDS block tables hold, so the stream runs
    64-z blocks): partial fields after a spread of sweep budgets, bitwise =
    the full-sweep twin."""
    dev = _dev()
    nx = ny = 136
    nz = 128
    scell, src = _problem(nx, ny, nz, 2, 59)
    scell, src = scell[1:], src[:1]                    # the fast-channel model, one station
    bs = _batch(nx, ny, nz, 32, 50)
    sl = torch.tensor(scell.reshape(1, -1), device=dev)
    full = bs.solve(torch.tensor(src), sl, want_fields=True)
    assert full["step_z"] == 16
    import ctypes as C
    from mceik_amd import _lib
    kname = _lib.lib().mceik_fsm_kernel_name(C.byref(bs.describe(1, 1, 1, 1))).decode()
    assert kname.startswith("fsm16_solve_kernel<0"), kname       # runtime kb
    _check(full, scell, src, nx, ny, nz, 32, 50)
    nsw = 8 * int(full["niter"].max())
    for ms in sorted({1, 2, 3, 5, 8, 9, 13, 16, 21, nsw // 2, nsw - 1}):
        if ms < nsw:
            out = bs.solve(torch.tensor(src), sl, want_fields=True, max_sweeps=ms)
            _check(out, scell, src, nx, ny, nz, 32, 50, max_sweeps=ms)


@pytest.mark.parametrize("precision", [32, 64], ids=["fp32_fsm16", "fp64_compact"])
@pytest.mark.parametrize("tol", [1e-3, 1e-12], ids=["tol1e-3", "tol1e-12"])
def test_convergence_paths_tol(precision, tol):
    """The convergence test's two paths under the held stream: with tol 1e-3
    no update is big enough to prove an iteration unconverged on its own
    (fp32: T = tol 2^24 s exceeds every travel time), so every iteration
    ends in the verify against the u0 copies; with tol 1e-12 nearly every
    change proves it, and once a wave knows, the rest of the iteration runs
    without the test or the u0 copies (MCEIK16_NC_SKIP / MCEIK8_NC_SKIP).
    Fields, iterations and ierr bitwise = the twin either way."""
    dev = _dev()
    nx, ny, nz = 30, 26, 67
    scell, src = _problem(nx, ny, nz, 2, 71)
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(nx, ny, nz, H, 0.0, 0.0, 0.0, 50, tol, precision, nref=NREF, fast_sqrt=True)
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(2, -1), device=dev), want_fields=True,
                   max_waves=1)
    ut = np.uint32 if precision == 32 else np.uint64
    dt = np.float32 if precision == 32 else np.float64
    u = out["u"].cpu().numpy().reshape(4, -1)
    for m in range(2):
        sfield = _expand(scell[m], nx, ny, nz).astype(dt)
        for s in range(2):
            t, ierr, it = O.eikonal_solve(nx, ny, nz, sfield, H, src[s], maxit=50, tol=tol, dtype=dt)
            q = m * 2 + s
            assert np.array_equal(u[q].view(ut), t.view(ut)), (m, s)
            assert int(out["niter"][q]) == it and int(out["ierr"][q]) == ierr, (m, s, int(out["niter"][q]), it)
