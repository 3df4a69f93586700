"""GPU parity of the batched FSM kernel (libmceik_hip.so) against the oracle.

* fp32 path: BITWISE equal to the fp32 twin (oracle/fsm_impl.inc, STABLE_UPDATE),
  fields, iteration counts and ierr; within the stated tolerance of fp64.
* fp64 path: BITWISE equal to the reference's own outputs (tests/golden) and
  to the fp64 oracle.
On a mismatch the test bisects the sweep budget to name the first bad sweep.
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _solver(nx, ny, nz, h, precision, maxit=50, tol=1e-8, nref=None):
    from mceik_amd.eikonal import BatchSolver
    return BatchSolver(nx, ny, nz, h, 0.0, 0.0, 0.0, maxit, tol, precision, nref=nref)


def _hetero(nx, ny, nz):
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return 3000.0 + 4000.0 * k / (nz - 1) + 500.0 * np.sin(0.3 * i) * np.cos(0.25 * j) * np.sin(0.2 * k)


def _rough(nx, ny, nz, seed):
    return 2000.0 + 4000.0 * np.random.default_rng(seed).random((nz, ny, nx))


def _first_bad_sweep(nx, ny, nz, h, slow32, src, maxit, tol):
    """Smallest sweep budget at which GPU and twin differ (debug aid)."""
    dev = _dev()
    bs = _solver(nx, ny, nz, h, 32, maxit, tol)
    for ms in range(0, 8 * maxit + 1):
        out = bs.solve(torch.tensor(src[None]), torch.tensor(slow32.reshape(1, nz, ny, nx), device=dev),
                       want_fields=True, max_sweeps=ms)
        g = out["u"].cpu().numpy().ravel()
        t, _, _ = O.eikonal_solve(nx, ny, nz, slow32, h, src, maxit=maxit, tol=tol, dtype=np.float32,
                                  max_sweeps=ms)
        if not np.array_equal(g.view(np.uint32), t.view(np.uint32)):
            bad = np.flatnonzero(g.view(np.uint32) != t.view(np.uint32))
            i = bad[0]
            return ms, len(bad), (i % nx, (i // nx) % ny, i // (nx * ny)), g[i], t[i]
    return None


CASES = [
    # (name, nx, ny, nz, velocity, sources[(ts,xs,ys,zs)...], maxit, tol)
    ("hetero_16^3_top", 16, 16, 16, "hetero", [(0.0, 737.0, 689.0, 1500.0)], 50, 1e-8),
    ("hetero_17x19x23", 17, 19, 23, "hetero", [(0.0, 837.0, 889.0, 2200.0)], 50, 1e-8),
    ("rough_24x20x16_onnode", 24, 20, 16, "rough", [(0.0, 1100.0, 600.0, 900.0)], 50, 1e-8),
    ("rough_13x9x11_xmax", 13, 9, 11, "rough", [(0.25, 1200.0, 330.0, 470.0)], 50, 1e-8),
    ("hetero_21x18x15_2src", 21, 18, 15, "hetero", [(0.0, 420.0, 390.0, 200.0), (0.05, 1550.0, 1225.0, 1160.0)], 50, 1e-8),
    ("rough_9x10x8_loose", 9, 10, 8, "rough", [(0.0, 260.0, 710.0, 40.0)], 50, 1e-3),
    ("hetero_40x33x90_deep", 40, 33, 90, "hetero", [(0.0, 2050.0, 1630.0, 8900.0)], 50, 1e-8),
    ("rough_70x12x30_wide", 70, 12, 30, "rough", [(0.0, 10.0, 1100.0, 2900.0)], 50, 1e-8),
    ("hetero_33x41x25_maxit2", 33, 41, 25, "hetero", [(0.0, 1610.0, 2030.0, 1240.0)], 2, 1e-8),
]


def _case_slow(kind, nx, ny, nz, seed=1):
    v = _hetero(nx, ny, nz) if kind == "hetero" else _rough(nx, ny, nz, seed)
    return (1.0 / v).ravel()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fp32_bitwise_vs_twin(case):
    name, nx, ny, nz, kind, srcs, maxit, tol = case
    dev = _dev()
    h = 100.0
    slow32 = _case_slow(kind, nx, ny, nz).astype(np.float32)
    src = np.asarray(srcs, dtype=np.float64)
    bs = _solver(nx, ny, nz, h, 32, maxit, tol)
    out = bs.solve(torch.tensor(src[None]), torch.tensor(slow32.reshape(1, nz, ny, nx), device=dev),
                   want_fields=True)
    g = out["u"].cpu().numpy().ravel()
    t, ierr, it = O.eikonal_solve(nx, ny, nz, slow32, h, src, maxit=maxit, tol=tol, dtype=np.float32)
    if not np.array_equal(g.view(np.uint32), t.view(np.uint32)):
        pytest.fail(f"{name}: fields differ; first bad sweep: {_first_bad_sweep(nx, ny, nz, h, slow32, src, maxit, tol)}")
    assert int(out["niter"][0]) == it
    assert int(out["ierr"][0]) == ierr


def test_fp32_batch_many_models_and_stations():
    """nmodel x nstat solves in one launch (more solves than resident waves is
    not needed here; the work queue path is the same)."""
    dev = _dev()
    nx, ny, nz, h = 20, 18, 22, 100.0
    rng = np.random.default_rng(3)
    nmodel, nstat = 3, 5
    slows = np.stack([(1.0 / _rough(nx, ny, nz, 10 + m)).ravel().astype(np.float32) for m in range(nmodel)])
    src = np.stack([np.array([[0.0, rng.uniform(0, 1900), rng.uniform(0, 1700), rng.uniform(0, 2100)]])
                    for _ in range(nstat)])
    ev = rng.integers(0, nx * ny * nz, 7).astype(np.int32)
    bs = _solver(nx, ny, nz, h, 32)
    out = bs.solve(torch.tensor(src), torch.tensor(slows.reshape(nmodel, nz, ny, nx), device=dev),
                   ev_node=torch.tensor(ev), want_fields=True)
    u = out["u"].cpu().numpy().reshape(nmodel * nstat, -1)
    tt = out["ttab"].cpu().numpy()
    for m in range(nmodel):
        for s in range(nstat):
            t, ierr, it = O.eikonal_solve(nx, ny, nz, slows[m], h, src[s], dtype=np.float32)
            k = m * nstat + s
            assert np.array_equal(u[k].view(np.uint32), t.view(np.uint32)), (m, s)
            assert np.array_equal(tt[k].view(np.uint32), t[ev].view(np.uint32))
            assert int(out["niter"][k]) == it


@pytest.mark.parametrize("fast,nz", [(False, 34), (True, 34), (True, 20), (True, 67)],
                         ids=["exact_sqrt_kb4", "fast_kb4", "fast_kb3", "fast_kb4_ragged"])
def test_fp32_inversion_grid_mode_bitwise(fast, nz):
    """slow_mode 1: per-cell slowness (nref refinement) == twin on the expanded field.
    fast=True runs the sampler's kernel (LDS cell cache, short sqrt); nz >= 25
    gives 4-brick z-blocks (the compile-time-kb variant used at 128^3)."""
    dev = _dev()
    nx, ny, h, nref = 30, 26, 100.0, (4, 4, 4)
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), nref)]
    rng = np.random.default_rng(9)
    v = rng.integers(2500, 6500, (ncz, ncy, ncx)).astype(np.int32)
    scell = (1.0 / v.astype(np.float32)).astype(np.float32)
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    sfield = scell[k // nref[2], j // nref[1], i // nref[0]].ravel()
    src = np.array([[[0.0, 1234.5, 987.6, (nz - 1) * h]], [[0.0, 300.0, 2200.0, (nz - 1) * h]]])
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(nx, ny, nz, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=fast)
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(1, -1), device=dev), want_fields=True)
    # the fast cell-cache instance with even z-blocks runs the 16-z-step kernel
    assert out["step_z"] == (16 if fast and nz != 20 else 8)
    u = out["u"].cpu().numpy().reshape(2, -1)
    for s in range(2):
        t, _, it = O.eikonal_solve(nx, ny, nz, sfield, h, src[s], dtype=np.float32)
        assert np.array_equal(u[s].view(np.uint32), t.view(np.uint32)), s
        assert int(out["niter"][s]) == it


FP64_CASES = [c for c in CASES if c[0] in ("hetero_16^3_top", "rough_24x20x16_onnode", "rough_13x9x11_xmax",
                                           "hetero_21x18x15_2src", "rough_9x10x8_loose", "hetero_40x33x90_deep",
                                           "hetero_33x41x25_maxit2")]


@pytest.mark.parametrize("case", FP64_CASES, ids=[c[0] for c in FP64_CASES])
def test_fp64_batch_bitwise_vs_oracle(case):
    """The batched fp64 kernel (per-node slowness, the reference's literal
    update, fsm3d.f90:562-693): fields bitwise = the fp64 oracle (itself
    bitwise = the reference on tests/golden), iterations and ierr equal."""
    name, nx, ny, nz, kind, srcs, maxit, tol = case
    dev = _dev()
    h = 100.0
    slow64 = _case_slow(kind, nx, ny, nz)
    src = np.asarray(srcs, dtype=np.float64)
    bs = _solver(nx, ny, nz, h, 64, maxit, tol)
    out = bs.solve(torch.tensor(src[None]), torch.tensor(slow64.reshape(1, nz, ny, nx), device=dev),
                   want_fields=True)
    g = out["u"].cpu().numpy().ravel()
    t, ierr, it = O.eikonal_solve(nx, ny, nz, slow64, h, src, maxit=maxit, tol=tol)
    assert np.array_equal(g.view(np.uint64), t.view(np.uint64)), name
    assert int(out["niter"][0]) == it
    assert int(out["ierr"][0]) == ierr


F64_GRID = {"kb4": "fsm_solve_kernel<double, 2, false, 2, 1, 4>",
            "kb4_short_sqrt": "fsm_solve_kernel<double, 2, true, 2, 1, 4>",
            "kb4_short_sqrt_ragged_reuse": "fsm_solve_kernel<double, 2, true, 2, 1, 4>",
            "kb3_runtime_kb": "fsm_solve_kernel<double, 2, false, 2, 1, 0>",
            "over_1024_blocks": "fsm_solve_kernel<double, 2, false, 2, 1, 0>"}


@pytest.mark.parametrize("nz,max_waves,fast,nxy,case",
                         [(34, 0, False, None, "kb4"), (34, 0, True, None, "kb4_short_sqrt"),
                          (67, 2, True, None, "kb4_short_sqrt_ragged_reuse"), (20, 0, True, None, "kb3_runtime_kb"),
                          (32, 0, True, 264, "over_1024_blocks")],
                         ids=list(F64_GRID))
def test_fp64_inversion_grid_mode_bitwise(nz, max_waves, fast, nxy, case):
    """The fp64 sampler's kernel (bench.py --precision 64): per-cell fp32
    slowness, fp64 fields and the literal update.  Several models and stations
    per launch (max_waves 2: several solves per wave in reused scratch);
    fields, event tables, iterations bitwise = the fp64 oracle on the expanded
    field.  fast=True is the instance the sampler launches (the short sqrt,
    bare v_min/v_max_f64: fsm_update.h godunov_fast64) with the compact LDS
    layout (16-bit block clocks rebased per iteration, whole-line own loads);
    kb != 4 and more than 1024 z-blocks fall back to the runtime-kb instance."""
    dev = _dev()
    nx, ny, h, nref = 30, 26, 100.0, (4, 4, 4)
    if nxy:
        nx = ny = nxy
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), nref)]
    rng = np.random.default_rng(23)
    nmodel = 2
    v = rng.integers(2500, 6500, (nmodel, ncz, ncy, ncx)).astype(np.int32)
    scell = (1.0 / v.astype(np.float32)).astype(np.float32)
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    src = np.array([[[0.0, 1234.5, 987.6, (nz - 1) * h]], [[0.0, 300.0, 2200.0, (nz - 1) * h]],
                    [[0.1, 1500.0, 1200.0, 1700.0]]])
    if nxy:
        nmodel, v, scell, src = 1, v[:1], scell[:1], src[:1]
    ev = rng.integers(0, nx * ny * nz, 7).astype(np.int32)
    from mceik_amd.eikonal import BatchSolver
    from mceik_amd import _lib
    bs = BatchSolver(nx, ny, nz, h, 0.0, 0.0, 0.0, 50, 1e-8, 64, nref=nref, fast_sqrt=fast)
    kname = _lib.lib().mceik_fsm_kernel_name(C.byref(bs.describe(nmodel, len(src), 1, 1, nev=len(ev)))).decode()
    assert kname == F64_GRID[case], kname
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(nmodel, -1), device=dev),
                   ev_node=torch.tensor(ev), want_fields=True, max_waves=max_waves)
    assert out["step_z"] == 8
    u = out["u"].cpu().numpy().reshape(nmodel * len(src), -1)
    tt = out["ttab"].cpu().numpy()
    for m in range(nmodel):
        sfield = scell[m][k // nref[2], j // nref[1], i // nref[0]].ravel().astype(np.float64)
        for s in range(len(src)):
            t, ierr, it = O.eikonal_solve(nx, ny, nz, sfield, h, src[s])
            q = m * len(src) + s
            assert np.array_equal(u[q].view(np.uint64), t.view(np.uint64)), (m, s)
            assert np.array_equal(tt[q].view(np.uint32), t[ev].astype(np.float32).view(np.uint32)), (m, s)
            assert int(out["niter"][q]) == it and int(out["ierr"][q]) == ierr


def test_solve_order_and_clock():
    """A permuted work order (mceik_fsm_batch.solve_order) gives bitwise the
    same fields, tables and iteration counts; solve_clock stamps every solve."""
    dev = _dev()
    nx, ny, nz, h = 20, 18, 22, 100.0
    rng = np.random.default_rng(5)
    nmodel, nstat = 3, 4
    slows = np.stack([(1.0 / _rough(nx, ny, nz, 20 + m)).ravel().astype(np.float32) for m in range(nmodel)])
    src = np.stack([np.array([[0.0, rng.uniform(0, 1900), rng.uniform(0, 1700), rng.uniform(0, 2100)]])
                    for _ in range(nstat)])
    ev = torch.tensor(rng.integers(0, nx * ny * nz, 5).astype(np.int32))
    sl = torch.tensor(slows.reshape(nmodel, nz, ny, nx), device=dev)
    bs = _solver(nx, ny, nz, h, 32)
    a = bs.solve(torch.tensor(src), sl, ev_node=ev, want_fields=True)
    perm = rng.permutation(nmodel * nstat).astype(np.int32)
    b = bs.solve(torch.tensor(src), sl, ev_node=ev, want_fields=True, solve_order=perm, solve_clock=True)
    assert torch.equal(a["u"].view(torch.int32), b["u"].view(torch.int32))
    assert torch.equal(a["ttab"].view(torch.int32), b["ttab"].view(torch.int32))
    assert torch.equal(a["niter"], b["niter"])
    clk = b["clock"].cpu().numpy()
    assert (clk[:, 0] > 0).all() and (clk[:, 1] >= clk[:, 0]).all()
    with pytest.raises(ValueError):
        bs.solve(torch.tensor(src), sl, solve_order=np.zeros(nmodel * nstat, np.int32))


def test_fp32_inversion_grid_mode_8brick_blocks():
    """136 x 136 x 128: 17 x 17 tiles x 16 z-bricks would be 1156 four-brick
    z-blocks, more than the LDS block tables hold (MCEIK_MAX_BLOCKS = 1024), so
    the stream runs 8-brick blocks -- the runtime-kb kernel that the 256^3
    configuration (C5) uses.  Bitwise == twin on the expanded field."""
    dev = _dev()
    nx = ny = 136
    nz, h, nref = 128, 100.0, (4, 4, 4)
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), nref)]
    rng = np.random.default_rng(11)
    v = rng.integers(2500, 6500, (ncz, ncy, ncx)).astype(np.int32)
    scell = (1.0 / v.astype(np.float32)).astype(np.float32)
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    sfield = scell[k // nref[2], j // nref[1], i // nref[0]].ravel()
    src = np.array([[[0.0, 6543.2, 7012.3, (nz - 1) * h]]])
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(nx, ny, nz, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
    out = bs.solve(torch.tensor(src), torch.tensor(scell.reshape(1, -1), device=dev), want_fields=True)
    assert out["step_z"] == 16          # runtime-kb instance of the 16-z-step kernel (kb16 = 4)
    u = out["u"].cpu().numpy().reshape(1, -1)
    t, _, it = O.eikonal_solve(nx, ny, nz, sfield, h, src[0], dtype=np.float32)
    assert np.array_equal(u[0].view(np.uint32), t.view(np.uint32))
    assert int(out["niter"][0]) == it


STEP_CASES = [
    # (name, nx, ny, nz, nmodel, sources per station, max_waves)
    ("ragged_30x26x67", 30, 26, 67, 2, [(0.0, 1234.5, 987.6, 6600.0), (0.0, 300.0, 2200.0, 6600.0),
                                        (0.1, 1500.0, 1200.0, 3300.0)], 2),
    ("c2_64cube_reuse", 64, 64, 64, 2, [(0.0, 3100.5, 2950.2, 6300.0), (0.0, 700.0, 5400.0, 6300.0)], 1),
    ("tall_24x16x200", 24, 16, 200, 1, [(0.0, 1150.0, 730.0, 19900.0), (0.0, 400.0, 200.0, 10000.0)], 0),
    # 1024 tiles: 16-brick z-blocks with 128 cells each (the C5 instance's cell cache of 4 per lane)
    ("cells128_256x256x128", 256, 256, 128, 1, [(0.0, 12345.6, 6789.0, 12700.0), (0.0, 900.0, 24000.0, 12700.0)], 0),
]


@pytest.mark.parametrize("case", STEP_CASES, ids=[c[0] for c in STEP_CASES])
def test_fsm16_steps_equal_8z_kernel_bitwise(case):
    """The 16-z-step kernel (fsm16_kernel.hip, the sampler's instance) and the
    8-z kernel give bitwise the same fields, tables and iteration counts:
    ragged tiles and a cut last 16-z brick (generic path), sources on nodes
    and inside the grid, several solves per wave in reused scratch."""
    name, nx, ny, nz, nmodel, srcs, max_waves = case
    dev = _dev()
    h, nref = 100.0, (4, 4, 4)
    ncx, ncy, ncz = [-(-a // r) for a, r in zip((nx, ny, nz), nref)]
    rng = np.random.default_rng(17)
    v = rng.integers(2500, 6500, (nmodel, ncz, ncy, ncx)).astype(np.int32)
    scell = torch.tensor((1.0 / v.astype(np.float32)).reshape(nmodel, -1), device=dev)
    src = torch.tensor(np.asarray(srcs, dtype=np.float64)[:, None, :])
    ev = torch.tensor(rng.integers(0, nx * ny * nz, 9).astype(np.int32))
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(nx, ny, nz, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
    a = bs.solve(src, scell, ev_node=ev, want_fields=True, max_waves=max_waves)
    b = bs.solve(src, scell, ev_node=ev, want_fields=True, max_waves=max_waves, step_z=8)
    assert (a["step_z"], b["step_z"]) == (16, 8)
    assert torch.equal(a["u"].view(torch.int32), b["u"].view(torch.int32))
    assert torch.equal(a["ttab"].view(torch.int32), b["ttab"].view(torch.int32))
    assert torch.equal(a["niter"], b["niter"]) and torch.equal(a["ierr"], b["ierr"])
    assert not a["ierr"].any()


FSM_FILES = sorted(glob.glob(os.path.join(GOLD, "fsm_*.npz")))


@pytest.mark.parametrize("path", FSM_FILES, ids=[os.path.basename(p)[4:-4] for p in FSM_FILES])
def test_fp64_serial_driver_bitwise_vs_reference(path):
    """The drop-in eikonal3d_serial_driver reproduces the reference's own output bit for bit."""
    from mceik_amd.eikonal import eikonal3d_serial_driver
    _dev()
    g = dict(np.load(path, allow_pickle=False))
    nx, ny, nz = int(g["nx"]), int(g["ny"]), int(g["nz"])
    if "slow" in g:
        slow = g["slow"]
    elif str(g["velocity_formula"]) == "uniform":
        slow = np.full(nx * ny * nz, 1.0 / float(g["velocity_const"]))
    else:
        slow = (1.0 / _hetero(nx, ny, nz)).ravel()
    s = g["sources"]
    u = np.zeros(nx * ny * nz)
    args = (int(g["maxit"]), len(s), nx, ny, nz, float(g["tol"]), float(g["h"]), 0.0, 0.0, 0.0,
            s[:, 0], s[:, 1], s[:, 2], s[:, 3], slow, u)
    assert eikonal3d_serial_driver(1, 0, *args) == 0
    assert eikonal3d_serial_driver(1, 0, *args) == 1          # already initialised
    ierr = eikonal3d_serial_driver(2, 0, *args)
    eikonal3d_serial_driver(3, 0, *args)
    assert eikonal3d_serial_driver(2, 0, *args) == 1          # not initialised
    assert ierr == int(g["ierr"])
    if "u" in g:
        assert np.array_equal(u.view(np.uint64), g["u"].view(np.uint64))
    else:
        assert np.array_equal(u[g["sample_idx"]].view(np.uint64), g["sample_u"].view(np.uint64))
        if "xfsm3d" in path:
            assert u.max() == 1.4308203212738235


def test_fp32_serial_driver_within_tolerance():
    from mceik_amd.eikonal import eikonal3d_serial_driver
    _dev()
    g = dict(np.load(os.path.join(GOLD, "fsm_hetero_17x19x23.npz"), allow_pickle=False))
    nx, ny, nz = int(g["nx"]), int(g["ny"]), int(g["nz"])
    s = g["sources"]
    u = np.zeros(nx * ny * nz)
    args = (50, 1, nx, ny, nz, 1e-8, 100.0, 0.0, 0.0, 0.0, s[:, 0], s[:, 1], s[:, 2], s[:, 3], g["slow"], u)
    eikonal3d_serial_driver(1, 0, *args, precision=32)
    assert eikonal3d_serial_driver(2, 0, *args, precision=32) == 0
    eikonal3d_serial_driver(3, 0, *args, precision=32)
    ref = g["u"]
    assert np.all(np.abs(u - ref) <= 1e-6 * ref + 1e-7)


def test_fp32_128cube_vs_twin_and_fp64():
    """Headline grid size: two stations of one heterogeneous 128^3 model."""
    dev = _dev()
    n, h = 128, 100.0
    slow64 = (1.0 / _hetero(n, n, n)).ravel()
    slow32 = slow64.astype(np.float32)
    src = np.array([[[0.0, h * 64 + 37.0, h * 64 - 11.0, h * 127]], [[0.0, 2345.0, 9876.0, h * 127]]])
    bs = _solver(n, n, n, h, 32)
    out = bs.solve(torch.tensor(src), torch.tensor(slow32.reshape(1, n, n, n), device=dev), want_fields=True)
    u = out["u"].cpu().numpy().reshape(2, -1)
    for s in range(2):
        t, _, it = O.eikonal_solve(n, n, n, slow32, h, src[s], dtype=np.float32)
        assert np.array_equal(u[s].view(np.uint32), t.view(np.uint32)), s
        assert int(out["niter"][s]) == it
        r, _, _ = O.eikonal_solve(n, n, n, slow64, h, src[s])
        assert np.all(np.abs(u[s] - r) <= 1e-6 * r + 1e-7), s


def test_locate_l2_gpu_bitwise_vs_reference():
    from mceik_amd.eikonal import aligned_empty, locate_l2_gridsearch
    _dev()
    g = dict(np.load(os.path.join(GOLD, "locate_l2.npz"), allow_pickle=False))
    ld, ng, no = int(g["ldgrd"]), int(g["ngrd"]), int(g["nobs"])
    test = aligned_empty(g["test"].size); test[:] = g["test"]
    t0 = aligned_empty(ng); obj = aligned_empty(ng)
    assert locate_l2_gridsearch(ld, ng, no, 1, 0.0, g["mask"], g["tobs"], g["tcorr"], g["varobs"], test, t0, obj) == 0
    assert np.array_equal(t0.view(np.uint64), g["ot_t0"].view(np.uint64))
    assert np.array_equal(obj.view(np.uint64), g["ot_objfn"].view(np.uint64))
    assert locate_l2_gridsearch(ld, ng, no, 0, 4.0, np.zeros(no), g["tobs"], None, g["varobs"], test, t0, obj) == 0
    assert np.array_equal(obj.view(np.uint64), g["fixed_objfn"].view(np.uint64))
    # reference error behaviour: ldgrd*8 % 64 != 0
    assert locate_l2_gridsearch(ld + 1, ng, no, 1, 0.0, g["mask"], g["tobs"], None, g["varobs"], test, t0, obj) == 1


def test_locate_l2_f32_gpu_bitwise_vs_reference():
    """locate_l2_gridSearch__float64 drop-in vs the compiled reference (golden)."""
    from mceik_amd.eikonal import aligned_empty, locate_l2_gridsearch_f32
    _dev()
    g = dict(np.load(os.path.join(GOLD, "locate_l2_f32.npz"), allow_pickle=False))
    ld, ng, no = int(g["ldgrd"]), int(g["ngrd"]), int(g["nobs"])
    test = aligned_empty(g["test"].size, np.float32); test[:] = g["test"]
    t0 = aligned_empty(ng, np.float32); obj = aligned_empty(ng, np.float32)
    assert locate_l2_gridsearch_f32(ld, ng, no, 1, 0.0, g["mask"], g["tobs"], g["tcorr"], g["varobs"],
                                    test, t0, obj) == 0
    assert np.array_equal(t0.view(np.uint32), g["ot_t0"].view(np.uint32))
    assert np.array_equal(obj.view(np.uint32), g["ot_objfn"].view(np.uint32))
    assert locate_l2_gridsearch_f32(ld, ng, no, 0, 4.0, np.zeros(no), g["tobs"], None, g["varobs"],
                                    test, t0, obj) == 0
    assert np.array_equal(obj.view(np.uint32), g["fixed_objfn"].view(np.uint32))
    # the reference's checks: ldgrd*4 % 64 != 0 -> ierr 1
    assert locate_l2_gridsearch_f32(ld + 1, ng, no, 1, 0.0, g["mask"], g["tobs"], None, g["varobs"],
                                    test, t0, obj) == 1


@pytest.mark.parametrize("single_pass", [True, False], ids=["lds_single_pass", "two_pass"])
def test_relocate_batch_matches_reference_per_event(single_pass):
    """Batched relocation (all events against shared tables, one launch) equals
    the reference fp32 L2 grid search event by event (oracle restatement,
    itself pinned to locate.c by the golden test)."""
    from mceik_amd.eikonal import relocate
    dev = _dev()
    g = dict(np.load(os.path.join(GOLD, "locate_l2_f32.npz"), allow_pickle=False))
    ld, ng, no = int(g["ldgrd"]), int(g["ngrd"]), int(g["nobs"])
    tables = torch.tensor(g["test"].reshape(no, ld), device=dev)
    rng = np.random.default_rng(11)
    events = []
    for e in range(5):
        rows = rng.permutation(no)[: 6 + e]
        mask = (rng.random(rows.size) < 0.2).astype(np.int32)
        events.append(dict(rows=rows, tobs=g["tobs"][rows] + np.float32(0.3 * e), varobs=g["varobs"][rows],
                           tcorr=g["tcorr"][rows], mask=mask))
    out, t0 = relocate(tables, events, log_pdf=True, single_pass=single_pass)
    out = out.cpu().numpy(); t0 = t0.cpu().numpy()
    for e, ev in enumerate(events):
        sub_test = g["test"].reshape(no, ld)[ev["rows"]].ravel()
        ierr, rt0, robj = O.locate_l2_f32(ld, ng, len(ev["rows"]), 1, 0.0, ev["mask"], ev["tobs"], ev["tcorr"],
                                          ev["varobs"], sub_test)
        assert ierr == 0
        assert np.array_equal(t0[e, :ng].view(np.uint32), rt0.view(np.uint32))
        assert np.array_equal((-out[e, :ng]).view(np.uint32), robj.view(np.uint32))


def test_relocate_single_pass_c3_catalogue():
    """C3-sized relocation: 32 station tables on the 128^3 grid, 32 events x 32
    P picks; the single-pass LDS kernel == the two-pass kernel bitwise."""
    from mceik_amd.eikonal import relocate
    dev = _dev()
    n, nst, nev = 128, 32, 32
    ngrd = n ** 3
    g = torch.Generator(device=dev).manual_seed(3)
    tables = torch.rand((nst, ngrd), generator=g, device=dev) * 4.0
    rng = np.random.default_rng(7)
    events = [dict(rows=np.arange(nst), tobs=rng.uniform(1.0, 5.0, nst).astype(np.float32),
                   varobs=rng.uniform(0.5, 2.0, nst).astype(np.float32)) for _ in range(nev)]
    a, ta = relocate(tables, events, log_pdf=True, single_pass=True)
    b, tb = relocate(tables, events, log_pdf=True, single_pass=False)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert torch.equal(ta.view(torch.int32), tb.view(torch.int32))


@pytest.mark.parametrize("bad", ["nobs_short", "row_past_nrows"])
def test_relocate_single_pass_rejects_a_broken_contract(bad):
    """The single-pass kernel sizes its LDS from the caller's nobs / nrows: a
    caller whose ev_ptr[nev] != nobs or whose obs_row reaches past nrows gets
    NaN everywhere (no out-of-bounds LDS, no plausible misfits); the honest
    description of the same batch gives finite values."""
    import ctypes as C
    from mceik_amd import _lib
    dev = _dev()
    nrows, ld, nev = 6, 1024, 3
    tables = torch.rand((nrows, ld), device=dev)
    ptr = [0, 4, 9, 12]
    rows = [0, 1, 2, 3, 1, 2, 3, 4, 5, 0, 5, 2]
    nobs = len(rows)
    t = lambda a, dt: torch.tensor(np.asarray(a, dtype=dt), device=dev)
    d_ptr, d_rows = t(ptr, np.int32), t(rows, np.int32)
    d_tc, d_wt = t(np.linspace(1, 2, nobs), np.float32), t(np.ones(nobs), np.float32)
    d_xn = t([4.0, 5.0, 3.0], np.float32)
    out = torch.zeros((nev, ld), device=dev)
    t0 = torch.zeros((nev, ld), device=dev)

    def run(nr, no):
        b = _lib.RelocateBatch()
        b.ldgrd, b.ngrd, b.nev, b.iwantOT, b.t0use = ld, ld, nev, 1, 0.0
        b.tables, b.ev_ptr, b.obs_row = tables.data_ptr(), d_ptr.data_ptr(), d_rows.data_ptr()
        b.tc, b.wt, b.xnorm = d_tc.data_ptr(), d_wt.data_ptr(), d_xn.data_ptr()
        b.t0, b.out, b.log_pdf = t0.data_ptr(), out.data_ptr(), 1
        b.nrows, b.nobs = nr, no
        assert _lib.lib().mceik_relocate(C.byref(b), C.c_void_p(0)) == 0
        torch.cuda.synchronize(dev)
        return out.clone(), t0.clone()

    good, _ = run(nrows, nobs)
    assert torch.isfinite(good).all()
    o, z = run(nrows, nobs - 3) if bad == "nobs_short" else run(nrows - 2, nobs)
    assert torch.isnan(o).all() and torch.isnan(z).all()


def test_batch_solve_captured_in_a_graph_bitwise():
    """mceik_fsm_batch_solve only enqueues work (no allocation, no host sync;
    include/mceik_eikonal.h): captured once in a HIP graph (torch.cuda.graph)
    and replayed on new slowness, its tables and iteration counts are bitwise
    those of eager launches -- the sampler's 16-z cell-cache instance."""
    dev = _dev()
    from mceik_amd.eikonal import BatchSolver
    n, h, nref, nm = 40, 100.0, (4, 4, 4), 3
    nc = (n // 4) ** 3
    rng = np.random.default_rng(21)
    src = torch.tensor(np.stack([np.zeros(4), rng.uniform(200, 3700, 4), rng.uniform(200, 3700, 4),
                                 np.full(4, 3900.0)], 1)[:, None, :])
    ev = torch.tensor(rng.integers(0, n ** 3, 12).astype(np.int32))
    src, ev = src.to(dev), ev.to(dev)                   # no host copies inside the capture
    bs = BatchSolver(n, n, n, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
    models = [torch.tensor((1.0 / rng.integers(2500, 6500, (nm, nc))).astype(np.float32), device=dev) for _ in range(3)]
    eager = []
    for m in models:
        o = bs.solve(src, m, ev_node=ev)
        torch.cuda.synchronize()
        eager.append((o["ttab"].clone(), o["niter"].clone()))
    slow = models[0].clone()
    bs.solve(src, slow, ev_node=ev)                      # warm: workspace allocated outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = bs.solve(src, slow, ev_node=ev, stream=s.cuda_stream)
    for m, (tt, it) in zip(models, eager):
        slow.copy_(m)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out["ttab"].view(torch.int32), tt.view(torch.int32))
        assert torch.equal(out["niter"], it)
