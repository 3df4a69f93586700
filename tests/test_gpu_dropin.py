"""The drop-in entry points a single-call user links (fsm3d.f90 / gridsearch.f90
BIND(C) names) on the GPU:

* eikonal3d_serial_driver (fp64) and _sp now run ONE solve on the whole GPU
  (fsm_single.hip brick-level dataflow): bitwise the reference's golden
  fields (test_gpu_fsm.py) and here bitwise the fp64 oracle / fp32 twin on
  multi-source, ragged and repeated calls, with the device state kept from
  job 1 to job 3;
* eikonal3d_initialize / _solve / _finalize from a C caller (tests/c) in the
  flow of the reference's xfsm3d program: its known answer
  max u = 1.4308203212738235;
* locate3d_gridsearch__double64 / __float64 bitwise the compiled
  gridsearch.f90 (tests/golden/gridsearch_f90.npz), with its error checks.
"""
import os
import subprocess
import time

import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _hetero(nx, ny, nz):
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return 3000.0 + 4000.0 * k / (nz - 1) + 500.0 * np.sin(0.3 * i) * np.cos(0.25 * j) * np.sin(0.2 * k)


def _serial(nx, ny, nz, slow, src, maxit=50, tol=1e-8, h=100.0, precision=64, reps=1):
    from mceik_amd.eikonal import eikonal3d_serial_driver
    s = np.atleast_2d(src)
    u = np.zeros(nx * ny * nz)
    args = (maxit, len(s), nx, ny, nz, tol, h, 0.0, 0.0, 0.0, s[:, 0], s[:, 1], s[:, 2], s[:, 3], slow, u)
    assert eikonal3d_serial_driver(1, 0, *args, precision=precision) == 0
    times, outs = [], []
    for _ in range(reps):
        t = time.perf_counter()
        ierr = eikonal3d_serial_driver(2, 0, *args, precision=precision)
        times.append(time.perf_counter() - t)
        outs.append((u.copy(), ierr))
    eikonal3d_serial_driver(3, 0, *args, precision=precision)
    return outs, times


@pytest.mark.parametrize("precision", [64, 32])
def test_serial_driver_many_sources_ragged(precision):
    """12 sources (no source-count limit), a ragged 37 x 29 x 21 grid (partial
    bricks in x, y and z), called twice on the kept device state."""
    _dev()
    nx, ny, nz = 37, 29, 21
    rng = np.random.default_rng(8)
    slow = (1.0 / (2500.0 + 3500.0 * rng.random(nx * ny * nz)))
    src = np.stack([rng.uniform(0.02, 0.3, 12), rng.uniform(100, 3500, 12), rng.uniform(100, 2700, 12),
                    rng.uniform(100, 1900, 12)], 1)
    outs, _ = _serial(nx, ny, nz, slow, src, precision=precision, reps=2)
    dt = np.float64 if precision == 64 else np.float32
    ref, ierr, _ = O.eikonal_solve(nx, ny, nz, slow.astype(dt), 100.0, src, dtype=dt)
    for u, e in outs:
        assert e == ierr == 0
        if precision == 64:
            assert np.array_equal(u.view(np.uint64), ref.view(np.uint64))
        else:
            assert np.array_equal(u.astype(np.float32).view(np.uint32), ref.view(np.uint32))


def test_serial_driver_128cube_time_and_bitwise():
    """One 128^3 heterogeneous fp64 call, bitwise the fp64 oracle (the
    reference's arithmetic); wall time of warm calls printed (one call with the
    one-wave-per-solve kernel took ~0.8 s; the CPU reference 0.7-4 s)."""
    _dev()
    n = 128
    slow = (1.0 / _hetero(n, n, n)).ravel()
    src = np.array([0.0, 6437.0, 6389.0, 12700.0])
    outs, times = _serial(n, n, n, slow, src, reps=3)
    ref, ierr, it = O.eikonal_solve(n, n, n, slow, 100.0, src)
    for u, e in outs:
        assert e == ierr
        assert np.array_equal(u.view(np.uint64), ref.view(np.uint64))
    print(f"\nserial_driver 128^3 fp64: {it} iterations, call times {[round(t, 4) for t in times]} s")
    assert min(times) < 1.0


def test_mpi_variant_from_c_caller(tmp_path):
    _dev()
    exe = str(tmp_path / "xfsm3d_gpu")
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "xfsm3d_gpu.c"),
                    "-L", os.path.join(ROOT, "mceik_amd"), "-lmceik_hip", "-Wl,-rpath," + os.path.join(ROOT, "mceik_amd"),
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = {ln.split()[0]: ln.split() for ln in out.stdout.splitlines() if ln.strip()}
    assert float(lines["mpi_variant"][4]) == 1.4308203212738235
    assert float(lines["mpi_variant"][2]) == 0.0
    # without MPI in the process, a call with n < nx*ny*nz acts as a non-master rank
    assert lines["non_master"][2] == "0" and float(lines["non_master"][4]) == -1.0
    assert float(lines["serial_driver"][4]) == 1.4308203212738235


def test_mpi_variant_collective_contract_two_ranks(tmp_path):
    """tests/c/xfsm3d_mpi.c under mpiexec -n 2: rank 0's parameters reach every
    rank (rank 1 passes nonsense, fsm3d.f90:1626-1639); rank 0's SETBCS error
    (source on the first node) is every rank's ierr (:1792); the solve gives
    xfsm3d's known answer on rank 0 and leaves rank 1's u alone; finalizing
    twice reports the reference's ierr = 1 (:1913-1916) on every rank."""
    _dev()
    mpi = "/opt/conda"
    if not (os.path.exists(f"{mpi}/bin/mpiexec") and os.path.exists(f"{mpi}/lib/libmpi.so")):
        pytest.skip("no MPI toolchain in this image")
    exe = str(tmp_path / "xfsm3d_mpi")
    lib = os.path.join(ROOT, "mceik_amd")
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), "-I", f"{mpi}/include",
                    os.path.join(ROOT, "tests", "c", "xfsm3d_mpi.c"), "-L", lib, "-lmceik_hip",
                    f"{mpi}/lib/libmpi.so", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}:{mpi}/lib", "-lm",
                    "-o", exe], check=True)
    out = subprocess.run([f"{mpi}/bin/mpiexec", "-n", "2", exe], capture_output=True, text=True, timeout=120)
    print(out.stdout, out.stderr[-2000:])
    assert out.returncode == 0, out.stdout + out.stderr
    got = {}
    for ln in out.stdout.splitlines():
        w = ln.split()
        if len(w) >= 5 and w[1] == "rank":
            got[(w[0], int(w[2]))] = w
    for r in (0, 1):
        assert got[("init", r)][4] == "0"
        assert got[("origin", r)][4] == "1", r          # the master's SETBCS error on every rank
        assert got[("solve", r)][4] == "0", r
        assert got[("finalize", r)][4] == "0" and got[("refinalize", r)][4] == "1", r
    assert float(got[("solve", 0)][6]) == 1.4308203212738235     # xfsm3d's known answer
    assert float(got[("solve", 1)][6]) == -1.0                   # rank 1 holds no field


@pytest.mark.parametrize("prec", [64, 32])
def test_locate3d_gridsearch_bitwise_vs_reference(prec):
    from mceik_amd.eikonal import locate3d_gridsearch
    _dev()
    g = dict(np.load(os.path.join(GOLD, "gridsearch_f90.npz"), allow_pickle=False))
    ld, ng, no = int(g["ldgrd"]), int(g["ngrd"]), int(g["nobs"])
    dt = np.float64 if prec == 64 else np.float32
    ut = np.uint64 if prec == 64 else np.uint32
    for iw in (1, 0):
        lp = np.zeros(ng, dt)
        assert locate3d_gridsearch(ld, ng, no, iw, g["mask"], g["tobs"], g["varobs"], g["test"], lp) == 0
        assert np.array_equal(lp.view(ut), g[f"logpdf{prec}_ot{iw}"].view(ut)), iw
    lp = np.zeros(ld + 64, dt)
    big = np.zeros(no * (ld + 64))
    assert locate3d_gridsearch(ld + 1, ng, no, 1, g["mask"], g["tobs"], g["varobs"], big, lp) == g[f"ierr{prec}_ld"] == 1
    assert locate3d_gridsearch(ld, ld + 64, no, 1, g["mask"], g["tobs"], g["varobs"], big, lp) == g[f"ierr{prec}_ng"] == 1
    assert locate3d_gridsearch(ld, ng, no, 1, np.ones(no), g["tobs"], g["varobs"], g["test"], lp[:ng]) == \
        g[f"ierr{prec}_allmasked"] == 1


def test_c_sampler_main_config_checkpoint_gather(tmp_path):
    """tests/c/mcmc_main.c: a C main using only include/mceik.h -- INI config +
    argv overrides, sampler run to mcparms.niter, checkpoint -> restore in a
    second sampler continuing bitwise, and the RCCL checkpoint gather."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path / "mcmc_main")
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "mcmc_main.c"),
                    "-L", os.path.join(ROOT, "mceik_amd"), "-lmceik_hip", "-Wl,-rpath," + os.path.join(ROOT, "mceik_amd"),
                    "-lm", "-o", exe], check=True)
    ini = tmp_path / "run.ini"
    ini.write_text("[grid]\nnx = 24\nny = 20\nnz = 28\ndx = 100\ndy = 100\ndz = 100\n"
                   "nrefx = 4\nnrefy = 4\nnrefz = 4\n[eikonal]\ntol = 1e-8\nmaxit = 30\n"
                   "[mcmc]\nnchains = 6\nniter = 8\nnburnIn = 2\nkeepK = 1\nmax_samples = 2\n"
                   "dvmax = 300\nvmin = 2000\nvmax = 7000\n")
    out = subprocess.run([exe, "--config", str(ini), "mcmc:seed=77"], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    checks = {ln.split()[1]: ln.split()[2] for ln in out.stdout.splitlines() if ln.startswith("check ")}
    assert len(checks) == 6 and all(v == "1" for v in checks.values()), checks
    assert "chains 6 step 8" in out.stdout


@pytest.mark.parametrize("where", ["host", "device"])
def test_eikonal3d_batch_solve_plain_arguments(where):
    """eikonal3d_batch_solve (SURVEY s.8b's batched extension): 2 models x 3
    stations of per-node slowness, host or device arrays, every field, niter
    and ierr bitwise = the fp32 twin."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    from mceik_amd import _lib
    nx, ny, nz, h, nm, ns = 26, 21, 30, 100.0, 2, 3
    rng = np.random.default_rng(17)
    slow = (1.0 / rng.uniform(2500.0, 6500.0, (nm, nz, ny, nx))).astype(np.float32)
    src = np.stack([np.zeros(ns), rng.uniform(100, (nx - 2) * h, ns), rng.uniform(100, (ny - 2) * h, ns),
                    rng.uniform(100, (nz - 2) * h, ns)], 1)
    u = np.zeros((nm * ns, nz, ny, nx), np.float32)
    it = np.zeros(nm * ns, np.int32)
    ie = np.full(nm * ns, 7, np.int32)
    L = _lib.lib()
    if where == "host":
        args = [src.ctypes.data, slow.ctypes.data, u.ctypes.data, it.ctypes.data, ie.ctypes.data]
    else:
        t = [torch.tensor(a, device="cuda:0") for a in (src, slow, u, it, ie)]
        args = [x.data_ptr() for x in t]
    assert L.eikonal3d_batch_solve(nm, ns, nx, ny, nz, h, 0.0, 0.0, 0.0, 50, 1e-8, *args) == 0
    if where == "device":
        u, it, ie = t[2].cpu().numpy(), t[3].cpu().numpy(), t[4].cpu().numpy()
    for m in range(nm):
        for s in range(ns):
            tw, ierr, nit = O.eikonal_solve(nx, ny, nz, slow[m].ravel(), h, src[s], dtype=np.float32)
            k = m * ns + s
            assert np.array_equal(u[k].ravel().view(np.uint32), tw.view(np.uint32)), (m, s)
            assert it[k] == nit and ie[k] == ierr == 0


def test_c_mpi_sampler_main_one_rank(tmp_path):
    """tests/c/mpi_sampler_main.c under mpiexec -n 1: problem broadcast from
    rank 0 (broadcast.c's role), chains sharded by rank, RCCL id over
    MPI_Bcast, the kept states gathered to rank 0 by mceik_mcmc_gather.  (RCCL
    takes one rank per GPU: more ranks need more GPUs.)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mpi = "/opt/conda"
    if not (os.path.exists(f"{mpi}/bin/mpiexec") and os.path.exists(f"{mpi}/lib/libmpi.so")):
        pytest.skip("no MPI toolchain in this image")
    exe = str(tmp_path / "mpi_sampler_main")
    lib = os.path.join(ROOT, "mceik_amd")
    # the system libstdc++ ahead of conda's (libamdhip64 needs the newer one)
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), "-I", f"{mpi}/include",
                    os.path.join(ROOT, "tests", "c", "mpi_sampler_main.c"), "-L", lib, "-lmceik_hip",
                    f"{mpi}/lib/libmpi.so", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}:{mpi}/lib", "-lm",
                    "-o", exe], check=True)
    out = subprocess.run([f"{mpi}/bin/mpiexec", "-n", "1", exe, "grid:nx=24", "grid:ny=20", "grid:nz=28",
                          "grid:dx=100", "grid:dy=100", "grid:dz=100", "grid:nrefx=4", "grid:nrefy=4",
                          "grid:nrefz=4", "mcmc:nchains=5", "mcmc:niter=4", "mcmc:max_samples=1"],
                         capture_output=True, text=True, timeout=120)
    print(out.stdout, out.stderr[-2000:])
    assert out.returncode == 0, out.stdout + out.stderr
    assert "check gather_own_shard 1" in out.stdout and "ranks 1 chains 5" in out.stdout


def _blocks_golden():
    d = np.load(os.path.join(ROOT, "tests", "golden", "blocks_mpi.npz"))
    return d, sorted({k[:-4] for k in d.files if k.endswith("_cfg")})


def _mpi_variant(nx, ny, nz, nd, nov, maxit, tol, h, slow, src):
    import ctypes as C
    from mceik_amd import _lib
    L = _lib.lib()
    i = lambda v: C.byref(C.c_int(v))
    d = lambda v: C.byref(C.c_double(v))
    ierr = C.c_int(0)
    L.eikonal3d_initialize(i(0), i(0), i(nx), i(ny), i(nz), i(nd[0]), i(nd[1]), i(nd[2]), i(nov), i(maxit),
                           d(0.0), d(0.0), d(0.0), d(h), d(tol), C.byref(ierr))
    assert ierr.value == 0
    n = nx * ny * nz
    u = np.zeros(n)
    s = [np.array([v], dtype=np.float64) for v in src]
    slow = np.ascontiguousarray(slow, dtype=np.float64)
    L.eikonal3d_solve(i(0), i(1), i(n), *[x.ctypes.data_as(C.POINTER(C.c_double)) for x in s],
                      slow.ctypes.data_as(C.POINTER(C.c_double)), u.ctypes.data_as(C.POINTER(C.c_double)),
                      C.byref(ierr))
    e = ierr.value
    L.eikonal3d_finalize(i(0), C.byref(ierr))
    return u, e


@pytest.mark.parametrize("case", _blocks_golden()[1])
def test_mpi_variant_blocks_bitwise_vs_reference_mpi_runs(case):
    """eikonal3d_initialize/solve/finalize with ndivx x ndivy x ndivz blocks:
    the block-decomposed FSM (EIKONAL3D_FSM_MPI semantics, one workgroup per
    block on one GPU) bitwise = the reference's own solver run under mpiexec
    with one rank per block (tests/golden/blocks_mpi.npz), ierr included."""
    _dev()
    d, _ = _blocks_golden()
    nx, ny, nz = (int(v) for v in d["grid"])
    cfg = d[f"{case}_cfg"]
    u, ierr = _mpi_variant(nx, ny, nz, tuple(int(v) for v in cfg[:3]), int(cfg[3]), int(cfg[4]), 1e-8,
                           float(d["h"]), d["slow"], d[f"{case}_src"])
    assert ierr == int(d[f"{case}_ierr"])
    if f"{case}_u" in d.files:
        assert np.array_equal(u.view(np.uint64), d[f"{case}_u"].view(np.uint64))


def test_mpi_variant_blocks_xfsm3d_digest():
    """The reference's xfsm3d case (70x80x90, 2x2x2 blocks, maxit 5, tol 1e-7):
    the field's sha256 equals the reference's 8-rank MPI run."""
    import hashlib
    _dev()
    d, _ = _blocks_golden()
    n = (70, 80, 90)
    u, ierr = _mpi_variant(*n, (2, 2, 2), 1, 5, 1e-7, 100.0, np.full(n[0] * n[1] * n[2], 1.0 / 5.0e3),
                           [0.0] + [100.0 * v / 2.0 for v in n])
    assert ierr == 0 and u.max() == 1.4308203212738235
    assert hashlib.sha256(u.tobytes()).hexdigest() == str(d["xfsm3d_sha256"])


@pytest.fixture(scope="module")
def blocks_mpi_exe(tmp_path_factory):
    _dev()
    mpi = "/opt/conda"
    if not (os.path.exists(f"{mpi}/bin/mpiexec") and os.path.exists(f"{mpi}/lib/libmpi.so")):
        pytest.skip("no MPI toolchain in this image")
    exe = str(tmp_path_factory.mktemp("bmpi") / "blocks_mpi_gpu")
    lib = os.path.join(ROOT, "mceik_amd")
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), "-I", f"{mpi}/include",
                    os.path.join(ROOT, "tests", "c", "blocks_mpi_gpu.c"), "-L", lib, "-lmceik_hip",
                    f"{mpi}/lib/libmpi.so", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}:{mpi}/lib", "-lm",
                    "-o", exe], check=True)
    return f"{mpi}/bin/mpiexec", exe


def _run_blocks_ranks(blocks_mpi_exe, tmp_path, n3, nd, nov, maxit, tol, h, slow, src):
    mpiexec, exe = blocks_mpi_exe
    sp, op = str(tmp_path / "slow.f64"), str(tmp_path / "u.f64")
    np.ascontiguousarray(slow, dtype=np.float64).tofile(sp)
    cmd = [mpiexec, "-n", str(nd[0] * nd[1] * nd[2]), exe, *map(str, n3), *map(str, nd), str(nov), str(maxit),
           repr(tol), repr(h), "0", "0", "0", *map(repr, (float(v) for v in src)), sp, op]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    print(out.stdout[-3000:], out.stderr[-2000:])
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    ranks = {int(ln.split()[1]): int(ln.split()[3]) for ln in out.stdout.splitlines() if ln.startswith("rank ")}
    assert sorted(ranks) == list(range(nd[0] * nd[1] * nd[2]))
    res = np.fromfile(op)
    return res[:-1], int(res[-1]), ranks


@pytest.mark.parametrize("case", _blocks_golden()[1])
def test_mpi_variant_blocks_across_ranks_bitwise_vs_reference(blocks_mpi_exe, tmp_path, case):
    """The distributed MPI variant (one rank per block, each sweeping its block
    on the GPU and swapping face layers with its neighbours after every sweep
    -- host-staged MPI here, the ranks sharing one GPU -- the master gathering
    u) under mpiexec with ndivx*ndivy*ndivz ranks: u and the master's ierr
    bitwise = the reference's own run with the same ranks and arguments
    (tests/golden/blocks_mpi.npz); SETBCS's error reaches every rank."""
    d, _ = _blocks_golden()
    cfg = d[f"{case}_cfg"]
    nd = tuple(int(v) for v in cfg[:3])
    u, ierr, ranks = _run_blocks_ranks(blocks_mpi_exe, tmp_path, tuple(int(v) for v in d["grid"]), nd, int(cfg[3]),
                                       int(cfg[4]), 1e-8, float(d["h"]), d["slow"], d[f"{case}_src"])
    assert ierr == ranks[0] == int(d[f"{case}_ierr"])
    if case.endswith("_err"):
        assert all(e == 1 for e in ranks.values()), ranks
    if f"{case}_u" in d.files:
        assert np.array_equal(u.view(np.uint64), d[f"{case}_u"].view(np.uint64))


def test_mpi_variant_xfsm3d_eight_ranks_digest(blocks_mpi_exe, tmp_path):
    """The reference's xfsm3d case (70x80x90, 2x2x2 blocks, maxit 5, tol 1e-7)
    on 8 ranks, one block each: the gathered field's sha256 equals the
    reference's 8-rank MPI run."""
    import hashlib
    d, _ = _blocks_golden()
    n3 = (70, 80, 90)
    u, ierr, ranks = _run_blocks_ranks(blocks_mpi_exe, tmp_path, n3, (2, 2, 2), 1, 5, 1e-7, 100.0,
                                       np.full(n3[0] * n3[1] * n3[2], 1.0 / 5.0e3),
                                       [0.0] + [100.0 * v / 2.0 for v in n3])
    assert ierr == 0 and u.max() == float(d["xfsm3d_max"]) == 1.4308203212738235
    assert hashlib.sha256(u.tobytes()).hexdigest() == str(d["xfsm3d_sha256"])


def test_mpi_variant_uneven_blocks_across_ranks_vs_one_gpu(blocks_mpi_exe, tmp_path):
    """A 3 x 2 x 1 decomposition with uneven blocks (the last block takes the
    remainder, fsm3d.f90:1096-1098) and a two-node ghost layer on 6 ranks:
    bitwise = the same decomposition run on one GPU (the single-process block
    iteration pinned by the reference goldens above)."""
    d, _ = _blocks_golden()
    n3 = tuple(int(v) for v in d["grid"])
    src = d["b222_src"]
    u, ierr, ranks = _run_blocks_ranks(blocks_mpi_exe, tmp_path, n3, (3, 2, 1), 2, 50, 1e-8, float(d["h"]),
                                       d["slow"], src)
    u1, e1 = _mpi_variant(*n3, (3, 2, 1), 2, 50, 1e-8, float(d["h"]), d["slow"], src)
    assert ierr == e1 == 0
    assert np.array_equal(u.view(np.uint64), u1.view(np.uint64))


def test_mpi_variant_rccl_halo_refused_on_shared_gpu(blocks_mpi_exe, tmp_path):
    """MCEIK_HALO=rccl with two ranks on one GPU: RCCL refuses the
    communicator (one rank per GPU), and initialize returns ierr = 1 on both
    ranks together instead of leaving one waiting in a collective."""
    mpiexec, exe = blocks_mpi_exe
    d, _ = _blocks_golden()
    sp = str(tmp_path / "slow.f64")
    d["slow"].tofile(sp)
    env = dict(os.environ, MCEIK_HALO="rccl")
    out = subprocess.run([mpiexec, "-n", "2", exe, *map(str, d["grid"]), "2", "1", "1", "1", "50", "1e-8", "100",
                          "0", "0", "0", "0", "834.5", "987.6", "1100", sp, str(tmp_path / "u.f64")],
                         capture_output=True, text=True, timeout=120, env=env)
    print(out.stdout[-2000:], out.stderr[-2000:])
    assert out.returncode == 0
    assert "rank 0 init_ierr 1" in out.stdout and "rank 1 init_ierr 1" in out.stdout
