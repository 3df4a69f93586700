#!/usr/bin/env python3
"""Generate golden vectors from the COMPILED REFERENCE (this container only).

Runs oracle/_ref/libfsm3d_ref.so (the reference's own fsm3d.f90 serial driver,
fsm3d.f90:1968-2052) and oracle/_ref/liblocate_ref.so (locate.c:923-1047), both
built from /root/reference by oracle/build_ref.sh, on small deterministic
inputs and writes inputs + outputs as .npz fixtures next to this script.
Only these data files are committed; the reference never travels.

Usage:  python tests/golden/make_golden.py        (rewrites tests/golden/*.npz)
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class RefFSM:
    """ctypes view of eikonal3d_serial_driver (all args by reference, fsm3d.f90:1968-1983)."""

    def __init__(self):
        self.lib = C.CDLL(os.path.join(REF, "libfsm3d_ref.so"))
        self.f = self.lib.eikonal3d_serial_driver

    def call(self, job, nx, ny, nz, slow, h, src, maxit=50, tol=1e-8, x0=0.0, y0=0.0, z0=0.0):
        i = lambda v: C.byref(C.c_int(v))
        d = lambda v: C.byref(C.c_double(v))
        src = np.atleast_2d(np.asarray(src, dtype=np.float64))
        ts = np.ascontiguousarray(src[:, 0]); xs = np.ascontiguousarray(src[:, 1])
        ys = np.ascontiguousarray(src[:, 2]); zs = np.ascontiguousarray(src[:, 3])
        u = np.zeros(nx * ny * nz)
        ierr = C.c_int(0)
        self.f(i(job), i(0), i(maxit), i(len(ts)), i(nx), i(ny), i(nz), d(tol), d(h),
               d(x0), d(y0), d(z0), _ptr(ts), _ptr(xs), _ptr(ys), _ptr(zs),
               _ptr(slow), _ptr(u), C.byref(ierr))
        return u, ierr.value

    def solve(self, nx, ny, nz, slow, h, src, **kw):
        _, e1 = self.call(1, nx, ny, nz, slow, h, src, **kw)
        assert e1 == 0
        u, ierr = self.call(2, nx, ny, nz, slow, h, src, **kw)
        self.call(3, nx, ny, nz, slow, h, src, **kw)
        return u, ierr


def hetero_velocity(nx, ny, nz):
    """Survey probe model v = 3000 + 4000 k/(nz-1) + 500 sin(.3i) cos(.25j) sin(.2k), x fastest."""
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return 3000.0 + 4000.0 * k / (nz - 1) + 500.0 * np.sin(0.3 * i) * np.cos(0.25 * j) * np.sin(0.2 * k)


def rough_velocity(nx, ny, nz, seed):
    rng = np.random.default_rng(seed)
    return 2000.0 + 4000.0 * rng.random((nz, ny, nx))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def fsm_cases():
    h = 100.0
    cases = []
    # (name, dims, velocity, h, sources[(ts,xs,ys,zs)], maxit, tol, store_full)
    n = (17, 19, 23)
    cases.append(("hetero_17x19x23", n, hetero_velocity(*n), h,
                  [(0.0, h * 8 + 37.0, h * 9 - 11.0, h * (n[2] - 1))], 50, 1e-8, True))
    n = (32, 32, 32)
    cases.append(("homog_32_onnode_top", n, np.full(n[::-1], 2000.0), 1000.0,
                  [(0.0, 13000.0, 7000.0, 31000.0)], 50, 1e-8, True))
    n = (24, 20, 16)
    cases.append(("rough_24x20x16_onnode_interior", n, rough_velocity(*n, 7), h,
                  [(0.0, h * 11, h * 6, h * 9)], 50, 1e-8, True))
    n = (13, 9, 11)
    cases.append(("rough_13x9x11_xmax_edge", n, rough_velocity(*n, 11), h,
                  [(0.25, h * (n[0] - 1), h * 3.3, h * 4.7)], 50, 1e-8, True))
    cases.append(("rough_13x9x11_beyond_xmax_err", n, rough_velocity(*n, 11), h,
                  [(0.0, h * (n[0] - 1) + 5.0, h * 3.3, h * 4.7)], 50, 1e-8, True))
    cases.append(("rough_13x9x11_at_origin_err", n, rough_velocity(*n, 11), h,
                  [(0.0, 0.0, h * 3.3, h * 4.7)], 50, 1e-8, True))
    n = (21, 18, 15)
    cases.append(("hetero_21x18x15_two_sources", n, hetero_velocity(*n), h,
                  [(0.0, h * 4.2, h * 3.9, h * 2.0), (0.05, h * 15.5, h * 12.25, h * 11.6)],
                  50, 1e-8, True))
    cases.append(("hetero_21x18x15_maxit1", n, hetero_velocity(*n), h,
                  [(0.0, h * 10.4, h * 8.8, h * 14.0)], 1, 1e-8, True))
    n = (9, 10, 8)
    cases.append(("rough_9x10x8_tol_loose", n, rough_velocity(*n, 3), h,
                  [(0.0, h * 2.6, h * 7.1, h * 0.4)], 50, 1e-3, True))
    n = (64, 64, 64)
    cases.append(("hetero_64_probe", n, hetero_velocity(*n), h,
                  [(0.0, h * 32 + 37.0, h * 32 - 11.0, h * 63)], 100, 1e-8, False))
    # the reference's own xfsm3d test (fsm3d.f90:2085-2146): known max 1.4308203212738235
    n = (70, 80, 90)
    cases.append(("xfsm3d_70x80x90", n, np.full(n[::-1], 5000.0), h,
                  [(0.0, h * 70 / 2.0, h * 80 / 2.0, h * 90 / 2.0)], 5, 1e-7, False))
    return cases


def make_fsm(ref):
    for name, (nx, ny, nz), vel, h, srcs, maxit, tol, full in fsm_cases():
        slow = np.ascontiguousarray((1.0 / vel).ravel(), dtype=np.float64)
        u, ierr = ref.solve(nx, ny, nz, slow, h, srcs, maxit=maxit, tol=tol)
        out = dict(nx=nx, ny=ny, nz=nz, h=h, x0=0.0, y0=0.0, z0=0.0, maxit=maxit, tol=tol,
                   sources=np.asarray(srcs, dtype=np.float64), ierr=ierr,
                   umin=u.min(), umax=u.max(), sha256=sha(u))
        if full:
            out["slow"] = slow
            out["u"] = u
        else:
            out["velocity_formula"] = "uniform" if np.all(vel == vel.flat[0]) else "hetero_probe"
            out["velocity_const"] = float(vel.flat[0])
            idx = np.arange(0, u.size, 97, dtype=np.int64)
            out["sample_idx"] = idx
            out["sample_u"] = u[idx]
        np.savez_compressed(os.path.join(HERE, f"fsm_{name}.npz"), **out)
        print(f"fsm_{name}: ierr={ierr} umax={u.max()!r}")


def make_gridsearch():
    """gridsearch.f90:382-540 (locate3d_gridsearch__double64 / __float64, the
    Fortran misfit variant) from oracle/_ref/libgridsearch_ref.so: straight-ray
    tables on a 31 x 27 x 9 grid, 12 stations, unequal variances, one masked
    observation and one mask value other than 0/1 (counts as used:
    gridsearch.f90:432 tests mask /= 1), with and without the origin time."""
    lib = C.CDLL(os.path.join(REF, "libgridsearch_ref.so"))
    nx, ny, nz, nobs, dx = 31, 27, 9, 12, 1.0e3
    ngrd = nx * ny * nz
    ldgrd = ngrd + 64 - ngrd % 64
    rng = np.random.default_rng(2024)
    rec = rng.random((nobs, 3)) * (np.array([nx, ny, nz]) - 1) * dx
    src = np.array([13.0, 19.0, 4.0]) * dx
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    pts = np.stack([i.ravel(), j.ravel(), k.ravel()], 1) * dx
    test = np.zeros(nobs * ldgrd)
    for o in range(nobs):
        test[o * ldgrd:o * ldgrd + ngrd] = np.sqrt(((pts - rec[o]) ** 2).sum(1)) / 5.0e3
    tobs = np.sqrt(((rec - src) ** 2).sum(1)) / 5.0e3 + 4.0 + rng.normal(0.0, 0.01, nobs)
    varobs = rng.uniform(0.5, 2.0, nobs)
    mask = np.zeros(nobs, np.int32)
    mask[3] = 1
    mask[7] = 2
    ip = lambda v: C.byref(C.c_int(v))
    out = dict(ldgrd=ldgrd, ngrd=ngrd, nobs=nobs, test=test, tobs=tobs, varobs=varobs, mask=mask)
    for prec, name in ((64, "locate3d_gridsearch__double64"), (32, "locate3d_gridsearch__float64")):
        dt = np.float64 if prec == 64 else np.float32
        f = getattr(lib, name)
        for iw in (1, 0):
            lp = np.zeros(ngrd, dt)
            ierr = C.c_int(-1)
            t, to, va = (np.ascontiguousarray(a, dtype=dt) for a in (test, tobs, varobs))
            f(ip(ldgrd), ip(ngrd), ip(nobs), ip(iw), _ptr(mask), _ptr(to), _ptr(va), _ptr(t), _ptr(lp),
              C.byref(ierr))
            assert ierr.value == 0
            out[f"logpdf{prec}_ot{iw}"] = lp
            print(f"gridsearch f{prec} iwantOT={iw}: argmin={int(np.argmin(lp))} true={(4 * ny + 19) * nx + 13}")
        # the reference's checks (ierr = 1): ldgrd % 64, ngrd > ldgrd, every observation masked
        for tag, args in (("ld", (ldgrd + 1, ngrd)), ("ng", (ldgrd, ldgrd + 64))):
            ierr = C.c_int(-1)
            lp = np.zeros(ldgrd + 64, dt)
            t, to, va = (np.ascontiguousarray(a, dtype=dt) for a in (np.zeros(nobs * (ldgrd + 64)), tobs, varobs))
            f(ip(args[0]), ip(args[1]), ip(nobs), ip(1), _ptr(mask), _ptr(to), _ptr(va), _ptr(t), _ptr(lp),
              C.byref(ierr))
            out[f"ierr{prec}_{tag}"] = ierr.value
        allm = np.ones(nobs, np.int32)
        ierr = C.c_int(-1)
        lp = np.zeros(ngrd, dt)
        t, to, va = (np.ascontiguousarray(a, dtype=dt) for a in (test, tobs, varobs))
        f(ip(ldgrd), ip(ngrd), ip(nobs), ip(1), _ptr(allm), _ptr(to), _ptr(va), _ptr(t), _ptr(lp), C.byref(ierr))
        out[f"ierr{prec}_allmasked"] = ierr.value
    np.savez_compressed(os.path.join(HERE, "gridsearch_f90.npz"), **out)


def make_locate():
    """locate.c main()-style inputs (locate.c:108-164) on a smaller grid,
    generated with the reference's own makeTest/makeObs and glibc rand()."""
    # lazy binding: locate.c's L1 path references weightedMedian__double, which
    # the reference never defines; only the L2 entry point is called.
    lib = C.CDLL(os.path.join(REF, "liblocate_ref.so"), mode=os.RTLD_LAZY)
    libc = C.CDLL("libc.so.6")
    libc.rand.restype = C.c_int
    RAND_MAX = 2147483647
    lib.makeObs.restype = C.c_double
    lib.makeObs.argtypes = [C.c_double] * 6
    lib.makeTest.argtypes = [C.c_int] * 3 + [C.c_double] * 6 + [C.c_void_p]
    f = lib.locate_l2_gridSearch__double64
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double] + [C.c_void_p] * 7
    libc.srand(4042)
    nx, ny, nz, nobs = 21, 17, 7, 12
    dx = dy = dz = 1.0e3
    ngrd = nx * ny * nz
    ldgrd = ngrd + 64 - ngrd % 64
    xsrc, ysrc, zsrc = 12 * dx, 9 * dy, 4 * dz

    def aligned(n, dtype=np.float64):
        raw = np.zeros(n + 16, dtype=dtype)
        off = (-raw.ctypes.data % 64) // raw.itemsize
        return raw[off:off + n]

    test = aligned(nobs * ldgrd)
    tobs = np.zeros(nobs); varobs = np.zeros(nobs)
    for i in range(nobs):
        xr = libc.rand() / RAND_MAX * (nx - 1) * dx
        yr = libc.rand() / RAND_MAX * (ny - 1) * dy
        zr = libc.rand() / RAND_MAX * (nz - 1) * dz
        tobs[i] = lib.makeObs(xr, yr, zr, xsrc, ysrc, zsrc)
        varobs[i] = libc.rand() / RAND_MAX
        lib.makeTest(nx, ny, nz, dx, dy, dz, xr, yr, zr, _ptr(test[ldgrd * i:]))
    tobs += 4.0
    tcorr = np.linspace(-0.05, 0.07, nobs)
    mask = np.zeros(nobs, dtype=np.int32); mask[[3, 8]] = 1
    out = dict(ldgrd=ldgrd, ngrd=ngrd, nobs=nobs, tobs=tobs, varobs=varobs,
               tcorr=tcorr, mask=mask, test=np.array(test))
    for tag, iwant, t0use, use_tc, m in (("ot", 1, 0.0, True, mask), ("fixed", 0, 4.0, False, np.zeros_like(mask))):
        t0 = aligned(ngrd); obj = aligned(ngrd)
        ierr = f(ldgrd, ngrd, nobs, iwant, t0use, _ptr(m), _ptr(tobs),
                 _ptr(tcorr) if use_tc else None, _ptr(varobs), _ptr(test), _ptr(t0), _ptr(obj))
        assert ierr == 0
        out[f"{tag}_t0"] = np.array(t0); out[f"{tag}_objfn"] = np.array(obj)
        out[f"{tag}_argmin"] = int(np.argmin(obj))
        print(f"locate_l2 {tag}: argmin={int(np.argmin(obj))} true={4*nx*ny+9*nx+12}")
    np.savez_compressed(os.path.join(HERE, "locate_l2.npz"), **out)

    # the fp32 variant (locate.c:1079-1203) on the same inputs cast to float32
    g = lib.locate_l2_gridSearch__float64
    g.restype = C.c_int
    g.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_float] + [C.c_void_p] * 7
    test32 = aligned(nobs * ldgrd, np.float32)
    test32[:] = np.asarray(test, dtype=np.float32)
    tobs32, varobs32, tcorr32 = (np.asarray(a, dtype=np.float32) for a in (tobs, varobs, tcorr))
    o32 = dict(ldgrd=ldgrd, ngrd=ngrd, nobs=nobs, tobs=tobs32, varobs=varobs32, tcorr=tcorr32, mask=mask,
               test=np.array(test32))
    for tag, iwant, t0use, use_tc, m in (("ot", 1, 0.0, True, mask), ("fixed", 0, 4.0, False, np.zeros_like(mask))):
        t0 = aligned(ngrd, np.float32); obj = aligned(ngrd, np.float32)
        ierr = g(ldgrd, ngrd, nobs, iwant, t0use, _ptr(m), _ptr(tobs32), _ptr(tcorr32) if use_tc else None,
                 _ptr(varobs32), _ptr(test32), _ptr(t0), _ptr(obj))
        assert ierr == 0
        o32[f"{tag}_t0"] = np.array(t0); o32[f"{tag}_objfn"] = np.array(obj)
        print(f"locate_l2 f32 {tag}: argmin={int(np.argmin(obj))}")
    np.savez_compressed(os.path.join(HERE, "locate_l2_f32.npz"), **o32)


def make_fsm_mpi():
    """The reference's MPI-variant solver (EIKONAL3D_INITIALIZE/_SOLVE,
    fsm3d.f90:1583-1852) on block decompositions, one MPI rank per block,
    through oracle/_ref/mpi_ref_driver (mpiexec).  The reference accepts
    1- or 2-way splits per axis here (3- and 4-way splits abort in its
    initialisation).  Fields are stored for the small grid; the xfsm3d
    70x80x90 case stores a digest, max u and the iteration-count-free ierr."""
    import subprocess
    import tempfile
    drv = os.path.join(REF, "mpi_ref_driver")
    mpiexec = "/opt/conda/bin/mpiexec"
    nx, ny, nz, h = 20, 18, 22, 100.0
    slow = np.ascontiguousarray((1.0 / hetero_velocity(nx, ny, nz)).ravel())
    src = (0.0, 834.5, 987.6, 1100.0)
    cases = [("b211", (2, 1, 1), 1, 50, src), ("b222", (2, 2, 2), 1, 50, src), ("b121_ov2", (1, 2, 1), 2, 50, src),
             ("b112", (1, 1, 2), 1, 50, src), ("b212_ov0", (2, 1, 2), 0, 50, src), ("b221_ov0", (2, 2, 1), 0, 50, src),
             ("b222_maxit1", (2, 2, 2), 1, 1, src), ("b222_onnode", (2, 2, 2), 1, 50, (0.5, 900.0, 800.0, 1000.0)),
             ("b222_origin_err", (2, 2, 2), 1, 50, (0.0, 0.0, 0.0, 0.0))]
    out = {"grid": np.array([nx, ny, nz]), "h": h, "slow": slow}
    with tempfile.TemporaryDirectory() as td:
        sp, op = os.path.join(td, "slow.f64"), os.path.join(td, "u.f64")
        slow.tofile(sp)
        for name, nd, nov, maxit, s in cases:
            cmd = [mpiexec, "-n", str(nd[0] * nd[1] * nd[2]), drv, str(nx), str(ny), str(nz), *map(str, nd), str(nov),
                   str(maxit), "1e-8", str(h), "0", "0", "0", *map(repr, s), sp, op]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if name.endswith("_err"):
                # SETBCS fails (source on the first node, fsm3d.f90:736-753): the
                # solve returns ierr = 1 on every rank before any sweep
                out[f"{name}_ierr"] = np.int32(1 if r.returncode == 0 and np.fromfile(op)[-1] == 1.0 else -1)
            else:
                assert r.returncode == 0, (name, r.stdout[-500:], r.stderr[-500:])
                res = np.fromfile(op)
                out[f"{name}_u"], out[f"{name}_ierr"] = res[:-1], np.int32(res[-1])
            out[f"{name}_cfg"] = np.array([*nd, nov, maxit])
            out[f"{name}_src"] = np.array(s)
        # the reference's own xfsm3d case (fsm3d.f90:2085-2100): 70x80x90, 2x2x2 blocks
        n3 = (70, 80, 90)
        sl = np.full(n3[0] * n3[1] * n3[2], 1.0 / 5.0e3)
        sl.tofile(sp)
        xs = tuple(100.0 * n / 2.0 for n in n3)
        cmd = [mpiexec, "-n", "8", drv, *map(str, n3), "2", "2", "2", "1", "5", "1e-7", "100", "0", "0", "0", "0",
               *map(repr, xs), sp, op]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-500:]
        res = np.fromfile(op)
        out["xfsm3d_sha256"] = np.array(hashlib.sha256(res[:-1].tobytes()).hexdigest())
        out["xfsm3d_max"], out["xfsm3d_ierr"] = res[:-1].max(), np.int32(res[-1])
    np.savez_compressed(os.path.join(HERE, "blocks_mpi.npz"), **out)


if __name__ == "__main__":
    if not os.path.exists(os.path.join(REF, "libfsm3d_ref.so")):
        sys.exit("build the reference first: oracle/build_ref.sh")
    make_fsm(RefFSM())
    make_locate()
    make_gridsearch()
    if os.path.exists(os.path.join(REF, "mpi_ref_driver")) and os.path.exists("/opt/conda/bin/mpiexec"):
        make_fsm_mpi()
