"""The reference's own fp64 serial driver (oracle/_ref/libfsm3d_ref.so, built
from fsm3d.f90:1968-2052 by oracle/build_ref.sh) run in a spawned worker
process -- test infrastructure, the checker only.

The Fortran driver keeps module state (its level structure), so it is not
called from threads; each call runs job 1 (initialise), job 2 (solve) and job
3 (finalise) in a process of its own.  The .so is built here and travels with
the tree (it is git-ignored, not gpurun-ignored); callers skip when it is
absent.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libfsm3d_ref.so")


def available():
    return os.path.exists(REF_SO)


def _solve_worker(args):
    """eikonal3d_serial_driver(job, iverb, maxit, nsrc, nx, ny, nz, tol, h,
    x0, y0, z0, ts, xs, ys, zs, slow, u, ierr) for jobs 1, 2, 3 on one grid;
    returns (u, ierr of job 2)."""
    so, n, h, src, slow, maxit, tol = args
    os.environ["OMP_NUM_THREADS"] = "1"
    lib = C.CDLL(so)
    slow = np.ascontiguousarray(slow, dtype=np.float64)
    u = np.zeros(n ** 3)
    ts, xs, ys, zs = (np.array([float(v)]) for v in src)
    ierr = C.c_int(0)
    i = lambda v: C.byref(C.c_int(v))
    d = lambda v: C.byref(C.c_double(v))
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    call = lambda job: lib.eikonal3d_serial_driver(i(job), i(0), i(maxit), i(1), i(n), i(n), i(n), d(tol), d(h),
                                                    d(0.0), d(0.0), d(0.0), P(ts), P(xs), P(ys), P(zs), P(slow),
                                                    P(u), C.byref(ierr))
    call(1)
    call(2)
    e = ierr.value
    call(3)
    return u, e


def solve_many(jobs, workers):
    """jobs: [(n, h, (t, x, y, z), slow fp64 [n^3], maxit, tol)] -> [(u, ierr)],
    each in a spawned single-threaded process."""
    import concurrent.futures as cf
    import multiprocessing as mp
    with cf.ProcessPoolExecutor(max_workers=max(1, workers), mp_context=mp.get_context("spawn")) as ex:
        return list(ex.map(_solve_worker, [(REF_SO,) + tuple(j) for j in jobs]))
