"""ctypes wrapper for oracle/liboracle.so -- the CPU checker.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg (never by mceik_amd/).  Builds the oracle on first use if it is missing.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        src = os.path.join(ORACLE_DIR, "mceik_oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        L = C.CDLL(path)
        for name in ("oracle_eikonal3d_solve_f64", "oracle_eikonal3d_solve_f32"):
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = [C.c_int] * 5 + [C.c_double] * 5 + [C.c_void_p] * 7
        for name in ("oracle_eikonal3d_solve_dbg_f64", "oracle_eikonal3d_solve_dbg_f32"):
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = [C.c_int] * 6 + [C.c_double] * 5 + [C.c_void_p] * 7
        L.oracle_batch_solve_f64.restype = C.c_int
        L.oracle_batch_solve_f64.argtypes = ([C.c_int] * 5 + [C.c_double] * 5 + [C.c_void_p] * 6
                                             + [C.c_int, C.c_int])
        L.oracle_locate_l2_gridsearch_f64.restype = C.c_int
        L.oracle_locate_l2_gridsearch_f64.argtypes = [C.c_int] * 4 + [C.c_double] + [C.c_void_p] * 7
        L.oracle_gridsearch_f90_f64.restype = C.c_int
        L.oracle_gridsearch_f90_f64.argtypes = [C.c_int] * 4 + [C.c_void_p] * 6
        L.oracle_det_log.restype = C.c_double
        L.oracle_det_log.argtypes = [C.c_double]
        L.oracle_philox4x32_10.argtypes = [C.c_void_p] * 3
        L.oracle_loglik.restype = C.c_double
        L.oracle_loglik.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_forward_f32.restype = C.c_int
        L.oracle_forward_f32.argtypes = [C.c_void_p] * 4
        L.oracle_mcmc_run.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_int] + [C.c_void_p] * 4
        _LIB = L
    return _LIB


def eikonal_solve(nx, ny, nz, slow, h, sources, maxit=50, tol=1e-8, x0=0.0, y0=0.0, z0=0.0,
                  dtype=np.float64, max_sweeps=-1):
    """Serial-driver job 2 semantics (SETBCS + FSM). Returns (u, ierr, niter).
    max_sweeps >= 0 stops after that many sweeps (debug bisection)."""
    src = np.atleast_2d(np.asarray(sources, dtype=np.float64))
    cols = [np.ascontiguousarray(src[:, k]) for k in range(4)]
    slow = np.ascontiguousarray(slow, dtype=dtype)
    u = np.zeros(nx * ny * nz, dtype=dtype)
    it = C.c_int(0)
    f = lib().oracle_eikonal3d_solve_dbg_f64 if dtype == np.float64 else lib().oracle_eikonal3d_solve_dbg_f32
    ierr = f(maxit, max_sweeps, len(cols[0]), nx, ny, nz, tol, h, x0, y0, z0, *[_p(c) for c in cols],
             _p(slow), _p(u), C.byref(it))
    return u, ierr, it.value


def eikonal_solve_blocks(nx, ny, nz, slow, h, src, ndiv, noverlap, maxit=50, tol=1e-8, x0=0.0, y0=0.0, z0=0.0):
    """oracle_eikonal3d_solve_blocks_f64: the MPI variant's block-decomposed
    solve (fp64).  Returns (u, ierr, niter)."""
    L = lib()
    f = L.oracle_eikonal3d_solve_blocks_f64
    f.restype = C.c_int
    f.argtypes = [C.c_int] * 9 + [C.c_double] * 5 + [C.c_void_p] * 7
    src = np.atleast_2d(np.asarray(src, dtype=np.float64))
    cols = [np.ascontiguousarray(src[:, k]) for k in range(4)]
    slow = np.ascontiguousarray(slow, dtype=np.float64)
    u = np.zeros(nx * ny * nz)
    it = C.c_int(0)
    ierr = f(maxit, len(cols[0]), nx, ny, nz, *ndiv, noverlap, tol, h, x0, y0, z0, *[_p(c) for c in cols],
             _p(slow), _p(u), C.byref(it))
    return u, ierr, it.value


def locate_l2(ldgrd, ngrd, nobs, iwant, t0use, mask, tobs, tcorr, varobs, test):
    t0 = np.zeros(ngrd); obj = np.zeros(ngrd)
    m = np.ascontiguousarray(mask, dtype=np.int32)
    ierr = lib().oracle_locate_l2_gridsearch_f64(ldgrd, ngrd, nobs, iwant, t0use, _p(m), _p(tobs),
                                                 _p(tcorr), _p(varobs), _p(test), _p(t0), _p(obj))
    return ierr, t0, obj


def locate_l2_f32(ldgrd, ngrd, nobs, iwant, t0use, mask, tobs, tcorr, varobs, test):
    t0 = np.zeros(ngrd, np.float32); obj = np.zeros(ngrd, np.float32)
    m = np.ascontiguousarray(mask, dtype=np.int32)
    f = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.float32)
    tobs, tcorr, varobs, test = f(tobs), f(tcorr), f(varobs), f(test)
    L = lib()
    L.oracle_locate_l2_gridsearch_f32.argtypes = [C.c_int] * 4 + [C.c_float] + [C.c_void_p] * 7
    ierr = L.oracle_locate_l2_gridsearch_f32(ldgrd, ngrd, nobs, iwant, t0use, _p(m), _p(tobs), _p(tcorr),
                                             _p(varobs), _p(test), _p(t0), _p(obj))
    return ierr, t0, obj


def gridsearch_f90(ldgrd, ngrd, nobs, iwant, mask, tobs, varobs, test):
    logpdf = np.zeros(ngrd); t0 = C.c_double(0)
    m = np.ascontiguousarray(mask, dtype=np.int32)
    iopt = lib().oracle_gridsearch_f90_f64(ldgrd, ngrd, nobs, iwant, _p(m), _p(tobs), _p(varobs),
                                           _p(test), _p(logpdf), C.byref(t0))
    return iopt, t0.value, logpdf


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32); k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


class McmcProblem(C.Structure):
    """Mirror of oracle_mcmc_problem (oracle/mceik_oracle.c)."""
    _fields_ = [(n, C.c_int) for n in ("nx", "ny", "nz", "nrx", "nry", "nrz", "ncx", "ncy", "ncz", "maxit")] + \
               [(n, C.c_double) for n in ("h", "x0", "y0", "z0", "tol")] + \
               [("nstat", C.c_int), ("nevents", C.c_int)] + \
               [(n, C.c_void_p) for n in ("sx", "sy", "sz", "ev_node", "obs_ptr", "obs_stat", "obs_mask",
                                          "tobs", "tcorr", "var")] + \
               [("vmin", C.c_int), ("vmax", C.c_int), ("dvmax", C.c_int), ("seed", C.c_uint32),
                ("ev_frac", C.c_void_p), ("nphase", C.c_int), ("vsmin", C.c_int), ("vsmax", C.c_int),
                ("obs_phase", C.c_void_p), ("skip", C.c_void_p), ("prec", C.c_int)]


def make_problem(pb, precision=32):
    """pb: mceik_amd.mcmc.Problem-like object holding numpy arrays. Keeps refs alive.
    precision 64: the fp64 sampler's forward (oracle_mcmc_problem.prec)."""
    P = McmcProblem()
    P.prec = int(precision)
    for n in ("nx", "ny", "nz", "nrx", "nry", "nrz", "ncx", "ncy", "ncz", "maxit", "nstat", "nevents",
              "vmin", "vmax", "dvmax"):
        setattr(P, n, int(getattr(pb, n)))
    for n in ("h", "x0", "y0", "z0", "tol"):
        setattr(P, n, float(getattr(pb, n)))
    P.seed = int(pb.seed)
    P.nphase = int(getattr(pb, "nphase", 1))
    P.vsmin, P.vsmax = int(getattr(pb, "vsmin", 0)), int(getattr(pb, "vsmax", 0))
    keep = []
    interp = bool(getattr(pb, "tt_interp", 0))
    ev_node, ev_frac = pb.ev_cell if interp else (pb.ev_node, None)
    vals = {"ev_node": ev_node}
    for n, dt in (("sx", np.float64), ("sy", np.float64), ("sz", np.float64), ("ev_node", np.int32),
                  ("obs_ptr", np.int32), ("obs_stat", np.int32), ("obs_mask", np.int32),
                  ("tobs", np.float64), ("tcorr", np.float64), ("var", np.float64)):
        a = np.ascontiguousarray(vals[n] if n in vals else getattr(pb, n), dtype=dt)
        keep.append(a)
        setattr(P, n, a.ctypes.data)
    if interp:
        a = np.ascontiguousarray(ev_frac, dtype=np.float32)
        keep.append(a)
        P.ev_frac = a.ctypes.data
    if P.nphase > 1:
        a = np.ascontiguousarray(pb.obs_phase, dtype=np.int32)
        keep.append(a)
        P.obs_phase = a.ctypes.data
    sk = getattr(pb, "skip", None)
    if sk is not None and np.asarray(sk).any():
        a = np.ascontiguousarray(sk, dtype=np.uint8)
        keep.append(a)
        P.skip = a.ctypes.data
    P._keep = keep
    return P


def forward_f32(P, v, phase=0):
    """Tables [nstat][nev] and iterations of one model of phase `phase` (the
    phase selects the skip row: stations without picks of it get FLT_MAX)."""
    tt = np.zeros(P.nstat * P.nevents, dtype=np.float32)
    it = np.zeros(P.nstat, dtype=np.int32)
    v = np.ascontiguousarray(v, dtype=np.int32)
    f = lib().oracle_forward_s_f32 if phase else lib().oracle_forward_f32
    f.restype = C.c_int
    f.argtypes = [C.c_void_p] * 4
    f(C.byref(P), _p(v), _p(tt), _p(it))
    return tt.reshape(P.nstat, P.nevents), it


def event_time(u, nx, ny, nz, node, w=None):
    """oracle_event_time: node value (w None) or the trilinear fp32 value."""
    L = lib()
    L.oracle_event_time.restype = C.c_float
    L.oracle_event_time.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    u = np.ascontiguousarray(u, dtype=np.float32)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float32)
    return np.float32(L.oracle_event_time(_p(u), nx, ny, nz, int(node), _p(w)))


def loglik(P, tt):
    """tt [nstat][nev] (P only) or [nphase][nstat][nev]."""
    tt = np.ascontiguousarray(tt, dtype=np.float32)
    return lib().oracle_loglik(C.byref(P), _p(tt))


def forward_all_f32(P, v):
    """Tables [nphase][nstat][nev] of every model of one chain (v [nphase*ncell])."""
    nph = max(1, int(P.nphase))
    tt = np.zeros(nph * P.nstat * P.nevents, dtype=np.float32)
    v = np.ascontiguousarray(v, dtype=np.int32)
    lib().oracle_forward_all_f32(C.byref(P), _p(v), _p(tt))
    return tt.reshape(nph, P.nstat, P.nevents)


def propose(P, chain, step, v):
    """oracle_propose: (cell over the chain's [nphase][ncell] entries, new v, in prior, log U)."""
    cell, vn, inp, logu = C.c_int(0), C.c_int(0), C.c_int(0), C.c_double(0.0)
    v = np.ascontiguousarray(v, dtype=np.int32)
    lib().oracle_propose(C.byref(P), C.c_uint32(chain), C.c_uint64(step), _p(v), C.byref(cell), C.byref(vn),
                         C.byref(inp), C.byref(logu))
    return cell.value, vn.value, bool(inp.value), logu.value


def mcmc_run(P, v, logl, gid0, step0, nsteps):
    v = np.ascontiguousarray(v, dtype=np.int32).copy()
    logl = np.ascontiguousarray(logl, dtype=np.float64).copy()
    nch = v.shape[0]        # v [nchains][ncell] or [nchains][nphase][ncell]
    acc = np.zeros((nsteps, nch), dtype=np.uint8)
    trace = np.zeros((nsteps, nch), dtype=np.float64)
    lib().oracle_mcmc_run(C.byref(P), nch, gid0, step0, nsteps, _p(v), _p(logl), _p(acc), _p(trace))
    return v, logl, acc, trace
