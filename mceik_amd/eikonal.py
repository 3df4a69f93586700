"""Host mirror of the reference's eikonal entry points, computed by libmceik_hip.so.

`eikonal3d_serial_driver` keeps the reference's calling convention
(fsm3d.f90:1968-2052: job 1 init / 2 solve / other free, ierr out, caller-owned
fp64 arrays x fastest).  `batch_solve` is the batched GPU path on torch device
tensors (one launch, nmodel x nstat solves).
"""
import ctypes as C

import numpy as np

from . import _lib


def _ip(v):
    return C.byref(C.c_int(int(v)))


def _dp(v):
    return C.byref(C.c_double(float(v)))


def _arr(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(C.c_void_p)


def eikonal3d_serial_driver(job, iverb, maxit, nsrc, nx, ny, nz, tol, h, x0, y0, z0,
                            ts, xs, ys, zs, slow, u, precision=64):
    """Same arguments and ierr behaviour as the reference; fills `u` in place.

    precision=64: bitwise the reference.  precision=32: fp32 GPU path within
    the stated tolerance (|du| <= 1e-6 u + 1e-7 s).
    """
    L = _lib.lib()
    f = L.eikonal3d_serial_driver if precision == 64 else L.eikonal3d_serial_driver_sp
    n = int(nx) * int(ny) * int(nz)
    keep = [_arr(np.atleast_1d(v)) for v in (ts, xs, ys, zs)]
    if job == 2:
        slow_a, slow_p = _arr(slow)
        if slow_a.size < n or u.size < n or u.dtype != np.float64 or not u.flags.c_contiguous:
            raise ValueError("slow/u must hold nx*ny*nz float64 values (u C-contiguous)")
        u_p = u.ctypes.data_as(C.c_void_p)
    else:
        slow_a, slow_p, u_p = None, None, None
    ierr = C.c_int(0)
    f(_ip(job), _ip(iverb), _ip(maxit), _ip(nsrc), _ip(nx), _ip(ny), _ip(nz), _dp(tol), _dp(h),
      _dp(x0), _dp(y0), _dp(z0), keep[0][1], keep[1][1], keep[2][1], keep[3][1], slow_p, u_p, C.byref(ierr))
    return ierr.value


def eikonal3d_initialize(iverb, nx, ny, nz, ndivx, ndivy, ndivz, noverlap, maxit, x0, y0, z0, h, tol, comm=0):
    """EIKONAL3D_INITIALIZE (fsm3d.f90:1583-1598); returns ierr.  One GPU holds
    the whole grid: comm and the decomposition are accepted, not used."""
    L = _lib.lib()
    ierr = C.c_int(0)
    L.eikonal3d_initialize(_ip(comm), _ip(iverb), _ip(nx), _ip(ny), _ip(nz), _ip(ndivx), _ip(ndivy), _ip(ndivz),
                           _ip(noverlap), _ip(maxit), _dp(x0), _dp(y0), _dp(z0), _dp(h), _dp(tol), C.byref(ierr))
    return ierr.value


def eikonal3d_solve(nsrc, n, ts, xs, ys, zs, slow, u, comm=0):
    """EIKONAL3D_SOLVE (fsm3d.f90:1754-1889): the master passes n = nx*ny*nz and
    gets u (float64, filled in place); n < nx*ny*nz is a non-master rank."""
    L = _lib.lib()
    keep = [_arr(np.atleast_1d(v)) for v in (ts, xs, ys, zs)]
    sl, slp = _arr(slow)
    if u.dtype != np.float64 or not u.flags.c_contiguous or u.size < n or sl.size < n:
        raise ValueError("slow/u must hold n float64 values (u C-contiguous)")
    ierr = C.c_int(0)
    L.eikonal3d_solve(_ip(comm), _ip(nsrc), _ip(n), keep[0][1], keep[1][1], keep[2][1], keep[3][1], slp,
                      u.ctypes.data_as(C.c_void_p), C.byref(ierr))
    return ierr.value


def eikonal3d_finalize(comm=0):
    L = _lib.lib()
    ierr = C.c_int(0)
    L.eikonal3d_finalize(_ip(comm), C.byref(ierr))
    return ierr.value


def locate3d_gridsearch(ldgrd, ngrd, nobs, iwantOT, mask, tobs, varobs, test, logpdf):
    """locate3d_gridsearch__double64 / __float64 (gridsearch.f90:382-540) by the
    dtype of `logpdf` (float64 / float32); test [nobs*ldgrd]; returns ierr."""
    L = _lib.lib()
    dt = logpdf.dtype
    f = L.locate3d_gridsearch__double64 if dt == np.float64 else L.locate3d_gridsearch__float64
    m = np.ascontiguousarray(mask, dtype=np.int32)
    to, va, te = (np.ascontiguousarray(a, dtype=dt) for a in (tobs, varobs, test))
    ierr = C.c_int(0)
    f(_ip(ldgrd), _ip(ngrd), _ip(nobs), _ip(iwantOT), m.ctypes.data_as(C.c_void_p), to.ctypes.data_as(C.c_void_p),
      va.ctypes.data_as(C.c_void_p), te.ctypes.data_as(C.c_void_p), logpdf.ctypes.data_as(C.c_void_p),
      C.byref(ierr))
    return ierr.value


def locate_l2_gridsearch(ldgrd, ngrd, nobs, iwantOT, t0use, mask, tobs, tcorr, varobs, test, t0, objfn):
    """locate_l2_gridSearch__double64 (locate.c:923-1047) on the GPU; returns ierr.
    t0/objfn/test must be 64-byte aligned float64 arrays, as the reference requires."""
    L = _lib.lib()
    m = np.ascontiguousarray(mask, dtype=np.int32)
    to, tp = _arr(tobs)
    va, vp = _arr(varobs)
    tc, tcp = (None, None) if tcorr is None else _arr(tcorr)
    return L.locate_l2_gridSearch__double64(int(ldgrd), int(ngrd), int(nobs), int(iwantOT), float(t0use),
                                            m.ctypes.data_as(C.c_void_p), tp, tcp, vp,
                                            test.ctypes.data_as(C.c_void_p), t0.ctypes.data_as(C.c_void_p),
                                            objfn.ctypes.data_as(C.c_void_p))


def locate_l2_gridsearch_f32(ldgrd, ngrd, nobs, iwantOT, t0use, mask, tobs, tcorr, varobs, test, t0, objfn):
    """locate_l2_gridSearch__float64 (locate.c:1079-1203, the fp32 variant) on the
    GPU; returns ierr.  test/t0/objfn: 64-byte aligned float32 arrays."""
    L = _lib.lib()
    m = np.ascontiguousarray(mask, dtype=np.int32)
    f = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.float32)
    to, va, tc = f(tobs), f(varobs), f(tcorr)
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    return L.locate_l2_gridSearch__float64(int(ldgrd), int(ngrd), int(nobs), int(iwantOT), float(t0use),
                                           p(m), p(to), p(tc), p(va), p(test), p(t0), p(objfn))


def relocate(tables, events, ldgrd=None, iwantOT=1, t0use=0.0, log_pdf=True, stream=0, single_pass=True,
             want_t0=True):
    """Relocation grid search (SURVEY s.8f row 2) of many events against one
    model's travel-time tables, one GPU launch (mceik_relocate).

    tables : torch float32 CUDA tensor [nrows, ldgrd] (row r = station r's
             travel times at every grid node, x fastest)
    events : list of dicts with 'rows' (int table row of each observation),
             'tobs', 'varobs', optional 'tcorr' and 'mask' (1 = masked),
             in the reference's observation order
    returns (out, t0): torch float32 [nev, ldgrd]; out = -objfn if log_pdf
    else objfn (locate.c L2 with the analytic origin time, fp32).
    """
    import torch
    L = _lib.lib()
    dev = tables.device
    nrows, ld = tables.shape
    ld = ldgrd or ld
    ptr, rows, tc, wt, xn = [0], [], [], [], []
    for ev in events:
        m = np.zeros(len(ev["rows"]), np.int32) if ev.get("mask") is None else np.asarray(ev["mask"])
        tcorr = ev.get("tcorr")
        x = np.float32(0.0)
        for i, r in enumerate(ev["rows"]):
            if m[i] != 0:
                continue
            to = np.float32(ev["tobs"][i])
            tc.append(to - np.float32(tcorr[i]) if tcorr is not None else to)
            rows.append(int(r))
            w = np.float32(1.0) / np.float32(ev["varobs"][i])
            wt.append(w)
            x = np.float32(x + w)
        xn.append(x)
        ptr.append(len(rows))
    nev = len(events)
    t = lambda a, dt: torch.tensor(np.asarray(a, dtype=dt), device=dev)
    d_ptr, d_rows = t(ptr, np.int32), t(rows if rows else [0], np.int32)
    d_tc, d_wt, d_xn = t(tc if tc else [0], np.float32), t(wt if wt else [0], np.float32), t(xn, np.float32)
    out = torch.empty((nev, ld), dtype=torch.float32, device=dev)
    t0 = torch.empty((nev, ld), dtype=torch.float32, device=dev)
    b = _lib.RelocateBatch()
    b.ldgrd, b.ngrd, b.nev, b.iwantOT, b.t0use = ld, int(tables.shape[1]) if ldgrd is None else int(ldgrd), nev, \
        int(iwantOT), float(t0use)
    b.ngrd = min(b.ngrd, ld)
    b.tables, b.ev_ptr, b.obs_row = tables.data_ptr(), d_ptr.data_ptr(), d_rows.data_ptr()
    b.tc, b.wt, b.xnorm = d_tc.data_ptr(), d_wt.data_ptr(), d_xn.data_ptr()
    b.t0, b.out, b.log_pdf = (t0.data_ptr() if want_t0 else None), out.data_ptr(), 1 if log_pdf else 0
    if single_pass:
        b.nrows, b.nobs = int(nrows), len(rows)
    if L.mceik_relocate(C.byref(b), C.c_void_p(stream)) != 0:
        raise RuntimeError("mceik_relocate failed")
    return out, (t0 if want_t0 else None)


def aligned_empty(n, dtype=np.float64, align=64):
    """numpy array whose data pointer is `align`-byte aligned (locate.c:967-974 requirement)."""
    itemsize = np.dtype(dtype).itemsize
    raw = np.zeros(n + align // itemsize, dtype=dtype)
    off = (-raw.ctypes.data % align) // itemsize
    return raw[off:off + n]


class BatchSolver:
    """Batched FSM solves on one GPU.  Tensors are torch CUDA(HIP) tensors.

    sources: [nstat, nsrc, 4] float64 (ts, xs, ys, zs)
    slow   : mode 'field': [nmodel, nz, ny, nx] (float32 or float64 = precision)
             mode 'cells': [nmodel, ncz, ncy, ncx] float32 slowness per inversion cell
    """

    def __init__(self, nx, ny, nz, h, x0=0.0, y0=0.0, z0=0.0, maxit=50, tol=1e-8, precision=32,
                 nref=None, fast_sqrt=False):
        self.nx, self.ny, self.nz, self.h = int(nx), int(ny), int(nz), float(h)
        # fast_sqrt (cells mode): the caller guarantees f = h * slowness >= 1e-12 (a
        # normal float), as the sampler does from vmax; results are unchanged
        self.fast_sqrt = bool(fast_sqrt)
        self.x0, self.y0, self.z0 = float(x0), float(y0), float(z0)
        self.maxit, self.tol, self.precision = int(maxit), float(tol), int(precision)
        self.nref = nref
        self._ws = None

    def describe(self, nmodel, nstat, nsrc, slow_mode, nev=0, max_sweeps=-1, max_waves=0, step_z=0):
        b = _lib.FsmBatch()
        b.nx, b.ny, b.nz = self.nx, self.ny, self.nz
        b.h, b.x0, b.y0, b.z0 = self.h, self.x0, self.y0, self.z0
        b.maxit, b.tol, b.precision = self.maxit, self.tol, self.precision
        b.nmodel, b.nstat, b.nsrc = nmodel, nstat, nsrc
        b.slow_mode = slow_mode
        nr = self.nref or (1, 1, 1)
        b.nrx, b.nry, b.nrz = nr
        b.nev = nev
        b.max_sweeps = max_sweeps
        b.fast_sqrt = 1 if (self.fast_sqrt and slow_mode == 1) else 0
        b.max_waves = int(max_waves)
        b.step_z = int(step_z)
        return b

    def solve(self, sources, slow, ev_node=None, want_fields=False, max_sweeps=-1, stream=None,
              solve_order=None, solve_clock=False, max_waves=0, step_z=0, ev_frac=None):
        """ev_node: [nev] x-fastest node per event -> out["ttab"] [nsolve][nev]
        (fp32): the node's value, or with ev_frac ([nev][3] float32 fractions,
        ev_node = the lowest corner of the event's cell; `cell_corners`) the
        trilinear interpolation in that cell (mceik_fsm_batch.ev_frac).
        solve_order: optional permutation of the nmodel*nstat solve ids (the
        order the work queues hand them out; results do not depend on it).
        solve_clock: also return out["clock"] [nsolve][2], the device realtime
        (100 MHz) at the start and end of every solve.  max_waves: cap on the
        resident solve waves (0 = occupancy x CUs); fewer waves than solves runs
        the production path (several solves per wave in reused scratch).
        step_z: 0 = the launch's kernel (16-z steps for the fp32 cell-cache
        instance, else 8-z; out["step_z"] says which ran), 8 = force the 8-z
        kernel; the results are identical."""
        import torch
        dev = slow.device
        sources = sources.to(device=dev, dtype=torch.float64).contiguous()
        nstat, nsrc = int(sources.shape[0]), int(sources.shape[1])
        nmodel = int(slow.shape[0])
        slow_mode = 1 if self.nref is not None else 0
        want_dtype = torch.float64 if self.precision == 64 else torch.float32
        if slow_mode == 0 and slow.dtype != want_dtype:
            raise TypeError(f"slowness field must be {want_dtype} for precision {self.precision}")
        if slow_mode == 1 and slow.dtype != torch.float32:
            raise TypeError("cell slowness must be float32")
        slow = slow.contiguous()
        nev = 0 if ev_node is None else int(ev_node.numel())
        b = self.describe(nmodel, nstat, nsrc, slow_mode, nev, max_sweeps, max_waves, step_z)
        nsolve = nmodel * nstat
        niter = torch.zeros(nsolve, dtype=torch.int32, device=dev)
        ierr = torch.zeros(nsolve, dtype=torch.int32, device=dev)
        out = {"niter": niter, "ierr": ierr}
        b.src = sources.data_ptr()
        b.slow = slow.data_ptr()
        b.niter, b.ierr = niter.data_ptr(), ierr.data_ptr()
        if solve_order is not None:
            solve_order = torch.as_tensor(solve_order, dtype=torch.int32).to(dev).contiguous()
            if solve_order.numel() != nsolve or not torch.equal(torch.sort(solve_order.cpu())[0],
                                                                torch.arange(nsolve, dtype=torch.int32)):
                raise ValueError("solve_order must be a permutation of the solve ids")
            b.solve_order = solve_order.data_ptr()
            out["_order"] = solve_order
        if solve_clock:
            clock = torch.zeros((nsolve, 2), dtype=torch.int64, device=dev)
            b.solve_clock = clock.data_ptr()
            out["clock"] = clock
        if nev:
            ev_node = ev_node.to(device=dev, dtype=torch.int32).contiguous()
            ttab = torch.empty((nsolve, nev), dtype=torch.float32, device=dev)
            b.ev_node, b.ttab = ev_node.data_ptr(), ttab.data_ptr()
            out["ttab"] = ttab
            out["_ev"] = ev_node
            if ev_frac is not None:
                ev_frac = torch.as_tensor(ev_frac, dtype=torch.float32).to(dev).contiguous()
                if ev_frac.numel() != 3 * nev:
                    raise ValueError("ev_frac must hold 3 fractions per event")
                b.ev_frac = ev_frac.data_ptr()
                out["_evf"] = ev_frac
        if want_fields:
            u = torch.empty((nsolve, self.nz, self.ny, self.nx), dtype=want_dtype, device=dev)
            b.u_out = u.data_ptr()
            out["u"] = u
        L = _lib.lib()
        nbytes = L.mceik_fsm_workspace_bytes(C.byref(b))
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        rc = L.mceik_fsm_batch_solve(C.byref(b), self._ws.data_ptr(), nbytes, C.c_void_p(st))
        if rc != 0:
            raise RuntimeError(f"mceik_fsm_batch_solve failed ({rc})")
        out["_keep"] = (sources, slow)
        out["bytes_per_node_sweep"] = L.mceik_fsm_bytes_per_node_sweep(C.byref(b))
        out["step_z"] = L.mceik_fsm_step_z(C.byref(b))
        return out
