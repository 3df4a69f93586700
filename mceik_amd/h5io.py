"""ctypes binding of libmceik_h5io.so (include/mceik_h5io.h) and the posterior
writer: the reference's h5io layout (h5io.c) for the kept MCMC samples.

`write_posterior` is the rank-0 step after the checkpoint gather (SURVEY s.8f
rows 1-2): for each kept velocity model it runs the fp32 forward with full
fields (one GPU launch per model, all stations), writes the P travel-time
tables to `<proj>_ttimes.h5`, relocates every event against those tables on
the GPU (`eikonal.relocate`, locate.c L2 with the analytic origin time) and
writes the log joint PDFs to `<proj>_locations.h5`.  Kept samples become
Model_1..Model_n.  Like the reference, files store fp32 grids with the
{nx,ny,nz} dataspace over x-fastest data (read back as [nz][ny][nx]).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmceik_h5io.so")
PATH_MAX = 4096
TRAVELTIME_FILE, LOCATION_FILE = 1, 2

EXPORTS = ("eikonal_h5io_setFileName", "eikonal_h5io_setTravelTimeName", "eikonal_h5io_setLocationName",
           "mceik_h5io_initTTables", "mceik_h5io_writeTravelTimes", "mceik_h5io_readTravelTimes",
           "mceik_h5io_initLocations", "mceik_h5io_writeLocationLogJPDF", "mceik_h5io_readLocationLogJPDF",
           "mceik_h5io_getModelDimensions", "mceik_h5io_readModel", "mceik_h5io_open", "mceik_h5io_exists",
           "mceik_h5io_finalize")

_lib = None


def lib():
    """Load libmceik_h5io.so (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"mceik_amd: {LIB_PATH} is missing; build it with `make -C {_HERE}`")
    L = C.CDLL(LIB_PATH)
    i, d, vp, i64p = C.c_int, C.c_double, C.c_void_p, C.POINTER(C.c_int64)
    L.eikonal_h5io_setFileName.argtypes = [i, C.c_char_p, C.c_char_p, C.c_char_p]
    L.eikonal_h5io_setTravelTimeName.argtypes = [i, i, i, C.c_char_p]
    L.eikonal_h5io_setTravelTimeName.restype = None
    L.eikonal_h5io_setLocationName.argtypes = [i, i, C.c_char_p]
    L.eikonal_h5io_setLocationName.restype = None
    L.mceik_h5io_initTTables.argtypes = [C.c_char_p, C.c_char_p] + [i] * 5 + [d] * 6 + [i64p]
    L.mceik_h5io_initLocations.argtypes = [C.c_char_p, C.c_char_p] + [i] * 5 + [d] * 6 + [i64p]
    for f in (L.mceik_h5io_writeTravelTimes, L.mceik_h5io_readTravelTimes):
        f.argtypes = [C.c_int64] + [i] * 6 + [vp]
    for f in (L.mceik_h5io_writeLocationLogJPDF, L.mceik_h5io_readLocationLogJPDF):
        f.argtypes = [C.c_int64] + [i] * 5 + [vp]
    L.mceik_h5io_getModelDimensions.argtypes = [C.c_int64] + [C.POINTER(C.c_int)] * 3
    L.mceik_h5io_readModel.argtypes = [C.c_int64] + [i] * 3 + [vp] * 3
    L.mceik_h5io_open.argtypes = [C.c_char_p, i, i64p]
    L.mceik_h5io_exists.argtypes = [C.c_int64, C.c_char_p]
    L.mceik_h5io_finalize.argtypes = [i64p]
    for name in EXPORTS:
        if getattr(L, name).restype is not None and name not in ("eikonal_h5io_setTravelTimeName",
                                                                  "eikonal_h5io_setLocationName"):
            getattr(L, name).restype = C.c_int
    _lib = L
    return L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


def file_name(job, dirnm, projnm):
    buf = C.create_string_buffer(PATH_MAX)
    _chk(lib().eikonal_h5io_setFileName(job, dirnm.encode() if dirnm else None, projnm.encode(), buf),
         "eikonal_h5io_setFileName")
    return buf.value.decode()


def travel_time_name(model, station, is_p=True):
    buf = C.create_string_buffer(512)
    lib().eikonal_h5io_setTravelTimeName(model, station, 1 if is_p else 0, buf)
    return buf.value.decode()


def location_name(model, event):
    buf = C.create_string_buffer(512)
    lib().eikonal_h5io_setLocationName(model, event, buf)
    return buf.value.decode()


class H5File:
    """An open ttimes or locations file (context manager)."""

    def __init__(self, fid):
        self.fid = C.c_int64(fid)

    @classmethod
    def open(cls, path, readwrite=False):
        fid = C.c_int64(-1)
        _chk(lib().mceik_h5io_open(path.encode(), 1 if readwrite else 0, C.byref(fid)), f"open {path}")
        return cls(fid.value)

    def exists(self, name):
        return lib().mceik_h5io_exists(self.fid, name.encode()) == 1

    def dims(self):
        nx, ny, nz = C.c_int(), C.c_int(), C.c_int()
        _chk(lib().mceik_h5io_getModelDimensions(self.fid, C.byref(nx), C.byref(ny), C.byref(nz)), "dims")
        return nx.value, ny.value, nz.value

    def model(self):
        nx, ny, nz = self.dims()
        x, y, z = (np.zeros(nx * ny * nz, np.float32) for _ in range(3))
        _chk(lib().mceik_h5io_readModel(self.fid, nx, ny, nz, *(a.ctypes.data_as(C.c_void_p) for a in (x, y, z))),
             "readModel")
        return x, y, z

    def write_ttimes(self, station, model, tt, iphase=1):
        nx, ny, nz = self.dims()
        a = np.ascontiguousarray(tt, dtype=np.float32).ravel()
        assert a.size == nx * ny * nz
        _chk(lib().mceik_h5io_writeTravelTimes(self.fid, station, model, iphase, nx, ny, nz,
                                               a.ctypes.data_as(C.c_void_p)), "writeTravelTimes")

    def read_ttimes(self, station, model, iphase=1):
        nx, ny, nz = self.dims()
        a = np.zeros(nx * ny * nz, np.float32)
        _chk(lib().mceik_h5io_readTravelTimes(self.fid, station, model, iphase, nx, ny, nz,
                                              a.ctypes.data_as(C.c_void_p)), "readTravelTimes")
        return a

    def write_logjpdf(self, model, event, v):
        nx, ny, nz = self.dims()
        a = np.ascontiguousarray(v, dtype=np.float32).ravel()
        assert a.size == nx * ny * nz
        _chk(lib().mceik_h5io_writeLocationLogJPDF(self.fid, model, event, nx, ny, nz,
                                                   a.ctypes.data_as(C.c_void_p)), "writeLocationLogJPDF")

    def read_logjpdf(self, model, event):
        nx, ny, nz = self.dims()
        a = np.zeros(nx * ny * nz, np.float32)
        _chk(lib().mceik_h5io_readLocationLogJPDF(self.fid, model, event, nx, ny, nz,
                                                  a.ctypes.data_as(C.c_void_p)), "readLocationLogJPDF")
        return a

    def close(self):
        if self.fid.value >= 0:
            _chk(lib().mceik_h5io_finalize(C.byref(self.fid)), "finalize")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def init_ttables(dirnm, projnm, nx, ny, nz, nmodels, nstations, x0, y0, z0, dx, dy, dz):
    fid = C.c_int64(-1)
    _chk(lib().mceik_h5io_initTTables(dirnm.encode(), projnm.encode(), nx, ny, nz, nmodels, nstations,
                                      x0, y0, z0, dx, dy, dz, C.byref(fid)), "initTTables")
    return H5File(fid.value)


def init_locations(dirnm, projnm, nx, ny, nz, nmodels, nevents, x0, y0, z0, dx, dy, dz):
    fid = C.c_int64(-1)
    _chk(lib().mceik_h5io_initLocations(dirnm.encode(), projnm.encode(), nx, ny, nz, nmodels, nevents,
                                        x0, y0, z0, dx, dy, dz, C.byref(fid)), "initLocations")
    return H5File(fid.value)


def write_posterior(p, models, dirnm, projnm, device=0, relocate_events=True):
    """Write kept velocity models (int32 [k, ncell] inversion-cell P velocities,
    or [k, 2, ncell] P and S models of a joint sampler, e.g. the gathered
    Sampler.samples()) as the reference's HDF5 posterior: the P travel-time
    table (and, with S models, the S table: PTravelTimes / STravelTimes,
    h5io.c:662-697) of every model x station (fp32 GPU forward, the sampler's
    arithmetic) and, if `relocate_events`, every event's log joint PDF on the
    grid for every model (GPU relocation over the event's fitted observations
    in catalog order -- an S pick against its station's S table -- masked
    picks excluded).  Returns the two file names."""
    import torch
    from . import eikonal
    nph = int(getattr(p, "nphase", 1))
    models = np.asarray(models, dtype=np.int32).reshape(-1, nph, p.ncell)
    nm = models.shape[0]
    dev = torch.device("cuda", device)
    nxyz = p.nx * p.ny * p.nz
    src = torch.tensor(np.stack([np.zeros(p.nstat), p.sx, p.sy, p.sz], 1)[:, None, :], dtype=torch.float64)
    bs = eikonal.BatchSolver(p.nx, p.ny, p.nz, p.h, p.x0, p.y0, p.z0, p.maxit, p.tol, 32, nref=p.nref)
    events = []
    mask_all, tcorr_all = p.obs_mask, p.tcorr
    row_all = p.obs_stat + p.nstat * (p.obs_phase if nph > 1 else 0)   # table row: phase-major
    for e in range(p.nevents):
        k = np.arange(p.obs_ptr[e], p.obs_ptr[e + 1])
        events.append(dict(rows=row_all[k], tobs=np.float32(p.tobs[k]), varobs=np.float32(p.var[k]),
                           tcorr=np.float32(tcorr_all[k]), mask=np.int32(mask_all[k])))
    ttf = init_ttables(dirnm, projnm, p.nx, p.ny, p.nz, nm, p.nstat, p.x0, p.y0, p.z0, p.h, p.h, p.h)
    locf = init_locations(dirnm, projnm, p.nx, p.ny, p.nz, nm, p.nevents, p.x0, p.y0, p.z0, p.h, p.h, p.h) \
        if relocate_events else None
    try:
        for m in range(nm):
            slow = torch.tensor((1.0 / models[m].astype(np.float32)).astype(np.float32).reshape(nph, -1), device=dev)
            u = bs.solve(src, slow, want_fields=True)["u"].reshape(nph * p.nstat, nxyz)
            host = u.cpu().numpy()
            for ph in range(nph):
                for s in range(p.nstat):
                    ttf.write_ttimes(s + 1, m + 1, host[ph * p.nstat + s], iphase=ph + 1)
            if locf is not None:
                logp, _ = eikonal.relocate(u.contiguous(), events, log_pdf=True)
                logp = logp[:, :nxyz].cpu().numpy()
                for e in range(p.nevents):
                    locf.write_logjpdf(m + 1, e + 1, logp[e])
    finally:
        ttf.close()
        if locf is not None:
            locf.close()
    return file_name(TRAVELTIME_FILE, dirnm, projnm), (file_name(LOCATION_FILE, dirnm, projnm)
                                                       if relocate_events else None)
