"""Run configuration: host side of include/mceik.h's mceik_parms_* (csrc/parms.c).

The reference hard-codes its parameters in its mains (homog.c:73-89,
fsm3d.f90:2085-2100); mceik_parms_struct (mceik_struct.h:68-90) is the
intended record (SURVEY s.5).  `load` fills it, plus the sampler options,
from an INI file and "section:key=value" overrides through the library's own
parser, so a C main and a Python driver read a file the same way.

    parms, opts = load("run.ini", ["mcmc:nchains=256", "eikonal:tol=1e-7"])
    kw = apply_to_problem(problem, parms, opts)     # -> Sampler(problem, **kw)
"""
import ctypes as C

from . import _lib


def _bind():
    L = _lib.lib()
    P, O = C.POINTER(_lib.MceikParms), C.POINTER(_lib.McmcOpts)
    L.mceik_parms_defaults.argtypes = [P, O]
    L.mceik_parms_set.argtypes = [P, O, C.c_char_p, C.c_char_p]
    L.mceik_parms_read.argtypes = [C.c_char_p, P, O]
    L.mceik_parms_args.argtypes = [C.c_int, C.POINTER(C.c_char_p), P, O]
    L.mceik_parms_write.argtypes = [C.c_char_p, P, O]
    for f in ("defaults", "set", "read", "args", "write"):
        getattr(L, "mceik_parms_" + f).restype = C.c_int
    return L


def defaults():
    """(MceikParms, McmcOpts) with mceik_parms_defaults' values (homog.c's grid)."""
    parms, opts = _lib.MceikParms(), _lib.McmcOpts()
    _bind().mceik_parms_defaults(C.byref(parms), C.byref(opts))
    return parms, opts


def set_key(parms, opts, key, value):
    """One "section:key" = value; raises KeyError / ValueError as the C call reports."""
    rc = _bind().mceik_parms_set(C.byref(parms), C.byref(opts), key.encode(), str(value).encode())
    if rc == 1:
        raise KeyError(key)
    if rc:
        raise ValueError(f"{key} = {value!r}")


def load(path=None, overrides=(), base=None):
    """Defaults (or `base`), then the INI file `path`, then each "section:key=value"
    of `overrides` in order.  Returns (MceikParms, McmcOpts)."""
    parms, opts = base if base is not None else defaults()
    if path is not None:
        rc = _bind().mceik_parms_read(str(path).encode(), C.byref(parms), C.byref(opts))
        if rc < 0:
            raise FileNotFoundError(path)
        if rc > 0:
            raise ValueError(f"{path}:{rc}: invalid configuration line")
    for ov in overrides:
        key, sep, value = ov.lstrip("-").partition("=")
        if not sep:
            raise ValueError(f"override {ov!r} is not section:key=value")
        set_key(parms, opts, key, value)
    return parms, opts


def write(path, parms, opts):
    if _bind().mceik_parms_write(str(path).encode(), C.byref(parms), C.byref(opts)) != 0:
        raise OSError(f"cannot write {path}")


def apply_to_problem(p, parms, opts):
    """Copies the grid / eikonal / MCMC settings into a mcmc.Problem (whose
    grid must match opts.nx/ny/nz) and returns the Sampler keyword arguments."""
    if (p.nx, p.ny, p.nz) != (opts.nx, opts.ny, opts.nz):
        raise ValueError(f"problem grid {(p.nx, p.ny, p.nz)} != configured {(opts.nx, opts.ny, opts.nz)}")
    if not (parms.dx == parms.dy == parms.dz):
        raise ValueError("the solver needs dx = dy = dz")
    p.h, p.x0, p.y0, p.z0 = parms.dx, parms.x0, parms.y0, parms.z0
    p.nref = (parms.nrefx, parms.nrefy, parms.nrefz)
    p.tol, p.maxit = parms.eikparms.tol, parms.eikparms.maxit
    p.nburn, p.keepk, p.niter = parms.mcparms.nburnIn, parms.mcparms.keepK, parms.mcparms.niter
    p.vmin, p.vmax, p.dvmax, p.seed = opts.vmin, opts.vmax, opts.dvmax, opts.seed
    p.tt_interp = opts.tt_interp
    if opts.nphase > 1 and p.nphase != opts.nphase:
        raise ValueError(f"configured nphase {opts.nphase} but the problem holds {p.nphase} model(s) per chain")
    if opts.nphase > 1 or p.nphase > 1:
        p.vsmin, p.vsmax = opts.vsmin or p.vsmin, opts.vsmax or p.vsmax
    p.mask_s = opts.mask_s
    return dict(nchains=opts.nchains, chain_offset=opts.chain_offset, max_samples=opts.max_samples,
                device=opts.device, precision=opts.precision or 32, max_waves=opts.max_waves)
