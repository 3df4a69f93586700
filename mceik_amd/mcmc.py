"""MCMC travel-time tomography sampler: host side of include/mceik.h.

A `Problem` carries the reference's driver data model (mceik_struct.h:
stations, CSR event catalogue, grid/MCMC/eikonal parameters); `Sampler`
drives one GPU's chains through libmceik_hip.so (propose -> batched FSM ->
L2 misfit with analytic origin time -> Metropolis).  Multi-GPU runs shard the
global chain ids over ranks (`shard`), one process per GPU.
"""
import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib

P_PRIMARY_PICK, S_PRIMARY_PICK = 1, 2

# the BASELINE.json configurations (SURVEY s.8): name -> (n, stations, events, chains)
CONFIGS = {
    "C1": dict(n=32, nstat=4, nev=4, nchains=1, h=1000.0, homogeneous=True),
    "C2": dict(n=64, nstat=16, nev=16, nchains=256, h=100.0, homogeneous=False),
    "C3": dict(n=128, nstat=32, nev=32, nchains=1024, h=100.0, homogeneous=False),
    "C4": dict(n=128, nstat=32, nev=32, nchains=8192, h=100.0, homogeneous=False),
    "C5": dict(n=256, nstat=64, nev=64, nchains=2048, h=100.0, homogeneous=False),
}


@dataclass
class Problem:
    """Grid, stations, events and picks of one tomography problem."""
    nx: int
    ny: int
    nz: int
    h: float
    nref: tuple = (4, 4, 4)
    x0: float = 0.0
    y0: float = 0.0
    z0: float = 0.0
    maxit: int = 50
    tol: float = 1e-8
    sx: np.ndarray = None           # station coordinates (m) = eikonal sources
    sy: np.ndarray = None
    sz: np.ndarray = None
    pcorr: np.ndarray = None
    ex: np.ndarray = None           # event coordinates (m)
    ey: np.ndarray = None
    ez: np.ndarray = None
    obs_ptr: np.ndarray = None      # CSR by event (0-based), mceik_catalog_struct.obsPtr
    obs_stat: np.ndarray = None     # 0-based station per observation
    pick_type: np.ndarray = None
    luse: np.ndarray = None
    tobs: np.ndarray = None
    var: np.ndarray = None
    vmin: int = 1500
    vmax: int = 9000
    dvmax: int = 50
    nphase: int = 1                 # velocity models per chain: 1 = P, 2 = P and S (homog.c:208-258)
    vsmin: int = 800                # S prior (nphase 2)
    vsmax: int = 5500
    mask_s: int = 0                 # nphase 1: ignore used S picks instead of refusing the catalog
    scorr: np.ndarray = None        # S static corrections (mceik_stations_struct.scorr)
    seed: int = 2016
    nburn: int = 0
    keepk: int = 1
    niter: int = 0                  # mcparms.niter: total proposals (Sampler.run(-1) runs the rest)
    tt_interp: int = 0              # 0: event times at the nearest node (reference); 1: trilinear in the cell
    v_true: np.ndarray = None       # [ncell] int, model used to make the picks
    vs_true: np.ndarray = None      # [ncell] int, S model of the picks (P/S problems)
    has_p: np.ndarray = None        # [nstat] lhasP (mceik_struct.h:43-46); None: stations with used P picks
    has_s: np.ndarray = None        # [nstat] lhasS; None: stations with used S picks
    lcartesian: int = 1             # mceik_stations_struct.lcartesian (the sampler takes metres only)
    _keep: list = field(default_factory=list, repr=False)

    @property
    def ncx(self):
        return -(-self.nx // self.nref[0])

    @property
    def ncy(self):
        return -(-self.ny // self.nref[1])

    @property
    def ncz(self):
        return -(-self.nz // self.nref[2])

    @property
    def ncell(self):
        return self.ncx * self.ncy * self.ncz

    @property
    def nstat(self):
        return len(self.sx)

    @property
    def nevents(self):
        return len(self.ex)

    # --- quantities the oracle mirror needs (tests/_oracle.make_problem) ---
    @property
    def nrx(self):
        return self.nref[0]

    @property
    def nry(self):
        return self.nref[1]

    @property
    def nrz(self):
        return self.nref[2]

    @property
    def ev_node(self):
        """Nearest node of each event, as the reference snaps sources (fsm3d.f90:697-711)."""
        def idx(n, x0, xs):
            xs = np.asarray(xs, dtype=np.float64)
            i = (((xs - x0) / self.h + 0.5).astype(np.int64))
            i = np.where(xs <= x0, 0, np.where(xs >= x0 + (n - 1) * self.h, n - 1, i))
            return i
        ix, iy, iz = idx(self.nx, self.x0, self.ex), idx(self.ny, self.y0, self.ey), idx(self.nz, self.z0, self.ez)
        return ((iz * self.ny + iy) * self.nx + ix).astype(np.int32)

    @property
    def ev_cell(self):
        """Trilinear mode (tt_interp = 1): (lowest corner node [nev] int32, fractions
        [nev][3] float32) of each event's grid cell, as mceik_mcmc_init computes them
        (capi.hip cell_corner: i = trunc((x - x0)/h) clamped to [0, n-2], w = f - i in
        [0, 1] rounded once to fp32)."""
        def corner(n, x0, xs):
            f = (np.asarray(xs, dtype=np.float64) - x0) / self.h
            i = np.where(f <= 0.0, 0, np.trunc(np.maximum(f, 0.0))).astype(np.int64)
            i = np.minimum(i, n - 2)
            w = np.clip(f - i, 0.0, 1.0).astype(np.float32)
            return i, w
        ix, wx = corner(self.nx, self.x0, self.ex)
        iy, wy = corner(self.ny, self.y0, self.ey)
        iz, wz = corner(self.nz, self.z0, self.ez)
        return ((iz * self.ny + iy) * self.nx + ix).astype(np.int32), np.stack([wx, wy, wz], 1)

    @property
    def obs_used(self):
        """Observations the sampler fits (mceik_mcmc_init): used P picks, and used
        S picks when the chains hold an S model."""
        k = self.obs_stat
        ok = (self.luse != 0) & (k >= 0) & (k < self.nstat)
        sel = self.pick_type == P_PRIMARY_PICK
        if self.nphase > 1:
            sel = sel | (self.pick_type == S_PRIMARY_PICK)
        return ok & sel

    @property
    def obs_mask(self):
        return (~self.obs_used).astype(np.int32)

    @property
    def obs_phase(self):
        """0 = P, 1 = S: the model an observation is fit against."""
        return (self.obs_used & (self.pick_type == S_PRIMARY_PICK)).astype(np.int32)

    @property
    def tcorr(self):
        sc = self.scorr if self.scorr is not None else np.zeros(self.nstat)
        corr = np.where(self.obs_phase == 1, sc[self.obs_stat], self.pcorr[self.obs_stat])
        return np.where(self.obs_mask == 0, corr, 0.0)

    def station_flags(self):
        """(lhasP, lhasS) [nstat] int: the explicit has_p / has_s, else whether
        the station has a used pick of the phase (homog.c:230-235 sets them per
        station from its picks).  The sampler solves a station's P (S) table
        only when its flag is set."""
        def has(t):
            sel = (self.luse != 0) & (self.pick_type == t)
            return np.array([bool((sel & (self.obs_stat == k)).any()) for k in range(self.nstat)], np.int32)
        hp = np.asarray(self.has_p, np.int32) if self.has_p is not None else has(P_PRIMARY_PICK)
        hs = np.asarray(self.has_s, np.int32) if self.has_s is not None else has(S_PRIMARY_PICK)
        return hp, hs

    @property
    def skip(self):
        """[nphase][nstat] uint8: solves the sampler skips (no picks of that phase)."""
        hp, hs = self.station_flags()
        return np.stack([hp == 0, hs == 0][:max(1, self.nphase)]).astype(np.uint8)

    @property
    def n_s_picks(self):
        k = self.obs_stat
        return int(((self.luse != 0) & (k >= 0) & (k < self.nstat) & (self.pick_type == S_PRIMARY_PICK)).sum())

    # --- mceik_struct.h views (ctypes), kept alive on the problem ---
    def structs(self):
        keep = self._keep
        keep.clear()

        def dp(a):
            a = np.ascontiguousarray(a, dtype=np.float64); keep.append(a)
            return a.ctypes.data_as(C.POINTER(C.c_double))

        def ip(a):
            a = np.ascontiguousarray(a, dtype=np.int32); keep.append(a)
            return a.ctypes.data_as(C.POINTER(C.c_int))

        parms = _lib.MceikParms()
        parms.mcparms.nburnIn = int(self.nburn)
        parms.mcparms.niter = int(self.niter)
        parms.mcparms.keepK = int(self.keepk)
        parms.eikparms.tol = float(self.tol)
        parms.eikparms.maxit = int(self.maxit)
        parms.projnm = b"mceik_amd"
        parms.x0, parms.y0, parms.z0 = self.x0, self.y0, self.z0
        parms.dx = parms.dy = parms.dz = float(self.h)
        parms.ndivx = parms.ndivy = parms.ndivz = 1
        parms.nrefx, parms.nrefy, parms.nrefz = (int(v) for v in self.nref)
        st = _lib.StationsStruct()
        st.nstat = self.nstat
        st.lcartesian = int(self.lcartesian)
        st.xrec, st.yrec, st.zrec = dp(self.sx), dp(self.sy), dp(self.sz)
        st.pcorr = dp(self.pcorr)
        st.scorr = dp(self.scorr if self.scorr is not None else np.zeros(self.nstat))
        hp, hs = self.station_flags()
        st.lhasP = ip(hp)
        st.lhasS = ip(hs)
        cat = _lib.CatalogStruct()
        cat.nevents = self.nevents
        cat.xsrc, cat.ysrc, cat.zsrc = dp(self.ex), dp(self.ey), dp(self.ez)
        cat.tori = dp(np.zeros(self.nevents))
        cat.tobs = dp(self.tobs)
        cat.test = dp(np.zeros_like(self.tobs))
        cat.varObs = dp(self.var)
        cat.luseObs = ip(self.luse)
        cat.pickType = ip(self.pick_type)
        cat.statPtr = ip(self.obs_stat + 1)          # 1-based, homog.c:227
        cat.obsPtr = ip(self.obs_ptr)
        return parms, st, cat


def cell_velocity(p: Problem):
    """Heterogeneous base model on the inversion grid (SURVEY s.8d), int m/s."""
    k, j, i = np.meshgrid(np.arange(p.ncz), np.arange(p.ncy), np.arange(p.ncx), indexing="ij")
    xi, eta, zeta = (i + 0.5) / p.ncx, (j + 0.5) / p.ncy, (k + 0.5) / p.ncz
    v = 3000.0 + 4000.0 * zeta + 500.0 * np.sin(6 * np.pi * xi) * np.cos(4 * np.pi * eta) * np.sin(4 * np.pi * zeta)
    return np.rint(v).astype(np.int32).ravel()


def make_problem(config="C3", n=None, nstat=None, nev=None, h=None, homogeneous=None, nref=(4, 4, 4),
                 seed=2016, maxit=50, tol=1e-8, picks="analytic", phases="P"):
    """Synthetic problem of a BASELINE configuration (SURVEY s.8d).

    picks: 'analytic' -> straight-ray times in the mean velocity (no GPU needed);
           a callable(problem, phase) -> [nstat, nev] travel times in the P
           (phase 0) or S (phase 1) model, e.g. the GPU forward of `v_true` /
           `vs_true` (see `picks_from_forward`).  Gaussian noise (sigma 0.05 s)
           is added, varObs = 0.25 s^2 (homog.c:55-56).
    phases: 'P' (every station picks P of every event) or 'PS' (a P and an S
           pick per station and event, in homog.c's order, homog.c:203-229;
           the chains then hold a P and an S model, vs = vp / sqrt(3) as
           homog.c:53-54).
    """
    cfg = dict(CONFIGS[config])
    n = n or cfg["n"]; nstat = nstat or cfg["nstat"]; nev = nev or cfg["nev"]
    h = h or cfg["h"]
    homogeneous = cfg["homogeneous"] if homogeneous is None else homogeneous
    rng = np.random.default_rng(seed)
    p = Problem(nx=n, ny=n, nz=n, h=h, nref=tuple(nref), maxit=maxit, tol=tol, seed=seed)
    ext = (n - 1) * h
    # stations on the top face, x/y off-grid and >= 2 nodes from the edges
    p.sx = rng.uniform(2 * h, ext - 2 * h, nstat)
    p.sy = rng.uniform(2 * h, ext - 2 * h, nstat)
    p.sz = np.full(nstat, ext)
    p.pcorr = np.zeros(nstat)
    p.scorr = np.zeros(nstat)
    p.ex = rng.uniform(h, ext - h, nev)
    p.ey = rng.uniform(h, ext - h, nev)
    p.ez = rng.uniform(h, ext - h, nev)
    p.v_true = np.full(p.ncell, 2000 if config == "C1" else 4000, np.int32) if homogeneous else cell_velocity(p)
    nph = 2 if phases == "PS" else 1
    if phases not in ("P", "PS"):
        raise ValueError(f"phases: 'P' or 'PS', not {phases!r}")
    p.nphase = nph
    if nph == 2:
        p.vs_true = np.rint(p.v_true / np.sqrt(3.0)).astype(np.int32)
    # every station sees every event, CSR by event; per station P (then S)
    per = nstat * nph
    p.obs_ptr = (np.arange(nev + 1) * per).astype(np.int32)
    p.obs_stat = np.tile(np.repeat(np.arange(nstat, dtype=np.int32), nph), nev)
    p.pick_type = np.tile(np.arange(1, nph + 1, dtype=np.int32), nev * nstat)
    p.luse = np.ones(nev * per, np.int32)
    p.var = np.full(nev * per, 0.25)
    tt = np.empty((nph, nstat, nev))
    for ph in range(nph):
        if picks == "analytic":
            vmean = float(np.mean(p.vs_true if ph else p.v_true))
            d = np.sqrt((p.sx[:, None] - p.ex[None]) ** 2 + (p.sy[:, None] - p.ey[None]) ** 2 +
                        (p.sz[:, None] - p.ez[None]) ** 2)
            tt[ph] = d / vmean                           # [nstat, nev]
        else:
            tt[ph] = np.asarray(picks(p, ph) if nph == 2 else picks(p), dtype=np.float64).reshape(nstat, nev)
    # observation (e, k, ph) at e*per + k*nph + ph
    p.tobs = (tt.transpose(2, 1, 0).ravel() + rng.normal(0.0, 0.05, nev * per)).astype(np.float64)
    return p


def initial_models(p: Problem, chain_ids, amp=50):
    """Per-chain start model: v_true + integer noise in [-amp, amp], keyed by the
    GLOBAL chain id so the chains do not depend on how they are sharded.
    [n, ncell] for P problems, [n, 2, ncell] (P, S) for P/S problems."""
    if p.nphase == 1:
        out = np.empty((len(chain_ids), p.ncell), np.int32)
        for r, gid in enumerate(chain_ids):
            g = np.random.default_rng([p.seed, int(gid)])
            out[r] = np.clip(p.v_true + g.integers(-amp, amp + 1, p.ncell), p.vmin, p.vmax)
        return out
    out = np.empty((len(chain_ids), 2, p.ncell), np.int32)
    for r, gid in enumerate(chain_ids):
        g = np.random.default_rng([p.seed, int(gid)])
        out[r, 0] = np.clip(p.v_true + g.integers(-amp, amp + 1, p.ncell), p.vmin, p.vmax)
        g = np.random.default_rng([p.seed, int(gid), 1])
        out[r, 1] = np.clip(p.vs_true + g.integers(-amp, amp + 1, p.ncell), p.vsmin, p.vsmax)
    return out


def shard(nchains_total, rank, world):
    """Contiguous block of global chain ids for `rank` (SURVEY s.8e)."""
    base, extra = divmod(nchains_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class Sampler:
    """One GPU's chains (include/mceik.h handle)."""

    def __init__(self, p: Problem, nchains, chain_offset=0, v0=None, max_samples=0, device=0, precision=32,
                 max_waves=0):
        self.p = p
        self.nchains = int(nchains)
        self.chain_offset = int(chain_offset)
        if v0 is None:
            v0 = initial_models(p, range(chain_offset, chain_offset + nchains))
        self.v0 = np.ascontiguousarray(v0, dtype=np.int32)
        assert self.v0.shape == self.model_shape, (self.v0.shape, self.model_shape)
        L = _lib.lib()
        parms, st, cat = p.structs()
        o = _lib.McmcOpts()
        o.nx, o.ny, o.nz = p.nx, p.ny, p.nz
        o.nchains, o.chain_offset = self.nchains, self.chain_offset
        o.vmin, o.vmax, o.dvmax, o.seed = p.vmin, p.vmax, p.dvmax, p.seed
        o.max_samples, o.device = int(max_samples), int(device)
        o.precision, o.max_waves = int(precision), int(max_waves)
        o.tt_interp = int(p.tt_interp)
        o.nphase, o.vsmin, o.vsmax, o.mask_s = int(p.nphase), int(p.vsmin), int(p.vsmax), int(p.mask_s)
        h = C.c_void_p()
        rc = L.mceik_mcmc_init(C.byref(parms), C.byref(st), C.byref(cat), C.byref(o),
                               self.v0.ctypes.data_as(C.c_void_p), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_init failed ({rc})")
        self._h = h
        self._L = L
        self.max_samples = int(max_samples)
        self._last_full = True          # the last forward solved every model (init / restore)

    @property
    def model_shape(self):
        """Shape of the chains' models: [nchains, ncell] (P) or [nchains, 2, ncell] (P, S)."""
        p = self.p
        return (self.nchains, p.ncell) if p.nphase == 1 else (self.nchains, p.nphase, p.ncell)

    def set_stream(self, stream_ptr):
        self._L.mceik_mcmc_set_stream(self._h, C.c_void_p(stream_ptr))

    def run(self, nsteps):
        rc = self._L.mceik_mcmc_run(self._h, int(nsteps))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_run failed ({rc})")
        if nsteps:
            self._last_full = False

    def sync(self):
        rc = self._L.mceik_mcmc_sync(self._h)
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_sync failed ({rc})")

    def info(self):
        """mceik_mcmc_get_info as a dict (pipes, kernel instance, waves, workspaces)."""
        i = _lib.McmcInfo()
        if self._L.mceik_mcmc_get_info(self._h, C.byref(i)) != 0:
            raise RuntimeError("mceik_mcmc_get_info failed")
        n = i.npipe
        return {"npipe": n, "nphase": i.nphase, "step_z": i.step_z, "fixed_layout": bool(i.fixed_layout),
                "chains": list(i.chains[:n]), "waves": list(i.waves[:n]),
                "workspace_bytes": list(i.workspace_bytes[:n]), "lds_bytes": int(i.lds_bytes),
                "masked_s": i.masked_s, "kernel": i.kernel.decode(), "multi_step": bool(i.multi_step)}

    def state(self):
        v = np.empty(self.model_shape, np.int32)
        logl = np.empty(self.nchains, np.float64)
        nacc = np.empty(self.nchains, np.int64)
        step = C.c_longlong(0)
        rc = self._L.mceik_mcmc_get_state(self._h, v.ctypes.data_as(C.c_void_p), logl.ctypes.data_as(C.c_void_p),
                                          nacc.ctypes.data_as(C.c_void_p), C.byref(step))
        if rc != 0:
            raise RuntimeError("mceik_mcmc_get_state failed")
        return v, logl, nacc, step.value

    def last(self, with_ierr=False):
        """Host copies of the last forward's travel-time tables, iteration counts and
        accept flags (and the per-solve reference ierr if with_ierr).  After a step:
        [nchains, nstat, nev] / [nchains, nstat] of the model each proposal changed
        (`last_phase`); after init / restore with two models: [nchains, 2, nstat, nev]
        / [nchains, 2, nstat]."""
        tt, it, acc, ie = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._L.mceik_mcmc_last(self._h, C.byref(tt), C.byref(it), C.byref(acc), C.byref(ie))
        p = self.p
        mid = (p.nphase,) if (self._last_full and p.nphase > 1) else ()
        ttab = np.empty((self.nchains,) + mid + (p.nstat, p.nevents), np.float32)
        niter = np.empty((self.nchains,) + mid + (p.nstat,), np.int32)
        ierr = np.empty((self.nchains,) + mid + (p.nstat,), np.int32)
        a = np.empty(self.nchains, np.uint8)
        self.sync()
        for dst, src in ((ttab, tt), (niter, it), (a, acc), (ierr, ie)):
            if self._L.mceik_memcpy(dst.ctypes.data_as(C.c_void_p), src, dst.nbytes, 1) != 0:
                raise RuntimeError("mceik_memcpy failed")
        return (ttab, niter, a, ierr) if with_ierr else (ttab, niter, a)

    def last_phase(self):
        """The model each chain's last proposal changed (0 = P, 1 = S)."""
        ph = C.c_void_p()
        self._L.mceik_mcmc_last_phase(self._h, C.byref(ph))
        out = np.empty(self.nchains, np.int32)
        self.sync()
        if self._L.mceik_memcpy(out.ctypes.data_as(C.c_void_p), ph, out.nbytes, 1) != 0:
            raise RuntimeError("mceik_memcpy failed")
        return out

    def checkpoint(self):
        """Complete chain state (mceik_mcmc_checkpoint): dict of v, logl, naccept,
        step, nkept -- restore() into a sampler of the same problem/shard resumes
        the chains bit for bit."""
        v = np.empty(self.model_shape, np.int32)
        logl = np.empty(self.nchains, np.float64)
        nacc = np.empty(self.nchains, np.int64)
        step, nkept = C.c_longlong(0), C.c_int(0)
        if self._L.mceik_mcmc_checkpoint(self._h, v.ctypes.data_as(C.c_void_p), logl.ctypes.data_as(C.c_void_p),
                                         nacc.ctypes.data_as(C.c_void_p), C.byref(step), C.byref(nkept)) != 0:
            raise RuntimeError("mceik_mcmc_checkpoint failed")
        return {"v": v, "logl": logl, "naccept": nacc, "step": step.value, "nkept": nkept.value,
                "chain_offset": self.chain_offset, "seed": self.p.seed}

    def restore(self, ck, recompute_logl=False):
        """Load a checkpoint() dict (mceik_mcmc_restore)."""
        if ck.get("chain_offset", self.chain_offset) != self.chain_offset or ck.get("seed", self.p.seed) != self.p.seed:
            raise ValueError("checkpoint belongs to another chain shard or seed")
        v = np.ascontiguousarray(ck["v"], dtype=np.int32)
        assert v.shape == self.model_shape
        logl = None if recompute_logl else np.ascontiguousarray(ck["logl"], dtype=np.float64)
        nacc = np.ascontiguousarray(ck["naccept"], dtype=np.int64)
        rc = self._L.mceik_mcmc_restore(self._h, v.ctypes.data_as(C.c_void_p),
                                        None if logl is None else logl.ctypes.data_as(C.c_void_p),
                                        nacc.ctypes.data_as(C.c_void_p), int(ck["step"]), int(ck.get("nkept", 0)))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_restore failed ({rc})")
        if recompute_logl:
            self._last_full = True

    def fsm_stats(self, reset=False):
        """(FSM kernel ms from hipEvents, launches, executed iterations summed over
        solves, (brick visits, column segments updated, segments changed, wave macro
        steps))."""
        ms, nl, it, tv = C.c_double(0), C.c_longlong(0), C.c_ulonglong(0), (C.c_ulonglong * 4)()
        if self._L.mceik_mcmc_fsm_stats(self._h, C.byref(ms), C.byref(nl), C.byref(it), tv, int(reset)) != 0:
            raise RuntimeError("mceik_mcmc_fsm_stats failed")
        return ms.value, nl.value, it.value, tuple(tv)

    def fsm_solves(self):
        """Solves executed since init or the last fsm_stats(reset=True) (mceik_mcmc_fsm_solves;
        solves of stations without picks of the phase are skipped, not counted)."""
        n = C.c_ulonglong(0)
        if self._L.mceik_mcmc_fsm_solves(self._h, C.byref(n)) != 0:
            raise RuntimeError("mceik_mcmc_fsm_solves failed")
        return n.value

    def samples(self, max_states=None, device_ptr=None):
        """Kept states [k, *model_shape] (host numpy, or copied into device_ptr)."""
        max_states = self.max_samples if max_states is None else max_states
        n = C.c_int(0)
        if device_ptr is not None:
            self._L.mceik_mcmc_get_samples(self._h, C.c_void_p(device_ptr), None, max_states, 1, C.byref(n))
            return n.value
        v = np.empty((max(max_states, 1),) + self.model_shape, np.int32)
        lg = np.empty((max(max_states, 1), self.nchains), np.float64)
        self._L.mceik_mcmc_get_samples(self._h, v.ctypes.data_as(C.c_void_p), lg.ctypes.data_as(C.c_void_p),
                                       max_states, 0, C.byref(n))
        return v[:n.value], lg[:n.value]

    def close(self):
        if self._h:
            self._L.mceik_mcmc_finalize(C.byref(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def picks_from_forward(device=0, precision=64):
    """picks callable for make_problem: GPU forward of the true model (fp64 by
    default: the reference's arithmetic, and a different kernel instance from
    the fp32 sampler so profiles of the two do not mix).  f(p) or f(p, phase):
    phase 1 solves the S model `vs_true`."""
    def f(p: Problem, phase=0):
        import torch
        from .eikonal import BatchSolver
        dev = torch.device("cuda", device)
        bs = BatchSolver(p.nx, p.ny, p.nz, p.h, p.x0, p.y0, p.z0, p.maxit, p.tol, precision, nref=p.nref)
        src = torch.tensor(np.stack([np.zeros(p.nstat), p.sx, p.sy, p.sz], 1)[:, None, :], dtype=torch.float64)
        vt = p.vs_true if phase else p.v_true
        slow = torch.tensor((1.0 / vt.astype(np.float32)).astype(np.float32).reshape(1, -1), device=dev)
        out = bs.solve(src, slow, ev_node=torch.tensor(p.ev_node))
        torch.cuda.synchronize(dev)
        return out["ttab"].cpu().numpy().reshape(p.nstat, p.nevents)
    return f


def bench_picks(p: Problem, sigma=5e-4, device=0):
    """bench.py's observations on `p` (in place): the GPU forward of the true
    model (`picks_from_forward`) plus N(0, sigma) noise drawn with seed
    p.seed + 1, and varObs = sigma^2 -- sigma at the scale one proposal moves
    a travel time (~1 ms for 50 m/s on a 400-m cell), so Metropolis both
    accepts and rejects (DESIGN.md s.7 "Accept rate")."""
    tt = picks_from_forward(device)(p)
    rng = np.random.default_rng(p.seed + 1)
    p.tobs = tt.T.ravel().astype(np.float64) + rng.normal(0.0, sigma, p.nevents * p.nstat)
    p.var[:] = sigma ** 2
    return p


def gather_kept(smp: Sampler, nchains_total, group=None, dst=0, device=None):
    """Checkpoint gather (SURVEY s.8e): the most recent kept state of every
    chain on every rank -> rank `dst`, in global chain order.

    One process per GPU; `smp` holds this rank's shard `shard(nchains_total,
    rank, world)`.  With `device` (a torch CUDA device) the states move as
    device tensors -- over RCCL for an nccl group, xGMI on one node -- else as
    host tensors (gloo).  Shards are padded to the largest one, as gather
    needs equal sizes.  Returns (v [nchains_total, ncell] int32, logl
    [nchains_total] float64) torch tensors on `dst`, (None, None) elsewhere."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    width = -(-nchains_total // world)
    ncell = smp.p.ncell * smp.p.nphase           # a chain's model entries
    if device is not None:
        v = torch.zeros((width, ncell), dtype=torch.int32, device=device)
        lg = torch.zeros((width,), dtype=torch.float64, device=device)
        got = C.c_int(0)
        rc = smp._L.mceik_mcmc_get_samples(smp._h, C.c_void_p(v.data_ptr()), C.c_void_p(lg.data_ptr()), 1, 1,
                                           C.byref(got))
        if rc != 0 or got.value != 1:
            raise RuntimeError("mceik_mcmc_get_samples: no kept state to gather")
    else:
        kv, kl = smp.samples(max_states=1)
        if len(kv) == 0:
            raise RuntimeError("no kept state to gather (max_samples = 0 or still in burn-in)")
        v = torch.zeros((width, ncell), dtype=torch.int32)
        lg = torch.zeros((width,), dtype=torch.float64)
        v[:smp.nchains] = torch.from_numpy(kv[0].reshape(smp.nchains, ncell))
        lg[:smp.nchains] = torch.from_numpy(kl[0])
    gv = [torch.empty_like(v) for _ in range(world)] if rank == dst else None
    gl = [torch.empty_like(lg) for _ in range(world)] if rank == dst else None
    dist.gather(v, gv, dst=dst, group=group)
    dist.gather(lg, gl, dst=dst, group=group)
    if rank != dst:
        return None, None
    parts = [shard(nchains_total, r, world) for r in range(world)]
    return (torch.cat([gv[r][:hi - lo] for r, (lo, hi) in enumerate(parts)]),
            torch.cat([gl[r][:hi - lo] for r, (lo, hi) in enumerate(parts)]))


def comm_ready():
    """(ok, reason) of this process for the library communicator: the library
    loads and RCCL has every entry point it uses (mceik_comm_available).  No
    GPU call."""
    try:
        L = _lib.lib()
    except (OSError, ImportError) as exc:
        return False, f"libmceik_hip.so: {exc}"
    if not L.mceik_comm_available():
        return False, "RCCL (librccl.so.1) cannot be loaded"
    return True, ""


class CommUnavailable(RuntimeError):
    """Raised on EVERY rank alike when some rank cannot build the communicator
    (agreed before the collective mceik_comm_init)."""


class Comm:
    """RCCL communicator of the library's checkpoint gather (include/mceik.h
    mceik_comm_*): one rank per GPU.  `bootstrap` moves the 128-byte id from
    rank 0 to the others (an MPI main uses MPI_Bcast; here any callable
    bytes -> bytes, e.g. over torch.distributed: see `from_torch`).  `agree`
    (world > 1) maps this rank's `comm_ready()` to every rank's, so that all
    ranks give up together, before any of them enters the collective
    mceik_comm_init (which would wait forever for a rank that cannot join)."""

    def __init__(self, rank, world, device, bootstrap=None, agree=None, ready=comm_ready):
        if world > 1 and agree is not None:
            every = agree(ready())
            bad = [(r, why) for r, (ok, why) in enumerate(every) if not ok]
            if bad:
                raise CommUnavailable("; ".join(f"rank {r}: {why}" for r, why in bad))
        L = _lib.lib()
        uid = (C.c_ubyte * 128)()
        mine = None
        if rank == 0 and L.mceik_comm_unique_id(uid) == 0:
            mine = bytes(uid)
        if world > 1:
            mine = bootstrap(mine if rank == 0 else None)     # every rank learns the id, or that there is none
        if mine is None:
            raise RuntimeError("mceik_comm_unique_id failed on rank 0")
        C.memmove(uid, mine, 128)
        h = C.c_void_p()
        if L.mceik_comm_init(uid, int(world), int(rank), int(device), C.byref(h)) != 0:
            raise RuntimeError("mceik_comm_init failed")
        self._h, self._L, self.rank, self.world = h, L, rank, world

    @classmethod
    def from_torch(cls, device, group=None, ready=comm_ready):
        """Bootstrap (and the readiness agreement) over an initialised
        torch.distributed group."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)

        def bcast(b):
            box = [b]
            dist.broadcast_object_list(box, src=0, group=group)
            return box[0]

        def agree(mine):
            every = [None] * world
            dist.all_gather_object(every, mine, group=group)
            return every
        return cls(rank, world, device, bcast, agree, ready)

    def gather(self, smp: Sampler, nchains_total, which=1, root=0, v_out=None, logl_out=None):
        """mceik_mcmc_gather: every rank's chains -> `root` in global chain order.
        which 0 = current state, 1 = most recent kept state.  v_out / logl_out:
        torch tensors (device: received in place) or numpy arrays on the root;
        by default the root gets host numpy arrays.  Returns (v, logl) on the
        root, (None, None) elsewhere."""
        is_root = self.rank == root
        if is_root and v_out is None:
            v_out = np.empty((nchains_total,) + smp.model_shape[1:], np.int32)
            logl_out = np.empty(nchains_total, np.float64) if logl_out is None else logl_out

        def ptr(a):
            if a is None or not is_root:
                return None
            return a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
        rc = self._L.mceik_mcmc_gather(smp._h, self._h, int(which), int(nchains_total), int(root),
                                       ptr(v_out), ptr(logl_out))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_gather failed ({rc})")
        return (v_out, logl_out) if is_root else (None, None)

    def close(self):
        if self._h:
            self._L.mceik_comm_finalize(C.byref(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
