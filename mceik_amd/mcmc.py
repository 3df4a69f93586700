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
    seed: int = 2016
    nburn: int = 0
    keepk: int = 1
    niter: int = 0                  # mcparms.niter: total proposals (Sampler.run(-1) runs the rest)
    tt_interp: int = 0              # 0: event times at the nearest node (reference); 1: trilinear in the cell
    v_true: np.ndarray = None       # [ncell] int, model used to make the picks
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
    def obs_mask(self):
        return (~((self.luse != 0) & (self.pick_type == P_PRIMARY_PICK))).astype(np.int32)

    @property
    def tcorr(self):
        return np.where(self.obs_mask == 0, self.pcorr[self.obs_stat], 0.0)

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
        st.lcartesian = 1
        st.xrec, st.yrec, st.zrec = dp(self.sx), dp(self.sy), dp(self.sz)
        st.pcorr = dp(self.pcorr)
        st.scorr = dp(np.zeros(self.nstat))
        st.lhasP = ip(np.ones(self.nstat))
        st.lhasS = ip(np.zeros(self.nstat))
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
                 seed=2016, maxit=50, tol=1e-8, picks="analytic"):
    """Synthetic problem of a BASELINE configuration (SURVEY s.8d).

    picks: 'analytic' -> straight-ray times in the mean velocity (no GPU needed);
           a callable(problem) -> [nstat, nev] travel times, e.g. the GPU forward
           of `v_true` (see `picks_from_forward`).  Gaussian noise (sigma 0.05 s)
           is added, varObs = 0.25 s^2 (homog.c:55).
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
    p.ex = rng.uniform(h, ext - h, nev)
    p.ey = rng.uniform(h, ext - h, nev)
    p.ez = rng.uniform(h, ext - h, nev)
    p.v_true = np.full(p.ncell, 2000 if config == "C1" else 4000, np.int32) if homogeneous else cell_velocity(p)
    # every station sees every event (P only), CSR by event
    p.obs_ptr = (np.arange(nev + 1) * nstat).astype(np.int32)
    p.obs_stat = np.tile(np.arange(nstat, dtype=np.int32), nev)
    p.pick_type = np.full(nev * nstat, P_PRIMARY_PICK, np.int32)
    p.luse = np.ones(nev * nstat, np.int32)
    p.var = np.full(nev * nstat, 0.25)
    if picks == "analytic":
        vmean = float(np.mean(p.v_true))
        d = np.sqrt((p.sx[:, None] - p.ex[None]) ** 2 + (p.sy[:, None] - p.ey[None]) ** 2 +
                    (p.sz[:, None] - p.ez[None]) ** 2)
        tt = d / vmean                               # [nstat, nev]
    else:
        tt = np.asarray(picks(p), dtype=np.float64).reshape(nstat, nev)
    p.tobs = (tt.T.ravel() + rng.normal(0.0, 0.05, nev * nstat)).astype(np.float64)
    return p


def initial_models(p: Problem, chain_ids, amp=50):
    """Per-chain start model: v_true + integer noise in [-amp, amp], keyed by the
    GLOBAL chain id so the chains do not depend on how they are sharded."""
    out = np.empty((len(chain_ids), p.ncell), np.int32)
    for r, gid in enumerate(chain_ids):
        g = np.random.default_rng([p.seed, int(gid)])
        out[r] = np.clip(p.v_true + g.integers(-amp, amp + 1, p.ncell), p.vmin, p.vmax)
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
        assert self.v0.shape == (self.nchains, p.ncell)
        L = _lib.lib()
        parms, st, cat = p.structs()
        o = _lib.McmcOpts()
        o.nx, o.ny, o.nz = p.nx, p.ny, p.nz
        o.nchains, o.chain_offset = self.nchains, self.chain_offset
        o.vmin, o.vmax, o.dvmax, o.seed = p.vmin, p.vmax, p.dvmax, p.seed
        o.max_samples, o.device = int(max_samples), int(device)
        o.precision, o.max_waves = int(precision), int(max_waves)
        o.tt_interp = int(p.tt_interp)
        h = C.c_void_p()
        rc = L.mceik_mcmc_init(C.byref(parms), C.byref(st), C.byref(cat), C.byref(o),
                               self.v0.ctypes.data_as(C.c_void_p), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_init failed ({rc})")
        self._h = h
        self._L = L
        self.max_samples = int(max_samples)

    def set_stream(self, stream_ptr):
        self._L.mceik_mcmc_set_stream(self._h, C.c_void_p(stream_ptr))

    def run(self, nsteps):
        rc = self._L.mceik_mcmc_run(self._h, int(nsteps))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_run failed ({rc})")

    def sync(self):
        self._L.mceik_mcmc_sync(self._h)

    def state(self):
        v = np.empty((self.nchains, self.p.ncell), np.int32)
        logl = np.empty(self.nchains, np.float64)
        nacc = np.empty(self.nchains, np.int64)
        step = C.c_longlong(0)
        rc = self._L.mceik_mcmc_get_state(self._h, v.ctypes.data_as(C.c_void_p), logl.ctypes.data_as(C.c_void_p),
                                          nacc.ctypes.data_as(C.c_void_p), C.byref(step))
        if rc != 0:
            raise RuntimeError("mceik_mcmc_get_state failed")
        return v, logl, nacc, step.value

    def last(self, with_ierr=False):
        """Host copies of the last step's travel-time table, iteration counts and
        accept flags (and the per-solve reference ierr if with_ierr)."""
        tt, it, acc, ie = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._L.mceik_mcmc_last(self._h, C.byref(tt), C.byref(it), C.byref(acc), C.byref(ie))
        p = self.p
        ttab = np.empty((self.nchains, p.nstat, p.nevents), np.float32)
        niter = np.empty((self.nchains, p.nstat), np.int32)
        ierr = np.empty((self.nchains, p.nstat), np.int32)
        a = np.empty(self.nchains, np.uint8)
        self.sync()
        for dst, src in ((ttab, tt), (niter, it), (a, acc), (ierr, ie)):
            if self._L.mceik_memcpy(dst.ctypes.data_as(C.c_void_p), src, dst.nbytes, 1) != 0:
                raise RuntimeError("mceik_memcpy failed")
        return (ttab, niter, a, ierr) if with_ierr else (ttab, niter, a)

    def checkpoint(self):
        """Complete chain state (mceik_mcmc_checkpoint): dict of v, logl, naccept,
        step, nkept -- restore() into a sampler of the same problem/shard resumes
        the chains bit for bit."""
        v = np.empty((self.nchains, self.p.ncell), np.int32)
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
        assert v.shape == (self.nchains, self.p.ncell)
        logl = None if recompute_logl else np.ascontiguousarray(ck["logl"], dtype=np.float64)
        nacc = np.ascontiguousarray(ck["naccept"], dtype=np.int64)
        rc = self._L.mceik_mcmc_restore(self._h, v.ctypes.data_as(C.c_void_p),
                                        None if logl is None else logl.ctypes.data_as(C.c_void_p),
                                        nacc.ctypes.data_as(C.c_void_p), int(ck["step"]), int(ck.get("nkept", 0)))
        if rc != 0:
            raise RuntimeError(f"mceik_mcmc_restore failed ({rc})")

    def fsm_stats(self, reset=False):
        """(FSM kernel ms from hipEvents, launches, executed iterations summed over
        solves, (tile visits, column segments updated, segments changed))."""
        ms, nl, it, tv = C.c_double(0), C.c_longlong(0), C.c_ulonglong(0), (C.c_ulonglong * 3)()
        if self._L.mceik_mcmc_fsm_stats(self._h, C.byref(ms), C.byref(nl), C.byref(it), tv, int(reset)) != 0:
            raise RuntimeError("mceik_mcmc_fsm_stats failed")
        return ms.value, nl.value, it.value, tuple(tv)

    def samples(self, max_states=None, device_ptr=None):
        """Kept states [k, nchains, ncell] (host numpy, or copied into device_ptr)."""
        max_states = self.max_samples if max_states is None else max_states
        n = C.c_int(0)
        if device_ptr is not None:
            self._L.mceik_mcmc_get_samples(self._h, C.c_void_p(device_ptr), None, max_states, 1, C.byref(n))
            return n.value
        v = np.empty((max(max_states, 1), self.nchains, self.p.ncell), np.int32)
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
    the fp32 sampler so profiles of the two do not mix)."""
    def f(p: Problem):
        import torch
        from .eikonal import BatchSolver
        dev = torch.device("cuda", device)
        bs = BatchSolver(p.nx, p.ny, p.nz, p.h, p.x0, p.y0, p.z0, p.maxit, p.tol, precision, nref=p.nref)
        src = torch.tensor(np.stack([np.zeros(p.nstat), p.sx, p.sy, p.sz], 1)[:, None, :], dtype=torch.float64)
        slow = torch.tensor((1.0 / p.v_true.astype(np.float32)).astype(np.float32).reshape(1, -1), device=dev)
        out = bs.solve(src, slow, ev_node=torch.tensor(p.ev_node))
        torch.cuda.synchronize(dev)
        return out["ttab"].cpu().numpy().reshape(p.nstat, p.nevents)
    return f


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
    ncell = smp.p.ncell
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
        v[:smp.nchains] = torch.from_numpy(kv[0])
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


class Comm:
    """RCCL communicator of the library's checkpoint gather (include/mceik.h
    mceik_comm_*): one rank per GPU.  `bootstrap` moves the 128-byte id from
    rank 0 to the others (an MPI main uses MPI_Bcast; here any callable
    bytes -> bytes, e.g. over torch.distributed: see `from_torch`)."""

    def __init__(self, rank, world, device, bootstrap=None):
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
    def from_torch(cls, device, group=None):
        """Bootstrap over an initialised torch.distributed group."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)

        def bcast(b):
            box = [b]
            dist.broadcast_object_list(box, src=0, group=group)
            return box[0]
        return cls(rank, world, device, bcast)

    def gather(self, smp: Sampler, nchains_total, which=1, root=0, v_out=None, logl_out=None):
        """mceik_mcmc_gather: every rank's chains -> `root` in global chain order.
        which 0 = current state, 1 = most recent kept state.  v_out / logl_out:
        torch tensors (device: received in place) or numpy arrays on the root;
        by default the root gets host numpy arrays.  Returns (v, logl) on the
        root, (None, None) elsewhere."""
        is_root = self.rank == root
        if is_root and v_out is None:
            v_out = np.empty((nchains_total, smp.p.ncell), np.int32)
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
