"""The reference's homog.c launch flow on torch.distributed (SURVEY s.8f row 3).

homog.c (homog.c:31-459) is the reference's MPI driver: rank 0 scatters six
receivers on the free surface and four events with glibc rand() seeded 2016,
attaches straight-ray P and S picks in a homogeneous medium (vp = 2000 m/s,
vs = vp/sqrt(3), varObs = 0.25 s^2), broadcasts the model, stations and
catalog (broadcast.c), splits the travel-time tables over the inter-table
communicator, writes them to `<proj>_<table group>_ttimes.h5` through h5io,
reads them back to verify (max |diff| <= 1e-5), initialises
`<proj>_locations.h5` and locates the events by grid search.

Here the same flow runs one process per GPU: communicator splitting becomes
torch.distributed groups (one table group per rank -- the build never
decomposes a grid over ranks, so the intra-table communicator has one rank),
broadcasts go over a gloo group (host metadata), tables are computed on the
rank's GPU by the FSM (`solver="fsm"`) or with homog.c's own analytic
formula (`solver="analytic"`, computeHomogeneousTraveltimes), gathered to
rank 0, written with libmceik_h5io.so, and the events are located by the GPU
relocation grid search (mceik_relocate).  The station/event generation is a
restatement (glibc rand() through ctypes, same call order): parity unpinned
by a reference run (homog.c needs parallel HDF5 and MPI, not in this image).

    python -m torch.distributed.run --nproc-per-node N -m mceik_amd.harness --dir OUT
"""
import argparse
import ctypes as C
import math
import os

import numpy as np

P_PRIMARY_PICK, S_PRIMARY_PICK = 1, 2          # mceik_struct.h:4-8
RAND_MAX = 2147483647


def homog_setup(seed=2016):
    """Stations, catalog and grid of homog.c:52-253 (glibc rand(), same order)."""
    libc = C.CDLL("libc.so.6")
    libc.rand.restype = C.c_int
    libc.srand(seed)
    rnd = lambda: libc.rand() / RAND_MAX
    x0 = y0 = z0 = 0.0
    x1, y1, z1 = 31.0e3, 28.0e3, 25.0e3
    dx = dy = dz = 1000.0
    nx = int((x1 - x0) / dx + 0.5) + 1
    ny = int((y1 - y0) / dy + 0.5) + 1
    nz = int((z1 - z0) / dz + 0.5) + 1
    const_vp = 2000.0
    const_vs = const_vp / math.sqrt(3.0)
    nxrec, nyrec, nevents = 2, 3, 4
    nstat = nxrec * nyrec
    xrec, yrec, zrec = np.zeros(nstat), np.zeros(nstat), np.zeros(nstat)
    for iy in range(nyrec):
        for ix in range(nxrec):
            k = iy * nxrec + ix
            xrec[k] = x0 + int(rnd() * (nx - 1)) * dx
            yrec[k] = y0 + int(rnd() * (ny - 1)) * dy
            zrec[k] = z1
    lhasP, lhasS = np.zeros(nstat, np.int32), np.zeros(nstat, np.int32)
    xsrc, ysrc, zsrc = np.zeros(nevents), np.zeros(nevents), np.zeros(nevents)
    tobs, var, luse, ptype, statptr, obsptr = [], [], [], [], [], [0]
    for i in range(nevents):
        xsrc[i] = x0 + (x1 - x0) * rnd()
        ysrc[i] = y0 + (y1 - y0) * rnd()
        zsrc[i] = z0 + (z1 - z0) * rnd()
        for k in range(nstat):
            dist = math.sqrt((xrec[k] - xsrc[i]) ** 2 + (yrec[k] - ysrc[i]) ** 2 + (zrec[k] - zsrc[i]) ** 2)
            for iphase in (P_PRIMARY_PICK, S_PRIMARY_PICK):
                tobs.append(dist / (const_vp if iphase == P_PRIMARY_PICK else const_vs))
                var.append(0.25)
                luse.append(1)
                ptype.append(iphase)
                statptr.append(k + 1)
            if i == 0:
                lhasP[k] = lhasS[k] = 1
        obsptr.append(len(tobs))
    grid = dict(nx=nx, ny=ny, nz=nz, x0=x0, y0=y0, z0=z0, dx=dx, dy=dy, dz=dz, vp=const_vp, vs=const_vs)
    stations = dict(xrec=xrec, yrec=yrec, zrec=zrec, pcorr=np.zeros(nstat), scorr=np.zeros(nstat),
                    lhasP=lhasP, lhasS=lhasS)
    catalog = dict(xsrc=xsrc, ysrc=ysrc, zsrc=zsrc, tori=np.zeros(nevents), tobs=np.array(tobs),
                   test=np.zeros(len(tobs)), varObs=np.array(var), luseObs=np.array(luse, np.int32),
                   pickType=np.array(ptype, np.int32), statPtr=np.array(statptr, np.int32),
                   obsPtr=np.array(obsptr, np.int32))
    return grid, stations, catalog


def homogeneous_traveltimes(nx, ny, nz, x0, y0, z0, dx, dy, dz, xs, ys, zs, vel):
    """homog.c computeHomogeneousTraveltimes: straight-ray times, x fastest."""
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    d = np.sqrt((x0 + i * dx - xs) ** 2 + (y0 + j * dy - ys) ** 2 + (z0 + k * dz - zs) ** 2)
    return (d / vel).ravel()


def table_list(stations):
    """homog.c:315-340: tables in station order, P then S where the station has them."""
    out = []
    for s in range(len(stations["xrec"])):
        if stations["lhasP"][s] == 1:
            out.append((s + 1, P_PRIMARY_PICK))
        if stations["lhasS"][s] == 1:
            out.append((s + 1, S_PRIMARY_PICK))
    return out


def _bcast_dict(d, root, group, keys):
    """broadcast.c pattern: sizes first, then every array, from `root`."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    for k in keys:
        if rank == root:
            a = np.ascontiguousarray(d[k])
            meta = torch.tensor([a.size, 0 if a.dtype.kind == "f" else 1], dtype=torch.int64)
        else:
            meta = torch.zeros(2, dtype=torch.int64)
        dist.broadcast(meta, root, group=group)
        dt = torch.float64 if int(meta[1]) == 0 else torch.int32
        t = torch.from_numpy(np.ascontiguousarray(d[k])).to(dt) if rank == root else \
            torch.zeros(int(meta[0]), dtype=dt)
        dist.broadcast(t, root, group=group)
        d[k] = t.numpy().astype(np.float64 if dt == torch.float64 else np.int32)
    return d


def broadcast_stations(stations, root=0, group=None):
    """broadcast.c:broadcast_stations over a (gloo) process group."""
    return _bcast_dict(stations, root, group, ("xrec", "yrec", "zrec", "pcorr", "scorr", "lhasP", "lhasS"))


def broadcast_catalog(catalog, root=0, group=None):
    """broadcast.c:98-150."""
    return _bcast_dict(catalog, root, group, ("xsrc", "ysrc", "zsrc", "tori", "tobs", "test", "varObs",
                                              "luseObs", "pickType", "statPtr", "obsPtr"))


def _fsm_tables(grid, stations, tables, device):
    """The rank's tables on its GPU: fp64 FSM (the reference's arithmetic),
    homogeneous slowness 1/v, one batched launch per phase."""
    import torch
    from .eikonal import BatchSolver
    g = grid
    n = g["nx"] * g["ny"] * g["nz"]
    out = {}
    for phase, vel in ((P_PRIMARY_PICK, g["vp"]), (S_PRIMARY_PICK, g["vs"])):
        mine = [(s, ph) for s, ph in tables if ph == phase]
        if not mine:
            continue
        src = torch.tensor([[[0.0, stations["xrec"][s - 1], stations["yrec"][s - 1], stations["zrec"][s - 1]]]
                            for s, _ in mine], dtype=torch.float64)
        slow = torch.full((1, g["nz"], g["ny"], g["nx"]), 1.0 / vel, dtype=torch.float64,
                          device=torch.device("cuda", device))
        bs = BatchSolver(g["nx"], g["ny"], g["nz"], g["dx"], g["x0"], g["y0"], g["z0"], maxit=50, tol=1e-8,
                         precision=64)
        res = bs.solve(src, slow, want_fields=True)
        u = res["u"].reshape(len(mine), n).cpu().numpy()
        ierr = res["ierr"].cpu().numpy()
        if np.any(ierr != 0):
            bad = [(mine[i][0], int(ierr[i])) for i in np.flatnonzero(ierr)]
            raise RuntimeError(f"eikonal solve failed for (station, ierr) {bad}: a station on the grid's "
                               "first node is the reference's SETBCS quirk (fsm3d.f90:736-745)")
        for i, key in enumerate(mine):
            out[key] = u[i]
    return out


def run_homog(dirnm, projnm="homog", solver="analytic", device=None, locate=True, seed=2016):
    """homog.c end to end.  Returns (hypocentres [nev, 3] or None, files)."""
    import torch.distributed as dist
    from . import h5io
    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank() if distributed else 0
    world = dist.get_world_size() if distributed else 1
    host_group = dist.new_group(backend="gloo") if distributed else None
    if rank == 0:
        grid, stations, catalog = homog_setup(seed)
    else:
        grid, stations, catalog = None, {}, {}
    if distributed:
        obj = [grid]
        dist.broadcast_object_list(obj, 0, group=host_group)
        grid = obj[0]
        stations = broadcast_stations(stations, 0, host_group)
        catalog = broadcast_catalog(catalog, 0, host_group)
    g = grid
    tables = table_list(stations)
    mine = tables[rank::world]                       # inter-table split, one rank per table group
    if solver == "fsm":
        tt = _fsm_tables(g, stations, mine, rank if device is None else device)
    else:
        tt = {(s, ph): homogeneous_traveltimes(g["nx"], g["ny"], g["nz"], g["x0"], g["y0"], g["z0"], g["dx"],
                                               g["dy"], g["dz"], stations["xrec"][s - 1], stations["yrec"][s - 1],
                                               stations["zrec"][s - 1], g["vp"] if ph == P_PRIMARY_PICK else g["vs"])
              for s, ph in mine}
    if distributed:
        parts = [None] * world if rank == 0 else None
        dist.gather_object(tt, parts, dst=0, group=host_group)
        if rank == 0:
            tt = {k: v for part in parts for k, v in part.items()}
    hypo, files = None, None
    if rank == 0:
        nmodels, model = 1, 1
        tproj = f"{projnm}_1"                            # homog.c:278: "<proj>_<table group>"
        tfile = h5io.init_ttables(dirnm, tproj, g["nx"], g["ny"], g["nz"], nmodels, len(stations["xrec"]),
                                  g["x0"], g["y0"], g["z0"], g["dx"], g["dy"], g["dz"])
        try:
            for (s, ph), t in sorted(tt.items()):
                t4 = t.astype(np.float32)                # double2FloatArray
                tfile.write_ttimes(s, model, t4, iphase=ph)
                back = tfile.read_ttimes(s, model, iphase=ph)
                if np.max(np.abs(back - t4)) > 1e-5:     # homog.c:388-397
                    raise RuntimeError("failed to read/write traveltime verification")
        finally:
            tfile.close()
        files = [h5io.file_name(1, dirnm, tproj)]
        if locate:
            hypo = _locate(dirnm, projnm, g, stations, catalog, tt, model)
            files.append(h5io.file_name(2, dirnm, projnm))
    if distributed:
        dist.barrier(group=host_group)
    return hypo, files


def _locate(dirnm, projnm, g, stations, catalog, tt, model):
    """Grid search location of every event against the written tables (the
    role of locate3d_gridsearch, homog.c:433-450): GPU relocation with the
    locate.c L2 objective; logJPDFs go to <proj>_locations.h5."""
    import torch
    from . import eikonal, h5io
    n = g["nx"] * g["ny"] * g["nz"]
    keys = sorted(tt)
    row = {k: i for i, k in enumerate(keys)}
    tables = torch.tensor(np.stack([tt[k].astype(np.float32) for k in keys]), device=torch.device("cuda"))
    events = []
    for e in range(len(catalog["xsrc"])):
        ks = range(catalog["obsPtr"][e], catalog["obsPtr"][e + 1])
        events.append(dict(rows=[row[(int(catalog["statPtr"][k]), int(catalog["pickType"][k]))] for k in ks],
                           tobs=np.float32([catalog["tobs"][k] for k in ks]),
                           varobs=np.float32([catalog["varObs"][k] for k in ks]),
                           mask=np.int32([0 if catalog["luseObs"][k] == 1 else 1 for k in ks])))
    logp, _ = eikonal.relocate(tables, events, log_pdf=True)
    logp = logp[:, :n].cpu().numpy()
    lfile = h5io.init_locations(dirnm, projnm, g["nx"], g["ny"], g["nz"], 1, len(events), g["x0"], g["y0"],
                                g["z0"], g["dx"], g["dy"], g["dz"])
    hypo = np.zeros((len(events), 3))
    try:
        for e in range(len(events)):
            lfile.write_logjpdf(model, e + 1, logp[e])
            idx = int(np.argmax(logp[e]))
            k, rem = divmod(idx, g["nx"] * g["ny"])
            j, i = divmod(rem, g["nx"])
            hypo[e] = (g["x0"] + i * g["dx"], g["y0"] + j * g["dy"], g["z0"] + k * g["dz"])
    finally:
        lfile.close()
    return hypo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=".")
    ap.add_argument("--proj", default="homog")
    ap.add_argument("--solver", default="fsm", choices=("fsm", "analytic"))
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    hypo, files = run_homog(args.dir, args.proj, solver=args.solver, device=local)
    if hypo is not None:
        for e, h in enumerate(hypo):
            print(f"event {e + 1}: located at x={h[0]:.0f} y={h[1]:.0f} z={h[2]:.0f} m")
        print("files:", " ".join(files))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
