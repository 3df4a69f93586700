"""Per-sweep change record of one fp32 solve (analysis tool, not product).

Runs the oracle's fp32 twin (oracle/fsm_impl.inc, bitwise the GPU's fields)
sweep by sweep on a C3 cell model -- each prefix of s sweeps from scratch
(oracle_eikonal3d_solve_dbg max_sweeps = s) -- and records, per sweep and
z-block (8x8 tile x 32 z, the fsm16 kernel's admission unit), whether the
block changed and which of its six face layers changed
(x-low, x-high, y-low, y-high, z-low, z-high; absolute orientation).
Output: npz with chg [nsweeps, nblocks], face [nsweeps, nblocks, 6], bc
(blocks holding boundary-condition nodes), geometry.

    python tools/sched/record.py OUT.npz [--chain 0] [--stations 0,5,10,...]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

ZB = int(os.environ.get("MCEIK_SIM_ZB", "32"))   # z per z-block (kb = 4 bricks of 8 z; 64: 4-step positions)


def block_flags(diff, nx, ny, nz):
    ntx, nty, nzk = -(-nx // 8), -(-ny // 8), -(-nz // ZB)
    d = np.zeros((nzk * ZB, nty * 8, ntx * 8), bool)
    d[:nz, :ny, :nx] = diff.reshape(nz, ny, nx)
    d = d.reshape(nzk, ZB, nty, 8, ntx, 8)
    chg = d.any(axis=(1, 3, 5))
    face = np.stack([d[:, :, :, :, :, 0].any(axis=(1, 3)), d[:, :, :, :, :, 7].any(axis=(1, 3)),
                     d[:, :, :, 0, :, :].any(axis=(1, 4)), d[:, :, :, 7, :, :].any(axis=(1, 4)),
                     d[:, 0, :, :, :, :].any(axis=(2, 4)), d[:, ZB - 1, :, :, :, :].any(axis=(2, 4))], -1)
    return chg.reshape(-1), face.reshape(-1, 6)


SWEEPS = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 1), (1, 1, 1)]


def relevance_flags_cons(u_prev, u, n, sweep, eps):
    """The kernel's cheap form of the rule: per node one upwind test (any of the
    three sweep-upwind neighbours, x / y / z) and one downwind test (x or y);
    an upwind hit marks the block itself and the upwind faces the node lies on,
    a downwind hit the downwind x / y faces it lies on; the downwind z face by
    the exact test of the block's last node."""
    rx, ry, rz = SWEEPS[sweep % 8]
    U, P = u.reshape(n, n, n), u_prev.reshape(n, n, n)
    chg = U != P
    one = U.dtype.type(1) + U.dtype.type(eps)
    up_any = np.zeros_like(chg)
    dn_any = np.zeros_like(chg)
    gedge = np.zeros_like(chg)
    face = {}
    hits = {}
    for ax, r, blk in ((2, rx, 8), (1, ry, 8), (0, rz, ZB)):
        for side in (-1, 1):
            upwind = (side == -1) == (r == 0)
            src = U if upwind else P
            nb = np.full_like(U, np.inf)
            sl_m = [slice(None)] * 3
            sl_n = [slice(None)] * 3
            if side == -1:
                sl_m[ax], sl_n[ax] = slice(1, None), slice(None, -1)
            else:
                sl_m[ax], sl_n[ax] = slice(None, -1), slice(1, None)
            nb[tuple(sl_m)] = src[tuple(sl_n)]
            rel = chg & (U < nb * one)
            idx = np.arange(n).reshape([-1 if a == ax else 1 for a in range(3)])
            on_face = (idx % blk == 0) if side == -1 else (idx % blk == blk - 1)
            edge = (idx == 0) if side == -1 else (idx == n - 1)
            gedge |= chg & edge
            hits[(ax, side)] = (rel & ~edge, on_face, upwind)
            if upwind:
                up_any |= rel & ~edge
            elif ax != 0:
                dn_any |= rel & ~edge
    own = up_any | gedge
    names = {(2, -1): 0, (2, 1): 1, (1, -1): 2, (1, 1): 3, (0, -1): 4, (0, 1): 5}
    fl = [None] * 6
    for (ax, side), (rel, on_face, upwind) in hits.items():
        if upwind:
            fl[names[(ax, side)]] = up_any & on_face
        elif ax != 0:
            fl[names[(ax, side)]] = dn_any & on_face
        else:
            fl[names[(ax, side)]] = rel & on_face
    def per_block(m):
        return block_flags(m.ravel(), n, n, n)[0]
    return per_block(own), np.stack([per_block(f) for f in fl], -1)


def relevance_flags(u_prev, u, n, sweep, eps):
    """Refined marks of one sweep (the relevance rule): a changed node m
    matters to a face neighbour n only if u_m(new) < u_n * (1 + eps), u_n the
    neighbour's value when m changed (new if n is sweep-upwind of m, i.e.
    already updated, else old).  own: some changed node of the block matters
    to a sweep-upwind neighbour inside the block (the block must be revisited
    next sweep); face[f]: a changed node on face f matters to the neighbour
    across it.  Absolute face order as block_flags."""
    rx, ry, rz = SWEEPS[sweep % 8]
    U, P = u.reshape(n, n, n), u_prev.reshape(n, n, n)
    chg = U != P
    own = np.zeros_like(chg)
    face = []
    one = U.dtype.type(1) + U.dtype.type(eps)
    for ax, r, blk in ((2, rx, 8), (1, ry, 8), (0, rz, ZB)):
        for side in (-1, 1):
            upwind = (side == -1) == (r == 0)        # the neighbour at side is updated before m
            src = U if upwind else P
            nb = np.full_like(U, np.inf)
            sl_m = [slice(None)] * 3
            sl_n = [slice(None)] * 3
            if side == -1:
                sl_m[ax], sl_n[ax] = slice(1, None), slice(None, -1)
            else:
                sl_m[ax], sl_n[ax] = slice(None, -1), slice(1, None)
            nb[tuple(sl_m)] = src[tuple(sl_n)]
            rel = chg & (U < nb * one)
            idx = np.arange(n).reshape([-1 if a == ax else 1 for a in range(3)])
            on_face = (idx % blk == 0) if side == -1 else (idx % blk == blk - 1)
            # on the grid boundary the update reads the node itself in place of the
            # missing neighbour (fsm3d.f90 UPDATE3D's edge rule): its own change is
            # an input of its next update -- the block must be revisited
            edge = (idx == 0) if side == -1 else (idx == n - 1)
            own |= chg & edge
            rel &= ~edge
            if upwind:
                own |= rel & ~on_face
            face.append(rel & on_face)
    # face order of block_flags: x-low, x-high, y-low, y-high, z-low, z-high
    def per_block(m):
        return block_flags(m.ravel(), n, n, n)[0]
    return per_block(own), np.stack([per_block(f) for f in face], -1)


def record_one(args):
    p_n, h, slow, src, maxit, tol, dt, eps = args
    import _oracle as O
    n = p_n
    u_prev = None
    _, _, niter = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt)
    nsw = 8 * niter
    chg, face, own_r, face_r = [], [], [], []
    # the field before the first sweep: SETBCS only (max_sweeps = 0)
    u_prev, _, _ = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt, max_sweeps=0)
    bcm = np.isfinite(u_prev) & (u_prev < np.float32(1e30))
    for s in range(1, nsw + 1):
        u, _, _ = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt, max_sweeps=s)
        c, f = block_flags(u != u_prev, n, n, n)
        chg.append(c); face.append(f)
        if eps is not None:
            o, fr = (relevance_flags_cons if os.environ.get("REL_CONS") else relevance_flags)(u_prev, u, n, s - 1, eps)
            own_r.append(o); face_r.append(fr)
        u_prev = u
    bc, _ = block_flags(bcm, n, n, n)
    return np.array(chg), np.array(face), bc, niter, np.array(own_r), np.array(face_r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--stations", default="0,5,10,15,20,25,30,31")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--prec", type=int, default=32, choices=(32, 64),
                    help="64: the fp64 sampler's forward (fp32 cell slowness promoted to fp64)")
    ap.add_argument("--rel", type=float, default=None,
                    help="also record the relevance rule's marks with this eps (own_rel, face_rel)")
    a = ap.parse_args()
    from mceik_amd import mcmc
    p = mcmc.make_problem("C3", picks="analytic")
    v = mcmc.initial_models(p, [a.chain])[0]
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    cell = ((k // p.nrz) * p.ncy + j // p.nry) * p.ncx + i // p.nrx
    slow = (1.0 / v.astype(np.float32)).astype(np.float32)[cell.ravel()]
    st = [int(s) for s in a.stations.split(",")]
    dt = np.float64 if a.prec == 64 else np.float32
    slow = slow.astype(dt)
    jobs = [(p.nx, p.h, slow, (0.0, p.sx[s], p.sy[s], p.sz[s]), p.maxit, p.tol, dt, a.rel) for s in st]
    import multiprocessing as mp
    with mp.get_context("fork").Pool(a.workers) as pool:
        res = pool.map(record_one, jobs)
    out = {"stations": np.array(st), "nx": p.nx, "ny": p.ny, "nz": p.nz, "zb": ZB}
    for k_, (c, f, bc, it, orl, frl) in enumerate(res):
        out[f"chg{k_}"], out[f"face{k_}"], out[f"bc{k_}"], out[f"niter{k_}"] = c, f, bc, it
        if a.rel is not None:
            out[f"own_rel{k_}"], out[f"face_rel{k_}"] = orl, frl
            print(f"station {st[k_]}: changed blocks {int(c.sum())}, self-relevant {int(orl.sum())}, "
                  f"changed faces {int(f.sum())}, relevant faces {int(frl.sum())}", flush=True)
        print(f"station {st[k_]}: {it} iterations, changed blocks per sweep {c.sum(1).tolist()}", flush=True)
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
