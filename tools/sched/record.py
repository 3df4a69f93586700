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

ZB = 32          # z per z-block (kb = 4 bricks of 8 z)


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


def record_one(args):
    p_n, h, slow, src, maxit, tol, dt = args
    import _oracle as O
    n = p_n
    u_prev = None
    _, _, niter = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt)
    nsw = 8 * niter
    chg, face = [], []
    # the field before the first sweep: SETBCS only (max_sweeps = 0)
    u_prev, _, _ = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt, max_sweeps=0)
    bcm = np.isfinite(u_prev) & (u_prev < np.float32(1e30))
    for s in range(1, nsw + 1):
        u, _, _ = O.eikonal_solve(n, n, n, slow, h, [src], maxit, tol, dtype=dt, max_sweeps=s)
        c, f = block_flags(u != u_prev, n, n, n)
        chg.append(c); face.append(f)
        u_prev = u
    bc, _ = block_flags(bcm, n, n, n)
    return np.array(chg), np.array(face), bc, niter


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--stations", default="0,5,10,15,20,25,30,31")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--prec", type=int, default=32, choices=(32, 64),
                    help="64: the fp64 sampler's forward (fp32 cell slowness promoted to fp64)")
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
    jobs = [(p.nx, p.h, slow, (0.0, p.sx[s], p.sy[s], p.sz[s]), p.maxit, p.tol, dt) for s in st]
    import multiprocessing as mp
    with mp.get_context("fork").Pool(a.workers) as pool:
        res = pool.map(record_one, jobs)
    out = {"stations": np.array(st), "nx": p.nx, "ny": p.ny, "nz": p.nz}
    for k_, (c, f, bc, it) in enumerate(res):
        out[f"chg{k_}"], out[f"face{k_}"], out[f"bc{k_}"], out[f"niter{k_}"] = c, f, bc, it
        print(f"station {st[k_]}: {it} iterations, changed blocks per sweep {c.sum(1).tolist()}", flush=True)
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
