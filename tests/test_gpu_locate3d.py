"""The reference's MPI location driver entry points (include/locate.h:
locate3d_initialize / gridsearch / finalize, reference locate.f90:322-689)
under homog.c's location step (homog.c:428-450), on the GPU.

tests/c/homog_h5io.c writes homog.c's travel-time tables through the h5io
entry points, then (argument "locate <job>") calls the three entry points as
homog.c does and prints the hypocentres.  The reference's locate.f90 does not
compile (SURVEY s.0.5), so parity is unpinned by the reference: the oracle
here is this build's own relocation (mceik_amd.eikonal.relocate =
mceik_relocate, bitwise = compiled locate.c's fp32 grid search,
tests/test_gpu_fsm.py) on the tables read back from the same file, with the
MAXLOC over each rank's block and over the blocks in block order
(locate.f90:469-498).  Hypocentres, origin times and the estimates are
compared bit for bit, for one rank and for the grid split over two ranks.
"""
import os
import re
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI = "/opt/conda"
NX, NY, NZ = 32, 29, 26                       # homog.c:76-89 (tests/c/homog_h5io.c)


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not (os.path.exists(f"{MPI}/include/mpi.h") and os.path.exists(f"{MPI}/bin/mpiexec")):
        pytest.skip("no MPI toolchain in this image")
    lib = os.path.join(ROOT, "mceik_amd")
    out = str(tmp_path_factory.mktemp("homog_loc") / "homog_h5io")
    subprocess.run(["gcc", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", f"{MPI}/include",
                    os.path.join(ROOT, "tests", "c", "homog_h5io.c"), "-L", lib, "-lmceik_hip", "-lmceik_h5io",
                    f"{MPI}/lib/libmpi.so", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}:{MPI}/lib", "-lm",
                    "-o", out], check=True)
    return out


def _catalog(tables_of):
    """The catalogue homog_h5io.c builds (rank 0, srand(2016)): 6 stations
    (station 3 without S), 4 events, a P and an S pick per station and event,
    varObs 0.25; tobs from the straight-ray times."""
    import ctypes as C
    libc = C.CDLL("libc.so.6")
    libc.srand(2016)
    rmax = 2147483647.0
    h, vp = 1000.0, 2000.0
    vs = vp / np.sqrt(3.0)
    st = []
    for _ in range(6):
        x = int(libc.rand() / rmax * (NX - 1)) * h
        y = int(libc.rand() / rmax * (NY - 1)) * h
        st.append((x, y, 25.e3))
    ev = []
    for i in range(4):
        xs = 31.e3 * libc.rand() / rmax
        ys = 28.e3 * libc.rand() / rmax
        zs = 25.e3 * libc.rand() / rmax
        obs = []
        for k, (x, y, z) in enumerate(st):
            d = np.sqrt((x - xs) ** 2 + (y - ys) ** 2 + (z - zs) ** 2)
            for ph in (1, 2):
                use = not (ph == 2 and k == 2)
                obs.append((k + 1, ph, d / (vp if ph == 1 else vs), 0.25, use))
        ev.append(obs)
    return ev


def _run(exe, n, ndivx, job, outdir):
    r = subprocess.run([f"{MPI}/bin/mpiexec", "-n", str(n), exe, str(outdir), "homog", str(ndivx), "locate",
                        str(job)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    hypo = {int(m[0]): [float(v) for v in m[1:]] for m in re.findall(r"^LOCATE (\d+) (\S+) (\S+) (\S+) (\S+)$",
                                                                           r.stdout, re.M)}
    test = [(int(u), float(t)) for u, t in re.findall(r"^TEST \d+ (\d) (\S+)$", r.stdout, re.M)]
    return hypo, test


def _expected(outdir, ndivx, job):
    """eikonal.relocate on the file's tables, MAXLOC per block (x split in
    ndivx blocks as homog.c / locate3d_initialize), first block with the
    largest log-PDF."""
    from mceik_amd import eikonal, h5io
    ev = _catalog(None)
    with h5io.H5File.open(os.path.join(str(outdir), "homog_1_ttimes.h5")) as f:
        xl, yl, zl = f.model()
        keys = sorted({(s, p) for obs in ev for s, p, _, _, u in obs if u})
        rowof = {k: i for i, k in enumerate(keys)}
        tabs = np.stack([f.read_ttimes(s, 1, p) for s, p in keys])
    dev = torch.device("cuda", 0)
    tables = torch.tensor(tabs, device=dev)
    events = [{"rows": [rowof[(s, p)] for s, p, _, _, u in obs if u], "tobs": [t for _, _, t, _, u in obs if u],
               "varobs": [v for _, _, _, v, u in obs if u]} for obs in ev]
    tori = [0.5 * i for i in range(4)]
    if job == 2:
        logp, t0 = eikonal.relocate(tables, events, log_pdf=True)
        logp, t0 = logp.cpu().numpy(), t0.cpu().numpy()
    else:
        parts = [eikonal.relocate(tables, [e], iwantOT=0, t0use=tori[i], log_pdf=True, single_pass=False)
                 for i, e in enumerate(events)]
        logp = np.concatenate([p[0].cpu().numpy() for p in parts])
    ndx = max(NX // ndivx, 1)
    k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(NX), indexing="ij")
    out = {}
    for e in range(4):
        best = None
        for b in range(ndivx):
            i1, i2 = ndx * b, (NX if b == ndivx - 1 else ndx * (b + 1))
            blk = np.flatnonzero(((i >= i1) & (i < i2)).ravel())   # x-fastest order within the block too
            g = blk[int(np.argmax(logp[e, blk]))]
            if best is None or logp[e, g] > logp[e, best]:
                best = g
        t0e = float(t0[e, best]) if job == 2 else tori[e]
        est = [(1 if u else 0, t0e + float(tabs[rowof[(s, p)], best]) if u else 0.0) for s, p, _, _, u in ev[e]]
        out[e + 1] = ([float(xl[best]), float(yl[best]), float(zl[best]), t0e], est)
    return out


@pytest.mark.parametrize("n,ndivx,job", [(1, 1, 2), (2, 2, 2), (1, 1, 1)])
def test_locate3d_entry_points_equal_relocation(exe, tmp_path, n, ndivx, job):
    """homog.c's location step through locate3d_* (one rank, and the grid
    split in two blocks over two ranks sharing the GPU): every hypocentre
    (x, y, z, t0) and event 1's estimates bitwise = the relocation oracle."""
    hypo, test = _run(exe, n, ndivx, job, tmp_path)
    want = _expected(tmp_path, ndivx, job)
    assert sorted(hypo) == [1, 2, 3, 4]
    for e in range(1, 5):
        assert hypo[e] == want[e][0], (e, hypo[e], want[e][0])
    assert test == want[1][1]
    print(f"LOCATE3D n={n} job={job}: " + "; ".join(f"{e}: {hypo[e]}" for e in range(1, 5)))
