"""The reference-signature harness entry points (include/h5io.h,
include/mceik_broadcast.h) under a homog.c-style MPI main, on the CPU.

tests/c/homog_h5io.c restates homog.c:31-451's table and location I/O: rank
0 builds homog.c's station list and catalog (srand(2016)), broadcast_stations
/ broadcast_catalog distribute them, every rank writes its block of each
table (one per lhasP / lhasS flag) with eikonal_h5io_writeTravelTimes, reads
it back and checks |d| <= 1e-5 (homog.c:389-413), then the location file.
The communicators come from mpiutils_initialize3d / getCommunicators as in
homog.c:90-110 (table groups of ndivx blocks).  It must build against
include/ and both libraries and pass under mpiexec -n 1, -n 2 and -n 4 (two
table groups).  The files it leaves are then checked here dataset by dataset:
with one rank they are bitwise what the serial Python writer (mceik_amd.h5io,
the posterior writer's path) writes for the same tables; with blocks they
hold exactly what the reference's collective hyperslab writes leave (each
rank's x-fastest block written through a {nxMax, nyMax, nzMax} memory space
at {ix0, iy0, iz0}, h5io.c:883-925), restated here in numpy.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from mceik_amd import h5io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI = "/opt/conda"
NX, NY, NZ, H = 32, 29, 26, 1000.0            # homog.c:76-89
VP = 2000.0
VS = VP / np.sqrt(3.0)


def _mpi():
    if not (os.path.exists(f"{MPI}/include/mpi.h") and os.path.exists(f"{MPI}/bin/mpiexec")):
        pytest.skip("no MPI toolchain in this image")


@pytest.fixture(scope="module")
def homog_exe(tmp_path_factory):
    _mpi()
    lib = os.path.join(ROOT, "mceik_amd")
    exe = str(tmp_path_factory.mktemp("homog") / "homog_h5io")
    subprocess.run(["gcc", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", f"{MPI}/include",
                    os.path.join(ROOT, "tests", "c", "homog_h5io.c"), "-L", lib, "-lmceik_hip", "-lmceik_h5io",
                    f"{MPI}/lib/libmpi.so", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}:{MPI}/lib", "-lm",
                    "-o", exe], check=True)
    return exe


def _run(exe, n, outdir, ndivx=None):
    ndivx = ndivx or n
    r = subprocess.run([f"{MPI}/bin/mpiexec", "-n", str(n), exe, str(outdir), "homog", str(ndivx)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"homog_h5io: {n} ranks, {n // ndivx} table groups, 11 tables ok" in r.stdout
    return r


def _stations():
    """homog.c:141-166 with glibc's rand() seeded by srand(2016)."""
    libc = C.CDLL("libc.so.6")
    libc.srand(2016)
    rmax = 2147483647.0
    xs, ys = [], []
    for _ in range(6):
        xs.append(((int(libc.rand() / rmax * (NX - 1)))) * H)
        ys.append(((int(libc.rand() / rmax * (NY - 1)))) * H)
    return np.array(xs), np.array(ys), np.full(6, 25.e3)


def _block_times(xs, ys, zs, vel, ix0, nxl):
    """homog.c:594-621 on the block [ix0, ix0 + nxl) x ny x nz, x fastest."""
    k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(nxl), indexing="ij")
    x, y, z = (ix0 + i) * H, j * H, k * H
    d = np.sqrt((xs - x) ** 2 + (ys - y) ** 2 + (zs - z) ** 2)
    return (d * (1.0 / vel)).astype(np.float32).ravel()


def _hyperslab_file(blocks, nmax):
    """What the reference's collective writes leave in the {nx, ny, nz}
    dataset: rank r's padded x-fastest block, read by HDF5 as a C-order
    {nxMax, nyMax, nzMax} array, lands at {ix0, 0, 0}; rank order."""
    f = np.zeros((NX, NY, NZ), np.float32)
    for ix0, blk in blocks:
        f[ix0:ix0 + nmax[0], :nmax[1], :nmax[2]] = blk.reshape(nmax)
    return f.ravel()


def _raw(f, name):
    """A dataset's raw contents (dataspace {nx, ny, nz}, C order)."""
    a = np.zeros(NX * NY * NZ, np.float32)
    L = h5io.lib()
    m = re.match(r"/TravelTimeTables/Model_(\d+)/Station_(\d+)/([PS])TravelTimes", name)
    if m:
        rc = L.mceik_h5io_readTravelTimes(f.fid, int(m.group(2)), int(m.group(1)), 1 if m.group(3) == "P" else 2,
                                          NX, NY, NZ, a.ctypes.data_as(C.c_void_p))
    else:
        m = re.match(r"/logJPDFs/Event_(\d+)/Model_(\d+)/logJPDF", name)
        rc = L.mceik_h5io_readLocationLogJPDF(f.fid, int(m.group(2)), int(m.group(1)), NX, NY, NZ,
                                              a.ctypes.data_as(C.c_void_p))
    assert rc == 0, name
    return a


def _tables():
    xs, ys, zs = _stations()
    return [(k + 1, ph, xs[k], ys[k], zs[k]) for k in range(6) for ph in (1, 2) if not (ph == 2 and k == 2)]


def test_homog_flow_one_rank_equals_python_writer(homog_exe, tmp_path):
    """mpiexec -n 1: the harness flow passes, and every dataset of both files
    is bitwise what the serial Python writer writes for the same tables."""
    _run(homog_exe, 1, tmp_path)
    py = tmp_path / "py"
    py.mkdir()
    ref = h5io.init_ttables(str(py), "homog", NX, NY, NZ, 1, 6, 0.0, 0.0, 0.0, H, H, H)
    for st, ph, x, y, z in _tables():
        ref.write_ttimes(st, 1, _block_times(x, y, z, VS if ph == 2 else VP, 0, NX), iphase=ph)
    loc = h5io.init_locations(str(py), "homog", NX, NY, NZ, 1, 4, 0.0, 0.0, 0.0, H, H, H)
    jp = -(np.arange(NX * NY * NZ) % 97).astype(np.float32)
    loc.write_logjpdf(1, 2, jp)
    got = h5io.H5File.open(str(tmp_path / "homog_1_ttimes.h5"))
    try:
        assert got.dims() == (NX, NY, NZ)
        for a, b in zip(got.model(), ref.model()):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        for st in range(1, 7):
            for ph in (1, 2):
                name = h5io.travel_time_name(1, st, ph == 1)
                assert np.array_equal(_raw(got, name).view(np.uint32), _raw(ref, name).view(np.uint32)), name
        assert not _raw(got, h5io.travel_time_name(1, 3, False)).any()     # lhasS = 0: the null table
    finally:
        got.close()
        ref.close()
    gl = h5io.H5File.open(str(tmp_path / "homog_locations.h5"))
    try:
        for e in range(1, 5):
            name = h5io.location_name(1, e)
            assert np.array_equal(_raw(gl, name).view(np.uint32), _raw(loc, name).view(np.uint32)), name
        assert gl.exists("/Model/priorLocationModel")
    finally:
        gl.close()
        loc.close()


@pytest.mark.parametrize("nranks", [2, 4])
def test_homog_flow_blocks_hyperslab_layout(homog_exe, tmp_path, nranks):
    """mpiexec -n 2 and -n 4 with ndivx = 2 (homog.c:82): mpiutils_initialize3d
    makes nranks / 2 table groups of two x blocks; the flow passes
    (broadcasts, per-rank write / read-back within 1e-5, readModel of each
    block), and each group's table file holds exactly the reference's
    collective hyperslab writes of its two 16-node x blocks."""
    _run(homog_exe, nranks, tmp_path, ndivx=2)
    nmax = (NX // 2, NY, NZ)
    for group in range(1, nranks // 2 + 1):
        got = h5io.H5File.open(str(tmp_path / f"homog_{group}_ttimes.h5"))
        try:
            for st, ph, x, y, z in _tables():
                vel = VS if ph == 2 else VP
                want = _hyperslab_file([(r * 16, _block_times(x, y, z, vel, r * 16, 16)) for r in range(2)], nmax)
                name = h5io.travel_time_name(1, st, ph == 1)
                assert np.array_equal(_raw(got, name).view(np.uint32), want.view(np.uint32)), (group, name)
            k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(16), indexing="ij")
            xl = _hyperslab_file([(r * 16, ((r * 16 + i) * H).astype(np.float32).ravel()) for r in range(2)], nmax)
            a = np.zeros(NX * NY * NZ, np.float32)
            assert h5io.lib().mceik_h5io_readModel(got.fid, NX, NY, NZ, a.ctypes.data_as(C.c_void_p), None,
                                                   None) == 0
            assert np.array_equal(a, xl)
        finally:
            got.close()
    gl = h5io.H5File.open(str(tmp_path / "homog_locations.h5"))
    try:
        blk = [(r * 16, (-(np.arange(16 * NY * NZ) % 97) - 0.25 * r).astype(np.float32)) for r in range(2)]
        assert np.array_equal(_raw(gl, h5io.location_name(1, 2)), _hyperslab_file(blk, nmax))
        assert not _raw(gl, h5io.location_name(1, 3)).any()
    finally:
        gl.close()


def test_reference_signature_exports():
    """Every function include/h5io.h declares is exported by libmceik_h5io.so,
    and mceik_broadcast.h's and mpiutils.h's by libmceik_hip.so."""
    def declared(h):
        txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", h)).read(), flags=re.S)
        return {m.group(1) for m in re.finditer(r"^\s*(?:int|void)\s+([A-Za-z_]\w*)\s*\(", txt, flags=re.M)}

    def exported(so):
        out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
        return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    d = declared("h5io.h")
    assert len(d) == 15 and d <= exported(h5io.LIB_PATH), d - exported(h5io.LIB_PATH)
    hip = exported(os.path.join(ROOT, "mceik_amd", "libmceik_hip.so"))
    b = declared("mceik_broadcast.h")
    assert b == {"broadcast_stations", "broadcast_catalog"} and b <= hip
    m = declared("mpiutils.h")
    assert len(m) == 5 and m <= hip, m - hip
