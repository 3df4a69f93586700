"""h5io posterior files (SURVEY s.8f row 1): the reference's names, layout and
quirks (h5io.c), checked by round trips through libmceik_h5io.so.  CPU only;
the GPU posterior writer test is in test_gpu_mcmc.py."""
import os
import re
import subprocess

import numpy as np
import pytest

from mceik_amd import h5io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_match_header():
    txt = open(os.path.join(ROOT, "include", "mceik_h5io.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    declared = {m.group(1) for m in re.finditer(r"^\s*(?:int|void)\s+([A-Za-z_]\w*)\s*\(", txt, flags=re.M)}
    assert declared == set(h5io.EXPORTS), declared ^ set(h5io.EXPORTS)
    h5io.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", h5io.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared <= exported


def test_file_and_dataset_names():
    """h5io.c:9-58, 164-190."""
    assert h5io.file_name(1, "/tmp/x", "proj") == "/tmp/x/proj_ttimes.h5"
    assert h5io.file_name(2, "/tmp/x/", "proj") == "/tmp/x/proj_locations.h5"
    assert h5io.file_name(1, None, "p") == "./p_ttimes.h5"
    assert h5io.file_name(1, "", "p") == "./p_ttimes.h5"
    with pytest.raises(RuntimeError):
        h5io.file_name(1, "/tmp", "")
    assert h5io.travel_time_name(3, 7, True) == "/TravelTimeTables/Model_3/Station_7/PTravelTimes"
    assert h5io.travel_time_name(1, 2, False) == "/TravelTimeTables/Model_1/Station_2/STravelTimes"
    assert h5io.location_name(4, 9) == "/logJPDFs/Event_9/Model_4/logJPDF"


def test_ttables_round_trip_and_layout(tmp_path):
    nx, ny, nz = 5, 4, 3
    x0, y0, z0, dx, dy, dz = 100.0, -50.0, 10.0, 25.0, 20.0, 15.0
    f = h5io.init_ttables(str(tmp_path), "t", nx, ny, nz, 2, 3, x0, y0, z0, dx, dy, dz)
    try:
        assert f.dims() == (nx, ny, nz)                    # the {nx,ny,nz} dataspace quirk
        for m in (1, 2):
            for s in (1, 2, 3):
                assert f.exists(f"/TravelTimeTables/Model_{m}/Station_{s}")
                assert f.exists(h5io.travel_time_name(m, s, True))
                assert f.exists(h5io.travel_time_name(m, s, False))
        assert not f.exists("/TravelTimeTables/Model_3")
        x, y, z = f.model()
        k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
        assert np.array_equal(x, (x0 + i * dx).astype(np.float32).ravel())   # x fastest in memory
        assert np.array_equal(y, (y0 + j * dy).astype(np.float32).ravel())
        assert np.array_equal(z, (z0 + k * dz).astype(np.float32).ravel())
        tt = np.random.default_rng(1).random(nx * ny * nz).astype(np.float32)
        f.write_ttimes(2, 1, tt)
        assert np.array_equal(f.read_ttimes(2, 1), tt)
        assert np.all(f.read_ttimes(3, 2) == 0)            # never written: the reference's null table
        assert np.all(f.read_ttimes(2, 1, iphase=2) == 0)
    finally:
        f.close()
    g = h5io.H5File.open(os.path.join(str(tmp_path), "t_ttimes.h5"))
    try:
        assert np.array_equal(g.read_ttimes(2, 1), tt)
        with pytest.raises(RuntimeError):
            g.read_ttimes(9, 1)                            # missing dataset
    finally:
        g.close()


def test_locations_round_trip(tmp_path):
    nx, ny, nz = 6, 5, 4
    f = h5io.init_locations(str(tmp_path), "loc", nx, ny, nz, 3, 2, 0.0, 0.0, 0.0, 1.0, 1.0, 1.0)
    try:
        assert f.exists("/Model/priorLocationModel")
        for e in (1, 2):
            for m in (1, 2, 3):
                assert f.exists(h5io.location_name(m, e))
        v = -np.arange(nx * ny * nz, dtype=np.float32)
        f.write_logjpdf(3, 2, v)
        assert np.array_equal(f.read_logjpdf(3, 2), v)
        assert np.all(f.read_logjpdf(1, 1) == 0)
    finally:
        f.close()
