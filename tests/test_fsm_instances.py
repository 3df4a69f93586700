"""Which sweep-kernel instance a batch launches and how much LDS a wave takes
(host-side: mceik_fsm_kernel_name / mceik_fsm_lds_bytes, no GPU).

The sampler's instances at the bench's C3 geometry, and the fp64 compact LDS
layout (fsm_common.h fsm_compact_layout: 16-bit block clocks, meta-only
column words) that gives the fp64 instance 8 waves per CU: 160 KiB of LDS
per CU / 8 = 20480 B per wave at most.  Geometries outside the compact
layout's bounds fall back to the runtime-kb instance."""
import ctypes as C

import pytest

pytest.importorskip("torch")

LDS_PER_CU = 160 * 1024


def _batch(n, precision, fast=True, nstat=32, nmodel=1024, nref=(4, 4, 4), nxy=None):
    from mceik_amd.eikonal import BatchSolver
    nx = ny = nxy or n
    bs = BatchSolver(nx, ny, n, 100.0, 0.0, 0.0, 0.0, 50, 1e-8, precision, nref=nref, fast_sqrt=fast)
    return bs.describe(nmodel, nstat, 1, 1, nev=32)


def _info(b):
    from mceik_amd import _lib
    L = _lib.lib()
    return L.mceik_fsm_kernel_name(C.byref(b)).decode(), int(L.mceik_fsm_lds_bytes(C.byref(b)))


def test_c3_fp32_sampler_instance():
    name, lds = _info(_batch(128, 32))
    assert name == "fsm16_solve_kernel<2, 1>"
    assert lds <= LDS_PER_CU // 8, lds                  # 8 waves/CU (the VGPR limit)


def test_c3_fp64_sampler_instance_compact_layout():
    """bench.py's f64 record: the short-sqrt fp64 instance, compact LDS."""
    name, lds = _info(_batch(128, 64))
    assert name == "fsm_solve_kernel<double, 2, true, 2, 1, 4>"
    assert lds <= LDS_PER_CU // 8, lds                  # 8 waves/CU; the int layout took 25456 B (6)
    exact, _ = _info(_batch(128, 64, fast=False))
    assert exact == "fsm_solve_kernel<double, 2, false, 2, 1, 4>"


@pytest.mark.parametrize("nz,nxy", [(20, None), (32, 264)], ids=["kb3", "over_1024_blocks"])
def test_fp64_runtime_kb_fallback(nz, nxy):
    """kb != MCEIK_KB (nz = 20: 3 bricks) or more than MCEIK_MAX_BLOCKS z-blocks
    (264 x 264 x 32: 33 x 33 tiles x 1 block): the runtime-kb instance with
    int clocks (the compact layout's 16-bit clocks are bounded for <= 1024)."""
    name, _ = _info(_batch(nz, 64, nxy=nxy, nstat=2, nmodel=1))
    assert name == "fsm_solve_kernel<double, 2, false, 2, 1, 0>"
