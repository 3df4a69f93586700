"""bench.py's roofline object on CPU (no GPU): the algorithmic-byte accounting
and the traffic record it attaches.

`profiles/traffic.json` holds the measured HBM bytes per launch of each
precision's sampler kernel, keyed by kernel revision; the line carries them
only while the revision matches bench.KERNEL_REVS.  These tests fail when a
kernel revision is bumped without a new PMC record (so `traffic` can no
longer drop to null silently), and pin the roofline arithmetic."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pytest.importorskip("torch")


def _tj():
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
        return json.load(f)


def test_traffic_records_match_the_kernel_revisions():
    import bench
    tj = _tj()
    for prec, rec in ((32, tj), (64, tj["f64"])):
        assert rec["kernel_rev"] == bench.KERNEL_REVS[prec], prec
        assert rec["workload"] == "C3" and rec["chains_per_gpu"] == 1024
        # FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md gfx950 correction)
        assert rec["hbm_bytes_per_launch"] == pytest.approx(2 * rec["fetch_size_bytes_raw"] + rec["write_size_bytes"])
        assert 1.0 <= rec["hbm_over_alg"] < 2.0


@pytest.mark.parametrize("precision", [32, 64])
def test_roofline_accounting(precision):
    """One one-pipe launch per step: alg bytes = visited bricks x 512 nodes x
    bytes per node sweep; achieved = alg / launch time; the traffic record of
    the precision is attached."""
    import bench
    from mceik_amd import mcmc
    p = mcmc.make_problem("C3", picks="analytic")
    tj = _tj()
    rec = tj if precision == 32 else tj["f64"]
    bricks, steps, ms = 5.0e9, 2, 10000.0
    stats = (ms * steps, steps, 1024 * 32 * 6 * steps, (bricks, 3.0e11, 1.0e11, 1.0e9))
    r = bench.roofline(p, 1024, precision, stats, ms * steps / 1e3, steps, "C3")
    bpn = 2.0 * (8 if precision == 64 else 4) + 4.0 / 64 / 32       # u read + write, cell slowness / 64 nodes / 32 stations
    assert r["bytes_per_node_sweep"] == pytest.approx(bpn)
    assert r["alg_bytes_per_step"] == pytest.approx(bricks * 512 * bpn / steps)
    assert r["achieved"] == pytest.approx(bricks * 512 * bpn / steps / (ms * 1e-3) / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-3)
    assert r["pipes"] == 1 and r["avg_launch_ms"] == pytest.approx(ms)
    assert r["traffic"] == rec["hbm_bytes_per_launch"]
    assert r["kernel_rev"] == bench.KERNEL_REVS[precision]
    assert ("fsm16_solve_kernel" in r["kernel"]) == (precision == 32)
