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


def _run_bench(args, env_extra=None, timeout=240):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` with no external launcher starts 2 ranks itself
    (torch.distributed.run on 127.0.0.1); --probe-ranks stops each rank before
    any GPU call and prints its rank and world size."""
    r = _run_bench(["--gpus", "2", "--probe-ranks"])
    assert r.returncode == 0, r.stderr[-2000:]
    probes = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"probe"')]
    assert sorted(q["rank"] for q in probes) == [0, 1], r.stdout
    assert all(q["world"] == 2 and q["gpus"] == 2 for q in probes)
    r1 = _run_bench(["--probe-ranks"])
    assert r1.returncode == 0 and [json.loads(l)["world"] for l in r1.stdout.splitlines()] == [1]


def test_world_size_must_equal_gpus():
    """Under an external launcher WORLD_SIZE must equal --gpus (the driver's
    SCALE line would otherwise mislabel its rank count)."""
    r = _run_bench(["--gpus", "4", "--probe-ranks"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr
    r = _run_bench(["--probe-ranks"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_rank_fields_of_an_n_gt_1_line():
    """Every N > 1 line carries ranks, rank_step_ms {min, max, ranks},
    gather_ms and gather {path, ms, equals_torch_gather, shards_match_ranks}."""
    import bench
    f = bench.rank_fields(2, 4, [[8.0, 0.002], [8.4, 0.003]], "mceik_mcmc_gather (RCCL)", True, True)
    assert f["ranks"] == 2
    assert f["rank_step_ms"] == {"min": 2000.0, "max": 2100.0, "ranks": 2}
    assert f["gather_ms"] == 3.0
    assert f["gather"] == {"path": "mceik_mcmc_gather (RCCL)", "ms": 3.0, "equals_torch_gather": True,
                           "shards_match_ranks": True, "library_comm": "ok"}
    one = bench.rank_fields(1, 4, [[8.0, 0.001]])
    assert "gather" not in one and one["rank_step_ms"]["ranks"] == 1


def test_shard_digest_detects_a_changed_state():
    import numpy as np
    import bench
    v = np.arange(12, dtype=np.int32).reshape(3, 4)
    lg = np.array([-1.0, -2.0, -3.0])
    d = bench.shard_digest(v, lg)
    assert bench.shard_digest(v.copy(), lg.copy()) == d
    v2 = v.copy(); v2[1, 2] += 1
    assert bench.shard_digest(v2, lg) != d
    assert bench.shard_digest(v, np.nextafter(lg, 0.0)) != d


def test_cpu_core_share_fields():
    """cpu_baseline carries the host's CPUs, the GPUs on the node and one GPU's
    share of the cores (None without a KFD topology, as on this CPU host)."""
    import bench
    c = bench.core_share({"value": 0.32, "cores": 16})
    assert c["host_cpus"] == (os.cpu_count() or 1)
    if c["gpus_on_node"]:
        share = c["host_cpus"] // c["gpus_on_node"]
        assert c["per_gpu_share_cores"] == share
        assert c["per_gpu_share_value"] == pytest.approx(0.32 * share / 16, rel=1e-4)
    else:
        assert c["per_gpu_share_cores"] is None and c["per_gpu_share_value"] is None


def test_gpus_8_launches_8_distinct_ranks():
    """C4 readiness (the driver's 8-GPU SCALE run is C4's first execution):
    `bench.py --gpus 8` starts 8 distinct ranks, LOCAL_RANK 0..7, world 8."""
    r = _run_bench(["--gpus", "8", "--probe-ranks"])
    assert r.returncode == 0, r.stderr[-2000:]
    probes = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"probe"')]
    assert sorted(q["rank"] for q in probes) == list(range(8)), r.stdout
    assert sorted(q["local_rank"] for q in probes) == list(range(8))
    assert all(q["world"] == 8 and q["gpus"] == 8 for q in probes)


@pytest.mark.parametrize("total,world", [(8192, 8), (2048, 8), (1024, 2), (1000, 8), (7, 8)])
def test_shards_tile_the_chains(total, world):
    """mcmc.shard(total, r, world) over r = 0..world-1 tiles [0, total) in
    order (C4: 8192 chains = 8 x 1024), sizes differing by at most one."""
    from mceik_amd import mcmc
    parts = [mcmc.shard(total, r, world) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == total
    assert all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
    sizes = [hi - lo for lo, hi in parts]
    assert max(sizes) - min(sizes) <= 1
    if total == 8192:
        assert parts == [(1024 * r, 1024 * (r + 1)) for r in range(8)]


def test_gather_path_is_reported():
    """Decided N > 1 behaviour without the library communicator: the run
    gathers with torch.distributed and the line names the path and why."""
    import bench
    assert bench.gather_path_name(True, False) == bench.LIB_GATHER
    assert bench.gather_path_name(False, False) == "torch.distributed gather (RCCL)"
    assert "rehearsal" in bench.gather_path_name(False, True)
    ok = bench.rank_fields(8, 2, [[4.0, 0.01]] * 8, bench.LIB_GATHER, True, True)
    assert ok["ranks"] == 8 and ok["rank_step_ms"]["ranks"] == 8 and ok["gather"]["library_comm"] == "ok"
    fb = bench.rank_fields(8, 2, [[4.0, 0.01]] * 8, bench.gather_path_name(False, False), None, True,
                           "rank 3: RCCL (librccl.so.1) cannot be loaded")
    assert fb["gather"]["path"] == "torch.distributed gather (RCCL)"
    assert fb["gather"]["library_comm"].startswith("rank 3")
    assert fb["gather"]["shards_match_ranks"] is True


def test_kfd_devices_count_partitions_once():
    """A CPX-partitioned MI3xx shows several KFD agents on one PCI function:
    the node's GPU count (for the per-GPU core share) counts the device once."""
    import bench
    cpu = {"simd_count": "0", "location_id": "0"}
    gpu = lambda loc: {"simd_count": "32", "location_id": str(loc), "domain": "0"}
    assert bench.kfd_devices([cpu] + [gpu(256 * k) for k in range(8)]) == (8, 8)
    assert bench.kfd_devices([cpu] + [gpu(256 * k) for k in range(8) for _ in range(4)]) == (8, 32)
    assert bench.kfd_devices([cpu]) == (0, 0)


def test_roofline_of_multi_step_launches():
    """A multi-step sampler (several steps per launch, e.g. 32 chains per
    rank in the 8-rank rehearsal: 0.5 launches per step) reports one pipe and
    prices a step's bytes on the wall time per step (round 6: it printed
    pipes 0 and the per-launch time as the step's)."""
    import bench
    from mceik_amd import mcmc
    p = mcmc.make_problem("C3", picks="analytic")
    stats = (2000.0, 1, 32 * 32 * 6 * 2, (1.0e8, 3.0e9, 1.0e9, 1.0e7))
    r = bench.roofline(p, 32, 32, stats, 1.5, 2, "C3", multi_step=True)
    assert r["pipes"] == 1 and r["launches_per_step"] == 0.5
    assert r["fsm_s_per_step"] == pytest.approx(0.75)
    assert r["achieved"] == pytest.approx(1.0e8 * 512 * r["bytes_per_node_sweep"] / 1.5 / 1e9, rel=1e-3)
    assert r["timing"].startswith("wall time per step (multi-step")
