#!/usr/bin/env python3
"""Headline benchmark: MCMC proposals/s (FSM eikonal + likelihood), BASELINE.json.

One step = one proposal for every chain on every GPU: propose (one inversion
cell per chain) -> batched FSM solves (chains x stations, HIP, fp32) ->
travel times at the events -> L2 misfit with analytic origin time ->
Metropolis (the sampler runs its chains as two halves on two streams, the
library default; --pipes 1 for one launch per step).  N=1 runs configs[2]
("C3": 1024 chains, 128^3, 32 stations);
--gpus N keeps 1024 chains per GPU (weak scaling; N=8 is configs[3], 8192
chains) and gathers the kept posterior states to rank 0 over RCCL at the
end of the timed region (the checkpoint).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (torch.distributed.run on 127.0.0.1, one process per GPU, before
anything touches the GPU) and exits with their status; under an external
launcher WORLD_SIZE must equal --gpus.  An N > 1 run exits non-zero when the
gathered posterior differs from the ranks' own shards.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MCMC proposals/sec (FSM eikonal + likelihood), 128³ grid, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
# sweep-kernel revision per precision (bump when that kernel changes; the
# profiles/traffic.json record of that precision must match)
KERNEL_REVS = {32: "fsm-v41", 64: "fsm-v42"}


# ---------------------------------------------------------------- CPU baseline
CPU_ROUNDS = 5


def _ref_solve_worker(args):
    """Single-threaded fp64 solves by the REFERENCE's own eikonal3d_serial_driver
    (oracle/_ref/libfsm3d_ref.so, built from fsm3d.f90): job 1 (level
    structure) and one warm-up solve untimed, then `rounds` job-2 solves, each
    timed alone.  Returns the per-solve seconds."""
    so, n, h, src, slow_path, rounds = args
    os.environ["OMP_NUM_THREADS"] = "1"
    lib = C.CDLL(so)
    slow = np.load(slow_path)
    u = np.zeros(n ** 3)
    i = lambda v: C.byref(C.c_int(v))
    d = lambda v: C.byref(C.c_double(v))
    ts, xs, ys, zs = (np.array([v]) for v in src)
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    ierr = C.c_int(0)
    args_ = lambda job: (i(job), i(0), i(50), i(1), i(n), i(n), i(n), d(1e-8), d(h), d(0.0), d(0.0), d(0.0),
                         P(ts), P(xs), P(ys), P(zs), P(slow), P(u), C.byref(ierr))
    lib.eikonal3d_serial_driver(*args_(1))
    lib.eikonal3d_serial_driver(*args_(2))              # warm-up
    times = []
    for _ in range(rounds):
        t = time.perf_counter()
        lib.eikonal3d_serial_driver(*args_(2))
        times.append(time.perf_counter() - t)
        if ierr.value != 0:
            raise RuntimeError(f"reference solve failed, ierr = {ierr.value}")
    lib.eikonal3d_serial_driver(*args_(3))
    return times


def cpu_cores():
    """Host cores for the CPU baseline: the CPUs this process may run on,
    capped by OMP_NUM_THREADS -- the GPU box allots 16 CPUs per GPU while
    nproc reports the whole machine."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", 0) or 0)
    return min(avail, cap) if cap > 0 else avail


def cpu_baseline(p, v0, cores, rounds=CPU_ROUNDS):
    """Reference proposals/s on this host (SURVEY s.8d protocol): `cores`
    single-threaded fp64 solves run concurrently, one per core (the reference's
    table-parallel design, mpiutils.f90:147-149); per core one warm-up solve,
    then `rounds` timed job-2 solves.  proposals/s = cores / median solve time
    / stations.  Runs before the GPU is initialised."""
    import multiprocessing as mp
    import tempfile
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    cell = ((k // p.nrz) * p.ncy + j // p.nry) * p.ncx + i // p.nrx
    slow = np.ascontiguousarray((1.0 / v0[cell.ravel()].astype(np.float64)))
    srcs = [(0.0, p.sx[s % p.nstat], p.sy[s % p.nstat], p.sz[s % p.nstat]) for s in range(cores)]
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libfsm3d_ref.so")
    nproc = os.cpu_count()
    if os.path.exists(ref_so):
        with tempfile.TemporaryDirectory() as td:
            sp = os.path.join(td, "slow.npy")
            np.save(sp, slow)
            ctx = mp.get_context("spawn")
            with ctx.Pool(cores) as pool:
                res = pool.map(_ref_solve_worker, [(ref_so, p.nx, p.h, s, sp, rounds) for s in srcs])
        kind = "reference"
        times = np.array(res).ravel()
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        L = O.lib()
        xs = np.array([s[1] for s in srcs]); ys = np.array([s[2] for s in srcs]); zs = np.array([s[3] for s in srcs])
        out = np.zeros(cores)
        idx = np.zeros(cores, np.int32)
        times = []
        for r in range(rounds + 1):
            t = time.perf_counter()
            L.oracle_batch_solve_f64(cores, 50, p.nx, p.ny, p.nz, 1e-8, p.h, 0.0, 0.0, 0.0, O._p(xs), O._p(ys),
                                     O._p(zs), O._p(slow), O._p(idx), O._p(out), 0, cores)
            if r:
                times.append(time.perf_counter() - t)     # wall of `cores` concurrent solves
        kind = "port"
        times = np.array(times)
    med = float(np.median(times))
    return {"value": round(cores / med / p.nstat, 5), "unit": "proposals/s", "cores": cores, "kind": kind,
            "sample": f"{p.nx}^3 fp64 solves of chain 0's model, stations 0..{cores - 1}: {cores} concurrent "
                      f"single-threaded solves (host nproc {nproc}, {cores} CPUs allotted), 1 warm-up + "
                      f"{rounds} timed job-2 solves per core; median solve {med:.3f} s, mean "
                      f"{float(np.mean(times)):.3f} s, min {float(np.min(times)):.3f} s, max "
                      f"{float(np.max(times)):.3f} s; proposals/s = cores / median / {p.nstat} stations"}


def kfd_devices(nodes):
    """(physical GPUs, GPU agents) of KFD topology nodes given as property
    dicts: agents are the nodes with SIMDs; a partitioned MI3xx (CPX / DPX
    modes) shows each compute partition as its own agent on the same PCI
    function, so devices are the distinct (domain, location_id) of the agents."""
    agents = [p for p in nodes if int(p.get("simd_count", 0)) > 0]
    devs = {(p.get("domain", "0"), p.get("location_id", str(i))) for i, p in enumerate(agents)}
    return len(devs), len(agents)


def node_gpus():
    """(GPUs of this host, source) from sysfs only (no GPU call): the physical
    devices of the KFD topology's GPU agents (partitions of one device counted
    once, `kfd_devices`), else the PCI functions of AMD (0x1002) processing
    accelerators / display controllers (every GPU of the node, whether or not
    this process may use it); (None, None) when neither is readable."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = []
        for d in os.listdir(base):
            with open(os.path.join(base, d, "properties")) as f:
                nodes.append(dict(line.split(None, 1) for line in f if len(line.split()) == 2))
        n, agents = kfd_devices([{k: v.strip() for k, v in p.items()} for p in nodes])
        if n:
            return n, "kfd topology" + (f" ({agents} partitions)" if agents != n else "")
    except (OSError, ValueError):
        pass
    try:
        n = 0
        pci = "/sys/bus/pci/devices"
        for d in os.listdir(pci):
            with open(os.path.join(pci, d, "vendor")) as f:
                vendor = f.read().strip()
            with open(os.path.join(pci, d, "class")) as f:
                cls = int(f.read().strip(), 16) >> 16
            if vendor == "0x1002" and cls in (0x12, 0x03):     # processing accelerator / display controller
                n += 1
        if n:
            return n, "pci (vendor 0x1002, class 0x12/0x03)"
    except (OSError, ValueError):
        pass
    return None, None


def core_share(cpu):
    """The baseline against one GPU's share of the node's cores (host CPUs /
    GPUs on the node), next to the allotted `cores` the leg actually used;
    the share's rate assumes the reference's table-parallel solves scale
    linearly with cores (they are independent single-threaded solves)."""
    host, (ngpu, src) = os.cpu_count() or 1, node_gpus()
    cpu["host_cpus"] = host
    cpu["gpus_on_node"] = ngpu
    cpu["gpus_on_node_source"] = src
    if ngpu:
        share = host // ngpu
        cpu["per_gpu_share_cores"] = share
        cpu["per_gpu_share_value"] = round(cpu["value"] * share / cpu["cores"], 5)
    else:
        cpu["per_gpu_share_cores"] = None        # no KFD topology (no GPU driver on this host)
        cpu["per_gpu_share_value"] = None
    return cpu


# ---------------------------------------------------------------- ranks
def launch_ranks(n):
    """Start the N ranks of `--gpus N` (one process per GPU) under
    torch.distributed.run on 127.0.0.1 with this command line, and return
    their exit status.  Runs before this process touches the GPU; the ranks
    find WORLD_SIZE set and run main() themselves."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


LIB_GATHER = "mceik_mcmc_gather (RCCL)"


def gather_path_name(library_comm, rehearse):
    """The checkpoint gather an N > 1 run times: the library's RCCL gather, or
    -- when some rank could not build the library communicator (agreed by all
    ranks) or on the one-GPU rehearsal -- torch.distributed's gather."""
    if library_comm:
        return LIB_GATHER
    return "torch.distributed gather (gloo; one-GPU rehearsal)" if rehearse else "torch.distributed gather (RCCL)"


def rank_fields(world, steps, per_rank, gather_path=None, gather_check=None, digest_check=None, comm_error=None):
    """The line's per-rank attribution: `rank_step_ms` {min, max, ranks} (each
    rank's own time per step up to its synchronise), `gather_ms` (the slowest
    rank's checkpoint gather) and, for N > 1, `ranks` and `gather` {path, ms,
    equals_torch_gather, shards_match_ranks, library_comm}.  per_rank: [[steps
    s, gather s]] of every rank.  library_comm: "ok", or why the run fell back
    to torch.distributed's gather."""
    st = [r[0] / steps * 1e3 for r in per_rank]
    out = {"rank_step_ms": {"min": round(min(st), 2), "max": round(max(st), 2), "ranks": len(st)},
           "gather_ms": round(max(r[1] for r in per_rank) * 1e3, 3)}
    if world > 1:
        out["ranks"] = world
        # equals_torch_gather: the library's RCCL gather against torch.distributed's
        # (None: no library communicator on this run, torch's gather was the timed path);
        # shards_match_ranks: each rank's block of the gathered posterior = its own kept states
        out["gather"] = {"path": gather_path, "ms": out["gather_ms"], "equals_torch_gather": gather_check,
                         "shards_match_ranks": digest_check,
                         "library_comm": ("ok" if gather_path == LIB_GATHER else
                                          comm_error or "not built: one-GPU rehearsal (RCCL takes one rank per GPU)")}
    return out


def shard_digest(v, logl):
    """sha256 of a block of kept states (int32 models, fp64 logL), as bytes."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(v, dtype=np.int32).tobytes())
    h.update(np.ascontiguousarray(logl, dtype=np.float64).tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------- roofline
def roofline(p, per_gpu, precision, stats, elapsed, nsteps, config, kname=None, multi_step=False):
    """The `roofline` object of a timed region: algorithmic bytes of the FSM
    launches (visited bricks x nodes x bytes per node sweep)
    over the FSM time of a step -- the HIP-event launch duration with one
    pipe, the wall time per step with overlapped pipes or with multi-step
    launches (several steps per launch, mceik_mcmc_get_info.multi_step)."""
    fsm_ms, nlaunch, iters, (bricks, segs, segs_changed, wsteps) = stats
    n_nodes = p.nx * p.ny * p.nz
    from mceik_amd import _lib
    b = _lib.FsmBatch(); b.precision = precision; b.slow_mode = 1; b.nstat = p.nstat
    b.nrx, b.nry, b.nrz = p.nref
    bpn = _lib.lib().mceik_fsm_bytes_per_node_sweep(C.byref(b))
    # the instance the sampler launches (same batch geometry as mceik_mcmc_init)
    b.nx, b.ny, b.nz, b.h = p.nx, p.ny, p.nz, p.h
    b.nmodel, b.nsrc, b.fast_sqrt, b.maxit, b.tol = per_gpu, 1, 1, p.maxit, p.tol
    b.nev = p.nevents
    if kname is None:
        kname = _lib.lib().mceik_fsm_kernel_name(C.byref(b)).decode()
    # algorithmic bytes: every node of every VISITED 8x8x8 brick (z-blocks whose
    # inputs did not change since their last visit are skipped)
    nbricks = -(-p.nx // 8) * -(-p.ny // 8) * -(-p.nz // 8)
    alg_bytes = bricks * (n_nodes / nbricks) * bpn    # this rank's launches
    full_bytes = iters * 8.0 * n_nodes * bpn          # the same iterations without skipping
    avg_ms = fsm_ms / max(nlaunch, 1)
    steps = max(nsteps, 1)
    solves_per_step = per_gpu * p.nstat                 # this rank's (chain, station) solves
    alg_step = alg_bytes / steps                        # algorithmic bytes of one step (all pipes)
    achieved = per_launch = alg_bytes / max(nlaunch, 1) / (avg_ms * 1e-3) / 1e9
    pipes = 1 if multi_step else round(nlaunch / steps)  # 1 if the sampler fell back to one pipe
    wall = pipes > 1 or multi_step
    if wall:
        # two half launches per step, overlapped: a half's HIP-event span also
        # covers the time it waits for the other half's waves, so price one
        # step's algorithmic bytes on the step's wall time instead (includes
        # propose/accept and the gather: conservative)
        achieved = alg_bytes / elapsed / 1e9                  # this rank's bytes, the timed region
    # the FSM time of one step: the single launch (HIP events) or, with pipes,
    # the wall time per step (the overlapped half launches' union is shorter)
    step_fsm_s = elapsed / steps if wall else avg_ms * 1e-3
    traffic = traffic_src = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tj = json.load(f)
        rec = tj.get("f64", {}) if precision == 64 else tj
        if (rec.get("workload") == config and rec.get("chains_per_gpu") == per_gpu
                and rec.get("kernel_rev") == KERNEL_REVS[precision]):
            traffic = rec.get("hbm_bytes_per_launch")     # one single-pipe launch = one step
            traffic_src = (f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes of kernel_rev {KERNEL_REVS[precision]} "
                           f"({rec.get('source', 'profiles/traffic.json')}); not measured in this run")
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": kname,
            "kernel_rev": KERNEL_REVS[precision],
            "timing": ("wall time per step (multi-step launches: several steps per launch)" if multi_step else
                       f"wall time per step ({pipes} overlapped partial launches, MCEIK_PIPES={pipes})"
                       if pipes > 1 else "HIP events around each FSM launch"),
            "per": "step: every per-unit field below is per step or per solve, whatever the pipes",
            "pipes": pipes,
            "alg_bytes_per_step": alg_step,
            "traffic_per_step": traffic, "traffic_source": traffic_src,
            "traffic_over_alg": round(traffic / alg_step, 4) if traffic else None,
            "bytes_per_node_sweep": bpn,
            "fsm_s_per_step": round(step_fsm_s, 4),
            "launches_per_step": round(nlaunch / steps, 3), "avg_launch_ms": round(avg_ms, 3),
            "frac_per_launch_events": round(per_launch / HBM_PEAK_GBS, 4),
            "solves_per_step": solves_per_step,
            "iterations_per_solve": round(iters / steps / solves_per_step, 3),
            "brick_visit_fraction": round(bricks / max(1.0, iters * 8.0 * nbricks), 4),
            "changed_segment_fraction": round(segs_changed / max(1.0, segs), 4),
            "wave_steps_per_step": wsteps / steps,
            "full_sweep_equiv_GBs": round(full_bytes / steps / step_fsm_s / 1e9, 1)}


def f64_record(p, v0, per_gpu, args, dev, stream):
    """The reference's own precision on the same workload, after the f32 timed
    region: a --precision 64 sampler (the literal fp64 update, fsm3d.f90:624-693)
    of the same chains, `f64_warmup` untimed + `f64_steps` timed steps bracketed
    like the headline's, with its own roofline.  One GPU only."""
    import torch
    from mceik_amd import mcmc
    torch.cuda.empty_cache()
    smp = mcmc.Sampler(p, nchains=per_gpu, chain_offset=0, v0=v0, max_samples=1, device=dev.index, precision=64)
    smp.set_stream(stream.cuda_stream)
    if args.f64_warmup:
        smp.run(args.f64_warmup)
    smp.fsm_stats(reset=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    smp.run(args.f64_steps)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    stats = smp.fsm_stats()
    info = smp.info()
    smp.close()
    rl = roofline(p, per_gpu, 64, stats, elapsed, args.f64_steps, args.config, kname=info["kernel"],
                  multi_step=info["multi_step"])
    rl["lds_bytes_per_wave"] = info["lds_bytes"]
    return {"value": round(per_gpu * args.f64_steps / elapsed, 3), "unit": "proposals/s", "dtype": "f64",
            "steps": args.f64_steps, "warmup": args.f64_warmup,
            "ms_per_step": round(elapsed / args.f64_steps * 1e3, 2), "roofline": rl}



# ---------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--chains", type=int, default=0, help="chains per GPU (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cores", type=int, default=0)
    ap.add_argument("--cpu-rounds", type=int, default=CPU_ROUNDS)
    ap.add_argument("--sigma", type=float, default=5e-4, help="pick noise (s); varObs = sigma^2")
    ap.add_argument("--raw-stats", action="store_true", help="add the raw FSM visit counters to the line")
    ap.add_argument("--precision", type=int, default=32, choices=(32, 64),
                    help="FSM arithmetic (64: the reference's literal fp64 update; tables fp32 either way)")
    ap.add_argument("--max-waves", type=int, default=0,
                    help="cap on the resident FSM waves per launch (0 = occupancy x CUs; experiments)")
    ap.add_argument("--f64-steps", type=int, default=2,
                    help="timed steps of the appended fp64 record (one GPU, --precision 32 runs; 0 = none)")
    ap.add_argument("--f64-warmup", type=int, default=1)
    ap.add_argument("--pipes", type=int, default=2, choices=(1, 2, 3, 4),
                    help="the sampler's chains as two halves on two streams (the library default, DESIGN.md "
                         "s.3.5) or one launch per step (1)")
    ap.add_argument("--probe-ranks", action="store_true",
                    help="each rank prints its rank and world size and exits before any GPU call "
                         "(tests the --gpus launcher on a CPU host)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no external launcher: start the N ranks here, before any GPU call
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: the launcher's rank count must equal --gpus",
              file=sys.stderr)
        sys.exit(2)
    os.environ["MCEIK_PIPES"] = str(args.pipes)

    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if args.probe_ranks:
        print(json.dumps({"probe": "rank", "rank": rank, "world": world, "local_rank": local_rank,
                          "gpus": args.gpus}), flush=True)
        return 0
    # MCEIK_BENCH_REHEARSAL=1: rehearse the N > 1 flow on ONE GPU (every rank on
    # device 0, torch.distributed over gloo, host-side gather; RCCL takes one
    # rank per GPU, so the library communicator is skipped).  A correctness
    # drill of sharding, barriers, max-over-ranks timing and the gather; its
    # throughput is not a scaling number.
    rehearse = os.environ.get("MCEIK_BENCH_REHEARSAL") == "1"
    if rehearse:
        local_rank = 0
    from mceik_amd import mcmc

    cfg = mcmc.CONFIGS[args.config]
    # C4 / C5 are quoted for 8 GPUs: their chain counts are totals
    per_gpu = args.chains or (cfg["nchains"] // 8 if args.config in ("C4", "C5") else cfg["nchains"])
    # problem geometry and start models are pure numpy: the CPU baseline runs
    # before anything touches the GPU (its workers are spawned processes)
    p = mcmc.make_problem(args.config, picks="analytic")
    lo, hi = mcmc.shard(per_gpu * world, rank, world)
    v0 = mcmc.initial_models(p, range(lo, hi))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = core_share(cpu_baseline(p, v0[0], args.cpu_cores or cpu_cores(), args.cpu_rounds))

    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    red_dev = torch.device("cpu") if rehearse else dev      # where the small reductions live
    # picks from the GPU forward of the true model (replaces the analytic ones)
    # (+ pick noise sigma, varObs = sigma^2: the scale one proposal moves a travel time)
    mcmc.bench_picks(p, args.sigma, local_rank)
    torch.cuda.empty_cache()             # the forward's workspace: the sampler sizes its waves to HBM
    p.nburn, p.keepk = args.warmup, max(1, args.steps)
    smp = mcmc.Sampler(p, nchains=hi - lo, chain_offset=lo, v0=v0, max_samples=1, device=local_rank,
                       precision=args.precision, max_waves=args.max_waves)
    stream = torch.cuda.current_stream(dev)
    smp.set_stream(stream.cuda_stream)

    comm = post = None
    gather_path = comm_error = None
    if world > 1:
        # the library's checkpoint gather (mceik_mcmc_gather, RCCL over xGMI);
        # the id travels over the torch.distributed group, as MPI_Bcast would carry it.
        # Decided behaviour when the library cannot build its communicator on
        # this node: every rank agrees on it BEFORE the collective init
        # (Comm.from_torch), all ranks gather with torch.distributed instead
        # (same bytes, RCCL underneath), and the line names the path used and
        # why (gather.path, gather.library_comm); the run still exits 0.
        ok = 0 if rehearse else 1
        if not rehearse:
            try:
                comm = mcmc.Comm.from_torch(local_rank)
            except Exception as exc:          # noqa: BLE001 - reported in the line, not hidden
                print(f"bench: mceik_comm unavailable ({exc}); gathering with torch.distributed", file=sys.stderr)
                comm_error = str(exc)
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=red_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()) and comm is not None:
            comm.close()
            comm = None
            comm_error = comm_error or "another rank could not build the communicator"
        gather_path = gather_path_name(comm is not None, rehearse)
        if rank == 0:
            post = torch.empty((per_gpu * world, p.ncell), dtype=torch.int32, device=dev)
            post_l = torch.empty(per_gpu * world, dtype=torch.float64, device=dev)
    else:
        post = torch.empty((hi - lo, p.ncell), dtype=torch.int32, device=dev)
    if args.warmup:
        smp.run(args.warmup)
    smp.fsm_stats(reset=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    smp.run(args.steps)
    # this rank's steps end here (the gather waits for them anyway): the split
    # attributes an N > 1 efficiency loss to the step spread or the gather
    torch.cuda.synchronize(dev)
    t_steps = time.perf_counter()
    # checkpoint: the kept posterior states of every chain -> rank 0 (RCCL over xGMI)
    if world > 1 and comm is not None:
        comm.gather(smp, per_gpu * world, which=1, root=0, v_out=post, logl_out=post_l if rank == 0 else None)
    elif world > 1:
        gv, gl = mcmc.gather_kept(smp, per_gpu * world, device=None if rehearse else dev)
        if rank == 0:
            post.copy_(gv)
            post_l.copy_(gl)
    else:
        smp.samples(max_states=1, device_ptr=post.data_ptr())
    torch.cuda.synchronize(dev)
    t_gather = time.perf_counter()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    per_rank = [[t_steps - t0, t_gather - t_steps]]            # [steps s, gather s] of each rank
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mine = torch.tensor(per_rank[0], dtype=torch.float64, device=red_dev)
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        per_rank = [e.tolist() for e in every]
    gather_check = digest_check = None
    if world > 1:
        # outside the timed region, two checks of the gathered posterior:
        # (1) with the library's RCCL gather, it equals torch.distributed's gather;
        # (2) whatever the path, each rank's block of it equals the rank's own
        #     kept states (sha256 of the shard, exchanged as objects)
        if comm is not None:
            tv, tl = mcmc.gather_kept(smp, per_gpu * world, device=None if rehearse else dev)
            if rank == 0:
                gather_check = bool(torch.equal(tv.to(dev), post) and torch.equal(tl.to(dev), post_l))
            comm.close()
        kv, kl = smp.samples(max_states=1)
        digests = [None] * world
        dist.all_gather_object(digests, (lo, hi, shard_digest(kv[0], kl[0])))
        if rank == 0:
            pv, pl = post.cpu().numpy(), post_l.cpu().numpy()
            digest_check = all(shard_digest(pv[a:b], pl[a:b]) == d for a, b, d in digests)
    stats = smp.fsm_stats()
    info = smp.info()
    _, logl, nacc, _ = smp.state()
    smp.close()
    f64 = None
    if world == 1 and args.precision == 32 and args.f64_steps > 0:
        f64 = f64_record(p, v0, per_gpu, args, dev, stream)

    if rank == 0:
        total = per_gpu * world * args.steps
        rl = roofline(p, per_gpu, args.precision, stats, elapsed, args.steps, args.config, kname=info["kernel"],
                      multi_step=info["multi_step"])
        rl["lds_bytes_per_wave"] = info["lds_bytes"]
        line = {
            "metric": METRIC,
            "value": round(total / elapsed, 3),
            "unit": "proposals/s",
            "n_gpus": 1 if rehearse else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == 32 else "f64",
            "data": f"synthetic (SURVEY s.8d heterogeneous model, picks = GPU forward of the true model + "
                    f"N(0, {args.sigma} s), varObs = {args.sigma}^2)",
            "config": {"workload": f"{args.config}: {per_gpu} chains/GPU, {p.nx}^3 grid, {p.nstat} stations, "
                                   f"{p.nevents} events, nref=4",
                       "chains_per_gpu": per_gpu, "chains_total": per_gpu * world, "grid": [p.nx, p.ny, p.nz],
                       "stations": p.nstat, "events": p.nevents, "parallelism": f"chains sharded over {world} GPU(s)",
                       "pipes": rl["pipes"]},
            "roofline": rl,
            "cpu_baseline": cpu,
            "accept_rate": round(float(nacc.sum()) / max(1, (hi - lo) * (args.warmup + args.steps)), 4),
        }
        if rehearse:
            line["rehearsal"] = "one GPU shared by all ranks (MCEIK_BENCH_REHEARSAL=1): not a scaling measurement"
        line.update(rank_fields(world, args.steps, per_rank, gather_path, gather_check, digest_check, comm_error))
        if cpu:
            line["speedup_vs_cpu_per_gpu_share"] = (round(line["value"] / cpu["per_gpu_share_value"], 1)
                                                    if cpu.get("per_gpu_share_value") else None)
        if args.raw_stats:
            ms, nl, it, (br, sg, sgc, ws) = stats
            line["fsm_raw"] = {"bricks": br, "segs": sg, "segs_changed": sgc, "iters": it, "wave_steps": ws,
                               "launches": nl}
        if f64 is not None:
            line["f64"] = f64
        if cpu:
            line["speedup_vs_cpu"] = round(line["value"] / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    bad = rank == 0 and (gather_check is False or digest_check is False)
    if world > 1:
        dist.destroy_process_group()
    if bad:
        print("bench: the gathered posterior differs from the ranks' own shards", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
