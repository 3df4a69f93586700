"""World-size-2 run of the sharded sampler on CPU (gloo): each rank advances
its block of global chain ids (CPU restatement as the compute), then the kept
states are gathered to rank 0 as bench.py does over RCCL.  The gathered
posterior must equal a single-process run of all chains."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem():
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", n=12, nstat=2, nev=3, picks="analytic")
    p.dvmax = 300
    return p


def _run_chains(p, lo, hi, nsteps):
    import _oracle as O
    from mceik_amd import mcmc
    P = O.make_problem(p)
    v0 = mcmc.initial_models(p, range(lo, hi))
    logl = [O.loglik(P, O.forward_f32(P, v)[0]) for v in v0]
    v, lg, acc, _ = O.mcmc_run(P, v0, logl, lo, 0, nsteps)
    return v, lg


def _worker(rank, world, port, nchains, nsteps, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here); sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    from mceik_amd import mcmc
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    p = _problem()
    lo, hi = mcmc.shard(nchains, rank, world)
    v, lg = _run_chains(p, lo, hi, nsteps)
    vt = torch.from_numpy(np.ascontiguousarray(v))
    gathered = [torch.empty_like(vt) for _ in range(world)] if rank == 0 else None
    dist.gather(vt, gathered, dst=0)
    if rank == 0:
        q.put(torch.cat(gathered).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather():
    import torch.multiprocessing as tmp
    nchains, nsteps, world = 4, 3, 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nchains, nsteps, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ref, _ = _run_chains(_problem(), 0, nchains, nsteps)
    assert np.array_equal(got, ref)


def _comm_worker(rank, world, port, bad_rank, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here); sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    from mceik_amd import mcmc
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)

    def ready():
        return (False, "RCCL (librccl.so.1) cannot be loaded") if rank == bad_rank else (True, "")
    try:
        mcmc.Comm.from_torch(rank, ready=ready)
        q.put((rank, "built"))
    except mcmc.CommUnavailable as exc:
        q.put((rank, str(exc)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, 1), (4, 2)])
def test_comm_unavailable_on_one_rank_is_agreed_by_all(world, bad_rank):
    """bench.py's N > 1 gather decision: one rank that cannot build the
    library communicator makes EVERY rank raise CommUnavailable before the
    collective mceik_comm_init (no rank is left waiting inside it), each
    naming the rank and the reason; bench.py then gathers with
    torch.distributed and reports gather.library_comm."""
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, bad_rank, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert sorted(got) == list(range(world))
    assert all(m == f"rank {bad_rank}: RCCL (librccl.so.1) cannot be loaded" for m in got.values()), got
