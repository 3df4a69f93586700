"""Two processes drive real Samplers (libmceik_hip.so) on the one GPU, each
with its shard of global chain ids, and gather the kept states to rank 0
through mcmc.gather_kept -- the code path bench.py runs over RCCL for N > 1,
here over gloo on host copies.  The gathered posterior must equal one
process running all chains."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

NCHAINS, NSTEPS, WORLD = 5, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem():
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", n=20, nstat=3, nev=4, seed=23, picks="analytic")
    p.dvmax, p.nburn, p.keepk = 300, 1, 1
    p.var[:] = 1e-4
    return p


def _worker(rank, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    from mceik_amd import mcmc
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    try:
        p = _problem()
        lo, hi = mcmc.shard(NCHAINS, rank, WORLD)
        smp = mcmc.Sampler(p, nchains=hi - lo, chain_offset=lo, max_samples=2)
        smp.run(NSTEPS)
        v, lg = mcmc.gather_kept(smp, NCHAINS)
        smp.close()
        if rank == 0:
            q.put((v.numpy(), lg.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_samplers_gather_equals_single_process():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for pr in procs:
        pr.start()
    got_v, got_l = q.get(timeout=100)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    from mceik_amd import mcmc
    s = mcmc.Sampler(_problem(), nchains=NCHAINS, max_samples=2)
    s.run(NSTEPS)
    v, lg = s.samples(max_states=1)
    s.close()
    assert got_v.shape == (NCHAINS, v.shape[2])
    assert np.array_equal(got_v, v[0]) and np.array_equal(got_l.view(np.uint64), lg[0].view(np.uint64))
