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


def test_library_rccl_gather_single_rank():
    """mceik_comm_* / mceik_mcmc_gather (the C multi-rank path, RCCL) with one
    rank: kept and current states land in global chain order, into host arrays
    or straight into a device tensor; shards that do not tile the chain range
    and a missing kept state are refused.  (More ranks need more GPUs: RCCL
    takes one rank per device; the driver's 8-GPU bench runs that path.)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mceik_amd import mcmc
    comm = mcmc.Comm(0, 1, 0)
    s = mcmc.Sampler(_problem(), nchains=NCHAINS, max_samples=2)
    s.run(NSTEPS)
    kv, kl = s.samples(max_states=1)
    v, lg, _, _ = s.state()
    gv, gl = comm.gather(s, NCHAINS, which=1)
    assert np.array_equal(gv, kv[0]) and np.array_equal(gl.view(np.uint64), kl[0].view(np.uint64))
    cv, cl = comm.gather(s, NCHAINS, which=0)
    assert np.array_equal(cv, v) and np.array_equal(cl.view(np.uint64), lg.view(np.uint64))
    dv = torch.zeros((NCHAINS, s.p.ncell), dtype=torch.int32, device="cuda:0")
    dl = torch.zeros(NCHAINS, dtype=torch.float64, device="cuda:0")
    comm.gather(s, NCHAINS, which=1, v_out=dv, logl_out=dl)
    assert np.array_equal(dv.cpu().numpy(), kv[0]) and np.array_equal(dl.cpu().numpy(), kl[0])
    with pytest.raises(RuntimeError):
        comm.gather(s, NCHAINS + 1)                       # chain NCHAINS is on no rank
    s.close()
    s0 = mcmc.Sampler(_problem(), nchains=NCHAINS, max_samples=0)
    with pytest.raises(RuntimeError):
        comm.gather(s0, NCHAINS, which=1)                 # nothing kept
    s0.close()
    comm.close()
