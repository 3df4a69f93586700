"""Probe (GPU box): can two processes on ONE GPU form an RCCL communicator
and run mceik_mcmc_gather?  RCCL normally wants one rank per device; this
records what this image's RCCL does.  Prints one line per rank."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from mceik_amd import mcmc
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    p = mcmc.make_problem("C2", n=20, nstat=3, nev=4, seed=23, picks="analytic")
    p.nburn, p.keepk = 1, 1
    lo, hi = mcmc.shard(5, rank, world)
    smp = mcmc.Sampler(p, nchains=hi - lo, chain_offset=lo, max_samples=2)
    smp.run(3)
    comm = mcmc.Comm.from_torch(0)
    v, lg = comm.gather(smp, 5, which=1)
    tv, tl = mcmc.gather_kept(smp, 5)
    if rank == 0:
        print("probe: library gather == torch gather:", np.array_equal(v, tv.numpy()) and
              np.array_equal(lg, tl.numpy()), flush=True)
    comm.close()
    smp.close()
    dist.destroy_process_group()
    print(f"probe rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
