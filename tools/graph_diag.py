import sys, numpy as np, torch
sys.path.insert(0, "/root/repo") if False else None
import os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from mceik_amd.eikonal import BatchSolver
dev = torch.device("cuda", 0)
n, h, nref, nm = 40, 100.0, (4, 4, 4), 3
nc = (n // 4) ** 3
rng = np.random.default_rng(21)
src = torch.tensor(np.stack([np.zeros(4), rng.uniform(200, 3700, 4), rng.uniform(200, 3700, 4), np.full(4, 3900.0)], 1)[:, None, :]).to(dev)
ev = torch.tensor(rng.integers(0, n ** 3, 12).astype(np.int32)).to(dev)
bs = BatchSolver(n, n, n, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=nref, fast_sqrt=True)
models = [torch.tensor((1.0 / rng.integers(2500, 6500, (nm, nc))).astype(np.float32), device=dev) for _ in range(3)]
eager = []
for m in models:
    o = bs.solve(src, m, ev_node=ev); torch.cuda.synchronize(); eager.append(o["ttab"].clone())
print("eager deterministic:", torch.equal(bs.solve(src, models[0], ev_node=ev)["ttab"], eager[0]))
slow = models[0].clone()
o2 = bs.solve(src, slow, ev_node=ev); torch.cuda.synchronize()
print("eager on clone:", torch.equal(o2["ttab"], eager[0]))
g = torch.cuda.CUDAGraph(); s = torch.cuda.Stream()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        out = bs.solve(src, slow, ev_node=ev, stream=s.cuda_stream)
torch.cuda.synchronize()
for k, m in enumerate(models):
    slow.copy_(m); g.replay(); torch.cuda.synchronize()
    print(k, [torch.equal(out["ttab"], e) for e in eager], float((out["ttab"] - eager[k]).abs().max()), out["niter"][:6].tolist())
