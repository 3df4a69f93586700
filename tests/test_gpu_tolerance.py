"""The fp32 sampler against the reference's fp64 FSM on the sampler's own
workload (north_star: "travel-time fields match reference fsm3d to a stated
fp32 tolerance"), and what fp32 costs the chains.

The stated bound is

    |u32 - u64| <= 4e-6 * u64 + 4e-7 s     at every node,

four times the largest error observed on the sampler's workloads (SURVEY
s.8c's rule; round 4 measured max |du|/u 9.56e-7 and |du| 1.80e-6 s at C3).
u32 comes from the GPU's fp32 cell-model path (the kernel instance the
sampler launches: 16-z steps, LDS cell cache, short sqrt), u64 from the
REFERENCE's own eikonal3d_serial_driver (fsm3d.f90:28-99,648-693, built into
oracle/_ref/libfsm3d_ref.so; the fp64 oracle, bitwise equal to it on every
golden, stands in when the .so is absent) on the same model expanded to fp64
slowness 1/(double)v per inversion cell.  Checked on full fields and at the
event nodes the sampler reads:

* C3 (128^3, the bench's geometry and picks): chains 0, 511 and 1023 x all 32
  stations, on their initial models AND on their models after the bench's 25
  steps (5 warm-up + 20 timed, bench.py's sigma and dvmax; chains are keyed by
  global id, so a one-chain sampler at offset c walks chain c of the bench);
* C5 (256^3, paths twice as long): chain 0 x 8 stations spread over the array.

The logL difference between the sampler's fp32 tables and the reference
pipeline's tables (fp64 solve exported to fp32, fsm3d.f90:1855-1875) is
reported, and the fp32 and fp64 samplers are run side by side from the same
seed at C2 (256 chains, 20 steps) to count identical accept decisions.
Observed maxima print as "TOLERANCE ..." / "ACCEPT ..." lines (run with -s).
"""
import os

import numpy as np
import pytest

import _oracle as O
import _refsolve as R

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL_REL, TOL_ABS = 4e-6, 4e-7
# bench.py's --sigma default; BENCH_STEPS = the driver's round-end bench command (`bench.py --warmup 5
# --steps 20`, BENCH_r05.json: 20 timed steps of 1643.86 ms), not bench.py's own defaults (--warmup 1 --steps 10)
BENCH_SIGMA, BENCH_STEPS = 5e-4, 25
# regression threshold on the observed largest |du| / bound (C3 0.225, C5 0.258 at round 5): the
# stated bound is 4x the observed maxima; this catches a precision regression of ~2x, not only 4x
RATIO_REGRESSION = 0.5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _cores():
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", 0) or 0)
    return max(1, min(avail, cap) if cap > 0 else avail)


def _node_slowness64(p, vcell):
    """Per-node fp64 slowness 1/(double)v of a cell model (x fastest)."""
    c = (1.0 / np.asarray(vcell, dtype=np.float64)).reshape(p.ncz, p.ncy, p.ncx)
    k, j, i = np.meshgrid(np.arange(p.nz), np.arange(p.ny), np.arange(p.nx), indexing="ij")
    return np.ascontiguousarray(c[k // p.nrz, j // p.nry, i // p.nrx].ravel())


def _reference_fields(p, jobs):
    """jobs [(vcell, station)] -> ([u64 [n^3]], which solver ran)."""
    srcs = [(0.0, p.sx[s], p.sy[s], p.sz[s]) for _, s in jobs]
    slows = [_node_slowness64(p, v) for v, _ in jobs]
    if R.available():
        res = R.solve_many([(p.nx, p.h, src, sl, p.maxit, p.tol) for src, sl in zip(srcs, slows)],
                           min(len(jobs), _cores()))
        assert all(e == 0 for _, e in res)
        return [u for u, _ in res], "reference eikonal3d_serial_driver (oracle/_ref/libfsm3d_ref.so)"
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(_cores()) as ex:
        res = list(ex.map(lambda a: O.eikonal_solve(p.nx, p.ny, p.nz, a[1], p.h, [a[0]], p.maxit, p.tol),
                          zip(srcs, slows)))
    assert all(e == 0 for _, e, _ in res)
    return [u for u, _, _ in res], "fp64 oracle (bitwise = reference on the goldens)"


def _excess(u32, u64):
    """(max |du| s, max |du|/u, max of |du| - bound, max of |du| / bound)."""
    u32 = np.asarray(u32, dtype=np.float64)
    d = np.abs(u32 - u64)
    bound = TOL_REL * u64 + TOL_ABS
    return d.max(), (d / np.maximum(u64, 1e-30)).max(), (d - bound).max(), (d / bound).max()


def _gpu_fields(p, vcells, stations, dev):
    """The sampler's fp32 kernel instance on cell models: fields + event tables."""
    from mceik_amd.eikonal import BatchSolver
    bs = BatchSolver(p.nx, p.ny, p.nz, p.h, p.x0, p.y0, p.z0, p.maxit, p.tol, 32, nref=p.nref, fast_sqrt=True)
    src = torch.tensor(np.stack([np.zeros(len(stations)), p.sx[stations], p.sy[stations], p.sz[stations]], 1)[:, None, :])
    slow = torch.tensor((1.0 / np.asarray(vcells, dtype=np.float32)).astype(np.float32), device=dev)
    out = bs.solve(src, slow, ev_node=torch.tensor(p.ev_node), want_fields=True)
    torch.cuda.synchronize(dev)
    nm, ns = len(vcells), len(stations)
    u = out["u"].cpu().numpy().reshape(nm, ns, -1)
    tt = out["ttab"].cpu().numpy().reshape(nm, ns, -1)
    assert out["step_z"] == 16
    return u, tt


def _check_models(p, label, chains, models, dev, sampler_tabs=None, logls=None):
    """Full fields and event times of `models` x every station within the
    bound of the reference; with `sampler_tabs` the sampler's own tables are
    the batched fields at the event nodes bit for bit.  Prints the maxima
    first, then asserts."""
    stations = np.arange(p.nstat)
    u32, tt32 = _gpu_fields(p, models, stations, dev)
    if sampler_tabs is not None:
        for m in range(len(chains)):
            assert np.array_equal(tt32[m].view(np.uint32), sampler_tabs[m].view(np.uint32)), chains[m]
    u64, who = _reference_fields(p, [(models[m], s) for m in range(len(chains)) for s in stations])
    P = O.make_problem(p)
    ev = p.ev_node
    worst_f = worst_e = (0.0, 0.0, -1.0, 0.0)
    fails = []
    for m, c in enumerate(chains):
        tt64 = np.empty((p.nstat, p.nevents), np.float32)
        for s in stations:
            ref = u64[m * p.nstat + s]
            f = _excess(u32[m, s], ref)
            e = _excess(tt32[m, s], ref[ev])
            if f[2] > 0.0 or e[2] > 0.0:
                fails.append((c, int(s), f, e))
            worst_f = max(worst_f, f, key=lambda t: t[3])
            worst_e = max(worst_e, e, key=lambda t: t[3])
            tt64[s] = ref[ev].astype(np.float32)          # the reference's fp64 -> fp32 table export
        l32 = O.loglik(P, tt32[m])
        l64 = O.loglik(P, tt64)
        if logls is not None:
            assert logls[m] == l32, c
        print(f"TOLERANCE {label} chain {c}: logL fp32 tables {l32:.9f}, reference tables {l64:.9f}, "
              f"|dlogL| {abs(l32 - l64):.3e} ({abs(l32 - l64) / abs(l64):.3e} relative)")
    print(f"TOLERANCE {label} fields ({who}): max |du| {worst_f[0]:.3e} s, max |du|/u {worst_f[1]:.3e}, "
          f"largest |du| / bound {worst_f[3]:.3f} (bound {TOL_REL:g} u + {TOL_ABS:g}); event nodes: "
          f"max |du| {worst_e[0]:.3e} s, max |du|/u {worst_e[1]:.3e}, |du| / bound {worst_e[3]:.3f}")
    assert not fails, fails[:4]
    assert worst_f[3] <= RATIO_REGRESSION and worst_e[3] <= RATIO_REGRESSION, (worst_f, worst_e)
    return worst_f, worst_e


def _bench_problem(config):
    """bench.py's problem: geometry, start models and picks (GPU forward +
    N(0, sigma), varObs = sigma^2)."""
    from mceik_amd import mcmc
    p = mcmc.make_problem(config, picks="analytic")
    return mcmc.bench_picks(p, BENCH_SIGMA, 0)


@pytest.mark.timeout(900)
def test_c3_sampler_fields_within_fp32_tolerance_of_reference():
    """C3 (the bench's geometry and picks): chains 0, 511, 1023 x all 32
    stations on their initial models.  The sampler's own tables equal the
    batched fields at the event nodes bit for bit; every node of every field
    and every event time is within the bound of the reference's fp64 solve."""
    dev = _dev()
    from mceik_amd import mcmc
    p = _bench_problem("C3")
    chains = (0, 511, 1023)
    v0, logl0, ttab = [], [], []
    for c in chains:
        s = mcmc.Sampler(p, nchains=1, chain_offset=c)
        v, lg, _, _ = s.state()
        tt, _, _ = s.last()
        s.close()
        v0.append(v[0]); logl0.append(lg[0]); ttab.append(tt[0])
    _check_models(p, "C3 init", chains, v0, dev, sampler_tabs=ttab, logls=logl0)


@pytest.mark.timeout(900)
def test_c3_fields_after_bench_steps_within_fp32_tolerance():
    """The same chains after the bench's 25 steps (its sigma and dvmax): the
    models have moved away from their start (cell contrasts up to +-dvmax per
    accepted step) and the bound still holds at every node."""
    dev = _dev()
    from mceik_amd import mcmc
    p = _bench_problem("C3")
    chains = (0, 511, 1023)
    models, moved = [], []
    for c in chains:
        s = mcmc.Sampler(p, nchains=1, chain_offset=c)
        v0, _, _, _ = s.state()
        s.run(BENCH_STEPS)
        v, _, nacc, step = s.state()
        s.close()
        assert step == BENCH_STEPS
        models.append(v[0])
        moved.append((int((v[0] != v0[0]).sum()), int(nacc[0])))
    print(f"TOLERANCE C3 after {BENCH_STEPS} steps: (cells changed, accepts) per chain {moved}")
    assert all(m[0] > 0 for m in moved)
    _check_models(p, f"C3 step {BENCH_STEPS}", chains, models, dev)


@pytest.mark.timeout(1200)
def test_c5_fields_within_fp32_tolerance_of_reference():
    """C5 (256^3, paths twice C3's): chain 0's cell model, 8 stations spread
    over the array: full fields and the sampler's event times within the
    bound of the reference's fp64 solve."""
    dev = _dev()
    torch.cuda.empty_cache()
    from mceik_amd import mcmc
    p = mcmc.make_problem("C5", picks="analytic")
    s = mcmc.Sampler(p, nchains=1)
    v, _, _, _ = s.state()
    ttab, _, _ = s.last()
    s.close()
    torch.cuda.empty_cache()
    stations = np.arange(0, p.nstat, p.nstat // 8)[:8]
    worst = (0.0, 0.0, -1.0, 0.0)
    u64, who = _reference_fields(p, [(v[0], s) for s in stations])
    fails = []
    for half in (stations[:4], stations[4:]):            # 4 fields of 64 MiB at a time
        u32, tt32 = _gpu_fields(p, [v[0]], half, dev)
        assert np.array_equal(tt32[0].view(np.uint32), ttab[0, half].view(np.uint32))
        for k, st in enumerate(half):
            ref = u64[int(np.flatnonzero(stations == st)[0])]
            f = _excess(u32[0, k], ref)
            e = _excess(ttab[0, st], ref[p.ev_node])
            print(f"TOLERANCE C5 station {st} ({who}): max |du| {f[0]:.3e} s, max |du|/u {f[1]:.3e}, "
                  f"|du| / bound {f[3]:.3f}; event nodes max |du|/u {e[1]:.3e}")
            worst = max(worst, f, key=lambda t: t[3])
            if f[2] > 0.0 or e[2] > 0.0:
                fails.append((int(st), f, e))
        del u32
        torch.cuda.empty_cache()
    print(f"TOLERANCE C5 fields: max |du|/u {worst[1]:.3e}, largest |du| / bound {worst[3]:.3f}")
    assert not fails, fails
    assert worst[3] <= RATIO_REGRESSION, worst


# identical accept decisions, fp32 vs fp64 sampler: observed at C2 0.99023 (50 of 5120
# differ, profiles/r05_a/gpu_tests_tolerance_phases_multistep.log); the floor leaves 2x that fraction of
# headroom.  C3's floor: see test_c3_fp32_and_fp64_samplers_accept_alike.
ACCEPT_FLOOR = 0.98


def _accept_sequences(p, offsets, nch, nsteps, prec):
    """[step, chain] accept flags of samplers of `nch` chains at each global
    chain offset (the library's default launch plan), stepped one by one."""
    from mceik_amd import mcmc
    out = []
    for off in offsets:
        s = mcmc.Sampler(p, nchains=nch, chain_offset=off, precision=prec)
        seq = []
        for _ in range(nsteps):
            s.run(1)
            seq.append(s.last()[2].astype(bool).copy())
        s.close()
        out.append(np.array(seq))
    return np.concatenate(out, axis=1)


def _compare_accepts(label, acc32, acc64, chain_ids):
    """Prints and returns (identical fraction, chains with identical
    sequences, first divergence (chain, step))."""
    same = acc32 == acc64
    frac = float(same.mean())
    chains_same = float(same.all(axis=0).mean())
    bad = np.argwhere(~same)
    first = None
    if len(bad):
        k = int(np.argmin(bad[:, 0] * same.shape[1] + bad[:, 1]))
        first = (int(chain_ids[bad[k, 1]]), int(bad[k, 0]))     # (global chain, step)
    print(f"ACCEPT {label} fp32 vs fp64 sampler, {same.shape[1]} chains x {same.shape[0]} steps: identical "
          f"decisions {frac:.5f} ({int((~same).sum())} differ), chains with identical sequences {chains_same:.4f}, "
          f"first divergence (chain, step) {first}; accept rate fp32 {acc32.mean():.3f} fp64 {acc64.mean():.3f}")
    return frac, chains_same, first


@pytest.mark.timeout(900)
def test_c2_fp32_and_fp64_samplers_accept_alike():
    """What fp32 costs the chain: the fp32 sampler (the headline) and the fp64
    sampler (the reference's arithmetic, fsm3d.f90:624-693) run from the same
    seed, start models and bench picks at C2 (256 chains, 20 steps).  Reports
    the fraction of identical accept decisions, the chains whose whole accept
    sequence agrees and the first divergent (chain, step); asserts the
    stated floor on identical decisions."""
    _dev()
    p = _bench_problem("C2")
    nch, nsteps = 256, 20
    acc = {prec: _accept_sequences(p, (0,), nch, nsteps, prec) for prec in (32, 64)}
    frac, _, _ = _compare_accepts("C2", acc[32], acc[64], np.arange(nch))
    assert frac >= ACCEPT_FLOOR


# C3 (the headline config): floor stated before the first measurement as C2's (0.98); the measured
# value is quoted in BASELINE.md beside the headline and in DESIGN.md s.5
ACCEPT_FLOOR_C3 = 0.98


@pytest.mark.timeout(900)
def test_c3_fp32_and_fp64_samplers_accept_alike():
    """The same at the headline config C3 (128^3, 32 stations, 32 events, the
    bench's picks and sigma): 128 chains -- global ids 0..63 and 512..575,
    i.e. from both halves (pipes) of the bench's 1024-chain sampler -- x the
    driver's 25 steps, fp32 against
    fp64 from the same seed.  Chains are keyed by global id, so these are
    the bench's own chains' decisions."""
    _dev()
    p = _bench_problem("C3")
    offsets, nch, nsteps = (0, 512), 64, BENCH_STEPS
    ids = np.concatenate([np.arange(o, o + nch) for o in offsets])
    acc = {prec: _accept_sequences(p, offsets, nch, nsteps, prec) for prec in (32, 64)}
    frac, chains_same, first = _compare_accepts("C3", acc[32], acc[64], ids)
    assert frac >= ACCEPT_FLOOR_C3
