"""Host logic on CPU: Philox known answers, deterministic log, problem builder,
sharding, event snapping (no GPU)."""
import math

import numpy as np

import _oracle as O
from mceik_amd import mcmc


def test_philox4x32_10_known_answers():
    """Random123 kat_vectors for philox4x32_10."""
    assert list(O.philox([0, 0, 0, 0], [0, 0])) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    f = 0xffffffff
    assert list(O.philox([f, f, f, f], [f, f])) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert list(O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0])) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_det_log_accuracy():
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.random(2000), [2.0 ** -32, 0.5, 1.0 - 2.0 ** -53, 1e-300, 3.7]])
    for x in xs:
        v = O.lib().oracle_det_log(float(x))
        assert abs(v - math.log(x)) <= 4e-16 * max(1.0, abs(math.log(x)))


def test_problem_csr_and_snapping():
    p = mcmc.make_problem("C2", n=40, nstat=5, nev=7)
    assert p.obs_ptr[0] == 0 and p.obs_ptr[-1] == len(p.tobs) == 35
    assert np.all(np.diff(p.obs_ptr) == 5)
    assert p.obs_mask.sum() == 0 and np.all(p.tcorr == 0)
    # nearest node = EIKONAL_SOURCE_INDEX (fsm3d.f90:697-711)
    for e in range(p.nevents):
        node = int(p.ev_node[e])
        ix, iy, iz = node % p.nx, (node // p.nx) % p.ny, node // (p.nx * p.ny)
        for xs, i in ((p.ex[e], ix), (p.ey[e], iy), (p.ez[e], iz)):
            assert i == int(xs / p.h + 0.5)
    parms, st, cat = p.structs()
    assert cat.nevents == 7 and st.nstat == 5 and cat.statPtr[0] == 1   # 1-based (homog.c:227)
    assert parms.nrefx == 4 and parms.dx == p.h


def test_shard_partitions_chain_ids():
    for total, world in ((1024, 1), (8192, 8), (10, 3), (3, 4)):
        ids = []
        for r in range(world):
            lo, hi = mcmc.shard(total, r, world)
            ids.extend(range(lo, hi))
        assert ids == list(range(total))


def test_initial_models_keyed_by_global_id():
    p = mcmc.make_problem("C2", n=24, nstat=3, nev=3)
    a = mcmc.initial_models(p, range(0, 6))
    b = np.concatenate([mcmc.initial_models(p, range(0, 2)), mcmc.initial_models(p, range(2, 6))])
    assert np.array_equal(a, b)
    assert a.min() >= p.vmin and a.max() <= p.vmax


def test_oracle_mcmc_accept_rejects_outside_prior():
    p = mcmc.make_problem("C2", n=16, nstat=2, nev=3, picks="analytic")
    p.vmin, p.vmax, p.dvmax = 3000, 3001, 100            # almost every proposal leaves the prior
    P = O.make_problem(p)
    v = np.full((1, p.ncell), 3000, np.int32)
    tt, _ = O.forward_f32(P, v[0])
    vo, lo, acc, _ = O.mcmc_run(P, v, [O.loglik(P, tt)], 0, 0, 5)
    assert acc.sum() <= 5 and np.all((vo >= 3000) & (vo <= 3001))


def test_trilinear_event_time_restatement():
    """oracle_event_time (the trilinear mode's checker): exact on a linear field
    with dyadic fractions, the node value at w = 0 or w = None, corner clamping
    on the grid's last plane."""
    nx, ny, nz = 5, 4, 3
    k, j, i = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    u = (1.0 + 2.0 * i + 4.0 * j + 8.0 * k).astype(np.float32).ravel()
    rng = np.random.default_rng(2)
    for _ in range(50):
        x, y, z = rng.integers(0, nx - 1), rng.integers(0, ny - 1), rng.integers(0, nz - 1)
        w = rng.integers(0, 5, 3) / 4.0
        node = (z * ny + y) * nx + x
        t = O.event_time(u, nx, ny, nz, node, w)
        assert t == np.float32(1.0 + 2.0 * (x + w[0]) + 4.0 * (y + w[1]) + 8.0 * (z + w[2]))
        assert O.event_time(u, nx, ny, nz, node, np.zeros(3)) == u[node] == O.event_time(u, nx, ny, nz, node)
    last = (nz - 1) * nx * ny + (ny - 1) * nx + nx - 1      # corners clamp to the grid
    assert O.event_time(u, nx, ny, nz, last, np.full(3, 0.5)) == u[last]


def test_event_cells_trilinear_mode():
    """Problem.ev_cell: lowest corner clamped to [0, n-2], fractions in [0, 1];
    on-node events get fraction 0 (or 1 on the last plane)."""
    p = mcmc.Problem(nx=10, ny=8, nz=6, h=100.0, x0=50.0)
    p.ex = np.array([50.0, 150.0, 925.0, -10.0, 2000.0, 925.0 - 1e-9])
    p.ey = np.array([0.0, 100.0, 700.0, 0.0, 0.0, 350.0])
    p.ez = np.array([0.0, 500.0, 250.0, -5.0, 0.0, 0.0])
    node, w = p.ev_cell
    ix, iy, iz = node % 10, (node // 10) % 8, node // 80
    assert list(ix) == [0, 1, 8, 0, 8, 8] and list(iy) == [0, 1, 6, 0, 0, 3] and list(iz) == [0, 4, 2, 0, 0, 0]
    assert w.dtype == np.float32 and np.all((w >= 0) & (w <= 1))
    assert list(w[:, 0]) == [0.0, 0.0, np.float32(0.75), 0.0, 1.0, np.float32(0.75 - 1e-11)]
    assert w[1, 2] == 1.0 and w[2, 1] == 1.0 and w[5, 1] == 0.5
