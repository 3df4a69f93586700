"""Trilinear station->event travel-time mode (north_star "station-to-event
travel-time interpolation"; mceik_fsm_batch.ev_frac, mceik_mcmc_opts.tt_interp).

The reference has no interpolation (it snaps sources and events to the
nearest node, fsm3d.f90:697-711; SURVEY s.0 #4), so this mode is parity
unpinned by the reference: the GPU tables are checked bit for bit against the
build's CPU restatement (oracle_event_time on the fp32 twin's field), and the
MCMC accept sequence in this mode against oracle_mcmc_run.
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("step_z", [0, 8], ids=["launch_choice", "z8"])
def test_batch_interp_tables_bitwise(step_z):
    """40^3 inversion-cell solves (the sampler's kernel family; step_z 0 = the
    16-z kernel), events anywhere incl. outside the grid and on faces."""
    dev = _dev()
    from mceik_amd.eikonal import BatchSolver
    from mceik_amd import mcmc
    n, h, nst, nmod = 40, 100.0, 3, 2
    p = mcmc.Problem(nx=n, ny=n, nz=n, h=h, nref=(4, 4, 4))
    rng = np.random.default_rng(5)
    ext = (n - 1) * h
    p.ex = np.concatenate([rng.uniform(0, ext, 20), [-50.0, ext + 10.0, 0.0, ext, 1234.5]])
    p.ey = np.concatenate([rng.uniform(0, ext, 20), [10.0, 20.0, 0.0, ext, ext + 300.0]])
    p.ez = np.concatenate([rng.uniform(0, ext, 20), [3000.0, 5.0, 0.0, ext, -1.0]])
    node, frac = p.ev_cell
    v = rng.integers(2500, 6000, size=(nmod, p.ncell)).astype(np.int32)
    slow = (1.0 / v.astype(np.float32)).astype(np.float32)
    src = np.stack([np.zeros(nst), rng.uniform(200, ext - 200, nst), rng.uniform(200, ext - 200, nst),
                    np.full(nst, ext)], 1)[:, None, :]
    bs = BatchSolver(n, n, n, h, 0.0, 0.0, 0.0, 50, 1e-8, 32, nref=(4, 4, 4), fast_sqrt=True)
    out = bs.solve(torch.tensor(src), torch.tensor(slow, device=dev), ev_node=torch.tensor(node),
                   ev_frac=torch.tensor(frac), want_fields=True, step_z=step_z)
    torch.cuda.synchronize()
    assert out["step_z"] == (16 if step_z == 0 else 8)
    tt = out["ttab"].cpu().numpy().reshape(nmod, nst, -1)
    u = out["u"].cpu().numpy().reshape(nmod, nst, -1)
    k, j, i = np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij")
    cell = (((k // 4) * p.ncy + j // 4) * p.ncx + i // 4).ravel()
    for m in range(nmod):
        sl = np.ascontiguousarray(slow[m][cell])
        for s in range(nst):
            tw, ierr, _ = O.eikonal_solve(n, n, n, sl, h, src[s], dtype=np.float32)
            assert ierr == 0
            assert np.array_equal(u[m, s].view(np.uint32), tw.view(np.uint32))
            want = np.array([O.event_time(tw, n, n, n, node[e], frac[e]) for e in range(len(node))], np.float32)
            assert np.array_equal(tt[m, s].view(np.uint32), want.view(np.uint32))


def test_mcmc_interp_accept_sequence_bitwise():
    """Sampler with tt_interp = 1: accept sequence, logL trace and models bitwise
    = oracle_mcmc_run in the same mode; the table differs from snapping."""
    _dev()
    from mceik_amd import mcmc
    p = mcmc.make_problem("C2", n=40, nstat=4, nev=6, seed=9, picks=mcmc.picks_from_forward(0))
    p.dvmax, p.var[:] = 400, 1e-4
    p.tt_interp = 1
    nch, nsteps, off = 4, 4, 3
    s = mcmc.Sampler(p, nchains=nch, chain_offset=off)
    v0, l0, _, _ = s.state()
    acc_g, trace_g = [], []
    for _ in range(nsteps):
        s.run(1)
        _, _, a = s.last()
        acc_g.append(a.copy())
        trace_g.append(s.state()[1].copy())
    v, logl, _, _ = s.state()
    ttab, _, _ = s.last()
    s.close()
    P = O.make_problem(p)
    vo, lo, acc, trace = O.mcmc_run(P, v0, l0, off, 0, nsteps)
    assert np.array_equal(np.array(acc_g), acc)
    assert np.array_equal(np.array(trace_g).view(np.uint64), trace.view(np.uint64))
    assert np.array_equal(v, vo) and np.array_equal(logl.view(np.uint64), lo.view(np.uint64))
    # the initial logL differs from the snapped mode's: the mode is really on
    p.tt_interp = 0
    tt_snap, _ = O.forward_f32(O.make_problem(p), v0[0])
    p.tt_interp = 1
    tt_int, _ = O.forward_f32(O.make_problem(p), v0[0])
    assert not np.array_equal(tt_snap, tt_int)
