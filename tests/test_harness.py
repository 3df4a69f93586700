"""homog.c launch flow (SURVEY s.8f row 3) on torch.distributed: problem
generation, broadcast, table split, h5io write/verify; CPU (gloo) here, GPU
location in the gpu-marked test."""
import math
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def test_homog_setup_matches_homog_c_geometry():
    from mceik_amd import harness as H
    g, st, cat = H.homog_setup()
    assert (g["nx"], g["ny"], g["nz"]) == (32, 29, 26)              # homog.c:76-89
    assert len(st["xrec"]) == 6 and np.all(st["zrec"] == 25.0e3)     # free surface
    assert np.all(np.mod(st["xrec"], 1000.0) == 0) and np.all(np.mod(st["yrec"], 1000.0) == 0)
    assert np.all((st["xrec"] >= 0) & (st["xrec"] <= 31.0e3) & (st["yrec"] >= 0) & (st["yrec"] <= 28.0e3))
    assert list(cat["obsPtr"]) == [0, 12, 24, 36, 48]
    assert list(cat["pickType"][:4]) == [1, 2, 1, 2] and list(cat["statPtr"][:4]) == [1, 1, 2, 2]
    d = math.dist((st["xrec"][0], st["yrec"][0], st["zrec"][0]), (cat["xsrc"][0], cat["ysrc"][0], cat["zsrc"][0]))
    assert cat["tobs"][0] == d / 2000.0 and cat["tobs"][1] == d / (2000.0 / math.sqrt(3.0))
    assert np.all(cat["varObs"] == 0.25) and np.all(st["lhasP"] == 1) and np.all(st["lhasS"] == 1)
    # deterministic under the seed
    _, st2, cat2 = H.homog_setup()
    assert np.array_equal(st["xrec"], st2["xrec"]) and np.array_equal(cat["xsrc"], cat2["xsrc"])


def test_single_process_tables_written_and_verified(tmp_path):
    from mceik_amd import h5io, harness as H
    hypo, files = H.run_homog(str(tmp_path), "homog", solver="analytic", locate=False)
    assert hypo is None and files[0].endswith("homog_1_ttimes.h5")
    g, st, _ = H.homog_setup()
    with h5io.H5File.open(files[0]) as f:
        assert f.dims() == (g["nx"], g["ny"], g["nz"])
        for s in range(1, 7):
            ref = H.homogeneous_traveltimes(g["nx"], g["ny"], g["nz"], 0.0, 0.0, 0.0, 1e3, 1e3, 1e3,
                                            st["xrec"][s - 1], st["yrec"][s - 1], st["zrec"][s - 1], g["vp"])
            assert np.array_equal(f.read_ttimes(s, 1, iphase=1), ref.astype(np.float32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here); sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    from mceik_amd import harness as H
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    st = {} if rank else H.homog_setup()[1]
    st = H.broadcast_stations(st, 0)
    _, files = H.run_homog(outdir, "homog", solver="analytic", locate=False)
    q.put((rank, st["xrec"].tolist(), files))
    dist.destroy_process_group()


def test_two_rank_broadcast_split_and_gather(tmp_path):
    import torch.multiprocessing as tmp
    from mceik_amd import h5io, harness as H
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    _, st, _ = H.homog_setup()
    assert res[0][1] == res[1][1] == st["xrec"].tolist()          # broadcast_stations
    assert res[1][2] is None and res[0][2][0].endswith("homog_1_ttimes.h5")
    g = H.homog_setup()[0]
    with h5io.H5File.open(res[0][2][0]) as f:                         # every table, from both ranks
        for s, ph in H.table_list(st):
            ref = H.homogeneous_traveltimes(g["nx"], g["ny"], g["nz"], 0.0, 0.0, 0.0, 1e3, 1e3, 1e3,
                                            st["xrec"][s - 1], st["yrec"][s - 1], st["zrec"][s - 1],
                                            g["vp"] if ph == 1 else g["vs"])
            assert np.array_equal(f.read_ttimes(s, 1, iphase=ph), ref.astype(np.float32))


@pytest.mark.gpu
def test_homog_locates_events_on_gpu(tmp_path):
    """The homog.c flow end to end on one GPU.  Location: the GPU relocation
    grid search over homog.c's analytic tables puts every event on the node
    the reference's fp32 L2 grid search picks (oracle restatement pinned to
    locate.c), within two nodes of the true hypocentre.  Tables: the fp64 FSM
    tables written by the harness are the fp64 FSM solutions (bitwise the
    oracle, itself bitwise the reference fsm3d), stored as fp32."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import _oracle as O
    from mceik_amd import h5io, harness as H
    g, st, cat = H.homog_setup()
    hypo, files = H.run_homog(str(tmp_path), "homog", solver="analytic", locate=True)
    keys = H.table_list(st)
    n = g["nx"] * g["ny"] * g["nz"]
    ld = n + (-n) % 16
    tabs = np.zeros((len(keys), ld), np.float32)
    for i, (s, ph) in enumerate(keys):
        tabs[i, :n] = H.homogeneous_traveltimes(g["nx"], g["ny"], g["nz"], 0.0, 0.0, 0.0, 1e3, 1e3, 1e3,
                                                st["xrec"][s - 1], st["yrec"][s - 1], st["zrec"][s - 1],
                                                g["vp"] if ph == 1 else g["vs"]).astype(np.float32)
    row = {k: i for i, k in enumerate(keys)}
    for e in range(4):
        ks = list(range(cat["obsPtr"][e], cat["obsPtr"][e + 1]))
        rows = [row[(int(cat["statPtr"][k]), int(cat["pickType"][k]))] for k in ks]
        _, _, obj = O.locate_l2_f32(ld, n, len(rows), 1, 0.0, np.zeros(len(rows), np.int32), cat["tobs"][ks], None,
                                    cat["varObs"][ks], tabs[rows].ravel())
        k, rem = divmod(int(np.argmin(obj)), g["nx"] * g["ny"])
        j, i = divmod(rem, g["nx"])
        assert tuple(hypo[e]) == (i * 1e3, j * 1e3, k * 1e3)
        # surface stations constrain depth least: within two nodes
        assert np.all(np.abs(hypo[e] - (cat["xsrc"][e], cat["ysrc"][e], cat["zsrc"][e])) <= 2e3)
    with h5io.H5File.open(files[1]) as f:
        for e in range(4):
            assert f.read_logjpdf(1, e + 1).max() <= 0.0
    os.makedirs(tmp_path / "fsm")
    _, files2 = H.run_homog(str(tmp_path / "fsm"), "homog", solver="fsm", locate=False)
    slow = np.full(n, 1.0 / g["vp"])
    with h5io.H5File.open(files2[0]) as f:
        for s_ in range(1, 7):
            src = np.array([[0.0, st["xrec"][s_ - 1], st["yrec"][s_ - 1], st["zrec"][s_ - 1]]])
            ref, ierr, _ = O.eikonal_solve(g["nx"], g["ny"], g["nz"], slow, 1e3, src, maxit=50, tol=1e-8)
            assert ierr == 0
            assert np.array_equal(f.read_ttimes(s_, 1, iphase=1), ref.astype(np.float32))
