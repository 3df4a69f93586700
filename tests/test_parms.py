"""Run configuration (include/mceik.h mceik_parms_*, csrc/parms.c): INI file +
section:key=value overrides into mceik_parms_struct / mceik_mcmc_opts.  Host
code only, runs on CPU.  The reference parses nothing (homog.c:73-89 hard-codes
its parameters; SURVEY s.5), so the defaults are pinned to homog.c's values."""
import ctypes as C

import numpy as np
import pytest

from mceik_amd import _lib, mcmc, parms as PM

INI = """
; sampler run
[General]
projnm = "tomo;run"      # quoted value keeps ';'
scratch_dir = /tmp/x
[grid]
x0 = 100.5
dx = 250 ; dy, dz below
dy = 250
dz = 250
NX = 40
ny = 36
nz = 30
nrefx = 4
nrefy = 4
nrefz = 2
tt_interp = 1
[eikonal]
tol = 1e-7
maxit = 12
[mcmc]
nburnIn = 10
niter = 500
keepK = 5
nchains = 256
seed = 0xfffffff0
vmin = 2000
vmax = 8000
nphase = 2
vsmin = 900
vsmax = 5000
mask_s = 1
"""


def test_defaults_follow_homog():
    parms, opts = PM.defaults()
    assert (opts.nx, opts.ny, opts.nz) == (32, 29, 26)            # homog.c:76-89
    assert parms.dx == parms.dy == parms.dz == 1000.0 and parms.x0 == 0.0
    assert opts.seed == 2016 and parms.eikparms.maxit == 50 and parms.mcparms.keepK == 1


def test_read_file_and_overrides(tmp_path):
    f = tmp_path / "run.ini"
    f.write_text(INI)
    parms, opts = PM.load(f, ["mcmc:nchains=64", "--eikonal:tol=2.5e-8", "grid:x0 = -3"])
    assert parms.projnm == b"tomo;run" and parms.scratch_dir == b"/tmp/x"
    assert parms.x0 == -3.0 and parms.dx == parms.dy == parms.dz == 250.0
    assert (opts.nx, opts.ny, opts.nz) == (40, 36, 30)
    assert (parms.nrefx, parms.nrefy, parms.nrefz) == (4, 4, 2) and opts.tt_interp == 1
    assert parms.eikparms.tol == 2.5e-8 and parms.eikparms.maxit == 12
    assert (parms.mcparms.nburnIn, parms.mcparms.niter, parms.mcparms.keepK) == (10, 500, 5)
    assert opts.nchains == 64 and opts.seed == 0xfffffff0 and (opts.vmin, opts.vmax) == (2000, 8000)
    assert opts.dvmax == 50                                        # untouched default
    assert (opts.nphase, opts.vsmin, opts.vsmax, opts.mask_s) == (2, 900, 5000, 1)


def test_write_read_roundtrip(tmp_path):
    f = tmp_path / "run.ini"
    f.write_text(INI)
    parms, opts = PM.load(f)
    g = tmp_path / "out.ini"
    PM.write(g, parms, opts)
    p2, o2 = PM.load(g, base=(_lib.MceikParms(), _lib.McmcOpts()))
    assert bytes(p2) == bytes(parms) and bytes(o2) == bytes(opts)
    assert (o2.nphase, o2.vsmin, o2.vsmax, o2.mask_s) == (2, 900, 5000, 1)    # a joint P/S run stays joint


@pytest.mark.parametrize("text, line", [("[grid]\nnx = 4x\n", 2), ("[grid]\nbogus = 1\n", 2),
                                        ("nx = 4\n", 1), ("[grid]\n\n[mcmc\n", 3),
                                        ("[mcmc]\nseed = -1\n", 2), ("[grid]\ndx = nan\n", 2)])
def test_bad_lines_report_line_number(tmp_path, text, line):
    f = tmp_path / "bad.ini"
    f.write_text(text)
    L = PM._bind()
    parms, opts = PM.defaults()
    assert L.mceik_parms_read(str(f).encode(), C.byref(parms), C.byref(opts)) == line
    with pytest.raises(ValueError):
        PM.load(f)


def test_missing_file_and_bad_override():
    with pytest.raises(FileNotFoundError):
        PM.load("/nonexistent/run.ini")
    with pytest.raises(KeyError):
        PM.load(None, ["mcmc:nosuch=1"])
    with pytest.raises(ValueError):
        PM.load(None, ["mcmc:nchains=many"])


def test_command_line_args(tmp_path):
    f = tmp_path / "run.ini"
    f.write_text(INI)
    argv = [b"prog", b"--config", str(f).encode(), b"--mcmc:nchains=8", b"positional", b"grid:tt_interp=0"]
    arr = (C.c_char_p * len(argv))(*argv)
    parms, opts = PM.defaults()
    assert PM._bind().mceik_parms_args(len(argv), arr, C.byref(parms), C.byref(opts)) == 4
    assert opts.nchains == 8 and opts.tt_interp == 0 and opts.nx == 40


def test_apply_to_problem(tmp_path):
    f = tmp_path / "run.ini"
    f.write_text(INI.replace("ny = 36", "ny = 40").replace("nz = 30", "nz = 40").replace("nrefz = 2", "nrefz = 4"))
    parms, opts = PM.load(f)
    p = mcmc.make_problem("C2", n=40, nstat=3, nev=2, phases="PS")
    kw = PM.apply_to_problem(p, parms, opts)
    assert (p.vsmin, p.vsmax, p.mask_s) == (900, 5000, 1)
    assert kw["nchains"] == 256 and kw["precision"] == 32
    assert p.h == 250.0 and p.x0 == 100.5 and p.nref == (4, 4, 4) and p.tt_interp == 1
    assert p.niter == 500 and p.maxit == 12 and np.isclose(p.tol, 1e-7)
    with pytest.raises(ValueError):
        PM.apply_to_problem(mcmc.make_problem("C2", n=24, nstat=3, nev=2), parms, opts)
    with pytest.raises(ValueError):                                # nphase 2 configured, a P-only problem
        PM.apply_to_problem(mcmc.make_problem("C2", n=40, nstat=3, nev=2), parms, opts)
