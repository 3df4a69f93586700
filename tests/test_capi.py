"""The C-ABI library loads and exports every symbol include/*.h declares, and
the data-model structs are ABI-identical to the reference's mceik_struct.h.
No compute calls (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
REF_INC = "/root/reference/include"


def _declared_functions():
    names = set()
    for h in ("mceik.h", "mceik_eikonal.h", "os.h", "locate.h"):
        txt = open(os.path.join(INC, h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:int|void|size_t|double|bool|const char)\s+\**\s*([A-Za-z_]\w*)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    from mceik_amd import _lib
    L = _lib.lib()
    declared = _declared_functions()
    assert len(declared) >= 14
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for name in declared:
        assert name in exported, name
        assert getattr(L, name) is not None


def test_os_helpers(tmp_path):
    """include/os.h (the reference's os.h, declared by its mceik.h): path tests,
    mkdir, and makedirs of nested, existing and trailing-slash paths."""
    from mceik_amd import _lib
    L = _lib.lib()
    for f in ("os_path_exists", "os_path_isdir", "os_path_isfile"):
        getattr(L, f).restype = C.c_bool
        getattr(L, f).argtypes = [C.c_char_p]
    L.os_makedirs.argtypes = L.os_mkdir.argtypes = [C.c_char_p]
    d = str(tmp_path).encode()
    f = os.path.join(str(tmp_path), "a.txt")
    open(f, "w").write("x")
    assert L.os_path_isdir(d) and not L.os_path_isfile(d) and L.os_path_exists(d)
    assert L.os_path_isfile(f.encode()) and not L.os_path_isdir(f.encode())
    assert not L.os_path_exists(d + b"/nope") and not L.os_path_isdir(b"") and not L.os_path_isdir(None)
    assert L.os_mkdir(d + b"/m") == 0 and L.os_path_isdir(d + b"/m")
    assert L.os_mkdir(d + b"/m") == -1 and L.os_mkdir(d + b"/x/y") == -1
    assert L.os_makedirs(d + b"/p/q/r") == 0 and L.os_path_isdir(d + b"/p/q/r")
    assert L.os_makedirs(d + b"/p/q/r") == 0 and L.os_makedirs(d + b"/s/t/") == 0 and L.os_path_isdir(d + b"/s/t")
    assert L.os_makedirs(f.encode() + b"/z") == -1 and L.os_makedirs(b"") == -1


def test_missing_library_fails_loudly(monkeypatch):
    from mceik_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libmceik_hip.so")
    with pytest.raises(ImportError):
        _lib.lib()


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "mceik_struct.h"
#define P(T, m) printf(#T "." #m " %zu\n", offsetof(struct T, m))
int main(void) {
  printf("catalog %zu stations %zu mcmc %zu eik %zu parms %zu\n", sizeof(struct mceik_catalog_struct),
         sizeof(struct mceik_stations_struct), sizeof(struct mcmc_parms_struct), sizeof(struct eik_parms_struct),
         sizeof(struct mceik_parms_struct));
  P(mceik_catalog_struct, xsrc); P(mceik_catalog_struct, varObs); P(mceik_catalog_struct, obsPtr);
  P(mceik_catalog_struct, nevents); P(mceik_stations_struct, xrec); P(mceik_stations_struct, lhasS);
  P(mceik_stations_struct, nstat); P(mceik_stations_struct, lcartesian); P(mcmc_parms_struct, keepK);
  P(mceik_parms_struct, eikparms); P(mceik_parms_struct, projnm); P(mceik_parms_struct, x0);
  P(mceik_parms_struct, dz); P(mceik_parms_struct, ndivz); P(mceik_parms_struct, nrefz);
  printf("P %d S %d\n", P_PRIMARY_PICK, S_PRIMARY_PICK);
  return 0;
}
"""


def _layout(incdir):
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "l.c")
        open(src, "w").write(LAYOUT_C)
        exe = os.path.join(td, "l")
        subprocess.run(["gcc", "-I", incdir, src, "-o", exe], check=True)
        return subprocess.run([exe], capture_output=True, text=True, check=True).stdout


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers not present (GPU box)")
def test_struct_layout_identical_to_reference_header():
    assert _layout(INC) == _layout(REF_INC)


def test_ctypes_mirrors_match_header():
    from mceik_amd import _lib
    out = _layout(INC).split()
    sizes = dict(zip(out[0:10:2], map(int, out[1:10:2])))
    assert C.sizeof(_lib.CatalogStruct) == sizes["catalog"]
    assert C.sizeof(_lib.StationsStruct) == sizes["stations"]
    assert C.sizeof(_lib.McmcParms) == sizes["mcmc"]
    assert C.sizeof(_lib.EikParms) == sizes["eik"]
    assert C.sizeof(_lib.MceikParms) == sizes["parms"]
    assert _lib.MceikParms.nrefz.offset == int(_layout(INC).split("mceik_parms_struct.nrefz ")[1].split()[0])


def _offsets_c(header, ctype, fields):
    """sizeof and offsetof(every field) of a C struct, from gcc on the public header."""
    body = "".join(f'  printf("{f} %zu\\n", offsetof({ctype}, {f}));\n' for f in fields)
    src = (f'#include <stdio.h>\n#include <stddef.h>\n#include "{header}"\n'
           f'int main(void) {{\n  printf("sizeof %zu\\n", sizeof({ctype}));\n{body}  return 0;\n}}\n')
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "o.c")
        open(p, "w").write(src)
        exe = os.path.join(td, "o")
        subprocess.run(["gcc", "-I", INC, p, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    return dict(zip(out[0::2], map(int, out[1::2])))


@pytest.mark.parametrize("header,ctype,pyname", [
    ("mceik_eikonal.h", "mceik_fsm_batch", "FsmBatch"),
    ("mceik_eikonal.h", "mceik_relocate_batch", "RelocateBatch"),
    ("mceik.h", "mceik_mcmc_opts", "McmcOpts"),
    ("mceik.h", "mceik_mcmc_info", "McmcInfo"),
])
def test_ctypes_batch_structs_match_public_headers(header, ctype, pyname):
    """Every field of the ctypes mirrors sits at the C offset (the batch
    descriptors are passed by pointer across the C-ABI)."""
    from mceik_amd import _lib
    cls = getattr(_lib, pyname)
    names = [f[0] for f in cls._fields_]
    c = _offsets_c(header, ctype, names)
    assert C.sizeof(cls) == c["sizeof"]
    for n in names:
        assert getattr(cls, n).offset == c[n], n


@pytest.mark.parametrize("src,mpi", [("xfsm3d_gpu.c", False), ("mcmc_main.c", False), ("xfsm3d_mpi.c", True),
                                     ("mpi_sampler_main.c", True), ("blocks_mpi_gpu.c", True)])
def test_c_callers_compile_and_link(tmp_path, src, mpi):
    """The C callers the GPU tests run (tests/c/*.c) build against include/ and
    link against libmceik_hip.so here on the CPU, so a header or ABI drift
    shows without a GPU (MPI callers against the image's MPICH)."""
    lib = os.path.join(ROOT, "mceik_amd")
    mpidir = "/opt/conda"
    if mpi and not (os.path.exists(f"{mpidir}/include/mpi.h") and os.path.exists(f"{mpidir}/lib/libmpi.so")):
        pytest.skip("no MPI toolchain in this image")
    cmd = ["gcc", "-O1", "-I", os.path.join(ROOT, "include")]
    if mpi:
        cmd += ["-I", f"{mpidir}/include"]
    cmd += [os.path.join(ROOT, "tests", "c", src), "-L", lib, "-lmceik_hip"]
    if mpi:
        cmd += [f"{mpidir}/lib/libmpi.so"]
    cmd += [f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{lib}" + (f":{mpidir}/lib" if mpi else ""), "-lm",
            "-o", str(tmp_path / "caller")]
    subprocess.run(cmd, check=True)


def test_locate3d_refuses_before_initialize_and_unknown_jobs():
    """include/locate.h (locate.f90:322-519): locate3d_gridsearch without a
    locate3d_initialize, and the jobs the reference leaves "not yet done" (3,
    5) or rejects, return ierr 1 before any GPU work (CPU host)."""
    import ctypes as C
    from mceik_amd import _lib
    L = _lib.lib()
    i = lambda v: C.byref(C.c_int(v))
    ierr = C.c_int(0)
    z = C.c_void_p(0)
    L.locate3d_finalize()
    L.locate3d_gridsearch(i(1), i(2), i(0), i(0), z, z, z, z, z, z, z, z, z, C.byref(ierr))
    assert ierr.value == 1
