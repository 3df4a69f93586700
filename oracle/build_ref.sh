#!/usr/bin/env bash
# Builds the REFERENCE's own hot-path sources, where they lie under
# /root/reference, into oracle/_ref/ (git-ignored; travels to the GPU box).
# Test infrastructure only: the product never links or loads anything here.
#
#  * libfsm3d_ref.so : module.F90 + mpiutils.f90 + fsm3d.f90 compiled with amdflang
#    (ROCm 7.2 flang).  fsm3d.f90/mpiutils.f90 say `USE MPI`; the image ships
#    MPICH's real mpif.h (/opt/conda/include) but its mpi.mod is gfortran-format,
#    so a module named MPI is generated from that real header (INCLUDE 'mpif.h').
#    No MPI routine is replaced: the objects link against the image's libmpi.
#  * liblocate_ref.so : locate.c (L2/L1 misfit).  locate.c:8 includes
#    <lapacke_utils.h> only for MIN/MAX; the image has no LAPACKE, so a -D pair
#    supplies those two macros and the include is satisfied from an empty dir.
#    Built without -fopenmp (locate.c:1308 does not compile under it).
#  * xgridsearch : gridsearch.f90 main program (known-answer: optimum 21124).
#  * mpi_ref_driver : oracle/mpi_ref_driver.c (ours) calling the reference's
#    MPI-variant solver on a block decomposition, for tests/golden/blocks_mpi.npz.
# Nothing from /root/reference is copied into the repository.
set -euo pipefail
R=${REFERENCE_DIR:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
F=/opt/rocm/lib/llvm/bin/amdflang
if [ ! -f "$R/fsm3d.f90" ]; then echo "build_ref: $R not present, skipping"; exit 0; fi
mkdir -p "$OUT" "$OUT/mod" "$OUT/inc"
cd "$OUT"
printf "      MODULE MPI\n      INCLUDE 'mpif.h'\n      END MODULE MPI\n" > mod/mpimod.f90
$F -c -fPIC -O2 -I/opt/conda/include -module-dir mod mod/mpimod.f90 -o mod/mpimod.o
$F -c -fPIC -O2 -module-dir mod -I mod "$R/module.F90" -o mod/module.o
$F -c -fPIC -O2 -module-dir mod -I mod -I/opt/conda/include "$R/mpiutils.f90" -o mod/mpiutils.o
$F -c -fPIC -O2 -fopenmp -module-dir mod -I mod -I/opt/conda/include "$R/fsm3d.f90" -o mod/fsm3d.o 2> mod/fsm3d.warn || { cat mod/fsm3d.warn; exit 1; }
$F -shared -fPIC -fopenmp -o libfsm3d_ref.so mod/mpimod.o mod/module.o mod/mpiutils.o mod/fsm3d.o \
   -L/opt/conda/lib -Wl,-rpath,/opt/conda/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib -lmpifort -lmpi
# the reference's own MPI test program (xfsm3d main, fsm3d.f90:2055-2183)
$F -O2 -fopenmp -o xfsm3d mod/mpimod.o mod/module.o mod/mpiutils.o mod/fsm3d.o \
   -L/opt/conda/lib -Wl,-rpath,/opt/conda/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib -lmpifort -lmpi
# golden generator for the MPI variant (our test driver oracle/mpi_ref_driver.c,
# linked against the reference build above; run under mpiexec by make_golden.py)
gcc -O1 -I/opt/conda/include "$HERE/mpi_ref_driver.c" -o mpi_ref_driver -L"$OUT" -lfsm3d_ref /opt/conda/lib/libmpi.so \
    -Wl,-rpath,"$OUT":/usr/lib/x86_64-linux-gnu:/opt/conda/lib:/opt/rocm/lib/llvm/lib
: > inc/lapacke_utils.h
gcc -O2 -fPIC -shared -I inc -I/opt/conda/include '-DMIN(a,b)=((a)<(b)?(a):(b))' '-DMAX(a,b)=((a)>(b)?(a):(b))' \
    -Dmain=locate_c_unused_main "$R/locate.c" -o liblocate_ref.so -lm 2> inc/locate.warn || { cat inc/locate.warn; exit 1; }
$F -O2 -module-dir mod "$R/gridsearch.f90" -o xgridsearch 2> mod/gridsearch.warn
# the same file's BIND(C) locate3d_gridsearch__double64/__float64 as a shared
# object (flang's main() lives in its runtime, so the PROGRAM unit links inert)
$F -O2 -fPIC -shared -module-dir mod "$R/gridsearch.f90" -o libgridsearch_ref.so 2>> mod/gridsearch.warn
echo "build_ref: built $(ls "$OUT" | tr '\n' ' ')"
