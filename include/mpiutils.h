/*
 * mpiutils.h -- the reference harness's communicator layout (reference
 * include/mpiutils.h, mpiutils.f90:99-426), implemented in libmceik_hip.so
 * over the caller's MPI (resolved at run time, csrc/mpi_rt.c).  Communicators
 * are Fortran handles (MPI_Comm_c2f; homog.c:91-109 converts both ways).
 *
 * mpiutils_initialize3d splits `comm` into ntables = nprocs / (ndivx ndivy
 * ndivz) table groups of one rank per block: global = a duplicate of comm
 * (the reference's path: its neighbour-graph variant is disabled,
 * mpiutils.f90:119,231-240), intra-table = ranks of one table (colour
 * rank / nblocks), inter-table = ranks holding the same block (colour rank
 * mod nblocks).  ierr = 1 (nothing created) unless every ndiv >= 1 and
 * nblocks divides the rank count.  ireord / iwt only weighted that disabled
 * graph and are accepted and ignored, as there.
 */
#ifndef __MPIUTILS_H__
#define __MPIUTILS_H__
#ifdef __cplusplus
extern "C" {
#endif
void mpiutils_getCommunicators(int *globalComm, int *intraTableComm, int *interTableComm, int *ierr);
/* block igrd (0-based, x fastest) -> (i, j, k); ierr counts the violated bounds */
void mpiutils_grd2ijk(const int *igrd, const int *nx, const int *ny, const int *nz, int *i, int *j, int *k,
                      int *ierr);
void mpiutils_initialize3d(const int *comm, const int *ireord, const int *iwt, const int *ndivx, const int *ndivy,
                           const int *ndivz, int *ierr);
/* ndivy = 1 (mpiutils.f90:307-325) */
void mpiutils_initialize2d(const int *comm, const int *ireord, const int *iwt, const int *ndivx, const int *ndivz,
                           int *ierr);
void mpiutils_finalize(void);
#ifdef __cplusplus
}
#endif
#endif
