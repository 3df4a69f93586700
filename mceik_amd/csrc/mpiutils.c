/* mpiutils.c -- include/mpiutils.h: the reference harness's table / block
 * communicators (mpiutils.f90:99-426) over the caller's MPI, resolved at run
 * time (mpi_rt.c).  Without an initialised MPI initialize3d fails (ierr 1),
 * as the reference's MPI calls would. */
#include <stdio.h>

#include "../../include/mpiutils.h"
#include "mpi_rt.h"

static struct {
    int init, global, intra, inter;
} g_comm;

void mpiutils_grd2ijk(const int *igrd, const int *nx, const int *ny, const int *nz, int *i, int *j, int *k,
                      int *ierr)
{
    const int nxy = *nx * *ny;
    *k = *igrd / nxy;
    *j = (*igrd - *k * nxy) / *nx;
    *i = *igrd - *k * nxy - *j * *nx;
    *ierr = (*i < 0 || *i >= *nx) + (*j < 0 || *j >= *ny) + (*k < 0 || *k >= *nz) +
            (*k * nxy + *j * *nx + *i != *igrd);
}

void mpiutils_initialize3d(const int *comm, const int *ireord, const int *iwt, const int *ndivx, const int *ndivy,
                           const int *ndivz, int *ierr)
{
    (void)ireord; (void)iwt;
    *ierr = 1;
    if (g_comm.init) printf("mpiutils_initialize3d: Warning communicator already initialized\n");
    const int nprocs = mceik_mpi_size(*comm), myid = mceik_mpi_rank(*comm);
    if (nprocs < 1 || myid < 0) {
        printf("mpiutils_initialize3d: no initialised MPI in this process\n");
        return;
    }
    if (*ndivx < 1 || *ndivy < 1 || *ndivz < 1) {
        printf("mpiutils_initialize3d: ndivx, ndivy and ndivz must be positive (%d %d %d)\n", *ndivx, *ndivy, *ndivz);
        return;
    }
    const int nblocks = *ndivx * *ndivy * *ndivz;
    if (nblocks > nprocs || nprocs % nblocks != 0) {
        printf("mpiutils_initialize3d: %d processes cannot hold tables of %d blocks\n", nprocs, nblocks);
        return;
    }
    const int table = myid / nblocks, block = myid % nblocks;
    int bi, bj, bk, e = 0;
    mpiutils_grd2ijk(&block, ndivx, ndivy, ndivz, &bi, &bj, &bk, &e);
    if (e) {
        printf("mpiutils_initialize3d: Error computing rank in grid %d %d\n", myid, block);
        return;
    }
    int g, a, b;
    if (mceik_mpi_comm_dup(*comm, &g)) return;
    const int gid = mceik_mpi_rank(g);
    if (mceik_mpi_comm_split(g, table, gid, &a) || mceik_mpi_comm_split(g, block, gid, &b)) return;
    if (mceik_mpi_size(a) != nblocks || mceik_mpi_size(b) != nprocs / nblocks) {
        printf("mpiutils_initialize3d: Error splitting the table communicators\n");
        return;
    }
    g_comm.global = g; g_comm.intra = a; g_comm.inter = b;
    g_comm.init = 1;
    *ierr = 0;
}

void mpiutils_initialize2d(const int *comm, const int *ireord, const int *iwt, const int *ndivx, const int *ndivz,
                           int *ierr)
{
    const int one = 1;
    mpiutils_initialize3d(comm, ireord, iwt, ndivx, &one, ndivz, ierr);
    if (*ierr) printf("mpiutils_initialize2d: Error splitting communicator!\n");
}

void mpiutils_getCommunicators(int *globalComm, int *intraTableComm, int *interTableComm, int *ierr)
{
    if (!g_comm.init) {
        printf("mpiutils_getCommunicators: Never initialized communicators\n");
        *ierr = 1;
        return;
    }
    *globalComm = g_comm.global;
    *intraTableComm = g_comm.intra;
    *interTableComm = g_comm.inter;
    *ierr = 0;
}

/* whether mpiutils_initialize3d has split the communicators (locate3d.hip:
 * the reference's linitComm, locate.f90:610) */
__attribute__((visibility("hidden"))) int mceik_mpiutils_initialized(void) { return g_comm.init; }

void mpiutils_finalize(void)
{
    if (!g_comm.init) return;
    mceik_mpi_comm_free(g_comm.global);
    mceik_mpi_comm_free(g_comm.intra);
    mceik_mpi_comm_free(g_comm.inter);
    g_comm.init = 0;
}
