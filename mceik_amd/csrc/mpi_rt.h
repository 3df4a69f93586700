/* mpi_rt.h -- internal: the MPI calls of the library, resolved at run time
 * from the calling process's (MPICH-ABI) MPI (mpi_rt.c).  Each returns -1
 * when the process runs no initialised MPI; communicators are Fortran
 * handles (MPI_Comm_c2f of a C communicator; the identity in MPICH). */
#pragma once
#ifdef __cplusplus
extern "C" {
#endif
#define MCEIK_HIDDEN __attribute__((visibility("hidden")))
MCEIK_HIDDEN int mceik_mpi_rank(int fcomm);
MCEIK_HIDDEN int mceik_mpi_size(int fcomm);
MCEIK_HIDDEN int mceik_mpi_bcast_int(int fcomm, int *v, int n, int root);
MCEIK_HIDDEN int mceik_mpi_bcast_double(int fcomm, double *v, int n, int root);
MCEIK_HIDDEN int mceik_mpi_allreduce_int(int fcomm, int *v, int n, int op);     /* op 0 sum, 1 max */
MCEIK_HIDDEN int mceik_mpi_allgather_bytes(int fcomm, const void *mine, void *all, int nbytes);
MCEIK_HIDDEN int mceik_mpi_gather_bytes(int fcomm, const void *mine, void *all, long long nbytes, int root);
MCEIK_HIDDEN int mceik_mpi_scatter_bytes(int fcomm, const void *all, void *mine, long long nbytes, int root);
MCEIK_HIDDEN int mceik_mpi_bcast_bytes(int fcomm, void *v, long long nbytes, int root);
MCEIK_HIDDEN int mceik_mpi_barrier(int fcomm);
MCEIK_HIDDEN int mceik_mpi_comm_dup(int fcomm, int *fout);
MCEIK_HIDDEN int mceik_mpi_comm_split(int fcomm, int color, int key, int *fout);
MCEIK_HIDDEN int mceik_mpi_comm_free(int fcomm);
#ifdef __cplusplus
}
#endif
