/* The MPI variant's block decomposition across ranks (fsm3d.f90:103-222,
 * 1583-1852): one MPI rank per block, every rank sweeping its own block on the
 * GPU and swapping face layers with its neighbours after every sweep, the
 * master gathering u.  Same command line and output file as the golden
 * generator's driver of the reference (oracle/mpi_ref_driver.c), so the test
 * compares the two runs file for file:
 *
 *   mpiexec -n ndivx*ndivy*ndivz blocks_mpi_gpu nx ny nz ndivx ndivy ndivz noverlap maxit tol h
 *           x0 y0 z0 ts xs ys zs slow.f64 out.f64
 *
 * The master reads the fp64 slowness (x fastest) and writes u followed by its
 * ierr (one fp64) to out.f64; every rank prints "rank <r> ierr <e>".  The
 * other ranks pass n = 1 as the reference's xfsm3d does (:2102-2106).
 * Written for this repository. */
#include <stdio.h>
#include <stdlib.h>

#include <mpi.h>

#include "mceik.h"

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    if (argc != 20) {
        fprintf(stderr, "usage: see the header of blocks_mpi_gpu.c\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    int rank;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    int nx = atoi(argv[1]), ny = atoi(argv[2]), nz = atoi(argv[3]);
    int ndx = atoi(argv[4]), ndy = atoi(argv[5]), ndz = atoi(argv[6]), nov = atoi(argv[7]), maxit = atoi(argv[8]);
    double tol = atof(argv[9]), h = atof(argv[10]), x0 = atof(argv[11]), y0 = atof(argv[12]), z0 = atof(argv[13]);
    double ts = atof(argv[14]), xs = atof(argv[15]), ys = atof(argv[16]), zs = atof(argv[17]);
    int comm = (int)MPI_Comm_c2f(MPI_COMM_WORLD), zero = 0, ierr = 0;
    const int n = rank == 0 ? nx * ny * nz : 1, nsrc = 1;
    double *slow = calloc((size_t)n, sizeof(double)), *u = calloc((size_t)n + 1, sizeof(double));
    if (rank == 0) {
        FILE *f = fopen(argv[18], "rb");
        if (!f || fread(slow, sizeof(double), (size_t)n, f) != (size_t)n) MPI_Abort(MPI_COMM_WORLD, 4);
        fclose(f);
    }
    eikonal3d_initialize(&comm, &zero, &nx, &ny, &nz, &ndx, &ndy, &ndz, &nov, &maxit, &x0, &y0, &z0, &h, &tol, &ierr);
    if (ierr) {                          /* every rank returns the same error: no rank is left waiting */
        printf("rank %d init_ierr %d\n", rank, ierr);
        free(slow);
        free(u);
        MPI_Finalize();
        return 0;
    }
    eikonal3d_solve(&comm, &nsrc, &n, &ts, &xs, &ys, &zs, slow, u, &ierr);
    printf("rank %d ierr %d\n", rank, ierr);
    if (rank == 0) {
        u[n] = (double)ierr;
        FILE *f = fopen(argv[19], "wb");
        if (!f || fwrite(u, sizeof(double), (size_t)n + 1, f) != (size_t)n + 1) MPI_Abort(MPI_COMM_WORLD, 6);
        fclose(f);
    }
    eikonal3d_finalize(&comm, &ierr);
    free(slow);
    free(u);
    MPI_Finalize();
    return 0;
}
