/*
 * mpi_ref_driver.c -- TEST INFRASTRUCTURE (golden-vector generator, never
 * shipped or loaded by the product): runs the REFERENCE's MPI-variant eikonal
 * solver (EIKONAL3D_INITIALIZE / _SOLVE / _FINALIZE, fsm3d.f90:1583-1929,
 * built from the reference's own sources into oracle/_ref/libfsm3d_ref.so by
 * build_ref.sh) on an ndivx x ndivy x ndivz block decomposition, one MPI rank
 * per block, the way the reference's xfsm3d main does (fsm3d.f90:2055-2146:
 * MPIUTILS_INITIALIZE3D, then the three calls on the global communicator).
 *
 * usage (mpiexec -n ndivx*ndivy*ndivz):
 *   mpi_ref_driver nx ny nz ndivx ndivy ndivz noverlap maxit tol h x0 y0 z0 ts xs ys zs slow.f64 out.f64
 * The master reads the fp64 slowness (x fastest) and writes u (fp64) followed
 * by ierr (as one fp64) to out.f64.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>

void mpiutils_initialize3d(const int *comm, const int *ireord, const int *iwt, const int *ndivx, const int *ndivy,
                           const int *ndivz, int *ierr);
void mpiutils_getCommunicators(int *global, int *intra, int *inter, int *ierr);
void eikonal3d_initialize(const int *comm, const int *iverb, const int *nx, const int *ny, const int *nz,
                          const int *ndivx, const int *ndivy, const int *ndivz, const int *noverlap,
                          const int *maxit, const double *x0, const double *y0, const double *z0,
                          const double *h, const double *tol, int *ierr);
void eikonal3d_solve(const int *comm, const int *nsrc, const int *n, const double *ts, const double *xs,
                     const double *ys, const double *zs, const double *slow, double *u, int *ierr);
void eikonal3d_finalize(const int *comm, int *ierr);

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    if (argc != 20) {
        fprintf(stderr, "usage: see the header of mpi_ref_driver.c\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    int rank;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    int nx = atoi(argv[1]), ny = atoi(argv[2]), nz = atoi(argv[3]);
    int ndx = atoi(argv[4]), ndy = atoi(argv[5]), ndz = atoi(argv[6]), nov = atoi(argv[7]), maxit = atoi(argv[8]);
    double tol = atof(argv[9]), h = atof(argv[10]), x0 = atof(argv[11]), y0 = atof(argv[12]), z0 = atof(argv[13]);
    double ts = atof(argv[14]), xs = atof(argv[15]), ys = atof(argv[16]), zs = atof(argv[17]);
    int world = (int)MPI_Comm_c2f(MPI_COMM_WORLD), one = 1, zero = 0, ierr = 0, g, intra, inter;
    mpiutils_initialize3d(&world, &one, &one, &ndx, &ndy, &ndz, &ierr);
    if (ierr) MPI_Abort(MPI_COMM_WORLD, 2);
    mpiutils_getCommunicators(&g, &intra, &inter, &ierr);
    if (ierr) MPI_Abort(MPI_COMM_WORLD, 3);
    const int n = rank == 0 ? nx * ny * nz : 1, nsrc = 1;
    double *slow = calloc((size_t)n, sizeof(double)), *u = calloc((size_t)n + 1, sizeof(double));
    if (rank == 0) {
        FILE *f = fopen(argv[18], "rb");
        if (!f || fread(slow, sizeof(double), (size_t)n, f) != (size_t)n) MPI_Abort(MPI_COMM_WORLD, 4);
        fclose(f);
    }
    eikonal3d_initialize(&g, &zero, &nx, &ny, &nz, &ndx, &ndy, &ndz, &nov, &maxit, &x0, &y0, &z0, &h, &tol, &ierr);
    if (ierr) MPI_Abort(MPI_COMM_WORLD, 5);
    eikonal3d_solve(&g, &nsrc, &n, &ts, &xs, &ys, &zs, slow, u, &ierr);
    if (rank == 0) {
        u[n] = (double)ierr;
        FILE *f = fopen(argv[19], "wb");
        if (!f || fwrite(u, sizeof(double), (size_t)n + 1, f) != (size_t)n + 1) MPI_Abort(MPI_COMM_WORLD, 6);
        fclose(f);
    }
    eikonal3d_finalize(&g, &ierr);
    free(slow);
    free(u);
    MPI_Finalize();
    return 0;
}
