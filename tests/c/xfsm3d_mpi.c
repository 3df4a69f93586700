/* The MPI variant's collective contract (fsm3d.f90:1583-1929) from a C/MPI
 * caller run under mpiexec with several ranks: rank 0's parameters are used
 * on every rank whatever the others pass (:1626-1639), rank 0's SETBCS error
 * reaches every rank (:1792), and finalizing an uninitialised solver reports
 * ierr = 1 (:1913-1916).  xfsm3d's problem (fsm3d.f90:2055-2146): 70 x 80 x 90
 * nodes, h = 100 m, v = 5000 m/s, centre source, maxit 5, tol 1e-7; the
 * non-master ranks pass n = 1 (:2102-2106).  Prints one line per rank and
 * call.  Written for this repository. */
#include <stdio.h>
#include <stdlib.h>

#include <mpi.h>

#include "mceik.h"

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    int comm = (int)MPI_Comm_c2f(MPI_COMM_WORLD);
    int iverb = 0, nsrc = 1, ierr = -7, ndiv = 1, noverlap = 1;
    /* only rank 0's grid counts: the others pass nonsense */
    int nx = rank ? 3 : 70, ny = rank ? 4 : 80, nz = rank ? 5 : 90, maxit = rank ? 1 : 5;
    double x0 = 0.0, y0 = 0.0, z0 = 0.0, h = rank ? 1.0 : 100.0, tol = rank ? 1.0 : 1.0e-7;
    eikonal3d_initialize(&comm, &iverb, &nx, &ny, &nz, &ndiv, &ndiv, &ndiv, &noverlap, &maxit, &x0, &y0, &z0, &h,
                         &tol, &ierr);
    printf("init rank %d ierr %d\n", rank, ierr);
    const int full = 70 * 80 * 90;
    int n = rank ? 1 : full;
    double *slow = malloc(sizeof(double) * full), *u = malloc(sizeof(double) * full);
    for (int i = 0; i < full; i++) { slow[i] = 1.0 / 5.0e3; u[i] = -1.0; }
    /* a source exactly on the first node: SETBCS's ierr = 1 (fsm3d.f90:736-753) on the master */
    double ts = 0.0, xs = rank ? 3000.0 : x0, ys = rank ? 3000.0 : y0, zs = rank ? 3000.0 : z0;
    ierr = -7;
    eikonal3d_solve(&comm, &nsrc, &n, &ts, &xs, &ys, &zs, slow, u, &ierr);
    printf("origin rank %d ierr %d\n", rank, ierr);
    xs = x0 + h * 70 / 2.0; ys = y0 + h * 80 / 2.0; zs = z0 + h * 90 / 2.0;
    if (rank) xs = ys = zs = 0.0;        /* ignored: only the master's sources are solved */
    ierr = -7;
    for (int i = 0; i < full; i++) u[i] = -1.0;
    eikonal3d_solve(&comm, &nsrc, &n, &ts, &xs, &ys, &zs, slow, u, &ierr);
    double mx = u[0];
    for (int i = 1; i < full; i++) mx = u[i] > mx ? u[i] : mx;
    printf("solve rank %d ierr %d max %.17g\n", rank, ierr, mx);
    eikonal3d_finalize(&comm, &ierr);
    printf("finalize rank %d ierr %d\n", rank, ierr);
    eikonal3d_finalize(&comm, &ierr);
    printf("refinalize rank %d ierr %d\n", rank, ierr);
    free(slow);
    free(u);
    MPI_Finalize();
    return 0;
}
