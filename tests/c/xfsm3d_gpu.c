/* A C caller of libmceik_hip.so's drop-in eikonal entry points, in the flow of
 * the reference's xfsm3d test program (fsm3d.f90:2055-2146): 70 x 80 x 90
 * nodes, h = 100 m, v = 5000 m/s, one source at the centre, maxit = 5,
 * tol = 1e-7.  First the MPI-variant initialize / solve / finalize, then the
 * serial driver job 1 / 2 / 3; prints min and max of both fields (the
 * reference's own known answer is max u = 1.4308203212738235) and the wall
 * time of each solve call.  Written for this repository; links only the
 * public headers and libmceik_hip.so. */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "mceik.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void minmax(const double *u, int n, double *mn, double *mx)
{
    *mn = u[0]; *mx = u[0];
    for (int i = 1; i < n; i++) {
        if (u[i] < *mn) *mn = u[i];
        if (u[i] > *mx) *mx = u[i];
    }
}

int main(void)
{
    int comm = 0, iverb = 0, nx = 70, ny = 80, nz = 90, ndiv = 2, noverlap = 1, maxit = 5, nsrc = 1, ierr = 0;
    double x0 = 0.0, y0 = 0.0, z0 = 0.0, h = 100.0, tol = 1.0e-7;
    double ts = 0.0, xs = x0 + h * nx / 2.0, ys = y0 + h * ny / 2.0, zs = z0 + h * nz / 2.0;
    int n = nx * ny * nz;
    double *slow = malloc(sizeof(double) * n), *u = malloc(sizeof(double) * n), mn, mx;
    for (int i = 0; i < n; i++) slow[i] = 1.0 / 5.0e3;
    eikonal3d_initialize(&comm, &iverb, &nx, &ny, &nz, &ndiv, &ndiv, &ndiv, &noverlap, &maxit, &x0, &y0, &z0, &h,
                         &tol, &ierr);
    if (ierr) { printf("initialize failed %d\n", ierr); return 1; }
    double t = now();
    eikonal3d_solve(&comm, &nsrc, &n, &ts, &xs, &ys, &zs, slow, u, &ierr);
    t = now() - t;
    if (ierr) { printf("solve failed %d\n", ierr); return 1; }
    minmax(u, n, &mn, &mx);
    printf("mpi_variant min %.17g max %.17g solve_s %.6f\n", mn, mx, t);
    {   /* a non-master rank passes n = 1 and gets nothing back */
        int one = 1;
        double u1 = -1.0, s1 = 1.0 / 5.0e3;
        eikonal3d_solve(&comm, &nsrc, &one, &ts, &xs, &ys, &zs, &s1, &u1, &ierr);
        printf("non_master ierr %d u1 %.1f\n", ierr, u1);
    }
    eikonal3d_finalize(&comm, &ierr);
    int job = 1;
    eikonal3d_serial_driver(&job, &iverb, &maxit, &nsrc, &nx, &ny, &nz, &tol, &h, &x0, &y0, &z0, &ts, &xs, &ys, &zs,
                            slow, u, &ierr);
    job = 2;
    for (int rep = 0; rep < 3; rep++) {
        t = now();
        eikonal3d_serial_driver(&job, &iverb, &maxit, &nsrc, &nx, &ny, &nz, &tol, &h, &x0, &y0, &z0, &ts, &xs, &ys,
                                &zs, slow, u, &ierr);
        t = now() - t;
        if (ierr) { printf("serial driver failed %d\n", ierr); return 1; }
        minmax(u, n, &mn, &mx);
        printf("serial_driver min %.17g max %.17g solve_s %.6f\n", mn, mx, t);
    }
    job = 3;
    eikonal3d_serial_driver(&job, &iverb, &maxit, &nsrc, &nx, &ny, &nz, &tol, &h, &x0, &y0, &z0, &ts, &xs, &ys, &zs,
                            slow, u, &ierr);
    free(slow);
    free(u);
    return 0;
}
