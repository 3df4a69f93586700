/* homog_h5io.c -- the reference harness's table and location I/O flow
 * (homog.c:31-451, minus its Fortran locator) on this build's drop-in C-ABI:
 * rank 0 makes homog.c's station list and catalog, broadcast_stations /
 * broadcast_catalog hand them to every rank, each rank takes its block of the
 * grid (ndivx = ranks, homog.c:264-287), eikonal_h5io_initTTables creates the
 * table file, every table (one per lhasP / lhasS flag, homog.c:311-335) is
 * computed, written, read back and checked to 1e-5 (homog.c:340-415) -- the
 * communicators from mpiutils_initialize3d / getCommunicators as homog.c
 * builds them (homog.c:90-110) -- then
 * eikonal_h5io_initLocations, a logJPDF write / read, readModel,
 * getModelDimensions and finalize.  Exit 0 when every check passes.
 * With a fourth argument "locate <job>" it also runs homog.c:428-450's
 * location step on the tables it wrote (locate3d_initialize / gridsearch /
 * finalize, include/locate.h) and rank 0 prints every hypocentre and the
 * estimates of event 1 ("LOCATE ...", "TEST ..." lines, %.17g); picks whose
 * table was not written (station 3's S picks) are not used.
 *
 *   mpiexec -n {1,2,4} homog_h5io <dir> <proj> [ndivx [locate <job>]]   (ndivx blocks per table:
 *   nprocs / ndivx table groups, each writing <proj>_<group>_ttimes.h5 through its intra-table
 *   communicator)
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mpi.h>

#include "h5io.h"
#include "locate.h"
#include "mceik_broadcast.h"
#include "mceik_struct.h"
#include "mpiutils.h"

#define CHECK(cond, ...)                                                    \
    do {                                                                    \
        if (!(cond)) {                                                      \
            fprintf(stderr, "rank %d: ", myid);                             \
            fprintf(stderr, __VA_ARGS__);                                   \
            fprintf(stderr, "\n");                                          \
            MPI_Abort(MPI_COMM_WORLD, 30);                                  \
        }                                                                   \
    } while (0)

/* homog.c:594-621: straight-ray times in a constant velocity */
static void homogeneous_times(int nx, int ny, int nz, double x0, double y0, double z0, double dx, double dy,
                              double dz, double xs, double ys, double zs, double vel, double *tt)
{
    const double slow = 1.0 / vel;
    for (int iz = 0; iz < nz; iz++)
        for (int iy = 0; iy < ny; iy++)
            for (int ix = 0; ix < nx; ix++) {
                const double x = x0 + (double)ix * dx, y = y0 + (double)iy * dy, z = z0 + (double)iz * dz;
                const double d = sqrt(pow(xs - x, 2) + pow(ys - y, 2) + pow(zs - z, 2));
                tt[((size_t)iz * ny + iy) * nx + ix] = d * slow;
            }
}

int main(int argc, char **argv)
{
    int myid = 0, nprocs = 1;
    MPI_Init(&argc, &argv);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    MPI_Comm_rank(MPI_COMM_WORLD, &myid);
    const char *dir = argc > 1 ? argv[1] : "./";
    const char *proj = argc > 2 ? argv[2] : "homog";
    const double vp = 2000.0, vs = vp / sqrt(3.0);
    const double x0 = 0.0, y0 = 0.0, z0 = 0.0, x1 = 31.e3, y1 = 28.e3, z1 = 25.e3, dx = 1000., dy = 1000., dz = 1000.;
    const int nx = (int)((x1 - x0) / dx + 0.5) + 1, ny = (int)((y1 - y0) / dy + 0.5) + 1,
              nz = (int)((z1 - z0) / dz + 0.5) + 1;
    const int nmodels = 1, model = 1, ndivx = argc > 3 ? atoi(argv[3]) : nprocs, ndivy = 1, ndivz = 1;
    /* the table / block communicators (homog.c:90-110) */
    int gcomm, intra, inter, ireord = 1, iwt = 0, ierr = 0;
    const int world = (int)MPI_Comm_c2f(MPI_COMM_WORLD);
    mpiutils_initialize3d(&world, &ireord, &iwt, &ndivx, &ndivy, &ndivz, &ierr);
    CHECK(ierr == 0, "mpiutils_initialize3d");
    mpiutils_getCommunicators(&gcomm, &intra, &inter, &ierr);
    CHECK(ierr == 0, "mpiutils_getCommunicators");
    const MPI_Comm intraComm = MPI_Comm_f2c((MPI_Fint)intra), interComm = MPI_Comm_f2c((MPI_Fint)inter);
    int myblock = 0, mytable = 0, nblk = 0, ntab = 0;
    MPI_Comm_rank(intraComm, &myblock);
    MPI_Comm_rank(interComm, &mytable);
    MPI_Comm_size(intraComm, &nblk);
    MPI_Comm_size(interComm, &ntab);
    CHECK(nblk == ndivx && ntab == nprocs / ndivx && myblock == myid % ndivx && mytable == myid / ndivx,
          "communicator layout");
    char tproj[256];
    snprintf(tproj, sizeof(tproj), "%s_%d", proj, mytable + 1);   /* one table file per table group (homog.c:290-293) */
    struct mceik_stations_struct st;
    struct mceik_catalog_struct cat;
    memset(&st, 0, sizeof(st));
    memset(&cat, 0, sizeof(cat));
    if (myid == 0) {                               /* homog.c:111-239 */
        srand(2016);
        const int nxrec = 2, nyrec = 3, nev = 4;
        st.nstat = nxrec * nyrec;
        st.lcartesian = 1;
        st.netw = calloc(st.nstat, sizeof(char *)); st.stnm = calloc(st.nstat, sizeof(char *));
        st.chan = calloc(st.nstat, sizeof(char *)); st.loc = calloc(st.nstat, sizeof(char *));
        for (int i = 0; i < st.nstat; i++) {
            st.netw[i] = calloc(64, 1); st.stnm[i] = calloc(64, 1);
            st.chan[i] = calloc(64, 1); st.loc[i] = calloc(64, 1);
            strcpy(st.netw[i], "NA"); sprintf(st.stnm[i], "RC%d", i + 1);
            strcpy(st.chan[i], "HH?"); strcpy(st.loc[i], "00");
        }
        st.xrec = calloc(st.nstat, sizeof(double)); st.yrec = calloc(st.nstat, sizeof(double));
        st.zrec = calloc(st.nstat, sizeof(double));
        for (int iy = 0; iy < nyrec; iy++)
            for (int ix = 0; ix < nxrec; ix++) {
                st.xrec[iy * nxrec + ix] = x0 + ((int)((double)rand() / RAND_MAX * (nx - 1))) * dx;
                st.yrec[iy * nxrec + ix] = y0 + ((int)((double)rand() / RAND_MAX * (ny - 1))) * dy;
                st.zrec[iy * nxrec + ix] = z1;
            }
        st.pcorr = calloc(st.nstat, sizeof(double)); st.scorr = calloc(st.nstat, sizeof(double));
        st.lhasP = calloc(st.nstat, sizeof(int)); st.lhasS = calloc(st.nstat, sizeof(int));
        cat.nevents = nev;
        const int nwork = 2 * nev * st.nstat;
        cat.xsrc = calloc(nev, sizeof(double)); cat.ysrc = calloc(nev, sizeof(double));
        cat.zsrc = calloc(nev, sizeof(double)); cat.tori = calloc(nev, sizeof(double));
        cat.tobs = calloc(nwork, sizeof(double)); cat.test = calloc(nwork, sizeof(double));
        cat.varObs = calloc(nwork, sizeof(double));
        cat.luseObs = calloc(nwork, sizeof(int)); cat.pickType = calloc(nwork, sizeof(int));
        cat.statPtr = calloc(nwork, sizeof(int)); cat.obsPtr = calloc(nev + 1, sizeof(int));
        int nkeep = 0;
        for (int i = 0; i < nev; i++) {
            cat.xsrc[i] = x0 + (x1 - x0) * (double)rand() / RAND_MAX;
            cat.ysrc[i] = y0 + (y1 - y0) * (double)rand() / RAND_MAX;
            cat.zsrc[i] = z0 + (z1 - z0) * (double)rand() / RAND_MAX;
            for (int k = 0; k < st.nstat; k++) {
                const double d = sqrt(pow(st.xrec[k] - cat.xsrc[i], 2) + pow(st.yrec[k] - cat.ysrc[i], 2) +
                                      pow(st.zrec[k] - cat.zsrc[i], 2));
                for (int ph = P_PRIMARY_PICK; ph <= S_PRIMARY_PICK; ph++) {
                    cat.tobs[nkeep] = d / (ph == P_PRIMARY_PICK ? vp : vs);
                    cat.varObs[nkeep] = 0.25;
                    cat.luseObs[nkeep] = 1;
                    cat.pickType[nkeep] = ph;
                    cat.statPtr[nkeep] = k + 1;
                    nkeep++;
                }
                /* the test's own twist: station 3 (1-based) has P picks only */
                if (i == 0) { st.lhasP[k] = 1; st.lhasS[k] = k != 2; }
            }
            cat.obsPtr[i + 1] = nkeep;
        }
    }
    broadcast_stations(MPI_COMM_WORLD, 0, &st);
    broadcast_catalog(MPI_COMM_WORLD, 0, &cat);
    CHECK(st.nstat == 6 && st.lcartesian == 1 && cat.nevents == 4 && cat.obsPtr[4] == 48, "broadcast sizes");
    CHECK(!strcmp(st.stnm[5], "RC6") && !strcmp(st.chan[0], "HH?") && st.lhasS[2] == 0 && st.lhasS[3] == 1,
          "broadcast station fields");
    CHECK(cat.pickType[1] == S_PRIMARY_PICK && cat.statPtr[47] == 6 && cat.varObs[17] == 0.25, "broadcast catalog");
    /* this rank's block (homog.c:264-287) */
    int imbx, imby, imbz, e = 0;
    mpiutils_grd2ijk(&myblock, &ndivx, &ndivy, &ndivz, &imbx, &imby, &imbz, &e);
    CHECK(e == 0, "grd2ijk");
    const int ndx = nx / ndivx > 1 ? nx / ndivx : 1, ndy = ny / ndivy > 1 ? ny / ndivy : 1,
              ndz = nz / ndivz > 1 ? nz / ndivz : 1;
    const int ix0 = imbx * ndx, iy0 = imby * ndy, iz0 = imbz * ndz;
    const int ix1 = imbx + 1 == ndivx ? nx : (imbx + 1) * ndx, iy1 = imby + 1 == ndivy ? ny : (imby + 1) * ndy,
              iz1 = imbz + 1 == ndivz ? nz : (imbz + 1) * ndz;
    const int nxL = ix1 - ix0, nyL = iy1 - iy0, nzL = iz1 - iz0;
    const size_t nloc = (size_t)nxL * nyL * nzL;
    hid_t tfid = -1, lfid = -1;
    ierr = eikonal_h5io_initTTables(intraComm, dir, tproj, ix0, iy0, iz0, nx, ny, nz, nxL, nyL, nzL, nmodels,
                                    st.nstat, false, x0, y0, z0, dx, dy, dz, &tfid);
    CHECK(ierr == 0, "initTTables");
    double *tt = calloc(nloc, sizeof(double));
    float *t4 = calloc(nloc, sizeof(float));
    int ntables = 0;
    for (int k = 0; k < st.nstat; k++)
        for (int ph = P_PRIMARY_PICK; ph <= S_PRIMARY_PICK; ph++) {
            if (!(ph == P_PRIMARY_PICK ? st.lhasP[k] : st.lhasS[k])) continue;
            ntables++;
            homogeneous_times(nxL, nyL, nzL, x0 + ix0 * dx, y0 + iy0 * dy, z0 + iz0 * dz, dx, dy, dz, st.xrec[k],
                              st.yrec[k], st.zrec[k], ph == S_PRIMARY_PICK ? vs : vp, tt);
            for (size_t i = 0; i < nloc; i++) t4[i] = (float)tt[i];
            /* homog.c:377 passes the 1-based table station number (k + 1 here) */
            ierr = eikonal_h5io_writeTravelTimes(intraComm, tfid, k + 1, model, ph, ix0, iy0, iz0, nxL, nyL,
                                                 nzL, t4);
            CHECK(ierr == 0, "writeTravelTimes station %d phase %d", k + 1, ph);
            memset(t4, 0, nloc * sizeof(float));
            ierr = eikonal_h5io_readTravelTimes(intraComm, tfid, k + 1, model, ph, ix0, iy0, iz0, nxL, nyL,
                                                nzL, t4);
            CHECK(ierr == 0, "readTravelTimes station %d phase %d", k + 1, ph);
            double dmax = 0.0;
            for (size_t i = 0; i < nloc; i++) dmax = fmax(dmax, fabs(t4[i] - (float)tt[i]));
            CHECK(dmax <= 1.e-5, "read/write verification: %g", dmax);
        }
    CHECK(ntables == 11, "table count %d", ntables);
    /* a missing dataset is an error on every rank */
    CHECK(eikonal_h5io_readTravelTimes(intraComm, tfid, 7, model, 1, ix0, iy0, iz0, nxL, nyL, nzL, t4) != 0,
          "station 7 does not exist");
    int gx = 0, gy = 0, gz = 0;
    CHECK(eikonal_h5io_getModelDimensions(tfid, &gx, &gy, &gz) == 0 && gx == nx && gy == ny && gz == nz,
          "getModelDimensions %d %d %d", gx, gy, gz);
    float *xl = calloc(nloc, sizeof(float)), *yl = calloc(nloc, sizeof(float)), *zl = calloc(nloc, sizeof(float));
    CHECK(eikonal_h5io_readModel(intraComm, tfid, ix0, iy0, iz0, nxL, nyL, nzL, xl, yl, zl) == 0, "readModel");
    for (int k = 0; k < nzL; k++)
        for (int j = 0; j < nyL; j++)
            for (int i = 0; i < nxL; i++) {
                const size_t n = ((size_t)k * nyL + j) * nxL + i;
                CHECK(xl[n] == (float)(x0 + (double)(i + ix0) * dx) && yl[n] == (float)(y0 + (double)(j + iy0) * dy) &&
                          zl[n] == (float)(z0 + (double)(k + iz0) * dz), "model coordinates at %zu", n);
            }
    ierr = eikonal_h5io_initLocations(MPI_COMM_WORLD, dir, proj, ix0, iy0, iz0, nx, ny, nz, nxL, nyL, nzL, nmodels,
                                      cat.nevents, x0, y0, z0, dx, dy, dz, &lfid);
    CHECK(ierr == 0, "initLocations");
    for (size_t i = 0; i < nloc; i++) t4[i] = -(float)(i % 97) - 0.25f * (float)myblock;
    CHECK(eikonal_h5io_writeLocationLogJPDF(MPI_COMM_WORLD, lfid, model, 2, ix0, iy0, iz0, nxL, nyL, nzL, t4) == 0,
          "writeLocationLogJPDF");
    if (argc > 5 && !strcmp(argv[4], "locate")) {   /* homog.c:428-450 */
        const int locJob = atoi(argv[5]);
        int iverb = 0;
        long tl = (long)tfid, ll = (long)lfid;
        locate3d_initialize(&intra, &iverb, &tl, &ll, &ndivx, &ndivy, &ndivz, &ierr);
        CHECK(ierr == 0, "locate3d_initialize");
        double *hypo = calloc((size_t)cat.nevents * 4, sizeof(double));
        int nobs = 2 * st.nstat;
        double *statCor = calloc((size_t)nobs, sizeof(double));
        for (int i = 0; i < cat.nevents; i++) cat.tori[i] = 0.5 * i;        /* job 1's fixed origin times */
        for (int i = 0; i < cat.nevents * nobs; i++)
            if (cat.pickType[i] == S_PRIMARY_PICK && !st.lhasS[cat.statPtr[i] - 1]) cat.luseObs[i] = 0;
        locate3d_gridsearch(&model, &locJob, &nobs, &cat.nevents, cat.luseObs, cat.statPtr, cat.pickType, statCor,
                            cat.tori, cat.varObs, cat.tobs, cat.test, hypo, &ierr);
        CHECK(ierr == 0, "locate3d_gridsearch");
        locate3d_finalize();
        if (myid == 0) {
            for (int i = 0; i < cat.nevents; i++)
                printf("LOCATE %d %.17g %.17g %.17g %.17g\n", i + 1, hypo[4 * i], hypo[4 * i + 1], hypo[4 * i + 2],
                       hypo[4 * i + 3]);
            for (int i = 0; i < nobs; i++) printf("TEST %d %d %.17g\n", i + 1, cat.luseObs[i], cat.test[i]);
        }
        free(hypo);
        free(statCor);
    }
    CHECK(eikonal_h5io_finalize(intraComm, &tfid) == 0 && eikonal_h5io_finalize(intraComm, &lfid) == 0,
          "finalize");
    mpiutils_finalize();
    MPI_Barrier(MPI_COMM_WORLD);
    if (myid == 0) printf("homog_h5io: %d ranks, %d table groups, %d tables ok\n", nprocs, ntab, ntables);
    MPI_Finalize();
    return 0;
}
