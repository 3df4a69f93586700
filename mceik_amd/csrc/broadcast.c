/* broadcast.c -- broadcast_stations / broadcast_catalog (include/mceik_broadcast.h;
 * reference broadcast.c:14-143) over the caller's MPI, resolved at run time
 * (mpi_rt.c).  Field order and allocation follow the reference so that a
 * homog.c-style main frees the result the same way. */
#include <stdlib.h>
#include <string.h>

#define MPICH_SKIP_MPICXX 1
#include <mpi.h>

#include "../../include/mceik_broadcast.h"
#include "mpi_rt.h"

static void *zalloc(int n, size_t sz) { return calloc((size_t)(n > 0 ? n : 1), sz); }

void broadcast_stations(MPI_Comm comm, const int root, struct mceik_stations_struct *st)
{
    const int fc = (int)MPI_Comm_c2f(comm);
    const int me = mceik_mpi_rank(fc);
    if (me < 0 || !st) return;                     /* no MPI: one rank, nothing to send */
    int hdr[2] = {st->nstat, st->lcartesian};
    mceik_mpi_bcast_int(fc, hdr, 2, root);
    st->nstat = hdr[0];
    st->lcartesian = hdr[1];
    const int n = st->nstat;
    if (n < 1) return;
    const int mine = me == root;
    if (!mine) {
        st->lhasP = (int *)zalloc(n, sizeof(int));
        st->lhasS = (int *)zalloc(n, sizeof(int));
    }
    mceik_mpi_bcast_int(fc, st->lhasP, n, root);
    mceik_mpi_bcast_int(fc, st->lhasS, n, root);
    double **d[5] = {&st->xrec, &st->yrec, &st->zrec, &st->pcorr, &st->scorr};
    for (int k = 0; k < 5; k++) {
        if (!mine) *d[k] = (double *)zalloc(n, sizeof(double));
        mceik_mpi_bcast_double(fc, *d[k], n, root);
    }
    char ***names[4] = {&st->netw, &st->stnm, &st->chan, &st->loc};
    if (!mine)
        for (int k = 0; k < 4; k++) {
            *names[k] = (char **)zalloc(n, sizeof(char *));
            for (int i = 0; i < n; i++) (*names[k])[i] = (char *)zalloc(64, 1);
        }
    /* the four 64-byte codes of a station together, station by station */
    char buf[4 * 64];
    for (int i = 0; i < n; i++) {
        if (mine)
            for (int k = 0; k < 4; k++) {
                const char *src = *names[k] ? (*names[k])[i] : NULL;
                if (src) memcpy(buf + 64 * k, src, 64);
                else memset(buf + 64 * k, 0, 64);
            }
        mceik_mpi_bcast_bytes(fc, buf, sizeof(buf), root);
        if (!mine)
            for (int k = 0; k < 4; k++) memcpy((*names[k])[i], buf + 64 * k, 64);
    }
}

void broadcast_catalog(MPI_Comm comm, const int root, struct mceik_catalog_struct *cat)
{
    const int fc = (int)MPI_Comm_c2f(comm);
    const int me = mceik_mpi_rank(fc);
    if (me < 0 || !cat) return;
    mceik_mpi_bcast_int(fc, &cat->nevents, 1, root);
    const int nev = cat->nevents;
    if (nev < 1) return;
    const int mine = me == root;
    int nobs = mine ? cat->obsPtr[nev] : 0;
    mceik_mpi_bcast_int(fc, &nobs, 1, root);
    int **iv[4] = {&cat->luseObs, &cat->pickType, &cat->statPtr, &cat->obsPtr};
    for (int k = 0; k < 4; k++) {
        const int cnt = k == 3 ? nev + 1 : nobs;
        if (!mine) *iv[k] = (int *)zalloc(cnt, sizeof(int));
        mceik_mpi_bcast_int(fc, *iv[k], cnt, root);
    }
    double **dv[7] = {&cat->xsrc, &cat->ysrc, &cat->zsrc, &cat->tori, &cat->tobs, &cat->test, &cat->varObs};
    for (int k = 0; k < 7; k++) {
        const int cnt = k < 4 ? nev : nobs;
        if (!mine) *dv[k] = (double *)zalloc(cnt, sizeof(double));
        mceik_mpi_bcast_double(fc, *dv[k], cnt, root);
    }
}
