/*
 * mpi_sampler_main.c -- the multi-rank flow of INTEGRATION.md s.3 as a C/MPI
 * main (one rank per GPU), the role homog.c:31-459 + broadcast.c:14-143 play
 * for the reference:
 *
 *   rank 0 makes the problem (stations on the top face, events inside,
 *   straight-ray picks) and broadcasts it (MPI_Bcast, as broadcast.c does);
 *   every rank takes its shard of the global chains, runs the sampler to
 *   mcparms.niter, and the kept states are gathered to rank 0 over RCCL
 *   (mceik_mcmc_gather; MPI only carries the 128-byte RCCL id).
 *
 * Rank 0 checks that its own shard in the gathered array equals its local
 * kept state and prints "check <name> <0|1>" lines and the gathered checksum.
 * Test program written for this repo (tests/test_gpu_dropin.py runs it with
 * mpiexec -n 1 where an MPI toolchain exists; RCCL takes one rank per GPU).
 */
#include <math.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mceik.h"

static unsigned lcg = 2016u;   /* homog.c:113 seeds with 2016 */
static double urand(void) { lcg = lcg * 1664525u + 1013904223u; return (lcg >> 8) * (1.0 / 16777216.0); }

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank, size, nfail = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    struct mceik_parms_struct parms;
    mceik_mcmc_opts o;
    mceik_parms_defaults(&parms, &o);
    if (mceik_parms_args(argc, argv, &parms, &o) < 0) MPI_Abort(MPI_COMM_WORLD, 30);
    const int nstat = 4, nev = 3, nobs = nstat * nev, ctot = o.nchains;
    /* problem on rank 0, then broadcast (broadcast.c) */
    double st_xyz[3 * 4], ev_xyz[3 * 3], tobs[12], var[12];
    if (rank == 0) {
        const double h = parms.dx, ex = (o.nx - 1) * h, ey = (o.ny - 1) * h, ez = (o.nz - 1) * h;
        for (int i = 0; i < nstat; i++) {
            st_xyz[3 * i] = h + urand() * (ex - 2 * h); st_xyz[3 * i + 1] = h + urand() * (ey - 2 * h);
            st_xyz[3 * i + 2] = ez;
        }
        for (int e = 0; e < nev; e++) {
            ev_xyz[3 * e] = h + urand() * (ex - 2 * h); ev_xyz[3 * e + 1] = h + urand() * (ey - 2 * h);
            ev_xyz[3 * e + 2] = h + urand() * (ez - 2 * h);
            for (int i = 0; i < nstat; i++) {
                double d = 0.0;
                for (int k = 0; k < 3; k++) d += (ev_xyz[3 * e + k] - st_xyz[3 * i + k]) * (ev_xyz[3 * e + k] - st_xyz[3 * i + k]);
                tobs[e * nstat + i] = sqrt(d) / 4000.0 + 0.002 * (urand() - 0.5);
                var[e * nstat + i] = 1e-4;
            }
        }
    }
    MPI_Bcast(st_xyz, 3 * nstat, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    MPI_Bcast(ev_xyz, 3 * nev, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    MPI_Bcast(tobs, nobs, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    MPI_Bcast(var, nobs, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    double xr[4], yr[4], zr[4], pc[4] = {0}, sc[4] = {0}, xs[3], ys[3], zs[3], tori[3] = {0}, test[12] = {0};
    int lhp[4] = {1, 1, 1, 1}, lhs[4] = {0}, luse[12], ptype[12], sptr[12], optr[4];
    for (int i = 0; i < nstat; i++) { xr[i] = st_xyz[3 * i]; yr[i] = st_xyz[3 * i + 1]; zr[i] = st_xyz[3 * i + 2]; }
    for (int e = 0; e < nev; e++) {
        xs[e] = ev_xyz[3 * e]; ys[e] = ev_xyz[3 * e + 1]; zs[e] = ev_xyz[3 * e + 2];
        optr[e] = e * nstat;
        for (int i = 0; i < nstat; i++) {
            luse[e * nstat + i] = 1; ptype[e * nstat + i] = P_PRIMARY_PICK; sptr[e * nstat + i] = i + 1;
        }
    }
    optr[nev] = nobs;
    struct mceik_stations_struct st;
    memset(&st, 0, sizeof(st));
    st.xrec = xr; st.yrec = yr; st.zrec = zr; st.pcorr = pc; st.scorr = sc; st.lhasP = lhp; st.lhasS = lhs;
    st.nstat = nstat; st.lcartesian = 1;
    struct mceik_catalog_struct cat;
    memset(&cat, 0, sizeof(cat));
    cat.xsrc = xs; cat.ysrc = ys; cat.zsrc = zs; cat.tori = tori; cat.tobs = tobs; cat.test = test;
    cat.varObs = var; cat.luseObs = luse; cat.pickType = ptype; cat.statPtr = sptr; cat.obsPtr = optr;
    cat.nevents = nev;
    /* this rank's shard of the global chains (SURVEY s.8e); one GPU per rank */
    const int base = ctot / size, extra = ctot % size;
    o.chain_offset = rank * base + (rank < extra ? rank : extra);
    o.nchains = base + (rank < extra ? 1 : 0);
    o.device = rank;
    const int ncell = ((o.nx + parms.nrefx - 1) / parms.nrefx) * ((o.ny + parms.nrefy - 1) / parms.nrefy) *
                      ((o.nz + parms.nrefz - 1) / parms.nrefz);
    int *v0 = malloc(sizeof(int) * (size_t)o.nchains * ncell);
    for (size_t i = 0; i < (size_t)o.nchains * ncell; i++) v0[i] = 4000 + (int)((i * 2654435761u) % 101) - 50;
    mceik_mcmc *s = NULL;
    if (mceik_mcmc_init(&parms, &st, &cat, &o, v0, &s)) MPI_Abort(MPI_COMM_WORLD, 31);
    unsigned char id[MCEIK_COMM_ID_BYTES];
    if (rank == 0 && mceik_comm_unique_id(id)) MPI_Abort(MPI_COMM_WORLD, 32);
    MPI_Bcast(id, MCEIK_COMM_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
    mceik_comm *comm = NULL;
    if (mceik_comm_init(id, size, rank, o.device, &comm)) MPI_Abort(MPI_COMM_WORLD, 33);
    if (mceik_mcmc_run(s, -1)) MPI_Abort(MPI_COMM_WORLD, 34);
    int *gv = rank == 0 ? malloc(sizeof(int) * (size_t)ctot * ncell) : NULL;
    double *gl = rank == 0 ? malloc(sizeof(double) * ctot) : NULL;
    int rc = mceik_mcmc_gather(s, comm, 1, ctot, 0, gv, gl);
    if (rank == 0) {
        int *kv = malloc(sizeof(int) * (size_t)o.nchains * ncell), got = 0;
        double *kl = malloc(sizeof(double) * o.nchains);
        mceik_mcmc_get_samples(s, kv, kl, 1, 0, &got);
        int ok = rc == 0 && got == 1 && !memcmp(gv + (size_t)o.chain_offset * ncell, kv, sizeof(int) * (size_t)o.nchains * ncell) &&
                 !memcmp(gl + o.chain_offset, kl, sizeof(double) * o.nchains);
        printf("check gather_own_shard %d\n", ok);
        nfail += !ok;
        unsigned long long sum = 0;
        for (size_t i = 0; i < (size_t)ctot * ncell; i++) sum = sum * 31u + (unsigned)gv[i];
        printf("ranks %d chains %d checksum %llu\n", size, ctot, sum);
        free(kv); free(kl);
    }
    mceik_comm_finalize(&comm);
    mceik_mcmc_finalize(&s);
    free(v0); free(gv); free(gl);
    MPI_Finalize();
    return nfail ? 1 : 0;
}
