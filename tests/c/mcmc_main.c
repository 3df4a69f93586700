/*
 * mcmc_main.c -- a C main driving the sampler through include/mceik.h only,
 * the way a homog.c-style MPI harness would (one rank here; an MPI main
 * broadcasts the RCCL id with MPI_Bcast):
 *
 *   configuration  mceik_parms_defaults + mceik_parms_args (--config FILE, section:key=value)
 *   problem        stations on the top face, events inside, straight-ray picks (homog.c-like)
 *   sampler        mceik_mcmc_init / run(-1) (mcparms.niter) / get_state / get_samples
 *   checkpoint     mceik_comm_* + mceik_mcmc_gather (RCCL), checkpoint -> restore in a
 *                  second sampler, both continue: identical chains
 *
 * Prints "check <name> <0|1>" lines; exit status 0 iff every check holds.
 * Test program written for this repo (tests/test_gpu_dropin.py).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mceik.h"

static unsigned lcg = 12345u;
static double urand(void) { lcg = lcg * 1664525u + 1013904223u; return (lcg >> 8) * (1.0 / 16777216.0); }

static int nfail = 0;
static void check(const char *name, int ok) { printf("check %s %d\n", name, ok); if (!ok) nfail++; }

int main(int argc, char **argv)
{
    struct mceik_parms_struct parms;
    mceik_mcmc_opts o;
    mceik_parms_defaults(&parms, &o);
    if (mceik_parms_args(argc, argv, &parms, &o) < 0) { fprintf(stderr, "bad arguments\n"); return 2; }
    const int nstat = 4, nev = 5, nch = o.nchains;
    const double h = parms.dx, ext[3] = {(o.nx - 1) * h, (o.ny - 1) * h, (o.nz - 1) * h};
    /* stations on the top face, events inside; P picks for every pair (CSR by event) */
    double xr[4], yr[4], zr[4], pc[4] = {0}, sc[4] = {0};
    int lhp[4] = {1, 1, 1, 1}, lhs[4] = {0};
    for (int i = 0; i < nstat; i++) {
        xr[i] = h + urand() * (ext[0] - 2 * h); yr[i] = h + urand() * (ext[1] - 2 * h); zr[i] = ext[2];
    }
    double xs[5], ys[5], zs[5], tori[5] = {0}, tobs[20], test[20] = {0}, var[20];
    int luse[20], ptype[20], sptr[20], optr[6];
    const double vel = 4000.0;
    for (int e = 0; e < nev; e++) {
        xs[e] = h + urand() * (ext[0] - 2 * h); ys[e] = h + urand() * (ext[1] - 2 * h);
        zs[e] = h + urand() * (ext[2] - 2 * h);
        optr[e] = e * nstat;
        for (int i = 0; i < nstat; i++) {
            const int j = e * nstat + i;
            const double d = sqrt((xs[e] - xr[i]) * (xs[e] - xr[i]) + (ys[e] - yr[i]) * (ys[e] - yr[i]) +
                                  (zs[e] - zr[i]) * (zs[e] - zr[i]));
            tobs[j] = d / vel + 0.002 * (urand() - 0.5);
            var[j] = 1e-4; luse[j] = 1; ptype[j] = P_PRIMARY_PICK; sptr[j] = i + 1;
        }
    }
    optr[nev] = nev * nstat;
    struct mceik_stations_struct st;
    memset(&st, 0, sizeof(st));
    st.xrec = xr; st.yrec = yr; st.zrec = zr; st.pcorr = pc; st.scorr = sc; st.lhasP = lhp; st.lhasS = lhs;
    st.nstat = nstat; st.lcartesian = 1;
    struct mceik_catalog_struct cat;
    memset(&cat, 0, sizeof(cat));
    cat.xsrc = xs; cat.ysrc = ys; cat.zsrc = zs; cat.tori = tori; cat.tobs = tobs; cat.test = test;
    cat.varObs = var; cat.luseObs = luse; cat.pickType = ptype; cat.statPtr = sptr; cat.obsPtr = optr;
    cat.nevents = nev;
    const int ncx = (o.nx + parms.nrefx - 1) / parms.nrefx, ncy = (o.ny + parms.nrefy - 1) / parms.nrefy,
              ncz = (o.nz + parms.nrefz - 1) / parms.nrefz, ncell = ncx * ncy * ncz;
    int *v0 = malloc(sizeof(int) * (size_t)nch * ncell);
    for (size_t i = 0; i < (size_t)nch * ncell; i++) v0[i] = (int)(vel + 100.0 * (urand() - 0.5));
    mceik_mcmc *s = NULL, *s2 = NULL;
    if (mceik_mcmc_init(&parms, &st, &cat, &o, v0, &s)) { fprintf(stderr, "init failed\n"); return 3; }
    const int half = parms.mcparms.niter / 2;
    if (mceik_mcmc_run(s, half)) return 4;
    /* checkpoint, restore into a second sampler, then both run the rest */
    int *cv = malloc(sizeof(int) * (size_t)nch * ncell);
    double *cl = malloc(sizeof(double) * nch);
    long long *cn = malloc(sizeof(long long) * nch), step = 0;
    int nkept = 0;
    if (mceik_mcmc_checkpoint(s, cv, cl, cn, &step, &nkept)) return 5;
    if (mceik_mcmc_init(&parms, &st, &cat, &o, v0, &s2) || mceik_mcmc_restore(s2, cv, cl, cn, step, nkept)) return 6;
    if (mceik_mcmc_run(s, -1) || mceik_mcmc_run(s2, -1)) return 7;
    int *v1 = malloc(sizeof(int) * (size_t)nch * ncell), *v2 = malloc(sizeof(int) * (size_t)nch * ncell);
    double *l1 = malloc(sizeof(double) * nch), *l2 = malloc(sizeof(double) * nch);
    long long *a1 = malloc(sizeof(long long) * nch), s1s = 0, s2s = 0;
    mceik_mcmc_get_state(s, v1, l1, a1, &s1s);
    mceik_mcmc_get_state(s2, v2, l2, NULL, &s2s);
    check("ran_niter", s1s == parms.mcparms.niter && s2s == s1s);
    check("restore_continues_bitwise", !memcmp(v1, v2, sizeof(int) * (size_t)nch * ncell) &&
                                       !memcmp(l1, l2, sizeof(double) * nch));
    long long acc = 0;
    for (int c = 0; c < nch; c++) acc += a1[c];
    check("accepts_and_rejects", acc > 0 && acc < (long long)nch * s1s);
    /* the checkpoint gather over RCCL (one rank: the id needs no broadcast) */
    unsigned char id[MCEIK_COMM_ID_BYTES];
    mceik_comm *comm = NULL;
    if (mceik_comm_unique_id(id) || mceik_comm_init(id, 1, 0, o.device, &comm)) return 8;
    int *gv = malloc(sizeof(int) * (size_t)nch * ncell), *kv = malloc(sizeof(int) * (size_t)nch * ncell);
    double *gl = malloc(sizeof(double) * nch), *kl = malloc(sizeof(double) * nch);
    int got = 0;
    check("gather_current", !mceik_mcmc_gather(s, comm, 0, nch, 0, gv, gl) &&
                            !memcmp(gv, v1, sizeof(int) * (size_t)nch * ncell) && !memcmp(gl, l1, sizeof(double) * nch));
    mceik_mcmc_get_samples(s, kv, kl, 1, 0, &got);
    {
        const int grc = mceik_mcmc_gather(s, comm, 1, nch, 0, gv, gl);
        const int vsame = !memcmp(gv, kv, sizeof(int) * (size_t)nch * ncell), lsame = !memcmp(gl, kl, sizeof(double) * nch);
        if (got != 1 || grc || !vsame || !lsame) printf("gather_kept: got %d rc %d v %d logl %d\n", got, grc, vsame, lsame);
        check("gather_kept", got == 1 && !grc && vsame && lsame);
    }
    check("gather_rejects_bad_tiling", mceik_mcmc_gather(s, comm, 0, nch + 3, 0, gv, gl) == 2);
    printf("chains %d step %lld accepted %lld logl0 %.17g\n", nch, s1s, acc, l1[0]);
    mceik_comm_finalize(&comm);
    mceik_mcmc_finalize(&s);
    mceik_mcmc_finalize(&s2);
    free(v0); free(cv); free(cl); free(cn); free(v1); free(v2); free(l1); free(l2); free(a1);
    free(gv); free(kv); free(gl); free(kl);
    return nfail ? 1 : 0;
}
