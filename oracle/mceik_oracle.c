/* mceik_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path, used solely as the CHECKER by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * mceik_amd/ links, loads or calls this file; the product fails loudly when its
 * HIP library is missing instead of falling back here.
 *
 * Contents (reference file:line followed by each piece):
 *   - eikonal serial solve, fp64 and fp32 twins (fsm_impl.inc; fsm3d.f90:28-99,
 *     419-840, 1968-2052)
 *   - L2 grid-search misfit with analytic origin time (locate.c:388-567,923-1047)
 *   - Fortran grid-search variant (gridsearch.f90:176-329,382-456), for the
 *     reference's own known-answer test (optimum 21124, t0 ~ 4 s)
 *   - Philox4x32-10, deterministic log, proposal and Metropolis step: the
 *     reference defines no MCMC (include/mceik.h:1-14 is empty), so these restate
 *     the build's own definition; parity there is between
 *     this file and the HIP kernels, not with the reference.
 * Build: gcc -O2 -ffp-contract=off -fopenmp (oracle/Makefile).  Pinned against
 * the compiled reference by tests/golden (tests/golden/make_golden.py).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* EIKONAL_SOURCE_INDEX (fsm3d.f90:697-711); returns a 1-based index. */
static int oracle_source_index(int nx, double x0, double dx, double xs)
{
    if (xs <= x0) return 1;
    if (xs >= x0 + (double)(nx - 1) * dx) return nx;
    return (int)((xs - x0) / dx + 0.5) + 1;
}

/* EIKONAL_INIT_GRID (fsm3d.f90:716-755).  Note the reference's quirks: an
 * on-node source always includes isx-1 (so isx=1 is an error) and includes
 * isx+1 only when isx < nx-1. */
static int oracle_init_grid(int nx, int isx, double x0, double dx, double xs, int loc[3])
{
    int np = 0, ierr = 0;
    loc[0] = loc[1] = loc[2] = -1;
    double xe = x0 + (double)(isx - 1) * dx;
    if (xe > xs)      { loc[0] = isx - 1; loc[1] = isx; np = 2; }
    else if (xe < xs) { loc[0] = isx; loc[1] = isx + 1; np = 2; }
    else {
        if (isx > 0) loc[np++] = isx - 1;
        loc[np++] = isx;
        if (isx < nx - 1) loc[np++] = isx + 1;
    }
    for (int i = 0; i < np; i++) if (loc[i] < 1 || loc[i] > nx) ierr = 1;
    return ierr;
}

/* ---- fp64 twin (bitwise the reference) ---- */
#define REAL double
#define FN(x) x##_f64
#define RC(x) (x)
#define UNAN DBL_MAX
#define SQRT sqrt
#define FABS fabs
#define THIRD (1.0 / 3.0)
#define TWO_THIRD (2.0 / 3.0)
#include "fsm_impl.inc"
#undef REAL
#undef FN
#undef RC
#undef UNAN
#undef SQRT
#undef FABS
#undef THIRD
#undef TWO_THIRD

/* ---- fp32 twin (bitwise the HIP fp32 kernel) ---- */
#define REAL float
#define FN(x) x##_f32
#define RC(x) ((float)(x))
#define UNAN FLT_MAX
#define SQRT sqrtf
#define FABS fabsf
#define THIRD (1.0f / 3.0f)
#define TWO_THIRD (2.0f / 3.0f)
#define STABLE_UPDATE 1
#include "fsm_impl.inc"
#undef REAL
#undef FN
#undef RC
#undef UNAN
#undef SQRT
#undef FABS
#undef THIRD
#undef TWO_THIRD
#undef STABLE_UPDATE

/* Batched fp64 solves for the CPU baseline: one (model, station) solve per
 * OpenMP thread, no nested parallelism -- the reference's table-parallel design
 * (mpiutils.f90:147-149: one serial solve per rank in inter_table_comm). */
int oracle_batch_solve_f64(int nsolve, int maxit, int nx, int ny, int nz, double tol,
                           double h, double x0, double y0, double z0,
                           const double *xs, const double *ys, const double *zs,
                           const double *slow, const int *slow_index, double *u_out,
                           int keep_fields, int nthreads)
{
    size_t n = (size_t)nx * ny * nz;
    int nerr = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : nerr)
#endif
    for (int s = 0; s < nsolve; s++) {
        double ts = 0.0;
        double *u = keep_fields ? u_out + (size_t)s * n : (double *)malloc(n * sizeof(double));
        const double *sl = slow + (size_t)slow_index[s] * n;
        int it;
        nerr += oracle_eikonal3d_solve_f64(maxit, 1, nx, ny, nz, tol, h, x0, y0, z0,
                                           &ts, &xs[s], &ys[s], &zs[s], sl, u, &it) != 0;
        if (!keep_fields) { u_out[s] = u[0]; free(u); }
    }
    return nerr;
}

/* ---------------- L2 misfit (locate.c:923-1047) ---------------- */
int oracle_locate_l2_gridsearch_f64(int ldgrd, int ngrd, int nobs, int iwantOT, double t0use,
                                    const int *mask, const double *tobs, const double *tcorr,
                                    const double *varobs, const double *test,
                                    double *t0, double *objfn)
{
    if (ldgrd < ngrd || nobs < 1 || !mask || !tobs || !varobs || !test || !t0 || !objfn)
        return 1;
    for (int g = 0; g < ngrd; g++) objfn[g] = 0.0;
    int *use = (int *)malloc(sizeof(int) * nobs);
    double *tc = (double *)malloc(sizeof(double) * nobs), *wt = (double *)malloc(sizeof(double) * nobs);
    int nuse = 0;
    double xnorm = 0.0;
    for (int i = 0; i < nobs; i++) {
        if (mask[i] != 0) continue;
        tc[nuse] = tcorr ? tobs[i] - tcorr[i] : tobs[i];
        use[nuse] = i;
        wt[nuse] = 1.0 / varobs[i];
        xnorm = xnorm + wt[nuse];
        nuse++;
    }
    if (iwantOT == 1) {
        for (int g = 0; g < ngrd; g++) t0[g] = 0.0;
        for (int j = 0; j < nuse; j++) {
            double w = wt[j] / xnorm, to = tc[j];
            const double *te = test + (size_t)ldgrd * use[j];
            for (int g = 0; g < ngrd; g++) t0[g] = t0[g] + w * (to - te[g]);
        }
    } else {
        for (int g = 0; g < ngrd; g++) t0[g] = t0use;
    }
    const double sqrt2i = 0.7071067811865475;
    for (int j = 0; j < nuse; j++) {
        double w = wt[j] * sqrt2i, to = tc[j];
        const double *te = test + (size_t)ldgrd * use[j];
        for (int g = 0; g < ngrd; g++) {
            double res = w * (to - (te[g] + t0[g]));
            objfn[g] = objfn[g] + res * res;
        }
    }
    free(use); free(tc); free(wt);
    return 0;
}

/* locate_l2_gridSearch__float64 (locate.c:1079-1203): the same loops in fp32
 * (the reference's float accumulations, 1.0f/var, sqrt2i as a float). */
int oracle_locate_l2_gridsearch_f32(int ldgrd, int ngrd, int nobs, int iwantOT, float t0use,
                                    const int *mask, const float *tobs, const float *tcorr,
                                    const float *varobs, const float *test,
                                    float *t0, float *objfn)
{
    if (ldgrd < ngrd || nobs < 1 || !mask || !tobs || !varobs || !test || !t0 || !objfn)
        return 1;
    for (int g = 0; g < ngrd; g++) objfn[g] = 0.0f;
    int *use = (int *)malloc(sizeof(int) * nobs);
    float *tc = (float *)malloc(sizeof(float) * nobs), *wt = (float *)malloc(sizeof(float) * nobs);
    int nuse = 0;
    float xnorm = 0.0f;
    for (int i = 0; i < nobs; i++) {
        if (mask[i] != 0) continue;
        tc[nuse] = tcorr ? tobs[i] - tcorr[i] : tobs[i];
        use[nuse] = i;
        wt[nuse] = 1.0f / varobs[i];
        xnorm = xnorm + wt[nuse];
        nuse++;
    }
    if (iwantOT == 1) {
        for (int g = 0; g < ngrd; g++) t0[g] = 0.0f;
        for (int j = 0; j < nuse; j++) {
            float w = wt[j] / xnorm, to = tc[j];
            const float *te = test + (size_t)ldgrd * use[j];
            for (int g = 0; g < ngrd; g++) t0[g] = t0[g] + w * (to - te[g]);
        }
    } else {
        for (int g = 0; g < ngrd; g++) t0[g] = t0use;
    }
    const float sqrt2i = 0.7071067811865475f;
    for (int j = 0; j < nuse; j++) {
        float w = wt[j] * sqrt2i, to = tc[j];
        const float *te = test + (size_t)ldgrd * use[j];
        for (int g = 0; g < ngrd; g++) {
            float res = w * (to - (te[g] + t0[g]));
            objfn[g] = objfn[g] + res * res;
        }
    }
    free(use); free(tc); free(wt);
    return 0;
}

/* Fortran variant (gridsearch.f90:382-456): t0 weight 1/(var_i * sum var),
 * logPDF weight sqrt(1/2)/var_i.  Returns the 0-based argmin (MINLOC). */
int oracle_gridsearch_f90_f64(int ldgrd, int ngrd, int nobs, int iwantOT, const int *mask,
                              const double *tobs, const double *varobs, const double *test,
                              double *logpdf, double *t0_at_opt)
{
    double *t0 = (double *)calloc((size_t)ngrd, sizeof(double));
    for (int g = 0; g < ngrd; g++) logpdf[g] = 0.0;
    if (iwantOT == 1) {
        double xnorm = 0.0;
        for (int i = 0; i < nobs; i++) if (mask[i] != 1) xnorm = xnorm + varobs[i];
        for (int i = 0; i < nobs; i++) {
            if (mask[i] == 1) continue;
            double wt = 1.0 / (varobs[i] * xnorm), to = tobs[i];
            const double *te = test + (size_t)ldgrd * i;
            for (int g = 0; g < ngrd; g++) t0[g] = t0[g] + wt * (to - te[g]);
        }
    }
    const double sqrt2i = 1.0 / sqrt(2.0);
    for (int i = 0; i < nobs; i++) {
        if (mask[i] == 1) continue;
        double wt = sqrt2i / varobs[i], to = tobs[i];
        const double *te = test + (size_t)ldgrd * i;
        for (int g = 0; g < ngrd; g++) {
            double res = wt * (to - (te[g] + t0[g]));
            logpdf[g] = logpdf[g] + res * res;
        }
    }
    int iopt = 0;
    for (int g = 1; g < ngrd; g++) if (logpdf[g] < logpdf[iopt]) iopt = g;
    if (t0_at_opt) *t0_at_opt = t0[iopt];
    free(t0);
    return iopt;
}

/* ---------------- MCMC restatement (build-defined) ---------- */
void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Natural log from IEEE +,-,*,/ only, so host and device agree bit for bit
 * (both compiled with -ffp-contract=off).  Domain: finite x > 0. */
double oracle_det_log(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    b = (b & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m;
    memcpy(&m, &b, 8);
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 1.0 / 25.0;
    p = p * s2 + 1.0 / 23.0; p = p * s2 + 1.0 / 21.0; p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0; p = p * s2 + 1.0 / 15.0; p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0; p = p * s2 + 1.0 / 9.0;  p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;  p = p * s2 + 1.0 / 3.0;  p = p * s2 + 1.0;
    double de = (double)e;
    return de * 6.93147180369123816490e-01 + (2.0 * s * p + de * 1.90821492927058770002e-10);
}

typedef struct {
    int nx, ny, nz, nrx, nry, nrz, ncx, ncy, ncz, maxit;
    double h, x0, y0, z0, tol;
    int nstat, nevents;
    const double *sx, *sy, *sz;   /* station coordinates = eikonal sources */
    const int *ev_node;           /* event nearest-node linear index (x fastest) */
    const int *obs_ptr;           /* CSR [nevents+1], 0-based */
    const int *obs_stat;          /* 0-based station of each observation */
    const int *obs_mask;          /* 1 = excluded (locate.c:981-1013 mask) */
    const double *tobs, *tcorr, *var;
    int vmin, vmax, dvmax;
    uint32_t seed;
    const float *ev_frac;         /* NULL, or trilinear mode: [nevents][3] fractions, ev_node = cell corner */
    int nphase;                   /* velocity models per chain: 1 = P, 2 = P and S (homog.c:208-258) */
    int vsmin, vsmax;             /* S prior (nphase 2) */
    const int *obs_phase;         /* NULL (all P) or [nobs] 0 = P, 1 = S: the model an observation fits */
    const unsigned char *skip;    /* NULL or [nphase][nstat]: no table for (phase, station) -- the station
                                     has no picks of that phase (lhasP / lhasS, homog.c:313-335); its
                                     table row is FLT_MAX (the sampler's rule, mceik_fsm_batch.skip) */
    int prec;                     /* 64: the fp64 sampler (--precision 64): per-cell fp32 slowness 1/(float)v
                                     promoted to fp64, the literal fp64 solve (bitwise the reference on the
                                     goldens), tables (float)u; otherwise the fp32 twin */
} oracle_mcmc_problem;

/* Travel time of an event from a solved fp32 field u (x fastest).  w == NULL:
 * the node value (the reference's nearest-node snapping, fsm3d.f90:697-711).
 * Else the build's trilinear mode (no reference counterpart, parity unpinned
 * by the reference): corners clamped to the grid, x then y then z, each lerp
 * a + w*(b - a) in fp32 (this file is compiled without contraction), the
 * GPU's event_time (mceik_amd/csrc/fsm_device.h) operation for operation. */
float oracle_event_time(const float *u, int nx, int ny, int nz, int node, const float *w)
{
    if (!w) return u[node];
    int nxy = nx * ny, z = node / nxy, y = (node - z * nxy) / nx, x = node - z * nxy - y * nx;
    int x1 = x + 1 < nx ? x + 1 : nx - 1, y1 = y + 1 < ny ? y + 1 : ny - 1, z1 = z + 1 < nz ? z + 1 : nz - 1;
    float c[8], a[4];
    for (int k = 0; k < 8; k++)
        c[k] = u[(size_t)((k & 4) ? z1 : z) * nxy + (size_t)((k & 2) ? y1 : y) * nx + ((k & 1) ? x1 : x)];
    for (int k = 0; k < 4; k++) {
        float d = c[2 * k + 1] - c[2 * k];
        float m = w[0] * d;
        a[k] = c[2 * k] + m;
    }
    float d0 = a[1] - a[0], m0 = w[1] * d0, b0 = a[0] + m0;
    float d1 = a[3] - a[2], m1 = w[1] * d1, b1 = a[2] + m1;
    float d2 = b1 - b0, m2 = w[2] * d2;
    return b0 + m2;
}

void oracle_expand_slowness(const oracle_mcmc_problem *p, const int *v, float *slow)
{
    for (int iz = 0; iz < p->nz; iz++)
        for (int iy = 0; iy < p->ny; iy++)
            for (int ix = 0; ix < p->nx; ix++) {
                int c = ((iz / p->nrz) * p->ncy + iy / p->nry) * p->ncx + ix / p->nrx;
                slow[((size_t)iz * p->ny + iy) * p->nx + ix] = 1.0f / (float)v[c];
            }
}

/* travel-time table [station][event] (fp32) of phase ph's velocity model */
static int oracle_forward_phase_f32(const oracle_mcmc_problem *p, int ph, const int *v, float *ttab, int *niter);

int oracle_forward_f32(const oracle_mcmc_problem *p, const int *v, float *ttab, int *niter)
{
    return oracle_forward_phase_f32(p, 0, v, ttab, niter);
}

int oracle_forward_s_f32(const oracle_mcmc_problem *p, const int *v, float *ttab, int *niter)
{
    return oracle_forward_phase_f32(p, 1, v, ttab, niter);
}

static int oracle_forward_phase_f32(const oracle_mcmc_problem *p, int ph, const int *v, float *ttab, int *niter)
{
    size_t n = (size_t)p->nx * p->ny * p->nz;
    float *slow = (float *)malloc(n * sizeof(float));
    oracle_expand_slowness(p, v, slow);
    int nerr = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : nerr)
#endif
    for (int s = 0; s < p->nstat; s++) {
        if (p->skip && p->skip[(size_t)ph * p->nstat + s]) {
            if (niter) niter[s] = 0;
            for (int e = 0; e < p->nevents; e++) ttab[(size_t)s * p->nevents + e] = FLT_MAX;
            continue;
        }
        float *u = (float *)malloc(n * sizeof(float));
        double ts = 0.0;
        int it = 0;
        if (p->prec == 64) {
            double *s64 = (double *)malloc(n * sizeof(double)), *u64 = (double *)malloc(n * sizeof(double));
            for (size_t i = 0; i < n; i++) s64[i] = (double)slow[i];
            nerr += oracle_eikonal3d_solve_f64(p->maxit, 1, p->nx, p->ny, p->nz, p->tol, p->h,
                                               p->x0, p->y0, p->z0, &ts, &p->sx[s], &p->sy[s],
                                               &p->sz[s], s64, u64, &it) != 0;
            for (size_t i = 0; i < n; i++) u[i] = (float)u64[i];    /* the GPU's table export, fsm_device.h event_time */
            free(s64); free(u64);
        } else {
            nerr += oracle_eikonal3d_solve_f32(p->maxit, 1, p->nx, p->ny, p->nz, p->tol, p->h,
                                               p->x0, p->y0, p->z0, &ts, &p->sx[s], &p->sy[s],
                                               &p->sz[s], slow, u, &it) != 0;
        }
        if (niter) niter[s] = it;
        for (int e = 0; e < p->nevents; e++)
            ttab[(size_t)s * p->nevents + e] = oracle_event_time(u, p->nx, p->ny, p->nz, p->ev_node[e],
                                                                 p->ev_frac ? p->ev_frac + 3 * e : NULL);
        free(u);
    }
    free(slow);
    return nerr;
}

/* logL = -sum_e objfn_e, objfn_e = locate.c L2 with analytic t0 at the
 * event's node (one grid point, iwantOT = 1), observations in CSR order.
 * ttab [phase][station][event]: an observation of phase ph (obs_phase, P if
 * NULL) is fit against model ph's table of its station -- the locator stacks
 * P and S picks alike (locate.f90:399,442; the build's definition, DESIGN s.4). */
double oracle_loglik(const oracle_mcmc_problem *p, const float *ttab)
{
    double logl = 0.0;
    const double sqrt2i = 0.7071067811865475;
    const size_t per = (size_t)p->nstat * p->nevents;
    for (int e = 0; e < p->nevents; e++) {
        int j0 = p->obs_ptr[e], j1 = p->obs_ptr[e + 1];
        double xnorm = 0.0, t0 = 0.0, obj = 0.0;
        for (int j = j0; j < j1; j++) if (!p->obs_mask[j]) xnorm = xnorm + 1.0 / p->var[j];
        for (int j = j0; j < j1; j++) {
            if (p->obs_mask[j]) continue;
            const int ph = p->obs_phase ? p->obs_phase[j] : 0;
            double te = (double)ttab[ph * per + (size_t)p->obs_stat[j] * p->nevents + e];
            double tc = p->tobs[j] - p->tcorr[j];
            t0 = t0 + ((1.0 / p->var[j]) / xnorm) * (tc - te);
        }
        for (int j = j0; j < j1; j++) {
            if (p->obs_mask[j]) continue;
            const int ph = p->obs_phase ? p->obs_phase[j] : 0;
            double te = (double)ttab[ph * per + (size_t)p->obs_stat[j] * p->nevents + e];
            double tc = p->tobs[j] - p->tcorr[j];
            double res = ((1.0 / p->var[j]) * sqrt2i) * (tc - (te + t0));
            obj = obj + res * res;
        }
        logl = logl - obj;
    }
    return logl;
}

static int oracle_nphase(const oracle_mcmc_problem *p) { return p->nphase > 1 ? p->nphase : 1; }

/* Proposal (build definition): one cell of the chain's nphase models, drawn
 * over [0, nphase*ncell) (cell / ncell = the model: 0 P, 1 S), moves by
 * +-[1, dvmax]; v is the chain's [nphase][ncell]. */
void oracle_propose(const oracle_mcmc_problem *p, uint32_t chain, uint64_t step,
                    const int *v, int *cell, int *vnew, int *in_prior, double *logu)
{
    uint32_t ctr[4] = {(uint32_t)step, (uint32_t)(step >> 32), 0u, 0u}, key[2] = {chain, p->seed}, r[4];
    oracle_philox4x32_10(ctr, key, r);
    uint32_t ncell = (uint32_t)(p->ncx * p->ncy * p->ncz);
    uint32_t ncm = ncell * (uint32_t)oracle_nphase(p);
    int c = (int)(((uint64_t)r[0] * ncm) >> 32);
    int mag = 1 + (int)(((uint64_t)r[1] * (uint32_t)p->dvmax) >> 32);
    int vn = v[c] + ((r[2] & 1u) ? -mag : mag);
    int sph = c >= (int)ncell;
    *cell = c; *vnew = vn;
    *in_prior = sph ? (vn >= p->vsmin && vn <= p->vsmax) : (vn >= p->vmin && vn <= p->vmax);
    *logu = oracle_det_log(((double)r[3] + 0.5) * (1.0 / 4294967296.0));
}

/* Tables [phase][station][event] of every model of one chain (v [nphase][ncell]). */
int oracle_forward_all_f32(const oracle_mcmc_problem *p, const int *v, float *ttab)
{
    const size_t ncell = (size_t)p->ncx * p->ncy * p->ncz, per = (size_t)p->nstat * p->nevents;
    int nerr = 0;
    for (int ph = 0; ph < oracle_nphase(p); ph++) nerr += oracle_forward_phase_f32(p, ph, v + ph * ncell, ttab + ph * per, NULL);
    return nerr;
}

/* Runs nsteps Metropolis steps for nchains chains (global ids gid0..); v is
 * [nchains][nphase][ncell] in/out, logl [nchains] in/out; accept
 * [nsteps][nchains].  Every proposal's logL comes from a forward of all of
 * the chain's models (the GPU re-solves only the changed one). */
void oracle_mcmc_run(const oracle_mcmc_problem *p, int nchains, uint32_t gid0, uint64_t step0,
                     int nsteps, int *v, double *logl, unsigned char *accept, double *logl_trace)
{
    size_t ncm = (size_t)p->ncx * p->ncy * p->ncz * oracle_nphase(p);
    int *vp = (int *)malloc(ncm * sizeof(int));
    float *tt = (float *)malloc(sizeof(float) * p->nstat * p->nevents * oracle_nphase(p));
    for (int st = 0; st < nsteps; st++) {
        for (int c = 0; c < nchains; c++) {
            int *vc = v + (size_t)c * ncm;
            int cell, vn, inp;
            double logu;
            oracle_propose(p, gid0 + (uint32_t)c, step0 + (uint64_t)st, vc, &cell, &vn, &inp, &logu);
            double ln = -HUGE_VAL;
            if (inp) {          /* outside the prior: rejected without a forward */
                memcpy(vp, vc, ncm * sizeof(int));
                vp[cell] = vn;
                oracle_forward_all_f32(p, vp, tt);
                ln = oracle_loglik(p, tt);
            }
            int acc = inp && (logu < ln - logl[c]);
            if (acc) { vc[cell] = vn; logl[c] = ln; }
            accept[(size_t)st * nchains + c] = (unsigned char)acc;
            if (logl_trace) logl_trace[(size_t)st * nchains + c] = logl[c];
        }
    }
    free(vp); free(tt);
}

/* EIKONAL3D_SOLVE of the MPI variant (fsm3d.f90:1754-1852) on an ndivx x
 * ndivy x ndivz block decomposition, every block in this process:
 * EIKONAL3D_GHOST_COMM's blocks (fsm3d.f90:1086-1101: nd = max(n/ndiv, 1),
 * block b owns [nd*b, nd*(b+1)-1], the last block up to n-1; a ghost layer of
 * width noverlap), EIKONAL3D_FSM_MPI's loop (:103-222): per sweep every block
 * runs its own Gauss-Seidel sweep over its nodes (ghosts and BC nodes are not
 * updated) reading ghost values as they were at the sweep's start, then
 * EIKONAL_EXCHANGE (:971-1046) refreshes the ghosts; with noverlap = 0 a block
 * face is a grid edge (GET_U*MIN3D's one-sided rule).  Convergence: every
 * owned node |u0-u| < tol.  ierr: the last EVAL_UPDATE3D of rank 0 (block
 * (0,0,0)): the update ierr of node (1,1,1) in the iteration's last sweep.
 * Pinned against the reference's own MPI runs (tests/golden/blocks_mpi.npz). */
int oracle_eikonal3d_solve_blocks_f64(int maxit, int nsrc, int nx, int ny, int nz, int ndivx, int ndivy,
                                      int ndivz, int noverlap, double tol, double h, double x0, double y0,
                                      double z0, const double *ts, const double *xs, const double *ys,
                                      const double *zs, const double *slow, double *u, int *niter_out)
{
    static const int sweeps[8][3] = {{0,0,0},{1,0,0},{0,1,0},{1,1,0},{0,0,1},{1,0,1},{0,1,1},{1,1,1}};
    const int nn[3] = {nx, ny, nz}, nd[3] = {ndivx, ndivy, ndivz};
    int step[3];
    for (int a = 0; a < 3; a++) step[a] = nn[a] / nd[a] > 1 ? nn[a] / nd[a] : 1;
    size_t n = (size_t)nx * ny * nz, nxy = (size_t)nx * ny;
    unsigned char *lisbc = (unsigned char *)malloc(n);
    if (niter_out) *niter_out = 0;
    int ierr = setbcs_f64(nx, ny, nz, nsrc, h, x0, y0, z0, ts, xs, ys, zs, slow, lisbc, u);
    if (ierr) { free(lisbc); return ierr; }
    double *u0 = (double *)malloc(n * sizeof(double)), *snap = (double *)malloc(n * sizeof(double));
    memcpy(u0, u, n * sizeof(double));
    int k;
    for (k = 1; k <= maxit; k++) {
        for (int sw = 0; sw < 8; sw++) {
            memcpy(snap, u, n * sizeof(double));
            for (int bz = 0; bz < ndivz; bz++)
            for (int by = 0; by < ndivy; by++)
            for (int bx = 0; bx < ndivx; bx++) {
                const int b[3] = {bx, by, bz};
                int lo[3], hi[3];
                for (int a = 0; a < 3; a++) {
                    lo[a] = step[a] * b[a];
                    hi[a] = b[a] + 1 == nd[a] ? nn[a] - 1 : step[a] * (b[a] + 1) - 1;
                }
                int last_ierr = 0;
                for (int kz = 0; kz <= hi[2] - lo[2]; kz++) {
                    int iz = sweeps[sw][2] ? hi[2] - kz : lo[2] + kz;
                    for (int ky = 0; ky <= hi[1] - lo[1]; ky++) {
                        int iy = sweeps[sw][1] ? hi[1] - ky : lo[1] + ky;
                        for (int kx = 0; kx <= hi[0] - lo[0]; kx++) {
                            int ix = sweeps[sw][0] ? hi[0] - kx : lo[0] + kx;
                            size_t ijk = (size_t)iz * nxy + (size_t)iy * nx + ix;
                            last_ierr = 0;
                            if (lisbc[ijk]) continue;
                            double self = u[ijk], f = slow[ijk] * h;
                            /* neighbour: outside the grid -> self; inside this block -> live;
                               another block's node -> the ghost (start of sweep), or self
                               without a ghost layer */
#define NB(cond_in, inblk, off) (!(cond_in) ? self : (inblk) ? u[ijk + (off)] : (noverlap > 0 ? snap[ijk + (off)] : self))
                            double xm = NB(ix > 0, ix - 1 >= lo[0], -1), xp = NB(ix < nx - 1, ix + 1 <= hi[0], 1);
                            double ym = NB(iy > 0, iy - 1 >= lo[1], -(long)nx), yp = NB(iy < ny - 1, iy + 1 <= hi[1], (long)nx);
                            double zm = NB(iz > 0, iz - 1 >= lo[2], -(long)nxy), zp = NB(iz < nz - 1, iz + 1 <= hi[2], (long)nxy);
#undef NB
                            double ux = xm < xp ? xm : xp, uy = ym < yp ? ym : yp, uz = zm < zp ? zm : zp;
                            int e1;
                            double ub = solve3d_f64(ux, uy, uz, f, &e1);
                            last_ierr = e1;
                            u[ijk] = self < ub ? self : ub;
                        }
                    }
                }
                if (bx == 0 && by == 0 && bz == 0) ierr = last_ierr;
            }
        }
        size_t lconv = 0;
        for (size_t i = 0; i < n; i++) {
            if (fabs(u0[i] - u[i]) < tol) lconv++;
            u0[i] = u[i];
        }
        if (lconv == n) break;
    }
    if (niter_out) *niter_out = (k > maxit ? maxit : k);
    free(u0); free(snap); free(lisbc);
    return ierr;
}
