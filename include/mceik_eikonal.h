/*
 * mceik_eikonal.h -- eikonal / misfit entry points of libmceik_hip.so (gfx950).
 *
 * The first group is a drop-in for the reference's Fortran BIND(C) symbols:
 * same names, every argument by pointer, caller-owned host arrays, ierr out.
 * The batched group is new: device pointers, many solves per launch.
 */
#ifndef MCEIK_EIKONAL_H_AMD
#define MCEIK_EIKONAL_H_AMD 1
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces EIKONAL3D_SERIAL_DRIVER (fsm3d.f90:1968-2052).
 * job 1: initialise (ierr=1 if already initialised); job 2: solve (ierr=1 if
 * not initialised; ierr from SETBCS / FSM as the reference); other: finalise.
 * Computes on the GPU in fp64 with the reference's arithmetic: u is bitwise
 * equal to the reference's output.  slow, u: [nx*ny*nz], x fastest.  Job 1
 * allocates the device state (freed by the finalising call); one solve runs
 * on the whole GPU (brick-level dataflow).  Any number of
 * sources. */
void eikonal3d_serial_driver(const int *job, const int *iverb, const int *maxit, const int *nsrc,
                             const int *nx, const int *ny, const int *nz, const double *tol,
                             const double *h, const double *x0, const double *y0, const double *z0,
                             const double *ts, const double *xs, const double *ys, const double *zs,
                             const double *slow, double *u, int *ierr);

/* Same contract computed in fp32 with the cancellation-free update
 * (DESIGN.md s.5): |u - u_ref| <= 1e-6 u_ref + 1e-7 s. */
void eikonal3d_serial_driver_sp(const int *job, const int *iverb, const int *maxit, const int *nsrc,
                                const int *nx, const int *ny, const int *nz, const double *tol,
                                const double *h, const double *x0, const double *y0, const double *z0,
                                const double *ts, const double *xs, const double *ys, const double *zs,
                                const double *slow, double *u, int *ierr);

/* Replaces the MPI variant EIKONAL3D_INITIALIZE / _SOLVE / _FINALIZE
 * (fsm3d.f90:1583-1598, 1754-1769, 1891-1899), every argument by pointer.
 * Collective over comm (MPI resolved at run time; no MPI = one rank): rank
 * 0's parameters and SETBCS error reach every rank.  The decomposition is
 * honoured: ndivx x ndivy x ndivz blocks (noverlap: ghost layer width, 0 =
 * block faces act as grid edges) run the reference's block-decomposed FSM
 * (EIKONAL3D_FSM_MPI: each block sweeps its nodes against ghost copies
 * refreshed after every sweep), so u and ierr are bitwise the reference's run
 * with one MPI rank per block; one block = the serial driver's solve.  With
 * as many ranks in comm as blocks (the reference's layout) every rank holds
 * only its block and the ghost layer on its GPU, sweeps the block and swaps
 * face layers with its neighbours after every sweep (host-staged MPI; MCEIK_HALO=rccl moves them device to
 * device over RCCL when each rank has a GPU of its own, unpinned), and the master gathers u; otherwise
 * the master's GPU runs every block.  The master passes the full arrays
 * (n = nx*ny*nz) and receives u; the other ranks pass n = 1 as the
 * reference's callers do and keep their u.  fp64 (xfsm3d: max u =
 * 1.4308203212738235). */
void eikonal3d_initialize(const int *comm, const int *iverb, const int *nx, const int *ny, const int *nz,
                          const int *ndivx, const int *ndivy, const int *ndivz, const int *noverlap,
                          const int *maxit, const double *x0, const double *y0, const double *z0,
                          const double *h, const double *tol, int *ierr);
void eikonal3d_solve(const int *comm, const int *nsrc, const int *n, const double *ts, const double *xs,
                     const double *ys, const double *zs, const double *slow, double *u, int *ierr);
void eikonal3d_finalize(const int *comm, int *ierr);

/* Replaces locate3d_gridsearch__double64 / __float64 (gridsearch.f90:382-540),
 * the Fortran misfit variant (t0 weight 1/(var_i * sum var), logPDF weight
 * sqrt(1/2)/var_i; SURVEY s.8a a12): same arguments by pointer, checks
 * (ldgrd % 64, ngrd <= ldgrd, some unmasked observation, sum var != 0) and
 * arithmetic order; host arrays, test [nobs][ldgrd]. */
void locate3d_gridsearch__double64(const int *ldgrd, const int *ngrd, const int *nobs, const int *iwantOT,
                                   const int *mask, const double *tobs, const double *varobs, const double *test,
                                   double *logPDF, int *ierr);
void locate3d_gridsearch__float64(const int *ldgrd, const int *ngrd, const int *nobs, const int *iwantOT,
                                  const int *mask, const float *tobs, const float *varobs, const float *test,
                                  float *logPDF, int *ierr);

/* Replaces locate_l2_gridSearch__double64 (locate.c:923-1047): same
 * arguments, errors and results (bitwise); host arrays, computed on the GPU.
 * test: [nobs][ldgrd]; tcorr may be NULL. */
int locate_l2_gridSearch__double64(int ldgrd, int ngrd, int nobs, int iwantOT, double t0use,
                                   const int *mask, const double *tobs, const double *tcorr,
                                   const double *varobs, const double *test,
                                   double *t0, double *objfn);

/* Replaces locate_l2_gridSearch__float64 (locate.c:1079-1203): the fp32
 * variant, same arguments, checks and arithmetic order; host arrays. */
int locate_l2_gridSearch__float64(int ldgrd, int ngrd, int nobs, int iwantOT, float t0use,
                                  const int *mask, const float *tobs, const float *tcorr,
                                  const float *varobs, const float *test, float *t0, float *objfn);

/* ---- relocation grid search over many events (device memory) ---------- */
/* For every event e and grid point g: the locate.c L2 objective with the
 * analytic origin time (fp32, locate_l2_gridSearch__float64 arithmetic) of
 * event e's observations against shared travel-time tables.  Observations
 * are compacted per event (masked ones removed, reference order): event e
 * owns [ev_ptr[e], ev_ptr[e+1]); obs_row[j] is the row of `tables` (e.g. the
 * station), tc[j] = tobs - tcorr, wt[j] = 1/var, xnorm[e] = sum of wt in
 * order.  out[e*ldgrd + g] = objfn, or -objfn (log joint PDF up to a
 * constant) when log_pdf != 0; t0 (may be NULL) the same layout. */
typedef struct mceik_relocate_batch {
    int ldgrd, ngrd, nev, iwantOT;
    float t0use;
    const float *tables;        /* device [nrows][ldgrd]                     */
    const int *ev_ptr;          /* device [nev+1]                            */
    const int *obs_row;         /* device [ev_ptr[nev]]                      */
    const float *tc, *wt;       /* device [ev_ptr[nev]]                      */
    const float *xnorm;         /* device [nev]                              */
    float *t0;                  /* device [nev][ldgrd] or NULL               */
    float *out;                 /* device [nev][ldgrd]                       */
    int log_pdf;
    int nrows;                  /* rows of `tables` (> every obs_row) and nobs = ev_ptr[nev] on the
                                   host: single-pass kernel (each table value read once per launch,
                                   LDS-staged; if ev_ptr[nev] != nobs or an obs_row >= nrows every
                                   output is NaN); 0 = unknown, two passes per event from HBM */
    int nobs;
} mceik_relocate_batch;
int mceik_relocate(const mceik_relocate_batch *b, void *stream);

/* ---- batched solves on device memory ---------------------------------- */
typedef struct mceik_fsm_batch {
    int nx, ny, nz;             /* grid nodes, dx = dy = dz = h              */
    double h, x0, y0, z0;
    int maxit;
    double tol;
    int precision;              /* 32 or 64                                  */
    int nmodel, nstat, nsrc;    /* solves = nmodel * nstat                   */
    const double *src;          /* device [nstat][nsrc][4] = (ts, xs, ys, zs) */
    int slow_mode;              /* 0: per-node field, 1: inversion grid      */
    const void *slow;           /* mode 0: device [nmodel][nx*ny*nz] (fp32/fp64 as precision,
                                   x fastest); mode 1: device float [nmodel][ncell] */
    int nrx, nry, nrz;          /* mode 1: refinement (cell = node / nr)     */
    int nev;                    /* events to sample (0: none)                */
    const int *ev_node;         /* device [nev], x-fastest node index         */
    float *ttab;                /* device [nmodel*nstat][nev]                */
    void *u_out;                /* device [nmodel*nstat][nx*ny*nz] or NULL   */
    int *niter, *ierr;          /* device [nmodel*nstat] or NULL             */
    int max_sweeps;             /* < 0: unlimited (debug)                    */
    unsigned long long *iter_total;  /* device counter += iterations of every solve, or NULL */
    int fast_sqrt;              /* 1: caller guarantees h*slowness >= 1e-12 (cells mode, fp32 AND
                                   fp64): fp32 uses the shorter correctly rounded sqrt, fp64 the
                                   sqrt expansion without input scaling (both exact only for normal
                                   radicands, hence the contract; same results within it).  0: the
                                   full-range sqrt */
    unsigned long long *visit_stats; /* device [4] += brick visits (8x8x8 nodes, one sweep; z-blocks
                                        whose inputs did not change are skipped), column segments
                                        (8 nodes) updated, segments that changed, macro steps of the
                                        sweep waves (one 64-lane step; 16 or 8 z per lane); or NULL */
    const int *solve_order;     /* device [nmodel*nstat]: work-queue slot -> solve id (a permutation;
                                   only the order solves start in changes), or NULL = model-major */
    unsigned long long *solve_clock; /* device [nmodel*nstat][2]: s_memrealtime (100 MHz) at the
                                        start and end of each solve (diagnostic), or NULL */
    int max_waves;              /* cap on the resident solve waves (0 = occupancy x CUs); with fewer
                                   waves than solves each wave runs several solves in its reused
                                   scratch field (the production path at C2/C3) */
    unsigned long long *traffic;/* device [8] += requested global-memory bytes by category (own segment
                                   loads, halo loads, z-upwind loads, own stores, u0 stores, cell loads,
                                   convergence-check loads, init fill + table gather); counted only by
                                   an accounting build (-DMCEIK_TRAFFIC), else untouched; or NULL */
    int step_z;                 /* z nodes per macro step of the sweep kernel: 0 = the launch's choice
                                   (16 for the fp32 cell-cache instance, else 8), 8 = force the 8-z
                                   kernel (A/B measurements, parity tests); results are identical */
    const float *ev_frac;       /* device [nev][3] (wx, wy, wz) in [0, 1], or NULL.  NULL: ttab holds the
                                   value at node ev_node (the reference's nearest-node snapping,
                                   fsm3d.f90:697-711).  Else trilinear interpolation in the cell whose
                                   lowest corner is ev_node (fp32, x then y then z, a + w*(b - a)) */
    const int *model_phase;     /* slow_mode 1: device [nmodel] or NULL.  Non-NULL: model m solves the
                                   slowness slow[(m*nphase + model_phase[m])*ncell ...] -- one of the
                                   nphase models (P, S) a sampler chain holds; NULL: slow[m*ncell ...] */
    int nphase;                 /* models per entry of `slow` when model_phase != NULL (1 or 2) */
    const unsigned char *skip;  /* device [nphase][nstat] or NULL: solve (m, s) of phase ph (model_phase[m];
                                   without a phase map m % nphase, i.e. models [chain][phase]) is skipped when skip[ph*nstat + s] != 0 -- a
                                   station with no picks of that phase (mceik_stations_struct lhasP /
                                   lhasS; homog.c:313-335 builds tables only for flagged stations): no
                                   sweep, niter 0, ierr 0, its ttab row FLT_MAX (the unreached value).
                                   Refused together with u_out (a skipped solve has no field) */
    unsigned long long *solve_count; /* device counter += solves executed (not skipped), or NULL */
} mceik_fsm_batch;

/* The batched extension of SURVEY s.8b with plain arguments: nmodels x
 * nstations single-source solves in one call, fp32 (the sampler's
 * arithmetic: bitwise the fp32 twin, within 1e-6 u + 1e-7 s of the fp64
 * reference).  src [nstations][4] = (ts, xs, ys, zs); slow [nmodels][nx*ny*nz]
 * s/m and u [nmodels*nstations][nx*ny*nz] x fastest, solve m*nstations + s;
 * niter, ierr [nmodels*nstations] or NULL.  Host or device pointers (host
 * arrays are staged); synchronous; allocates per call (use
 * mceik_fsm_batch_solve with a kept workspace for repeated calls).  0 = ok. */
int eikonal3d_batch_solve(int nmodels, int nstations, int nx, int ny, int nz, double h, double x0, double y0,
                          double z0, int maxit, double tol, const double *src, const float *slow, float *u,
                          int *niter, int *ierr);

/* Device workspace (bytes) a launch of this batch needs. */
size_t mceik_fsm_workspace_bytes(const mceik_fsm_batch *b);
/* Enqueue the batch on `stream` (hipStream_t; NULL = default).  No host
 * synchronisation and no allocation: capturable in a hipGraph. 0 = ok. */
int mceik_fsm_batch_solve(const mceik_fsm_batch *b, void *workspace, size_t workspace_bytes,
                          void *stream);

/* z nodes per macro step the launch of this batch runs (8 or 16; diagnostic). */
int mceik_fsm_step_z(const mceik_fsm_batch *b);

/* The kernel instance the launch of this batch runs (the name rocprofv3
 * traces show) and its LDS bytes per wave; host-side, no GPU needed. */
const char *mceik_fsm_kernel_name(const mceik_fsm_batch *b);
size_t mceik_fsm_lds_bytes(const mceik_fsm_batch *b);

/* Algorithmic HBM bytes of one node visit in one sweep (roofline accounting). */
double mceik_fsm_bytes_per_node_sweep(const mceik_fsm_batch *b);

/* Synchronous copy helper for hosts without a device runtime binding
 * (kind: 0 host->device, 1 device->host, 2 device->device). 0 = ok. */
int mceik_memcpy(void *dst, const void *src, size_t bytes, int kind);

#ifdef __cplusplus
}
#endif
#endif
