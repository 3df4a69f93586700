/*
 * mceik_struct.h -- driver data model of the mceik MCMC tomography code.
 *
 * ABI-identical re-declaration of the reference's include/mceik_struct.h:4-90
 * (same type names, member names, member order and types), so a harness built
 * against the reference headers links against libmceik_hip.so unchanged.
 * tests/test_capi.py checks sizeof/offsetof of every struct against the
 * layout the reference header implies.
 */
#ifndef _mceik_struct_h__
#define _mceik_struct_h__ 1   /* the reference's own guard: one definition when both are included */

/* phase of an observation (mceik_struct.h:4-8) */
enum pick_type_enum {
    P_PRIMARY_PICK = 1,
    S_PRIMARY_PICK = 2,
};

/* Event catalogue, observations in CSR by event (mceik_struct.h:10-32).
 * obsPtr[e]..obsPtr[e+1]-1 are event e's observations (0-based); statPtr is
 * 1-based into the station list (homog.c:227). */
struct mceik_catalog_struct {
    double *xsrc, *ysrc, *zsrc;  /* event position (m), z up from model base  */
    double *tori;                /* origin time (s)                          */
    double *tobs;                /* observed pick time (s)                   */
    double *test;                /* estimated pick time (s)                  */
    double *varObs;              /* pick variance (s^2)                      */
    int *luseObs;                /* 0: observation not used                  */
    int *pickType;               /* P_PRIMARY_PICK / S_PRIMARY_PICK           */
    int *statPtr;                /* station of each observation (1-based)    */
    int *obsPtr;                 /* [nevents+1]                              */
    int nevents;
};

/* Receivers (mceik_struct.h:34-49). */
struct mceik_stations_struct {
    char **netw, **stnm, **chan, **loc;
    double *xrec, *yrec, *zrec;  /* position (m)                             */
    double *pcorr, *scorr;       /* static corrections (s)                   */
    int *lhasP, *lhasS;
    int nstat;
    int lcartesian;
};

struct catalog_struct {
    int nevents;
};

/* MCMC controls (mceik_struct.h:54-60). */
struct mcmc_parms_struct {
    char resdir[512];
    int nburnIn;                 /* proposals before samples are kept        */
    int niter;                   /* total proposals (forward problems)       */
    int keepK;                   /* keep every keepK-th state after burn-in  */
};

/* Eikonal controls (mceik_struct.h:62-66). */
struct eik_parms_struct {
    double tol;                  /* convergence tolerance (s)                */
    int maxit;                   /* max sweep iterations                     */
};

/* Global parameters (mceik_struct.h:68-90). */
struct mceik_parms_struct {
    struct mcmc_parms_struct mcparms;
    struct eik_parms_struct eikparms;
    char projnm[128];
    char scratch_dir[512];
    double x0, y0, z0;           /* grid origin (m)                          */
    double dx, dy, dz;           /* grid spacing (m); the solver needs dx=dy=dz */
    int ndivx, ndivy, ndivz;     /* MPI domain divisions (unused on one GPU) */
    int nrefx, nrefy, nrefz;     /* inversion -> eikonal grid refinement     */
};

#endif
