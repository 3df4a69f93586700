/*
 * mceik.h -- MCMC travel-time tomography driver API (libmceik_hip.so, gfx950).
 *
 * The reference's include/mceik.h:1-14 declares nothing; its data model
 * (mceik_struct.h) is kept and this header fills the driver slot that
 * homog.c:343-415 occupies.  One process drives one GPU; an MPI harness
 * passes its rank/size and shards chains.  Every function
 * returns 0 on success (h5io.c convention).
 */
#ifndef _mceik_h__
#define _mceik_h__ 1   /* the reference's guard (include/mceik.h:1-2): this header replaces it */
#include <stdint.h>
/* the reference's mceik.h pulls in <mpi.h> and "os.h" (include/mceik.h:3-4):
 * a harness built with an MPI compiler gets the MPI declarations from here as
 * before; the library itself needs no MPI at build or link time */
#if defined(__has_include)
#if __has_include(<mpi.h>)
#include <mpi.h>
#endif
#endif
#include "os.h"
#include "mceik_struct.h"
#include "mceik_eikonal.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mceik_mcmc mceik_mcmc;   /* opaque per-GPU sampler */

/* Sampler options beyond mceik_parms_struct. */
typedef struct mceik_mcmc_opts {
    int nx, ny, nz;            /* eikonal grid (parms->dx = dy = dz = h)     */
    int nchains;               /* chains on this GPU                         */
    int chain_offset;          /* global id of the first chain (rank shard)  */
    int vmin, vmax;            /* uniform prior on cell velocity (m/s)       */
    int dvmax;                 /* proposal: +-[1, dvmax] m/s on one cell     */
    uint32_t seed;             /* Philox key                                 */
    int max_samples;           /* device sample ring capacity (states)       */
    int device;                /* HIP device ordinal                         */
    int precision;             /* FSM arithmetic: 32 (0 = default) or 64; tables are fp32 at rest
                                  either way (fsm3d.f90:1855-1875)           */
    int max_waves;             /* cap on resident FSM waves (0 = occupancy x CUs) */
    int tt_interp;             /* event travel times: 0 = value at the event's nearest node (the
                                  reference's snapping, fsm3d.f90:697-711); 1 = trilinear
                                  interpolation in the event's grid cell (mceik_fsm_batch.ev_frac) */
    int nphase;                /* velocity models per chain: 1 (or 0) = P only; 2 = joint P and S
                                  (homog.c:208-258 makes both; the catalog's pickType selects the
                                  model an observation is fit against, mceik_struct.h:4-8)   */
    int vsmin, vsmax;          /* nphase 2: uniform prior on S cell velocity (m/s)          */
    int mask_s;                /* nphase 1 and the catalog holds used S picks: 0 = init fails
                                  (naming the count), 1 = fit the P picks and ignore the S picks */
} mceik_mcmc_opts;

/* What mceik_mcmc_init set up (diagnostic; mceik_mcmc_info). */
typedef struct mceik_mcmc_info {
    int npipe;                 /* chain groups on streams of their own (1 = one FSM launch per step) */
    int nphase;                /* velocity models per chain (1 = P, 2 = P and S)              */
    int step_z;                /* z nodes per macro step of the sampler's FSM kernel (16 or 8) */
    int fixed_layout;          /* 1: the compile-time LDS layout instance                   */
    int chains[4];             /* chains of pipe k (k < npipe)                               */
    int waves[4];              /* resident FSM waves of pipe k's launch                     */
    size_t workspace_bytes[4]; /* FSM scratch of pipe k                                     */
    size_t lds_bytes;          /* LDS per FSM wave                                           */
    int masked_s;              /* S observations ignored (nphase 1 with mask_s = 1)          */
    char kernel[64];           /* the FSM kernel instance (rocprof name)                    */
    int multi_step;            /* 1: one FSM launch runs up to 64 steps, no barrier between
                                  them (the chain epilogue in the kernel; default when a step
                                  is <= 4 solves per wave, MCEIK_PERSIST=1/0 forces);
                                  0: per-step propose / FSM / accept launches               */
} mceik_mcmc_info;

/* ---- run configuration (host only; csrc/parms.c) ----------------------
 * The reference's mains hard-code their parameters (homog.c:73-89,
 * fsm3d.f90:2085-2100); these fill mceik_parms_struct (mceik_struct.h:68-90)
 * and the sampler options from an INI file ([general] projnm scratch_dir;
 * [grid] x0 y0 z0 dx dy dz nx ny nz ndivx ndivy ndivz nrefx nrefy nrefz
 * tt_interp; [eikonal] tol maxit precision max_waves; [mcmc] resdir nburnIn
 * niter keepK nchains chain_offset vmin vmax dvmax seed max_samples device),
 * names case-insensitive, ';'/'#' comments.  Either record pointer may be NULL. */
/* homog.c's grid (32 x 29 x 26 nodes at 1 km), tol 1e-8, maxit 50, seed 2016. */
int mceik_parms_defaults(struct mceik_parms_struct *parms, mceik_mcmc_opts *opts);
/* key "section:name": 0 ok, 1 unknown key, 2 invalid value (message on stderr). */
int mceik_parms_set(struct mceik_parms_struct *parms, mceik_mcmc_opts *opts, const char *key, const char *value);
/* 0 ok, -1 cannot open, > 0 the line number of the first bad line. */
int mceik_parms_read(const char *path, struct mceik_parms_struct *parms, mceik_mcmc_opts *opts);
/* Applies [--]section:key=value arguments and --config FILE / --config=FILE
 * (in argument order, argv[0] skipped); returns the count consumed or -1. */
int mceik_parms_args(int argc, char **argv, struct mceik_parms_struct *parms, mceik_mcmc_opts *opts);
/* Writes every key back in INI form (0 ok). */
int mceik_parms_write(const char *path, const struct mceik_parms_struct *parms, const mceik_mcmc_opts *opts);

/* v0: host [nchains][nphase][ncell] int m/s (P model, then S model when
 * nphase = 2), ncell = ceil(nx/nrefx)*ceil(ny/nrefy)*ceil(nz/nrefz), cell
 * index x fastest.  Computes each chain's initial logL.  Stations need
 * Cartesian coordinates (lcartesian = 1); a station gets a P table only when
 * lhasP[k] and an S table only when lhasS[k] is set (NULL arrays: every
 * station), the other solves are skipped.  Returns 1 on invalid arguments
 * (lcartesian != 1, a used pick at a station without its phase flag, used S
 * picks with nphase 1 unless mask_s), 2 when a station's solve fails (the
 * reference's ierr), -1 on a device failure.  A failed multi-step queue
 * (mceik_mcmc_get_info multi_step) is reported as -1 by the next
 * synchronising call (sync, get_state, get_samples, checkpoint).
 * Every array below sized [nchains][ncell] is [nchains][nphase][ncell]. */
int mceik_mcmc_init(const struct mceik_parms_struct *parms,
                    const struct mceik_stations_struct *stations,
                    const struct mceik_catalog_struct *catalog,
                    const mceik_mcmc_opts *opts, const int *v0, mceik_mcmc **out);
/* Enqueue nsteps proposals for every chain (propose -> FSM -> misfit ->
 * Metropolis); keeps states per mcparms (nburnIn, keepK). Asynchronous.
 * nsteps < 0: run the remaining mcparms.niter - step proposals (mceik_struct.h:58). */
int mceik_mcmc_run(mceik_mcmc *s, int nsteps);
int mceik_mcmc_set_stream(mceik_mcmc *s, void *stream);
int mceik_mcmc_sync(mceik_mcmc *s);
/* Host copies of the chain state. Any pointer may be NULL. */
int mceik_mcmc_get_state(mceik_mcmc *s, int *v, double *logl, long long *naccept, long long *step);
/* Kept samples: copies the n = min(max, kept, max_samples) most recent kept
 * states, oldest first, into v_out [n][nchains][ncell] and logl_out
 * [n][nchains] (both host memory for kind 0, both device memory for kind 1);
 * returns n in *nkept. */
int mceik_mcmc_get_samples(mceik_mcmc *s, void *v_out, double *logl_out, int max, int kind, int *nkept);
/* Diagnostics of the last step: device pointers to the travel-time table
 * [nchains][nstat][nev] (fp32), per-solve iteration counts and reference ierr
 * [nchains][nstat] (int), and accept flags [nchains].  With nphase 2 a step
 * re-solves only the model its proposal changed: the tables are that phase's
 * (mceik_mcmc_last_phase); after init they are [nchains][nphase][nstat][nev]
 * and niter/ierr [nchains][nphase][nstat].  Any pointer may be NULL. */
int mceik_mcmc_last(mceik_mcmc *s, const float **ttab, const int **niter, const unsigned char **accept,
                    const int **ierr);
/* Device pointer to the last step's proposed phase per chain [nchains] (0 = P, 1 = S). */
int mceik_mcmc_last_phase(mceik_mcmc *s, const int **phase);
/* Fills *info (host). */
int mceik_mcmc_get_info(mceik_mcmc *s, mceik_mcmc_info *info);
/* Checkpoint / resume.  The proposal RNG is Philox keyed by (global chain,
 * step), so (v, logl, naccept, step, nkept) is the complete chain state:
 * restoring it into a sampler built with the same problem, seed and chain
 * shard continues the chains bit for bit.  checkpoint: host copies
 * (synchronises; any pointer may be NULL).  restore: host arrays for this
 * sampler's chains; logl == NULL recomputes it with one forward. */
int mceik_mcmc_checkpoint(mceik_mcmc *s, int *v, double *logl, long long *naccept, long long *step, int *nkept);
int mceik_mcmc_restore(mceik_mcmc *s, const int *v, const double *logl, const long long *naccept,
                       long long step, int nkept);
/* FSM accounting since init (or the last reset): kernel time of every FSM
 * launch from hipEvents on the sampler's stream (ms), launches, and the
 * sum over solves of executed iterations (8 sweeps each) and visits[4] = brick
 * visits (8x8x8 nodes in one sweep; unchanged z-blocks are skipped), column
 * segments updated, segments changed, wave macro steps (mceik_fsm_batch.visit_stats).
 * Synchronises. */
int mceik_mcmc_fsm_stats(mceik_mcmc *s, double *fsm_ms, long long *nlaunch, unsigned long long *iters,
                         unsigned long long *visits, int reset);
/* Solves executed since init (or the last fsm_stats reset): solves of a
 * station without picks of the solve's phase are skipped (lhasP / lhasS,
 * homog.c:313-335) and not counted.  Synchronises. */
int mceik_mcmc_fsm_solves(mceik_mcmc *s, unsigned long long *solves);
int mceik_mcmc_finalize(mceik_mcmc **s);

/* ---- multi-rank runs (one process per GPU; csrc/comm.hip) ---------------
 * The sampler's only collective is the checkpoint gather (SURVEY s.8e) over
 * RCCL (xGMI on one node).  Bootstrap as RCCL's: rank 0 calls
 * mceik_comm_unique_id, the launcher broadcasts the bytes (MPI_Bcast in a
 * C/MPI main -- MPI keeps launch and bootstrap, the role of broadcast.c and
 * mpiutils.f90:346-426), then every rank calls mceik_comm_init with its GPU. */
#define MCEIK_COMM_ID_BYTES 128
typedef struct mceik_comm mceik_comm;
/* 1 if this process can build a communicator (RCCL loads and has every entry
 * point the library uses), else 0.  Local, no GPU call: a launcher agrees on
 * it over all ranks BEFORE mceik_comm_init, which is collective and would
 * leave the other ranks waiting for a rank that cannot join. */
int mceik_comm_available(void);
int mceik_comm_unique_id(unsigned char id[MCEIK_COMM_ID_BYTES]);
int mceik_comm_init(const unsigned char id[MCEIK_COMM_ID_BYTES], int nranks, int rank, int device,
                    mceik_comm **out);
int mceik_comm_finalize(mceik_comm **c);
/* Collective over c: every rank's chains -> root, in global chain order.
 * which = 0 the current state (mceik_mcmc_get_state), 1 the most recent kept
 * state (every rank must hold one).  The ranks' shards [chain_offset,
 * chain_offset + nchains) must tile [0, nchains_total) (else every rank
 * returns 2).  On the root v_out [nchains_total][ncell] and logl_out
 * [nchains_total] are host or device memory (either may be NULL; device
 * memory of the communicator's GPU is received into directly, without
 * staging); other ranks pass NULL.
 * Synchronises the sampler's stream. */
int mceik_mcmc_gather(mceik_mcmc *s, mceik_comm *c, int which, int nchains_total, int root, int *v_out,
                      double *logl_out);

#ifdef __cplusplus
}
#endif
#endif
