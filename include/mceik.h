/*
 * mceik.h -- MCMC travel-time tomography driver API (libmceik_hip.so, gfx950).
 *
 * The reference's include/mceik.h:1-14 declares nothing; its data model
 * (mceik_struct.h) is kept and this header fills the driver slot that
 * homog.c:343-415 occupies.  One process drives one GPU; an MPI harness
 * passes its rank/size and shards chains.  Every function
 * returns 0 on success (h5io.c convention).
 */
#ifndef MCEIK_H_AMD
#define MCEIK_H_AMD 1
#include <stdint.h>
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
} mceik_mcmc_opts;

/* v0: host [nchains][ncell] int m/s, ncell = ceil(nx/nrefx)*ceil(ny/nrefy)*
 * ceil(nz/nrefz), cell index x fastest.  Computes each chain's initial logL. */
int mceik_mcmc_init(const struct mceik_parms_struct *parms,
                    const struct mceik_stations_struct *stations,
                    const struct mceik_catalog_struct *catalog,
                    const mceik_mcmc_opts *opts, const int *v0, mceik_mcmc **out);
/* Enqueue nsteps proposals for every chain (propose -> FSM -> misfit ->
 * Metropolis); keeps states per mcparms (nburnIn, keepK). Asynchronous. */
int mceik_mcmc_run(mceik_mcmc *s, int nsteps);
int mceik_mcmc_set_stream(mceik_mcmc *s, void *stream);
int mceik_mcmc_sync(mceik_mcmc *s);
/* Host copies of the chain state. Any pointer may be NULL. */
int mceik_mcmc_get_state(mceik_mcmc *s, int *v, double *logl, long long *naccept, long long *step);
/* Kept samples: copies up to max states (device or host pointers via kind:
 * 0 host, 1 device); returns the count in *nkept. Layout [k][nchains][ncell]. */
int mceik_mcmc_get_samples(mceik_mcmc *s, void *v_out, double *logl_out, int max, int kind, int *nkept);
/* Diagnostics of the last step: device pointers (travel-time table, per-solve
 * iteration counts, accept flags) and sizes. */
int mceik_mcmc_last(mceik_mcmc *s, const float **ttab, const int **niter, const unsigned char **accept);
/* FSM accounting since init (or the last reset): kernel time of every FSM
 * launch from hipEvents on the sampler's stream (ms), launches, and the
 * sum over solves of executed iterations (8 sweeps each) and visits[3] = brick
 * visits (8x8x8 nodes in one sweep; unchanged z-blocks are skipped), column
 * segments updated, segments changed (mceik_fsm_batch.visit_stats). Synchronises. */
int mceik_mcmc_fsm_stats(mceik_mcmc *s, double *fsm_ms, long long *nlaunch, unsigned long long *iters,
                         unsigned long long *visits, int reset);
int mceik_mcmc_finalize(mceik_mcmc **s);

#ifdef __cplusplus
}
#endif
#endif
