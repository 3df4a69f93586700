// mcmc_common.h -- device-side state of the per-GPU sampler (not public).
#pragma once
#include <stddef.h>
#include <stdint.h>

struct McmcDev {
    int nchains, chain_offset, ncell, nstat, nev;
    int nphase;                    // velocity models per chain: 1 (P) or 2 (P, S)
    int ncm;                       // ncell * nphase: one chain's model entries
    int vmin, vmax, dvmax;         // P prior, proposal step
    int vsmin, vsmax;              // S prior (nphase 2)
    uint32_t seed;
    int *v;                        // [nchains][nphase][ncell] current models (m/s)
    float *slow_cur, *slow_prop;   // [nchains][nphase][ncell] 1/v of current / proposed
    double *logl;                  // [nchains]
    long long *naccept;            // [nchains]
    int *prop_cell, *prop_v, *prop_inprior;   // prop_cell indexes the chain's [nphase][ncell] entries
    int *prop_phase;               // [nchains] the model the proposal changes (cell / ncell)
    double *prop_logu;
    unsigned char *accept;         // [nchains] last step
    const float *ttab;             // [nchains][nstat][nev]: the proposed model's tables (its phase)
    float *ttab_cur;               // nphase 2: [nchains][nphase][nstat][nev] tables of the current models
    const int *obs_ptr, *obs_stat, *obs_mask;
    const int *obs_phase;          // [nobs] 0 = P, 1 = S (null: all P)
    const double *tobs, *tcorr, *var;
    int *keep_v;                   // [max_samples][keep_stride][nphase][ncell]
    double *keep_logl;             // [max_samples][keep_stride]
    int keep_stride;               // chains per kept slot: the sampler's nchains (a pipe's view covers a part)
};

// One rank's chain shard as the checkpoint gather sees it (capi.hip
// mcmc_shard_view -> comm.hip).  stream is a hipStream_t.
struct mceik_mcmc;
struct McmcShard {
    int device, nchains, chain_offset, ncell;
    void *stream;
    const int *v;                  // device [nchains][ncell] (ncell = the chain's model entries)
    const double *logl;            // device [nchains]
};
// Returns 0, 1 (which = 1 and no state kept yet) or -1 (the sampler's stream
// failed or a multi-step launch broke its work queue: no valid state).
int mcmc_shard_view(mceik_mcmc *s, int which, McmcShard *out);
