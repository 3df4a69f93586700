// mcmc_common.h -- device-side state of the per-GPU sampler (not public).
#pragma once
#include <stddef.h>
#include <stdint.h>

struct McmcDev {
    int nchains, chain_offset, ncell, nstat, nev;
    int vmin, vmax, dvmax;
    uint32_t seed;
    int *v;                        // [nchains][ncell] current model (m/s)
    float *slow_cur, *slow_prop;   // [nchains][ncell] 1/v of current / proposed
    double *logl;                  // [nchains]
    long long *naccept;            // [nchains]
    int *prop_cell, *prop_v, *prop_inprior;
    double *prop_logu;
    unsigned char *accept;         // [nchains] last step
    const float *ttab;             // [nchains][nstat][nev]
    const int *obs_ptr, *obs_stat, *obs_mask;
    const double *tobs, *tcorr, *var;
    int *keep_v;                   // [max_samples][keep_stride][ncell]
    double *keep_logl;             // [max_samples][keep_stride]
    int keep_stride;               // chains per kept slot: the sampler's nchains (a pipe's view covers a part)
};

// One rank's chain shard as the checkpoint gather sees it (capi.hip
// mcmc_shard_view -> comm.hip).  stream is a hipStream_t.
struct mceik_mcmc;
struct McmcShard {
    int device, nchains, chain_offset, ncell;
    void *stream;
    const int *v;                  // device [nchains][ncell]
    const double *logl;            // device [nchains]
};
int mcmc_shard_view(mceik_mcmc *s, int which, McmcShard *out);
