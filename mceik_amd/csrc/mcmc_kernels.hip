// mcmc_kernels.hip -- proposal, L2 misfit + Metropolis, and the L2 grid
// search, on gfx950.
//
// The per-chain step pieces live in mcmc_device.h (shared with the chain
// epilogue of the multi-step FSM launch).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcmc_common.h"
#include "mcmc_device.h"

namespace {


// One proposal per chain (mcmc_device.h chain_propose).
__global__ void propose_kernel(McmcDev D, uint64_t step)
{
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= D.nchains) return;
    mcmcd::chain_propose(D, c, step);
}

__global__ void init_loglik_kernel(McmcDev D)
{
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= D.nchains) return;
    D.logl[c] = mcmcd::chain_loglik(D, c, D.nphase > 1 ? -1 : 0);
}

// Metropolis accept/reject (mcmc_device.h chain_accept); with two models an
// accepted proposal's tables become its phase's current tables.
__global__ void accept_kernel(McmcDev D, int keep_slot)
{
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= D.nchains) return;
    const int inp = D.prop_inprior[c], ph = D.prop_phase[c];
    const double ln = inp ? mcmcd::chain_loglik(D, c, ph) : 0.0;
    if (mcmcd::chain_accept(D, c, ln, keep_slot) && D.nphase > 1) mcmcd::chain_copy_tables(D, c, ph, 0, 1);
}

// Kept state copy: [slot][chain][nphase][ncell] int (after accept_kernel).
__global__ void keep_kernel(McmcDev D, int keep_slot)
{
    size_t n = (size_t)D.nchains * D.ncm;
    int *dst = D.keep_v + (size_t)keep_slot * D.keep_stride * D.ncm;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = D.v[i];
}

// ---- L2 grid search (locate.c:923-1047) over all grid points -----------------
// obs already compacted on the host in the reference's order: use[j] (row of
// test), tc[j] = tobs - tcorr, wt[j] = 1/var; xnorm = sum wt (host, same order).
__global__ void l2_gridsearch_kernel(int ldgrd, int ngrd, int nuse, int iwantOT, double t0use,
                                     const int *use, const double *tc, const double *wt, double xnorm,
                                     const double *test, double *t0, double *objfn)
{
    const double sqrt2i = 0.7071067811865475;
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < ngrd; g += gridDim.x * blockDim.x) {
        double t = 0.0;
        if (iwantOT == 1) {
            for (int j = 0; j < nuse; j++) {
                double w = wt[j] / xnorm;
                t = t + w * (tc[j] - test[(size_t)ldgrd * use[j] + g]);
            }
        } else {
            t = t0use;
        }
        double o = 0.0;
        for (int j = 0; j < nuse; j++) {
            double w = wt[j] * sqrt2i;
            double res = w * (tc[j] - (test[(size_t)ldgrd * use[j] + g] + t));
            o = o + res * res;
        }
        t0[g] = t;
        objfn[g] = o;
    }
}

// fp32 twin of the above (locate.c:1079-1203, locate_l2_gridSearch__float64),
// batched over events that share travel-time tables: event e uses
// observations [ev_ptr[e], ev_ptr[e+1]) of the compacted arrays (mask already
// applied, reference order), row obs_row[j] of `test` (leading dimension
// ldgrd), tc = tobs - tcorr, wt = 1/var, xnorm[e] = sum wt (host, in order).
// grid (ceil(ngrd/256), nev): thread = (grid point, event).
__global__ void l2_gridsearch_f32_kernel(int ldgrd, int ngrd, int iwantOT, float t0use, const int *ev_ptr,
                                         const int *obs_row, const float *tc, const float *wt, const float *xnorm,
                                         const float *test, float *t0, float *objfn, int negate)
{
    const float sqrt2i = 0.7071067811865475f;
    const int e = blockIdx.y;
    const int j0 = ev_ptr[e], j1 = ev_ptr[e + 1];
    const float xn = xnorm[e];
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < ngrd; g += gridDim.x * blockDim.x) {
        float t = 0.0f;
        if (iwantOT == 1) {
            for (int j = j0; j < j1; j++) {
                const float w = wt[j] / xn;
                t = t + w * (tc[j] - test[(size_t)ldgrd * obs_row[j] + g]);
            }
        } else {
            t = t0use;
        }
        float o = 0.0f;
        for (int j = j0; j < j1; j++) {
            const float w = wt[j] * sqrt2i;
            const float res = w * (tc[j] - (test[(size_t)ldgrd * obs_row[j] + g] + t));
            o = o + res * res;
        }
        if (t0) t0[(size_t)e * ldgrd + g] = t;
        objfn[(size_t)e * ldgrd + g] = negate ? -o : o;
    }
}

// Single-pass relocation (SURVEY s.8f row 2): a block stages the travel-time
// tables of its TG grid points -- every row, once -- in LDS, and each thread
// then evaluates ALL events at its grid point from its own LDS column, so a
// table value leaves HBM once per launch instead of twice per event that
// observes it.  The per-observation weights wt/xnorm and wt*sqrt(1/2) are
// formed once per block (the same fp32 operations as l2_gridsearch_f32_kernel,
// so every output is bitwise the same) into per-event groups aligned to 4, read
// back as 16-B uniform (broadcast) LDS loads by the 4-way unrolled pair loops.
// LDS: [nrows][TG] tables | per event 4-aligned (tc, w0, w1, row*TG) | offsets.
template <int TG>
__global__ __launch_bounds__(TG) void relocate_lds_kernel(int ldgrd, int ngrd, int nrows, int nev, int nobs,
                                                          int iwantOT, float t0use, const int *ev_ptr,
                                                          const int *obs_row, const float *tc, const float *wt,
                                                          const float *xnorm, const float *test, float *t0,
                                                          float *objfn, int negate)
{
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef int i4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *tile = sm;                                   // [nrows][TG]
    const int cap = (nobs + 3 * nev + 3) & ~3;          // obs slots with per-event padding to 4
    float *stc = sm + (size_t)nrows * TG, *sw0 = stc + cap, *sw1 = sw0 + cap;
    int *srow = (int *)(sw1 + cap), *soff = srow + cap;    // soff [nev + 1]
    const float sqrt2i = 0.7071067811865475f;
    const int tid = threadIdx.x;
    __shared__ int bad;                                 // the caller's nobs / nrows do not hold
    if (tid == 0) {
        int o = 0, b = ev_ptr[0] != 0 || ev_ptr[nev] != nobs;
        for (int e = 0; e < nev && !b; e++) {
            b = ev_ptr[e + 1] < ev_ptr[e];
            soff[e] = o;
            o += (ev_ptr[e + 1] - ev_ptr[e] + 3) & ~3;
        }
        soff[nev] = o;
        bad = b;
    }
    __syncthreads();
    if (!bad) {
        int b = 0;
        for (int e = 0; e < nev; e++) {
            const float xn = xnorm[e];
            const int j0 = ev_ptr[e], base = soff[e] - j0;
            for (int j = j0 + tid; j < ev_ptr[e + 1]; j += TG) {
                const int r = obs_row[j];
                b |= r < 0 || r >= nrows;
                stc[base + j] = tc[j];
                sw0[base + j] = wt[j] / xn;
                sw1[base + j] = wt[j] * sqrt2i;
                srow[base + j] = (b ? 0 : r) * TG;
            }
        }
        if (b) bad = 1;
    }
    const int g = blockIdx.x * TG + tid;
    const bool in = g < ngrd;
    __syncthreads();
    if (bad) {
        // contract violated: every output of the block is NaN (no LDS access
        // out of bounds, and no plausible-looking misfits)
        if (in)
            for (int e = 0; e < nev; e++) {
                if (t0) t0[(size_t)e * ldgrd + g] = __builtin_nanf("");
                objfn[(size_t)e * ldgrd + g] = __builtin_nanf("");
            }
        return;
    }
    for (int r = 0; r < nrows; r++) tile[r * TG + tid] = in ? test[(size_t)ldgrd * r + g] : 0.0f;
    __syncthreads();
    if (!in) return;
    const float *col = tile + tid;
    for (int e = 0; e < nev; e++) {
        const int b = soff[e], n = ev_ptr[e + 1] - ev_ptr[e], n4 = n & ~3;
        float t = 0.0f;
        if (iwantOT == 1) {
            for (int k = 0; k < n4; k += 4) {
                const f4 c4 = *(const f4 *)(stc + b + k), w4 = *(const f4 *)(sw0 + b + k);
                const i4 r4 = *(const i4 *)(srow + b + k);
                const float te0 = col[r4.x], te1 = col[r4.y], te2 = col[r4.z], te3 = col[r4.w];
                t = t + w4.x * (c4.x - te0);
                t = t + w4.y * (c4.y - te1);
                t = t + w4.z * (c4.z - te2);
                t = t + w4.w * (c4.w - te3);
            }
            for (int k = n4; k < n; k++) t = t + sw0[b + k] * (stc[b + k] - col[srow[b + k]]);
        } else {
            t = t0use;
        }
        float o = 0.0f;
        for (int k = 0; k < n4; k += 4) {
            const f4 c4 = *(const f4 *)(stc + b + k), w4 = *(const f4 *)(sw1 + b + k);
            const i4 r4 = *(const i4 *)(srow + b + k);
            const float te0 = col[r4.x], te1 = col[r4.y], te2 = col[r4.z], te3 = col[r4.w];
            float res = w4.x * (c4.x - (te0 + t));
            o = o + res * res;
            res = w4.y * (c4.y - (te1 + t));
            o = o + res * res;
            res = w4.z * (c4.z - (te2 + t));
            o = o + res * res;
            res = w4.w * (c4.w - (te3 + t));
            o = o + res * res;
        }
        for (int k = n4; k < n; k++) {
            const float res = sw1[b + k] * (stc[b + k] - (col[srow[b + k]] + t));
            o = o + res * res;
        }
        if (t0) t0[(size_t)e * ldgrd + g] = t;
        objfn[(size_t)e * ldgrd + g] = negate ? -o : o;
    }
}

// Fortran misfit variant (gridsearch.f90:176-540): per grid point the t0 stack
// (LOCATE3D_STACK_T0_*, weight 1/(var_i * sum var)) then the logPDF stack
// (LOCATE3D_STACK_LOGPDF_*, weight sqrt(1/2)/var_i), observations in order.
// Host-compacted arrays: row[j] of test, tob[j], w0[j] = 1/(var*xnorm),
// wl[j] = sqrt2i/var, computed in T exactly as the Fortran does.
template <typename T>
__global__ void gridsearch_f90_kernel(int ldgrd, int ngrd, int nuse, int iwantOT, const int *row, const T *tob,
                                      const T *w0, const T *wl, const T *test, T *logpdf)
{
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < ngrd; g += gridDim.x * blockDim.x) {
        T t0 = (T)0;
        if (iwantOT == 1)
            for (int j = 0; j < nuse; j++) t0 = t0 + w0[j] * (tob[j] - test[(size_t)ldgrd * row[j] + g]);
        T lp = (T)0;
        for (int j = 0; j < nuse; j++) {
            const T res = wl[j] * (tob[j] - (test[(size_t)ldgrd * row[j] + g] + t0));
            lp = lp + res * res;
        }
        logpdf[g] = lp;
    }
}

}  // namespace

hipError_t gridsearch_f90(int is_double, int ldgrd, int ngrd, int nuse, int iwantOT, const int *row,
                          const void *tob, const void *w0, const void *wl, const void *test, void *logpdf,
                          hipStream_t st)
{
    int bx = (ngrd + 255) / 256;
    if (bx > 4096) bx = 4096;
    if (is_double)
        hipLaunchKernelGGL(gridsearch_f90_kernel<double>, dim3(bx), dim3(256), 0, st, ldgrd, ngrd, nuse, iwantOT,
                           row, (const double *)tob, (const double *)w0, (const double *)wl, (const double *)test,
                           (double *)logpdf);
    else
        hipLaunchKernelGGL(gridsearch_f90_kernel<float>, dim3(bx), dim3(256), 0, st, ldgrd, ngrd, nuse, iwantOT,
                           row, (const float *)tob, (const float *)w0, (const float *)wl, (const float *)test,
                           (float *)logpdf);
    return hipGetLastError();
}

// Longest-first queue order for the next FSM launch.  The persistent waves
// pull solves from 8 queues (fsm_device.h next_solve: group g drains slots
// [nsolve*g/8, nsolve*(g+1)/8) and then steals); a chain's proposal changes
// one cell, so a solve costs about what it cost last step.  Each group's
// solves are ranked by last launch's duration (s_memrealtime stamps, the
// kernel's solve_clock), longest first, ties by solve id, and written to
// the group's own slots: the set of solves per group -- hence per XCD -- is
// unchanged, only the order within it.  Results do not depend on the order.
// Rank by counting over the group's keys staged through LDS (n^2 / group:
// 4096-solve groups at C3 take well under a millisecond).
#define LPT_TILE 2048
__global__ __launch_bounds__(256) void lpt_order_kernel(const unsigned long long *clk, int nsolve, int *order)
{
    __shared__ unsigned key[LPT_TILE];
    const int g = blockIdx.y;
    const int lo = (int)((long long)nsolve * g / 8), hi = (int)((long long)nsolve * (g + 1) / 8), n = hi - lo;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if ((int)blockIdx.x * 256 >= n) return;                 // uniform per block
    auto dur = [&](int j) -> unsigned {
        const unsigned long long d = clk[2 * (size_t)j + 1] - clk[2 * (size_t)j];
        return d > 0xffffffffull ? 0xffffffffu : (unsigned)d;
    };
    const unsigned ki = i < n ? dur(lo + i) : 0u;
    int rank = 0;
    for (int t0 = 0; t0 < n; t0 += LPT_TILE) {
        const int m = min(LPT_TILE, n - t0);
        __syncthreads();
        for (int j = threadIdx.x; j < m; j += 256) key[j] = dur(lo + t0 + j);
        __syncthreads();
        for (int j = 0; j < m; j++) {
            const unsigned kj = key[j];
            rank += (kj > ki) || (kj == ki && t0 + j < i);
        }
    }
    if (i < n) order[lo + rank] = lo + i;
}

hipError_t mcmc_lpt_order(const unsigned long long *clk, int nsolve, int *order, hipStream_t st)
{
    const int nmax = (nsolve + 7) / 8;
    hipLaunchKernelGGL(lpt_order_kernel, dim3((nmax + 255) / 256, 8), dim3(256), 0, st, clk, nsolve, order);
    return hipGetLastError();
}

hipError_t mcmc_propose(const McmcDev &D, uint64_t step, hipStream_t st)
{
    hipLaunchKernelGGL(propose_kernel, dim3((D.nchains + 255) / 256), dim3(256), 0, st, D, step);
    return hipGetLastError();
}

hipError_t mcmc_init_loglik(const McmcDev &D, hipStream_t st)
{
    hipLaunchKernelGGL(init_loglik_kernel, dim3((D.nchains + 63) / 64), dim3(64), 0, st, D);
    return hipGetLastError();
}

hipError_t mcmc_accept(const McmcDev &D, int keep_slot, hipStream_t st)
{
    hipLaunchKernelGGL(accept_kernel, dim3((D.nchains + 63) / 64), dim3(64), 0, st, D, keep_slot);
    if (keep_slot >= 0)
        hipLaunchKernelGGL(keep_kernel, dim3(512), dim3(256), 0, st, D, keep_slot);
    return hipGetLastError();
}

hipError_t l2_gridsearch(int ldgrd, int ngrd, int nuse, int iwantOT, double t0use, const int *use,
                         const double *tc, const double *wt, double xnorm, const double *test,
                         double *t0, double *objfn, hipStream_t st)
{
    int blocks = (ngrd + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(l2_gridsearch_kernel, dim3(blocks), dim3(256), 0, st, ldgrd, ngrd, nuse, iwantOT,
                       t0use, use, tc, wt, xnorm, test, t0, objfn);
    return hipGetLastError();
}

#define RELOC_TG 256
size_t relocate_lds_bytes(int nrows, int nobs, int nev)
{
    return (size_t)nrows * RELOC_TG * 4 + (size_t)((nobs + 3 * nev + 3) & ~3) * 16 + (size_t)(nev + 1) * 4;
}

hipError_t relocate_lds(int ldgrd, int ngrd, int nrows, int nev, int nobs, int iwantOT, float t0use,
                        const int *ev_ptr, const int *obs_row, const float *tc, const float *wt, const float *xnorm,
                        const float *test, float *t0, float *objfn, int negate, hipStream_t st)
{
    const size_t lds = relocate_lds_bytes(nrows, nobs, nev);
    hipLaunchKernelGGL(relocate_lds_kernel<RELOC_TG>, dim3((ngrd + RELOC_TG - 1) / RELOC_TG), dim3(RELOC_TG), lds, st,
                       ldgrd, ngrd, nrows, nev, nobs, iwantOT, t0use, ev_ptr, obs_row, tc, wt, xnorm, test, t0, objfn,
                       negate);
    return hipGetLastError();
}

hipError_t l2_gridsearch_f32(int ldgrd, int ngrd, int nev, int iwantOT, float t0use, const int *ev_ptr,
                             const int *obs_row, const float *tc, const float *wt, const float *xnorm,
                             const float *test, float *t0, float *objfn, int negate, hipStream_t st)
{
    int bx = (ngrd + 255) / 256;
    if (bx > 2048) bx = 2048;
    hipLaunchKernelGGL(l2_gridsearch_f32_kernel, dim3(bx, nev), dim3(256), 0, st, ldgrd, ngrd, iwantOT, t0use,
                       ev_ptr, obs_row, tc, wt, xnorm, test, t0, objfn, negate);
    return hipGetLastError();
}
