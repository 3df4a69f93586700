// mcmc_device.h -- the per-chain pieces of a sampler step (proposal, L2
// misfit, Metropolis, kept state), shared by the per-step kernels
// (mcmc_kernels.hip: one thread per chain) and the chain epilogue of the
// multi-step FSM launch (fsm16_kernel.hip: one wave per chain).  Both run the
// same arithmetic in the same order, so the two paths agree bit for bit.
//
// The reference defines no MCMC (include/mceik.h:1-14 is empty; only
// mcmc_parms_struct, mceik_struct.h:54-60).  The definition
// is restated on the CPU in oracle/mceik_oracle.c: integer Philox4x32-10
// draws, a log built from IEEE +,-,*,/ only, an fp64 misfit summed in
// observation order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcmc_common.h"

namespace mcmcd {

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

// Natural log from IEEE basic operations only (host twin: oracle_det_log).
__device__ __forceinline__ double det_log(double x)
{
    uint64_t b = __double_as_longlong(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    double m = __longlong_as_double((long long)((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
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

// A load of chain state through a vector-register address.  Inside a
// multi-step launch the chain state changes, and a wave-uniform load may
// otherwise become a scalar-cache load, which nothing invalidates.
template <typename T>
__device__ __forceinline__ T ldv(const T *p)
{
    asm volatile("" : "+v"(p));
    return *p;
}

// One proposal for chain c: a single inversion cell of one of the chain's
// nphase models moves by +-[1, dvmax] m/s (cell drawn over [0, nphase*ncell):
// with one model exactly the P-only draw).  slow_prop (== slow_cur everywhere
// but the proposed cell) gets the new cell.
__device__ __forceinline__ void chain_propose(const McmcDev &D, int c, uint64_t step)
{
    uint32_t ctr[4] = {(uint32_t)step, (uint32_t)(step >> 32), 0u, 0u};
    philox4x32_10(ctr, (uint32_t)(D.chain_offset + c), D.seed);
    const int cell = (int)(((uint64_t)ctr[0] * (uint32_t)D.ncm) >> 32);
    const int mag = 1 + (int)(((uint64_t)ctr[1] * (uint32_t)D.dvmax) >> 32);
    const int ph = cell >= D.ncell ? 1 : 0;
    const int vold = ldv(&D.v[(size_t)c * D.ncm + cell]);
    const int vn = vold + ((ctr[2] & 1u) ? -mag : mag);
    const int inp = ph ? (vn >= D.vsmin && vn <= D.vsmax) : (vn >= D.vmin && vn <= D.vmax);
    D.prop_cell[c] = cell;
    D.prop_phase[c] = ph;
    D.prop_v[c] = vn;
    D.prop_inprior[c] = inp;
    D.prop_logu[c] = det_log(((double)ctr[3] + 0.5) * (1.0 / 4294967296.0));
    if (inp) D.slow_prop[(size_t)c * D.ncm + cell] = 1.0f / (float)vn;
}

// objfn of event e for chain c: the L2 misfit with analytic origin time
// (locate.c:923-1047 at one grid point, iwantOT = 1), observations in CSR
// order; an S observation is fit against the S model's table of its station
// (the locator stacks both phases, locate.f90:399,442).  Tables of phase pph
// come from the proposal's tables, the others from the current ones (pph < 0:
// every phase from ttab_cur; nphase 1 uses pph = 0).
__device__ __forceinline__ double event_obj(const McmcDev &D, int c, int pph, int e)
{
    const float *tp = D.ttab + (size_t)c * D.nstat * D.nev;
    const float *tcur = D.ttab_cur ? D.ttab_cur + (size_t)c * D.nphase * D.nstat * D.nev : nullptr;
    const double sqrt2i = 0.7071067811865475;
    auto te_of = [&](int j) -> double {
        const int ph = D.obs_phase ? D.obs_phase[j] : 0;
        const size_t k = (size_t)D.obs_stat[j] * D.nev + e;
        return (double)(ph == pph ? ldv(tp + k) : ldv(tcur + (size_t)ph * D.nstat * D.nev + k));
    };
    const int j0 = D.obs_ptr[e], j1 = D.obs_ptr[e + 1];
    double xnorm = 0.0, t0 = 0.0, obj = 0.0;
    for (int j = j0; j < j1; j++) if (!D.obs_mask[j]) xnorm = xnorm + 1.0 / D.var[j];
    for (int j = j0; j < j1; j++) {
        if (D.obs_mask[j]) continue;
        double te = te_of(j);
        double tc = D.tobs[j] - D.tcorr[j];
        t0 = t0 + ((1.0 / D.var[j]) / xnorm) * (tc - te);
    }
    for (int j = j0; j < j1; j++) {
        if (D.obs_mask[j]) continue;
        double te = te_of(j);
        double tc = D.tobs[j] - D.tcorr[j];
        double res = ((1.0 / D.var[j]) * sqrt2i) * (tc - (te + t0));
        obj = obj + res * res;
    }
    return obj;
}

// logL = -sum_e objfn_e, events in order.
__device__ __forceinline__ double chain_loglik(const McmcDev &D, int c, int pph)
{
    double logl = 0.0;
    for (int e = 0; e < D.nev; e++) logl = logl - event_obj(D, c, pph, e);
    return logl;
}

// Metropolis accept/reject of chain c's pending proposal given its logL ln
// (ignored outside the prior); keeps slot_cur / slot_prop identical except
// while a proposal is pending, so each step touches one cell per chain.
// Returns 1 when accepted.  The table copy of an accepted two-model proposal
// is the caller's (chain_copy_tables).
__device__ __forceinline__ int chain_accept(const McmcDev &D, int c, double ln, int keep_slot)
{
    const int cell = ldv(&D.prop_cell[c]);
    const size_t ci = (size_t)c * D.ncm + cell;
    int acc = 0;
    if (ldv(&D.prop_inprior[c])) {
        acc = ldv(&D.prop_logu[c]) < ln - ldv(&D.logl[c]);
        if (acc) {
            D.logl[c] = ln;
            D.v[ci] = ldv(&D.prop_v[c]);
            D.slow_cur[ci] = ldv(&D.slow_prop[ci]);
            D.naccept[c] = ldv(&D.naccept[c]) + 1;
        } else {
            D.slow_prop[ci] = ldv(&D.slow_cur[ci]);
        }
    }
    D.accept[c] = (unsigned char)acc;
    if (keep_slot >= 0) D.keep_logl[(size_t)keep_slot * D.keep_stride + c] = ldv(&D.logl[c]);
    return acc;
}

// An accepted proposal's tables become its phase's current tables (nphase 2);
// elements first, first + stride, ...
__device__ __forceinline__ void chain_copy_tables(const McmcDev &D, int c, int ph, int first, int stride)
{
    const size_t n = (size_t)D.nstat * D.nev;
    const float *src = D.ttab + (size_t)c * n;
    float *dst = D.ttab_cur + ((size_t)c * D.nphase + ph) * n;
    for (size_t k = first; k < n; k += stride) dst[k] = ldv(src + k);
}

}  // namespace mcmcd
