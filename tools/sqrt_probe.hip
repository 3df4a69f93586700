// sqrt_probe.hip -- is the hardware v_sqrt_f32 correctly rounded on gfx950?
// Exhaustive over every normal positive float (bits 0x00800000 .. 0x7f7fffff):
// counts, per binary exponent, the inputs where __builtin_amdgcn_sqrtf (one
// v_sqrt_f32) differs from the correctly rounded square root (LLVM's
// __builtin_sqrtf expansion, and the kernels' sqrt_normal), and prints the
// first few.  Experiment tool, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -o sqrt_probe tools/sqrt_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "../mceik_amd/csrc/fsm_update.h"

__global__ void probe(unsigned lo, unsigned n, unsigned long long *cnt_exp, unsigned *first, unsigned *nfirst,
                      unsigned long long *cnt_sn, unsigned long long *sn_exp, unsigned *sn_first, unsigned *sn_nfirst)
{
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned b = lo + i;
        const float x = __builtin_bit_cast(float, b);
        const float hw = __builtin_amdgcn_sqrtf(x);
        const float cr = __builtin_sqrtf(x);
        const float sn = sqrt_normal(x);
        if (__builtin_bit_cast(unsigned, sn) != __builtin_bit_cast(unsigned, cr)) {
            atomicAdd(cnt_sn, 1ull);
            atomicAdd(&sn_exp[b >> 23], 1ull);
            const unsigned k = atomicAdd(sn_nfirst, 1u);
            if (k < 4096) sn_first[k] = b;
        }
        if (__builtin_bit_cast(unsigned, hw) != __builtin_bit_cast(unsigned, cr)) {
            atomicAdd(&cnt_exp[b >> 23], 1ull);
            const unsigned k = atomicAdd(nfirst, 1u);
            if (k < 16) first[k] = b;
        }
    }
}

__global__ void eval(const unsigned *b, int n, unsigned *sn, unsigned *cr)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = __builtin_bit_cast(float, b[i]);
    sn[i] = __builtin_bit_cast(unsigned, sqrt_normal(x));
    cr[i] = __builtin_bit_cast(unsigned, __builtin_sqrtf(x));
}

int main()
{
    unsigned long long *cnt, *csn;
    unsigned *first, *nfirst;
    hipMalloc(&cnt, 256 * 8);
    hipMalloc(&csn, 8);
    hipMalloc(&first, 16 * 4);
    hipMalloc(&nfirst, 4);
    unsigned long long *snx;
    unsigned *snf, *snn;
    hipMalloc(&snx, 256 * 8);
    hipMalloc(&snf, 4096 * 4);
    hipMalloc(&snn, 4);
    hipMemset(snx, 0, 256 * 8);
    hipMemset(snn, 0, 4);
    hipMemset(cnt, 0, 256 * 8);
    hipMemset(csn, 0, 8);
    hipMemset(nfirst, 0, 4);
    const unsigned lo = 0x00800000u, hi = 0x7f800000u;
    hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, lo, hi - lo, cnt, first, nfirst, csn, snx, snf, snn);
    unsigned long long h[256], hs;
    unsigned f[16], nf;
    hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(&hs, csn, 8, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    hipMemcpy(&nf, nfirst, 4, hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int e = 0; e < 256; e++) tot += h[e];
    printf("inputs %u  hw != correctly rounded: %llu  sqrt_normal != correctly rounded: %llu\n", hi - lo, tot, hs);
    for (int e = 0; e < 256; e++)
        if (h[e]) printf("  exponent field %3d (2^%4d): %llu of 8388608\n", e, e - 127, h[e]);
    for (unsigned k = 0; k < nf && k < 16; k++) {
        const float x = __builtin_bit_cast(float, f[k]);
        printf("  x = %.9g (0x%08x)\n", x, f[k]);
    }
    unsigned long long hx[256];
    unsigned sf[4096], sn;
    hipMemcpy(hx, snx, sizeof(hx), hipMemcpyDeviceToHost);
    hipMemcpy(sf, snf, sizeof(sf), hipMemcpyDeviceToHost);
    hipMemcpy(&sn, snn, 4, hipMemcpyDeviceToHost);
    printf("sqrt_normal vs LLVM's sqrtf by exponent:\n");
    for (int e = 0; e < 256; e++)
        if (hx[e]) printf("  exponent field %3d (2^%4d): %llu\n", e, e - 127, hx[e]);
    // which one is correctly rounded: the host's IEEE sqrtf on the first mismatches
    const int ns = sn < 4096 ? (int)sn : 4096;
    unsigned *dsn, *dcr, vsn[4096], vcr[4096];
    hipMalloc(&dsn, 4096 * 4);
    hipMalloc(&dcr, 4096 * 4);
    if (ns) hipLaunchKernelGGL(eval, dim3((ns + 255) / 256), dim3(256), 0, 0, snf, ns, dsn, dcr);
    hipMemcpy(vsn, dsn, sizeof(vsn), hipMemcpyDeviceToHost);
    hipMemcpy(vcr, dcr, sizeof(vcr), hipMemcpyDeviceToHost);
    int bad_sn = 0, bad_llvm = 0;
    for (int k = 0; k < ns; k++) {
        const float x = __builtin_bit_cast(float, sf[k]);
        const unsigned ref = __builtin_bit_cast(unsigned, sqrtf(x));
        bad_sn += vsn[k] != ref;
        bad_llvm += vcr[k] != ref;
        if (k < 8) printf("  x = %.9g (0x%08x): sqrt_normal 0x%08x  llvm 0x%08x  host 0x%08x\n", x, sf[k], vsn[k], vcr[k], ref);
    }
    printf("of %d sampled mismatches: sqrt_normal != host sqrtf %d, llvm != host sqrtf %d\n", ns, bad_sn, bad_llvm);
    return 0;
}
