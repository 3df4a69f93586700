// sqrt_dir_probe.hip -- direction of v_sqrt_f32's error on gfx950, and
// whether a one-sided rounding correction is exact.  Exhaustive over every
// normal positive float: counts inputs where the hardware root is one ulp
// above / one ulp below / further from the correctly rounded root
// (__builtin_sqrtf, LLVM's exact expansion), and checks two 5-instruction
// candidates against it (a one-sided Tuckerman test: hw in {cr - 1, cr} needs
// only the upper test, hw in {cr, cr + 1} only the lower one).  Experiment
// tool, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -o sqrt_dir_probe tools/sqrt_dir_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ float sqrt_up_test(float x)    // hw in {cr - 1, cr}
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const int sb = __builtin_bit_cast(int, s);
    const float up = __builtin_bit_cast(float, sb + 1);
    const int eup = __builtin_bit_cast(int, __builtin_fmaf(-up, s, x));
    int p;
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(p) : "v"(eup));
    return __builtin_bit_cast(float, sb + p);
}
__device__ __forceinline__ float sqrt_dn_test(float x)    // hw in {cr, cr + 1}
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const int sb = __builtin_bit_cast(int, s);
    const float dn = __builtin_bit_cast(float, sb - 1);
    const int edn = __builtin_bit_cast(int, __builtin_fmaf(-dn, s, x));
    int p;
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(p) : "v"(edn));
    return __builtin_bit_cast(float, (sb - 1) + p);
}

__global__ void probe(unsigned lo, unsigned n, unsigned long long *c)
{
    unsigned long long above = 0, below = 0, far = 0, bad_up = 0, bad_dn = 0;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, lo + i);
        const int hw = __builtin_bit_cast(int, __builtin_amdgcn_sqrtf(x));
        const int cr = __builtin_bit_cast(int, __builtin_sqrtf(x));
        above += hw == cr + 1;
        below += hw == cr - 1;
        far += hw > cr + 1 || hw < cr - 1;
        bad_up += __builtin_bit_cast(int, sqrt_up_test(x)) != cr;
        bad_dn += __builtin_bit_cast(int, sqrt_dn_test(x)) != cr;
    }
    atomicAdd(c + 0, above);
    atomicAdd(c + 1, below);
    atomicAdd(c + 2, far);
    atomicAdd(c + 3, bad_up);
    atomicAdd(c + 4, bad_dn);
}

int main()
{
    unsigned long long *c, h[5];
    hipMalloc(&c, sizeof(h));
    // every normal positive float, and the domain the kernels use (x >= 2^-104)
    const unsigned ranges[2][2] = {{0x00800000u, 0x7f800000u}, {0x0b800000u, 0x7f800000u}};
    for (int r = 0; r < 2; r++) {
        hipMemset(c, 0, sizeof(h));
        hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, ranges[r][0], ranges[r][1] - ranges[r][0], c);
        hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
        printf("x in [0x%08x, 0x%08x): hw = cr + 1ulp %llu, hw = cr - 1ulp %llu, further %llu; "
               "upper-test-only != cr %llu, lower-test-only != cr %llu\n",
               ranges[r][0], ranges[r][1], h[0], h[1], h[2], h[3], h[4]);
    }
    return 0;
}
