// XCC_ID of each workgroup of a 2048-workgroup launch (one wave each):
// histogram and agreement with blockIdx % 8 (hardware probe for the
// multi-step launch's XCD-owned chain groups).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void probe(unsigned *out)
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
    // keep the wave resident a while so the dispatch spreads
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100000) __builtin_amdgcn_s_sleep(10);
}
int main()
{
    const int n = 2048;
    unsigned *d, h[n];
    hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(probe, dim3(n), dim3(64), 0, 0, d);
    hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    int hist[16] = {0}, agree = 0;
    for (int i = 0; i < n; i++) { hist[h[i] & 15]++; agree += (h[i] & 15) == (unsigned)(i % 8); }
    printf("raw[0..9]:");
    for (int i = 0; i < 10; i++) printf(" %u", h[i]);
    printf("\nhist:");
    for (int i = 0; i < 16; i++) printf(" %d", hist[i]);
    printf("\nagree with blockIdx %% 8: %d of %d\n", agree, n);
    return 0;
}
