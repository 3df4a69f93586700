// Microbenchmark: does the gfx950 L2 read (fill) lines that a kernel writes
// only partially?  Each wave owns a disjoint 2 KiB block per iteration and
// writes a pattern of it; run under rocprofv3 --pmc TCC_EA0_RDREQ_sum
// TCC_EA0_WRREQ_sum.  Patterns: 0 = all 64 lanes x 32 B (full lines);
// 1 = every other lane (32 B of each 64 B); 2 = one lane in four (32 B per
// 128-B line); 3 = 16 B per lane, all lanes (full lines, two instructions);
// 4 = 16 B per lane, every other lane (16-B holes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(float4 *buf, int pattern, int iters, size_t blocks)
{
    const int lane = threadIdx.x;
    for (int it = 0; it < iters; it++) {
        size_t blk = ((size_t)blockIdx.x * iters + it) % blocks;
        float4 *b = buf + blk * 128;                  // 2 KiB = 128 float4
        float4 v = make_float4(lane, it, 1.f, 2.f);
        bool w = pattern == 0 || pattern == 3 || (pattern == 1 && (lane & 1) == 0) || (pattern == 2 && (lane & 3) == 0);
        if (pattern == 4) {
            if (lane & 1) { b[lane] = v; b[64 + lane] = v; }
        } else if (pattern == 3) {
            b[lane] = v; b[64 + lane] = v;
        } else if (w) {
            b[2 * lane] = v; b[2 * lane + 1] = v;
        }
    }
}

int main(int argc, char **argv)
{
    size_t blocks = (size_t)1 << 17;                  // 256 MiB
    float4 *buf;
    hipMalloc(&buf, blocks * 2048);
    hipMemset(buf, 0, blocks * 2048);
    for (int p = 0; p < 5; p++) {
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(probe, dim3(4096), dim3(64), 0, 0, buf, p, 64, blocks);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("pattern %d: %.3f ms\n", p, ms);
    }
    hipFree(buf);
    return 0;
}
