// fsm_device.h -- device helpers shared by the two batched sweep kernels
// (fsm_kernel.hip: 8-z steps, every precision and slowness mode;
// fsm16_kernel.hip: 16-z steps, the fp32 cell-cache sampler instance): buffer
// resources, the field layout, the per-solve setup (EIKONAL3D_SETBCS,
// fsm3d.f90:697-840), the work queue, and the fast fp32 Godunov update.
// Not a public header.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fsm_common.h"
#include "fsm_update.h"

namespace {

// ---- buffer resources: 32-bit offsets, out-of-range reads return 0 and
// out-of-range writes are dropped, so predicated memory ops need no branches.
#define OOB 0x80000000u
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc make_rsrc(const void *p, uint32_t bytes)
{
    // wave-uniform by construction (kernel args / readfirstlane'd solve id)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

// NOTE (ROCm 7.2 clang): extracting elements of the uint4 returned by
// __builtin_amdgcn_raw_buffer_load_b128 miscompiles into one buffer_load_dword;
// bit-casting the whole vector to float4 / double2 keeps the dwordx4.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void bload8(Rsrc r, uint32_t off, float (&v)[8])
{
    f4v a = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    f4v b = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void bstore8(Rsrc r, uint32_t off, const float (&v)[8])
{
    f4v a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, a), r, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, b), r, off + 16, 0, 0);
}
__device__ __forceinline__ void bload8(Rsrc r, uint32_t off, double (&v)[8])
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        d2v a = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * k, 0, 0));
        v[2 * k] = a.x; v[2 * k + 1] = a.y;
    }
}
__device__ __forceinline__ void bstore8(Rsrc r, uint32_t off, const double (&v)[8])
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        d2v a = {v[2 * k], v[2 * k + 1]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, a), r, off + 16 * k, 0, 0);
    }
}
__device__ __forceinline__ void bstore4(Rsrc r, uint32_t off, float a0, float a1, float a2, float a3)
{
    f4v a = {a0, a1, a2, a3};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, a), r, off, 0, 0);
}
__device__ __forceinline__ float bload1f(Rsrc r, uint32_t off)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// Column order inside a brick: the tile perimeter first -- rows ly = 0 and
// ly = 7 (slots 0..15), then the x faces lx = 0 and lx = 7 (16..27), then the
// interior -- so each face a neighbour tile reads as its halo spans 2-4
// 128-B lines instead of 8 (row-major order puts every x-face column in its
// own line).
__host__ __device__ __forceinline__ int colpos(int lx, int ly)
{
    if (ly == 0) return lx;
    if (ly == 7) return 8 + lx;
    if (lx == 0) return 15 + ly;
    if (lx == 7) return 21 + ly;
    return 28 + (ly - 1) * 6 + (lx - 1);
}
__host__ __device__ __forceinline__ void colpos_inv(int p, int &lx, int &ly)
{
    if (p < 8) { lx = p; ly = 0; }
    else if (p < 16) { lx = p - 8; ly = 7; }
    else if (p < 22) { lx = 0; ly = p - 15; }
    else if (p < 28) { lx = 7; ly = p - 21; }
    else { lx = 1 + (p - 28) % 6; ly = 1 + (p - 28) / 6; }
}

// Field layout: per tile, groups of 128-B lines, one per column (colpos
// order), each holding ZQ = 128/es consecutive z of that column.  A lane
// reads and writes its 8-z segment of a line in BPL consecutive steps, so a
// line is fetched once per tile visit (a row-of-bricks layout spreads each
// line over 4 columns that different lane diagonals reach up to 14 steps
// apart, and the L2 refetches it).
template <typename R> struct Lay {
    static constexpr int ZQ = 128 / (int)sizeof(R);      // z per line
    static constexpr int BPL = ZQ / 8;                   // 8-z bricks per line
};
template <typename R>
__device__ __forceinline__ uint32_t zoff_bytes(int zb)
{
    // shifts, not the (zb / BPL) * (8192 - 128) + zb * 32 the compiler would
    // otherwise form (v_mul_lo_u32 is quarter rate); zb >= 0 wherever used
    constexpr int LB = Lay<R>::BPL == 4 ? 2 : 1, LS = sizeof(R) == 4 ? 5 : 6;
    const uint32_t u = (uint32_t)zb;
    return ((u >> LB) << 13) | ((u & (uint32_t)(Lay<R>::BPL - 1)) << LS);
}
template <typename R>
__device__ __forceinline__ uint32_t tile_bytes(const FsmLaunch &L) { return (uint32_t)L.nzq * 8192u; }

// x-fastest node -> field element index
template <typename R>
__device__ __forceinline__ size_t brick_index(const FsmLaunch &L, int x, int y, int z)
{
    constexpr int ZQ = Lay<R>::ZQ;
    const int tile = (y >> 3) * L.ntx + (x >> 3);
    return (((size_t)tile * L.nzq + z / ZQ) * 64 + colpos(x & 7, y & 7)) * ZQ + z % ZQ;
}

// Travel time of event e from a finished field (fp32 table value).  ev_frac ==
// nullptr: the value at node ev_node[e] (the reference snaps sources to the
// nearest node, fsm3d.f90:697-711).  Otherwise trilinear interpolation in the
// cell whose lowest corner is ev_node[e], with fractions ev_frac[3e..3e+2]:
// x first, then y, then z, each lerp a + w*(b - a) in fp32 with every
// operation rounded (no contraction) -- oracle/mceik_oracle.c
// oracle_event_time restates it operation for operation.
template <typename R>
__device__ __forceinline__ float event_time(const FsmLaunch &L, const R *u, int e)
{
    const int node = L.ev_node[e];
    const int nxy = L.nx * L.ny;
    const int z = node / nxy, rem = node - z * nxy, y = rem / L.nx, x = rem - y * L.nx;
    if (!L.ev_frac) return (float)u[brick_index<R>(L, x, y, z)];
    const float wx = L.ev_frac[3 * e], wy = L.ev_frac[3 * e + 1], wz = L.ev_frac[3 * e + 2];
    const int x1 = min(x + 1, L.nx - 1), y1 = min(y + 1, L.ny - 1), z1 = min(z + 1, L.nz - 1);
    float c[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
        c[k] = (float)u[brick_index<R>(L, (k & 1) ? x1 : x, (k & 2) ? y1 : y, (k & 4) ? z1 : z)];
    float a[4];
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = __fadd_rn(c[2 * k], __fmul_rn(wx, __fsub_rn(c[2 * k + 1], c[2 * k])));
    const float b0 = __fadd_rn(a[0], __fmul_rn(wy, __fsub_rn(a[1], a[0])));
    const float b1 = __fadd_rn(a[2], __fmul_rn(wy, __fsub_rn(a[3], a[2])));
    return __fadd_rn(b0, __fmul_rn(wz, __fsub_rn(b1, b0)));
}

// A skipped solve (mceik_fsm_batch.skip: the station has no picks of the
// solve's phase): no sweep; iterations 0, ierr 0, its table row FLT_MAX.
template <typename R>
__device__ __forceinline__ void skip_solve(const FsmLaunch &L, unsigned solve)
{
    const int lane = threadIdx.x;
    if (lane == 0) {
        if (L.solve_clock) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            L.solve_clock[2 * (size_t)solve] = t;
            L.solve_clock[2 * (size_t)solve + 1] = t;
        }
        if (L.niter) L.niter[solve] = 0;
        if (L.ierr) L.ierr[solve] = 0;
    }
    if (L.ttab)
        for (int e = lane; e < L.nev; e += 64) L.ttab[(size_t)solve * L.nev + e] = FLT_MAX;
}

// Per-solve boundary-condition boxes (EIKONAL3D_SETBCS nodes, lupd = .FALSE.).
// Wave-uniform, kept in LDS: box k = {xlo, xhi, ylo, yhi, zlo, zhi} (0-based, inclusive).
struct BcBoxes {
    int n;
    int *box;          // LDS, [nsrc][6]
};

// Traffic accounting (MCEIK_TRAFFIC builds): lane 0 adds bytes x (lanes where
// pred holds) to the wave's LDS counter of category k.
#ifdef MCEIK_TRAFFIC
#define TRAF(S, k, pred, bytes)                                                                         \
    do {                                                                                                \
        const unsigned n_ = (unsigned)__builtin_popcountll(__ballot(pred));                             \
        if (threadIdx.x == 0) (S).scratch[8 + (k)] += (int)(n_ * (unsigned)(bytes));                     \
    } while (0)
#define TRAFU(S, k, bytes)                                                                              \
    do {                                                                                                \
        if (threadIdx.x == 0) (S).scratch[8 + (k)] += (int)(bytes);                                     \
    } while (0)
#endif
#ifdef MCEIK_TRAFFIC
// flush the wave's counters to the launch totals (after every sweep / solve)
#define TRAF_FLUSH(L, S)                                                                                \
    do {                                                                                                \
        asm volatile("" ::: "memory");                                                                  \
        if (threadIdx.x == 0 && (L).traffic)                                                            \
            for (int k_ = 0; k_ < MCEIK_TRAFFIC_N; k_++) {                                              \
                atomicAdd((L).traffic + k_, (unsigned long long)(unsigned)(S).scratch[8 + k_]);         \
                (S).scratch[8 + k_] = 0;                                                                \
            }                                                                                           \
        asm volatile("" ::: "memory");                                                                  \
    } while (0)
#else
#define TRAF(S, k, pred, bytes) do { } while (0)
#define TRAFU(S, k, bytes) do { } while (0)
#define TRAF_FLUSH(L, S) do { } while (0)
#endif

// Cell range of a tile along one axis: first cell and count.
__device__ __forceinline__ void tile_cells(int t, int n, unsigned magic, int &c0, int &nc)
{
    const int a = t * 8, b = min(t * 8 + 7, n - 1);
    c0 = (int)(((unsigned)a * magic) >> 20);
    nc = (int)(((unsigned)b * magic) >> 20) - c0 + 1;
}
// Cell range of z-block tz.
__device__ __forceinline__ void block_zcells(const FsmLaunch &L, int kb, int tz, int &cz0, int &ncz)
{
    const int a = tz * kb * 8, b = min(a + kb * 8, L.nz) - 1;
    cz0 = (int)(((unsigned)a * L.magic_rz) >> 20);
    ncz = (int)(((unsigned)b * L.magic_rz) >> 20) - cz0 + 1;
}

__device__ __forceinline__ void bload4(Rsrc r, uint32_t off, float (&v)[4])
{
    f4v a = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
__device__ __forceinline__ void bload4(Rsrc r, uint32_t off, double (&v)[4])
{
    d2v a = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    d2v b = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}
__device__ __forceinline__ void bstore1(Rsrc r, uint32_t off, float v)
{
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}
__device__ __forceinline__ void bstore1(Rsrc r, uint32_t off, double v)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, off, 0, 0);
}
__device__ __forceinline__ float bload1(Rsrc r, uint32_t off, float)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ double bload1(Rsrc r, uint32_t off, double)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

template <typename R, int SLOWMODE>
__device__ __forceinline__ double slow_at(const FsmLaunch &L, const void *slow_model, int x, int y, int z)
{
    if (SLOWMODE == 0)
        return (double)reinterpret_cast<const R *>(slow_model)[brick_index<R>(L, x, y, z)];   // modes 1, 2: cells
    // (a vector load: the sampler's multi-step launch changes the cells between
    // solves, and a wave-uniform address would make this a scalar-cache load)
    const float *si = reinterpret_cast<const float *>(slow_model);
    asm volatile("" : "+v"(si));
    return (double)si[((size_t)(z / L.nrz) * L.ncy + y / L.nry) * L.ncx + x / L.nrx];
}

__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// Godunov update without the error code (fast path): fp32 values identical to
// godunov_bl (a1 == UN or an overflowing / NaN candidate gives UN either way).
// ff = f*f, ff2 = ff + ff and ff3 = 3*ff come from the caller (once per
// slowness cell).
template <bool FAST>
__device__ __forceinline__ float godunov_v(float a, float b, float c, float f, float ff, float ff2, float ff3)
{
    // sort by bit pattern (non-negative, non-NaN inputs; see fmin_): v_min3 / v_max3 / v_med3
    const unsigned ia = __builtin_bit_cast(unsigned, a), ib = __builtin_bit_cast(unsigned, b),
                   ic = __builtin_bit_cast(unsigned, c);
    unsigned u1, u2, u3;
    // (written as asm: the instruction selector shares min(a,b) / max(a,b)
    // between the three and emits five ops)
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(u1) : "v"(ia), "v"(ib), "v"(ic));
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(u2) : "v"(ia), "v"(ib), "v"(ic));
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(u3) : "v"(ia), "v"(ib), "v"(ic));
    const float a1 = __builtin_bit_cast(float, u1), a2 = __builtin_bit_cast(float, u2),
                a3 = __builtin_bit_cast(float, u3);
    const float d2 = a2 - a1, d3 = a3 - a1;
    const float e = d3 - d2;
    const float d22 = d2 * d2, d33 = d3 * d3;
    const float t = d33 + e * e;
    const bool two = t >= ff;
    const float r2 = ff2 - d22;
    const float sm = d2 + d3;
    const float disc = ff3 - (d22 + t);     // 3D radicand, t shared with the 2D/3D test
    const float rad = two ? r2 : disc;
    const float s = FAST ? sqrt_normal(rad) : __builtin_sqrtf(rad);
    // two: 0.5 * (d2 + s); else (sm + s) * (1/3)  (same products, one multiply)
    const float y23 = ((two ? d2 : sm) + s) * (two ? 0.5f : (1.0f / 3.0f));
    // (an integer-mask choice, v_bfi_b32 on the sign of bits(d2) - bits(f),
    // measured no faster: DESIGN.md s.7, rejected variants)
    const float y = !(f > d2) ? f : y23;
    // x >= UN, +inf or NaN -> UN: unsigned min with the bits of FLT_MAX (x >= +0)
    const unsigned ix = __builtin_bit_cast(unsigned, a1 + y);
    return __builtin_bit_cast(float, __builtin_elementwise_min(ix, 0x7f7fffffu));
}
template <bool FAST>
__device__ __forceinline__ double godunov_v(double a, double b, double c, double f, double, double, double)
{
    return godunov_fast64<FAST>(a, b, c, f);
}

// ---- per-solve setup: u = u_nan, then the source boxes (EIKONAL3D_SETBCS) ----
template <typename R, int SLOWMODE>
__device__ __forceinline__ bool init_field(const FsmLaunch &L, R *u, Rsrc ur, const void *slow_model, const double *src,
                           BcBoxes &bc)
{
    const int lane = threadIdx.x;
    const R UN = Num<R>::unan();
    const uint32_t nvec = (uint32_t)(L.field_elems / 8);
    R fill[8];
#pragma unroll
    for (int i = 0; i < 8; i++) fill[i] = UN;
    for (uint32_t i = lane; i < nvec; i += 64) bstore8(ur, i * 8u * (uint32_t)sizeof(R), fill);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    bc.n = L.nsrc;
    bool ok = true;
    for (int s = 0; s < L.nsrc; s++) {
        const double *sp = src + (size_t)s * 4;
        const double ts = sp[0];
        int loc[3][3];
        const int nn[3] = {L.nx, L.ny, L.nz};
        const double org[3] = {L.x0, L.y0, L.z0};
        for (int a = 0; a < 3; a++) {
            double xs = sp[1 + a], x0 = org[a], dx = L.h;
            int n = nn[a], is;
            if (xs <= x0) is = 1;                                   // EIKONAL_SOURCE_INDEX
            else if (xs >= x0 + (double)(n - 1) * dx) is = n;
            else is = (int)((xs - x0) / dx + 0.5) + 1;
            int np = 0;                                             // EIKONAL_INIT_GRID
            loc[a][0] = loc[a][1] = loc[a][2] = -1;
            double xe = x0 + (double)(is - 1) * dx;
            if (xe > xs) { loc[a][0] = is - 1; loc[a][1] = is; np = 2; }
            else if (xe < xs) { loc[a][0] = is; loc[a][1] = is + 1; np = 2; }
            else {
                loc[a][np++] = is - 1;          // is > 0 always: the reference's isx-1 quirk
                loc[a][np++] = is;
                if (is < n - 1) loc[a][np++] = is + 1;
            }
            for (int i = 0; i < np; i++) if (loc[a][i] < 1 || loc[a][i] > n) ok = false;
            int lo = 1 << 30, hi = -1;
            for (int i = 0; i < np; i++) { lo = min(lo, loc[a][i] - 1); hi = max(hi, loc[a][i] - 1); }
            if (lane == 0) { bc.box[6 * s + 2 * a] = lo; bc.box[6 * s + 2 * a + 1] = hi; }
        }
        if (!ok) { bc.n = s; break; }
        // lanes 0..26 each own one node of the 3x3x3 candidate box
        if (lane < 27) {
            int i = lane % 3, j = (lane / 3) % 3, k = lane / 9;
            int ix = loc[0][i], iy = loc[1][j], iz = loc[2][k];
            if (ix != -1 && iy != -1 && iz != -1) {
                double x = L.x0 + (double)(ix - 1) * L.h, y = L.y0 + (double)(iy - 1) * L.h,
                       z = L.z0 + (double)(iz - 1) * L.h;
                double ddx = sp[1] - x, ddy = sp[2] - y, ddz = sp[3] - z;
                double dd = __builtin_sqrt((ddx * ddx + ddy * ddy) + ddz * ddz);
                double sl = slow_at<R, SLOWMODE>(L, slow_model, ix - 1, iy - 1, iz - 1);
                R t = (R)(ts + dd * sl);
                size_t idx = brick_index<R>(L, ix - 1, iy - 1, iz - 1);
                R cur = u[idx];
                u[idx] = (__builtin_fabs(dd) < 1.e-10) ? t : (cur < t ? cur : t);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    return ok;
}

// Work queue: 8 groups (blockIdx % 8, which the dispatcher deals round-robin
// over the XCDs -- speed only, never correctness); group g first drains the
// contiguous solve range [g*S/8, (g+1)*S/8) -- consecutive solves share a model,
// so a model's cells stay in one XCD's L2 -- then steals from the others.
__device__ __forceinline__ int next_solve(const FsmLaunch &L, int &pass)
{
    const int g0 = blockIdx.x & 7;
    while (pass < 8) {
        const int g = (g0 + pass) & 7;
        const int lo = (int)((long long)L.nsolve * g / 8), hi = (int)((long long)L.nsolve * (g + 1) / 8);
        unsigned i = 0;
        if (threadIdx.x == 0) i = atomicAdd(L.counter + 32 * g, 1u);
        i = __builtin_amdgcn_readfirstlane(__shfl(i, 0, 64));
        if ((int)i < hi - lo) return L.solve_order ? L.solve_order[lo + (int)i] : lo + (int)i;
        pass++;
    }
    return -1;
}

// Diagonal order of the tiles for the (+x, +y) sweep: by txs + tys, then tys.
// Other directions flip tx / ty; every tile comes after its upwind neighbours.
__device__ __forceinline__ void build_order(const FsmLaunch &L, int *order)
{
    for (int id = threadIdx.x; id < L.ntiles; id += 64) {
        const int txs = id % L.ntx, tys = id / L.ntx, dg = txs + tys;
        int rank = 0;
        for (int e = 0; e < dg; e++)
            rank += min(e, L.nty - 1) - max(0, e - L.ntx + 1) + 1;
        rank += tys - max(0, dg - L.ntx + 1);
        order[rank] = txs | (tys << 16);
    }
}

// ---- stream machinery shared by both sweep kernels ----------------------
// Position of a lane in the stream of one sweep: stream position sp, its ring
// slot ri = sp mod nr, and the step zbs (0..kb-1) inside the position,
// advanced one virtual brick per macro step.
struct Pos {
    int vb, sp, zbs, ri;
};
__device__ __forceinline__ void pos_init(Pos &p, int vb, int kb, int nr)
{
    p.vb = vb;
    const int v = vb < 0 ? 0 : vb;
    p.sp = v / kb; p.zbs = v - p.sp * kb;
    p.ri = p.sp % nr;
}
__device__ __forceinline__ void pos_adv(Pos &p, int kb, int nr)
{
    // branch-free (lanes differ in vb): selects instead of exec-mask branches
    const int z1 = p.zbs + (p.vb >= 0 ? 1 : 0);
    const bool wrap = z1 == kb;
    const int r1 = p.ri + (wrap ? 1 : 0);
    p.zbs = wrap ? 0 : z1;
    p.sp += wrap ? 1 : 0;
    p.ri = r1 == nr ? 0 : r1;
    p.vb++;
}
__device__ __forceinline__ bool pos_valid(const Pos &p, int nstream)
{
    return p.vb >= 0 && p.sp < nstream;
}

// Column flags (written at admission, per lane and position) and brick flags.
enum {
    C_ACT = 1,      // column inside the grid
    C_U0 = 2,       // first visit of the z-block in this iteration: store u0
    C_PART = 4,     // tile cut by the grid's x or y end (generic path)
    C_00 = 8,       // column of node (0,0,0) (ierr, generic path)
    C_BC = 16,      // column crosses a boundary-condition box in x and y
    C_BLK = 32,     // the position holds a z-block (not a bubble)
    C_ZH = 64,      // run start inside the column: the z-upwind value comes from HBM
    C_XOWN = 128,   // x-edge lane whose x neighbour is outside the grid: its x halo is its own column
    C_YOWN = 256,   // the same for the y halo
    F_VALID = 128, F_FIRST = 256, F_LAST = 512, F_SLOW = 1024, F_ZH = 2048   // BInfo.fl (meta bits 0-6 +)
};
// column info word w: flags (bits 0-8) | tz << 9 (7 bits) | (signed) cell-cache base << 16
__device__ __forceinline__ int ci_tz(unsigned w) { return (int)((w >> 9) & 0x7f); }
__device__ __forceinline__ int ci_ccb(unsigned w) { return (int)w >> 16; }

// Column info of this lane for the tile of a run (entry: tx | ty << 12): the
// own column offset, the tile-level flags and the lane's cell column
// (cyl * ncxt + cxl).  The x/y halo of a tile-edge lane is the neighbour
// column (a lane-constant offset from the own column, halo_delta), or the
// lane's own column where the grid ends (C_XOWN / C_YOWN: the reference's
// missing neighbour is the node itself, so the halo then holds exactly the
// node's old value).
struct ColTile {
    int tile;                    // tx | ty << 12 of the cached tile, -1 none
    uint32_t col;
    int fl, cl;
};
template <typename R>
__device__ __forceinline__ void column_tile(const FsmLaunch &L, const BcBoxes &bc, int entry, int lx, int ly,
                                            int lxs, int lys, int rx, int ry, ColTile &t)
{
    const int tx = entry & 0xfff, ty = (entry >> 12) & 0xfff;
    const int x = tx * 8 + lx, y = ty * 8 + ly;
    const uint32_t st = tile_bytes<R>(L);
    const uint32_t col = (uint32_t)(ty * L.ntx + tx) * st + (uint32_t)colpos(lx, ly) * 128u;
    int m = (x < L.nx && y < L.ny) ? C_ACT : 0;
    if (lxs == 0 || lxs == 7) {
        const int xn = x + (((lxs == 0) != (rx != 0)) ? -1 : 1);
        if (!(xn >= 0 && xn < L.nx)) m |= C_XOWN;
    }
    if (lys == 0 || lys == 7) {
        const int yn = y + (((lys == 0) != (ry != 0)) ? -1 : 1);
        if (!(yn >= 0 && yn < L.ny)) m |= C_YOWN;
    }
    if (tx * 8 + 8 > L.nx || ty * 8 + 8 > L.ny) m |= C_PART;
    if (x == 0 && y == 0) m |= C_00;
    for (int k = 0; k < bc.n; k++) {
        const int *q = bc.box + 6 * k;
        if (x >= q[0] && x <= q[1] && y >= q[2] && y <= q[3]) m |= C_BC;
    }
    int cx0, ncxt, cy0, ncyt;
    tile_cells(tx, L.nx, L.magic_rx, cx0, ncxt);
    tile_cells(ty, L.ny, L.magic_ry, cy0, ncyt);
    const int xc = x < L.nx ? x : L.nx - 1, yc = y < L.ny ? y : L.ny - 1;
    const int cxl = (int)(((unsigned)xc * L.magic_rx) >> 20) - cx0;
    const int cyl = (int)(((unsigned)yc * L.magic_ry) >> 20) - cy0;
    t.tile = entry & 0xffffff;
    t.col = col;
    t.fl = m;
    t.cl = cyl * ncxt + cxl;
}
// Column info word of block tz of the cached tile at ring slot ri:
// flags | tz << 8 | cell-cache base << 16, cell of node z = cc[base + z cell].
__device__ __forceinline__ unsigned column_word(const FsmLaunch &L, int kb, const ColTile &t, int tz, int ri,
                                                int u0flag, int zh)
{
    int cz0, nczb;
    block_zcells(L, kb, tz, cz0, nczb);
    const int ccb = ri * L.ccb + t.cl * nczb - cz0;
    const int m = t.fl | C_BLK | (u0flag ? C_U0 : 0) | (zh ? C_ZH : 0);
    return (unsigned)(m | (tz << 9) | (ccb << 16));
}

// Halo columns of a tile (sweep-relative lanes): j = 0..7 the x-upwind halos
// of lanes (0, j), 8..15 the x-downwind halos of lanes (7, j - 8), 16..23 the
// y-upwind halos of lanes (j - 16, 0), 24..31 the y-downwind halos of lanes
// (j - 24, 7).  All 64 lanes load them: lane k fetches half k & 1 (4 z) of
// column k >> 1's segment for that edge lane's brick vb+2, so one 16-B (fp32)
// load per lane replaces four 32-B loads of which 48 lanes were idle.
__device__ __forceinline__ int halo_edge_lane(int j)
{
    return j < 8 ? j * 8 : j < 16 ? (j - 8) * 8 + 7 : j < 24 ? j - 16 : 56 + (j - 24);
}
// Byte offset from a tile-edge lane's own column to the neighbour column
// its halo column j reads (sweep direction rx, ry; he = the edge lane): the
// neighbour tile (+-1 in x, +-ntx in y) and the column on that tile's facing
// edge.
__device__ __forceinline__ uint32_t halo_delta(const FsmLaunch &L, uint32_t tile_bytes, int j, int he, int rx, int ry)
{
    const int lxs = he & 7, lys = he >> 3;
    const int lx = rx ? 7 - lxs : lxs, ly = ry ? 7 - lys : lys;
    if (j < 16) {
        const int dx = ((j < 8) != (rx != 0)) ? -1 : 1;
        return (uint32_t)(dx * (int)tile_bytes) + (uint32_t)((colpos((lx + dx) & 7, ly) - colpos(lx, ly)) * 128);
    }
    const int dy = ((j < 24) != (ry != 0)) ? -1 : 1;
    return (uint32_t)(dy * L.ntx * (int)tile_bytes) + (uint32_t)((colpos(lx, (ly + dy) & 7) - colpos(lx, ly)) * 128);
}
__device__ __forceinline__ unsigned dpp_swap_pair(unsigned v)
{
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
}
// Cell cache (SLOWMODE 2): the slowness cells of a z-block (2 x 2 x 8 at
// nref = 4, kb = 4), one buffer per ring slot.  Loads for the block at
// position k are issued two macro steps before lane (0,0) enters it and
// written at the end of that step; the slot's previous block (position
// k - nr) has no reader left.  fp32 entries hold f = s*h (the product the
// update uses, rounded once as before); fp64 entries hold s.
template <int CCR>
__device__ __forceinline__ void cc_issue(const FsmLaunch &L, int kb, Rsrc sr, int entry, float (&v)[CCR], int &size)
{
    const int lane = threadIdx.x;
    const int tx = entry & 0xfff, ty = (entry >> 12) & 0xfff, tz = (entry >> 24) & 0xff;
    int cx0, ncxt, cy0, ncyt, cz0, nczb;
    tile_cells(tx, L.nx, L.magic_rx, cx0, ncxt);
    tile_cells(ty, L.ny, L.magic_ry, cy0, ncyt);
    block_zcells(L, kb, tz, cz0, nczb);
    size = entry >= 0 ? ncxt * ncyt * nczb : 0;
    // small exact divisions (idx < 64 * CCR <= 256, divisors <= 256): the
    // quotient of (a + 1/2) / d is >= 1/512 away from an integer, far above
    // the error of v_rcp_f32 and one rounding, so truncation gives floor(a / d)
    const float rz = __builtin_amdgcn_rcpf((float)nczb), rx = __builtin_amdgcn_rcpf((float)ncxt);
#pragma unroll
    for (int r = 0; r < CCR; r++) {
        const int idx = lane + 64 * r;
        const int t = (int)(((float)idx + 0.5f) * rz), cz = idx - t * nczb;
        const int cyl = (int)(((float)t + 0.5f) * rx), cxl = t - cyl * ncxt;
        const uint32_t off = (uint32_t)((((cz0 + cz) * L.ncy + cy0 + cyl) * L.ncx) + cx0 + cxl) * 4u;
        v[r] = bload1f(sr, idx < size ? off : OOB);
    }
}
template <typename R, int CCR>
__device__ __forceinline__ void cc_write(const FsmLaunch &L, float *cc, int ri, const float (&v)[CCR], int size,
                                         float h)
{
    const int lane = threadIdx.x;
#pragma unroll
    for (int r = 0; r < CCR; r++) {
        const int idx = lane + 64 * r;
        if (idx < size) cc[ri * L.ccb + idx] = sizeof(R) == 4 ? v[r] * h : v[r];
    }
}

// Stream state of a sweep (wave-uniform): the next tile (diagonal order) to
// scan, the run in progress (tile, next sweep-relative z-block, first block
// of the run) and the bubbles still owed before it.
struct Stream {
    int cursor, tile, k, k0, wait;
};

}  // namespace
