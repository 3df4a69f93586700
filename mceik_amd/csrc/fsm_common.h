// fsm_common.h -- shared host/device definitions for the batched fast-sweeping
// eikonal solve (MI355X / gfx950).  Not a public header: the C-ABI lives in
// include/mceik_eikonal.h and include/mceik.h.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

#define MCEIK_MAX_SRC 8          // point sources per solve (box BCs, fsm3d.f90:762-840)
#define MCEIK_TILE 8             // 8x8 column tile = one 64-lane wave
#define MCEIK_BRICK 512          // 8x8 columns x 8 z = one brick
#define MCEIK_MIN_SB 12          // virtual bricks per tile (>= nzb); halo lags need >= 12

// One batched launch: nsolve = nmodel * nstat solves; solve id = model*nstat + station.
struct FsmLaunch {
    int nx, ny, nz;              // eikonal grid (nodes); dx = dy = dz = h
    int ntx, nty, nzb, sb, ntiles;
    int maxit, max_sweeps;       // max_sweeps < 0: unlimited (debug bisection aid)
    double tol, h, x0, y0, z0;
    double conv_thresh;          // T: nodes >= T converge iff unchanged
    int nsolve, nstat, nsrc;     // sources of station s: src[(s*nsrc + k)*4 + {0:ts,1:xs,2:ys,3:zs}]
    const double *src;
    int slow_mode;               // 0: per-node field (brick layout, R); 1: inversion grid (float)
    const void *slow;            // mode 0: [nmodel][field_elems] R ; mode 1: [nmodel][ncell] float
    int ncx, ncy, ncz, nrx, nry, nrz;
    unsigned magic_rx, magic_ry, magic_rz;   // ceil(2^20 / nr*): cell = (node * magic) >> 20
    int nzq;                     // 128-B line groups per column: ceil(nzb / (16 / es))
    size_t field_elems;          // ntiles * nzq * 64 * (128 / es)
    void *u;                     // travel-time fields (brick layout, R)
    void *u0;                    // convergence side field (same layout)
    int slot_per_solve;          // 1: field slot = solve id; 0: slot = blockIdx.x (scratch)
    const int *ev_node;          // event nodes (x-fastest linear index), may be null
    int nev;
    float *ttab;                 // [nsolve][nev] travel times at events (fp32), may be null
    int *niter;                  // [nsolve] iterations executed, may be null
    int *ierr;                   // [nsolve] reference ierr semantics, may be null
    int cell_cache;              // slow_mode 1: every tile's cells fit the LDS cell cache
    int fast_sqrt;               // host-validated: f = s*h is a normal float >= 1e-18
    unsigned *counter;           // 8 work-queue heads, 128 B apart (zeroed before the launch)
    unsigned long long *iter_total;   // += iterations of every solve (roofline accounting), may be null
    unsigned long long *visit_stats;  // [3] += tile visits, column-segment updates, changed segments; may be null
};

static inline int mceik_div_up(int a, int b) { return (a + b - 1) / b; }

// LDS of one solve wave (byte offsets, shared by host and device):
//  0 BC boxes [MAX_SRC][6] int | 1 cell cache [3][256] float (cached mode) |
//  2 diagonal tile order int | 3 lastproc int | 4 lastchg int | 5 u0 epoch u16 |
//  (all [ntiles]) 6 unused | 7 stream ring [4] int |
//  8 staged f [8][64] R (uncached) | 9 x halos [8][2][8] R | 10 y halos [8][2][8] R |
//  11 column info [4][64] uint4
#define MCEIK_CC_MAX 256
#define MCEIK_SMEM_ARRAYS 12
static inline __host__ __device__ size_t mceik_align16(size_t v) { return (v + 15) & ~(size_t)15; }
static inline __host__ __device__ size_t fsm_smem_layout(const FsmLaunch &L, size_t es, size_t *off)
{
    const bool cached = L.slow_mode != 0 && L.cell_cache;
    const size_t nt = (size_t)L.ntiles;
    size_t o = 0;
    off[0] = o; o += mceik_align16(MCEIK_MAX_SRC * 6 * 4);
    off[1] = o; o += cached ? 3 * MCEIK_CC_MAX * 4 : 0;
    off[2] = o; o += mceik_align16(nt * 4);
    off[3] = o; o += mceik_align16(nt * 4);
    off[4] = o; o += mceik_align16(nt * 4);
    off[5] = o; o += mceik_align16(nt * 2);
    off[6] = o;                                   // (unused)
    off[7] = o; o += 32;                          // ring[4] + debug[4]
    off[8] = o; o += cached ? 0 : 512 * es;
    off[9] = o; o += 128 * es;
    off[10] = o; o += 128 * es;
    off[11] = o; o += 4 * 64 * 16;
    return o;
}
static inline size_t fsm_lds_bytes(const FsmLaunch &L, size_t es)
{
    size_t off[MCEIK_SMEM_ARRAYS];
    return fsm_smem_layout(L, es, off);
}
#define MCEIK_MAX_LDS (64 * 1024)   // dynamic LDS without a launch attribute

// Fills the tile geometry of a launch from nx, ny, nz (es: element bytes).
// Field layout: per 8x8 column tile, z-major groups of one
// 128-B line per column (32 fp32 / 16 fp64 z values), columns in colpos order.
static inline void fsm_geometry(FsmLaunch *L, int es)
{
    L->ntx = mceik_div_up(L->nx, MCEIK_TILE);
    L->nty = mceik_div_up(L->ny, MCEIK_TILE);
    L->nzb = mceik_div_up(L->nz, MCEIK_TILE);
    L->sb = L->nzb > MCEIK_MIN_SB ? L->nzb : MCEIK_MIN_SB;
    L->ntiles = L->ntx * L->nty;
    const int bpl = 16 / es;                     // 8-z bricks per 128-B line
    L->nzq = mceik_div_up(L->nzb, bpl);
    L->field_elems = (size_t)L->ntiles * L->nzq * 64 * (128 / es);
}
