// fsm_common.h -- shared host/device definitions for the batched fast-sweeping
// eikonal solve (MI355X / gfx950).  Not a public header: the C-ABI lives in
// include/mceik_eikonal.h and include/mceik.h.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

#define MCEIK_TILE 8             // 8x8 column tile = one 64-lane wave
#define MCEIK_BRICK 512          // 8x8 columns x 8 z = one brick
#define MCEIK_KB 4               // bricks per z-block (stream position) when the block tables fit in LDS
#define MCEIK_MAX_BLOCKS 1024    // per-block clocks in LDS: at most this many z-blocks per field
#define MCEIK_AHEAD 2            // own segments are loaded this many macro steps ahead (3 measured slower:
                                 // DESIGN.md s.7, rejected variants)

// One batched launch: nsolve = nmodel * nstat solves; solve id = model*nstat + station.
struct FsmLaunch {
    int nx, ny, nz;              // eikonal grid (nodes); dx = dy = dz = h
    int ntx, nty, nzb, ntiles;
    int kb, nzk, nblocks, nr;    // bricks per z-block (= steps per stream position), z-blocks per column,
                                 // z-blocks per field, stream ring size (positions in flight)
    int infl, vis;               // positions a visit stays in flight / min distance to an upwind x/y visit
    int ccb;                     // cell-cache floats per stream position (SLOWMODE 2)
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
    void *zf;                    // held stream: per-wave copies of every z-block's lowest and highest node per
                                 // column, [nblocks][2][64 columns lx + 8 ly] R (zf_bytes), the values a run
                                 // start / end reads across a z-block boundary
    int slot_per_solve;          // 1: field slot = solve id; 0: slot = blockIdx.x (scratch)
    const int *ev_node;          // event nodes (x-fastest linear index), may be null
    int nev;
    float *ttab;                 // [nsolve][nev] travel times at events (fp32), may be null
    int *niter;                  // [nsolve] iterations executed, may be null
    int *ierr;                   // [nsolve] reference ierr semantics, may be null
    int cell_cache;              // slow_mode 1: every tile's cells fit the LDS cell cache
    int fast_sqrt;               // host-validated: f = s*h >= 1e-12 (sqrt_normal is exact for x >= 2^-104, profiles/r03_sqrt)
    unsigned *counter;           // 8 work-queue heads, 128 B apart (zeroed before the launch)
    unsigned long long *iter_total;   // += iterations of every solve (roofline accounting), may be null
    unsigned long long *visit_stats;  // [4] += brick visits, column-segment updates, changed segments, macro steps; may be null
    const int *solve_order;      // queue slot -> solve id, or null (slot = solve)
    unsigned long long *solve_clock;  // [nsolve][2] realtime at solve start / end, or null
    int max_waves;               // host only: cap on resident waves (0 = occupancy x CUs)
    unsigned long long *traffic; // [MCEIK_TRAFFIC_N] requested bytes by category (MCEIK_TRAFFIC builds), or null
    int step_z;                  // host only: 8 forces the 8-z kernel, 0 = the launch's choice
    const float *ev_frac;        // [nev][3] trilinear fractions (ev_node = lowest corner), or null = node value
    const int *model_phase;      // slow_mode 1: model m uses slow entry m * nphase + model_phase[m], or null
    int nphase;
    const unsigned char *skip;   // [nphase][nstat]: solve of (phase, station) skipped when set, or null
    unsigned long long *solve_count;  // += solves executed, or null
    // Multi-step sampler launch (fsm16 kernel only; null mc_dev: a plain
    // batch).  Solves of steps mc_step0 .. mc_step0 + mc_nsteps - 1; the wave
    // that completes a chain's solves of a step runs the chain's accept, kept
    // state and next proposal (mcmc_device.h).  mc_sync: [8] group owner (XCD
    // id + 1) | [8][32] group tickets | [nchains] steps ready | [nchains]
    // solves done (zeroed before every launch) | [1] broken-queue flag (zeroed
    // once at init; the sampler checks it at every synchronisation).
    const void *mc_dev;          // the sampler's McmcDev (device copy)
    unsigned *mc_sync;
    unsigned mc_spin_limit;      // polls of a step-ready wait before the queue counts as broken
    int mc_step0, mc_nsteps;
    int mc_nburn, mc_keepk, mc_maxs, mc_nkept0;   // kept-state slots (mceik_mcmc_run's bookkeeping)
};
#define MC_SYNC_WORDS(nchains) (8 + 8 * 32 + 2 * (nchains) + 1)

// Phase of model m of a batch without a phase map: models [chain][phase]
// when nphase > 1 (the sampler's full forward), else 0.
static inline __host__ __device__ int fsm_plain_phase(const FsmLaunch &L, int m)
{
    return L.nphase > 1 ? m % L.nphase : 0;
}

// Inversion-grid slowness entry of model m (slow_mode 1).
static inline __host__ __device__ size_t fsm_slow_entry(const FsmLaunch &L, int m)
{
    return L.model_phase ? (size_t)m * L.nphase + L.model_phase[m] : (size_t)m;
}

static inline __host__ __device__ int mceik_div_up(int a, int b) { return (a + b - 1) / b; }
// bytes of one wave's z-face copies (FsmLaunch.zf)
static inline __host__ __device__ size_t zf_bytes(const FsmLaunch &L, size_t es) { return (size_t)L.nblocks * 128 * es; }

// Debug / accounting counters in LDS: [0..3] visit statistics; MCEIK_TRAFFIC
// builds add [8..15], the requested global-memory bytes of the wave's current
// sweep by category (flushed to FsmLaunch.traffic after every sweep).
#if defined(MCEIK_TRAFFIC)
#define MCEIK_SCRATCH_BYTES 64
#else
#define MCEIK_SCRATCH_BYTES 32
#endif
#define MCEIK_TRAFFIC_N 8       // categories: own load, halo load, z-upwind load, own store, u0 store,
                                // cell-cache load, verify loads (u + u0), init fill + BC + table gather

// LDS of one solve wave (byte offsets, shared by host and device):
//  0 BC boxes [nsrc][6] int (EIKONAL3D_SETBCS, fsm3d.f90:762-840; no source limit beyond LDS) | 1 cell cache [nr][ccb] float (cached mode) |
//  2 diagonal tile order int [ntiles] | 3 lastproc int [nblocks] | 4 lastchg int [nblocks] |
//  5 (unused: a block's first visit in an iteration is lastproc < the iteration's first clock) |
//  6 stream entries int [nr] + block ids int [nr] | 7 run scratch int [8] | 8 staged f [8][64] R (uncached) |
//  9 neighbour rows XR, 10 neighbour rows XN: [2 halves][80 rows][4] R each -- row l < 64 holds lane l's
//    8 z values (XR: its results of the last step, XN: its next brick), rows 64..79 the tile's halo columns |
//  11 column info [nr][64] uint2 {own column offset, flags | tz | cell-cache base}
//    (fp64: XN is followed by HOLD [2][64] x 16 B, the held later halves of the whole-line own
//    loads of the compile-time-kb instances, fsm_kernel.hip line_issue64)
#define MCEIK_CC_MAX 256         // cell-cache floats per position, upper bound
#define MCEIK_F64_HOLD (2 * 64 * 16)
#define MCEIK_SMEM_ARRAYS 14      // (+ 12 tile frontier u8 [ntiles], 13 two block bitmaps: the held stream of
                                  //  the compact layout, fsm_hold.h)
#define MCEIK_XROWS 80           // neighbour-row array: 64 lanes + 8 x-halo + 8 y-halo rows
static inline __host__ __device__ size_t mceik_align16(size_t v) { return (v + 15) & ~(size_t)15; }
// The compile-time-kb cell-cache kernel (fsm_kernel.hip variant 8, the C3
// sampler instance) uses a FIXED layout: every array base is a constant, so
// LDS addresses fold into instruction offsets instead of occupying SGPRs
// (the kernel runs at the SGPR limit).  Runtime-sized arrays (tile order,
// BC boxes) come last; the block tables are sized for MCEIK_MAX_BLOCKS.
#define FSMF_NR (2 + (16 + MCEIK_KB - 1) / MCEIK_KB)
#define FSMF_CINFO 0
#define FSMF_XR (FSMF_CINFO + FSMF_NR * 64 * 8)
#define FSMF_XN (FSMF_XR + 2 * MCEIK_XROWS * 16)
#define FSMF_CC (FSMF_XN + 2 * MCEIK_XROWS * 16)
#define FSMF_RING (FSMF_CC + FSMF_NR * 64 * 4)
#define FSMF_SCRATCH (FSMF_RING + 64)
#define FSMF_LASTPROC (FSMF_SCRATCH + MCEIK_SCRATCH_BYTES)
#define FSMF_LASTCHG (FSMF_LASTPROC + MCEIK_MAX_BLOCKS * 4)
#define FSMF_ORDER (FSMF_LASTCHG + MCEIK_MAX_BLOCKS * 4)
static inline __host__ __device__ bool fsm_fixed_layout(const FsmLaunch &L, size_t es)
{
    return es == 4 && L.slow_mode != 0 && L.cell_cache && L.fast_sqrt && L.nrz == 4 && L.ccb <= 64 &&
           L.kb == MCEIK_KB && L.nr == FSMF_NR && L.nblocks <= MCEIK_MAX_BLOCKS;
}
// The compact layout of the fp64 compile-time-kb instances (fsm_kernel.hip
// variants 15, 16; Smem<R, true>): 16-bit block clocks rebased per iteration
// (an iteration takes at most 8 (nblocks (1 + vis) + infl) + 64 < 2^16
// clocks at nblocks <= MCEIK_MAX_BLOCKS, kb = MCEIK_KB), one meta word per
// lane and position, the tile base per position in the ring.
static inline __host__ __device__ bool fsm_compact_layout(const FsmLaunch &L, size_t es)
{
    return es == 8 && L.slow_mode != 0 && L.cell_cache && L.nrz == 4 && L.ccb <= 64 && L.kb == MCEIK_KB &&
           L.nblocks <= MCEIK_MAX_BLOCKS;
}
static inline __host__ __device__ size_t fsm_smem_layout(const FsmLaunch &L, size_t es, size_t *off)
{
    if (fsm_fixed_layout(L, es)) {
        off[11] = FSMF_CINFO; off[9] = FSMF_XR; off[10] = FSMF_XN; off[1] = FSMF_CC;
        off[6] = FSMF_RING; off[7] = FSMF_SCRATCH; off[3] = FSMF_LASTPROC; off[4] = FSMF_LASTCHG;
        off[5] = FSMF_ORDER; off[2] = FSMF_ORDER; off[8] = FSMF_ORDER;          // sf: unused (cells cached)
        off[0] = FSMF_ORDER + mceik_align16((size_t)L.ntiles * 4);
        off[12] = off[13] = off[0];                                       // (no held stream)
        return off[0] + mceik_align16((size_t)(L.nsrc > 0 ? L.nsrc : 1) * 6 * 4);
    }
    const bool cached = L.slow_mode != 0 && L.cell_cache;
    const size_t nt = (size_t)L.ntiles, nb = (size_t)L.nblocks, nr = (size_t)L.nr;
    size_t o = 0;
    off[0] = o; o += mceik_align16((size_t)(L.nsrc > 0 ? L.nsrc : 1) * 6 * 4);
    off[1] = o; o += cached ? mceik_align16(nr * L.ccb * 4) : 0;
    const bool cmp = fsm_compact_layout(L, es);
    off[2] = o; o += mceik_align16(nt * 4);
    off[3] = o; o += mceik_align16(nb * (cmp ? 2 : 4));
    off[4] = o; o += mceik_align16(nb * (cmp ? 2 : 4));
    off[5] = o;
    off[6] = o; o += mceik_align16(nr * (cmp ? 16 : 8));       // (cmp: + the held stream's change masks)
    off[12] = o; o += cmp ? mceik_align16(nt) : 0;
    off[13] = o; o += cmp ? mceik_align16((nb + 31) / 32 * 4 * 2) : 0;
    off[7] = o; o += MCEIK_SCRATCH_BYTES;
    off[8] = o; o += cached ? 0 : 512 * es;
    off[9] = o; o += 2 * MCEIK_XROWS * 4 * es;
    off[10] = o; o += 2 * MCEIK_XROWS * 4 * es + (es == 8 ? MCEIK_F64_HOLD : 0);
    off[11] = o; o += nr * 64 * (cmp ? 4 : 8);
    return o;
}
static inline size_t fsm_lds_bytes(const FsmLaunch &L, size_t es)
{
    size_t off[MCEIK_SMEM_ARRAYS];
    return fsm_smem_layout(L, es, off);
}
#define MCEIK_MAX_LDS (64 * 1024)   // dynamic LDS without a launch attribute

// ---- 16-z-step kernel (fsm16_kernel.hip, the fp32 cell-cache sampler
// instance).  A macro step updates 16 z of every lane's column (half of its
// 128-B line), so a line is consumed in two pieces instead of four.  Stream
// positions are the same z-blocks: L.kb 8-z bricks = kb/2 steps; L.kb must be
// even and >= 4 (the 16-bit block clocks below need at most 1 + vis <= 7
// positions per block and sweep).  Timing rules in steps, as for the 8-z
// kernel (fsm_geometry): infl = 1 + ceil((14 + AH) / kb16), vis =
// ceil(12 / kb16), nr = 1 + ceil((15 + AH) / kb16).
#define MCEIK_AHEAD16 2
struct Fsm16Geo {
    int nzb, kb, nr, infl, vis;  // 16-z bricks per column, steps per position, ring, in-flight, visibility
};
static inline __host__ __device__ Fsm16Geo fsm16_geo(const FsmLaunch &L)
{
    Fsm16Geo g;
    g.nzb = mceik_div_up(L.nz, 16);
    g.kb = L.kb / 2;
    g.infl = 1 + mceik_div_up(14 + MCEIK_AHEAD16, g.kb);
    g.vis = mceik_div_up(12, g.kb);
    g.nr = 1 + mceik_div_up(15 + MCEIK_AHEAD16, g.kb);
    return g;
}
static inline __host__ __device__ bool fsm16_eligible(const FsmLaunch &L, size_t es)
{
    return es == 4 && L.slow_mode != 0 && L.cell_cache && L.fast_sqrt && L.nrz == 4 && L.ccb <= MCEIK_CC_MAX &&
           L.kb >= 4 && (L.kb & 1) == 0 && L.nblocks <= MCEIK_MAX_BLOCKS && L.ntx <= 256 && L.nty <= 256;
}
// LDS of one fsm16 solve wave: 0 BC boxes | 1 cell cache [nr][ccb] float | 2 tile order int [ntiles] |
// 2 is u16 (txs | tys << 8) | 3 lastproc u16 [nblocks] | 4 lastchg u16 [nblocks] (clocks relative to the
// iteration; with the held stream (fsm_hold.h): relative to the sweep, and lastchg holds
// "need", the clock of the last settled change of the block or of a neighbour's face it shares) |
// 5 ring: entry int [nr], block id int [nr], tile base u32 [nr], change mask u32 [nr] | 6 scratch |
// 7 neighbour rows XR then XN, each [4 quarters][80 rows][4] float | 8 column meta u32 [nr][64] |
// 9 tile frontier u8 [ntiles] (z-blocks decided in this sweep) | 10 two block bitmaps u32 [nblocks / 32]
// (visited / changed in this iteration)
#define MCEIK_SMEM16_ARRAYS 11
// floats per quarter array of the neighbour rows: 80 rows of 4 plus a 16-B pad,
// so that the x-pair exchange (even lane: quarter 0, odd lane: quarter 1 of the
// same row) falls in different LDS banks (unpadded, 320 floats = 5 x 64 banks)
#define MCEIK_X16PAD 4
#define MCEIK_X16Q (MCEIK_XROWS * 4 + MCEIK_X16PAD)
#define F16_NR (1 + (15 + MCEIK_AHEAD16 + 1) / 2)      // nr at kb16 = 2
#define F16_CINFO 0
#define F16_XR (F16_CINFO + F16_NR * 64 * 4)
#define F16_CC (F16_XR + 2 * 4 * MCEIK_X16Q * 4)
#define F16_RING (F16_CC + F16_NR * 32 * 4)
#define F16_SCRATCH (F16_RING + 176)
#define F16_LASTPROC (F16_SCRATCH + MCEIK_SCRATCH_BYTES)
#define F16_LASTCHG (F16_LASTPROC + MCEIK_MAX_BLOCKS * 2)
#define F16_ORDER (F16_LASTCHG + MCEIK_MAX_BLOCKS * 2)
static inline __host__ __device__ bool fsm16_fixed_layout(const FsmLaunch &L)
{
    return fsm16_eligible(L, 4) && L.kb == 4 && L.ccb <= 32 && fsm16_geo(L).nr == F16_NR;
}
static inline __host__ __device__ size_t f16_bitmap_bytes(const FsmLaunch &L)
{
    return mceik_align16((size_t)((L.nblocks + 31) / 32) * 4 * 2);
}
static inline __host__ __device__ size_t fsm16_smem_layout(const FsmLaunch &L, size_t *off)
{
    const size_t nbox = mceik_align16((size_t)(L.nsrc > 0 ? L.nsrc : 1) * 6 * 4);
    if (fsm16_fixed_layout(L)) {
        off[8] = F16_CINFO; off[7] = F16_XR; off[1] = F16_CC; off[5] = F16_RING; off[6] = F16_SCRATCH;
        off[3] = F16_LASTPROC; off[4] = F16_LASTCHG; off[2] = F16_ORDER;
        off[9] = F16_ORDER + mceik_align16((size_t)L.ntiles * 2);
        off[10] = off[9] + mceik_align16((size_t)L.ntiles);
        off[0] = off[10] + f16_bitmap_bytes(L);
        return off[0] + nbox;
    }
    const Fsm16Geo g = fsm16_geo(L);
    const size_t nr = (size_t)g.nr, nb = (size_t)L.nblocks;
    size_t o = 0;
    off[0] = o; o += nbox;
    off[1] = o; o += mceik_align16(nr * L.ccb * 4);
    off[2] = o; o += mceik_align16((size_t)L.ntiles * 2);
    off[3] = o; o += mceik_align16(nb * 2);
    off[4] = o; o += mceik_align16(nb * 2);
    off[9] = o; o += mceik_align16((size_t)L.ntiles);
    off[10] = o; o += f16_bitmap_bytes(L);
    off[5] = o; o += mceik_align16(nr * 16);
    off[6] = o; o += MCEIK_SCRATCH_BYTES;
    off[7] = o; o += 2 * 4 * MCEIK_X16Q * 4;
    off[8] = o; o += nr * 64 * 4;
    return o;
}
static inline size_t fsm16_lds_bytes(const FsmLaunch &L)
{
    size_t off[MCEIK_SMEM16_ARRAYS];
    return fsm16_smem_layout(L, off);
}

// The held stream (fsm_hold.h) keeps 16-bit clocks relative to the sweep: a
// sweep needs at most nblocks (1 + infl) + 64 of them (between two visits at
// most infl bubbles).
// The bound at the tables' capacity and the largest infl of either kernel:
// the 16-z kernel's at kb16 = 2 (its smallest z-block) and the 8-z compact
// instances' at kb = MCEIK_KB (fsm16_geo / fsm_geometry).  The host checks
// every launch as well (mceik_fsm_batch_solve).
static inline __host__ __device__ constexpr int hold_clock_bound(int nblocks, int infl)
{
    return nblocks * (1 + infl) + 64;
}
static_assert(hold_clock_bound(MCEIK_MAX_BLOCKS, 1 + (14 + MCEIK_AHEAD16 + 1) / 2) < 65536,
              "16-bit held-stream clocks: MCEIK_MAX_BLOCKS / MCEIK_AHEAD16 too large");
static_assert(hold_clock_bound(MCEIK_MAX_BLOCKS, 1 + (14 + MCEIK_AHEAD + MCEIK_KB - 1) / MCEIK_KB) < 65536,
              "16-bit held-stream clocks: MCEIK_MAX_BLOCKS / MCEIK_AHEAD too large");

// Fills the tile geometry of a launch from nx, ny, nz (es: element bytes).
// Field layout: per 8x8 column tile, z-major groups of one
// 128-B line per column (32 fp32 / 16 fp64 z values), columns in colpos order.
// Stream: positions of kb z-bricks (a z-block); kb = 4 when
// the per-block tables fit, else the smallest power of two that fits (up to
// the whole column).  Timing rules of the lane pipeline (lag <= 14 steps;
// own segments loaded AHEAD = MCEIK_AHEAD steps ahead, so a position is
// decided AHEAD steps before lane (0,0) enters it; halos loaded 2 steps ahead; a store is visible to
// loads issued >= 3 steps later): a visit stays in flight (its changes
// unknown) for infl = 1 + ceil((14 + AHEAD) / kb) positions (decision at step Q*kb - AHEAD
// must follow the last lane's last step P*kb + kb - 1 + 14); an upwind x/y
// neighbour visit must be >= vis = ceil(12 / kb) positions back; the ring
// keeps nr = 2 + ceil(16 / kb) positions (the oldest lane reads its
// position's ring entry and cells up to kb + 13 steps after the position
// starts, the slot is rewritten nr*kb - AHEAD steps after it starts).
static inline void fsm_geometry(FsmLaunch *L, int es)
{
    L->ntx = mceik_div_up(L->nx, MCEIK_TILE);
    L->nty = mceik_div_up(L->ny, MCEIK_TILE);
    L->nzb = mceik_div_up(L->nz, MCEIK_TILE);
    L->ntiles = L->ntx * L->nty;
    int kb = L->nzb < MCEIK_KB ? L->nzb : MCEIK_KB;
    // (a z-block index must fit the 7-bit tz field of the column info word)
    while (kb < L->nzb && ((long)L->ntiles * mceik_div_up(L->nzb, kb) > MCEIK_MAX_BLOCKS || mceik_div_up(L->nzb, kb) > 128))
        kb *= 2;
    if (kb > L->nzb) kb = L->nzb;
    L->kb = kb;
    L->nzk = mceik_div_up(L->nzb, kb);
    L->nblocks = L->ntiles * L->nzk;
    L->infl = 1 + mceik_div_up(14 + MCEIK_AHEAD, kb);
    L->vis = mceik_div_up(12, kb);
    L->nr = 2 + mceik_div_up(16, kb);
    const int bpl = 16 / es;                     // 8-z bricks per 128-B line
    L->nzq = mceik_div_up(L->nzb, bpl);
    L->field_elems = (size_t)L->ntiles * L->nzq * 64 * (128 / es);
}
