// fsm16_kernel.hip -- the fp32 cell-cache sampler instance of the batched
// fast-sweeping solve with 16-z macro steps (gfx950).
//
// Same schedule and update DAG as fsm_kernel.hip (EIKONAL3D_FSM /
// EVAL_UPDATE3D / UPDATE3D / SOLVE_HAMILTONIAN3D, fsm3d.f90:28-99, 419-693;
// DESIGN.md s.3): one 64-lane wave per (model, station) solve, an 8x8 column
// tile per stream position, lane (lx, ly) one step behind its upwind x/y
// neighbours, z-blocks admitted only when their inputs changed.  What differs
// is the step: a lane updates 16 z per step, half of its column's 128-B line
// (32 fp32 z), so every line is read in two 64-B pieces one step apart instead
// of four 32-B pieces over four steps.  With ~100 lines open per wave and 256
// waves per XCD sharing a 4 MB L2, the 8-z kernel re-fetched lines between
// pieces (1.7x the requested read bytes) and wrote every changed 32-B segment
// as a 64-B request (2x); the 16-z step halves both the re-fetch chances and
// the write granularity loss, and the per-step bookkeeping is spread over
// twice the nodes.  Results are bitwise those of the 8-z kernel and the fp32
// twin (oracle/fsm_impl.inc): the node update order is a topological order of
// the same DAG and every skipped block is provably unchanged.
//
// Instance: fp32, inversion-cell slowness through the LDS cell cache
// (f = s*h per cell), nrz = 4 (a brick's 16 slots cover 4 cells in z), the
// correctly rounded fast sqrt (host-validated), L.kb even and >= 4.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fsm_common.h"
#include "fsm_device.h"
#include "fsm_hold.h"
#include "fsm_update.h"
#include "mcmc_device.h"

namespace {

// byte offset of 16-z brick zb inside a column's line group (two per line)
__device__ __forceinline__ uint32_t zoff16(int zb)
{
    const uint32_t u = (uint32_t)zb;
    return ((u >> 1) << 13) | ((u & 1u) << 6);
}

// Phase clocks (MCEIK_PHASECLK instrumentation builds, with MCEIK_TRAFFIC for
// the counters' plumbing): shader-clock cycles of a step's phases, summed per
// wave into the traffic categories 0..6 in place of bytes -- 0 prefetch issue,
// 1 u0 copies, 2 brick update, 3 load waits / row writes / stores, 4 stream
// decision (fsm_hold.h hold_decide), 5 its admission (ring, column meta, cell
// cache loads), 6 the sweep outside its step loop; 7 counts hold_decide's
// window rounds.  The clock reads wait for the
// wave's outstanding LDS and scalar loads, so phases are slightly serialised.
#ifdef MCEIK_PHASECLK
#undef TRAF
#undef TRAFU
#define TRAF(S, k, pred, bytes) do { } while (0)
#define TRAFU(S, k, bytes) do { } while (0)
#define PCLK(k)                                                                                         \
    do {                                                                                                \
        const unsigned long long t_ = __builtin_readcyclecounter();                                     \
        if (threadIdx.x == 0) S.scratch[8 + (k)] += (int)(t_ - pclk_t);                                 \
        pclk_t = t_;                                                                                    \
    } while (0)
#else
#define PCLK(k) do { } while (0)
#endif

// ---- LDS ------------------------------------------------------------------
struct Smem16 {
    int *box;                    // BC boxes [nsrc][6]
    float *cc;                   // cell cache [nr][ccb] (f = s*h)
    unsigned short *order;       // diagonal tile order: txs | tys << 8 (ntx, nty <= 256)
    unsigned short *lastproc;    // per z-block clock (relative to the iteration) of the last visit
    unsigned short *lastchg;     //   ... of the last visit that changed it
    int *ring_e, *ring_b;        // per position (mod nr): entry tx | ty << 12 | tz << 24 (bubble -1), block id
    unsigned *ring_base;         //   ... byte offset of the tile's line groups
    unsigned *fmask;             //   ... held stream: what the visit changed (fsm_hold.h)
    int *scratch;                // visit statistics / traffic counters
    float *xr;                   // neighbour rows XR [4][80][4], then XN (same shape)
    unsigned *meta;              // [nr][64] column meta (flags | tz << 9 | cell-cache base << 16)
    unsigned char *fz;           // held stream: per tile, the z-blocks decided in this sweep (sweep z order)
    unsigned *vbits, *cbits;     // held stream: blocks visited / changed in this iteration (bitmaps)
};
template <bool FIXED>
__device__ __forceinline__ Smem16 smem16_bind(const FsmLaunch &L, unsigned char *base)
{
    size_t off[MCEIK_SMEM16_ARRAYS];
    if (FIXED) {         // fsm16_fixed_layout(): constants (checked on the host)
        off[8] = F16_CINFO; off[7] = F16_XR; off[1] = F16_CC; off[5] = F16_RING; off[6] = F16_SCRATCH;
        off[3] = F16_LASTPROC; off[4] = F16_LASTCHG; off[2] = F16_ORDER;
        off[9] = F16_ORDER + mceik_align16((size_t)L.ntiles * 2);
        off[10] = off[9] + mceik_align16((size_t)L.ntiles);
        off[0] = off[10] + f16_bitmap_bytes(L);
    } else {
        fsm16_smem_layout(L, off);
    }
    const int nr = fsm16_geo(L).nr;
    Smem16 S;
    S.box = reinterpret_cast<int *>(base + off[0]);
    S.cc = reinterpret_cast<float *>(base + off[1]);
    S.order = reinterpret_cast<unsigned short *>(base + off[2]);
    S.lastproc = reinterpret_cast<unsigned short *>(base + off[3]);
    S.lastchg = reinterpret_cast<unsigned short *>(base + off[4]);
    S.ring_e = reinterpret_cast<int *>(base + off[5]);
    S.ring_b = S.ring_e + (FIXED ? F16_NR : nr);
    S.ring_base = reinterpret_cast<unsigned *>(S.ring_b + (FIXED ? F16_NR : nr));
    S.fmask = S.ring_base + (FIXED ? F16_NR : nr);
    S.fz = base + off[9];
    S.vbits = reinterpret_cast<unsigned *>(base + off[10]);
    S.cbits = S.vbits + (L.nblocks + 31) / 32;
    S.scratch = reinterpret_cast<int *>(base + off[6]);
    S.xr = reinterpret_cast<float *>(base + off[7]);
    S.meta = reinterpret_cast<unsigned *>(base + off[8]);
    return S;
}

// Neighbour rows (element offsets into S.xr): array arr (0 = XR: a lane's
// results of its last step; 1 = XN: its next brick), quarter q (4 z), row
// (lane 0..63, halo rows 64..79 as in fsm_kernel.hip).
#define XROW16(arr, q, row) (((arr) * 4 + (q)) * MCEIK_X16Q + (row) * 4)
typedef float f4v16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_w4(float *p, float a, float b, float c, float d)
{
    *reinterpret_cast<f4v16 *>(p) = f4v16{a, b, c, d};
}
__device__ __forceinline__ void lds_r4(const float *p, float &a, float &b, float &c, float &d)
{
    const f4v16 v = *reinterpret_cast<const f4v16 *>(p);
    a = v.x; b = v.y; c = v.z; d = v.w;
}
__device__ __forceinline__ void store_row16(float *x, int arr, int lane, const float (&v)[16])
{
#pragma unroll
    for (int q = 0; q < 4; q++) lds_w4(x + XROW16(arr, q, lane), v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}
__device__ __forceinline__ void load_row16(const float *x, int arr, int row, float (&v)[16])
{
#pragma unroll
    for (int q = 0; q < 4; q++) lds_r4(x + XROW16(arr, q, row), v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}
// half h (8 z: quarters 2h, 2h+1) of a row
__device__ __forceinline__ void load_half16(const float *x, int arr, int row, int h, float (&v)[8])
{
    lds_r4(x + XROW16(arr, 2 * h, row), v[0], v[1], v[2], v[3]);
    lds_r4(x + XROW16(arr, 2 * h + 1, row), v[4], v[5], v[6], v[7]);
}
// halo staging: lane k holds half (k & 1) of halo column j = k >> 1
__device__ __forceinline__ void halo_stage16(float *x, int lane, const float (&v)[8])
{
    const int j = lane >> 1, h = lane & 1;
    const int arr = (j >> 3) & 1, row = 64 + ((j >> 4) << 3) + (j & 7);
    lds_w4(x + XROW16(arr, 2 * h, row), v[0], v[1], v[2], v[3]);
    lds_w4(x + XROW16(arr, 2 * h + 1, row), v[4], v[5], v[6], v[7]);
}

// The fixed instance (2-step positions) loads whole own lines (FL), decodes
// lean position words (LEAN) and loads whole halo lines (HFL); every instance
// runs the held stream (fsm_hold.h: face-level change marks, blocks with an
// in-flight dependency and no settled reason wait instead of being visited).
// The brick update reads its neighbour rows in four passes of 4 z (v39: half
// the neighbour registers of two 8-z passes).
#define NPASS16 4
// BInfo16.w1 bit 24: the brick is the last of its position below the column end, so its z-downwind
// node is loaded from HBM (into the z-boundary register with the run-start node) for a run that
// does not continue
#define W1_ZD (1u << 24)

// ---- global loads / stores of 64-B segments ------------------------------
// Pair-coalesced (lanes 2i, 2i+1 = x neighbours): each instruction makes both
// lanes of a pair read the same line, so it touches 32 lines instead of 64.
//   i0: even own q0,     odd partner's q1     (even's line)
//   i1: even own q2,     odd partner's q3     (even's line)
//   i2: even partner q0, odd own q1           (odd's line)
//   i3: even partner q2, odd own q3           (odd's line)
// even then holds E0 E2 O0 O2 and odd E1 E3 O1 O3, written straight into
// the neighbour rows they belong to (raw_write below).
__device__ __forceinline__ void seg_issue(Rsrc r, uint32_t seg, float (&a)[16])
{
    const bool odd = threadIdx.x & 1;
    const uint32_t segp = dpp_swap_pair(seg);
    float t[4];
    bload4(r, odd ? segp + 16u : seg, t);
    a[0] = t[0]; a[1] = t[1]; a[2] = t[2]; a[3] = t[3];
    bload4(r, odd ? segp + 48u : seg + 32u, t);
    a[4] = t[0]; a[5] = t[1]; a[6] = t[2]; a[7] = t[3];
    bload4(r, odd ? seg + 16u : segp, t);
    a[8] = t[0]; a[9] = t[1]; a[10] = t[2]; a[11] = t[3];
    bload4(r, odd ? seg + 48u : segp + 32u, t);
    a[12] = t[0]; a[13] = t[1]; a[14] = t[2]; a[15] = t[3];
}
// The pair exchange through the neighbour rows instead of DPP swaps (no
// VALU): the raw quarters of seg_issue are written straight into the rows
// they belong to -- even lane: own q0, own q2, odd's q0, odd's q2; odd lane:
// even's q1, even's q3, own q1, own q3, i.e. base pair_row(arr) + {0, 2Q, 4,
// 2Q + 4} floats -- and a paired store reads its operands back the same way
// from the XR rows (raw_read), so both lanes of an instruction hit one line.
#define XQE MCEIK_X16Q           // floats per quarter array
__device__ __forceinline__ int pair_row(int arr, int lane)
{
    return (lane & 1) ? XROW16(arr, 1, lane - 1) : XROW16(arr, 0, lane);
}
__device__ __forceinline__ void raw_write(float *x, int pb, const float (&a)[16])
{
    lds_w4(x + pb, a[0], a[1], a[2], a[3]);
    lds_w4(x + pb + 2 * XQE, a[4], a[5], a[6], a[7]);
    lds_w4(x + pb + 4, a[8], a[9], a[10], a[11]);
    lds_w4(x + pb + 2 * XQE + 4, a[12], a[13], a[14], a[15]);
}
__device__ __forceinline__ void raw_read(const float *x, int pb, float (&a)[16])
{
    lds_r4(x + pb, a[0], a[1], a[2], a[3]);
    lds_r4(x + pb + 2 * XQE, a[4], a[5], a[6], a[7]);
    lds_r4(x + pb + 4, a[8], a[9], a[10], a[11]);
    lds_r4(x + pb + 2 * XQE + 4, a[12], a[13], a[14], a[15]);
}
template <int P>
struct Par16 {
    static constexpr int value = P;
};

// ---- full-line own loads (FL: positions of 2 steps = one 128-B line per column)
// A lane's position covers its column's whole 128-B line (two 16-z bricks);
// x-adjacent lanes (a pair) run one step apart, so at every step exactly one
// lane of a pair -- the "loader", whose prefetch target is the first brick of
// its position -- needs a new line, and the other lane's target is the second
// brick of the line its partner... of the line it loaded itself one step
// earlier.  Both lanes of the pair load the loader's whole line in 4
// instructions (lane parity p: quarters p and p+2 of each half, so an
// instruction touches 32 lines, 32 B of each): the first half goes to the
// loader's next-brick row at the end of the step, the second half is held in
// registers for one step and then goes to the (then) non-loader's row.  Every
// line is fetched once per visit instead of in two 64-B halves a step apart,
// which the L2 re-fetched between the halves.
struct LineLd {
    float a[8];                  // now half: quarters p, p+2 of the loader's line
    int rowl, rowo;              // XN rows: the loader's, the other lane's
};
// the later half (quarters p, p+2) goes to h, held one step
__device__ __forceinline__ void line_issue(Rsrc r, uint32_t seg, bool isl, LineLd &q, float (&h)[8])
{
    const int lane = threadIdx.x, par = lane & 1;
    const bool islp = dpp_swap_pair((unsigned)isl) != 0u;
    const uint32_t segp = dpp_swap_pair(seg);
    const uint32_t sl = isl ? seg : (islp ? segp : OOB);       // the loader's now-half segment
    const uint32_t o = (uint32_t)par * 16u;
    float t[4];
    bload4(r, sl + o, t);
    q.a[0] = t[0]; q.a[1] = t[1]; q.a[2] = t[2]; q.a[3] = t[3];
    bload4(r, sl + o + 32u, t);
    q.a[4] = t[0]; q.a[5] = t[1]; q.a[6] = t[2]; q.a[7] = t[3];
    const uint32_t sh = sl ^ 64u;                               // the other half of the line (OOB stays OOB)
    bload4(r, sh + o, t);
    h[0] = t[0]; h[1] = t[1]; h[2] = t[2]; h[3] = t[3];
    bload4(r, sh + o + 32u, t);
    h[4] = t[0]; h[5] = t[1]; h[6] = t[2]; h[7] = t[3];
    q.rowl = isl ? lane : (lane ^ 1);
    q.rowo = lane ^ (q.rowl == lane ? 1 : 0);
}
// end of step: the loader's next brick (this step's now half) and the other
// lane's (the half held since the previous step) into the XN rows
__device__ __forceinline__ void line_write(float *x, const LineLd &q, const float (&hp)[8])
{
    const int par = threadIdx.x & 1;
    lds_w4(x + XROW16(1, par, q.rowl), q.a[0], q.a[1], q.a[2], q.a[3]);
    lds_w4(x + XROW16(1, par + 2, q.rowl), q.a[4], q.a[5], q.a[6], q.a[7]);
    lds_w4(x + XROW16(1, par, q.rowo), hp[0], hp[1], hp[2], hp[3]);
    lds_w4(x + XROW16(1, par + 2, q.rowo), hp[4], hp[5], hp[6], hp[7]);
}

// paired write-back of changed segments from raw_read operands t
__device__ __forceinline__ void raw_store(Rsrc r, uint32_t seg, bool chg, const float (&t)[16])
{
    const bool odd = threadIdx.x & 1;
    const uint32_t own = chg ? seg : OOB;
    const uint32_t oth = dpp_swap_pair(own);
    const uint32_t o = odd ? 16u : 0u;
    const uint32_t b01 = (odd ? oth : own) + o, b23 = (odd ? own : oth) + o;
    bstore4(r, b01, t[0], t[1], t[2], t[3]);
    bstore4(r, b01 + 32u, t[4], t[5], t[6], t[7]);
    bstore4(r, b23, t[8], t[9], t[10], t[11]);
    bstore4(r, b23 + 32u, t[12], t[13], t[14], t[15]);
}
__device__ __forceinline__ void store16_plain(Rsrc r, uint32_t off, const float (&v)[16])
{
#pragma unroll
    for (int q = 0; q < 4; q++) bstore4(r, off + 16u * q, v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// ---- brick / halo addressing ------------------------------------------------
__device__ __forceinline__ void bload4h(Rsrc r, uint32_t off, float (&v)[4])
{
    f4v a = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
// Brick info of one lane's brick, packed (b0 / b1 ride two steps in VGPRs):
// w1 = flags (12 bits) | zb << 12 (8) | ring slot << 20; w2 = cell-cache base
// (signed 16) | position clock << 16; w3 = block id | BC z-slot mask << 16.
struct BInfo16 {
    uint32_t seg;            // own 64-B segment (OOB if none)
    uint32_t zh;             // z-boundary node (prefetch only): the z-upwind node of a run start (first
                             // brick of a position) or the z-downwind node (last brick, W1_ZD)
    uint32_t lseg;           // this brick's half of its column line if the line holds a valid brick
                             // (prefetch only: a line loader whose own brick is past the grid end)
    uint32_t w1, w2, w3;
    __device__ __forceinline__ int fl() const { return (int)(w1 & 0xfffu); }
    __device__ __forceinline__ int zb() const { return (int)((w1 >> 12) & 0xffu); }   // (lean: the phase)
    __device__ __forceinline__ int ri() const { return (int)((w1 >> 20) & 0xfu); }
    __device__ __forceinline__ int ccb() const { return (int)(w2 << 16) >> 16; }
    __device__ __forceinline__ int clk() const { return (int)(w2 >> 16); }
    __device__ __forceinline__ int bid() const { return (int)(w3 & 0xffffu); }
    __device__ __forceinline__ int bcm() const { return (int)(w3 >> 16); }
};
template <bool RZ>
__device__ __forceinline__ BInfo16 brick_info16(const FsmLaunch &L, const Fsm16Geo &g, int kb, const Smem16 &S,
                                                const Pos &p, int nstream, int lx, int ly, const BcBoxes &bc,
                                                unsigned meta, uint32_t col)
{
    BInfo16 b;
    const int tz = ci_tz(meta);
    const int zb = tz * kb + (RZ ? kb - 1 - p.zbs : p.zbs);   // kb: compile-time in the fixed instance
    const bool valid = pos_valid(p, nstream) && (meta & C_BLK) && zb < g.nzb;
    b.seg = valid ? col + zoff16(zb) : OOB;
    b.lseg = pos_valid(p, nstream) && (meta & C_BLK) && (zb & ~1) < g.nzb ? col + zoff16(zb) : OOB;
    const int zu = RZ ? zb * 16 + 16 : zb * 16 - 1;          // z-upwind node of the brick's first slot
    b.zh = (valid && (meta & C_ZH) && p.zbs == 0) ? col + zoff16(zu >> 4) + (uint32_t)(zu & 15) * 4u : OOB;
    int fl = valid ? (int)((meta & 0x7f) | F_VALID) : 0;
    if (zb == (RZ ? g.nzb - 1 : 0)) fl |= F_FIRST;
    if (zb == (RZ ? 0 : g.nzb - 1)) fl |= F_LAST;
    // held stream: the z-boundary nodes come from the z-face copies (zf), the run end's z-downwind
    // node of the position's last brick below the column end included
    const bool zd = valid && p.zbs == kb - 1 && !(fl & F_LAST);
    if (b.zh != OOB) b.zh = zf_boundary<float, RZ>(L, S.ring_b[p.ri], false, lx, ly);
    if (zd) b.zh = zf_boundary<float, RZ>(L, S.ring_b[p.ri], true, lx, ly);
    if ((meta & C_ZH) && p.zbs == 0) fl |= F_ZH;
    bool slow = (fl & C_PART) || ((fl & C_00) && zb == 0) || (valid && zb * 16 + 16 > L.nz);
    unsigned bcm = 0;
    if (__any(fl & C_BC)) {
        // BC z-slots of this column segment (rare: columns through a source box)
        const int e = S.ring_e[p.ri];
        const int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        unsigned m = 0;
        if (fl & C_BC) {
            for (int k = 0; k < bc.n; k++) {
                const int *q = bc.box + 6 * k;
                if (x >= q[0] && x <= q[1] && y >= q[2] && y <= q[3]) {
                    int lo = q[4] - zb * 16, hi = q[5] - zb * 16;
                    lo = lo < 0 ? 0 : lo; hi = hi > 15 ? 15 : hi;
                    if (lo <= hi) m |= ((2u << hi) - (1u << lo));
                }
            }
        }
        bcm = m;
        slow |= m != 0;
    }
    if (slow) fl |= F_SLOW;
    const int ccb = ci_ccb(meta) + zb * 4;                     // nrz = 4: cell of node z = base + z / 4
    b.w1 = (uint32_t)fl | ((uint32_t)(valid ? zb : 0) << 12) | ((uint32_t)p.ri << 20) | (zd ? W1_ZD : 0u);
    b.w2 = ((uint32_t)ccb & 0xffffu) | ((uint32_t)p.sp << 16);
    b.w3 = ((uint32_t)S.ring_b[p.ri] & 0xffffu) | (bcm << 16);
    return b;
}
// this lane's half (8 z) of halo column j at the edge lane's position pe
template <bool RZ>
__device__ __forceinline__ uint32_t halo_offset16(const Fsm16Geo &g, int kb, const Pos &pe, int nstream, int half,
                                                  unsigned meta, uint32_t col, unsigned hbit, uint32_t hdelta)
{
    const int zb = ci_tz(meta) * kb + (RZ ? kb - 1 - pe.zbs : pe.zbs);
    const bool valid = pos_valid(pe, nstream) && (meta & C_BLK) && zb < g.nzb;
    const uint32_t base = col + ((meta & hbit) ? 0u : hdelta);
    return valid ? base + zoff16(zb) + (uint32_t)half * 32u : OOB;
}

// ---- lean position words (the fixed instance: 2-step positions) ---------
// At admission every lane's position word holds its column flags (bits 0-8,
// as column_word's), per sweep-order phase p a group g_p = FIRST | LAST << 1
// | SLOW << 2 | ZH << 3 | VALID << 4 at bits 9 + 5p, and the cell-cache base
// of the phase-0 brick at bits 19-31; ring_base holds the position's line
// base (tile offset + tz << 13).  A step then decodes its brick with a few
// shifts instead of rederiving zb, validity and the brick flags from tz.
#define LW_G(p) (9 + 5 * (p))
#define LW_CCB 19
template <bool RZ>
__device__ __forceinline__ unsigned lean_word(const FsmLaunch &L, const Fsm16Geo &g, const ColTile &ct, int tz, int ri,
                                              int u0flag, int zh)
{
    int cz0, nczb;
    block_zcells(L, L.kb, tz, cz0, nczb);
    const int m = ct.fl | C_BLK | (u0flag ? C_U0 : 0) | (zh ? C_ZH : 0);
    const int zb0 = 2 * tz + (RZ ? 1 : 0);                      // the phase-0 brick (sweep order)
    unsigned w = (unsigned)m & 0x1ffu;
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const int zb = RZ ? zb0 - p : zb0 + p;
        unsigned gp = zb < g.nzb ? 16u : 0u;
        if (zb == (RZ ? g.nzb - 1 : 0)) gp |= 1u;
        if (zb == (RZ ? 0 : g.nzb - 1)) gp |= 2u;
        if ((m & C_PART) || ((m & C_00) && zb == 0) || zb * 16 + 16 > L.nz) gp |= 4u;
        if (p == 0 && (m & C_ZH)) gp |= 8u;
        w |= gp << LW_G(p);
    }
    const int ccb0 = ri * L.ccb + ct.cl * nczb - cz0 + zb0 * 4;
    return w | ((unsigned)ccb0 << LW_CCB);
}
template <bool RZ>
__device__ __forceinline__ BInfo16 brick_info_lean(const FsmLaunch &L, const Smem16 &S, const Pos &p, int nstream,
                                                   int lx, int ly, const BcBoxes &bc, unsigned w, uint32_t base)
{
    BInfo16 b;
    const int ph = p.zbs;
    const unsigned gp = (w >> (ph ? LW_G(1) : LW_G(0))) & 31u;
    const bool pv = pos_valid(p, nstream);
    const bool valid = pv && (gp & 16u);
    const uint32_t off = base + ((uint32_t)(ph ^ (RZ ? 1 : 0)) << 6);
    b.seg = valid ? off : OOB;
    b.lseg = pv && (w & ((16u << LW_G(0)) | (16u << LW_G(1)))) ? off : OOB;
    b.zh = valid && (gp & 8u) ? off + (RZ ? 8192u - 64u : 124u - 8192u) : OOB;
    // held stream: the z-boundary nodes come from the z-face copies (zf), the run end's z-downwind
    // node of the position's last brick below the column end included
    const bool zd = valid && ph == 1 && !(gp & 2u);
    if (b.zh != OOB) b.zh = zf_boundary<float, RZ>(L, S.ring_b[p.ri], false, lx, ly);
    if (zd) b.zh = zf_boundary<float, RZ>(L, S.ring_b[p.ri], true, lx, ly);
    int fl = valid ? (int)((w & 0x7fu) | F_VALID | ((gp & 15u) << 8)) : 0;
    unsigned bcm = 0;
    if (__any(fl & C_BC)) {
        // BC z-slots of this column segment (rare: columns through a source box)
        const int e = S.ring_e[p.ri];
        const int zb = 2 * ((e >> 24) & 0xff) + (RZ ? 1 - ph : ph);
        const int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        if (fl & C_BC) {
            for (int k = 0; k < bc.n; k++) {
                const int *q = bc.box + 6 * k;
                if (x >= q[0] && x <= q[1] && y >= q[2] && y <= q[3]) {
                    int lo = q[4] - zb * 16, hi = q[5] - zb * 16;
                    lo = lo < 0 ? 0 : lo; hi = hi > 15 ? 15 : hi;
                    if (lo <= hi) bcm |= ((2u << hi) - (1u << lo));
                }
            }
        }
        if (bcm) fl |= F_SLOW;
    }
    const int ccb = (int)(w >> LW_CCB) + (RZ ? -4 * ph : 4 * ph);
    b.w1 = (uint32_t)fl | ((uint32_t)ph << 12) | ((uint32_t)p.ri << 20) | (zd ? W1_ZD : 0u);
    b.w2 = ((uint32_t)ccb & 0xffffu) | ((uint32_t)p.sp << 16);
    b.w3 = ((uint32_t)S.ring_b[p.ri] & 0xffffu) | (bcm << 16);
    return b;
}
template <bool RZ>
__device__ __forceinline__ uint32_t halo_offset_lean(const Pos &pe, int nstream, int half, unsigned me, uint32_t base,
                                                     unsigned hbit, uint32_t hdelta)
{
    const int ph = pe.zbs;
    const bool valid = pos_valid(pe, nstream) && ((me >> (ph ? LW_G(1) : LW_G(0))) & 16u);
    const uint32_t o = base + ((me & hbit) ? 0u : hdelta) + ((uint32_t)(ph ^ (RZ ? 1 : 0)) << 6) + (uint32_t)half * 32u;
    return valid ? o : OOB;
}
// Whole-line halo loads (the fixed instance): the line base of halo column
// j at the edge lane's position pe, valid when the position and either of
// its bricks are.  Halo columns 2i and 2i+1 belong to edge lanes of adjacent
// skews, so at every step exactly one of them targets the first brick of a
// position: the four lanes of quad i then load that column's whole line (the
// first brick staged at the end of the next step, the second one step
// later), lane r taking quarter r of both halves.
template <bool RZ>
__device__ __forceinline__ uint32_t halo_line_lean(const Pos &pe, int nstream, unsigned me, uint32_t base,
                                                   unsigned hbit, uint32_t hdelta)
{
    const bool valid = pos_valid(pe, nstream) && (me & ((16u << LW_G(0)) | (16u << LW_G(1))));
    return valid ? base + ((me & hbit) ? 0u : hdelta) : OOB;
}
// lanes r <-> r ^ 2 within each quad (quad_perm 2, 3, 0, 1)
__device__ __forceinline__ unsigned dpp_swap_quad_half(unsigned v)
{
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
}
// the brick info / halo offset of a step: lean (fixed instance) or general
template <bool RZ, bool LEAN>
__device__ __forceinline__ BInfo16 brick_info_any(const FsmLaunch &L, const Fsm16Geo &g, int kb, const Smem16 &S,
                                                  const Pos &p, int nstream, int lx, int ly, const BcBoxes &bc,
                                                  unsigned meta, uint32_t col)
{
    if (LEAN) return brick_info_lean<RZ>(L, S, p, nstream, lx, ly, bc, meta, col);
    return brick_info16<RZ>(L, g, kb, S, p, nstream, lx, ly, bc, meta, col);
}
template <bool RZ, bool LEAN>
__device__ __forceinline__ uint32_t halo_offset_any(const Fsm16Geo &g, int kb, const Pos &pe, int nstream, int half,
                                                    unsigned meta, uint32_t col, unsigned hbit, uint32_t hdelta)
{
    if (LEAN) return halo_offset_lean<RZ>(pe, nstream, half, meta, col, hbit, hdelta);
    return halo_offset16<RZ>(g, kb, pe, nstream, half, meta, col, hbit, hdelta);
}

// Diagonal order of the tiles for the (+x, +y) sweep (build_order in
// fsm_device.h, 16-bit entries txs | tys << 8).
__device__ __forceinline__ void build_order16(const FsmLaunch &L, unsigned short *order)
{
    for (int id = threadIdx.x; id < L.ntiles; id += 64) {
        const int txs = id % L.ntx, tys = id / L.ntx, dg = txs + tys;
        int rank = 0;
        for (int e = 0; e < dg; e++)
            rank += min(e, L.nty - 1) - max(0, e - L.ntx + 1) + 1;
        rank += tys - max(0, dg - L.ntx + 1);
        order[rank] = (unsigned short)(txs | (tys << 8));
    }
}


// the held stream's LDS arrays (fsm_hold.h)
__device__ __forceinline__ HoldLds<unsigned short> hold_lds16(const Smem16 &S)
{
    HoldLds<unsigned short> H;
    H.order = S.order; H.fz = S.fz; H.lastproc = S.lastproc; H.need = S.lastchg; H.fmask = S.fmask;
    H.ring_e = S.ring_e; H.vbits = S.vbits; H.cbits = S.cbits;
    return H;
}


// Admit position (ring slot ri, relative clock C): every lane writes its
// column meta, lane 0 the ring entry, block id, tile base and the block's
// visit clock.  u0flag: the block's first visit in this iteration (no visit
// since the iteration started: the held stream's clocks restart every sweep,
// so the iteration's visits are a bitmap, read by hold_decide).
template <bool RZ, bool LEAN>
__device__ __forceinline__ void admit16(const FsmLaunch &L, const Fsm16Geo &g, const Smem16 &S, const BcBoxes &bc,
                                        int entry, int zh, int u0flag, int ri, int C, int lx, int ly, int lxs,
                                        int lys, int rx, int ry, ColTile &ct)
{
    unsigned meta = 0;
    int bid = 0, nbv = 0;
    uint32_t base = 0;
    if (entry >= 0) {
        const int tz = (entry >> 24) & 0xff, tx = entry & 0xfff, ty = (entry >> 12) & 0xfff;
        bid = tz * L.ntiles + tx + ty * L.ntx;
        nbv = min(L.kb, L.nzb - tz * L.kb);          // 8-z bricks of the block (visit statistics)
        if ((entry & 0xffffff) != ct.tile) column_tile<float>(L, bc, entry, lx, ly, lxs, lys, rx, ry, ct);
        meta = LEAN ? lean_word<RZ>(L, g, ct, tz, ri, u0flag, zh) : column_word(L, L.kb, ct, tz, ri, u0flag, zh);
        base = (uint32_t)(ty * L.ntx + tx) * tile_bytes<float>(L) + (LEAN ? (uint32_t)tz << 13 : 0u);
    }
    const int nact = L.visit_stats && entry >= 0 ? __builtin_popcountll(__ballot(ct.fl & C_ACT)) : 0;
    asm volatile("" ::: "memory");
    S.meta[ri * 64 + threadIdx.x] = meta;
    if (threadIdx.x == 0) {
        if (entry >= 0) {
            S.lastproc[bid] = (unsigned short)C;
            S.vbits[bid >> 5] |= 1u << (bid & 31);
            if (L.visit_stats) {
                S.scratch[0] += nbv;
                S.scratch[1] += nbv * nact;
            }
        }
        S.ring_e[ri] = entry;
        S.ring_b[ri] = bid;
        S.ring_base[ri] = base;
    }
    asm volatile("" ::: "memory");
}


// The 16 z-slots of the current brick, updated in place (v).  GENERIC as in
// fsm_kernel.hip brick_update (grid-edge columns of cut tiles, cut z-bricks,
// BC nodes, node (0,0,0)); otherwise every lane's missing x/y neighbours are
// already its own old values (the halo of a grid-edge lane is its column).
// NC: evaluate the "changed while >= T" test (nc).  Once a lane of the wave
// has found the iteration unconverged, the test cannot change the outcome
// (the iteration runs again, its verify and u0 copies are not used), so the
// sweep drops it for the rest of the iteration.
template <bool RZ, bool GENERIC, bool LEAN, bool NC = true>
__device__ __forceinline__ void brick16(const FsmLaunch &L, const Smem16 &S, const BInfo16 &b0, float (&v)[16],
                                        float zprev0, float znext, int lx, int ly, int rx, int ry, bool &changed,
                                        bool &nc, int &ierr_last, bool &c0, bool &c15)
{
    const int lane = threadIdx.x;
    const float T = (float)L.conv_thresh;
    const int fl = b0.fl();
    bool xp = true, xn = true, yp = true, yn = true, act = true;
    int zbg = 0;                                             // the brick's zb (generic path)
    if (GENERIC) {
        const int e = S.ring_e[b0.ri()];
        zbg = LEAN ? 2 * ((e >> 24) & 0xff) + (RZ ? 1 - b0.zb() : b0.zb()) : b0.zb();
        const int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        const bool xlo = x > 0, xhi = x < L.nx - 1, ylo = y > 0, yhi = y < L.ny - 1;
        xp = rx ? xhi : xlo; xn = rx ? xlo : xhi; yp = ry ? yhi : ylo; yn = ry ? ylo : yhi;
        act = (fl & C_ACT) != 0;
    }
    const bool first = (fl & F_FIRST) != 0, last = (fl & F_LAST) != 0;
    const int lxs = lane & 7, lys = lane >> 3;
    const int rxm = lxs > 0 ? lane - 1 : 64 + lys, rym = lys > 0 ? lane - 8 : 72 + lxs;
    const int rxp = lxs < 7 ? lane + 1 : 64 + lys, ryp = lys < 7 ? lane + 8 : 72 + lxs;
    float fc = 0.f, ffc = 0.f, ff2c = 0.f, ff3c = 0.f;
#pragma unroll
    for (int hh = 0; hh < NPASS16; hh++) {
        // the quarter of the brick this pass updates (4 z; sweep order: low z
        // first unless RZ) and the four neighbour rows' values for it
        constexpr int PZ = 16 / NPASS16;
        const int h = RZ ? NPASS16 - 1 - hh : hh;
        float xm[PZ], xq[PZ], ym[PZ], yq[PZ];
        lds_r4(S.xr + XROW16(0, h, rxm), xm[0], xm[1], xm[2], xm[3]);
        lds_r4(S.xr + XROW16(0, h, rym), ym[0], ym[1], ym[2], ym[3]);
        lds_r4(S.xr + XROW16(1, h, rxp), xq[0], xq[1], xq[2], xq[3]);
        lds_r4(S.xr + XROW16(1, h, ryp), yq[0], yq[1], yq[2], yq[3]);
#pragma unroll
        for (int jj = 0; jj < PZ; jj++) {
            const int j = hh * PZ + jj;                     // sweep-order slot
            const int pj = RZ ? 15 - j : j;                 // z slot
            const int ph = pj % PZ;                         // index in the pass
            const int pprev = RZ ? pj + 1 : pj - 1, pnext = RZ ? pj - 1 : pj + 1;
            const float self = v[pj];
            if (!GENERIC) {
                if ((j & 3) == 0) {                        // a new cell (4 z per cell) in sweep order
                    fc = S.cc[b0.ccb() + (pj >> 2)];
                    ffc = fc * fc;
                    ff2c = ffc + ffc;
                    ff3c = 3.0f * ffc;
                }
            }
            float xup = xm[ph], xdn = xq[ph], yup = ym[ph], ydn = yq[ph];
            float zup, zdn;
            if (GENERIC) {
                xup = xp ? xup : self; xdn = xn ? xdn : self; yup = yp ? yup : self; ydn = yn ? ydn : self;
                const int zabs = zbg * 16 + pj;
                const bool zp_ex = RZ ? (zabs < L.nz - 1) : (zabs > 0);
                const bool zn_ex = RZ ? (zabs > 0) : (zabs < L.nz - 1);
                zup = zp_ex ? (j > 0 ? v[pprev] : zprev0) : self;
                zdn = zn_ex ? (j < 15 ? v[pnext] : znext) : self;
            } else {
                zup = j > 0 ? v[pprev] : (first ? self : zprev0);
                zdn = j < 15 ? v[pnext] : (last ? self : znext);
            }
            const float ux = fmin_(xup, xdn), uy = fmin_(yup, ydn), uz = fmin_(zup, zdn);
            float nv;
            if (GENERIC) {
                const int zabs = zbg * 16 + pj;
                const int zc_ = zabs < L.nz ? zabs : L.nz - 1;          // cut brick: clamp the cell
                const float f = S.cc[b0.ccb() - zbg * 4 + (zc_ >> 2)];
                int e;
                const float ub = godunov_bl<true>(ux, uy, uz, f, e);
                const bool upd = act && zabs < L.nz && !((b0.bcm() >> pj) & 1);
                nv = upd ? fmin_(self, ub) : self;
                if ((fl & C_00) && zabs == 0) ierr_last = upd ? e : 0;
            } else {
                nv = fmin_(self, godunov_v<true>(ux, uy, uz, fc, ffc, ff2c, ff3c));
            }
            const bool dec = nv < self;
            if (NC) nc |= dec && self >= T;
            changed |= dec;
            if (pj == 0) c0 = dec;                          // the brick's lowest / highest node changed
            if (pj == 15) c15 = dec;                        //   (z faces of its block, held stream)
            v[pj] = nv;
        }
    }
}

// One Gauss-Seidel sweep in direction (rx, ry, RZ) over the admitted
// z-blocks; returns the stream positions used.  The step structure follows
// fsm_kernel.hip sweep() (prefetch AH = 2 steps ahead, loads consumed before
// the step's stores, the next position decided at the end of a step), with
// 16-z bricks and the brick values updated in place: a lane's next brick
// lives in its XN row and is read back into v at the end of the step.
template <bool RZ, int KB16, int CCR>
__device__ __forceinline__ int sweep16(const FsmLaunch &L, const Fsm16Geo &g, Rsrc ur, Rsrc u0r, Rsrc sr, Rsrc zfr,
                                       const BcBoxes &bc, const Smem16 &S, int rx, int ry, int clock0, bool &notconv,
                                       int &ierr_last, unsigned &nchg, unsigned &nsteps)
{
    const Rsrc zr_ = zfr;                            // the z-boundary nodes: the z-face copies
#ifdef MCEIK_PHASECLK
    unsigned long long pclk_t = __builtin_readcyclecounter();
#endif
    const int lane = threadIdx.x, lxs = lane & 7, lys = lane >> 3, d = lxs + lys;
    const int lx = rx ? 7 - lxs : lxs, ly = ry ? 7 - lys : lys;
    const float UN = FLT_MAX;
    const int kb = KB16 > 0 ? KB16 : g.kb;
    const int nr = KB16 > 0 ? F16_NR : g.nr;
    const uint32_t lanecol = (uint32_t)colpos(lx, ly) * 128u;

    // halo loader role: half hh of halo column hj (edge lane he, lag hd)
    const int hj = lane >> 1, hh = lane & 1, he = halo_edge_lane(hj), hd = (he & 7) + (he >> 3);
    const unsigned hbit = hj < 16 ? C_XOWN : C_YOWN;
    const uint32_t hdelta = halo_delta(L, tile_bytes<float>(L), hj, he, rx, ry);
    const int hlx = rx ? 7 - (he & 7) : (he & 7), hly = ry ? 7 - (he >> 3) : (he >> 3);
    const uint32_t hcol = (uint32_t)colpos(hlx, hly) * 128u;

    const HoldLds<unsigned short> H = hold_lds16(S);
    // (the held stream's scan state -- first incomplete tile, previous position's tile and its cached
    // status inputs -- lives in LDS scratch [4..6]: fewer scalar registers live across the step loop)
    // this lane's change-mask bits of a changed brick: the block, and its x / y faces when the
    // lane's column is a tile edge (absolute orientation)
    const unsigned xyface = HOLD_OWN | (lx == 0 ? 2u : 0u) | (lx == 7 ? 4u : 0u) | (ly == 0 ? 8u : 0u) |
                            (ly == 7 ? 16u : 0u);
    hold_norm(L, H);
    if (lane == 0) { S.scratch[4] = 0; S.scratch[5] = -1; }
    clock0 = 64;
    // the next position's block (after settling the visit infl positions back)
    auto decide_any = [&](int pos, int ri, int &zh, int &u0) __attribute__((always_inline)) -> int {
        // positions are decided one after another: settle the one infl back
        const HoldSt hs = hold_state(S.scratch + 4);
        const int q = pos - g.infl;
        if (q >= 0) hold_settle(L, H, q % nr, clock0 + q);
        return hold_decide<RZ>(L, H, S.scratch + 4, hs, clock0 + pos, rx, ry, ri == 0 ? nr - 1 : ri - 1, g.infl,
                               g.vis, zh, u0);
    };
    constexpr bool FL = KB16 == 2;                   // full-line own loads (2-step positions)
    constexpr bool LEAN = KB16 == 2;                 // lean position words (2-step positions)
    // ping-pong register sets by step parity (the step loop runs in pairs, so
    // no register copies at the loop latch): halo values hs[p] loaded at the
    // step before, staged at the end of step p, hs[1 - p] loading; FL's held
    // line half hps[p] from the step before, hps[1 - p] loading
    float v[16], qa[16], hs[2][8];
    LineLd lq;                                       // FL: this step's line loads
    float hps[2][8];                                 // FL: held line halves
    float (&hq)[8] = hs[0];                          // prologue names: halo of step 0, of step 1
    // HFL (whole halo lines): quad i = halo columns 2i, 2i+1; column 2i + hfl(P)
    // loads its line at steps of parity P (hpi: parity of column 2i's lag).
    // hA[P]: the first brick loaded at a step of parity P, staged at the end
    // of the next step; hB[P]: the second brick, staged two steps later (hBs
    // holds it over the step that reloads hB[P])
    constexpr bool HFL = FL && LEAN;
    const int hr = lane & 3, hpi = (lane >> 4) & 1, hcme = (lane >> 1) & 1;
    const int hj0 = (lane >> 1) & ~1;
    const int hst = XROW16((hj0 >> 3) & 1, hr, 64 + ((hj0 >> 4) << 3) + (hj0 & 7));   // column 2i's row, quarter r
    float hA[2][4], hB[2][4], hBs[4];
    float (&hn)[8] = hs[1];
    float (&hp)[8] = hps[0];
    float zc, zn, zq;
    float ccv[CCR];
    int ccsize = 0;
    ColTile ct;
    ct.tile = -1;
    // prologue decisions: positions of lane (0,0)'s bricks 0 .. AH-1
    constexpr int AH = MCEIK_AHEAD16;
    int ndecided = 0, nstream = 0x7fffffff, dri = 0;
    for (int pos = 0; pos <= (AH - 1) / kb; pos++) {
        int zh, u0;
        const int e = decide_any(pos, dri, zh, u0);
        if (e == -2) {
            if (pos == 0) return 0;                         // nothing changed near any block: skip the sweep
            nstream = pos;
            break;
        }
        admit16<RZ, LEAN>(L, g, S, bc, e, zh, u0, dri, clock0 + pos, lx, ly, lxs, lys, rx, ry, ct);
        if (e >= 0) {
            cc_issue<CCR>(L, L.kb, sr, e, ccv, ccsize);
            TRAFU(S, 5, ccsize * 4);
            cc_write<float, CCR>(L, S.cc, dri, ccv, ccsize, (float)L.h);
        }
        ndecided = pos + 1;
        if (++dri == nr) dri = 0;
    }
    asm volatile("" ::: "memory");
    // bricks vb (b0) and vb+1 (b1); the loop computes vb+2's (b3) and carries it
    Pos p3, pe;
    pos_init(p3, -d, kb, nr);
    BInfo16 b0 = brick_info_any<RZ, LEAN>(L, g, kb, S, p3, nstream, lx, ly, bc, S.meta[p3.ri * 64 + lane],
                                  S.ring_base[p3.ri] + lanecol);
    const int pbr = pair_row(0, lane), pbn = pair_row(1, lane);
    {
        float t[16];
        seg_issue(ur, b0.seg, t);
        raw_write(S.xr, pbn, t);                      // through this lane's XN row
        load_row16(S.xr, 1, lane, v);
    }
    pos_init(pe, -hd, kb, nr);
    {
        const uint32_t ho = halo_offset_any<RZ, LEAN>(g, kb, pe, nstream, hh, S.meta[pe.ri * 64 + he],
                                              S.ring_base[pe.ri] + hcol, hbit, hdelta);
        bload4h(ur, ho, *reinterpret_cast<float (*)[4]>(&hq[0]));
        bload4h(ur, ho + 16u, *reinterpret_cast<float (*)[4]>(&hq[4]));
        TRAF(S, 1, ho != OOB, 32);
    }
    zc = bload1(zr_, b0.zh, 0.0f);
    TRAF(S, 0, b0.seg != OOB, 64);
    TRAF(S, 2, b0.zh != OOB, 4);
    pos_adv(p3, kb, nr);
    BInfo16 b1 = brick_info_any<RZ, LEAN>(L, g, kb, S, p3, nstream, lx, ly, bc, S.meta[p3.ri * 64 + lane],
                                  S.ring_base[p3.ri] + lanecol);
    {
        float t[16];
        seg_issue(ur, b1.seg, t);
        raw_write(S.xr, pbn, t);                        // brick vb0 + 1: the XN rows
    }
    if (FL) {
        // the held half for step 0: the lane whose step-0 target is the second
        // brick of its position (it would have loaded the line one step
        // earlier) gets it from its own segment, quarters split over the pair
        Pos pn = p3;
        pos_adv(pn, kb, nr);
        const bool nl = pn.vb >= 0 && pn.zbs == 1;
        const uint32_t sn = nl ? brick_info_any<RZ, LEAN>(L, g, kb, S, pn, nstream, lx, ly, bc, S.meta[pn.ri * 64 + lane],
                                                  S.ring_base[pn.ri] + lanecol).seg
                               : OOB;
        const bool nlp = dpp_swap_pair((unsigned)nl) != 0u;
        const uint32_t snp = dpp_swap_pair(sn);
        const uint32_t s0 = (nl ? sn : (nlp ? snp : OOB)) + (uint32_t)(lane & 1) * 16u;
        float t[4];
        bload4(ur, s0, t);
        hp[0] = t[0]; hp[1] = t[1]; hp[2] = t[2]; hp[3] = t[3];
        bload4(ur, s0 + 32u, t);
        hp[4] = t[0]; hp[5] = t[1]; hp[6] = t[2]; hp[7] = t[3];
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("" : "+v"(hp[i]));
    }
    pos_adv(pe, kb, nr);
    if (HFL) {
        // bricks vb = 1 - hd of both columns (staged at the end of step 0) and
        // the second brick of the loader of parity 1 (staged at the end of
        // step 1): the loader of parity 1 starts its line at 1 - hd, the one
        // of parity 0 holds 1 - hd as its second brick.  Both positions are
        // decided (vb <= 1).
        const uint32_t lo = halo_line_lean<RZ>(pe, nstream, S.meta[pe.ri * 64 + he], S.ring_base[pe.ri] + hcol, hbit,
                                               hdelta);
        const uint32_t lp = dpp_swap_quad_half(lo);
        const uint32_t l1 = hcme == (hpi ^ 1) ? lo : lp, l0 = hcme == hpi ? lo : lp;
        const uint32_t qo = 16u * (uint32_t)hr, oa = (RZ ? 64u : 0u) + qo, ob = (RZ ? 0u : 64u) + qo;
        bload4h(ur, l1 + oa, hA[1]);
        bload4h(ur, l0 + ob, hB[0]);
        bload4h(ur, l1 + ob, hB[1]);
        TRAF(S, 1, l1 != OOB, 32);
    } else {
        const uint32_t ho = halo_offset_any<RZ, LEAN>(g, kb, pe, nstream, hh, S.meta[pe.ri * 64 + he],
                                              S.ring_base[pe.ri] + hcol, hbit, hdelta);
        bload4h(ur, ho, *reinterpret_cast<float (*)[4]>(&hn[0]));
        bload4h(ur, ho + 16u, *reinterpret_cast<float (*)[4]>(&hn[4]));
        TRAF(S, 1, ho != OOB, 32);
    }
    zn = bload1(zr_, b1.zh, 0.0f);
    TRAF(S, 0, b1.seg != OOB, 64);
    TRAF(S, 2, b1.zh != OOB, 4);
    {
        float un[16];
#pragma unroll
        for (int i = 0; i < 16; i++) un[i] = UN;
        store_row16(S.xr, 0, lane, un);             // no results yet
    }
    halo_stage16(S.xr, lane, hq);
    float zprev = UN;                                // last slot of the previous brick (sweep order)
    // the prologue's loads are waited for here, once per sweep; step 0 stages
    // hs[0] = the halos loaded second (hn)
    if (HFL) {
#pragma unroll
        for (int i = 0; i < 4; i++) asm volatile("" : "+v"(hA[1][i]), "+v"(hB[0][i]), "+v"(hB[1][i]));
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) hs[0][i] = hs[1][i];
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("" : "+v"(hs[0][i]));
    }
#pragma unroll
    for (int i = 0; i < 16; i++) asm volatile("" : "+v"(v[i]));
    asm volatile("" : "+v"(zc), "+v"(zn));
    asm volatile("" ::: "memory");

    int ph = AH % kb;
    int cc_pend = -1;
    int B = 0;
    bool ccfill = false;
    int ccri = 0;
    auto decide_step = [&]() __attribute__((always_inline)) {
        ccfill = false;
        ccri = 0;
        if (ph == 0 && nstream == 0x7fffffff) {
            const int pos = ndecided;
            int zh, u0;
            const int e = decide_any(pos, dri, zh, u0);
            PCLK(4);
            if (e == -2) {
                nstream = pos;
            } else {
                admit16<RZ, LEAN>(L, g, S, bc, e, zh, u0, dri, clock0 + pos, lx, ly, lxs, lys, rx, ry, ct);
                if (e >= 0) {
                    cc_issue<CCR>(L, L.kb, sr, e, ccv, ccsize);
                    TRAFU(S, 5, ccsize * 4);
                    ccfill = true;
                    ccri = dri;
                }
                ndecided = pos + 1;
                if (++dri == nr) dri = 0;
            }
        }
    };
    auto more = [&]() __attribute__((always_inline)) -> bool {
        return !(nstream != 0x7fffffff && B >= nstream * kb + 14);
    };
    auto step = [&](auto par) __attribute__((always_inline)) -> bool {
        constexpr int P = FL ? decltype(par)::value : 0;   // other instances: one set + copies
        float (&hcur)[8] = hs[P];                    // staged at the end of this step
        float (&hnew)[8] = hs[1 - P];                // loaded this step
        float (&hpcur)[8] = hps[P];                  // FL: written to XN at the end of this step
        float (&hpnew)[8] = hps[1 - P];              // FL: loaded this step
        // ---- prefetch: own segment and halos of vb+2 (consumed at the end of
        // this step, before its stores; halos staged at the end of the next)
        pos_adv(p3, kb, nr);
        pos_adv(pe, kb, nr);
        const unsigned m3 = S.meta[p3.ri * 64 + lane], me = S.meta[pe.ri * 64 + he];
        const uint32_t c3 = S.ring_base[p3.ri] + lanecol, ce = S.ring_base[pe.ri] + hcol;
        __builtin_amdgcn_sched_barrier(0);
        const BInfo16 b3 = brick_info_any<RZ, LEAN>(L, g, kb, S, p3, nstream, lx, ly, bc, m3, c3);
        if (FL)
            line_issue(ur, b3.lseg, p3.vb >= 0 && p3.zbs == 0, lq, hpnew);
        else
            seg_issue(ur, b3.seg, qa);
        zq = __any(b3.zh != OOB) ? bload1(zr_, b3.zh, 0.0f) : 0.0f;
        if (HFL) {
            const uint32_t lo = halo_line_lean<RZ>(pe, nstream, me, ce, hbit, hdelta);
            const uint32_t lp = dpp_swap_quad_half(lo);
            const uint32_t sl = hcme == (hpi ^ P) ? lo : lp;         // this step's loader column's line
            const uint32_t qo = 16u * (uint32_t)hr;
#pragma unroll
            for (int i = 0; i < 4; i++) hBs[i] = hB[P][i];
            bload4h(ur, sl + (RZ ? 64u : 0u) + qo, hA[P]);
            bload4h(ur, sl + (RZ ? 0u : 64u) + qo, hB[P]);
            TRAF(S, 1, sl != OOB, 32);
            TRAF(S, 0, b3.seg != OOB, 64);
            TRAF(S, 2, b3.zh != OOB, 4);
        } else {
            const uint32_t ho = halo_offset_any<RZ, LEAN>(g, kb, pe, nstream, hh, me, ce, hbit, hdelta);
            bload4h(ur, ho, *reinterpret_cast<float (*)[4]>(&hnew[0]));
            bload4h(ur, ho + 16u, *reinterpret_cast<float (*)[4]>(&hnew[4]));
            TRAF(S, 1, ho != OOB, 32);
            TRAF(S, 0, b3.seg != OOB, 64);
            TRAF(S, 2, b3.zh != OOB, 4);
        }
        PCLK(0);
        __builtin_amdgcn_s_setprio(0);               // the update at the SIMD's low priority (below)
        // ---- u0: old values of a block's first visit in the iteration (< T only); none once the
        // iteration is known unconverged (the verify that reads them does not run)
        const bool wnc = !__any(notconv);
        if (wnc && __any(b0.fl() & C_U0)) {
            unsigned m = __builtin_bit_cast(unsigned, v[0]);
#pragma unroll
            for (int i = 1; i < 16; i++) m = min(m, __builtin_bit_cast(unsigned, v[i]));
            const bool st0 = __builtin_bit_cast(float, m) < (float)L.conv_thresh && (b0.fl() & C_U0);
            if (__any(st0)) store16_plain(u0r, st0 ? b0.seg : OOB, v);
            TRAF(S, 4, st0, 64);
        }
        // ---- the 16 z-slots of the current brick (next brick's first value
        // in sweep order from this lane's XN row)
        float znext = S.xr[XROW16(1, RZ ? 3 : 0, lane) + (RZ ? 3 : 0)];
        // the position's last brick: its z-downwind node is the next brick's first (XN row) only
        // when the run continues, else the node loaded from HBM
        const unsigned fmk = S.fmask[b0.ri()];
        if ((b0.w1 & W1_ZD) && !(fmk & HOLD_CONT)) znext = zc;
        const float zp0 = (b0.fl() & F_ZH) ? zc : zprev;
        PCLK(1);
        bool changed = false, nc = false, c0 = false, c15 = false;
        if (__any(b0.fl() & F_SLOW))
            brick16<RZ, true, LEAN>(L, S, b0, v, zp0, znext, lx, ly, rx, ry, changed, nc, ierr_last, c0, c15);
        else if (wnc)
            brick16<RZ, false, LEAN>(L, S, b0, v, zp0, znext, lx, ly, rx, ry, changed, nc, ierr_last, c0, c15);
        else
            brick16<RZ, false, LEAN, false>(L, S, b0, v, zp0, znext, lx, ly, rx, ry, changed, nc, ierr_last, c0, c15);
        const bool val = (b0.fl() & F_VALID) != 0;
        changed = changed && val;
        notconv |= nc && val;
        nchg += changed ? 2u : 0u;                   // in 8-z segment equivalents
        // From here to the next step's loads the wave issues at raised priority:
        // its bookkeeping (load waits, row writes, stores, the stream decision and
        // the next prefetch) is a chain of dependent short instructions, and the
        // other wave of the SIMD, inside its update, fills the cycles in between
        // (+0.7%, profiles/r06_prio2).
        PCLK(2);
        __builtin_amdgcn_s_setprio(2);

        // ---- consume this step's loads before any store of the step
        if (cc_pend >= 0) cc_write<float, CCR>(L, S.cc, cc_pend, ccv, ccsize, (float)L.h);
        cc_pend = ccfill ? ccri : -1;
        float nn[16];
        if (FL) {
#pragma unroll
            for (int i = 0; i < 8; i++) asm volatile("" : "+v"(lq.a[i]), "+v"(hpnew[i]));
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) nn[i] = qa[i];     // raw quarters (raw_write below)
        }
        if (HFL) {
            // the first brick loaded last step -> the other column (this
            // step's non-loader), the second brick loaded two steps ago ->
            // this step's loader column
            const int lc = hpi ^ P;
            lds_w4(S.xr + hst + 4 * (1 - lc), hA[1 - P][0], hA[1 - P][1], hA[1 - P][2], hA[1 - P][3]);
            lds_w4(S.xr + hst + 4 * lc, hBs[0], hBs[1], hBs[2], hBs[3]);
        } else {
            halo_stage16(S.xr, lane, hcur);
        }
        zc = zn; zn = zq;
        if (!FL) {
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("" : "+v"(nn[i]));
        }
        if (!FL) {
#pragma unroll
            for (int i = 0; i < 8; i++) hcur[i] = hnew[i];
        }
        if (HFL) {
#pragma unroll
            for (int i = 0; i < 4; i++) asm volatile("" : "+v"(hA[P][i]), "+v"(hB[P][i]));
        } else {
            asm volatile("" : "+v"(hnew[0]), "+v"(hnew[1]), "+v"(hnew[2]), "+v"(hnew[3]), "+v"(hnew[4]),
                         "+v"(hnew[5]), "+v"(hnew[6]), "+v"(hnew[7]));
        }
        asm volatile("" : "+v"(zn));
        asm volatile("" ::: "memory");
        // ---- rows for the next step: results (XR), then this lane's next
        // brick back into v and the brick after it into XN
        store_row16(S.xr, 0, lane, v);
        zprev = v[RZ ? 0 : 15];
        if (__any(changed)) {
            float t[16];
            raw_read(S.xr, pbr, t);
            raw_store(ur, b0.seg, changed, t);
        }
        TRAF(S, 3, changed, 64);
        {
            // what this lane changed: the block, its x / y faces (edge columns), its z faces (the
            // block's lowest / highest node of the column)
            const int zr = LEAN ? (b0.zb() ^ (RZ ? 1 : 0)) : b0.zb() % kb;   // brick index in the block
            const bool zlo = changed && zr == 0 && c0, zhi = changed && zr == kb - 1 && c15;
            if (changed) atomicOr(&S.fmask[b0.ri()], xyface | (zlo ? HOLD_ZLO : 0u) | (zhi ? HOLD_ZHI : 0u));
            // the block's lowest / highest node of this column changed: its z-face copy too
            if (__any(zlo || zhi)) {
                bstore1(zfr, zlo ? zf_off<float>(b0.bid(), 0, lx, ly) : OOB, v[0]);
                bstore1(zfr, zhi ? zf_off<float>(b0.bid(), 1, lx, ly) : OOB, v[15]);
            }
        }
        load_row16(S.xr, 1, lane, v);
        if (FL) {
            line_write(S.xr, lq, hpcur);
        } else {
            raw_write(S.xr, pbn, nn);
        }
        asm volatile("" ::: "memory");
        b0 = b1;
        b1 = b3;
        if (++ph == kb) ph = 0;
        B++;
        PCLK(3);
        decide_step();
        PCLK(5);
        return more();
    };
    decide_step();
    PCLK(6);
    if (more()) {
        if (FL) {
            do {
                if (!step(Par16<0>())) break;
            } while (step(Par16<1>()));
        } else {
            do {
            } while (step(Par16<0>()));
        }
    }
    __builtin_amdgcn_s_setprio(0);
    nsteps += (unsigned)B;                           // macro steps of this sweep (visit statistics)
    // the last visits' changes (every lane is past them)
    for (int q = max(0, nstream - g.infl + 1); q < nstream; q++) hold_settle(L, H, q % nr, clock0 + q);
    PCLK(6);
    return nstream;
}

// End-of-iteration check of the nodes below T (only when no node >= T
// changed): the z-blocks changed in this iteration; u0 was stored at their
// first visit (fsm_kernel.hip verify_small, 16-bit clocks).
__device__ __forceinline__ void verify16(const FsmLaunch &L, Rsrc ur, Rsrc u0r, const Smem16 &S, bool &notconv)
{
    const int lane = threadIdx.x, lx = lane & 7, ly = lane >> 3;
    const float T = (float)L.conv_thresh, tolr = (float)L.tol;
    for (int base = 0; base < L.nblocks; base += 64) {
        const int k = base + lane;
        const bool flag = k < L.nblocks && ((S.cbits[k >> 5] >> (k & 31)) & 1u) != 0;
        unsigned long long m = __ballot(flag);
        while (m) {
            const int bid = base + __builtin_ctzll(m);
            m &= m - 1;
            const int tz = bid / L.ntiles, id = bid - tz * L.ntiles;
            const int tx = id % L.ntx, ty = id / L.ntx;
            const int x = tx * 8 + lx, y = ty * 8 + ly;
            const int zend = min(tz * L.kb + L.kb, L.nzb);
            for (int zb = tz * L.kb; zb < zend; zb++) {
                const uint32_t seg = (uint32_t)id * tile_bytes<float>(L) + zoff_bytes<float>(zb) +
                                     (uint32_t)colpos(lx, ly) * 128u;
                float u[8], v0[8];
                bload8(ur, seg, u);
                bload8(u0r, seg, v0);
                TRAF(S, 6, x < L.nx && y < L.ny, 64);
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    float dl = v0[i] - u[i];
                    dl = dl < 0.0f ? -dl : dl;
                    if (x < L.nx && y < L.ny && zb * 8 + i < L.nz && u[i] < T && !(dl < tolr)) notconv = true;
                }
            }
        }
    }
}

// ---- multi-step sampler launch (L.mc_dev) ----------------------------------
// The solves of mc_nsteps sampler steps in one launch, without a barrier
// between steps: the chains are split into 8 groups, each group's solves of
// all steps handed out by its own ticket counter in step-major, chain-major
// order.  A chain's solves of step k wait until its step k - 1 is accepted
// and step k proposed; the wave that completes the chain's last solve of a
// step does both (mcmc_device.h: the per-step kernels' arithmetic, so the
// results equal the step-by-step launches bit for bit).
//
// Coherence: hipMalloc memory is coherent within one XCD's L2 only, so a
// group is owned by one XCD (the first that claims it: XCD id + 1 by CAS)
// and only that XCD's waves serve it; a chain's solves, tables, state and
// proposal then stay behind one L2.  Writers wait for their stores
// (s_waitcnt) before the L2 atomics that publish them; readers invalidate
// their CU's L1 (buffer_inv sc1) after observing them and load chain state
// through vector loads (mcmcd::ldv).  A wave first serves its own XCD's
// group, then any group its XCD owns or can claim, and exits when none has
// tickets left, so every group is served whatever the XCD ids.  A ticket
// only waits on earlier tickets of its own group, all held by running
// waves: no deadlock, whatever the residency.
struct McQueue {
    unsigned xcc;                // this wave's XCD id + 1
    int cur;                     // group being served, -1 none
};
__device__ __forceinline__ unsigned mc_group_tickets(const FsmLaunch &L, int g, int &clo)
{
    const int nch = L.nsolve / L.nstat;
    clo = (int)((long long)nch * g / 8);
    const int chi = (int)((long long)nch * (g + 1) / 8);
    return (unsigned)(chi - clo) * (unsigned)L.nstat;
}
// (sc1: the agent-scope acquire's invalidate, which is what reaches the CU's
// L1 -- workgroup scope (sc0) leaves a non-split workgroup's L1 alone; local
// memory's L2 lines are not dropped by it)
__device__ __forceinline__ void mc_l1_invalidate()
{
    asm volatile("buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
}
// every store issued so far has completed (reached L2) before what follows
// is issued (the asm is also a compiler barrier: no store sinks past it)
__device__ __forceinline__ void mc_stores_done()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ bool mc_next(const FsmLaunch &L, McQueue &q, int &solve, int &k)
{
    const int lane = threadIdx.x;
    unsigned *owner = L.mc_sync, *tick = L.mc_sync + 8;
    int *ready = reinterpret_cast<int *>(L.mc_sync + 8 + 8 * 32);
    for (;;) {
        if (q.cur >= 0) {
            int clo;
            const unsigned gs = mc_group_tickets(L, q.cur, clo), tot = gs * (unsigned)L.mc_nsteps;
            unsigned t = 0;
            if (lane == 0) t = atomicAdd(tick + 32 * q.cur, 1u);
            t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
            if (t < tot) {
                k = (int)(t / gs);
                solve = clo * L.nstat + (int)(t - (unsigned)k * gs);
                const int c = solve / L.nstat;
                unsigned broken = 0;
                if (lane == 0) {
                    // (a safety net, never expected: after ~30 s the wave stops
                    // waiting, raises the sync buffer's broken-queue flag, which
                    // the host reports as a failed run, and leaves the launch
                    // without solving from a state that is not ready)
                    for (unsigned it = 0; atomicAdd(ready + c, 0) < k; it++) {
                        if (it >= L.mc_spin_limit) {
                            atomicExch(L.mc_sync + MC_SYNC_WORDS(L.nsolve / L.nstat) - 1, 1u);
                            broken = 1;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(32);
                    }
                }
                broken = __builtin_amdgcn_readfirstlane(__shfl(broken, 0, 64));
                if (broken) return false;
                __builtin_amdgcn_wave_barrier();
                mc_l1_invalidate();
                return true;
            }
            q.cur = -1;
        }
        int found = -1;
        for (int j = 0; j < 8 && found < 0; j++) {
            const int g = (int)((q.xcc - 1u + (unsigned)j) & 7u);
            unsigned own = 0, left = 0;
            if (lane == 0) {
                own = atomicCAS(owner + g, 0u, q.xcc);
                if (own == 0u) own = q.xcc;
                int clo;
                const unsigned tot = mc_group_tickets(L, g, clo) * (unsigned)L.mc_nsteps;
                left = own == q.xcc && atomicAdd(tick + 32 * g, 0u) < tot ? 1u : 0u;
            }
            left = __builtin_amdgcn_readfirstlane(__shfl(left, 0, 64));
            if (left) found = g;
        }
        if (found < 0) return false;
        q.cur = found;
    }
}
// kept-state slot of global step gs (mceik_mcmc_run's rule), or -1
__device__ __forceinline__ int mc_keep_slot(const FsmLaunch &L, long long gs)
{
    if (!L.mc_maxs || gs < L.mc_nburn || (gs - L.mc_nburn) % L.mc_keepk) return -1;
    auto nk = [&](long long x) -> long long {       // kept steps in [0, x)
        return x <= L.mc_nburn ? 0 : (x - L.mc_nburn + L.mc_keepk - 1) / L.mc_keepk;
    };
    return (int)((L.mc_nkept0 + nk(gs) - nk(L.mc_step0)) % L.mc_maxs);
}
// After solve (c, station) of launch step k wrote its tables: count it; the
// chain's last solve of the step runs the chain's accept (step mc_step0 + k),
// kept state and next proposal, then marks step k + 1 ready.
__device__ __forceinline__ void mc_finish(const FsmLaunch &L, int solve, int k)
{
    const int lane = threadIdx.x;
    const int nch = L.nsolve / L.nstat, c = solve / L.nstat;
    int *ready = reinterpret_cast<int *>(L.mc_sync + 8 + 8 * 32);
    unsigned *done = L.mc_sync + 8 + 8 * 32 + nch;
    mc_stores_done();                               // this solve's tables are in L2
    unsigned old = 0;
    if (lane == 0) old = atomicAdd(done + c, 1u);
    old = __builtin_amdgcn_readfirstlane(__shfl(old, 0, 64));
    if (old + 1u != (unsigned)(k + 1) * (unsigned)L.nstat) return;
    mc_l1_invalidate();
    const McmcDev &D = *reinterpret_cast<const McmcDev *>(L.mc_dev);
    const long long gstep = (long long)L.mc_step0 + k;
    const int keep_slot = mc_keep_slot(L, gstep);
    // the proposal's logL: objfn of event e on lane e % 64, summed in event order
    const int inp = mcmcd::ldv(&D.prop_inprior[c]), ph = mcmcd::ldv(&D.prop_phase[c]);
    double ln = 0.0;
    if (inp) {
        for (int e0 = 0; e0 < D.nev; e0 += 64) {
            const int e = e0 + lane, n = min(64, D.nev - e0);
            const double obj = e < D.nev ? mcmcd::event_obj(D, c, ph, e) : 0.0;
            for (int i = 0; i < n; i++) ln = ln - __shfl(obj, i, 64);
        }
    }
    int acc = 0;
    if (lane == 0) acc = mcmcd::chain_accept(D, c, ln, keep_slot);
    acc = __builtin_amdgcn_readfirstlane(__shfl(acc, 0, 64));
    if (acc && D.nphase > 1) mcmcd::chain_copy_tables(D, c, ph, lane, 64);
    if (keep_slot >= 0) {                           // keep_kernel's copy of this chain (after the accept)
        const int cell = mcmcd::ldv(&D.prop_cell[c]), pv = mcmcd::ldv(&D.prop_v[c]);
        int *dst = D.keep_v + ((size_t)keep_slot * D.keep_stride + c) * D.ncm;
        const int *src = D.v + (size_t)c * D.ncm;
        for (int j = lane; j < D.ncm; j += 64) dst[j] = (acc && j == cell) ? pv : mcmcd::ldv(src + j);
    }
    if (k + 1 < L.mc_nsteps && lane == 0) mcmcd::chain_propose(D, c, (uint64_t)(gstep + 1));
    mc_stores_done();                               // the chain's new state is in L2
    if (lane == 0) atomicExch(ready + c, k + 1);
}

// MC: the multi-step sampler instance (L.mc_dev set); the plain batch
// instances carry none of its code
template <int KB16, int CCR, bool MC>
__device__ __forceinline__ void fsm16_body(const FsmLaunch &L)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem16 S = smem16_bind<KB16 == 2>(L, smem);
    const Fsm16Geo g = fsm16_geo(L);
    const int lane = threadIdx.x;
    const uint32_t fbytes = (uint32_t)(L.field_elems * 4);
    build_order16(L, S.order);
    int pass = 0;
    McQueue mq;
    mq.cur = -1;
    mq.xcc = 1u;
    if (MC) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        mq.xcc = (x & 0xfu) + 1u;
    }
    for (;;) {
        int snext, mk = 0;
        if (MC) {
            if (!mc_next(L, mq, snext, mk)) break;
        } else {
            snext = next_solve(L, pass);
            if (snext < 0) break;
        }
        const unsigned solve = (unsigned)snext;
        if (L.solve_clock && lane == 0) L.solve_clock[2 * (size_t)solve] = __builtin_amdgcn_s_memrealtime();
        const int model = (int)solve / L.nstat, station = (int)solve - model * L.nstat;
        const size_t slot = L.slot_per_solve ? solve : blockIdx.x;
        float *u = reinterpret_cast<float *>(L.u) + slot * L.field_elems;
        float *u0 = reinterpret_cast<float *>(L.u0) + (size_t)blockIdx.x * L.field_elems;   // per-wave scratch
        const size_t ncell = (size_t)L.ncx * L.ncy * L.ncz;
        // (a multi-step launch's model phase changes between steps: vector load)
        const int phase = L.model_phase ? (MC ? mcmcd::ldv(L.model_phase + model) : L.model_phase[model])
                                        : fsm_plain_phase(L, model);
        if (L.skip && L.skip[phase * L.nstat + station]) {      // no picks of this phase at this station
            skip_solve<float>(L, solve);
            if (MC) mc_finish(L, (int)solve, mk);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            continue;
        }
        const size_t sentry = !L.model_phase ? (size_t)model : (size_t)model * L.nphase + phase;
        const void *slow_model = reinterpret_cast<const float *>(L.slow) + sentry * ncell;
        const Rsrc ur = make_rsrc(u, fbytes), u0r = make_rsrc(u0, fbytes),
                   sr = make_rsrc(slow_model, (uint32_t)(ncell * 4));
        const size_t zfb = zf_bytes(L, 4);
        const Rsrc zfr = make_rsrc(reinterpret_cast<char *>(L.zf) + (size_t)blockIdx.x * zfb, (uint32_t)zfb);
        if (lane == 0) { S.scratch[0] = 0; S.scratch[1] = 0; S.scratch[2] = 0; S.scratch[3] = 0; }
#ifdef MCEIK_TRAFFIC
        if (lane == 0)
            for (int k = 0; k < MCEIK_TRAFFIC_N; k++) S.scratch[8 + k] = 0;
#endif
        unsigned nchg = 0, nsteps = 0;
        BcBoxes bc;
        bc.box = S.box;
        const bool ok = init_field<float, 1>(L, u, ur, slow_model, L.src + (size_t)station * L.nsrc * 4, bc);
        // (before the first sweep only the blocks holding boundary-condition nodes are dirty: a block
        // whose nodes and neighbours are all u_nan updates to u_nan; hold_solve_start)
        hold_solve_start(L, hold_lds16(S), bc, g.nr);
        zf_init<float>(L, zfr, u, bc);
        asm volatile("" ::: "memory");
        int iters = 0, ierr_last = 0;
        if (ok) {
            int sweeps_left = L.max_sweeps < 0 ? 0x7fffffff : L.max_sweeps;
            for (int it = 0; it < L.maxit && sweeps_left > 0; it++) {
                bool notconv = false;
                hold_iter_start(L, hold_lds16(S));     // (the held stream rebases its clocks every sweep)
                int clock = 64;
                for (int sw = 0; sw < 8 && sweeps_left > 0; sw++, sweeps_left--) {
                    const int rx = sw & 1, ry = (sw >> 1) & 1;
                    // positions used + a gap of infl: the previous sweep's visits are
                    // never in flight (nor within vis) for the next one
                    if (sw & 4)
                        clock += g.infl + sweep16<true, KB16, CCR>(L, g, ur, u0r, sr, zfr, bc, S, rx, ry, clock, notconv,
                                                              ierr_last, nchg, nsteps);
                    else
                        clock += g.infl + sweep16<false, KB16, CCR>(L, g, ur, u0r, sr, zfr, bc, S, rx, ry, clock, notconv,
                                                               ierr_last, nchg, nsteps);
                    __builtin_amdgcn_s_waitcnt(0);      // stores of this sweep land before the next sweep's loads
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    TRAF_FLUSH(L, S);
                }
                iters = it + 1;
                if (sweeps_left > 0 || L.max_sweeps < 0) {
                    if (!__any(notconv)) verify16(L, ur, u0r, S, notconv);
                    if (!__any(notconv)) break;
                }
            }
        }
        // ierr: from the last evaluation of node (0,0,0) (the reference's last update)
        int ierr = ierr_last;
        for (int o = 32; o > 0; o >>= 1) ierr = max(ierr, __shfl_xor(ierr, o, 64));
        if (!ok) ierr = 1;
        if (L.visit_stats) {
            for (int o = 32; o > 0; o >>= 1) nchg += __shfl_xor(nchg, o, 64);
            asm volatile("" ::: "memory");
            if (lane == 0) {
                atomicAdd(L.visit_stats, (unsigned long long)(unsigned)S.scratch[0]);
                atomicAdd(L.visit_stats + 1, (unsigned long long)(unsigned)S.scratch[1]);
                atomicAdd(L.visit_stats + 2, (unsigned long long)nchg);
                atomicAdd(L.visit_stats + 3, (unsigned long long)nsteps);
            }
        }
        if (lane == 0) {
            if (L.solve_clock) L.solve_clock[2 * (size_t)solve + 1] = __builtin_amdgcn_s_memrealtime();
            if (L.iter_total) atomicAdd(L.iter_total, (unsigned long long)iters);
            if (L.solve_count) atomicAdd(L.solve_count, 1ull);
            if (L.niter) L.niter[solve] = iters;
            if (L.ierr) L.ierr[solve] = ierr;
        }
        TRAFU(S, 7, (unsigned)(L.field_elems * 4) + (L.ttab ? (unsigned)L.nev * (4u + 64u) : 0u));
        TRAF_FLUSH(L, S);
        if (L.ttab) {
            for (int e = lane; e < L.nev; e += 64) L.ttab[(size_t)solve * L.nev + e] = event_time<float>(L, u, e);
        }
        if (MC) mc_finish(L, (int)solve, mk);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
}

// register budget: two waves per SIMD (<= 256 VGPRs)
#define FSM16_WPE __attribute__((amdgpu_waves_per_eu(2, 2)))
template <int KB16, int CCR, bool MC>
__global__ __launch_bounds__(64) FSM16_WPE void fsm16_solve_kernel(FsmLaunch L)
{
    fsm16_body<KB16, CCR, MC>(L);
}

}  // namespace

// ---- host-side launchers (used by fsm_kernel.hip's dispatcher) -------------
// instances: <2, 1> the fixed layout (kb16 = 2, <= 32 cells per z-block: C2,
// C3), <0, 1> runtime kb with <= 64 cells per block, <0, 4> up to 256 (C5)
hipError_t fsm16_launch(const FsmLaunch &L, int nwaves, hipStream_t st)
{
    if (!fsm16_eligible(L, 4)) return hipErrorInvalidValue;
    const size_t lds = fsm16_lds_bytes(L);
    const bool mc = L.mc_dev != nullptr;
    if (fsm16_fixed_layout(L)) {
        if (mc) hipLaunchKernelGGL((fsm16_solve_kernel<2, 1, true>), dim3(nwaves), dim3(64), lds, st, L);
        else hipLaunchKernelGGL((fsm16_solve_kernel<2, 1, false>), dim3(nwaves), dim3(64), lds, st, L);
    } else if (L.ccb <= 64) {
        if (mc) hipLaunchKernelGGL((fsm16_solve_kernel<0, 1, true>), dim3(nwaves), dim3(64), lds, st, L);
        else hipLaunchKernelGGL((fsm16_solve_kernel<0, 1, false>), dim3(nwaves), dim3(64), lds, st, L);
    } else {
        if (mc) hipLaunchKernelGGL((fsm16_solve_kernel<0, 4, true>), dim3(nwaves), dim3(64), lds, st, L);
        else hipLaunchKernelGGL((fsm16_solve_kernel<0, 4, false>), dim3(nwaves), dim3(64), lds, st, L);
    }
    return hipGetLastError();
}

int fsm16_occupancy(const FsmLaunch &L)
{
    int nb = 0;
    const size_t lds = fsm16_lds_bytes(L);
    hipError_t e;
    if (fsm16_fixed_layout(L))
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm16_solve_kernel<2, 1, false>, 64, lds);
    else if (L.ccb <= 64)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm16_solve_kernel<0, 1, false>, 64, lds);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm16_solve_kernel<0, 4, false>, 64, lds);
    return e == hipSuccess ? nb : 1;
}
