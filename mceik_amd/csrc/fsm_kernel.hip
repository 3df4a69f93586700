// fsm_kernel.hip -- batched 3D fast-sweeping eikonal solve for gfx950.
//
// Replaces the reference's CPU hot loop EIKONAL3D_FSM / EVAL_UPDATE3D /
// UPDATE3D / SOLVE_HAMILTONIAN3D (fsm3d.f90:28-99, 419-693) and the boundary
// conditions EIKONAL3D_SETBCS (fsm3d.f90:697-840).  Results are bitwise equal to
// the reference's Gauss-Seidel order (fp64 build) or to the stable fp32 twin
// (fp32 build); see DESIGN.md s.3 for the schedule and its proof.
//
// Execution model: ONE 64-lane wave per (model, station) solve, persistent
// over a work queue.  The wave owns an 8x8 column tile; lane (lx,ly) holds its
// column's values in registers and runs 8*(lx+ly) steps behind lane (0,0), so
// every lane sits on the same intra-brick z slot and a lane's upwind x/y
// neighbours (already updated) and downwind ones (still old) are one brick
// ahead/behind in neighbour lanes' registers.  Tiles are streamed through the
// wave back to back in sweep order; the x-halo of the previous tile goes
// through LDS, the y-halos and the next tile's x-halo come from HBM.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "fsm_common.h"
#include "fsm_device.h"
#include "fsm_hold.h"
#include "fsm_update.h"

// The compact-layout fp64 instances run the held z-block stream (fsm_hold.h),
// their z-boundary nodes read from the field (the z-face copies of the fp32
// kernel measured 2.4% slower here: their stores and buffer descriptor spill
// registers; profiles/r05_zf).

namespace {

// ---- neighbour exchange through LDS rows.  At the end of every step each
// lane writes its 8 results (XR row) and its next brick (XN row); the next
// step reads the x/y-upwind lanes' XR rows (new values of its own z brick)
// and the downwind lanes' XN rows (old values), tile-edge lanes the halo
// rows staged in the same arrays.  The row offsets are lane constants, so a
// node's four x/y neighbours cost no VALU (no DPP moves, no halo selects).

// ---- LDS working set of one solve wave -------------------------------------
// The stream of a sweep is a sequence of positions of kb z-bricks each: the
// z-blocks (tile, tz) that need an update, tiles in diagonal (wavefront)
// order of the sweep direction and, inside a tile, a run of consecutive
// z-blocks from the first one whose inputs changed to the column's end (a
// block's z-upwind neighbour is still in flight when the next block is
// decided, so a run never stops early).  Bubble positions keep an upwind x/y
// neighbour's visit >= vis positions back (halo visibility).  Per-block
// clocks live in LDS.
// CMP (the compact layout, fsm_compact_layout(): the fp64 compile-time-kb
// instances): 16-bit block clocks relative to the sweep (the held stream,
// fsm_hold.h, as fsm16_kernel.hip), and per position one meta word per lane plus the tile
// base (ring) instead of {own column, meta} -- 25.4 -> 19.9 KB of LDS at C3,
// 6 -> 8 resident waves per CU.
template <typename R, bool CMP = false>
struct Smem {
    using clk_t = typename std::conditional<CMP, unsigned short, int>::type;
    int *box;                    // BC boxes [nsrc][6]
    float *cc;                   // cell cache [nr][ccb]                   (SLOWMODE 2)
    int *order;                  // diagonal tile order: txs | tys << 16   [ntiles]
    clk_t *lastproc, *lastchg;   // per z-block stream clock of the last visit / last visit with a change
    int *ring;                   // per position (mod nr): block entry tx | ty << 12 | tz << 24, bubble -1;
                                 // then [nr] the z-block ids (CMP: then [nr] the tile base offsets)
    int *scratch;                // debug counters
    u2v *cinfo;                  // [nr][64] column info of every lane per position: {own column, meta}
    unsigned *meta;              // CMP: [nr][64] the meta word only (own column = tile base + lane column)
    R *sf;                       // staged slowness*h (modes 0,1)
    R *xr;                       // neighbour rows: XR [2 halves][80 rows][4], then XN (same shape)
    unsigned *fmask;             // CMP, held stream: per ring slot, what the position's visit changed
    unsigned char *fz;           // CMP, held stream: per tile, z-blocks decided in this sweep
    unsigned *vbits, *cbits;     // CMP, held stream: blocks visited / changed in this iteration
};

template <typename R, bool FIXED, bool CMP>
__device__ __forceinline__ Smem<R, CMP> smem_bind(const FsmLaunch &L, unsigned char *base)
{
    size_t off[MCEIK_SMEM_ARRAYS];
    if (FIXED) {         // fsm_fixed_layout(): constants (the host checked the predicate)
        off[11] = FSMF_CINFO; off[9] = FSMF_XR; off[1] = FSMF_CC; off[6] = FSMF_RING; off[7] = FSMF_SCRATCH;
        off[3] = FSMF_LASTPROC; off[4] = FSMF_LASTCHG; off[2] = FSMF_ORDER; off[8] = FSMF_ORDER;
        off[0] = FSMF_ORDER + mceik_align16((size_t)L.ntiles * 4);
    } else {
        fsm_smem_layout(L, sizeof(R), off);
    }
    Smem<R, CMP> S;
    S.box = reinterpret_cast<int *>(base + off[0]);
    S.cc = reinterpret_cast<float *>(base + off[1]);
    S.order = reinterpret_cast<int *>(base + off[2]);
    S.lastproc = reinterpret_cast<typename Smem<R, CMP>::clk_t *>(base + off[3]);
    S.lastchg = reinterpret_cast<typename Smem<R, CMP>::clk_t *>(base + off[4]);
    S.ring = reinterpret_cast<int *>(base + off[6]);
    S.scratch = reinterpret_cast<int *>(base + off[7]);
    S.sf = reinterpret_cast<R *>(base + off[8]);
    S.xr = reinterpret_cast<R *>(base + off[9]);       // arrays 9 (XR) and 10 (XN) are contiguous
    S.cinfo = reinterpret_cast<u2v *>(base + off[11]);
    S.meta = reinterpret_cast<unsigned *>(base + off[11]);
    S.fmask = reinterpret_cast<unsigned *>(S.ring + 3 * L.nr);
    S.fz = base + off[12];
    S.vbits = reinterpret_cast<unsigned *>(base + off[13]);
    S.cbits = S.vbits + (L.nblocks + 31) / 32;
    return S;
}
// the held stream's LDS arrays (compact layout only: 16-bit clocks)
template <typename R>
__device__ __forceinline__ HoldLds<int> hold_lds(const Smem<R, true> &S)
{
    HoldLds<int> H;
    H.order = S.order; H.fz = S.fz; H.lastproc = S.lastproc; H.need = S.lastchg; H.fmask = S.fmask;
    H.ring_e = S.ring; H.vbits = S.vbits; H.cbits = S.cbits;
    return H;
}
// column info {own column, meta} of lane l at ring slot ri (col: lane l's
// column offset inside its tile, used by the compact layout)
template <typename R, bool CMP>
__device__ __forceinline__ u2v cinfo_at(const FsmLaunch &L, const Smem<R, CMP> &S, int ri, int l, uint32_t col)
{
    if (!CMP) return S.cinfo[ri * 64 + l];
    u2v c;
    c.x = (uint32_t)S.ring[2 * L.nr + ri] + col;
    c.y = S.meta[ri * 64 + l];
    return c;
}

// What a lane needs about one of its bricks.
struct BInfo {
    uint32_t seg;            // byte offset (u buffer) of the own segment (OOB if none)
    uint32_t zh;             // the z-upwind node of a run start (prefetch only)
    uint32_t lseg;           // this brick's half of its column line if the line holds a valid brick
                             // (FL64 prefetch only: a loader whose own brick is past the grid end)
    int zb8, fl, ccb, ri;    // fl: C_* | F_*; ccb: cell-cache index of the brick (SLOWMODE 2); ri: ring slot
    int bid;                 // z-block id (stamps)
    int clk;                 // stream position of the brick (stamps)
    int bcm;                 // BC z-slots of the segment (generic path)
    bool zd;                 // held stream: the position's last brick below the column end -- zh is then
                             // its z-downwind node, the next brick's first only when the run continues
};

template <typename R, bool RZ, int ZSH, bool CMP>
__device__ __forceinline__ BInfo brick_info(const FsmLaunch &L, int kb, const Smem<R, CMP> &S, const Pos &p, int nstream,
                                            int lx, int ly, const BcBoxes &bc, const u2v ci)
{
    BInfo b;
    const unsigned meta = ci.y;
    const int tz = ci_tz(meta);
    const int zb = tz * kb + (RZ ? kb - 1 - p.zbs : p.zbs);
    const bool valid = pos_valid(p, nstream) && (meta & C_BLK) && zb < L.nzb;
    const uint32_t zoff = zoff_bytes<R>(zb);
    b.seg = valid ? ci.x + zoff : OOB;
    b.lseg = pos_valid(p, nstream) && (meta & C_BLK) && (zb & ~1) < L.nzb ? ci.x + zoff : OOB;
    const int zu = RZ ? zb * 8 + 8 : zb * 8 - 1;             // z-upwind node of the brick's first slot
    b.zh = (valid && (meta & C_ZH) && p.zbs == 0)
               ? ci.x + zoff_bytes<R>(zu >> 3) + (uint32_t)(zu & 7) * (uint32_t)sizeof(R) : OOB;
    b.zb8 = valid ? zb * 8 : 0;
    b.ri = p.ri;
    b.clk = p.sp;
    b.bid = S.ring[L.nr + p.ri];                              // z-block id (admit)
    int fl = valid ? (int)((meta & 0x7f) | F_VALID) : 0;
    if (zb == (RZ ? L.nzb - 1 : 0)) fl |= F_FIRST;
    if (zb == (RZ ? 0 : L.nzb - 1)) fl |= F_LAST;
    if ((meta & C_ZH) && p.zbs == 0) fl |= F_ZH;
    // held stream: the run end's z-downwind node of the position's last brick below the column end
    b.zd = CMP && valid && p.zbs == kb - 1 && !(fl & F_LAST);
    if (b.zd) {
        const int zn = RZ ? zb * 8 - 1 : zb * 8 + 8;          // z-downwind node of the brick's last slot
        b.zh = ci.x + zoff_bytes<R>(zn >> 3) + (uint32_t)(zn & 7) * (uint32_t)sizeof(R);
    }
    bool slow = (fl & C_PART) || ((fl & C_00) && zb == 0) || (valid && b.zb8 + 8 > L.nz);
    b.bcm = 0;
    if (__any(fl & C_BC)) {
        // BC z-slots of this column segment (rare: columns through a source box)
        const int e = S.ring[p.ri];
        const int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        unsigned m = 0;
        if (fl & C_BC) {
            for (int k = 0; k < bc.n; k++) {
                const int *q = bc.box + 6 * k;
                if (x >= q[0] && x <= q[1] && y >= q[2] && y <= q[3]) {
                    int lo = q[4] - b.zb8, hi = q[5] - b.zb8;
                    lo = lo < 0 ? 0 : lo; hi = hi > 7 ? 7 : hi;
                    if (lo <= hi) m |= ((2u << hi) - (1u << lo));
                }
            }
        }
        b.bcm = (int)m;
        slow |= m != 0;
    }
    if (slow) fl |= F_SLOW;
    b.fl = fl;
    b.ccb = ci_ccb(meta) + (ZSH >= 0 ? (b.zb8 >> (ZSH < 0 ? 0 : ZSH)) : 0);
    return b;
}

// offset of this lane's half of halo column j at the edge lane's position pe
// (ci: the edge lane's column info at pe; hbit: C_XOWN for x halos, C_YOWN
// for y halos; hdelta: halo_delta)
template <typename R, bool RZ>
__device__ __forceinline__ uint32_t halo_offset(const FsmLaunch &L, int kb, const Pos &pe, int nstream, int half,
                                                const u2v ci, unsigned hbit, uint32_t hdelta)
{
    const unsigned meta = ci.y;
    const int zb = ci_tz(meta) * kb + (RZ ? kb - 1 - pe.zbs : pe.zbs);
    const bool valid = pos_valid(pe, nstream) && (meta & C_BLK) && zb < L.nzb;
    const uint32_t base = ci.x + ((meta & hbit) ? 0u : hdelta);
    return valid ? base + zoff_bytes<R>(zb) + (uint32_t)half * 4u * (uint32_t)sizeof(R) : OOB;
}
// Neighbour rows: XR = S.xr[0 .. 640), XN = S.xr[640 .. 1280), each
// [half][80 rows][4] (element offsets).  Halo columns go to rows 64..79:
// j = 0..7 (x-upwind of lanes (0, j)) XR 64 + j, 8..15 (x-downwind of
// (7, j - 8)) XN 64 + j - 8, 16..23 (y-upwind of (j - 16, 0)) XR 72 + j - 16,
// 24..31 (y-downwind of (j - 24, 7)) XN 72 + j - 24.
#define XROW(arr, half, row) ((((arr) * 2 + (half)) * MCEIK_XROWS + (row)) * 4)
// Element offsets by precision: xrow = slot 0 of a row, xz(z) = z-slot z (0..7)
// from there.  fp32: [arr][half][row][4] (XROW, a row's four slots contiguous);
// fp64: [arr][z][row], so that a wave's ds_read_b64 of one z from 32 rows spans
// all 64 banks (as [row][4] it put rows r, r + 8, r + 16, r + 24 on one bank
// pair: 4-way conflicts, 69% of the fp64 kernel's LDS cycles, profiles/r06_lds).
template <typename R>
__device__ __forceinline__ constexpr int xrow(int arr, int row)
{
    return sizeof(R) == 8 ? arr * 8 * MCEIK_XROWS + row : XROW(arr, 0, row);
}
template <typename R>
__device__ __forceinline__ constexpr int xz(int z)
{
    return sizeof(R) == 8 ? z * MCEIK_XROWS : (z >> 2) * 4 * MCEIK_XROWS + (z & 3);
}
// the halo half this lane stages (slot 0 of it)
template <typename R>
__device__ __forceinline__ int halo_row_off(int lane)
{
    const int j = lane >> 1, half = lane & 1;
    return xrow<R>((j >> 3) & 1, 64 + ((j >> 4) << 3) + (j & 7)) + xz<R>(4 * half);
}
template <typename R>
__device__ __forceinline__ void store4(R *d, const R (&v)[4])
{
#pragma unroll
    for (int i = 0; i < 4; i++) d[xz<R>(i)] = v[i];
}
template <typename R>
__device__ __forceinline__ void store_row(R *x, int arr, int lane, const R (&v)[8])
{
    R *a = x + xrow<R>(arr, lane);
#pragma unroll
    for (int z = 0; z < 8; z++) a[xz<R>(z)] = v[z];
}
template <typename R>
__device__ __forceinline__ void load_row(const R *x, int off0, R (&v)[8])   // off0 = xrow(arr, row)
{
    const R *a = x + off0;
#pragma unroll
    for (int z = 0; z < 8; z++) v[z] = a[xz<R>(z)];
}

// Loads / stores that most lanes skip (z-upwind nodes of run starts, u0
// copies, unchanged segments) are issued only when some lane needs them:
// every wave-instruction costs address-unit time for all 64 lanes.
// Pair-coalesced segment loads (fp32): lanes 2i and 2i+1
// read the two 16-B halves of lane 2i's segment with one instruction and of
// lane 2i+1's with the other, so each wave-instruction touches 32 lines
// instead of 64; pair_finish() swaps the halves into place (DPP quad_perm
// [1,0,3,2]) once the data has arrived.
__device__ __forceinline__ void pair_issue(Rsrc r, uint32_t seg, float (&a)[4], float (&b)[4])
{
    const bool odd = threadIdx.x & 1;
    const uint32_t segp = dpp_swap_pair(seg);
    bload4(r, odd ? segp + 16u : seg, a);       // even: own [0,4)  odd: partner's [4,8)
    bload4(r, odd ? seg + 16u : segp, b);       // even: partner's [0,4)  odd: own [4,8)
}
__device__ __forceinline__ void pair_finish(const float (&a)[4], const float (&b)[4], float (&v)[8])
{
    const bool odd = threadIdx.x & 1;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float send = odd ? a[i] : b[i];
        const float recv = __builtin_bit_cast(float, dpp_swap_pair(__builtin_bit_cast(unsigned, send)));
        v[i] = odd ? recv : a[i];
        v[4 + i] = odd ? b[i] : recv;
    }
}

// Pair-coalesced segment store (fp32): the same pairing for the write-back of
// changed segments (each instruction stores the two halves of one lane's
// segment, predicated on that lane's change).
__device__ __forceinline__ void pair_store(Rsrc r, uint32_t seg, bool chg, const float (&v)[8])
{
    const bool odd = threadIdx.x & 1;
    const uint32_t own = chg ? seg : OOB;
    const uint32_t oth = dpp_swap_pair(own);    // partner's offset (OOB if unchanged)
    float x[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        x[i] = __builtin_bit_cast(float, dpp_swap_pair(__builtin_bit_cast(unsigned, odd ? v[i] : v[4 + i])));
    // even: own [0,4) | odd: even's [4,8)         even: odd's [0,4) | odd: own [4,8)
    // (branch-free selects: both instructions carry all 64 lanes)
    bstore4(r, odd ? oth + 16u : own, odd ? x[0] : v[0], odd ? x[1] : v[1], odd ? x[2] : v[2], odd ? x[3] : v[3]);
    bstore4(r, odd ? own + 16u : oth, odd ? v[4] : x[0], odd ? v[5] : x[1], odd ? v[6] : x[2], odd ? v[7] : x[3]);
}

// ---- FL64: whole-line own loads of the fp64 compile-time-kb instances.
// A 128-B column line holds two 8-z fp64 bricks, which a
// lane visits in two consecutive steps (kb even: a position's bricks pair up
// as zbs 0/1, 2/3 in either z direction).  x-adjacent lanes (a pair) run one
// step apart, so at every step exactly one lane of a pair -- the loader,
// whose prefetch target is the first brick of a line in sweep order --
// starts a line.  Both lanes load the loader's whole line in 4 dwordx4 loads
// (lane parity p: quarters p and p + 2 of each half, so an instruction
// touches 32 lines, 32 B of each): the now half goes to the loader's XN row
// at the end of the step; the later half waits one step in LDS (HOLD) and
// then goes to the row of the same lane, the non-loader of the next step.
// As fsm16's FL, with the held half in LDS instead of registers (this
// instance runs at its VGPR limit).  Without it a line was read as two 64-B
// halves a step apart and the L2 re-fetched part of them in between.
#define XHOLD(k) (xrow<double>(2, 0) + (k) * 128)   // HOLD quarter k of lane l: 2 values at + 2 l
__device__ __forceinline__ void line_issue64(Rsrc r, uint32_t lseg, bool isl, double (&a)[4], double (&h)[4],
                                             int &rowl, int &rowo)
{
    const int lane = threadIdx.x, par = lane & 1;
    const bool islp = dpp_swap_pair((unsigned)isl) != 0u;
    const uint32_t segp = dpp_swap_pair(lseg);
    const uint32_t sl = isl ? lseg : (islp ? segp : OOB);     // the loader's now half
    const uint32_t sh = sl ^ 64u;                             // its later half (OOB stays OOB)
    const uint32_t o = (uint32_t)par * 16u;
    d2v x = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, sl + o, 0, 0));
    d2v y = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, sl + o + 32u, 0, 0));
    d2v z = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, sh + o, 0, 0));
    d2v w = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, sh + o + 32u, 0, 0));
    a[0] = x.x; a[1] = x.y; a[2] = y.x; a[3] = y.y;
    h[0] = z.x; h[1] = z.y; h[2] = w.x; h[3] = w.y;
    rowl = isl ? lane : (lane ^ 1);
    rowo = lane ^ (rowl == lane ? 1 : 0);
}
// end of step: the loader's next brick (this step's now half) and the other
// lane's (the half held since the previous step) into the XN rows; this
// step's later half into HOLD.  Quarter q of a row: half q >> 1, values
// 2 (q & 1) .. + 1.
__device__ __forceinline__ void line_write64(double *x, int rowl, int rowo, const double (&a)[4], const double (&h)[4])
{
    const int lane = threadIdx.x, par = lane & 1;
    double *hd = x + XHOLD(0) + 2 * lane;
    const double p0 = hd[0], p1 = hd[1], p2 = hd[128], p3 = hd[129];
    hd[0] = h[0]; hd[1] = h[1]; hd[128] = h[2]; hd[129] = h[3];
    double *l = x + xrow<double>(1, rowl) + xz<double>(2 * par), *o = x + xrow<double>(1, rowo) + xz<double>(2 * par);
    l[0] = a[0]; l[xz<double>(1)] = a[1]; l[xz<double>(4)] = a[2]; l[xz<double>(5)] = a[3];
    o[0] = p0; o[xz<double>(1)] = p1; o[xz<double>(4)] = p2; o[xz<double>(5)] = p3;
}

// Slowness of the 8 nodes of a segment (prefetch; multiplied by h when staged).
// Modes 0 and 1 only; the column's x, y come from the stream ring.
template <typename R, int SLOWMODE, bool CMP>
__device__ __forceinline__ void prefetch_slow(const FsmLaunch &L, const Smem<R, CMP> &S, Rsrc sr, const BInfo &b,
                                              int lx, int ly, R (&s)[8])
{
    if (SLOWMODE == 0) {
        bload8(sr, b.seg, s);
    } else {
        const int e = S.ring[b.ri];
        const uint32_t mx = L.magic_rx, my = L.magic_ry, mz = L.magic_rz;
        int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        x = x < L.nx ? x : L.nx - 1; y = y < L.ny ? y : L.ny - 1;
        const uint32_t col = ((uint32_t)y * my >> 20) * (uint32_t)L.ncx + ((uint32_t)x * mx >> 20);
        const uint32_t plane = (uint32_t)L.ncx * L.ncy;
        const bool v = (b.fl & F_VALID) != 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            int z = b.zb8 + i;
            z = z < L.nz ? z : L.nz - 1;
            const uint32_t off = (col + ((uint32_t)z * mz >> 20) * plane) * 4u;
            s[i] = (R)bload1f(sr, v ? off : OOB);
        }
    }
}

// Decide stream position `pos` (global clock C = clock0 + pos): a z-block
// (returns its entry, *zh = run start inside the column), a bubble (-1) or the
// end of the sweep (-2).  A z-block needs an update iff it changed at its
// last visit, a face neighbour changed since, or a sweep-upwind x/y neighbour
// is still in flight (its changes are not known yet); otherwise its update
// would recompute every node from unchanged inputs and return the current
// value.  Once a run starts, the next block's z-upwind neighbour is in flight,
// so the run covers the rest of the column.
template <typename R, bool RZ, bool CMP>
__device__ __forceinline__ int decide(const FsmLaunch &L, const Smem<R, CMP> &S, Stream &st, int C, int rx, int ry, int &zh)
{
    const int lane = threadIdx.x;
    const int nt = L.ntiles, nzk = L.nzk;
    zh = 0;
    if (st.tile < 0) {
        while (st.cursor < nt) {
            const int k = st.cursor + lane;
            int k0 = nzk, entry = 0;
            if (k < nt) {
                const int o = S.order[k];
                const int txs = o & 0xffff, tys = o >> 16;
                const int tx = rx ? L.ntx - 1 - txs : txs, ty = ry ? L.nty - 1 - tys : tys;
                const int id = ty * L.ntx + tx;
                const int xu = txs > 0 ? id + (rx ? 1 : -1) : -1;
                const int yu = tys > 0 ? id + (ry ? L.ntx : -L.ntx) : -1;
                entry = tx | (ty << 12);
                for (int kz = 0; kz < nzk; kz++) {
                    const int tz = RZ ? nzk - 1 - kz : kz;
                    const int b = tz * nt + id;
                    const int lp = S.lastproc[b];
                    bool d = S.lastchg[b] >= lp;
                    if (tx > 0) d |= S.lastchg[b - 1] > lp;
                    if (tx < L.ntx - 1) d |= S.lastchg[b + 1] > lp;
                    if (ty > 0) d |= S.lastchg[b - L.ntx] > lp;
                    if (ty < L.nty - 1) d |= S.lastchg[b + L.ntx] > lp;
                    if (tz > 0) d |= S.lastchg[b - nt] > lp;
                    if (tz < nzk - 1) d |= S.lastchg[b + nt] > lp;
                    if (xu >= 0) d |= S.lastproc[tz * nt + xu] > C - L.infl;
                    if (yu >= 0) d |= S.lastproc[tz * nt + yu] > C - L.infl;
                    if (d) { k0 = kz; break; }
                }
            }
            const unsigned long long m = __ballot(k0 < nzk);
            if (m) {
                const int first = __builtin_ctzll(m);
                st.cursor += first + 1;
                st.tile = __builtin_amdgcn_readfirstlane(__shfl(entry, first, 64));
                st.k0 = st.k = __builtin_amdgcn_readfirstlane(__shfl(k0, first, 64));
                break;
            }
            st.cursor += 64;
        }
        if (st.tile < 0) return -2;
        // bubbles before the run: block k sits at position pos + wait + (k - k0),
        // which must be >= vis positions after its upwind x/y neighbours' visits
        const int tx = st.tile & 0xfff, ty = st.tile >> 12;
        const int txs = rx ? L.ntx - 1 - tx : tx, tys = ry ? L.nty - 1 - ty : ty;
        const int id = ty * L.ntx + tx;
        int need = 0;
        for (int kz = st.k0 + lane; kz < nzk; kz += 64) {
            const int tz = RZ ? nzk - 1 - kz : kz;
            int p = -0x40000000;
            if (txs > 0) p = max(p, (int)S.lastproc[tz * nt + id + (rx ? 1 : -1)]);
            if (tys > 0) p = max(p, (int)S.lastproc[tz * nt + id + (ry ? L.ntx : -L.ntx)]);
            need = max(need, p + L.vis - (kz - st.k0) - C);
        }
        st.wait = __builtin_amdgcn_readfirstlane(wave_max(need));
    }
    if (st.wait > 0) {
        st.wait--;
        return -1;
    }
    const int kz = st.k;
    zh = kz == st.k0 && kz > 0;
    const int tz = RZ ? nzk - 1 - kz : kz;
#ifdef MCEIK_STEPSTATS
    if (kz > st.k0 && lane == 0) {           // experiment: continuation block clean except its z-upwind
        const int tx = st.tile & 0xfff, ty = st.tile >> 12, id = ty * L.ntx + tx, b = tz * nt + id;
        const int txs = rx ? L.ntx - 1 - tx : tx, tys = ry ? L.nty - 1 - ty : ty;
        const int lp = S.lastproc[b];
        bool d = S.lastchg[b] >= lp;
        if (tx > 0) d |= S.lastchg[b - 1] > lp;
        if (tx < L.ntx - 1) d |= S.lastchg[b + 1] > lp;
        if (ty > 0) d |= S.lastchg[b - L.ntx] > lp;
        if (ty < L.nty - 1) d |= S.lastchg[b + L.ntx] > lp;
        const int zdn = RZ ? tz - 1 : tz + 1;
        if (zdn >= 0 && zdn < nzk) d |= S.lastchg[zdn * nt + id] > lp;
        if (txs > 0) d |= S.lastproc[b + (rx ? 1 : -1)] > C - L.infl;
        if (tys > 0) d |= S.lastproc[b + (ry ? L.ntx : -L.ntx)] > C - L.infl;
        if (!d) S.scratch[2]++;
    }
#endif
    const int e = st.tile | (tz << 24);
    if (++st.k == nzk) st.tile = -1;
    return e;
}

// Admit stream position pos (ring slot ri): a z-block (every lane writes its
// column info -- the tile part is computed once per run -- and lane 0 the
// ring entry, the block id and the block's clocks) or a bubble.  Visit
// statistics: the bricks lane (0,0) will update (= z-bricks of the block in
// the grid) and the column segments of all lanes (S.scratch[0], [1]).
template <typename R, bool CMP>
__device__ __forceinline__ void admit(const FsmLaunch &L, int kb, const Smem<R, CMP> &S, const BcBoxes &bc, int entry,
                                      int zh, int ri, int clock, int clock_it, int lx, int ly, int lxs, int lys, int rx,
                                      int ry, ColTile &ct)
{
    u2v ci;
    int bid = 0, nbv = 0;
    uint32_t tbase = 0;
    if (entry >= 0) {
        const int tz = (entry >> 24) & 0xff;
        bid = tz * L.ntiles + (entry & 0xfff) + ((entry >> 12) & 0xfff) * L.ntx;
        tbase = (uint32_t)((entry & 0xfff) + ((entry >> 12) & 0xfff) * L.ntx) * tile_bytes<R>(L);
        nbv = min(kb, L.nzb - tz * kb);
        // first visit of the block in this iteration: no visit since the iteration's first clock
        // (held stream: its clocks restart every sweep, the iteration's visits are a bitmap)
        const int u0flag = CMP ? !((S.vbits[bid >> 5] >> (bid & 31)) & 1u)
                                                : (int)S.lastproc[bid] < clock_it;
        if ((entry & 0xffffff) != ct.tile) column_tile<R>(L, bc, entry, lx, ly, lxs, lys, rx, ry, ct);
        ci.x = ct.col;
        ci.y = column_word(L, kb, ct, tz, ri, u0flag, zh);
    } else {
        ci.x = OOB; ci.y = 0;
    }
    const int nact = L.visit_stats && entry >= 0 ? __builtin_popcountll(__ballot(ct.fl & C_ACT)) : 0;
    asm volatile("" ::: "memory");
    if (CMP)
        S.meta[ri * 64 + threadIdx.x] = ci.y;
    else
        S.cinfo[ri * 64 + threadIdx.x] = ci;
    if (threadIdx.x == 0) {
        if (CMP) S.ring[2 * L.nr + ri] = (int)tbase;
        if (entry >= 0) {
            S.lastproc[bid] = (typename Smem<R, CMP>::clk_t)clock;
            if (CMP) S.vbits[bid >> 5] |= 1u << (bid & 31);
            if (L.visit_stats) {
                S.scratch[0] += nbv;
                S.scratch[1] += nbv * nact;
            }
        }
        S.ring[ri] = entry;
        S.ring[L.nr + ri] = bid;
    }
    asm volatile("" ::: "memory");
}

// x/y neighbour minima and f = s*h of slot pj.  The four neighbour rows
// (x/y-upwind lanes' new values, downwind lanes' old values, or the halo
// rows for tile-edge lanes) were read from LDS at the start of the brick.
template <typename R, int SLOWMODE, int ZSH, bool GENERIC, bool WANTF, bool CMP>
__device__ __forceinline__ void gather_xy(const FsmLaunch &L, const Smem<R, CMP> &S, const BInfo &b0, const R (&c)[8],
                                          const R (&xmr)[8], const R (&xpr)[8], const R (&ymr)[8], const R (&ypr)[8],
                                          int pj, bool xp, bool xn, bool yp, bool yn, R &ux, R &uy, R &fv)
{
    const int lane = threadIdx.x;
    const R self = c[pj];
    if (!WANTF) {
    } else if (SLOWMODE == 2) {
        if (ZSH >= 0 && !GENERIC) {
            fv = (R)S.cc[b0.ccb + (pj >> (ZSH < 0 ? 0 : ZSH))];
        } else {
            const int zabs = b0.zb8 + pj;
            fv = (R)S.cc[b0.ccb + (ZSH >= 0 ? (pj >> (ZSH < 0 ? 0 : ZSH))
                                            : (int)(((unsigned)(zabs < L.nz ? zabs : L.nz - 1) * L.magic_rz) >> 20))];
        }
        if (sizeof(R) == 8) fv *= (R)L.h;        // fp32 entries already hold s*h
    } else {
        fv = S.sf[pj * 64 + lane];
    }
    R xup = xmr[pj], xdn = xpr[pj], yup = ymr[pj], ydn = ypr[pj];
    if (GENERIC) {
        xup = xp ? xup : self; xdn = xn ? xdn : self; yup = yp ? yup : self; ydn = yn ? ydn : self;
    }
    ux = fmin_(xup, xdn);
    uy = fmin_(yup, ydn);
}

// The 8 z-slots of the current brick.  GENERIC: any brick (grid-edge columns
// of cut tiles, cut z-bricks, BC nodes, node (0,0,0) with the reference's
// ierr); otherwise the brick is interior to the grid in x, y and z up to the
// sweep-order first/last brick, no lane holds a BC node, and every lane's
// missing x/y neighbours are already its own old values (column_info).
// NC: evaluate the unconverged test (nc); the sweep drops it once a lane of
// the wave has found the iteration unconverged (the outcome cannot change, as
// for the fp64 u0 copies skipped after a big step)
template <typename R, int SLOWMODE, bool FAST, bool RZ, int ZSH, bool GENERIC, bool CMP, bool NC = true>
__device__ __forceinline__ void brick_update(const FsmLaunch &L, const Smem<R, CMP> &S, const BInfo &b0, R (&c)[8],
                                             R (&n)[8], R (&r)[8], R zc, int lx, int ly, int rx, int ry,
                                             bool &changed, bool &nc, int &ierr_last, bool zdsel, bool &c0,
                                             bool &c7)
{
    const int lane = threadIdx.x;
    const R T = (R)L.conv_thresh;
    // fp64 (v34, "big step"): a node that drops by >= tol (1 + 2^-50) in one
    // update moved by >= tol over the iteration (values only fall), so the
    // reference's |u0 - u| < tol fails: not converged, as the >= T rule says
    // in fp32 (where T = 2^26 s makes that rule empty in fp64)
    const R TB = (R)(L.tol * (1.0 + 0x1p-50));
    const int fl = b0.fl;
    bool xp = true, xn = true, yp = true, yn = true, act = true;
    if (GENERIC) {
        const int e = S.ring[b0.ri];
        const int x = (e & 0xfff) * 8 + lx, y = ((e >> 12) & 0xfff) * 8 + ly;
        const bool xlo = x > 0, xhi = x < L.nx - 1, ylo = y > 0, yhi = y < L.ny - 1;
        xp = rx ? xhi : xlo; xn = rx ? xlo : xhi; yp = ry ? yhi : ylo; yn = ry ? ylo : yhi;
        act = (fl & C_ACT) != 0;
    }
    const bool first = (fl & F_FIRST) != 0, last = (fl & F_LAST) != 0;
    // z-upwind value of slot 0: the previous brick of the lane's sequence, or
    // (run start inside the column) the node loaded from HBM
    const R zprev = (fl & F_ZH) ? zc : r[RZ ? 0 : 7];
    // the four neighbour rows (sweep-relative lanes: -1 / -8 upwind in XR,
    // +1 / +8 downwind in XN; tile-edge lanes read the halo rows)
    // fp64: each slot's four neighbours are read when the slot is updated (the
    // four whole rows would hold 64 VGPRs for the brick)
    constexpr bool LAZY = sizeof(R) == 8;
    R xmr[8], xpr[8], ymr[8], ypr[8];
    const int lxs = lane & 7, lys = lane >> 3;
    const int oxm = xrow<R>(0, lxs > 0 ? lane - 1 : 64 + lys), oym = xrow<R>(0, lys > 0 ? lane - 8 : 72 + lxs);
    const int oxp = xrow<R>(1, lxs < 7 ? lane + 1 : 64 + lys), oyp = xrow<R>(1, lys < 7 ? lane + 8 : 72 + lxs);
    // fp64: the next brick's first slot from this lane's XN row (the sweep
    // keeps no register copy of the next brick)
    R nfirst = LAZY ? S.xr[xrow<R>(1, lane) + xz<R>(RZ ? 7 : 0)] : n[RZ ? 7 : 0];
    if (zdsel) nfirst = zc;                  // held stream: a run end below the column end (HBM node)
    if (!LAZY) {
        load_row(S.xr, oxm, xmr);
        load_row(S.xr, oym, ymr);
        load_row(S.xr, oxp, xpr);
        load_row(S.xr, oyp, ypr);
    }
    // fast fp32 path over the LDS cell cache: f, f*f, 2f*f, 3f*f per cell
    constexpr bool CELLF = SLOWMODE == 2 && ZSH >= 0 && !GENERIC && sizeof(R) == 4;
    R fc = 0, ffc = 0, ff2c = 0, ff3c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int pj = RZ ? 7 - j : j;
        const int pprev = RZ ? pj + 1 : pj - 1;
        const int pnext = RZ ? pj - 1 : pj + 1;
        const R self = c[pj];
        if (LAZY) {
            const int sl = xz<R>(pj);
            xmr[pj] = S.xr[oxm + sl]; ymr[pj] = S.xr[oym + sl];
            xpr[pj] = S.xr[oxp + sl]; ypr[pj] = S.xr[oyp + sl];
        }
        R ux, uy, fv;
        gather_xy<R, SLOWMODE, ZSH, GENERIC, !CELLF>(L, S, b0, c, xmr, xpr, ymr, ypr, pj, xp, xn, yp, yn, ux, uy, fv);
        if (CELLF) {
            // one LDS read and one f*f per slowness cell (2^ZSH slots)
            if (j == 0 || (pj >> (ZSH < 0 ? 0 : ZSH)) != (pprev >> (ZSH < 0 ? 0 : ZSH))) {
                fc = (R)S.cc[b0.ccb + (pj >> (ZSH < 0 ? 0 : ZSH))];
                ffc = fc * fc;
                ff2c = ffc + ffc;
                ff3c = (R)3 * ffc;
            }
            fv = fc;
        }
        R zup, zdn;
        if (GENERIC) {
            const int zabs = b0.zb8 + pj;
            const bool zp_ex = RZ ? (zabs < L.nz - 1) : (zabs > 0);
            const bool zn_ex = RZ ? (zabs > 0) : (zabs < L.nz - 1);
            zup = zp_ex ? (j > 0 ? r[pprev] : zprev) : self;
            zdn = zn_ex ? (j < 7 ? c[pnext] : nfirst) : self;
        } else {
            zup = j > 0 ? r[pprev] : (first ? self : zprev);
            zdn = j < 7 ? c[pnext] : (last ? self : nfirst);
        }
        const R uz = fmin_(zup, zdn);
        R nv;
        if (GENERIC) {
            const int zabs = b0.zb8 + pj;
            int e;
            const R ub = godunov_bl<FAST>(ux, uy, uz, fv, e);
            const bool upd = act && zabs < L.nz && !((b0.bcm >> pj) & 1);
            nv = upd ? fmin_(self, ub) : self;
            if ((fl & C_00) && zabs == 0) ierr_last = upd ? e : 0;
        } else {
            const R ffv = CELLF ? ffc : fv * fv;
            nv = fmin_(self, godunov_v<FAST>(ux, uy, uz, fv, ffv, CELLF ? ff2c : ffv + ffv, CELLF ? ff3c : (R)3 * ffv));
        }
        const bool dec = nv < self;
        if (NC) nc |= dec && (self >= T || (sizeof(R) == 8 && self - nv >= TB));
        changed |= dec;
        if (pj == 0) c0 = dec;               // the brick's lowest / highest node changed (z faces of
        if (pj == 7) c7 = dec;               //   its block, held stream)
        r[pj] = nv;
    }
}

// One Gauss-Seidel sweep over the grid in direction (rx, ry, RZ): only the
// z-blocks admitted by decide() are visited.  Returns the number of stream
// positions used (z-blocks and bubbles).
// KB > 0: the launch's kb (bricks per z-block) as a compile-time constant
// (the ring then has nr = 2 + 16 / KB slots); 0: runtime L.kb / L.nr.
// nchg: per-lane count of changed column segments (visit statistics).
template <typename R, int SLOWMODE, bool FAST, bool RZ, int ZSH, int CCR, int KB, bool CMP>
__device__ __forceinline__ int sweep(const FsmLaunch &L, Rsrc ur, Rsrc u0r, Rsrc sr, const BcBoxes &bc,
                                     const Smem<R, CMP> &S, int rx, int ry, int clock_it, int clock0,
                                     bool &notconv, int &ierr_last, unsigned &nchg, unsigned &nsteps)
{
    const int lane = threadIdx.x, lxs = lane & 7, lys = lane >> 3, d = lxs + lys;
    const int lx = rx ? 7 - lxs : lxs, ly = ry ? 7 - lys : lys;
    const R UN = Num<R>::unan();
    const R hr = (R)L.h;
    const int kb = KB > 0 ? KB : L.kb;
    const int nr = KB > 0 ? 2 + (16 + KB - 1) / (KB > 0 ? KB : 1) : L.nr;

    // halo loader role of this lane (halo_edge_lane)
    const int hj = lane >> 1, hh = lane & 1, he = halo_edge_lane(hj), hd = (he & 7) + (he >> 3);
    const unsigned hbit = hj < 16 ? C_XOWN : C_YOWN;
    const uint32_t hdelta = halo_delta(L, tile_bytes<R>(L), hj, he, rx, ry);
    const int hso = halo_row_off<R>(lane);
    // column offsets inside a tile (the compact layout's cinfo_at): this lane's, the halo edge lane's
    const uint32_t lanecol = (uint32_t)colpos(lx, ly) * 128u;
    const uint32_t hcol = (uint32_t)colpos(rx ? 7 - (he & 7) : (he & 7), ry ? 7 - (he >> 3) : (he >> 3)) * 128u;

    // stream bookkeeping (wave-uniform)
    Stream st;
    st.cursor = 0; st.tile = -1; st.k = 0; st.k0 = 0; st.wait = 0;
    // the held stream (compact layout; fsm_hold.h): clocks restart at 64 every sweep
    constexpr bool HOLD = CMP;
    // (its scan state -- first incomplete tile, previous position's tile -- lives in LDS scratch
    // [4], [5]: fewer scalar registers live across the step loop)
    // this lane's change-mask bits of a changed brick: the block, and its x / y faces when the
    // lane's column is a tile edge (absolute orientation)
    const unsigned xyface = HOLD_OWN | (lx == 0 ? 2u : 0u) | (lx == 7 ? 4u : 0u) | (ly == 0 ? 8u : 0u) |
                            (ly == 7 ? 16u : 0u);
    if constexpr (HOLD) {
        hold_norm(L, hold_lds(S));
        if (lane == 0) { S.scratch[4] = 0; S.scratch[5] = -1; }
        clock0 = 64;
    }
    // the next position's block (held stream: after settling the visit infl positions back)
    auto decide_any = [&](int pos, int ri, int &zh) __attribute__((always_inline)) -> int {
        if constexpr (HOLD) {
            const HoldLds<int> H = hold_lds(S);
            // positions are decided one after another: settle the one infl back
            const int q = pos - L.infl;
            if (q >= 0) hold_settle(L, H, q % nr, clock0 + q);
            return hold_decide_scan<RZ>(L, H, S.scratch + 4, clock0 + pos, rx, ry, ri == 0 ? nr - 1 : ri - 1, L.infl,
                                        L.vis, zh);
        } else {
            return decide<R, RZ>(L, S, st, clock0 + pos, rx, ry, zh);
        }
    };
    R c[8], n[8], q[8], r[8], fq[8], hq[4], hn[4];
    constexpr bool PAIR = sizeof(R) == 4;
    // FL64: whole-line own loads (line_issue64): la / lh this step's quarters
    // of the loader's now / later half, rowl / rowo the XN rows they go to
    constexpr bool FL64 = sizeof(R) == 8 && KB > 0 && (KB & 1) == 0;
    double la[4], lh[4];
    int rowl = 0, rowo = 0;
    float qa[4], qb[4];                  // PAIR: raw halves of q
    R zc, zn, zq;                    // z-upwind values of run starts (vb .. vb+2)
    float ccv[CCR];
    int ccsize = 0;
    ColTile ct;
    ct.tile = -1;
    // prologue decisions: the positions of lane (0,0)'s bricks 0..AH-1; the
    // loop then decides position (B+AH)/kb (own segments are loaded AH = 2
    // steps ahead)
    int ndecided = 0, nstream = 0x7fffffff, dri = 0;
    constexpr int AH = MCEIK_AHEAD;      // own segments loaded AH = 2 steps ahead
    for (int pos = 0; pos <= (AH - 1) / kb; pos++) {
        int zh;
        const int e = decide_any(pos, dri, zh);
        if (e == -2) {
            if (pos == 0) return 0;                         // nothing changed near any block: skip the sweep
            nstream = pos;
            break;
        }
        admit<R>(L, kb, S, bc, e, zh, dri, clock0 + pos, clock_it, lx, ly, lxs, lys, rx, ry, ct);
        if (SLOWMODE == 2 && e >= 0) {
            cc_issue<CCR>(L, kb, sr, e, ccv, ccsize);
            TRAFU(S, 5, ccsize * 4);
            cc_write<R, CCR>(L, S.cc, dri, ccv, ccsize, (float)L.h);
        }
        ndecided = pos + 1;
        if (++dri == nr) dri = 0;
    }
    asm volatile("" ::: "memory");
    // Brick info of vb (b0), vb+1 (b1); the loop computes vb+AH's (b3) once, uses its offsets for the own-segment
    // prefetch and carries it (one column-info read and decode per brick).
    Pos p3;
    pos_init(p3, -d, kb, nr);
    BInfo b0 = brick_info<R, RZ, ZSH>(L, kb, S, p3, nstream, lx, ly, bc, cinfo_at(L, S, p3.ri, lane, lanecol));
    // prologue: c, n, q = bricks vb0 .. vb0+2; stage f and halos of vb0
    bload8(ur, b0.seg, c);
    if (SLOWMODE != 2) prefetch_slow<R, SLOWMODE>(L, S, sr, b0, lx, ly, fq);
    Pos pe;                              // the halo's edge lane position (vb+2 in the loop)
    pos_init(pe, -hd, kb, nr);
    {
        const uint32_t ho = halo_offset<R, RZ>(L, kb, pe, nstream, hh, cinfo_at(L, S, pe.ri, he, hcol), hbit, hdelta);
        bload4(ur, ho, hq);
        TRAF(S, 1, ho != OOB, 4 * sizeof(R));
    }
    zc = bload1(ur, b0.zh, R());
    TRAF(S, 0, b0.seg != OOB, 8 * sizeof(R));
    TRAF(S, 2, b0.zh != OOB, sizeof(R));
    pos_adv(p3, kb, nr);
    BInfo b1 = brick_info<R, RZ, ZSH>(L, kb, S, p3, nstream, lx, ly, bc, cinfo_at(L, S, p3.ri, lane, lanecol));
    bload8(ur, b1.seg, n);
    pos_adv(pe, kb, nr);
    {
        const uint32_t ho = halo_offset<R, RZ>(L, kb, pe, nstream, hh, cinfo_at(L, S, pe.ri, he, hcol), hbit, hdelta);
        bload4(ur, ho, hn);   // halos of vb+1
        TRAF(S, 1, ho != OOB, 4 * sizeof(R));
    }
    zn = bload1(ur, b1.zh, R());
    TRAF(S, 0, b1.seg != OOB, 8 * sizeof(R));
    TRAF(S, 2, b1.zh != OOB, sizeof(R));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r[i] = UN;
        if (SLOWMODE != 2) S.sf[i * 64 + lane] = fq[i] * hr;
    }
    store4(S.xr + hso, hq);                       // halos of vb0
    store_row(S.xr, 0, lane, r);                   // no results yet (u_nan)
    store_row(S.xr, 1, lane, n);                   // brick vb0 + 1
    if (FL64) {
        // HOLD for step 0: quarters p, p + 2 of the brick the pair's step-0
        // non-loader targets (the second brick of a line it would have started
        // one step earlier), loaded from that lane's own segment
        Pos pn = p3;
        pos_adv(pn, kb, nr);
        const bool nl = pn.vb >= 0 && (pn.zbs & 1) == 1;
        const uint32_t sn = nl ? brick_info<R, RZ, ZSH>(L, kb, S, pn, nstream, lx, ly, bc,
                                                         cinfo_at(L, S, pn.ri, lane, lanecol)).seg
                               : OOB;
        const bool nlp = dpp_swap_pair((unsigned)nl) != 0u;
        const uint32_t snp = dpp_swap_pair(sn);
        const uint32_t s0 = (nl ? sn : (nlp ? snp : OOB)) + (uint32_t)(lane & 1) * 16u;
        d2v x = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(ur, s0, 0, 0));
        d2v y = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(ur, s0 + 32u, 0, 0));
        double *hd = reinterpret_cast<double *>(S.xr) + XHOLD(0) + 2 * lane;
        hd[0] = x.x; hd[1] = x.y; hd[128] = y.x; hd[129] = y.y;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) hq[i] = hn[i];
    // Wait for the prologue's loads here, once per sweep: a register the loop
    // carries in from a prologue load would otherwise count as a pending load
    // at the loop head, and its first use in every step would wait on vmcnt --
    // i.e. for the previous step's write-back stores as well.
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("" : "+v"(c[i]), "+v"(n[i]));
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(hq[i]));
    asm volatile("" : "+v"(zc), "+v"(zn));
    asm volatile("" ::: "memory");

    int ph = AH % kb;                // (B + AH) mod kb: 0 when lane (0,0)'s vb+AH starts a new position
    int cc_pend = -1;                // ring slot whose cell loads (ccv) are written next step
    int B = 0;
    // The stream decision for step B is made at the end of step B-1 (after
    // its write-back, so it reads the same block clocks) and the loop tests
    // its exit at the bottom: one path around the loop, so the loop-carried
    // registers need no phi copies on a second edge
    bool ccfill = false;
    int ccri = 0;
    auto decide_step = [&]() __attribute__((always_inline)) {
        // ---- stream decision for the position lane (0,0) prefetches in step B
        ccfill = false;
        ccri = 0;
        if (ph == 0 && nstream == 0x7fffffff) {
            const int pos = ndecided;
            int zh;
            const int e = decide_any(pos, dri, zh);
            if (e == -2) {
                nstream = pos;
            } else {
                admit<R>(L, kb, S, bc, e, zh, dri, clock0 + pos, clock_it, lx, ly, lxs, lys, rx, ry, ct);
                if (SLOWMODE == 2 && e >= 0) {
                    cc_issue<CCR>(L, kb, sr, e, ccv, ccsize);
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
    auto step = [&](R (&c)[8], R (&n)[8], R (&hq)[4], R (&hn)[4]) __attribute__((always_inline)) -> bool {
        // ---- prefetch: own segment and halos of vb+AH (consumed at the end
        // of this step, before its stores; halos staged to LDS at the end of
        // the next), slowness of vb+1 (modes 0/1)
        // (both column-info reads issued before either is decoded: one LDS
        // latency per step instead of two)
        pos_adv(p3, kb, nr);
        pos_adv(pe, kb, nr);
        const u2v ci3 = cinfo_at(L, S, p3.ri, lane, lanecol), cie = cinfo_at(L, S, pe.ri, he, hcol);
        __builtin_amdgcn_sched_barrier(0);     // keep the two reads ahead of every use
        const BInfo b3 = brick_info<R, RZ, ZSH>(L, kb, S, p3, nstream, lx, ly, bc, ci3);
        if (PAIR)
            pair_issue(ur, b3.seg, qa, qb);
        else if (FL64)
            line_issue64(ur, b3.lseg, p3.vb >= 0 && (p3.zbs & 1) == 0, la, lh, rowl, rowo);
        else
            bload8(ur, b3.seg, q);
        zq = __any(b3.zh != OOB) ? bload1(ur, b3.zh, R()) : R(0);
        {
            const uint32_t ho = halo_offset<R, RZ>(L, kb, pe, nstream, hh, cie, hbit, hdelta);
            bload4(ur, ho, hn);
            TRAF(S, 1, ho != OOB, 4 * sizeof(R));
            TRAF(S, 0, b3.seg != OOB, 8 * sizeof(R));
            TRAF(S, 2, b3.zh != OOB, sizeof(R));
        }
        if (SLOWMODE != 2) prefetch_slow<R, SLOWMODE>(L, S, sr, b1, lx, ly, fq);

        // ---- the 8 z-slots of the current brick (held stream: a run end's z-downwind node is the
        // one loaded from HBM)
        __builtin_amdgcn_s_setprio(0);          // the update at the SIMD's low priority (fsm16_kernel.hip)
        bool changed = false, nc = false, c0 = false, c7 = false;
        const bool zdsel = HOLD && b0.zd && !(S.fmask[b0.ri] & HOLD_CONT);
        if (__any(b0.fl & F_SLOW))
            brick_update<R, SLOWMODE, FAST, RZ, ZSH, true>(L, S, b0, c, n, r, zc, lx, ly, rx, ry, changed, nc,
                                                           ierr_last, zdsel, c0, c7);
        else if (!__any(notconv))
            brick_update<R, SLOWMODE, FAST, RZ, ZSH, false>(L, S, b0, c, n, r, zc, lx, ly, rx, ry, changed, nc,
                                                            ierr_last, zdsel, c0, c7);
        else
            brick_update<R, SLOWMODE, FAST, RZ, ZSH, false, CMP, false>(L, S, b0, c, n, r, zc, lx, ly, rx, ry,
                                                                        changed, nc, ierr_last, zdsel, c0, c7);
        const bool val = (b0.fl & F_VALID) != 0;
        changed = changed && val;
        notconv |= nc && val;
        nchg += changed ? 1u : 0u;
        __builtin_amdgcn_s_setprio(2);          // the bookkeeping to the next loads at raised priority

        // ---- consume this step's loads before any store of the step is issued.
        // gfx9's vmcnt retires loads and stores in issue order, so a wait for a
        // load placed after the write-back (the loop's register copies of the
        // prefetched values) would also wait for those stores to complete.
        // Stage the prefetched slowness/halos of vb+1 for the next step (the
        // update has read this step's halos), finish the brick after next and
        // rotate the z-upwind and halo registers.
        if (SLOWMODE == 2) {
            // cells of the position admitted one step earlier: lane (0,0)
            // enters it at the next step, so a step of latency cover is free
            // (kb >= 2: the next admission, which reloads ccv, is >= 2 steps on)
            if (kb >= 2) {
                if (cc_pend >= 0) cc_write<R, CCR>(L, S.cc, cc_pend, ccv, ccsize, (float)L.h);
                cc_pend = ccfill ? ccri : -1;
            } else if (ccfill) {
                cc_write<R, CCR>(L, S.cc, ccri, ccv, ccsize, (float)L.h);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) S.sf[i * 64 + lane] = fq[i] * hr;
        }
        store4(S.xr + hso, hq);
        R nn[8];
        if (PAIR) {
            pair_finish(qa, qb, reinterpret_cast<float (&)[8]>(nn));
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (!FL64) nn[i] = q[i];
            }
        }
        // u0: a block's first visit in the iteration (old values c)
        // (once the iteration is known unconverged its verify never runs, so
        // its remaining u0 copies are not needed)
        auto u0_store = [&]() __attribute__((always_inline)) {
            if (__any(b0.fl & C_U0) && !__any(notconv)) {
                R m = fmin_(fmin_(fmin_(c[0], c[1]), fmin_(c[2], c[3])), fmin_(fmin_(c[4], c[5]), fmin_(c[6], c[7])));
                const bool st0 = m < (R)L.conv_thresh && (b0.fl & C_U0);
                if (__any(st0)) bstore8(u0r, st0 ? b0.seg : OOB, c);
                TRAF(S, 4, st0, 8 * sizeof(R));
            }
        };
        // neighbour rows for the next step: this step's results, the next brick
        // (fp64: the brick of the next step is read back from the XN row first,
        // so c's u0 copy is stored before)
        constexpr bool LAZYN = sizeof(R) == 8;
        if (LAZYN) u0_store();
        store_row(S.xr, 0, lane, r);
        if (LAZYN) load_row(S.xr, xrow<R>(1, lane), c);
        if (FL64)
            line_write64(reinterpret_cast<double *>(S.xr), rowl, rowo, la, lh);
        else
            store_row(S.xr, 1, lane, nn);
#pragma unroll
        for (int i = 0; i < 4; i++) hq[i] = hn[i];
        zc = zn; zn = zq;
        // materialise the copies here (the loads' waits land here, before the
        // stores); otherwise they become the loop's phi copies at the latch
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (!FL64) asm volatile("" : "+v"(nn[i]));
        }
        if (FL64) {
#pragma unroll
            for (int i = 0; i < 4; i++) asm volatile("" : "+v"(la[i]), "+v"(lh[i]));
        }
        asm volatile("" : "+v"(hq[0]), "+v"(hq[1]), "+v"(hq[2]), "+v"(hq[3]));
        asm volatile("" : "+v"(zn));
        asm volatile("" ::: "memory");

        // ---- write-back, u0 at a block's first visit of the iteration, change stamps
        if (__any(changed)) {
            if (PAIR)
                pair_store(ur, b0.seg, changed, reinterpret_cast<const float (&)[8]>(r));
            else
                bstore8(ur, changed ? b0.seg : OOB, r);
            TRAF(S, 3, changed, 8 * sizeof(R));
        }
        if (!LAZYN) u0_store();
        if constexpr (HOLD) {
            // what this lane changed: the block, its x / y faces (edge columns), its z faces (the
            // block's lowest / highest node of the column)
            const int zr = (b0.zb8 >> 3) % kb;                     // brick index in the block
            const bool zlo = changed && zr == 0 && c0, zhi = changed && zr == kb - 1 && c7;
            if (changed) atomicOr(&S.fmask[b0.ri], xyface | (zlo ? HOLD_ZLO : 0u) | (zhi ? HOLD_ZHI : 0u));
        } else if (changed) {
            S.lastchg[b0.bid] = (typename Smem<R, CMP>::clk_t)(clock0 + b0.clk);   // lanes of one block write the same value
        }
        asm volatile("" ::: "memory");
        if (!LAZYN) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                c[i] = n[i];
                n[i] = nn[i];
            }
        }
        b0 = b1;
        b1 = b3;
        if (++ph == kb) ph = 0;
        B++;
        decide_step();
        return more();
    };
    decide_step();
    if (more()) {
        do {
        } while (step(c, n, hq, hn));
    }
    __builtin_amdgcn_s_setprio(0);
    nsteps += (unsigned)B;                           // macro steps of this sweep (visit statistics)
    if constexpr (HOLD) {
        // the last visits' changes (every lane is past them)
        const HoldLds<int> H = hold_lds(S);
        for (int q = max(0, nstream - L.infl + 1); q < nstream; q++) hold_settle(L, H, q % nr, clock0 + q);
    }
    return nstream;
}

// End-of-iteration check of the nodes below T (run only when no node >= T
// changed): the z-blocks that changed in this iteration (lastchg >= the
// iteration's first clock); u0 was stored at their first visit.
template <typename R, bool CMP>
__device__ __forceinline__ void verify_small(const FsmLaunch &L, Rsrc ur, Rsrc u0r, const Smem<R, CMP> &S, int clock_it, bool &notconv)
{
    const int lane = threadIdx.x, lx = lane & 7, ly = lane >> 3;
    const R T = (R)L.conv_thresh, tolr = (R)L.tol;
    for (int base = 0; base < L.nblocks; base += 64) {
        const int k = base + lane;
        const bool flag = k < L.nblocks && (CMP ? ((S.cbits[k >> 5] >> (k & 31)) & 1u) != 0
                                                 : S.lastchg[k] >= clock_it);
        unsigned long long m = __ballot(flag);
        while (m) {
            const int bid = base + __builtin_ctzll(m);
            m &= m - 1;
            const int tz = bid / L.ntiles, id = bid - tz * L.ntiles;
            const int tx = id % L.ntx, ty = id / L.ntx;
            const int x = tx * 8 + lx, y = ty * 8 + ly;
            const int zend = min(tz * L.kb + L.kb, L.nzb);
            for (int zb = tz * L.kb; zb < zend; zb++) {
                const uint32_t seg = (uint32_t)id * tile_bytes<R>(L) + zoff_bytes<R>(zb) + (uint32_t)colpos(lx, ly) * 128u;
                R u[8], v0[8];
                bload8(ur, seg, u);
                bload8(u0r, seg, v0);
                TRAF(S, 6, x < L.nx && y < L.ny, 16 * sizeof(R));
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    R dl = v0[i] - u[i];
                    dl = dl < (R)0 ? -dl : dl;
                    if (x < L.nx && y < L.ny && zb * 8 + i < L.nz && u[i] < T && !(dl < tolr)) notconv = true;
                }
            }
            // the iteration is not converged once any node fails: the rest of
            // the scan cannot change the answer (its only output), so stop
            if (__any(notconv)) return;
        }
    }
}

// fp64: two waves per SIMD (the register budget that allows it: 4 B of
// spills outside the step loop, against one wave with AGPR spills)
#define FSM_WPE __attribute__((amdgpu_waves_per_eu(sizeof(R) == 8 ? 2 : 1)))
template <typename R, int SLOWMODE, bool FAST, int ZSH, int CCR, int KB>
__global__ __launch_bounds__(64) FSM_WPE void fsm_solve_kernel(FsmLaunch L)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool CMP = sizeof(R) == 8 && KB > 0;     // fsm_compact_layout() (the host checked it)
    const Smem<R, CMP> S = smem_bind<R, KB == MCEIK_KB && sizeof(R) == 4 && SLOWMODE == 2, CMP>(L, smem);
    const int lane = threadIdx.x;
    const uint32_t fbytes = (uint32_t)(L.field_elems * sizeof(R));
    build_order(L, S.order);
    int pass = 0;
    for (;;) {
        const int snext = next_solve(L, pass);
        if (snext < 0) break;
        const unsigned solve = (unsigned)snext;
        if (L.solve_clock && lane == 0) L.solve_clock[2 * (size_t)solve] = __builtin_amdgcn_s_memrealtime();
        const int model = (int)solve / L.nstat, station = (int)solve - model * L.nstat;
        if (L.skip && L.skip[(L.model_phase && SLOWMODE != 0 ? L.model_phase[model] : fsm_plain_phase(L, model)) *
                                 L.nstat + station]) {
            skip_solve<R>(L, solve);                    // no picks of this phase at this station
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            continue;
        }
        const size_t slot = L.slot_per_solve ? solve : blockIdx.x;
        R *u = reinterpret_cast<R *>(L.u) + slot * L.field_elems;
        R *u0 = reinterpret_cast<R *>(L.u0) + (size_t)blockIdx.x * L.field_elems;   // per-wave scratch
        const void *slow_model;
        uint32_t slow_bytes;
        if (SLOWMODE == 0) {
            slow_model = reinterpret_cast<const R *>(L.slow) + (size_t)model * L.field_elems;
            slow_bytes = fbytes;
        } else {
            const size_t ncell = (size_t)L.ncx * L.ncy * L.ncz;
            slow_model = reinterpret_cast<const float *>(L.slow) + fsm_slow_entry(L, model) * ncell;
            slow_bytes = (uint32_t)(ncell * 4);
        }
        const Rsrc ur = make_rsrc(u, fbytes), u0r = make_rsrc(u0, fbytes), sr = make_rsrc(slow_model, slow_bytes);
        // Clocks before the first sweep: every block "visited" at -2 and
        // unchanged since (-3), except the blocks holding boundary-condition
        // nodes (changed at -1).  Exact: a block whose nodes and neighbours
        // are all u_nan updates to u_nan (a1 == u_nan), so it needs no visit
        // until a neighbour changes.  The stream clock starts at 64, so no
        // initial visit counts as in flight.
        // (compact layout: the held stream, hold_solve_start)
        constexpr bool HOLD = CMP;
        if (!HOLD) {
            for (int t = lane; t < L.nblocks; t += 64) {
                S.lastproc[t] = -2; S.lastchg[t] = -3;
            }
        }
        if (lane == 0) { S.scratch[0] = 0; S.scratch[1] = 0; S.scratch[2] = 0; S.scratch[3] = 0; }
#ifdef MCEIK_TRAFFIC
        if (lane == 0)
            for (int k = 0; k < MCEIK_TRAFFIC_N; k++) S.scratch[8 + k] = 0;
#endif
        unsigned nchg = 0, nsteps = 0;
        BcBoxes bc;
        bc.box = S.box;
        const bool ok = init_field<R, SLOWMODE>(L, u, ur, slow_model, L.src + (size_t)station * L.nsrc * 4, bc);
        if constexpr (HOLD) {
            hold_solve_start(L, hold_lds(S), bc, L.nr);
        } else if (lane == 0) {
            for (int k = 0; k < bc.n; k++) {
                const int *q = bc.box + 6 * k;
                for (int tz = q[4] / (8 * L.kb); tz <= q[5] / (8 * L.kb); tz++)
                    for (int ty = q[2] >> 3; ty <= q[3] >> 3; ty++)
                        for (int tx = q[0] >> 3; tx <= q[1] >> 3; tx++)
                            S.lastchg[(tz * L.nty + ty) * L.ntx + tx] = -1;
            }
        }
        asm volatile("" ::: "memory");
        int iters = 0, ierr_last = 0, clock = 64;
        if (ok) {
            int sweeps_left = L.max_sweeps < 0 ? 0x7fffffff : L.max_sweeps;
            for (int it = 0; it < L.maxit && sweeps_left > 0; it++) {
                bool notconv = false;
                if constexpr (HOLD) {
                    hold_iter_start(L, hold_lds(S));      // (the held stream rebases its clocks every sweep)
                    clock = 64;
                }
                const int clock_it = clock;
                for (int sw = 0; sw < 8 && sweeps_left > 0; sw++, sweeps_left--) {
                    const int rx = sw & 1, ry = (sw >> 1) & 1;
#ifdef MCEIK_STEPSTATS
                    const int clock_sw = clock;
#endif
                    // positions used + a gap of infl: the previous sweep's visits are
                    // never in flight (nor within vis) for the next one
                    if (sw & 4)
                        clock += L.infl + sweep<R, SLOWMODE, FAST, true, ZSH, CCR, KB>(
                                              L, ur, u0r, sr, bc, S, rx, ry, clock_it, clock, notconv, ierr_last, nchg,
                                              nsteps);
                    else
                        clock += L.infl + sweep<R, SLOWMODE, FAST, false, ZSH, CCR, KB>(
                                              L, ur, u0r, sr, bc, S, rx, ry, clock_it, clock, notconv, ierr_last, nchg,
                                              nsteps);
#ifdef MCEIK_STEPSTATS
                    {   // experiment: visited blocks of this sweep that did not change
                        const int c1 = clock - L.infl;
                        unsigned nu = 0;
                        for (int t = lane; t < L.nblocks; t += 64) {
                            const int lp = S.lastproc[t];
                            nu += (lp >= c1 - 0x100000 && lp > 63 && lp >= clock_sw && S.lastchg[t] < lp) ? 1u : 0u;
                        }
                        for (int o = 32; o > 0; o >>= 1) nu += __shfl_xor(nu, o, 64);
                        if (lane == 0) S.scratch[3] += nu;
                    }
#endif
                    __builtin_amdgcn_s_waitcnt(0);      // stores of this sweep land before the next sweep's loads
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    TRAF_FLUSH(L, S);
                }
                iters = it + 1;
                if (sweeps_left > 0 || L.max_sweeps < 0) {
                    if (!__any(notconv)) verify_small<R>(L, ur, u0r, S, clock_it, notconv);
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
#ifdef MCEIK_STEPSTATS
                atomicAdd(L.visit_stats + 1, (unsigned long long)(unsigned)S.scratch[2]);
                atomicAdd(L.visit_stats + 2, (unsigned long long)(unsigned)S.scratch[3]);
#else
                atomicAdd(L.visit_stats + 1, (unsigned long long)(unsigned)S.scratch[1]);
                atomicAdd(L.visit_stats + 2, (unsigned long long)nchg);
                atomicAdd(L.visit_stats + 3, (unsigned long long)nsteps);
#endif
            }
        }
        if (lane == 0) {
            if (L.solve_clock) L.solve_clock[2 * (size_t)solve + 1] = __builtin_amdgcn_s_memrealtime();
            if (L.iter_total) atomicAdd(L.iter_total, (unsigned long long)iters);
            if (L.solve_count) atomicAdd(L.solve_count, 1ull);
            if (L.niter) L.niter[solve] = iters;
            if (L.ierr) L.ierr[solve] = ierr;
        }
        TRAFU(S, 7, (unsigned)(L.field_elems * sizeof(R)) + (L.ttab ? (unsigned)L.nev * (4u + 64u) : 0u));
        TRAF_FLUSH(L, S);
        if (L.ttab) {
            for (int e = lane; e < L.nev; e += 64) L.ttab[(size_t)solve * L.nev + e] = event_time<R>(L, u, e);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
}

// ---- layout conversion (x-fastest <-> brick), drop-in entry points only ----
template <typename RS, typename RD>
__global__ void to_brick_kernel(const RS *src, RD *dst, FsmLaunch L, int nfield)
{
    size_t n = L.field_elems * (size_t)nfield;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        size_t fld = i / L.field_elems, e = i - fld * L.field_elems;
        constexpr int ZQ = Lay<RD>::ZQ;                   // destination layout (brick_index<RD>)
        const int zi = (int)(e % ZQ);
        size_t t = e / ZQ;
        const int col = (int)(t & 63); t >>= 6;
        const int zq = (int)(t % L.nzq); const int tile = (int)(t / L.nzq);
        int ty = tile / L.ntx, tx = tile - ty * L.ntx;
        int clx, cly;
        colpos_inv(col, clx, cly);
        int x = tx * 8 + clx, y = ty * 8 + cly, z = zq * ZQ + zi;
        RD v = 0;
        if (x < L.nx && y < L.ny && z < L.nz)
            v = (RD)src[fld * (size_t)L.nx * L.ny * L.nz + ((size_t)z * L.ny + y) * L.nx + x];
        dst[i] = v;
    }
}

template <typename RS, typename RD>
__global__ void from_brick_kernel(const RS *src, RD *dst, FsmLaunch L, int nfield)
{
    size_t nn = (size_t)L.nx * L.ny * L.nz, n = nn * nfield;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        size_t fld = i / nn, e = i - fld * nn;
        int x = (int)(e % L.nx); size_t t = e / L.nx;
        int y = (int)(t % L.ny); int z = (int)(t / L.ny);
        dst[i] = (RD)src[fld * L.field_elems + brick_index<RS>(L, x, y, z)];
    }
}

}  // namespace

// ---- host-side launchers (C++ linkage, used by capi.hip) ---------------------
template <typename R, int SLOWMODE, bool FAST, int ZSH, int CCR, int KB>
static hipError_t launch_fsm(const FsmLaunch &L, int nwaves, hipStream_t st)
{
    size_t lds = fsm_lds_bytes(L, sizeof(R));
    if (KB == MCEIK_KB && sizeof(R) == 4 && SLOWMODE == 2 && !fsm_fixed_layout(L, 4)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fsm_solve_kernel<R, SLOWMODE, FAST, ZSH, CCR, KB>), dim3(nwaves), dim3(64), lds, st, L);
    return hipGetLastError();
}

template <typename R, int SLOWMODE, bool FAST, int ZSH, int CCR, int KB>
static int occupancy_of(size_t lds)
{
    int nb = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_solve_kernel<R, SLOWMODE, FAST, ZSH, CCR, KB>, 64,
                                                        lds) == hipSuccess ? nb : 1;
}

// Kernel variant of a launch: slowness source, sqrt form, and (cell cache)
// whether the z refinement is 4 (cell offsets of a brick's slots are
// constants) with at most 64 cells per z-block (one cell register per lane).
static int variant(const FsmLaunch &L, int is_double)
{
    const int mode = L.slow_mode == 0 ? 0 : (L.cell_cache ? 2 : 1);
    if (is_double) {
        // compile-time kb (15, 16) iff the compact LDS layout applies (nblocks <= MCEIK_MAX_BLOCKS)
        const int v = 9 + mode * 2 + (mode == 2 && L.nrz == 4 && L.ccb <= 64 ? (fsm_compact_layout(L, 8) ? 2 : 1) : 0);
        return v == 15 && L.fast_sqrt ? 16 : v;      // the fp64 sampler instance with the short sqrt
    }
    if (mode != 2) return mode * 2;
    return 4 + (L.fast_sqrt ? 1 : 0) + (L.nrz == 4 && L.fast_sqrt && L.ccb <= 64 ? (L.kb == MCEIK_KB ? 3 : 2) : 0);
}

#define FSM_VARIANTS(X)                         \
    X(0, float, 0, false, -1, 1, 0)             \
    X(2, float, 1, false, -1, 1, 0)             \
    X(4, float, 2, false, -1, 4, 0)             \
    X(5, float, 2, true, -1, 4, 0)              \
    X(7, float, 2, true, 2, 1, 0)               \
    X(8, float, 2, true, 2, 1, MCEIK_KB)        \
    X(9, double, 0, false, -1, 1, 0)            \
    X(11, double, 1, false, -1, 1, 0)           \
    X(13, double, 2, false, -1, 4, 0)           \
    X(14, double, 2, false, 2, 1, 0)            \
    X(15, double, 2, false, 2, 1, MCEIK_KB)     \
    X(16, double, 2, true, 2, 1, MCEIK_KB)

// the 16-z-step kernel (fsm16_kernel.hip) serves the fp32 cell-cache
// instances (variants 7, 8) when fsm16_eligible(); MCEIK_FSM16=0 keeps the
// 8-z kernel (A/B measurements)
hipError_t fsm16_launch(const FsmLaunch &L, int nwaves, hipStream_t st);
int fsm16_occupancy(const FsmLaunch &L);
static bool use_fsm16(const FsmLaunch &L, int is_double)
{
    static const bool on = [] { const char *e = getenv("MCEIK_FSM16"); return !(e && e[0] == '0'); }();
    const int v = variant(L, is_double);
    return on && L.step_z != 8 && (v == 5 || v == 7 || v == 8) && fsm16_eligible(L, 4);
}
size_t fsm_launch_lds_bytes(const FsmLaunch &L, int is_double)
{
    return use_fsm16(L, is_double) ? fsm16_lds_bytes(L) : fsm_lds_bytes(L, is_double ? 8 : 4);
}
int fsm_launch_kind(const FsmLaunch &L, int is_double) { return use_fsm16(L, is_double) ? 16 : 8; }
// The kernel instance a launch runs (names as in the rocprof traces).
const char *fsm_launch_name(const FsmLaunch &L, int is_double)
{
    if (use_fsm16(L, is_double))
        return fsm16_fixed_layout(L) ? "fsm16_solve_kernel<2, 1>" : L.ccb <= 64 ? "fsm16_solve_kernel<0, 1>"
                                                                                 : "fsm16_solve_kernel<0, 4>";
    switch (variant(L, is_double)) {
    case 0: return "fsm_solve_kernel<float, 0, false, -1, 1, 0>";
    case 2: return "fsm_solve_kernel<float, 1, false, -1, 1, 0>";
    case 4: return "fsm_solve_kernel<float, 2, false, -1, 4, 0>";
    case 5: return "fsm_solve_kernel<float, 2, true, -1, 4, 0>";
    case 7: return "fsm_solve_kernel<float, 2, true, 2, 1, 0>";
    case 8: return "fsm_solve_kernel<float, 2, true, 2, 1, 4>";
    case 9: return "fsm_solve_kernel<double, 0, false, -1, 1, 0>";
    case 11: return "fsm_solve_kernel<double, 1, false, -1, 1, 0>";
    case 13: return "fsm_solve_kernel<double, 2, false, -1, 4, 0>";
    case 14: return "fsm_solve_kernel<double, 2, false, 2, 1, 0>";
    case 15: return "fsm_solve_kernel<double, 2, false, 2, 1, 4>";
    case 16: return "fsm_solve_kernel<double, 2, true, 2, 1, 4>";
    }
    return "?";
}

// Zeroes the launch's work-queue heads with a kernel rather than
// hipMemsetAsync: inside a captured HIP graph the memset node was not replayed
// (ROCm 7.2; every replay after the first found the queues drained and ran no
// solve, tests/test_gpu_fsm.py::test_batch_solve_captured_in_a_graph_bitwise).
__global__ void fsm_zero_words_kernel(unsigned *p, int n)
{
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0u;
}
hipError_t fsm_zero_words(unsigned *p, int n, hipStream_t st)
{
    hipLaunchKernelGGL(fsm_zero_words_kernel, dim3(1), dim3(256), 0, st, p, n);
    return hipGetLastError();
}

hipError_t fsm_launch(const FsmLaunch &L, int is_double, int nwaves, hipStream_t st)
{
    if (use_fsm16(L, is_double)) return fsm16_launch(L, nwaves, st);
    switch (variant(L, is_double)) {
#define X(v, R, M, F, Z, CR, K) case v: return launch_fsm<R, M, F, Z, CR, K>(L, nwaves, st);
        FSM_VARIANTS(X)
#undef X
    default: return hipErrorInvalidValue;
    }
}

int fsm_occupancy(const FsmLaunch &L, int is_double)
{
    if (use_fsm16(L, is_double)) return fsm16_occupancy(L);
    const size_t lds = fsm_lds_bytes(L, is_double ? 8 : 4);
    switch (variant(L, is_double)) {
#define X(v, R, M, F, Z, CR, K) case v: return occupancy_of<R, M, F, Z, CR, K>(lds);
        FSM_VARIANTS(X)
#undef X
    default: return 1;
    }
}

hipError_t fsm_to_brick_f64(const double *src, void *dst, int dst_double, const FsmLaunch &L, int nfield, hipStream_t st)
{
    if (dst_double) hipLaunchKernelGGL((to_brick_kernel<double, double>), dim3(1024), dim3(256), 0, st, src, (double *)dst, L, nfield);
    else hipLaunchKernelGGL((to_brick_kernel<double, float>), dim3(1024), dim3(256), 0, st, src, (float *)dst, L, nfield);
    return hipGetLastError();
}

hipError_t fsm_from_brick_f64(const void *src, int src_double, double *dst, const FsmLaunch &L, int nfield, hipStream_t st)
{
    if (src_double) hipLaunchKernelGGL((from_brick_kernel<double, double>), dim3(1024), dim3(256), 0, st, (const double *)src, dst, L, nfield);
    else hipLaunchKernelGGL((from_brick_kernel<float, double>), dim3(1024), dim3(256), 0, st, (const float *)src, dst, L, nfield);
    return hipGetLastError();
}

hipError_t fsm_from_brick_f32(const float *src, float *dst, const FsmLaunch &L, int nfield, hipStream_t st)
{
    hipLaunchKernelGGL((from_brick_kernel<float, float>), dim3(1024), dim3(256), 0, st, src, dst, L, nfield);
    return hipGetLastError();
}

hipError_t fsm_to_brick_f32(const float *src, float *dst, const FsmLaunch &L, int nfield, hipStream_t st)
{
    hipLaunchKernelGGL((to_brick_kernel<float, float>), dim3(1024), dim3(256), 0, st, src, dst, L, nfield);
    return hipGetLastError();
}
