// fsm_hold.h -- the held z-block stream of the batched sweep kernels
// (fsm16_kernel.hip, and fsm_kernel.hip's compact-layout fp64 instances;
// DESIGN.md s.3.8).
//
// EVAL_UPDATE3D (fsm3d.f90:419-456) sweeps every node of the grid in every
// direction.  The kernels visit only the z-blocks (8x8 column tile x kb
// bricks) whose inputs changed; skipping the others is exact because a node's
// update is a pure function of itself, its six neighbours and its slowness,
// and only lowers it.  The held stream decides which blocks those are:
//
// The z-blocks of a sweep are decided tile by tile in diagonal order, but a
// tile's blocks one at a time (frontier fz, sweep z order), and a block only
// once the blocks it reads new values from are decided: its sweep-upwind x and
// y neighbours (the upwind tiles' frontiers are past it) and its z-below (the
// frontier).  Then, with 16-bit clocks relative to the sweep:
//   need >= lastproc (it changed at its last visit, or a neighbour changed
//     the face layer it shares with it since: settled marks)  -> visit, once
//     its upwind visits are >= vis positions back (a z-below visited at the
//     previous position continues the run in registers);
//   else an upwind neighbour or the z-below still in flight   -> wait (held);
//   else                                                      -> skip.
// The earlier stream visited every block whose upwind neighbour was still in
// flight and ran every tile to its column end; those visits almost never
// changed anything (profiles/r05_admit/bench_admit_stats.log).
// A visit's changes are "settled" infl positions after it (every lane is past
// it): the change mask its lanes collected (fmask) then marks need of the
// block itself and of the neighbours across the faces it changed.
#pragma once
#include <hip/hip_runtime.h>

#include "fsm_common.h"
#include "fsm_device.h"

// the per-position change mask (fmask): bit 0 the block changed, bits 1-6 the
// face layer it changed (x-low, x-high, y-low, y-high, z-low, z-high; absolute
// orientation), and HOLD_CONT: the next position continues this position's
// z-run (same tile, next block in sweep z order)
#define HOLD_OWN 1u
#define HOLD_ZLO 32u
#define HOLD_ZHI 64u
#define HOLD_CONT 256u

namespace {

// The stream's LDS arrays (OrderT: u16 order entries txs | tys << 8, or int
// entries txs | tys << 16)
template <typename OrderT>
struct HoldLds {
    const OrderT *order;         // diagonal tile order of the (+x, +y) sweep
    unsigned char *fz;           // per tile: z-blocks decided in this sweep (sweep z order)
    unsigned short *lastproc;    // per block: clock of its last visit (sweep-relative)
    unsigned short *need;        // per block: clock of the last settled change of it or of a shared face
    unsigned *fmask;             // per ring slot: what the position's visit changed | HOLD_CONT
    const int *ring_e;           // per ring slot: entry tx | ty << 12 | tz << 24, bubble -1
    unsigned *vbits, *cbits;     // blocks visited / changed in this iteration (bitmaps)
};
// scan state (int [2] in LDS): [0] tiles [0, done) of the diagonal order are
// complete, [1] diagonal index of the previous position's tile, -1 none
enum { HOLD_DONE = 0, HOLD_BLOCKED, HOLD_HELD, HOLD_WAIT, HOLD_SKIP, HOLD_READY };

template <typename OrderT>
__device__ __forceinline__ void hold_txy(const HoldLds<OrderT> &H, int ti, int &txs, int &tys)
{
    constexpr int SH = 4 * (int)sizeof(OrderT);
    const int o = (int)H.order[ti];
    txs = o & ((1 << SH) - 1);
    tys = o >> SH;
}
// The next undecided block (sweep-z index k) of tile id at clock C, its upwind
// x / y tiles xu / yu (-1: none): HOLD_DONE (k >= nzk) / BLOCKED (an upwind
// tile has not decided that far) / HELD / WAIT (a reason, but an upwind visit
// is < vis back) / SKIP / READY; runon: its z-below is the previous position.
// Every read is issued up front (absent neighbours and a DONE tile read the
// tile's own entries, unused): one LDS round trip per call.  u0: the block
// has not been visited in this iteration (the admission's u0 flag).
template <bool RZ, typename OrderT>
__device__ __forceinline__ int hold_status(const FsmLaunch &L, const HoldLds<OrderT> &H, int id, int xu, int yu, int k,
                                           int C, int infl, int vis, int &runon, int &u0)
{
    const int nt = L.ntiles, nzk = L.nzk;
    const int kc = min(k, nzk - 1);
    const int tz = RZ ? nzk - 1 - kc : kc;
    const int b = tz * nt + id;
    int fxu = H.fz[xu >= 0 ? xu : id], fyu = H.fz[yu >= 0 ? yu : id];
    int nb = H.need[b], lb = H.lastproc[b];
    int lxu = H.lastproc[tz * nt + (xu >= 0 ? xu : id)], lyu = H.lastproc[tz * nt + (yu >= 0 ? yu : id)];
    int lzl = H.lastproc[kc > 0 ? b + (RZ ? nt : -nt) : b];
    unsigned vw = H.vbits[b >> 5];
    asm volatile("" : "+v"(fxu), "+v"(fyu), "+v"(nb), "+v"(lb), "+v"(lxu), "+v"(lyu), "+v"(lzl), "+v"(vw));
    u0 = !((vw >> (b & 31)) & 1u);                       // no visit of the block in this iteration yet
    runon = 0;
    if (k >= nzk) return HOLD_DONE;
    if ((xu >= 0 && fxu <= k) || (yu >= 0 && fyu <= k)) return HOLD_BLOCKED;
    const bool reason = nb >= lb;
    int dep = -0x40000000;                               // latest upwind visit (this sweep's clocks)
    if (xu >= 0) dep = max(dep, lxu);
    if (yu >= 0) dep = max(dep, lyu);
    const int zl = k > 0 ? lzl : -0x40000000;
    runon = zl == C - 1;
    if (!runon) dep = max(dep, zl);
    if (reason) return dep + vis <= C ? HOLD_READY : HOLD_WAIT;
    return (runon || dep > C - infl) ? HOLD_HELD : HOLD_SKIP;
}
// The scan state a decision starts from (LDS sst[0..2]): [0] tiles [0, done)
// of the diagonal order are complete, [1] diagonal index of the previous
// position's tile (-1 none), [2] that tile's id | its next sweep-z index << 16
// | upwind x / y tile flags << 24.  Read before the same decision's settle, so
// the two round trips overlap (values per lane; hold_decide makes them scalar).
struct HoldSt {
    int done, last, lc;
};
__device__ __forceinline__ HoldSt hold_state(const int *sst)
{
    asm volatile("" ::: "memory");
    return HoldSt{sst[0], sst[1], sst[2]};
}
// The block of position C (the previous position's ring slot rprev): the next
// block of the previous position's tile when it is ready, else the first ready
// block in diagonal order -- windows of 64 tiles from the first incomplete one,
// every lane deciding its tile's next block per round, until a block is ready
// or no lane can skip.  Returns the entry tx | ty << 12 | tz << 24, -1 (a
// bubble) or -2 (every tile decided: the sweep's stream ends); zh: a run start
// above the column's first block (its z-upwind node comes from HBM).
// Progress: the first incomplete tile's upwind tiles are complete, so within
// infl positions its next block is ready or skipped.
// Round trips: the previous tile's status from the cached state (one); the
// front scan (tile order, frontiers: two), whose window the first round reuses
// when the front did not move; one per round (a lane's own frontier is
// tracked in registers: only its lane advances it within a window).
template <bool RZ, typename OrderT>
__device__ __forceinline__ int hold_decide(const FsmLaunch &L, const HoldLds<OrderT> &H, int *sst, const HoldSt &sr,
                                           int C, int rx, int ry, int rprev, int infl, int vis, int &zh, int &u0)
{
    const int lane = threadIdx.x, nt = L.ntiles, nzk = L.nzk;
    const int dxu = rx ? 1 : -1, dyu = ry ? L.ntx : -L.ntx;
    zh = 0;
    u0 = 0;
    int pick = -1, pid = 0, pk = 0, pro = 0, pfl = 0, pu0 = 0;
    int done = __builtin_amdgcn_readfirstlane(sr.done);
    const int last = __builtin_amdgcn_readfirstlane(sr.last), lc = __builtin_amdgcn_readfirstlane(sr.lc);
    if (last >= 0) {
        const int id = lc & 0xffff, k = (lc >> 16) & 0xff, fl = (lc >> 24) & 3;
        int ro, v0;
        const int s = hold_status<RZ>(L, H, id, (fl & 1) ? id + dxu : -1, (fl & 2) ? id + dyu : -1, k, C, infl, vis,
                                      ro, v0);
        if (__builtin_amdgcn_readfirstlane(s) == HOLD_READY) {
            pick = last;
            pid = id;
            pk = k;
            pro = __builtin_amdgcn_readfirstlane(ro);
            pu0 = __builtin_amdgcn_readfirstlane(v0);
            pfl = fl;
        }
    }
    if (pick < 0) {
        // this lane's tile of the window at wbase: id, upwind tiles, frontier (255: none)
        int wbase = -1, ti = 0, id = 0, xu = -1, yu = -1, k = 255;
        auto window = [&](int base) __attribute__((always_inline)) {
            wbase = base;
            ti = base + lane;
            const bool in = ti < nt;
            int txs, tys;
            hold_txy(H, in ? ti : 0, txs, tys);
            const int tx = rx ? L.ntx - 1 - txs : txs, ty = ry ? L.nty - 1 - tys : tys;
            id = ty * L.ntx + tx;
            xu = txs > 0 ? id + dxu : -1;
            yu = tys > 0 ? id + dyu : -1;
            const int f = H.fz[id];
            k = in ? f : 255;
        };
        for (;;) {                                   // the complete tiles at the front
            window(done);
            const unsigned long long m = ~__ballot(ti < nt && k >= nzk);
            const int n = m ? __builtin_ctzll(m) : 64;
            done += n;
            if (n < 64) break;
        }
        if (done >= nt) {
            asm volatile("" ::: "memory");
            if (lane == 0) { sst[0] = done; sst[1] = -1; }
            asm volatile("" ::: "memory");
            return -2;
        }
        for (int base = done; base < nt && pick < 0; base += 64) {
            if (base != wbase) window(base);
            for (;;) {
#ifdef MCEIK_PHASECLK
                if (lane == 0) sst[4 + 7] += 1;           // traffic category 7: window rounds
#endif
                int ro, v0;
                const int s0 = hold_status<RZ>(L, H, id, xu, yu, k, C, infl, vis, ro, v0);
                const int s = ti < nt ? s0 : HOLD_DONE;
                const bool sk = s == HOLD_SKIP;
                if (sk) H.fz[id] = (unsigned char)(k + 1);
                const unsigned long long rm = __ballot(s == HOLD_READY);
                if (rm) {
                    const int f = __builtin_ctzll(rm);
                    pick = base + f;
                    pid = __builtin_amdgcn_readfirstlane(__shfl(id, f, 64));
                    pk = __builtin_amdgcn_readfirstlane(__shfl(k, f, 64));
                    pro = __builtin_amdgcn_readfirstlane(__shfl(ro, f, 64));
                    pu0 = __builtin_amdgcn_readfirstlane(__shfl(v0, f, 64));
                    pfl = __builtin_amdgcn_readfirstlane(__shfl((xu >= 0 ? 1 : 0) | (yu >= 0 ? 2 : 0), f, 64));
                    break;
                }
                if (!__ballot(sk)) break;
                k += sk ? 1 : 0;
                asm volatile("" ::: "memory");       // this round's frontiers feed the next
            }
        }
    }
    asm volatile("" ::: "memory");
    if (pick < 0) {
        if (lane == 0) { sst[0] = done; sst[1] = -1; }
        asm volatile("" ::: "memory");
        return -1;
    }
    if (lane == 0) {
        H.fz[pid] = (unsigned char)(pk + 1);
        if (pro) atomicOr(&H.fmask[rprev], HOLD_CONT);   // the previous position's run continues here
        sst[0] = done;
        sst[1] = pick;
        sst[2] = pid | ((pk + 1) << 16) | (pfl << 24);
    }
    asm volatile("" ::: "memory");
    zh = pk > 0 && !pro;
    u0 = pu0;
    const int ty = pid / L.ntx, tx = pid - ty * L.ntx;
    return tx | (ty << 12) | ((RZ ? L.nzk - 1 - pk : pk) << 24);
}
template <typename OrderT>
__device__ __forceinline__ int hold_tile_id(const FsmLaunch &L, const HoldLds<OrderT> &H, int ti, int rx, int ry)
{
    int txs, tys;
    hold_txy(H, ti, txs, tys);
    return (ry ? L.nty - 1 - tys : tys) * L.ntx + (rx ? L.ntx - 1 - txs : txs);
}
// ---- the decision as the fp64 instances make it (fsm_kernel.hip) ----------
// Same decisions as hold_decide below, with the tile geometry read from the
// order table on every call and no cached state (four LDS round trips for the
// previous tile's status, two for the front scan, three per window round).
// The fp64 kernel keeps this form: the round-trip-lean one moved its register
// allocation and measured 0.7% slower there (profiles/r06_hd).
// The next undecided block of the tile at diagonal index ti at clock C:
// HOLD_DONE / BLOCKED (an upwind tile has not decided that far) / HELD / WAIT
// (a reason, but an upwind visit is < vis back) / SKIP / READY; id, k: the
// tile and the block's sweep-z index, runon: its z-below is the previous position.
template <bool RZ, typename OrderT>
__device__ __forceinline__ int hold_status_scan(const FsmLaunch &L, const HoldLds<OrderT> &H, int ti, int C, int rx, int ry,
                                           int infl, int vis, int &id, int &k, int &runon)
{
    int txs, tys;
    hold_txy(H, ti, txs, tys);
    const int tx = rx ? L.ntx - 1 - txs : txs, ty = ry ? L.nty - 1 - tys : tys;
    const int nt = L.ntiles, nzk = L.nzk;
    id = ty * L.ntx + tx;
    k = H.fz[id];
    runon = 0;
    if (k >= nzk) return HOLD_DONE;
    const int xu = txs > 0 ? id + (rx ? 1 : -1) : -1;
    const int yu = tys > 0 ? id + (ry ? L.ntx : -L.ntx) : -1;
    if ((xu >= 0 && (int)H.fz[xu] <= k) || (yu >= 0 && (int)H.fz[yu] <= k)) return HOLD_BLOCKED;
    const int tz = RZ ? nzk - 1 - k : k;
    const int b = tz * nt + id;
    const bool reason = H.need[b] >= H.lastproc[b];
    int dep = -0x40000000;                               // latest upwind visit (this sweep's clocks)
    if (xu >= 0) dep = max(dep, (int)H.lastproc[tz * nt + xu]);
    if (yu >= 0) dep = max(dep, (int)H.lastproc[tz * nt + yu]);
    const int zl = k > 0 ? (int)H.lastproc[b + (RZ ? nt : -nt)] : -0x40000000;
    runon = zl == C - 1;
    if (!runon) dep = max(dep, zl);
    if (reason) return dep + vis <= C ? HOLD_READY : HOLD_WAIT;
    return (runon || dep > C - infl) ? HOLD_HELD : HOLD_SKIP;
}
// The block of position C (the previous position's ring slot rprev): the next
// block of the previous position's tile when it is ready, else the first ready
// block in diagonal order -- windows of 64 tiles from the first incomplete one,
// every lane deciding its tile's next block per round, until a block is ready
// or no lane can skip.  Returns the entry tx | ty << 12 | tz << 24, -1 (a
// bubble) or -2 (every tile decided: the sweep's stream ends); zh: a run start
// above the column's first block (its z-upwind node comes from HBM).
// Progress: the first incomplete tile's upwind tiles are complete, so within
// infl positions its next block is ready or skipped.
template <bool RZ, typename OrderT>
__device__ __forceinline__ int hold_decide_scan(const FsmLaunch &L, const HoldLds<OrderT> &H, int *sst, int C, int rx,
                                           int ry, int rprev, int infl, int vis, int &zh)
{
    const int lane = threadIdx.x, nt = L.ntiles;
    zh = 0;
    int pick = -1, pid = 0, pk = 0, pro = 0;
    asm volatile("" ::: "memory");
    struct { int done, last; } st = {__builtin_amdgcn_readfirstlane(sst[0]), __builtin_amdgcn_readfirstlane(sst[1])};
    if (st.last >= 0) {
        int id, k, ro;
        const int s = hold_status_scan<RZ>(L, H, st.last, C, rx, ry, infl, vis, id, k, ro);
        if (__builtin_amdgcn_readfirstlane(s) == HOLD_READY) {
            pick = st.last;
            pid = __builtin_amdgcn_readfirstlane(id);
            pk = __builtin_amdgcn_readfirstlane(k);
            pro = __builtin_amdgcn_readfirstlane(ro);
        }
    }
    if (pick < 0) {
        for (;;) {                                   // the complete tiles at the front
            const int ti = st.done + lane;
            const bool cpl = ti < nt && (int)H.fz[hold_tile_id(L, H, ti, rx, ry)] >= L.nzk;
            const unsigned long long m = ~__ballot(cpl);
            const int n = m ? __builtin_ctzll(m) : 64;
            st.done += n;
            if (n < 64) break;
        }
        if (st.done >= nt) {
            asm volatile("" ::: "memory");
            if (lane == 0) { sst[0] = st.done; sst[1] = -1; }
            asm volatile("" ::: "memory");
            return -2;
        }
        for (int base = st.done; base < nt && pick < 0; base += 64) {
            const int ti = base + lane;
            for (;;) {
                int s = HOLD_DONE, id = 0, k = 0, ro = 0;
                if (ti < nt) s = hold_status_scan<RZ>(L, H, ti, C, rx, ry, infl, vis, id, k, ro);
                const bool sk = s == HOLD_SKIP;
                if (sk) H.fz[id] = (unsigned char)(k + 1);
                const unsigned long long rm = __ballot(s == HOLD_READY);
                if (rm) {
                    const int f = __builtin_ctzll(rm);
                    pick = base + f;
                    pid = __builtin_amdgcn_readfirstlane(__shfl(id, f, 64));
                    pk = __builtin_amdgcn_readfirstlane(__shfl(k, f, 64));
                    pro = __builtin_amdgcn_readfirstlane(__shfl(ro, f, 64));
                    break;
                }
                if (!__ballot(sk)) break;
                asm volatile("" ::: "memory");       // this round's frontiers feed the next
            }
        }
    }
    asm volatile("" ::: "memory");
    if (pick < 0) {
        if (lane == 0) { sst[0] = st.done; sst[1] = -1; }
        asm volatile("" ::: "memory");
        return -1;
    }
    if (lane == 0) {
        H.fz[pid] = (unsigned char)(pk + 1);
        if (pro) atomicOr(&H.fmask[rprev], HOLD_CONT);   // the previous position's run continues here
        sst[0] = st.done;
        sst[1] = pick;
    }
    asm volatile("" ::: "memory");
    zh = pk > 0 && !pro;
    const int ty = pid / L.ntx, tx = pid - ty * L.ntx;
    return tx | (ty << 12) | ((RZ ? L.nzk - 1 - pk : pk) << 24);
}
// Settle the visit of ring slot ri (clock clk): its change mask marks need of
// the block (and the iteration's changed bitmap) and of the neighbours across
// the changed faces; lanes 0-6 take one target each.
template <typename OrderT>
__device__ __forceinline__ void hold_settle(const FsmLaunch &L, const HoldLds<OrderT> &H, int ri, int clk)
{
    const int lane = threadIdx.x;
    asm volatile("" ::: "memory");
    const int e = H.ring_e[ri];
    const unsigned m = H.fmask[ri];
    if (e >= 0 && lane < 7 && ((m >> lane) & 1u)) {
        const int tx = e & 0xfff, ty = (e >> 12) & 0xfff, tz = (e >> 24) & 0xff;
        const int nt = L.ntiles, b = tz * nt + ty * L.ntx + tx;
        const int t = lane == 0 ? b
                    : lane == 1 ? (tx > 0 ? b - 1 : -1)
                    : lane == 2 ? (tx < L.ntx - 1 ? b + 1 : -1)
                    : lane == 3 ? (ty > 0 ? b - L.ntx : -1)
                    : lane == 4 ? (ty < L.nty - 1 ? b + L.ntx : -1)
                    : lane == 5 ? (tz > 0 ? b - nt : -1)
                    : (tz < L.nzk - 1 ? b + nt : -1);
        if (t >= 0) H.need[t] = (unsigned short)clk;
        if (lane == 0) H.cbits[b >> 5] |= 1u << (b & 31);
    }
    asm volatile("" ::: "memory");
    if (lane == 0) H.fmask[ri] = 0;
    asm volatile("" ::: "memory");
}
// Start of a sweep: every block's pending state (need >= lastproc) becomes
// need 1 / 0 against lastproc 1, the frontiers restart, and the sweep's clock
// starts at 64 (a sweep needs at most nblocks (1 + infl) + 64 < 2^16 clocks:
// between two visits at most infl bubbles; fsm_common.h hold_clock_bound).
template <typename OrderT>
__device__ __forceinline__ void hold_norm(const FsmLaunch &L, const HoldLds<OrderT> &H)
{
    asm volatile("" ::: "memory");
    for (int b = threadIdx.x; b < L.nblocks; b += 64) {
        const bool pend = H.need[b] >= H.lastproc[b];
        H.lastproc[b] = 1;
        H.need[b] = pend ? 1 : 0;
    }
    for (int t = threadIdx.x; t < L.ntiles; t += 64) H.fz[t] = 0;
    asm volatile("" ::: "memory");
}
// Start of an iteration: no block visited or changed yet.
template <typename OrderT>
__device__ __forceinline__ void hold_iter_start(const FsmLaunch &L, const HoldLds<OrderT> &H)
{
    for (int w = threadIdx.x; w < (L.nblocks + 31) / 32; w += 64) {
        H.vbits[w] = 0;
        H.cbits[w] = 0;
    }
    asm volatile("" ::: "memory");
}
// Start of a solve (before the first sweep): every block visited at 2 and
// not pending (need 1), except the blocks holding boundary-condition nodes
// and their face neighbours (need 3): a block whose nodes and neighbours are
// all u_nan updates to u_nan.  Lane 0 marks the boxes' blocks.
template <typename OrderT>
__device__ __forceinline__ void hold_solve_start(const FsmLaunch &L, const HoldLds<OrderT> &H, const BcBoxes &bc, int nr)
{
    const int lane = threadIdx.x;
    for (int t = lane; t < L.nblocks; t += 64) {
        H.lastproc[t] = 2;
        H.need[t] = 1;
    }
    if (lane < nr) H.fmask[lane] = 0;
    asm volatile("" ::: "memory");
    if (lane == 0) {
        for (int k = 0; k < bc.n; k++) {
            const int *q = bc.box + 6 * k;
            for (int tz = q[4] / (8 * L.kb); tz <= q[5] / (8 * L.kb); tz++)
                for (int ty = q[2] >> 3; ty <= q[3] >> 3; ty++)
                    for (int tx = q[0] >> 3; tx <= q[1] >> 3; tx++) {
                        const int b = (tz * L.nty + ty) * L.ntx + tx;
                        H.need[b] = 3;
                        if (tx > 0) H.need[b - 1] = 3;
                        if (tx < L.ntx - 1) H.need[b + 1] = 3;
                        if (ty > 0) H.need[b - L.ntx] = 3;
                        if (ty < L.nty - 1) H.need[b + L.ntx] = 3;
                        if (tz > 0) H.need[b - L.ntiles] = 3;
                        if (tz < L.nzk - 1) H.need[b + L.ntiles] = 3;
                    }
        }
    }
    asm volatile("" ::: "memory");
}

// ---- z-face copies (FsmLaunch.zf) -----------------------------------------
// A run that starts above a column's first block reads its z-upwind node, and
// one that ends below the column's last block its z-downwind node, across a
// z-block boundary.  Read from the field those are one value per 128-B line
// of 64 columns; the held stream starts and ends runs at about half its
// positions, so the kernels keep a copy of every block's lowest and highest
// node per column (zf, [nblocks][2][64] R, columns lx + 8 ly), rewritten with
// the field whenever such a node changes, and read 64 columns from 256 B.
// Offset of block b's side (0: lowest node, 1: highest) of column (lx, ly).
template <typename R>
__device__ __forceinline__ uint32_t zf_off(int b, int side, int lx, int ly)
{
    return ((uint32_t)(b * 2 + side) * 64u + (uint32_t)(lx + 8 * ly)) * (uint32_t)sizeof(R);
}
// The z-boundary node a brick of block b reads in sweep direction RZ: the
// z-upwind node of a run start (the z-below block's facing side), or the
// z-downwind node of a run end (zd: the z-above block's facing side).
template <typename R, bool RZ>
__device__ __forceinline__ uint32_t zf_boundary(const FsmLaunch &L, int b, bool zd, int lx, int ly)
{
    // sweep z ascending: below = tz - 1 (its highest node), above = tz + 1 (its lowest)
    const bool up = zd != RZ;                               // the neighbour is at tz + 1
    return zf_off<R>(b + (up ? L.ntiles : -L.ntiles), up ? 0 : 1, lx, ly);
}
// Start of a solve (after init_field, whose stores have completed): every
// copy is u_nan except the boundary-condition nodes on a block's lowest or
// highest layer, copied from the field (lanes 0-26: the 3 x 3 x 3 candidate
// nodes of each source box).
template <typename R>
__device__ __forceinline__ void zf_init(const FsmLaunch &L, Rsrc zfr, const R *u, const BcBoxes &bc)
{
    const int lane = threadIdx.x;
    const R UN = Num<R>::unan();
    R fill[8];
#pragma unroll
    for (int i = 0; i < 8; i++) fill[i] = UN;
    const uint32_t nvec = (uint32_t)(zf_bytes(L, sizeof(R)) / (8 * sizeof(R)));
    for (uint32_t i = lane; i < nvec; i += 64) bstore8(zfr, i * 8u * (uint32_t)sizeof(R), fill);
    __builtin_amdgcn_s_waitcnt(0);
    const int zbk = 8 * L.kb;                                  // z per block
    for (int s = 0; s < bc.n; s++) {
        const int *q = bc.box + 6 * s;
        const int x = q[0] + lane % 3, y = q[2] + (lane / 3) % 3, z = q[4] + lane / 9;
        if (lane < 27 && x <= q[1] && y <= q[3] && z <= q[5]) {
            const int zr = z % zbk;
            if (zr == 0 || zr == zbk - 1) {
                const int b = ((z / zbk) * L.nty + (y >> 3)) * L.ntx + (x >> 3);
                bstore1(zfr, zf_off<R>(b, zr == 0 ? 0 : 1, x & 7, y & 7), u[brick_index<R>(L, x, y, z)]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

}  // namespace
