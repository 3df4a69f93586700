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

#include "fsm_common.h"

namespace {

template <typename R> struct Num;
template <> struct Num<float> {
    static __device__ __forceinline__ float unan() { return FLT_MAX; }
    static __device__ __forceinline__ float sqrt_(float x) { return __builtin_sqrtf(x); }
};
template <> struct Num<double> {
    static __device__ __forceinline__ double unan() { return DBL_MAX; }
    static __device__ __forceinline__ double sqrt_(double x) { return __builtin_sqrt(x); }
};

// ---- the Godunov local solve ------------------------------------------------
// fp32: cancellation-free form (increments relative to a1), bitwise equal to
// oracle/fsm_impl.inc STABLE_UPDATE.  fp64: the reference's literal
// SOLVE_HAMILTONIAN2D/3D (fsm3d.f90:624-693).
__device__ __forceinline__ float godunov(float a, float b, float c, float f, int &ierr)
{
    const float UN = FLT_MAX;
    float lo = a < b ? a : b, hi = a < b ? b : a;
    float a1 = lo < c ? lo : c;
    float a3 = hi < c ? c : hi;
    float a2 = lo < c ? (hi < c ? hi : c) : lo;
    ierr = 0;
    if (a1 == UN) return UN;
    float d2 = a2 - a1, d3 = a3 - a1, y;
    if (!(f > d2)) {
        y = f;
    } else {
        y = 0.5f * (d2 + __builtin_sqrtf((2.0f * f) * f - d2 * d2));
        if (y > d3) {
            float sm = d2 + d3;
            float q = ((d2 * d2) + (d3 * d3)) - f * f;
            float disc = sm * sm - 3.0f * q;
            if (disc < 0.0f) ierr = 1;
            y = (sm + __builtin_sqrtf(disc)) * (1.0f / 3.0f);
        }
    }
    float x = a1 + y;
    if (x < UN) return x;
    ierr = 3;
    return UN;
}

__device__ __forceinline__ double godunov(double a, double b, double c, double f, int &ierr)
{
    const double UN = DBL_MAX;
    double a1, a2, a3;
    bool lab = !(a > b), lac = !(a > c), lbc = !(b > c);
    if (lab && lac) { a1 = a; a2 = lbc ? b : c; a3 = lbc ? c : b; }
    else if (!lab && lbc) { a1 = b; a2 = lac ? a : c; a3 = lac ? c : a; }
    else { a1 = c; a2 = lab ? a : b; a3 = lab ? b : a; }
    ierr = 0;
    if (a1 == UN) return UN;
    double x = a1 + f;
    if (!(x > a2)) return x;
    double amb = a1 - a2;
    if (__builtin_fabs(amb) < f) {
        double arg = (2.0 * f) * f - amb * amb;
        x = 0.5 * ((a1 + a2) + __builtin_sqrt(arg));
    } else {
        x = (a1 < a2 ? a1 : a2) + f;
    }
    if (!(x > a3)) return x;
    double qb = -((2.0 / 3.0) * ((a1 + a2) + a3));
    double qc = ((((a1 * a1) + (a2 * a2)) + (a3 * a3)) - f * f) * (1.0 / 3.0);
    double disc = qb * qb - 4.0 * qc;
    if (disc < 0.0) ierr = 1;
    x = 0.5 * (-qb + __builtin_sqrt(disc));
    if (x < 0.0) ierr = 2;
    if (x < UN) return x;
    ierr = 3;
    return UN;
}

// ---- 8-value column segments (32 B fp32 / 64 B fp64, always aligned) ------
__device__ __forceinline__ void load8(const float *p, float (&v)[8])
{
    float4 a = reinterpret_cast<const float4 *>(p)[0], b = reinterpret_cast<const float4 *>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(float *p, const float (&v)[8])
{
    reinterpret_cast<float4 *>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4 *>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void load8(const double *p, double (&v)[8])
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double2 a = reinterpret_cast<const double2 *>(p)[i];
        v[2 * i] = a.x; v[2 * i + 1] = a.y;
    }
}
__device__ __forceinline__ void store8(double *p, const double (&v)[8])
{
#pragma unroll
    for (int i = 0; i < 4; i++) reinterpret_cast<double2 *>(p)[i] = make_double2(v[2 * i], v[2 * i + 1]);
}

template <typename R>
__device__ __forceinline__ R shfl_up_(R v, int d) { return __shfl_up(v, d, 64); }
template <typename R>
__device__ __forceinline__ R shfl_down_(R v, int d) { return __shfl_down(v, d, 64); }

// x-fastest node -> brick-layout element index
__device__ __forceinline__ size_t brick_index(const FsmLaunch &L, int x, int y, int z)
{
    int tile = (y >> 3) * L.ntx + (x >> 3);
    return ((((size_t)tile * L.nzb + (z >> 3)) * 64 + ((y & 7) * 8 + (x & 7))) << 3) + (z & 7);
}

// Where a lane stands in the tile/brick stream of one sweep.
struct Brick {
    bool valid;       // a real brick (not before/after the stream or z padding)
    bool in_xy;       // this lane's column is inside the grid
    bool xp, xn, yp, yn;   // sweep-upwind / sweep-downwind neighbour exists (grid edge rule)
    int x, y, zb;     // physical column and z-brick
    size_t seg;       // element offset of this lane's 8-value column segment
    size_t hx_seg;    // x-downwind halo segment (lane lx=7), next tile
    size_t hy_seg;    // y halo segment (ly=0: upwind tile, ly=7: downwind tile)
};

template <bool RZ>
__device__ __forceinline__ Brick brick_at(const FsmLaunch &L, int vb, int lxs, int lys, int rx, int ry)
{
    Brick b;
    b.valid = false; b.in_xy = false; b.xp = b.xn = b.yp = b.yn = false;
    b.x = b.y = b.zb = 0; b.seg = b.hx_seg = b.hy_seg = 0;
    if (vb < 0) return b;
    int k = vb / L.sb, zbs = vb - k * L.sb;
    if (k >= L.ntiles || zbs >= L.nzb) return b;
    b.valid = true;
    int tys = k / L.ntx, txs = k - tys * L.ntx;
    int tx = rx ? L.ntx - 1 - txs : txs, ty = ry ? L.nty - 1 - tys : tys;
    b.zb = RZ ? L.nzb - 1 - zbs : zbs;
    int lx = rx ? 7 - lxs : lxs, ly = ry ? 7 - lys : lys;
    b.x = tx * 8 + lx; b.y = ty * 8 + ly;
    b.in_xy = b.x < L.nx && b.y < L.ny;
    bool xlo = b.x > 0, xhi = b.x < L.nx - 1, ylo = b.y > 0, yhi = b.y < L.ny - 1;
    b.xp = rx ? xhi : xlo; b.xn = rx ? xlo : xhi;
    b.yp = ry ? yhi : ylo; b.yn = ry ? ylo : yhi;
    b.seg = ((((size_t)(ty * L.ntx + tx) * L.nzb + b.zb) * 64 + (ly * 8 + lx)) << 3);
    // x-downwind halo: first column of the next tile in sweep order
    int txn = rx ? tx - 1 : tx + 1, lxn = rx ? 7 : 0;
    if (lxs == 7 && b.xn)
        b.hx_seg = ((((size_t)(ty * L.ntx + txn) * L.nzb + b.zb) * 64 + (ly * 8 + lxn)) << 3);
    // y halos: upwind tile's last row (new values), downwind tile's first row (old values)
    if (lys == 0 && b.yp) {
        int tyh = ry ? ty + 1 : ty - 1, lyh = ry ? 0 : 7;
        b.hy_seg = ((((size_t)(tyh * L.ntx + tx) * L.nzb + b.zb) * 64 + (lyh * 8 + lx)) << 3);
    } else if (lys == 7 && b.yn) {
        int tyh = ry ? ty - 1 : ty + 1, lyh = ry ? 7 : 0;
        b.hy_seg = ((((size_t)(tyh * L.ntx + tx) * L.nzb + b.zb) * 64 + (lyh * 8 + lx)) << 3);
    }
    return b;
}

// Per-solve boundary-condition boxes (EIKONAL3D_SETBCS nodes, lupd = .FALSE.).
// Wave-uniform, kept in LDS: box k = {xlo, xhi, ylo, yhi, zlo, zhi} (0-based, inclusive).
struct BcBoxes {
    int n;
    int *box;          // LDS, [MCEIK_MAX_SRC][6]
};
#define BC_LDS_BYTES (MCEIK_MAX_SRC * 6 * 4)

__device__ __forceinline__ bool in_bc_xy(const BcBoxes &bc, int k, int x, int y)
{
    const int *b = bc.box + 6 * k;
    return x >= b[0] && x <= b[1] && y >= b[2] && y <= b[3];
}

// Slowness*h for the 8 nodes of a lane's segment.
template <typename R, int SLOWMODE>
__device__ __forceinline__ void load_f(const FsmLaunch &L, const void *slow_model, const Brick &b,
                                       R hr, R (&f)[8])
{
    if (SLOWMODE == 0) {
        R s[8];
        load8(reinterpret_cast<const R *>(slow_model) + b.seg, s);
#pragma unroll
        for (int i = 0; i < 8; i++) f[i] = s[i] * hr;
    } else {
        const float *si = reinterpret_cast<const float *>(slow_model);
        int cx = min(b.x, L.nx - 1) / L.nrx, cy = min(b.y, L.ny - 1) / L.nry;
        const float *col = si + (size_t)cy * L.ncx + cx;
        size_t plane = (size_t)L.ncx * L.ncy;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            int z = min(b.zb * 8 + i, L.nz - 1);
            f[i] = (R)col[(size_t)(z / L.nrz) * plane] * hr;
        }
    }
}

template <typename R, int SLOWMODE>
__device__ __forceinline__ double slow_at(const FsmLaunch &L, const void *slow_model, int x, int y, int z)
{
    if (SLOWMODE == 0)
        return (double)reinterpret_cast<const R *>(slow_model)[brick_index(L, x, y, z)];
    const float *si = reinterpret_cast<const float *>(slow_model);
    return (double)si[((size_t)(z / L.nrz) * L.ncy + y / L.nry) * L.ncx + x / L.nrx];
}

// One Gauss-Seidel sweep over the whole grid in direction (rx, ry, RZ).
template <typename R, int SLOWMODE, bool RZ>
__device__ __forceinline__ void sweep(const FsmLaunch &L, R *__restrict__ u, R *__restrict__ u0,
                                      const void *slow_model, const BcBoxes &bc, R *xh,
                                      int rx, int ry, bool first_sweep, bool last_sweep,
                                      bool &notconv, int &ierr_last)
{
    const int lane = threadIdx.x, lxs = lane & 7, lys = lane >> 3, d = lxs + lys;
    const R UN = Num<R>::unan();
    const R hr = (R)L.h, T = (R)L.conv_thresh, tolr = (R)L.tol;
    const int nmacro = L.ntiles * L.sb + 14;

    R c[8], n[8], q[8], r[8], hx[8], hy[8], hxq[8], hyq[8], f[8], fq[8];
#pragma unroll
    for (int i = 0; i < 8; i++) { c[i] = n[i] = q[i] = r[i] = hx[i] = hy[i] = hxq[i] = hyq[i] = UN; f[i] = fq[i] = 0; }

    // prologue: resident c = brick(vb0), n = brick(vb0+1), halo/f of vb0
    {
        Brick b0 = brick_at<RZ>(L, -d, lxs, lys, rx, ry), b1 = brick_at<RZ>(L, 1 - d, lxs, lys, rx, ry);
        if (b0.valid) {
            load8(u + b0.seg, c);
            load_f<R, SLOWMODE>(L, slow_model, b0, hr, f);
            if (b0.hx_seg) load8(u + b0.hx_seg, hx);
            if (b0.hy_seg) load8(u + b0.hy_seg, hy);
        }
        if (b1.valid) load8(u + b1.seg, n);
    }

    for (int B = 0; B < nmacro; B++) {
        const int vb = B - d;
        const Brick b = brick_at<RZ>(L, vb, lxs, lys, rx, ry);
        // prefetch: u of brick vb+2 (becomes n next step), halo + f of vb+1
        {
            Brick b1 = brick_at<RZ>(L, vb + 1, lxs, lys, rx, ry), b2 = brick_at<RZ>(L, vb + 2, lxs, lys, rx, ry);
            if (b2.valid) load8(u + b2.seg, q);
            if (b1.valid) {
                load_f<R, SLOWMODE>(L, slow_model, b1, hr, fq);
                if (b1.hx_seg) load8(u + b1.hx_seg, hxq);
                if (b1.hy_seg) load8(u + b1.hy_seg, hyq);
            }
        }
        // BC membership of this column for each source box
        unsigned bcxy = 0;
        for (int k = 0; k < bc.n; k++) bcxy |= (in_bc_xy(bc, k, b.x, b.y) ? 1u : 0u) << k;
        const bool colact = b.valid && b.in_xy;
        bool changed = false;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int pj = RZ ? 7 - j : j;                 // physical slot of sweep slot j
            const int pprev = RZ ? pj + 1 : pj - 1;         // physical slot of sweep slot j-1
            const int pnext = RZ ? pj - 1 : pj + 1;         // physical slot of sweep slot j+1
            const int zabs = b.zb * 8 + pj;
            const R self = c[pj];
            // neighbour lanes: upwind lanes are one brick ahead (their r[pj] still
            // holds this brick's slot j), downwind lanes one brick behind (their n[pj])
            const R xm = shfl_up_(r[pj], 1), xpv = shfl_down_(n[pj], 1);
            const R ym = shfl_up_(r[pj], 8), ypv = shfl_down_(n[pj], 8);
            R xup = self, xdn = self, yup = self, ydn = self, zup = self, zdn = self;
            if (b.xp) xup = lxs > 0 ? xm : xh[zabs * 8 + lys];
            if (b.xn) xdn = lxs < 7 ? xpv : hx[pj];
            if (b.yp) yup = lys > 0 ? ym : hy[pj];
            if (b.yn) ydn = lys < 7 ? ypv : hy[pj];
            const bool zp_ex = RZ ? (zabs < L.nz - 1) : (zabs > 0);
            const bool zn_ex = RZ ? (zabs > 0) : (zabs < L.nz - 1);
            if (zp_ex) zup = j > 0 ? r[pprev] : r[RZ ? 0 : 7];
            if (zn_ex) zdn = j < 7 ? c[pnext] : n[RZ ? 7 : 0];
            const R ux = xup < xdn ? xup : xdn;
            const R uy = yup < ydn ? yup : ydn;
            const R uz = zup < zdn ? zup : zdn;
            int e;
            const R ub = godunov(ux, uy, uz, f[pj], e);
            bool isbc = false;
            for (int k = 0; k < bc.n; k++)
                isbc |= ((bcxy >> k) & 1u) && zabs >= bc.box[6 * k + 4] && zabs <= bc.box[6 * k + 5];
            const bool upd = colact && zabs < L.nz && !isbc;
            const R nv = upd ? (self < ub ? self : ub) : self;
            if (upd && nv < self && self >= T) notconv = true;
            if (last_sweep && colact && b.x == 0 && b.y == 0 && zabs == 0) ierr_last = upd ? e : 0;
            changed |= nv != self;
            r[pj] = nv;
            if (lxs == 7 && b.valid) xh[zabs * 8 + lys] = nv;
        }
        if (b.valid) {
            if (changed) store8(u + b.seg, r);
            if (first_sweep) {
                bool need = false;
#pragma unroll
                for (int i = 0; i < 8; i++) need |= c[i] < T;
                if (need) store8(u0 + b.seg, c);
            }
            if (last_sweep && !notconv && colact) {
                bool need = false;
#pragma unroll
                for (int i = 0; i < 8; i++) need |= (r[i] < T) && (b.zb * 8 + i < L.nz);
                if (need) {
                    R v0[8];
                    load8(u0 + b.seg, v0);
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        R dlt = v0[i] - r[i];
                        dlt = dlt < (R)0 ? -dlt : dlt;
                        if (b.zb * 8 + i < L.nz && !(dlt < tolr)) notconv = true;
                    }
                }
            }
        }
        asm volatile("" ::: "memory");   // order LDS halo traffic across steps (one wave, in-order LDS)
#pragma unroll
        for (int i = 0; i < 8; i++) { c[i] = n[i]; n[i] = q[i]; hx[i] = hxq[i]; hy[i] = hyq[i]; f[i] = fq[i]; }
    }
}

// ---- per-solve setup: u = u_nan, then the source boxes (EIKONAL3D_SETBCS) ----
template <typename R, int SLOWMODE>
__device__ bool init_field(const FsmLaunch &L, R *u, const void *slow_model, const double *src,
                           BcBoxes &bc)
{
    const int lane = threadIdx.x;
    const R UN = Num<R>::unan();
    const size_t nvec = L.field_elems / 8;
    R fill[8];
#pragma unroll
    for (int i = 0; i < 8; i++) fill[i] = UN;
    for (size_t i = lane; i < nvec; i += 64) store8(u + i * 8, fill);
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
        if (!ok) { bc.n = s; return false; }
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
                size_t idx = brick_index(L, ix - 1, iy - 1, iz - 1);
                R cur = u[idx];
                u[idx] = (__builtin_fabs(dd) < 1.e-10) ? t : (cur < t ? cur : t);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    return true;
}

template <typename R, int SLOWMODE>
__global__ __launch_bounds__(64) void fsm_solve_kernel(FsmLaunch L)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int *bcbox = reinterpret_cast<int *>(smem);                 // 192 B, 16-B multiple
    R *xh = reinterpret_cast<R *>(smem + BC_LDS_BYTES);
    const int lane = threadIdx.x;
    for (;;) {
        unsigned solve = 0;
        if (lane == 0) solve = atomicAdd(L.counter, 1u);
        solve = __shfl(solve, 0, 64);
        if (solve >= (unsigned)L.nsolve) break;
        const int model = (int)solve / L.nstat, station = (int)solve - model * L.nstat;
        const size_t slot = L.slot_per_solve ? solve : blockIdx.x;
        R *u = reinterpret_cast<R *>(L.u) + slot * L.field_elems;
        R *u0 = reinterpret_cast<R *>(L.u0) + (size_t)blockIdx.x * L.field_elems;   // per-wave scratch
        const void *slow_model = SLOWMODE == 0
            ? (const void *)(reinterpret_cast<const R *>(L.slow) + (size_t)model * L.field_elems)
            : (const void *)(reinterpret_cast<const float *>(L.slow) + (size_t)model * L.ncx * L.ncy * L.ncz);
        BcBoxes bc;
        bc.box = bcbox;
        const bool ok = init_field<R, SLOWMODE>(L, u, slow_model, L.src + (size_t)station * L.nsrc * 4, bc);
        int iters = 0, ierr_last = 0;
        if (ok) {
            int sweeps_left = L.max_sweeps < 0 ? 0x7fffffff : L.max_sweeps;
            for (int it = 0; it < L.maxit && sweeps_left > 0; it++) {
                bool notconv = false;
                for (int sw = 0; sw < 8 && sweeps_left > 0; sw++, sweeps_left--) {
                    const int rx = sw & 1, ry = (sw >> 1) & 1;
                    const bool first = sw == 0, last = sw == 7;
                    if (sw & 4)
                        sweep<R, SLOWMODE, true>(L, u, u0, slow_model, bc, xh, rx, ry, first, last, notconv, ierr_last);
                    else
                        sweep<R, SLOWMODE, false>(L, u, u0, slow_model, bc, xh, rx, ry, first, last, notconv, ierr_last);
                    __builtin_amdgcn_s_waitcnt(0);      // stores of this sweep land before the next sweep's loads
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                }
                iters = it + 1;
                if (sweeps_left > 0 || L.max_sweeps < 0) {
                    if (!__any(notconv)) break;
                }
            }
        }
        // reduce ierr over lanes (only the lane owning node (0,0,0) sets it)
        int ierr = ierr_last;
        for (int o = 32; o > 0; o >>= 1) ierr = max(ierr, __shfl_xor(ierr, o, 64));
        if (!ok) ierr = 1;
        if (lane == 0) {
            if (L.iter_total) atomicAdd(L.iter_total, (unsigned long long)iters);
            if (L.niter) L.niter[solve] = iters;
            if (L.ierr) L.ierr[solve] = ierr;
        }
        if (L.ttab) {
            for (int e = lane; e < L.nev; e += 64) {
                int node = L.ev_node[e];
                int nxy = L.nx * L.ny;
                int z = node / nxy, rem = node - z * nxy, y = rem / L.nx, x = rem - y * L.nx;
                L.ttab[(size_t)solve * L.nev + e] = (float)u[brick_index(L, x, y, z)];
            }
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
        int zi = e & 7; size_t t = e >> 3;
        int col = t & 63; t >>= 6;
        int zb = (int)(t % L.nzb); int tile = (int)(t / L.nzb);
        int ty = tile / L.ntx, tx = tile - ty * L.ntx;
        int x = tx * 8 + (col & 7), y = ty * 8 + (col >> 3), z = zb * 8 + zi;
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
        dst[i] = (RD)src[fld * L.field_elems + brick_index(L, x, y, z)];
    }
}

}  // namespace

// ---- host-side launchers (C++ linkage, used by capi.hip) ---------------------
int fsm_max_resident_waves(int dev, size_t lds_bytes, int is_double, int slow_mode);

template <typename R, int SLOWMODE>
static hipError_t launch_fsm(const FsmLaunch &L, int nwaves, hipStream_t st)
{
    size_t lds = BC_LDS_BYTES + (size_t)L.nzb * 8 * 8 * sizeof(R);
    hipLaunchKernelGGL((fsm_solve_kernel<R, SLOWMODE>), dim3(nwaves), dim3(64), lds, st, L);
    return hipGetLastError();
}

hipError_t fsm_launch(const FsmLaunch &L, int is_double, int nwaves, hipStream_t st)
{
    if (is_double) return L.slow_mode ? launch_fsm<double, 1>(L, nwaves, st) : launch_fsm<double, 0>(L, nwaves, st);
    return L.slow_mode ? launch_fsm<float, 1>(L, nwaves, st) : launch_fsm<float, 0>(L, nwaves, st);
}

int fsm_occupancy(int is_double, int slow_mode, size_t lds)
{
    int nb = 0;
    hipError_t e;
    if (is_double)
        e = slow_mode ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_solve_kernel<double, 1>, 64, lds)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_solve_kernel<double, 0>, 64, lds);
    else
        e = slow_mode ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_solve_kernel<float, 1>, 64, lds)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_solve_kernel<float, 0>, 64, lds);
    return e == hipSuccess ? nb : 1;
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
