// fsm_single.hip -- ONE eikonal solve spread over the whole GPU: the path of
// the drop-in entry points eikonal3d_serial_driver (fsm3d.f90:1968-2052) and
// eikonal3d_solve (fsm3d.f90:1754-1889), where a caller asks for one table at
// a time and the batched kernel (one wave per solve) would leave 2047 of 2048
// wave slots idle.
//
// Schedule: the grid is cut into 8x8x8 bricks; a task is (sweep g, brick),
// and the tasks of sweep g are handed out level by level of the brick
// hyperplanes bx+by+bz in g's direction -- MAKE_LEVEL_STRUCT (fsm3d.f90:226-308)
// at brick granularity.  A persistent wave takes the next task from one
// atomic counter and waits (relaxed polls + one agent-scope acquire,
// cdna_hip_programming.md s.6 G16) until
//   * the brick has finished sweep g-1,
//   * every face neighbour that is upwind in g has finished sweep g, and
//   * every downwind face neighbour has finished sweep g-1 (it cannot have
//     started g: it waits for this brick),
// so every node sees exactly the new / old neighbour values of the
// reference's Gauss-Seidel order and the result is bitwise the reference's.
// Sweeps overlap (sweep g+1 starts in the corner sweep g finished first); the
// iterations are separated by the convergence test (|u0-u| < tol at every
// node, fsm3d.f90:86-95), decided by the last brick to finish the iteration.
// Inside a brick the 22 node hyperplanes run one after another, a level's
// nodes on different lanes, all in LDS.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include <algorithm>

#include "fsm_common.h"
#include "fsm_update.h"
#include "fsm_single.h"

namespace {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ unsigned poll32(const unsigned *p)
{
    return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every wait is bounded (a schedule bug must not hang the GPU): after ~2^22
// polls (seconds) the wave records the failure in ctl[1] and exits; the host
// reports it as a device failure.
#define SPIN_LIMIT (1u << 22)
__device__ __noinline__ void spin_fail(const SingleLaunch &L, unsigned code)
{
    if (threadIdx.x == 0) {
        __hip_atomic_store((gu32 *)(L.ctl + 1), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu32 *)(L.ctl + 2 + code), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Update of one node from its 6 neighbours in the LDS brick (+1 halo), with the
// one-sided edge rule of GET_U{X,Y,Z}MIN3D (fsm3d.f90:484-546): a neighbour
// outside the grid is replaced by the node itself.
template <typename R>
__device__ __forceinline__ R node_update(const R *ext, int e, R self, bool xm, bool xp, bool ym, bool yp, bool zm,
                                         bool zp, R f, int &ierr)
{
    const R a = xm ? ext[e - 1] : self, b = xp ? ext[e + 1] : self;
    const R c = ym ? ext[e - 10] : self, d = yp ? ext[e + 10] : self;
    const R g = zm ? ext[e - 100] : self, k = zp ? ext[e + 100] : self;
    const R ux = fmin_(a, b), uy = fmin_(c, d), uz = fmin_(g, k);
    return godunov_bl<false>(ux, uy, uz, f, ierr);
}

// Write-through (sc1) 16-B stores of one brick row: the payload of a hand-off
// (G16 R1).  r: wave-uniform resource of the whole field; off: this lane's row.
template <typename R>
__device__ __forceinline__ void st_row_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const R (&v)[8])
{
    constexpr int PER = 16 / sizeof(R);
#pragma unroll
    for (int k = 0; k < 8 / PER; k++) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        R w[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) w[i] = v[k * PER + i];
        u4 bits;
        __builtin_memcpy(&bits, w, 16);
        __builtin_amdgcn_raw_buffer_store_b128(bits, r, off + 16 * k, 0, 16);
    }
}

template <typename R>
__device__ __forceinline__ void ld_row(const R *p, R (&v)[8])
{
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = p[i];
}

template <typename R>
__global__ __launch_bounds__(64) void fsm_single_kernel(SingleLaunch L)
{
    __shared__ __attribute__((aligned(16))) R ext[1000];     // brick + 1-node halo, [z][y][x] 10^3
    __shared__ __attribute__((aligned(16))) R fsl[512];      // s*h of the brick's nodes
    __shared__ unsigned char bcl[512];                       // boundary-condition node (lupd = .FALSE.)
    __shared__ unsigned short order[512];                    // brick nodes by sweep-local level
    __shared__ int lvl[24];
    const int lane = threadIdx.x;
    const R tol = (R)L.tol, hr = (R)L.h, UN = Num<R>::unan();
    // node order of a brick by level i+j+k (sweep-local coordinates)
    if (lane == 0) {
        int n = 0;
        for (int l = 0; l <= 21; l++) {
            lvl[l] = n;
            for (int k = 0; k < 8; k++)
                for (int j = 0; j < 8; j++) {
                    const int i = l - k - j;
                    if (i >= 0 && i < 8) order[n++] = (unsigned short)(i | (j << 3) | (k << 6));
                }
        }
        lvl[22] = n;
    }
    __syncthreads();
    const size_t sy = (size_t)L.nxp, sz = (size_t)L.nxp * L.nyp;
    R *u = (R *)L.u, *u0 = (R *)L.u0;
    const R *slow = (const R *)L.slow;
    const uint32_t fbytes = (uint32_t)((size_t)L.nxp * L.nyp * L.nzp * sizeof(R));
    const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(u, 0, fbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t u0r = __builtin_amdgcn_make_buffer_rsrc(u0, 0, fbytes, 0x00020000);
    int known = 0;                       // iterations < known are decided "not converged"
    if (*L.bcerr) return;                // SETBCS failed: the reference returns before EIKONAL3D_FSM
    for (;;) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(L.ctl, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, 64));
        const int g = (int)(t / (unsigned)L.nb), r = (int)(t % (unsigned)L.nb);
        const int it = g >> 3, s = g & 7;
        if (it >= L.maxit) break;
        // iteration barrier: every earlier iteration must be decided "not
        // converged" (in order: a task two iterations ahead must not wait for
        // a decision that an earlier convergence makes never happen)
        bool stop = false;
        for (; known < it && !stop; known++) {
            unsigned dec = 0;
            for (unsigned spins = 0;; spins++) {
                if (lane == 0) dec = poll32(L.ctl + 32 + known);
                dec = __builtin_amdgcn_readfirstlane(__shfl(dec, 0, 64));
                if (dec) break;
                if (spins > SPIN_LIMIT) { spin_fail(L, 2); return; }
                __builtin_amdgcn_s_sleep(2);
            }
            stop = dec == 2;             // converged: no task of a later iteration runs
        }
        if (stop) break;
        const int rx = s & 1, ry = (s >> 1) & 1, rz = (s >> 2) & 1;   // evalSweep order (fsm3d.f90:46-53)
        const int w = L.border[r];
        const int bx = rx ? L.nbx - 1 - (w & 1023) : (w & 1023);
        const int by = ry ? L.nby - 1 - ((w >> 10) & 1023) : ((w >> 10) & 1023);
        const int bz = rz ? L.nbz - 1 - (w >> 20) : (w >> 20);
        const int b = (bz * L.nby + by) * L.nbx + bx;
        // dependencies: lane 0 self (>= g), lanes 1..6 the face neighbours
        {
            int nb = -1;
            unsigned need = (unsigned)g;
            if (lane == 0) nb = b;
            else if (lane <= 6) {
                const int ax = (lane - 1) >> 1, up = (lane - 1) & 1;    // axis, upwind side?
                const int dir = ax == 0 ? rx : ax == 1 ? ry : rz;       // 1: sweep runs downwards
                const int step = (up ? -1 : 1) * (dir ? -1 : 1);        // offset to that neighbour
                const int cx = bx + (ax == 0 ? step : 0), cy = by + (ax == 1 ? step : 0),
                          cz = bz + (ax == 2 ? step : 0);
                if (cx >= 0 && cx < L.nbx && cy >= 0 && cy < L.nby && cz >= 0 && cz < L.nbz) {
                    nb = (cz * L.nby + cy) * L.nbx + cx;
                    need = up ? (unsigned)g + 1u : (unsigned)g;
                }
            }
            for (unsigned spins = 0;; spins++) {
                const bool ok = nb < 0 || poll32(L.done + nb) >= need;
                if (__all(ok)) break;
                if (spins > SPIN_LIMIT) { spin_fail(L, 1); return; }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // load the brick (row per lane: y = lane & 7, z = lane >> 3) and its face halos
        const int x0 = bx * 8, y0 = by * 8, z0 = bz * 8;
        const int ly = lane & 7, lz = lane >> 3;
        const size_t row = (size_t)(z0 + lz) * sz + (size_t)(y0 + ly) * sy + (size_t)x0;
        R v[8], f[8];
        ld_row(u + row, v);
        ld_row(slow + row, f);
        const unsigned long long bcw = *(const unsigned long long *)(L.bc + row);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            ext[(lz + 1) * 100 + (ly + 1) * 10 + i + 1] = v[i];
            fsl[lane * 8 + i] = f[i] * hr;
            bcl[lane * 8 + i] = (unsigned char)((bcw >> (8 * i)) & 0xff);
        }
        {
            // faces: x (y = ly, z = lz), y (x = ly, z = lz), z (x = ly, y = lz); outside the grid unused
            const int X = x0 - 1, X8 = x0 + 8, Y = y0 - 1, Y8 = y0 + 8, Z = z0 - 1, Z8 = z0 + 8;
            const size_t ry0 = (size_t)(z0 + lz) * sz + (size_t)(y0 + ly) * sy;
            const size_t rx0 = (size_t)(z0 + lz) * sz + (size_t)(x0 + ly);
            const size_t rz0 = (size_t)(y0 + lz) * sy + (size_t)(x0 + ly);
            const R hxm = X >= 0 ? u[ry0 + X] : UN, hxp = X8 < L.nxp ? u[ry0 + X8] : UN;
            const R hym = Y >= 0 ? u[rx0 + (size_t)Y * sy] : UN, hyp = Y8 < L.nyp ? u[rx0 + (size_t)Y8 * sy] : UN;
            const R hzm = Z >= 0 ? u[rz0 + (size_t)Z * sz] : UN, hzp = Z8 < L.nzp ? u[rz0 + (size_t)Z8 * sz] : UN;
            ext[(lz + 1) * 100 + (ly + 1) * 10 + 0] = hxm;
            ext[(lz + 1) * 100 + (ly + 1) * 10 + 9] = hxp;
            ext[(lz + 1) * 100 + 0 * 10 + ly + 1] = hym;
            ext[(lz + 1) * 100 + 9 * 10 + ly + 1] = hyp;
            ext[0 * 100 + (lz + 1) * 10 + ly + 1] = hzm;
            ext[9 * 100 + (lz + 1) * 10 + ly + 1] = hzp;
        }
        if (s == 0) st_row_wt<R>(u0r, (uint32_t)(row * sizeof(R)), v);   // start-of-iteration values
        __syncthreads();
        // the 22 node levels of the brick in the sweep's direction
        int ierr0 = 0;
        for (int l = 0; l <= 21; l++) {
            const int k0 = lvl[l], cnt = lvl[l + 1] - k0;
            if (lane < cnt) {
                const int o = order[k0 + lane];
                const int i = o & 7, j = (o >> 3) & 7, k = o >> 6;
                const int x = rx ? 7 - i : i, y = ry ? 7 - j : j, z = rz ? 7 - k : k;
                const int gx = x0 + x, gy = y0 + y, gz = z0 + z;
                const int nid = (z * 8 + y) * 8 + x;
                if (gx < L.nx && gy < L.ny && gz < L.nz && !bcl[nid]) {
                    const int e = (z + 1) * 100 + (y + 1) * 10 + x + 1;
                    const R self = ext[e];
                    int ie = 0;
                    const R ub = node_update<R>(ext, e, self, gx > 0, gx < L.nx - 1, gy > 0, gy < L.ny - 1, gz > 0,
                                                gz < L.nz - 1, fsl[nid], ie);
                    ext[e] = fmin_(self, ub);
                    if ((gx | gy | gz) == 0) ierr0 = ie;
                }
            }
            __syncthreads();
        }
        // write back; the last sweep of an iteration also tests convergence
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = ext[(lz + 1) * 100 + (ly + 1) * 10 + i + 1];
        st_row_wt<R>(ur, (uint32_t)(row * sizeof(R)), v);
        bool nc = false;
        if (s == 7) {
            R a[8];
            ld_row(u0 + row, a);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                R dl = a[i] - v[i];
                dl = dl < (R)0 ? -dl : dl;
                if (x0 + i < L.nx && y0 + ly < L.ny && z0 + lz < L.nz && !(dl < tol)) nc = true;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every lane's payload has landed
        const bool anync = __any(nc);
        for (int o = 32; o > 0; o >>= 1) ierr0 = max(ierr0, __shfl_xor(ierr0, o, 64));
        if (lane == 0) {
            if (s == 7 && b == 0) L.ierr_it[it] = ierr0;       // node (0,0,0): the reference's last ierr
            __hip_atomic_store((gu32 *)(L.done + b), (unsigned)g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (s == 7) {
                const unsigned long long add = 1ull | (anync ? (1ull << 32) : 0ull);
                const unsigned long long old =
                    __hip_atomic_fetch_add((gu64 *)(L.arrive + it), add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((unsigned)(old & 0xffffffffu) == (unsigned)L.nb - 1u) {
                    const bool conv = ((old >> 32) == 0) && !anync;
                    __hip_atomic_store((gu32 *)(L.ctl + 32 + it), conv ? 2u : 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
}

// u = u_nan on the padded grid, bc = 0.
template <typename R>
__global__ void single_fill_kernel(R *u, unsigned char *bc, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        u[i] = Num<R>::unan();
        bc[i] = 0;
    }
}

// EIKONAL3D_SETBCS (fsm3d.f90:762-840) with EIKONAL_SOURCE_INDEX / EIKONAL_INIT_GRID
// (:697-755), sources in order: one wave, lanes 0..26 own the 3x3x3 candidates.
template <typename R>
__global__ void single_setbcs_kernel(SingleLaunch L, const double *src, int nsrc, int *ierr)
{
    const int lane = threadIdx.x;
    R *u = (R *)L.u;
    const R *slow = (const R *)L.slow;
    const size_t sy = (size_t)L.nxp, sz = (size_t)L.nxp * L.nyp;
    int bad = 0;
    for (int s = 0; s < nsrc && !bad; s++) {
        const double *sp = src + (size_t)s * 4;
        int loc[3][3];
        const int nn[3] = {L.gx, L.gy, L.gz};
        const double org[3] = {L.x0, L.y0, L.z0};
        for (int a = 0; a < 3; a++) {
            const double xs = sp[1 + a], x0 = org[a], dx = L.h;
            const int n = nn[a];
            int is;
            if (xs <= x0) is = 1;
            else if (xs >= x0 + (double)(n - 1) * dx) is = n;
            else is = (int)((xs - x0) / dx + 0.5) + 1;
            int np = 0;
            loc[a][0] = loc[a][1] = loc[a][2] = -1;
            const double xe = x0 + (double)(is - 1) * dx;
            if (xe > xs) { loc[a][0] = is - 1; loc[a][1] = is; np = 2; }
            else if (xe < xs) { loc[a][0] = is; loc[a][1] = is + 1; np = 2; }
            else {
                loc[a][np++] = is - 1;          // the reference's isx-1 (0 when the source is on node 1)
                loc[a][np++] = is;
                if (is < n - 1) loc[a][np++] = is + 1;
            }
            for (int i = 0; i < np; i++) if (loc[a][i] < 1 || loc[a][i] > n) bad = 1;
        }
        if (bad) break;
        if (lane < 27) {
            const int i = lane % 3, j = (lane / 3) % 3, k = lane / 9;
            const int ix = loc[0][i], iy = loc[1][j], iz = loc[2][k];
            // local node (the fields may hold a box of the grid: nodes outside it are skipped)
            const int lx = ix - 1 - L.ox, ly = iy - 1 - L.oy, lz = iz - 1 - L.oz;
            if (ix != -1 && iy != -1 && iz != -1 && lx >= 0 && lx < L.nx && ly >= 0 && ly < L.ny && lz >= 0 &&
                lz < L.nz) {
                const double x = L.x0 + (double)(ix - 1) * L.h, y = L.y0 + (double)(iy - 1) * L.h,
                             z = L.z0 + (double)(iz - 1) * L.h;
                const double ddx = sp[1] - x, ddy = sp[2] - y, ddz = sp[3] - z;
                const double dd = __builtin_sqrt((ddx * ddx + ddy * ddy) + ddz * ddz);
                const size_t idx = (size_t)lz * sz + (size_t)ly * sy + (size_t)lx;
                const R t = (R)(sp[0] + dd * (double)slow[idx]);
                const R cur = u[idx];
                u[idx] = (__builtin_fabs(dd) < 1.e-10) ? t : (cur < t ? cur : t);
                L.bc[idx] = 1;
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    if (lane == 0) *ierr = bad;
}

// dense x-fastest <-> padded layout
template <typename RS, typename RD>
__global__ void single_pad_kernel(const RS *src, RD *dst, int nx, int ny, int nz, int nxp, int nyp, int to_padded)
{
    const size_t n = (size_t)nx * ny * nz;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % nx);
        const size_t t = i / nx;
        const int y = (int)(t % ny), z = (int)(t / ny);
        const size_t p = ((size_t)z * nyp + y) * nxp + x;
        if (to_padded) dst[p] = (RD)src[i];
        else dst[i] = (RD)src[p];
    }
}

// ---- the MPI variant's block decomposition (EIKONAL3D_FSM_MPI) --------------
// fsm3d.f90:103-222 with EIKONAL3D_GHOST_COMM's blocks (:1086-1101) and
// EIKONAL_EXCHANGE after every sweep (:971-1046): per sweep every block runs
// its own Gauss-Seidel sweep over the nodes it owns, reading a neighbour that
// another block owns as that block's ghost copy, i.e. its value at the start
// of the sweep (snap), or -- without a ghost layer (noverlap = 0) -- as a
// missing neighbour (GET_U*MIN3D's one-sided rule: the node itself).  One
// workgroup per block walks the block's node hyperplanes in sweep order (the
// nodes of a level are independent), so the result is bitwise the reference's
// run with one MPI rank per block.  fp64, the padded layout of SingleLaunch.
//
// Across ranks (one block per rank, blocks_solve_ranks in capi.hip) a rank
// sweeps block b0 alone on a grid whose other nodes change only in the halo
// swap between sweeps, so snap is u itself.  ierr: the reference's EVAL_UPDATE3D
// ierr of the last level, the corner node of the rank's local grid (its block
// extended by the ghost layer, fsm3d.f90:1099-1104), which is an updated node
// only when the ghost layer does not extend it there (block 0 always).
__global__ __launch_bounds__(256) void block_sweep_kernel(SingleLaunch L, BlockDecomp D, const double *snap, int g,
                                                          int *ierr, int b0, int ierr_b)
{
    const int b = blockIdx.x + b0;
    const int bi[3] = {b % D.nd[0], (b / D.nd[0]) % D.nd[1], b / (D.nd[0] * D.nd[1])};
    const int nn[3] = {L.gx, L.gy, L.gz};
    int lo[3], ext[3];
    for (int a = 0; a < 3; a++) {
        lo[a] = D.step[a] * bi[a];
        const int hi = bi[a] + 1 == D.nd[a] ? nn[a] - 1 : D.step[a] * (bi[a] + 1) - 1;
        ext[a] = hi - lo[a] + 1;
        if (ext[a] <= 0) return;                       // an empty block (more blocks than nodes)
    }
    const bool rev[3] = {(g & 1) != 0, (g & 2) != 0, (g & 4) != 0};
    double *u = (double *)L.u;
    const double *slow = (const double *)L.slow;
    const size_t sy = (size_t)L.nxp, sz = (size_t)L.nxp * L.nyp;
    const bool ierr_here = b == ierr_b && (D.nov == 0 || (lo[0] == 0 && lo[1] == 0 && lo[2] == 0));
    const int nlev = ext[0] + ext[1] + ext[2] - 2;
    for (int lev = 0; lev < nlev; lev++) {
        const int zlo = max(0, lev - (ext[0] - 1) - (ext[1] - 1)), zhi = min(ext[2] - 1, lev);
        const int npairs = (zhi - zlo + 1) * ext[1];
        for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
            const int kz = zlo + p / ext[1], ky = p % ext[1], kx = lev - kz - ky;
            if (kx < 0 || kx >= ext[0]) continue;
            const int k3[3] = {kx, ky, kz};
            int c[3];
            for (int a = 0; a < 3; a++) c[a] = rev[a] ? lo[a] + ext[a] - 1 - k3[a] : lo[a] + k3[a];
            const size_t idx = (size_t)(c[2] - L.oz) * sz + (size_t)(c[1] - L.oy) * sy + (size_t)(c[0] - L.ox);
            if (L.bc[idx]) continue;                   // lupd = .FALSE. (SETBCS node)
            const double self = u[idx];
            double nb[6];
            const size_t stride[3] = {1, sy, sz};
            for (int a = 0; a < 3; a++)
                for (int s = 0; s < 2; s++) {
                    const int q = c[a] + (s ? 1 : -1);
                    const size_t qi = s ? idx + stride[a] : idx - stride[a];
                    double v;
                    if (q < 0 || q >= nn[a]) v = self;                          // outside the grid
                    else if (q >= lo[a] && q < lo[a] + ext[a]) v = u[qi];        // this block: live
                    else v = D.nov > 0 ? snap[qi] : self;                        // ghost / no ghost layer
                    nb[2 * a + s] = v;
                }
            const double ux = fmin_(nb[0], nb[1]), uy = fmin_(nb[2], nb[3]), uz = fmin_(nb[4], nb[5]);
            int e;
            const double ub = godunov(ux, uy, uz, slow[idx] * L.h, e);
            u[idx] = self < ub ? self : ub;
            if (ierr_here && c[0] == lo[0] && c[1] == lo[1] && c[2] == lo[2]) *ierr = e;   // last level
        }
        __syncthreads();
    }
}

// nodes of the box (global coordinates) with !(|u0 - u| < tol) (the FSM_MPI
// convergence count, fsm3d.f90:195-205; the whole grid, or the nodes a rank owns)
__global__ void block_unconverged_kernel(SingleLaunch L, BlockBox B, double tol, unsigned *count)
{
    const size_t n = (size_t)B.ext[0] * B.ext[1] * B.ext[2];
    unsigned c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int x = B.lo[0] + (int)(i % B.ext[0]);
        const size_t t = i / B.ext[0];
        const int y = B.lo[1] + (int)(t % B.ext[1]), z = B.lo[2] + (int)(t / B.ext[1]);
        const size_t p = ((size_t)(z - L.oz) * L.nyp + (y - L.oy)) * L.nxp + (x - L.ox);
        const double d = ((const double *)L.u0)[p] - ((const double *)L.u)[p];
        c += !(__builtin_fabs(d) < tol);
    }
    if (c) atomicAdd(count, c);
}

// Boxes of the padded fp64 grid (global coordinates, inside the fields' box)
// <-> one contiguous buffer, box k at off[k], x fastest inside a box: the halo faces a rank swaps after every sweep
// (EIKONAL_EXCHANGE, fsm3d.f90:971-1046) and the owned block it sends to the
// master at the end (EIKONAL_GATHER_TRAVELTIMES).
__global__ void box_copy_kernel(SingleLaunch L, BoxList bl, double *buf, int to_buf)
{
    const size_t total = bl.off[bl.n];
    double *u = (double *)L.u;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        int k = 0;
        while (i >= bl.off[k + 1]) k++;
        const BlockBox &B = bl.box[k];
        const size_t j = i - bl.off[k];
        const int x = B.lo[0] + (int)(j % B.ext[0]);
        const size_t t = j / B.ext[0];
        const int y = B.lo[1] + (int)(t % B.ext[1]), z = B.lo[2] + (int)(t / B.ext[1]);
        const size_t p = ((size_t)(z - L.oz) * L.nyp + (y - L.oy)) * L.nxp + (x - L.ox);
        if (to_buf) buf[i] = u[p];
        else u[p] = buf[i];
    }
}

}  // namespace

hipError_t fsm_single_setbcs(const SingleLaunch &L, const double *d_src, int nsrc, int *d_ierr_bc, hipStream_t st)
{
    const size_t np = (size_t)L.nxp * L.nyp * L.nzp;
    hipLaunchKernelGGL(single_fill_kernel<double>, dim3(1024), dim3(256), 0, st, (double *)L.u, L.bc, np);
    hipLaunchKernelGGL(single_setbcs_kernel<double>, dim3(1), dim3(64), 0, st, L, d_src, nsrc, d_ierr_bc);
    return hipGetLastError();
}

hipError_t fsm_block_sweep(const SingleLaunch &L, const BlockDecomp &D, const double *snap, int g, int *ierr,
                           hipStream_t st, int b0, int nblk, int ierr_b)
{
    if (nblk < 0) nblk = D.nd[0] * D.nd[1] * D.nd[2];
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(block_sweep_kernel, dim3(nblk), dim3(256), 0, st, L, D, snap, g, ierr, b0, ierr_b);
    return hipGetLastError();
}

hipError_t fsm_block_unconverged(const SingleLaunch &L, const BlockBox &B, double tol, unsigned *count,
                                 hipStream_t st)
{
    if ((size_t)B.ext[0] * B.ext[1] * B.ext[2] == 0) return hipSuccess;
    hipLaunchKernelGGL(block_unconverged_kernel, dim3(512), dim3(256), 0, st, L, B, tol, count);
    return hipGetLastError();
}

hipError_t fsm_box_copy(const SingleLaunch &L, const BoxList &bl, double *buf, int to_buf, hipStream_t st)
{
    if (bl.n < 1 || bl.off[bl.n] == 0) return hipSuccess;
    const size_t total = bl.off[bl.n];
    const unsigned nblk = (unsigned)std::min<size_t>(1024, (total + 255) / 256);
    hipLaunchKernelGGL(box_copy_kernel, dim3(nblk), dim3(256), 0, st, L, bl, buf, to_buf);
    return hipGetLastError();
}

int fsm_single_occupancy(int is_double)
{
    int nb = 0;
    hipError_t e = is_double ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_single_kernel<double>, 64, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fsm_single_kernel<float>, 64, 0);
    return e == hipSuccess && nb > 0 ? nb : 1;
}

hipError_t fsm_single_solve(const SingleLaunch &L, int is_double, const double *d_src, int nsrc, int *d_ierr_bc,
                            int nwaves, hipStream_t st)
{
    const size_t np = (size_t)L.nxp * L.nyp * L.nzp;
    if (is_double) {
        hipLaunchKernelGGL(single_fill_kernel<double>, dim3(1024), dim3(256), 0, st, (double *)L.u, L.bc, np);
        hipLaunchKernelGGL(single_setbcs_kernel<double>, dim3(1), dim3(64), 0, st, L, d_src, nsrc, d_ierr_bc);
        hipLaunchKernelGGL(fsm_single_kernel<double>, dim3(nwaves), dim3(64), 0, st, L);
    } else {
        hipLaunchKernelGGL(single_fill_kernel<float>, dim3(1024), dim3(256), 0, st, (float *)L.u, L.bc, np);
        hipLaunchKernelGGL(single_setbcs_kernel<float>, dim3(1), dim3(64), 0, st, L, d_src, nsrc, d_ierr_bc);
        hipLaunchKernelGGL(fsm_single_kernel<float>, dim3(nwaves), dim3(64), 0, st, L);
    }
    return hipGetLastError();
}

hipError_t fsm_single_pad(const double *src, void *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                          hipStream_t st)
{
    if (is_double)
        hipLaunchKernelGGL((single_pad_kernel<double, double>), dim3(1024), dim3(256), 0, st, src, (double *)dst, nx,
                           ny, nz, nxp, nyp, 1);
    else
        hipLaunchKernelGGL((single_pad_kernel<double, float>), dim3(1024), dim3(256), 0, st, src, (float *)dst, nx,
                           ny, nz, nxp, nyp, 1);
    return hipGetLastError();
}

hipError_t fsm_single_unpad(const void *src, double *dst, int is_double, int nx, int ny, int nz, int nxp, int nyp,
                            hipStream_t st)
{
    if (is_double)
        hipLaunchKernelGGL((single_pad_kernel<double, double>), dim3(1024), dim3(256), 0, st, (const double *)src,
                           dst, nx, ny, nz, nxp, nyp, 0);
    else
        hipLaunchKernelGGL((single_pad_kernel<float, double>), dim3(1024), dim3(256), 0, st, (const float *)src,
                           dst, nx, ny, nz, nxp, nyp, 0);
    return hipGetLastError();
}
