// capi.hip -- C-ABI of libmceik_hip.so (include/mceik.h, include/mceik_eikonal.h).
//
// Host orchestration only: argument checks with the reference's error
// behaviour, device allocation at init time, and kernel enqueueing.  The
// numerics live in fsm_kernel.hip and mcmc_kernels.hip.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "../../include/mceik.h"
#include "fsm_common.h"
#include "mcmc_common.h"
#include "fsm_single.h"
#include "rccl_rt.h"

hipError_t fsm_launch(const FsmLaunch &L, int is_double, int nwaves, hipStream_t st);
hipError_t fsm_zero_words(unsigned *p, int n, hipStream_t st);
int fsm_occupancy(const FsmLaunch &L, int is_double);
size_t fsm_launch_lds_bytes(const FsmLaunch &L, int is_double);
int fsm_launch_kind(const FsmLaunch &L, int is_double);
const char *fsm_launch_name(const FsmLaunch &L, int is_double);
hipError_t fsm_to_brick_f64(const double *src, void *dst, int dst_double, const FsmLaunch &L, int nfield, hipStream_t st);
hipError_t fsm_from_brick_f64(const void *src, int src_double, double *dst, const FsmLaunch &L, int nfield, hipStream_t st);
hipError_t fsm_from_brick_f32(const float *src, float *dst, const FsmLaunch &L, int nfield, hipStream_t st);
hipError_t fsm_to_brick_f32(const float *src, float *dst, const FsmLaunch &L, int nfield, hipStream_t st);
hipError_t mcmc_propose(const McmcDev &D, uint64_t step, hipStream_t st);
hipError_t mcmc_init_loglik(const McmcDev &D, hipStream_t st);
hipError_t mcmc_accept(const McmcDev &D, int keep_slot, hipStream_t st);
hipError_t mcmc_lpt_order(const unsigned long long *clk, int nsolve, int *order, hipStream_t st);
hipError_t l2_gridsearch_f32(int ldgrd, int ngrd, int nev, int iwantOT, float t0use, const int *ev_ptr,
                             const int *obs_row, const float *tc, const float *wt, const float *xnorm,
                             const float *test, float *t0, float *objfn, int negate, hipStream_t st);
size_t relocate_lds_bytes(int nrows, int nobs, int nev);
hipError_t relocate_lds(int ldgrd, int ngrd, int nrows, int nev, int nobs, int iwantOT, float t0use,
                        const int *ev_ptr, const int *obs_row, const float *tc, const float *wt, const float *xnorm,
                        const float *test, float *t0, float *objfn, int negate, hipStream_t st);
hipError_t gridsearch_f90(int is_double, int ldgrd, int ngrd, int nuse, int iwantOT, const int *row,
                          const void *tob, const void *w0, const void *wl, const void *test, void *logpdf,
                          hipStream_t st);
hipError_t l2_gridsearch(int ldgrd, int ngrd, int nuse, int iwantOT, double t0use, const int *use,
                         const double *tc, const double *wt, double xnorm, const double *test,
                         double *t0, double *objfn, hipStream_t st);

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "mceik_hip: %s failed: %s (%s:%d)\n", #x,                  \
                    hipGetErrorString(e_), __FILE__, __LINE__);                        \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

// ---------------------------------------------------------------------------
// Convergence threshold T: the smallest power of two with
// spacing(T^-) = T * 2^-p >= tol, p = 24 (fp32) or 53 (fp64).  A node whose
// value was >= T when it changed has moved by >= tol, so only nodes below T
// need their start-of-iteration value kept for the |u0 - u| < tol test.
static double conv_threshold(double tol, int is_double)
{
    double tolr = is_double ? tol : (double)(float)tol;
    if (!(tolr > 0.0)) return HUGE_VAL;
    int p = is_double ? 53 : 24;
    int k = (int)ceil(log2(tolr)) + p;
    while (ldexp(1.0, k - p) < tolr) k++;
    while (ldexp(1.0, k - 1 - p) >= tolr) k--;
    double T = ldexp(1.0, k);
    double big = is_double ? DBL_MAX : (double)FLT_MAX;
    return T > big ? HUGE_VAL : T;
}

static void fill_launch(FsmLaunch &L, const mceik_fsm_batch *b)
{
    memset(&L, 0, sizeof(L));
    L.nx = b->nx; L.ny = b->ny; L.nz = b->nz;
    fsm_geometry(&L, b->precision == 64 ? 8 : 4);
    L.maxit = b->maxit; L.max_sweeps = b->max_sweeps;
    L.tol = b->tol; L.h = b->h; L.x0 = b->x0; L.y0 = b->y0; L.z0 = b->z0;
    int is_double = b->precision == 64;
    double T = conv_threshold(b->tol, is_double);
    L.conv_thresh = is_double ? (T == HUGE_VAL ? DBL_MAX : T) : (T == HUGE_VAL ? (double)FLT_MAX : T);
    L.nsolve = b->nmodel * b->nstat; L.nstat = b->nstat; L.nsrc = b->nsrc;
    L.src = b->src;
    L.slow_mode = b->slow_mode;
    L.nrx = b->nrx > 0 ? b->nrx : 1; L.nry = b->nry > 0 ? b->nry : 1; L.nrz = b->nrz > 0 ? b->nrz : 1;
    L.ncx = mceik_div_up(L.nx, L.nrx); L.ncy = mceik_div_up(L.ny, L.nry); L.ncz = mceik_div_up(L.nz, L.nrz);
    L.magic_rx = ((1u << 20) + L.nrx - 1) / L.nrx;
    L.magic_ry = ((1u << 20) + L.nry - 1) / L.nry;
    L.magic_rz = ((1u << 20) + L.nrz - 1) / L.nrz;
    L.ev_node = b->ev_node; L.nev = b->nev; L.ttab = b->ttab; L.ev_frac = b->ev_frac;
    L.model_phase = b->slow_mode == 1 ? b->model_phase : nullptr;
    L.skip = b->skip;
    L.solve_count = b->solve_count;
    L.nphase = b->nphase > 0 ? b->nphase : 1;
    // LDS cell cache when every z-block's cells fit (2 x 2 x 8 at nref = 4, kb = 4)
    {
        auto span = [](int a, int e, int nr) { return e / nr - a / nr + 1; };
        int mx = 0, my = 0, mz = 0;
        for (int t = 0; t < L.ntx; t++) {
            int v = span(t * 8, t * 8 + 7 < L.nx - 1 ? t * 8 + 7 : L.nx - 1, L.nrx); mx = v > mx ? v : mx;
        }
        for (int t = 0; t < L.nty; t++) {
            int v = span(t * 8, t * 8 + 7 < L.ny - 1 ? t * 8 + 7 : L.ny - 1, L.nry); my = v > my ? v : my;
        }
        for (int t = 0; t < L.nzk; t++) {
            int a = t * L.kb * 8, e = a + L.kb * 8 - 1 < L.nz - 1 ? a + L.kb * 8 - 1 : L.nz - 1;
            int v = span(a, e, L.nrz); mz = v > mz ? v : mz;
        }
        L.ccb = mx * my * mz;
        L.cell_cache = b->slow_mode == 1 && L.ccb <= MCEIK_CC_MAX && L.nx < 4096 && L.ny < 4096 && L.nz < 4096;
        if (!L.cell_cache) L.ccb = 0;
    }
    L.fast_sqrt = b->fast_sqrt;
    L.niter = b->niter; L.ierr = b->ierr;
    L.iter_total = b->iter_total;
    L.visit_stats = b->visit_stats;
    L.solve_order = b->solve_order;
    L.solve_clock = b->solve_clock;
    L.max_waves = b->max_waves;
    L.traffic = b->traffic;
    L.step_z = b->step_z;
}

static int g_device_cus = 0;

static int device_cus()
{
    if (g_device_cus == 0) {
        int dev = 0;
        hipDeviceProp_t p;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
            g_device_cus = p.multiProcessorCount;
        else
            g_device_cus = 256;
    }
    return g_device_cus;
}

// Scratch budget for the per-wave u / u0 fields, fixed at the first call (so
// workspace_bytes and batch_solve agree): MCEIK_FSM_WS_GB if set, else the
// device memory free at that moment less an 8-GiB margin (the sampler's other
// arrays, the caller's tensors), at most 80% of the total (230 GB on a 288-GB
// MI355X).  A sampler with several pipes splits it between them (pipes_setup).
static size_t ws_budget_bytes()
{
    static size_t budget = 0;
    if (budget == 0) {
        const char *e = getenv("MCEIK_FSM_WS_GB");
        double gb = e ? atof(e) : 0.0;
        if (gb > 0.0) {
            budget = (size_t)(gb * 1073741824.0);
        } else {
            size_t fr = 0, tot = 0;
            const size_t margin = (size_t)8 << 30;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot) {
                // at 256^3 (128 MiB of u + u0 per wave): 6.7 waves/CU
                budget = tot / 5 * 4;
                const size_t avail = fr > 2 * margin ? fr - margin : fr / 2;
                if (avail < budget) budget = avail;
            } else {
                budget = (size_t)96 << 30;
            }
        }
    }
    return budget;
}

// Waves a launch keeps resident (one solve each): occupancy x CUs, at most nsolve.
static int batch_waves(const FsmLaunch &L, int is_double)
{
    int per_cu = fsm_occupancy(L, is_double);
    if (per_cu < 1) per_cu = 1;
    // tuning knob: fewer resident waves per CU (L2 working set experiments)
    static const int env_cap = [] { const char *e = getenv("MCEIK_WAVES_PER_CU"); return e ? atoi(e) : 0; }();
    if (env_cap > 0 && env_cap < per_cu) per_cu = env_cap;
    long w = (long)per_cu * device_cus();
    if (L.max_waves > 0 && w > L.max_waves) w = L.max_waves;
    if (w > L.nsolve) w = L.nsolve;
    static const bool report = getenv("MCEIK_LAUNCH_REPORT") != nullptr;
    if (report)
        fprintf(stderr, "mceik fsm launch: %d-z steps, %d waves/CU (occupancy), %ld resident waves, %zu B LDS per wave\n",
                fsm_launch_kind(L, is_double), per_cu, w, fsm_launch_lds_bytes(L, is_double));
    return (int)(w < 1 ? 1 : w);
}

// Waves of a batch before the scratch budget caps them.
static int fsm_batch_waves_uncapped(const mceik_fsm_batch *b)
{
    FsmLaunch L;
    fill_launch(L, b);
    return batch_waves(L, b->precision == 64);
}

// Workspace: [8 queue heads, 1 KiB][slow brick copy (mode 0)][u scratch][u0 scratch]
struct WsLayout {
    size_t counter, slow, u, u0, zf, total;
    int nwaves;
};

static WsLayout ws_layout(const mceik_fsm_batch *b)
{
    FsmLaunch L;
    fill_launch(L, b);
    int is_double = b->precision == 64;
    size_t es = is_double ? 8 : 4;
    WsLayout w;
    w.nwaves = batch_waves(L, is_double);
    // the held stream's per-wave z-face copies: read only by the 16-z kernel (the 8-z / fp64
    // instances read the z-boundary nodes from the field)
    const size_t zfw = fsm_launch_kind(L, is_double) == 16 ? zf_bytes(L, es) : 0;
    // Every resident wave owns a u and a u0 scratch field: cap the waves so the
    // scratch stays within a fixed budget (deterministic across calls; 256^3
    // fp32 fields are 67 MB, 2048 waves would need 275 GB).  Waves then take
    // several solves each from the queue.
    {
        const size_t per_wave = 2 * L.field_elems * es + zfw;
        const long cap = (long)(ws_budget_bytes() / (per_wave ? per_wave : 1));
        if (cap >= 1 && w.nwaves > cap) w.nwaves = (int)cap;
    }
    w.counter = 0;
    w.slow = 1024;
    size_t slow_bytes = b->slow_mode == 0 ? (size_t)b->nmodel * L.field_elems * es : 0;
    w.u = w.slow + ((slow_bytes + 255) & ~(size_t)255);
    size_t nu = b->u_out ? (size_t)L.nsolve : (size_t)w.nwaves;
    w.u0 = w.u + nu * L.field_elems * es;
    w.zf = w.u0 + (size_t)w.nwaves * L.field_elems * es;          // the held stream's z-face copies
    w.total = w.zf + (size_t)w.nwaves * zfw;
    return w;
}

extern "C" size_t mceik_fsm_workspace_bytes(const mceik_fsm_batch *b)
{
    return ws_layout(b).total;
}

extern "C" int mceik_fsm_step_z(const mceik_fsm_batch *b)
{
    if (!b) return 0;
    FsmLaunch L;
    fill_launch(L, b);
    return fsm_launch_kind(L, b->precision == 64);
}

extern "C" const char *mceik_fsm_kernel_name(const mceik_fsm_batch *b)
{
    if (!b) return "";
    FsmLaunch L;
    fill_launch(L, b);
    return fsm_launch_name(L, b->precision == 64);
}

extern "C" size_t mceik_fsm_lds_bytes(const mceik_fsm_batch *b)
{
    if (!b) return 0;
    FsmLaunch L;
    fill_launch(L, b);
    return fsm_launch_lds_bytes(L, b->precision == 64);
}

extern "C" double mceik_fsm_bytes_per_node_sweep(const mceik_fsm_batch *b)
{
    // u read + u write per node visit; slowness read once per node per model
    // pass, shared by the nstat stations of that model (SURVEY s.8d: N(8+4/S)).
    double es = b->precision == 64 ? 8.0 : 4.0;
    double s = b->slow_mode == 0 ? es : 4.0 / ((double)b->nrx * b->nry * b->nrz);
    return 2.0 * es + s / (b->nstat > 0 ? b->nstat : 1);
}

// The sampler's multi-step launch (FsmLaunch mc_*): not part of the public batch.
#define MCEIK_MC_CHUNK 64        // steps per multi-step launch (bounds one kernel's duration)
struct McmcExt {
    const void *dev;             // device copy of the sampler's McmcDev
    unsigned *sync;              // MC_SYNC_WORDS(nchains) words, zeroed here before the launch (but the last)
    unsigned spin_limit;
    int step0, nsteps, nburn, keepk, maxs, nkept0;
};

static int fsm_batch_solve_impl(const mceik_fsm_batch *b, void *workspace, size_t workspace_bytes, void *stream,
                                const McmcExt *ext);

extern "C" int mceik_fsm_batch_solve(const mceik_fsm_batch *b, void *workspace, size_t workspace_bytes,
                                     void *stream)
{
    return fsm_batch_solve_impl(b, workspace, workspace_bytes, stream, nullptr);
}

static int fsm_batch_solve_impl(const mceik_fsm_batch *b, void *workspace, size_t workspace_bytes, void *stream,
                                const McmcExt *ext)
{
    if (!b || b->nx < 2 || b->ny < 2 || b->nz < 2 || b->nx > 4096 || b->ny > 4096 || b->nz > 4096 ||
        b->nsrc < 1 ||
        b->nmodel < 1 || b->nstat < 1 || !(b->precision == 32 || b->precision == 64)) {
        fprintf(stderr, "mceik_fsm_batch_solve: invalid batch description\n");
        return 1;
    }
    if (b->slow_mode == 1 && b->precision != 32 && b->precision != 64) return 1;
    WsLayout w = ws_layout(b);
    {
        FsmLaunch G;
        fill_launch(G, b);
        if (G.field_elems * (b->precision == 64 ? 8 : 4) >= (size_t)1 << 31) {
            fprintf(stderr, "mceik_fsm_batch_solve: one travel-time field must stay below 2 GiB\n");
            return 1;
        }
        if (fsm_launch_lds_bytes(G, b->precision == 64) > MCEIK_MAX_LDS) {
            fprintf(stderr, "mceik_fsm_batch_solve: %d x %d x %d z-blocks exceed the LDS block tables\n", G.ntx, G.nty,
                    G.nzk);
            return 1;
        }
        // the held stream's 16-bit sweep clocks (fsm_hold.h hold_clock_bound)
        const bool held = fsm_launch_kind(G, b->precision == 64) == 16 || fsm_compact_layout(G, 8);
        const int infl = fsm_launch_kind(G, b->precision == 64) == 16 ? fsm16_geo(G).infl : G.infl;
        if (held && hold_clock_bound(G.nblocks, infl) >= 65536) {
            fprintf(stderr, "mceik_fsm_batch_solve: %d z-blocks overflow the held stream's 16-bit clocks\n", G.nblocks);
            return 1;
        }
    }
    if (!workspace || workspace_bytes < w.total) {
        fprintf(stderr, "mceik_fsm_batch_solve: workspace too small (%zu < %zu)\n", workspace_bytes, w.total);
        return 1;
    }
    if (b->skip && b->u_out) {
        // a skipped solve never sweeps, so its u slot would hold stale workspace
        fprintf(stderr, "mceik_fsm_batch_solve: skip and u_out cannot be combined (a skipped solve has no field)\n");
        return 1;
    }
    hipStream_t st = (hipStream_t)stream;
    int is_double = b->precision == 64;
    FsmLaunch L;
    fill_launch(L, b);
    char *ws = (char *)workspace;
    L.counter = (unsigned *)(ws + w.counter);
    HIPCHK(fsm_zero_words(L.counter, 256, st));          // 8 queue heads, 128 B apart (graph-safe)
    if (b->slow_mode == 0) {
        void *sb = ws + w.slow;
        if (is_double)
            HIPCHK(fsm_to_brick_f64((const double *)b->slow, sb, 1, L, b->nmodel, st));
        else
            HIPCHK(fsm_to_brick_f32((const float *)b->slow, (float *)sb, L, b->nmodel, st));
        L.slow = sb;
    } else {
        L.slow = b->slow;
    }
    L.u = ws + w.u;
    L.u0 = ws + w.u0;
    L.zf = ws + w.zf;
    L.slot_per_solve = b->u_out ? 1 : 0;
    if (ext) {
        if (is_double || fsm_launch_kind(L, 0) != 16 || b->solve_order || b->u_out) return 1;
        L.mc_dev = ext->dev;
        L.mc_sync = ext->sync;
        L.mc_spin_limit = ext->spin_limit;
        L.mc_step0 = ext->step0; L.mc_nsteps = ext->nsteps;
        L.mc_nburn = ext->nburn; L.mc_keepk = ext->keepk; L.mc_maxs = ext->maxs; L.mc_nkept0 = ext->nkept0;
        // the broken-queue flag (last word) persists until the sampler reports it
        HIPCHK(fsm_zero_words(ext->sync, MC_SYNC_WORDS(L.nsolve / L.nstat) - 1, st));
    }
    HIPCHK(fsm_launch(L, is_double, w.nwaves, st));
    if (b->u_out) {
        if (is_double) HIPCHK(fsm_from_brick_f64(L.u, 1, (double *)b->u_out, L, L.nsolve, st));
        else HIPCHK(fsm_from_brick_f32((const float *)L.u, (float *)b->u_out, L, L.nsolve, st));
    }
    return 0;
}

// The plain-argument batched extension SURVEY s.8b names: nmodels x
// nstations single-source solves (fp32, the sampler's arithmetic) of
// per-node slowness fields in one call.  Pointers may be host or device
// memory (host arrays are staged); synchronous.  Solve m*nstations + s
// uses model m and station s.
static bool is_device_ptr(const void *p)
{
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

extern "C" int eikonal3d_batch_solve(int nmodels, int nstations, int nx, int ny, int nz, double h, double x0,
                                     double y0, double z0, int maxit, double tol, const double *src,
                                     const float *slow, float *u, int *niter, int *ierr)
{
    if (nmodels < 1 || nstations < 1 || !src || !slow || !u) return 1;
    const size_t n = (size_t)nx * ny * nz, nsolve = (size_t)nmodels * nstations;
    mceik_fsm_batch b;
    memset(&b, 0, sizeof(b));
    b.nx = nx; b.ny = ny; b.nz = nz; b.h = h; b.x0 = x0; b.y0 = y0; b.z0 = z0;
    b.maxit = maxit; b.tol = tol; b.precision = 32;
    b.nmodel = nmodels; b.nstat = nstations; b.nsrc = 1; b.slow_mode = 0; b.max_sweeps = -1;
    std::vector<void *> tmp;
    auto stage = [&](const void *p, size_t bytes, bool in) -> void * {
        if (is_device_ptr(p)) return const_cast<void *>(p);
        void *d = nullptr;
        if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
        tmp.push_back(d);
        if (in && hipMemcpy(d, p, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    };
    int rc = 0;
    void *d_src = stage(src, (size_t)nstations * 4 * sizeof(double), true);
    void *d_slow = stage(slow, (size_t)nmodels * n * sizeof(float), true);
    void *d_u = stage(u, nsolve * n * sizeof(float), false);
    void *d_it = niter ? stage(niter, nsolve * sizeof(int), false) : nullptr;
    void *d_ie = ierr ? stage(ierr, nsolve * sizeof(int), false) : nullptr;
    void *ws = nullptr;
    if (!d_src || !d_slow || !d_u || (niter && !d_it) || (ierr && !d_ie)) rc = -1;
    if (!rc) {
        b.src = (const double *)d_src; b.slow = d_slow; b.u_out = d_u;
        b.niter = (int *)d_it; b.ierr = (int *)d_ie;
        const size_t wsb = mceik_fsm_workspace_bytes(&b);
        if (hipMalloc(&ws, wsb) != hipSuccess) rc = -1;
        else rc = mceik_fsm_batch_solve(&b, ws, wsb, nullptr);
        if (!rc && hipDeviceSynchronize() != hipSuccess) rc = -1;
    }
    if (!rc && d_u != u) rc = hipMemcpy(u, d_u, nsolve * n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess;
    if (!rc && niter && d_it != niter) rc = hipMemcpy(niter, d_it, nsolve * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess;
    if (!rc && ierr && d_ie != ierr) rc = hipMemcpy(ierr, d_ie, nsolve * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess;
    if (ws) hipFree(ws);
    for (void *p : tmp) hipFree(p);
    return rc;
}

extern "C" int mceik_memcpy(void *dst, const void *src, size_t bytes, int kind)
{
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIPCHK(hipMemcpy(dst, src, bytes, k));
    return 0;
}

// ---------------------------------------------------------------------------
// Drop-in single-solve entry points: the serial driver (fsm3d.f90:1968-2052)
// and the MPI variant eikonal3d_initialize / _solve / _finalize
// (fsm3d.f90:1583-1929).  One solve at a time runs on the whole GPU
// (fsm_single.hip).  The reference's job-1 state (SAVE lstruct, linit,
// fsm3d.f90:1985-1988) becomes the device state below: the brick level
// order (MAKE_LEVEL_STRUCT at brick granularity) and every device buffer,
// allocated at init and freed at finalize, so a solve call only copies the
// model in, runs, and copies the field out.
struct SingleState {
    int init;
    int nx, ny, nz, maxit_cap, nsrc_cap;
    int is_double;
    SingleLaunch L;
    void *mem;                   // one allocation: fields, flags, tables
    double *dense, *src;         // fp64 x-fastest staging [n], sources [nsrc][4]
    int *ierr_bc;
    int nwaves;
    int bcfail;                  // the last solve stopped in SETBCS
    hipStream_t st;
    // MPI-variant parameters (eikonal3d_initialize)
    int iverb, maxit;
    double x0, y0, z0, h, tol;
    BlockDecomp D;               // the reference's block decomposition (more than one block: blocks_solve)
    double *snap;                // ghost copies: u at the start of the sweep (padded layout)
    unsigned *d_count;           // unconverged-node count
};
static SingleState g_single[3];          // [0] serial fp32, [1] serial fp64, [2] MPI variant (fp64)

// Frees the device state; the caller's parameters (init flag, the MPI
// variant's eikonal3d_initialize arguments and decomposition) survive.
static void single_free(SingleState &S)
{
    if (S.snap) hipFree(S.snap);
    if (S.d_count) hipFree(S.d_count);
    if (S.mem) hipFree(S.mem);
    if (S.st) hipStreamDestroy(S.st);
    const SingleState keep = S;
    memset(&S, 0, sizeof(S));
    S.init = keep.init;
    S.iverb = keep.iverb; S.maxit = keep.maxit;
    S.x0 = keep.x0; S.y0 = keep.y0; S.z0 = keep.z0; S.h = keep.h; S.tol = keep.tol;
    S.D = keep.D;
}

// Ghost snapshot and counters of the block-decomposed solve (allocated once
// per grid; single_alloc reallocations drop them).
static int blocks_buffers(SingleState &S)
{
    const size_t np = (size_t)S.L.nxp * S.L.nyp * S.L.nzp;
    if (!S.snap && hipMalloc(&S.snap, np * 8) != hipSuccess) { S.snap = nullptr; return 1; }
    if (!S.d_count && hipMalloc(&S.d_count, 16) != hipSuccess) { S.d_count = nullptr; return 1; }
    return 0;
}

// Device buffers of a solve on nx x ny x nz (maxit iterations, nsrc sources).
static int single_alloc(SingleState &S, int is_double, int nx, int ny, int nz, int maxit, int nsrc)
{
    if (S.mem && S.is_double == is_double && S.nx == nx && S.ny == ny && S.nz == nz && maxit <= S.maxit_cap &&
        nsrc <= S.nsrc_cap)
        return 0;
    const int keep = S.init;
    single_free(S);
    S.init = keep;
    if (nx < 1 || ny < 1 || nz < 1 || (long)nx * ny * nz >= (1L << 31)) return 1;
    SingleLaunch &L = S.L;
    L.nx = nx; L.ny = ny; L.nz = nz;
    L.gx = nx; L.gy = ny; L.gz = nz;             // the whole grid (rank_alloc: a box of it)
    L.nbx = mceik_div_up(nx, 8); L.nby = mceik_div_up(ny, 8); L.nbz = mceik_div_up(nz, 8);
    if (L.nbx > 1024 || L.nby > 1024 || L.nbz > 1024) return 1;
    L.nxp = 8 * L.nbx; L.nyp = 8 * L.nby; L.nzp = 8 * L.nbz;
    L.nb = L.nbx * L.nby * L.nbz;
    if ((size_t)L.nxp * L.nyp * L.nzp * (is_double ? 8 : 4) >= ((size_t)1 << 31)) return 1;   // 32-bit offsets
    const int mcap = maxit > 0 ? maxit : 1, scap = nsrc > 0 ? nsrc : 1;
    const size_t es = is_double ? 8 : 4, np = (size_t)L.nxp * L.nyp * L.nzp, n = (size_t)nx * ny * nz;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    size_t off[12], o = 0;
    off[0] = o; o += al(np * es);                      // u
    off[1] = o; o += al(np * es);                      // u0
    off[2] = o; o += al(np * es);                      // slow
    off[3] = o; o += al(np);                           // bc
    off[4] = o; o += al((size_t)L.nb * 4);             // border
    off[5] = o; o += al((size_t)L.nb * 4);             // done
    off[6] = o; o += al((size_t)(32 + mcap) * 4);      // ctl
    off[7] = o; o += al((size_t)mcap * 8);             // arrive
    off[8] = o; o += al((size_t)mcap * 4);             // ierr_it
    off[9] = o; o += al(n * 8);                        // dense fp64 staging
    off[10] = o; o += al((size_t)scap * 32);           // sources
    off[11] = o; o += al(16);                          // SETBCS ierr
    if (hipMalloc(&S.mem, o) != hipSuccess) { S.mem = nullptr; return 1; }
    char *m = (char *)S.mem;
    L.u = m + off[0]; L.u0 = m + off[1]; L.slow = m + off[2]; L.bc = (unsigned char *)(m + off[3]);
    L.border = (const int *)(m + off[4]); L.done = (unsigned *)(m + off[5]); L.ctl = (unsigned *)(m + off[6]);
    L.arrive = (unsigned long long *)(m + off[7]); L.ierr_it = (int *)(m + off[8]);
    S.dense = (double *)(m + off[9]); S.src = (double *)(m + off[10]); S.ierr_bc = (int *)(m + off[11]);
    L.bcerr = S.ierr_bc;
    // brick level order in sweep coordinates (any order inside a level)
    std::vector<int> ord;
    ord.reserve(L.nb);
    for (int lev = 0; lev <= L.nbx + L.nby + L.nbz - 3; lev++)
        for (int bz = 0; bz < L.nbz; bz++)
            for (int by = 0; by < L.nby; by++) {
                const int bx = lev - bz - by;
                if (bx >= 0 && bx < L.nbx) ord.push_back(bx | (by << 10) | (bz << 20));
            }
    if ((int)ord.size() != L.nb ||
        hipMemcpy((void *)L.border, ord.data(), ord.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess) {
        single_free(S);
        return 1;
    }
    // persistent waves: every wave of the grid is resident (tasks are taken
    // in dependency order, so a waiting wave only ever waits for running ones)
    static const int wpc = [] { const char *e = getenv("MCEIK_SINGLE_WAVES_PER_CU"); return e ? atoi(e) : 2; }();
    int occ = fsm_single_occupancy(is_double);
    S.nwaves = device_cus() * std::max(1, std::min(wpc, occ));
    S.is_double = is_double; S.nx = nx; S.ny = ny; S.nz = nz; S.maxit_cap = mcap; S.nsrc_cap = scap;
    return 0;
}

// SETBCS + FSM of one model on the GPU; slow/u: host fp64 [nx*ny*nz].  Returns
// the reference's ierr (1: SETBCS, fsm3d.f90:736-753; else the ierr of node
// (1,1,1) in the last sweep, :78-82) or -1 on a device failure.
static int single_solve(SingleState &S, int maxit, int nsrc, double tol, double h, double x0, double y0, double z0,
                        const double *ts, const double *xs, const double *ys, const double *zs, const double *slow,
                        double *u, int *niter_out)
{
    SingleLaunch &L = S.L;
    const size_t n = (size_t)L.nx * L.ny * L.nz;
    L.maxit = maxit; L.tol = tol; L.h = h; L.x0 = x0; L.y0 = y0; L.z0 = z0;
    std::vector<double> src((size_t)nsrc * 4);
    for (int k = 0; k < nsrc; k++) {
        src[k * 4 + 0] = ts[k]; src[k * 4 + 1] = xs[k]; src[k * 4 + 2] = ys[k]; src[k * 4 + 3] = zs[k];
    }
    const int mcap = maxit > 0 ? maxit : 1;
    std::vector<unsigned> ctl(32 + mcap);
    std::vector<int> ierr_it(mcap);
    int ierr_bc = 0;
    hipStream_t st = S.st;
    if (hipMemcpyAsync(S.dense, slow, n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(S.src, src.data(), src.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        fsm_single_pad(S.dense, (void *)L.slow, S.is_double, L.nx, L.ny, L.nz, L.nxp, L.nyp, st) != hipSuccess ||
        hipMemsetAsync(L.done, 0, (size_t)L.nb * 4, st) != hipSuccess ||
        hipMemsetAsync(L.ctl, 0, (size_t)(32 + mcap) * 4, st) != hipSuccess ||
        hipMemsetAsync(L.arrive, 0, (size_t)mcap * 8, st) != hipSuccess ||
        hipMemsetAsync(L.ierr_it, 0, (size_t)mcap * 4, st) != hipSuccess ||
        fsm_single_solve(L, S.is_double, S.src, nsrc, S.ierr_bc, S.nwaves, st) != hipSuccess ||
        fsm_single_unpad(L.u, S.dense, S.is_double, L.nx, L.ny, L.nz, L.nxp, L.nyp, st) != hipSuccess ||
        hipMemcpyAsync(u, S.dense, n * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(ctl.data(), L.ctl, ctl.size() * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(ierr_it.data(), L.ierr_it, ierr_it.size() * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&ierr_bc, S.ierr_bc, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return -1;
    if (ctl[1] != 0) {
        std::vector<unsigned> done(L.nb);
        std::vector<unsigned long long> arr(mcap);
        hipMemcpy(done.data(), L.done, done.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(arr.data(), L.arrive, arr.size() * 8, hipMemcpyDeviceToHost);
        unsigned dmin = ~0u, dmax = 0;
        for (unsigned d : done) { dmin = std::min(dmin, d); dmax = std::max(dmax, d); }
        fprintf(stderr, "mceik_hip: single-solve schedule timed out (code %u; waits timed out: deps %u, "
                        "iteration %u; tasks taken %u, nb %d, done %u..%u, arrivals it0 %llu/%llu it1 %llu, "
                        "decisions %u %u %u)\n", ctl[1], ctl[3], ctl[4], ctl[0], L.nb, dmin, dmax,
                arr[0] & 0xffffffffull, arr[0] >> 32, mcap > 1 ? arr[1] & 0xffffffffull : 0ull, ctl[32],
                mcap > 1 ? ctl[33] : 0u, mcap > 2 ? ctl[34] : 0u);
        return -1;
    }
    S.bcfail = ierr_bc != 0;
    if (ierr_bc) {
        if (niter_out) *niter_out = 0;
        return 1;
    }
    int niter = maxit > 0 ? maxit : 0;
    for (int it = 0; it < maxit; it++)
        if (ctl[32 + it] == 2) { niter = it + 1; break; }
    if (niter_out) *niter_out = niter;
    return niter > 0 ? ierr_it[niter - 1] : 0;
}

static void serial_driver(int is_double, const int *job, const int *iverb, const int *maxit,
                          const int *nsrc, const int *nx, const int *ny, const int *nz,
                          const double *tol, const double *h, const double *x0, const double *y0,
                          const double *z0, const double *ts, const double *xs, const double *ys,
                          const double *zs, const double *slow, double *u, int *ierr)
{
    SingleState &S = g_single[is_double];
    *ierr = 0;
    if (*job == 1) {
        if (S.init) { printf(" eikonal3d_serial_driver: Already initialized!\n"); *ierr = 1; return; }
        if (*iverb > 0) printf(" eikonal3d_serial_driver: Generating levels...\n");
        if (single_alloc(S, is_double, *nx, *ny, *nz, *maxit, *nsrc)) {
            printf(" eikonal3d_serial_driver: Error generating level structure\n");
            *ierr = 1;
            return;
        }
        S.init = 1;
        return;
    }
    if (*job != 2) {
        if (!S.init) printf(" eikonal3d_serial_driver: Never initialized!\n");
        single_free(S);
        S.init = 0;
        return;
    }
    if (!S.init) { printf(" eikonal3d_serial_driver: Solver not initalized!\n"); *ierr = 1; return; }
    if (*nsrc < 1) {
        printf(" eikonal3d_serial_driver: nsrc must be >= 1\n");
        *ierr = 1;
        return;
    }
    // a solve on another grid than job 1's (the reference's level structure
    // would not match): reallocate rather than fail
    if (single_alloc(S, is_double, *nx, *ny, *nz, *maxit, *nsrc)) {
        printf(" eikonal3d_serial_driver: device allocation failed\n");
        *ierr = 1;
        return;
    }
    if (*iverb > 0) printf(" eikonal3d_serial_driver: Setting boundary conditions...\n");
    const int rc = single_solve(S, *maxit, *nsrc, *tol, *h, *x0, *y0, *z0, ts, xs, ys, zs, slow, u, nullptr);
    if (rc < 0) {
        printf(" eikonal3d_serial_driver: device failure\n");
        *ierr = 1;
        return;
    }
    *ierr = rc;
    if (S.bcfail) printf(" eikonal3d_serial_driver: Error setting boundary conditions\n");
    else if (rc != 0) printf(" eikonal3d_serial_driver: Error solving eikonal equation\n");
}

extern "C" void eikonal3d_serial_driver(const int *job, const int *iverb, const int *maxit, const int *nsrc,
                                        const int *nx, const int *ny, const int *nz, const double *tol,
                                        const double *h, const double *x0, const double *y0, const double *z0,
                                        const double *ts, const double *xs, const double *ys, const double *zs,
                                        const double *slow, double *u, int *ierr)
{
    serial_driver(1, job, iverb, maxit, nsrc, nx, ny, nz, tol, h, x0, y0, z0, ts, xs, ys, zs, slow, u, ierr);
}

extern "C" void eikonal3d_serial_driver_sp(const int *job, const int *iverb, const int *maxit, const int *nsrc,
                                           const int *nx, const int *ny, const int *nz, const double *tol,
                                           const double *h, const double *x0, const double *y0, const double *z0,
                                           const double *ts, const double *xs, const double *ys, const double *zs,
                                           const double *slow, double *u, int *ierr)
{
    serial_driver(0, job, iverb, maxit, nsrc, nx, ny, nz, tol, h, x0, y0, z0, ts, xs, ys, zs, slow, u, ierr);
}

// MPI variant (fsm3d.f90:1583-1929) on one GPU.  The reference decomposes the
// grid over ndivx*ndivy*ndivz ranks of `comm` and gathers u on rank 0; here
// the whole grid lives on the calling process's GPU and `comm` is not used,
// but the decomposition is: with more than one block the solve runs the
// reference's block-decomposed iteration (blocks_solve: per sweep every block
// sweeps its own nodes against ghost copies refreshed after the sweep), so u,
// the iteration count and ierr are bitwise those of the reference's run with
// one MPI rank per block (tests/golden/blocks_mpi.npz); one block is the
// serial driver's solve.  Collective semantics are kept by the reference's own
// convention: the master passes the full arrays (n = nx*ny*nz) and gets the
// travel times; every other rank passes n < nx*ny*nz (the reference's callers
// use n = 1, fsm3d.f90:2102-2106) and returns at once with ierr = 0.
// The block-decomposed solve of the MPI variant on one GPU (EIKONAL3D_FSM_MPI,
// fsm3d.f90:103-222; fsm_single.hip block_sweep_kernel): SETBCS, then per
// iteration 8 sweeps, each preceded by the ghost snapshot (the state every
// block's EIKONAL_EXCHANGE leaves), then the convergence count.  Returns the
// reference's ierr (rank 0's) or -1 on a device failure.
static int blocks_solve(SingleState &S, int nsrc, const double *ts, const double *xs, const double *ys,
                        const double *zs, const double *slow, double *u, int *niter_out)
{
    SingleLaunch &L = S.L;
    const size_t n = (size_t)L.nx * L.ny * L.nz, np = (size_t)L.nxp * L.nyp * L.nzp;
    L.maxit = S.maxit; L.tol = S.tol; L.h = S.h; L.x0 = S.x0; L.y0 = S.y0; L.z0 = S.z0;
    std::vector<double> src((size_t)nsrc * 4);
    for (int k = 0; k < nsrc; k++) {
        src[k * 4 + 0] = ts[k]; src[k * 4 + 1] = xs[k]; src[k * 4 + 2] = ys[k]; src[k * 4 + 3] = zs[k];
    }
    hipStream_t st = S.st;
    int ierr_bc = 0, ierr = 0, niter = 0;
    if (hipMemcpyAsync(S.dense, slow, n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(S.src, src.data(), src.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        fsm_single_pad(S.dense, (void *)L.slow, 1, L.nx, L.ny, L.nz, L.nxp, L.nyp, st) != hipSuccess ||
        fsm_single_setbcs(L, S.src, nsrc, S.ierr_bc, st) != hipSuccess ||
        hipMemcpyAsync(&ierr_bc, S.ierr_bc, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return -1;
    S.bcfail = ierr_bc != 0;
    int *d_ierr = (int *)(S.d_count + 1);
    for (int k = 1; k <= S.maxit && !ierr_bc; k++) {
        niter = k;
        if (hipMemcpyAsync(L.u0, L.u, np * 8, hipMemcpyDeviceToDevice, st) != hipSuccess) return -1;
        for (int g = 0; g < 8; g++)
            if (hipMemcpyAsync(S.snap, L.u, np * 8, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipMemsetAsync(d_ierr, 0, 4, st) != hipSuccess ||
                fsm_block_sweep(L, S.D, S.snap, g, d_ierr, st) != hipSuccess)
                return -1;
        unsigned count = 0;
        if (hipMemsetAsync(S.d_count, 0, 4, st) != hipSuccess ||
            fsm_block_unconverged(L, BlockBox{{0, 0, 0}, {L.nx, L.ny, L.nz}}, S.tol, S.d_count, st) != hipSuccess ||
            hipMemcpyAsync(&count, S.d_count, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(&ierr, d_ierr, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return -1;
        if (count == 0) break;
    }
    if (fsm_single_unpad(L.u, S.dense, 1, L.nx, L.ny, L.nz, L.nxp, L.nyp, st) != hipSuccess ||
        hipMemcpyAsync(u, S.dense, n * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return -1;
    if (niter_out) *niter_out = niter;
    return ierr_bc ? 1 : ierr;
}

// MPI of the calling process, resolved at run time (csrc/mpi_rt.c): -1 = the
// caller runs no MPI (a single process: rank 0 of one).
extern "C" int mceik_mpi_rank(int fcomm);
extern "C" int mceik_mpi_size(int fcomm);
extern "C" int mceik_mpi_bcast_int(int fcomm, int *v, int n, int root);
extern "C" int mceik_mpi_bcast_double(int fcomm, double *v, int n, int root);
extern "C" int mceik_mpi_allreduce_int(int fcomm, int *v, int n, int op);
extern "C" int mceik_mpi_allgather_bytes(int fcomm, const void *mine, void *all, int nbytes);
extern "C" int mceik_mpi_exchange_double(int fcomm, int nmsg, const int *dir, const int *peer, const int *tag,
                                         double *const *buf, const int *count);

// ---- the MPI variant across ranks: one block per rank -----------------------
// With as many ranks in comm as blocks (the reference's own layout,
// fsm3d.f90:1069-1074: rank r owns block r, x fastest, MPIUTILS_GRD2IJK), the
// solve is distributed as the reference's EIKONAL3D_FSM_MPI: every rank sweeps
// the block it owns on its own GPU, swaps the one-node face layers with the
// ranks owning the adjacent blocks after every sweep (EIKONAL_EXCHANGE,
// :971-1046; only the first ghost layer is ever read), sums the unconverged
// nodes over ranks after every iteration (:198-211) and sends its block to the
// master at the end (EIKONAL_GATHER_TRAVELTIMES).  Each rank keeps the grid in
// the padded global layout (nodes outside its block and its faces stay at their
// SETBCS values; a 512^3 fp64 field is 1 GiB of the 288 GB), so the sweep is
// the one-GPU block kernel restricted to block b0 with the ghost snapshot
// being u itself.  Transport of the face layers: RCCL device to device when
// every rank has a GPU of its own (xGMI), host-staged MPI when ranks share a
// GPU (RCCL takes one rank per GPU).  Default MPI; MCEIK_HALO=rccl|auto opts in.
struct RankHalo {
    int on;                      // the solve runs one block per rank
    int fcomm, rank, nranks;
    int gn[3];                   // the global grid
    BlockBox own;                // the block this rank owns (= its rank)
    BlockBox hbox;               // the nodes this rank holds: its block and the ghost layer
    int kind;                    // 1: host-staged MPI, 2: RCCL
    int peer[6], tag_send[6], tag_recv[6];
    BoxList send, recv;          // faces sent / received, in the same face order
    double *d_buf;               // device: send faces, then receive faces
    double *h_buf;               // pinned host staging (MPI transport)
    ncclComm_t nc;
};
static RankHalo g_halo;

// Block b of the decomposition (fsm3d.f90:1086-1098; ext may be <= 0 when
// there are more blocks than nodes, which the reference rejects).
static void decomp_block(const BlockDecomp &D, const int nn[3], int b, int lo[3], int ext[3])
{
    const int bi[3] = {b % D.nd[0], (b / D.nd[0]) % D.nd[1], b / (D.nd[0] * D.nd[1])};
    for (int a = 0; a < 3; a++) {
        lo[a] = D.step[a] * bi[a];
        const int hi = bi[a] + 1 == D.nd[a] ? nn[a] - 1 : D.step[a] * (bi[a] + 1) - 1;
        ext[a] = hi - lo[a] + 1;
    }
}

// The reference's check that the blocks tile the grid (fsm3d.f90:1105-1112).
static bool decomp_tiles(const BlockDecomp &D, const int nn[3])
{
    long long tot = 0;
    for (int b = 0; b < D.nd[0] * D.nd[1] * D.nd[2]; b++) {
        int lo[3], ext[3];
        decomp_block(D, nn, b, lo, ext);
        tot += (long long)ext[0] * ext[1] * ext[2];
    }
    return tot == (long long)nn[0] * nn[1] * nn[2];
}

// The nodes rank r holds: its block extended by the one-node ghost layer the
// sweep reads (clamped to the grid); a 1-node dummy for an empty block.
static BlockBox halo_box(const BlockDecomp &D, const int nn[3], int r)
{
    int lo[3], ext[3];
    decomp_block(D, nn, r, lo, ext);
    BlockBox b{{0, 0, 0}, {1, 1, 1}};
    if (ext[0] <= 0 || ext[1] <= 0 || ext[2] <= 0) return b;
    for (int a = 0; a < 3; a++) {
        const int l = std::max(0, lo[a] - 1), h = std::min(nn[a] - 1, lo[a] + ext[a]);
        b.lo[a] = l;
        b.ext[a] = h - l + 1;
    }
    return b;
}

// Device state of a rank's box (reallocated when nsrc outgrows it): the
// fields hold hbox of the global grid.
static int rank_alloc(SingleState &S, const RankHalo &H, int maxit, int nsrc)
{
    if (single_alloc(S, 1, H.hbox.ext[0], H.hbox.ext[1], H.hbox.ext[2], maxit, nsrc)) return 1;
    SingleLaunch &L = S.L;
    L.gx = H.gn[0]; L.gy = H.gn[1]; L.gz = H.gn[2];
    L.ox = H.hbox.lo[0]; L.oy = H.hbox.lo[1]; L.oz = H.hbox.lo[2];
    return 0;
}

static void halo_free(RankHalo &H)
{
    if (H.nc) mceik_rccl().CommDestroy(H.nc);
    if (H.d_buf) hipFree(H.d_buf);
    if (H.h_buf) hipHostFree(H.h_buf);
    memset(&H, 0, sizeof(H));
}

// Face plan, buffers and transport of this rank (collective over comm).
// Returns 0, or 1 when any rank failed (every rank returns alike).
static int halo_setup(RankHalo &H, const BlockDecomp &D, const int nn[3], int fcomm, int rank, int nranks)
{
    halo_free(H);
    H.fcomm = fcomm; H.rank = rank; H.nranks = nranks;
    for (int a = 0; a < 3; a++) H.gn[a] = nn[a];
    H.hbox = halo_box(D, nn, rank);
    int lo[3], ext[3];
    decomp_block(D, nn, rank, lo, ext);
    for (int a = 0; a < 3; a++) { H.own.lo[a] = lo[a]; H.own.ext[a] = ext[a]; }
    const int bi[3] = {rank % D.nd[0], (rank / D.nd[0]) % D.nd[1], rank / (D.nd[0] * D.nd[1])};
    int nf = 0;
    H.send.off[0] = H.recv.off[0] = 0;
    const bool empty = ext[0] <= 0 || ext[1] <= 0 || ext[2] <= 0;
    for (int a = 0; a < 3 && D.nov > 0 && !empty; a++)
        for (int s = 0; s < 2; s++) {
            const int nb = bi[a] + (s ? 1 : -1);
            if (nb < 0 || nb >= D.nd[a]) continue;
            int nbi[3] = {bi[0], bi[1], bi[2]};
            nbi[a] = nb;
            int nlo[3], next[3];
            decomp_block(D, nn, nbi[0] + D.nd[0] * (nbi[1] + D.nd[1] * nbi[2]), nlo, next);
            if (next[0] <= 0 || next[1] <= 0 || next[2] <= 0) continue;      // an empty neighbour sends nothing
            BlockBox sb = H.own, rb = H.own;
            sb.ext[a] = rb.ext[a] = 1;
            sb.lo[a] = s ? lo[a] + ext[a] - 1 : lo[a];
            rb.lo[a] = s ? lo[a] + ext[a] : lo[a] - 1;
            H.peer[nf] = nbi[0] + D.nd[0] * (nbi[1] + D.nd[1] * nbi[2]);
            H.tag_send[nf] = 2 * a + s;
            H.tag_recv[nf] = 2 * a + 1 - s;
            H.send.box[nf] = sb;
            H.recv.box[nf] = rb;
            const size_t cnt = (size_t)sb.ext[0] * sb.ext[1] * sb.ext[2];
            H.send.off[nf + 1] = H.send.off[nf] + cnt;
            H.recv.off[nf + 1] = H.recv.off[nf] + cnt;
            nf++;
        }
    H.send.n = H.recv.n = nf;
    const size_t nsend = H.send.off[nf], nrecv = H.recv.off[nf];
    int e = 0;
    if (nsend + nrecv > 0 &&
        (hipMalloc(&H.d_buf, (nsend + nrecv) * 8) != hipSuccess ||
         hipHostMalloc(&H.h_buf, (nsend + nrecv) * 8, hipHostMallocDefault) != hipSuccess))
        e = 1;
    // transport: host-staged MPI by default (the transport the bitwise
    // across-ranks tests pin); MCEIK_HALO=rccl forces RCCL device to device,
    // MCEIK_HALO=auto picks RCCL when no two ranks share a GPU.  The RCCL face
    // swap needs one GPU per rank, which this build's test pool never had, so
    // its parity is unpinned and it stays opt-in.
    const char *env = getenv("MCEIK_HALO");
    int want = env && !strcmp(env, "rccl") ? 2 : env && !strcmp(env, "auto") ? 0 : 1;
    if (!want) {
        char id[128] = {0};
        int dev = 0;
        gethostname(id, 64);
        id[63] = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(id + 64, 64, dev) != hipSuccess) e = 1;
        std::vector<char> all((size_t)nranks * 128);
        want = 2;
        if (mceik_mpi_allgather_bytes(fcomm, id, all.data(), 128)) e = 1;
        for (int r = 0; r < nranks && want == 2; r++)
            for (int q = 0; q < r; q++)
                if (!memcmp(&all[(size_t)r * 128], &all[(size_t)q * 128], 128)) { want = 1; break; }
    }
    if (mceik_mpi_allreduce_int(fcomm, &e, 1, 1)) e = 1;
    if (!e && want == 2) {
        int idw[MCEIK_COMM_ID_BYTES / 4] = {0};
        int ie = !mceik_rccl().ok;
        if (mceik_mpi_allreduce_int(fcomm, &ie, 1, 1) || ie) e = 1;
        ncclUniqueId uid;
        if (!e && rank == 0) {
            ie = mceik_rccl().GetUniqueId(&uid) != ncclSuccess;
            memcpy(idw, &uid, sizeof(uid));
        }
        if (!e && (mceik_mpi_bcast_int(fcomm, &ie, 1, 0) || ie || mceik_mpi_bcast_int(fcomm, idw, MCEIK_COMM_ID_BYTES / 4, 0)))
            e = 1;
        if (!e) {
            memcpy(&uid, idw, sizeof(uid));
            ie = mceik_rccl().CommInitRank(&H.nc, nranks, uid, rank) != ncclSuccess;
            if (ie) H.nc = nullptr;
            if (mceik_mpi_allreduce_int(fcomm, &ie, 1, 1) || ie) e = 1;
        }
    }
    H.kind = want;
    if (e) {
        halo_free(H);
        return 1;
    }
    H.on = 1;
    return 0;
}

// One face swap after a sweep: pack the faces this rank owns, swap them with
// the neighbours, unpack the ones received.  Returns nonzero on a failure
// (a failing rank still takes part in the messages, so none is left waiting).
static int halo_swap(RankHalo &H, const SingleLaunch &L, hipStream_t st, int fail)
{
    const int nf = H.send.n;
    if (nf == 0) return fail;
    const size_t nsend = H.send.off[nf], nrecv = H.recv.off[nf];
    double *d_recv = H.d_buf + nsend;
    if (H.kind == 2) {
        if (!fail && fsm_box_copy(L, H.send, H.d_buf, 1, st) != hipSuccess) fail = 1;
        bool ok = mceik_rccl().GroupStart() == ncclSuccess;
        for (int f = 0; f < nf && ok; f++)
            ok = mceik_rccl().Send(H.d_buf + H.send.off[f], H.send.off[f + 1] - H.send.off[f], ncclFloat64, H.peer[f],
                                   H.nc, st) == ncclSuccess &&
                 mceik_rccl().Recv(d_recv + H.recv.off[f], H.recv.off[f + 1] - H.recv.off[f], ncclFloat64, H.peer[f],
                                   H.nc, st) == ncclSuccess;
        ok = mceik_rccl().GroupEnd() == ncclSuccess && ok;
        if (!ok) fail = 1;
        if (!fail && fsm_box_copy(L, H.recv, d_recv, 0, st) != hipSuccess) fail = 1;
        return fail;
    }
    if (!fail && (fsm_box_copy(L, H.send, H.d_buf, 1, st) != hipSuccess ||
                  hipMemcpyAsync(H.h_buf, H.d_buf, nsend * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                  hipStreamSynchronize(st) != hipSuccess))
        fail = 1;
    int dir[12], peer[12], tag[12], cnt[12];
    double *buf[12];
    for (int f = 0; f < nf; f++) {
        dir[2 * f] = 0; peer[2 * f] = H.peer[f]; tag[2 * f] = H.tag_send[f];
        buf[2 * f] = H.h_buf + H.send.off[f]; cnt[2 * f] = (int)(H.send.off[f + 1] - H.send.off[f]);
        dir[2 * f + 1] = 1; peer[2 * f + 1] = H.peer[f]; tag[2 * f + 1] = H.tag_recv[f];
        buf[2 * f + 1] = H.h_buf + nsend + H.recv.off[f]; cnt[2 * f + 1] = (int)(H.recv.off[f + 1] - H.recv.off[f]);
    }
    if (mceik_mpi_exchange_double(H.fcomm, 2 * nf, dir, peer, tag, buf, cnt)) fail = 1;
    if (!fail && (hipMemcpyAsync(d_recv, H.h_buf + nsend, nrecv * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
                  fsm_box_copy(L, H.recv, d_recv, 0, st) != hipSuccess))
        fail = 1;
    return fail;
}

// Node box B (global coordinates) of the dense x-fastest grid g <-> a packed
// x-fastest buffer (host side of the model scatter and the field gather).
static void host_box(double *grid, const int g[3], const BlockBox &B, double *buf, bool to_buf)
{
    size_t i = 0;
    for (int z = 0; z < B.ext[2]; z++)
        for (int y = 0; y < B.ext[1]; y++) {
            double *row = grid + ((size_t)(B.lo[2] + z) * g[1] + B.lo[1] + y) * g[0] + B.lo[0];
            if (to_buf) memcpy(buf + i, row, (size_t)B.ext[0] * 8);
            else memcpy(row, buf + i, (size_t)B.ext[0] * 8);
            i += B.ext[0];
        }
}
static size_t box_count(const BlockBox &B)
{
    return B.ext[0] > 0 && B.ext[1] > 0 && B.ext[2] > 0 ? (size_t)B.ext[0] * B.ext[1] * B.ext[2] : 0;
}

// The distributed solve (collective over comm; the master's slow/u are the
// whole grid, the others' are not read or written).  The master sends every
// rank the slowness of the nodes it holds (EIKONAL_SCATTER_MODEL) and the
// sources; every rank runs SETBCS on its box (the same nodes and values as on
// the whole grid), sweeps its block with a face swap after every sweep, and
// sends its block back (EIKONAL_GATHER_TRAVELTIMES).  Every rank returns its
// own ierr as the reference's (SETBCS: the same on every rank; the solver: the
// ierr of its local grid's last level), -1 on a failure on any rank.
static int blocks_solve_ranks(SingleState &S, RankHalo &H, int nsrc, const double *ts, const double *xs,
                              const double *ys, const double *zs, const double *slow, double *u)
{
    SingleLaunch &L = S.L;
    const size_t nloc = (size_t)L.nx * L.ny * L.nz, np = (size_t)L.nxp * L.nyp * L.nzp;
    L.maxit = S.maxit; L.tol = S.tol; L.h = S.h; L.x0 = S.x0; L.y0 = S.y0; L.z0 = S.z0;
    const bool master = H.rank == 0;
    std::vector<double> src((size_t)nsrc * 4), mine(nloc);
    if (master)
        for (int k = 0; k < nsrc; k++) {
            src[k * 4 + 0] = ts[k]; src[k * 4 + 1] = xs[k]; src[k * 4 + 2] = ys[k]; src[k * 4 + 3] = zs[k];
        }
    if (mceik_mpi_bcast_double(H.fcomm, src.data(), nsrc * 4, 0)) return -1;
    int fail = 0;
    {   // the slowness of every rank's box from the master
        std::vector<std::vector<double>> out;
        std::vector<int> dir, peer, tag, cnt;
        std::vector<double *> buf;
        if (master) {
            host_box((double *)slow, H.gn, H.hbox, mine.data(), true);
            out.resize(H.nranks);
            for (int r = 1; r < H.nranks; r++) {
                const BlockBox b = halo_box(S.D, H.gn, r);
                out[r].resize(box_count(b));
                host_box((double *)slow, H.gn, b, out[r].data(), true);
                dir.push_back(0); peer.push_back(r); tag.push_back(98); cnt.push_back((int)out[r].size());
                buf.push_back(out[r].data());
            }
        } else {
            dir.push_back(1); peer.push_back(0); tag.push_back(98); cnt.push_back((int)nloc); buf.push_back(mine.data());
        }
        if (mceik_mpi_exchange_double(H.fcomm, (int)dir.size(), dir.data(), peer.data(), tag.data(), buf.data(),
                                      cnt.data()))
            return -1;
    }
    hipStream_t st = S.st;
    const BlockBox own = H.own;
    const bool empty = own.ext[0] <= 0 || own.ext[1] <= 0 || own.ext[2] <= 0;
    int ierr_bc = 0, ierr = 0;
    if (hipMemcpyAsync(S.dense, mine.data(), nloc * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(S.src, src.data(), src.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        fsm_single_pad(S.dense, (void *)L.slow, 1, L.nx, L.ny, L.nz, L.nxp, L.nyp, st) != hipSuccess ||
        fsm_single_setbcs(L, S.src, nsrc, S.ierr_bc, st) != hipSuccess ||
        hipMemcpyAsync(&ierr_bc, S.ierr_bc, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        fail = 1;
    int agree[2] = {fail, ierr_bc};                  // SETBCS's checks run alike everywhere
    if (mceik_mpi_allreduce_int(H.fcomm, agree, 2, 1)) return -1;
    if (agree[0]) return -1;
    S.bcfail = agree[1] != 0;
    if (S.bcfail) return 1;
    int *d_ierr = (int *)(S.d_count + 1);
    for (int k = 1; k <= S.maxit; k++) {
        if (!fail && hipMemcpyAsync(L.u0, L.u, np * 8, hipMemcpyDeviceToDevice, st) != hipSuccess) fail = 1;
        for (int g = 0; g < 8; g++) {
            if (!fail && (hipMemsetAsync(d_ierr, 0, 4, st) != hipSuccess ||
                          fsm_block_sweep(L, S.D, (const double *)L.u, g, d_ierr, st, H.rank, empty ? 0 : 1,
                                          H.rank) != hipSuccess))
                fail = 1;
            fail = halo_swap(H, L, st, fail);
        }
        unsigned count = 0;
        if (!fail && (hipMemsetAsync(S.d_count, 0, 4, st) != hipSuccess ||
                      (!empty && fsm_block_unconverged(L, own, S.tol, S.d_count, st) != hipSuccess) ||
                      hipMemcpyAsync(&count, S.d_count, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                      hipMemcpyAsync(&ierr, d_ierr, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                      hipStreamSynchronize(st) != hipSuccess))
            fail = 1;
        // the reference sums the unconverged counts (fsm3d.f90:198-211) and tests
        // for zero: a max over "any left" flags is that test without the sum's
        // overflow on large blocks
        int tot[2] = {count ? 1 : 0, fail};
        if (mceik_mpi_allreduce_int(H.fcomm, tot, 2, 1)) return -1;
        if (tot[1]) return -1;
        if (tot[0] == 0) break;
    }
    // every block to the master
    BoxList bl;
    bl.n = 1; bl.box[0] = own; bl.off[0] = 0; bl.off[1] = empty ? 0 : box_count(own);
    std::vector<double> blk(bl.off[1]);
    if (!fail && bl.off[1] &&
        (fsm_box_copy(L, bl, S.dense, 1, st) != hipSuccess ||
         hipMemcpyAsync(blk.data(), S.dense, blk.size() * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
         hipStreamSynchronize(st) != hipSuccess))
        fail = 1;
    {
        std::vector<std::vector<double>> got(H.nranks);
        std::vector<BlockBox> box(H.nranks);
        std::vector<int> dir, peer, tag, cnt;
        std::vector<double *> buf;
        if (master) {
            for (int r = 1; r < H.nranks; r++) {
                int lo[3], ext[3];
                decomp_block(S.D, H.gn, r, lo, ext);
                for (int a = 0; a < 3; a++) { box[r].lo[a] = lo[a]; box[r].ext[a] = ext[a]; }
                got[r].resize(box_count(box[r]));
                if (got[r].empty()) continue;
                dir.push_back(1); peer.push_back(r); tag.push_back(99); cnt.push_back((int)got[r].size());
                buf.push_back(got[r].data());
            }
        } else if (!blk.empty()) {
            dir.push_back(0); peer.push_back(0); tag.push_back(99); cnt.push_back((int)blk.size()); buf.push_back(blk.data());
        }
        if (mceik_mpi_exchange_double(H.fcomm, (int)dir.size(), dir.data(), peer.data(), tag.data(), buf.data(),
                                      cnt.data()))
            fail = 1;
        if (master && !fail) {
            if (!blk.empty()) host_box(u, H.gn, own, blk.data(), false);
            for (int r = 1; r < H.nranks; r++)
                if (!got[r].empty()) host_box(u, H.gn, box[r], got[r].data(), false);
        }
    }
    if (mceik_mpi_allreduce_int(H.fcomm, &fail, 1, 1) || fail) return -1;
    return ierr;
}

// The MPI variant is collective over comm as the reference's
// (fsm3d.f90:1583-1929): the master (rank 0) broadcasts its parameters at
// initialize (:1626-1639) and its error at solve (:1792) and every rank
// returns it.  With as many ranks as blocks the solve is distributed, one
// block per rank (RankHalo above).  Otherwise one GPU holds the whole grid and
// the master alone solves (every block, when there are several, by the
// one-GPU block iteration); the other ranks take part in the broadcasts and
// keep their u untouched.  A process without MPI is the master of one rank,
// except that a call passing n < nx*ny*nz to solve acts as a non-master rank
// (the reference's callers pass n = 1 there, fsm3d.f90:2102-2106) and returns
// ierr = 0.
static int mpi_variant_rank(const int *comm) { return comm ? mceik_mpi_rank(*comm) : -1; }

extern "C" void eikonal3d_initialize(const int *comm, const int *iverb, const int *nx, const int *ny, const int *nz,
                                     const int *ndivx, const int *ndivy, const int *ndivz, const int *noverlap,
                                     const int *maxit, const double *x0, const double *y0, const double *z0,
                                     const double *h, const double *tol, int *ierr)
{
    SingleState &S = g_single[2];
    *ierr = 0;
    const int rank = mpi_variant_rank(comm);
    const int nranks = rank >= 0 ? mceik_mpi_size(*comm) : 1;
    // the master's parameters on every rank
    int ip[9] = {*iverb, *nx, *ny, *nz, *ndivx, *ndivy, *ndivz, *noverlap, *maxit};
    double dp[5] = {*x0, *y0, *z0, *h, *tol};
    if (rank >= 0 && (mceik_mpi_bcast_int(*comm, ip, 9, 0) || mceik_mpi_bcast_double(*comm, dp, 5, 0))) {
        printf(" eikonal3d_initialize: Error broadcasting parameters\n");
        *ierr = 1;
        return;
    }
    if (ip[0] > 0 && rank <= 0) printf(" eikonal3d_initialize: Broadcasting parameters...\n");
    int e = 0;
    const int nd[3] = {ip[4], ip[5], ip[6]}, nn[3] = {ip[1], ip[2], ip[3]};
    BlockDecomp D{};
    if (ip[4] < 1 || ip[5] < 1 || ip[6] < 1 || ip[7] < 0 || nn[0] < 1 || nn[1] < 1 || nn[2] < 1) {
        e = 1;
    } else {
        for (int a = 0; a < 3; a++) {
            D.nd[a] = nd[a];
            D.step[a] = nn[a] / nd[a] > 1 ? nn[a] / nd[a] : 1;       // fsm3d.f90:1086-1088
        }
        D.nov = ip[7];
        if (!decomp_tiles(D, nn)) e = 1;
    }
    if (e && rank <= 0) printf(" eikonal3d_initialize: Error computing local domain\n");
    const bool ranks = !e && rank >= 0 && nranks > 1 && nranks == nd[0] * nd[1] * nd[2];
    halo_free(g_halo);
    if (ranks) {                                 // every rank holds its block and the ghost layer
        if (halo_setup(g_halo, D, nn, *comm, rank, nranks)) {
            if (rank == 0) printf(" eikonal3d_initialize: Error making the ghost communication structure\n");
            e = 1;
        } else {
            if (rank_alloc(S, g_halo, ip[8], 1)) e = 2;
            S.D = D;
            if (!e && blocks_buffers(S)) e = 2;
        }
    } else if (!e && rank <= 0) {                // the grid on the master's GPU
        if (single_alloc(S, 1, nn[0], nn[1], nn[2], ip[8], 1)) e = 2;
        S.D = D;
        if (!e && (nd[0] * nd[1] * nd[2] > 1) && blocks_buffers(S)) e = 2;
    }
    if (e == 2) printf(" eikonal3d_initialize: Error making the device structures on process %d\n", rank > 0 ? rank : 0);
    // a failure on any rank's device is every rank's failure
    if (rank >= 0 && mceik_mpi_allreduce_int(*comm, &e, 1, 1)) e = 1;
    if (e) {
        halo_free(g_halo);
        *ierr = 1;
        return;
    }
    if (!ranks) { S.nx = nn[0]; S.ny = nn[1]; S.nz = nn[2]; }   // (ranks: S.n* are the box's, g_halo.gn the grid's)
    S.iverb = ip[0]; S.maxit = ip[8]; S.x0 = dp[0]; S.y0 = dp[1]; S.z0 = dp[2]; S.h = dp[3]; S.tol = dp[4];
    S.init = 1;
}

extern "C" void eikonal3d_solve(const int *comm, const int *nsrc, const int *n, const double *ts, const double *xs,
                                const double *ys, const double *zs, const double *slow, double *u, int *ierr)
{
    SingleState &S = g_single[2];
    *ierr = 0;
    const int rank = mpi_variant_rank(comm);
    if (!S.init) {
        printf(" eikonal3d_solve: solver not initialized\n");
        *ierr = 1;
        return;
    }
    int e = 0;
    const bool master = rank == 0 || (rank < 0 && (long)*n >= (long)S.nx * S.ny * S.nz);
    if (g_halo.on) {
        // the master's source count and argument check on every rank
        const RankHalo &H = g_halo;
        int mp[2] = {*nsrc, 0};
        if (master && (*nsrc < 1 || (long)*n < (long)H.gn[0] * H.gn[1] * H.gn[2])) mp[1] = 1;
        if (mceik_mpi_bcast_int(*comm, mp, 2, 0)) mp[1] = 1;
        if (!mp[1] && (rank_alloc(S, H, S.maxit, mp[0]) || blocks_buffers(S))) mp[1] = 2;
        if (mceik_mpi_allreduce_int(*comm, &mp[1], 1, 1)) mp[1] = 1;
        if (mp[1]) {
            if (master) printf(" eikonal3d_solve: Error setting bcs\n");
            *ierr = 1;
            return;
        }
        if (master && S.iverb > 0) printf(" eikonal3d_solve: Setting boundary conditions...\n");
        const int rc = blocks_solve_ranks(S, g_halo, mp[0], ts, xs, ys, zs, slow, u);
        if (S.bcfail) {
            if (master) printf(" eikonal3d_solve: Error setting bcs\n");
        } else if (rc != 0) {
            printf(" eikonal3d_solve: Error calling solver on process %d\n", rank);
        }
        *ierr = rc < 0 ? 1 : rc;
        return;
    }
    if (master) {
        const bool blocks = S.D.nd[0] * S.D.nd[1] * S.D.nd[2] > 1;
        if (*nsrc < 1 || (long)*n < (long)S.nx * S.ny * S.nz || single_alloc(S, 1, S.nx, S.ny, S.nz, S.maxit, *nsrc) ||
            (blocks && blocks_buffers(S))) {
            printf(" eikonal3d_solve: Error setting bcs\n");
            e = 1;
        } else {
            if (S.iverb > 0) printf(" eikonal3d_solve: Setting boundary conditions...\n");
            const int rc = blocks ? blocks_solve(S, *nsrc, ts, xs, ys, zs, slow, u, nullptr)
                                  : single_solve(S, S.maxit, *nsrc, S.tol, S.h, S.x0, S.y0, S.z0, ts, xs, ys, zs,
                                                 slow, u, nullptr);
            if (S.bcfail) printf(" eikonal3d_solve: Error setting bcs\n");
            else if (rc != 0) printf(" eikonal3d_solve: Error calling solver\n");
            e = rc < 0 ? 1 : rc;
        }
    }
    // the master's error on every rank (fsm3d.f90:1792)
    if (rank >= 0 && mceik_mpi_bcast_int(*comm, &e, 1, 0)) e = 1;
    *ierr = e;
}

extern "C" void eikonal3d_finalize(const int *comm, int *ierr)
{
    SingleState &S = g_single[2];
    *ierr = 0;
    if (!S.init) {                       // fsm3d.f90:1913-1916
        printf(" eikonal3d_finalize: Solver was never initialized\n");
        *ierr = 1;
    }
    if (mpi_variant_rank(comm) <= 0 && S.iverb > 0) printf(" eikonal3d_finalize: Freeing memory...\n");
    halo_free(g_halo);
    single_free(S);
    S.init = 0;
}

// ---------------------------------------------------------------------------
// locate3d_gridsearch__double64 / __float64 drop-ins (gridsearch.f90:382-540).
template <typename T>
static void gridsearch_f90_dropin(const char *fcnm, const int *ldgrd, const int *ngrd, const int *nobs,
                                  const int *iwantOT, const int *mask, const T *tobs, const T *varobs, const T *test,
                                  T *logPDF, int *ierr)
{
    *ierr = 0;
    if (*ldgrd % 64 != 0) {
        printf(" %s: Require arrays be 64 byte aligned %d %d\n", fcnm, *ldgrd,
               sizeof(T) == 8 ? (8 * *ldgrd) % 64 : *ldgrd % 64);
        *ierr = 1;
        return;
    }
    if (*ngrd > *ldgrd) {
        printf(" %s: ngrd cannot be greater than ldgrd\n", fcnm);
        *ierr = 1;
        return;
    }
    long msum = 0;
    T vsum = (T)0;
    for (int i = 0; i < *nobs; i++) { msum += mask[i]; vsum = vsum + varobs[i]; }
    if (msum == *nobs) {
        printf(" %s: No observations\n", fcnm);
        *ierr = 1;
        return;
    }
    const T eps = sizeof(T) == 8 ? (T)DBL_EPSILON : (T)FLT_EPSILON;
    if ((vsum < (T)0 ? -vsum : vsum) < eps) {
        printf(" %s: Will be division by zero\n", fcnm);
        *ierr = 1;
        return;
    }
    T xnorm = (T)0;
    for (int i = 0; i < *nobs; i++) if (mask[i] != 1) xnorm = xnorm + varobs[i];
    const T one = (T)1, sqrt2i = one / (sizeof(T) == 8 ? (T)sqrt(2.0) : (T)sqrtf(2.0f));
    std::vector<int> row;
    std::vector<T> tob, w0, wl;
    for (int i = 0; i < *nobs; i++) {
        if (mask[i] == 1) continue;
        row.push_back(i);
        tob.push_back(tobs[i]);
        w0.push_back(one / (varobs[i] * xnorm));
        wl.push_back(sqrt2i / varobs[i]);
    }
    const int nuse = (int)row.size();
    const size_t tb = (size_t)*ldgrd * *nobs * sizeof(T);
    char *d = nullptr;
    const size_t a = ((size_t)nuse * 16 + 255) & ~(size_t)255;
    if (hipMalloc(&d, 4 * a + tb + (size_t)*ngrd * sizeof(T) + 64) != hipSuccess) {
        printf(" %s: device allocation failed\n", fcnm);
        *ierr = 1;
        return;
    }
    int *d_row = (int *)d;
    T *d_tob = (T *)(d + a), *d_w0 = (T *)(d + 2 * a), *d_wl = (T *)(d + 3 * a);
    T *d_test = (T *)(d + 4 * a), *d_lp = (T *)(d + 4 * a + tb);
    bool ok = hipMemcpy(d_row, row.data(), nuse * 4, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_tob, tob.data(), nuse * sizeof(T), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_w0, w0.data(), nuse * sizeof(T), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_wl, wl.data(), nuse * sizeof(T), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_test, test, tb, hipMemcpyHostToDevice) == hipSuccess &&
              gridsearch_f90(sizeof(T) == 8, *ldgrd, *ngrd, nuse, *iwantOT, d_row, d_tob, d_w0, d_wl, d_test, d_lp,
                             nullptr) == hipSuccess &&
              hipMemcpy(logPDF, d_lp, (size_t)*ngrd * sizeof(T), hipMemcpyDeviceToHost) == hipSuccess;
    hipFree(d);
    if (!ok) {
        printf(" %s: device failure\n", fcnm);
        *ierr = 1;
    }
}

extern "C" void locate3d_gridsearch__double64(const int *ldgrd, const int *ngrd, const int *nobs, const int *iwantOT,
                                              const int *mask, const double *tobs, const double *varobs,
                                              const double *test, double *logPDF, int *ierr)
{
    gridsearch_f90_dropin<double>("locate3d_gridsearch_double64", ldgrd, ngrd, nobs, iwantOT, mask, tobs, varobs,
                                  test, logPDF, ierr);
}

extern "C" void locate3d_gridsearch__float64(const int *ldgrd, const int *ngrd, const int *nobs, const int *iwantOT,
                                             const int *mask, const float *tobs, const float *varobs,
                                             const float *test, float *logPDF, int *ierr)
{
    gridsearch_f90_dropin<float>("locate3d_gridsearch_float64", ldgrd, ngrd, nobs, iwantOT, mask, tobs, varobs,
                                 test, logPDF, ierr);
}

// ---------------------------------------------------------------------------
// locate_l2_gridSearch__double64 drop-in (locate.c:923-1047).
extern "C" int locate_l2_gridSearch__double64(int ldgrd, int ngrd, int nobs, int iwantOT, double t0use,
                                              const int *mask, const double *tobs, const double *tcorr,
                                              const double *varobs, const double *test,
                                              double *t0, double *objfn)
{
    const char *fcnm = "locate_l2_gridSearch__double64";
    if ((sizeof(double) * (size_t)ldgrd) % 64 != 0 || ldgrd < ngrd || nobs < 1 || !mask || !tobs ||
        !varobs || !test || !t0 || !objfn) {
        if ((sizeof(double) * (size_t)ldgrd) % 64 != 0) printf("%s: Error ldgrd must be divisible by 64\n", fcnm);
        if (ldgrd < ngrd) printf("%s: Error ldgrd < ngrd\n", fcnm);
        if (!mask) printf("%s: mask is null\n", fcnm);
        if (!tobs) printf("%s: tobs is null\n", fcnm);
        if (!varobs) printf("%s: varobs is null\n", fcnm);
        if (!test) printf("%s: test is null\n", fcnm);
        if (!t0) printf("%s: t0 is null\n", fcnm);
        if (!objfn) printf("%s: objfn is null\n", fcnm);
        return 1;
    }
    if (((uintptr_t)t0 % 64) || ((uintptr_t)test % 64) || ((uintptr_t)objfn % 64)) {
        printf("%s: Input arrays are not 64 bit aligned\n", fcnm);
        return 1;
    }
    std::vector<int> use;
    std::vector<double> tc, wt;
    double xnorm = 0.0;
    for (int i = 0; i < nobs; i++) {
        if (mask[i] != 0) continue;
        tc.push_back(tcorr ? tobs[i] - tcorr[i] : tobs[i]);
        use.push_back(i);
        wt.push_back(1.0 / varobs[i]);
        xnorm = xnorm + wt.back();
    }
    int nuse = (int)use.size();
    int *d_use = nullptr;
    double *d_tc = nullptr, *d_wt = nullptr, *d_test = nullptr, *d_t0 = nullptr, *d_obj = nullptr;
    int rc = 1;
    size_t tb = (size_t)ldgrd * nobs * 8;
    if (hipMalloc(&d_use, (nuse + 1) * 4) != hipSuccess || hipMalloc(&d_tc, (nuse + 1) * 8) != hipSuccess ||
        hipMalloc(&d_wt, (nuse + 1) * 8) != hipSuccess || hipMalloc(&d_test, tb) != hipSuccess ||
        hipMalloc(&d_t0, (size_t)ngrd * 8 + 8) != hipSuccess || hipMalloc(&d_obj, (size_t)ngrd * 8 + 8) != hipSuccess)
        goto out;
    if (nuse) {
        hipMemcpy(d_use, use.data(), nuse * 4, hipMemcpyHostToDevice);
        hipMemcpy(d_tc, tc.data(), nuse * 8, hipMemcpyHostToDevice);
        hipMemcpy(d_wt, wt.data(), nuse * 8, hipMemcpyHostToDevice);
    }
    hipMemcpy(d_test, test, tb, hipMemcpyHostToDevice);
    if (l2_gridsearch(ldgrd, ngrd, nuse, iwantOT, t0use, d_use, d_tc, d_wt, xnorm, d_test, d_t0, d_obj, nullptr) != hipSuccess)
        goto out;
    if (hipMemcpy(t0, d_t0, (size_t)ngrd * 8, hipMemcpyDeviceToHost) != hipSuccess) goto out;
    if (hipMemcpy(objfn, d_obj, (size_t)ngrd * 8, hipMemcpyDeviceToHost) != hipSuccess) goto out;
    rc = 0;
out:
    hipFree(d_use); hipFree(d_tc); hipFree(d_wt); hipFree(d_test); hipFree(d_t0); hipFree(d_obj);
    if (rc) printf("%s: device failure\n", fcnm);
    return rc;
}

// ---------------------------------------------------------------------------
// locate_l2_gridSearch__float64 drop-in (locate.c:1079-1203): fp32 arithmetic.
extern "C" int locate_l2_gridSearch__float64(int ldgrd, int ngrd, int nobs, int iwantOT, float t0use,
                                             const int *mask, const float *tobs, const float *tcorr,
                                             const float *varobs, const float *test, float *t0, float *objfn)
{
    const char *fcnm = "locate_l2_gridSearch__float64";
    if ((sizeof(float) * (size_t)ldgrd) % 64 != 0 || ldgrd < ngrd || nobs < 1 || !mask || !tobs ||
        !varobs || !test || !t0 || !objfn) {
        if ((sizeof(float) * (size_t)ldgrd) % 64 != 0) printf("%s: Error ldgrd must be divisible by 64\n", fcnm);
        if (ldgrd < ngrd) printf("%s: Error ldgrd < ngrd\n", fcnm);
        if (!mask) printf("%s: mask is null\n", fcnm);
        if (!tobs) printf("%s: tobs is null\n", fcnm);
        if (!varobs) printf("%s: varobs is null\n", fcnm);
        if (!test) printf("%s: test is null\n", fcnm);
        if (!t0) printf("%s: t0 is null\n", fcnm);
        if (!objfn) printf("%s: objfn is null\n", fcnm);
        return 1;
    }
    if (((uintptr_t)t0 % 64) || ((uintptr_t)test % 64) || ((uintptr_t)objfn % 64)) {
        printf("%s: Input arrays are not 64 bit aligned\n", fcnm);
        return 1;
    }
    std::vector<int> row;
    std::vector<float> tc, wt;
    float xnorm = 0.0f;
    for (int i = 0; i < nobs; i++) {
        if (mask[i] != 0) continue;
        tc.push_back(tcorr ? tobs[i] - tcorr[i] : tobs[i]);
        row.push_back(i);
        wt.push_back(1.0f / varobs[i]);
        xnorm = xnorm + wt.back();
    }
    const int nuse = (int)row.size();
    const int ptr[2] = {0, nuse};
    int *d_row = nullptr, *d_ptr = nullptr;
    float *d_tc = nullptr, *d_wt = nullptr, *d_xn = nullptr, *d_test = nullptr, *d_t0 = nullptr, *d_obj = nullptr;
    int rc = 1;
    const size_t tb = (size_t)ldgrd * nobs * 4, gb = (size_t)ldgrd * 4;
    if (hipMalloc(&d_row, (nuse + 1) * 4) != hipSuccess || hipMalloc(&d_ptr, 8) != hipSuccess ||
        hipMalloc(&d_tc, (nuse + 1) * 4) != hipSuccess || hipMalloc(&d_wt, (nuse + 1) * 4) != hipSuccess ||
        hipMalloc(&d_xn, 4) != hipSuccess || hipMalloc(&d_test, tb) != hipSuccess ||
        hipMalloc(&d_t0, gb) != hipSuccess || hipMalloc(&d_obj, gb) != hipSuccess)
        goto out;
    if (nuse) {
        hipMemcpy(d_row, row.data(), nuse * 4, hipMemcpyHostToDevice);
        hipMemcpy(d_tc, tc.data(), nuse * 4, hipMemcpyHostToDevice);
        hipMemcpy(d_wt, wt.data(), nuse * 4, hipMemcpyHostToDevice);
    }
    hipMemcpy(d_ptr, ptr, 8, hipMemcpyHostToDevice);
    hipMemcpy(d_xn, &xnorm, 4, hipMemcpyHostToDevice);
    hipMemcpy(d_test, test, tb, hipMemcpyHostToDevice);
    if (l2_gridsearch_f32(ldgrd, ngrd, 1, iwantOT, t0use, d_ptr, d_row, d_tc, d_wt, d_xn, d_test, d_t0, d_obj, 0,
                          nullptr) != hipSuccess)
        goto out;
    if (hipMemcpy(t0, d_t0, (size_t)ngrd * 4, hipMemcpyDeviceToHost) != hipSuccess) goto out;
    if (hipMemcpy(objfn, d_obj, (size_t)ngrd * 4, hipMemcpyDeviceToHost) != hipSuccess) goto out;
    rc = 0;
out:
    hipFree(d_row); hipFree(d_ptr); hipFree(d_tc); hipFree(d_wt); hipFree(d_xn);
    hipFree(d_test); hipFree(d_t0); hipFree(d_obj);
    if (rc) printf("%s: device failure\n", fcnm);
    return rc;
}

// Relocation grid search of many events against one model's station tables
// (SURVEY s.8f row 2): device arrays, one launch, enqueued on `stream`.
extern "C" int mceik_relocate(const mceik_relocate_batch *b, void *stream)
{
    if (!b || b->ngrd < 1 || b->ldgrd < b->ngrd || b->nev < 1 || !b->tables || !b->ev_ptr || !b->obs_row ||
        !b->tc || !b->wt || !b->xnorm || !b->out) {
        fprintf(stderr, "mceik_relocate: invalid batch description\n");
        return 1;
    }
    if (b->nrows > 0 && b->nobs >= 0 && relocate_lds_bytes(b->nrows, b->nobs, b->nev) <= 64 * 1024)
        return relocate_lds(b->ldgrd, b->ngrd, b->nrows, b->nev, b->nobs, b->iwantOT, b->t0use, b->ev_ptr, b->obs_row,
                            b->tc, b->wt, b->xnorm, b->tables, b->t0, b->out, b->log_pdf ? 1 : 0,
                            (hipStream_t)stream) != hipSuccess;
    return l2_gridsearch_f32(b->ldgrd, b->ngrd, b->nev, b->iwantOT, b->t0use, b->ev_ptr, b->obs_row, b->tc, b->wt,
                             b->xnorm, b->tables, b->t0, b->out, b->log_pdf ? 1 : 0, (hipStream_t)stream) != hipSuccess;
}

// ---------------------------------------------------------------------------
// MCMC sampler (include/mceik.h)
#define MCEIK_EV_RING 32           // hipEvent pairs around timed FSM launches (fixed ring)
#define MCEIK_MAX_PIPES 4
#define MCEIK_ITERS_N (6 + MCEIK_TRAFFIC_N)   // d_iters: iterations, 4 visit statistics, solves, traffic

struct mceik_mcmc {
    McmcDev D;
    hipEvent_t ev[2 * MCEIK_EV_RING];  // pairs around FSM launches (timing)
    int ev_made;                       // pairs created so far
    long long nlaunch;                 // timed launches since the last reset
    long long ev_folded;               // launches whose pair has been folded into fsm_ms
    double fsm_ms;                     // folded kernel time (ms)
    unsigned long long *d_iters;
    int *d_ierr;
    unsigned long long *d_clock;       // per-solve start/end stamps of the last launch (queue order, report)
    int *d_order;                      // longest-first queue order for the next launch (MCEIK_LPT=1), or null
    bool report;                       // MCEIK_SOLVE_CLOCK_REPORT=1
    // Two pipes (default; MCEIK_PIPES=1 turns them off): the chains run as two
    // halves on two streams of their own, each half's next FSM launch queued
    // behind its own accept, so one half's launch fills the waves the other
    // half's queue tail leaves idle.  Results are those of
    // one pipe bit for bit.
    int npipe;
    // Multi-step launches (MCEIK_PERSIST=1, where the 16-z kernel runs): one
    // FSM launch runs up to MCEIK_MC_CHUNK steps, the
    // chain epilogue (accept, kept state, next proposal) inside the kernel
    // (fsm16_kernel.hip mc_finish), so no step waits for the slowest chain of
    // the one before.  d_dev: device copy of D; d_sync: the launch's queues.
    bool persist;
    unsigned spin_limit;               // multi-step launches: polls before a wait counts as a broken queue
    McmcDev *d_dev;
    unsigned *d_sync;
    hipStream_t pst[MCEIK_MAX_PIPES];
    hipEvent_t pfork, pjoin[MCEIK_MAX_PIPES];
    McmcDev pD[MCEIK_MAX_PIPES];
    mceik_fsm_batch pfb[MCEIK_MAX_PIPES];
    void *pws[MCEIK_MAX_PIPES];        // pipe k's workspace: a part of ws, ws itself, or its own
    size_t pws_bytes[MCEIK_MAX_PIPES];
    bool pws_own[MCEIK_MAX_PIPES];     // pws[k] was allocated for the pipe
    mceik_fsm_batch fb;                // a step's batch: every chain's proposed model x stations
    mceik_fsm_batch fb_all;            // init / restore: every model of every chain (= fb with one model)
    const float *last_ttab;            // tables of the last forward (mceik_mcmc_last)
    int masked_s;                      // S picks ignored (nphase 1, mask_s)
    int device, max_samples, nburn, keepk, nkept, niter_total;
    int nkept_base;                    // nkept at the last restore: earlier states are not in the ring
    long long step;
    hipStream_t stream;
    void *ws;
    size_t ws_bytes;
    std::vector<void *> allocs;
};

// Every entry point runs on the sampler's device and restores the caller's.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceScope()
    {
        if (prev >= 0) hipSetDevice(prev);
    }
};

template <typename T>
static int dalloc(mceik_mcmc *s, T **p, size_t count)
{
    void *q = nullptr;
    if (hipMalloc(&q, count * sizeof(T) + 16) != hipSuccess) return -1;
    hipMemset(q, 0, count * sizeof(T) + 16);
    s->allocs.push_back(q);
    *p = (T *)q;
    return 0;
}

template <typename T>
static int dput(mceik_mcmc *s, T **p, const T *host, size_t count)
{
    if (dalloc(s, p, count)) return -1;
    if (count && hipMemcpy(*p, host, count * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return -1;
    return 0;
}

static int source_index(int n, double x0, double dx, double xs)   // fsm3d.f90:697-711 (0-based)
{
    if (xs <= x0) return 0;
    if (xs >= x0 + (double)(n - 1) * dx) return n - 1;
    return (int)((xs - x0) / dx + 0.5);
}

// Trilinear mode (mceik_mcmc_opts.tt_interp; no reference counterpart): the
// lowest corner i of the grid cell holding xs, clamped to [0, n-2], and the
// fraction w = (xs - x0)/dx - i in [0, 1] rounded once to fp32.  Positions
// outside the grid clamp to its faces (w = 0 or 1), the snapping rule's
// clamping (fsm3d.f90:697-711).
static int cell_corner(int n, double x0, double dx, double xs, float *w)
{
    if (n < 2) { *w = 0.0f; return 0; }
    const double f = (xs - x0) / dx;
    int i = f <= 0.0 ? 0 : (int)f;
    if (i > n - 2) i = n - 2;
    double r = f - (double)i;
    r = r < 0.0 ? 0.0 : (r > 1.0 ? 1.0 : r);
    *w = (float)r;
    return i;
}

// Adds the elapsed time of timed launch k (its pair is complete once its end
// event is) to fsm_ms.  Blocks only when MCEIK_EV_RING launches are queued.
static int fold_launch(mceik_mcmc *s, long long k)
{
    const int r = (int)(k % MCEIK_EV_RING);
    float t = 0.f;
    HIPCHK(hipEventSynchronize(s->ev[2 * r + 1]));
    HIPCHK(hipEventElapsedTime(&t, s->ev[2 * r], s->ev[2 * r + 1]));
    s->fsm_ms += t;
    return 0;
}

static int mcmc_forward(mceik_mcmc *s, bool timed, int pipe = -1, const McmcExt *ext = nullptr)
{
    mceik_fsm_batch &fb = pipe < 0 ? s->fb : s->pfb[pipe];
    void *ws = pipe >= 0 ? s->pws[pipe] : s->ws;
    const size_t ws_bytes = pipe >= 0 ? s->pws_bytes[pipe] : s->ws_bytes;
    const hipStream_t st = pipe < 0 ? s->stream : s->pst[pipe];
    int r = 0;
    if (timed) {
        // the ring slot of launch nlaunch - RING is reused: fold that launch first
        while (s->ev_folded <= s->nlaunch - MCEIK_EV_RING) {
            if (fold_launch(s, s->ev_folded)) return -1;
            s->ev_folded++;
        }
        r = (int)(s->nlaunch % MCEIK_EV_RING);
        while (s->ev_made <= r) {
            HIPCHK(hipEventCreate(&s->ev[2 * s->ev_made]));
            HIPCHK(hipEventCreate(&s->ev[2 * s->ev_made + 1]));
            s->ev_made++;
        }
        HIPCHK(hipEventRecord(s->ev[2 * r], st));
    }
    if (fsm_batch_solve_impl(&fb, ws, ws_bytes, st, ext)) return -1;
    s->last_ttab = s->fb.ttab;
    if (timed) {
        HIPCHK(hipEventRecord(s->ev[2 * r + 1], st));
        s->nlaunch++;
    }
    if (s->d_order && pipe < 0) {       // the next launch pulls this launch's longest solves first
        HIPCHK(mcmc_lpt_order(s->d_clock, s->fb.nmodel * s->fb.nstat, s->d_order, s->stream));
        s->fb.solve_order = s->d_order;
    }
    return 0;
}

// Untimed forward of every model of every chain (init, restore): tables into
// ttab_cur (nphase 2) or the step tables (nphase 1).
static int mcmc_forward_all(mceik_mcmc *s)
{
    if (mceik_fsm_batch_solve(&s->fb_all, s->ws, s->ws_bytes, s->stream)) return -1;
    s->last_ttab = s->fb_all.ttab;
    return 0;
}

// MCEIK_SOLVE_CLOCK_REPORT=1: how busy the persistent waves were in the last
// launch (sum of solve durations / (waves x launch span)); synchronises.
static void clock_report(mceik_mcmc *s, const char *tag)
{
    const size_t n = (size_t)s->fb.nmodel * s->fb.nstat;
    std::vector<unsigned long long> clk(n * 2);
    if ((s->npipe > 1 ? hipDeviceSynchronize() : hipStreamSynchronize(s->stream)) != hipSuccess ||
        hipMemcpy(clk.data(), s->d_clock, clk.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    unsigned long long t0 = ~0ull, t1 = 0;
    double busy = 0.0, dmin = 1e30, dmax = 0.0;
    for (size_t i = 0; i < clk.size(); i += 2) {
        t0 = clk[i] < t0 ? clk[i] : t0;
        t1 = clk[i + 1] > t1 ? clk[i + 1] : t1;
        const double d = (double)(clk[i + 1] - clk[i]);
        busy += d;
        dmin = d < dmin ? d : dmin;
        dmax = d > dmax ? d : dmax;
    }
    const int nw = ws_layout(&s->fb).nwaves;
    fprintf(stderr, "mceik solve clock (%s, %s order): %zu solves on %d waves, launch %.1f ms, solve %.1f..%.1f ms "
                    "(mean %.1f), waves busy %.2f%%\n", tag, s->d_order ? "longest-first" : "id", n, nw,
            (t1 - t0) * 1e-5, dmin * 1e-5, dmax * 1e-5, busy / n * 1e-5, 100.0 * busy / ((double)nw * (double)(t1 - t0)));
}

// A view of chains [off, off + n) of the sampler's device state / batch.
static McmcDev dev_view(const McmcDev &D, int off, int n)
{
    McmcDev V = D;
    const size_t o = (size_t)off, oc = o * D.ncm;
    V.nchains = n;
    V.chain_offset = D.chain_offset + off;
    V.v += oc; V.slow_cur += oc; V.slow_prop += oc;
    V.logl += o; V.naccept += o;
    V.prop_cell += o; V.prop_phase += o; V.prop_v += o; V.prop_inprior += o; V.prop_logu += o; V.accept += o;
    V.ttab += o * D.nstat * D.nev;
    if (V.ttab_cur) V.ttab_cur += o * D.nphase * D.nstat * D.nev;
    if (V.keep_v) V.keep_v += oc;
    if (V.keep_logl) V.keep_logl += o;
    return V;
}

static mceik_fsm_batch batch_view(const mceik_fsm_batch &b, int off, int n, size_t ncm)
{
    mceik_fsm_batch V = b;
    const size_t o = (size_t)off, os = o * b.nstat;
    V.nmodel = n;
    V.slow = (const float *)b.slow + o * ncm;       // a chain's models are ncm = nphase * ncell floats
    if (V.model_phase) V.model_phase = b.model_phase + o;
    V.ttab = b.ttab + os * b.nev;
    V.niter = b.niter + os;
    V.ierr = b.ierr + os;
    V.solve_order = nullptr;
    V.solve_clock = b.solve_clock ? b.solve_clock + 2 * os : nullptr;
    return V;
}

// np pipes: parts of the chains, their own streams and workspaces (pipe 0
// reuses the sampler's).  Returns nonzero on a HIP failure; falls back to one
// pipe (with a message) when the extra workspaces do not fit.
static int pipes_setup(mceik_mcmc *s, int np)
{
    const int nch = s->D.nchains;
    const size_t ncm = (size_t)s->D.ncm;
    // The scratch budget binds (large grids: fewer resident waves than the
    // occupancy allows): pipes would have to share those waves, and splitting
    // them lengthens each half's queue tail more than the other half fills
    // (C5: 24.3 vs 25.1 proposals/s, profiles/r03_cfg): run one pipe.
    const int w1 = ws_layout(&s->fb).nwaves;
    if (w1 < fsm_batch_waves_uncapped(&s->fb)) {
        fprintf(stderr, "mceik_mcmc_init: the FSM scratch budget caps the waves (%d); running one pipe\n", w1);
        return 0;
    }
    for (int k = 0; k < np; k++) {
        const int lo = (int)((long long)nch * k / np), hi = (int)((long long)nch * (k + 1) / np);
        s->pD[k] = dev_view(s->D, lo, hi - lo);
        s->pfb[k] = batch_view(s->fb, lo, hi - lo, ncm);
    }
    // workspaces: carved out of the sampler's own when they fit in it together
    // (budget-capped grids), else pipe 0 reuses it and the others get their own
    size_t sum = 0;
    for (int k = 0; k < np; k++) sum += (s->pws_bytes[k] = (mceik_fsm_workspace_bytes(&s->pfb[k]) + 255) & ~(size_t)255);
    bool fit = true;
    size_t extra = 0;
    if (sum <= s->ws_bytes) {
        size_t off = 0;
        for (int k = 0; k < np; k++) {
            s->pws[k] = (char *)s->ws + off;
            s->pws_own[k] = false;
            off += s->pws_bytes[k];
        }
    } else {
        fit = s->pws_bytes[0] <= s->ws_bytes;
        s->pws[0] = s->ws;
        s->pws_bytes[0] = s->ws_bytes;
        for (int k = 1; k < np && fit; k++) {
            extra += s->pws_bytes[k];
            if (hipMalloc(&s->pws[k], s->pws_bytes[k]) != hipSuccess) {
                (void)hipGetLastError();
                s->pws[k] = nullptr;
                fit = false;
            } else {
                s->pws_own[k] = true;
            }
        }
    }
    if (!fit) {
        for (int k = 0; k < np; k++) {
            if (s->pws_own[k] && s->pws[k]) hipFree(s->pws[k]);
            s->pws[k] = nullptr;
            s->pws_own[k] = false;
        }
        fprintf(stderr, "mceik_mcmc_init: %d pipes need %zu B more FSM workspace; running one pipe\n", np, extra);
        return 0;
    }
    s->npipe = np;                     // finalize releases whatever was created
    for (int k = 0; k < np; k++) {
        HIPCHK(hipStreamCreateWithFlags(&s->pst[k], hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&s->pjoin[k], hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&s->pfork, hipEventDisableTiming));
    return 0;
}

// After a forward: every solve's reference ierr must be 0 (a station on the
// grid's first node is the SETBCS quirk, fsm3d.f90:736-745, ierr = 1; its table
// would stay u_nan).  Synchronises; names the failing stations.
static int check_forward_ierr(mceik_mcmc *s, const char *who)
{
    const int np = s->D.nphase, ns = s->D.nstat;
    const size_t n = (size_t)s->D.nchains * np * ns;     // the full batch: [chain][phase][station]
    std::vector<int> ie(n);
    HIPCHK(hipStreamSynchronize(s->stream));
    HIPCHK(hipMemcpy(ie.data(), s->d_ierr, n * sizeof(int), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int ph = 0; ph < np; ph++)
        for (int st = 0; st < ns; st++) {
            int e = 0;
            for (int c = 0; c < s->D.nchains && !e; c++) e = ie[((size_t)c * np + ph) * ns + st];
            if (e) {
                fprintf(stderr, "%s: station %d (0-based)%s: eikonal solve ierr = %d%s\n", who, st,
                        np > 1 ? (ph ? ", S model" : ", P model") : "", e,
                        e == 1 ? " (source on the grid's first node or outside it, fsm3d.f90:736-745)" : "");
                bad = 1;
            }
        }
    return bad;
}

extern "C" int mceik_mcmc_init(const struct mceik_parms_struct *parms, const struct mceik_stations_struct *st,
                               const struct mceik_catalog_struct *cat, const mceik_mcmc_opts *o,
                               const int *v0, mceik_mcmc **out)
{
    if (!parms || !st || !cat || !o || !v0 || !out) return 1;
    *out = nullptr;
    if (parms->dx != parms->dy || parms->dx != parms->dz || parms->dx <= 0.0) {
        fprintf(stderr, "mceik_mcmc_init: the eikonal solver needs dx = dy = dz\n");
        return 1;
    }
    const int nphase = o->nphase <= 1 ? 1 : o->nphase;
    if (o->nx < 2 || o->ny < 2 || o->nz < 2 || o->nchains < 1 || st->nstat < 1 || cat->nevents < 1 ||
        o->vmin < 1 || o->vmax < o->vmin || o->dvmax < 1 || !(o->precision == 0 || o->precision == 32 ||
                                                              o->precision == 64) ||
        nphase > 2 || (nphase == 2 && (o->vsmin < 1 || o->vsmax < o->vsmin))) {
        fprintf(stderr, "mceik_mcmc_init: invalid options\n");
        return 1;
    }
    for (int e = 0; e < cat->nevents; e++)
        if (cat->obsPtr[e + 1] < cat->obsPtr[e]) {
            fprintf(stderr, "mceik_mcmc_init: obsPtr must be non-decreasing\n");
            return 1;
        }
    const int nstat = st->nstat, nev = cat->nevents, nch = o->nchains;
    const int nobs = cat->obsPtr[nev];
    // observations fit: used P picks, and used S picks against the S model
    // (nphase 2); a P-only sampler refuses a catalog with S picks unless told
    // to ignore them (mask_s), so no observation disappears silently
    int nsused = 0;
    for (int j = 0; j < nobs; j++) {
        const int k = cat->statPtr[j] - 1;
        if (cat->luseObs[j] != 0 && cat->pickType[j] == S_PRIMARY_PICK && k >= 0 && k < nstat) nsused++;
    }
    if (nphase == 1 && nsused > 0) {
        if (!o->mask_s) {
            fprintf(stderr, "mceik_mcmc_init: the catalog holds %d used S picks; set nphase = 2 (joint P and S "
                            "models) or mask_s = 1 (fit the P picks only)\n", nsused);
            return 1;
        }
        fprintf(stderr, "mceik_mcmc_init: ignoring %d S picks (nphase 1, mask_s)\n", nsused);
    }
    auto fit_obs = [&](int j) {
        const int k = cat->statPtr[j] - 1;
        return cat->luseObs[j] != 0 && k >= 0 && k < nstat &&
               (cat->pickType[j] == P_PRIMARY_PICK || (nphase == 2 && cat->pickType[j] == S_PRIMARY_PICK));
    };
    for (int j = 0; j < nobs; j++)
        if (fit_obs(j) && !(cat->varObs[j] > 0.0)) {
            fprintf(stderr, "mceik_mcmc_init: observation %d has varObs <= 0\n", j);
            return 1;
        }
    // station coordinates are metres on the grid (lcartesian = 1, as homog.c
    // sets them); geographic station lists are not converted
    if (st->lcartesian != 1) {
        fprintf(stderr, "mceik_mcmc_init: stations.lcartesian = %d: only Cartesian station coordinates (metres, "
                        "lcartesian = 1) are supported\n", st->lcartesian);
        return 1;
    }
    // Tables only for the phases a station has picks of (lhasP / lhasS,
    // mceik_struct.h:43-46; homog.c:313-335 builds exactly those): the other
    // solves are skipped.  A fit pick at a station without its flag would
    // read a table never made, so the catalog is refused.
    std::vector<unsigned char> skip((size_t)nphase * nstat, 0);
    for (int k = 0; k < nstat; k++) {
        skip[k] = st->lhasP ? st->lhasP[k] == 0 : 0;
        if (nphase == 2) skip[(size_t)nstat + k] = st->lhasS ? st->lhasS[k] == 0 : 0;
    }
    for (int j = 0; j < nobs; j++)
        if (fit_obs(j)) {
            const int k = cat->statPtr[j] - 1, sph = cat->pickType[j] == S_PRIMARY_PICK;
            if (skip[(size_t)sph * nstat + k]) {
                fprintf(stderr, "mceik_mcmc_init: observation %d is a used %s pick at station %d (1-based) whose "
                                "%s = 0\n", j, sph ? "S" : "P", k + 1, sph ? "lhasS" : "lhasP");
                return 1;
            }
        }
    int nskip = 0;
    for (unsigned char c : skip) nskip += c;
    DeviceScope dg(o->device);
    if (hipSetDevice(o->device) != hipSuccess) return -1;
    mceik_mcmc *s = new mceik_mcmc();
    s->device = o->device;
    s->stream = nullptr;
    s->step = 0;
    s->nkept = 0;
    s->masked_s = nphase == 1 ? nsused : 0;
    s->nburn = parms->mcparms.nburnIn;
    s->keepk = parms->mcparms.keepK > 0 ? parms->mcparms.keepK : 1;
    s->niter_total = parms->mcparms.niter;
    s->max_samples = o->max_samples > 0 ? o->max_samples : 0;
    int nrx = parms->nrefx > 0 ? parms->nrefx : 1, nry = parms->nrefy > 0 ? parms->nrefy : 1,
        nrz = parms->nrefz > 0 ? parms->nrefz : 1;
    int ncx = mceik_div_up(o->nx, nrx), ncy = mceik_div_up(o->ny, nry), ncz = mceik_div_up(o->nz, nrz);
    int ncell = ncx * ncy * ncz;
    const int ncm = ncell * nphase;
    McmcDev &D = s->D;
    memset(&D, 0, sizeof(D));
    D.nchains = nch; D.chain_offset = o->chain_offset; D.ncell = ncell; D.nstat = nstat; D.nev = nev;
    D.nphase = nphase; D.ncm = ncm;
    D.keep_stride = nch;
    D.vmin = o->vmin; D.vmax = o->vmax; D.dvmax = o->dvmax; D.seed = o->seed;
    D.vsmin = nphase == 2 ? o->vsmin : 0; D.vsmax = nphase == 2 ? o->vsmax : 0;
    // host-side problem tables
    std::vector<double> src((size_t)nstat * 4);
    for (int i = 0; i < nstat; i++) {
        src[i * 4 + 0] = 0.0; src[i * 4 + 1] = st->xrec[i]; src[i * 4 + 2] = st->yrec[i]; src[i * 4 + 3] = st->zrec[i];
    }
    std::vector<int> ev(nev);
    std::vector<float> evf(o->tt_interp ? (size_t)nev * 3 : 0);
    for (int e = 0; e < nev; e++) {
        int ix, iy, iz;
        if (o->tt_interp) {   // lowest corner of the event's cell + fractions (trilinear mode)
            ix = cell_corner(o->nx, parms->x0, parms->dx, cat->xsrc[e], &evf[3 * e]);
            iy = cell_corner(o->ny, parms->y0, parms->dx, cat->ysrc[e], &evf[3 * e + 1]);
            iz = cell_corner(o->nz, parms->z0, parms->dx, cat->zsrc[e], &evf[3 * e + 2]);
        } else {
            ix = source_index(o->nx, parms->x0, parms->dx, cat->xsrc[e]);
            iy = source_index(o->ny, parms->y0, parms->dx, cat->ysrc[e]);
            iz = source_index(o->nz, parms->z0, parms->dx, cat->zsrc[e]);
        }
        ev[e] = (iz * o->ny + iy) * o->nx + ix;
    }
    std::vector<int> ostat(nobs > 0 ? nobs : 1), omask(nobs > 0 ? nobs : 1), ophase(nobs > 0 ? nobs : 1);
    std::vector<double> tcorr(nobs > 0 ? nobs : 1);
    for (int j = 0; j < nobs; j++) {
        int k = cat->statPtr[j] - 1;
        int use = fit_obs(j);
        int sph = use && cat->pickType[j] == S_PRIMARY_PICK;
        ostat[j] = use ? k : 0;
        omask[j] = !use;
        ophase[j] = sph;
        const double *corr = sph ? st->scorr : st->pcorr;       // static corrections (mceik_struct.h:42-44)
        tcorr[j] = (use && corr) ? corr[k] : 0.0;
    }
    std::vector<float> sl((size_t)nch * ncm);
    for (size_t i = 0; i < sl.size(); i++) sl[i] = 1.0f / (float)v0[i];
    int rc = 0;
    double *d_src = nullptr;
    int *d_ev = nullptr, *d_optr = nullptr;
    float *d_tt = nullptr;
    int *d_niter = nullptr;
    rc |= dput(s, &d_src, src.data(), src.size());
    rc |= dput(s, &d_ev, ev.data(), ev.size());
    float *d_evf = nullptr;
    if (o->tt_interp) rc |= dput(s, &d_evf, evf.data(), evf.size());
    rc |= dput(s, &d_optr, (const int *)cat->obsPtr, (size_t)nev + 1);
    int *d_ostat = nullptr, *d_omask = nullptr, *d_ophase = nullptr;
    double *d_tobs = nullptr, *d_tcorr = nullptr, *d_var = nullptr;
    rc |= dput(s, &d_ostat, ostat.data(), ostat.size());
    rc |= dput(s, &d_omask, omask.data(), omask.size());
    rc |= dput(s, &d_ophase, ophase.data(), ophase.size());
    rc |= dput(s, &d_tobs, (const double *)cat->tobs, (size_t)(nobs > 0 ? nobs : 0));
    rc |= dput(s, &d_tcorr, tcorr.data(), tcorr.size());
    rc |= dput(s, &d_var, (const double *)cat->varObs, (size_t)(nobs > 0 ? nobs : 0));
    unsigned char *d_skip = nullptr;
    if (nskip) rc |= dput(s, &d_skip, skip.data(), skip.size());
    rc |= dput(s, &D.v, v0, (size_t)nch * ncm);
    rc |= dput(s, &D.slow_cur, sl.data(), sl.size());
    rc |= dput(s, &D.slow_prop, sl.data(), sl.size());
    rc |= dalloc(s, &D.logl, nch);
    rc |= dalloc(s, &D.naccept, nch);
    rc |= dalloc(s, &D.prop_cell, nch);
    rc |= dalloc(s, &D.prop_phase, nch);
    rc |= dalloc(s, &D.prop_v, nch);
    rc |= dalloc(s, &D.prop_inprior, nch);
    rc |= dalloc(s, &D.prop_logu, nch);
    rc |= dalloc(s, &D.accept, nch);
    rc |= dalloc(s, &d_tt, (size_t)nch * nstat * nev);
    if (nphase > 1) rc |= dalloc(s, &D.ttab_cur, (size_t)nch * nphase * nstat * nev);
    rc |= dalloc(s, &d_niter, (size_t)nch * nphase * nstat);
    rc |= dalloc(s, &s->d_ierr, (size_t)nch * nphase * nstat);
    rc |= dalloc(s, &s->d_iters, MCEIK_ITERS_N);       // [0] iterations, [1..4] visit_stats, [5] solves, [6..] traffic
    if (s->max_samples) {
        rc |= dalloc(s, &D.keep_v, (size_t)s->max_samples * nch * ncm);
        rc |= dalloc(s, &D.keep_logl, (size_t)s->max_samples * nch);
    }
    if (rc) { mceik_mcmc_finalize(&s); return -1; }
    D.ttab = d_tt; D.obs_ptr = d_optr; D.obs_stat = d_ostat; D.obs_mask = d_omask;
    D.obs_phase = nphase > 1 ? d_ophase : nullptr;
    D.tobs = d_tobs; D.tcorr = d_tcorr; D.var = d_var;
    // the step batch: one solve per (chain, station) of the model the proposal
    // changed (model_phase = prop_phase: the other model's tables stay valid)
    mceik_fsm_batch &b = s->fb;
    memset(&b, 0, sizeof(b));
    b.nx = o->nx; b.ny = o->ny; b.nz = o->nz; b.h = parms->dx;
    b.x0 = parms->x0; b.y0 = parms->y0; b.z0 = parms->z0;
    b.maxit = parms->eikparms.maxit; b.tol = parms->eikparms.tol;
    b.precision = o->precision == 64 ? 64 : 32;
    b.nmodel = nch; b.nstat = nstat; b.nsrc = 1; b.src = d_src;
    b.slow_mode = 1; b.slow = D.slow_prop; b.nrx = nrx; b.nry = nry; b.nrz = nrz;
    b.model_phase = nphase > 1 ? D.prop_phase : nullptr;
    b.nphase = nphase;
    b.nev = nev; b.ev_node = d_ev; b.ev_frac = d_evf; b.ttab = d_tt; b.u_out = nullptr; b.niter = d_niter; b.ierr = s->d_ierr;
    b.max_sweeps = -1;
    b.iter_total = s->d_iters;
    b.visit_stats = s->d_iters + 1;
    b.solve_count = s->d_iters + 5;
    b.traffic = s->d_iters + 6;
    b.skip = d_skip;
    b.max_waves = o->max_waves > 0 ? o->max_waves : 0;
    // f = h/v stays a normal float: the short correctly rounded sqrt (fp32 only)
    const int vhi = nphase == 2 ? std::max(o->vmax, o->vsmax) : o->vmax;
    b.fast_sqrt = parms->dx / (double)vhi >= 1e-12 ? 1 : 0;      // f = h*s >= 1e-12: the short sqrt (fp32, fp64)
    // the full batch (init, restore): every model of every chain, models
    // [chain][phase] in place of model_phase, tables into ttab_cur
    s->fb_all = b;
    if (nphase > 1) {
        s->fb_all.nmodel = nch * nphase;
        s->fb_all.model_phase = nullptr;
        s->fb_all.ttab = D.ttab_cur;
    }
    s->last_ttab = s->fb_all.ttab;
    s->ws_bytes = std::max(mceik_fsm_workspace_bytes(&b), mceik_fsm_workspace_bytes(&s->fb_all));
    if (hipMalloc(&s->ws, s->ws_bytes) != hipSuccess) {
        fprintf(stderr, "mceik_mcmc_init: cannot allocate %zu B of FSM workspace\n", s->ws_bytes);
        s->ws = nullptr;
        mceik_mcmc_finalize(&s);
        return -1;
    }
    // initial log-likelihood of every chain.  Every launch stamps its solves
    // (solve_clock) and with MCEIK_LPT=1 the next launch drains each queue
    // longest solve first (mcmc_lpt_order; the init forward runs in id order).
    // Off by default: at C3 the waves are 96.6% busy in id order and longest-
    // first made the mean solve 4% slower.
    // MCEIK_SOLVE_CLOCK_REPORT=1: print how busy the persistent waves were
    // (init forward; diagnostic for the work-queue tail)
    const char *lpt_env = getenv("MCEIK_LPT");
    const bool lpt = lpt_env && lpt_env[0] == '1';
    const char *rep_env = getenv("MCEIK_SOLVE_CLOCK_REPORT");
    const bool report = rep_env && rep_env[0] == '1';
    if ((lpt || report) && dalloc(s, &s->d_clock, (size_t)nch * nphase * nstat * 2)) {
        mceik_mcmc_finalize(&s);
        return -1;
    }
    if (lpt && dalloc(s, &s->d_order, (size_t)nch * nstat)) {
        mceik_mcmc_finalize(&s);
        return -1;
    }
    b.solve_clock = s->d_clock;
    b.solve_order = nullptr;
    s->fb_all.solve_clock = s->d_clock;
    s->fb_all.solve_order = nullptr;
    if (mcmc_forward_all(s) || mcmc_init_loglik(D, s->stream) != hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess) {
        mceik_mcmc_finalize(&s);
        return -1;
    }
    if (check_forward_ierr(s, "mceik_mcmc_init")) {
        mceik_mcmc_finalize(&s);
        return 2;
    }
    s->report = report;
    if (report) clock_report(s, "init");
    s->npipe = 1;
    // Multi-step launches by default where a step is at most
    // 4 solves per resident wave (the per-step tail is then a large share: C2
    // +1.1% over two pipes; at C3's 16 solves per wave two pipes are 1% ahead);
    // MCEIK_PERSIST=1 / 0 forces them on / off
    const char *persist_env = getenv("MCEIK_PERSIST");
    const bool short_steps = (long long)b.nmodel * b.nstat <= 4LL * ws_layout(&b).nwaves;
    s->persist = (persist_env ? persist_env[0] == '1' : short_steps) && b.precision == 32 &&
                 mceik_fsm_step_z(&b) == 16 && !lpt;
    if (s->persist && (dalloc(s, &s->d_sync, MC_SYNC_WORDS(nch)) || dput(s, &s->d_dev, &D, 1))) {
        mceik_mcmc_finalize(&s);
        return -1;
    }
    // MCEIK_MC_SPIN_LIMIT (test hook): polls before a multi-step wait gives up
    const char *spin_env = getenv("MCEIK_MC_SPIN_LIMIT");
    s->spin_limit = spin_env ? (unsigned)strtoul(spin_env, nullptr, 10) : 1u << 24;
    const char *pipe_env = getenv("MCEIK_PIPES");       // default 2; MCEIK_PIPES=1: one pipe
    int np = s->persist ? 1 : pipe_env ? atoi(pipe_env) : 2;
    np = np < 1 ? 1 : np > MCEIK_MAX_PIPES ? MCEIK_MAX_PIPES : np;
    if (np > nch) np = nch;
    if (np > 1 && pipes_setup(s, np)) {
        mceik_mcmc_finalize(&s);
        return -1;
    }
    hipMemset(s->d_iters, 0, MCEIK_ITERS_N * sizeof(unsigned long long));
    *out = s;
    return 0;
}

extern "C" int mceik_mcmc_set_stream(mceik_mcmc *s, void *stream)
{
    if (!s) return 1;
    s->stream = (hipStream_t)stream;
    return 0;
}

// Steps of one call.  Returns -1 on a HIP failure; the caller joins the pipes
// whatever happened, so the caller's stream is always ordered after every
// kernel this call queued on the internal streams.
static int mcmc_steps(mceik_mcmc *s, int nsteps)
{
    if (s->persist) {
        // the first step's proposals here, then up to MCEIK_MC_CHUNK steps per
        // FSM launch (the kernel accepts, keeps and proposes the rest)
        for (int done = 0; done < nsteps;) {
            const int n = std::min(nsteps - done, MCEIK_MC_CHUNK);
            McmcExt x;
            x.dev = s->d_dev; x.sync = s->d_sync; x.spin_limit = s->spin_limit;
            x.step0 = (int)s->step; x.nsteps = n;
            x.nburn = s->nburn; x.keepk = s->keepk; x.maxs = s->max_samples; x.nkept0 = s->nkept;
            HIPCHK(mcmc_propose(s->D, (uint64_t)s->step, s->stream));
            if (mcmc_forward(s, true, -1, &x)) return -1;
            for (int i = 0; i < n; i++, s->step++)
                if (s->max_samples && s->step >= s->nburn && (s->step - s->nburn) % s->keepk == 0) s->nkept++;
            if (s->report) clock_report(s, "steps");
            done += n;
        }
        return 0;
    }
    const int np = s->npipe;
    for (int i = 0; i < nsteps; i++) {
        uint64_t step = (uint64_t)s->step;
        int slot = -1;
        if (s->max_samples && s->step >= s->nburn && (s->step - s->nburn) % s->keepk == 0) {
            slot = s->nkept % s->max_samples;
            s->nkept++;
        }
        if (np > 1) {
            for (int k = 0; k < np; k++) {
                HIPCHK(mcmc_propose(s->pD[k], step, s->pst[k]));
                if (mcmc_forward(s, true, k)) return -1;
                HIPCHK(mcmc_accept(s->pD[k], slot, s->pst[k]));
            }
        } else {
            HIPCHK(mcmc_propose(s->D, step, s->stream));
            if (mcmc_forward(s, true)) return -1;
            HIPCHK(mcmc_accept(s->D, slot, s->stream));
        }
        if (s->report) clock_report(s, "step");
        s->step++;
    }
    return 0;
}

extern "C" int mceik_mcmc_run(mceik_mcmc *s, int nsteps)
{
    if (!s) return 1;
    if (nsteps < 0) {
        const long long left = (long long)s->niter_total - s->step;
        nsteps = left > 0 ? (int)left : 0;
    }
    DeviceScope dg(s->device);
    const int np = s->npipe;
    if (np > 1) {                       // both pipes start after the caller's stream
        HIPCHK(hipEventRecord(s->pfork, s->stream));
        for (int k = 0; k < np; k++) HIPCHK(hipStreamWaitEvent(s->pst[k], s->pfork, 0));
    }
    int rc = mcmc_steps(s, nsteps);
    if (np > 1) {                       // the caller's stream continues after every pipe, also on failure
        for (int k = 0; k < np; k++) {
            if (hipEventRecord(s->pjoin[k], s->pst[k]) != hipSuccess ||
                hipStreamWaitEvent(s->stream, s->pjoin[k], 0) != hipSuccess) {
                // cannot order the caller's stream after pipe k: wait for it here
                if (hipStreamSynchronize(s->pst[k]) != hipSuccess) rc = -1;
                rc = rc ? rc : -1;
            }
        }
    }
    return rc;
}

// After a stream synchronisation: a multi-step launch whose wave gave up
// waiting for a chain's step (the broken-queue flag) failed, and the chains'
// state is not to be trusted; every later synchronising call (and the
// gather, through mcmc_shard_view) reports it until mceik_mcmc_restore
// reloads a state.
static int mc_queue_check(mceik_mcmc *s, const char *who)
{
    if (!s->persist) return 0;
    unsigned flag = 0;
    HIPCHK(hipMemcpy(&flag, s->d_sync + MC_SYNC_WORDS(s->D.nchains) - 1, sizeof(flag), hipMemcpyDeviceToHost));
    if (!flag) return 0;
    fprintf(stderr, "%s: a multi-step launch timed out waiting for a chain's previous step (broken work queue); "
                    "the chain state is invalid\n", who);
    return -1;
}

extern "C" int mceik_mcmc_sync(mceik_mcmc *s)
{
    if (!s) return 1;
    DeviceScope dg(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    return mc_queue_check(s, "mceik_mcmc_sync");
}

extern "C" int mceik_mcmc_get_state(mceik_mcmc *s, int *v, double *logl, long long *naccept, long long *step)
{
    if (!s) return 1;
    DeviceScope dg(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    if (mc_queue_check(s, "mceik_mcmc_get_state")) return -1;
    const McmcDev &D = s->D;
    if (v) HIPCHK(hipMemcpy(v, D.v, (size_t)D.nchains * D.ncm * 4, hipMemcpyDeviceToHost));
    if (logl) HIPCHK(hipMemcpy(logl, D.logl, (size_t)D.nchains * 8, hipMemcpyDeviceToHost));
    if (naccept) HIPCHK(hipMemcpy(naccept, D.naccept, (size_t)D.nchains * 8, hipMemcpyDeviceToHost));
    if (step) *step = s->step;
    return 0;
}

extern "C" int mceik_mcmc_checkpoint(mceik_mcmc *s, int *v, double *logl, long long *naccept, long long *step,
                                     int *nkept)
{
    if (!s) return 1;
    if (mceik_mcmc_get_state(s, v, logl, naccept, step)) return -1;
    if (nkept) *nkept = s->nkept;
    return 0;
}

extern "C" int mceik_mcmc_restore(mceik_mcmc *s, const int *v, const double *logl, const long long *naccept,
                                  long long step, int nkept)
{
    if (!s || !v || step < 0 || nkept < 0) return 1;
    DeviceScope dg(s->device);
    McmcDev &D = s->D;
    const size_t n = (size_t)D.nchains * D.ncm;
    for (size_t i = 0; i < n; i++) {
        const bool sph = (int)(i % (size_t)D.ncm) >= D.ncell;
        const int lo = sph ? D.vsmin : D.vmin, hi = sph ? D.vsmax : D.vmax;
        if (v[i] < lo || v[i] > hi) {
            fprintf(stderr, "mceik_mcmc_restore: v[%zu] = %d outside the prior [%d, %d]\n", i, v[i], lo, hi);
            return 1;
        }
    }
    std::vector<float> sl(n);
    for (size_t i = 0; i < n; i++) sl[i] = 1.0f / (float)v[i];
    HIPCHK(hipStreamSynchronize(s->stream));
    HIPCHK(hipMemcpy(D.v, v, n * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D.slow_cur, sl.data(), n * sizeof(float), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D.slow_prop, sl.data(), n * sizeof(float), hipMemcpyHostToDevice));
    if (naccept) HIPCHK(hipMemcpy(D.naccept, naccept, (size_t)D.nchains * 8, hipMemcpyHostToDevice));
    else HIPCHK(hipMemset(D.naccept, 0, (size_t)D.nchains * 8));
    if (logl) {
        HIPCHK(hipMemcpy(D.logl, logl, (size_t)D.nchains * 8, hipMemcpyHostToDevice));
    } else {
        // one forward of the restored models (not timed, not counted in the FSM stats)
        unsigned long long keep[MCEIK_ITERS_N];
        HIPCHK(hipMemcpy(keep, s->d_iters, sizeof(keep), hipMemcpyDeviceToHost));
        if (mcmc_forward_all(s)) return -1;
        HIPCHK(mcmc_init_loglik(D, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipMemcpy(s->d_iters, keep, sizeof(keep), hipMemcpyHostToDevice));
        if (check_forward_ierr(s, "mceik_mcmc_restore")) return 2;
    }
    s->step = step;
    s->nkept = nkept;
    s->nkept_base = nkept;
    if (s->persist) {
        // the restored state replaces whatever a broken multi-step launch left: clear its flag
        HIPCHK(hipMemset(s->d_sync + MC_SYNC_WORDS(s->D.nchains) - 1, 0, sizeof(unsigned)));
    }
    return 0;
}

extern "C" int mceik_mcmc_get_samples(mceik_mcmc *s, void *v_out, double *logl_out, int max, int kind, int *nkept)
{
    if (!s) return 1;
    int have = std::min(s->nkept - s->nkept_base, s->max_samples);
    int n = have < max ? have : max;
    if (nkept) *nkept = n;
    if (n <= 0) return 0;
    DeviceScope dg(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    if (mc_queue_check(s, "mceik_mcmc_get_samples")) return -1;
    hipMemcpyKind k = kind ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const size_t per = (size_t)s->D.nchains * s->D.ncm;
    // ring slot of the i-th of the n most recent states: (nkept - n + i) mod max_samples
    int i = 0;
    while (i < n) {
        const int slot = (int)(((long long)s->nkept - n + i) % s->max_samples);
        const int run = std::min(n - i, s->max_samples - slot);     // contiguous slots
        if (v_out)
            HIPCHK(hipMemcpy((int *)v_out + (size_t)i * per, s->D.keep_v + (size_t)slot * per,
                             (size_t)run * per * 4, k));
        if (logl_out)
            HIPCHK(hipMemcpy(logl_out + (size_t)i * s->D.nchains, s->D.keep_logl + (size_t)slot * s->D.nchains,
                             (size_t)run * s->D.nchains * 8, k));
        i += run;
    }
    return 0;
}

// Device view of this sampler's chain shard for comm.hip's gather: which = 0
// the current state, 1 the most recent kept state (1 if none is kept).
int mcmc_shard_view(mceik_mcmc *s, int which, McmcShard *out)
{
    if (!s || !out) return 1;
    const McmcDev &D = s->D;
    out->device = s->device; out->stream = s->stream;
    out->nchains = D.nchains; out->chain_offset = D.chain_offset; out->ncell = D.ncm;
    {   // a broken multi-step launch left no valid state to gather (-1)
        DeviceScope dg(s->device);
        if (hipStreamSynchronize(s->stream) != hipSuccess || mc_queue_check(s, "mceik_mcmc_gather")) return -1;
    }
    if (which == 0) {
        out->v = D.v; out->logl = D.logl;
        return 0;
    }
    if (s->max_samples <= 0 || s->nkept - s->nkept_base <= 0) return 1;
    const int slot = (int)(((long long)s->nkept - 1) % s->max_samples);
    out->v = D.keep_v + (size_t)slot * D.nchains * D.ncm;
    out->logl = D.keep_logl + (size_t)slot * D.nchains;
    return 0;
}

extern "C" int mceik_mcmc_last(mceik_mcmc *s, const float **ttab, const int **niter, const unsigned char **accept,
                               const int **ierr)
{
    if (!s) return 1;
    if (ttab) *ttab = s->last_ttab;
    if (niter) *niter = s->fb.niter;
    if (accept) *accept = s->D.accept;
    if (ierr) *ierr = s->d_ierr;
    return 0;
}

extern "C" int mceik_mcmc_last_phase(mceik_mcmc *s, const int **phase)
{
    if (!s || !phase) return 1;
    *phase = s->D.prop_phase;
    return 0;
}

extern "C" int mceik_mcmc_get_info(mceik_mcmc *s, mceik_mcmc_info *info)
{
    if (!s || !info) return 1;
    DeviceScope dg(s->device);
    memset(info, 0, sizeof(*info));
    info->npipe = s->npipe;
    info->multi_step = s->persist ? 1 : 0;
    info->nphase = s->D.nphase;
    info->masked_s = s->masked_s;
    FsmLaunch L;
    fill_launch(L, &s->fb);
    const int is_double = s->fb.precision == 64;
    info->step_z = fsm_launch_kind(L, is_double);
    info->fixed_layout = info->step_z == 16 && fsm16_fixed_layout(L) ? 1 : 0;
    info->lds_bytes = fsm_launch_lds_bytes(L, is_double);
    snprintf(info->kernel, sizeof(info->kernel), "%s", fsm_launch_name(L, is_double));
    for (int k = 0; k < s->npipe && k < 4; k++) {
        const mceik_fsm_batch &b = s->npipe > 1 ? s->pfb[k] : s->fb;
        info->chains[k] = b.nmodel;
        info->waves[k] = ws_layout(&b).nwaves;
        info->workspace_bytes[k] = s->npipe > 1 ? s->pws_bytes[k] : s->ws_bytes;
    }
    return 0;
}

extern "C" int mceik_mcmc_fsm_stats(mceik_mcmc *s, double *fsm_ms, long long *nlaunch, unsigned long long *iters,
                                    unsigned long long *visits, int reset)
{
    if (!s) return 1;
    DeviceScope dg(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    if (mc_queue_check(s, "mceik_mcmc_fsm_stats")) return -1;
    while (s->ev_folded < s->nlaunch) {
        if (fold_launch(s, s->ev_folded)) return -1;
        s->ev_folded++;
    }
    unsigned long long it[MCEIK_ITERS_N] = {0};
    HIPCHK(hipMemcpy(it, s->d_iters, sizeof(it), hipMemcpyDeviceToHost));
    {   // accounting build: requested bytes per launch by category
        unsigned long long tsum = 0;
        for (int k = 0; k < MCEIK_TRAFFIC_N; k++) tsum += it[6 + k];
        if (tsum && s->nlaunch) {
            static const char *nm[MCEIK_TRAFFIC_N] = {"own_load", "halo_load", "zup_load", "own_store",
                                                      "u0_store", "cell_load", "verify_load", "init_gather"};
            fprintf(stderr, "mceik traffic (requested bytes per FSM launch, %lld launches):", s->nlaunch);
            for (int k = 0; k < MCEIK_TRAFFIC_N; k++) fprintf(stderr, " %s=%.6e", nm[k], (double)it[6 + k] / s->nlaunch);
            fprintf(stderr, " total=%.6e\n", (double)tsum / s->nlaunch);
        }
    }
    if (fsm_ms) *fsm_ms = s->fsm_ms;
    if (nlaunch) *nlaunch = s->nlaunch;
    if (iters) *iters = it[0];
    if (visits) { visits[0] = it[1]; visits[1] = it[2]; visits[2] = it[3]; visits[3] = it[4]; }
    if (reset) {
        s->fsm_ms = 0.0;
        s->nlaunch = 0;
        s->ev_folded = 0;
        HIPCHK(hipMemset(s->d_iters, 0, MCEIK_ITERS_N * sizeof(unsigned long long)));
    }
    return 0;
}

extern "C" int mceik_mcmc_fsm_solves(mceik_mcmc *s, unsigned long long *solves)
{
    if (!s || !solves) return 1;
    DeviceScope dg(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    if (mc_queue_check(s, "mceik_mcmc_fsm_solves")) return -1;
    HIPCHK(hipMemcpy(solves, s->d_iters + 5, sizeof(*solves), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int mceik_mcmc_finalize(mceik_mcmc **ps)
{
    if (!ps || !*ps) return 0;
    mceik_mcmc *s = *ps;
    DeviceScope dg(s->device);
    hipStreamSynchronize(s->stream);
    for (int k = 0; k < MCEIK_MAX_PIPES; k++) {
        if (s->pst[k]) {
            hipStreamSynchronize(s->pst[k]);
            hipStreamDestroy(s->pst[k]);
        }
        if (s->pjoin[k]) hipEventDestroy(s->pjoin[k]);
    }
    if (s->pfork) hipEventDestroy(s->pfork);
    for (int k = 0; k < MCEIK_MAX_PIPES; k++) if (s->pws_own[k] && s->pws[k]) hipFree(s->pws[k]);
    for (void *p : s->allocs) hipFree(p);
    for (int i = 0; i < 2 * s->ev_made; i++) hipEventDestroy(s->ev[i]);
    if (s->ws) hipFree(s->ws);
    delete s;
    *ps = nullptr;
    return 0;
}
