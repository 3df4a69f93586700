// fsm_update.h -- the Godunov local update shared by the batched sweep kernel
// (fsm_kernel.hip) and the single-solve kernel (fsm_single.hip):
// SOLVE_HAMILTONIAN2D/3D + SORT3 (fsm3d.f90:562-693) in fp64, literally, and
// the stable fp32 form that oracle/fsm_impl.inc STABLE_UPDATE restates.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

#ifndef MCEIK_SQRT_ADD3_ASM
#define MCEIK_SQRT_ADD3_ASM 0     // 1: the add as an asm statement too (the compiler pads its use: +0.2% slower, tools A/B)
#endif
#ifndef MCEIK_SQRT_INT
#define MCEIK_SQRT_INT 1     // sqrt_normal's rounding choice in integer arithmetic (0: compares + selects)
#endif

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
// fp64: the reference's literal SOLVE_HAMILTONIAN2D/3D (fsm3d.f90:624-693).
// fp32: godunov_bl / godunov_v below, bitwise equal to oracle/fsm_impl.inc
// STABLE_UPDATE (increments relative to a1, one square root per solve).
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

// The same update without branches (MCEIK_F64_SELECT): the sorted triple by
// min / max / median, the 1D, 2D and 3D candidates all computed, the
// reference's choice made by selects.  Values and ierr identical to godunov()
// (inputs are never NaN; a root of a negative radicand is NaN only in a
// candidate that is not selected, or gives the reference's ierr 3).  A wave
// whose lanes take different branches runs every branch anyway; this form
// drops the exec-mask bookkeeping and branches of the divergent code.
#ifndef MCEIK_F64_SELECT
#define MCEIK_F64_SELECT 1
#endif
#ifndef MCEIK_F64_ONE_SQRT
#define MCEIK_F64_ONE_SQRT 0     // 1: one square root per node (bitwise; measured 13% slower, profiles/r03_f64one)
#endif
__device__ __forceinline__ double godunov_sel(double a, double b, double c, double f, int &ierr)
{
    const double UN = DBL_MAX;
    const double a1 = __builtin_fmin(__builtin_fmin(a, b), c);
    const double a3 = __builtin_fmax(__builtin_fmax(a, b), c);
    const double a2 = __builtin_fmax(__builtin_fmin(a, b), __builtin_fmin(__builtin_fmax(a, b), c));
    const double x1 = a1 + f;
    const double amb = a1 - a2;
    const double arg = (2.0 * f) * f - amb * amb;
#if MCEIK_F64_ONE_SQRT
    // One square root per node.  The reference takes the 3D root when the 2D
    // value x2 = 0.5*((a1 + a2) + sqrt(arg)) exceeds a3 (|a1 - a2| < f), i.e.
    // when sqrt(arg) > T = 2*a3 - (a1 + a2).  Outside a band of half-width
    // E = 2^-40 * (a1 + a2 + 2*a3 + 2*f) around T -- 2^11 times the rounding
    // of every quantity involved (all of them are sums of a1..a3, f and
    // sqrt(arg) <= sqrt(2) f) -- comparing arg with (T +- E)^2 gives the
    // reference's decision on its rounded x2, so only the chosen radicand is
    // square-rooted.  Inside the band (and for non-finite T or E) the lane
    // decides on the literal x2.  Values and ierr identical to godunov().
    const bool use2 = __builtin_fabs(amb) < f;
    const double S = a1 + a2;
    const double x2b = (a1 < a2 ? a1 : a2) + f;
    const double T = 2.0 * a3 - S;
    const double E = 0x1p-40 * ((S + 2.0 * a3) + 2.0 * f);
    const double tp = T + E, tm = T - E;
    const bool fin = E < 0x1p400;                           // T, E and their squares are finite
    const bool open3 = a3 == UN;                            // x2 is finite: never above DBL_MAX
    const bool sure3 = fin && !open3 && (tp < 0.0 || arg > tp * tp);   // sqrt(arg) > T + E: x2 > a3
    const bool sure2 = open3 || (fin && tm > 0.0 && arg < tm * tm);    // sqrt(arg) < T - E: x2 < a3
    const bool r1 = !(x1 > a2), nan_in = a1 == UN;
    bool d3 = use2 ? sure3 : x2b > a3;                      // the reference's 3D case
    if (use2 && !(sure3 || sure2)) d3 = 0.5 * (S + __builtin_sqrt(arg)) > a3;   // the band: its literal test
    const double qb = -((2.0 / 3.0) * ((a1 + a2) + a3));
    const double qc = ((((a1 * a1) + (a2 * a2)) + (a3 * a3)) - f * f) * (1.0 / 3.0);
    const double disc = qb * qb - 4.0 * qc;
    const double sq = __builtin_sqrt(d3 ? disc : arg);
    const double x2 = use2 ? 0.5 * (S + sq) : x2b;
    const double x3 = 0.5 * (-qb + sq);
    const bool in3 = x3 < UN;
    const int e3 = in3 ? (x3 < 0.0 ? 2 : (disc < 0.0 ? 1 : 0)) : 3;
    ierr = (nan_in || r1 || !d3) ? 0 : e3;
    return nan_in ? UN : r1 ? x1 : !d3 ? x2 : (in3 ? x3 : UN);
#else
    const double x2 = __builtin_fabs(amb) < f ? 0.5 * ((a1 + a2) + __builtin_sqrt(arg)) : (a1 < a2 ? a1 : a2) + f;
    const double qb = -((2.0 / 3.0) * ((a1 + a2) + a3));
    const double qc = ((((a1 * a1) + (a2 * a2)) + (a3 * a3)) - f * f) * (1.0 / 3.0);
    const double disc = qb * qb - 4.0 * qc;
    const double x3 = 0.5 * (-qb + __builtin_sqrt(disc));
    const bool in3 = x3 < UN;
    const bool r1 = !(x1 > a2), r2 = !(x2 > a3), nan_in = a1 == UN;
    const int e3 = in3 ? (x3 < 0.0 ? 2 : (disc < 0.0 ? 1 : 0)) : 3;
    ierr = (nan_in || r1 || r2) ? 0 : e3;
    return nan_in ? UN : r1 ? x1 : r2 ? x2 : (in3 ? x3 : UN);
#endif
}

// Correctly rounded sqrt for normal positive x (LLVM's expansion without the
// denormal rescale and zero/inf fix-up).  Used only where the radicand that
// is finally selected is provably a normal float: on the MCMC path f = h*s >=
// h/vmax (checked on the host) and the selected radicand exceeds f^2 (2D:
// 2f^2 - d2^2 with d2 < f; 3D: 3f^2 - (d2^2 + (d3^2 + (d3-d2)^2)) with both
// terms < f^2).
//
// The choice among dn = s - 1 ulp, s, up = s + 1 ulp (LLVM's: edn <= 0 -> dn,
// eup > 0 -> up, else s; eup > 0 implies edn > 0) is made in integer
// arithmetic: result bits = dn + [eup > 0] + [edn > 0], each [v > 0] the
// clamp med3_i32(bits(v), 0, 1) (v is finite: a positive float has positive
// bits, +-0 and negatives do not).  Same values as the compare/select form
// without its compare -> lane-mask -> select hazard wait states (gfx950 puts
// two wait states between a VALU write of an SGPR mask and its use).
#ifndef MCEIK_SQRT_ONESIDED
#define MCEIK_SQRT_ONESIDED 0    // 1: only the upper test (v_sqrt_f32 never above the correctly rounded
                                 // root), -1: only the lower test (never below); see tools/sqrt_dir_probe.hip
#endif
__device__ __forceinline__ float sqrt_normal(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const int sb = __builtin_bit_cast(int, s);
#if MCEIK_SQRT_ONESIDED != 0
    {
        // The exhaustive probe (tools/sqrt_dir_probe.hip) shows the hardware
        // root is off by at most one ulp and only on one side over the domain
        // x >= 2^-104, so one Tuckerman test decides: +1 ulp when x > up*s
        // (MCEIK_SQRT_ONESIDED 1), -1 ulp unless x > dn*s (-1).
        const float t = __builtin_bit_cast(float, sb + MCEIK_SQRT_ONESIDED);
        const int e = __builtin_bit_cast(int, __builtin_fmaf(-t, s, x));
        int p;
        asm("v_med3_i32 %0, %1, 0, 1" : "=v"(p) : "v"(e));
        return __builtin_bit_cast(float, MCEIK_SQRT_ONESIDED > 0 ? sb + p : (sb - 1) + p);
    }
#endif
    const float dn = __builtin_bit_cast(float, sb - 1);
    const float up = __builtin_bit_cast(float, sb + 1);
    const int edn = __builtin_bit_cast(int, __builtin_fmaf(-dn, s, x));
    const int eup = __builtin_bit_cast(int, __builtin_fmaf(-up, s, x));
#if MCEIK_SQRT_INT
    // (asm: the instruction selector turns the clamp back into compares + carry adds)
    int pdn, pup, r;
#if MCEIK_SQRT_ADD3_ASM == 2
    // one asm statement: the compiler pads a use of an asm result by a wait
    // state (it cannot see whether the asm wrote a transcendental result), so
    // the three instructions are one block and only r's use can be padded
    asm("v_med3_i32 %1, %3, 0, 1\n\tv_med3_i32 %2, %4, 0, 1\n\tv_add3_u32 %0, %5, %1, %2"
        : "=v"(r), "=&v"(pdn), "=&v"(pup) : "v"(edn), "v"(eup), "v"(sb - 1));
#else
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(pdn) : "v"(edn));
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(pup) : "v"(eup));
#if MCEIK_SQRT_ADD3_ASM
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(sb - 1), "v"(pdn), "v"(pup));
#else
    r = (sb - 1) + pdn + pup;           // v_add3_u32 from the selector
#endif
#endif
    return __builtin_bit_cast(float, r);
#else
    const float t = __builtin_bit_cast(float, edn) <= 0.0f ? dn : s;
    return __builtin_bit_cast(float, eup) > 0.0f ? up : t;
#endif
}

// min / max of two doubles as single instructions.  In IEEE mode the
// compiler quiets both operands of v_min_f64 / v_max_f64 first (a
// canonicalising v_max_f64 x, x, x per operand not known to be the result of
// arithmetic: every value loaded from LDS or HBM) in case one is a signalling
// NaN; travel times, slownesses and their sums are never NaN, so the bare
// instruction returns the same value.
__device__ __forceinline__ double dmin_(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double dmax_(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Correctly rounded fp64 sqrt for normal positive x below +inf: LLVM's
// expansion of __builtin_sqrt (v_rsq_f64 and two Newton-Raphson / Goldschmidt
// corrections, the same operations in the same order) without its input
// scaling for x < 2^-767 and its +-0 / +inf fix-up, so the result is bitwise
// __builtin_sqrt's for every such x.  Used only where the radicand finally
// selected is provably normal: the 2D radicand 2f^2 - (a1 - a2)^2 > f^2 when
// |a1 - a2| < f, the 3D one (4/9)(3f^2 - sum of the squared pairwise
// differences) > (4/9) f^2 when the 3D case is taken, and the host validates
// f = h * s >= 1e-12 (fp32's sqrt_normal, the same bound).  An unselected
// radicand may be anything: a negative or zero one gives NaN, never selected.
__device__ __forceinline__ double sqrt_normal_f64(double x)
{
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}

#ifndef MCEIK_F64_NOCLAMP
#define MCEIK_F64_NOCLAMP 0      // 1: drop the 3D root clamp (measured 1.1% slower, profiles/r04_ncl)
#endif
#ifndef MCEIK_F64_NOBRANCH
#define MCEIK_F64_NOBRANCH 0     // 1: the fast fp64 update as straight-line code (A/B)
#endif
// The literal fp64 update for the fast path (no ierr): godunov_sel's values
// with the sort and the minima as bare v_min_f64 / v_max_f64, the 2D root
// computed unconditionally and no early return (no divergent branch: the
// node updates of a brick form one basic block, so the scheduler can overlap
// the next node's LDS neighbour reads), and (FAST) the short sqrt.
// min(a1, a2) + f of the 2D fallback is x1 (a1 <= a2 by the sort).
template <bool FAST>
__device__ __forceinline__ double godunov_fast64(double a, double b, double c, double f)
{
    const double UN = DBL_MAX;
    const double mn = dmin_(a, b), mx = dmax_(a, b);
    const double a1 = dmin_(mn, c), a3 = dmax_(mx, c), a2 = dmax_(mn, dmin_(mx, c));
    const double x1 = a1 + f;
    const double amb = a1 - a2;
    const double arg = (2.0 * f) * f - amb * amb;
    const double s2 = FAST ? sqrt_normal_f64(arg) : __builtin_sqrt(arg);
    const double x2 = __builtin_fabs(amb) < f ? 0.5 * ((a1 + a2) + s2) : x1;
    const double qb = -((2.0 / 3.0) * ((a1 + a2) + a3));
    const double qc = ((((a1 * a1) + (a2 * a2)) + (a3 * a3)) - f * f) * (1.0 / 3.0);
    const double disc = qb * qb - 4.0 * qc;
    const double x3 = 0.5 * (-qb + (FAST ? sqrt_normal_f64(disc) : __builtin_sqrt(disc)));
    // (a1 == UN needs no test of its own: then a2 = UN too, x1 = UN + f rounds
    // to UN and the 1D case returns it -- the reference's early return)
    const bool r1 = !(x1 > a2), r2 = !(x2 > a3);
#if MCEIK_F64_NOBRANCH
    // the choice as masks on the bit patterns: no ternary for the optimiser to
    // turn into exec-masked branches (with the 2D / 3D arithmetic sunk into
    // them); instcombine folds each mask pair back into one select
    const unsigned long long m1 = 0ull - (unsigned long long)r1, m2 = 0ull - (unsigned long long)r2;
    const unsigned long long b3 = __builtin_bit_cast(unsigned long long, dmin_(x3, UN));
    const unsigned long long b23 = (__builtin_bit_cast(unsigned long long, x2) & m2) | (b3 & ~m2);
    return __builtin_bit_cast(double, (__builtin_bit_cast(unsigned long long, x1) & m1) | (b23 & ~m1));
#elif MCEIK_F64_NOCLAMP
    // The reference clamps the 3D root at u_nan.  The 3D case is selected
    // only when x1 > a2 and x2 > a3: with a2 = u_nan x1 = a1 + f cannot exceed
    // it (a1 + f rounds to u_nan at most), with a3 = u_nan the 2D root cannot
    // (it is a1-based, finite or x1), so a1..a3 are travel times, all finite
    // and far below u_nan / 4, and x3 = (-qb + sqrt(disc)) / 2 is too: the
    // clamp never acts on a selected value.  Dropping it drops the u_nan
    // constant (an SGPR pair the kernel spills) from the node update.
    return r1 ? x1 : r2 ? x2 : x3;
#else
    return r1 ? x1 : r2 ? x2 : (x3 < UN ? x3 : UN);
#endif
}

// Branchless fp32 Godunov update, values and ierr identical to the twin
// (oracle/fsm_impl.inc STABLE_UPDATE): 1D if f <= d2, else the 2D root unless
// d3^2 + (d3 - d2)^2 < f^2 (the 2D root would exceed d3), then the 3D root;
// only the selected radicand is square-rooted.
template <bool FAST>
__device__ __forceinline__ float godunov_bl(float a, float b, float c, float f, int &ierr)
{
    const float UN = FLT_MAX;
    const float a1 = fminf(fminf(a, b), c);
    const float a3 = fmaxf(fmaxf(a, b), c);
    const float a2 = __builtin_amdgcn_fmed3f(a, b, c);
    const float d2 = a2 - a1, d3 = a3 - a1;
    const float ff = f * f, e = d3 - d2;
    const float d22 = d2 * d2, d33 = d3 * d3;
    const float t = d33 + e * e;
    const bool two = t >= ff;
    const float r2 = (ff + ff) - d22;
    const float sm = d2 + d3;
    const float disc = (3.0f * ff) - (d22 + t);      // 3f^2 - (d2^2 + d3^2 + (d3-d2)^2)
    const float rad = two ? r2 : disc;
    const float s = FAST ? sqrt_normal(rad) : __builtin_sqrtf(rad);
    const float y23 = two ? 0.5f * (d2 + s) : (sm + s) * (1.0f / 3.0f);
    const bool one = !(f > d2);
    const float y = one ? f : y23;
    const float x = a1 + y;
    const bool ok = x < UN;
    const bool nan_in = a1 == UN;
    ierr = nan_in ? 0 : (!ok ? 3 : ((!one && !two && disc < 0.0f) ? 1 : 0));
    return (nan_in || !ok) ? UN : x;
}
template <bool FAST>
__device__ __forceinline__ double godunov_bl(double a, double b, double c, double f, int &ierr)
{
    return MCEIK_F64_SELECT ? godunov_sel(a, b, c, f, ierr) : godunov(a, b, c, f, ierr);   // fp64: literal form
}

// min of two travel times.  Values in the field are never NaN or -0 (every
// update is clamped to FLT_MAX, sources are ts + d*s >= +0), so for fp32 the
// unsigned order of the bit patterns is the float order: v_min_u32 needs no
// IEEE canonicalisation of its inputs (v_min_f32 does).
__device__ __forceinline__ float fmin_(float a, float b)
{
    const unsigned ia = __builtin_bit_cast(unsigned, a), ib = __builtin_bit_cast(unsigned, b);
    return __builtin_bit_cast(float, __builtin_elementwise_min(ia, ib));
}
__device__ __forceinline__ double fmin_(double a, double b) { return dmin_(a, b); }

}  // namespace
