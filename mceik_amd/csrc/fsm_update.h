// fsm_update.h -- the Godunov local update shared by the batched sweep kernel
// (fsm_kernel.hip) and the single-solve kernel (fsm_single.hip):
// SOLVE_HAMILTONIAN2D/3D + SORT3 (fsm3d.f90:562-693) in fp64, literally, and
// the stable fp32 form that oracle/fsm_impl.inc STABLE_UPDATE restates.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

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

// The same update without branches: the sorted triple by
// min / max / median, the 1D, 2D and 3D candidates all computed, the
// reference's choice made by selects.  Values and ierr identical to godunov()
// (inputs are never NaN; a root of a negative radicand is NaN only in a
// candidate that is not selected, or gives the reference's ierr 3).  A wave
// whose lanes take different branches runs every branch anyway; this form
// drops the exec-mask bookkeeping and branches of the divergent code.
__device__ __forceinline__ double godunov_sel(double a, double b, double c, double f, int &ierr)
{
    const double UN = DBL_MAX;
    const double a1 = __builtin_fmin(__builtin_fmin(a, b), c);
    const double a3 = __builtin_fmax(__builtin_fmax(a, b), c);
    const double a2 = __builtin_fmax(__builtin_fmin(a, b), __builtin_fmin(__builtin_fmax(a, b), c));
    const double x1 = a1 + f;
    const double amb = a1 - a2;
    const double arg = (2.0 * f) * f - amb * amb;
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
__device__ __forceinline__ float sqrt_normal(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const int sb = __builtin_bit_cast(int, s);
    const float dn = __builtin_bit_cast(float, sb - 1);
    const float up = __builtin_bit_cast(float, sb + 1);
    const int edn = __builtin_bit_cast(int, __builtin_fmaf(-dn, s, x));
    const int eup = __builtin_bit_cast(int, __builtin_fmaf(-up, s, x));
    // (asm: the instruction selector turns the clamp back into compares + carry adds)
    int pdn, pup;
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(pdn) : "v"(edn));
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(pup) : "v"(eup));
    return __builtin_bit_cast(float, (sb - 1) + pdn + pup);     // v_add3_u32 from the selector
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
    return r1 ? x1 : r2 ? x2 : (x3 < UN ? x3 : UN);
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
    return godunov_sel(a, b, c, f, ierr);   // fp64: the literal form's values without its branches
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
