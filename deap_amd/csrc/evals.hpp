// evals.hpp — device restatements of the DEAP objective functions
// (deap/benchmarks/__init__.py) for rows distributed over a lane group.
//
// Layout contract: a group of G lanes owns one genome row; in chunk c, lane
// `sub` holds genes [c*4G + 4*sub, +4) as doubles (float rows are widened
// exactly, as CPython does for array('f') items).  Each per-gene term below
// evaluates the reference expression in the reference's operation order
// (every binary op left to right, no FMA contraction: built with
// -ffp-contract=off); only the order of the final sum differs (tree vs
// left-to-right), which the 1e-12 relative tolerance of the parity tests
// covers.
#pragma once
#include "common.hpp"

namespace dm {

constexpr double PI = 3.141592653589793;  // math.pi

// Classification of objectives by the evaluation template they need.
enum EvalClass {
    EC_NONE = 0,
    EC_SUM = 1,    // single-objective sums, objective chosen at run time
    EC_MO = 2,     // ZDT / DTLZ
    EC_RAST = 3,   // rastrigin, specialised (benchmark hot path)
    EC_ROSEN = 4   // rosenbrock, specialised
};
__host__ __device__ constexpr bool ec_single(int ec) {
    return ec == EC_SUM || ec == EC_RAST || ec == EC_ROSEN;
}

__host__ __device__ inline int eval_class(int fn) {
    switch (fn) {
        case DM_EVAL_NONE: return EC_NONE;
        case DM_EVAL_RASTRIGIN: return EC_RAST;
        case DM_EVAL_ROSENBROCK: return EC_ROSEN;
        case DM_EVAL_ONEMAX:
        case DM_EVAL_SPHERE: return EC_SUM;
        default: return EC_MO;
    }
}
__host__ __device__ inline int eval_nobj(const dm_eval& ev) {
    switch (ev.fn) {
        case DM_EVAL_NONE: return 0;
        case DM_EVAL_ONEMAX:
        case DM_EVAL_RASTRIGIN:
        case DM_EVAL_ROSENBROCK:
        case DM_EVAL_SPHERE: return 1;
        case DM_EVAL_ZDT1:
        case DM_EVAL_ZDT2:
        case DM_EVAL_ZDT3:
        case DM_EVAL_ZDT4:
        case DM_EVAL_ZDT6: return 2;
        default: return ev.obj;
    }
}
// First gene index that enters the tail sum of a multi-objective function.
__host__ __device__ inline int mo_tail_start(const dm_eval& ev) {
    switch (ev.fn) {
        case DM_EVAL_ZDT1:
        case DM_EVAL_ZDT2:
        case DM_EVAL_ZDT3:
        case DM_EVAL_ZDT4:
        case DM_EVAL_ZDT6: return 1;
        default: return ev.obj - 1;  // DTLZ: xm = individual[obj-1:]
    }
}

// cos(a) for an already-rounded fp64 argument a (the reference evaluates
// cos(2*pi*gene) on the rounded product).  Cody-Waite reduction by pi/2 with
// three FMA terms (exact enough for |a| < 2^20*pi/2) and fdlibm's
// __kernel_sin/__kernel_cos minimax polynomials on |r| <= pi/4: <= 1 ulp,
// i.e. agrees with glibc's correctly rounded cos to within 1 ulp.  Larger
// arguments take ocml's Payne-Hanek path (never on the benchmark inputs).
// Explicit fma() is used only where the algorithm requires it; the build's
// -ffp-contract=off still forbids implicit contraction everywhere else.
__device__ __noinline__ double cos_slow(double a) { return cos(a); }

// Reduction + polynomials only (caller guarantees |a| < 1.6e6).
__device__ __forceinline__ double cos_core(double a) {
    constexpr double TWO_OVER_PI = 0.63661977236758138243;
    constexpr double PIO2_HI = 1.5707963267948966e+00;     // 0x3FF921FB54442D18
    constexpr double PIO2_MID = 6.123233995736766e-17;     // 0x3C91A62633145C07
    constexpr double PIO2_LO = -1.4973849048591698e-33;    // 0xB91F1976B7ED8FBC
    const double q = rint(a * TWO_OVER_PI);
    double r = fma(-q, PIO2_HI, a);
    r = fma(-q, PIO2_MID, r);
    r = fma(-q, PIO2_LO, r);
    const int quad = (int)(int64_t)q & 3;
    const double z = r * r;
    // __kernel_cos (y = 0), Horner with explicit FMAs
    double cr = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    cr = fma(z, cr, -2.75573143513906633035e-07);
    cr = fma(z, cr, 2.48015872894767294178e-05);
    cr = fma(z, cr, -1.38888888888741095749e-03);
    cr = fma(z, cr, 4.16666666666666019037e-02);
    cr = z * cr;
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + fma(z, cr, (1.0 - w) - hz);
    // __kernel_sin (y = 0)
    double sr = fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    sr = fma(z, sr, 2.75573137070700676789e-06);
    sr = fma(z, sr, -1.98412698298579493134e-04);
    sr = fma(z, sr, 8.33333333332248946124e-03);
    const double v = z * r;
    const double sn = fma(v, fma(z, sr, -1.66666666666666324348e-01), r);
    const double mag = (quad & 1) ? sn : c;
    return (quad == 1 || quad == 2) ? -mag : mag;
}
__device__ __forceinline__ double cos_fast(double a) {
    if (__builtin_expect(!(fabs(a) < 1.6e6), 0)) return cos_slow(a);
    return cos_core(a);
}
// Rastrigin term gene*gene - 10*cos(2*pi*gene)                            :239-240
__device__ __forceinline__ double rast_term(double x) {
    const double a = (2.0 * PI) * x;
    double c = cos_core(a);
    if (__builtin_expect(!(fabs(a) < 1.6e6), 0)) c = cos_slow(a);
    return x * x - 10.0 * c;
}

// Per-gene term of a single-objective sum (EC_SUM) for gene x.
__device__ __forceinline__ double sum_term(int fn, double x) {
    switch (fn) {
        case DM_EVAL_RASTRIGIN:  // gene*gene - 10*cos(2*pi*gene)          :239-240
            return x * x - 10.0 * cos_fast((2.0 * PI) * x);
        case DM_EVAL_SPHERE:  // gene*gene                                   :77
            return x * x;
        default:  // ONEMAX on real-valued genes: sum(individual)
            return x;
    }
}
// Rosenbrock pair term: 100*(x*x - y)**2 + (1. - x)**2                  :117-118
__device__ __forceinline__ double rosen_term(double x, double y) {
    const double a = x * x - y;
    const double b = 1.0 - x;
    return 100.0 * (a * a) + b * b;
}
// Tail term of the multi-objective functions.
__device__ __forceinline__ double mo_term(int fn, double x) {
    switch (fn) {
        case DM_EVAL_ZDT4: {  // xi**2 - 10*cos(4*pi*xi)                    :447
            return x * x - 10.0 * cos_fast((4.0 * PI) * x);
        }
        case DM_EVAL_DTLZ1:
        case DM_EVAL_DTLZ3: {  // (xi-0.5)**2 - cos(20*pi*(xi-0.5))    :489,:544
            // cos_fast: fdlibm's polynomials (<= 1 ulp, as ocml's cos) with one
            // small inlined copy; ocml's inlined cos took the lane-group kernels
            // past 240 VGPRs
            const double d = x - 0.5;
            return d * d - cos_fast((20.0 * PI) * d);
        }
        case DM_EVAL_DTLZ2:
        case DM_EVAL_DTLZ4: {  // (xi-0.5)**2                           :518,:574
            const double d = x - 0.5;
            return d * d;
        }
        default:  // ZDT1/2/3/6: sum(individual[1:])
            return x;
    }
}

// Final fitness of a multi-objective function from its tail sum S and the
// head genes x[0..7] (values, unweighted).  Writes nobj values into f.
__device__ inline void mo_finalize(const dm_eval& ev, int n, double S, const double* h,
                                   double* f) {
    switch (ev.fn) {
        case DM_EVAL_ZDT1: {  // :400-403
            const double g = 1.0 + 9.0 * S / (double)(n - 1);
            f[0] = h[0];
            f[1] = g * (1.0 - sqrt(h[0] / g));
            return;
        }
        case DM_EVAL_ZDT2: {  // :416-419
            const double g = 1.0 + 9.0 * S / (double)(n - 1);
            const double r = h[0] / g;
            f[0] = h[0];
            f[1] = g * (1.0 - r * r);
            return;
        }
        case DM_EVAL_ZDT3: {  // :432-435
            const double g = 1.0 + 9.0 * S / (double)(n - 1);
            const double r = h[0] / g;
            f[0] = h[0];
            f[1] = g * (1.0 - sqrt(r) - r * sin((10.0 * PI) * h[0]));
            return;
        }
        case DM_EVAL_ZDT4: {  // :447-450  (1 + 10*(n-1) is an int in Python)
            const double g = (double)(1 + 10 * (n - 1)) + S;
            f[0] = h[0];
            f[1] = g * (1.0 - sqrt(h[0] / g));
            return;
        }
        case DM_EVAL_ZDT6: {  // :462-465
            const double g = 1.0 + 9.0 * pow(S / (double)(n - 1), 0.25);
            const double f1 = 1.0 - exp(-4.0 * h[0]) * pow(sin((6.0 * PI) * h[0]), 6.0);
            const double r = f1 / g;
            f[0] = f1;
            f[1] = g * (1.0 - r * r);
            return;
        }
        case DM_EVAL_DTLZ1: {  // :489-492
            const int M = ev.obj;
            const double g = 100.0 * ((double)(n - (M - 1)) + S);
            double P = 1.0;
            for (int j = 0; j < M - 1; ++j) P = P * h[j];
            f[0] = 0.5 * P * (1.0 + g);
            int o = 1;
            for (int m = M - 2; m >= 0; --m) {
                double Pm = 1.0;
                for (int j = 0; j < m; ++j) Pm = Pm * h[j];
                f[o++] = 0.5 * Pm * (1.0 - h[m]) * (1.0 + g);
            }
            return;
        }
        default: {  // DTLZ2 / DTLZ3 / DTLZ4                 :516-520, :544-547, :574-576
            const int M = ev.obj;
            double g = S;
            if (ev.fn == DM_EVAL_DTLZ3) g = 100.0 * ((double)(n - (M - 1)) + S);
            double c[DM_MAX_OBJ], s[DM_MAX_OBJ];
            for (int j = 0; j < M - 1; ++j) {
                const double xj = (ev.fn == DM_EVAL_DTLZ4) ? pow(h[j], ev.alpha) : h[j];
                const double ang = 0.5 * xj * PI;
                c[j] = cos(ang);
                s[j] = sin(ang);
            }
            double P = 1.0;
            for (int j = 0; j < M - 1; ++j) P = P * c[j];
            f[0] = (1.0 + g) * P;
            int o = 1;
            for (int m = M - 2; m >= 0; --m) {
                double Pm = 1.0;
                for (int j = 0; j < m; ++j) Pm = Pm * c[j];
                f[o++] = (1.0 + g) * Pm * s[m];
            }
            return;
        }
    }
}

// ZDT1 / ZDT2 / ZDT4 only, the same arithmetic as mo_finalize (square roots
// and divisions): the short-row kernel's light variant, whose registers are
// not sized by the sine / power paths of ZDT3 / ZDT6 / DTLZ
__device__ __forceinline__ void mo_finalize_light(const dm_eval& ev, int n, double S, double h0,
                                                  double* f) {
    const double g = ev.fn == DM_EVAL_ZDT4 ? (double)(1 + 10 * (n - 1)) + S
                                           : 1.0 + 9.0 * S / (double)(n - 1);
    f[0] = h0;
    if (ev.fn == DM_EVAL_ZDT2) {
        const double r = h0 / g;
        f[1] = g * (1.0 - r * r);
    } else {
        f[1] = g * (1.0 - sqrt(h0 / g));
    }
}

// Per-row evaluation state carried across the chunks of one row.
struct EvalState {
    double s;      // running per-lane partial sum
    double carry;  // last gene of the previous chunk (Rosenbrock)
    double head[8];
};

__device__ __forceinline__ void eval_init(EvalState& st) {
    st.s = 0.0;
    st.carry = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) st.head[j] = 0.0;
}

// Feed one chunk of 4 genes per lane.  gbase = index of y[0] for this lane,
// cbase = index of the chunk's first gene.  All G lanes of the group must
// call this together (shuffles), `active` gates accumulation only.
template <int G, int EC>
__device__ __forceinline__ void eval_chunk(const dm_eval& ev, int dim, int gbase, int cbase,
                                           const double (&y)[4], bool active, EvalState& st) {
    const int lane = threadIdx.x & 63;
    const int gl0 = lane & ~(G - 1);  // first lane of this group
    const int sub = lane & (G - 1);
    if constexpr (ec_single(EC)) {
        const int fn = EC == EC_RAST ? (int)DM_EVAL_RASTRIGIN
                       : EC == EC_ROSEN ? (int)DM_EVAL_ROSENBROCK : ev.fn;
        if (fn == DM_EVAL_ROSENBROCK) {
            const double nb = __shfl(y[0], gl0 + ((sub + 1) & (G - 1)), 64);
            const double last = __shfl(y[3], gl0 + G - 1, 64);
            if (active) {
                double acc = 0.0;
                if (sub == 0 && cbase > 0 && cbase < dim) acc += rosen_term(st.carry, y[0]);
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    if (gbase + j + 1 < dim) acc += rosen_term(y[j], y[j + 1]);
                if (sub < G - 1 && gbase + 4 < dim) acc += rosen_term(y[3], nb);
                st.s += acc;
            }
            st.carry = last;
        } else if (EC == EC_RAST) {
            if (active) {
                if (gbase + 3 < dim) {  // full slot: four independent cosines (ILP)
                    const double t0 = rast_term(y[0]), t1 = rast_term(y[1]);
                    const double t2 = rast_term(y[2]), t3 = rast_term(y[3]);
                    st.s += (t0 + t1) + (t2 + t3);
                } else {
                    double acc = 0.0;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (gbase + j < dim) acc += rast_term(y[j]);
                    st.s += acc;
                }
            }
        } else {
            if (active) {
                // one (not four) inlined copy of the transcendental: keeps VGPRs low
                double acc = 0.0;
                const int nj = min(4, dim - gbase);
#pragma unroll 1
                for (int j = 0; j < nj; ++j) {
                    const double x = j == 0 ? y[0] : j == 1 ? y[1] : j == 2 ? y[2] : y[3];
                    acc += sum_term(fn, x);
                }
                st.s += acc;
            }
        }
    } else if constexpr (EC == EC_MO) {
        if (cbase == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                double v;
                switch (j & 3) {
                    case 0: v = y[0]; break;
                    case 1: v = y[1]; break;
                    case 2: v = y[2]; break;
                    default: v = y[3]; break;
                }
                st.head[j] = __shfl(v, gl0 + ((j >> 2) & (G - 1)), 64);
            }
        }
        if (active) {
            const int t0 = mo_tail_start(ev);
            double acc = 0.0;
            const int nj = min(4, dim - gbase);
#pragma unroll 1
            for (int j = 0; j < nj; ++j) {
                const double x = j == 0 ? y[0] : j == 1 ? y[1] : j == 2 ? y[2] : y[3];
                if (gbase + j >= t0) acc += mo_term(ev.fn, x);
            }
            st.s += acc;
        }
    }
}

// Reduce + finalize.  Returns nobj unweighted values in f (valid in every lane).
template <int G, int EC>
__device__ __forceinline__ void eval_finish(const dm_eval& ev, int dim, EvalState& st,
                                            double* f) {
    const double S = group_sum<G>(st.s);
    if constexpr (ec_single(EC)) {
        if (EC == EC_RAST || (EC == EC_SUM && ev.fn == DM_EVAL_RASTRIGIN))
            f[0] = (double)(10 * (int64_t)dim) + S;  // 10*len(individual) + sum(...)
        else
            f[0] = S;
    } else if constexpr (EC == EC_MO) {
        mo_finalize(ev, dim, S, st.head, f);
    }
}

}  // namespace dm
