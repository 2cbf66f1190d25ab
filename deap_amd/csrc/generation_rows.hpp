// generation_rows.hpp — the native hot path for SHORT float rows (at most 64
// genes: Rastrigin-30D, ZDT / DTLZ genomes), any objective count.
//
// Two launches per generation, as for long rows (generation_pipe.hpp):
//  1. pair_plan_kernel — every per-pair decision (tournaments of one or more
//     objectives, crossover flag and cuts, mutation flags) into a 32-B plan;
//  2. gen_rows_kernel — a lane group of G lanes per offspring pair (4 genes
//     per lane: G = 4 / 8 / 16 for rows of <= 16 / 32 / 64 genes), 64 / G pairs
//     per wave on a persistent grid.  A group keeps the rows of PD pairs (the
//     one it varies and the next PD - 1) and the plan of the pair after them in
//     flight: the only dependent chain per pair is plan -> row loads, issued
//     PD pairs ahead.
// The general kernel (generation.hpp gen_float_kernel) draws the tournaments
// inside the lane group -- t dependent random fitness loads per child -- and
// spilled 320-1,000 B per lane to scratch: 0.054 of the HBM roofline on
// Rastrigin-30D (profiles/r06a).  Decisions come from the same Philox
// counters (gene4_words, zig_normal), so the children are bit-identical to the
// replay kernel's dump mode, which the oracle replays.
#pragma once
#include "generation_pipe.hpp"

namespace dm {

template <typename T>
struct RowRaw;
template <>
struct RowRaw<double> {
    dm_d2 a, b;  // genes g .. g + 3 of one row
    __device__ __forceinline__ void load(const char* row, int g) {
        const dm_d2* p = reinterpret_cast<const dm_d2*>(row + (size_t)g * 8);
        a = p[0];
        b = p[1];
    }
    __device__ __forceinline__ void unpack(double (&x)[4]) const {
        x[0] = a.x;
        x[1] = a.y;
        x[2] = b.x;
        x[3] = b.y;
    }
};
template <>
struct RowRaw<float> {
    dm_f4 v;
    __device__ __forceinline__ void load(const char* row, int g) {
        v = *reinterpret_cast<const dm_f4*>(row + (size_t)g * 4);
    }
    __device__ __forceinline__ void unpack(double (&x)[4]) const {
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    }
};

// A plan as 2 x 16 B (every lane of the group loads it; one request per group)
__device__ __forceinline__ PairPlan load_plan_vec(const PairPlan* plans, int64_t p) {
    const int4* q = reinterpret_cast<const int4*>(plans + p);
    const int4 u = q[0], v = q[1];
    PairPlan r;
    r.s0 = u.x;
    r.s1 = u.y;
    r.cuts = (uint32_t)u.z;
    r.flags = (uint32_t)u.w;
    r.f0 = __hiloint2double(v.y, v.x);
    r.f1 = __hiloint2double(v.w, v.z);
    return r;
}

// Fitness of both children of a pair, 4 genes per lane (genes g .. g + 3,
// lanes of one group): per-gene terms in the reference's operation order
// (evals.hpp), one group sum per child; lane sub = 0 returns child 0's
// unweighted values in f, lane sub = 1 child 1's.  Both children run through
// ONE copy of each term and of the final formula (an 8-step loop over the two
// children's genes, the finalisation with per-lane data), so the objective's
// transcendental code is inlined once.
// ZDT1 / ZDT2 / ZDT4 on short rows: EC_MO's terms with the light final
// formula (evals.hpp mo_finalize_light), two objectives
constexpr int EC_MO_LIGHT = 7;
__host__ __device__ constexpr bool ec_mo(int ec) { return ec == EC_MO || ec == EC_MO_LIGHT; }
__host__ __device__ inline bool mo_light(int fn) {
    return fn == DM_EVAL_ZDT1 || fn == DM_EVAL_ZDT2 || fn == DM_EVAL_ZDT4;
}

template <int G, int EC>
__device__ __forceinline__ void rows_eval(const dm_eval& ev, int dim, int g, int sub,
                                          const double (&y0)[4], const double (&y1)[4], bool inv0,
                                          bool inv1, double* f) {
    const int lane = threadIdx.x & 63;
    const int gl0 = lane & ~(G - 1);
    double acc0 = 0.0, acc1 = 0.0;
    if (ec_single(EC) && ev.fn == DM_EVAL_ROSENBROCK) {
        // 100*(x*x - y)**2 + (1. - x)**2 over consecutive genes     (:117-118)
        const double nb0 = __shfl(y0[0], gl0 + ((sub + 1) & (G - 1)), 64);
        const double nb1 = __shfl(y1[0], gl0 + ((sub + 1) & (G - 1)), 64);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (g + j + 1 < dim) {
                acc0 += rosen_term(y0[j], y0[j + 1]);
                acc1 += rosen_term(y1[j], y1[j + 1]);
            }
        if (sub < G - 1 && g + 4 < dim) {
            acc0 += rosen_term(y0[3], nb0);
            acc1 += rosen_term(y1[3], nb1);
        }
    } else {
        const int t0 = ec_mo(EC) ? mo_tail_start(ev) : 0;
#pragma unroll 1
        for (int k = 0; k < 8; ++k) {
            const int j = k & 3;
            const bool second = k >= 4;
            const double xa = j == 0 ? y0[0] : j == 1 ? y0[1] : j == 2 ? y0[2] : y0[3];
            const double xb = j == 0 ? y1[0] : j == 1 ? y1[1] : j == 2 ? y1[2] : y1[3];
            const double x = second ? xb : xa;
            if (g + j < dim && g + j >= t0 && (second ? inv1 : inv0)) {
                const double t = ec_mo(EC) ? mo_term(ev.fn, x) : sum_term(ev.fn, x);
                if (second)
                    acc1 += t;
                else
                    acc0 += t;
            }
        }
    }
    const double S0 = group_sum<G>(acc0), S1 = group_sum<G>(acc1);
    const bool second = sub == 1;
    const double S = second ? S1 : S0;
    if constexpr (ec_single(EC)) {
        f[0] = ev.fn == DM_EVAL_RASTRIGIN ? (double)(10 * (int64_t)dim) + S : S;  // 10*len + sum
    } else if constexpr (EC == EC_MO_LIGHT) {
        const double h0 = __shfl(y0[0], gl0, 64), h1 = __shfl(y1[0], gl0, 64);  // gene 0
        mo_finalize_light(ev, dim, S, second ? h1 : h0, f);
    } else if constexpr (EC == EC_MO) {
        double h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // head genes x[0..7] of this lane's child
            const double v0 = (j & 3) == 0 ? y0[0] : (j & 3) == 1 ? y0[1] : (j & 3) == 2 ? y0[2] : y0[3];
            const double v1 = (j & 3) == 0 ? y1[0] : (j & 3) == 1 ? y1[1] : (j & 3) == 2 ? y1[2] : y1[3];
            const double h0 = __shfl(v0, gl0 + ((j >> 2) & (G - 1)), 64);
            const double h1 = __shfl(v1, gl0 + ((j >> 2) & (G - 1)), 64);
            h[j] = second ? h1 : h0;
        }
        mo_finalize(ev, dim, S, h, f);
    }
}

// PD: pairs whose rows are in flight per lane group (the current one included)
#ifndef DM_ROWS_PD
#define DM_ROWS_PD 3
#endif
template <typename T, int G, int CX, int MUT, int EC, int PD = DM_ROWS_PD>
__global__ __launch_bounds__(256) void gen_rows_kernel(GenArgs a, const PairPlan* __restrict__ plans) {
    __shared__ double szig[MUT == DM_MUT_GAUSSIAN ? ZIG_N + 1 : 1];
    if (MUT == DM_MUT_GAUSSIAN) {
        for (int i = threadIdx.x; i <= ZIG_N; i += blockDim.x) szig[i] = a.zig[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t ng = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    if (p >= npairs) return;  // group-uniform
    const int dim = a.dim;
    const int g = 4 * sub;  // this lane's first gene
    const bool in = g < dim;
    const double gamma_scale = 1.0 + 2.0 * a.alpha;

    // ring of PD pairs whose rows are in flight (slot k: pair p + k ng), and
    // the plan of the pair after them
    PairPlan plq[PD];
    RowRaw<T> rq0[PD], rq1[PD];
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        const int64_t pk = p + k * ng;
        plq[k] = load_plan_vec(plans, pk < npairs ? pk : p);
    }
#pragma unroll
    for (int k = 0; k < PD; ++k)
        if (in && p + k * ng < npairs) {
            rq0[k].load(a.pgenes + (int64_t)plq[k].s0 * a.pstride, g);
            rq1[k].load(a.pgenes + (int64_t)plq[k].s1 * a.pstride, g);
        }
    PairPlan nx = load_plan_vec(plans, p + PD * ng < npairs ? p + PD * ng : p);
    // pair p from ring slot sl (compile-time after unrolling)
    auto pair_step = [&](const int sl) {
        const PairPlan pl = plq[sl];
        double y0[4] = {0, 0, 0, 0}, y1[4] = {0, 0, 0, 0};
        if (in) {
            rq0[sl].unpack(y0);
            rq1[sl].unpack(y1);
        }
        // refill the slot: the rows of pair p + PD ng, the plan after it
        {
            const int64_t pn = p + PD * ng, pn2 = pn + ng;
            if (in && pn < npairs) {
                rq0[sl].load(a.pgenes + (int64_t)nx.s0 * a.pstride, g);
                rq1[sl].load(a.pgenes + (int64_t)nx.s1 * a.pstride, g);
            }
            plq[sl] = nx;
            nx = load_plan_vec(plans, pn2 < npairs ? pn2 : p);
        }
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        const uint32_t fl = pl.flags;
        const bool cx = fl & PF_CX, mut0 = fl & PF_MUT0, mut1 = fl & PF_MUT1;
        const bool has1 = fl & PF_HAS1, inv0 = fl & PF_INV0, inv1 = fl & PF_INV1;
        if (in && CX == DM_CX_BLEND && cx) {
            // gamma = (1. + 2.*alpha)*random() - alpha ; blend   (crossover.py:255-258)
            const u32x4 w = gene4_words<T>(a.rng, ST_BLEND, (uint32_t)p, g);
            const uint32_t us[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (g + j < dim) {
                    const double gm = gamma_scale * u01_32(us[j]) - a.alpha;
                    const double x1 = y0[j], x2 = y1[j];
                    y0[j] = (1.0 - gm) * x1 + gm * x2;
                    y1[j] = gm * x1 + (1.0 - gm) * x2;
                }
            }
        } else if (in && CX == DM_CX_TWOPOINT && cx) {
            const int cp1 = (int)(pl.cuts & 0xFFFFu), cp2 = (int)(pl.cuts >> 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (g + j >= cp1 && g + j < cp2) {  // crossover.py:71-72 slice swap
                    const double t = y0[j];
                    y0[j] = y1[j];
                    y1[j] = t;
                }
            }
        }
        if constexpr (sizeof(T) == 4) {
            // array('f') stores the crossover result (rounded) before mutation reads it
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                y0[j] = (double)(float)y0[j];
                y1[j] = (double)(float)y1[j];
            }
        }
        if (MUT == DM_MUT_GAUSSIAN && in && (mut0 || mut1)) {
            // per-gene Bernoulli(indpb) + gauss(mu, sigma)   (mutation.py:44-46)
            uint32_t bits = 0;
            if (mut0) {
                const u32x4 w = gene4_words<T>(a.rng, ST_MASK, (uint32_t)c0, g);
                bits |= ((uint64_t)w.x < a.thr_ind ? 1u : 0u) | ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                        ((uint64_t)w.z < a.thr_ind ? 4u : 0u) | ((uint64_t)w.w < a.thr_ind ? 8u : 0u);
            }
            if (mut1) {
                const u32x4 w = gene4_words<T>(a.rng, ST_MASK, (uint32_t)c1, g);
                bits |= (((uint64_t)w.x < a.thr_ind ? 1u : 0u) | ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                         ((uint64_t)w.z < a.thr_ind ? 4u : 0u) | ((uint64_t)w.w < a.thr_ind ? 8u : 0u))
                        << 4;
            }
            const int valid = dim - g;
            if (valid < 4) {
                const uint32_t keep = (1u << valid) - 1u;
                bits &= keep | (keep << 4);
            }
#pragma unroll 1
            while (bits) {
                const int b = __builtin_ctz(bits);
                bits &= bits - 1;
                const int j = b & 3;
                const int gi = g + j;
                const double nrm =
                    zig_normal_lds(szig, a.zig, a.rng, (uint32_t)(c0 + (b >> 2)), (uint32_t)gi);
                const double m = a.mu_vec ? a.mu_vec[gi] : a.mu;
                const double s = a.sigma_vec ? a.sigma_vec[gi] : a.sigma;
                const double gv = m + nrm * s;  // random.gauss(mu, sigma)
                if (b < 4) {
                    y0[0] = j == 0 ? y0[0] + gv : y0[0];
                    y0[1] = j == 1 ? y0[1] + gv : y0[1];
                    y0[2] = j == 2 ? y0[2] + gv : y0[2];
                    y0[3] = j == 3 ? y0[3] + gv : y0[3];
                } else {
                    y1[0] = j == 0 ? y1[0] + gv : y1[0];
                    y1[1] = j == 1 ? y1[1] + gv : y1[1];
                    y1[2] = j == 2 ? y1[2] + gv : y1[2];
                    y1[3] = j == 3 ? y1[3] + gv : y1[3];
                }
            }
        }
        if (in) {
            Vec4<T>::store_nt(a.cgenes + c0 * a.cstride, g, y0);
            if (has1) Vec4<T>::store_nt(a.cgenes + c1 * a.cstride, g, y1);
        }
        if constexpr (sizeof(T) == 4) {
            // evaluate the stored (fp32-rounded) genes, as DEAP reads array('f')
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                y0[j] = (double)(float)y0[j];
                y1[j] = (double)(float)y1[j];
            }
        }
        // fitness: lane sub = 0 finalises child 0, sub = 1 child 1 (one inlined
        // copy of the objective's code for both children)
        double f[DM_MAX_OBJ];
        if constexpr (EC != EC_NONE) rows_eval<G, EC>(a.ev, dim, g, sub, y0, y1, inv0, inv1, f);
        if (sub < 2) {
            const int m = a.nobj;
            const bool second = sub == 1;
            const int64_t c = second ? c1 : c0;
            const bool inv = second ? inv1 : inv0;
            const int64_t s = second ? pl.s1 : pl.s0;
            if (!second || has1) {
                if constexpr (ec_single(EC)) {
                    a.cwv[c] = inv ? f[0] * a.w0 : (second ? pl.f1 : pl.f0);
                } else if constexpr (EC == EC_MO_LIGHT) {
#pragma unroll
                    for (int o = 0; o < 2; ++o)
                        a.cwv[c * 2 + o] = inv ? f[o] * a.ev.weights[o] : a.pwv[s * 2 + o];
                } else if constexpr (EC == EC_MO) {
                    for (int o = 0; o < m; ++o)
                        a.cwv[c * m + o] = inv ? f[o] * a.ev.weights[o] : a.pwv[s * m + o];
                } else {  // no evaluation requested: every child keeps its parent's fitness
                    for (int o = 0; o < m; ++o) a.cwv[c * m + o] = a.pwv[s * m + o];
                }
                a.cvalid[c] = EC != EC_NONE ? 1 : (inv ? 0 : 1);
            }
        }
    };
    for (;;) {
#pragma unroll
        for (int sl = 0; sl < PD; ++sl) {
            if (p >= npairs) return;  // group-uniform
            pair_step(sl);
            p += ng;
        }
    }
}

template <typename T, int G, int CX, int MUT>
void launch_rows_e(const GenArgs& a, const PairPlan* plans, int ec, dim3 grid, hipStream_t s) {
    if (ec_single(ec))
        gen_rows_kernel<T, G, CX, MUT, EC_SUM><<<grid, 256, 0, s>>>(a, plans);
    else if (ec == EC_MO && mo_light(a.ev.fn) && a.nobj == 2)
        gen_rows_kernel<T, G, CX, MUT, EC_MO_LIGHT><<<grid, 256, 0, s>>>(a, plans);
    else if (ec == EC_MO)
        gen_rows_kernel<T, G, CX, MUT, EC_MO><<<grid, 256, 0, s>>>(a, plans);
    else
        gen_rows_kernel<T, G, CX, MUT, EC_NONE><<<grid, 256, 0, s>>>(a, plans);
}
template <typename T, int G>
void launch_rows_ops(const GenArgs& a, const PairPlan* plans, int ec, dim3 grid, hipStream_t s) {
    const bool mg = a.mut == DM_MUT_GAUSSIAN;
    switch (a.cx) {
        case DM_CX_BLEND:
            mg ? launch_rows_e<T, G, DM_CX_BLEND, DM_MUT_GAUSSIAN>(a, plans, ec, grid, s)
               : launch_rows_e<T, G, DM_CX_BLEND, DM_MUT_NONE>(a, plans, ec, grid, s);
            break;
        case DM_CX_TWOPOINT:
            mg ? launch_rows_e<T, G, DM_CX_TWOPOINT, DM_MUT_GAUSSIAN>(a, plans, ec, grid, s)
               : launch_rows_e<T, G, DM_CX_TWOPOINT, DM_MUT_NONE>(a, plans, ec, grid, s);
            break;
        default:
            mg ? launch_rows_e<T, G, DM_CX_NONE, DM_MUT_GAUSSIAN>(a, plans, ec, grid, s)
               : launch_rows_e<T, G, DM_CX_NONE, DM_MUT_NONE>(a, plans, ec, grid, s);
    }
}
template <typename T>
void launch_rows_t(const GenArgs& a, const PairPlan* plans, int ec, int num_cus, hipStream_t s) {
    const int G = a.dim <= 16 ? 4 : a.dim <= 32 ? 8 : 16;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t per_block = 256 / G;
    const int64_t blocks =
        std::min<int64_t>((npairs + per_block - 1) / per_block, (int64_t)num_cus * 8);
    const dim3 grid((unsigned)std::max<int64_t>(blocks, 1));
    if (G == 4)
        launch_rows_ops<T, 4>(a, plans, ec, grid, s);
    else if (G == 8)
        launch_rows_ops<T, 8>(a, plans, ec, grid, s);
    else
        launch_rows_ops<T, 16>(a, plans, ec, grid, s);
}

}  // namespace dm
