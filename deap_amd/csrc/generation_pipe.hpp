// generation_pipe.hpp — the hot-path kernels of the fused eaSimple generation
// (native RNG, float genomes of 65..1024 genes).
//
// Two launches per generation:
//  1. pair_plan_kernel — one thread per offspring pair draws every per-pair
//     decision (tournament aspirants, crossover flag and cuts, mutation flags;
//     same Philox counters as the replay kernels) and writes a 32-byte
//     PairPlan: the two parent rows, the cut slice, the flags and the parents'
//     weighted fitness (what a clone inherits).  16 MB of plans per 2^20
//     children: 0.1% of the generation's traffic.
//  2. gen_pipe_kernel — one wave per pair, persistent grid, rolling pipeline:
//     the wave holds all NCH x 4 genes per lane of both parent rows in
//     registers; as soon as chunk c of pair p has been varied, stored and
//     evaluated, chunk c of the parents of pair p + W is loaded into the same
//     registers, so 2 x NCH x 2 KB per wave stay in flight while it computes.
//     Nothing inside the compute phase may issue a vector load or a call
//     (vmcnt is in-order on CDNA, a callee starts with a full wait): plans
//     come through SCALAR loads (lgkmcnt) two pairs ahead, the ziggurat tables
//     live in LDS, and the rare ziggurat rejection (~0.6% of draws) is inlined.
// Results are bit-identical to the replay kernel:
// tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel.
#pragma once
#include "generation.hpp"

namespace dm {

typedef __attribute__((address_space(4))) const uint32_t c4_u32;

struct PairPlan {
    int32_t s0, s1;    // parent rows
    uint32_t cuts;     // cxTwoPoint slice [cp1, cp2): cp1 | cp2 << 16
    uint32_t flags;    // PF_*
    double f0, f1;     // parents' wvalues[0] (inherited by an unchanged clone)
};
static_assert(sizeof(PairPlan) == 32, "PairPlan layout");
enum : uint32_t { PF_CX = 1, PF_MUT0 = 2, PF_MUT1 = 4, PF_HAS1 = 8, PF_INV0 = 16, PF_INV1 = 32 };

// Scalar (SMEM) load of a plan: wave-uniform index, tracked by lgkmcnt.
__device__ __forceinline__ PairPlan load_plan(const PairPlan* plans, int64_t p) {
    const c4_u32* q = (const c4_u32*)(const void*)(plans + p);
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = q[i];
    PairPlan r;
    r.s0 = (int32_t)v[0];
    r.s1 = (int32_t)v[1];
    r.cuts = v[2];
    r.flags = v[3];
    r.f0 = __hiloint2double((int)v[5], (int)v[4]);
    r.f1 = __hiloint2double((int)v[7], (int)v[6]);
    return r;
}

// Ziggurat draw with the tables in LDS: the rectangle test accepts ~99.4% of
// draws; otherwise the full sampler (common.hpp zig_normal) recomputes the
// same draw from attempt 0 — identical value either way.
// Inlined on purpose: a call would start with a full s_waitcnt and drain the
// row prefetches (measured 4.20 vs 3.84 ms per C3 generation).
__device__ __forceinline__ double zig_normal_slow(const double* zig, Rng rng, uint32_t c, uint32_t gi) {
    return zig_normal(zig, rng, ST_GAUSS, c, gi);
}
__device__ __forceinline__ double zig_normal_lds(const double* szig, const double* gzig,
                                                 const Rng& rng, uint32_t c, uint32_t gi) {
    const u32x4 w = rng(ST_GAUSS, c, gi);
    const int layer = (int)(w.x & (ZIG_N - 1));
    const bool neg = (w.x >> 8) & 1;
    const double u = u01_53(w.y & 0xFFFFF800u, w.z);
    const double x = u * szig[layer];
    if (x < szig[layer + 1]) return neg ? -x : x;
    return zig_normal_slow(gzig, rng, c, gi);
}

struct PipeArgs {
    const char* pgenes;
    char* cgenes;
    double* cwv;
    uint8_t* cvalid;
    const PairPlan* plans;
    const double* pwv;  // nobj > 1 clones only
    const double* mu_vec;
    const double* sigma_vec;
    const double* zig;
    int64_t* nevals;
    int64_t nc, pstride, cstride;
    int32_t dim, nobj;
    Rng rng;
    uint64_t thr_ind;
    double alpha, mu, sigma, w0;
    dm_eval ev;
};

#ifndef DM_PIPE_MINWAVES
#define DM_PIPE_MINWAVES 2
#endif

#ifndef DM_PIPE_DEPTH
#define DM_PIPE_DEPTH 2
#endif

template <typename T, int NCH, int CX, int MUT, int EC>
__global__ __launch_bounds__(256, DM_PIPE_MINWAVES) void gen_pipe_kernel(PipeArgs a) {
    constexpr int D = NCH < DM_PIPE_DEPTH ? NCH : DM_PIPE_DEPTH;
    static_assert(NCH % D == 0, "ring depth must divide the chunk count");
    __shared__ double szig[ZIG_N + 1];
    if (MUT == DM_MUT_GAUSSIAN) {
        for (int i = threadIdx.x; i <= ZIG_N; i += blockDim.x) szig[i] = a.zig[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (p >= npairs) return;
    int64_t evals = 0;
    const double gamma_scale = 1.0 + 2.0 * a.alpha;

    PairPlan pl = load_plan(a.plans, p);
    PairPlan nx = load_plan(a.plans, p + nw < npairs ? p + nw : p);
    // ring of D chunk slots over the chunk sequence (p,0..NCH-1), (p+W,0..), ...
    double y0[D][4], y1[D][4];
#pragma unroll
    for (int ch = 0; ch < D; ++ch) {
        const int g = ch * 256 + 4 * lane;
        if (g < a.dim) {
            Vec4<T>::load(a.pgenes + (int64_t)pl.s0 * a.pstride, g, y0[ch]);
            Vec4<T>::load(a.pgenes + (int64_t)pl.s1 * a.pstride, g, y1[ch]);
        }
    }
    for (; p < npairs; p += nw) {
        const bool more = p + nw < npairs;
        const int64_t p2 = p + 2 * nw;
        const PairPlan nn = load_plan(a.plans, p2 < npairs ? p2 : p);  // two ahead
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        const uint32_t fl = pl.flags;
        const bool cx = fl & PF_CX, mut0 = fl & PF_MUT0, mut1 = fl & PF_MUT1;
        const bool has1 = fl & PF_HAS1, inv0 = fl & PF_INV0, inv1 = fl & PF_INV1;
        const int cp1 = (int)(pl.cuts & 0xFFFFu), cp2 = (int)(pl.cuts >> 16);
        char* w0 = a.cgenes + c0 * a.cstride;
        char* w1 = a.cgenes + c1 * a.cstride;
        const char* r0 = a.pgenes + (int64_t)pl.s0 * a.pstride;
        const char* r1 = a.pgenes + (int64_t)pl.s1 * a.pstride;
        const char* n0 = a.pgenes + (int64_t)nx.s0 * a.pstride;
        const char* n1 = a.pgenes + (int64_t)nx.s1 * a.pstride;
        EvalState e0, e1;
        eval_init(e0);
        eval_init(e1);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int cbase = ch * 256;
            const int g = cbase + 4 * lane;
            const bool in = g < a.dim;
            double x0[4], x1[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x0[k] = in ? y0[ch % D][k] : 0.0;
                x1[k] = in ? y1[ch % D][k] : 0.0;
            }
            // ring: the chunk D ahead into the freed slot (this pair's rows or
            // the next pair's)
            {
                const int ca = ch + D;
                const int ga = (ca < NCH ? ca : ca - NCH) * 256 + 4 * lane;
                if (ca < NCH) {
                    if (ga < a.dim) {
                        Vec4<T>::load(r0, ga, y0[ch % D]);
                        Vec4<T>::load(r1, ga, y1[ch % D]);
                    }
                } else if (more && ga < a.dim) {
                    Vec4<T>::load(n0, ga, y0[ch % D]);
                    Vec4<T>::load(n1, ga, y1[ch % D]);
                }
            }
            if (CX == DM_CX_BLEND && cx && in) {
                const u32x4 u = a.rng(ST_BLEND, (uint32_t)p, (uint32_t)(g >> 2));
                const uint32_t us[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (g + k < a.dim) {
                        // gamma = (1.+2.*alpha)*random()-alpha; blend   (crossover.py:255-258)
                        const double gm = gamma_scale * u01_32(us[k]) - a.alpha;
                        const double v1 = x0[k], v2 = x1[k];
                        x0[k] = (1.0 - gm) * v1 + gm * v2;
                        x1[k] = gm * v1 + (1.0 - gm) * v2;
                    }
                }
            } else if (CX == DM_CX_TWOPOINT && cx && in) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (g + k >= cp1 && g + k < cp2) {  // crossover.py:71-72 slice swap
                        const double tt = x0[k];
                        x0[k] = x1[k];
                        x1[k] = tt;
                    }
                }
            }
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x0[k] = (double)(float)x0[k];
                    x1[k] = (double)(float)x1[k];
                }
            }
            if (MUT == DM_MUT_GAUSSIAN && in && (mut0 || mut1)) {
                // per-gene Bernoulli(indpb) + gauss(mu, sigma)   (mutation.py:44-46)
                uint32_t bits = 0;
                const int lim = a.dim - g < 4 ? a.dim - g : 4;
                const uint32_t keep = (1u << lim) - 1u;
                if (mut0) {
                    const u32x4 w = a.rng(ST_MASK, (uint32_t)c0, (uint32_t)(g >> 2));
                    bits |= (((uint64_t)w.x < a.thr_ind ? 1u : 0u) |
                             ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                             ((uint64_t)w.z < a.thr_ind ? 4u : 0u) |
                             ((uint64_t)w.w < a.thr_ind ? 8u : 0u)) & keep;
                }
                if (mut1) {
                    const u32x4 w = a.rng(ST_MASK, (uint32_t)c1, (uint32_t)(g >> 2));
                    bits |= ((((uint64_t)w.x < a.thr_ind ? 1u : 0u) |
                              ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                              ((uint64_t)w.z < a.thr_ind ? 4u : 0u) |
                              ((uint64_t)w.w < a.thr_ind ? 8u : 0u)) & keep) << 4;
                }
#pragma unroll 1
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    bits &= bits - 1;
                    const int j = b & 3, gi = g + j;
                    const double nrm =
                        zig_normal_lds(szig, a.zig, a.rng, (uint32_t)(c0 + (b >> 2)), (uint32_t)gi);
                    const double m = a.mu_vec ? a.mu_vec[gi] : a.mu;
                    const double s = a.sigma_vec ? a.sigma_vec[gi] : a.sigma;
                    const double gv = m + nrm * s;  // random.gauss(mu, sigma)
                    if (b < 4) {
                        x0[0] = j == 0 ? x0[0] + gv : x0[0];
                        x0[1] = j == 1 ? x0[1] + gv : x0[1];
                        x0[2] = j == 2 ? x0[2] + gv : x0[2];
                        x0[3] = j == 3 ? x0[3] + gv : x0[3];
                    } else {
                        x1[0] = j == 0 ? x1[0] + gv : x1[0];
                        x1[1] = j == 1 ? x1[1] + gv : x1[1];
                        x1[2] = j == 2 ? x1[2] + gv : x1[2];
                        x1[3] = j == 3 ? x1[3] + gv : x1[3];
                    }
                }
            }
            if (in) {
                Vec4<T>::store_nt(w0, g, x0);
                if (has1) Vec4<T>::store_nt(w1, g, x1);
            }
            if constexpr (sizeof(T) == 4) {
                // evaluate the stored (fp32-rounded) genes, as DEAP reads array('f')
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x0[k] = (double)(float)x0[k];
                    x1[k] = (double)(float)x1[k];
                }
            }
            if (EC != EC_NONE) {
                eval_chunk<64, EC>(a.ev, a.dim, g, cbase, x0, inv0, e0);
                eval_chunk<64, EC>(a.ev, a.dim, g, cbase, x1, inv1, e1);
            }
        }
        double f0[DM_MAX_OBJ], f1[DM_MAX_OBJ];
        if (EC != EC_NONE) {
            eval_finish<64, EC>(a.ev, a.dim, e0, f0);
            eval_finish<64, EC>(a.ev, a.dim, e1, f1);
        }
        if (lane == 0) {
            const bool de = EC != EC_NONE;
            if constexpr (ec_single(EC)) {
                a.cwv[c0] = inv0 ? f0[0] * a.w0 : pl.f0;
                if (has1) a.cwv[c1] = inv1 ? f1[0] * a.w0 : pl.f1;
            } else if (a.nobj == 1) {  // no evaluation requested
                a.cwv[c0] = pl.f0;
                if (has1) a.cwv[c1] = pl.f1;
            } else {
                const int m = a.nobj;
                for (int o = 0; o < m; ++o) {
                    a.cwv[c0 * m + o] = a.pwv[(int64_t)pl.s0 * m + o];
                    if (has1) a.cwv[c1 * m + o] = a.pwv[(int64_t)pl.s1 * m + o];
                }
            }
            a.cvalid[c0] = de ? 1 : (inv0 ? 0 : 1);
            if (has1) a.cvalid[c1] = de ? 1 : (inv1 ? 0 : 1);
            evals += (int64_t)inv0 + (int64_t)inv1;
        }
        pl = nx;
        nx = nn;
    }
    if (a.nevals && EC != EC_NONE) {
        int64_t tot = evals;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)a.nevals, (unsigned long long)tot);
    }
}

template <typename T, int NCH, int CX, int MUT>
void launch_pipe_e(const PipeArgs& a, int ec, dim3 grid, hipStream_t s) {
    if (ec == EC_RAST)
        gen_pipe_kernel<T, NCH, CX, MUT, EC_RAST><<<grid, 256, 0, s>>>(a);
    else if (ec == EC_ROSEN)
        gen_pipe_kernel<T, NCH, CX, MUT, EC_ROSEN><<<grid, 256, 0, s>>>(a);
    else if (ec_single(ec))
        gen_pipe_kernel<T, NCH, CX, MUT, EC_SUM><<<grid, 256, 0, s>>>(a);
    else
        gen_pipe_kernel<T, NCH, CX, MUT, EC_NONE><<<grid, 256, 0, s>>>(a);
}
template <typename T, int NCH>
void launch_pipe_ops(const PipeArgs& a, int ec, int cx, int mut, dim3 grid, hipStream_t s) {
    const bool mg = mut == DM_MUT_GAUSSIAN;
    switch (cx) {
        case DM_CX_BLEND:
            mg ? launch_pipe_e<T, NCH, DM_CX_BLEND, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_pipe_e<T, NCH, DM_CX_BLEND, DM_MUT_NONE>(a, ec, grid, s);
            break;
        case DM_CX_TWOPOINT:
            mg ? launch_pipe_e<T, NCH, DM_CX_TWOPOINT, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_pipe_e<T, NCH, DM_CX_TWOPOINT, DM_MUT_NONE>(a, ec, grid, s);
            break;
        default:
            mg ? launch_pipe_e<T, NCH, DM_CX_NONE, DM_MUT_GAUSSIAN>(a, ec, grid, s)
               : launch_pipe_e<T, NCH, DM_CX_NONE, DM_MUT_NONE>(a, ec, grid, s);
    }
}

// Decisions of every pair (thread per pair), generation_pipe_f64.hip.
void launch_pair_plans(const GenArgs& a, PairPlan* plans, hipStream_t s);
void launch_gen_pipe_f64(const PipeArgs& a, int ec, int cx, int mut, int nch, dim3 grid,
                         hipStream_t s);
void launch_gen_pipe_f32(const PipeArgs& a, int ec, int cx, int mut, int nch, dim3 grid,
                         hipStream_t s);

}  // namespace dm
