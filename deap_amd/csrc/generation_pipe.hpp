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
//     a row is streamed in chunks of 256 genes; the wave keeps D chunks of
//     both parent rows in flight in registers, and as soon as chunk c of pair
//     p has been varied, stored and evaluated, chunk c + D (or a chunk of the
//     parents of pair p + W) is loaded into the freed registers.
//     Nothing inside the compute phase may issue a vector load or a call
//     (vmcnt is in-order on CDNA, a callee starts with a full wait): plans
//     come through SCALAR loads (lgkmcnt) two pairs ahead, the ziggurat and
//     cosine tables live in LDS, and the rare ziggurat rejection (~0.6% of
//     draws) is inlined.
//
// Lane layout of a chunk (ChunkLayout<T>): every load / store instruction of
// the wave covers ONE contiguous KiB (16 B per lane).  fp64: two pieces per
// row, lane L holds genes {256c + 2L, +1} and {256c + 128 + 2L, +1}; fp32:
// one piece, lane L holds genes 256c + 4L .. +3.  (The earlier 32-B-per-lane
// layout made every instruction span 2 KiB with holes and capped the row
// copy at 4.4 TB/s against 5.6 TB/s for whole-KiB instructions — measured
// with tools_gpu/bwtest2.hip.)  The per-gene Philox slots follow the same
// layout (gene4_words in generation.hpp), so one Philox call feeds a lane's four
// genes in every kernel.
//
// Genomes are bit-identical to the replay kernel's:
// tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel.
#pragma once
#include "generation.hpp"

namespace dm {

typedef __attribute__((address_space(4))) const uint32_t c4_u32;

#ifndef DM_RAST_ILP
#define DM_RAST_ILP 2  // Rastrigin terms evaluated side by side (VGPR pressure)
#endif

struct PairPlan {
    int32_t s0, s1;    // parent rows
    uint32_t cuts;     // cxTwoPoint slice [cp1, cp2): cp1 | cp2 << 16
    uint32_t flags;    // PF_*; parent-ordered plans: the pair index << PF_PAIR_SHIFT
    double f0, f1;     // parents' wvalues[0] (inherited by an unchanged clone)
};
static_assert(sizeof(PairPlan) == 32, "PairPlan layout");
enum : uint32_t { PF_CX = 1, PF_MUT0 = 2, PF_MUT1 = 4, PF_HAS1 = 8, PF_INV0 = 16, PF_INV1 = 32 };
constexpr int PF_PAIR_SHIFT = 8;  // parent-ordered plans: the pair index above the flags

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

// The ziggurat's wedge / tail sampler (~0.6% of draws).  Out of line by
// default: inlined, its exp / log1p temporaries pushed the hot kernel past
// 128 VGPRs; the call's vmcnt(0) drain is paid only on those rare draws.
#ifndef DM_ZIG_SLOW_NOINLINE
#define DM_ZIG_SLOW_NOINLINE 1
#endif
#if DM_ZIG_SLOW_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
double zig_normal_slow(const double* zig, Rng rng, uint32_t c, uint32_t gi) {
    return zig_normal(zig, rng, ST_GAUSS, c, gi);
}

// Ziggurat draw with the tables in LDS: the rectangle test accepts ~99.4% of
// draws; otherwise the full sampler (common.hpp zig_normal) recomputes the
// same draw from attempt 0 — identical value either way.
// The fast path is inlined: a call would start with a full s_waitcnt and
// drain the row prefetches on every draw (measured 4.20 vs 3.84 ms per C3
// generation).
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

// cos(2*pi*x) for the Rastrigin term `gene*gene - 10*cos(2*pi*gene)`
// (deap/benchmarks/__init__.py:239-240).  Reduction in turns: k = rint(64x),
// f = x - k/64 (exact, |f| <= 1/128), and
//   cos(2pi(k/64 + f)) = C_k cos(2pi f) - S_k sin(2pi f)
// with (C_k, S_k) = (cos, sin)(2pi k/64) from a 1-KiB LDS table and Taylor
// polynomials in f (truncation < 1e-15).  Against glibc's cos of the rounded
// product 2*pi*gene the difference is the reference's own rounding of that
// product (<= 4e-15 absolute per term), far inside the 1e-12 relative
// fitness tolerance.  ~17 fp64 operations vs ~28 for a pi/2 reduction that
// evaluates both the sine and cosine kernels.
__device__ __forceinline__ double cos2pi_lds(const double2* tab, double x) {
    const double k = rint(x * 64.0);
    const double f = fma(-k, 0.015625, x);
    const double2 cs = tab[(int)k & 63];
    const double z = f * f;
    const double c = fma(z, fma(z, fma(z, -85.45681720669373, 64.9393940226683),
                                -19.739208802178716), 1.0);
    const double s = f * fma(z, fma(z, fma(z, -76.70585975306139, 81.60524927607506),
                                    -41.34170224039976), 6.283185307179586);
    return fma(cs.x, c, -(cs.y * s));
}

// Lane layout of one 256-gene chunk (see the header comment).
template <typename T>
struct ChunkLayout;
template <>
struct ChunkLayout<double> {
    // a chunk of one row as loaded: lane L's two 16-B pieces
    struct Raw {
        dm_d2 a, b;
    };
    __device__ __forceinline__ static int gene(int c, int lane, int k) {
        return (c << 8) + ((k >> 1) << 7) + 2 * lane + (k & 1);
    }
    __device__ __forceinline__ static void load(const char* row, int c, int lane, int dim, Raw& r) {
        const int g0 = gene(c, lane, 0), g2 = gene(c, lane, 2);
        if (g0 < dim) r.a = *reinterpret_cast<const dm_d2*>(row + (size_t)g0 * 8);
        if (g2 < dim) r.b = *reinterpret_cast<const dm_d2*>(row + (size_t)g2 * 8);
    }
    __device__ __forceinline__ static void unpack(const Raw& r, double (&x)[4]) {
        x[0] = r.a.x;
        x[1] = r.a.y;
        x[2] = r.b.x;
        x[3] = r.b.y;
    }
    // streaming store: the child row is not re-read in this launch
    __device__ __forceinline__ static void store_nt(char* row, int c, int lane, int dim,
                                                    const double (&x)[4]) {
        const int g0 = gene(c, lane, 0), g2 = gene(c, lane, 2);
        if (g0 < dim)
            __builtin_nontemporal_store(dm_d2{x[0], x[1]}, reinterpret_cast<dm_d2*>(row + (size_t)g0 * 8));
        if (g2 < dim)
            __builtin_nontemporal_store(dm_d2{x[2], x[3]}, reinterpret_cast<dm_d2*>(row + (size_t)g2 * 8));
    }
};
// fp32 rows: the ring keeps the loaded floats and widens them only where the
// chunk is used -- a conversion next to the load would wait for it there
// (vmcnt), and the ring would hold no load in flight
template <>
struct ChunkLayout<float> {
    typedef dm_f4 Raw;
    __device__ __forceinline__ static int gene(int c, int lane, int k) {
        return (c << 8) + 4 * lane + k;
    }
    __device__ __forceinline__ static void load(const char* row, int c, int lane, int dim, Raw& r) {
        const int g = gene(c, lane, 0);
        if (g < dim) r = *reinterpret_cast<const dm_f4*>(row + (size_t)g * 4);
    }
    __device__ __forceinline__ static void unpack(const Raw& r, double (&x)[4]) {
        x[0] = r.x;
        x[1] = r.y;
        x[2] = r.z;
        x[3] = r.w;
    }
    __device__ __forceinline__ static void store_nt(char* row, int c, int lane, int dim,
                                                    const double (&x)[4]) {
        const int g = gene(c, lane, 0);
        if (g < dim) Vec4<float>::store_nt(row, g, x);
    }
};

// Single-objective evaluation of one chunk in ChunkLayout<T> (Rastrigin,
// Rosenbrock, or a per-gene sum).  Called by every lane of the wave (the
// Rosenbrock neighbours come through shuffles); `carry` is the previous
// chunk's last gene.
template <typename T, int EC>
__device__ __forceinline__ void pipe_eval_chunk(const dm_eval& ev, int dim, int c, int lane,
                                                const double (&x)[4], const double2* cstab,
                                                bool active, double& acc, double& carry) {
    typedef ChunkLayout<T> L;
    if constexpr (EC == EC_ROSEN) {
        // 100*(x*x - y)**2 + (1. - x)**2 over consecutive genes     (:117-118)
        const int up = (lane + 1) & 63;
        const double s0 = __shfl(x[0], up, 64);
        const double s2 = __shfl(x[2], up, 64);
        const double last = __shfl(x[3], 63, 64);
        if (active) {
            double t = 0.0;
            if (lane == 0 && c > 0 && (c << 8) < dim) t += rosen_term(carry, x[0]);
            if constexpr (sizeof(T) == 8) {
                const int a0 = L::gene(c, lane, 0), b0 = L::gene(c, lane, 2);
                if (a0 + 1 < dim) t += rosen_term(x[0], x[1]);
                if (a0 + 2 < dim) t += rosen_term(x[1], lane < 63 ? s0 : s2);
                if (b0 + 1 < dim) t += rosen_term(x[2], x[3]);
                if (lane < 63 && b0 + 2 < dim) t += rosen_term(x[3], s2);
            } else {
                const int g = L::gene(c, lane, 0);
                if (g + 1 < dim) t += rosen_term(x[0], x[1]);
                if (g + 2 < dim) t += rosen_term(x[1], x[2]);
                if (g + 3 < dim) t += rosen_term(x[2], x[3]);
                if (lane < 63 && g + 4 < dim) t += rosen_term(x[3], s0);
            }
            acc += t;
        }
        carry = last;
    } else if constexpr (EC == EC_RAST) {
        if (active) {
            if (L::gene(c, lane, 3) < dim) {  // all four genes in the row
#if DM_RAST_ILP == 4
                const double t0 = x[0] * x[0] - 10.0 * cos2pi_lds(cstab, x[0]);
                const double t1 = x[1] * x[1] - 10.0 * cos2pi_lds(cstab, x[1]);
                const double t2 = x[2] * x[2] - 10.0 * cos2pi_lds(cstab, x[2]);
                const double t3 = x[3] * x[3] - 10.0 * cos2pi_lds(cstab, x[3]);
                acc += (t0 + t1) + (t2 + t3);
#else
#pragma unroll 1
                for (int h = 0; h < 2; ++h) {  // two independent terms at a time
                    const double a0 = h ? x[2] : x[0], a1 = h ? x[3] : x[1];
                    const double t0 = a0 * a0 - 10.0 * cos2pi_lds(cstab, a0);
                    const double t1 = a1 * a1 - 10.0 * cos2pi_lds(cstab, a1);
                    acc += t0 + t1;
                }
#endif
            } else {
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (L::gene(c, lane, k) < dim) t += x[k] * x[k] - 10.0 * cos2pi_lds(cstab, x[k]);
                acc += t;
            }
        }
    } else if constexpr (EC == EC_SUM) {
        if (active) {
            double t = 0.0;
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const double v = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : x[3];
                if (L::gene(c, lane, k) < dim) t += sum_term(ev.fn, v);
            }
            acc += t;
        }
    }
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
    int32_t bpc;  // dm_knobs.pipe_bpc: workgroups per CU (0 = default)
    // 1: the plans are in parent order (plan_order_kernel), each carries its
    // pair index (flags >> PF_PAIR_SHIFT); a workgroup takes a contiguous run
    // of them, its waves interleaved, so the pairs that share a parent row are
    // varied together on one CU and the row's repeated reads hit its L2
    int32_t ordered;
    Rng rng;
    uint64_t thr_ind;
    double alpha, mu, sigma, w0;
    dm_eval ev;
};

#ifndef DM_PIPE_MINWAVES
#define DM_PIPE_MINWAVES 2
#endif

// Ablation switches for profiling builds only (bit 1: skip evaluation, 2:
// cxBlend without Philox (u = 0.5), 4: skip mutation).  Results are wrong
// in such builds; the product build has DM_PIPE_ABLATE = 0.
#ifndef DM_PIPE_ABLATE
#define DM_PIPE_ABLATE 0
#endif

#ifndef DM_PIPE_DEPTH
#define DM_PIPE_DEPTH 2
#endif

// DEPTH: ring slots (chunks in flight per row); fp32 chunks are half the bytes,
// so their ring is twice as deep (the same 8 KiB in flight per wave)
template <typename T, int NCH, int CX, int MUT, int EC,
          int DEPTH = sizeof(T) == 4 ? 2 * DM_PIPE_DEPTH : DM_PIPE_DEPTH>
__global__ __launch_bounds__(256, DM_PIPE_MINWAVES) void gen_pipe_kernel(PipeArgs a) {
    typedef ChunkLayout<T> L;
    // NCH = 0: rows of any length, the chunk count read at run time (rounded
    // up to whole rings; chunks past the row load and store nothing)
    constexpr int D = NCH == 0 ? DEPTH : NCH < DEPTH ? NCH : DEPTH;
    static_assert(NCH % D == 0, "ring depth must divide the chunk count");
    __shared__ double szig[ZIG_N + 1];
    __shared__ double2 cstab[64];
    if (MUT == DM_MUT_GAUSSIAN)
        for (int i = threadIdx.x; i <= ZIG_N; i += blockDim.x) szig[i] = a.zig[i];
    if (EC == EC_RAST && threadIdx.x < 64) {
        double sn, cn;
        sincospi((double)threadIdx.x / 32.0, &sn, &cn);  // (sin, cos)(2 pi k / 64)
        cstab[threadIdx.x] = make_double2(cn, sn);
    }
    if (MUT == DM_MUT_GAUSSIAN || EC == EC_RAST) __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    // plan slots of this wave: j = wid, wid + nw, ... (pair order), or a
    // contiguous run (parent order); the pair of slot j is j, or the index the
    // ordered plan carries
    int64_t j, jend, jstep;
    if (a.ordered) {
        const int64_t wpb = blockDim.x >> 6;
        const int64_t per = ((npairs + gridDim.x - 1) / gridDim.x + wpb - 1) / wpb * wpb;
        j = (int64_t)blockIdx.x * per + (threadIdx.x >> 6);
        jend = std::min<int64_t>(npairs, (int64_t)blockIdx.x * per + per);
        jstep = wpb;
    } else {
        j = wid;
        jend = npairs;
        jstep = nw;
    }
    if (j >= jend) return;
    int64_t evals = 0;
    const int dim = a.dim;
    const int nchr = NCH > 0 ? NCH : ((dim + 255) / 256 + D - 1) / D * D;
    const double gamma_scale = 1.0 + 2.0 * a.alpha;

    PairPlan pl = load_plan(a.plans, j);
    PairPlan nx = load_plan(a.plans, j + jstep < jend ? j + jstep : j);
    // ring of D chunk slots over the chunk sequence (p,0..NCH-1), (p+W,0..), ...
    typename L::Raw y0[D], y1[D];
#pragma unroll
    for (int ch = 0; ch < D; ++ch) {
        L::load(a.pgenes + (int64_t)pl.s0 * a.pstride, ch, lane, dim, y0[ch]);
        L::load(a.pgenes + (int64_t)pl.s1 * a.pstride, ch, lane, dim, y1[ch]);
    }
    for (; j < jend; j += jstep) {
        const bool more = j + jstep < jend;
        const int64_t j2 = j + 2 * jstep;
        const PairPlan nn = load_plan(a.plans, j2 < jend ? j2 : j);  // two ahead
        const int64_t p = a.ordered ? (int64_t)(pl.flags >> PF_PAIR_SHIFT) : j;
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
        double acc0 = 0.0, acc1 = 0.0, carry0 = 0.0, carry1 = 0.0;
        // chunk ch of the pair, its ring slot sl (compile-time after unrolling)
        auto chunk = [&](const int ch, const int sl) {
            double x0[4], x1[4];
            L::unpack(y0[sl], x0);
            L::unpack(y1[sl], x1);
            // ring: the chunk D ahead into the freed slot (this pair's rows or
            // the next pair's)
            {
                const int ca = ch + D;
                if (ca < nchr) {
                    L::load(r0, ca, lane, dim, y0[sl]);
                    L::load(r1, ca, lane, dim, y1[sl]);
                } else if (more) {
                    L::load(n0, ca - nchr, lane, dim, y0[sl]);
                    L::load(n1, ca - nchr, lane, dim, y1[sl]);
                }
            }
            const uint32_t slot = (uint32_t)((ch << 6) + lane);  // gene_slot of this lane's genes
            if (CX == DM_CX_BLEND && cx) {
                const u32x4 u = (DM_PIPE_ABLATE & 2) ? u32x4{1u << 31, 1u << 31, 1u << 31, 1u << 31}
                                                     : a.rng(ST_BLEND, (uint32_t)p, slot);
                const uint32_t us[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // gamma = (1.+2.*alpha)*random()-alpha; blend   (crossover.py:255-258)
                    const double gm = gamma_scale * u01_32(us[k]) - a.alpha;
                    const double v1 = x0[k], v2 = x1[k];
                    x0[k] = (1.0 - gm) * v1 + gm * v2;
                    x1[k] = gm * v1 + (1.0 - gm) * v2;
                }
            } else if (CX == DM_CX_TWOPOINT && cx) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int gk = L::gene(ch, lane, k);
                    if (gk >= cp1 && gk < cp2) {  // crossover.py:71-72 slice swap
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
            if (MUT == DM_MUT_GAUSSIAN && !(DM_PIPE_ABLATE & 4) && (mut0 || mut1)) {
                // per-gene Bernoulli(indpb) + gauss(mu, sigma)   (mutation.py:44-46)
                uint32_t keep = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) keep |= (L::gene(ch, lane, k) < dim ? 1u : 0u) << k;
                uint32_t bits = 0;
                if (mut0) {
                    const u32x4 w = a.rng(ST_MASK, (uint32_t)c0, slot);
                    bits |= ((uint64_t)w.x < a.thr_ind ? 1u : 0u) | ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                            ((uint64_t)w.z < a.thr_ind ? 4u : 0u) | ((uint64_t)w.w < a.thr_ind ? 8u : 0u);
                }
                if (mut1) {
                    const u32x4 w = a.rng(ST_MASK, (uint32_t)c1, slot);
                    bits |= (((uint64_t)w.x < a.thr_ind ? 1u : 0u) | ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
                             ((uint64_t)w.z < a.thr_ind ? 4u : 0u) | ((uint64_t)w.w < a.thr_ind ? 8u : 0u))
                            << 4;
                }
                bits &= keep | (keep << 4);
#pragma unroll 1
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    bits &= bits - 1;
                    const int j = b & 3;
                    const int gi = L::gene(ch, lane, j);
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
            L::store_nt(w0, ch, lane, dim, x0);
            if (has1) L::store_nt(w1, ch, lane, dim, x1);
            if constexpr (sizeof(T) == 4) {
                // evaluate the stored (fp32-rounded) genes, as DEAP reads array('f')
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x0[k] = (double)(float)x0[k];
                    x1[k] = (double)(float)x1[k];
                }
            }
            if (EC != EC_NONE && !(DM_PIPE_ABLATE & 1)) {
                pipe_eval_chunk<T, EC>(a.ev, dim, ch, lane, x0, cstab, inv0, acc0, carry0);
                pipe_eval_chunk<T, EC>(a.ev, dim, ch, lane, x1, cstab, inv1, acc1, carry1);
            }
        };
        if constexpr (NCH > 0) {
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) chunk(ch, ch % D);
        } else {
#pragma unroll 1
            for (int cb = 0; cb < nchr; cb += D) {
#pragma unroll
                for (int sl = 0; sl < D; ++sl) chunk(cb + sl, sl);
            }
        }
        if (lane == 0) evals += (int64_t)inv0 + (int64_t)inv1;
        if (EC != EC_NONE) {
            const double S0 = group_sum<64>(acc0), S1 = group_sum<64>(acc1);
            if (lane == 0) {
                const double base = EC == EC_RAST || (EC == EC_SUM && a.ev.fn == DM_EVAL_RASTRIGIN)
                                        ? (double)(10 * (int64_t)dim)  // 10*len(individual) + sum
                                        : 0.0;
                a.cwv[c0] = inv0 ? (base + S0) * a.w0 : pl.f0;
                if (has1) a.cwv[c1] = inv1 ? (base + S1) * a.w0 : pl.f1;
                a.cvalid[c0] = 1;
                if (has1) a.cvalid[c1] = 1;
            }
        } else if (lane == 0) {  // no evaluation requested: clones keep their fitness
            if (a.nobj == 1) {
                a.cwv[c0] = pl.f0;
                if (has1) a.cwv[c1] = pl.f1;
            } else {
                const int m = a.nobj;
                for (int o = 0; o < m; ++o) {
                    a.cwv[c0 * m + o] = a.pwv[(int64_t)pl.s0 * m + o];
                    if (has1) a.cwv[c1 * m + o] = a.pwv[(int64_t)pl.s1 * m + o];
                }
            }
            a.cvalid[c0] = inv0 ? 0 : 1;
            if (has1) a.cvalid[c1] = inv1 ? 0 : 1;
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

// Persistent grid of 256-thread workgroups, never more than one wave per
// pair: 64 workgroups per CU in pair order (>= 16x the resident ones): the
// grid drains in many waves of blocks, so late blocks fill CUs whose first
// blocks finished early (A/B on C3, profiles/r01m: 2 resident/CU 3.47 ms;
// 8/CU 3.33-3.40; 32/CU 3.10; 48-64/CU 2.88; 128/CU 2.95; one pair per wave
// 4.84; r01s on a slower box: 32/CU 3.31 ms, 64/CU 3.25).  With the plans in
// label order 32 per CU (runs of 64 pairs per workgroup: more of a bin in one
// L2): 3.102-3.104 ms per step against 3.118-3.123 at 64, 16 / 24 / 48 in
// between, 96 3.15 (profiles/r04_labels/ab_bpc.txt).  bpc > 0 (dm_knobs,
// DM_PIPE_BPC) overrides the per-CU count (A/B experiments).
inline dim3 pipe_grid(int num_cus, int64_t npairs, int bpc, bool ordered) {
    const int occ = bpc > 0 ? bpc : ordered ? 32 : 64;
    const int64_t blocks = std::min<int64_t>((npairs + 3) / 4, (int64_t)num_cus * occ);
    return dim3((unsigned)std::max<int64_t>(blocks, 1));
}
template <typename T, int NCH, int CX, int MUT, int EC>
void launch_pipe_k(const PipeArgs& a, int num_cus, hipStream_t s) {
    auto kern = gen_pipe_kernel<T, NCH, CX, MUT, EC>;
    kern<<<pipe_grid(num_cus, (a.nc + 1) / 2, a.bpc, a.ordered != 0), 256, 0, s>>>(a);
}
template <typename T, int NCH, int CX, int MUT>
void launch_pipe_e(const PipeArgs& a, int ec, int num_cus, hipStream_t s) {
    if (ec == EC_RAST)
        launch_pipe_k<T, NCH, CX, MUT, EC_RAST>(a, num_cus, s);
    else if (ec == EC_ROSEN)
        launch_pipe_k<T, NCH, CX, MUT, EC_ROSEN>(a, num_cus, s);
    else if (ec_single(ec))
        launch_pipe_k<T, NCH, CX, MUT, EC_SUM>(a, num_cus, s);
    else
        launch_pipe_k<T, NCH, CX, MUT, EC_NONE>(a, num_cus, s);
}
template <typename T, int NCH>
void launch_pipe_ops(const PipeArgs& a, int ec, int cx, int mut, int num_cus, hipStream_t s) {
    const bool mg = mut == DM_MUT_GAUSSIAN;
    switch (cx) {
        case DM_CX_BLEND:
            mg ? launch_pipe_e<T, NCH, DM_CX_BLEND, DM_MUT_GAUSSIAN>(a, ec, num_cus, s)
               : launch_pipe_e<T, NCH, DM_CX_BLEND, DM_MUT_NONE>(a, ec, num_cus, s);
            break;
        case DM_CX_TWOPOINT:
            mg ? launch_pipe_e<T, NCH, DM_CX_TWOPOINT, DM_MUT_GAUSSIAN>(a, ec, num_cus, s)
               : launch_pipe_e<T, NCH, DM_CX_TWOPOINT, DM_MUT_NONE>(a, ec, num_cus, s);
            break;
        default:
            mg ? launch_pipe_e<T, NCH, DM_CX_NONE, DM_MUT_GAUSSIAN>(a, ec, num_cus, s)
               : launch_pipe_e<T, NCH, DM_CX_NONE, DM_MUT_NONE>(a, ec, num_cus, s);
    }
}

// Decisions of every pair (thread per pair), generation_pipe_f64.hip.  With
// keys / hist (zeroed, one counter per parent row): key[p] = the plan's sort
// key (its fitter parent), tick[p] = its place among the plans of that key
// (the counter's old value) and hist[key] their count.
// lab64 / epoch: the first label-propagation round of the parent order
// (epoch-tagged labels, generation_pipe_f64.hip lab_of); zero / nzero: ints
// the launch clears for a later launch of the generation
void launch_pair_plans(const GenArgs& a, PairPlan* plans, long long* count_evals, hipStream_t s,
                       int32_t* keys = nullptr, int32_t* hist = nullptr,
                       int32_t* tick = nullptr, uint64_t* lab64 = nullptr, uint32_t epoch = 0,
                       int2* pairs2 = nullptr, int32_t* zero = nullptr, int64_t nzero = 0);
// Parent order: ordered[start[key[p]] + tick[p]] = plans[p] with p in its
// flags (start = the exclusive scan of hist).
void launch_plan_order(const PairPlan* plans, const int32_t* keys, const int32_t* tick,
                       const int32_t* start, PairPlan* ordered, int64_t npairs, hipStream_t s);
// Degree keys (the default; DM_PIPE_KEY_FITTER keys by the fitter parent in
// the plan kernel instead): after launch_pair_plans(..., hist = deg) counted
// every parent slot, key[p] = the parent of more slots, ticketed into hist2.
// jump: the bin also takes the labels of the parents' labels (one more
// propagation round as gathers)
void launch_plan_degree_keys(const PairPlan* plans, const int2* pairs2, const int32_t* deg,
                             const uint64_t* lab64, uint32_t epoch, bool jump, int32_t* keys,
                             int32_t* tick, int32_t* hist2, int64_t npairs, hipStream_t s);
void launch_plan_labels(const int2* pairs2, uint64_t* lab64, uint32_t epoch, int64_t npairs,
                        int rounds, hipStream_t s);
void launch_gen_bits_fused(const GenArgs& a, bool eval, long long* spread, hipStream_t s);
void launch_fit_keys(const GenArgs& a, int16_t* keys, hipStream_t s);
// num_cus: CUs of the device (the persistent grid is sized from it).
void launch_gen_pipe_f64(const PipeArgs& a, int ec, int cx, int mut, int nch, int num_cus,
                         hipStream_t s);
void launch_gen_pipe_f32(const PipeArgs& a, int ec, int cx, int mut, int nch, int num_cus,
                         hipStream_t s);
// rows of at most 64 genes (any objective count), generation_rows_{f64,f32}.hip
void launch_gen_rows_f64(const GenArgs& a, const PairPlan* plans, int ec, int num_cus,
                         hipStream_t s);
void launch_gen_rows_f32(const GenArgs& a, const PairPlan* plans, int ec, int num_cus,
                         hipStream_t s);
// rows of more than 1,024 genes (nch 0: run-time chunk count), generation_pipe_long.hip
void launch_gen_pipe_long(const PipeArgs& a, bool f64, int ec, int cx, int mut, int num_cus,
                          hipStream_t s);
// Packed-bit hot path (generation_pipe_bits.hip): rows of <= 64 words, one objective.
void launch_gen_bits_pipe(const GenArgs& a, const PairPlan* plans, bool eval, int num_cus,
                          hipStream_t s);

}  // namespace dm
