// common.hpp — shared device/host helpers for libdeapmi (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/deapmi.h"

// ---------------------------------------------------------------------------
// Error plumbing: thread-local message + status codes (no exceptions cross the
// C ABI; the ctypes layer maps codes back to DEAP's Python exception types).
// ---------------------------------------------------------------------------
namespace dm {

void set_error(const char* fmt, ...);

#define DM_CHECK_ARG(cond, ...)                 \
    do {                                        \
        if (!(cond)) {                          \
            ::dm::set_error(__VA_ARGS__);       \
            return DM_ERR_INVALID;              \
        }                                       \
    } while (0)

#define DM_HIP(expr)                                                          \
    do {                                                                      \
        hipError_t e_ = (expr);                                               \
        if (e_ != hipSuccess) {                                               \
            ::dm::set_error("HIP error %s at %s:%d: %s", hipGetErrorName(e_), \
                            __FILE__, __LINE__, #expr);                       \
            return DM_ERR_HIP;                                                \
        }                                                                     \
    } while (0)

#define DM_LAUNCH_CHECK() DM_HIP(hipGetLastError())

}  // namespace dm

// Opaque context: one device, one stream, grow-only scratch arena.
constexpr int kEvalSpread = 64, kEvalSpreadStride = 16;  // counters, int64 stride
// evals_spread layout (int64 words): count[g] at g*16, ticket[g] at (64+g)*16,
// the total at 128*16 and its ticket at 129*16 (g < kEvalSpread)
constexpr int kEvalSpreadWords = (2 * kEvalSpread + 2) * kEvalSpreadStride;
// Tuning switches for A/B measurements (tools_gpu/), read ONCE from the
// environment at dm_ctx_create; all off by default.  None of them changes a
// result: every one selects between bit-identical kernels (one exception:
// DM_DISABLE_PIPE's general kernel evaluates Rastrigin's cosine with the
// fdlibm form, the hot kernel with its LDS table -- fitness within 1e-12
// relative), and every one is run against the default by a GPU test
// (tests/test_gpu_knobs.py, test_gpu_fullsize.py).
struct dm_knobs {
    bool disable_pipe = false;      // DM_DISABLE_PIPE: general kernels instead of the hot ones
    bool bits_plan = false;         // DM_BITS_PLAN: C2 through the plan + burst kernels
    bool bits_nokeys = false;       // DM_BITS_NOKEYS: C2 tournaments read wvalues, no int16 keys
    bool lex_full = false;          // DM_LEX_FULL: full lexicographic sort in the grouping
    bool lex_no32 = false;          // DM_LEX_NO32: whole-key objective-0 sort in the grouping
    int32_t pipe_label_rounds = 2;  // DM_PIPE_LABEL_ROUNDS: label propagation rounds of the plan order (2: round 1 + a gather jump)
    bool selbest_fullsort = false;  // DM_SELBEST_FULLSORT: selBest by the full radix sort
    int pipe_bpc = 0;               // DM_PIPE_BPC: C3 workgroups per CU (0 = 32 ordered / 64)
    bool pipe_noorder = false;      // DM_PIPE_NOORDER: C3 plans in pair order (no parent order)
    bool pipe_key_fitter = false;   // DM_PIPE_KEY_FITTER: parent order keyed by the fitter parent
};

struct dm_ctx {
    static constexpr int kSlots = 5;
    int device = 0;
    hipStream_t stream = nullptr;
    void* scratch[kSlots] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t scratch_bytes[kSlots] = {0, 0, 0, 0, 0};
    void* pinned = nullptr;  // small host staging area for host-synchronising calls
    size_t pinned_bytes = 0;
    int num_cus = 256;
    int peel_hint = 4;  // fronts the last fast sortNondominated peeled (first status batch)
    int peel_trend = 0;  // ... and how many more than the call before it
    int64_t peel_hint_U = 0, peel_hint_N = 0;  // ... its unique fitnesses and its k
    double* zig = nullptr;  // ziggurat tables (device), see zig_normal
    // nevals counters (kEvalSpreadWords, zero between launches; see
    // evals_fold): a kernel's workgroups add their counts to 64 counters 128 B
    // apart, the last workgroup of the launch adds the total to nevals
    long long* evals_spread = nullptr;
    // Hot-kernel timing (dm_ctx_set_timing): HIP event pairs recorded on the
    // launch stream around each generation kernel, for bench.py's roofline.
    std::vector<hipEvent_t> tev;
    int tev_used = 0;  // pairs recorded so far
    int timing_target = 0;  // DM_TIME_GENERATION / DM_TIME_DOMINANCE: which launches
    dm_knobs knobs;
    // C3 parent order (generation.hip): the parent graph's labels, persistent
    // and tagged with a per-call epoch in the high 32 bits (nothing zeroes them
    // between generations: a label of an older epoch reads as unset)
    uint64_t* plan_lab = nullptr;
    int64_t plan_lab_n = 0;
    uint32_t plan_epoch = 0;
    // sortNondominated dominance path (dm_ctx_set_dom_path): DM_DOM_DEFAULT or
    // one of the cross-check paths the parity tests compare against it
    int32_t dom_path = 0;
};

namespace dm {
// Called by ONE thread of every workgroup of a launch (all of them, count 0
// included) with the workgroup's count: adds it into counter blockIdx % 64,
// and the workgroup that completes the launch adds the total to *nevals and
// leaves every counter at zero.  Same-address atomics stay bounded (one
// atomic per workgroup into ONE address serialised at one L2 channel: 0.19
// ms per C2 generation).  Ordering uses returning atomics and a vmcnt wait
// (each is performed before the next issues), never a fence: an agent-scope
// release writes the L2 back and cost 0.7 ms per C2 launch.
__device__ __forceinline__ unsigned long long atomic_add_ret(unsigned long long* p,
                                                            unsigned long long v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long atomic_exch_ret(unsigned long long* p,
                                                             unsigned long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void evals_fold(long long* spread, int64_t* nevals, long long count) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(spread);
    const unsigned nb = gridDim.x;
    const unsigned g = blockIdx.x % kEvalSpread;
    const unsigned gsize = nb / kEvalSpread + (g < nb % kEvalSpread ? 1u : 0u);
    // each atomic is performed (returned) before the next issues
    atomic_add_ret(w + g * kEvalSpreadStride, (unsigned long long)count);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long tk = atomic_add_ret(w + (kEvalSpread + g) * kEvalSpreadStride, 1ull);
    if (tk != gsize - 1) return;
    // last workgroup of group g: every count of the group is in
    const unsigned long long gt = atomic_exch_ret(w + g * kEvalSpreadStride, 0ull);
    atomic_exch_ret(w + (kEvalSpread + g) * kEvalSpreadStride, 0ull);
    atomic_add_ret(w + 2 * kEvalSpread * kEvalSpreadStride, gt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned ngroups = nb < (unsigned)kEvalSpread ? nb : (unsigned)kEvalSpread;
    const unsigned long long tt = atomic_add_ret(w + (2 * kEvalSpread + 1) * kEvalSpreadStride, 1ull);
    if (tt != ngroups - 1) return;
    const unsigned long long tot = atomic_exch_ret(w + 2 * kEvalSpread * kEvalSpreadStride, 0ull);
    atomic_exch_ret(w + (2 * kEvalSpread + 1) * kEvalSpreadStride, 0ull);
    *nevals += (int64_t)tot;
}

// Event pair i around the next launch of the timed kind (target: 0 = the
// generation kernel, 1 = the NSGA-II dominance kernel; no-op when timing is
// off, another kind is timed, or every pair has been used).
inline void timing_begin(dm_ctx* ctx, int target = 0) {
    const int i = ctx->tev_used;
    if (target == ctx->timing_target && 2 * i + 1 < (int)ctx->tev.size())
        (void)hipEventRecord(ctx->tev[2 * i], ctx->stream);
}
inline void timing_end(dm_ctx* ctx, int target = 0) {
    const int i = ctx->tev_used;
    if (target == ctx->timing_target && 2 * i + 1 < (int)ctx->tev.size()) {
        (void)hipEventRecord(ctx->tev[2 * i + 1], ctx->stream);
        ctx->tev_used = i + 1;
    }
}
}  // namespace dm

namespace dm {
// Grow-only scratch arenas; returns nullptr on failure (error set).  Growing
// a slot discards its contents.  Slot 0 = general temporaries, 1 = NSGA-II
// dominance matrix, 2 = NSGA-II order buffers, 3 = migration placement,
// 4 = migration emigrant / immigrant / receive blocks.
void* scratch_slot(dm_ctx* ctx, int slot, size_t bytes);
inline void* scratch(dm_ctx* ctx, size_t bytes) { return scratch_slot(ctx, 0, bytes); }
void* pinned(dm_ctx* ctx, size_t bytes);
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace dm

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Counter layout of the whole library
// (DESIGN.md §RNG): ctr = {item, sub, gen, (stage << 16) | island},
// key = {seed lo, seed hi}.
// ---------------------------------------------------------------------------
namespace dm {

enum Stage : uint32_t {
    ST_SEL = 1,     // tournament / selRandom aspirants: item = child, sub = draw/2
    ST_CX = 2,      // pair flag + cxTwoPoint raw cut draws: item = pair
    ST_BLEND = 3,   // cxBlend per-gene u: item = pair, sub = gene/4
    ST_MUT = 4,     // per-individual mutation flag: item = child
    ST_MASK = 5,    // per-gene Bernoulli(indpb) (float genomes): sub = gene/4
    ST_GAUSS = 6,   // per-gene normal: sub = gene
    ST_FLIP = 7,    // packed-bit geometric skips: sub = (word << 8) | call
    ST_VAROR = 8,   // varOr op choice + indices: item = child
    ST_INIT = 9,    // initial population
    ST_DCD = 10,    // selTournamentDCD: tie coins (item = tournament slot, sub = 2),
                    // permutation q's sort keys (item = index, sub = 4 + q)
    ST_SBX_PAIR = 11,  // NSGA-II loop pair random() <= cxpb: item = pair
    ST_SBX = 12,       // cxSimulatedBinaryBounded per gene: item = pair, sub = gene
                       // (| 1 << 24 for the swap coin)
    ST_POLY = 13,      // mutPolynomialBounded per gene: item = child, sub = gene
    ST_SAMPLE = 14,    // random.sample: item = attempt (rejection) or row (keys), sub = 0 / 1
};

struct u32x4 {
    uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

struct Rng {
    uint32_t k0 = 0, k1 = 0, gen = 0, island = 0;
    Rng() = default;
    __host__ __device__ Rng(const dm_rng& r)
        : k0((uint32_t)r.seed), k1((uint32_t)(r.seed >> 32)), gen(r.gen), island(r.island) {}
    __host__ __device__ __forceinline__ u32x4 operator()(uint32_t stage, uint32_t item,
                                                         uint32_t sub) const {
        return philox4x32_10(u32x4{item, sub, gen, (stage << 16) | (island & 0xFFFFu)}, k0, k1);
    }
};

// Bernoulli threshold: P(w < thr) = thr / 2^32 = floor(p * 2^32) / 2^32.
__host__ __device__ __forceinline__ uint64_t prob_threshold(double p) {
    if (!(p > 0.0)) return 0;
    if (p >= 1.0) return 1ull << 32;
    return (uint64_t)(p * 4294967296.0);
}
// Bounded integer in [0, n) from a 64-bit word: floor(v * n / 2^64).
// Exactly uniform when n is a power of two; otherwise bias <= n / 2^64.
__host__ __device__ __forceinline__ uint32_t bounded64(uint32_t lo, uint32_t hi, uint32_t n) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
#ifdef __HIP_DEVICE_COMPILE__
    return (uint32_t)__umul64hi(v, (uint64_t)n);
#else
    return (uint32_t)(((unsigned __int128)v * n) >> 64);
#endif
}
// 32-bit uniform in [0,1): exact in fp64.
__host__ __device__ __forceinline__ double u01_32(uint32_t w) { return (double)w * 2.3283064365386963e-10; }
// 53-bit uniform in [0,1) from two words.
__host__ __device__ __forceinline__ double u01_53(uint32_t lo, uint32_t hi) {
    const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)v * 1.1102230246251565e-16;
}

// ---------------------------------------------------------------------------
// Standard normal by the 256-layer ziggurat (Marsaglia & Tsang 2000, fp64,
// 53-bit uniforms): ~98.8% of draws are one table lookup and one multiply;
// the rest test the wedge with exp() or sample the tail with log().  Tables
// live in a small device buffer of the context, filled by dm_ctx_create
// (zig_make_tables).  Draw `attempt` of (stream, item, sub < 2^23) uses Philox
// call (item, sub | attempt << 24): 4 words = layer/sign, 53-bit uniform,
// wedge uniform; the tail takes a fresh call with bit 23 of sub set.
// ---------------------------------------------------------------------------
constexpr int ZIG_N = 256;
// zig[0..256] = layer edges (zig[0] = V/f(R), zig[1] = R, zig[256] = 0),
// zig[257..513] = f(edge) = exp(-edge^2/2).  Device copy owned by the ctx.
int zig_make_tables(double* host513x2);

__device__ __forceinline__ double zig_normal(const double* __restrict__ zig, const Rng& rng,
                                             uint32_t stage, uint32_t item, uint32_t sub) {
    const double* zig_x = zig;
    const double* zig_f = zig + (ZIG_N + 1);
    constexpr double R = 3.6541528853610088;
    for (uint32_t attempt = 0; attempt < 64; ++attempt) {
        const u32x4 w = rng(stage, item, sub | (attempt << 24));
        const int layer = (int)(w.x & (ZIG_N - 1));
        const bool neg = (w.x >> 8) & 1;
        const double u = u01_53(w.y & 0xFFFFF800u, w.z);  // 53-bit uniform in [0,1)
        const double x = u * zig_x[layer];
        if (x < zig_x[layer + 1]) return neg ? -x : x;  // inside the rectangle
        if (layer == 0) {
            // tail beyond R (Marsaglia 1964): x = -ln(u1)/R, y = -ln(u2), accept 2y > x^2
            const u32x4 t = rng(stage, item, sub | (attempt << 24) | (1u << 23));
            const double u1 = u01_53(t.x, t.y);
            const double u2 = u01_53(t.z, t.w);
            const double xt = -log1p(-u1) / R;
            const double yt = -log1p(-u2);
            if (yt + yt > xt * xt) return neg ? -(R + xt) : (R + xt);
            continue;
        }
        const double y = zig_f[layer + 1] + u01_32(w.w) * (zig_f[layer] - zig_f[layer + 1]);
        if (y < exp(-0.5 * x * x)) return neg ? -x : x;  // wedge
    }
    return 0.0;  // unreachable in practice (acceptance ~0.99 per attempt)
}

}  // namespace dm

// ---------------------------------------------------------------------------
// Wave helpers (wave64).
// ---------------------------------------------------------------------------
namespace dm {
template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int G>
__device__ __forceinline__ int64_t group_sum_i(int64_t v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// DEAP Fitness.__gt__ (base.py:234-235) = not (a.wvalues <= b.wvalues), with
// Python tuple semantics: first index whose elements are not ==, then <=.
__host__ __device__ __forceinline__ bool fit_gt(const double* a, const double* b, int m) {
    for (int j = 0; j < m; ++j) {
        if (!(a[j] == b[j])) return !(a[j] <= b[j]);
    }
    return false;  // equal tuples: a <= b holds
}
// a < b lexicographic (tuple __lt__).
__host__ __device__ __forceinline__ bool fit_lt(const double* a, const double* b, int m) {
    for (int j = 0; j < m; ++j) {
        if (!(a[j] == b[j])) return a[j] < b[j];
    }
    return false;
}
}  // namespace dm
