// nsga2.hip — sortNondominated / assignCrowdingDist / selNSGA2
// (deap/tools/emo.py:15-143) for gfx950.
//
// sortNondominated reproduces DEAP's exact front order:
//   1. equal fitnesses are grouped (dict keyed by Fitness, first-appearance
//      order) -> unique fits U in order of their first individual;
//   2. the dominance relation over U is materialised as a bit matrix
//      D[u][v] = fit_u dominates fit_v  (U x ceil(U/64) words, LDS-tiled
//      O(M*U^2) pass) together with count[v] = #dominators of v;
//   3. front 0 = {count == 0} in U order; front r+1 = the v whose last
//      remaining dominators are in front r, ordered by (position in front r
//      of the *last* dominator that releases v, U index) — the order in which
//      the reference's peel loop appends them (emo.py:106-115).  Each peel
//      reads the D rows of the front's members once: a wave transposes 64x64
//      bit blocks (64 members x one 64-wide word of v) with lane shuffles and
//      accumulates per-v dominator counts and last positions;
//   4. unique fits expand to their individuals in population order, fronts are
//      emitted until >= min(n, k) individuals are sorted.
// assignCrowdingDist reproduces the reference's chained stable sorts: for
// objective i the order is lexicographic in (v_i, v_{i-1}, ..., v_0, front
// position), distances accumulate in objective order with IEEE division.
#include "sort.hpp"

namespace dm {

int validate_pop(const dm_pop* p, const char* what);
int sort_by_fitness(dm_ctx* ctx, const double* wv, int nobj, int64_t n, bool desc,
                    int32_t* vals_out);
// dominance.hip: integer ranks in objective-0 order, lower-triangle dominance,
// device-driven peel
size_t fast_dom_bytes(int64_t n, int64_t U);
int64_t fast_dom_words(int64_t U);
int fast_dom_build(dm_ctx* ctx, const double* wv, int m, int64_t n,
                   const int32_t* perm, const int32_t* segin, const int32_t* uidx,
                   const double* ufit, int64_t U, uint64_t* D, int32_t* count, char* ws);
int fast_rank_keys(dm_ctx* ctx, const char* ws, int64_t n, int64_t U, int m, const int32_t* ui,
                   const int32_t* order, int64_t T, int32_t* rk);
bool fast_table_peel(const dm_ctx* ctx, int m);
int fast_fronts(dm_ctx* ctx, const uint64_t* D, int m, int64_t n, int64_t U, const int32_t* F0,
                const int64_t* sorted0,
                int64_t N, const int32_t* gsize, int32_t* ulist, int32_t* rankU, int32_t* count,
                int32_t* fstarts, char* ws, std::vector<int32_t>& ufront, int64_t* sorted,
                int64_t* last_inds, int64_t* max_inds = nullptr);

// ---------------------------------------------------------------------------
// Workspace bump allocator over the context scratch
// ---------------------------------------------------------------------------
struct Bump {
    char* base;
    size_t off = 0;
    template <typename T>
    T* take(int64_t count) {
        T* p = reinterpret_cast<T*>(base + off);
        off += align_up((size_t)std::max<int64_t>(count, 1) * sizeof(T), 256);
        return p;
    }
};

static dim3 g1(int64_t n) {
    return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65535)));
}

#define GRID_LOOP(i, n)                                                          \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
         i += (int64_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------------------------
// 1. grouping of equal fitnesses
// ---------------------------------------------------------------------------
// isrep is written for every row (perm is a permutation: no zeroing pass);
// *nanflag (zeroed by the caller) is set when any objective value is NaN
__global__ void seg_flag_kernel(const double* wv, int m, const int32_t* perm, int64_t n,
                                int32_t* segstart_in, int32_t* isrep, int32_t* nanflag) {
    GRID_LOOP(j, n) {
        const double* a = wv + (int64_t)perm[j] * m;
        bool start = j == 0, nan = false;
        for (int o = 0; o < m; ++o) nan |= a[o] != a[o];
        if (!start) {
            const double* b = wv + (int64_t)perm[j - 1] * m;
            for (int o = 0; o < m; ++o)
                if (!(a[o] == b[o])) start = true;
        }
        segstart_in[j] = start ? (int32_t)j : 0;
        isrep[perm[j]] = start ? 1 : 0;
        if (nan) *nanflag = 1;
    }
}
// After a stable sort by objective 0 alone (keys0: the sorted objective-0
// keys): the runs of equal objective 0 that are out of lexicographic order in
// the other objectives are sorted in place, which gives the order of the full
// lexicographic sort.  lex_bad_kernel flags the start of every run holding an
// adjacent pair out of order (a run starts in index order, and identical rows
// -- clones -- are in order); lex_run_sort_kernel sorts each flagged run with
// one wave (a bitonic sort over the lanes of (objectives 1.., index)).  A
// flagged run longer than LEX_RUN_CAP = 64 sets *overflow: the caller then
// sorts in full.
constexpr int LEX_RUN_CAP = 64;
// o0: the first objective compared (1 after the whole-key objective-0 sort; 0
// after the 32-bit one, whose runs of equal top bits may differ in objective 0)
__device__ __forceinline__ bool lex_less_rest(const double* wv, int m, int32_t x, int32_t y,
                                              int o0) {
    const double* a = wv + (int64_t)x * m;
    const double* b = wv + (int64_t)y * m;
    for (int o = o0; o < m; ++o) {
        const uint64_t ka = ordered_key(a[o]), kb = ordered_key(b[o]);
        if (ka != kb) return ka < kb;
    }
    return x < y;
}
// kshift: runs are rows whose objective-0 keys agree above bit kshift (0: the
// whole key; 32: the top half, what a 4-pass radix sort orders)
__global__ void lex_bad_kernel(const double* wv, int m, const uint64_t* keys0, const int32_t* perm,
                               int64_t n, int32_t* runflag, int32_t* overflow, int kshift) {
    const int o0 = kshift ? 0 : 1;
    GRID_LOOP(j, n) {
        const uint64_t kj = keys0[j] >> kshift;
        if (j == 0 || kj != keys0[j - 1] >> kshift) continue;
        if (lex_less_rest(wv, m, perm[j - 1], perm[j], o0)) continue;
        int64_t st = j - 1;
        while (st > 0 && keys0[st - 1] >> kshift == kj && j - st < LEX_RUN_CAP) --st;
        if (st > 0 && keys0[st - 1] >> kshift == kj) {
            *overflow = 1;
            continue;
        }
        runflag[st] = 1;
    }
}
struct LexRest {
    uint64_t k[3];
    int32_t x;
};
__device__ __forceinline__ bool lex_rest_less(const LexRest& a, const LexRest& b) {
    for (int o = 0; o < 3; ++o)
        if (a.k[o] != b.k[o]) return a.k[o] < b.k[o];
    return a.x < b.x;
}
__device__ __forceinline__ uint64_t shfl_xor_u64l(uint64_t v, int mask) {
    const int lo = __shfl_xor((int)(uint32_t)v, mask, 64);
    const int hi = __shfl_xor((int)(uint32_t)(v >> 32), mask, 64);
    return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}
__global__ __launch_bounds__(256) void lex_run_sort_kernel(const double* wv, int m,
                                                           const uint64_t* keys0, int32_t* perm,
                                                           int64_t n, const int32_t* runflag,
                                                           int32_t* overflow, int kshift) {
    const int lane = threadIdx.x & 63;
    const int o0 = kshift ? 0 : 1;  // the whole-key sort leaves objective 0 equal in a run
    const int64_t base = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64;
    if (base >= n) return;
    uint64_t todo = __ballot(base + lane < n && runflag[base + lane] != 0);
    while (todo) {  // wave-uniform
        const int64_t st = base + __ffsll((long long)todo) - 1;
        todo &= todo - 1;
        const uint64_t k0 = keys0[st] >> kshift;
        if (st + LEX_RUN_CAP < n && keys0[st + LEX_RUN_CAP] >> kshift == k0) {
            if (lane == 0) *overflow = 1;
            continue;
        }
        const int64_t i = st + lane;
        const bool in = i < n && keys0[i] >> kshift == k0;
        LexRest r;
        r.x = in ? perm[i] : INT32_MAX;
        for (int o = 0; o < 3; ++o)
            r.k[o] = in && o + o0 < m ? ordered_key(wv[(int64_t)r.x * m + o + o0]) : (in ? 0ull : ~0ull);
        for (int size = 2; size <= 64; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                LexRest p;
                for (int o = 0; o < 3; ++o) p.k[o] = shfl_xor_u64l(r.k[o], stride);
                p.x = __shfl_xor(r.x, stride, 64);
                const bool lower = (lane & stride) == 0;
                const bool up = (lane & size) == 0;
                const bool pl = lex_rest_less(p, r);
                // lower lane of an ascending pair keeps the minimum
                if ((lower == up) ? pl : !pl && (p.x != r.x)) r = p;
            }
        }
        if (in) perm[i] = r.x;
    }
}
__global__ void zero_i32_kernel(int32_t* p, int64_t n) {
    GRID_LOOP(i, n) p[i] = 0;
}
__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
    GRID_LOOP(i, n) p[i] = v;
}
// the per-unique-fit arrays of a sort: group sizes and counts 0, ranks -1
__global__ void unique_init_kernel(int32_t* gsize, int32_t* count, int32_t* rankU, int64_t U) {
    GRID_LOOP(i, U) {
        gsize[i] = 0;
        count[i] = 0;
        rankU[i] = -1;
    }
}
// ui[i] = unique index of individual i; ufit / useg / gsize per unique fit.
__global__ void unique_kernel(const double* wv, int m, const int32_t* perm, const int32_t* segstart,
                              const int32_t* uidx_of_rep, int64_t n, int32_t* ui, double* ufit,
                              int32_t* useg, int32_t* gsize) {
    GRID_LOOP(j, n) {
        const int32_t s = segstart[j];
        const int32_t rep = perm[s];
        const int32_t u = uidx_of_rep[rep];
        const int32_t i = perm[j];
        ui[i] = u;
        atomicAdd(&gsize[u], 1);
        if (s == j) {
            useg[u] = (int32_t)j;
            for (int o = 0; o < m; ++o) ufit[(int64_t)u * m + o] = wv[(int64_t)i * m + o];
        }
    }
}

// ---------------------------------------------------------------------------
// 2. dominance bit matrix + dominator counts
// ---------------------------------------------------------------------------
constexpr int DT_WORDS = 32;   // words of v per tile -> 2048 v
constexpr int DT_ROWS = 256;   // rows u per block

__global__ __launch_bounds__(256) void dom_build_kernel(const double* ufit, int m, int64_t U,
                                                        int64_t W, uint64_t* D, int32_t* count) {
    extern __shared__ __attribute__((aligned(16))) double sfit[];  // [m][64][DT_WORDS]
    const int64_t w0 = (int64_t)blockIdx.x * DT_WORDS;
    for (int e = threadIdx.x; e < m * 64 * DT_WORDS; e += blockDim.x) {
        const int o = e / (64 * DT_WORDS);
        const int b = (e / DT_WORDS) % 64;
        const int wl = e % DT_WORDS;
        const int64_t v = (w0 + wl) * 64 + b;
        sfit[e] = v < U ? ufit[v * m + o] : __builtin_nan("");
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wl = lane & 31;
    const int half = lane >> 5;
    const int64_t w = w0 + wl;
    const int64_t u_begin = (int64_t)blockIdx.y * DT_ROWS;
    const int64_t u_end = std::min<int64_t>(U, u_begin + DT_ROWS);
    for (int64_t u = u_begin + wave * 2 + half; u < u_end; u += 8) {
        double fu[DM_MAX_OBJ];
        for (int o = 0; o < m; ++o) fu[o] = ufit[u * m + o];
        uint64_t bits = 0;
        int cnt = 0;
        for (int b = 0; b < 64; ++b) {
            bool gt = false, lt = false;  // NaN objectives compare equal (base.py:209-224)
            for (int o = 0; o < m; ++o) {
                const double x = fu[o];
                const double y = sfit[(o * 64 + b) * DT_WORDS + wl];
                gt |= x > y;
                lt |= x < y;
            }
            bits |= (uint64_t)(gt && !lt) << b;  // u dominates v
            cnt += (lt && !gt) ? 1 : 0;          // v dominates u
        }
        if (w < W) D[u * W + w] = bits;
        // reduce cnt over the 32 lanes of this half-wave
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if (wl == 0 && cnt) atomicAdd(&count[u], cnt);
    }
}

// Ballot form (the path taken for 2..4 objectives).  A wave owns DB_WPW
// consecutive words of v (lane L of word k <-> v = 64*(w0+k) + L, fitness in
// VGPRs) and sweeps a tile of DB_ROWS rows u with u wave-uniform (fitness
// from scalar loads).  Fitness.dominates (base.py:209-224) returns False at
// the first objective with x < y and needs one with x > y — an objective where
// either side is NaN counts as equal — so with one wave mask per objective
// and compare over the 64 lanes:
//   D[u][w]                = ANY(x > y) & ~ANY(x < y)     (u dominates v)
//   #v in w dominating u   = popcount(ANY(x < y) & ~ANY(x > y))
// The mask of row u is parked in lane u%64 and every 64 rows each lane stores
// its row's DB_WPW words; dominator counts go to per-word-group partials
// cpart[g][u] (summed by dom_count_reduce_kernel, no atomics).
// Tile A/B on C5 (2^18 rows, M = 3; r01t): 8 words x 512 rows 29.8 ms/gen,
// 4 x 1024 29.0-29.4, 4 x 512 29.2, 16 x 512 35.0, 2 x 2048 36.4.
#ifndef DM_DB_WPW
#define DM_DB_WPW 4
#endif
#ifndef DM_DB_ROWS
#define DM_DB_ROWS 1024
#endif
constexpr int DB_WPW = DM_DB_WPW;    // words per wave (256 v)
constexpr int DB_ROWS = DM_DB_ROWS;  // rows u per wave

template <int M>
__global__ __launch_bounds__(256) void dom_ballot_kernel(const double* __restrict__ ufit, int64_t U,
                                                         int64_t W, int64_t ngroups,
                                                         int64_t ntiles, uint64_t* __restrict__ D,
                                                         int32_t* __restrict__ cpart) {
    const int lane = threadIdx.x & 63;
    const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (gw >= ngroups * ntiles) return;
    const int64_t grp = gw % ngroups, tile = gw / ngroups;
    const int64_t w0 = grp * DB_WPW;
    double y[DB_WPW][M];
    uint64_t vmask[DB_WPW];
#pragma unroll
    for (int k = 0; k < DB_WPW; ++k) {
        const int64_t v = (w0 + k) * 64 + lane;
        const bool in = v < U;
#pragma unroll
        for (int o = 0; o < M; ++o) y[k][o] = in ? ufit[v * M + o] : 0.0;
        vmask[k] = __ballot(in);
    }
    const int64_t u_begin = tile * DB_ROWS;
    const int64_t u_end = u_begin + DB_ROWS < U ? u_begin + DB_ROWS : U;
    for (int64_t ub = u_begin; ub < u_end; ub += 64) {
        const int nb = (int)(u_end - ub < 64 ? u_end - ub : 64);
        uint64_t acc[DB_WPW];
#pragma unroll
        for (int k = 0; k < DB_WPW; ++k) acc[k] = 0;
        int32_t cacc = 0;
        for (int j = 0; j < nb; ++j) {
            const int64_t u = ub + j;
            double x[M];
#pragma unroll
            for (int o = 0; o < M; ++o) x[o] = ufit[u * M + o];
            int32_t cnt = 0;
#pragma unroll
            for (int k = 0; k < DB_WPW; ++k) {
                uint64_t gt = 0, lt = 0;
#pragma unroll
                for (int o = 0; o < M; ++o) {
                    gt |= __ballot(x[o] > y[k][o]);
                    lt |= __ballot(x[o] < y[k][o]);
                }
                const uint64_t dom = gt & ~lt & vmask[k];
                cnt += __popcll(lt & ~gt & vmask[k]);
                acc[k] = lane == j ? dom : acc[k];
            }
            cacc = lane == j ? cnt : cacc;
        }
        if (lane < nb) {
            uint64_t* row = D + (ub + lane) * W + w0;
#pragma unroll
            for (int k = 0; k < DB_WPW; ++k)
                if (w0 + k < W) row[k] = acc[k];
            cpart[grp * U + ub + lane] = cacc;
        }
    }
}

__global__ void dom_count_reduce_kernel(const int32_t* __restrict__ cpart, int64_t ngroups,
                                        int64_t U, int32_t* __restrict__ count) {
    GRID_LOOP(u, U) {
        int32_t c = 0;
        for (int64_t g = 0; g < ngroups; ++g) c += cpart[g * U + u];
        count[u] = c;
    }
}

template <int M>
static void launch_dom_ballot(const double* ufit, int64_t U, int64_t W, uint64_t* D,
                              int32_t* cpart, hipStream_t s) {
    const int64_t ngroups = (W + DB_WPW - 1) / DB_WPW;
    const int64_t ntiles = (U + DB_ROWS - 1) / DB_ROWS;
    const int64_t waves = ngroups * ntiles;
    dom_ballot_kernel<M><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(ufit, U, W, ngroups,
                                                                        ntiles, D, cpart);
}

// ---------------------------------------------------------------------------
// 3. fronts
// ---------------------------------------------------------------------------
__global__ void flag_zero_count_kernel(const int32_t* count, int64_t U, int32_t* flag) {
    GRID_LOOP(u, U) flag[u] = count[u] == 0 ? 1 : 0;
}
// Compaction: members in U order.  keys (optional) from key_src.
__global__ void compact_kernel(const int32_t* flag, const int32_t* pos, int64_t U, int32_t* out,
                               const int32_t* key_src, uint64_t* keys_out, int32_t* rankU,
                               int32_t rank) {
    GRID_LOOP(u, U) {
        if (flag[u]) {
            out[pos[u]] = (int32_t)u;
            if (keys_out) keys_out[pos[u]] = (uint64_t)(uint32_t)key_src[u];
            rankU[u] = rank;
        }
    }
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)x, m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
// 64x64 bit transpose across the wave: in lane i bit j = A[i][j]; out lane j
// bit i = A[i][j].
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane) {
    const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull,
                               0x00FF00FF00FF00FFull, 0x0F0F0F0F0F0F0F0Full,
                               0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int s = 32 >> st;
        const uint64_t mlo = masks[st];
        const uint64_t y = shfl_xor64(x, s);
        if (lane & s)
            x = (x & ~mlo) | ((y & ~mlo) >> s);
        else
            x = (x & mlo) | ((y & mlo) << s);
    }
    return x;
}

constexpr int PEEL_WORDS = 16;

// part_dec[c][v] = #members of chunk c dominating v; part_last[c][v] = last
// (max) front position among them, or -1.
__global__ __launch_bounds__(256) void peel_kernel(const uint64_t* D, int64_t W, int64_t U,
                                                   const int32_t* members, int64_t F,
                                                   int64_t chunk, int64_t tiles, int64_t nchunks,
                                                   int32_t* part_dec, int32_t* part_last) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wid >= tiles * nchunks) return;
    const int64_t t = wid % tiles;
    const int64_t c = wid / tiles;
    const int64_t wbase = t * PEEL_WORDS;
    int32_t dec[PEEL_WORDS], last[PEEL_WORDS];
#pragma unroll
    for (int k = 0; k < PEEL_WORDS; ++k) {
        dec[k] = 0;
        last[k] = -1;
    }
    const int64_t jb = c * chunk, je = std::min<int64_t>(F, jb + chunk);
    for (int64_t j0 = jb; j0 < je; j0 += 64) {
        const int64_t j = j0 + lane;
        const bool ok = j < je;
        const int64_t u = ok ? members[j] : 0;
        const uint64_t* row = D + u * W;
#pragma unroll
        for (int k = 0; k < PEEL_WORDS; ++k) {
            const int64_t w = wbase + k;
            const uint64_t x = (ok && w < W) ? row[w] : 0ull;
            const uint64_t tcol = transpose64(x, lane);  // lane b: bit i = member j0+i dominates v
            dec[k] += __popcll(tcol);
            if (tcol) last[k] = (int32_t)(j0 + 63 - __clzll(tcol));
        }
    }
#pragma unroll
    for (int k = 0; k < PEEL_WORDS; ++k) {
        const int64_t v = (wbase + k) * 64 + lane;
        if (v < U) {
            part_dec[c * U + v] = dec[k];
            part_last[c * U + v] = last[k];
        }
    }
}

__global__ void peel_combine_kernel(const int32_t* part_dec, const int32_t* part_last,
                                    int64_t nchunks, int64_t U, int32_t* count,
                                    const int32_t* rankU, int32_t* flag, int32_t* lastpos) {
    GRID_LOOP(v, U) {
        int32_t dec = 0, last = -1;
        for (int64_t c = 0; c < nchunks; ++c) {
            dec += part_dec[c * U + v];
            last = max(last, part_last[c * U + v]);
        }
        int32_t f = 0;
        if (dec > 0 && rankU[v] < 0) {
            const int32_t left = count[v] - dec;
            count[v] = left;
            if (left == 0) f = 1;
        }
        flag[v] = f;
        lastpos[v] = last;
    }
}

__global__ void sum_gsize_kernel(const int32_t* members, int64_t F, const int32_t* gsize,
                                 int64_t* total) {
    __shared__ int64_t sh[256];
    int64_t acc = 0;
    GRID_LOOP(j, F) acc += gsize[members[j]];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && sh[0]) atomicAdd((unsigned long long*)total, (unsigned long long)sh[0]);
}
__global__ void sum_gsize_dev_kernel(const int32_t* members, const int32_t* Fp, const int32_t* gsize,
                                     int64_t* total) {
    __shared__ int64_t sh[256];
    const int64_t F = *Fp;
    int64_t acc = 0;
    GRID_LOOP(j, F) acc += gsize[members[j]];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && sh[0]) atomicAdd((unsigned long long*)total, (unsigned long long)sh[0]);
}

// ---------------------------------------------------------------------------
// 4. expansion to individuals
// ---------------------------------------------------------------------------
__global__ void member_sizes_kernel(const int32_t* ulist, int64_t T, const int32_t* gsize,
                                    int32_t* sizes) {
    GRID_LOOP(j, T) sizes[j] = gsize[ulist[j]];
}
__global__ void expand_kernel(const int32_t* ulist, int64_t T, const int32_t* outpos,
                              const int32_t* useg, const int32_t* gsize, const int32_t* perm,
                              int32_t* order) {
    GRID_LOOP(j, T) {
        const int32_t u = ulist[j];
        const int32_t s = useg[u], g = gsize[u], o = outpos[j];
        for (int32_t t = 0; t < g; ++t) order[o + t] = perm[s + t];
    }
}
__global__ void ind_rank_kernel(const int32_t* ui, const int32_t* rankU, int64_t n, int32_t* rank) {
    GRID_LOOP(i, n) rank[i] = rankU[ui[i]];
}
__global__ void front_start_kernel(const int32_t* ufront_start, int32_t nfronts,
                                   const int32_t* outpos, int64_t T, int32_t total,
                                   int32_t* fstart) {
    GRID_LOOP(f, (int64_t)nfronts + 1) {
        const int32_t us = ufront_start[f];
        fstart[f] = us < T ? outpos[us] : total;
    }
}

// Host-side driver ----------------------------------------------------------
struct SortResult {
    int64_t nsorted = 0;
    int32_t nfronts = 0;
    int64_t last_inds = 0;  // individuals of the last emitted front
    int64_t max_inds = INT64_MAX;  // individuals of the largest emitted front (if known)
    int64_t U = 0;          // unique fitnesses
    bool rank_keys = false; // rank_keys filled (fast path)
};

// rank_keys (nullable, m * n int32): filled with the emitted individuals'
// per-objective integer ranks when the fast path runs (res->rank_keys).
static int sort_nondominated_impl(dm_ctx* ctx, const dm_pop* pop, int64_t k, bool first_only,
                                  int32_t* order, int32_t* front_start, int32_t* rank,
                                  SortResult* res, int32_t* rank_keys = nullptr) {
    hipStream_t s = ctx->stream;
    const int64_t n = pop->n;
    const int m = pop->nobj;
    const double* wv = pop->wvalues;
    if (n == 0 || k == 0) {
        res->nsorted = 0;
        res->nfronts = 0;
        if (rank && n) fill_i32_kernel<<<g1(n), 256, 0, s>>>(rank, n, -1);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    // ---- workspace: everything O(n) in slot 0 (U <= n), D in slot 1 ----
    const int64_t max_chunks = 64;
    const size_t nb8 = align_up((size_t)n * 8, 256), nb4 = align_up((size_t)(n + 2) * 4, 256);
    const size_t need = 2 * nb8 + 20 * nb4 + align_up((size_t)n * m * 8, 256) +
                        2 * align_up((size_t)max_chunks * n * 4, 256) +
                        radix_sort_temp_bytes(n) + scan_temp_bytes(n) + 8192;
    char* base = (char*)scratch(ctx, need);
    if (!base) return DM_ERR_NOMEM;
#ifdef DM_BD_CHECK
    DM_HIP(hipMemsetAsync(base, 0x7F, need, s));
#endif
    int32_t* hostv = (int32_t*)pinned(ctx, 2048);  // the size fast_fronts asks for: no realloc
    if (!hostv) return DM_ERR_NOMEM;
    Bump bp{base};
    uint64_t* keys = bp.take<uint64_t>(n);
    uint64_t* ktmp = bp.take<uint64_t>(n);
    int32_t* perm = bp.take<int32_t>(n + 2);
    int32_t* vtmp = bp.take<int32_t>(n + 2);
    int32_t* segin = bp.take<int32_t>(n + 2);
    int32_t* segstart = bp.take<int32_t>(n + 2);
    int32_t* isrep = bp.take<int32_t>(n + 2);
    int32_t* uidx = bp.take<int32_t>(n + 2);
    int32_t* ui = bp.take<int32_t>(n + 2);
    int32_t* small = bp.take<int32_t>(n + 2);  // scalars
    void* rtemp = bp.take<char>(radix_sort_temp_bytes(n));
    void* stemp = bp.take<char>(scan_temp_bytes(n));
    int32_t* utotal = small;
    int32_t* nanflag = small + 2;
    int32_t* ftotal = small + 4;
    int64_t* dtotal = (int64_t*)(small + 8);
    // lexicographic ascending sort of wvalues (ties by index: stable): by
    // objective 0 alone (8 radix passes instead of 8m), then the runs of equal
    // objective 0 that are out of order in the others are sorted in place
    // (lex_bad_kernel, lex_run_sort_kernel); only when such a run is longer than LEX_RUN_CAP (flag
    // read with U below) are the full sort and the grouping redone.  (C5's
    // populations hold near-clones equal in objective 0 and a few ulps apart
    // in the others: the full redo cost 24 radix passes per selection.)
    int32_t* tieflag = small + 6;
    const bool full_lex = ctx->knobs.lex_full;
    // the in-place run sort keys objectives 1..3 (LexRest): up to 4 objectives;
    // with at most 3 (LexRest then holds objectives 0..2) the objective-0 sort
    // orders only the top 32 key bits (4 radix passes instead of 8) and the
    // runs of equal top bits are fixed up the same way
    const bool quick = m > 1 && m <= 4 && !full_lex;
    const bool q32 = quick && m <= 3 && !ctx->knobs.lex_no32;
    int rc;
    auto group = [&](int nlex, int kshift) -> int {
        // the scalars: unique count, NaN flag, front-0 size, tie flag, front-0 individuals
        DM_HIP(hipMemsetAsync(small, 0, 48, s));
        int r = lex_sort_rows(s, wv, m, n, false, keys, ktmp, perm, vtmp, rtemp, nlex, kshift);
        if (r) return r;
        if (nlex < m) {
            zero_i32_kernel<<<g1(n), 256, 0, s>>>(vtmp, n);
            lex_bad_kernel<<<g1(n), 256, 0, s>>>(wv, m, keys, perm, n, vtmp, tieflag, kshift);
            lex_run_sort_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, s>>>(
                wv, m, keys, perm, n, vtmp, tieflag, kshift);
        }
        seg_flag_kernel<<<g1(n), 256, 0, s>>>(wv, m, perm, n, segin, isrep, nanflag);
        if ((r = inclusive_max_scan_i32(s, segin, segstart, n, stemp))) return r;
        return exclusive_scan_i32(s, isrep, uidx, n, utotal, stemp);
    };
    if ((rc = group(quick ? 1 : m, q32 ? 32 : 0))) return rc;
    DM_HIP(hipMemcpyAsync(hostv, utotal, 28, hipMemcpyDeviceToHost, s));
    DM_HIP(hipStreamSynchronize(s));
    // a run longer than LEX_RUN_CAP: the whole-key objective-0 sort, then the
    // full lexicographic sort
    if (q32 && hostv[6]) {
        if ((rc = group(1, 0))) return rc;
        DM_HIP(hipMemcpyAsync(hostv, utotal, 28, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
    }
    if (quick && hostv[6]) {
        if ((rc = group(m, 0))) return rc;
        DM_HIP(hipMemcpyAsync(hostv, utotal, 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
    }
    const int64_t U = hostv[0];
    const bool has_nan = hostv[2] != 0;
    // integer ranks + bitset tables + device-driven peel (dominance.hip);
    // the cross-check paths DM_DOM_LDS / DM_DOM_BALLOT select the fp64 kernels
    const bool fast = m >= 2 && m <= 4 && !has_nan && ctx->dom_path != DM_DOM_LDS &&
                      ctx->dom_path != DM_DOM_BALLOT;
    const int64_t W = (U + 63) / 64;
    const int64_t tiles = (W + PEEL_WORDS - 1) / PEEL_WORDS;
    const double dbytes = (double)U * (double)W * 8.0;
    DM_CHECK_ARG(dbytes < 120e9, "too many distinct fitnesses for the dominance matrix (%lld)",
                 (long long)U);
    double* ufit = bp.take<double>(U * m);
    int32_t* useg = bp.take<int32_t>(U);
    int32_t* gsize = bp.take<int32_t>(U);
    int32_t* count = bp.take<int32_t>(U);
    int32_t* rankU = bp.take<int32_t>(U);
    int32_t* flag = bp.take<int32_t>(U);
    int32_t* fpos = bp.take<int32_t>(U);
    int32_t* lastpos = bp.take<int32_t>(U);
    int32_t* ulist = bp.take<int32_t>(U + 2);  // unique fits in front order
    int32_t* ufs = bp.take<int32_t>(U + 2);    // front starts in ulist
    int32_t* outpos = bp.take<int32_t>(U + 2);
    uint64_t* ukeys = keys;  // the n-sized key buffers are free again
    uint64_t* uktmp = ktmp;
    int32_t* part_dec = bp.take<int32_t>(max_chunks * U);
    int32_t* part_last = bp.take<int32_t>(max_chunks * U);
    void* urtemp = rtemp;
    void* ustemp = stemp;
    if (bp.off > need) {
        set_error("internal workspace overflow");
        return DM_ERR_INVALID;
    }
    uint64_t* D = (uint64_t*)scratch_slot(
        ctx, 1, fast ? (fast_table_peel(ctx, m) ? 256 : (size_t)fast_dom_words(U) * 8) : (size_t)U * W * 8);
    if (!D) return DM_ERR_NOMEM;
    char* fwork = nullptr;  // fast path workspace (dominance.hip)
    if (fast) {
        fwork = (char*)scratch_slot(ctx, 4, fast_dom_bytes(n, U));
#ifdef DM_BD_CHECK
        // diagnostics: poison the fast path's workspace (a read before write
        // then shows up as an out-of-range index in the range checks)
        if (fwork) DM_HIP(hipMemsetAsync(fwork, 0x7F, fast_dom_bytes(n, U), s));
#endif
        if (!fwork) return DM_ERR_NOMEM;
    }

    unique_init_kernel<<<g1(U), 256, 0, s>>>(gsize, count, rankU, U);
    unique_kernel<<<g1(n), 256, 0, s>>>(wv, m, perm, segstart, uidx, n, ui, ufit, useg, gsize);
    if (fast) {
        if ((rc = fast_dom_build(ctx, wv, m, n, perm, segin, uidx, ufit, U, D, count,
                                 fwork)))
            return rc;
    } else if (m >= 2 && m <= 4 && ctx->dom_path != DM_DOM_LDS) {
        const int64_t ngroups = (W + DB_WPW - 1) / DB_WPW;
        int32_t* cpart = (int32_t*)scratch_slot(ctx, 4, (size_t)ngroups * U * 4);
        if (!cpart) return DM_ERR_NOMEM;
        if (m == 2)
            launch_dom_ballot<2>(ufit, U, W, D, cpart, s);
        else if (m == 3)
            launch_dom_ballot<3>(ufit, U, W, D, cpart, s);
        else
            launch_dom_ballot<4>(ufit, U, W, D, cpart, s);
        DM_LAUNCH_CHECK();
        dom_count_reduce_kernel<<<g1(U), 256, 0, s>>>(cpart, ngroups, U, count);
    } else {
        dim3 grid((unsigned)((W + DT_WORDS - 1) / DT_WORDS), (unsigned)((U + DT_ROWS - 1) / DT_ROWS));
        const size_t lds = (size_t)m * 64 * DT_WORDS * sizeof(double);
        dom_build_kernel<<<grid, 256, lds, s>>>(ufit, m, U, W, D, count);
    }
    // front 0
    flag_zero_count_kernel<<<g1(U), 256, 0, s>>>(count, U, flag);
    if ((rc = exclusive_scan_i32(s, flag, fpos, U, ftotal, ustemp))) return rc;
    compact_kernel<<<g1(U), 256, 0, s>>>(flag, fpos, U, ulist, nullptr, nullptr, rankU, 0);
    // dtotal is zero (the grouping's scalar memset)
    const int64_t N = std::min<int64_t>(n, k);
    std::vector<int32_t> ufront{0};
    int64_t F = 0, sorted_inds = 0;
    int64_t ustart = 0;  // start of the current front in ulist
    int32_t rnk = 0;
    int64_t* hostd = (int64_t*)(hostv + 8);
    const bool device_fronts = fast && !first_only;
    int64_t last_inds = 0, max_inds = 0;
    if (device_fronts) {
        // front 0's size and individual count stay on the device: the peel's
        // first kernel reads them (no host round trip)
        sum_gsize_dev_kernel<<<g1(U), 256, 0, s>>>(ulist, ftotal, gsize, dtotal);
        int64_t total = 0;
        // ufs doubles as the device front-start array
        if ((rc = fast_fronts(ctx, D, m, n, U, ftotal, dtotal, N, gsize, ulist, rankU, count, ufs,
                              fwork, ufront, &total, &last_inds, &max_inds)))
            return rc;
        sorted_inds = total;
    } else {
        DM_HIP(hipMemcpyAsync(hostv, ftotal, 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        F = hostv[0];
        sum_gsize_kernel<<<g1(F), 256, 0, s>>>(ulist, F, gsize, dtotal);
        DM_HIP(hipMemcpyAsync(hostd, dtotal, 8, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        sorted_inds = hostd[0];
        last_inds = hostd[0];
        max_inds = last_inds;
        ufront.push_back((int32_t)F);
    }
    while (!fast && !first_only && sorted_inds < N && ustart + F < U && F > 0) {
        // peel front `rnk` (ulist[ustart, ustart+F)) -> front rnk+1
        const int64_t waves_target = 8192;
        int64_t nchunks = std::max<int64_t>(1, std::min<int64_t>(max_chunks, waves_target / tiles));
        nchunks = std::min<int64_t>(nchunks, (F + 63) / 64);
        int64_t chunk = (F + nchunks - 1) / nchunks;
        chunk = (chunk + 63) / 64 * 64;
        nchunks = (F + chunk - 1) / chunk;
        const int64_t waves = tiles * nchunks;
        peel_kernel<<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(D, W, U, ulist + ustart, F, chunk,
                                                                tiles, nchunks, part_dec,
                                                                part_last);
        peel_combine_kernel<<<g1(U), 256, 0, s>>>(part_dec, part_last, nchunks, U, count, rankU,
                                                  flag, lastpos);
        if ((rc = exclusive_scan_i32(s, flag, fpos, U, ftotal, ustemp))) return rc;
        const int64_t nstart = ustart + F;
        compact_kernel<<<g1(U), 256, 0, s>>>(flag, fpos, U, ulist + nstart, lastpos, ukeys, rankU,
                                             rnk + 1);
        DM_HIP(hipMemcpyAsync(hostv, ftotal, 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        const int64_t F2 = hostv[0];
        if (F2 == 0) break;
        // stable order by position of the releasing dominator (candidates are in U order)
        int bits = 8;
        while (bits < 32 && (1ll << bits) <= F) bits += 8;
        if ((rc = radix_sort_pairs(s, ukeys, ulist + nstart, uktmp, vtmp, F2, 0, bits, urtemp)))
            return rc;
        DM_HIP(hipMemsetAsync(dtotal, 0, 8, s));
        sum_gsize_kernel<<<g1(F2), 256, 0, s>>>(ulist + nstart, F2, gsize, dtotal);
        DM_HIP(hipMemcpyAsync(hostd, dtotal, 8, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        sorted_inds += hostd[0];
        last_inds = hostd[0];
        max_inds = std::max(max_inds, last_inds);
        ustart = nstart;
        F = F2;
        ++rnk;
        ufront.push_back((int32_t)(ustart + F));
    }
    const int32_t nfronts = (int32_t)ufront.size() - 1;
    const int64_t T = ufront.back();  // unique fits in emitted fronts
    // expansion (the device peel already wrote ufs)
    if (!device_fronts)
        DM_HIP(hipMemcpyAsync(ufs, ufront.data(), ufront.size() * 4, hipMemcpyHostToDevice, s));
    member_sizes_kernel<<<g1(T), 256, 0, s>>>(ulist, T, gsize, flag);
    if ((rc = exclusive_scan_i32(s, flag, outpos, T, ftotal, ustemp))) return rc;
    expand_kernel<<<g1(T), 256, 0, s>>>(ulist, T, outpos, useg, gsize, perm, order);
    front_start_kernel<<<g1(nfronts + 1), 256, 0, s>>>(ufs, nfronts, outpos, T,
                                                        (int32_t)sorted_inds, front_start);
    if (rank) {
        // individuals outside the emitted fronts keep rankU = -1
        ind_rank_kernel<<<g1(n), 256, 0, s>>>(ui, rankU, n, rank);
    }
    res->U = U;
    res->rank_keys = false;
    if (rank_keys && fast) {
        if ((rc = fast_rank_keys(ctx, fwork, n, U, m, ui, order, sorted_inds, rank_keys)))
            return rc;
        res->rank_keys = true;
    }
    if (!device_fronts) DM_HIP(hipStreamSynchronize(s));  // ufront host vector goes out of scope
    res->nsorted = sorted_inds;
    res->nfronts = nfronts;
    res->last_inds = last_inds;
    res->max_inds = max_inds;
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// ---------------------------------------------------------------------------
// crowding distance
// ---------------------------------------------------------------------------
struct Weights {
    double w[DM_MAX_OBJ];
};
__global__ void crowd_key_kernel(const double* wv, int m, int obj, Weights wt, const int32_t* order,
                                 const int32_t* pos, uint64_t* keys, int64_t T) {
    GRID_LOOP(j, T) {
        const int32_t ind = order[pos[j]];
        keys[j] = ordered_key(wv[(int64_t)ind * m + obj] / wt.w[obj]);
    }
}
__global__ void fid_key_kernel(const int32_t* fid, const int32_t* pos, uint64_t* keys, int64_t T) {
    GRID_LOOP(j, T) keys[j] = (uint64_t)(uint32_t)fid[pos[j]];
}
// front ids, crowding zeroed and the identity order in one pass
__global__ void crowd_setup_kernel(const int32_t* fstart, int32_t nf, const int32_t* order,
                                   int64_t T, int32_t* fid, double* crowd, int32_t* pos) {
    GRID_LOOP(j, T) {
        int lo = 0, hi = nf - 1;  // last f with fstart[f] <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (fstart[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        fid[j] = lo;
        crowd[order[j]] = 0.0;
        pos[j] = (int32_t)j;
    }
}
__global__ void crowd_update_kernel(const double* wv, int m, int obj, Weights wt,
                                    const int32_t* order, const int32_t* spos,
                                    const int32_t* fid_of_pos, const int32_t* fstart, int64_t T,
                                    double* crowd) {
    GRID_LOOP(j, T) {
        const int32_t f = fid_of_pos[j];  // fronts occupy the same ranges after the sort
        const int64_t first = fstart[f], last = fstart[f + 1] - 1;
        const int32_t ind = order[spos[j]];
        const double w = wt.w[obj];
        if (j == first || j == last) {
            crowd[ind] = INFINITY;  // distances[crowd[0][1]] = inf   (emo.py:134-135)
            continue;
        }
        const double vmin = wv[(int64_t)order[spos[first]] * m + obj] / w;
        const double vmax = wv[(int64_t)order[spos[last]] * m + obj] / w;
        if (vmax == vmin) continue;  // emo.py:136-137
        const double norm = (double)m * (vmax - vmin);
        const double nxt = wv[(int64_t)order[spos[j + 1]] * m + obj] / w;
        const double prv = wv[(int64_t)order[spos[j - 1]] * m + obj] / w;
        crowd[ind] = crowd[ind] + (nxt - prv) / norm;
    }
}

// (front, rank) key of objective obj: ascending in the unweighted value
// (values = wvalues / weights: a negative weight reverses the rank order)
__global__ void crowd_rank_key_kernel(const int32_t* rk, int64_t U, bool neg, const int32_t* fid,
                                      const int32_t* pos, int rbits, uint64_t* keys, int64_t T) {
    GRID_LOOP(j, T) {
        const int32_t p = pos[j];
        const uint32_t r = (uint32_t)(neg ? (int32_t)(U - 1) - rk[p] : rk[p]);
        keys[j] = fid ? ((uint64_t)(uint32_t)fid[p] << rbits) | r : (uint64_t)r;  // fid null: rank alone
    }
}

// rk (nullable): per-objective integer ranks of the T individuals (m x T,
// sort_nondominated_impl's rank_keys) over U unique fitnesses.
// max_front: individuals of the largest front, when known -- at most
// LDS_SORT_CAP32 and each objective's order is ONE segmented LDS sort (a
// workgroup per front, by rank alone: a front never leaves its range)
// instead of a 24-bit (front, rank) one-sweep radix sort of all T.
static int crowding_impl(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                         const int32_t* order, const int32_t* fstart_dev, int32_t nfronts,
                         int64_t T, double* crowd, const int32_t* rk = nullptr, int64_t U = 0,
                         int64_t max_front = INT64_MAX) {
    hipStream_t s = ctx->stream;
    const int m = pop->nobj;
    if (T <= 0 || nfronts <= 0) return DM_OK;
    Weights wt{};
    for (int o = 0; o < m; ++o) wt.w[o] = weights[o];
    char* base = (char*)scratch(ctx, 2 * align_up((size_t)T * 8, 256) +
                                         4 * align_up((size_t)T * 4, 256) +
                                         radix_sort_temp_bytes(T) + 4096);
    if (!base) return DM_ERR_NOMEM;
    Bump bp{base};
    uint64_t* keys = bp.take<uint64_t>(T);
    uint64_t* ktmp = bp.take<uint64_t>(T);
    int32_t* pos = bp.take<int32_t>(T);
    int32_t* vtmp = bp.take<int32_t>(T);
    int32_t* fid = bp.take<int32_t>(T);
    int32_t* fpos = bp.take<int32_t>(T);
    void* rtemp = bp.take<char>(radix_sort_temp_bytes(T));
    crowd_setup_kernel<<<g1(T), 256, 0, s>>>(fstart_dev, nfronts, order, T, fid, crowd, pos);
    int fbits = 8;
    while (fbits < 32 && (1ll << fbits) <= nfronts) fbits += 8;
    // The reference sorts one `crowd` list by objective 0, then 1, ...
    // (emo.py:131-133, stable): the order for objective i is the previous
    // one stably sorted by v_i, i.e. lexicographic in (v_i, ..., v_0,
    // position) — one 64-bit sort per objective carried over; the grouping
    // by front (a stable sort by front id) works on a copy.
    bool zero_w = false;
    for (int o = 0; o < m; ++o) zero_w = zero_w || weights[o] == 0.0;
    if (rk && !zero_w) {
        // sorted by (front, rank_i) carrying the previous objective's order:
        // within a front lexicographic in (v_i, ..., v_0, position), fronts
        // grouped — one sort of rbits + fbits bits per objective
        int rbits = 1;
        while (rbits < 31 && (1ll << rbits) < U) ++rbits;
        int kbits = rbits;
        while (kbits < 64 && (1ll << (kbits - rbits)) <= nfronts) ++kbits;
        if (max_front <= (rbits <= 32 ? LDS_SORT_CAP32 : LDS_SORT_CAP)) {
            for (int i = 0; i < m; ++i) {
                crowd_rank_key_kernel<<<g1(T), 256, 0, s>>>(rk + (int64_t)i * T, U,
                                                            weights[i] < 0.0, nullptr, pos, rbits,
                                                            keys, T);
                int rc = seg_sort_pairs_small(s, keys, pos, fstart_dev, nfronts, 0, rbits, ktmp,
                                              vtmp);
                if (rc) return rc;
                crowd_update_kernel<<<g1(T), 256, 0, s>>>(pop->wvalues, m, i, wt, order, pos, fid,
                                                          fstart_dev, T, crowd);
            }
            DM_LAUNCH_CHECK();
            return DM_OK;
        }
        for (int i = 0; i < m; ++i) {
            crowd_rank_key_kernel<<<g1(T), 256, 0, s>>>(rk + (int64_t)i * T, U, weights[i] < 0.0,
                                                        fid, pos, rbits, keys, T);
            // an odd pass count leaves the pairs in the tmp buffers: swap
            // the roles instead of copying back (the keys are rebuilt per
            // objective, only pos carries over)
            bool in_tmp = false;
            int rc = radix_sort_pairs_any(s, keys, pos, ktmp, vtmp, T, 0, kbits, rtemp, &in_tmp);
            if (rc) return rc;
            if (in_tmp) {
                std::swap(keys, ktmp);
                std::swap(pos, vtmp);
            }
            crowd_update_kernel<<<g1(T), 256, 0, s>>>(pop->wvalues, m, i, wt, order, pos, fid,
                                                      fstart_dev, T, crowd);
        }
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    for (int i = 0; i < m; ++i) {
        crowd_key_kernel<<<g1(T), 256, 0, s>>>(pop->wvalues, m, i, wt, order, pos, keys, T);
        int rc = radix_sort_pairs(s, keys, pos, ktmp, vtmp, T, 0, 64, rtemp);
        if (rc) return rc;
        DM_HIP(hipMemcpyAsync(fpos, pos, (size_t)T * 4, hipMemcpyDeviceToDevice, s));
        fid_key_kernel<<<g1(T), 256, 0, s>>>(fid, fpos, keys, T);
        rc = radix_sort_pairs(s, keys, fpos, ktmp, vtmp, T, 0, fbits, rtemp);
        if (rc) return rc;
        crowd_update_kernel<<<g1(T), 256, 0, s>>>(pop->wvalues, m, i, wt, order, fpos, fid,
                                                  fstart_dev, T, crowd);
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

__global__ void crowd_desc_key_kernel(const double* crowd, const int32_t* vals, uint64_t* keys,
                                      int64_t T) {
    GRID_LOOP(j, T) keys[j] = ~ordered_key(crowd[vals[j]]);
}

// selNSGA2's choice from sorted fronts (emo.py:38-48): the fronts before the
// last one whole, then the last front (its L individuals at the end of
// order[0, T)) by decreasing crowding distance, stable (sorted(...,
// reverse=True) keeps equal distances in front order).
static int take_chosen(dm_ctx* ctx, const int32_t* order, const SortResult& r, int64_t k,
                       const double* crowd, int32_t* out_idx) {
    const int64_t chosen = r.nfronts > 0 ? r.nsorted - r.last_inds : 0;
    if (chosen > 0)
        DM_HIP(hipMemcpyAsync(out_idx, order, (size_t)std::min(chosen, k) * 4,
                              hipMemcpyDeviceToDevice, ctx->stream));
    const int64_t rem = k - chosen;
    if (rem > 0 && r.nfronts > 0) {
        const int64_t L = r.last_inds;  // last front size
        char* base = (char*)scratch(ctx, 2 * align_up((size_t)L * 8, 256) +
                                             2 * align_up((size_t)L * 4, 256) +
                                             radix_sort_temp_bytes(L) + 4096);
        if (!base) return DM_ERR_NOMEM;
        Bump bp{base};
        uint64_t* keys = bp.take<uint64_t>(L);
        uint64_t* ktmp = bp.take<uint64_t>(L);
        int32_t* vals = bp.take<int32_t>(L);
        int32_t* vtmp = bp.take<int32_t>(L);
        void* rtemp = bp.take<char>(radix_sort_temp_bytes(L));
        DM_HIP(hipMemcpyAsync(vals, order + chosen, (size_t)L * 4, hipMemcpyDeviceToDevice,
                              ctx->stream));
        crowd_desc_key_kernel<<<g1(L), 256, 0, ctx->stream>>>(crowd, vals, keys, L);
        int rc = radix_sort_pairs(ctx->stream, keys, vals, ktmp, vtmp, L, 0, 64, rtemp);
        if (rc) return rc;
        DM_HIP(hipMemcpyAsync(out_idx + chosen, vals, (size_t)std::min(rem, L) * 4,
                              hipMemcpyDeviceToDevice, ctx->stream));
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// ---------------------------------------------------------------------------
// sortLogNondominated order (emo.py:246-276).  Fortin's sort computes the
// same Pareto ranks as the standard one, so the ranks come
// from sort_nondominated_impl; the log version's fronts list the unique
// fitnesses in ``fitnesses.sort(reverse=True)`` order (descending
// lexicographic wvalues, emo.py:257) and each one's individuals in population
// order (``unique_fits[...].append``, emo.py:249-250): a stable descending
// lexicographic sort of the rows (ties = equal fitnesses keep index order),
// then a stable sort by rank (rows outside the emitted fronts last).
// ---------------------------------------------------------------------------
__global__ void log_rank_key_kernel(const int32_t* rank, const int32_t* perm, int64_t n,
                                    uint64_t unsorted, uint64_t* keys) {
    GRID_LOOP(j, n) {
        const int32_t r = rank[perm[j]];
        keys[j] = r < 0 ? unsorted : (uint64_t)(uint32_t)r;
    }
}
__global__ void log_front_start_kernel(const uint64_t* keys, int64_t T, int32_t nf,
                                       int32_t* fstart) {
    GRID_LOOP(j, T) {
        if (j == 0 || keys[j] != keys[j - 1]) fstart[keys[j]] = (int32_t)j;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) fstart[nf] = (int32_t)T;
}

// order [n] / fstart [n + 1]: device outputs, not in scratch slots 0, 1, 3, 4.
static int log_sort_impl(dm_ctx* ctx, const dm_pop* pop, int64_t k, bool first_only,
                         int32_t* order, int32_t* fstart, SortResult* res) {
    hipStream_t s = ctx->stream;
    const int64_t n = pop->n;
    int32_t* w = (int32_t*)scratch_slot(ctx, 3, (size_t)(3 * n + 4) * 4);
    if (!w) return DM_ERR_NOMEM;
    int32_t* rank = w;
    int32_t* perm = w + n;
    int32_t* std_fstart = w + 2 * n;  // the standard front starts (unused)
    int rc = sort_nondominated_impl(ctx, pop, k, first_only, order, std_fstart, rank, res);
    if (rc) return rc;
    if ((rc = sort_by_fitness(ctx, pop->wvalues, pop->nobj, n, true, perm))) return rc;
    const size_t kb = align_up((size_t)n * 8, 256), vb = align_up((size_t)n * 4, 256);
    char* t = (char*)scratch(ctx, 2 * kb + vb + radix_sort_temp_bytes(n));
    if (!t) return DM_ERR_NOMEM;
    uint64_t* keys = (uint64_t*)t;
    uint64_t* ktmp = (uint64_t*)(t + kb);
    int32_t* vtmp = (int32_t*)(t + 2 * kb);
    void* rtemp = t + 2 * kb + vb;
    int bits = 8;
    while (bits < 32 && (1ll << bits) <= (int64_t)res->nfronts) bits += 8;
    log_rank_key_kernel<<<g1(n), 256, 0, s>>>(rank, perm, n, (1ull << bits) - 1, keys);
    if ((rc = radix_sort_pairs(s, keys, perm, ktmp, vtmp, n, 0, bits, rtemp))) return rc;
    const int64_t T = res->nsorted;
    if (T > 0) DM_HIP(hipMemcpyAsync(order, perm, (size_t)T * 4, hipMemcpyDeviceToDevice, s));
    log_front_start_kernel<<<g1(std::max<int64_t>(T, 1)), 256, 0, s>>>(keys, T, res->nfronts,
                                                                      fstart);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

__global__ void gather_f64_kernel(const double* src, const int32_t* idx, int64_t n, double* dst) {
    GRID_LOOP(i, n) dst[i] = src[idx ? idx[i] : i];
}

}  // namespace dm

using namespace dm;

extern "C" int dm_sort_nondominated(dm_ctx* ctx, const dm_pop* pop, int64_t k,
                                    int32_t first_front_only, int32_t* order,
                                    int32_t* front_start, int32_t* rank, int64_t* nsorted,
                                    int32_t* nfronts) {
    DM_CHECK_ARG(ctx && order && front_start && nsorted && nfronts, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    DM_CHECK_ARG(pop->n < (1ll << 31), "population too large");
    SortResult r;
    rc = sort_nondominated_impl(ctx, pop, k, first_front_only != 0, order, front_start, rank, &r);
    if (rc) return rc;
    *nsorted = r.nsorted;
    *nfronts = r.nfronts;
    return DM_OK;
}

extern "C" int dm_sort_log_nondominated(dm_ctx* ctx, const dm_pop* pop, int64_t k,
                                        int32_t first_front_only, int32_t* order,
                                        int32_t* front_start, int64_t* nsorted,
                                        int32_t* nfronts) {
    DM_CHECK_ARG(ctx && order && front_start && nsorted && nfronts, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    DM_CHECK_ARG(pop->n < (1ll << 31), "population too large");
    *nsorted = 0;
    *nfronts = 0;
    if (pop->n == 0 || k == 0) return DM_OK;
    SortResult r;
    rc = log_sort_impl(ctx, pop, k, first_front_only != 0, order, front_start, &r);
    if (rc) return rc;
    DM_HIP(hipStreamSynchronize(ctx->stream));
    *nsorted = r.nsorted;
    *nfronts = r.nfronts;
    return DM_OK;
}

extern "C" int dm_crowding_dist(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                                const int32_t* order, const int32_t* front_start, int32_t nfronts,
                                double* crowd) {
    DM_CHECK_ARG(ctx && pop && weights && crowd, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    if (nfronts <= 0) return DM_OK;
    DM_CHECK_ARG(order && front_start, "null order/front_start");
    int32_t last = 0;
    DM_HIP(hipMemcpyAsync(&last, front_start + nfronts, 4, hipMemcpyDeviceToHost, ctx->stream));
    DM_HIP(hipStreamSynchronize(ctx->stream));
    return crowding_impl(ctx, pop, weights, order, front_start, nfronts, last, crowd);
}

extern "C" int dm_sel_nsga2(dm_ctx* ctx, const dm_pop* pop, const double* weights, int64_t k,
                            int32_t* out_idx, double* crowd) {
    DM_CHECK_ARG(ctx && pop && weights && out_idx && crowd, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    const int64_t n = pop->n;
    if (n == 0 || k == 0) return DM_OK;
    // order / front starts / integer crowding keys outlive the sort's slot-0
    // workspace: slot 2
    const int m = pop->nobj;
    int32_t* order = (int32_t*)scratch_slot(ctx, 2, (size_t)(2 * n + 2 + (int64_t)m * n) * 4);
    if (!order) return DM_ERR_NOMEM;
    int32_t* fstart = order + n;
    int32_t* rkeys = order + 2 * n + 2;
    SortResult r;
    rc = sort_nondominated_impl(ctx, pop, k, false, order, fstart, nullptr, &r, rkeys);
    if (rc) return rc;
    rc = crowding_impl(ctx, pop, weights, order, fstart, r.nfronts, r.nsorted, crowd,
                       r.rank_keys ? rkeys : nullptr, r.U, r.max_inds);
    if (rc) return rc;
    return take_chosen(ctx, order, r, k, crowd, out_idx);
}

extern "C" int dm_sel_nsga2_log(dm_ctx* ctx, const dm_pop* pop, const double* weights, int64_t k,
                                int32_t* out_idx, double* crowd) {
    DM_CHECK_ARG(ctx && pop && weights && out_idx && crowd, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    DM_CHECK_ARG(pop->n < (1ll << 31), "population too large");
    const int64_t n = pop->n;
    if (n == 0 || k == 0) return DM_OK;
    int32_t* order = (int32_t*)scratch_slot(ctx, 2, (size_t)(2 * n + 2) * 4);
    if (!order) return DM_ERR_NOMEM;
    int32_t* fstart = order + n;
    SortResult r;
    if ((rc = log_sort_impl(ctx, pop, k, false, order, fstart, &r))) return rc;
    // crowding on every front in its log order (emo.py:41-42)
    rc = crowding_impl(ctx, pop, weights, order, fstart, r.nfronts, r.nsorted, crowd);
    if (rc) return rc;
    return take_chosen(ctx, order, r, k, crowd, out_idx);
}

extern "C" int dm_gather_f64(dm_ctx* ctx, const double* src, const int32_t* idx, int64_t n,
                             double* dst) {
    DM_CHECK_ARG(ctx && (n == 0 || (src && dst)), "null argument");
    DM_CHECK_ARG(n >= 0, "negative n");
    if (n == 0) return DM_OK;
    gather_f64_kernel<<<g1(n), 256, 0, ctx->stream>>>(src, idx, n, dst);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// ---------------------------------------------------------------------------
// selTournamentDCD (emo.py:145-195)
// ---------------------------------------------------------------------------
namespace dm {

// Fitness.dominates on wvalues (base.py:209-224): an objective with a NaN side
// compares equal.
__device__ __forceinline__ bool dominates_wv(const double* a, const double* b, int m) {
    bool not_equal = false;
    for (int o = 0; o < m; ++o) {
        if (a[o] > b[o])
            not_equal = true;
        else if (a[o] < b[o])
            return false;
    }
    return not_equal;
}

// random.sample(individuals, len(individuals)) twice (emo.py:186-187): the
// permutations are the orders of 2 n Philox keys (stage ST_DCD, item = i, sub
// = 4 + q), sorted as ONE batched radix sort of two segments (stable: a tie of
// two 64-bit keys keeps index order).  Uniform random keys give uniformly
// distributed permutations, as random.sample's are.  (Round 5 used a keyed
// 4-round Feistel network cycle-walked into [0, n) instead -- one pass, but a
// simulation of it with ideal round functions (tools_gpu/dcd_perm_sim.py) puts
// the position-of-i histogram 11-31 % off uniform at n = 5..33 (chi-square p
// < 1e-12): not random.sample's distribution; removed in round 6.)
__global__ void dcd_keys_kernel(Rng rng, int64_t n, uint64_t* keys, int32_t* vals) {
    GRID_LOOP(t, 2 * n) {
        const uint32_t q = t >= n ? 1u : 0u;
        const int64_t i = t - (int64_t)q * n;
        const u32x4 w = rng(ST_DCD, (uint32_t)i, 4u + q);
        keys[t] = ((uint64_t)w.x << 32) | w.y;
        vals[t] = (int32_t)i;
    }
}

// Slot j of the output: tournament j%4 of group j/4 — (P1[i], P1[i+1]),
// (P1[i+2], P1[i+3]), (P2[i], P2[i+1]), (P2[i+2], P2[i+3]) with i = 4*(j/4)
// (emo.py:188-192); dominance, then the larger crowding distance, then
// random() <= 0.5 keeps the first (emo.py:170-183).
__global__ void dcd_kernel(const double* wv, int m, const double* crowd, const int32_t* p1,
                           const int32_t* p2, int64_t k4, Rng rng, int mode, uint8_t* coin,
                           int32_t* out) {
    GRID_LOOP(j, k4) {
        const int64_t i = (j >> 2) << 2;
        const int r = (int)(j & 3);
        const int32_t* P = r < 2 ? p1 : p2;
        const int64_t o = i + 2 * (r & 1);
        const int32_t a = P[o], b = P[o + 1];
        int32_t res;
        if (dominates_wv(wv + (int64_t)a * m, wv + (int64_t)b * m, m)) {
            res = a;
        } else if (dominates_wv(wv + (int64_t)b * m, wv + (int64_t)a * m, m)) {
            res = b;
        } else if (crowd[a] < crowd[b]) {
            res = b;
        } else if (crowd[a] > crowd[b]) {
            res = a;
        } else {
            bool first;
            if (mode == DM_RNG_INJECT) {
                first = coin[j] != 0;
            } else {
                const u32x4 w = rng(ST_DCD, (uint32_t)j, 2u);
                first = u01_53(w.x, w.y) <= 0.5;
                if (mode == DM_RNG_DUMP) coin[j] = first ? 1 : 0;
            }
            res = first ? a : b;
        }
        out[j] = res;
    }
}

}  // namespace dm

extern "C" int dm_sel_tournament_dcd(dm_ctx* ctx, const dm_pop* pop, const double* crowd,
                                     int64_t k, dm_rng rng, int32_t mode, int32_t* perm1,
                                     int32_t* perm2, uint8_t* coin, int32_t* out_idx) {
    using namespace dm;
    DM_CHECK_ARG(ctx && crowd && out_idx, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    const int64_t n = pop->n;
    DM_CHECK_ARG(k >= 0, "bad k");
    DM_CHECK_ARG(n < (1ll << 31), "population too large");
    if (k > n) {
        set_error("selTournamentDCD: k must be less than or equal to individuals length");
        return DM_ERR_INVALID;
    }
    if (k == n && k % 4 != 0) {
        set_error("selTournamentDCD: k must be divisible by four if k == len(individuals)");
        return DM_ERR_INVALID;
    }
    const int64_t k4 = (k + 3) / 4 * 4;
    if (k4 > n) {  // individuals_1[i+3] past the end (emo.py:188-192)
        set_error("list index out of range");
        return DM_ERR_INDEX;
    }
    if (mode == DM_RNG_INJECT) {
        DM_CHECK_ARG(perm1 && perm2 && coin, "decisions perm1 / perm2 / coin required");
    } else if (mode == DM_RNG_DUMP) {
        DM_CHECK_ARG(perm1 && perm2 && coin, "dump buffers perm1 / perm2 / coin required");
    }
    if (k == 0) return DM_OK;
    hipStream_t s = ctx->stream;
    if (mode != DM_RNG_INJECT) {
        // random.sample(individuals, len(individuals)) twice: the two segments'
        // key orders (dcd_keys_kernel + one batched radix sort)
        const size_t kb = align_up((size_t)2 * n * 8, 256), vb = align_up((size_t)2 * n * 4, 256);
        char* w = (char*)scratch(ctx, 2 * kb + 2 * vb + radix_sort_batched_temp_bytes(2, n));
        if (!w) return DM_ERR_NOMEM;
        uint64_t* keys = (uint64_t*)w;
        uint64_t* ktmp = (uint64_t*)(w + kb);
        int32_t* vals = (int32_t*)(w + 2 * kb);
        int32_t* vtmp = (int32_t*)(w + 2 * kb + vb);
        dcd_keys_kernel<<<g1(2 * n), 256, 0, s>>>(Rng(rng), n, keys, vals);
        bool in_tmp = false;
        int rc = radix_sort_pairs_batched(s, keys, vals, ktmp, vtmp, 2, n, 0, 64, w + 2 * kb + 2 * vb,
                                          &in_tmp);
        if (rc) return rc;
        const int32_t* sorted = in_tmp ? vtmp : vals;
        if (perm1 && perm2) {  // dump mode: the caller's buffers
            DM_HIP(hipMemcpyAsync(perm1, sorted, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
            DM_HIP(hipMemcpyAsync(perm2, sorted + n, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        } else {
            perm1 = const_cast<int32_t*>(sorted);
            perm2 = const_cast<int32_t*>(sorted + n);
        }
    }
    dcd_kernel<<<g1(k4), 256, 0, s>>>(pop->wvalues, pop->nobj, crowd, perm1, perm2, k4, Rng(rng),
                                      mode, coin, out_idx);
    DM_LAUNCH_CHECK();
    return DM_OK;
}
