// dominance.hip — fast path of sortNondominated (deap/tools/emo.py:53-117)
// for 2..4 objectives and NaN-free fitnesses: the unique fitnesses' dominance
// relation over integer ranks, each unordered pair of 64-blocks computed once,
// and a front-peeling loop driven by the device.
//
// 1. Ranks.  Fitness.dominates (base.py:209-224) only asks, per objective,
//    whether x > y, x < y or neither; replacing every objective value by its
//    dense rank among the U unique values (-0.0 == 0.0, as Python compares)
//    preserves all three answers, so the O(M U^2) pass compares int32 ranks
//    (full-rate VALU compares) instead of fp64 values.  A NaN compares neither
//    way with anything and has no rank: populations holding one take the fp64
//    kernels of nsga2.hip.
// 2. Dominance.  A wave owns SD_WPW 64-v blocks (ranks in VGPRs, lane = v) and
//    sweeps the u rows of the blocks I <= J below them (ranks by scalar loads,
//    u wave-uniform).  One pair of compare masks per (u, 64 v) gives both
//    directions: D[u][J] = ANY(x > y) & ~ANY(x < y) is parked in lane u%64
//    (v_writelane), and "v dominates u" is shifted lane-locally into the
//    transposed word D[v][I] — the lower triangle of the matrix comes from the
//    same compares as the upper one.  Dominator counts accumulate as int16
//    partials per (v-group, u) and per (u-chunk, v), reduced afterwards.
//    D is stored in 64 x 8-word tiles (tile (I, G): rows 64I..64I+63, words
//    8G..8G+7, 64 B per row): a wave's direct stores (64 rows x 32 B) and its
//    transposed stores (64 rows x 64 B, after 8 u-blocks) are contiguous, and
//    a row segment read by the peel is one 64-B line.
// 3. Fronts.  Front 0 = count 0 in U order (nsga2.hip).  Then per front a
//    peel kernel transposes 64 x 64 bit blocks of the members' rows and
//    decrements the dominator counts atomically; the wave whose decrement
//    reaches zero appends v to the next front's candidates and every wave
//    raises v's (front, last releasing position) with a 64-bit atomicMax.
//    One workgroup then orders the candidates by (last releasing position,
//    U index) — the order the reference's peel loop appends them in
//    (emo.py:106-115) — with a bitonic sort in LDS, writes
//    the front, its ranks and its individual count, and decides termination
//    on the device.  The host only checks a status word every few fronts.
#include "sort.hpp"

namespace dm {

#define DGRID_LOOP(i, n)                                                         \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
         i += (int64_t)gridDim.x * blockDim.x)

static dim3 dg1(int64_t n) {
    return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65535)));
}

// ---------------------------------------------------------------------------
// 1. dense ranks per objective: R[u] = int4 {rank_0, .., rank_{m-1}, pad}
// ---------------------------------------------------------------------------
__global__ void rank_key_kernel(const double* ufit, int m, int o, int64_t U, uint64_t* keys,
                                int32_t* vals) {
    DGRID_LOOP(u, U) {
        keys[u] = ordered_key(ufit[u * m + o]);
        vals[u] = (int32_t)u;
    }
}
__global__ void rank_flag_kernel(const uint64_t* keys, int64_t U, int32_t* flag) {
    DGRID_LOOP(j, U) flag[j] = (j > 0 && keys[j] != keys[j - 1]) ? 1 : 0;
}
__global__ void rank_scatter_kernel(const int32_t* vals, const int32_t* excl, const int32_t* flag,
                                    int64_t U, int o, int32_t* R4) {
    DGRID_LOOP(j, U) R4[(int64_t)vals[j] * 4 + o] = excl[j] + flag[j];
}

// ---------------------------------------------------------------------------
// 2. symmetric dominance over ranks
// ---------------------------------------------------------------------------
constexpr int SD_WPW = 4;     // 64-v blocks per wave (a v-group)
constexpr int SD_CHUNK = 16;  // u-blocks per task
#ifndef DM_SD_TG
#define DM_SD_TG 4
#endif
constexpr int SD_TG = DM_SD_TG;  // u-blocks per transposed store (8: one 64-B row segment)
static_assert(SD_TG == 4 || SD_TG == 8, "transposed store group");


// word w of row u in the tiled layout (NG = 8-word groups per row)
__host__ __device__ __forceinline__ int64_t tword(int64_t u, int64_t w, int64_t NG) {
    return ((((u >> 6) * NG + (w >> 3)) << 6) + (u & 63)) * 8 + (w & 7);
}

// tasks are (h, c, g%2) with v-groups g = 2h, 2h+1 and u-chunks c <= h/2:
// S(h) = sum_{h' < h} (h'/2 + 1) = (q + r)(q + 1) for h = 2q + r
__device__ __forceinline__ int64_t sd_tasks_before(int64_t h) {
    const int64_t q = h >> 1, r = h & 1;
    return (q + r) * (q + 1);
}
int64_t sd_task_count(int64_t ngroups) {
    const int64_t nh = (ngroups + 1) / 2;
    const int64_t q = nh >> 1, r = nh & 1;
    return 2 * (q + r) * (q + 1);
}

typedef __attribute__((address_space(4))) const int32_t c4_i32;

// min / max over the M rank differences d_o = y_o - x_o: some x_o > y_o iff
// min < 0, some x_o < y_o iff max > 0 (ranks < 2^31: no overflow)
template <int M>
__device__ __forceinline__ void diff_minmax(const int32_t (&x)[M], const int32_t (&y)[M],
                                            int32_t& mn, int32_t& mx) {
    int32_t d[M];
#pragma unroll
    for (int o = 0; o < M; ++o) d[o] = y[o] - x[o];
    mn = d[0];
    mx = d[0];
#pragma unroll
    for (int o = 1; o < M; ++o) {
        mn = min(mn, d[o]);
        mx = max(mx, d[o]);
    }
}

// t + t + (bit `lane` of mask): one v_addc_co_u32 with the wave mask as the
// carry-in (lane-local "shift in the bit of this lane" / "count this lane").
__device__ __forceinline__ uint32_t add2_carry(uint32_t t, uint32_t a, uint64_t mask) {
    uint32_t out;
    uint64_t cout;
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %3, %4"
                 : "=v"(out), "=s"(cout)
                 : "v"(t), "v"(a), "s"(mask));
    return out;
}

// One u-block I (64 rows, nb valid) against the wave's SD_WPW v-blocks.
// FULL: every v-block J is above I (J > I) — both directions are recorded;
// otherwise the diagonal band: J < I skipped, J == I direct only.  Rows are
// walked in descending order so the transposed words build up by doubling
// (t = 2t + bit): bit j of the word <-> row 64I + j; rows 63..32 feed the
// high half, 31..0 the low half.
template <int M, bool FULL, bool HI>
__device__ __forceinline__ void sd_rows(const int32_t* Rs, int64_t I, int nb, int64_t J0,
                                        const int32_t (&y)[SD_WPW][M], int lane,
                                        uint32_t (&acc_lo)[SD_WPW], uint32_t (&acc_hi)[SD_WPW],
                                        uint32_t (&tw)[SD_WPW], int32_t (&vcnt)[SD_WPW],
                                        int32_t& cpark) {
    const int jtop = HI ? 63 : 31, jbot = HI ? 32 : 0;
    // four rows per step: their ranks arrive with one 64-B scalar load, so a
    // wave waits on the scalar cache once per four rows
    // the next row's ranks are loaded (scalar) before this row is compared,
    // so the scalar-cache latency overlaps a row's worth of compares
    const c4_i32* xrow = (const c4_i32*)(const void*)Rs;
    int32_t xn[M];
#pragma unroll
    for (int o = 0; o < M; ++o) xn[o] = xrow[(I * 64 + jtop) * 4 + o];
    for (int j = jtop; j >= jbot; --j) {
        int32_t x[M];
#pragma unroll
        for (int o = 0; o < M; ++o) x[o] = xn[o];
        if (j > jbot) {
#pragma unroll
            for (int o = 0; o < M; ++o) xn[o] = xrow[(I * 64 + j - 1) * 4 + o];
        }
        if (j >= nb) {  // rows past the end of the population: shift in zeros
#pragma unroll
            for (int k = 0; k < SD_WPW; ++k) tw[k] += tw[k];
            continue;
        }
        int32_t ucnt = 0;
        const bool me = lane == j;
#pragma unroll
        for (int k = 0; k < SD_WPW; ++k) {
            if (!FULL && J0 + k < I) continue;  // pair handled with the roles swapped
            int32_t mn, mx;
            diff_minmax<M>(x, y[k], mn, mx);
            const uint64_t gm = __ballot(mn < 0);  // some x > y
            const uint64_t lm = __ballot(mx > 0);  // some x < y
            const uint64_t duv = gm & ~lm;         // u dominates v (v = lane)
            const uint64_t dvu = lm & ~gm;         // v dominates u
            acc_lo[k] = me ? (uint32_t)duv : acc_lo[k];  // park the direct word in lane j
            acc_hi[k] = me ? (uint32_t)(duv >> 32) : acc_hi[k];
            ucnt += __popcll(dvu);
            if (FULL || J0 + k > I) {  // off-diagonal: the transposed word and v's count too
                tw[k] = add2_carry(tw[k], tw[k], dvu);
                vcnt[k] = (int32_t)add2_carry((uint32_t)vcnt[k], 0u, duv);
            }
        }
        cpark = me ? ucnt : cpark;
    }
}

template <int M, bool FULL>
__device__ __forceinline__ void sd_block(const int32_t* Rs, int64_t I, int nb, int64_t J0,
                                         const int32_t (&y)[SD_WPW][M], int lane,
                                         uint32_t (&acc_lo)[SD_WPW], uint32_t (&acc_hi)[SD_WPW],
                                         uint32_t (&t_lo)[SD_WPW], uint32_t (&t_hi)[SD_WPW],
                                         int32_t (&vcnt)[SD_WPW], int32_t& cpark) {
    sd_rows<M, FULL, true>(Rs, I, nb, J0, y, lane, acc_lo, acc_hi, t_hi, vcnt, cpark);
    sd_rows<M, FULL, false>(Rs, I, nb, J0, y, lane, acc_lo, acc_hi, t_lo, vcnt, cpark);
}

template <int M>
__global__ __launch_bounds__(256) void sym_dom_kernel(const int4* __restrict__ R4, int64_t U,
                                                      int64_t NB, int64_t NG, int64_t ngroups,
                                                      int64_t ntasks, uint64_t* __restrict__ D,
                                                      int16_t* __restrict__ crow,
                                                      int16_t* __restrict__ ccol) {
    const int lane = threadIdx.x & 63;
    // wave-uniform task index (SGPR): everything derived from it is scalar
    const int64_t t = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    if (t >= ntasks) return;
    // decode (h, c, g) from the task index
    const int64_t pair = t >> 1;
    int64_t lo = 0, hi = (ngroups + 1) / 2;  // largest h with S(h) <= pair
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (sd_tasks_before(mid) <= pair) lo = mid;
        else hi = mid;
    }
    const int64_t h = lo;
    const int64_t c = pair - sd_tasks_before(h);
    const int64_t g = 2 * h + (t & 1);
    if (g >= ngroups) return;
    const int64_t J0 = g * SD_WPW;
    int32_t y[SD_WPW][M];
#pragma unroll
    for (int k = 0; k < SD_WPW; ++k) {
        const int64_t v = (J0 + k) * 64 + lane;
        if (v < U) {
            const int4 r = R4[v];
            y[k][0] = r.x;
            y[k][1] = r.y;
            if constexpr (M > 2) y[k][2] = r.z;
            if constexpr (M > 3) y[k][3] = r.w;
        } else {
            // a lane past the end: x > y in objective 0 and x < y in
            // objective 1 for every u, so neither side dominates
            y[k][0] = -1;
            y[k][1] = INT32_MAX;
            if constexpr (M > 2) y[k][2] = 0;
            if constexpr (M > 3) y[k][3] = 0;
        }
    }
    int32_t vcnt[SD_WPW] = {0, 0, 0, 0};
    const int64_t I_begin = c * SD_CHUNK;
    const int64_t I_end = std::min<int64_t>(std::min<int64_t>(I_begin + SD_CHUNK, J0 + SD_WPW), NB);
    const int32_t* Rs = (const int32_t*)(const void*)R4;
    for (int64_t IG = I_begin; IG < I_end; IG += SD_TG) {
        uint32_t t_lo[SD_WPW][SD_TG], t_hi[SD_WPW][SD_TG];
#pragma unroll
        for (int k = 0; k < SD_WPW; ++k)
#pragma unroll
            for (int ii = 0; ii < SD_TG; ++ii) t_lo[k][ii] = t_hi[k][ii] = 0;
#pragma unroll
        for (int ii = 0; ii < SD_TG; ++ii) {
            const int64_t I = IG + ii;
            if (I >= I_end) break;
            const int nb = (int)std::min<int64_t>(64, U - I * 64);
            uint32_t acc_lo[SD_WPW], acc_hi[SD_WPW], tl[SD_WPW], th[SD_WPW];
#pragma unroll
            for (int k = 0; k < SD_WPW; ++k) acc_lo[k] = acc_hi[k] = tl[k] = th[k] = 0;
            int32_t cpark = 0;
            if (I < J0)
                sd_block<M, true>(Rs, I, nb, J0, y, lane, acc_lo, acc_hi, tl, th, vcnt, cpark);
            else
                sd_block<M, false>(Rs, I, nb, J0, y, lane, acc_lo, acc_hi, tl, th, vcnt, cpark);
#pragma unroll
            for (int k = 0; k < SD_WPW; ++k) {
                t_lo[k][ii] = tl[k];
                t_hi[k][ii] = th[k];
            }
            // direct words: row 64I + lane, words J >= I of this v-group
            const int64_t u = I * 64 + lane;
            if (u < U) {
#pragma unroll
                for (int k = 0; k < SD_WPW; ++k) {
                    const int64_t J = J0 + k;
                    if (J >= I && J < NB) D[tword(u, J, NG)] = ((uint64_t)acc_hi[k] << 32) | acc_lo[k];
                }
                crow[g * U + u] = (int16_t)cpark;
            }
        }
        // transposed words: row 64J + lane, words I (< J) of this 8-block group
#pragma unroll
        for (int k = 0; k < SD_WPW; ++k) {
            const int64_t J = J0 + k;
            const int64_t v = J * 64 + lane;
            if (J >= NB || v >= U || IG >= J) continue;
            uint64_t* seg = D + tword(v, IG, NG);  // 64-B aligned row segment
            if (IG + SD_TG <= J && IG + SD_TG <= I_end) {
                uint4* q = reinterpret_cast<uint4*>(seg);
#pragma unroll
                for (int p = 0; p < SD_TG / 2; ++p)
                    q[p] = make_uint4(t_lo[k][2 * p], t_hi[k][2 * p], t_lo[k][2 * p + 1],
                                      t_hi[k][2 * p + 1]);
            } else {
#pragma unroll
                for (int ii = 0; ii < SD_TG; ++ii)
                    if (IG + ii < J && IG + ii < I_end)
                        seg[ii] = ((uint64_t)t_hi[k][ii] << 32) | t_lo[k][ii];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < SD_WPW; ++k) {
        const int64_t v = (J0 + k) * 64 + lane;
        if (v < U) ccol[c * U + v] = (int16_t)vcnt[k];
    }
}

// count[x] = sum over the v-groups g >= I(x)/4 of crow[g][x] + sum over the
// u-chunks c <= (I(x)/4)/4 of ccol[c][x]
__global__ void sym_count_reduce_kernel(const int16_t* __restrict__ crow,
                                        const int16_t* __restrict__ ccol, int64_t U,
                                        int64_t ngroups, int32_t* __restrict__ count) {
    DGRID_LOOP(x, U) {
        const int64_t g0 = (x >> 6) / SD_WPW;
        int32_t cnt = 0;
        for (int64_t g = g0; g < ngroups; ++g) cnt += crow[g * U + x];
        const int64_t cmax = g0 / 4;  // chunks of the tasks of v-group g0
        for (int64_t c = 0; c <= cmax; ++c) cnt += ccol[c * U + x];
        count[x] = cnt;
    }
}

// ---------------------------------------------------------------------------
// 3. device-driven front peeling
// ---------------------------------------------------------------------------
struct FrontState {
    int32_t F;         // size of the current front (ulist[ustart, ustart + F))
    int32_t ustart;
    int32_t nfronts;   // fronts emitted after front 0
    int32_t done;
    int32_t overflow;  // candidates exceed the LDS sort: the host orders them
    int32_t ncand;     // candidates of the next front appended by the peel
    int64_t sorted;    // individuals in the emitted fronts
    int64_t pending;   // individuals of the released candidates (gsize sums)
    int64_t N;         // min(n, k)
    int64_t U;
};

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)x, m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
// 64x64 bit transpose across the wave: in lane i bit j = A[i][j]; out lane j
// bit i = A[i][j].
__device__ __forceinline__ uint64_t transpose64_w(uint64_t x, int lane) {
    const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull,
                               0x00FF00FF00FF00FFull, 0x0F0F0F0F0F0F0F0Full,
                               0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int s = 32 >> st;
        const uint64_t mlo = masks[st];
        const uint64_t y = shfl_xor_u64(x, s);
        if (lane & s)
            x = (x & ~mlo) | ((y & ~mlo) >> s);
        else
            x = (x & mlo) | ((y & mlo) << s);
    }
    return x;
}

constexpr int PEEL_WAVES = 16;  // waves of a peel workgroup (they split the front's members)

// One workgroup owns one 8-word row segment s (v in [512 s, 512 s + 512)):
// its waves take interleaved 64-member slices of the front, transpose the
// members' row segments, and the per-wave (dominators, last position) of each
// v are reduced in LDS.  v is written by this workgroup only, so count and
// lastpos need no atomics; a v whose count reaches zero is released: its
// rank, its sort key (last releasing position, U index) and its individual
// count are recorded here, so the ordering kernel only sorts.
__global__ __launch_bounds__(1024) void peel_owned_kernel(const uint64_t* __restrict__ D,
                                                          int64_t NG,
                                                          const int32_t* __restrict__ ulist,
                                                          const int32_t* __restrict__ gsize,
                                                          FrontState* st, int32_t* count,
                                                          uint64_t* ckey, int32_t* rankU) {
    __shared__ int32_t sdec[PEEL_WAVES][512];
    __shared__ int32_t slast[PEEL_WAVES][512];
    __shared__ int32_t sF, sust, sstop, snf;
    if (threadIdx.x == 0) {
        sF = st->F;
        sust = st->ustart;
        snf = st->nfronts;
        sstop = st->done | st->overflow;
    }
    __syncthreads();
    if (sstop) return;
    const int64_t F = sF, U = st->U, s = blockIdx.x;
    const int32_t* members = ulist + sust;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int32_t dec[8], last[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        dec[w] = 0;
        last[w] = -1;
    }
    for (int64_t j0 = (int64_t)wave * 64; j0 < F; j0 += PEEL_WAVES * 64) {
        const int64_t j = j0 + lane;
        uint64_t seg[8];
        if (j < F) {
            const uint4* q = reinterpret_cast<const uint4*>(D + tword(members[j], s * 8, NG));
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const uint4 v = q[p];
                seg[2 * p] = ((uint64_t)v.y << 32) | v.x;
                seg[2 * p + 1] = ((uint64_t)v.w << 32) | v.z;
            }
        } else {
#pragma unroll
            for (int w = 0; w < 8; ++w) seg[w] = 0;
        }
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint64_t tcol = transpose64_w(seg[w], lane);  // bit i: member j0+i dominates v
            dec[w] += __popcll(tcol);
            if (tcol) last[w] = (int32_t)(j0 + 63 - __clzll(tcol));
        }
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        sdec[wave][w * 64 + lane] = dec[w];
        slast[wave][w * 64 + lane] = last[w];
    }
    __syncthreads();
    if (threadIdx.x >= 512) return;
    const int t = threadIdx.x;
    int32_t d = 0, l = -1;
#pragma unroll
    for (int wv = 0; wv < PEEL_WAVES; ++wv) {
        d += sdec[wv][t];
        l = max(l, slast[wv][t]);
    }
    const int64_t v = s * 512 + t;
    bool fresh = false;
    if (v < U && d > 0) {
        const int32_t left = count[v] - d;
        count[v] = left;
        fresh = left == 0;
    }
    const unsigned long long fm = __ballot(fresh);
    if (fm) {
        const int first = __ffsll(fm) - 1;
        int32_t base = 0;
        if (lane == first) base = atomicAdd(&st->ncand, __popcll(fm));
        base = __shfl(base, first, 64);
        int64_t gs = 0;
        if (fresh) {
            ckey[base + __popcll(fm & ((1ull << lane) - 1))] =
                ((uint64_t)(uint32_t)l << 32) | (uint32_t)v;
            rankU[v] = snf + 1;
            gs = gsize[v];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) gs += __shfl_xor(gs, o, 64);
        if (lane == first) atomicAdd((unsigned long long*)&st->pending, (unsigned long long)gs);
    }
}

constexpr int ORDER_CAP = 16384;  // candidates sorted in registers + LDS by one workgroup

// Bitonic sort of P = 1024 * E keys held E per thread (element i = tid*E + e),
// ascending: compare-exchanges of stride < E stay in registers, strides below
// 64 E go through lane shuffles, only the longer ones through LDS (one
// barrier per stage), so a 2,048-key sort needs 18 barriers instead of 66.
template <int E>
__device__ void block_bitonic(uint64_t (&k)[E], uint64_t* lds) {
    constexpr int P = 1024 * E;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int size = 2; size <= P; size <<= 1) {
        int stride = size >> 1;
        if (stride >= 64 * E) {
#pragma unroll
            for (int e = 0; e < E; ++e) lds[tid * E + e] = k[e];
            __syncthreads();
            for (; stride >= 64 * E; stride >>= 1) {
                for (int q = tid; q < P / 2; q += 1024) {
                    const int a = 2 * q - (q & (stride - 1));
                    const int b = a + stride;
                    const bool up = (a & size) == 0;
                    const uint64_t ka = lds[a], kb = lds[b];
                    if ((ka > kb) == up) {
                        lds[a] = kb;
                        lds[b] = ka;
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (int e = 0; e < E; ++e) k[e] = lds[tid * E + e];
            __syncthreads();
        }
        for (; stride >= E; stride >>= 1) {
            const int ls = stride / E;
            const bool lower = (lane & ls) == 0;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint64_t p = shfl_xor_u64(k[e], ls);
                const bool up = ((tid * E + e) & size) == 0;
                const bool take_min = lower == up;
                k[e] = take_min ? (p < k[e] ? p : k[e]) : (p > k[e] ? p : k[e]);
            }
        }
        // strides below E: registers of this thread (compile-time indices)
#pragma unroll
        for (int st2 = E / 2; st2 > 0; st2 >>= 1) {
            if (st2 >= size) continue;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                if (e & st2) continue;
                const int f = e | st2;
                const bool up = ((tid * E + e) & size) == 0;
                const uint64_t a = k[e], b = k[f];
                const bool sw = (a > b) == up;
                k[e] = sw ? b : a;
                k[f] = sw ? a : b;
            }
        }
    }
}

template <int E>
__device__ void order_sorted(const uint64_t* ckey, int32_t n, int32_t* out, uint64_t* lds) {
    uint64_t k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        k[e] = i < n ? ckey[i] : ~0ull;
    }
    block_bitonic<E>(k, lds);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        if (i < n) out[i] = (int32_t)(uint32_t)k[e];
    }
}

// Orders the released candidates by (last releasing position, U index),
// appends them to ulist as the next front and updates the state.
// presorted: ckey already ordered (the host's radix-sort fallback for fronts
// larger than ORDER_CAP).
__global__ __launch_bounds__(1024) void front_order_kernel(FrontState* st, const uint64_t* ckey,
                                                           int32_t* ulist, int32_t* fstarts,
                                                           int presorted) {
    __shared__ uint64_t lds[ORDER_CAP];
    __shared__ int32_t sn, sgo, snstart;
    if (threadIdx.x == 0) {
        sgo = !(st->done || (st->overflow && !presorted));
        sn = st->ncand;
        snstart = st->ustart + st->F;
    }
    __syncthreads();
    if (!sgo) return;
    const int32_t n = sn;
    if (n == 0) {  // nothing released: the reference's `if F2 == 0: break`
        if (threadIdx.x == 0) st->done = 1;
        return;
    }
    if (!presorted && n > ORDER_CAP) {
        if (threadIdx.x == 0) st->overflow = 1;
        return;
    }
    int32_t* out = ulist + snstart;
    if (presorted) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = (int32_t)(uint32_t)ckey[i];
    } else if (n <= 1024) {
        order_sorted<1>(ckey, n, out, lds);
    } else if (n <= 2048) {
        order_sorted<2>(ckey, n, out, lds);
    } else if (n <= 4096) {
        order_sorted<4>(ckey, n, out, lds);
    } else if (n <= 8192) {
        order_sorted<8>(ckey, n, out, lds);
    } else {
        order_sorted<16>(ckey, n, out, lds);
    }
    if (threadIdx.x == 0) {
        const int32_t nstart = snstart, r = st->nfronts;
        const int64_t sorted = st->sorted + st->pending;
        st->sorted = sorted;
        st->pending = 0;
        st->ustart = nstart;
        st->F = n;
        st->nfronts = r + 1;
        st->ncand = 0;
        st->overflow = 0;
        fstarts[r + 2] = nstart + n;
        // emo.py:109: continue while pareto_sorted < N (and fronts remain)
        if (sorted >= st->N || nstart + n >= st->U) st->done = 1;
    }
}

__global__ void front_init_kernel(FrontState* st, int32_t F0, int64_t sorted0, int64_t N, int64_t U,
                                  int32_t* fstarts) {
    st->F = F0;
    st->ustart = 0;
    st->nfronts = 0;
    st->done = (sorted0 >= N || F0 >= U || F0 == 0) ? 1 : 0;
    st->overflow = 0;
    st->ncand = 0;
    st->sorted = sorted0;
    st->pending = 0;
    st->N = N;
    st->U = U;
    fstarts[0] = 0;
    fstarts[1] = F0;
}

// ---------------------------------------------------------------------------
// host drivers (called from nsga2.hip)
// ---------------------------------------------------------------------------
size_t fast_dom_ranks_bytes(int64_t U) {
    return 2 * align_up((size_t)U * 8, 256) +
           3 * align_up((size_t)U * 4, 256) + radix_sort_temp_bytes(U) + scan_temp_bytes(U);
}

// Dense ranks of each objective; `work` holds fast_dom_ranks_bytes(U) bytes.
int fast_dom_ranks(hipStream_t s, const double* ufit, int m, int64_t U, int4* R4, char* work) {
    uint64_t* keys = (uint64_t*)work;
    uint64_t* ktmp = (uint64_t*)(work + align_up((size_t)U * 8, 256));
    char* p = work + 2 * align_up((size_t)U * 8, 256);
    int32_t* vals = (int32_t*)p;
    int32_t* vtmp = (int32_t*)(p + align_up((size_t)U * 4, 256));
    int32_t* flag = (int32_t*)(p + 2 * align_up((size_t)U * 4, 256));
    void* rtemp = p + 3 * align_up((size_t)U * 4, 256);
    void* stemp = (char*)rtemp + radix_sort_temp_bytes(U);
    DM_HIP(hipMemsetAsync(R4, 0, (size_t)U * 16, s));
    for (int o = 0; o < m; ++o) {
        rank_key_kernel<<<dg1(U), 256, 0, s>>>(ufit, m, o, U, keys, vals);
        int rc = radix_sort_pairs(s, keys, vals, ktmp, vtmp, U, 0, 64, rtemp);
        if (rc) return rc;
        rank_flag_kernel<<<dg1(U), 256, 0, s>>>(keys, U, flag);
        // the scan may not alias its input: the exclusive prefix goes to vtmp
        if ((rc = exclusive_scan_i32(s, flag, vtmp, U, nullptr, stemp))) return rc;
        rank_scatter_kernel<<<dg1(U), 256, 0, s>>>(vals, vtmp, flag, U, o, (int32_t*)R4);
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int64_t fast_dom_words(int64_t U) {
    const int64_t NB = (U + 63) / 64, NG = (NB + 7) / 8;
    return NB * 64 * NG * 8;
}
size_t fast_dom_partial_bytes(int64_t U) {
    const int64_t NB = (U + 63) / 64;
    const int64_t ngroups = (NB + SD_WPW - 1) / SD_WPW;
    const int64_t nchunks = (NB + SD_CHUNK - 1) / SD_CHUNK;
    return align_up((size_t)ngroups * U * 2, 256) + align_up((size_t)nchunks * U * 2, 256);
}

// D (tiled, fast_dom_words(U) words) and count[U] from the ranks.
int fast_dom_matrix(hipStream_t s, const int4* R4, int m, int64_t U, uint64_t* D, char* partials,
                    int32_t* count) {
    const int64_t NB = (U + 63) / 64, NG = (NB + 7) / 8;
    const int64_t ngroups = (NB + SD_WPW - 1) / SD_WPW;
    int16_t* crow = (int16_t*)partials;
    int16_t* ccol = (int16_t*)(partials + align_up((size_t)ngroups * U * 2, 256));
    const int64_t ntasks = sd_task_count(ngroups);
    const unsigned blocks = (unsigned)((ntasks + 3) / 4);
    switch (m) {
        case 2: sym_dom_kernel<2><<<blocks, 256, 0, s>>>(R4, U, NB, NG, ngroups, ntasks, D, crow, ccol); break;
        case 3: sym_dom_kernel<3><<<blocks, 256, 0, s>>>(R4, U, NB, NG, ngroups, ntasks, D, crow, ccol); break;
        default: sym_dom_kernel<4><<<blocks, 256, 0, s>>>(R4, U, NB, NG, ngroups, ntasks, D, crow, ccol); break;
    }
    DM_LAUNCH_CHECK();
    sym_count_reduce_kernel<<<dg1(U), 256, 0, s>>>(crow, ccol, U, ngroups, count);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

size_t fast_fronts_bytes(int64_t U) {
    return align_up(sizeof(FrontState), 256) + 2 * align_up((size_t)U * 8, 256) +
           align_up((size_t)U * 8, 256) + 2 * align_up((size_t)U * 4, 256) +
           radix_sort_temp_bytes(U);
}

// Fronts 1.. after front 0 (ulist[0, F0), rankU set): peel on the device,
// checking the status every few fronts.  Fills ufront (front starts in ulist,
// host) and *sorted (individuals).  `work`: fast_fronts_bytes(U).
int fast_fronts(dm_ctx* ctx, const uint64_t* D, int64_t U, int32_t F0, int64_t sorted0, int64_t N,
                const int32_t* gsize, int32_t* ulist, int32_t* rankU, int32_t* count,
                int32_t* fstarts, char* work, std::vector<int32_t>& ufront, int64_t* sorted) {
    hipStream_t s = ctx->stream;
    const int64_t NB = (U + 63) / 64, NG = (NB + 7) / 8;
    char* p = work;
    FrontState* st = (FrontState*)p;
    p += align_up(sizeof(FrontState), 256);
    uint64_t* ckey = (uint64_t*)p;
    p += align_up((size_t)U * 8, 256);
    uint64_t* ktmp = (uint64_t*)p;
    p += align_up((size_t)U * 8, 256);
    uint64_t* kspare = (uint64_t*)p;  // keep the layout of fast_fronts_bytes
    p += align_up((size_t)U * 8, 256);
    int32_t* vals = (int32_t*)p;
    p += align_up((size_t)U * 4, 256);
    int32_t* vtmp = (int32_t*)p;
    p += align_up((size_t)U * 4, 256);
    void* rtemp = p;
    (void)kspare;
    front_init_kernel<<<1, 1, 0, s>>>(st, F0, sorted0, N, U, fstarts);
    FrontState* hst = (FrontState*)pinned(ctx, sizeof(FrontState));
    if (!hst) return DM_ERR_NOMEM;
    int batch = 4;
    for (;;) {
        for (int b = 0; b < batch; ++b) {
            peel_owned_kernel<<<(unsigned)NG, 1024, 0, s>>>(D, NG, ulist, gsize, st, count, ckey,
                                                            rankU);
            front_order_kernel<<<1, 1024, 0, s>>>(st, ckey, ulist, fstarts, 0);
        }
        DM_LAUNCH_CHECK();
        DM_HIP(hipMemcpyAsync(hst, st, sizeof(FrontState), hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        if (hst->done) break;
        if (hst->overflow) {
            // a front too large for the LDS sort: the radix sort orders its keys
            const int32_t n = hst->ncand;
            DM_HIP(hipMemsetAsync(vals, 0, (size_t)n * 4, s));
            int rc = radix_sort_pairs(s, ckey, vals, ktmp, vtmp, n, 0, 64, rtemp);
            if (rc) return rc;
            front_order_kernel<<<1, 1024, 0, s>>>(st, ckey, ulist, fstarts, 1);
            DM_LAUNCH_CHECK();
        }
        batch = std::min(batch * 2, 32);
    }
    const int32_t nf = hst->nfronts + 1;  // front 0 plus the peeled ones
    ufront.resize(nf + 1);
    DM_HIP(hipMemcpyAsync(ufront.data(), fstarts, (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, s));
    DM_HIP(hipStreamSynchronize(s));
    *sorted = hst->sorted;
    return DM_OK;
}

}  // namespace dm
