// bitdom.hpp — bitset-table dominance (bitdom.hip): constants, the tables'
// layout and the device helpers shared by the table passes and the
// table-fed front peel (dominance.hip peel_order_kernel).
#pragma once
#include "dominance.hpp"

namespace dm {

constexpr int BD_CW = 512;        // v of a chunk
constexpr int BD_K = BD_CW + 1;   // prefix sets per chunk and objective
constexpr int BD_RT = 16384;      // rows (row pass) / v (count pass) per task
constexpr int BD_THREADS = 512;
// bucket starts per chunk and objective: bucket b holds the ranks in
// [b << sh, (b + 1) << sh), sh the smallest shift with U >> sh <= 1024
constexpr int BD_BKN = 1026;
__host__ __device__ __forceinline__ int bd_bucket_shift(int64_t U) {
    int sh = 0;
    while ((U >> sh) > 1024) ++sh;
    return sh;
}

#ifndef DM_BD_ABLATE
#define DM_BD_ABLATE 0
#endif

struct BitdomLayout {
    int64_t NB, NG, Upad;
    size_t part, P, R, BK, first, last, span, rowfirst, reach, toffD, toffC, total;
};
static inline BitdomLayout bitdom_layout(int64_t U, int m) {
    BitdomLayout L;
    const int64_t F = m - 1;
    L.NB = (U + 63) / 64;
    L.NG = (L.NB + 7) / 8;
    L.Upad = L.NB * 64;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(std::max<size_t>(bytes, 1), 256);
        return o;
    };
    L.part = take((size_t)L.NG * L.Upad * 2);
    L.P = take((size_t)L.NG * F * BD_K * 64);
    L.R = take((size_t)L.NG * F * BD_CW * 4);
    L.BK = take((size_t)L.NG * F * BD_BKN * 2);
    L.first = take((size_t)U * 4);
    L.last = take((size_t)U * 4);
    L.span = take((size_t)U * 8);
    L.rowfirst = take((size_t)L.NG * 4);
    L.reach = take((size_t)L.NG * 4);
    L.toffD = take((size_t)(L.NG + 1) * 4);
    L.toffC = take((size_t)(L.NG + 1) * 4);
    L.total = off;
    return L;
}
// #{j : sr[j] <= x} (LE) or #{j : sr[j] < x} over 512 ascending values held
// in LDS with one pad word after every 32 (value j at j + j / 32, bd_rpad),
// starting from the bucket table sb: sb[b] = #{j : sr[j] < b << sh}, so only
// the values of x's own bucket are scanned (0.6 of them on average at 512
// values per ~830 buckets) — two or three dependent LDS reads where a binary
// search over the 512 needs ten.
constexpr int BD_RP = BD_CW + BD_CW / 32;  // padded sorted-rank array
__device__ __forceinline__ int bd_rpad(int j) { return j + (j >> 5); }
template <bool LE>
__device__ __forceinline__ int bd_count_below(const int32_t* sr, const uint16_t* sb, int sh,
                                              int32_t x) {
    const int b = x >> sh;
    int j = sb[b];
    const int e = sb[b + 1];
    while (j < e) {
        const int32_t y = sr[bd_rpad(j)];
        if (!(LE ? y <= x : y < x)) break;
        ++j;
    }
    return j;
}

// dword d of a chunk holds positions 32d..32d+31
__device__ __forceinline__ uint32_t upto_mask(int32_t lim, int d) {  // positions <= lim
    const int32_t x = lim - 32 * d;
    return x >= 31 ? ~0u : x < 0 ? 0u : (2u << x) - 1u;
}
__device__ __forceinline__ uint32_t from_mask(int32_t lo, int d) {  // positions >= lo
    const int32_t x = lo - 32 * d;
    return x <= 0 ? ~0u : x > 31 ? 0u : ~0u << x;
}
// positions <= lim without position ps, for dword d: dl = lim >> 5, part =
// the mask of dword dl, ds = ps >> 5 (-1: none), sb = ~bit(ps)
__device__ __forceinline__ uint32_t row_mask(int32_t dl, uint32_t part, int32_t ds, uint32_t sb,
                                             int d) {
    const uint32_t m = d < dl ? ~0u : (d == dl ? part : 0u);
    return d == ds ? (m & sb) : m;
}

// The task's chunk (last c with toff[c] <= t) and the tables of that chunk
// into LDS.
template <int F>
__device__ __forceinline__ int64_t bd_task_chunk(const int32_t* toff, int64_t NG, int32_t t) {
    int64_t lo = 0, hi = NG - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (toff[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// The chunk's bucket tables (F x BD_BKN uint16) into LDS: the first F of the
// FG objectives the global tables hold per chunk.
template <int F, int FG = F>
__device__ __forceinline__ void bd_load_buckets(const uint16_t* BK, int64_t c,
                                                uint16_t (&sB)[F][BD_BKN]) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(BK + c * FG * BD_BKN);
    uint32_t* l = reinterpret_cast<uint32_t*>(&sB[0][0]);
    for (int i = threadIdx.x; i < F * BD_BKN / 2; i += blockDim.x) l[i] = g[i];
}
template <int F, int FG = F>
__device__ __forceinline__ void bd_load_tables(const uint32_t* P, const int32_t* R, const uint16_t* BK,
                                               int64_t c, uint4 (&sP)[F][BD_K * 4],
                                               int32_t (&sR)[F][BD_RP], uint16_t (&sB)[F][BD_BKN]) {
    bd_load_buckets<F, FG>(BK, c, sB);
    // batches of 4 global loads in flight, then their LDS stores: the staging
    // stays in registers (a whole-table register array of up to 13 pieces was
    // placed in scratch memory by the compiler)
    constexpr int NP = F * BD_K * 4, NR = F * BD_CW / 4;
    const uint4* gP = reinterpret_cast<const uint4*>(P + c * FG * BD_K * 16);
    const int4* gR = reinterpret_cast<const int4*>(R + c * FG * BD_CW);
    uint4* lP = &sP[0][0];
    for (int i0 = threadIdx.x; i0 < NP; i0 += 4 * BD_THREADS) {
        uint4 t0 = make_uint4(0, 0, 0, 0), t1 = t0, t2 = t0, t3 = t0;
        const int i1 = i0 + BD_THREADS, i2 = i1 + BD_THREADS, i3 = i2 + BD_THREADS;
        t0 = gP[i0];
        if (i1 < NP) t1 = gP[i1];
        if (i2 < NP) t2 = gP[i2];
        if (i3 < NP) t3 = gP[i3];
        lP[i0] = t0;
        if (i1 < NP) lP[i1] = t1;
        if (i2 < NP) lP[i2] = t2;
        if (i3 < NP) lP[i3] = t3;
    }
    for (int i = threadIdx.x; i < NR; i += BD_THREADS) {  // values 4i..4i+3 of the F arrays
        const int4 t = gR[i];
        const int f = (4 * i) / BD_CW, e = (4 * i) % BD_CW;
        int32_t* d = &sR[f][0];
        d[bd_rpad(e)] = t.x;
        d[bd_rpad(e + 1)] = t.y;
        d[bd_rpad(e + 2)] = t.z;
        d[bd_rpad(e + 3)] = t.w;
    }
    __syncthreads();
}

// Sources of the 64-byte prefix sets P_f[C][k] (four 16-byte pieces j):
// the chunk's tables in LDS, or its slice of the global table (the peel reads
// only the sets its members need).
template <int F>
struct BdLdsSets {
    const uint4 (&sP)[F][BD_K * 4];
    __device__ __forceinline__ uint4 operator()(int f, int k, int j) const { return sP[f][k * 4 + j]; }
};
struct BdGlobalSets {
    const uint4* gP;  // the chunk's F x BD_K x 4 pieces
    __device__ __forceinline__ uint4 operator()(int f, int k, int j) const {
        return gP[(f * BD_K + k) * 4 + j];
    }
};

// Row u's 512 bits over chunk C (positions v0 + p): prefix0(u) (p <= lim) and
// the prefix sets of its other ranks, without its own bit (position ps when
// in C); piece i of w holds dwords 4j..4j+3 with j = (i + rot) & 3.
template <int M, typename Sets>
__device__ __forceinline__ void bd_row_words(const int4 su, int32_t lim, int32_t ps, const Sets& sets,
                                             const int32_t (&sR)[M - 1][BD_RP],
                                             const uint16_t (&sB)[M - 1][BD_BKN], int sh, int rot,
                                             uint4 (&w)[4]) {
    constexpr int F = M - 1;
    if (lim < 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = make_uint4(0, 0, 0, 0);
        return;
    }
    int k[F];
#pragma unroll
    for (int f = 0; f < F; ++f) k[f] = bd_count_below<true>(sR[f], sB[f], sh, icomp(su, f));
#ifdef DM_BD_CHECK
    for (int f = 0; f < F; ++f)
        if (!BD_OK(k[f], BD_K, "rows k")) k[f] = 0;
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = (i + rot) & 3;
        w[i] = sets(0, k[0], j);
#pragma unroll
        for (int f = 1; f < F; ++f) {
            const uint4 y = sets(f, k[f], j);
            w[i].x &= y.x;
            w[i].y &= y.y;
            w[i].z &= y.z;
            w[i].w &= y.w;
        }
    }
    const bool self = (uint32_t)ps < (uint32_t)BD_CW;
    if (lim < BD_CW - 1 || self) {  // prefix0 ends in C, or u is in C
        const int32_t dl = lim >= BD_CW - 1 ? 16 : lim >> 5;
        const uint32_t part = (2u << (lim & 31)) - 1u;
        const int32_t ds = self ? ps >> 5 : -1;
        const uint32_t sb = ~(1u << (ps & 31));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d0 = 4 * ((i + rot) & 3);
            w[i].x &= row_mask(dl, part, ds, sb, d0);
            w[i].y &= row_mask(dl, part, ds, sb, d0 + 1);
            w[i].z &= row_mask(dl, part, ds, sb, d0 + 2);
            w[i].w &= row_mask(dl, part, ds, sb, d0 + 3);
        }
    }
}

// The pieces of bd_row_words for a software pipeline (the table peel): the
// searches, the set pieces (raw: loads in flight until used), and the merge.
template <int F>
__device__ __forceinline__ void bd_row_k(const int4 su, const int32_t (&sR)[F][BD_RP],
                                         const uint16_t (&sB)[F][BD_BKN], int sh, int (&k)[F]) {
#pragma unroll
    for (int f = 0; f < F; ++f) k[f] = bd_count_below<true>(sR[f], sB[f], sh, icomp(su, f));
}
template <int F, typename Sets>
__device__ __forceinline__ void bd_row_fetch(const Sets& sets, const int (&k)[F], uint4 (&raw)[F][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int f = 0; f < F; ++f) raw[f][i] = sets(f, k[f], i);
}
// SELF = false (the peel): u's own bit is left set — u is a member of the
// front being peeled, its count is already zero and one more decrement
// releases nothing; only the objective-0 prefix is masked.
template <int F, bool SELF = true>
__device__ __forceinline__ void bd_row_merge(const uint4 (&raw)[F][4], int32_t lim, int32_t ps,
                                             uint4 (&w)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[i] = raw[0][i];
#pragma unroll
        for (int f = 1; f < F; ++f) {
            w[i].x &= raw[f][i].x;
            w[i].y &= raw[f][i].y;
            w[i].z &= raw[f][i].z;
            w[i].w &= raw[f][i].w;
        }
    }
    const bool self = SELF && (uint32_t)ps < (uint32_t)BD_CW;
    if (lim < BD_CW - 1 || self) {
        const int32_t dl = lim >= BD_CW - 1 ? 16 : (lim < 0 ? -1 : lim >> 5);
        const uint32_t part = lim < 0 ? 0u : (2u << (lim & 31)) - 1u;
        if (SELF) {
            const int32_t ds = self ? ps >> 5 : -1;
            const uint32_t sb = ~(1u << (ps & 31));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[i].x &= row_mask(dl, part, ds, sb, 4 * i);
                w[i].y &= row_mask(dl, part, ds, sb, 4 * i + 1);
                w[i].z &= row_mask(dl, part, ds, sb, 4 * i + 2);
                w[i].w &= row_mask(dl, part, ds, sb, 4 * i + 3);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[i].x &= 4 * i < dl ? ~0u : (4 * i == dl ? part : 0u);
                w[i].y &= 4 * i + 1 < dl ? ~0u : (4 * i + 1 == dl ? part : 0u);
                w[i].z &= 4 * i + 2 < dl ? ~0u : (4 * i + 2 == dl ? part : 0u);
                w[i].w &= 4 * i + 3 < dl ? ~0u : (4 * i + 3 == dl ? part : 0u);
            }
        }
    }
}

// The chunk's sorted-rank arrays into LDS (padded, bd_rpad).
template <int F>
__device__ __forceinline__ void bd_load_ranks(const int32_t* R, int64_t c, int32_t (&sR)[F][BD_RP]) {
    const int32_t* g = R + c * F * BD_CW;
    for (int i = threadIdx.x; i < F * BD_CW; i += blockDim.x)
        sR[i / BD_CW][bd_rpad(i % BD_CW)] = g[i];
    __syncthreads();
}

}  // namespace dm
