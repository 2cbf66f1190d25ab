// dominance.hpp — definitions shared by the fast sortNondominated kernels
// (dominance.hip: ranks, compare kernel, peel; bitdom.hip: bitset tables).
#pragma once
#include "sort.hpp"

namespace dm {

#define DGRID_LOOP(i, n)                                                         \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
         i += (int64_t)gridDim.x * blockDim.x)

static inline dim3 dg1(int64_t n) {
    return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65535)));
}

// 64-row blocks per A-group: the unit of a row's reach (nseg[g], in 512-v
// halves) that the peel reads D words up to.
#ifndef DM_TD_WPW
#define DM_TD_WPW 4
#endif
constexpr int TD_WPW = DM_TD_WPW;

// component c of S[q] = int4 {rank_1, .., rank_{m-1}, rank_0, pad}
__host__ __device__ __forceinline__ int32_t icomp(const int4& r, int c) {
    return c == 0 ? r.x : c == 1 ? r.y : c == 2 ? r.z : r.w;
}

// word w of row u in the tiled layout: tiles of 64 rows x TW = 16 words (one
// 128-byte line per row, 8 KB), NQ = 16-word groups per row.  Word w of a row
// holds the bits of v in [64 w, 64 w + 64) (bit j <-> v = 64 w + j); words
// 8h..8h+7 of a line are the row's 512-v half h of that 1,024-v segment.
constexpr int TW = 16;
__host__ __device__ __forceinline__ int64_t tword(int64_t u, int64_t w, int64_t NQ) {
    return ((((u >> 6) * NQ + w / TW) << 6) + (u & 63)) * TW + (w % TW);
}

// bitdom.hip: dominator counts and (when D is not null) the D words by bitset
// tables (the default dominance pass of the fast path).  ws: that pass's
// scratch of bitdom_bytes(U, m) bytes, which keeps the tables for the
// table-fed peel.
size_t bitdom_bytes(int64_t U, int m);
int bitdom_build(dm_ctx* ctx, const int4* S, int m, int64_t U, int64_t NQ, int64_t ngroups,
                 const int32_t* nseg, const int32_t* sigma, uint64_t* D, int32_t* count,
                 int32_t* countq, char* ws);

}  // namespace dm
