// dominance.hpp — definitions shared by the fast sortNondominated kernels
// (dominance.hip: ranks, compare kernel, peel; bitdom.hip: bitset tables).
#pragma once
#include "sort.hpp"

namespace dm {

// DM_BD_CHECK builds (diagnostics only): the global indices of the bitset
// dominance pass, the table-fed peel and the front ordering are range-checked
// and an out-of-range one is printed and skipped; the fast path's workspace
// is filled with a poison pattern first (a read before write shows up as an
// out-of-range index).
#ifdef DM_BD_CHECK
__device__ __forceinline__ bool bd_ok(int64_t i, int64_t n, const char* tag) {
    if (i >= 0 && i < n) return true;
    printf("bitdom OOB %s: %lld of %lld (block %d,%d thread %d)\n", tag, (long long)i,
           (long long)n, (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);
    return false;
}
#define BD_OK(i, n, tag) bd_ok((int64_t)(i), (int64_t)(n), tag)
#else
#define BD_OK(i, n, tag) true
#endif


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

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)x, m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(x >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Bitonic sort of P = NT * E keys held E per thread (element i = tid*E + e),
// ascending: compare-exchanges of stride < E stay in registers, strides below
// 64 E go through lane shuffles, only the longer ones through LDS (one
// barrier per stage), so a 2,048-key sort needs 18 barriers instead of 66.
template <int NT, int E>
__device__ void block_bitonic(uint64_t (&k)[E], uint64_t* lds) {
    constexpr int P = NT * E;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int size = 2; size <= P; size <<= 1) {
        int stride = size >> 1;
        if (stride >= 64 * E) {
#pragma unroll
            for (int e = 0; e < E; ++e) lds[tid * E + e] = k[e];
            __syncthreads();
            for (; stride >= 64 * E; stride >>= 1) {
                for (int q = tid; q < P / 2; q += NT) {
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

// bitdom.hip: dominator counts and (when D is not null) the D words by bitset
// tables (the default dominance pass of the fast path).  ws: that pass's
// scratch of bitdom_bytes(U, m) bytes, which keeps the tables for the
// table-fed peel.
size_t bitdom_bytes(int64_t U, int m);
int bitdom_build(dm_ctx* ctx, const int4* S, int m, int64_t U, int64_t NQ, int64_t ngroups,
                 const int32_t* nseg, const int32_t* sigma, uint64_t* D, int32_t* count,
                 int32_t* countq, char* ws);

}  // namespace dm
