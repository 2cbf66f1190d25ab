// sort.hpp — device sort / scan primitives used by selBest, NSGA-II and
// migration: a stable LSD radix sort of (uint64 key, int32 value) pairs with
// 8-bit digits, and int32 prefix scans.  All launches are asynchronous on the
// given stream; temporaries come from the caller.
#pragma once
#include "common.hpp"

namespace dm {

// Order-preserving map double -> uint64 (ascending); -0.0 == +0.0 as in
// Python's float comparison.
__host__ __device__ __forceinline__ uint64_t ordered_key(double x) {
    if (x == 0.0) x = 0.0;
    uint64_t b;
    memcpy(&b, &x, 8);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Scratch needed by radix_sort_pairs for n elements.
size_t radix_sort_temp_bytes(int64_t n);

// Stable sort of (keys, vals) by keys bits [begin_bit, end_bit).  Results end
// in keys/vals (the tmp buffers are ping-pong storage of n elements each).
// `temp` must hold radix_sort_temp_bytes(n) bytes.
int radix_sort_pairs(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                     int32_t* vals_tmp, int64_t n, int begin_bit, int end_bit, void* temp);
// nseg independent segments of seglen keys each (segment g at [g seglen,
// (g + 1) seglen)), sorted in the same launches; `temp` must hold
// radix_sort_batched_temp_bytes(nseg, seglen) bytes.
size_t radix_sort_batched_temp_bytes(int64_t nseg, int64_t seglen);
int radix_sort_pairs_batched(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                             int32_t* vals_tmp, int64_t nseg, int64_t seglen, int begin_bit,
                             int end_bit, void* temp, bool* in_tmp = nullptr);
// radix_sort_pairs without the copy back after an odd number of passes:
// *in_tmp tells whether the sorted pairs are in keys_tmp / vals_tmp.
int radix_sort_pairs_any(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                         int32_t* vals_tmp, int64_t n, int begin_bit, int end_bit, void* temp,
                         bool* in_tmp);

// Pairs one workgroup sorts in LDS; keys of at most 32 bits: twice as many.
constexpr int LDS_SORT_CAP = 4096;
constexpr int LDS_SORT_CAP32 = 8192;
// Stable sort of nseg variable-length segments [starts[g], starts[g + 1])
// (starts on the device), each of at most LDS_SORT_CAP pairs (LDS_SORT_CAP32
// when begin_bit = 0 and end_bit <= 32, keys then < 2^32) by key bits
// [begin_bit, end_bit): one workgroup per segment, in LDS, one launch.  A
// segment over that capacity is still sorted exactly, by its workgroup
// through keys_tmp / vals_tmp (n entries, same offsets) in global memory.
int seg_sort_pairs_small(hipStream_t s, uint64_t* keys, int32_t* vals, const int32_t* starts,
                         int64_t nseg, int begin_bit, int end_bit, uint64_t* keys_tmp,
                         int32_t* vals_tmp);

// Inclusive scan (sum, or max when MAX) of a wave through DPP moves: within
// each row of 16 lanes by row_shr 1, 2, 4, 8, then row 0's / rows 0-1's last
// lane broadcast into the rows above (row_bcast:15, row_bcast:31).  Lanes a
// move does not reach take the identity.  Six VALU ops with DPP operands
// instead of six ds_bpermute round trips through the LDS crossbar.
template <bool MAX>
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x, int width = 64) {
    constexpr int32_t ident = MAX ? INT32_MIN : 0;
    auto op = [](int32_t a, int32_t b) { return MAX ? max(a, b) : a + b; };
    x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x111, 0xF, 0xF, false));  // row_shr:1
    x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x112, 0xF, 0xF, false));  // row_shr:2
    x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x114, 0xF, 0xF, false));  // row_shr:4
    x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x118, 0xF, 0xF, false));  // row_shr:8
    if (width > 16)
        x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    if (width > 32)
        x = op(x, __builtin_amdgcn_update_dpp(ident, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return x;
}

// Inclusive scan (sum, or max when MAX) over the NT threads of a workgroup:
// a DPP scan within each wave, one wave scans the wave totals -- two
// barriers (an LDS Hillis-Steele scan over 256 slots takes 16).  sh: NT / 64
// ints of LDS.  Every thread must call it.
template <int NT, bool MAX>
__device__ __forceinline__ int32_t block_incl_scan(int32_t v, int32_t* sh) {
    static_assert(NT % 64 == 0 && NT / 64 <= 64, "whole waves, at most 64");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int32_t x = wave_incl_scan<MAX>(v);
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    if (wave == 0) {
        int32_t w = lane < NT / 64 ? sh[lane] : (MAX ? INT32_MIN : 0);
        w = wave_incl_scan<MAX>(w, NT / 64);
        if (lane < NT / 64) sh[lane] = w;
    }
    __syncthreads();
    return wave ? (MAX ? max(x, sh[wave - 1]) : x + sh[wave - 1]) : x;
}

size_t scan_temp_bytes(int64_t n);
// out[i] = sum_{j<i} in[j] (exclusive); *total (device, may be null) = sum.
int exclusive_scan_i32(hipStream_t s, const int32_t* in, int32_t* out, int64_t n,
                       int32_t* total, void* temp);
// out[i] = max_{j<=i} in[j] (inclusive).
int inclusive_max_scan_i32(hipStream_t s, const int32_t* in, int32_t* out, int64_t n,
                           void* temp);

// Stable lexicographic sort of rows by wvalues with caller buffers; nlex
// (default: all) sorts by the first nlex objectives only.
int lex_sort_rows(hipStream_t s, const double* wv, int nobj, int64_t n, bool desc, uint64_t* keys,
                  uint64_t* ktmp, int32_t* vals, int32_t* vtmp, void* rtemp, int nlex = -1,
                  int begin_bit = 0);

}  // namespace dm
