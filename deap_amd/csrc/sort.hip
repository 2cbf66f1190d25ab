// sort.hip — stable LSD radix sort + scans (see sort.hpp), and the selBest /
// selWorst entry points (deap/tools/selection.py:27-48) built on them.
#include "sort.hpp"

namespace dm {

// One-sweep LSD radix sort (8-bit digits).  Per sort: one memset (global
// digit histograms + look-back status), one histogram launch for all passes,
// then ONE launch per pass: each 1,024-key tile ranks its keys stably (wave
// ballots over the 8 bit-planes of the digit, per-(round, wave) digit counts
// in LDS), publishes its digit counts and finds the counts of all earlier
// tiles by decoupled look-back (thread d follows digit d), then scatters.
constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 4;                       // rounds of 256 keys per tile
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;    // 1,024 keys per tile
constexpr int RS_BINS = 256;
constexpr int RS_MAX_PASSES = 8;
constexpr int RS_HIST_BLOCKS = 512;

// temp layout: global digit histograms | one tile-id counter per pass |
// look-back status words
constexpr size_t RS_GHIST_BYTES = (RS_MAX_PASSES * RS_BINS * 4 + 255) / 256 * 256;
constexpr size_t RS_TICKET_BYTES = 256;

size_t radix_sort_batched_temp_bytes(int64_t nseg, int64_t seglen) {
    const int64_t tiles = nseg * ((seglen + RS_TILE - 1) / RS_TILE);
    return (size_t)nseg * RS_GHIST_BYTES + RS_TICKET_BYTES +
           align_up((size_t)tiles * RS_MAX_PASSES * RS_BINS * 4, 256);
}
size_t radix_sort_temp_bytes(int64_t n) { return radix_sort_batched_temp_bytes(1, n); }

// ghist[p][d] += count of digit d of pass p (shift begin + 8p); segment
// blockIdx.y of the batch: keys + y seglen, histograms + y RS_GHIST_BYTES
__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const uint64_t* __restrict__ keys,
                                                             int64_t n, int begin, int passes,
                                                             int32_t* __restrict__ ghist) {
    keys += (int64_t)blockIdx.y * n;
    ghist += (int64_t)blockIdx.y * (RS_GHIST_BYTES / 4);
    __shared__ int32_t h[RS_MAX_PASSES][RS_BINS];
    for (int p = 0; p < passes; ++p) h[p][threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * RS_THREADS + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * RS_THREADS) {
        const uint64_t k = keys[i] >> begin;
        for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 0xFF], 1);
    }
    __syncthreads();
    for (int p = 0; p < passes; ++p) {
        const int32_t c = h[p][threadIdx.x];
        if (c) atomicAdd(&ghist[p * RS_BINS + threadIdx.x], c);
    }
}

// look-back status word of (tile, digit): flag (1 = tile count, 2 = inclusive
// prefix) in bits 30-31, the count below
constexpr uint32_t RS_AGG = 1u << 30, RS_PREFIX = 2u << 30, RS_COUNT = (1u << 30) - 1;

// A batch of independent segments of `seglen` keys (tps tiles each) sorts in
// the same launches: a tile's digit offsets, look-back and output stay
// inside its segment.  One segment: seglen = n.
__global__ __launch_bounds__(RS_THREADS) void rs_pass_kernel(
    const uint64_t* __restrict__ keys_in, const int32_t* __restrict__ vals_in,
    uint64_t* __restrict__ keys_out, int32_t* __restrict__ vals_out, int64_t seglen, int64_t tps,
    int shift, const int32_t* __restrict__ ghist, uint32_t* status, uint32_t* ticket,
    const uint8_t* __restrict__ dig = nullptr) {
    __shared__ int32_t cnt[RS_ROUNDS][RS_THREADS / 64][RS_BINS];
    __shared__ int32_t gofs[RS_BINS];
    __shared__ uint32_t tile_id;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // tile ids in the order workgroups START (an atomic ticket, not blockIdx):
    // every tile a workgroup waits on in the look-back below is then already
    // running, whatever order the dispatcher launches workgroups in
    if (tid == 0) tile_id = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t tile = tile_id;
    const int64_t seg = tile / tps, lt = tile - seg * tps;  // segment, tile within it
    const int64_t sbase = seg * seglen;
    const int64_t base = sbase + lt * RS_TILE;
    const int64_t n = sbase + seglen;  // end of the segment
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r)
#pragma unroll
        for (int w = 0; w < RS_THREADS / 64; ++w) cnt[r][w][tid] = 0;
    // exclusive scan of the global digit histogram (thread d -> digit d)
    gofs[tid] = ghist[seg * (RS_GHIST_BYTES / 4) + tid];
    __syncthreads();
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint64_t k[RS_ROUNDS];
    int32_t v[RS_ROUNDS];
    int d[RS_ROUNDS], rk[RS_ROUNDS];
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const int64_t i = base + r * RS_THREADS + tid;
        const bool ok = i < n;
        k[r] = ok ? keys_in[i] : 0;
        v[r] = ok ? vals_in[i] : 0;
        // dig (sample sort): the digit is the key's bucket, stored by ss_classify_kernel
        d[r] = ok ? (dig ? (int)dig[i] : (int)((k[r] >> shift) & 0xFF)) : -1;
    }
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const bool ok = d[r] >= 0;
        uint64_t same = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t plane = __ballot(ok && ((d[r] >> b) & 1));
            same &= ((d[r] >> b) & 1) ? plane : ~plane;
        }
        rk[r] = __popcll(same & below);
        if (ok && rk[r] == 0) cnt[r][wave][d[r]] = __popcll(same);
    }
    static_assert(RS_BINS == RS_THREADS, "thread d owns digit d");
    __shared__ int32_t wsum[RS_THREADS / 64];
    // global exclusive offset of digit tid (the scan's barriers also order
    // the per-(round, wave) counts above before the offsets below)
    const int32_t gx = gofs[tid];
    const int32_t gex = block_incl_scan<RS_THREADS, false>(gx, wsum) - gx;
    // tile-local exclusive offsets per (round, wave) in key order; tile total
    int32_t run = 0;
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r)
#pragma unroll
        for (int w = 0; w < RS_THREADS / 64; ++w) {
            const int32_t c = cnt[r][w][tid];
            cnt[r][w][tid] = run;
            run += c;
        }
    // decoupled look-back over the earlier tiles for digit tid
    uint32_t* my = status + tile * RS_BINS + tid;
    int32_t excl = 0;
    if (lt == 0) {
        __hip_atomic_store(my, RS_PREFIX | (uint32_t)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(my, RS_AGG | (uint32_t)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int64_t t = tile - 1; t >= seg * tps;) {
            const uint32_t st = __hip_atomic_load(status + t * RS_BINS + tid, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            if (st == 0) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += (int32_t)(st & RS_COUNT);
            if (st & RS_PREFIX) break;
            --t;
        }
        __hip_atomic_store(my, RS_PREFIX | (uint32_t)(excl + run), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    gofs[tid] = gex + excl;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        if (d[r] >= 0) {
            const int64_t pos = sbase + gofs[d[r]] + cnt[r][wave][d[r]] + rk[r];
            keys_out[pos] = k[r];
            vals_out[pos] = v[r];
        }
    }
}

// ---------------------------------------------------------------------------
// Small and mid-size sorts.  The one-sweep pass above costs a launch per 8-bit
// digit whatever n is, and at the sizes NSGA-II sorts (a last front of a few
// thousand, 2^18 objective values) a pass is latency, not bytes: 17-21 us per
// pass of 2^18 keys, 8 passes per 64-bit key (profiles/r05fin4).
//  - seglen <= LS_CAP: one workgroup per segment sorts the pairs in LDS
//    (lds_radix below) -- one launch.
//  - SS_MIN <= seglen <= SS_MAX with at least SS_MIN_PASSES digits: sample
//    sort.  255 splitters per segment from a sorted jittered-regular sample
//    of (key bits, position) pairs; a classify pass stores each key's bucket
//    byte and histograms the buckets; ONE one-sweep pass (rs_pass_kernel on
//    the bytes) scatters the pairs into bucket order, stably; one workgroup
//    per bucket sorts it in LDS, stably (lds_radix).  The splitters carry
//    the position, so equal keys spread over buckets and every pair is
//    distinct: the result is exactly the stable order.  A bucket larger than
//    LS_CAP (a sample that missed a cluster) is sorted by a workgroup-local
//    LSD radix sort through global memory instead: slower, same result.
// Five launches (memset, splitters, classify, scatter, buckets) instead of ten.
// ---------------------------------------------------------------------------
constexpr int LS_THREADS = 1024;
constexpr int LS_WAVES = LS_THREADS / 64;
constexpr int LS_CAP = LDS_SORT_CAP;  // pairs one workgroup sorts in LDS
constexpr int SS_SAMPLE = 4096;    // sample per segment (16 per bucket)
constexpr int SS_BUCKETS = 256;    // = RS_BINS: the bucket is the scatter digit
constexpr int64_t SS_MIN = 1 << 16;  // below, its fixed ~90 us (splitter + bucket sorts) loses to radix
constexpr int64_t SS_MAX = 1 << 19;
constexpr int SS_MIN_PASSES = 5;
static_assert(SS_SAMPLE <= LS_CAP, "the sample is sorted in LDS");

// the bits [begin, begin + width) of a key that the sort compares
template <bool FULL>
__device__ __forceinline__ uint64_t kbits(uint64_t k, int begin, uint64_t mask) {
    return FULL ? k : (k >> begin) & mask;
}

// A workgroup's LSD radix sort in LDS: n <= LS_CAP (key, index) pairs in
// k[0] / i[0], 8-bit digits.  Wave w owns the contiguous elements [w chunk,
// (w + 1) chunk) in rounds of 64; a digit's rank inside a round is a ballot
// match over the 8 bit planes (as in rs_pass_kernel) plus the wave's running
// count of that digit; one thread per digit turns the per-wave counts into
// offsets; the scatter goes to the other buffer.  Stable, ~5 barriers per
// digit.  (A bitonic network over the same LDS arrays ran 52-104 us for
// 4,096 pairs -- 78 stages of LDS-bandwidth-bound compare-exchanges; r05_ssort.)
struct LdsRadix {
    using Key = uint64_t;
    using Idx = uint32_t;
    static constexpr int cap = LS_CAP;
    uint64_t k[2][LS_CAP];
    uint32_t i[2][LS_CAP];
    int32_t wc[LS_WAVES][RS_BINS];  // per-wave digit counts -> offsets
    int32_t wsum[LS_WAVES];
    int32_t same;                   // the pass's digit is one value: no scatter
};
// keys of at most 32 bits: twice the pairs in the same LDS (with the values,
// 144 KiB for 8,192) -- the crowding distance's per-front rank sorts
constexpr int LS_CAP32 = LDS_SORT_CAP32;
struct LdsRadix32 {
    using Key = uint32_t;
    using Idx = uint16_t;
    static constexpr int cap = LS_CAP32;
    uint32_t k[2][LS_CAP32];
    uint16_t i[2][LS_CAP32];
    int32_t wc[LS_WAVES][RS_BINS];
    int32_t wsum[LS_WAVES];
    int32_t same;
};

// the digit passes the n pairs in k[0] need: the high digits their minimum
// and maximum share are constant in all of them (LSD: only the low digits
// below run); one workgroup-wide min / max in LDS
template <bool FULL, class LR>
__device__ __forceinline__ int lds_passes_needed(LR& L, int n, int begin, uint64_t mask,
                                                 int passes) {
    __shared__ unsigned long long mn, mx;
    if (threadIdx.x == 0) {
        mn = ~0ull;
        mx = 0ull;
    }
    __syncthreads();
    uint64_t a = ~0ull, z = 0ull;
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        const uint64_t b = kbits<FULL>(L.k[0][i], begin, mask);
        a = b < a ? b : a;
        z = b > z ? b : z;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a2 = __shfl_xor(a, o, 64), z2 = __shfl_xor(z, o, 64);
        a = a2 < a ? a2 : a;
        z = z2 > z ? z2 : z;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mn, (unsigned long long)a);
        atomicMax(&mx, (unsigned long long)z);
    }
    __syncthreads();
    const uint64_t d = (uint64_t)mn ^ (uint64_t)mx;
    const int vary = d == 0 ? 0 : 64 - __clzll((long long)d);
    return min(passes, (vary + 7) / 8);
}

// returns the buffer (0 or 1) holding the sorted pairs
template <bool FULL, class LR>
__device__ __forceinline__ int lds_radix(LR& L, int n, int begin, uint64_t mask, int passes) {
    constexpr int PER = LR::cap / LS_THREADS;  // rounds per wave at most
    using Key = typename LR::Key;
    using Idx = typename LR::Idx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int chunk = (n + LS_THREADS - 1) / LS_THREADS * 64;  // per wave, whole rounds
    const int rounds = chunk / 64;                             // <= PER
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int cur = 0;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        for (int q = lane; q < RS_BINS; q += 64) L.wc[wave][q] = 0;
        if (tid == 0) L.same = 0;
        Key kk[PER];
        Idx ii[PER];
        int dd[PER], rr[PER];
#pragma unroll
        for (int r = 0; r < PER; ++r) {
            dd[r] = -1;
            if (r < rounds) {  // wave-uniform
                const int e = wave * chunk + r * 64 + lane;
                const bool ok = e < n;
                kk[r] = ok ? L.k[cur][e] : 0;
                ii[r] = ok ? L.i[cur][e] : 0;
                const int d = ok ? (int)((kbits<FULL>(kk[r], begin, mask) >> shift) & 0xFF) : -1;
                uint64_t same = __ballot(ok);
#pragma unroll
                for (int bit = 0; bit < 8; ++bit) {
                    const uint64_t plane = __ballot(ok && ((d >> bit) & 1));
                    same &= ((d >> bit) & 1) ? plane : ~plane;
                }
                const int rk = __popcll(same & below);
                // in-order LDS within the wave: every lane reads the running
                // count before the digit's first lane advances it
                const int base = ok ? L.wc[wave][d] : 0;
                if (ok && rk == 0) L.wc[wave][d] = base + __popcll(same);
                dd[r] = d;
                rr[r] = base + rk;
            }
        }
        __syncthreads();
        int32_t tot = 0;
        if (tid < RS_BINS)
#pragma unroll
            for (int w = 0; w < LS_WAVES; ++w) {
                const int32_t c = L.wc[w][tid];
                L.wc[w][tid] = tot;
                tot += c;
            }
        const int32_t ex = block_incl_scan<LS_THREADS, false>(tid < RS_BINS ? tot : 0, L.wsum) - tot;
        if (tid < RS_BINS) {
#pragma unroll
            for (int w = 0; w < LS_WAVES; ++w) L.wc[w][tid] += ex;
            if (tot == n) L.same = 1;
        }
        __syncthreads();
        if (!L.same) {  // workgroup-uniform
#pragma unroll
            for (int r = 0; r < PER; ++r)
                if (dd[r] >= 0) {
                    const int pos = L.wc[wave][dd[r]] + rr[r];
                    L.k[cur ^ 1][pos] = kk[r];
                    L.i[cur ^ 1][pos] = ii[r];
                }
            cur ^= 1;
        }
        __syncthreads();
    }
    return cur;
}

// A workgroup's stable LSD radix sort of cnt pairs through global memory
// (src <-> dst at the same offsets; the sorted pairs end in dst): chunks of
// LS_THREADS pairs ranked by wave ballots as in rs_pass_kernel.  The sample
// sort's fallback for a bucket its sample missed, and the segmented LDS sorts'
// for a segment over their capacity (slower, same result: never a silently
// unsorted tail).  L's per-wave counts and index array are its LDS scratch.
template <bool FULL, class LR>
__device__ __noinline__ void wg_global_radix(LR& L, int32_t* dbase, uint64_t* __restrict__ ksrc,
                                             int32_t* __restrict__ vsrc, uint64_t* __restrict__ kdst,
                                             int32_t* __restrict__ vdst, int cnt, int begin,
                                             uint64_t mask, int passes) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint64_t* kin = ksrc;
    int32_t* vin = vsrc;
    uint64_t* kout = kdst;
    int32_t* vout = vdst;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        if (tid < RS_BINS) dbase[tid] = 0;
        __syncthreads();
        for (int i = tid; i < cnt; i += LS_THREADS)
            atomicAdd(&dbase[(kbits<FULL>(kin[i], begin, mask) >> shift) & 0xFF], 1);
        __syncthreads();
        if (wave == 0) {  // exclusive scan of the 256 digit counts, 4 per lane
            int32_t c[4], run = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = dbase[lane * 4 + q];
                run += c[q];
            }
            int32_t x = run;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            int32_t e = x - run;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                dbase[lane * 4 + q] = e;
                e += c[q];
            }
        }
        __syncthreads();
        for (int c0 = 0; c0 < cnt; c0 += LS_THREADS) {
            const int i = c0 + tid;
            const bool ok = i < cnt;
            const uint64_t k = ok ? kin[i] : 0;
            const int32_t val = ok ? vin[i] : 0;
            const int d = ok ? (int)((kbits<FULL>(k, begin, mask) >> shift) & 0xFF) : -1;
            uint64_t same = __ballot(ok);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit) {
                const uint64_t plane = __ballot(ok && ((d >> bit) & 1));
                same &= ((d >> bit) & 1) ? plane : ~plane;
            }
            const int rk = __popcll(same & below);
            for (int q = lane; q < RS_BINS; q += 64) L.wc[wave][q] = 0;
            __syncthreads();
            if (ok && rk == 0) L.wc[wave][d] = __popcll(same);
            __syncthreads();
            if (tid < RS_BINS) {  // digit tid: waves' exclusive offsets, the chunk's total
                int32_t run = 0;
#pragma unroll
                for (int w = 0; w < LS_WAVES; ++w) {
                    const int32_t t = L.wc[w][tid];
                    L.wc[w][tid] = run;
                    run += t;
                }
                L.i[0][tid] = (typename LR::Idx)run;
            }
            __syncthreads();
            if (ok) {
                const int pos = dbase[d] + L.wc[wave][d] + rk;
                kout[pos] = k;
                vout[pos] = val;
            }
            __syncthreads();
            if (tid < RS_BINS) dbase[tid] += (int32_t)L.i[0][tid];
            __syncthreads();
        }
        uint64_t* kt = kin;
        kin = kout;
        kout = kt;
        int32_t* vt = vin;
        vin = vout;
        vout = vt;
        __syncthreads();
    }
    if ((passes & 1) == 0) {  // the result is back in src
        for (int i = tid; i < cnt; i += LS_THREADS) {
            kdst[i] = ksrc[i];
            vdst[i] = vsrc[i];
        }
    }
}

// a segment over the LDS sorts' capacity: sorted in global memory through
// the tmp buffers (at the segment's offset), the result copied back; no tmp
// buffers: flagged, left as it is
template <bool FULL, class LR>
__device__ __forceinline__ void seg_oversize(LR& L, int32_t* dbase, uint64_t* k, int32_t* v,
                                             uint64_t* ktmp, int32_t* vtmp, int64_t base, int n,
                                             int begin, uint64_t mask, int passes,
                                             int32_t* oversize) {
    if (!ktmp || !vtmp) {
        if (threadIdx.x == 0 && oversize) atomicMax(oversize, n);
        return;
    }
    wg_global_radix<FULL>(L, dbase, k, v, ktmp + base, vtmp + base, n, begin, mask, passes);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        k[i] = ktmp[base + i];
        v[i] = vtmp[base + i];
    }
}

// one workgroup per segment of at most LS_CAP pairs, sorted in place: segment
// g is [g seglen, (g + 1) seglen), or [starts[g], starts[g + 1]) with starts.
// A variable segment over LS_CAP pairs (the caller's bound on it was wrong)
// is sorted through ktmp / vtmp (same offsets) by wg_global_radix: slower,
// never a silently unsorted tail; without tmp buffers it is left unsorted
// and *oversize is set (the callers pass the buffers).
template <bool FULL>
__global__ __launch_bounds__(LS_THREADS) void ls_sort_kernel(uint64_t* __restrict__ keys,
                                                             int32_t* __restrict__ vals,
                                                             int64_t seglen, int begin,
                                                             uint64_t mask, int passes,
                                                             const int32_t* __restrict__ starts,
                                                             uint64_t* __restrict__ ktmp = nullptr,
                                                             int32_t* __restrict__ vtmp = nullptr,
                                                             int32_t* __restrict__ oversize = nullptr) {
    __shared__ LdsRadix L;
    __shared__ int32_t sv[LS_CAP];
    __shared__ int32_t dbase[RS_BINS];
    const int64_t base = starts ? (int64_t)starts[blockIdx.x] : (int64_t)blockIdx.x * seglen;
    const int n = starts ? starts[blockIdx.x + 1] - starts[blockIdx.x] : (int)seglen;
    if (n <= 1) return;  // workgroup-uniform
    if (n > LS_CAP) {
        seg_oversize<FULL>(L, dbase, keys + base, vals + base, ktmp, vtmp, base, n, begin, mask,
                           passes, oversize);
        return;
    }
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        L.k[0][i] = keys[base + i];
        L.i[0][i] = (uint32_t)i;
        sv[i] = vals[base + i];
    }
    __syncthreads();
    passes = lds_passes_needed<FULL>(L, n, begin, mask, passes);
    const int c = lds_radix<FULL>(L, n, begin, mask, passes);
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        keys[base + i] = L.k[c][i];
        vals[base + i] = sv[L.i[c][i]];
    }
}

// ls_sort_kernel for keys of at most 32 bits (< 2^32; sorted by bits [0,
// width)) over segments [starts[g], starts[g + 1]) of at most LS_CAP32 pairs
// (larger ones as in ls_sort_kernel)
__global__ __launch_bounds__(LS_THREADS) void ls_sort32_kernel(uint64_t* __restrict__ keys,
                                                               int32_t* __restrict__ vals,
                                                               uint64_t mask, int passes,
                                                               const int32_t* __restrict__ starts,
                                                               uint64_t* __restrict__ ktmp,
                                                               int32_t* __restrict__ vtmp,
                                                               int32_t* __restrict__ oversize) {
    __shared__ LdsRadix32 L;
    __shared__ int32_t sv[LS_CAP32];
    __shared__ int32_t dbase[RS_BINS];
    const int64_t base = starts[blockIdx.x];
    const int n = starts[blockIdx.x + 1] - starts[blockIdx.x];
    if (n <= 1) return;  // workgroup-uniform
    if (n > LS_CAP32) {
        seg_oversize<false>(L, dbase, keys + base, vals + base, ktmp, vtmp, base, n, 0, mask,
                            passes, oversize);
        return;
    }
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        L.k[0][i] = (uint32_t)keys[base + i];
        L.i[0][i] = (uint16_t)i;
        sv[i] = vals[base + i];
    }
    __syncthreads();
    passes = lds_passes_needed<false>(L, n, 0, mask, passes);
    const int c = lds_radix<false>(L, n, 0, mask, passes);
    for (int i = threadIdx.x; i < n; i += LS_THREADS) {
        keys[base + i] = L.k[c][i];
        vals[base + i] = sv[L.i[c][i]];
    }
}

// splitters of segment blockIdx.x: a jittered regular sample of (bits,
// position) pairs, sorted (stable by bits = by (bits, position): the sample
// positions ascend); splitter j = sample (j + 1) * 16 (j < 255)
template <bool FULL>
__global__ __launch_bounds__(LS_THREADS) void ss_splitter_kernel(const uint64_t* __restrict__ keys,
                                                                 int64_t seglen, int begin,
                                                                 uint64_t mask, int passes,
                                                                 uint64_t* __restrict__ spk,
                                                                 uint32_t* __restrict__ spp) {
    __shared__ LdsRadix L;
    const int64_t base = (int64_t)blockIdx.x * seglen;
    const int64_t stride = seglen / SS_SAMPLE;  // >= 16: seglen >= SS_MIN
    for (int i = threadIdx.x; i < SS_SAMPLE; i += LS_THREADS) {
        const uint32_t h = (uint32_t)i * 2654435761u;
        const int64_t p = (int64_t)i * stride + (int64_t)((h >> 8) % (uint32_t)stride);
        L.k[0][i] = kbits<FULL>(keys[base + p], begin, mask);
        L.i[0][i] = (uint32_t)p;
    }
    __syncthreads();
    passes = lds_passes_needed<true>(L, SS_SAMPLE, 0, ~0ull, passes);
    const int c = lds_radix<true>(L, SS_SAMPLE, 0, ~0ull, passes);
    constexpr int per = SS_SAMPLE / SS_BUCKETS;
    if (threadIdx.x < SS_BUCKETS - 1) {
        spk[(int64_t)blockIdx.x * SS_BUCKETS + threadIdx.x] = L.k[c][(threadIdx.x + 1) * per];
        spp[(int64_t)blockIdx.x * SS_BUCKETS + threadIdx.x] = L.i[c][(threadIdx.x + 1) * per];
    }
}

// bucket of every key (the number of splitters below its (bits, position)
// pair) -> dig, and the segment's bucket histogram -> ghist (pass-0 row)
template <bool FULL>
__global__ __launch_bounds__(RS_THREADS) void ss_classify_kernel(
    const uint64_t* __restrict__ keys, int64_t seglen, int64_t tps, int begin, uint64_t mask,
    const uint64_t* __restrict__ spk, const uint32_t* __restrict__ spp, uint8_t* __restrict__ dig,
    int32_t* __restrict__ ghist) {
    __shared__ uint64_t sk[SS_BUCKETS];
    __shared__ uint32_t sp[SS_BUCKETS];
    __shared__ int32_t h[SS_BUCKETS];
    static_assert(SS_BUCKETS == RS_THREADS, "thread b loads splitter b");
    const int tid = threadIdx.x;
    const int64_t seg = blockIdx.x / tps, lt = blockIdx.x - seg * tps;
    if (tid < SS_BUCKETS - 1) {
        sk[tid] = spk[seg * SS_BUCKETS + tid];
        sp[tid] = spp[seg * SS_BUCKETS + tid];
    }
    h[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
        const int64_t p = lt * RS_TILE + r * RS_THREADS + tid;
        if (p < seglen) {
            const uint64_t b = kbits<FULL>(keys[seg * seglen + p], begin, mask);
            int lo = 0, hi = SS_BUCKETS - 1;  // lower bound over the 255 splitters
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                const bool below = sk[mid] < b || (sk[mid] == b && sp[mid] < (uint32_t)p);
                if (below) lo = mid + 1;
                else hi = mid;
            }
            dig[seg * seglen + p] = (uint8_t)lo;
            atomicAdd(&h[lo], 1);
        }
    }
    __syncthreads();
    if (h[tid]) atomicAdd(&ghist[seg * (RS_GHIST_BYTES / 4) + tid], h[tid]);
}

// bucket (blockIdx.x % 256) of segment (blockIdx.x / 256): its pairs, in input
// order at [start, start + cnt) of ksrc / vsrc, sorted into kdst / vdst
template <bool FULL>
__global__ __launch_bounds__(LS_THREADS) void ss_bucket_kernel(
    uint64_t* __restrict__ ksrc, int32_t* __restrict__ vsrc, uint64_t* __restrict__ kdst,
    int32_t* __restrict__ vdst, int64_t seglen, int begin, uint64_t mask, int passes,
    const int32_t* __restrict__ ghist, const uint64_t* __restrict__ spk) {
    __shared__ LdsRadix L;
    __shared__ int32_t dbase[RS_BINS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t seg = blockIdx.x / SS_BUCKETS;
    const int b = (int)(blockIdx.x % SS_BUCKETS);
    const int32_t* gh = ghist + seg * (RS_GHIST_BYTES / 4);
    // start = the counts of the buckets before b
    int32_t v = tid < b ? gh[tid] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) L.wsum[wave] = v;
    __syncthreads();
    int32_t start = 0;
#pragma unroll
    for (int w = 0; w < LS_WAVES; ++w) start += L.wsum[w];
    const int cnt = gh[b];
    const int64_t off = seg * seglen + start;
    // the bucket's keys lie between its two splitters: the high digits the
    // splitters share are constant in it, only the digits below need passes
    // (a bucket of 1/256 of a 2^18 key range: 5-6 of 8)
    {
        const uint64_t lo = b > 0 ? spk[seg * SS_BUCKETS + b - 1] : 0ull;
        const uint64_t hi = b < SS_BUCKETS - 1 ? spk[seg * SS_BUCKETS + b] : ~0ull;
        const int vary = lo == hi ? 0 : 64 - __clzll((long long)(lo ^ hi));
        passes = min(passes, (vary + 7) / 8);
    }
    if (cnt <= 1 || passes == 0) {  // one pair, or one key value: input order is the order
        for (int i = tid; i < cnt; i += LS_THREADS) {
            kdst[off + i] = ksrc[off + i];
            vdst[off + i] = vsrc[off + i];
        }
        return;
    }
    if (cnt <= LS_CAP) {
        for (int i = tid; i < cnt; i += LS_THREADS) {
            L.k[0][i] = ksrc[off + i];
            L.i[0][i] = (uint32_t)i;
        }
        __syncthreads();
        const int c = lds_radix<FULL>(L, cnt, begin, mask, passes);
        for (int i = tid; i < cnt; i += LS_THREADS) {
            kdst[off + i] = L.k[c][i];
            vdst[off + i] = vsrc[off + L.i[c][i]];
        }
        return;
    }
    // fallback: the bucket is larger than LS_CAP (a sample that missed a cluster)
    wg_global_radix<FULL>(L, dbase, ksrc + off, vsrc + off, kdst + off, vdst + off, cnt, begin,
                          mask, passes);
}

int radix_sort_pairs_batched(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                             int32_t* vals_tmp, int64_t nseg, int64_t seglen, int begin_bit,
                             int end_bit, void* temp, bool* in_tmp) {
    if (in_tmp) *in_tmp = false;
    if (nseg <= 0 || seglen <= 1 || end_bit <= begin_bit) return DM_OK;
    const int64_t n = nseg * seglen;
    DM_CHECK_ARG(n < (1ll << 30), "radix sort of more than 2^30 keys");
    DM_CHECK_ARG(nseg <= 65535, "radix sort of more than 65,535 segments");
    const int64_t tps = (seglen + RS_TILE - 1) / RS_TILE;
    const int64_t tiles = nseg * tps;
    const int passes = std::min(RS_MAX_PASSES, (end_bit - begin_bit + 7) / 8);
    int32_t* ghist = (int32_t*)temp;
    uint32_t* ticket = (uint32_t*)((char*)temp + nseg * RS_GHIST_BYTES);
    uint32_t* status = (uint32_t*)((char*)temp + nseg * RS_GHIST_BYTES + RS_TICKET_BYTES);
    const int width = std::min(64, end_bit - begin_bit);
    const bool full = begin_bit == 0 && width == 64;
    const uint64_t mask = width == 64 ? ~0ull : ((1ull << width) - 1);
    if (seglen <= LS_CAP) {
        if (full)
            ls_sort_kernel<true><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, vals, seglen, 0, mask,
                                                                     passes, nullptr);
        else
            ls_sort_kernel<false><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, vals, seglen,
                                                                      begin_bit, mask, passes,
                                                                      nullptr);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    if (passes >= SS_MIN_PASSES && seglen >= SS_MIN && seglen <= SS_MAX) {
        // temp: ghist | ticket | one pass of look-back status | bucket bytes | splitters
        // (within radix_sort_batched_temp_bytes: tiles * 8 KB covers them)
        uint8_t* dig = (uint8_t*)status + align_up((size_t)tiles * RS_BINS * 4, 256);
        uint64_t* spk = (uint64_t*)(dig + align_up((size_t)n, 256));
        uint32_t* spp = (uint32_t*)(spk + nseg * SS_BUCKETS);
        DM_HIP(hipMemsetAsync(temp, 0,
                              nseg * RS_GHIST_BYTES + RS_TICKET_BYTES + (size_t)tiles * RS_BINS * 4,
                              s));
        if (full) {
            ss_splitter_kernel<true><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, seglen, 0, mask,
                                                                           passes, spk, spp);
            ss_classify_kernel<true><<<(unsigned)tiles, RS_THREADS, 0, s>>>(
                keys, seglen, tps, 0, mask, spk, spp, dig, ghist);
        } else {
            ss_splitter_kernel<false><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, seglen, begin_bit,
                                                                            mask, passes, spk, spp);
            ss_classify_kernel<false><<<(unsigned)tiles, RS_THREADS, 0, s>>>(
                keys, seglen, tps, begin_bit, mask, spk, spp, dig, ghist);
        }
        rs_pass_kernel<<<(unsigned)tiles, RS_THREADS, 0, s>>>(keys, vals, keys_tmp, vals_tmp, seglen,
                                                             tps, 0, ghist, status, ticket, dig);
        const unsigned nb = (unsigned)(nseg * SS_BUCKETS);
        if (full)
            ss_bucket_kernel<true><<<nb, LS_THREADS, 0, s>>>(keys_tmp, vals_tmp, keys, vals, seglen,
                                                             0, mask, passes, ghist, spk);
        else
            ss_bucket_kernel<false><<<nb, LS_THREADS, 0, s>>>(keys_tmp, vals_tmp, keys, vals, seglen,
                                                              begin_bit, mask, passes, ghist, spk);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    DM_HIP(hipMemsetAsync(temp, 0,
                          nseg * RS_GHIST_BYTES + RS_TICKET_BYTES +
                              (size_t)passes * tiles * RS_BINS * 4,
                          s));
    const unsigned hb = (unsigned)std::min<int64_t>(
        RS_HIST_BLOCKS, (seglen + RS_THREADS * 8 - 1) / (RS_THREADS * 8));
    rs_hist_kernel<<<dim3(hb, (unsigned)nseg), RS_THREADS, 0, s>>>(keys, seglen, begin_bit, passes,
                                                                   ghist);
    uint64_t* kin = keys;
    int32_t* vin = vals;
    uint64_t* kout = keys_tmp;
    int32_t* vout = vals_tmp;
    for (int p = 0; p < passes; ++p) {
        rs_pass_kernel<<<(unsigned)tiles, RS_THREADS, 0, s>>>(kin, vin, kout, vout, seglen, tps,
                                                             begin_bit + 8 * p, ghist + p * RS_BINS,
                                                             status + (size_t)p * tiles * RS_BINS,
                                                             ticket + p);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    if ((passes & 1) && in_tmp) {
        *in_tmp = true;  // the caller takes the result from the tmp buffers
    } else if (passes & 1) {
        DM_HIP(hipMemcpyAsync(keys, kin, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
        DM_HIP(hipMemcpyAsync(vals, vin, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int seg_sort_pairs_small(hipStream_t s, uint64_t* keys, int32_t* vals, const int32_t* starts,
                         int64_t nseg, int begin_bit, int end_bit, uint64_t* keys_tmp,
                         int32_t* vals_tmp) {
    if (nseg <= 0 || end_bit <= begin_bit) return DM_OK;
    DM_CHECK_ARG(nseg <= (1ll << 31) - 1, "too many segments");
    const int width = std::min(64, end_bit - begin_bit);
    const int passes = std::min(RS_MAX_PASSES, (width + 7) / 8);
    const uint64_t mask = width == 64 ? ~0ull : ((1ull << width) - 1);
    if (begin_bit == 0 && width <= 32)
        ls_sort32_kernel<<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, vals, mask, passes, starts,
                                                               keys_tmp, vals_tmp, nullptr);
    else if (begin_bit == 0 && width == 64)
        ls_sort_kernel<true><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, vals, 0, 0, mask, passes,
                                                                 starts, keys_tmp, vals_tmp);
    else
        ls_sort_kernel<false><<<(unsigned)nseg, LS_THREADS, 0, s>>>(keys, vals, 0, begin_bit, mask,
                                                                  passes, starts, keys_tmp, vals_tmp);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int radix_sort_pairs(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                     int32_t* vals_tmp, int64_t n, int begin_bit, int end_bit, void* temp) {
    return radix_sort_pairs_batched(s, keys, vals, keys_tmp, vals_tmp, 1, n, begin_bit, end_bit,
                                    temp, nullptr);
}
int radix_sort_pairs_any(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* keys_tmp,
                         int32_t* vals_tmp, int64_t n, int begin_bit, int end_bit, void* temp,
                         bool* in_tmp) {
    return radix_sort_pairs_batched(s, keys, vals, keys_tmp, vals_tmp, 1, n, begin_bit, end_bit,
                                    temp, in_tmp);
}

// ---------------------------------------------------------------------------
// Scans: reduce-then-scan up to 4 Mi elements; beyond, block-local scan ->
// scan of block sums -> add back.
// ---------------------------------------------------------------------------
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 8;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

size_t scan_temp_bytes(int64_t n) {
    int64_t blocks = (n + SC_TILE - 1) / SC_TILE;
    size_t b = 0;
    while (blocks > 1) {
        b += align_up((size_t)blocks * 8, 256) * 2;
        blocks = (blocks + SC_TILE - 1) / SC_TILE;
    }
    return b + 512;
}

template <bool MAX>
__device__ __forceinline__ int32_t op2(int32_t a, int32_t b) {
    return MAX ? max(a, b) : a + b;
}

// Each block scans its tile; writes block aggregate.  INCL: inclusive.
template <bool MAX, bool INCL>
__global__ __launch_bounds__(SC_THREADS) void scan_tile_kernel(const int32_t* in, int32_t* out,
                                                               int64_t n, int32_t* block_sums) {
    __shared__ int32_t sh[SC_THREADS];
    const int64_t base = (int64_t)blockIdx.x * SC_TILE + (int64_t)threadIdx.x * SC_ITEMS;
    const int32_t ident = MAX ? INT32_MIN : 0;
    int32_t v[SC_ITEMS];
    int32_t acc = ident;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j;
        v[j] = i < n ? in[i] : ident;
        acc = op2<MAX>(acc, v[j]);
    }
    const int32_t incl = block_incl_scan<SC_THREADS, MAX>(acc, sh);
    // exclusive: the previous thread's inclusive value
    int32_t run = __shfl_up(incl, 1, 64);
    if ((threadIdx.x & 63) == 0) run = threadIdx.x > 0 ? sh[(threadIdx.x >> 6) - 1] : ident;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j;
        const int32_t nxt = op2<MAX>(run, v[j]);
        if (i < n) out[i] = INCL ? nxt : run;
        run = nxt;
    }
    if (threadIdx.x == SC_THREADS - 1 && block_sums) block_sums[blockIdx.x] = incl;
}

template <bool MAX>
__global__ void scan_add_kernel(int32_t* out, int64_t n, const int32_t* block_prefix) {
    const int64_t i = (int64_t)blockIdx.x * SC_TILE + (int64_t)threadIdx.x * SC_ITEMS;
    const int32_t p = block_prefix[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j)
        if (i + j < n) out[i + j] = op2<MAX>(out[i + j], p);
}

__global__ void scan_total_kernel(const int32_t* in, const int32_t* ex, int64_t n, int32_t* total) {
    *total = n > 0 ? ex[n - 1] + in[n - 1] : 0;
}

// Reduce-then-scan for up to SC_TILE tiles (n <= 4 Mi): block b's aggregate
// (scan_reduce_kernel), then every block combines the aggregates before it
// -- at most SC_DIRECT ints, from the L2 -- and scans its tile from that
// prefix (scan_down_kernel).  Two launches and no look-back, where the
// tile / block-sum / add-back form took three (four with the total).  Past
// SC_DIRECT tiles (1 Mi elements) that combination is O(blocks^2) L2 reads
// (ADVICE r5): one workgroup scans the aggregates first and each block reads
// its own prefix (three launches).
constexpr int64_t SC_DIRECT = 512;
template <bool MAX>
__device__ __forceinline__ int32_t sc_block_reduce(int32_t v, int32_t* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op2<MAX>(v, __shfl_xor(v, o, 64));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int32_t r = sh[0];
#pragma unroll
    for (int w = 1; w < SC_THREADS / 64; ++w) r = op2<MAX>(r, sh[w]);
    return r;
}
template <bool MAX>
__global__ __launch_bounds__(SC_THREADS) void scan_reduce_kernel(const int32_t* in, int64_t n,
                                                                 int32_t* sums) {
    __shared__ int32_t sh[SC_THREADS / 64];
    const int64_t base = (int64_t)blockIdx.x * SC_TILE + (int64_t)threadIdx.x * SC_ITEMS;
    int32_t acc = MAX ? INT32_MIN : 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j)
        if (base + j < n) acc = op2<MAX>(acc, in[base + j]);
    acc = sc_block_reduce<MAX>(acc, sh);
    if (threadIdx.x == 0) sums[blockIdx.x] = acc;
}
// total (may be null): the whole input's aggregate, from the last block
template <bool MAX, bool INCL>
__global__ __launch_bounds__(SC_THREADS) void scan_down_kernel(const int32_t* in, int32_t* out,
                                                               int64_t n, const int32_t* sums,
                                                               int32_t* total,
                                                               const int32_t* pref = nullptr) {
    __shared__ int32_t sh[SC_THREADS];
    __shared__ int32_t shr[SC_THREADS / 64];
    const int32_t ident = MAX ? INT32_MIN : 0;
    const int64_t base = (int64_t)blockIdx.x * SC_TILE + (int64_t)threadIdx.x * SC_ITEMS;
    int32_t v[SC_ITEMS];
    int32_t acc = ident;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j;
        v[j] = i < n ? in[i] : ident;
        acc = op2<MAX>(acc, v[j]);
    }
    int32_t p = ident;
    if (pref) {
        p = pref[blockIdx.x];  // the scanned aggregates (exclusive)
    } else {
        for (int64_t b = threadIdx.x; b < (int64_t)blockIdx.x; b += SC_THREADS)
            p = op2<MAX>(p, sums[b]);
        p = sc_block_reduce<MAX>(p, shr);
    }
    const int32_t incl = block_incl_scan<SC_THREADS, MAX>(acc, sh);
    int32_t run = __shfl_up(incl, 1, 64);
    if ((threadIdx.x & 63) == 0) run = threadIdx.x > 0 ? sh[(threadIdx.x >> 6) - 1] : ident;
    run = op2<MAX>(p, run);
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const int64_t i = base + j;
        const int32_t nxt = op2<MAX>(run, v[j]);
        if (i < n) out[i] = INCL ? nxt : run;
        run = nxt;
    }
    if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == SC_THREADS - 1) *total = run;
}

// total (may be null): the aggregate of the whole input, on the device
template <bool MAX, bool INCL>
static int scan_impl(hipStream_t s, const int32_t* in, int32_t* out, int64_t n, void* temp,
                     int32_t* total) {
    if (n <= 0) {
        if (total) DM_HIP(hipMemsetAsync(total, 0, 4, s));
        return DM_OK;
    }
    const int64_t blocks = (n + SC_TILE - 1) / SC_TILE;
    if (blocks == 1) {
        scan_tile_kernel<MAX, INCL><<<1, SC_THREADS, 0, s>>>(in, out, n, total);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    int32_t* sums = (int32_t*)temp;
    int32_t* pref = (int32_t*)((char*)temp + align_up((size_t)blocks * 8, 256));
    if (blocks <= SC_TILE) {
        scan_reduce_kernel<MAX><<<(unsigned)blocks, SC_THREADS, 0, s>>>(in, n, sums);
        if (blocks <= SC_DIRECT) {
            scan_down_kernel<MAX, INCL><<<(unsigned)blocks, SC_THREADS, 0, s>>>(in, out, n, sums,
                                                                                total);
        } else {
            scan_tile_kernel<MAX, false><<<1, SC_THREADS, 0, s>>>(sums, pref, blocks, nullptr);
            scan_down_kernel<MAX, INCL><<<(unsigned)blocks, SC_THREADS, 0, s>>>(in, out, n, sums,
                                                                                total, pref);
        }
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    void* next = (char*)temp + 2 * align_up((size_t)blocks * 8, 256);
    scan_tile_kernel<MAX, INCL><<<(unsigned)blocks, SC_THREADS, 0, s>>>(in, out, n, sums);
    // exclusive scan of block aggregates
    int rc = scan_impl<MAX, false>(s, sums, pref, blocks, next, nullptr);
    if (rc) return rc;
    scan_add_kernel<MAX><<<(unsigned)blocks, SC_THREADS, 0, s>>>(out, n, pref);
    if (total) {
        if (MAX) return DM_ERR_INVALID;  // no caller asks for the total of a max scan
        scan_total_kernel<<<1, 1, 0, s>>>(in, out, n, total);
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int exclusive_scan_i32(hipStream_t s, const int32_t* in, int32_t* out, int64_t n,
                       int32_t* total, void* temp) {
    return scan_impl<false, false>(s, in, out, n, temp, total);
}

int inclusive_max_scan_i32(hipStream_t s, const int32_t* in, int32_t* out, int64_t n,
                           void* temp) {
    return scan_impl<true, true>(s, in, out, n, temp, nullptr);
}

// ---------------------------------------------------------------------------
// selBest / selWorst: sorted(individuals, key=fitness, reverse=best)[:k]
// ---------------------------------------------------------------------------
__global__ void key_obj_kernel(const double* wv, int nobj, int obj, const int32_t* vals,
                               uint64_t* keys, int64_t n, bool desc) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = ordered_key(wv[(int64_t)vals[i] * nobj + obj]);
        keys[i] = desc ? ~k : k;
    }
}
// key_obj_kernel over the identity order, which it also writes to vals
__global__ void key_obj_iota_kernel(const double* wv, int nobj, int obj, int32_t* vals,
                                    uint64_t* keys, int64_t n, bool desc) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = ordered_key(wv[i * nobj + obj]);
        keys[i] = desc ? ~k : k;
        vals[i] = (int32_t)i;
    }
}
__global__ void iota_kernel(int32_t* v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (int32_t)i;
}

int validate_pop(const dm_pop* p, const char* what);

// Stable lexicographic sort of rows by wvalues (asc or desc) with caller
// buffers; the permutation ends in vals.
int lex_sort_rows(hipStream_t s, const double* wv, int nobj, int64_t n, bool desc, uint64_t* keys,
                  uint64_t* ktmp, int32_t* vals, int32_t* vtmp, void* rtemp, int nlex,
                  int begin_bit) {
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    if (nlex < 0 || nlex > nobj) nlex = nobj;
    if (nlex == 0) iota_kernel<<<g, 256, 0, s>>>(vals, n);
    for (int o = nlex - 1; o >= 0; --o) {  // LSD over objectives: last objective first
        if (o == nlex - 1)
            key_obj_iota_kernel<<<g, 256, 0, s>>>(wv, nobj, o, vals, keys, n, desc);
        else
            key_obj_kernel<<<g, 256, 0, s>>>(wv, nobj, o, vals, keys, n, desc);
        int rc = radix_sort_pairs(s, keys, vals, ktmp, vtmp, n, begin_bit, 64, rtemp);
        if (rc) return rc;
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// Same on the context scratch (slot 0); vals_out must not live in slot 0.
int sort_by_fitness(dm_ctx* ctx, const double* wv, int nobj, int64_t n, bool desc,
                    int32_t* vals_out) {
    const size_t kb = align_up((size_t)n * 8, 256), vb = align_up((size_t)n * 4, 256);
    char* s = (char*)scratch(ctx, 2 * kb + vb + radix_sort_temp_bytes(n));
    if (!s) return DM_ERR_NOMEM;
    return lex_sort_rows(ctx->stream, wv, nobj, n, desc, (uint64_t*)s, (uint64_t*)(s + kb),
                         vals_out, (int32_t*)(s + 2 * kb), s + 2 * kb + vb);
}


// Top-k of a single-objective population (k <= TOPK_MAX): the order of the
// first k entries of the stable sort without sorting n keys.  A wave holds
// 1,024 (key, index) pairs in registers (16 per lane) and extracts its k
// smallest in k rounds (lane minimum, 6-step shuffle minimum, the winner's
// slot cleared); a pass turns n pairs into ceil(n / 1024) * k candidates and
// is repeated until one wave's span remains (2^20 -> 15,360 -> 225 -> k for
// k = 15).  Pairs are distinct (the index breaks ties), so the result is
// exactly the stable order: ties by ascending index.  (The previous version
// bitonic-sorted 4,096-pair slices in LDS and then all candidates in one
// workgroup: 0.21 ms per selBest of 2^20; profiles/r02h.)
constexpr int TOPK_MAX = 128;  // HallOfFame candidate sets are 64+
constexpr int TOPK_PER = 16;            // pairs per lane
constexpr int TOPK_SPAN = 64 * TOPK_PER;  // pairs per wave

// (key, index) minimum over a row of 16 lanes through DPP (quad xor 1, quad
// xor 2, half-row mirror, row mirror: every lane ends with its row's
// minimum), then over the 4 rows by readlane: wave-uniform result, no LDS
// round trips (the __shfl_xor butterfly was 18 ds_bpermute per round).
template <int CTRL>
__device__ __forceinline__ void dpp_min_step(uint64_t& k, int32_t& i) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)k, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(k >> 32), CTRL, 0xF, 0xF, false);
    const int32_t oi = __builtin_amdgcn_mov_dpp(i, CTRL, 0xF, 0xF, false);
    const uint64_t ok = ((uint64_t)hi << 32) | lo;
    if (ok < k || (ok == k && oi < i)) {
        k = ok;
        i = oi;
    }
}
__device__ __forceinline__ void wave_min_pair(uint64_t& k, int32_t& i) {
    dpp_min_step<0xB1>(k, i);   // quad_perm(1,0,3,2)
    dpp_min_step<0x4E>(k, i);   // quad_perm(2,3,0,1)
    dpp_min_step<0x141>(k, i);  // row_half_mirror
    dpp_min_step<0x140>(k, i);  // row_mirror
    uint64_t bk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), 0) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, 0);
    int32_t bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const uint64_t rk =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k >> 32), r) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, r);
        const int32_t ri = __builtin_amdgcn_readlane(i, r);
        if (rk < bk || (rk == bk && ri < bi)) {
            bk = rk;
            bi = ri;
        }
    }
    k = bk;
    i = bi;
}

template <bool FROM_WV>
__global__ __launch_bounds__(256) void topk_wave_kernel(const double* __restrict__ wv, bool desc,
                                                        const uint64_t* __restrict__ ikey,
                                                        const int32_t* __restrict__ iidx, int64_t n,
                                                        int k, uint64_t* __restrict__ okey,
                                                        int32_t* __restrict__ oidx,
                                                        int32_t* __restrict__ out_final,
                                                        const int32_t* __restrict__ skip) {
    if (skip && *skip) return;  // the bucket selection already wrote the result
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t base = wave * TOPK_SPAN;
    if (base >= n) return;  // wave-uniform
    uint64_t key[TOPK_PER];
    int32_t idx[TOPK_PER];
#pragma unroll
    for (int j = 0; j < TOPK_PER; ++j) {
        const int64_t r = base + j * 64 + lane;
        key[j] = ~0ull;
        idx[j] = INT32_MAX;
        if (r < n) {
            if (FROM_WV) {
                const uint64_t q = ordered_key(wv[r]);
                key[j] = desc ? ~q : q;
                idx[j] = (int32_t)r;
            } else {
                key[j] = ikey[r];
                idx[j] = iidx[r];
            }
        }
    }
    for (int round = 0; round < k; ++round) {
        uint64_t bk = key[0];
        int32_t bi = idx[0];
#pragma unroll
        for (int j = 1; j < TOPK_PER; ++j)
            if (key[j] < bk || (key[j] == bk && idx[j] < bi)) {
                bk = key[j];
                bi = idx[j];
            }
        wave_min_pair(bk, bi);
#pragma unroll
        for (int j = 0; j < TOPK_PER; ++j)
            if (idx[j] == bi && key[j] == bk) {
                key[j] = ~0ull;
                idx[j] = INT32_MAX;
            }
        if (lane == 0) {
            if (out_final) {
                out_final[round] = bi;
            } else {
                okey[wave * k + round] = bk;
                oidx[wave * k + round] = bi;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Bucket selection (the usual path for n > one wave's span): the keys' range
// [kmin, kmax] is cut into 2,048 equal buckets (a monotone map of the key),
// a histogram finds the bucket B holding the k-th key, every element of a
// bucket <= B (at most TK_CAP of them) is compacted and ranked by (key,
// index) among the others: rank < k goes to out[rank].  A few full-width
// passes instead of k sequential extraction rounds (0.33 ms for k = 64 at
// 2^20, profiles/r02 bookkeeping run).  When more than TK_CAP elements share
// the buckets <= B (massive ties) the wave passes above run instead; they
// read the flag and return at once otherwise.
constexpr int TK_BUCKETS = 2048, TK_CAP = 16384, TK_BLOCKS = 64;
struct TkState {
    unsigned long long kmin, kmax;
    int32_t B, ncand, fallback, count;
};
__device__ __forceinline__ uint64_t tk_key(const double* wv, int64_t i, bool best) {
    const uint64_t q = ordered_key(wv[i]);
    return best ? ~q : q;
}
__device__ __forceinline__ int tk_bucket(uint64_t key, const TkState& st) {
    const uint64_t width = (st.kmax - st.kmin) / TK_BUCKETS + 1;
    return (int)((key - st.kmin) / width);
}
__global__ __launch_bounds__(256) void tk_minmax_kernel(const double* __restrict__ wv, int64_t n,
                                                        bool best, TkState* st) {
    uint64_t mn = ~0ull, mx = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = tk_key(wv, i, best);
        mn = key < mn ? key : mn;
        mx = key > mx ? key : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    __shared__ uint64_t smn[4], smx[4];
    if ((threadIdx.x & 63) == 0) {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            mn = smn[w] < mn ? smn[w] : mn;
            mx = smx[w] > mx ? smx[w] : mx;
        }
        atomicMin(&st->kmin, (unsigned long long)mn);
        atomicMax(&st->kmax, (unsigned long long)mx);
    }
}
__global__ __launch_bounds__(256) void tk_hist_kernel(const double* __restrict__ wv, int64_t n,
                                                      bool best, const TkState* st,
                                                      int32_t* __restrict__ part) {
    __shared__ int32_t h[TK_BUCKETS];
    for (int b = threadIdx.x; b < TK_BUCKETS; b += blockDim.x) h[b] = 0;
    __syncthreads();
    const TkState s = *st;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[tk_bucket(tk_key(wv, i, best), s)], 1);
    __syncthreads();
    for (int b = threadIdx.x; b < TK_BUCKETS; b += blockDim.x)
        part[(int64_t)blockIdx.x * TK_BUCKETS + b] = h[b];
}
// one workgroup of 1024: bucket totals, their inclusive scan, the boundary
__global__ __launch_bounds__(1024) void tk_bound_kernel(const int32_t* __restrict__ part, int nparts,
                                                        int64_t k, TkState* st) {
    __shared__ int32_t tot[TK_BUCKETS];
    __shared__ int32_t wsum[16];
    constexpr int PER = TK_BUCKETS / 1024;
    int32_t c[PER];
    int32_t run = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int b = threadIdx.x * PER + j;
        int32_t t = 0;
        for (int q = 0; q < nparts; ++q) t += part[(int64_t)q * TK_BUCKETS + b];
        run += t;
        c[j] = run;  // inclusive within the thread's buckets
    }
    // scan of the per-thread totals
    int32_t x = run;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int32_t off = 0;
    for (int i = 0; i < w; ++i) off += wsum[i];
    const int32_t excl = off + x - run;
#pragma unroll
    for (int j = 0; j < PER; ++j) tot[threadIdx.x * PER + j] = excl + c[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int b = threadIdx.x * PER + j;
        const int32_t prev = b ? tot[b - 1] : 0;
        if (prev < k && tot[b] >= k) {  // exactly one bucket
            st->B = b;
            st->ncand = tot[b];
            st->fallback = tot[b] > TK_CAP ? 1 : 0;
        }
    }
}
__global__ __launch_bounds__(256) void tk_compact_kernel(const double* __restrict__ wv, int64_t n,
                                                         bool best, TkState* st,
                                                         uint64_t* __restrict__ ckey,
                                                         int32_t* __restrict__ cidx) {
    if (st->fallback) return;
    const TkState s = *st;
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        uint64_t key = 0;
        bool in = false;
        if (i < n) {
            key = tk_key(wv, i, best);
            in = tk_bucket(key, s) <= s.B;
        }
        const uint64_t m = __ballot(in);
        if (!m) continue;
        int32_t base = 0;
        if (lane == 0) base = atomicAdd(&st->count, __popcll(m));
        base = __shfl(base, 0, 64);
        if (in) {
            const int32_t slot = base + __popcll(m & ((1ull << lane) - 1));
            ckey[slot] = key;
            cidx[slot] = (int32_t)i;
        }
    }
}
// rank of each candidate by (key, index) among all candidates; rank < k -> out
__global__ __launch_bounds__(256) void tk_rank_kernel(const uint64_t* __restrict__ ckey,
                                                      const int32_t* __restrict__ cidx,
                                                      const TkState* st, int64_t k,
                                                      int32_t* __restrict__ out) {
    if (st->fallback) return;
    const int c = st->ncand;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(blockIdx.x * blockDim.x) >= c) return;  // whole workgroup idle
    const uint64_t ki = i < c ? ckey[i] : ~0ull;
    const int32_t ii = i < c ? cidx[i] : INT32_MAX;
    __shared__ uint64_t tk[1024];
    __shared__ int32_t ti[1024];
    int32_t rank = 0;
    for (int t0 = 0; t0 < c; t0 += 1024) {
        __syncthreads();
        for (int j = threadIdx.x; j < 1024; j += blockDim.x) {
            tk[j] = t0 + j < c ? ckey[t0 + j] : ~0ull;
            ti[j] = t0 + j < c ? cidx[t0 + j] : INT32_MAX;
        }
        __syncthreads();
        const int m = c - t0 < 1024 ? c - t0 : 1024;
        for (int j = 0; j < m; ++j) rank += (tk[j] < ki || (tk[j] == ki && ti[j] < ii)) ? 1 : 0;
    }
    if (i < c && rank < k) out[rank] = ii;
}
__global__ void tk_flip_kernel(TkState* st) { st->fallback = !st->fallback; }
__global__ void tk_init_kernel(TkState* st) {
    st->kmin = ~0ull;
    st->kmax = 0;
    st->B = 0;
    st->ncand = 0;
    st->fallback = 0;
    st->count = 0;
}

static int sel_topk(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx, bool best) {
    const int64_t n = pop->n;
    auto waves = [](int64_t m) { return (m + TOPK_SPAN - 1) / TOPK_SPAN; };
    hipStream_t s = ctx->stream;
    if (n <= TOPK_SPAN) {
        topk_wave_kernel<true><<<1, 64, 0, s>>>(pop->wvalues, best, nullptr, nullptr, n, (int)k,
                                                nullptr, nullptr, out_idx, nullptr);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    const int64_t c1 = waves(n) * k;  // candidates after the first wave pass
    const size_t kb = align_up((size_t)c1 * 8, 256), ib = align_up((size_t)c1 * 4, 256);
    const size_t pb = align_up((size_t)TK_BLOCKS * TK_BUCKETS * 4, 256);
    const size_t cb = align_up((size_t)TK_CAP * 8, 256) + align_up((size_t)TK_CAP * 4, 256);
    char* w = (char*)scratch_slot(ctx, 3, 2 * (kb + ib) + pb + cb + 256);
    if (!w) return DM_ERR_NOMEM;
    uint64_t* key[2] = {(uint64_t*)w, (uint64_t*)(w + kb + ib)};
    int32_t* idx[2] = {(int32_t*)(w + kb), (int32_t*)(w + 2 * kb + ib)};
    char* t = w + 2 * (kb + ib);
    int32_t* part = (int32_t*)t;
    uint64_t* ckey = (uint64_t*)(t + pb);
    int32_t* cidx = (int32_t*)(t + pb + align_up((size_t)TK_CAP * 8, 256));
    TkState* st = (TkState*)(t + pb + cb);
    const int32_t* skip = &st->fallback;  // 0 after a bucket selection: wave passes skip
    // bucket selection
    tk_init_kernel<<<1, 1, 0, s>>>(st);
    tk_minmax_kernel<<<TK_BLOCKS * 4, 256, 0, s>>>(pop->wvalues, n, best, st);
    tk_hist_kernel<<<TK_BLOCKS, 256, 0, s>>>(pop->wvalues, n, best, st, part);
    tk_bound_kernel<<<1, 1024, 0, s>>>(part, TK_BLOCKS, k, st);
    tk_compact_kernel<<<TK_BLOCKS * 4, 256, 0, s>>>(pop->wvalues, n, best, st, ckey, cidx);
    tk_rank_kernel<<<TK_CAP / 256, 256, 0, s>>>(ckey, cidx, st, k, out_idx);
    // wave passes: only when the buckets <= B hold more than TK_CAP elements
    tk_flip_kernel<<<1, 1, 0, s>>>(st);  // skip = !fallback
    auto grid = [&](int64_t m) { return dim3((unsigned)((waves(m) + 3) / 4)); };
    topk_wave_kernel<true><<<grid(n), 256, 0, s>>>(pop->wvalues, best, nullptr, nullptr, n, (int)k,
                                                   key[0], idx[0], nullptr, skip);
    int64_t m = c1;
    int cur = 0;
    while (m > TOPK_SPAN) {
        topk_wave_kernel<false><<<grid(m), 256, 0, s>>>(nullptr, best, key[cur], idx[cur], m, (int)k,
                                                        key[cur ^ 1], idx[cur ^ 1], nullptr, skip);
        m = waves(m) * k;
        cur ^= 1;
    }
    topk_wave_kernel<false><<<1, 64, 0, s>>>(nullptr, best, key[cur], idx[cur], m, (int)k, nullptr,
                                             nullptr, out_idx, skip);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

}  // namespace dm

using namespace dm;

static int sel_sorted(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx, bool best) {
    DM_CHECK_ARG(ctx && out_idx, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    k = std::min(k, pop->n);
    if (k == 0) return DM_OK;
    DM_CHECK_ARG(pop->n < (1ll << 31), "population too large");
    // small k of a single objective (migRing emigrants, HallOfFame candidates)
    if (pop->nobj == 1 && k <= TOPK_MAX && pop->n > 4 * k &&
        !ctx->knobs.selbest_fullsort)
        return sel_topk(ctx, pop, k, out_idx, best);
    int32_t* full = out_idx;
    if (k < pop->n) {
        full = (int32_t*)scratch_slot(ctx, 3, (size_t)pop->n * 4);
        if (!full) return DM_ERR_NOMEM;
    }
    rc = sort_by_fitness(ctx, pop->wvalues, pop->nobj, pop->n, best, full);
    if (rc) return rc;
    if (full != out_idx)
        DM_HIP(hipMemcpyAsync(out_idx, full, (size_t)k * 4, hipMemcpyDeviceToDevice, ctx->stream));
    return DM_OK;
}

extern "C" int dm_sel_best(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx) {
    return sel_sorted(ctx, pop, k, out_idx, true);
}
extern "C" int dm_sel_worst(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx) {
    return sel_sorted(ctx, pop, k, out_idx, false);
}

// Test hook (not part of include/deapmi.h): sort nseg segments of seglen
// (key, value) pairs in place by key bits [begin_bit, end_bit), stably,
// through the dispatcher above (LDS / sample / radix sort by size), then wait.
extern "C" int dm_test_sort_pairs(dm_ctx* ctx, uint64_t* keys, int32_t* vals, int64_t nseg,
                                  int64_t seglen, int begin_bit, int end_bit) {
    DM_CHECK_ARG(ctx && keys && vals, "null argument");
    DM_CHECK_ARG(nseg >= 0 && seglen >= 0 && begin_bit >= 0 && end_bit <= 64, "bad sort shape");
    const int64_t n = nseg * seglen;
    const size_t kb = align_up((size_t)std::max<int64_t>(n, 1) * 8, 256);
    const size_t vb = align_up((size_t)std::max<int64_t>(n, 1) * 4, 256);
    char* t = (char*)scratch(ctx, kb + vb + radix_sort_batched_temp_bytes(nseg, seglen));
    if (!t) return DM_ERR_NOMEM;
    int rc = radix_sort_pairs_batched(ctx->stream, keys, vals, (uint64_t*)t, (int32_t*)(t + kb),
                                      nseg, seglen, begin_bit, end_bit, t + kb + vb);
    if (rc) return rc;
    DM_HIP(hipStreamSynchronize(ctx->stream));
    return DM_OK;
}

// Test hook: seg_sort_pairs_small over device segment starts (nseg + 1 ints);
// n = starts[nseg] pairs (the tmp buffers of oversized segments).
extern "C" int dm_test_seg_sort_pairs(dm_ctx* ctx, uint64_t* keys, int32_t* vals,
                                      const int32_t* starts, int64_t nseg, int begin_bit,
                                      int end_bit, int64_t n) {
    DM_CHECK_ARG(ctx && keys && vals && starts && n >= 0, "null argument");
    char* t = (char*)scratch(ctx, align_up((size_t)n * 8, 256) + (size_t)n * 4 + 256);
    if (!t) return DM_ERR_NOMEM;
    int rc = seg_sort_pairs_small(ctx->stream, keys, vals, starts, nseg, begin_bit, end_bit,
                                  (uint64_t*)t, (int32_t*)(t + align_up((size_t)n * 8, 256)));
    if (rc) return rc;
    DM_HIP(hipStreamSynchronize(ctx->stream));
    return DM_OK;
}

// Test hook: the device scans over n ints (kind 0: exclusive sum with its
// total in *total, 1: inclusive max) -- one tile, reduce-then-scan with the
// direct and the scanned-aggregate prefixes, and the block-sum form past 4 Mi.
extern "C" int dm_test_scan_i32(dm_ctx* ctx, const int32_t* in, int32_t* out, int64_t n, int kind,
                                int32_t* total) {
    DM_CHECK_ARG(ctx && in && out && n >= 0 && (kind == 0 || kind == 1), "bad scan arguments");
    void* t = scratch(ctx, scan_temp_bytes(n));
    if (!t) return DM_ERR_NOMEM;
    int rc = kind == 0 ? exclusive_scan_i32(ctx->stream, in, out, n, total, t)
                       : inclusive_max_scan_i32(ctx->stream, in, out, n, t);
    if (rc) return rc;
    DM_HIP(hipStreamSynchronize(ctx->stream));
    return DM_OK;
}
