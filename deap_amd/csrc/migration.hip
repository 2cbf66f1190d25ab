// migration.hip — migRing building blocks (deap/tools/migration.py:4-51).
//
// Emigrants / immigrants travel as packed blocks (dm_pack_rows): this is the
// payload exchanged between GPUs with RCCL point-to-point.  Placement
// (dm_mig_place) reproduces the reference's sequential
//     indx = populations[to].index(immigrant); populations[to][indx] = emigrant
// including its aliasing quirk (a later equal-valued immigrant can hit the
// slot just filled by an equal emigrant):
//   1. one parallel pass over the deme marks, per immigrant j, the rows whose
//      genome equals immigrant j (fitness prefilter, then exact element
//      compare: float ==, so -0.0 == 0.0 as in Python) in a bitmap;
//   2. a k x k pass compares emigrant and immigrant genomes;
//   3. one workgroup resolves j = 0..k-1 in order: the first row that still
//      holds an original match, or an already-placed emigrant equal to
//      immigrant j, whichever index is smaller -- decisions first, in LDS,
//      then every row copied in parallel by its last taker.
#include "common.hpp"
#include "sort.hpp"

namespace dm {

int validate_pop(const dm_pop* p, const char* what);

struct Block {  // views into a packed block of k rows
    char* genes;
    double* wv;
    uint8_t* valid;
    int32_t* src;
};
static int64_t block_bytes(const dm_pop* p, int64_t k) {
    return k * p->stride + k * p->nobj * 8 + (int64_t)align_up((size_t)k, 8) + k * 4;
}
__host__ __device__ inline Block block_view(void* base, int64_t stride, int nobj, int64_t k) {
    char* b = (char*)base;
    Block v;
    v.genes = b;
    v.wv = (double*)(b + k * stride);
    v.valid = (uint8_t*)(b + k * stride + k * nobj * 8);
    v.src = (int32_t*)(b + k * stride + k * nobj * 8 + ((k + 7) / 8) * 8);
    return v;
}

__global__ void pack_kernel(const char* genes, const double* wv, const uint8_t* valid,
                            int64_t stride, int nobj, const int32_t* idx, int64_t k, void* block) {
    Block b = block_view(block, stride, nobj, k);
    const int lane = threadIdx.x & 63;
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= k) return;
    const int64_t s = idx[r];
    const uint4* src = reinterpret_cast<const uint4*>(genes + s * stride);
    uint4* dst = reinterpret_cast<uint4*>(b.genes + r * stride);
    for (int64_t i = lane; i < stride / 16; i += 64) dst[i] = src[i];
    if (lane < nobj) b.wv[r * nobj + lane] = wv[s * nobj + lane];
    if (lane == 0) {
        b.valid[r] = valid[s];
        b.src[r] = (int32_t)s;
    }
}

// Genome equality of row a and row b (value semantics of the genome type).
__device__ __forceinline__ bool genome_eq(const char* a, const char* b, int gtype, int dim) {
    if (gtype == DM_BITS) {
        const uint64_t* x = (const uint64_t*)a;
        const uint64_t* y = (const uint64_t*)b;
        for (int w = 0; w < (dim + 63) / 64; ++w)
            if (x[w] != y[w]) return false;
        return true;
    }
    if (gtype == DM_F32) {
        const float* x = (const float*)a;
        const float* y = (const float*)b;
        for (int i = 0; i < dim; ++i)
            if (!(x[i] == y[i])) return false;
        return true;
    }
    const double* x = (const double*)a;
    const double* y = (const double*)b;
    for (int i = 0; i < dim; ++i)
        if (!(x[i] == y[i])) return false;
    return true;
}

__device__ __forceinline__ bool fit_prefilter(const double* a, uint8_t va, const double* b,
                                              uint8_t vb, int nobj) {
    if (!va || !vb) return true;  // cannot use fitness, compare genomes
    for (int o = 0; o < nobj; ++o)
        if (!(a[o] == b[o])) return false;
    return true;
}

// Genome equality of rows a and b computed by a whole wave (value semantics
// of the genome type; lanes stride the genes, pad bytes never read).
__device__ __forceinline__ bool wave_genome_eq(const char* a, const char* b, int gtype, int dim,
                                               int lane) {
    bool ok = true;
    if (gtype == DM_BITS) {
        const uint64_t* x = (const uint64_t*)a;
        const uint64_t* y = (const uint64_t*)b;
        for (int w = lane; w < (dim + 63) / 64; w += 64) ok = ok && x[w] == y[w];
    } else if (gtype == DM_F32) {
        const float* x = (const float*)a;
        const float* y = (const float*)b;
        for (int i = lane; i < dim; i += 64) ok = ok && x[i] == y[i];
    } else {
        const double* x = (const double*)a;
        const double* y = (const double*)b;
        for (int i = lane; i < dim; i += 64) ok = ok && x[i] == y[i];
    }
    return __ballot(!ok) == 0;
}

// bitmap[j][w]: bit r%64 of word r/64 set iff row r equals immigrant j;
// first[j] = the lowest such row.  dirty (nullable): rows an earlier hop of
// the same migration overwrote — the immigrant object that was there is no
// longer in the list, so list.index's identity test cannot hit that row.  A wave owns 64 consecutive rows (one bitmap
// word per immigrant, written with a plain store), lane = row: the row's
// fitness / validity are loaded once and compared with a tile of 64
// immigrants staged in LDS; a fitness match (or an invalid fitness on either
// side) is confirmed by a genome comparison done by the whole wave.
__global__ __launch_bounds__(256) void match_kernel(const char* genes, const double* wv,
                                                    const uint8_t* valid, int64_t n, int64_t stride,
                                                    int dim, int gtype, int nobj,
                                                    const void* imm_block, int64_t k, int64_t words,
                                                    const unsigned long long* dirty,
                                                    unsigned long long* bitmap, int32_t* first) {
    Block im = block_view((void*)imm_block, stride, nobj, k);
    __shared__ double swv[64 * DM_MAX_OBJ];
    __shared__ int32_t ssrc[64];
    __shared__ uint8_t sval[64];
    const int lane = threadIdx.x & 63;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t jt = 0; jt < k; jt += 64) {
        const int jn = (int)(k - jt < 64 ? k - jt : 64);
        __syncthreads();
        if (threadIdx.x < jn) {
            const int64_t j = jt + threadIdx.x;
            ssrc[threadIdx.x] = im.src[j];
            sval[threadIdx.x] = im.valid[j];
            for (int o = 0; o < nobj; ++o) swv[threadIdx.x * nobj + o] = im.wv[j * nobj + o];
        }
        __syncthreads();
        for (int64_t r0 = wave0 * 64; r0 < n; r0 += nwaves * 64) {
            const int64_t r = r0 + lane;
            const bool in = r < n;
            double f[DM_MAX_OBJ];
#pragma unroll
            for (int o = 0; o < DM_MAX_OBJ; ++o) f[o] = (in && o < nobj) ? wv[r * nobj + o] : 0.0;
            const uint8_t vr = in ? valid[r] : 0;
            const bool clean = !(in && dirty && ((dirty[r >> 6] >> (r & 63)) & 1ull));
            for (int jj = 0; jj < jn; ++jj) {
                const int64_t j = jt + jj;
                // list.index tests `is` before `==` (PyObject_RichCompareBool):
                // the immigrant's own row matches even when its genome holds a NaN
                const bool self = in && clean && r == ssrc[jj];
                bool eq = self;
                // fitness prefilter (fit_prefilter, registers unrolled)
                bool pre = in && !self;
                if (pre && vr && sval[jj]) {
#pragma unroll
                    for (int o = 0; o < DM_MAX_OBJ; ++o)
                        if (o < nobj && !(f[o] == swv[jj * nobj + o])) pre = false;
                }
                uint64_t hits = __ballot(pre);
                while (hits) {  // wave-uniform
                    const int l = __ffsll((long long)hits) - 1;
                    hits &= hits - 1;
                    const bool e = wave_genome_eq(genes + (r0 + l) * stride, im.genes + j * stride,
                                                  gtype, dim, lane);
                    if (lane == l) eq = e;
                }
                const uint64_t m = __ballot(eq);
                if (lane == 0 && m) {
                    bitmap[j * words + (r0 >> 6)] = m;
                    atomicMin(&first[j], (int32_t)(r0 + __ffsll((long long)m) - 1));
                }
            }
        }
    }
}

// E[j*k + e] = emigrant e == immigrant j (genome), stored per immigrant
__global__ void em_im_eq_kernel(const void* em_block, const void* im_block, int64_t k,
                                int64_t stride, int dim, int gtype, int nobj, uint8_t* E) {
    Block em = block_view((void*)em_block, stride, nobj, k);
    Block im = block_view((void*)im_block, stride, nobj, k);
    // stored by immigrant: E[j * k + e] = emigrant e equals immigrant j (the
    // placement of immigrant j reads row j of it)
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k * k;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = t / k, e = t % k;
        E[t] = genome_eq(em.genes + e * stride, im.genes + j * stride, gtype, dim) ? 1 : 0;
    }
}

// Sequential resolution, decisions first: immigrant j's slot
// depends only on which rows earlier immigrants took and which emigrants are
// still where they were put, so the k decisions run in LDS -- (a) the first
// original match not taken by an earlier placement (first[j], unless taken:
// then the bitmap from there with the taken rows masked), (b) a smaller row
// still holding an earlier emigrant equal to immigrant j -- and only then are
// the rows copied, in parallel, each slot by its last writer.  Same result as
// placing and copying one immigrant at a time (what round 3 did: 124 us per
// deme at k = 15), without a global round trip and a row copy per immigrant.
// Row copies of a placement, flattened over (row, 16-B piece) and eight
// pieces per thread in flight: a wave copying one 8-KB row at a time with one
// load outstanding took ~12 us per row.  dst_slot(j) < 0: row j not copied.
template <typename SlotFn>
__device__ __forceinline__ void copy_em_rows(char* genes, int64_t stride, const Block& em,
                                             int64_t nrows, SlotFn dst_slot) {
    const int64_t per = stride / 16, total = nrows * per;
    const int64_t nt = blockDim.x;
    constexpr int U = 8;
    for (int64_t t0 = threadIdx.x; t0 < total; t0 += nt * U) {
        uint4 v[U];
        int64_t slot[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t = t0 + u * nt;
            slot[u] = -1;
            if (t < total) {
                const int64_t j = t / per;
                slot[u] = dst_slot(j);
                if (slot[u] >= 0) v[u] = reinterpret_cast<const uint4*>(em.genes + j * stride)[t - j * per];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t = t0 + u * nt;
            if (slot[u] >= 0) {
                const int64_t j = t / per;
                reinterpret_cast<uint4*>(genes + slot[u] * stride)[t - j * per] = v[u];
            }
        }
    }
}

constexpr int RES_MAX = 4096;  // placements tracked in LDS = the API's k limit (dm_mig_place)
constexpr int MLIST = 64;      // leading matches of each immigrant listed before the resolution

// mlist[j][0..mcount[j]): the first min(j + 1, MLIST) rows whose genome
// equals immigrant j, ascending (at most j rows can be taken before
// immigrant j is placed, so j + 1 leading matches always hold its answer when
// the list is complete).  One workgroup per immigrant, from first[j]'s word.
__global__ __launch_bounds__(256) void first_matches_kernel(const unsigned long long* bitmap,
                                                            int64_t words, const int32_t* first,
                                                            int64_t n, int32_t* mlist,
                                                            int32_t* mcount) {
    const int64_t j = blockIdx.x;
    const int L = (int)std::min<int64_t>(MLIST, j + 1);
    __shared__ int32_t sh[4];
    if (first[j] >= n) {
        if (threadIdx.x == 0) mcount[j] = 0;
        return;
    }
    // 16 consecutive words per thread per pass (4,096 words = 262,144 rows):
    // the loads of a pass are all in flight together
    constexpr int WPT = 16;
    const unsigned long long* row = bitmap + j * words;
    int got = 0;
    for (int64_t wb = first[j] >> 6; wb < words && got < L; wb += 256 * WPT) {
        const int64_t w0 = wb + (int64_t)threadIdx.x * WPT;
        unsigned long long x[WPT];
        int c = 0;
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            x[i] = w0 + i < words ? row[w0 + i] : 0ull;
            c += __popcll(x[i]);
        }
        int pos = got + block_incl_scan<256, false>(c, sh) - c;
        const int total = sh[3];
#pragma unroll
        for (int i = 0; i < WPT; ++i)
            for (unsigned long long y = x[i]; y && pos < L; y &= y - 1)
                mlist[j * MLIST + pos++] = (int32_t)((w0 + i) * 64 + __ffsll((long long)y) - 1);
        __syncthreads();  // sh is reused by the next pass's scan
        got += total;
    }
    if (threadIdx.x == 0) mcount[j] = std::min(got, L);
}

// The identity bitmap of a receiving deme (rows whose original object is no
// longer in the list, so list.index may not match them by identity), set
// from each row's FINAL occupant of a hop: a row whose last taker is its own
// object (a self hop's emigrant from that row, self_rows[j] == slot) has its
// identity back -- even if an earlier placement of this hop or an earlier hop
// took it -- every other final occupant is foreign.  Stale placements (a
// later one took the row) leave the bit alone.
__device__ __forceinline__ void mark_identity(unsigned long long* dirty, const int32_t* self_rows,
                                              int64_t j, int64_t slot) {
    const unsigned long long bit = 1ull << (slot & 63);
    if (self_rows && self_rows[j] == slot)
        atomicAnd(&dirty[slot >> 6], ~bit);
    else
        atomicOr(&dirty[slot >> 6], bit);
}

__device__ void resolve_decide_then_copy(char* genes, double* wv, uint8_t* valid, int64_t n,
                                         int64_t stride, int nobj, const Block& em, int64_t k,
                                         int64_t words, const unsigned long long* bitmap,
                                         const uint8_t* E, const int32_t* mlist,
                                         const int32_t* mcount, int32_t* slots,
                                         unsigned long long* dirty, const int32_t* self_rows,
                                         int32_t* err) {
    __shared__ int32_t sl[RES_MAX];     // slot of placement j
    __shared__ uint8_t stale[RES_MAX];  // placement j's row was taken by a later one
    __shared__ int32_t smc[RES_MAX];
    // the rows taken so far, an open-addressing set (load <= 1/2): rule (a)'s
    // "taken?" is one or two LDS probes instead of a scan over every earlier
    // placement (O(k^2) per lane at k = 4,096)
    constexpr int TH = 2 * RES_MAX;
    __shared__ int32_t taken_set[TH];
    auto slot_of = [](int32_t row) { return (int)(((uint32_t)row * 2654435761u) >> 19) & (TH - 1); };
    auto is_taken = [&](int32_t row) {
        for (int h = slot_of(row);; h = (h + 1) & (TH - 1)) {
            const int32_t v = taken_set[h];
            if (v == row) return true;
            if (v < 0) return false;
        }
    };
    constexpr int SM = 64;              // E and the match lists staged in LDS up to k = 64 (C4: 15)
    __shared__ uint8_t sE[SM * SM];
    __shared__ int32_t sml[SM * MLIST];
    __shared__ unsigned long long sbest;
    __shared__ int nplaced;
    const int tid = threadIdx.x, nt = blockDim.x;
    const bool small = k <= SM;
    for (int64_t j = tid; j < k; j += nt) smc[j] = mcount[j];
    for (int t = tid; t < TH; t += nt) taken_set[t] = -1;
    if (small) {
        for (int64_t t = tid; t < k * k; t += nt) sE[t] = E[t];
        for (int64_t t = tid; t < k * MLIST; t += nt) sml[t] = mlist[t];
    }
    if (tid == 0) nplaced = (int)k;
    __syncthreads();
    for (int64_t j = 0; j < k; ++j) {
        if (tid == 0) sbest = ~0ull;
        __syncthreads();
        // (a) the first listed match no earlier placement took (rows ascend)
        const int mc = smc[j];
        if (tid < mc) {
            const int32_t row = small ? sml[j * MLIST + tid] : mlist[j * MLIST + tid];
            if (!is_taken(row)) atomicMin(&sbest, (unsigned long long)row);
        }
        __syncthreads();
        if (sbest == ~0ull && mc == MLIST) {
            // every listed match taken (j >= MLIST): scan on past the list,
            // taken rows masked
            const int64_t start = (int64_t)(small ? sml[j * MLIST + MLIST - 1]
                                                  : mlist[j * MLIST + MLIST - 1]) + 1;
            for (int64_t wb = start >> 6; wb < words; wb += nt) {
                const int64_t w = wb + tid;
                unsigned long long x = w < words ? bitmap[j * words + w] : 0ull;
                if (w == (start >> 6) && (start & 63)) x &= ~0ull << (start & 63);
                for (unsigned long long y = x; y; y &= y - 1) {
                    const int b = __ffsll((long long)y) - 1;
                    if (is_taken((int32_t)(w * 64 + b))) x &= ~(1ull << b);
                    else break;  // the lowest untaken row of the word is all rule (a) needs
                }
                if (x) atomicMin(&sbest, (unsigned long long)(w * 64 + __ffsll((long long)x) - 1));
                __syncthreads();
                if (sbest != ~0ull) break;
                __syncthreads();
            }
        }
        // (b) an earlier emigrant equal to immigrant j, still in its row, at a smaller row
        for (int64_t p = tid; p < j; p += nt)
            if (!stale[p] && (small ? sE[j * k + p] : E[j * k + p]) &&
                (unsigned long long)sl[p] < sbest)
                atomicMin(&sbest, (unsigned long long)sl[p]);
        __syncthreads();
        const unsigned long long slot = sbest;
        if (slot >= (unsigned long long)n) {  // list.index -> ValueError
            if (tid == 0) {
                *err = (int32_t)j + 1;
                nplaced = (int)j;
            }
            __syncthreads();
            break;
        }
        if (tid == 0) {
            sl[j] = (int32_t)slot;
            stale[j] = 0;
            if (!is_taken((int32_t)slot)) {
                int h = slot_of((int32_t)slot);
                while (taken_set[h] >= 0) h = (h + 1) & (TH - 1);
                taken_set[h] = (int32_t)slot;
            }
        }
        for (int64_t p = tid; p < j; p += nt)
            if ((unsigned long long)sl[p] == slot) stale[p] = 1;
        __syncthreads();
    }
    __syncthreads();
    const int np = nplaced;
    // copies: a row taken twice is written by its last taker
    copy_em_rows(genes, stride, em, np, [&](int64_t j) { return stale[j] ? -1ll : (long long)sl[j]; });
    for (int64_t j = tid; j < np; j += nt) {
        const int64_t slot = sl[j];
        if (!stale[j]) {
            for (int o = 0; o < nobj; ++o) wv[slot * nobj + o] = em.wv[j * nobj + o];
            valid[slot] = em.valid[j];
        }
        slots[j] = (int32_t)slot;
        if (dirty && !stale[j]) mark_identity(dirty, self_rows, j, slot);
    }
}

// Placement of one deme's k immigrants; one workgroup of 256 threads.
__global__ __launch_bounds__(256) void resolve_kernel(char* genes, double* wv, uint8_t* valid,
                                                      int64_t n, int64_t stride, int nobj,
                                                      const void* em_block, int64_t k,
                                                      int64_t words, unsigned long long* bitmap,
                                                      const uint8_t* E, const int32_t* first,
                                                      const int32_t* mlist, const int32_t* mcount,
                                                      int32_t* slots, unsigned long long* dirty,
                                                      const int32_t* self_rows, int32_t* err) {
    Block em = block_view((void*)em_block, stride, nobj, k);
    __shared__ int fast;
    if (threadIdx.x == 0) fast = 1;
    __syncthreads();
    // Fast path: when every immigrant has a first match, the first matches
    // are pairwise distinct and no emigrant equals any immigrant, no
    // placement can change another immigrant's match, so the decisions
    // below would put emigrant j into first[j] for every j: copy directly.
    for (int64_t t = threadIdx.x; t < k * k; t += blockDim.x) {
        const int64_t e = t / k, j = t % k;
        if (E[t] || first[j] >= n || (e < j && first[e] == first[j])) fast = 0;
    }
    __syncthreads();
    if (fast) {
        copy_em_rows(genes, stride, em, k, [&](int64_t j) { return (long long)first[j]; });
        for (int64_t j = threadIdx.x; j < k; j += blockDim.x) {
            const int64_t slot = first[j];
            for (int o = 0; o < nobj; ++o) wv[slot * nobj + o] = em.wv[j * nobj + o];
            valid[slot] = em.valid[j];
            slots[j] = (int32_t)slot;
            if (dirty) mark_identity(dirty, self_rows, j, slot);
        }
        return;
    }
    resolve_decide_then_copy(genes, wv, valid, n, stride, nobj, em, k, words, bitmap, E, mlist,
                             mcount, slots, dirty, self_rows, err);
}

}  // namespace dm

using namespace dm;

extern "C" int64_t dm_pack_bytes(const dm_pop* pop, int64_t k) {
    if (!pop || k < 0) return 0;
    return block_bytes(pop, k);
}

extern "C" int dm_pack_rows(dm_ctx* ctx, const dm_pop* pop, const int32_t* idx, int64_t k,
                            void* block) {
    DM_CHECK_ARG(ctx && pop && block, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0, "negative k");
    if (k == 0) return DM_OK;
    DM_CHECK_ARG(idx != nullptr, "null idx");
    pack_kernel<<<(unsigned)((k + 3) / 4), 256, 0, ctx->stream>>>(
        (const char*)pop->genes, pop->wvalues, pop->valid, pop->stride, pop->nobj, idx, k, block);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

namespace dm {
// Placement for one receiving deme, asynchronous: *err (device int32) gets
// j + 1 when immigrant j is not found (list.index ValueError), else stays 0.
// dirty (nullable, ceil(n/64) words): rows overwritten by earlier hops into
// this deme in the same migration (read by the identity test, and the rows
// this placement overwrites are added).
// self_rows (nullable): for a hop from the deme into itself, the emigrants'
// rows in it.
static int mig_place_async(dm_ctx* ctx, dm_pop* pop, const void* immigrant_block,
                           const void* emigrant_block, int64_t k, int32_t* out_slots,
                           unsigned long long* dirty, int32_t* err,
                           const int32_t* self_rows = nullptr) {
    const int64_t n = pop->n;
    const int64_t words = (n + 63) / 64;
    const size_t bm = align_up((size_t)k * words * 8, 256);
    DM_CHECK_ARG(k <= RES_MAX, "k must be in [0, 4096]");
    const size_t kb = align_up((size_t)k * 4, 256);
    char* base = (char*)scratch_slot(ctx, 3, bm + align_up((size_t)k * k, 256) + 2 * kb +
                                                 align_up((size_t)k * MLIST * 4, 256));
    if (!base) return DM_ERR_NOMEM;
    unsigned long long* bitmap = (unsigned long long*)base;
    uint8_t* E = (uint8_t*)(base + bm);
    int32_t* first = (int32_t*)(base + bm + align_up((size_t)k * k, 256));
    int32_t* mcount = (int32_t*)((char*)first + kb);
    int32_t* mlist = (int32_t*)((char*)mcount + kb);
    hipStream_t s = ctx->stream;
    DM_HIP(hipMemsetAsync(bitmap, 0, (size_t)k * words * 8, s));
    DM_HIP(hipMemsetAsync(first, 0x7F, (size_t)k * 4, s));  // INT32 ~max: no match yet
    // one wave per 64 rows, at most 16 waves per CU slot pass
    const unsigned grid = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((words + 3) / 4, (int64_t)ctx->num_cus * 16));
    match_kernel<<<grid, 256, 0, s>>>((const char*)pop->genes, pop->wvalues, pop->valid, n,
                                      pop->stride, pop->dim, pop->gtype, pop->nobj,
                                      immigrant_block, k, words, dirty, bitmap, first);
    em_im_eq_kernel<<<(unsigned)std::max<int64_t>(1, (k * k + 255) / 256), 256, 0, s>>>(
        emigrant_block, immigrant_block, k, pop->stride, pop->dim, pop->gtype, pop->nobj, E);
    first_matches_kernel<<<(unsigned)k, 256, 0, s>>>(bitmap, words, first, n, mlist, mcount);
    resolve_kernel<<<1, 256, 0, s>>>((char*)pop->genes, pop->wvalues, pop->valid, n, pop->stride,
                                     pop->nobj, emigrant_block, k, words, bitmap, E, first,
                                     mlist, mcount, out_slots, dirty, self_rows, err);
    DM_LAUNCH_CHECK();
    return DM_OK;
}
}  // namespace dm

extern "C" int dm_mig_place(dm_ctx* ctx, dm_pop* pop, const void* immigrant_block,
                            const void* emigrant_block, int64_t k, int32_t* out_slots) {
    DM_CHECK_ARG(ctx && pop && immigrant_block && emigrant_block && out_slots, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0 && k <= 4096, "k must be in [0, 4096]");
    if (k == 0) return DM_OK;
    int32_t* err = (int32_t*)scratch_slot(ctx, 4, 256);
    if (!err) return DM_ERR_NOMEM;
    DM_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
    if ((rc = mig_place_async(ctx, pop, immigrant_block, emigrant_block, k, out_slots, nullptr,
                              err)))
        return rc;
    int32_t herr = 0;
    DM_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, ctx->stream));
    DM_HIP(hipStreamSynchronize(ctx->stream));
    DM_CHECK_ARG(herr == 0, "migRing: immigrant %d is not in the receiving population", herr - 1);
    return DM_OK;
}

// ---------------------------------------------------------------------------
// random.sample(range(n), k) on the device (migRing's `replacement`).
// ---------------------------------------------------------------------------
namespace dm {

// k <= 4096 and 2k <= n: sequential rejection sampling in one workgroup —
// candidate a = Philox(SAMPLE, a, 0) mod n (64-bit bounded), rejected when it
// is already among the accepted ones (the 256 threads test the accepted list
// in parallel).  Expected attempts <= 2k.
__global__ __launch_bounds__(256) void sample_reject_kernel(Rng rng, int64_t n, int64_t k,
                                                            int32_t* out) {
    __shared__ int32_t acc[4096];
    __shared__ int dup;
    int cnt = 0;
    for (uint32_t a = 0; cnt < k; ++a) {
        const u32x4 w = rng(ST_SAMPLE, a, 0u);
        const int32_t c = (int32_t)bounded64(w.x, w.y, (uint32_t)n);
        if (threadIdx.x == 0) dup = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += blockDim.x)
            if (acc[i] == c) dup = 1;
        __syncthreads();
        if (!dup) {
            if (threadIdx.x == 0) {
                acc[cnt] = c;
                out[cnt] = c;
            }
            ++cnt;
        }
        __syncthreads();
    }
}

__global__ void sample_keys_kernel(Rng rng, int64_t n, uint64_t* keys, int32_t* vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const u32x4 w = rng(ST_SAMPLE, (uint32_t)i, 1u);
        keys[i] = ((uint64_t)w.x << 32) | w.y;
        vals[i] = (int32_t)i;
    }
}

}  // namespace dm

#include "sort.hpp"

extern "C" int dm_sel_sample(dm_ctx* ctx, int64_t n, int64_t k, dm_rng rng, int32_t* out_idx) {
    DM_CHECK_ARG(ctx && out_idx, "null argument");
    DM_CHECK_ARG(n >= 0 && n < (1ll << 31), "bad population size");
    if (k < 0 || k > n) {
        set_error("Sample larger than population or is negative");
        return DM_ERR_INVALID;
    }
    if (k == 0) return DM_OK;
    hipStream_t s = ctx->stream;
    if (k <= 4096 && 2 * k <= n) {
        sample_reject_kernel<<<1, 256, 0, s>>>(Rng(rng), n, k, out_idx);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    // otherwise: the first k rows of a random permutation (Philox keys, stable
    // radix sort, ties by index)
    const size_t kb = align_up((size_t)n * 8, 256), vb = align_up((size_t)n * 4, 256);
    char* w = (char*)scratch(ctx, 2 * kb + 2 * vb + radix_sort_temp_bytes(n));
    if (!w) return DM_ERR_NOMEM;
    uint64_t* keys = (uint64_t*)w;
    uint64_t* ktmp = (uint64_t*)(w + kb);
    int32_t* vals = (int32_t*)(w + 2 * kb);
    int32_t* vtmp = (int32_t*)(w + 2 * kb + vb);
    void* rtemp = w + 2 * kb + 2 * vb;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    sample_keys_kernel<<<g, 256, 0, s>>>(Rng(rng), n, keys, vals);
    DM_LAUNCH_CHECK();
    int rc = radix_sort_pairs(s, keys, vals, ktmp, vtmp, n, 0, 64, rtemp);
    if (rc) return rc;
    DM_HIP(hipMemcpyAsync(out_idx, vals, (size_t)k * 4, hipMemcpyDeviceToDevice, s));
    return DM_OK;
}

// ---------------------------------------------------------------------------
// Whole migRing in one call: local demes (dm_mig_ring) and across ranks over
// RCCL point-to-point (dm_mig_ring_rccl).
// ---------------------------------------------------------------------------
#include <rccl/rccl.h>
#include <cstring>
#include <string>

struct dm_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    int32_t* flag = nullptr;  // device word for mig_agree
};

namespace dm {

static int plan_hops(int32_t n_demes, const int32_t* migarray, const int32_t* owner, int32_t me,
                     int32_t flags, std::vector<dm_mig_hop>& hops) {
    hops.clear();
    for (int32_t from = 0; from < n_demes; ++from) {
        const int32_t to = migarray ? migarray[from] : (from + 1) % n_demes;
        DM_CHECK_ARG(to >= 0 && to < n_demes, "migarray[%d] = %d is not a deme index", from, to);
        const int32_t src = owner ? owner[from] : 0, dst = owner ? owner[to] : 0;
        if (src == me && dst == me) {
            if ((flags & DM_MIG_FORCE_P2P) && from != to) {
                hops.push_back(dm_mig_hop{DM_HOP_SEND, from, to, me});
                hops.push_back(dm_mig_hop{DM_HOP_RECV, from, to, me});
            } else {
                hops.push_back(dm_mig_hop{DM_HOP_LOCAL, from, to, me});
            }
        } else if (src == me) {
            hops.push_back(dm_mig_hop{DM_HOP_SEND, from, to, dst});
        } else if (dst == me) {
            hops.push_back(dm_mig_hop{DM_HOP_RECV, from, to, src});
        }
    }
    return DM_OK;
}

#define DM_NCCL(expr)                                                              \
    do {                                                                           \
        ncclResult_t r_ = (expr);                                                  \
        if (r_ != ncclSuccess) {                                                   \
            ::dm::set_error("RCCL error %s at %s:%d: %s", ncclGetErrorString(r_),  \
                            __FILE__, __LINE__, #expr);                            \
            return DM_ERR_HIP;                                                     \
        }                                                                          \
    } while (0)

// Every per-rank check of a migration, and the scratch it needs, before any
// communication: a rank that fails here must not leave its peers waiting in
// ncclSend / ncclRecv (see mig_agree).
struct MigPlan {
    std::vector<int32_t> local_of;
    std::vector<dm_mig_hop> hops;
    char* base = nullptr;
    size_t bb = 0;
    int nrecv = 0;
    std::vector<int32_t> hops_into;  // per local deme: hops that place into it
};

static int mig_prepare(dm_ctx* ctx, dm_comm* comm, int32_t n_local, dm_pop* demes,
                       const int32_t* deme_ids, int32_t n_demes, const int32_t* migarray,
                       const int32_t* owner, int64_t k, int32_t* const* emig_idx, int32_t flags,
                       MigPlan& P) {
    DM_CHECK_ARG(n_demes >= 1 && n_local >= 0 && n_local <= n_demes, "bad deme counts");
    DM_CHECK_ARG(n_local == 0 || (demes && deme_ids && emig_idx), "null deme arrays");
    DM_CHECK_ARG(k >= 0 && k <= 4096, "k must be in [0, 4096]");
    const int me = comm ? comm->rank : 0;
    // local index of every global deme held here
    P.local_of.assign(n_demes, -1);
    for (int32_t i = 0; i < n_local; ++i) {
        DM_CHECK_ARG(deme_ids[i] >= 0 && deme_ids[i] < n_demes, "deme id %d out of range",
                     deme_ids[i]);
        DM_CHECK_ARG(P.local_of[deme_ids[i]] < 0, "deme %d listed twice", deme_ids[i]);
        if (owner) DM_CHECK_ARG(owner[deme_ids[i]] == me, "deme %d is not owned by rank %d",
                                deme_ids[i], me);
        P.local_of[deme_ids[i]] = i;
        int rc = validate_pop(&demes[i], "deme");
        if (rc) return rc;
        DM_CHECK_ARG(emig_idx[i] != nullptr || k == 0, "null emigrant indices");
        DM_CHECK_ARG(k <= demes[i].n, "k exceeds deme size");
    }
    if (owner)
        for (int32_t d = 0; d < n_demes; ++d)
            DM_CHECK_ARG(owner[d] >= 0 && (!comm || owner[d] < comm->nranks), "bad owner[%d]", d);
    if (!owner) DM_CHECK_ARG(n_local == n_demes, "without owner every deme must be local");
    int rc = plan_hops(n_demes, migarray, owner, me, flags, P.hops);
    if (rc) return rc;
    if (k == 0 || n_local == 0) return DM_OK;
    // every deme shares one layout (the blocks travel between them)
    for (int32_t i = 1; i < n_local; ++i)
        DM_CHECK_ARG(demes[i].stride == demes[0].stride && demes[i].dim == demes[0].dim &&
                         demes[i].gtype == demes[0].gtype && demes[i].nobj == demes[0].nobj,
                     "demes differ in layout");
    const bool p2p = std::any_of(P.hops.begin(), P.hops.end(),
                                 [](const dm_mig_hop& h) { return h.kind != DM_HOP_LOCAL; });
    DM_CHECK_ARG(!p2p || comm != nullptr, "cross-rank hops need an RCCL communicator");
    P.bb = align_up((size_t)block_bytes(&demes[0], k), 256);
    P.hops_into.assign(n_local, 0);
    for (const dm_mig_hop& h : P.hops) {
        P.nrecv += h.kind == DM_HOP_RECV;
        if (h.kind != DM_HOP_SEND) ++P.hops_into[P.local_of[h.to]];
    }
    // dirty-row bitmaps for demes that receive more than one hop
    size_t dirty_bytes = 0;
    for (int32_t i = 0; i < n_local; ++i)
        if (P.hops_into[i] > 1) dirty_bytes += align_up((size_t)(demes[i].n + 63) / 64 * 8, 256);
    // [emigrant block | immigrant block] per local deme, then one per receive,
    // the placement slots, the per-hop status words, the dirty bitmaps
    P.base = (char*)scratch_slot(ctx, 4, P.bb * (2 * (size_t)n_local + P.nrecv) +
                                             align_up((size_t)k * 4, 256) +
                                             align_up(P.hops.size() * 4, 256) + dirty_bytes);
    if (!P.base) return DM_ERR_NOMEM;
    return DM_OK;
}

// All ranks of the communicator agree that every rank prepared its part of
// the migration (min-reduction of a flag over RCCL on the ctx stream) before
// any rank posts a send or receive; a rank whose check failed reports its own
// error, the others a ValueError naming the failure elsewhere.
static int mig_agree(dm_ctx* ctx, dm_comm* comm, bool ok_here, bool* ok_all) {
    hipStream_t s = ctx->stream;
    DM_HIP(hipMemsetAsync(comm->flag, ok_here ? 1 : 0, sizeof(int32_t), s));
    DM_NCCL(ncclAllReduce(comm->flag, comm->flag, 1, ncclInt32, ncclMin, comm->comm, s));
    int32_t v = 0;
    DM_HIP(hipMemcpyAsync(&v, comm->flag, sizeof(v), hipMemcpyDeviceToHost, s));
    DM_HIP(hipStreamSynchronize(s));
    *ok_all = v != 0;
    return DM_OK;
}

static int mig_ring_impl(dm_ctx* ctx, dm_comm* comm, int32_t n_local, dm_pop* demes,
                         const int32_t* deme_ids, int32_t n_demes, const int32_t* migarray,
                         const int32_t* owner, int64_t k, int32_t* const* emig_idx,
                         int32_t* const* immig_idx, int32_t* const* out_slots, int32_t flags) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    MigPlan P;
    int rc = mig_prepare(ctx, comm, n_local, demes, deme_ids, n_demes, migarray, owner, k,
                         emig_idx, flags, P);
    if (comm && comm->nranks > 1) {
        std::string mine = rc ? std::string(dm_last_error()) : std::string();
        bool all = false;
        int arc = mig_agree(ctx, comm, rc == DM_OK, &all);
        if (arc) return arc;
        if (rc) {
            set_error("%s", mine.c_str());
            return rc;
        }
        DM_CHECK_ARG(all, "migRing: another rank rejected this migration (see its error)");
    } else if (rc) {
        return rc;
    }
    if (k == 0 || n_local == 0) return DM_OK;
    const std::vector<dm_mig_hop>& hops = P.hops;
    const std::vector<int32_t>& local_of = P.local_of;
    const size_t bb = P.bb;
    char* base = P.base;
    hipStream_t s = ctx->stream;
    std::vector<char*> emig(n_local), immig(n_local);
    // migration.py:39-46: every deme's emigrants / immigrants first
    for (int32_t i = 0; i < n_local; ++i) {
        emig[i] = base + 2 * (size_t)i * bb;
        if ((rc = dm_pack_rows(ctx, &demes[i], emig_idx[i], k, emig[i]))) return rc;
        if (immig_idx && immig_idx[i]) {
            immig[i] = emig[i] + bb;
            if ((rc = dm_pack_rows(ctx, &demes[i], immig_idx[i], k, immig[i]))) return rc;
        } else {
            immig[i] = emig[i];
        }
    }
    // exchange: the incoming block of every hop into a local deme
    std::vector<char*> incoming(hops.size(), nullptr);
    if (P.nrecv || std::any_of(hops.begin(), hops.end(),
                               [](const dm_mig_hop& h) { return h.kind == DM_HOP_SEND; })) {
        const size_t bytes = (size_t)block_bytes(&demes[0], k);
        char* rb = base + 2 * (size_t)n_local * bb;
        DM_NCCL(ncclGroupStart());
        for (size_t h = 0; h < hops.size(); ++h) {
            const dm_mig_hop& hp = hops[h];
            if (hp.kind == DM_HOP_SEND) {
                DM_NCCL(ncclSend(emig[local_of[hp.from]], bytes, ncclUint8, hp.peer, comm->comm, s));
            } else if (hp.kind == DM_HOP_RECV) {
                incoming[h] = rb;
                rb += bb;
                DM_NCCL(ncclRecv(incoming[h], bytes, ncclUint8, hp.peer, comm->comm, s));
            }
        }
        DM_NCCL(ncclGroupEnd());
    }
    for (size_t h = 0; h < hops.size(); ++h)
        if (hops[h].kind == DM_HOP_LOCAL) incoming[h] = emig[local_of[hops[h].from]];
    // migration.py:48-51: placements in from_deme order, asynchronous; one
    // status word per hop, copied back and checked once at the end
    int32_t* slot_scratch = (int32_t*)(base + 2 * (size_t)n_local * bb + (size_t)P.nrecv * bb);
    int32_t* errs = (int32_t*)((char*)slot_scratch + align_up((size_t)k * 4, 256));
    char* dptr = (char*)errs + align_up(hops.size() * 4, 256);
    std::vector<unsigned long long*> dirty(n_local, nullptr);
    for (int32_t i = 0; i < n_local; ++i) {
        if (P.hops_into[i] <= 1) continue;
        const size_t db = (size_t)(demes[i].n + 63) / 64 * 8;
        dirty[i] = (unsigned long long*)dptr;
        DM_HIP(hipMemsetAsync(dirty[i], 0, db, s));
        dptr += align_up(db, 256);
    }
    DM_HIP(hipMemsetAsync(errs, 0, hops.size() * 4, s));
    for (size_t h = 0; h < hops.size(); ++h) {
        if (!incoming[h]) continue;
        const int32_t t = local_of[hops[h].to];
        int32_t* slots = out_slots && out_slots[t] ? out_slots[t] : slot_scratch;
        const bool self_hop = hops[h].kind == DM_HOP_LOCAL && hops[h].from == hops[h].to;
        if ((rc = mig_place_async(ctx, &demes[t], immig[t], incoming[h], k, slots, dirty[t],
                                  errs + h, self_hop ? emig_idx[t] : nullptr)))
            return rc;
    }
    std::vector<int32_t> herr(hops.size(), 0);
    DM_HIP(hipMemcpyAsync(herr.data(), errs, hops.size() * 4, hipMemcpyDeviceToHost, s));
    DM_HIP(hipStreamSynchronize(s));
    for (size_t h = 0; h < hops.size(); ++h)
        DM_CHECK_ARG(herr[h] == 0, "migRing: immigrant %d of deme %d is not in the receiving "
                     "population", herr[h] - 1, hops[h].to);
    return DM_OK;
}

}  // namespace dm

extern "C" int dm_mig_plan(int32_t n_demes, const int32_t* migarray, const int32_t* owner,
                           int32_t me, int32_t flags, dm_mig_hop* hops, int32_t cap,
                           int32_t* nhops) {
    DM_CHECK_ARG(nhops != nullptr && n_demes >= 1 && cap >= 0 && (hops || cap == 0),
                 "bad argument");
    std::vector<dm_mig_hop> v;
    int rc = plan_hops(n_demes, migarray, owner, me, flags, v);
    if (rc) return rc;
    *nhops = (int32_t)v.size();
    DM_CHECK_ARG((int32_t)v.size() <= cap, "hop buffer too small (%d needed)", (int)v.size());
    std::copy(v.begin(), v.end(), hops);
    return DM_OK;
}

extern "C" int dm_mig_ring(dm_ctx* ctx, int32_t n_demes, dm_pop* demes, const int32_t* migarray,
                           int64_t k, int32_t* const* emig_idx, int32_t* const* immig_idx,
                           int32_t* const* out_slots) {
    DM_CHECK_ARG(n_demes >= 1 && n_demes <= 65536, "bad deme count");
    std::vector<int32_t> ids(n_demes);
    for (int32_t i = 0; i < n_demes; ++i) ids[i] = i;
    return mig_ring_impl(ctx, nullptr, n_demes, demes, ids.data(), n_demes, migarray, nullptr, k,
                         emig_idx, immig_idx, out_slots, 0);
}

extern "C" int dm_mig_ring_rccl(dm_ctx* ctx, dm_comm* comm, int32_t n_local, dm_pop* demes,
                                const int32_t* deme_ids, int32_t n_demes,
                                const int32_t* migarray, const int32_t* owner, int64_t k,
                                int32_t* const* emig_idx, int32_t* const* immig_idx,
                                int32_t* const* out_slots, int32_t flags) {
    DM_CHECK_ARG(comm != nullptr && owner != nullptr, "null comm / owner");
    return mig_ring_impl(ctx, comm, n_local, demes, deme_ids, n_demes, migarray, owner, k,
                         emig_idx, immig_idx, out_slots, flags);
}

extern "C" int dm_comm_get_unique_id(uint8_t* id_out) {
    DM_CHECK_ARG(id_out != nullptr, "null id");
    static_assert(sizeof(ncclUniqueId) == DM_COMM_ID_BYTES, "unique id size");
    ncclUniqueId id;
    DM_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return DM_OK;
}

extern "C" int dm_comm_init(dm_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id,
                            dm_comm** out) {
    DM_CHECK_ARG(ctx && id && out, "null argument");
    DM_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank %d of %d", rank, nranks);
    DM_HIP(hipSetDevice(ctx->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    dm_comm* c = new dm_comm();
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        delete c;
        return DM_ERR_HIP;
    }
    c->nranks = nranks;
    c->rank = rank;
    if (hipMalloc(&c->flag, 256) != hipSuccess) {
        set_error("hipMalloc of the communicator's flag word failed");
        ncclCommDestroy(c->comm);
        delete c;
        return DM_ERR_NOMEM;
    }
    *out = c;
    return DM_OK;
}

extern "C" int dm_comm_destroy(dm_comm* comm) {
    if (!comm) return DM_OK;
    ncclResult_t r = comm->comm ? ncclCommDestroy(comm->comm) : ncclSuccess;
    if (comm->flag) (void)hipFree(comm->flag);
    delete comm;
    if (r != ncclSuccess) {
        set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return DM_ERR_HIP;
    }
    return DM_OK;
}
