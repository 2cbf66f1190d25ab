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
//      immigrant j, whichever index is smaller; it copies emigrant j there and
//      clears that row from the later bitmaps.
#include "common.hpp"

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

// bitmap[j][w]: bit r%64 of word r/64 set iff row r equals immigrant j.
__global__ void match_kernel(const char* genes, const double* wv, const uint8_t* valid, int64_t n,
                             int64_t stride, int dim, int gtype, int nobj, const void* imm_block,
                             int64_t k, int64_t words, unsigned long long* bitmap) {
    Block im = block_view((void*)imm_block, stride, nobj, k);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        for (int64_t j = 0; j < k; ++j) {
            if (!fit_prefilter(wv + r * nobj, valid[r], im.wv + j * nobj, im.valid[j], nobj))
                continue;
            if (genome_eq(genes + r * stride, im.genes + j * stride, gtype, dim))
                atomicOr(&bitmap[j * words + (r >> 6)], 1ull << (r & 63));
        }
    }
}

// E[e*k + j] = emigrant e == immigrant j (genome)
__global__ void em_im_eq_kernel(const void* em_block, const void* im_block, int64_t k,
                                int64_t stride, int dim, int gtype, int nobj, uint8_t* E) {
    Block em = block_view((void*)em_block, stride, nobj, k);
    Block im = block_view((void*)im_block, stride, nobj, k);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k * k;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = t / k, j = t % k;
        E[t] = genome_eq(em.genes + e * stride, im.genes + j * stride, gtype, dim) ? 1 : 0;
    }
}

// Sequential resolution; one workgroup of 256 threads.
__global__ __launch_bounds__(256) void resolve_kernel(char* genes, double* wv, uint8_t* valid,
                                                      int64_t n, int64_t stride, int nobj,
                                                      const void* em_block, int64_t k,
                                                      int64_t words, unsigned long long* bitmap,
                                                      const uint8_t* E, int32_t* slots,
                                                      int32_t* content, int32_t* err) {
    Block em = block_view((void*)em_block, stride, nobj, k);
    __shared__ int64_t best;
    __shared__ int32_t placed_slot[256];
    __shared__ int32_t placed_em[256];
    __shared__ int nplaced;
    if (threadIdx.x == 0) nplaced = 0;
    __syncthreads();
    for (int64_t j = 0; j < k; ++j) {
        if (threadIdx.x == 0) best = INT64_MAX;
        __syncthreads();
        // (a) first original match still present: scan words in blocks of 256
        for (int64_t wb = 0; wb < words; wb += blockDim.x) {
            const int64_t w = wb + threadIdx.x;
            if (w < words) {
                const unsigned long long x = bitmap[j * words + w];
                if (x) atomicMin((unsigned long long*)&best, (unsigned long long)(w * 64 + __ffsll(x) - 1));
            }
            __syncthreads();
            if (best != INT64_MAX) break;
            __syncthreads();
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t slot = best;
            // (b) already-placed emigrants equal to immigrant j
            for (int p = 0; p < nplaced; ++p) {
                const int32_t s = placed_slot[p];
                if (content[s] == placed_em[p] && E[(int64_t)placed_em[p] * k + j] && s < slot)
                    slot = s;
            }
            if (slot == INT64_MAX || slot >= n) {
                *err = (int32_t)j + 1;  // list.index -> ValueError
                best = -1;
            } else {
                best = slot;
                slots[j] = (int32_t)slot;
                content[slot] = (int32_t)j;
                if (nplaced < 256) {
                    placed_slot[nplaced] = (int32_t)slot;
                    placed_em[nplaced] = (int32_t)j;
                    ++nplaced;
                }
            }
        }
        __syncthreads();
        const int64_t slot = best;
        if (slot < 0) return;
        // copy emigrant j into the slot
        const uint4* src = reinterpret_cast<const uint4*>(em.genes + j * stride);
        uint4* dst = reinterpret_cast<uint4*>(genes + slot * stride);
        for (int64_t i = threadIdx.x; i < stride / 16; i += blockDim.x) dst[i] = src[i];
        if (threadIdx.x < nobj) wv[slot * nobj + threadIdx.x] = em.wv[j * nobj + threadIdx.x];
        if (threadIdx.x == 0) valid[slot] = em.valid[j];
        // the row no longer holds its original genome
        for (int64_t jj = j + 1 + threadIdx.x; jj < k; jj += blockDim.x)
            bitmap[jj * words + (slot >> 6)] &= ~(1ull << (slot & 63));
        __threadfence_block();
        __syncthreads();
    }
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

extern "C" int dm_mig_place(dm_ctx* ctx, dm_pop* pop, const void* immigrant_block,
                            const void* emigrant_block, int64_t k, int32_t* out_slots) {
    DM_CHECK_ARG(ctx && pop && immigrant_block && emigrant_block && out_slots, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0 && k <= 4096, "k must be in [0, 4096]");
    if (k == 0) return DM_OK;
    const int64_t n = pop->n;
    const int64_t words = (n + 63) / 64;
    const size_t bm = align_up((size_t)k * words * 8, 256);
    char* base = (char*)scratch_slot(ctx, 3, bm + align_up((size_t)k * k, 256) +
                                                 align_up((size_t)std::max<int64_t>(n, 1) * 4, 256) + 256);
    if (!base) return DM_ERR_NOMEM;
    unsigned long long* bitmap = (unsigned long long*)base;
    uint8_t* E = (uint8_t*)(base + bm);
    int32_t* content = (int32_t*)(base + bm + align_up((size_t)k * k, 256));
    int32_t* err = (int32_t*)(base + bm + align_up((size_t)k * k, 256) +
                              align_up((size_t)std::max<int64_t>(n, 1) * 4, 256));
    hipStream_t s = ctx->stream;
    DM_HIP(hipMemsetAsync(bitmap, 0, (size_t)k * words * 8, s));
    DM_HIP(hipMemsetAsync(err, 0, 4, s));
    DM_HIP(hipMemsetAsync(content, 0xFF, (size_t)std::max<int64_t>(n, 1) * 4, s));
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
    match_kernel<<<grid, 256, 0, s>>>((const char*)pop->genes, pop->wvalues, pop->valid, n,
                                      pop->stride, pop->dim, pop->gtype, pop->nobj,
                                      immigrant_block, k, words, bitmap);
    em_im_eq_kernel<<<(unsigned)std::max<int64_t>(1, (k * k + 255) / 256), 256, 0, s>>>(
        emigrant_block, immigrant_block, k, pop->stride, pop->dim, pop->gtype, pop->nobj, E);
    resolve_kernel<<<1, 256, 0, s>>>((char*)pop->genes, pop->wvalues, pop->valid, n, pop->stride,
                                     pop->nobj, emigrant_block, k, words, bitmap, E, out_slots,
                                     content, err);
    DM_LAUNCH_CHECK();
    int32_t herr = 0;
    DM_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
    DM_HIP(hipStreamSynchronize(s));
    DM_CHECK_ARG(herr == 0, "migRing: immigrant %d is not in the receiving population", herr - 1);
    return DM_OK;
}
