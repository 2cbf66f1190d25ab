// Host stand-ins for the library pieces the emulated NSGA-II units call but
// that are not under test here (tools_cpu/bdemu): the sort / scan primitives
// (sort.hip; exercised against numpy by tests/test_gpu_sort.py), the context's
// scratch arenas and the error string (capi.hip).  The sorts are the same
// stable orders the device primitives produce.
#include <stdarg.h>

#include <numeric>
#include <vector>

#if defined(__has_feature)
#if __has_feature(memory_sanitizer)
#include <sanitizer/msan_interface.h>
#endif
#endif
#include "common.hpp"
#include "sort.hpp"

#if defined(__SANITIZE_ADDRESS__)
#include <sanitizer/asan_interface.h>
#define EMU_POISON(p, n) __asan_poison_memory_region((p), (n))
#define EMU_UNPOISON(p, n) __asan_unpoison_memory_region((p), (n))
#else
#define EMU_POISON(p, n) ((void)(p), (void)(n))
#define EMU_UNPOISON(p, n) ((void)(p), (void)(n))
#endif

namespace dm {

static thread_local char g_err[1024];
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    fprintf(stderr, "dm error: %s\n", g_err);
}

int validate_pop(const dm_pop* p, const char* what) {
    DM_CHECK_ARG(p != nullptr, "%s: null population", what);
    DM_CHECK_ARG(p->n >= 0, "%s: negative size", what);
    DM_CHECK_ARG(p->nobj >= 1 && p->nobj <= DM_MAX_OBJ, "%s: nobj", what);
    return DM_OK;
}

// Grow-only arenas as the library keeps them, with every byte past the size
// of the latest request poisoned for ASan: an access past what the caller
// asked for is reported even when the arena is larger.
struct Arena {
    char* p = nullptr;
    size_t cap = 0;
};
static Arena g_slots[dm_ctx::kSlots + 1];
static void* arena_get(Arena& a, size_t bytes) {
    if (bytes > a.cap) {
        if (a.p) {
            EMU_UNPOISON(a.p, a.cap);
            free(a.p);
        }
        a.cap = (bytes + 255) / 256 * 256;
        a.p = (char*)aligned_alloc(256, a.cap);
        // EMU_ARENA_FILL: the byte new arenas start with (0xC3 by default, so
        // a read before any write shows; 0 mimics a fresh process's memory)
        static const int fill =
            getenv("EMU_ARENA_FILL") ? (int)strtol(getenv("EMU_ARENA_FILL"), nullptr, 0) : 0xC3;
        memset(a.p, fill, a.cap);
#if defined(__has_feature)
#if __has_feature(memory_sanitizer)
        // a new device allocation holds no defined values; EMU_MSAN_ARENA=0 keeps
        // them defined (the epoch-stamped front state is read before it is
        // written by design: a stale entry never carries the call's epoch)
        if (!getenv("EMU_MSAN_ARENA") || atoi(getenv("EMU_MSAN_ARENA")) != 0) __msan_poison(a.p, a.cap);
#endif
#endif
    }
    EMU_UNPOISON(a.p, a.cap);
    EMU_POISON(a.p + bytes, a.cap - bytes);
    return a.p;
}
void* scratch_slot(dm_ctx*, int slot, size_t bytes) { return arena_get(g_slots[slot], bytes); }
void* pinned(dm_ctx*, size_t bytes) { return arena_get(g_slots[dm_ctx::kSlots], bytes); }

size_t radix_sort_temp_bytes(int64_t) { return 256; }
size_t radix_sort_batched_temp_bytes(int64_t, int64_t) { return 256; }
size_t scan_temp_bytes(int64_t) { return 256; }

static void stable_sort_bits(uint64_t* keys, int32_t* vals, int64_t n, int b, int e) {
    const uint64_t mask = (e - b >= 64) ? ~0ull : (((1ull << (e - b)) - 1) << b);
    std::vector<int64_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(),
                     [&](int64_t x, int64_t y) { return (keys[x] & mask) < (keys[y] & mask); });
    std::vector<uint64_t> k(n);
    std::vector<int32_t> v(n);
    for (int64_t i = 0; i < n; ++i) {
        k[i] = keys[idx[i]];
        v[i] = vals[idx[i]];
    }
    std::copy(k.begin(), k.end(), keys);
    std::copy(v.begin(), v.end(), vals);
}
int radix_sort_pairs(hipStream_t, uint64_t* keys, int32_t* vals, uint64_t*, int32_t*, int64_t n,
                     int b, int e, void*) {
    stable_sort_bits(keys, vals, n, b, e);
    return DM_OK;
}
int radix_sort_pairs_any(hipStream_t s, uint64_t* keys, int32_t* vals, uint64_t* kt, int32_t* vt,
                         int64_t n, int b, int e, void* t, bool* in_tmp) {
    *in_tmp = false;
    return radix_sort_pairs(s, keys, vals, kt, vt, n, b, e, t);
}
int radix_sort_pairs_batched(hipStream_t, uint64_t* keys, int32_t* vals, uint64_t*, int32_t*,
                             int64_t nseg, int64_t seglen, int b, int e, void*, bool* in_tmp) {
    for (int64_t g = 0; g < nseg; ++g) stable_sort_bits(keys + g * seglen, vals + g * seglen, seglen, b, e);
    if (in_tmp) *in_tmp = false;
    return DM_OK;
}
int exclusive_scan_i32(hipStream_t, const int32_t* in, int32_t* out, int64_t n, int32_t* total,
                       void*) {
    int32_t acc = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t x = in[i];
        out[i] = acc;
        acc += x;
    }
    if (total) *total = acc;
    return DM_OK;
}
int inclusive_max_scan_i32(hipStream_t, const int32_t* in, int32_t* out, int64_t n, void*) {
    int32_t acc = INT32_MIN;
    for (int64_t i = 0; i < n; ++i) out[i] = acc = std::max(acc, in[i]);
    return DM_OK;
}
// sort.hip lex_sort_rows: LSD over objectives (last first), each a stable
// sort of the ordered keys of that objective.
#ifdef EMU_PRE
int lex_sort_rows(hipStream_t s, const double* wv, int nobj, int64_t n, bool desc, uint64_t* keys,
                  uint64_t* ktmp, int32_t* vals, int32_t* vtmp, void* rtemp, int nlex) {
    const int begin_bit = 0;
#else
int lex_sort_rows(hipStream_t s, const double* wv, int nobj, int64_t n, bool desc, uint64_t* keys,
                  uint64_t* ktmp, int32_t* vals, int32_t* vtmp, void* rtemp, int nlex,
                  int begin_bit) {
#endif
    for (int64_t i = 0; i < n; ++i) vals[i] = (int32_t)i;
    if (nlex < 0 || nlex > nobj) nlex = nobj;
    for (int o = nlex - 1; o >= 0; --o) {
        for (int64_t i = 0; i < n; ++i) {
            const uint64_t k = ordered_key(wv[(int64_t)vals[i] * nobj + o]);
            keys[i] = desc ? ~k : k;
        }
        radix_sort_pairs(s, keys, vals, ktmp, vtmp, n, begin_bit, 64, rtemp);
    }
    return DM_OK;
}
int sort_by_fitness(dm_ctx* ctx, const double* wv, int nobj, int64_t n, bool desc, int32_t* out) {
    std::vector<uint64_t> k(n), kt(n);
    std::vector<int32_t> vt(n);
    return lex_sort_rows(ctx->stream, wv, nobj, n, desc, k.data(), kt.data(), out, vt.data(), nullptr);
}
#ifndef EMU_PRE
// sort.hip seg_sort_pairs_small: every segment [starts[g], starts[g + 1])
// stably by key bits [begin_bit, end_bit)
int seg_sort_pairs_small(hipStream_t, uint64_t* keys, int32_t* vals, const int32_t* starts,
                         int64_t nseg, int b, int e, uint64_t*, int32_t*) {
    for (int64_t g = 0; g < nseg; ++g)
        stable_sort_bits(keys + starts[g], vals + starts[g], starts[g + 1] - starts[g], b, e);
    return DM_OK;
}
#endif

}  // namespace dm
