// Host emulation of the HIP subset the NSGA-II fast path uses (tools_cpu/bdemu).
//
// NOT a GPU runtime: it exists to run the library's own kernel sources on the
// CPU under AddressSanitizer / UBSan / gdb (the m = 4
// bitset fault).  Every lane of a workgroup is an OS thread; __syncthreads is
// a block barrier; wave operations (ballot, shuffles, DPP, permlane swaps,
// readfirstlane) exchange values through a per-wave slot array between two
// wave barriers.  __shared__ arrays become function-static objects, so each
// one gets its own ASan redzones: an out-of-range LDS index is reported.
// Workgroups of a launch run one after another in blockIdx order (a
// last-arriver or look-back pattern sees every earlier workgroup done).
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <functional>
#include <type_traits>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static
#define __HIP_MEMORY_SCOPE_AGENT 0
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define __HIP_MEMORY_SCOPE_SYSTEM 0
#define __HIP_MEMORY_SCOPE_WAVEFRONT 0

struct dim3 {
    unsigned x = 1, y = 1, z = 1;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct emu_u3 {
    unsigned x = 0, y = 0, z = 0;
};
extern thread_local emu_u3 threadIdx, blockIdx, blockDim, gridDim;

#define EMU_VEC4(T, N)                                  \
    struct alignas(4 * sizeof(T)) N {                   \
        T x, y, z, w;                                   \
    };                                                  \
    inline N make_##N(T a, T b, T c, T d) { return N{a, b, c, d}; }
#define EMU_VEC2(T, N)                     \
    struct alignas(2 * sizeof(T)) N {      \
        T x, y;                            \
    };                                     \
    inline N make_##N(T a, T b) { return N{a, b}; }
EMU_VEC4(int, int4)
EMU_VEC4(unsigned, uint4)
EMU_VEC4(float, float4)
EMU_VEC2(int, int2)
EMU_VEC2(unsigned, uint2)
EMU_VEC2(double, double2)
EMU_VEC2(long long, longlong2)
EMU_VEC2(float, float2)

// ---- runtime API subset ----
typedef void* hipStream_t;
typedef void* hipEvent_t;
enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2 };
enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4
};
inline const char* hipGetErrorName(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hipError"; }
inline const char* hipGetErrorString(hipError_t e) { return hipGetErrorName(e); }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipPeekAtLastError() { return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t = nullptr) {
    memset(p, v, n);
    return hipSuccess;
}
inline hipError_t hipMemset(void* p, int v, size_t n) { return hipMemsetAsync(p, v, n); }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t = nullptr) {
    memmove(d, s, n);
    return hipSuccess;
}
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind k) {
    return hipMemcpyAsync(d, s, n, k);
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t = nullptr) { return hipSuccess; }

// ---- emulator core (emu_runtime.cpp) ----
namespace emu {
struct Cfg {
    dim3 g, b;
    size_t shm;
};
inline Cfg cfg(dim3 g, dim3 b, size_t shm = 0, hipStream_t = nullptr) { return Cfg{g, b, shm}; }
void launch(const Cfg& c, const char* name, const std::function<void()>& body);
void syncthreads();
int lane();
int wave_size();
// every live lane of the wave publishes v; returns the published values (64
// slots, lanes that exited keep their last value) and the live mask
const uint64_t* wave_exchange(uint64_t v, uint64_t* live);
void* dyn_lds();
void fence();
// LDS arrays (prep.py appends EMU_LDS after each __shared__ declaration): the
// runtime fills every registered array with a poison pattern before each
// workgroup, as LDS content is undefined when a workgroup starts
void lds_register(void* p, size_t n);
[[noreturn]] void check_failed(const char* what, long long v, const char* file, int line);
}  // namespace emu
#define EMU_LDS(name)                                                         \
    do {                                                                      \
        static std::atomic<bool> emu_reg_{false};                             \
        if (!emu_reg_.exchange(true)) emu::lds_register((void*)&(name), sizeof(name)); \
    } while (0)
#define EMU_CHECK(cond, what, v) \
    ((cond) ? (void)0 : emu::check_failed(what, (long long)(v), __FILE__, __LINE__))

namespace emu {
int syncthreads_count(int p);
}
inline void __syncthreads() { emu::syncthreads(); }
inline int __syncthreads_count(int p) { return emu::syncthreads_count(p); }
inline int __syncthreads_and(int p) { return emu::syncthreads_count(!p) == 0; }
inline int __syncthreads_or(int p) { return emu::syncthreads_count(p != 0) != 0; }
inline void __threadfence() { std::atomic_thread_fence(std::memory_order_seq_cst); }
inline void __threadfence_block() { std::atomic_thread_fence(std::memory_order_seq_cst); }
inline unsigned __lane_id() { return (unsigned)emu::lane(); }

inline int __popc(unsigned x) { return __builtin_popcount(x); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __ffs(unsigned x) { return __builtin_ffs((int)x); }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __clz(unsigned x) { return x ? __builtin_clz(x) : 32; }
inline int __clzll(unsigned long long x) { return x ? __builtin_clzll(x) : 64; }
inline unsigned __brev(unsigned x) {
    unsigned r = 0;
    for (int i = 0; i < 32; ++i) r |= ((x >> i) & 1u) << (31 - i);
    return r;
}

template <class T>
inline uint64_t emu_bits(T v) {
    static_assert(sizeof(T) <= 8, "wave values of at most 8 bytes");
    uint64_t b = 0;
    memcpy(&b, &v, sizeof(T));
    return b;
}
template <class T>
inline T emu_from(uint64_t b) {
    T v;
    memcpy(&v, &b, sizeof(T));
    return v;
}

inline unsigned long long __ballot(int pred) {
    uint64_t live = 0;
    const uint64_t* s = emu::wave_exchange(pred ? 1 : 0, &live);
    unsigned long long m = 0;
    for (int i = 0; i < 64; ++i)
        if (((live >> i) & 1) && s[i]) m |= 1ull << i;
    return m;
}
inline int __any(int p) { return __ballot(p) != 0; }
inline int __all(int p) {
    uint64_t live = 0;
    const uint64_t* s = emu::wave_exchange(p ? 1 : 0, &live);
    for (int i = 0; i < 64; ++i)
        if (((live >> i) & 1) && !s[i]) return 0;
    return 1;
}

// shuffles (width divides 64; source lane computed as HIP does)
template <class T>
inline T __shfl(T v, int src, int width = 64) {
    const int l = emu::lane();
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    const int base = l & ~(width - 1);
    const int j = base + (((src % width) + width) % width);
    return emu_from<T>(s[j]);
}
template <class T>
inline T __shfl_xor(T v, int m, int width = 64) {
    const int l = emu::lane();
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    const int j = l ^ m;
    const bool ok = (j & ~(width - 1)) == (l & ~(width - 1)) && j < 64;
    return ok ? emu_from<T>(s[j]) : v;
}
template <class T>
inline T __shfl_up(T v, unsigned d, int width = 64) {
    const int l = emu::lane();
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    const int base = l & ~(width - 1);
    const int j = l - (int)d;
    return j >= base ? emu_from<T>(s[j]) : v;
}
template <class T>
inline T __shfl_down(T v, unsigned d, int width = 64) {
    const int l = emu::lane();
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    const int base = l & ~(width - 1);
    const int j = l + (int)d;
    return j < base + width ? emu_from<T>(s[j]) : v;
}

// DPP source lane of lane l for control ctrl (-1: no source)
inline int emu_dpp_src(int l, int ctrl) {
    const int r = l & ~15, i = l & 15;
    if (ctrl <= 0xFF) return (l & ~3) | ((ctrl >> (2 * (l & 3))) & 3);  // quad_perm
    if (ctrl >= 0x101 && ctrl <= 0x10F) {                             // row_shl
        const int j = i + (ctrl - 0x100);
        return j < 16 ? r + j : -1;
    }
    if (ctrl >= 0x111 && ctrl <= 0x11F) {  // row_shr
        const int j = i - (ctrl - 0x110);
        return j >= 0 ? r + j : -1;
    }
    if (ctrl >= 0x121 && ctrl <= 0x12F) return r + ((i + (ctrl - 0x120)) & 15);  // row_ror
    if (ctrl == 0x140) return r + (15 - i);                                    // row_mirror
    if (ctrl == 0x141) return (l & ~7) | (7 - (l & 7));                        // row_half_mirror
    if (ctrl == 0x142) return r >= 16 ? r - 1 : -1;                            // row_bcast:15
    if (ctrl == 0x143) return l >= 32 ? 31 : -1;                               // row_bcast:31
    if (ctrl == 0x130) return l + 1 < 64 ? l + 1 : -1;                         // wave_shl:1
    if (ctrl == 0x134) return (l + 1) & 63;                                    // wave_rol:1
    if (ctrl == 0x138) return l >= 1 ? l - 1 : -1;                             // wave_shr:1
    if (ctrl == 0x13C) return (l + 63) & 63;                                   // wave_ror:1
    fprintf(stderr, "emu: unsupported DPP control 0x%x\n", ctrl);
    abort();
}
template <class T>
inline T __builtin_amdgcn_update_dpp(T old, T src, int ctrl, int row_mask, int bank_mask, bool bound_ctrl) {
    const int l = emu::lane();
    const uint64_t* s = emu::wave_exchange(emu_bits(src), nullptr);
    if (!((row_mask >> (l >> 4)) & 1) || !((bank_mask >> ((l >> 2) & 3)) & 1)) return old;
    const int j = emu_dpp_src(l, ctrl);
    if (j < 0) return bound_ctrl ? T(0) : old;
    return emu_from<T>(s[j]);
}
template <class T>
inline T __builtin_amdgcn_mov_dpp(T src, int ctrl, int row_mask, int bank_mask, bool bound_ctrl) {
    return __builtin_amdgcn_update_dpp(T(0), src, ctrl, row_mask, bank_mask, bound_ctrl);
}
template <class T>
inline T __builtin_amdgcn_readfirstlane(T v) {
    uint64_t live = 0;
    const uint64_t* s = emu::wave_exchange(emu_bits(v), &live);
    return emu_from<T>(s[live ? __builtin_ctzll(live) : 0]);
}
template <class T>
inline T __builtin_amdgcn_readlane(T v, int j) {
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    return emu_from<T>(s[j & 63]);
}
template <class T>
inline T __builtin_amdgcn_ds_bpermute(int addr, T v) {
    const uint64_t* s = emu::wave_exchange(emu_bits(v), nullptr);
    return emu_from<T>(s[(addr >> 2) & 63]);
}
struct emu_u32pair {
    uint32_t v[2];
    uint32_t operator[](int i) const { return v[i]; }
};
// v_permlane16_swap: the odd rows of the first operand trade places with the
// even rows of the second; v_permlane32_swap: the first operand's upper half
// with the second's lower half.  Returns {first, second} after the swap.
inline emu_u32pair __builtin_amdgcn_permlane16_swap(uint32_t a, uint32_t b, bool, bool) {
    const int l = emu::lane();
    uint64_t both = ((uint64_t)b << 32) | a;
    const uint64_t* s = emu::wave_exchange(both, nullptr);
    const bool odd = (l >> 4) & 1;
    const uint32_t na = odd ? (uint32_t)(s[l - 16] >> 32) : a;  // odd row of a <- even row of b
    const uint32_t nb = odd ? b : (uint32_t)s[l + 16];          // even row of b <- odd row of a
    return emu_u32pair{{na, nb}};
}
inline emu_u32pair __builtin_amdgcn_permlane32_swap(uint32_t a, uint32_t b, bool, bool) {
    const int l = emu::lane();
    uint64_t both = ((uint64_t)b << 32) | a;
    const uint64_t* s = emu::wave_exchange(both, nullptr);
    const bool up = l >= 32;
    const uint32_t na = up ? (uint32_t)(s[l - 32] >> 32) : a;  // upper half of a <- lower half of b
    const uint32_t nb = up ? b : (uint32_t)s[l + 32];          // lower half of b <- upper half of a
    return emu_u32pair{{na, nb}};
}
inline uint32_t __builtin_amdgcn_perm(uint32_t a, uint32_t b, uint32_t sel) {
    const uint64_t c = ((uint64_t)a << 32) | b;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFF;
        uint32_t byte;
        if (s < 8) byte = (uint32_t)(c >> (8 * s)) & 0xFF;
        else if (s == 12) byte = 0x00;
        else if (s > 12) byte = 0xFF;
        else {
            fprintf(stderr, "emu: unsupported v_perm selector %u\n", s);
            abort();
        }
        r |= byte << (8 * i);
    }
    return r;
}
inline uint32_t __builtin_amdgcn_alignbit(uint32_t a, uint32_t b, uint32_t sh) {
    return (uint32_t)((((uint64_t)a << 32) | b) >> (sh & 31));
}
inline void __builtin_amdgcn_s_sleep(int) {}
inline void __builtin_amdgcn_wave_barrier() { (void)emu::wave_exchange(0, nullptr); }
inline void __builtin_amdgcn_s_setprio(int) {}
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
#define __builtin_nontemporal_load(p) (*(p))

// v_writelane_b32 / v_addc_co_u32 as the prep step rewrites the inline asm
template <class T, class U>
inline void emu_writelane(T& old, U val, int L) {
    if (emu::lane() == L) old = (T)val;
}

// ---- atomics (sequentially consistent on the host) ----
// (renamed: clang knows the __hip_atomic_* names as builtins on every target)
#define __hip_atomic_fetch_add emu__hip_atomic_fetch_add
#define __hip_atomic_fetch_max emu__hip_atomic_fetch_max
#define __hip_atomic_fetch_min emu__hip_atomic_fetch_min
#define __hip_atomic_exchange emu__hip_atomic_exchange
#define __hip_atomic_load emu__hip_atomic_load
#define __hip_atomic_store emu__hip_atomic_store
template <class T>
inline T emu__hip_atomic_fetch_add(T* p, T v, int, int) {
    return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
template <class T>
inline T emu__hip_atomic_fetch_max(T* p, T v, int, int) {
    T cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
    }
    return cur;
}
template <class T>
inline T emu__hip_atomic_fetch_min(T* p, T v, int, int) {
    T cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (cur > v && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
    }
    return cur;
}
template <class T>
inline T emu__hip_atomic_exchange(T* p, T v, int, int) {
    return __atomic_exchange_n(p, v, __ATOMIC_SEQ_CST);
}
template <class T>
inline T emu__hip_atomic_load(T* p, int, int) {
    return __atomic_load_n(p, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline void emu__hip_atomic_store(T* p, U v, int, int) {
    __atomic_store_n(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicAdd(T* p, U v) {
    return __atomic_fetch_add(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicSub(T* p, U v) {
    return __atomic_fetch_sub(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicMax(T* p, U v) {
    return __hip_atomic_fetch_max(p, (T)v, 0, 0);
}
template <class T, class U>
inline T atomicMin(T* p, U v) {
    return __hip_atomic_fetch_min(p, (T)v, 0, 0);
}
template <class T, class U>
inline T atomicOr(T* p, U v) {
    return __atomic_fetch_or(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicAnd(T* p, U v) {
    return __atomic_fetch_and(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicExch(T* p, U v) {
    return __atomic_exchange_n(p, (T)v, __ATOMIC_SEQ_CST);
}
template <class T, class U>
inline T atomicCAS(T* p, U cmp, U v) {
    T c = (T)cmp;
    __atomic_compare_exchange_n(p, &c, (T)v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
    return c;
}

// HIP's integer min / max overloads
#define EMU_MINMAX(T)                                  \
    inline T max(T a, T b) { return a > b ? a : b; } \
    inline T min(T a, T b) { return a < b ? a : b; }
EMU_MINMAX(int)
EMU_MINMAX(unsigned)
EMU_MINMAX(long)
EMU_MINMAX(unsigned long)
EMU_MINMAX(long long)
EMU_MINMAX(unsigned long long)
using ::fmax;
using ::fmin;
inline double __longlong_as_double(long long x) { return emu_from<double>((uint64_t)x); }
inline long long __double_as_longlong(double x) { return (long long)emu_bits(x); }
inline unsigned __float_as_uint(float x) { return (unsigned)emu_bits(x); }
inline float __uint_as_float(unsigned x) { return emu_from<float>(x); }
inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
inline unsigned __umulhi(unsigned a, unsigned b) { return (unsigned)(((uint64_t)a * b) >> 32); }
