// HBM ceilings for the packed-bit generation's access pattern (not part of the
// product): 512-B rows (OneMax-4096), one wave per offspring pair, random
// parent rows, sequential child rows.  A: lane L moves word L of each row
// (8 B/lane, 512 B per instruction, 2 loads + 2 stores per pair); B: lanes
// 0-31 move row s0 and lanes 32-63 row s1 as 16 B/lane (1 KiB per
// instruction, 1 load + 1 store per pair); PP pairs per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned long long u64;
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int PP>
__global__ __launch_bounds__(256) void rows8(const char* __restrict__ a, char* __restrict__ b,
                                             const int* __restrict__ idx, int npairs) {
    const int lane = threadIdx.x & 63;
    const int w = (blockIdx.x * 256 + threadIdx.x) >> 6;
    u64 x[PP], y[PP];
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int p = w * PP + k;
        if (p < npairs) {
            x[k] = ((const u64*)(a + (long)idx[2 * p] * 512))[lane];
            y[k] = ((const u64*)(a + (long)idx[2 * p + 1] * 512))[lane];
        }
    }
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int p = w * PP + k;
        if (p < npairs) {
            __builtin_nontemporal_store(x[k] ^ y[k], (u64*)(b + (long)(2 * p) * 512) + lane);
            __builtin_nontemporal_store(x[k] + y[k], (u64*)(b + (long)(2 * p + 1) * 512) + lane);
        }
    }
}
template <int PP>
__global__ __launch_bounds__(256) void rows16(const char* __restrict__ a, char* __restrict__ b,
                                              const int* __restrict__ idx, int npairs) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const int w = (blockIdx.x * 256 + threadIdx.x) >> 6;
    u4 x[PP];
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int p = w * PP + k;
        if (p < npairs) x[k] = ((const u4*)(a + (long)idx[2 * p + h] * 512))[l];
    }
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int p = w * PP + k;
        if (p < npairs) {
            u4 o;
            o.x = __shfl_xor(x[k].x, 32, 64); o.y = __shfl_xor(x[k].y, 32, 64);
            o.z = __shfl_xor(x[k].z, 32, 64); o.w = __shfl_xor(x[k].w, 32, 64);
            __builtin_nontemporal_store(x[k] ^ o, (u4*)(b + (long)(2 * p + h) * 512) + l);
        }
    }
}

int main() {
    const int rows = 1 << 20;
    const size_t bytes = (size_t)rows * 512;
    char *a, *b;
    int* ir;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&ir, rows * 4);
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    std::vector<int> h(rows);
    unsigned s = 1;
    for (int i = 0; i < rows; ++i) { s = s * 1664525u + 1013904223u; h[i] = (s >> 8) % rows; }
    hipMemcpy(ir, h.data(), rows * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, double traffic, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 20;
        printf("%-36s %8.4f ms  %7.1f GB/s\n", name, ms, traffic / ms / 1e6);
        fflush(stdout);
    };
    const double copyb = 2.0 * 512.0 * rows;
    const int np = rows / 2;
#define R8(PP) run("rows8 pp=" #PP, copyb, [&] { rows8<PP><<<(np / PP * 64 + 255) / 256, 256>>>(a, b, ir, np); });
#define R16(PP) run("rows16 pp=" #PP, copyb, [&] { rows16<PP><<<(np / PP * 64 + 255) / 256, 256>>>(a, b, ir, np); });
    R8(1) R8(2) R8(4) R8(8) R16(1) R16(2) R16(4) R16(8)
    return 0;
}
