// HBM ceilings on this box for the generation's traffic (not part of the
// product): flat float4 copy / read / write of 8.4 GB beside the row-pair
// gather-copy the hot kernel performs (one wave per pair, 1 KiB per wave
// instruction, random parents, 8064-B row stride).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void flat_copy(const u4* __restrict__ a, u4* __restrict__ b, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        u4 v = a[i];
        if (NT) __builtin_nontemporal_store(v, b + i); else b[i] = v;
    }
}
// 4 independent loads per thread before the stores (more bytes in flight)
template <bool NT>
__global__ __launch_bounds__(256) void flat_copy4(const u4* __restrict__ a, u4* __restrict__ b, long n) {
    const long st = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i + 3 * st < n; i += 4 * st) {
        u4 v0 = a[i], v1 = a[i + st], v2 = a[i + 2 * st], v3 = a[i + 3 * st];
        if (NT) {
            __builtin_nontemporal_store(v0, b + i); __builtin_nontemporal_store(v1, b + i + st);
            __builtin_nontemporal_store(v2, b + i + 2 * st); __builtin_nontemporal_store(v3, b + i + 3 * st);
        } else { b[i] = v0; b[i + st] = v1; b[i + 2 * st] = v2; b[i + 3 * st] = v3; }
    }
}
__global__ __launch_bounds__(256) void flat_read(const u4* __restrict__ a, u4* __restrict__ out, long n) {
    u4 acc = {0, 0, 0, 0};
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}
template <bool NT>
__global__ __launch_bounds__(256) void flat_write(u4* __restrict__ b, long n) {
    const u4 v = {1, 2, 3, 4};
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store(v, b + i); else b[i] = v;
    }
}
// row-pair gather-copy (the hot kernel's memory pattern); SPLIT: the four
// waves of a workgroup share one pair (each a quarter of both rows)
template <bool NT, bool SPLIT>
__global__ __launch_bounds__(256) void pair_copy(const char* __restrict__ a, char* __restrict__ b,
                                                 const int* __restrict__ idx, int npairs, long stride) {
    const int lane = threadIdx.x & 63;
    if (!SPLIT) {
        const int nw = (gridDim.x * 256) >> 6;
        for (int p = (blockIdx.x * 256 + threadIdx.x) >> 6; p < npairs; p += nw) {
            const u4* r0 = (const u4*)(a + (long)idx[2 * p] * stride);
            const u4* r1 = (const u4*)(a + (long)idx[2 * p + 1] * stride);
            u4* w0 = (u4*)(b + (long)(2 * p) * stride);
            u4* w1 = (u4*)(b + (long)(2 * p + 1) * stride);
            u4 v0[8], v1[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { const int q = lane + 64 * u; if (q < 500) { v0[u] = r0[q]; v1[u] = r1[q]; } }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = lane + 64 * u;
                if (q < 500) {
                    if (NT) { __builtin_nontemporal_store(v0[u], w0 + q); __builtin_nontemporal_store(v1[u], w1 + q); }
                    else { w0[q] = v0[u]; w1[q] = v1[u]; }
                }
            }
        }
    } else {
        const int wv = threadIdx.x >> 6;
        for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
            const u4* r0 = (const u4*)(a + (long)idx[2 * p] * stride);
            const u4* r1 = (const u4*)(a + (long)idx[2 * p + 1] * stride);
            u4* w0 = (u4*)(b + (long)(2 * p) * stride);
            u4* w1 = (u4*)(b + (long)(2 * p + 1) * stride);
            u4 v0[2], v1[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) { const int q = lane + 64 * (2 * wv + u); if (q < 500) { v0[u] = r0[q]; v1[u] = r1[q]; } }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = lane + 64 * (2 * wv + u);
                if (q < 500) {
                    if (NT) { __builtin_nontemporal_store(v0[u], w0 + q); __builtin_nontemporal_store(v1[u], w1 + q); }
                    else { w0[q] = v0[u]; w1[q] = v1[u]; }
                }
            }
        }
    }
}

int main() {
    const int rows = 1 << 20;
    const long stride = 8064;
    const size_t bytes = (size_t)rows * stride;
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
    int dev; hipGetDevice(&dev); hipDeviceProp_t pr; hipGetDeviceProperties(&pr, dev);
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char* name, double traffic, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, traffic / ms / 1e6);
        fflush(stdout);
    };
    const long n4 = (long)rows * 8000 / 16;  // float4 elements of 8.0 GB
    const double copyb = 2.0 * 8000.0 * rows;
    char nm[96];
    for (int bpc : {4, 8, 16, 32}) {
        const int g = cus * bpc;
        snprintf(nm, 96, "flat copy plain bpc=%d", bpc);
        run(nm, copyb, [&] { flat_copy<false><<<g, 256>>>((const u4*)a, (u4*)b, n4); });
        snprintf(nm, 96, "flat copy nt bpc=%d", bpc);
        run(nm, copyb, [&] { flat_copy<true><<<g, 256>>>((const u4*)a, (u4*)b, n4); });
        snprintf(nm, 96, "flat copy4 nt bpc=%d", bpc);
        run(nm, copyb, [&] { flat_copy4<true><<<g, 256>>>((const u4*)a, (u4*)b, n4); });
        snprintf(nm, 96, "flat read bpc=%d", bpc);
        run(nm, copyb / 2, [&] { flat_read<<<g, 256>>>((const u4*)a, (u4*)b, n4); });
        snprintf(nm, 96, "flat write nt bpc=%d", bpc);
        run(nm, copyb / 2, [&] { flat_write<true><<<g, 256>>>((u4*)b, n4); });
        snprintf(nm, 96, "flat write plain bpc=%d", bpc);
        run(nm, copyb / 2, [&] { flat_write<false><<<g, 256>>>((u4*)b, n4); });
    }
    {
        const long nn = n4;
        const int g = (int)((nn + 255) / 256);
        run("flat copy plain one-shot grid", copyb, [&] { flat_copy<false><<<g, 256>>>((const u4*)a, (u4*)b, nn); });
        run("flat copy nt one-shot grid", copyb, [&] { flat_copy<true><<<g, 256>>>((const u4*)a, (u4*)b, nn); });
    }
    const int np = rows / 2;
    for (int bpc : {2, 4, 8}) {
        const int g = cus * bpc;
        snprintf(nm, 96, "pair copy nt rand bpc=%d", bpc);
        run(nm, copyb, [&] { pair_copy<true, false><<<g, 256>>>(a, b, ir, np, stride); });
        snprintf(nm, 96, "pair copy nt rand split bpc=%d", bpc);
        run(nm, copyb, [&] { pair_copy<true, true><<<g, 256>>>(a, b, ir, np, stride); });
        snprintf(nm, 96, "pair copy plain rand split bpc=%d", bpc);
        run(nm, copyb, [&] { pair_copy<false, true><<<g, 256>>>(a, b, ir, np, stride); });
    }
    return 0;
}
