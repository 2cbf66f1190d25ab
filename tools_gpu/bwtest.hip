// Streaming-bandwidth ceilings on this box (not part of the product):
// copy / read / write of a 8.4 GB buffer with 16-B lanes, U loads in flight.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <int U>
__global__ __launch_bounds__(256) void copy_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n) v[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n) b[i + u * 256] = v[u];
    }
}
template <int U>
__global__ __launch_bounds__(256) void copy_nt_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n) v[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n) { typedef unsigned int u4 __attribute__((ext_vector_type(4))); u4 t = {v[u].x, v[u].y, v[u].z, v[u].w}; __builtin_nontemporal_store(t, (u4*)&b[i + u * 256]); }
    }
}
// row gather: one wave per 8000-B row, random source rows, all 8 pieces in flight
__global__ __launch_bounds__(256) void gather_k(const char* a, char* b, const int* idx, int rows, int rowb) {
    const int lane = threadIdx.x & 63;
    for (int r = (blockIdx.x * 256 + threadIdx.x) >> 6; r < rows; r += (gridDim.x * 256) >> 6) {
        const uint4* s = (const uint4*)(a + (size_t)idx[r] * rowb);
        uint4* d = (uint4*)(b + (size_t)r * rowb);
        const int q = rowb / 16;
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) if (lane + 64 * u < q) v[u] = s[lane + 64 * u];
#pragma unroll
        for (int u = 0; u < 8; ++u) if (lane + 64 * u < q) d[lane + 64 * u] = v[u];
    }
}
int main() {
    const size_t bytes = (size_t)(1 << 20) * 8000;
    const size_t n = bytes / 16;
    uint4 *a, *b;
    int* idx;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&idx, (1 << 20) * 4);
    hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
    std::vector<int> h(1 << 20);
    unsigned s = 1; for (int i = 0; i < (1 << 20); ++i) { s = s * 1664525u + 1013904223u; h[i] = (s >> 8) % (1 << 20); }
    hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0); for (int r = 0; r < 10; ++r) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 10;
        printf("%-28s %8.3f ms  %7.1f GB/s (read+write)\n", name, ms, 2.0 * bytes / ms / 1e6);
    };
    for (int g : {1024, 2048, 4096, 16384}) {
        char nm[64];
        snprintf(nm, 64, "copy U=4 grid=%d", g); run(nm, [&] { copy_k<4><<<g, 256>>>(a, b, n); });
        snprintf(nm, 64, "copy U=8 grid=%d", g); run(nm, [&] { copy_k<8><<<g, 256>>>(a, b, n); });
        snprintf(nm, 64, "copy_nt U=8 grid=%d", g); run(nm, [&] { copy_nt_k<8><<<g, 256>>>(a, b, n); });
    }
    for (int g : {1024, 4096, 16384})  {
        char nm[64]; snprintf(nm, 64, "gather rows grid=%d", g);
        run(nm, [&] { gather_k<<<g, 256>>>((const char*)a, (char*)b, idx, 1 << 20, 8000); });
    }
    return 0;
}
