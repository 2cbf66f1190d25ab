// HBM ceilings for the generation's access pattern, one-shot grids (not part
// of the product): one wave per offspring pair reads two random parent rows
// (8000 B of an 8064-B stride) and writes two sequential child rows, the grid
// covering every pair once (no persistent loop), beside the persistent form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// WPP waves per pair: wave w of a pair handles u4 slots [w*500/WPP, (w+1)*500/WPP)
template <bool NT, int WPP>
__global__ __launch_bounds__(256) void pair_oneshot(const char* __restrict__ a, char* __restrict__ b,
                                                    const int* __restrict__ idx, int npairs, long stride) {
    constexpr int PER = (500 + 64 * WPP - 1) / (64 * WPP);
    const int lane = threadIdx.x & 63;
    const int gw = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int p = gw / WPP, w = gw % WPP;
    if (p >= npairs) return;
    const u4* r0 = (const u4*)(a + (long)idx[2 * p] * stride);
    const u4* r1 = (const u4*)(a + (long)idx[2 * p + 1] * stride);
    u4* w0 = (u4*)(b + (long)(2 * p) * stride);
    u4* w1 = (u4*)(b + (long)(2 * p + 1) * stride);
    u4 v0[PER], v1[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int q = w * PER * 64 + lane + 64 * u;
        if (q < 500) { v0[u] = r0[q]; v1[u] = r1[q]; }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int q = w * PER * 64 + lane + 64 * u;
        if (q < 500) {
            u4 x = v0[u] + v1[u], y = v0[u] - v1[u];
            if (NT) { __builtin_nontemporal_store(x, w0 + q); __builtin_nontemporal_store(y, w1 + q); }
            else { w0[q] = x; w1[q] = y; }
        }
    }
}

int main() {
    const int rows = 1 << 20;
    const long stride = 8064;
    const size_t bytes = (size_t)rows * stride;
    char *a, *b;
    int *ir, *is;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&ir, rows * 4);
    hipMalloc(&is, rows * 4);
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    std::vector<int> h(rows), hs(rows);
    unsigned s = 1;
    for (int i = 0; i < rows; ++i) { s = s * 1664525u + 1013904223u; h[i] = (s >> 8) % rows; hs[i] = i; }
    hipMemcpy(ir, h.data(), rows * 4, hipMemcpyHostToDevice);
    hipMemcpy(is, hs.data(), rows * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
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
    const double copyb = 2.0 * 8000.0 * rows;
    const int np = rows / 2;
    for (int ri = 0; ri < 2; ++ri) {
        const int* id = ri ? is : ir;
        const char* tag = ri ? "seq" : "rand";
        char nm[96];
#define ONE(NT, WPP)                                                                          \
        {                                                                                     \
            const int g = (int)(((long)np * WPP * 64 + 255) / 256);                           \
            snprintf(nm, 96, "pair oneshot %s %s wpp=%d", tag, NT ? "nt" : "plain", WPP);     \
            run(nm, copyb, [&] { pair_oneshot<NT, WPP><<<g, 256>>>(a, b, id, np, stride); }); \
        }
        ONE(true, 1) ONE(false, 1) ONE(true, 2) ONE(false, 2) ONE(true, 4) ONE(true, 8)
    }
    return 0;
}
