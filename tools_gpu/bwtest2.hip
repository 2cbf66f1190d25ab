// Row-gather ceilings for the generation's access pattern (not part of the
// product): 2^20 child rows of 8000 B, each copied from a (random or
// identity) parent row, one wave per row pair, persistent grid.
//   MODE 0: each load/store instruction covers 1 KB contiguous (16 B / lane)
//   MODE 1: each lane owns 32 contiguous bytes (two dwordx4 at stride 32 B),
//           the layout of the hot kernel's 4-genes-per-lane chunks
//   NT    : non-temporal child stores
//   D     : chunks of 1 KB (MODE 0) / 2 KB (MODE 1) per row in flight
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int MODE, bool NT>
__device__ __forceinline__ void st(u4* p, u4 v) {
    if (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void gather2(const char* __restrict__ a, char* __restrict__ b,
                                               const int* __restrict__ idx, int npairs, long stride) {
    const int lane = threadIdx.x & 63;
    const int nw = (gridDim.x * 256) >> 6;
    for (int p = (blockIdx.x * 256 + threadIdx.x) >> 6; p < npairs; p += nw) {
        const int s0 = idx[2 * p], s1 = idx[2 * p + 1];
        const u4* r0 = (const u4*)(a + (long)s0 * stride);
        const u4* r1 = (const u4*)(a + (long)s1 * stride);
        u4* w0 = (u4*)(b + (long)(2 * p) * stride);
        u4* w1 = (u4*)(b + (long)(2 * p + 1) * stride);
        u4 v0[8], v1[8];
        if (MODE == 0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = lane + 64 * u;
                if (q < 500) { v0[u] = r0[q]; v1[u] = r1[q]; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = lane + 64 * u;
                if (q < 500) { st<MODE, NT>(w0 + q, v0[u]); st<MODE, NT>(w1 + q, v1[u]); }
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = 2 * (lane + 64 * u);
                if (q < 500) { v0[2*u] = r0[q]; v0[2*u+1] = r0[q+1]; v1[2*u] = r1[q]; v1[2*u+1] = r1[q+1]; }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = 2 * (lane + 64 * u);
                if (q < 500) {
                    st<MODE, NT>(w0 + q, v0[2*u]); st<MODE, NT>(w0 + q + 1, v0[2*u+1]);
                    st<MODE, NT>(w1 + q, v1[2*u]); st<MODE, NT>(w1 + q + 1, v1[2*u+1]);
                }
            }
        }
    }
}

int main() {
    const int rows = 1 << 20;
    const long maxstride = 8320;
    char *a, *b;
    int *ir, *ii;
    hipMalloc(&a, (size_t)rows * maxstride);
    hipMalloc(&b, (size_t)rows * maxstride);
    hipMalloc(&ir, rows * 4);
    hipMalloc(&ii, rows * 4);
    hipMemset(a, 1, (size_t)rows * maxstride);
    std::vector<int> h(rows), id(rows);
    unsigned s = 1;
    for (int i = 0; i < rows; ++i) { s = s * 1664525u + 1013904223u; h[i] = (s >> 8) % rows; id[i] = i; }
    hipMemcpy(ir, h.data(), rows * 4, hipMemcpyHostToDevice);
    hipMemcpy(ii, id.data(), rows * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev; hipGetDevice(&dev); hipDeviceProp_t pr; hipGetDeviceProperties(&pr, dev);
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("%-48s %8.3f ms  %7.1f GB/s (2 x 8000 B / row)\n", name, ms, 2.0 * 8000.0 * rows / ms / 1e6);
        fflush(stdout);
    };
    const int np = rows / 2;
    for (long stride : {8000L, 8064L, 8192L, 8320L}) {
        for (int bpc : {2, 4, 8, 64}) {
            const int g = cus * bpc > np / 4 ? np / 4 : cus * bpc;
            char nm[96];
            for (int rnd = 0; rnd < 2; ++rnd) {
                const int* ix = rnd ? ir : ii;
                const char* rn = rnd ? "rand" : "ident";
                snprintf(nm, 96, "m0 nt stride=%ld bpc=%d %s", stride, bpc, rn);
                run(nm, [&] { gather2<0, true><<<g, 256>>>(a, b, ix, np, stride); });
                snprintf(nm, 96, "m1 nt stride=%ld bpc=%d %s", stride, bpc, rn);
                run(nm, [&] { gather2<1, true><<<g, 256>>>(a, b, ix, np, stride); });
                if (bpc == 8) {
                    snprintf(nm, 96, "m0 plain stride=%ld bpc=%d %s", stride, bpc, rn);
                    run(nm, [&] { gather2<0, false><<<g, 256>>>(a, b, ix, np, stride); });
                    snprintf(nm, 96, "m1 plain stride=%ld bpc=%d %s", stride, bpc, rn);
                    run(nm, [&] { gather2<1, false><<<g, 256>>>(a, b, ix, np, stride); });
                }
            }
        }
    }
    return 0;
}
