// lds_probe.hip — does a workgroup with a large static LDS allocation run
// correctly on this box?  Each block fills its LDS with a block-specific
// pattern (16-B stores), waits at a barrier, reads it back in a rotated order
// and counts mismatches.  Sizes: 69,760 B (the m = 3 bitset kernels),
// 104,640 B (m = 4), 139,520 B (two chunks of m = 3 tables).
// Build: hipcc --offload-arch=gfx950 -O3 lds_probe.hip -o lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N16>
__global__ __launch_bounds__(512) void lds_fill_check(unsigned* errors, int rounds) {
    __shared__ uint4 buf[N16];
    unsigned bad = 0;
    for (int r = 0; r < rounds; ++r) {
        const unsigned key = blockIdx.x * 2654435761u + r * 40503u;
        for (int i = threadIdx.x; i < N16; i += blockDim.x)
            buf[i] = make_uint4(key ^ i, key + i, i, ~key);
        __syncthreads();
        for (int i = (threadIdx.x * 7) % N16, n = 0; n < (N16 + 511) / 512; ++n, i = (i + 512) % N16) {
            const uint4 v = buf[i];
            bad += (v.x != (key ^ i)) + (v.y != key + i) + (v.z != (unsigned)i) + (v.w != ~key);
        }
        __syncthreads();
    }
    if (bad) atomicAdd(errors, bad);
}

template <int N16>
static int run(const char* name, unsigned* d_err) {
    hipMemset(d_err, 0, 4);
    lds_fill_check<N16><<<4096, 512>>>(d_err, 8);
    hipError_t e = hipDeviceSynchronize();
    unsigned h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d_err, 4, hipMemcpyDeviceToHost);
    printf("%-10s %7d B LDS: %s, mismatches %u\n", name, N16 * 16, hipGetErrorString(e), h);
    return e != hipSuccess || h != 0;
}

int main(int argc, char** argv) {
    unsigned* d_err = nullptr;
    if (hipMalloc(&d_err, 4) != hipSuccess) return 2;
    int which = argc > 1 ? atoi(argv[1]) : 0;
    int rc = 0;
    if (which == 0 || which == 1) rc |= run<4360>("m3", d_err);
    if (rc) return rc;
    if (which == 0 || which == 2) rc |= run<6540>("m4", d_err);
    if (rc) return rc;
    if (which == 0 || which == 3) rc |= run<8720>("m3x2", d_err);
    return rc;
}
