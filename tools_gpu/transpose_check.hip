// Checks the two wave transposes of deap_amd/csrc/transpose.hpp against a
// host transpose on random words (build: hipcc --offload-arch=gfx950 -O3).
#include "../deap_amd/csrc/transpose.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>

template <class T>
__global__ void k(const uint64_t* in, uint64_t* out) {
    const int lane = threadIdx.x;
    const T tr(lane);
    uint32_t lo[8], hi[8];
    for (int w = 0; w < 8; ++w) {
        lo[w] = (uint32_t)in[w * 64 + lane];
        hi[w] = (uint32_t)(in[w * 64 + lane] >> 32);
    }
    tr.template run<8>(lo, hi);
    for (int w = 0; w < 8; ++w) out[w * 64 + lane] = ((uint64_t)hi[w] << 32) | lo[w];
}

int main() {
    std::vector<uint64_t> h(512), r(512), ref(512);
    srand(7);
    for (auto& x : h) x = ((uint64_t)rand() << 42) ^ ((uint64_t)rand() << 21) ^ (uint64_t)rand();
    for (int w = 0; w < 8; ++w)
        for (int i = 0; i < 64; ++i) {
            uint64_t o = 0;
            for (int j = 0; j < 64; ++j) o |= ((h[w * 64 + j] >> i) & 1ull) << j;
            ref[w * 64 + i] = o;
        }
    uint64_t *din, *dout;
    if (hipMalloc(&din, 4096) || hipMalloc(&dout, 4096)) return 2;
    hipMemcpy(din, h.data(), 4096, hipMemcpyHostToDevice);
    int bad = 0;
    for (int v = 0; v < 2; ++v) {
        if (v == 0) k<dm::Transposer><<<1, 64>>>(din, dout);
        else k<dm::TransposerX><<<1, 64>>>(din, dout);
        hipMemcpy(r.data(), dout, 4096, hipMemcpyDeviceToHost);
        int mism = 0;
        for (int i = 0; i < 512; ++i) mism += r[i] != ref[i];
        printf("%s: %d of 512 words differ\n", v ? "TransposerX (dpp/permlane)" : "Transposer (bpermute)", mism);
        bad |= mism != 0;
    }
    return bad;
}
