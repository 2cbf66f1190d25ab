// transpose.hpp — 64 x 64-bit transposes across a wave (the peel of
// dominance.hip): the LDS-shuffle form and the DPP / permlane form.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace dm {

// 64x64 bit transposes across the wave (in lane i bit j = A[i][j]; out lane j
// bit i = A[i][j]) of N words at once, stage by stage so that the lane
// exchanges of all N words are in flight together, without branches: the
// stage of distance s swaps 2s-bit blocks between lanes i and i^s.  s = 32
// moves whole 32-bit halves; s = 16 and 8 recombine bytes with one v_perm;
// s = 4, 2, 1 rotate the partner's half and merge with one bit-field insert,
// the per-lane selectors and masks computed once.
struct Transposer {
    uint32_t sel16, sel8, m4, m2, m1, r4, r2, r1;
    bool low32;
    __device__ explicit Transposer(int lane) {
        sel16 = (lane & 16) ? 0x03020706u : 0x05040100u;
        sel8 = (lane & 8) ? 0x03070105u : 0x06020400u;
        m4 = (lane & 4) ? ~0x0F0F0F0Fu : 0x0F0F0F0Fu;
        m2 = (lane & 2) ? ~0x33333333u : 0x33333333u;
        m1 = (lane & 1) ? ~0x55555555u : 0x55555555u;
        r4 = (lane & 4) ? 4u : 28u;
        r2 = (lane & 2) ? 2u : 30u;
        r1 = (lane & 1) ? 1u : 31u;
        low32 = (lane & 32) == 0;
    }
    template <int N>
    __device__ __forceinline__ void run(uint32_t (&lo)[N], uint32_t (&hi)[N]) const {
        {  // s = 32: lanes < 32 take the partner's low half as their high half
            uint32_t r[N];
#pragma unroll
            for (int w = 0; w < N; ++w) r[w] = __shfl_xor(low32 ? hi[w] : lo[w], 32, 64);
#pragma unroll
            for (int w = 0; w < N; ++w) {
                hi[w] = low32 ? r[w] : hi[w];
                lo[w] = low32 ? lo[w] : r[w];
            }
        }
        bytes<N>(lo, hi, 16, sel16);
        bytes<N>(lo, hi, 8, sel8);
        bits<N>(lo, hi, 4, m4, r4);
        bits<N>(lo, hi, 2, m2, r2);
        bits<N>(lo, hi, 1, m1, r1);
    }
    template <int N>
    __device__ __forceinline__ static void bytes(uint32_t (&lo)[N], uint32_t (&hi)[N], int s,
                                                 uint32_t sel) {
        uint32_t rl[N], rh[N];
#pragma unroll
        for (int w = 0; w < N; ++w) {
            rl[w] = __shfl_xor(lo[w], s, 64);
            rh[w] = __shfl_xor(hi[w], s, 64);
        }
#pragma unroll
        for (int w = 0; w < N; ++w) {
            lo[w] = __builtin_amdgcn_perm(rl[w], lo[w], sel);
            hi[w] = __builtin_amdgcn_perm(rh[w], hi[w], sel);
        }
    }
    template <int N>
    __device__ __forceinline__ static void bits(uint32_t (&lo)[N], uint32_t (&hi)[N], int s,
                                                uint32_t m, uint32_t rot) {
        uint32_t rl[N], rh[N];
#pragma unroll
        for (int w = 0; w < N; ++w) {
            rl[w] = __shfl_xor(lo[w], s, 64);
            rh[w] = __shfl_xor(hi[w], s, 64);
        }
#pragma unroll
        for (int w = 0; w < N; ++w) {
            const uint32_t tl = __builtin_amdgcn_alignbit(rl[w], rl[w], rot);
            const uint32_t th = __builtin_amdgcn_alignbit(rh[w], rh[w], rot);
            lo[w] = (m & lo[w]) | (~m & tl);
            hi[w] = (m & hi[w]) | (~m & th);
        }
    }
};

// The same transposes with no LDS traffic: the distance-32 and -16 exchanges
// by v_permlane32_swap / v_permlane16_swap, the distance-8/4/2/1 partners by
// DPP row and quad permutations (l^8 = half_mirror(mirror), l^4 =
// quad_perm[3,2,1,0](half_mirror), l^2 / l^1 = quad_perm).  The peel issued
// 11 ds_bpermute per word with the LDS pipe busy ~8 cycles each, which bound
// it; these run on the VALU.
struct TransposerX {
    uint32_t sel16, sel8, m4, m2, m1, r4, r2, r1;
    bool odd16;
    __device__ explicit TransposerX(int lane) {
        sel16 = (lane & 16) ? 0x03020706u : 0x05040100u;
        sel8 = (lane & 8) ? 0x03070105u : 0x06020400u;
        m4 = (lane & 4) ? ~0x0F0F0F0Fu : 0x0F0F0F0Fu;
        m2 = (lane & 2) ? ~0x33333333u : 0x33333333u;
        m1 = (lane & 1) ? ~0x55555555u : 0x55555555u;
        r4 = (lane & 4) ? 4u : 28u;
        r2 = (lane & 2) ? 2u : 30u;
        r1 = (lane & 1) ? 1u : 31u;
        odd16 = (lane & 16) != 0;
    }
    template <int CTRL>
    __device__ __forceinline__ static uint32_t dpp(uint32_t x) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
    }
    __device__ __forceinline__ uint32_t x16(uint32_t x) const {
        const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return odd16 ? p[0] : p[1];
    }
    template <int N>
    __device__ __forceinline__ void run(uint32_t (&lo)[N], uint32_t (&hi)[N]) const {
#pragma unroll
        for (int w = 0; w < N; ++w) {  // s = 32: lanes >= 32 take the partner's high half as low
            const auto p = __builtin_amdgcn_permlane32_swap(lo[w], hi[w], false, false);
            lo[w] = p[0];
            hi[w] = p[1];
        }
#pragma unroll
        for (int w = 0; w < N; ++w) {
            const uint32_t rl = x16(lo[w]), rh = x16(hi[w]);
            lo[w] = __builtin_amdgcn_perm(rl, lo[w], sel16);
            hi[w] = __builtin_amdgcn_perm(rh, hi[w], sel16);
        }
        {
            // the two-step DPP partners: every word's first step before any
            // second step (a DPP reading the VGPR the previous VALU wrote needs
            // wait states, s_nop when nothing else can fill them)
            uint32_t tl[N], th[N];
#pragma unroll
            for (int w = 0; w < N; ++w) {
                tl[w] = dpp<0x140>(lo[w]);
                th[w] = dpp<0x140>(hi[w]);
            }
#pragma unroll
            for (int w = 0; w < N; ++w) {
                const uint32_t rl = dpp<0x141>(tl[w]), rh = dpp<0x141>(th[w]);
                lo[w] = __builtin_amdgcn_perm(rl, lo[w], sel8);
                hi[w] = __builtin_amdgcn_perm(rh, hi[w], sel8);
            }
        }
        bits<N, 0x1B, true>(lo, hi, m4, r4);
        bits<N, 0x4E, false>(lo, hi, m2, r2);
        bits<N, 0xB1, false>(lo, hi, m1, r1);
    }
    template <int N, int QP, bool HM>
    __device__ __forceinline__ static void bits(uint32_t (&lo)[N], uint32_t (&hi)[N], uint32_t m,
                                                uint32_t rot) {
        uint32_t rl[N], rh[N];
#pragma unroll
        for (int w = 0; w < N; ++w) {
            rl[w] = HM ? dpp<0x141>(lo[w]) : lo[w];
            rh[w] = HM ? dpp<0x141>(hi[w]) : hi[w];
        }
#pragma unroll
        for (int w = 0; w < N; ++w) {
            rl[w] = dpp<QP>(rl[w]);
            rh[w] = dpp<QP>(rh[w]);
        }
#pragma unroll
        for (int w = 0; w < N; ++w) {
            const uint32_t tl = __builtin_amdgcn_alignbit(rl[w], rl[w], rot);
            const uint32_t th = __builtin_amdgcn_alignbit(rh[w], rh[w], rot);
            lo[w] = (m & lo[w]) | (~m & tl);
            hi[w] = (m & hi[w]) | (~m & th);
        }
    }
};

}  // namespace dm
