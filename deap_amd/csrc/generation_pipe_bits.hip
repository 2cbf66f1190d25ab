// generation_pipe_bits.hip — hot path of the packed-bit eaSimple generation
// (OneMax-4096, config C2): native RNG, tournament / random selection, rows
// of at most 64 u64 words (4096 genes), one objective.
//
// Same two-launch structure as the float hot path (generation_pipe.hpp):
//  1. pair_plan_kernel (generation_pipe_f64.hip) — one thread per pair draws
//     the tournaments, the crossover flag and cxTwoPoint cuts, the mutation
//     flags (same Philox counters as gen_bits_kernel);
//     With evaluation on it also counts `nevals` (one atomic per workgroup).
//  2. gen_bits_burst_kernel — one-shot grid, each wave takes DM_BITS_PP
//     consecutive pairs: all their plans (scalar loads) and then all their
//     parent rows (lane L holds word L, one 512-B load per row) are issued
//     before the first pair is varied.  A persistent grid with a D-deep row
//     ring (r01c: 0.315 ms per C2 generation) ran at 3.5 TB/s where a
//     one-shot copy of the same rows reaches 6.0-6.6 TB/s
//     (tools_gpu/bwtest5.hip, profiles/r01f).
//
// Per pair: cxTwoPoint = masked word swap (crossover.py:37-60), mutFlipBit =
// geometric-skip flip masks (flip_mask_word, mutation.py:124-142), OneMax =
// popcount (README.md:85-86) of both children reduced in ONE wave reduction
// (two 16-bit counts packed in a 32-bit lane value; a row has <= 4096 ones).
// Children are bit-identical to gen_bits_kernel's native mode:
// tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel.
#include "generation_pipe.hpp"

namespace dm {

#ifndef DM_BITS_PP
#define DM_BITS_PP 4  // pairs per wave (tools_gpu/bwtest5.hip: 2-4 best)
#endif

template <int CX, int MUT, bool EVAL>
__global__ __launch_bounds__(256) void gen_bits_burst_kernel(GenArgs a, const PairPlan* plans) {
    constexpr int PP = DM_BITS_PP;
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t p0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * PP;
    if (p0 >= npairs) return;
    const int words = a.words64;
    const bool lw = lane < words;
    auto row = [&](int32_t s) {
        return reinterpret_cast<const uint64_t*>(a.pgenes + (int64_t)s * a.pstride);
    };
    // every plan (scalar loads) and then every parent row of the wave's PP
    // pairs are issued before the first pair is varied
    PairPlan pl[PP];
#pragma unroll
    for (int k = 0; k < PP; ++k) pl[k] = load_plan(plans, p0 + k < npairs ? p0 + k : p0);
    uint64_t y0[PP], y1[PP];
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        y0[k] = 0;
        y1[k] = 0;
        if (lw && p0 + k < npairs) {
            y0[k] = row(pl[k].s0)[lane];
            y1[k] = row(pl[k].s1)[lane];
        }
    }
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int64_t p = p0 + k;
        if (p >= npairs) break;
        const PairPlan& cur = pl[k];
        uint64_t x0 = y0[k], x1 = y1[k];
        const uint32_t fl = cur.flags;
        const bool has1 = fl & PF_HAS1, inv0 = fl & PF_INV0, inv1 = fl & PF_INV1;
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        if (lw) {
            if (CX == DM_CX_TWOPOINT && (fl & PF_CX)) {
                const int cp1 = (int)(cur.cuts & 0xFFFFu), cp2 = (int)(cur.cuts >> 16);
                const uint64_t m = range_mask(cp1 - lane * 64, cp2 - lane * 64);
                const uint64_t t = (x0 ^ x1) & m;
                x0 ^= t;
                x1 ^= t;
            }
            if (MUT == DM_MUT_FLIPBIT) {
                if (fl & PF_MUT0) x0 ^= flip_mask_word<false>(a, c0, lane);
                if (fl & PF_MUT1) x1 ^= flip_mask_word<false>(a, c1, lane);
            }
            uint64_t* w0 = reinterpret_cast<uint64_t*>(a.cgenes + c0 * a.cstride);
            uint64_t* w1 = reinterpret_cast<uint64_t*>(a.cgenes + c1 * a.cstride);
            __builtin_nontemporal_store(x0, w0 + lane);
            if (has1) __builtin_nontemporal_store(x1, w1 + lane);
        }
        if (EVAL) {
            uint32_t pc = lw ? ((uint32_t)__popcll(x0) | ((uint32_t)__popcll(x1) << 16)) : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) pc += __shfl_xor(pc, o, 64);
            if (lane == 0) {
                a.cwv[c0] = inv0 ? (double)(pc & 0xFFFFu) * a.w0 : cur.f0;
                if (has1) a.cwv[c1] = inv1 ? (double)(pc >> 16) * a.w0 : cur.f1;
                a.cvalid[c0] = 1;
                if (has1) a.cvalid[c1] = 1;
            }
        } else if (lane == 0) {  // no evaluation requested: clones keep their fitness
            a.cwv[c0] = cur.f0;
            if (has1) a.cwv[c1] = cur.f1;
            a.cvalid[c0] = inv0 ? 0 : 1;
            if (has1) a.cvalid[c1] = inv1 ? 0 : 1;
        }
    }
}

template <int CX, int MUT, bool EVAL>
static void launch_bp(const GenArgs& a, const PairPlan* plans, int num_cus, hipStream_t s) {
    // one-shot grid: every wave takes DM_BITS_PP consecutive pairs once
    const int64_t waves = ((a.nc + 1) / 2 + DM_BITS_PP - 1) / DM_BITS_PP;
    gen_bits_burst_kernel<CX, MUT, EVAL><<<dim3((unsigned)((waves + 3) / 4)), 256, 0, s>>>(a, plans);
}
template <int CX, int MUT>
static void launch_bp_e(const GenArgs& a, const PairPlan* plans, bool eval, int num_cus,
                        hipStream_t s) {
    eval ? launch_bp<CX, MUT, true>(a, plans, num_cus, s)
         : launch_bp<CX, MUT, false>(a, plans, num_cus, s);
}

void launch_gen_bits_pipe(const GenArgs& a, const PairPlan* plans, bool eval, int num_cus,
                          hipStream_t s) {
    const bool mf = a.mut == DM_MUT_FLIPBIT;
    if (a.cx == DM_CX_TWOPOINT)
        mf ? launch_bp_e<DM_CX_TWOPOINT, DM_MUT_FLIPBIT>(a, plans, eval, num_cus, s)
           : launch_bp_e<DM_CX_TWOPOINT, DM_MUT_NONE>(a, plans, eval, num_cus, s);
    else
        mf ? launch_bp_e<DM_CX_NONE, DM_MUT_FLIPBIT>(a, plans, eval, num_cus, s)
           : launch_bp_e<DM_CX_NONE, DM_MUT_NONE>(a, plans, eval, num_cus, s);
}

}  // namespace dm
