// generation_pipe_bits.hip — hot path of the packed-bit eaSimple generation
// (OneMax-4096, config C2): native RNG, tournament / random selection, rows
// of at most 64 u64 words (4096 genes), one objective.
//
// Same two-launch structure as the float hot path (generation_pipe.hpp):
//  1. pair_plan_kernel (generation_pipe_f64.hip) — one thread per pair draws
//     the tournaments, the crossover flag and cxTwoPoint cuts, the mutation
//     flags (same Philox counters as gen_bits_kernel);
//  2. gen_bits_pipe_kernel — one wave per pair on a persistent grid; lane L
//     holds word L of both parent rows (one 512-B load instruction per row).
//     The rows of the next D pairs of the wave are in flight while a pair is
//     varied, so the per-pair latency chain (plan -> rows -> store) that
//     bounds gen_bits_kernel (tournament loads, then row loads, per pair, in
//     every wave) is paid once per wave instead of once per pair.
//
// Per pair: cxTwoPoint = masked word swap (crossover.py:37-60), mutFlipBit =
// geometric-skip flip masks (flip_mask_word, mutation.py:124-142), OneMax =
// popcount (README.md:85-86) of both children reduced in ONE wave reduction
// (two 16-bit counts packed in a 32-bit lane value; a row has <= 4096 ones).
// Children are bit-identical to gen_bits_kernel's native mode:
// tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel.
#include "generation_pipe.hpp"

namespace dm {

#ifndef DM_BITS_PIPE_DEPTH
#define DM_BITS_PIPE_DEPTH 4
#endif

template <int CX, int MUT, bool EVAL>
__global__ __launch_bounds__(256) void gen_bits_pipe_kernel(GenArgs a, const PairPlan* plans) {
    constexpr int D = DM_BITS_PIPE_DEPTH;
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (p >= npairs) return;
    const int words = a.words64;
    const bool lw = lane < words;
    auto clampq = [&](int64_t q) { return q < npairs ? q : p; };
    auto row = [&](int32_t s) {
        return reinterpret_cast<const uint64_t*>(a.pgenes + (int64_t)s * a.pstride);
    };

    // ring: plans of pairs p + d*nw (d = 0..D), rows of pairs p + d*nw (d < D)
    PairPlan pl[D + 1];
    uint64_t y0[D], y1[D];
#pragma unroll
    for (int d = 0; d <= D; ++d) pl[d] = load_plan(plans, clampq(p + d * nw));
#pragma unroll
    for (int d = 0; d < D; ++d) {
        y0[d] = 0;
        y1[d] = 0;
        if (lw && p + d * nw < npairs) {
            y0[d] = row(pl[d].s0)[lane];
            y1[d] = row(pl[d].s1)[lane];
        }
    }
    int64_t evals = 0;
    for (; p < npairs; p += nw) {
        const PairPlan cur = pl[0];
        // issue the rows of pair p + D*nw before touching this pair's rows
        const int64_t pf = p + D * nw;
        uint64_t n0 = 0, n1 = 0;
        if (lw && pf < npairs) {
            n0 = row(pl[D].s0)[lane];
            n1 = row(pl[D].s1)[lane];
        }
        uint64_t x0 = y0[0], x1 = y1[0];
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            y0[d] = y0[d + 1];
            y1[d] = y1[d + 1];
        }
        y0[D - 1] = n0;
        y1[D - 1] = n1;
#pragma unroll
        for (int d = 0; d < D; ++d) pl[d] = pl[d + 1];
        pl[D] = load_plan(plans, clampq(p + (D + 1) * nw));

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
                evals += (int64_t)inv0 + (int64_t)inv1;
            }
        } else if (lane == 0) {  // no evaluation requested: clones keep their fitness
            a.cwv[c0] = cur.f0;
            if (has1) a.cwv[c1] = cur.f1;
            a.cvalid[c0] = inv0 ? 0 : 1;
            if (has1) a.cvalid[c1] = inv1 ? 0 : 1;
        }
    }
    if (a.nevals && EVAL && lane == 0 && evals)
        atomicAdd((unsigned long long*)a.nevals, (unsigned long long)evals);
}

template <int CX, int MUT, bool EVAL>
static void launch_bp(const GenArgs& a, const PairPlan* plans, int num_cus, hipStream_t s) {
    auto kern = gen_bits_pipe_kernel<CX, MUT, EVAL>;
    kern<<<pipe_grid(kern, num_cus, (a.nc + 1) / 2), 256, 0, s>>>(a, plans);
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
