// generation_pipe_bits.hip — hot path of the packed-bit eaSimple generation
// (OneMax-4096, config C2): native RNG, tournament / random selection, rows
// of at most 64 u64 words (4096 genes) -- the fused kernel up to 256 words
// (16,384 genes, round 6) --, one objective.
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
// row-level geometric-skip flip masks (flip_mask_row, mutation.py:124-142), OneMax =
// popcount (README.md:85-86) of both children reduced in ONE wave reduction
// (two 16-bit counts packed in a 32-bit lane value; a row has <= 4096 ones).
// Children are bit-identical to gen_bits_kernel's native mode:
// tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel.
#include "generation_pipe.hpp"

namespace dm {

// Flip mask of word `lane` of child c's row (<= 64 words): the row-level
// geometric stream of flip_mask_chunk drawn by the whole wave.
__device__ __forceinline__ uint64_t flip_mask_row(const GenArgs& a, int64_t c, int lane,
                                                  uint64_t* lds) {
    FlipRow<64> st;
    flip_begin<64>(a, c, lane, st);
    return flip_mask_chunk<64, false>(a, c, 0, lane, st, lds);
}

// flip_mask_row for rows of WPL x 64 words (lane L: words L + 64 k)
template <int WPL>
__device__ __forceinline__ void flip_mask_row_w(const GenArgs& a, int64_t c, int lane,
                                                uint64_t* lds, uint64_t (&f)[WPL]) {
    FlipRow<64> st;
    flip_begin<64>(a, c, lane, st);
#pragma unroll
    for (int k = 0; k < WPL; ++k) f[k] = flip_mask_chunk<64, false>(a, c, 64 * k, lane, st, lds);
}

// The flip masks of every mutated child of a group (bit c of `mut_bits` =
// child 2 p0 + c) into that child's 64 LDS words: issued right after the
// group's row loads, so this VALU / LDS work overlaps their latency.
// Slots of 64 LDS words per wave for precomputed flip masks (children ranked
// by index among the group's mutated ones; P(more than 6 of 16) = 2.7 % at
// mutpb 0.2) plus one scratch slot for the rest, computed in bits_finish.
constexpr int FLIP_SLOTS = 6;

// Rows of WPL x 64 words: lane L holds words L + 64 k (k < WPL), a slot is
// 64 WPL words, the row's chunks of 64 words drawn in order from one
// geometric stream (the same positions as flip_mask_chunk's).
template <int NCH, int WPL>
__device__ __forceinline__ void flip_rows_to_lds(const GenArgs& a, int64_t cbase, uint64_t mut_bits,
                                                 int lane, uint64_t* lds) {
    if (a.thr_ind == 0) return;
    int slot = 0;
    for (uint64_t mb = mut_bits; mb && slot < FLIP_SLOTS; mb &= mb - 1, ++slot) {  // wave-uniform
        const int ch = __ffsll((long long)mb) - 1;
        uint64_t* w = lds + slot * 64 * WPL;
        if (a.thr_ind >= (1ull << 32)) {
#pragma unroll
            for (int k = 0; k < WPL; ++k) {
                const int wi = lane + 64 * k;
                const int nbits = min(64, a.dim - wi * 64);
                w[64 * k + lane] = wi >= a.words64 ? 0ull : nbits >= 64 ? ~0ull : ((1ull << nbits) - 1);
            }
            continue;
        }
        FlipRow<64> st;
        flip_begin<64>(a, cbase + ch, lane, st);
#pragma unroll
        for (int k = 0; k < WPL; ++k) flip_chunk_lds<64>(a, cbase + ch, 64 * k, lane, st, w + 64 * k);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Sum of a u32 over the wave, wave-uniform result: DPP adds within each row
// of 16 lanes (quad xor 1, quad xor 2, half-row mirror, row mirror), then
// the four row sums by readlane — no LDS round trips (a __shfl_xor butterfly
// is six ds_bpermute).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm(1,0,3,2)
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm(2,3,0,1)
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Profiling-only ablations of the fused kernel (product build: 0): bit 0
// skips the mutFlipBit masks, bit 1 the aspirants' fitness loads, bit 2 the
// Philox evaluation of the decisions.
#ifndef DM_BITS_ABLATE
#define DM_BITS_ABLATE 0
#endif

// Non-temporal parent-row loads (0 disables): the streamed rows no longer
// evict the aspirants' 2 MiB key array from the L2 (A/B r04 c2ntl: kernel
// 0.2255 -> 0.2227 ms, HBM bytes per launch 1.242e9 -> 1.101e9 = 0.99 x the
// algorithmic 1.107e9).
#ifndef DM_BITS_NTLOAD
#define DM_BITS_NTLOAD 1
#endif

// Wave priority over the decision chain (0 disables; A/B r04 c2prio: 1 and
// 3 both -1.3 to -2 % kernel time; keeping it through the flip masks: no gain)
#ifndef DM_BITS_PRIO
#define DM_BITS_PRIO 1
#endif

#ifndef DM_BITS_PP
#define DM_BITS_PP 4  // pairs per wave (tools_gpu/bwtest5.hip: 2-4 best)
#endif

template <int CX, int MUT, bool EVAL>
__global__ __launch_bounds__(256) void gen_bits_burst_kernel(GenArgs a, const PairPlan* plans) {
    constexpr int PP = DM_BITS_PP;
    __shared__ uint64_t flip_lds_all[256];
    uint64_t* flip_lds = flip_lds_all + (threadIdx.x & ~63);
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
        uint64_t f0 = 0, f1 = 0;  // flip masks, drawn by the whole wave per row
        if (MUT == DM_MUT_FLIPBIT) {
            if (fl & PF_MUT0) f0 = flip_mask_row(a, c0, lane, flip_lds);
            if (fl & PF_MUT1) f1 = flip_mask_row(a, c1, lane, flip_lds);
        }
        if (lw) {
            if (CX == DM_CX_TWOPOINT && (fl & PF_CX)) {
                const int cp1 = (int)(cur.cuts & 0xFFFFu), cp2 = (int)(cur.cuts >> 16);
                const uint64_t m = range_mask(cp1 - lane * 64, cp2 - lane * 64);
                const uint64_t t = (x0 ^ x1) & m;
                x0 ^= t;
                x1 ^= t;
            }
            x0 ^= f0;  // mutation after the crossover (algorithms.py:72-81)
            x1 ^= f1;
            uint64_t* w0 = reinterpret_cast<uint64_t*>(a.cgenes + c0 * a.cstride);
            uint64_t* w1 = reinterpret_cast<uint64_t*>(a.cgenes + c1 * a.cstride);
            __builtin_nontemporal_store(x0, w0 + lane);
            if (has1) __builtin_nontemporal_store(x1, w1 + lane);
        }
        if (EVAL) {
            const uint32_t pc =
                wave_sum_u32(lw ? ((uint32_t)__popcll(x0) | ((uint32_t)__popcll(x1) << 16)) : 0u);
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

// ---------------------------------------------------------------------------
// Single-launch form (the C2 hot path): the per-pair decisions are drawn
// inside the burst kernel, so the plan kernel, its 32-B plans and its
// separate pass over the parents' fitness disappear.  A wave owns DM_BITS_PP
// = 4 pairs = 8 children; for the selection phase lane L takes child L & 7
// and Philox call L >> 3 (its two aspirants), lanes 32-39 the crossover
// calls of the 4 pairs and lanes 40-47 the mutation flags of the 8 children,
// so ONE Philox evaluation per lane draws every decision of the wave (t <=
// 8); each aspirant's fitness and validity come from one vector load, the
// tournament (first-drawn wins, a later aspirant replaces only on
// Fitness.__gt__ = not(a <= b), selection.py:68) runs over lane shuffles.  The
// winners reach the row loads through readlane (scalar row addresses), the
// clone's inherited fitness stays in the child's lane, and each wave stores
// its 8 fitness values and 8 validity bytes as one contiguous store each.
// `nevals`: per-workgroup partials (ballot + LDS), summed by a second launch.
// Same Philox counters as pair_plan_kernel / gen_bits_kernel: bit-identical
// children (tests/test_gpu_parity.py::test_native_hot_kernel_equals_replay_kernel).
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Parent fitness keys.  The tournaments read t random parent fitnesses per
// child; as 8-B loads from the 8 MiB wvalues array (2^20 rows) each pulls a
// whole line past the 4 MiB L2 of its XCD (PMC: 1.31x the algorithmic bytes,
// profiles/r02x).  OneMax fitnesses are small integers times the weight, so
// one coalesced pass writes every parent's wvalue as an int16 q with
// wv == q * |w0| EXACTLY (2 MiB, L2-resident), or FIT_KEY_NONE when the row
// is invalid or its value is not such a multiple.  The tournament rebuilds
// the exact fp64 wvalue from the key (falls back to wvalues / valid for
// FIT_KEY_NONE), so the comparisons are the reference's own
// (Fitness.__gt__ on wvalues, selection.py:68), not an approximation.
// ---------------------------------------------------------------------------
constexpr int16_t FIT_KEY_NONE = -32768;

__global__ __launch_bounds__(256) void fit_key_kernel(const double* __restrict__ wv,
                                                      const uint8_t* __restrict__ valid, int64_t n,
                                                      double scale, int16_t* __restrict__ keys) {
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i0 >= n) return;
    int16_t k[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        k[j] = FIT_KEY_NONE;
        const int64_t i = i0 + j;
        if (i < n && valid[i]) {
            const double v = wv[i];
            const double q = rint(v / scale);
            // -0.0 (a zero count under a negative weight) has no key: the
            // rebuild q * |w0| would give +0.0, and clones keep -0.0
            if (fabs(q) <= 32767.0 && q * scale == v && !(v == 0.0 && signbit(v)))
                k[j] = (int16_t)q;
        }
    }
    if (i0 + 3 < n) {
        *reinterpret_cast<uint64_t*>(keys + i0) =
            (uint64_t)(uint16_t)k[0] | ((uint64_t)(uint16_t)k[1] << 16) |
            ((uint64_t)(uint16_t)k[2] << 32) | ((uint64_t)(uint16_t)k[3] << 48);
    } else {
        for (int j = 0; j < 4 && i0 + j < n; ++j) keys[i0 + j] = k[j];
    }
}

void launch_fit_keys(const GenArgs& a, int16_t* keys, hipStream_t s) {
    const int64_t threads = (a.np + 3) / 4;
    fit_key_kernel<<<dim3((unsigned)((threads + 255) / 256)), 256, 0, s>>>(
        a.pwv, a.pvalid, a.np, fabs(a.w0), keys);
}

// wvalue of parent k: from its key when it has one (exact), else wvalues
__device__ __forceinline__ double parent_fit(const GenArgs& a, int32_t k) {
    if (a.pkeys) {
        const int16_t q = a.pkeys[k];
        if (q != FIT_KEY_NONE) return (double)q * fabs(a.w0);
    }
    return a.pwv[k];
}

// Decision draws of one group (PP pairs) of a wave, before the tournament:
// the Philox words of every lane and the aspirants' fitness loads in flight.
struct BitsDraw {
    int32_t k0, k1;
    double f0, f1;
    uint32_t cxf_l, cuts;
    bool mut_l;
};
// A group after its tournament: winners, flags and parent rows in flight.
template <int PP, int WPL>
struct BitsGroup {
    int64_t p0;
    int32_t s0[PP], s1[PP];
    uint32_t cut[PP], cxf[PP];
    uint64_t y0[PP][WPL], y1[PP][WPL];  // lane L: words L + 64 k
    uint64_t mut_bits;
    double f;      // lane L < 2PP: child L's winner fitness (the clone's)
    uint32_t v;    // ... its validity
    bool cx_c, mut;
};

template <int PP, int CX, int MUT, bool TOURN>
__device__ __forceinline__ BitsDraw bits_draw(const GenArgs& a, int64_t p0, int lane) {
    constexpr int NCH = 2 * PP;
    constexpr int CXL = 32, MUTL = 32 + 2 * PP;  // first crossover / mutation lane
    const int64_t cbase = 2 * p0;
    const uint32_t np = (uint32_t)a.np;
    //   lanes 0-31: selection, child L % NCH, call L / NCH (aspirants 2call, 2call+1)
    //   lanes CXL..CXL+2PP-1: crossover of pair (L - CXL) % PP, call (L - CXL) / PP
    //   lanes MUTL..MUTL+NCH-1: mutation flag of child L - MUTL
    const int t = TOURN ? a.tournsize : 1;
    const int S = (t + 1) >> 1;  // selection calls per child (t <= 64 / NCH)
    uint32_t stage = ST_SEL, item = 0, sub = 0;
    bool draw = false;
    if (lane < CXL) {
        item = (uint32_t)(cbase + (lane % NCH));
        sub = (uint32_t)(lane / NCH);
        draw = (int)sub < S && cbase + (lane % NCH) < a.nc;
    } else if (lane < MUTL) {
        const int64_t pp = p0 + ((lane - CXL) % PP);
        stage = ST_CX;
        item = (uint32_t)pp;
        sub = (uint32_t)((lane - CXL) / PP);
        draw = CX != DM_CX_NONE && 2 * pp + 1 < a.nc;
    } else if (lane < MUTL + NCH) {
        stage = ST_MUT;
        item = (uint32_t)(cbase + lane - MUTL);
        draw = MUT != DM_MUT_NONE && cbase + lane - MUTL < a.nc;
    }
    u32x4 w{};
    if (draw) {
        if (DM_BITS_ABLATE & 4)
            w = u32x4{item * 2654435761u ^ sub, item * 40503u + stage, item ^ 0x9E3779B9u, sub + item};
        else
            w = a.rng(stage, item, sub);
    }
    BitsDraw d{};
    // selection lanes: both aspirants of the call and their fitness
    if (draw && lane < CXL) {
        d.k0 = (int32_t)bounded64(w.x, w.y, np);
        d.f0 = (DM_BITS_ABLATE & 2) ? (double)(d.k0 & 255) : parent_fit(a, d.k0);
        if (2 * (int)sub + 1 < t) {
            d.k1 = (int32_t)bounded64(w.z, w.w, np);
            d.f1 = (DM_BITS_ABLATE & 2) ? (double)(d.k1 & 255) : parent_fit(a, d.k1);
        }
    }
    // crossover lanes CXL..CXL+PP-1: flag and cxTwoPoint cuts of pair L - CXL
    // (call 1's words come from lane L + PP)
    const uint32_t w2x = (uint32_t)__shfl((int)w.x, (lane + PP) & 63, 64);
    const uint32_t w2y = (uint32_t)__shfl((int)w.y, (lane + PP) & 63, 64);
    if (draw && lane >= CXL && lane < CXL + PP && (uint64_t)w.x < a.thr_cx) {
        d.cxf_l = 1;
        if (CX == DM_CX_TWOPOINT) {
            int32_t r1 = 1 + (int32_t)bounded64(w.z, w.w, (uint32_t)a.dim);
            int32_t r2 = 1 + (int32_t)bounded64(w2x, w2y, (uint32_t)(a.dim - 1));
            if (r2 >= r1) {
                r2 += 1;
            } else {
                const int32_t tt = r1;
                r1 = r2;
                r2 = tt;
            }
            d.cuts = (uint32_t)r1 | ((uint32_t)r2 << 16);
        }
    }
    d.mut_l = draw && lane >= MUTL && lane < MUTL + NCH && (uint64_t)w.x < a.thr_mut;
    return d;
}

// tournament of child L (lanes 0..2PP-1): first-drawn wins, a later aspirant
// replaces only on Fitness.__gt__ (one objective: not(a <= b))
template <int PP, bool TOURN>
__device__ __forceinline__ void bits_tournament(const BitsDraw& d, int t, int lane, int32_t& k,
                                                double& f) {
    constexpr int NCH = 2 * PP;
    k = d.k0;
    f = d.f0;
    if (TOURN) {
        for (int jj = 1; jj < t; ++jj) {
            const int src = (jj >> 1) * NCH + (lane % NCH);
            const double fj = __shfl((jj & 1) ? d.f1 : d.f0, src, 64);
            const int32_t kj = __shfl((jj & 1) ? d.k1 : d.k0, src, 64);
            if (!(fj <= f)) {
                f = fj;
                k = kj;
            }
        }
    }
}

template <int PP, int WPL, bool TOURN>
__device__ __forceinline__ void bits_resolve(const GenArgs& a, const BitsDraw& d, int64_t p0,
                                             int lane, BitsGroup<PP, WPL>& g) {
    constexpr int NCH = 2 * PP;
    constexpr int CXL = 32, MUTL = 32 + 2 * PP;
    const int t = TOURN ? a.tournsize : 1;
    // tournament of child L (lanes 0..NCH-1): first-drawn wins, a later
    // aspirant replaces only on Fitness.__gt__ (one objective: not(a <= b))
    int32_t k;
    double f;
    bits_tournament<PP, TOURN>(d, t, lane, k, f);
    // per child (lanes 0..NCH-1): its pair's crossover flag, its mutation flag
    // (shuffles outside any condition: a bpermute reads 0 from inactive lanes)
    const int ch = lane % NCH;
    const bool live = lane < NCH && 2 * p0 + ch < a.nc;
    g.p0 = p0;
    g.f = f;
    g.cx_c = __shfl((int)d.cxf_l, CXL + (ch >> 1), 64) != 0;
    const int mut_c = __shfl((int)d.mut_l, MUTL + ch, 64);
    g.mut = live && mut_c != 0;
    g.mut_bits = __ballot(g.mut);
    // the winner's validity is only needed for the fitness store: loaded with
    // the rows, off the decision chain (one random byte per child, not t)
    g.v = 1;
    if (live && !(g.cx_c || g.mut))
        g.v = (a.pkeys && a.pkeys[k] != FIT_KEY_NONE) ? 1u : a.pvalid[k];
    const int64_t npairs = (a.nc + 1) / 2;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        g.s0[q] = __builtin_amdgcn_readlane(k, 2 * q);
        g.s1[q] = __builtin_amdgcn_readlane(k, 2 * q + 1);
        g.cut[q] = (uint32_t)__builtin_amdgcn_readlane((int)d.cuts, CXL + q);
        g.cxf[q] = (uint32_t)__builtin_amdgcn_readlane((int)d.cxf_l, CXL + q);
    }
#pragma unroll
    for (int w = 0; w < WPL; ++w) {  // every row's first 512 B, then the next ones
        const bool lw = lane + 64 * w < a.words64;
#pragma unroll
        for (int q = 0; q < PP; ++q) {
            g.y0[q][w] = 0;
            g.y1[q][w] = 0;
            if (lw && p0 + q < npairs) {
                const uint64_t* r0 =
                    reinterpret_cast<const uint64_t*>(a.pgenes + (int64_t)g.s0[q] * a.pstride) + 64 * w;
                const uint64_t* r1 =
                    reinterpret_cast<const uint64_t*>(a.pgenes + (int64_t)g.s1[q] * a.pstride) + 64 * w;
#if DM_BITS_NTLOAD
                g.y0[q][w] = __builtin_nontemporal_load(r0 + lane);
                if (2 * (p0 + q) + 1 < a.nc) g.y1[q][w] = __builtin_nontemporal_load(r1 + lane);
#else
                g.y0[q][w] = r0[lane];
                if (2 * (p0 + q) + 1 < a.nc) g.y1[q][w] = r1[lane];
#endif
            }
        }
    }
}

// Vary, store and evaluate the group's children; returns how many fitnesses
// were invalidated (nevals).
template <int PP, int WPL, int CX, int MUT, bool EVAL>
__device__ __forceinline__ int bits_finish(const GenArgs& a, BitsGroup<PP, WPL>& g, int lane,
                                           uint64_t* flip_lds) {
    constexpr int NCH = 2 * PP;
    const int64_t npairs = (a.nc + 1) / 2;
    uint32_t my_count = 0;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
        const int64_t pq = g.p0 + q;
        if (pq >= npairs) break;
        const int64_t c0 = 2 * pq, c1 = 2 * pq + 1;
        const bool h1 = c1 < a.nc;
        uint64_t f0[WPL], f1[WPL];  // flip masks: precomputed slot, or drawn now
#pragma unroll
        for (int w = 0; w < WPL; ++w) f0[w] = f1[w] = 0;
        if (MUT == DM_MUT_FLIPBIT && !(DM_BITS_ABLATE & 1)) {
            const uint64_t below = g.mut_bits & ((1ull << (2 * q)) - 1);
            const int r0 = __popcll(below), r1 = r0 + (int)((g.mut_bits >> (2 * q)) & 1);
            uint64_t* spare = flip_lds + FLIP_SLOTS * 64 * WPL;
            if ((g.mut_bits >> (2 * q)) & 1) {
                if (r0 < FLIP_SLOTS) {
#pragma unroll
                    for (int w = 0; w < WPL; ++w) f0[w] = flip_lds[(r0 * WPL + w) * 64 + lane];
                } else {
                    flip_mask_row_w<WPL>(a, c0, lane, spare, f0);
                }
            }
            if ((g.mut_bits >> (2 * q + 1)) & 1) {
                if (r1 < FLIP_SLOTS) {
#pragma unroll
                    for (int w = 0; w < WPL; ++w) f1[w] = flip_lds[(r1 * WPL + w) * 64 + lane];
                } else {
                    flip_mask_row_w<WPL>(a, c1, lane, spare, f1);
                }
            }
        }
        uint32_t pc_l = 0;
#pragma unroll
        for (int w = 0; w < WPL; ++w) {
            const int wi = lane + 64 * w;
            if (wi < a.words64) {
                uint64_t x0 = g.y0[q][w], x1 = g.y1[q][w];
                if (CX == DM_CX_TWOPOINT && g.cxf[q]) {
                    const int cp1 = (int)(g.cut[q] & 0xFFFFu), cp2 = (int)(g.cut[q] >> 16);
                    const uint64_t m = range_mask(cp1 - wi * 64, cp2 - wi * 64);
                    const uint64_t tt = (x0 ^ x1) & m;
                    x0 ^= tt;
                    x1 ^= tt;
                }
                x0 ^= f0[w];  // mutation after the crossover (algorithms.py:72-81)
                x1 ^= f1[w];
                uint64_t* w0 = reinterpret_cast<uint64_t*>(a.cgenes + c0 * a.cstride);
                uint64_t* w1 = reinterpret_cast<uint64_t*>(a.cgenes + c1 * a.cstride);
                __builtin_nontemporal_store(x0, w0 + wi);
                if (h1) __builtin_nontemporal_store(x1, w1 + wi);
                pc_l += (uint32_t)__popcll(x0) | ((uint32_t)__popcll(x1) << 16);
            }
        }
        if (EVAL) {
            // both children's counts in one 32-bit sum (a row of <= 16,384 genes)
            const uint32_t pc = wave_sum_u32(pc_l);
            if ((lane >> 1) == q) my_count = (lane & 1) ? (pc >> 16) : (pc & 0xFFFFu);
        }
    }
    // fitness / validity of the group's children (contiguous stores)
    const int64_t c = 2 * g.p0 + (lane % NCH);
    const bool live = lane < NCH && c < a.nc;
    const bool inv = live && (g.cx_c || g.mut || !g.v);
    if (live) {
        if (EVAL) {
            a.cwv[c] = inv ? (double)my_count * a.w0 : g.f;
            a.cvalid[c] = 1;
        } else {  // no evaluation requested: clones keep their fitness
            a.cwv[c] = g.f;
            a.cvalid[c] = inv ? 0 : 1;
        }
    }
    return __popcll(__ballot(inv));
}

#ifndef DM_BITS_MINW
#define DM_BITS_MINW 1  // minimum waves per SIMD the fused kernel is compiled for (A/B)
#endif

// WPL: 64-word pieces per row (lane L holds words L + 64 k): rows of up to
// 4,096 / 8,192 / 16,384 genes
template <int PP, int CX, int MUT, bool EVAL, bool TOURN, int WPL = 1>
__global__ __launch_bounds__(256, DM_BITS_MINW) void gen_bits_fused_kernel(GenArgs a,
                                                                           long long* spread) {
    static_assert(PP == 4 || PP == 8, "lane layout: 4 or 8 pairs per wave");
    // FLIP_SLOTS + 1 flip-mask rows of 64 WPL words per wave (3.5 KiB per piece)
    __shared__ uint64_t flip_lds_all[4 * (FLIP_SLOTS + 1) * 64 * WPL];
    uint64_t* flip_lds = flip_lds_all + (threadIdx.x >> 6) * ((FLIP_SLOTS + 1) * 64 * WPL);
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t ngroups = (npairs + PP - 1) / PP;
    const int64_t grp = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int evals = 0;
    if (grp < ngroups) {  // one group per wave
        BitsGroup<PP, WPL> g;
#if DM_BITS_PRIO
        // the decision chain (Philox -> aspirant keys -> tournament) gates the
        // wave's row loads: it issues ahead of the other waves' streaming work
        __builtin_amdgcn_s_setprio(DM_BITS_PRIO);
#endif
        const BitsDraw d = bits_draw<PP, CX, MUT, TOURN>(a, grp * PP, lane);
        bits_resolve<PP, WPL, TOURN>(a, d, grp * PP, lane, g);
#if DM_BITS_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        if (MUT == DM_MUT_FLIPBIT && !(DM_BITS_ABLATE & 1))
            flip_rows_to_lds<2 * PP, WPL>(a, 2 * grp * PP, g.mut_bits, lane, flip_lds);
        evals = bits_finish<PP, WPL, CX, MUT, EVAL>(a, g, lane, flip_lds);
    }
    if (EVAL && spread) {  // nevals: workgroup count, folded by the last workgroup
        __shared__ int32_t wave_evals[4];
        if (lane == 0) wave_evals[threadIdx.x >> 6] = evals;
        __syncthreads();
        if (threadIdx.x == 0)
            evals_fold(spread, a.nevals,
                       (long long)wave_evals[0] + wave_evals[1] + wave_evals[2] + wave_evals[3]);
    }
}


// 8 pairs per wave (ONE Philox call per lane draws every decision of the
// wave: 16 children x 2 selection calls, 8 x 2 crossover calls, 16 mutation
// flags) when t <= 4; 4 pairs per wave for 4 < t <= 8.
static int fused_pp(const GenArgs& a) {
    return (a.sel != DM_SEL_TOURNAMENT || a.tournsize <= 4) ? 8 : 4;
}

// One-shot grid: one wave per group.
template <int PP, int CX, int MUT, bool EVAL, bool TOURN>
static void launch_bf(const GenArgs& a, long long* wg, hipStream_t s) {
    const int64_t waves = ((a.nc + 1) / 2 + PP - 1) / PP;
    const dim3 grid((unsigned)((waves + 3) / 4));
    if (a.words64 <= 64)
        gen_bits_fused_kernel<PP, CX, MUT, EVAL, TOURN, 1><<<grid, 256, 0, s>>>(a, wg);
    else if (a.words64 <= 128)
        gen_bits_fused_kernel<PP, CX, MUT, EVAL, TOURN, 2><<<grid, 256, 0, s>>>(a, wg);
    else
        gen_bits_fused_kernel<PP, CX, MUT, EVAL, TOURN, 4><<<grid, 256, 0, s>>>(a, wg);
}
template <int PP, int CX, int MUT>
static void launch_bf_e(const GenArgs& a, bool eval, long long* wg, hipStream_t s) {
    const bool tourn = a.sel == DM_SEL_TOURNAMENT;
    if (eval)
        tourn ? launch_bf<PP, CX, MUT, true, true>(a, wg, s)
              : launch_bf<PP, CX, MUT, true, false>(a, wg, s);
    else
        tourn ? launch_bf<PP, CX, MUT, false, true>(a, wg, s)
              : launch_bf<PP, CX, MUT, false, false>(a, wg, s);
}
template <int PP>
static void launch_bf_pp(const GenArgs& a, bool eval, long long* wg, hipStream_t s) {
    const bool mf = a.mut == DM_MUT_FLIPBIT;
    if (a.cx == DM_CX_TWOPOINT)
        mf ? launch_bf_e<PP, DM_CX_TWOPOINT, DM_MUT_FLIPBIT>(a, eval, wg, s)
           : launch_bf_e<PP, DM_CX_TWOPOINT, DM_MUT_NONE>(a, eval, wg, s);
    else
        mf ? launch_bf_e<PP, DM_CX_NONE, DM_MUT_FLIPBIT>(a, eval, wg, s)
           : launch_bf_e<PP, DM_CX_NONE, DM_MUT_NONE>(a, eval, wg, s);
}

// spread: the context's zeroed nevals counters, or null when nevals is not
// counted (the kernel's last workgroup adds the total to a.nevals).
void launch_gen_bits_fused(const GenArgs& a, bool eval, long long* spread, hipStream_t s) {
    long long* wg = (eval && a.nevals) ? spread : nullptr;
    if (fused_pp(a) == 8)
        launch_bf_pp<8>(a, eval, wg, s);
    else
        launch_bf_pp<4>(a, eval, wg, s);
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
