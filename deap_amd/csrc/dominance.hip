// dominance.hip — fast path of sortNondominated (deap/tools/emo.py:53-117)
// for 2..4 objectives and NaN-free fitnesses: the unique fitnesses' dominance
// relation over integer ranks, each unordered pair of 64-blocks computed once,
// and a front-peeling loop driven by the device.
//
// 1. Ranks.  Fitness.dominates (base.py:209-224) only asks, per objective,
//    whether x > y, x < y or neither; replacing every objective value by its
//    dense rank among the U unique values (-0.0 == 0.0, as Python compares)
//    preserves all three answers, so the O(M U^2) pass compares int32 ranks
//    (full-rate VALU compares) instead of fp64 values.  A NaN compares neither
//    way with anything and has no rank: populations holding one take the fp64
//    kernels of nsga2.hip.
// 2. Dominance.  Rows are ordered by objective 0 (q order), so a row can only
//    dominate the rows before it: tri_dom_kernel computes the lower triangle
//    only (section 2 below), D[a][b] one bit, with b's dominator count as
//    int16 partials per (A-group, b) summed by tri_count.  D is stored in
//    tiles of 64 rows x 16 words (tword): one 128-byte line per row and
//    1024-v segment.
// 3. Fronts.  Front 0 = count 0 in U order (nsga2.hip).  Then per front a
//    peel kernel reads the members' row lines (whole lines), transposes the
//    64 x 64-bit blocks with DPP / permlane moves (transpose.hpp) and
//    subtracts the dominator counts; a v whose count reaches zero joins the
//    next front's candidates with the key (last releasing position, U index).
//    One workgroup then orders the candidates by that key — the order the
//    reference's peel loop appends them in (emo.py:106-115, SURVEY.md
//    §8a-a21) — writes the front, its ranks and its individual count, and
//    decides termination on the device.  The host only checks a status word
//    every few fronts.
#include "bitdom.hpp"

#include <atomic>
#include "transpose.hpp"

namespace dm {

// ---------------------------------------------------------------------------
// 1. ranks in objective-0 order
// ---------------------------------------------------------------------------
// Unique fitness u gets the position q = pos[u] of its group in the
// population's lexicographic order (sigma[q] = u), so objective 0 ascends
// with q.  S[q] = int4 {rank_1, .., rank_{m-1}, rank_0, pad}: objective 0's
// dense rank is component m-1.
__global__ void lex_flags_kernel(const double* wv, int m, const int32_t* perm,
                                 const int32_t* segin, int64_t n, int32_t* fst, int32_t* f0) {
    DGRID_LOOP(j, n) {
        fst[j] = (j == 0 || segin[j] != 0) ? 1 : 0;
        f0[j] = (j == 0 || !(wv[(int64_t)perm[j] * m] == wv[(int64_t)perm[j - 1] * m])) ? 1 : 0;
    }
}
__global__ void lex_sigma_kernel(const int32_t* perm, const int32_t* uidx, const int32_t* fst,
                                 const int32_t* qex, const int32_t* f0, const int32_t* rex,
                                 int64_t n, int m, int32_t* sigma, int32_t* pos, int32_t* S) {
    DGRID_LOOP(j, n) {
        if (fst[j]) {
            const int32_t q = qex[j], u = uidx[perm[j]];
            sigma[q] = u;
            pos[u] = q;
            S[(int64_t)q * 4 + (m - 1)] = rex[j] + f0[j] - 1;
        }
    }
}
// Dense ranks of objectives 1..m-1 over the U unique fitnesses, batched:
// element j of segment g = j / U holds objective g + 1 of unique row j % U.
__global__ void rank_key_kernel(const double* ufit, int m, int64_t U, int64_t nb, uint64_t* keys,
                                int32_t* vals) {
    DGRID_LOOP(j, nb) {
        const int64_t g = j / U, u = j - g * U;
        keys[j] = ordered_key(ufit[u * m + g + 1]);
        vals[j] = (int32_t)u;
    }
}
__global__ void rank_flag_kernel(const uint64_t* keys, int64_t U, int64_t nb, int32_t* flag) {
    DGRID_LOOP(j, nb) flag[j] = (j % U != 0 && keys[j] != keys[j - 1]) ? 1 : 0;
}
// rank within the segment: the prefix count of new values since its start
__global__ void rank_scatter_kernel(const int32_t* vals, const int32_t* excl, const int32_t* flag,
                                    const int32_t* pos, int64_t U, int64_t nb, int32_t* S) {
    DGRID_LOOP(j, nb) {
        const int64_t g = j / U;
        S[(int64_t)pos[vals[j]] * 4 + g] = excl[j] + flag[j] - excl[g * U];
    }
}

// ---------------------------------------------------------------------------
// 2. dominance below the objective-0 diagonal
// ---------------------------------------------------------------------------
// a can dominate b only if rank_0(a) >= rank_0(b), i.e. (with ties aside)
// only for b before a in q order.  A wave owns an A-group of TD_WPW 64-row
// blocks (dominators a in the lanes, ranks in VGPRs) and sweeps the 64-v
// blocks B that the group's largest rank_0 can reach (v wave-uniform, ranks
// by scalar loads).  When every rank_0 of B is below every rank_0 of the
// group ("strict" block pair) objective 0 is decided, and a dominates b iff
// its other m-1 ranks are >= b's: m-1 compares whose wave masks are ANDed by
// the SALU.  Otherwise (the group's own blocks, rank_0 ties across blocks)
// the full test: min(x - y) >= 0 and max(x - y) > 0 over all m ranks.  The
// mask bit of lane a is shifted into a's word D[a][B] lane-locally
// (t = 2t + bit, one v_addc); the mask's popcount is b's dominator count
// contribution, parked in lane b%64 and stored as an int16 partial per
// (A-group, b).  Words above the reach of a group are never written (the
// peel skips them), so the matrix costs about half the bytes and compares of
// the symmetric pass and the strict inner step is m-1 compares + 1 add.
constexpr int TD_SEGS = 2;  // 8-block row segments (512 v) per task

// D layout: tword (dominance.hpp).  A wave's store of 4 words of its 64 rows
// is 64 pieces of 32 bytes that fill the tile's lines over four such stores;
// a peel read of a row segment is one whole line.

// nseg[g]: 8-block segments of v the rows of A-group g reach (every v whose
// rank_0 <= the group's largest); toff[g]: first task of g (TD_SEGS segments
// per task), toff[ngroups] = tasks.  One workgroup; nseg is nondecreasing.
// nseg[g] = the 512-v segments row group g (TD_WPW 64-row blocks) can
// reach: up to the last q whose rank_0 does not exceed the group's largest
// (rank_0 ascends with q).
__device__ __forceinline__ int32_t group_reach(const int4* S, int m, int64_t U, int64_t NG,
                                               int64_t g) {
    const int64_t last = std::min<int64_t>((g + 1) * TD_WPW * 64, U) - 1;
    const int32_t rmax = icomp(S[last], m - 1);
    int64_t lo = last, hi = U - 1;  // last q with rank_0 <= rmax
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (icomp(S[mid], m - 1) <= rmax) lo = mid;
        else hi = mid - 1;
    }
    return (int32_t)std::min<int64_t>(NG, (lo >> 9) + 1);
}
// the bitset path needs only nseg (no compare-kernel tile offsets): one
// thread per group over the whole grid instead of tri_plan_kernel's single
// workgroup (18.6 us at C5)
__global__ void group_reach_kernel(const int4* S, int m, int64_t U, int64_t NG, int64_t ngroups,
                                   int32_t* nseg) {
    DGRID_LOOP(g, ngroups) nseg[g] = group_reach(S, m, U, NG, g);
}

__global__ __launch_bounds__(1024) void tri_plan_kernel(const int4* S, int m, int64_t U,
                                                        int64_t NG, int64_t ngroups,
                                                        int32_t* nseg, int32_t* toff,
                                                        int32_t* counter) {
    __shared__ int32_t sh[1024];
    __shared__ int32_t carry;
    const int tid = threadIdx.x;
    if (tid == 0) {
        carry = 0;
        *counter = 0;
    }
    __syncthreads();
    for (int64_t base = 0; base < ngroups; base += 1024) {
        const int64_t g = base + tid;
        int32_t nt = 0;
        if (g < ngroups) {
            const int32_t ns = group_reach(S, m, U, NG, g);
            nseg[g] = ns;
            nt = (ns + TD_SEGS - 1) / TD_SEGS;
        }
        sh[tid] = nt;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const int32_t add = tid >= off ? sh[tid - off] : 0;
            __syncthreads();
            sh[tid] += add;
            __syncthreads();
        }
        const int32_t c0 = carry;
        if (g < ngroups) toff[g] = c0 + sh[tid] - nt;
        __syncthreads();
        if (tid == 1023) carry = c0 + sh[1023];
        __syncthreads();
    }
    if (tid == 0) toff[ngroups] = carry;
}

// t + t + (bit `lane` of mask): one v_addc_co_u32 with the wave mask as the
// carry-in (lane-local "shift in the bit of this lane").
#ifndef DM_TD_ILP
#define DM_TD_ILP 1  // 0: the round-2 per-A-block order (A/B)
#endif
// Not volatile: a pure function of its operands, so the scheduler may
// interleave the independent shift-ins of the 4 A-blocks (a volatile asm kept
// them in program order, each waiting on its own compare -> s_and chain).
__device__ __forceinline__ uint32_t add2_carry(uint32_t t, uint32_t a, uint64_t mask) {
    uint32_t out;
    uint64_t cout;
#if DM_TD_ILP
    asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4"
        : "=v"(out), "=s"(cout)
        : "v"(t), "v"(a), "s"(mask));
#else
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %3, %4"
                 : "=v"(out), "=s"(cout)
                 : "v"(t), "v"(a), "s"(mask));
#endif
    return out;
}

// v_writelane_b32 with an immediate lane: lane L of old <- the wave-uniform val
template <int L>
__device__ __forceinline__ int32_t writelane(int32_t old, int32_t val) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(val), "i"(L));
    return old;
}

// Dominator counts.  DM_TD_TCOUNT = 1 (default): after each 64-row block the
// group's words (lane a: bit j <-> a dominates row j of the block) are
// transposed across the wave (TransposerX, DPP / permlane moves) so that lane
// j holds the dominators of row j and counts them with v_bcnt — per block and
// A-block one transpose (~31 VALU) instead of 64 s_bcnt1 + s_add on the SALU
// and a v_writelane per row (r02: 1.16e9 SALU beside 1.36e9 VALU
// instructions per launch, profiles/r03b).  0: the per-row SALU count.
#ifndef DM_TD_TCOUNT
#define DM_TD_TCOUNT 1
#endif
// DM_TD_WQ = 1: the D words of 4 consecutive v blocks are kept and stored
// as two 16-B pieces per row; 0: one 8-B store per row and block.
#ifndef DM_TD_WQ
#define DM_TD_WQ 1
#endif
// DM_TD_SROWS = 1: the v block's ranks (wave-uniform) come by scalar loads
// into SGPRs instead of an LDS broadcast into VGPRs.
#ifndef DM_TD_SROWS
#define DM_TD_SROWS 1
#endif

// one row b (ranks y) against the group's lanes: shift the dominance bits
// into tw, return b's dominator count over the group (0 when counted by
// transposes)
template <int M, bool STRICT>
__device__ __forceinline__ int32_t td_row(const int4 y4, const int32_t (&x)[TD_WPW][M],
                                          uint32_t (&tw)[TD_WPW]) {
    int32_t y[M];
    y[0] = y4.x;
    y[1] = y4.y;
    if constexpr (M > 2) y[2] = y4.z;
    if constexpr (M > 3) y[3] = y4.w;
    int32_t cnt = 0;
    // all compares of the row first (independent wave masks), then the ANDs,
    // then the shift-ins: the VALU -> SALU -> VALU chains of the 4 A-blocks
    // overlap instead of running one after the other
    uint64_t msk[TD_WPW];
#pragma unroll
    for (int k = 0; k < TD_WPW; ++k) {
        if constexpr (STRICT) {
            msk[k] = __ballot(x[k][0] >= y[0]);
        } else {
            int32_t mn = x[k][0] - y[0], mx = mn;
#pragma unroll
            for (int o = 1; o < M; ++o) {
                const int32_t d = x[k][o] - y[o];
                mn = min(mn, d);
                mx = max(mx, d);
            }
            msk[k] = __ballot(mn >= 0) & __ballot(mx > 0);
        }
    }
    if constexpr (STRICT) {
#pragma unroll
        for (int o = 1; o < M - 1; ++o)
#pragma unroll
            for (int k = 0; k < TD_WPW; ++k) msk[k] &= __ballot(x[k][o] >= y[o]);
    }
#pragma unroll
    for (int k = 0; k < TD_WPW; ++k) {
        tw[k] = add2_carry(tw[k], tw[k], msk[k]);
#if !defined(DM_TD_NOCOUNT) && !DM_TD_TCOUNT
        cnt += __popcll(msk[k]);
#endif
    }
    return cnt;
}

// rows JTOP..JTOP-31 of a full block (descending: bit j of the word <-> row
// j); the block's ranks are in the wave's LDS buffer (broadcast reads), the
// next four rows read ahead
template <int M, bool STRICT, int JTOP, int J4 = 0>
__device__ __forceinline__ void td_half(const int4* L, const int32_t (&x)[TD_WPW][M],
                                        uint32_t (&tw)[TD_WPW], int32_t& cpark, const int4 (&cur)[4]) {
    int4 nxt[4];
    if constexpr (J4 + 4 < 32) {
#pragma unroll
        for (int i = 0; i < 4; ++i) nxt[i] = L[JTOP - J4 - 4 - i];
    }
    if constexpr (DM_TD_TCOUNT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) (void)td_row<M, STRICT>(cur[i], x, tw);
    } else {
        cpark = writelane<JTOP - J4>(cpark, td_row<M, STRICT>(cur[0], x, tw));
        cpark = writelane<JTOP - J4 - 1>(cpark, td_row<M, STRICT>(cur[1], x, tw));
        cpark = writelane<JTOP - J4 - 2>(cpark, td_row<M, STRICT>(cur[2], x, tw));
        cpark = writelane<JTOP - J4 - 3>(cpark, td_row<M, STRICT>(cur[3], x, tw));
    }
    if constexpr (J4 + 4 < 32) td_half<M, STRICT, JTOP, J4 + 4>(L, x, tw, cpark, nxt);
}
template <int M, bool STRICT, int JTOP>
__device__ __forceinline__ void td_half(const int4* L, const int32_t (&x)[TD_WPW][M],
                                        uint32_t (&tw)[TD_WPW], int32_t& cpark) {
    int4 cur[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cur[i] = L[JTOP - i];
    td_half<M, STRICT, JTOP, 0>(L, x, tw, cpark, cur);
}

// the last, partial block (nb < 64 rows): rows past the end shift in zeros
template <int M, bool STRICT>
__device__ void td_partial_half(const int4* L, int jtop, int nb,
                                const int32_t (&x)[TD_WPW][M], uint32_t (&tw)[TD_WPW],
                                int32_t& cpark) {
    for (int j = jtop; j > jtop - 32; --j) {
        if (j >= nb) {
#pragma unroll
            for (int k = 0; k < TD_WPW; ++k) tw[k] += tw[k];
            continue;
        }
        const int32_t cnt = td_row<M, STRICT>(L[j], x, tw);
        if constexpr (!DM_TD_TCOUNT) cpark = (int)(threadIdx.x & 63) == j ? cnt : cpark;
    }
}

// Persistent: each wave takes tasks (A-group g, TD_SEGS segments of B) from
// an atomic counter until toff[ngroups] are done.
template <int M>
__global__ __launch_bounds__(256) void tri_dom_kernel(const int4* __restrict__ S, int64_t U,
                                                      int64_t NB, int64_t NQ, int64_t ngroups,
                                                      const int32_t* __restrict__ nseg,
                                                      const int32_t* __restrict__ toff,
                                                      int32_t* counter, uint64_t* __restrict__ D,
                                                      int16_t* __restrict__ part) {
#if !DM_TD_SROWS
    __shared__ int4 sbuf[4][64];  // per wave: the ranks of the current v block
    int4* Lw = sbuf[threadIdx.x >> 6];
#endif
    const int lane = threadIdx.x & 63;
    const TransposerX tr(lane);
    const int64_t Upad = NB * 64;
    const int32_t total = toff[ngroups];
    for (;;) {
        int32_t t = 0;
        if (lane == 0) t = atomicAdd(counter, 1);
        t = __builtin_amdgcn_readfirstlane(t);
        if (t >= total) break;
        int64_t lo = 0, hi = ngroups - 1;  // last g with toff[g] <= t
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (toff[mid] <= t) lo = mid;
            else hi = mid - 1;
        }
        const int64_t g = lo, c = t - toff[g];
        const int64_t A0 = g * TD_WPW;
        int32_t x[TD_WPW][M];
#pragma unroll
        for (int k = 0; k < TD_WPW; ++k) {
            const int64_t r = (A0 + k) * 64 + lane;
            const int4 xr = r < U ? S[r] : make_int4(-1, -1, -1, -1);  // past the end: no bits
            x[k][0] = xr.x;
            x[k][1] = xr.y;
            if constexpr (M > 2) x[k][2] = xr.z;
            if constexpr (M > 3) x[k][3] = xr.w;
        }
        const int32_t rmin = __builtin_amdgcn_readfirstlane(icomp(S[A0 * 64], M - 1));
        const int64_t B0 = c * TD_SEGS * 8;
        const int64_t B1 = std::min<int64_t>(std::min<int64_t>((int64_t)nseg[g], (c + 1) * TD_SEGS) * 8, NB);
#if !DM_TD_SROWS
        int4 nxt = B0 < B1 ? S[B0 * 64 + lane] : make_int4(0, 0, 0, 0);
#endif
        // words of 4 consecutive v blocks, stored together (whole 2 KB tiles)
        uint64_t wq[TD_WPW][4];
#pragma unroll
        for (int k = 0; k < TD_WPW; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) wq[k][i] = 0;
        for (int64_t B = B0; B < B1; ++B) {
            const int nb = (int)std::min<int64_t>(64, U - B * 64);
#if DM_TD_SROWS
            // the block's ranks are wave-uniform: scalar loads into SGPRs (no
            // LDS staging, no VGPRs for the rows in flight)
            const int4* L = S + B * 64;
            const bool strict = icomp(L[nb - 1], M - 1) < rmin;
#else
            int4* L = Lw;
            L[lane] = nxt;  // the previous block's reads were issued before (in-order LDS)
            if (B + 1 < B1) nxt = S[(B + 1) * 64 + lane];
            const bool strict = __builtin_amdgcn_readfirstlane(icomp(L[nb - 1], M - 1)) < rmin;
#endif
            uint32_t th[TD_WPW], tl[TD_WPW];
#pragma unroll
            for (int k = 0; k < TD_WPW; ++k) th[k] = tl[k] = 0;
            int32_t cpark = 0;
            if (nb == 64) {
                if (strict) {
                    td_half<M, true, 63>(L, x, th, cpark);
                    td_half<M, true, 31>(L, x, tl, cpark);
                } else {
                    td_half<M, false, 63>(L, x, th, cpark);
                    td_half<M, false, 31>(L, x, tl, cpark);
                }
            } else if (strict) {
                td_partial_half<M, true>(L, 63, nb, x, th, cpark);
                td_partial_half<M, true>(L, 31, nb, x, tl, cpark);
            } else {
                td_partial_half<M, false>(L, 63, nb, x, th, cpark);
                td_partial_half<M, false>(L, 31, nb, x, tl, cpark);
            }
            if constexpr (DM_TD_TCOUNT) {
                uint32_t lo[TD_WPW], hi[TD_WPW];
#pragma unroll
                for (int k = 0; k < TD_WPW; ++k) {
                    lo[k] = tl[k];
                    hi[k] = th[k];
                }
                tr.run<TD_WPW>(lo, hi);  // lane j: bit a <-> lane a dominates row j
                cpark = 0;
#pragma unroll
                for (int k = 0; k < TD_WPW; ++k) cpark += __popc(lo[k]) + __popc(hi[k]);
            }
            part[g * Upad + B * 64 + lane] = (int16_t)cpark;
#if !DM_TD_WQ
            // one 8-B word per row and block, stored at once (no VGPRs for the
            // 4-block line pieces; L2 merges the pieces of a line)
#pragma unroll
            for (int k = 0; k < TD_WPW; ++k)
                if (A0 + k < NB)
                    D[tword((A0 + k) * 64 + lane, B, NQ)] = ((uint64_t)th[k] << 32) | tl[k];
            continue;
#endif
            const int bq = (int)(B & 3);
#pragma unroll
            for (int k = 0; k < TD_WPW; ++k) {
                const uint64_t w = ((uint64_t)th[k] << 32) | tl[k];
#pragma unroll
                for (int i = 0; i < 4; ++i) wq[k][i] = bq == i ? w : wq[k][i];
            }
            if (bq == 3 || B + 1 == B1) {
#pragma unroll
                for (int k = 0; k < TD_WPW; ++k) {
                    if (A0 + k < NB) {
                        uint4* q = reinterpret_cast<uint4*>(D + tword((A0 + k) * 64 + lane, B & ~3ll, NQ));
                        const uint4 v0 = make_uint4((uint32_t)wq[k][0], (uint32_t)(wq[k][0] >> 32),
                                                    (uint32_t)wq[k][1], (uint32_t)(wq[k][1] >> 32));
                        const uint4 v1 = make_uint4((uint32_t)wq[k][2], (uint32_t)(wq[k][2] >> 32),
                                                    (uint32_t)wq[k][3], (uint32_t)(wq[k][3] >> 32));
                        // plain stores: the four 32-B pieces of a line merge in L2
                        // (nontemporal stores of the pieces measured 3x slower)
                        q[0] = v0;
                        q[1] = v1;
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) wq[k][i] = 0;
                }
            }
        }
    }
}

// count[sigma[q]] (U order, front 0) = countq[q] (q order, the peel) = sum
// over the A-groups reaching q's segment of part[g][q].  The column sums are
// split over TC_CHUNKS ranges of g (grid y) so that enough loads are in
// flight (a column of segment 0 has ngroups partials): a thread sums 4
// adjacent q (one 8-byte load per g, 8 in flight) into tmp[chunk][q], and
// tri_count_sum_kernel adds the chunks.
constexpr int TC_CHUNKS = 4;
__global__ __launch_bounds__(256) void tri_count_part_kernel(const int16_t* __restrict__ part,
                                                             const int32_t* __restrict__ nseg,
                                                             int64_t U, int64_t Upad, int64_t ngroups,
                                                             int32_t* __restrict__ tmp) {
    const int64_t q0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (q0 >= U) return;
    const int32_t sq = (int32_t)(q0 >> 9);
    int64_t lo = 0, hi = ngroups;  // first g with nseg[g] > sq
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (nseg[mid] > sq) hi = mid;
        else lo = mid + 1;
    }
    const int64_t ch = (ngroups + TC_CHUNKS - 1) / TC_CHUNKS;
    const int64_t g0 = std::max<int64_t>(lo, blockIdx.y * ch);
    const int64_t g1 = std::min<int64_t>(ngroups, (blockIdx.y + 1) * ch);
    int32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    const uint2* col = reinterpret_cast<const uint2*>(part + q0);  // Upad % 64 == 0: aligned
    const int64_t rs = Upad / 4;                                    // row stride in uint2
    auto add = [&](uint2 x) {
        c0 += (int16_t)(x.x & 0xFFFF);
        c1 += (int16_t)(x.x >> 16);
        c2 += (int16_t)(x.y & 0xFFFF);
        c3 += (int16_t)(x.y >> 16);
    };
    int64_t g = g0;
    for (; g + 8 <= g1; g += 8) {
        uint2 x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = col[(g + i) * rs];
#pragma unroll
        for (int i = 0; i < 8; ++i) add(x[i]);
    }
    for (; g < g1; ++g) add(col[g * rs]);
    int32_t* out = tmp + blockIdx.y * U + q0;
    out[0] = c0;
    if (q0 + 1 < U) out[1] = c1;
    if (q0 + 2 < U) out[2] = c2;
    if (q0 + 3 < U) out[3] = c3;
}
__global__ void tri_count_sum_kernel(const int32_t* __restrict__ tmp, const int32_t* __restrict__ sigma,
                                     int64_t U, int32_t* __restrict__ count,
                                     int32_t* __restrict__ countq) {
    DGRID_LOOP(q, U) {
        int32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < TC_CHUNKS; ++c) cnt += tmp[c * U + q];
        count[sigma[q]] = cnt;
        countq[q] = cnt;
    }
}

// ---------------------------------------------------------------------------
// 3. device-driven front peeling
// ---------------------------------------------------------------------------
struct FrontState {
    int32_t F;         // size of the current front (ulist[ustart, ustart + F))
    int32_t ustart;
    int32_t nfronts;   // fronts emitted after front 0
    int32_t done;
    int32_t overflow;  // candidates exceed the LDS sort: the host orders them
    int32_t ncand;     // candidates of the next front appended by the peel
    int64_t sorted;    // individuals in the emitted fronts
    int64_t pending;   // individuals of the released candidates (gsize sums)
    int64_t lastinds;  // individuals of the last emitted front
    int64_t N;         // min(n, k)
    int64_t U;
};

// Released candidates go to eight slot buckets (bucket = the releasing
// workgroup's chunk or segment index mod 8) instead of one shared counter:
// every workgroup of a peel launch that releases something took a returning
// atomic on st->ncand and st->pending, and ~400 of them serialised on those
// two addresses (the release phase's slowest workgroup took 7-19 us on the
// fronts of a few hundred members, profiles/r05_peelphase).  Bucket b's
// counters live in their own 4-KB page after the state (st + 4096 (b + 1):
// slot count, and the released individuals at +64), its candidates in slots
// [b cap, b cap + count) of ckey / cq / crec, cap = cand_cap(U) (room for
// every v of the chunks of 512 or segments of 1,024 that map to it).  The
// ordering reads the eight ranges as one list (CandMap) and resets the
// counters.
constexpr int CAND_BUCKETS = 8;
constexpr size_t CAND_PAGE = 4096;
__host__ __device__ __forceinline__ int64_t cand_cap(int64_t U) { return (U + 8191) / 8192 * 1024; }
__device__ __forceinline__ int32_t* cand_count(FrontState* st, int b) {
    return reinterpret_cast<int32_t*>(reinterpret_cast<char*>(st) + CAND_PAGE * (b + 1));
}
__device__ __forceinline__ unsigned long long* cand_pending(FrontState* st, int b) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(st) + CAND_PAGE * (b + 1) + 64);
}
// candidate i of the ordering's list -> its slot
struct CandMap {
    int32_t pre[CAND_BUCKETS + 1];  // bucket starts in the list (pre[8] = n)
    int64_t cap;                    // 0: the list is contiguous (presorted, overflow path)
    // static indices only (a dynamic pre[b] put the map in scratch memory)
    __device__ __forceinline__ int64_t slot(int32_t i) const {
        if (!cap) return i;
        int32_t base = 0;
        int64_t off = 0;
#pragma unroll
        for (int k = 1; k < CAND_BUCKETS; ++k)
            if (i >= pre[k]) {
                base = pre[k];
                off = k * cap;
            }
        return off + (i - base);
    }
    // the workgroup-uniform map in scalar registers
    __device__ __forceinline__ CandMap uniform() const {
        CandMap m;
#pragma unroll
        for (int k = 0; k <= CAND_BUCKETS; ++k) m.pre[k] = __builtin_amdgcn_readfirstlane(pre[k]);
        m.cap = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)cap) |
                ((int64_t)__builtin_amdgcn_readfirstlane((int32_t)(cap >> 32)) << 32);
        return m;
    }
};

#ifndef DM_PEEL_WAVES
#define DM_PEEL_WAVES 8
#endif
constexpr int PEEL_WAVES = DM_PEEL_WAVES;  // waves of a peel workgroup (they split the front's members)
#ifndef DM_PEEL_BATCH
#define DM_PEEL_BATCH 2
#endif
constexpr int PEEL_BATCH = DM_PEEL_BATCH;  // member chunks per wave in flight
constexpr int PEEL_WORDS = TW;  // words of a row segment (one line)
// One workgroup (8 waves) owns one row segment s of D: PEEL_WORDS = 16 words,
// v in [1024 s, 1024 s + 1024) in q order, one 128-byte line of a row.  Its
// waves take interleaved 64-member chunks of the front, load each member's
// line (whole lines: the reads of a front's random rows fetch no bytes of
// other rows), transpose the 64 x 64-bit blocks, and the per-wave
// (dominators, last position) of each v are reduced in LDS.  v is written by
// this workgroup only, so countq needs no atomics; a v whose count reaches
// zero is released: its rank, its sort key (last releasing position, U index),
// its row and its individual count are recorded here, so the ordering kernel
// only sorts.  A row's reach (mrow.y) counts 512-v halves: the words of a half
// past it were never stored and read as zero.
// Slices of the front's members for segment s (grid y = K): a row reaches the
// segments up to its own, so segment s is read by about (1 - s/NS) of the
// members and the low segments carry the most work; they are split over up
// to K workgroups (at least PEEL_SLICE_MIN members each).
#ifndef DM_PEEL_SLICES
#define DM_PEEL_SLICES 4
#endif
constexpr int PEEL_SLICES = DM_PEEL_SLICES;
#ifndef DM_PEEL_SLICE_MIN
#define DM_PEEL_SLICE_MIN 1024
#endif
constexpr int64_t PEEL_SLICE_MIN = DM_PEEL_SLICE_MIN;
// the table peel's slices hold at least 2,048 members: its workgroups repeat
// the chunk's table loads and release per slice, and C5 measured 3.58 ms/gen
// with 2,048-8,192 against 3.69 with 1,024 (profiles/r03y)
#ifndef DM_PEEL_TAB_SLICE_MIN
#define DM_PEEL_TAB_SLICE_MIN 2048
#endif
__device__ __forceinline__ int64_t peel_slices(int64_t F, int64_t s, int64_t NS, int64_t K,
                                               int64_t smin = PEEL_SLICE_MIN) {
    const int64_t byload = (K * (NS - s) + NS - 1) / NS;
    return std::max<int64_t>(1, std::min<int64_t>(byload, F / smin));
}
// Data one phase of the persistent peel hands to another crosses workgroups
// on different XCDs, whose L2s are not coherent with each other: those
// accesses are agent-scope relaxed loads / stores (sc1, served coherently)
// when COH; plain otherwise (separate launches: the kernel boundary makes
// them visible).
template <bool COH, typename T>
__device__ __forceinline__ T cld(const T* p) {
    if constexpr (COH)
        return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        return *p;
}
template <bool COH, typename T>
__device__ __forceinline__ void cst(T* p, T v) {
    if constexpr (COH)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}
template <bool COH>
__device__ __forceinline__ int2 cld2(const int2* p) {
    if constexpr (COH) {
        const unsigned long long x = __hip_atomic_load(
            reinterpret_cast<unsigned long long*>(const_cast<int2*>(p)), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        return make_int2((int32_t)(uint32_t)x, (int32_t)(uint32_t)(x >> 32));
    } else {
        return *p;
    }
}
template <bool COH>
__device__ __forceinline__ void cst2(int2* p, int2 v) {
    if constexpr (COH)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                           (unsigned long long)(uint32_t)v.x | ((unsigned long long)(uint32_t)v.y << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

constexpr int PEEL_PV = PEEL_WORDS * 64;                 // v of a row segment
constexpr int PEEL_IT = PEEL_PV / (PEEL_WAVES * 64);      // v per thread
template <int PV>
struct PeelLdsT {
    int32_t sdec[PEEL_WAVES][PV];
    int32_t slast[PEEL_WAVES][PV];
};
template <int PV>
struct PeelSmallT {
    static constexpr int IT = PV / (PEEL_WAVES * 64);
    int32_t wcnt[IT][PEEL_WAVES];
    int64_t wgs[IT][PEEL_WAVES];
    int32_t sbase;
};
typedef PeelLdsT<PEEL_PV> PeelLds;
typedef PeelSmallT<PEEL_PV> PeelSmall;

template <bool COH, int PW>
__device__ void peel_release(const int32_t (&dec)[PW], const int32_t (&last)[PW], int64_t vbase,
                             const int32_t* __restrict__ gsize, const int32_t* __restrict__ sigma,
                             FrontState* st, int32_t* countq, unsigned long long* lastq,
                             uint64_t* ckey, int32_t* cq, int32_t* rankU, int64_t U, int32_t snf,
                             int64_t nsl, PeelLdsT<PW * 64>& L, PeelSmallT<PW * 64>& S);

// Slice y of the nsl slices of row segment s for the front of sF unique
// fitnesses starting at sust in ulist / mrow (front number snf).
template <bool COH>
__device__ void peel_segment(const uint64_t* __restrict__ D, int64_t NQ, const int2* mrow,
                             const int32_t* __restrict__ gsize, const int32_t* __restrict__ sigma,
                             FrontState* st, int32_t* countq, unsigned long long* lastq,
                             uint64_t* ckey, int32_t* cq, int32_t* rankU, int64_t U, int32_t sF,
                             int32_t sust, int32_t snf, int64_t s, int64_t y, int64_t nsl,
                             PeelLds& L, PeelSmall& S) {
    constexpr int PW = PEEL_WORDS, PV = PEEL_PV;
    // members of this workgroup's slice [j0s, F)
    const int64_t slen = ((sF + nsl - 1) / nsl + 63) & ~63ll;
    const int64_t j0s = y * slen;
    const int64_t F = std::min<int64_t>(sF, j0s + slen);
    const int2* members = mrow + sust;  // (row in q order, 512-v halves it reaches)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const TransposerX tr(lane);
    int32_t dec[PW], last[PW];
#pragma unroll
    for (int w = 0; w < PW; ++w) {
        dec[w] = 0;
        last[w] = -1;
    }
    constexpr int64_t STEP = PEEL_WAVES * 64;
    // member rows of the next batch are loaded one batch ahead
    int2 mr[PEEL_BATCH];
#pragma unroll
    for (int b = 0; b < PEEL_BATCH; ++b) {
        const int64_t j = j0s + (int64_t)wave * 64 + b * STEP + lane;
        mr[b] = j < F ? cld2<COH>(members + j) : make_int2(0, 0);
    }
    for (int64_t jb = j0s + (int64_t)wave * 64; jb < F; jb += STEP * PEEL_BATCH) {
        uint4 seg[PEEL_BATCH][PW / 2];
        bool has[PEEL_BATCH][2];
#pragma unroll
        for (int b = 0; b < PEEL_BATCH; ++b) {
            const uint4* q = reinterpret_cast<const uint4*>(D + tword(mr[b].x, s * PW, NQ));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                has[b][h] = 2 * s + h < mr[b].y;
#pragma unroll
                for (int i = 0; i < PW / 4; ++i)
                    seg[b][h * (PW / 4) + i] = has[b][h] ? q[h * (PW / 4) + i] : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int b = 0; b < PEEL_BATCH; ++b) {
            const int64_t j = jb + (PEEL_BATCH + b) * STEP + lane;
            mr[b] = j < F ? cld2<COH>(members + j) : make_int2(0, 0);
        }
#pragma unroll
        for (int b = 0; b < PEEL_BATCH; ++b) {
            const int64_t j0 = jb + b * STEP;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (__ballot(has[b][h]) == 0) continue;  // no member of the chunk reaches the half
                uint32_t lo[8], hi[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint4 x = seg[b][h * 4 + i];
                    lo[2 * i] = x.x;
                    hi[2 * i] = x.y;
                    lo[2 * i + 1] = x.z;
                    hi[2 * i + 1] = x.w;
                }
                tr.run<8>(lo, hi);  // lane v: bit i <-> member j0+i dominates v
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    dec[h * 8 + w] += __popc(lo[w]) + __popc(hi[w]);
                    const int32_t top = hi[w] ? 63 - __clz(hi[w]) : (lo[w] ? 31 - __clz(lo[w]) : -1);
                    if (top >= 0) last[h * 8 + w] = (int32_t)(j0 + top);
                }
            }
        }
    }
    peel_release<COH, PW>(dec, last, s * PV, gsize, sigma, st, countq, lastq, ckey, cq, rankU, U,
                          snf, nsl, L, S);
}

// The workgroup's (dominators, last releasing position) per v of its segment
// [vbase, vbase + 64 PW) (dec / last: word w of this thread = v 64 w + lane,
// per wave) are reduced in LDS and applied to countq; a v whose count reaches
// zero is released into the next front's candidates.
template <bool COH, int PW>
__device__ void peel_release(const int32_t (&dec)[PW], const int32_t (&last)[PW], int64_t vbase,
                             const int32_t* __restrict__ gsize, const int32_t* __restrict__ sigma,
                             FrontState* st, int32_t* countq, unsigned long long* lastq,
                             uint64_t* ckey, int32_t* cq, int32_t* rankU, int64_t U, int32_t snf,
                             int64_t nsl, PeelLdsT<PW * 64>& L, PeelSmallT<PW * 64>& S) {
    constexpr int PEEL_IT = PeelSmallT<PW * 64>::IT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int w = 0; w < PW; ++w) {
        L.sdec[wave][w * 64 + lane] = dec[w];
        L.slast[wave][w * 64 + lane] = last[w];
    }
    __syncthreads();
    // release: one atomic per workgroup on the shared counters (a
    // same-address atomic per wave serialised ~6 ns each over thousands of
    // waves on the large fronts)
    bool fresh[PEEL_IT];
    int32_t lk[PEEL_IT], vu[PEEL_IT];
    unsigned long long fm[PEEL_IT];
#pragma unroll
    for (int it = 0; it < PEEL_IT; ++it) {
        const int t = threadIdx.x + it * PEEL_WAVES * 64;
        int32_t d = 0, l = -1;
#pragma unroll
        for (int wv = 0; wv < PEEL_WAVES; ++wv) {
            d += L.sdec[wv][t];
            l = max(l, L.slast[wv][t]);
        }
        const int64_t v = vbase + t;  // q order
        fresh[it] = false;
        if (v < U && d > 0) {
            if (nsl == 1) {
                const int32_t left = cld<COH>(countq + v) - d;
                cst<COH>(countq + v, left);
                fresh[it] = left == 0;
            } else {
                // several slices: publish the last position, then subtract;
                // the subtraction that reaches zero is ordered after every
                // slice's max (each waits for its max before subtracting)
                const unsigned long long key = ((unsigned long long)(snf + 1) << 32) | (uint32_t)l;
                __hip_atomic_fetch_max(lastq + v, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int32_t old = __hip_atomic_fetch_add(countq + v, -d, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (old == d) {
                    fresh[it] = true;
                    l = (int32_t)(uint32_t)__hip_atomic_fetch_max(lastq + v, key, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        lk[it] = l;
        vu[it] = fresh[it] ? sigma[v] : 0;
        fm[it] = __ballot(fresh[it]);
        int64_t gs = fresh[it] ? gsize[vu[it]] : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) gs += __shfl_xor(gs, o, 64);
        if (lane == 0) {
            S.wcnt[it][wave] = __popcll(fm[it]);
            S.wgs[it][wave] = gs;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t tot = 0;
        int64_t gtot = 0;
        for (int it = 0; it < PEEL_IT; ++it)
            for (int wv = 0; wv < PEEL_WAVES; ++wv) {
                const int32_t c = S.wcnt[it][wv];
                S.wcnt[it][wv] = tot;
                tot += c;
                gtot += S.wgs[it][wv];
            }
        const int b = (int)((vbase / (PW * 64)) & (CAND_BUCKETS - 1));
        S.sbase = tot ? (int32_t)(b * cand_cap(U)) + atomicAdd(cand_count(st, b), tot) : 0;
        if (gtot) atomicAdd(cand_pending(st, b), (unsigned long long)gtot);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PEEL_IT; ++it) {
        if (!fresh[it]) continue;
        const int64_t v = vbase + threadIdx.x + it * PEEL_WAVES * 64;
        const int32_t slot = S.sbase + S.wcnt[it][wave] + __popcll(fm[it] & ((1ull << lane) - 1));
        if (!BD_OK(slot, CAND_BUCKETS * cand_cap(U), "release slot") || !BD_OK(vu[it], U, "release vu")) continue;
        cst<COH>(ckey + slot, ((uint64_t)(uint32_t)lk[it] << 32) | (uint32_t)vu[it]);
        cst<COH>(cq + slot, (int32_t)v);
        cst<COH>(rankU + vu[it], snf + 1);
    }
    __syncthreads();  // the LDS is reused by the caller's next task
}

#ifndef DM_PEEL_MINW
#define DM_PEEL_MINW 1  // min waves per SIMD (4: two 512-thread workgroups per CU)
#endif
__global__ __launch_bounds__(PEEL_WAVES * 64, DM_PEEL_MINW) void peel_owned_kernel(const uint64_t* __restrict__ D,
                                                         int64_t NQ,
                                                         const int2* __restrict__ mrow,
                                                         const int32_t* __restrict__ gsize,
                                                         const int32_t* __restrict__ sigma,
                                                         FrontState* st, int32_t* countq,
                                                         unsigned long long* lastq,
                                                         uint64_t* ckey, int32_t* cq,
                                                         int32_t* rankU) {
    __shared__ PeelLds L;
    __shared__ PeelSmall S;
    __shared__ int32_t sF, sust, sstop, snf;
    if (threadIdx.x == 0) {
        sF = st->F;
        sust = st->ustart;
        snf = st->nfronts;
        sstop = st->done | st->overflow;
    }
    __syncthreads();
    if (sstop) return;
    const int64_t s = blockIdx.x;
    const int64_t nsl = peel_slices(sF, s, gridDim.x, gridDim.y);
    if ((int64_t)blockIdx.y >= nsl) return;
    peel_segment<false>(D, NQ, mrow, gsize, sigma, st, countq, lastq, ckey, cq, rankU, st->U, sF,
                        sust, snf, s, blockIdx.y, nsl, L, S);
}

#ifndef DM_PEEL_TAB_MINW
#define DM_PEEL_TAB_MINW 4  // min waves per SIMD (4: two 512-thread workgroups per CU)
#endif
#ifdef DM_PEEL_PROF
// phase clocks of each table-peel workgroup (diagnostic builds only):
// {chunk, slice, F, t_start, t_tables, t_members, t_release, 0}
__device__ unsigned long long g_pprof[1 << 20];
__device__ unsigned int g_pprof_n;
#define PPROF_T(x) const unsigned long long x = wall_clock64()
#else
#define PPROF_T(x)
#endif
constexpr int ORDER_CAP = 16384;  // candidates sorted in registers + LDS by one workgroup

// member i of a front: (its row in q order, the row segments it reaches)
__device__ __forceinline__ int2 member_row(int32_t u, const int32_t* pos, const int32_t* nseg) {
    const int32_t r = pos[u];
    return make_int2(r, nseg[r / (64 * TD_WPW)]);
}
// gsq (nullable): gsize[sigma[q]] per q, so the table peel's prologue loads
// it without a dependent second load
__global__ void member_rec_kernel(const int4* S, const int2* span, const int32_t* nseg, int64_t U,
                                  int4* qrec, unsigned long long* lastq,
                                  const int32_t* sigma = nullptr, const int32_t* gsize = nullptr,
                                  int32_t* gsq = nullptr, int32_t* qrec3 = nullptr) {
    DGRID_LOOP(q, U) {
        const int4 s = S[q];
        qrec[q] = make_int4(nseg[q / (64 * TD_WPW)], span[q].y, s.x, s.y);
        if (qrec3) qrec3[q] = s.z;  // four objectives: S[q].z is rank 3
        if (lastq) lastq[q] = 0;  // the sliced peels' (front, last position) per v
        if (gsq) gsq[q] = gsize[sigma[q]];
    }
}

template <int NT, int E, bool COH>
__device__ void order_sorted(const uint64_t* ckey, int32_t n, int32_t* out, int2* mout,
                             const int32_t* pos, const int32_t* nseg, uint64_t* lds,
                             const CandMap& cm) {
    uint64_t k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        k[e] = i < n ? cld<COH>(ckey + cm.slot(i)) : ~0ull;
    }
    block_bitonic<NT, E>(k, lds);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        if (i < n) {
            const int32_t u = (int32_t)(uint32_t)k[e];
            cst<COH>(out + i, u);
            cst2<COH>(mout + i, member_row(u, pos, nseg));
        }
    }
}

template <int CAP>
union OrderLds {
    uint64_t keys[CAP];
    struct {
        int32_t base[CAP + 1];
        int32_t tmp[CAP];
    } cs;
};
struct OrderScalars {
    int32_t sn, sgo, snstart, sF, smax;
    int64_t spending;  // individuals of the candidates (the buckets' sums)
    CandMap cm;
};

// Orders the released candidates by (last releasing position l, U index) and
// appends them to ulist / mrow as the next front, then updates the state
// (one workgroup of NT threads).  Counting sort: l < F (the current front's
// size), so the candidates are binned by l in LDS and ranked inside their bin
// by U index; a bin of more than ORDER_BIN_MAX candidates (or too many
// candidates) takes the bitonic sort of the whole key.  More than CAP
// candidates: overflow, the host's radix sort orders them (presorted: ckey
// already ordered).
constexpr int ORDER_BIN_MAX = 64;
// Exclusive prefix sum over the workgroup's threads: lane shuffles within
// each wave, one wave scans the wave totals (two barriers; a Hillis-Steele
// scan over 1,024 LDS slots took 20).  sh: NT / 64 ints of LDS.
template <int NT>
__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t* sh) {
    static_assert(NT % 64 == 0 && NT / 64 <= 64, "whole waves, at most 64");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    if (wave == 0) {
        int32_t w = lane < NT / 64 ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < NT / 64; o <<= 1) {
            const int32_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < NT / 64) sh[lane] = w;
    }
    __syncthreads();
    return x - v + (wave ? sh[wave - 1] : 0);
}

// The counting-sort ordering with E candidate slots per thread (E x NT >= n):
// the candidates binned by their last releasing position l < Fr, ranked in
// their bin by U index.  Returns false when a bin is too large for the
// in-bin scan (the caller's bitonic fallback orders them).  Templated on E so
// that the common fronts of a few thousand candidates do not carry the
// registers (and scratch spills) of the 16-slot form.
template <int NT, int E, int CAP, bool COH>
__device__ bool order_count(const uint64_t* ckey, const int32_t* cq, int32_t* out, int2* mout,
                            const int32_t* nseg,
                            const CandMap& cm, int32_t n, int32_t Fr, OrderLds<CAP>& lds,
                            int32_t* part, OrderScalars& sc) {
    const int tid = threadIdx.x;
    bool sorted_here = false;
    for (int i = tid; i <= Fr; i += NT) lds.cs.base[i] = 0;
    __syncthreads();
    uint64_t key[E];
    int32_t qv[E], slot[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        if (i < n) {
            const int64_t sl = cm.slot(i);
            key[e] = cld<COH>(ckey + sl);
            qv[e] = cld<COH>(cq + sl);
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        if (i < n) slot[e] = atomicAdd(&lds.cs.base[(int32_t)(key[e] >> 32)], 1);
    }
    __syncthreads();
    // exclusive prefix of the bin counts: thread t owns C consecutive bins
    const int C = (Fr + NT - 1) / NT;
    const int b0 = tid * C, b1 = min(Fr, b0 + C);
    int32_t sum = 0, mx = 0;
    for (int b = b0; b < b1; ++b) {
        const int32_t c = lds.cs.base[b];
        sum += c;
        mx = max(mx, c);
    }
    if (mx > ORDER_BIN_MAX) atomicMax(&sc.smax, mx);
    int32_t run = block_excl_scan<NT>(sum, part);
    for (int b = b0; b < b1; ++b) {
        const int32_t c = lds.cs.base[b];
        lds.cs.base[b] = run;
        run += c;
    }
    if (tid == 0) lds.cs.base[Fr] = n;
    __syncthreads();
    if (sc.smax == 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = tid + e * NT;
            if (i < n) lds.cs.tmp[lds.cs.base[(int32_t)(key[e] >> 32)] + slot[e]] = (int32_t)(uint32_t)key[e];
        }
        __syncthreads();
        // ranks first, then the member rows
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = tid + e * NT;
            if (i < n) {
                const int32_t l = (int32_t)(key[e] >> 32), vu = (int32_t)(uint32_t)key[e];
                const int32_t beg = lds.cs.base[l], end = lds.cs.base[l + 1];
                int32_t r = beg;
                for (int32_t j = beg; j < end; ++j) r += lds.cs.tmp[j] < vu ? 1 : 0;
                cst<COH>(out + r, vu);
                slot[e] = r;
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = tid + e * NT;
            if (i < n) cst2<COH>(mout + slot[e], make_int2(qv[e], nseg[qv[e] / (64 * TD_WPW)]));
        }
        sorted_here = true;
    }
    __syncthreads();  // the bitonic fallback reuses the LDS
    return sorted_here;
}

template <int NT, int CAP, bool COH>
__device__ void order_front(FrontState* st, const uint64_t* ckey, const int32_t* cq,
                            int32_t* ulist, int2* mrow, const int32_t* pos, const int32_t* nseg,
                            int32_t* fstarts, int presorted, OrderLds<CAP>& lds, int32_t* part,
                            OrderScalars& sc) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        const int32_t done = cld<COH>(&st->done), ovf = cld<COH>(&st->overflow);
        sc.sgo = !(done || (ovf && !presorted));
        // the candidate list: the eight slot buckets in order, or (presorted,
        // after the host's compaction and radix sort) ckey[0, ncand)
        int32_t run = 0;
        int64_t pend = 0;
        for (int b = 0; b < CAND_BUCKETS; ++b) {
            sc.cm.pre[b] = run;
            run += cld<COH>(cand_count(st, b));
            pend += (int64_t)cld<COH>(cand_pending(st, b));
        }
        sc.cm.pre[CAND_BUCKETS] = run;
        sc.cm.cap = presorted ? 0 : cand_cap(st->U);
        sc.sn = presorted ? cld<COH>(&st->ncand) : run;
        sc.spending = pend;
        sc.snstart = cld<COH>(&st->ustart) + cld<COH>(&st->F);
        sc.sF = cld<COH>(&st->F);
        sc.smax = 0;
    }
    __syncthreads();
    if (!sc.sgo) return;
    const int32_t n = sc.sn;
    const CandMap cm = sc.cm.uniform();
    if (!BD_OK(sc.snstart + (int64_t)n - 1, st->U, "order front end")) return;
    if (n == 0) {  // nothing released: the reference's `if F2 == 0: break`
        if (tid == 0) cst<COH>(&st->done, 1);
        return;
    }
    if (!presorted && n > CAP) {
        if (tid == 0) {
            cst<COH>(&st->ncand, n);  // the host compacts the buckets and sorts them
            cst<COH>(&st->overflow, 1);
        }
        return;
    }
    int32_t* out = ulist + sc.snstart;
    int2* mout = mrow + sc.snstart;
    bool sorted_here = false;
    if (presorted) {
        for (int i = tid; i < n; i += NT) {
            const int32_t u = (int32_t)(uint32_t)cld<COH>(ckey + i);
            cst<COH>(out + i, u);
            cst2<COH>(mout + i, member_row(u, pos, nseg));
        }
        sorted_here = true;
    } else if (sc.sF <= CAP) {
        // slots per thread for this front: 4 covers the C5 fronts (< 4,096)
        if (n <= 4 * NT)
            sorted_here = order_count<NT, 4, CAP, COH>(ckey, cq, out, mout, nseg, cm, n,
                                                       sc.sF, lds, part, sc);
        else if (n <= 8 * NT)
            sorted_here = order_count<NT, 8, CAP, COH>(ckey, cq, out, mout, nseg, cm, n,
                                                       sc.sF, lds, part, sc);
        else
            sorted_here = order_count<NT, CAP / NT, CAP, COH>(ckey, cq, out, mout, nseg,
                                                              cm, n, sc.sF, lds, part, sc);
    }
    if (!sorted_here) {
        uint64_t* keys = lds.keys;
        if (n <= NT) {
            order_sorted<NT, 1, COH>(ckey, n, out, mout, pos, nseg, keys, cm);
        } else if (n <= 2 * NT) {
            order_sorted<NT, 2, COH>(ckey, n, out, mout, pos, nseg, keys, cm);
        } else if (n <= 4 * NT) {
            order_sorted<NT, 4, COH>(ckey, n, out, mout, pos, nseg, keys, cm);
        } else if (n <= 8 * NT) {
            order_sorted<NT, 8, COH>(ckey, n, out, mout, pos, nseg, keys, cm);
        } else {
            static_assert(CAP <= 16 * NT, "order capacity exceeds the bitonic sizes");
            order_sorted<NT, 16, COH>(ckey, n, out, mout, pos, nseg, keys, cm);
        }
    }
    if (tid == 0) {
        const int32_t nstart = sc.snstart, r = cld<COH>(&st->nfronts);
        const int64_t pending = sc.spending;
        const int64_t sorted = cld<COH>(&st->sorted) + pending;
        cst<COH>(&st->sorted, sorted);
        cst<COH>(&st->lastinds, pending);

        cst<COH>(&st->ustart, nstart);
        cst<COH>(&st->F, n);
        cst<COH>(&st->nfronts, r + 1);
        __hip_atomic_store(&st->ncand, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int b = 0; b < CAND_BUCKETS; ++b) {  // empty buckets for the next peel
            __hip_atomic_store(cand_count(st, b), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cand_pending(st, b), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        cst<COH>(&st->overflow, 0);
        cst<COH>(fstarts + r + 2, nstart + n);
        // emo.py:109: continue while pareto_sorted < N (and fronts remain)
        if (sorted >= cld<COH>(&st->N) || nstart + n >= cld<COH>(&st->U)) cst<COH>(&st->done, 1);
    }
}

__global__ __launch_bounds__(1024) void front_order_kernel(FrontState* st, const uint64_t* ckey,
                                                           const int32_t* cq, int32_t* ulist,
                                                           int2* mrow, const int32_t* pos,
                                                           const int32_t* nseg, int32_t* fstarts,
                                                           int presorted) {
    __shared__ OrderLds<ORDER_CAP> lds;
    __shared__ int32_t part[1024];
    __shared__ OrderScalars sc;
    order_front<1024, ORDER_CAP, false>(st, ckey, cq, ulist, mrow, pos, nseg, fstarts, presorted,
                                        lds, part, sc);
}

// The overflow path's compaction: bucket blockIdx.y's candidates to
// out[pre_b + j] (pre_b: the earlier buckets' counts).
__global__ void cand_compact_kernel(FrontState* st, const uint64_t* ckey, int64_t cap,
                                    uint64_t* out) {
    const int b = blockIdx.y;
    int32_t pre = 0;
    for (int k = 0; k < b; ++k) pre += *cand_count(st, k);
    const int32_t cnt = *cand_count(st, b);
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < cnt;
         j += (int64_t)gridDim.x * blockDim.x)
        out[pre + j] = ckey[b * cap + j];
}

__global__ void member_rows_kernel(const int32_t* ulist, const int32_t* Fp, const int32_t* pos,
                                   const int32_t* nseg, int2* mrow) {
    const int64_t F = *Fp;
    DGRID_LOOP(j, F) {
        mrow[j] = member_row(ulist[j], pos, nseg);
    }
}

// one workgroup per 4-KB page of the state and its candidate buckets: the
// pages zeroed, then (workgroup 0) the state of front 0
__global__ void front_init_kernel(FrontState* st, const int32_t* F0p, const int64_t* sorted0p,
                                  int64_t N, int64_t U, int32_t* fstarts) {
    uint4* page = reinterpret_cast<uint4*>(reinterpret_cast<char*>(st) + CAND_PAGE * blockIdx.x);
    for (int i = threadIdx.x; i < (int)(CAND_PAGE / 16); i += blockDim.x) page[i] = make_uint4(0, 0, 0, 0);
    if (blockIdx.x != 0) return;
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int32_t F0 = *F0p;
    const int64_t sorted0 = *sorted0p;
    st->F = F0;
    st->ustart = 0;
    st->nfronts = 0;
    st->done = (sorted0 >= N || F0 >= U || F0 == 0) ? 1 : 0;
    st->overflow = 0;
    st->ncand = 0;
    st->sorted = sorted0;
    st->lastinds = sorted0;
    st->pending = 0;
    st->N = N;
    st->U = U;
    fstarts[0] = 0;
    fstarts[1] = F0;
}

// ---------------------------------------------------------------------------
// 3b. the table peel with the ordering one launch behind it (2-3 objectives)
// ---------------------------------------------------------------------------
// Which fits form front j+1 depends only on front j's membership: a v is
// released when the front's members that dominate it bring its count to
// zero, whatever their order.  Only the ORDER of front j+1 (emo.py:96-104:
// a fit is appended when its last dominator -- in front order -- is
// processed, after the ones that dominator released before it, in U order)
// needs front j's order.  So the two chains are separated:
//  * the peel of front j (the chunk workgroups) takes its members in slot
//    order and only counts; it releases front j+1's members into candidate
//    buffer (j+1) % 3 (eight slot buckets, as above);
//  * TAB_NA search workgroups of the same launch find, for each member v of
//    front j (released by the previous launch), its last dominator: front
//    j-1's members sit in front order in the record table (mtab), and a scan
//    from the end of that front stops at the first member u with q(v) <=
//    tie-group end(u) and r_i(v) <= r_i(u) -- the relation the bitset rows
//    encode -- which is the one of largest position.  The key (position, U
//    index) goes to the candidate's slot with a coherent store; the last
//    search workgroup to arrive sorts front j by it (counting sort), writes
//    it to ulist and its records to mtab in front order, and hands the state
//    to launch j+1.
// One launch per front, where the peel and the ordering took two dependent
// ones; the ordering is off the peel chain as long as it finishes within the
// peel's launch.
struct FrontStep {
    int64_t sorted;  // individuals in the fronts before j
    int32_t ustart;  // front j's start in ulist / mtab
    int32_t Fprev;   // size of front j - 1
    uint32_t valid;  // the call's epoch when written (entries of earlier calls stay in the workspace)
    int32_t done;    // no front j (emo.py:109, or every fit sorted)
    int32_t pad[2];
};
struct FrontSum {      // read by the host after each batch of launches
    int32_t nfronts;   // the last front ordered (fronts 1..nfronts after front 0)
    int32_t done;
    int32_t overflow;  // front nfronts + 1 has more members than the sorting workgroup holds
    int32_t ncand;
    int64_t sorted, lastinds;
    int64_t maxinds;    // individuals of the largest front so far (crowding's segmented sort)
    int32_t arrive[3];  // search workgroups done, per candidate buffer
};
// Four objectives on the bitset tables: diagnostic builds only (-DDM_BD_M4,
// see fast_bitset); the product build compiles the rank-3 copies out.
#ifdef DM_BD_M4
constexpr bool kBitsetM4 = true;
#else
constexpr bool kBitsetM4 = false;
#endif
struct CandBufs {
    char* pages;     // [3][8] counter pages: slot count at +0, released individuals at +64
    uint64_t* ckey;  // [3][8 cap]: U index, then (last position << 32 | U index)
    int32_t* cq;     // [3][8 cap]: q
    int4* crec;      // [3][8 cap]: the member record (reach, tie-group end, rank 1, rank 2)
    int32_t* crec3;  // [3][8 cap]: rank 3 of the record (four objectives), else null
    int64_t cap;
    __device__ __forceinline__ int32_t* count(int buf, int b) const {
        return reinterpret_cast<int32_t*>(pages + CAND_PAGE * (buf * CAND_BUCKETS + b));
    }
    __device__ __forceinline__ unsigned long long* pending(int buf, int b) const {
        return reinterpret_cast<unsigned long long*>(pages + CAND_PAGE * (buf * CAND_BUCKETS + b) + 64);
    }
    __device__ __forceinline__ int64_t base(int buf) const { return (int64_t)buf * CAND_BUCKETS * cap; }
};
struct TabArgs {
    const uint32_t* P;
    const int32_t* R;
    const uint16_t* BK;
    const int4* qrec;
    const int32_t* qrec3;  // rank 3 per q (four objectives), else null
    const int32_t* gsize;
    const int32_t* gsq;  // gsize[sigma[q]] per q (member_rec_kernel)
    const int32_t* sigma;
    const int32_t* pos;  // U index -> q
    int32_t* countq;
    int32_t* rankU;
    int32_t* ulist;
    int32_t* fstarts;
    int4* mtab;  // [U] member records in front order: front j at [ustart_j, ustart_j + n_j)
    int32_t* mtab3;  // [U] their rank 3 (four objectives), else null
    int32_t* gslot;  // [U] a large front's members' places in their bins (tab_sort_big)
    int32_t* gtmp;   // [U] ... its U indices binned
    uint64_t* gkey;  // [U] ... and its keys
    FrontStep* stf;
    FrontSum* sum;
    CandBufs cb;
    int64_t U, N;
    int64_t gx;      // chunk workgroups per slice row (NG rounded up to 8)
    uint32_t epoch;  // this call's stamp for stf entries
};
constexpr int TAB_NT = PEEL_WAVES * 64;       // the launch's workgroup size
constexpr int TAB_NA = 128;                   // search workgroups per launch (a multiple of 8)
constexpr int TAB_WIN = 2048;                 // peel members per window
constexpr int TAB_SWIN = 2048;                // previous-front members per search window
constexpr int TAB_ORDER_CAP = 16 * TAB_NT;    // members the sorting workgroup orders
template <int F>
struct TabLds {  // byte offsets in the launch's shared buffer
    static constexpr size_t sR = 0;
    static constexpr size_t sB = sR + 4 * F * BD_RP;
    static constexpr size_t dec = (sB + 2 * F * BD_BKN + 15) / 16 * 16;
    static constexpr size_t sM = dec + 4 * PEEL_WAVES * BD_CW;
    static constexpr size_t peel = sM + 16 * TAB_WIN;
    static constexpr size_t search = 16 * TAB_SWIN;
    static constexpr size_t order = sizeof(OrderLds<TAB_ORDER_CAP>);
    static constexpr size_t bytes = std::max(std::max(peel, search), order);
};
struct TabScalars {
    FrontStep sf;
    CandMap cm;
    int64_t pend;
    int32_t n, go, smax, sbase, last;
    int32_t wcnt[PEEL_WAVES];
    int64_t wgs[PEEL_WAVES];
    int32_t part[64];
};

// buffer `buf`'s candidate list (thread 0)
__device__ __forceinline__ void tab_cand_list(const CandBufs& cb, int buf, TabScalars& sc) {
    int32_t run = 0;
    int64_t p = 0;
    for (int b = 0; b < CAND_BUCKETS; ++b) {
        sc.cm.pre[b] = run;
        run += *cb.count(buf, b);
        p += (int64_t)*cb.pending(buf, b);
    }
    sc.cm.pre[CAND_BUCKETS] = run;
    sc.cm.cap = cb.cap;
    sc.n = run;
    sc.pend = p;
}

// Front j is ordered: empty front j-1's buffer and this launch's arrival
// count, hand the state to launch j+1 (thread 0).
__device__ void tab_finish(const TabArgs& a, int32_t j, int32_t n, int64_t pend, const FrontStep& sf) {
    const int rb = (j + 2) % 3;
    for (int b = 0; b < CAND_BUCKETS; ++b) {
        *a.cb.count(rb, b) = 0;
        *a.cb.pending(rb, b) = 0ull;
    }
    a.sum->arrive[j % 3] = 0;
    FrontStep nx{};
    nx.sorted = sf.sorted + pend;
    nx.ustart = sf.ustart + n;
    nx.Fprev = n;
    nx.valid = a.epoch;
    nx.done = (nx.sorted >= a.N || nx.ustart >= a.U) ? 1 : 0;
    a.stf[j + 1] = nx;
    a.fstarts[j + 1] = nx.ustart;
    a.sum->nfronts = j;
    a.sum->sorted = nx.sorted;
    a.sum->lastinds = pend;
    a.sum->maxinds = pend > a.sum->maxinds ? pend : a.sum->maxinds;
    a.sum->done = nx.done;
    a.sum->overflow = 0;
}

// counting sort of front j by its keys (last position l < Fr, U index):
// binned in LDS, ranked inside the bin (as order_count); false when a bin
// holds more than ORDER_BIN_MAX (the bitonic sort orders them)
template <int NT, int E>
__device__ bool tab_sort_count(const TabArgs& a, int64_t bbase, const CandMap& cm, int32_t n,
                               int32_t Fr, int32_t ustart, OrderLds<TAB_ORDER_CAP>& lds,
                               TabScalars& sc) {
    const int tid = threadIdx.x;
    for (int i = tid; i <= Fr; i += NT) lds.cs.base[i] = 0;
    uint64_t key[E];
    int32_t sidx[E], slot[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        sidx[e] = i < n ? (int32_t)cm.slot(i) : 0;
        key[e] = i < n ? cld<true>(a.cb.ckey + bbase + sidx[e]) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        if (i < n) {
            int32_t l = (int32_t)(key[e] >> 32);
            if (!BD_OK(l, Fr, "tab sort bin")) l = 0;
            slot[e] = atomicAdd(&lds.cs.base[l], 1);
        }
    }
    __syncthreads();
    const int C = (Fr + NT - 1) / NT;
    const int b0 = tid * C, b1 = min(Fr, b0 + C);
    int32_t sum = 0, mx = 0;
    for (int b = b0; b < b1; ++b) {
        const int32_t c = lds.cs.base[b];
        sum += c;
        mx = max(mx, c);
    }
    if (mx > ORDER_BIN_MAX) atomicMax(&sc.smax, mx);
    int32_t run = block_excl_scan<NT>(sum, sc.part);
    for (int b = b0; b < b1; ++b) {
        const int32_t c = lds.cs.base[b];
        lds.cs.base[b] = run;
        run += c;
    }
    if (tid == 0) lds.cs.base[Fr] = n;
    __syncthreads();
    if (sc.smax != 0) {
        __syncthreads();  // the bitonic fallback reuses the LDS
        return false;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        if (i < n) lds.cs.tmp[lds.cs.base[(int32_t)(key[e] >> 32)] + slot[e]] = (int32_t)(uint32_t)key[e];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * NT;
        if (i < n) {
            const int32_t l = (int32_t)(key[e] >> 32), vu = (int32_t)(uint32_t)key[e];
            const int32_t beg = lds.cs.base[l], end = lds.cs.base[l + 1];
            int32_t r = beg;
            for (int32_t q = beg; q < end; ++q) r += lds.cs.tmp[q] < vu ? 1 : 0;
            a.ulist[ustart + r] = vu;
            a.mtab[ustart + r] = a.cb.crec[bbase + sidx[e]];
            if (kBitsetM4 && a.mtab3) a.mtab3[ustart + r] = a.cb.crec3[bbase + sidx[e]];
        }
    }
    return true;
}
template <int NT, int E>
__device__ void tab_sort_bitonic(const TabArgs& a, int64_t bbase, const CandMap& cm, int32_t n,
                                 int32_t ustart, uint64_t* lds) {
    uint64_t k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        k[e] = i < n ? cld<true>(a.cb.ckey + bbase + cm.slot(i)) : ~0ull;
    }
    block_bitonic<NT, E>(k, lds);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = threadIdx.x * E + e;
        if (i < n) {
            const int32_t vu = (int32_t)(uint32_t)k[e];
            a.ulist[ustart + i] = vu;
            if (BD_OK(vu, a.U, "tab sorted vu")) {
                a.mtab[ustart + i] = a.qrec[a.pos[vu]];
                if (kBitsetM4 && a.mtab3) a.mtab3[ustart + i] = a.qrec3[a.pos[vu]];
            }
        }
    }
}

// A front of more than TAB_ORDER_CAP members: the same counting sort with
// the bins' starts in LDS (Fr + 1 <= TAB_BIG_BINS) and each member's place
// in its bin and the binned U indices in global memory (L2; agent-scope
// accesses); false when a bin holds more than TAB_BIG_BIN_MAX members (the
// host sorts the front then).
constexpr int TAB_BIG_BINS = TAB_ORDER_CAP * 2;  // ints of OrderLds<TAB_ORDER_CAP>
constexpr int TAB_BIG_BIN_MAX = 512;
template <int NT>
__device__ bool tab_sort_big(const TabArgs& a, int64_t bbase, const CandMap& cm, int32_t n,
                             int32_t Fr, int32_t ustart, int32_t* base, TabScalars& sc) {
    // the keys are read coherently once (the search workgroups stored them)
    // into the workgroup's own scratch (plain accesses from here on: one
    // workgroup, ordered by its barriers), four members per thread in flight
    constexpr int B = 4;
    const int tid = threadIdx.x;
    for (int i = tid; i <= Fr; i += NT) base[i] = 0;
    __syncthreads();
    for (int i0 = tid; i0 < n; i0 += B * NT) {
        uint64_t k[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b * NT;
            k[b] = i < n ? cld<true>(a.cb.ckey + bbase + cm.slot(i)) : 0;
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b * NT;
            if (i < n) {
                int32_t l = (int32_t)(k[b] >> 32);
                if (!BD_OK(l, Fr, "tab big bin")) l = 0;
                a.gkey[i] = k[b];
                a.gslot[i] = atomicAdd(&base[l], 1);
            }
        }
    }
    __syncthreads();
    const int C = (Fr + NT - 1) / NT;
    const int b0 = tid * C, b1 = min(Fr, b0 + C);
    int32_t sum = 0, mx = 0;
    for (int b = b0; b < b1; ++b) {
        const int32_t c = base[b];
        sum += c;
        mx = max(mx, c);
    }
    if (mx > TAB_BIG_BIN_MAX) atomicMax(&sc.smax, mx);
    int32_t run = block_excl_scan<NT>(sum, sc.part);
    for (int b = b0; b < b1; ++b) {
        const int32_t c = base[b];
        base[b] = run;
        run += c;
    }
    if (tid == 0) base[Fr] = n;
    __syncthreads();
    if (sc.smax != 0) return false;
    for (int i0 = tid; i0 < n; i0 += B * NT) {
        uint64_t k[B];
        int32_t g[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b * NT;
            k[b] = i < n ? a.gkey[i] : 0;
            g[b] = i < n ? a.gslot[i] : 0;
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (i0 + b * NT < n) a.gtmp[base[(int32_t)(k[b] >> 32)] + g[b]] = (int32_t)(uint32_t)k[b];
    }
    __syncthreads();
    for (int i0 = tid; i0 < n; i0 += B * NT) {
        uint64_t k[B];
        int4 rec[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int i = i0 + b * NT;
            k[b] = i < n ? a.gkey[i] : 0;
            rec[b] = i < n ? a.cb.crec[bbase + cm.slot(i)] : make_int4(0, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (i0 + b * NT >= n) continue;
            const int32_t l = (int32_t)(k[b] >> 32), vu = (int32_t)(uint32_t)k[b];
            const int32_t beg = base[l], end = base[l + 1];
            int32_t r = beg;
            for (int32_t q = beg; q < end; ++q) r += a.gtmp[q] < vu ? 1 : 0;
            a.ulist[ustart + r] = vu;
            a.mtab[ustart + r] = rec[b];
            if (kBitsetM4 && a.mtab3) a.mtab3[ustart + r] = a.cb.crec3[bbase + cm.slot(i0 + b * NT)];
        }
    }
    return true;
}

// the last search workgroup of launch j: front j in order (n <= TAB_ORDER_CAP)
template <int NT>
__device__ void tab_sort_front(const TabArgs& a, int32_t j, char* smem, TabScalars& sc) {
    const int32_t n = sc.n;
    const CandMap cm = sc.cm.uniform();
    const int64_t bbase = a.cb.base(j % 3);
    const int32_t Fr = sc.sf.Fprev, ustart = sc.sf.ustart;
    auto& lds = *reinterpret_cast<OrderLds<TAB_ORDER_CAP>*>(smem);
    if (threadIdx.x == 0) sc.smax = 0;
    __syncthreads();
    bool done = false;
    if (Fr <= TAB_ORDER_CAP) {
        if (n <= 4 * NT)
            done = tab_sort_count<NT, 4>(a, bbase, cm, n, Fr, ustart, lds, sc);
        else if (n <= 8 * NT)
            done = tab_sort_count<NT, 8>(a, bbase, cm, n, Fr, ustart, lds, sc);
        else
            done = tab_sort_count<NT, 16>(a, bbase, cm, n, Fr, ustart, lds, sc);
    }
    if (!done) {
        if (n <= 2 * NT)
            tab_sort_bitonic<NT, 2>(a, bbase, cm, n, ustart, lds.keys);
        else if (n <= 4 * NT)
            tab_sort_bitonic<NT, 4>(a, bbase, cm, n, ustart, lds.keys);
        else if (n <= 8 * NT)
            tab_sort_bitonic<NT, 8>(a, bbase, cm, n, ustart, lds.keys);
        else
            tab_sort_bitonic<NT, 16>(a, bbase, cm, n, ustart, lds.keys);
    }
    if (threadIdx.x == 0) tab_finish(a, j, n, sc.pend, sc.sf);
}

// Search workgroup aw of launch j >= 1 (see the top of this section).
#ifdef DM_PEEL_PROF
// search workgroup stamps (diagnostic builds): aw, j, n, start, state read,
// search done, end (after the sort for the last arriver), 1 + 2 last
__device__ void sprof_rec(int aw, int32_t j, int32_t n, unsigned long long t0,
                          unsigned long long t1, unsigned long long t2, bool last) {
    const unsigned long long t3 = wall_clock64();
    if (threadIdx.x != 0) return;
    const unsigned int e = atomicAdd(&g_pprof_n, 1u);
    if (e < (1u << 17)) {
        unsigned long long* o = g_pprof + (size_t)e * 8;
        o[0] = aw; o[1] = j; o[2] = n; o[3] = t0; o[4] = t1; o[5] = t2; o[6] = t3;
        o[7] = 1 + 2 * (unsigned long long)last + ((unsigned long long)j << 8);
    }
}
#define SPROF(last) sprof_rec(aw, j, sc.n, st0, st1, st2, last)
#else
#define SPROF(last)
#endif

template <int F>
__device__ void tab_search(const TabArgs& a, int32_t j, int aw, char* smem, TabScalars& sc) {
    PPROF_T(st0);
    const int tid = threadIdx.x;
    const int buf = j % 3;
    if (tid == 0) {
        sc.sf = a.stf[j];
        sc.go = sc.sf.valid == a.epoch && !sc.sf.done;
        if (sc.go) tab_cand_list(a.cb, buf, sc);
    }
    __syncthreads();
    if (!sc.go) return;
    PPROF_T(st1);
    const int32_t n = sc.n;
    if (n == 0) {  // nothing released: every fit is in a front
        if (aw == 0 && tid == 0) {
            FrontStep nx{};
            nx.valid = a.epoch;
            nx.done = 1;
            a.stf[j + 1] = nx;
            a.sum->done = 1;
        }
        return;
    }
    const CandMap cm = sc.cm.uniform();
    const int64_t bbase = a.cb.base(buf);
    const int32_t n1 = sc.sf.Fprev;
    const int64_t us0 = (int64_t)sc.sf.ustart - n1;  // front j-1 in mtab
    int4* sP = reinterpret_cast<int4*>(smem);         // (tie-group end, rank 1, rank 2, rank 3) per member
    const int32_t per = (n + TAB_NA - 1) / TAB_NA;
    const int32_t i0 = aw * per, i1 = min(n, i0 + per);
    // the share in chunks of TAB_NT candidates, 64 per wave; a wave tests 64
    // members of front j-1 per step for one candidate (one ballot), its
    // members read from the LDS window 512 at a time into registers, so the
    // candidates of the wave reuse them
    const int lane = tid & 63;
    for (int32_t c0 = i0; c0 < i1; c0 += TAB_NT) {  // workgroup-uniform
        // candidate c0 + 8 lane + wave: a small share spreads over every wave
        const int32_t i = c0 + 8 * lane + (tid >> 6);
        const bool mine = i < i1;
        int64_t sl = 0;
        int32_t vq = 0, vr1 = 0, vr2 = 0, vr3 = 0;
        uint32_t vu = 0;
        if (mine) {
            sl = bbase + cm.slot(i);
            const int4 rec = a.cb.crec[sl];
            vq = a.cb.cq[sl];
            vr1 = rec.z;
            vr2 = rec.w;
            if (F == 3) vr3 = a.cb.crec3[sl];
            vu = (uint32_t)a.cb.ckey[sl];
        }
        int32_t last = -1;
        uint64_t open = __ballot(mine);  // the wave's candidates without their last dominator yet
        for (int32_t wend = n1; wend > 0; wend -= TAB_SWIN) {
            if (__syncthreads_and(open == 0)) break;  // all found (and the window read out)
            const int32_t wb = max(0, wend - TAB_SWIN);
            for (int32_t t = wb + tid; t < wend; t += TAB_NT) {
                const int4 r = a.mtab[us0 + t];
                sP[t - wb] = make_int4(r.y, r.z, r.w, F == 3 ? a.mtab3[us0 + t] : 0);
            }
            __syncthreads();
            // 512-member segments from the window's end; member k of this lane
            // is position sb - 1 - 64 k - lane (descending in k and lane)
            for (int32_t sb = wend; sb > wb && open; sb -= 8 * 64) {
                int4 mk[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int32_t pk = sb - 1 - 64 * k - lane;
                    mk[k] = pk >= wb ? sP[pk - wb] : make_int4(-1, 0, 0, 0);  // te -1: dominates nothing
                }
                uint64_t todo = open;
                while (todo) {
                    const int cl = __ffsll((unsigned long long)todo) - 1;
                    todo &= todo - 1;
                    const int32_t cq1 = __builtin_amdgcn_readlane(vq, cl);
                    const int32_t cr1 = __builtin_amdgcn_readlane(vr1, cl);
                    const int32_t cr2 = __builtin_amdgcn_readlane(vr2, cl);
                    const int32_t cr3 = F == 3 ? __builtin_amdgcn_readlane(vr3, cl) : 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        bool dom = cq1 <= mk[k].x && cr1 <= mk[k].y;
                        if (F >= 2) dom = dom && cr2 <= mk[k].z;
                        if (F == 3) dom = dom && cr3 <= mk[k].w;
                        const uint64_t hit = __ballot(dom);
                        if (hit) {  // the lowest lane holds the largest position
                            if (lane == cl) last = sb - 1 - 64 * k - (__ffsll((unsigned long long)hit) - 1);
                            open &= ~(1ull << cl);
                            break;
                        }
                    }
                }
            }
        }
        if (mine) {
            if (!BD_OK(last, n1, "tab last dominator")) last = 0;
            cst<true>(a.cb.ckey + sl, ((uint64_t)(uint32_t)last << 32) | vu);
        }
        __syncthreads();  // the next chunk's first window overwrites sP
    }
    // every key stored (coherently) before this workgroup counts itself in
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PPROF_T(st2);
    __syncthreads();
    if (tid == 0)
        sc.last = __hip_atomic_fetch_add(a.sum->arrive + buf, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == TAB_NA - 1;
    __syncthreads();
    if (!sc.last) {
        SPROF(false);
        return;
    }
    if (!BD_OK(sc.sf.ustart + (int64_t)n - 1, a.U, "tab front end")) return;
    if (n > TAB_ORDER_CAP) {
        if (tid == 0) sc.smax = 0;
        __syncthreads();
        if (sc.sf.Fprev < TAB_BIG_BINS &&
            tab_sort_big<TAB_NT>(a, a.cb.base(buf), sc.cm.uniform(), n, sc.sf.Fprev, sc.sf.ustart,
                                 reinterpret_cast<int32_t*>(smem), sc)) {
            if (tid == 0) tab_finish(a, j, n, sc.pend, sc.sf);
        } else if (tid == 0) {  // the host sorts this front (tab_presorted_kernel)
            a.sum->ncand = n;
            a.sum->overflow = 1;
        }
        return;
    }
    tab_sort_front<TAB_NT>(a, j, smem, sc);
    SPROF(true);
}

// The members [wb, we) of the front being peeled (member i at slot bbase +
// cm.slot(i)) whose row reaches chunk c, into LDS: sM = (rank 1, rank 2,
// tie-group end, 0).  Returns how many.
template <int F>
__device__ int tab_window(const TabArgs& a, int64_t bbase, const CandMap& cm, int64_t wb,
                          int64_t we, int64_t c, int4* sM, TabScalars& sc) {
    constexpr int WR = TAB_WIN / TAB_NT;  // members per thread
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t bal[WR];
    int4 mr[WR];
    int32_t m3[WR];  // rank 3 (four objectives)
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        const int64_t i = wb + (int64_t)(wave * WR + r) * 64 + lane;
        mr[r] = i < we ? a.cb.crec[bbase + cm.slot((int32_t)i)] : make_int4(0, 0, 0, 0);
        m3[r] = F == 3 && i < we ? a.cb.crec3[bbase + cm.slot((int32_t)i)] : 0;
    }
    int nw = 0;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        const int64_t i = wb + (int64_t)(wave * WR + r) * 64 + lane;
        bal[r] = __ballot(i < we && c < mr[r].x);
        nw += __popcll(bal[r]);
    }
    if (lane == 0) sc.wcnt[wave] = nw;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < PEEL_WAVES; ++w) {
        const int x = sc.wcnt[w];
        base += w < wave ? x : 0;
        total += x;
    }
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
        if ((bal[r] >> lane) & 1)  // (rank 1, rank 2, tie-group end, rank 3)
            sM[base + __popcll(bal[r] & below)] = make_int4(mr[r].z, mr[r].w, mr[r].y, m3[r]);
        base += __popcll(bal[r]);
    }
    __syncthreads();
    return total;
}

// chunk c, member slice y of launch j: front j's dominators subtracted from
// countq; the v whose count reaches zero go to buffer (j + 1) % 3
template <int F>
__device__ void tab_peel(const TabArgs& a, int32_t j, int64_t c, int64_t y, int64_t nslices,
                         char* smem, TabScalars& sc) {
    constexpr int PW = BD_CW / 64;
    PPROF_T(pt0);
    const int64_t U = a.U;
    const int64_t NG = (U + BD_CW - 1) / BD_CW;
    if (c >= NG) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t* gR = a.R + c * F * BD_CW;
    int32_t rr[F];
#pragma unroll
    for (int f = 0; f < F; ++f) rr[f] = gR[f * BD_CW + tid];
    const int buf = j % 3, nbuf = (j + 1) % 3;
    if (tid == 0) {
        sc.sf = a.stf[j];
        sc.go = 0;
        if (sc.sf.valid == a.epoch && !sc.sf.done) {
            tab_cand_list(a.cb, buf, sc);
            // emo.py:109: front j is peeled while pareto_sorted < N
            sc.go = sc.n > 0 && sc.sf.sorted + sc.pend < a.N && (int64_t)sc.sf.ustart + sc.n < U;
        }
    }
    const int64_t v = c * BD_CW + tid;
    // v's count, U index, individuals and record, all in flight with the state
    // read (no dependent second load: the record is needed only if v is
    // released, but a load after the count update would lengthen the release)
    int32_t pcnt = 0, pvu = 0, pgs = 0;
    int4 rq = make_int4(0, 0, 0, 0);
    int32_t rq3 = 0;
    if (v < U) {
        pcnt = a.countq[v];
        pvu = a.sigma[v];
        pgs = a.gsq[v];
        rq = a.qrec[v];
        if (F == 3) rq3 = a.qrec3[v];
    }
    if (!BD_OK(pvu, U, "tab sigma")) pvu = 0;
    __syncthreads();
    if (!sc.go) return;
    const int32_t n = sc.n;
    const int64_t nsl = peel_slices(n, c, NG, nslices, DM_PEEL_TAB_SLICE_MIN);
    if (y >= nsl) return;
    const CandMap cm = sc.cm.uniform();
    const int64_t bbase = a.cb.base(buf);
    auto& sR = *reinterpret_cast<int32_t(*)[F][BD_RP]>(smem + TabLds<F>::sR);
    auto& sB = *reinterpret_cast<uint16_t(*)[F][BD_BKN]>(smem + TabLds<F>::sB);
    int32_t* sdec = reinterpret_cast<int32_t*>(smem + TabLds<F>::dec);
    int4* sM = reinterpret_cast<int4*>(smem + TabLds<F>::sM);
#pragma unroll
    for (int f = 0; f < F; ++f) sR[f][bd_rpad(tid)] = rr[f];
    bd_load_buckets<F>(a.BK, c, sB);
    const int sh = bd_bucket_shift(U);
    const BdGlobalSets sets{reinterpret_cast<const uint4*>(a.P + c * F * BD_K * 16)};
    const TransposerX tr(lane);
    const int64_t slen = ((n + nsl - 1) / nsl + 63) & ~63ll;
    const int64_t j0s = y * slen;
    const int64_t Fm = std::min<int64_t>(n, j0s + slen);
    const int64_t v0 = c * BD_CW;
    int32_t dec[PW];
#pragma unroll
    for (int w = 0; w < PW; ++w) dec[w] = 0;
    PPROF_T(pt1);
    for (int64_t wb = j0s; wb < Fm; wb += TAB_WIN) {
        const int total = tab_window<F>(a, bbase, cm, wb, std::min<int64_t>(Fm, wb + TAB_WIN), c, sM, sc);
        for (int g0 = wave * 64; g0 < total; g0 += TAB_NT) {
            const int g = g0 + lane;
            const int4 mA = g < total ? sM[g] : make_int4(0, 0, 0, 0);
            const int32_t lim =
                g < total ? (int32_t)std::max<int64_t>(-1, std::min<int64_t>((int64_t)mA.z - v0, BD_CW)) : -1;
            int k[F];
            if (lim >= 0) {
                bd_row_k<F>(make_int4(mA.x, mA.y, mA.w, 0), sR, sB, sh, k);
#ifdef DM_BD_CHECK
                for (int f = 0; f < F; ++f)
                    if (!BD_OK(k[f], BD_K, "tab peel k")) k[f] = 0;
#endif
            } else {
#pragma unroll
                for (int f = 0; f < F; ++f) k[f] = 0;
            }
            uint4 raw[F][4], w[4];
            bd_row_fetch<F>(sets, k, raw);
            bd_row_merge<F, false>(raw, lim, -1, w);
            uint32_t lo[8], hi[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                lo[2 * i] = w[i].x;
                hi[2 * i] = w[i].y;
                lo[2 * i + 1] = w[i].z;
                hi[2 * i + 1] = w[i].w;
            }
            tr.run<8>(lo, hi);  // lane v: bit i <-> group member i dominates v
#pragma unroll
            for (int w2 = 0; w2 < 8; ++w2) dec[w2] += __popc(lo[w2]) + __popc(hi[w2]);
        }
        __syncthreads();  // the window's list is read out before the next one
    }
    PPROF_T(pt2);
    // release: the waves' counts reduced in LDS, applied to countq
#pragma unroll
    for (int w = 0; w < PW; ++w) sdec[wave * BD_CW + w * 64 + lane] = dec[w];
    __syncthreads();
    int32_t d = 0;
#pragma unroll
    for (int wv = 0; wv < PEEL_WAVES; ++wv) d += sdec[wv * BD_CW + tid];
    bool fresh = false;
    if (v < U && d > 0) {
        if (nsl == 1) {
            const int32_t left = pcnt - d;
            a.countq[v] = left;
            fresh = left == 0;
        } else {
            const int32_t old = __hip_atomic_fetch_add(a.countq + v, -d, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            fresh = old == d;
        }
    }
    const uint64_t fm = __ballot(fresh);
    int64_t gs = fresh ? pgs : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) gs += __shfl_xor(gs, o, 64);
    if (lane == 0) {
        sc.wcnt[wave] = __popcll(fm);
        sc.wgs[wave] = gs;
    }
    __syncthreads();
    if (tid == 0) {
        int32_t tot = 0;
        int64_t gtot = 0;
        for (int wv = 0; wv < PEEL_WAVES; ++wv) {
            const int32_t x = sc.wcnt[wv];
            sc.wcnt[wv] = tot;
            tot += x;
            gtot += sc.wgs[wv];
        }
        const int b = (int)(c & (CAND_BUCKETS - 1));
        sc.sbase = tot ? (int32_t)(b * a.cb.cap) + atomicAdd(a.cb.count(nbuf, b), tot) : 0;
        if (gtot) atomicAdd(a.cb.pending(nbuf, b), (unsigned long long)gtot);
    }
    __syncthreads();
    if (fresh) {
        const int32_t at = sc.sbase + sc.wcnt[wave] + __popcll(fm & ((1ull << lane) - 1));
        const int64_t slot = a.cb.base(nbuf) + at;
        if (BD_OK(at, CAND_BUCKETS * a.cb.cap, "tab slot") && BD_OK(pvu, U, "tab vu")) {
            a.cb.ckey[slot] = (uint64_t)(uint32_t)pvu;
            a.cb.cq[slot] = (int32_t)v;
            a.cb.crec[slot] = rq;
            if (F == 3) a.cb.crec3[slot] = rq3;
            a.rankU[pvu] = j + 1;
        }
    }
#ifdef DM_PEEL_PROF
    PPROF_T(pt3);
    if (tid == 0) {
        const unsigned int e = atomicAdd(&g_pprof_n, 1u);
        if (e < (1u << 17)) {
            unsigned long long* o = g_pprof + (size_t)e * 8;
            o[0] = c; o[1] = y; o[2] = n; o[3] = pt0; o[4] = pt1; o[5] = pt2; o[6] = pt3;
            o[7] = (unsigned long long)j << 8;
        }
    }
#endif
}

// Launch j: workgroups [0, TAB_NA) search and sort front j, the others peel
// it (chunk c, slice y; TAB_NA and gx are multiples of 8, so the slices of a
// chunk land on one XCD).
template <int F>
__global__ __launch_bounds__(TAB_NT, DM_PEEL_TAB_MINW) void peel_order_kernel(TabArgs a, int32_t j) {
    __shared__ __attribute__((aligned(16))) char smem[TabLds<F>::bytes];
    __shared__ TabScalars sc;
    if (blockIdx.x < TAB_NA) {
        if (j >= 1) tab_search<F>(a, j, blockIdx.x, smem, sc);
        return;
    }
    const int64_t t = (int64_t)blockIdx.x - TAB_NA;
    tab_peel<F>(a, j, t % a.gx, t / a.gx, PEEL_SLICES, smem, sc);
}

// front 0 (ulist[0, F0), U order): buffer 0's members, its records in mtab,
// and the state of launches 0 and 1 (workgroup 0, thread 0)
__global__ void tab_front0_kernel(TabArgs a, const int32_t* F0p, const int64_t* sorted0p) {
    const int64_t F0 = *F0p;
    DGRID_LOOP(i, F0) {
        const int32_t u = a.ulist[i];
        if (!BD_OK(u, a.U, "tab front 0")) continue;
        const int32_t q = a.pos[u];
        const int4 rec = a.qrec[q];
        a.cb.ckey[i] = (uint64_t)(uint32_t)u;
        a.cb.cq[i] = q;
        a.cb.crec[i] = rec;
        a.mtab[i] = rec;
        if (kBitsetM4 && a.mtab3) {
            const int32_t r3 = a.qrec3[q];
            a.cb.crec3[i] = r3;
            a.mtab3[i] = r3;
        }
    }
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const int64_t s0 = *sorted0p;
    for (int b = 0; b < CAND_BUCKETS; ++b) {
        *a.cb.count(0, b) = (int32_t)std::max<int64_t>(0, std::min<int64_t>(a.cb.cap, F0 - b * a.cb.cap));
        *a.cb.pending(0, b) = b == 0 ? (unsigned long long)s0 : 0ull;
    }
    FrontStep s{};
    s.valid = a.epoch;
    s.done = F0 == 0;
    a.stf[0] = s;
    FrontStep s1{};
    s1.sorted = s0;
    s1.ustart = (int32_t)F0;
    s1.Fprev = (int32_t)F0;
    s1.valid = a.epoch;
    s1.done = (s0 >= a.N || F0 >= a.U || F0 == 0) ? 1 : 0;
    a.stf[1] = s1;
    a.sum->nfronts = 0;
    a.sum->done = s1.done;
    a.sum->overflow = 0;
    a.sum->ncand = 0;
    a.sum->sorted = s0;
    a.sum->lastinds = s0;
    a.sum->maxinds = s0;
    a.fstarts[0] = 0;
    a.fstarts[1] = (int32_t)F0;
}
// A front past the sorting workgroup: its keys (bucket blockIdx.y after the
// earlier buckets) and slots into keys / vals for a radix sort ...
__global__ void tab_compact_kernel(TabArgs a, int buf, uint64_t* keys, int32_t* vals) {
    const int b = blockIdx.y;
    int32_t pre = 0;
    for (int k = 0; k < b; ++k) pre += *a.cb.count(buf, k);
    const int32_t cnt = *a.cb.count(buf, b);
    const int64_t src = a.cb.base(buf) + b * a.cb.cap;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt;
         i += (int64_t)gridDim.x * blockDim.x) {
        keys[pre + i] = a.cb.ckey[src + i];
        vals[pre + i] = (int32_t)(b * a.cb.cap + i);
    }
}
// ... and written out in that order as front j
__global__ __launch_bounds__(1024) void tab_presorted_kernel(TabArgs a, int32_t j, const uint64_t* keys,
                                                             const int32_t* vals) {
    __shared__ TabScalars sc;
    if (threadIdx.x == 0) {
        sc.sf = a.stf[j];
        tab_cand_list(a.cb, j % 3, sc);
    }
    __syncthreads();
    const int32_t n = sc.n;
    if (!BD_OK(sc.sf.ustart + (int64_t)n - 1, a.U, "tab presorted end")) return;
    const int64_t bbase = a.cb.base(j % 3);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        a.ulist[sc.sf.ustart + i] = (int32_t)(uint32_t)keys[i];
        a.mtab[sc.sf.ustart + i] = a.cb.crec[bbase + vals[i]];
        if (kBitsetM4 && a.mtab3) a.mtab3[sc.sf.ustart + i] = a.cb.crec3[bbase + vals[i]];
    }
    if (threadIdx.x == 0) tab_finish(a, j, n, sc.pend, sc.sf);
}

// ---------------------------------------------------------------------------
// host drivers (called from nsga2.hip)
// ---------------------------------------------------------------------------
// Workspace of the fast path: the buffers that live from the ranks to the
// last front, then the scratch shared by the rank sorts and the peel loop.
struct FastLayout {
    int64_t NB, NG, NQ, ngroups, Upad;  // NG: 512-v segments (tri_dom), NQ: TW-word lines (peel)
    size_t part, S, sigma, pos, nseg, toff, counter, mrow, mtab, qrec, crec, countq, cq, work, total;
    size_t mtab3, qrec3, crec3;  // rank 3 of the records (four objectives)
};
// elements of the rank pass's key / value buffers: the population (objective
// 0's q order) or the M-1 <= 3 objectives' unique values sorted as one batch
static int64_t ranks_elems(int64_t n, int64_t U) { return std::max<int64_t>(n, 3 * U); }
static size_t ranks_work_bytes(int64_t n, int64_t U) {
    const int64_t e = ranks_elems(n, U);
    return 2 * align_up((size_t)e * 8, 256) + 3 * align_up((size_t)e * 4, 256) +
           std::max(radix_sort_temp_bytes(n), radix_sort_batched_temp_bytes(3, U)) +
           scan_temp_bytes(e);
}
// the peel loop's part of the work region: the state page and the three
// candidate buffers' counter pages, their keys, the overflow sort's buffers
// (ktmp2 is the D peel's lastq) and the per-front state of the table peel
struct FrontsWork {
    size_t pages, ckey, ktmp, ktmp2, vals, vtmp, rtemp, stf, total;
};
static FrontsWork fronts_work(int64_t U) {
    FrontsWork W;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(std::max<size_t>(bytes, 1), 256);
        return o;
    };
    W.pages = take(CAND_PAGE * (1 + 3 * CAND_BUCKETS));
    W.ckey = take((size_t)3 * CAND_BUCKETS * cand_cap(U) * 8);
    W.ktmp = take((size_t)U * 8);
    W.ktmp2 = take((size_t)U * 8);
    W.vals = take((size_t)U * 4);
    W.vtmp = take((size_t)U * 4);
    W.rtemp = take(radix_sort_temp_bytes(U));
    W.stf = take((size_t)(U + 2) * sizeof(FrontStep));
    W.total = off;
    return W;
}
static size_t fronts_work_bytes(int64_t U) { return fronts_work(U).total; }
static FastLayout fast_layout(int64_t n, int64_t U) {
    FastLayout L;
    L.NB = (U + 63) / 64;
    L.NG = (L.NB + 7) / 8;
    L.NQ = (L.NB + TW - 1) / TW;
    L.ngroups = (L.NB + TD_WPW - 1) / TD_WPW;
    L.Upad = L.NB * 64;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(std::max<size_t>(bytes, 1), 256);
        return o;
    };
    // the compare kernel's int16 partials, or the bitset pass's scratch
    L.part = take(std::max((size_t)L.ngroups * L.Upad * 2, bitdom_bytes(U, 4)));
    L.S = take((size_t)L.Upad * 16);
    L.sigma = take((size_t)U * 4);
    L.pos = take((size_t)U * 4);
    L.nseg = take((size_t)(L.ngroups + 1) * 4);
    L.toff = take((size_t)(L.ngroups + 1) * 4);
    L.counter = take(4);
    L.mrow = take((size_t)U * 8);
    L.mtab = take((size_t)U * 16);
    L.qrec = take((size_t)U * 16);
    L.crec = take((size_t)3 * CAND_BUCKETS * cand_cap(U) * 16);
    L.countq = take((size_t)U * 4);
    L.cq = take((size_t)3 * CAND_BUCKETS * cand_cap(U) * 4);
    L.mtab3 = take((size_t)U * 4);
    L.qrec3 = take((size_t)U * 4);
    L.crec3 = take((size_t)3 * CAND_BUCKETS * cand_cap(U) * 4);
    L.work = take(std::max(ranks_work_bytes(n, U), fronts_work_bytes(U)));
    L.total = off;
    return L;
}
size_t fast_dom_bytes(int64_t n, int64_t U) { return fast_layout(n, U).total; }
int64_t fast_dom_words(int64_t U) {
    const int64_t NB = (U + 63) / 64, NQ = (NB + TW - 1) / TW;
    return NB * 64 * NQ * TW;
}

// Bitset tables (bitdom.hip) are the dominance pass for 2 and 3 objectives;
// four take the integer compare kernel + D peel.  (An m = 4 bitset pass was
// built and deleted in round 4: its first call in a fresh process faulted
// deterministically in the product build -- with the tables in LDS and with
// them read from global memory alike -- and never in the range-checked,
// workspace-poisoning DM_BD_CHECK build, which printed no out-of-range index;
// DESIGN.md §8.)  With the bitset pass the peel reads the tables, not a D
// matrix (peel_order_kernel), unless the DM_DOM_PEEL_D cross-check asks for the
// D peel.
// Four objectives on the bitset tables (rank 3 beside the member records) are
// built only into diagnostic builds (-DDM_BD_M4: tools_cpu/bdemu runs them on
// the host): on the GPU the path faulted in both of round 6's forms, with the
// count pass's tables in LDS and out of it, while running clean under ASan in
// the host emulation ("the m = 4 fault").
bool fast_bitset(const dm_ctx* ctx, int m) {
    return m >= 2 && (m <= 3 || (kBitsetM4 && m == 4 && ctx->dom_path != DM_DOM_PEEL_D)) &&
           ctx->dom_path != DM_DOM_COMPARE;
}
bool fast_table_peel(const dm_ctx* ctx, int m) {
    return fast_bitset(ctx, m) && ctx->dom_path != DM_DOM_PEEL_D;
}

// Ranks (objective 0 from the population's lexicographic order perm, whose
// group starts segin marks; uidx: U index of each group's representative),
// the dominance words D (fast_dom_words(U)) and count[U] (U order).
int fast_dom_build(dm_ctx* ctx, const double* wv, int m, int64_t n,
                   const int32_t* perm, const int32_t* segin, const int32_t* uidx,
                   const double* ufit, int64_t U, uint64_t* D, int32_t* count, char* ws) {
    hipStream_t s = ctx->stream;
    const int num_cus = ctx->num_cus;
    const FastLayout L = fast_layout(n, U);
    int4* S = (int4*)(ws + L.S);
    int32_t* sigma = (int32_t*)(ws + L.sigma);
    int32_t* pos = (int32_t*)(ws + L.pos);
    int32_t* nseg = (int32_t*)(ws + L.nseg);
    int32_t* toff = (int32_t*)(ws + L.toff);
    int32_t* counter = (int32_t*)(ws + L.counter);
    int16_t* part = (int16_t*)(ws + L.part);
    char* w = ws + L.work;
    const int64_t e = ranks_elems(n, U);
    uint64_t* keys = (uint64_t*)w;
    uint64_t* ktmp = (uint64_t*)(w + align_up((size_t)e * 8, 256));
    char* p = w + 2 * align_up((size_t)e * 8, 256);
    int32_t* vals = (int32_t*)p;
    int32_t* vtmp = (int32_t*)(p + align_up((size_t)e * 4, 256));
    int32_t* flag = (int32_t*)(p + 2 * align_up((size_t)e * 4, 256));
    void* rtemp = p + 3 * align_up((size_t)e * 4, 256);
    void* stemp = (char*)rtemp + std::max(radix_sort_temp_bytes(n), radix_sort_batched_temp_bytes(3, U));
    DM_HIP(hipMemsetAsync(S, 0, (size_t)L.Upad * 16, s));
    // objective 0 and the q order from the lexicographic order
    lex_flags_kernel<<<dg1(n), 256, 0, s>>>(wv, m, perm, segin, n, vals, vtmp);
    int rc;
    if ((rc = exclusive_scan_i32(s, vals, flag, n, nullptr, stemp))) return rc;
    if ((rc = exclusive_scan_i32(s, vtmp, (int32_t*)keys, n, nullptr, stemp))) return rc;
    lex_sigma_kernel<<<dg1(n), 256, 0, s>>>(perm, uidx, vals, flag, vtmp, (int32_t*)keys, n, m,
                                            sigma, pos, (int32_t*)S);
    // objectives 1..m-1: dense ranks by ONE batched sort of the unique values
    // (segment o - 1 = objective o), one flag pass, one scan, one scatter
    if (m > 1) {
        const int64_t nb = (int64_t)(m - 1) * U;
        rank_key_kernel<<<dg1(nb), 256, 0, s>>>(ufit, m, U, nb, keys, vals);
        if ((rc = radix_sort_pairs_batched(s, keys, vals, ktmp, vtmp, m - 1, U, 0, 64, rtemp)))
            return rc;
        rank_flag_kernel<<<dg1(nb), 256, 0, s>>>(keys, U, nb, flag);
        // the scan may not alias its input: the exclusive prefix goes to vtmp
        if ((rc = exclusive_scan_i32(s, flag, vtmp, nb, nullptr, stemp))) return rc;
        rank_scatter_kernel<<<dg1(nb), 256, 0, s>>>(vals, vtmp, flag, pos, U, nb, (int32_t*)S);
    }
    if (fast_bitset(ctx, m)) {  // bitset tables (bitdom.hip; DM_TIME_DOMINANCE: its count pass)
        group_reach_kernel<<<dg1(L.ngroups), 256, 0, s>>>(S, m, U, L.NG, L.ngroups, nseg);
        return bitdom_build(ctx, S, m, U, L.NQ, L.ngroups, nseg, sigma,
                            fast_table_peel(ctx, m) ? nullptr : D, count, (int32_t*)(ws + L.countq),
                            (char*)part);
    }
    tri_plan_kernel<<<1, 1024, 0, s>>>(S, m, U, L.NG, L.ngroups, nseg, toff, counter);
    const unsigned blocks = (unsigned)std::max(1, num_cus) * 8;
    timing_begin(ctx, DM_TIME_DOMINANCE);
    switch (m) {
        case 2: tri_dom_kernel<2><<<blocks, 256, 0, s>>>(S, U, L.NB, L.NQ, L.ngroups, nseg, toff, counter, D, part); break;
        case 3: tri_dom_kernel<3><<<blocks, 256, 0, s>>>(S, U, L.NB, L.NQ, L.ngroups, nseg, toff, counter, D, part); break;
        default: tri_dom_kernel<4><<<blocks, 256, 0, s>>>(S, U, L.NB, L.NQ, L.ngroups, nseg, toff, counter, D, part); break;
    }
    timing_end(ctx, DM_TIME_DOMINANCE);
    DM_LAUNCH_CHECK();
    // the rank sorts' keys / ktmp (2 n x 8 bytes) hold the TC_CHUNKS column sums
    static_assert(TC_CHUNKS * 4 <= 16, "tri_count scratch exceeds keys + ktmp");
    int32_t* ctmp = (int32_t*)keys;
    const int64_t cthreads = (U + 3) / 4;
    tri_count_part_kernel<<<dim3((unsigned)((cthreads + 255) / 256), TC_CHUNKS), 256, 0, s>>>(
        part, nseg, U, L.Upad, L.ngroups, ctmp);
    tri_count_sum_kernel<<<dg1(U), 256, 0, s>>>(ctmp, sigma, U, count, (int32_t*)(ws + L.countq));
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// Integer crowding keys (selNSGA2's fast path): rk[o * T + j] = the dense rank
// of objective o (weighted-value order, equal values equal ranks) of the
// emitted individual order[j], from the ranks the dominance pass already
// holds (S in q order).  assignCrowdingDist's per-objective sorts then run on
// (front, rank) keys of ~26 bits — 4 radix passes instead of 8 + 1.
__global__ void rank_keys_kernel(const int4* S, const int32_t* pos, const int32_t* ui,
                                 const int32_t* order, int64_t T, int m, int32_t* rk) {
    DGRID_LOOP(j, T) {
        const int4 r = S[pos[ui[order[j]]]];
        for (int o = 0; o < m; ++o) rk[o * T + j] = icomp(r, o == 0 ? m - 1 : o - 1);
    }
}
int fast_rank_keys(dm_ctx* ctx, const char* ws, int64_t n, int64_t U, int m, const int32_t* ui,
                   const int32_t* order, int64_t T, int32_t* rk) {
    const FastLayout L = fast_layout(n, U);
    if (T <= 0) return DM_OK;
    rank_keys_kernel<<<dg1(T), 256, 0, ctx->stream>>>((const int4*)(ws + L.S),
                                                      (const int32_t*)(ws + L.pos), ui, order, T,
                                                      m, rk);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

// fast_fronts for the bitset tables: one launch per front (peel_order_kernel:
// the peel of front j beside the search and sort of front j), the status
// read after each batch.
static int fast_fronts_tab(dm_ctx* ctx, int m, int64_t n, int64_t U, const int32_t* F0,
                           const int64_t* sorted0, int64_t N, const int32_t* gsize, int32_t* ulist,
                           int32_t* rankU, int32_t* fstarts, char* ws, std::vector<int32_t>& ufront,
                           int64_t* sorted, int64_t* last_inds, int64_t* max_inds) {
    hipStream_t s = ctx->stream;
    const FastLayout L = fast_layout(n, U);
    const FrontsWork W = fronts_work(U);
    char* p = ws + L.work;
    const BitdomLayout TL = bitdom_layout(U, m);
    const char* tws = ws + L.part;
    DM_CHECK_ARG(U < (1ll << 31) - 1, "more than 2^31 unique fitnesses");
    TabArgs a;
    a.P = (const uint32_t*)(tws + TL.P);
    a.R = (const int32_t*)(tws + TL.R);
    a.BK = (const uint16_t*)(tws + TL.BK);
    a.qrec = (const int4*)(ws + L.qrec);
    a.gsize = gsize;
    a.sigma = (const int32_t*)(ws + L.sigma);
    a.pos = (const int32_t*)(ws + L.pos);
    a.countq = (int32_t*)(ws + L.countq);
    a.rankU = rankU;
    a.ulist = ulist;
    a.fstarts = fstarts;
    a.mtab = (int4*)(ws + L.mtab);
    a.gslot = (int32_t*)(p + W.vals);
    a.gtmp = (int32_t*)(p + W.vtmp);
    a.gkey = (uint64_t*)(p + W.ktmp2);
    a.stf = (FrontStep*)(p + W.stf);
    a.sum = (FrontSum*)(p + W.pages);
    a.cb.pages = p + W.pages + CAND_PAGE;
    a.cb.ckey = (uint64_t*)(p + W.ckey);
    a.cb.cq = (int32_t*)(ws + L.cq);
    a.cb.crec = (int4*)(ws + L.crec);
    // four objectives: rank 3 travels beside every record
    a.qrec3 = m == 4 ? (const int32_t*)(ws + L.qrec3) : nullptr;
    a.mtab3 = m == 4 ? (int32_t*)(ws + L.mtab3) : nullptr;
    a.cb.crec3 = m == 4 ? (int32_t*)(ws + L.crec3) : nullptr;
    a.cb.cap = cand_cap(U);
    a.U = U;
    a.N = N;
    a.gx = (TL.NG + 7) & ~7ll;
    static std::atomic<uint32_t> epochs{0};
    do {
        a.epoch = ++epochs;
    } while (a.epoch == 0);
    DM_HIP(hipMemsetAsync(p + W.pages, 0, CAND_PAGE * (1 + 3 * CAND_BUCKETS), s));
    // gsq: gsize[sigma[q]] in the D peel's member-row area (unused by this peel)
    int32_t* gsq = (int32_t*)(ws + L.mrow);
    a.gsq = gsq;
    member_rec_kernel<<<dg1(U), 256, 0, s>>>((const int4*)(ws + L.S), (const int2*)(tws + TL.span),
                                             (const int32_t*)(ws + L.nseg), U, (int4*)(ws + L.qrec),
                                             nullptr, a.sigma, gsize, gsq,
                                             m == 4 ? (int32_t*)(ws + L.qrec3) : nullptr);
    tab_front0_kernel<<<dg1(U), 256, 0, s>>>(a, F0, sorted0);
    char* hbuf = (char*)pinned(ctx, 2048);
    if (!hbuf) return DM_ERR_NOMEM;
    FrontSum* hsum = (FrontSum*)hbuf;
    int32_t* hfs = (int32_t*)(hbuf + 256);
    const int64_t npre = std::min<int64_t>((2048 - 256) / 4, U + 2);
    // as fast_fronts: the first batch from the previous call's front count
    // and its trend; launch j orders front j, so the fronts up to J take J+1
    constexpr int PEEL_BATCH_MAX = 96;
    const bool hinted = 4 * U >= 3 * ctx->peel_hint_U && 3 * U <= 4 * ctx->peel_hint_U &&
                        N == ctx->peel_hint_N;
    const int hint = hinted ? ctx->peel_hint : 4;
    const int trend = hinted ? std::max(0, std::min(ctx->peel_trend, 4)) : 0;
    int batch = std::max(2, std::min(hint + 1 + trend, PEEL_BATCH_MAX));
    const unsigned grid = (unsigned)(TAB_NA + a.gx * PEEL_SLICES);
    int32_t j = 0;  // the next launch's front
    for (;;) {
        timing_begin(ctx, DM_TIME_PEEL_CHAIN);
        for (int b = 0; b < batch; ++b) {
            timing_begin(ctx, DM_TIME_PEEL);
            if (m == 2)
                peel_order_kernel<1><<<grid, TAB_NT, 0, s>>>(a, j + b);
            else if (m == 3)
                peel_order_kernel<2><<<grid, TAB_NT, 0, s>>>(a, j + b);
            else
                peel_order_kernel<3><<<grid, TAB_NT, 0, s>>>(a, j + b);
            timing_end(ctx, DM_TIME_PEEL);
        }
        timing_end(ctx, DM_TIME_PEEL_CHAIN);
        DM_LAUNCH_CHECK();
        DM_HIP(hipMemcpyAsync(hsum, a.sum, sizeof(FrontSum), hipMemcpyDeviceToHost, s));
        DM_HIP(hipMemcpyAsync(hfs, fstarts, (size_t)npre * 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        if (hsum->done) break;
        if (hsum->overflow) {
            // front js has more members than the sorting workgroup holds:
            // the radix sort orders their (final) keys
            const int32_t js = hsum->nfronts + 1, nc = hsum->ncand;
            uint64_t* ktmp = (uint64_t*)(p + W.ktmp);
            uint64_t* ktmp2 = (uint64_t*)(p + W.ktmp2);
            int32_t* vals = (int32_t*)(p + W.vals);
            int32_t* vtmp = (int32_t*)(p + W.vtmp);
            tab_compact_kernel<<<dim3((unsigned)((a.cb.cap + 255) / 256), CAND_BUCKETS), 256, 0, s>>>(
                a, js % 3, ktmp, vals);
            int rc = radix_sort_pairs(s, ktmp, vals, ktmp2, vtmp, nc, 0, 64, p + W.rtemp);
            if (rc) return rc;
            tab_presorted_kernel<<<1, 1024, 0, s>>>(a, js, ktmp, vals);
            DM_LAUNCH_CHECK();
            j = js + 1;
        } else {
            j += batch;
        }
        // the next batch from what is left (as fast_fronts)
        const double mean = (double)hsum->sorted / (double)(hsum->nfronts + 1);
        const double per = std::max(mean, (double)hsum->lastinds);
        const double left = (double)(N - hsum->sorted);
        int need = per > 0 ? (int)std::ceil(left / per) : 32;
        if (hint > hsum->nfronts) need = std::min(need, hint - hsum->nfronts + 1);
        batch = std::max(2, std::min(need + 2, PEEL_BATCH_MAX));
    }
    const int32_t nf = hsum->nfronts + 1;
    ctx->peel_trend = hinted ? hsum->nfronts - ctx->peel_hint : 0;
    ctx->peel_hint = hsum->nfronts;
    ctx->peel_hint_U = U;
    ctx->peel_hint_N = N;
    ufront.resize(nf + 1);
    if (nf + 1 <= npre) {
        std::copy(hfs, hfs + nf + 1, ufront.begin());
    } else {
        DM_HIP(hipMemcpyAsync(ufront.data(), fstarts, (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
    }
    *sorted = hsum->sorted;
    *last_inds = hsum->lastinds;
    if (max_inds) *max_inds = hsum->maxinds;
    return DM_OK;
}

// Fronts 1.. after front 0 (ulist[0, *F0), rankU set): peel on the device,
// checking the status every few fronts.  F0 and sorted0 (front 0's unique
// fitnesses and individuals) stay on the device.  Fills ufront (front starts
// in ulist, host; fstarts on the device) and *sorted (individuals).  ws: the
// fast_dom_build workspace.
int fast_fronts(dm_ctx* ctx, const uint64_t* D, int m, int64_t n, int64_t U, const int32_t* F0,
                const int64_t* sorted0,
                int64_t N, const int32_t* gsize, int32_t* ulist, int32_t* rankU, int32_t* count,
                int32_t* fstarts, char* ws, std::vector<int32_t>& ufront, int64_t* sorted,
                int64_t* last_inds, int64_t* max_inds) {
    hipStream_t s = ctx->stream;
    const FastLayout L = fast_layout(n, U);
    const int32_t* sigma = (const int32_t*)(ws + L.sigma);
    if (max_inds) *max_inds = INT64_MAX;  // unknown unless the table peel reports it
    const int32_t* pos = (const int32_t*)(ws + L.pos);
    const int32_t* nseg = (const int32_t*)(ws + L.nseg);
    int2* mrow = (int2*)(ws + L.mrow);
    int32_t* countq = (int32_t*)(ws + L.countq);
    int32_t* cq = (int32_t*)(ws + L.cq);
    if (fast_table_peel(ctx, m))
        return fast_fronts_tab(ctx, m, n, U, F0, sorted0, N, gsize, ulist, rankU, fstarts, ws,
                               ufront, sorted, last_inds, max_inds);
    char* p = ws + L.work;
    const FrontsWork W = fronts_work(U);
    FrontState* st = (FrontState*)(p + W.pages);  // + the eight candidate-bucket pages
    uint64_t* ckey = (uint64_t*)(p + W.ckey);
    uint64_t* ktmp = (uint64_t*)(p + W.ktmp);
    int32_t* vals = (int32_t*)(p + W.vals);
    int32_t* vtmp = (int32_t*)(p + W.vtmp);
    // sliced peels: per v the max (front + 1, last releasing position)
    unsigned long long* lastq = (unsigned long long*)(p + W.ktmp2);
    void* rtemp = p + W.rtemp;
    front_init_kernel<<<CAND_BUCKETS + 1, 256, 0, s>>>(st, F0, sorted0, N, U, fstarts);
    DM_HIP(hipMemsetAsync(lastq, 0, (size_t)U * 8, s));
    // the D peel reads member rows (mrow), which its ordering writes
    member_rows_kernel<<<dg1(U), 256, 0, s>>>(ulist, F0, pos, nseg, mrow);
    // status word and the first front starts come back together: when the
    // peel is done they are usually all that is needed (one round trip)
    char* hbuf = (char*)pinned(ctx, 2048);
    if (!hbuf) return DM_ERR_NOMEM;
    FrontState* hst = (FrontState*)hbuf;
    int32_t* hfs = (int32_t*)(hbuf + 256);
    const int64_t npre = std::min<int64_t>((2048 - 256) / 4, U + 2);
    // launch pairs (peel, order) per front: first status check after as many
    // fronts as the previous call needed
    // (the previous call's front count + 1, so that a selection like the last
    // one needs a single status read; up to PEEL_BATCH_MAX launch pairs)
    constexpr int PEEL_BATCH_MAX = 96;
    // the hint counts only for a problem of about the same size
    const bool hinted = 4 * U >= 3 * ctx->peel_hint_U && 3 * U <= 4 * ctx->peel_hint_U &&
                        N == ctx->peel_hint_N;
    const int hint = hinted ? ctx->peel_hint : 4;
    // while a run's front count still grows (its first generations: a few
    // more fronts per call) the first batch adds the last change
    const int trend = hinted ? std::max(0, std::min(ctx->peel_trend, 4)) : 0;
    int batch = std::max(2, std::min(hint + 1 + trend, PEEL_BATCH_MAX));
    for (;;) {
        timing_begin(ctx, DM_TIME_PEEL_CHAIN);
        for (int b = 0; b < batch; ++b) {
            timing_begin(ctx, DM_TIME_PEEL);
            peel_owned_kernel<<<dim3((unsigned)L.NQ, PEEL_SLICES), PEEL_WAVES * 64, 0, s>>>(
                D, L.NQ, mrow, gsize, sigma, st, countq, lastq, ckey, cq, rankU);
            timing_end(ctx, DM_TIME_PEEL);
            front_order_kernel<<<1, 1024, 0, s>>>(st, ckey, cq, ulist, mrow, pos, nseg, fstarts, 0);
        }
        timing_end(ctx, DM_TIME_PEEL_CHAIN);
        DM_LAUNCH_CHECK();
        DM_HIP(hipMemcpyAsync(hst, st, sizeof(FrontState), hipMemcpyDeviceToHost, s));
        DM_HIP(hipMemcpyAsync(hfs, fstarts, (size_t)npre * 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
        if (hst->done) break;
        if (hst->overflow) {
            // a front too large for the LDS sort: the radix sort orders its keys
            const int32_t nc = hst->ncand;
            // the buckets' candidates gathered into one list (ktmp), sorted,
            // and back into ckey[0, nc) for the presorted ordering
            cand_compact_kernel<<<dim3((unsigned)((cand_cap(U) + 255) / 256), CAND_BUCKETS), 256, 0,
                                  s>>>(st, ckey, cand_cap(U), ktmp);
            DM_HIP(hipMemsetAsync(vals, 0, (size_t)nc * 4, s));
            int rc = radix_sort_pairs(s, ktmp, vals, ckey, vtmp, nc, 0, 64, rtemp);
            if (rc) return rc;
            DM_HIP(hipMemcpyAsync(ckey, ktmp, (size_t)nc * 8, hipMemcpyDeviceToDevice, s));
            front_order_kernel<<<1, 1024, 0, s>>>(st, ckey, cq, ulist, mrow, pos, nseg, fstarts, 1);
            DM_LAUNCH_CHECK();
        }
        // next batch from what is left: fronts grow along the peel, so the
        // remaining individuals over the last front's (or the mean front's,
        // if larger) bound the fronts still needed (each launch past `done`
        // returns at once but costs ~10 us; each extra status check a round
        // trip; the bench's growing generations left 4-12 launch pairs idle
        // per selection with the mean alone and two spare pairs)
        const double mean = (double)hst->sorted / (double)(hst->nfronts + 1);
        const double per = std::max(mean, (double)hst->lastinds);
        const double left = (double)(hst->N - hst->sorted);
        int need = per > 0 ? (int)std::ceil(left / per) : 32;
        // the previous call's front count, when it had more fronts than done
        // so far, is the better estimate
        if (hint > hst->nfronts) need = std::min(need, hint - hst->nfronts + 1);
        batch = std::max(2, std::min(need + 1, PEEL_BATCH_MAX));
    }
    const int32_t nf = hst->nfronts + 1;  // front 0 plus the peeled ones
    ctx->peel_trend = hinted ? hst->nfronts - ctx->peel_hint : 0;
    ctx->peel_hint = hst->nfronts;
    ctx->peel_hint_U = U;
    ctx->peel_hint_N = N;
    ufront.resize(nf + 1);
    if (nf + 1 <= npre) {
        std::copy(hfs, hfs + nf + 1, ufront.begin());
    } else {
        DM_HIP(hipMemcpyAsync(ufront.data(), fstarts, (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, s));
        DM_HIP(hipStreamSynchronize(s));
    }
    *sorted = hst->sorted;
    *last_inds = hst->lastinds;
    return DM_OK;
}

}  // namespace dm

#ifdef DM_PEEL_PROF
// diagnostic builds: copy out and reset the table-peel phase clocks
extern "C" int dm_debug_peel_prof(unsigned long long* host, int64_t cap) {
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(dm::g_pprof_n), 4) != hipSuccess) return -1;
    n = std::min<unsigned int>(n, 1u << 17);
    const int64_t k = std::min<int64_t>(n, cap);
    if (k > 0 && hipMemcpyFromSymbol(host, HIP_SYMBOL(dm::g_pprof), (size_t)k * 64) != hipSuccess) return -1;
    const unsigned int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(dm::g_pprof_n), &z, 4) != hipSuccess) return -1;
    return (int)k;
}
#endif
