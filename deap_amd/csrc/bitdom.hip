// bitdom.hip — the dominance words D and dominator counts of the fast
// sortNondominated path (deap/tools/emo.py:53-117) from bitset tables.
//
// Over integer ranks (dominance.hip §1) Fitness.dominates (base.py:209-224)
// factorises per objective:  u dominates v  <=>  r_i(u) >= r_i(v) for every
// objective i and u != v (distinct unique fitnesses have distinct rank
// vectors, so "not all equal" is u != v).  Over a chunk C of 512 consecutive
// v of the q order, the set {v in C : r_i(v) <= t} is, for any threshold t,
// a prefix of C sorted by r_i: one of only 513 sets.  bd_table_kernel stores
// them all per chunk and objective i >= 1 (P_i[C][k], k = 0..512, 64 bytes
// each, built by wave ballots), beside C's sorted ranks R_i[C].  Row u of D
// over C is then
//     prefix0(u) & P_1[C][k_1] & .. & P_{m-1}[C][k_{m-1}]  without bit u,
//     k_i = #{v in C : r_i(v) <= r_i(u)}  (a binary search of R_i[C] in LDS),
// and prefix0(u) = every v up to the last q of u's objective-0 tie group (q
// order ascends in r_0).  16 dword ANDs per objective decide 512 pairs, where
// the compare kernel (dominance.hip tri_dom_kernel) spends a VALU compare per
// objective and 64 pairs; what is left is storing D (one 64-byte half line
// per row and chunk).  The dominator counts use the same tables transposed:
//     #{u in C : u dominates v} = popcount(suffix0(v) & ~(P_1[lb_1] | ..)) - [v in C],
//     lb_i = #{u in C : r_i(u) < r_i(v)},
// int16 partials per (chunk, v), summed per v over the chunks that reach it.
//
// Output = tri_dom_kernel's + tri_count's: the same D words for every row and
// every 512-v half its A-group reaches (nseg), the same count / countq, so the
// peel is unchanged.  DM_DOM_TRI=1 selects the compare kernel (A/B, tests).
#include "bitdom.hpp"

namespace dm {

size_t bitdom_bytes(int64_t U, int m) { return bitdom_layout(U, m).total; }

// first[r] / last[r]: the first / last q whose objective-0 rank is r (r_0 is
// a dense rank and ascends with q).
__global__ void bd_ties_kernel(const int4* __restrict__ S, int m, int64_t U, int32_t* first,
                               int32_t* last) {
    DGRID_LOOP(q, U) {
        const int32_t r = icomp(S[q], m - 1);
        if (!BD_OK(r, U, "ties r")) continue;
        if (q == 0 || icomp(S[q - 1], m - 1) != r) first[r] = (int32_t)q;
        if (q == U - 1 || icomp(S[q + 1], m - 1) != r) last[r] = (int32_t)q;
    }
}

// span[q] = (first, last) q of q's objective-0 tie group: prefix0(u) is every
// v <= span[u].y, suffix0(v) every u >= span[v].x.
__global__ void bd_span_kernel(const int4* __restrict__ S, int m, int64_t U,
                               const int32_t* __restrict__ first, const int32_t* __restrict__ last,
                               int2* __restrict__ span) {
    DGRID_LOOP(q, U) {
        const int32_t r = icomp(S[q], m - 1);
        if (!BD_OK(r, U, "span r")) continue;
        span[q] = make_int2(first[r], last[r]);
    }
}

// Tables of chunk c (blockIdx.x) for objective f + 1 (blockIdx.y; S component
// f):  R[(cF + f) 512 + j] = the j-th smallest rank of C (positions past U:
// INT32_MAX, last);  P[((cF + f) 513 + k) 16 + d] = dword d of the set of
// positions whose local rank (rank, position) is below k — for k = 0..512 by
// one ballot per 64 positions and k.
__global__ __launch_bounds__(BD_THREADS) void bd_table_kernel(const int4* __restrict__ S,
                                                              int64_t U, int F,
                                                              uint32_t* __restrict__ P,
                                                              int32_t* __restrict__ R,
                                                              uint16_t* __restrict__ BK) {
    __shared__ uint64_t sk[BD_CW];  // the bitonic sort's long strides
    __shared__ int32_t lrs[BD_CW];
    __shared__ int32_t sorted[BD_CW];
    const int64_t c = blockIdx.x;
    const int f = blockIdx.y;
    const int t = threadIdx.x;
    const int64_t v = c * BD_CW + t;
    const int32_t rv = v < U ? icomp(S[v], f) : INT32_MAX;  // ranks >= 0
    // local rank of v = its place in the chunk sorted by (rank, position): a
    // bitonic sort of (rank << 32 | position) (the direct count compared
    // every pair of the chunk, 512 LDS reads and compares per thread)
    uint64_t key[1] = {((uint64_t)(uint32_t)rv << 32) | (uint32_t)t};
    block_bitonic<BD_THREADS, 1>(key, sk);
    lrs[(uint32_t)key[0]] = t;
    sorted[t] = (int32_t)(key[0] >> 32);
    const int64_t cf = c * F + f;
    R[cf * BD_CW + t] = sorted[t];
    __syncthreads();
    const int32_t lr = lrs[t];
    // bucket starts: BK[b] = #{sorted ranks < b << sh}
    const int sh = bd_bucket_shift(U);
    for (int b = t; b < BD_BKN; b += BD_THREADS) {
        const int64_t th = (int64_t)b << sh;
        int lo = 0, hi = BD_CW;  // first j with sorted[j] >= th
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((int64_t)sorted[mid] < th) lo = mid + 1;
            else hi = mid;
        }
        BK[cf * BD_BKN + b] = (uint16_t)lo;
    }
    // the sets are built in LDS (wave w owns word w of every set) and then
    // stored as whole 64-B sets by consecutive threads: 16-B stores, each
    // wave instruction one contiguous KiB (the direct form wrote 8 B per lane
    // into 64 different lines per instruction)
    __shared__ uint64_t sP[BD_K][BD_CW / 64];
    const int wave = t >> 6, lane = t & 63;
    for (int k0 = 0; k0 < BD_K; k0 += 64) {
        uint64_t mine = 0;
#pragma unroll 16
        for (int i = 0; i < 64; ++i) {
            const uint64_t b = __ballot(lr < k0 + i);
            mine = lane == i ? b : mine;
        }
        const int k = k0 + lane;
        if (k < BD_K) sP[k][wave] = mine;
    }
    __syncthreads();
    uint4* Pc = reinterpret_cast<uint4*>(P + cf * BD_K * 16);
    const uint4* src = reinterpret_cast<const uint4*>(&sP[0][0]);
    for (int i = t; i < BD_K * 4; i += BD_THREADS) Pc[i] = src[i];
}

// Per chunk c: rowfirst[c] = first row of the A-groups whose reach includes c
// (nseg[g] > c; nseg is nondecreasing), reach[c] = 1 + the last q whose r_0
// is at most chunk c's largest (the v a row of c can dominate); toffD /
// toffC: first task of c in the row / count pass (BD_RT rows or v per task).
__global__ __launch_bounds__(1024) void bd_plan_kernel(const int4* __restrict__ S, int m,
                                                       const int32_t* __restrict__ last,
                                                       const int32_t* __restrict__ nseg, int64_t U,
                                                       int64_t NG, int64_t ngroups,
                                                       int32_t* rowfirst, int32_t* reach,
                                                       int32_t* toffD, int32_t* toffC) {
    __shared__ int32_t shD[1024 / 64], shC[1024 / 64];  // wave totals of the scans
    __shared__ int32_t carryD, carryC;
    const int tid = threadIdx.x;
    if (tid == 0) carryD = carryC = 0;
    __syncthreads();
    for (int64_t base = 0; base < NG; base += 1024) {
        const int64_t c = base + tid;
        int32_t nD = 0, nC = 0;
        if (c < NG) {
            if (!BD_OK(ngroups - 1, U, "plan ngroups")) continue;
            int64_t lo = 0, hi = ngroups;  // first g with nseg[g] > c
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (nseg[mid] > c) hi = mid;
                else lo = mid + 1;
            }
            const int64_t r0 = lo * TD_WPW * 64;
            rowfirst[c] = (int32_t)r0;
            nD = r0 < U ? (int32_t)((U - r0 + BD_RT - 1) / BD_RT) : 0;
            const int64_t qe = std::min<int64_t>(c * BD_CW + BD_CW - 1, U - 1);
            const int32_t rq = icomp(S[qe], m - 1);
            const int32_t re = BD_OK(rq, U, "plan last") ? last[rq] + 1 : 0;
            reach[c] = re;
            nC = (re + BD_RT - 1) / BD_RT;
        }
        const int32_t iD = block_incl_scan<1024, false>(nD, shD);
        const int32_t iC = block_incl_scan<1024, false>(nC, shC);
        const int32_t cD = carryD, cC = carryC;
        if (c < NG) {
            toffD[c] = cD + iD - nD;
            toffC[c] = cC + iC - nC;
        }
        __syncthreads();
        if (tid == 1023) {
            carryD = cD + iD;
            carryC = cC + iC;
        }
        __syncthreads();
    }
    if (tid == 0) {
        toffD[NG] = carryD;
        toffC[NG] = carryC;
    }
}

// Row pass: task = (chunk c, BD_RT rows from rowfirst[c]); lane = row u, a
// wave takes 64 rows at a time.  The 64-byte row of a table set is read as
// four 16-byte pieces in a lane-rotated order (piece (i + lane) & 3 at step
// i): random sets start on only 4 of the 16 bank quads, the rotation spreads
// a lane group's reads over all 16.  The next row's ranks and span are loaded
// before this row's D stores are issued: loads and stores share the in-order
// vmcnt counter, so a load issued after the stores would wait for them.
template <int M>
__global__ __launch_bounds__(BD_THREADS) void bd_rows_kernel(
    const int4* __restrict__ S, const int2* __restrict__ span, int64_t U, int64_t NQ, int64_t NG,
    const int32_t* __restrict__ rowfirst, const int32_t* __restrict__ toffD,
    const uint32_t* __restrict__ P, const int32_t* __restrict__ R, const uint16_t* __restrict__ BK,
    uint64_t* __restrict__ D) {
    constexpr int F = M - 1;
    static_assert(F <= 3, "the prefix-set tables of 2-4 objectives fit in LDS (110,988 B at F = 3)");
    __shared__ uint4 sP[F][BD_K * 4];
    __shared__ int32_t sR[F][BD_RP];
    __shared__ uint16_t sB[F][BD_BKN];
    const int sh = bd_bucket_shift(U);
    const int32_t t = blockIdx.x;
    if (t >= toffD[NG]) return;
    const int64_t c = bd_task_chunk<F>(toffD, NG, t);
    const int64_t row0 = rowfirst[c] + (int64_t)(t - toffD[c]) * BD_RT;
    const int64_t row1 = std::min<int64_t>(U, row0 + BD_RT);
    int64_t u = row0 + threadIdx.x;
    int4 su = u < row1 ? S[u] : make_int4(0, 0, 0, 0);
    int2 sp = u < row1 ? span[u] : make_int2(0, 0);
    bd_load_tables<F>(P, R, BK, c, sP, sR, sB);
    const int rot = threadIdx.x & 3;
    const int64_t v0 = c * BD_CW;
    for (; u < row1; u += BD_THREADS) {
        const int4 cu = su;
        const int64_t lim = (int64_t)sp.y - v0;  // prefix0(u): positions <= lim
        const int64_t un = u + BD_THREADS;
        if (un < row1) {
            su = S[un];
            sp = span[un];
        }
        uint4 w[4];
        bd_row_words<M>(cu, (int32_t)std::min<int64_t>(lim, BD_CW), (int32_t)std::max<int64_t>(-1, std::min<int64_t>(u - v0, BD_CW)), BdLdsSets<F>{sP}, sR, sB, sh, rot, w);
        if (!BD_OK(tword(u, 8 * c, NQ) + 7, (U + 63) / 64 * 64 * NQ * TW, "rows D")) continue;
        uint4* dst = reinterpret_cast<uint4*>(D + tword(u, 8 * c, NQ));
#if DM_BD_ABLATE & 1  // profiling only: no D stores
        if (w[0].x == 0x12345u && w[1].y == 0x777u) dst[0] = w[2];
        continue;
#elif DM_BD_ABLATE & 2  // profiling only (wrong D): whole 128-B lines, both halves
        uint4* line = reinterpret_cast<uint4*>(D + tword(u, 16 * (c >> 1), NQ));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            line[(i + rot) & 3] = w[i];
            line[4 + ((i + rot) & 3)] = w[i];
        }
        continue;
#endif
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[(i + rot) & 3] = w[i];
    }
}

// Count pass: task = (chunk c of dominators u, BD_RT v below reach[c]); lane
// = v: the u of C that dominate v, as an int16 partial part[c][v].  The next
// v's ranks and span are loaded ahead (as in the row pass).
template <int M>
__global__ __launch_bounds__(BD_THREADS) void bd_count_kernel(
    const int4* __restrict__ S, const int2* __restrict__ span, int64_t U, int64_t Upad, int64_t NG,
    const int32_t* __restrict__ reach, const int32_t* __restrict__ toffC,
    const uint32_t* __restrict__ P, const int32_t* __restrict__ R, const uint16_t* __restrict__ BK,
    int16_t* __restrict__ part) {
    constexpr int F = M - 1;
    static_assert(F <= 3, "2 to 4 objectives");
    // objectives 1-2 in LDS (73,992 B, as for three objectives); a fourth
    // objective's tables are read from the global table, whose chunk slice
    // (35 KB) stays in the L2: the 110,988-B LDS form of four objectives
    // faulted on the GPU twice while running clean in the host emulation
    // ("the m = 4 fault")
    constexpr int FL = F < 3 ? F : 2;
    __shared__ uint4 sP[FL][BD_K * 4];
    __shared__ int32_t sR[FL][BD_RP];
    __shared__ uint16_t sB[FL][BD_BKN];
    const int sh = bd_bucket_shift(U);
    const int32_t t = blockIdx.x;
    if (t >= toffC[NG]) return;
    const int64_t c = bd_task_chunk<F>(toffC, NG, t);
    const int64_t vb = (int64_t)(t - toffC[c]) * BD_RT;
    const int64_t ve = std::min<int64_t>(reach[c], vb + BD_RT);
    if (!BD_OK(c, NG, "count c") || !BD_OK(reach[c] - 1, U, "count reach")) return;
    int64_t v = vb + threadIdx.x;
    int4 sv = v < ve ? S[v] : make_int4(0, 0, 0, 0);
    int32_t sf = v < ve ? span[v].x : 0;
    bd_load_tables<FL, F>(P, R, BK, c, sP, sR, sB);
    const uint4* gP3 = reinterpret_cast<const uint4*>(P + (c * F + 2) * BD_K * 16);  // F = 3 only
    const int32_t* gR3 = R + (c * F + 2) * BD_CW;
    const uint16_t* gB3 = BK + (c * F + 2) * BD_BKN;
    const int rot = threadIdx.x & 3;
    const int64_t v0 = c * BD_CW;
    const int32_t nvalid = (int32_t)std::min<int64_t>(U - v0, BD_CW);  // positions < nvalid are real rows
    for (; v < ve; v += BD_THREADS) {
        const int4 cv = sv;
        const int32_t lo = (int32_t)std::max<int64_t>(-1, (int64_t)sf - v0);  // suffix0(v): positions >= lo
        const int64_t vn = v + BD_THREADS;
        if (vn < ve) {
            sv = S[vn];
            sf = span[vn].x;
        }
        int k[F];
#pragma unroll
        for (int f = 0; f < FL; ++f) k[f] = bd_count_below<false>(sR[f], sB[f], sh, icomp(cv, f));
        if constexpr (F == 3) {  // #{j : R_3[j] < r_3(v)} from the global sorted ranks
            const int32_t x = icomp(cv, 2);
            const int b = x >> sh;
            int j = gB3[b];
            const int e = gB3[b + 1];
            while (j < e && gR3[j] < x) ++j;
            k[2] = j;
        }
        uint32_t cnt = 0;
        const bool edge = lo > 0 || nvalid < BD_CW;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = (i + rot) & 3;
            uint4 o = sP[0][k[0] * 4 + j];
#pragma unroll
            for (int f = 1; f < F; ++f) {
                const uint4 y = f < FL ? sP[f < FL ? f : 0][k[f] * 4 + j] : gP3[k[f] * 4 + j];
                o.x |= y.x;
                o.y |= y.y;
                o.z |= y.z;
                o.w |= y.w;
            }
            uint32_t x0 = ~o.x, x1 = ~o.y, x2 = ~o.z, x3 = ~o.w;
            if (edge) {
                const int d0 = 4 * j;
                x0 &= from_mask(lo, d0) & upto_mask(nvalid - 1, d0);
                x1 &= from_mask(lo, d0 + 1) & upto_mask(nvalid - 1, d0 + 1);
                x2 &= from_mask(lo, d0 + 2) & upto_mask(nvalid - 1, d0 + 2);
                x3 &= from_mask(lo, d0 + 3) & upto_mask(nvalid - 1, d0 + 3);
            }
            cnt += __popc(x0) + __popc(x1) + __popc(x2) + __popc(x3);
        }
        if (v >= v0 && v < v0 + BD_CW) cnt -= 1;  // v itself
        if (BD_OK(c * Upad + v, NG * Upad, "count part")) part[c * Upad + v] = (int16_t)cnt;
    }
}

// count[sigma[q]] = countq[q] = sum of part[c][q] over the chunks c that
// reach q: every c from the chunk of q's objective-0 tie group start on.
__global__ void bd_sum_kernel(const int16_t* __restrict__ part, const int2* __restrict__ span,
                              int64_t U, int64_t Upad, int64_t NG,
                              const int32_t* __restrict__ sigma, int32_t* __restrict__ count,
                              int32_t* __restrict__ countq) {
    DGRID_LOOP(q, U) {
        if (!BD_OK(sigma[q], U, "sum sigma")) continue;
        if (!BD_OK(span[q].x, U, "sum span")) continue;
        const int64_t c0 = span[q].x / BD_CW;
        int32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        int64_t c = c0;
        for (; c + 4 <= NG; c += 4) {
            a0 += part[c * Upad + q];
            a1 += part[(c + 1) * Upad + q];
            a2 += part[(c + 2) * Upad + q];
            a3 += part[(c + 3) * Upad + q];
        }
        for (; c < NG; ++c) a0 += part[c * Upad + q];
        const int32_t cnt = (a0 + a1) + (a2 + a3);
        count[sigma[q]] = cnt;
        countq[q] = cnt;
    }
}

template <int M>
static void bitdom_launch(dm_ctx* ctx, const int4* S, int64_t U, int64_t NQ, const BitdomLayout& L,
                          char* ws, uint64_t* D) {
    hipStream_t s = ctx->stream;
    const int2* span = (const int2*)(ws + L.span);
    const uint32_t* P = (const uint32_t*)(ws + L.P);
    const int32_t* R = (const int32_t*)(ws + L.R);
    const uint16_t* BK = (const uint16_t*)(ws + L.BK);
    const int64_t maxtasks = L.NG * ((U + BD_RT - 1) / BD_RT);
    // D words only for the D-reading peel (the table-fed peel needs none);
    // four objectives never write D here (fast_bitset: DM_DOM_PEEL_D at M = 4
    // takes the compare kernel), so no 110,988-B LDS kernel is ever launched
    if constexpr (M <= 3)
        if (D)
            bd_rows_kernel<M><<<dim3((unsigned)maxtasks), BD_THREADS, 0, s>>>(
        S, span, U, NQ, L.NG, (const int32_t*)(ws + L.rowfirst), (const int32_t*)(ws + L.toffD), P,
        R, BK, D);
    timing_begin(ctx, DM_TIME_DOMINANCE);
    bd_count_kernel<M><<<dim3((unsigned)maxtasks), BD_THREADS, 0, s>>>(
        S, span, U, L.Upad, L.NG, (const int32_t*)(ws + L.reach), (const int32_t*)(ws + L.toffC), P,
        R, BK, (int16_t*)(ws + L.part));
    timing_end(ctx, DM_TIME_DOMINANCE);
}

int bitdom_build(dm_ctx* ctx, const int4* S, int m, int64_t U, int64_t NQ, int64_t ngroups,
                 const int32_t* nseg, const int32_t* sigma, uint64_t* D, int32_t* count,
                 int32_t* countq, char* ws) {
    hipStream_t s = ctx->stream;
    DM_CHECK_ARG(m >= 2 && m <= 4, "bitdom: 2 to 4 objectives");
    const BitdomLayout L = bitdom_layout(U, m);
    int32_t* first = (int32_t*)(ws + L.first);
    int32_t* last = (int32_t*)(ws + L.last);
    int2* span = (int2*)(ws + L.span);
    bd_ties_kernel<<<dg1(U), 256, 0, s>>>(S, m, U, first, last);
    bd_span_kernel<<<dg1(U), 256, 0, s>>>(S, m, U, first, last, span);
    bd_table_kernel<<<dim3((unsigned)L.NG, (unsigned)(m - 1)), BD_THREADS, 0, s>>>(
        S, U, m - 1, (uint32_t*)(ws + L.P), (int32_t*)(ws + L.R), (uint16_t*)(ws + L.BK));
    bd_plan_kernel<<<1, 1024, 0, s>>>(S, m, last, nseg, U, L.NG, ngroups,
                                      (int32_t*)(ws + L.rowfirst), (int32_t*)(ws + L.reach),
                                      (int32_t*)(ws + L.toffD), (int32_t*)(ws + L.toffC));
    switch (m) {
        case 2: bitdom_launch<2>(ctx, S, U, NQ, L, ws, D); break;
        case 3: bitdom_launch<3>(ctx, S, U, NQ, L, ws, D); break;
        default: bitdom_launch<4>(ctx, S, U, NQ, L, ws, D); break;
    }
    bd_sum_kernel<<<dg1(U), 256, 0, s>>>((const int16_t*)(ws + L.part), span, U, L.Upad, L.NG,
                                         sigma, count, countq);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

}  // namespace dm
