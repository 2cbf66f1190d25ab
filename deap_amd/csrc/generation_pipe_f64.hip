// generation_pipe_f64.hip — double instantiations of the rolling-pipeline hot
// kernel and the per-pair decision kernel (generation_pipe.hpp).
#include "generation_pipe.hpp"

namespace dm {

// One thread per pair: the decisions the replay kernels consume, drawn from
// the same Philox counters — selTournament / selRandom of
// both children (selection.py:55-70, 36-48), the varAnd crossover flag and
// cxTwoPoint cuts (algorithms.py:72-76, crossover.py:62-70), the two mutation
// flags (algorithms.py:78-81) and which children need evaluation
// (algorithms.py:75-81 `del fitness.values`, algorithms.py:155-158).
// Decisions of pair p -> plans[p]; returns the plan's flags.
// Parent-graph labels (the parent order's bins): lab64[r] = (epoch << 32) |
// (INT32_MAX - label); an entry of another epoch is unset, so the persistent
// array needs no zeroing between generations (ctx->plan_lab).  A row's label
// is min(that label, r).
__device__ __forceinline__ int32_t lab_of(const uint64_t* lab64, int32_t r, uint32_t epoch) {
    const uint64_t u = lab64[r];
    return (uint32_t)(u >> 32) == epoch ? min(INT32_MAX - (int32_t)(uint32_t)u, r) : r;
}
// Profiling-only ablations (product build: 0): bit 0 skips the label
// atomics, bit 1 replaces the aspirants' fitness loads by a hash.
#ifndef DM_PLAN_ABLATE
#define DM_PLAN_ABLATE 0
#endif
__device__ __forceinline__ void lab_lower(uint64_t* lab64, int32_t r, int32_t m, uint32_t epoch) {
    if (DM_PLAN_ABLATE & 1) return;
    atomicMax((unsigned long long*)(lab64 + r),
              ((unsigned long long)epoch << 32) | (uint32_t)(INT32_MAX - m));
}

// MF: objectives the register tournaments take (1, or up to 3 for the ZDT /
// DTLZ shapes: pair_plan_kernel<3> for 2-3 objectives, t <= 4)
template <int MF>
__device__ __forceinline__ uint32_t plan_one(const GenArgs& a, PairPlan* __restrict__ plans,
                                             int64_t p, int32_t* __restrict__ keys,
                                             int32_t* __restrict__ hist,
                                             int32_t* __restrict__ tick,
                                             uint64_t* __restrict__ lab64, uint32_t epoch,
                                             int2* __restrict__ pairs2) {
    const int64_t c0 = 2 * p, c1 = 2 * p + 1;
    const bool has1 = c1 < a.nc;
    const int m = a.nobj;
    const uint32_t np = (uint32_t)a.np;
    int32_t s[2];
    // One objective, t <= 8 (C3, C4): every aspirant of both tournaments is
    // drawn first and their fitnesses loaded together, then the tournaments run
    // in registers -- one round of random loads instead of a chain of 2t
    // dependent ones (the same aspirants, the same first-drawn-wins rule).  A
    // winner's validity is read afterwards and only for a clone (no crossover
    // and no mutation: 0.4 of the children at cxpb 0.5, mutpb 0.2): the 2t
    // validity bytes loaded beside the fitnesses were half of the kernel's
    // random requests (round 6).
    // Several objectives (MF = 3): the same with each aspirant's m values
    // loaded together and compared lexicographically (Fitness.__gt__ on the
    // wvalues tuples, base.py:231-238), t <= 4.
    constexpr int TM = MF == 1 ? 8 : 4;
    bool fast = a.sel == DM_SEL_TOURNAMENT && (MF == 1 ? m == 1 : (m >= 2 && m <= MF)) &&
                a.tournsize >= 1 && a.tournsize <= TM;
    double fw[2] = {0.0, 0.0};
    uint8_t vw[2] = {1, 1};
    if (fast && MF > 1) {
        const int t = a.tournsize;
        int32_t kk[2][TM];
        double ff[2][TM][MF];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = (uint32_t)(h ? c1 : c0);
            u32x4 w{};
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                if (j < t && (h == 0 || has1)) {
                    if (!(j & 1)) w = a.rng(ST_SEL, c, (uint32_t)(j >> 1));
                    kk[h][j] = (int32_t)((j & 1) ? bounded64(w.z, w.w, np) : bounded64(w.x, w.y, np));
                } else {
                    kk[h][j] = 0;
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int o = 0; o < MF; ++o)
                    ff[h][j][o] = (j < t && (h == 0 || has1) && o < m)
                                      ? a.pwv[(int64_t)kk[h][j] * m + o] : 0.0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int b = 0;
#pragma unroll
            for (int j = 1; j < TM; ++j) {
                if (!(j < t && (h == 0 || has1))) continue;
                // fit_gt(ff[h][j], ff[h][b]) over the first m objectives
                bool gt = false, decided = false;
#pragma unroll
                for (int o = 0; o < MF; ++o) {
                    double x = ff[h][j][o], y = ff[h][0][o];
#pragma unroll
                    for (int q = 1; q < TM; ++q) y = b == q ? ff[h][q][o] : y;
                    if (!decided && o < m && !(x == y)) {
                        gt = !(x <= y);
                        decided = true;
                    }
                }
                if (gt) b = j;
            }
            int32_t best = kk[h][0];
            double fb = ff[h][0][0];
#pragma unroll
            for (int q = 1; q < TM; ++q) {
                best = b == q ? kk[h][q] : best;
                fb = b == q ? ff[h][q][0] : fb;
            }
            s[h] = best;
            fw[h] = fb;
        }
    } else if (fast) {
        const int t = a.tournsize;
        int32_t kk[2][TM];
        double ff[2][TM];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = (uint32_t)(h ? c1 : c0);
            u32x4 w{};
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                if (j < t && (h == 0 || has1)) {
                    if (!(j & 1)) w = a.rng(ST_SEL, c, (uint32_t)(j >> 1));
                    kk[h][j] = (int32_t)((j & 1) ? bounded64(w.z, w.w, np) : bounded64(w.x, w.y, np));
                } else {
                    kk[h][j] = 0;
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < TM; ++j)
                if (j < t && (h == 0 || has1))
                    ff[h][j] = (DM_PLAN_ABLATE & 2) ? (double)(kk[h][j] & 1023) : a.pwv[kk[h][j]];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int32_t best = kk[h][0];
            double fb = ff[h][0];
#pragma unroll
            for (int j = 1; j < TM; ++j)
                if (j < t && (h == 0 || has1) && !(ff[h][j] == fb) && !(ff[h][j] <= fb)) {
                    best = kk[h][j];
                    fb = ff[h][j];
                }
            s[h] = best;
            fw[h] = fb;
        }
    }
    for (int h = 0; h < (has1 ? 2 : 1) && !fast; ++h) {
        const uint32_t c = (uint32_t)(h ? c1 : c0);
        if (a.sel == DM_SEL_RANDOM) {
            const u32x4 w = a.rng(ST_SEL, c, 0);
            s[h] = (int32_t)bounded64(w.x, w.y, np);
            continue;
        }
        // first-drawn aspirant wins ties: replace only on fit_gt (selection.py:68)
        int32_t best = 0;
        u32x4 w{};
        for (int j = 0; j < a.tournsize; ++j) {
            if (!(j & 1)) w = a.rng(ST_SEL, c, (uint32_t)(j >> 1));
            const int32_t k = (int32_t)((j & 1) ? bounded64(w.z, w.w, np) : bounded64(w.x, w.y, np));
            if (j == 0 || fit_gt(a.pwv + (int64_t)k * m, a.pwv + (int64_t)best * m, m)) best = k;
        }
        s[h] = best;
    }
    if (!has1) s[1] = s[0];
    uint32_t fl = has1 ? PF_HAS1 : 0u;
    uint32_t cuts = 0;
    if (a.cx != DM_CX_NONE && has1) {
        const u32x4 w = a.rng(ST_CX, (uint32_t)p, 0);
        if ((uint64_t)w.x < a.thr_cx) {
            fl |= PF_CX;
            if (a.cx == DM_CX_TWOPOINT) {
                const u32x4 w2 = a.rng(ST_CX, (uint32_t)p, 1);
                int32_t r1 = 1 + (int32_t)bounded64(w.z, w.w, (uint32_t)a.dim);
                int32_t r2 = 1 + (int32_t)bounded64(w2.x, w2.y, (uint32_t)(a.dim - 1));
                if (r2 >= r1) {
                    r2 += 1;
                } else {
                    const int32_t t = r1;
                    r1 = r2;
                    r2 = t;
                }
                cuts = (uint32_t)r1 | ((uint32_t)r2 << 16);
            }
        }
    }
    if (a.mut != DM_MUT_NONE) {
        if ((uint64_t)a.rng(ST_MUT, (uint32_t)c0, 0).x < a.thr_mut) fl |= PF_MUT0;
        if (has1 && (uint64_t)a.rng(ST_MUT, (uint32_t)c1, 0).x < a.thr_mut) fl |= PF_MUT1;
    }
    const bool cx = fl & PF_CX;
    if (!fast) {
        vw[0] = a.pvalid[s[0]];
        vw[1] = a.pvalid[s[1]];
        fw[0] = a.pwv[(int64_t)s[0] * m];
        fw[1] = a.pwv[(int64_t)s[1] * m];
    } else {
        // a varied child is invalid whatever its parent was: only clones read it
        if (!cx && !(fl & PF_MUT0)) vw[0] = a.pvalid[s[0]];
        if (has1 && !cx && !(fl & PF_MUT1)) vw[1] = a.pvalid[s[1]];
        if (!has1) {
            vw[1] = vw[0];
            fw[1] = fw[0];
        }
    }
    if (cx || (fl & PF_MUT0) || !vw[0]) fl |= PF_INV0;
    if (has1 && (cx || (fl & PF_MUT1) || !vw[1])) fl |= PF_INV1;
    PairPlan pl;
    pl.s0 = s[0];
    pl.s1 = s[1];
    pl.cuts = cuts;
    pl.flags = fl;
    pl.f0 = fw[0];
    pl.f1 = fw[1];
    plans[p] = pl;
    if (keys && tick) {
        // sort key: the fitter parent (tournament winners repeat with their
        // fitness: a fitter row is the likelier one to recur in other pairs)
        const int32_t key = pl.f1 > pl.f0 ? s[1] : s[0];
        keys[p] = key;
        tick[p] = atomicAdd(hist + key, 1);
    } else if (lab64) {
        // neighbourhood bins: the first label-propagation round (plan_label_kernel);
        // the pair's parents also go to a compact array the label rounds and
        // the bin kernel read (8 B per pair instead of 32-B plans)
        if (pairs2) pairs2[p] = make_int2(s[0], s[1]);
        // only the larger row can take a smaller label from this pair (a row's
        // label is at most the row itself): one random atomic per pair, not two
        // (each is a memory-side round trip: the two took 23 of the kernel's
        // 68 us, profiles/r06_prelude)
        if (has1 && s[0] != s[1]) lab_lower(lab64, max(s[0], s[1]), min(s[0], s[1]), epoch);
    } else if (hist) {
        // degree keys (plan_degree_key_kernel): count both parents' slots
        atomicAdd(hist + s[0], 1);
        if (has1) atomicAdd(hist + s[1], 1);
    }
    return fl;
}

// With count_evals set (the context's spread counters), the plan kernel also
// counts the generation's `nevals` (children whose fitness is invalidated,
// algorithms.py:171-174) into a.nevals: one ballot per wave, evals_fold per
// workgroup.
// zero (nullable): nzero ints this launch clears for a later one (the parent
// order's ticket counters: no separate fill launch)
template <int MF>
__global__ __launch_bounds__(256) void pair_plan_kernel(GenArgs a, PairPlan* __restrict__ plans,
                                                        long long* __restrict__ count_evals,
                                                        int32_t* __restrict__ keys,
                                                        int32_t* __restrict__ hist,
                                                        int32_t* __restrict__ tick,
                                                        uint64_t* __restrict__ lab64,
                                                        uint32_t epoch,
                                                        int2* __restrict__ pairs2,
                                                        int32_t* __restrict__ zero, int64_t nzero) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npairs = (a.nc + 1) / 2;
    if (zero)
        for (int64_t i = p; i < nzero; i += (int64_t)gridDim.x * blockDim.x) zero[i] = 0;
    if (count_evals) {
        __shared__ int32_t wave_evals[4];
        uint32_t fl = 0;
        if (p < npairs) fl = plan_one<MF>(a, plans, p, keys, hist, tick, lab64, epoch, pairs2);
        const int32_t cnt = __popcll(__ballot((fl & PF_INV0) != 0)) +
                            __popcll(__ballot((fl & PF_INV1) != 0));
        if ((threadIdx.x & 63) == 0) wave_evals[threadIdx.x >> 6] = cnt;
        __syncthreads();
        if (threadIdx.x == 0)
            evals_fold(count_evals, a.nevals,
                       (long long)wave_evals[0] + wave_evals[1] + wave_evals[2] + wave_evals[3]);
        return;
    }
    if (p < npairs) plan_one<MF>(a, plans, p, keys, hist, tick, lab64, epoch, pairs2);
}

void launch_pair_plans(const GenArgs& a, PairPlan* plans, long long* count_evals, hipStream_t s,
                       int32_t* keys, int32_t* hist, int32_t* tick, uint64_t* lab64,
                       uint32_t epoch, int2* pairs2, int32_t* zero, int64_t nzero) {
    const int64_t npairs = (a.nc + 1) / 2;
    const dim3 grid((unsigned)((npairs + 255) / 256));
    if (a.nobj >= 2 && a.nobj <= 3)
        pair_plan_kernel<3><<<grid, 256, 0, s>>>(a, plans, count_evals, keys, hist, tick, lab64, epoch,
                                                 pairs2, zero, nzero);
    else
        pair_plan_kernel<1><<<grid, 256, 0, s>>>(a, plans, count_evals, keys, hist, tick, lab64, epoch,
                                                 pairs2, zero, nzero);
}

// Counting-sort placement of the plans by key: slot start[key] + tick of pair
// p, the plan copied with p in its flags (the hot kernel then reads its plans
// contiguously; an index array read before each plan was 1.2 % slower,
// profiles/r04i).  The order inside a key's run is whatever the plan
// kernel's atomics gave: the processing order never changes a result (every
// child is a function of its own plan and counters).
__global__ __launch_bounds__(256) void plan_order_kernel(const PairPlan* __restrict__ plans,
                                                         const int32_t* __restrict__ keys,
                                                         const int32_t* __restrict__ tick,
                                                         const int32_t* __restrict__ start,
                                                         PairPlan* __restrict__ ordered,
                                                         int64_t npairs) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npairs) return;
    PairPlan pl = plans[p];
    pl.flags |= (uint32_t)p << PF_PAIR_SHIFT;
    ordered[start[keys[p]] + tick[p]] = pl;
}

// Degree keys: the parent that appears in more pair slots of this generation
// (a greedy vertex cover of the pairs: fewer distinct key rows than the fitter
// parent gives), ticketed into the zeroed hist2.
// With lab (label propagation below) the bin is the pair's label -- the
// smaller of its parents' labels -- instead of a degree key: the pairs of one
// neighbourhood of the parent graph land together, so more of their rows
// (not only one shared parent's) are re-read from the L2.
__global__ __launch_bounds__(256) void plan_degree_key_kernel(const PairPlan* __restrict__ plans,
                                                              const int2* __restrict__ pairs2,
                                                              const int32_t* __restrict__ deg,
                                                              const uint64_t* __restrict__ lab64,
                                                              uint32_t epoch, int jump,
                                                              int32_t* __restrict__ keys,
                                                              int32_t* __restrict__ tick,
                                                              int32_t* __restrict__ hist2,
                                                              int64_t npairs) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npairs) return;
    const int2 pr = pairs2 ? pairs2[p] : make_int2(plans[p].s0, plans[p].s1);
    const int32_t s0 = pr.x, s1 = pr.y;
    int32_t bin;
    if (lab64) {
        const int32_t l0 = lab_of(lab64, s0, epoch), l1 = lab_of(lab64, s1, epoch);
        bin = min(l0, l1);
        // jump: the labels of the two labels (rows themselves) -- a second
        // propagation round as gathers, no atomics: the label kernel's round
        // took 27 us, 22 of them its random atomics (profiles/r06_prelude),
        // and a jump groups the pairs as well (tools_gpu/plan_order_sim.py:
        // 0.657 of the parent reads left at runs of 64, as a second round)
        if (jump) bin = min(bin, min(lab_of(lab64, l0, epoch), lab_of(lab64, l1, epoch)));
    } else {
        bin = deg[s1] > deg[s0] ? s1 : s0;
    }
    keys[p] = bin;
    tick[p] = atomicAdd(hist2 + bin, 1);
}
void launch_plan_degree_keys(const PairPlan* plans, const int2* pairs2, const int32_t* deg,
                             const uint64_t* lab64, uint32_t epoch, bool jump, int32_t* keys,
                             int32_t* tick, int32_t* hist2, int64_t npairs, hipStream_t s) {
    plan_degree_key_kernel<<<dim3((unsigned)((npairs + 255) / 256)), 256, 0, s>>>(
        plans, pairs2, deg, lab64, epoch, jump ? 1 : 0, keys, tick, hist2, npairs);
}

// One round of label propagation over the parent graph (rows = vertices, a
// pair's two parents = an edge): every parent takes the smallest label among
// itself and its pair partner (lab_of / lab_lower above: epoch-tagged, never
// zeroed).  In place -- the rounds are a heuristic for locality, any
// interleaving of the atomics is a valid labelling and the order never changes
// a child.  The first round runs inside the plan kernel.
__global__ __launch_bounds__(256) void plan_label_kernel(const int2* __restrict__ pairs2,
                                                         uint64_t* __restrict__ lab64,
                                                         uint32_t epoch, int64_t npairs) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npairs) return;
    const int2 pr = pairs2[p];
    const int32_t s0 = pr.x, s1 = pr.y;
    const int32_t l0 = lab_of(lab64, s0, epoch), l1 = lab_of(lab64, s1, epoch);
    const int32_t m = min(l0, l1);
    if (m < l0) lab_lower(lab64, s0, m, epoch);
    if (m < l1) lab_lower(lab64, s1, m, epoch);
}
void launch_plan_labels(const int2* pairs2, uint64_t* lab64, uint32_t epoch, int64_t npairs,
                        int rounds, hipStream_t s) {
    for (int r = 0; r < rounds; ++r)
        plan_label_kernel<<<dim3((unsigned)((npairs + 255) / 256)), 256, 0, s>>>(pairs2, lab64,
                                                                                 epoch, npairs);
}

void launch_plan_order(const PairPlan* plans, const int32_t* keys, const int32_t* tick,
                       const int32_t* start, PairPlan* ordered, int64_t npairs, hipStream_t s) {
    plan_order_kernel<<<dim3((unsigned)((npairs + 255) / 256)), 256, 0, s>>>(plans, keys, tick,
                                                                            start, ordered, npairs);
}

void launch_gen_pipe_f64(const PipeArgs& a, int ec, int cx, int mut, int nch, int num_cus,
                         hipStream_t s) {
    if (nch == 0)
        launch_gen_pipe_long(a, true, ec, cx, mut, num_cus, s);
    else if (nch <= 2)
        launch_pipe_ops<double, 2>(a, ec, cx, mut, num_cus, s);
    else
        launch_pipe_ops<double, 4>(a, ec, cx, mut, num_cus, s);
}

}  // namespace dm
