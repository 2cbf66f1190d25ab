// generation.hpp — fused eaSimple generation body for gfx950:
//   selTournament / selRandom / index / identity  (selection.py:12-24, 51-69)
//   -> toolbox.clone                              (base.py:49, algorithms.py:68)
//   -> varAnd: pair crossover + per-child mutation (algorithms.py:33-82)
//   -> evaluate invalid children                  (algorithms.py:171-174)
//
// One lane group of G lanes produces one offspring pair (children 2p, 2p+1),
// streaming the two parent rows through registers in chunks of 4 genes per
// lane (floats: 2x16-B or 16-B loads per lane; packed bits: one u64 word per
// lane) so each individual-generation reads its parent genome once and writes
// the child genome once: B = 2G + (t+1)F algorithmic bytes.
// Randomness: Philox4x32-10 keyed by (seed, island, gen) with the counter
// layout in common.hpp, or injected / dumped decisions (DM_RNG_INJECT/_DUMP).
#pragma once
#include "common.hpp"
#include "evals.hpp"

namespace dm {

struct GenArgs {
    const char* pgenes;
    const double* pwv;
    const uint8_t* pvalid;
    int64_t np, pstride;
    char* cgenes;
    double* cwv;
    uint8_t* cvalid;
    int64_t nc, cstride;
    int32_t dim, nobj, words64;  // words64 = ceil(dim/64)
    int32_t sel, tournsize;
    const int32_t* sel_index;
    int32_t cx, mut;
    uint64_t thr_cx, thr_mut, thr_ind;
    double alpha, indpb, mu, sigma;
    const double* mu_vec;
    const double* sigma_vec;
    float flip_inv_log2;  // 1 / log2(1 - indpb) for geometric skips
    int32_t eval_fn;
    double w0;  // ev.weights[0]
    // C2 fitness keys (fit_key_kernel, generation_pipe_bits.hip): the parents'
    // wvalues as exact int16 multiples of |w0| (or FIT_KEY_NONE), nullable
    const int16_t* pkeys;
    dm_eval ev;
    Rng rng;
    const double* zig;
    int32_t mode;
    dm_decisions dec;
    int64_t* nevals;
};

// ---------------------------------------------------------------------------
// Selection of the parent of child c (all lanes of the group compute the same
// value; only the group leader writes dumped decisions).
// ---------------------------------------------------------------------------
template <bool RP>
__device__ __forceinline__ int64_t parent_of(const GenArgs& a, int64_t c, bool leader) {
    if (a.sel == DM_SEL_IDENTITY) return c;
    if (a.sel == DM_SEL_INDEX) return a.sel_index[c];
    const int t = a.tournsize;
    const int m = a.nobj;
    int64_t best = 0;
    for (int j = 0; j < t; ++j) {
        int64_t cand;
        if ((RP && a.mode == DM_RNG_INJECT)) {
            cand = a.dec.aspirants[c * t + j];
        } else {
            const u32x4 w = a.rng(ST_SEL, (uint32_t)c, (uint32_t)(j >> 1));
            cand = (j & 1) ? bounded64(w.z, w.w, (uint32_t)a.np) : bounded64(w.x, w.y, (uint32_t)a.np);
            if ((RP && a.mode == DM_RNG_DUMP) && leader) a.dec.aspirants[c * t + j] = (int32_t)cand;
        }
        if (a.sel == DM_SEL_RANDOM) return cand;  // selRandom: k draws of one aspirant
        if (j == 0) {
            best = cand;
        } else if (fit_gt(a.pwv + cand * m, a.pwv + best * m, m)) {
            best = cand;  // max(): replace only when strictly greater  (selection.py:68)
        }
    }
    return best;
}

struct PairDecisions {
    bool cx;
    int32_t c1, c2;  // cxTwoPoint slice [c1, c2)
    bool mut0, mut1;
};

template <bool RP>
__device__ __forceinline__ PairDecisions pair_decisions(const GenArgs& a, int64_t p, bool has1,
                                                        bool leader) {
    PairDecisions d{};
    const int64_t c0 = 2 * p, c1i = 2 * p + 1;
    int32_t r1 = 0, r2 = 0;
    if (has1 && a.cx != DM_CX_NONE) {
        if ((RP && a.mode == DM_RNG_INJECT)) {
            d.cx = a.dec.cx_flag[p] != 0;
            if (a.cx == DM_CX_TWOPOINT && d.cx) {
                r1 = a.dec.cx_raw[2 * p];
                r2 = a.dec.cx_raw[2 * p + 1];
            }
        } else {
            const u32x4 w = a.rng(ST_CX, (uint32_t)p, 0);
            d.cx = (uint64_t)w.x < a.thr_cx;
            if (a.cx == DM_CX_TWOPOINT && d.cx) {
                // randint(1, size); randint(1, size - 1)       (crossover.py:50-51)
                const u32x4 w2 = a.rng(ST_CX, (uint32_t)p, 1);
                r1 = 1 + (int32_t)bounded64(w.z, w.w, (uint32_t)a.dim);
                r2 = 1 + (int32_t)bounded64(w2.x, w2.y, (uint32_t)(a.dim - 1));
            }
            if ((RP && a.mode == DM_RNG_DUMP) && leader) {
                a.dec.cx_flag[p] = d.cx;
                if (a.dec.cx_raw) {
                    a.dec.cx_raw[2 * p] = r1;
                    a.dec.cx_raw[2 * p + 1] = r2;
                }
            }
        }
        if (a.cx == DM_CX_TWOPOINT && d.cx) {
            // if cxpoint2 >= cxpoint1: cxpoint2 += 1 else swap      (crossover.py:52-55)
            if (r2 >= r1) {
                r2 += 1;
            } else {
                const int32_t t = r1;
                r1 = r2;
                r2 = t;
            }
            d.c1 = r1;
            d.c2 = r2;
        }
    }
    if (a.mut != DM_MUT_NONE) {
        if ((RP && a.mode == DM_RNG_INJECT)) {
            d.mut0 = a.dec.mut_flag[c0] != 0;
            d.mut1 = has1 && a.dec.mut_flag[c1i] != 0;
        } else {
            d.mut0 = (uint64_t)a.rng(ST_MUT, (uint32_t)c0, 0).x < a.thr_mut;
            d.mut1 = has1 && (uint64_t)a.rng(ST_MUT, (uint32_t)c1i, 0).x < a.thr_mut;
            if ((RP && a.mode == DM_RNG_DUMP) && leader) {
                a.dec.mut_flag[c0] = d.mut0;
                if (has1) a.dec.mut_flag[c1i] = d.mut1;
            }
        }
    }
    return d;
}

// ---------------------------------------------------------------------------
// Float genomes (T = float | double): chunk = 4 genes per lane.
// ---------------------------------------------------------------------------
template <typename T>
struct Vec4;
typedef double dm_d2 __attribute__((ext_vector_type(2)));
typedef float dm_f4 __attribute__((ext_vector_type(4)));
#ifndef DM_NT_STORES
#define DM_NT_STORES 1
#endif

template <>
struct Vec4<double> {
    // streaming store: the child row is not re-read in this launch, keep it
    // out of L2/MALL (non-temporal: measured 6.07 vs 3.9-5.8 TB/s on copies)
    __device__ __forceinline__ static void store_nt(char* row, int g, const double (&x)[4]) {
        dm_d2* p = reinterpret_cast<dm_d2*>(row + (size_t)g * 8);
        const dm_d2 a = {x[0], x[1]}, b = {x[2], x[3]};
        if (DM_NT_STORES) {
            __builtin_nontemporal_store(a, p);
            __builtin_nontemporal_store(b, p + 1);
        } else {
            p[0] = a;
            p[1] = b;
        }
    }
    __device__ __forceinline__ static void load(const char* row, int g, double (&x)[4]) {
        const double2* p = reinterpret_cast<const double2*>(row + (size_t)g * 8);
        const double2 a = p[0], b = p[1];
        x[0] = a.x;
        x[1] = a.y;
        x[2] = b.x;
        x[3] = b.y;
    }
    __device__ __forceinline__ static void store(char* row, int g, const double (&x)[4]) {
        double2* p = reinterpret_cast<double2*>(row + (size_t)g * 8);
        p[0] = make_double2(x[0], x[1]);
        p[1] = make_double2(x[2], x[3]);
    }
};
template <>
struct Vec4<float> {
    __device__ __forceinline__ static void store_nt(char* row, int g, const double (&x)[4]) {
        const dm_f4 v = {(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
        if (DM_NT_STORES)
            __builtin_nontemporal_store(v, reinterpret_cast<dm_f4*>(row + (size_t)g * 4));
        else
            *reinterpret_cast<dm_f4*>(row + (size_t)g * 4) = v;
    }
    __device__ __forceinline__ static void load(const char* row, int g, double (&x)[4]) {
        const float4 a = *reinterpret_cast<const float4*>(row + (size_t)g * 4);
        x[0] = a.x;
        x[1] = a.y;
        x[2] = a.z;
        x[3] = a.w;
    }
    __device__ __forceinline__ static void store(char* row, int g, const double (&x)[4]) {
        // array('f') semantics: fp64 arithmetic, round-to-nearest on store.
        *reinterpret_cast<float4*>(row + (size_t)g * 4) =
            make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]);
    }
};

// Per-gene Philox slots (streams ST_BLEND, ST_MASK): the four words of call
// (stage, item, sub = 64c + L) feed the four genes lane L holds in chunk c of
// the hot kernel's lane layout (generation_pipe.hpp ChunkLayout): fp64 genes
// {256c + 2L, +1, 256c + 128 + 2L, +1}, fp32 genes 256c + 4L .. +3.  Here the
// words of four consecutive genes g .. g+3 (g % 4 == 0) are gathered from
// that layout: one call for fp32 rows, two for fp64 rows.
template <typename T>
__device__ __forceinline__ u32x4 gene4_words(const Rng& rng, uint32_t stage, uint32_t item, int g) {
    if constexpr (sizeof(T) == 4) {
        return rng(stage, item, (uint32_t)(g >> 2));
    } else {
        const int r = g & 255;
        const uint32_t sub = (uint32_t)(((g >> 8) << 6) + ((r & 127) >> 1));
        const u32x4 a = rng(stage, item, sub), b = rng(stage, item, sub + 1);
        return (r & 128) ? u32x4{a.z, a.w, b.z, b.w} : u32x4{a.x, a.y, b.x, b.y};
    }
}

// Per-gene Gaussian mutation of one child's chunk (mutation.py:44-46).
// Returns the 4-bit mask of mutated genes; the normal draws happen in
// gauss_apply so only one inlined copy of log/cos/sqrt exists.
// Standard normal draw for (child, gene): 256-layer ziggurat (common.hpp).
// Out of line: the draw is rare (indpb of the genes of mutated children) and
// keeping its wedge/tail transcendental paths out of the streaming loop saves
// VGPRs there.
__device__ __noinline__ double std_normal(const double* zig, Rng rng, int64_t c, int gi) {
    return zig_normal(zig, rng, ST_GAUSS, (uint32_t)c, (uint32_t)gi);
}

template <typename T, bool RP>
__device__ __forceinline__ uint32_t gauss_mask(const GenArgs& a, int64_t c, int g) {
    uint32_t bits = 0;
    if ((RP && a.mode == DM_RNG_INJECT)) {
        const uint64_t word = a.dec.mut_mask[c * a.words64 + (g >> 6)];
        bits = (uint32_t)(word >> (g & 63)) & 0xFu;
    } else {
        const u32x4 w = gene4_words<T>(a.rng, ST_MASK, (uint32_t)c, g);
        bits = ((uint64_t)w.x < a.thr_ind ? 1u : 0u) | ((uint64_t)w.y < a.thr_ind ? 2u : 0u) |
               ((uint64_t)w.z < a.thr_ind ? 4u : 0u) | ((uint64_t)w.w < a.thr_ind ? 8u : 0u);
        if ((RP && a.mode == DM_RNG_DUMP) && bits) {
            atomicOr((unsigned long long*)&a.dec.mut_mask[c * a.words64 + (g >> 6)],
                     (unsigned long long)bits << (g & 63));
        }
    }
    const int valid = a.dim - g;  // genes of this lane inside the row
    if (valid < 4) bits &= (1u << max(valid, 0)) - 1u;
    return bits;
}
template <bool RP>
__device__ __forceinline__ double gauss_value(const GenArgs& a, int64_t c, int gi) {
    if ((RP && a.mode == DM_RNG_INJECT)) return a.dec.gauss[c * a.dim + gi];
    const double nrm = std_normal(a.zig, a.rng, c, gi);
    const double m = a.mu_vec ? a.mu_vec[gi] : a.mu;
    const double s = a.sigma_vec ? a.sigma_vec[gi] : a.sigma;
    const double gv = m + nrm * s;  // random.gauss(mu, sigma) = mu + z*sigma
    if ((RP && a.mode == DM_RNG_DUMP)) a.dec.gauss[c * a.dim + gi] = gv;
    return gv;
}
// Apply the Gaussian steps of both children: bits 0-3 child 0, 4-7 child 1.
template <bool RP>
__device__ __forceinline__ void gauss_apply(const GenArgs& a, int64_t c0, int g, uint32_t bits,
                                            double (&y0)[4], double (&y1)[4]) {
#pragma unroll 1
    while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const int j = b & 3;
        const double gv = gauss_value<RP>(a, c0 + (b >> 2), g + j);
        if (b < 4) {
            y0[0] = j == 0 ? y0[0] + gv : y0[0];
            y0[1] = j == 1 ? y0[1] + gv : y0[1];
            y0[2] = j == 2 ? y0[2] + gv : y0[2];
            y0[3] = j == 3 ? y0[3] + gv : y0[3];
        } else {
            y1[0] = j == 0 ? y1[0] + gv : y1[0];
            y1[1] = j == 1 ? y1[1] + gv : y1[1];
            y1[2] = j == 2 ? y1[2] + gv : y1[2];
            y1[3] = j == 3 ? y1[3] + gv : y1[3];
        }
    }
}

#ifndef DM_GEN_MINWAVES
#define DM_GEN_MINWAVES 4
#endif
#ifndef DM_GEN_PREFETCH
#define DM_GEN_PREFETCH 1
#endif
template <typename T, int G, int CX, int MUT, int EC, bool RP>
__global__ __launch_bounds__(256, DM_GEN_MINWAVES) void gen_float_kernel(GenArgs a) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const bool leader = sub == 0;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t evals = 0;
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; p < npairs;
         p += gstride) {
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        const bool has1 = c1 < a.nc;
        const int64_t s0 = parent_of<RP>(a, c0, leader);
        const int64_t s1 = has1 ? parent_of<RP>(a, c1, leader) : s0;
        const PairDecisions d = pair_decisions<RP>(a, p, has1, leader);
        const bool inv0 = d.cx || d.mut0 || !a.pvalid[s0];
        const bool inv1 = has1 && (d.cx || d.mut1 || !a.pvalid[s1]);
        const bool do_eval = EC != EC_NONE;

        const char* r0 = a.pgenes + s0 * a.pstride;
        const char* r1 = a.pgenes + s1 * a.pstride;
        char* w0 = a.cgenes + c0 * a.cstride;
        char* w1 = a.cgenes + c1 * a.cstride;
        EvalState e0, e1;
        eval_init(e0);
        eval_init(e1);
        const double gamma_scale = 1.0 + 2.0 * a.alpha;  // (1. + 2. * alpha)

        // software pipeline: the next chunk's parent loads are in flight while
        // the current chunk is varied, evaluated and stored
        double n0[4] = {0, 0, 0, 0}, n1[4] = {0, 0, 0, 0};
        if (DM_GEN_PREFETCH && 4 * sub < a.dim) {
            Vec4<T>::load(r0, 4 * sub, n0);
            if (has1) Vec4<T>::load(r1, 4 * sub, n1);
        }
        for (int cbase = 0; cbase < a.dim; cbase += 4 * G) {
            const int g = cbase + 4 * sub;
            double y0[4], y1[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                y0[j] = n0[j];
                y1[j] = n1[j];
            }
            const bool in = g < a.dim;
            if (DM_GEN_PREFETCH) {
                const int gn = g + 4 * G;
                if (gn < a.dim) {
                    Vec4<T>::load(r0, gn, n0);
                    if (has1) Vec4<T>::load(r1, gn, n1);
                }
            } else if (in) {
                Vec4<T>::load(r0, g, y0);
                if (has1) Vec4<T>::load(r1, g, y1);
            }
            if (CX == DM_CX_BLEND && d.cx && in) {
                // gamma = (1. + 2.*alpha)*random() - alpha ; y1/y2 blend  (crossover.py:255-258)
                double u[4];
                if ((RP && a.mode == DM_RNG_INJECT)) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        u[j] = (g + j < a.dim) ? a.dec.blend_u[p * a.dim + g + j] : 0.0;
                } else {
                    const u32x4 w = gene4_words<T>(a.rng, ST_BLEND, (uint32_t)p, g);
                    u[0] = u01_32(w.x);
                    u[1] = u01_32(w.y);
                    u[2] = u01_32(w.z);
                    u[3] = u01_32(w.w);
                    if ((RP && a.mode == DM_RNG_DUMP)) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (g + j < a.dim) a.dec.blend_u[p * a.dim + g + j] = u[j];
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (g + j < a.dim) {
                        const double gm = gamma_scale * u[j] - a.alpha;
                        const double x1 = y0[j], x2 = y1[j];
                        y0[j] = (1.0 - gm) * x1 + gm * x2;
                        y1[j] = gm * x1 + (1.0 - gm) * x2;
                    }
                }
            } else if (CX == DM_CX_TWOPOINT && d.cx && in) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int gi = g + j;
                    if (gi >= d.c1 && gi < d.c2) {
                        const double t = y0[j];
                        y0[j] = y1[j];
                        y1[j] = t;
                    }
                }
            }
            if constexpr (sizeof(T) == 4) {
                // array('f') stores the crossover result (rounded) before mutation reads it
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y0[j] = (double)(float)y0[j];
                    y1[j] = (double)(float)y1[j];
                }
            }
            if (MUT == DM_MUT_GAUSSIAN && in) {
                uint32_t bits = 0;
                if (d.mut0) bits |= gauss_mask<T, RP>(a, c0, g);
                if (d.mut1) bits |= gauss_mask<T, RP>(a, c1, g) << 4;
                gauss_apply<RP>(a, c0, g, bits, y0, y1);
            }
            if (in) {
                Vec4<T>::store_nt(w0, g, y0);
                if (has1) Vec4<T>::store_nt(w1, g, y1);
            }
            if constexpr (sizeof(T) == 4) {
                // Evaluate the stored (fp32-rounded) genes, as DEAP reads array('f').
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y0[j] = (double)(float)y0[j];
                    y1[j] = (double)(float)y1[j];
                }
            }
            if (do_eval) {
                eval_chunk<G, EC>(a.ev, a.dim, g, cbase, y0, inv0, e0);
                eval_chunk<G, EC>(a.ev, a.dim, g, cbase, y1, inv1, e1);
            }
        }
        double f0[DM_MAX_OBJ], f1[DM_MAX_OBJ];
        if (do_eval) {
            eval_finish<G, EC>(a.ev, a.dim, e0, f0);
            eval_finish<G, EC>(a.ev, a.dim, e1, f1);
        }
        if (leader) {
            if constexpr (ec_single(EC)) {  // one objective
                a.cwv[c0] = inv0 ? f0[0] * a.w0 : a.pwv[s0];
                if (has1) a.cwv[c1] = inv1 ? f1[0] * a.w0 : a.pwv[s1];
            } else {
                const int m = a.nobj;
                for (int o = 0; o < m; ++o) {
                    a.cwv[c0 * m + o] =
                        (do_eval && inv0) ? f0[o] * a.ev.weights[o] : a.pwv[s0 * m + o];
                    if (has1)
                        a.cwv[c1 * m + o] =
                            (do_eval && inv1) ? f1[o] * a.ev.weights[o] : a.pwv[s1 * m + o];
                }
            }
            a.cvalid[c0] = do_eval ? 1 : (inv0 ? 0 : 1);
            if (has1) a.cvalid[c1] = do_eval ? 1 : (inv1 ? 0 : 1);
            evals += (int64_t)inv0 + (int64_t)inv1;
        }
    }
    if (a.nevals && EC != EC_NONE) {
        // one atomic per wave: sum the leaders' counts
        int64_t tot = evals;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)a.nevals, (unsigned long long)tot);
    }
}

// ---------------------------------------------------------------------------
// Packed-bit genomes: chunk = one u64 word per lane (64 genes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t range_mask(int lo, int hi) {  // bits [lo, hi) of a word
    lo = max(lo, 0);
    hi = min(hi, 64);
    if (hi <= lo) return 0;
    const uint64_t up = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
    const uint64_t dn = lo <= 0 ? 0ull : ((1ull << lo) - 1);
    return up & ~dn;
}

// mutFlipBit (mutation.py:124-142): Bernoulli(indpb) per gene, drawn as ONE
// geometric-skip sequence over the whole row: uniform i of
// child c is word i & 3 of Philox(ST_FLIP, c, i >> 2), u = (w + 1) / 2^32,
// gap_i = min(floor(log2f(u) / log2(1 - indpb)), 65536) (fp32), and the
// flipped genes are P_m = P_{m-1} + 1 + gap_m (P_{-1} = -1) while P_m < dim.
// A group of G lanes draws 4G gaps per round (lane `sub` = Philox call
// round * G + sub) and places them with a group prefix sum, so a 4096-gene
// row at indpb 0.05 takes one Philox call per lane.  The positions of the
// current round stay in registers across the G-word chunks of a row; a
// chunk's words are assembled in LDS (G words per group, ds_or).
template <int G>
struct FlipRow {
    int32_t pos[4];  // this lane's positions in the current round (ascending)
    int32_t last;    // last position of the round (group-uniform)
    uint32_t round;
};

template <int G>
__device__ __forceinline__ void flip_round(const GenArgs& a, int64_t c, int sub, int32_t base,
                                           FlipRow<G>& st) {
    const u32x4 w = a.rng(ST_FLIP, (uint32_t)c, st.round * G + (uint32_t)sub);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    int32_t s = 0, loc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float u = ((float)ws[j] + 1.0f) * 2.3283064365386963e-10f;
        const float gap = floorf(__log2f(fminf(u, 1.0f)) * a.flip_inv_log2);
        s += 1 + (int32_t)fminf(gap, 65536.0f);
        loc[j] = s;
    }
    int32_t incl = s;  // group inclusive scan of the lanes' sums
#pragma unroll
    for (int d = 1; d < G; d <<= 1) {
        const int32_t t = __shfl_up(incl, d, G);
        if (sub >= d) incl += t;
    }
    const int32_t excl = base + incl - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) st.pos[j] = excl + loc[j];
    st.last = base + __shfl(incl, G - 1, G);
}

template <int G>
__device__ __forceinline__ void flip_begin(const GenArgs& a, int64_t c, int sub, FlipRow<G>& st) {
    st.round = 0;
    if (a.thr_ind > 0 && a.thr_ind < (1ull << 32)) flip_round<G>(a, c, sub, -1, st);
}

// Flip bits of chunk [64 wb, 64 (wb + G)) of child c's row ORed into the G
// LDS words `lds` (zeroed first); 0 < indpb < 1.
template <int G>
__device__ __forceinline__ void flip_chunk_lds(const GenArgs& a, int64_t c, int wb, int sub,
                                               FlipRow<G>& st, uint64_t* lds) {
    const int32_t lo = wb * 64;
    const int32_t hi = min(a.dim, (wb + G) * 64);
    lds[sub] = 0;
    __builtin_amdgcn_wave_barrier();
    while (true) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int32_t q = st.pos[j];
            if (q >= lo && q < hi) atomicOr((unsigned long long*)&lds[(q - lo) >> 6], 1ull << (q & 63));
        }
        if (st.last >= hi) break;  // the round reaches the next chunk (kept)
        st.round += 1;
        flip_round<G>(a, c, sub, st.last, st);
    }
}

// The flip mask of word wb + sub of child c (chunk [64 wb, 64 (wb + G)) of the
// row); called by every lane of the group, chunks in ascending order.
// `lds`: this group's G words.  Inject / dump as the replay modes need.
template <int G, bool RP>
__device__ __forceinline__ uint64_t flip_mask_chunk(const GenArgs& a, int64_t c, int wb, int sub,
                                                    FlipRow<G>& st, uint64_t* lds) {
    const int wi = wb + sub;
    const bool in = wi < a.words64;
    if ((RP && a.mode == DM_RNG_INJECT)) return in ? a.dec.mut_mask[c * a.words64 + wi] : 0ull;
    uint64_t mask = 0;
    if (a.thr_ind >= (1ull << 32)) {
        const int nbits = min(64, a.dim - wi * 64);
        mask = !in ? 0ull : nbits >= 64 ? ~0ull : ((1ull << nbits) - 1);
    } else if (a.thr_ind > 0) {
        flip_chunk_lds<G>(a, c, wb, sub, st, lds);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        mask = lds[sub];
        __builtin_amdgcn_wave_barrier();
    }
    if ((RP && a.mode == DM_RNG_DUMP) && in) a.dec.mut_mask[c * a.words64 + wi] = mask;
    return mask;
}

template <int G, int CX, int MUT, int EC, bool RP>
__global__ __launch_bounds__(256) void gen_bits_kernel(GenArgs a) {
    __shared__ uint64_t flip_lds_all[256];
    uint64_t* flip_lds = flip_lds_all + (threadIdx.x & ~(G - 1));
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const bool leader = sub == 0;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t evals = 0;
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; p < npairs;
         p += gstride) {
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        const bool has1 = c1 < a.nc;
        const int64_t s0 = parent_of<RP>(a, c0, leader);
        const int64_t s1 = has1 ? parent_of<RP>(a, c1, leader) : s0;
        const PairDecisions d = pair_decisions<RP>(a, p, has1, leader);
        const bool inv0 = d.cx || d.mut0 || !a.pvalid[s0];
        const bool inv1 = has1 && (d.cx || d.mut1 || !a.pvalid[s1]);
        const uint64_t* r0 = reinterpret_cast<const uint64_t*>(a.pgenes + s0 * a.pstride);
        const uint64_t* r1 = reinterpret_cast<const uint64_t*>(a.pgenes + s1 * a.pstride);
        uint64_t* w0 = reinterpret_cast<uint64_t*>(a.cgenes + c0 * a.cstride);
        uint64_t* w1 = reinterpret_cast<uint64_t*>(a.cgenes + c1 * a.cstride);
        int64_t pc0 = 0, pc1 = 0;
        FlipRow<G> fr0, fr1;
        if (MUT == DM_MUT_FLIPBIT) {
            if (d.mut0) flip_begin<G>(a, c0, sub, fr0);
            if (d.mut1) flip_begin<G>(a, c1, sub, fr1);
        }
        for (int wb = 0; wb < a.words64; wb += G) {
            const int wi = wb + sub;
            uint64_t f0 = 0, f1 = 0;  // flip masks: every lane of the group takes part
            if (MUT == DM_MUT_FLIPBIT) {
                if (d.mut0) f0 = flip_mask_chunk<G, RP>(a, c0, wb, sub, fr0, flip_lds);
                if (d.mut1) f1 = flip_mask_chunk<G, RP>(a, c1, wb, sub, fr1, flip_lds);
            }
            if (wi < a.words64) {
                uint64_t x0 = r0[wi];
                uint64_t x1 = has1 ? r1[wi] : 0ull;
                if (CX == DM_CX_TWOPOINT && d.cx) {
                    const uint64_t m = range_mask(d.c1 - wi * 64, d.c2 - wi * 64);
                    const uint64_t t = (x0 ^ x1) & m;
                    x0 ^= t;
                    x1 ^= t;
                }
                x0 ^= f0;
                x1 ^= f1;
                __builtin_nontemporal_store(x0, &w0[wi]);
                if (has1) __builtin_nontemporal_store(x1, &w1[wi]);
                pc0 += __popcll(x0);
                pc1 += __popcll(x1);
            }
        }
        if (EC != EC_NONE) {
            pc0 = group_sum_i<G>(pc0);
            pc1 = group_sum_i<G>(pc1);
        }
        if (leader) {
            const int m = a.nobj;
            const bool do_eval = EC != EC_NONE;
            for (int o = 0; o < m; ++o) {
                a.cwv[c0 * m + o] =
                    (do_eval && inv0) ? (double)pc0 * a.ev.weights[o] : a.pwv[s0 * m + o];
                if (has1)
                    a.cwv[c1 * m + o] =
                        (do_eval && inv1) ? (double)pc1 * a.ev.weights[o] : a.pwv[s1 * m + o];
            }
            a.cvalid[c0] = do_eval ? 1 : (inv0 ? 0 : 1);
            if (has1) a.cvalid[c1] = do_eval ? 1 : (inv1 ? 0 : 1);
            evals += (int64_t)inv0 + (int64_t)inv1;
        }
    }
    if (a.nevals && EC != EC_NONE) {
        int64_t tot = evals;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)a.nevals, (unsigned long long)tot);
    }
}

void launch_gen_f64_native(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s);
void launch_gen_f64_replay(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s);
void launch_gen_f32_native(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s);
void launch_gen_f32_replay(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s);
void launch_gen_bits(const GenArgs& a, int ec, int G, dim3 grid, hipStream_t s);

}  // namespace dm
