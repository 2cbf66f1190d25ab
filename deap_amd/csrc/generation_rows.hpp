// generation_rows.hpp — the hot-path variant of the fused generation kernel
// (native RNG, float genomes, one wave per offspring pair, dim <= 256*NCH).
//
// Differences from the streaming kernel in generation.hpp (same results,
// same decisions — the Philox words come from the same counters):
//  * every per-pair decision is drawn lane-parallel: lanes [0,t) draw child
//    0's tournament aspirants, lanes [32,32+t) child 1's, lanes 30/31 the
//    crossover flag and cut draws, lanes 62/63 the two mutation flags — one
//    Philox latency per pair instead of ~8 sequential ones; aspirant fitnesses
//    are fetched by their own lane and the first-wins max is a shuffle scan;
//  * both parent rows are loaded whole (NCH chunks of 4 genes per lane) before
//    any compute, so 2 x 8 KB per wave are in flight while the previous
//    pair's stores drain — the kernel streams HBM instead of alternating
//    load / compute phases.
#pragma once
#include "generation.hpp"

namespace dm {

// Which lanes draw what (requires tournsize <= 30).
constexpr int LANE_CX0 = 30, LANE_CX1 = 31, LANE_MUT0 = 62, LANE_MUT1 = 63;

__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, 64); }

template <typename T, int NCH, int CX, int MUT, int EC>
#ifndef DM_ROWS_MINWAVES
#define DM_ROWS_MINWAVES 2
#endif
__global__ __launch_bounds__(256, DM_ROWS_MINWAVES) void gen_rows_kernel(GenArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t npairs = (a.nc + 1) / 2;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int t = a.tournsize;
    const bool tourn = a.sel == DM_SEL_TOURNAMENT;
    const int m = a.nobj;
    int64_t evals = 0;
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < npairs;
         p += nwaves) {
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        const bool has1 = c1 < a.nc;
        // ---- lane-parallel decisions -------------------------------------
        const int half = lane >> 5, j = lane & 31;
        uint32_t stage, item, subc;
        if (j < t) {
            stage = ST_SEL;
            item = (uint32_t)(half ? c1 : c0);
            subc = (uint32_t)(j >> 1);
        } else if (lane == LANE_CX0 || lane == LANE_CX1) {
            stage = ST_CX;
            item = (uint32_t)p;
            subc = (uint32_t)(lane - LANE_CX0);
        } else {  // LANE_MUT0 / LANE_MUT1 (and idle lanes, harmless)
            stage = ST_MUT;
            item = (uint32_t)(lane == LANE_MUT1 ? c1 : c0);
            subc = 0;
        }
        const u32x4 w = a.rng(stage, item, subc);
        int64_t cand = 0;
        double fa = 0.0;
        if (j < t) {
            cand = (j & 1) ? bounded64(w.z, w.w, (uint32_t)a.np) : bounded64(w.x, w.y, (uint32_t)a.np);
            if (tourn && m == 1) fa = a.pwv[cand];
        }
        int64_t s0, s1;
        if (!tourn) {  // selRandom: one aspirant
            s0 = __shfl((int)cand, 0, 64);
            s1 = __shfl((int)cand, 32, 64);
        } else if (m == 1) {
            // first-drawn aspirant wins ties: replace only on fit_gt (selection.py:68)
            int b0 = 0, b1 = 0;
            double f0 = shfl_d(fa, 0), f1 = shfl_d(fa, 32);
            for (int k = 1; k < t; ++k) {
                const double x0 = shfl_d(fa, k), x1 = shfl_d(fa, 32 + k);
                if (!(x0 <= f0)) {
                    f0 = x0;
                    b0 = k;
                }
                if (!(x1 <= f1)) {
                    f1 = x1;
                    b1 = k;
                }
            }
            s0 = __shfl((int)cand, b0, 64);
            s1 = __shfl((int)cand, 32 + b1, 64);
        } else {
            int b0 = 0, b1 = 0;
            for (int k = 1; k < t; ++k) {
                const int64_t k0 = __shfl((int)cand, k, 64), bb0 = __shfl((int)cand, b0, 64);
                const int64_t k1 = __shfl((int)cand, 32 + k, 64), bb1 = __shfl((int)cand, 32 + b1, 64);
                if (fit_gt(a.pwv + k0 * m, a.pwv + bb0 * m, m)) b0 = k;
                if (fit_gt(a.pwv + k1 * m, a.pwv + bb1 * m, m)) b1 = k;
            }
            s0 = __shfl((int)cand, b0, 64);
            s1 = __shfl((int)cand, 32 + b1, 64);
        }
        if (!has1) s1 = s0;
        bool cx = false;
        int32_t cp1 = 0, cp2 = 0;
        if (CX != DM_CX_NONE && has1) {
            const uint32_t wx = __shfl(w.x, LANE_CX0, 64);
            cx = (uint64_t)wx < a.thr_cx;
            if (CX == DM_CX_TWOPOINT && cx) {
                const uint32_t z0 = __shfl(w.z, LANE_CX0, 64), z1 = __shfl(w.w, LANE_CX0, 64);
                const uint32_t q0 = __shfl(w.x, LANE_CX1, 64), q1 = __shfl(w.y, LANE_CX1, 64);
                int32_t r1 = 1 + (int32_t)bounded64(z0, z1, (uint32_t)a.dim);
                int32_t r2 = 1 + (int32_t)bounded64(q0, q1, (uint32_t)(a.dim - 1));
                if (r2 >= r1) {
                    r2 += 1;
                } else {
                    const int32_t tt = r1;
                    r1 = r2;
                    r2 = tt;
                }
                cp1 = r1;
                cp2 = r2;
            }
        }
        bool mut0 = false, mut1 = false;
        if (MUT != DM_MUT_NONE) {
            mut0 = (uint64_t)__shfl(w.x, LANE_MUT0, 64) < a.thr_mut;
            mut1 = has1 && (uint64_t)__shfl(w.x, LANE_MUT1, 64) < a.thr_mut;
        }
        const bool inv0 = cx || mut0 || !a.pvalid[s0];
        const bool inv1 = has1 && (cx || mut1 || !a.pvalid[s1]);

        // ---- whole parent rows in flight ----------------------------------
        const char* r0 = a.pgenes + s0 * a.pstride;
        const char* r1 = a.pgenes + s1 * a.pstride;
        double y0[NCH][4], y1[NCH][4];
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int g = ch * 256 + 4 * lane;
            if (g < a.dim) {
                Vec4<T>::load(r0, g, y0[ch]);
                Vec4<T>::load(r1, g, y1[ch]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) y0[ch][k] = y1[ch][k] = 0.0;
            }
        }
        char* w0 = a.cgenes + c0 * a.cstride;
        char* w1 = a.cgenes + c1 * a.cstride;
        EvalState e0, e1;
        eval_init(e0);
        eval_init(e1);
        const double gamma_scale = 1.0 + 2.0 * a.alpha;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int cbase = ch * 256;
            const int g = cbase + 4 * lane;
            const bool in = g < a.dim;
            double (&x0)[4] = y0[ch];
            double (&x1)[4] = y1[ch];
            if (CX == DM_CX_BLEND && cx && in) {
                const u32x4 u = a.rng(ST_BLEND, (uint32_t)p, (uint32_t)(g >> 2));
                const uint32_t us[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (g + k < a.dim) {
                        const double gm = gamma_scale * u01_32(us[k]) - a.alpha;
                        const double v1 = x0[k], v2 = x1[k];
                        x0[k] = (1.0 - gm) * v1 + gm * v2;
                        x1[k] = gm * v1 + (1.0 - gm) * v2;
                    }
                }
            } else if (CX == DM_CX_TWOPOINT && cx && in) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (g + k >= cp1 && g + k < cp2) {
                        const double tt = x0[k];
                        x0[k] = x1[k];
                        x1[k] = tt;
                    }
                }
            }
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x0[k] = (double)(float)x0[k];
                    x1[k] = (double)(float)x1[k];
                }
            }
            if (MUT == DM_MUT_GAUSSIAN && in && (mut0 || mut1)) {
                uint32_t bits = 0;
                if (mut0) bits |= gauss_mask<false>(a, c0, g);
                if (mut1) bits |= gauss_mask<false>(a, c1, g) << 4;
                gauss_apply<false>(a, c0, g, bits, x0, x1);
            }
            if (in) {
                Vec4<T>::store_nt(w0, g, x0);
                if (has1) Vec4<T>::store_nt(w1, g, x1);
            }
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    x0[k] = (double)(float)x0[k];
                    x1[k] = (double)(float)x1[k];
                }
            }
            if (EC != EC_NONE) {
                eval_chunk<64, EC>(a.ev, a.dim, g, cbase, x0, inv0, e0);
                eval_chunk<64, EC>(a.ev, a.dim, g, cbase, x1, inv1, e1);
            }
        }
        double f0[DM_MAX_OBJ], f1[DM_MAX_OBJ];
        if (EC != EC_NONE) {
            eval_finish<64, EC>(a.ev, a.dim, e0, f0);
            eval_finish<64, EC>(a.ev, a.dim, e1, f1);
        }
        if (lane == 0) {
            if constexpr (ec_single(EC)) {
                a.cwv[c0] = inv0 ? f0[0] * a.w0 : a.pwv[s0];
                if (has1) a.cwv[c1] = inv1 ? f1[0] * a.w0 : a.pwv[s1];
            } else {
                const bool de = EC != EC_NONE;
                for (int o = 0; o < m; ++o) {
                    a.cwv[c0 * m + o] = (de && inv0) ? f0[o] * a.ev.weights[o] : a.pwv[s0 * m + o];
                    if (has1)
                        a.cwv[c1 * m + o] =
                            (de && inv1) ? f1[o] * a.ev.weights[o] : a.pwv[s1 * m + o];
                }
            }
            const bool de = EC != EC_NONE;
            a.cvalid[c0] = de ? 1 : (inv0 ? 0 : 1);
            if (has1) a.cvalid[c1] = de ? 1 : (inv1 ? 0 : 1);
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

void launch_gen_rows_f64(const GenArgs& a, int ec, int nch, dim3 grid, hipStream_t s);
void launch_gen_rows_f32(const GenArgs& a, int ec, int nch, dim3 grid, hipStream_t s);

}  // namespace dm
