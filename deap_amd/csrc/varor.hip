// varor.hip — varOr (algorithms.py:192-245): lambda offspring, each from
// exactly one of crossover (first child of a random.sample pair), mutation
// (clone of a random.choice) or reproduction (random.choice, not cloned).
// One lane group of G lanes per child; the child row streams through
// registers in chunks of 4 genes per lane like the fused generation kernel.
#include "generation.hpp"

namespace dm {

struct ChildDecisions {
    int op;             // 0 cx, 1 mut, 2 repro
    int64_t a, b;       // parent indices (b only for cx)
    int32_t c1, c2;     // cxTwoPoint slice
};

__device__ __forceinline__ ChildDecisions child_decisions(const GenArgs& a, int64_t c,
                                                          double cxpb, double cxmutpb,
                                                          bool leader) {
    ChildDecisions d{};
    int32_t r1 = 0, r2 = 0;
    if (a.mode == DM_RNG_INJECT) {
        d.op = a.dec.varor_op[c];
        d.a = a.dec.varor_idx[2 * c];
        d.b = a.dec.varor_idx[2 * c + 1];
        if (d.op == 0 && a.cx == DM_CX_TWOPOINT) {
            r1 = a.dec.cx_raw[2 * c];
            r2 = a.dec.cx_raw[2 * c + 1];
        }
    } else {
        const u32x4 w = a.rng(ST_VAROR, (uint32_t)c, 0);
        const u32x4 w2 = a.rng(ST_VAROR, (uint32_t)c, 1);
        const double u = u01_53(w.x, w.y);  // op_choice = random.random()
        d.op = u < cxpb ? 0 : (u < cxmutpb ? 1 : 2);
        const uint32_t n = (uint32_t)a.np;
        d.a = bounded64(w.z, w.w, n);
        d.b = 0;
        if (d.op == 0) {
            // random.sample(population, 2): two distinct indices
            uint32_t b = bounded64(w2.x, w2.y, n - 1);
            if (b >= (uint32_t)d.a) ++b;
            d.b = b;
            if (a.cx == DM_CX_TWOPOINT) {
                const u32x4 w3 = a.rng(ST_CX, (uint32_t)c, 0);
                r1 = 1 + (int32_t)bounded64(w3.x, w3.y, (uint32_t)a.dim);
                r2 = 1 + (int32_t)bounded64(w3.z, w3.w, (uint32_t)(a.dim - 1));
            }
        }
        if (a.mode == DM_RNG_DUMP && leader) {
            a.dec.varor_op[c] = d.op;
            a.dec.varor_idx[2 * c] = (int32_t)d.a;
            a.dec.varor_idx[2 * c + 1] = (int32_t)d.b;
            if (a.dec.cx_raw) {
                a.dec.cx_raw[2 * c] = r1;
                a.dec.cx_raw[2 * c + 1] = r2;
            }
        }
    }
    if (d.op == 0 && a.cx == DM_CX_TWOPOINT) {
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
    return d;
}

template <typename T, int G, int EC>
__global__ __launch_bounds__(256) void varor_float_kernel(GenArgs a, double cxpb, double cxmutpb) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const bool leader = sub == 0;
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t evals = 0;
    for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; c < a.nc; c += gstride) {
        const ChildDecisions d = child_decisions(a, c, cxpb, cxmutpb, leader);
        const bool inv = d.op != 2 || !a.pvalid[d.a];
        const char* ra = a.pgenes + d.a * a.pstride;
        const char* rb = a.pgenes + d.b * a.pstride;
        char* wc = a.cgenes + c * a.cstride;
        EvalState e;
        eval_init(e);
        const double gamma_scale = 1.0 + 2.0 * a.alpha;
        for (int cbase = 0; cbase < a.dim; cbase += 4 * G) {
            const int g = cbase + 4 * sub;
            double y[4] = {0, 0, 0, 0}, x2[4] = {0, 0, 0, 0};
            const bool in = g < a.dim;
            if (in) {
                Vec4<T>::load(ra, g, y);
                if (d.op == 0) Vec4<T>::load(rb, g, x2);
            }
            if (d.op == 0 && in) {
                if (a.cx == DM_CX_BLEND) {
                    double u[4];
                    if (a.mode == DM_RNG_INJECT) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            u[j] = (g + j < a.dim) ? a.dec.blend_u[c * a.dim + g + j] : 0.0;
                    } else {
                        const u32x4 w = gene4_words<T>(a.rng, ST_BLEND, (uint32_t)c, g);
                        u[0] = u01_32(w.x);
                        u[1] = u01_32(w.y);
                        u[2] = u01_32(w.z);
                        u[3] = u01_32(w.w);
                        if (a.mode == DM_RNG_DUMP) {
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (g + j < a.dim) a.dec.blend_u[c * a.dim + g + j] = u[j];
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (g + j < a.dim) {
                            const double gm = gamma_scale * u[j] - a.alpha;
                            y[j] = (1.0 - gm) * y[j] + gm * x2[j];  // first child only
                        }
                    }
                } else if (a.cx == DM_CX_TWOPOINT) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (g + j >= d.c1 && g + j < d.c2) y[j] = x2[j];
                }
            }
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (double)(float)y[j];
            }
            if (d.op == 1 && in && a.mut == DM_MUT_GAUSSIAN) {
                double dummy[4] = {0, 0, 0, 0};
                gauss_apply<true>(a, c, g, gauss_mask<T, true>(a, c, g), y, dummy);
            }
            if (in) Vec4<T>::store(wc, g, y);
            if constexpr (sizeof(T) == 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (double)(float)y[j];
            }
            if (EC != EC_NONE) eval_chunk<G, EC>(a.ev, a.dim, g, cbase, y, inv, e);
        }
        double f[DM_MAX_OBJ];
        if (EC != EC_NONE) eval_finish<G, EC>(a.ev, a.dim, e, f);
        if (leader) {
            const int m = a.nobj;
            for (int o = 0; o < m; ++o)
                a.cwv[c * m + o] =
                    (EC != EC_NONE && inv) ? f[o] * a.ev.weights[o] : a.pwv[d.a * m + o];
            a.cvalid[c] = EC != EC_NONE ? 1 : (inv ? 0 : 1);
            evals += inv;
        }
    }
    if (a.nevals && EC != EC_NONE) {
        int64_t tot = evals;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)a.nevals, (unsigned long long)tot);
    }
}

template <int G>
__global__ __launch_bounds__(256) void varor_bits_kernel(GenArgs a, double cxpb, double cxmutpb) {
    __shared__ uint64_t flip_lds_all[256];
    uint64_t* flip_lds = flip_lds_all + (threadIdx.x & ~(G - 1));
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const bool leader = sub == 0;
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t evals = 0;
    const bool do_eval = a.eval_fn != DM_EVAL_NONE;
    for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; c < a.nc; c += gstride) {
        const ChildDecisions d = child_decisions(a, c, cxpb, cxmutpb, leader);
        const bool inv = d.op != 2 || !a.pvalid[d.a];
        const uint64_t* ra = reinterpret_cast<const uint64_t*>(a.pgenes + d.a * a.pstride);
        const uint64_t* rb = reinterpret_cast<const uint64_t*>(a.pgenes + d.b * a.pstride);
        uint64_t* wc = reinterpret_cast<uint64_t*>(a.cgenes + c * a.cstride);
        int64_t pc = 0;
        const bool flip = d.op == 1 && a.mut == DM_MUT_FLIPBIT;  // group-uniform
        FlipRow<G> fr;
        if (flip) flip_begin<G>(a, c, sub, fr);
        for (int wb = 0; wb < a.words64; wb += G) {
            const int wi = wb + sub;
            const uint64_t fm = flip ? flip_mask_chunk<G, true>(a, c, wb, sub, fr, flip_lds) : 0ull;
            if (wi >= a.words64) continue;
            uint64_t x = ra[wi];
            if (d.op == 0 && a.cx == DM_CX_TWOPOINT) {
                const uint64_t m = range_mask(d.c1 - wi * 64, d.c2 - wi * 64);
                x = (x & ~m) | (rb[wi] & m);
            }
            x ^= fm;
            wc[wi] = x;
            pc += __popcll(x);
        }
        pc = group_sum_i<G>(pc);
        if (leader) {
            const int m = a.nobj;
            for (int o = 0; o < m; ++o)
                a.cwv[c * m + o] = (do_eval && inv) ? (double)pc * a.ev.weights[o] : a.pwv[d.a * m + o];
            a.cvalid[c] = do_eval ? 1 : (inv ? 0 : 1);
            evals += inv;
        }
    }
    if (a.nevals && do_eval) {
        int64_t tot = evals;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)a.nevals, (unsigned long long)tot);
    }
}

int validate_pop(const dm_pop* p, const char* what);
int validate_eval(const dm_eval* ev, const dm_pop* p);
int validate_variation(const dm_variation* v, const dm_pop* p);

template <typename T, int G>
static void launch_varor_float(const GenArgs& a, int ec, dim3 grid, hipStream_t s, double cxpb,
                               double cxmutpb) {
    if (ec_single(ec))
        varor_float_kernel<T, G, EC_SUM><<<grid, 256, 0, s>>>(a, cxpb, cxmutpb);
    else if (ec == EC_MO)
        varor_float_kernel<T, G, EC_MO><<<grid, 256, 0, s>>>(a, cxpb, cxmutpb);
    else
        varor_float_kernel<T, G, EC_NONE><<<grid, 256, 0, s>>>(a, cxpb, cxmutpb);
}

}  // namespace dm

using namespace dm;

extern "C" int dm_var_or(dm_ctx* ctx, const dm_pop* parents, dm_pop* children,
                         const dm_variation* var, const dm_eval* ev, dm_rng rng, int32_t mode,
                         const dm_decisions* dec, int64_t* nevals) {
    DM_CHECK_ARG(ctx && parents && children && var, "null argument");
    int rc;
    if ((rc = validate_pop(parents, "parents")) || (rc = validate_pop(children, "children")))
        return rc;
    DM_CHECK_ARG(parents->gtype == children->gtype && parents->dim == children->dim &&
                     parents->nobj == children->nobj,
                 "parents and children must share genome type, dim and nobj");
    DM_CHECK_ARG(parents->genes != children->genes, "children must not alias parents");
    // assert (cxpb + mutpb) <= 1.0                                  (algorithms.py:225-227)
    DM_CHECK_ARG(var->cxpb + var->mutpb <= 1.0,
                 "The sum of the crossover and mutation probabilities must be smaller or equal "
                 "to 1.0.");
    if ((rc = validate_variation(var, parents))) return rc;
    dm_eval none{};
    if (!ev) ev = &none;
    if ((rc = validate_eval(ev, parents))) return rc;
    DM_CHECK_ARG(mode >= DM_RNG_NATIVE && mode <= DM_RNG_DUMP, "bad rng mode");
    DM_CHECK_ARG(parents->n < (1ll << 31), "population too large");
    if (children->n == 0) return DM_OK;
    DM_CHECK_ARG(parents->n >= 1, "cannot vary an empty population");
    if (var->cxpb > 0.0)
        DM_CHECK_ARG(parents->n >= 2, "random.sample needs at least 2 individuals");
    dm_decisions d{};
    if (dec) d = *dec;
    if (mode != DM_RNG_NATIVE) {
        DM_CHECK_ARG(dec && d.varor_op && d.varor_idx, "decisions.varor_op/varor_idx required");
        if (var->cx == DM_CX_TWOPOINT && mode == DM_RNG_INJECT)
            DM_CHECK_ARG(d.cx_raw, "decisions.cx_raw required");
        if (var->cx == DM_CX_BLEND) DM_CHECK_ARG(d.blend_u, "decisions.blend_u required");
        if (var->mut != DM_MUT_NONE) DM_CHECK_ARG(d.mut_mask, "decisions.mut_mask required");
        if (var->mut == DM_MUT_GAUSSIAN) DM_CHECK_ARG(d.gauss, "decisions.gauss required");
    }
    if (mode == DM_RNG_DUMP && var->mut == DM_MUT_GAUSSIAN)
        DM_HIP(hipMemsetAsync(d.mut_mask, 0,
                              (size_t)children->n * ((parents->dim + 63) / 64) * 8, ctx->stream));

    GenArgs a{};
    a.pgenes = (const char*)parents->genes;
    a.pwv = parents->wvalues;
    a.pvalid = parents->valid;
    a.np = parents->n;
    a.pstride = parents->stride;
    a.cgenes = (char*)children->genes;
    a.cwv = children->wvalues;
    a.cvalid = children->valid;
    a.nc = children->n;
    a.cstride = children->stride;
    a.dim = parents->dim;
    a.nobj = parents->nobj;
    a.words64 = (parents->dim + 63) / 64;
    a.cx = var->cx;
    a.mut = var->mut;
    a.thr_ind = prob_threshold(var->indpb);
    a.alpha = var->alpha;
    a.indpb = var->indpb;
    a.mu = var->mu;
    a.sigma = var->sigma;
    a.mu_vec = var->mu_vec;
    a.sigma_vec = var->sigma_vec;
    a.flip_inv_log2 = (var->indpb > 0.0 && var->indpb < 1.0)
                          ? (float)(1.0 / std::log2(1.0 - var->indpb))
                          : 0.0f;
    a.eval_fn = ev->fn;
    a.w0 = ev->weights[0];
    a.ev = *ev;
    a.rng = Rng(rng);
    a.zig = ctx->zig;
    a.mode = mode;
    a.dec = d;
    a.nevals = nevals;
    const double cxpb = var->cxpb, cxmutpb = var->cxpb + var->mutpb;
    const int ec = eval_class(ev->fn);
    hipStream_t s = ctx->stream;
    auto grid_of = [&](int G) {
        int64_t b = (children->n + (256 / G) - 1) / (256 / G);
        b = std::min<int64_t>(std::max<int64_t>(b, 1), (int64_t)ctx->num_cus * 16);
        return dim3((unsigned)b);
    };
    if (parents->gtype == DM_BITS) {
        const int G = a.words64 <= 2 ? 2 : a.words64 <= 8 ? 8 : 64;
        if (G == 2) varor_bits_kernel<2><<<grid_of(2), 256, 0, s>>>(a, cxpb, cxmutpb);
        else if (G == 8) varor_bits_kernel<8><<<grid_of(8), 256, 0, s>>>(a, cxpb, cxmutpb);
        else varor_bits_kernel<64><<<grid_of(64), 256, 0, s>>>(a, cxpb, cxmutpb);
    } else {
        const int q = (parents->dim + 3) / 4;
        const int G = q <= 4 ? 4 : q <= 16 ? 16 : 64;
        if (parents->gtype == DM_F64) {
            if (G == 4) launch_varor_float<double, 4>(a, ec, grid_of(4), s, cxpb, cxmutpb);
            else if (G == 16) launch_varor_float<double, 16>(a, ec, grid_of(16), s, cxpb, cxmutpb);
            else launch_varor_float<double, 64>(a, ec, grid_of(64), s, cxpb, cxmutpb);
        } else {
            if (G == 4) launch_varor_float<float, 4>(a, ec, grid_of(4), s, cxpb, cxmutpb);
            else if (G == 16) launch_varor_float<float, 16>(a, ec, grid_of(16), s, cxpb, cxmutpb);
            else launch_varor_float<float, 64>(a, ec, grid_of(64), s, cxpb, cxmutpb);
        }
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}
