// bounded.hip — the variation body of DEAP's NSGA-II loop
// (examples/ga/nsga2.py:96-105): clone the selected parents, simulated binary
// bounded crossover of consecutive pairs (crossover.py:291-360) and bounded
// polynomial mutation of both children (mutation.py:51-95), fitness deleted.
//
// Once its random() values are fixed every gene of a pair is independent of
// the others, so the kernel runs one lane per (pair, gene): the lane loads the
// two parent genes, applies SBX, mutates both child genes and stores them.
// Consecutive lanes cover consecutive genes of a pair, so the two gathered
// parent rows are read and the two child rows written in whole lines.
// HBM per pair: 2 rows in + 2 rows out (+ the decision arrays in replay modes).
#include "common.hpp"

namespace dm {

struct BoundedArgs {
    const char* pgenes;
    const double* pwv;
    const uint8_t* pvalid;
    int64_t np, pstride;
    const int32_t* idx;
    char* cgenes;
    double* cwv;
    uint8_t* cvalid;
    int64_t nc, cstride;
    int64_t pairs, units;  // units = pairs + (nc odd)
    int dim, nobj;
    int cx, mut;
    double cxpb, eta_cx, eta_mut, indpb, low, up;
    const double* low_vec;
    const double* up_vec;
    Rng rng;
    int mode;
    double* cx_u;
    double* sbx_u;
    double* mut_u;
};

// beta_q of crossover.py:334-338 / :343-347 (Python `**` = libm pow).
__device__ __forceinline__ double sbx_beta_q(double beta, double rand, double eta) {
    const double alpha = 2.0 - pow(beta, -(eta + 1.0));
    if (rand <= 1.0 / alpha) return pow(rand * alpha, 1.0 / (eta + 1.0));
    return pow(1.0 / (2.0 - rand * alpha), 1.0 / (eta + 1.0));
}

// min(max(c, xl), xu) with Python's builtin semantics: max(c, xl) keeps c
// unless xl > c; min(., xu) keeps it unless xu < it (NaN stays NaN).
__device__ __forceinline__ double py_clamp(double c, double xl, double xu) {
    if (xl > c) c = xl;
    if (xu < c) c = xu;
    return c;
}

// mutation.py:76-94 for one gene whose gate random() passed.
__device__ __forceinline__ double poly_mutate(double x, double xl, double xu, double rand,
                                              double eta) {
    const double delta_1 = (x - xl) / (xu - xl);
    const double delta_2 = (xu - x) / (xu - xl);
    const double mut_pow = 1.0 / (eta + 1.0);
    double delta_q;
    if (rand < 0.5) {
        const double xy = 1.0 - delta_1;
        const double val = 2.0 * rand + (1.0 - 2.0 * rand) * pow(xy, eta + 1.0);
        delta_q = pow(val, mut_pow) - 1.0;
    } else {
        const double xy = 1.0 - delta_2;
        const double val = 2.0 * (1.0 - rand) + 2.0 * (rand - 0.5) * pow(xy, eta + 1.0);
        delta_q = 1.0 - pow(val, mut_pow);
    }
    x = x + delta_q * (xu - xl);
    return py_clamp(x, xl, xu);
}

// Per-gene (gate, rand) of the polynomial mutation of child c.
__device__ __forceinline__ void poly_draw(const BoundedArgs& a, int64_t c, int g, double& gate,
                                          double& rand) {
    double* slot = a.mut_u + ((size_t)c * a.dim + g) * 2;
    if (a.mode == DM_RNG_INJECT) {
        gate = slot[0];
        rand = slot[1];
        return;
    }
    const u32x4 w = a.rng(ST_POLY, (uint32_t)c, (uint32_t)g);
    gate = u01_53(w.x, w.y);
    rand = u01_53(w.z, w.w);
    if (a.mode == DM_RNG_DUMP) {
        slot[0] = gate;
        slot[1] = rand;
    }
}

__global__ __launch_bounds__(256) void bounded_vary_kernel(BoundedArgs a) {
    const int64_t total = a.units * a.dim;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += step) {
        const int64_t p = t / a.dim;
        const int g = (int)(t - p * a.dim);
        const int64_t c0 = 2 * p, c1 = 2 * p + 1;
        int64_t s0 = a.idx ? a.idx[c0] : c0;
        double* w0 = reinterpret_cast<double*>(a.cgenes + c0 * a.cstride);
        // out-of-range selection index: never read outside the parent rows;
        // the child becomes NaN + invalid (the host layer raises IndexError
        // for host-side indices before launching)
        bool bad = s0 < 0 || s0 >= a.np;
        if (p < a.pairs) {
            const int64_t s1c = a.idx ? a.idx[c1] : c1;
            bad = bad || s1c < 0 || s1c >= a.np;
        }
        if (bad) {
            w0[g] = __builtin_nan("");
            if (p < a.pairs) reinterpret_cast<double*>(a.cgenes + c1 * a.cstride)[g] = __builtin_nan("");
            if (g == 0) {
                a.cvalid[c0] = 0;
                if (p < a.pairs) a.cvalid[c1] = 0;
            }
            continue;
        }
        const double x0 = reinterpret_cast<const double*>(a.pgenes + s0 * a.pstride)[g];
        if (p == a.pairs) {
            // odd last offspring: outside zip(offspring[::2], offspring[1::2]) a
            // plain clone (fitness kept); mutation-only (the batch form of
            // mutPolynomialBounded) mutates it like every other individual.
            const bool mutate = a.mut && !a.cx;
            double y = x0;
            if (mutate) {
                const double xl = a.low_vec ? a.low_vec[g] : a.low;
                const double xu = a.up_vec ? a.up_vec[g] : a.up;
                double gate, rand;
                poly_draw(a, c0, g, gate, rand);
                if (gate <= a.indpb) y = poly_mutate(y, xl, xu, rand, a.eta_mut);
            }
            w0[g] = y;
            if (g == 0) {
                for (int o = 0; o < a.nobj; ++o) a.cwv[c0 * a.nobj + o] = a.pwv[s0 * a.nobj + o];
                a.cvalid[c0] = mutate ? 0 : a.pvalid[s0];
            }
            continue;
        }
        const int64_t s1 = a.idx ? a.idx[c1] : c1;
        double* w1 = reinterpret_cast<double*>(a.cgenes + c1 * a.cstride);
        double y0 = x0;
        double y1 = reinterpret_cast<const double*>(a.pgenes + s1 * a.pstride)[g];
        const double xl = a.low_vec ? a.low_vec[g] : a.low;
        const double xu = a.up_vec ? a.up_vec[g] : a.up;

        if (a.cx) {
            // if random.random() <= CXPB                              (nsga2.py:100)
            double ucx;
            if (a.mode == DM_RNG_INJECT) {
                ucx = a.cx_u[p];
            } else {
                const u32x4 w = a.rng(ST_SBX_PAIR, (uint32_t)p, 0);
                ucx = u01_53(w.x, w.y);
                if (a.mode == DM_RNG_DUMP && g == 0) a.cx_u[p] = ucx;
            }
            if (ucx <= a.cxpb) {
                double* slot = a.sbx_u ? a.sbx_u + ((size_t)p * a.dim + g) * 3 : nullptr;
                double gate, rand, swap;
                if (a.mode == DM_RNG_INJECT) {
                    gate = slot[0];
                    rand = slot[1];
                    swap = slot[2];
                } else {
                    const u32x4 w = a.rng(ST_SBX, (uint32_t)p, (uint32_t)g);
                    const u32x4 v = a.rng(ST_SBX, (uint32_t)p, (uint32_t)g | (1u << 24));
                    gate = u01_53(w.x, w.y);
                    rand = u01_53(w.z, w.w);
                    swap = u01_53(v.x, v.y);
                    if (a.mode == DM_RNG_DUMP) {
                        slot[0] = gate;
                        slot[1] = rand;
                        slot[2] = swap;
                    }
                }
                // crossover.py:325-358
                if (gate <= 0.5 && fabs(y0 - y1) > 1e-14) {
                    const double x1 = (y1 < y0) ? y1 : y0;  // min(ind1[i], ind2[i])
                    const double x2 = (y1 > y0) ? y1 : y0;  // max(ind1[i], ind2[i])
                    double beta = 1.0 + (2.0 * (x1 - xl) / (x2 - x1));
                    double bq = sbx_beta_q(beta, rand, a.eta_cx);
                    double ca = 0.5 * (x1 + x2 - bq * (x2 - x1));
                    beta = 1.0 + (2.0 * (xu - x2) / (x2 - x1));
                    bq = sbx_beta_q(beta, rand, a.eta_cx);
                    double cb = 0.5 * (x1 + x2 + bq * (x2 - x1));
                    ca = py_clamp(ca, xl, xu);
                    cb = py_clamp(cb, xl, xu);
                    if (swap <= 0.5) {
                        y0 = cb;
                        y1 = ca;
                    } else {
                        y0 = ca;
                        y1 = cb;
                    }
                }
            }
        }
        if (a.mut) {
            // toolbox.mutate(ind1); toolbox.mutate(ind2)       (nsga2.py:103-104)
            double gate, rand;
            poly_draw(a, c0, g, gate, rand);
            if (gate <= a.indpb) y0 = poly_mutate(y0, xl, xu, rand, a.eta_mut);
            poly_draw(a, c1, g, gate, rand);
            if (gate <= a.indpb) y1 = poly_mutate(y1, xl, xu, rand, a.eta_mut);
        }
        w0[g] = y0;
        w1[g] = y1;
        if (g == 0) {  // del ind1.fitness.values, ind2.fitness.values  (nsga2.py:105)
            for (int o = 0; o < a.nobj; ++o) {
                a.cwv[c0 * a.nobj + o] = a.pwv[s0 * a.nobj + o];
                a.cwv[c1 * a.nobj + o] = a.pwv[s1 * a.nobj + o];
            }
            a.cvalid[c0] = 0;
            a.cvalid[c1] = 0;
        }
    }
}

int validate_pop(const dm_pop* p, const char* what);

}  // namespace dm

using namespace dm;

extern "C" int dm_vary_bounded(dm_ctx* ctx, const dm_pop* parents, const int32_t* idx,
                               dm_pop* children, const dm_bounded_var* var, dm_rng rng,
                               int32_t mode, double* cx_u, double* sbx_u, double* mut_u) {
    DM_CHECK_ARG(ctx && parents && children && var, "null argument");
    int rc;
    if ((rc = validate_pop(parents, "parents")) || (rc = validate_pop(children, "children")))
        return rc;
    if (parents->gtype != DM_F64) {
        set_error("cxSimulatedBinaryBounded / mutPolynomialBounded need f64 genomes");
        return DM_ERR_UNSUPPORTED;
    }
    DM_CHECK_ARG(parents->gtype == children->gtype && parents->dim == children->dim &&
                     parents->nobj == children->nobj,
                 "parents and children must share genome type, dim and nobj");
    DM_CHECK_ARG(parents->genes != children->genes, "children must not alias parents");
    DM_CHECK_ARG(mode >= DM_RNG_NATIVE && mode <= DM_RNG_DUMP, "bad rng mode");
    DM_CHECK_ARG(var->cx == 0 || var->cx == 1, "bad cx flag %d", var->cx);
    DM_CHECK_ARG(var->mut == 0 || var->mut == 1, "bad mut flag %d", var->mut);
    DM_CHECK_ARG(children->n < (1ll << 31) && parents->n < (1ll << 31), "population too large");
    if (children->n == 0 || parents->dim == 0) return DM_OK;
    DM_CHECK_ARG(idx || children->n <= parents->n,
                 "identity variation needs children->n <= parents->n");
    DM_CHECK_ARG(parents->n >= 1, "cannot vary an empty population");
    if (mode != DM_RNG_NATIVE) {
        if (var->cx) DM_CHECK_ARG(cx_u && sbx_u, "decisions cx_u / sbx_u required");
        if (var->mut) DM_CHECK_ARG(mut_u, "decisions mut_u required");
    }

    BoundedArgs a{};
    a.pgenes = (const char*)parents->genes;
    a.pwv = parents->wvalues;
    a.pvalid = parents->valid;
    a.np = parents->n;
    a.pstride = parents->stride;
    a.idx = idx;
    a.cgenes = (char*)children->genes;
    a.cwv = children->wvalues;
    a.cvalid = children->valid;
    a.nc = children->n;
    a.cstride = children->stride;
    a.pairs = children->n / 2;
    a.units = a.pairs + (children->n & 1);
    a.dim = parents->dim;
    a.nobj = parents->nobj;
    a.cx = var->cx;
    a.mut = var->mut;
    a.cxpb = var->cxpb;
    a.eta_cx = var->eta_cx;
    a.eta_mut = var->eta_mut;
    a.indpb = var->indpb;
    a.low = var->low;
    a.up = var->up;
    a.low_vec = var->low_vec;
    a.up_vec = var->up_vec;
    a.rng = Rng(rng);
    a.mode = mode;
    a.cx_u = cx_u;
    a.sbx_u = sbx_u;
    a.mut_u = mut_u;
    const int64_t total = a.units * a.dim;
    int64_t blocks = (total + 255) / 256;
    blocks = std::min<int64_t>(std::max<int64_t>(blocks, 1), (int64_t)ctx->num_cus * 32);
    bounded_vary_kernel<<<dim3((unsigned)blocks), 256, 0, ctx->stream>>>(a);
    DM_LAUNCH_CHECK();
    return DM_OK;
}
