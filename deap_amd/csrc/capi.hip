// capi.hip — context, errors, validation, RNG/init, evaluation, selection
// and gather entry points of libdeapmi.
#include <stdarg.h>
#include <stdio.h>

#include "common.hpp"
#include "evals.hpp"

namespace dm {

// Layer edges of the 256-layer normal ziggurat: equal-area (V) layers under
// f(x) = exp(-x^2/2), R = 3.6541528853610088 (Marsaglia & Tsang 2000).
int zig_make_tables(double* t) {
    const double R = 3.6541528853610088, V = 0.00492867323399;
    double* x = t;
    double* f = t + (ZIG_N + 1);
    x[0] = V / std::exp(-0.5 * R * R);
    x[1] = R;
    for (int i = 2; i < ZIG_N; ++i)
        x[i] = std::sqrt(-2.0 * std::log(V / x[i - 1] + std::exp(-0.5 * x[i - 1] * x[i - 1])));
    x[ZIG_N] = 0.0;
    for (int i = 0; i <= ZIG_N; ++i) f[i] = std::exp(-0.5 * x[i] * x[i]);
    return DM_OK;
}

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void* scratch_slot(dm_ctx* ctx, int slot, size_t bytes) {
    bytes = align_up(std::max<size_t>(bytes, 256), 256);
    if (bytes <= ctx->scratch_bytes[slot]) return ctx->scratch[slot];
    if (ctx->scratch[slot]) {
        // the stream may still use the old arena
        if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
            hipFree(ctx->scratch[slot]) != hipSuccess) {
            set_error("scratch release failed");
            return nullptr;
        }
        ctx->scratch[slot] = nullptr;
        ctx->scratch_bytes[slot] = 0;
    }
    if (hipMalloc(&ctx->scratch[slot], bytes) != hipSuccess) {
        set_error("hipMalloc(%zu) for scratch slot %d failed", bytes, slot);
        ctx->scratch[slot] = nullptr;
        return nullptr;
    }
    ctx->scratch_bytes[slot] = bytes;
    return ctx->scratch[slot];
}

void* pinned(dm_ctx* ctx, size_t bytes) {
    bytes = align_up(std::max<size_t>(bytes, 256), 256);
    if (bytes <= ctx->pinned_bytes) return ctx->pinned;
    if (ctx->pinned) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
    }
    if (hipHostMalloc(&ctx->pinned, bytes, hipHostMallocDefault) != hipSuccess) {
        set_error("hipHostMalloc(%zu) failed", bytes);
        ctx->pinned = nullptr;
        return nullptr;
    }
    ctx->pinned_bytes = bytes;
    return ctx->pinned;
}

int validate_pop(const dm_pop* p, const char* what) {
    DM_CHECK_ARG(p != nullptr, "%s: null population", what);
    DM_CHECK_ARG(p->n >= 0, "%s: negative size", what);
    DM_CHECK_ARG(p->gtype == DM_BITS || p->gtype == DM_F32 || p->gtype == DM_F64,
                 "%s: bad genome type %d", what, p->gtype);
    DM_CHECK_ARG(p->dim >= 1, "%s: dim must be >= 1", what);
    DM_CHECK_ARG(p->nobj >= 1 && p->nobj <= DM_MAX_OBJ, "%s: nobj must be in [1, %d]", what,
                 DM_MAX_OBJ);
    DM_CHECK_ARG(p->stride % 16 == 0, "%s: row stride must be a multiple of 16", what);
    const int64_t need = p->gtype == DM_BITS ? (int64_t)((p->dim + 63) / 64) * 8
                         : p->gtype == DM_F32 ? (int64_t)((p->dim + 3) / 4) * 16
                                              : (int64_t)((p->dim + 3) / 4) * 32;
    DM_CHECK_ARG(p->stride >= need, "%s: row stride %lld < %lld bytes needed", what,
                 (long long)p->stride, (long long)need);
    if (p->n > 0)
        DM_CHECK_ARG(p->genes && p->wvalues && p->valid, "%s: null device buffer", what);
    return DM_OK;
}

int validate_eval(const dm_eval* ev, const dm_pop* p) {
    if (ev->fn == DM_EVAL_NONE) return DM_OK;
    DM_CHECK_ARG(ev->fn >= DM_EVAL_ONEMAX && ev->fn <= DM_EVAL_SPHERE, "bad eval fn %d", ev->fn);
    if (p->gtype == DM_BITS)
        DM_CHECK_ARG(ev->fn == DM_EVAL_ONEMAX, "packed-bit genomes support only OneMax");
    const int m = eval_nobj(*ev);
    DM_CHECK_ARG(m == p->nobj, "objective returns %d values but the fitness has %d weights", m,
                 p->nobj);
    if (ev->fn >= DM_EVAL_DTLZ1 && ev->fn <= DM_EVAL_DTLZ4) {
        DM_CHECK_ARG(ev->obj >= 2 && ev->obj <= DM_MAX_OBJ, "DTLZ obj must be in [2, %d]",
                     DM_MAX_OBJ);
        DM_CHECK_ARG(p->dim >= ev->obj, "DTLZ needs at least obj genes");
        DM_CHECK_ARG(ev->obj - 1 <= 8, "DTLZ supports at most 9 objectives");
    }
    if (ev->fn >= DM_EVAL_ZDT1 && ev->fn <= DM_EVAL_ZDT6)
        DM_CHECK_ARG(p->dim >= 2, "ZDT needs at least 2 genes");
    return DM_OK;
}

int validate_variation(const dm_variation* v, const dm_pop* p) {
    DM_CHECK_ARG(v->cx >= DM_CX_NONE && v->cx <= DM_CX_BLEND, "bad crossover %d", v->cx);
    DM_CHECK_ARG(v->mut >= DM_MUT_NONE && v->mut <= DM_MUT_GAUSSIAN, "bad mutation %d", v->mut);
    if (p->gtype == DM_BITS) {
        DM_CHECK_ARG(v->cx != DM_CX_BLEND, "cxBlend needs real-valued genomes");
        DM_CHECK_ARG(v->mut != DM_MUT_GAUSSIAN, "mutGaussian needs real-valued genomes");
    } else {
        DM_CHECK_ARG(v->mut != DM_MUT_FLIPBIT, "mutFlipBit needs packed-bit genomes");
    }
    if (v->cx == DM_CX_TWOPOINT) DM_CHECK_ARG(p->dim >= 2, "cxTwoPoint needs at least 2 genes");
    return DM_OK;
}

// ---------------------------------------------------------------------------
// RNG blocks (known-answer tests) and initialisation
// ---------------------------------------------------------------------------
__global__ void philox_blocks_kernel(u32x4 c0, uint32_t k0, uint32_t k1, int64_t n, uint32_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        u32x4 c = c0;
        c.x += (uint32_t)i;
        const u32x4 r = philox4x32_10(c, k0, k1);
        reinterpret_cast<uint4*>(out)[i] = make_uint4(r.x, r.y, r.z, r.w);
    }
}

__global__ void init_bits_kernel(uint64_t* genes, int64_t n, int64_t stride_words, int words,
                                 int dim, Rng rng, uint8_t* valid) {
    const int64_t total = n * words;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / words;
        const int w = (int)(i % words);
        const u32x4 v = rng(ST_INIT, (uint32_t)r, (uint32_t)w);
        uint64_t x = ((uint64_t)v.y << 32) | v.x;
        const int nb = dim - w * 64;
        if (nb < 64) x &= (1ull << nb) - 1;
        genes[r * stride_words + w] = x;
        if (w == 0) valid[r] = 0;
    }
}

template <typename T>
__global__ void init_float_kernel(char* genes, int64_t n, int64_t stride, int dim, double low,
                                  double high, Rng rng, uint8_t* valid) {
    const int q = (dim + 3) / 4;
    const int64_t total = n * q;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / q;
        const int g = (int)(i % q) * 4;
        const u32x4 v = rng(ST_INIT, (uint32_t)r, (uint32_t)(g >> 2));
        const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
        T* row = reinterpret_cast<T*>(genes + r * stride);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // random.uniform(a, b) = a + (b - a) * random()
            const double u = u01_32(ws[j]);
            row[g + j] = (g + j < dim) ? (T)(low + (high - low) * u) : (T)0;
        }
        if (g == 0) valid[r] = 0;
    }
}

// ---------------------------------------------------------------------------
// Batch evaluation: one lane group per row.
// ---------------------------------------------------------------------------
template <typename T, int G, int EC>
__global__ __launch_bounds__(256) void eval_float_kernel(const char* genes, int64_t stride,
                                                         double* wv, uint8_t* valid, int64_t n,
                                                         int dim, int nobj, dm_eval ev,
                                                         int only_invalid, int64_t* nevals) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t cnt = 0;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; r < n; r += gstride) {
        const bool todo = !only_invalid || !valid[r];
        if (!todo) continue;  // uniform within the group
        const char* row = genes + r * stride;
        EvalState st;
        eval_init(st);
        for (int cbase = 0; cbase < dim; cbase += 4 * G) {
            const int g = cbase + 4 * sub;
            double y[4] = {0, 0, 0, 0};
            if (g < dim) {
                if constexpr (sizeof(T) == 8) {
                    const double2* p = reinterpret_cast<const double2*>(row + (size_t)g * 8);
                    const double2 a = p[0], b = p[1];
                    y[0] = a.x;
                    y[1] = a.y;
                    y[2] = b.x;
                    y[3] = b.y;
                } else {
                    const float4 a = *reinterpret_cast<const float4*>(row + (size_t)g * 4);
                    y[0] = a.x;
                    y[1] = a.y;
                    y[2] = a.z;
                    y[3] = a.w;
                }
            }
            eval_chunk<G, EC>(ev, dim, g, cbase, y, true, st);
        }
        double f[DM_MAX_OBJ];
        eval_finish<G, EC>(ev, dim, st, f);
        if (sub == 0) {
            for (int o = 0; o < nobj; ++o) wv[r * nobj + o] = f[o] * ev.weights[o];
            valid[r] = 1;
            ++cnt;
        }
    }
    if (nevals) {
        int64_t tot = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)nevals, (unsigned long long)tot);
    }
}

template <int G>
__global__ __launch_bounds__(256) void eval_bits_kernel(const char* genes, int64_t stride,
                                                        double* wv, uint8_t* valid, int64_t n,
                                                        int words, int nobj, dm_eval ev,
                                                        int only_invalid, int64_t* nevals) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & (G - 1);
    const int64_t gstride = (int64_t)gridDim.x * (blockDim.x / G);
    int64_t cnt = 0;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; r < n; r += gstride) {
        if (only_invalid && valid[r]) continue;
        const uint64_t* row = reinterpret_cast<const uint64_t*>(genes + r * stride);
        int64_t pc = 0;
        for (int w = sub; w < words; w += G) pc += __popcll(row[w]);
        pc = group_sum_i<G>(pc);
        if (sub == 0) {
            for (int o = 0; o < nobj; ++o) wv[r * nobj + o] = (double)pc * ev.weights[o];
            valid[r] = 1;
            ++cnt;
        }
    }
    if (nevals) {
        int64_t tot = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (lane == 0 && tot) atomicAdd((unsigned long long*)nevals, (unsigned long long)tot);
    }
}

template <typename T, int G>
static void launch_eval_float(const dm_pop* p, const dm_eval* ev, int oi, int64_t* ne,
                              dim3 grid, hipStream_t s) {
    const int ec = eval_class(ev->fn);
    if (ec_single(ec))
        eval_float_kernel<T, G, EC_SUM><<<grid, 256, 0, s>>>((const char*)p->genes, p->stride,
                                                            p->wvalues, p->valid, p->n, p->dim,
                                                            p->nobj, *ev, oi, ne);
    else
        eval_float_kernel<T, G, EC_MO><<<grid, 256, 0, s>>>((const char*)p->genes, p->stride,
                                                           p->wvalues, p->valid, p->n, p->dim,
                                                           p->nobj, *ev, oi, ne);
}

static dim3 grid_for(dm_ctx* ctx, int64_t items, int per_block) {
    int64_t b = (items + per_block - 1) / per_block;
    b = std::min<int64_t>(std::max<int64_t>(b, 1), (int64_t)ctx->num_cus * 16);
    return dim3((unsigned)b);
}

// ---------------------------------------------------------------------------
// Selection (standalone) and gather
// ---------------------------------------------------------------------------
__global__ void sel_tournament_kernel(const double* wv, int nobj, int64_t n, int64_t k, int t,
                                      Rng rng, int mode, int32_t* asp, int32_t* out) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < k;
         c += (int64_t)gridDim.x * blockDim.x) {
        int64_t best = 0;
        for (int j = 0; j < t; ++j) {
            int64_t cand;
            if (mode == DM_RNG_INJECT) {
                cand = asp[c * t + j];
            } else {
                const u32x4 w = rng(ST_SEL, (uint32_t)c, (uint32_t)(j >> 1));
                cand = (j & 1) ? bounded64(w.z, w.w, (uint32_t)n) : bounded64(w.x, w.y, (uint32_t)n);
                if (mode == DM_RNG_DUMP) asp[c * t + j] = (int32_t)cand;
            }
            if (j == 0 || fit_gt(wv + cand * nobj, wv + best * nobj, nobj)) best = cand;
        }
        out[c] = (int32_t)best;
    }
}

// Rows copied in 16-B pieces by lpr lanes each (a power of two up to 64):
// 64 / lpr rows per wave.  One wave per row left most lanes idle on short
// rows (C5's 96-B genomes used 6 of 64, and its chosen-row gather ran ~8
// dependent row copies per wave in sequence).
__global__ void gather_kernel(const char* sg, const double* swv, const uint8_t* sv, int64_t sstride,
                              char* dg, double* dwv, uint8_t* dv, int64_t dstride,
                              const int32_t* idx, int64_t k, int64_t row_bytes, int nobj, int lpr) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & (lpr - 1);
    const int64_t rpw = 64 / lpr;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t q = row_bytes / 16;
    for (int64_t r = wave * rpw + lane / lpr; r < k; r += nw * rpw) {
        const int64_t s = idx ? idx[r] : r;
        const uint4* src = reinterpret_cast<const uint4*>(sg + s * sstride);
        uint4* dst = reinterpret_cast<uint4*>(dg + r * dstride);
        for (int64_t i = sub; i < q; i += lpr) dst[i] = src[i];
        for (int o = sub; o < nobj; o += lpr) dwv[r * nobj + o] = swv[s * nobj + o];
        if (sub == 0) dv[r] = sv[s];
    }
}

// Host-evaluated fitness written back (the scatter half of the host-evaluate
// bridge): row idx[i] takes wvalues src[i][0..nobj) and becomes valid; a row
// index outside [0, n) is skipped and counted in *bad.
__global__ void set_fitness_kernel(double* wv, uint8_t* valid, int nobj, int64_t nrows,
                                   const int32_t* idx, int64_t k, const double* src, int32_t* bad) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k * nobj;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / nobj;
        const int o = (int)(t % nobj);
        const int64_t r = idx[i];
        if (r < 0 || r >= nrows) {
            if (o == 0) atomicAdd(bad, 1);
            continue;
        }
        wv[r * nobj + o] = src[i * nobj + o];
        if (o == 0) valid[r] = 1;
    }
}

// Fitness statistics (tools.Statistics over fitness.values, support.py:199-210):
// per objective the min / max with first-occurrence argmin / argmax (numpy
// semantics), the count, mean and M2 = sum of squared deviations combined with
// Chan et al.'s pairwise update (stable where sumsq - n*mean^2 cancels), the
// plain sum, and NaN propagation as numpy's reducers do.
struct StatAcc {
    double mn, mx, mean, m2, sum;
    int64_t amn, amx, cnt, nan;
    int64_t anan;  // first row holding NaN (numpy's argmin / argmax return it), -1: none
};
__device__ __forceinline__ void stat_merge(StatAcc& x, const StatAcc& y) {
    if (y.amn >= 0 && (x.amn < 0 || y.mn < x.mn || (y.mn == x.mn && y.amn < x.amn))) {
        x.mn = y.mn;
        x.amn = y.amn;
    }
    if (y.amx >= 0 && (x.amx < 0 || y.mx > x.mx || (y.mx == x.mx && y.amx < x.amx))) {
        x.mx = y.mx;
        x.amx = y.amx;
    }
    if (y.cnt) {
        const int64_t n = x.cnt + y.cnt;
        const double d = y.mean - x.mean;
        x.mean += d * ((double)y.cnt / (double)n);
        x.m2 += y.m2 + d * d * ((double)x.cnt * (double)y.cnt / (double)n);
        x.cnt = n;
    }
    x.sum += y.sum;
    x.nan += y.nan;
    if (y.anan >= 0 && (x.anan < 0 || y.anan < x.anan)) x.anan = y.anan;
}
__global__ __launch_bounds__(256) void stats_kernel(const double* wv, const uint8_t* valid,
                                                    int64_t n, int nobj, dm_eval w, StatAcc* part,
                                                    int64_t nparts) {
    // w.weights: the fitness weights (values = wvalues / weights, base.py:184-185)
    const int o = blockIdx.y;
    StatAcc a{INFINITY, -INFINITY, 0.0, 0.0, 0.0, -1, -1, 0, 0, -1};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (!valid[i]) continue;
        const double v = wv[i * nobj + o] / w.weights[o];
        if (v != v) {
            ++a.nan;
            if (a.anan < 0) a.anan = i;  // rows ascend per thread
            continue;
        }
        if (a.amn < 0 || v < a.mn) {
            a.mn = v;
            a.amn = i;
        }
        if (a.amx < 0 || v > a.mx) {
            a.mx = v;
            a.amx = i;
        }
        ++a.cnt;  // Welford step
        const double d = v - a.mean;
        a.mean += d / (double)a.cnt;
        a.m2 += d * (v - a.mean);
        a.sum += v;
    }
    __shared__ StatAcc sh[256];
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) stat_merge(sh[threadIdx.x], sh[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(int64_t)o * nparts + blockIdx.x] = sh[0];
}
// One workgroup per objective: the partials merged in LDS as a fixed binary
// tree (deterministic; a serial merge of 256 partials by one thread took
// 0.18 ms of dependent loads per call, profiles/r02 bookkeeping run).
__global__ __launch_bounds__(256) void stats_combine_kernel(const StatAcc* part, int64_t nparts,
                                                            int nobj, double* out) {
    const int o = blockIdx.x;
    __shared__ StatAcc sh[256];
    StatAcc a{INFINITY, -INFINITY, 0.0, 0.0, 0.0, -1, -1, 0, 0, -1};
    for (int64_t b = threadIdx.x; b < nparts; b += blockDim.x)  // nparts <= 1024
        stat_merge(a, part[(int64_t)o * nparts + b]);
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) stat_merge(sh[threadIdx.x], sh[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x) return;
    a = sh[0];
    double* q = out + o * 8;
    const double qnan = __longlong_as_double(0x7FF8000000000000ll);
    const bool nan = a.nan > 0;
    q[0] = nan ? qnan : a.mn;
    q[1] = nan ? qnan : a.mx;
    q[2] = nan || a.cnt == 0 ? qnan : a.mean;
    q[3] = nan || a.cnt == 0 ? qnan : a.m2;
    q[4] = nan ? qnan : a.sum;
    q[5] = (double)(nan ? a.anan : a.amn);  // numpy: the first NaN is both arg-extrema
    q[6] = (double)(nan ? a.anan : a.amx);
    q[7] = (double)(a.cnt + a.nan);
}

bool fast_bitset(const dm_ctx* ctx, int m);  // dominance.hip
}  // namespace dm

using namespace dm;

extern "C" {

const char* dm_last_error(void) { return dm::g_err; }
const char* dm_version(void) { return "deapmi 0.1 gfx950"; }

static int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? atoi(v) : dflt;
}

static void read_knobs(dm_knobs& kn) {
    kn.disable_pipe = std::getenv("DM_DISABLE_PIPE") != nullptr;
    kn.bits_plan = std::getenv("DM_BITS_PLAN") != nullptr;
    kn.bits_nokeys = std::getenv("DM_BITS_NOKEYS") != nullptr;
    kn.lex_full = std::getenv("DM_LEX_FULL") != nullptr;
    kn.lex_no32 = std::getenv("DM_LEX_NO32") != nullptr;
    kn.pipe_label_rounds = std::max(0, std::min(8, env_int("DM_PIPE_LABEL_ROUNDS", 2)));
    kn.selbest_fullsort = std::getenv("DM_SELBEST_FULLSORT") != nullptr;
    kn.pipe_bpc = std::max(0, env_int("DM_PIPE_BPC", 0));
    kn.pipe_noorder = std::getenv("DM_PIPE_NOORDER") != nullptr;
    kn.pipe_key_fitter = std::getenv("DM_PIPE_KEY_FITTER") != nullptr;
}

int dm_ctx_reload_knobs(dm_ctx* ctx) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    read_knobs(ctx->knobs);
    return DM_OK;
}

int dm_ctx_create(int device, void* hip_stream, dm_ctx** out) {
    DM_CHECK_ARG(out != nullptr, "null out");
    DM_HIP(hipSetDevice(device));
    dm_ctx* c = new dm_ctx();
    c->device = device;
    c->stream = (hipStream_t)hip_stream;
    read_knobs(c->knobs);  // A/B switches, read once (common.hpp)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        c->num_cus = cus;
    double tab[2 * (ZIG_N + 1)];
    zig_make_tables(tab);
    if (hipMalloc(&c->zig, sizeof(tab)) != hipSuccess ||
        hipMemcpy(c->zig, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("ziggurat table upload failed");
        delete c;
        return DM_ERR_HIP;
    }
    const size_t spread = sizeof(long long) * kEvalSpreadWords;
    if (hipMalloc(&c->evals_spread, spread) != hipSuccess ||
        hipMemset(c->evals_spread, 0, spread) != hipSuccess) {
        set_error("counter allocation failed");
        (void)hipFree(c->zig);
        delete c;
        return DM_ERR_HIP;
    }
    *out = c;
    return DM_OK;
}

int dm_ctx_set_dom_path(dm_ctx* ctx, int32_t path) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    DM_CHECK_ARG(path >= DM_DOM_DEFAULT && path <= DM_DOM_LDS, "unknown dominance path %d", path);
    ctx->dom_path = path;
    return DM_OK;
}

int dm_ctx_dom_bitset(dm_ctx* ctx, int32_t nobj) {
    return ctx && dm::fast_bitset(ctx, nobj) && ctx->dom_path != DM_DOM_LDS &&
           ctx->dom_path != DM_DOM_BALLOT ? 1 : 0;
}

int dm_ctx_destroy(dm_ctx* ctx) {
    if (!ctx) return DM_OK;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < dm_ctx::kSlots; ++i)
        if (ctx->scratch[i]) (void)hipFree(ctx->scratch[i]);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->zig) (void)hipFree(ctx->zig);
    if (ctx->evals_spread) (void)hipFree(ctx->evals_spread);
    if (ctx->plan_lab) (void)hipFree(ctx->plan_lab);
    for (hipEvent_t e : ctx->tev) (void)hipEventDestroy(e);
    delete ctx;
    return DM_OK;
}

int dm_ctx_set_timing(dm_ctx* ctx, int32_t max_launches) {
    DM_CHECK_ARG(ctx != nullptr && max_launches >= 0, "bad argument");
    if (ctx->stream) DM_HIP(hipStreamSynchronize(ctx->stream));
    for (hipEvent_t e : ctx->tev) (void)hipEventDestroy(e);
    ctx->tev.clear();
    ctx->tev_used = 0;
    for (int i = 0; i < 2 * max_launches; ++i) {
        hipEvent_t e;
        DM_HIP(hipEventCreate(&e));
        ctx->tev.push_back(e);
    }
    return DM_OK;
}

int dm_ctx_set_timing_target(dm_ctx* ctx, int32_t target) {
    DM_CHECK_ARG(ctx != nullptr && (target >= DM_TIME_GENERATION && target <= DM_TIME_PEEL_CHAIN),
                 "bad timing target %d", target);
    ctx->timing_target = target;
    return DM_OK;
}

int dm_ctx_kernel_times(dm_ctx* ctx, float* ms, int32_t cap, int32_t* count) {
    DM_CHECK_ARG(ctx != nullptr && count != nullptr && (ms != nullptr || cap == 0), "bad argument");
    const int n = std::min(ctx->tev_used, (int)cap);
    for (int i = 0; i < n; ++i) {
        DM_HIP(hipEventSynchronize(ctx->tev[2 * i + 1]));
        DM_HIP(hipEventElapsedTime(&ms[i], ctx->tev[2 * i], ctx->tev[2 * i + 1]));
    }
    *count = ctx->tev_used;
    return DM_OK;
}

int dm_ctx_set_stream(dm_ctx* ctx, void* hip_stream) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    hipStream_t next = (hipStream_t)hip_stream;
    if (next != ctx->stream) {
        // The scratch slots are reused by the next launch on the new stream:
        // order it after everything already queued on the old one.
        hipEvent_t e;
        DM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        hipError_t err = hipEventRecord(e, ctx->stream);
        if (err == hipSuccess) err = hipStreamWaitEvent(next, e, 0);
        (void)hipEventDestroy(e);
        DM_HIP(err);
    }
    ctx->stream = next;
    return DM_OK;
}

int dm_ctx_sync(dm_ctx* ctx) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    DM_HIP(hipStreamSynchronize(ctx->stream));
    return DM_OK;
}

int dm_zero(dm_ctx* ctx, void* ptr, int64_t bytes) {
    DM_CHECK_ARG(ctx != nullptr && bytes >= 0 && (ptr != nullptr || bytes == 0), "bad argument");
    if (bytes) DM_HIP(hipMemsetAsync(ptr, 0, (size_t)bytes, ctx->stream));
    return DM_OK;
}

int dm_philox_blocks(dm_ctx* ctx, const uint32_t ctr0[4], const uint32_t key[2], int64_t nblocks,
                     uint32_t* out) {
    DM_CHECK_ARG(ctx && ctr0 && key && out && nblocks >= 0, "bad argument");
    if (nblocks == 0) return DM_OK;
    philox_blocks_kernel<<<grid_for(ctx, nblocks, 256), 256, 0, ctx->stream>>>(
        u32x4{ctr0[0], ctr0[1], ctr0[2], ctr0[3]}, key[0], key[1], nblocks, out);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_init_uniform(dm_ctx* ctx, dm_pop* pop, double low, double high, dm_rng rng) {
    DM_CHECK_ARG(ctx != nullptr, "null ctx");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    if (pop->n == 0) return DM_OK;
    if (pop->gtype == DM_BITS) {
        const int words = (pop->dim + 63) / 64;
        init_bits_kernel<<<grid_for(ctx, pop->n * words, 256), 256, 0, ctx->stream>>>(
            (uint64_t*)pop->genes, pop->n, pop->stride / 8, words, pop->dim, Rng(rng), pop->valid);
    } else {
        const int64_t items = pop->n * ((pop->dim + 3) / 4);
        if (pop->gtype == DM_F64)
            init_float_kernel<double><<<grid_for(ctx, items, 256), 256, 0, ctx->stream>>>(
                (char*)pop->genes, pop->n, pop->stride, pop->dim, low, high, Rng(rng), pop->valid);
        else
            init_float_kernel<float><<<grid_for(ctx, items, 256), 256, 0, ctx->stream>>>(
                (char*)pop->genes, pop->n, pop->stride, pop->dim, low, high, Rng(rng), pop->valid);
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_evaluate(dm_ctx* ctx, dm_pop* pop, const dm_eval* ev, int only_invalid, int64_t* nevals) {
    DM_CHECK_ARG(ctx && ev, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(ev->fn != DM_EVAL_NONE, "no objective function");
    if ((rc = validate_eval(ev, pop))) return rc;
    if (pop->n == 0) return DM_OK;
    hipStream_t s = ctx->stream;
    if (pop->gtype == DM_BITS) {
        const int words = (pop->dim + 63) / 64;
        const int G = words <= 2 ? 2 : words <= 8 ? 8 : words <= 32 ? 32 : 64;
        dim3 grid = grid_for(ctx, pop->n, 256 / G);
        switch (G) {
            case 2: eval_bits_kernel<2><<<grid, 256, 0, s>>>((const char*)pop->genes, pop->stride, pop->wvalues, pop->valid, pop->n, words, pop->nobj, *ev, only_invalid, nevals); break;
            case 8: eval_bits_kernel<8><<<grid, 256, 0, s>>>((const char*)pop->genes, pop->stride, pop->wvalues, pop->valid, pop->n, words, pop->nobj, *ev, only_invalid, nevals); break;
            case 32: eval_bits_kernel<32><<<grid, 256, 0, s>>>((const char*)pop->genes, pop->stride, pop->wvalues, pop->valid, pop->n, words, pop->nobj, *ev, only_invalid, nevals); break;
            default: eval_bits_kernel<64><<<grid, 256, 0, s>>>((const char*)pop->genes, pop->stride, pop->wvalues, pop->valid, pop->n, words, pop->nobj, *ev, only_invalid, nevals); break;
        }
    } else {
        const int q = (pop->dim + 3) / 4;
        const int G = q <= 2 ? 2 : q <= 4 ? 4 : q <= 8 ? 8 : q <= 16 ? 16 : q <= 32 ? 32 : 64;
        dim3 grid = grid_for(ctx, pop->n, 256 / G);
        const int oi = only_invalid;
        if (pop->gtype == DM_F64) {
            switch (G) {
                case 2: launch_eval_float<double, 2>(pop, ev, oi, nevals, grid, s); break;
                case 4: launch_eval_float<double, 4>(pop, ev, oi, nevals, grid, s); break;
                case 8: launch_eval_float<double, 8>(pop, ev, oi, nevals, grid, s); break;
                case 16: launch_eval_float<double, 16>(pop, ev, oi, nevals, grid, s); break;
                case 32: launch_eval_float<double, 32>(pop, ev, oi, nevals, grid, s); break;
                default: launch_eval_float<double, 64>(pop, ev, oi, nevals, grid, s); break;
            }
        } else {
            switch (G) {
                case 2: launch_eval_float<float, 2>(pop, ev, oi, nevals, grid, s); break;
                case 4: launch_eval_float<float, 4>(pop, ev, oi, nevals, grid, s); break;
                case 8: launch_eval_float<float, 8>(pop, ev, oi, nevals, grid, s); break;
                case 16: launch_eval_float<float, 16>(pop, ev, oi, nevals, grid, s); break;
                case 32: launch_eval_float<float, 32>(pop, ev, oi, nevals, grid, s); break;
                default: launch_eval_float<float, 64>(pop, ev, oi, nevals, grid, s); break;
            }
        }
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_sel_tournament(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t tournsize, dm_rng rng,
                      int32_t mode, const dm_decisions* dec, int32_t* out_idx) {
    DM_CHECK_ARG(ctx && out_idx, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    DM_CHECK_ARG(k >= 0 && tournsize >= 1, "bad k / tournsize");
    DM_CHECK_ARG(pop->n > 0 || k == 0, "cannot select from an empty population");
    DM_CHECK_ARG(pop->n < (1ll << 31), "population too large");
    int32_t* asp = nullptr;
    if (mode != DM_RNG_NATIVE) {
        DM_CHECK_ARG(dec && dec->aspirants, "decisions.aspirants required");
        asp = dec->aspirants;
    }
    if (k == 0) return DM_OK;
    sel_tournament_kernel<<<grid_for(ctx, k, 256), 256, 0, ctx->stream>>>(
        pop->wvalues, pop->nobj, pop->n, k, tournsize, Rng(rng), mode, asp, out_idx);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_sel_random(dm_ctx* ctx, int64_t n, int64_t k, dm_rng rng, int32_t mode,
                  const dm_decisions* dec, int32_t* out_idx) {
    DM_CHECK_ARG(ctx && out_idx, "null argument");
    DM_CHECK_ARG(k >= 0 && n >= 0 && n < (1ll << 31), "bad sizes");
    DM_CHECK_ARG(n > 0 || k == 0, "cannot select from an empty population");
    int32_t* asp = nullptr;
    if (mode != DM_RNG_NATIVE) {
        DM_CHECK_ARG(dec && dec->aspirants, "decisions.aspirants required");
        asp = dec->aspirants;
    }
    if (k == 0) return DM_OK;
    // a one-aspirant tournament never compares: it is selRandom
    sel_tournament_kernel<<<grid_for(ctx, k, 256), 256, 0, ctx->stream>>>(
        nullptr, 1, n, k, 1, Rng(rng), mode, asp, out_idx);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_gather(dm_ctx* ctx, const dm_pop* src, const int32_t* idx, dm_pop* dst) {
    DM_CHECK_ARG(ctx && src && dst, "null argument");
    int rc;
    if ((rc = validate_pop(src, "src")) || (rc = validate_pop(dst, "dst"))) return rc;
    DM_CHECK_ARG(src->gtype == dst->gtype && src->dim == dst->dim && src->nobj == dst->nobj,
                 "src/dst layout mismatch");
    if (!idx) DM_CHECK_ARG(dst->n <= src->n, "identity gather needs dst.n <= src.n");
    if (dst->n == 0) return DM_OK;
    const int64_t row_bytes = std::min(src->stride, dst->stride);
    int lpr = 1;  // lanes per row: the row's 16-B pieces, rounded up to a power of two
    while (lpr < 64 && lpr * 16 < row_bytes) lpr *= 2;
    const int64_t rows_per_block = 4 * (64 / lpr);
    gather_kernel<<<grid_for(ctx, dst->n, (int)rows_per_block), 256, 0, ctx->stream>>>(
        (const char*)src->genes, src->wvalues, src->valid, src->stride, (char*)dst->genes,
        dst->wvalues, dst->valid, dst->stride, idx, dst->n, row_bytes, src->nobj, lpr);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

int dm_set_fitness(dm_ctx* ctx, dm_pop* pop, const int32_t* idx, int64_t k, const double* wv) {
    DM_CHECK_ARG(ctx && pop && (k == 0 || (idx && wv)), "null argument");
    DM_CHECK_ARG(k >= 0, "negative count");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    if (k == 0) return DM_OK;
    int32_t* bad = (int32_t*)scratch(ctx, 16);
    if (!bad) return DM_ERR_NOMEM;
    DM_HIP(hipMemsetAsync(bad, 0, 4, ctx->stream));
    set_fitness_kernel<<<grid_for(ctx, k * pop->nobj, 256), 256, 0, ctx->stream>>>(
        pop->wvalues, pop->valid, pop->nobj, pop->n, idx, k, wv, bad);
    DM_LAUNCH_CHECK();
    int32_t hbad = 0;
    DM_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, ctx->stream));
    DM_HIP(hipStreamSynchronize(ctx->stream));
    if (hbad) {
        set_error("dm_set_fitness: %d row indices outside [0, %lld)", hbad, (long long)pop->n);
        return DM_ERR_INDEX;
    }
    return DM_OK;
}

int dm_fitness_stats(dm_ctx* ctx, const dm_pop* pop, const double* weights, double* out) {
    DM_CHECK_ARG(ctx && weights && out, "null argument");
    int rc = validate_pop(pop, "pop");
    if (rc) return rc;
    dm_eval w{};
    for (int o = 0; o < pop->nobj; ++o) {
        DM_CHECK_ARG(weights[o] != 0.0, "zero fitness weight");
        w.weights[o] = weights[o];
    }
    const int64_t nparts = std::min<int64_t>(std::max<int64_t>((pop->n + 4095) / 4096, 1), 1024);
    StatAcc* part = (StatAcc*)scratch(ctx, (size_t)nparts * pop->nobj * sizeof(StatAcc));
    if (!part) return DM_ERR_NOMEM;
    stats_kernel<<<dim3((unsigned)nparts, pop->nobj), 256, 0, ctx->stream>>>(
        pop->wvalues, pop->valid, pop->n, pop->nobj, w, part, nparts);
    stats_combine_kernel<<<pop->nobj, 256, 0, ctx->stream>>>(part, nparts, pop->nobj, out);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

}  // extern "C"
