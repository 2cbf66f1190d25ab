// generation.hip — host side of the fused generation (see generation.hpp for
// the kernels; per-genome-type instantiations live in generation_{f64,f32,bits}.hip
// so they compile in parallel).
#include "generation_pipe.hpp"
#include "sort.hpp"

namespace dm {

// Lanes per offspring pair: enough lanes to cover the row in few chunks.
// zero two int arrays of n entries in one launch (16-B stores): the ordered
// plans' slot counts and labels, two hipMemsetAsync fills of 4 MB at 2^20
// that ran 8.6 us each (profiles/r05fin2/c3_kernel_stats.csv)
__global__ __launch_bounds__(256) void zero2_kernel(int32_t* __restrict__ a, int32_t* __restrict__ b,
                                                    int64_t n) {
    const int64_t n4 = n >> 2;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += step) {
        reinterpret_cast<int4*>(a)[i] = make_int4(0, 0, 0, 0);
        if (b) reinterpret_cast<int4*>(b)[i] = make_int4(0, 0, 0, 0);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        a[i] = 0;
        if (b) b[i] = 0;
    }
}

static int pick_group_float(int dim) {
    const int q = (dim + 3) / 4;  // lane-slots of 4 genes
    if (q <= 4) return 4;
    if (q <= 16) return 16;
    return 64;
}
static int pick_group_bits(int words) {
    if (words <= 2) return 2;
    if (words <= 8) return 8;
    return 64;
}

int validate_pop(const dm_pop* p, const char* what);
int validate_eval(const dm_eval* ev, const dm_pop* p);
int validate_variation(const dm_variation* v, const dm_pop* p);

// The context's persistent parent-graph labels for n rows and this call's
// epoch (generation_pipe_f64.hip lab_of): grown (and zeroed) on demand, and
// zeroed again when the 32-bit epoch wraps.
static uint64_t* plan_labels(dm_ctx* ctx, int64_t n, uint32_t* epoch) {
    if (n > ctx->plan_lab_n || ctx->plan_epoch == 0xFFFFFFFFu) {
        if (n > ctx->plan_lab_n) {
            if (ctx->plan_lab) {
                if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
                (void)hipFree(ctx->plan_lab);
                ctx->plan_lab = nullptr;
                ctx->plan_lab_n = 0;
            }
            if (hipMalloc(&ctx->plan_lab, (size_t)n * 8) != hipSuccess) {
                ctx->plan_lab = nullptr;
                return nullptr;
            }
            ctx->plan_lab_n = n;
        }
        if (hipMemsetAsync(ctx->plan_lab, 0, (size_t)ctx->plan_lab_n * 8, ctx->stream) != hipSuccess)
            return nullptr;
        ctx->plan_epoch = 0;
    }
    *epoch = ++ctx->plan_epoch;
    return ctx->plan_lab;
}

int launch_generation(dm_ctx* ctx, const dm_pop* parents, dm_pop* children, int32_t sel,
                      int32_t tournsize, const int32_t* sel_index, const dm_variation* var,
                      const dm_eval* ev, dm_rng rng, int32_t mode, const dm_decisions* dec,
                      int64_t* nevals) {
    int rc;
    if ((rc = validate_pop(parents, "parents"))) return rc;
    if ((rc = validate_pop(children, "children"))) return rc;
    DM_CHECK_ARG(parents->gtype == children->gtype && parents->dim == children->dim &&
                     parents->nobj == children->nobj,
                 "parents and children must share genome type, dim and nobj");
    DM_CHECK_ARG(parents->genes != children->genes, "children must not alias parents");
    DM_CHECK_ARG(sel >= DM_SEL_IDENTITY && sel <= DM_SEL_RANDOM, "bad selection kind %d", sel);
    if (sel == DM_SEL_IDENTITY)
        DM_CHECK_ARG(children->n <= parents->n, "identity selection needs k <= n");
    if (sel == DM_SEL_INDEX) DM_CHECK_ARG(sel_index != nullptr, "sel_index required");
    if (sel == DM_SEL_TOURNAMENT || sel == DM_SEL_RANDOM) {
        DM_CHECK_ARG(parents->n > 0 && parents->n < (1ll << 31), "population size out of range");
        if (sel == DM_SEL_TOURNAMENT) DM_CHECK_ARG(tournsize >= 1, "tournsize must be >= 1");
        else tournsize = 1;
    }
    DM_CHECK_ARG(var != nullptr, "variation required");
    if ((rc = validate_variation(var, parents))) return rc;
    dm_eval none{};
    if (!ev) ev = &none;
    if ((rc = validate_eval(ev, parents))) return rc;
    DM_CHECK_ARG(mode >= DM_RNG_NATIVE && mode <= DM_RNG_DUMP, "bad rng mode");
    dm_decisions d{};
    if (dec) d = *dec;
    if (mode != DM_RNG_NATIVE) {
        DM_CHECK_ARG(dec != nullptr, "decisions required for inject/dump");
        if (sel == DM_SEL_TOURNAMENT || sel == DM_SEL_RANDOM)
            DM_CHECK_ARG(d.aspirants, "decisions.aspirants required");
        if (var->cx != DM_CX_NONE) DM_CHECK_ARG(d.cx_flag, "decisions.cx_flag required");
        if (var->cx == DM_CX_TWOPOINT && mode == DM_RNG_INJECT)
            DM_CHECK_ARG(d.cx_raw, "decisions.cx_raw required");
        if (var->cx == DM_CX_BLEND) DM_CHECK_ARG(d.blend_u, "decisions.blend_u required");
        if (var->mut != DM_MUT_NONE)
            DM_CHECK_ARG(d.mut_flag && d.mut_mask, "decisions.mut_flag/mut_mask required");
        if (var->mut == DM_MUT_GAUSSIAN) DM_CHECK_ARG(d.gauss, "decisions.gauss required");
    }
    if (children->n == 0) return DM_OK;
    if (mode == DM_RNG_DUMP && var->mut == DM_MUT_GAUSSIAN) {
        DM_HIP(hipMemsetAsync(d.mut_mask, 0,
                              (size_t)children->n * ((parents->dim + 63) / 64) * 8, ctx->stream));
    }

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
    a.sel = sel;
    a.tournsize = tournsize;
    a.sel_index = sel_index;
    a.cx = var->cx;
    a.mut = var->mut;
    a.thr_cx = prob_threshold(var->cxpb);
    a.thr_mut = prob_threshold(var->mutpb);
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

    const int ec = eval_class(ev->fn);
    const int64_t npairs = (children->n + 1) / 2;
    // hot path: native RNG, float rows of more than 64 genes, fused tournament /
    // random selection -> per-pair decision kernel + rolling-pipeline kernel on
    // a persistent grid (generation_pipe.hpp); rows past 1,024 genes take its
    // run-time chunk count (nch 0)
    if (mode == DM_RNG_NATIVE && parents->gtype != DM_BITS && parents->dim > 64 &&
        parents->dim <= 65535 && (sel == DM_SEL_TOURNAMENT || sel == DM_SEL_RANDOM) &&
        ec != EC_MO && !ctx->knobs.disable_pipe) {
        const int nch = parents->dim <= 512 ? 2 : parents->dim <= 1024 ? 4 : 0;
        // parent order: the plans sorted by a key parent -- of
        // the two, the one in more pair slots of this generation (a greedy
        // vertex cover of the pairs) -- so the pairs that share that row are
        // varied together and the row's repeated reads hit the L2, not HBM
        const bool ordered = !ctx->knobs.pipe_noorder && npairs >= 4096 &&
                             npairs < (1ll << (32 - PF_PAIR_SHIFT));
        const size_t pb = align_up((size_t)npairs * sizeof(PairPlan), 256);
        const size_t hb = align_up((size_t)(a.np + 1) * 4, 256);
        const size_t kb = align_up((size_t)npairs * 4, 256);
        char* w = (char*)scratch(ctx, ordered ? 2 * pb + 3 * hb + 4 * kb +
                                                    align_up(scan_temp_bytes(a.np), 256) : pb);
        if (!w) return DM_ERR_NOMEM;
        PairPlan* plans = (PairPlan*)w;
        // nevals is counted by the plan kernel (spread counters + fold): one
        // same-address atomic per hot-kernel wave serialised 65,536 atomics
        const bool count = ec != EC_NONE && a.nevals;
        if (ordered) {
            PairPlan* sorted = (PairPlan*)(w + pb);
            int32_t* hist = (int32_t*)(w + 2 * pb);
            int32_t* start = (int32_t*)(w + 2 * pb + hb);
            int32_t* keys = (int32_t*)(w + 2 * pb + 2 * hb);
            int32_t* tick = (int32_t*)(w + 2 * pb + 2 * hb + kb);
            void* stemp = w + 2 * pb + 2 * hb + 2 * kb;
            const unsigned zg = (unsigned)std::min<int64_t>(2048, (a.np / 4 + 255) / 256 + 1);
            if (!ctx->knobs.pipe_key_fitter && ctx->knobs.pipe_label_rounds > 0) {
                // bins: labels of the parent graph's neighbourhoods (round 1
                // inside the plan kernel, further rounds after it), persistent
                // and epoch-tagged; the plan kernel clears the bins' ticket
                // counters (hist) for the key kernel: no fill launch
                uint32_t epoch = 0;
                uint64_t* lab64 = plan_labels(ctx, a.np, &epoch);
                if (!lab64) return DM_ERR_NOMEM;
                int2* pairs2 = (int2*)((char*)stemp + align_up(scan_temp_bytes(a.np), 256));  // 2 kb
                launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream,
                                  nullptr, nullptr, nullptr, lab64, epoch, pairs2, hist, a.np + 1);
                // DM_PIPE_LABEL_ROUNDS = r: round 1 in the plan kernel; r >= 2: r - 2
                // scatter rounds (plan_label_kernel, atomics) and the gather jump in
                // the key kernel (the default r = 2: no label kernel)
                const int rounds = ctx->knobs.pipe_label_rounds;
                if (rounds > 2)
                    launch_plan_labels(pairs2, lab64, epoch, npairs, rounds - 2, ctx->stream);
                launch_plan_degree_keys(plans, pairs2, nullptr, lab64, epoch, rounds >= 2, keys,
                                        tick, hist, npairs, ctx->stream);
            } else if (!ctx->knobs.pipe_key_fitter) {
                // DM_PIPE_LABEL_ROUNDS=0: degree keys (counted into the zeroed deg)
                int32_t* deg = (int32_t*)((char*)stemp + align_up(scan_temp_bytes(a.np), 256));
                zero2_kernel<<<zg, 256, 0, ctx->stream>>>(hist, deg, a.np);
                launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream,
                                  nullptr, deg);
                launch_plan_degree_keys(plans, nullptr, deg, nullptr, 0, false, keys, tick, hist,
                                        npairs, ctx->stream);
            } else {
                zero2_kernel<<<zg, 256, 0, ctx->stream>>>(hist, nullptr, a.np);
                launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream, keys,
                                  hist, tick);
            }
            int rc = exclusive_scan_i32(ctx->stream, hist, start, a.np, nullptr, stemp);
            if (rc) return rc;
            launch_plan_order(plans, keys, tick, start, sorted, npairs, ctx->stream);
            plans = sorted;
        } else {
            launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream);
        }
        DM_LAUNCH_CHECK();
        PipeArgs q{};
        q.pgenes = a.pgenes;
        q.cgenes = a.cgenes;
        q.cwv = a.cwv;
        q.cvalid = a.cvalid;
        q.plans = plans;
        q.pwv = a.pwv;
        q.mu_vec = a.mu_vec;
        q.sigma_vec = a.sigma_vec;
        q.zig = a.zig;
        q.nevals = nullptr;
        q.nc = a.nc;
        q.pstride = a.pstride;
        q.cstride = a.cstride;
        q.dim = a.dim;
        q.nobj = a.nobj;
        q.rng = a.rng;
        q.thr_ind = a.thr_ind;
        q.alpha = a.alpha;
        q.mu = a.mu;
        q.sigma = a.sigma;
        q.w0 = a.w0;
        q.ev = a.ev;
        q.bpc = ctx->knobs.pipe_bpc;
        q.ordered = ordered ? 1 : 0;
        timing_begin(ctx);
        if (parents->gtype == DM_F64)
            launch_gen_pipe_f64(q, ec, a.cx, a.mut, nch, ctx->num_cus, ctx->stream);
        else
            launch_gen_pipe_f32(q, ec, a.cx, a.mut, nch, ctx->num_cus, ctx->stream);
        timing_end(ctx);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    // short float rows (at most 64 genes, any objective count): the per-pair
    // decision kernel + the lane-group streaming kernel (generation_rows.hpp)
    if (mode == DM_RNG_NATIVE && parents->gtype != DM_BITS && parents->dim <= 64 &&
        (sel == DM_SEL_TOURNAMENT || sel == DM_SEL_RANDOM) && !ctx->knobs.disable_pipe) {
        PairPlan* plans = (PairPlan*)scratch(ctx, align_up((size_t)npairs * sizeof(PairPlan), 256));
        if (!plans) return DM_ERR_NOMEM;
        const bool count = ec != EC_NONE && a.nevals;
        launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream);
        DM_LAUNCH_CHECK();
        timing_begin(ctx);
        if (parents->gtype == DM_F64)
            launch_gen_rows_f64(a, plans, ec, ctx->num_cus, ctx->stream);
        else
            launch_gen_rows_f32(a, plans, ec, ctx->num_cus, ctx->stream);
        timing_end(ctx);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    // packed-bit hot path (C2): one fused burst kernel for tournaments of at most
    // 8 aspirants (decisions drawn in-kernel), else the plan kernel (which also
    // counts nevals) + the burst kernel (generation_pipe_bits.hip)
    if (mode == DM_RNG_NATIVE && parents->gtype == DM_BITS && a.words64 <= 256 &&
        parents->nobj == 1 && (sel == DM_SEL_TOURNAMENT || sel == DM_SEL_RANDOM) &&
        !ctx->knobs.disable_pipe &&
        (a.words64 <= 64 || ((sel == DM_SEL_RANDOM || tournsize <= 8) && !ctx->knobs.bits_plan))) {
        // rows of 65-256 words: the fused kernel only (64-word pieces per lane)
        if ((sel == DM_SEL_RANDOM || tournsize <= 8) && !ctx->knobs.bits_plan) {
            // one launch: decisions drawn inside the burst kernel (+ the
            // nevals reduction of its per-workgroup partials)
            const bool count = ec != EC_NONE && a.nevals;
            // tournaments read the parents' fitness through int16 keys (one
            // coalesced pass, timed with the generation kernel)
            const bool keys = sel == DM_SEL_TOURNAMENT && a.w0 != 0.0 && !ctx->knobs.bits_nokeys;
            if (keys) {
                int16_t* kb = (int16_t*)scratch(ctx, (size_t)a.np * 2 + 16);
                if (!kb) return DM_ERR_NOMEM;
                a.pkeys = kb;
            }
            timing_begin(ctx);
            if (keys) launch_fit_keys(a, (int16_t*)a.pkeys, ctx->stream);
            launch_gen_bits_fused(a, ec != EC_NONE, count ? ctx->evals_spread : nullptr,
                                  ctx->stream);
            timing_end(ctx);
            DM_LAUNCH_CHECK();
            return DM_OK;
        }
        PairPlan* plans = (PairPlan*)scratch(ctx, (size_t)npairs * sizeof(PairPlan));
        if (!plans) return DM_ERR_NOMEM;
        const bool count = ec != EC_NONE && a.nevals;
        launch_pair_plans(a, plans, count ? ctx->evals_spread : nullptr, ctx->stream);
        DM_LAUNCH_CHECK();
        timing_begin(ctx);
        launch_gen_bits_pipe(a, plans, ec != EC_NONE, ctx->num_cus, ctx->stream);
        timing_end(ctx);
        DM_LAUNCH_CHECK();
        return DM_OK;
    }
    const int G = parents->gtype == DM_BITS ? pick_group_bits(a.words64)
                                            : pick_group_float(parents->dim);
    const int64_t groups_per_block = 256 / G;
    int64_t blocks = (npairs + groups_per_block - 1) / groups_per_block;
    blocks = std::min<int64_t>(blocks, (int64_t)ctx->num_cus * 16);
    const dim3 grid((unsigned)std::max<int64_t>(blocks, 1));
    timing_begin(ctx);
    if (parents->gtype == DM_BITS)
        launch_gen_bits(a, ec, G, grid, ctx->stream);
    else if (parents->gtype == DM_F64)
        (mode == DM_RNG_NATIVE ? launch_gen_f64_native : launch_gen_f64_replay)(a, ec, G, grid,
                                                                                 ctx->stream);
    else
        (mode == DM_RNG_NATIVE ? launch_gen_f32_native : launch_gen_f32_replay)(a, ec, G, grid,
                                                                                 ctx->stream);
    timing_end(ctx);
    DM_LAUNCH_CHECK();
    return DM_OK;
}

}  // namespace dm

extern "C" int dm_generation(dm_ctx* ctx, const dm_pop* parents, dm_pop* children, int32_t sel,
                             int32_t tournsize, const int32_t* sel_index,
                             const dm_variation* var, const dm_eval* ev, dm_rng rng,
                             int32_t mode, const dm_decisions* dec, int64_t* nevals) {
    DM_CHECK_ARG(ctx && parents && children, "null argument");
    return dm::launch_generation(ctx, parents, children, sel, tournsize, sel_index, var, ev, rng,
                                 mode, dec, nevals);
}
