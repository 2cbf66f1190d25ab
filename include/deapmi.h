/*
 * deapmi.h — C ABI of libdeapmi.so, the MI355X (gfx950) engine for DEAP's
 * per-generation population hot path.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, returns an
 * int status (DM_OK = 0) and never throws.  On failure `dm_last_error()` holds
 * a thread-local message.  Device buffers are owned by the caller (PyTorch
 * tensors in the Python host layer); the library never frees or retains them.
 * Scratch lives in the opaque `dm_ctx`, bound to one device and one stream.
 * Every launch is asynchronous on the context's stream; no entry point below
 * synchronises the host unless its comment says so.
 *
 * Each function cites the DEAP 1.3.1 interface (file:line under the reference
 * tree) whose behaviour it reproduces at population granularity.  Randomness
 * comes either from the counter-based Philox RNG (mode DM_RNG_NATIVE; stream
 * layout in DESIGN.md §RNG), from caller-supplied decisions (DM_RNG_INJECT —
 * the same pre-drawn decisions replayed into the DEAP reference give the same
 * offspring), or natively with every decision written out (DM_RNG_DUMP).
 */
#ifndef DEAPMI_H
#define DEAPMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------- */
enum dm_status {
    DM_OK = 0,
    DM_ERR_INVALID = 1,   /* bad argument: maps to ValueError / TypeError  */
    DM_ERR_INDEX = 2,     /* short mu/sigma/low/up sequence: IndexError     */
    DM_ERR_HIP = 3,       /* HIP runtime error                               */
    DM_ERR_NOMEM = 4,     /* scratch allocation failed                       */
    DM_ERR_UNSUPPORTED = 5
};

/* ---- genome / operator enums -------------------------------------------- */
enum dm_gtype { DM_BITS = 0, DM_F32 = 1, DM_F64 = 2 };

enum dm_cx { DM_CX_NONE = 0, DM_CX_TWOPOINT = 1, DM_CX_BLEND = 2 };
enum dm_mut { DM_MUT_NONE = 0, DM_MUT_FLIPBIT = 1, DM_MUT_GAUSSIAN = 2 };

enum dm_sel {
    DM_SEL_IDENTITY = 0,   /* child k <- parent k (varAnd on a population)   */
    DM_SEL_INDEX = 1,      /* child k <- parent index[k] (any select + clone) */
    DM_SEL_TOURNAMENT = 2, /* child k <- selTournament winner (fused)         */
    DM_SEL_RANDOM = 3      /* child k <- selRandom draw (fused)               */
};

enum dm_eval_fn {
    DM_EVAL_NONE = 0,
    DM_EVAL_ONEMAX = 1,      /* README.md:85-86 sum(individual)                 */
    DM_EVAL_RASTRIGIN = 2,   /* deap/benchmarks/__init__.py:220-240             */
    DM_EVAL_ROSENBROCK = 3,  /* deap/benchmarks/__init__.py:98-118              */
    DM_EVAL_ZDT1 = 4,        /* deap/benchmarks/__init__.py:391-403             */
    DM_EVAL_ZDT2 = 5,        /* :405-419 */
    DM_EVAL_ZDT3 = 6,        /* :421-435 */
    DM_EVAL_ZDT4 = 7,        /* :437-450 */
    DM_EVAL_ZDT6 = 8,        /* :452-465 */
    DM_EVAL_DTLZ1 = 9,       /* :467-493 */
    DM_EVAL_DTLZ2 = 10,      /* :495-521 */
    DM_EVAL_DTLZ3 = 11,      /* :523-548 */
    DM_EVAL_DTLZ4 = 12,      /* :550-577 */
    DM_EVAL_SPHERE = 13      /* :62-78 (sum of squares; cheap test objective)   */
};

enum dm_rng_mode { DM_RNG_NATIVE = 0, DM_RNG_INJECT = 1, DM_RNG_DUMP = 2 };

#define DM_MAX_OBJ 8

/* ---- structures (all pointers are device pointers unless noted) --------- */

/* Structure-of-arrays population (deap/base.py:125-270 Fitness + creator
 * Individual types deap/creator.py:76-93).  Genome row r starts at
 * (char*)genes + r*stride.  DM_BITS rows hold ceil(dim/64) uint64 words, gene
 * i at word i>>6, bit i&63 (LSB first); bits >= dim are zero.  wvalues holds
 * the *weighted* fitness (values*weights, base.py:187-198), valid[r] != 0
 * iff the fitness is valid (base.py:226-229). */
typedef struct dm_pop {
    void* genes;
    double* wvalues;   /* [n][nobj] */
    uint8_t* valid;    /* [n]       */
    int64_t n;
    int64_t stride;    /* bytes per genome row, multiple of 16 */
    int32_t dim;
    int32_t gtype;     /* enum dm_gtype */
    int32_t nobj;
    int32_t reserved;
} dm_pop;

/* Objective function + the fitness weights it is stored under. */
typedef struct dm_eval {
    int32_t fn;        /* enum dm_eval_fn */
    int32_t obj;       /* number of objectives for DTLZ (its `obj` argument) */
    double alpha;      /* DTLZ4 alpha */
    double weights[DM_MAX_OBJ];
} dm_eval;

/* Variation parameters: varAnd/varOr probabilities plus the registered
 * mate/mutate partial keywords (crossover.py:37-60,241-260;
 * mutation.py:17-48,124-142). */
typedef struct dm_variation {
    int32_t cx;        /* enum dm_cx  */
    int32_t mut;       /* enum dm_mut */
    double cxpb;
    double mutpb;
    double alpha;      /* cxBlend */
    double indpb;      /* mutFlipBit / mutGaussian */
    double mu;         /* mutGaussian scalar mean  (used when mu_vec == NULL)    */
    double sigma;      /* mutGaussian scalar sigma (used when sigma_vec == NULL) */
    const double* mu_vec;    /* optional device [dim] */
    const double* sigma_vec; /* optional device [dim] */
} dm_variation;

/* Counter-based RNG coordinates: (seed, island, generation) select the
 * stream; stage/individual/gene select the word. */
typedef struct dm_rng {
    uint64_t seed;
    uint32_t island;
    uint32_t gen;
} dm_rng;

/* Pre-drawn random decisions in DEAP's vocabulary.  INJECT reads them,
 * DUMP writes them; any pointer may be NULL when the operator is unused.
 * Shapes refer to the number of children k and genes dim. */
typedef struct dm_decisions {
    int32_t* aspirants; /* [k][tournsize] selRandom indices (selection.py:24) */
    uint8_t* cx_flag;   /* [k/2] random() < cxpb           (algorithms.py:72) */
    int32_t* cx_raw;    /* [k/2][2] raw randint(1,size), randint(1,size-1)  */
    double* blend_u;    /* [k/2][dim] random() per gene (crossover.py:256)  */
    uint8_t* mut_flag;  /* [k] random() < mutpb            (algorithms.py:78) */
    uint64_t* mut_mask; /* [k][ceil(dim/64)] per-gene random() < indpb      */
    double* gauss;      /* [k][dim] random.gauss(mu,sigma) where masked     */
    int32_t* varor_op;  /* [k] 0 = crossover, 1 = mutation, 2 = reproduction */
    int32_t* varor_idx; /* [k][2] random.sample / random.choice indices      */
} dm_decisions;

typedef struct dm_ctx dm_ctx;

/* ---- context ------------------------------------------------------------- */
const char* dm_last_error(void);
const char* dm_version(void);
int dm_ctx_create(int device, void* hip_stream, dm_ctx** out);
int dm_ctx_destroy(dm_ctx* ctx);
int dm_ctx_set_stream(dm_ctx* ctx, void* hip_stream);
int dm_ctx_sync(dm_ctx* ctx);  /* hipStreamSynchronize on the ctx stream */
/* Zero `bytes` bytes of device memory at `ptr` on the ctx stream
 * (hipMemsetAsync): buffer set-up (population rows, counters, crowding
 * distances) without a host-framework fill kernel. */
int dm_zero(dm_ctx* ctx, void* ptr, int64_t bytes);
/* Measurement hook (no reference counterpart; used by bench.py): record a HIP
 * event pair on the ctx stream around each of the next `max_launches`
 * generation-kernel launches of dm_generation (0 = off).  dm_ctx_kernel_times
 * waits for them and writes up to `cap` durations in ms; *count = pairs
 * recorded. */
int dm_ctx_set_timing(dm_ctx* ctx, int32_t max_launches);
int dm_ctx_kernel_times(dm_ctx* ctx, float* ms, int32_t cap, int32_t* count);
/* Which launches the event pairs bracket: DM_TIME_GENERATION (default, the
 * dm_generation kernel), DM_TIME_DOMINANCE (the all-pairs dominance kernel of
 * dm_sort_nondominated / dm_sel_nsga2), DM_TIME_PEEL (every front-peel
 * launch of the bitset path, in front order; launches issued after the last
 * front exit at once) or DM_TIME_PEEL_CHAIN (each batch of peel launches as
 * one pair). */
enum dm_time_target {
    DM_TIME_GENERATION = 0,
    DM_TIME_DOMINANCE = 1,
    DM_TIME_PEEL = 2,
    DM_TIME_PEEL_CHAIN = 3 /* each batch of front-peel launches as one pair: the chain's GPU time
                              without per-launch events (each event pair adds ~5 us) */
};
int dm_ctx_set_timing_target(dm_ctx* ctx, int32_t target);
/* Dominance path of dm_sort_nondominated / dm_sel_nsga2 (and the log
 * versions): DM_DOM_DEFAULT (bitset tables + table-fed peel for 2-3
 * objectives, integer compare kernel + D-matrix peel for 4, fp64 kernels
 * with NaN or more objectives) or a cross-check path the parity tests
 * compare the default against.  Every path gives the same fronts. */
enum dm_dom_path {
    DM_DOM_DEFAULT = 0,
    DM_DOM_COMPARE = 1,  /* integer compare kernel + D-matrix peel (2-4 objectives) */
    DM_DOM_PEEL_D = 2,   /* bitset rows written as D + D-matrix peel (bitset objectives) */
    DM_DOM_BALLOT = 3,   /* fp64 ballot kernel + peel (2-4 objectives) */
    DM_DOM_LDS = 4       /* fp64 LDS-tiled kernel + peel (any objectives) */
};
int dm_ctx_set_dom_path(dm_ctx* ctx, int32_t path);
/* Re-read the A/B tuning switches (DM_PIPE_BPC, DM_BITS_PP4, ... DESIGN.md
 * §3) from the environment; dm_ctx_create reads them once.  Measurement
 * tools only: every switch selects between bit-identical kernels. */
int dm_ctx_reload_knobs(dm_ctx* ctx);
/* 1 when the context's dominance pass for nobj objectives (NaN-free
 * fitnesses) is the bitset-table pass, else 0 (introspection for tests). */
int dm_ctx_dom_bitset(dm_ctx* ctx, int32_t nobj);

/* ---- RNG (test + init) ---------------------------------------------------- */
/* Raw Philox4x32-10 blocks: out[i*4..i*4+3] = philox(ctr_i, key) with
 * ctr_i = {ctr0[0]+i, ctr0[1], ctr0[2], ctr0[3]}. */
int dm_philox_blocks(dm_ctx* ctx, const uint32_t ctr0[4], const uint32_t key[2],
                     int64_t nblocks, uint32_t* out);

/* Population initialisation (tools.initRepeat/initIterate stand-in,
 * deap/tools/init.py:3-51): bits i.i.d. Bernoulli(1/2), floats U[low, high).
 * Marks every fitness invalid. */
int dm_init_uniform(dm_ctx* ctx, dm_pop* pop, double low, double high, dm_rng rng);

/* ---- evaluation ------------------------------------------------------------ */
/* toolbox.map(toolbox.evaluate, invalid_ind) + fitness.values = fit
 * (algorithms.py:149-152 / :171-174).  only_invalid != 0 evaluates rows
 * with valid == 0 only; *nevals (device int64, may be NULL) is incremented
 * by the number of rows evaluated. */
int dm_evaluate(dm_ctx* ctx, dm_pop* pop, const dm_eval* ev, int only_invalid,
                int64_t* nevals);

/* ---- selection ------------------------------------------------------------- */
/* selTournament (selection.py:51-69): out_idx[k] = winner of tournsize
 * aspirants (selRandom, :12-24); ties keep the first-drawn aspirant,
 * comparison is DEAP's lexicographic Fitness.__gt__ on wvalues. */
int dm_sel_tournament(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t tournsize,
                      dm_rng rng, int32_t mode, const dm_decisions* dec,
                      int32_t* out_idx);
/* selRandom (selection.py:12-24). */
int dm_sel_random(dm_ctx* ctx, int64_t n, int64_t k, dm_rng rng, int32_t mode,
                  const dm_decisions* dec, int32_t* out_idx);
/* selBest (selection.py:27-36): indices of the k best, stable (ties by
 * ascending index), via a device sort of the lexicographic wvalues. */
int dm_sel_best(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx);
/* selWorst (selection.py:39-48), same machinery ascending. */
int dm_sel_worst(dm_ctx* ctx, const dm_pop* pop, int64_t k, int32_t* out_idx);

/* toolbox.clone over a selection (base.py:49, algorithms.py:68):
 * dst row r <- src row idx[r] (genome, wvalues, valid). */
int dm_gather(dm_ctx* ctx, const dm_pop* src, const int32_t* idx, dm_pop* dst);

/* The scatter half of the host-evaluate bridge (a plain Python `evaluate`
 * such as the reference README's evalOneMax, algorithms.py:171-174
 * `ind.fitness.values = fit`): wvalues[idx[i]] = wv[i][0..nobj) and
 * valid[idx[i]] = 1 for i < k (wv: device, k x nobj weighted values).
 * DM_ERR_INDEX if an index is outside [0, pop->n).  Host-synchronising. */
int dm_set_fitness(dm_ctx* ctx, dm_pop* pop, const int32_t* idx, int64_t k, const double* wv);

/* ---- variation / fused generation ----------------------------------------- */
/* One eaSimple generation body (algorithms.py:163-181), fused:
 *   select (per `sel`) -> clone -> varAnd (algorithms.py:33-82) -> evaluate
 *   invalid children (per `ev`, fn NONE = leave them invalid).
 * children->n offspring are produced (children may not alias parents).
 * sel_index is used for DM_SEL_INDEX.  *nevals += #invalid children. */
int dm_generation(dm_ctx* ctx, const dm_pop* parents, dm_pop* children,
                  int32_t sel, int32_t tournsize, const int32_t* sel_index,
                  const dm_variation* var, const dm_eval* ev, dm_rng rng,
                  int32_t mode, const dm_decisions* dec, int64_t* nevals);

/* varOr (algorithms.py:192-245): children->n = lambda offspring from
 * parents, optionally evaluated.  Requires cxpb + mutpb <= 1. */
int dm_var_or(dm_ctx* ctx, const dm_pop* parents, dm_pop* children,
              const dm_variation* var, const dm_eval* ev, dm_rng rng,
              int32_t mode, const dm_decisions* dec, int64_t* nevals);

/* ---- multi-objective selection (deap/tools/emo.py) ----------------------- */
/* sortNondominated (emo.py:53-117).  Outputs, over the n individuals of pop:
 *   order[0..nsorted)   individual indices in DEAP's front order;
 *   front_start[0..nfronts]  offsets into order (front f = order[fs[f]..fs[f+1]));
 *   rank[n]             front index, or -1 if not sorted (truncated).
 * Sorting stops once >= min(n, k) individuals are placed (or after the first
 * front if first_front_only).  Host-synchronising (front count is data
 * dependent).  *nsorted / *nfronts are host pointers. */
int dm_sort_nondominated(dm_ctx* ctx, const dm_pop* pop, int64_t k,
                         int32_t first_front_only, int32_t* order,
                         int32_t* front_start, int32_t* rank,
                         int64_t* nsorted, int32_t* nfronts);
/* assignCrowdingDist (emo.py:119-143) on every front of a sorted order:
 * crowd[order[j]] = crowding distance within its front (weights unapply
 * values = wvalues / weights as in base.py:184-185). weights: host [nobj]. */
int dm_crowding_dist(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                     const int32_t* order, const int32_t* front_start,
                     int32_t nfronts, double* crowd);
/* selNSGA2 (emo.py:15-50), nd='standard': out_idx[k] chosen indices in
 * DEAP's order; crowd[n] receives fitness.crowding_dist of sorted rows.
 * Host-synchronising. */
int dm_sel_nsga2(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                 int64_t k, int32_t* out_idx, double* crowd);
/* sortLogNondominated (emo.py:234-276): the same fronts as
 * dm_sort_nondominated (Fortin's sort computes the same Pareto ranks) in the
 * log version's order: inside a front, unique fitnesses by descending
 * lexicographic wvalues (emo.py:257 fitnesses.sort(reverse=True)), equal
 * fitnesses in population order (emo.py:249-250).  order [n], front_start
 * [n+1] as dm_sort_nondominated.  Host-synchronising. */
int dm_sort_log_nondominated(dm_ctx* ctx, const dm_pop* pop, int64_t k,
                             int32_t first_front_only, int32_t* order,
                             int32_t* front_start, int64_t* nsorted,
                             int32_t* nfronts);
/* selNSGA2(nd='log') (emo.py:15-50 over sortLogNondominated): as
 * dm_sel_nsga2 with crowding on the log-ordered fronts. */
int dm_sel_nsga2_log(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                     int64_t k, int32_t* out_idx, double* crowd);
/* dst[i] = src[idx[i]] for i < n (fitness.crowding_dist carried with a
 * selection's clones, algorithms.py:329 select + base.py:252-261); idx NULL:
 * dst[i] = src[i]. */
int dm_gather_f64(dm_ctx* ctx, const double* src, const int32_t* idx, int64_t n,
                  double* dst);

/* selTournamentDCD (emo.py:145-195): out_idx[4*ceil(k/4)] — for every group
 * of four slots, tournaments (P1[i],P1[i+1]), (P1[i+2],P1[i+3]),
 * (P2[i],P2[i+1]), (P2[i+2],P2[i+3]) where P1, P2 are the two
 * random.sample(individuals, n) permutations; a tournament keeps the
 * dominating individual, else the larger crowd[] (device [n],
 * fitness.crowding_dist), else the first one iff random() <= 0.5.
 * perm1/perm2 [n] and coin [4*ceil(k/4)] (1 = first kept on a tie) are read
 * (INJECT), written (DUMP) or optional scratch (NATIVE).  k > n or
 * (k == n, k % 4 != 0): DM_ERR_INVALID (the reference's ValueError);
 * 4*ceil(k/4) > n: DM_ERR_INDEX (its IndexError). */
int dm_sel_tournament_dcd(dm_ctx* ctx, const dm_pop* pop, const double* crowd, int64_t k,
                          dm_rng rng, int32_t mode, int32_t* perm1, int32_t* perm2,
                          uint8_t* coin, int32_t* out_idx);

/* ---- bounded real-valued variation (NSGA-II example loop) ---------------- */
/* Parameters of cxSimulatedBinaryBounded(eta, low, up) (crossover.py:291-360)
 * and mutPolynomialBounded(eta, low, up, indpb) (mutation.py:51-95).  low/up
 * are the scalars unless low_vec/up_vec (device [dim]) are given. */
typedef struct dm_bounded_var {
    int32_t cx;        /* 1 = apply cxSimulatedBinaryBounded to pairs          */
    int32_t mut;       /* 1 = apply mutPolynomialBounded to both children      */
    double cxpb;       /* pair crossed iff random() <= cxpb (nsga2.py:100)     */
    double eta_cx;
    double eta_mut;
    double indpb;
    double low, up;
    const double* low_vec;
    const double* up_vec;
} dm_bounded_var;

/* The variation body of the NSGA-II loop (examples/ga/nsga2.py:96-105):
 *   offspring = [clone(pop[i]) for i in idx]          (idx NULL: identity)
 *   for ind1, ind2 in zip(offspring[::2], offspring[1::2]):
 *       if random() <= cxpb: cxSimulatedBinaryBounded(ind1, ind2)   (if cx)
 *       mutPolynomialBounded(ind1); mutPolynomialBounded(ind2)      (if mut)
 *       del ind1.fitness.values, ind2.fitness.values
 * children->n = k offspring; an odd last child is a plain clone (fitness
 * kept) — except with cx == 0 (mutation only, the batch form of
 * mutPolynomialBounded), which mutates every child.  F64 genomes only.  Decisions (INJECT read / DUMP write / NATIVE
 * unused, may be NULL): cx_u[k/2] the pair random(); sbx_u[k/2][dim][3] the
 * per-gene (gate, rand, swap) random()s of SBX; mut_u[2*(k/2)][dim][2] the
 * per-gene (gate, rand) random()s of the polynomial mutation ([k] rows when
 * cx == 0).  A value is
 * only consumed where the reference would draw it.  An idx entry outside
 * [0, parents->n) is never dereferenced: its pair's children become NaN rows
 * with invalid fitness. */
int dm_vary_bounded(dm_ctx* ctx, const dm_pop* parents, const int32_t* idx, dm_pop* children,
                    const dm_bounded_var* var, dm_rng rng, int32_t mode, double* cx_u,
                    double* sbx_u, double* mut_u);

/* ---- island migration (deap/tools/migration.py:4-51) --------------------- */
/* Pack rows idx[0..k) of pop into a contiguous emigrant block:
 * [k][stride] genomes, then [k][nobj] wvalues, then [k] valid (padded to 8 B),
 * then [k] int32 source row indices.  dm_pack_bytes gives its size. */
int dm_pack_rows(dm_ctx* ctx, const dm_pop* pop, const int32_t* idx, int64_t k,
                 void* block);
int64_t dm_pack_bytes(const dm_pop* pop, int64_t k);
/* migRing placement for one receiving deme (migration.py:48-51): for j in
 * 0..k-1 in order, slot = first row of the *current* deme whose genome equals
 * immigrant j (list.index value equality), then that row <- emigrant j.
 * immigrants: rows of `pop` as selected before any placement (idx[k]);
 * emigrants: a packed block from dm_pack_rows.  out_slots[k] (device) gets the
 * slots written.  An immigrant absent from the deme is DM_ERR_INVALID (the
 * reference's list.index ValueError).  Host-synchronising. */
int dm_mig_place(dm_ctx* ctx, dm_pop* pop, const void* immigrant_block,
                 const void* emigrant_block, int64_t k, int32_t* out_slots);

/* random.sample(population, k) as migRing's `replacement`
 * (examples/ga/onemax_multidemic.py:46-47, migration.py:42-44): out_idx[k]
 * (device) = k distinct row indices of [0, n) in draw order, from the
 * counter-based RNG (stage SAMPLE).  k > n is DM_ERR_INVALID (the reference's
 * "Sample larger than population" ValueError). */
int dm_sel_sample(dm_ctx* ctx, int64_t n, int64_t k, dm_rng rng, int32_t* out_idx);

/* The hops of one migRing (migration.py:34,48-51: from_deme ->
 * migarray[from_deme], in from_deme order) as seen by rank `me`, given
 * owner[d] = rank holding deme d.  Host-only (no device work): hops[i] =
 * {kind, from, to, peer} with kind DM_HOP_LOCAL (both demes on `me`),
 * DM_HOP_SEND (from on `me`, to on peer) or DM_HOP_RECV (to on `me`, from on
 * peer); hops involving neither side are skipped.  flags & DM_MIG_FORCE_P2P
 * turns every local hop between two different demes into a send/recv pair
 * to `me` itself (exercises the RCCL data path on one GPU). */
enum dm_hop_kind { DM_HOP_LOCAL = 0, DM_HOP_SEND = 1, DM_HOP_RECV = 2 };
enum dm_mig_flags { DM_MIG_FORCE_P2P = 1 };
typedef struct dm_mig_hop {
    int32_t kind, from, to, peer;
} dm_mig_hop;
int dm_mig_plan(int32_t n_demes, const int32_t* migarray, const int32_t* owner, int32_t me,
                int32_t flags, dm_mig_hop* hops, int32_t cap, int32_t* nhops);

/* migRing(populations, k, selection, replacement, migarray) over the demes
 * held by this process (migration.py:4-51), whole migration in one call:
 * every local deme's emigrants (rows emig_idx[i][0..k), the result of
 * `selection`) and immigrants (rows immig_idx[i][0..k) = `replacement`, or
 * the emigrants when immig_idx or immig_idx[i] is NULL) are packed first;
 * then the blocks move along migarray (NULL = ring d -> d+1) and each
 * receiving deme applies the sequential list.index placement (dm_mig_place)
 * in from_deme order.  Host arrays: demes[n_local], deme_ids[n_local] (global
 * ids), emig_idx/immig_idx/out_slots[n_local] of device pointers (out_slots
 * may be NULL; else out_slots[i] receives the k slots written into local deme
 * i by its last incoming hop).  dm_mig_ring: every deme is local
 * (deme_ids = 0..n_demes-1).  Host-synchronising. */
int dm_mig_ring(dm_ctx* ctx, int32_t n_demes, dm_pop* demes, const int32_t* migarray,
                int64_t k, int32_t* const* emig_idx, int32_t* const* immig_idx,
                int32_t* const* out_slots);

/* ---- RCCL communicator for islands across GPUs -------- */
/* One process per GPU; rank 0 creates the unique id and shares its
 * DM_COMM_ID_BYTES bytes out of band (the Python layer broadcasts them over
 * torch.distributed); every rank then calls dm_comm_init collectively. */
#define DM_COMM_ID_BYTES 128
typedef struct dm_comm dm_comm;
int dm_comm_get_unique_id(uint8_t* id_out);
int dm_comm_init(dm_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id, dm_comm** out);
int dm_comm_destroy(dm_comm* comm);
/* dm_mig_ring across ranks: owner[n_demes] (host) gives each deme's rank;
 * this rank holds demes[n_local] with global ids deme_ids[n_local].  Cross-
 * rank hops are grouped ncclSend / ncclRecv of the packed emigrant blocks
 * (ncclGroupStart/End, RCCL point-to-point over xGMI) on the ctx stream;
 * placement is local to the receiver.  Must be called by every rank with the
 * same n_demes / migarray / owner / k — a rank holding no deme included
 * (n_local = 0, demes / deme_ids / emig_idx may be NULL).  With more than one
 * rank, every per-rank check (ids, owners, k against deme sizes, layouts,
 * scratch) runs first and the ranks agree on the outcome (one ncclAllReduce
 * of an ok flag) before any send or receive is posted: a rank whose check
 * failed returns its own error, the others DM_ERR_INVALID, none hangs.
 * flags: DM_MIG_FORCE_P2P. */
int dm_mig_ring_rccl(dm_ctx* ctx, dm_comm* comm, int32_t n_local, dm_pop* demes,
                     const int32_t* deme_ids, int32_t n_demes, const int32_t* migarray,
                     const int32_t* owner, int64_t k, int32_t* const* emig_idx,
                     int32_t* const* immig_idx, int32_t* const* out_slots, int32_t flags);

/* ---- statistics (tools.Statistics / Logbook helpers) --------------------- */
/* tools.Statistics(key=lambda ind: ind.fitness.values) reductions
 * (support.py:199-210) in one pass: per objective j, out[j*8 + {0..7}] =
 * {min, max, mean, m2, sum, argmin, argmax, count} of fitness.values
 * (= wvalues / weights, base.py:184-185) over valid rows, device doubles;
 * m2 = sum of squared deviations from the mean (np.var = m2 / count,
 * np.std = sqrt(np.var)), combined pairwise (Chan et al.); argmin / argmax
 * are first occurrences; a NaN value makes min / max / mean / m2 / sum NaN
 * and argmin / argmax the first NaN row, as numpy's reducers do.  weights:
 * host [nobj].  Asynchronous. */
int dm_fitness_stats(dm_ctx* ctx, const dm_pop* pop, const double* weights,
                     double* out);

#ifdef __cplusplus
}
#endif
#endif /* DEAPMI_H */
