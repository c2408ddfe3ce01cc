/*
 * wsmc.h — C ABI of the MI355X-native SMC inner loop for WeightedSampling.jl.
 *
 * This library replaces the per-particle hot path that sits behind the reference's
 * store / state / operator interface. Each entry point names the reference interface it
 * stands in for (paths relative to the reference repository root):
 *
 *   store      AbstractParticleStore            src/stores.jl:1-35, ColumnStore :70-128
 *   state      SMCState weights / flags         src/types.jl:48-65
 *   operators  apply!(Assign|Sample|Observe|Weight|Resample|Move, state)
 *                                               src/transformers.jl:28, 172, 228, 283, 474, 588
 *   numerics   exp_norm / ess_perc / logsumexp / stratified_resample / icdf
 *                                               src/resampling.jl:13-77
 *   proposals  RW / autoRW                      src/move_kernels.jl:189-253
 *   kernels    default_kernels Normal / MvNormal / Uniform, the example HalfNormal
 *                                               src/default_kernels.jl:83-102,
 *                                               examples/damped_oscillator.jl:24-28
 *   score fold score_logpdf! / score!          src/types.jl:198-206, src/transformers.jl:193-302
 *
 * Conventions
 *   - All functions return WSMC_OK (0) or a nonzero wsmc_status; wsmc_last_error()
 *     returns a thread-local message for the last failure.
 *   - A context owns every device buffer of one particle shard on one GPU. Host pointers
 *     are borrowed for the duration of a call. Downloads synchronise; everything else is
 *     enqueued on the context's stream.
 *   - Columns are particle-major SoA f64: a column of dimension d is d contiguous arrays
 *     of N doubles (component-major), so component k of particle i is data[k*N + i].
 *   - Particle, slot and column indices are 0-based (the reference is 1-based).
 *   - One context per host thread (the reference is single-threaded, src/types.jl:24-26).
 *   - No host pointers to device memory escape except through wsmc_col_device_ptr.
 */
#ifndef WSMC_H
#define WSMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    WSMC_OK = 0,
    WSMC_EARG = 1,     /* invalid argument (reference: ArgumentError, src/move_kernels.jl:26) */
    WSMC_EHIP = 2,     /* HIP runtime failure */
    WSMC_ENOTPD = 3,   /* proposal covariance not positive definite (reference: PosDefException) */
    WSMC_ERCCL = 4,    /* RCCL failure */
    WSMC_ESTATE = 5,   /* operation invalid in the current state */
    WSMC_ENOMEM = 6
} wsmc_status;

typedef struct wsmc_ctx wsmc_ctx;

/* ---- argument forms -------------------------------------------------------
 * The reference passes opaque Julia closures (argfn). The device path accepts the
 * argument shapes @model's `vectorize` produces for the supported kernels: constants
 * (Ref), columns, and affine combinations of up to two column components.
 *   value(i) = c0 + coef[0]*col[0][comp[0]][i] + coef[1]*col[1][comp[1]][i]
 * Unused slots have col = -1.                                                  */
typedef struct {
    double  c0;
    int32_t col[2];
    int32_t comp[2];
    double  coef[2];
} wsmc_operand;

typedef enum {
    WSMC_FAM_NORMAL = 0,        /* Normal(mu, sigma), sigma a std               */
    WSMC_FAM_HALFNORMAL = 1,    /* Truncated(Normal(0, sigma), 0, Inf)          */
    WSMC_FAM_UNIFORM = 2,       /* Uniform(a, b) = param[0], param[1]           */
    WSMC_FAM_MVNORMAL_ISO = 3,  /* MvNormal(mu, var*I), dim <= 4                */
    WSMC_FAM_MVNORMAL = 4,      /* MvNormal(mu, Sigma), constant covariance Sigma, dim <= 3:
                                   build it with wsmc_dist_mvnormal_cov (the factor is
                                   packed into the dist, see wsmc_terms.h)       */
    /* scalar families of src/default_kernels.jl:83-102 with closed-form draws (one uniform
       word pair each) and Distributions.jl's logpdf formulas; location mu[0], scale `scale`: */
    WSMC_FAM_BERNOULLI = 5,     /* Bernoulli(p = mu[0]): x in {0.0, 1.0}            */
    WSMC_FAM_BERNOULLI_LOGIT = 6, /* BernoulliLogit(logitp = mu[0])                   */
    WSMC_FAM_EXPONENTIAL = 7,   /* Exponential(theta = scale), theta the mean       */
    WSMC_FAM_LOGNORMAL = 8,     /* LogNormal(mu, sigma)                             */
    WSMC_FAM_LAPLACE = 9,       /* Laplace(mu, theta)                               */
    WSMC_FAM_CAUCHY = 10,       /* Cauchy(mu, sigma)                                */
    WSMC_FAM_LOGISTIC = 11,     /* Logistic(mu, theta)                              */
    WSMC_FAM_GUMBEL = 12,       /* Gumbel(mu, theta)                                */
    WSMC_FAM_RAYLEIGH = 13,     /* Rayleigh(sigma = scale)                          */
    WSMC_FAM_GEOMETRIC = 14     /* Geometric(p = mu[0]): failures before the first success */
} wsmc_family;

typedef enum {
    WSMC_MEAN_AFFINE = 0,       /* mean component k = mu[k]                      */
    WSMC_MEAN_OSCILLATOR = 1    /* mean = mu[0]*exp(-mu[2]*t)*cos(mu[1]*t+mu[3]), t = param[0]
                                   (examples/damped_oscillator.jl:11)            */
} wsmc_mean_fn;

typedef struct {
    int32_t family;
    int32_t mean_fn;
    int32_t dim;                /* 1 for scalar families */
    int32_t reserved;
    wsmc_operand mu[4];
    wsmc_operand scale;         /* sigma (NORMAL, HALFNORMAL) or variance (MVNORMAL_ISO) */
    double param[2];
} wsmc_dist;

/* MvNormal(mu, Sigma) with a constant covariance Sigma (src/default_kernels.jl:93; the
 * reference builds Distributions' MvNormal, whose PDMat factors Sigma once). On entry d->dim
 * (1..3) and d->mu[0..dim-1] are set; Sigma is dim x dim row-major. Sets family
 * WSMC_FAM_MVNORMAL and packs the Cholesky factor and log det Sigma into d. Host only (no
 * device call). WSMC_EARG: bad dim or Sigma not exactly symmetric (LinearAlgebra.cholesky's
 * ishermitian check); WSMC_ENOTPD: Sigma not positive definite (PosDefException). */
int wsmc_dist_mvnormal_cov(wsmc_dist* d, const double* cov);

typedef enum { WSMC_TERM_SAMPLE = 0, WSMC_TERM_OBSERVE = 1, WSMC_TERM_WEIGHT = 2 } wsmc_term_kind;

/* One entry of the score tape: the statement's log-density contribution as
 * score!(Sample|Observe|Weight) recomputes it (src/transformers.jl:193-199, 243-249, 297-302). */
typedef struct {
    wsmc_dist    dist;
    wsmc_operand x[4];          /* the scored value (Sample: the drawn column) */
    int32_t      kind;
    int32_t      depth;         /* execution depth of the statement (src/types.jl:162-177) */
} wsmc_term;

typedef enum {
    WSMC_RESAMPLE_STRATIFIED = 0,   /* the reference's stratified_resample (src/resampling.jl:35-43) */
    WSMC_RESAMPLE_SYSTEMATIC = 1,   /* one uniform for all strata (north-star addition) */
    WSMC_RESAMPLE_MULTINOMIAL = 2   /* independent draws (north-star addition) */
} wsmc_scheme;
typedef enum { WSMC_PROPOSAL_RW = 0, WSMC_PROPOSAL_AUTORW = 1 } wsmc_proposal;

typedef struct {
    int32_t resampled;          /* SMCState.resampled */
    int32_t weights_changed;    /* SMCState.weights_changed */
    int32_t depth;              /* SMCState.depth */
    int32_t n_terms;            /* score tape length */
    double  last_ess_perc;      /* last ESS/N computed by a Resample */
    uint64_t op_counter;        /* stochastic-statement counter (RNG stream position) */
    int64_t n_resamples;
} wsmc_state;

/* ---- context --------------------------------------------------------------- */
const char* wsmc_last_error(void);
int wsmc_version(int32_t* major, int32_t* minor);
int wsmc_device_count(int32_t* n);
/* SMCState(n_particles; rng) — src/types.jl:62-78. The seed keys the Philox streams. */
int wsmc_create(wsmc_ctx** out, int64_t n_particles, int32_t device, uint64_t seed);
int wsmc_destroy(wsmc_ctx* ctx);
/* SMCState over n_gpus devices in ONE handle ("multi-GPU inside one
 * context"): the population [0, n_particles) is split into n_gpus contiguous shards (ragged),
 * shard g on devices[g] (NULL: device g). transport WSMC_TRANSPORT_RCCL: one communicator per
 * device from ncclCommInitAll (distinct devices); WSMC_TRANSPORT_HOST: records exchanged in
 * host memory between the shards' threads (several shards may share a device). Every other
 * entry point accepts the handle: a call runs on every shard concurrently (one host thread per
 * shard, so each shard's collectives meet the others', as one process per GPU would) and host
 * buffers of n_particles are split / joined by shard. Island sharding by default
 * (wsmc_comm_set_shard_mode applies to every shard). Per-shard-only calls
 * (wsmc_col_device_ptr, wsmc_store_resample, wsmc_debug_kernel_bench) need n_gpus = 1. */
typedef enum { WSMC_TRANSPORT_RCCL = 0, WSMC_TRANSPORT_HOST = 1 } wsmc_transport;
int wsmc_create_multi(wsmc_ctx** out, int64_t n_particles, int32_t n_gpus, const int32_t* devices,
                      uint64_t seed, int32_t transport);
int wsmc_sync(wsmc_ctx* ctx);
int wsmc_nparticles(wsmc_ctx* ctx, int64_t* n);
int wsmc_get_state(wsmc_ctx* ctx, wsmc_state* out);
/* Test hooks used by the reference's own tests (test/move_test.jl:36-37 set state.depth). */
int wsmc_set_depth(wsmc_ctx* ctx, int32_t depth);
int wsmc_set_op_counter(wsmc_ctx* ctx, uint64_t op);

/* ---- multi-GPU shard (one process per GPU) ----------------------------------
 * A context may own the shard [global_offset, global_offset + N) of a global
 * population of global_n particles; RNG streams are keyed by the global index.
 * RCCL is initialised from a unique id distributed by the caller (rank 0 creates it). */
int wsmc_comm_unique_id(uint8_t out_id[128]);
int wsmc_comm_init(wsmc_ctx* ctx, const uint8_t id[128], int32_t world, int32_t rank,
                   int64_t global_offset, int64_t global_n);
/* The same sharding with a host-side exchange instead of RCCL: `exchange` receives this
 * shard's record (`words` u64) and must return every rank's record in rank order in `all`
 * (world * words), returning 0 on success. For hosts that carry their own transport (an
 * MPI binding, a test harness putting several shards on one device); the device path is
 * otherwise identical. */
typedef int (*wsmc_exchange_fn)(void* user, const uint64_t* mine, int32_t words, uint64_t* all);
int wsmc_comm_init_host(wsmc_ctx* ctx, wsmc_exchange_fn exchange, void* user, int32_t world, int32_t rank,
                        int64_t global_offset, int64_t global_n);
/* How a sharded Resample draws:
 *  WSMC_SHARD_ISLAND (default): one record all-gather per step; each shard resamples
 *    within itself and resets to its own log-mean (evidence-preserving). Not the
 *    single-GPU ancestors.
 *  WSMC_SHARD_EXACT: the reference's stratified/systematic Resample over the whole
 *    population — identical bits to one context holding every particle (ancestors as
 *    global indices, columns, weights, evidence): the global max is exchanged first,
 *    the records are summed as integers, each shard fills its contiguous window of
 *    global slots and the particles move to their owners (grouped send/recv).
 * Exact mode covers the statement operators and wsmc_ssm2d_run (history traced back
 * across ranks); multinomial draws on exact shards return WSMC_EARG. */
typedef enum { WSMC_SHARD_ISLAND = 0, WSMC_SHARD_EXACT = 1 } wsmc_shard_mode;
int wsmc_comm_set_shard_mode(wsmc_ctx* ctx, int32_t mode);
/* A watchdog on every wait for the context's stream (each shard's, on a multi-device handle)
 * while it holds an RCCL communicator: a wait longer than `seconds` (a collective whose peer
 * never arrives) aborts the communicator (ncclCommAbort) and the call returns WSMC_ERCCL, so a
 * lost rank ends the job instead of hanging the node. 0 (the default) waits without bound. */
int wsmc_comm_set_timeout(wsmc_ctx* ctx, double seconds);
/* What a context (or a multi-device handle) is sharded over, as the communicator itself
 * reports it — for a benchmark line that must say how many devices it measured (no reference
 * counterpart: the reference is single-threaded, /root/reference/TODO.md:28).
 *   shards      shards in this handle (1 for a plain context, G for wsmc_create_multi)
 *   world/rank  the sharding (world 1: unsharded)
 *   rccl_ranks  ncclCommCount of the (first) shard's communicator, 0 when it has none
 *   transport   WSMC_TRANSPORT_RCCL, WSMC_TRANSPORT_HOST, or -1 (unsharded)
 *   shard_mode  WSMC_SHARD_ISLAND / WSMC_SHARD_EXACT
 *   devices[g], shard_n[g]  HIP device and particle count of shard g < min(shards, 8) */
typedef struct {
    int32_t shards, world, rank, rccl_ranks, transport, shard_mode;
    int32_t devices[8];
    int64_t shard_n[8];
} wsmc_comm_info_t;
int wsmc_comm_info(wsmc_ctx* ctx, wsmc_comm_info_t* out);

/* ---- store: AbstractParticleStore (src/stores.jl:1-35) ----------------------- */
/* broadcast_setcol! column creation (src/stores.jl:85-96); existing name => same id */
int wsmc_col_create(wsmc_ctx* ctx, const char* name, int32_t dim, int32_t* col_id);
/* hascol / lookup; *col_id = -1 when absent */
int wsmc_col_find(wsmc_ctx* ctx, const char* name, int32_t* col_id);
/* colnames (insertion order) */
int wsmc_col_count(wsmc_ctx* ctx, int32_t* n);
int wsmc_col_info(wsmc_ctx* ctx, int32_t col_id, char* name_buf, int32_t buf_len, int32_t* dim);
/* getcol (host copy, synchronising) */
int wsmc_col_download(wsmc_ctx* ctx, int32_t col_id, double* host);
/* broadcast_setcol!(store, name, identity, (v,)) with a host vector */
int wsmc_col_upload(wsmc_ctx* ctx, int32_t col_id, const double* host);
/* device pointer of the live buffer (valid until the next resample/gather) */
int wsmc_col_device_ptr(wsmc_ctx* ctx, int32_t col_id, double** dptr);
/* resample!(store, indices) with caller-supplied 0-based indices (src/stores.jl:105-128) */
int wsmc_store_resample(wsmc_ctx* ctx, const int32_t* host_indices);
/* Lazy genealogy of the store (the default; ColumnStore.resample! gathers every column at
 * every resample, src/stores.jl:105-128, which is O(T^2 N) over a run that keeps a history
 * column per step). A Resample logs its int32 ancestors and gathers only the columns an
 * operator touched since the previous Resample; the others are brought up to date, all in
 * one trace over the log, when a later operator or getcol reads one. Values are bit-identical
 * to the eager gathers (a gather is a copy). lazy = 0 restores the eager gathers (after
 * bringing every column up to date); exact shards are always eager.
 * wsmc_store_info: log entries held and columns currently behind the log. */
int wsmc_store_set_lazy(wsmc_ctx* ctx, int32_t lazy);
/* bring every column up to date now (one trace over the log; what a DataFrame(state) export
 * or a run's end needs), without a host copy */
int wsmc_store_materialize(wsmc_ctx* ctx);
int wsmc_store_info(wsmc_ctx* ctx, int64_t* log_entries, int32_t* stale_columns);

/* ---- weights: SMCState.weights (src/types.jl:48-60) ------------------------- */
int wsmc_weights_upload(wsmc_ctx* ctx, const double* host);
int wsmc_weights_download(wsmc_ctx* ctx, double* host);
/* logsumexp(weights) - log(N)  (src/utils.jl:21) */
int wsmc_log_evidence(wsmc_ctx* ctx, double* out);

/* ---- analysis reductions (src/utils.jl), no N-sized download -------------------------
 * Weighted moments under w = exp_norm(weights) of up to 4 expressions (operand form):
 * mean[k] = sum w_i v_k(i) / sum w_i           expectation / @E (src/utils.jl:11, 23-58)
 * cov[a*d+b] = sum w_i (v_a - mean_a)(v_b - mean_b) / sum w_i
 *                                             describe's std(..., corrected=false) (:233-240)
 * in the canonical reduction order of the autoRW moments; cov may be NULL. */
int wsmc_weighted_moments(wsmc_ctx* ctx, const wsmc_operand* exprs, int32_t d, double* mean, double* cov);
/* unweighted minimum / maximum of a column component (describe, src/utils.jl:238-239) */
int wsmc_col_minmax(wsmc_ctx* ctx, int32_t col_id, int32_t comp, double* min_out, double* max_out);
/* ess_perc(exp_norm(weights)) (src/resampling.jl:51-54) without resampling or any state change */
int wsmc_ess(wsmc_ctx* ctx, double* ess_perc);
/* describe()'s weighted median (StatsBase.quantile(v, Weights(w), 0.5)) and 8-bin sparkline
 * histogram levels (1..8, src/utils.jl:134-141) of one column component, on the integer
 * weights (include/wsmc_math.h). On shards both are population-wide: the median takes the
 * union of every rank's (value, q) pairs, the sparkline sums integer bins taken at the
 * population's max log-weight — the bits of one context holding every particle. */
int wsmc_weighted_median(wsmc_ctx* ctx, int32_t col_id, int32_t comp, double* out);
int wsmc_histogram(wsmc_ctx* ctx, int32_t col_id, int32_t comp, int32_t levels[8]);
/* sample(state, n; replace) (src/utils.jl:92-118): n particle indices (0-based) drawn by
 * the normalised weights — with replacement independent draws in draw order, without
 * replacement the n largest Efraimidis–Spirakis keys (include/wsmc_math.h wsmc_es_key).
 * Consumes one op counter (the reference draws from the global RNG). WSMC_EARG for n <= 0
 * or (!replace && n > N), as the reference's ArgumentError. On shards the indices are
 * global and the draws are the single-context draws (each target located by the rank whose
 * CDF range holds it; without replacement the union of the ranks' top-n keys). */
int wsmc_sample_particles(wsmc_ctx* ctx, int64_t n, int32_t replace, int64_t* idx_out);
/* rows idx[0..n) of a column, [dim][n] (getcol(store, c)[indices], src/utils.jl:117) */
int wsmc_col_gather_rows(wsmc_ctx* ctx, int32_t col_id, const int64_t* idx, int64_t n, double* out);

/* ---- operators (apply!) ------------------------------------------------------ */
/* Assign: out[k] .= expr[k] for k < dim(out)            src/transformers.jl:28-32 */
int wsmc_assign(wsmc_ctx* ctx, int32_t out_col, const wsmc_operand* expr);
/* Assign of a general expression: out[k] .= f_k(columns...) for k < dim(out).
 * The reference's `vectorize` (src/rewrites.jl:146-219) turns the right-hand side into one
 * fused broadcast over the columns: calls f.(args...), `cond ? a : b` as ifelse.(...),
 * `a || b` / `a && b` as .| / .&, `x[j]` component reads. The device form is one postfix
 * program per output component, the components' programs back to back in `prog`, len[k]
 * instructions for component k (k < dim(out)); at most WSMC_XPROG_MAX instructions in all and
 * WSMC_XSTACK_MAX values on the stack. Binary operators pop b (the top) then a and push
 * f(a, b); each component's program must leave exactly one value. The arithmetic is
 * wsmc_xop1 / wsmc_xop2 (include/wsmc_terms.h). Columns read one lazy Resample behind are
 * read through its ancestors (as wsmc_assign). WSMC_EARG: a malformed program, an unknown
 * column or component. Domain errors Julia throws (sqrt / log of a negative, a negative
 * base to a fractional power) give NaN. */
typedef enum {
    WSMC_X_CONST = 0,   /* push c                                                         */
    WSMC_X_COL = 1,     /* push column col, component comp                                */
    WSMC_X_NEG = 2, WSMC_X_ABS = 3, WSMC_X_SQRT = 4, WSMC_X_EXP = 5, WSMC_X_LOG = 6,
    WSMC_X_LOG1P = 7, WSMC_X_SIN = 8, WSMC_X_COS = 9,
    WSMC_X_POWI = 10,   /* a^n, n = c (an integer, |n| < 2^62): Base.literal_pow for
                           n in -2..3, else Base's compensated power by squaring       */
    WSMC_X_NOT = 11,    /* !a: 1 if a == 0 else 0                                        */
    WSMC_X_ADD = 16, WSMC_X_SUB = 17, WSMC_X_MUL = 18, WSMC_X_DIV = 19,
    WSMC_X_MIN = 20, WSMC_X_MAX = 21,   /* Base.min / max (NaN-propagating, -0.0 < 0.0)   */
    WSMC_X_POW = 22,    /* a^b: integer b as POWI, else exp(b * log(a))                   */
    WSMC_X_LT = 23, WSMC_X_LE = 24, WSMC_X_GT = 25, WSMC_X_GE = 26, WSMC_X_EQ = 27,
    WSMC_X_NE = 28,     /* comparisons: 1.0 / 0.0                                         */
    WSMC_X_AND = 29, WSMC_X_OR = 30,    /* (a != 0) & (b != 0), (a != 0) | (b != 0)       */
    WSMC_X_IFELSE = 31  /* pops f, t, cond: cond != 0 ? t : f (both evaluated)            */
} wsmc_xop;
typedef struct {
    int32_t op;         /* wsmc_xop */
    int32_t col;        /* WSMC_X_COL: the column */
    int32_t comp;       /* WSMC_X_COL: its component */
    int32_t reserved;
    double  c;          /* WSMC_X_CONST: the value; WSMC_X_POWI: the exponent */
} wsmc_xinst;
#define WSMC_XPROG_MAX 96
#define WSMC_XSTACK_MAX 8
int wsmc_assign_expr(wsmc_ctx* ctx, int32_t out_col, const wsmc_xinst* prog, const int32_t* len);
/* Sample: out ~ dist (weighter === nothing)            src/transformers.jl:172-182 */
int wsmc_sample(wsmc_ctx* ctx, int32_t out_col, const wsmc_dist* dist);
/* Sample with importance_kernel(proposal, target)      src/default_kernels.jl:69-73 */
int wsmc_sample_importance(wsmc_ctx* ctx, int32_t out_col, const wsmc_dist* proposal,
                           const wsmc_dist* target);
/* Observe: weights .+= logpdf(dist, x)                  src/transformers.jl:228-235 */
int wsmc_observe(wsmc_ctx* ctx, const wsmc_dist* dist, const wsmc_operand* x);
/* Weight (_ ~ f(args)): weights .+= logpdf(dist, x)     src/transformers.jl:283-289 */
int wsmc_weight(wsmc_ctx* ctx, const wsmc_dist* dist, const wsmc_operand* x);
/* Resample (gated on weights_changed, strict ESS test, log-mean reset)
 *                                                       src/transformers.jl:474-498
 *   resampled_out / ess_perc_out both NULL: asynchronous — the decision stays on the device
 *   (gated gather and weight reset, no host wait) and is folded into wsmc_get_state's
 *   resampled / n_resamples / last_ess_perc at the next read (exact shards always wait). */
int wsmc_resample(wsmc_ctx* ctx, double ess_perc_min, int32_t scheme,
                  int32_t* resampled_out, double* ess_perc_out);
/* Move with RW / autoRW (src/transformers.jl:588-623, src/move_kernels.jl:189-253).
 *   targets: d <= 4 scalar columns; lo/hi: per-target bounds (NULL = unbounded);
 *   step: RW step size (std) or autoRW min_step; target_depth: state.depth at the move
 *   (pass -1 to use the context's current depth); diversity: NaN = ungated.
 *   *accepted_out (may be NULL) receives the number of accepted proposals. With
 *   accepted_out NULL the Move is asynchronous (no host wait, as the reference's Move
 *   returns nothing): a not-positive-definite autoRW covariance leaves the Move's targets
 *   untouched and is reported as WSMC_ENOTPD by the next synchronizing call (wsmc_sync,
 *   get_state, a download, a waited Resample or Move). Operators enqueued in between have
 *   run (later asynchronous Moves skip on the same flag): nothing is rolled back, the state
 *   is the one those statements produce with the failed Moves left out, where the reference
 *   would have thrown at the failing Move. Callers that need the reference's stop-at-the-
 *   failure behaviour pass accepted_out.                                                  */
int wsmc_move(wsmc_ctx* ctx, int32_t proposal, const int32_t* targets, int32_t d, double step,
              const double* lo, const double* hi, int32_t target_depth, double diversity,
              int64_t* accepted_out);
/* Move.apply! inside `if resampled ... end` (the Cond of src/rewrites.jl:360-368;
 * examples/linear_regression.jl:23-24, examples/damped_oscillator.jl:38-41) with the condition
 * decided on the device: the Move runs only if the last Resample resampled, and the host never
 * reads the flag (an asynchronous Resample followed by gated Moves keeps the whole step on the
 * stream). Asynchronous like wsmc_move with accepted_out NULL. A gated Move consumes its two
 * op counters whether or not it runs, so its streams do not depend on the decision. With a
 * diversity gate or on shards the decision is read on the host first.                       */
int wsmc_move_gated(wsmc_ctx* ctx, int32_t proposal, const int32_t* targets, int32_t d, double step,
                    const double* lo, const double* hi, int32_t target_depth, double diversity);
/* One Move of a block (wsmc_move_block): wsmc_move's arguments without the diversity gate. */
typedef struct {
    int32_t proposal;        /* WSMC_PROPOSAL_RW / WSMC_PROPOSAL_AUTORW */
    int32_t d;               /* 1..4 targets */
    int32_t targets[4];
    int32_t bounded;         /* 0: lo / hi ignored (wsmc_move's NULL lo and hi) */
    int32_t target_depth;    /* < 0: the current depth */
    double step;             /* RW step / autoRW min_step */
    double lo[4], hi[4];
} wsmc_move_spec;
/* A statement block of consecutive Moves — `α << autoRW(); β << autoRW()` in the body of
 * `if resampled ... end` (examples/linear_regression.jl:23-24) or a sweep of
 * examples/damped_oscillator.jl:38-41 without its diversity gate: exactly n wsmc_move calls
 * in order (gated != 0: n wsmc_move_gated calls), the same results bit for bit, op counters
 * taken two per Move in order. Autorw Moves on disjoint targets (4 at most in all) with one
 * target depth run as one moments pass, one combine and one Move kernel; anything else runs
 * the Moves one by one. accepted_out: n counts (synchronizing, the ENOTPD check of the first
 * failing Move as wsmc_move's) or NULL (asynchronous).                                     */
int wsmc_move_block(wsmc_ctx* ctx, int32_t n, const wsmc_move_spec* specs, int32_t gated, int64_t* accepted_out);
/* score_logpdf!(scores, state, targets, target_depth) (src/types.jl:198-206) -> host */
int wsmc_score(wsmc_ctx* ctx, int32_t target_depth, double* host_scores);
/* marginal_diversity(store, targets)  (src/transformers.jl:560-565) */
int wsmc_marginal_diversity(wsmc_ctx* ctx, const int32_t* targets, int32_t d, double* out);
/* the last resample's ancestors (0-based; debug/parity; synchronising); a multi-device
 * handle returns population indices (island shards resample within their own range) */
int wsmc_last_ancestors(wsmc_ctx* ctx, int32_t* host);

/* ---- fused runners (whole model loops; one HIP graph per run) ------------------
 * 2D SSM bootstrap filter (examples/2D_ssm.jl:7-17) on a fresh context:
 *   x{1} .= x0; v .= v0; for t: x{t+1} .= x{t} + v; dv ~ MvNormal(0, q_var I);
 *   v .= v + dv; o_t => MvNormal(x{t+1}, r_var I)   (+ the auto-inserted Resamples)
 * Columns created: x_1 .. x_{T+1} (dim 2, when keep_history), x (dim 2, otherwise), v, dv.
 * Produces the same columns, weights and RNG stream positions as issuing the same
 * statements one by one through the operators above.                                   */
int wsmc_ssm2d_run(wsmc_ctx* ctx, const double* obs /* T x 2, row-major */, int32_t T,
                   const double* x0, const double* v0, double q_var, double r_var,
                   double ess_perc_min, int32_t scheme, int32_t keep_history,
                   double* log_evidence_out);
/* per-kernel timing of the last fused run (HIP events on the ctx stream), ms */
typedef struct {
    double total_ms;            /* whole run, first kernel to last                       */
    double propagate_ms;        /* sum over steps of the propagate/observe kernel         */
    double reduce_ms;           /* sum over steps of the weight-statistics kernel         */
    double resample_ms;         /* sum over steps of the scan/ancestor kernel             */
    double finalize_ms;         /* trace-back + final gather                              */
    int32_t steps;
    int32_t n_resamples;
} wsmc_run_timing;
int wsmc_run_set_timing(wsmc_ctx* ctx, int32_t enabled);
int wsmc_run_get_timing(wsmc_ctx* ctx, wsmc_run_timing* out);

/* ---- diagnostics ---------------------------------------------------------------
 * Average time (us) of `iters` back-to-back launches of one resample kernel on the
 * context's current weights: kernel 0 = weight statistics, 1 = reduce, 2 = ancestor scan;
 * mode 0 = production variant, > 0 = ablations (see csrc/wsmc_kernels.hip).        */
int wsmc_debug_kernel_bench(wsmc_ctx* ctx, int32_t kernel, int32_t mode, int32_t iters, double* avg_us);
/* Test hook: shard `shard` of the handle (0 for a single context) fails its nth next shard
 * record exchange (a Resample's or an evidence query's) with WSMC_EHIP before exchanging.
 * On a multi-device handle the other shards then leave their exchange with WSMC_ERCCL
 * instead of waiting for it; shards that left in different states mark the handle failed
 * (every later call returns WSMC_ESTATE). nth = 0 disarms. nth >= 1000: the failure is a
 * WSMC_EARG at exchange nth - 1000 (an argument error one shard meets alone past an exchange:
 * it requests the abort at once rather than waiting for peers that meet the same error). */
int wsmc_debug_inject_failure(wsmc_ctx* ctx, int32_t shard, int32_t nth);
/* Exact-sharded fused run: the fixed neighbour block (slots per step) and
 * trace window (ids per level) sizes — > 0 sets, 0 restores the defaults, < 0 leaves as is —
 * and, in stats_out[6] (may be NULL), the last run's largest block needed, its largest
 * lineage excursion, the runs re-done on the eager path after a block overflow, the block
 * size, the runs whose history was traced across ranks after a window overflow, and 1 when
 * later runs ship no trace windows (lineages wander past half a shard). */
int wsmc_debug_exact(wsmc_ctx* ctx, int64_t cap, int64_t ctr, int64_t* stats_out);
/* Statement batches compiled for their shape at run time (hiprtc; csrc/wsmc_jit.hip):
 * stats_out[5] = signatures compiled, signatures that failed to compile (their batches run on
 * the interpreter kernel), batches launched on compiled kernels, batches run on the
 * interpreter, total compile time (us) — process-wide. */
int wsmc_debug_jit_stats(int64_t* stats_out);
/* Compile a representative batch signature (the 2D SSM step) for gfx950 without a device:
 * WSMC_OK, or WSMC_EHIP with hiprtc's log in wsmc_last_error(). */
int wsmc_debug_jit_selfcheck(void);
/* The Move acceptance screen (csrc/wsmc_kernels.hip move_accept) on the current device: for each
 * u[i], out[2i] = the single-precision estimate of log u and out[2i+1] = the restated double log,
 * so a test can check the screen's band bound. Host buffers of n and 2n doubles. */
int wsmc_debug_log_screen(const double* u, int64_t n, double* out);
/* Move blocks compiled for their shape at run time (hiprtc; csrc/wsmc_mv_body.h): stats_out[5]
 * = signatures compiled, signatures that failed to compile, blocks launched on compiled kernels,
 * blocks run on the interpreter kernels, total compile time (us) — process-wide. */
int wsmc_debug_mv_jit_stats(int64_t* stats_out);
/* Compile a representative Move block (C3's shape) for gfx950 without a device: WSMC_OK, or
 * WSMC_EHIP with hiprtc's log in wsmc_last_error(). */
int wsmc_debug_mv_jit_selfcheck(void);
/* The fused 2D-SSM run's Resample statistics, cumulative over the context's
 * runs: stats_out[0] = the steps whose propagate guessed the reference point wrong (one GPU: found
 * by the fill; sharded: recomputed in place, k_rs_qfix), stats_out[1] = where the statistics are
 * taken (0 = their own kernel, 1 = the propagate with q stored, 2 = the propagate, the fill
 * recomputing q), stats_out[2] = the runs re-done on the exact path after a miss (one GPU),
 * stats_out[3] = the generic Resamples whose statistics the statement batch took (round 6; its
 * misses, recomputed by k_rs_qfix, count in stats_out[0]). stats_out holds 4 values. */
int wsmc_debug_run_stats(wsmc_ctx* ctx, int64_t* stats_out);

#ifdef __cplusplus
}
#endif
#endif /* WSMC_H */
