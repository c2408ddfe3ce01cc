/*
 * wsmc_oracle.c — CPU restatement of the WeightedSampling.jl SMC inner loop.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline. The product (weightedsampling.jl_amd) never links or calls it.
 *
 * Parity status: the reference is Julia and no Julia toolchain exists here (SURVEY.md
 * §8c), so the reference cannot be executed. This restatement is pinned by
 *   (1) the reference's own known-answer tests re-run against it
 *       (test/score_test.jl:20-54 fold + depth cutoff; test/importance_kernel_test.jl:18-19
 *        exact weighter; test/move_test.jl:23-58 cancellation; test/move_test.jl:116-208
 *        diversity gating), and
 *   (2) the analytic oracles the reference's tests use (Kalman evidence,
 *       test/models.jl:272-288; conjugate-normal posterior, test/move_test.jl:69-98),
 * at the reference's tolerances; see tests/test_oracle.py. Bit-level parity with the
 * Julia RNG stream is impossible by construction, so the HIP path is
 * checked bit-exactly against THIS restatement on the shared Philox streams.
 *
 * Structure follows the reference step by step (file:line cited at each function):
 *   store        ColumnStore, eager ping-pong gather of EVERY column at each resample
 *                (src/stores.jl:105-128) — deliberately the reference's O(#cols) cost
 *   operators    src/transformers.jl:28-32, 172-182, 228-235, 283-289, 474-498, 588-623
 *   numerics     src/resampling.jl:13-77 on the integer CDF of wsmc_math.h
 *   proposals    src/move_kernels.jl:116-253
 * Island resampling for G > 1 shards is the build's documented multi-GPU semantics
 * (DESIGN.md §5): global ESS decision, per-shard stratified resampling, per-shard
 * log-mean reset (evidence preserving, src/transformers.jl:446-459).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "wsmc.h"
#include "wsmc_math.h"
#include "wsmc_terms.h"

#define OR_MAX_COLS 4096
#define OR_MAX_SHARDS 64
#define OR_TILE 2048
#define OR_BLOCK 256

typedef struct {
    char name[64];
    int32_t dim;
    double* front;
    double* back;
} or_col;

typedef struct oracle {
    int64_t N;
    uint64_t seed;
    int32_t ncols;
    or_col cols[OR_MAX_COLS];
    double* colptr[OR_MAX_COLS];
    double* w;                 /* SMCState.weights */
    int32_t resampled, weights_changed, depth;
    double last_ess;
    uint64_t op;
    int64_t n_resamples;
    wsmc_term* tape;
    int32_t nterms, cap_terms;
    int32_t nshards;
    int32_t exact;     /* exact sharding: Resample/ESS/evidence over the whole population */
    int64_t shard_off[OR_MAX_SHARDS + 1];
    int64_t goff;              /* global index of particle 0 (one shard of a multi-process run) */
    int32_t* last_anc;
    double* scratch;
    double* tmp;               /* 4*N staging for statements that read their own output */
} oracle;

/* ------------------------------------------------------------------------- */
oracle* or_create(int64_t N, uint64_t seed) {
    if (N <= 0) return NULL;
    oracle* o = (oracle*)calloc(1, sizeof(oracle));
    o->N = N;
    o->seed = seed;
    o->w = (double*)calloc((size_t)N, sizeof(double));   /* zeros(N), src/types.jl:63 */
    o->last_anc = (int32_t*)calloc((size_t)N, sizeof(int32_t));
    o->scratch = (double*)calloc((size_t)N, sizeof(double));
    o->tmp = (double*)calloc((size_t)(4 * N), sizeof(double));
    o->nshards = 1;
    o->shard_off[0] = 0;
    o->shard_off[1] = N;
    o->last_ess = WSMC_NAN;
    return o;
}

void or_destroy(oracle* o) {
    if (!o) return;
    for (int c = 0; c < o->ncols; ++c) { free(o->cols[c].front); free(o->cols[c].back); }
    free(o->w); free(o->last_anc); free(o->scratch); free(o->tmp); free(o->tape);
    free(o);
}

/* WSMC_SHARD_EXACT: the device shards resample the whole population (the single-context
 * bits) while the autoRW moments stay per-shard canonical sums in rank order */
void or_set_shard_exact(oracle* o, int32_t exact) { o->exact = exact != 0; }
/* the partition Resample / ESS / evidence use: the shards, or one part when exact */
static int rs_parts(const oracle* o, int64_t* off) {
    if (o->exact) { off[0] = 0; off[1] = o->N; return 1; }
    for (int g = 0; g <= o->nshards; ++g) off[g] = o->shard_off[g];
    return o->nshards;
}

int or_set_shards(oracle* o, int32_t G) {
    if (G < 1 || G > OR_MAX_SHARDS || G > o->N) return -1;
    o->nshards = G;
    for (int g = 0; g <= G; ++g) o->shard_off[g] = (o->N * g) / G;
    return 0;
}

int64_t or_nparticles(oracle* o) { return o->N; }
void or_set_global_offset(oracle* o, int64_t goff) { o->goff = goff; }
uint64_t or_get_op(oracle* o) { return o->op; }
void or_set_op(oracle* o, uint64_t op) { o->op = op; }
int32_t or_get_depth(oracle* o) { return o->depth; }
void or_set_depth(oracle* o, int32_t d) { o->depth = d; }
int32_t or_resampled(oracle* o) { return o->resampled; }
int32_t or_weights_changed(oracle* o) { return o->weights_changed; }
double or_last_ess(oracle* o) { return o->last_ess; }
int64_t or_n_resamples(oracle* o) { return o->n_resamples; }
int32_t or_nterms(oracle* o) { return o->nterms; }
double* or_weights(oracle* o) { return o->w; }
int32_t* or_last_anc(oracle* o) { return o->last_anc; }

/* ---- store (src/stores.jl:85-128) ---------------------------------------- */
int32_t or_col_find(oracle* o, const char* name) {
    for (int c = 0; c < o->ncols; ++c)
        if (strncmp(o->cols[c].name, name, 63) == 0) return c;
    return -1;
}
int32_t or_col_create(oracle* o, const char* name, int32_t dim) {
    int32_t c = or_col_find(o, name);
    if (c >= 0) return o->cols[c].dim == dim ? c : -1;
    if (o->ncols >= OR_MAX_COLS || dim < 1 || dim > 4) return -1;
    c = o->ncols++;
    strncpy(o->cols[c].name, name, 63);
    o->cols[c].dim = dim;
    o->cols[c].front = (double*)calloc((size_t)(dim * o->N), sizeof(double));
    o->cols[c].back = (double*)calloc((size_t)(dim * o->N), sizeof(double));
    o->colptr[c] = o->cols[c].front;
    return c;
}
int32_t or_col_dim(oracle* o, int32_t c) { return o->cols[c].dim; }
int32_t or_col_count(oracle* o) { return o->ncols; }
const char* or_col_name(oracle* o, int32_t c) { return o->cols[c].name; }
double* or_col_data(oracle* o, int32_t c) { return o->cols[c].front; }

/* resample!(store, indices): gather every column front->back, swap (src/stores.jl:105-111) */
void or_store_resample(oracle* o, const int32_t* idx) {
    int64_t N = o->N;
    // resample!(store, idx) with caller indices: they are the last ancestors too
    if (idx != o->last_anc) memcpy(o->last_anc, idx, sizeof(int32_t) * (size_t)N);
    for (int c = 0; c < o->ncols; ++c) {
        or_col* col = &o->cols[c];
        for (int k = 0; k < col->dim; ++k) {
            const double* src = col->front + (int64_t)k * N;
            double* dst = col->back + (int64_t)k * N;
            for (int64_t i = 0; i < N; ++i) dst[i] = src[idx[i]];
        }
        double* t = col->front; col->front = col->back; col->back = t;
        o->colptr[c] = col->front;
    }
}

static void or_tape_push(oracle* o, const wsmc_term* t) {
    if (o->nterms == o->cap_terms) {
        o->cap_terms = o->cap_terms ? 2 * o->cap_terms : 64;
        o->tape = (wsmc_term*)realloc(o->tape, (size_t)o->cap_terms * sizeof(wsmc_term));
    }
    o->tape[o->nterms++] = *t;
}

static wsmc_operand col_operand(int32_t col, int32_t comp) {
    wsmc_operand r;
    memset(&r, 0, sizeof(r));
    r.col[0] = col; r.comp[0] = comp; r.coef[0] = 1.0;
    r.col[1] = -1;
    return r;
}

/* ---- operators -------------------------------------------------------------- */
/* Assign (src/transformers.jl:28-32) */
int or_assign(oracle* o, int32_t out, const wsmc_operand* expr) {
    int64_t N = o->N;
    int dim = o->cols[out].dim;
    double* tmp = o->tmp;
    for (int k = 0; k < dim; ++k)
        for (int64_t i = 0; i < N; ++i)
            tmp[(int64_t)k * N + i] = wsmc_operand_eval(&expr[k], o->colptr, N, i, 0);
    memcpy(o->cols[out].front, tmp, sizeof(double) * (size_t)(dim * N));
    o->depth += 1;
    return 0;
}

/* Assign of a general expression (src/transformers.jl:28-32 over the fused broadcast
   src/rewrites.jl:146-219 emits): component k of every particle by wsmc_xeval */
int or_assign_expr(oracle* o, int32_t out, const wsmc_xinst* prog, const int32_t* len) {
    int64_t N = o->N;
    int dim = o->cols[out].dim;
    if (wsmc_xprog_check(prog, len, dim)) return -1;
    double* tmp = o->tmp;
    int pc = 0;
    for (int k = 0; k < dim; ++k) {
        for (int64_t i = 0; i < N; ++i)
            tmp[(int64_t)k * N + i] = wsmc_xeval(prog + pc, len[k], o->colptr, N, i);
        pc += len[k];
    }
    memcpy(o->cols[out].front, tmp, sizeof(double) * (size_t)(dim * N));
    o->depth += 1;
    return 0;
}

static void sample_into(oracle* o, int32_t out, const wsmc_dist* d, uint64_t op, double* tmp) {
    int64_t N = o->N;
    int dim = o->cols[out].dim;
    for (int64_t i = 0; i < N; ++i) {
        double x[4];
        wsmc_dist_sample(d, x, o->seed, op, (uint64_t)(o->goff + i), o->colptr, N, i);
        for (int k = 0; k < dim; ++k) tmp[(int64_t)k * N + i] = x[k];
    }
}

/* Sample (src/transformers.jl:172-182), weighter === nothing */
int or_sample(oracle* o, int32_t out, const wsmc_dist* d) {
    int64_t N = o->N;
    int dim = o->cols[out].dim;
    if (d->dim != dim) return -1;
    uint64_t op = o->op++;
    sample_into(o, out, d, op, o->tmp);
    memcpy(o->cols[out].front, o->tmp, sizeof(double) * (size_t)(dim * N));
    wsmc_term t;
    memset(&t, 0, sizeof(t));
    t.dist = *d;
    for (int k = 0; k < 4; ++k) t.x[k] = col_operand(k < dim ? out : -1, k);
    t.kind = WSMC_TERM_SAMPLE;
    t.depth = o->depth;
    or_tape_push(o, &t);
    o->depth += 1;
    return 0;
}

/* Sample with importance_kernel(proposal, target): weighter = lp_target - lp_proposal,
 * logpdf field = target (src/default_kernels.jl:69-73) */
int or_sample_importance(oracle* o, int32_t out, const wsmc_dist* prop, const wsmc_dist* targ) {
    int64_t N = o->N;
    int dim = o->cols[out].dim;
    if (prop->dim != dim || targ->dim != dim) return -1;
    uint64_t op = o->op++;
    sample_into(o, out, prop, op, o->tmp);
    memcpy(o->cols[out].front, o->tmp, sizeof(double) * (size_t)(dim * N));
    for (int64_t i = 0; i < N; ++i) {
        double x[4];
        for (int k = 0; k < dim; ++k) x[k] = o->cols[out].front[(int64_t)k * N + i];
        double lt = wsmc_dist_logpdf(targ, x, o->colptr, N, i, 0);
        double lp = wsmc_dist_logpdf(prop, x, o->colptr, N, i, 0);
        o->w[i] = o->w[i] + (lt - lp);
    }
    o->weights_changed = 1;
    wsmc_term t;
    memset(&t, 0, sizeof(t));
    t.dist = *targ;
    for (int k = 0; k < 4; ++k) t.x[k] = col_operand(k < dim ? out : -1, k);
    t.kind = WSMC_TERM_SAMPLE;
    t.depth = o->depth;
    or_tape_push(o, &t);
    o->depth += 1;
    return 0;
}

static int or_weigh(oracle* o, const wsmc_dist* d, const wsmc_operand* x, int kind) {
    int64_t N = o->N;
    wsmc_term t;
    memset(&t, 0, sizeof(t));
    t.dist = *d;
    for (int k = 0; k < 4; ++k) t.x[k] = x[k < d->dim ? k : 0];
    t.kind = kind;
    t.depth = o->depth;
    wsmc_osc_link(o->nterms ? &o->tape[o->nterms - 1] : 0, &t);   /* before its first evaluation */
    for (int64_t i = 0; i < N; ++i) o->w[i] = o->w[i] + wsmc_term_logpdf(&t, o->colptr, N, i, 0);
    o->weights_changed = 1;
    or_tape_push(o, &t);
    o->depth += 1;
    return 0;
}
/* Observe (src/transformers.jl:228-235) */
int or_observe(oracle* o, const wsmc_dist* d, const wsmc_operand* x) { return or_weigh(o, d, x, WSMC_TERM_OBSERVE); }
/* Weight (src/transformers.jl:283-289) */
int or_weight(oracle* o, const wsmc_dist* d, const wsmc_operand* x) { return or_weigh(o, d, x, WSMC_TERM_WEIGHT); }

/* ---- resampling (src/transformers.jl:474-498, src/resampling.jl:13-77) ------- */
typedef wsmc_shard_stats or_stats;

static or_stats shard_stats(const double* lw, int64_t n, int K) {
    or_stats s;
    double M = -WSMC_INF;
    int nan = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (wsmc_isnan(lw[i])) nan = 1;
        else if (lw[i] > M) M = lw[i];
    }
    s.M = nan ? WSMC_NAN : M;                    /* maximum() propagates NaN */
    s.Q = 0; s.Q2 = 0; s.Wf2 = 0; s.Wf = 0; s.n = (uint64_t)n;
    const double R = wsmc_qref(s.M);             /* the reference point (round 6) */
    for (int64_t i = 0; i < n; ++i) {
        wsmc_qparts p = wsmc_qparts_of(lw[i], R, K);
        s.Q += p.q;
        s.Q2 += p.q2;
        s.Wf2 += p.wf2;
        s.Wf += p.wf;
    }
    return s;
}

/* the icdf merge (src/resampling.jl:13-26) on the integer CDF, one shard */
static void shard_ancestors(const double* lw, int64_t n, int K, double M, uint64_t Q, int scheme,
                            uint64_t seed, uint64_t op, uint64_t slot_base, int32_t* anc) {
    M = wsmc_qref(M);                               /* M: the shard max; q against its reference point */
    if (scheme == WSMC_RESAMPLE_MULTINOMIAL) {
        /* sorted draws from exponential spacings, then the same merge as the strata */
        uint64_t PN = 0;
        for (int64_t k = 0; k <= n; ++k) PN += wsmc_multi_e(seed, op, slot_base, (uint64_t)k, (uint64_t)n);
        uint64_t P = 0, C = wsmc_qweight(lw[0], M, K);
        int64_t m = 0;
        for (int64_t s = 0; s < n; ++s) {
            P += wsmc_multi_e(seed, op, slot_base, (uint64_t)s, (uint64_t)n);
            while (!wsmc_multi_above(C, Q, P, PN)) {   /* while C_m <= x_s */
                m += 1;
                C += wsmc_qweight(lw[m], M, K);
            }
            anc[s] = (int32_t)m;
        }
        return;
    }
    uint64_t C = wsmc_qweight(lw[0], M, K);       /* s = weights[1] */
    int64_t m = 0;
    uint32_t R0 = wsmc_strat_word(seed, op, slot_base);
    for (int64_t s = 0; s < n; ++s) {
        uint32_t R = scheme == WSMC_RESAMPLE_SYSTEMATIC ? R0 : wsmc_strat_word(seed, op, slot_base + (uint64_t)s);
        uint64_t x = wsmc_target((uint64_t)s, R, Q, (uint64_t)n);
        while (C <= x) {                            /* while s < us[n] */
            m += 1;
            C += wsmc_qweight(lw[m], M, K);
        }
        anc[s] = (int32_t)m;
    }
}

int or_resample(oracle* o, double ess_min, int32_t scheme, int32_t* resampled_out, double* ess_out) {
    uint64_t op = o->op++;
    if (!o->weights_changed) {                    /* src/transformers.jl:475-477 */
        if (resampled_out) *resampled_out = o->resampled;
        if (ess_out) *ess_out = o->last_ess;
        return 0;
    }
    int64_t off[OR_MAX_SHARDS + 1];
    int G = rs_parts(o, off);
    or_stats st[OR_MAX_SHARDS];
    for (int g = 0; g < G; ++g) {
        int64_t a = off[g], b = off[g + 1];
        st[g] = shard_stats(o->w + a, b - a, wsmc_qbits((uint64_t)(b - a)));
    }
    double ess = wsmc_global_ess(st, G);
    o->last_ess = ess;
    if (ess < ess_min) {                          /* strict, src/transformers.jl:484 */
        for (int g = 0; g < G; ++g) {
            int64_t a = off[g], b = off[g + 1], n = b - a;
            int K = wsmc_qbits((uint64_t)n);
            shard_ancestors(o->w + a, n, K, st[g].M, st[g].Q, scheme, o->seed, op, (uint64_t)(o->goff + a),
                            o->last_anc + a);
            for (int64_t s = 0; s < n; ++s) o->last_anc[a + s] += (int32_t)a;
        }
        for (int g = 0; g < G; ++g) {
            int64_t a = off[g], b = off[g + 1];
            /* logsumexp(logW) - log(N): m + log(sum exp(x - m)) - log(n) */
            double mean = wsmc_shard_mean(&st[g]);
            for (int64_t i = a; i < b; ++i) o->w[i] = mean;      /* fill!(weights, mean) */
        }
        or_store_resample(o, o->last_anc);
        o->resampled = 1;
        o->n_resamples += 1;
    } else {
        o->resampled = 0;
    }
    o->weights_changed = 0;
    if (resampled_out) *resampled_out = o->resampled;
    if (ess_out) *ess_out = ess;
    return 0;
}

/* ---- sample(state, n; replace) (src/utils.jl:92-118) ---------------------------------- */
static uint64_t* g_sort_keys;   /* qsort context (single-threaded test infrastructure) */
static int cmp_es(const void* a, const void* b) {
    const int64_t i = *(const int64_t*)a, j = *(const int64_t*)b;
    if (g_sort_keys[i] != g_sort_keys[j]) return g_sort_keys[i] > g_sort_keys[j] ? -1 : 1;   /* key desc */
    return i < j ? -1 : (i > j);                                                           /* index asc */
}
double or_es_key(uint64_t seed, uint64_t op, uint64_t i, uint64_t q) { return wsmc_es_key(seed, op, i, q); }
/* the oscillator mean's math (include/wsmc_math.h), for the known-answer tests */
void or_sincos(double x, double* s, double* c) { wsmc_sincos(x, s, c); }
double or_oscillator(double t, double A, double om, double ga, double ph) { return wsmc_oscillator(t, A, om, ga, ph); }
double or_osc_rolled(double ta, double d, int32_t m, double A, double om, double ga, double ph) {
    return wsmc_osc_rolled(ta, d, m, A, om, ga, ph);
}
int or_sample_particles(oracle* o, int64_t n, int32_t replace, int64_t* out) {
    const int64_t N = o->N;
    if (n <= 0 || (!replace && n > N)) return WSMC_EARG;
    const uint64_t op = o->op++;
    or_stats st = shard_stats(o->w, N, wsmc_qbits((uint64_t)N));
    if (st.Q == 0) return WSMC_ESTATE;                  /* exp_norm of these weights is NaN */
    const int K = wsmc_qbits((uint64_t)N);
    uint64_t* q = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N);
    for (int64_t i = 0; i < N; ++i) q[i] = wsmc_qweight(o->w[i], wsmc_qref(st.M), K);
    if (replace) {
        uint64_t* C = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N);
        uint64_t acc = 0;
        for (int64_t i = 0; i < N; ++i) { acc += q[i]; C[i] = acc; }
        for (int64_t j = 0; j < n; ++j) {
            const uint64_t x = wsmc_multi_target(wsmc_multi_word(o->seed, op, (uint64_t)j), st.Q);
            int64_t lo = 0, hi = N - 1;
            while (lo < hi) {
                const int64_t mid = lo + (hi - lo) / 2;
                if (C[mid] > x) hi = mid; else lo = mid + 1;
            }
            out[j] = lo;
        }
        free(C);
    } else {
        uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N);
        int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)N);
        for (int64_t i = 0; i < N; ++i) {
            keys[i] = wsmc_ord_enc(wsmc_es_key(o->seed, op, (uint64_t)i, q[i]));
            idx[i] = i;
        }
        g_sort_keys = keys;
        qsort(idx, (size_t)N, sizeof(int64_t), cmp_es);
        for (int64_t j = 0; j < n; ++j) out[j] = idx[j];
        free(keys); free(idx);
    }
    free(q);
    return 0;
}

/* ---- describe(): weighted median and sparkline histogram (src/utils.jl:94-141, :233-240) */
typedef struct { uint64_t v; uint64_t q; } or_vq;
static int cmp_vq(const void* a, const void* b) {
    const or_vq *x = (const or_vq*)a, *y = (const or_vq*)b;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;     /* value (ordered encoding) asc */
    return x->q < y->q ? -1 : (x->q > y->q);           /* then weight asc */
}
static uint64_t* or_qvec(oracle* o) {
    or_stats st = shard_stats(o->w, o->N, wsmc_qbits((uint64_t)o->N));
    const int K = wsmc_qbits((uint64_t)o->N);
    uint64_t* q = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)o->N);
    for (int64_t i = 0; i < o->N; ++i) q[i] = wsmc_qweight(o->w[i], wsmc_qref(st.M), K);
    return q;
}
int or_weighted_median(oracle* o, int32_t col, int32_t comp, double* out) {
    if (col < 0 || col >= o->ncols || comp < 0 || comp >= o->cols[col].dim) return WSMC_EARG;
    const int64_t N = o->N;
    const double* x = o->cols[col].front + (int64_t)comp * N;
    for (int64_t i = 0; i < N; ++i)
        if (wsmc_isnan(x[i])) { *out = x[i]; return 0; }     /* a NaN value: NaN */
    uint64_t* q = or_qvec(o);
    or_vq* a = (or_vq*)malloc(sizeof(or_vq) * (size_t)(N > 0 ? N : 1));
    int64_t n = 0;
    uint64_t Q = 0;
    for (int64_t i = 0; i < N; ++i)
        if (q[i]) { a[n].v = wsmc_ord_enc(x[i]); a[n].q = q[i]; Q += q[i]; ++n; }   /* zero weights dropped */
    free(q);
    if (n == 0) { free(a); return WSMC_ESTATE; }       /* weights cannot sum to zero */
    qsort(a, (size_t)n, sizeof(or_vq), cmp_vq);
    const uint64_t q1 = a[0].q;
    const wsmc_u128 H2 = (wsmc_u128)Q + q1;             /* 2 h */
    uint64_t Sk = 0, Skold = 0;
    double vk = 0.0, vkold = 0.0;
    int64_t k = 0;
    *out = wsmc_ord_dec(a[n - 1].v);                    /* the largest value */
    while (2 * (wsmc_u128)Sk <= H2) {
        if (k == n) { free(a); return 0; }
        Skold = Sk; vkold = vk;
        vk = wsmc_ord_dec(a[k].v);
        Sk += a[k].q;
        ++k;
    }
    *out = wsmc_median_interp(vkold, vk, Q, q1, Skold, a[k - 1].q);
    free(a);
    return 0;
}
int or_histogram(oracle* o, int32_t col, int32_t comp, int32_t* levels) {
    if (col < 0 || col >= o->ncols || comp < 0 || comp >= o->cols[col].dim) return WSMC_EARG;
    const int64_t N = o->N;
    const double* x = o->cols[col].front + (int64_t)comp * N;
    double lo = WSMC_INF, hi = -WSMC_INF;
    int nan = 0;
    for (int64_t i = 0; i < N; ++i) {
        if (wsmc_isnan(x[i])) nan = 1;
        if (x[i] < lo) lo = x[i];
        if (x[i] > hi) hi = x[i];
    }
    if (nan) lo = hi = WSMC_NAN;                        /* extrema propagate NaN: every value in bin 1 */
    if (lo == hi) { for (int b = 0; b < 8; ++b) levels[b] = 8; return 0; }
    double edges[9];
    for (int k = 0; k <= 8; ++k) edges[k] = wsmc_linspace_edge(lo, hi, k, 8);
    uint64_t* q = or_qvec(o);
    uint64_t Qs = 0;
    for (int64_t i = 0; i < N; ++i) Qs += q[i];
    if (Qs == 0) { free(q); return WSMC_ESTATE; }       /* the weights do not normalise */
    uint64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = 0; i < N; ++i) cnt[wsmc_hist_bin(x[i], edges, 8)] += q[i];
    free(q);
    uint64_t mx = 0;
    for (int b = 0; b < 8; ++b) mx = cnt[b] > mx ? cnt[b] : mx;
    for (int b = 0; b < 8; ++b) levels[b] = wsmc_spark_level(cnt[b], mx);
    return 0;
}

/* ---- one shard of an exact-sharded run: the device ranks' protocol ----
 * record of this shard's weights relative to a given (global) max, K from the global N */
void or_exact_record(oracle* o, double M, int64_t gN, uint64_t* out) {
    const int K = wsmc_qbits((uint64_t)gN);
    uint64_t Q = 0, Q2 = 0;
    wsmc_u128 Wf2 = 0, Wf = 0;
    for (int64_t i = 0; i < o->N; ++i) {
        wsmc_qparts p = wsmc_qparts_of(o->w[i], wsmc_qref(M), K);
        Q += p.q; Q2 += p.q2; Wf2 += p.wf2; Wf += p.wf;
    }
    out[0] = wsmc_d2bits(M); out[1] = Q; out[2] = Q2;
    out[3] = (uint64_t)Wf2; out[4] = (uint64_t)(Wf2 >> 64);
    out[5] = (uint64_t)Wf; out[6] = (uint64_t)(Wf >> 64);
    out[7] = (uint64_t)o->N;
}
/* the records summed as integers: the single-population statistics */
void or_combine_records(const uint64_t* recs, int32_t G, uint64_t* out) {
    uint64_t Q = 0, Q2 = 0, n = 0;
    wsmc_u128 Wf2 = 0, Wf = 0;
    for (int g = 0; g < G; ++g) {
        const uint64_t* r = recs + 8 * g;
        Q += r[1]; Q2 += r[2];
        Wf2 += ((wsmc_u128)r[4] << 64) | r[3];
        Wf += ((wsmc_u128)r[6] << 64) | r[5];
        n += r[7];
    }
    out[0] = recs[0]; out[1] = Q; out[2] = Q2;
    out[3] = (uint64_t)Wf2; out[4] = (uint64_t)(Wf2 >> 64);
    out[5] = (uint64_t)Wf; out[6] = (uint64_t)(Wf >> 64);
    out[7] = n;
}
/* ESS%, post-resample log-mean and log-evidence of one (combined) record */
void or_record_summary(const uint64_t* rec, double* ess, double* mean, double* evidence) {
    or_stats st;
    st.M = wsmc_bits2d(rec[0]); st.Q = rec[1]; st.Q2 = rec[2];
    st.Wf2 = ((wsmc_u128)rec[4] << 64) | rec[3];
    st.Wf = ((wsmc_u128)rec[6] << 64) | rec[5];
    st.n = rec[7];
    *ess = wsmc_global_ess(&st, 1);
    *mean = wsmc_shard_mean(&st);
    *evidence = wsmc_global_log_evidence(&st, 1);
}
/* this shard's window of global slots [a, b) and its ancestors (local ids): particle m owns
 * [rank(C_{m-1}), rank(C_m)) of the global CDF (cbase + the local prefix) */
int or_exact_window(oracle* o, double M, int64_t gN, uint64_t Q, uint64_t cbase, int32_t scheme, uint64_t op,
                    int32_t* anc_out, uint64_t* ab) {
    const int K = wsmc_qbits((uint64_t)gN);
    uint64_t C = cbase;
    const uint64_t a = wsmc_rank(C, Q, (uint64_t)gN, scheme, o->seed, op, 0);
    uint64_t lo = a;
    for (int64_t m = 0; m < o->N; ++m) {
        C += wsmc_qweight(o->w[m], wsmc_qref(M), K);
        const uint64_t hi = wsmc_rank(C, Q, (uint64_t)gN, scheme, o->seed, op, 0);
        for (uint64_t sl = lo; sl < hi; ++sl) anc_out[sl - a] = (int32_t)m;
        lo = hi;
    }
    ab[0] = a; ab[1] = lo;
    return 0;
}
/* test hook: the flags a Resample leaves (an exchange driven from outside the oracle) */
void or_set_resample_flags(oracle* o, int32_t resampled, int32_t weights_changed, double last_ess) {
    o->resampled = resampled; o->weights_changed = weights_changed; o->last_ess = last_ess;
    if (resampled) o->n_resamples += 1;
}

/* ---- one shard of a multi-process run: record exchange ------------------------------
 * record layout (8 x u64): M bits, Q, Q2, Wf2 lo, Wf2 hi, Wf lo, Wf hi, n — the payload the GPU
 * ranks exchange with ncclAllGather each step (weightedsampling.jl_amd/csrc, ShardRec). */
void or_shard_record(oracle* o, uint64_t* out) {
    or_stats s = shard_stats(o->w, o->N, wsmc_qbits((uint64_t)o->N));
    out[0] = wsmc_d2bits(s.M); out[1] = s.Q;
    out[2] = s.Q2;
    out[3] = (uint64_t)s.Wf2; out[4] = (uint64_t)(s.Wf2 >> 64);
    out[5] = (uint64_t)s.Wf; out[6] = (uint64_t)(s.Wf >> 64);
    out[7] = s.n;
}
static or_stats record_stats(const uint64_t* r) {
    or_stats s;
    s.M = wsmc_bits2d(r[0]); s.Q = r[1];
    s.Q2 = r[2];
    s.Wf2 = ((wsmc_u128)r[4] << 64) | r[3];
    s.Wf = ((wsmc_u128)r[6] << 64) | r[5];
    s.n = r[7];
    return s;
}
/* Resample of this shard given every shard's record (rank order): global ESS decision,
 * island resampling, shard log-mean reset. Same semantics as or_resample with shards. */
int or_resample_records(oracle* o, double ess_min, int32_t scheme, const uint64_t* recs, int32_t G,
                        int32_t rank, int32_t* resampled_out, double* ess_out) {
    uint64_t op = o->op++;
    if (!o->weights_changed) {
        if (resampled_out) *resampled_out = o->resampled;
        if (ess_out) *ess_out = o->last_ess;
        return 0;
    }
    or_stats st[OR_MAX_SHARDS];
    for (int g = 0; g < G; ++g) st[g] = record_stats(recs + 8 * g);
    double ess = wsmc_global_ess(st, G);
    o->last_ess = ess;
    if (ess < ess_min) {
        int K = wsmc_qbits((uint64_t)o->N);
        shard_ancestors(o->w, o->N, K, st[rank].M, st[rank].Q, scheme, o->seed, op, (uint64_t)o->goff,
                        o->last_anc);
        double mean = wsmc_shard_mean(&st[rank]);
        for (int64_t i = 0; i < o->N; ++i) o->w[i] = mean;
        or_store_resample(o, o->last_anc);
        o->resampled = 1;
        o->n_resamples += 1;
    } else {
        o->resampled = 0;
    }
    o->weights_changed = 0;
    if (resampled_out) *resampled_out = o->resampled;
    if (ess_out) *ess_out = ess;
    return 0;
}
double or_log_evidence_records(const uint64_t* recs, int32_t G) {
    or_stats st[OR_MAX_SHARDS];
    for (int g = 0; g < G; ++g) st[g] = record_stats(recs + 8 * g);
    return wsmc_global_log_evidence(st, G);
}

double or_canon_sum(const double* v, int64_t n);
static int move_apply(oracle* o, const int32_t* targets, int32_t d, int bounded, const double* l, const double* h,
                      const double* L, int32_t target_depth, uint64_t op_prop, uint64_t op_acc,
                      int64_t* accepted_out);
/* ---- one shard's part of a sharded autoRW move (the device ranks' protocol) ----
 * out = this oracle's canonical totals {sum e, sum e d_k, sum (e d_a) d_b (a <= b)} with
 * e = exp(w - M) for the given global M and d = z - pivot (include/wsmc_math.h
 * wsmc_autorw_factor); pivot: the unconstrained values of the population's particle 0 */
static void autorw_totals(oracle* o, int64_t a0, int64_t a1, const double* e, const double* z, int32_t d,
                          const double* pivot, double* out) {
    int64_t N = o->N, n = a1 - a0;
    double* v = o->scratch;
    int nv = 0;
    out[nv++] = or_canon_sum(e + a0, n);
    for (int k = 0; k < d; ++k) {
        for (int64_t i = a0; i < a1; ++i) v[i - a0] = e[i] * (z[(int64_t)k * N + i] - pivot[k]);
        out[nv++] = or_canon_sum(v, n);
    }
    for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b) {
            for (int64_t i = a0; i < a1; ++i)
                v[i - a0] = (e[i] * (z[(int64_t)a * N + i] - pivot[a])) * (z[(int64_t)b * N + i] - pivot[b]);
            out[nv++] = or_canon_sum(v, n);
        }
}
static void autorw_values(oracle* o, const int32_t* targets, int32_t d, const double* lo, const double* hi,
                          double M, double* e, double* z) {
    int64_t N = o->N;
    for (int64_t i = 0; i < N; ++i) e[i] = wsmc_exp(o->w[i] - M);
    for (int k = 0; k < d; ++k) {
        const double* x = o->cols[targets[k]].front;
        double l = lo ? lo[k] : -WSMC_INF, h = hi ? hi[k] : WSMC_INF;
        for (int64_t i = 0; i < N; ++i) z[(int64_t)k * N + i] = wsmc_to_unc(x[i], l, h);
    }
}
int or_moment_totals(oracle* o, const int32_t* targets, int32_t d, const double* lo, const double* hi,
                     double M, const double* pivot, double* out) {
    int64_t N = o->N;
    if (d < 1 || d > 4) return WSMC_EARG;
    double* e = (double*)malloc(sizeof(double) * (size_t)N);
    double* z = (double*)malloc(sizeof(double) * (size_t)(N * d));
    autorw_values(o, targets, d, lo, hi, M, e, z);
    autorw_totals(o, 0, N, e, z, d, pivot, out);
    free(e); free(z);
    return 0;
}
/* the unconstrained values of this oracle's particle 0 (rank 0's: the sharded pivot) */
int or_autorw_pivot(oracle* o, const int32_t* targets, int32_t d, const double* lo, const double* hi, double* out) {
    if (d < 1 || d > 4 || o->N < 1) return WSMC_EARG;
    for (int k = 0; k < d; ++k)
        out[k] = wsmc_to_unc(o->cols[targets[k]].front[0], lo ? lo[k] : -WSMC_INF, hi ? hi[k] : WSMC_INF);
    return 0;
}
/* the factor from rank-order combined totals (the device ranks' k_autorw_combine) */
int or_autorw_factor(const double* tot, int32_t d, double min_step, double* L) {
    double S[16];
    return wsmc_autorw_factor(tot, d, min_step, S, L);
}
/* covariance S (d x d, already divided by S0) -> zeros to min_step, x 2.38/sqrt(d), Cholesky */
int or_factor(const double* S_in, int32_t d, double min_step, double* L) {
    double S[16];
    double lam = 2.38 / wsmc_sqrt((double)d);
    for (int k = 0; k < d * d; ++k) {
        S[k] = S_in[k];
        if (S[k] == 0.0) S[k] = min_step;
        S[k] = lam * S[k];
    }
    return wsmc_cholesky(S, L, d);
}
/* a Move with a given factor L (consumes the Move's two op counters like or_move) */
int or_move_factor(oracle* o, const int32_t* targets, int32_t d, const double* lo, const double* hi,
                   const double* L, int32_t target_depth, int64_t* accepted_out) {
    uint64_t op_prop = o->op++, op_acc = o->op++;
    if (accepted_out) *accepted_out = 0;
    if (target_depth < 0) target_depth = o->depth;
    int bounded = 0;
    double l[4], h[4];
    for (int k = 0; k < d; ++k) {
        l[k] = lo ? lo[k] : -WSMC_INF; h[k] = hi ? hi[k] : WSMC_INF;
        if (wsmc_isfinite(l[k]) || wsmc_isfinite(h[k])) bounded = 1;
    }
    if (!lo && !hi) bounded = 0;
    return move_apply(o, targets, d, bounded, l, h, L, target_depth, op_prop, op_acc, accepted_out);
}
/* consume a Move's two op counters without moving (a shard whose factor failed) */
void or_skip_move(oracle* o) { o->op += 2; }

/* ---- analysis reductions (src/utils.jl) ------------------------------------------------
 * Weighted moments under exp_norm(weights) of d <= 4 operand expressions, in the canonical
 * reduction order the device uses (or_canon_sum): expectation / @E (src/utils.jl:11, 23-58)
 * and describe's mean and std(corrected=false) (:233-240). */
double or_canon_sum(const double* vals, int64_t n);
int or_weighted_moments(oracle* o, const wsmc_operand* ex, int32_t d, double* mean, double* cov) {
    int64_t N = o->N;
    if (d < 1 || d > 4) return WSMC_EARG;
    double M = -WSMC_INF;
    for (int64_t i = 0; i < N; ++i) if (o->w[i] > M || wsmc_isnan(o->w[i])) M = o->w[i];
    double* e = (double*)malloc(sizeof(double) * (size_t)N);
    double* z = (double*)malloc(sizeof(double) * (size_t)(N * d));
    double* v = o->scratch;
    for (int64_t i = 0; i < N; ++i) e[i] = wsmc_exp(o->w[i] - M);
    for (int k = 0; k < d; ++k)
        for (int64_t i = 0; i < N; ++i) z[(int64_t)k * N + i] = wsmc_operand_eval(&ex[k], o->colptr, N, i, 0);
    double S0 = or_canon_sum(e, N);
    for (int k = 0; k < d; ++k) {
        for (int64_t i = 0; i < N; ++i) v[i] = e[i] * z[(int64_t)k * N + i];
        mean[k] = or_canon_sum(v, N) / S0;
    }
    if (cov)
        for (int a = 0; a < d; ++a)
            for (int b = a; b < d; ++b) {
                for (int64_t i = 0; i < N; ++i)
                    v[i] = (e[i] * (z[(int64_t)a * N + i] - mean[a])) * (z[(int64_t)b * N + i] - mean[b]);
                double c = or_canon_sum(v, N) / S0;
                cov[a * d + b] = c; cov[b * d + a] = c;
            }
    free(e); free(z);
    return 0;
}
/* minimum / maximum of a column component; NaN propagates (Base.minimum / maximum) */
int or_col_minmax(oracle* o, int32_t col, int32_t comp, double* mn, double* mx) {
    if (col < 0 || col >= o->ncols || comp < 0 || comp >= o->cols[col].dim) return WSMC_EARG;
    const double* x = o->cols[col].front + (int64_t)comp * o->N;
    uint64_t a = 0, b = 0;
    for (int64_t i = 0; i < o->N; ++i) {
        uint64_t ea = wsmc_ord_enc(x[i]), eb = wsmc_ord_enc(-x[i]);
        if (ea > a) a = ea;
        if (eb > b) b = eb;
    }
    *mx = wsmc_ord_dec(a);
    *mn = -wsmc_ord_dec(b);
    return 0;
}
/* ess_perc of the current weights, no state change (src/resampling.jl:51-54) */
double or_ess(oracle* o) {
    or_stats st[OR_MAX_SHARDS];
    int64_t off[OR_MAX_SHARDS + 1];
    int G = rs_parts(o, off);
    for (int g = 0; g < G; ++g) {
        int64_t a = off[g], b = off[g + 1];
        st[g] = shard_stats(o->w + a, b - a, wsmc_qbits((uint64_t)(b - a)));
    }
    return wsmc_global_ess(st, G);
}

/* logsumexp(weights) - log(N) via the same fixed point (src/utils.jl:21) */
double or_log_evidence(oracle* o) {
    or_stats st[OR_MAX_SHARDS];
    int64_t off[OR_MAX_SHARDS + 1];
    int G = rs_parts(o, off);
    for (int g = 0; g < G; ++g) {
        int64_t a = off[g], b = off[g + 1];
        st[g] = shard_stats(o->w + a, b - a, wsmc_qbits((uint64_t)(b - a)));
    }
    return wsmc_global_log_evidence(st, G);
}

/* ---- canonical reduction order (shared with the HIP moment kernels) -------- */
/* tile of 2048 = 256 threads x 8: thread t sums items base + j*256 + t (j = 0..7) from
 * 0.0, then a xor-butterfly over each 64-lane wave (offsets 1..32), then
 * (w0 + w1) + (w2 + w3). Tiles are combined the same way with thread t summing tiles
 * t, t+256, ... */
static double canon_block(const double* vals, int64_t n, int64_t base, int per_thread_fixed) {
    double t[OR_BLOCK], nt[64];
    for (int th = 0; th < OR_BLOCK; ++th) {
        double acc = 0.0;
        if (per_thread_fixed) {
            for (int j = 0; j < OR_TILE / OR_BLOCK; ++j) {
                int64_t idx = base + (int64_t)j * OR_BLOCK + th;
                acc = acc + (idx < n ? vals[idx] : 0.0);
            }
        } else {
            for (int64_t idx = th; idx < n; idx += OR_BLOCK) acc = acc + vals[idx];
        }
        t[th] = acc;
    }
    double ws[4];
    for (int w = 0; w < 4; ++w) {
        double* l = t + 64 * w;
        for (int off = 1; off < 64; off <<= 1) {
            for (int ln = 0; ln < 64; ++ln) nt[ln] = l[ln] + l[ln ^ off];
            for (int ln = 0; ln < 64; ++ln) l[ln] = nt[ln];
        }
        ws[w] = l[0];
    }
    return (ws[0] + ws[1]) + (ws[2] + ws[3]);
}

double or_canon_sum(const double* vals, int64_t n) {
    int64_t ntiles = (n + OR_TILE - 1) / OR_TILE;
    if (ntiles == 0) return 0.0;
    double* P = (double*)malloc(sizeof(double) * (size_t)ntiles);
    for (int64_t b = 0; b < ntiles; ++b) P[b] = canon_block(vals, n, b * OR_TILE, 1);
    double r = canon_block(P, ntiles, 0, 0);
    free(P);
    return r;
}

/* ---- Move (src/transformers.jl:588-623, src/move_kernels.jl:116-253) --------- */
static uint64_t canon_key(double x) {
    return wsmc_isnan(x) ? 0x7ff8000000000000ULL : wsmc_d2bits(x);   /* isequal semantics */
}
static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}
/* marginal_diversity (src/transformers.jl:560-565) */
double or_marginal_diversity(oracle* o, const int32_t* targets, int32_t d) {
    int64_t N = o->N;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N);
    double best = WSMC_INF;
    for (int k = 0; k < d; ++k) {
        const double* x = o->cols[targets[k]].front;
        for (int64_t i = 0; i < N; ++i) keys[i] = canon_key(x[i]);
        qsort(keys, (size_t)N, sizeof(uint64_t), cmp_u64);
        int64_t u = N > 0 ? 1 : 0;
        for (int64_t i = 1; i < N; ++i) u += keys[i] != keys[i - 1];
        double frac = wsmc_u64_to_d((uint64_t)u) / wsmc_u64_to_d((uint64_t)N);
        if (frac < best) best = frac;
    }
    free(keys);
    return best;
}

/* autoRW covariance: exp_norm(weights)-weighted, uncorrected (StatsBase cov with
 * ProbabilityWeights, corrected=false), zero entries -> min_step, times 2.38/sqrt(d);
 * returns the lower Cholesky factor in L (row-major d x d), 0 if not PD. */
double or_canon_sum(const double* vals, int64_t n);
int or_autorw_chol(oracle* o, const int32_t* targets, int32_t d, double min_step, const double* lo,
                   const double* hi, double* L, double* cov_out) {
    int64_t N = o->N;
    double M = -WSMC_INF;
    for (int64_t i = 0; i < N; ++i) if (o->w[i] > M || wsmc_isnan(o->w[i])) M = o->w[i];
    double* e = (double*)malloc(sizeof(double) * (size_t)N);
    double* z = (double*)malloc(sizeof(double) * (size_t)(N * d));
    autorw_values(o, targets, d, lo, hi, M, e, z);
    /* one pass relative to the pivot (the population's particle 0), canonical totals per
       shard combined in rank order (one shard: the plain canonical sums); the device ranks
       exchange exactly these per-shard totals (include/wsmc_math.h wsmc_autorw_factor) */
    double pivot[4];
    for (int k = 0; k < d; ++k) pivot[k] = z[(int64_t)k * N];
    int G = o->nshards;
    double tot[15], part[15];
    const int nv = 1 + d + d * (d + 1) / 2;
    for (int g = 0; g < G; ++g) {
        autorw_totals(o, o->shard_off[g], o->shard_off[g + 1], e, z, d, pivot, part);
        for (int k = 0; k < nv; ++k) tot[k] = g == 0 ? part[k] : tot[k] + part[k];
    }
    double S[16];
    const int ok = wsmc_autorw_factor(tot, d, min_step, S, L);
    if (cov_out) for (int k = 0; k < d * d; ++k) cov_out[k] = S[k];
    free(e); free(z);
    return ok;
}

static int move_apply(oracle* o, const int32_t* targets, int32_t d, int bounded, const double* l, const double* h,
                      const double* L, int32_t target_depth, uint64_t op_prop, uint64_t op_acc,
                      int64_t* accepted_out);
int or_move(oracle* o, int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
            const double* hi, int32_t target_depth, double diversity, int64_t* accepted_out) {
    uint64_t op_prop = o->op++, op_acc = o->op++;
    if (accepted_out) *accepted_out = 0;
    if (d < 1 || d > 4) return WSMC_EARG;
    if (!wsmc_isnan(diversity) && or_marginal_diversity(o, targets, d) >= diversity) return 0;
    if (target_depth < 0) target_depth = o->depth;
    int bounded = 0;
    double l[4], h[4];
    for (int k = 0; k < d; ++k) {
        l[k] = lo ? lo[k] : -WSMC_INF; h[k] = hi ? hi[k] : WSMC_INF;
        if (wsmc_isfinite(l[k]) || wsmc_isfinite(h[k])) bounded = 1;
    }
    if (!lo && !hi) bounded = 0;
    double L[16];
    if (proposal == WSMC_PROPOSAL_AUTORW) {
        if (!or_autorw_chol(o, targets, d, step, bounded ? l : 0, bounded ? h : 0, L, 0)) return WSMC_ENOTPD;
    } else {
        for (int k = 0; k < d * d; ++k) L[k] = 0.0;
        for (int k = 0; k < d; ++k) L[k * d + k] = step;
    }
    return move_apply(o, targets, d, bounded, l, h, L, target_depth, op_prop, op_acc, accepted_out);
}

/* the proposal + accept/reject of a Move given its factor L (src/transformers.jl:604-621) */
static int move_apply(oracle* o, const int32_t* targets, int32_t d, int bounded, const double* l, const double* h,
                      const double* L, int32_t target_depth, uint64_t op_prop, uint64_t op_acc,
                      int64_t* accepted_out) {
    int64_t N = o->N;
    int64_t acc = 0;
    double* newv = (double*)malloc(sizeof(double) * (size_t)(N * d));
    unsigned char* ok = (unsigned char*)malloc((size_t)N);
    /* particles are independent (counter-based draws, per-particle folds): OpenMP changes no bit */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        double xi[4], dz[4];
        wsmc_override ov;
        ov.n = d;
        for (int k = 0; k < d; ++k) xi[k] = wsmc_normal_k(o->seed, op_prop, (uint64_t)(o->goff + i), (uint32_t)k);
        for (int k = 0; k < d; ++k) {
            double s = 0.0;
            for (int j = 0; j <= k; ++j) s = s + L[k * d + j] * xi[j];
            dz[k] = s;
        }
        double lpr = 0.0;
        for (int k = 0; k < d; ++k) {
            double x = o->cols[targets[k]].front[i];
            double xn = x + dz[k];
            if (bounded) {   /* to_unc, the step, from_unc and the Jacobian difference */
                const int fl = wsmc_isfinite(l[k]), fh = wsmc_isfinite(h[k]);
                double dj;
                xn = wsmc_bounded_step(x, dz[k], l[k], h[k], fl && fh ? wsmc_log(h[k] - l[k]) : 0.0, fl, fh, &dj);
                lpr = lpr + dj;
            }
            ov.col[k] = targets[k];
            ov.val[k] = xn;
            newv[(int64_t)k * N + i] = xn;
        }
        double s_old = wsmc_fold(o->tape, o->nterms, target_depth, o->colptr, N, i, 0);
        double s_new = wsmc_fold(o->tape, o->nterms, target_depth, o->colptr, N, i, &ov);
        double u = wsmc_uniform_k(o->seed, op_acc, (uint64_t)(o->goff + i), 0);
        ok[i] = wsmc_log(u) < (lpr + s_new) - s_old;   /* src/transformers.jl:615 */
    }
    for (int64_t i = 0; i < N; ++i) {
        if (!ok[i]) continue;
        acc += 1;
        for (int k = 0; k < d; ++k) o->cols[targets[k]].front[i] = newv[(int64_t)k * N + i];
    }
    free(newv); free(ok);
    if (accepted_out) *accepted_out = acc;
    return 0;
}

/* score_logpdf (src/types.jl:198-206) */
void or_score(oracle* o, int32_t target_depth, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < o->N; ++i)
        out[i] = wsmc_fold(o->tape, o->nterms, target_depth, o->colptr, o->N, i, 0);
}

/* ---- raw primitives exported for the unit tests ------------------------------ */
void or_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    wsmc_u32x4 r = wsmc_philox(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
    for (int k = 0; k < 4; ++k) out[k] = r.v[k];
}
double or_exp(double x) { return wsmc_exp(x); }
double or_expw(double x) { return wsmc_expw(x); }
double or_log(double x) { return wsmc_log(x); }
double or_log1p(double x) { return wsmc_log1p(x); }
double or_cos(double x) { return wsmc_cos(x); }
double or_sin(double x) { return wsmc_sin(x); }
void or_sincos2pi(double u, double* s, double* c) { wsmc_sincos2pi(u, s, c); }
double or_normal_k(uint64_t seed, uint64_t op, uint64_t idx, uint32_t k) { return wsmc_normal_k(seed, op, idx, k); }
double or_uniform_k(uint64_t seed, uint64_t op, uint64_t idx, uint32_t k) { return wsmc_uniform_k(seed, op, idx, k); }
uint64_t or_rank(uint64_t c, uint64_t Q, uint64_t N, int scheme, uint64_t seed, uint64_t op, uint64_t base) {
    return wsmc_rank(c, Q, N, scheme, seed, op, base);
}
uint64_t or_target(uint64_t n, uint32_t R, uint64_t Q, uint64_t N) { return wsmc_target(n, R, Q, N); }
uint32_t or_strat_word(uint64_t seed, uint64_t op, uint64_t n) { return wsmc_strat_word(seed, op, n); }
uint64_t or_qweight(double lw, double M, int K) { return wsmc_qweight(lw, M, K); }
double or_qref(double M) { return wsmc_qref(M); }
int or_qbits(uint64_t n) { return wsmc_qbits(n); }
int32_t or_sizeof_term(void) { return (int32_t)sizeof(wsmc_term); }
int32_t or_sizeof_dist(void) { return (int32_t)sizeof(wsmc_dist); }
