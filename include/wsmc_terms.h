/*
 * wsmc_terms.h — per-particle evaluation of operator arguments, draws, log-densities
 * and the score fold. Shared verbatim by the HIP kernels and the CPU oracle so that
 * every per-particle value is computed by the same sequence of IEEE operations.
 *
 *   operand     argfn shapes of @model `vectorize` (src/rewrites.jl:146-219)
 *   sample      WeightedKernel.sampler = rand(D(args...))   (src/default_kernels.jl:18)
 *   logpdf      WeightedKernel.logpdf  = logpdf(D(args...), x) (src/default_kernels.jl:20)
 *   fold        score_logpdf!: scores start at 0.0 and every counted statement executed
 *               before target_depth adds its term in program order
 *               (src/types.jl:198-206, Sequence early stop src/transformers.jl:343-349)
 */
#ifndef WSMC_TERMS_H
#define WSMC_TERMS_H

#include "wsmc.h"
#include "wsmc_math.h"

/* MH proposal values substituted for target columns during the s_new fold */
typedef struct {
    int32_t n;
    int32_t col[4];
    double  val[4];
} wsmc_override;

WSMC_HD double wsmc_colval(double* const* cols, int64_t N, int32_t col, int32_t comp, int64_t i,
                           const wsmc_override* ov) {
    if (ov) {
        for (int k = 0; k < ov->n; ++k)
            if (ov->col[k] == col && comp == 0) return ov->val[k];
    }
    return cols[col][(int64_t)comp * N + i];
}

WSMC_HD double wsmc_operand_eval(const wsmc_operand* o, double* const* cols, int64_t N, int64_t i,
                                 const wsmc_override* ov) {
    double v = o->c0;
    if (o->col[0] >= 0) v = v + o->coef[0] * wsmc_colval(cols, N, o->col[0], o->comp[0], i, ov);
    if (o->col[1] >= 0) v = v + o->coef[1] * wsmc_colval(cols, N, o->col[1], o->comp[1], i, ov);
    return v;
}

/* ---- expressions (wsmc_assign_expr): one postfix program per output component ----------
 * The operators of the fused broadcast `vectorize` emits (src/rewrites.jl:146-219), each a
 * fixed IEEE sequence shared by the device and the oracle. */
WSMC_HD double wsmc_xop1(int op, double a, double c) {
    switch (op) {
        case WSMC_X_NEG: return -a;
        case WSMC_X_ABS: return wsmc_fabs(a);
        case WSMC_X_SQRT: return a < 0.0 ? WSMC_NAN : wsmc_sqrt(a);
        case WSMC_X_EXP: return wsmc_exp(a);
        case WSMC_X_LOG: return wsmc_log(a);
        case WSMC_X_LOG1P: return wsmc_log1p(a);
        case WSMC_X_SIN: return wsmc_sin(a);
        case WSMC_X_COS: return wsmc_cos(a);
        case WSMC_X_POWI: return wsmc_powi(a, (int64_t)c);
        case WSMC_X_NOT: return a == 0.0 ? 1.0 : 0.0;
        default: return WSMC_NAN;
    }
}
WSMC_HD double wsmc_xop2(int op, double a, double b) {
    switch (op) {
        case WSMC_X_ADD: return a + b;
        case WSMC_X_SUB: return a - b;
        case WSMC_X_MUL: return a * b;
        case WSMC_X_DIV: return a / b;
        case WSMC_X_MIN: return wsmc_min(a, b);
        case WSMC_X_MAX: return wsmc_max(a, b);
        case WSMC_X_POW: return wsmc_pow(a, b);
        case WSMC_X_LT: return a < b ? 1.0 : 0.0;
        case WSMC_X_LE: return a <= b ? 1.0 : 0.0;
        case WSMC_X_GT: return a > b ? 1.0 : 0.0;
        case WSMC_X_GE: return a >= b ? 1.0 : 0.0;
        case WSMC_X_EQ: return a == b ? 1.0 : 0.0;
        case WSMC_X_NE: return a != b ? 1.0 : 0.0;
        case WSMC_X_AND: return (a != 0.0 && b != 0.0) ? 1.0 : 0.0;
        case WSMC_X_OR: return (a != 0.0 || b != 0.0) ? 1.0 : 0.0;
        default: return WSMC_NAN;
    }
}
/* stack effect of one instruction (pops, pushes); pops < 0: not an operator */
WSMC_HD int wsmc_xarity(int op) {
    if (op == WSMC_X_CONST || op == WSMC_X_COL) return 0;
    if (op >= WSMC_X_NEG && op <= WSMC_X_NOT) return 1;
    if (op >= WSMC_X_ADD && op <= WSMC_X_OR) return 2;
    if (op == WSMC_X_IFELSE) return 3;
    return -1;
}
/* the program's shape (columns are the caller's to check): 0, or -1 for an unknown
   operator, -2 a stack underflow, -3 more than WSMC_XSTACK_MAX values, -4 a component not
   leaving one value, -5 too many instructions, -6 a POWI exponent that is no integer */
WSMC_HD int wsmc_xprog_check(const wsmc_xinst* prog, const int32_t* len, int dim) {
    int64_t total = 0;
    for (int k = 0; k < dim; ++k) {
        if (len[k] < 1) return -4;
        total += len[k];
    }
    if (total > WSMC_XPROG_MAX) return -5;
    int pc = 0;
    for (int k = 0; k < dim; ++k) {
        int sp = 0;
        for (int e = pc + len[k]; pc < e; ++pc) {
            const int a = wsmc_xarity(prog[pc].op);
            if (a < 0) return -1;
            if (sp < a) return -2;
            sp += 1 - a;
            if (sp > WSMC_XSTACK_MAX) return -3;
            if (prog[pc].op == WSMC_X_POWI) {
                const double c = prog[pc].c;
                if (!(wsmc_fabs(c) < 4611686018427387904.0) || c != (double)(int64_t)c) return -6;
            }
        }
        if (sp != 1) return -4;
    }
    return 0;
}
/* one component of one particle, a plain stack (the oracle's machine; the device keeps its
   stack in registers and applies the same operators) */
WSMC_HD double wsmc_xeval(const wsmc_xinst* p, int n, double* const* cols, int64_t N, int64_t i) {
    double st[WSMC_XSTACK_MAX];
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        const int op = p[k].op;
        if (op == WSMC_X_CONST) {
            st[sp++] = p[k].c;
        } else if (op == WSMC_X_COL) {
            st[sp++] = cols[p[k].col][(int64_t)p[k].comp * N + i];
        } else if (op == WSMC_X_IFELSE) {
            const double f = st[--sp], t = st[--sp];
            st[sp - 1] = st[sp - 1] != 0.0 ? t : f;
        } else if (wsmc_xarity(op) == 1) {
            st[sp - 1] = wsmc_xop1(op, st[sp - 1], p[k].c);
        } else {
            const double b = st[--sp];
            st[sp - 1] = wsmc_xop2(op, st[sp - 1], b);
        }
    }
    return st[0];
}

/* feat: the mean functions and families a caller may meet (WSMC_FEAT_OSC: the oscillator,
 * WSMC_FEAT_MVN: the full-covariance MvNormal). A device kernel launched without them passes
 * 0 (or OSC alone), so their code is not compiled into it (registers); every other caller
 * passes WSMC_FEAT_ALL. The arithmetic is the same. */
#define WSMC_FEAT_OSC 1u
#define WSMC_FEAT_MVN 2u   /* the full-covariance MvNormal family */
#define WSMC_FEAT_EXT 4u   /* the scalar families from WSMC_FAM_BERNOULLI on */
#define WSMC_FEAT_ALL 7u
WSMC_HD double wsmc_dist_mean_f(const wsmc_dist* d, int k, double* const* cols, int64_t N, int64_t i,
                                const wsmc_override* ov, unsigned feat) {
    if ((feat & WSMC_FEAT_OSC) && d->mean_fn == WSMC_MEAN_OSCILLATOR) {
        double A = wsmc_operand_eval(&d->mu[0], cols, N, i, ov);
        double om = wsmc_operand_eval(&d->mu[1], cols, N, i, ov);
        double ga = wsmc_operand_eval(&d->mu[2], cols, N, i, ov);
        double ph = wsmc_operand_eval(&d->mu[3], cols, N, i, ov);
        /* reserved = m > 0: a linked Observe term, the mean at param[0] + m param[1] by rotation */
        if (d->reserved > 0) return wsmc_osc_rolled(d->param[0], d->param[1], d->reserved, A, om, ga, ph);
        return wsmc_oscillator(d->param[0], A, om, ga, ph);
    }
    return wsmc_operand_eval(&d->mu[k], cols, N, i, ov);
}
WSMC_HD double wsmc_dist_mean(const wsmc_dist* d, int k, double* const* cols, int64_t N, int64_t i,
                              const wsmc_override* ov) {
    return wsmc_dist_mean_f(d, k, cols, N, i, ov, WSMC_FEAT_ALL);
}

/* log and reciprocal of a scale parameter, remembered across the terms of one fold: a
 * particle's terms often share one sigma / variance value (e.g. a sigma column), and the
 * log / reciprocal of the same bits are the same bits, so reusing them changes nothing but
 * the work. */
typedef struct {
    uint64_t arg;
    double val;      /* log(arg) */
    double rcp;      /* 1 / arg  */
    int valid;
} wsmc_logmemo;
WSMC_HD void wsmc_scale_memo(wsmc_logmemo* m, double x, double* lg, double* rc) {
    if (!m) {
        *lg = wsmc_log(x);
        *rc = 1.0 / x;
        return;
    }
    uint64_t b = wsmc_d2bits(x);
    if (!(m->valid && m->arg == b)) {
        m->arg = b;
        m->val = wsmc_log(x);
        m->rcp = 1.0 / x;
        m->valid = 1;
    }
    *lg = m->val;
    *rc = m->rcp;
}
WSMC_HD double wsmc_log_memo(wsmc_logmemo* m, double x) {
    double lg, rc;
    wsmc_scale_memo(m, x, &lg, &rc);
    return lg;
}

/* WSMC_FAM_MVNORMAL (constant covariance, dim <= 3). Sigma = L L' with L lower triangular;
 * the packed numbers are L row by row (dim (dim + 1) / 2 values), then log det Sigma. They sit
 * in the double fields (c0, coef[0], coef[1]) of the unused mean operands mu[dim..3], then of
 * scale, then in param[0..1]: every operand stays a constant (col = -1), so the code that
 * scans operands for the columns a statement reads (lazy gathers, statement batches, remaps)
 * never sees them. Capacity 3 (4 - dim) + 5 doubles: 8 at dim 3 (7 needed). */
#define WSMC_MVN_MAXDIM 3
/* packed number j of a dist of dimension n; called with constant n and j (the per-dimension
 * instances below unroll), so every access is a fixed field of the argument struct */
WSMC_HD double wsmc_mvn_get(const wsmc_dist* d, int n, int j) {
    const int nfree = 4 - n;
    const int q = j / 3, r = j - 3 * q;
    if (q > nfree) return d->param[j - 3 * (nfree + 1)];
    const wsmc_operand* o = q < nfree ? &d->mu[n + q] : &d->scale;
    return r == 0 ? o->c0 : o->coef[r - 1];
}
WSMC_HD void wsmc_mvn_set(wsmc_dist* d, int j, double v) {
    const int nfree = 4 - d->dim;
    const int q = j / 3, r = j - 3 * q;
    if (q > nfree) {
        d->param[j - 3 * (nfree + 1)] = v;
        return;
    }
    wsmc_operand* o = q < nfree ? &d->mu[d->dim + q] : &d->scale;
    if (r == 0) o->c0 = v; else o->coef[r - 1] = v;
}
/* wsmc_dist_mvnormal_cov's packing (host): 0, -1 bad dim / not exactly symmetric, -2 not
 * positive definite. Cholesky–Banachiewicz, each entry's dot product summed left to right;
 * log det = 2 (log L00 + log L11 + ...). */
WSMC_HD int wsmc_mvn_pack(wsmc_dist* d, const double* S) {
    const int n = d->dim;
    if (n < 1 || n > WSMC_MVN_MAXDIM) return -1;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j)
            if (!(S[i * n + j] == S[j * n + i])) return -1;
    double L[WSMC_MVN_MAXDIM][WSMC_MVN_MAXDIM] = {{0.0}};
    double hl = 0.0;
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j <= i; ++j) {
            double s = S[i * n + j];
            for (int k = 0; k < j; ++k) s = s - L[i][k] * L[j][k];
            if (i == j) {
                if (!(s > 0.0) || !wsmc_isfinite(s)) return -2;
                L[i][i] = wsmc_sqrt(s);
                hl = hl + wsmc_log(L[i][i]);
            } else {
                L[i][j] = s / L[j][j];
            }
        }
    }
    d->family = WSMC_FAM_MVNORMAL;
    for (int k = n; k < 4; ++k) {
        d->mu[k].c0 = 0.0;
        d->mu[k].col[0] = d->mu[k].col[1] = -1;
        d->mu[k].comp[0] = d->mu[k].comp[1] = 0;
        d->mu[k].coef[0] = d->mu[k].coef[1] = 0.0;
    }
    d->scale.c0 = 0.0;
    d->scale.col[0] = d->scale.col[1] = -1;
    d->scale.comp[0] = d->scale.comp[1] = 0;
    d->scale.coef[0] = d->scale.coef[1] = 0.0;
    d->param[0] = d->param[1] = 0.0;
    int p = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) wsmc_mvn_set(d, p++, L[i][j]);
    wsmc_mvn_set(d, p, 2.0 * hl);
    return 0;
}

/* WSMC_FAM_MVNORMAL of dimension n (a constant at every call):
 * -(n log2pi + log det Sigma + |L^-1 (x - mu)|^2)/2, L^-1 r by forward substitution */
WSMC_HD double wsmc_mvn_logpdf_n(const wsmc_dist* d, const int n, const double* x, double* const* cols,
                                 int64_t N, int64_t i, const wsmc_override* ov, unsigned feat) {
    double y[WSMC_MVN_MAXDIM] = {0.0, 0.0, 0.0};
    double s = 0.0;
    int p = 0;
    WSMC_UNROLL
    for (int k = 0; k < n; ++k) {   /* row k of L at p */
        double r = x[k] - wsmc_dist_mean_f(d, k, cols, N, i, ov, feat);
        WSMC_UNROLL
        for (int m = 0; m < k; ++m) r = r - wsmc_mvn_get(d, n, p + m) * y[m];
        y[k] = r / wsmc_mvn_get(d, n, p + k);
        s = s + y[k] * y[k];
        p += k + 1;
    }
    return -(((double)n * WSMC_LOG2PI + wsmc_mvn_get(d, n, p)) + s) * 0.5;
}
/* mu + L z, z drawn in pairs as for the isotropic family */
WSMC_HD void wsmc_mvn_sample_n(const wsmc_dist* d, const int n, double* x, uint64_t seed, uint64_t op,
                               uint64_t idx, double* const* cols, int64_t N, int64_t i, unsigned feat) {
    double z[4] = {0.0, 0.0, 0.0, 0.0};
    WSMC_UNROLL
    for (int k = 0; k < n; k += 2)
        wsmc_normal_pair(wsmc_rng_block(seed, op, idx, (uint32_t)(k >> 1)), &z[k], &z[k + 1]);
    int p = 0;
    WSMC_UNROLL
    for (int k = 0; k < n; ++k) {
        double acc = 0.0;
        WSMC_UNROLL
        for (int m = 0; m <= k; ++m) acc = acc + wsmc_mvn_get(d, n, p + m) * z[m];
        x[k] = wsmc_dist_mean_f(d, k, cols, N, i, 0, feat) + acc;
        p += k + 1;
    }
}

/* the feature bits a dist needs in a kernel (wsmc_dist_logpdf_mf / wsmc_dist_sample_mf's feat) */
WSMC_HD unsigned wsmc_dist_feat(const wsmc_dist* d) {
    return (d->mean_fn == WSMC_MEAN_OSCILLATOR ? WSMC_FEAT_OSC : 0u) |
           (d->family == WSMC_FAM_MVNORMAL ? WSMC_FEAT_MVN : 0u) |
           (d->family >= WSMC_FAM_BERNOULLI ? WSMC_FEAT_EXT : 0u);
}

/* ---- the scalar families from WSMC_FAM_BERNOULLI on (src/default_kernels.jl:83-102) -----
 * location m = mu[0] (p, logitp for the Bernoullis and Geometric), scale s = `scale`.
 * logpdf: Distributions.jl's formulas, operation for operation where they are written out
 * (zval as the Normal family's (x - m) * (1/s)); outside the support -Inf. */
WSMC_HD double wsmc_ext_logpdf(int fam, double x, double m, double s, wsmc_logmemo* lm) {
    switch (fam) {
        case WSMC_FAM_BERNOULLI:   /* x == 0 ? log(failprob) : x == 1 ? log(succprob) : -Inf */
            return x == 0.0 ? wsmc_log(1.0 - m) : (x == 1.0 ? wsmc_log(m) : -WSMC_INF);
        case WSMC_FAM_BERNOULLI_LOGIT:   /* -log1pexp(x ? -logitp : logitp) */
            return x == 0.0 ? -wsmc_log1pexp(m) : (x == 1.0 ? -wsmc_log1pexp(-m) : -WSMC_INF);
        case WSMC_FAM_EXPONENTIAL: {   /* λ = rate = 1/θ: log(λ) - λ x */
            const double r = 1.0 / s;
            return x < 0.0 ? -WSMC_INF : wsmc_log(r) - r * x;
        }
        case WSMC_FAM_LOGNORMAL: {   /* normlogpdf(μ, σ, log x) - log x */
            if (!(x > 0.0)) return -WSMC_INF;
            const double lx = wsmc_log(x);
            double lg, rc;
            wsmc_scale_memo(lm, s, &lg, &rc);
            return wsmc_normal_lh((lx - m) * wsmc_normal_rh(rc), wsmc_normal_c(lg)) - lx;
        }
        case WSMC_FAM_LAPLACE:   /* -(|x - μ| / θ + log(2θ)) */
            return -(wsmc_fabs(x - m) / s + wsmc_log(2.0 * s));
        case WSMC_FAM_CAUCHY: {   /* -(log1psq((x - μ)/σ) + log π + log σ) */
            double lg, rc;
            wsmc_scale_memo(lm, s, &lg, &rc);
            const double az = wsmc_fabs((x - m) * rc);
            const double l1 = az < 9007199254740992.0 ? wsmc_log1p(az * az) : 2.0 * wsmc_log(az);
            return -((l1 + 1.14472988584940017414) + lg);
        }
        case WSMC_FAM_LOGISTIC: {   /* u = -|z|: u - 2 log1pexp(u) - log θ */
            double lg, rc;
            wsmc_scale_memo(lm, s, &lg, &rc);
            const double u = -wsmc_fabs((x - m) * rc);
            return (u - 2.0 * wsmc_log1pexp(u)) - lg;
        }
        case WSMC_FAM_GUMBEL: {   /* -(z + exp(-z) + log θ) */
            double lg, rc;
            wsmc_scale_memo(lm, s, &lg, &rc);
            const double z = (x - m) * rc;
            return -((z + wsmc_exp(-z)) + lg);
        }
        case WSMC_FAM_RAYLEIGH: {   /* σ² = σ^2: x < 0 ? -Inf : log(x / σ²) - x^2 / (2σ²) */
            const double s2 = s * s;
            return x < 0.0 ? -WSMC_INF : wsmc_log(x / s2) - (x * x) / (2.0 * s2);
        }
        default: {   /* WSMC_FAM_GEOMETRIC: insupport ? log(p) + log1p(-p) x : -Inf */
            if (!(x >= 0.0 && x == wsmc_floor(x))) return -WSMC_INF;
            return wsmc_log(m) + wsmc_log1p(-m) * x;
        }
    }
}
/* one draw: u the op's first uniform in [0, 1), e = -log(1 - u) an Exp(1) variate (a
 * uniform's inverse CDF; Julia's randexp draws the same distribution by a ziggurat) */
WSMC_HD double wsmc_ext_sample(int fam, double m, double s, uint64_t seed, uint64_t op, uint64_t idx) {
    if (fam == WSMC_FAM_LOGNORMAL) return wsmc_exp(m + s * wsmc_normal_k(seed, op, idx, 0));
    const wsmc_u32x4 w = wsmc_rng_block(seed, op, idx, 0x80u);
    const double u = wsmc_u01(w.v[0], w.v[1]);
    const double e = -wsmc_log(1.0 - u);
    switch (fam) {
        case WSMC_FAM_BERNOULLI: return u < m ? 1.0 : 0.0;
        case WSMC_FAM_BERNOULLI_LOGIT: return u < 1.0 / (1.0 + wsmc_exp(-m)) ? 1.0 : 0.0;
        case WSMC_FAM_EXPONENTIAL: return s * e;
        case WSMC_FAM_LAPLACE: return m + s * ((w.v[2] >> 31) ? e : -e);   /* randexp * ±1 */
        case WSMC_FAM_CAUCHY: {   /* μ + σ tan(π (u - 1/2)) = μ - σ cos(π u) / sin(π u) */
            double sn, cs;
            wsmc_sincos2pi(0.5 * u, &sn, &cs);
            return m - s * (cs / sn);
        }
        case WSMC_FAM_LOGISTIC: return m + s * wsmc_log(u / (1.0 - u));   /* μ + θ logit(u) */
        case WSMC_FAM_GUMBEL: return m - s * wsmc_log(e);                 /* μ - θ log(randexp) */
        case WSMC_FAM_RAYLEIGH: return s * wsmc_sqrt(2.0 * e);            /* σ sqrt(2 randexp) */
        default: return wsmc_floor(-e / wsmc_log1p(-m));                   /* Geometric */
    }
}

/* logpdf(D(args...), x) for the supported families */
WSMC_HD double wsmc_dist_logpdf_mf(const wsmc_dist* d, const double* x, double* const* cols, int64_t N,
                                   int64_t i, const wsmc_override* ov, wsmc_logmemo* lm, unsigned feat) {
    switch (d->family) {
        case WSMC_FAM_NORMAL: {   /* wsmc_normal_logpdf with a remembered log(sigma), 1/sigma */
            double mu = wsmc_dist_mean_f(d, 0, cols, N, i, ov, feat);
            double sg = wsmc_operand_eval(&d->scale, cols, N, i, ov);
            double lg, rc;
            wsmc_scale_memo(lm, sg, &lg, &rc);
            return wsmc_normal_lh((x[0] - mu) * wsmc_normal_rh(rc), wsmc_normal_c(lg));
        }
        case WSMC_FAM_HALFNORMAL: {   /* wsmc_halfnormal_logpdf likewise */
            double sg = wsmc_operand_eval(&d->scale, cols, N, i, ov);
            if (!(x[0] >= 0.0)) return -WSMC_INF;
            double lg, rc;
            wsmc_scale_memo(lm, sg, &lg, &rc);
            return wsmc_normal_lh((x[0] - 0.0) * wsmc_normal_rh(rc), wsmc_normal_c(lg)) + WSMC_LOG2;
        }
        case WSMC_FAM_UNIFORM:
            return wsmc_uniform_logpdf(d->param[0], d->param[1], x[0]);
        case WSMC_FAM_BERNOULLI: case WSMC_FAM_BERNOULLI_LOGIT: case WSMC_FAM_EXPONENTIAL:
        case WSMC_FAM_LOGNORMAL: case WSMC_FAM_LAPLACE: case WSMC_FAM_CAUCHY: case WSMC_FAM_LOGISTIC:
        case WSMC_FAM_GUMBEL: case WSMC_FAM_RAYLEIGH: case WSMC_FAM_GEOMETRIC:
            if (!(feat & WSMC_FEAT_EXT)) return __builtin_nan("");   /* never launched so */
            return wsmc_ext_logpdf(d->family, x[0], wsmc_operand_eval(&d->mu[0], cols, N, i, ov),
                                   wsmc_operand_eval(&d->scale, cols, N, i, ov), lm);
        case WSMC_FAM_MVNORMAL:
            if (!(feat & WSMC_FEAT_MVN)) return __builtin_nan("");   /* never launched so */
            if (d->dim == 2) return wsmc_mvn_logpdf_n(d, 2, x, cols, N, i, ov, feat);
            if (d->dim == 3) return wsmc_mvn_logpdf_n(d, 3, x, cols, N, i, ov, feat);
            return wsmc_mvn_logpdf_n(d, 1, x, cols, N, i, ov, feat);
        default: { /* WSMC_FAM_MVNORMAL_ISO: -(d log2pi + d log var + |x-mu|^2/var)/2 */
            double var = wsmc_operand_eval(&d->scale, cols, N, i, ov);
            double s = 0.0;
            for (int k = 0; k < d->dim && k < 4; ++k) {
                double dx = x[k] - wsmc_dist_mean_f(d, k, cols, N, i, ov, feat);
                s = s + dx * dx;
            }
            double dd = (double)d->dim;
            return -((dd * WSMC_LOG2PI + dd * wsmc_log_memo(lm, var)) + s / var) * 0.5;
        }
    }
}
WSMC_HD double wsmc_dist_logpdf_m(const wsmc_dist* d, const double* x, double* const* cols, int64_t N,
                                  int64_t i, const wsmc_override* ov, wsmc_logmemo* lm) {
    return wsmc_dist_logpdf_mf(d, x, cols, N, i, ov, lm, WSMC_FEAT_ALL);
}
WSMC_HD double wsmc_dist_logpdf(const wsmc_dist* d, const double* x, double* const* cols, int64_t N,
                                int64_t i, const wsmc_override* ov) {
    return wsmc_dist_logpdf_m(d, x, cols, N, i, ov, 0);
}

/* rand(D(args...)) for particle i (global RNG index idx). sd_pre: for an MvNormal whose
 * variance operand is a constant, wsmc_sqrt of it evaluated once by the caller (the same
 * function of the same bits, so the same result as evaluating it per particle); else null. */
WSMC_HD void wsmc_dist_sample_mf(const wsmc_dist* d, double* x, uint64_t seed, uint64_t op, uint64_t idx,
                                 double* const* cols, int64_t N, int64_t i, const double* sd_pre, unsigned feat) {
    switch (d->family) {
        case WSMC_FAM_NORMAL: {
            double mu = wsmc_dist_mean_f(d, 0, cols, N, i, 0, feat);
            double sg = wsmc_operand_eval(&d->scale, cols, N, i, 0);
            x[0] = mu + sg * wsmc_normal_k(seed, op, idx, 0);
            break;
        }
        case WSMC_FAM_HALFNORMAL: {
            double sg = wsmc_operand_eval(&d->scale, cols, N, i, 0);
            x[0] = sg * wsmc_fabs(wsmc_normal_k(seed, op, idx, 0));
            break;
        }
        case WSMC_FAM_UNIFORM: {
            double a = d->param[0], b = d->param[1];
            x[0] = a + (b - a) * wsmc_uniform_k(seed, op, idx, 0);
            break;
        }
        case WSMC_FAM_BERNOULLI: case WSMC_FAM_BERNOULLI_LOGIT: case WSMC_FAM_EXPONENTIAL:
        case WSMC_FAM_LOGNORMAL: case WSMC_FAM_LAPLACE: case WSMC_FAM_CAUCHY: case WSMC_FAM_LOGISTIC:
        case WSMC_FAM_GUMBEL: case WSMC_FAM_RAYLEIGH: case WSMC_FAM_GEOMETRIC:
            if (!(feat & WSMC_FEAT_EXT)) break;   /* never launched so */
            x[0] = wsmc_ext_sample(d->family, wsmc_operand_eval(&d->mu[0], cols, N, i, 0),
                                   wsmc_operand_eval(&d->scale, cols, N, i, 0), seed, op, idx);
            break;
        case WSMC_FAM_MVNORMAL:
            if (!(feat & WSMC_FEAT_MVN)) break;   /* never launched so */
            if (d->dim == 2) wsmc_mvn_sample_n(d, 2, x, seed, op, idx, cols, N, i, feat);
            else if (d->dim == 3) wsmc_mvn_sample_n(d, 3, x, seed, op, idx, cols, N, i, feat);
            else wsmc_mvn_sample_n(d, 1, x, seed, op, idx, cols, N, i, feat);
            break;
        default: {
            double sd = sd_pre ? *sd_pre : wsmc_sqrt(wsmc_operand_eval(&d->scale, cols, N, i, 0));
            for (int k = 0; k < d->dim && k < 4; k += 2) {
                double z0, z1;
                wsmc_normal_pair(wsmc_rng_block(seed, op, idx, (uint32_t)(k >> 1)), &z0, &z1);
                x[k] = wsmc_dist_mean_f(d, k, cols, N, i, 0, feat) + sd * z0;
                if (k + 1 < d->dim) x[k + 1] = wsmc_dist_mean_f(d, k + 1, cols, N, i, 0, feat) + sd * z1;
            }
            break;
        }
    }
}
WSMC_HD void wsmc_dist_sample_m(const wsmc_dist* d, double* x, uint64_t seed, uint64_t op, uint64_t idx,
                                double* const* cols, int64_t N, int64_t i, const double* sd_pre) {
    wsmc_dist_sample_mf(d, x, seed, op, idx, cols, N, i, sd_pre, WSMC_FEAT_ALL);
}

WSMC_HD void wsmc_dist_sample(const wsmc_dist* d, double* x, uint64_t seed, uint64_t op, uint64_t idx,
                              double* const* cols, int64_t N, int64_t i) {
    wsmc_dist_sample_m(d, x, seed, op, idx, cols, N, i, 0);
}
/* the operand is a constant (reads no column) */
WSMC_HD int wsmc_operand_is_const(const wsmc_operand* o) { return o->col[0] < 0 && o->col[1] < 0; }

/* Link an oscillator Observe term to the tape's previous term (prev, null at the start): when
 * prev is an oscillator Observe of the same operands and the times continue its block's
 * regular step (|t - (t_a + m d)| <= 64 eps (1 + |t|)), the term becomes (t_a, d, m) =
 * (dist.param[0], dist.param[1], dist.reserved) of its block; blocks hold at most
 * WSMC_OSC_BLOCK terms. Otherwise it opens a block (m = 0: the direct evaluation). Called
 * before the term is first evaluated, by the device library and the oracle alike. */
#ifndef WSMC_OSC_BLOCK
#define WSMC_OSC_BLOCK 64
#endif
WSMC_HD int wsmc_operand_same(const wsmc_operand* a, const wsmc_operand* b) {
    return wsmc_d2bits(a->c0) == wsmc_d2bits(b->c0) && wsmc_d2bits(a->coef[0]) == wsmc_d2bits(b->coef[0]) &&
           wsmc_d2bits(a->coef[1]) == wsmc_d2bits(b->coef[1]) && a->col[0] == b->col[0] && a->col[1] == b->col[1] &&
           a->comp[0] == b->comp[0] && a->comp[1] == b->comp[1];
}
WSMC_HD int wsmc_osc_term(const wsmc_term* t) {
    return t->kind == WSMC_TERM_OBSERVE && t->dist.family == WSMC_FAM_NORMAL && t->dist.dim <= 1 &&
           t->dist.mean_fn == WSMC_MEAN_OSCILLATOR;
}
WSMC_HD void wsmc_osc_link(const wsmc_term* prev, wsmc_term* t) {
    if (t->dist.mean_fn != WSMC_MEAN_OSCILLATOR) return;
    t->dist.reserved = 0;
    t->dist.param[1] = 0.0;
    if (!prev || !wsmc_osc_term(t) || !wsmc_osc_term(prev)) return;
    for (int k = 0; k < 4; ++k)
        if (!wsmc_operand_same(&prev->dist.mu[k], &t->dist.mu[k])) return;
    if (!wsmc_operand_same(&prev->dist.scale, &t->dist.scale)) return;
    const int mp = prev->dist.reserved;
    if (mp + 1 >= WSMC_OSC_BLOCK) return;
    const double ta = prev->dist.param[0], tk = t->dist.param[0];
    if (!wsmc_isfinite(ta) || !wsmc_isfinite(tk)) return;
    const double d = mp == 0 ? tk - ta : prev->dist.param[1];   /* a block's step: its second term */
    if (!wsmc_isfinite(d) || d == 0.0) return;
    if (mp > 0 && wsmc_fabs((ta + (double)(mp + 1) * d) - tk) > 1.4210854715202004e-14 * (1.0 + wsmc_fabs(tk)))
        return;
    t->dist.param[0] = ta;
    t->dist.param[1] = d;
    t->dist.reserved = mp + 1;
}

/* a scalar Normal (affine mean) / HalfNormal / Uniform term: wsmc_term_logpdf_m's arithmetic
 * for those families, without the other families' code (the device Move's lean fold) */
WSMC_HD int wsmc_term_is_scalar(const wsmc_term* t) {
    return t->dist.dim <= 1 && t->dist.mean_fn != WSMC_MEAN_OSCILLATOR &&
           (t->dist.family == WSMC_FAM_NORMAL || t->dist.family == WSMC_FAM_HALFNORMAL ||
            t->dist.family == WSMC_FAM_UNIFORM);
}
/* a Normal's per-sigma pair (c, rh) of wsmc_normal_logpdf through the fold's memo */
WSMC_HD void wsmc_normal_scale(wsmc_logmemo* lm, double sigma, double* c, double* rh) {
    double lg, rc;
    wsmc_scale_memo(lm, sigma, &lg, &rc);
    *c = wsmc_normal_c(lg);
    *rh = wsmc_normal_rh(rc);
}
/* pre: for a constant scale operand, the pair (c, rh) evaluated once by the caller
 * (wsmc_scale_pre: the same functions of the same bits as wsmc_normal_scale's), else null */
WSMC_HD double wsmc_scalar_term_logpdf_p(const wsmc_term* t, double* const* cols, int64_t N, int64_t i,
                                         const wsmc_override* ov, wsmc_logmemo* lm, const double* pre) {
    const wsmc_dist* d = &t->dist;
    const double x0 = wsmc_operand_eval(&t->x[0], cols, N, i, ov);
    if (d->family == WSMC_FAM_NORMAL || d->family == WSMC_FAM_HALFNORMAL) {
        const int half = d->family == WSMC_FAM_HALFNORMAL;
        if (half && !(x0 >= 0.0)) return -WSMC_INF;
        const double mu = half ? 0.0 : wsmc_operand_eval(&d->mu[0], cols, N, i, ov);
        double c, rh;
        if (pre) {
            c = pre[0];
            rh = pre[1];
        } else {
            wsmc_normal_scale(lm, wsmc_operand_eval(&d->scale, cols, N, i, ov), &c, &rh);
        }
        const double l = wsmc_normal_lh((x0 - mu) * rh, c);
        return half ? l + WSMC_LOG2 : l;
    }
    return wsmc_uniform_logpdf(d->param[0], d->param[1], x0);
}
WSMC_HD double wsmc_scalar_term_logpdf_m(const wsmc_term* t, double* const* cols, int64_t N, int64_t i,
                                         const wsmc_override* ov, wsmc_logmemo* lm) {
    return wsmc_scalar_term_logpdf_p(t, cols, N, i, ov, lm, 0);
}
/* the (c, rh) pair of a constant scale (wsmc_scalar_term_logpdf_p's pre) */
WSMC_HD void wsmc_scale_pre(double sigma, double* pre) {
    pre[0] = wsmc_normal_c(wsmc_log(sigma));
    pre[1] = wsmc_normal_rh(1.0 / sigma);
}

WSMC_HD double wsmc_term_logpdf_mf(const wsmc_term* t, double* const* cols, int64_t N, int64_t i,
                                   const wsmc_override* ov, wsmc_logmemo* lm, unsigned feat) {
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    int dim = t->dist.dim < 1 ? 1 : (t->dist.dim > 4 ? 4 : t->dist.dim);
    for (int k = 0; k < dim; ++k) x[k] = wsmc_operand_eval(&t->x[k], cols, N, i, ov);
    return wsmc_dist_logpdf_mf(&t->dist, x, cols, N, i, ov, lm, feat);
}
WSMC_HD double wsmc_term_logpdf_m(const wsmc_term* t, double* const* cols, int64_t N, int64_t i,
                                  const wsmc_override* ov, wsmc_logmemo* lm) {
    return wsmc_term_logpdf_mf(t, cols, N, i, ov, lm, WSMC_FEAT_ALL);
}
WSMC_HD double wsmc_term_logpdf(const wsmc_term* t, double* const* cols, int64_t N, int64_t i,
                                const wsmc_override* ov) {
    return wsmc_term_logpdf_m(t, cols, N, i, ov, 0);
}

/* score_logpdf! for one particle: 0.0 then += each term with depth < target_depth */
WSMC_HD double wsmc_fold(const wsmc_term* terms, int32_t n, int32_t target_depth, double* const* cols,
                         int64_t N, int64_t i, const wsmc_override* ov) {
    double s = 0.0;
    wsmc_logmemo lm = {0, 0.0, 0.0, 0};
    for (int32_t j = 0; j < n; ++j) {
        if (terms[j].depth >= target_depth) break;
        s = s + wsmc_term_logpdf_m(&terms[j], cols, N, i, ov, &lm);
    }
    return s;
}

/* the same left fold continued from s0 over terms [j0, n) — bit-identical to wsmc_fold when
 * s0 is the fold over [0, j0) of the same values (the carried score of a Move) */
WSMC_HD double wsmc_fold_from(double s0, const wsmc_term* terms, int32_t j0, int32_t n, int32_t target_depth,
                              double* const* cols, int64_t N, int64_t i, const wsmc_override* ov) {
    double s = s0;
    wsmc_logmemo lm = {0, 0.0, 0.0, 0};
    for (int32_t j = j0; j < n; ++j) {
        if (terms[j].depth >= target_depth) break;
        s = s + wsmc_term_logpdf_m(&terms[j], cols, N, i, ov, &lm);
    }
    return s;
}

#endif /* WSMC_TERMS_H */
