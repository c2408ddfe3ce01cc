/*
 * wsmc_port_fast.c — "reference-speed" CPU ports of the path (bench cpu_baseline legs).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/ and bench.py's cpu_baseline leg call it.
 *
 * The bit-exact ports (wsmc_oracle.c, wsmc_port_mt.c) evaluate the canonical draws and
 * transcendentals (Philox4x32-10 + Box–Muller, fdlibm-style exp/log/sincos), which cost
 * several times what the reference's Julia path spends per particle-step (Xoshiro256++,
 * ziggurat randn, libm). SURVEY.md §8(d) asks that the 1-thread CPU baseline land within
 * about 2x of the reference's published single-thread rate, or the baseline is unfair. This
 * file is the reference's algorithm at the reference's speed, NOT bit-exact:
 *   - RNG: xoshiro256++ (the algorithm of Julia's default RNG), one stream per thread,
 *     normals by the Marsaglia–Tsang ziggurat (Julia's randn is a ziggurat too); the
 *     stratified offsets are a counter hash per slot so that threads agree on them;
 *   - transcendentals: libm exp/log;
 *   - Resample.apply! exactly as src/transformers.jl:474-498 with src/resampling.jl:13-77
 *     in f64: max, exp(lw - m), Σ, ESS% = 1/(N Σ w²) with w = e/Σe (strict <),
 *     stratified u_n = (n - 1 + U_n)/N against the running cumulative sum (icdf), the
 *     column gather, and the weights reset to logsumexp(lw) - log N.
 * Results are statistically equivalent (tests/test_port_fast.py checks the Kalman
 * evidence), not equal, to the oracle's. Threads: OpenMP over particles; the cumulative
 * sum is blocked (chunk sums, offsets) and each thread merges its own range of slots.
 */
#include <malloc.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

/*
 * Keep freed run buffers in the heap (glibc otherwise maps and unmaps every buffer above
 * 128 KB), so a timed run after a same-size warm-up does not pay first-touch page faults —
 * as the device run, which reuses its HBM buffers, does not. Process-wide; bench.py calls it
 * before its CPU warm-ups.
 */
int fp_keep_heap(void) {
    return mallopt(M_MMAP_THRESHOLD, 32 << 20) && mallopt(M_TRIM_THRESHOLD, 1 << 30) ? 0 : -1;
}

/* ---- xoshiro256++ (Blackman & Vigna), seeded through splitmix64 ---- */
typedef struct { uint64_t s[4]; uint64_t pad[4]; } xo_t;   /* one cache line per thread */

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static inline uint64_t xo_next(xo_t* r) {
    const uint64_t res = rotl64(r->s[0] + r->s[3], 23) + r->s[0];
    const uint64_t t = r->s[1] << 17;
    r->s[2] ^= r->s[0]; r->s[3] ^= r->s[1]; r->s[1] ^= r->s[2]; r->s[0] ^= r->s[3];
    r->s[2] ^= t;
    r->s[3] = rotl64(r->s[3], 45);
    return res;
}
static void xo_seed(xo_t* r, uint64_t seed, uint64_t stream) {
    uint64_t x = seed ^ (0xd1b54a32d192ed03ull * (stream + 1));
    for (int k = 0; k < 4; ++k) r->s[k] = splitmix64(&x);
}
static inline double xo_unif(xo_t* r) { return (double)(xo_next(r) >> 11) * 0x1.0p-53; }   /* [0, 1) */

/* ---- Marsaglia–Tsang ziggurat, 128 layers (J. Stat. Softw. 5(8), 2000) ---- */
static uint32_t zk[128];
static double zw[128], zf[128];
static int z_ready = 0;

static void zig_init(void) {
    if (z_ready) return;
    const double m1 = 2147483648.0, vn = 9.91256303526217e-3;
    double dn = 3.442619855899, tn = dn;
    const double q = vn / exp(-0.5 * dn * dn);
    zk[0] = (uint32_t)((dn / q) * m1);
    zk[1] = 0;
    zw[0] = q / m1;
    zw[127] = dn / m1;
    zf[0] = 1.0;
    zf[127] = exp(-0.5 * dn * dn);
    for (int i = 126; i >= 1; --i) {
        dn = sqrt(-2.0 * log(vn / dn + exp(-0.5 * dn * dn)));
        zk[i + 1] = (uint32_t)((dn / tn) * m1);
        tn = dn;
        zf[i] = exp(-0.5 * dn * dn);
        zw[i] = dn / m1;
    }
    z_ready = 1;
}

static double zig_tail(xo_t* r, int32_t hz, uint32_t iz) {
    const double rr = 3.442619855899;
    for (;;) {
        const double x = hz * zw[iz];
        if (iz == 0) {
            double xx, y;
            do {
                xx = -log(1.0 - xo_unif(r)) / rr;
                y = -log(1.0 - xo_unif(r));
            } while (y + y < xx * xx);
            return hz > 0 ? rr + xx : -rr - xx;
        }
        if (zf[iz] + xo_unif(r) * (zf[iz - 1] - zf[iz]) < exp(-0.5 * x * x)) return x;
        hz = (int32_t)(uint32_t)(xo_next(r) >> 32);
        iz = (uint32_t)hz & 127u;
        if ((uint32_t)(hz < 0 ? -(int64_t)hz : hz) < zk[iz]) return hz * zw[iz];
    }
}
static inline double zig_normal(xo_t* r) {
    const int32_t hz = (int32_t)(uint32_t)(xo_next(r) >> 32);
    const uint32_t iz = (uint32_t)hz & 127u;
    if ((uint32_t)(hz < 0 ? -(int64_t)hz : hz) < zk[iz]) return hz * zw[iz];
    return zig_tail(r, hz, iz);
}

/* the stratified offset U_n of slot n at step t: a counter hash, so every thread agrees */
static inline double strat_u(uint64_t seed, uint64_t t, uint64_t n) {
    uint64_t x = seed ^ (t * 0xa0761d6478bd642full) ^ (n * 0xe7037ed1a0b428dbull);
    return (double)(splitmix64(&x) >> 11) * 0x1.0p-53;
}

/*
 * Resample.apply! (src/transformers.jl:474-498) on a state whose max log-weight is M.
 * Fills anc[n] (the slot's ancestor) when it resamples; returns 1 if it resampled.
 * e: scratch [N]; cs: per-thread chunk sums [nthreads + 1].
 */
static int resample_f64(int64_t N, double* w, double M, double ess_min, uint64_t seed, uint64_t t, int nth,
                        double* e, double* cs, int32_t* anc, double* mean_out) {
    double S = 0.0, S2 = 0.0;
    const int64_t chunk = (N + nth - 1) / nth;
#pragma omp parallel num_threads(nth) reduction(+ : S, S2)
    {
        const int th = omp_get_thread_num();
        const int64_t lo = th * chunk < N ? th * chunk : N, hi = lo + chunk < N ? lo + chunk : N;
        double s = 0.0, s2 = 0.0;
        for (int64_t i = lo; i < hi; ++i) {           /* exp_norm (src/resampling.jl:72-77) */
            const double v = exp(w[i] - M);
            e[i] = v;
            s += v;
            s2 += v * v;
        }
        cs[th + 1] = s;
        S += s;
        S2 += s2;
    }
    const double ess = (S * S) / ((double)N * S2);    /* ess_perc = 1/(N Σ (e/S)^2) (:51-54) */
    if (!(ess < ess_min)) return 0;                    /* strict, src/transformers.jl:484 */
    *mean_out = M + log(S) - log((double)N);           /* logsumexp(lw) - log N (:486-489) */
    cs[0] = 0.0;
    for (int k = 0; k < nth; ++k) cs[k + 1] += cs[k];
    const double inv = 1.0 / (double)N;
#pragma omp parallel num_threads(nth)
    {
        /* this thread's slots [slo, shi): merge u_n = (n + U_n)/N · S against the running
         * cumulative sum (icdf, src/resampling.jl:13-26), starting from the chunk that holds
         * u_slo */
        const int th = omp_get_thread_num();
        const int64_t slo = th * chunk < N ? th * chunk : N, shi = slo + chunk < N ? slo + chunk : N;
        if (slo < shi) {
            const double u0 = ((double)slo + strat_u(seed, t, (uint64_t)slo)) * inv * S;
            int k = 0;
            while (k + 1 < nth && cs[k + 1] < u0) ++k;
            int64_t m = k * chunk;
            double c;
            if (m < N) {
                c = cs[k] + e[m];
            } else {                                   /* u0 past the total (round-off): clamp */
                m = N - 1;
                c = cs[nth];
            }
            for (int64_t n = slo; n < shi; ++n) {
                const double u = ((double)n + strat_u(seed, t, (uint64_t)n)) * inv * S;
                while (c < u && m + 1 < N) c += e[++m];    /* clamp at N (round-off overrun) */
                anc[n] = (int32_t)m;
            }
        }
    }
    return 1;
}

/*
 * The reference's CPU benchmark model (benchmarks/ssm/WeightedSampling/lgssm1d.jl:18-24):
 * x ~ Normal(0, x0_std); per y: x ~ Normal(a x, q); y => Normal(x, r); Resample.
 * Returns 0; out: log_evidence, the final weighted posterior mean of x, the resample count.
 */
int fp_lgssm1d_run(int64_t N, int32_t T, const double* data, double a, double q, double r, double x0_std,
                   double ess_min, uint64_t seed, int32_t nthreads, double* log_evidence, double* post_mean,
                   int32_t* n_resamples) {
    if (N <= 0 || T < 1 || !data || N >= ((int64_t)1 << 31)) return -1;
    const int nth = nthreads < 1 ? 1 : nthreads;
    zig_init();
    double* x = malloc(sizeof(double) * (size_t)N);
    double* xb = malloc(sizeof(double) * (size_t)N);
    double* w = malloc(sizeof(double) * (size_t)N);
    double* e = malloc(sizeof(double) * (size_t)N);
    int32_t* anc = malloc(sizeof(int32_t) * (size_t)N);
    double* cs = calloc((size_t)nth + 1, sizeof(double));
    double* tm = calloc((size_t)nth, sizeof(double));
    xo_t* rng = malloc(sizeof(xo_t) * (size_t)nth);
    if (!x || !xb || !w || !e || !anc || !cs || !tm || !rng) {
        free(x); free(xb); free(w); free(e); free(anc); free(cs); free(tm); free(rng);
        return -1;
    }
    for (int k = 0; k < nth; ++k) xo_seed(&rng[k], seed, (uint64_t)k);
    const double lr = log(r), l2pi = log(2.0 * M_PI);
    int nrs = 0;
#pragma omp parallel for num_threads(nth) schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        x[i] = x0_std * zig_normal(&rng[omp_get_thread_num()]);
        w[i] = 0.0;
    }
    for (int t = 1; t <= T; ++t) {
        const double y = data[t - 1];
#pragma omp parallel num_threads(nth)
        {
            const int th = omp_get_thread_num();
            xo_t* g = &rng[th];
            double M = -INFINITY;
#pragma omp for schedule(static)
            for (int64_t i = 0; i < N; ++i) {
                const double xn = a * x[i] + q * zig_normal(g);          /* x ~ Normal(a x, q) */
                const double z = (y - xn) / r;                          /* y => Normal(x, r) */
                const double wn = w[i] - 0.5 * (z * z + l2pi) - lr;
                x[i] = xn;
                w[i] = wn;
                if (wn > M) M = wn;
            }
            tm[th] = M;
        }
        double M = -INFINITY;
        for (int k = 0; k < nth; ++k) M = tm[k] > M ? tm[k] : M;
        double mean = 0.0;
        if (resample_f64(N, w, M, ess_min, seed, (uint64_t)t, nth, e, cs, anc, &mean)) {
#pragma omp parallel for num_threads(nth) schedule(static)
            for (int64_t n = 0; n < N; ++n) {                           /* resample!(store, idx) */
                xb[n] = x[anc[n]];
                w[n] = mean;                                            /* fill!(weights, mean) */
            }
            double* sw = x; x = xb; xb = sw;
            ++nrs;
        }
    }
    double M = -INFINITY, S = 0.0, SX = 0.0;
    for (int64_t i = 0; i < N; ++i) M = w[i] > M ? w[i] : M;
    for (int64_t i = 0; i < N; ++i) {
        const double v = exp(w[i] - M);
        S += v;
        SX += v * x[i];
    }
    if (log_evidence) *log_evidence = M + log(S) - log((double)N);      /* src/utils.jl:21 */
    if (post_mean) *post_mean = SX / S;
    if (n_resamples) *n_resamples = nrs;
    free(x); free(xb); free(w); free(e); free(anc); free(cs); free(tm); free(rng);
    return 0;
}

/*
 * examples/2D_ssm.jl:7-17 with the history kept (x_1..x_{T+1} materialised), organised like
 * wsmc_port_mt.c (gather-on-read through the ancestor log, one trace-back at the end).
 * xs (optional): (T+1) columns, each SoA [2][N]. Returns 0.
 */
int fp_ssm2d_run(int64_t N, int32_t T, const double* obs, const double* x0, const double* v0, double q_var,
                 double r_var, double ess_min, uint64_t seed, int32_t nthreads, double* xs, double* log_evidence,
                 int32_t* n_resamples) {
    if (N <= 0 || T < 1 || !obs || !x0 || !v0 || N >= ((int64_t)1 << 31)) return -1;
    const int nth = nthreads < 1 ? 1 : nthreads;
    zig_init();
    double** hist = calloc((size_t)T + 2, sizeof(double*));
    double* vb[2] = {malloc(sizeof(double) * 2 * (size_t)N), malloc(sizeof(double) * 2 * (size_t)N)};
    double* w = malloc(sizeof(double) * (size_t)N);
    double* e = malloc(sizeof(double) * (size_t)N);
    int32_t* anc = malloc(sizeof(int32_t) * (size_t)N * (size_t)T);
    int32_t* rs = calloc((size_t)T + 1, sizeof(int32_t));
    double* mean = calloc((size_t)T + 1, sizeof(double));
    double* cs = calloc((size_t)nth + 1, sizeof(double));
    double* tm = calloc((size_t)nth, sizeof(double));
    xo_t* rng = malloc(sizeof(xo_t) * (size_t)nth);
    int ok = hist && vb[0] && vb[1] && w && e && anc && rs && mean && cs && tm && rng;
    for (int k = 2; ok && k <= T + 1; ++k) ok = (hist[k] = malloc(sizeof(double) * 2 * (size_t)N)) != NULL;
    if (!ok) {
        if (hist) for (int k = 0; k <= T + 1; ++k) free(hist[k]);
        free(hist); free(vb[0]); free(vb[1]); free(w); free(e); free(anc); free(rs); free(mean); free(cs);
        free(tm); free(rng);
        return -1;
    }
    for (int k = 0; k < nth; ++k) xo_seed(&rng[k], seed, (uint64_t)k);
    const double q_sd = sqrt(q_var);
    const double cpre = 2.0 * log(2.0 * M_PI) + 2.0 * log(r_var);   /* log|2π Σ| for Σ = r I₂ */
    memset(w, 0, sizeof(double) * (size_t)N);
    int nrs = 0;
    for (int t = 1; t <= T; ++t) {
        const int rsp = t > 1 && rs[t - 1];
        const double meanp = rsp ? mean[t - 1] : 0.0;
        const int32_t* ap = t > 1 ? anc + (size_t)(t - 2) * (size_t)N : NULL;
        const double* xp = t > 1 ? hist[t] : NULL;
        double* xn = hist[t + 1];
        const double* vp = vb[t & 1];
        double* vn = vb[(t + 1) & 1];
        const double o0 = obs[2 * (t - 1)], o1 = obs[2 * (t - 1) + 1];
#pragma omp parallel num_threads(nth)
        {
            const int th = omp_get_thread_num();
            xo_t* g = &rng[th];
            double M = -INFINITY;
#pragma omp for schedule(static)
            for (int64_t n = 0; n < N; ++n) {
                const int64_t s = rsp ? ap[n] : n;
                const double xa = t > 1 ? xp[2 * s] : x0[0], xc = t > 1 ? xp[2 * s + 1] : x0[1];
                const double va = t > 1 ? vp[2 * s] : v0[0], vc = t > 1 ? vp[2 * s + 1] : v0[1];
                const double xn0 = xa + va, xn1 = xc + vc;                      /* x{t+1} .= x{t} + v */
                const double vn0 = va + q_sd * zig_normal(g);                    /* dv ~ MvNormal(0, q I) */
                const double vn1 = vc + q_sd * zig_normal(g);                    /* v .= v + dv */
                const double d0 = o0 - xn0, d1 = o1 - xn1;                       /* o => MvNormal(x, r I) */
                const double wn = (rsp ? meanp : w[n]) - 0.5 * (cpre + (d0 * d0 + d1 * d1) / r_var);
                xn[2 * n] = xn0; xn[2 * n + 1] = xn1;
                vn[2 * n] = vn0; vn[2 * n + 1] = vn1;
                w[n] = wn;
                if (wn > M) M = wn;
            }
            tm[th] = M;
        }
        double M = -INFINITY;
        for (int k = 0; k < nth; ++k) M = tm[k] > M ? tm[k] : M;
        rs[t] = resample_f64(N, w, M, ess_min, seed, (uint64_t)t, nth, e, cs, anc + (size_t)(t - 1) * (size_t)N,
                             &mean[t]);
        nrs += rs[t];
    }
    /* trace-back: the columns the reference's per-resample gathers leave (src/stores.jl:105-128) */
#pragma omp parallel for num_threads(nth) schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        int64_t s = rs[T] ? anc[(size_t)(T - 1) * (size_t)N + i] : i;
        if (rs[T]) w[i] = mean[T];
        const int64_t col = 2 * N;
        double xa = hist[T + 1][2 * s], xc = hist[T + 1][2 * s + 1];
        if (xs) { xs[(size_t)T * col + i] = xa; xs[(size_t)T * col + N + i] = xc; }
        for (int u = T - 1; u >= 1; --u) {
            if (rs[u]) s = anc[(size_t)(u - 1) * (size_t)N + s];
            xa = hist[u + 1][2 * s]; xc = hist[u + 1][2 * s + 1];
            if (xs) { xs[(size_t)u * col + i] = xa; xs[(size_t)u * col + N + i] = xc; }
        }
        if (xs) { xs[i] = x0[0]; xs[N + i] = x0[1]; }
    }
    if (log_evidence) {
        double M = -INFINITY, S = 0.0;
        for (int64_t i = 0; i < N; ++i) M = w[i] > M ? w[i] : M;
        for (int64_t i = 0; i < N; ++i) S += exp(w[i] - M);
        *log_evidence = M + log(S) - log((double)N);
    }
    if (n_resamples) *n_resamples = nrs;
    for (int k = 0; k <= T + 1; ++k) free(hist[k]);
    free(hist); free(vb[0]); free(vb[1]); free(w); free(e); free(anc); free(rs); free(mean); free(cs); free(tm);
    free(rng);
    return 0;
}
