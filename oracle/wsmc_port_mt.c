/*
 * wsmc_port_mt.c — multi-threaded CPU port of the fused 2D SSM run (bench cpu_baseline).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/ and bench.py's cpu_baseline leg call it: the
 * tests check it bit for bit against the statement-by-statement oracle (wsmc_oracle.c),
 * and bench.py times it on the GPU box's host cores as the all-cores CPU baseline of
 * SURVEY.md §8(d) ("(ii) all host cores with OpenMP over particles; the scan is blocked").
 *
 * It runs examples/2D_ssm.jl:7-17 (x{t+1} .= x{t} + v; dv ~ MvNormal(0, q I); v .= v + dv;
 * o => MvNormal(x{t+1}, r I); the auto-inserted Resample of src/transformers.jl:474-498)
 * with the canonical arithmetic of include/wsmc_math.h, organised the way a good CPU
 * implementation would be rather than the way the reference's store is:
 *   - gather-on-read through the previous step's ancestors instead of the eager per-resample
 *     gather of every column (src/stores.jl:105-128, O(T^2) per run), with the history
 *     traced back once at the end (the device's k_ssm2d_final);
 *   - OpenMP over particles for the propagate, the statistics, the per-particle rank of the
 *     icdf merge (src/resampling.jl:13-26) and the trace-back; the CDF prefix is blocked
 *     (per-thread chunk sums, then offsets).
 * The statistics are exact integers and the ancestor of a slot does not depend on how the
 * particles are split, so the result is identical for every thread count and equal to the
 * oracle's statements and the device's fused run.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "wsmc.h"
#include "wsmc_math.h"

/* c0 + 1*a + 1*b: the affine operand order of the assign operator (k_ssm2d_prop's aff2) */
static inline double aff2(double a, double b) {
    double v = 0.0;
    v = v + 1.0 * a;
    v = v + 1.0 * b;
    return v;
}

typedef struct {
    double M;
    int nan;
    uint64_t Q, Q2;
    wsmc_u128 Wf2, Wf;
} part_stats;

/*
 * outputs (each may be NULL; the trace-back runs regardless, it is part of the timed run):
 *   xs      (T+1) columns x_1..x_{T+1}, each SoA [2][N] (keep_history), or x (one column)
 *   v, dv   SoA [2][N];  w [N];  flags [T] (resampled per step)
 * returns 0, or -1 on a bad argument / allocation failure
 */
int or_ssm2d_run_mt(int64_t N, uint64_t seed, uint64_t op_base, uint64_t goff, const double* w0, const double* obs,
                    int32_t T,
                    const double* x0, const double* v0, double q_var, double r_var, double ess_min, int32_t scheme,
                    int32_t keep_history, int32_t nthreads, double* xs, double* v_out, double* dv_out, double* w_out,
                    int32_t* flags, double* log_evidence) {
    if (N <= 0 || T < 1 || !obs || !x0 || !v0 || N >= ((int64_t)1 << 31)) return -1;
    if (scheme != WSMC_RESAMPLE_STRATIFIED && scheme != WSMC_RESAMPLE_SYSTEMATIC) return -1;
    if (nthreads < 1) nthreads = 1;
    const int keep = keep_history != 0;
    const int nh = keep ? T + 2 : 2;            /* history buffers x_2..x_{T+1} (pairs), or a ping-pong */
    double** hist = (double**)calloc((size_t)nh, sizeof(double*));
    double* vb[2] = {malloc(sizeof(double) * 2 * (size_t)N), malloc(sizeof(double) * 2 * (size_t)N)};
    double* dvw = malloc(sizeof(double) * 2 * (size_t)N);
    double* w = malloc(sizeof(double) * (size_t)N);
    uint64_t* q = malloc(sizeof(uint64_t) * (size_t)N);
    int32_t* anc = malloc(sizeof(int32_t) * (size_t)N * (size_t)T);
    int32_t* rs = calloc((size_t)T + 1, sizeof(int32_t));
    double* mean = calloc((size_t)T + 1, sizeof(double));
    part_stats* ps = calloc((size_t)nthreads, sizeof(part_stats));
    uint64_t* coff = calloc((size_t)nthreads + 1, sizeof(uint64_t));
    int ok = hist && vb[0] && vb[1] && dvw && w && q && anc && rs && mean && ps && coff;
    for (int k = 0; ok && k < nh; ++k)
        if (keep ? k >= 2 : 1) ok = (hist[k] = malloc(sizeof(double) * 2 * (size_t)N)) != NULL;
    if (!ok) {
        if (hist) for (int k = 0; k < nh; ++k) free(hist[k]);
        free(hist); free(vb[0]); free(vb[1]); free(dvw); free(w); free(q); free(anc); free(rs); free(mean);
        free(ps); free(coff);
        return -1;
    }
    if (w0) memcpy(w, w0, sizeof(double) * (size_t)N);
    else memset(w, 0, sizeof(double) * (size_t)N);
    const int K = wsmc_qbits((uint64_t)N);
    const double q_sd = wsmc_sqrt(q_var);
    const double c0 = 2.0 * WSMC_LOG2PI + 2.0 * wsmc_log(r_var);
#define XBUF(t) (keep ? hist[(t)] : hist[(t) & 1])   /* x_t, t >= 2 */

    for (int t = 1; t <= T; ++t) {
        const uint64_t op_dv = op_base + 3ull * (uint64_t)(t - 1);
        const uint64_t op_rs = op_dv + 2ull;
        const int rsp = t > 1 && rs[t - 1];
        const double meanp = rsp ? mean[t - 1] : 0.0;
        const int32_t* ap = t > 1 ? anc + (size_t)(t - 2) * (size_t)N : NULL;
        const double* xp = t > 1 ? XBUF(t) : NULL;
        double* xn = XBUF(t + 1);
        const double* vp = vb[t & 1];
        double* vn = vb[(t + 1) & 1];
        const double o0 = obs[2 * (t - 1)], o1 = obs[2 * (t - 1) + 1];
        /* ---- propagate + observe, per-thread max ---- */
#pragma omp parallel num_threads(nthreads)
        {
            const int th = omp_get_thread_num();
            double M = -WSMC_INF;
            int nan = 0;
#pragma omp for schedule(static)
            for (int64_t n = 0; n < N; ++n) {
                const int64_t s = rsp ? ap[n] : n;
                const double xa = t > 1 ? xp[2 * s] : x0[0], xb = t > 1 ? xp[2 * s + 1] : x0[1];
                const double va = t > 1 ? vp[2 * s] : v0[0], vbb = t > 1 ? vp[2 * s + 1] : v0[1];
                double z0, z1;
                wsmc_normal_pair(wsmc_rng_block(seed, op_dv, goff + (uint64_t)n, 0u), &z0, &z1);
                const double xn0 = aff2(xa, va), xn1 = aff2(xb, vbb);            /* x{t+1} .= x{t} + v */
                const double dv0 = 0.0 + q_sd * z0, dv1 = 0.0 + q_sd * z1;       /* dv ~ MvNormal(0, q I) */
                const double vn0 = aff2(va, dv0), vn1 = aff2(vbb, dv1);          /* v .= v + dv */
                const double m0 = 0.0 + 1.0 * xn0, m1 = 0.0 + 1.0 * xn1;
                double ss = 0.0;
                const double d0 = o0 - m0, d1 = o1 - m1;
                ss = ss + d0 * d0;
                ss = ss + d1 * d1;
                const double lp = -(c0 + ss / r_var) * 0.5;                     /* o => MvNormal(x{t+1}, r I) */
                const double wn = (rsp ? meanp : w[n]) + lp;
                xn[2 * n] = xn0; xn[2 * n + 1] = xn1;
                vn[2 * n] = vn0; vn[2 * n + 1] = vn1;
                if (t == T) { dvw[2 * n] = dv0; dvw[2 * n + 1] = dv1; }
                w[n] = wn;
                if (wsmc_isnan(wn)) nan = 1;
                else if (wn > M) M = wn;
            }
            ps[th].M = M;
            ps[th].nan = nan;
        }
        double M = -WSMC_INF;
        int nan = 0;
        for (int k = 0; k < nthreads; ++k) {
            if (ps[k].nan) nan = 1;
            else if (ps[k].M > M) M = ps[k].M;
        }
        if (nan) M = WSMC_NAN;                    /* maximum() propagates NaN */
        /* ---- exact integer statistics (order-free), against the reference point ---- */
        const double R = wsmc_qref(M);
#pragma omp parallel num_threads(nthreads)
        {
            const int th = omp_get_thread_num();
            uint64_t Q = 0, Q2 = 0;
            wsmc_u128 Wf2 = 0, Wf = 0;
#pragma omp for schedule(static)
            for (int64_t n = 0; n < N; ++n) {
                const wsmc_qparts p = wsmc_qparts_of(w[n], R, K);
                q[n] = p.q;
                Q += p.q;
                Q2 += p.q2;
                Wf2 += p.wf2;
                Wf += p.wf;
            }
            ps[th].Q = Q; ps[th].Q2 = Q2; ps[th].Wf2 = Wf2; ps[th].Wf = Wf;
        }
        wsmc_shard_stats st;
        st.M = M; st.Q = 0; st.Q2 = 0; st.Wf2 = 0; st.Wf = 0; st.n = (uint64_t)N;
        for (int k = 0; k < nthreads; ++k) {
            st.Q += ps[k].Q; st.Q2 += ps[k].Q2; st.Wf2 += ps[k].Wf2; st.Wf += ps[k].Wf;
        }
        const double ess = wsmc_global_ess(&st, 1);
        rs[t] = ess < ess_min;                    /* strict, src/transformers.jl:484 */
        if (flags) flags[t - 1] = rs[t];
        if (!rs[t]) continue;
        mean[t] = wsmc_shard_mean(&st);           /* fill!(weights, mean), src/transformers.jl:486-489 */
        /* ---- ancestors: blocked CDF prefix, then per-particle rank ---- */
        const uint64_t Q = st.Q;
        const double ratio = wsmc_u64_to_d((uint64_t)N) / wsmc_u64_to_d(Q);
        int32_t* a = anc + (size_t)(t - 1) * (size_t)N;
        const int64_t chunk = (N + nthreads - 1) / nthreads;
#pragma omp parallel num_threads(nthreads)
        {
            const int th = omp_get_thread_num();
            const int64_t lo = th * chunk < N ? th * chunk : N, hi = lo + chunk < N ? lo + chunk : N;
            uint64_t cs = 0;
            for (int64_t n = lo; n < hi; ++n) cs += q[n];
            coff[th + 1] = cs;
#pragma omp barrier
#pragma omp single
            for (int k = 0; k < nthreads; ++k) coff[k + 1] += coff[k];
            /* particle m owns the slots [rank(C_{m-1}), rank(C_m)) */
            uint64_t C = coff[th];
            uint64_t prev = wsmc_rank_r(C, Q, (uint64_t)N, ratio, scheme, seed, op_rs, goff);
            for (int64_t m = lo; m < hi; ++m) {
                C += q[m];
                const uint64_t h = q[m] ? wsmc_rank_r(C, Q, (uint64_t)N, ratio, scheme, seed, op_rs, goff) : prev;
                for (uint64_t s = prev; s < h; ++s) a[s] = (int32_t)m;
                prev = h;
            }
        }
    }
    /* ---- trace-back (k_ssm2d_final): the columns the per-resample gathers would leave ---- */
    const double* vw = vb[(T + 1) & 1];
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        int64_t s = rs[T] ? anc[(size_t)(T - 1) * (size_t)N + i] : i;
        if (v_out) { v_out[i] = vw[2 * s]; v_out[N + i] = vw[2 * s + 1]; }
        if (dv_out) { dv_out[i] = dvw[2 * s]; dv_out[N + i] = dvw[2 * s + 1]; }
        if (rs[T]) w[i] = mean[T];
        if (!keep) {
            if (xs) { xs[i] = XBUF(T + 1)[2 * s]; xs[N + i] = XBUF(T + 1)[2 * s + 1]; }
            continue;
        }
        const int64_t col = 2 * N;                 /* x_t is column t-1 of xs */
        double xa = hist[T + 1][2 * s], xb = hist[T + 1][2 * s + 1];
        if (xs) { xs[(size_t)T * col + i] = xa; xs[(size_t)T * col + N + i] = xb; }
        for (int u = T - 1; u >= 1; --u) {
            if (rs[u]) s = anc[(size_t)(u - 1) * (size_t)N + s];
            xa = hist[u + 1][2 * s]; xb = hist[u + 1][2 * s + 1];
            if (xs) { xs[(size_t)u * col + i] = xa; xs[(size_t)u * col + N + i] = xb; }
        }
        if (xs) { xs[i] = x0[0]; xs[N + i] = x0[1]; }
    }
#undef XBUF
    if (w_out) memcpy(w_out, w, sizeof(double) * (size_t)N);
    if (log_evidence) {                           /* logsumexp(w) - log N (src/utils.jl:21) */
        double M = -WSMC_INF;
        int nan = 0;
        for (int64_t i = 0; i < N; ++i) {
            if (wsmc_isnan(w[i])) nan = 1;
            else if (w[i] > M) M = w[i];
        }
        wsmc_shard_stats st;
        st.M = nan ? WSMC_NAN : M; st.Q = 0; st.Q2 = 0; st.Wf2 = 0; st.Wf = 0; st.n = (uint64_t)N;
        for (int64_t i = 0; i < N; ++i) {
            const wsmc_qparts p = wsmc_qparts_of(w[i], wsmc_qref(st.M), K);
            st.Q += p.q; st.Q2 += p.q2; st.Wf2 += p.wf2; st.Wf += p.wf;
        }
        *log_evidence = wsmc_global_log_evidence(&st, 1);
    }
    for (int k = 0; k < nh; ++k) free(hist[k]);
    free(hist); free(vb[0]); free(vb[1]); free(dvw); free(w); free(q); free(anc); free(rs); free(mean);
    free(ps); free(coff);
    return 0;
}
