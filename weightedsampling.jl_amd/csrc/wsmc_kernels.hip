// wsmc_kernels.hip — gfx950 kernels of the SMC inner loop.
//
// Per-particle arithmetic comes from include/wsmc_math.h / wsmc_terms.h, the same source
// the CPU oracle compiles, built with -ffp-contract=off: every per-particle value is
// bit-identical to the oracle's. Reductions that feed decisions are integer (exact,
// order-independent); floating reductions (autoRW moments) follow the canonical tile
// order documented in oracle/wsmc_oracle.c (canon_block).
//
// Layout: particle-major SoA f64 (component k of particle i at data[k*N + i]); one thread
// per particle for streaming kernels (coalesced 8-B lanes), 256-thread workgroups of
// 4 wave64s; tile kernels own 2048 particles (8 per thread).
#include "wsmc_internal.h"

namespace wsmc {

typedef unsigned long long u64;

// ------------------------------------------------------------------------------------
// wave / block primitives (wave64)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        u64 o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}
// canonical f64 block sum: xor butterfly 1..32 inside each wave, then (w0+w1)+(w2+w3)
__device__ __forceinline__ double block_sum_canon(double v, double* lds4) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v = v + __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ u64 block_sum_u64(u64 v, u64* lds4) {
    v = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    u64 r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ u64 block_max_u64(u64 v, u64* lds4) {
    v = wave_max_u64(v);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    u64 a = lds4[0] > lds4[1] ? lds4[0] : lds4[1];
    u64 b = lds4[2] > lds4[3] ? lds4[2] : lds4[3];
    __syncthreads();
    return a > b ? a : b;
}
// exclusive prefix sum over the block (thread order), also returns the block total
__device__ __forceinline__ u64 block_excl_scan_u64(u64 v, u64* lds4, u64* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u64 x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        u64 y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    u64 pre = 0;
    for (int k = 0; k < w; ++k) pre += lds4[k];
    *total = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();
    return pre + x - v;
}
// exclusive prefix max over the block (int, -1 = empty)
__device__ __forceinline__ int block_excl_max_i32(int v, int* lds4, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int y = __shfl_up(x, off, 64);
        if (lane >= off) x = y > x ? y : x;
    }
    int ex = __shfl_up(x, 1, 64);
    if (lane == 0) ex = -1;
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    int pre = -1;
    for (int k = 0; k < w; ++k) pre = lds4[k] > pre ? lds4[k] : pre;
    int t = lds4[0];
    for (int k = 1; k < 4; ++k) t = lds4[k] > t ? lds4[k] : t;
    *total = t;
    __syncthreads();
    return ex > pre ? ex : pre;
}

__device__ __forceinline__ void atomic_max_filtered(u64* p, u64 v) {
    u64 cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v > cur) atomicMax(p, v);
}

__device__ __forceinline__ uint64_t op_eff(uint64_t op, const uint64_t* op_dev) {
    return op_dev ? op_dev[0] + op : op;
}

// ------------------------------------------------------------------------------------
// elementwise operators: Assign / Sample / Observe / Weight
// ------------------------------------------------------------------------------------
struct AssignArgs { wsmc_operand e[4]; };

__global__ __launch_bounds__(kBlock) void k_assign(double* out, int dim, AssignArgs a,
                                                   double* const* cols, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    double x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) x[k] = wsmc_operand_eval(&a.e[k], cols, N, i, nullptr);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
}

__global__ __launch_bounds__(kBlock) void k_sample(double* out, int dim, wsmc_dist d, uint64_t seed,
                                                   uint64_t op, int64_t goff, double* const* cols,
                                                   int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    double x[4];
    wsmc_dist_sample(&d, x, seed, op, (uint64_t)(goff + i), cols, N, i);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
}

__global__ __launch_bounds__(kBlock) void k_sample_importance(double* out, int dim, wsmc_dist prop,
                                                              wsmc_dist targ, double* w, uint64_t seed,
                                                              uint64_t op, int64_t goff,
                                                              double* const* cols, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    double x[4];
    wsmc_dist_sample(&prop, x, seed, op, (uint64_t)(goff + i), cols, N, i);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
    double lt = wsmc_dist_logpdf(&targ, x, cols, N, i, nullptr);
    double lp = wsmc_dist_logpdf(&prop, x, cols, N, i, nullptr);
    w[i] = w[i] + (lt - lp);
}

__global__ __launch_bounds__(kBlock) void k_weigh(wsmc_term t, double* w, double* const* cols, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    w[i] = w[i] + wsmc_term_logpdf(&t, cols, N, i, nullptr);
}

// ------------------------------------------------------------------------------------
// Resample: max, integer sums, scan + ancestor fill (src/transformers.jl:474-498)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_rs_max(const double* __restrict__ w, int64_t N, ShardRec* rec) {
    __shared__ u64 lds[4];
    u64 m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock)
        m = max(m, (u64)wsmc_ord_enc(w[i]));
    m = block_max_u64(m, lds);
    if (threadIdx.x == 0) atomic_max_filtered(&rec->v[blockIdx.x % kSlots][0], m);
}

// slot reductions by one wave: lane l owns slot l (kSlots == 64)
static_assert(kSlots == 64, "one lane per accumulator slot");
__device__ __forceinline__ u64 wave_rec_max_enc(const ShardRec* r) {
    return wave_max_u64(r->v[threadIdx.x & 63][0]);
}
// block-uniform max of the record (all threads); uses one wave + LDS
__device__ __forceinline__ double block_rec_max(const ShardRec* r, u64* lds1) {
    if (threadIdx.x < 64) {
        const u64 m = wave_rec_max_enc(r);
        if (threadIdx.x == 0) lds1[0] = m;
    }
    __syncthreads();
    const double M = wsmc_ord_dec(lds1[0]);
    __syncthreads();
    return M;
}
// full shard statistics, computed by one wave (every lane returns the same value)
__device__ __forceinline__ wsmc_shard_stats wave_rec_stats(const ShardRec* r) {
    const int l = threadIdx.x & 63;
    wsmc_shard_stats st;
    st.M = wsmc_ord_dec(wave_max_u64(r->v[l][0]));
    st.Q = wave_sum_u64(r->v[l][1]);
    u64 lim[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) lim[k] = wave_sum_u64(r->v[l][2 + k]);
    st.Q2 = (wsmc_u128)lim[0] + ((wsmc_u128)lim[1] << 32) + ((wsmc_u128)lim[2] << 64) + ((wsmc_u128)lim[3] << 96);
    st.W = (wsmc_u128)lim[4] + ((wsmc_u128)lim[5] << 32) + ((wsmc_u128)lim[6] << 64) + ((wsmc_u128)lim[7] << 96);
    st.n = r->v[0][10];
    return st;
}

// one resample tile (1024 particles) per block, striped items (coalesced): sum q,
// sum q^2 (4 x 32-bit limbs), sum fix96(e) (4 limbs) into the shard record (atomics spread
// over kSlots copies); the tile's sum q -> tileQ (scan offsets).
__global__ __launch_bounds__(kBlock) void k_rs_sums(const double* __restrict__ w, int64_t N, ShardRec* rec,
                                                    u64* __restrict__ tileQ, u64* __restrict__ qbuf) {
    __shared__ u64 lds[4][9];
    __shared__ u64 s_m[1];
    const int64_t base = (int64_t)blockIdx.x * kRsTile;
    double lw[kRsItems];
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        const int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
        lw[j] = i < N ? w[i] : -WSMC_INF;
    }
    const double M = block_rec_max(rec, s_m);
    const int K = wsmc_qbits((uint64_t)N);
    const double scale = wsmc_pow2i(K);
    u64 acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        const double e = wsmc_exp(lw[j] - M);
        const u64 q = (e > 0.0) ? (u64)wsmc_d_to_u64_trunc(e * scale) : 0ull;
        const int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
        if (i < N) qbuf[i] = q;
        const wsmc_u128 q2 = (wsmc_u128)q * q;
        const wsmc_u128 f = wsmc_fix96(e);
        acc[0] += q;
        acc[1] += (uint32_t)q2;
        acc[2] += (uint32_t)(q2 >> 32);
        acc[3] += (uint32_t)(q2 >> 64);
        acc[4] += (uint32_t)(q2 >> 96);
        acc[5] += (uint32_t)f;
        acc[6] += (uint32_t)(f >> 32);
        acc[7] += (uint32_t)(f >> 64);
        acc[8] += (uint32_t)(f >> 96);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        u64 v = wave_sum_u64(acc[k]);
        if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 9) {
        const int k = threadIdx.x;
        const u64 v = (lds[0][k] + lds[1][k]) + (lds[2][k] + lds[3][k]);
        if (k == 0) tileQ[blockIdx.x] = v;
        if (v) atomicAdd(&rec->v[blockIdx.x % kSlots][1 + k], v);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) rec->v[0][10] = (u64)N;
}

// Global Resample decision from the shard records (rank order), the same arithmetic as
// wsmc_global_ess / wsmc_shard_mean. Called by all 64 lanes of one wave.
__device__ void decide(const ShardRec* recs, int world, int rank, double ess_min, double* ess_out,
                       int* rs_out, wsmc_shard_stats* mine) {
    double M = -WSMC_INF;
    uint64_t N = 0;
    int nan = 0;
    for (int g = 0; g < world; ++g) {
        const double Mg = wsmc_ord_dec(wave_rec_max_enc(&recs[g]));
        if (wsmc_isnan(Mg)) nan = 1;
        else if (Mg > M) M = Mg;
        N += recs[g].v[0][10];
    }
    if (nan) M = WSMC_NAN;
    double sq = 0.0, sq2 = 0.0;
    for (int g = 0; g < world; ++g) {
        const wsmc_shard_stats st = wave_rec_stats(&recs[g]);
        const double f = wsmc_exp(st.M - M);
        const double sc = wsmc_pow2i(-wsmc_qbits(st.n));
        const double qd = wsmc_u64_to_d(st.Q), q2d = wsmc_u128_to_d(st.Q2);
        sq = sq + (qd * sc) * f;
        sq2 = sq2 + ((q2d * sc) * sc) * (f * f);
        if (g == rank) *mine = st;
    }
    const double ess = (sq * sq) / (wsmc_u64_to_d(N) * sq2);
    *ess_out = ess;
    *rs_out = ess < ess_min;
}

// Decision + inclusive integer CDF + ancestor fill for one tile.
// ancestor(slot) = smallest m with C_m > x_slot (src/resampling.jl:13-26); particle m owns
// slots [rank(C_{m-1}), rank(C_m)) and the block fills its contiguous slot range through
// an LDS mark array + max-scan (load-balanced within the block).
__global__ __launch_bounds__(kBlock) void k_rs_scan(const double* __restrict__ w, int64_t N,
                                                    const ShardRec* recs, int world, int rank,
                                                    double ess_min, int scheme, uint64_t seed,
                                                    uint64_t op, const uint64_t* op_dev,
                                                    int64_t slot_base, const u64* __restrict__ tileQ,
                                                    const u64* __restrict__ qbuf,
                                                    int32_t* __restrict__ anc, Decision* dec) {
    __shared__ u64 s_u4[4];
    __shared__ int s_i4[4];
    __shared__ u64 s_hi[kBlock];
    __shared__ int marks[kRsChunk];
    __shared__ u64 s_Q, s_L;
    __shared__ int s_rs;
    const int th = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kRsTile;

    // issue this tile's loads and the offset loads before the decision
    u64 q[kRsItems];
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        const int64_t i = base + (int64_t)th * kRsItems + j;
        q[j] = i < N ? qbuf[i] : 0ull;
    }
    u64 part = 0;
    for (int64_t b = th; b < (int64_t)blockIdx.x; b += kBlock) part += tileQ[b];

    if (th < 64) {
        double ess;
        int rs;
        wsmc_shard_stats me;
        decide(recs, world, rank, ess_min, &ess, &rs, &me);
        if (th == 0) {
            s_Q = me.Q;
            s_rs = rs;
        }
        if (blockIdx.x == 0 && th == 0) {
            dec->resampled = rs;
            dec->ess = ess;
            dec->M = me.M;
            dec->mean = rs ? wsmc_shard_mean(&me) : 0.0;
        }
    }
    __syncthreads();
    if (!s_rs) return;
    const uint64_t opx = op_eff(op, op_dev);
    const u64 Q = s_Q;
    const double ratio = wsmc_u64_to_d((uint64_t)N) / wsmc_u64_to_d(Q);
    const u64 off = block_sum_u64(part, s_u4);

    // blocked items: thread th owns particles base + th*4 .. +3
    u64 tsum = 0;
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) tsum += q[j];
    u64 tot;
    const u64 pre = block_excl_scan_u64(tsum, s_u4, &tot);
    // hi_j = rank(C_j); lo_0 = rank(C_{-1})
    u64 hi[kRsItems];
    u64 C = off + pre;
    const u64 lo0 = wsmc_rank_r(C, Q, (uint64_t)N, ratio, scheme, seed, opx, (uint64_t)slot_base);
    u64 prev = lo0;
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        C += q[j];
        hi[j] = q[j] ? wsmc_rank_r(C, Q, (uint64_t)N, ratio, scheme, seed, opx, (uint64_t)slot_base) : prev;
        prev = hi[j];
    }
    s_hi[th] = hi[kRsItems - 1];
    if (th == 0) s_L = lo0;
    __syncthreads();
    const u64 Ls = s_L, H = s_hi[kBlock - 1];

    int carry = -1;
    constexpr int PT = kRsChunk / kBlock;   // slots per thread per chunk
    for (u64 cb = Ls; cb < H; cb += kRsChunk) {
#pragma unroll
        for (int k = 0; k < PT; ++k) marks[k * kBlock + th] = -1;
        __syncthreads();
        u64 lo = lo0;
#pragma unroll
        for (int j = 0; j < kRsItems; ++j) {
            if (lo < hi[j] && lo >= cb && lo < cb + kRsChunk) marks[lo - cb] = th * kRsItems + j;
            lo = hi[j];
        }
        __syncthreads();
        int run[PT];
        int m = -1;
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int v = marks[th * PT + k];
            m = v > m ? v : m;
            run[k] = m;
        }
        int ctot;
        const int ex = block_excl_max_i32(m, s_i4, &ctot);
        const int lead = ex > carry ? ex : carry;
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const u64 slot = cb + (u64)(th * PT + k);
            if (slot < H) {
                const int a = run[k] > lead ? run[k] : lead;
                anc[slot] = (int32_t)(base + a);
            }
        }
        carry = ctot > carry ? ctot : carry;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBlock) void k_gather(double* __restrict__ dst, const double* __restrict__ src,
                                                   const int32_t* __restrict__ anc, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    dst[i] = src[anc[i]];
}

__global__ __launch_bounds__(kBlock) void k_fill_weights(double* w, const Decision* dec, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N || !dec->resampled) return;
    w[i] = dec->mean;
}

// ------------------------------------------------------------------------------------
// score fold, autoRW moments, MH move (src/transformers.jl:588-623)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_score(const wsmc_term* tape, int32_t n, int32_t depth,
                                                  double* const* cols, int64_t N, double* out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    out[i] = wsmc_fold(tape, n, depth, cols, N, i, nullptr);
}

struct MomArgs {
    int32_t tcol[4];
    double lo[4], hi[4];
};

// pass 1: values {e, e*z_k};  pass 2: values {(e*(z_a-mean_a))*(z_b-mean_b), a <= b}
// written as canonical tile partials tilepart[v * ntiles + tile]
__global__ __launch_bounds__(kBlock) void k_moments(const double* __restrict__ w, const ShardRec* rec,
                                                    double* const* cols, MomArgs ma, int d, int pass,
                                                    const double* mom, int64_t N, int64_t ntiles,
                                                    double* tilepart) {
    __shared__ double lds4[4];
    __shared__ u64 s_m[1];
    const double M = block_rec_max(rec, s_m);
    const int64_t base = (int64_t)blockIdx.x * kTile;
    double acc[10];
    const int nv = pass == 1 ? 1 + d : d * (d + 1) / 2;
#pragma unroll
    for (int v = 0; v < 10; ++v) acc[v] = 0.0;
    double mean[4] = {0.0, 0.0, 0.0, 0.0};
    if (pass == 2)
        for (int k = 0; k < d; ++k) mean[k] = mom[k];
    for (int j = 0; j < kItems; ++j) {
        const int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
        double vals[10];
#pragma unroll
        for (int v = 0; v < 10; ++v) vals[v] = 0.0;
        if (i < N) {
            const double e = wsmc_exp(w[i] - M);
            double z[4];
            for (int k = 0; k < d; ++k) z[k] = wsmc_to_unc(cols[ma.tcol[k]][i], ma.lo[k], ma.hi[k]);
            if (pass == 1) {
                vals[0] = e;
                for (int k = 0; k < d; ++k) vals[1 + k] = e * z[k];
            } else {
                int v = 0;
                for (int a = 0; a < d; ++a)
                    for (int b = a; b < d; ++b) vals[v++] = (e * (z[a] - mean[a])) * (z[b] - mean[b]);
            }
        }
#pragma unroll
        for (int v = 0; v < 10; ++v) acc[v] = acc[v] + vals[v];
    }
    for (int v = 0; v < nv; ++v) {
        const double s = block_sum_canon(acc[v], lds4);
        if (threadIdx.x == 0) tilepart[(int64_t)v * ntiles + blockIdx.x] = s;
    }
}

// one block: canonical combine of tile partials; pass 1 -> mom[0..d) = mean, mom[8] = S0;
// pass 2 -> mom[16..16+d*d) = lambda*Sigma (zeros -> min_step), mom[32..32+d*d) = chol
__global__ __launch_bounds__(kBlock) void k_moments_final(const double* tilepart, int64_t ntiles, int d,
                                                          int pass, double min_step, double* mom,
                                                          int32_t* flag) {
    __shared__ double lds4[4];
    __shared__ double tot[10];
    const int nv = pass == 1 ? 1 + d : d * (d + 1) / 2;
    for (int v = 0; v < nv; ++v) {
        double acc = 0.0;
        for (int64_t b = threadIdx.x; b < ntiles; b += kBlock) acc = acc + tilepart[(int64_t)v * ntiles + b];
        const double s = block_sum_canon(acc, lds4);
        if (threadIdx.x == 0) tot[v] = s;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (pass == 1) {
        const double S0 = tot[0];
        for (int k = 0; k < d; ++k) mom[k] = tot[1 + k] / S0;
        mom[8] = S0;
        return;
    }
    const double S0 = mom[8];
    double S[16], L[16];
    int v = 0;
    for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b) {
            const double c = tot[v++] / S0;
            S[a * d + b] = c;
            S[b * d + a] = c;
        }
    const double lam = 2.38 / wsmc_sqrt((double)d);
    for (int k = 0; k < d * d; ++k) {
        if (S[k] == 0.0) S[k] = min_step;
        S[k] = lam * S[k];
        mom[16 + k] = S[k];
    }
    const int ok = wsmc_cholesky(S, L, d);
    for (int k = 0; k < d * d; ++k) mom[32 + k] = L[k];
    if (!ok) flag[0] = 1;
}

__global__ __launch_bounds__(kBlock) void k_move(const wsmc_term* tape, int32_t nterms, int32_t depth,
                                                 double* const* cols, MomArgs ma, int d, int bounded,
                                                 const double* Lm, uint64_t seed, uint64_t op_prop,
                                                 uint64_t op_acc, int64_t goff, int64_t N, u64* accepted) {
    __shared__ u64 lds4[4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    u64 acc = 0;
    if (i < N) {
        double xi[4], dz[4];
        for (int k = 0; k < d; ++k) xi[k] = wsmc_normal_k(seed, op_prop, (uint64_t)(goff + i), (uint32_t)k);
        for (int k = 0; k < d; ++k) {
            double s = 0.0;
            for (int j = 0; j <= k; ++j) s = s + Lm[k * d + j] * xi[j];
            dz[k] = s;
        }
        wsmc_override ov;
        ov.n = d;
        double lpr = 0.0;
        for (int k = 0; k < d; ++k) {
            const double x = cols[ma.tcol[k]][i];
            const double zo = bounded ? wsmc_to_unc(x, ma.lo[k], ma.hi[k]) : x;
            const double zn = zo + dz[k];
            const double xn = bounded ? wsmc_from_unc(zn, ma.lo[k], ma.hi[k]) : zn;
            if (bounded)
                lpr = lpr + (wsmc_log_abs_jac(zn, ma.lo[k], ma.hi[k]) - wsmc_log_abs_jac(zo, ma.lo[k], ma.hi[k]));
            ov.col[k] = ma.tcol[k];
            ov.val[k] = xn;
        }
        const double s_old = wsmc_fold(tape, nterms, depth, cols, N, i, nullptr);
        const double s_new = wsmc_fold(tape, nterms, depth, cols, N, i, &ov);
        const double u = wsmc_uniform_k(seed, op_acc, (uint64_t)(goff + i), 0);
        if (wsmc_log(u) < (lpr + s_new) - s_old) {
            for (int k = 0; k < d; ++k) cols[ma.tcol[k]][i] = ov.val[k];
            acc = 1;
        }
    }
    acc = block_sum_u64(acc, lds4);
    if (threadIdx.x == 0 && acc) atomicAdd(accepted, acc);
}

// marginal_diversity keys: isequal semantics (all NaN equal, -0.0 != 0.0)
__global__ __launch_bounds__(kBlock) void k_div_keys(const double* x, u64* keys, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    const double v = x[i];
    keys[i] = wsmc_isnan(v) ? 0x7ff8000000000000ull : wsmc_d2bits(v);
}
__global__ __launch_bounds__(kBlock) void k_count_unique(const u64* keys, int64_t N, u64* count) {
    __shared__ u64 lds4[4];
    u64 c = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock)
        c += (i == 0) || (keys[i] != keys[i - 1]);
    c = block_sum_u64(c, lds4);
    if (threadIdx.x == 0 && c) atomicAdd(count, c);
}

// ------------------------------------------------------------------------------------
// fused 2D SSM step (examples/2D_ssm.jl:10-16): gather-on-read through the previous
// step's ancestors, x{t+1} = x{t} + v, dv ~ MvNormal(0, q I), v = v + dv,
// weights += logpdf(MvNormal(x{t+1}, r I), o_t), block max -> record.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double aff2(double a, double b) {
    double v = 0.0;        // operand c0
    v = v + 1.0 * a;       // coef[0] * col[0]
    v = v + 1.0 * b;       // coef[1] * col[1]
    return v;
}

__global__ __launch_bounds__(kBlock) void k_ssm2d_prop(Ssm2dArgs a) {
    __shared__ u64 lds4[4];
    const int64_t N = a.N;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    u64 menc = 0;
    if (i < N) {
        const bool rs = a.t > 1 && a.dec_prev->resampled;
        const int64_t src = rs ? (int64_t)a.anc_prev[i] : i;
        double x0, x1, v0, v1;
        if (a.t == 1) {
            x0 = a.x0[0]; x1 = a.x0[1]; v0 = a.v0[0]; v1 = a.v0[1];
        } else {
            x0 = a.x_prev[src]; x1 = a.x_prev[N + src];
            v0 = a.v_prev[src]; v1 = a.v_prev[N + src];
        }
        // x{t+1} .= x{t} + v
        const double xn0 = aff2(x0, v0), xn1 = aff2(x1, v1);
        // dv ~ MvNormal([0,0], q*I)
        const uint64_t op_dv = a.op_dev[0] + 3ull * (uint64_t)(a.t - 1);
        double z0, z1;
        wsmc_normal_pair(wsmc_rng_block(a.seed, op_dv, (uint64_t)(a.goff + i), 0u), &z0, &z1);
        const double dv0 = 0.0 + a.q_sd * z0, dv1 = 0.0 + a.q_sd * z1;
        // v .= v + dv
        const double vn0 = aff2(v0, dv0), vn1 = aff2(v1, dv1);
        // o => MvNormal(x{t+1}, r*I)
        const double o0 = a.obs[2 * (a.t - 1)], o1 = a.obs[2 * (a.t - 1) + 1];
        const double m0 = 0.0 + 1.0 * xn0, m1 = 0.0 + 1.0 * xn1;
        double s = 0.0;
        const double d0 = o0 - m0, d1 = o1 - m1;
        s = s + d0 * d0;
        s = s + d1 * d1;
        const double lp = -(a.c0 + s / a.r_var) * 0.5;
        const double wb = rs ? a.dec_prev->mean : a.w[i];
        const double wn = wb + lp;
        a.x_next[i] = xn0; a.x_next[N + i] = xn1;
        a.v_next[i] = vn0; a.v_next[N + i] = vn1;
        a.dv[i] = dv0; a.dv[N + i] = dv1;
        a.w[i] = wn;
        menc = wsmc_ord_enc(wn);
    }
    menc = block_max_u64(menc, lds4);
    if (threadIdx.x == 0) atomic_max_filtered(&a.rec->v[blockIdx.x % kSlots][0], menc);
}

// trace the ancestor log back once and materialise the final columns — the result
// ColumnStore's per-resample gather of every column would have produced (src/stores.jl:105-128)
__global__ __launch_bounds__(kBlock) void k_ssm2d_final(Ssm2dFinal f) {
    const int64_t N = f.N;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    const int T = f.T;
    int64_t a = i;
    if (f.dec[T].resampled) a = f.anc_log[(int64_t)(T - 1) * N + i];
    f.v_out[i] = f.v_work[a]; f.v_out[N + i] = f.v_work[N + a];
    f.dv_out[i] = f.dv_work[a]; f.dv_out[N + i] = f.dv_work[N + a];
    if (f.dec[T].resampled) f.w[i] = f.dec[T].mean;
    if (!f.keep_history) {
        f.x_out[i] = f.x_work[a]; f.x_out[N + i] = f.x_work[N + a];
        return;
    }
    // x_{T+1} was written at step T
    {
        const double* src = f.hist_work[T + 1];
        double* dst = f.hist_out[T + 1];
        dst[i] = src[a]; dst[N + i] = src[N + a];
    }
    for (int s = T - 1; s >= 1; --s) {
        if (f.dec[s].resampled) a = f.anc_log[(int64_t)(s - 1) * N + a];
        const double* src = f.hist_work[s + 1];
        double* dst = f.hist_out[s + 1];
        dst[i] = src[a]; dst[N + i] = src[N + a];
    }
    double* d1 = f.hist_out[1];
    d1[i] = f.x0[0]; d1[N + i] = f.x0[1];
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static inline dim3 grid_for(int64_t N) { return dim3((unsigned)((N + kBlock - 1) / kBlock)); }
static inline dim3 tiles_for(int64_t N) { return dim3((unsigned)((N + kTile - 1) / kTile)); }
static inline dim3 rs_tiles_for(int64_t N) { return dim3((unsigned)((N + kRsTile - 1) / kRsTile)); }

hipError_t launch_assign(hipStream_t s, double* out, int dim, const wsmc_operand* expr,
                         double* const* cols, int64_t N) {
    AssignArgs a;
    for (int k = 0; k < 4; ++k) a.e[k] = expr[k < dim ? k : 0];
    hipLaunchKernelGGL(k_assign, grid_for(N), dim3(kBlock), 0, s, out, dim, a, cols, N);
    return hipGetLastError();
}
hipError_t launch_sample(hipStream_t s, double* out, int dim, const wsmc_dist& d, uint64_t seed, uint64_t op,
                         int64_t goff, double* const* cols, int64_t N) {
    hipLaunchKernelGGL(k_sample, grid_for(N), dim3(kBlock), 0, s, out, dim, d, seed, op, goff, cols, N);
    return hipGetLastError();
}
hipError_t launch_sample_importance(hipStream_t s, double* out, int dim, const wsmc_dist& prop,
                                    const wsmc_dist& targ, double* w, uint64_t seed, uint64_t op,
                                    int64_t goff, double* const* cols, int64_t N) {
    hipLaunchKernelGGL(k_sample_importance, grid_for(N), dim3(kBlock), 0, s, out, dim, prop, targ, w, seed,
                       op, goff, cols, N);
    return hipGetLastError();
}
hipError_t launch_weigh(hipStream_t s, const wsmc_term& t, double* w, double* const* cols, int64_t N) {
    hipLaunchKernelGGL(k_weigh, grid_for(N), dim3(kBlock), 0, s, t, w, cols, N);
    return hipGetLastError();
}
hipError_t launch_rs_max(hipStream_t s, const double* w, int64_t N, ShardRec* rec) {
    int64_t nb = (N + kBlock * 4 - 1) / (kBlock * 4);
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_rs_max, dim3((unsigned)nb), dim3(kBlock), 0, s, w, N, rec);
    return hipGetLastError();
}
hipError_t launch_rs_sums(hipStream_t s, const double* w, int64_t N, ShardRec* rec, u64* tileQ, u64* qbuf) {
    hipLaunchKernelGGL(k_rs_sums, rs_tiles_for(N), dim3(kBlock), 0, s, w, N, rec, tileQ, qbuf);
    return hipGetLastError();
}
hipError_t launch_rs_scan(hipStream_t s, const double* w, int64_t N, const ShardRec* recs, int world, int rank,
                          double ess_min, int scheme, uint64_t seed, uint64_t op, const uint64_t* op_dev,
                          int64_t slot_base, const u64* tileQ, const u64* qbuf, int32_t* anc, Decision* dec) {
    hipLaunchKernelGGL(k_rs_scan, rs_tiles_for(N), dim3(kBlock), 0, s, w, N, recs, world, rank, ess_min, scheme,
                       seed, op, op_dev, slot_base, tileQ, qbuf, anc, dec);
    return hipGetLastError();
}
hipError_t launch_gather(hipStream_t s, double* dst, const double* src, const int32_t* anc, int64_t N) {
    hipLaunchKernelGGL(k_gather, grid_for(N), dim3(kBlock), 0, s, dst, src, anc, N);
    return hipGetLastError();
}
hipError_t launch_fill_weights(hipStream_t s, double* w, const Decision* dec, int64_t N) {
    hipLaunchKernelGGL(k_fill_weights, grid_for(N), dim3(kBlock), 0, s, w, dec, N);
    return hipGetLastError();
}
hipError_t launch_log_evidence_stats(hipStream_t s, const double* w, int64_t N, ShardRec* rec, u64* tileQ,
                                     u64* qbuf) {
    hipError_t e = launch_rs_max(s, w, N, rec);
    if (e != hipSuccess) return e;
    return launch_rs_sums(s, w, N, rec, tileQ, qbuf);
}
hipError_t launch_score(hipStream_t s, const wsmc_term* tape, int32_t n, int32_t depth, double* const* cols,
                        int64_t N, double* out) {
    hipLaunchKernelGGL(k_score, grid_for(N), dim3(kBlock), 0, s, tape, n, depth, cols, N, out);
    return hipGetLastError();
}
hipError_t launch_moments(hipStream_t s, const double* w, const ShardRec* rec, double* const* cols,
                          const int32_t* tcols, int d, const double* lo, const double* hi, int pass,
                          const double* mom, int64_t N, double* tilepart) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
    }
    const int64_t nt = (N + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_moments, tiles_for(N), dim3(kBlock), 0, s, w, rec, cols, ma, d, pass, mom, N, nt,
                       tilepart);
    return hipGetLastError();
}
hipError_t launch_moments_final(hipStream_t s, const double* tilepart, int64_t ntiles, int d, int pass,
                                double min_step, double* mom, int32_t* flag) {
    hipLaunchKernelGGL(k_moments_final, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, d, pass, min_step, mom,
                       flag);
    return hipGetLastError();
}
hipError_t launch_move(hipStream_t s, const wsmc_term* tape, int32_t nterms, int32_t depth, double* const* cols,
                       const int32_t* tcols, int d, const double* lo, const double* hi, int bounded,
                       const double* L, uint64_t seed, uint64_t op_prop, uint64_t op_acc, int64_t goff,
                       int64_t N, u64* accepted) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
    }
    hipLaunchKernelGGL(k_move, grid_for(N), dim3(kBlock), 0, s, tape, nterms, depth, cols, ma, d, bounded, L,
                       seed, op_prop, op_acc, goff, N, accepted);
    return hipGetLastError();
}
hipError_t launch_diversity_keys(hipStream_t s, const double* x, u64* keys, int64_t N) {
    hipLaunchKernelGGL(k_div_keys, grid_for(N), dim3(kBlock), 0, s, x, keys, N);
    return hipGetLastError();
}
hipError_t launch_count_unique(hipStream_t s, const u64* keys, int64_t N, u64* count) {
    int64_t nb = (N + kBlock * 4 - 1) / (kBlock * 4);
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_count_unique, dim3((unsigned)nb), dim3(kBlock), 0, s, keys, N, count);
    return hipGetLastError();
}
hipError_t launch_ssm2d_propagate(hipStream_t s, const Ssm2dArgs& a) {
    hipLaunchKernelGGL(k_ssm2d_prop, grid_for(a.N), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}
// bounded spin on the 100 MHz constant clock (always exits): queue-filling delay for
// instrumented runs
__global__ void k_delay(int microseconds) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long ticks = (unsigned long long)microseconds * 100ull;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
hipError_t launch_delay(hipStream_t s, int microseconds) {
    if (microseconds > 100000) microseconds = 100000;
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, microseconds);
    return hipGetLastError();
}

hipError_t launch_ssm2d_finalize(hipStream_t s, const Ssm2dFinal& f) {
    hipLaunchKernelGGL(k_ssm2d_final, grid_for(f.N), dim3(kBlock), 0, s, f);
    return hipGetLastError();
}

}  // namespace wsmc
