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
#include <hip/hip_ext.h>

#include <cstdlib>
#include "wsmc_internal.h"

namespace wsmc {

typedef double d2 __attribute__((ext_vector_type(2)));

typedef unsigned long long u64;

// ------------------------------------------------------------------------------------
// wave / block primitives (wave64)
// Cross-lane moves are DPP (a VALU operand modifier) rather than ds_bpermute (an LDS
// round trip per step): quad_perm 1,0,3,2 / 2,3,0,1, row_ror 4 / 8 reduce within each row
// of 16 lanes, row_bcast 15 / 31 carry the rows up to lane 63. Lanes without a source read
// the identity (update_dpp's `old`).
// ------------------------------------------------------------------------------------
enum : int {
    kDppQuad1032 = 0xb1, kDppQuad2301 = 0x4e, kDppRowRor4 = 0x124, kDppRowRor8 = 0x128,
    kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr3 = 0x113, kDppRowShr4 = 0x114,
    kDppRowShr8 = 0x118, kDppBcast15 = 0x142, kDppBcast31 = 0x143, kDppWaveShr1 = 0x138
};
// lanes with no source read 0 (the identity of every use: sums, unsigned max). With full row
// and bank masks that is bound_ctrl, and no `old` value has to be materialised first.
template <int CTRL, int ROW = 0xf, int BANK = 0xf>
__device__ __forceinline__ u64 dpp_u64(u64 v) {
    constexpr bool full = ROW == 0xf && BANK == 0xf;
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW, BANK, full);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW, BANK, full);
    return ((u64)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {   // identity 0.0 (bits 0)
    return __builtin_bit_cast(double, dpp_u64<CTRL>(__builtin_bit_cast(u64, v)));
}
__device__ __forceinline__ u64 lane63_u64(u64 v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((u64)hi << 32) | lo;
}
// wave totals (every lane gets the result)
__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
    v += dpp_u64<kDppQuad1032>(v);
    v += dpp_u64<kDppQuad2301>(v);
    v += dpp_u64<kDppRowRor4>(v);
    v += dpp_u64<kDppRowRor8>(v);
    v += dpp_u64<kDppBcast15>(v);
    v += dpp_u64<kDppBcast31>(v);
    return lane63_u64(v);
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
    u64 o;
    o = dpp_u64<kDppQuad1032>(v); v = o > v ? o : v;
    o = dpp_u64<kDppQuad2301>(v); v = o > v ? o : v;
    o = dpp_u64<kDppRowRor4>(v); v = o > v ? o : v;
    o = dpp_u64<kDppRowRor8>(v); v = o > v ? o : v;
    o = dpp_u64<kDppBcast15>(v); v = o > v ? o : v;
    o = dpp_u64<kDppBcast31>(v); v = o > v ? o : v;
    return lane63_u64(v);
}
// wave total of f64 values that are exact integers whose sum stays below 2^53 (any order
// gives the same bits); NOT for canonical floating sums (block_sum_canon)
__device__ __forceinline__ double wave_sum_f64_exact(double v) {
    v = v + dpp_f64<kDppQuad1032>(v);
    v = v + dpp_f64<kDppQuad2301>(v);
    v = v + dpp_f64<kDppRowRor4>(v);
    v = v + dpp_f64<kDppRowRor8>(v);
    v = v + dpp_f64<kDppBcast15>(v);
    v = v + dpp_f64<kDppBcast31>(v);
    return __builtin_bit_cast(double, lane63_u64(__builtin_bit_cast(u64, v)));
}
// inclusive prefix sum over the wave (lane order)
__device__ __forceinline__ u64 wave_incl_scan_u64(u64 v) {
    u64 x = v + dpp_u64<kDppRowShr1>(v);
    x += dpp_u64<kDppRowShr2>(v);
    x += dpp_u64<kDppRowShr3>(v);
    x += dpp_u64<kDppRowShr4, 0xf, 0xe>(x);
    x += dpp_u64<kDppRowShr8, 0xf, 0xc>(x);
    x += dpp_u64<kDppBcast15, 0xa, 0xf>(x);
    x += dpp_u64<kDppBcast31, 0xc, 0xf>(x);
    return x;
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
// block_sum_canon_n (NV values at once): csrc/wsmc_mv_body.h, shared with the compiled Move blocks
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
// exclusive prefix sum over a block of NW waves (thread order), also returns the total
template <int NW = 4>
__device__ __forceinline__ u64 block_excl_scan_u64(u64 v, u64* ldsw, u64* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u64 x = wave_incl_scan_u64(v);
    if (lane == 63) ldsw[w] = x;
    __syncthreads();
    u64 pre = 0, t = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const u64 s = ldsw[k];
        pre += k < w ? s : 0ull;
        t += s;
    }
    *total = t;
    __syncthreads();
    return pre + x - v;
}
// exclusive prefix max over a block of NW waves (int, -1 = empty)
template <int NW = 4>
__device__ __forceinline__ int block_excl_max_i32(int v, int* ldsw, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int y = __shfl_up(x, off, 64);
        if (lane >= off) x = y > x ? y : x;
    }
    int ex = __shfl_up(x, 1, 64);
    if (lane == 0) ex = -1;
    if (lane == 63) ldsw[w] = x;
    __syncthreads();
    int pre = -1, t = -1;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const int s = ldsw[k];
        if (k < w) pre = s > pre ? s : pre;
        t = s > t ? s : t;
    }
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
// the expressions and their operand columns resolved by the host to component pointers
// (p[k][m] = column col[m] of expression k at its component), so the kernel reads no table
struct AssignArgs {
    wsmc_operand e[4];
    const double* p[4][2];
};

// Assign (src/transformers.jl:28-32). Gather-on-read (lazy genealogy): operand column slot
// s = 2k + m (expression k, column m) with bit s of ind.mask reads its column one log entry
// behind, through that entry's ancestors — ColumnStore's gather fused into the read. The
// arithmetic is wsmc_operand_eval's, term for term. ind.tab_col >= 0: `out` is written to a
// fresh buffer whose address goes into the device pointer table (the host swaps front/back).
__global__ __launch_bounds__(kBlock) void k_assign(double* out, int dim, AssignArgs a,
                                                   double* const* cols, int64_t N, Indirect ind) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    if (i == 0 && ind.tab_col >= 0) ind.tab[ind.tab_col] = out;
    const int64_t j = (ind.mask && (!ind.dec || ind.dec->resampled)) ? (int64_t)ind.row[i] : i;
    double x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= dim) continue;
        const wsmc_operand& o = a.e[k];
        double v = o.c0;
        if (o.col[0] >= 0) v = v + o.coef[0] * a.p[k][0][(ind.mask >> (2 * k)) & 1 ? j : i];
        if (o.col[1] >= 0) v = v + o.coef[1] * a.p[k][1][(ind.mask >> (2 * k + 1)) & 1 ? j : i];
        x[k] = v;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
}

// Assign of a general expression (wsmc_assign_expr; the fused broadcast of src/rewrites.jl:146-219
// into src/transformers.jl:28-32). The program (XProg, the only argument) is read in place through
// the kernarg segment pointer: every lane runs the same instruction, so the loads are scalar and
// the branches uniform, and the stack index is uniform too (the stack stays in registers, indexed
// through M0). Each operator is wsmc_xop1 / wsmc_xop2, as in the oracle's wsmc_xeval; a COL read
// with `lag` goes through the newest log entry's ancestors (k_assign's gather-on-read).
__global__ __launch_bounds__(kBlock) void k_assign_expr(XProg) {
    const XProg* X = (const XProg*)(const char*)__builtin_amdgcn_kernarg_segment_ptr();
    const int64_t N = X->N;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    if (i == 0 && X->tab_col >= 0) X->tab[X->tab_col] = X->out;
    const int64_t j = (X->any_lag && (!X->dec || X->dec->resampled)) ? (int64_t)X->row[i] : i;
    int pc = 0;
    double res[4];   // every component before any store: a component may read another of `out`
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= X->dim) break;
        double st[WSMC_XSTACK_MAX];
        int sp = 0;
        for (const int e = pc + X->len[k]; pc < e; ++pc) {
            const XIns& I = X->ins[pc];
            const int op = I.op;
            if (op == WSMC_X_CONST) {
                st[sp++] = I.c;
            } else if (op == WSMC_X_COL) {
                st[sp++] = I.p[I.lag ? j : i];
            } else if (op == WSMC_X_IFELSE) {
                const double f = st[sp - 1], t = st[sp - 2];
                sp -= 2;
                st[sp - 1] = st[sp - 1] != 0.0 ? t : f;
            } else if (op < WSMC_X_ADD) {
                st[sp - 1] = wsmc_xop1(op, st[sp - 1], I.c);
            } else {
                const double b = st[--sp];
                st[sp - 1] = wsmc_xop2(op, st[sp - 1], b);
            }
        }
        res[k] = st[0];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < X->dim) X->out[(int64_t)k * N + i] = res[k];
}

// FEAT (wsmc_terms.h): WSMC_FEAT_ALL, WSMC_FEAT_OSC, or 0 for affine means (no oscillator or
// full-covariance code: registers)
template <unsigned FEAT>
__global__ __launch_bounds__(kBlock) void k_sample(double* out, int dim, wsmc_dist d, uint64_t seed,
                                                   uint64_t op, int64_t goff, double* const* cols,
                                                   int64_t N, int has_sd, double sd) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    double x[4];
    // has_sd: a constant MvNormal variance, its sqrt evaluated once by the host (the same
    // restated function of the same bits each particle would evaluate)
    const double sdl = sd;   // a local (the parameter's address would live in scratch)
    wsmc_dist_sample_mf(&d, x, seed, op, (uint64_t)(goff + i), cols, N, i, has_sd ? &sdl : nullptr, FEAT);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
}

template <unsigned FEAT>
__global__ __launch_bounds__(kBlock) void k_sample_importance(double* out, int dim, wsmc_dist prop,
                                                              wsmc_dist targ, double* w, uint64_t seed,
                                                              uint64_t op, int64_t goff,
                                                              double* const* cols, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    wsmc_dist_sample_mf(&prop, x, seed, op, (uint64_t)(goff + i), cols, N, i, nullptr, FEAT);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < dim) out[(int64_t)k * N + i] = x[k];
    double lt = wsmc_dist_logpdf_mf(&targ, x, cols, N, i, nullptr, nullptr, FEAT);
    double lp = wsmc_dist_logpdf_mf(&prop, x, cols, N, i, nullptr, nullptr, FEAT);
    w[i] = w[i] + (lt - lp);
}

// Observe / Weight: weights += logpdf, and the block max of the new weights into the 64
// slots of `ms` (zero on entry), so the Resample that follows needs no max pass; block 0
// zeroes `ms_next`, the slots the next launch will use (k_rs_max's encoding and slots)
// wreset != null: a Resample's weight reset still pending (the fused generic Resample defers
// it to its first reader): a particle's weight is wreset->mean when that step resampled
template <unsigned FEAT>
__global__ __launch_bounds__(kBlock) void k_weigh(wsmc_term t, double* w, double* const* cols, int64_t N,
                                                  MaxSlots* ms, MaxSlots* ms_next, wsmc_logmemo lm0,
                                                  const Decision* wreset) {
    __shared__ u64 lds[4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    u64 m = 0;
    if (i < N) {
        // lm0: a constant scale operand's log, evaluated once by the host and handed to the
        // term through the fold's log memo (the same bits every particle would compute)
        wsmc_logmemo lm = lm0;
        const double w0 = (wreset && wreset->resampled) ? wreset->mean : w[i];
        const double v = w0 + wsmc_term_logpdf_mf(&t, cols, N, i, nullptr, &lm, FEAT);
        w[i] = v;
        m = wsmc_ord_enc(v);
    }
    m = block_max_u64(m, lds);
    if (threadIdx.x == 0) atomic_max_filtered(&ms->v[blockIdx.x % kSlots][0], m);
    if (blockIdx.x == 0)
        for (int k = threadIdx.x; k < kSlots * 16; k += kBlock) ms_next->v[k >> 4][k & 15] = 0ull;
}

// A batch of elementwise statements (EwBatch, the first argument: read in place through the
// kernarg segment pointer): per particle, each statement in order with k_assign's, k_sample's
// and k_weigh's arithmetic — one launch for a model step's Assign / Sample / Observe run.
// Values a later statement reads are kept in LDS rows (one per column component, a value per
// thread): a statement's output is written to its global column and, when staged, to its rows;
// the Sample / weight terms evaluate against a pointer table of rows (stride kBlock, index =
// the thread), the columns no earlier statement wrote loaded into rows at the start — so no
// statement re-reads from memory what an earlier one just stored. The weights stay in a
// register across the weight terms (the first applies a pending reset); the block max of the
// final weights goes to the batch's slots.
template <unsigned FEAT>
__global__ __launch_bounds__(kBlock) void k_ew_batch(EwBatch, uint64_t seed, int64_t goff, int64_t N) {
    const EwBatch* B = (const EwBatch*)(const char*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ u64 lds[4];
    extern __shared__ double rows[];   // [B->nrows][kBlock], sized by the launch
    __shared__ double* ctab[kEwSlots];
    const int th = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * kBlock + th;
    const bool in = i < N;
    if (i == 0)
        for (int t = 0; t < B->ntab; ++t) B->tab[B->tab_col[t]] = B->tab_out[t];
    if (th < B->nslots) ctab[th] = rows + (int)B->slot_row[th] * kBlock;
    // every load that depends on no statement, up front: the preloaded rows, the ancestor, the
    // weight
    const int64_t j = (in && B->anc && (!B->dec || B->dec->resampled)) ? (int64_t)B->anc[i] : i;
    // unrolled over the capacity: the loads issue back to back (a rolled loop stored each
    // value to LDS before issuing the next load, one memory latency per column)
    const int npre = B->npre;
    double pv[kEwPre];
#pragma unroll
    for (int p = 0; p < kEwPre; ++p) pv[p] = (p < npre && in) ? B->pre_src[p][B->pre_lag[p] ? j : i] : 0.0;
#pragma unroll
    for (int p = 0; p < kEwPre; ++p)
        if (p < npre) rows[(int)B->pre_row[p] * kBlock + th] = pv[p];
    double wv = 0.0;
    if (in && B->has_w) wv = (B->wreset && B->wreset->resampled) ? B->wreset->mean : B->w[i];
    __syncthreads();
    double* const* cols = ctab;
    u64 m = 0;
    if (in) {
        for (int k = 0; k < B->nops; ++k) {
            const EwOp& op = B->ops[k];
            const int dim = op.dim;
            double x[4] = {0.0, 0.0, 0.0, 0.0};
            if (op.kind == 0) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q >= dim) continue;
                    const wsmc_operand& o = op.a.e[q];
                    double v = o.c0;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (o.col[c] < 0) continue;
                        const int f = op.a.fwd[q][c];
                        const double xv = f >= 0 ? rows[f * kBlock + th]
                                                 : op.a.p[q][c][(op.a.lag >> (2 * q + c)) & 1 ? j : i];
                        v = v + o.coef[c] * xv;
                    }
                    x[q] = v;
                }
            } else if (op.kind == 1) {
                const double sdl = op.s.sd;   // (a pointer chosen by a select would live in scratch)
                if (op.s.has_sd)
                    wsmc_dist_sample_mf(&op.s.d, x, seed, op.s.op, (uint64_t)(goff + i), cols, kBlock, th, &sdl, FEAT);
                else
                    wsmc_dist_sample_mf(&op.s.d, x, seed, op.s.op, (uint64_t)(goff + i), cols, kBlock, th, nullptr,
                                        FEAT);
            } else {
                wsmc_logmemo lm = op.w.lm0;
                wv = wv + wsmc_term_logpdf_mf(&op.w.t, cols, kBlock, th, nullptr, &lm, FEAT);
                continue;
            }
            if (!op.nostore)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < dim) op.out[(int64_t)q * N + i] = x[q];
            if (op.out_row >= 0)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < dim) rows[(op.out_row + q) * kBlock + th] = x[q];
        }
        if (B->has_w) {
            B->w[i] = wv;
            m = wsmc_ord_enc(wv);
        }
    }
    if (!B->has_w) return;
    m = block_max_u64(m, lds);
    if (threadIdx.x == 0) atomic_max_filtered(&B->ms->v[blockIdx.x % kSlots][0], m);
    if (blockIdx.x == 0)
        for (int k = threadIdx.x; k < kSlots * 16; k += kBlock) B->ms_next->v[k >> 4][k & 15] = 0ull;
}

// ------------------------------------------------------------------------------------
// Resample (src/transformers.jl:474-498) as four passes per invocation:
//   max      block max of the log-weights -> 64 slots (read-filtered atomicMax)
//   sums     per 1024-particle tile: q_i = floor(exp(lw_i - M) 2^K) (stored), and the exact
//            integer partials sum q, sum q^2, sum floor(exp(lw_i - M) 2^96) (plain stores)
//   reduce   one block: shard totals (ShardRecord), exclusive tile offsets, and — on one
//            GPU — the ESS decision and post-resample log-mean
//   scan     per tile: inclusive integer CDF from the offsets and the stratified /
//            systematic ancestor fill (the icdf merge, src/resampling.jl:13-26)
// Every decision-relevant quantity is an integer, so results do not depend on the order
// of any reduction, the grid shape or the shard count.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_rs_max(const double* __restrict__ w, int64_t N, MaxSlots* ms) {
    __shared__ u64 lds[4];
    u64 m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock)
        m = max(m, (u64)wsmc_ord_enc(w[i]));
    m = block_max_u64(m, lds);
    if (threadIdx.x == 0) atomic_max_filtered(&ms->v[blockIdx.x % kSlots][0], m);
}

static_assert(kSlots == 64, "one lane per max slot");
// max over the 64 slots by one wave (every lane of the calling wave gets it); no barrier
__device__ __forceinline__ double wave_slots_max(const MaxSlots* ms) {
    return wsmc_ord_dec(wave_max_u64(ms->v[threadIdx.x & 63][0]));
}
// the same over nms consecutive slot sets (exact shards: every rank's, all-gathered)
__device__ __forceinline__ double wave_slots_max_n(const MaxSlots* ms, int nms) {
    u64 m = 0;
    for (int g = 0; g < nms; ++g) {
        const u64 v = ms[g].v[threadIdx.x & 63][0];
        m = v > m ? v : m;
    }
    return wsmc_ord_dec(wave_max_u64(m));
}
// exact integer block sums of P values through LDS (transpose, two levels)
template <int NT, int P>
__device__ __forceinline__ void block_sum_parts(const u64 (&acc)[P], u64 (*red)[NT], u64 (*red2)[16],
                                                u64* out /* P, valid in threads < P */) {
    const int th = threadIdx.x;
#pragma unroll
    for (int k = 0; k < P; ++k) red[k][th] = acc[k];
    __syncthreads();
    if (th < P * 16) {
        const int k = th >> 4, seg = th & 15;
        u64 t = 0;
#pragma unroll 8
        for (int j = 0; j < NT / 16; ++j) t += red[k][j * 16 + seg];
        red2[k][seg] = t;
    }
    __syncthreads();
    if (th < P) {
        u64 t = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += red2[th][j];
        out[th] = t;
    }
}

// The per-particle Resample statistics: QAcc, qacc_add (csrc/wsmc_ew.h).
// a block's QAcc -> the tile partials (sum q, sum q2, sum wf2, sum wf) in threads < kPart;
// s_f [4][nw] LDS; returns the tile's sum q in thread 0 (0 elsewhere)
template <int NB>
__device__ __forceinline__ u64 qacc_tile(QAcc a, double (*s_f)[NB / 64], u64* out) {
    const int th = threadIdx.x;
    a.Q = wave_sum_f64_exact(a.Q);
    a.Q2 = wave_sum_f64_exact(a.Q2);
    a.WF2 = wave_sum_f64_exact(a.WF2);
    a.WF = wave_sum_f64_exact(a.WF);
    const int wv = th >> 6;
    if ((th & 63) == 0) {
        s_f[0][wv] = a.Q; s_f[1][wv] = a.Q2;
        s_f[2][wv] = a.WF2; s_f[3][wv] = a.WF;
    }
    __syncthreads();
    u64 t = 0;
    if (th < kPart) {
        double f = 0.0;
#pragma unroll
        for (int v = 0; v < NB / 64; ++v) f = f + s_f[th][v];
        t = (u64)f;                                         // exact integer <= 2^53
        out[th] = t;
    }
    return t;   // thread k < kPart: part k (thread 0: the tile's sum q), 0 elsewhere
}

// Weight statistics of one 1024-particle tile (256 threads x 4 particles, coalesced):
// q (stored for the fill) and the tile partials of qacc_tile.
// MODE (diagnostics only; production = 0): 1 = no exp, 4 = load/store only.
template <int MODE, bool MULTI = false>
__global__ __launch_bounds__(kSumBlock) void k_rs_sums_t(const double* __restrict__ w, int64_t N,
                                                         const MaxSlots* __restrict__ ms, u64* __restrict__ tilep,
                                                         u64* __restrict__ qbuf, u64* __restrict__ grp, int G,
                                                         int64_t Nk, int nms, int gall) {
    constexpr int IT = kRsTile / kSumBlock;
    __shared__ double s_f[kPart][kSumBlock / 64];
    const int th = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kRsTile;
    u64 mv = MODE == 4 ? 0ull : ms[0].v[th & 63][0];
    double lw[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = base + (int64_t)k * kSumBlock + th;
        lw[k] = i < N ? w[i] : -WSMC_INF;
    }
    if (MULTI)   // exact shards: every rank's slots (a separate instance: the loop's loads would
                 // make the single-rank path wait for the weights' loads too)
        for (int g = 1; g < nms; ++g) {
            const u64 v = ms[g].v[th & 63][0];
            mv = v > mv ? v : mv;
        }
    const double M = MODE == 4 ? 0.0 : wsmc_qref(wsmc_ord_dec(wave_max_u64(mv)));   // the reference point
    const double sK = wsmc_pow2i(wsmc_qbits((uint64_t)Nk));   // Nk: the global N when exact-sharded
    QAcc acc;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = base + (int64_t)k * kSumBlock + th;
        if (MODE == 4) {
            if (i < N) qbuf[i] = (u64)wsmc_d2bits(lw[k]);
            continue;
        }
        const double e = MODE == 1 ? (lw[k] > M - 1.0 ? 1.0 : 0.5) : wsmc_expw(lw[k] - M);
        const u64 q = qacc_add(acc, e, sK);
        if (i < N) qbuf[i] = q;
    }
    if (MODE == 4) return;
    const u64 t = qacc_tile<kSumBlock>(acc, s_f, tilep + (int64_t)blockIdx.x * kPart);
    // group sums of q (fused runs; integer atomics, so order-free): the fill's CDF
    // offsets and the shard record's Q
    // word 1: the group's largest tile sum (the fill's overflow blocks exit early when no
    // tile can own more than one chunk of slots)
    if (grp && th == 0) {
        u64* gl = grp + (int64_t)(blockIdx.x / G) * kGroupLine;
        atomicAdd(gl, t);
        atomicMax(gl + 1, t);
    }
    // exact shards: the group lines carry every part (they are all-gathered in place of the
    // record): word 2 sum q2, 3 sum wf2, 4 sum wf (integer atomics, order-free); word 7 of
    // line 0 the shard size
    if (gall && th >= 1 && th < kPart) atomicAdd(grp + (int64_t)(blockIdx.x / G) * kGroupLine + 1 + th, t);
    if (gall && blockIdx.x == 0 && th == kPart) atomicAdd(grp + 7, (u64)N);
}

// The fused run's statistics check (round 6): the propagate took every q against its guess R_g
// (k_ssm2d_prop QS); they are the canonical ones iff R_g == wsmc_qref(M) (numerically: -0.0 and
// +0.0 give the same expw). Then every block returns at once. Otherwise (M and the bound straddle
// an integer, the first step, a NaN) the blocks recompute, grid-stride, each tile's q (when the
// fill reads it from qbuf), its partials, and correct the group lines by the difference of the
// tile's sum (u64 wrap-around arithmetic: exact) and a max with the new one (the overflow plan's
// gate only needs an upper bound). nfix counts the steps that took this path.
__global__ __launch_bounds__(kSumBlock) void k_rs_qfix(const double* __restrict__ w, int64_t N,
                                                     const MaxSlots* __restrict__ ms, const double* __restrict__ rg,
                                                     u64* __restrict__ tilep, u64* __restrict__ qbuf,
                                                     u64* __restrict__ grp, int G, u64* nfix) {
    constexpr int IT = kRsTile / kSumBlock;
    __shared__ double s_f[kPart][kSumBlock / 64];
    const double R = wsmc_qref(wave_slots_max(ms));
    if (R == *rg) return;                                   // uniform: the guess was the reference point
    if (nfix && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(nfix, 1ull);
    const int th = threadIdx.x;
    const int ntiles = (int)((N + kRsTile - 1) / kRsTile);
    const double sK = wsmc_pow2i(wsmc_qbits((uint64_t)N));
    for (int b = blockIdx.x; b < ntiles; b += gridDim.x) {
        const int64_t base = (int64_t)b * kRsTile;
        const u64 old = th == 0 ? tilep[(int64_t)b * kPart] : 0ull;
        QAcc acc;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int64_t i = base + (int64_t)k * kSumBlock + th;
            const double lw = i < N ? w[i] : -WSMC_INF;
            const u64 q = qacc_add(acc, wsmc_expw(lw - R), sK);
            if (qbuf && i < N) qbuf[i] = q;
        }
        const u64 t = qacc_tile<kSumBlock>(acc, s_f, tilep + (int64_t)b * kPart);
        if (th == 0) {
            u64* gl = grp + (int64_t)(b / G) * kGroupLine;
            atomicAdd(gl, t - old);
            atomicMax(gl + 1, t);
        }
        __syncthreads();                                    // s_f is reused by the next tile
    }
}

__device__ __forceinline__ wsmc_shard_stats record_stats(const ShardRecord& r) {
    wsmc_shard_stats st;
    st.M = wsmc_ord_dec(r.menc);
    st.Q = r.Q;
    st.Q2 = r.q2;
    st.Wf2 = ((wsmc_u128)r.wf2hi << 64) | r.wf2lo;
    st.Wf = ((wsmc_u128)r.wfhi << 64) | r.wflo;
    st.n = r.n;
    return st;
}

// Global decision from the shard records (rank order): the same arithmetic as
// wsmc_global_ess / wsmc_shard_mean, streamed over the records (no local arrays).
__device__ void decide_records(const ShardRecord* recs, int world, int rank, double ess_min, Decision* dec) {
    double R = -WSMC_INF;
    uint64_t N = 0;
    int nan = 0, flat = world > 0;
    const double M0 = wsmc_ord_dec(recs[0].menc);
    for (int g = 0; g < world; ++g) {
        const wsmc_shard_stats st = record_stats(recs[g]);
        const double Rg = wsmc_qref(st.M);
        if (wsmc_isnan(Rg)) nan = 1;
        else if (Rg > R) R = Rg;
        N += recs[g].n;
        flat = flat && wsmc_shard_flat(&st) && st.M == M0;   // wsmc_all_flat
    }
    if (nan) R = WSMC_NAN;
    double s1 = 0.0, s2 = 0.0;
    for (int g = 0; g < world; ++g) {
        // the arithmetic of wsmc_global_ess, streamed over the records
        const wsmc_shard_stats st = record_stats(recs[g]);
        const double f = wsmc_exp(wsmc_qref(st.M) - R);
        s1 = s1 + wsmc_shard_expsum(&st) * f;
        s2 = s2 + wsmc_shard_expsum2(&st) * (f * f);
    }
    const double ess = flat ? 1.0 : (s1 * s1) / (wsmc_u64_to_d(N) * s2);
    const int rs = ess < ess_min;
    const wsmc_shard_stats me = record_stats(recs[rank]);
    dec->resampled = rs;
    dec->ess = ess;
    dec->M = me.M;
    dec->mean = rs ? wsmc_shard_mean(&me) : 0.0;
}

__device__ void decide_exact(const ShardRecord* recs, int world, int rank, double ess_min, const FillPlan& plan,
                             ShardRecord* comb, Decision* dec, ExactPlan* xp);
// one block: shard totals, tile offsets, the ancestor-fill task plan and (one GPU) the decision
// overflow chunks (past the first) a tile with integer weight sum qb may need
__device__ __forceinline__ int ovf_chunks(u64 qb, double ratio) {
    if (qb == 0) return 0;
    const double bound = wsmc_u64_to_d(qb) * ratio + 3.0;   // >= cnt_b + 1 (estimate error << 1)
    const int k = (int)(bound * (1.0 / kRsChunk));          // floor(bound / chunk)
    return k;                                               // ceil(bound / chunk) - 1 <= k
}

// MODE (diagnostics only; production = 0): 1 = no fill plan, 2 = no decision,
// 3 = partial sums + record only
template <int MODE>
__global__ __launch_bounds__(kRsBlock) void k_rs_reduce_t(const MaxSlots* __restrict__ ms,
                                                        const u64* __restrict__ tilep, int64_t ntiles, int64_t N,
                                                        u64* __restrict__ tileOff, ShardRecord* rec,
                                                        int decide_local, double ess_min, Decision* dec,
                                                        FillPlan plan, u64* __restrict__ esum, int nms) {
    __shared__ u64 red[kRedPart][kRsBlock];
    __shared__ u64 red2[kRedPart][16];
    __shared__ u64 tot[kRedPart];
    __shared__ u64 s_w[kRsBlock / 64];
    constexpr int kHeavyTasks = 4, kHeavyQueue = 256;
    __shared__ int s_heavy[kHeavyQueue][3];
    __shared__ int s_nheavy;
    const int th = threadIdx.x;
    // exact shards: the single-GPU decision and every rank's slot window first (the plan
    // below reads them)
    if (plan.dx_recs) {
        if (th == 0)
            decide_exact(plan.dx_recs, plan.dx_world, plan.dx_rank, plan.dx_ess, plan, plan.dx_comb, plan.dx_dec,
                         plan.dx_xp);
        __syncthreads();
    }
    // the max slots are read first so their latency overlaps the partials' loads
    u64 mslot = 0;
    for (int g = 0; g < nms; ++g) {
        const u64 v = th < kSlots ? ms[g].v[th][0] : 0ull;
        mslot = v > mslot ? v : mslot;
    }
    // thread th owns the contiguous tiles [b0, b1): loads each tile's partials once
    const int64_t per = (ntiles + kRsBlock - 1) / kRsBlock;
    const int64_t b0 = (int64_t)th * per < ntiles ? (int64_t)th * per : ntiles;
    const int64_t b1 = b0 + per < ntiles ? b0 + per : ntiles;
    u64 t4[kPart] = {0, 0, 0, 0};
    for (int64_t b = b0; b < b1; ++b)
#pragma unroll
        for (int k = 0; k < kPart; ++k) t4[k] += tilep[b * kPart + k];
    // Q and Q2 totals fit u64; Wf2 and Wf are summed as 32-bit limbs into u128
    const u64 acc[kRedPart] = {t4[0], t4[1], t4[2] & 0xffffffffull, t4[2] >> 32, t4[3] & 0xffffffffull,
                               t4[3] >> 32};
    block_sum_parts<kRsBlock, kRedPart>(acc, red, red2, tot);
    u64 total;
    u64 pre = block_excl_scan_u64<kRsBlock / 64>(acc[0], s_w, &total);
    // tile offsets; overflow fill tasks sized from the tile sums alone: a tile owns
    // cnt_b <= Q_b N / Q + 2 slots (stratified and systematic targets are one per 1/N
    // stratum), so ceil((Q_b N / Q + 3) / kRsChunk) - 1 chunks past the first always
    // suffice (a chunk found empty exits). Fill blocks rank their own tile's boundaries.
    const bool planned = MODE != 1 && MODE != 3 && plan.taskOff != nullptr;   // log-evidence: unplanned
    // targets are one per 1/N stratum of the CDF being filled: the global one when exact
    const double ratio = plan.xp ? wsmc_u64_to_d(plan.xp->N) / wsmc_u64_to_d(plan.xp->Q)
                                 : total ? wsmc_u64_to_d((uint64_t)N) / wsmc_u64_to_d(total) : 0.0;
    int nt = 0;
    {
        u64 c = pre;
        for (int64_t b = b0; b < b1; ++b) {
            tileOff[b] = c;
            const u64 qb = b1 - b0 == 1 ? t4[0] : tilep[b * kPart];
            c += qb;
            if (planned) nt += ovf_chunks(qb, ratio);
        }
    }
    // multinomial: exclusive offsets of the exponential-spacing tile sums, in place, and
    // their total in esum[ntiles]
    if (esum) {
        u64 es = 0;
        for (int64_t b = b0; b < b1; ++b) es += esum[b];
        u64 etot;
        u64 ec = block_excl_scan_u64<kRsBlock / 64>(es, s_w, &etot);
        for (int64_t b = b0; b < b1; ++b) {
            const u64 v = esum[b];
            esum[b] = ec;
            ec += v;
        }
        if (th == 0) esum[ntiles] = etot;
    }
    u64 tt = 0;
    if (planned) {
        // overflow task -> tile map; exclusive scan of the per-tile counts -> taskOff
        int tpre = (int)block_excl_scan_u64<kRsBlock / 64>((u64)nt, s_w, &tt);
        // a tile with many tasks (a dominant particle) is queued and its map entries are
        // written by the whole block, so one thread never loops over N / kRsChunk entries
        if (th == 0) s_nheavy = 0;
        __syncthreads();
        for (int64_t b = b0; b < b1; ++b) {
            const int k = ovf_chunks(b1 - b0 == 1 ? t4[0] : tilep[b * kPart], ratio);
            plan.taskOff[b] = tpre;
            int q = -1;
            if (k > kHeavyTasks) {
                q = atomicAdd(&s_nheavy, 1);
                if (q < kHeavyQueue) { s_heavy[q][0] = (int)b; s_heavy[q][1] = tpre; s_heavy[q][2] = k; }
            }
            if (q < 0 || q >= kHeavyQueue)
                for (int j = 0; j < k; ++j) plan.taskTile[tpre + j] = (int32_t)b;
            tpre += k;
        }
        __syncthreads();
        const int nh = s_nheavy < kHeavyQueue ? s_nheavy : kHeavyQueue;
        for (int e = 0; e < nh; ++e)
            for (int j = th; j < s_heavy[e][2]; j += kRsBlock) plan.taskTile[s_heavy[e][1] + j] = s_heavy[e][0];
    }
    if (th < 64) {
        const u64 menc = wave_max_u64(mslot);
        if (th == 0) {
            ShardRecord r;
            r.menc = menc;
            r.Q = tot[0];
            r.q2 = tot[1];
            const wsmc_u128 Wf2 = (wsmc_u128)tot[2] + ((wsmc_u128)tot[3] << 32);
            const wsmc_u128 Wf = (wsmc_u128)tot[4] + ((wsmc_u128)tot[5] << 32);
            r.wf2lo = (u64)Wf2; r.wf2hi = (u64)(Wf2 >> 64);
            r.wflo = (u64)Wf; r.wfhi = (u64)(Wf >> 64);
            r.n = (u64)N;
            *rec = r;
            if (dec) {
                dec->ntasks = (int32_t)tt;
                if (decide_local && MODE != 2 && MODE != 3) decide_records(&r, 1, 0, ess_min, dec);
            }
        }
    }
}

// multi-GPU: decision from the all-gathered records
__global__ void k_rs_decide(const ShardRecord* recs, int world, int rank, double ess_min, Decision* dec) {
    if (threadIdx.x == 0) decide_records(recs, world, rank, ess_min, dec);
}

// ---- exact sharding ----------------------------------------------------
__global__ void k_max_publish(const MaxSlots* ms, u64* word) {
    const u64 m = wave_max_u64(ms->v[threadIdx.x & 63][0]);
    if (threadIdx.x == 0) *word = m;
}
// the global max (ordered encodings: NaN dominates, as the device max does) into slot 0
__global__ void k_max_adopt(const u64* words, int world, MaxSlots* ms) {
    const int th = threadIdx.x;
    u64 m = 0;
    for (int g = 0; g < world; ++g) m = words[g] > m ? words[g] : m;
    ms->v[th & 63][0] = th == 0 ? m : 0ull;
}
// Sum the records as integers (every shard's q is relative to the global max with K from
// the global N, so the sums are exactly the single-GPU ones) and decide once, as one GPU
// does; then the global CDF offsets and every rank's window of global slots.
__device__ void decide_exact(const ShardRecord* recs, int world, int rank, double ess_min, const FillPlan& plan,
                             ShardRecord* comb, Decision* dec, ExactPlan* xp) {
    ShardRecord r = recs[0];
    wsmc_u128 Wf2 = 0, Wf = 0;
    u64 Q = 0, Q2 = 0, n = 0;
    u64 cb[kMaxShards + 1];
    for (int g = 0; g < world; ++g) {
        cb[g] = Q;
        xp->gofs[g] = n;
        Q += recs[g].Q;
        Q2 += recs[g].q2;
        Wf2 += ((wsmc_u128)recs[g].wf2hi << 64) | recs[g].wf2lo;
        Wf += ((wsmc_u128)recs[g].wfhi << 64) | recs[g].wflo;
        n += recs[g].n;
        r.menc = recs[g].menc > r.menc ? recs[g].menc : r.menc;
    }
    cb[world] = Q;
    xp->gofs[world] = n;
    r.Q = Q;
    r.q2 = Q2;
    r.wf2lo = (u64)Wf2; r.wf2hi = (u64)(Wf2 >> 64);
    r.wflo = (u64)Wf; r.wfhi = (u64)(Wf >> 64);
    r.n = n;
    *comb = r;
    decide_records(&r, 1, 0, ess_min, dec);
    const uint64_t opx = op_eff(plan.op, plan.op_dev);
    xp->Q = Q;
    xp->N = n;
    for (int g = 0; g <= world; ++g)
        xp->seg[g] = Q ? wsmc_rank(cb[g], Q, n, plan.scheme, plan.seed, opx, 0) : 0;
    xp->cbase = cb[rank];
    xp->a = xp->seg[rank];
    xp->b = xp->seg[rank + 1];
}
__global__ void k_rs_decide_exact(const ShardRecord* recs, int world, int rank, double ess_min, FillPlan plan,
                                  ShardRecord* comb, Decision* dec, ExactPlan* xp) {
    if (threadIdx.x == 0) decide_exact(recs, world, rank, ess_min, plan, comb, dec, xp);
}
// slot j of the window: its owner keeps its components (written straight into the back
// buffers if that is this rank, packed into the peer's send block otherwise)
__global__ __launch_bounds__(kBlock) void k_exact_pack(ExactRoute rt, const int32_t* __restrict__ anc_out,
                                                       const double* const* __restrict__ src,
                                                       double* const* __restrict__ dst, int32_t* __restrict__ anc_local,
                                                       u64* __restrict__ sendbuf) {
    const u64 cnt = rt.b - rt.a;
    const u64 j = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (j >= cnt) return;
    const u64 sl = rt.a + j;
    int r = 0;
    while (r + 1 < rt.world && sl >= rt.gofs[r + 1]) ++r;
    const int32_t m = anc_out[j];
    const u64 gid = rt.gofs[rt.rank] + (u64)m;      // the ancestor's global index
    if (r == rt.rank) {
        const u64 li = sl - rt.gofs[rt.rank];
        for (int c = 0; c < rt.ncomp; ++c) dst[c][li * rt.stride] = src[c][(u64)m * rt.stride];
        anc_local[li] = (int32_t)gid;
        return;
    }
    const u64 lo = rt.a > rt.gofs[r] ? rt.a : rt.gofs[r];
    const u64 hi = rt.b < rt.gofs[r + 1] ? rt.b : rt.gofs[r + 1];
    const u64 len = hi - lo, idx = sl - lo;
    u64* blk = sendbuf + rt.sendoff[r];
    for (int c = 0; c < rt.ncomp; ++c) blk[(u64)c * len + idx] = (u64)wsmc_d2bits(src[c][(u64)m * rt.stride]);
    blk[(u64)rt.ncomp * len + idx] = gid;
}
__global__ __launch_bounds__(kBlock) void k_exact_unpack(ExactRoute rt, const u64* __restrict__ recvbuf,
                                                         double* const* __restrict__ dst,
                                                         int32_t* __restrict__ anc_local) {
    const u64 j = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (j >= rt.recvpre[rt.world]) return;
    int g = 0;
    while (j >= rt.recvpre[g + 1]) ++g;
    const u64 idx = j - rt.recvpre[g], len = rt.recvlen[g];
    const u64* blk = recvbuf + rt.recvoff[g];
    const u64 li = rt.recvdst[g] + idx;
    for (int c = 0; c < rt.ncomp; ++c) dst[c][li * rt.stride] = wsmc_bits2d(blk[(u64)c * len + idx]);
    anc_local[li] = (int32_t)blk[(u64)rt.ncomp * len + idx];
}

// ---- exact shards without host round trips (ExactStep, wsmc_internal.h) -------------------
__device__ __forceinline__ u64 overlap_d(u64 a0, u64 a1, u64 b0, u64 b1) {
    const u64 lo = a0 > b0 ? a0 : b0, hi = a1 < b1 ? a1 : b1;
    return hi > lo ? hi - lo : 0ull;
}
__device__ __forceinline__ void stat_overflow(u64* stat, u64 bit) { atomicOr(stat, bit); }

// the filled window's slots to their owners: the fill wrote this rank's slots straight into
// its ancestor row (global ids); the slots it wrote into the row's margins belong to a
// neighbour and are packed, with the ancestor's state, into that neighbour's fixed block
__global__ __launch_bounds__(kBlock) void k_exact_route(ExactStep e) {
    if (!e.dec->resampled) return;
    const ExactPlan* xp = e.xp;
    const u64 a = xp->a, b = xp->b;
    const int64_t lo = (int64_t)xp->gofs[e.rank];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the blocks this step needs: a slot of a rank further than a neighbour, or more
        // than `cap` slots for one neighbour, cannot be moved this way
        u64 need = 0;
        for (int g = 0; g < e.world; ++g) {
            if (g == e.rank) continue;
            const u64 n = overlap_d(a, b, xp->gofs[g], xp->gofs[g + 1]);
            if (!n) continue;
            if (g != e.rank - 1 && g != e.rank + 1) stat_overflow(e.stat, 1ull);
            need = n > need ? n : need;
        }
        if (need > (u64)e.cap) stat_overflow(e.stat, 1ull);
        if (need) atomicMax(e.stat + 1, need);
    }
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= 2 * e.cap) return;
    const int side = t >= e.cap ? 1 : 0;
    const int64_t r = side ? e.cap + e.N + (t - e.cap) : t;   // index in the row
    const int64_t sl = lo - e.cap + r;                          // its global slot
    if (sl < 0 || (u64)sl < a || (u64)sl >= b) return;
    const int nb = side ? e.rank + 1 : e.rank - 1;
    if (nb < 0 || nb >= e.world || (u64)sl < xp->gofs[nb] || (u64)sl >= xp->gofs[nb + 1]) return;   // flagged
    const u64 first = a > xp->gofs[nb] ? a : xp->gofs[nb];
    const u64 idx = (u64)sl - first;
    if (idx >= (u64)e.cap) return;                                                                 // flagged
    const int32_t gid = e.row[r];
    const int64_t m = (int64_t)gid - e.goff;
    u64* blk = e.send[side] + idx * kXWords;
    const d2 x = *reinterpret_cast<const d2*>(e.x + 2 * m);
    const d2 v = *reinterpret_cast<const d2*>(e.v + 2 * m);
    const d2 dv = *reinterpret_cast<const d2*>(e.dv + 2 * m);
    blk[0] = (u64)wsmc_d2bits(x.x); blk[1] = (u64)wsmc_d2bits(x.y);
    blk[2] = (u64)wsmc_d2bits(v.x); blk[3] = (u64)wsmc_d2bits(v.y);
    blk[4] = (u64)wsmc_d2bits(dv.x); blk[5] = (u64)wsmc_d2bits(dv.y);
    blk[6] = (u64)(uint32_t)gid;
}
// the slots of this rank filled by a neighbour: the ancestor's pairs by slot, its global id
// into the ancestor row (threads [0, cap) the left block, [cap, 2 cap) the right one)
__global__ __launch_bounds__(kBlock) void k_exact_recv(ExactStep e) {
    if (!e.dec->resampled) return;
    const u64 t = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (t >= 2 * (u64)e.cap) return;
    const int side = t >= (u64)e.cap ? 1 : 0;
    const u64 j = t - (side ? (u64)e.cap : 0ull);
    const int nb = side ? e.rank + 1 : e.rank - 1;
    if (nb < 0 || nb >= e.world) return;
    const ExactPlan* xp = e.xp;
    const u64 lo = xp->gofs[e.rank], hi = xp->gofs[e.rank + 1];
    const u64 cnt = overlap_d(xp->seg[nb], xp->seg[nb + 1], lo, hi);
    if (j >= cnt) return;                       // cnt > cap: the sender flagged it
    const u64 li = (xp->seg[nb] > lo ? xp->seg[nb] : lo) - lo + j;
    const u64* blk = e.recv[side] + j * kXWords;
    *reinterpret_cast<d2*>(e.xr + 2 * li) = d2{wsmc_bits2d(blk[0]), wsmc_bits2d(blk[1])};
    *reinterpret_cast<d2*>(e.vr + 2 * li) = d2{wsmc_bits2d(blk[2]), wsmc_bits2d(blk[3])};
    *reinterpret_cast<d2*>(e.dvr + 2 * li) = d2{wsmc_bits2d(blk[4]), wsmc_bits2d(blk[5])};
    e.anc_row[li] = (int32_t)blk[6];
}
// trace-back windows: out[side][L-1][j][3] for the first (side 0, to the left neighbour) and
// last (side 1, to the right neighbour) ctr ids of this rank's range
__global__ __launch_bounds__(kBlock) void k_exact_window_pack(ExactWin w) {
    const int64_t per = (int64_t)w.T * w.ctr;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= 2 * per) return;
    const int side = t >= per ? 1 : 0;
    if (side == 0 && !w.has_left) return;
    if (side == 1 && !w.has_right) return;
    const int64_t r = t - (side ? per : 0);
    const int L = (int)(r / w.ctr) + 1;
    const int64_t j = r - (int64_t)(L - 1) * w.ctr;
    const int64_t loc = side ? w.N - w.ctr + j : j;
    const d2 x = *reinterpret_cast<const d2*>(w.hist_work[L + 1] + 2 * loc);
    const int32_t an = (L >= 2 && w.dec[L - 1].resampled) ? w.anc_log[(int64_t)(L - 2) * w.anc_stride + loc]
                                                          : (int32_t)(w.goff + loc);
    u64* o = w.out + ((int64_t)side * per + r) * 3;
    o[0] = (u64)wsmc_d2bits(x.x);
    o[1] = (u64)wsmc_d2bits(x.y);
    o[2] = (u64)(uint32_t)an;
}
// the window entry of global id g at level L (the left neighbour's last ids or the right
// neighbour's first ones); nullptr (and the overflow bit) outside both
__device__ __forceinline__ const u64* exact_win(const ExactFinal& f, int L, int64_t g) {
    if (f.win[0] && g >= f.goff - f.ctr && g < f.goff)
        return f.win[0] + ((int64_t)(L - 1) * f.ctr + (g - (f.goff - f.ctr))) * 3;
    if (f.win[1] && g >= f.goff + f.N && g < f.goff + f.N + f.ctr)
        return f.win[1] + ((int64_t)(L - 1) * f.ctr + (g - (f.goff + f.N))) * 3;
    return nullptr;
}
// the owner of global index g among the ranks' peer words (W <= kMaxShards): its ancestor row
// entry at level L (row L - 1) and its history pair at level L; false if no rank holds g
__device__ __forceinline__ bool exact_peer_of(const ExactFinal& f, int64_t g, int& h, int64_t& loc) {
    for (int r = 0; r < f.world; ++r) {
        const int64_t o = (int64_t)f.peer[8 * r + 3], n = (int64_t)f.peer[8 * r + 4];
        if (g >= o && g < o + n) {
            h = r;
            loc = g - o;
            return true;
        }
    }
    return false;
}
__global__ void k_put_words(unsigned long long* dst, PutWords w) {
    if (threadIdx.x < 8) dst[threadIdx.x] = w.w[threadIdx.x];
}
hipError_t launch_put_words(hipStream_t s, unsigned long long* dst, const unsigned long long (&w)[8]) {
    PutWords pw;
    for (int k = 0; k < 8; ++k) pw.w[k] = w[k];
    hipLaunchKernelGGL(k_put_words, dim3(1), dim3(64), 0, s, dst, pw);
    return hipGetLastError();
}
// k_ssm2d_final on exact shards: ancestors are global ids; ids of this rank read its own
// buffers, a neighbour's come from the last step's received pairs (level T) or the trace
// windows (levels below), or — shards of one process (f.peer) — the owner's buffers in place
__global__ __launch_bounds__(kBlock) void k_exact_final(ExactFinal f) {
    __shared__ u64 lds4[4];
    const int64_t N = f.N;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int T = f.T;
    const int64_t S = f.anc_stride;
    u64 exc = 0, bad = 0;
    if (i < N) {
        const bool rsT = f.dec[T].resampled;
        int64_t g = rsT ? (int64_t)f.anc_log[(int64_t)(T - 1) * S + i] : f.goff + i;
        int64_t loc = g - f.goff;
        const bool here = loc >= 0 && loc < N;
        const d2 v = *reinterpret_cast<const d2*>(here ? f.v_work + 2 * loc : f.vr + 2 * i);
        f.v_out[i] = v.x; f.v_out[N + i] = v.y;
        const d2 dv = *reinterpret_cast<const d2*>(here ? f.dv_work + 2 * loc : f.dvr + 2 * i);
        f.dv_out[i] = dv.x; f.dv_out[N + i] = dv.y;
        if (rsT) f.w[i] = f.dec[T].mean;
        const double* xt = f.keep_history ? f.hist_work[T + 1] : f.x_work;
        const d2 xT = *reinterpret_cast<const d2*>(here ? xt + 2 * loc : f.xr + 2 * i);
        double* dT = f.keep_history ? f.hist_out[T + 1] : f.x_out;
        dT[i] = xT.x; dT[N + i] = xT.y;
        if (f.keep_history) {
            for (int s = T - 1; s >= 1; --s) {
                loc = g - f.goff;
                bool in = loc >= 0 && loc < N;
                const u64* wv = in ? nullptr : exact_win(f, s + 1, g);
                if (!in) {
                    const u64 d = (u64)(g < f.goff ? f.goff - g : g - (f.goff + N) + 1);
                    exc = d > exc ? d : exc;
                }
                if (f.dec[s].resampled) {
                    int h;
                    int64_t pl;
                    if (in) g = f.anc_log[(int64_t)(s - 1) * S + loc];
                    else if (wv) g = (int64_t)(int32_t)(uint32_t)wv[2];
                    else if (f.peer && exact_peer_of(f, g, h, pl))   // the owner's row, in place
                        g = reinterpret_cast<const int32_t*>(f.peer[8 * h])[(int64_t)(s - 1) * (int64_t)f.peer[8 * h + 1] + pl];
                    else bad = 1;
                }
                loc = g - f.goff;
                in = loc >= 0 && loc < N;
                d2 x = d2{0.0, 0.0};
                if (in) {
                    x = *reinterpret_cast<const d2*>(f.hist_work[s + 1] + 2 * loc);
                } else {
                    const u64 d = (u64)(g < f.goff ? f.goff - g : g - (f.goff + N) + 1);
                    exc = d > exc ? d : exc;
                    const u64* wx = exact_win(f, s, g);
                    int h;
                    int64_t pl;
                    if (wx) x = d2{wsmc_bits2d(wx[0]), wsmc_bits2d(wx[1])};
                    else if (f.peer && exact_peer_of(f, g, h, pl))   // the owner's history, in place
                        x = *reinterpret_cast<const d2*>(reinterpret_cast<double* const*>(f.peer[8 * h + 2])[s + 1] + 2 * pl);
                    else bad = 1;
                }
                double* dst = f.hist_out[s + 1];
                dst[i] = x.x; dst[N + i] = x.y;
            }
            double* d1 = f.hist_out[1];
            d1[i] = f.x0[0]; d1[N + i] = f.x0[1];
        }
    }
    exc = block_max_u64(exc, lds4);
    bad = block_max_u64(bad, lds4);
    if (threadIdx.x == 0) {
        if (exc) atomicMax(f.stat + 2, exc);
        if (bad) stat_overflow(f.stat, 2ull);
    }
}

constexpr int kOverflowBlocks = 256;   // fill blocks serving overflow chunks (grid-stride)

// ---- the ancestor fill of one chunk of a tile's slots --------------------------------------
// Particle m owns the output slots [hi_{m-1}, hi_m), hi_m = rank(C_m), rank(c) = #{n : x_n < c}
// (include/wsmc_math.h wsmc_rank_r), so a chunk [cs, ce) of the tile's slot range [L, H) is
// filled in three data-parallel passes with no per-slot loop:
//   ranks    every thread ranks its 4 (blocked) particles from the tile's local f64 prefix of q
//            (exact: a tile's q sum stays below 2^53), by the fast path below, exact fallback;
//   marks    a particle owning slots of the chunk writes its id at its first one (one LDS
//            store; the chunk's slots start at -1);
//   expand   a block max-scan over the chunk's slots (8 a thread: running max, DPP wave scan,
//            one LDS round) gives every slot the last mark at or before it — its owner, since
//            ids increase with the slot — and the thread stores its slots with 16-B stores.
// A particle owning many slots (a dominant weight) costs one mark, not a loop.
// Fast rank: y = fma(cl, N/Q, fl(off) N/Q) estimates z = c N / Q (c = off + cl) to within
// 6 * 2^-53 * N <= 2^-19 for N < 2^31; if frac(y) is further than 2^-15 from 0 and 1,
// floor(z) = floor(y), and rank(c) = floor(z) + [R / 2^32 < frac(z)] (R the stratum word of
// slot floor(z)) is decided unless R / 2^32 is within 2^-15 of frac(y). The rest (about 1e-4
// of the particles, and c = 0 or c >= Q) take the exact 64x32-bit path.
constexpr int kFillSlots = kRsChunk / kScanBlock;   // slots a thread expands (8)
constexpr int kFillWin = kRsChunk + 4;              // the chunk, placed 16-B aligned (<= 3 slots of head)
static_assert(kRsTile / kScanBlock == 4 && kFillSlots == 8, "fill: 4 particles and 8 slots a thread");

struct FillLds {
    u64 LH[2];                              // the tile's slot range [L, H)
    double uw[kScanBlock / 64];             // block scan of the tile's q
    u64 red[kScanBlock / 64][2];            // fused fill: the tile's CDF offset and the total Q
    uint32_t last[kScanBlock / 64];         // each wave's last particle's end slot
    int wmax[kScanBlock / 64];              // each wave's last mark
    alignas(16) int32_t out[kFillWin];      // marks -> ancestors, window slot p = slot - cs + head
};

// slot words: R = wsmc_strat_hash(key, slot_base + n) with the 64-bit slot split once per
// launch when its high word is constant over the slots (always on one GPU)
struct SlotHash {
    uint64_t key, base;
    uint32_t kx, blo;
    int fast;          // hi32(base + n) == hi32(base) for every slot n < Nr
    int sys;           // systematic: one word for every slot
    double rsys;       // its R / 2^32
};
__device__ __forceinline__ SlotHash slot_hash_of(const FillPlan& plan, uint64_t opx, uint64_t Nr) {
    SlotHash h;
    h.key = wsmc_strat_key(plan.seed, opx);
    h.base = (uint64_t)plan.slot_base;
    h.fast = (h.base >> 32) == ((h.base + Nr) >> 32);
    h.kx = (uint32_t)h.key ^ ((uint32_t)(h.base >> 32) * 0x85EBCA6Bu ^ (uint32_t)(h.key >> 32));
    h.blo = (uint32_t)h.base;
    h.sys = plan.scheme == 1;
    h.rsys = (double)wsmc_strat_hash(h.key, h.base) * 2.3283064365386963e-10;
    return h;
}
// R / 2^32 of slot ns (exact), branch-free; valid when h.fast (the rank's caller sends the other
// case, a slot range crossing a 2^32 boundary, to the exact path)
__device__ __forceinline__ double slot_word_d(const SlotHash& h, uint32_t ns) {
    const double r = (double)wsmc_strat_fin((h.blo + ns) ^ h.kx) * 2.3283064365386963e-10;
    return h.sys ? h.rsys : r;
}

// an exact integer u64 below 2^52 -> double (q <= 2^43)
__device__ __forceinline__ double u64_small_to_d(u64 v) {
    return __builtin_bit_cast(double, v | 0x4330000000000000ull) - 4503599627370496.0;
}

// rank(c) exactly, c = off + cl; the fast path above, else wsmc_rank_r
__device__ __forceinline__ u64 rank_fast(u64 c, u64 Q, u64 N, double ratio, int scheme, uint64_t seed,
                                         uint64_t op, uint64_t slot_base, uint64_t key) {
    if (c == 0) return 0;
    if (c >= Q) return N;
    constexpr double kMargin = 3.0517578125e-05;    // 2^-15
    const double y = wsmc_u64_to_d(c) * ratio;
    const double fl = wsmc_floor(y);
    const double f = y - fl;                        // exact
    if (f > kMargin && f < 1.0 - kMargin) {
        const u64 ns = (u64)fl;
        if (ns < N) {
            const uint32_t R = wsmc_strat_hash(key, scheme == 1 ? slot_base : slot_base + ns);
            const double dd = f - (double)R * 2.3283064365386963e-10;   // f - R / 2^32
            if (dd > kMargin) return ns + 1;
            if (dd < -kMargin) return ns;
        }
    }
    return wsmc_rank_r(c, Q, N, ratio, scheme, seed, op, slot_base);
}

template <int CTRL, int ROW = 0xf, int BANK = 0xf>
__device__ __forceinline__ int dpp_i32_or(int v, int idn) {
    return __builtin_amdgcn_update_dpp(idn, v, CTRL, ROW, BANK, false);
}
// inclusive max over the wave's lanes (identity -1)
__device__ __forceinline__ int wave_incl_max_i32(int v) {
    int x = max(v, dpp_i32_or<kDppRowShr1>(v, -1));
    x = max(x, dpp_i32_or<kDppRowShr2>(v, -1));
    x = max(x, dpp_i32_or<kDppRowShr3>(v, -1));
    x = max(x, dpp_i32_or<kDppRowShr4, 0xf, 0xe>(x, -1));
    x = max(x, dpp_i32_or<kDppRowShr8, 0xf, 0xc>(x, -1));
    x = max(x, dpp_i32_or<kDppBcast15, 0xa, 0xf>(x, -1));
    x = max(x, dpp_i32_or<kDppBcast31, 0xc, 0xf>(x, -1));
    return x;
}
// inclusive prefix sum of exact-integer f64 values over the wave (sums below 2^53)
__device__ __forceinline__ double wave_incl_scan_f64(double v) {
    double x = v + dpp_f64<kDppRowShr1>(v);
    x = x + dpp_f64<kDppRowShr2>(v);
    x = x + dpp_f64<kDppRowShr3>(v);
    x = x + __builtin_bit_cast(double, dpp_u64<kDppRowShr4, 0xf, 0xe>(__builtin_bit_cast(u64, x)));
    x = x + __builtin_bit_cast(double, dpp_u64<kDppRowShr8, 0xf, 0xc>(__builtin_bit_cast(u64, x)));
    x = x + __builtin_bit_cast(double, dpp_u64<kDppBcast15, 0xa, 0xf>(__builtin_bit_cast(u64, x)));
    x = x + __builtin_bit_cast(double, dpp_u64<kDppBcast31, 0xc, 0xf>(__builtin_bit_cast(u64, x)));
    return x;
}

// the tile's q in registers (4 blocked particles a thread) as exact doubles, and the thread's
// inclusive local prefixes (exact: a tile's sum is at most 2^53)
template <int IT>
__device__ __forceinline__ void load_tile_q(int64_t N, int b, const u64* __restrict__ qbuf, u64 (&q)[IT]) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = (int64_t)b * kRsTile + (int64_t)threadIdx.x * IT + k;
        q[k] = i < N ? qbuf[i] : 0ull;
    }
}

// the same q recomputed from the log-weights against the reference point (the fused run's fill
// when the propagate did not store q: qacc_add's arithmetic, bit for bit)
// (against the guessed reference point rref when the fill checks a guess: consistent with the tile
// partials the propagate took, whether or not the guess was right)
template <int IT>
__device__ __forceinline__ void load_tile_qw(int64_t N, int b, const double* __restrict__ w,
                                             const MaxSlots* __restrict__ ms, const double* rref, u64 (&q)[IT]) {
    double lw[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = (int64_t)b * kRsTile + (int64_t)threadIdx.x * IT + k;
        lw[k] = i < N ? w[i] : -WSMC_INF;
    }
    const double R = rref ? *rref : wsmc_qref(wave_slots_max(ms));
    const double sK = wsmc_pow2i(wsmc_qbits((uint64_t)N));
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        double e = wsmc_expw(lw[k] - R);
        e = e > 0.0 ? e : 0.0;
        q[k] = d_small_to_u64(wsmc_floor(e * sK));
    }
}

// every slot of the window starts at -1 (no mark); the caller's next barrier orders it
__device__ __forceinline__ void fill_clear(FillLds& sh) {
    const int4 m1 = make_int4(-1, -1, -1, -1);
    int4* o = reinterpret_cast<int4*>(sh.out);
    o[2 * threadIdx.x] = m1;
    o[2 * threadIdx.x + 1] = m1;
    if (threadIdx.x == 0) o[2 * kScanBlock] = m1;
}

// store window slots [p0, p0 + 4) (16-B aligned in dst) keeping those in [a, e)
__device__ __forceinline__ void fill_store4(int32_t* __restrict__ dst, int p0, int a, int e, int4 v) {
    if (p0 >= a && p0 + 4 <= e) {
        *reinterpret_cast<int4*>(dst + p0) = v;
    } else if (p0 + 4 > a && p0 < e) {
        if (p0 >= a && p0 < e) dst[p0] = v.x;
        if (p0 + 1 >= a && p0 + 1 < e) dst[p0 + 1] = v.y;
        if (p0 + 2 >= a && p0 + 2 < e) dst[p0 + 2] = v.z;
        if (p0 + 3 >= a && p0 + 3 < e) dst[p0 + 3] = v.w;
    }
}

// Fill chunk j of tile b, given the tile's CDF offset `off`, the total Q, the thread's q and
// its exclusive local prefix `pre` (f64). Entered after a barrier that published `pre` and
// after fill_clear; ends with a barrier when `reuse` (the window is used again).
// MODE (diagnostics only; production = 0): 1 = no exact rank (the estimate, clamped),
// 2 = ranks only (no marks / stores), 3 = scan only
template <int MODE>
__device__ __forceinline__ void fill_chunk_core(int64_t N, int b, int j, u64 Q, u64 off, u64 qb, double pre,
                                                const FillPlan& plan, uint64_t opx,
                                                const u64 (&q)[kRsTile / kScanBlock], int32_t* __restrict__ anc,
                                                FillLds& sh, bool reuse) {
    constexpr int IT = kRsTile / kScanBlock;
    constexpr double kMargin = 3.0517578125e-05;    // 2^-15
    const int th = threadIdx.x, lane = th & 63, wv = th >> 6;
    // exact sharding: targets over the global population, slots written window-relative
    const uint64_t Nr = plan.n_global ? plan.n_global : plan.xp ? plan.xp->N : (uint64_t)N;
    // exact shards without host round trips: slots land in this rank's ancestor row, which
    // covers [row_lo, row_hi) (its own range and a margin per neighbour); global ids
    const u64 s0 = plan.row_hi ? plan.row_lo : plan.xp ? plan.xp->a : 0ull;
    const double ratio = wsmc_u64_to_d(Nr) / wsmc_u64_to_d(Q);
    const double yoff = wsmc_u64_to_d(off) * ratio;
    const SlotHash sh_ = slot_hash_of(plan, opx, Nr);
    // the tile's slot range [L, H) = [rank(off), rank(off + Q_b)), ranked by two threads
    // while the others rank their particles; the next barrier publishes them
    if (th < 2) {
        const u64 c = th == 0 ? off : off + qb;
        sh.LH[th] = rank_fast(c, Q, Nr, ratio, plan.scheme, plan.seed, opx, sh_.base, sh_.key);
    }
    if (MODE == 3) {
        if (pre == 0.123) anc[0] = 1;
        return;
    }
    // ---- ranks: hi[k] = rank(off + cl_k) as a slot index (< 2^31) ----
    const double Nd = wsmc_u64_to_d(Nr);
    uint32_t hi[IT];
    uint32_t slow = 0;                             // particles left to the exact path (bits)
    double cl = pre;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        cl = cl + u64_small_to_d(q[k]);
        const double y = __builtin_fma(cl, ratio, yoff);
        const double fl = wsmc_floor(y);
        const double f = y - fl;                   // exact
        const bool inr = fl < Nd;
        const uint32_t ns = (uint32_t)(inr ? fl : 0.0);
        uint32_t h = ns;
        bool ok = f > kMargin && f < 1.0 - kMargin && inr && sh_.fast;
        if (MODE == 1) {
            ok = true;
            h = fl < Nd ? ns : (uint32_t)Nr;
        } else {
            const double dd = f - slot_word_d(sh_, ns);
            ok = ok && (dd > kMargin || dd < -kMargin);
            h = ns + (dd > kMargin ? 1u : 0u);
        }
        if (k > 0 && q[k] == 0) {                  // no slots: ends where the previous particle ends
            h = hi[k - 1];
            ok = !((slow >> (k - 1)) & 1u);        // final once the previous one is
        }
        hi[k] = h;
        slow |= (ok ? 0u : 1u) << k;
    }
    if (MODE != 1 && slow) {                       // the exact path (rare; c = 0 and c >= Q too)
        double c2 = pre;
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            c2 = c2 + u64_small_to_d(q[k]);
            if (slow >> k & 1u) {
                if (k > 0 && q[k] == 0) {
                    hi[k] = hi[k - 1];
                } else {
                    const u64 c = off + (u64)c2;
                    hi[k] = (uint32_t)wsmc_rank_r(c, Q, Nr, ratio, plan.scheme, plan.seed, opx, sh_.base);
                }
            }
        }
    }
    // first slot of the thread's first particle = the previous thread's last end
    uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi[IT - 1], kDppWaveShr1, 0xf, 0xf, false);
    if (lane == 63) sh.last[wv] = hi[IT - 1];
    __syncthreads();
    const u64 L = sh.LH[0], H = sh.LH[1];
    if (lane == 0) lo = wv > 0 ? sh.last[wv - 1] : (uint32_t)L;
    if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < IT; ++k) hi[k] = hi[k] < (uint32_t)L ? (uint32_t)L : hi[k] > (uint32_t)H ? (uint32_t)H : hi[k];
        lo = lo < (uint32_t)L ? (uint32_t)L : lo > (uint32_t)H ? (uint32_t)H : lo;
    }
    const u64 cs64 = L + (u64)j * kRsChunk;
    const u64 ce64 = cs64 + kRsChunk < H ? cs64 + kRsChunk : H;
    if (cs64 >= ce64) {                            // uniform: no slots in this chunk
        if (reuse) __syncthreads();
        return;
    }
    if (MODE == 2) {
        if (lo == 0x12345678u) anc[0] = 1;
        if (reuse) __syncthreads();
        return;
    }
    const uint32_t cs = (uint32_t)cs64, ce = (uint32_t)ce64;
    // the window: slot s at p = s - cs + head, with p = 0 mod 4 on 16-B boundaries of the row
    int32_t* const dst0 = anc + (cs64 - s0);
    const int head = (int)(((uintptr_t)dst0 >> 2) & 3);
    // ---- marks ----
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t a = lo > cs ? lo : cs;
        const uint32_t e = hi[k] < ce ? hi[k] : ce;
        if (a < e) sh.out[a - cs + head] = (int32_t)(b * kRsTile + th * IT + k) + plan.id_base;
        lo = hi[k];
    }
    __syncthreads();
    // ---- expand: block max-scan over the window, 8 slots a thread ----
    const int4* o4 = reinterpret_cast<const int4*>(sh.out);
    int4 v0 = o4[2 * th], v1 = o4[2 * th + 1];
    v0.y = max(v0.y, v0.x); v0.z = max(v0.z, v0.y); v0.w = max(v0.w, v0.z);
    v1.x = max(v1.x, v0.w); v1.y = max(v1.y, v1.x); v1.z = max(v1.z, v1.y); v1.w = max(v1.w, v1.z);
    const int inc = wave_incl_max_i32(v1.w);
    int carry = __builtin_amdgcn_update_dpp(-1, inc, kDppWaveShr1, 0xf, 0xf, false);
    if (lane == 63) sh.wmax[wv] = inc;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanBlock / 64 - 1; ++k)
        if (k < wv) carry = max(carry, sh.wmax[k]);
    v0.x = max(v0.x, carry); v0.y = max(v0.y, carry); v0.z = max(v0.z, carry); v0.w = max(v0.w, carry);
    v1.x = max(v1.x, carry); v1.y = max(v1.y, carry); v1.z = max(v1.z, carry); v1.w = max(v1.w, carry);
    // ---- stores: the window's [a, e) (exact shards: the part of the chunk the row covers;
    // the rest cannot be routed) ----
    int a = head, e = head + (int)(ce - cs);
    if (plan.row_hi) {
        const u64 w0 = cs64 > plan.row_lo ? cs64 : plan.row_lo, w1 = ce64 < plan.row_hi ? ce64 : plan.row_hi;
        if (th == 0 && (w0 != cs64 || w1 != ce64)) atomicOr(plan.xstat, 1ull);
        a = w1 > w0 ? head + (int)(w0 - cs64) : 0;
        e = w1 > w0 ? head + (int)(w1 - cs64) : 0;
    }
    int32_t* const dst = dst0 - head;              // window slot p lands at dst[p]
    fill_store4(dst, 8 * th, a, e, v0);
    fill_store4(dst, 8 * th + 4, a, e, v1);
    if (th == kScanBlock - 1 && e > kRsChunk) {    // the window's last (head) slots
        int4 v2 = o4[2 * kScanBlock];
        v2.x = max(v2.x, v1.w); v2.y = max(v2.y, v2.x); v2.z = max(v2.z, v2.y); v2.w = max(v2.w, v2.z);
        fill_store4(dst, kRsChunk, a, e, v2);
    }
    if (reuse) __syncthreads();
}

// block exclusive prefix of the threads' tile-q sums (exact f64); ends with the barrier that
// publishes it
__device__ __forceinline__ double fill_scan_q(double tsum, FillLds& sh) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double x = wave_incl_scan_f64(tsum);
    if (lane == 63) sh.uw[wv] = x;
    __syncthreads();
    double pre = 0.0;
#pragma unroll
    for (int k = 0; k < kScanBlock / 64 - 1; ++k)
        if (k < wv) pre = pre + sh.uw[k];
    return pre + (x - tsum);
}

__device__ __forceinline__ double tile_q_sum(const u64 (&q)[kRsTile / kScanBlock]) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kRsTile / kScanBlock; ++k) s = s + u64_small_to_d(q[k]);
    return s;
}

// a whole chunk given the tile's offset and Q (generic Resample, overflow chunks); QW: q from the
// log-weights wq against the reference point of the max slots ms
template <int MODE, bool QW = false>
__device__ __forceinline__ void fill_chunk(int64_t N, int b, int j, u64 Q, u64 off, const FillPlan& plan,
                                           uint64_t opx, const u64* __restrict__ qbuf, int32_t* __restrict__ anc,
                                           FillLds& sh, const double* __restrict__ wq = nullptr,
                                           const MaxSlots* __restrict__ ms = nullptr) {
    u64 q[kRsTile / kScanBlock];
    if (QW)
        load_tile_qw(N, b, wq, ms, plan.rg_check, q);
    else
        load_tile_q(N, b, qbuf, q);
    const u64 qb = plan.tilep[(int64_t)b * kPart];
    fill_clear(sh);
    const double pre = fill_scan_q(tile_q_sum(q), sh);
    fill_chunk_core<MODE>(N, b, j, Q, off, qb, pre, plan, opx, q, anc, sh, true);
}

// Ancestor fill (the icdf merge, src/resampling.jl:13-26): ancestor(slot n) = smallest m
// with C_m > x_n, i.e. particle m owns the slots [rank(C_{m-1}), rank(C_m)) with
// rank(c) = #{n : x_n < c}. Block b < ntiles fills the first chunk
// (<= kRsChunk slots) of tile b: no lookup, every load independent. kOverflowBlocks more
// blocks take, grid-stride, the later chunks of tiles owning more than kRsChunk slots
// (a dominant particle adds chunks, never a long loop in one block).
// MODE (diagnostics only; production = 0): 1 = no rank (cheap estimate), 2 = no fill,
// 3 = scan only
template <int MODE>
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(6))) void k_rs_scan_t(int64_t N, const ShardRecord* __restrict__ rec,
                                                          const Decision* __restrict__ dec, FillPlan plan,
                                                          const u64* __restrict__ tileOff,
                                                          const u64* __restrict__ qbuf, int32_t* __restrict__ anc) {
    __shared__ FillLds sh;
    const int t = blockIdx.x;
    const int ntiles = (int)((N + kRsTile - 1) / kRsTile);
    if (t == 0 && threadIdx.x == 0 && plan.host_dec) *plan.host_dec = *dec;   // the host's copy
    const int rs = dec->resampled;
    if (!rs) return;
    // exact sharding: the global CDF (this shard's tiles offset by the lower ranks' Q)
    const u64 Q = plan.xp ? plan.xp->Q : rec->Q;
    const u64 cb = plan.xp ? plan.xp->cbase : 0ull;
    const uint64_t opx = op_eff(plan.op, plan.op_dev);
    if (t < ntiles) {
        fill_chunk<MODE>(N, t, 0, Q, cb + tileOff[t], plan, opx, qbuf, anc, sh);
        if (plan.w_reset) {   // the weights reset to the log-mean (the fill read q, not w)
            const double mean = dec->mean;
            for (int k = threadIdx.x; k < kRsTile; k += kScanBlock) {
                const int64_t i = (int64_t)t * kRsTile + k;
                if (i < N) plan.w_reset[i] = mean;
            }
        }
        return;
    }
    const int ntasks = dec->ntasks;
    for (int o = t - ntiles; o < ntasks; o += kOverflowBlocks) {
        const int b = plan.taskTile[o];
        fill_chunk<MODE>(N, b, 1 + o - plan.taskOff[b], Q, cb + tileOff[b], plan, opx, qbuf, anc, sh);
    }
}

// ---- multinomial resampling (include/wsmc_math.h wsmc_multi_e) ----------------------
// Weight statistics for a multinomial Resample: the tile partials of k_rs_sums_t (the same
// exact integers), plus per particle the tile-local inclusive prefix of q (C_m =
// tileOff[tile] + lcdf[m]) and per tile the sum of the slots' exponential spacings E.
// 4 blocked particles per thread so one block scan gives the prefix.
__global__ __launch_bounds__(kSumBlock) void k_rs_sums_multi(const double* __restrict__ w, int64_t N,
                                                             const MaxSlots* __restrict__ ms, FillPlan plan,
                                                             u64* __restrict__ tilep, u64* __restrict__ lcdf,
                                                             u64* __restrict__ esum, uint32_t* __restrict__ ebuf) {
    constexpr int IT = kRsTile / kSumBlock;
    __shared__ double s_f[kPart][kSumBlock / 64];
    __shared__ u64 s_e[kSumBlock / 64];
    __shared__ u64 s_w[kSumBlock / 64];
    const int th = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kRsTile + (int64_t)th * IT;
    double lw[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) lw[k] = base + k < N ? w[base + k] : -WSMC_INF;
    const double M = wsmc_qref(wave_slots_max(ms));   // the reference point
    const double sK = wsmc_pow2i(wsmc_qbits((uint64_t)N));
    const uint64_t opx = op_eff(plan.op, plan.op_dev);
    u64 q[IT], E = 0;
    QAcc acc;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        q[k] = qacc_add(acc, wsmc_expw(lw[k] - M), sK);
        if (base + k < N) {
            const u64 ek = wsmc_multi_e(plan.seed, opx, (uint64_t)plan.slot_base, (uint64_t)(base + k), (uint64_t)N);
            E += ek;
            ebuf[base + k] = (uint32_t)ek;                  // E < 2^30 (-log u <= 36.8)
        }
    }
    u64 qtot;
    u64 c = block_excl_scan_u64<kSumBlock / 64>(d_small_to_u64(acc.Q), s_w, &qtot);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        c += q[k];
        if (base + k < N) lcdf[base + k] = c;
    }
    E = wave_sum_u64(E);
    if ((th & 63) == 0) s_e[th >> 6] = E;
    qacc_tile<kSumBlock>(acc, s_f, tilep + (int64_t)blockIdx.x * kPart);   // its barrier publishes s_e
    if (th == kPart) {
        u64 t = 0;
#pragma unroll
        for (int v = 0; v < kSumBlock / 64; ++v) t += s_e[v];
        esum[blockIdx.x] = t;
    }
}

__device__ __forceinline__ u64 multi_cval(const u64* __restrict__ tileOff, const u64* __restrict__ lcdf, int64_t m) {
    return tileOff[m / kRsTile] + lcdf[m];
}
// the ancestor of one slot from scratch, by one wave: a 64-ary search of m -> [C_m > x]
// (false ... false true ... true; C_{N-1} = Q > x): each round the 64 lanes probe
// evenly spaced particles in parallel and the ballot narrows the range 64-fold, so 1M
// particles take 4 rounds of two independent loads instead of a 20-load serial chain
__device__ int64_t multi_locate_wave(int64_t N, const u64* __restrict__ tileOff, const u64* __restrict__ lcdf, u64 Q,
                                     u64 P, u64 PN) {
    const int lane = threadIdx.x & 63;
    int64_t lo = 0, hi = N - 1;
    while (hi > lo) {
        const int64_t S = hi - lo + 1;
        const int64_t step = (S + 63) / 64;
        int64_t m = lo + (int64_t)(lane + 1) * step - 1;
        if (m > hi) m = hi;
        const bool t = wsmc_multi_above(multi_cval(tileOff, lcdf, m), Q, P, PN);
        const int f = __popcll(~__ballot(t));        // lanes probing a "false" (a prefix)
        if (S <= 64) return lo + f;                  // every particle of [lo, hi] was probed
        const int64_t lo2 = f == 0 ? lo : lo + (int64_t)f * step;
        const int64_t hi2 = lo + (int64_t)(f + 1) * step - 1;
        lo = lo2;
        hi = hi2 < hi ? hi2 : hi;
    }
    return lo;
}

// Slots of one tile (4 consecutive per thread): E recomputed, block scan + the tile's
// offset (reduce kernel) -> P_n; P_N = total + the terminal E_N. The first and last slot
// are located from scratch; the CDF between their ancestors is staged in LDS when it
// spans <= kMultiStage particles (the usual case), and every slot searches from the
// previous slot's answer.
constexpr int kMultiStage = 4096;
__global__ __launch_bounds__(kScanBlock) void k_multi_fill(int64_t N, const ShardRecord* __restrict__ rec,
                                                           const Decision* __restrict__ dec, FillPlan plan,
                                                           const u64* __restrict__ tileOff,
                                                           const u64* __restrict__ lcdf, const u64* __restrict__ esum,
                                                           const uint32_t* __restrict__ ebuf, int32_t* __restrict__ anc) {
    constexpr int IT = kRsTile / kScanBlock;
    __shared__ u64 s_w[kScanBlock / 64];
    __shared__ int64_t s_m[2];
    __shared__ u64 sC[kMultiStage];
    if (blockIdx.x == 0 && threadIdx.x == 0 && plan.host_dec) *plan.host_dec = *dec;   // the host's copy
    if (!dec->resampled) return;
    const int th = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kRsTile;
    const int64_t last = (base + kRsTile < N ? base + kRsTile : N) - 1;
    const int64_t nt = (N + kRsTile - 1) / kRsTile;
    const uint64_t opx = op_eff(plan.op, plan.op_dev);
    const u64 Q = rec->Q;
    const u64 PN = esum[nt] + wsmc_multi_e(plan.seed, opx, (uint64_t)plan.slot_base, (uint64_t)N, (uint64_t)N);
    u64 e[IT], t = 0;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = base + (int64_t)th * IT + k;
        e[k] = i <= last ? (u64)ebuf[i] : 0ull;
        t += e[k];
    }
    u64 tot;
    u64 P = esum[blockIdx.x] + block_excl_scan_u64<kScanBlock / 64>(t, s_w, &tot);
    u64 Pk[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) { P += e[k]; Pk[k] = P; }
    // first slot: wave 0 (thread 0's P); last slot: the wave of the thread holding it
    const int64_t lt = last - base;
    const int tl = (int)(lt / IT), wv = th >> 6;
    if (wv == 0) {
        const u64 P0 = __shfl(Pk[0], 0, 64);
        const int64_t m = multi_locate_wave(N, tileOff, lcdf, Q, P0, PN);
        if (th == 0) s_m[0] = m;
    }
    if (wv == tl >> 6) {
        u64 Pl = Pk[0];
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (k == lt % IT) Pl = Pk[k];
        Pl = __shfl(Pl, tl & 63, 64);
        const int64_t m = multi_locate_wave(N, tileOff, lcdf, Q, Pl, PN);
        if (th == tl) s_m[1] = m;
    }
    __syncthreads();
    const int64_t mlo = s_m[0], mhi = s_m[1];
    const int64_t span = mhi - mlo + 1;
    if (span <= kMultiStage) {
        for (int64_t j = th; j < span; j += kScanBlock) sC[j] = multi_cval(tileOff, lcdf, mlo + j);
        __syncthreads();
        // gallop from the previous answer (sorted slots: usually 0-2 particles ahead), then
        // bisect the last doubling interval
        int lo = 0;
        const int hi = (int)(span - 1);
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int64_t i = base + (int64_t)th * IT + k;
            if (i > last) break;
            int a = lo, b = lo, g = 1;
            while (b < hi && !wsmc_multi_above(sC[b], Q, Pk[k], PN)) {
                a = b + 1;
                b = b + g < hi ? b + g : hi;
                g <<= 1;
            }
            while (a < b) {
                const int mid = (a + b) >> 1;
                if (wsmc_multi_above(sC[mid], Q, Pk[k], PN)) b = mid; else a = mid + 1;
            }
            lo = a;
            anc[i] = (int32_t)(mlo + a);
        }
        return;
    }
    int64_t lo = mlo;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int64_t i = base + (int64_t)th * IT + k;
        if (i > last) break;
        int64_t a = lo, b = mhi;
        while (a < b) {
            const int64_t mid = (a + b) >> 1;
            if (wsmc_multi_above(multi_cval(tileOff, lcdf, mid), Q, Pk[k], PN)) b = mid; else a = mid + 1;
        }
        lo = a;
        anc[i] = (int32_t)a;
    }
}

// ---- sample(state, n; replace) (src/utils.jl:92-118; include/wsmc_math.h) -------------
// with replacement: one independent draw per thread, located in the integer CDF
__global__ __launch_bounds__(kBlock) void k_sample_draws(int64_t n, int64_t N, const ShardRecord* __restrict__ rec,
                                                         const u64* __restrict__ tileOff,
                                                         const u64* __restrict__ lcdf, uint64_t seed, uint64_t op,
                                                         int64_t* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const u64 x = wsmc_multi_target(wsmc_multi_word(seed, op, (uint64_t)j), rec->Q);
    const int64_t nt = (N + kRsTile - 1) / kRsTile;
    int64_t lo = 0, hi = nt;                         // largest tile b with tileOff[b] <= x
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (tileOff[mid] <= x) lo = mid; else hi = mid;
    }
    const u64 off = tileOff[lo];
    int64_t m0 = lo * kRsTile, m1 = (m0 + kRsTile < N ? m0 + kRsTile : N) - 1;
    while (m0 < m1) {                                // smallest m in the tile with C_m > x
        const int64_t mid = (m0 + m1) >> 1;
        if (off + lcdf[mid] > x) m1 = mid; else m0 = mid + 1;
    }
    out[j] = m0;
}
// without replacement: Efraimidis–Spirakis keys (ordered encoding) and indices to sort
__global__ __launch_bounds__(kBlock) void k_es_keys(const double* __restrict__ w, int64_t N,
                                                    const MaxSlots* __restrict__ ms, uint64_t seed, uint64_t op,
                                                    u64* __restrict__ keys, u64* __restrict__ idx) {
    const double M = wsmc_qref(wave_slots_max(ms));   // the reference point
    const int K = wsmc_qbits((uint64_t)N);
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    keys[i] = wsmc_ord_enc(wsmc_es_key(seed, op, (uint64_t)i, wsmc_qweight(w[i], M, K)));
    idx[i] = (u64)i;
}
// sample(state, n; replace=true) on a shard: draw j's target x (the single-context formula
// over the population's Q) lands in this shard iff base <= x < base + Qloc; then its
// ancestor is the smallest local m with base + C_m > x. out[j] = global index + 1, or 0.
__global__ __launch_bounds__(kBlock) void k_sample_draws_shard(int64_t n, int64_t N, const u64* __restrict__ cdf,
                                                               u64 base, u64 Qloc, u64 Q, uint64_t seed,
                                                               uint64_t op, int64_t goff, int64_t* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const u64 x = wsmc_multi_target(wsmc_multi_word(seed, op, (uint64_t)j), Q);
    if (x < base || x - base >= Qloc) {
        out[j] = 0;
        return;
    }
    const u64 xl = x - base;
    int64_t lo = 0, hi = N - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cdf[mid] > xl) hi = mid; else lo = mid + 1;
    }
    out[j] = goff + lo + 1;
}
hipError_t launch_sample_draws_shard(hipStream_t s, int64_t n, int64_t N, const u64* cdf, u64 base, u64 Qloc, u64 Q,
                                     uint64_t seed, uint64_t op, int64_t goff, int64_t* out) {
    hipLaunchKernelGGL(k_sample_draws_shard, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, N,
                       cdf, base, Qloc, Q, seed, op, goff, out);
    return hipGetLastError();
}
// Efraimidis–Spirakis keys of a shard: the global index keys the draw, the integer weight is
// relative to the population's max with the global N's K
__global__ __launch_bounds__(kBlock) void k_es_keys_shard(const double* __restrict__ w, int64_t N, int64_t gN,
                                                          int64_t goff, const MaxSlots* __restrict__ ms,
                                                          uint64_t seed, uint64_t op, u64* __restrict__ keys,
                                                          u64* __restrict__ idx) {
    const double M = wsmc_qref(wave_slots_max(ms));   // the reference point
    const int K = wsmc_qbits((uint64_t)gN);
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    keys[i] = wsmc_ord_enc(wsmc_es_key(seed, op, (uint64_t)(goff + i), wsmc_qweight(w[i], M, K)));
    idx[i] = (u64)(goff + i);
}
hipError_t launch_es_keys_shard(hipStream_t s, const double* w, int64_t N, int64_t gN, int64_t goff,
                                const MaxSlots* ms, uint64_t seed, uint64_t op, u64* keys, u64* idx) {
    hipLaunchKernelGGL(k_es_keys_shard, dim3((unsigned)((N + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w, N, gN, goff,
                       ms, seed, op, keys, idx);
    return hipGetLastError();
}
// rows of a column: out[k][j] = col[k][idx[j]]
__global__ __launch_bounds__(kBlock) void k_gather_rows(const double* __restrict__ src, int64_t N, int dim,
                                                        const int64_t* __restrict__ idx, int64_t n,
                                                        double* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const int64_t i = idx[j];
    for (int k = 0; k < dim; ++k) out[(int64_t)k * n + j] = src[(int64_t)k * N + i];
}

// ---- describe(): weighted median / histogram (include/wsmc_math.h) --------------------
__global__ __launch_bounds__(kBlock) void k_median_keys(const double* __restrict__ x, const u64* __restrict__ q,
                                                        int64_t N, u64* __restrict__ kq, u64* __restrict__ kv) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    kq[i] = q[i];
    kv[i] = wsmc_ord_enc(x[i]);
}
// first index in [0, N) with S[i] >= t (S non-decreasing); N if none
__device__ int64_t lower_bound_u64(const u64* S, int64_t N, u64 t) {
    int64_t lo = 0, hi = N;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (S[mid] >= t) hi = mid; else lo = mid + 1;
    }
    return lo;
}
// sorted (value, q) pairs + inclusive prefix S of q: StatsBase's walk by binary search
__global__ void k_median_pick(const u64* __restrict__ v, const u64* __restrict__ q, const u64* __restrict__ S,
                              int64_t N, double* out) {
    if (threadIdx.x != 0) return;
    const u64 Q = S[N - 1];
    const int64_t i1 = lower_bound_u64(S, N, 1);                 // the first nonzero weight
    const u64 q1 = q[i1];
    const wsmc_u128 H2 = (wsmc_u128)Q + q1;                       // 2 h
    int64_t lo = 0, hi = N;                                       // first k with 2 S_k > 2 h
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (2 * (wsmc_u128)S[mid] > H2) hi = mid; else lo = mid + 1;
    }
    if (lo == N) {                                                // h beyond the total: the largest value
        *out = wsmc_ord_dec(v[lower_bound_u64(S, N, Q)]);
        return;
    }
    const u64 wk = q[lo], Skold = S[lo] - wk;
    const double vkold = Skold ? wsmc_ord_dec(v[lower_bound_u64(S, N, Skold)]) : 0.0;
    *out = wsmc_median_interp(vkold, wsmc_ord_dec(v[lo]), Q, q1, Skold, wk);
}
struct HistEdges { double e[9]; };
__global__ __launch_bounds__(kBlock) void k_hist(const double* __restrict__ x, const u64* __restrict__ q, int64_t N,
                                                 HistEdges ed, u64* __restrict__ cnt) {
    __shared__ u64 s_c[8];
    if (threadIdx.x < 8) s_c[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
        const u64 w = q[i];
        if (w) atomicAdd(&s_c[wsmc_hist_bin(x[i], ed.e, 8)], w);   // integers: order-free
    }
    __syncthreads();
    if (threadIdx.x < 8 && s_c[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], s_c[threadIdx.x]);
}

// ---- fused single-GPU resample: no reduce kernel ----------------------------------
// block sum of two u64 values (all threads get the totals)
__device__ __forceinline__ void block_sum2_u64(u64& a, u64& b, u64 (*lds)[2]) {
    a = wave_sum_u64(a);
    b = wave_sum_u64(b);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { lds[wv][0] = a; lds[wv][1] = b; }
    __syncthreads();
    a = 0; b = 0;
#pragma unroll
    for (int v = 0; v < kScanBlock / 64; ++v) { a += lds[v][0]; b += lds[v][1]; }
    __syncthreads();
}

// The decision and the ancestor fill of one Resample in one launch (single GPU, fused run).
// The weight-statistics kernel left per-tile partials and per-group sums (G tiles a group):
//  * block ntiles + kOverflowBlocks builds the shard record from the tile partials, the
//    group sums and the max slots and takes the decision (strict ESS test, log-mean) —
//    concurrently with the fill;
//  * block b < ntiles fills the first chunk of tile b, its CDF offset being the groups
//    before it plus the tiles before it in its group (O(sqrt(ntiles)) loads, no reduce pass);
//  * kOverflowBlocks blocks plan the overflow chunks from the tile sums and fill them.
// The fill does not wait for the decision: when the step does not resample, the row it
// writes is never read (the next step and the trace-back check the decision).
// MODE (diagnostics only, results wrong; production = 0): 1 = the record block only marks
// the step resampled with mean 0 (the same fill work under forced resampling: q depends on
// lw - M only)
// QW (round 6, the fused run after a propagate that took the statistics): the tile blocks
// recompute q from the weights wq instead of loading it (no q in HBM)
#ifndef WSMC_FILL_WAVES   // build-time override for occupancy experiments (tools/build_variant.py)
#define WSMC_FILL_WAVES 6
#endif
template <int MODE, bool QW = false>
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(WSMC_FILL_WAVES))) void k_rs_fill_fused(int64_t N, FillPlan plan, const u64* __restrict__ grp,
                                                              int G, const MaxSlots* __restrict__ ms, double ess_min,
                                                              ShardRecord* rec, Decision* dec,
                                                              const u64* __restrict__ qbuf, int32_t* __restrict__ anc,
                                                              const double* __restrict__ wq) {
    __shared__ FillLds sh;
    __shared__ u64 s_red[kScanBlock / 64][2];
    __shared__ u64 s_parts[kScanBlock / 64][kRedPart];
    __shared__ u64 s_task[3];
    __shared__ u64 s_u[kScanBlock / 64];
    const int th = threadIdx.x;
    const int ntiles = (int)((N + kRsTile - 1) / kRsTile);
    const int ngroups = (ntiles + G - 1) / G;
    // block 0 (dispatched first: its serial decision is the longest chain) is the record
    // block; blocks 1..ntiles fill the tiles' first chunks, the rest serve overflow chunks
#ifndef WSMC_FILL_XCD
#define WSMC_FILL_XCD 1
#endif
#if WSMC_FILL_XCD
    // tile t on block t + 8: the XCD (blockIdx % 8) of the propagate block that wrote its q,
    // tile partials and group line (k_ssm2d_prop: tile t on block t), so the first loads can hit
    // that XCD's L2; blocks 1..7 serve overflow chunks 0..6, the blocks after the tiles the rest
    const int bx = (int)blockIdx.x;
    const int t = bx == 0 ? ntiles + kOverflowBlocks
                : bx < 8 ? ntiles + (bx - 1)
                : bx < 8 + ntiles ? bx - 8
                : ntiles + 7 + (bx - 8 - ntiles);
    static_assert(kOverflowBlocks >= 7, "blocks 1..7 are overflow blocks");
#else
    const int t = blockIdx.x == 0 ? ntiles + kOverflowBlocks : (int)blockIdx.x - 1;
#endif
    if (MODE == 1 && t == ntiles + kOverflowBlocks) {
        if (th == 0 && dec) { dec->resampled = 1; dec->mean = 0.0; dec->ess = 0.0; dec->M = 0.0; }
        return;
    }
    if (t == ntiles + kOverflowBlocks && plan.xlines) {
        // ---- exact shards: every rank's record from its all-gathered group lines and max
        // slots, then the single-GPU decision and the slot windows (decide_exact) ----
        __shared__ ShardRecord s_recs[kMaxShards];
        const int W = plan.dx_world;
        const int ngw = (int)(plan.xstride / kGroupLine);
        for (int g = 0; g < W; ++g) {
            const u64* L = plan.xlines + (int64_t)g * plan.xstride;
            u64 q = 0, q2 = 0, f2lo = 0, f2hi = 0, flo = 0, fhi = 0;
            for (int k = th; k < ngw; k += kScanBlock) {
                const u64* l = L + (int64_t)k * kGroupLine;
                q += l[0]; q2 += l[2];
                f2lo += l[3] & 0xffffffffull; f2hi += l[3] >> 32;
                flo += l[4] & 0xffffffffull; fhi += l[4] >> 32;
            }
            const u64 mv = th < kSlots ? plan.xms[g].v[th][0] : 0ull;
            const u64 menc = wave_max_u64(mv);
            u64 acc[kRedPart] = {q, q2, f2lo, f2hi, flo, fhi};
#pragma unroll
            for (int k = 0; k < kRedPart; ++k) acc[k] = wave_sum_u64(acc[k]);
            if ((th & 63) == 0)
#pragma unroll
                for (int k = 0; k < kRedPart; ++k) s_parts[th >> 6][k] = acc[k];
            __syncthreads();
            if (th == 0) {
                u64 tot[kRedPart] = {0, 0, 0, 0, 0, 0};
                for (int v = 0; v < kScanBlock / 64; ++v)
                    for (int k = 0; k < kRedPart; ++k) tot[k] += s_parts[v][k];
                ShardRecord r;
                r.menc = menc;
                r.Q = tot[0];
                r.q2 = tot[1];
                const wsmc_u128 Wf2 = (wsmc_u128)tot[2] + ((wsmc_u128)tot[3] << 32);
                const wsmc_u128 Wf = (wsmc_u128)tot[4] + ((wsmc_u128)tot[5] << 32);
                r.wf2lo = (u64)Wf2; r.wf2hi = (u64)(Wf2 >> 64);
                r.wflo = (u64)Wf; r.wfhi = (u64)(Wf >> 64);
                r.n = L[7];
                s_recs[g] = r;
                if (g == plan.dx_rank) *rec = r;
            }
            __syncthreads();
        }
        if (th == 0)
            decide_exact(s_recs, W, plan.dx_rank, plan.dx_ess, plan, plan.dx_comb, plan.dx_dec, plan.dx_xp);
        return;
    }
    if (t == ntiles + kOverflowBlocks) {
        // ---- the shard record and (one GPU, dec != null) the decision; a sharded run
        // all-gathers the records and decides afterwards (k_rs_decide) ----
        for (int64_t k = th; k < plan.grp_zero_words; k += kScanBlock) plan.grp_zero[k] = 0ull;
        u64 acc[kRedPart] = {0, 0, 0, 0, 0, 0};
        for (int g = th; g < ngroups; g += kScanBlock) acc[0] += grp[(int64_t)g * kGroupLine];
        for (int b = th; b < ntiles; b += kScanBlock) {
            const u64 q2 = plan.tilep[(int64_t)b * kPart + 1], wf2 = plan.tilep[(int64_t)b * kPart + 2],
                      wf = plan.tilep[(int64_t)b * kPart + 3];
            acc[1] += q2;
            acc[2] += wf2 & 0xffffffffull; acc[3] += wf2 >> 32;
            acc[4] += wf & 0xffffffffull; acc[5] += wf >> 32;
        }
        const u64 menc = th < kSlots ? wave_max_u64(ms->v[th & (kSlots - 1)][0]) : 0ull;
#pragma unroll
        for (int k = 0; k < kRedPart; ++k) acc[k] = wave_sum_u64(acc[k]);
        if ((th & 63) == 0)
#pragma unroll
            for (int k = 0; k < kRedPart; ++k) s_parts[th >> 6][k] = acc[k];
        __syncthreads();
        if (th == 0) {
            u64 tot[kRedPart] = {0, 0, 0, 0, 0, 0};
            for (int v = 0; v < kScanBlock / 64; ++v)
                for (int k = 0; k < kRedPart; ++k) tot[k] += s_parts[v][k];
            ShardRecord r;
            r.menc = menc;
            r.Q = tot[0];
            r.q2 = tot[1];
            const wsmc_u128 Wf2 = (wsmc_u128)tot[2] + ((wsmc_u128)tot[3] << 32);
            const wsmc_u128 Wf = (wsmc_u128)tot[4] + ((wsmc_u128)tot[5] << 32);
            r.wf2lo = (u64)Wf2; r.wf2hi = (u64)(Wf2 >> 64);
            r.wflo = (u64)Wf; r.wfhi = (u64)(Wf >> 64);
            r.n = (u64)N;
            *rec = r;
            // the propagate took the statistics against its guess: a miss makes this step's
            // decision and fill non-canonical (but consistent with one another: no hazard); the
            // host re-does the run on the exact path
            if (plan.rg_check && !(wsmc_qref(wsmc_ord_dec(menc)) == *plan.rg_check)) atomicAdd(plan.rg_miss, 1);
            if (dec) {
                decide_records(&r, 1, 0, ess_min, dec);
                if (plan.host_dec) *plan.host_dec = *dec;   // the generic Resample's host copy
                if (plan.base_out) *plan.base_out = dec->resampled ? dec->mean : wsmc_ord_dec(menc);
                // the generic Resample defers its weight reset: the max of the reset (equal)
                // weights goes into the slots now (the fill's other blocks never read them)
                if (plan.ms_reset && dec->resampled) {
                    plan.ms_reset->v[0][0] = wsmc_ord_enc(dec->mean);
                    for (int k = 1; k < kSlots; ++k) plan.ms_reset->v[k][0] = 0ull;
                }
            }
        }
        return;
    }
    const uint64_t opx = op_eff(plan.op, plan.op_dev);
    if (t < ntiles) {
        // ---- first chunk of tile t (its q loads in flight while the offset is summed) ----
        u64 q[kRsTile / kScanBlock];
        if (QW)
            load_tile_qw(N, t, wq, ms, plan.rg_check, q);
        else
            load_tile_q(N, t, qbuf, q);
        const u64 qb = plan.tilep[(int64_t)t * kPart];   // every load of the block is issued here
        const int g = t / G;
        u64 pre = 0, tot = 0;
        if (plan.xlines) {   // exact shards: the global Q; the lower ranks' Q, then this rank's groups before
            const int ngw = (int)(plan.xstride / kGroupLine);
            for (int k = th; k < plan.dx_world * ngw; k += kScanBlock) {
                const int r = k / ngw, kk = k - r * ngw;
                const u64 v = plan.xlines[(int64_t)r * plan.xstride + (int64_t)kk * kGroupLine];
                tot += v;
                pre += (r < plan.dx_rank || (r == plan.dx_rank && kk < g)) ? v : 0ull;
            }
        } else {
            for (int k = th; k < ngroups; k += kScanBlock) {
                const u64 v = grp[(int64_t)k * 8];
                tot += v;
                pre += k < g ? v : 0ull;
            }
        }
        for (int b = g * G + th; b < t; b += kScanBlock) pre += plan.tilep[(int64_t)b * kPart];
        fill_clear(sh);
        // one barrier for the tile's CDF offset, the total Q and the scan of its q
        const int lane = th & 63, wv = th >> 6;
        pre = wave_sum_u64(pre);
        tot = wave_sum_u64(tot);
        const double tsum = tile_q_sum(q);
        const double x = wave_incl_scan_f64(tsum);
        if (lane == 63) {
            sh.uw[wv] = x;
            sh.red[wv][0] = pre;
            sh.red[wv][1] = tot;
        }
        __syncthreads();
        u64 off = 0, Q = 0;
        double lp = 0.0;
#pragma unroll
        for (int k = 0; k < kScanBlock / 64; ++k) {
            off += sh.red[k][0];
            Q += sh.red[k][1];
            if (k < wv) lp = lp + sh.uw[k];
        }
        fill_chunk_core<0>(N, t, 0, Q, off, qb, lp + (x - tsum), plan, opx, q, anc, sh, false);
        return;
    }
    // ---- overflow chunks: plan from the tile sums (contiguous tiles per thread) ----
    u64 Q = 0, qmax = 0, cbase = 0;
    for (int k = th; k < ngroups; k += kScanBlock) {
        Q += grp[(int64_t)k * kGroupLine];
        const u64 m = grp[(int64_t)k * kGroupLine + 1];
        qmax = m > qmax ? m : qmax;
    }
    if (plan.xlines) {   // exact shards: the global Q and this rank's CDF base
        Q = 0;
        const int ngw = (int)(plan.xstride / kGroupLine);
        for (int k = th; k < plan.dx_world * ngw; k += kScanBlock) {
            const int r = k / ngw, kk = k - r * ngw;
            const u64 v = plan.xlines[(int64_t)r * plan.xstride + (int64_t)kk * kGroupLine];
            Q += v;
            cbase += r < plan.dx_rank ? v : 0ull;
        }
    }
    qmax = block_max_u64(qmax, s_u);
    block_sum2_u64(Q, cbase, s_red);
    const uint64_t Nr = plan.n_global ? plan.n_global : (uint64_t)N;
    const double ratio = Q ? wsmc_u64_to_d(Nr) / wsmc_u64_to_d(Q) : 0.0;
    if (ovf_chunks(qmax, ratio) == 0) return;   // no tile owns more than its first chunk

    const int per = (ntiles + kScanBlock - 1) / kScanBlock;
    const int b0 = th * per < ntiles ? th * per : ntiles;
    const int b1 = b0 + per < ntiles ? b0 + per : ntiles;
    u64 qs = 0, ns = 0;
    for (int b = b0; b < b1; ++b) {
        const u64 qb = plan.tilep[(int64_t)b * kPart];
        qs += qb;
        ns += (u64)ovf_chunks(qb, ratio);
    }
    u64 qtot, ntasks;
    const u64 qpre = block_excl_scan_u64<kScanBlock / 64>(qs, s_u, &qtot);
    const u64 npre = block_excl_scan_u64<kScanBlock / 64>(ns, s_u, &ntasks);
    // the plan goes to LDS: nothing per thread stays live across the chunk fills (their
    // registers bound the whole kernel's occupancy, the tile blocks' included)
    __shared__ uint32_t s_npre[kScanBlock], s_ns[kScanBlock];
    __shared__ u64 s_c0[kScanBlock];
    s_npre[th] = (uint32_t)npre;
    s_ns[th] = (uint32_t)ns;
    s_c0[th] = cbase + qpre;
    const u64 Qu = ((u64)__builtin_amdgcn_readfirstlane((int)(Q >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)Q);
    const uint32_t nt = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ntasks);
    for (uint32_t o = (uint32_t)(t - ntiles); o < nt; o += kOverflowBlocks) {
        const uint32_t n0_ = s_npre[th], k_ = s_ns[th];
        if (o >= n0_ && o < n0_ + k_) {            // exactly one thread owns task o
            u64 c = s_c0[th];
            uint32_t n0 = n0_;
            const int per_ = (ntiles + kScanBlock - 1) / kScanBlock;
            const int bb0 = th * per_ < ntiles ? th * per_ : ntiles;
            const int bb1 = bb0 + per_ < ntiles ? bb0 + per_ : ntiles;
            for (int b = bb0; b < bb1; ++b) {
                const u64 qb = plan.tilep[(int64_t)b * kPart];
                const uint32_t k = (uint32_t)ovf_chunks(qb, ratio);
                if (o < n0 + k) {
                    s_task[0] = (u64)b;
                    s_task[1] = 1 + (o - n0);
                    s_task[2] = c;
                    break;
                }
                n0 += k;
                c += qb;
            }
        }
        __syncthreads();
        const int b = __builtin_amdgcn_readfirstlane((int)s_task[0]);
        const int j = __builtin_amdgcn_readfirstlane((int)s_task[1]);
        const u64 off = ((u64)__builtin_amdgcn_readfirstlane((int)(s_task[2] >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s_task[2]);
        fill_chunk<0, QW>(N, b, j, Qu, off, plan, opx, qbuf, anc, sh, wq, ms);   // ends with a barrier
    }
}

// Lazy genealogy: bring stale columns up to date through the Resample log (ColumnStore's
// per-resample gathers, src/stores.jl:105-128, composed). Per particle i: a = i, then for
// each entry from the newest back (a = anc[a] where that Resample resampled) the columns
// whose values predate the entries applied so far read src[a]. Rows are monotone
// (stratified / systematic / sorted multinomial), so the gathers stay nearly coalesced.
// The walk is a chain of dependent loads (the entry of each row at the lineage so far), so
// its speed is the number of chains in flight: P = 2 particles a thread (two chains, 16-B
// stores of the outputs; N even, 16-B aligned outputs) keeps a 1M population resident in one
// round of waves, and each level's entry is loaded before that level's column gathers (every
// row exists; the entry is used only if its Resample resampled), so a level costs one memory
// latency, not two.
template <int P>
__global__ __launch_bounds__(kBlock) void k_lazy_trace(TraceArgs t, int64_t N) {
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * P;
    // every level's decision up front, one per lane, before any lane leaves (ballots: a
    // decision read inside the walk is a vector load the next level waits for, together with
    // every store in flight)
    const TraceArgs* T = (const TraceArgs*)(const char*)__builtin_amdgcn_kernarg_segment_ptr();
    const int lane = threadIdx.x & 63;
    static_assert(kTraceLev <= 128, "two decision words");
    const u64 rs0 = __ballot(lane < t.nlev && T->decs[lane]->resampled);
    const u64 rs1 = __ballot(lane + 64 < t.nlev && T->decs[lane + 64]->resampled);
    if (i0 >= N) return;
    if (i0 == 0)   // the columns' new fronts into the device pointer table
        for (int c = 0; c < t.ncomp; ++c)
            if (t.comp[c].col >= 0) t.tab[t.comp[c].col] = t.comp[c].dst;
    int64_t a[P];
    if (t.a_in) {
        if constexpr (P == 2) {
            const int2 v = *reinterpret_cast<const int2*>(t.a_in + i0);
            a[0] = v.x;
            a[1] = v.y;
        } else {
            a[0] = t.a_in[i0];
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; ++p) a[p] = i0 + p;
    }
    int32_t nx[P];
#pragma unroll
    for (int p = 0; p < P; ++p) nx[p] = t.nlev > 0 ? t.rows[0][a[p]] : 0;
    int k = 0;
    for (int lev = 0; lev < t.nlev; ++lev) {
        if (((lev < 64 ? rs0 : rs1) >> (lev & 63)) & 1)
#pragma unroll
            for (int p = 0; p < P; ++p) a[p] = nx[p];
        if (lev + 1 < t.nlev)
#pragma unroll
            for (int p = 0; p < P; ++p) nx[p] = t.rows[lev + 1][a[p]];
        for (; k < t.ncomp && t.comp[k].level == lev + 1; ++k) {
            const double* src = t.comp[k].src;
            if constexpr (P == 2) {
                *reinterpret_cast<d2*>(t.comp[k].dst + i0) = d2{src[a[0]], src[a[1]]};
            } else {
                t.comp[k].dst[i0] = src[a[0]];
            }
        }
    }
    if (t.a_out) {
        if constexpr (P == 2) {
            *reinterpret_cast<int2*>(t.a_out + i0) = int2{(int)a[0], (int)a[1]};
        } else {
            t.a_out[i0] = (int32_t)a[0];
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_gather(double* __restrict__ dst, const double* __restrict__ src,
                                                   const int32_t* __restrict__ anc, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    dst[i] = src[anc[i]];
}

// the gated weight reset: four weights a thread, 16-B stores (w is 16-B aligned)
__global__ __launch_bounds__(kBlock) void k_fill_weights(double* w, const Decision* dec, int64_t N, MaxSlots* ms) {
    const int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (!dec->resampled) return;
    const double m = dec->mean;
    // the max of N equal weights, in k_rs_max's encoding and slots (slot 0, the rest zero)
    if (ms && blockIdx.x == 0 && threadIdx.x < kSlots) ms->v[threadIdx.x][0] = threadIdx.x == 0 ? wsmc_ord_enc(m) : 0ull;
    if (i >= N) return;
    if (i + 4 <= N) {
        *reinterpret_cast<d2*>(w + i) = d2{m, m};
        *reinterpret_cast<d2*>(w + i + 2) = d2{m, m};
    } else {
        for (int64_t k = i; k < N; ++k) w[k] = m;
    }
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
    double lgw[4];           // log(hi - lo) of a bounded interval (host-evaluated), else 0
    int32_t use_ex;          // analysis moments: values are operand expressions (identity transform)
    wsmc_operand ex[4];
};
// targets one lazy Resample behind (bit k of mask: target k read through anc when dec resampled)

// one block: canonical combine of tile partials; pass 1 -> mom[0..d) = mean, mom[8] = S0;
// pass 2 -> mom[16..16+d*d) = lambda*Sigma (zeros -> min_step), mom[32..32+d*d) = chol
__device__ __forceinline__ void moments_final_block(const double* tilepart, int64_t ntiles, int d, int pass,
                                                    double min_step, double* mom, int32_t* flag, int raw,
                                                    double* lds4, double* tot) {
    const int nv = pass == 1 ? 1 + d : d * (d + 1) / 2;
    for (int v = 0; v < nv; ++v) {
        double acc = 0.0;
        for (int64_t b = threadIdx.x; b < ntiles; b += kBlock) acc = acc + tilepart[(int64_t)v * ntiles + b];
        const double s = block_sum_canon(acc, lds4);
        if (threadIdx.x == 0) tot[v] = s;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int v = 0; v < nv; ++v) mom[48 + v] = tot[v];   // raw shard totals (sharded moves combine them)
    if (raw == 2) return;                                // sharded: the host combines and factorises
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
    if (raw) {   // analysis moments: the weighted covariance itself
        for (int k = 0; k < d * d; ++k) mom[16 + k] = S[k];
        return;
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

// pass 1: values {e, e*z_k};  pass 2: values {(e*(z_a-mean_a))*(z_b-mean_b), a <= b}
// written as canonical tile partials tilepart[v * ntiles + tile]. D = d (1..4), a template
// parameter so every per-particle array is unrolled into registers (the same operations in the
// same order as a runtime d); EX: the values are operand expressions (analysis moments)
template <int D, bool EX>
__global__ __launch_bounds__(kBlock) void k_moments(const double* __restrict__ w, const MaxSlots* ms,
                                                    double* const* cols, MomArgs ma, int pass,
                                                    const double* mom, int64_t N, int64_t ntiles,
                                                    double* tilepart) {
    constexpr int d = D;
    __shared__ double lds4[4];
    const double M = wave_slots_max(ms);
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
#pragma unroll
            for (int k = 0; k < d; ++k)
                z[k] = EX ? wsmc_operand_eval(&ma.ex[k], cols, N, i, nullptr)
                          : wsmc_to_unc(cols[ma.tcol[k]][i], ma.lo[k], ma.hi[k]);
            if (pass == 1) {
                vals[0] = e;
#pragma unroll
                for (int k = 0; k < d; ++k) vals[1 + k] = e * z[k];
            } else {
                int v = 0;
#pragma unroll
                for (int a = 0; a < d; ++a)
#pragma unroll
                    for (int b = a; b < d; ++b) vals[v++] = (e * (z[a] - mean[a])) * (z[b] - mean[b]);
            }
        }
#pragma unroll
        for (int v = 0; v < 10; ++v) acc[v] = acc[v] + vals[v];
    }
#pragma unroll
    for (int v = 0; v < 10; ++v) {
        if (v >= nv) break;
        const double s = block_sum_canon(acc[v], lds4);
        if (threadIdx.x == 0) tilepart[(int64_t)v * ntiles + blockIdx.x] = s;
    }
}

// Sharded autoRW: the ranks' raw moment totals, all-gathered as `stride` u64
// words per rank (the bits of the doubles), summed in rank order; pass 1 -> the means and S0,
// pass 2 -> min_step, 2.38/sqrt(d), Cholesky (not PD -> flag): the host combine's arithmetic,
// on the device (no host round trip per pass).
__global__ void k_autorw_combine(const u64* __restrict__ xchg, int world, int stride, int d, int pass,
                                 double min_step, double* mom, int32_t* flag) {
    if (threadIdx.x != 0) return;
    auto total = [&](int v) {
        double acc = 0.0;
        for (int g = 0; g < world; ++g) {
            const double x = __builtin_bit_cast(double, xchg[(int64_t)g * stride + v]);
            acc = g == 0 ? x : acc + x;
        }
        return acc;
    };
    if (pass == 1) {
        const double S0 = total(0);
        for (int k = 0; k < d; ++k) mom[k] = total(1 + k) / S0;
        mom[8] = S0;
        return;
    }
    const double S0 = mom[8];
    double S[16], L[16];
    int v = 0;
    for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b, ++v) {
            const double cv = total(v) / S0;
            S[a * d + b] = cv;
            S[b * d + a] = cv;
        }
    const double lam = 2.38 / wsmc_sqrt((double)d);
    for (int k = 0; k < d * d; ++k) {
        if (S[k] == 0.0) S[k] = min_step;
        S[k] = lam * S[k];
    }
    const int ok = wsmc_cholesky(S, L, d);
    for (int k = 0; k < 16; ++k) mom[32 + k] = k < d * d ? L[k] : 0.0;
    if (!ok) flag[0] = 1;
}

__global__ __launch_bounds__(kBlock) void k_moments_final(const double* tilepart, int64_t ntiles, int d,
                                                          int pass, double min_step, double* mom,
                                                          int32_t* flag, int raw) {
    __shared__ double lds4[4];
    __shared__ double tot[10];
    moments_final_block(tilepart, ntiles, d, pass, min_step, mom, flag, raw, lds4, tot);
}

// ---- autoRW in one pass (include/wsmc_math.h wsmc_autorw_factor) ------------------------
// the pivot: the unconstrained values of the population's particle 0 (a sharded run passes
// rank 0's, all-gathered, as the bits of doubles in pv; nullptr: this context's particle 0)
template <int D>
__device__ __forceinline__ void autorw_pivot(double* const* cols, const MomArgs& ma, const u64* pv, double (&p)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k)
        p[k] = pv ? wsmc_bits2d(pv[k]) : wsmc_to_unc(cols[ma.tcol[k]][0], ma.lo[k], ma.hi[k]);
}
// the canonical tile partials tilepart[v * ntiles + tile] of {e, e d_k, (e d_a) d_b (a <= b)}
// with e = exp(w - M), d = z - pivot: the same per-thread order, butterfly and tile order as
// k_moments, one pass
template <int D>
__global__ __launch_bounds__(kBlock) void k_moments1(const double* __restrict__ w, const MaxSlots* ms,
                                                     double* const* cols, MomArgs ma, const u64* pv, int64_t N,
                                                     int64_t ntiles, double* tilepart, const Decision* wreset,
                                                     const Decision* gate, MomLag lg, MomZero z) {
    constexpr int d = D, NV = 1 + D + D * (D + 1) / 2;
    __shared__ double lds4[4];
    // the Move block's flag words and accepted counters, zeroed here rather than by two memset
    // launches (the combine and the Move kernel, which use them, run after this kernel)
    if (blockIdx.x == 0) {   // 4 moves x 64 count slots: one a thread
        if (z.count) *acc_slot(z.count, (int)threadIdx.x / kAccSlots, threadIdx.x) = 0;
        if (z.flag && threadIdx.x < 4) z.flag[threadIdx.x] = 0;
    }
    if (gate && !gate->resampled) return;   // a gated Move that does not run
    const double M = wave_slots_max(ms);
    // a fused Resample's weight reset still pending (the next Observe applies it): the
    // weights are its log-mean, all equal (the max slots already hold it)
    const bool reset = wreset && wreset->resampled;
    // the log / exp tables from LDS copies for the 3- and 4-target passes when they evaluate
    // them per particle (bounded targets, weights not reset): C5's 4-target pass, 154.3 ->
    // 152.1 ms a run on one box; C3's 2-target pass measured 3 % slower with the copy's LDS
    // and barrier in the kernel, so it keeps the cached gathers (uniform branch); the 1-target
    // pass with the copies measured even (C5 143.8 ms either way, round 5)
#ifndef WSMC_MOM_LDS_TABLES   // 0: the cached gathers everywhere, for comparison
#define WSMC_MOM_LDS_TABLES 1
#endif
    constexpr bool kLds = WSMC_MOM_LDS_TABLES && D >= 3;
    __shared__ double s_logtab[kLds ? 2 * WSMC_LOG_TABLE_N : 1];
    __shared__ uint64_t s_exptab[kLds ? 2 * WSMC_EXP_TABLE_N : 1];
    if constexpr (kLds) {
        bool bnd = false;
#pragma unroll
        for (int k = 0; k < D; ++k) bnd = bnd || wsmc_isfinite(ma.lo[k]) || wsmc_isfinite(ma.hi[k]);
        if (bnd || !reset) {
            const double* lt = wsmc_log_table();
            const uint64_t* et = wsmc_exp_table();
            for (int k = (int)threadIdx.x; k < 2 * WSMC_LOG_TABLE_N; k += kBlock) s_logtab[k] = lt[k];
            for (int k = (int)threadIdx.x; k < 2 * WSMC_EXP_TABLE_N; k += kBlock) s_exptab[k] = et[k];
            __syncthreads();
        }
    }
    // read only when filled: without bounds to_unc takes no log, with the reset no exp is taken
    const double* logtab = kLds ? (const double*)s_logtab : wsmc_log_table();
    const uint64_t* exptab = kLds ? (const uint64_t*)s_exptab : wsmc_exp_table();
    // all equal: one exp for the block (the same bits every particle's would give)
    const double er = reset ? wsmc_exp(wreset->mean - M) : 0.0;
    // targets one lazy Resample behind (lg.mask): read through its ancestors, gated by its
    // decision (the values the trace would have gathered)
    const int lmask = (lg.anc && lg.dec->resampled) ? lg.mask : 0;
    // the column pointers come from a device table: cast to the global address space, so the
    // gathers are global loads (a generic pointer's flat loads also count in lgkmcnt)
    typedef const double __attribute__((address_space(1)))* gdp_t;
    typedef const int32_t __attribute__((address_space(1)))* gip_t;
    gdp_t tp[D];
#pragma unroll
    for (int k = 0; k < d; ++k) tp[k] = (gdp_t)cols[ma.tcol[k]];
    const gip_t lanc = (gip_t)lg.anc;
    const gdp_t gw = (gdp_t)w;
    double p[4];
    if (pv) {
        autorw_pivot<D>(cols, ma, pv, p);
    } else {
        const int64_t i0 = lmask ? (int64_t)lg.anc[0] : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = k < d ? wsmc_to_unc(tp[k][(lmask >> k) & 1 ? i0 : 0], ma.lo[k], ma.hi[k]) : 0.0;
    }
    const int64_t base = (int64_t)blockIdx.x * kTile;
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    // the tile's loads in chunks of CH items (a few memory latencies per thread, not kItems in
    // a row; CH bounded so the loaded values stay in registers), then the canonical per-item
    // accumulation
#ifndef WSMC_MOM_CH
#define WSMC_MOM_CH 0
#endif
    // measured (tools/ab.sh, round 5): twice these (8, 8, 4) slower on C3 and C5 (1.02 / 0.96 ms,
    // 162 / 156 ms: the registers cost more waves than the extra loads in flight gain); half of
    // them (4, 2, 1: WSMC_MOM_CH=2) even (0.93 / 0.93 ms, 155.0 / 155.5 ms)
    constexpr int CH = WSMC_MOM_CH == 2 ? (D <= 1 ? 4 : (D == 2 ? 2 : 1)) : (D <= 1 ? 8 : (D == 2 ? 4 : 2));
    static_assert(kItems % CH == 0, "chunking");
#pragma unroll 1
    for (int j0 = 0; j0 < kItems; j0 += CH) {
    double xv[CH][D], wv[CH];
    int32_t ai[CH];
    // every load of the chunk unconditional (an index past N reads particle N - 1, unused), so
    // they issue back to back with one wait: a load under its own `i < N` branch waited for
    // each in turn
    if (lmask) {   // uniform: one branch around the chunk's ancestor loads
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int64_t i = base + (int64_t)(j0 + c) * kBlock + threadIdx.x;
            ai[c] = lanc[i < N ? i : N - 1];
        }
    } else {
#pragma unroll
        for (int c = 0; c < CH; ++c) ai[c] = 0;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int64_t i = base + (int64_t)(j0 + c) * kBlock + threadIdx.x;
        const int64_t ic = i < N ? i : N - 1;
        wv[c] = reset ? 0.0 : gw[ic];
#pragma unroll
        for (int k = 0; k < d; ++k) xv[c][k] = tp[k][(lmask >> k) & 1 ? (int64_t)ai[c] : ic];
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int j = j0 + c;
        const int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
        double vals[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) vals[v] = 0.0;
        if (i < N) {
            const double e = reset ? er : wsmc_exp_t(wv[c] - M, exptab);
            double dz[4];
#pragma unroll
            for (int k = 0; k < d; ++k) dz[k] = wsmc_to_unc_t(xv[c][k], ma.lo[k], ma.hi[k], logtab) - p[k];
            vals[0] = e;
#pragma unroll
            for (int k = 0; k < d; ++k) vals[1 + k] = e * dz[k];
            int v = 1 + d;
#pragma unroll
            for (int a = 0; a < d; ++a)
#pragma unroll
                for (int b = a; b < d; ++b) vals[v++] = (e * dz[a]) * dz[b];
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = acc[v] + vals[v];
    }
    }
    __shared__ double ldsn[NV][4];
    double tot[NV];
    block_sum_canon_n<NV>(acc, ldsn, tot);
    if (threadIdx.x == 0)
#pragma unroll
        for (int v = 0; v < NV; ++v) tilepart[(int64_t)v * ntiles + blockIdx.x] = tot[v];
}
// a thread's strided sums of the tile partials, value by value in the combine's order (tiles
// th, th + kBlock, ... ascending), the loads of four tiles issued before their adds (measured:
// C5's 4-target combine 15.2 -> 14.8 us a launch, the others 2-3 % less)
template <int NV>
__device__ __forceinline__ void combine_partials(const double* __restrict__ tilepart, int64_t ntiles,
                                                 double (&acc)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    int64_t b = threadIdx.x;
    for (; b + 3 * kBlock < ntiles; b += 4 * kBlock) {
        double x[4][NV];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) x[u][v] = tilepart[(int64_t)v * ntiles + b + u * kBlock];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[v] = acc[v] + x[u][v];
    }
    for (; b < ntiles; b += kBlock)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] = acc[v] + tilepart[(int64_t)v * ntiles + b];
}
// one block: the canonical combine of the tile partials (k_moments_final's order); raw: the
// totals to mom[48..] (a sharded run all-gathers them), else the factor: mom[16..] the scaled
// covariance, mom[32..] its Cholesky factor, flag[0] = 1 if not positive definite
template <int D>
__global__ __launch_bounds__(kBlock) void k_autorw_final(const double* tilepart, int64_t ntiles, double min_step,
                                                         double* mom, int32_t* flag, int raw, const Decision* gate) {
    constexpr int NV = 1 + D + D * (D + 1) / 2;
    __shared__ double lds4[4];
    __shared__ double tot[NV];
    if (gate && !gate->resampled) return;
    // every value's partials in one walk (each value's sum in its own order), then the sums
    double acc[NV];
    combine_partials<NV>(tilepart, ntiles, acc);
    {
        __shared__ double ldsn[NV][4];
        double t[NV];
        block_sum_canon_n<NV>(acc, ldsn, t);
        if (threadIdx.x == 0)
#pragma unroll
            for (int v = 0; v < NV; ++v) tot[v] = t[v];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (raw) {
        for (int v = 0; v < NV; ++v) mom[48 + v] = tot[v];
        return;
    }
    double S[16], L[16];
    const int ok = wsmc_autorw_factor(tot, D, min_step, S, L);
    for (int k = 0; k < D * D; ++k) {
        mom[16 + k] = S[k];
        mom[32 + k] = L[k];
    }
    if (!ok) flag[0] = 1;
}
// sharded: this rank's max word and its particle 0's unconstrained values (rank 0's are the
// pivot), 1 + d words
template <int D>
__global__ void k_autorw_publish(const MaxSlots* ms, double* const* cols, MomArgs ma, u64* out) {
    const u64 m = wave_max_u64(ms->v[threadIdx.x & 63][0]);
    if (threadIdx.x != 0) return;
    out[0] = m;
    double p[4];
    autorw_pivot<D>(cols, ma, nullptr, p);
    for (int k = 0; k < D; ++k) out[1 + k] = wsmc_d2bits(p[k]);
}
// sharded: the ranks' totals summed in rank order, then the factor (k_autorw_final's arithmetic)
__global__ void k_autorw_combine1(const u64* __restrict__ xchg, int world, int stride, int d, double min_step,
                                  double* mom, int32_t* flag) {
    if (threadIdx.x != 0) return;
    const int nv = 1 + d + d * (d + 1) / 2;
    double tot[15];
    for (int v = 0; v < nv; ++v) {
        double acc = 0.0;
        for (int g = 0; g < world; ++g) {
            const double x = __builtin_bit_cast(double, xchg[(int64_t)g * stride + v]);
            acc = g == 0 ? x : acc + x;
        }
        tot[v] = acc;
    }
    double S[16], L[16];
    const int ok = wsmc_autorw_factor(tot, d, min_step, S, L);
    for (int k = 0; k < 16; ++k) mom[32 + k] = k < d * d ? L[k] : 0.0;
    if (!ok) flag[0] = 1;
}

// its band half-width and estimate, for the device check of the bound
__global__ void k_debug_log_screen(const double* u, int64_t n, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double L = (double)__builtin_amdgcn_logf((float)u[i]) * 0.69314718055994530942;
    out[2 * i] = L;
    out[2 * i + 1] = wsmc_log(u[i]);
}

hipError_t launch_debug_log_screen(hipStream_t s, const double* u, int64_t n, double* out) {
    hipLaunchKernelGGL(k_debug_log_screen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, n, out);
    return hipGetLastError();
}

// Move (src/transformers.jl:588-623). scache carries each particle's score from its last
// move (the fold is a left-to-right sum, so continuing it over the terms appended since
// [cache_from, nterms) gives the same bits as refolding); cache_from < 0 = refold.
// A non-PD autoRW covariance (flag set by the moments pass) skips the move untouched,
// as the reference throws before modifying anything.
__global__ __launch_bounds__(kBlock) void k_move(const wsmc_term* tape, int32_t nterms, int32_t depth,
                                                 double* const* cols, MomArgs ma, int d, int bounded,
                                                 const double* Lm, uint64_t seed, uint64_t op_prop,
                                                 uint64_t op_acc, int64_t goff, int64_t N, u64* accepted,
                                                 const int32_t* flag, double* scache, int32_t cache_from) {
    __shared__ u64 lds4[4];
    if (flag && flag[0]) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    u64 acc = 0;
    if (i < N) {
        double xi[4] = {0.0, 0.0, 0.0, 0.0}, dz[4];
        for (int k = 0; k < d; k += 2)   // one Box-Muller pair per two targets (wsmc_normal_k's values)
            wsmc_normal_pair(wsmc_rng_block(seed, op_prop, (uint64_t)(goff + i), (uint32_t)(k >> 1)), &xi[k], &xi[k + 1]);
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
            double xn = x + dz[k];
            if (bounded) {
                double dj;
                xn = wsmc_bounded_step(x, dz[k], ma.lo[k], ma.hi[k], ma.lgw[k], wsmc_isfinite(ma.lo[k]),
                                       wsmc_isfinite(ma.hi[k]), &dj);
                lpr = lpr + dj;
            }
            ov.col[k] = ma.tcol[k];
            ov.val[k] = xn;
        }
        const double s_old = cache_from >= 0
                                 ? wsmc_fold_from(scache[i], tape, cache_from, nterms, depth, cols, N, i, nullptr)
                                 : wsmc_fold(tape, nterms, depth, cols, N, i, nullptr);
        const double s_new = wsmc_fold(tape, nterms, depth, cols, N, i, &ov);
        const double u = wsmc_uniform_k(seed, op_acc, (uint64_t)(goff + i), 0);
        if (move_accept(u, (lpr + s_new) - s_old)) {   // strict; NaN rejects (src/transformers.jl:615)
            for (int k = 0; k < d; ++k) cols[ma.tcol[k]][i] = ov.val[k];
            acc = 1;
        }
        scache[i] = acc ? s_new : s_old;
    }
    acc = block_sum_u64(acc, lds4);
    if (threadIdx.x == 0 && acc) atomicAdd(acc_slot(accepted, 0, blockIdx.x), acc);
}

// The same Move over a compiled tape: the host renumbers every (column, component) the
// fold reads into slots (the targets first), each thread loads its slot values once — all
// loads independent, in flight together — into LDS, and the shared fold (include/
// wsmc_terms.h, unchanged arithmetic) reads them through LDS slot pointers. The generic
// fold's per-term chain term -> column pointer -> global value becomes LDS reads.
// K particles per thread: the program is walked once per thread for K particles, so the
// interpreter's serial chain of scalar term loads and branches (what the one-particle
// kernel waits on: VALU active 10%) is shared; each particle keeps its own accumulator and
// log memo, so every fold is the same left fold as wsmc_fold / wsmc_fold_from.
//
// The fold runs a segment program (FoldProgram): one-term segments go through the shared
// term evaluator; a run segment evaluates its per-particle invariants once and then only the
// per-term arithmetic, its constants read as wave-uniform scalars. Every term's arithmetic is
// wsmc_term_logpdf_m's (the same operations in the same order, the same log memo), so the
// fold is bit-identical to the term-by-term one.
// LEAN (a template flag, chosen by the host from the program): 0 = any term; 1 = runs and
// scalar Normal/HalfNormal/Uniform one-term segments only (wsmc_scalar_term_logpdf_m: the
// same arithmetic), no oscillator; 2 = the same with oscillator runs. The lean variants carry
// no code for the other families, so they need far fewer registers (occupancy: the fold is
// latency-bound).
template <int K, int LEAN = 0>
__device__ __forceinline__ void fold_seg(double (&s)[K], const wsmc_term* tape, const FoldSeg* segs, int32_t nseg,
                                         const double* __restrict__ cst, double* const* cols, const int (&ix)[K],
                                         const bool (&ok)[K]) {
    wsmc_logmemo lm[K];
#pragma unroll
    for (int p = 0; p < K; ++p) lm[p] = wsmc_logmemo{0, 0.0, 0.0, 0};
    for (int32_t g = 0; g < nseg; ++g) {
        const FoldSeg sg = segs[g];
        const wsmc_term* tp = &tape[sg.tmpl];
        if (LEAN != 1 && sg.kind == kSegNormalOsc) {
            // Normal(A exp(-gamma t) cos(omega t + phi), sigma) observed at y, over (t, y) pairs
            double A[K], om[K], ga[K], ph[K], rh[K], nc[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                A[p] = wsmc_operand_eval(&tp->dist.mu[0], cols, 0, ix[p], nullptr);
                om[p] = wsmc_operand_eval(&tp->dist.mu[1], cols, 0, ix[p], nullptr);
                ga[p] = wsmc_operand_eval(&tp->dist.mu[2], cols, 0, ix[p], nullptr);
                ph[p] = wsmc_operand_eval(&tp->dist.mu[3], cols, 0, ix[p], nullptr);
                if (sg.soff >= 0) {   // a constant sigma: its pair from the host (uniform branch)
                    nc[p] = cst[sg.soff];
                    rh[p] = cst[sg.soff + 1];
                } else {
                    wsmc_normal_scale(&lm[p], wsmc_operand_eval(&tp->dist.scale, cols, 0, ix[p], nullptr), &nc[p],
                                     &rh[p]);
                }
            }
            // the mean by rotation (wsmc_osc_rolled's operations): a block's first term (m = 0)
            // is the direct phasor, each next term of the block one complex multiply by R; a
            // fold entering a block mid-way (the carried score's continuation) anchors and rolls
            // there, so every term has the bits of the term-by-term evaluation
            // over the segment's rotation runs (t_a, d, m, n, y_0 .. y_{n-1}; csrc/wsmc_mv.h)
            const double* c = cst + sg.coff;
            double zr[K], zi[K], rr[K], ri[K];
            double r_d = WSMC_NAN;
            for (int32_t left = sg.count; left > 0;) {   // uniform
                const double ta = c[0], dl = c[1];
                const int32_t m = osc_run_int(c[2]);
                const int32_t n0 = osc_run_int(c[3]), n = n0 < 1 ? 1 : n0;
                const double* yv = c + 4;
                c = yv + n;
                left -= n;
                if ((m > 0 || n > 1) && wsmc_d2bits(dl) != wsmc_d2bits(r_d)) {   // uniform branch
#pragma unroll
                    for (int p = 0; p < K; ++p) wsmc_osc_step(dl, om[p], ga[p], &rr[p], &ri[p]);
                    r_d = dl;
                }
                for (int32_t k = 0; k < n; ++k) {
                    const double y = yv[k];
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        if (k > 0) {
                            wsmc_osc_rotate(&zr[p], &zi[p], rr[p], ri[p]);
                        } else {
                            wsmc_osc_anchor(ta, A[p], om[p], ga[p], ph[p], &zr[p], &zi[p]);
                            for (int j = 0; j < m; ++j) wsmc_osc_rotate(&zr[p], &zi[p], rr[p], ri[p]);
                        }
                    }
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        if (!ok[p]) continue;
                        s[p] = s[p] + wsmc_normal_lh((y - zr[p]) * rh[p], nc[p]);
                    }
                }
            }
            continue;
        }
        if (sg.kind == kSegNormalAff) {
            // Normal(c0 + coef0 col0 + coef1 col1, sigma) observed at y, over (c0, coef0, coef1, y)
            const wsmc_operand& m = tp->dist.mu[0];
            const bool h0 = m.col[0] >= 0, h1 = m.col[1] >= 0;
            double v0[K], v1[K], rh[K], nc[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                v0[p] = h0 ? cols[m.col[0]][ix[p]] : 0.0;
                v1[p] = h1 ? cols[m.col[1]][ix[p]] : 0.0;
                if (sg.soff >= 0) {
                    nc[p] = cst[sg.soff];
                    rh[p] = cst[sg.soff + 1];
                } else {
                    wsmc_normal_scale(&lm[p], wsmc_operand_eval(&tp->dist.scale, cols, 0, ix[p], nullptr), &nc[p],
                                     &rh[p]);
                }
            }
            const double* c = cst + sg.coff;
            const bool any = sg.count > 0;   // the next term's constants, loaded ahead
            double q0 = any ? c[0] : 0.0, q1 = any ? c[1] : 0.0, q2 = any ? c[2] : 0.0, q3 = any ? c[3] : 0.0;
            for (int32_t k = 0; k < sg.count; ++k) {
                const double c0 = q0, a0 = q1, a1 = q2, y = q3;
                if (k + 1 < sg.count) {   // uniform
                    q0 = c[4 * k + 4];
                    q1 = c[4 * k + 5];
                    q2 = c[4 * k + 6];
                    q3 = c[4 * k + 7];
                }
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    if (!ok[p]) continue;
                    double mu = c0;
                    if (h0) mu = mu + a0 * v0[p];
                    if (h1) mu = mu + a1 * v1[p];
                    s[p] = s[p] + wsmc_normal_lh((y - mu) * rh[p], nc[p]);
                }
            }
            continue;
        }
        if (LEAN) {
            const double* pre = sg.soff >= 0 ? cst + sg.soff : nullptr;
#pragma unroll
            for (int p = 0; p < K; ++p)
                if (ok[p]) s[p] = s[p] + wsmc_scalar_term_logpdf_p(tp, cols, 0, ix[p], nullptr, &lm[p], pre);
            continue;
        }
#pragma unroll
        for (int p = 0; p < K; ++p)
            if (ok[p]) s[p] = s[p] + wsmc_term_logpdf_m(tp, cols, 0, ix[p], nullptr, &lm[p]);
    }
}

// The same Move over a compiled tape (slots; targets are slots 0..d-1), K particles per
// thread: slot values staged once in LDS ([slot][K * kBlock]), proposals in their own LDS
// rows so the s_new fold reads them through its own pointer table (no override lookups).
// a Move's slot values into LDS: loaded in chunks of 8 / K slots, every load of a chunk issued
// before its LDS stores (a rolled slot loop waited out one memory latency per slot: the stores
// may alias the generic slot pointers, so the compiler cannot hoist the next load)
template <int K>
__device__ __forceinline__ void stage_slots(double* sv, int W, const FoldSlots& fs, const int (&ix)[K],
                                            const int64_t (&gi)[K], const int64_t (&ai)[K], const bool (&ok)[K],
                                            int smask) {
    constexpr int C = 8 / K;
    for (int s0 = 0; s0 < fs.n; s0 += C) {
        double v[C][K];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int p = 0; p < K; ++p) {
                const int sl = s0 + c;
                v[c][p] = (sl < fs.n && ok[p]) ? fs.p[sl][(smask >> sl) & 1 ? ai[p] : gi[p]] : 0.0;
            }
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int p = 0; p < K; ++p)
                if (s0 + c < fs.n) sv[(s0 + c) * W + ix[p]] = v[c][p];
    }
}

template <int K, int LEAN>
__device__ __forceinline__ void move_c_body(const wsmc_term* ctape, const FoldSlots& fs, const MomArgs& ma, int d,
                                            int bounded, const double* Lm, uint64_t seed, uint64_t op_prop,
                                            uint64_t op_acc, int64_t goff, int64_t N, u64* accepted,
                                            const int32_t* flag, const MoveCarry& mc, int32_t cache_from,
                                            const FoldProgram& prog) {
    constexpr int W = K * kBlock;            // LDS row length
    extern __shared__ double sv[];           // [fs.n][W] current values, then [d][W] proposals
    __shared__ double* sp[kFoldSlots];
    __shared__ double* spn[kFoldSlots];
    __shared__ u64 lds4[4];
    if (flag && flag[0]) return;
    const int th = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * W;
    double* prop = sv + fs.n * W;
    if (th < fs.n) {
        sp[th] = sv + th * W;
        spn[th] = th < d ? prop + th * W : sv + th * W;
    }
    int ix[K];
    bool ok[K];
    int64_t gi[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        ix[p] = p * kBlock + th;
        gi[p] = base + ix[p];
        ok[p] = gi[p] < N;
    }
    stage_slots<K>(sv, W, fs, ix, gi, gi, ok, 0);
    double so[K], sn[K], lpr[K];
    const bool lag = mc.anc && mc.dec->resampled;
    const bool run = !mc.gate || mc.gate->resampled;   // a gated Move that does not run only carries
                                                       // its scores on over the new terms
#pragma unroll
    for (int p = 0; p < K; ++p) {
        so[p] = (ok[p] && cache_from >= 0) ? mc.in[lag ? (int64_t)mc.anc[gi[p]] : gi[p]] : 0.0;
        sn[p] = 0.0;
        lpr[p] = 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (!ok[p] || !run) continue;
        // the proposal's normals: one Box-Muller pair per two targets (wsmc_normal_k(k) is
        // component k & 1 of the pair of block k >> 1: the same values, half the work)
        double xi[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; k += 2)
            if (k < d) wsmc_normal_pair(wsmc_rng_block(seed, op_prop, (uint64_t)(goff + gi[p]), (uint32_t)(k >> 1)),
                                        &xi[k], &xi[k + 1]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k >= d) break;
            double dz = 0.0;
#pragma unroll
            for (int j = 0; j <= k; ++j) dz = dz + Lm[k * d + j] * xi[j];
            const double x = sv[k * W + ix[p]];
            double xn = x + dz;
            if (bounded) {
                double dj;
                xn = wsmc_bounded_step(x, dz, ma.lo[k], ma.hi[k], ma.lgw[k], wsmc_isfinite(ma.lo[k]),
                                       wsmc_isfinite(ma.hi[k]), &dj);
                lpr[p] = lpr[p] + dj;
            }
            prop[k * W + ix[p]] = xn;
        }
    }
    // s_old: the carried score continued over the new terms, or the full fold
    fold_seg<K, LEAN>(so, ctape, prog.seg_old, prog.nseg_old, prog.cst, sp, ix, ok);
#ifndef WSMC_ABL_NOFOLD
    if (run) fold_seg<K, LEAN>(sn, ctape, prog.seg_new, prog.nseg_new, prog.cst, spn, ix, ok);
#else
#pragma unroll
    for (int p = 0; p < K; ++p) sn[p] = -0.5 * prop[ix[p]] * prop[ix[p]];
#endif
    u64 acc = 0;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (!ok[p]) continue;
        if (!run) {
            mc.out[gi[p]] = so[p];
            continue;
        }
        const double u = wsmc_uniform_k(seed, op_acc, (uint64_t)(goff + gi[p]), 0);
        const bool a = move_accept(u, (lpr[p] + sn[p]) - so[p]);   // strict; NaN rejects (src/transformers.jl:615)
        if (a) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < d) fs.t[k][gi[p]] = prop[k * W + ix[p]];
            acc += 1;
        }
        mc.out[gi[p]] = a ? sn[p] : so[p];
    }
    acc = block_sum_u64(acc, lds4);
    if (threadIdx.x == 0 && acc) atomicAdd(acc_slot(accepted, 0, blockIdx.x), acc);
}
template <int K, int LEAN>
__global__ __launch_bounds__(kBlock) void k_move_c(const wsmc_term* ctape, FoldSlots fs, MomArgs ma, int d,
                                                   int bounded, const double* Lm, uint64_t seed, uint64_t op_prop,
                                                   uint64_t op_acc, int64_t goff, int64_t N, u64* accepted,
                                                   const int32_t* flag, MoveCarry mc, int32_t cache_from,
                                                   FoldProgram prog) {
    move_c_body<K, LEAN>(ctape, fs, ma, d, bounded, Lm, seed, op_prop, op_acc, goff, N, accepted, flag, mc,
                         cache_from, prog);
}
// the program in the kernel's arguments (ProgInline, the first argument: offset 0 of the
// kernarg segment): its templates, segments and constants are read in place through the
// segment pointer with scalar loads (naming the by-value argument would copy it to scratch)
template <int K, int LEAN>
__global__ __launch_bounds__(kBlock) void k_move_ci(ProgInline, FoldSlots fs, MomArgs ma, int d, int bounded,
                                                    const double* Lm, uint64_t seed, uint64_t op_prop,
                                                    uint64_t op_acc, int64_t goff, int64_t N, u64* accepted,
                                                    const int32_t* flag, MoveCarry mc, int32_t cache_from,
                                                    int32_t nseg_new, int32_t nseg_old) {
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    const int32_t* hdr = reinterpret_cast<const int32_t*>(ka);   // seg_off, cst_off, seg_old0
    const char* b = ka + offsetof(ProgInline, w);
    FoldProgram prog;
    prog.seg_new = reinterpret_cast<const FoldSeg*>(b + hdr[0]);
    prog.seg_old = prog.seg_new + hdr[2];
    prog.nseg_new = nseg_new;
    prog.nseg_old = nseg_old;
    prog.cst = reinterpret_cast<const double*>(b + hdr[1]);
    move_c_body<K, LEAN>(reinterpret_cast<const wsmc_term*>(b), fs, ma, d, bounded, Lm, seed, op_prop, op_acc, goff,
                         N, accepted, flag, mc, cache_from, prog);
}

// ---- a block of Moves in one pass (wsmc_move_block) ----------------------------------------
// Consecutive autoRW Moves on disjoint targets with one fold (the same target depth): each
// move's covariance reads only its own targets and the weights, which the earlier moves of
// the block leave alone, so one moments pass over the union of the targets serves them all
// (each move's totals are a sub-block of the union's: the same per-value arithmetic, order
// and tile combine as a pass over its targets alone), and one kernel runs the moves one after
// the other per particle — the later moves' folds see the earlier moves' accepted values and
// continue from their scores, as the sequential Moves do.
// The factors: move m's at mom[64 + 16 m ..]; flag[0] = 1 if one is not PD, flag[2] = the
// moves that run (those before the first non-PD one; 0 when an earlier failure is pending).
template <int D>
__global__ __launch_bounds__(kBlock) void k_autorw_final_blk(const double* tilepart, int64_t ntiles, MoveBlk mb,
                                                             double* mom, int32_t* flag, const Decision* gate) {
    constexpr int NV = 1 + D + D * (D + 1) / 2;
    __shared__ double lds4[4];
    __shared__ double tot[NV];
    if (gate && !gate->resampled) return;
    // every value's partials in one walk (each value's sum in its own order), then the sums
    double acc[NV];
    combine_partials<NV>(tilepart, ntiles, acc);
    {
        __shared__ double ldsn[NV][4];
        double t[NV];
        block_sum_canon_n<NV>(acc, ldsn, t);
        if (threadIdx.x == 0)
#pragma unroll
            for (int v = 0; v < NV; ++v) tot[v] = t[v];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int prior = flag[0];
    int nrun = mb.nm;
    for (int m = 0; m < mb.nm; ++m) {
        const int o = mb.off[m], dm = mb.off[m + 1] - o;
        double sub[15];
        sub[0] = tot[0];
        for (int k = 0; k < dm; ++k) sub[1 + k] = tot[1 + o + k];
        int v = 1 + dm;
        for (int a = 0; a < dm; ++a)
            for (int b = a; b < dm; ++b) {
                const int ua = o + a, ub = o + b;
                int pi = 0;   // (ua, ub) in the union's a <= b enumeration
                for (int x = 0; x < ua; ++x) pi += D - x;
                sub[v++] = tot[1 + D + pi + (ub - ua)];
            }
        double S[16], L[16];
        const int ok = wsmc_autorw_factor(sub, dm, mb.min_step[m], S, L);
        for (int k = 0; k < 16; ++k) mom[64 + 16 * m + k] = k < dm * dm ? L[k] : 0.0;
        if (!ok) {
            flag[0] = 1;
            nrun = m;
            break;
        }
    }
    flag[2] = prior ? 0 : nrun;
}
// the same with one moments pass per move (a union of more than 4 targets): move m's totals at
// tilepart + toff[m] * ntiles, each combined exactly as k_autorw_final<d_m> combines them
struct BlkOff {
    int32_t t[4];
};
__global__ __launch_bounds__(kBlock) void k_autorw_final_sep(const double* tilepart, int64_t ntiles, MoveBlk mb,
                                                             BlkOff toff, double* mom, int32_t* flag,
                                                             const Decision* gate) {
    __shared__ double lds4[4];
    __shared__ double tot[4][15];
    if (gate && !gate->resampled) return;
    for (int m = 0; m < mb.nm; ++m) {
        const int dm = mb.off[m + 1] - mb.off[m], nv = 1 + dm + dm * (dm + 1) / 2;
        const double* tp = tilepart + (int64_t)toff.t[m] * ntiles;
        double acc[15];
#pragma unroll
        for (int v = 0; v < 15; ++v) acc[v] = 0.0;
        for (int64_t b = threadIdx.x; b < ntiles; b += kBlock)
#pragma unroll
            for (int v = 0; v < 15; ++v)
                if (v < nv) acc[v] = acc[v] + tp[(int64_t)v * ntiles + b];
#pragma unroll
        for (int v = 0; v < 15; ++v) {
            if (v >= nv) break;
            const double s = block_sum_canon(acc[v], lds4);
            if (threadIdx.x == 0) tot[m][v] = s;
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int prior = flag[0];
    int nrun = mb.nm;
    for (int m = 0; m < mb.nm; ++m) {
        const int dm = mb.off[m + 1] - mb.off[m];
        double S[16], L[16];
        const int ok = wsmc_autorw_factor(tot[m], dm, mb.min_step[m], S, L);
        for (int k = 0; k < 16; ++k) mom[64 + 16 * m + k] = k < dm * dm ? L[k] : 0.0;
        if (!ok) {
            flag[0] = 1;
            nrun = m;
            break;
        }
    }
    flag[2] = prior ? 0 : nrun;
}

// BND = 0: no union target is bounded (the host checks mb.bnd), so the transforms' code is left
// out (with it the unrolled per-target bodies carry 2K copies of log / exp / log1p: code size)
template <int K, int LEAN, int BND = 1>
__device__ __forceinline__ void move_blk_body(const wsmc_term* ctape, const FoldSeg* seg_new, const FoldSeg* seg_old,
                                              const double* cst, int32_t nseg_new, int32_t nseg_old,
                                              const FoldSlots& fs, const MoveBlk& mb, const double* Lb,
                                              uint64_t seed, int64_t goff, int64_t N, u64* accepted,
                                              const int32_t* flag, const MoveCarry& mc, int32_t cache_from,
                                              const MomLag& lg, double** tab) {
    constexpr int W = K * kBlock;
    extern __shared__ double sv[];           // [fs.n][W] current values, then [D][W] proposals
    __shared__ double* sp[kFoldSlots];
    __shared__ double* spn[4][kFoldSlots];
    __shared__ u64 lds4[4];
    const int th = threadIdx.x;
    const int nm = mb.nm;
    double* prop = sv + fs.n * W;
    if (th < fs.n) {
        sp[th] = sv + th * W;
        for (int m = 0; m < nm; ++m)
            spn[m][th] = (th >= mb.off[m] && th < mb.off[m + 1]) ? prop + th * W : sv + th * W;
    }
    int ix[K];
    bool ok[K];
    int64_t gi[K], ai[K];
    // slots one lazy Resample behind read through its ancestors (gated by its decision), as
    // are the carried scores (MoveCarry)
    const int smask = (lg.anc && lg.dec->resampled) ? lg.mask : 0;
    const bool slag = mc.anc && mc.dec->resampled;
    const int32_t* arow = smask ? lg.anc : mc.anc;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        ix[p] = p * kBlock + th;
        gi[p] = (int64_t)blockIdx.x * W + ix[p];
        ok[p] = gi[p] < N;
        ai[p] = (ok[p] && (smask || slag)) ? (int64_t)arow[gi[p]] : gi[p];
    }
    stage_slots<K>(sv, W, fs, ix, gi, ai, ok, smask);
    double so[K], sn[K], lpr[K];
    int chg[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        so[p] = (ok[p] && cache_from >= 0) ? mc.in[slag ? ai[p] : gi[p]] : 0.0;
        chg[p] = 0;
    }
    const bool run = !mc.gate || mc.gate->resampled;
    const int nrun = run ? flag[2] : 0;   // the final's count (uniform)
    __syncthreads();
    fold_seg<K, LEAN>(so, ctape, seg_old, nseg_old, cst, sp, ix, ok);
    for (int m = 0; m < nrun; ++m) {
        const int o = mb.off[m], dm = mb.off[m + 1] - o;
        const double* Lm = Lb + 16 * m;
        u64 acc = 0;
#pragma unroll
        for (int p = 0; p < K; ++p) {
            sn[p] = 0.0;
            lpr[p] = 0.0;
            if (!ok[p]) continue;
            double xi[4] = {0.0, 0.0, 0.0, 0.0};
#ifndef WSMC_ABL_NODRAW   // ablation builds only (tools/build_variant.sh): what each part of the block costs
#pragma unroll
            for (int k = 0; k < 4; k += 2)
                if (k < dm)
                    wsmc_normal_pair(wsmc_rng_block(seed, mb.op_prop[m], (uint64_t)(goff + gi[p]), (uint32_t)(k >> 1)),
                                     &xi[k], &xi[k + 1]);
#else
            xi[0] = xi[1] = xi[2] = xi[3] = 0.01 * (double)(gi[p] & 7);
#endif
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k >= dm) break;
                const int u = o + k;
                double dz = 0.0;
#pragma unroll
                for (int jj = 0; jj <= k; ++jj) dz = dz + Lm[k * dm + jj] * xi[jj];
                const double x = sv[u * W + ix[p]];
                const bool bd = BND && ((mb.bnd >> u) & 1);
                double xn = x + dz;
                if (bd) {
                    double dj;
                    xn = wsmc_bounded_step(x, dz, mb.lo[u], mb.hi[u], mb.lgw[u], wsmc_isfinite(mb.lo[u]),
                                           wsmc_isfinite(mb.hi[u]), &dj);
                    lpr[p] = lpr[p] + dj;
                }
                prop[u * W + ix[p]] = xn;
            }
        }
#ifndef WSMC_ABL_NOFOLD
        fold_seg<K, LEAN>(sn, ctape, seg_new, nseg_new, cst, spn[m], ix, ok);
#else
#pragma unroll
        for (int p = 0; p < K; ++p) sn[p] = -0.5 * prop[o * W + ix[p]] * prop[o * W + ix[p]];
#endif
#pragma unroll
        for (int p = 0; p < K; ++p) {
            if (!ok[p]) continue;
#ifndef WSMC_ABL_NOACC
            const double uu = wsmc_uniform_k(seed, mb.op_acc[m], (uint64_t)(goff + gi[p]), 0);
#else
            const double uu = 0.25 + 0.0625 * (double)(gi[p] & 7);
#endif
            const bool a = move_accept(uu, (lpr[p] + sn[p]) - so[p]);   // strict; NaN rejects (src/transformers.jl:615)
            if (a) {
                for (int u = o; u < o + dm; ++u) sv[u * W + ix[p]] = prop[u * W + ix[p]];
                chg[p] |= ((1 << dm) - 1) << o;
                acc += 1;
                so[p] = sn[p];
            }
        }
        if (accepted) {   // uniform
            acc = block_sum_u64(acc, lds4);
            if (th == 0 && acc) atomicAdd(acc_slot(accepted, m, blockIdx.x), acc);
        }
    }
    const int D = mb.off[nm];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (!ok[p]) continue;
        for (int u = 0; u < D; ++u)
            if (((mb.lag_targets | chg[p]) >> u) & 1) mb.tout[u][gi[p]] = sv[u * W + ix[p]];
        mc.out[gi[p]] = so[p];
    }
    if (mb.lag_targets && blockIdx.x == 0 && th == 0)   // the device column table follows the moved fronts
        for (int u = 0; u < D; ++u)
            if ((mb.lag_targets >> u) & 1) tab[mb.tcol[u]] = mb.tout[u];
}
// the program in the kernel's arguments (ProgInlineBlk first: offset 0 of the kernarg segment)
#ifndef WSMC_MOVE_WAVES
#define WSMC_MOVE_WAVES 1
#endif
#ifndef WSMC_BLK_K   // particles a thread of the unbounded lean block
#define WSMC_BLK_K 2
#endif
template <int K, int LEAN, int BND>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WSMC_MOVE_WAVES))) void k_move_blk(ProgInlineBlk, FoldSlots fs, MoveBlk mb, const double* Lb,
                                                     uint64_t seed, int64_t goff, int64_t N, u64* accepted,
                                                     const int32_t* flag, MoveCarry mc, int32_t cache_from,
                                                     int32_t nseg_new, int32_t nseg_old, MomLag lg, double** tab) {
    const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    const int32_t* hdr = reinterpret_cast<const int32_t*>(ka);
    const char* pb = ka + offsetof(ProgInlineBlk, w);
    const FoldSeg* seg_new = reinterpret_cast<const FoldSeg*>(pb + hdr[0]);
    move_blk_body<K, LEAN, BND>(reinterpret_cast<const wsmc_term*>(pb), seg_new, seg_new + hdr[2],
                           reinterpret_cast<const double*>(pb + hdr[1]), nseg_new, nseg_old, fs, mb, Lb, seed, goff,
                           N, accepted, flag, mc, cache_from, lg, tab);
}
// the program uploaded to device memory (too large for the arguments)
template <int K, int LEAN>
__global__ __launch_bounds__(kBlock) void k_move_blk_g(const wsmc_term* ctape, FoldProgram prog, FoldSlots fs,
                                                       MoveBlk mb, const double* Lb, uint64_t seed, int64_t goff,
                                                       int64_t N, u64* accepted, const int32_t* flag, MoveCarry mc,
                                                       int32_t cache_from, MomLag lg, double** tab) {
    move_blk_body<K, LEAN>(ctape, prog.seg_new, prog.seg_old, prog.cst, prog.nseg_new, prog.nseg_old, fs, mb, Lb, seed,
                           goff, N, accepted, flag, mc, cache_from, lg, tab);
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

// One step of the fused 2D SSM (examples/2D_ssm.jl:11-16) for two adjacent particles per
// thread. The run's working state is particle-major pairs ([N][2]: x_t, v, dv), so each
// gather through an ancestor is one 16-B load and every store (x, v, w pairs) is 16 B per
// lane. Gathers x_t, v through the previous step's ancestors, draws dv, x_{t+1} = x_t + v,
// v += dv, observes, and folds the block's max log-weight into one of 64 line-strided slots.
// MODE (diagnostics only, results wrong; production = 0): bit 1 = no draw (dv = 0),
// bit 2 = no ancestor gather (src = i), bit 4 = no block max / atomic, bit 8 = per-wave
// unfiltered atomics. Measured (1M, bench timing): 17.0 (0) / 15.3 (1) / 16.4 (2) / 15.0 (3) /
// 16.3 (4) / 14.3 (7) / 17.0 (8) us — draws ~1.8 us, the max tail ~0.7 us, the rest is the
// 36 B read + 40 B write per particle. Write-through (sc1) or nontemporal 16-B stores were
// slower (22-25 us); loading the ancestors speculatively beside the decision flag changed
// nothing.
#ifndef WSMC_PROP_LDS_LOG   // the draws' log table from an LDS copy (0: the cached gathers, for comparison)
#define WSMC_PROP_LDS_LOG 1
#endif
// QS (round 6, the single-GPU and island runs): NT = 512 threads, so a block is one 1024-particle
// Resample tile, and the block also takes the tile's Resample statistics (k_rs_sums_t's q, tile
// partials and group sums) against a guessed reference point R_g = ceil(U), U = (the previous
// step's log-mean, or its max when it did not resample) + the observation density's maximum
// -c0/2: every weight of the step is <= U (rounding is monotone), so R_g >= ceil(M), and R_g is
// the canonical ceil(M) unless M and U straddle an integer. k_rs_qfix checks that once M is
// known and recomputes the statistics when it is not (include/wsmc_math.h wsmc_qref).
template <int MODE, int IT = 1, int NT = kBlock, bool QS = false>
__global__ __launch_bounds__(NT) void k_ssm2d_prop(Ssm2dArgs a) {
    __shared__ u64 lds4[NT / 64];
    __shared__ double s_logtab[2 * WSMC_LOG_TABLE_N];
    if (WSMC_PROP_LDS_LOG && (MODE & 1) == 0) {   // every thread, before the first draw
        const double* lt = wsmc_log_table();
        for (int k = (int)threadIdx.x; k < 2 * WSMC_LOG_TABLE_N; k += NT) s_logtab[k] = lt[k];
        __syncthreads();
    }
    const double* logtab = WSMC_PROP_LDS_LOG ? s_logtab : wsmc_log_table();
    const int64_t N = a.N;
    bool rs;
    double mean;
    if (a.recs_prev && a.t > 1) {
        __shared__ Decision s_dec;
        if (threadIdx.x == 0) {
            Decision dd;
            decide_records(a.recs_prev, a.world, a.rank, a.ess_min, &dd);
            s_dec = dd;
            if (blockIdx.x == 0) *a.dec_out = dd;
        }
        __syncthreads();
        rs = s_dec.resampled;
        mean = rs ? s_dec.mean : 0.0;
    } else {
        rs = a.t > 1 && a.dec_prev->resampled;
        mean = rs ? a.dec_prev->mean : 0.0;
    }
    const uint64_t op_dv = a.op_dev[0] + 3ull * (uint64_t)(a.t - 1);
    const double o0 = a.obs[2 * (a.t - 1)], o1 = a.obs[2 * (a.t - 1) + 1];
    // IT pairs per thread, a grid apart: every pair's loads are issued before any pair is
    // computed and stored, so one pair's stores overlap the next pair's reads
    const int64_t stride = (int64_t)gridDim.x * NT * 2;
    const int64_t ib = ((int64_t)blockIdx.x * NT + threadIdx.x) * 2;
    int64_t src[IT][2];
    bool ok[IT], two[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int64_t i0 = ib + (int64_t)j * stride;
        ok[j] = i0 < N;
        two[j] = i0 + 1 < N;
        src[j][0] = i0; src[j][1] = i0 + 1;
        // the ancestors are loaded speculatively (the previous step's row always exists at
        // t > 1), in parallel with the decision flag, not after it
        if (ok[j] && a.t > 1 && (MODE & 2) == 0 && !a.identity) {
            int2 s2;
            if (two[j]) {
                s2 = *reinterpret_cast<const int2*>(a.anc_prev + i0);
            } else {
                s2.x = a.anc_prev[i0];
                s2.y = 0;
            }
            if (rs) { src[j][0] = s2.x; src[j][1] = s2.y; }
        }
    }
    d2 xp[IT][2], vp[IT][2];
    double wb[IT][2];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int64_t i0 = ib + (int64_t)j * stride;
        wb[j][0] = wb[j][1] = mean;
        if (!ok[j]) continue;
        if (!rs) {
            if (two[j]) {
                const d2 w2 = *reinterpret_cast<const d2*>(a.w + i0);
                wb[j][0] = w2.x; wb[j][1] = w2.y;
                if (a.w_save) *reinterpret_cast<d2*>(a.w_save + i0) = w2;
            } else {
                wb[j][0] = a.w[i0];
                if (a.w_save) a.w_save[i0] = wb[j][0];
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (a.t == 1) {
                xp[j][k] = d2{a.x0[0], a.x0[1]};
                vp[j][k] = d2{a.v0[0], a.v0[1]};
            } else if (k == 0 || two[j]) {
                if (MODE & 16) {   // exact shards: global ids; a neighbour's particle arrived at the slot
                    const int64_t loc = rs ? src[j][k] - a.goff : src[j][k];
                    const bool here = loc >= 0 && loc < N;
                    const double* xs = here ? a.x_prev + 2 * loc : a.xr + 2 * (i0 + k);
                    const double* vs = here ? a.v_prev + 2 * loc : a.vr + 2 * (i0 + k);
                    xp[j][k] = *reinterpret_cast<const d2*>(xs);
                    vp[j][k] = *reinterpret_cast<const d2*>(vs);
                } else {
                    xp[j][k] = *reinterpret_cast<const d2*>(a.x_prev + 2 * src[j][k]);
                    vp[j][k] = *reinterpret_cast<const d2*>(a.v_prev + 2 * src[j][k]);
                }
            }
        }
    }
    u64 menc = 0;
    QAcc acc;          // QS: the tile's Resample statistics
    double Rg = 0.0, sK = 0.0;
    if (QS) {
        // the guess: every weight of this step is wb + lp <= base + lpmax (lp <= -c0/2, wb <= base)
        double base = WSMC_NAN;   // the first step: no bound (k_rs_qfix takes the statistics)
        if (a.t > 1 && a.ms_prev) base = rs ? mean : wave_slots_max(a.ms_prev);
        const double lpmax = -(a.c0 + 0.0) * 0.5;
        Rg = wsmc_qref(base + lpmax);
        sK = wsmc_pow2i(wsmc_qbits((uint64_t)N));
        if (blockIdx.x == 0 && threadIdx.x == 0) *a.rg_out = Rg;
    }
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        if (!ok[j]) continue;
        const int64_t i0 = ib + (int64_t)j * stride;
        // the draws need no loaded data: computed while the gathers are in flight
        double z[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
        if ((MODE & 1) == 0) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                wsmc_normal_pair_t(wsmc_rng_block(a.seed, op_dv, (uint64_t)(a.goff + i0 + k), 0u), &z[k][0], &z[k][1],
                                   logtab);
        }
        d2 xn[2], vn[2], dvv[2];
        double wn[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            // x{t+1} .= x{t} + v
            const double xn0 = aff2(xp[j][k].x, vp[j][k].x), xn1 = aff2(xp[j][k].y, vp[j][k].y);
            // dv ~ MvNormal([0,0], q*I)
            const double dv0 = 0.0 + a.q_sd * z[k][0], dv1 = 0.0 + a.q_sd * z[k][1];
            // v .= v + dv
            const double vn0 = aff2(vp[j][k].x, dv0), vn1 = aff2(vp[j][k].y, dv1);
            // o => MvNormal(x{t+1}, r*I)
            const double m0 = 0.0 + 1.0 * xn0, m1 = 0.0 + 1.0 * xn1;
            double s = 0.0;
            const double d0 = o0 - m0, d1 = o1 - m1;
            s = s + d0 * d0;
            s = s + d1 * d1;
            const double lp = -(a.c0 + s / a.r_var) * 0.5;
            wn[k] = wb[j][k] + lp;
            xn[k] = d2{xn0, xn1};
            vn[k] = d2{vn0, vn1};
            dvv[k] = d2{dv0, dv1};
        }
        *reinterpret_cast<d2*>(a.x_next + 2 * i0) = xn[0];
        *reinterpret_cast<d2*>(a.v_next + 2 * i0) = vn[0];
        if (a.dv) *reinterpret_cast<d2*>(a.dv + 2 * i0) = dvv[0];
        u64 e0 = wsmc_ord_enc(wn[0]);
        menc = e0 > menc ? e0 : menc;
        u64 q0 = 0, q1 = 0;
        if (QS) q0 = qacc_add(acc, wsmc_expw(wn[0] - Rg), sK);
        if (two[j]) {
            *reinterpret_cast<d2*>(a.x_next + 2 * i0 + 2) = xn[1];
            *reinterpret_cast<d2*>(a.v_next + 2 * i0 + 2) = vn[1];
            if (a.dv) *reinterpret_cast<d2*>(a.dv + 2 * i0 + 2) = dvv[1];
            *reinterpret_cast<d2*>(a.w + i0) = d2{wn[0], wn[1]};
            const u64 e1 = wsmc_ord_enc(wn[1]);
            menc = e1 > menc ? e1 : menc;
            if (QS) q1 = qacc_add(acc, wsmc_expw(wn[1] - Rg), sK);
            if (QS && a.qbuf) *reinterpret_cast<ulonglong2*>(a.qbuf + i0) = make_ulonglong2(q0, q1);
        } else {
            a.w[i0] = wn[0];
            if (QS && a.qbuf) a.qbuf[i0] = q0;
        }
    }
    if (QS) {
        // one barrier for the block max and the tile partials (qacc_tile's layout, the group lines
        // of k_rs_sums_t)
        __shared__ double s_f[kPart][NT / 64];
        const int th = threadIdx.x, wv = th >> 6;
        acc.Q = wave_sum_f64_exact(acc.Q);
        acc.Q2 = wave_sum_f64_exact(acc.Q2);
        acc.WF2 = wave_sum_f64_exact(acc.WF2);
        acc.WF = wave_sum_f64_exact(acc.WF);
        menc = wave_max_u64(menc);
        if ((th & 63) == 0) {
            s_f[0][wv] = acc.Q; s_f[1][wv] = acc.Q2;
            s_f[2][wv] = acc.WF2; s_f[3][wv] = acc.WF;
            lds4[wv] = menc;
        }
        __syncthreads();
        if (th < kPart) {
            double f = 0.0;
#pragma unroll
            for (int v = 0; v < NT / 64; ++v) f = f + s_f[th][v];
            const u64 t = (u64)f;                     // exact integer <= 2^53
            a.tilep[(int64_t)blockIdx.x * kPart + th] = t;
            if (th == 0) {
                u64* gl = a.grp + (int64_t)(blockIdx.x / a.G) * kGroupLine;
                atomicAdd(gl, t);
                atomicMax(gl + 1, t);
            }
        } else if (th == 64) {
            u64 m = 0;
#pragma unroll
            for (int v = 0; v < NT / 64; ++v) m = lds4[v] > m ? lds4[v] : m;
            atomic_max_filtered(&a.ms->v[blockIdx.x % kSlots][0], m);
        }
        return;
    }
    if (MODE & 4) {                                  // diag: no block max / atomic
        if (menc == 0x123456789ull) a.w[0] = 0.0;
        return;
    }
    if (MODE & 8) {                                  // diag: wave max + unfiltered atomic per wave
        menc = wave_max_u64(menc);
        if ((threadIdx.x & 63) == 0) atomicMax(&a.ms->v[(blockIdx.x * 4 + (threadIdx.x >> 6)) % kSlots][0], menc);
        return;
    }
    menc = block_max_u64(menc, lds4);
    if (threadIdx.x == 0) atomic_max_filtered(&a.ms->v[blockIdx.x % kSlots][0], menc);
}

// ---- exact-sharded fused run: distributed trace-back -------------------
// words per global index: x pair (2 doubles) + the ancestor id of the step before
__global__ __launch_bounds__(kBlock) void k_trace_pack(const double* __restrict__ xpairs,
                                                       const int32_t* __restrict__ arow, int64_t start, int64_t count,
                                                       u64* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= count) return;
    const d2 x = *reinterpret_cast<const d2*>(xpairs + 2 * (start + j));
    out[3 * j] = (u64)wsmc_d2bits(x.x);
    out[3 * j + 1] = (u64)wsmc_d2bits(x.y);
    out[3 * j + 2] = arow ? (u64)(uint32_t)arow[start + j] : 0ull;
}
__global__ __launch_bounds__(kBlock) void k_trace_lookup(const u64* __restrict__ recv, int64_t lo,
                                                         const int32_t* __restrict__ a, int64_t n,
                                                         double* __restrict__ xout, int32_t* __restrict__ anext,
                                                         int use_a) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t o = (int64_t)a[i] - lo;
    xout[i] = wsmc_bits2d(recv[3 * o]);
    xout[n + i] = wsmc_bits2d(recv[3 * o + 1]);
    anext[i] = use_a ? (int32_t)(uint32_t)recv[3 * o + 2] : a[i];
}
__global__ __launch_bounds__(kBlock) void k_pairs_to_soa(const double* __restrict__ pairs, double* __restrict__ soa,
                                                         int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const d2 v = *reinterpret_cast<const d2*>(pairs + 2 * i);
    soa[i] = v.x;
    soa[n + i] = v.y;
}
__global__ __launch_bounds__(kBlock) void k_fill_const2(double* __restrict__ soa, double v0, double v1, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    soa[i] = v0;
    soa[n + i] = v1;
}
__global__ __launch_bounds__(kBlock) void k_iota(int32_t* __restrict__ a, int64_t n, int64_t base) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] = (int32_t)(base + i);
}

// trace the ancestor log back once and materialise the final columns — the result
// ColumnStore's per-resample gather of every column would have produced (src/stores.jl:105-128)
// ISL: island shards decide the last step here, from its records (the single-GPU instance
// reads the decision: no barrier or decide code ahead of the trace)
// P = 2: two particles a thread (N even): two lineage chains in flight per thread, so a 1M
// population is resident in one round of waves, and every SoA output is a 16-B store.
// The walk is software-pipelined so that a step waits for one memory latency, its ancestor
// entry, and nothing else: the step's decision and its history pointers come from LDS (staged
// 64 steps at a time), and the x gathered at a step is stored one step later, after the next
// step's loads are issued (stores count in vmcnt: storing at once would make the next step's
// wait for its ancestor entry also wait for the store acknowledgements).
constexpr int kFinChunk = 64;   // steps whose decisions and history pointers are staged at a time
// a pointer read back from LDS is a generic (flat) pointer, and flat accesses count in both
// vmcnt and lgkmcnt (every LDS wait then also waits for them): cast to the global address space
typedef const double __attribute__((address_space(1)))* gcdp;
typedef double __attribute__((address_space(1)))* gdp;
// DG (diagnostic build only; results wrong): 1 = the walk and its gathers without the history
// stores, 2 = the ancestor chain alone
template <bool ISL, int P, int DG = 0>
__global__ __launch_bounds__(kBlock) void k_ssm2d_final(Ssm2dFinal f) {
    const int64_t N = f.N;
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * P;
    const int T = f.T;
    bool rsT;
    double meanT;
    Decision decT{};   // island shards: the last step's decision, taken here
    if (ISL) {
        __shared__ Decision s_dec;
        if (threadIdx.x == 0) {
            Decision dd;
            decide_records(f.recs_last, f.world, f.rank, f.ess_min, &dd);
            s_dec = dd;
            if (blockIdx.x == 0) *f.dec_out = dd;
        }
        __syncthreads();
        decT = s_dec;
        rsT = s_dec.resampled;
        meanT = s_dec.mean;
    } else {
        rsT = f.dec[T].resampled;
        meanT = f.dec[T].mean;
    }
    // lanes past N take the last particles' walk and store the same bits again: every lane
    // stays in the block's barriers and every step has the same memory operations
    const int64_t ib = i0 < N ? i0 : N - P;
    const int64_t S = f.anc_stride;
    // component pairs of P particles: (x.x of each, x.y of each) -> SoA dst[ib..], dst[N + ib..]
// WSMC_FIN_NT=1 (diagnostics): nontemporal history stores. Measured (tools/ab_bench.sh, round 5):
// 447 against 438 us a run, the bench line even (2.51e10 both): not kept
#ifndef WSMC_FIN_NT
#define WSMC_FIN_NT 0
#endif
// WSMC_FIN_SC1=1 (diagnostics): the history stores write-through (buffer stores with sc1, aux 16),
// so the streamed history does not stay in the XCD L2 over the walk's reused ancestor entries
#ifndef WSMC_FIN_SC1
#define WSMC_FIN_SC1 0
#endif
    auto put = [&](double* dst0, const d2 (&x)[P]) {
        gdp dst = (gdp)dst0;
        if constexpr (P >= 2 && WSMC_FIN_SC1) {
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            const uint64_t base = (uint64_t)(uintptr_t)dst0;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32));
            void* ub = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(ub, 0, (int)(16 * N), 0x00020000);
#pragma unroll
            for (int p = 0; p < P; p += 2) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, d2{x[p].x, x[p + 1].x}), rs,
                                                       (int)(8 * (ib + p)), 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, d2{x[p].y, x[p + 1].y}), rs,
                                                       (int)(8 * (N + ib + p)), 0, 16);
            }
        } else if constexpr (P >= 2) {
#pragma unroll
            for (int p = 0; p < P; p += 2) {
                if (WSMC_FIN_NT) {
                    typedef double __attribute__((ext_vector_type(2))) v2d;
                    __builtin_nontemporal_store(v2d{x[p].x, x[p + 1].x}, reinterpret_cast<__attribute__((address_space(1))) v2d*>(dst + ib + p));
                    __builtin_nontemporal_store(v2d{x[p].y, x[p + 1].y}, reinterpret_cast<__attribute__((address_space(1))) v2d*>(dst + N + ib + p));
                } else {
                    *reinterpret_cast<__attribute__((address_space(1))) d2*>(dst + ib + p) = d2{x[p].x, x[p + 1].x};
                    *reinterpret_cast<__attribute__((address_space(1))) d2*>(dst + N + ib + p) = d2{x[p].y, x[p + 1].y};
                }
            }
        } else {
            dst[ib] = x[0].x;
            dst[N + ib] = x[0].y;
        }
    };
    int64_t a[P];
#pragma unroll
    for (int p = 0; p < P; ++p) a[p] = rsT ? f.anc_log[(int64_t)(T - 1) * S + ib + p] : ib + p;
    // the run's read-back: block 0 copies the decisions to the host's pinned words (island
    // shards: the last one is this kernel's); every thread copies its particles' entry of the
    // last resampled row (step T's is a, already loaded; else the newest step that resampled,
    // found by the first wave, 64 steps a ballot; none: last_anc is left as it was)
    if (f.hdec && blockIdx.x == 0)
        for (int t = (int)threadIdx.x; t <= T; t += kBlock) {
            f.hdec[t] = (ISL && t == T) ? decT : f.dec[t];
        }
    if (f.last_anc) {
        if (rsT) {
#pragma unroll
            for (int p = 0; p < P; ++p) f.last_anc[ib + p] = (int32_t)a[p];
        } else {
            __shared__ int s_tl;
            if (threadIdx.x < 64) {
                int best = 0;
                for (int top = T - 1; top >= 1 && best == 0; top -= 64) {   // steps (top - 64, top]
                    const int t = top - (int)threadIdx.x;
                    const u64 m = __ballot(t >= 1 && f.dec[t].resampled);
                    if (m) best = top - __builtin_ctzll(m);                  // the lowest lane: the newest
                }
                if (threadIdx.x == 0) s_tl = best;
            }
            __syncthreads();
            const int tl = s_tl;
            if (tl > 0)
#pragma unroll
                for (int p = 0; p < P; ++p) f.last_anc[ib + p] = f.anc_log[(int64_t)(tl - 1) * S + ib + p];
        }
    }
    // working buffers are particle-major pairs; output columns are SoA [2][N]
    {
        d2 v[P], dv[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            v[p] = *reinterpret_cast<const d2*>(f.v_work + 2 * a[p]);
            dv[p] = *reinterpret_cast<const d2*>(f.dv_work + 2 * a[p]);
        }
        put(f.v_out, v);
        put(f.dv_out, dv);
    }
    if (rsT) {
        if constexpr (P >= 2) {
#pragma unroll
            for (int p = 0; p < P; p += 2) *reinterpret_cast<d2*>(f.w + ib + p) = d2{meanT, meanT};
        } else {
            f.w[ib] = meanT;
        }
    }
    if (!f.keep_history) {
        d2 x[P];
#pragma unroll
        for (int p = 0; p < P; ++p) x[p] = *reinterpret_cast<const d2*>(f.x_work + 2 * a[p]);
        put(f.x_out, x);
        return;
    }
    // The lineage a_s (x_{s+1} is read at a_s): a_s = anc_log row s-1 at a_{s+1} when step s
    // resampled, else a_{s+1}. x_{T+1} was written at step T (read at a_T = a).
    __shared__ const double* s_work[kFinChunk];
    __shared__ double* s_out[kFinChunk];
    __shared__ u64 s_rs;
    d2 xp[P];   // gathered, not yet stored
#pragma unroll
    for (int p = 0; p < P; ++p) xp[p] = *reinterpret_cast<const d2*>(f.hist_work[T + 1] + 2 * a[p]);
    double* outp = f.hist_out[T + 1];
    // the entry of step T - 1's row (T - 2 in the log) at the lineage so far; every later entry
    // is loaded by the step before (across chunks too), so the inner loop's entry state is the
    // same from the chunk prologue and from its own back edge (one wait a step, for the entry)
    int32_t raw[P];
#pragma unroll
    for (int p = 0; p < P; ++p) raw[p] = f.anc_log[(int64_t)(T - 2 > 0 ? T - 2 : 0) * S + a[p]];
    double sink = 0.0;   // (DG: keeps the walk's loads live)
    for (int s0 = T - 1; s0 >= 1; s0 -= kFinChunk) {
        const int n = s0 < kFinChunk ? s0 : kFinChunk;   // steps s0, s0 - 1, ..., s0 - n + 1
        __syncthreads();   // the previous chunk's readers are done
        if (threadIdx.x < kFinChunk) {
            const int k = threadIdx.x, s = s0 - k;
            const bool rs = k < n && f.dec[s].resampled;
            s_work[k] = k < n ? f.hist_work[s + 1] : nullptr;
            s_out[k] = k < n ? f.hist_out[s + 1] : nullptr;
            const u64 m = __ballot(rs);
            if (k == 0) s_rs = m;
        }
        __syncthreads();
        const u64 rsw = s_rs;
        for (int k = 0; k < n; ++k) {
            const int s = s0 - k;
            if ((rsw >> k) & 1)
#pragma unroll
                for (int p = 0; p < P; ++p) a[p] = raw[p];
            const int64_t ro = (int64_t)(s - 2 > 0 ? s - 2 : 0) * S;
            gcdp src = (gcdp)s_work[k];
            d2 xn[P];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                raw[p] = f.anc_log[ro + a[p]];
                if (DG == 2)
                    xn[p] = d2{(double)raw[p], 0.0};
                else
                    xn[p] = *reinterpret_cast<const __attribute__((address_space(1))) d2*>(src + 2 * a[p]);
            }
            if (DG == 0)
                put(outp, xp);
            else
#pragma unroll
                for (int p = 0; p < P; ++p) sink += xp[p].x + xp[p].y;
            outp = s_out[k];
#pragma unroll
            for (int p = 0; p < P; ++p) xp[p] = xn[p];
        }
    }
    put(outp, xp);
    d2 x1[P];
#pragma unroll
    for (int p = 0; p < P; ++p) x1[p] = d2{f.x0[0], f.x0[1]};
    put(f.hist_out[1], x1);
    if (DG) f.w[ib] = sink;
}

// A fused run's head (RunHead): the per-step words its kernels accumulate into, zeroed, and its
// op-base word and observations copied from pinned host memory (the last block; coherent
// memory, read once, 16 B a run per observation pair)
__global__ __launch_bounds__(kBlock) void k_run_head(RunHead h) {
    const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x, nth = (int64_t)gridDim.x * kBlock;
#pragma unroll
    for (int r = 0; r < 3; ++r)
        for (int64_t i = tid; i < h.zwords[r]; i += nth) h.z[r][i] = 0ull;
    if (blockIdx.x == gridDim.x - 1) {
        for (int i = (int)threadIdx.x; i < h.nobs; i += kBlock) h.obs[i] = h.hstage[2 + i];
        if (threadIdx.x == 0) *h.op = (uint64_t)wsmc_d2bits(h.hstage[0]);
    }
}
hipError_t launch_run_head(hipStream_t s, const RunHead& h) {
    int64_t w = h.zwords[0] > h.zwords[1] ? h.zwords[0] : h.zwords[1];
    w = w > h.zwords[2] ? w : h.zwords[2];
    int64_t nb = (w + kBlock * 4 - 1) / (kBlock * 4);
    nb = nb < 1 ? 1 : nb > 256 ? 256 : nb;
    hipLaunchKernelGGL(k_run_head, dim3((unsigned)nb), dim3(kBlock), 0, s, h);
    return hipGetLastError();
}

// the 4 moves' accepted counts from their 64 slots each (one wave a move, DPP-free shuffles),
// and the 4 flag words, written straight into the host's pinned words (a synchronous Move's
// read-back: no copy launches behind it)
__global__ __launch_bounds__(kBlock) void k_acc_sum(const u64* __restrict__ acc, u64* __restrict__ out,
                                                    const int32_t* __restrict__ flag, int32_t* __restrict__ flag_out) {
    const int m = threadIdx.x >> 6, s = threadIdx.x & 63;
    u64 v = acc[(size_t)m * kAccMove + (size_t)s * kAccStride];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (s == 0) out[m] = v;
    if (flag_out && threadIdx.x < 4) flag_out[threadIdx.x] = flag[threadIdx.x];
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static inline dim3 grid_for(int64_t N) { return dim3((unsigned)((N + kBlock - 1) / kBlock)); }
static inline dim3 tiles_for(int64_t N) { return dim3((unsigned)((N + kTile - 1) / kTile)); }
static inline dim3 rs_tiles_for(int64_t N) { return dim3((unsigned)((N + kRsTile - 1) / kRsTile)); }

hipError_t launch_assign(hipStream_t s, double* out, int dim, const wsmc_operand* expr,
                         double* const* cols, int64_t N, const Indirect& ind) {
    AssignArgs a;
    for (int k = 0; k < 4; ++k) {
        a.e[k] = expr[k < dim ? k : 0];
        for (int m = 0; m < 2; ++m)
            a.p[k][m] = a.e[k].col[m] >= 0 ? ind.front[a.e[k].col[m]] + (int64_t)a.e[k].comp[m] * N : nullptr;
    }
    hipLaunchKernelGGL(k_assign, grid_for(N), dim3(kBlock), 0, s, out, dim, a, cols, N, ind);
    return hipGetLastError();
}
hipError_t launch_assign_expr(hipStream_t s, const XProg& x) {
    static_assert(sizeof(XProg) + 32 <= 4096, "the program rides in the kernel arguments");
    if (x.N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_assign_expr, grid_for(x.N), dim3(kBlock), 0, s, x);
    return hipGetLastError();
}
hipError_t launch_sample(hipStream_t s, double* out, int dim, const wsmc_dist& d, uint64_t seed, uint64_t op,
                         int64_t goff, double* const* cols, int64_t N) {
    const int has_sd = d.family == WSMC_FAM_MVNORMAL_ISO && wsmc_operand_is_const(&d.scale);
    const double sd = has_sd ? wsmc_sqrt(wsmc_operand_eval(&d.scale, nullptr, N, 0, nullptr)) : 0.0;
    if (wsmc_dist_feat(&d) & (WSMC_FEAT_MVN | WSMC_FEAT_EXT))
        hipLaunchKernelGGL(k_sample<WSMC_FEAT_ALL>, grid_for(N), dim3(kBlock), 0, s, out, dim, d, seed, op, goff, cols,
                           N, has_sd, sd);
    else if (d.mean_fn == WSMC_MEAN_OSCILLATOR)
        hipLaunchKernelGGL(k_sample<WSMC_FEAT_OSC>, grid_for(N), dim3(kBlock), 0, s, out, dim, d, seed, op, goff, cols,
                           N, has_sd, sd);
    else
        hipLaunchKernelGGL(k_sample<0u>, grid_for(N), dim3(kBlock), 0, s, out, dim, d, seed, op, goff, cols, N, has_sd,
                           sd);
    return hipGetLastError();
}
hipError_t launch_ew_assign1(hipStream_t s, const EwBatch& b, double* const* cols, int64_t N) {
    const EwOp& op = b.ops[0];
    AssignArgs a;
    for (int k = 0; k < 4; ++k) {
        a.e[k] = op.a.e[k];
        for (int m = 0; m < 2; ++m) a.p[k][m] = op.a.p[k][m];
    }
    Indirect ind;
    ind.row = b.anc;
    ind.dec = b.dec;
    ind.mask = op.a.lag;
    if (b.ntab > 0) {
        ind.tab_col = b.tab_col[0];
        ind.tab = b.tab;
    }
    hipLaunchKernelGGL(k_assign, grid_for(N), dim3(kBlock), 0, s, op.out, (int)op.dim, a, cols, N, ind);
    return hipGetLastError();
}
hipError_t launch_ew_batch(hipStream_t s, const EwBatch& b, unsigned feat, uint64_t seed, int64_t goff, int64_t N) {
    static_assert(sizeof(EwBatch) + 32 <= 4096, "the batch rides in the kernel arguments");
    const size_t rows = sizeof(double) * kBlock * (size_t)b.nrows;   // only the rows used: occupancy
    if (feat & (WSMC_FEAT_MVN | WSMC_FEAT_EXT))
        hipLaunchKernelGGL(k_ew_batch<WSMC_FEAT_ALL>, grid_for(N), dim3(kBlock), rows, s, b, seed, goff, N);
    else if (feat)
        hipLaunchKernelGGL(k_ew_batch<WSMC_FEAT_OSC>, grid_for(N), dim3(kBlock), rows, s, b, seed, goff, N);
    else
        hipLaunchKernelGGL(k_ew_batch<0u>, grid_for(N), dim3(kBlock), rows, s, b, seed, goff, N);
    return hipGetLastError();
}
hipError_t launch_sample_importance(hipStream_t s, double* out, int dim, const wsmc_dist& prop,
                                    const wsmc_dist& targ, double* w, uint64_t seed, uint64_t op,
                                    int64_t goff, double* const* cols, int64_t N) {
    if ((wsmc_dist_feat(&prop) | wsmc_dist_feat(&targ)) & (WSMC_FEAT_MVN | WSMC_FEAT_EXT))
        hipLaunchKernelGGL(k_sample_importance<WSMC_FEAT_ALL>, grid_for(N), dim3(kBlock), 0, s, out, dim, prop, targ, w,
                           seed, op, goff, cols, N);
    else
        hipLaunchKernelGGL(k_sample_importance<WSMC_FEAT_OSC>, grid_for(N), dim3(kBlock), 0, s, out, dim, prop, targ, w,
                           seed, op, goff, cols, N);
    return hipGetLastError();
}
hipError_t launch_weigh(hipStream_t s, const wsmc_term& t, double* w, double* const* cols, int64_t N, MaxSlots* ms,
                        MaxSlots* ms_next, const Decision* wreset) {
    wsmc_logmemo lm0 = {0, 0.0, 0.0, 0};
    if (t.dist.family != WSMC_FAM_UNIFORM && wsmc_operand_is_const(&t.dist.scale)) {
        const double sc = wsmc_operand_eval(&t.dist.scale, nullptr, N, 0, nullptr);
        lm0.arg = wsmc_d2bits(sc);
        lm0.val = wsmc_log(sc);
        lm0.rcp = 1.0 / sc;
        lm0.valid = 1;
    }
    if (wsmc_dist_feat(&t.dist) & (WSMC_FEAT_MVN | WSMC_FEAT_EXT))
        hipLaunchKernelGGL(k_weigh<WSMC_FEAT_ALL>, grid_for(N), dim3(kBlock), 0, s, t, w, cols, N, ms, ms_next, lm0,
                           wreset);
    else if (t.dist.mean_fn == WSMC_MEAN_OSCILLATOR)
        hipLaunchKernelGGL(k_weigh<WSMC_FEAT_OSC>, grid_for(N), dim3(kBlock), 0, s, t, w, cols, N, ms, ms_next, lm0,
                           wreset);
    else
        hipLaunchKernelGGL(k_weigh<0u>, grid_for(N), dim3(kBlock), 0, s, t, w, cols, N, ms, ms_next, lm0, wreset);
    return hipGetLastError();
}
template <typename K, typename... Args>
static hipError_t launch_timed(K kernel, dim3 grid, dim3 block, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                               Args... args) {
    if (e0 || e1)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, e0, e1, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
    return hipGetLastError();
}

hipError_t launch_lazy_trace(hipStream_t s, const TraceArgs& a, int64_t N) {
    bool pair = (N & 1) == 0 && (!a.a_in || ((uintptr_t)a.a_in & 7) == 0) && (!a.a_out || ((uintptr_t)a.a_out & 7) == 0);
    for (int c = 0; c < a.ncomp; ++c) pair = pair && ((uintptr_t)a.comp[c].dst & 15) == 0;
    if (pair)
        hipLaunchKernelGGL(k_lazy_trace<2>, grid_for(N / 2), dim3(kBlock), 0, s, a, N);
    else
        hipLaunchKernelGGL(k_lazy_trace<1>, grid_for(N), dim3(kBlock), 0, s, a, N);
    return hipGetLastError();
}
hipError_t launch_rs_max(hipStream_t s, const double* w, int64_t N, MaxSlots* ms) {
    int64_t nb = (N + kBlock * 4 - 1) / (kBlock * 4);
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_rs_max, dim3((unsigned)nb), dim3(kBlock), 0, s, w, N, ms);
    return hipGetLastError();
}
hipError_t launch_rs_sums(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, u64* tilep, u64* qbuf,
                          hipEvent_t e0, hipEvent_t e1, u64* grp, int G, int64_t Nk, int nms, int gall) {
    if (nms > 1)
        return launch_timed(k_rs_sums_t<0, true>, rs_tiles_for(N), dim3(kSumBlock), s, e0, e1, w, N, ms, tilep, qbuf,
                            grp, G, Nk > 0 ? Nk : N, nms, gall);
    return launch_timed(k_rs_sums_t<0>, rs_tiles_for(N), dim3(kSumBlock), s, e0, e1, w, N, ms, tilep, qbuf, grp, G,
                        Nk > 0 ? Nk : N, nms, gall);
}
hipError_t launch_rs_fill_fused(hipStream_t s, int64_t N, const FillPlan& plan, const u64* grp, int G,
                                const MaxSlots* ms, double ess_min, ShardRecord* rec, Decision* dec, const u64* qbuf,
                                int32_t* anc, hipEvent_t e0, hipEvent_t e1, const double* wq) {
    const dim3 g((unsigned)((N + kRsTile - 1) / kRsTile + kOverflowBlocks + 1));
    if (wq)
        return launch_timed(k_rs_fill_fused<0, true>, g, dim3(kScanBlock), s, e0, e1, N, plan, grp, G, ms, ess_min,
                            rec, dec, qbuf, anc, wq);
#ifdef WSMC_DIAG_BUILD
    static const int diag = [] {
        const char* e = diag_env("WSMC_DIAG_FILL");
        return e ? atoi(e) : 0;
    }();
    if (diag == 1)
        return launch_timed(k_rs_fill_fused<1>, g, dim3(kScanBlock), s, e0, e1, N, plan, grp, G, ms, ess_min,
                            rec, dec, qbuf, anc, wq);
#endif
    return launch_timed(k_rs_fill_fused<0>, g, dim3(kScanBlock), s, e0, e1, N, plan, grp, G, ms, ess_min,
                        rec, dec, qbuf, anc, wq);
}
hipError_t launch_rs_qfix(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, const double* rg, u64* tilep,
                          u64* qbuf, u64* grp, int G, u64* nfix, hipEvent_t e0, hipEvent_t e1) {
    // few blocks: in the common case each one only reads the slots and returns
    const int64_t nt = (N + kRsTile - 1) / kRsTile;
    int64_t nb = 256;
#ifdef WSMC_DIAG_BUILD
    static const int diag = [] {   // blocks; 0 = no check at all (wrong results on a miss: timing only)
        const char* e = diag_env("WSMC_DIAG_QFIX_BLOCKS");
        return e ? atoi(e) : -1;
    }();
    if (diag == 0) {
        if (e0) (void)hipEventRecord(e0, s);
        if (e1) (void)hipEventRecord(e1, s);
        return hipSuccess;
    }
    if (diag > 0) nb = diag;
#endif
    const dim3 g((unsigned)(nt < nb ? nt : nb));
    return launch_timed(k_rs_qfix, g, dim3(kSumBlock), s, e0, e1, w, N, ms, rg, tilep, qbuf, grp, G, nfix);
}
hipError_t launch_rs_reduce(hipStream_t s, const MaxSlots* ms, const u64* tilep, int64_t N, u64* tileOff,
                            ShardRecord* rec, int decide_local, double ess_min, Decision* dec,
                            const FillPlan* plan, hipEvent_t e0, hipEvent_t e1, u64* esum, int nms) {
    const int64_t nt = (N + kRsTile - 1) / kRsTile;
    FillPlan p{};
    if (plan) p = *plan;
    return launch_timed(k_rs_reduce_t<0>, dim3(1), dim3(kRsBlock), s, e0, e1, ms, tilep, nt, N, tileOff, rec,
                        decide_local, ess_min, dec, p, esum, nms);
}
hipError_t launch_rs_decide(hipStream_t s, const ShardRecord* recs, int world, int rank, double ess_min,
                            Decision* dec) {
    hipLaunchKernelGGL(k_rs_decide, dim3(1), dim3(64), 0, s, recs, world, rank, ess_min, dec);
    return hipGetLastError();
}
hipError_t launch_max_publish(hipStream_t s, const MaxSlots* ms, u64* word) {
    hipLaunchKernelGGL(k_max_publish, dim3(1), dim3(64), 0, s, ms, word);
    return hipGetLastError();
}
// the global max from the ranks' words `stride` apart (k_max_adopt's rule)
__global__ void k_autorw_max(const u64* words, int world, int stride, MaxSlots* ms) {
    const int th = threadIdx.x;
    u64 m = 0;
    for (int g = 0; g < world; ++g) m = words[(int64_t)g * stride] > m ? words[(int64_t)g * stride] : m;
    ms->v[th & 63][0] = th == 0 ? m : 0ull;
}
hipError_t launch_autorw_max(hipStream_t s, const u64* words, int world, int stride, MaxSlots* ms) {
    hipLaunchKernelGGL(k_autorw_max, dim3(1), dim3(64), 0, s, words, world, stride, ms);
    return hipGetLastError();
}
hipError_t launch_autorw_combine(hipStream_t s, const u64* xchg, int world, int stride, int d, int pass,
                                 double min_step, double* mom, int32_t* flag) {
    hipLaunchKernelGGL(k_autorw_combine, dim3(1), dim3(64), 0, s, xchg, world, stride, d, pass, min_step, mom, flag);
    return hipGetLastError();
}
hipError_t launch_max_adopt(hipStream_t s, const u64* words, int world, MaxSlots* ms) {
    hipLaunchKernelGGL(k_max_adopt, dim3(1), dim3(64), 0, s, words, world, ms);
    return hipGetLastError();
}
hipError_t launch_rs_decide_exact(hipStream_t s, const ShardRecord* recs, int world, int rank, double ess_min,
                                  const FillPlan& plan, ShardRecord* comb, Decision* dec, ExactPlan* xp) {
    hipLaunchKernelGGL(k_rs_decide_exact, dim3(1), dim3(64), 0, s, recs, world, rank, ess_min, plan, comb, dec, xp);
    return hipGetLastError();
}
hipError_t launch_exact_pack(hipStream_t s, const ExactRoute& rt, const int32_t* anc_out, const double* const* src,
                             double* const* dst, int32_t* anc_local, u64* sendbuf) {
    const u64 cnt = rt.b - rt.a;
    if (!cnt) return hipSuccess;
    hipLaunchKernelGGL(k_exact_pack, dim3((unsigned)((cnt + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rt, anc_out,
                       src, dst, anc_local, sendbuf);
    return hipGetLastError();
}
hipError_t launch_exact_route(hipStream_t s, const ExactStep& e) {
    hipLaunchKernelGGL(k_exact_route, dim3((unsigned)((2 * e.cap + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, e);
    return hipGetLastError();
}
hipError_t launch_exact_recv(hipStream_t s, const ExactStep& e) {
    hipLaunchKernelGGL(k_exact_recv, dim3((unsigned)((2 * e.cap + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, e);
    return hipGetLastError();
}
hipError_t launch_exact_window_pack(hipStream_t s, const ExactWin& w) {
    const int64_t n = 2 * (int64_t)w.T * w.ctr;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_exact_window_pack, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w);
    return hipGetLastError();
}
hipError_t launch_exact_final(hipStream_t s, const ExactFinal& f) {
    hipLaunchKernelGGL(k_exact_final, grid_for(f.N), dim3(kBlock), 0, s, f);
    return hipGetLastError();
}
hipError_t launch_exact_unpack(hipStream_t s, const ExactRoute& rt, const u64* recvbuf, double* const* dst,
                               int32_t* anc_local) {
    const u64 cnt = rt.recvpre[rt.world];
    if (!cnt) return hipSuccess;
    hipLaunchKernelGGL(k_exact_unpack, dim3((unsigned)((cnt + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rt,
                       recvbuf, dst, anc_local);
    return hipGetLastError();
}
hipError_t launch_sample_draws(hipStream_t s, int64_t n, int64_t N, const ShardRecord* rec, const u64* tileOff,
                               const u64* lcdf, uint64_t seed, uint64_t op, int64_t* out) {
    hipLaunchKernelGGL(k_sample_draws, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, N, rec,
                       tileOff, lcdf, seed, op, out);
    return hipGetLastError();
}
hipError_t launch_es_keys(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, uint64_t seed, uint64_t op,
                          u64* keys, u64* idx) {
    hipLaunchKernelGGL(k_es_keys, grid_for(N), dim3(kBlock), 0, s, w, N, ms, seed, op, keys, idx);
    return hipGetLastError();
}
hipError_t launch_gather_rows(hipStream_t s, const double* src, int64_t N, int dim, const int64_t* idx, int64_t n,
                              double* out) {
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, src, N, dim,
                       idx, n, out);
    return hipGetLastError();
}
hipError_t launch_median_keys(hipStream_t s, const double* x, const u64* q, int64_t N, u64* kq, u64* kv) {
    hipLaunchKernelGGL(k_median_keys, grid_for(N), dim3(kBlock), 0, s, x, q, N, kq, kv);
    return hipGetLastError();
}
hipError_t launch_median_pick(hipStream_t s, const u64* v, const u64* q, const u64* S, int64_t N, double* out) {
    hipLaunchKernelGGL(k_median_pick, dim3(1), dim3(64), 0, s, v, q, S, N, out);
    return hipGetLastError();
}
hipError_t launch_hist(hipStream_t s, const double* x, const u64* q, int64_t N, const double* edges, u64* cnt) {
    HistEdges ed;
    for (int k = 0; k < 9; ++k) ed.e[k] = edges[k];
    int64_t nb = (N + kBlock - 1) / kBlock;
    if (nb > 2048) nb = 2048;
    hipLaunchKernelGGL(k_hist, dim3((unsigned)nb), dim3(kBlock), 0, s, x, q, N, ed, cnt);
    return hipGetLastError();
}
// one block per tile (its first chunk) + grid-stride overflow blocks
static inline dim3 fill_tasks_for(int64_t N) {
    return dim3((unsigned)((N + kRsTile - 1) / kRsTile + kOverflowBlocks));
}
hipError_t launch_rs_scan(hipStream_t s, int64_t N, const ShardRecord* rec, const Decision* dec,
                          const FillPlan& plan, const u64* tileOff, const u64* qbuf, int32_t* anc, hipEvent_t e0,
                          hipEvent_t e1) {
    return launch_timed(k_rs_scan_t<0>, fill_tasks_for(N), dim3(kScanBlock), s, e0, e1, N, rec, dec, plan, tileOff,
                        qbuf, anc);
}

hipError_t launch_rs_sums_multi(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, const FillPlan& plan,
                                u64* tilep, u64* lcdf, u64* esum, uint32_t* ebuf, hipEvent_t e0, hipEvent_t e1) {
    return launch_timed(k_rs_sums_multi, rs_tiles_for(N), dim3(kSumBlock), s, e0, e1, w, N, ms, plan, tilep, lcdf,
                        esum, ebuf);
}
hipError_t launch_rs_multinomial(hipStream_t s, int64_t N, const ShardRecord* rec, const Decision* dec,
                                 const FillPlan& plan, const u64* tileOff, const u64* lcdf, const u64* esum,
                                 const uint32_t* ebuf, int32_t* anc, hipEvent_t e0, hipEvent_t e1) {
    const unsigned nt = (unsigned)((N + kRsTile - 1) / kRsTile);
    return launch_timed(k_multi_fill, dim3(nt), dim3(kScanBlock), s, e0, e1, N, rec, dec, plan, tileOff, lcdf, esum,
                        ebuf, anc);
}

// diagnostics: the propagate kernel's memory pattern with no arithmetic — per particle a
// 4-B index + 2 x 16-B reads, 2 x 16-B + 8-B writes (76 B), 2 particles per thread.
// MODE 0: identity index; 1: index gather through anc (the step's ancestors)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_stream_like_prop(const int32_t* __restrict__ anc,
                                                            const double* __restrict__ xs,
                                                            const double* __restrict__ vs, double* __restrict__ xd,
                                                            double* __restrict__ vd, double* __restrict__ wd,
                                                            int64_t N) {
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 2;
    if (i0 + 1 >= N) return;
    const int2 s2 = *reinterpret_cast<const int2*>(anc + i0);
    const int64_t a0 = MODE ? s2.x : i0, a1 = MODE ? s2.y : i0 + 1;
    const d2 x0 = *reinterpret_cast<const d2*>(xs + 2 * a0), x1 = *reinterpret_cast<const d2*>(xs + 2 * a1);
    const d2 v0 = *reinterpret_cast<const d2*>(vs + 2 * a0), v1 = *reinterpret_cast<const d2*>(vs + 2 * a1);
    *reinterpret_cast<d2*>(xd + 2 * i0) = x0 + v0;
    *reinterpret_cast<d2*>(xd + 2 * i0 + 2) = x1 + v1;
    *reinterpret_cast<d2*>(vd + 2 * i0) = v0;
    *reinterpret_cast<d2*>(vd + 2 * i0 + 2) = v1;
    *reinterpret_cast<d2*>(wd + i0) = d2{x0.x + (double)s2.x, x1.x};
}

// diagnostics: time `iters` launches of a kernel variant on the context's current buffers
hipError_t debug_kernel_bench(hipStream_t s, int kernel, int mode, int iters, const double* w, int64_t N,
                              MaxSlots* ms, u64* tilep, u64* qbuf, u64* tileOff, ShardRecord* rec, Decision* dec,
                              const FillPlan& plan, int32_t* anc, double* stream4, float* ms_out) {
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e0 = hipEventCreate(&a);
    if (e0 == hipSuccess) e0 = hipEventCreate(&b);
    if (e0 == hipSuccess) e0 = hipEventRecord(a, s);
    if (e0 != hipSuccess) {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
        return e0;
    }
    const dim3 g = rs_tiles_for(N), blk(kSumBlock), gs = fill_tasks_for(N), bs(kScanBlock);
#ifndef WSMC_DIAG_BUILD
    // the ablations (mode > 0) and the streaming calibration kernel exist in the diagnostic
    // build only (tools/build_variant.py NAME -DWSMC_DIAG_BUILD)
    if (mode != 0 || kernel == 3) {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        return hipErrorNotSupported;
    }
    for (int it = 0; it < iters; ++it) {
        if (kernel == 0)
            hipLaunchKernelGGL(k_rs_sums_t<0>, g, blk, 0, s, w, N, ms, tilep, qbuf, nullptr, 1, N, 1, 0);
        else if (kernel == 1)
            hipLaunchKernelGGL(k_rs_reduce_t<0>, dim3(1), dim3(kRsBlock), 0, s, ms, tilep,
                               (N + kRsTile - 1) / kRsTile, N, tileOff, rec, 1, 2.0, dec, plan, nullptr, 1);
        else
            hipLaunchKernelGGL(k_rs_scan_t<0>, gs, bs, 0, s, N, rec, dec, plan, tileOff, qbuf, anc);
    }
    (void)stream4;
#else
    for (int it = 0; it < iters; ++it) {
        if (kernel == 0) {
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_rs_sums_t<0>, g, blk, 0, s, w, N, ms, tilep, qbuf, nullptr, 1, N, 1, 0); break;
                case 1: hipLaunchKernelGGL(k_rs_sums_t<1>, g, blk, 0, s, w, N, ms, tilep, qbuf, nullptr, 1, N, 1, 0); break;
                default: hipLaunchKernelGGL(k_rs_sums_t<4>, g, blk, 0, s, w, N, ms, tilep, qbuf, nullptr, 1, N, 1, 0); break;
            }
        } else if (kernel == 3) {
            // scratch: stream4 = 4 x [2N] doubles (x src, v src, x dst, v dst), wd = w
            const dim3 gp((unsigned)((N + 2 * kBlock - 1) / (2 * kBlock)));
            double* b4 = stream4;
            if (mode == 0)
                hipLaunchKernelGGL(k_stream_like_prop<0>, gp, dim3(kBlock), 0, s, anc, b4, b4 + 2 * N, b4 + 4 * N,
                                   b4 + 6 * N, const_cast<double*>(w), N);
            else
                hipLaunchKernelGGL(k_stream_like_prop<1>, gp, dim3(kBlock), 0, s, anc, b4, b4 + 2 * N, b4 + 4 * N,
                                   b4 + 6 * N, const_cast<double*>(w), N);
        } else if (kernel == 1) {
            const int64_t nt = (N + kRsTile - 1) / kRsTile;
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_rs_reduce_t<0>, dim3(1), dim3(kRsBlock), 0, s, ms, tilep, nt, N, tileOff, rec, 1, 2.0, dec, plan, nullptr, 1); break;
                case 1: hipLaunchKernelGGL(k_rs_reduce_t<1>, dim3(1), dim3(kRsBlock), 0, s, ms, tilep, nt, N, tileOff, rec, 1, 2.0, dec, plan, nullptr, 1); break;
                case 2: hipLaunchKernelGGL(k_rs_reduce_t<2>, dim3(1), dim3(kRsBlock), 0, s, ms, tilep, nt, N, tileOff, rec, 1, 2.0, dec, plan, nullptr, 1); break;
                default: hipLaunchKernelGGL(k_rs_reduce_t<3>, dim3(1), dim3(kRsBlock), 0, s, ms, tilep, nt, N, tileOff, rec, 1, 2.0, dec, plan, nullptr, 1); break;
            }
        } else {
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_rs_scan_t<0>, gs, bs, 0, s, N, rec, dec, plan, tileOff, qbuf, anc); break;
                case 1: hipLaunchKernelGGL(k_rs_scan_t<1>, gs, bs, 0, s, N, rec, dec, plan, tileOff, qbuf, anc); break;
                case 2: hipLaunchKernelGGL(k_rs_scan_t<2>, gs, bs, 0, s, N, rec, dec, plan, tileOff, qbuf, anc); break;
                default: hipLaunchKernelGGL(k_rs_scan_t<3>, gs, bs, 0, s, N, rec, dec, plan, tileOff, qbuf, anc); break;
            }
        }
    }
#endif
    hipError_t e = hipEventRecord(b, s);
    if (e == hipSuccess) e = hipEventSynchronize(b);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, a, b);
    *ms_out = t;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return e != hipSuccess ? e : hipGetLastError();
}

// ColumnStore.resample! of every column component (and the carried Move scores) plus the
// weight reset in one launch: blockIdx.y selects a (dst, src) pair, y == n the weights.
// dec: gate on the device-side decision (identity copy when it did not resample) — the
// asynchronous Resample; null: the host has seen a resample. w null: no weight reset.
__global__ __launch_bounds__(kBlock) void k_resample_apply(GatherSet gs, const int32_t* __restrict__ anc,
                                                           const Decision* dec, double* w, int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    const int k = blockIdx.y;
    const bool rs = dec ? dec->resampled != 0 : true;
    if (i == 0 && k < gs.n && gs.tab && gs.col[k] >= 0) gs.tab[gs.col[k]] = gs.dst[k];   // new front
    if (k == gs.n) {
        if (rs && dec) w[i] = dec->mean;
        return;
    }
    gs.dst[k][i] = gs.src[k][rs ? (int64_t)anc[i] : i];
}
hipError_t launch_resample_apply(hipStream_t s, const GatherSet& gs, const int32_t* anc, const Decision* dec,
                                 double* w, int64_t N) {
    const dim3 g((unsigned)((N + kBlock - 1) / kBlock), (unsigned)(gs.n + (w ? 1 : 0)));
    if (g.y == 0) return hipSuccess;
    hipLaunchKernelGGL(k_resample_apply, g, dim3(kBlock), 0, s, gs, anc, dec, w, N);
    return hipGetLastError();
}
// the ColumnStore gather of an asynchronous Resample (the host has not seen the decision):
// through the ancestors if it resampled, else an identity copy, so the host's front/back
// swap is right either way
__global__ __launch_bounds__(kBlock) void k_gather_dec(double* __restrict__ dst, const double* __restrict__ src,
                                                       const int32_t* __restrict__ anc, const Decision* dec,
                                                       int64_t N) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= N) return;
    dst[i] = src[dec->resampled ? (int64_t)anc[i] : i];
}
hipError_t launch_gather_dec(hipStream_t s, double* dst, const double* src, const int32_t* anc, const Decision* dec,
                             int64_t N) {
    hipLaunchKernelGGL(k_gather_dec, grid_for(N), dim3(kBlock), 0, s, dst, src, anc, dec, N);
    return hipGetLastError();
}
hipError_t launch_gather(hipStream_t s, double* dst, const double* src, const int32_t* anc, int64_t N) {
    hipLaunchKernelGGL(k_gather, grid_for(N), dim3(kBlock), 0, s, dst, src, anc, N);
    return hipGetLastError();
}
hipError_t launch_fill_weights(hipStream_t s, double* w, const Decision* dec, int64_t N, MaxSlots* ms) {
    hipLaunchKernelGGL(k_fill_weights, dim3((unsigned)((N + 4 * kBlock - 1) / (4 * kBlock))), dim3(kBlock), 0, s, w,
                       dec, N, ms);
    return hipGetLastError();
}
hipError_t launch_log_evidence_stats(hipStream_t s, const double* w, int64_t N, MaxSlots* ms, u64* tilep,
                                     u64* qbuf, u64* tileOff, ShardRecord* rec) {
    hipError_t e = launch_rs_max(s, w, N, ms);
    if (e == hipSuccess) e = launch_rs_sums(s, w, N, ms, tilep, qbuf);
    if (e == hipSuccess) e = launch_rs_reduce(s, ms, tilep, N, tileOff, rec, 0, 0.0, nullptr, nullptr);
    return e;
}
hipError_t launch_score(hipStream_t s, const wsmc_term* tape, int32_t n, int32_t depth, double* const* cols,
                        int64_t N, double* out) {
    hipLaunchKernelGGL(k_score, grid_for(N), dim3(kBlock), 0, s, tape, n, depth, cols, N, out);
    return hipGetLastError();
}
hipError_t launch_moments(hipStream_t s, const double* w, const MaxSlots* rec, double* const* cols,
                          const int32_t* tcols, int d, const double* lo, const double* hi, int pass,
                          const double* mom, int64_t N, double* tilepart) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
        ma.lgw[k] = (wsmc_isfinite(ma.lo[k]) && wsmc_isfinite(ma.hi[k])) ? wsmc_log(ma.hi[k] - ma.lo[k]) : 0.0;
    }
    ma.use_ex = 0;
    const int64_t nt = (N + kTile - 1) / kTile;
    switch (d) {
        case 1: hipLaunchKernelGGL((k_moments<1, false>), tiles_for(N), dim3(kBlock), 0, s, w, rec, cols, ma, pass, mom, N, nt, tilepart); break;
        case 2: hipLaunchKernelGGL((k_moments<2, false>), tiles_for(N), dim3(kBlock), 0, s, w, rec, cols, ma, pass, mom, N, nt, tilepart); break;
        case 3: hipLaunchKernelGGL((k_moments<3, false>), tiles_for(N), dim3(kBlock), 0, s, w, rec, cols, ma, pass, mom, N, nt, tilepart); break;
        default: hipLaunchKernelGGL((k_moments<4, false>), tiles_for(N), dim3(kBlock), 0, s, w, rec, cols, ma, pass, mom, N, nt, tilepart); break;
    }
    return hipGetLastError();
}
hipError_t launch_moments_expr(hipStream_t s, const double* w, const MaxSlots* ms, double* const* cols,
                               const wsmc_operand* ex, int d, int pass, const double* mom, int64_t N,
                               double* tilepart) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = 0;
        ma.lo[k] = -WSMC_INF;
        ma.hi[k] = WSMC_INF;
        ma.lgw[k] = (wsmc_isfinite(ma.lo[k]) && wsmc_isfinite(ma.hi[k])) ? wsmc_log(ma.hi[k] - ma.lo[k]) : 0.0;
        ma.ex[k] = ex[k < d ? k : 0];
    }
    ma.use_ex = 1;
    const int64_t nt = (N + kTile - 1) / kTile;
    switch (d) {
        case 1: hipLaunchKernelGGL((k_moments<1, true>), tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pass, mom, N, nt, tilepart); break;
        case 2: hipLaunchKernelGGL((k_moments<2, true>), tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pass, mom, N, nt, tilepart); break;
        case 3: hipLaunchKernelGGL((k_moments<3, true>), tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pass, mom, N, nt, tilepart); break;
        default: hipLaunchKernelGGL((k_moments<4, true>), tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pass, mom, N, nt, tilepart); break;
    }
    return hipGetLastError();
}
// unweighted min / max of one column component (describe): ordered-encoding maxima of x and
// of -x into the line-strided slots (NaN propagates, as Base.minimum / maximum)
__global__ __launch_bounds__(kBlock) void k_minmax(const double* __restrict__ x, int64_t N, MaxSlots* ms) {
    __shared__ u64 lds4[4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    u64 a = 0, b = 0;
    if (i < N) {
        a = wsmc_ord_enc(x[i]);
        b = wsmc_ord_enc(-x[i]);
    }
    a = block_max_u64(a, lds4);
    b = block_max_u64(b, lds4);
    if (threadIdx.x == 0) {
        atomic_max_filtered(&ms->v[blockIdx.x % kSlots][0], a);
        atomic_max_filtered(&ms->v[blockIdx.x % kSlots][1], b);
    }
}
hipError_t launch_minmax(hipStream_t s, const double* x, int64_t N, MaxSlots* ms) {
    hipLaunchKernelGGL(k_minmax, grid_for(N), dim3(kBlock), 0, s, x, N, ms);
    return hipGetLastError();
}
static MomArgs mom_args(const int32_t* tcols, int d, const double* lo, const double* hi) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
        ma.lgw[k] = (wsmc_isfinite(ma.lo[k]) && wsmc_isfinite(ma.hi[k])) ? wsmc_log(ma.hi[k] - ma.lo[k]) : 0.0;
    }
    ma.use_ex = 0;
    return ma;
}
hipError_t launch_autorw_moments(hipStream_t s, const double* w, const MaxSlots* ms, double* const* cols,
                                 const int32_t* tcols, int d, const double* lo, const double* hi, const u64* pv,
                                 int64_t N, double* tilepart, const Decision* wreset, const Decision* gate,
                                 const int32_t* lag_anc, const Decision* lag_dec, int lag_mask, int32_t* zflag,
                                 u64* zcount) {
    const MomArgs ma = mom_args(tcols, d, lo, hi);
    const int64_t nt = (N + kTile - 1) / kTile;
    const MomLag lg{lag_mask ? lag_anc : nullptr, lag_dec, lag_mask};
    const MomZero z{zflag, zcount};
    switch (d) {
        case 1: hipLaunchKernelGGL(k_moments1<1>, tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pv, N, nt, tilepart, wreset, gate, lg, z); break;
        case 2: hipLaunchKernelGGL(k_moments1<2>, tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pv, N, nt, tilepart, wreset, gate, lg, z); break;
        case 3: hipLaunchKernelGGL(k_moments1<3>, tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pv, N, nt, tilepart, wreset, gate, lg, z); break;
        default: hipLaunchKernelGGL(k_moments1<4>, tiles_for(N), dim3(kBlock), 0, s, w, ms, cols, ma, pv, N, nt, tilepart, wreset, gate, lg, z); break;
    }
    return hipGetLastError();
}
hipError_t launch_acc_sum(hipStream_t s, const u64* acc, u64* out, const int32_t* flag, int32_t* flag_out) {
    hipLaunchKernelGGL(k_acc_sum, dim3(1), dim3(kBlock), 0, s, acc, out, flag, flag_out);
    return hipGetLastError();
}
hipError_t launch_autorw_final(hipStream_t s, const double* tilepart, int64_t ntiles, int d, double min_step,
                               double* mom, int32_t* flag, int raw, const Decision* gate) {
    switch (d) {
        case 1: hipLaunchKernelGGL(k_autorw_final<1>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, min_step, mom, flag, raw, gate); break;
        case 2: hipLaunchKernelGGL(k_autorw_final<2>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, min_step, mom, flag, raw, gate); break;
        case 3: hipLaunchKernelGGL(k_autorw_final<3>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, min_step, mom, flag, raw, gate); break;
        default: hipLaunchKernelGGL(k_autorw_final<4>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, min_step, mom, flag, raw, gate); break;
    }
    return hipGetLastError();
}
hipError_t launch_autorw_final_blk(hipStream_t s, const double* tilepart, int64_t ntiles, const MoveBlk& mb,
                                   int sep, const int32_t* toff, double* mom, int32_t* flag, const Decision* gate) {
    if (sep) {
        BlkOff o{};
        for (int m = 0; m < mb.nm; ++m) o.t[m] = toff[m];
        hipLaunchKernelGGL(k_autorw_final_sep, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, mb, o, mom, flag, gate);
        return hipGetLastError();
    }
    switch (mb.off[mb.nm]) {
        case 1: hipLaunchKernelGGL(k_autorw_final_blk<1>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, mb, mom, flag, gate); break;
        case 2: hipLaunchKernelGGL(k_autorw_final_blk<2>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, mb, mom, flag, gate); break;
        case 3: hipLaunchKernelGGL(k_autorw_final_blk<3>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, mb, mom, flag, gate); break;
        default: hipLaunchKernelGGL(k_autorw_final_blk<4>, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, mb, mom, flag, gate); break;
    }
    return hipGetLastError();
}
hipError_t launch_move_blk(hipStream_t s, const ProgInlineBlk* pin, const wsmc_term* ctape, const FoldProgram& prog,
                           const FoldSlots& fs, const MoveBlk& mb, const double* Lb, uint64_t seed, int64_t goff,
                           int64_t N, unsigned long long* accepted, const int32_t* flag, const MoveCarry& mc,
                           int32_t cache_from, const int32_t* lag_anc, const Decision* lag_dec, int lag_mask,
                           double** tab) {
    const MomLag lg{lag_mask ? lag_anc : nullptr, lag_dec, lag_mask};
    const size_t row = sizeof(double) * kBlock * (size_t)(fs.n + mb.off[mb.nm]);
    const dim3 g1((unsigned)((N + kBlock - 1) / kBlock)), g2((unsigned)((N + 2 * kBlock - 1) / (2 * kBlock)));
    const dim3 gk((unsigned)((N + WSMC_BLK_K * kBlock - 1) / (WSMC_BLK_K * kBlock)));
    if (pin) {
        const bool bnd = mb.bnd != 0;
        if (fs.heavy && bnd)
            hipLaunchKernelGGL((k_move_blk<1, 2, 1>), g1, dim3(kBlock), row, s, *pin, fs, mb, Lb, seed, goff, N, accepted,
                               flag, mc, cache_from, prog.nseg_new, prog.nseg_old, lg, tab);
        else if (fs.heavy)
            hipLaunchKernelGGL((k_move_blk<1, 2, 0>), g1, dim3(kBlock), row, s, *pin, fs, mb, Lb, seed, goff, N, accepted,
                               flag, mc, cache_from, prog.nseg_new, prog.nseg_old, lg, tab);
        else if (bnd)
            hipLaunchKernelGGL((k_move_blk<2, 1, 1>), g2, dim3(kBlock), 2 * row, s, *pin, fs, mb, Lb, seed, goff, N,
                               accepted, flag, mc, cache_from, prog.nseg_new, prog.nseg_old, lg, tab);
        else
            hipLaunchKernelGGL((k_move_blk<WSMC_BLK_K, 1, 0>), gk, dim3(kBlock), WSMC_BLK_K * row, s, *pin, fs, mb, Lb,
                               seed, goff, N, accepted, flag, mc, cache_from, prog.nseg_new, prog.nseg_old, lg, tab);
    } else {
        if (fs.heavy)
            hipLaunchKernelGGL((k_move_blk_g<1, 2>), g1, dim3(kBlock), row, s, ctape, prog, fs, mb, Lb, seed, goff, N,
                               accepted, flag, mc, cache_from, lg, tab);
        else
            hipLaunchKernelGGL((k_move_blk_g<2, 1>), g2, dim3(kBlock), 2 * row, s, ctape, prog, fs, mb, Lb, seed, goff,
                               N, accepted, flag, mc, cache_from, lg, tab);
    }
    return hipGetLastError();
}
hipError_t launch_autorw_publish(hipStream_t s, const MaxSlots* ms, double* const* cols, const int32_t* tcols, int d,
                                 const double* lo, const double* hi, u64* out) {
    const MomArgs ma = mom_args(tcols, d, lo, hi);
    switch (d) {
        case 1: hipLaunchKernelGGL(k_autorw_publish<1>, dim3(1), dim3(64), 0, s, ms, cols, ma, out); break;
        case 2: hipLaunchKernelGGL(k_autorw_publish<2>, dim3(1), dim3(64), 0, s, ms, cols, ma, out); break;
        case 3: hipLaunchKernelGGL(k_autorw_publish<3>, dim3(1), dim3(64), 0, s, ms, cols, ma, out); break;
        default: hipLaunchKernelGGL(k_autorw_publish<4>, dim3(1), dim3(64), 0, s, ms, cols, ma, out); break;
    }
    return hipGetLastError();
}
hipError_t launch_autorw_combine1(hipStream_t s, const u64* xchg, int world, int stride, int d, double min_step,
                                  double* mom, int32_t* flag) {
    hipLaunchKernelGGL(k_autorw_combine1, dim3(1), dim3(64), 0, s, xchg, world, stride, d, min_step, mom, flag);
    return hipGetLastError();
}
hipError_t launch_moments_final(hipStream_t s, const double* tilepart, int64_t ntiles, int d, int pass,
                                double min_step, double* mom, int32_t* flag, int raw) {
    hipLaunchKernelGGL(k_moments_final, dim3(1), dim3(kBlock), 0, s, tilepart, ntiles, d, pass, min_step, mom,
                       flag, raw);
    return hipGetLastError();
}
hipError_t launch_move(hipStream_t s, const wsmc_term* tape, int32_t nterms, int32_t depth, double* const* cols,
                       const int32_t* tcols, int d, const double* lo, const double* hi, int bounded,
                       const double* L, uint64_t seed, uint64_t op_prop, uint64_t op_acc, int64_t goff,
                       int64_t N, u64* accepted, const int32_t* flag, double* scache,
                       int32_t cache_from) {
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
        ma.lgw[k] = (wsmc_isfinite(ma.lo[k]) && wsmc_isfinite(ma.hi[k])) ? wsmc_log(ma.hi[k] - ma.lo[k]) : 0.0;
    }
    hipLaunchKernelGGL(k_move, grid_for(N), dim3(kBlock), 0, s, tape, nterms, depth, cols, ma, d, bounded, L,
                       seed, op_prop, op_acc, goff, N, accepted, flag, scache, cache_from);
    return hipGetLastError();
}
hipError_t launch_move_c(hipStream_t s, const wsmc_term* ctape, int32_t nterms, int32_t depth, const FoldSlots& fs,
                         const int32_t* tcols, int d, const double* lo, const double* hi, int bounded,
                         const double* L, uint64_t seed, uint64_t op_prop, uint64_t op_acc, int64_t goff, int64_t N,
                         u64* accepted, const int32_t* flag, const MoveCarry& mc, int32_t cache_from,
                         const FoldProgram& prog, const ProgInline* pin) {
    (void)nterms;
    (void)depth;
    MomArgs ma;
    for (int k = 0; k < 4; ++k) {
        ma.tcol[k] = k < d ? tcols[k] : 0;
        ma.lo[k] = (k < d && lo) ? lo[k] : -WSMC_INF;
        ma.hi[k] = (k < d && hi) ? hi[k] : WSMC_INF;
        ma.lgw[k] = (wsmc_isfinite(ma.lo[k]) && wsmc_isfinite(ma.hi[k])) ? wsmc_log(ma.hi[k] - ma.lo[k]) : 0.0;
    }
    // particles per thread: 2 when the terms are cheap (the scalar term chain dominates:
    // C3 3.7 vs 4.3 ms per run), 1 when they are transcendental-heavy (occupancy wins: C5
    // 0.76 vs 0.88 s); 4 was slower for both
    const size_t row = sizeof(double) * kBlock * (size_t)(fs.n + d);
    static const int kdiag = [] {   // diagnostics only: force 1 or 2 particles per thread
        const char* e = diag_env("WSMC_DIAG_MOVE_K");
        return e ? atoi(e) : 0;
    }();
    static const int nolean = [] {   // diagnostics only: the generic fold for every program
        const char* e = diag_env("WSMC_DIAG_MOVE_GENERIC");
        return e ? atoi(e) : 0;
    }();
    // lean variant: 1 = scalar terms and runs without oscillators, 2 = with them, 0 = generic
    const int lean = nolean ? 0 : (fs.lean ? (fs.heavy ? 2 : 1) : 0);
#define WSMC_MOVE_LAUNCH(KK, LL)                                                                               \
    hipLaunchKernelGGL((k_move_c<KK, LL>), dim3((unsigned)((N + KK * kBlock - 1) / (KK * kBlock))), dim3(kBlock),  \
                       KK * row, s, ctape, fs, ma, d, bounded, L, seed, op_prop, op_acc, goff, N, accepted, flag, mc, \
                       cache_from, prog)
#define WSMC_MOVE_LAUNCH_I(KK, LL)                                                                             \
    hipLaunchKernelGGL((k_move_ci<KK, LL>), dim3((unsigned)((N + KK * kBlock - 1) / (KK * kBlock))), dim3(kBlock), \
                       KK * row, s, *pin, fs, ma, d, bounded, L, seed, op_prop, op_acc, goff, N, accepted, flag,    \
                       mc, cache_from, prog.nseg_new, prog.nseg_old)
    if (pin) {   // lean programs only (the host inlines no other; WSMC_DIAG_MOVE_GENERIC
                 // applies to uploaded programs: pair it with WSMC_DIAG_PROG_COPY)
        const bool one = kdiag == 1 || (kdiag != 2 && fs.heavy);
        if (one) {
            if (fs.heavy) WSMC_MOVE_LAUNCH_I(1, 2);
            else WSMC_MOVE_LAUNCH_I(1, 1);
        } else {
            if (fs.heavy) WSMC_MOVE_LAUNCH_I(2, 2);
            else WSMC_MOVE_LAUNCH_I(2, 1);
        }
        return hipGetLastError();
    }
    if (kdiag == 1 || (kdiag != 2 && fs.heavy)) {
        if (lean == 2) WSMC_MOVE_LAUNCH(1, 2);
        else if (lean == 1) WSMC_MOVE_LAUNCH(1, 1);
        else WSMC_MOVE_LAUNCH(1, 0);
    } else {
        if (lean == 2) WSMC_MOVE_LAUNCH(2, 2);
        else if (lean == 1) WSMC_MOVE_LAUNCH(2, 1);
        else WSMC_MOVE_LAUNCH(2, 0);
    }
#undef WSMC_MOVE_LAUNCH
#undef WSMC_MOVE_LAUNCH_I
    return hipGetLastError();
}
hipError_t launch_trace_pack(hipStream_t s, const double* xpairs, const int32_t* arow, int64_t start, int64_t count,
                             u64* out) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_trace_pack, dim3((unsigned)((count + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, xpairs, arow,
                       start, count, out);
    return hipGetLastError();
}
hipError_t launch_trace_lookup(hipStream_t s, const u64* recv, int64_t lo, const int32_t* a, int64_t n, double* xout,
                               int32_t* anext, int use_a) {
    hipLaunchKernelGGL(k_trace_lookup, grid_for(n), dim3(kBlock), 0, s, recv, lo, a, n, xout, anext, use_a);
    return hipGetLastError();
}
hipError_t launch_pairs_to_soa(hipStream_t s, const double* pairs, double* soa, int64_t n) {
    hipLaunchKernelGGL(k_pairs_to_soa, grid_for(n), dim3(kBlock), 0, s, pairs, soa, n);
    return hipGetLastError();
}
hipError_t launch_fill_const2(hipStream_t s, double* soa, double v0, double v1, int64_t n) {
    hipLaunchKernelGGL(k_fill_const2, grid_for(n), dim3(kBlock), 0, s, soa, v0, v1, n);
    return hipGetLastError();
}
hipError_t launch_iota(hipStream_t s, int32_t* a, int64_t n, int64_t base) {
    hipLaunchKernelGGL(k_iota, grid_for(n), dim3(kBlock), 0, s, a, n, base);
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
#ifdef WSMC_DIAG_BUILD
static int prop_mode() {
    static int v = [] {
        const char* e = diag_env("WSMC_DIAG_PROP_MODE");   // diagnostics only: ablated propagate
        return e ? atoi(e) & 15 : 0;
    }();
    return v;
}
#endif
hipError_t launch_ssm2d_propagate(hipStream_t s, const Ssm2dArgs& a, hipEvent_t e0, hipEvent_t e1) {
    if (a.qstat)   // one 1024-particle Resample tile a block
        return launch_timed(k_ssm2d_prop<0, 1, 512, true>, rs_tiles_for(a.N), dim3(512), s, e0, e1, a);
    const dim3 g((unsigned)((a.N + 2 * kBlock - 1) / (2 * kBlock)));
    // IT = 2 / 4 pairs per thread (grid / 2, / 4) measured 18.8 / 22.2 us against 17.0 (1M)
    if (a.xr) return launch_timed(k_ssm2d_prop<16>, g, dim3(kBlock), s, e0, e1, a);   // exact shards
#ifndef WSMC_DIAG_BUILD
    return launch_timed(k_ssm2d_prop<0>, g, dim3(kBlock), s, e0, e1, a);
#else
    switch (prop_mode()) {
        case 1: return launch_timed(k_ssm2d_prop<1>, g, dim3(kBlock), s, e0, e1, a);
        case 2: return launch_timed(k_ssm2d_prop<2>, g, dim3(kBlock), s, e0, e1, a);
        case 3: return launch_timed(k_ssm2d_prop<3>, g, dim3(kBlock), s, e0, e1, a);
        case 4: return launch_timed(k_ssm2d_prop<4>, g, dim3(kBlock), s, e0, e1, a);
        case 7: return launch_timed(k_ssm2d_prop<7>, g, dim3(kBlock), s, e0, e1, a);
        case 8: return launch_timed(k_ssm2d_prop<8>, g, dim3(kBlock), s, e0, e1, a);
        default: return launch_timed(k_ssm2d_prop<0>, g, dim3(kBlock), s, e0, e1, a);
    }
#endif
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

hipError_t launch_ssm2d_finalize(hipStream_t s, const Ssm2dFinal& f, hipEvent_t e0, hipEvent_t e1) {
    // two particles a thread when the SoA outputs' second components stay 16-B aligned
    bool pair = (f.N & 1) == 0 && ((uintptr_t)f.w & 15) == 0;
    static const int diag_p = [] {   // diagnostics (tools/): particles a thread, 1 / 2 / 4
        const char* e = diag_env("WSMC_DIAG_FINAL_P");
        return e ? atoi(e) : 0;
    }();
    if (diag_p == 4 && (f.N & 3) == 0 && pair) {
        if (f.recs_last) return launch_timed(k_ssm2d_final<true, 4>, grid_for(f.N / 4), dim3(kBlock), s, e0, e1, f);
        return launch_timed(k_ssm2d_final<false, 4>, grid_for(f.N / 4), dim3(kBlock), s, e0, e1, f);
    }
    if (diag_p == 1) pair = false;
#ifdef WSMC_DIAG_BUILD
    // 1: no history stores, 2: the ancestor chain alone (timing only, results wrong)
    static const int diag_fin = [] {
        const char* e = diag_env("WSMC_DIAG_FIN");
        return e ? atoi(e) : 0;
    }();
    if (pair && !f.recs_last && diag_fin == 1)
        return launch_timed(k_ssm2d_final<false, 2, 1>, grid_for(f.N / 2), dim3(kBlock), s, e0, e1, f);
    if (pair && !f.recs_last && diag_fin == 2)
        return launch_timed(k_ssm2d_final<false, 2, 2>, grid_for(f.N / 2), dim3(kBlock), s, e0, e1, f);
#endif
    if (pair) {
        if (f.recs_last) return launch_timed(k_ssm2d_final<true, 2>, grid_for(f.N / 2), dim3(kBlock), s, e0, e1, f);
        return launch_timed(k_ssm2d_final<false, 2>, grid_for(f.N / 2), dim3(kBlock), s, e0, e1, f);
    }
    if (f.recs_last) return launch_timed(k_ssm2d_final<true, 1>, grid_for(f.N), dim3(kBlock), s, e0, e1, f);
    return launch_timed(k_ssm2d_final<false, 1>, grid_for(f.N), dim3(kBlock), s, e0, e1, f);
}

}  // namespace wsmc
