// wsmc_ew_body.h — a statement batch (EwBatch, csrc/wsmc_ew.h) specialised for its shape.
//
// The interpreter (k_ew_batch, csrc/wsmc_kernels.hip) reads the batch's structure at run time:
// a loop over kernarg ops, every column value staged in LDS rows behind a pointer table, one
// particle per thread. This body takes the structure as a compile-time signature (EwSig: the
// op kinds and dims, which operand reads which row, which column is read through the ancestors)
// and the values (pointers, constants, op counters) from the same EwBatch in the kernel
// arguments. libwsmc generates one tiny translation unit per signature and compiles it with
// hiprtc the first time the signature is launched (csrc/wsmc_jit.hip) — the batch of a model's
// step has the same signature every step, so a run compiles once. After the ops are unrolled:
//   * every row is a register (r[p][row]); the header functions read them through a local
//     pointer table whose indices are constants, so nothing is left in memory;
//   * two adjacent particles a thread (PAIR): every direct column access, the weights and the
//     ancestors are 16-B (8-B) loads and stores; only reads through the ancestors stay 8-B
//     gathers. PAIR needs N even and 16-B aligned buffers (the host checks, else P = 1);
//   * the arithmetic is the interpreter's, call for call (wsmc_operand_eval's Assign order,
//     wsmc_dist_sample_mf, wsmc_term_logpdf_mf with the op's log memo), so the values are the
//     same bits as the interpreter's and the oracle's.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include "wsmc_ew.h"

namespace wsmc {

enum : int8_t { kSrcNone = 0, kSrcRow = 1, kSrcMem = 2, kSrcLag = 3 };
struct EwSigOp {
    int8_t kind, dim, out_row;          // EwOp's; out_row -1: the output has no rows
    int8_t family, mean_fn, ddim, has_sd, nostore;   // nostore: the output stays in its rows
    int8_t asrc[4][2];                  // Assign operand (component q, column c): kSrc*
    int8_t arow[4][2];                  // ... its row (kSrcRow)
    int8_t mrow[4][2];                  // Sample / weight dist mean operands: row (-1: no column)
    int8_t srow[2];                     // ... the scale operand
    int8_t xrow[4][2];                  // weight term value operands
};
struct EwSig {
    int8_t nops, has_w, has_reset, has_anc, has_dec, ntab, npre;
    int8_t qs;                          // the Resample statistics of the final weights (EwBatch)
    int8_t pre_row[kEwPre];
    int8_t pre_lag[kEwPre];
    uint32_t feat;
    EwSigOp op[kEwOps];
};

template <int P>
struct EwLanes {
    double r[P][kEwRows];   // the rows (registers after unrolling)
    double wv[P];
    int64_t j[P];           // ancestor (or own index) of each particle
};

// one 16-B (P = 2) or 8-B (P = 1) load / store of particles i0 .. i0 + P - 1
template <int P>
__device__ __forceinline__ void ew_load(const double* p, int64_t i0, double (&v)[P]) {
    if constexpr (P == 2) {
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v x = *reinterpret_cast<const d2v*>(p + i0);
        v[0] = x.x;
        v[1] = x.y;
    } else {
        v[0] = p[i0];
    }
}
template <int P>
__device__ __forceinline__ void ew_store(double* p, int64_t i0, const double (&v)[P]) {
    if constexpr (P == 2) {
        typedef double d2v __attribute__((ext_vector_type(2)));
        *reinterpret_cast<d2v*>(p + i0) = d2v{v[0], v[1]};
    } else {
        p[i0] = v[0];
    }
}

// the operands of a dist with their columns renumbered to rows (comp 0: the row is the
// component); the structural fields become constants, the numbers stay the batch's
__device__ __forceinline__ void ew_fix_operand(wsmc_operand& o, const int8_t (&row)[2]) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        o.col[m] = row[m];
        o.comp[m] = 0;
    }
}
template <class S, int K>
__device__ __forceinline__ void ew_fix_dist(wsmc_dist& d) {
    constexpr EwSigOp o = S::sig.op[K];
    d.family = o.family;
    d.mean_fn = o.mean_fn;
    d.dim = o.ddim;
#pragma unroll
    for (int q = 0; q < 4; ++q) ew_fix_operand(d.mu[q], o.mrow[q]);
    ew_fix_operand(d.scale, o.srow);
}

template <class S, int K, int P>
__device__ __forceinline__ void ew_op(const EwBatch* B, EwLanes<P>& L, uint64_t seed, int64_t goff, int64_t N,
                                      int64_t i0) {
    constexpr EwSig g = S::sig;
    constexpr EwSigOp o = g.op[K];
    const EwOp& op = B->ops[K];
    double x[P][4];
    if constexpr (o.kind == 0) {   // Assign (k_assign's arithmetic)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q >= o.dim) continue;
            const wsmc_operand& e = op.a.e[q];
            double v[P];
#pragma unroll
            for (int p = 0; p < P; ++p) v[p] = e.c0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (o.asrc[q][c] == kSrcNone) continue;
                double xv[P];
                if (o.asrc[q][c] == kSrcRow) {
#pragma unroll
                    for (int p = 0; p < P; ++p) xv[p] = L.r[p][o.arow[q][c]];
                } else if (o.asrc[q][c] == kSrcMem) {
                    ew_load<P>(op.a.p[q][c], i0, xv);
                } else {
#pragma unroll
                    for (int p = 0; p < P; ++p) xv[p] = op.a.p[q][c][L.j[p]];
                }
#pragma unroll
                for (int p = 0; p < P; ++p) v[p] = v[p] + e.coef[c] * xv[p];
            }
#pragma unroll
            for (int p = 0; p < P; ++p) x[p][q] = v[p];
        }
    } else if constexpr (o.kind == 1) {   // Sample (k_sample's)
        wsmc_dist d = op.s.d;
        ew_fix_dist<S, K>(d);
        const double sdl = op.s.sd;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            double* cols[kEwRows];
#pragma unroll
            for (int k = 0; k < kEwRows; ++k) cols[k] = &L.r[p][k];
            double xs[4] = {0.0, 0.0, 0.0, 0.0};
            wsmc_dist_sample_mf(&d, xs, seed, op.s.op, (uint64_t)(goff + i0 + p), cols, 0, 0,
                                o.has_sd ? &sdl : nullptr, g.feat);
#pragma unroll
            for (int q = 0; q < 4; ++q) x[p][q] = xs[q];
        }
    } else {   // Observe / Weight (k_weigh's)
        wsmc_term t = op.w.t;
        ew_fix_dist<S, K>(t.dist);
#pragma unroll
        for (int q = 0; q < 4; ++q) ew_fix_operand(t.x[q], o.xrow[q]);
#pragma unroll
        for (int p = 0; p < P; ++p) {
            double* cols[kEwRows];
#pragma unroll
            for (int k = 0; k < kEwRows; ++k) cols[k] = &L.r[p][k];
            wsmc_logmemo lm = op.w.lm0;
            L.wv[p] = L.wv[p] + wsmc_term_logpdf_mf(&t, cols, 0, 0, nullptr, &lm, g.feat);
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q >= o.dim) continue;
        double v[P];
#pragma unroll
        for (int p = 0; p < P; ++p) v[p] = x[p][q];
        if constexpr (!o.nostore) ew_store<P>(op.out + (int64_t)q * N, i0, v);
        if (o.out_row >= 0)
#pragma unroll
            for (int p = 0; p < P; ++p) L.r[p][o.out_row + q] = v[p];
    }
}

template <class S, int K, int P>
struct EwOps {
    static __device__ __forceinline__ void run(const EwBatch* B, EwLanes<P>& L, uint64_t seed, int64_t goff,
                                               int64_t N, int64_t i0) {
        if constexpr (K < S::sig.nops) {
            ew_op<S, K, P>(B, L, seed, goff, N, i0);
            EwOps<S, K + 1, P>::run(B, L, seed, goff, N, i0);
        }
    }
};

// P particles a thread: i0 = P * (global thread index); with P = 2 the host guarantees N even.
// NT threads a block; with the statistics (g.qs) P = 2 and NT = 512: a block is one Resample tile
template <class S, int P, int NT = kBlock>
__device__ __forceinline__ void ew_body(uint64_t seed, int64_t goff, int64_t N) {
    constexpr EwSig g = S::sig;
    static_assert(!g.qs || (g.has_w && P * NT == kRsTile), "the statistics: one tile a block");
    constexpr int NW = NT / 64;
    const EwBatch* B = (const EwBatch*)(const char*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ unsigned long long ldsw[NW];
#ifdef WSMC_TABLES_LDS
    wsmc_tables_to_lds();   // before any log / exp (every thread: it ends in a barrier)
#endif
    const int th = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * NT + th;
    const int64_t i0 = t * P;
    const bool in = i0 < N;
    if (t == 0)
#pragma unroll
        for (int k = 0; k < g.ntab; ++k) B->tab[B->tab_col[k]] = B->tab_out[k];
    EwLanes<P> L;
    unsigned long long m = 0;
    if (in) {
#pragma unroll
        for (int p = 0; p < P; ++p) L.j[p] = i0 + p;
        if constexpr (g.has_anc) {
            const bool rs = !g.has_dec || B->dec->resampled;
            if (rs) {
                if constexpr (P == 2) {
                    const int2 a = *reinterpret_cast<const int2*>(B->anc + i0);
                    L.j[0] = a.x;
                    L.j[1] = a.y;
                } else {
                    L.j[0] = B->anc[i0];
                }
            }
        }
        // every load that depends on no statement, up front
#pragma unroll
        for (int k = 0; k < kEwPre; ++k) {
            if (k >= g.npre) continue;
            double v[P];
            if (g.pre_lag[k]) {
#pragma unroll
                for (int p = 0; p < P; ++p) v[p] = B->pre_src[k][L.j[p]];
            } else {
                ew_load<P>(B->pre_src[k], i0, v);
            }
#pragma unroll
            for (int p = 0; p < P; ++p) L.r[p][g.pre_row[k]] = v[p];
        }
        if constexpr (g.has_w) {
            if (g.has_reset && B->wreset->resampled) {
#pragma unroll
                for (int p = 0; p < P; ++p) L.wv[p] = B->wreset->mean;
            } else {
                ew_load<P>(B->w, i0, L.wv);
            }
        }
        EwOps<S, 0, P>::run(B, L, seed, goff, N, i0);
        if constexpr (g.has_w) {
            ew_store<P>(B->w, i0, L.wv);
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const unsigned long long e = wsmc_ord_enc(L.wv[p]);
                m = e > m ? e : m;
            }
        }
    }
    // the Resample statistics (g.qs): q against the guessed reference point, the tile's exact
    // partials (k_rs_sums_t's arithmetic: qacc_add on the final weights, 0 past N)
    QAcc acc;
    if constexpr (g.qs) {
        double U = *B->qs_base;
        for (int k = 0; k < B->nqb; ++k) U = U + B->qb[k];   // (uniform)
        const double R = wsmc_qref(U);
        const double sK = wsmc_pow2i(wsmc_qbits((uint64_t)N));
        unsigned long long q[P];
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] = qacc_add(acc, in ? wsmc_expw(L.wv[p] - R) : 0.0, sK);
        if (in) *reinterpret_cast<ulonglong2*>(B->qbuf + i0) = make_ulonglong2(q[0], q[1]);
        if (blockIdx.x == 0 && th == 0) *B->rg_out = R;
    }
    if constexpr (g.has_w) {
        // block max (a wave's by DPP-free shuffles; the batch is not on the resample leg's
        // critical path), one filtered atomic per block into slot blockIdx % 64; with the
        // statistics, the tile's partials in the same barrier round (exact integers in f64:
        // any order gives the same sums)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(m, off, 64);
            m = o > m ? o : m;
            if constexpr (g.qs) {
                acc.Q = acc.Q + __shfl_xor(acc.Q, off, 64);
                acc.Q2 = acc.Q2 + __shfl_xor(acc.Q2, off, 64);
                acc.WF2 = acc.WF2 + __shfl_xor(acc.WF2, off, 64);
                acc.WF = acc.WF + __shfl_xor(acc.WF, off, 64);
            }
        }
        __shared__ double ldsq[g.qs ? kPart : 1][NW];
        if ((th & 63) == 0) {
            ldsw[th >> 6] = m;
            if constexpr (g.qs) {
                ldsq[0][th >> 6] = acc.Q;
                ldsq[1][th >> 6] = acc.Q2;
                ldsq[2][th >> 6] = acc.WF2;
                ldsq[3][th >> 6] = acc.WF;
            }
        }
        __syncthreads();
        if (th == 0) {
            unsigned long long a = 0;
#pragma unroll
            for (int k = 0; k < NW; ++k) a = ldsw[k] > a ? ldsw[k] : a;
            unsigned long long* slot = &B->ms->v[blockIdx.x % kSlots][0];
            const unsigned long long cur = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a > cur) atomicMax(slot, a);
        }
        if constexpr (g.qs) {
            if (th < kPart) {
                double f = 0.0;
#pragma unroll
                for (int k = 0; k < NW; ++k) f = f + ldsq[th][k];
                const unsigned long long tsum = (unsigned long long)f;   // exact integer <= 2^53
                B->tilep[(int64_t)blockIdx.x * kPart + th] = tsum;
                if (th == 0) {   // the tile's sum q into its group's line (integer atomics: order-free)
                    unsigned long long* gl = B->grp + (int64_t)(blockIdx.x / B->G) * kGroupLine;
                    atomicAdd(gl, tsum);
                    atomicMax(gl + 1, tsum);
                }
            }
        }
        if (blockIdx.x == 0)
            for (int k = th; k < kSlots * 16; k += NT) B->ms_next->v[k >> 4][k & 15] = 0ull;
    }
}

}  // namespace wsmc
