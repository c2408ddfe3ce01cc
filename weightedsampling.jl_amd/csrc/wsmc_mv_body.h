// wsmc_mv_body.h — a block of autoRW Moves (wsmc_move_block, src/transformers.jl:588-623)
// specialised for its shape.
//
// The interpreter kernels (k_move_blk, csrc/wsmc_kernels.hip) walk the fold program at run
// time: segment headers and term templates are scalar loads the next step depends on, the
// term evaluator carries every lean family and operand form, and slot values sit in LDS rows
// read through a pointer table (flat loads). Measured on C3 (examples/linear_regression.jl,
// 1M particles), the fold was 18.6 of the block's 53.7 us and the draws 11, with the
// arithmetic a few us of either (tools/abl_moves.sh, profiles/r04_abl*).
// This body takes the shape as a compile-time signature (MvSig): the block's moves and their
// dims, which targets are bounded, which slots are read through the lazy Resample's ancestors,
// and the fold program's segments — their kinds, term families and which slots each operand
// reads. The values stay run-time and are read where the interpreter reads them: the program
// ([templates | segments | constants], the same bytes) in the kernel arguments or in device
// memory, at offsets the signature fixes; counts, constants, coefficients, scales, the factors
// and the op counters. So:
//   * every slot value is a register (v[p][slot]), proposals too;
//   * a segment's header and its template's fields are independent scalar loads at constant
//     offsets, issued together;
//   * each fold is straight-line code for its segments (runs keep a run-time term count).
// The arithmetic is the interpreter's operation for operation (wsmc_operand_eval's order,
// wsmc_scalar_term_logpdf_p, the run loops of fold_seg, the draws, wsmc_bounded_step,
// move_accept), so the bits are the interpreter's and the oracle's.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include "wsmc_mv.h"

namespace wsmc {

constexpr int kMvSegs = 10;   // segments a program (new or old fold) may have in a compiled block
struct MvSigOp {
    int8_t c[2];              // the operand's slots (-1: none)
};
struct MvSigSeg {
    int8_t kind;              // kSegTerm / kSegNormalOsc / kSegNormalAff
    int8_t fam;               // a one-term segment's family: WSMC_FAM_NORMAL / HALFNORMAL / UNIFORM
    int8_t pre;               // a constant scale: its Normal pair (c, rh) at the segment's soff
    int8_t pad;
    MvSigOp x, mu[4], sc;     // the template's operand slots
};
struct MvSig {
    int8_t K, nm, D, ns;      // particles a thread, moves, union targets, slots
    int8_t ntmpl, nnew, nold, carry;   // templates; segments of the new / old fold; carried scores in
    int8_t off[5];            // move m owns union targets [off[m], off[m+1])
    uint8_t bnd;              // union target u bounded (bit u)
    uint8_t lagt;             // lag_targets: written in full (bit u)
    uint8_t flo, fhi;         // a bounded target's finite lower / upper bound (bit u): the
                              // transform's case, fixed at compile time
    uint16_t smask;           // slots read through the lag row when its decision resampled
    MvSigSeg seg[2 * kMvSegs];   // new fold [0, nnew), old fold [kMvSegs, kMvSegs + nold)
};
// the block's run-time arguments (after the program, ProgInlineBlk, in the kernel arguments)
struct MvArgs {
    FoldSlots fs;
    MoveBlk mb;
    const double* Lb;
    unsigned long long seed;
    int64_t goff, N;
    unsigned long long* accepted;
    const int32_t* flag;
    MoveCarry mc;
    MomLag lg;
    double** tab;
    const char* prog;         // the program in device memory, or null: in the kernel arguments
};

// canonical f64 block sum of NV values at once (256 threads): an xor butterfly 1..32 inside each
// wave, then (w0 + w1) + (w2 + w3), every value in the same order (the autoRW moments' tile and
// combine order, oracle/wsmc_oracle.c canon_block); lds [NV][4]
template <int NV>
__device__ __forceinline__ void block_sum_canon_n(const double (&v)[NV], double (*lds)[4], double (&out)[NV]) {
    double x[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) x[k] = v[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
#pragma unroll
        for (int k = 0; k < NV; ++k) x[k] = x[k] + __shfl_xor(x[k], off, 64);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[k][threadIdx.x >> 6] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = (lds[k][0] + lds[k][1]) + (lds[k][2] + lds[k][3]);
    __syncthreads();
}

__device__ __forceinline__ unsigned long long mv_block_sum(unsigned long long v, unsigned long long* lds4) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    const unsigned long long r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    __syncthreads();
    return r;
}

// wsmc_operand_eval with the slot reads resolved at compile time
template <int NS>
__device__ __forceinline__ double mv_opv(const wsmc_operand* o, MvSigOp q, const double (&v)[NS]) {
    double r = o->c0;
    if (q.c[0] >= 0) r = r + o->coef[0] * v[q.c[0]];
    if (q.c[1] >= 0) r = r + o->coef[1] * v[q.c[1]];
    return r;
}

// one fold over the segments [first, first + n) of the signature; rt: their run-time headers
template <class S, int FIRST, int NSEG, int K, int NS>
__device__ __forceinline__ void mv_fold(double (&s)[K], const double (&v)[K][NS], const wsmc_term* tp,
                                        const FoldSeg* rt, const double* cst) {
    constexpr MvSig G = S::sig;
#pragma unroll
    for (int g = 0; g < NSEG; ++g) {
        const MvSigSeg q = G.seg[FIRST + g];
        const FoldSeg h = rt[g];
        const wsmc_term* t = tp + h.tmpl;
        if (q.kind == kSegTerm) {
            // wsmc_scalar_term_logpdf_p
#pragma unroll
            for (int p = 0; p < K; ++p) {
                const double x0 = mv_opv<NS>(&t->x[0], q.x, v[p]);
                double term;
                if (q.fam == WSMC_FAM_NORMAL || q.fam == WSMC_FAM_HALFNORMAL) {
                    double nc, rh;
                    if (q.pre) {
                        nc = cst[h.soff];
                        rh = cst[h.soff + 1];
                    } else {
                        wsmc_normal_scale(nullptr, mv_opv<NS>(&t->dist.scale, q.sc, v[p]), &nc, &rh);
                    }
                    if (q.fam == WSMC_FAM_NORMAL) {
                        const double mu = mv_opv<NS>(&t->dist.mu[0], q.mu[0], v[p]);
                        term = wsmc_normal_lh((x0 - mu) * rh, nc);
                    } else {
                        term = (x0 >= 0.0) ? wsmc_normal_lh((x0 - 0.0) * rh, nc) + WSMC_LOG2 : -WSMC_INF;
                    }
                } else {
                    term = wsmc_uniform_logpdf(t->dist.param[0], t->dist.param[1], x0);
                }
                s[p] = s[p] + term;
            }
        } else if (q.kind == kSegNormalAff) {
            // Normal(c0 + coef0 col0 + coef1 col1, sigma) at y over (c0, coef0, coef1, y) per term
            const bool h0 = q.mu[0].c[0] >= 0, h1 = q.mu[0].c[1] >= 0;
            double v0[K], v1[K], rh[K], nc[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                v0[p] = h0 ? v[p][q.mu[0].c[0] < 0 ? 0 : q.mu[0].c[0]] : 0.0;
                v1[p] = h1 ? v[p][q.mu[0].c[1] < 0 ? 0 : q.mu[0].c[1]] : 0.0;
                if (q.pre) {
                    nc[p] = cst[h.soff];
                    rh[p] = cst[h.soff + 1];
                } else {
                    wsmc_normal_scale(nullptr, mv_opv<NS>(&t->dist.scale, q.sc, v[p]), &nc[p], &rh[p]);
                }
            }
            const double* c = cst + h.coff;
            const bool any = h.count > 0;
            double q0 = any ? c[0] : 0.0, q1 = any ? c[1] : 0.0, q2 = any ? c[2] : 0.0, q3 = any ? c[3] : 0.0;
            for (int32_t k = 0; k < h.count; ++k) {
                const double c0 = q0, a0 = q1, a1 = q2, y = q3;
                if (k + 1 < h.count) {
                    q0 = c[4 * k + 4];
                    q1 = c[4 * k + 5];
                    q2 = c[4 * k + 6];
                    q3 = c[4 * k + 7];
                }
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    double mu = c0;
                    if (h0) mu = mu + a0 * v0[p];
                    if (h1) mu = mu + a1 * v1[p];
                    s[p] = s[p] + wsmc_normal_lh((y - mu) * rh[p], nc[p]);
                }
            }
        } else {
            // Normal(A exp(-gamma t) cos(omega t + phi), sigma) at y, over (t_a, d, m, y) per term:
            // fold_seg's rotation walk (a block's first term the direct phasor, each next term one
            // complex multiply, a fold entering a block mid-way anchors and rolls there)
            double A[K], om[K], ga[K], ph[K], rh[K], nc[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                A[p] = mv_opv<NS>(&t->dist.mu[0], q.mu[0], v[p]);
                om[p] = mv_opv<NS>(&t->dist.mu[1], q.mu[1], v[p]);
                ga[p] = mv_opv<NS>(&t->dist.mu[2], q.mu[2], v[p]);
                ph[p] = mv_opv<NS>(&t->dist.mu[3], q.mu[3], v[p]);
                if (q.pre) {
                    nc[p] = cst[h.soff];
                    rh[p] = cst[h.soff + 1];
                } else {
                    wsmc_normal_scale(nullptr, mv_opv<NS>(&t->dist.scale, q.sc, v[p]), &nc[p], &rh[p]);
                }
            }
            const double* c = cst + h.coff;
            double zr[K], zi[K], rr[K], ri[K];
            // the segment's rotation runs (wsmc_mv.h): a run's first term is its anchor and m
            // rotations by the block's step R, each next term one rotation — the term-by-term
            // evaluation's operations bit for bit; the step is recomputed only when a run needs it
            // and its bits change. The inner loop is a rotation and a score per term, one scalar
            // load (the next observation, issued a term ahead)
            double r_d = WSMC_NAN;
            for (int32_t left = h.count; left > 0;) {   // uniform
                const double ta = c[0], dl = c[1];
                const int32_t m = osc_run_int(c[2]);
                const int32_t n0 = osc_run_int(c[3]), n = n0 < 1 ? 1 : n0;
                const double* yv = c + 4;
                c = yv + n;
                left -= n;
                if ((m > 0 || n > 1) && wsmc_d2bits(dl) != wsmc_d2bits(r_d)) {
#pragma unroll
                    for (int p = 0; p < K; ++p) wsmc_osc_step(dl, om[p], ga[p], &rr[p], &ri[p]);
                    r_d = dl;
                }
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    wsmc_osc_anchor(ta, A[p], om[p], ga[p], ph[p], &zr[p], &zi[p]);
                    for (int j = 0; j < m; ++j) wsmc_osc_rotate(&zr[p], &zi[p], rr[p], ri[p]);
                }
                // yv[k + 1] is in the program for every k < n (the next run's header or the
                // segment's pad word), so the next observation's load is unconditional
                double yn = yv[1];
#pragma unroll
                for (int p = 0; p < K; ++p) s[p] = s[p] + wsmc_normal_lh((yv[0] - zr[p]) * rh[p], nc[p]);
#pragma unroll 2
                for (int32_t k = 1; k < n; ++k) {
                    const double y = yn;
                    yn = yv[k + 1];
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        wsmc_osc_rotate(&zr[p], &zi[p], rr[p], ri[p]);
                        s[p] = s[p] + wsmc_normal_lh((y - zr[p]) * rh[p], nc[p]);
                    }
                }
            }
        }
    }
}

// move_blk_body (csrc/wsmc_kernels.hip) for one signature
template <class S>
__device__ __forceinline__ void mv_body(const char* pb, const MvArgs& a) {
    constexpr MvSig G = S::sig;
    constexpr int K = G.K, NS = G.ns, D = G.D;
    static_assert(NS > 0 && NS <= kFoldSlots && D > 0 && D <= NS, "block shape");
    constexpr int W = K * kBlock;
    __shared__ unsigned long long lds4[4];
#ifdef WSMC_TABLES_LDS
    wsmc_tables_to_lds();   // before any log / exp (every thread: it ends in a barrier)
#endif
    const wsmc_term* tp = reinterpret_cast<const wsmc_term*>(pb);
    const FoldSeg* segs = reinterpret_cast<const FoldSeg*>(pb + G.ntmpl * (int)sizeof(wsmc_term));
    const double* cst =
        reinterpret_cast<const double*>(pb + G.ntmpl * (int)sizeof(wsmc_term) + (G.nnew + G.nold) * (int)sizeof(FoldSeg));
    const int th = threadIdx.x;
    // slots one lazy Resample behind read through its ancestors (gated by its decision), as are
    // the carried scores
    const int smask = (G.smask && a.lg.anc && a.lg.dec->resampled) ? G.smask : 0;
    const bool slag = a.mc.anc && a.mc.dec->resampled;
    const int32_t* arow = smask ? a.lg.anc : a.mc.anc;
    bool ok[K];
    int64_t gi[K], ai[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        gi[p] = (int64_t)blockIdx.x * W + p * kBlock + th;
        ok[p] = gi[p] < a.N;
        ai[p] = (ok[p] && (smask || slag)) ? (int64_t)arow[gi[p]] : gi[p];
    }
    double v[K][NS];
#pragma unroll
    for (int p = 0; p < K; ++p)
#pragma unroll
        for (int q = 0; q < NS; ++q) v[p][q] = ok[p] ? a.fs.p[q][((smask >> q) & 1) ? ai[p] : gi[p]] : 0.0;
    double so[K], sn[K], lpr[K];
    int chg[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        so[p] = (ok[p] && G.carry) ? a.mc.in[slag ? ai[p] : gi[p]] : 0.0;
        chg[p] = 0;
    }
    const bool run = !a.mc.gate || a.mc.gate->resampled;
    const int nrun = run ? a.flag[2] : 0;   // the combine's count (uniform)
    mv_fold<S, kMvSegs, G.nold, K, NS>(so, v, tp, segs + G.nnew, cst);
#pragma unroll
    for (int m = 0; m < G.nm; ++m) {
        if (m >= nrun) break;   // uniform
        const int o = G.off[m], dm = G.off[m + 1] - G.off[m];
        const double* Lm = a.Lb + 16 * m;
        double pr[K][4];
        unsigned long long acc = 0;
#pragma unroll
        for (int p = 0; p < K; ++p) {
            lpr[p] = 0.0;
            double xi[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < 4; k += 2)
                if (k < dm)
                    wsmc_normal_pair(wsmc_rng_block(a.seed, a.mb.op_prop[m], (uint64_t)(a.goff + gi[p]), (uint32_t)(k >> 1)),
                                     &xi[k], &xi[k + 1]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pr[p][k] = 0.0;
                if (k >= dm) continue;
                const int u = o + k;
                double dz = 0.0;
#pragma unroll
                for (int jj = 0; jj <= k; ++jj) dz = dz + Lm[k * dm + jj] * xi[jj];
                const double x = v[p][u];
                const bool bd = (G.bnd >> u) & 1, flo = (G.flo >> u) & 1, fhi = (G.fhi >> u) & 1;
                double xn = x + dz;
                if (bd) {   // the bounds' finiteness known at compile time: only its case's code
                    double dj;
                    xn = wsmc_bounded_step(x, dz, a.mb.lo[u], a.mb.hi[u], a.mb.lgw[u], flo, fhi, &dj);
                    lpr[p] = lpr[p] + dj;
                }
                pr[p][k] = xn;
            }
        }
        // the proposal's fold reads the proposed values at this move's targets
        double vn[K][NS];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            sn[p] = 0.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) vn[p][q] = (q >= o && q < o + dm) ? pr[p][q - o < 0 ? 0 : (q - o) & 3] : v[p][q];
        }
        mv_fold<S, 0, G.nnew, K, NS>(sn, vn, tp, segs, cst);
#pragma unroll
        for (int p = 0; p < K; ++p) {
            if (!ok[p]) continue;
            const double uu = wsmc_uniform_k(a.seed, a.mb.op_acc[m], (uint64_t)(a.goff + gi[p]), 0);
            const bool ac = move_accept(uu, (lpr[p] + sn[p]) - so[p]);   // strict; NaN rejects (src/transformers.jl:615)
            if (ac) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < dm) v[p][o + k] = pr[p][k];
                chg[p] |= ((1 << dm) - 1) << o;
                acc += 1;
                so[p] = sn[p];
            }
        }
        if (a.accepted) {   // uniform
            acc = mv_block_sum(acc, lds4);
            if (th == 0 && acc) atomicAdd(acc_slot(a.accepted, m, blockIdx.x), acc);
        }
    }
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (!ok[p]) continue;
#pragma unroll
        for (int u = 0; u < D; ++u)
            if (((G.lagt | chg[p]) >> u) & 1) a.mb.tout[u][gi[p]] = v[p][u];
        a.mc.out[gi[p]] = so[p];
    }
    if (G.lagt && blockIdx.x == 0 && th == 0)   // the device column table follows the moved fronts
#pragma unroll
        for (int u = 0; u < D; ++u)
            if ((G.lagt >> u) & 1) a.tab[a.mb.tcol[u]] = a.mb.tout[u];
}

}  // namespace wsmc
