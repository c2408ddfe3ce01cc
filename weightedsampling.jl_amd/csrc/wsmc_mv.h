// wsmc_mv.h — the Move kernels' argument structures and acceptance test, shared by the library
// (csrc/wsmc_kernels.hip) and the Move blocks compiled for their shape at run time
// (csrc/wsmc_mv_body.h, csrc/wsmc_jit.hip); hiprtc-compilable.
#pragma once

#include "wsmc_ew.h"

namespace wsmc {

// A Move's accepted count: 64 line-separated slots per move (block b adds into slot b mod 64;
// one address for every block serialised the atomics: 15.6k blocks of a 4M Move at one
// particle a thread cost 40 us a Move), summed by launch_acc_sum before the host reads them
constexpr int kAccSlots = 64, kAccStride = 16, kAccMove = kAccSlots * kAccStride;
__host__ __device__ inline unsigned long long* acc_slot(unsigned long long* acc, int m, unsigned block) {
    return acc + (size_t)m * kAccMove + (size_t)(block % kAccSlots) * kAccStride;
}

// Move over a compiled tape (operands renumbered to slots; the targets are slots 0..d-1)
constexpr int kFoldSlots = 16;
struct FoldSlots {
    const double* p[kFoldSlots];   // slot s = column component values [N]
    double* t[4];                  // the target columns (written on accept)
    int32_t n;
    int32_t heavy;                 // transcendental-heavy terms (oscillator means): one particle per thread
    int32_t lean;                  // every term is a run term or scalar (wsmc_term_is_scalar): the lean fold
};
// The fold as a program of segments over the compiled tape: a run of consecutive Normal
// terms that differ only in their constants (the observations of a model's loop, e.g.
// examples/damped_oscillator.jl:36 or examples/linear_regression.jl:21) is one segment whose
// per-particle invariants (the mean's column reads, sigma and its log) are evaluated once;
// its terms' constants are packed in `cst`. Aff: (c0, coef0, coef1, y) per term. Osc: rotation
// runs back to back, each (t_a, d, m, n, y_0 .. y_{n-1}) — n terms of one rotation block of
// wsmc_osc_link, the first the block's term m (its anchor and m rotations by the step d), each
// next one rotation further (m and n ride as osc_run_word bits). Every other term is a
// one-term segment.
enum { kSegTerm = 0, kSegNormalOsc = 1, kSegNormalAff = 2 };
WSMC_HD double osc_run_word(int32_t v) { return wsmc_bits2d((uint64_t)(uint32_t)v); }
WSMC_HD int32_t osc_run_int(double w) { return (int32_t)(uint32_t)wsmc_d2bits(w); }
struct FoldSeg {
    int32_t kind;
    int32_t count;   // terms in the segment
    int32_t tmpl;    // index of its first term in the compiled tape
    int32_t coff;    // offset of its constants (the layouts above)
    int32_t soff;    // a constant scale: offset of its Normal pair (c, rh) in the constants
                     // (wsmc_scale_pre, evaluated once on the host), else -1
    int32_t pad;     // 24 B: the constants after the segments stay 8-aligned
};
// the carried Move scores of one Move (ping-pong when a lazy Resample came in between: the
// scores are then read through its ancestors, gated by its decision, and written to `out`)
struct MoveCarry {
    const double* in;
    double* out;
    const int32_t* anc = nullptr;
    const Decision* dec = nullptr;
    const Decision* gate = nullptr;   // a gated Move (wsmc_move_gated): only the scores are carried
                                      // on when !gate->resampled
};
// targets one lazy Resample behind: read through its ancestors, gated by its decision
struct MomLag {
    const int32_t* anc;
    const Decision* dec;
    int32_t mask;
};
// a block of autoRW Moves on disjoint targets in one pass (wsmc_move_block): union targets
// u = 0..D-1 (the fold's slots 0..D-1, D <= 8), move m owns [off[m], off[m+1])
constexpr int kBlkTargets = 8;
struct MoveBlk {
    int32_t nm;
    int8_t off[5];
    int8_t pad[3];
    int32_t bnd;                 // bit u: the bounded transform applies to union target u
    int32_t lag_targets;         // bit u: target u read through the lag row, written in full to tout
    int16_t tcol[kBlkTargets];   // column ids (device table entries moved to tout when lagged)
    double min_step[4];          // per move
    unsigned long long op_prop[4], op_acc[4];
    double* tout[kBlkTargets];   // per union target: where its values go
    double lo[kBlkTargets], hi[kBlkTargets];
    double lgw[kBlkTargets];     // log(hi - lo) of a bounded interval (host-evaluated)
};
// a block's fold program in its kernel's arguments (the block's other arguments are larger
// than a single Move's, so fewer words than ProgInline). Layout: [templates | segments |
// constants], offsets in bytes
constexpr int kProgBlkWords = 360;
struct ProgInlineBlk {
    int32_t seg_off, cst_off, seg_old0, pad;
    unsigned long long w[kProgBlkWords];
};

// The Metropolis test `wsmc_log(u) < d` (src/transformers.jl:615: strict, NaN rejects), with the
// same decision bits and without the double log wherever a single-precision log settles it:
// L = v_log_f32((float)u) ln 2 is within 2^-24 (the rounding of u) plus a few float ulps of log u
// for u >= 2^-60, so |L - wsmc_log(u)| < 2^-13 + 2^-16 |L| leaves the comparison decided unless d
// lies within that band of L (a fraction ~1e-4 of the draws); those, u < 2^-60 and a non-finite d
// take the restated log (tests/test_gpu_moves_accept.py checks the bound on the device).
__device__ __forceinline__ bool move_accept(double u, double d) {
    if (u >= 8.673617379884035e-19 && wsmc_fabs(d) <= 1e300) {   // the second also rejects NaN
        const double L = (double)__builtin_amdgcn_logf((float)u) * 0.69314718055994530942;
        const double e = 1.220703125e-4 + 1.52587890625e-5 * wsmc_fabs(L);
        if (L + e < d) return true;
        if (L - e >= d) return false;
    }
    return wsmc_log(u) < d;
}

}  // namespace wsmc
