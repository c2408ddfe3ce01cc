// wsmc_ew.h — the device-visible records shared by libwsmc and the statement-batch kernels it
// compiles at run time (csrc/wsmc_jit.hip): nothing here includes the HIP runtime, so hiprtc
// builds it from the embedded text (build.py) exactly as hipcc builds it into the library.
#pragma once

#include "wsmc.h"
#include "wsmc_math.h"
#include "wsmc_terms.h"

namespace wsmc {

constexpr int kBlock = 256;            // threads per workgroup (4 waves of 64)
constexpr int kSlots = 64;             // max-accumulator slots (blockIdx % 64)

// Max accumulator of one Resample: 64 ordered-encoded slots, one per block group
// (blockIdx % 64), filled with read-filtered atomicMax. One 128-B line per slot: memory-side
// atomics and filtered loads to one line serialise, so the slots must not share lines.
struct MaxSlots {
    unsigned long long v[kSlots][16];
};

// Resample outcome for one invocation (one step of a fused run).
constexpr int kDecRing = 1024;   // asynchronous Resample decisions held before a forced resolve
struct Decision {
    int32_t resampled;
    int32_t ntasks;     // ancestor-fill tasks of this shard (<= ntiles + N / kRsChunk + 1)
    double mean;        // this shard's post-resample log-weight
    double ess;         // global ESS/N
    double M;           // this shard's max log-weight
};

// The Resample statistics' tiles and per-particle parts (include/wsmc_math.h wsmc_qparts),
// shared by the library's kernels and the statement batches compiled at run time
constexpr int kRsTile = 1024;    // particles per resample tile
constexpr int kPart = 4;         // per-tile partials: sum q, sum q2, sum wf2, sum wf (all exact)
constexpr int kGroupLine = 8;    // u64 words of a tile group's line (sum q, max tile sum, ...)
// q and the tile accumulators of q, q2, wf2, wf: all four are exact integers held in f64
// (q, q2 <= 2^K <= 2^43 and wf, wf2 < 2^42), so a 1024-particle tile's sums stay below 2^53
// (wsmc_qbits) and f64 accumulation is exact and order-free — no 64-bit integer arithmetic or
// conversion per particle.
struct QAcc {
    double Q = 0.0, Q2 = 0.0, WF2 = 0.0, WF = 0.0;
};
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
// an exact integer-valued double in [0, 2^52) -> u64 (the low mantissa bits of d + 2^52)
__device__ __forceinline__ unsigned long long d_small_to_u64(double d) {
    return __builtin_bit_cast(unsigned long long, d + 4503599627370496.0) - 0x4330000000000000ull;
}
__device__ __forceinline__ unsigned long long qacc_add(QAcc& a, double e, double sK) {
    e = e > 0.0 ? e : 0.0;                                  // -inf weights, NaN: all parts 0
    const double sc = e * sK;
    const double qd = wsmc_floor(sc);
    const double wf = wsmc_floor((sc - qd) * 4398046511104.0);      // 2^42
    const double sc2 = (e * e) * sK;
    const double q2d = wsmc_floor(sc2);
    const double wf2 = wsmc_floor((sc2 - q2d) * 4398046511104.0);
    a.Q = a.Q + qd;
    a.Q2 = a.Q2 + q2d;
    a.WF2 = a.WF2 + wf2;
    a.WF = a.WF + wf;
    return d_small_to_u64(qd);
}
#endif

// A batch of consecutive elementwise statements (Assign / Sample / Observe / Weight) run as one
// kernel, each particle taking the statements in order (csrc/wsmc_api.hip ew_*). The batch
// travels in the kernel's arguments (read in place through the kernarg segment).
constexpr int kEwOps = 6;       // statements a batch holds
constexpr int kEwSlots = 16;    // columns the Sample / weight terms read
constexpr int kEwRows = 12;     // LDS rows (one column component each, a value per thread)
constexpr int kEwPre = 10;      // components loaded into LDS rows at the start
struct EwAssign {
    wsmc_operand e[4];
    const double* p[4][2];      // operand components resolved to pointers
    uint32_t lag;               // bit 2k+m: operand read one lazy Resample behind (the batch's row)
    int8_t fwd[4][2];           // >= 0: the operand is an LDS row (an earlier statement's output)
};
struct EwSample {
    wsmc_dist d;                // operand columns renumbered to the batch's slots
    unsigned long long op;
    int32_t has_sd, pad;
    double sd;                  // a constant MvNormal variance's sqrt (host-evaluated)
};
struct EwWeigh {
    wsmc_term t;                // operand columns renumbered to the batch's slots
    wsmc_logmemo lm0;           // a constant scale's log / reciprocal (host-evaluated)
};
struct EwOp {
    int16_t kind;               // 0 Assign, 1 Sample, 2 Observe / Weight
    int16_t nostore;            // a Sample whose output is recomputed when read (VirtCol): rows only
    int16_t dim;
    int16_t out_row;            // >= 0: the output's components also go to LDS rows out_row..
                                // (later statements of the batch read them there)
    double* out;                // Assign / Sample destination (components N apart)
    union {
        EwAssign a;
        EwSample s;
        EwWeigh w;
    };
};
struct EwBatch {
    int32_t nops, ntab;
    int32_t has_w, nslots;
    const int32_t* anc;         // the newest lazy Resample's ancestors (lagged Assign operands)
    const Decision* dec;        // and its decision
    double* w;
    const Decision* wreset;     // a pending weight reset (the first weight term applies it)
    MaxSlots* ms;               // the max of the final weights (zero on entry)
    MaxSlots* ms_next;          // zeroed by block 0
    double** tab;               // device column table: entries moved by Assigns into fresh buffers
    double* tab_out[4];
    int32_t tab_col[4];
    // the Sample / weight terms read their columns from LDS: slot s at rows slot_row[s] +
    // component (an earlier statement's output, or loaded at the start: pre_src -> pre_row)
    const double* slot[kEwSlots];
    int8_t slot_row[kEwSlots];
    int32_t nrows, npre;
    const double* pre_src[kEwPre];
    int8_t pre_row[kEwPre];
    int8_t pre_lag[kEwPre];     // loaded through the ancestor row
    EwOp ops[kEwOps];
    // the Resample statistics of the final weights (EwSig::qs, round 6; the statement path's
    // form of the fused run's statistics in the propagate): every particle's q against the
    // guessed reference point R_g = wsmc_qref(fl(fl(*qs_base + qb[0]) + qb[1]) ...) — the
    // entering weights' max plus each weight term's largest value, a bound of the new max —
    // into qbuf, each 1024-particle tile's partials into tilep and its sum q into its group's
    // line (grp, G tiles a group); R_g into rg_out, which k_rs_qfix checks against the max
    const double* qs_base;
    double* rg_out;
    unsigned long long* qbuf;
    unsigned long long* tilep;
    unsigned long long* grp;
    int32_t G, nqb;
    double qb[kEwOps];
};
}  // namespace wsmc
