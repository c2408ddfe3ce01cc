// wsmc_internal.h — runtime structures of libwsmc (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <deque>
#include <atomic>
#include <functional>
#include <string>
#include <vector>

#include "wsmc.h"
#include "wsmc_math.h"
#include "wsmc_terms.h"
#include "wsmc_ew.h"
#include "wsmc_mv.h"
#include "wsmc_mv_body.h"

namespace wsmc {

// Environment switches for A/B experiments (tools/): kernel variants, ablations and
// alternative paths, read only by a diagnostic build (tools/build_variant.py NAME -DWSMC_DIAG_BUILD,
// selected with WSMC_LIB). The product library ignores them, so no stray variable in a user's
// environment can change its results. The ones it honours change no result (tests select paths
// with them, or they only print): WSMC_DIAG_NO_GRAPH (the fused run enqueued eagerly, for kernel
// tracers), WSMC_DIAG_NO_JIT (the interpreter kernels in place of the run-time compiled ones),
// WSMC_DIAG_CAPTURE_FAIL (the eager fallback after a failed graph capture), WSMC_DIAG_NO_PEER
// (exact shards trace lineages through windows instead of peer reads), WSMC_EXACT_EAGER (the
// host-driven exact-shard run), WSMC_EAGER_GATHER (columns gathered at each Resample instead of
// lazily), and WSMC_JIT_DUMP / WSMC_JIT_VERBOSE / WSMC_TRACE_DEBUG (diagnostic output only).
inline const char* diag_env(const char* name) {
#ifdef WSMC_DIAG_BUILD
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

constexpr int kItems = 8;              // particles per thread in the tile kernels
constexpr int kTile = kBlock * kItems; // 2048 particles per tile (canonical reduction tile)
constexpr int kRsBlock = 1024;         // threads of the reduce workgroup
#ifndef WSMC_SUM_BLOCK
#define WSMC_SUM_BLOCK 256                // build-time override for block-size experiments (tools/)
#endif
#ifndef WSMC_SCAN_BLOCK
#define WSMC_SCAN_BLOCK 256
#endif
constexpr int kSumBlock = WSMC_SUM_BLOCK;   // threads of the weight-statistics workgroup (1024 / kSumBlock particles each)
constexpr int kScanBlock = WSMC_SCAN_BLOCK;   // threads of the ancestor-fill workgroup (1024 / kScanBlock particles each)
constexpr int kRsChunk = 2048;         // ancestor slots per fill task
constexpr int kMaxCols = 4096;
constexpr int kMaxShards = 8;     // one node: up to 8 GPUs

// One shard's weight statistics: what the ranks exchange (64 B per step).
struct ShardRecord {
    unsigned long long menc;   // ordered encoding of the shard max log-weight
    unsigned long long Q;      // sum q_i
    unsigned long long q2;     // sum q2_i (ESS: the fixed point of e^2, include/wsmc_math.h wsmc_qparts)
    unsigned long long wf2lo, wf2hi;  // sum wf2_i (u128): sum floor(e^2 2^(K+42)) = Q2 2^42 + Wf2
    unsigned long long wflo, wfhi;  // sum wf_i (u128): sum floor(e 2^(K+42)) = Q 2^42 + Wf
    unsigned long long n;      // shard size
};

constexpr int kRedPart = 6;   // reduce-kernel parts: Q, Q2, Wf2 lo32/hi, Wf lo32/hi

// Exact cross-shard resampling: the global CDF and the slot windows,
// built on the device from the all-gathered records (k_rs_decide_exact). Shard g's
// particles own the contiguous global slots [seg[g], seg[g+1]) (ancestors are monotone).
struct ExactPlan {
    unsigned long long Q;       // global sum q (q relative to the global max, K from the global N)
    unsigned long long N;       // global particle count
    unsigned long long cbase;   // this shard's CDF offset: sum of the lower ranks' Q
    unsigned long long a, b;    // this shard's slot window [a, b)
    unsigned long long seg[kMaxShards + 1];    // slot windows of every rank
    unsigned long long gofs[kMaxShards + 1];   // particle offsets of every rank
};

struct Column {
    std::string name;
    int32_t dim = 1;
    double* front = nullptr;   // live data (what getcol returns) as of `epoch`
    double* back = nullptr;    // ping-pong / scratch buffer
    int64_t epoch = 0;         // lazy genealogy: front holds the values before log entry `epoch`
    int64_t touch = -1;        // the last epoch in which an operator read or wrote the column
};

// Lazy genealogy of the generic store (ColumnStore.resample!, src/stores.jl:105-128): a
// Resample records its ancestor row and its device-side decision as one log entry; only the
// columns an operator touched since the previous Resample are gathered at once. A column
// left behind (history such as x{t}) is brought up to date by one trace over the log when
// something reads it — bit-identical, since a gather is a copy.
struct AncRow {
    int32_t* anc = nullptr;        // [N] ancestors of the entry
    Decision* dec = nullptr;       // the entry's decision (gates the trace: identity if it did not resample)
    int32_t known = -1;            // host knowledge of dec->resampled: -1 pending (asynchronous Resample)
};
constexpr int kTraceLev = 96;      // log entries one trace launch walks
constexpr int kTraceCols = 48;     // column components one trace launch writes
struct TraceComp {
    double* dst;
    const double* src;
    int32_t level;                 // entries to apply (1 = the newest only), ascending in the table
    int32_t col;                   // column id when this is its component 0 (-1 otherwise): the
                                   // device pointer table entry is set to dst (the new front)
};
struct TraceArgs {
    const int32_t* rows[kTraceLev];      // rows[0] = the newest entry
    const Decision* decs[kTraceLev];
    TraceComp comp[kTraceCols];
    int32_t nlev, ncomp;
    const int32_t* a_in;                 // composed indices before rows[0] (null = identity)
    int32_t* a_out;                      // composed indices after the last row (null = not kept)
    double** tab;                        // the context's device column-pointer table
};

// cached HIP graph of one fused-run configuration
struct RunGraph {
    std::string key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    void* owned = nullptr;     // device tables baked into the graph
};

struct MultiState;   // wsmc_multi.hip
struct EwBatch;      // below
}  // namespace wsmc

struct wsmc_ctx {
    wsmc::MultiState* multi = nullptr;   // a handle over several shards (wsmc_create_multi)
    int device = 0;
    hipStream_t stream = nullptr;
    // asynchronous Resamples (no flag requested): their decisions are copied into a pinned
    // ring and folded into resampled / n_resamples / last_ess at the next host read
    wsmc::Decision* dec_ring = nullptr;
    wsmc::Decision* dec_ring_dev = nullptr;   // the ring as the device addresses it (host-mapped)
    void* pinned_dev = nullptr;               // `pinned` as the device addresses it
    int dec_pending = 0;
    bool no_graph = false;   // a sharded run's capture failed once: run it eagerly
    // the max of the weights as the last Observe / Weight left them (double-buffered slots:
    // each such launch maxes into wslots[wnext] and zeroes the other); valid while
    // wmax_seq == wseq, the count of weight writes
    wsmc::MaxSlots* wslots[2] = {nullptr, nullptr};
    int wnext = 0, wmax_buf = -1;
    uint64_t wseq = 0, wmax_seq = ~0ull;
    // slots holding the max of the current weights (an Observe's, or a fused Resample's after
    // its weight reset), valid while cur_max_seq == wseq: a Move's autoRW skips its max pass
    wsmc::MaxSlots* cur_max = nullptr;
    uint64_t cur_max_seq = ~0ull;
    // a fused generic Resample's weight reset, not yet applied to `w` (the decision on the
    // device): the next Observe / Weight applies it in its kernel, any other call first runs
    // the gated reset (settle_weights, from CHECK_CTX)
    wsmc::Decision* w_reset_pending = nullptr;
    int64_t N = 0;
    uint64_t seed = 0;

    // shard / RCCL
    int world = 1, rank = 0;
    int64_t goff = 0, gN = 0;
    ncclComm_t comm = nullptr;
    // a shard of a multi-device handle (wsmc_multi.hip): the handle's abort request. Only the
    // shard's own thread touches its communicator: before every collective and while it waits
    // for its stream it checks the request and, when set, aborts its own communicator (a
    // collective missing a failed peer would never complete) and leaves with `released` set
    const std::atomic<bool>* peer_abort = nullptr;
    bool released = false;
    double comm_timeout_s = 0.0;                // wsmc_comm_set_timeout: bound on a stream wait (0: none)
    wsmc_exchange_fn host_exchange = nullptr;   // host-side record exchange (instead of RCCL)
    bool host_inproc = false;                   // ... between threads of this process (a multi-device
                                                // handle's: a memcpy), not a caller's transport
    int32_t inject_fail = 0;                    // wsmc_debug_inject_failure: fail the nth next record exchange
    bool inject_earg = false;                   // ... as WSMC_EARG (nth >= 1000) instead of WSMC_EHIP
    int64_t exchanges = 0;                      // exchanges (collectives / host rendezvous) issued so far
    unsigned long long* run_grp = nullptr;      // [T+1][ngroups][kGroupLine] fused-run group sums
    // Move score cache: each particle's fold over the first scache_terms tape terms (its
    // score after its last move); -1 = invalid (a column the tape reads was rewritten)
    unsigned long long* xchg = nullptr;   // sharded moves: small all-gather buffer (16 words per rank)
    double* scache = nullptr;
    double* scache_back = nullptr;
    int32_t scache_terms = -1;
    void* host_user = nullptr;

    // store
    std::vector<wsmc::Column> cols;
    double** d_colptr = nullptr;     // device table of front pointers
    bool colptr_dirty = true;

    // SMCState
    double* w = nullptr;
    int32_t resampled = 0, weights_changed = 0, depth = 0;
    double last_ess = 0.0;
    uint64_t op = 0;
    int64_t n_resamples = 0;

    // score tape
    std::vector<wsmc_term> tape;
    wsmc_term* d_tape = nullptr;
    int64_t d_tape_cap = 0, d_tape_n = 0;

    // scratch
    int32_t* anc = nullptr;                 // last ancestors [N]
    double* tmp = nullptr;                  // [4N]
    unsigned long long* tilep = nullptr;    // [nrstiles * kPart] per-tile integer partials
    unsigned long long* tileOff = nullptr;  // [nrstiles] exclusive prefix of the tiles' sum q
    int32_t* taskOff = nullptr;             // [nrstiles] first overflow fill task of each tile
    int32_t* taskTile = nullptr;            // [N / kRsChunk + nrstiles + 1] tile of each overflow task
    unsigned long long* qbuf = nullptr;     // [N] integer weights q_i of the last weight-statistics pass
    unsigned long long* cdf = nullptr;      // [N] tile-local CDF of q + spacing tile sums (multinomial; lazy)
    // exact sharding (wsmc_comm_set_shard_mode)
    int32_t shard_mode = 0;                 // WSMC_SHARD_ISLAND / WSMC_SHARD_EXACT
    wsmc::ExactPlan* xp = nullptr;          // [1] device plan
    wsmc::ShardRecord* comb = nullptr;      // [1] combined (global) record
    int32_t* anc_out = nullptr;             // [gN] the window's ancestors (local particle ids)
    bool task_global = false;               // taskTile sized for a window of up to gN slots
    unsigned long long* xbuf = nullptr;     // send + receive buffers (words)
    size_t xbuf_cap = 0;
    double** d_comp = nullptr;              // [2 * cap] component pointer tables (src, dst)
    double* xrun[9] = {};                    // exact-sharded fused run: gathered / scratch pair buffers
    int32_t* lineage[2] = {};                // [N] global lineage ids (distributed trace-back)
    // exact-sharded fused run without host round trips (enqueue_ssm2d_exact)
    double* xpairs = nullptr;               // [6N] x, v, dv pairs received from a neighbour, by slot
    unsigned long long* xnb = nullptr;      // [4][x_cap][kXWords]: send left, right; receive left, right
    int64_t xnb_cap = 0;                    // slots per block allocated
    unsigned long long* xwin = nullptr;     // [4][T][x_ctr][3]: trace windows sent left, right; received
    int64_t xwin_words = 0;                 // words per block allocated
    unsigned long long* xstat = nullptr;    // [kMaxShards][kXStat], this rank's at rank * kXStat
    double* w_save = nullptr;               // [N] the weights at the run's start (re-run after an overflow)
    wsmc::MaxSlots* xms = nullptr;          // [T+1][world] every rank's max slots per step (all-gathered)
    int64_t xms_n = 0;
    int32_t* xanc = nullptr;                // [T][xanc_stride] ancestor rows: margin, this rank's N slots, margin
    unsigned long long* xlines = nullptr;   // [T+1][world][line words] every rank's statistics group lines
    int64_t xlines_words = 0;
    int64_t xanc_words = 0, xanc_stride = 0;
    int64_t x_cap = 0, x_ctr = 0;           // block / window sizes in use (0: defaults; grown on overflow)
    unsigned long long x_need = 0, x_exc = 0;   // the last run's largest block / lineage excursion
    int64_t x_overflows = 0;                // runs re-done on the eager path
    bool x_eager = false;                   // the blocks grew past half a shard (particles move
                                            // far): later runs take the eager path directly
    bool x_trace = false;                   // the trace windows would need half a shard (lineages
                                            // wander far): later runs ship no windows and trace the
                                            // history across ranks after the run (exact_trace_history)
    int64_t x_traces = 0;                   // runs whose history was traced across ranks
    bool peer_ok = false;                   // every rank is a shard of this process's multi-device
                                            // handle and can read the others' memory (same device,
                                            // or peer access over xGMI): the exact trace-back reads
                                            // the owners' ancestor rows and history in place
    unsigned long long* xpeer = nullptr;    // [kMaxShards][8] every rank's trace-back words (all-gathered)
    wsmc_term* d_ctape = nullptr;           // compiled Move tape (slot operands)
    int64_t d_ctape_cap = 0;
    void* d_prog = nullptr;                 // compiled fold program: segments, then constants
    int64_t d_prog_cap = 0;                 // bytes
    // device copies of the last few fold programs, keyed by content: a sweep alternates a few
    // programs (C5's two Moves repeat theirs five times a step), so most Moves upload nothing
    struct ProgSlot {
        std::vector<char> host;             // the bytes the device copy holds
        void* dev = nullptr;
        int64_t cap = 0;
        uint64_t used = 0;                  // LRU stamp
    };
    ProgSlot prog_slots[4];
    uint64_t prog_tick = 0;
    int64_t prog_uploads = 0, prog_hits = 0;
    wsmc::EwBatch* ew = nullptr;            // elementwise statements not launched yet (one kernel at
    unsigned ew_feat = 0;                   // the next other entry point); the oscillator mean seen
    std::vector<int32_t> ew_lag;            // columns the batch reads one Resample behind
    struct EwRow {
        const double* p;                    // column buffer
        int lag;                            // read through the batch's ancestor row
        int row;                            // its first LDS row in the batch
    };
    std::vector<EwRow> ew_rows;
    std::vector<const double*> ew_unstaged; // outputs of the batch without rows (no later LDS reads)
    // Sample outputs not stored (EwOp.nostore): a Sample whose distribution reads no column
    // (dv ~ MvNormal(0, 0.1 I)) has values that are a function of (seed, op, particle) alone,
    // so the batch keeps them in rows for its later statements and the column is written only
    // if something reads it before the next full overwrite (the next step's Sample): VirtCol
    // entries, materialised by every reader (virt_*), dropped by an overwrite
    struct VirtCol {
        int32_t col;
        const double* buf;                  // the column's front when sampled (checked on use)
        wsmc_dist d;
        uint64_t op;
    };
    std::vector<VirtCol> virt;              // launched batches' unstored Sample outputs
    std::vector<VirtCol> ew_virt;           // ... of the open batch (moved to virt at its launch)
    wsmc_term ew_first;                     // the batch's first statement as called (a batch of one
                                            // launches the statement's own kernel)
    char* prog_stage = nullptr;             // pinned staging ring of the programs too large to ride
    int64_t prog_stage_cap = 0, prog_stage_at = 0;   // in the Move's arguments (ProgInline)
    unsigned long long* rs_grp[2] = {nullptr, nullptr};   // generic Resample's group lines (double-buffered)
    int rs_grp_cur = 0;
    // the Resample statistics in the statement batch (round 6): rs_qs[0] the max of the weights
    // the last fused Resample left (its record block writes it), rs_qs[1] the batch's guessed
    // reference point; valid for the next batch while rs_base_seq == wseq. ew_qs_ok: the open
    // batch's weight terms all have a bound (EwBatch::qb) and it started from that base
    double* rs_qs = nullptr;
    uint64_t rs_base_seq = ~0ull;
    bool ew_qs_ok = false;
    int64_t rs_qs_batches = 0;   // Resamples whose statistics the batch took (wsmc_debug_run_stats)
    size_t d_comp_cap = 0;
    double* tilepart = nullptr;             // [16 * ntiles] canonical-sum tile partials
    wsmc::MaxSlots* mslots = nullptr;       // [1] max slots of one generic resample / evidence
    wsmc::ShardRecord* rec = nullptr;       // [world] shard records of one generic resample
    wsmc::Decision* dec = nullptr;          // [1] decision of one generic resample
    double* mom = nullptr;                  // [64] moment / covariance / Cholesky results
    int32_t* dflag = nullptr;               // [4] device error flags
    unsigned long long* ucount = nullptr;   // 4 moves x kAccSlots line-separated count slots, then [4] sums
    void* pinned = nullptr;                 // 4 KB pinned staging
    int64_t ntiles = 0;      // canonical-sum tiles (2048)
    int64_t nrstiles = 0;    // resample tiles (1024)

    // lazy genealogy (AncRow): entries for epochs [log_base, epoch)
    bool lazy = true;
    int64_t epoch = 0, log_base = 0;
    std::deque<wsmc::AncRow> alog;
    std::vector<wsmc::AncRow> row_pool;     // free rows (ancestors + decision)
    std::vector<void*> row_slabs;           // the rows' memory: slabs of several rows, one hipMalloc each
    int64_t rows_made = 0;
    // each pending asynchronous decision's ancestors: a lazy log entry (epoch >= 0) or an eager
    // store's own row (epoch -1), held until the decision is read back
    struct PendingRow {
        int64_t epoch;
        wsmc::AncRow row;
    };
    std::vector<PendingRow> dec_rows;
    // carried Move scores one lazy Resample behind (their gather deferred to the next Move,
    // which reads them through this log entry's ancestors)
    const int32_t* scache_anc = nullptr;
    const wsmc::Decision* scache_dec = nullptr;
    int64_t scache_lag_epoch = -1;
    int32_t* anc_last = nullptr;            // wsmc_last_ancestors: newest row known to have resampled
    int64_t anc_last_epoch = -1;            // its log entry (lazy), -1 otherwise
    wsmc::AncRow anc_keep{};                // eager store: the row anc_last points at (owned)
    wsmc::Decision* dec_always = nullptr;   // [1] resampled = 1 (explicit resample!(store, idx))
    bool move_pending = false;              // an asynchronous Move's PD flag not yet read back
    bool dflag_zero = false;                // dflag known to be all zero (no memset needed)
    const wsmc::Decision* move_gate = nullptr;   // wsmc_move_gated: the deciding Resample's device decision

    // fused runner state
    int32_t T_alloc = 0;
    wsmc::MaxSlots* run_max = nullptr;      // [T+1]
    double* run_rg = nullptr;               // [T+1] the propagate's guessed reference points (round 6)
    unsigned long long* run_nfix = nullptr; // [1] steps whose statistics k_rs_qfix recomputed (cumulative)
    double* run_w0 = nullptr;               // [2][N] the weights a run started from (its replay's start), by parity
    // asynchronous fused runs (round 6): wsmc_ssm2d_run returns once its graph is launched; the
    // decisions come back into pinned memory behind it and the next entry point (or the next run,
    // after its own launch) folds them in — and re-does the run if its guessed reference point
    // missed. A run's per-call buffers alternate by parity so the next run can be enqueued while
    // it executes.
    struct RunPend* run_pend = nullptr;     // the run whose decisions are still on the device
    int run_par = 0;                        // the next run's buffer parity
    uint64_t* run_op = nullptr;             // this run's op-base word: run_params + 4 parity
    wsmc::Decision* run_hdec = nullptr;     // pinned, coherent [2][T+1]: each parity's decisions, written
                                            // by the run's trace-back kernel
    double* run_hstage = nullptr;           // pinned, coherent [2][2T + 4]: each parity's op-base word
                                            // (bits) and observations, read by the run's head kernel
    hipEvent_t run_ev[2] = {nullptr, nullptr};   // recorded behind each parity's read-back
    int64_t run_missed = 0, run_replays = 0; // single GPU: steps whose guess missed, runs re-done
    wsmc::ShardRecord* run_rec = nullptr;   // [(T+1) * world]
    wsmc::Decision* run_dec = nullptr;      // [T+1]
    int32_t* anc_log = nullptr;             // [T][N]
    double* obs = nullptr;                  // [T*2] this run's observations (obs_buf + parity)
    double* obs_buf = nullptr;              // [2][T+1][2]
    double* vscratch = nullptr;             // [2N] second ping-pong buffer for v / x
    double* xscratch = nullptr;             // [2N]
    uint64_t* run_params = nullptr;         // [8] device copy of per-run values (op base)
    std::vector<wsmc::RunGraph> graphs;
    bool timing = false;
    std::vector<hipEvent_t> events;
    wsmc_run_timing last_timing{};
};

namespace wsmc {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define WSMC_HIP(expr)                                                                   \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return ::wsmc::fail(WSMC_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// a multi-device handle asked its shards to abort (a peer failed): this shard's communicator
// is aborted by its own thread, the call leaves with WSMC_ERCCL (released)
bool peer_aborted(wsmc_ctx* c);
// hipStreamSynchronize that a peer's abort request interrupts (multi-device shards poll)
hipError_t ctx_sync(wsmc_ctx* c, hipStream_t s);
#define WSMC_RCCL_GUARD(ctx)                                                             \
    if (::wsmc::peer_aborted(ctx)) return ::wsmc::fail(WSMC_ERCCL, "communicator aborted: a peer shard failed")
#define WSMC_RCCL(expr)                                                                  \
    do {                                                                                 \
        ncclResult_t _r = (expr);                                                        \
        if (_r != ncclSuccess)                                                           \
            return ::wsmc::fail(WSMC_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// ---- kernel launchers (wsmc_kernels.hip) -------------------------------------------
// gather-on-read of operand columns one lazy-log entry behind (k_assign)
struct Indirect {
    const int32_t* row = nullptr;     // the newest log entry's ancestors
    const Decision* dec = nullptr;    // its decision (identity when it did not resample)
    uint32_t mask = 0;                // operand slots read through the row
    int32_t tab_col = -1;             // column whose table entry becomes `out`
    double** tab = nullptr;
    const double* const* front = nullptr;   // host: every column's front buffer (resolves operands)
};
hipError_t launch_assign(hipStream_t s, double* out, int dim, const wsmc_operand* expr,
                         double* const* cols, int64_t N, const Indirect& ind);
// Assign of a general expression (wsmc_assign_expr): the program with its column reads resolved
// to component pointers; lag = read through `row` (one lazy Resample behind)
struct XIns {
    int32_t op, lag;
    const double* p;   // WSMC_X_COL: the component
    double c;
};
struct XProg {
    double* out;
    int64_t N;
    const int32_t* row;
    const Decision* dec;
    double** tab;      // tab_col >= 0: `out` becomes that column's table entry
    int32_t tab_col, dim, any_lag, pad;
    int32_t len[4];
    XIns ins[WSMC_XPROG_MAX];
};
hipError_t launch_assign_expr(hipStream_t s, const XProg& x);
// the statement batch (csrc/wsmc_ew.h) on the interpreter kernel, or on its signature's kernel
// compiled at run time (csrc/wsmc_jit.hip; hipErrorNotSupported: none, run the interpreter)
hipError_t launch_ew_jit(hipStream_t s, const EwBatch& b, unsigned feat, uint64_t seed, int64_t goff, int64_t N,
                         int device);
void ew_jit_stats(int64_t* out);   // compiled, failed, launched, interpreted, compile time (us)
bool ew_pair_ok(const EwBatch& b, int64_t N);   // the batch can run two particles a thread
int ew_jit_selfcheck(std::string& err);   // hiprtc builds a representative signature (no device)
hipError_t launch_ew_batch(hipStream_t s, const EwBatch& b, unsigned feat, uint64_t seed, int64_t goff, int64_t N);
// a batch of one Assign: k_assign with the batch's resolved pointers
hipError_t launch_ew_assign1(hipStream_t s, const EwBatch& b, double* const* cols, int64_t N);
hipError_t launch_sample(hipStream_t s, double* out, int dim, const wsmc_dist& d, uint64_t seed,
                         uint64_t op, int64_t goff, double* const* cols, int64_t N);
hipError_t launch_sample_importance(hipStream_t s, double* out, int dim, const wsmc_dist& prop,
                                    const wsmc_dist& targ, double* w, uint64_t seed, uint64_t op,
                                    int64_t goff, double* const* cols, int64_t N);
hipError_t launch_weigh(hipStream_t s, const wsmc_term& t, double* w, double* const* cols, int64_t N, MaxSlots* ms,
                        MaxSlots* ms_next, const Decision* wreset = nullptr);
hipError_t launch_rs_max(hipStream_t s, const double* w, int64_t N, MaxSlots* ms);
hipError_t launch_rs_sums(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms,
                          unsigned long long* tilep, unsigned long long* qbuf,
                          hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr,
                          unsigned long long* grp = nullptr, int G = 1,
                          int64_t Nk = 0 /* N of K = 63 - ceil(log2 N): the global N when exact */,
                          int nms = 1 /* slot sets in ms (exact shards: every rank's, all-gathered) */,
                          int gall = 0 /* exact shards: every part into the group lines (grp) */);
struct FillPlan {          // ancestor-fill task planning (in the reduce kernel)
    const unsigned long long* tilep;   // per-tile partials (sum q first)
    int32_t* taskOff;
    int32_t* taskTile;
    int scheme;
    uint64_t seed, op;
    const uint64_t* op_dev;
    int64_t slot_base;
    const ExactPlan* xp = nullptr;     // exact sharding: global Q / N / offsets, window-relative slots
    double* w_reset = nullptr;         // generic Resample: the tile blocks reset the weights to dec->mean
    Decision* host_dec = nullptr;      // generic Resample: the decision also written to host-mapped memory
    unsigned long long* grp_zero = nullptr;   // fused fill: the next call's group lines, zeroed by its record block
    MaxSlots* ms_reset = nullptr;      // fused fill: the record block writes the reset weights' max here
    int64_t grp_zero_words = 0;
    // exact shards without host round trips: the fill writes global ids (id_base + local) into
    // a row covering the global slots [row_lo, row_hi), and a slot outside sets xstat bit 0
    int32_t id_base = 0;
    unsigned long long row_lo = 0, row_hi = 0;
    unsigned long long* xstat = nullptr;
    // ... the fused fill (k_rs_fill_fused) takes its totals from every rank's all-gathered
    // group lines (xlines, xstride words per rank) and its record block decides for all
    const unsigned long long* xlines = nullptr;
    int64_t xstride = 0;
    const MaxSlots* xms = nullptr;              // every rank's max slots (all-gathered)
    unsigned long long n_global = 0;
    // ... and the reduce kernel takes the single-GPU decision first (k_rs_decide_exact's work)
    const ShardRecord* dx_recs = nullptr;
    ShardRecord* dx_comb = nullptr;
    Decision* dx_dec = nullptr;
    ExactPlan* dx_xp = nullptr;
    int32_t dx_world = 0, dx_rank = 0;
    double dx_ess = 0.0;
    // the fused run's guessed reference point (round 6): the record block compares it with
    // wsmc_qref of the step's max and counts a miss (the run is then re-done on the exact path)
    const double* rg_check = nullptr;
    int32_t* rg_miss = nullptr;
    // generic Resample (round 6): the record block writes the max of the weights it leaves (the
    // log-mean if it resampled, else the max it read) — the next statement batch's guess starts
    // from it (EwBatch::qs_base)
    double* base_out = nullptr;
};
hipError_t launch_rs_reduce(hipStream_t s, const MaxSlots* ms, const unsigned long long* tilep, int64_t N,
                            unsigned long long* tileOff, ShardRecord* rec, int decide_local, double ess_min,
                            Decision* dec, const FillPlan* plan, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr,
                            unsigned long long* esum = nullptr, int nms = 1);
hipError_t launch_rs_decide(hipStream_t s, const ShardRecord* recs, int world, int rank, double ess_min,
                            Decision* dec);
// describe(): median sort keys, the StatsBase walk on the sorted prefix, histogram counts
hipError_t launch_median_keys(hipStream_t s, const double* x, const unsigned long long* q, int64_t N,
                              unsigned long long* kq, unsigned long long* kv);
hipError_t launch_median_pick(hipStream_t s, const unsigned long long* v, const unsigned long long* q,
                              const unsigned long long* S, int64_t N, double* out);
hipError_t launch_hist(hipStream_t s, const double* x, const unsigned long long* q, int64_t N, const double* edges,
                       unsigned long long* cnt);
struct FoldProgram {
    const FoldSeg* seg_new;    // the s_new fold, terms [0, n)
    const FoldSeg* seg_old;    // the s_old fold, terms [cache_from or 0, n)
    int32_t nseg_new, nseg_old;
    const double* cst;
};
// a lean fold program small enough to travel in the Move kernel's own arguments (read from
// the kernarg segment with scalar loads): no upload copy per Move. Layout as the device
// program: [templates | segments | constants], offsets in bytes
constexpr int kProgInlineWords = 416;   // 3328 B (the kernel's other arguments stay under 4 KB)
struct ProgInline {
    int32_t seg_off, cst_off, seg_old0, pad;
    unsigned long long w[kProgInlineWords];
};
// the moments of a block: one pass over the union of the targets (sep = 0, D <= 4: every
// move's totals a sub-block of the union's), or one pass per move (its totals at
// tilepart + toff[m] * ntiles)
// a Move block on its signature's compiled kernel (csrc/wsmc_jit.hip); hipErrorNotSupported: none
// (JIT off or the signature failed to compile) — the caller runs the interpreter kernels
hipError_t launch_mv_jit(hipStream_t s, const MvSig& sig, const ProgInlineBlk* pin, const MvArgs& a, int device);
int mv_jit_selfcheck(std::string& err);
void mv_jit_stats(int64_t* out);
hipError_t launch_debug_log_screen(hipStream_t s, const double* u, int64_t n, double* out);
hipError_t launch_autorw_final_blk(hipStream_t s, const double* tilepart, int64_t ntiles, const MoveBlk& mb,
                                   int sep, const int32_t* toff, double* mom, int32_t* flag, const Decision* gate);
hipError_t launch_move_blk(hipStream_t s, const ProgInlineBlk* pin, const wsmc_term* ctape, const FoldProgram& prog,
                           const FoldSlots& fs, const MoveBlk& mb, const double* Lb, uint64_t seed, int64_t goff,
                           int64_t N, unsigned long long* accepted, const int32_t* flag, const MoveCarry& mc,
                           int32_t cache_from, const int32_t* lag_anc, const Decision* lag_dec, int lag_mask,
                           double** tab);
hipError_t launch_move_c(hipStream_t s, const wsmc_term* ctape, int32_t nterms, int32_t depth, const FoldSlots& fs,
                         const int32_t* tcols, int d, const double* lo, const double* hi, int bounded,
                         const double* L, uint64_t seed, uint64_t op_prop, uint64_t op_acc, int64_t goff, int64_t N,
                         unsigned long long* accepted, const int32_t* flag, const MoveCarry& mc, int32_t cache_from,
                         const FoldProgram& prog, const ProgInline* pin = nullptr);
// exact-sharded fused run: contiguous slices of (x pair, ancestor) by global index for the
// distributed trace-back, the lineage lookup, pairs -> SoA
hipError_t launch_trace_pack(hipStream_t s, const double* xpairs, const int32_t* arow, int64_t start, int64_t count,
                             unsigned long long* out);
hipError_t launch_trace_lookup(hipStream_t s, const unsigned long long* recv, int64_t lo, const int32_t* a, int64_t n,
                               double* xout, int32_t* anext, int use_a);
hipError_t launch_pairs_to_soa(hipStream_t s, const double* pairs, double* soa, int64_t n);
hipError_t launch_fill_const2(hipStream_t s, double* soa, double v0, double v1, int64_t n);
hipError_t launch_iota(hipStream_t s, int32_t* a, int64_t n, int64_t base);
// sample(state, n; replace): draws on the integer CDF / Efraimidis-Spirakis keys / row gather
hipError_t launch_sample_draws(hipStream_t s, int64_t n, int64_t N, const ShardRecord* rec,
                               const unsigned long long* tileOff, const unsigned long long* lcdf, uint64_t seed,
                               uint64_t op, int64_t* out);
hipError_t launch_es_keys(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, uint64_t seed, uint64_t op,
                          unsigned long long* keys, unsigned long long* idx);
hipError_t launch_gather_rows(hipStream_t s, const double* src, int64_t N, int dim, const int64_t* idx, int64_t n,
                              double* out);
// exact sharding: global max from the all-gathered per-rank maxima (words[world]) into ms
hipError_t launch_max_adopt(hipStream_t s, const unsigned long long* words, int world, MaxSlots* ms);
hipError_t launch_autorw_max(hipStream_t s, const unsigned long long* words, int world, int stride, MaxSlots* ms);
// sharded autoRW: rank-order combine of the all-gathered moment totals (pass 1 means, pass 2 factor)
hipError_t launch_autorw_combine(hipStream_t s, const unsigned long long* xchg, int world, int stride, int d,
                                 int pass, double min_step, double* mom, int32_t* flag);
hipError_t launch_max_publish(hipStream_t s, const MaxSlots* ms, unsigned long long* word);
// autoRW in one pass (include/wsmc_math.h wsmc_autorw_factor): pivoted canonical tile partials,
// their one-block combine and factor; sharded: publish (max word, pivot), rank-order combine
struct MomZero {   // words the moments kernel zeroes first (block 0): a Move block's flags, counters
    int32_t* flag;
    unsigned long long* count;
};
hipError_t launch_autorw_moments(hipStream_t s, const double* w, const MaxSlots* ms, double* const* cols,
                                 const int32_t* tcols, int d, const double* lo, const double* hi,
                                 const unsigned long long* pv, int64_t N, double* tilepart,
                                 const Decision* wreset = nullptr, const Decision* gate = nullptr,
                                 const int32_t* lag_anc = nullptr, const Decision* lag_dec = nullptr, int lag_mask = 0,
                                 int32_t* zflag = nullptr, unsigned long long* zcount = nullptr);
hipError_t launch_acc_sum(hipStream_t s, const unsigned long long* acc, unsigned long long* out,
                          const int32_t* flag = nullptr, int32_t* flag_out = nullptr);
hipError_t launch_autorw_final(hipStream_t s, const double* tilepart, int64_t ntiles, int d, double min_step,
                               double* mom, int32_t* flag, int raw, const Decision* gate = nullptr);
hipError_t launch_autorw_publish(hipStream_t s, const MaxSlots* ms, double* const* cols, const int32_t* tcols, int d,
                                 const double* lo, const double* hi, unsigned long long* out);
hipError_t launch_autorw_combine1(hipStream_t s, const unsigned long long* xchg, int world, int stride, int d,
                                  double min_step, double* mom, int32_t* flag);
// exact sharding: records summed as integers (the single-GPU decision bits), slot windows
hipError_t launch_rs_decide_exact(hipStream_t s, const ShardRecord* recs, int world, int rank, double ess_min,
                                  const FillPlan& plan, ShardRecord* comb, Decision* dec, ExactPlan* xp);
// exact sharding: slot -> owner routing of the filled window (local slots written in place,
// the rest packed per peer as [component][slot] u64 blocks), and the receive side
struct ExactRoute {
    int32_t world, rank, ncomp;                 // ncomp double components (+1 ancestor id word)
    int32_t stride = 1;                         // element stride of every component (2: pair layout)
    unsigned long long a, b;                    // this rank's window
    unsigned long long gofs[kMaxShards + 1];
    unsigned long long sendoff[kMaxShards];     // words, per peer
    unsigned long long recvoff[kMaxShards];     // words, per source
    unsigned long long recvlen[kMaxShards];     // slots, per source
    unsigned long long recvdst[kMaxShards];     // first local slot, per source
    unsigned long long recvpre[kMaxShards + 1]; // prefix of recvlen (slots)
};
hipError_t launch_exact_pack(hipStream_t s, const ExactRoute& rt, const int32_t* anc_out,
                             const double* const* src, double* const* dst, int32_t* anc_local,
                             unsigned long long* sendbuf);
hipError_t launch_exact_unpack(hipStream_t s, const ExactRoute& rt, const unsigned long long* recvbuf,
                               double* const* dst, int32_t* anc_local);
// exact-sharded fused run without host round trips: every count comes from the
// device plan (ExactPlan), particles move between neighbouring ranks only, through fixed-size
// blocks of `cap` slots per side (a collective's size must be fixed at enqueue / capture
// time); a slot that needs a farther rank or a larger block sets the overflow flag and the
// host re-runs the filter on the eager path (it starts from constants: the same bits).
constexpr int kXWords = 7;                      // a moving slot: x pair, v pair, dv pair, global ancestor id
constexpr int kXStat = 8;                       // u64 stats: [0] overflow bits, [1] largest block needed
                                                // (slots), [2] largest trace-back excursion (ids)
struct ExactStep {
    const ExactPlan* xp;
    const Decision* dec;
    const int32_t* row;                         // this step's ancestor row from its left margin (cap slots
                                                // before the rank's range; global ids)
    const double* x;                            // this rank's particles at the step (pairs, pre-resample)
    const double* v;
    const double* dv;                           // valid at the last step only (moved anyway)
    int32_t* anc_row;                           // row + cap: [N] global ancestor ids of this rank's slots
    unsigned long long* send[2];                // [cap * kXWords] to the left (0) / right (1) neighbour
    const unsigned long long* recv[2];          // from the left / right neighbour
    double* xr;                                 // [2N] pairs received, by slot
    double* vr;
    double* dvr;
    unsigned long long* stat;                   // [kXStat]
    int64_t cap, N, goff;
    int32_t rank, world;
};
hipError_t launch_exact_route(hipStream_t s, const ExactStep& e);
hipError_t launch_exact_recv(hipStream_t s, const ExactStep& e);
// trace-back windows: for every level L = 1..T and each side, `ctr` ids at the edge of this
// rank's range: x_{L+1} (pair) and the ancestor of step L-1 (the id itself if it did not
// resample), 3 words each, [L-1][side][ctr][3]
struct ExactWin {
    const double* const* hist_work;             // [T+2] x_t working buffers (pairs)
    const int32_t* anc_log;
    int64_t anc_stride;
    const Decision* dec;                        // [T+1]
    unsigned long long* out;
    int64_t ctr, N, goff;
    int32_t T, has_left, has_right;
};
hipError_t launch_exact_window_pack(hipStream_t s, const ExactWin& w);
struct PutWords {   // eight words for k_put_words (kernel arguments: capturable, no host buffer)
    unsigned long long w[8];
};
struct ExactFinal {
    int32_t T, keep_history;
    int64_t N, goff, ctr;
    double x0[2];
    double* const* hist_work;
    double* const* hist_out;
    const double* x_work;                       // no-history: x_{T+1}
    double* x_out;
    const double* v_work;
    double* v_out;
    const double* dv_work;
    double* dv_out;
    const double* xr;                           // the last step's received pairs
    const double* vr;
    const double* dvr;
    double* w;
    const int32_t* anc_log;
    int64_t anc_stride;
    const Decision* dec;
    const unsigned long long* win[2];           // windows received from the left / right neighbour
    unsigned long long* stat;
    // peer reads (ctx peer_ok): every rank's {ancestor rows at its own slot 0, row stride,
    // history table, first global index, N} (8 words a rank); lineages outside this shard read
    // the owner's rows and history in place, no windows
    const unsigned long long* peer = nullptr;
    int32_t world = 1;
};
hipError_t launch_exact_final(hipStream_t s, const ExactFinal& f);
hipError_t launch_put_words(hipStream_t s, unsigned long long* dst, const unsigned long long (&w)[8]);
hipError_t launch_rs_scan(hipStream_t s, int64_t N, const ShardRecord* rec, const Decision* dec,
                          const FillPlan& plan, const unsigned long long* tileOff,
                          const unsigned long long* qbuf, int32_t* anc, hipEvent_t e0 = nullptr,
                          hipEvent_t e1 = nullptr);
// multinomial: weight statistics + tile-local CDF + spacing tile sums, then the fill
// (the reduce kernel turns the spacing sums into offsets when given esum)
hipError_t launch_rs_sums_multi(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, const FillPlan& plan,
                                unsigned long long* tilep, unsigned long long* lcdf, unsigned long long* esum,
                                uint32_t* ebuf, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_rs_multinomial(hipStream_t s, int64_t N, const ShardRecord* rec, const Decision* dec,
                                 const FillPlan& plan, const unsigned long long* tileOff,
                                 const unsigned long long* lcdf, const unsigned long long* esum,
                                 const uint32_t* ebuf, int32_t* anc, hipEvent_t e0 = nullptr,
                                 hipEvent_t e1 = nullptr);
// fused run: group sums of q (kGroupLine u64 per group, one line each, csrc/wsmc_ew.h) replace
// the reduce kernel
constexpr int kMaxWorld = kMaxShards;   // ranks of one node
inline int group_tiles(int64_t N) {   // tiles per group: ~sqrt(ntiles), >= 16
    const int64_t nt = (N + kRsTile - 1) / kRsTile;
    int G = 16;
    while ((int64_t)G * G < nt) ++G;
    return G;
}
hipError_t launch_rs_fill_fused(hipStream_t s, int64_t N, const FillPlan& plan, const unsigned long long* grp,
                                int G, const MaxSlots* ms, double ess_min, ShardRecord* rec, Decision* dec,
                                const unsigned long long* qbuf, int32_t* anc, hipEvent_t e0 = nullptr,
                                hipEvent_t e1 = nullptr, const double* wq = nullptr);
hipError_t launch_gather(hipStream_t s, double* dst, const double* src, const int32_t* anc, int64_t N);
hipError_t launch_lazy_trace(hipStream_t s, const TraceArgs& a, int64_t N);
// up to kGatherSet (dst, src) column-component pairs of one Resample, passed by value
constexpr int kGatherSet = 48;
struct GatherSet {
    double* dst[kGatherSet];
    const double* src[kGatherSet];
    int32_t col[kGatherSet];       // column id for its component 0 (-1 otherwise): table entry := dst
    double** tab;                  // the device column-pointer table (null: not updated)
    int n;
};
hipError_t launch_resample_apply(hipStream_t s, const GatherSet& gs, const int32_t* anc, const Decision* dec,
                                 double* w, int64_t N);
hipError_t launch_gather_dec(hipStream_t s, double* dst, const double* src, const int32_t* anc, const Decision* dec,
                             int64_t N);
hipError_t launch_sample_draws_shard(hipStream_t s, int64_t n, int64_t N, const unsigned long long* cdf,
                                     unsigned long long base, unsigned long long Qloc, unsigned long long Q,
                                     uint64_t seed, uint64_t op, int64_t goff, int64_t* out);
hipError_t launch_es_keys_shard(hipStream_t s, const double* w, int64_t N, int64_t gN, int64_t goff,
                                const MaxSlots* ms, uint64_t seed, uint64_t op, unsigned long long* keys,
                                unsigned long long* idx);
// ms != null: when the step resampled, ms is rewritten to hold the max of the reset weights
hipError_t launch_fill_weights(hipStream_t s, double* w, const Decision* dec, int64_t N, MaxSlots* ms = nullptr);
hipError_t launch_log_evidence_stats(hipStream_t s, const double* w, int64_t N, MaxSlots* ms,
                                     unsigned long long* tilep, unsigned long long* qbuf,
                                     unsigned long long* tileOff, ShardRecord* rec);
hipError_t launch_score(hipStream_t s, const wsmc_term* tape, int32_t n, int32_t depth,
                        double* const* cols, int64_t N, double* out);
hipError_t launch_moments(hipStream_t s, const double* w, const MaxSlots* ms, double* const* cols,
                          const int32_t* tcols, int d, const double* lo, const double* hi,
                          int pass, const double* mom, int64_t N, double* tilepart);
hipError_t launch_moments_final(hipStream_t s, const double* tilepart, int64_t ntiles, int d,
                                int pass, double min_step, double* mom, int32_t* flag, int raw = 0);
hipError_t launch_moments_expr(hipStream_t s, const double* w, const MaxSlots* ms, double* const* cols,
                               const wsmc_operand* ex, int d, int pass, const double* mom, int64_t N,
                               double* tilepart);
hipError_t launch_minmax(hipStream_t s, const double* x, int64_t N, MaxSlots* ms);
hipError_t launch_move(hipStream_t s, const wsmc_term* tape, int32_t nterms, int32_t depth,
                       double* const* cols, const int32_t* tcols, int d, const double* lo,
                       const double* hi, int bounded, const double* L, uint64_t seed,
                       uint64_t op_prop, uint64_t op_acc, int64_t goff, int64_t N,
                       unsigned long long* accepted, const int32_t* flag, double* scache, int32_t cache_from);
hipError_t launch_diversity_keys(hipStream_t s, const double* x, unsigned long long* keys, int64_t N);
hipError_t launch_count_unique(hipStream_t s, const unsigned long long* keys, int64_t N,
                               unsigned long long* count);

// fused 2D SSM
struct Ssm2dArgs {
    int32_t t;                 // 1-based step
    int32_t keep_history;
    int64_t N;
    int64_t goff;
    uint64_t seed;
    const uint64_t* op_dev;    // op base of the run (device)
    const double* obs;         // [T][2]
    double x0[2], v0[2];
    double q_sd;               // sqrt(q_var)
    double r_var;
    double c0;                 // -(2 log 2pi + 2 log r_var)/2 (host-computed, shared math)
    // working buffers are particle-major pairs [N][2] (the output columns are SoA [2][N])
    const double* x_prev;      // x_t (pre-resample numbering of step t-1), unused at t = 1
    double* x_next;
    const double* v_prev;
    double* v_next;
    double* dv;                // written at the last step only (the column keeps the latest draw)
    double* w;                 // [N]
    const int32_t* anc_prev;   // [N] ancestors of step t-1 (8-B aligned row)
    const Decision* dec_prev;  // decision of step t-1 (nullptr at t = 1)
    MaxSlots* ms;              // this step's max slots
    int32_t identity = 0;      // exact shards: the previous state is already in slot order (no gather)
    // exact shards without host round trips: anc_prev holds global ids; an ancestor outside
    // [goff, goff + N) arrived from a neighbour and its pair is xr / vr at the slot itself
    const double* xr = nullptr;
    const double* vr = nullptr;
    // island shards: the previous step's decision is taken here from its all-gathered records
    // (every block, the same bits as k_rs_decide) instead of by its own launch; block 0 stores
    // it at dec_out for the host and the trace-back
    const ShardRecord* recs_prev = nullptr;
    Decision* dec_out = nullptr;
    int32_t world = 1, rank = 0;
    double ess_min = 0.0;
    // the Resample statistics in the propagate (round 6, k_ssm2d_prop QS): the previous step's max
    // slots (the bound when it did not resample), where the guessed reference point goes (for
    // k_rs_qfix), this step's tile partials and group lines, and q itself when the fill reads it
    // (null: the fill recomputes q from the weights)
    bool qstat = false;
    double* w_save = nullptr;          // the first step's incoming weights go here (a replay's start)
    const MaxSlots* ms_prev = nullptr;
    double* rg_out = nullptr;
    unsigned long long* tilep = nullptr;
    unsigned long long* grp = nullptr;
    int32_t G = 1;
    unsigned long long* qbuf = nullptr;
};
// k_rs_qfix: the statistics again against ceil(M) when the propagate's guess was not it
hipError_t launch_rs_qfix(hipStream_t s, const double* w, int64_t N, const MaxSlots* ms, const double* rg,
                          unsigned long long* tilep, unsigned long long* qbuf, unsigned long long* grp, int G,
                          unsigned long long* nfix, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_ssm2d_propagate(hipStream_t s, const Ssm2dArgs& a, hipEvent_t e0 = nullptr,
                                  hipEvent_t e1 = nullptr);
struct Ssm2dFinal {
    int32_t T;
    int32_t keep_history;
    int64_t N;
    double x0[2];
    double* const* hist_work;  // device table [T+2]: working buffers x_t (pre-resample), t=2..T+1
    double* const* hist_out;   // device table [T+2]: final (front) buffers of x_t, t=1..T+1
    const double* x_work;      // no-history: x_{T+1} working buffer
    double* x_out;
    const double* v_work;
    double* v_out;
    const double* dv_work;
    double* dv_out;
    double* w;
    const int32_t* anc_log;    // [T][anc_stride]
    int64_t anc_stride;        // row stride of the ancestor log (N rounded up to 4)
    const Decision* dec;       // [T+1], index t
    // the run's read-back (block 0): every step's decision into pinned host memory; and the row
    // of the last step that resampled into last_anc (wsmc_last_ancestors after run!)
    Decision* hdec = nullptr;
    int32_t* last_anc = nullptr;
    // island shards: the last step's decision from its all-gathered records (see Ssm2dArgs)
    const ShardRecord* recs_last = nullptr;
    Decision* dec_out = nullptr;
    int32_t world = 1, rank = 0;
    double ess_min = 0.0;
};
// a fused run's head: zeroes its per-step max slots, decisions and group sums and copies its
// op-base word and observations from pinned host memory (one launch for three memsets and two
// copies)
struct RunHead {
    unsigned long long* z[3];
    int64_t zwords[3];
    const double* hstage;      // [op bits, pad, obs...]
    double* obs;
    int32_t nobs;
    uint64_t* op;
};
hipError_t launch_run_head(hipStream_t s, const RunHead& h);
hipError_t launch_ssm2d_finalize(hipStream_t s, const Ssm2dFinal& f, hipEvent_t e0 = nullptr,
                                 hipEvent_t e1 = nullptr);
hipError_t launch_delay(hipStream_t s, int microseconds);
// one handle over several devices (wsmc_multi.hip): the ABI entry points fan out
int multi_destroy(wsmc_ctx* c);
wsmc_ctx* multi_first(wsmc_ctx* c);
int multi_G(wsmc_ctx* c);
int multi_sync(wsmc_ctx* c);
int multi_get_state(wsmc_ctx* c, wsmc_state* out);
int multi_each(wsmc_ctx* c, const std::function<int(wsmc_ctx*)>& f);
int multi_col_download(wsmc_ctx* c, int32_t col, double* host);
int multi_col_upload(wsmc_ctx* c, int32_t col, const double* host);
int multi_weights(wsmc_ctx* c, const double* up, double* down);
int multi_score(wsmc_ctx* c, int32_t depth, double* host);
int multi_last_ancestors(wsmc_ctx* c, int32_t* host);
int multi_inject_failure(wsmc_ctx* c, int32_t shard, int32_t nth);
int multi_comm_info(wsmc_ctx* c, wsmc_comm_info_t* out);
int multi_gather_rows(wsmc_ctx* c, int32_t col, const int64_t* idx, int64_t n, double* out);
int multi_move(wsmc_ctx* c, int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
               const double* hi, int32_t target_depth, double diversity, int64_t* accepted_out);
hipError_t debug_kernel_bench(hipStream_t s, int kernel, int mode, int iters, const double* w, int64_t N,
                              MaxSlots* ms, unsigned long long* tilep, unsigned long long* qbuf,
                              unsigned long long* tileOff, ShardRecord* rec, Decision* dec, const FillPlan& plan,
                              int32_t* anc, double* stream4, float* ms_out);

}  // namespace wsmc
