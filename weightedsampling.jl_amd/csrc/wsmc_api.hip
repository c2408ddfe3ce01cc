// wsmc_api.hip — C ABI implementation: context, store, operators, fused runner, RCCL.
//
// Reference interfaces replaced (see include/wsmc.h for the per-function mapping):
//   AbstractParticleStore / ColumnStore   src/stores.jl:1-128
//   SMCState                              src/types.jl:48-78
//   apply!(...)                           src/transformers.jl:28-623
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <memory>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "wsmc_internal.h"

using namespace wsmc;

namespace wsmc {
bool peer_aborted(wsmc_ctx* c) {
    if (!c->peer_abort || !c->peer_abort->load(std::memory_order_acquire)) return false;
    if (c->comm) {   // this shard's thread is the only user of its communicator
        (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
    }
    c->released = true;
    return true;
}
hipError_t ctx_sync(wsmc_ctx* c, hipStream_t s) {
    const bool watch = c->comm && c->comm_timeout_s > 0.0;
    if (!c->peer_abort && !watch) return hipStreamSynchronize(s);
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return e;
        if (peer_aborted(c)) {
            // the abort ends the collectives in flight; what remains on the stream completes
            (void)hipStreamSynchronize(s);
            return hipErrorLaunchFailure;
        }
        if (watch && (spin & 255) == 255 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->comm_timeout_s) {
            // the watchdog (wsmc_comm_set_timeout): a collective's peer never arrived
            std::fprintf(stderr, "wsmc: a stream wait exceeded %.0f s (rank %d of %d): aborting its communicator\n",
                         c->comm_timeout_s, c->rank, c->world);
            (void)ncclCommAbort(c->comm);
            c->comm = nullptr;
            c->released = true;
            (void)hipStreamSynchronize(s);
            return hipErrorLaunchFailure;
        }
        if (spin < 4096)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace wsmc

// every entry point: the device, then any deferred weight reset applied before the call reads
// or writes the weights (CHECK_CTX_KEEP: the Observe / Weight path, which applies it itself)
// CHECK_CTX_EW: the elementwise statements (Assign / Sample / Observe / Weight), which join the
// pending batch (ew_*); every other entry point launches the batch first (CHECK_CTX_KEEP)
// CHECK_CTX_DEV: the device only (column creation: no state an asynchronous run changes);
// every other entry point first folds in an asynchronous fused run (resolve_run)
#define CHECK_CTX_DEV(ctx)                                               \
    do {                                                                 \
        if (!(ctx)) return fail(WSMC_EARG, "null context");              \
        WSMC_HIP(hipSetDevice((ctx)->device));                           \
    } while (0)
#define CHECK_CTX_EW(ctx)                                                \
    do {                                                                 \
        CHECK_CTX_DEV(ctx);                                              \
        if (int _r = resolve_run(ctx)) return _r;                        \
    } while (0)
#define CHECK_CTX_KEEP(ctx)                                              \
    do {                                                                 \
        CHECK_CTX_EW(ctx);                                               \
        if (int _r = ew_flush(ctx)) return _r;                           \
        if (int _r = virt_all(ctx)) return _r;                           \
    } while (0)
#define CHECK_CTX(ctx)                                                   \
    do {                                                                 \
        CHECK_CTX_KEEP(ctx);                                             \
        if ((ctx)->w_reset_pending) {                                    \
            WSMC_HIP(launch_fill_weights((ctx)->stream, (ctx)->w, (ctx)->w_reset_pending, (ctx)->N)); \
            (ctx)->w_reset_pending = nullptr;                            \
        }                                                                \
    } while (0)


static int resolve_run(wsmc_ctx* c);        // an asynchronous fused run's decisions (wsmc_ssm2d_run)
static int run_qstat_mode(int64_t N);       // where the Resample statistics are taken (0: their own kernel)
static void run_pend_free(RunPend* r);

// ---- the elementwise batch (EwBatch, csrc/wsmc_internal.h) ---------------------------------
// Consecutive Assign / Sample / Observe / Weight statements join one batch, launched as one
// kernel by the next other entry point (or when full). Each particle takes the statements in
// order, so a statement reading what an earlier one wrote reads its own particle's value; the
// one cross-particle read is an Assign operand one Resample behind (through the ancestors), so
// a statement writing such a column in place launches the batch first. One context only
// (shards exchange inside their operators); WSMC_DIAG_NO_BATCH=1 launches every statement alone.
static bool ew_enabled(const wsmc_ctx* c) {
    static const bool off = [] {
        const char* e = diag_env("WSMC_DIAG_NO_BATCH");
        return e && atoi(e) != 0;
    }();
    return !off && !(c->world > 1 || c->comm || c->host_exchange);
}
// qs_done: the batch carried the Resample statistics (EwBatch::qs_base, set by wsmc_resample)
// and its compiled kernel took them
static int ew_flush(wsmc_ctx* c, bool* qs_done = nullptr) {
    EwBatch* b = c->ew;
    if (qs_done) *qs_done = false;
    if (!b || b->nops == 0) return WSMC_OK;
    // the batch's signature compiled for its shape (csrc/wsmc_jit.hip); without it a batch of
    // one statement runs its own kernel (leaner than the interpreter's: no rows, no table)
    hipError_t e = launch_ew_jit(c->stream, *b, c->ew_feat, c->seed, c->goff, c->N, c->device);
    const bool launched_jit = e != hipErrorNotSupported;
    const EwOp& o0 = b->ops[0];
    if (launched_jit)
        ;
    else if (b->nops > 1)
        e = launch_ew_batch(c->stream, *b, c->ew_feat, c->seed, c->goff, c->N);
    else if (o0.kind == 0)
        e = launch_ew_assign1(c->stream, *b, c->d_colptr, c->N);
    else if (o0.kind == 1)
        e = launch_sample(c->stream, o0.out, o0.dim, c->ew_first.dist, c->seed, o0.s.op, c->goff, c->d_colptr, c->N);
    else
        e = launch_weigh(c->stream, c->ew_first, b->w, c->d_colptr, c->N, b->ms, b->ms_next, b->wreset);
    // the compiled batch and the interpreter leave nostore outputs unwritten (a batch of one
    // on its own kernel writes them): they become VirtCol entries
    const bool honoured = launched_jit || b->nops > 1;
    for (auto& v : c->ew_virt)
        if (honoured) c->virt.push_back(v);
    c->ew_virt.clear();
    if (qs_done) *qs_done = launched_jit && b->qs_base != nullptr && e == hipSuccess;
    b->qs_base = nullptr;
    b->nqb = 0;
    c->ew_qs_ok = false;
    b->nops = b->ntab = b->has_w = b->nslots = b->nrows = b->npre = 0;
    b->anc = nullptr;
    b->dec = nullptr;
    c->ew_feat = 0;
    c->ew_lag.clear();
    c->ew_rows.clear();
    c->ew_unstaged.clear();
    if (e != hipSuccess) return fail(WSMC_EHIP, std::string("statement batch: ") + hipGetErrorString(e));
    return WSMC_OK;
}
static EwBatch* ew_open(wsmc_ctx* c) {
    if (!c->ew) {
        c->ew = new EwBatch;
        std::memset(c->ew, 0, sizeof(EwBatch));
    }
    return c->ew;
}
// ---- unstored Sample outputs (wsmc_ctx::VirtCol) ------------------------------------------
// write column `col`'s values now: the Sample kernel of its entry, into the buffer it would
// have written (the same function of the same seed, op and particle indices: the same bits)
static int virt_write(wsmc_ctx* c, const wsmc_ctx::VirtCol& v) {
    if (c->cols[v.col].front != v.buf)
        return fail(WSMC_ESTATE, "unstored Sample output of column " + c->cols[v.col].name + " lost its buffer");
    WSMC_HIP(launch_sample(c->stream, const_cast<double*>(v.buf), v.d.dim, v.d, c->seed, v.op, c->goff, c->d_colptr,
                           c->N));
    return WSMC_OK;
}
// a statement or a kernel is about to read `col`: materialise it if its Sample left it unstored
static int virt_one(wsmc_ctx* c, int32_t col) {
    for (size_t k = 0; k < c->virt.size(); ++k)
        if (c->virt[k].col == col) {
            const wsmc_ctx::VirtCol v = c->virt[k];
            c->virt.erase(c->virt.begin() + (long)k);
            return virt_write(c, v);
        }
    return WSMC_OK;
}
static int virt_all(wsmc_ctx* c) {
    while (!c->virt.empty()) {
        const wsmc_ctx::VirtCol v = c->virt.back();
        c->virt.pop_back();
        if (int r = virt_write(c, v)) return r;
    }
    return WSMC_OK;
}
// `col` is about to be overwritten in full: its unstored values (of a launched batch or of the
// open one, whose later statements read them from rows) are never needed
static void virt_drop(wsmc_ctx* c, int32_t col) {
    for (auto* v : {&c->virt, &c->ew_virt})
        for (size_t k = 0; k < v->size(); ++k)
            if ((*v)[k].col == col) {
                v->erase(v->begin() + (long)k);
                break;
            }
}

static bool ew_reads_lagged(const wsmc_ctx* c, int32_t col) {
    for (int32_t x : c->ew_lag)
        if (x == col) return true;
    return false;
}
// the LDS rows of a column buffer in the batch, read directly or through the ancestors (-1: none)
static int ew_row_of(const wsmc_ctx* c, const double* p, int lag = 0) {
    for (const auto& e : c->ew_rows)
        if (e.p == p && e.lag == lag) return e.row;
    return -1;
}
// rows loaded at the start for a column (all its components); -1: no room
static int ew_preload(wsmc_ctx* c, EwBatch* b, const double* p, int dim, int lag) {
    if (b->nrows + dim > kEwRows || b->npre + dim > kEwPre) return -1;
    const int r = b->nrows;
    b->nrows += dim;
    for (int q = 0; q < dim; ++q) {
        b->pre_src[b->npre] = p + (int64_t)q * c->N;
        b->pre_row[b->npre] = (int8_t)(r + q);
        b->pre_lag[b->npre] = (int8_t)lag;
        b->npre += 1;
    }
    c->ew_rows.push_back({p, lag, r});
    return r;
}
// rows for a statement's output (its buffer keeps the rows it has: later readers see the new
// values there); -1: none left (the output is unstaged)
static int ew_out_rows(wsmc_ctx* c, EwBatch* b, const double* p, int dim) {
    int r = ew_row_of(c, p);
    if (r >= 0) return r;
    if (b->nrows + dim > kEwRows) {
        c->ew_unstaged.push_back(p);
        return -1;
    }
    r = b->nrows;
    b->nrows += dim;
    c->ew_rows.push_back({p, 0, r});
    return r;
}
// an operand's columns renumbered to the batch's slots, each slot's rows an earlier output's
// or loaded at the start; false: no room, or a column an earlier statement wrote without rows
static bool ew_remap(wsmc_ctx* c, EwBatch* b, wsmc_operand& o) {
    for (int m = 0; m < 2; ++m) {
        if (o.col[m] < 0) continue;
        const Column& col = c->cols[o.col[m]];
        const double* p = col.front;
        for (const double* u : c->ew_unstaged)
            if (u == p) return false;
        int s = -1;
        for (int k = 0; k < b->nslots; ++k)
            if (b->slot[k] == p) s = k;
        if (s < 0) {
            if (b->nslots == kEwSlots) return false;
            int r = ew_row_of(c, p);
            if (r < 0) r = ew_preload(c, b, p, col.dim, 0);   // not written in the batch: loaded at the start
            if (r < 0) return false;
            s = b->nslots++;
            b->slot[s] = p;
            b->slot_row[s] = (int8_t)r;
        }
        o.col[m] = s;
    }
    return true;
}
// a statement's operand columns staged all or none (the batch state restored on failure)
template <typename F>
static bool ew_stage(wsmc_ctx* c, EwBatch* b, F&& remap_all) {
    const int32_t ns = b->nslots, nr = b->nrows, np = b->npre;
    const size_t nrow = c->ew_rows.size();
    if (remap_all()) return true;
    b->nslots = ns;
    b->nrows = nr;
    b->npre = np;
    c->ew_rows.resize(nrow);
    return false;
}
static bool ew_remap_dist(wsmc_ctx* c, EwBatch* b, wsmc_dist& d) {
    for (int k = 0; k < 4; ++k)
        if (!ew_remap(c, b, d.mu[k])) return false;
    return ew_remap(c, b, d.scale);
}

// ---- helpers -------------------------------------------------------------------------
static int upload_colptr(wsmc_ctx* c) {
    if (!c->colptr_dirty) return WSMC_OK;
    WSMC_HIP(ctx_sync(c, c->stream));   // the pinned table may still be in flight
    double** host = reinterpret_cast<double**>(c->pinned);
    // pinned staging holds 512 pointers; larger tables go through a synchronous copy
    if (c->cols.size() <= 256) {
        for (size_t k = 0; k < c->cols.size(); ++k) host[k] = c->cols[k].front;
        WSMC_HIP(hipMemcpyAsync(c->d_colptr, host, sizeof(double*) * c->cols.size(), hipMemcpyHostToDevice,
                                c->stream));
    } else {
        std::vector<double*> tab(c->cols.size());
        for (size_t k = 0; k < c->cols.size(); ++k) tab[k] = c->cols[k].front;
        WSMC_HIP(hipMemcpyAsync(c->d_colptr, tab.data(), sizeof(double*) * tab.size(), hipMemcpyHostToDevice,
                                c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
    }
    c->colptr_dirty = false;
    return WSMC_OK;
}

static int upload_tape(wsmc_ctx* c) {
    const int64_t n = (int64_t)c->tape.size();
    if (c->d_tape_n == n) return WSMC_OK;
    if (n > c->d_tape_cap) {
        int64_t cap = c->d_tape_cap ? c->d_tape_cap : 64;
        while (cap < n) cap *= 2;
        WSMC_HIP(ctx_sync(c, c->stream));
        if (c->d_tape) WSMC_HIP(hipFree(c->d_tape));
        WSMC_HIP(hipMalloc(&c->d_tape, sizeof(wsmc_term) * cap));
        c->d_tape_cap = cap;
        c->d_tape_n = 0;
    }
    WSMC_HIP(hipMemcpyAsync(c->d_tape + c->d_tape_n, c->tape.data() + c->d_tape_n,
                            sizeof(wsmc_term) * (n - c->d_tape_n), hipMemcpyHostToDevice, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    c->d_tape_n = n;
    return WSMC_OK;
}

static bool valid_col(const wsmc_ctx* c, int32_t col) { return col >= 0 && col < (int32_t)c->cols.size(); }

static int check_operand(const wsmc_ctx* c, const wsmc_operand& o) {
    for (int k = 0; k < 2; ++k) {
        if (o.col[k] < 0) continue;
        if (!valid_col(c, o.col[k])) return fail(WSMC_EARG, "operand references an unknown column");
        if (o.comp[k] < 0 || o.comp[k] >= c->cols[o.col[k]].dim)
            return fail(WSMC_EARG, "operand component out of range for column " + c->cols[o.col[k]].name);
    }
    return WSMC_OK;
}

static int check_dist(const wsmc_ctx* c, const wsmc_dist& d) {
    if (d.family < WSMC_FAM_NORMAL || d.family > WSMC_FAM_GEOMETRIC) return fail(WSMC_EARG, "unknown family");
    if (d.dim < 1 || d.dim > 4) return fail(WSMC_EARG, "dist dim must be 1..4");
    if (d.family == WSMC_FAM_MVNORMAL && d.dim > WSMC_MVN_MAXDIM)
        return fail(WSMC_EARG, "MvNormal with a full covariance: dim must be 1..3");
    if (d.family != WSMC_FAM_MVNORMAL_ISO && d.family != WSMC_FAM_MVNORMAL && d.dim != 1)
        return fail(WSMC_EARG, "scalar family with dim != 1");
    if (d.mean_fn == WSMC_MEAN_OSCILLATOR && (d.family != WSMC_FAM_NORMAL))
        return fail(WSMC_EARG, "oscillator mean only for Normal");
    int r;
    for (int k = 0; k < 4; ++k)
        if ((r = check_operand(c, d.mu[k])) != WSMC_OK) return r;
    return check_operand(c, d.scale);
}

static wsmc_operand col_operand(int32_t col, int32_t comp) {
    wsmc_operand r;
    std::memset(&r, 0, sizeof(r));
    r.col[0] = col;
    r.comp[0] = comp;
    r.coef[0] = 1.0;
    r.col[1] = -1;
    return r;
}

// does any tape term read column `col` (its value, its distribution's arguments)?
static bool tape_reads(const wsmc_ctx* c, int32_t col) {
    auto uses = [&](const wsmc_operand& o) { return o.col[0] == col || o.col[1] == col; };
    for (const wsmc_term& t : c->tape) {
        for (int k = 0; k < 4; ++k)
            if (uses(t.x[k]) || uses(t.dist.mu[k])) return true;
        if (uses(t.dist.scale)) return true;
    }
    return false;
}
// the carried Move scores are no longer valid (they are refolded by the next Move)
static void scores_invalidate(wsmc_ctx* c) {
    c->scache_terms = -1;
    c->scache_anc = nullptr;
    c->scache_dec = nullptr;
    c->scache_lag_epoch = -1;
}
// a write to a column the tape reads changes past terms' values: the carried scores are stale
static void scores_touch(wsmc_ctx* c, int32_t col) {
    if (c->scache_terms >= 0 && tape_reads(c, col)) scores_invalidate(c);
}

// ColumnStore.resample! (src/stores.jl:105-128) of the given columns (and the carried Move
// scores) through `anc`, in k_resample_apply launches of up to kGatherSet components; the
// last one also resets the weights to dec->mean when w_reset is given. dec != null gates
// everything on the device-side decision (the asynchronous Resample: identity copies when it
// did not resample, so the front/back swap holds); null = an explicit resample!(store, idx).
// The gathered columns' values become those of epoch `to_epoch`.
static int gather_columns(wsmc_ctx* c, const std::vector<int32_t>& which, const int32_t* anc, const Decision* dec,
                          double* w_reset, int64_t to_epoch) {
    for (int32_t id : which)
        if (int r = virt_one(c, id)) return r;
    GatherSet gs;
    gs.n = 0;
    gs.tab = c->d_colptr;   // the kernel moves each gathered column's table entry to its new front
    auto flush = [&](bool last) -> hipError_t {
        const hipError_t e = launch_resample_apply(c->stream, gs, anc, dec, last ? w_reset : nullptr, c->N);
        gs.n = 0;
        return e;
    };
    auto add = [&](double* dst, const double* src, int32_t col) -> hipError_t {
        if (gs.n == kGatherSet) {
            const hipError_t e = flush(false);
            if (e != hipSuccess) return e;
        }
        gs.dst[gs.n] = dst;
        gs.src[gs.n] = src;
        gs.col[gs.n] = col;
        gs.n += 1;
        return hipSuccess;
    };
    for (int32_t id : which) {
        Column& col = c->cols[id];
        for (int k = 0; k < col.dim; ++k)
            WSMC_HIP(add(col.back + (int64_t)k * c->N, col.front + (int64_t)k * c->N, k == 0 ? id : -1));
        std::swap(col.front, col.back);
        col.epoch = to_epoch;
    }
    if (c->scache && c->scache_terms >= 0) {   // carried Move scores follow their particles
        WSMC_HIP(add(c->scache_back, c->scache, -1));
        std::swap(c->scache, c->scache_back);
    }
    WSMC_HIP(flush(true));
    return WSMC_OK;
}

// the carried scores' deferred gather, now (k_resample_apply through the lagged entry)
static int resolve_scache_lag(wsmc_ctx* c) {
    if (!c->scache_anc) return WSMC_OK;
    const int32_t* anc = c->scache_anc;
    const Decision* dec = c->scache_dec;
    c->scache_anc = nullptr;
    c->scache_dec = nullptr;
    c->scache_lag_epoch = -1;
    if (c->scache && c->scache_terms >= 0) return gather_columns(c, {}, anc, dec, nullptr, c->epoch);
    return WSMC_OK;
}

// ---- lazy genealogy (AncRow, wsmc_internal.h) ---------------------------------------------
static inline size_t row_anc_bytes(int64_t N) { return (sizeof(int32_t) * (size_t)N + 255) & ~(size_t)255; }
static int acquire_row(wsmc_ctx* c, AncRow* out) {
    if (c->row_pool.empty()) {
        // a slab of as many rows as exist (at least 4): a lazy log that keeps growing (columns
        // read one Resample behind) costs a hipMalloc every few Resamples, not one each — a
        // hipMalloc is tens of microseconds of host time, more than a step's launches. Capped at
        // 8 rows and 256 MB a slab (doubling at 8M particles, 32 MB a row, one row past
        // 32 took another 1 GB); slabs are freed with the context
        const size_t stride = row_anc_bytes(c->N) + 256;
        const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(8, (int64_t)((256u << 20) / stride)));
        const int64_t n = std::min<int64_t>(std::max<int64_t>(4, c->rows_made), std::max<int64_t>(cap, 1));
        void* p = nullptr;
        WSMC_HIP(hipMalloc(&p, stride * (size_t)n));
        c->row_slabs.push_back(p);
        c->rows_made += n;
        for (int64_t k = n - 1; k >= 0; --k) {
            char* q = reinterpret_cast<char*>(p) + stride * (size_t)k;
            AncRow r{};
            r.anc = reinterpret_cast<int32_t*>(q);
            r.dec = reinterpret_cast<Decision*>(q + row_anc_bytes(c->N));
            c->row_pool.push_back(r);
        }
    }
    *out = c->row_pool.back();
    c->row_pool.pop_back();
    out->known = -1;
    return WSMC_OK;
}
// entries no column, no pending decision and no last_ancestors query can reach return to the pool
static void gc_log(wsmc_ctx* c) {
    int64_t keep = c->epoch;
    for (const auto& col : c->cols) keep = std::min(keep, col.epoch);
    if (c->anc_last_epoch >= 0) keep = std::min(keep, c->anc_last_epoch);
    if (c->scache_lag_epoch >= 0) keep = std::min(keep, c->scache_lag_epoch);
    for (const auto& p : c->dec_rows)
        if (p.epoch >= 0) keep = std::min(keep, p.epoch);
    while (c->log_base < keep && !c->alog.empty()) {
        c->row_pool.push_back(c->alog.front());
        c->alog.pop_front();
        c->log_base += 1;
    }
}
// the newest ancestors known to have resampled (wsmc_last_ancestors, the oracle's last_anc):
// a lazy log entry (epoch >= 0), an eager store's row (epoch -1, owned as anc_keep until the
// next resampling Resample), or row == nullptr: c->anc, which only the fused run and exact
// shards write, and only when they resample
static void set_anc_last(wsmc_ctx* c, const AncRow* row, int64_t epoch) {
    if (c->anc_keep.anc && (!row || row->anc != c->anc_keep.anc)) {
        c->row_pool.push_back(c->anc_keep);
        c->anc_keep = AncRow{};
    }
    if (row && epoch < 0) c->anc_keep = *row;
    c->anc_last = row ? row->anc : nullptr;
    c->anc_last_epoch = row ? epoch : -1;
    gc_log(c);
}
// Bring every stale column to the current epoch: one walk over the log per particle, from
// the newest entry back to the oldest a stale column needs (kTraceLev entries per launch,
// the composed index carried between launches), each column read where its epoch is reached.
static int materialize(wsmc_ctx* c, const std::vector<int32_t>* only) {
    if (only) {   // an unstored Sample output is written before it is traced
        for (int32_t id : *only)
            if (int r = virt_one(c, id)) return r;
    } else if (int r = virt_all(c)) {
        return r;
    }
    std::vector<std::pair<int64_t, int32_t>> stale;   // (levels to apply, column)
    std::vector<char> want(c->cols.size(), only ? 0 : 1);
    if (only)
        for (int32_t id : *only)
            if (id >= 0 && id < (int32_t)c->cols.size()) want[id] = 1;
    for (int32_t id = 0; id < (int32_t)c->cols.size(); ++id)
        if (want[id] && c->cols[id].epoch < c->epoch) stale.emplace_back(c->epoch - c->cols[id].epoch, id);
    if (stale.empty()) return WSMC_OK;
    std::sort(stale.begin(), stale.end());
    const int64_t maxlev = stale.back().first;
    if (c->epoch - maxlev < c->log_base) return fail(WSMC_ESTATE, "lazy genealogy: log entry already released");
    int32_t* scratch[2] = {reinterpret_cast<int32_t*>(c->tmp), reinterpret_cast<int32_t*>(c->tmp) + c->N};
    const int32_t* a_in = nullptr;
    size_t next = 0;
    // launches over consecutive level ranges, each walking its entries once and carrying the
    // composed index to the next; a range ends at kTraceLev entries or where its columns'
    // components would pass kTraceCols (a single level with more repeats its walk)
    for (int64_t base = 0, pass = 0; base < maxlev; ++pass) {
        int64_t hi = std::min<int64_t>(base + kTraceLev, maxlev);
        size_t ncomp = 0, end = next;
        while (end < stale.size() && stale[end].first <= hi) {
            const int d = c->cols[stale[end].second].dim;
            if (ncomp + d > (size_t)kTraceCols && ncomp > 0 && stale[end].first > stale[next].first) {
                hi = stale[end].first - 1;   // close the range before this column's level
                break;
            }
            ncomp += d;
            ++end;
        }
        const int nl = (int)(hi - base);
        TraceArgs t{};
        t.nlev = nl;
        t.tab = c->d_colptr;
        for (int j = 0; j < nl; ++j) {
            const AncRow& r = c->alog[(size_t)(c->epoch - 1 - (base + j) - c->log_base)];
            t.rows[j] = r.anc;
            t.decs[j] = r.dec;
        }
        int32_t* a_out = hi < maxlev ? scratch[pass & 1] : nullptr;
        t.a_in = a_in;
        std::vector<TraceComp> comps;
        for (; next < stale.size() && stale[next].first <= hi; ++next) {
            Column& col = c->cols[stale[next].second];
            for (int k = 0; k < col.dim; ++k)
                comps.push_back({col.back + (int64_t)k * c->N, col.front + (int64_t)k * c->N,
                                 (int32_t)(stale[next].first - base), k == 0 ? stale[next].second : -1});
        }
        size_t done = 0;
        do {   // more than kTraceCols components in the range: repeat the walk per batch
            const size_t n = std::min<size_t>(kTraceCols, comps.size() - done);
            t.ncomp = (int32_t)n;
            for (size_t k = 0; k < n; ++k) t.comp[k] = comps[done + k];
            done += n;
            t.a_out = done >= comps.size() ? a_out : nullptr;
            WSMC_HIP(launch_lazy_trace(c->stream, t, c->N));
        } while (done < comps.size());
        a_in = a_out;
        base = hi;
    }
    for (const auto& sc : stale) {
        Column& col = c->cols[sc.second];
        std::swap(col.front, col.back);
        col.epoch = c->epoch;
    }
    gc_log(c);
    return WSMC_OK;
}
static int materialize_all(wsmc_ctx* c) {
    if (int r = resolve_scache_lag(c)) return r;
    return materialize(c, nullptr);
}
// an operator reads these columns: bring the stale ones among them up to date first (one
// walk of the log for all of them); history the operator does not read stays behind
static int need_cols(wsmc_ctx* c, const std::vector<int32_t>& ids) {
    bool stale = false;
    for (int32_t id : ids) {
        if (id < 0 || id >= (int32_t)c->cols.size()) continue;
        c->cols[id].touch = c->epoch;
        stale |= c->cols[id].epoch < c->epoch;
    }
    return stale ? materialize(c, &ids) : WSMC_OK;
}
static void cols_of(const wsmc_operand& o, std::vector<int32_t>& v) {
    for (int k = 0; k < 2; ++k)
        if (o.col[k] >= 0) v.push_back(o.col[k]);
}
static void cols_of(const wsmc_dist& d, std::vector<int32_t>& v) {
    for (int k = 0; k < 4; ++k) cols_of(d.mu[k], v);
    cols_of(d.scale, v);
}
static void cols_of(const wsmc_term& t, std::vector<int32_t>& v) {
    cols_of(t.dist, v);
    for (int k = 0; k < 4; ++k) cols_of(t.x[k], v);
}
// a column an operator overwrites in full: its old values (of any epoch) are dead
static void wrote_col(wsmc_ctx* c, int32_t id) {
    c->cols[id].epoch = c->epoch;
    c->cols[id].touch = c->epoch;
}
// the ColumnStore.resample! of one Resample / resample!(store, idx) with ancestors `row`:
// lazy — log the row; every column is left behind until an operator reads it (the carried
// Move scores and the weight reset are applied now); eager (exact shards, store_set_lazy(0)
// or WSMC_EAGER_GATHER) — every column gathered, as ColumnStore does
static int store_resample_row(wsmc_ctx* c, const AncRow& row, const Decision* dec, double* w_reset) {
    std::vector<int32_t> which;
    if (!c->lazy) {   // every column is current: no log entry
        for (int32_t id = 0; id < (int32_t)c->cols.size(); ++id) which.push_back(id);
        return gather_columns(c, which, row.anc, dec, w_reset, c->epoch);
    }
    c->alog.push_back(row);
    c->epoch += 1;
    if (w_reset) {
        if (int r = resolve_scache_lag(c)) return r;
        if (int r = gather_columns(c, which, row.anc, dec, w_reset, c->epoch)) return r;
    } else if (c->scache && c->scache_terms >= 0) {
        // the carried Move scores follow their particles at the next Move, which reads them
        // through this entry's ancestors (no gather launch now); one entry at most
        if (int r = resolve_scache_lag(c)) return r;
        c->scache_anc = row.anc;
        c->scache_dec = dec ? dec : c->dec_always;
        c->scache_lag_epoch = c->epoch - 1;
    }
    gc_log(c);
    return WSMC_OK;
}

static wsmc_shard_stats host_record_stats(const ShardRecord& r) {
    wsmc_shard_stats st;
    st.M = wsmc_ord_dec(r.menc);
    st.Q = r.Q;
    st.Q2 = r.q2;
    st.Wf2 = ((wsmc_u128)r.wf2hi << 64) | r.wf2lo;
    st.Wf = ((wsmc_u128)r.wfhi << 64) | r.wflo;
    st.n = r.n;
    return st;
}

// ---- context -------------------------------------------------------------------------
extern "C" {

const char* wsmc_last_error(void) { return g_err.c_str(); }

int wsmc_version(int32_t* major, int32_t* minor) {
    if (major) *major = 0;
    if (minor) *minor = 1;
    return WSMC_OK;
}

// MvNormal(mu, Sigma) with a constant Sigma (src/default_kernels.jl:93): the factor is packed
// into the dist once, on the host (wsmc_terms.h wsmc_mvn_pack)
int wsmc_dist_mvnormal_cov(wsmc_dist* d, const double* cov) {
    if (!d || !cov) return fail(WSMC_EARG, "null argument");
    if (d->dim < 1 || d->dim > WSMC_MVN_MAXDIM) return fail(WSMC_EARG, "MvNormal with a full covariance: dim must be 1..3");
    if (d->mean_fn != WSMC_MEAN_AFFINE) return fail(WSMC_EARG, "MvNormal mean must be affine");
    const int r = wsmc_mvn_pack(d, cov);
    if (r == -1) return fail(WSMC_EARG, "covariance is not symmetric");
    if (r == -2) return fail(WSMC_ENOTPD, "covariance is not positive definite");
    return WSMC_OK;
}

int wsmc_device_count(int32_t* n) {
    int k = 0;
    WSMC_HIP(hipGetDeviceCount(&k));
    *n = k;
    return WSMC_OK;
}

int wsmc_create(wsmc_ctx** out, int64_t n_particles, int32_t device, uint64_t seed) {
    if (!out) return fail(WSMC_EARG, "null out");
    if (n_particles < 1 || n_particles >= (int64_t(1) << 31))
        return fail(WSMC_EARG, "n_particles must be in [1, 2^31)");
    WSMC_HIP(hipSetDevice(device));
    wsmc_ctx* c = new wsmc_ctx();
    c->device = device;
    c->N = n_particles;
    c->gN = n_particles;
    c->seed = seed;
    c->ntiles = (n_particles + kTile - 1) / kTile;
    c->nrstiles = (n_particles + kRsTile - 1) / kRsTile;
    hipError_t e = hipSuccess;
#define ALLOC(ptr, bytes)                                          \
    if (e == hipSuccess) e = hipMalloc((void**)&(ptr), (bytes));
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    ALLOC(c->w, sizeof(double) * c->N);
    ALLOC(c->anc, sizeof(int32_t) * c->N);
    ALLOC(c->tmp, sizeof(double) * 4 * c->N);
    ALLOC(c->xchg, sizeof(unsigned long long) * 16 * kMaxWorld);
    ALLOC(c->tilep, sizeof(unsigned long long) * kPart * c->nrstiles);
    ALLOC(c->tileOff, sizeof(unsigned long long) * c->nrstiles);
    ALLOC(c->taskOff, sizeof(int32_t) * c->nrstiles);
    ALLOC(c->taskTile, sizeof(int32_t) * (c->nrstiles + n_particles / kRsChunk + 1));
    ALLOC(c->mslots, sizeof(MaxSlots));
    ALLOC(c->wslots[0], sizeof(MaxSlots));
    ALLOC(c->wslots[1], sizeof(MaxSlots));
    ALLOC(c->qbuf, sizeof(unsigned long long) * c->N);
    ALLOC(c->tilepart, sizeof(double) * 64 * c->ntiles);   // a Move block's per-move moment sets
    ALLOC(c->rec, sizeof(ShardRecord) * kMaxWorld);
    ALLOC(c->dec, sizeof(Decision));
    ALLOC(c->dec_always, sizeof(Decision));
    ALLOC(c->mom, sizeof(double) * 128);   // [64..128): a Move block's factors
    ALLOC(c->dflag, sizeof(int32_t) * 4);
    ALLOC(c->ucount, sizeof(unsigned long long) * (4 * kAccMove + 4));
    ALLOC(c->d_colptr, sizeof(double*) * kMaxCols);
    ALLOC(c->run_params, sizeof(uint64_t) * 8);
#undef ALLOC
    if (e == hipSuccess) e = hipHostMalloc(&c->pinned, 4096, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->dec_ring, sizeof(Decision) * kDecRing, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->dec_ring_dev, c->dec_ring, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&c->pinned_dev, c->pinned, 0);
    if (e == hipSuccess) e = hipMemsetAsync(c->w, 0, sizeof(double) * c->N, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->wslots[0], 0, sizeof(MaxSlots), c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->wslots[1], 0, sizeof(MaxSlots), c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->anc, 0, sizeof(int32_t) * c->N, c->stream);
    if (e == hipSuccess) {
        Decision always{};
        always.resampled = 1;
        e = hipMemcpy(c->dec_always, &always, sizeof(Decision), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = ctx_sync(c, c->stream);
    {   // diagnostics / A-B: the reference's eager gather of every column at every resample
        const char* eg = getenv("WSMC_EAGER_GATHER");
        c->lazy = !(eg && atoi(eg) != 0);
    }
    if (e != hipSuccess) {
        std::string m = std::string("wsmc_create: ") + hipGetErrorString(e);
        wsmc_destroy(c);
        return fail(WSMC_EHIP, m);
    }
    c->last_ess = std::nan("");
    *out = c;
    return WSMC_OK;
}

int wsmc_destroy(wsmc_ctx* c) {
    if (c && c->multi) return multi_destroy(c);
    if (!c) return WSMC_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& g : c->graphs) {
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        if (g.graph) (void)hipGraphDestroy(g.graph);
        if (g.owned) (void)hipFree(g.owned);
    }
    for (auto ev : c->events) (void)hipEventDestroy(ev);
    for (auto ev : c->run_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->run_hdec) (void)hipHostFree(c->run_hdec);
    if (c->run_hstage) (void)hipHostFree(c->run_hstage);
    run_pend_free(c->run_pend);   // (its run completed with the stream above; nothing to fold in any more)
    c->run_pend = nullptr;
    for (auto& col : c->cols) {
        (void)hipFree(col.front);
        (void)hipFree(col.back);
    }
    for (void* p : c->row_slabs) (void)hipFree(p);   // every row (log, pool, eager, anc_keep) lives in a slab
    void* bufs[] = {c->dec_always, c->xchg, c->scache, c->scache_back, c->w, c->anc, c->tmp, c->tilep, c->tileOff, c->taskOff, c->taskTile, c->mslots, c->qbuf, c->cdf, c->tilepart, c->rec, c->dec, c->mom, c->dflag, c->ucount, c->wslots[0], c->wslots[1],
                    c->d_colptr, c->run_params, c->d_tape, c->run_max, c->run_rec, c->run_dec, c->anc_log, c->obs_buf, c->run_grp, c->run_rg, c->run_nfix, c->run_w0,
                    c->vscratch, c->xscratch, c->xp, c->comb, c->anc_out, c->xbuf, c->d_comp, c->d_ctape, c->d_prog, c->rs_grp[0], c->rs_grp[1], c->rs_qs,
                    c->xpairs, c->xnb, c->xwin, c->xstat, c->w_save, c->xms, c->xanc, c->xlines, c->xpeer};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (double* p : c->xrun)
        if (p) (void)hipFree(p);
    for (int32_t* p : c->lineage)
        if (p) (void)hipFree(p);
    if (c->pinned) (void)hipHostFree(c->pinned);
    for (auto& sl : c->prog_slots)
        if (sl.dev) (void)hipFree(sl.dev);
    if (c->prog_stage) (void)hipHostFree(c->prog_stage);
    delete c->ew;   // statements never launched: the context goes with them
    if (c->dec_ring) (void)hipHostFree(c->dec_ring);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return WSMC_OK;
}

// fold the decisions of asynchronous Resamples (pinned ring, in issue order) into the host
// mirror of state.resampled / n_resamples / last_ess
static int resolve_decisions(wsmc_ctx* c) {
    if (!c->dec_pending) return WSMC_OK;
    WSMC_HIP(ctx_sync(c, c->stream));
    for (int i = 0; i < c->dec_pending; ++i) {
        const Decision& d = c->dec_ring[i];
        c->last_ess = d.ess;
        c->resampled = d.resampled;
        if (d.resampled) c->n_resamples += 1;
        if (i < (int)c->dec_rows.size()) {
            const wsmc_ctx::PendingRow& p = c->dec_rows[i];
            if (p.epoch < 0) {   // an eager store's row: kept only if this Resample resampled
                if (d.resampled) set_anc_last(c, &p.row, -1);
                else c->row_pool.push_back(p.row);
            } else if (p.epoch >= c->log_base && p.epoch - c->log_base < (int64_t)c->alog.size()) {
                AncRow& r = c->alog[(size_t)(p.epoch - c->log_base)];   // the lazy log entry
                r.known = d.resampled;
                if (d.resampled) set_anc_last(c, &r, p.epoch);
            }
        }
    }
    c->dec_pending = 0;
    c->dec_rows.clear();
    gc_log(c);
    return WSMC_OK;
}

// an asynchronous Move (no accepted count requested) leaves its not-positive-definite flag on
// the device; the next synchronizing call reads it and reports the reference's PosDefException
static int check_deferred(wsmc_ctx* c) {
    if (!c->move_pending) return WSMC_OK;
    int32_t* hf = reinterpret_cast<int32_t*>(c->pinned) + 1000;
    WSMC_HIP(hipMemcpyAsync(hf, c->dflag, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    c->move_pending = false;
    if (hf[0]) {
        scores_invalidate(c);
        WSMC_HIP(hipMemsetAsync(c->dflag, 0, sizeof(int32_t) * 4, c->stream));
        c->dflag_zero = true;
        return fail(WSMC_ENOTPD, "autoRW proposal covariance is not positive definite (an asynchronous Move)");
    }
    c->dflag_zero = true;   // read back as zero: the next Move needs no reset
    return WSMC_OK;
}

int wsmc_sync(wsmc_ctx* c) {
    if (c && c->multi) return multi_sync(c);
    CHECK_CTX(c);
    WSMC_HIP(ctx_sync(c, c->stream));
    if (int r = check_deferred(c)) return r;
    return WSMC_OK;
}

int wsmc_nparticles(wsmc_ctx* c, int64_t* n) {
    if (!c || !n) return fail(WSMC_EARG, "null argument");
    *n = c->N;
    return WSMC_OK;
}

int wsmc_get_state(wsmc_ctx* c, wsmc_state* s) {
    if (c && c->multi) return s ? multi_get_state(c, s) : fail(WSMC_EARG, "null argument");
    if (!c || !s) return fail(WSMC_EARG, "null argument");
    if (int r = resolve_decisions(c)) return r;
    if (int r = check_deferred(c)) return r;
    s->resampled = c->resampled;
    s->weights_changed = c->weights_changed;
    s->depth = c->depth;
    s->n_terms = (int32_t)c->tape.size();
    s->last_ess_perc = c->last_ess;
    s->op_counter = c->op;
    s->n_resamples = c->n_resamples;
    return WSMC_OK;
}

int wsmc_set_depth(wsmc_ctx* c, int32_t depth) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_set_depth(x, depth); });
    if (!c) return fail(WSMC_EARG, "null context");
    c->depth = depth;
    scores_invalidate(c);
    return WSMC_OK;
}

int wsmc_set_op_counter(wsmc_ctx* c, uint64_t op) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_set_op_counter(x, op); });
    if (!c) return fail(WSMC_EARG, "null context");
    c->op = op;
    return WSMC_OK;
}

// ---- RCCL ----------------------------------------------------------------------------
int wsmc_comm_unique_id(uint8_t out_id[128]) {
    ncclUniqueId id;
    WSMC_RCCL(ncclGetUniqueId(&id));
    std::memcpy(out_id, id.internal, 128);
    return WSMC_OK;
}

int wsmc_comm_init(wsmc_ctx* c, const uint8_t id[128], int32_t world, int32_t rank, int64_t goff, int64_t gN) {
    if (c && c->multi) return fail(WSMC_EARG, "a multi-device handle is sharded at creation");
    CHECK_CTX(c);
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) return fail(WSMC_EARG, "bad world/rank");
    if (goff < 0 || goff + c->N > gN) return fail(WSMC_EARG, "shard outside the global population");
    // ancestor ids are int32 and the exact fill keeps slot ranks in 32 bits: a population of
    // 2^31 or more would truncate them
    if (gN >= (int64_t(1) << 31)) return fail(WSMC_EARG, "global population of 2^31 particles or more");
    c->world = world;
    c->rank = rank;
    c->goff = goff;
    c->gN = gN;
    {   // world 1 too: a one-rank communicator runs the exchange paths on one GPU
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, 128);
        WSMC_RCCL(ncclCommInitRank(&c->comm, world, uid, rank));
    }
    return WSMC_OK;
}

int wsmc_comm_init_host(wsmc_ctx* c, wsmc_exchange_fn exchange, void* user, int32_t world, int32_t rank,
                        int64_t goff, int64_t gN) {
    if (c && c->multi) return fail(WSMC_EARG, "a multi-device handle is sharded at creation");
    CHECK_CTX(c);
    if (!exchange) return fail(WSMC_EARG, "null exchange");
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world) return fail(WSMC_EARG, "bad world/rank");
    if (goff < 0 || goff + c->N > gN) return fail(WSMC_EARG, "shard outside the global population");
    // ancestor ids are int32 and the exact fill keeps slot ranks in 32 bits: a population of
    // 2^31 or more would truncate them
    if (gN >= (int64_t(1) << 31)) return fail(WSMC_EARG, "global population of 2^31 particles or more");
    c->world = world;
    c->rank = rank;
    c->goff = goff;
    c->gN = gN;
    c->host_exchange = exchange;
    c->host_user = user;
    return WSMC_OK;
}

int wsmc_comm_info(wsmc_ctx* c, wsmc_comm_info_t* out) {
    if (!out) return fail(WSMC_EARG, "null argument");
    if (c && c->multi) return multi_comm_info(c, out);
    CHECK_CTX(c);
    *out = wsmc_comm_info_t{};
    out->shards = 1;
    out->world = c->world;
    out->rank = c->rank;
    out->transport = c->comm ? WSMC_TRANSPORT_RCCL : c->host_exchange ? WSMC_TRANSPORT_HOST : -1;
    out->shard_mode = c->shard_mode;
    if (c->comm) {
        int n = 0;
        WSMC_RCCL(ncclCommCount(c->comm, &n));
        out->rccl_ranks = n;
    }
    for (int g = 0; g < 8; ++g) out->devices[g] = -1;
    out->devices[0] = c->device;
    out->shard_n[0] = c->N;
    return WSMC_OK;
}

int wsmc_comm_set_timeout(wsmc_ctx* c, double seconds) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_comm_set_timeout(x, seconds); });
    CHECK_CTX(c);
    if (!(seconds >= 0.0)) return fail(WSMC_EARG, "timeout must be >= 0");
    c->comm_timeout_s = seconds;
    return WSMC_OK;
}

int wsmc_comm_set_shard_mode(wsmc_ctx* c, int32_t mode) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_comm_set_shard_mode(x, mode); });
    CHECK_CTX(c);
    if (mode != WSMC_SHARD_ISLAND && mode != WSMC_SHARD_EXACT) return fail(WSMC_EARG, "unknown shard mode");
    // pending asynchronous decisions are read back under the store mode they were issued in
    if (int r = resolve_decisions(c)) return r;
    // exact shards move every column between ranks at each Resample: the store stays eager
    if (mode == WSMC_SHARD_EXACT) {
        if (int r = materialize_all(c)) return r;
        c->lazy = false;
    } else {
        const char* eg = getenv("WSMC_EAGER_GATHER");
        c->lazy = !(eg && atoi(eg) != 0);
    }
    c->shard_mode = mode;
    return WSMC_OK;
}

// ---- store ---------------------------------------------------------------------------
int wsmc_col_create(wsmc_ctx* c, const char* name, int32_t dim, int32_t* col_id) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { int32_t id = -1; int r = wsmc_col_create(x, name, dim, &id); if (x == multi_first(c) && col_id) *col_id = id; return r; });
    CHECK_CTX_DEV(c);   // no weights touched; a pending statement batch keeps its pointers
    if (!name || !col_id) return fail(WSMC_EARG, "null argument");
    for (size_t k = 0; k < c->cols.size(); ++k)
        if (c->cols[k].name == name) {
            if (c->cols[k].dim != dim) return fail(WSMC_EARG, std::string("column ") + name + " exists with another dim");
            *col_id = (int32_t)k;
            return WSMC_OK;
        }
    if (dim < 1 || dim > 4) return fail(WSMC_EARG, "column dim must be 1..4");
    if ((int)c->cols.size() >= kMaxCols) return fail(WSMC_ENOMEM, "too many columns");
    Column col;
    col.name = name;
    col.dim = dim;
    WSMC_HIP(hipMalloc(&col.front, sizeof(double) * dim * c->N));
    WSMC_HIP(hipMalloc(&col.back, sizeof(double) * dim * c->N));
    WSMC_HIP(hipMemsetAsync(col.front, 0, sizeof(double) * dim * c->N, c->stream));
    col.epoch = c->epoch;   // zeros, current
    c->cols.push_back(col);
    c->colptr_dirty = true;
    *col_id = (int32_t)(c->cols.size() - 1);
    return WSMC_OK;
}

int wsmc_col_find(wsmc_ctx* c, const char* name, int32_t* col_id) {
    if (c && c->multi) return wsmc_col_find(multi_first(c), name, col_id);
    if (!c || !name || !col_id) return fail(WSMC_EARG, "null argument");
    *col_id = -1;
    for (size_t k = 0; k < c->cols.size(); ++k)
        if (c->cols[k].name == name) *col_id = (int32_t)k;
    return WSMC_OK;
}

int wsmc_col_count(wsmc_ctx* c, int32_t* n) {
    if (c && c->multi) return wsmc_col_count(multi_first(c), n);
    if (!c || !n) return fail(WSMC_EARG, "null argument");
    *n = (int32_t)c->cols.size();
    return WSMC_OK;
}

int wsmc_col_info(wsmc_ctx* c, int32_t col, char* buf, int32_t len, int32_t* dim) {
    if (c && c->multi) return wsmc_col_info(multi_first(c), col, buf, len, dim);
    if (!c || !valid_col(c, col)) return fail(WSMC_EARG, "bad column");
    if (buf && len > 0) {
        std::strncpy(buf, c->cols[col].name.c_str(), len - 1);
        buf[len - 1] = 0;
    }
    if (dim) *dim = c->cols[col].dim;
    return WSMC_OK;
}

int wsmc_col_download(wsmc_ctx* c, int32_t col, double* host) {
    if (c && c->multi) return host ? multi_col_download(c, col, host) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!valid_col(c, col) || !host) return fail(WSMC_EARG, "bad column or null buffer");
    if (int r = need_cols(c, {col})) return r;
    if (int r = check_deferred(c)) return r;
    WSMC_HIP(hipMemcpyAsync(host, c->cols[col].front, sizeof(double) * c->cols[col].dim * c->N,
                            hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

int wsmc_col_upload(wsmc_ctx* c, int32_t col, const double* host) {
    if (c && c->multi) return host ? multi_col_upload(c, col, host) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!valid_col(c, col) || !host) return fail(WSMC_EARG, "bad column or null buffer");
    scores_touch(c, col);
    wrote_col(c, col);
    WSMC_HIP(hipMemcpyAsync(c->cols[col].front, host, sizeof(double) * c->cols[col].dim * c->N,
                            hipMemcpyHostToDevice, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

int wsmc_col_device_ptr(wsmc_ctx* c, int32_t col, double** dptr) {
    if (c && c->multi) return multi_G(c) == 1 ? wsmc_col_device_ptr(multi_first(c), col, dptr) : fail(WSMC_EARG, "a column of a multi-device handle lives on several devices");
    if (!c || !valid_col(c, col) || !dptr) return fail(WSMC_EARG, "bad column");
    WSMC_HIP(hipSetDevice(c->device));
    if (int r = ew_flush(c)) return r;   // the caller reads the column on the stream
    if (int r = need_cols(c, {col})) return r;
    *dptr = c->cols[col].front;
    return WSMC_OK;
}

int wsmc_store_resample(wsmc_ctx* c, const int32_t* idx) {
    if (c && c->multi) return multi_G(c) == 1 ? wsmc_store_resample(multi_first(c), idx) : fail(WSMC_EARG, "resample!(store, idx) with global indices needs one shard");
    CHECK_CTX(c);
    if (!idx) return fail(WSMC_EARG, "null indices");
    for (int64_t i = 0; i < c->N; ++i)
        if (idx[i] < 0 || idx[i] >= c->N) return fail(WSMC_EARG, "index out of range");
    // pending asynchronous Resamples come first (their rows would otherwise overtake this one)
    int r = resolve_decisions(c);
    if (r) return r;
    // logged like a Resample that resampled (its decision: always); an eager store keeps the
    // row as the last ancestors
    AncRow row;
    if ((r = acquire_row(c, &row))) return r;
    WSMC_HIP(hipMemcpyAsync(row.anc, idx, sizeof(int32_t) * c->N, hipMemcpyHostToDevice, c->stream));
    WSMC_HIP(hipMemcpyAsync(row.dec, c->dec_always, sizeof(Decision), hipMemcpyDeviceToDevice, c->stream));
    row.known = 1;
    if ((r = store_resample_row(c, row, nullptr, nullptr))) return r;
    set_anc_last(c, &row, c->lazy ? c->epoch - 1 : -1);
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

static bool exact_mode(const wsmc_ctx* c);
int wsmc_store_set_lazy(wsmc_ctx* c, int32_t lazy) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_store_set_lazy(x, lazy); });
    CHECK_CTX(c);
    if (!lazy || exact_mode(c)) {
        if (int r = resolve_decisions(c)) return r;
        if (int r = materialize_all(c)) return r;
        c->lazy = false;
        gc_log(c);
        return WSMC_OK;
    }
    c->lazy = true;
    return WSMC_OK;
}

int wsmc_store_materialize(wsmc_ctx* c) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_store_materialize(x); });
    CHECK_CTX(c);
    return materialize_all(c);
}

int wsmc_store_info(wsmc_ctx* c, int64_t* log_entries, int32_t* stale_columns) {
    if (c && c->multi) return wsmc_store_info(multi_first(c), log_entries, stale_columns);
    if (!c) return fail(WSMC_EARG, "null context");
    if (log_entries) *log_entries = (int64_t)c->alog.size();
    if (stale_columns) {
        int32_t n = 0;
        for (const auto& col : c->cols) n += col.epoch < c->epoch ? 1 : 0;
        *stale_columns = n;
    }
    return WSMC_OK;
}

// ---- weights -------------------------------------------------------------------------
int wsmc_weights_upload(wsmc_ctx* c, const double* host) {
    if (c && c->multi) return host ? multi_weights(c, host, nullptr) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!host) return fail(WSMC_EARG, "null buffer");
    c->wseq += 1;
    WSMC_HIP(hipMemcpyAsync(c->w, host, sizeof(double) * c->N, hipMemcpyHostToDevice, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

int wsmc_weights_download(wsmc_ctx* c, double* host) {
    if (c && c->multi) return host ? multi_weights(c, nullptr, host) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!host) return fail(WSMC_EARG, "null buffer");
    if (int r = check_deferred(c)) return r;
    WSMC_HIP(hipMemcpyAsync(host, c->w, sizeof(double) * c->N, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

static int exchange_recs(wsmc_ctx* c, ShardRecord* recs);
// The exchange (sharded) code paths run when the population is split over ranks, and also
// for a one-rank communicator (world 1 with an RCCL comm or a host exchange): one shard is
// the whole population, so the results equal the unsharded path's, which lets one GPU
// exercise the RCCL calls themselves (tests/test_gpu_multishard.py).
static inline bool is_sharded(const wsmc_ctx* c) { return c->world > 1 || c->comm || c->host_exchange; }
// max (unless the caller's kernel already filled the slots), sums, reduce, [exchange + decide]
static FillPlan fill_plan(wsmc_ctx* c, int scheme, uint64_t op, const uint64_t* op_dev) {
    FillPlan p;
    p.tilep = c->tilep;
    p.taskOff = c->taskOff;
    p.taskTile = c->taskTile;
    p.scheme = scheme;
    p.seed = c->seed;
    p.op = op;
    p.op_dev = op_dev;
    p.slot_base = c->goff;
    return p;
}

static bool valid_scheme(int32_t s) {
    return s == WSMC_RESAMPLE_STRATIFIED || s == WSMC_RESAMPLE_SYSTEMATIC || s == WSMC_RESAMPLE_MULTINOMIAL;
}
static int ensure_cdf(wsmc_ctx* c) {
    // [N] tile-local CDF + the exponential-spacing tile sums (one per tile, + the total)
    const size_t words = (size_t)c->N + (size_t)((c->N + kRsTile - 1) / kRsTile) + 1;
    if (!c->cdf) WSMC_HIP(hipMalloc(&c->cdf, sizeof(unsigned long long) * words));
    return WSMC_OK;
}

// multinomial: c->cdf holds the tile-local CDF [N], then the spacing tile sums / offsets
static unsigned long long* multi_esum(wsmc_ctx* c) { return c->cdf + c->N; }
// and the slots' spacings E (u32) in the q buffer, which the multinomial path does not use
static uint32_t* multi_ebuf(wsmc_ctx* c) { return reinterpret_cast<uint32_t*>(c->qbuf); }

static int enqueue_resample_stats(wsmc_ctx* c, const double* w, MaxSlots* ms, ShardRecord* recs, double ess_min,
                                  Decision* dec, bool run_max, const FillPlan& plan, hipEvent_t* ev = nullptr) {
    if (run_max) {
        WSMC_HIP(hipMemsetAsync(ms, 0, sizeof(MaxSlots), c->stream));
        WSMC_HIP(launch_rs_max(c->stream, w, c->N, ms));
    }
    const bool multi = plan.scheme == WSMC_RESAMPLE_MULTINOMIAL;
    if (multi)
        WSMC_HIP(launch_rs_sums_multi(c->stream, w, c->N, ms, plan, c->tilep, c->cdf, multi_esum(c), multi_ebuf(c),
                                      ev ? ev[0] : nullptr, ev ? ev[1] : nullptr));
    else
        WSMC_HIP(launch_rs_sums(c->stream, w, c->N, ms, c->tilep, c->qbuf, ev ? ev[0] : nullptr, ev ? ev[1] : nullptr));
    WSMC_HIP(launch_rs_reduce(c->stream, ms, c->tilep, c->N, c->tileOff, recs + c->rank, !is_sharded(c), ess_min, dec,
                              &plan, ev ? ev[2] : nullptr, ev ? ev[3] : nullptr, multi ? multi_esum(c) : nullptr));
    if (is_sharded(c)) {
        int r = exchange_recs(c, recs);
        if (r) return r;
        WSMC_HIP(launch_rs_decide(c->stream, recs, c->world, c->rank, ess_min, dec));
    }
    return WSMC_OK;
}

// all-gather `words` u64 per rank in place (rank r's block at buf + r * words) on stream s
// a host-provided exchange (wsmc_comm_init_host), counted: a multi-device handle's shard that
// fails after its first exchange of a call requests the abort at once (csrc/wsmc_multi.hip)
static inline int host_xchg(wsmc_ctx* c, const uint64_t* mine, int32_t words, uint64_t* all) {
    c->exchanges += 1;
    return c->host_exchange(c->host_user, mine, words, all);
}

static int exchange_words(wsmc_ctx* c, unsigned long long* buf, int64_t words, hipStream_t s) {
    if (!is_sharded(c)) return WSMC_OK;
    if (c->host_exchange) {
        std::vector<unsigned long long> h((size_t)words * c->world);
        WSMC_HIP(hipMemcpyAsync(h.data() + (size_t)c->rank * words, buf + (size_t)c->rank * words,
                                sizeof(unsigned long long) * words, hipMemcpyDeviceToHost, s));
        WSMC_HIP(ctx_sync(c, s));
        const std::vector<unsigned long long> mine(h.begin() + (size_t)c->rank * words,
                                                   h.begin() + (size_t)(c->rank + 1) * words);
        if (host_xchg(c, reinterpret_cast<const uint64_t*>(mine.data()), (int32_t)words,
                             reinterpret_cast<uint64_t*>(h.data())) != 0)
            return fail(WSMC_ERCCL, "host exchange failed");
        WSMC_HIP(hipMemcpyAsync(buf, h.data(), sizeof(unsigned long long) * h.size(), hipMemcpyHostToDevice, s));
        WSMC_HIP(ctx_sync(c, s));
        return WSMC_OK;
    }
    WSMC_RCCL_GUARD(c);
    c->exchanges += 1;
    WSMC_RCCL(ncclAllGather(buf + (size_t)c->rank * words, buf, (size_t)words, ncclUint64, c->comm, s));
    return WSMC_OK;
}

static int exchange_recs(wsmc_ctx* c, ShardRecord* recs) {
    if (c->inject_fail > 0 && --c->inject_fail == 0)
        return c->inject_earg ? fail(WSMC_EARG, "injected shard argument error (wsmc_debug_inject_failure)")
                              : fail(WSMC_EHIP, "injected shard failure (wsmc_debug_inject_failure)");
    if (!is_sharded(c)) return WSMC_OK;
    const int words = (int)(sizeof(ShardRecord) / sizeof(unsigned long long));
    if (c->host_exchange) {
        std::vector<ShardRecord> h(c->world);
        WSMC_HIP(hipMemcpyAsync(&h[c->rank], recs + c->rank, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        const ShardRecord mine = h[c->rank];
        if (host_xchg(c, reinterpret_cast<const uint64_t*>(&mine), words,
                             reinterpret_cast<uint64_t*>(h.data())) != 0)
            return fail(WSMC_ERCCL, "host record exchange failed");
        WSMC_HIP(hipMemcpyAsync(recs, h.data(), sizeof(ShardRecord) * c->world, hipMemcpyHostToDevice, c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        return WSMC_OK;
    }
    WSMC_RCCL_GUARD(c);
    c->exchanges += 1;
    WSMC_RCCL(ncclAllGather(recs + c->rank, recs, words, ncclUint64, c->comm, c->stream));
    return WSMC_OK;
}

// ---- exact sharding ---------------------------------------------------
static bool exact_mode(const wsmc_ctx* c) { return is_sharded(c) && c->shard_mode == WSMC_SHARD_EXACT; }

static int ensure_exact(wsmc_ctx* c) {
    if (!c->xp) WSMC_HIP(hipMalloc(&c->xp, sizeof(ExactPlan)));
    if (!c->comb) WSMC_HIP(hipMalloc(&c->comb, sizeof(ShardRecord)));
    if (!c->anc_out) WSMC_HIP(hipMalloc(&c->anc_out, sizeof(int32_t) * (size_t)c->gN));
    if (!c->task_global) {
        // a shard may own up to all gN slots: sum_b floor((Q_b gN / Q + 3) / kRsChunk)
        // <= gN / kRsChunk + ntiles overflow tasks
        WSMC_HIP(ctx_sync(c, c->stream));
        WSMC_HIP(hipFree(c->taskTile));
        WSMC_HIP(hipMalloc(&c->taskTile, sizeof(int32_t) * (size_t)(c->nrstiles + c->gN / kRsChunk + 1)));
        c->task_global = true;
    }
    return WSMC_OK;
}

// the global max (the ranks' local maxima all-gathered), the shard's q relative to it with
// K from the global N, its record, and every rank's record: their integer sums are exactly
// the statistics one context holding all particles computes
static int exact_records(wsmc_ctx* c) {
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    WSMC_HIP(launch_max_publish(c->stream, c->mslots, c->xchg + c->rank));
    int r = exchange_words(c, c->xchg, 1, c->stream);
    if (r) return r;
    WSMC_HIP(launch_max_adopt(c->stream, c->xchg, c->world, c->mslots));
    WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, nullptr, nullptr, nullptr, 1,
                            c->gN));
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec + c->rank, 0, 0.0, nullptr,
                              nullptr));
    return exchange_recs(c, c->rec);
}
static int exact_global_stats(wsmc_ctx* c, wsmc_shard_stats* st) {
    int r = exact_records(c);
    if (r) return r;
    std::vector<ShardRecord> h(c->world);
    WSMC_HIP(hipMemcpyAsync(h.data(), c->rec, sizeof(ShardRecord) * c->world, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    *st = host_record_stats(h[0]);
    st->Q = 0; st->Q2 = 0; st->Wf2 = 0; st->Wf = 0; st->n = 0;
    for (int g = 0; g < c->world; ++g) {
        const wsmc_shard_stats x = host_record_stats(h[g]);
        st->Q += x.Q; st->Q2 += x.Q2; st->Wf2 += x.Wf2; st->Wf += x.Wf; st->n += x.n;
    }
    return WSMC_OK;
}

static inline unsigned long long overlap(unsigned long long a0, unsigned long long a1, unsigned long long b0,
                                         unsigned long long b1) {
    const unsigned long long lo = a0 > b0 ? a0 : b0, hi = a1 < b1 ? a1 : b1;
    return hi > lo ? hi - lo : 0ull;
}

// the window's slots move to their owners: local ones in place, the rest packed per peer,
// exchanged (grouped RCCL send/recv, or the host exchange), unpacked. src/dst: component
// arrays (element stride `stride`); anc_local receives the global ancestor ids.
static int exact_route(wsmc_ctx* c, const ExactPlan& x, const std::vector<const double*>& src,
                       const std::vector<double*>& dst, int stride, int32_t* anc_local) {
    const int W = c->world, me = c->rank;
    const int nc = (int)src.size();
    const size_t need = 2 * (size_t)(nc > 0 ? nc : 1);
    if (c->d_comp_cap < need) {
        WSMC_HIP(ctx_sync(c, c->stream));
        if (c->d_comp) WSMC_HIP(hipFree(c->d_comp));
        WSMC_HIP(hipMalloc(&c->d_comp, sizeof(double*) * need));
        c->d_comp_cap = need;
    }
    std::vector<double*> tab(need, nullptr);
    for (int k = 0; k < nc; ++k) {
        tab[k] = const_cast<double*>(src[k]);
        tab[nc + k] = dst[k];
    }
    WSMC_HIP(hipMemcpyAsync(c->d_comp, tab.data(), sizeof(double*) * need, hipMemcpyHostToDevice, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));   // `tab` is pageable and local
    // routing tables (every rank derives every rank's blocks from the same plan)
    const unsigned long long D = (unsigned long long)nc + 1;
    auto sendlen = [&](int g, int r) { return overlap(x.seg[g], x.seg[g + 1], x.gofs[r], x.gofs[r + 1]); };
    ExactRoute rt{};
    rt.world = W; rt.rank = me; rt.ncomp = nc; rt.stride = stride;
    rt.a = x.a; rt.b = x.b;
    for (int g = 0; g <= W; ++g) rt.gofs[g] = x.gofs[g];
    unsigned long long S = 0, R = 0;
    std::vector<unsigned long long> Sg(W, 0);
    for (int g = 0; g < W; ++g)
        for (int r = 0; r < W; ++r)
            if (r != g) Sg[g] += sendlen(g, r) * D;
    for (int r = 0; r < W; ++r) {
        rt.sendoff[r] = S;
        if (r != me) S += sendlen(me, r) * D;
    }
    rt.recvpre[0] = 0;
    for (int g = 0; g < W; ++g) {
        const unsigned long long n = g == me ? 0ull : sendlen(g, me);
        rt.recvoff[g] = R;
        rt.recvlen[g] = n;
        rt.recvdst[g] = (x.seg[g] > x.gofs[me] ? x.seg[g] : x.gofs[me]) - x.gofs[me];
        rt.recvpre[g + 1] = rt.recvpre[g] + n;
        R += n * D;
    }
    const size_t words = (size_t)(S + R) + 1;
    if (c->xbuf_cap < words) {
        WSMC_HIP(ctx_sync(c, c->stream));
        if (c->xbuf) WSMC_HIP(hipFree(c->xbuf));
        WSMC_HIP(hipMalloc(&c->xbuf, sizeof(unsigned long long) * words));
        c->xbuf_cap = words;
    }
    unsigned long long* sendbuf = c->xbuf;
    unsigned long long* recvbuf = c->xbuf + S;
    WSMC_HIP(launch_exact_pack(c->stream, rt, c->anc_out, c->d_comp, c->d_comp + nc, anc_local, sendbuf));
    if (c->host_exchange) {
        // test transport: every rank all-gathers its whole send area (padded to the largest)
        unsigned long long maxS = 0;
        for (int g = 0; g < W; ++g) maxS = Sg[g] > maxS ? Sg[g] : maxS;
        if (maxS > 0) {
            if (maxS > 0x7fffffffull) return fail(WSMC_EARG, "host exchange block too large");
            std::vector<unsigned long long> mine(maxS, 0ull), all((size_t)maxS * W);
            if (S) WSMC_HIP(hipMemcpyAsync(mine.data(), sendbuf, sizeof(unsigned long long) * S, hipMemcpyDeviceToHost,
                                           c->stream));
            WSMC_HIP(ctx_sync(c, c->stream));
            if (host_xchg(c, reinterpret_cast<const uint64_t*>(mine.data()), (int32_t)maxS,
                                 reinterpret_cast<uint64_t*>(all.data())) != 0)
                return fail(WSMC_ERCCL, "host particle exchange failed");
            std::vector<unsigned long long> rv((size_t)R + 1);
            for (int g = 0; g < W; ++g) {
                if (g == me || !rt.recvlen[g]) continue;
                unsigned long long off = 0;
                for (int r = 0; r < me; ++r)
                    if (r != g) off += sendlen(g, r) * D;
                std::memcpy(rv.data() + rt.recvoff[g], all.data() + (size_t)g * maxS + off,
                            sizeof(unsigned long long) * rt.recvlen[g] * D);
            }
            if (R) WSMC_HIP(hipMemcpyAsync(recvbuf, rv.data(), sizeof(unsigned long long) * R, hipMemcpyHostToDevice,
                                           c->stream));
            WSMC_HIP(ctx_sync(c, c->stream));
        }
    } else {
        WSMC_RCCL_GUARD(c);
        c->exchanges += 1;
        WSMC_RCCL(ncclGroupStart());
        for (int r = 0; r < W; ++r) {
            if (r == me) continue;
            const unsigned long long ns = sendlen(me, r) * D, nr = rt.recvlen[r] * D;
            if (ns) WSMC_RCCL(ncclSend(sendbuf + rt.sendoff[r], (size_t)ns, ncclUint64, r, c->comm, c->stream));
            if (nr) WSMC_RCCL(ncclRecv(recvbuf + rt.recvoff[r], (size_t)nr, ncclUint64, r, c->comm, c->stream));
        }
        WSMC_RCCL(ncclGroupEnd());
    }
    WSMC_HIP(launch_exact_unpack(c->stream, rt, recvbuf, c->d_comp + nc, anc_local));
    return WSMC_OK;
}

// every column (and the carried Move scores) follows the window's ancestors
static int exact_move_particles(wsmc_ctx* c, const ExactPlan& x) {
    std::vector<const double*> src;
    std::vector<double*> dst;
    for (auto& col : c->cols)
        for (int k = 0; k < col.dim; ++k) {
            src.push_back(col.front + (int64_t)k * c->N);
            dst.push_back(col.back + (int64_t)k * c->N);
        }
    const bool cache = c->scache && c->scache_terms >= 0;   // carried Move scores follow their particles
    if (cache) {
        src.push_back(c->scache);
        dst.push_back(c->scache_back);
    }
    int r = exact_route(c, x, src, dst, 1, c->anc);
    if (r) return r;
    for (auto& col : c->cols) std::swap(col.front, col.back);
    if (cache) std::swap(c->scache, c->scache_back);
    c->colptr_dirty = true;
    return WSMC_OK;
}

// decide (the single-context bits) and fill this shard's window of global slots (anc_out)
static int exact_decide_fill(wsmc_ctx* c, double ess_min, int32_t scheme, uint64_t op, Decision* dec_dev,
                             Decision* hd, ExactPlan* hx) {
    int r = ensure_exact(c);
    if (r) return r;
    if ((r = exact_records(c))) return r;
    FillPlan plan = fill_plan(c, scheme, op, nullptr);
    plan.slot_base = 0;                       // slots are global: their keys too
    WSMC_HIP(launch_rs_decide_exact(c->stream, c->rec, c->world, c->rank, ess_min, plan, c->comb, dec_dev, c->xp));
    plan.xp = c->xp;
    // fill tasks planned with the global strata (N / Q of the whole population)
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec + c->rank, 0, ess_min, dec_dev,
                              &plan));
    WSMC_HIP(launch_rs_scan(c->stream, c->N, c->comb, dec_dev, plan, c->tileOff, c->qbuf, c->anc_out));
    struct Host { Decision d; ExactPlan x; };
    Host* h = reinterpret_cast<Host*>(c->pinned);
    static_assert(sizeof(Host) <= 4096, "pinned staging");
    WSMC_HIP(hipMemcpyAsync(&h->d, dec_dev, sizeof(Decision), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(hipMemcpyAsync(&h->x, c->xp, sizeof(ExactPlan), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    *hd = h->d;
    *hx = h->x;
    return WSMC_OK;
}

// Resample over the whole population: the single-GPU decision,
// ancestors, columns, weights and evidence, bit for bit
static int exact_resample(wsmc_ctx* c, double ess_min, int32_t scheme, uint64_t op, Decision* out) {
    ExactPlan x;
    int r = exact_decide_fill(c, ess_min, scheme, op, c->dec, out, &x);
    if (r || !out->resampled) return r;
    if ((r = exact_move_particles(c, x))) return r;
    c->wseq += 1;
    WSMC_HIP(launch_fill_weights(c->stream, c->w, c->dec, c->N));
    return WSMC_OK;
}

// One level of the distributed trace-back: every rank's lineage ids a[0..n) are sorted
// (stratified / systematic ancestors are monotone, so are their compositions), so a rank
// needs one contiguous range [a[0], a[n-1]] of global indices. Owners send their part of
// (x pair of hist, ancestor of arow) for it; xout gets hist[a] (SoA), anext arow[a] (or a).
static int trace_level(wsmc_ctx* c, const ExactPlan& x, const double* hist, const int32_t* arow, const int32_t* a,
                       int32_t* anext, double* xout) {
    const int W = c->world, me = c->rank;
    const int64_t n = c->N;
    int32_t* h2 = reinterpret_cast<int32_t*>(c->pinned);
    WSMC_HIP(hipMemcpyAsync(h2, a, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(hipMemcpyAsync(h2 + 1, a + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    std::vector<unsigned long long> rng(2 * (size_t)W);
    {
        unsigned long long* mine = reinterpret_cast<unsigned long long*>(c->pinned) + 64;   // pinned staging
        mine[0] = (unsigned long long)(uint32_t)h2[0];
        mine[1] = (unsigned long long)(uint32_t)h2[1] + 1;                                  // [lo, hi)
        WSMC_HIP(hipMemcpyAsync(c->xchg + 2 * me, mine, sizeof(unsigned long long) * 2, hipMemcpyHostToDevice,
                                c->stream));
        int r = exchange_words(c, c->xchg, 2, c->stream);
        if (r) return r;
        WSMC_HIP(hipMemcpyAsync(rng.data(), c->xchg, sizeof(unsigned long long) * 2 * W, hipMemcpyDeviceToHost,
                                c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
    }
    static const bool dbg = [] {   // diagnostics: every level's requested id range
        const char* e = getenv("WSMC_TRACE_DEBUG");
        return e && atoi(e) != 0;
    }();
    if (dbg && me == 0)
        std::fprintf(stderr, "[trace_level] ranges:%s\n", [&] {
            std::string t;
            for (int g = 0; g < W; ++g) t += " [" + std::to_string(rng[2 * g]) + "," + std::to_string(rng[2 * g + 1]) + ")";
            return t;
        }().c_str());
    auto part = [&](int owner, int req) {   // [start, end) global of owner's rows requester needs
        const unsigned long long lo = rng[2 * req] > x.gofs[owner] ? rng[2 * req] : x.gofs[owner];
        const unsigned long long hi = rng[2 * req + 1] < x.gofs[owner + 1] ? rng[2 * req + 1] : x.gofs[owner + 1];
        return std::make_pair(lo, hi > lo ? hi : lo);
    };
    const unsigned long long lome = rng[2 * me], R = (rng[2 * me + 1] - lome) * 3;
    unsigned long long S = 0;
    std::vector<unsigned long long> soff(W, 0), Sg(W, 0);
    for (int g = 0; g < W; ++g)
        for (int r = 0; r < W; ++r)
            if (r != g) { auto pr = part(g, r); Sg[g] += (pr.second - pr.first) * 3; }
    for (int r = 0; r < W; ++r) {
        soff[r] = S;
        if (r != me) { auto pr = part(me, r); S += (pr.second - pr.first) * 3; }
    }
    const size_t words = (size_t)(S + R) + 1;
    if (c->xbuf_cap < words) {
        WSMC_HIP(ctx_sync(c, c->stream));
        if (c->xbuf) WSMC_HIP(hipFree(c->xbuf));
        WSMC_HIP(hipMalloc(&c->xbuf, sizeof(unsigned long long) * words));
        c->xbuf_cap = words;
    }
    unsigned long long* sendbuf = c->xbuf;
    unsigned long long* recvbuf = c->xbuf + S;
    const unsigned long long g0 = x.gofs[me];
    for (int r = 0; r < W; ++r) {
        auto pr = part(me, r);
        if (pr.second <= pr.first) continue;
        unsigned long long* dst = r == me ? recvbuf + (pr.first - lome) * 3 : sendbuf + soff[r];
        WSMC_HIP(launch_trace_pack(c->stream, hist, arow, (int64_t)(pr.first - g0), (int64_t)(pr.second - pr.first),
                                   dst));
    }
    if (c->host_exchange) {
        unsigned long long maxS = 0;
        for (int g = 0; g < W; ++g) maxS = Sg[g] > maxS ? Sg[g] : maxS;
        if (maxS > 0) {
            if (maxS > 0x7fffffffull) return fail(WSMC_EARG, "host exchange block too large");
            std::vector<unsigned long long> mine(maxS, 0ull), all((size_t)maxS * W);
            if (S) WSMC_HIP(hipMemcpyAsync(mine.data(), sendbuf, sizeof(unsigned long long) * S, hipMemcpyDeviceToHost,
                                           c->stream));
            WSMC_HIP(ctx_sync(c, c->stream));
            if (host_xchg(c, reinterpret_cast<const uint64_t*>(mine.data()), (int32_t)maxS,
                                 reinterpret_cast<uint64_t*>(all.data())) != 0)
                return fail(WSMC_ERCCL, "host trace-back exchange failed");
            for (int g = 0; g < W; ++g) {
                if (g == me) continue;
                auto pr = part(g, me);
                if (pr.second <= pr.first) continue;
                unsigned long long off = 0;
                for (int r = 0; r < me; ++r)
                    if (r != g) { auto q = part(g, r); off += (q.second - q.first) * 3; }
                WSMC_HIP(hipMemcpyAsync(recvbuf + (pr.first - lome) * 3, all.data() + (size_t)g * maxS + off,
                                        sizeof(unsigned long long) * (pr.second - pr.first) * 3, hipMemcpyHostToDevice,
                                        c->stream));
            }
            WSMC_HIP(ctx_sync(c, c->stream));
        }
    } else {
        WSMC_RCCL_GUARD(c);
        c->exchanges += 1;
        WSMC_RCCL(ncclGroupStart());
        for (int r = 0; r < W; ++r) {
            if (r == me) continue;
            auto ps = part(me, r), pr = part(r, me);
            if (ps.second > ps.first)
                WSMC_RCCL(ncclSend(sendbuf + soff[r], (size_t)(ps.second - ps.first) * 3, ncclUint64, r, c->comm,
                                   c->stream));
            if (pr.second > pr.first)
                WSMC_RCCL(ncclRecv(recvbuf + (pr.first - lome) * 3, (size_t)(pr.second - pr.first) * 3, ncclUint64,
                                   r, c->comm, c->stream));
        }
        WSMC_RCCL(ncclGroupEnd());
    }
    WSMC_HIP(launch_trace_lookup(c->stream, recvbuf, (int64_t)lome, a, n, xout, anext, arow ? 1 : 0));
    return WSMC_OK;
}

// ---- analysis reductions (src/utils.jl) ----------------------------------------------
// all-gather `words` (<= 16) host words per rank through the exchange buffer; all[W * words]
static int allgather_host_words(wsmc_ctx* c, const unsigned long long* mine, int words, unsigned long long* all) {
    unsigned long long* dbuf = c->xchg;   // 16 words per rank
    WSMC_HIP(hipMemcpyAsync(dbuf + (size_t)c->rank * words, mine, sizeof(unsigned long long) * words,
                            hipMemcpyHostToDevice, c->stream));
    int r = exchange_words(c, dbuf, words, c->stream);
    if (r) return r;
    WSMC_HIP(hipMemcpyAsync(all, dbuf, sizeof(unsigned long long) * words * c->world, hipMemcpyDeviceToHost,
                            c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}
// the population's max log-weight into c->mslots (slot 0; the others zero), so that every
// shard's exp(lw - M) and integer weights are relative to the same M
static int adopt_global_max(wsmc_ctx* c) {
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    MaxSlots hs;
    WSMC_HIP(hipMemcpyAsync(&hs, c->mslots, sizeof(MaxSlots), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    unsigned long long menc = 0;
    for (int k = 0; k < kSlots; ++k) menc = hs.v[k][0] > menc ? hs.v[k][0] : menc;
    std::vector<unsigned long long> ex(c->world);
    int r = allgather_host_words(c, &menc, 1, ex.data());
    if (r) return r;
    for (int g = 0; g < c->world; ++g) menc = ex[g] > menc ? ex[g] : menc;
    std::memset(&hs, 0, sizeof(hs));
    hs.v[0][0] = menc;
    WSMC_HIP(hipMemcpyAsync(c->mslots, &hs, sizeof(MaxSlots), hipMemcpyHostToDevice, c->stream));
    return WSMC_OK;
}

int wsmc_weighted_moments(wsmc_ctx* c, const wsmc_operand* exprs, int32_t d, double* mean, double* cov) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double m[4], v[16]; int r = wsmc_weighted_moments(x, exprs, d, mean ? m : nullptr, cov ? v : nullptr); if (!r && x == multi_first(c)) { if (mean) std::memcpy(mean, m, sizeof(double) * (d > 0 && d <= 4 ? d : 0)); if (cov) std::memcpy(cov, v, sizeof(double) * (d > 0 && d <= 4 ? d * d : 0)); } return r; });
    CHECK_CTX(c);
    if (!exprs || !mean || d < 1 || d > 4) return fail(WSMC_EARG, "need 1..4 expressions and a mean buffer");
    std::vector<int32_t> reads;
    if (int r = check_deferred(c)) return r;   // the moment kernels share the flag word
    for (int k = 0; k < d; ++k) {
        int r = check_operand(c, exprs[k]);
        if (r) return r;
        cols_of(exprs[k], reads);
    }
    int r = need_cols(c, reads);
    if (!r) r = upload_colptr(c);
    if (r) return r;
    wsmc_operand ex[4];
    for (int k = 0; k < 4; ++k) ex[k] = exprs[k < d ? k : 0];
    if (is_sharded(c)) {
        // population-wide: the global max, then each shard's canonical totals combined in
        // rank order (the sharded autoRW's moment protocol), means, then centred products
        if ((r = adopt_global_max(c))) return r;
        const int W = c->world, n1 = 1 + d, n2 = d * (d + 1) / 2;
        std::vector<unsigned long long> all(16 * W);
        double mom[64];
        auto rank_sums = [&](int n, double* out) {
            for (int v = 0; v < n; ++v) {
                double acc = 0.0;
                for (int g = 0; g < W; ++g) {
                    double x;
                    std::memcpy(&x, &all[(size_t)g * n + v], 8);
                    acc = g == 0 ? x : acc + x;
                }
                out[v] = acc;
            }
        };
        WSMC_HIP(launch_moments_expr(c->stream, c->w, c->mslots, c->d_colptr, ex, d, 1, c->mom, c->N, c->tilepart));
        WSMC_HIP(launch_moments_final(c->stream, c->tilepart, c->ntiles, d, 1, 0.0, c->mom, c->dflag, 2));
        WSMC_HIP(hipMemcpyAsync(mom, c->mom, sizeof(mom), hipMemcpyDeviceToHost, c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        if ((r = allgather_host_words(c, reinterpret_cast<const unsigned long long*>(mom + 48), n1, all.data())))
            return r;
        double t1[5];
        rank_sums(n1, t1);
        const double S0 = t1[0];
        for (int k = 0; k < d; ++k) mean[k] = mom[k] = t1[1 + k] / S0;
        mom[8] = S0;
        if (!cov) return WSMC_OK;
        WSMC_HIP(hipMemcpyAsync(c->mom, mom, sizeof(double) * 16, hipMemcpyHostToDevice, c->stream));
        WSMC_HIP(launch_moments_expr(c->stream, c->w, c->mslots, c->d_colptr, ex, d, 2, c->mom, c->N, c->tilepart));
        WSMC_HIP(launch_moments_final(c->stream, c->tilepart, c->ntiles, d, 2, 0.0, c->mom, c->dflag, 2));
        WSMC_HIP(hipMemcpyAsync(mom + 48, c->mom + 48, sizeof(double) * 16, hipMemcpyDeviceToHost, c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        if ((r = allgather_host_words(c, reinterpret_cast<const unsigned long long*>(mom + 48), n2, all.data())))
            return r;
        double t2[10];
        rank_sums(n2, t2);
        int v = 0;
        for (int a = 0; a < d; ++a)
            for (int b = a; b < d; ++b) {
                const double cv = t2[v++] / S0;
                cov[a * d + b] = cv;
                cov[b * d + a] = cv;
            }
        return WSMC_OK;
    }
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    WSMC_HIP(launch_moments_expr(c->stream, c->w, c->mslots, c->d_colptr, ex, d, 1, c->mom, c->N, c->tilepart));
    WSMC_HIP(launch_moments_final(c->stream, c->tilepart, c->ntiles, d, 1, 0.0, c->mom, c->dflag, 1));
    if (cov) {
        WSMC_HIP(launch_moments_expr(c->stream, c->w, c->mslots, c->d_colptr, ex, d, 2, c->mom, c->N, c->tilepart));
        WSMC_HIP(launch_moments_final(c->stream, c->tilepart, c->ntiles, d, 2, 0.0, c->mom, c->dflag, 1));
    }
    double h[32];
    WSMC_HIP(hipMemcpyAsync(h, c->mom, sizeof(double) * 32, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    for (int k = 0; k < d; ++k) mean[k] = h[k];
    if (cov)
        for (int k = 0; k < d * d; ++k) cov[k] = h[16 + k];
    return WSMC_OK;
}

int wsmc_col_minmax(wsmc_ctx* c, int32_t col, int32_t comp, double* mn, double* mx) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double a, b; int r = wsmc_col_minmax(x, col, comp, mn ? &a : nullptr, mx ? &b : nullptr); if (!r && x == multi_first(c)) { *mn = a; *mx = b; } return r; });
    CHECK_CTX(c);
    if (col < 0 || col >= (int32_t)c->cols.size()) return fail(WSMC_EARG, "bad column");
    if (comp < 0 || comp >= c->cols[col].dim) return fail(WSMC_EARG, "bad component");
    if (!mn || !mx) return fail(WSMC_EARG, "null output");
    if (int r = need_cols(c, {col})) return r;
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_minmax(c->stream, c->cols[col].front + (int64_t)comp * c->N, c->N, c->mslots));
    MaxSlots h;
    WSMC_HIP(hipMemcpyAsync(&h, c->mslots, sizeof(MaxSlots), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    unsigned long long a = 0, b = 0;
    for (int k = 0; k < kSlots; ++k) {
        a = h.v[k][0] > a ? h.v[k][0] : a;
        b = h.v[k][1] > b ? h.v[k][1] : b;
    }
    if (is_sharded(c)) {   // the population's extremes (order-free)
        const unsigned long long mine[2] = {a, b};
        std::vector<unsigned long long> all(2 * c->world);
        const int r = allgather_host_words(c, mine, 2, all.data());
        if (r) return r;
        for (int g = 0; g < c->world; ++g) {
            a = all[2 * g] > a ? all[2 * g] : a;
            b = all[2 * g + 1] > b ? all[2 * g + 1] : b;
        }
    }
    *mx = wsmc_ord_dec(a);
    *mn = -wsmc_ord_dec(b);
    return WSMC_OK;
}

// integer weights q of the current log-weights into qbuf; their total (0: not normalisable)
static int local_q(wsmc_ctx* c, unsigned long long* Q) {
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf));
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 0, 0.0, nullptr, nullptr));
    ShardRecord* hr = reinterpret_cast<ShardRecord*>(c->pinned);
    WSMC_HIP(hipMemcpyAsync(hr, c->rec, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    *Q = hr->Q;
    return WSMC_OK;
}

// StatsBase's weighted median of n (value, integer weight) pairs; zero weights drop out, so
// zero-weight padding is harmless
static int median_of(wsmc_ctx* c, const double* x, const unsigned long long* q, int64_t n, double* out) {
    using u64 = unsigned long long;
    u64* buf = nullptr;
    WSMC_HIP(hipMalloc(&buf, sizeof(u64) * 4 * (size_t)n));
    u64 *kin = buf, *kout = buf + n, *vin = buf + 2 * n, *vout = buf + 3 * n;
    hipError_t e = launch_median_keys(c->stream, x, q, n, kin, vin);
    // (value, weight) order: stable radix sorts by weight, then by value
    size_t tb1 = 0, tb2 = 0;
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb1, kin, kout, vin, vout, (int)n, 0, 64, c->stream);
    if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(nullptr, tb2, vin, kout, (int)n, c->stream);
    const size_t tb = (tb1 > tb2 ? tb1 : tb2) + 16;
    void* ts = nullptr;
    double* dout = nullptr;
    if (e == hipSuccess) e = hipMalloc(&ts, tb);
    if (e == hipSuccess) e = hipMalloc(&dout, sizeof(double));
    size_t t = tb;
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(ts, t, kin, kout, vin, vout, (int)n, 0, 64, c->stream);
    t = tb;
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(ts, t, vout, kin, kout, vin, (int)n, 0, 64, c->stream);
    t = tb;
    if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(ts, t, vin, kout, (int)n, c->stream);
    if (e == hipSuccess) e = launch_median_pick(c->stream, kin, vin, kout, n, dout);
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = ctx_sync(c, c->stream);
    if (ts) (void)hipFree(ts);
    if (dout) (void)hipFree(dout);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(WSMC_EHIP, std::string("weighted median: ") + hipGetErrorString(e));
    return WSMC_OK;
}

int wsmc_weighted_median(wsmc_ctx* c, int32_t col, int32_t comp, double* out) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double v; int r = wsmc_weighted_median(x, col, comp, out ? &v : nullptr); if (!r && x == multi_first(c)) *out = v; return r; });
    CHECK_CTX(c);
    if (!out) return fail(WSMC_EARG, "null output");
    double mn, mx;
    int r = wsmc_col_minmax(c, col, comp, &mn, &mx);   // population-wide on shards
    if (r) return r;
    if (wsmc_isnan(mx)) { *out = mx; return WSMC_OK; }          // a NaN value: NaN (StatsBase)
    const double* x = c->cols[col].front + (int64_t)comp * c->N;
    if (!is_sharded(c)) {
        unsigned long long Q = 0;
        if ((r = local_q(c, &Q))) return r;
        if (Q == 0) return fail(WSMC_ESTATE, "weight vector cannot sum to zero");
        return median_of(c, x, c->qbuf, c->N, out);
    }
    // shards: integer weights relative to the population's max (the single-context q), then
    // every rank's (value, q) all-gathered, zero-weight padded to the largest shard, and the
    // median taken over the union on every rank
    using u64 = unsigned long long;
    if ((r = adopt_global_max(c))) return r;
    WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, nullptr, nullptr, nullptr, 1, c->gN));
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 0, 0.0, nullptr, nullptr));
    ShardRecord* hr = reinterpret_cast<ShardRecord*>(c->pinned);
    WSMC_HIP(hipMemcpyAsync(hr, c->rec, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    const u64 mine[2] = {(u64)c->N, hr->Q};
    std::vector<u64> all(2 * c->world);
    if ((r = allgather_host_words(c, mine, 2, all.data()))) return r;
    u64 nmax = 1, Q = 0;
    for (int g = 0; g < c->world; ++g) {
        nmax = all[2 * g] > nmax ? all[2 * g] : nmax;
        Q += all[2 * g + 1];
    }
    if (Q == 0) return fail(WSMC_ESTATE, "weight vector cannot sum to zero");
    const int64_t U = (int64_t)nmax * c->world;
    u64* g = nullptr;
    WSMC_HIP(hipMalloc(&g, sizeof(u64) * 2 * (size_t)U));
    u64 *gx = g, *gq = g + U;
    hipError_t e = hipMemsetAsync(g, 0, sizeof(u64) * 2 * (size_t)U, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(gx + nmax * c->rank, x, sizeof(double) * c->N, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(gq + nmax * c->rank, c->qbuf, sizeof(u64) * c->N, hipMemcpyDeviceToDevice, c->stream);
    if (e != hipSuccess) {
        (void)hipFree(g);
        return fail(WSMC_EHIP, std::string("weighted median: ") + hipGetErrorString(e));
    }
    r = exchange_words(c, gx, (int64_t)nmax, c->stream);
    if (!r) r = exchange_words(c, gq, (int64_t)nmax, c->stream);
    if (!r) r = median_of(c, reinterpret_cast<const double*>(gx), gq, U, out);
    (void)hipFree(g);
    return r;
}

int wsmc_histogram(wsmc_ctx* c, int32_t col, int32_t comp, int32_t levels[8]) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { int32_t lv[8]; int r = wsmc_histogram(x, col, comp, levels ? lv : nullptr); if (!r && x == multi_first(c)) std::memcpy(levels, lv, sizeof(lv)); return r; });
    CHECK_CTX(c);
    if (!levels) return fail(WSMC_EARG, "null output");
    double lo, hi;
    int r = wsmc_col_minmax(c, col, comp, &lo, &hi);   // population-wide on shards
    if (r) return r;
    if (lo == hi) {                                                // _sparkline(fill(sum(w), 8))
        for (int b = 0; b < 8; ++b) levels[b] = 8;
        return WSMC_OK;
    }
    unsigned long long Q = 0;
    const bool sh = is_sharded(c);
    if (sh) {
        // integer weights relative to the population's max with the global N's K: exactly
        // the single-context q, so the summed bins are the unsharded bins
        if ((r = adopt_global_max(c))) return r;
        WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, nullptr, nullptr, nullptr, 1,
                                c->gN));
        WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 0, 0.0, nullptr,
                                  nullptr));
        ShardRecord* hr = reinterpret_cast<ShardRecord*>(c->pinned);
        WSMC_HIP(hipMemcpyAsync(hr, c->rec, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        const unsigned long long mine = hr->Q;
        std::vector<unsigned long long> all(c->world);
        if ((r = allgather_host_words(c, &mine, 1, all.data()))) return r;
        for (int g = 0; g < c->world; ++g) Q += all[g];
    } else if ((r = local_q(c, &Q))) {
        return r;
    }
    if (Q == 0) return fail(WSMC_ESTATE, "the weights do not normalise (all -Inf or NaN)");
    double edges[9];
    for (int k = 0; k <= 8; ++k) edges[k] = wsmc_linspace_edge(lo, hi, k, 8);
    unsigned long long* cnt = c->xchg;
    WSMC_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * 8, c->stream));
    WSMC_HIP(launch_hist(c->stream, c->cols[col].front + (int64_t)comp * c->N, c->qbuf, c->N, edges, cnt));
    unsigned long long h[8];
    WSMC_HIP(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    if (sh) {   // integer bin sums: order-free
        std::vector<unsigned long long> all(8 * c->world);
        if ((r = allgather_host_words(c, h, 8, all.data()))) return r;
        for (int b = 0; b < 8; ++b) {
            h[b] = 0;
            for (int g = 0; g < c->world; ++g) h[b] += all[(size_t)g * 8 + b];
        }
    }
    unsigned long long mxc = 0;
    for (int b = 0; b < 8; ++b) mxc = h[b] > mxc ? h[b] : mxc;
    for (int b = 0; b < 8; ++b) levels[b] = wsmc_spark_level(h[b], mxc);
    return WSMC_OK;
}

int wsmc_ess(wsmc_ctx* c, double* ess_perc) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double v; int r = wsmc_ess(x, &v); if (x == multi_first(c) && ess_perc) *ess_perc = v; return r; });
    CHECK_CTX(c);
    if (!ess_perc) return fail(WSMC_EARG, "null output");
    if (exact_mode(c)) {
        wsmc_shard_stats st;
        int r = exact_global_stats(c, &st);
        if (r) return r;
        *ess_perc = wsmc_global_ess(&st, 1);
        return WSMC_OK;
    }
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_log_evidence_stats(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, c->tileOff,
                                       c->rec + c->rank));
    int r = exchange_recs(c, c->rec);
    if (r) return r;
    std::vector<ShardRecord> h(c->world);
    WSMC_HIP(hipMemcpyAsync(h.data(), c->rec, sizeof(ShardRecord) * c->world, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    wsmc_shard_stats st[kMaxWorld];
    for (int g = 0; g < c->world; ++g) st[g] = host_record_stats(h[g]);
    *ess_perc = wsmc_global_ess(st, c->world);
    return WSMC_OK;
}

// sample(state, n; replace) over a sharded population (global indices, the single-context
// draws): integer weights relative to the population's max with the global N's K.
//   replace: every rank locates the draws whose target falls in its CDF range (its base is
//   the lower ranks' Q); the owners' answers are all-gathered.
//   no replace: each rank's top-min(n, N) Efraimidis–Spirakis keys (keyed by global index)
//   are all-gathered and the union re-sorted: by global index, then stably by key
//   (descending), as one context's stable sort orders them.
static int sample_particles_sharded(wsmc_ctx* c, int64_t n, int32_t replace, int64_t* idx_out) {
    using u64 = unsigned long long;
    const uint64_t op = c->op++;
    const int W = c->world;
    int r = adopt_global_max(c);
    if (r) return r;
    WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, nullptr, nullptr, nullptr, 1, c->gN));
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 0, 0.0, nullptr, nullptr));
    ShardRecord* hr = reinterpret_cast<ShardRecord*>(c->pinned);
    WSMC_HIP(hipMemcpyAsync(hr, c->rec, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    const u64 mine = hr->Q, mine2[2] = {hr->Q, (u64)c->N};
    std::vector<u64> qs(2 * W);
    if ((r = allgather_host_words(c, mine2, 2, qs.data()))) return r;
    u64 Q = 0, base = 0, nmax = 1;
    for (int g = 0; g < W; ++g) {
        if (g < c->rank) base += qs[2 * g];
        Q += qs[2 * g];
        nmax = qs[2 * g + 1] > nmax ? qs[2 * g + 1] : nmax;
    }
    if (Q == 0) return fail(WSMC_ESTATE, "the weights do not normalise (all -Inf or NaN)");
    std::vector<void*> owned;
    auto done = [&](int rc) {
        for (void* p : owned) (void)hipFree(p);
        return rc;
    };
    auto dalloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
        owned.push_back(p);
        return p;
    };
#define SP_HIP(x)                                                                                  \
    do {                                                                                           \
        const hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return done(fail(WSMC_EHIP, std::string("sample: ") + hipGetErrorString(e_))); \
    } while (0)
    if (replace) {
        u64* cdf = static_cast<u64*>(dalloc(sizeof(u64) * c->N));
        int64_t* all = static_cast<int64_t*>(dalloc(sizeof(int64_t) * (size_t)n * W));
        if (!cdf || !all) return done(fail(WSMC_EHIP, "sample: out of device memory"));
        size_t tb = 0;
        SP_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, c->qbuf, cdf, (int)c->N, c->stream));
        void* ts = dalloc(tb);
        if (!ts) return done(fail(WSMC_EHIP, "sample: out of device memory"));
        SP_HIP(hipcub::DeviceScan::InclusiveSum(ts, tb, c->qbuf, cdf, (int)c->N, c->stream));
        SP_HIP(launch_sample_draws_shard(c->stream, n, c->N, cdf, base, mine, Q, c->seed, op, c->goff,
                                         all + (size_t)n * c->rank));
        if ((r = exchange_words(c, reinterpret_cast<u64*>(all), n, c->stream))) return done(r);
        std::vector<int64_t> h((size_t)n * W);
        SP_HIP(hipMemcpyAsync(h.data(), all, sizeof(int64_t) * h.size(), hipMemcpyDeviceToHost, c->stream));
        SP_HIP(ctx_sync(c, c->stream));
        for (int64_t j = 0; j < n; ++j) {   // exactly one rank owns each draw
            int64_t v = 0;
            for (int g = 0; g < W; ++g) v = h[(size_t)g * n + j] ? h[(size_t)g * n + j] : v;
            idx_out[j] = v - 1;
        }
        return done(WSMC_OK);
    }
    // a shard contributes at most its top m (the same m on every rank; shorter shards pad)
    const int64_t m = n < (int64_t)nmax ? n : (int64_t)nmax, mloc = m < c->N ? m : c->N;
    u64* kin = reinterpret_cast<u64*>(c->tmp);
    u64* kout = kin + c->N;
    u64* vin = kout + c->N;
    u64* vout = vin + c->N;
    SP_HIP(launch_es_keys_shard(c->stream, c->w, c->N, c->gN, c->goff, c->mslots, c->seed, op, kin, vin));
    size_t tb = 0;
    SP_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, kin, kout, vin, vout, (int)c->N, 0, 64,
                                                        c->stream));
    const int64_t U = m * W;
    u64* gk = static_cast<u64*>(dalloc(sizeof(u64) * 2 * (size_t)U));   // keys, then indices
    u64* t4 = static_cast<u64*>(dalloc(sizeof(u64) * 4 * (size_t)U));
    size_t tb2 = 0, tb3 = 0;
    if (!gk || !t4) return done(fail(WSMC_EHIP, "sample: out of device memory"));
    SP_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, gk, t4, gk, t4, (int)U, 0, 64, c->stream));
    SP_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb3, gk, t4, gk, t4, (int)U, 0, 64, c->stream));
    size_t tmax = tb > tb2 ? tb : tb2;
    tmax = tmax > tb3 ? tmax : tb3;
    void* ts = dalloc(tmax + 16);
    if (!ts) return done(fail(WSMC_EHIP, "sample: out of device memory"));
    size_t t = tmax;
    SP_HIP(hipcub::DeviceRadixSort::SortPairsDescending(ts, t, kin, kout, vin, vout, (int)c->N, 0, 64, c->stream));
    u64* gkeys = gk;
    u64* gidx = gk + U;
    SP_HIP(hipMemsetAsync(gk, 0, sizeof(u64) * 2 * (size_t)U, c->stream));   // padding never wins: key 0
    SP_HIP(hipMemcpyAsync(gkeys + m * c->rank, kout, sizeof(u64) * mloc, hipMemcpyDeviceToDevice, c->stream));
    SP_HIP(hipMemcpyAsync(gidx + m * c->rank, vout, sizeof(u64) * mloc, hipMemcpyDeviceToDevice, c->stream));
    if ((r = exchange_words(c, gkeys, m, c->stream))) return done(r);
    if ((r = exchange_words(c, gidx, m, c->stream))) return done(r);
    // by global index, then stably by key, descending
    u64 *i1 = t4, *k1 = t4 + U, *k2 = t4 + 2 * U, *i2 = t4 + 3 * U;
    t = tmax;
    SP_HIP(hipcub::DeviceRadixSort::SortPairs(ts, t, gidx, i1, gkeys, k1, (int)U, 0, 64, c->stream));
    t = tmax;
    SP_HIP(hipcub::DeviceRadixSort::SortPairsDescending(ts, t, k1, k2, i1, i2, (int)U, 0, 64, c->stream));
    SP_HIP(hipMemcpyAsync(idx_out, i2, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream));
    SP_HIP(ctx_sync(c, c->stream));
#undef SP_HIP
    return done(WSMC_OK);
}

int wsmc_sample_particles(wsmc_ctx* c, int64_t n, int32_t replace, int64_t* idx_out) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { std::vector<int64_t> v(n > 0 ? (size_t)n : 1); int r = wsmc_sample_particles(x, n, replace, idx_out ? v.data() : nullptr); if (!r && x == multi_first(c)) std::memcpy(idx_out, v.data(), sizeof(int64_t) * (size_t)n); return r; });
    CHECK_CTX(c);
    if (!idx_out) return fail(WSMC_EARG, "null output");
    if (n <= 0) return fail(WSMC_EARG, "Number of samples must be positive");
    if (!replace && n > c->gN) return fail(WSMC_EARG, "Cannot sample more particles than N without replacement");
    if (is_sharded(c)) return sample_particles_sharded(c, n, replace, idx_out);
    const uint64_t op = c->op++;
    // the integer weights relative to the max (and, with replacement, their CDF)
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    if (replace) {
        if (ensure_cdf(c)) return WSMC_EHIP;
        const FillPlan plan = fill_plan(c, WSMC_RESAMPLE_MULTINOMIAL, op, nullptr);
        WSMC_HIP(launch_rs_sums_multi(c->stream, c->w, c->N, c->mslots, plan, c->tilep, c->cdf, multi_esum(c),
                                      multi_ebuf(c)));
    } else {
        WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf));
    }
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 0, 0.0, nullptr, nullptr));
    ShardRecord* hr = reinterpret_cast<ShardRecord*>(c->pinned);
    WSMC_HIP(hipMemcpyAsync(hr, c->rec, sizeof(ShardRecord), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    if (hr->Q == 0) return fail(WSMC_ESTATE, "the weights do not normalise (all -Inf or NaN)");
    if (replace) {
        int64_t* d = nullptr;
        WSMC_HIP(hipMalloc(&d, sizeof(int64_t) * (size_t)n));
        hipError_t e = launch_sample_draws(c->stream, n, c->N, c->rec, c->tileOff, c->cdf, c->seed, op, d);
        if (e == hipSuccess) e = hipMemcpyAsync(idx_out, d, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = ctx_sync(c, c->stream);
        (void)hipFree(d);
        if (e != hipSuccess) return fail(WSMC_EHIP, std::string("sample: ") + hipGetErrorString(e));
        return WSMC_OK;
    }
    // keys, then a stable descending radix sort of (key, index): the first n are the sample
    unsigned long long* kin = reinterpret_cast<unsigned long long*>(c->tmp);
    unsigned long long* kout = kin + c->N;
    unsigned long long* vin = kout + c->N;
    unsigned long long* vout = vin + c->N;
    WSMC_HIP(launch_es_keys(c->stream, c->w, c->N, c->mslots, c->seed, op, kin, vin));
    size_t tbytes = 0;
    WSMC_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tbytes, kin, kout, vin, vout, (int)c->N, 0, 64,
                                                          c->stream));
    void* tstore = nullptr;
    WSMC_HIP(hipMalloc(&tstore, tbytes + 16));
    hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(tstore, tbytes, kin, kout, vin, vout, (int)c->N, 0, 64,
                                                                c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(idx_out, vout, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = ctx_sync(c, c->stream);
    (void)hipFree(tstore);
    if (e != hipSuccess) return fail(WSMC_EHIP, std::string("sample: ") + hipGetErrorString(e));
    return WSMC_OK;
}

int wsmc_col_gather_rows(wsmc_ctx* c, int32_t col, const int64_t* idx, int64_t n, double* out) {
    if (c && c->multi) return (idx && out && n >= 0) ? multi_gather_rows(c, col, idx, n, out) : fail(WSMC_EARG, "bad arguments");
    CHECK_CTX(c);
    if (!valid_col(c, col) || !idx || !out || n < 0) return fail(WSMC_EARG, "bad arguments");
    if (n == 0) return WSMC_OK;
    for (int64_t j = 0; j < n; ++j)
        if (idx[j] < 0 || idx[j] >= c->N) return fail(WSMC_EARG, "row index out of range");
    if (int r = need_cols(c, {col})) return r;
    const int dim = c->cols[col].dim;
    int64_t* d = nullptr;
    double* o = nullptr;
    WSMC_HIP(hipMalloc(&d, sizeof(int64_t) * (size_t)n));
    hipError_t e = hipMalloc(&o, sizeof(double) * (size_t)n * dim);
    if (e == hipSuccess) e = hipMemcpyAsync(d, idx, sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_gather_rows(c->stream, c->cols[col].front, c->N, dim, d, n, o);
    if (e == hipSuccess) e = hipMemcpyAsync(out, o, sizeof(double) * n * dim, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = ctx_sync(c, c->stream);
    (void)hipFree(d);
    if (o) (void)hipFree(o);
    if (e != hipSuccess) return fail(WSMC_EHIP, std::string("gather rows: ") + hipGetErrorString(e));
    return WSMC_OK;
}

int wsmc_log_evidence(wsmc_ctx* c, double* out) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double v; int r = wsmc_log_evidence(x, &v); if (x == multi_first(c) && out) *out = v; return r; });
    CHECK_CTX(c);
    if (!out) return fail(WSMC_EARG, "null out");
    if (exact_mode(c)) {
        wsmc_shard_stats st;
        int r = exact_global_stats(c, &st);
        if (r) return r;
        *out = wsmc_global_log_evidence(&st, 1);
        return WSMC_OK;
    }
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_log_evidence_stats(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf, c->tileOff,
                                       c->rec + c->rank));
    int r = exchange_recs(c, c->rec);
    if (r) return r;
    std::vector<ShardRecord> h(c->world);
    WSMC_HIP(hipMemcpyAsync(h.data(), c->rec, sizeof(ShardRecord) * c->world, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    wsmc_shard_stats st[kMaxWorld];
    for (int g = 0; g < c->world; ++g) st[g] = host_record_stats(h[g]);
    *out = wsmc_global_log_evidence(st, c->world);
    return WSMC_OK;
}

// ---- operators -----------------------------------------------------------------------
int wsmc_assign(wsmc_ctx* c, int32_t out, const wsmc_operand* expr) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_assign(x, out, expr); });
    CHECK_CTX_EW(c);   // reads and writes no weights: a pending reset stays pending
    if (!valid_col(c, out) || !expr) return fail(WSMC_EARG, "bad output column");
    const int dim = c->cols[out].dim;
    for (int k = 0; k < dim; ++k) {
        int r = check_operand(c, expr[k]);
        if (r) return r;
    }
    // an operand column its Sample left unstored is written first; the output is overwritten
    for (int k = 0; k < dim; ++k)
        for (int m = 0; m < 2; ++m)
            if (expr[k].col[m] >= 0)
                if (int rv = virt_one(c, expr[k].col[m])) return rv;
    virt_drop(c, out);
    // operand columns one Resample behind are read through that Resample's ancestors inside
    // the kernel (no materialising pass); any further behind are brought up to date first
    std::vector<int32_t> deep;
    for (int k = 0; k < dim; ++k)
        for (int m = 0; m < 2; ++m) {
            const int32_t id = expr[k].col[m];
            if (id >= 0 && c->cols[id].epoch < c->epoch - 1) deep.push_back(id);
        }
    int r = deep.empty() ? WSMC_OK : materialize(c, &deep);
    if (!r) r = upload_colptr(c);
    if (r) return r;
    Indirect ind;
    bool out_read_behind = false;
    for (int k = 0; k < dim; ++k)
        for (int m = 0; m < 2; ++m) {
            const int32_t id = expr[k].col[m];
            if (id < 0) continue;
            c->cols[id].touch = c->epoch;
            if (c->cols[id].epoch < c->epoch) {
                ind.mask |= 1u << (2 * k + m);
                out_read_behind |= id == out;
            }
        }
    if (ind.mask) {
        const AncRow& nr = c->alog.back();   // entry epoch - 1 (kept alive by the stale column)
        ind.row = nr.anc;
        ind.dec = nr.dec;
    }
    std::vector<const double*> fronts(c->cols.size());
    for (size_t k = 0; k < c->cols.size(); ++k) fronts[k] = c->cols[k].front;   // before any swap
    ind.front = fronts.data();
    double* dst = c->cols[out].front;
    EwBatch* b = ew_enabled(c) ? ew_open(c) : nullptr;
    // the batch: full, another ancestor row, a full table-move list, or an in-place write of a
    // column the batch reads through the ancestors -> launch it first
    if (b && b->nops > 0 &&
        (b->nops == kEwOps || (ind.mask && b->anc && b->anc != ind.row) || (out_read_behind && b->ntab == 4) ||
         (!out_read_behind && ew_reads_lagged(c, out))))
        if ((r = ew_flush(c))) return r;
    if (out_read_behind) {   // out read through the ancestors: write a fresh buffer (no read/write race)
        dst = c->cols[out].back;
        ind.tab_col = out;
        ind.tab = c->d_colptr;
        std::swap(c->cols[out].front, c->cols[out].back);
    }
    scores_touch(c, out);
    wrote_col(c, out);
    if (b) {
        EwOp& op = b->ops[b->nops];
        std::memset(&op, 0, sizeof(op));
        op.kind = 0;
        op.dim = dim;
        op.out = dst;
        for (int k = 0; k < 4; ++k) {
            op.a.e[k] = expr[k < dim ? k : 0];
            for (int m = 0; m < 2; ++m) {
                const int32_t id = op.a.e[k].col[m];
                op.a.p[k][m] = id >= 0 ? fronts[id] + (int64_t)op.a.e[k].comp[m] * c->N : nullptr;
                op.a.fwd[k][m] = -1;
                if (id < 0 || k >= dim) continue;
                const int lag = (ind.mask >> (2 * k + m)) & 1;
                if (lag) c->ew_lag.push_back(id);
                // its LDS rows: an earlier statement's output, or loaded at the start (directly
                // or through the ancestors); without room the kernel reads the column itself
                int rr = ew_row_of(c, fronts[id], lag);
                if (rr < 0) {
                    bool unstaged = false;
                    for (const double* u : c->ew_unstaged) unstaged |= u == fronts[id];
                    if (!unstaged) rr = ew_preload(c, b, fronts[id], c->cols[id].dim, lag);
                }
                if (rr >= 0) op.a.fwd[k][m] = (int8_t)(rr + op.a.e[k].comp[m]);
            }
        }
        op.a.lag = ind.mask;
        op.out_row = (int16_t)ew_out_rows(c, b, dst, dim);
        if (ind.mask) {
            b->anc = ind.row;
            b->dec = ind.dec;
        }
        if (ind.tab_col >= 0) {
            b->tab = ind.tab;
            b->tab_out[b->ntab] = dst;
            b->tab_col[b->ntab] = ind.tab_col;
            b->ntab += 1;
        }
        b->nops += 1;
    } else {
        WSMC_HIP(launch_assign(c->stream, dst, dim, expr, c->d_colptr, c->N, ind));
    }
    gc_log(c);
    c->depth += 1;
    return WSMC_OK;
}

// Assign of a general expression (include/wsmc.h): the program checked on the host, its column
// reads resolved to component pointers; columns one lazy Resample behind are read through that
// Resample's ancestors (deeper ones are brought up to date first), as wsmc_assign's
int wsmc_assign_expr(wsmc_ctx* c, int32_t out, const wsmc_xinst* prog, const int32_t* len) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_assign_expr(x, out, prog, len); });
    CHECK_CTX_EW(c);   // reads and writes no weights: a pending reset stays pending
    if (!valid_col(c, out) || !prog || !len) return fail(WSMC_EARG, "bad output column or program");
    const int dim = c->cols[out].dim;
    static const char* const kWhy[] = {"", "an unknown operator", "a stack underflow",
                                       "more than WSMC_XSTACK_MAX values on the stack",
                                       "a component program that does not leave one value",
                                       "more than WSMC_XPROG_MAX instructions", "a POWI exponent that is no integer"};
    if (int e = wsmc_xprog_check(prog, len, dim)) return fail(WSMC_EARG, std::string("expression: ") + kWhy[-e]);
    int total = 0;
    for (int k = 0; k < dim; ++k) total += len[k];
    std::vector<int32_t> reads;
    for (int q = 0; q < total; ++q) {
        if (prog[q].op != WSMC_X_COL) continue;
        const int32_t id = prog[q].col;
        if (!valid_col(c, id)) return fail(WSMC_EARG, "expression references an unknown column");
        if (prog[q].comp < 0 || prog[q].comp >= c->cols[id].dim)
            return fail(WSMC_EARG, "expression component out of range for column " + c->cols[id].name);
        reads.push_back(id);
    }
    // the statement batch runs first (program order); unstored Sample outputs read here are
    // written, the output's is dropped (overwritten)
    if (int r = ew_flush(c)) return r;
    for (int32_t id : reads)
        if (int r = virt_one(c, id)) return r;
    virt_drop(c, out);
    std::vector<int32_t> deep;
    for (int32_t id : reads)
        if (c->cols[id].epoch < c->epoch - 1) deep.push_back(id);
    int r = deep.empty() ? WSMC_OK : materialize(c, &deep);
    if (!r) r = upload_colptr(c);
    if (r) return r;
    XProg x;
    std::memset(&x, 0, sizeof(x));
    x.N = c->N;
    x.dim = dim;
    x.tab_col = -1;
    for (int k = 0; k < dim; ++k) x.len[k] = len[k];
    bool out_read_behind = false;
    for (int q = 0; q < total; ++q) {
        XIns& I = x.ins[q];
        I.op = prog[q].op;
        I.c = prog[q].c;
        if (I.op != WSMC_X_COL) continue;
        const int32_t id = prog[q].col;
        c->cols[id].touch = c->epoch;
        I.p = c->cols[id].front + (int64_t)prog[q].comp * c->N;
        I.lag = c->cols[id].epoch < c->epoch;
        x.any_lag |= I.lag;
        out_read_behind |= I.lag && id == out;
    }
    if (x.any_lag) {
        const AncRow& nr = c->alog.back();   // entry epoch - 1 (kept alive by the stale column)
        x.row = nr.anc;
        x.dec = nr.dec;
    }
    x.out = c->cols[out].front;
    if (out_read_behind) {   // out read through the ancestors: write a fresh buffer (no read/write race)
        x.out = c->cols[out].back;
        x.tab_col = out;
        x.tab = c->d_colptr;
        std::swap(c->cols[out].front, c->cols[out].back);
    }
    scores_touch(c, out);
    wrote_col(c, out);
    WSMC_HIP(launch_assign_expr(c->stream, x));
    gc_log(c);
    c->depth += 1;
    return WSMC_OK;
}

static void push_sample_term(wsmc_ctx* c, int32_t out, const wsmc_dist& d) {
    wsmc_term t;
    std::memset(&t, 0, sizeof(t));
    t.dist = d;
    for (int k = 0; k < 4; ++k) t.x[k] = col_operand(k < d.dim ? out : -1, k);
    t.kind = WSMC_TERM_SAMPLE;
    t.depth = c->depth;
    c->tape.push_back(t);
}

int wsmc_sample(wsmc_ctx* c, int32_t out, const wsmc_dist* d) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_sample(x, out, d); });
    CHECK_CTX_EW(c);   // reads and writes no weights: a pending reset stays pending
    if (!valid_col(c, out) || !d) return fail(WSMC_EARG, "bad output column");
    int r = check_dist(c, *d);
    if (r) return r;
    if (d->dim != c->cols[out].dim) return fail(WSMC_EARG, "dist dim != column dim");
    std::vector<int32_t> reads;
    cols_of(*d, reads);
    for (int32_t id : reads)
        if ((r = virt_one(c, id))) return r;
    virt_drop(c, out);   // overwritten in full: earlier unstored values are never needed
    if ((r = need_cols(c, reads))) return r;
    if ((r = upload_colptr(c))) return r;
    const uint64_t op = c->op++;
    bool queued = false;
    if (ew_enabled(c)) {   // join the batch (its kernel writes the column in place)
        EwBatch* b = ew_open(c);
        if (b->nops > 0 && (b->nops == kEwOps || ew_reads_lagged(c, out)))
            if ((r = ew_flush(c))) return r;
        EwOp& eo = b->ops[b->nops];
        std::memset(&eo, 0, sizeof(eo));
        eo.s.d = *d;
        auto stage = [&] { return ew_stage(c, b, [&] { return ew_remap_dist(c, b, eo.s.d); }); };
        if (!stage()) {   // no room, or a column written without rows: launch the batch first
            if ((r = ew_flush(c))) return r;
            eo.s.d = *d;
            queued = stage();
        } else {
            queued = true;
        }
    }
    if (queued) {
        EwBatch* b = c->ew;
        EwOp& eo = b->ops[b->nops];
        if (b->nops == 0) c->ew_first.dist = *d;   // as called (a batch of one replays it)
        eo.kind = 1;
        eo.dim = (int16_t)d->dim;
        eo.out = c->cols[out].front;
        eo.out_row = (int16_t)ew_out_rows(c, b, eo.out, d->dim);
        eo.s.op = op;
        eo.s.has_sd = d->family == WSMC_FAM_MVNORMAL_ISO && wsmc_operand_is_const(&d->scale);
        eo.s.sd = eo.s.has_sd ? wsmc_sqrt(wsmc_operand_eval(&d->scale, nullptr, c->N, 0, nullptr)) : 0.0;
        c->ew_feat |= wsmc_dist_feat(d);
        // a distribution that reads no column: the values are a function of (seed, op,
        // particle), kept in the batch's rows and written only when read (lazy store: a
        // Resample gathers nothing). WSMC_DIAG_STORE_SAMPLES=1 stores them (A/B)
        static const bool store_all = [] {
            const char* e = diag_env("WSMC_DIAG_STORE_SAMPLES");
            return e && atoi(e) != 0;
        }();
        eo.nostore = (int16_t)(reads.empty() && c->lazy && eo.out_row >= 0 && !store_all);
        if (eo.nostore) c->ew_virt.push_back({out, eo.out, *d, op});
        b->nops += 1;
    }
    scores_touch(c, out);
    wrote_col(c, out);
    if (!queued)
        WSMC_HIP(launch_sample(c->stream, c->cols[out].front, d->dim, *d, c->seed, op, c->goff, c->d_colptr, c->N));
    push_sample_term(c, out, *d);
    c->depth += 1;
    return WSMC_OK;
}

int wsmc_sample_importance(wsmc_ctx* c, int32_t out, const wsmc_dist* prop, const wsmc_dist* targ) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_sample_importance(x, out, prop, targ); });
    CHECK_CTX(c);
    if (!valid_col(c, out) || !prop || !targ) return fail(WSMC_EARG, "bad arguments");
    int r = check_dist(c, *prop);
    if (!r) r = check_dist(c, *targ);
    if (r) return r;
    if (prop->dim != c->cols[out].dim || targ->dim != c->cols[out].dim) return fail(WSMC_EARG, "dim mismatch");
    std::vector<int32_t> reads;
    cols_of(*prop, reads);
    cols_of(*targ, reads);
    if ((r = need_cols(c, reads))) return r;
    if ((r = upload_colptr(c))) return r;
    const uint64_t op = c->op++;
    scores_touch(c, out);
    wrote_col(c, out);
    c->wseq += 1;
    WSMC_HIP(launch_sample_importance(c->stream, c->cols[out].front, prop->dim, *prop, *targ, c->w, c->seed, op,
                                      c->goff, c->d_colptr, c->N));
    c->weights_changed = 1;
    push_sample_term(c, out, *targ);
    c->depth += 1;
    return WSMC_OK;
}

// the largest value a weight term's log density can take, computed as the kernels compute it
// (the same header functions): a constant-scale Normal is fma(-h, h, c) <= c, HalfNormal that
// plus log 2 (or -inf), an isotropic MvNormal -((d log 2pi + d log var) + s / var) / 2 with
// s >= 0. Rounding is monotone, so w + lp <= base + bound for every particle. None: false.
static bool term_lp_bound(const wsmc_term& t, double* b) {
    const wsmc_dist& d = t.dist;
    if (!wsmc_operand_is_const(&d.scale)) return false;
    const double sc = wsmc_operand_eval(&d.scale, nullptr, 0, 0, nullptr);
    if (!(sc > 0.0) || !(sc < WSMC_INF)) return false;
    switch (d.family) {
        case WSMC_FAM_NORMAL: *b = wsmc_normal_c(wsmc_log(sc)); return true;
        case WSMC_FAM_HALFNORMAL: *b = wsmc_normal_c(wsmc_log(sc)) + WSMC_LOG2; return true;
        case WSMC_FAM_MVNORMAL_ISO: {
            const double dd = (double)d.dim;
            *b = -((dd * WSMC_LOG2PI + dd * wsmc_log(sc)) + 0.0) * 0.5;
            return true;
        }
        default: return false;
    }
}

static int weigh(wsmc_ctx* c, const wsmc_dist* d, const wsmc_operand* x, int kind) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* s) { return weigh(s, d, x, kind); });
    CHECK_CTX_EW(c);   // a pending weight reset is applied by the kernel itself
    if (!d || !x) return fail(WSMC_EARG, "null argument");
    int r = check_dist(c, *d);
    if (r) return r;
    wsmc_term t;
    std::memset(&t, 0, sizeof(t));
    t.dist = *d;
    for (int k = 0; k < 4; ++k) {
        t.x[k] = x[k < d->dim ? k : 0];
        if ((r = check_operand(c, t.x[k]))) return r;
    }
    t.kind = kind;
    t.depth = c->depth;
    wsmc_osc_link(c->tape.empty() ? nullptr : &c->tape.back(), &t);   // before its first evaluation
    std::vector<int32_t> reads;
    cols_of(t, reads);
    for (int32_t id : reads)
        if ((r = virt_one(c, id))) return r;
    if ((r = need_cols(c, reads))) return r;
    if ((r = upload_colptr(c))) return r;
    int wb = c->wnext;
    bool queued = false;
    if (ew_enabled(c)) {   // join the batch: its weight terms share one register and one max
        EwBatch* b = ew_open(c);
        if (b->nops == kEwOps)
            if ((r = ew_flush(c))) return r;
        EwOp& eo = b->ops[b->nops];
        std::memset(&eo, 0, sizeof(eo));
        eo.w.t = t;
        auto stage = [&] {
            return ew_stage(c, b, [&] {
                if (!ew_remap_dist(c, b, eo.w.t.dist)) return false;
                for (int k = 0; k < 4; ++k)
                    if (!ew_remap(c, b, eo.w.t.x[k])) return false;
                return true;
            });
        };
        if (!stage()) {   // no room, or a column written without rows: launch the batch first
            if ((r = ew_flush(c))) return r;
            eo.w.t = t;
            queued = stage();
        } else {
            queued = true;
        }
    }
    if (queued) {
        EwBatch* b = c->ew;
        EwOp& eo = b->ops[b->nops];
        if (b->nops == 0) c->ew_first = t;   // as called (a batch of one replays it)
        eo.kind = 2;
        eo.dim = (int16_t)t.dist.dim;
        eo.out_row = -1;
        eo.w.lm0 = wsmc_logmemo{0, 0.0, 0.0, 0};
        if (t.dist.family != WSMC_FAM_UNIFORM && wsmc_operand_is_const(&t.dist.scale)) {
            const double sc = wsmc_operand_eval(&t.dist.scale, nullptr, c->N, 0, nullptr);
            eo.w.lm0 = wsmc_logmemo{wsmc_d2bits(sc), wsmc_log(sc), 1.0 / sc, 1};
        }
        c->ew_feat |= wsmc_dist_feat(&t.dist);
        if (!b->has_w) {   // the batch's first weight term: the pending reset, the slot pair
            b->has_w = 1;
            b->w = c->w;
            b->wreset = c->w_reset_pending;
            b->ms = c->wslots[wb];
            b->ms_next = c->wslots[wb ^ 1];
            c->wnext = wb ^ 1;
            // the weights entering the batch are the last fused Resample's (statistics guess)
            c->ew_qs_ok = c->rs_base_seq == c->wseq;
            b->nqb = 0;
        } else {
            wb = c->wmax_buf;   // the batch's max goes to its first term's slots
        }
        double bd = 0.0;
        if (c->ew_qs_ok && b->nqb < kEwOps && term_lp_bound(t, &bd))
            b->qb[b->nqb++] = bd;
        else
            c->ew_qs_ok = false;
        b->nops += 1;
    } else {
        WSMC_HIP(launch_weigh(c->stream, t, c->w, c->d_colptr, c->N, c->wslots[wb], c->wslots[wb ^ 1],
                              c->w_reset_pending));
        c->wnext = wb ^ 1;
    }
    c->w_reset_pending = nullptr;
    c->wmax_buf = wb;
    c->wseq += 1;
    c->wmax_seq = c->wseq;
    c->cur_max = c->wslots[wb];
    c->cur_max_seq = c->wseq;
    c->tape.push_back(t);
    c->weights_changed = 1;
    c->depth += 1;
    return WSMC_OK;
}

int wsmc_observe(wsmc_ctx* c, const wsmc_dist* d, const wsmc_operand* x) { return weigh(c, d, x, WSMC_TERM_OBSERVE); }
int wsmc_weight(wsmc_ctx* c, const wsmc_dist* d, const wsmc_operand* x) { return weigh(c, d, x, WSMC_TERM_WEIGHT); }

// diagnostics: the generic Resample's reduce-kernel sequence instead of the fused pair
static bool no_fused_resample() {
    static const bool v = [] {
        const char* e = diag_env("WSMC_DIAG_RESAMPLE_REDUCE");
        return e && atoi(e) != 0;
    }();
    return v;
}
static inline int64_t run_grp_words(int64_t N);

int wsmc_resample(wsmc_ctx* c, double ess_min, int32_t scheme, int32_t* resampled_out, double* ess_out) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { int32_t rs = 0; double e = 0; const bool f = x == multi_first(c); int r = wsmc_resample(x, ess_min, scheme, resampled_out ? &rs : nullptr, ess_out ? &e : nullptr); if (!r && f) { if (resampled_out) *resampled_out = rs; if (ess_out) *ess_out = e; } return r; });
    CHECK_CTX_EW(c);   // a gated no-op Resample leaves a pending weight reset pending (settled below)
    if (!valid_scheme(scheme)) return fail(WSMC_EARG, "unknown resampling scheme");
    if (scheme == WSMC_RESAMPLE_MULTINOMIAL && exact_mode(c))
        return fail(WSMC_EARG, "multinomial draws on exact shards are not supported (island mode is)");
    if (scheme == WSMC_RESAMPLE_MULTINOMIAL && ensure_cdf(c)) return WSMC_EHIP;
    const uint64_t op = c->op++;
    // no flag requested: the decision stays on the device (gated gather / weight reset), no
    // host round trip; it is folded into the host state at the next read
    const bool async = !resampled_out && !ess_out && !exact_mode(c);
    if (!async) {
        if (int r = resolve_decisions(c)) return r;
        if (int r = check_deferred(c)) return r;
    }
    if (!c->weights_changed) {   // a no-op: the statement batch stays open
        if (resampled_out) *resampled_out = c->resampled;
        if (ess_out) *ess_out = c->last_ess;
        return WSMC_OK;
    }
    // the statistics in the statement batch (round 6; the fused run's statistics in the
    // propagate, for the drop-in statements): when the open batch writes the weights from the
    // last fused Resample's and each of its weight terms has a bound, its kernel takes q and the
    // tile partials against the guessed reference point ceil(base + bounds); k_rs_qfix then
    // checks the guess against the max (a miss recomputes them) in place of k_rs_sums_t
    const bool fused_rs = !is_sharded(c) && !exact_mode(c) && scheme != WSMC_RESAMPLE_MULTINOMIAL && !no_fused_resample();
    if (fused_rs && !c->rs_grp[0]) {
        const int64_t gw = run_grp_words(c->N);
        for (int k = 0; k < 2; ++k) WSMC_HIP(hipMalloc(&c->rs_grp[k], sizeof(unsigned long long) * gw));
        WSMC_HIP(hipMemsetAsync(c->rs_grp[0], 0, sizeof(unsigned long long) * gw, c->stream));
        c->rs_grp_cur = 0;
    }
    bool qs_done = false;
    if (fused_rs && c->ew && c->ew->nops > 0 && c->ew->has_w && c->ew_qs_ok && c->rs_qs && run_qstat_mode(c->N) != 0 &&
        ew_pair_ok(*c->ew, c->N)) {
        if (!c->run_nfix) {
            WSMC_HIP(hipMalloc(&c->run_nfix, sizeof(unsigned long long)));
            WSMC_HIP(hipMemsetAsync(c->run_nfix, 0, sizeof(unsigned long long), c->stream));
        }
        EwBatch* b = c->ew;
        b->qs_base = c->rs_qs;
        b->rg_out = c->rs_qs + 1;
        b->qbuf = c->qbuf;
        b->tilep = c->tilep;
        b->grp = c->rs_grp[c->rs_grp_cur];
        b->G = group_tiles(c->N);
    }
    if (int r = ew_flush(c, &qs_done)) return r;
    if (!c->lazy || is_sharded(c))   // every column gathered now: the unstored ones written first
        if (int r = virt_all(c)) return r;
    if (c->w_reset_pending) {   // (a weight write settles it first, so this does not happen)
        WSMC_HIP(launch_fill_weights(c->stream, c->w, c->w_reset_pending, c->N));
        c->w_reset_pending = nullptr;
    }
    if (exact_mode(c)) {
        Decision d;
        int r = exact_resample(c, ess_min, scheme, op, &d);
        if (r) return r;
        c->last_ess = d.ess;
        c->resampled = d.resampled;
        if (d.resampled) {
            c->n_resamples += 1;
            set_anc_last(c, nullptr, -1);   // the exact route wrote c->anc
        }
        c->weights_changed = 0;
        if (resampled_out) *resampled_out = c->resampled;
        if (ess_out) *ess_out = d.ess;
        return WSMC_OK;
    }
    // the ancestors and the decision land in a row of their own: a log entry (lazy genealogy),
    // or (eager store) a row kept as the last ancestors only if this Resample resamples
    AncRow row;
    int r;
    if ((r = acquire_row(c, &row))) return r;
    FillPlan plan = fill_plan(c, scheme, op, nullptr);
    // stratified / systematic: the fill's tile blocks also reset the weights to the log-mean
    const bool fill_resets = scheme != WSMC_RESAMPLE_MULTINOMIAL;
    if (fill_resets) plan.w_reset = c->w;
    // the last weight write was an Observe / Weight: its kernel left the max in wslots
    const bool pre = c->wmax_buf >= 0 && c->wmax_seq == c->wseq;
    MaxSlots* ms = pre ? c->wslots[c->wmax_buf] : c->mslots;
    // the fill kernel writes the decision straight into host-mapped memory (no copy op): the
    // asynchronous ring's next slot, or the pinned staging the synchronous path reads
    if (async && c->dec_pending == kDecRing)
        if ((r = resolve_decisions(c))) return r;
    Decision* hd = reinterpret_cast<Decision*>(c->pinned);
    plan.host_dec = async ? c->dec_ring_dev + c->dec_pending : reinterpret_cast<Decision*>(c->pinned_dev);
    bool max_kept = false;   // ms holds the max of the weights after this Resample
    if (fused_rs) {
        // one GPU: the fused run's two launches (statistics with group sums, then the fill
        // whose extra block decides), then the gated weight reset — no reduce kernel. The
        // group lines are double-buffered: each fill's record block zeroes the next call's.
        const int64_t gw = run_grp_words(c->N);
        unsigned long long* grp = c->rs_grp[c->rs_grp_cur];
        c->rs_grp_cur ^= 1;
        plan.w_reset = nullptr;
        plan.grp_zero = c->rs_grp[c->rs_grp_cur];
        plan.grp_zero_words = gw;
        plan.ms_reset = pre ? ms : nullptr;
        if (!pre) {
            WSMC_HIP(hipMemsetAsync(ms, 0, sizeof(MaxSlots), c->stream));
            WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, ms));
        }
        const int G = group_tiles(c->N);
        if (qs_done) {   // the batch took the statistics: check its guess (a miss recomputes them)
            c->rs_qs_batches += 1;
            WSMC_HIP(launch_rs_qfix(c->stream, c->w, c->N, ms, c->rs_qs + 1, c->tilep, c->qbuf, grp, G, c->run_nfix));
        } else {
            WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, ms, c->tilep, c->qbuf, nullptr, nullptr, grp, G));
        }
        if (!c->rs_qs) WSMC_HIP(hipMalloc(&c->rs_qs, sizeof(double) * 2));
        plan.base_out = c->rs_qs;   // the next batch's guess starts from the max this leaves
        WSMC_HIP(launch_rs_fill_fused(c->stream, c->N, plan, grp, G, ms, ess_min, c->rec + c->rank, row.dec, c->qbuf,
                                      row.anc));
        // the weight reset is deferred to the first reader (the next Observe applies it in
        // its kernel; any other call runs it first, CHECK_CTX); the fill's record block
        // already leaves the max of the reset weights in ms (an Observe's slots: nothing else
        // writes them before the next Observe, which moves on to the other buffer)
        static const bool eager_reset = [] {   // diagnostics: reset in the Resample (A/B)
            const char* e = diag_env("WSMC_DIAG_EAGER_RESET");
            return e && atoi(e) != 0;
        }();
        if (eager_reset) WSMC_HIP(launch_fill_weights(c->stream, c->w, row.dec, c->N));
        else c->w_reset_pending = row.dec;
        max_kept = pre;
    } else {
        if ((r = enqueue_resample_stats(c, c->w, ms, c->rec, ess_min, row.dec, !pre, plan))) return r;
        if (scheme == WSMC_RESAMPLE_MULTINOMIAL)
        WSMC_HIP(launch_rs_multinomial(c->stream, c->N, c->rec + c->rank, row.dec, plan, c->tileOff, c->cdf,
                                       multi_esum(c), multi_ebuf(c), row.anc));
        else
            WSMC_HIP(launch_rs_scan(c->stream, c->N, c->rec + c->rank, row.dec, plan, c->tileOff, c->qbuf, row.anc));
    }
    if (async) {
        c->dec_pending += 1;
        c->dec_rows.push_back({c->lazy ? c->epoch : -1, row});   // the log entry this Resample becomes
        c->wseq += 1;
        if ((r = store_resample_row(c, row, row.dec, fill_resets ? nullptr : c->w))) return r;   // gated
        c->weights_changed = 0;
        if (max_kept) {
            c->cur_max = ms;
            c->cur_max_seq = c->wseq;
        }
        if (fused_rs) c->rs_base_seq = c->wseq;
        return WSMC_OK;
    }
    WSMC_HIP(ctx_sync(c, c->stream));
    const Decision d = *hd;
    c->last_ess = d.ess;
    if (d.resampled) {
        c->wseq += 1;
        row.known = 1;
        if ((r = store_resample_row(c, row, row.dec, fill_resets ? nullptr : c->w))) return r;
        set_anc_last(c, &row, c->lazy ? c->epoch - 1 : -1);
        c->resampled = 1;
        c->n_resamples += 1;
    } else {
        c->row_pool.push_back(row);   // nothing to log: no particle moved
        c->resampled = 0;
    }
    c->weights_changed = 0;
    if (max_kept) {
        c->cur_max = ms;
        c->cur_max_seq = c->wseq;
    }
    if (fused_rs) c->rs_base_seq = c->wseq;
    if (resampled_out) *resampled_out = c->resampled;
    if (ess_out) *ess_out = d.ess;
    return WSMC_OK;
}

int wsmc_last_ancestors(wsmc_ctx* c, int32_t* host) {
    if (c && c->multi) return host ? multi_last_ancestors(c, host) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!host) return fail(WSMC_EARG, "null buffer");
    if (int r = resolve_decisions(c)) return r;   // which pending Resample resampled last
    const int32_t* src = c->anc_last ? c->anc_last : c->anc;
    WSMC_HIP(hipMemcpyAsync(host, src, sizeof(int32_t) * c->N, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

int wsmc_score(wsmc_ctx* c, int32_t depth, double* host) {
    if (c && c->multi) return host ? multi_score(c, depth, host) : fail(WSMC_EARG, "null buffer");
    CHECK_CTX(c);
    if (!host) return fail(WSMC_EARG, "null buffer");
    std::vector<int32_t> reads;
    for (const auto& t : c->tape) cols_of(t, reads);
    int r = need_cols(c, reads);
    if (!r) r = upload_colptr(c);
    if (!r) r = upload_tape(c);
    if (r) return r;
    WSMC_HIP(launch_score(c->stream, c->d_tape, (int32_t)c->tape.size(), depth, c->d_colptr, c->N, c->tmp));
    WSMC_HIP(hipMemcpyAsync(host, c->tmp, sizeof(double) * c->N, hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    return WSMC_OK;
}

// The population-wide unique count of a shard's sorted keys: each rank
// compacts its unique keys, the ranks all-gather them (padded to the largest count, after
// an all-gather of the counts), and every rank sorts the union and counts it. Every rank
// gets the same count; it equals the unsharded count. `sorted` is N keys; scratch is
// allocated per call (the gate runs once per move).
static int global_unique(wsmc_ctx* c, const unsigned long long* sorted, unsigned long long* u_out) {
    using u64 = unsigned long long;
    const int W = c->world, me = c->rank;
    const int64_t N = c->N;
    std::vector<void*> owned;
    auto dalloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
        owned.push_back(p);
        return p;
    };
    auto done = [&](int rc) {
        for (void* p : owned) (void)hipFree(p);
        return rc;
    };
#define GU_HIP(x)                                                                                  \
    do {                                                                                           \
        const hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return done(fail(WSMC_EHIP, std::string("global_unique: ") + hipGetErrorString(e_))); \
    } while (0)
    u64* uq = static_cast<u64*>(dalloc(sizeof(u64) * N));
    u64* cnt = static_cast<u64*>(dalloc(sizeof(u64) * W));
    u64* nsel = static_cast<u64*>(dalloc(sizeof(u64)));
    if (!uq || !cnt || !nsel) return done(fail(WSMC_EHIP, "global_unique: out of device memory"));
    size_t tb = 0;
    if (hipcub::DeviceSelect::Unique(nullptr, tb, sorted, uq, nsel, (int)N, c->stream) != hipSuccess)
        return done(fail(WSMC_EHIP, "global_unique: select"));
    void* tmp = dalloc(tb);
    if (!tmp) return done(fail(WSMC_EHIP, "global_unique: out of device memory"));
    GU_HIP(hipcub::DeviceSelect::Unique(tmp, tb, sorted, uq, nsel, (int)N, c->stream));
    GU_HIP(hipMemcpyAsync(cnt + me, nsel, sizeof(u64), hipMemcpyDeviceToDevice, c->stream));
    int r = exchange_words(c, cnt, 1, c->stream);
    if (r) return done(r);
    std::vector<u64> hc(W);
    GU_HIP(hipMemcpyAsync(hc.data(), cnt, sizeof(u64) * W, hipMemcpyDeviceToHost, c->stream));
    GU_HIP(ctx_sync(c, c->stream));
    u64 M = 1, tot = 0;
    for (int g = 0; g < W; ++g) {
        M = hc[g] > M ? hc[g] : M;
        tot += hc[g];
    }
    u64* gbuf = static_cast<u64*>(dalloc(sizeof(u64) * M * W));
    u64* all = static_cast<u64*>(dalloc(sizeof(u64) * tot));
    u64* alls = static_cast<u64*>(dalloc(sizeof(u64) * tot));
    if (!gbuf || !all || !alls) return done(fail(WSMC_EHIP, "global_unique: out of device memory"));
    if (hc[me]) GU_HIP(hipMemcpyAsync(gbuf + M * me, uq, sizeof(u64) * hc[me], hipMemcpyDeviceToDevice, c->stream));
    if ((r = exchange_words(c, gbuf, (int64_t)M, c->stream))) return done(r);
    u64 off = 0;
    for (int g = 0; g < W; ++g) {   // the valid prefix of every rank's block
        if (hc[g]) GU_HIP(hipMemcpyAsync(all + off, gbuf + M * g, sizeof(u64) * hc[g], hipMemcpyDeviceToDevice,
                                           c->stream));
        off += hc[g];
    }
    size_t sb = 0;
    GU_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, sb, all, alls, (int)tot, 0, 64, c->stream));
    void* stmp = dalloc(sb);
    if (!stmp) return done(fail(WSMC_EHIP, "global_unique: out of device memory"));
    GU_HIP(hipcub::DeviceRadixSort::SortKeys(stmp, sb, all, alls, (int)tot, 0, 64, c->stream));
    GU_HIP(hipMemsetAsync(nsel, 0, sizeof(u64), c->stream));
    GU_HIP(launch_count_unique(c->stream, alls, (int64_t)tot, nsel));
    GU_HIP(hipMemcpyAsync(u_out, nsel, sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    GU_HIP(ctx_sync(c, c->stream));
    return done(WSMC_OK);
#undef GU_HIP
}

int wsmc_marginal_diversity(wsmc_ctx* c, const int32_t* targets, int32_t d, double* out) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { double v; int r = wsmc_marginal_diversity(x, targets, d, out ? &v : nullptr); if (!r && x == multi_first(c)) *out = v; return r; });
    CHECK_CTX(c);
    if (!targets || d < 1 || !out) return fail(WSMC_EARG, "bad targets");
    for (int k = 0; k < d; ++k)
        if (!valid_col(c, targets[k]) || c->cols[targets[k]].dim != 1)
            return fail(WSMC_EARG, "diversity targets must be scalar columns");
    if (int r = need_cols(c, std::vector<int32_t>(targets, targets + d))) return r;
    unsigned long long* kin = reinterpret_cast<unsigned long long*>(c->tmp);
    unsigned long long* kout = kin + c->N;
    size_t tbytes = 0;
    WSMC_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tbytes, kin, kout, (int)c->N, 0, 64, c->stream));
    void* tstore = nullptr;
    WSMC_HIP(hipMalloc(&tstore, tbytes + 16));
    // one shard: length(unique(col)) / N; sharded: the population-wide count over the global N
    const bool global = is_sharded(c);
    const uint64_t Nd = global ? (uint64_t)c->gN : (uint64_t)c->N;
    double best = INFINITY;
    for (int k = 0; k < d; ++k) {
        hipError_t e = launch_diversity_keys(c->stream, c->cols[targets[k]].front, kin, c->N);
        if (e == hipSuccess)
            e = hipcub::DeviceRadixSort::SortKeys(tstore, tbytes, kin, kout, (int)c->N, 0, 64, c->stream);
        unsigned long long u = 0;
        if (global) {
            if (e != hipSuccess) {
                (void)hipFree(tstore);
                return fail(WSMC_EHIP, std::string("marginal_diversity: ") + hipGetErrorString(e));
            }
            const int r = global_unique(c, kout, &u);
            if (r) {
                (void)hipFree(tstore);
                return r;
            }
        } else {
            if (e == hipSuccess) e = hipMemsetAsync(c->ucount, 0, sizeof(unsigned long long), c->stream);
            if (e == hipSuccess) e = launch_count_unique(c->stream, kout, c->N, c->ucount);
            if (e == hipSuccess)
                e = hipMemcpyAsync(&u, c->ucount, sizeof(u), hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = ctx_sync(c, c->stream);
            if (e != hipSuccess) {
                (void)hipFree(tstore);
                return fail(WSMC_EHIP, std::string("marginal_diversity: ") + hipGetErrorString(e));
            }
        }
        const double frac = wsmc_u64_to_d(u) / wsmc_u64_to_d(Nd);
        if (frac < best) best = frac;
    }
    (void)hipFree(tstore);
    *out = best;
    return WSMC_OK;
}

// autoRW proposal factor on a sharded context: global max log-weight, then
// each rank's canonical moment totals all-gathered and combined in rank order (the
// oracle's sharded restatement), then the same min_step / 2.38/sqrt(d) / Cholesky as the
// single-GPU kernel — all on the stream (k_max_publish/adopt, k_autorw_combine), no host
// round trip: a not-PD factor sets the device flag, the Move skips on it and the host reports
// WSMC_ENOTPD after the Move (state untouched, as the reference throws before changing it).
static int sharded_autorw(wsmc_ctx* c, const int32_t* targets, int d, const double* lo, const double* hi,
                          double min_step) {
    const int W = c->world;
    constexpr int kStride = 16;   // u64 words per rank in c->xchg
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    // each rank's max word and its particle 0's unconstrained values; rank 0's are the pivot
    WSMC_HIP(launch_autorw_publish(c->stream, c->mslots, c->d_colptr, targets, d, lo, hi,
                                   c->xchg + (size_t)c->rank * kStride));
    int r = exchange_words(c, c->xchg, kStride, c->stream);
    if (r) return r;
    // the ranks' maxima sit kStride words apart: gather them into the first W words
    WSMC_HIP(launch_autorw_max(c->stream, c->xchg, W, kStride, c->mslots));
    // one pass: this rank's canonical totals relative to the pivot, all-gathered, combined in
    // rank order (include/wsmc_math.h wsmc_autorw_factor)
    const int nv = 1 + d + d * (d + 1) / 2;
    WSMC_HIP(launch_autorw_moments(c->stream, c->w, c->mslots, c->d_colptr, targets, d, lo, hi, c->xchg + 1, c->N,
                                   c->tilepart));
    WSMC_HIP(launch_autorw_final(c->stream, c->tilepart, c->ntiles, d, min_step, c->mom, c->dflag, 1));
    WSMC_HIP(hipMemcpyAsync(c->xchg + (size_t)c->rank * kStride, c->mom + 48, sizeof(double) * nv,
                            hipMemcpyDeviceToDevice, c->stream));
    if ((r = exchange_words(c, c->xchg, kStride, c->stream))) return r;
    WSMC_HIP(launch_autorw_combine1(c->stream, c->xchg, W, kStride, d, min_step, c->mom, c->dflag));
    return WSMC_OK;
}

// ---- the fold as a segment program (FoldProgram, csrc/wsmc_internal.h) ----------------
static bool same_bits(double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; }
static bool same_operand(const wsmc_operand& a, const wsmc_operand& b, bool c0, bool coef0, bool coef1) {
    return (c0 || same_bits(a.c0, b.c0)) && (coef0 || same_bits(a.coef[0], b.coef[0])) &&
           (coef1 || same_bits(a.coef[1], b.coef[1])) && a.col[0] == b.col[0] && a.col[1] == b.col[1] &&
           a.comp[0] == b.comp[0] && a.comp[1] == b.comp[1];
}
static bool const_operand(const wsmc_operand& o) { return o.col[0] < 0 && o.col[1] < 0; }
// the run kind a term can open: a scalar Normal whose scored value is a constant
static int run_kind(const wsmc_term& t) {
    if (t.dist.family != WSMC_FAM_NORMAL || t.dist.dim != 1 || !const_operand(t.x[0])) return kSegTerm;
    return t.dist.mean_fn == WSMC_MEAN_OSCILLATOR ? kSegNormalOsc : kSegNormalAff;
}
// b continues a's run: everything equal except the run's per-term constants
static bool same_run(const wsmc_term& a, const wsmc_term& b, int kind) {
    if (run_kind(b) != kind || a.dist.mean_fn != b.dist.mean_fn) return false;
    const bool osc = kind == kSegNormalOsc;
    for (int k = 0; k < 4; ++k)
        if (!same_operand(a.dist.mu[k], b.dist.mu[k], !osc && k == 0, !osc && k == 0, !osc && k == 0)) return false;
    if (!same_operand(a.dist.scale, b.dist.scale, false, false, false)) return false;
    // oscillator runs: param[0], param[1], reserved are the per-term (t_a, d, m) (wsmc_osc_link)
    if (!osc && (!same_bits(a.dist.param[0], b.dist.param[0]) || !same_bits(a.dist.param[1], b.dist.param[1])))
        return false;
    return same_operand(a.x[0], b.x[0], true, false, false);   // x[0].c0 = the observation
}
// segments of terms [j0, j1) appended to segs (constants to cst); returns their count
static int32_t compile_fold(const std::vector<wsmc_term>& ct, int32_t j0, int32_t j1, std::vector<FoldSeg>& segs,
                            std::vector<double>& cst) {
    const size_t s0 = segs.size();
    // a constant sigma's log and reciprocal, once here instead of per particle (the shared
    // functions of the same bits: the values the per-particle memo would give)
    auto scale_pre = [&](const wsmc_term& t) -> int32_t {
        const bool scaled = t.dist.family == WSMC_FAM_NORMAL || t.dist.family == WSMC_FAM_HALFNORMAL;
        if (!scaled || !wsmc_term_is_scalar(&t) || !const_operand(t.dist.scale)) return -1;
        double pre[2];
        wsmc_scale_pre(t.dist.scale.c0, pre);
        cst.push_back(pre[0]);
        cst.push_back(pre[1]);
        return (int32_t)cst.size() - 2;
    };
    for (int32_t j = j0; j < j1;) {
        const int kind = run_kind(ct[j]);
        int32_t e = j + 1;
        if (kind != kSegTerm)
            while (e < j1 && same_run(ct[j], ct[e], kind)) ++e;
        // a lone Normal-affine term stays a one-term segment; a lone oscillator term is a run
        // of one (the lean fold carries no generic oscillator evaluation)
        if (kind == kSegTerm || (kind == kSegNormalAff && e - j < 2)) {
            const int32_t so = scale_pre(ct[j]);
            segs.push_back(FoldSeg{kSegTerm, 1, j, 0, so, 0});
            ++j;
            continue;
        }
        int32_t soff = -1;   // runs are scalar Normals: their sigma
        if (const_operand(ct[j].dist.scale)) {
            double pre[2];
            wsmc_scale_pre(ct[j].dist.scale.c0, pre);
            soff = (int32_t)cst.size();
            cst.push_back(pre[0]);
            cst.push_back(pre[1]);
        }
        segs.push_back(FoldSeg{kind, e - j, j, (int32_t)cst.size(), soff, 0});
        if (kind == kSegNormalOsc) {
            // rotation runs (wsmc_mv.h): a term continues the open run when it is the next
            // rotation of the same block (m = m' + 1, the same t_a and step bits) — the
            // continuation test of the term-by-term evaluation; any other term opens a run
            // (anchor, m rotations)
            size_t head = 0;
            int32_t run_m = 0, run_n = 0;
            for (int32_t k = j; k < e; ++k) {
                const wsmc_term& t = ct[k];
                const int32_t m = t.dist.reserved;
                const bool next = run_n > 0 && m > 0 && m == run_m + run_n &&
                                  same_bits(t.dist.param[0], cst[head]) &&
                                  (run_n == 1 && run_m == 0 ? true : same_bits(t.dist.param[1], cst[head + 1]));
                if (next) {
                    if (run_n == 1 && run_m == 0) cst[head + 1] = t.dist.param[1];   // the block's step
                    ++run_n;
                    cst[head + 3] = osc_run_word(run_n);
                } else {
                    head = cst.size();
                    run_m = m;
                    run_n = 1;
                    cst.push_back(t.dist.param[0]);
                    cst.push_back(t.dist.param[1]);
                    cst.push_back(osc_run_word(m));
                    cst.push_back(osc_run_word(1));
                }
                cst.push_back(t.x[0].c0);
            }
            cst.push_back(0.0);   // the pad word: the device loads a run's next observation ahead
        } else {
            for (int32_t k = j; k < e; ++k) {
                const wsmc_term& t = ct[k];
                cst.push_back(t.dist.mu[0].c0);
                cst.push_back(t.dist.mu[0].coef[0]);
                cst.push_back(t.dist.mu[0].coef[1]);
                cst.push_back(t.x[0].c0);
            }
        }
        j = e;
    }
    return (int32_t)(segs.size() - s0);
}

// the device copy of a fold program written at hp (prog_bytes, `need` bytes of the staging ring):
// a content hit in the context's few program slots uploads nothing (and returns the ring space),
// a miss copies into the least recently used slot
static int prog_device(wsmc_ctx* c, const char* hp, size_t prog_bytes, int64_t need, char** dev) {
    const uint64_t tick = ++c->prog_tick;
    for (auto& sl : c->prog_slots)
        if (sl.dev && sl.host.size() == prog_bytes && std::memcmp(sl.host.data(), hp, prog_bytes) == 0) {
            sl.used = tick;
            c->prog_stage_at -= need;   // the staged bytes are not needed (nothing was enqueued from them)
            c->prog_hits += 1;
            *dev = reinterpret_cast<char*>(sl.dev);
            return WSMC_OK;
        }
    wsmc_ctx::ProgSlot* v = &c->prog_slots[0];
    for (auto& sl : c->prog_slots)
        if (sl.used < v->used) v = &sl;
    if ((int64_t)prog_bytes > v->cap) {
        int64_t cap = v->cap ? v->cap : 4096;
        while (cap < (int64_t)prog_bytes) cap *= 2;
        WSMC_HIP(ctx_sync(c, c->stream));   // launches still reading the slot
        if (v->dev) WSMC_HIP(hipFree(v->dev));
        v->dev = nullptr;
        WSMC_HIP(hipMalloc(&v->dev, cap));
        v->cap = cap;
    }
    WSMC_HIP(hipMemcpyAsync(v->dev, hp, prog_bytes, hipMemcpyHostToDevice, c->stream));
    v->host.assign(hp, hp + prog_bytes);
    v->used = tick;
    c->prog_uploads += 1;
    *dev = reinterpret_cast<char*>(v->dev);
    return WSMC_OK;
}

static int move_block_fused(wsmc_ctx* c, int32_t n, const wsmc_move_spec* specs, int32_t gated,
                            int64_t* accepted_out, bool* done);
// WSMC_DIAG_NO_BLOCK1=1: single Moves keep their own kernels (k_move_c / k_move_ci), for comparison
static bool no_block1() {
    static const bool v = [] {
        const char* e = diag_env("WSMC_DIAG_NO_BLOCK1");
        return e && atoi(e) != 0;
    }();
    return v;
}
// a single Move as a block of one: wsmc_move's arguments as a wsmc_move_spec (false: not
// expressible — the Move takes its own path)
static bool move_spec_of(int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
                         const double* hi, int32_t target_depth, wsmc_move_spec& sp) {
    if (proposal != WSMC_PROPOSAL_AUTORW || !targets || d < 1 || d > 4) return false;
    std::memset(&sp, 0, sizeof(sp));
    sp.proposal = proposal;
    sp.d = d;
    for (int k = 0; k < d; ++k) {
        sp.targets[k] = targets[k];
        sp.lo[k] = lo ? lo[k] : -INFINITY;
        sp.hi[k] = hi ? hi[k] : INFINITY;
    }
    sp.bounded = (lo || hi) ? 1 : 0;
    sp.target_depth = target_depth;
    sp.step = step;
    return true;
}

int wsmc_move(wsmc_ctx* c, int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
              const double* hi, int32_t target_depth, double diversity, int64_t* accepted_out) {
    if (c && c->multi)
        return multi_move(c, proposal, targets, d, step, lo, hi, target_depth, diversity, accepted_out);
    // the weights are read by the autoRW moments only, which apply a pending fused-Resample
    // reset themselves (the next Observe applies it to the weights); sharded: settled below
    CHECK_CTX_KEEP(c);
    // an autoRW Move without a diversity gate: a block of one (the fused block path, compiled for
    // its shape), the same bits (tests/test_gpu_parity.py)
    wsmc_move_spec sp1;
    if (std::isnan(diversity) && !c->move_gate && !is_sharded(c) && !no_block1() &&
        move_spec_of(proposal, targets, d, step, lo, hi, target_depth, sp1)) {
        bool done = false;
        const int r = move_block_fused(c, 1, &sp1, 0, accepted_out, &done);
        if (done) return r;
    }
    const uint64_t op_prop = c->op++, op_acc = c->op++;
    if (accepted_out) *accepted_out = 0;
    if (!targets || d < 1 || d > 4) return fail(WSMC_EARG, "move needs 1..4 targets");
    if (proposal != WSMC_PROPOSAL_RW && proposal != WSMC_PROPOSAL_AUTORW) return fail(WSMC_EARG, "unknown proposal");
    for (int k = 0; k < d; ++k)
        if (!valid_col(c, targets[k]) || c->cols[targets[k]].dim != 1)
            return fail(WSMC_EARG, "move targets must be existing scalar columns");
    if (!std::isnan(diversity)) {
        double div = 0;
        int r = wsmc_marginal_diversity(c, targets, d, &div);
        if (r) return r;
        if (div >= diversity) return WSMC_OK;
    }
    if (target_depth < 0) target_depth = c->depth;
    // a gated Move (wsmc_move_gated) decided on the device; a diversity gate or shards read
    // the decision on the host first (the Move then runs or not as an ordinary one)
    const Decision* gate = c->move_gate;
    c->move_gate = nullptr;
    if (gate && (is_sharded(c) || proposal != WSMC_PROPOSAL_AUTORW && proposal != WSMC_PROPOSAL_RW)) gate = nullptr;
    double l[4], h[4];
    bool bounded = false;
    for (int k = 0; k < d; ++k) {
        l[k] = lo ? lo[k] : -INFINITY;
        h[k] = hi ? hi[k] : INFINITY;
        if (std::isfinite(l[k]) || std::isfinite(h[k])) bounded = true;
    }
    if (!lo && !hi) bounded = false;
    // the move reads its targets and every column of the score tape, and rewrites the targets
    std::vector<int32_t> reads(targets, targets + d);
    for (const auto& t : c->tape) cols_of(t, reads);
    int r = need_cols(c, reads);
    if (!r) r = upload_colptr(c);   // the generic fold's tape is uploaded below, only when used
    if (r) return r;
    // asynchronous (no count requested): no host wait; a pending failure flag stays set (the
    // kernels skip on it) until the next synchronizing call reports it
    const bool async = !accepted_out;   // sharded too: the factor and its PD flag are device-side
    if (!async && (r = check_deferred(c))) return r;
    // the flag words and accepted counters: zeroed by the moments kernel on the one-context
    // autoRW path (block 0, before anything reads them), else by memsets
    int32_t* zflag = (!c->move_pending && !c->dflag_zero) ? c->dflag : nullptr;
    c->dflag_zero = true;
    unsigned long long* zcount = accepted_out ? c->ucount : nullptr;
    if (proposal != WSMC_PROPOSAL_AUTORW || is_sharded(c)) {
        if (zflag) WSMC_HIP(hipMemsetAsync(zflag, 0, sizeof(int32_t) * 4, c->stream));
        if (zcount) WSMC_HIP(hipMemsetAsync(zcount, 0, sizeof(unsigned long long) * 4 * kAccMove, c->stream));
    }
    if (proposal == WSMC_PROPOSAL_AUTORW && is_sharded(c)) {
        if (c->w_reset_pending) {   // the sharded max pass reads the weights
            WSMC_HIP(launch_fill_weights(c->stream, c->w, c->w_reset_pending, c->N));
            c->w_reset_pending = nullptr;
        }
        c->dflag_zero = false;
        int rr = sharded_autorw(c, targets, d, bounded ? l : nullptr, bounded ? h : nullptr, step);
        if (rr) return rr;
    } else if (proposal == WSMC_PROPOSAL_AUTORW) {
        // the max of the weights: kept by the last Observe / fused Resample when still
        // current (Moves leave the weights alone), else a max pass
        const bool kept = c->cur_max && c->cur_max_seq == c->wseq;
        MaxSlots* mms = kept ? c->cur_max : c->mslots;
        if (!kept) {
            if (c->w_reset_pending) {   // the max pass reads the weights themselves
                WSMC_HIP(launch_fill_weights(c->stream, c->w, c->w_reset_pending, c->N));
                c->w_reset_pending = nullptr;
            }
            WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
            WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
        }
        const double* lp = bounded ? l : nullptr;
        const double* hp = bounded ? h : nullptr;
        // one pass relative to the pivot (particle 0), then the one-block combine and factor
        // (a last-block combine inside the moments kernel, an arrival counter behind a
        // device-scope fence per block, measured 2x slower than the separate combine launch:
        // 113.6 vs 57.7 + 13.5 us at 4M — every block's fence writes back its L2)
        WSMC_HIP(launch_autorw_moments(c->stream, c->w, mms, c->d_colptr, targets, d, lp, hp, nullptr, c->N,
                                       c->tilepart, c->w_reset_pending, gate, nullptr, nullptr, 0, zflag, zcount));
        WSMC_HIP(launch_autorw_final(c->stream, c->tilepart, c->ntiles, d, step, c->mom, c->dflag, 0, gate));
        c->dflag_zero = false;
    } else {
        WSMC_HIP(ctx_sync(c, c->stream));
        double* L = reinterpret_cast<double*>(c->pinned);
        for (int k = 0; k < 16; ++k) L[k] = 0.0;
        for (int k = 0; k < d; ++k) L[k * d + k] = step;
        WSMC_HIP(hipMemcpyAsync(c->mom + 32, L, sizeof(double) * 16, hipMemcpyHostToDevice, c->stream));
    }
    // carried scores: the fold prefix of this move is the terms before the first one at or
    // beyond target_depth; continue the cache if it covers a prefix of it
    int32_t kD = 0;
    while (kD < (int32_t)c->tape.size() && c->tape[kD].depth < target_depth) ++kD;
    if (!c->scache) {
        WSMC_HIP(hipMalloc(&c->scache, sizeof(double) * c->N));
        WSMC_HIP(hipMalloc(&c->scache_back, sizeof(double) * c->N));
    }
    const int32_t cache_from = (c->scache_terms >= 0 && c->scache_terms <= kD) ? c->scache_terms : -1;
    // compile the fold's tape prefix: every (column, component) it reads becomes a slot
    // (targets first); > kFoldSlots distinct reads keep the generic interpreter
    std::vector<std::pair<int32_t, int32_t>> slots;
    auto slot_of = [&](int32_t col, int32_t comp) -> int32_t {
        for (size_t s = 0; s < slots.size(); ++s)
            if (slots[s].first == col && slots[s].second == comp) return (int32_t)s;
        slots.emplace_back(col, comp);
        return (int32_t)slots.size() - 1;
    };
    for (int k = 0; k < d; ++k) slot_of(targets[k], 0);
    std::vector<wsmc_term> ct(c->tape.begin(), c->tape.begin() + kD);
    auto remap = [&](wsmc_operand& o) {
        for (int k = 0; k < 2; ++k)
            if (o.col[k] >= 0) {
                o.col[k] = slot_of(o.col[k], o.comp[k]);
                o.comp[k] = 0;
            }
    };
    for (auto& t : ct) {
        for (int k = 0; k < 4; ++k) { remap(t.x[k]); remap(t.dist.mu[k]); }
        remap(t.dist.scale);
    }
    const int32_t* mflag = proposal == WSMC_PROPOSAL_AUTORW ? c->dflag : nullptr;
    if ((int)slots.size() <= kFoldSlots) {
        // the fold program: s_new over [0, kD), s_old over [cache_from or 0, kD)
        std::vector<FoldSeg> segs;
        std::vector<double> cst;
        const int32_t nseg_new = compile_fold(ct, 0, kD, segs, cst);
        const int32_t seg_old0 = (int32_t)segs.size();
        const int32_t nseg_old = compile_fold(ct, cache_from >= 0 ? cache_from : 0, kD, segs, cst);
        // the templates the segments read, compacted (the fold reads no other term)
        std::vector<int32_t> tmap(ct.size(), -1);
        std::vector<wsmc_term> tmpls;
        for (auto& sg : segs) {
            if (tmap[sg.tmpl] < 0) {
                tmap[sg.tmpl] = (int32_t)tmpls.size();
                tmpls.push_back(ct[sg.tmpl]);
            }
            sg.tmpl = tmap[sg.tmpl];
        }
        // [templates | segments | constants]: in the kernel's arguments when it fits (no
        // copy), else one upload through the pinned staging ring
        const size_t ct_bytes = sizeof(wsmc_term) * tmpls.size();
        const size_t seg_bytes = sizeof(FoldSeg) * segs.size();
        const size_t prog_bytes = ct_bytes + seg_bytes + sizeof(double) * cst.size();
        static_assert(sizeof(wsmc_term) % 8 == 0 && sizeof(FoldSeg) % 8 == 0, "program alignment");
        static const bool no_inline = [] {   // diagnostics only: always upload the program
            const char* e = diag_env("WSMC_DIAG_PROG_COPY");
            return e && atoi(e) != 0;
        }();
        // lean fold: every one-term segment scalar (runs are evaluated by their own code)
        bool lean = true;
        for (const auto& sg : segs)
            if (sg.kind == kSegTerm && !wsmc_term_is_scalar(&tmpls[sg.tmpl])) lean = false;
        const bool inl = !no_inline && lean && prog_bytes <= sizeof(ProgInline::w);
        ProgInline pin;
        char* hp = nullptr;
        int64_t need = 0;
        if (inl) {
            hp = reinterpret_cast<char*>(pin.w);
            pin.seg_off = (int32_t)ct_bytes;
            pin.cst_off = (int32_t)(ct_bytes + seg_bytes);
            pin.seg_old0 = seg_old0;
            pin.pad = 0;
        } else {
            need = ((int64_t)prog_bytes + 255) & ~(int64_t)255;
            if (c->prog_stage_at + need > c->prog_stage_cap) {   // wrap: the ring's copies are done
                WSMC_HIP(ctx_sync(c, c->stream));
                c->prog_stage_at = 0;
                if (need > c->prog_stage_cap) {
                    if (c->prog_stage) WSMC_HIP(hipHostFree(c->prog_stage));
                    c->prog_stage = nullptr;
                    int64_t cap = std::max<int64_t>(262144, need);
                    WSMC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->prog_stage), cap, hipHostMallocDefault));
                    c->prog_stage_cap = cap;
                }
            }
            hp = c->prog_stage + c->prog_stage_at;
            c->prog_stage_at += need;
        }
        if (!tmpls.empty()) std::memcpy(hp, tmpls.data(), ct_bytes);
        if (seg_bytes) std::memcpy(hp + ct_bytes, segs.data(), seg_bytes);
        if (!cst.empty()) std::memcpy(hp + ct_bytes + seg_bytes, cst.data(), sizeof(double) * cst.size());
        char* pbase = nullptr;
        if (!inl && prog_bytes && (r = prog_device(c, hp, prog_bytes, need, &pbase))) return r;
        const wsmc_term* d_ct = reinterpret_cast<const wsmc_term*>(pbase);
        FoldProgram prog;
        prog.seg_new = reinterpret_cast<const FoldSeg*>(pbase + ct_bytes);
        prog.seg_old = prog.seg_new + seg_old0;
        prog.nseg_new = nseg_new;
        prog.nseg_old = nseg_old;
        prog.cst = reinterpret_cast<const double*>(pbase + ct_bytes + seg_bytes);
        FoldSlots fs{};
        fs.n = (int32_t)slots.size();
        for (const auto& t : ct) fs.heavy |= t.dist.mean_fn == WSMC_MEAN_OSCILLATOR ? 1 : 0;
        fs.lean = lean ? 1 : 0;
        for (size_t s = 0; s < slots.size(); ++s)
            fs.p[s] = c->cols[slots[s].first].front + (int64_t)slots[s].second * c->N;
        for (int k = 0; k < d; ++k) fs.t[k] = c->cols[targets[k]].front;
        // carried scores one lazy Resample behind: read through its ancestors, written to the
        // other buffer (no gather launch at the Resample)
        MoveCarry mc;
        mc.in = c->scache;
        mc.out = c->scache;
        mc.gate = gate;
        if (c->scache_anc && cache_from >= 0) {
            mc.anc = c->scache_anc;
            mc.dec = c->scache_dec;
            mc.out = c->scache_back;
        }
        WSMC_HIP(launch_move_c(c->stream, d_ct, kD, target_depth, fs, targets, d, bounded ? l : nullptr,
                               bounded ? h : nullptr, bounded ? 1 : 0, c->mom + 32, c->seed, op_prop, op_acc, c->goff,
                               c->N, c->ucount, mflag, mc, cache_from, prog, inl ? &pin : nullptr));
        if (mc.out != mc.in) std::swap(c->scache, c->scache_back);
        c->scache_anc = nullptr;   // written in slot order now (or refolded from scratch)
        c->scache_dec = nullptr;
        c->scache_lag_epoch = -1;
    } else {
        if (gate) {   // the generic kernel has no gate: decide on the host
            if ((r = resolve_decisions(c))) return r;
            if (!c->resampled) return WSMC_OK;   // skipped (its op counters are consumed)
        }
        if ((r = resolve_scache_lag(c))) return r;   // the generic kernel reads its scores in place
        if ((r = upload_tape(c))) return r;
        WSMC_HIP(launch_move(c->stream, c->d_tape, (int32_t)c->tape.size(), target_depth, c->d_colptr, targets, d,
                             bounded ? l : nullptr, bounded ? h : nullptr, bounded ? 1 : 0, c->mom + 32, c->seed,
                             op_prop, op_acc, c->goff, c->N, c->ucount, mflag, c->scache, cache_from));
    }
    if (async) {
        c->scache_terms = kD;
        c->move_pending = true;
        return WSMC_OK;
    }
    struct {
        int32_t flag[4];
        unsigned long long acc[4];
    }* hb = reinterpret_cast<decltype(hb)>(c->pinned);
    // the counts and flags into the pinned words by the summing kernel itself
    auto* hbd = reinterpret_cast<decltype(hb)>(c->pinned_dev);
    WSMC_HIP(launch_acc_sum(c->stream, c->ucount, hbd->acc, c->dflag, hbd->flag));
    WSMC_HIP(ctx_sync(c, c->stream));
    if (hb->flag[0]) return fail(WSMC_ENOTPD, "autoRW proposal covariance is not positive definite");
    c->dflag_zero = true;
    c->scache_terms = kD;
    if (accepted_out) *accepted_out = (int64_t)hb->acc[0];
    return WSMC_OK;
}

int wsmc_move_gated(wsmc_ctx* c, int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
                    const double* hi, int32_t target_depth, double diversity) {
    if (c && c->multi)
        return multi_each(c, [&](wsmc_ctx* x) {
            return wsmc_move_gated(x, proposal, targets, d, step, lo, hi, target_depth, diversity);
        });
    CHECK_CTX_KEEP(c);
    // the deciding Resample: the newest one still pending on the device, else the host flag
    const Decision* gate = c->dec_pending > 0 && !c->dec_rows.empty() ? c->dec_rows.back().row.dec : nullptr;
    if (gate && (is_sharded(c) || !std::isnan(diversity))) {
        if (int r = resolve_decisions(c)) return r;
        gate = nullptr;
    }
    if (!gate) {
        if (!c->resampled) {   // does not run: its two op counters are consumed all the same
            c->op += 2;
            return WSMC_OK;
        }
        return wsmc_move(c, proposal, targets, d, step, lo, hi, target_depth, diversity, nullptr);
    }
    wsmc_move_spec sp1;
    if (!no_block1() && move_spec_of(proposal, targets, d, step, lo, hi, target_depth, sp1)) {
        bool done = false;
        const int r = move_block_fused(c, 1, &sp1, 1, nullptr, &done);
        if (done) return r;
    }
    c->move_gate = gate;
    const int r = wsmc_move(c, proposal, targets, d, step, lo, hi, target_depth, diversity, nullptr);
    c->move_gate = nullptr;
    return r;
}

// ---- a block of Moves (wsmc_move_block) -----------------------------------------------------
// The moves one by one (the definition the fused path reproduces bit for bit)
static int move_block_each(wsmc_ctx* c, int32_t n, const wsmc_move_spec* specs, int32_t gated, int64_t* accepted_out) {
    for (int32_t m = 0; m < n; ++m) {
        const wsmc_move_spec& sp = specs[m];
        const double* lo = sp.bounded ? sp.lo : nullptr;
        const double* hi = sp.bounded ? sp.hi : nullptr;
        int r;
        if (gated && !accepted_out) {
            r = wsmc_move_gated(c, sp.proposal, sp.targets, sp.d, sp.step, lo, hi, sp.target_depth, WSMC_NAN);
        } else if (gated) {   // counts requested: the host reads the condition
            if (c->multi) {
                r = wsmc_move_gated(c, sp.proposal, sp.targets, sp.d, sp.step, lo, hi, sp.target_depth, WSMC_NAN);
                accepted_out[m] = 0;
            } else {
                if ((r = resolve_decisions(c))) return r;
                if (!c->resampled) {
                    c->op += 2;
                    accepted_out[m] = 0;
                    continue;
                }
                r = wsmc_move(c, sp.proposal, sp.targets, sp.d, sp.step, lo, hi, sp.target_depth, WSMC_NAN,
                              &accepted_out[m]);
            }
        } else {
            r = wsmc_move(c, sp.proposal, sp.targets, sp.d, sp.step, lo, hi, sp.target_depth, WSMC_NAN,
                          accepted_out ? &accepted_out[m] : nullptr);
        }
        if (r) return r;
    }
    return WSMC_OK;
}

// oscillator (heavy) blocks compiled one particle a thread. Round 4 measured two a thread
// faster (the run loop's per-term control shared: 0.242 -> 0.235 s); with the loop reduced to a
// rotation and a score per term and the log / exp tables in LDS, the halved registers win:
// C5 151.7 -> 143.9 ms asynchronous on one box (round 5, tools/ab_env.sh). WSMC_DIAG_MV_K1=0
// compiles two a thread, for comparison
static bool mv_heavy_k1() {
    static const bool v = [] {
        const char* e = diag_env("WSMC_DIAG_MV_K1");
        return !(e && *e && atoi(e) == 0);
    }();
    return v;
}
// WSMC_DIAG_MV_K=1|2|4: particles a thread of the compiled lean (non-oscillator) blocks (2)
static int mv_lean_k() {
    static const int v = [] {
        const char* e = diag_env("WSMC_DIAG_MV_K");
        const int k = e ? atoi(e) : 2;
        return (k == 1 || k == 4) ? k : 2;
    }();
    return v;
}
// a Move block's shape for csrc/wsmc_mv_body.h (false: outside what it compiles — the
// interpreter kernels run the block): its moves, which targets are bounded or read through the
// lag row, and the lean fold program's segments with the slots each template operand reads
static bool mv_signature(const FoldSlots& fs, const MoveBlk& mb, int D, int lag_slots, int lag_targets,
                         int32_t cache_from, const std::vector<wsmc_term>& tmpls, const std::vector<FoldSeg>& segs,
                         int32_t nseg_new, int32_t nseg_old, MvSig& g) {
    std::memset(&g, 0, sizeof(g));
    if (fs.n < 1 || fs.n > kFoldSlots || D < 1 || D > kBlkTargets || mb.nm < 1 || mb.nm > 4) return false;
    if (nseg_new > kMvSegs || nseg_old > kMvSegs || tmpls.size() > 64) return false;
    g.K = (fs.heavy && mv_heavy_k1()) ? 1 : (fs.heavy ? 2 : mv_lean_k());
    g.nm = (int8_t)mb.nm;
    g.D = (int8_t)D;
    g.ns = (int8_t)fs.n;
    g.ntmpl = (int8_t)tmpls.size();
    g.nnew = (int8_t)nseg_new;
    g.nold = (int8_t)nseg_old;
    g.carry = cache_from >= 0 ? 1 : 0;
    for (int k = 0; k <= mb.nm; ++k) g.off[k] = mb.off[k];
    for (int k = mb.nm + 1; k < 5; ++k) g.off[k] = mb.off[mb.nm];
    g.bnd = (uint8_t)(mb.bnd & 0xff);
    for (int u = 0; u < D; ++u) {
        if (!((mb.bnd >> u) & 1)) continue;
        if (std::isfinite(mb.lo[u])) g.flo |= (uint8_t)(1 << u);
        if (std::isfinite(mb.hi[u])) g.fhi |= (uint8_t)(1 << u);
    }
    g.lagt = (uint8_t)(lag_targets & 0xff);
    g.smask = (uint16_t)(lag_slots & 0xffff);
    auto shape = [](const wsmc_operand& o, MvSigOp& q) {
        for (int k = 0; k < 2; ++k) q.c[k] = (int8_t)(o.col[k] >= 0 ? o.col[k] : -1);
    };
    for (int32_t i = 0; i < nseg_new + nseg_old; ++i) {
        const FoldSeg& sg = segs[i];
        MvSigSeg& q = g.seg[i < nseg_new ? i : kMvSegs + (i - nseg_new)];
        const wsmc_term& t = tmpls[sg.tmpl];
        q.kind = (int8_t)sg.kind;
        q.fam = (int8_t)t.dist.family;
        q.pre = sg.soff >= 0 ? 1 : 0;
        shape(t.x[0], q.x);
        for (int k = 0; k < 4; ++k) shape(t.dist.mu[k], q.mu[k]);
        shape(t.dist.scale, q.sc);
        if (sg.kind == kSegTerm) {
            if (!wsmc_term_is_scalar(&t)) return false;
        } else if (sg.kind == kSegNormalOsc) {
            if (!fs.heavy) return false;
        } else if (sg.kind != kSegNormalAff) {
            return false;
        }
    }
    for (int i = nseg_new; i < kMvSegs; ++i) g.seg[i].kind = 0;
    return true;
}

int wsmc_move_block(wsmc_ctx* c, int32_t n, const wsmc_move_spec* specs, int32_t gated, int64_t* accepted_out) {
    if (!c) return fail(WSMC_EARG, "null context");
    if (n < 0 || (n > 0 && !specs)) return fail(WSMC_EARG, "move block needs n >= 0 specs");
    if (accepted_out)
        for (int32_t m = 0; m < n; ++m) accepted_out[m] = 0;
    if (n == 0) return WSMC_OK;
    if (c->multi) return move_block_each(c, n, specs, gated, accepted_out);
    CHECK_CTX_KEEP(c);
    bool done = false;
    const int r = move_block_fused(c, n, specs, gated, accepted_out, &done);
    return done ? r : move_block_each(c, n, specs, gated, accepted_out);
}

// The fused path of a block (also a single autoRW Move's, wsmc_move / wsmc_move_gated): *done
// false when the block is outside it — nothing has been changed then, and the caller runs the
// moves one by one
static int move_block_fused(wsmc_ctx* c, int32_t n, const wsmc_move_spec* specs, int32_t gated,
                            int64_t* accepted_out, bool* done) {
    *done = false;
    // the fused path: autoRW Moves on disjoint scalar targets (8 in all), one target depth, one
    // GPU, a lean fold program
    int32_t depth = specs[0].target_depth < 0 ? c->depth : specs[0].target_depth;
    bool fuse = !is_sharded(c) && n <= 4 && !c->move_gate;
    int32_t D = 0;
    int32_t utg[kBlkTargets] = {};
    MoveBlk mb{};
    mb.nm = n;
    for (int32_t m = 0; m < n && fuse; ++m) {
        const wsmc_move_spec& sp = specs[m];
        const int32_t dm = sp.target_depth < 0 ? c->depth : sp.target_depth;
        if (sp.proposal != WSMC_PROPOSAL_AUTORW || sp.d < 1 || sp.d > 4 || D + sp.d > kBlkTargets || dm != depth) {
            fuse = false;
            break;
        }
        mb.off[m] = (int8_t)D;
        bool bounded = false;
        for (int k = 0; k < sp.d; ++k) {
            const int32_t t = sp.targets[k];
            if (!valid_col(c, t) || c->cols[t].dim != 1) return fail(WSMC_EARG, "move targets must be existing scalar columns");
            for (int u = 0; u < D; ++u)
                if (utg[u] == t) fuse = false;   // overlapping targets: the moves one by one
            for (int j = 0; j < k; ++j)
                if (sp.targets[j] == t) fuse = false;
            if (sp.bounded && (std::isfinite(sp.lo[k]) || std::isfinite(sp.hi[k]))) bounded = true;
        }
        for (int k = 0; k < sp.d; ++k) {
            const int u = D + k;
            utg[u] = sp.targets[k];
            mb.lo[u] = bounded ? sp.lo[k] : -INFINITY;
            mb.hi[u] = bounded ? sp.hi[k] : INFINITY;
            mb.lgw[u] = (std::isfinite(mb.lo[u]) && std::isfinite(mb.hi[u])) ? wsmc_log(mb.hi[u] - mb.lo[u]) : 0.0;
            if (bounded) mb.bnd |= 1 << u;
            mb.tcol[u] = (int16_t)utg[u];
        }
        mb.min_step[m] = sp.step;
        D += sp.d;
    }
    if (!fuse) return WSMC_OK;
    mb.off[n] = (int8_t)D;
    // the fold program over the union's slots (targets first), compiled before anything runs
    int32_t kD = 0;
    while (kD < (int32_t)c->tape.size() && c->tape[kD].depth < depth) ++kD;
    const int32_t cache_from = (c->scache && c->scache_terms >= 0 && c->scache_terms <= kD) ? c->scache_terms : -1;
    std::vector<std::pair<int32_t, int32_t>> slots;
    auto slot_of = [&](int32_t col, int32_t comp) -> int32_t {
        for (size_t q = 0; q < slots.size(); ++q)
            if (slots[q].first == col && slots[q].second == comp) return (int32_t)q;
        slots.emplace_back(col, comp);
        return (int32_t)slots.size() - 1;
    };
    for (int u = 0; u < D; ++u) slot_of(utg[u], 0);
    std::vector<wsmc_term> ct(c->tape.begin(), c->tape.begin() + kD);
    auto remap = [&](wsmc_operand& o) {
        for (int k = 0; k < 2; ++k)
            if (o.col[k] >= 0) {
                o.col[k] = slot_of(o.col[k], o.comp[k]);
                o.comp[k] = 0;
            }
    };
    for (auto& t : ct) {
        for (int k = 0; k < 4; ++k) { remap(t.x[k]); remap(t.dist.mu[k]); }
        remap(t.dist.scale);
    }
    std::vector<FoldSeg> segs;
    std::vector<double> cst;
    const int32_t nseg_new = compile_fold(ct, 0, kD, segs, cst);
    const int32_t seg_old0 = (int32_t)segs.size();
    const int32_t nseg_old = compile_fold(ct, cache_from >= 0 ? cache_from : 0, kD, segs, cst);
    std::vector<int32_t> tmap(ct.size(), -1);
    std::vector<wsmc_term> tmpls;
    for (auto& sg : segs) {
        if (tmap[sg.tmpl] < 0) {
            tmap[sg.tmpl] = (int32_t)tmpls.size();
            tmpls.push_back(ct[sg.tmpl]);
        }
        sg.tmpl = tmap[sg.tmpl];
    }
    bool lean = (int)slots.size() <= kFoldSlots;
    for (const auto& sg : segs)
        if (sg.kind == kSegTerm && !wsmc_term_is_scalar(&tmpls[sg.tmpl])) lean = false;
    if (!lean) return WSMC_OK;
    *done = true;
    const size_t ct_bytes = sizeof(wsmc_term) * tmpls.size();
    const size_t seg_bytes = sizeof(FoldSeg) * segs.size();
    const size_t prog_bytes = ct_bytes + seg_bytes + sizeof(double) * cst.size();

    // the condition: the newest Resample still pending on the device, else the host flag
    const Decision* gate = nullptr;
    if (gated) {
        gate = c->dec_pending > 0 && !c->dec_rows.empty() ? c->dec_rows.back().row.dec : nullptr;
        if (!gate && !c->resampled) {   // does not run: the op counters are consumed all the same
            c->op += 2 * (uint64_t)n;
            return WSMC_OK;
        }
    }
    for (int32_t m = 0; m < n; ++m) {
        mb.op_prop[m] = c->op++;
        mb.op_acc[m] = c->op++;
    }
    // columns: current, one lazy Resample behind (read through its row by the kernels, no
    // trace), or further behind (brought up to date first)
    std::vector<int32_t> reads;
    for (const auto& sl : slots) reads.push_back(sl.first);
    const bool has_lag_row = c->lazy && !c->alog.empty() && c->epoch - 1 >= c->log_base;
    const AncRow* lrow = has_lag_row ? &c->alog.back() : nullptr;
    std::vector<int32_t> far;
    for (int32_t id : reads) {
        c->cols[id].touch = c->epoch;
        const int64_t e = c->cols[id].epoch;
        if (e < c->epoch && !(lrow && e == c->epoch - 1)) far.push_back(id);
    }
    int r;
    if (!far.empty() && (r = materialize(c, &far))) return r;
    int lag_slots = 0, lag_targets = 0;
    for (size_t q = 0; q < slots.size(); ++q)
        if (c->cols[slots[q].first].epoch == c->epoch - 1 && lrow) lag_slots |= 1 << q;
    lag_targets = lag_slots & ((1 << D) - 1);
    if ((r = upload_colptr(c))) return r;
    const bool async = !accepted_out;
    if (!async && (r = check_deferred(c))) return r;
    // the flag words and accepted counters are zeroed by the first moments launch (block 0)
    int32_t* zflag = (!c->move_pending && !c->dflag_zero) ? c->dflag : nullptr;
    unsigned long long* zcount = accepted_out ? c->ucount : nullptr;
    // the moments: one pass over the union of the targets (4 at most), else one pass per move;
    // one combine into every move's factor
    const bool kept = c->cur_max && c->cur_max_seq == c->wseq;
    MaxSlots* mms = kept ? c->cur_max : c->mslots;
    if (!kept) {
        if (c->w_reset_pending) {
            WSMC_HIP(launch_fill_weights(c->stream, c->w, c->w_reset_pending, c->N));
            c->w_reset_pending = nullptr;
        }
        WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
        WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    }
    const int sep = D > 4;
    int32_t toff[4] = {0, 0, 0, 0};
    const int32_t* lanc = lrow ? lrow->anc : nullptr;
    const Decision* ldec = lrow ? lrow->dec : nullptr;
    if (!sep) {
        WSMC_HIP(launch_autorw_moments(c->stream, c->w, mms, c->d_colptr, utg, D, mb.lo, mb.hi, nullptr, c->N,
                                       c->tilepart, c->w_reset_pending, gate, lanc, ldec, lag_targets, zflag, zcount));
    } else {
        int32_t at = 0;
        for (int32_t m = 0; m < n; ++m) {
            const int o = mb.off[m], dm = mb.off[m + 1] - o;
            toff[m] = at;
            WSMC_HIP(launch_autorw_moments(c->stream, c->w, mms, c->d_colptr, utg + o, dm, mb.lo + o, mb.hi + o,
                                           nullptr, c->N, c->tilepart + (int64_t)at * c->ntiles, c->w_reset_pending,
                                           gate, lanc, ldec, (lag_targets >> o) & ((1 << dm) - 1), m == 0 ? zflag : nullptr,
                                           m == 0 ? zcount : nullptr));
            at += 1 + dm + dm * (dm + 1) / 2;
        }
    }
    WSMC_HIP(launch_autorw_final_blk(c->stream, c->tilepart, c->ntiles, mb, sep, toff, c->mom, c->dflag, gate));
    c->dflag_zero = false;
    if (!c->scache) {
        WSMC_HIP(hipMalloc(&c->scache, sizeof(double) * c->N));
        WSMC_HIP(hipMalloc(&c->scache_back, sizeof(double) * c->N));
    }
    // the program: in the kernel's arguments when it fits, else uploaded through the ring
    ProgInlineBlk pin;
    const bool inl = prog_bytes <= sizeof(ProgInlineBlk::w);
    char* hp;
    int64_t need = 0;
    if (inl) {
        hp = reinterpret_cast<char*>(pin.w);
        pin.seg_off = (int32_t)ct_bytes;
        pin.cst_off = (int32_t)(ct_bytes + seg_bytes);
        pin.seg_old0 = seg_old0;
        pin.pad = 0;
    } else {
        need = ((int64_t)prog_bytes + 255) & ~(int64_t)255;
        if (c->prog_stage_at + need > c->prog_stage_cap) {
            WSMC_HIP(ctx_sync(c, c->stream));
            c->prog_stage_at = 0;
            if (need > c->prog_stage_cap) {
                if (c->prog_stage) WSMC_HIP(hipHostFree(c->prog_stage));
                c->prog_stage = nullptr;
                const int64_t cap = std::max<int64_t>(262144, need);
                WSMC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->prog_stage), cap, hipHostMallocDefault));
                c->prog_stage_cap = cap;
            }
        }
        hp = c->prog_stage + c->prog_stage_at;
        c->prog_stage_at += need;
    }
    if (!tmpls.empty()) std::memcpy(hp, tmpls.data(), ct_bytes);
    if (seg_bytes) std::memcpy(hp + ct_bytes, segs.data(), seg_bytes);
    if (!cst.empty()) std::memcpy(hp + ct_bytes + seg_bytes, cst.data(), sizeof(double) * cst.size());
    char* pbase = nullptr;
    if (!inl && (r = prog_device(c, hp, prog_bytes, need, &pbase))) return r;
    FoldProgram prog;
    prog.seg_new = inl ? nullptr : reinterpret_cast<const FoldSeg*>(pbase + ct_bytes);
    prog.seg_old = inl ? nullptr : prog.seg_new + seg_old0;
    prog.nseg_new = nseg_new;
    prog.nseg_old = nseg_old;
    prog.cst = inl ? nullptr : reinterpret_cast<const double*>(pbase + ct_bytes + seg_bytes);
    FoldSlots fs{};
    fs.n = (int32_t)slots.size();
    for (const auto& t : tmpls) fs.heavy |= t.dist.mean_fn == WSMC_MEAN_OSCILLATOR ? 1 : 0;
    fs.lean = 1;
    for (size_t q = 0; q < slots.size(); ++q)
        fs.p[q] = c->cols[slots[q].first].front + (int64_t)slots[q].second * c->N;
    for (int u = 0; u < D; ++u) {
        Column& col = c->cols[utg[u]];
        mb.tout[u] = ((lag_targets >> u) & 1) ? col.back : col.front;
    }
    mb.lag_targets = lag_targets;
    MoveCarry mc;
    mc.in = c->scache;
    mc.out = c->scache;
    mc.gate = gate;
    if (c->scache_anc && cache_from >= 0) {
        mc.anc = c->scache_anc;
        mc.dec = c->scache_dec;
        mc.out = c->scache_back;
    }
    // the block on its shape's compiled kernel (csrc/wsmc_mv_body.h), else the interpreter
    MvSig sig;
    hipError_t je = hipErrorNotSupported;
    if (mv_signature(fs, mb, D, lag_slots, lag_targets, cache_from, tmpls, segs, nseg_new, nseg_old, sig)) {
        MvArgs ma;
        ma.fs = fs;
        ma.mb = mb;
        ma.Lb = c->mom + 64;
        ma.seed = c->seed;
        ma.goff = c->goff;
        ma.N = c->N;
        ma.accepted = accepted_out ? c->ucount : nullptr;
        ma.flag = c->dflag;
        ma.mc = mc;
        ma.lg = MomLag{lag_slots ? lanc : nullptr, ldec, lag_slots};
        ma.tab = c->d_colptr;
        ma.prog = inl ? nullptr : pbase;
        je = launch_mv_jit(c->stream, sig, inl ? &pin : nullptr, ma, c->device);
        if (je != hipSuccess && je != hipErrorNotSupported) WSMC_HIP(je);
    }
    if (je == hipErrorNotSupported)
        WSMC_HIP(launch_move_blk(c->stream, inl ? &pin : nullptr, reinterpret_cast<const wsmc_term*>(pbase), prog, fs,
                                 mb, c->mom + 64, c->seed, c->goff, c->N, accepted_out ? c->ucount : nullptr, c->dflag,
                                 mc, cache_from, lanc, ldec, lag_slots, c->d_colptr));
    if (mc.out != mc.in) std::swap(c->scache, c->scache_back);
    c->scache_anc = nullptr;
    c->scache_dec = nullptr;
    c->scache_lag_epoch = -1;
    c->scache_terms = kD;
    for (int u = 0; u < D; ++u) {   // the moved targets are current (the lagged ones in their back buffers)
        Column& col = c->cols[utg[u]];
        if ((lag_targets >> u) & 1) std::swap(col.front, col.back);
        wrote_col(c, utg[u]);
    }
    gc_log(c);
    if (async) {
        c->move_pending = true;
        return WSMC_OK;
    }
    struct {
        int32_t flag[4];
        unsigned long long acc[4];
    }* hb = reinterpret_cast<decltype(hb)>(c->pinned);
    // the counts and flags into the pinned words by the summing kernel itself
    auto* hbd = reinterpret_cast<decltype(hb)>(c->pinned_dev);
    WSMC_HIP(launch_acc_sum(c->stream, c->ucount, hbd->acc, c->dflag, hbd->flag));
    WSMC_HIP(ctx_sync(c, c->stream));
    for (int32_t m = 0; m < n; ++m) accepted_out[m] = (int64_t)hb->acc[m];
    if (hb->flag[0]) return fail(WSMC_ENOTPD, "autoRW proposal covariance is not positive definite");
    c->dflag_zero = true;   // (flag[2] is rewritten by every block's combine before it is read)
    return WSMC_OK;
}

// ---- fused 2D SSM runner --------------------------------------------------------------
// ancestor-log rows are padded to 16 B so every row start is aligned for paired loads
static inline int64_t anc_stride(int64_t N) { return (N + 3) & ~(int64_t)3; }
// per-step group sums of the fused single-GPU resample
static inline int64_t run_grp_words(int64_t N) {
    const int64_t nt = (N + kRsTile - 1) / kRsTile, G = group_tiles(N);
    return ((nt + G - 1) / G) * kGroupLine;
}
static inline size_t run_grp_bytes(int64_t N, int32_t T) {
    return sizeof(unsigned long long) * (size_t)run_grp_words(N) * (size_t)(T + 1);
}

static int ensure_run_buffers(wsmc_ctx* c, int32_t T) {
    if (c->T_alloc >= T && c->run_rec) return WSMC_OK;
    if (int r = resolve_run(c)) return r;   // (a pending run reads these buffers)
    WSMC_HIP(ctx_sync(c, c->stream));
    void* old[] = {c->run_max, c->run_rec, c->run_dec, c->anc_log, c->obs_buf, c->run_grp, c->run_rg};
    for (void* p : old)
        if (p) WSMC_HIP(hipFree(p));
    if (c->run_hdec) WSMC_HIP(hipHostFree(c->run_hdec));
    if (c->run_hstage) WSMC_HIP(hipHostFree(c->run_hstage));
    WSMC_HIP(hipMalloc(&c->run_max, sizeof(MaxSlots) * (T + 1)));
    WSMC_HIP(hipMalloc(&c->run_rg, sizeof(double) * (T + 1)));
    if (!c->run_w0) WSMC_HIP(hipMalloc(&c->run_w0, sizeof(double) * 2 * c->N));
    // coherent: written by the trace-back kernel / read by the head kernel in place
    WSMC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->run_hdec), sizeof(Decision) * 2 * (T + 1), hipHostMallocCoherent));
    WSMC_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->run_hstage), sizeof(double) * 2 * (2 * (size_t)T + 4),
                           hipHostMallocCoherent));
    for (int k = 0; k < 2; ++k)
        if (!c->run_ev[k]) WSMC_HIP(hipEventCreateWithFlags(&c->run_ev[k], hipEventDisableTiming));
    if (!c->run_nfix) {
        WSMC_HIP(hipMalloc(&c->run_nfix, sizeof(unsigned long long)));
        WSMC_HIP(hipMemsetAsync(c->run_nfix, 0, sizeof(unsigned long long), c->stream));
    }
    WSMC_HIP(hipMalloc(&c->run_rec, sizeof(ShardRecord) * (T + 1) * kMaxWorld));
    WSMC_HIP(hipMalloc(&c->run_dec, sizeof(Decision) * (T + 1)));
    WSMC_HIP(hipMalloc(&c->anc_log, sizeof(int32_t) * (size_t)T * anc_stride(c->N)));
    WSMC_HIP(hipMalloc(&c->obs_buf, sizeof(double) * 4 * (T + 1)));
    c->obs = c->obs_buf;
    WSMC_HIP(hipMalloc(&c->run_grp, run_grp_bytes(c->N, T)));
    if (!c->vscratch) WSMC_HIP(hipMalloc(&c->vscratch, sizeof(double) * 2 * c->N));
    if (!c->xscratch) WSMC_HIP(hipMalloc(&c->xscratch, sizeof(double) * 2 * c->N));
    c->T_alloc = T;
    for (auto& g : c->graphs) {  // graphs bake old pointers
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        if (g.graph) (void)hipGraphDestroy(g.graph);
        if (g.owned) (void)hipFree(g.owned);
    }
    c->graphs.clear();
    return WSMC_OK;
}

struct RunPlan {
    int32_t T = 0, keep = 0, scheme = 0;
    bool exact_stats = false;   // the statistics' own kernel at every step (a replay after a missed guess)
    double ess_min = 0, q_var = 0, r_var = 0;
    double x0[2] = {0, 0}, v0[2] = {0, 0};
    int32_t colx = -1, colv = -1, coldv = -1;
    std::vector<int32_t> xcols;  // x_1 .. x_{T+1}
    double** d_hist_work = nullptr;
    double** d_hist_out = nullptr;
};

// where the fused run takes the Resample statistics (see enqueue_ssm2d); measured in round 6
// (DESIGN.md §3). A diagnostic build (tools/build_variant.py -DWSMC_DIAG_BUILD) reads
// WSMC_DIAG_QSTAT for A/B runs; the product library ignores the environment.
// q stored by the propagate (1) or recomputed by the fill from the weights (2): stored is ahead
// while a step's working set stays in the MALL, recomputed (8 B a particle less traffic) beyond
// it — measured alternated on one box (profiles/r06_p*): 1M 3.035 / 3.096 against 3.008 / 3.010e10,
// 2M 3.752 / 3.766 against 3.735 / 3.741e10, 4M 3.994 / 3.998 against 4.010 / 4.009e10, 8M 4.082
// / 4.081 against 4.151 / 4.164e10
constexpr int64_t kQstatRecomputeN = 3000000;   // between the 2M and 4M measurements
static int run_qstat_mode(int64_t N) {
    const int dflt = N >= kQstatRecomputeN ? 2 : 1;
#ifdef WSMC_DIAG_BUILD
    static const int v = [] {
        const char* e = diag_env("WSMC_DIAG_QSTAT");
        return e ? atoi(e) : -1;
    }();
    return v >= 0 ? v : dflt;
#else
    return dflt;
#endif
}

// events (timing mode): per step 8 = {prop, sums, reduce, scan} x {start, stop} bound to the
// dispatches themselves (hipExtLaunchKernelGGL), then 2 for the finalize kernel
// a parity's pinned staging: [op-base bits, pad, obs 2T] (ensure_run_buffers sizes it)
static inline double* run_stage(wsmc_ctx* c, int par) {
    return c->run_hstage + (size_t)par * (2 * (size_t)c->T_alloc + 4);
}
static void run_stage_fill(wsmc_ctx* c, int par, uint64_t op_base, const double* obs, int T) {
    double* st = run_stage(c, par);
    st[0] = wsmc_bits2d(op_base);
    st[1] = 0.0;
    std::memcpy(st + 2, obs, sizeof(double) * 2 * (size_t)T);
}

static int enqueue_ssm2d(wsmc_ctx* c, const RunPlan& p, const std::vector<hipEvent_t>* ev) {
    const int T = p.T;
    const int64_t N = c->N;
    const double r_var = p.r_var;
    const double cpre = 2.0 * WSMC_LOG2PI + 2.0 * wsmc_log(r_var);
    auto E = [&](int k) -> hipEvent_t { return ev ? (*ev)[k] : nullptr; };
    const bool sharded = is_sharded(c);
    const int G = group_tiles(N);
    // this run's parity (its op word, observations, saved weights and read-back)
    const int64_t par = (c->run_op - c->run_params) / 4;
    {   // the head: per-step words zeroed, op word and observations in (one launch)
        RunHead h;
        h.z[0] = reinterpret_cast<unsigned long long*>(c->run_max);
        h.zwords[0] = (int64_t)(sizeof(MaxSlots) / 8) * (T + 1);
        h.z[1] = reinterpret_cast<unsigned long long*>(c->run_dec);
        h.zwords[1] = (int64_t)(sizeof(Decision) / 8) * (T + 1);
        h.z[2] = c->run_grp;
        h.zwords[2] = (int64_t)(run_grp_bytes(N, T) / 8);
        h.hstage = run_stage(c, (int)par);
        h.obs = c->obs;
        h.nobs = 2 * T;
        h.op = c->run_op;
        WSMC_HIP(launch_run_head(c->stream, h));
    }
    double* vbuf[2] = {c->cols[p.colv].back, c->vscratch};
    double* xbuf[2] = {p.keep ? nullptr : c->cols[p.colx].back, c->xscratch};
    // the Resample statistics' place (round 6): 0 = their own kernel (k_rs_sums_t), 1 = in the
    // propagate with q stored for the fill, 2 = in the propagate, the fill recomputing q
    // From step 2 on the propagate guesses the reference point from a bound (k_ssm2d_prop QS); the
    // first step has no bound and takes the statistics' own kernel. One GPU: the fill's record
    // block checks the guess and counts a miss into run_dec[0].ntasks, and the host re-does a run
    // with a miss on the exact path (wsmc_ssm2d_run); sharded: k_rs_qfix checks and recomputes in
    // place (the shards' decisions are global, so a replay would have to be too).
    const int qs = p.scheme == WSMC_RESAMPLE_MULTINOMIAL || p.exact_stats ? 0 : run_qstat_mode(N);
    for (int t = 1; t <= T; ++t) {
        const bool guess = qs && t > 1;
        Ssm2dArgs a;
        a.t = t;
        a.keep_history = p.keep;
        a.N = N;
        a.goff = c->goff;
        a.seed = c->seed;
        a.op_dev = c->run_op;
        a.obs = c->obs;
        a.x0[0] = p.x0[0]; a.x0[1] = p.x0[1];
        a.v0[0] = p.v0[0]; a.v0[1] = p.v0[1];
        a.q_sd = wsmc_sqrt(p.q_var);
        a.r_var = r_var;
        a.c0 = cpre;
        if (p.keep) {
            a.x_prev = t > 1 ? c->cols[p.xcols[t]].back : nullptr;   // x_t (written at step t-1)
            a.x_next = c->cols[p.xcols[t + 1]].back;                  // x_{t+1}
        } else {
            a.x_prev = t > 1 ? xbuf[t & 1] : nullptr;
            a.x_next = xbuf[(t + 1) & 1];
        }
        a.v_prev = t > 1 ? vbuf[t & 1] : nullptr;
        a.v_next = vbuf[(t + 1) & 1];
        // the reference's dv column holds the latest draw only: earlier steps' draws are
        // overwritten before anything reads them, so only step T stores it
        a.dv = t == T ? c->cols[p.coldv].back : nullptr;
        a.w = c->w;
        a.anc_prev = t > 1 ? c->anc_log + (size_t)(t - 2) * anc_stride(N) : nullptr;
        a.dec_prev = t > 1 ? c->run_dec + (t - 1) : nullptr;
        MaxSlots* ms = c->run_max + t;
        ShardRecord* recs = c->run_rec + (size_t)t * c->world;
        if (sharded && p.scheme != WSMC_RESAMPLE_MULTINOMIAL && t > 1) {
            // island: the previous step's decision is taken in this kernel from its records
            a.recs_prev = c->run_rec + (size_t)(t - 1) * c->world;
            a.dec_out = c->run_dec + (t - 1);
            a.world = c->world;
            a.rank = c->rank;
            a.ess_min = p.ess_min;
        }
        a.ms = ms;
        if (qs && t == 1 && !sharded)   // a replay starts from these weights (this run's parity)
            a.w_save = c->run_w0 + (size_t)par * N;
        if (guess) {   // stratified / systematic: the propagate takes the Resample statistics too
            a.qstat = true;
            a.ms_prev = t > 1 ? c->run_max + (t - 1) : nullptr;
            a.rg_out = c->run_rg + t;
            a.tilep = c->tilep;
            a.grp = c->run_grp + (size_t)t * run_grp_words(N);
            a.G = G;
            a.qbuf = qs == 1 ? c->qbuf : nullptr;
        }
        const int k0 = 8 * (t - 1);
        WSMC_HIP(launch_ssm2d_propagate(c->stream, a, E(k0), E(k0 + 1)));
        const FillPlan plan = fill_plan(c, p.scheme, 3ull * (uint64_t)(t - 1) + 2ull, c->run_op);
        int32_t* anc_row = c->anc_log + (size_t)(t - 1) * anc_stride(N);
        if (p.scheme == WSMC_RESAMPLE_MULTINOMIAL) {
            // unsorted draws: sums, reduce (tile offsets, record), [exchange + decide], CDF + search
            WSMC_HIP(launch_rs_sums_multi(c->stream, c->w, N, ms, plan, c->tilep, c->cdf, multi_esum(c), multi_ebuf(c), E(k0 + 2),
                                          E(k0 + 3)));
            WSMC_HIP(launch_rs_reduce(c->stream, ms, c->tilep, N, c->tileOff, recs + c->rank, !sharded, p.ess_min,
                                      c->run_dec + t, &plan, E(k0 + 6), nullptr, multi_esum(c)));
            if (sharded) {
                int r = exchange_recs(c, recs);
                if (r) return r;
                WSMC_HIP(launch_rs_decide(c->stream, recs, c->world, c->rank, p.ess_min, c->run_dec + t));
            }
            WSMC_HIP(launch_rs_multinomial(c->stream, N, recs + c->rank, c->run_dec + t, plan, c->tileOff, c->cdf,
                                           multi_esum(c), multi_ebuf(c), anc_row, nullptr, E(k0 + 7)));
            continue;
        }
        // group sums of q + one fill launch whose extra block builds the shard record (and,
        // on one GPU, decides). Sharded: the records are all-gathered on the same stream and
        // every rank decides in rank order (k_rs_decide); island resampling fills from the
        // shard's own Q, so the fill never waits for the collective.
        unsigned long long* grp = c->run_grp + (size_t)t * run_grp_words(N);
        FillPlan fp = plan;
        if (guess && sharded) {   // check the propagate's reference point (usually a no-op) and fix
            WSMC_HIP(launch_rs_qfix(c->stream, c->w, N, ms, c->run_rg + t, c->tilep, qs == 1 ? c->qbuf : nullptr, grp, G,
                                    c->run_nfix, E(k0 + 2), E(k0 + 3)));
        } else if (guess) {       // checked by the fill's record block
            fp.rg_check = c->run_rg + t;
            fp.rg_miss = &c->run_dec[0].ntasks;
            if (E(k0 + 2)) {      // (instrumented runs: no statistics kernel, an empty interval)
                WSMC_HIP(hipEventRecord(E(k0 + 2), c->stream));
                WSMC_HIP(hipEventRecord(E(k0 + 3), c->stream));
            }
        } else {
            WSMC_HIP(launch_rs_sums(c->stream, c->w, N, ms, c->tilep, c->qbuf, E(k0 + 2), E(k0 + 3), grp, G));
        }
        WSMC_HIP(launch_rs_fill_fused(c->stream, N, fp, grp, G, ms, p.ess_min, recs + c->rank,
                                      sharded ? nullptr : c->run_dec + t, c->qbuf, anc_row, E(k0 + 6), E(k0 + 7),
                                      guess && qs == 2 ? c->w : nullptr));
        if (sharded) {   // the next propagate (or the trace-back) decides from the records
            int r = exchange_recs(c, recs);
            if (r) return r;
        }
    }
    Ssm2dFinal f;
    f.T = T;
    f.keep_history = p.keep;
    f.N = N;
    f.x0[0] = p.x0[0]; f.x0[1] = p.x0[1];
    f.hist_work = p.d_hist_work;
    f.hist_out = p.d_hist_out;
    f.x_work = p.keep ? nullptr : xbuf[(T + 1) & 1];
    f.x_out = p.keep ? nullptr : c->cols[p.colx].front;
    f.v_work = vbuf[(T + 1) & 1];
    f.v_out = c->cols[p.colv].front;
    f.dv_work = c->cols[p.coldv].back;
    f.dv_out = c->cols[p.coldv].front;
    f.w = c->w;
    f.anc_log = c->anc_log;
    f.anc_stride = anc_stride(N);
    f.dec = c->run_dec;
    f.hdec = c->run_hdec + (size_t)par * (c->T_alloc + 1);
    f.last_anc = c->anc;
    if (sharded && p.scheme != WSMC_RESAMPLE_MULTINOMIAL) {
        f.recs_last = c->run_rec + (size_t)T * c->world;
        f.dec_out = c->run_dec + T;
        f.world = c->world;
        f.rank = c->rank;
        f.ess_min = p.ess_min;
    }
    WSMC_HIP(launch_ssm2d_finalize(c->stream, f, E(8 * T), E(8 * T + 1)));
    return WSMC_OK;
}

// ---- exact shards without host round trips -------------------------------------------------
// Fixed-size blocks to the neighbours: send[0] to rank - 1, send[1] to rank + 1; recv[0] from
// rank - 1, recv[1] from rank + 1. RCCL: one group of send / recv on the stream (sizes fixed, so
// it is captured with the run); host exchange (tests): every rank all-gathers its two blocks.
static int exchange_neighbors(wsmc_ctx* c, unsigned long long* const send[2], unsigned long long* const recv[2],
                              int64_t words, hipStream_t s) {
    const int W = c->world, me = c->rank;
    if (W < 2 || words <= 0) return WSMC_OK;
    if (c->host_exchange) {
        // in pieces of at most 2^22 words a block (the callback counts words in an int32, a
        // gathered message stays far below the host transport's 1 GB limit at 8 ranks, and
        // every rank cuts the same pieces: words is the same on all of them)
        const int64_t piece = (int64_t)1 << 22;
        for (int64_t at = 0; at < words; at += piece) {
            const int64_t n = std::min(piece, words - at);
            std::vector<unsigned long long> mine(2 * (size_t)n), all(2 * (size_t)n * W);
            WSMC_HIP(hipMemcpyAsync(mine.data(), send[0] + at, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost, s));
            WSMC_HIP(hipMemcpyAsync(mine.data() + n, send[1] + at, sizeof(unsigned long long) * n,
                                    hipMemcpyDeviceToHost, s));
            WSMC_HIP(ctx_sync(c, s));
            if (host_xchg(c, reinterpret_cast<const uint64_t*>(mine.data()), (int32_t)(2 * n),
                                 reinterpret_cast<uint64_t*>(all.data())) != 0)
                return fail(WSMC_ERCCL, "host neighbour exchange failed");
            if (me > 0)   // the left rank's right block
                WSMC_HIP(hipMemcpyAsync(recv[0] + at, all.data() + (size_t)(me - 1) * 2 * n + n,
                                        sizeof(unsigned long long) * n, hipMemcpyHostToDevice, s));
            if (me + 1 < W)   // the right rank's left block
                WSMC_HIP(hipMemcpyAsync(recv[1] + at, all.data() + (size_t)(me + 1) * 2 * n,
                                        sizeof(unsigned long long) * n, hipMemcpyHostToDevice, s));
            WSMC_HIP(ctx_sync(c, s));
        }
        return WSMC_OK;
    }
    WSMC_RCCL_GUARD(c);
    c->exchanges += 1;
        WSMC_RCCL(ncclGroupStart());
    if (me > 0) {
        WSMC_RCCL(ncclSend(send[0], (size_t)words, ncclUint64, me - 1, c->comm, s));
        WSMC_RCCL(ncclRecv(recv[0], (size_t)words, ncclUint64, me - 1, c->comm, s));
    }
    if (me + 1 < W) {
        WSMC_RCCL(ncclSend(send[1], (size_t)words, ncclUint64, me + 1, c->comm, s));
        WSMC_RCCL(ncclRecv(recv[1], (size_t)words, ncclUint64, me + 1, c->comm, s));
    }
    WSMC_RCCL(ncclGroupEnd());
    return WSMC_OK;
}

// the block (slots per neighbour per step) and window (ids per neighbour per level) sizes:
// every rank derives the same values (from the global size, and the overflow statistics all
// ranks see), so their fixed-size collectives match
static void exact_sizes(const wsmc_ctx* c, int64_t* cap, int64_t* ctr) {
    const int64_t nmin = c->gN / c->world;   // the smallest (ragged) shard
    // the default block: a shard's slot window moves by the weight mass its particles hold
    // beyond their share, which grows like sqrt(n) (C4's 2 x 1M forced run needed 6.2k slots;
    // the blocks a run settles at after a first overflow were 4x that): 16 sqrt(n), so a first
    // run at that shape does not overflow and re-run eagerly, at most half a shard
    int64_t cdef = 1024;
    while (cdef * cdef < 256 * nmin && 2 * cdef <= nmin) cdef *= 2;
    int64_t cp = c->x_cap ? c->x_cap : cdef;
    int64_t ct = c->x_ctr ? c->x_ctr : std::max<int64_t>(1024, nmin / 128);
    *cap = std::max<int64_t>(1, std::min(cp, nmin));
    *ctr = std::max<int64_t>(1, std::min(ct, nmin));
}
static bool exact_eager_forced() {   // diagnostics / A-B: the host-driven exact run only
    static const bool v = [] {
        const char* e = getenv("WSMC_EXACT_EAGER");
        return e && atoi(e) != 0;
    }();
    return v;
}
// group-line words per rank in the all-gathered statistics: the same on every rank (the
// larger of the two shard sizes a ragged split can give)
static inline int64_t run_grp_words(int64_t N);
static int64_t exact_line_words(const wsmc_ctx* c) {
    const int64_t lo = c->gN / c->world, hi = (c->gN + c->world - 1) / c->world;
    return std::max(run_grp_words(lo), run_grp_words(hi));
}
static int ensure_exact_async(wsmc_ctx* c, int32_t T, int64_t cap, int64_t ctr) {
    int r = ensure_exact(c);
    if (r) return r;
    const int64_t N = c->N;
    const int64_t wwords = (int64_t)T * ctr * 3;
    const int64_t astride = (N + 2 * cap + 3) & ~(int64_t)3;
    const int64_t awords = (int64_t)T * astride;
    const int64_t msn = (int64_t)(T + 1) * c->world;
    const int64_t lwords = msn * exact_line_words(c);
    const bool grow = !c->xpairs || cap > c->xnb_cap || wwords > c->xwin_words || awords > c->xanc_words ||
                      msn > c->xms_n || lwords > c->xlines_words;
    c->xanc_stride = astride;
    if (!grow && c->xstat && c->w_save) return WSMC_OK;
    WSMC_HIP(ctx_sync(c, c->stream));
    if (!c->xpairs) WSMC_HIP(hipMalloc(&c->xpairs, sizeof(double) * 6 * (size_t)N));
    if (!c->xstat) WSMC_HIP(hipMalloc(&c->xstat, sizeof(unsigned long long) * kMaxShards * kXStat));
    if (c->peer_ok && !c->xpeer) WSMC_HIP(hipMalloc(&c->xpeer, sizeof(unsigned long long) * kMaxShards * 8));
    if (!c->w_save) WSMC_HIP(hipMalloc(&c->w_save, sizeof(double) * (size_t)N));
    if (cap > c->xnb_cap) {
        if (c->xnb) WSMC_HIP(hipFree(c->xnb));
        WSMC_HIP(hipMalloc(&c->xnb, sizeof(unsigned long long) * 4 * (size_t)cap * kXWords));
        c->xnb_cap = cap;
    }
    if (wwords > c->xwin_words) {
        if (c->xwin) WSMC_HIP(hipFree(c->xwin));
        WSMC_HIP(hipMalloc(&c->xwin, sizeof(unsigned long long) * 4 * (size_t)wwords));
        c->xwin_words = wwords;
    }
    if (awords > c->xanc_words) {
        if (c->xanc) WSMC_HIP(hipFree(c->xanc));
        WSMC_HIP(hipMalloc(&c->xanc, sizeof(int32_t) * (size_t)awords));
        c->xanc_words = awords;
    }
    if (msn > c->xms_n) {
        if (c->xms) WSMC_HIP(hipFree(c->xms));
        WSMC_HIP(hipMalloc(&c->xms, sizeof(MaxSlots) * (size_t)msn));
        c->xms_n = msn;
    }
    if (lwords > c->xlines_words) {
        if (c->xlines) WSMC_HIP(hipFree(c->xlines));
        WSMC_HIP(hipMalloc(&c->xlines, sizeof(unsigned long long) * (size_t)lwords));
        c->xlines_words = lwords;
    }
    return WSMC_OK;
}

// The fused 2D SSM run on exact shards with no host round trip: per step the
// propagate (ancestors as global ids: a neighbour's particle is read from the pairs it sent),
// the global max and the records all-gathered, the single-GPU decision and window fill
// (k_rs_decide_exact, the fill), then k_exact_route / the neighbour exchange / k_exact_recv
// move the window's slots to their owners through fixed-size blocks; at the end the trace
// windows are exchanged once and k_exact_final traces every lineage back, and every rank's
// overflow statistics are all-gathered. A slot or lineage the blocks cannot carry sets an
// overflow bit: the host then re-runs the filter on the eager path.
static int enqueue_ssm2d_exact(wsmc_ctx* c, const RunPlan& p, int64_t cap, int64_t ctr) {
    const int T = p.T;
    const int64_t N = c->N;
    const int W = c->world, me = c->rank;
    const double cpre = 2.0 * WSMC_LOG2PI + 2.0 * wsmc_log(p.r_var);
    WSMC_HIP(hipMemsetAsync(c->xms, 0, sizeof(MaxSlots) * (size_t)(T + 1) * W, c->stream));
    const int64_t xstride = exact_line_words(c);
    const int G = group_tiles(N);
    WSMC_HIP(hipMemsetAsync(c->xlines, 0, sizeof(unsigned long long) * (size_t)(T + 1) * W * xstride, c->stream));
    WSMC_HIP(hipMemsetAsync(c->run_dec, 0, sizeof(Decision) * (T + 1), c->stream));
    WSMC_HIP(hipMemsetAsync(c->xstat, 0, sizeof(unsigned long long) * kMaxShards * kXStat, c->stream));
    const int64_t S = c->xanc_stride;
    auto row = [&](int t) { return c->xanc + (size_t)(t - 1) * S; };   // step t's row, from its left margin
    const int64_t glo = c->goff - cap;                                  // the global slot of row index 0
    const unsigned long long row_lo = glo > 0 ? (unsigned long long)glo : 0ull;
    const unsigned long long row_hi = std::min<unsigned long long>((unsigned long long)c->gN,
                                                                   (unsigned long long)(c->goff + N + cap));
    WSMC_HIP(hipMemcpyAsync(c->w_save, c->w, sizeof(double) * N, hipMemcpyDeviceToDevice, c->stream));
    double* Xr = c->xpairs;
    double* Vr = Xr + 2 * N;
    double* DVr = Vr + 2 * N;
    const int64_t bw = cap * kXWords;
    unsigned long long* const snd[2] = {c->xnb, c->xnb + bw};
    unsigned long long* const rcv[2] = {c->xnb + 2 * bw, c->xnb + 3 * bw};
    double* vbuf[2] = {c->cols[p.colv].back, c->vscratch};
    double* xbuf[2] = {p.keep ? nullptr : c->cols[p.colx].back, c->xscratch};
    double* dvw = c->cols[p.coldv].back;
    unsigned long long* stat = c->xstat + (size_t)me * kXStat;
    int r;
    for (int t = 1; t <= T; ++t) {
        Ssm2dArgs a;
        a.t = t;
        a.keep_history = p.keep;
        a.N = N;
        a.goff = c->goff;
        a.seed = c->seed;
        a.op_dev = c->run_op;
        a.obs = c->obs;
        a.x0[0] = p.x0[0]; a.x0[1] = p.x0[1];
        a.v0[0] = p.v0[0]; a.v0[1] = p.v0[1];
        a.q_sd = wsmc_sqrt(p.q_var);
        a.r_var = p.r_var;
        a.c0 = cpre;
        if (p.keep) {
            a.x_prev = t > 1 ? c->cols[p.xcols[t]].back : nullptr;
            a.x_next = c->cols[p.xcols[t + 1]].back;
        } else {
            a.x_prev = t > 1 ? xbuf[t & 1] : nullptr;
            a.x_next = xbuf[(t + 1) & 1];
        }
        a.v_prev = t > 1 ? vbuf[t & 1] : nullptr;
        a.v_next = vbuf[(t + 1) & 1];
        a.dv = t == T ? dvw : nullptr;
        a.w = c->w;
        a.anc_prev = t > 1 ? row(t - 1) + cap : nullptr;
        a.dec_prev = t > 1 ? c->run_dec + (t - 1) : nullptr;
        MaxSlots* msx = c->xms + (size_t)t * W;   // every rank's slots of this step
        a.ms = msx + me;
        a.identity = 0;
        a.xr = Xr;
        a.vr = Vr;
        WSMC_HIP(launch_ssm2d_propagate(c->stream, a));
        // every rank's max slots (the global max), this shard's record relative to it (K from
        // the global N), every rank's record: exactly the single-context statistics
        if ((r = exchange_words(c, reinterpret_cast<unsigned long long*>(msx), sizeof(MaxSlots) / 8, c->stream)))
            return r;
        // the statistics into this rank's group lines (every part), all-gathered in place of
        // the record: the fill's blocks take the global Q and their CDF offsets from them, its
        // record block builds every rank's record and decides (the single-GPU bits)
        unsigned long long* lines = c->xlines + (size_t)t * W * xstride;
        WSMC_HIP(launch_rs_sums(c->stream, c->w, N, msx, c->tilep, c->qbuf, nullptr, nullptr, lines + me * xstride,
                                G, c->gN, W, 1));
        if ((r = exchange_words(c, lines, xstride, c->stream))) return r;
        FillPlan plan = fill_plan(c, p.scheme, 3ull * (uint64_t)(t - 1) + 2ull, c->run_op);
        plan.slot_base = 0;   // slots are global: their keys too
        plan.xlines = lines;
        plan.xstride = xstride;
        plan.xms = msx;
        plan.n_global = (unsigned long long)c->gN;
        plan.dx_world = W;
        plan.dx_rank = me;
        plan.dx_ess = p.ess_min;
        plan.dx_comb = c->comb;
        plan.dx_dec = c->run_dec + t;
        plan.dx_xp = c->xp;
        plan.id_base = (int32_t)c->goff;
        plan.row_lo = row_lo;
        plan.row_hi = row_hi;
        plan.xstat = stat;
        // the fill stores slot s at anc[s - row_lo]: the row index of s is s - glo
        WSMC_HIP(launch_rs_fill_fused(c->stream, N, plan, lines + me * xstride, G, msx, p.ess_min, c->rec + me,
                                      c->run_dec + t, c->qbuf, row(t) + ((int64_t)row_lo - glo)));
        ExactStep e;
        e.xp = c->xp;
        e.dec = c->run_dec + t;
        e.row = row(t);
        e.x = a.x_next;
        e.v = a.v_next;
        e.dv = dvw;
        e.anc_row = row(t) + cap;
        e.send[0] = snd[0]; e.send[1] = snd[1];
        e.recv[0] = rcv[0]; e.recv[1] = rcv[1];
        e.xr = Xr; e.vr = Vr; e.dvr = DVr;
        e.stat = stat;
        e.cap = cap;
        e.N = N;
        e.goff = c->goff;
        e.rank = me;
        e.world = W;
        if (W > 1) {
            WSMC_HIP(launch_exact_route(c->stream, e));
            if ((r = exchange_neighbors(c, snd, rcv, bw, c->stream))) return r;
            WSMC_HIP(launch_exact_recv(c->stream, e));
        }
    }
    const int64_t ww = (int64_t)T * ctr * 3;
    unsigned long long* const wsnd[2] = {c->xwin, c->xwin + ww};
    unsigned long long* const wrcv[2] = {c->xwin + 2 * ww, c->xwin + 3 * ww};
    // shards of one process that can read each other's memory trace lineages through the
    // owners' rows and history in place (no windows, no cross-rank trace after the run)
    const bool peer = c->peer_ok && p.keep && W > 1 && c->xpeer;
    const bool wins = p.keep && W > 1 && !c->x_trace && !peer;
    if (peer) {
        const unsigned long long pw[8] = {(unsigned long long)(uintptr_t)(c->xanc + cap), (unsigned long long)S,
                                          (unsigned long long)(uintptr_t)p.d_hist_work,
                                          (unsigned long long)c->goff, (unsigned long long)N, 0ull, 0ull, 0ull};
        WSMC_HIP(launch_put_words(c->stream, c->xpeer + (size_t)me * 8, pw));
        if ((r = exchange_words(c, c->xpeer, 8, c->stream))) return r;
    }
    if (wins) {
        ExactWin w;
        w.hist_work = p.d_hist_work;
        w.anc_log = c->xanc + cap;
        w.anc_stride = S;
        w.dec = c->run_dec;
        w.out = c->xwin;
        w.ctr = ctr;
        w.N = N;
        w.goff = c->goff;
        w.T = T;
        w.has_left = me > 0;
        w.has_right = me + 1 < W;
        WSMC_HIP(launch_exact_window_pack(c->stream, w));
        if ((r = exchange_neighbors(c, wsnd, wrcv, ww, c->stream))) return r;
    }
    ExactFinal f;
    f.T = T;
    f.keep_history = p.keep;
    f.N = N;
    f.goff = c->goff;
    f.ctr = ctr;
    f.x0[0] = p.x0[0]; f.x0[1] = p.x0[1];
    f.hist_work = p.d_hist_work;
    f.hist_out = p.d_hist_out;
    f.x_work = p.keep ? nullptr : xbuf[(T + 1) & 1];
    f.x_out = p.keep ? nullptr : c->cols[p.colx].front;
    f.v_work = vbuf[(T + 1) & 1];
    f.v_out = c->cols[p.colv].front;
    f.dv_work = dvw;
    f.dv_out = c->cols[p.coldv].front;
    f.xr = Xr; f.vr = Vr; f.dvr = DVr;
    f.w = c->w;
    f.anc_log = c->xanc + cap;
    f.anc_stride = S;
    f.dec = c->run_dec;
    f.win[0] = wins && me > 0 ? wrcv[0] : nullptr;
    f.win[1] = wins && me + 1 < W ? wrcv[1] : nullptr;
    f.stat = stat;
    f.peer = peer ? c->xpeer : nullptr;
    f.world = W;
    WSMC_HIP(launch_exact_final(c->stream, f));
    // every rank's overflow bits: all ranks take the same branch (re-run or not) afterwards
    return exchange_words(c, c->xstat, kXStat, c->stream);
}

// The fused 2D SSM run on exact shards (SURVEY §8(e) item 4, C4 with the single-GPU bits),
// eager and host-driven. Each step:
//   propagate from the state already gathered in slot order (identity read);
//   exact statistics, decision and the window fill (exact_decide_fill);
//   on a resample the state (x, v; dv at the last step) moves to the owners of its slots,
//   with the global ancestor ids into the ancestor log.
// The history x_1..x_{T+1} is traced back across ranks: one range exchange per step
// (trace_level).
static int ssm2d_run_exact(wsmc_ctx* c, const RunPlan& p, uint64_t op_base) {
    const int T = p.T;
    const int64_t N = c->N;
    int r = ensure_exact(c);
    if (r) return r;
    for (int k = 0; k < 9; ++k)
        if (!c->xrun[k]) WSMC_HIP(hipMalloc(&c->xrun[k], sizeof(double) * 2 * (size_t)N));
    for (int k = 0; k < 2; ++k)
        if (!c->lineage[k]) WSMC_HIP(hipMalloc(&c->lineage[k], sizeof(int32_t) * (size_t)N));
    double* Gx[2] = {c->xrun[0], c->xrun[1]};
    double* Gv[2] = {c->xrun[2], c->xrun[3]};
    double* Gdv = c->xrun[4];
    double* Xt[2] = {c->xrun[5], c->xrun[6]};
    double* Vt[2] = {c->xrun[7], c->xrun[8]};
    WSMC_HIP(hipMemsetAsync(c->run_max, 0, sizeof(MaxSlots) * (T + 1), c->stream));
    WSMC_HIP(hipMemsetAsync(c->run_dec, 0, sizeof(Decision) * (T + 1), c->stream));
    const double cpre = 2.0 * WSMC_LOG2PI + 2.0 * wsmc_log(p.r_var);
    const double* cur_x = nullptr;
    const double* cur_v = nullptr;
    double* dvw = c->cols[p.coldv].back;   // pairs: the last step's draws
    const double* cur_dv = dvw;
    std::vector<int> rs(T + 1, 0);
    ExactPlan hx{};
    for (int t = 1; t <= T; ++t) {
        Ssm2dArgs a;
        a.t = t;
        a.keep_history = p.keep;
        a.N = N;
        a.goff = c->goff;
        a.seed = c->seed;
        a.op_dev = c->run_op;
        a.obs = c->obs;
        a.x0[0] = p.x0[0]; a.x0[1] = p.x0[1];
        a.v0[0] = p.v0[0]; a.v0[1] = p.v0[1];
        a.q_sd = wsmc_sqrt(p.q_var);
        a.r_var = p.r_var;
        a.c0 = cpre;
        a.x_prev = cur_x;
        a.v_prev = cur_v;
        a.x_next = p.keep ? c->cols[p.xcols[t + 1]].back : Xt[t & 1];
        a.v_next = Vt[t & 1];
        a.dv = t == T ? dvw : nullptr;
        a.w = c->w;
        a.anc_prev = nullptr;
        a.identity = 1;
        a.dec_prev = t > 1 ? c->run_dec + (t - 1) : nullptr;
        a.ms = c->run_max + t;
        WSMC_HIP(launch_ssm2d_propagate(c->stream, a));
        Decision hd;
        if ((r = exact_decide_fill(c, p.ess_min, p.scheme, op_base + 3ull * (uint64_t)(t - 1) + 2ull, c->run_dec + t,
                                   &hd, &hx)))
            return r;
        rs[t] = hd.resampled;
        if (!hd.resampled) {
            cur_x = a.x_next;
            cur_v = a.v_next;
            continue;
        }
        std::vector<const double*> src = {a.x_next, a.x_next + 1, a.v_next, a.v_next + 1};
        std::vector<double*> dst = {Gx[t & 1], Gx[t & 1] + 1, Gv[t & 1], Gv[t & 1] + 1};
        if (t == T) {
            src.push_back(dvw); src.push_back(dvw + 1);
            dst.push_back(Gdv); dst.push_back(Gdv + 1);
            cur_dv = Gdv;
        }
        if ((r = exact_route(c, hx, src, dst, 2, c->anc_log + (size_t)(t - 1) * anc_stride(N)))) return r;
        cur_x = Gx[t & 1];
        cur_v = Gv[t & 1];
    }
    if (rs[T]) WSMC_HIP(launch_fill_weights(c->stream, c->w, c->run_dec + T, N));
    WSMC_HIP(launch_pairs_to_soa(c->stream, cur_v, c->cols[p.colv].front, N));
    WSMC_HIP(launch_pairs_to_soa(c->stream, cur_dv, c->cols[p.coldv].front, N));
    if (!p.keep) {
        WSMC_HIP(launch_pairs_to_soa(c->stream, cur_x, c->cols[p.colx].front, N));
        return WSMC_OK;
    }
    WSMC_HIP(launch_fill_const2(c->stream, c->cols[p.xcols[1]].front, p.x0[0], p.x0[1], N));
    // lineage at step T: the last ancestors (global ids), then one range exchange per step:
    // level t gives x_{t+1} = hist[t+1][a_t] and a_{t-1} = ancestors of step t-1 at a_t
    int32_t* A = c->lineage[0];
    int32_t* B = c->lineage[1];
    if (rs[T])
        WSMC_HIP(hipMemcpyAsync(A, c->anc_log + (size_t)(T - 1) * anc_stride(N), sizeof(int32_t) * N,
                                hipMemcpyDeviceToDevice, c->stream));
    else
        WSMC_HIP(launch_iota(c->stream, A, N, c->goff));
    for (int t = T; t >= 1; --t) {
        const int32_t* arow = (t >= 2 && rs[t - 1]) ? c->anc_log + (size_t)(t - 2) * anc_stride(N) : nullptr;
        if ((r = trace_level(c, hx, c->cols[p.xcols[t + 1]].back, arow, A, B, c->cols[p.xcols[t + 1]].front)))
            return r;
        std::swap(A, B);
    }
    return WSMC_OK;
}

// The history of an exact-shard run whose filter completed on the device but whose lineages
// left the trace windows (overflow bit 1 only: every particle moved within its blocks, so the
// weights, the final columns and the global-id ancestor rows are right): x_2..x_{T+1} traced
// across ranks level by level (trace_level, the eager path's exchange) over the rows the run
// wrote, instead of re-running the filter.
static int exact_trace_history(wsmc_ctx* c, const RunPlan& p, int64_t cap) {
    const int T = p.T;
    const int64_t N = c->N;
    int r = ensure_exact(c);
    if (r) return r;
    for (int k = 0; k < 2; ++k)
        if (!c->lineage[k]) WSMC_HIP(hipMalloc(&c->lineage[k], sizeof(int32_t) * (size_t)N));
    ExactPlan hx;
    std::vector<Decision> hdec(T + 1);
    WSMC_HIP(hipMemcpyAsync(&hx, c->xp, sizeof(ExactPlan), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(hipMemcpyAsync(hdec.data(), c->run_dec, sizeof(Decision) * (T + 1), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    const int64_t S = c->xanc_stride;
    auto arow_of = [&](int t) { return c->xanc + (size_t)(t - 1) * S + cap; };   // step t's global ancestor ids
    int32_t* A = c->lineage[0];
    int32_t* B = c->lineage[1];
    if (hdec[T].resampled)
        WSMC_HIP(hipMemcpyAsync(A, arow_of(T), sizeof(int32_t) * N, hipMemcpyDeviceToDevice, c->stream));
    else
        WSMC_HIP(launch_iota(c->stream, A, N, c->goff));
    for (int t = T; t >= 1; --t) {
        const int32_t* arow = (t >= 2 && hdec[t - 1].resampled) ? arow_of(t - 1) : nullptr;
        if ((r = trace_level(c, hx, c->cols[p.xcols[t + 1]].back, arow, A, B, c->cols[p.xcols[t + 1]].front)))
            return r;
        std::swap(A, B);
    }
    c->x_traces += 1;
    return WSMC_OK;
}

int wsmc_run_set_timing(wsmc_ctx* c, int32_t enabled) {
    if (c && c->multi) return multi_each(c, [&](wsmc_ctx* x) { return wsmc_run_set_timing(x, enabled); });
    if (!c) return fail(WSMC_EARG, "null context");
    c->timing = enabled != 0;
    return WSMC_OK;
}

int wsmc_run_get_timing(wsmc_ctx* c, wsmc_run_timing* out) {
    if (c && c->multi) return wsmc_run_get_timing(multi_first(c), out);
    if (!c || !out) return fail(WSMC_EARG, "null argument");
    *out = c->last_timing;
    return WSMC_OK;
}

// ---- asynchronous fused runs (round 6) -----------------------------------------------------
// A run enqueued without anything the caller reads back returns at once; its decisions land in
// pinned memory behind it (wsmc_ctx::run_hdec, by parity) and are folded in by the next entry
// point, or by the next run right after that run's own launch, so the device goes from one run
// to the next without waiting for the host. A run whose guessed reference point missed (the
// fill's record block counted it) is re-done then on the exact path, from the weights it
// started with — and so is a run enqueued after it, which started from its state.
struct RunPend {
    int par = 0;                   // buffer parity
    RunPlan p;
    uint64_t op_base = 0;
    std::vector<double> hobs;      // its observations (a replay uploads them again)
    bool guessed = false;          // the statistics were guessed (a miss is possible)
    void* temp_tables = nullptr;   // an eagerly enqueued run's history tables, freed when folded
};
static void run_book(wsmc_ctx* c, const RunPlan& p, const double* obs);
static void run_fold_decisions(wsmc_ctx* c, const Decision* hdec, int T);
static int fold_run(wsmc_ctx* c, RunPend* P, RunPend* Q);

int wsmc_ssm2d_run(wsmc_ctx* c, const double* obs, int32_t T, const double* x0, const double* v0, double q_var,
                   double r_var, double ess_min, int32_t scheme, int32_t keep_history, double* log_evidence_out) {
    if (c && c->multi)
        return multi_each(c, [&](wsmc_ctx* x) {
            double ev = 0;
            int r = wsmc_ssm2d_run(x, obs, T, x0, v0, q_var, r_var, ess_min, scheme, keep_history,
                                   log_evidence_out ? &ev : nullptr);
            if (!r && log_evidence_out && x == multi_first(c)) *log_evidence_out = ev;
            return r;
        });
    CHECK_CTX_DEV(c);
    static const bool no_graph = [] {   // diagnostics only: the same run enqueued eagerly
        const char* e = getenv("WSMC_DIAG_NO_GRAPH");
        return e && atoi(e) != 0;
    }();
    // asynchronous (round 6) when nothing in the call needs the run's results on the host: the
    // call returns once the run is enqueued, the previous asynchronous run is folded in after
    // this one's launch (so the device never waits for the host between runs)
    const bool async_run = !exact_mode(c) && !c->timing && !c->host_exchange && !log_evidence_out && !no_graph;
    if (!async_run)
        if (int r = resolve_run(c)) return r;
    if (int r = ew_flush(c)) return r;
    if (int r = virt_all(c)) return r;
    if (c->w_reset_pending) {
        WSMC_HIP(launch_fill_weights(c->stream, c->w, c->w_reset_pending, c->N));
        c->w_reset_pending = nullptr;
    }
    if (int r = resolve_decisions(c)) return r;
    scores_invalidate(c);   // the run rewrites columns the tape reads
    c->wseq += 1;           // ... and the weights
    if (!obs || T < 1 || !x0 || !v0) return fail(WSMC_EARG, "bad arguments");
    if (!valid_scheme(scheme)) return fail(WSMC_EARG, "unknown resampling scheme");
    if (exact_mode(c) && scheme == WSMC_RESAMPLE_MULTINOMIAL)
        return fail(WSMC_EARG, "multinomial draws on exact shards are not supported (island mode is)");
    if (scheme == WSMC_RESAMPLE_MULTINOMIAL && ensure_cdf(c)) return WSMC_EHIP;
    if (!(q_var > 0) || !(r_var > 0)) return fail(WSMC_EARG, "variances must be positive");
    RunPlan p;
    p.T = T;
    p.keep = keep_history ? 1 : 0;
    p.scheme = scheme;
    p.ess_min = ess_min;
    p.q_var = q_var;
    p.r_var = r_var;
    p.x0[0] = x0[0]; p.x0[1] = x0[1];
    p.v0[0] = v0[0]; p.v0[1] = v0[1];
    int r;
    // columns, in the order @model's statements create them (examples/2D_ssm.jl:8-16)
    if (p.keep) {
        p.xcols.assign(T + 2, -1);
        int32_t id;
        if ((r = wsmc_col_create(c, "x_1", 2, &id))) return r;
        p.xcols[1] = id;
        if ((r = wsmc_col_create(c, "v", 2, &p.colv))) return r;
        for (int t = 1; t <= T; ++t) {
            const std::string nm = "x_" + std::to_string(t + 1);
            if ((r = wsmc_col_create(c, nm.c_str(), 2, &id))) return r;
            p.xcols[t + 1] = id;
            if (t == 1 && (r = wsmc_col_create(c, "dv", 2, &p.coldv))) return r;
        }
    } else {
        if ((r = wsmc_col_create(c, "x", 2, &p.colx))) return r;
        if ((r = wsmc_col_create(c, "v", 2, &p.colv))) return r;
        if ((r = wsmc_col_create(c, "dv", 2, &p.coldv))) return r;
    }
    if ((r = ensure_run_buffers(c, T))) return r;
    // per-run values: obs, op base — in this run's parity of the buffers (the previous run may
    // still read the other one; the one before it has been folded in, so it is done)
    const int par = c->run_par;
    c->run_par ^= 1;
    c->obs = c->obs_buf + (size_t)par * 2 * (c->T_alloc + 1);
    c->run_op = c->run_params + 4 * par;
    const uint64_t op_base = c->op;
    std::vector<double> hobs(obs, obs + 2 * (size_t)T);
    // this parity's pinned staging (the run two calls back, its last reader, has been folded in):
    // the head kernel of the run copies it; the exact-shard paths copy it here
    run_stage_fill(c, par, op_base, obs, T);
    if (exact_mode(c)) {
        const double* st = run_stage(c, par);
        WSMC_HIP(hipMemcpyAsync(c->obs, st + 2, sizeof(double) * 2 * T, hipMemcpyHostToDevice, c->stream));
        WSMC_HIP(hipMemcpyAsync(c->run_op, st, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    }

    char keybuf[512];
    std::snprintf(keybuf, sizeof(keybuf), "ssm2d T=%d keep=%d sch=%d ess=%.17g q=%.17g r=%.17g x0=%.17g,%.17g v0=%.17g,%.17g w=%d tm=%d",
                  T, p.keep, scheme, ess_min, q_var, r_var, x0[0], x0[1], v0[0], v0[1], c->world, (int)c->timing);
    // the graph bakes column buffers: key on their addresses too
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* q) { h = (h ^ (uint64_t)(uintptr_t)q) * 1099511628211ull; };
    for (auto& col : c->cols) { mix(col.front); mix(col.back); }
    mix(c->w); mix(c->anc_log); mix(c->run_rec); mix(c->run_max); mix(c->obs);
    mix(c->comm);   // a captured collective bakes its communicator
    // exact shards: the run without host round trips unless it is switched off (A/B) or the
    // scheme needs the eager path; its block / window sizes are part of the graph
    // a caller's host transport (wsmc_comm_init_host: a test vehicle, every exchange a host
    // round trip) ships the async run's fixed blocks of cap slots every step; the eager path
    // ships only the slots that move, so it runs there
    const bool exact_async = exact_mode(c) && !exact_eager_forced() && !c->x_eager &&
                             (!c->host_exchange || c->host_inproc);
    int64_t xcap = 0, xctr = 0;
    if (exact_async) {
        exact_sizes(c, &xcap, &xctr);
        if ((r = ensure_exact_async(c, T, xcap, xctr))) return r;
        const void* xb[] = {c->xpairs, c->xnb, c->xwin, c->xstat, c->w_save, c->xms, c->xanc, c->xlines, c->taskTile, c->xp,
                            c->comb, c->rec, c->tilep, c->tileOff, c->qbuf, c->taskOff};
        for (const void* q : xb) mix(q);
    }
    const std::string key = std::string(keybuf) + " ptr=" + std::to_string(h) +
                            (exact_async ? " exact cap=" + std::to_string(xcap) + " ctr=" + std::to_string(xctr) +
                                               " trace=" + std::to_string((int)c->x_trace)
                                         : "");
    auto build_tables = [&](double*** work, double*** outp) -> int {
        *work = *outp = nullptr;
        if (!p.keep) return WSMC_OK;
        std::vector<double*> hw(T + 2, nullptr), ho(T + 2, nullptr);
        for (int t = 1; t <= T + 1; ++t) {
            hw[t] = c->cols[p.xcols[t]].back;
            ho[t] = c->cols[p.xcols[t]].front;
        }
        double** tabs = nullptr;
        WSMC_HIP(hipMalloc(&tabs, sizeof(double*) * 2 * (T + 2)));
        WSMC_HIP(hipMemcpyAsync(tabs, hw.data(), sizeof(double*) * (T + 2), hipMemcpyHostToDevice, c->stream));
        WSMC_HIP(hipMemcpyAsync(tabs + (T + 2), ho.data(), sizeof(double*) * (T + 2), hipMemcpyHostToDevice,
                                c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        *work = tabs;
        *outp = tabs + (T + 2);
        return WSMC_OK;
    };
    // HIP cannot time events captured in graphs; a host exchange (test mode) synchronises
    // inside the run, and exact shards are host-driven. RCCL collectives are captured.
    const bool use_graph = !c->timing && !no_graph && !c->no_graph && (!exact_mode(c) || exact_async) &&
                           !c->host_exchange;
    if (exact_mode(c) && c->timing) return fail(WSMC_ESTATE, "run timing is not available on exact shards");
    const int nev = 8 * T + 2;
    std::vector<hipEvent_t> evs;
    if (c->timing) {
        while ((int)c->events.size() < nev) {
            hipEvent_t e;
            WSMC_HIP(hipEventCreate(&e));
            c->events.push_back(e);
        }
        evs.assign(c->events.begin(), c->events.begin() + nev);
    }
    void* temp_tables = nullptr;
    auto enqueue_run = [&]() {
        return exact_async ? enqueue_ssm2d_exact(c, p, xcap, xctr) : enqueue_ssm2d(c, p, c->timing ? &evs : nullptr);
    };
    if (exact_mode(c) && !exact_async) {
        if ((r = ssm2d_run_exact(c, p, op_base))) return r;
    } else {
        bool graphed = false;
        if (use_graph) {
            RunGraph* g = nullptr;
            for (auto& gg : c->graphs)
                if (gg.key == key) g = &gg;
            if (!g) {
                RunGraph ng;
                ng.key = key;
                if ((r = build_tables(&p.d_hist_work, &p.d_hist_out))) return r;
                ng.owned = p.d_hist_work;
                WSMC_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
                r = enqueue_run();
                static const bool diag_fail = [] {   // diagnostics: exercise the eager fallback
                    const char* e = getenv("WSMC_DIAG_CAPTURE_FAIL");
                    return e && atoi(e) != 0;
                }();
                if (!r && diag_fail) r = fail(WSMC_EHIP, "diagnostic capture failure");
                hipGraph_t graph = nullptr;
                hipError_t ee = hipStreamEndCapture(c->stream, &graph);
                hipGraphExec_t exec = nullptr;
                if (!r && ee == hipSuccess) ee = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
                if (r || ee != hipSuccess) {
                    if (graph) (void)hipGraphDestroy(graph);
                    if (ng.owned) (void)hipFree(ng.owned);
                    p.d_hist_work = p.d_hist_out = nullptr;
                    if (!is_sharded(c)) {
                        if (r) return r;
                        WSMC_HIP(ee);
                    }
                    // a sharded run whose collectives would not capture runs eagerly from now on
                    (void)hipGetLastError();
                    std::fprintf(stderr, "wsmc: capturing the sharded run failed (%s); running it eagerly\n",
                                 r ? wsmc_last_error() : hipGetErrorString(ee));
                    c->no_graph = true;
                } else {
                    ng.graph = graph;
                    ng.exec = exec;
                    c->graphs.push_back(ng);
                    g = &c->graphs.back();
                }
            }
            if (g) {
                WSMC_HIP(hipGraphLaunch(g->exec, c->stream));
                graphed = true;
            }
        }
        if (!graphed) {
            if ((r = build_tables(&p.d_hist_work, &p.d_hist_out))) return r;
            temp_tables = p.d_hist_work;
            // instrumented runs: a bounded delay kernel keeps the GPU busy while the host
            // queues the whole run, so no host-submission gap lands inside an event pair
            if (c->timing) WSMC_HIP(launch_delay(c->stream, 20000));
            r = enqueue_run();
            if (r) {
                if (temp_tables) (void)hipFree(temp_tables);
                return r;
            }
        }
    }
    if (async_run) {
        // the trace-back kernel wrote the decisions into this parity's pinned slots and the last
        // resampled row into the last-ancestors buffer
        WSMC_HIP(hipEventRecord(c->run_ev[par], c->stream));
        run_book(c, p, obs);
        RunPend* P = new RunPend;
        P->par = par;
        P->p = p;
        P->p.d_hist_work = P->p.d_hist_out = nullptr;
        P->op_base = op_base;
        P->hobs = std::move(hobs);
        P->guessed = !is_sharded(c) && p.scheme != WSMC_RESAMPLE_MULTINOMIAL && run_qstat_mode(c->N) != 0;
        P->temp_tables = temp_tables;
        RunPend* prev = c->run_pend;
        c->run_pend = P;
        if (prev) return fold_run(c, prev, P);
        return WSMC_OK;
    }
    bool rows_x = exact_async;   // the ancestor rows are the exact run's (not the eager re-run's)
    if (exact_async) {
        // every rank's overflow statistics (all-gathered by the run): the same on all ranks, so
        // all of them re-run on the eager path together, from the weights the run started with
        std::vector<unsigned long long> st((size_t)kMaxShards * kXStat);
        WSMC_HIP(hipMemcpyAsync(st.data(), c->xstat, sizeof(unsigned long long) * st.size(), hipMemcpyDeviceToHost,
                                c->stream));
        WSMC_HIP(ctx_sync(c, c->stream));
        unsigned long long bits = 0, need = 0, exc = 0;
        for (int g = 0; g < c->world; ++g) {
            bits |= st[(size_t)g * kXStat];
            need = std::max(need, st[(size_t)g * kXStat + 1]);
            exc = std::max(exc, st[(size_t)g * kXStat + 2]);
        }
        c->x_need = need;
        c->x_exc = exc;
        c->x_overflows += bits ? 1 : 0;
        const int64_t nmax = (c->gN + c->world - 1) / c->world;
        // trace windows cost T x ctr x 24 B a side every run, the distributed trace one range
        // exchange a level: windows grow at most to 4x their default, past that (lineages
        // wander far: coalescence) they are dropped and the history is traced across ranks
        auto grow_windows = [&]() {
            int64_t d_cap = 0, d_ctr = 0;
            const int64_t saved = c->x_ctr;
            c->x_ctr = 0;
            exact_sizes(c, &d_cap, &d_ctr);
            c->x_ctr = saved;
            const int64_t grown = std::min<int64_t>(nmax, std::max<int64_t>(4 * xctr, 2 * (int64_t)exc));
            if (grown > 4 * d_ctr || 2 * grown >= nmax)
                c->x_trace = true;
            else
                c->x_ctr = grown;
        };
        if (!(bits & 1ull) && need > 0 && 8 * (int64_t)need < xcap && xcap > 256) {
            // the blocks ship cap slots a side every step whatever moves: shrink them toward
            // the need (4x margin, a power of two, so a captured graph is rebuilt rarely)
            int64_t cp = 256;
            while (cp < 4 * (int64_t)need) cp *= 2;
            c->x_cap = cp;
        }
        if (bits & 1ull) {
            // a block overflowed: particles are missing, re-run the filter on the eager path.
            // Grown for the next runs, never past a shard (a block cannot need more than a
            // neighbour's particles); blocks of half a shard or more would ship most of a
            // neighbour's state every step: the eager path's exchanges cost less from then on
            c->x_cap = std::min<int64_t>(nmax, std::max<int64_t>(4 * xcap, 2 * (int64_t)need));
            if (bits & 2ull) grow_windows();
            if (2 * c->x_cap >= nmax) c->x_eager = true;
            WSMC_HIP(hipMemcpyAsync(c->w, c->w_save, sizeof(double) * c->N, hipMemcpyDeviceToDevice, c->stream));
            rows_x = false;
            if ((r = ssm2d_run_exact(c, p, op_base))) {
                if (temp_tables) (void)hipFree(temp_tables);
                return r;
            }
        } else if (bits & 2ull) {
            // only the trace windows overflowed: the filter is right, the history is traced
            // across ranks now
            grow_windows();
            if ((r = exact_trace_history(c, p, xcap))) {
                if (temp_tables) (void)hipFree(temp_tables);
                return r;
            }
        }
    }
    // the decisions: exact shards copy them back; every other run's trace-back kernel wrote them
    // into this parity's pinned slots (and the last resampled row into c->anc)
    const bool kernel_rb = !exact_mode(c);
    const Decision* hd = c->run_hdec + (size_t)par * (c->T_alloc + 1);
    std::vector<Decision> hdec(T + 1);
    if (!kernel_rb)
        WSMC_HIP(hipMemcpyAsync(hdec.data(), c->run_dec, sizeof(Decision) * (T + 1), hipMemcpyDeviceToHost, c->stream));
    WSMC_HIP(ctx_sync(c, c->stream));
    if (kernel_rb) std::memcpy(hdec.data(), hd, sizeof(Decision) * (T + 1));
    if (temp_tables) (void)hipFree(temp_tables);
    temp_tables = nullptr;
    if (hdec[0].ntasks > 0 && !exact_mode(c)) {
        // a step's guessed reference point missed (the max and its bound straddle an integer, an
        // outlier observation): the run is re-done from the weights it started with, every step
        // taking its statistics against the exact max — the canonical bits, as if never guessed
        c->run_missed += hdec[0].ntasks;
        c->run_replays += 1;
        WSMC_HIP(hipMemcpyAsync(c->w, c->run_w0 + (size_t)par * c->N, sizeof(double) * c->N, hipMemcpyDeviceToDevice,
                                c->stream));
        p.exact_stats = true;
        if ((r = build_tables(&p.d_hist_work, &p.d_hist_out))) return r;
        temp_tables = p.d_hist_work;
        r = enqueue_ssm2d(c, p, nullptr);
        if (!r) {
            r = ctx_sync(c, c->stream) == hipSuccess ? WSMC_OK : fail(WSMC_EHIP, "replay sync failed");
            if (!r) std::memcpy(hdec.data(), hd, sizeof(Decision) * (T + 1));
        }
        (void)hipFree(temp_tables);
        temp_tables = nullptr;
        if (r) return r;
    }
    // wsmc_last_ancestors reports the run's last resample, as after the statement sequence
    for (int t = T; t >= 1; --t)
        if (hdec[t].resampled) {
            if (!kernel_rb) {
                const int32_t* src = rows_x ? c->xanc + (size_t)(t - 1) * c->xanc_stride + xcap
                                            : c->anc_log + (size_t)(t - 1) * anc_stride(c->N);
                WSMC_HIP(hipMemcpyAsync(c->anc, src, sizeof(int32_t) * c->N, hipMemcpyDeviceToDevice, c->stream));
            }
            set_anc_last(c, nullptr, -1);
            break;
        }
    run_book(c, p, obs);
    run_fold_decisions(c, hdec.data(), T);
    if (c->timing) {
        int32_t nres = 0;
        for (int t = 1; t <= T; ++t) nres += hdec[t].resampled ? 1 : 0;
        wsmc_run_timing tm{};
        float ms = 0.f;
        for (int t = 1; t <= T; ++t) {
            const int k = 8 * (t - 1);
            WSMC_HIP(hipEventElapsedTime(&ms, evs[k], evs[k + 1]));
            tm.propagate_ms += ms;
            WSMC_HIP(hipEventElapsedTime(&ms, evs[k + 2], evs[k + 3]));
            tm.reduce_ms += ms;
            WSMC_HIP(hipEventElapsedTime(&ms, evs[k + 6], evs[k + 7]));
            tm.resample_ms += ms;
        }
        WSMC_HIP(hipEventElapsedTime(&ms, evs[8 * T], evs[8 * T + 1]));
        tm.finalize_ms = ms;
        WSMC_HIP(hipEventElapsedTime(&ms, evs[0], evs[8 * T + 1]));
        tm.total_ms = ms;
        tm.steps = T;
        tm.n_resamples = nres;
        c->last_timing = tm;
    }
    if (log_evidence_out) return wsmc_log_evidence(c, log_evidence_out);
    return WSMC_OK;
}

// the decision-independent bookkeeping of a run: the state issuing the statements one by one
// leaves (columns current, the score tape, depth, op counter)
static void run_book(wsmc_ctx* c, const RunPlan& p, const double* obs) {
    const int T = p.T;
    // the run wrote its columns in full (traced back): current
    if (p.keep) {
        for (int t = 1; t <= T + 1; ++t) wrote_col(c, p.xcols[t]);
    } else {
        wrote_col(c, p.colx);
    }
    wrote_col(c, p.colv);
    wrote_col(c, p.coldv);
    gc_log(c);

    // bookkeeping identical to issuing the statements one by one
    const uint64_t op_base = c->op;
    c->depth += 2;  // x{1} .= x0, v .= v0
    for (int t = 1; t <= T; ++t) {
        wsmc_dist dv;
        std::memset(&dv, 0, sizeof(dv));
        dv.family = WSMC_FAM_MVNORMAL_ISO;
        dv.mean_fn = WSMC_MEAN_AFFINE;
        dv.dim = 2;
        for (int k = 0; k < 4; ++k) {
            dv.mu[k].col[0] = dv.mu[k].col[1] = -1;
        }
        dv.scale.c0 = p.q_var;
        dv.scale.col[0] = dv.scale.col[1] = -1;
        c->depth += 1;  // x{t+1} .= x{t} + v
        push_sample_term(c, p.coldv, dv);
        c->depth += 1;  // dv ~ ...
        c->depth += 1;  // v .= v + dv
        wsmc_term ob;
        std::memset(&ob, 0, sizeof(ob));
        ob.dist.family = WSMC_FAM_MVNORMAL_ISO;
        ob.dist.mean_fn = WSMC_MEAN_AFFINE;
        ob.dist.dim = 2;
        const int32_t xc = p.keep ? p.xcols[t + 1] : p.colx;
        for (int k = 0; k < 4; ++k) ob.dist.mu[k] = col_operand(k < 2 ? xc : -1, k);
        ob.dist.scale.c0 = p.r_var;
        ob.dist.scale.col[0] = ob.dist.scale.col[1] = -1;
        for (int k = 0; k < 4; ++k) {
            std::memset(&ob.x[k], 0, sizeof(wsmc_operand));
            ob.x[k].c0 = k < 2 ? obs[2 * (t - 1) + k] : 0.0;
            ob.x[k].col[0] = ob.x[k].col[1] = -1;
        }
        ob.kind = WSMC_TERM_OBSERVE;
        ob.depth = c->depth;
        c->tape.push_back(ob);
        c->depth += 1;  // o => ...
    }
    c->op = op_base + 3ull * (uint64_t)T;
    c->weights_changed = 0;
    c->colptr_dirty = true;
}

// the decision-dependent part, from the run's decisions [T+1] on the host
static void run_fold_decisions(wsmc_ctx* c, const Decision* hdec, int T) {
    int32_t nres = 0;
    for (int t = 1; t <= T; ++t) nres += hdec[t].resampled ? 1 : 0;
    c->resampled = hdec[T].resampled;
    c->last_ess = hdec[T].ess;
    c->n_resamples += nres;
    if (nres) set_anc_last(c, nullptr, -1);   // the last resampled row is in c->anc
}

// a run's history tables (x_t working / output buffers by step), uploaded (synchronous)
static int build_run_tables(wsmc_ctx* c, RunPlan& p) {
    p.d_hist_work = p.d_hist_out = nullptr;
    if (!p.keep) return WSMC_OK;
    const int T = p.T;
    std::vector<double*> hw(T + 2, nullptr), ho(T + 2, nullptr);
    for (int t = 1; t <= T + 1; ++t) {
        hw[t] = c->cols[p.xcols[t]].back;
        ho[t] = c->cols[p.xcols[t]].front;
    }
    double** tabs = nullptr;
    WSMC_HIP(hipMalloc(&tabs, sizeof(double*) * 2 * (T + 2)));
    WSMC_HIP(hipMemcpy(tabs, hw.data(), sizeof(double*) * (T + 2), hipMemcpyHostToDevice));
    WSMC_HIP(hipMemcpy(tabs + (T + 2), ho.data(), sizeof(double*) * (T + 2), hipMemcpyHostToDevice));
    p.d_hist_work = tabs;
    p.d_hist_out = tabs + (T + 2);
    return WSMC_OK;
}

// an event's wait, bounded like ctx_sync's (a peer's abort, the communicator watchdog)
static hipError_t ev_sync(wsmc_ctx* c, hipEvent_t ev) {
    const bool watch = c->comm && c->comm_timeout_s > 0.0;
    if (!c->peer_abort && !watch) return hipEventSynchronize(ev);
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        if (peer_aborted(c)) return ctx_sync(c, c->stream);
        if (watch && (spin & 255) == 255 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->comm_timeout_s)
            return ctx_sync(c, c->stream);   // (aborts the communicator past the same bound)
        if (spin < 4096)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// re-do a run on the exact path (every step's statistics against the exact max), synchronously:
// from the weights it started with (restore_w) or from the current ones (the run after a re-done
// one); its decisions into its parity's pinned slots
static int replay_run(wsmc_ctx* c, RunPend* R, bool restore_w) {
    const int T = R->p.T;
    if (restore_w)
        WSMC_HIP(hipMemcpyAsync(c->w, c->run_w0 + (size_t)R->par * c->N, sizeof(double) * c->N,
                                hipMemcpyDeviceToDevice, c->stream));
    c->obs = c->obs_buf + (size_t)R->par * 2 * (c->T_alloc + 1);
    c->run_op = c->run_params + 4 * R->par;
    WSMC_HIP(ctx_sync(c, c->stream));   // (nothing in flight reads the staging now)
    run_stage_fill(c, R->par, R->op_base, R->hobs.data(), T);
    RunPlan p = R->p;
    p.exact_stats = true;
    if (int r = build_run_tables(c, p)) return r;
    // the head copies the staging in; the trace-back writes the decisions and the last row
    int r = enqueue_ssm2d(c, p, nullptr);
    if (!r && ctx_sync(c, c->stream) != hipSuccess) r = fail(WSMC_EHIP, "replay sync failed");
    if (p.d_hist_work) (void)hipFree(p.d_hist_work);
    return r;
}

static int fold_run(wsmc_ctx* c, RunPend* P, RunPend* Q) {
    std::unique_ptr<RunPend> own(P);
    WSMC_HIP(ev_sync(c, c->run_ev[P->par]));
    if (P->temp_tables) {
        (void)hipFree(P->temp_tables);
        P->temp_tables = nullptr;
    }
    const Decision* hd = c->run_hdec + (size_t)P->par * (c->T_alloc + 1);
    if (P->guessed && hd[0].ntasks > 0) {
        c->run_missed += hd[0].ntasks;
        c->run_replays += 1;
        WSMC_HIP(ctx_sync(c, c->stream));   // (the run after it, if any, ends too)
        if (int r = replay_run(c, P, true)) return r;
        if (Q) {
            if (int r = replay_run(c, Q, false)) return r;
            Q->guessed = false;   // folded later from its replayed decisions
        }
    }
    run_fold_decisions(c, hd, P->p.T);
    return WSMC_OK;
}

static int resolve_run(wsmc_ctx* c) {
    if (!c->run_pend) return WSMC_OK;
    RunPend* P = c->run_pend;
    c->run_pend = nullptr;
    return fold_run(c, P, nullptr);
}
static void run_pend_free(RunPend* r) {
    if (r && r->temp_tables) (void)hipFree(r->temp_tables);
    delete r;
}

int wsmc_debug_exact(wsmc_ctx* c, int64_t cap, int64_t ctr, int64_t* stats_out) {
    if (c && c->multi) {
        int64_t st[6];
        int r = multi_each(c, [&](wsmc_ctx* x) { return wsmc_debug_exact(x, cap, ctr, x == multi_first(c) ? st : nullptr); });
        if (!r && stats_out) std::memcpy(stats_out, st, sizeof(st));
        return r;
    }
    if (!c) return fail(WSMC_EARG, "null context");
    if (cap >= 0) c->x_cap = cap;
    if (ctr >= 0) c->x_ctr = ctr;
    if (cap >= 0 || ctr >= 0) c->x_eager = c->x_trace = false;   // margins set by hand: the async run again
    if (stats_out) {
        int64_t cp = 0, ct = 0;
        if (c->world > 0 && c->gN > 0) exact_sizes(c, &cp, &ct);
        stats_out[0] = (int64_t)c->x_need;
        stats_out[1] = (int64_t)c->x_exc;
        stats_out[2] = c->x_overflows - c->x_traces;
        stats_out[3] = cp;
        stats_out[4] = c->x_traces;
        stats_out[5] = c->x_trace ? 1 : 0;
    }
    return WSMC_OK;
}

int wsmc_debug_inject_failure(wsmc_ctx* c, int32_t shard, int32_t nth) {
    if (c && c->multi) return multi_inject_failure(c, shard, nth);
    if (!c) return fail(WSMC_EARG, "null context");
    if (shard != 0 || nth < 0) return fail(WSMC_EARG, "bad shard or count");
    c->inject_earg = nth >= 1000;
    c->inject_fail = nth >= 1000 ? nth - 1000 : nth;
    return WSMC_OK;
}

int wsmc_debug_kernel_bench(wsmc_ctx* c, int32_t kernel, int32_t mode, int32_t iters, double* avg_us) {
    if (c && c->multi) return multi_G(c) == 1 ? wsmc_debug_kernel_bench(multi_first(c), kernel, mode, iters, avg_us) : fail(WSMC_EARG, "diagnostics need one shard");
    CHECK_CTX(c);
    if (!avg_us || iters < 1) return fail(WSMC_EARG, "bad arguments");
    // populate max slots / partials / offsets / record from the current weights; force a resample
    WSMC_HIP(hipMemsetAsync(c->mslots, 0, sizeof(MaxSlots), c->stream));
    WSMC_HIP(launch_rs_max(c->stream, c->w, c->N, c->mslots));
    WSMC_HIP(launch_rs_sums(c->stream, c->w, c->N, c->mslots, c->tilep, c->qbuf));
    const FillPlan plan = fill_plan(c, WSMC_RESAMPLE_STRATIFIED, c->op, nullptr);
    WSMC_HIP(launch_rs_reduce(c->stream, c->mslots, c->tilep, c->N, c->tileOff, c->rec, 1, 2.0, c->dec, &plan));
    double* stream4 = nullptr;
    if (kernel == 3) WSMC_HIP(hipMalloc(&stream4, sizeof(double) * 8 * (size_t)c->N));
    if (stream4) WSMC_HIP(hipMemsetAsync(stream4, 0, sizeof(double) * 8 * (size_t)c->N, c->stream));
    float ms = 0.f;
    const hipError_t e = debug_kernel_bench(c->stream, kernel, mode, iters, c->w, c->N, c->mslots, c->tilep, c->qbuf,
                                            c->tileOff, c->rec, c->dec, plan, c->anc, stream4, &ms);
    if (stream4) (void)hipFree(stream4);
    WSMC_HIP(e);
    *avg_us = 1e3 * ms / iters;
    return WSMC_OK;
}

}  // extern "C"

int wsmc_debug_jit_stats(int64_t* stats_out) {
    if (!stats_out) return fail(WSMC_EARG, "null stats_out");
    ew_jit_stats(stats_out);
    return WSMC_OK;
}

int wsmc_debug_run_stats(wsmc_ctx* c, int64_t* stats_out) {
    if (c && c->multi) return wsmc_debug_run_stats(multi_first(c), stats_out);
    if (!c || !stats_out) return fail(WSMC_EARG, "null argument");
    unsigned long long nfix = 0;
    if (c->run_nfix) {
        WSMC_HIP(ctx_sync(c, c->stream));
        WSMC_HIP(hipMemcpy(&nfix, c->run_nfix, sizeof(nfix), hipMemcpyDeviceToHost));
    }
    stats_out[0] = (int64_t)nfix + c->run_missed;
    stats_out[1] = run_qstat_mode(c->N);
    stats_out[2] = c->run_replays;
    stats_out[3] = c->rs_qs_batches;
    return WSMC_OK;
}

int wsmc_debug_mv_jit_stats(int64_t* stats_out) {
    if (!stats_out) return fail(WSMC_EARG, "null stats_out");
    mv_jit_stats(stats_out);
    return WSMC_OK;
}

int wsmc_debug_mv_jit_selfcheck(void) {
    std::string err;
    if (mv_jit_selfcheck(err)) return fail(WSMC_EHIP, "Move-block JIT: " + err);
    return WSMC_OK;
}

int wsmc_debug_log_screen(const double* u, int64_t n, double* out) {
    if (!u || !out || n < 0) return fail(WSMC_EARG, "null buffer or n < 0");
    if (n == 0) return WSMC_OK;
    double *du = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc(&du, n * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&dout, 2 * n * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(du, u, n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_debug_log_screen(nullptr, du, n, dout);
    if (e == hipSuccess) e = hipMemcpy(out, dout, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
    hipFree(du);
    hipFree(dout);
    return e == hipSuccess ? WSMC_OK : fail(WSMC_EHIP, std::string("log screen: ") + hipGetErrorString(e));
}

int wsmc_debug_jit_selfcheck(void) {
    std::string err;
    if (ew_jit_selfcheck(err)) return fail(WSMC_EHIP, "statement-batch JIT: " + err);
    return WSMC_OK;
}
