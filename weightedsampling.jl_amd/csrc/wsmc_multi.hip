// wsmc_multi.hip — one handle over several devices (`wsmc_create(…, n_gpus, …)`,
// "multi-GPU inside one context"), so a single-threaded host — the reference's model,
// src/types.jl:24-26 — can hold one SMCState spanning the node without an MPI launcher.
//
// The population [0, N) is split into G contiguous shards [N g / G, N (g+1) / G); shard g is an ordinary sharded context on its device, exactly what one
// process per GPU would create (wsmc_comm_init / wsmc_comm_init_host), so every sharded code
// path and its bit-exactness carry over unchanged. A call on the handle fans out to one host
// thread per shard (persistent workers; shard 0 runs on the caller's thread): each shard
// issues its own RCCL collectives from its own thread, as one process per GPU would, and
// the collectives of the G shards meet. Host buffers of N particles are split by shard on the
// way in and joined on the way out; population-wide results (evidence, ESS, moments, median,
// histogram, diversity, sample, flags) are identical on every shard and taken from shard 0.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "wsmc_internal.h"

namespace wsmc {

struct MultiState;

namespace {

struct Worker {
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    std::function<void()> job;
    bool has = false, done = false, quit = false;
};

struct XArg {
    MultiState* M;
    int rank;
};

}  // namespace

struct MultiState {
    int G = 1;
    int64_t N = 0;
    std::vector<int64_t> off;          // shard g = [off[g], off[g+1])
    std::vector<wsmc_ctx*> sub;
    std::vector<std::unique_ptr<Worker>> workers;   // workers[g] for g >= 1
    // in-process record exchange (transport 1)
    std::mutex xm;
    std::condition_variable xcv;
    int arrived = 0, departed = 0;
    uint64_t gen_in = 0, gen_out = 0;
    std::vector<uint64_t> xbuf;
    std::vector<XArg> xargs;
    // A shard that fails by itself during a fan-out (a HIP or exchange failure: its peers may
    // be waiting in a collective for it) sets `abort`: shards waiting in the host exchange leave
    // it with an error, and RCCL shards abort their own communicators (each from its own thread,
    // before its next collective or while it waits for its stream: a collective missing its
    // peer would never complete) and leave with WSMC_ERCCL. An error every shard meets at the
    // same point — an argument error before any collective, a population-wide not-PD
    // covariance after the same collectives — sets nothing: the failing shard waits for its
    // peers (at most kPeerWaitS, then it requests the abort after all). Shards that left the
    // call with different results may hold different states: the handle is marked failed.
    bool rccl = false;
    std::atomic<bool> abort{false};   // written under xm
    int finished = 0;                 // shards back from this fan-out's call (guarded by xm)
    bool failed = false;              // set between fan-outs only
};

// seconds a shard that met a symmetric error waits for its peers before requesting the abort
constexpr double kPeerWaitS = 30.0;
// errors every shard meets at the same point: an argument error before the call's first
// exchange (validation, the same arguments on every shard), and a not-PD autoRW covariance (it
// is factored from all-gathered totals, so every shard computes the same); anything else a shard
// meets alone — an argument error past an exchange included — requests the abort at once
static bool symmetric_error(const wsmc_ctx* s, int code) {
    return code == WSMC_ENOTPD || (code == WSMC_EARG && s->exchanges == 0);
}

static void worker_loop(Worker* w) {
    for (;;) {
        std::function<void()> job;
        {
            std::unique_lock<std::mutex> lk(w->m);
            w->cv.wait(lk, [&] { return w->has || w->quit; });
            if (w->quit && !w->has) return;
            job = std::move(w->job);
            w->has = false;
        }
        job();
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->done = true;
        }
        w->cv.notify_all();
    }
}

// a shard failed by itself: release the shards waiting for it in the host exchange, and ask
// the RCCL shards to abort their communicators (they do it on their own threads)
static void request_abort(MultiState* M) {
    std::lock_guard<std::mutex> lk(M->xm);
    if (M->abort.load()) return;
    M->abort.store(true, std::memory_order_release);
    M->xcv.notify_all();
}

// shard g is back from its call with code rc
static void shard_done(MultiState* M, int g, int rc) {
    const bool sym = symmetric_error(M->sub[g], rc);
    if (rc && !sym && M->G > 1) request_abort(M);   // one shard: no peer waits for it
    bool wait_peers = false;
    {
        std::lock_guard<std::mutex> lk(M->xm);
        M->finished += 1;
        M->xcv.notify_all();
        wait_peers = rc && sym && M->G > 1;
    }
    if (!wait_peers) return;
    // every shard should meet the same error at the same point: wait for them, and abort the
    // call after all if one is still inside it (then it was waiting for this shard)
    std::unique_lock<std::mutex> lk(M->xm);
    const bool all = M->xcv.wait_for(lk, std::chrono::duration<double>(kPeerWaitS),
                                     [&] { return M->finished == M->G || M->abort.load(); });
    lk.unlock();
    if (!all) {
        fprintf(stderr, "[wsmc multi] shard %d met error %d and its peers did not return within %.0f s: aborting\n",
                g, rc, kPeerWaitS);
        request_abort(M);
    }
}

// fn(g, shard) on every shard concurrently; the first failing shard's code and message
static int run_all(MultiState* M, const std::function<int(int, wsmc_ctx*)>& fn) {
    if (M->failed) return fail(WSMC_ESTATE, "multi-device handle failed in an earlier call (its shards diverged)");
    {
        std::lock_guard<std::mutex> lk(M->xm);
        M->abort.store(false);
        M->arrived = M->departed = 0;
        M->finished = 0;
    }
    for (auto* s : M->sub) {
        s->released = false;
        s->exchanges = 0;   // this call's exchanges
    }
    std::vector<int> rc(M->G, 0);
    std::vector<std::string> msg(M->G);
    for (int g = 1; g < M->G; ++g) {
        Worker* w = M->workers[g].get();
        std::lock_guard<std::mutex> lk(w->m);
        w->job = [&, g] {
            rc[g] = fn(g, M->sub[g]);
            if (rc[g]) msg[g] = wsmc_last_error();
            shard_done(M, g, rc[g]);
        };
        w->has = true;
        w->done = false;
        w->cv.notify_all();
    }
    rc[0] = fn(0, M->sub[0]);
    if (rc[0]) msg[0] = wsmc_last_error();
    shard_done(M, 0, rc[0]);
    for (int g = 1; g < M->G; ++g) {
        Worker* w = M->workers[g].get();
        std::unique_lock<std::mutex> lk(w->m);
        w->cv.wait(lk, [&] { return w->done; });
    }
    if (M->abort.load() && M->rccl) {
        // every thread is back: the communicators no shard aborted (shards that had finished
        // before the request) are aborted here, and the handle is done with RCCL
        for (auto* s : M->sub)
            if (s->comm) {
                (void)ncclCommAbort(s->comm);
                s->comm = nullptr;
            }
        M->failed = true;
    }
    bool same = true;
    for (int g = 1; g < M->G; ++g) same &= rc[g] == rc[0];
    if (!same) M->failed = true;
    // report the first shard that failed by itself, not one released by the abort
    for (int pass = 0; pass < 2; ++pass)
        for (int g = 0; g < M->G; ++g)
            if (rc[g] && (pass == 1 || (rc[g] != WSMC_ERCCL && !M->sub[g]->released)))
                return fail(rc[g], "shard " + std::to_string(g) + ": " + msg[g]);
    return WSMC_OK;
}

// all-gather of one u64 record per shard through host memory (the shards are threads of this
// process): a two-phase barrier so no shard overwrites the buffer before every shard copied it
static int multi_exchange(void* user, const uint64_t* mine, int32_t words, uint64_t* all) {
    XArg* a = static_cast<XArg*>(user);
    MultiState* M = a->M;
    std::unique_lock<std::mutex> lk(M->xm);
    if (M->xbuf.size() < (size_t)M->G * (size_t)words) M->xbuf.resize((size_t)M->G * (size_t)words);
    std::memcpy(M->xbuf.data() + (size_t)a->rank * words, mine, sizeof(uint64_t) * (size_t)words);
    const uint64_t g_in = M->gen_in;
    if (M->abort) return -1;
    if (++M->arrived == M->G) {
        M->arrived = 0;
        M->gen_in += 1;
        M->xcv.notify_all();
    } else {
        M->xcv.wait(lk, [&] { return M->gen_in != g_in || M->abort; });
        if (M->gen_in == g_in) return -1;   // a shard failed before arriving
    }
    std::memcpy(all, M->xbuf.data(), sizeof(uint64_t) * (size_t)M->G * (size_t)words);
    const uint64_t g_out = M->gen_out;
    if (++M->departed == M->G) {
        M->departed = 0;
        M->gen_out += 1;
        M->xcv.notify_all();
    } else {
        M->xcv.wait(lk, [&] { return M->gen_out != g_out || M->abort; });
        if (M->gen_out == g_out) return -1;
    }
    return 0;
}

static inline int64_t nloc(const MultiState* M, int g) { return M->off[g + 1] - M->off[g]; }

// [dim][N] host <-> per-shard [dim][n_g]
static void split_rows(const MultiState* M, int g, const double* host, int dim, std::vector<double>& out) {
    const int64_t n = nloc(M, g);
    out.resize((size_t)dim * n);
    for (int k = 0; k < dim; ++k)
        std::memcpy(out.data() + (size_t)k * n, host + (size_t)k * M->N + M->off[g], sizeof(double) * n);
}
static void join_rows(const MultiState* M, int g, const std::vector<double>& in, int dim, double* host) {
    const int64_t n = nloc(M, g);
    for (int k = 0; k < dim; ++k)
        std::memcpy(host + (size_t)k * M->N + M->off[g], in.data() + (size_t)k * n, sizeof(double) * n);
}

int multi_destroy(wsmc_ctx* c) {
    MultiState* M = c->multi;
    for (int g = 1; g < M->G; ++g) {
        Worker* w = M->workers[g].get();
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->quit = true;
        }
        w->cv.notify_all();
        if (w->th.joinable()) w->th.join();
    }
    for (auto* s : M->sub)
        if (s) wsmc_destroy(s);
    delete M;
    delete c;
    return WSMC_OK;
}

}  // namespace wsmc

using namespace wsmc;

// ---- the per-function fan-out (called from the ABI entry points when ctx->multi) -------------
namespace wsmc {

wsmc_ctx* multi_first(wsmc_ctx* c) { return c->multi->sub[0]; }
int multi_G(wsmc_ctx* c) { return c->multi->G; }
int multi_sync(wsmc_ctx* c) { return run_all(c->multi, [](int, wsmc_ctx* s) { return wsmc_sync(s); }); }
int multi_get_state(wsmc_ctx* c, wsmc_state* out) {
    std::vector<wsmc_state> st(c->multi->G);
    int r = run_all(c->multi, [&](int g, wsmc_ctx* s) { return wsmc_get_state(s, &st[g]); });
    if (!r) *out = st[0];
    return r;
}
int multi_each(wsmc_ctx* c, const std::function<int(wsmc_ctx*)>& f) {
    return run_all(c->multi, [&](int, wsmc_ctx* s) { return f(s); });
}
int multi_col_download(wsmc_ctx* c, int32_t col, double* host) {
    MultiState* M = c->multi;
    int32_t dim = 0;
    int r = wsmc_col_info(M->sub[0], col, nullptr, 0, &dim);
    if (r) return r;
    std::vector<std::vector<double>> buf(M->G);
    r = run_all(M, [&](int g, wsmc_ctx* s) {
        buf[g].resize((size_t)dim * nloc(M, g));
        return wsmc_col_download(s, col, buf[g].data());
    });
    if (r) return r;
    for (int g = 0; g < M->G; ++g) join_rows(M, g, buf[g], dim, host);
    return WSMC_OK;
}
int multi_col_upload(wsmc_ctx* c, int32_t col, const double* host) {
    MultiState* M = c->multi;
    int32_t dim = 0;
    int r = wsmc_col_info(M->sub[0], col, nullptr, 0, &dim);
    if (r) return r;
    std::vector<std::vector<double>> buf(M->G);
    for (int g = 0; g < M->G; ++g) split_rows(M, g, host, dim, buf[g]);
    return run_all(M, [&](int g, wsmc_ctx* s) { return wsmc_col_upload(s, col, buf[g].data()); });
}
int multi_weights(wsmc_ctx* c, const double* up, double* down) {
    MultiState* M = c->multi;
    std::vector<std::vector<double>> buf(M->G);
    if (up)
        for (int g = 0; g < M->G; ++g) split_rows(M, g, up, 1, buf[g]);
    int r = run_all(M, [&](int g, wsmc_ctx* s) {
        if (up) return wsmc_weights_upload(s, buf[g].data());
        buf[g].resize(nloc(M, g));
        return wsmc_weights_download(s, buf[g].data());
    });
    if (!r && down)
        for (int g = 0; g < M->G; ++g) join_rows(M, g, buf[g], 1, down);
    return r;
}
int multi_score(wsmc_ctx* c, int32_t depth, double* host) {
    MultiState* M = c->multi;
    std::vector<std::vector<double>> buf(M->G);
    int r = run_all(M, [&](int g, wsmc_ctx* s) {
        buf[g].resize(nloc(M, g));
        return wsmc_score(s, depth, buf[g].data());
    });
    if (!r)
        for (int g = 0; g < M->G; ++g) join_rows(M, g, buf[g], 1, host);
    return r;
}
int multi_last_ancestors(wsmc_ctx* c, int32_t* host) {
    MultiState* M = c->multi;
    std::vector<std::vector<int32_t>> buf(M->G);
    int r = run_all(M, [&](int g, wsmc_ctx* s) {
        buf[g].resize(nloc(M, g));
        return wsmc_last_ancestors(s, buf[g].data());
    });
    if (!r)
        for (int g = 0; g < M->G; ++g) {
            // population indices: exact shards hold global ids already, island shards their own
            const int32_t base = M->sub[g]->shard_mode == WSMC_SHARD_EXACT ? 0 : (int32_t)M->off[g];
            for (int64_t i = 0; i < nloc(M, g); ++i) host[M->off[g] + i] = buf[g][(size_t)i] + base;
        }
    return r;
}
int multi_gather_rows(wsmc_ctx* c, int32_t col, const int64_t* idx, int64_t n, double* out) {
    MultiState* M = c->multi;
    int32_t dim = 0;
    int r = wsmc_col_info(M->sub[0], col, nullptr, 0, &dim);
    if (r) return r;
    std::vector<std::vector<int64_t>> li(M->G), pos(M->G);
    for (int64_t j = 0; j < n; ++j) {
        if (idx[j] < 0 || idx[j] >= M->N) return fail(WSMC_EARG, "row index out of range");
        int g = 0;
        while (idx[j] >= M->off[g + 1]) ++g;
        li[g].push_back(idx[j] - M->off[g]);
        pos[g].push_back(j);
    }
    std::vector<std::vector<double>> buf(M->G);
    r = run_all(M, [&](int g, wsmc_ctx* s) {   // local reads only: no collective
        if (li[g].empty()) return (int)WSMC_OK;
        buf[g].resize((size_t)dim * li[g].size());
        return wsmc_col_gather_rows(s, col, li[g].data(), (int64_t)li[g].size(), buf[g].data());
    });
    if (r) return r;
    for (int g = 0; g < M->G; ++g) {
        const size_t m = li[g].size();
        for (size_t q = 0; q < m; ++q)
            for (int k = 0; k < dim; ++k) out[(size_t)k * n + pos[g][q]] = buf[g][(size_t)k * m + q];
    }
    return WSMC_OK;
}
int multi_move(wsmc_ctx* c, int32_t proposal, const int32_t* targets, int32_t d, double step, const double* lo,
               const double* hi, int32_t target_depth, double diversity, int64_t* accepted_out) {
    std::vector<int64_t> acc(c->multi->G, 0);
    int r = run_all(c->multi, [&](int g, wsmc_ctx* s) {
        return wsmc_move(s, proposal, targets, d, step, lo, hi, target_depth, diversity, &acc[g]);
    });
    if (!r && accepted_out) {
        int64_t t = 0;
        for (int64_t a : acc) t += a;
        *accepted_out = t;
    }
    return r;
}

int multi_inject_failure(wsmc_ctx* c, int32_t shard, int32_t nth) {
    MultiState* M = c->multi;
    if (shard < 0 || shard >= M->G || nth < 0) return fail(WSMC_EARG, "bad shard or count");
    M->sub[shard]->inject_earg = nth >= 1000;
    M->sub[shard]->inject_fail = nth >= 1000 ? nth - 1000 : nth;
    return WSMC_OK;
}

int multi_comm_info(wsmc_ctx* c, wsmc_comm_info_t* out) {
    MultiState* M = c->multi;
    wsmc_comm_info_t first{};
    if (int r = wsmc_comm_info(M->sub[0], &first)) return r;
    *out = first;
    out->shards = M->G;
    for (int g = 0; g < 8; ++g) {
        out->devices[g] = g < M->G ? M->sub[g]->device : -1;
        out->shard_n[g] = g < M->G ? nloc(M, g) : 0;
    }
    return WSMC_OK;
}

}  // namespace wsmc

extern "C" int wsmc_create_multi(wsmc_ctx** out, int64_t n_particles, int32_t n_gpus, const int32_t* devices,
                                 uint64_t seed, int32_t transport) {
    if (!out) return fail(WSMC_EARG, "null out");
    *out = nullptr;
    if (n_gpus < 1 || n_gpus > kMaxWorld) return fail(WSMC_EARG, "n_gpus must be 1..8");
    if (n_particles < n_gpus) return fail(WSMC_EARG, "fewer particles than shards");
    if (n_particles >= (int64_t(1) << 31)) return fail(WSMC_EARG, "global population of 2^31 particles or more");
    if (transport != WSMC_TRANSPORT_RCCL && transport != WSMC_TRANSPORT_HOST) return fail(WSMC_EARG, "unknown transport");
    const int G = n_gpus;
    std::vector<int32_t> devs(G);
    for (int g = 0; g < G; ++g) devs[g] = devices ? devices[g] : g;
    if (transport == WSMC_TRANSPORT_RCCL)
        for (int g = 0; g < G; ++g)
            for (int h = 0; h < g; ++h)
                if (devs[g] == devs[h]) return fail(WSMC_EARG, "RCCL shards need distinct devices (transport 1 shares one)");
    MultiState* M = new MultiState();
    M->G = G;
    M->N = n_particles;
    M->off.resize(G + 1);
    for (int g = 0; g <= G; ++g) M->off[g] = n_particles * g / G;   // the oracle's shard layout
    M->sub.assign(G, nullptr);
    M->xargs.resize(G);
    auto cleanup = [&](int code) {
        for (auto* s : M->sub)
            if (s) wsmc_destroy(s);
        delete M;
        return code;
    };
    for (int g = 0; g < G; ++g) {
        int r = wsmc_create(&M->sub[g], M->off[g + 1] - M->off[g], devs[g], seed);
        if (r) return cleanup(r);
    }
    M->rccl = transport == WSMC_TRANSPORT_RCCL;
    if (transport == WSMC_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms(G);
        const ncclResult_t nr = ncclCommInitAll(comms.data(), G, devs.data());
        if (nr != ncclSuccess) return cleanup(fail(WSMC_ERCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(nr)));
        for (int g = 0; g < G; ++g) {
            wsmc_ctx* s = M->sub[g];
            s->world = G;
            s->rank = g;
            s->goff = M->off[g];
            s->gN = n_particles;
            s->comm = comms[g];   // the shard's destroy releases it
            s->peer_abort = &M->abort;
        }
    } else {
        for (int g = 0; g < G; ++g) {
            M->xargs[g] = XArg{M, g};
            int r = wsmc_comm_init_host(M->sub[g], multi_exchange, &M->xargs[g], G, g, M->off[g], n_particles);
            if (r) return cleanup(r);
            M->sub[g]->host_inproc = true;
        }
    }
    // the shards can read each other's device memory (one device, or peer access over xGMI):
    // the exact trace-back then reads lineages in their owners' buffers (csrc/wsmc_kernels.hip
    // k_exact_final); WSMC_DIAG_NO_PEER=1 keeps the trace windows and the cross-rank trace
    bool peer = G > 1;
    {
        const char* e = getenv("WSMC_DIAG_NO_PEER");
        if (e && atoi(e) != 0) peer = false;
    }
    int cur = 0;
    hipGetDevice(&cur);
    for (int g = 0; g < G && peer; ++g)
        for (int h = 0; h < G && peer; ++h) {
            if (devs[g] == devs[h]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devs[g], devs[h]) != hipSuccess || !can) {
                peer = false;
                break;
            }
            hipSetDevice(devs[g]);
            const hipError_t e = hipDeviceEnablePeerAccess(devs[h], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) peer = false;
        }
    (void)hipGetLastError();
    hipSetDevice(cur);
    for (int g = 0; g < G; ++g) M->sub[g]->peer_ok = peer;
    M->workers.resize(G);
    for (int g = 1; g < G; ++g) {
        M->workers[g] = std::make_unique<Worker>();
        M->workers[g]->th = std::thread(worker_loop, M->workers[g].get());
    }
    wsmc_ctx* c = new wsmc_ctx();
    c->multi = M;
    c->device = devs[0];
    c->N = n_particles;
    c->gN = n_particles;
    c->seed = seed;
    c->world = G;
    *out = c;
    return WSMC_OK;
}
