// wsmc_jit.hip — statement batches compiled for their shape at run time (hiprtc).
//
// A model's step issues the same statements every step (examples/2D_ssm.jl:11-16: Assign,
// Sample, Assign, Observe), so the batch csrc/wsmc_api.hip collects for it has the same shape
// every step: the same op kinds and dims, the same rows, the same columns read through the
// ancestors. Only the values change (buffer pointers, constants, observations, op counters).
// The shape is the signature (EwSig, csrc/wsmc_ew_body.h); the first launch of a signature on a
// device generates a translation unit that instantiates ew_body<signature>, compiles it with
// hiprtc for the device's architecture from the headers embedded at build time (the same text
// hipcc compiled into this library, -ffp-contract=off, no fast math: the same bits), loads the
// code object and keeps it for the process. This is the device analogue of the reference's
// per-model specialisation: Julia compiles the broadcasts `vectorize` emits for each @model
// (src/rewrites.jl:146-219) the first time the model runs.
//
// A batch whose signature fails to compile (or WSMC_DIAG_NO_JIT=1) runs on the interpreter
// kernel k_ew_batch, which computes the same bits; wsmc_debug_jit_stats counts both.
#include <hip/hiprtc.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "wsmc_ew_body.h"
#include "wsmc_internal.h"

namespace wsmc {
namespace {

struct JitHeader {
    const char* name;
    const char* text;
};
const JitHeader kJitHeaders[] = {
#include "wsmc_jit_headers.inc"
};

struct JitKernel {
    hipModule_t mod = nullptr;
    hipFunction_t f[2] = {nullptr, nullptr};   // P = 1, P = 2
    bool ok = false;
};

struct JitCache {
    std::mutex mu;
    std::map<std::pair<int, std::string>, JitKernel> k;
    int64_t compiled = 0, failed = 0, launched = 0, interpreted = 0;
    double compile_s = 0.0;
    int64_t mv_compiled = 0, mv_failed = 0, mv_launched = 0, mv_interpreted = 0;   // Move blocks
    double mv_compile_s = 0.0;
};
JitCache& cache() {
    static JitCache* c = new JitCache;   // never destroyed: modules live for the process
    return *c;
}

bool jit_off() {
    static const bool v = [] {
        const char* e = getenv("WSMC_DIAG_NO_JIT");
        return e && atoi(e) != 0;
    }();
    return v;
}
// diagnostics: WSMC_JIT_DUMP=<dir> writes each compiled code object (<dir>/<kind>_<n>.co) and its
// signature (<dir>/<kind>_<n>.sig), for the ISA and register counts of the run-time kernels
void jit_dump(const char* kind, int64_t n, const std::string& key, const std::string& code) {
    const char* d = getenv("WSMC_JIT_DUMP");
    if (!d || !*d) return;
    const std::string base = std::string(d) + "/" + kind + "_" + std::to_string(n);
    if (FILE* f = fopen((base + ".co").c_str(), "wb")) {
        fwrite(code.data(), 1, code.size(), f);
        fclose(f);
    }
    if (FILE* f = fopen((base + ".sig").c_str(), "w")) {
        fwrite(key.data(), 1, key.size(), f);
        fclose(f);
    }
}
bool jit_verbose() {
    static const bool v = [] {
        const char* e = getenv("WSMC_JIT_VERBOSE");
        return e && atoi(e) != 0;
    }();
    return v;
}

// the row an operand of a Sample / weight term reads (its column renumbered to a batch slot)
int8_t slot_rowc(const EwBatch& b, int32_t col, int32_t comp) {
    return col < 0 ? (int8_t)-1 : (int8_t)(b.slot_row[col] + comp);
}

EwSig signature(const EwBatch& b, unsigned feat) {
    EwSig g;
    std::memset(&g, 0, sizeof(g));
    g.nops = (int8_t)b.nops;
    g.has_w = (int8_t)(b.has_w != 0);
    g.has_reset = (int8_t)(b.has_w && b.wreset != nullptr);
    g.has_anc = (int8_t)(b.anc != nullptr);
    g.has_dec = (int8_t)(b.dec != nullptr);
    g.ntab = (int8_t)b.ntab;
    g.npre = (int8_t)b.npre;
    g.qs = (int8_t)(b.has_w && b.qs_base != nullptr);
    for (int k = 0; k < b.npre; ++k) {
        g.pre_row[k] = b.pre_row[k];
        g.pre_lag[k] = b.pre_lag[k];
    }
    g.feat = feat;
    for (int k = 0; k < b.nops; ++k) {
        const EwOp& op = b.ops[k];
        EwSigOp& o = g.op[k];
        std::memset(&o, -1, sizeof(o));
        o.kind = (int8_t)op.kind;
        o.dim = (int8_t)op.dim;
        o.out_row = (int8_t)op.out_row;
        o.family = o.mean_fn = o.ddim = o.has_sd = 0;
        o.nostore = (int8_t)(op.kind == 1 && op.nostore);
        for (int q = 0; q < 4; ++q)
            for (int m = 0; m < 2; ++m) {
                o.asrc[q][m] = kSrcNone;
                o.arow[q][m] = 0;
            }
        if (op.kind == 0) {
            for (int q = 0; q < op.dim; ++q)
                for (int m = 0; m < 2; ++m) {
                    if (op.a.e[q].col[m] < 0) continue;
                    if (op.a.fwd[q][m] >= 0) {
                        o.asrc[q][m] = kSrcRow;
                        o.arow[q][m] = op.a.fwd[q][m];
                    } else {
                        o.asrc[q][m] = ((op.a.lag >> (2 * q + m)) & 1) ? kSrcLag : kSrcMem;
                    }
                }
            continue;
        }
        const wsmc_dist& d = op.kind == 1 ? op.s.d : op.w.t.dist;
        o.family = (int8_t)d.family;
        o.mean_fn = (int8_t)d.mean_fn;
        o.ddim = (int8_t)d.dim;
        o.has_sd = (int8_t)(op.kind == 1 && op.s.has_sd);
        for (int q = 0; q < 4; ++q)
            for (int m = 0; m < 2; ++m) o.mrow[q][m] = slot_rowc(b, d.mu[q].col[m], d.mu[q].comp[m]);
        for (int m = 0; m < 2; ++m) o.srow[m] = slot_rowc(b, d.scale.col[m], d.scale.comp[m]);
        if (op.kind == 2)
            for (int q = 0; q < 4; ++q)
                for (int m = 0; m < 2; ++m) o.xrow[q][m] = slot_rowc(b, op.w.t.x[q].col[m], op.w.t.x[q].comp[m]);
    }
    return g;
}

// the signature as a C++ aggregate initializer (also the cache key)
std::string sig_text(const EwSig& g) {
    std::string s;
    auto num = [&](int v) { s += std::to_string(v); s += ','; };
    auto arr = [&](const int8_t* a, int n) {
        s += '{';
        for (int k = 0; k < n; ++k) num(a[k]);
        s += "},";
    };
    s += '{';
    num(g.nops); num(g.has_w); num(g.has_reset); num(g.has_anc); num(g.has_dec); num(g.ntab); num(g.npre); num(g.qs);
    arr(g.pre_row, kEwPre);
    arr(g.pre_lag, kEwPre);
    s += std::to_string(g.feat) + "u,{";
    for (int k = 0; k < kEwOps; ++k) {
        const EwSigOp& o = g.op[k];
        s += '{';
        num(o.kind); num(o.dim); num(o.out_row); num(o.family); num(o.mean_fn); num(o.ddim); num(o.has_sd);
        num(o.nostore);
        s += '{'; for (int q = 0; q < 4; ++q) arr(o.asrc[q], 2); s += "},";
        s += '{'; for (int q = 0; q < 4; ++q) arr(o.arow[q], 2); s += "},";
        s += '{'; for (int q = 0; q < 4; ++q) arr(o.mrow[q], 2); s += "},";
        arr(o.srow, 2);
        s += '{'; for (int q = 0; q < 4; ++q) arr(o.xrow[q], 2); s += "}";
        s += "},";
    }
    s += "}}";
    return s;
}

bool tables_global();
// the log / exp tables in LDS for a batch that draws (a Sample's normals take a log each);
// the copy and its barrier are pure cost to a batch without draws (C3's Observe batch: 2 %)
bool ew_tables_lds(const EwSig& g) {
    if (tables_global()) return false;
    for (int k = 0; k < g.nops; ++k)
        if (g.op[k].kind == 1) return true;
    return false;
}
std::string tu_source(const std::string& sig, bool lds, bool qs) {
    const std::string head = std::string(lds ? "#define WSMC_TABLES_LDS 1\n" : "") + "#include \"wsmc_ew_body.h\"\n"
                             "struct WsmcSig { static constexpr wsmc::EwSig sig = " + sig + "; };\n";
    if (qs)   // the statistics: two particles a thread, 512 threads = one Resample tile a block
        return head +
               "extern \"C\" __global__ void wsmc_ew_p1(wsmc::EwBatch, uint64_t, int64_t, int64_t) {}\n"
               "extern \"C\" __global__ __launch_bounds__(512) void wsmc_ew_p2(wsmc::EwBatch, uint64_t seed, "
               "int64_t goff, int64_t N) { wsmc::ew_body<WsmcSig, 2, 512>(seed, goff, N); }\n";
    return head +
           "extern \"C\" __global__ __launch_bounds__(256) void wsmc_ew_p1(wsmc::EwBatch, uint64_t seed, int64_t goff, "
           "int64_t N) { wsmc::ew_body<WsmcSig, 1>(seed, goff, N); }\n"
           "extern \"C\" __global__ __launch_bounds__(256) void wsmc_ew_p2(wsmc::EwBatch, uint64_t seed, int64_t goff, "
           "int64_t N) { wsmc::ew_body<WsmcSig, 2>(seed, goff, N); }\n";
}

// compile a translation unit for `arch` (the code object in `code`)
bool compile_src(const std::string& arch, const std::string& src, std::string& code, std::string& err) {
    const int nh = (int)(sizeof(kJitHeaders) / sizeof(kJitHeaders[0]));
    std::vector<const char*> htext(nh), hname(nh);   // sized from the generated list (build.py JIT_HEADERS)
    for (int k = 0; k < nh; ++k) {
        htext[k] = kJitHeaders[k].text;
        hname[k] = kJitHeaders[k].name;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "wsmc_ew_jit.hip", nh, htext.data(), hname.data()) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return false;
    }
    const std::string arch_opt = "--offload-arch=" + arch;
    const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                          "-munsafe-fp-atomics", "-Wno-unused-result",
#ifdef WSMC_LDS_TABLE_CHECK   // the library's check build checks its run-time compiled kernels too
                          "-DWSMC_LDS_TABLE_CHECK",
#endif
    };
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof(opts) / sizeof(opts[0])), opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        err = std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(rc) + "\n" + log;
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code.assign(n, '\0');
    hiprtcGetCode(prog, &code[0]);
    hiprtcDestroyProgram(&prog);
    return true;
}

bool compile_code(const std::string& arch, const std::string& sig, std::string& code, std::string& err, bool lds,
                  bool qs) {
    return compile_src(arch, tu_source(sig, lds, qs), code, err);
}

bool device_arch(int device, std::string& arch, std::string& err) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        err = "hipGetDeviceProperties failed";
        return false;
    }
    arch = prop.gcnArchName;   // e.g. "gfx950:sramecc+:xnack-": the processor alone
    arch = arch.substr(0, arch.find(':'));
    return true;
}

// load a code object on `device` and look up its kernels f[0], f[1]
bool load_module(int device, const std::string& code, const char* f0, const char* f1, JitKernel& out,
                 std::string& err) {
    int cur = 0;
    hipGetDevice(&cur);
    hipSetDevice(device);
    hipError_t e = hipModuleLoadData(&out.mod, code.data());
    if (e == hipSuccess) e = hipModuleGetFunction(&out.f[0], out.mod, f0);
    if (e == hipSuccess) e = hipModuleGetFunction(&out.f[1], out.mod, f1);
    hipSetDevice(cur);
    if (e != hipSuccess) {
        err = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
        return false;
    }
    return true;
}

bool compile(int device, const std::string& sig, JitKernel& out, std::string& err, bool lds, bool qs) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        err = "hipGetDeviceProperties failed";
        return false;
    }
    std::string arch = prop.gcnArchName;   // e.g. "gfx950:sramecc+:xnack-": the processor alone
    arch = arch.substr(0, arch.find(':'));
    std::string code;
    if (!compile_code(arch, sig, code, err, lds, qs)) return false;
    int cur = 0;
    hipGetDevice(&cur);
    hipSetDevice(device);
    hipError_t e = hipModuleLoadData(&out.mod, code.data());
    if (e == hipSuccess) e = hipModuleGetFunction(&out.f[0], out.mod, "wsmc_ew_p1");
    if (e == hipSuccess) e = hipModuleGetFunction(&out.f[1], out.mod, "wsmc_ew_p2");
    hipSetDevice(cur);
    if (e != hipSuccess) {
        err = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
        return false;
    }
    return true;
}

bool aligned(const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

// two particles a thread: N even and every direct (not gathered) access 16-B aligned
bool pair_ok(const EwBatch& b, int64_t N) {
    if (N & 1) return false;
    if (b.anc && !aligned(b.anc, 8)) return false;
    if (b.has_w && !aligned(b.w, 16)) return false;
    for (int k = 0; k < b.npre; ++k)
        if (!b.pre_lag[k] && !aligned(b.pre_src[k], 16)) return false;
    for (int k = 0; k < b.nops; ++k) {
        const EwOp& op = b.ops[k];
        if (op.kind != 2 && !aligned(op.out, 16)) return false;
        if (op.kind == 0)
            for (int q = 0; q < op.dim; ++q)
                for (int m = 0; m < 2; ++m)
                    if (op.a.e[q].col[m] >= 0 && op.a.fwd[q][m] < 0 && !((op.a.lag >> (2 * q + m)) & 1) &&
                        !aligned(op.a.p[q][m], 16))
                        return false;
    }
    return true;
}

}  // namespace

// the batch on its signature's compiled kernel; hipErrorNotSupported: no kernel (JIT off or the
// signature failed to compile) — the caller runs the interpreter
hipError_t launch_ew_jit(hipStream_t s, const EwBatch& b, unsigned feat, uint64_t seed, int64_t goff, int64_t N,
                         int device) {
    JitCache& C = cache();
    if (jit_off()) {
        std::lock_guard<std::mutex> lk(C.mu);
        C.interpreted += 1;
        return hipErrorNotSupported;
    }
    const EwSig sg = signature(b, feat);
    const std::string key = sig_text(sg);
    JitKernel* jk = nullptr;
    {
        std::lock_guard<std::mutex> lk(C.mu);
        auto it = C.k.find({device, key});
        if (it == C.k.end()) {
            JitKernel k;
            std::string err;
            const auto t0 = std::chrono::steady_clock::now();
            k.ok = compile(device, key, k, err, ew_tables_lds(sg), sg.qs != 0);
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            C.compile_s += dt;
            if (k.ok) {
                C.compiled += 1;
                if (jit_verbose()) fprintf(stderr, "[wsmc jit] device %d: signature compiled in %.2f s\n", device, dt);
            } else {
                C.failed += 1;
                fprintf(stderr, "[wsmc jit] device %d: a statement-batch signature did not compile; it runs on the "
                                "interpreter kernel\n%s\n", device, err.c_str());
            }
            it = C.k.emplace(std::make_pair(device, key), k).first;
        }
        jk = &it->second;
        if (!jk->ok) {
            C.interpreted += 1;
            return hipErrorNotSupported;
        }
        C.launched += 1;
    }
    const int P = pair_ok(b, N) ? 2 : 1;
    if (sg.qs && P != 2) return hipErrorInvalidValue;   // (the caller checked ew_pair_ok)
    const int NT = sg.qs ? 512 : kBlock;
    const int64_t threads = (N + P - 1) / P;
    const unsigned grid = (unsigned)((threads + NT - 1) / NT);
    EwBatch bb = b;   // the kernel arguments (copied by the launch)
    void* args[] = {&bb, &seed, &goff, &N};
    return hipModuleLaunchKernel(jk->f[P - 1], grid, 1, 1, NT, 1, 1, 0, s, args, nullptr);
}
bool ew_pair_ok(const EwBatch& b, int64_t N) { return pair_ok(b, N); }

// compile a representative signature (the 2D SSM step: Assign through the ancestors, Sample,
// Assign, Observe) for gfx950 without a device: the embedded headers build under hiprtc
int ew_jit_selfcheck(std::string& err) {
    EwSig g;
    std::memset(&g, 0, sizeof(g));
    g.nops = 4; g.has_w = 1; g.has_reset = 1; g.has_anc = 1; g.has_dec = 1; g.ntab = 1; g.npre = 4;
    for (int k = 0; k < 4; ++k) { g.pre_row[k] = (int8_t)k; g.pre_lag[k] = 1; }
    const int8_t rows[4][2][2] = {{{0, 2}, {1, 3}}, {{0, 0}, {0, 0}}, {{2, 6}, {3, 7}}, {{0, 0}, {0, 0}}};
    for (int k = 0; k < 4; ++k) {
        EwSigOp& o = g.op[k];
        std::memset(&o, -1, sizeof(o));
        o.kind = (int8_t)(k == 3 ? 2 : (k == 1 ? 1 : 0));
        o.dim = 2;
        o.out_row = (int8_t)(k == 3 ? -1 : 4 + 2 * k);
        o.family = (int8_t)(o.kind == 0 ? 0 : WSMC_FAM_MVNORMAL_ISO);
        o.mean_fn = 0;
        o.ddim = (int8_t)(o.kind == 0 ? 0 : 2);
        o.has_sd = (int8_t)(k == 1);
        o.nostore = 0;
        for (int q = 0; q < 4; ++q)
            for (int m = 0; m < 2; ++m) {
                o.asrc[q][m] = (o.kind == 0 && q < 2) ? kSrcRow : kSrcNone;
                o.arow[q][m] = (o.kind == 0 && q < 2) ? rows[k][q][m] : 0;
            }
        if (k == 3) {
            o.mrow[0][0] = 4;
            o.mrow[1][0] = 5;
        }
    }
    std::string code;
    if (!compile_code("gfx950", sig_text(g), code, err, ew_tables_lds(g), false)) return -1;
    g.qs = 1;   // and its form with the Resample statistics
    return compile_code("gfx950", sig_text(g), code, err, ew_tables_lds(g), true) ? 0 : -1;
}

void ew_jit_stats(int64_t* out) {
    JitCache& C = cache();
    std::lock_guard<std::mutex> lk(C.mu);
    out[0] = C.compiled;
    out[1] = C.failed;
    out[2] = C.launched;
    out[3] = C.interpreted;
    out[4] = (int64_t)(C.compile_s * 1e6);
}

// ---- Move blocks compiled for their shape (csrc/wsmc_mv_body.h) ------------------------
namespace {
std::string mv_sig_text(const MvSig& g) {
    std::string s;
    auto num = [&](int v) { s += std::to_string(v); s += ','; };
    auto op = [&](const MvSigOp& o) { s += '{'; s += '{'; num(o.c[0]); num(o.c[1]); s += "}},"; };
    s += '{';
    num(g.K); num(g.nm); num(g.D); num(g.ns); num(g.ntmpl); num(g.nnew); num(g.nold); num(g.carry);
    s += '{';
    for (int k = 0; k < 5; ++k) num(g.off[k]);
    s += "},";
    num(g.bnd); num(g.lagt); num(g.flo); num(g.fhi); num(g.smask);
    s += '{';
    for (int k = 0; k < 2 * kMvSegs; ++k) {
        const MvSigSeg& q = g.seg[k];
        s += '{';
        num(q.kind); num(q.fam); num(q.pre); num(0);
        op(q.x);
        s += '{';
        for (int j = 0; j < 4; ++j) op(q.mu[j]);
        s += "},";
        op(q.sc);
        s += "},";
    }
    s += "}}";
    return s;
}

// two entries: the program in the kernel arguments (read through the kernarg segment, scalar
// loads) or in device memory; MvArgs after ProgInlineBlk at its own alignment
// WSMC_DIAG_MV_WAVES=n: the blocks compiled for n waves a SIMD (amdgpu_waves_per_eu), for comparison
std::string mv_waves_attr() {
    static const std::string a = [] {
        const char* e = diag_env("WSMC_DIAG_MV_WAVES");
        const int n = e ? atoi(e) : 0;
        return n > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(n) + ")))" : std::string();
    }();
    return a;
}
// the run-time compiled kernels whose work is transcendental-heavy read the log / exp tables
// from LDS copies (WSMC_TABLES_LDS, include/wsmc_math.h); WSMC_DIAG_MV_TABLES_GLOBAL=1 keeps
// the gathers through the caches everywhere, for comparison
bool tables_global() {
    static const bool g = [] {
        const char* e = diag_env("WSMC_DIAG_MV_TABLES_GLOBAL");
        return e && *e && *e != '0';
    }();
    return g;
}
// a Move block with bounded targets (log / exp transforms) or oscillator terms (anchors):
// C5's blocks 158.5 -> 153.5 ms; C3's unbounded affine blocks measured 2 % slower with the copy
bool mv_tables_lds(const MvSig& g) {
    if (tables_global()) return false;
    if (g.bnd) return true;
    for (int k = 0; k < 2 * kMvSegs; ++k)
        if (g.seg[k].kind == kSegNormalOsc) return true;
    return false;
}
std::string mv_tu(const std::string& sig, bool lds) {
    const std::string lb = "__launch_bounds__(256)" + mv_waves_attr();
    return std::string(lds ? "#define WSMC_TABLES_LDS 1\n" : "") + "#include \"wsmc_mv_body.h\"\n"
           "struct WsmcMvSig { static constexpr wsmc::MvSig sig = " + sig + "; };\n"
           "constexpr unsigned kMvArgsAt = (sizeof(wsmc::ProgInlineBlk) + alignof(wsmc::MvArgs) - 1) & "
           "~(unsigned)(alignof(wsmc::MvArgs) - 1);\n"
           "extern \"C\" __global__ " + lb + " void wsmc_mv_i(wsmc::ProgInlineBlk, wsmc::MvArgs) {\n"
           "  const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();\n"
           "  wsmc::mv_body<WsmcMvSig>(ka + __builtin_offsetof(wsmc::ProgInlineBlk, w), "
           "*reinterpret_cast<const wsmc::MvArgs*>(ka + kMvArgsAt));\n}\n"
           "extern \"C\" __global__ " + lb + " void wsmc_mv_g(wsmc::ProgInlineBlk, wsmc::MvArgs) {\n"
           "  const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();\n"
           "  const wsmc::MvArgs& a = *reinterpret_cast<const wsmc::MvArgs*>(ka + kMvArgsAt);\n"
           "  wsmc::mv_body<WsmcMvSig>(a.prog, a);\n}\n";
}
}  // namespace

hipError_t launch_mv_jit(hipStream_t s, const MvSig& sig, const ProgInlineBlk* pin, const MvArgs& a, int device) {
    JitCache& C = cache();
    if (jit_off()) {
        std::lock_guard<std::mutex> lk(C.mu);
        C.mv_interpreted += 1;
        return hipErrorNotSupported;
    }
    const std::string key = "mv:" + mv_sig_text(sig);
    JitKernel* jk = nullptr;
    {
        std::lock_guard<std::mutex> lk(C.mu);
        auto it = C.k.find({device, key});
        if (it == C.k.end()) {
            JitKernel k;
            std::string err, arch, code;
            const auto t0 = std::chrono::steady_clock::now();
            k.ok = device_arch(device, arch, err) && compile_src(arch, mv_tu(key.substr(3), mv_tables_lds(sig)), code, err) &&
                   load_module(device, code, "wsmc_mv_i", "wsmc_mv_g", k, err);
            if (k.ok) jit_dump("mv", C.mv_compiled, key, code);
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            C.mv_compile_s += dt;
            if (k.ok) {
                C.mv_compiled += 1;
                if (jit_verbose()) fprintf(stderr, "[wsmc jit] device %d: Move block compiled in %.2f s\n", device, dt);
            } else {
                C.mv_failed += 1;
                fprintf(stderr, "[wsmc jit] device %d: a Move-block signature did not compile; it runs on the "
                                "interpreter kernel\n%s\n", device, err.c_str());
            }
            it = C.k.emplace(std::make_pair(device, key), k).first;
        }
        jk = &it->second;
        if (!jk->ok) {
            C.mv_interpreted += 1;
            return hipErrorNotSupported;
        }
        C.mv_launched += 1;
    }
    const unsigned grid = (unsigned)((a.N + sig.K * kBlock - 1) / (sig.K * kBlock));
    ProgInlineBlk pb;
    if (pin) {
        pb = *pin;
    } else {
        std::memset(&pb, 0, sizeof(pb));
    }
    MvArgs aa = a;
    void* args[] = {&pb, &aa};
    return hipModuleLaunchKernel(jk->f[pin ? 0 : 1], grid, 1, 1, kBlock, 1, 1, 0, s, args, nullptr);
}

// compile a representative Move block (C3's: two 1-D unbounded moves, two Normal priors and an
// affine Normal run; the old fold one Normal term) for gfx950 without a device
int mv_jit_selfcheck(std::string& err) {
    MvSig g;
    std::memset(&g, 0, sizeof(g));
    for (auto& q : g.seg) {
        q.x.c[0] = q.x.c[1] = q.sc.c[0] = q.sc.c[1] = -1;
        for (auto& m : q.mu) m.c[0] = m.c[1] = -1;
    }
    g.K = 2; g.nm = 2; g.D = 2; g.ns = 2; g.ntmpl = 4; g.nnew = 3; g.nold = 1; g.carry = 1;
    g.off[0] = 0; g.off[1] = 1; g.off[2] = 2; g.off[3] = 2; g.off[4] = 2;
    for (int k = 0; k < 2; ++k) {
        g.seg[k].kind = kSegTerm;
        g.seg[k].fam = WSMC_FAM_NORMAL;
        g.seg[k].pre = 1;
        g.seg[k].x.c[0] = (int8_t)k;
    }
    g.seg[2].kind = kSegNormalAff;
    g.seg[2].pre = 1;
    g.seg[2].mu[0].c[0] = 0;
    g.seg[2].mu[0].c[1] = 1;
    g.seg[kMvSegs] = g.seg[0];
    g.seg[kMvSegs].mu[0].c[0] = 0;
    std::string code;
    return compile_src("gfx950", mv_tu(mv_sig_text(g), mv_tables_lds(g)), code, err) ? 0 : -1;
}

void mv_jit_stats(int64_t* out) {
    JitCache& C = cache();
    std::lock_guard<std::mutex> lk(C.mu);
    out[0] = C.mv_compiled;
    out[1] = C.mv_failed;
    out[2] = C.mv_launched;
    out[3] = C.mv_interpreted;
    out[4] = (int64_t)(C.mv_compile_s * 1e6);
}

}  // namespace wsmc
