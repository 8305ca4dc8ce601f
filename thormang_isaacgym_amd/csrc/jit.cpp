// jit.cpp -- run-time model specialisations (tg_model_jit).
//
// The reference loads its URDF at run time (gym.load_asset,
// isaacgymenvs/tasks/gogoro_new.py:198-213).  libtgsim.so ships constexpr
// specialisations of the articulation kernels for the models compiled in
// (generated/Model_*.inc); a model that is not among them is compiled here,
// at run time, by hipRTC for gfx950: the same kernel templates
// (articulation_kernels.h) instantiated with the model's constexpr tables (the
// text model/codegen.py emits), so a changed URDF needs no library rebuild.
// The code object is cached on disk by (model hash, digest of the model text
// and the kernel headers) and loaded per device with hipModuleLoadData; the
// launchers in articulation.hip fall through to the jit_* functions below
// when no compiled specialisation matches the hash.  The task epilogues
// (tg_walk_step / tg_gogoro_step fusion) are not instantiated for run-time
// models: those calls fall back to the separate task kernels.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "tg_kernels.h"

namespace tg {
namespace {

constexpr int JIT_COMPOSE_WPB = 8;   // articulation_kernels.h COMPOSE_WPB
enum { K_COMPOSE, K_STEP, K_STEP_HF, K_BODY, K_RBF, NK };
const char *const KERNEL_EXPR[NK] = {
    "tg::compose_kernel<TgJitModel>",
    "tg::step_par_kernel<TgJitModel, TgJitModel::EPB, false, tg::NoPost>",
    "tg::step_par_kernel<TgJitModel, TgJitModel::EPB, true, tg::NoPost>",
    "tg::body_state_kernel<TgJitModel>",
    "tg::rb_force_kernel<TgJitModel>",
};
// the per-model launch figures the host needs, read back from the module
// (tgjit_meta, same order)
struct JitMeta {
    int kc, epb, lpe, lds, nl, ng, nd, pad;
};
struct JitCode {
    std::vector<char> code;   // gfx950 code object
    std::string names[NK];    // lowered kernel names
};
struct JitLoaded {
    hipModule_t mod = nullptr;
    hipFunction_t f[NK] = {};
    JitMeta meta{};
};

std::mutex g_mu;
std::map<uint64_t, JitCode> g_code;                            // by model hash
std::map<std::pair<uint64_t, int>, JitLoaded> g_loaded;       // by (hash, device)

const char *const HEADERS[] = {"articulation_kernels.h", "step_par.h", "tg_math.h", "gogoro_math.h", "paper_math.h",
                               "tg_kernels.h",
                               "../../include/tgsim.h", "../../include/tg_gogoro.h",
                               "../../include/tg_gogoro_paper.h", "../../include/tg_walk.h"};

uint64_t fnv1a(uint64_t h, const std::string &s) {
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

bool read_file(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// directory of this shared library + "/csrc" (the in-tree kernel headers)
std::string default_include_dir() {
    Dl_info info{};
    if (!dladdr((void *)&default_include_dir, &info) || !info.dli_fname) return "";
    std::string p = info.dli_fname;
    const size_t k = p.rfind('/');
    return (k == std::string::npos ? std::string(".") : p.substr(0, k)) + "/csrc";
}

std::string source_text(const char *struct_name, const char *model_source) {
    std::string s;
    s += "// run-time specialisation (libtgsim jit.cpp)\n";
    s += "#include \"articulation_kernels.h\"\n";
    s += model_source;
    s += "\nusing TgJitModel = ";
    s += struct_name;
    s += ";\nextern \"C\" __device__ const int tgjit_meta[8] = {TgJitModel::KC, TgJitModel::EPB, TgJitModel::LPE,\n"
         "    (int)tg::ParLayout<TgJitModel>::template bytes<TgJitModel::EPB>(), TgJitModel::NL, TgJitModel::NG,\n"
         "    TgJitModel::ND, 0};\n";
    return s;
}

// the flags of the compiled-in articulation unit (build_ext.py UNITS); part of
// the on-disk cache key (jit_compile), so a flag-only change never reuses a
// code object built under other semantics
const char *const JIT_OPTS[] = {"--offload-arch=gfx950", "-std=c++17", "-O3", "-ffast-math", "-fno-associative-math",
                                "-ffp-contract=fast-honor-pragmas", "-munsafe-fp-atomics", "-fno-slp-vectorize",
                                "-DTG_JIT=1"};
constexpr int N_JIT_OPTS = (int)(sizeof JIT_OPTS / sizeof JIT_OPTS[0]);

int compile(const std::string &src, const std::string &incdir, JitCode &out, std::string &err) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "tgjit_model.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return TG_ERR_HIP;
    }
    for (int k = 0; k < NK; ++k) hiprtcAddNameExpression(prog, KERNEL_EXPR[k]);
    const std::string inc = "-I" + incdir;
    const char *opts[N_JIT_OPTS + 1];
    for (int k = 0; k < N_JIT_OPTS; ++k) opts[k] = JIT_OPTS[k];
    opts[N_JIT_OPTS] = inc.c_str();
    const hiprtcResult rc = hiprtcCompileProgram(prog, N_JIT_OPTS + 1, opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        err = std::string("hipRTC compile failed: ") + hiprtcGetErrorString(rc) + "\n" +
              (log.size() > 4000 ? log.substr(0, 4000) : log);
        hiprtcDestroyProgram(&prog);
        return TG_ERR_MODEL;
    }
    for (int k = 0; k < NK; ++k) {
        const char *nm = nullptr;
        if (hiprtcGetLoweredName(prog, KERNEL_EXPR[k], &nm) != HIPRTC_SUCCESS || !nm) {
            err = std::string("hipRTC: no lowered name for ") + KERNEL_EXPR[k];
            hiprtcDestroyProgram(&prog);
            return TG_ERR_MODEL;
        }
        out.names[k] = nm;
    }
    size_t sz = 0;
    hiprtcGetCodeSize(prog, &sz);
    out.code.resize(sz);
    hiprtcGetCode(prog, out.code.data());
    hiprtcDestroyProgram(&prog);
    return 0;
}

// cache file: "TGJIT1\n", one lowered name per line, then the code object
bool cache_load(const std::string &path, JitCode &out) {
    std::string s;
    if (!read_file(path, s)) return false;
    size_t pos = 0;
    auto line = [&](std::string &l) {
        const size_t e = s.find('\n', pos);
        if (e == std::string::npos) return false;
        l = s.substr(pos, e - pos);
        pos = e + 1;
        return true;
    };
    std::string magic;
    if (!line(magic) || magic != "TGJIT1") return false;
    for (int k = 0; k < NK; ++k)
        if (!line(out.names[k]) || out.names[k].empty()) return false;
    if (pos >= s.size()) return false;
    out.code.assign(s.begin() + pos, s.end());
    return true;
}

void cache_store(const std::string &path, const JitCode &c) {
    const std::string tmp = path + ".tmp" + std::to_string((unsigned long)getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;
        f << "TGJIT1\n";
        for (int k = 0; k < NK; ++k) f << c.names[k] << "\n";
        f.write(c.code.data(), (std::streamsize)c.code.size());
        if (!f) return;
    }
    std::rename(tmp.c_str(), path.c_str());   // atomic publish: concurrent ranks never read a partial file
}

// the module of `hash` on the current device, loaded on first use (g_mu held)
JitLoaded *loaded_locked(uint64_t hash) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    auto it = g_loaded.find({hash, dev});
    if (it != g_loaded.end()) return &it->second;
    auto c = g_code.find(hash);
    if (c == g_code.end()) return nullptr;
    JitLoaded L;
    if (hipModuleLoadData(&L.mod, c->second.code.data()) != hipSuccess) return nullptr;
    for (int k = 0; k < NK; ++k)
        if (hipModuleGetFunction(&L.f[k], L.mod, c->second.names[k].c_str()) != hipSuccess) return nullptr;
    hipDeviceptr_t p = nullptr;
    size_t bytes = 0;
    if (hipModuleGetGlobal(&p, &bytes, L.mod, "tgjit_meta") != hipSuccess || bytes != sizeof(JitMeta)) return nullptr;
    if (hipMemcpyDtoH(&L.meta, p, sizeof(JitMeta)) != hipSuccess) return nullptr;
    if (L.meta.lds > 160 * 1024) return nullptr;
    // dynamic LDS above the 64 KB default (large trees): best effort, the
    // launch reports a failure if the device refuses it
    if (L.meta.lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void *)L.f[K_STEP], hipFuncAttributeMaxDynamicSharedMemorySize, L.meta.lds);
    return &g_loaded.emplace(std::make_pair(hash, dev), L).first->second;
}

JitLoaded *find(uint64_t hash) {
    std::lock_guard<std::mutex> lk(g_mu);
    return loaded_locked(hash);
}

int launch(hipFunction_t f, unsigned gx, unsigned bx, unsigned lds, hipStream_t s, void **args) {
    if (hipModuleLaunchKernel(f, gx, 1, 1, bx, 1, 1, lds, s, args, nullptr) != hipSuccess) return TG_ERR_HIP;
    return 0;
}

}  // namespace

int jit_compile(uint64_t hash, const char *struct_name, const char *model_source, const char *include_dir,
                const char *cache_dir, std::string &err) {
    const std::string inc = include_dir && *include_dir ? include_dir : default_include_dir();
    uint64_t digest = fnv1a(14695981039346656037ull, struct_name);
    digest = fnv1a(digest, model_source);
    for (const char *h : HEADERS) {
        std::string t;
        if (!read_file(inc + "/" + h, t)) {
            err = "kernel header " + inc + "/" + h + " not found (tg_model_jit include_dir)";
            return TG_ERR_ARG;
        }
        digest = fnv1a(digest, t);
    }
    // the compile flags and the hipRTC version are part of the key too
    for (int k = 0; k < N_JIT_OPTS; ++k) digest = fnv1a(digest, JIT_OPTS[k]);
    int rtc_major = 0, rtc_minor = 0;
    (void)hiprtcVersion(&rtc_major, &rtc_minor);
    digest = fnv1a(digest, ("hiprtc " + std::to_string(rtc_major) + "." + std::to_string(rtc_minor)).c_str());
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_code.count(hash)) return 0;
    }
    char fname[96];
    snprintf(fname, sizeof fname, "tgjit_%016llx_%016llx.co", (unsigned long long)hash, (unsigned long long)digest);
    const std::string path = cache_dir && *cache_dir ? std::string(cache_dir) + "/" + fname : "";
    JitCode code;
    if (path.empty() || !cache_load(path, code)) {
        if (int rc = compile(source_text(struct_name, model_source), inc, code, err)) return rc;
        if (!path.empty()) cache_store(path, code);
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_code.emplace(hash, std::move(code));
    if (!loaded_locked(hash)) {
        g_code.erase(hash);
        err = "loading the run-time code object failed (hipModuleLoadData / kernel lookup / LDS budget)";
        return TG_ERR_HIP;
    }
    return 0;
}

bool jit_has(uint64_t hash) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_code.count(hash) != 0;
}

int jit_kc(uint64_t hash) {
    JitLoaded *L = find(hash);
    return L ? L->meta.kc : -1;
}

int jit_launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    JitLoaded *L = find(hash);
    if (!L) return TG_ERR_MODEL;
    StepArgs aa = a;
    void *cargs[] = {&aa};
    if (!a.skip_compose)
        if (int rc = launch(L->f[K_COMPOSE], (unsigned)((a.N + JIT_COMPOSE_WPB - 1) / JIT_COMPOSE_WPB),
                            64 * JIT_COMPOSE_WPB, 0, stream, cargs))
            return rc;
    if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
    char pa = 0;   // the step kernel's empty NoPost::Args
    void *sargs[] = {&aa, &pa};
    const int e = L->meta.epb;
    if (int rc = launch(L->f[a.hf ? K_STEP_HF : K_STEP], (unsigned)((a.N + e - 1) / e), (unsigned)(e * L->meta.lpe),
                        (unsigned)L->meta.lds, stream, sargs))
        return rc;
    if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
    return 0;
}

int jit_launch_body_states(uint64_t hash, const float *root, const float *dof, int n, float *out, hipStream_t stream) {
    JitLoaded *L = find(hash);
    if (!L) return TG_ERR_MODEL;
    void *args[] = {&root, &dof, &n, &out};
    return launch(L->f[K_BODY], (unsigned)n, 64, 0, stream, args);
}

int jit_launch_rb_forces(uint64_t hash, const float *root, const float *dof, const float *comp, int n,
                         const float *mass_scale, const float *forces, const float *torques, int space, float *out,
                         const float *props, hipStream_t stream) {
    JitLoaded *L = find(hash);
    if (!L) return TG_ERR_MODEL;
    void *args[] = {&root, &dof, &comp, &n, &mass_scale, &forces, &torques, &space, &out, &props};
    return launch(L->f[K_RBF], (unsigned)((n + JIT_COMPOSE_WPB - 1) / JIT_COMPOSE_WPB), 64 * JIT_COMPOSE_WPB, 0, stream,
                  args);
}

}  // namespace tg
