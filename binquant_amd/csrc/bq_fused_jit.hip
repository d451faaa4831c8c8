// Native fused element-wise programs: each validated bq_fused_program is
// translated into straight-line HIP source (one SSA value per instruction,
// operand layouts specialised), compiled for gfx950 with hiprtc once per
// program STRUCTURE and launched as an ordinary kernel. Constants travel in
// the kernel arguments (exact doubles), not in the source: a stage called
// with new threshold values every message reuses its compiled kernel. The interpreter in bq_fused.hip decodes every instruction per
// element group and keeps program registers in LDS; here the compiler
// allocates VGPRs and schedules the loads, so a stage costs its HBM traffic
// plus the arithmetic, not the decode.
//
// Semantics are the interpreter's, operation for operation (same IEEE fp64
// expressions, -ffp-contract=off): tests/test_fused_gpu.py runs both and
// requires identical bits.
//
// Cache: compiled code objects are kept per process (key = generated source)
// and, when a cache directory is set (bq_fused_set_cache_dir), on disk under
// the FNV-1a hash of the source, so later processes skip the compile.
#include "bq_device.h"
#include "binquant_amd.h"
#include "bq_fused_jit.h"

#include <hip/hiprtc.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int JIT_NT = 256;   // threads per block; a block covers JIT_NT * K candles of one symbol

// kernel argument block (mirrored in the generated source)
struct JitArgs {
  const void* in[BQ_FUSED_MAX_IN];
  long long ss_in[BQ_FUSED_MAX_IN], st_in[BQ_FUSED_MAX_IN];
  void* out[BQ_FUSED_MAX_OUT];
  long long ss_out[BQ_FUSED_MAX_OUT], st_out[BQ_FUSED_MAX_OUT];
  double c[BQ_FUSED_MAX_CONST];
  int T, nbt;
};

const char* kArgsDecl =
    "struct JitArgs {\n"
    "  const void* in[" BQ_STR(BQ_FUSED_MAX_IN) "];\n"
    "  long long ss_in[" BQ_STR(BQ_FUSED_MAX_IN) "], st_in[" BQ_STR(BQ_FUSED_MAX_IN) "];\n"
    "  void* out[" BQ_STR(BQ_FUSED_MAX_OUT) "];\n"
    "  long long ss_out[" BQ_STR(BQ_FUSED_MAX_OUT) "], st_out[" BQ_STR(BQ_FUSED_MAX_OUT) "];\n"
    "  double c[" BQ_STR(BQ_FUSED_MAX_CONST) "];\n"
    "  int T, nbt;\n"
    "};\n";

// stride_t class of an operand: 1 (contiguous along t), 0 (one value per symbol), else general
int tclass(int64_t st) { return st == 1 ? 1 : st == 0 ? 0 : 2; }

std::string addr(const char* ss, const char* st, int cls, const std::string& t) {
  std::string s = std::string("sym * a.") + ss;
  if (cls == 1) return s + " + (long long)(" + t + ")";
  if (cls == 2) return s + " + (long long)(" + t + ") * a." + st;
  return s;
}

int arity(int op) {
  switch (op) {
    case BQ_F_LD: case BQ_F_CONST: case BQ_F_INRANGE: return 0;
    case BQ_F_NOT: case BQ_F_ABS: case BQ_F_NEG: case BQ_F_ISNAN: case BQ_F_SQRT: case BQ_F_LOG: case BQ_F_ST:
      return 1;
    case BQ_F_WHERE: return 3;
    default: return 2;
  }
}

// Generated source for the program: kernels bq_fk1 / bq_fk2 / bq_fk4 (K
// candles per thread at t = block start + k * 256 + thread). Every load of
// all K candles is issued before any arithmetic; then each candle's program
// runs and stores its outputs (the stores cannot alias a later load).
const char* kOpts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"};

std::string generate(const bq_fused_program& P) {
  std::string s;
  s.reserve(16384);
  // the compile options head the source (a comment), so they are part of the cache key
  s += "//";
  for (const char* o : kOpts) s += std::string(" ") + o;
  s += "\n";
  s += kArgsDecl;
  char b[512];
  // per-operand element readers
  for (int i = 0; i < P.n_in; ++i) {
    const bq_fused_operand& X = P.in[i];
    snprintf(b, sizeof b, "ss_in[%d]", i);
    std::string ss = b;
    snprintf(b, sizeof b, "st_in[%d]", i);
    std::string st = b;
    const std::string off = addr(ss.c_str(), st.c_str(), tclass(X.stride_t), "ts");
    if (X.dtype == BQ_F_U8)
      snprintf(b, sizeof b,
               "__device__ __forceinline__ double rd%d(const JitArgs& a, long long sym, int ts) "
               "{ return (double)(static_cast<const unsigned char*>(a.in[%d])[%s] != 0); }\n",
               i, i, off.c_str());
    else
      snprintf(b, sizeof b,
               "__device__ __forceinline__ double rd%d(const JitArgs& a, long long sym, int ts) "
               "{ return static_cast<const double*>(a.in[%d])[%s]; }\n",
               i, i, off.c_str());
    s += b;
  }
  s += "template <int K>\n__device__ __forceinline__ void body(const JitArgs& a) {\n";
  s += "  const int T = a.T;\n";
  s += "  const long long sym = blockIdx.x / a.nbt;\n";
  snprintf(b, sizeof b, "  const int t0 = (int)(blockIdx.x %% a.nbt) * (%d * K) + threadIdx.x;\n", JIT_NT);
  s += b;
  for (int j = 0; j < P.n_const; ++j) {
    snprintf(b, sizeof b, "  const double C%d = a.c[%d];\n", j, j);
    s += b;
  }
  // loads (every LD instruction, wherever the program placed it)
  for (int pc = 0; pc < P.n_ins; ++pc) {
    const uint64_t in = P.ins[pc];
    if ((int)(in & 0xff) != BQ_F_LD) continue;
    const int bi = (int)((in >> 24) & 0xff), ci = (int)((in >> 32) & 0xff);
    const int sh = (int)((int64_t)in >> 40);
    snprintf(b, sizeof b,
             "  double L%d[K];\n"
             "#pragma unroll\n"
             "  for (int k = 0; k < K; ++k) {\n"
             "    const int t = t0 + k * %d, ts = t - (%d);\n"
             "    L%d[k] = (t < T && ts >= 0 && ts < T) ? rd%d(a, sym, ts) : C%d;\n"
             "  }\n",
             pc, JIT_NT, sh, pc, bi, ci);
    s += b;
  }
  snprintf(b, sizeof b, "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n    const int t = t0 + k * %d;\n", JIT_NT);
  s += b;
  // SSA: register r currently holds value name[r]
  std::vector<std::string> name(BQ_FUSED_MAX_REGS > 256 ? BQ_FUSED_MAX_REGS : 256);
  for (int pc = 0; pc < P.n_ins; ++pc) {
    const uint64_t in = P.ins[pc];
    const int op = (int)(in & 0xff);
    const int d = (int)((in >> 8) & 0xff), ra = (int)((in >> 16) & 0xff), rb = (int)((in >> 24) & 0xff),
              rc = (int)((in >> 32) & 0xff);
    const int64_t imm = (int64_t)in >> 40;
    const int idx[3] = {ra, rb, rc};
    std::string o[3];
    if (op != BQ_F_LD && op != BQ_F_CONST && op != BQ_F_INRANGE && op != BQ_F_ST)
      for (int k = 0; k < arity(op); ++k) {
        snprintf(b, sizeof b, "C%d", idx[k]);
        o[k] = ((imm >> k) & 1) ? std::string(b) : name[idx[k]];
      }
    const std::string& u = o[0];
    const std::string& v = o[1];
    const std::string& w = o[2];
    std::string e;
    switch (op) {
      case BQ_F_LD: snprintf(b, sizeof b, "L%d[k]", pc); e = b; break;
      case BQ_F_CONST: snprintf(b, sizeof b, "C%d", (int)imm); e = b; break;
      case BQ_F_INRANGE:
        snprintf(b, sizeof b, "((t - (%d) >= 0 && t - (%d) < T) ? 1.0 : 0.0)", (int)imm, (int)imm);
        e = b;
        break;
      case BQ_F_ADD: e = u + " + " + v; break;
      case BQ_F_SUB: e = u + " - " + v; break;
      case BQ_F_MUL: e = u + " * " + v; break;
      case BQ_F_DIV: e = u + " / " + v; break;
      case BQ_F_NEG: e = "-" + u; break;
      case BQ_F_FMAX: e = "fmax(" + u + ", " + v + ")"; break;
      case BQ_F_FMIN: e = "fmin(" + u + ", " + v + ")"; break;
      case BQ_F_MAXIMUM:
        e = "((" + u + " != " + u + " || " + v + " != " + v + ") ? __builtin_nan(\"\") : (" + u + " > " + v +
            " ? " + u + " : " + v + "))";
        break;
      case BQ_F_MINIMUM:
        e = "((" + u + " != " + u + " || " + v + " != " + v + ") ? __builtin_nan(\"\") : (" + u + " < " + v +
            " ? " + u + " : " + v + "))";
        break;
      case BQ_F_GT: e = "((" + u + " > " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_GE: e = "((" + u + " >= " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_LT: e = "((" + u + " < " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_LE: e = "((" + u + " <= " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_EQ: e = "((" + u + " == " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_NE: e = "((" + u + " != " + v + ") ? 1.0 : 0.0)"; break;
      case BQ_F_AND: e = "((" + u + " != 0.0 && " + v + " != 0.0) ? 1.0 : 0.0)"; break;
      case BQ_F_OR: e = "((" + u + " != 0.0 || " + v + " != 0.0) ? 1.0 : 0.0)"; break;
      case BQ_F_NOT: e = "((" + u + " == 0.0) ? 1.0 : 0.0)"; break;
      case BQ_F_ABS: e = "fabs(" + u + ")"; break;
      case BQ_F_ISNAN: e = "((" + u + " != " + u + ") ? 1.0 : 0.0)"; break;
      case BQ_F_SQRT: e = "sqrt(" + u + ")"; break;
      case BQ_F_LOG: e = "log(" + u + ")"; break;
      case BQ_F_WHERE: e = "((" + u + " != 0.0) ? " + v + " : " + w + ")"; break;
      case BQ_F_ST: {
        const int oi = (int)imm;
        const bq_fused_operand& Y = P.out[oi];
        snprintf(b, sizeof b, "ss_out[%d]", oi);
        std::string ss = b;
        snprintf(b, sizeof b, "st_out[%d]", oi);
        std::string st = b;
        const std::string off = addr(ss.c_str(), st.c_str(), tclass(Y.stride_t), "t");
        if (Y.dtype == BQ_F_U8)
          snprintf(b, sizeof b, "    if (t < T) static_cast<unsigned char*>(a.out[%d])[%s] = %s != 0.0;\n", oi,
                   off.c_str(), name[ra].c_str());
        else
          snprintf(b, sizeof b, "    if (t < T) static_cast<double*>(a.out[%d])[%s] = %s;\n", oi, off.c_str(),
                   name[ra].c_str());
        s += b;
        continue;
      }
      default: e = "0.0"; break;
    }
    snprintf(b, sizeof b, "v%d", pc);
    name[d] = b;
    s += "    const double " + name[d] + " = " + e + ";\n";
  }
  s += "  }\n}\n";
  for (int K : {1, 2, 4}) {
    snprintf(b, sizeof b,
             "extern \"C\" __global__ __launch_bounds__(%d) void bq_fk%d(const JitArgs a) { body<%d>(a); }\n",
             JIT_NT, K, K);
    s += b;
  }
  return s;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// hiprtc compile; returns false (log in err) on failure
bool compile(const std::string& src, std::vector<char>& code, std::string& err) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "bq_fused_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)(sizeof kOpts / sizeof kOpts[0]), kOpts);
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    err.assign(n + 1, '\0');
    hiprtcGetProgramLog(prog, &err[0]);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.resize(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return true;
}

struct Entry {
  std::vector<char> code;
  std::unordered_map<int, std::pair<hipModule_t, hipFunction_t[3]>> mods;   // per device
};

std::mutex g_mu;
std::unordered_map<std::string, Entry>* g_cache = nullptr;
std::string g_dir;
int g_mode = -1;   // -1: from BQ_FUSED_NATIVE (default on), 0 interpreter, 1 native
long long g_compiles = 0, g_disk_hits = 0;

bool disk_read(const std::string& path, std::vector<char>& code) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  code.resize(n > 0 ? (size_t)n : 0);
  const bool ok = n > 0 && fread(code.data(), 1, (size_t)n, f) == (size_t)n;
  fclose(f);
  return ok;
}

void disk_write(const std::string& path, const std::vector<char>& code) {
  char tmp[64];
  snprintf(tmp, sizeof tmp, ".tmp.%d", (int)getpid());
  const std::string t = path + tmp;
  FILE* f = fopen(t.c_str(), "wb");
  if (!f) return;
  const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
  fclose(f);
  if (ok) rename(t.c_str(), path.c_str());   // atomic: concurrent processes see a whole file or none
  else remove(t.c_str());
}

// the code object for this source (process cache, disk cache, compile)
Entry* lookup(const std::string& src, std::string& err) {
  if (!g_cache) g_cache = new std::unordered_map<std::string, Entry>();
  auto it = g_cache->find(src);
  if (it != g_cache->end()) return &it->second;
  Entry e;
  std::string path;
  if (!g_dir.empty()) {
    char h[40];
    snprintf(h, sizeof h, "/%016llx.gfx950.co", (unsigned long long)fnv1a(src));
    path = g_dir + h;
    // the source is stored next to the code object: a hash collision is detected, not trusted
    std::vector<char> s;
    if (disk_read(path + ".src", s) && std::string(s.begin(), s.end()) == src && disk_read(path, e.code)) ++g_disk_hits;
    else e.code.clear();
  }
  if (e.code.empty()) {
    if (!compile(src, e.code, err)) return nullptr;
    ++g_compiles;
    if (!path.empty()) {
      disk_write(path, e.code);
      disk_write(path + ".src", std::vector<char>(src.begin(), src.end()));
    }
  }
  return &g_cache->emplace(src, std::move(e)).first->second;
}

}  // namespace

namespace bq {

bool fused_native_enabled() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_mode < 0) {
    const char* e = getenv("BQ_FUSED_NATIVE");
    g_mode = (e && e[0] == '0') ? 0 : 1;
  }
  return g_mode == 1;
}

int fused_native_eval(const bq_fused_program& P, int64_t S, int64_t T, hipStream_t stream) {
  const std::string src = generate(P);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return BQ_EHIP;
  hipFunction_t fn[3];
  {
    std::lock_guard<std::mutex> g(g_mu);
    std::string err;
    Entry* e = lookup(src, err);
    if (!e) {
      fprintf(stderr, "bq_fused_eval: native compile failed:\n%s\n", err.c_str());
      return BQ_EHIP;
    }
    auto m = e->mods.find(dev);
    if (m == e->mods.end()) {
      hipModule_t mod;
      if (hipModuleLoadData(&mod, e->code.data()) != hipSuccess) return BQ_EHIP;
      // resolve every entry before caching the module: a failure leaves no
      // half-initialised entry behind (and unloads the module)
      const char* names[3] = {"bq_fk1", "bq_fk2", "bq_fk4"};
      hipFunction_t got[3];
      for (int i = 0; i < 3; ++i)
        if (hipModuleGetFunction(&got[i], mod, names[i]) != hipSuccess) {
          (void)hipModuleUnload(mod);
          return BQ_EHIP;
        }
      auto& slot = e->mods[dev];
      slot.first = mod;
      for (int i = 0; i < 3; ++i) slot.second[i] = got[i];
      m = e->mods.find(dev);
    }
    for (int i = 0; i < 3; ++i) fn[i] = m->second.second[i];
  }
  // candles per thread: K loads of every operand are in flight per thread
  // before the arithmetic; short rows (live frames) keep one so no thread
  // idles on the tail
  int nld = 0;
  for (int pc = 0; pc < P.n_ins; ++pc) nld += (int)(P.ins[pc] & 0xff) == BQ_F_LD;
  const int K = T < 4 * JIT_NT ? 1 : nld <= 8 ? 4 : nld <= 24 ? 2 : 1;
  const int fi = K == 4 ? 2 : K == 2 ? 1 : 0;
  JitArgs A;
  memset(&A, 0, sizeof A);
  for (int i = 0; i < P.n_in; ++i) {
    A.in[i] = P.in[i].ptr;
    A.ss_in[i] = P.in[i].stride_s;
    A.st_in[i] = P.in[i].stride_t;
  }
  for (int i = 0; i < P.n_out; ++i) {
    A.out[i] = const_cast<void*>(P.out[i].ptr);
    A.ss_out[i] = P.out[i].stride_s;
    A.st_out[i] = P.out[i].stride_t;
  }
  memcpy(A.c, P.consts, sizeof(A.c));
  A.T = (int)T;
  const int span = JIT_NT * K;
  A.nbt = (int)((T + span - 1) / span);
  const int64_t blocks = S * A.nbt;
  if (blocks > 0x7fffffff) return BQ_EINVAL;
  void* params[] = {&A};
  if (hipModuleLaunchKernel(fn[fi], (unsigned)blocks, 1, 1, JIT_NT, 1, 1, 0, stream, params, nullptr) != hipSuccess)
    return BQ_EHIP;
  return BQ_OK;
}

}  // namespace bq

extern "C" {

int bq_fused_set_native(int on) {
  std::lock_guard<std::mutex> g(g_mu);
  const int prev = g_mode < 0 ? -1 : g_mode;
  g_mode = on < 0 ? -1 : (on ? 1 : 0);
  return prev;
}

int bq_fused_set_cache_dir(const char* dir) {
  std::lock_guard<std::mutex> g(g_mu);
  g_dir = dir ? dir : "";
  return BQ_OK;
}

int bq_fused_source(const bq_fused_program* P, char* buf, int64_t cap, int64_t* len) {
  if (!P || !len || bq::fused_validate(*P) != BQ_OK) return BQ_EINVAL;
  const std::string s = generate(*P);
  *len = (int64_t)s.size();
  if (buf && cap > 0) {
    const size_t n = s.size() < (size_t)(cap - 1) ? s.size() : (size_t)(cap - 1);
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return BQ_OK;
}

int bq_fused_compile(const bq_fused_program* P) {
  if (!P || bq::fused_validate(*P) != BQ_OK) return BQ_EINVAL;
  const std::string src = generate(*P);
  std::lock_guard<std::mutex> g(g_mu);
  std::string err;
  if (!lookup(src, err)) {
    fprintf(stderr, "bq_fused_compile: %s\n", err.c_str());
    return BQ_EHIP;
  }
  return BQ_OK;
}

int bq_fused_stats(int64_t* compiles, int64_t* disk_hits, int64_t* cached) {
  std::lock_guard<std::mutex> g(g_mu);
  if (compiles) *compiles = g_compiles;
  if (disk_hits) *disk_hits = g_disk_hits;
  if (cached) *cached = g_cache ? (int64_t)g_cache->size() : 0;
  return BQ_OK;
}

}  // extern "C"
