// mq_api.cpp — implementation of the C-ABI in include/mq.h (libmq.so).
//
// Host side of the quick-sat evaluator: owns the device copies of the candidate models
// (ModelCache contents, mythril/support/support_utils.py:56-58), compiles boundary tapes into
// GPU stack programs (tape_compiler.cpp) and launches the gfx950 kernels (qs_kernels.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mq.h"
#include "gprog.h"
#include "qs_launch.h"
#include "tape_compiler.h"

using namespace mq;

namespace {

inline int nl_of(int w) { return w == 0 ? 1 : (w + 31) / 32; }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 16));
    if (e == hipSuccess) bytes = std::max<size_t>(n, 16);
    return e;
  }
  template <class T>
  hipError_t upload(const T* src, size_t count, hipStream_t st) {
    hipError_t e = ensure(sizeof(T) * count);
    if (e != hipSuccess || count == 0) return e;
    return hipMemcpyAsync(p, src, sizeof(T) * count, hipMemcpyHostToDevice, st);
  }
  template <class T>
  T* as() const { return (T*)p; }
};

}  // namespace

struct mq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool have_models = false;
  // models
  int64_t M = 0, index_base = 0;
  int n_vars = 0, n_funcs = 0;
  std::vector<uint16_t> var_width;
  DevBuf vars, var_off, var_nl, funcs, entry_ptr, entry_words, else_words;
  DevBuf counters;
  DevBuf best_tmp;  // scratch first-hit buffer for the synchronous API
  DevBuf verdict_buf;
};

struct mq_tapes {
  mq_ctx* ctx = nullptr;
  int32_t n_tapes = 0;
  int32_t n_unsupported = 0;
  std::vector<uint8_t> unsupported;
  std::vector<uint32_t> n_nodes;
  std::vector<double> alg_ops;
  double total_nodes = 0, total_alg_ops = 0;
  DevBuf descs, prog, consts, unsup_dev;
  struct Variant {
    int L = 0;
    int begin = 0, count = 0;  // range in descs
    int max_temps = 0;
  };
  std::vector<Variant> variants;
};

static thread_local std::string g_last_error;

static int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return MQ_ERR_HIP;
}

#define HIPCHK(expr)                                   \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return hip_fail(_e, #expr); \
  } while (0)

extern "C" {

const char* mq_version(void) { return "mq 0.1.0 gfx950"; }

int mq_tape_compile_info(const mq_tape_batch* tb, int32_t t, int32_t* supported, int32_t* limbs, int32_t* depth,
                         int32_t* n_temps, int32_t* prog_words, char* why, int32_t why_len) {
  if (!tb || t < 0 || t >= tb->n_tapes) return MQ_ERR_ARG;
  CompileLimits lim;
  CompiledTape c = compile_tape(tb, t, lim);
  if (supported) *supported = c.supported ? 1 : 0;
  if (limbs) *limbs = c.L;
  if (depth) *depth = c.depth;
  if (n_temps) *n_temps = c.n_temps;
  if (prog_words) *prog_words = (int32_t)c.prog.size();
  if (why && why_len > 0) {
    std::strncpy(why, c.why.c_str(), (size_t)why_len - 1);
    why[why_len - 1] = 0;
  }
  return MQ_OK;
}

const char* mq_strerror(int code) {
  switch (code) {
    case MQ_OK: return "ok";
    case MQ_ERR_ARG: return "invalid argument";
    case MQ_ERR_HIP: return g_last_error.empty() ? "HIP runtime error" : g_last_error.c_str();
    case MQ_ERR_NOMEM: return "device out of memory";
    case MQ_ERR_NO_MODELS: return "no candidate models uploaded";
    case MQ_ERR_NODEV: return "no usable gfx950 device";
    case MQ_ERR_TAPE: return "malformed tape";
    case MQ_ERR_STATE: return "invalid context state";
    default: return "unknown error";
  }
}

int mq_ctx_create(int n_dev, const int* dev_ids, mq_ctx** out) {
  if (!out || n_dev != 1) return MQ_ERR_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return MQ_ERR_NODEV;
  int dev = dev_ids ? dev_ids[0] : 0;
  if (dev < 0 || dev >= count) return MQ_ERR_NODEV;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_last_error = std::string("device arch ") + prop.gcnArchName + " is not gfx950";
    return MQ_ERR_NODEV;
  }
  HIPCHK(hipSetDevice(dev));
  auto* c = new mq_ctx();
  c->device = dev;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    delete c;
    return MQ_ERR_HIP;
  }
  if (c->counters.ensure(4 * sizeof(unsigned long long)) != hipSuccess) {
    delete c;
    return MQ_ERR_NOMEM;
  }
  *out = c;
  return MQ_OK;
}

void mq_ctx_destroy(mq_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int mq_models_upload(mq_ctx* c, const mq_model_batch* mb) {
  if (!c || !mb || mb->n_models <= 0 || mb->n_vars < 0 || mb->n_funcs < 0) return MQ_ERR_ARG;
  if (mb->n_models > 0x7FFFFFFF || mb->index_base + mb->n_models > 0x7FFFFFFE) return MQ_ERR_ARG;
  HIPCHK(hipSetDevice(c->device));
  const int64_t M = mb->n_models;
  std::vector<uint32_t> voff(std::max(mb->n_vars, 1)), vnl(std::max(mb->n_vars, 1));
  int64_t rows = 0;
  for (int v = 0; v < mb->n_vars; v++) {
    voff[v] = (uint32_t)rows;
    vnl[v] = (uint32_t)nl_of(mb->var_width[v]);
    rows += vnl[v];
  }
  if (rows > 0 && !mb->var_words) return MQ_ERR_ARG;
  // functions: SoA else block, CSR entries copied as is
  const int F = mb->n_funcs;
  std::vector<FuncDev> fd(std::max(F, 1));
  std::vector<uint32_t> else_soa;
  int64_t ew_total = 0;
  for (int f = 0; f < F; f++) {
    const mq_func_desc& d = mb->funcs[f];
    if (d.arity < 1 || d.arity > 2) return MQ_ERR_ARG;
    FuncDev& x = fd[f];
    x.arity = d.arity;
    x.nl_a0 = nl_of(d.arg_width[0]);
    x.nl_a1 = d.arity > 1 ? nl_of(d.arg_width[1]) : 0;
    x.nl_res = nl_of(d.result_width);
    x.stride = x.nl_a0 + x.nl_a1 + x.nl_res;
    x.entry_base = mb->entry_base[f];
    x.ptr_base = (int64_t)f * (M + 1);
    x.else_base = (int64_t)else_soa.size();
    const uint32_t* ew = mb->else_words + mb->else_base[f];
    const size_t start = else_soa.size();
    else_soa.resize(start + (size_t)x.nl_res * M);
    for (int64_t m = 0; m < M; m++)
      for (uint32_t l = 0; l < x.nl_res; l++) else_soa[start + (size_t)l * M + m] = ew[m * x.nl_res + l];
    const int64_t last = mb->entry_base[f] + mb->entry_ptr[(int64_t)f * (M + 1) + M] * (int64_t)x.stride;
    if (last > mb->n_entry_words) return MQ_ERR_ARG;
    ew_total = std::max(ew_total, last);
  }
  if (else_soa.empty()) else_soa.push_back(0);
  c->have_models = false;
  HIPCHK(c->vars.upload(mb->var_words, (size_t)std::max<int64_t>(rows * M, 1), c->stream));
  HIPCHK(c->var_off.upload(voff.data(), voff.size(), c->stream));
  HIPCHK(c->var_nl.upload(vnl.data(), vnl.size(), c->stream));
  HIPCHK(c->funcs.upload(fd.data(), fd.size(), c->stream));
  if (F > 0) {
    HIPCHK(c->entry_ptr.upload(mb->entry_ptr, (size_t)F * (M + 1), c->stream));
    HIPCHK(c->entry_words.upload(mb->entry_words, (size_t)std::max<int64_t>(ew_total, 1), c->stream));
  } else {
    int64_t z = 0;
    uint32_t zw = 0;
    HIPCHK(c->entry_ptr.upload(&z, 1, c->stream));
    HIPCHK(c->entry_words.upload(&zw, 1, c->stream));
  }
  HIPCHK(c->else_words.upload(else_soa.data(), else_soa.size(), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->M = M;
  c->index_base = mb->index_base;
  c->n_vars = mb->n_vars;
  c->n_funcs = F;
  c->var_width.assign(mb->var_width, mb->var_width + mb->n_vars);
  c->have_models = true;
  return MQ_OK;
}

int mq_tapes_upload(mq_ctx* c, const mq_tape_batch* tb, mq_tapes** out, int32_t* n_unsup_out) {
  if (!c || !tb || !out || tb->n_tapes < 0 || (tb->n_tapes > 0 && (!tb->tape_offsets || !tb->nodes))) return MQ_ERR_ARG;
  *out = nullptr;
  HIPCHK(hipSetDevice(c->device));
  auto T = std::make_unique<mq_tapes>();
  T->ctx = c;
  T->n_tapes = tb->n_tapes;
  T->unsupported.assign(std::max(tb->n_tapes, 1), 0);
  T->n_nodes.assign(tb->n_tapes, 0);
  T->alg_ops.assign(tb->n_tapes, 0);
  CompileLimits lim;
  std::vector<CompiledTape> ct(tb->n_tapes);
  for (int t = 0; t < tb->n_tapes; t++) {
    if (tb->tape_offsets[t + 1] < tb->tape_offsets[t]) return MQ_ERR_ARG;
  }
  // compile (independent per tape)
#pragma omp parallel for schedule(dynamic, 64)
  for (int t = 0; t < tb->n_tapes; t++) ct[t] = compile_tape(tb, t, lim);
  // order descriptors by variant (L)
  std::vector<uint32_t> prog, consts;
  std::vector<GDesc> descs;
  for (int L : {8, 16}) {
    mq_tapes::Variant v;
    v.L = L;
    v.begin = (int)descs.size();
    for (int t = 0; t < tb->n_tapes; t++) {
      const CompiledTape& x = ct[t];
      if (!x.supported || x.L != L) continue;
      GDesc d{};
      d.prog_off = (uint32_t)prog.size();
      d.prog_len = (uint32_t)x.prog.size();
      d.tape = (uint32_t)t;
      d.const_base = (uint32_t)consts.size();
      d.n_nodes = x.n_nodes;
      d.n_temps = (uint32_t)x.n_temps;
      d.depth = (uint32_t)x.depth;
      d.alg_ops = (uint32_t)std::min(x.alg_ops, 4.0e9);
      prog.insert(prog.end(), x.prog.begin(), x.prog.end());
      consts.insert(consts.end(), x.consts.begin(), x.consts.end());
      // pad so that the scalar loads of the last constant never run past the buffer
      descs.push_back(d);
      v.max_temps = std::max(v.max_temps, x.n_temps);
    }
    v.count = (int)descs.size() - v.begin;
    if (v.count) T->variants.push_back(v);
  }
  consts.resize(consts.size() + 16, 0);
  prog.push_back(gword(G_END, 0, 0));
  for (int t = 0; t < tb->n_tapes; t++) {
    T->unsupported[t] = ct[t].supported ? 0 : 1;
    T->n_unsupported += ct[t].supported ? 0 : 1;
    T->n_nodes[t] = ct[t].n_nodes;
    T->alg_ops[t] = ct[t].alg_ops;
  }
  if (descs.empty()) descs.push_back(GDesc{});
  HIPCHK(T->descs.upload(descs.data(), descs.size(), c->stream));
  HIPCHK(T->prog.upload(prog.data(), prog.size(), c->stream));
  HIPCHK(T->consts.upload(consts.data(), consts.size(), c->stream));
  HIPCHK(T->unsup_dev.upload(T->unsupported.data(), T->unsupported.size(), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (n_unsup_out) *n_unsup_out = T->n_unsupported;
  *out = T.release();
  return MQ_OK;
}

void mq_tapes_free(mq_tapes* t) { delete t; }

static KArgs make_args(mq_ctx* c, mq_tapes* T, const mq_tapes::Variant& v) {
  KArgs a{};
  a.descs = T->descs.as<GDesc>() + v.begin;
  a.n_desc = v.count;
  const int64_t tiles = (c->M + 255) / 256;
  // ~8k workgroups: enough to fill 256 CUs many times over with a short tail
  int64_t tpg = (int64_t(v.count) * tiles + 8191) / 8192;
  tpg = std::max<int64_t>(1, std::min<int64_t>(tpg, v.count));
  a.tapes_per_group = (int)tpg;
  a.prog = T->prog.as<uint32_t>();
  a.consts = T->consts.as<uint32_t>();
  a.vars = c->vars.as<uint32_t>();
  a.var_off = c->var_off.as<uint32_t>();
  a.var_nl = c->var_nl.as<uint32_t>();
  a.n_vars = c->n_vars;
  a.n_funcs = c->n_funcs;
  a.funcs = c->funcs.as<FuncDev>();
  a.entry_ptr = c->entry_ptr.as<int64_t>();
  a.entry_words = c->entry_words.as<uint32_t>();
  a.else_words = c->else_words.as<uint32_t>();
  a.M = c->M;
  a.index_base = c->index_base;
  a.counters = c->counters.as<unsigned long long>();
  a.tmp_words_per_wave = v.max_temps * v.L * 64;
  a.early_exit = 1;
  return a;
}

int mq_launch_first_hit(mq_ctx* c, mq_tapes* T, int32_t* d_best, void* stream) {
  if (!c || !T || !d_best) return MQ_ERR_ARG;
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  if (T->ctx != c) return MQ_ERR_STATE;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(launch_init_best(d_best, T->n_tapes, st));
  for (const auto& v : T->variants) {
    KArgs a = make_args(c, T, v);
    a.best = d_best;
    HIPCHK(launch_qs(a, v.L, false, st));
  }
  return MQ_OK;
}

int mq_finalize_first_hit(mq_ctx* c, mq_tapes* T, int32_t* d_best, void* stream) {
  if (!c || !T || !d_best) return MQ_ERR_ARG;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(launch_finalize_best(d_best, T->unsup_dev.as<uint8_t>(), T->n_tapes, st));
  return MQ_OK;
}

int mq_counters(mq_ctx* c, double* out3, int reset) {
  if (!c || !out3) return MQ_ERR_ARG;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());
  unsigned long long cnt[3] = {0, 0, 0};
  HIPCHK(hipMemcpy(cnt, c->counters.p, sizeof(cnt), hipMemcpyDeviceToHost));
  for (int i = 0; i < 3; i++) out3[i] = (double)cnt[i];
  if (reset) HIPCHK(hipMemset(c->counters.p, 0, 4 * sizeof(unsigned long long)));
  return MQ_OK;
}

int mq_eval_tapes_first_hit(mq_ctx* c, mq_tapes* T, int32_t* out, mq_stats* stats) {
  if (!c || !T || (!out && T->n_tapes)) return MQ_ERR_ARG;
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  HIPCHK(hipSetDevice(c->device));
  if (T->n_tapes == 0) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    return MQ_OK;
  }
  HIPCHK(c->best_tmp.ensure(sizeof(int32_t) * T->n_tapes));
  HIPCHK(hipMemsetAsync(c->counters.p, 0, 4 * sizeof(unsigned long long), c->stream));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  int rc = mq_launch_first_hit(c, T, c->best_tmp.as<int32_t>(), c->stream);
  if (rc) return rc;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  rc = mq_finalize_first_hit(c, T, c->best_tmp.as<int32_t>(), c->stream);
  if (rc) return rc;
  unsigned long long cnt[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(out, c->best_tmp.p, sizeof(int32_t) * T->n_tapes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(cnt, c->counters.p, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (stats) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    stats->kernel_ms = ms;
    stats->pairs_evaluated = (int64_t)cnt[0];
    stats->node_evals = (double)cnt[1];
    stats->alg_ops = (double)cnt[2];  // exact: per evaluated (tape, model) pair, the tape's cost
    int hits = 0;
    for (int t = 0; t < T->n_tapes; t++) hits += out[t] >= 0;
    stats->n_hits = hits;
    stats->n_unsupported = T->n_unsupported;
  }
  return MQ_OK;
}

int mq_eval_first_hit(mq_ctx* c, const mq_tape_batch* tb, int32_t* out, mq_stats* stats) {
  mq_tapes* T = nullptr;
  int rc = mq_tapes_upload(c, tb, &T, nullptr);
  if (rc) return rc;
  rc = mq_eval_tapes_first_hit(c, T, out, stats);
  mq_tapes_free(T);
  return rc;
}

int mq_eval_verdicts(mq_ctx* c, const mq_tape_batch* tb, uint8_t* bits, int32_t* first_hit_out) {
  if (!c || !tb || !bits) return MQ_ERR_ARG;
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  mq_tapes* T = nullptr;
  int rc = mq_tapes_upload(c, tb, &T, nullptr);
  if (rc) return rc;
  std::unique_ptr<mq_tapes> guard(T);
  const size_t nbytes = (size_t)T->n_tapes * (size_t)c->M;
  HIPCHK(c->verdict_buf.ensure(std::max<size_t>(nbytes, 1)));
  HIPCHK(hipMemsetAsync(c->verdict_buf.p, 0, std::max<size_t>(nbytes, 1), c->stream));
  for (const auto& v : T->variants) {
    KArgs a = make_args(c, T, v);
    a.verdicts = c->verdict_buf.as<uint8_t>();
    a.early_exit = 0;
    HIPCHK(launch_qs(a, v.L, true, c->stream));
  }
  std::vector<uint8_t> host(nbytes);
  if (nbytes) HIPCHK(hipMemcpyAsync(host.data(), c->verdict_buf.p, nbytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  std::memset(bits, 0, (nbytes + 7) / 8);
  for (size_t i = 0; i < nbytes; i++)
    if (host[i]) bits[i >> 3] |= (uint8_t)(1u << (i & 7));
  if (first_hit_out) {
    for (int t = 0; t < T->n_tapes; t++) {
      int32_t h = -1;
      if (T->unsupported[t]) h = -2;
      else
        for (int64_t m = 0; m < c->M; m++)
          if (host[(size_t)t * c->M + m]) {
            h = (int32_t)(c->index_base + m);
            break;
          }
      first_hit_out[t] = h;
    }
  }
  return MQ_OK;
}

double mq_tape_alg_ops(const mq_tape_batch* tb, int32_t t) {
  if (!tb || t < 0 || t >= tb->n_tapes) return -1;
  return tape_alg_ops(tb, t);
}

int mq_keccak256(mq_ctx* c, const uint8_t* data, const int64_t* offsets, int32_t n, uint8_t* out) {
  if (!c || (n > 0 && (!data || !offsets || !out)) || n < 0) return MQ_ERR_ARG;
  if (n == 0) return MQ_OK;
  HIPCHK(hipSetDevice(c->device));
  const int64_t total = offsets[n];
  DevBuf d_data, d_off, d_out;
  HIPCHK(d_data.upload(data, (size_t)std::max<int64_t>(total, 1), c->stream));
  HIPCHK(d_off.upload(offsets, (size_t)n + 1, c->stream));
  HIPCHK(d_out.ensure((size_t)32 * n));
  HIPCHK(launch_keccak(d_data.as<uint8_t>(), d_off.as<int64_t>(), n, d_out.as<uint8_t>(), c->stream));
  HIPCHK(hipMemcpyAsync(out, d_out.p, (size_t)32 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MQ_OK;
}

}  // extern "C"
