// mq_api.cpp — implementation of the C-ABI in include/mq.h (libmq.so).
//
// Host side of the quick-sat evaluator: owns the device copies of the candidate models
// (ModelCache contents, mythril/support/support_utils.py:56-58), compiles boundary tapes into
// GPU stack programs (tape_compiler.cpp) and launches the gfx950 kernels (qs_kernels.hip).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <pthread.h>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <unordered_set>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mq.h"
#include "gprog.h"
#include "qs_launch.h"
#include "qsa_table.h"
#include "tape_compiler.h"
#include "host_keccak.h"

using namespace mq;

namespace {

inline int nl_of(int w) { return w == 0 ? 1 : (w + 31) / 32; }

// Device allocations are cached per device by size class instead of going back to hipFree: the
// drop-in path builds a fresh mq_tapes (a dozen buffers) per query batch, and a hipMalloc /
// hipFree pair per buffer (hipFree synchronises the device) cost more than compiling the batch.
// A released block may be handed out again at once, so whoever releases a buffer must have
// ordered the kernels that read it before any later use: every product path synchronises its
// stream before freeing (mq_tapes_free, mq_ctx_destroy).
class DevPool {
 public:
  static DevPool& get() {
    static DevPool* p = new DevPool();
    return *p;
  }
  static size_t size_class(size_t n) {
    n = std::max<size_t>(n, 256);
    if (n <= (size_t(64) << 20)) {
      size_t c = 256;
      while (c < n) c <<= 1;
      return c;
    }
    const size_t g = size_t(2) << 20;
    return (n + g - 1) / g * g;
  }
  void* take(int dev, size_t cls) {
    std::lock_guard<std::mutex> g(mu_);
    auto& fl = free_[dev & 15];
    auto it = fl.find(cls);
    if (it == fl.end()) return nullptr;
    void* p = it->second;
    fl.erase(it);
    cached_[dev & 15] -= cls;
    return p;
  }
  // a kernel was launched on a caller's stream (mq_launch_first_hit): a block released on this
  // device may still be read there, so the next release synchronises the device first (what
  // hipFree would have done)
  void mark_foreign(int dev) { foreign_[dev & 15].store(true); }
  // the library's own streams per device (each context's), so a growing buffer drains those
  // instead of the whole device
  void register_stream(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> g(mu_);
    streams_[dev & 15].push_back(s);
  }
  void unregister_stream(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> g(mu_);
    auto& v = streams_[dev & 15];
    v.erase(std::remove(v.begin(), v.end(), s), v.end());
  }
  // before a block is handed out again: the library's streams on dev are drained, and the device
  // when a caller's stream may hold a reader (mark_foreign)
  void drain(int dev) {
    if (foreign_[dev & 15].load()) {
      (void)hipDeviceSynchronize();
      return;
    }
    std::vector<hipStream_t> v;
    {
      std::lock_guard<std::mutex> g(mu_);
      v = streams_[dev & 15];
    }
    for (hipStream_t s : v) (void)hipStreamSynchronize(s);
  }
  void put(int dev, void* p, size_t cls) {
    if (foreign_[dev & 15].exchange(false)) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(dev);
      (void)hipDeviceSynchronize();
      (void)hipSetDevice(cur);
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (cached_[dev & 15] + cls <= kMaxCached) {
        free_[dev & 15].emplace(cls, p);
        cached_[dev & 15] += cls;
        return;
      }
    }
    (void)hipFree(p);
  }
  void trim(int dev) {   // give the cached blocks back (an allocation failed)
    std::multimap<size_t, void*> fl;
    {
      std::lock_guard<std::mutex> g(mu_);
      fl.swap(free_[dev & 15]);
      cached_[dev & 15] = 0;
    }
    for (auto& kv : fl) (void)hipFree(kv.second);
  }

 private:
  static constexpr size_t kMaxCached = size_t(4) << 30;
  std::mutex mu_;
  std::multimap<size_t, void*> free_[16];
  size_t cached_[16] = {};
  std::atomic<bool> foreign_[16] = {};
  std::vector<hipStream_t> streams_[16];
};

// page-locked host staging (readbacks of small batches skip the runtime's pageable bounce)
struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    size_t want = 4096;
    while (want < n) want *= 2;
    const hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) bytes = want;
    return e;
  }
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int dev = 0;
  bool own = true;   // false: a view into another buffer (UploadPack), released with it
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes), dev(o.dev), own(o.own) {
    o.p = nullptr;
    o.bytes = 0;
    o.own = true;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      dev = o.dev;
      own = o.own;
      o.p = nullptr;
      o.bytes = 0;
      o.own = true;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p && own) DevPool::get().put(dev, p, bytes);
    p = nullptr;
    bytes = 0;
    own = true;
  }
  void set_view(void* q, size_t n) {
    release();
    p = q;
    bytes = n;
    own = false;
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    // growing: a kernel queued on one of the library's streams (or a caller's) may still read the
    // old block, and the pool hands it out again at once -- drain those first (growth is rare:
    // size classes double)
    if (p) DevPool::get().drain(dev);
    release();
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return e;
    const size_t cls = DevPool::size_class(n);
    p = DevPool::get().take(d, cls);
    if (!p) {
      e = hipMalloc(&p, cls);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        DevPool::get().trim(d);
        e = hipMalloc(&p, cls);
      }
      if (e != hipSuccess) {
        p = nullptr;
        return e;
      }
    }
    bytes = cls;
    dev = d;
    return hipSuccess;
  }
  template <class T>
  hipError_t upload(const T* src, size_t count, hipStream_t st) {
    hipError_t e = ensure(sizeof(T) * count);
    if (e != hipSuccess || count == 0) return e;
    return hipMemcpyAsync(p, src, sizeof(T) * count, hipMemcpyHostToDevice, st);
  }
  // the same through the staging ring (StageRing, defined below): the source may be freed at once
  template <class T, class Ring>
  hipError_t upload_staged(const T* src, size_t count, hipStream_t st, Ring& ring) {
    hipError_t e = ensure(sizeof(T) * count);
    if (e != hipSuccess || count == 0) return e;
    const size_t n = sizeof(T) * count;
    void* h = n <= Ring::kMaxStaged ? ring.put(src, n, st) : nullptr;
    if (!h) {
      e = hipMemcpyAsync(p, src, n, hipMemcpyHostToDevice, st);
      return e != hipSuccess ? e : hipStreamSynchronize(st);
    }
    return hipMemcpyAsync(p, h, n, hipMemcpyHostToDevice, st);
  }
  template <class T>
  T* as() const { return (T*)p; }
};

// Small host-to-device uploads of the drop-in path (tape tables, translated programs, argument
// blocks: ~10 per query batch) through a page-locked ring: the copy is a DMA from pinned memory
// that the host does not wait for, so the stream syncs that kept pageable sources alive until
// their copy ran are gone (profiles/r06f: 10 pageable hipMemcpyAsync + ~6 stream syncs per batch,
// ~0.14 ms of a 0.23 ms batch).  A source is staged at the ring's head; when the ring is full the
// streams that copied out of it are drained and it starts over (every ~8 MB of uploads).
struct StageRing {
  static constexpr size_t kMaxStaged = size_t(256) << 10;   // larger uploads: pageable + a sync
  static constexpr size_t kBytes = size_t(8) << 20;
  PinnedBuf buf;
  size_t head = 0;
  std::vector<hipStream_t> used;
  // pinned copy of src (n <= kMaxStaged; src nullptr: n bytes the caller fills) for an async copy
  // on st; nullptr: stage failed
  void* put(const void* src, size_t n, hipStream_t st) {
    if (!buf.p && buf.ensure(kBytes) != hipSuccess) return nullptr;
    const size_t a = (n + 255) & ~size_t(255);
    if (head + a > buf.bytes) {
      for (hipStream_t s : used)
        if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
      used.clear();
      head = 0;
    }
    if (std::find(used.begin(), used.end(), st) == used.end()) used.push_back(st);
    void* d = (char*)buf.p + head;
    if (src) std::memcpy(d, src, n);
    head += a;
    return d;
  }
};

// Several small host arrays copied to the device as ONE block (one staged copy instead of one
// copy each: the drop-in path's per-batch tables); the DevBufs become views into it.  The block
// DevBuf must outlive its views (both live in the same mq_tapes).
struct UploadPack {
  std::vector<uint8_t> host;
  struct V {
    DevBuf* buf;
    size_t off, bytes;
  };
  std::vector<V> views;
  // (pad: that many zero elements after the copied ones, inside the view)
  template <class T>
  void add(DevBuf& v, const T* src, size_t count, size_t pad = 0) {
    const size_t off = (host.size() + 255) & ~size_t(255), n = sizeof(T) * count, b = std::max<size_t>(n + sizeof(T) * pad, 1);
    host.resize(off + b, 0);
    if (n) std::memcpy(host.data() + off, src, n);
    views.push_back(V{&v, off, b});
  }
  hipError_t commit(DevBuf& block, hipStream_t st, StageRing& ring) {
    for (const V& x : views) x.buf->release();   // (views of the previous block, if any)
    const hipError_t e = block.upload_staged(host.data(), host.size(), st, ring);
    if (e != hipSuccess) return e;
    for (const V& x : views) x.buf->set_view((char*)block.p + x.off, x.bytes);
    return hipSuccess;
  }
};

}  // namespace

// words past the function entries that reads may touch (8 entries of the widest G table)
static constexpr size_t kEntryPadWords = 512;
// most entry slots per model a function may have to get dense lookup slots (FuncDev dense_e)
static constexpr int64_t kDenseMaxE = 16;

// the assembly interpreter keeps temps in LDS (2 KB per temp per wave, 4 waves per workgroup)
static constexpr int kQsaMaxTemps = 16;

// HIP C++ interpreter variants (qs_kernels.hip launch_qs): limbs per stack slot and whether the
// variant carries the interpreted-keccak handler.  Kind 0 (L = 8) is where 256-bit tapes the
// assembly interpreters cannot take run; 32 / 64 limbs hold the > 512-bit values of keccak
// inputs longer than 64 bytes (Concat / Extract / EQ / ITE / UF keys) and always carry keccak.
static constexpr int kGen = 5;
static constexpr int kGenL[kGen] = {8, 16, 16, 32, 64};
static constexpr bool kGenK[kGen] = {false, false, true, true, true};
static int gen_kind(const CompiledTape& x) {
  if (x.L == 8) return 0;
  if (x.L == 16) return x.keccak ? 2 : 1;
  return x.L == 32 ? 3 : 4;
}
static constexpr int64_t kColAsmMinNodes = 1;    // hoisted columns on qsg_kernel from this size

// Guards every context's live_tapes and every mq_tapes::ctx: a batch freed on one thread while
// its context is destroyed on another must not read the context after it is deleted.
static std::mutex g_live_mu;

// mq_keccak256 hashes a batch of at most this many 136-byte blocks on the host (measured crossover
// against one launch + two copies: profiles/r05*/bench_c2.json keccak_service)
static constexpr int64_t kKeccakHostBlocks = 128;

struct mq_ctx {
  // compiled batches made on this context, detached (ctx = nullptr) when it is destroyed first:
  // mq_tapes_free after mq_ctx_destroy must not touch the freed context (a Python finalizer may
  // run in either order); both under g_live_mu
  std::unordered_set<mq_tapes*> live_tapes;
  // per model function: the most table entries any model of the WHOLE batch holds (all shards):
  // a wide-key lookup (MQ_OP_UF_WIDE) tracks at most 64 entries per model
  std::vector<int64_t> func_max_entries;
  uint64_t batch_gen = 0;   // bumped by every mq_models_upload (all devices of a context alike)
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // a column level's kernels are independent of each other (a column reads only lower levels):
  // the keccak columns run on aux[0], the bit-gather and flat columns on aux[1], next to the
  // interpreters on the launch stream, forked and joined per level with these events
  hipStream_t aux[2] = {nullptr, nullptr};
  hipEvent_t fork_ev = nullptr, join_ev[2] = {nullptr, nullptr};
  bool have_models = false;
  // models
  int64_t M = 0, index_base = 0;
  int n_vars = 0, n_funcs = 0;
  std::vector<uint16_t> var_width;
  DevBuf vars, var_off, var_nl, funcs, entry_ptr, entry_words, else_words, dense_words;
  int64_t entry_words_n = 0;   // words of function entries (G scans them with 32-bit offsets)
  DevBuf counters;
  DevBuf best_tmp;  // scratch first-hit buffer for the synchronous API
  DevBuf scratch;   // per-wave temp slots of the HIP C++ interpreter (persistent grid)
  DevBuf kec_data, kec_off, kec_out;   // mq_keccak256 buffers, grown and kept across calls
  DevBuf rowmask;   // per-row masks applied to uploaded variable words
  DevBuf mpack;     // UploadPack block of the model batch's small tables (upload_one: the views above point in)
  // Bool variables as packed lane masks [tile][n_bmask] (G kernel PUSH_PKB): bmask_of_var[v] =
  // mask index of Bool variable v (-1: none); bmask_rows[j] = its variable row
  std::vector<int32_t> bmask_of_var;
  int32_t n_bmask = 0;
  DevBuf bmasks, bmask_rows;
  DevBuf prof;   // G profile build (kQsaProfBytes > 0): per-kind (cycles, count), mq_qsa_profile
  DevBuf prof_sink;   // ... the launches MQ_PROF_LEVEL leaves out write here
  DevBuf verdict_buf;
  PinnedBuf verdict_host;   // verdict bytes read back (batches up to kPinnedVerdictBytes)
  PinnedBuf readback_host;  // a first-hit launch's counter slots and first hits
  StageRing stage;          // small uploads (DevBuf::upload_staged)
  hipEvent_t stage_ev = nullptr;   // a launch on a caller's stream waits for the context stream's copies
  // assembly interpreters (qsa.hip): handler byte offsets read back at context creation;
  // k = 0 the P kernel (preloaded variables), k = 1 the G kernel (general)
  bool qsa_ready = false;
  std::vector<uint32_t> qsa_off[2];
  int qsa_index[2][QK_COUNT][kQsaStack][kQsaSel + 1];
  // G kinds that wait for every vector load themselves (PUSH_MEMB, MEQK*, UF1*)
  bool qsa_vm_drain[QK_COUNT] = {};
  uint32_t qsa_var_row[64];
  std::vector<uint8_t> qsa_data_words;
  uint32_t qsa_hbase_lo[2] = {0, 0};   // low 32 bits of each interpreter's handler base
  std::vector<int16_t> qsa_kind_of[2];  // handler byte offset / 4 -> QsaKind (histograms)
  DevBuf qsa_args;
  // host copies of the model batch layout the QSA translation depends on
  std::vector<uint32_t> var_off_h, var_nl_h;
  std::vector<mq_func_desc> funcs_h;
  uint64_t models_gen = 0;      // bumped by every mq_models_upload
  // bumped by an upload whose layout differs from the previous batch's (variables and their
  // widths, Bool lane-mask indices, function signatures): the tape translations, column plans and
  // keccak maps depend on the layout only, so a drop-in batch that differs in its models (a solver
  // model inserted, another LRU subset) keeps them
  uint64_t layout_gen = 0;
  std::vector<uint8_t> layout_sig;
  int use_asm = 1;      // MQ_OPT_USE_ASM
  int early_exit = 1;   // MQ_OPT_EARLY_EXIT
  int64_t latency_waves = 0;   // MQ_OPT_LATENCY_WAVES
  int64_t keccak_host_blocks = kKeccakHostBlocks;   // MQ_OPT_KECCAK_HOST_BLOCKS
  // MQ_OPT_TIME_KERNELS: one HIP event pair bracketing the evaluation kernels of each launch
  int time_kernels = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kev;
  size_t kev_used = 0;
  // ... and, on a context that reduces in-library (comms), per launch: the event pair around the
  // ncclGroup of the MIN all-reduce on the lead stream, the host milliseconds the launch call
  // spent issuing every device's kernels and the reduce, and those of the peers' launch loop
  // (mq_launch_times)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> rev;
  size_t rev_used = 0;
  std::vector<double> issue_ms, peer_issue_ms;
  // Several devices from one process (mq_ctx_create(n_dev > 1)): this context is
  // the lead (dev_ids[0]); peers[i] is a single-device context on dev_ids[i + 1].  The candidate
  // axis is split contiguously over [lead, peers...] (shard_lo[g] = first local model of device
  // g); per-tape first hits are combined by an in-library RCCL MIN all-reduce (comms, lead first).
  double host_t[MQ_HOST_PHASES] = {};   // mq_host_times
  std::vector<mq_ctx*> peers;
  std::vector<ncclComm_t> comms;
  std::vector<int64_t> shard_lo;
  int64_t M_total = 0;
};

struct FcaPlanSeg {   // one fca_kernel launch (fca_plan)
  int atom_off, n_atoms, group_off, n_groups, tape_first, n_tapes, chunk_first, smask_off, n_smask;
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
  // wide-key lookups (MQ_OP_UF_WIDE): per tape the functions, the compile-time unsupported flags,
  // and the batch the flags were last re-derived for (a function with more than kWideMaxEntries
  // entries in some model makes its tapes unsupported under that batch)
  std::vector<std::vector<uint32_t>> wide_funcs;
  std::vector<uint8_t> unsupported_base;
  bool wide_any = false;
  uint64_t wide_gen = ~0ull;
  struct Variant {
    int L = 0;
    int begin = 0, count = 0;  // range in descs
    int max_temps = 0;
    int max_depth = 1;
    bool keccak = false;
  };
  // descs layout: [L8 QSA-eligible | gen[0] (L8 other) | gen[1..] (wider kinds)]; the QSA view
  // (qdescs/qprog) holds the eligible tapes translated to threaded code.  The translation depends
  // on the model batch (variable rows, function table), so it is redone at launch when the models
  // changed: each eligible tape goes to the P kernel (only preloaded variables) or the G kernel.
  Variant l8_all, qsa;
  Variant gen[kGen];                         // HIP C++ interpreter kinds (kGenL / kGenK)
  std::vector<CompiledTape> qct;             // compiled programs of the QSA-eligible tapes
  std::vector<GDesc> qbase;                  // their descriptors (const_base into consts)
  uint64_t qsa_gen = ~0ull;                  // layout_gen of the current translation
  bool qsa_live = false;                     // the translation succeeded for every tape
  int q_count[2] = {0, 0}, q_temps[2] = {0, 0};
  // G kernel preload for the current translation: gpre[var] = VGPR slot (or -1) of the (at
  // most 8) variables the G tapes push most; g_var_row = their limb rows (QArgs.var_row)
  std::vector<int> gpre;
  uint32_t g_var_row[64];
  // G rows staged in LDS per workgroup: gstage[var] = LDS slot of its first limb row (or -1),
  // stage_rows = global row of every slot (padded to a multiple of 8 with the zero row)
  std::vector<int> gstage;
  std::vector<uint32_t> stage_rows;
  DevBuf stage_dev;
  // handler-kind histograms of the current translation (mq_tapes_qsa_histogram): [0] P tapes,
  // [1] G tapes, [2] G column programs; qpairs = (kind, next kind) counts over the G tapes,
  // qpairs_p over the P tapes
  std::vector<int64_t> qhist[3], qpairs, qpairs_p;
  DevBuf qdescs, qprog, qargs[2];
  QArgs qargs_dev_copy[2];   // what qargs[k] currently holds on the device
  bool qargs_valid[2] = {false, false};
  // batch-level hoisting: column programs evaluated once per model before the tapes, one
  // launch per (nesting level, kernel variant); GDesc.tape = the model variable written
  // v8 begins with the v8q columns the G assembly interpreter can take (structurally); when
  // their translation for the current model batch succeeds (cq_live) they run on qsg_kernel in
  // mode 3 and the HIP C++ column kernel takes the rest of v8
  struct ColumnLevel {
    Variant v[kGen];    // v[0]: L = 8 (its first v8q columns are the G-eligible ones)
    int v8q = 0;
    int cq_begin = 0;   // first of the level's columns in cq_ct / cqdescs
  };
  std::vector<ColumnLevel> clevels;
  std::vector<int32_t> col_var, col_width, col_level;
  // per column level: mask indices of its Bool columns, repacked after the level ran
  std::vector<std::vector<int32_t>> lvl_bmask_h;
  std::vector<DevBuf> lvl_bmask;
  // the same for the Bool columns NOT on the G column path (when it runs, G stores its Bool
  // columns' masks itself: gen_qsa.py store_column)
  std::vector<std::vector<int32_t>> lvl_bmask_cpp_h;
  std::vector<DevBuf> lvl_bmask_cpp;
  uint64_t bmask_gen = ~0ull;
  DevBuf cdescs, cprog, cconsts;
  std::vector<CompiledTape> cq_ct;   // the G-eligible columns, level by level
  std::vector<int32_t> cq_var;
  std::vector<uint8_t> cq_bool;
  uint64_t cq_gen = ~0ull;
  bool cq_live = false;
  DevBuf cqdescs, cqprog, cqconsts, cqargs;
  std::vector<QArgs> cqargs_host;   // what cqargs holds on the device, per level
  std::vector<uint32_t> cq_stage_rows;                   // staged rows of every level, level by level
  std::vector<uint32_t> cq_lvl_stage_off, cq_lvl_stage_n;  // per level: its rows in cq_stage_rows
  std::vector<int> cq_lvl_temps;                         // per level: LDS temp slots
  DevBuf cq_stage_dev;
  // keccak columns (launch_keccak_columns): columns that are exactly keccak(concat of variables
  // and constants); per column its pieces, most significant first (var >= 0: a model variable of
  // nl limbs; var < 0: nl constant limbs at kc_consts[coff]); grouped by level
  struct KcPiece {
    int32_t var;
    uint32_t nl, coff;
  };
  struct KcPredHost {   // a Bool column h OP c evaluated from the keccak column's digest
    int32_t target;
    uint32_t kind, bits;
    uint32_t c[8];
  };
  struct KcHost {
    int32_t target;
    uint32_t n_nodes, alg_ops;   // (its predicate columns' included)
    std::vector<KcPiece> pieces;
    std::vector<KcPredHost> preds;
  };
  std::vector<KcHost> kc;
  std::vector<uint32_t> kc_consts;
  std::vector<std::pair<int, int>> kc_level;   // (first, count) in kc, per column level
  uint64_t kc_gen = ~0ull;                      // layout_gen of the uploaded map
  DevBuf kc_cols_dev, kc_map_dev, kc_pred_dev;
  // bit-gather columns (cw.hip, cw_compile): columns that are an arrangement of variable bits and
  // constants, runs gated by `i <s size` (calldata words); per output limb its slots
  struct CwSlotHost {
    int32_t var;
    uint32_t vlimb, mask, shifts, gate;
  };
  struct CwHost {
    int32_t target = -1, size_var = -1;   // size_var -1: no gated slot
    uint32_t n_nodes = 0, alg_ops = 0;
    std::vector<std::vector<CwSlotHost>> limb_slots;
    std::vector<uint32_t> const_or;
  };
  std::vector<CwHost> cw;
  std::vector<std::pair<int, int>> cw_level;   // (first, count) in cw, per column level
  uint64_t cw_gen = ~0ull;
  DevBuf cw_cols_dev, cw_chunks_dev;
  std::vector<char> col_direct_mask;            // per column: its lane masks are stored by its kernel
  // flat conjunctions (fc.hip): QSA-eligible tapes that are an AND of Bool variables and
  // variable-constant compares, run on fc_kernel instead of P / G (per model batch: qsa_prepare)
  int fc_count = 0;
  int fc_stage_n = 0, fc_smask_n = 0;
  DevBuf fc_tapes_dev, fc_mask_dev, fc_cmp_dev, fc_stage_dev, fc_smask_dev, fc_prefix_dev;
  // the two-phase form (fca_kernel; MQ_FC_ONEPHASE=1: fc_kernel): atoms in fc_cmp_dev, lists in
  // fc_mask_dev
  bool fca = false;
  bool fca_any_xf = false;   // the tape plan has unary atoms (FcaPlan::any_xf)
  int fca_atoms = 0;
  std::vector<FcaPlanSeg> fca_segs;
  DevBuf fca_chunk_dev, fca_out_dev, fca_metric_dev, fca_group_dev, fca_xf_dev;
  // the G-eligible Bool columns of a level that are flat (fc_match) run on fc_kernel, mode 3,
  // before the level's G launch (cq_prepare); the level's G descriptors are the others
  struct FcLevel {   // fca_kernel mode 3 (fca_plan per level)
    int count = 0;
    bool any_xf = false;   // (FcaPlan::any_xf)
    std::vector<FcaPlanSeg> segs;
    DevBuf atoms, xfs, groups, lists, chunk, out, metric, smask, colmask;
  };
  std::vector<std::unique_ptr<FcLevel>> fc_lvl;
  std::vector<int> cq_lvl_desc_off, cq_lvl_desc_n;
  std::vector<uint32_t> cq_group_tab, cq_lvl_tab_off;   // per level: its G groups' descriptor bounds
  std::vector<int> cq_lvl_groups;
  DevBuf cq_group_dev;
  // multi-device context: the same batch compiled on each peer device (ctx->peers order)
  std::vector<mq_tapes*> peers;
  DevBuf pack0, pack1;   // UploadPack blocks: the upload's tables / qsa_prepare's (the views above point in)
  bool in_flight = false;   // copies or launches the host has not waited for (mq_tapes_free)
  ~mq_tapes() {
    for (mq_tapes* p : peers) delete p;
    std::lock_guard<std::mutex> g(g_live_mu);
    if (ctx) ctx->live_tapes.erase(this);
  }
};

static thread_local std::string g_last_error;

static constexpr size_t kCounterBytes = sizeof(unsigned long long) * kCounterSlots * kCounterStride;

// the three work counters, summed over the slots (qs_launch.h)
static void sum_counter_slots(const std::vector<unsigned long long>& raw, unsigned long long out[3]) {
  out[0] = out[1] = out[2] = 0;
  for (int s = 0; s < kCounterSlots; s++)
    for (int i = 0; i < 3; i++) out[i] += raw[(size_t)s * kCounterStride + i];
}

// Host-side parallel loop over independent items (tape compilation): std::threads pulling
// chunks off a shared counter.  Threads: MQ_HOST_THREADS, else OMP_NUM_THREADS, else the
// hardware concurrency, at most 64.  (No OpenMP runtime: the library shares its process with
// torch's own.)
// The workers are created once and park on a condition variable between calls: a drop-in query
// compiles a few dozen tapes, and spawning threads per call cost more than the compilation.
// set in a thread while it runs a pool job (a nested parallel_for runs serially: run() holds
// call_mu_), and in a forked child (the pool's workers do not exist there)
static thread_local bool tl_in_pool = false;
static std::atomic<bool> g_forked_child{false};
struct InPool {   // tl_in_pool for a job's extent, cleared when the job throws too
  InPool() { tl_in_pool = true; }
  ~InPool() { tl_in_pool = false; }
};

class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = [] {
      pthread_atfork(nullptr, nullptr, [] { g_forked_child.store(true); });
      return new HostPool();   // (never destroyed: workers may outlive static dtors)
    }();
    return *p;
  }
  int threads() const { return n_; }
  // run job(tid) on tids 0 .. k-1 (0 on the caller), return when all are done
  void run(int k, const std::function<void(int)>& job) {
    std::lock_guard<std::mutex> serial(call_mu_);   // one parallel region at a time
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &job;
      want_ = k - 1;
      done_ = 0;
      epoch_++;
    }
    cv_.notify_all();
    {
      InPool in;
      job(0);
    }
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return done_ == want_; });
    job_ = nullptr;
  }

 private:
  HostPool() {
    n_ = [] {
      for (const char* v : {"MQ_HOST_THREADS", "OMP_NUM_THREADS"})
        if (const char* e = std::getenv(v)) {
          const int t = std::atoi(e);
          if (t > 0) return std::min(t, 64);
        }
      return (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
    }();
    for (int t = 1; t < n_; t++) std::thread([this, t] { loop(t); }).detach();
  }
  void loop(int tid) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return epoch_ != seen; });
        seen = epoch_;
        if (tid > want_) continue;   // not needed this time
        job = job_;
      }
      {
        InPool in;
        (*job)(tid);
      }
      std::lock_guard<std::mutex> g(mu_);
      if (++done_ == want_) done_cv_.notify_one();
    }
  }
  int n_ = 1;
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int want_ = 0, done_ = 0;
  uint64_t epoch_ = 0;
};

template <class F>
static void parallel_for(int64_t n, int64_t chunk, F&& fn) {
  if (tl_in_pool || g_forked_child.load(std::memory_order_relaxed)) {   // nested, or no workers
    fn(0, 0, n);
    return;
  }
  HostPool& pool = HostPool::get();
  const int T = (int)std::min<int64_t>(pool.threads(), (n + chunk - 1) / std::max<int64_t>(chunk, 1));
  if (T <= 1) {
    fn(0, 0, n);
    return;
  }
  std::atomic<int64_t> next{0};
  const std::function<void(int)> work = [&](int tid) {
    for (;;) {
      const int64_t b = next.fetch_add(chunk);
      if (b >= n) break;
      fn(tid, b, std::min(n, b + chunk));
    }
  };
  pool.run(T, work);
}

// adds the scope's wall time to ctx->host_t[phase] (mq_host_times)
struct PhaseTimer {
  double* acc;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit PhaseTimer(double* a) : acc(a) {}
  ~PhaseTimer() { *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};

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

int mq_tape_compile_info_g(const mq_tape_batch* tb, int32_t t, int32_t* depth_g, int32_t* n_temps_g,
                           int32_t* prog_words_g) {
  if (!tb || t < 0 || t >= tb->n_tapes) return MQ_ERR_ARG;
  CompileLimits lim;
  lim.g_depth = kQsaStackG;
  lim.value_root = true;   // (a hoisted column program reports like a tape)
  CompiledTape c = compile_tape(tb, t, lim);
  if (!c.supported) return MQ_ERR_TAPE;
  const bool alt = !c.prog_g.empty();
  if (depth_g) *depth_g = alt ? c.depth_g : c.depth;
  if (n_temps_g) *n_temps_g = alt ? c.n_temps_g : c.n_temps;
  if (prog_words_g) *prog_words_g = (int32_t)(alt ? c.prog_g.size() : c.prog.size());
  return MQ_OK;
}

int mq_tape_program(const mq_tape_batch* tb, int32_t t, uint32_t* words, int32_t cap, int32_t* n_words) {
  if (!tb || t < 0 || t >= tb->n_tapes || !n_words) return MQ_ERR_ARG;
  CompileLimits lim;
  CompiledTape c = compile_tape(tb, t, lim);
  if (!c.supported) return MQ_ERR_TAPE;
  *n_words = (int32_t)c.prog.size();
  if (words && cap >= (int32_t)c.prog.size()) std::memcpy(words, c.prog.data(), c.prog.size() * sizeof(uint32_t));
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

// Handler byte offset -> the 16-bit word field that encodes it: P / G handlers are 4-byte
// aligned (shift 2); the diagnostic G profile build aligns them to 8 bytes (shift 3, 512 KB reach)
static inline uint32_t hword(int k, uint32_t off) { return off >> (k == 1 ? kQsaHandlerShiftG : 2); }

// Read back the byte offset of every handler of the assembly interpreters (kernel mode 2).
static int qsa_init(mq_ctx* c) {
  bool ok = true;
  for (int k = 0; k < 2; k++) {
    const int nh = k == 0 ? kQsaHandlersP : kQsaHandlersG;
    static_assert(kQsaStackP <= kQsaStack && kQsaStackG <= kQsaStack, "qsa_index holds both stacks");
    const QsaHandlerKey* keys = k == 0 ? kQsaHandlerKeysP : kQsaHandlerKeysG;
    for (int q = 0; q < QK_COUNT; q++)
      for (int d = 0; d < kQsaStack; d++)
        for (int v = 0; v <= kQsaSel; v++) c->qsa_index[k][q][d][v] = -1;
    for (int h = 0; h < nh; h++) c->qsa_index[k][keys[h].kind][keys[h].d < 0 ? 0 : keys[h].d][keys[h].v + 1] = h;
    DevBuf table;   // nh handler offsets, then the absolute handler base (lo, hi)
    HIPCHK(table.ensure(sizeof(uint32_t) * (nh + 2)));
    HIPCHK(hipMemsetAsync(table.p, 0xFF, sizeof(uint32_t) * (nh + 2), c->stream));
    QArgs qa{};
    qa.table_out = table.as<uint32_t>();
    qa.mode = 2;
    HIPCHK(c->qsa_args.upload(&qa, 1, c->stream));
    HIPCHK(launch_qsa(k, c->qsa_args.as<QArgs>(), 1, 1, 0, c->stream));
    c->qsa_off[k].resize(nh + 2);
    HIPCHK(hipMemcpyAsync(c->qsa_off[k].data(), table.p, sizeof(uint32_t) * (nh + 2), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->qsa_hbase_lo[k] = c->qsa_off[k][nh];
    c->qsa_kind_of[k].assign(1 << 16, -1);
    for (int h = 0; h < nh; h++)
      if (hword(k, c->qsa_off[k][h]) < (1u << 16)) c->qsa_kind_of[k][hword(k, c->qsa_off[k][h])] = (int16_t)keys[h].kind;
    uint32_t max_off = 0;
    for (int h = 0; h < nh; h++) {
      ok = ok && c->qsa_off[k][h] != 0xFFFFFFFFu && hword(k, c->qsa_off[k][h]) < (1u << 16) &&
           (c->qsa_off[k][h] & ((k == 1 ? (1u << kQsaHandlerShiftG) : 4u) - 1)) == 0;
      max_off = std::max(max_off, c->qsa_off[k][h]);
    }
    // P program entries and G's decoded program window hold the low 32 bits of absolute handler
    // addresses: they must share the high half (the kernels keep it in s19)
    ok = ok && (uint64_t)c->qsa_hbase_lo[k] + max_off < (1ull << 32);
    c->qsa_off[k].resize(nh);
  }
  // G handler word index -> inline data words that follow it (generated: the window words the
  // handler body reads, gen_qsa.py handler_data_words)
  c->qsa_data_words.assign(1 << 16, 0);
  for (int h = 0; ok && h < kQsaHandlersG; h++)
    if (kQsaHandlerDataWordsG[h] > 0) c->qsa_data_words[hword(1, c->qsa_off[1][h]) & 0xFFFFu] = kQsaHandlerDataWordsG[h];
  for (int q = 0; q < QK_COUNT; q++) {
    const std::string n = kQsaKindNames[q];
    c->qsa_vm_drain[q] = n == "PUSH_MEMB" || n.rfind("MEQK", 0) == 0 || n.rfind("UF1", 0) == 0;
  }
  c->qsa_ready = ok && std::getenv("MQ_DISABLE_QSA") == nullptr;
  return MQ_OK;
}

static int create_one(int dev, mq_ctx** out) {
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return MQ_ERR_NODEV;
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
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux[0], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux[1], hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->join_ev[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->join_ev[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming) != hipSuccess) {
    mq_ctx_destroy(c);
    return MQ_ERR_HIP;
  }
  DevPool::get().register_stream(dev, c->stream);
  DevPool::get().register_stream(dev, c->aux[0]);
  DevPool::get().register_stream(dev, c->aux[1]);
  if (c->counters.ensure(kCounterBytes) != hipSuccess) {
    mq_ctx_destroy(c);
    return MQ_ERR_NOMEM;
  }
  int rc = qsa_init(c);
  if (rc) {
    mq_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return MQ_OK;
}

static int rccl_fail(ncclResult_t r, const char* what) {
  g_last_error = std::string(what) + ": " + ncclGetErrorString(r);
  return MQ_ERR_HIP;
}

// One RCCL communicator per device of the context (lead first), single process: ncclCommInitAll.
static int rccl_init(mq_ctx* c) {
  if (!c->comms.empty()) return MQ_OK;
  std::vector<int> devs{c->device};
  for (mq_ctx* p : c->peers) devs.push_back(p->device);
  std::vector<ncclComm_t> comms(devs.size());
  ncclResult_t r = ncclCommInitAll(comms.data(), (int)devs.size(), devs.data());
  if (r != ncclSuccess) return rccl_fail(r, "ncclCommInitAll");
  c->comms = comms;
  return MQ_OK;
}

// [lead, peers...]
static std::vector<mq_ctx*> devices_of(mq_ctx* c) {
  std::vector<mq_ctx*> v{c};
  v.insert(v.end(), c->peers.begin(), c->peers.end());
  return v;
}

int mq_ctx_create(int n_dev, const int* dev_ids, mq_ctx** out) {
  if (!out || n_dev < 1 || (n_dev > 1 && !dev_ids)) return MQ_ERR_ARG;
  *out = nullptr;
  for (int i = 0; i < n_dev; i++)
    for (int j = 0; j < i; j++)
      if (dev_ids[i] == dev_ids[j]) return MQ_ERR_ARG;   // one context per device
  mq_ctx* lead = nullptr;
  int rc = create_one(dev_ids ? dev_ids[0] : 0, &lead);
  if (rc) return rc;
  for (int i = 1; i < n_dev; i++) {
    mq_ctx* p = nullptr;
    rc = create_one(dev_ids[i], &p);
    if (rc) {
      mq_ctx_destroy(lead);
      return rc;
    }
    lead->peers.push_back(p);
  }
  if (n_dev > 1) {
    rc = rccl_init(lead);
    if (rc) {
      mq_ctx_destroy(lead);
      return rc;
    }
  }
  *out = lead;
  return MQ_OK;
}

void mq_ctx_destroy(mq_ctx* c) {
  if (!c) return;
  for (ncclComm_t cm : c->comms) (void)ncclCommDestroy(cm);
  c->comms.clear();
  for (mq_ctx* p : c->peers) mq_ctx_destroy(p);
  c->peers.clear();
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (hipStream_t a : c->aux)
    if (a) {
      (void)hipStreamSynchronize(a);
      (void)hipStreamDestroy(a);
      DevPool::get().unregister_stream(c->device, a);
    }
  if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
  if (c->stage_ev) (void)hipEventDestroy(c->stage_ev);
  for (hipEvent_t e : c->join_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (auto& e : c->kev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  for (auto& e : c->rev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  DevPool::get().unregister_stream(c->device, c->stream);
  {
    std::lock_guard<std::mutex> g(g_live_mu);
    for (mq_tapes* t : c->live_tapes) t->ctx = nullptr;   // their launches were synchronised above
    c->live_tapes.clear();
    delete c;
  }
}

// Upload a model batch to ONE device (n_models may be 0: an empty shard evaluates to "no hit").
static int upload_one(mq_ctx* c, const mq_model_batch* mb) {
  if (!c || !mb || mb->n_models < 0 || mb->n_vars < 0 || mb->n_funcs < 0) return MQ_ERR_ARG;
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
  // dense lookup slots for the G interpreter's table scan (gen_qsa.py sub_uf1): functions of one
  // argument whose per-model entry count is small (keccak inverse tables, C4) get every model's
  // entries as slot-major SoA rows as well, so the 64 lanes of a wave probing slot e read one
  // coalesced row per key limb instead of 64 scattered entries.  MQ_NO_DENSE_TABLES=1: off.
  std::vector<uint32_t> dense;
  {
    const bool no_dense = std::getenv("MQ_NO_DENSE_TABLES") != nullptr;
    for (int f = 0; f < F && !no_dense && M > 0; f++) {
      FuncDev& x = fd[f];
      if (x.arity != 1 || x.nl_a0 > 8 || x.nl_res > 8) continue;
      const int64_t* ep = mb->entry_ptr + (int64_t)f * (M + 1);
      int64_t emax = 0;
      for (int64_t m = 0; m < M; m++) emax = std::max(emax, ep[m + 1] - ep[m]);
      const int64_t total = ep[M] - ep[0];
      const int64_t words = emax * (int64_t)(x.nl_a0 + x.nl_res) * M;
      // bounded: at most kDenseMaxE slots, and not much more memory than the CSR entries
      if (emax == 0 || emax > kDenseMaxE || words > 2 * total * (int64_t)x.stride + 16 * M) continue;
      x.dense_e = (uint32_t)emax;
      x.dense_base = (int64_t)dense.size();
      dense.resize(dense.size() + (size_t)words, 0);
      uint32_t* kd = dense.data() + x.dense_base;
      uint32_t* vd = kd + (size_t)emax * x.nl_a0 * M;
      const uint32_t* base = mb->entry_words + mb->entry_base[f];
      for (int64_t m = 0; m < M; m++)
        for (int64_t e = 0; e < ep[m + 1] - ep[m]; e++) {
          const uint32_t* ent = base + (ep[m] + e) * (int64_t)x.stride;
          for (uint32_t l = 0; l < x.nl_a0; l++) kd[((size_t)e * x.nl_a0 + l) * M + m] = ent[l];
          for (uint32_t l = 0; l < x.nl_res; l++) vd[((size_t)e * x.nl_res + l) * M + m] = ent[x.nl_a0 + l];
        }
    }
  }
  if (dense.empty()) dense.push_back(0);
  c->have_models = false;
  // the batch's small tables (row masks, Bool mask rows, variable offsets / limbs, functions,
  // entries, else values, dense slots) go up as ONE staged block (UploadPack: c->mpack, the
  // buffers below views into it); the variable rows, which can be large, stay a buffer of their own
  UploadPack pk;
  // variable rows followed by one all-zero row (the QSA preload points absent limbs at it)
  HIPCHK(c->vars.ensure(sizeof(uint32_t) * (size_t)(rows + 1) * M));
  {
    const size_t n = sizeof(uint32_t) * (size_t)rows * M, nz = sizeof(uint32_t) * (size_t)M;
    if (n + nz <= StageRing::kMaxStaged) {
      // (a drop-in batch's rows are a few KB: the rows and the zero row in one staged copy, no sync)
      void* h = c->stage.put(nullptr, n + nz, c->stream);
      if (h) {
        if (n) std::memcpy(h, mb->var_words, n);
        std::memset((char*)h + n, 0, nz);
        HIPCHK(hipMemcpyAsync(c->vars.p, h, n + nz, hipMemcpyHostToDevice, c->stream));
      } else {
        if (n) HIPCHK(hipMemcpyAsync(c->vars.p, mb->var_words, n, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemsetAsync((uint32_t*)c->vars.p + (size_t)rows * M, 0, nz, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
      }
    } else {
      // a large batch: pageable + a sync
      if (n) HIPCHK(hipMemcpyAsync(c->vars.p, mb->var_words, n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemsetAsync((uint32_t*)c->vars.p + (size_t)rows * M, 0, nz, c->stream));
      if (n) HIPCHK(hipStreamSynchronize(c->stream));
    }
  }
  // canonical values: bits above a variable's width are cleared on the device (the kernels
  // and the asm interpreter read rows unmasked)
  std::vector<uint32_t> rowmask((size_t)rows + 1, 0xFFFFFFFFu);
  bool need_mask = false;
  for (int v = 0; v < mb->n_vars; v++) {
    const int w = mb->var_width[v];
    const uint32_t top = w == 0 ? 1u : ((w % 32) ? ((1u << (w % 32)) - 1u) : 0xFFFFFFFFu);
    if (top != 0xFFFFFFFFu) {
      rowmask[voff[v] + vnl[v] - 1] = top;
      need_mask = true;
    }
  }
  if (need_mask) pk.add(c->rowmask, rowmask.data(), rowmask.size());
  // P kernel preload rows: var v < 8, limb l (the zero row where absent; a variable wider
  // than 256 bits is never preloaded: the translator sends its tapes to the G kernel)
  for (int v = 0; v < 8; v++)
    for (int l = 0; l < 8; l++) {
      uint32_t row = (uint32_t)rows;  // zero row
      if (v < mb->n_vars && mb->var_width[v] <= 256 && (uint32_t)l < vnl[v]) row = voff[v] + l;
      c->qsa_var_row[8 * v + l] = row;
    }
  // Bool variables as lane masks (at most 65535 of them; the others are read as rows;
  // MQ_BMASK_CAP lowers the cap so tests reach the row path)
  std::vector<uint32_t> brows;
  {
    c->bmask_of_var.assign(mb->n_vars, -1);
    size_t cap = 65535;
    if (const char* e = std::getenv("MQ_BMASK_CAP")) cap = std::min<size_t>(cap, (size_t)std::atol(e));
    for (int v = 0; v < mb->n_vars && brows.size() < cap; v++)
      if (mb->var_width[v] == 0) {
        c->bmask_of_var[v] = (int32_t)brows.size();
        brows.push_back(voff[v]);
      }
    c->n_bmask = (int32_t)brows.size();
    const int64_t tiles = (M + 63) / 64;
    HIPCHK(c->bmasks.ensure(std::max<size_t>(8, sizeof(uint64_t) * (size_t)tiles * brows.size())));
    if (brows.empty()) brows.push_back(0);
    pk.add(c->bmask_rows, brows.data(), brows.size());
  }
  c->var_off_h.assign(voff.begin(), voff.begin() + mb->n_vars);
  c->var_nl_h.assign(vnl.begin(), vnl.begin() + mb->n_vars);
  c->funcs_h.assign(mb->funcs, mb->funcs + F);
  c->entry_words_n = F > 0 ? ew_total : 0;
  c->models_gen++;
  {
    std::vector<uint8_t> sig;
    auto put = [&](const void* p, size_t n) {
      const uint8_t* b = (const uint8_t*)p;
      sig.insert(sig.end(), b, b + n);
    };
    const int32_t nv = mb->n_vars;
    put(&nv, sizeof nv);
    put(mb->var_width, sizeof(uint16_t) * (size_t)nv);
    put(c->bmask_of_var.data(), sizeof(int32_t) * c->bmask_of_var.size());
    put(&F, sizeof F);
    put(c->funcs_h.data(), sizeof(mq_func_desc) * c->funcs_h.size());
    const uint8_t fits = (uint64_t)(c->entry_words_n + (int64_t)kEntryPadWords) * 4 < (1ull << 32) ? 1 : 0;
    put(&fits, 1);
    if (sig != c->layout_sig) {
      c->layout_sig.swap(sig);
      c->layout_gen++;
    }
  }
  pk.add(c->var_off, voff.data(), voff.size());
  pk.add(c->var_nl, vnl.data(), vnl.size());
  pk.add(c->funcs, fd.data(), fd.size());
  if (F > 0) {
    pk.add(c->entry_ptr, mb->entry_ptr, (size_t)F * (M + 1));
    // (padded: G's table scan reads the first word of up to 7 entries past a model's last one,
    // gen_qsa.py sub_uf1)
    pk.add(c->entry_words, mb->entry_words, (size_t)std::max<int64_t>(ew_total, 1), kEntryPadWords);
  } else {
    const int64_t z = 0;
    const uint32_t zw = 0;
    pk.add(c->entry_ptr, &z, 1);
    pk.add(c->entry_words, &zw, 1, kEntryPadWords);
  }
  pk.add(c->else_words, else_soa.data(), else_soa.size());
  pk.add(c->dense_words, dense.data(), dense.size());
  HIPCHK(pk.commit(c->mpack, c->stream, c->stage));
  if (need_mask) HIPCHK(launch_mask_rows(c->vars.as<uint32_t>(), c->rowmask.as<uint32_t>(), rows, M, c->stream));
  HIPCHK(launch_pack_bool(c->vars.as<uint32_t>(), c->bmasks.as<uint64_t>(), c->bmask_rows.as<uint32_t>(), nullptr,
                          c->n_bmask, c->n_bmask, M, c->stream));
  c->M = M;
  c->index_base = mb->index_base;
  c->n_vars = mb->n_vars;
  c->n_funcs = F;
  c->var_width.assign(mb->var_width, mb->var_width + mb->n_vars);
  c->have_models = true;
  return MQ_OK;
}

// Models [lo, hi) of mb as a batch of their own (global index base + lo).  Variable rows and the
// entries of every function are packed into `keep`; else values are a view into mb.
struct ShardBuffers {
  std::vector<uint32_t> var_words, entry_words;
  std::vector<int64_t> entry_ptr, entry_base, else_base;
};
static mq_model_batch shard_view(const mq_model_batch* mb, int64_t lo, int64_t hi, ShardBuffers& keep) {
  const int64_t M = mb->n_models, Ms = hi - lo;
  mq_model_batch s = *mb;
  s.n_models = Ms;
  s.index_base = mb->index_base + lo;
  int64_t rows = 0;
  for (int v = 0; v < mb->n_vars; v++) rows += nl_of(mb->var_width[v]);
  keep.var_words.resize((size_t)std::max<int64_t>(rows * Ms, 1));
  for (int64_t r = 0; r < rows; r++)
    std::memcpy(keep.var_words.data() + r * Ms, mb->var_words + r * M + lo, sizeof(uint32_t) * (size_t)Ms);
  s.var_words = keep.var_words.data();
  const int F = mb->n_funcs;
  keep.entry_ptr.assign((size_t)F * (Ms + 1) + 1, 0);
  keep.entry_base.assign((size_t)F + 1, 0);
  keep.else_base.assign((size_t)F + 1, 0);
  keep.entry_words.clear();
  for (int f = 0; f < F; f++) {
    const mq_func_desc& d = mb->funcs[f];
    int64_t stride = nl_of(d.result_width);
    for (int i = 0; i < d.arity && i < 2; i++) stride += nl_of(d.arg_width[i]);
    const int64_t* ptr = mb->entry_ptr + (int64_t)f * (M + 1);
    const int64_t a = ptr[lo], b = ptr[hi];
    keep.entry_base[f] = (int64_t)keep.entry_words.size();
    const uint32_t* src = mb->entry_words + mb->entry_base[f] + a * stride;
    keep.entry_words.insert(keep.entry_words.end(), src, src + (b - a) * stride);
    for (int64_t m = 0; m <= Ms; m++) keep.entry_ptr[(size_t)f * (Ms + 1) + m] = ptr[lo + m] - a;
    keep.else_base[f] = mb->else_base[f] + lo * nl_of(d.result_width);
  }
  if (keep.entry_words.empty()) keep.entry_words.push_back(0);
  s.entry_ptr = keep.entry_ptr.data();
  s.entry_base = keep.entry_base.data();
  s.entry_words = keep.entry_words.data();
  s.n_entry_words = (int64_t)keep.entry_words.size();
  s.else_base = keep.else_base.data();
  return s;
}

int mq_models_shard(const mq_model_batch* mb, int64_t lo, int64_t hi, mq_model_batch* out, void** handle) {
  if (!mb || !out || !handle || lo < 0 || hi < lo || hi > mb->n_models || mb->n_funcs < 0 || mb->n_vars < 0)
    return MQ_ERR_ARG;
  auto* keep = new ShardBuffers();
  *out = shard_view(mb, lo, hi, *keep);
  *handle = keep;
  return MQ_OK;
}

void mq_models_shard_free(void* handle) { delete static_cast<ShardBuffers*>(handle); }

static constexpr int64_t kWideMaxEntries = 64;

int mq_models_upload(mq_ctx* c, const mq_model_batch* mb) {
  if (!c || !mb || mb->n_models < 0) return MQ_ERR_ARG;
  PhaseTimer pt(&c->host_t[8]);
  {
    std::vector<int64_t> mx((size_t)std::max(mb->n_funcs, 0), 0);
    if (mb->entry_ptr)
      for (int f = 0; f < mb->n_funcs; f++) {
        const int64_t* p = mb->entry_ptr + (int64_t)f * (mb->n_models + 1);
        for (int64_t m = 0; m < mb->n_models; m++) mx[f] = std::max(mx[f], p[m + 1] - p[m]);
      }
    for (mq_ctx* d : devices_of(c)) {
      d->func_max_entries = mx;
      d->batch_gen++;
    }
  }
  if (c->peers.empty()) {
    c->shard_lo.assign(1, 0);
    c->M_total = mb->n_models;
    return upload_one(c, mb);
  }
  // contiguous model-axis shards in global candidate order; a device whose range
  // is empty (fewer models than devices) holds zero models and reports no hit
  const std::vector<mq_ctx*> devs = devices_of(c);
  const int64_t G = (int64_t)devs.size(), M = mb->n_models;
  std::vector<int64_t> lo(G);
  for (int64_t g = 0; g < G; g++) {
    lo[g] = M * g / G;
    const int64_t hi = M * (g + 1) / G;
    ShardBuffers keep;
    const mq_model_batch sb = shard_view(mb, lo[g], hi, keep);
    const int rc = upload_one(devs[g], &sb);
    if (rc) return rc;
  }
  c->shard_lo = lo;
  c->M_total = M;
  return MQ_OK;
}

// G profile build: the zeroed per-kind (cycles, count) accumulator, nullptr in product builds.
// level: the launch's column level, -1 for the tape launch; MQ_PROF_LEVEL=k (diagnostic) keeps
// only column level k's launch ("t": the tape launch), the others accumulate into a sink.
static unsigned long long* prof_buffer(mq_ctx* c, int level) {
  if (kQsaProfBytes <= 0) return nullptr;
  if (!c->prof.p) {
    if (c->prof.ensure((size_t)kQsaProfBytes) != hipSuccess) return nullptr;
    if (hipMemset(c->prof.p, 0, (size_t)kQsaProfBytes) != hipSuccess) return nullptr;
  }
  static const char* only = std::getenv("MQ_PROF_LEVEL");
  if (only && *only && (only[0] == 't' ? level != -1 : std::atoi(only) != level)) {
    if (!c->prof_sink.p && c->prof_sink.ensure((size_t)kQsaProfBytes) != hipSuccess) return nullptr;
    return c->prof_sink.as<unsigned long long>();
  }
  return c->prof.as<unsigned long long>();
}

// Count the handler kinds of one translated program (k = 0: P three-word entries; 1: G words,
// inline constant words skipped) into hist[QK_COUNT] and, if given, kind bigrams into pairs.
static void qsa_count(const mq_ctx* c, int k, const std::vector<uint32_t>& tr, std::vector<int64_t>& hist,
                      std::vector<int64_t>* pairs) {
  if (hist.size() != (size_t)QK_COUNT) hist.assign(QK_COUNT, 0);
  if (pairs && pairs->size() != (size_t)QK_COUNT * QK_COUNT) pairs->assign((size_t)QK_COUNT * QK_COUNT, 0);
  int prev = -1;
  for (size_t i = 0; i < tr.size();) {
    const uint32_t key = k == 0 ? ((tr[i] - c->qsa_hbase_lo[0]) >> 2) & 0xFFFFu : tr[i] & 0xFFFFu;
    const int kind = c->qsa_kind_of[k].empty() ? -1 : c->qsa_kind_of[k][key];
    i += k == 0 ? 3 : 1;
    if (kind < 0) continue;
    hist[kind]++;
    if (pairs && prev >= 0 && kind != QK_REFILL) (*pairs)[(size_t)prev * QK_COUNT + kind]++;
    if (kind != QK_REFILL) prev = kind;
    if (k == 1) i += c->qsa_data_words[key];
  }
}

// The program the assembly interpreter k runs: G's stack has kQsaStackG slots, so a deeper
// program runs its spilled variant (tape_compiler.cpp CompiledTape::prog_g).
static inline const std::vector<uint32_t>& qsa_prog(const CompiledTape& x, int k) {
  return (k == 1 && !x.prog_g.empty()) ? x.prog_g : x.prog;
}
static inline int qsa_temps(const CompiledTape& x, int k) { return (k == 1 && !x.prog_g.empty()) ? x.n_temps_g : x.n_temps; }
static inline int qsa_depth(const CompiledTape& x, int k) { return (k == 1 && !x.prog_g.empty()) ? x.depth_g : x.depth; }

// Translate a compiled stack program into QSA threaded code for kernel k (0 = P, 1 = G).
// models == false: structural check only (upload time: variable rows and function tables are
// not known yet, any variable / lookup is assumed expressible).  extra: the tape's derived
// constants (divisor reciprocals), appended after its own constants in the same order every
// time.  Returns false if any instruction is outside the interpreter's set (those tapes run on
// the HIP C++ kernel).
static bool qsa_translate(const mq_ctx* c, int k, bool models, const CompiledTape& x, std::vector<uint32_t>* out_p,
                          std::vector<uint32_t>* extra_p, const std::vector<int>* gpre = nullptr,
                          const std::vector<int>* gstage = nullptr) {
  std::vector<uint32_t> dummy_out, dummy_extra;
  std::vector<uint32_t>& out = out_p ? *out_p : dummy_out;
  std::vector<uint32_t>& extra = extra_p ? *extra_p : dummy_extra;
  out.clear();
  extra.clear();
  const bool P = k == 0;
  if (x.L != 8 || qsa_depth(x, k) > (P ? kQsaStackP : kQsaStackG) || qsa_temps(x, k) > kQsaMaxTemps) return false;
  const std::vector<uint32_t>& xprog = qsa_prog(x, k);
  const size_t wpi = P ? 3 : 1;   // program words per interpreter instruction
  // every handler word emitted so far (position, key, immediate, inline data words): the
  // fusions below rewrite the last ones while nothing follows them
  struct Emit {
    size_t pos;
    int kind, d, v;
    uint32_t imm;
    size_t nd;
  };
  std::vector<Emit> log;
  auto ends_at = [&](const Emit& e) { return e.pos + wpi + e.nd; };
  auto drop_last = [&](size_t n) {   // forget the last n words (and their data)
    out.resize(log[log.size() - n].pos);
    log.resize(log.size() - n);
  };
  auto word = [&](int kind, int d, int v, uint32_t imm, bool imm32 = false) -> bool {
    if (d < 0 || d >= kQsaStack || v < -1 || v >= kQsaSel || (imm > 0xFFFFu && !(imm32 && P))) return false;
    const int h = c->qsa_index[k][kind][d][v + 1];
    if (h < 0) return false;
    log.push_back(Emit{out.size(), kind, d, v, imm, 0});
    if (P) {   // entry: absolute handler address (low half), immediate, constant prefetch
      out.push_back(c->qsa_hbase_lo[0] + c->qsa_off[0][h]);
      out.push_back(imm);
      out.push_back(0);
    } else {
      out.push_back(hword(k, c->qsa_off[k][h]) | (imm << 16));
    }
    return true;
  };
  // slot d holds a value of width W < 256: clear the bits above W
  auto mask = [&](int d, uint32_t W) -> bool {
    if (W >= 256) return true;
    const int n = (int)(W + 31) / 32;
    if (W % 32) return word(QK_MASKP, d, n - 1, W % 32);
    return word(QK_MASKZ, d, n - 1, 0);
  };
  auto lshr = [&](int d, uint32_t kbits, bool arith) -> bool {
    if (kbits == 0) return true;
    return word(arith ? QK_ASHRI : QK_LSHRI, d, (int)(kbits >> 5), kbits & 31);
  };
  auto shl = [&](int d, uint32_t kbits) -> bool {
    if (kbits == 0) return true;
    if (kbits & 31) return word(QK_SHLI, d, (int)(kbits >> 5), 32 - (kbits & 31));
    return word(QK_SHLW, d, (int)(kbits >> 5), 0);
  };
  // the constant pushed by the previous instruction (the right operand of a shift / division)
  auto const_value = [&](uint32_t off, uint32_t (&v)[8]) -> bool {
    if ((size_t)off + 8 > x.consts.size()) return false;
    for (int l = 0; l < 8; l++) v[l] = x.consts[off + l];
    return true;
  };
  // re-emit a word under another kind (same slot, selector, immediate and inline data)
  auto rekind = [&](int kind) -> bool {
    const Emit e = log.back();
    if (c->qsa_index[k][kind][e.d][e.v + 1] < 0) return false;
    std::vector<uint32_t> data(out.begin() + (long)(e.pos + wpi), out.begin() + (long)ends_at(e));
    drop_last(1);
    if (!word(kind, e.d, e.v, e.imm)) return false;
    out.insert(out.end(), data.begin(), data.end());
    log.back().nd = data.size();
    return true;
  };
  // slot where the last word left a Bool result, or -1 (it is not a fusable Bool producer, or
  // something was emitted after it)
  auto last_bool_slot = [&]() -> int {
    if (log.empty() || out.size() != ends_at(log.back()) || kQsaKindBoolRes[log.back().kind] < 0) return -1;
    return kQsaKindBoolRes[log.back().kind] == 0 ? log.back().d : log.back().d - 1;
  };
  // AND / OR at slot d whose right operand the last word just produced: that word's fused form
  auto fuse_acc = [&](int d, bool is_and) -> bool {
    if (last_bool_slot() != d) return false;
    const int fk = is_and ? kQsaKindAndForm[log.back().kind] : kQsaKindOrForm[log.back().kind];
    return fk >= 0 && rekind(fk);
  };
  // NOT of a compare the last word just made: the complementary compare
  auto fuse_not = [&](int d) -> bool {
    if (last_bool_slot() != d || kQsaKindNot[log.back().kind] < 0) return false;
    return rekind(kQsaKindNot[log.back().kind]);
  };
  // G: a constant push as the operand of a compare -> the compare-with-inline-constant handler.
  // (cls, data words) of the constant pushed by e (PUSH_CONSTI / PUSH_CONSTW), or cls -1
  auto const_of = [&](const Emit& e, std::vector<uint32_t>& words) -> int {
    words.clear();
    if (e.kind == QK_PUSH_CONSTI) return 0;
    if (e.kind != QK_PUSH_CONSTW) return -1;
    const size_t n = e.nd;
    words.assign(out.begin() + (long)(e.pos + 1), out.begin() + (long)(e.pos + 1 + n));
    const int cls = n <= (size_t)kQsaKClassWords[1] ? 1 : 2;
    words.resize((size_t)kQsaKClassWords[cls], 0);
    return cls;
  };
  auto emit_k = [&](int kind, int x, int sel, uint32_t imm, const std::vector<uint32_t>& words) -> bool {
    if (!word(kind, x, sel, imm)) return false;
    out.insert(out.end(), words.begin(), words.end());
    log.back().nd = words.size();
    return true;
  };
  // compare `kind` at slot d (operands S(d-1), S(d)); kk = its constant form, mk = the constant
  // form of the mirrored compare (c OP x == x MIRROR(OP) c)
  auto fuse_const = [&](int d, int kk, int mk) -> bool {
    if (P || log.empty() || d < 1) return false;
    std::vector<uint32_t> words;
    const Emit e1 = log.back();
    if (out.size() != ends_at(e1)) return false;
    // constant on the right: S(d-1) OP c
    if (e1.d == d) {
      const int cls = const_of(e1, words);
      if (cls >= 0 && c->qsa_index[k][kk][d - 1][cls + 1] >= 0) {
        const uint32_t imm = e1.imm;
        drop_last(1);
        return emit_k(kk, d - 1, cls, cls == 0 ? imm : 0, words);
      }
    }
    // constant on the left, value pushed right after it: the value moves down one slot
    if (log.size() >= 2 && e1.d == d && e1.nd == 0 &&
        (e1.kind == QK_PUSH_MEM || e1.kind == QK_PUSH_MEMS || e1.kind == QK_PUSH_TMP || e1.kind == QK_PUSH_VAR)) {
      const Emit e0 = log[log.size() - 2];
      const int cls = e0.d == d - 1 && ends_at(e0) == e1.pos ? const_of(e0, words) : -1;
      if (cls >= 0 && c->qsa_index[k][mk][d - 1][cls + 1] >= 0 && c->qsa_index[k][e1.kind][d - 1][e1.v + 1] >= 0) {
        const uint32_t imm = e0.imm;
        drop_last(2);
        return word(e1.kind, d - 1, e1.v, e1.imm) && emit_k(mk, d - 1, cls, cls == 0 ? imm : 0, words);
      }
    }
    return false;
  };
  // G: consecutive "B(d - 1) &= packed mask" words (PUSH_PKB_A at slot d) as one PKBN_A word
  // with up to four masks: their scalar loads share one wait
  // ... and a PUSH_PKB at slot d - 1 followed by such words as one PKBP word at d - 1 (their AND
  // pushed); up to six masks a word
  auto merge_pkb = [&](int d) {
    if (log.size() < 2) return;
    const Emit e1 = log.back();
    if (e1.kind != QK_PUSH_PKB_A || e1.d != d || out.size() != ends_at(e1)) return;
    const Emit e0 = log[log.size() - 2];
    if (ends_at(e0) != e1.pos) return;
    int n0, kind, x;   // masks after the first one in e0; merged kind and slot
    if (e0.d == d && e0.kind == QK_PUSH_PKB_A) n0 = 0, kind = QK_PKBN_A, x = d;
    else if (e0.d == d && e0.kind == QK_PKBN_A) n0 = e0.v, kind = QK_PKBN_A, x = d;
    else if (e0.d == d - 1 && e0.kind == QK_PUSH_PKB) n0 = 0, kind = QK_PKBP, x = d - 1;
    else if (e0.d == d - 1 && e0.kind == QK_PKBP) n0 = e0.v, kind = QK_PKBP, x = d - 1;
    else return;
    if (n0 + 1 > 5 || c->qsa_index[k][kind][x][n0 + 2] < 0) return;
    std::vector<uint32_t> data(out.begin() + (long)(e0.pos + 1), out.begin() + (long)ends_at(e0));
    data.push_back(e1.imm);
    const uint32_t imm0 = e0.imm;
    drop_last(2);
    emit_k(kind, x, n0 + 1, imm0, data);
  };
  // G: "PUSH_MEM / PUSH_MEMS x (n limbs); EQK_A x" (a model variable compared with an inline
  // constant, AND-ed into the conjunction) as one M/SEQK{2,8}_A word: row / slot in the
  // immediate, the constant in 2 or 8 inline data words (a 16-bit immediate constant travels
  // as two)
  // (and "PUSH_MEMS x; ULTK_A / UGTK_A x" as one S{ULT,UGT}K{2,8}_A word, same layout)
  auto merge_memk = [&]() {
    if (log.size() < 2) return;
    const Emit e1 = log.back();
    if ((e1.kind != QK_EQK_A && e1.kind != QK_ULTK_A && e1.kind != QK_UGTK_A) || out.size() != ends_at(e1)) return;
    const Emit e0 = log[log.size() - 2];
    if (ends_at(e0) != e1.pos || e0.d != e1.d || e0.nd != 0 || e0.v < 0) return;
    const bool wide = e1.v == 2;
    int fk;
    if (e1.kind == QK_ULTK_A) {
      if (e0.kind != QK_PUSH_MEMS) return;
      fk = wide ? QK_SULTK8_A : QK_SULTK2_A;
    } else if (e1.kind == QK_UGTK_A) {
      if (e0.kind != QK_PUSH_MEMS) return;
      fk = wide ? QK_SUGTK8_A : QK_SUGTK2_A;
    } else if (e0.kind == QK_PUSH_MEM) fk = wide ? QK_MEQK8_A : QK_MEQK2_A;
    else if (e0.kind == QK_PUSH_MEMS) fk = wide ? QK_SEQK8_A : QK_SEQK2_A;
    else return;
    if (c->qsa_index[k][fk][e1.d][e0.v + 1] < 0) return;
    std::vector<uint32_t> data;
    if (e1.v == 0) data = {e1.imm, 0u};
    else data.assign(out.begin() + (long)(e1.pos + 1), out.begin() + (long)ends_at(e1));
    const int x = e1.d, nsel = e0.v;
    const uint32_t imm0 = e0.imm;
    drop_last(2);
    emit_k(fk, x, nsel, imm0, data);
  };
  // G: "PUSH_MEMS x (n limbs); SLTK / SGTK x" as one S{SLT,SGT}K{2,8} word (layout as merge_memk's)
  auto merge_mems_k = [&]() {
    if (P || log.size() < 2) return;
    const Emit e1 = log.back();
    if ((e1.kind != QK_SLTK && e1.kind != QK_SGTK) || out.size() != ends_at(e1)) return;
    const Emit e0 = log[log.size() - 2];
    if (e0.kind != QK_PUSH_MEMS || ends_at(e0) != e1.pos || e0.d != e1.d || e0.nd != 0 || e0.v < 0) return;
    const bool wide = e1.v == 2;
    const int fk = e1.kind == QK_SLTK ? (wide ? QK_SSLTK8 : QK_SSLTK2) : (wide ? QK_SSGTK8 : QK_SSGTK2);
    if (c->qsa_index[k][fk][e1.d][e0.v + 1] < 0) return;
    std::vector<uint32_t> data;
    if (e1.v == 0) data = {e1.imm, 0u};
    else data.assign(out.begin() + (long)(e1.pos + 1), out.begin() + (long)ends_at(e1));
    const int x = e1.d, nsel = e0.v;
    const uint32_t imm0 = e0.imm;
    drop_last(2);
    emit_k(fk, x, nsel, imm0, data);
  };
  uint32_t prev_op = G_END, prev_d = 0, prev_imm = 0;
  size_t prev_out = 0;
  int prev_pre = -1;   // preload slot of the variable the previous instruction pushed
  // preload slot of variable v in this kernel, or -1 (P: v itself; G: the batch's choice)
  auto pre_slot = [&](uint32_t v) -> int {
    if (P) return v < (uint32_t)kQsaVars ? (int)v : -1;
    if (!models || !gpre || v >= gpre->size()) return -1;
    return (*gpre)[v];
  };
  // a binary op at slot d whose right operand was just pushed from a preloaded variable runs
  // as the fused handler kindv(d, slot) (the push word is dropped)
  // (P) likewise a right operand just pushed from the constants, for the kinds with a kindc
  // handler (operand read from SGPRs)
  auto binop = [&](int d, int kind, int kindv, int kindc = -1, int kindk = -1, int kindkm = -1) -> bool {
    // G: EQ of a constant (left) and a preloaded variable (right) -> EQVK, no stack traffic
    if (!P && kind == QK_EQ && prev_op == G_PUSH_VAR && prev_pre >= 0 && (int)prev_d == d && log.size() >= 2 &&
        out.size() == prev_out + wpi && log.back().pos == prev_out) {
      const Emit e0 = log[log.size() - 2];
      std::vector<uint32_t> words;
      int cls = e0.d == d - 1 && ends_at(e0) == prev_out ? const_of(e0, words) : -1;
      if (cls == 0) {   // the 16-bit immediate travels as a two-word constant here
        words.assign((size_t)kQsaKClassWords[1], 0);
        words[0] = e0.imm;
        cls = 1;
      }
      const int sel = 2 * prev_pre + (cls - 1);
      if (cls >= 1 && sel < kQsaSel && c->qsa_index[k][QK_EQVK][d - 1][sel + 1] >= 0) {
        drop_last(2);
        return emit_k(QK_EQVK, d - 1, sel, 0, words);
      }
    }
    if (kindk >= 0 && fuse_const(d, kindk, kindkm)) return true;
    if (prev_op == G_PUSH_VAR && prev_pre >= 0 && (int)prev_d == d && out.size() == prev_out + wpi &&
        c->qsa_index[k][kindv][d][prev_pre + 1] >= 0) {
      drop_last(1);
      // (P) the left operand is a leaf pushed right before at slot d - 1: both leaves in one
      // handler at d - 1 (gen_qsa.py kindVV / MULVV / kindCV, the right variable through M0)
      int kvv = -1, kcv = -1;
      bool vv_by_v1 = true;
      switch (kindv) {
        case QK_ADDV: kvv = QK_ADDVV; kcv = QK_ADDCV; break;
        case QK_SUBV: kvv = QK_SUBVV; kcv = QK_SUBCV; break;
        case QK_BANDV: kvv = QK_BANDVV; kcv = QK_BANDCV; break;
        case QK_BORV: kvv = QK_BORVV; kcv = QK_BORCV; break;
        case QK_BXORV: kvv = QK_BXORVV; kcv = QK_BXORCV; break;
        case QK_MULV: kvv = QK_MULVV; kcv = QK_MULCV; vv_by_v1 = false; break;
        default: break;
      }
      if (P && kvv >= 0 && d >= 1 && !log.empty() && out.size() == ends_at(log.back()) && log.back().d == d - 1) {
        const Emit e0 = log.back();
        const uint32_t v2 = 8u * (uint32_t)prev_pre;
        if (e0.kind == QK_PUSH_VAR && e0.v >= 0 && c->qsa_index[k][kvv][d - 1][vv_by_v1 ? e0.v + 1 : 0] >= 0) {
          drop_last(1);
          return vv_by_v1 ? word(kvv, d - 1, e0.v, v2) : word(kvv, d - 1, -1, 8u * (uint32_t)e0.v | v2 << 16, true);
        }
        if (e0.kind == QK_PUSH_CONST && c->qsa_index[k][kcv][d - 1][0] >= 0) {
          drop_last(1);
          return word(kcv, d - 1, -1, e0.imm | v2 << 16, true);
        }
      }
      return word(kindv, d, prev_pre, 0);
    }
    if (kindc >= 0 && P && prev_op == G_PUSH_CONST && (int)prev_d == d && out.size() == prev_out + wpi &&
        c->qsa_index[k][kindc][d][0] >= 0) {
      drop_last(1);
      return word(kindc, d, -1, prev_imm);
    }
    return word(kind, d, -1, 0);
  };
  for (size_t pc = 0; pc < xprog.size(); pc++) {
    const uint32_t w = xprog[pc];
    const uint32_t op = w & 0xFFu, imm = w >> 12;
    const int d = (int)((w >> 8) & 0xFu);
    uint32_t imm2 = 0;
    if (has_imm2(op)) {
      if (++pc >= xprog.size()) return false;
      imm2 = xprog[pc];
    }
    const size_t out_before = out.size();
    const bool after_const = prev_op == G_PUSH_CONST && (int)prev_d == d;
    int pushed_pre = -1;
    bool ok;
    switch (op) {
      case G_END: ok = word(QK_END, 0, -1, 0); break;
      case G_PUSH_VAR:
      case G_PUSH_VAR_B: {
        const bool b = op == G_PUSH_VAR_B;
        const int ps = pre_slot(imm);
        if (P) {
          // preloaded variables only (var < 8, at most 256 bits)
          ok = ps >= 0 && (!models || (imm < c->var_nl_h.size() && c->var_nl_h[imm] <= 8)) &&
               word(b ? QK_PUSH_VARB : QK_PUSH_VAR, d, ps, 0);
          pushed_pre = ps;
        } else if (ps >= 0) {
          ok = word(b ? QK_PUSH_VARB : QK_PUSH_VAR, d, ps, 0);
          pushed_pre = ps;
        } else if (!models) {
          ok = word(b ? QK_PUSH_MEMB : QK_PUSH_MEM, d, b ? -1 : 7, 0);
        } else if (b && imm < c->bmask_of_var.size() && c->bmask_of_var[imm] >= 0) {
          // the tile's lane mask, one scalar load (qs_pack_bool)
          ok = word(QK_PUSH_PKB, d, -1, (uint32_t)c->bmask_of_var[imm]);
        } else if (gstage && imm < gstage->size() && (*gstage)[imm] >= 0 && c->var_nl_h[imm] <= 8) {
          // a row staged in LDS by the workgroup (gen_qsa.py stage_rows)
          ok = word(b ? QK_PUSH_MEMSB : QK_PUSH_MEMS, d, b ? -1 : (int)c->var_nl_h[imm] - 1, (uint32_t)(*gstage)[imm]);
        } else {
          ok = imm < c->var_off_h.size() && c->var_nl_h[imm] <= 8 && c->var_off_h[imm] <= 0xFFFFu &&
               word(b ? QK_PUSH_MEMB : QK_PUSH_MEM, d, b ? -1 : (int)c->var_nl_h[imm] - 1, c->var_off_h[imm]);
        }
        break;
      }
      case G_PUSH_CONST: {
        if (P) {
          ok = word(QK_PUSH_CONST, d, -1, imm);
          break;
        }
        // G: the constant travels inline in the program stream (no scalar load)
        uint32_t cv[8];
        ok = const_value(imm, cv);
        if (!ok) break;
        int n = 8;
        while (n > 1 && cv[n - 1] == 0) n--;
        if (n == 1 && cv[0] <= 0xFFFFu) {
          ok = word(QK_PUSH_CONSTI, d, -1, cv[0]);
        } else {
          ok = word(QK_PUSH_CONSTW, d, n - 1, 0);
          for (int l = 0; ok && l < n; l++) out.push_back(cv[l]);
          if (ok) log.back().nd = (size_t)n;
        }
        break;
      }
      case G_PUSH_TMP: ok = word(QK_PUSH_TMP, d, -1, imm); break;
      case G_PUSH_TMP_B: ok = word(QK_PUSH_TMP_BOOL, d, -1, imm); break;
      case G_STORE_TMP: ok = d == 0 && word(QK_STORE_TMP, 0, -1, imm); break;
      case G_STORE_TMP_B: ok = d == 0 && word(QK_STORE_TMP_BOOL, 0, -1, imm); break;
      case G_PUSH_BOOL: ok = word(QK_PUSH_BOOL, d, -1, imm); break;
      case G_NOT: ok = fuse_not(d) || word(QK_NOT, d, -1, 0); break;
      case G_AND:
        ok = fuse_acc(d, true) || word(QK_AND, d, -1, 0);
        if (ok && !P) merge_pkb(d);
        if (ok && !P) merge_memk();
        break;
      case G_OR: ok = fuse_acc(d, false) || word(QK_OR, d, -1, 0); break;
      case G_XOR: ok = word(QK_XOR, d, -1, 0); break;
      case G_IFF: ok = word(QK_IFF, d, -1, 0); break;
      case G_IMPLIES: ok = word(QK_IMPLIES, d, -1, 0); break;
      case G_BITE: ok = word(QK_BITE, d, -1, 0); break;
      case G_BITE_EF: ok = word(QK_BITE_EF, d, -1, 0); break;
      // unsigned predicates / bitwise / ite are exact on canonical values of any width <= 256
      case G_EQ: ok = imm >= 1 && binop(d, QK_EQ, QK_EQV, QK_EQC, QK_EQK, QK_EQK); break;
      case G_ULT: ok = imm >= 1 && binop(d, QK_ULT, QK_ULTV, QK_ULTC, QK_ULTK, QK_UGTK); break;
      case G_ULE: ok = imm >= 1 && binop(d, QK_ULE, QK_ULEV, QK_ULEC, QK_ULEK, QK_UGEK); break;
      case G_UGT: ok = imm >= 1 && binop(d, QK_UGT, QK_UGTV, QK_UGTC, QK_UGTK, QK_ULTK); break;
      case G_UGE: ok = imm >= 1 && binop(d, QK_UGE, QK_UGEV, QK_UGEC, QK_UGEK, QK_ULEK); break;
      case G_BAND: ok = binop(d, QK_BAND, QK_BANDV, QK_BANDC); break;
      case G_BOR: ok = binop(d, QK_BOR, QK_BORV, QK_BORC); break;
      case G_BXOR: ok = binop(d, QK_BXOR, QK_BXORV, QK_BXORC); break;
      case G_ITE: {
        // G: ite(c, x, 0) with the zero pushed last -> ITEZ at the then-slot (the push dropped)
        const Emit* e = log.empty() ? nullptr : &log.back();
        if (!P && d >= 2 && e && e->kind == QK_PUSH_CONSTI && e->imm == 0 && e->d == d && out.size() == ends_at(*e) &&
            c->qsa_index[k][QK_ITEZ][d - 1][0] >= 0) {
          drop_last(1);
          // "SS{LT,GT}K x; PUSH_MEM x + 1": the load goes first, so it is in flight while the
          // compare reads LDS (the compare touches slot x, T and B(x) only)
          if (log.size() >= 2) {
            const Emit ep = log.back(), ec = log[log.size() - 2];
            const bool cmp = ec.kind == QK_SSLTK2 || ec.kind == QK_SSGTK2 || ec.kind == QK_SSLTK8 || ec.kind == QK_SSGTK8;
            if (cmp && ep.kind == QK_PUSH_MEM && ep.nd == 0 && ep.d == d - 1 && ec.d == d - 2 &&
                ends_at(ec) == ep.pos && out.size() == ends_at(ep)) {
              std::vector<uint32_t> data(out.begin() + (long)(ec.pos + 1), out.begin() + (long)ends_at(ec));
              drop_last(2);
              ok = word(ep.kind, ep.d, ep.v, ep.imm) && emit_k(ec.kind, ec.d, ec.v, ec.imm, data);
              if (!ok) break;
            }
          }
          // a staged then-value pushed right before: ITEZS reads the row itself
          const Emit ev = log.empty() ? Emit{} : log.back();
          if (!log.empty() && ev.kind == QK_PUSH_MEMS && ev.nd == 0 && ev.d == d - 1 && ev.v >= 0 && out.size() == ends_at(ev) &&
              c->qsa_index[k][QK_ITEZS][d - 1][ev.v + 1] >= 0) {
            const int nsel = ev.v;
            const uint32_t row = ev.imm;
            drop_last(1);
            ok = word(QK_ITEZS, d - 1, nsel, row);
            break;
          }
          ok = word(QK_ITEZ, d - 1, -1, 0);
        } else ok = word(QK_ITE, d, -1, 0);
        break;
      }
      case G_ITE_EF: ok = word(QK_ITE_EF, d, -1, 0); break;
      // signed predicates: at 256 bits the handler flips bit 255; below, flip bit W-1 of both
      // operands (FLIP2) and compare unsigned
      case G_SLT: case G_SLE: case G_SGT: case G_SGE: {
        const int su = op == G_SLT ? QK_SLT : op == G_SLE ? QK_SLE : op == G_SGT ? QK_SGT : QK_SGE;
        const int uu = op == G_SLT ? QK_ULT : op == G_SLE ? QK_ULE : op == G_SGT ? QK_UGT : QK_UGE;
        if (imm == 256 && (op == G_SLT || op == G_SGT) &&
            fuse_const(d, op == G_SLT ? QK_SLTK : QK_SGTK, op == G_SLT ? QK_SGTK : QK_SLTK)) {
          // G: a compare with a constant operand; a staged variable pushed right before it is
          // read by the compare itself (S{SLT,SGT}K{2,8})
          merge_mems_k();
          ok = true;
        } else if (imm == 256) ok = word(su, d, -1, 0);
        else ok = imm >= 1 && imm < 256 && word(QK_FLIP2, d, (int)((imm - 1) >> 5), (imm - 1) & 31) && word(uu, d, -1, 0);
        break;
      }
      // wrapping arithmetic: 256-bit handlers, results below 256 bits re-masked
      case G_ADD: ok = imm <= 256 && binop(d, QK_ADD, QK_ADDV, QK_ADDC) && mask(d - 1, imm); break;
      case G_SUB: ok = imm <= 256 && binop(d, QK_SUB, QK_SUBV, QK_SUBC) && mask(d - 1, imm); break;
      case G_MUL: ok = imm <= 256 && binop(d, QK_MUL, QK_MULV, QK_MULC) && mask(d - 1, imm); break;
      case G_NEG: ok = imm <= 256 && word(QK_NEG, d, -1, 0) && mask(d, imm); break;
      case G_BNOT: ok = imm <= 256 && word(QK_BNOT, d, -1, 0) && mask(d, imm); break;
      // shifts by a constant amount (the previous instruction pushed it): in place on slot d-1
      case G_SHL: case G_LSHR: case G_ASHR: {
        uint32_t cv[8];
        if (!after_const) {   // by a variable amount: G's SHLV / LSHRV / ASHRV (ASHR at 256 bits);
          // the immediate is the width W: the handler replaces results of amounts >= W by the fill
          ok = d >= 1 && imm >= 1 && imm <= 256 && (op != G_ASHR || imm == 256) &&
               word(op == G_SHL ? QK_SHLV : op == G_LSHR ? QK_LSHRV : QK_ASHRV, d - 1, -1, imm) &&
               (op != G_SHL || mask(d - 1, imm));
          break;
        }
        ok = after_const && d >= 1 && imm >= 1 && imm <= 256 && const_value(prev_imm, cv);
        if (!ok) break;
        if (log.empty() || log.back().pos != prev_out) return false;
        drop_last(1);  // drop the amount push
        bool big = false;
        for (int l = 1; l < 8; l++) big = big || cv[l] != 0;
        const uint32_t kb = big || cv[0] >= imm ? imm : cv[0];  // >= width: everything shifted out
        if (op == G_ASHR) {
          ok = imm == 256 && lshr(d - 1, std::min<uint32_t>(kb, 255), true);
        } else if (kb >= imm) {
          ok = word(QK_MASKP, d - 1, 0, 0);  // zero
        } else if (op == G_LSHR) {
          ok = lshr(d - 1, kb, false);
        } else {
          ok = shl(d - 1, kb) && mask(d - 1, imm);
        }
        break;
      }
      // division by a constant divisor (the previous instruction pushed it), in place on d-1
      case G_UDIV: case G_UREM: case G_SDIV: case G_SREM: case G_SMOD: {
        uint32_t cv[8];
        if (!after_const) {
          // by a variable divisor: G's UDIVV / UREMV (both slots; the quotient of x / 0 is all
          // ones, masked back to the width) and, at 256 bits, SDIVV / SREMV / SMODV
          int kind = op == G_UDIV ? QK_UDIVV : op == G_UREM ? QK_UREMV : op == G_SDIV ? QK_SDIVV
                   : op == G_SREM ? QK_SREMV : QK_SMODV;
          const bool sgn = op == G_SDIV || op == G_SREM || op == G_SMOD;
          ok = d >= 1 && imm >= 1 && imm <= 256 && (!sgn || imm == 256) && word(kind, d - 1, -1, 0) &&
               (op != G_UDIV || mask(d - 1, imm));
          break;
        }
        if (op == G_UDIV || op == G_UREM) {
          // unsigned by a constant that is not a non-zero 32-bit value: UDIVV / UREMV on it
          bool small = const_value(prev_imm, cv) && cv[0] != 0;
          for (int l = 1; small && l < 8; l++) small = cv[l] == 0;
          if (!small) {
            ok = d >= 1 && imm >= 1 && imm <= 256 && word(op == G_UDIV ? QK_UDIVV : QK_UREMV, d - 1, -1, 0) &&
                 (op == G_UREM || mask(d - 1, imm));
            break;
          }
        }
        ok = after_const && d >= 1 && imm >= 1 && imm <= 256 && const_value(prev_imm, cv);
        if (!ok) break;
        const bool sgn = op == G_SDIV || op == G_SREM || op == G_SMOD;
        bool neg = false;
        if (sgn) {
          if (imm != 256) { ok = false; break; }
          neg = (cv[7] >> 31) != 0;
          if (neg) {  // |c| = -c
            uint64_t br = 1;
            for (int l = 0; l < 8; l++) {
              const uint64_t t = (uint64_t)(uint32_t)~cv[l] + br;
              cv[l] = (uint32_t)t;
              br = t >> 32;
            }
          }
        }
        bool hi = false;
        for (int l = 1; l < 8; l++) hi = hi || cv[l] != 0;
        if (sgn && (hi || cv[0] == 0)) {
          // a signed divisor of 0 or of magnitude >= 2^32: SDIVV / SREMV / SMODV on the pushed
          // constant, as the unsigned case routes such divisors to UDIVV / UREMV (G only)
          ok = word(op == G_SDIV ? QK_SDIVV : op == G_SREM ? QK_SREMV : QK_SMODV, d - 1, -1, 0);
          break;
        }
        if (log.empty() || log.back().pos != prev_out) return false;
        drop_last(1);  // drop the divisor push
        if (!sgn && !hi && cv[0] != 0 && (cv[0] & (cv[0] - 1)) == 0) {
          // unsigned power of two: shift / mask
          const uint32_t kb = (uint32_t)__builtin_ctz(cv[0]);
          ok = op == G_UDIV ? lshr(d - 1, kb, false)
                            : (kb == 0 ? word(QK_MASKP, d - 1, 0, 0) : mask(d - 1, kb));
          break;
        }
        if (hi || cv[0] == 0) { ok = false; break; }
        const uint32_t cabs = cv[0];
        const uint32_t sh = (uint32_t)__builtin_clz(cabs);
        const uint32_t dn = cabs << sh;
        const uint64_t inv = ~0ull / dn - (1ull << 32);
        const uint32_t off = (uint32_t)(x.consts.size() + extra.size());
        extra.push_back(dn);
        extra.push_back((uint32_t)inv);
        extra.push_back(sh);
        extra.push_back(cabs);
        int kind;
        switch (op) {
          case G_UDIV: kind = QK_UDIVC; break;
          case G_UREM: kind = QK_UREMC; break;
          case G_SREM: kind = QK_SREMC; break;
          case G_SMOD: kind = neg ? QK_SMODCN : QK_SMODCP; break;
          default: kind = neg ? QK_SDIVCN : QK_SDIVCP; break;
        }
        ok = word(kind, d - 1, -1, off);
        break;
      }
      case G_EXTRACT:  // imm = lo, imm2 = result width
        ok = imm < 256 && imm2 >= 1 && imm2 <= 256 && lshr(d, imm, false) && mask(d, imm2);
        break;
      case G_CONCAT:  // imm = width of the low operand (slot d), imm2 = result width
        ok = imm >= 1 && imm < 256 && imm2 <= 256;
        if (ok && !P && (imm & 31) && c->qsa_index[k][QK_SHLOR][d][(imm >> 5) + 1] >= 0)
          ok = word(QK_SHLOR, d, (int)(imm >> 5), 32 - (imm & 31));   // G: shift and OR in one
        else ok = ok && shl(d - 1, imm) && word(QK_BOR, d, -1, 0);
        break;
      case G_SEXT: {  // imm = source width, imm2 = result width
        ok = imm >= 1 && imm <= 256 && imm2 <= 256;
        if (!ok) break;
        const int p = (int)((imm - 1) >> 5);
        const uint32_t nb = ((imm - 1) & 31) + 1;
        if (nb < 32) ok = word(QK_SEXTB, d, p, nb);
        else if (p < 7) ok = word(QK_SEXTA, d, p, 0);
        ok = ok && mask(d, imm2);
        break;
      }
      case G_UF1: {  // imm = function id, imm2 = result width (0 = Bool)
        // (G scans the entries with 32-bit byte offsets)
        ok = !P && imm2 <= 256 && (uint64_t)(c->entry_words_n + (int64_t)kEntryPadWords) * 4 < (1ull << 32);
        if (ok && models) {
          // a function absent from the model batch evaluates to 0 (as in the C++ kernel)
          ok = imm >= c->funcs_h.size() || (c->funcs_h[imm].arity == 1 && c->funcs_h[imm].arg_width[0] <= 256 &&
                                            c->funcs_h[imm].result_width <= 256);
        }
        if (!ok) break;
        if (imm2 == 0) ok = word(QK_UF1B, d, -1, imm);
        else ok = word(QK_UF1, d, -1, imm) && mask(d, imm2);
        break;
      }
      default: ok = false;
    }
    if (!ok) {
      // MQ_QSA_DEBUG=1: name the stack-program instruction a translation stops at (diagnostic)
      static const bool dbg = std::getenv("MQ_QSA_DEBUG") != nullptr;
      if (dbg) std::fprintf(stderr, "qsa_translate(%s): op %u at slot %d imm %u not translated\n", P ? "P" : "G", op, d, imm);
      return false;
    }
    prev_op = op;
    prev_d = (uint32_t)d;
    prev_imm = imm;
    prev_out = out_before;
    prev_pre = op == G_PUSH_VAR ? pushed_pre : -1;
  }
  static const bool no_lwait = std::getenv("MQ_NO_LWAIT") != nullptr;   // (diagnostic A/B)
  if (!P) {
    // final pass: a stack reader waits for the vector loads of a PUSH_MEM only when one may be
    // outstanding; otherwise its "_L" variant waits for LDS / scalar loads alone, and the
    // prefetch of the next program window (gen_qsa.py load_window) stays in flight
    // (MQ_NO_LWAIT: no _L variants; END_V is needed either way)
    bool pending = false;
    for (const Emit& e : log) {
      if (e.kind == QK_PUSH_MEM) {
        pending = true;
        continue;
      }
      if (e.kind == QK_END) {
        // the value a column stores may still be a load in flight: END_V waits for it (the
        // tape end's column store waits for LDS / scalar loads only)
        const int h = c->qsa_index[k][QK_END_V][0][0];
        if (pending && h >= 0) out[e.pos] = hword(k, c->qsa_off[k][h]);
        continue;
      }
      const int lk = kQsaKindLForm[e.kind];
      if (lk >= 0) {
        const int h = c->qsa_index[k][lk][e.d][e.v + 1];
        if (!pending && h >= 0 && !no_lwait) out[e.pos] = hword(k, c->qsa_off[k][h]) | (e.imm << 16);
        pending = false;   // (the VMWAIT form drained every load)
        continue;
      }
      if (c->qsa_vm_drain[e.kind]) pending = false;
    }
  }
  if (P) {
    // constant prefetch (gen_qsa.py NEXT_P): a constant handler whose predecessor is not itself
    // a prefetched one becomes its PF_ variant, and the predecessor's entry names its constant
    // (the dispatch of the predecessor loads it into CB); a PF_ handler whose successor is not
    // one re-loads its own constant (an in-flight load then writes CB's current contents)
    auto pf_kind = [](int kind) -> int {
      switch (kind) {
        case QK_PUSH_CONST: return QK_PF_PUSH_CONST;
        case QK_ADDC: return QK_PF_ADDC;
        case QK_SUBC: return QK_PF_SUBC;
        case QK_MULC: return QK_PF_MULC;
        case QK_BANDC: return QK_PF_BANDC;
        case QK_BORC: return QK_PF_BORC;
        case QK_BXORC: return QK_PF_BXORC;
        case QK_ADDCV: return QK_PF_ADDCV;
        case QK_SUBCV: return QK_PF_SUBCV;
        case QK_MULCV: return QK_PF_MULCV;
        case QK_BANDCV: return QK_PF_BANDCV;
        case QK_BORCV: return QK_PF_BORCV;
        case QK_BXORCV: return QK_PF_BXORCV;
        default: return -1;
      }
    };
    std::vector<char> pf(log.size(), 0);
    auto coff_bytes = [&](const Emit& e) -> uint32_t {
      const bool cv = e.kind == QK_ADDCV || e.kind == QK_SUBCV || e.kind == QK_MULCV || e.kind == QK_BANDCV ||
                      e.kind == QK_BORCV || e.kind == QK_BXORCV;
      return 4u * (cv ? (e.imm & 0xFFFFu) : e.imm);
    };
    for (size_t j = 1; j < log.size(); j++) {
      const Emit& e = log[j];
      const int fk = pf_kind(e.kind);
      if (fk < 0 || pf[j - 1] || c->qsa_index[0][fk][e.d][e.v + 1] < 0) continue;
      pf[j] = 1;
      out[e.pos] = c->qsa_hbase_lo[0] + c->qsa_off[0][c->qsa_index[0][fk][e.d][e.v + 1]];
      out[log[j - 1].pos + 2] = coff_bytes(e);
    }
    for (size_t j = 0; j < log.size(); j++)
      if (pf[j] && !(j + 1 < log.size() && pf[j + 1])) out[log[j].pos + 2] = coff_bytes(log[j]);
  }
  return x.consts.size() + extra.size() <= 0x10000u;
}

// Upload a compiled batch to ONE device.  may_move: the batch's last device takes the QSA-eligible
// tapes' programs out of ct instead of copying them (~3 000 tapes of a fresh drop-in batch).
static int tapes_upload_one(mq_ctx* c, int32_t n_tapes, std::vector<CompiledTape>& ct, mq_tapes** out,
                            bool may_move) {
  *out = nullptr;
  HIPCHK(hipSetDevice(c->device));
  auto T = std::make_unique<mq_tapes>();
  T->ctx = c;
  {
    std::lock_guard<std::mutex> g(g_live_mu);
    c->live_tapes.insert(T.get());
  }
  T->n_tapes = n_tapes;
  T->unsupported.assign(std::max(n_tapes, 1), 0);
  T->n_nodes.assign(n_tapes, 0);
  T->alg_ops.assign(n_tapes, 0);
  // descriptor groups: [L8 QSA-eligible | gen[0] | gen[1..]] (see mq_tapes)
  std::vector<uint32_t> prog, consts;
  std::vector<GDesc> descs;
  auto push_desc = [&](int t, const CompiledTape& x) {
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
    descs.push_back(d);
    return d;
  };
  // QSA eligibility is structural here (G kernel set, no model information); the derived
  // constants of an eligible tape (divisor reciprocals) follow its own constants in the pool
  std::vector<char> qsa_ok(n_tapes, 0);
  std::vector<std::vector<uint32_t>> qextra(n_tapes);
  std::unique_ptr<PhaseTimer> pt(new PhaseTimer(&c->host_t[1]));
  if (c->qsa_ready)
    parallel_for(n_tapes, 32, [&](int, int64_t b, int64_t e) {
      for (int64_t t = b; t < e; t++)
        if (ct[t].supported && ct[t].L == 8 && ct[t].n_temps <= kQsaMaxTemps)
          qsa_ok[t] = qsa_translate(c, 1, false, ct[t], nullptr, &qextra[t]) ? 1 : 0;
    });
  pt.reset(new PhaseTimer(&c->host_t[2]));
  // (before the descriptor passes: with may_move they empty the eligible tapes' vectors)
  T->wide_funcs.assign(n_tapes, {});
  for (int t = 0; t < n_tapes; t++) {
    T->wide_funcs[t] = ct[t].wide_funcs;
    T->wide_any = T->wide_any || !ct[t].wide_funcs.empty();
  }
  for (int t = 0; t < n_tapes; t++) {
    T->unsupported[t] = ct[t].supported ? 0 : 1;
    T->n_unsupported += ct[t].supported ? 0 : 1;
    T->n_nodes[t] = ct[t].n_nodes;
    T->alg_ops[t] = ct[t].alg_ops;
  }
  size_t prog_words = 1, const_words = 24;
  for (int t = 0; t < n_tapes; t++) {
    prog_words += ct[t].prog.size();
    const_words += ct[t].consts.size() + qextra[t].size();
  }
  prog.reserve(prog_words);
  consts.reserve(const_words);
  descs.reserve((size_t)n_tapes + 1);
  for (int pass = -1; pass < kGen; pass++) {
    mq_tapes::Variant& v = pass < 0 ? T->qsa : T->gen[pass];
    v.L = pass < 0 ? 8 : kGenL[pass];
    v.keccak = pass < 0 ? false : kGenK[pass];
    v.begin = (int)descs.size();
    for (int t = 0; t < n_tapes; t++) {
      const CompiledTape& x = ct[t];
      if (!x.supported) continue;
      if (pass < 0 ? !(x.L == 8 && qsa_ok[t]) : (gen_kind(x) != pass || (pass == 0 && qsa_ok[t]))) continue;
      GDesc d = push_desc(t, x);
      if (pass < 0) {
        consts.insert(consts.end(), qextra[t].begin(), qextra[t].end());
        T->qbase.push_back(d);
        if (may_move)
          T->qct.push_back(std::move(ct[t]));
        else
          T->qct.push_back(x);
      }
      v.max_temps = std::max(v.max_temps, x.n_temps);
      v.max_depth = std::max(v.max_depth, x.depth);
    }
    v.count = (int)descs.size() - v.begin;
  }
  T->l8_all.L = 8;
  T->l8_all.begin = 0;
  T->l8_all.count = T->qsa.count + T->gen[0].count;
  T->l8_all.max_temps = std::max(T->qsa.max_temps, T->gen[0].max_temps);
  T->l8_all.max_depth = std::max(T->qsa.max_depth, T->gen[0].max_depth);
  consts.resize(consts.size() + 16, 0);
  prog.push_back(gword(G_END, 0, 0));
  if (descs.empty()) descs.push_back(GDesc{});
  HIPCHK(T->qargs[0].ensure(sizeof(QArgs)));
  HIPCHK(T->qargs[1].ensure(sizeof(QArgs)));
  // P's constant prefetch reads 8 words at a tape's constants + 0 even for a tape without any
  consts.insert(consts.end(), 8, 0u);
  {
    UploadPack pk;   // descriptors, programs, constants, unsupported flags: one copy
    pk.add(T->descs, descs.data(), descs.size());
    pk.add(T->prog, prog.data(), prog.size());
    pk.add(T->consts, consts.data(), consts.size());
    pk.add(T->unsup_dev, T->unsupported.data(), T->unsupported.size());
    HIPCHK(pk.commit(T->pack0, c->stream, c->stage));
  }
  T->in_flight = true;
  T->unsupported_base = T->unsupported;
  *out = T.release();
  return MQ_OK;
}

// Upload compiled tapes to every device of the context (lead + peers).
static int tapes_upload_all(mq_ctx* c, int32_t n_tapes, std::vector<CompiledTape>& ct, mq_tapes** out,
                            int32_t* n_unsup_out) {
  // the peers copy the compiled programs, the lead (uploaded last) takes them
  std::vector<mq_tapes*> peers;
  for (mq_ctx* p : c->peers) {
    mq_tapes* pt = nullptr;
    const int rc = tapes_upload_one(p, n_tapes, ct, &pt, false);
    if (rc) {
      for (mq_tapes* q : peers) mq_tapes_free(q);
      return rc;
    }
    peers.push_back(pt);
  }
  mq_tapes* T = nullptr;
  int rc = tapes_upload_one(c, n_tapes, ct, &T, true);
  if (rc) {
    for (mq_tapes* q : peers) mq_tapes_free(q);
    return rc;
  }
  std::unique_ptr<mq_tapes> guard(T);
  T->peers = peers;
  if (n_unsup_out) *n_unsup_out = T->n_unsupported;
  *out = guard.release();
  return MQ_OK;
}

int mq_tapes_upload(mq_ctx* c, const mq_tape_batch* tb, mq_tapes** out, int32_t* n_unsup_out) {
  if (!c || !tb || !out || tb->n_tapes < 0 || (tb->n_tapes > 0 && (!tb->tape_offsets || !tb->nodes))) return MQ_ERR_ARG;
  *out = nullptr;
  for (int t = 0; t < tb->n_tapes; t++) {
    if (tb->tape_offsets[t + 1] < tb->tape_offsets[t]) return MQ_ERR_ARG;
  }
  // compile once (independent per tape), upload to every device of the context
  CompileLimits lim;
  lim.g_depth = kQsaStackG;
  std::vector<CompiledTape> ct(tb->n_tapes);
  {
    PhaseTimer pt(&c->host_t[0]);
    parallel_for(tb->n_tapes, 16, [&](int, int64_t b, int64_t e) {
      for (int64_t t = b; t < e; t++) ct[t] = compile_tape(tb, (int32_t)t, lim);
    });
  }
  return tapes_upload_all(c, tb->n_tapes, ct, out, n_unsup_out);
}

// ---------------------------------------------------------------- DAG batches (the query stream)
// Node fields that reference other nodes (include/mq.h operand conventions).
static int node_refs(const mq_node& n, uint32_t r[3]) {
  switch (n.op) {
    case MQ_OP_CONST: case MQ_OP_VAR: case MQ_OP_TRUE: case MQ_OP_FALSE: case MQ_OP_ARRAY_VAR:
      return 0;
    case MQ_OP_NOT: case MQ_OP_NEG: case MQ_OP_BNOT: case MQ_OP_EXTRACT: case MQ_OP_ZEXT: case MQ_OP_SEXT:
    case MQ_OP_CONST_ARRAY: case MQ_OP_KECCAK:
      r[0] = n.a;
      return 1;
    case MQ_OP_BITE: case MQ_OP_ITE: case MQ_OP_STORE:
      r[0] = n.a; r[1] = n.b; r[2] = n.c;
      return 3;
    case MQ_OP_UF:
    case MQ_OP_UF_CHUNK:
      r[0] = n.b;
      if (n.c == MQ_NONE) return 1;
      r[1] = n.c;
      return 2;
    case MQ_OP_UF_WIDE:
      r[0] = n.b;
      return 1;
    default:
      r[0] = n.a; r[1] = n.b;
      return 2;
  }
}

// Tape t of a DAG batch as a self-contained postfix block: the nodes reachable from its conjunct
// roots in ascending DAG order (the DAG is postfix, so that order is topological), references
// renumbered, then an AND chain over the roots.  CONST nodes keep indexing the shared pool.
// mark: per-thread scratch of dag->n_nodes entries, stamp unique per call.
static bool expand_dag_tape(const mq_dag_batch* dag, int32_t t, std::vector<int32_t>& mark, int32_t stamp,
                            std::vector<mq_node>& out) {
  out.clear();
  const int64_t r0 = dag->root_offsets[t], r1 = dag->root_offsets[t + 1];
  std::vector<uint32_t> reach, st;
  for (int64_t i = r0; i < r1; i++) {
    const uint32_t r = dag->roots[i];
    if ((int64_t)r >= dag->n_nodes) return false;
    if (mark[r] != stamp) {
      mark[r] = stamp;
      st.push_back(r);
    }
  }
  while (!st.empty()) {
    const uint32_t x = st.back();
    st.pop_back();
    reach.push_back(x);
    uint32_t kids[3];
    const int nk = node_refs(dag->nodes[x], kids);
    for (int k = 0; k < nk; k++) {
      const uint32_t c = kids[k];
      if (c >= x) return false;   // not postfix
      if (mark[c] != stamp) {
        mark[c] = stamp;
        st.push_back(c);
      }
    }
  }
  std::sort(reach.begin(), reach.end());
  // renumber: mark[x] = -(local index) - 2 for reached nodes (distinct from any stamp >= 1)
  for (size_t i = 0; i < reach.size(); i++) mark[reach[i]] = -(int32_t)i - 2;
  out.reserve(reach.size() + (size_t)std::max<int64_t>(r1 - r0, 1));
  for (uint32_t x : reach) {
    mq_node n = dag->nodes[x];
    uint32_t* f[3] = {&n.a, &n.b, &n.c};
    switch (n.op) {   // rewrite exactly the reference fields
      case MQ_OP_CONST: case MQ_OP_VAR: case MQ_OP_TRUE: case MQ_OP_FALSE: case MQ_OP_ARRAY_VAR:
        break;
      case MQ_OP_NOT: case MQ_OP_NEG: case MQ_OP_BNOT: case MQ_OP_EXTRACT: case MQ_OP_ZEXT: case MQ_OP_SEXT:
      case MQ_OP_CONST_ARRAY: case MQ_OP_KECCAK:
        n.a = (uint32_t)(-mark[n.a] - 2);
        break;
      case MQ_OP_BITE: case MQ_OP_ITE: case MQ_OP_STORE:
        for (int k = 0; k < 3; k++) *f[k] = (uint32_t)(-mark[*f[k]] - 2);
        break;
      case MQ_OP_UF:
      case MQ_OP_UF_CHUNK:
        n.b = (uint32_t)(-mark[n.b] - 2);
        if (n.c != MQ_NONE) n.c = (uint32_t)(-mark[n.c] - 2);
        break;
      case MQ_OP_UF_WIDE:
        n.b = (uint32_t)(-mark[n.b] - 2);
        break;
      default:
        n.a = (uint32_t)(-mark[n.a] - 2);
        n.b = (uint32_t)(-mark[n.b] - 2);
    }
    out.push_back(n);
  }
  if (r1 == r0) {   // And() of nothing: true
    out.push_back(mq_node{MQ_OP_TRUE, 0, 0, 0, 0});
  } else {
    uint32_t acc = (uint32_t)(-mark[dag->roots[r0]] - 2);
    for (int64_t i = r0 + 1; i < r1; i++) {
      out.push_back(mq_node{MQ_OP_AND, 0, acc, (uint32_t)(-mark[dag->roots[i]] - 2), 0});
      acc = (uint32_t)out.size() - 1;
    }
    // the root must be the last node: a single-conjunct tape whose root is not last gets an
    // AND with itself (idempotent)
    if (r1 - r0 == 1 && acc != (uint32_t)out.size() - 1) out.push_back(mq_node{MQ_OP_AND, 0, acc, acc, 0});
  }
  for (uint32_t x : reach) mark[x] = stamp;   // back to "seen in this call"
  return true;
}

static bool dag_ok(const mq_dag_batch* d) {
  return d && d->n_tapes >= 0 && d->n_nodes >= 0 && (d->n_tapes == 0 || (d->root_offsets && d->roots)) &&
         (d->n_nodes == 0 || d->nodes) && d->n_nodes < 0x7FFFFFFF;
}

// Compile every tape of a DAG batch (parallel over tapes).
static std::vector<CompiledTape> compile_dag(const mq_dag_batch* dag, const CompileLimits& lim) {
  std::vector<CompiledTape> ct(dag->n_tapes);
  // per-thread scratch kept across calls: the mark array spans the whole persistent DAG (up to
  // 2^20 nodes), so re-zeroing it per call cost more than compiling a query's few tapes; stamps
  // keep increasing across calls instead (the array is reset only when it grows or they wrap)
  struct Scratch {
    std::vector<int32_t> mark;
    std::vector<mq_node> block;
    int32_t stamp = 0;
  };
  static thread_local Scratch sc_tls;
  parallel_for(dag->n_tapes, 4, [&](int, int64_t b, int64_t e) {
    Scratch& sc = sc_tls;
    if ((int64_t)sc.mark.size() < dag->n_nodes || sc.stamp > (1 << 30)) {
      sc.mark.assign((size_t)std::max<int64_t>(dag->n_nodes, 1), 0);
      sc.stamp = 0;
    }
    for (int64_t t = b; t < e; t++) {
      if (!expand_dag_tape(dag, (int32_t)t, sc.mark, ++sc.stamp, sc.block)) {
        ct[t].why = "malformed DAG (operand does not precede its user)";
        continue;
      }
      const int64_t offs[2] = {0, (int64_t)sc.block.size()};
      mq_tape_batch one{1, offs, sc.block.data(), dag->const_words, dag->n_const_words};
      ct[t] = compile_tape(&one, 0, lim);
    }
  });
  return ct;
}

int mq_tapes_upload_dag(mq_ctx* c, const mq_dag_batch* dag, mq_tapes** out, int32_t* n_unsup_out) {
  if (!c || !out || !dag_ok(dag)) return MQ_ERR_ARG;
  *out = nullptr;
  for (int t = 0; t < dag->n_tapes; t++)
    if (dag->root_offsets[t + 1] < dag->root_offsets[t]) return MQ_ERR_ARG;
  CompileLimits lim;
  lim.g_depth = kQsaStackG;
  std::vector<CompiledTape> ct;
  {
    PhaseTimer pt(&c->host_t[0]);
    ct = compile_dag(dag, lim);
  }
  return tapes_upload_all(c, dag->n_tapes, ct, out, n_unsup_out);
}

int mq_dag_expand(const mq_dag_batch* dag, int32_t t, mq_node* nodes_out, int64_t cap, int64_t* n_out) {
  if (!dag_ok(dag) || t < 0 || t >= dag->n_tapes || !n_out) return MQ_ERR_ARG;
  std::vector<int32_t> mark((size_t)std::max<int64_t>(dag->n_nodes, 1), 0);
  std::vector<mq_node> block;
  if (!expand_dag_tape(dag, t, mark, 1, block)) return MQ_ERR_TAPE;
  *n_out = (int64_t)block.size();
  if (nodes_out && cap >= (int64_t)block.size()) std::memcpy(nodes_out, block.data(), block.size() * sizeof(mq_node));
  return MQ_OK;
}

void mq_tapes_free(mq_tapes* t) {
  // the batch's buffers go back to the pool: the launches on the context streams that read them
  // must be done (caller streams: DevPool::mark_foreign)
  if (!t) return;
  double* acc = t->ctx ? &t->ctx->host_t[9] : nullptr;
  double dummy = 0;
  PhaseTimer pt(acc ? acc : &dummy);
  // (a batch whose copies and launches the host has already waited for needs no sync: the
  // drop-in path frees one per query batch)
  if (t->ctx && t->ctx->stream && t->in_flight) (void)hipStreamSynchronize(t->ctx->stream);
  delete t;
}

// A column program that is exactly keccak256(concat of variables and constants) with every piece
// a whole number of 32-bit words and at most 2048 bits in all (lower.py keccak_subterms makes
// them): its pieces, most significant first, for the keccak column kernel.
static bool kc_match(const mq_tape_batch* progs, int32_t k, std::vector<mq_tapes::KcPiece>& pieces,
                     std::vector<uint32_t>& consts) {
  const int64_t base = progs->tape_offsets[k];
  const int64_t nn = progs->tape_offsets[k + 1] - base;
  if (nn < 2) return false;
  const mq_node* nd = progs->nodes + base;
  const mq_node& root = nd[nn - 1];
  if (root.op != MQ_OP_KECCAK || root.width != 256 || root.a >= (uint32_t)(nn - 1)) return false;
  pieces.clear();
  const size_t c0 = consts.size();
  uint32_t words = 0;
  std::vector<uint32_t> stack{root.a};
  while (!stack.empty()) {
    const uint32_t i = stack.back();
    stack.pop_back();
    const mq_node& n = nd[i];
    if (n.op == MQ_OP_CONCAT) {
      if (n.a >= i || n.b >= i) return false;
      stack.push_back(n.b);   // low part after the high part
      stack.push_back(n.a);
      continue;
    }
    if ((n.op != MQ_OP_VAR && n.op != MQ_OP_CONST) || n.width == 0 || n.width % 32) {
      consts.resize(c0);
      return false;
    }
    const uint32_t nl = n.width / 32;
    words += nl;
    if (n.op == MQ_OP_VAR) {
      pieces.push_back(mq_tapes::KcPiece{(int32_t)n.a, nl, 0});
    } else {
      if ((int64_t)n.a + nl > progs->n_const_words) {
        consts.resize(c0);
        return false;
      }
      pieces.push_back(mq_tapes::KcPiece{-1, nl, (uint32_t)consts.size()});
      consts.insert(consts.end(), progs->const_words + n.a, progs->const_words + n.a + nl);
    }
  }
  if (words == 0 || words > 64) {
    consts.resize(c0);
    return false;
  }
  return true;
}

// A column program comparing a variable with a constant, as lower.py keccak_predicates makes
// them (root ULT / EQ of a VAR and a CONST, possibly under NOT; or EQ(EXTRACT(k-1, 0, VAR), 0)):
// the variable and the predicate, for the keccak column kernel.
static bool kp_match(const mq_tape_batch* progs, int32_t k, int32_t* var, uint32_t* kind, uint32_t* bits,
                     uint32_t (&c)[8]) {
  const int64_t base = progs->tape_offsets[k];
  const int64_t nn = progs->tape_offsets[k + 1] - base;
  if (nn < 3 || nn > 5) return false;
  const mq_node* nd = progs->nodes + base;
  int64_t r = nn - 1;
  bool neg = false;
  if (nd[r].op == MQ_OP_NOT) {
    neg = true;
    if (nd[r].a >= (uint32_t)r) return false;
    r = nd[r].a;
  }
  const mq_node& p = nd[r];
  if ((p.op != MQ_OP_ULT && p.op != MQ_OP_EQ) || p.a >= (uint32_t)r || p.b >= (uint32_t)r) return false;
  const mq_node &x = nd[p.a], &y = nd[p.b];
  auto konst = [&](const mq_node& n) -> bool {
    if (n.op != MQ_OP_CONST || n.width == 0 || n.width > 256 || (int64_t)n.a + (n.width + 31) / 32 > progs->n_const_words)
      return false;
    for (int i = 0; i < 8; i++) c[i] = i < (int)((n.width + 31) / 32) ? progs->const_words[n.a + i] : 0u;
    if (n.width % 32) c[(n.width - 1) / 32] &= (1u << (n.width % 32)) - 1u;
    return true;
  };
  *bits = 0;
  if (p.op == MQ_OP_EQ && x.op == MQ_OP_EXTRACT && !neg && x.c == 0 && x.a < p.a && nd[x.a].op == MQ_OP_VAR &&
      nd[x.a].width == 256 && konst(y)) {   // EQ(EXTRACT(k-1, 0, h), 0): the low k bits are zero
    for (int i = 0; i < 8; i++)
      if (c[i]) return false;
    *var = (int32_t)nd[x.a].a;
    *kind = KP_LOWZ;
    *bits = x.width;
    return x.width > 0 && x.width <= 256;
  }
  bool h_left;
  if (x.op == MQ_OP_VAR && x.width == 256 && konst(y)) h_left = true;
  else if (y.op == MQ_OP_VAR && y.width == 256 && konst(x)) h_left = false;
  else return false;
  *var = (int32_t)(h_left ? x.a : y.a);
  if (p.op == MQ_OP_EQ) {
    if (neg) return false;
    *kind = KP_EQ;
  } else if (h_left) {
    *kind = neg ? KP_GE : KP_LT;   // h < c  /  not (h < c)
  } else {
    *kind = neg ? KP_LE : KP_GT;   // c < h  /  not (c < h)
  }
  return true;
}

// A column program that only arranges bits (cw.hip): VAR, CONST, CONCAT, EXTRACT, ZEXT, BAND
// with a constant operand, and ITE(SLT(CONST i, VAR size), x, 0) with 0 <= i < 2^31 and one
// 256-bit size variable per column (lower.py's calldata bytes, calldata.py:234-247), over a
// bit-vector root of at most 256 bits.  Each node's value is evaluated symbolically bit by bit
// (a source variable bit or a constant, and the gate); the root's bits are then grouped into
// runs of consecutive bits of one variable limb under one gate: the slots of its output limbs.
static bool cw_compile(const mq_tape_batch* progs, int32_t k, mq_tapes::CwHost& h) {
  const int64_t base = progs->tape_offsets[k];
  const int64_t nn = progs->tape_offsets[k + 1] - base;
  if (nn < 2 || nn > 4096) return false;
  const mq_node* nd = progs->nodes + base;
  const mq_node& root = nd[nn - 1];
  if (root.width == 0 || root.width > 256) return false;
  struct Bit {
    int32_t var;    // >= 0: a variable; -1: constant 0; -2: constant 1
    uint32_t bit;   // the variable's bit
    uint32_t gate;  // ~0u: ungated; else i of `i <s size`
  };
  std::vector<std::vector<Bit>> val(nn);
  std::vector<char> need(nn, 0);
  need[nn - 1] = 1;
  // which nodes the root reaches (a dead node of any op does not block the match)
  for (int64_t i = nn - 1; i >= 0; i--) {
    if (!need[i]) continue;
    const mq_node& n = nd[i];
    auto mark = [&](uint32_t j) -> bool {
      if (j >= (uint32_t)i) return false;
      need[j] = 1;
      return true;
    };
    switch (n.op) {
      case MQ_OP_VAR: case MQ_OP_CONST: break;
      case MQ_OP_EXTRACT: case MQ_OP_ZEXT: if (!mark(n.a)) return false; break;
      case MQ_OP_CONCAT: case MQ_OP_BAND: case MQ_OP_SLT: if (!mark(n.a) || !mark(n.b)) return false; break;
      case MQ_OP_ITE: if (!mark(n.a) || !mark(n.b) || !mark(n.c)) return false; break;
      default: return false;
    }
  }
  int32_t size_var = -1;
  const Bit zero{-1, 0, ~0u};
  auto is_const = [&](const std::vector<Bit>& v) {
    for (const Bit& b : v)
      if (b.var >= 0) return false;
    return true;
  };
  for (int64_t i = 0; i < nn; i++) {
    if (!need[i]) continue;
    const mq_node& n = nd[i];
    std::vector<Bit>& r = val[i];
    switch (n.op) {
      case MQ_OP_VAR:
        if (n.width == 0 || n.width > 256) return false;
        for (uint32_t b = 0; b < n.width; b++) r.push_back(Bit{(int32_t)n.a, b, ~0u});
        break;
      case MQ_OP_CONST: {
        if (n.width == 0 || n.width > 256 || (int64_t)n.a + (n.width + 31) / 32 > progs->n_const_words) return false;
        for (uint32_t b = 0; b < n.width; b++)
          r.push_back((progs->const_words[n.a + b / 32] >> (b % 32)) & 1u ? Bit{-2, 0, ~0u} : zero);
        break;
      }
      case MQ_OP_CONCAT:
        r = val[n.b];
        r.insert(r.end(), val[n.a].begin(), val[n.a].end());
        break;
      case MQ_OP_EXTRACT:
        if (n.c > n.b || n.b >= val[n.a].size()) return false;
        r.assign(val[n.a].begin() + n.c, val[n.a].begin() + n.b + 1);
        break;
      case MQ_OP_ZEXT:
        r = val[n.a];
        r.resize(n.width, zero);
        break;
      case MQ_OP_BAND: {
        const std::vector<Bit>&x = val[n.a], &y = val[n.b];
        if (x.size() != y.size()) return false;
        const bool cy = is_const(y), cx = is_const(x);
        if (!cx && !cy) return false;
        const std::vector<Bit>&v = cy ? x : y, &c = cy ? y : x;
        for (size_t b = 0; b < v.size(); b++) r.push_back(c[b].var == -2 ? v[b] : zero);
        break;
      }
      case MQ_OP_SLT: {   // only as an ITE condition: checked there
        const mq_node &a = nd[n.a], &s = nd[n.b];
        if (a.op != MQ_OP_CONST || a.width != 256 || s.op != MQ_OP_VAR || s.width != 256) return false;
        if ((int64_t)a.a + 8 > progs->n_const_words) return false;
        for (int l = 1; l < 8; l++)
          if (progs->const_words[a.a + l]) return false;
        if (progs->const_words[a.a] >= 0x80000000u) return false;
        if (size_var >= 0 && size_var != (int32_t)s.a) return false;
        size_var = (int32_t)s.a;
        break;
      }
      case MQ_OP_ITE: {
        const mq_node& cnd = nd[n.a];
        if (cnd.op != MQ_OP_SLT) return false;
        const uint32_t gate = progs->const_words[nd[cnd.a].a];
        const std::vector<Bit>&t = val[n.b], &e = val[n.c];
        if (t.size() != e.size()) return false;
        for (const Bit& b : e)
          if (b.var != -1) return false;   // else branch: 0
        for (const Bit& b : t) {
          if (b.gate != ~0u) return false;   // nested gates
          r.push_back(b.var == -1 ? zero : Bit{b.var, b.bit, gate});   // (a constant 1 bit would need a gated const)
          if (b.var == -2) return false;
        }
        break;
      }
      default: return false;
    }
    if (n.op != MQ_OP_SLT && r.size() != n.width) return false;
  }
  const std::vector<Bit>& out = val[nn - 1];
  const uint32_t W = root.width, nl = (W + 31) / 32;
  h.size_var = size_var;
  h.limb_slots.assign(nl, {});
  h.const_or.assign(nl, 0);
  for (uint32_t l = 0; l < nl; l++) {
    for (uint32_t b = 32 * l; b < std::min(W, 32 * l + 32);) {
      const Bit& s = out[b];
      if (s.var < 0) {
        if (s.var == -2) h.const_or[l] |= 1u << (b - 32 * l);
        b++;
        continue;
      }
      uint32_t len = 1;
      while (b + len < std::min(W, 32 * l + 32)) {
        const Bit& t = out[b + len];
        if (t.var != s.var || t.gate != s.gate || t.bit != s.bit + len || t.bit / 32 != s.bit / 32) break;
        len++;
      }
      const uint32_t mask = len == 32 ? ~0u : (1u << len) - 1u;
      h.limb_slots[l].push_back(
          mq_tapes::CwSlotHost{s.var, s.bit / 32, mask, (s.bit % 32) | ((b - 32 * l) << 8), s.gate});
      b += len;
    }
  }
  return true;
}

static int set_columns_one(mq_tapes* T, const mq_tape_batch* progs, const int32_t* var_index, const int32_t* level_in,
                           int32_t n_columns) {
  mq_ctx* c = T->ctx;
  if (!c) return MQ_ERR_STATE;   // the context was destroyed
  HIPCHK(hipSetDevice(c->device));
  T->clevels.clear();
  T->col_var.assign(var_index, var_index + n_columns);
  T->col_level.assign(level_in, level_in + n_columns);
  T->col_direct_mask.assign(n_columns, 0);
  T->bmask_gen = ~0ull;
  T->col_width.assign(n_columns, 0);
  T->kc.clear();
  T->kc_level.clear();
  T->cw.clear();
  T->cw_level.clear();
  if (n_columns == 0) return MQ_OK;
  CompileLimits lim;
  lim.g_depth = kQsaStackG;
  lim.value_root = true;
  std::vector<CompiledTape> ct(n_columns);
  parallel_for(n_columns, 16, [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; k++) ct[k] = compile_tape(progs, (int32_t)k, lim);
  });
  for (int k = 0; k < n_columns; k++) {
    if (!ct[k].supported) {
      g_last_error = "column program " + std::to_string(k) + " unsupported: " + ct[k].why;
      return MQ_ERR_TAPE;
    }
    if (level_in[k] < 0) return MQ_ERR_ARG;
    const int64_t last = progs->tape_offsets[k + 1] - 1;
    T->col_width[k] = progs->nodes[last].width;
  }
  // keccak columns (MQ_NO_KECCAK_COLUMNS=1: leave them to the interpreters), and the predicate
  // columns over them (lower.py keccak_predicates), which the keccak column kernel evaluates
  // from the digest it computed (MQ_NO_KECCAK_PREDICATES=1: on the interpreters)
  std::vector<char> kcm(n_columns, 0), kpm(n_columns, 0);
  std::vector<mq_tapes::KcPiece> kc_pieces_tmp;
  std::vector<std::vector<mq_tapes::KcPiece>> kpieces(n_columns);
  std::unordered_map<int32_t, int> kcol_of_var;   // keccak column target variable -> column
  T->kc_consts.clear();
  if (!std::getenv("MQ_NO_KECCAK_COLUMNS")) {
    for (int k = 0; k < n_columns; k++)
      if (kc_match(progs, k, kpieces[k], T->kc_consts)) {
        kcm[k] = 1;
        kcol_of_var[var_index[k]] = k;
      }
  }
  // bit-gather columns (calldata words; MQ_NO_GATHER_COLUMNS=1: leave them to the interpreters)
  std::vector<char> cwm(n_columns, 0);
  std::vector<mq_tapes::CwHost> cwh(n_columns);
  if (!std::getenv("MQ_NO_GATHER_COLUMNS")) {
    parallel_for(n_columns, 16, [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; k++)
        if (!kcm[k] && T->col_width[k] != 0 && cw_compile(progs, (int32_t)k, cwh[k])) cwm[k] = 1;
    });
  }
  std::vector<int> kp_of(n_columns, -1);   // predicate column -> its keccak column
  std::vector<mq_tapes::KcPredHost> kp_host(n_columns);
  if (!kcol_of_var.empty() && !std::getenv("MQ_NO_KECCAK_PREDICATES")) {
    for (int k = 0; k < n_columns; k++) {
      if (kcm[k] || T->col_width[k] != 0) continue;
      int32_t v;
      mq_tapes::KcPredHost ph{};
      if (!kp_match(progs, k, &v, &ph.kind, &ph.bits, ph.c)) continue;
      auto it = kcol_of_var.find(v);
      if (it == kcol_of_var.end()) continue;
      ph.target = var_index[k];
      kp_of[k] = it->second;
      kp_host[k] = ph;
      kpm[k] = 1;
    }
  }
  // levels from the programs: a column is one level past the deepest column it reads, and a
  // predicate column sits at its keccak column's level (computed in the same launch); otherwise
  // this is the lowering's own level (lower.py lower_batch), which the C-ABI also passes
  std::vector<int> level(n_columns, -1);
  {
    std::unordered_map<int32_t, int> col_of_var;
    for (int k = 0; k < n_columns; k++) col_of_var[var_index[k]] = k;
    std::vector<std::vector<int>> reads(n_columns);
    for (int k = 0; k < n_columns; k++)
      for (int64_t i = progs->tape_offsets[k]; i < progs->tape_offsets[k + 1]; i++) {
        const mq_node& n = progs->nodes[i];
        if (n.op != MQ_OP_VAR) continue;
        auto it = col_of_var.find((int32_t)n.a);
        if (it != col_of_var.end() && it->second != k) reads[k].push_back(it->second);
      }
    std::vector<char> state(n_columns, 0);   // 1 = on the DFS stack
    std::function<int(int)> lv = [&](int k) -> int {
      if (level[k] >= 0) return level[k];
      if (state[k]) throw std::runtime_error("cyclic columns");
      state[k] = 1;
      int l;
      if (kp_of[k] >= 0) {
        l = lv(kp_of[k]);
      } else {
        l = 0;
        for (int j : reads[k]) l = std::max(l, lv(j) + 1);
      }
      state[k] = 0;
      return level[k] = l;
    };
    try {
      for (int k = 0; k < n_columns; k++) lv(k);
    } catch (const std::exception&) {
      g_last_error = "hoisted columns read each other in a cycle";
      return MQ_ERR_ARG;
    }
  }
  int max_level = 0;
  for (int k = 0; k < n_columns; k++) max_level = std::max(max_level, level[k]);
  T->col_level.assign(level.begin(), level.end());
  T->col_direct_mask.assign(kpm.begin(), kpm.end());
  std::vector<uint32_t> prog, consts;
  std::vector<GDesc> descs;
  // G assembly eligibility is structural here, as for tapes (mq_tapes_upload).  Columns shorter
  // than kColAsmMinNodes stay on the HIP C++ column kernel.  With slotted counters and the
  // decoded program window every column size runs faster on qsg_kernel (profiles/r02n_*: C3
  // 90.5 -> 84.4 ms with all columns there; before, r01p_*, short columns lost 45 vs 24 ms).
  // MQ_G_COL_MIN_NODES overrides the threshold.
  int64_t min_nodes = kColAsmMinNodes;
  if (const char* e = std::getenv("MQ_G_COL_MIN_NODES")) min_nodes = std::atol(e);
  // keccak columns level by level, each with its predicate columns
  T->kc.clear();
  T->kc_gen = ~0ull;
  T->kc_level.assign((size_t)max_level + 1, {0, 0});
  for (int lv = 0; lv <= max_level; lv++) {
    T->kc_level[lv].first = (int)T->kc.size();
    for (int k = 0; k < n_columns; k++) {
      if (level[k] != lv || !kcm[k]) continue;
      mq_tapes::KcHost h;
      h.pieces = std::move(kpieces[k]);
      h.target = var_index[k];
      double nodes = ct[k].n_nodes, ops = ct[k].alg_ops;
      for (int j = 0; j < n_columns; j++)
        if (kp_of[j] == k) {
          h.preds.push_back(kp_host[j]);
          nodes += ct[j].n_nodes;
          ops += ct[j].alg_ops;
        }
      h.n_nodes = (uint32_t)std::min(nodes, 4.0e9);
      h.alg_ops = (uint32_t)std::min(ops, 4.0e9);
      T->kc.push_back(std::move(h));
    }
    T->kc_level[lv].second = (int)T->kc.size() - T->kc_level[lv].first;
  }
  T->cw.clear();
  T->cw_gen = ~0ull;
  T->cw_level.assign((size_t)max_level + 1, {0, 0});
  for (int lv = 0; lv <= max_level; lv++) {
    T->cw_level[lv].first = (int)T->cw.size();
    for (int k = 0; k < n_columns; k++) {
      if (level[k] != lv || !cwm[k]) continue;
      mq_tapes::CwHost& h = cwh[k];
      h.target = var_index[k];
      h.n_nodes = ct[k].n_nodes;
      h.alg_ops = (uint32_t)std::min(ct[k].alg_ops, 4.0e9);
      T->cw.push_back(std::move(h));
    }
    T->cw_level[lv].second = (int)T->cw.size() - T->cw_level[lv].first;
  }
  for (int k = 0; k < n_columns; k++)
    if (cwm[k]) kcm[k] = 2;   // (off the interpreters below, as keccak columns)
  std::vector<char> gq(n_columns, 0);
  if (c->qsa_ready)
    for (int k = 0; k < n_columns; k++)
      gq[k] = !kcm[k] && !kpm[k] && ct[k].L == 8 && !ct[k].keccak && ct[k].n_temps <= kQsaMaxTemps &&
              (int64_t)ct[k].n_nodes >= min_nodes && qsa_translate(c, 1, false, ct[k], nullptr, nullptr);
  T->cq_ct.clear();
  T->cq_var.clear();
  T->cq_bool.clear();
  T->cq_gen = ~0ull;
  T->cq_live = false;
  T->clevels.resize((size_t)max_level + 1);
  for (int lv = 0; lv <= max_level; lv++) {
    T->clevels[lv].cq_begin = (int)T->cq_ct.size();
    // pass -1: the G-eligible L = 8 columns (front of v[0]); pass g: kind g (qs_column_kernel)
    for (int pass = -1; pass < kGen; pass++) {
      mq_tapes::Variant& v = T->clevels[lv].v[pass < 0 ? 0 : pass];
      v.L = pass < 0 ? 8 : kGenL[pass];
      v.keccak = pass < 0 ? false : kGenK[pass];
      if (pass != 0) v.begin = (int)descs.size();
      for (int k = 0; k < n_columns; k++) {
        const CompiledTape& x = ct[k];
        if (level[k] != lv || kcm[k] || kpm[k]) continue;
        if (pass == -1 && !gq[k]) continue;
        if (pass >= 0 && (gen_kind(x) != pass || (pass == 0 && gq[k]))) continue;
        GDesc d{};
        d.prog_off = (uint32_t)prog.size();
        d.prog_len = (uint32_t)x.prog.size();
        d.tape = (uint32_t)var_index[k];
        d.const_base = (uint32_t)consts.size();
        d.n_nodes = x.n_nodes;
        d.n_temps = (uint32_t)x.n_temps;
        d.depth = (uint32_t)x.depth;
        d.alg_ops = (uint32_t)std::min(x.alg_ops, 4.0e9);
        prog.insert(prog.end(), x.prog.begin(), x.prog.end());
        consts.insert(consts.end(), x.consts.begin(), x.consts.end());
        descs.push_back(d);
        v.max_temps = std::max(v.max_temps, x.n_temps);
        v.max_depth = std::max(v.max_depth, x.depth);
        if (pass == -1) {
          T->cq_ct.push_back(x);
          T->cq_var.push_back(var_index[k]);
          T->cq_bool.push_back(T->col_width[k] == 0 ? 1 : 0);
        }
      }
      if (pass == -1) T->clevels[lv].v8q = (int)descs.size() - v.begin;
      if (pass != -1) v.count = (int)descs.size() - v.begin;
    }
  }
  consts.resize(consts.size() + 16, 0);
  prog.push_back(gword(G_END, 0, 0));
  HIPCHK(T->cdescs.upload(descs.data(), descs.size(), c->stream));
  HIPCHK(T->cprog.upload(prog.data(), prog.size(), c->stream));
  HIPCHK(T->cconsts.upload(consts.data(), consts.size(), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MQ_OK;
}

int mq_tapes_set_columns(mq_tapes* T, const mq_tape_batch* progs, const int32_t* var_index, const int32_t* level,
                         int32_t n_columns) {
  if (!T || n_columns < 0 || (n_columns > 0 && (!progs || !var_index || !level || progs->n_tapes != n_columns)))
    return MQ_ERR_ARG;
  int rc = set_columns_one(T, progs, var_index, level, n_columns);
  for (size_t i = 0; rc == MQ_OK && i < T->peers.size(); i++) rc = set_columns_one(T->peers[i], progs, var_index, level, n_columns);
  return rc;
}

// Workgroups (one wave each) of the persistent HIP C++ kernels: 16 per CU on 256 CUs; each
// strides over the (model tile, tape group) items.  Bounds the temp scratch to
// grid * temps * 2 KB (L = 8).
static constexpr int64_t kPersistentGroups = 4096;

static KArgs make_args(mq_ctx* c, mq_tapes* T, const mq_tapes::Variant& v) {
  KArgs a{};
  a.descs = T->descs.as<GDesc>() + v.begin;
  a.n_desc = v.count;
  const int64_t tiles = (c->M + 63) / 64;
  // ~8k (tile, tape group) items: enough to fill 256 CUs many times over with a short tail
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
  const int64_t groups = (int64_t(v.count) + tpg - 1) / tpg;
  a.tiles = tiles;
  a.n_items = tiles * groups;
  // the 1024/2048-bit kinds: 64-128 KB of LDS stack per wave, so fewer resident waves; a smaller
  // persistent grid also bounds their temp scratch (grid x temps x 8-16 KB)
  a.grid = (int)std::min<int64_t>(a.n_items, v.L >= 32 ? kPersistentGroups / 4 : kPersistentGroups);
  a.scratch = nullptr;
  a.stack_slots = std::max(1, v.max_depth);
  return a;
}

static KArgs make_col_args(mq_ctx* c, mq_tapes* T, const mq_tapes::Variant& v) {
  KArgs a = make_args(c, T, v);
  a.descs = T->cdescs.as<GDesc>() + v.begin;
  a.prog = T->cprog.as<uint32_t>();
  a.consts = T->cconsts.as<uint32_t>();
  a.mode = 2;
  return a;
}

// G programs stream through a 64-word VGPR window (gen_qsa.py NEXT_G): insert a REFILL word
// wherever the next handler word and its inline data would not fit in the current window (the
// refilled window starts right after the REFILL word).
static void qsa_window_layout(const mq_ctx* c, std::vector<uint32_t>& prog) {
  // Windows are the program's aligned 64-word blocks: a handler group (word + inline data) that
  // does not fit the rest of a block is preceded by REFILL and moves to the next block (the gap
  // is padded with END), and the program is padded to a whole block.  So the window after the
  // current one is always 256 bytes further, which the kernel prefetches (gen_qsa.py NWIN), and
  // the programs of consecutive descriptors are contiguous blocks: the next tape's first window
  // is the prefetch of the current tape's last one.
  const std::vector<uint8_t>& data_words = c->qsa_data_words;
  const uint32_t refill = hword(1, c->qsa_off[1][c->qsa_index[1][QK_REFILL][0][0]]);
  const uint32_t endw = hword(1, c->qsa_off[1][c->qsa_index[1][QK_END][0][0]]);
  std::vector<uint32_t> out;
  out.reserve(prog.size() + prog.size() / 32 + 64);
  size_t pos = 0;
  for (size_t i = 0; i < prog.size();) {
    const size_t g = 1 + (size_t)data_words[prog[i] & 0xFFFFu];
    if (pos + g > 63) {
      out.push_back(refill);
      out.insert(out.end(), 63 - pos, endw);
      pos = 0;
    }
    for (size_t j = 0; j < g && i + j < prog.size(); j++) out.push_back(prog[i + j]);
    pos += g;
    i += g;
  }
  if (pos) out.insert(out.end(), 64 - pos, endw);
  prog.swap(out);
}

// Column programs are short (C3: ~6 nodes): padding each to whole 64-word blocks made every column
// start with a window load, a memory round trip per column program (the G profile charged it to
// FRAME3: ~20 % of C3's cycles).  They are packed back to back instead: a program starts at the
// next word (or, when its first handler group would not fit the block, at the next block), the
// REFILL rule of qsa_window_layout applies inside it, and the kernel starts a program that lies in
// its current window without a load (gen_qsa.py load_window).  Returns the program's word offset;
// pos = the next word's position in its block.
static uint32_t qsa_pack_program(const mq_ctx* c, std::vector<uint32_t>& out, size_t& pos,
                                 const std::vector<uint32_t>& prog) {
  const std::vector<uint8_t>& data_words = c->qsa_data_words;
  const uint32_t refill = hword(1, c->qsa_off[1][c->qsa_index[1][QK_REFILL][0][0]]);
  const uint32_t endw = hword(1, c->qsa_off[1][c->qsa_index[1][QK_END][0][0]]);
  if (!prog.empty() && pos + 1 + (size_t)data_words[prog[0] & 0xFFFFu] > 63) {
    out.insert(out.end(), 64 - pos, endw);
    pos = 0;
  }
  const uint32_t start = (uint32_t)out.size();
  for (size_t i = 0; i < prog.size();) {
    const size_t g = 1 + (size_t)data_words[prog[i] & 0xFFFFu];
    if (pos + g > 63) {
      out.push_back(refill);
      out.insert(out.end(), 63 - pos, endw);
      pos = 0;
    }
    for (size_t j = 0; j < g && i + j < prog.size(); j++) out.push_back(prog[i + j]);
    pos += g;
    i += g;
  }
  return start;
}

// Push counts of the variables (<= 256 bits) a set of compiled programs reads.
static std::vector<int64_t> count_pushes(const mq_ctx* c, const std::vector<CompiledTape>& cts,
                                         const std::vector<char>* skip = nullptr) {
  std::vector<int64_t> pushes(c->var_nl_h.size(), 0);
  for (size_t i = 0; i < cts.size(); i++) {
    if (skip && (*skip)[i]) continue;
    const auto& pr = cts[i].prog;
    for (size_t pc = 0; pc < pr.size(); pc++) {
      const uint32_t op = pr[pc] & 0xFFu, imm = pr[pc] >> 12;
      if ((op == G_PUSH_VAR || (op == G_PUSH_VAR_B && !(imm < c->bmask_of_var.size() && c->bmask_of_var[imm] >= 0))) &&
          imm < pushes.size() && c->var_nl_h[imm] <= 8)
        pushes[imm]++;
      if (has_imm2(op)) pc++;
    }
  }
  return pushes;
}

// G kernel LDS staging plan: the most pushed variables (not preloaded) whose rows fit the
// workgroup's staging budget get consecutive LDS slots (gen_qsa.py stage_rows); their pushes
// become LDS reads.  Budget: MQ_G_STAGE_KB (default 26: the 80-VGPR G runs 6 waves per SIMD =
// 6 workgroups of 4 waves per CU, and 6 x 26 KB fit the CU's 160 KB; 40 KB, the budget of the
// 5-wave layout, capped C5 at 4 workgroups per CU: 70.5 vs 61.6 ms, profiles/r04c) KB per
// workgroup minus the temps of its 4 waves.  Every workgroup loads its rows
// once, so a variable is staged only when the workgroup's tapes (wg_share of the batch's
// programs) push it at least MQ_G_STAGE_MIN (default 1.5) times on average
// (profiles/r02t_*: 40 KB with no such floor sped C3 up and slowed C5, whose groups cover few
// tapes).  stage_rows is padded to a multiple of 8 with the zero row.
static int64_t g_tapes_per_group(int64_t n, int64_t M);
static int64_t cq_tapes_per_group(int64_t n, int64_t M);


static void plan_stage(const mq_ctx* c, const std::vector<int64_t>& pushes, const std::vector<int>* gpre, int temps,
                       double wg_share, std::vector<int>& gstage, std::vector<uint32_t>& rows) {
  int64_t kb = 26;
  if (const char* e = std::getenv("MQ_G_STAGE_KB")) kb = std::atol(e);
  double min_pushes = 1.5;
  if (const char* e = std::getenv("MQ_G_STAGE_MIN")) min_pushes = std::atof(e);
  const int64_t budget = (kb * 1024 - 4 * (int64_t)temps * 2048) / 256;
  gstage.assign(c->var_nl_h.size(), -1);
  rows.clear();
  std::vector<int> order;
  for (size_t v = 0; v < pushes.size(); v++)
    if (pushes[v] > 0 && !(gpre && v < gpre->size() && (*gpre)[v] >= 0)) order.push_back((int)v);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pushes[a] > pushes[b]; });
  for (int v : order) {
    const int64_t nl = c->var_nl_h[v];
    if ((double)pushes[v] * wg_share < min_pushes) break;   // (sorted by pushes)
    if ((int64_t)rows.size() + nl > budget) continue;
    gstage[v] = (int)rows.size();
    for (int64_t l = 0; l < nl; l++) rows.push_back(c->var_off_h[v] + (uint32_t)l);
  }
  const uint32_t zero_row = (uint32_t)(c->var_off_h.empty() ? 0 : c->var_off_h.back() + c->var_nl_h.back());
  while (rows.size() % 8) rows.push_back(zero_row);
}

// (Re)translate the QSA-eligible tapes for the current model batch (variable rows, function
// table): the P kernel when every variable a tape reads is preloaded, the G kernel otherwise.
// If one tape does not translate, the whole group runs on the HIP C++ kernel for this batch.
// A flat conjunction (fc.hip): the stack program of x, run abstractly, leaves an AND of Bool
// variables (negated or not) and compares of one model variable of at most 256 bits with a
// constant; temps, arithmetic and anything else do not match.  A Bool variable without a lane-mask
// index is a compare of its 0/1 row with 1.  Appends its masks (index | negated << 31) and
// compares (FcCmpH: the variable's first row and limbs, the predicate as an accept mask over
// (x < c, x == c, x > c), the constant; signed compares have the sign bit flipped) to the lists.
struct FcCmpH {
  uint32_t row, nl, accept;
  uint32_t c[8], f[8];
  uint32_t src_nl = 0;   // limbs of the compared variable's rows (0: nl; fewer when it was zero-extended)
  uint32_t nx = 0;       // unary atoms (fca only): the variable's transform, nx steps
  FcXop xf[kFcMaxXops] = {};
};
// accept masks: bit 0 x < c, bit 1 x == c, bit 2 x > c
static constexpr uint32_t kAccEq = 2, kAccNe = 5, kAccLt = 1, kAccLe = 3, kAccGt = 4, kAccGe = 6;
// LDS budget of the flat-conjunction kernel's staging, per tile (fc.hip stages FC_TILES = 4
// tiles a workgroup): rows of 256 B (40 KB for 4 tiles) and masks of 8 B (8 KB for 4 tiles);
// only what a launch uses is allocated (C4's tapes: ~5 KB)
static constexpr int kFcStageRows = 40;
static constexpr int kFcStageMasks = 256;

// A program that is a flat conjunction of atoms (Bool variables, variable-constant compares),
// or the negation of one: ORs of atoms and of negated conjunctions are taken by De Morgan
// (OR(a, b) = NOT(AND(NOT a, NOT b))), the result negation returned in *neg.
// With `unary` (the two-phase kernel only) an atom may also compare a constant with a unary
// function of its variable: zero extension (free: values are canonical), sign extension, extract,
// shifts by constants, and division / remainder by small constants (FcXop, fc.hip fx_apply).
static bool fc_match(const mq_ctx* c, const CompiledTape& x, std::vector<uint32_t>& masks, std::vector<FcCmpH>& cmps,
                     bool* neg = nullptr, bool unary = false) {
  struct Item {
    int kind = 0;   // 0 model variable (BV, through xf), 1 constant, 2 conjunction (negated when neg)
    uint32_t v = 0;
    uint32_t w = 0;   // kind 0: the width of its current value
    bool neg = false;
    std::vector<uint32_t> m;
    std::vector<FcCmpH> q;
    std::vector<FcXop> xf;
  };
  // the 256-bit constant at word offset k of the tape's pool, limb by limb (8 limbs, zero padded)
  auto const_limbs = [&](uint32_t k, uint32_t out[8]) {
    for (int i = 0; i < 8; i++) out[i] = x.consts[k + i];
  };
  // value (< 2^32 or saturated) of a constant of width w: its limbs above 0 are zero?
  auto small_value = [&](const uint32_t l[8], uint64_t* v) {
    for (int i = 2; i < 8; i++)
      if (l[i]) return false;
    *v = (uint64_t)l[0] | ((uint64_t)l[1] << 32);
    return true;
  };
  // NOT of an item as a plain conjunction: a single atom negated, or a negated conjunction's body
  auto negate_to_conj = [](Item& a) -> bool {
    if (a.neg) {
      a.neg = false;
      return true;
    }
    if (a.m.size() + a.q.size() != 1) return false;
    if (!a.m.empty()) a.m[0] ^= 0x80000000u;
    else a.q[0].accept ^= 7u;
    return true;
  };
  std::vector<Item> st;
  const auto& pr = x.prog;
  auto bool_item = [&](uint32_t v, Item& it) {
    it.kind = 2;
    if (v < c->bmask_of_var.size() && c->bmask_of_var[v] >= 0) {
      it.m.push_back((uint32_t)c->bmask_of_var[v]);
    } else {
      FcCmpH q{};
      q.row = c->var_off_h[v];
      q.nl = 1;
      q.accept = kAccEq;
      q.c[0] = 1;
      it.q.push_back(q);
    }
  };
  for (size_t pc = 0; pc < pr.size(); pc++) {
    const uint32_t w = pr[pc], op = w & 0xFFu, imm = w >> 12;
    if (op == G_END) break;
    if (unary && op == G_CONCAT && pc + 1 < pr.size()) {
      // Concat(0, x): a zero extension (bitvec.py:16-22 pads a narrower operand so; EVM BYTE)
      const uint32_t w2 = pr[++pc];
      if (st.size() < 2 || st.back().kind != 0 || st[st.size() - 2].kind != 1 || st.back().w > imm || w2 > 256) return false;
      uint32_t hl[8];
      const_limbs(st[st.size() - 2].v, hl);
      for (int i = 0; i < 8; i++)
        if (hl[i]) return false;
      Item v = std::move(st.back());
      st.pop_back();
      st.back() = std::move(v);
      st.back().w = w2;
      continue;
    }
    if (unary && (op == G_EXTRACT || op == G_SEXT) && pc + 1 < pr.size()) {
      // (the two ops with a second word: the result width)
      const uint32_t w2 = pr[++pc];
      if (st.empty() || st.back().kind != 0 || st.back().xf.size() >= (size_t)kFcMaxXops) return false;
      Item& a = st.back();
      // (a value narrower than the op's operand was zero-extended: canonical values are, so the
      // op reads it at the wider width as is)
      if (op == G_EXTRACT) {
        if (imm + w2 > 256 || w2 == 0) return false;
        a.xf.push_back(FcXop{FX_EXTRACT | (std::max(a.w, imm + w2) << 8), imm, w2, 0});
      } else {
        if (imm < a.w || w2 <= imm || w2 > 256) return false;
        a.xf.push_back(FcXop{FX_SEXT | (imm << 8), w2, 0, 0});
      }
      a.w = w2;
      continue;
    }
    if (has_imm2(op)) return false;
    Item it;
    switch (op) {
      case G_PUSH_VAR:
        if (imm >= c->var_nl_h.size() || c->var_width[imm] == 0 || c->var_nl_h[imm] > 8) return false;
        it.kind = 0;
        it.v = imm;
        it.w = c->var_width[imm];
        st.push_back(std::move(it));
        break;
      case G_LSHR: case G_SHL: case G_ASHR: case G_UREM: case G_UDIV: case G_SMOD: case G_SREM: case G_SDIV: {
        // a unary step: the variable (through its steps so far) OP a constant
        if (!unary || st.size() < 2 || st.back().kind != 1 || st[st.size() - 2].kind != 0) return false;
        const uint32_t kc = st.back().v;
        st.pop_back();
        Item& a = st.back();
        const uint32_t w = imm;   // (>= the value's width: a zero-extended value, read as is)
        if (imm < a.w || w == 0 || w > 256 || a.xf.size() >= (size_t)kFcMaxXops) return false;
        uint32_t l[8];
        const_limbs(kc, l);
        uint64_t k = 0;
        const bool small = small_value(l, &k);
        if (op == G_LSHR || op == G_SHL || op == G_ASHR) {
          const uint32_t sh = (!small || k >= w) ? w : (uint32_t)k;   // (>= w: the kernel's saturation)
          a.xf.push_back(FcXop{(op == G_LSHR ? FX_LSHR : op == G_SHL ? FX_SHL : FX_ASHR) | (w << 8), sh, 0, 0});
        } else if (op == G_UREM || op == G_UDIV) {
          if (!small || k == 0 || k >= (1u << 21)) return false;
          a.xf.push_back(FcXop{(op == G_UREM ? FX_UREM : FX_UDIV) | (w << 8), (uint32_t)k, 0, 0});
        } else {
          // signed divisor: |d| and its sign at width w (two's complement of the w-bit constant)
          bool dneg = ((l[(w - 1) / 32] >> ((w - 1) % 32)) & 1u) != 0;
          uint32_t m[8];
          for (int i = 0; i < 8; i++) m[i] = l[i];
          if (dneg) {   // |d| = -d mod 2^w
            uint64_t cy = 1;
            for (int i = 0; i < 8; i++) {
              const uint64_t t = (uint64_t)(~m[i]) + cy;
              m[i] = (uint32_t)t;
              cy = t >> 32;
            }
            for (int i = 0; i < 8; i++) {
              const uint32_t lo = 32u * i;
              if (w <= lo) m[i] = 0;
              else if (w < lo + 32) m[i] &= (1u << (w - lo)) - 1u;
            }
          }
          uint64_t ad = 0;
          if (!small_value(m, &ad) || ad == 0 || ad >= (1u << 21)) return false;
          const uint32_t code = op == G_SMOD ? FX_SMOD : op == G_SREM ? FX_SREM : FX_SDIV;
          a.xf.push_back(FcXop{code | (w << 8), (uint32_t)ad, dneg ? 1u : 0u, 0});
        }
        a.w = w;
        break;
      }
      case G_PUSH_VAR_B:
        if (imm >= c->var_nl_h.size() || c->var_width[imm] != 0) return false;
        bool_item(imm, it);
        st.push_back(std::move(it));
        break;
      case G_PUSH_CONST:
        if ((size_t)imm + 8 > x.consts.size()) return false;
        it.kind = 1;
        it.v = imm;
        st.push_back(std::move(it));
        break;
      case G_PUSH_BOOL:
        if (imm != 1) return false;
        it.kind = 2;   // TRUE: the empty conjunction
        st.push_back(std::move(it));
        break;
      case G_NOT: {
        if (st.empty() || st.back().kind != 2) return false;
        Item& a = st.back();
        if (!negate_to_conj(a)) a.neg = true;   // NOT of a conjunction of several atoms
        break;
      }
      case G_AND: case G_OR: {
        if (st.size() < 2 || st.back().kind != 2 || st[st.size() - 2].kind != 2) return false;
        Item b = std::move(st.back());
        st.pop_back();
        Item& a = st.back();
        if (op == G_OR) {   // NOT(AND(NOT a, NOT b))
          if (!negate_to_conj(a) || !negate_to_conj(b)) return false;
          a.neg = true;
        } else if (a.neg || b.neg) {
          return false;
        }
        a.m.insert(a.m.end(), b.m.begin(), b.m.end());
        a.q.insert(a.q.end(), b.q.begin(), b.q.end());
        break;
      }
      case G_EQ: case G_ULT: case G_ULE: case G_UGT: case G_UGE:
      case G_SLT: case G_SLE: case G_SGT: case G_SGE: {
        if (st.size() < 2) return false;
        Item r = std::move(st.back());
        st.pop_back();
        Item l = std::move(st.back());
        st.pop_back();
        bool swap;
        if (l.kind == 0 && r.kind == 1) swap = false;
        else if (l.kind == 1 && r.kind == 0) swap = true;
        else if (unary && l.kind == 1 && r.kind == 1 && imm > 0 && imm <= 256 && !c->var_off_h.empty()) {
          // two constants (an unfolded compare): its truth value — TRUE is the empty
          // conjunction, FALSE an atom that accepts nothing
          uint32_t a[8], b[8];
          const_limbs(l.v, a);
          const_limbs(r.v, b);
          if (op >= G_SLT) {
            a[(imm - 1) / 32] ^= 1u << ((imm - 1) % 32);
            b[(imm - 1) / 32] ^= 1u << ((imm - 1) % 32);
          }
          int cmp = 0;
          for (int i = 7; i >= 0 && !cmp; i--) cmp = a[i] < b[i] ? -1 : (a[i] > b[i] ? 1 : 0);
          bool t;
          switch (op) {
            case G_EQ: t = cmp == 0; break;
            case G_ULT: case G_SLT: t = cmp < 0; break;
            case G_ULE: case G_SLE: t = cmp <= 0; break;
            case G_UGT: case G_SGT: t = cmp > 0; break;
            default: t = cmp >= 0; break;
          }
          it.kind = 2;
          if (!t) {
            FcCmpH q{};
            q.row = c->var_off_h[0];
            q.nl = 1;
            q.accept = 0;
            it.q.push_back(q);
          }
          st.push_back(std::move(it));
          break;
        } else {
          return false;
        }
        const Item& var = swap ? r : l;
        const Item& cst = swap ? l : r;
        const uint32_t wdt = imm;
        // (a narrower value compared at a wider width: a zero-extended column read, free)
        if (wdt == 0 || wdt > 256 || var.w > wdt || (!unary && (var.w != wdt || !var.xf.empty()))) return false;
        FcCmpH q{};
        q.row = c->var_off_h[var.v];
        q.nl = (wdt + 31) / 32;
        q.src_nl = c->var_nl_h[var.v];
        q.nx = (uint32_t)var.xf.size();
        for (size_t k = 0; k < var.xf.size(); k++) q.xf[k] = var.xf[k];
        for (uint32_t i = 0; i < q.nl; i++) q.c[i] = x.consts[cst.v + i];
        // x OP c with the variable on the left; a constant on the left mirrors the order
        switch (op) {
          case G_EQ: q.accept = kAccEq; break;
          case G_ULT: case G_SLT: q.accept = swap ? kAccGt : kAccLt; break;
          case G_ULE: case G_SLE: q.accept = swap ? kAccGe : kAccLe; break;
          case G_UGT: case G_SGT: q.accept = swap ? kAccLt : kAccGt; break;
          default: q.accept = swap ? kAccLe : kAccGe; break;
        }
        if (op >= G_SLT) {   // signed: flip the sign bit of both sides, then compare unsigned
          q.f[q.nl - 1] = 1u << ((wdt - 1) % 32);
          q.c[q.nl - 1] ^= q.f[q.nl - 1];
        }
        it.kind = 2;
        it.q.push_back(q);
        st.push_back(std::move(it));
        break;
      }
      default:
        return false;
    }
  }
  if (st.size() != 1 || st[0].kind != 2) return false;
  if (st[0].neg && !neg) return false;
  if (neg) *neg = st[0].neg;
  masks.insert(masks.end(), st[0].m.begin(), st[0].m.end());
  cmps.insert(cmps.end(), st[0].q.begin(), st[0].q.end());
  return true;
}

// The flat-conjunction kernel's tables for the tapes (or columns) `cand` of the lists `fm` / `fq`
// (fc_match): the compared variables and the masks the most compares / tapes read are staged in
// LDS within the budgets; a candidate reading one that is not staged is dropped from `cand`'s
// kernel (keep[i] = 0: it stays on the interpreter).  out_of(i) and mask_out(i) give FcTape.out /
// .mask_out, nodes_ops(i) its metric words.
struct FcPlan {
  std::vector<FcTape> tapes;
  std::vector<uint32_t> mask_lds;
  std::vector<FcCmp> cmps;
  std::vector<uint32_t> stage_rows, stage_masks;
  std::vector<unsigned long long> prefix;
};
static void fc_plan(const mq_ctx* c, const std::vector<std::vector<uint32_t>>& fm, const std::vector<std::vector<FcCmpH>>& fq,
                    const std::vector<char>& negated, std::vector<char>& keep, const std::function<uint32_t(size_t)>& out_of,
                    const std::function<int32_t(size_t)>& mask_out,
                    const std::function<std::pair<uint32_t, uint32_t>(size_t)>& nodes_ops, FcPlan& P) {
  const uint32_t zero_row = (uint32_t)(c->var_off_h.empty() ? 0 : c->var_off_h.back() + c->var_nl_h.back());
  std::map<uint32_t, int64_t> row_use, mask_use;
  std::map<uint32_t, uint32_t> row_nl;
  for (size_t i = 0; i < keep.size(); i++) {
    if (!keep[i]) continue;
    for (const auto& q : fq[i]) {
      row_use[q.row]++;
      row_nl[q.row] = q.nl;
    }
    for (uint32_t e : fm[i]) mask_use[e & 0x7FFFFFFFu]++;
  }
  auto by_use = [](const std::map<uint32_t, int64_t>& u) {
    std::vector<std::pair<int64_t, uint32_t>> o;
    for (const auto& kv : u) o.push_back({kv.second, kv.first});
    std::stable_sort(o.begin(), o.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    return o;
  };
  std::map<uint32_t, uint32_t> slot_of, mslot_of;
  for (const auto& o : by_use(row_use)) {
    const uint32_t nl = row_nl[o.second], width = nl <= 2 ? 2 : 8;   // (padded with the zero row)
    if (P.stage_rows.size() + width > (size_t)kFcStageRows) continue;
    slot_of[o.second] = (uint32_t)P.stage_rows.size();
    for (uint32_t l = 0; l < width; l++) P.stage_rows.push_back(l < nl ? o.second + l : zero_row);
  }
  for (const auto& o : by_use(mask_use)) {
    if (P.stage_masks.size() >= (size_t)kFcStageMasks) break;
    mslot_of[o.second] = (uint32_t)P.stage_masks.size();
    P.stage_masks.push_back(o.second);
  }
  P.prefix.assign(2, 0);
  for (size_t i = 0; i < keep.size(); i++) {
    if (!keep[i]) continue;
    bool ok = true;
    for (const auto& q : fq[i]) ok = ok && slot_of.count(q.row);
    for (uint32_t e : fm[i]) ok = ok && mslot_of.count(e & 0x7FFFFFFFu);
    if (!ok) {
      keep[i] = 0;
      continue;
    }
    FcTape f{};
    f.out = out_of(i);
    f.mask_out = mask_out(i);
    f.mask_off = (uint32_t)P.mask_lds.size();
    f.n_mask = (uint32_t)fm[i].size() | (negated[i] ? 0x80000000u : 0u);
    for (uint32_t e : fm[i]) P.mask_lds.push_back(8u * mslot_of[e & 0x7FFFFFFFu] | (e >> 31));
    if (!fm[i].empty())
      while (P.mask_lds.size() % 16) P.mask_lds.push_back(P.mask_lds.back());   // (the same AND again)
    f.cmp_off = (uint32_t)P.cmps.size();
    f.n_cmp = (uint32_t)fq[i].size();
    for (const auto& h : fq[i]) {
      FcCmp q{};
      q.h.slot = slot_of[h.row];
      q.h.nl = h.nl;
      q.h.accept = h.accept;
      q.h.c01 = (uint64_t)h.c[0] | ((uint64_t)h.c[1] << 32);
      q.h.f01 = (uint64_t)h.f[0] | ((uint64_t)h.f[1] << 32);
      for (int l = 0; l < 6; l++) {
        q.t.c[l] = h.c[2 + l];
        q.t.f[l] = h.f[2 + l];
      }
      P.cmps.push_back(q);
    }
    const auto no = nodes_ops(i);
    f.n_nodes = no.first;
    f.alg_ops = no.second;
    P.tapes.push_back(f);
    P.prefix.push_back(P.prefix[P.prefix.size() - 2] + f.n_nodes);
    P.prefix.push_back(P.prefix[P.prefix.size() - 2] + f.alg_ops);
  }
}

// The two-phase kernel's tables for the tapes `keep` of fm / fq (fca_kernel).  Tapes are taken
// in order into launches ("segments") of at most kFcaMaxAtoms distinct compares ("atoms": a
// compare and its negation are one atom, accept canonicalised to {1, 2, 3} and the negation moved
// into the list entry) and kFcStageMasks distinct Bool masks; a segment's atoms are ordered by
// the variable they read (one group per variable: its limbs are loaded once per tile).
struct FcaPlan {
  std::vector<FcCmp> atoms;
  std::vector<FcXf> xfs;   // parallel to atoms
  bool any_xf = false;     // some atom has a unary transform (else the launches pass xfs = nullptr)
  std::vector<FcaGroup> groups;
  std::vector<uint32_t> lists, chunk_off, tape_out, metric, stage_masks;
  std::vector<int32_t> col_mask;   // (columns: per kept column its lane-mask index)
  std::vector<FcaPlanSeg> segs;
};
static constexpr int kFcaMaxAtoms = 1024;   // 32 KB of LDS masks for the 4 tiles of a workgroup
static constexpr int kFcaGroupAtoms = 16;   // (C4 fca: 4 -> 213 us, 8 -> 196, 16 -> 186, 32 -> 199)
static void fca_plan(const mq_ctx* c, const std::vector<std::vector<uint32_t>>& fm, const std::vector<std::vector<FcCmpH>>& fq,
                     const std::vector<char>& negated, std::vector<char>& keep, const std::function<uint32_t(size_t)>& out_of,
                     const std::function<std::pair<uint32_t, uint32_t>(size_t)>& nodes_ops, FcaPlan& P,
                     const std::function<int32_t(size_t)>& mask_out = nullptr) {
  const uint32_t zero_row = (uint32_t)(c->var_off_h.empty() ? 0 : c->var_off_h.back() + c->var_nl_h.back());
  // key: row, source limbs, path (1: the 8-limb path — wide compares, zero-extended reads wider
  // than 64 bits, unary atoms), accept, compare limbs, then the constant / flip limbs and the
  // transform steps (atoms of one (row, source limbs, path) form groups)
  auto atom_key = [](const FcCmpH& h, bool* ng) {
    *ng = h.accept >= 4;
    const uint32_t src = h.src_nl ? h.src_nl : h.nl;
    const uint32_t general = (h.nx > 0 || h.nl > 2 || src > 2) ? 1u : 0u;
    std::vector<uint32_t> key{h.row, src, general, *ng ? (h.accept ^ 7u) : h.accept, h.nl, h.nx};
    for (uint32_t l = 0; l < h.nl; l++) {
      key.push_back(h.c[l]);
      key.push_back(h.f[l]);
    }
    for (uint32_t k = 0; k < h.nx; k++) {
      key.push_back(h.xf[k].code);
      key.push_back(h.xf[k].p0);
      key.push_back(h.xf[k].p1);
      key.push_back(h.xf[k].p2);
    }
    return key;
  };
  // the segment being built: its atoms / masks in arrival order, and its tapes' symbolic entries
  // (kind 0 mask slot, 1 atom; local id; negated)
  struct Ent {
    uint32_t kind, id, neg;
  };
  std::map<std::vector<uint32_t>, uint32_t> atom_of;
  std::vector<std::vector<uint32_t>> akeys;
  std::map<uint32_t, uint32_t> mask_of;
  std::vector<uint32_t> masks;
  std::vector<std::vector<Ent>> tl;
  std::vector<size_t> tsrc;
  P.chunk_off.assign(1, 0);
  auto close = [&]() {
    if (tl.empty()) return;
    FcaPlanSeg sg{};
    sg.atom_off = (int)P.atoms.size();
    sg.n_atoms = (int)akeys.size();
    sg.group_off = (int)P.groups.size();
    sg.tape_first = (int)P.tape_out.size();
    sg.n_tapes = (int)tl.size();
    sg.chunk_first = (int)P.chunk_off.size() - 1;
    sg.smask_off = (int)P.stage_masks.size();
    sg.n_smask = (int)masks.size();

    // atoms ordered by (variable row, limbs): groups
    std::vector<uint32_t> ord(akeys.size());
    for (size_t i = 0; i < ord.size(); i++) ord[i] = (uint32_t)i;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
      for (int f = 0; f < 3; f++)
        if (akeys[x][f] != akeys[y][f]) return akeys[x][f] < akeys[y][f];
      return false;
    });
    static const uint32_t group_atoms = [] {
      const char* e = std::getenv("MQ_FCA_GROUP_ATOMS");
      return e ? (uint32_t)std::max(1, std::atoi(e)) : (uint32_t)kFcaGroupAtoms;
    }();
    std::vector<uint32_t> pos(akeys.size());
    for (size_t r = 0; r < ord.size(); r++) {
      const std::vector<uint32_t>& key = akeys[ord[r]];
      pos[ord[r]] = (uint32_t)r;
      // (a group holds at most kFcaGroupAtoms atoms: the 4 waves take every fourth group, so one
      // variable's many compares must not land on one wave)
      if (r == 0 || akeys[ord[r - 1]][0] != key[0] || akeys[ord[r - 1]][1] != key[1] ||
          akeys[ord[r - 1]][2] != key[2] || P.groups.back().count >= group_atoms) {
        FcaGroup g{};
        const uint32_t nl = key[1];
        for (uint32_t l = 0; l < 8; l++) g.rows[l] = l < nl ? key[0] + l : zero_row;
        g.first = (uint32_t)r;
        g.nl = key[2] ? 8u : nl;   // (the kernel's 8-limb path for nl > 2)
        P.groups.push_back(g);
      }
      P.groups.back().count++;
      FcCmp q{};
      q.h.slot = 0;
      const uint32_t cnl = key[4], nx = key[5];
      q.h.nl = cnl;
      q.h.accept = key[3];
      uint32_t cc[8] = {0}, ff[8] = {0};
      for (uint32_t l = 0; l < cnl; l++) {
        cc[l] = key[6 + 2 * l];
        ff[l] = key[7 + 2 * l];
      }
      FcXf xf{};
      xf.n = nx;
      for (uint32_t k = 0; k < nx; k++) {
        const size_t o = 6 + 2 * cnl + 4 * k;
        xf.op[k] = FcXop{key[o], key[o + 1], key[o + 2], key[o + 3]};
      }
      P.xfs.push_back(xf);
      P.any_xf |= nx > 0;
      q.h.c01 = (uint64_t)cc[0] | ((uint64_t)cc[1] << 32);
      q.h.f01 = (uint64_t)ff[0] | ((uint64_t)ff[1] << 32);
      for (int l = 0; l < 6; l++) {
        q.t.c[l] = cc[2 + l];
        q.t.f[l] = ff[2 + l];
      }
      P.atoms.push_back(q);
    }
    sg.n_groups = (int)P.groups.size() - sg.group_off;
    P.stage_masks.insert(P.stage_masks.end(), masks.begin(), masks.end());
    const uint32_t abase = 1u + (uint32_t)masks.size();
    // chunks of 64 tapes, entries k-major; short lists padded with entry 0 (all ones)
    for (size_t c0 = 0; c0 < tl.size(); c0 += 64) {
      size_t kmax = 0;
      for (size_t t = c0; t < std::min(tl.size(), c0 + 64); t++) kmax = std::max(kmax, tl[t].size());
      for (size_t k = 0; k < kmax; k++)
        for (size_t l = 0; l < 64; l++) {
          const size_t t = c0 + l;
          uint32_t e = 0;
          if (t < tl.size() && k < tl[t].size()) {
            const Ent& x = tl[t][k];
            e = (x.kind == 0 ? 1u + x.id : abase + pos[x.id]) | (x.neg ? 0x80000000u : 0u);
          }
          P.lists.push_back(e);
        }
      P.chunk_off.push_back((uint32_t)P.lists.size());
    }
    for (size_t t = 0; t < tl.size(); t++) {
      P.tape_out.push_back(out_of(tsrc[t]) | (negated[tsrc[t]] ? 0x80000000u : 0u));
      const auto no = nodes_ops(tsrc[t]);
      P.metric.push_back(no.first);
      P.metric.push_back(no.second);
      if (mask_out) P.col_mask.push_back(mask_out(tsrc[t]));
    }
    P.segs.push_back(sg);
    atom_of.clear();
    akeys.clear();
    mask_of.clear();
    masks.clear();
    tl.clear();
    tsrc.clear();
  };
  for (size_t i = 0; i < keep.size(); i++) {
    if (!keep[i]) continue;
    if (fq[i].size() > (size_t)kFcaMaxAtoms || fm[i].size() > (size_t)kFcStageMasks) {
      keep[i] = 0;
      continue;
    }
    // this tape's new atoms / masks; a new segment when they do not fit
    size_t new_a = 0, new_m = 0;
    {
      std::set<std::vector<uint32_t>> fa;
      std::set<uint32_t> fmk;
      for (const auto& h : fq[i]) {
        bool ng;
        auto key = atom_key(h, &ng);
        if (!atom_of.count(key)) fa.insert(key);
      }
      for (uint32_t e : fm[i])
        if (!mask_of.count(e & 0x7FFFFFFFu)) fmk.insert(e & 0x7FFFFFFFu);
      new_a = fa.size();
      new_m = fmk.size();
    }
    if (akeys.size() + new_a > (size_t)kFcaMaxAtoms || masks.size() + new_m > (size_t)kFcStageMasks) close();
    std::vector<Ent> ent;
    for (uint32_t e : fm[i]) {
      const uint32_t v = e & 0x7FFFFFFFu;
      auto it = mask_of.find(v);
      uint32_t id;
      if (it == mask_of.end()) {
        id = (uint32_t)masks.size();
        mask_of[v] = id;
        masks.push_back(v);
      } else {
        id = it->second;
      }
      ent.push_back(Ent{0, id, e >> 31});
    }
    for (const auto& h : fq[i]) {
      bool ng;
      auto key = atom_key(h, &ng);
      auto it = atom_of.find(key);
      uint32_t id;
      if (it == atom_of.end()) {
        id = (uint32_t)akeys.size();
        atom_of[key] = id;
        akeys.push_back(key);
      } else {
        id = it->second;
      }
      ent.push_back(Ent{1, id, ng ? 1u : 0u});
    }
    tl.push_back(std::move(ent));
    tsrc.push_back(i);
  }
  close();
}

static int qsa_prepare(mq_ctx* c, mq_tapes* T, bool latency) {
  if (T->qsa_gen == c->layout_gen) return MQ_OK;
  T->qsa_gen = c->layout_gen;
  T->qsa_live = false;
  std::vector<uint32_t> words[2], tr, extra;
  std::vector<GDesc> ds[2];
  int temps[2] = {0, 0};
  // pass 1: tapes the P kernel takes; the others go to G, which preloads the (at most 8)
  // variables of at most 256 bits those tapes push most often
  const int64_t nq = (int64_t)T->qct.size();
  std::vector<char> on_p(nq, 0);
  std::unique_ptr<PhaseTimer> pt(new PhaseTimer(&c->host_t[3]));
  // flat conjunctions first: they run on fc_kernel (no interpreter); MQ_NO_FLAT=1 keeps them on P / G
  const bool no_flat = std::getenv("MQ_NO_FLAT") != nullptr;
  std::vector<char> on_fc(nq, 0);
  std::vector<std::vector<uint32_t>> fc_m(nq);
  std::vector<std::vector<FcCmpH>> fc_q(nq);
  std::vector<char> fc_neg(nq, 0);
  T->fca = std::getenv("MQ_FC_ONEPHASE") == nullptr;
  // unary atoms (fca only) are opt-in, MQ_FC_UNARY=1: they move C3's tapes off G (all 1 000 are
  // flat with them) but measured slower there — C3 18.6 -> 40.9 ms, C5 49 -> 69 ms (profiles/r06c):
  // C3's 8 854 compares are 8 442 distinct atoms, so the flat kernel's phase 1 does the tapes' work
  // with no sharing to win, for every tile, while G's per-tape cost is no higher per atom
  const bool unary = T->fca && std::getenv("MQ_FC_UNARY") != nullptr;
  if (!no_flat)
    parallel_for(nq, 32, [&](int, int64_t b, int64_t e) {
      for (int64_t i = b; i < e; i++) {
        bool ng = false;
        on_fc[i] = fc_match(c, T->qct[i], fc_m[i], fc_q[i], &ng, unary) ? 1 : 0;
        fc_neg[i] = ng ? 1 : 0;
      }
    });
  FcPlan fcp;
  FcaPlan fap;
  if (T->fca)
    fca_plan(c, fc_m, fc_q, fc_neg, on_fc, [&](size_t i) { return T->qbase[i].tape; },
             [&](size_t i) { return std::make_pair(T->qbase[i].n_nodes, T->qbase[i].alg_ops); }, fap);
  else
    fc_plan(c, fc_m, fc_q, fc_neg, on_fc, [&](size_t i) { return T->qbase[i].tape; }, [](size_t) { return (int32_t)-1; },
            [&](size_t i) { return std::make_pair(T->qbase[i].n_nodes, T->qbase[i].alg_ops); }, fcp);
  // (P preloads variables 0-7 only: a program pushing any other variable is not tried on P)
  auto p_candidate = [](const CompiledTape& x) {
    for (size_t pc = 0; pc < x.prog.size(); pc++) {
      const uint32_t op = x.prog[pc] & 0xFFu;
      if ((op == G_PUSH_VAR || op == G_PUSH_VAR_B) && (x.prog[pc] >> 12) >= (uint32_t)kQsaVars) return false;
      if (has_imm2(op)) pc++;
    }
    return true;
  };
  // (a latency-bound launch runs everything on G, one tape per wave: no P attempt.  Chunks of
  // 32 tapes: a drop-in batch of a few conjunct tapes is translated on the calling thread, which
  // is cheaper than waking the pool)
  if (!latency)
    parallel_for(nq, 32, [&](int, int64_t b, int64_t e) {
      for (int64_t i = b; i < e; i++)
        on_p[i] = !on_fc[i] && p_candidate(T->qct[i]) && qsa_translate(c, 0, true, T->qct[i], nullptr, nullptr) ? 1 : 0;
    });
  std::vector<int64_t> pushes(c->var_nl_h.size(), 0);
  for (size_t i = 0; i < T->qct.size(); i++) {
    if (on_p[i] || on_fc[i]) continue;
    const auto& pr = T->qct[i].prog;
    for (size_t pc = 0; pc < pr.size(); pc++) {
      const uint32_t op = pr[pc] & 0xFFu, imm = pr[pc] >> 12;
      // (Bool variables with a lane mask are neither preloaded nor staged: PUSH_PKB)
      if ((op == G_PUSH_VAR || (op == G_PUSH_VAR_B && !(imm < c->bmask_of_var.size() && c->bmask_of_var[imm] >= 0))) &&
          imm < pushes.size() && c->var_nl_h[imm] <= 8)
        pushes[imm]++;
      if (has_imm2(op)) pc++;
    }
  }
  std::vector<int> order;
  for (size_t v = 0; v < pushes.size(); v++)
    if (pushes[v] > 0) order.push_back((int)v);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pushes[a] > pushes[b]; });
  if (order.size() > (size_t)kQsaVarsG) order.resize(kQsaVarsG);
  T->gpre.assign(c->var_nl_h.size(), -1);
  const uint32_t zero_row = (uint32_t)(c->var_off_h.empty() ? 0 : c->var_off_h.back() + c->var_nl_h.back());
  for (int j = 0; j < 64; j++) T->g_var_row[j] = zero_row;
  for (size_t j = 0; j < order.size(); j++) {
    const int v = order[j];
    T->gpre[v] = (int)j;
    for (uint32_t l = 0; l < c->var_nl_h[v]; l++) T->g_var_row[8 * j + l] = c->var_off_h[v] + l;
  }
  int g_temps = 0;
  for (size_t i = 0; i < T->qct.size(); i++)
    if (!on_p[i] && !on_fc[i]) g_temps = std::max(g_temps, qsa_temps(T->qct[i], 1));
  int64_t n_g = 0;
  for (size_t i = 0; i < T->qct.size(); i++) n_g += (on_p[i] || on_fc[i]) ? 0 : 1;
  const double g_share = n_g ? std::min(1.0, 4.0 * (double)g_tapes_per_group(n_g, c->M) / (double)n_g) : 1.0;
  plan_stage(c, pushes, &T->gpre, g_temps, g_share, T->gstage, T->stage_rows);
  T->qhist[0].assign(QK_COUNT, 0);
  T->qhist[1].assign(QK_COUNT, 0);
  T->qpairs.assign((size_t)QK_COUNT * QK_COUNT, 0);
  T->qpairs_p.assign((size_t)QK_COUNT * QK_COUNT, 0);
  // per-tape translations in parallel (independent; ~50 ns per node), then concatenated in order
  pt.reset(new PhaseTimer(&c->host_t[4]));
  std::vector<std::vector<uint32_t>> trs(nq);
  std::vector<char> kind_of(nq, 0);
  std::atomic<bool> g_fail{false};
  parallel_for(nq, 32, [&](int, int64_t b, int64_t e) {
    std::vector<uint32_t> ex;
    for (int64_t i = b; i < e && !g_fail.load(std::memory_order_relaxed); i++) {
      if (on_fc[i]) {
        kind_of[i] = 2;
        continue;
      }
      if (on_p[i] && qsa_translate(c, 0, true, T->qct[i], &trs[i], &ex)) continue;
      kind_of[i] = 1;
      if (!qsa_translate(c, 1, true, T->qct[i], &trs[i], &ex, &T->gpre, &T->gstage)) {
        g_fail = true;
        break;
      }
      qsa_window_layout(c, trs[i]);
    }
  });
  if (g_fail) return MQ_OK;
  for (int64_t i = 0; i < nq; i++) {
    const int k = kind_of[i];
    if (k == 2) continue;
    const std::vector<uint32_t>& t = trs[i];
    qsa_count(c, k, t, T->qhist[k], k == 1 ? &T->qpairs : &T->qpairs_p);
    GDesc d = T->qbase[i];
    d.prog_off = (uint32_t)words[k].size();
    d.prog_len = (uint32_t)t.size();
    words[k].insert(words[k].end(), t.begin(), t.end());
    ds[k].push_back(d);
    temps[k] = std::max(temps[k], qsa_temps(T->qct[i], k));
  }
  // [P programs | END END | G programs | END END]: the dispatch tail prefetches one word past
  // each program's END
  pt.reset(new PhaseTimer(&c->host_t[5]));
  std::vector<uint32_t> prog;
  std::vector<GDesc> descs;
  for (int k = 0; k < 2; k++) {
    // G's program windows are the buffer's aligned 64-word blocks (gen_qsa.py load_window rounds
    // a program's address down to its block): G's programs start at a block boundary
    if (k == 1) prog.resize((prog.size() + 63) / 64 * 64, 0);
    const uint32_t base = (uint32_t)prog.size();
    for (GDesc d : ds[k]) {
      d.prog_off += base;
      descs.push_back(d);
    }
    prog.insert(prog.end(), words[k].begin(), words[k].end());
    const uint32_t endo = c->qsa_off[k][c->qsa_index[k][QK_END][0][0]];
    const uint32_t endw = hword(1, endo);
    if (k == 0) {   // P entries are (handler address, imm, prefetch); the x4 entry load reads one more word
      for (int r = 0; r < 2; r++) {
        prog.push_back(c->qsa_hbase_lo[0] + endo);
        prog.push_back(0);
        prog.push_back(0);
      }
      prog.push_back(0);
    } else {
      prog.push_back(endw);
      prog.push_back(endw);
    }
    // G's window loads read up to 63 words past a program's last word
    if (k == 1) prog.insert(prog.end(), 128, endw);   // window + next-window prefetch past the last END
    T->q_count[k] = (int)ds[k].size();
    T->q_temps[k] = temps[k];
  }
  if (descs.empty()) descs.push_back(GDesc{});
  UploadPack pk;
  pk.add(T->qdescs, descs.data(), descs.size());
  pk.add(T->qprog, prog.data(), prog.size());
  if (T->fca) {
    T->fc_count = (int)fap.tape_out.size();
    T->fca_atoms = (int)fap.atoms.size();
    T->fca_segs = fap.segs;
    T->fca_any_xf = fap.any_xf;
    if (T->fc_count > 0) {
      if (fap.stage_masks.empty()) fap.stage_masks.push_back(0);
      if (fap.atoms.empty()) fap.atoms.push_back(FcCmp{});
      if (fap.xfs.empty()) fap.xfs.push_back(FcXf{});
      if (fap.groups.empty()) fap.groups.push_back(FcaGroup{});
      if (fap.lists.empty()) fap.lists.push_back(0);
      pk.add(T->fc_cmp_dev, fap.atoms.data(), fap.atoms.size());
      pk.add(T->fca_xf_dev, fap.xfs.data(), fap.xfs.size());
      pk.add(T->fca_group_dev, fap.groups.data(), fap.groups.size());
      pk.add(T->fc_mask_dev, fap.lists.data(), fap.lists.size());
      pk.add(T->fca_chunk_dev, fap.chunk_off.data(), fap.chunk_off.size());
      pk.add(T->fca_out_dev, fap.tape_out.data(), fap.tape_out.size());
      pk.add(T->fca_metric_dev, fap.metric.data(), fap.metric.size());
      pk.add(T->fc_smask_dev, fap.stage_masks.data(), fap.stage_masks.size());
    }
  } else {
    T->fc_count = (int)fcp.tapes.size();
    T->fc_stage_n = (int)fcp.stage_rows.size();
    T->fc_smask_n = (int)fcp.stage_masks.size();
  }
  if (!T->fca && !fcp.tapes.empty()) {
    if (fcp.stage_rows.empty()) fcp.stage_rows.push_back(0);
    if (fcp.stage_masks.empty()) fcp.stage_masks.push_back(0);
    if (fcp.mask_lds.empty()) fcp.mask_lds.push_back(0);
    if (fcp.cmps.empty()) fcp.cmps.push_back(FcCmp{});
    pk.add(T->fc_tapes_dev, fcp.tapes.data(), fcp.tapes.size());
    pk.add(T->fc_mask_dev, fcp.mask_lds.data(), fcp.mask_lds.size());
    pk.add(T->fc_cmp_dev, fcp.cmps.data(), fcp.cmps.size());
    pk.add(T->fc_stage_dev, fcp.stage_rows.data(), fcp.stage_rows.size());
    pk.add(T->fc_smask_dev, fcp.stage_masks.data(), fcp.stage_masks.size());
    pk.add(T->fc_prefix_dev, fcp.prefix.data(), fcp.prefix.size());
  }
  {
    const uint32_t zero = 0;
    if (T->stage_rows.empty()) pk.add(T->stage_dev, &zero, 1);
    else pk.add(T->stage_dev, T->stage_rows.data(), T->stage_rows.size());
  }
  // (translated programs, descriptors, flat-kernel tables and staging rows: one copy)
  HIPCHK(pk.commit(T->pack1, c->stream, c->stage));
  T->qargs_valid[0] = T->qargs_valid[1] = false;
  T->qsa_live = true;
  return MQ_OK;
}

// Latency weight of a G program on one tile: its ops, plus the round trips of its variable
// pushes and table lookups (a store chain's select ends in a lookup; these dominate a column level)
static double g_cost(const CompiledTape& x) {
  double w = 0;
  for (size_t pc = 0; pc < x.prog.size(); pc++) {
    const uint32_t op = x.prog[pc] & 0xFFu;
    w += 1;
    if (op == G_PUSH_VAR || op == G_PUSH_VAR_B) w += 4;
    if (op == G_UF1 || op == G_UF2 || op == G_UFK0 || op == G_UFK || op == G_UFKV) w += 24;
    if (has_imm2(op)) pc++;
  }
  return w;
}

// Split a column level's G programs into groups (a group = one wave of G on one tile; group g
// = descriptors [tab[g], tab[g+1]), the table gen_qsa.py's mode-3 prologue reads) so the
// heaviest group is as light as it can be: longest processing time first over
// min(n, ceil(n / tpg) rounded up to the workgroup's 4 waves) groups, of any sizes.  A workgroup
// holds its LDS until its slowest wave ends, so a level's time follows its heaviest group (C4
// level 2, five store chains: three in one wave of three 0.69 ms; 2-2-1 0.50 ms).  Reorders idx
// group by group; tab gets groups rounded up to 4, + 1 entries (empty groups past the last).
static void balance_groups(const std::vector<CompiledTape>& ct, std::vector<int>& idx, int tpg,
                           std::vector<uint32_t>& tab) {
  const int n = (int)idx.size();
  const int groups = std::max(1, std::min(n, ((n + tpg - 1) / tpg + 3) / 4 * 4));
  std::vector<std::pair<double, int>> w;
  for (int i : idx) w.push_back({g_cost(ct[i]), i});
  std::stable_sort(w.begin(), w.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  std::vector<double> load(groups, 0);
  std::vector<std::vector<int>> members(groups);
  for (const auto& x : w) {
    int best = 0;
    for (int g = 1; g < groups; g++)
      if (load[g] < load[best]) best = g;
    members[best].push_back(x.second);
    load[best] += x.first;
  }
  idx.clear();
  tab.assign(1, 0);
  for (const auto& m : members) {
    idx.insert(idx.end(), m.begin(), m.end());
    tab.push_back((uint32_t)idx.size());
  }
  while ((tab.size() - 1) % 4) tab.push_back((uint32_t)n);
}

// Translate the G-eligible column programs for the current model batch (variable rows): one
// program segment and descriptor list, levels contiguous.  GDesc for mode 3: tape = first row
// of the target variable, n_temps = its limbs, depth = Bool root (gen_qsa.py store_column).
// If one column does not translate, all columns run on the HIP C++ column kernel.
static int cq_prepare(mq_ctx* c, mq_tapes* T) {
  if (T->cq_gen == c->layout_gen) return MQ_OK;
  T->cq_gen = c->layout_gen;
  T->cq_live = false;
  if (T->cq_ct.empty()) return MQ_OK;
  std::vector<uint32_t> prog, consts, tr, extra;
  std::vector<GDesc> descs;
  // column programs packed back to back (qsa_pack_program; MQ_G_COL_BLOCKS=1: each padded to
  // whole blocks, as tape programs are)
  const bool pack_block = std::getenv("MQ_G_COL_BLOCKS") != nullptr;
  size_t pack_pos = 0;
  // one LDS staging plan per column level: a level's launch stages only the rows its own
  // programs push (one plan for all levels made every level stage every level's rows)
  T->cq_stage_rows.clear();
  T->cq_lvl_stage_off.assign(T->clevels.size(), 0);
  T->cq_lvl_stage_n.assign(T->clevels.size(), 0);
  T->cq_lvl_temps.assign(T->clevels.size(), 0);
  T->cq_lvl_desc_off.assign(T->clevels.size(), 0);
  T->cq_lvl_desc_n.assign(T->clevels.size(), 0);
  T->cq_lvl_tab_off.assign(T->clevels.size(), 0);
  T->cq_lvl_groups.assign(T->clevels.size(), 0);
  T->cq_group_tab.clear();
  T->fc_lvl.clear();
  T->fc_lvl.resize(T->clevels.size());
  const bool no_flat = std::getenv("MQ_NO_FLAT") != nullptr;
  for (size_t li = 0; li < T->clevels.size(); li++) {
    T->fc_lvl[li].reset(new mq_tapes::FcLevel());
    T->cq_lvl_desc_off[li] = (int)descs.size();
    const int b = T->clevels[li].cq_begin, n0 = T->clevels[li].v8q;
    if (n0 <= 0) continue;
    // the level's flat Bool columns (fc_kernel, mode 3)
    std::vector<char> on_fc(n0, 0), fneg(n0, 0);
    std::vector<std::vector<uint32_t>> fm(n0);
    std::vector<std::vector<FcCmpH>> fq(n0);
    if (!no_flat)
      for (int i = 0; i < n0; i++) {
        bool ng = false;
        on_fc[i] = T->cq_bool[b + i] && fc_match(c, T->cq_ct[b + i], fm[i], fq[i], &ng) ? 1 : 0;
        fneg[i] = ng ? 1 : 0;
      }
    FcaPlan fap;
    fca_plan(c, fm, fq, fneg, on_fc, [&](size_t i) { return c->var_off_h[T->cq_var[b + i]]; },
             [&](size_t i) {
               const CompiledTape& x = T->cq_ct[b + i];
               return std::make_pair(x.n_nodes, (uint32_t)std::min(x.alg_ops, 4.0e9));
             },
             fap,
             [&](size_t i) {
               const int v = T->cq_var[b + i];
               return (int32_t)(v < (int)c->bmask_of_var.size() ? c->bmask_of_var[v] : -1);
             });
    mq_tapes::FcLevel& fl = *T->fc_lvl[li];
    fl.count = (int)fap.tape_out.size();
    fl.segs = fap.segs;
    fl.any_xf = fap.any_xf;
    if (fl.count > 0) {
      if (fap.stage_masks.empty()) fap.stage_masks.push_back(0);
      if (fap.atoms.empty()) fap.atoms.push_back(FcCmp{});
      if (fap.xfs.empty()) fap.xfs.push_back(FcXf{});
      if (fap.groups.empty()) fap.groups.push_back(FcaGroup{});
      if (fap.lists.empty()) fap.lists.push_back(0);
      HIPCHK(fl.atoms.upload(fap.atoms.data(), fap.atoms.size(), c->stream));
      HIPCHK(fl.xfs.upload(fap.xfs.data(), fap.xfs.size(), c->stream));
      HIPCHK(fl.groups.upload(fap.groups.data(), fap.groups.size(), c->stream));
      HIPCHK(fl.lists.upload(fap.lists.data(), fap.lists.size(), c->stream));
      HIPCHK(fl.chunk.upload(fap.chunk_off.data(), fap.chunk_off.size(), c->stream));
      HIPCHK(fl.out.upload(fap.tape_out.data(), fap.tape_out.size(), c->stream));
      HIPCHK(fl.metric.upload(fap.metric.data(), fap.metric.size(), c->stream));
      HIPCHK(fl.smask.upload(fap.stage_masks.data(), fap.stage_masks.size(), c->stream));
      HIPCHK(fl.colmask.upload(fap.col_mask.data(), fap.col_mask.size(), c->stream));
    }
    std::vector<int> rest;   // the level's columns left to G
    for (int i = 0; i < n0; i++)
      if (!on_fc[i]) rest.push_back(b + i);
    const int n = (int)rest.size();
    T->cq_lvl_desc_n[li] = n;
    if (n <= 0) continue;
    {
      std::vector<uint32_t> tab;
      balance_groups(T->cq_ct, rest, (int)std::max<int64_t>(1, std::min<int64_t>(cq_tapes_per_group(n, c->M), n)), tab);
      T->cq_lvl_tab_off[li] = (uint32_t)T->cq_group_tab.size();
      T->cq_lvl_groups[li] = (int)tab.size() - 1;
      T->cq_group_tab.insert(T->cq_group_tab.end(), tab.begin(), tab.end());
    }
    std::vector<CompiledTape> lvl;
    for (int i : rest) lvl.push_back(T->cq_ct[i]);
    int temps = 0;
    for (const CompiledTape& x : lvl) temps = std::max(temps, qsa_temps(x, 1));
    const double share = std::min(1.0, 4.0 * (double)cq_tapes_per_group(n, c->M) / (double)n);
    std::vector<int> gstage;
    std::vector<uint32_t> rows;
    plan_stage(c, count_pushes(c, lvl), nullptr, temps, share, gstage, rows);
    T->cq_lvl_stage_off[li] = (uint32_t)T->cq_stage_rows.size();
    T->cq_lvl_stage_n[li] = (uint32_t)rows.size();
    T->cq_lvl_temps[li] = temps;
    T->cq_stage_rows.insert(T->cq_stage_rows.end(), rows.begin(), rows.end());
    for (int i : rest) {
      const CompiledTape& x = T->cq_ct[i];
      if (!qsa_translate(c, 1, true, x, &tr, &extra, nullptr, &gstage)) return MQ_OK;
      qsa_count(c, 1, tr, T->qhist[2], nullptr);
      const int v = T->cq_var[i];
      GDesc d{};
      d.prog_len = (uint32_t)tr.size();
      d.prog_off = pack_block ? (qsa_window_layout(c, tr), (uint32_t)prog.size()) : qsa_pack_program(c, prog, pack_pos, tr);
      d.tape = c->var_off_h[v];
      d.const_base = (uint32_t)consts.size();
      d.n_nodes = x.n_nodes;
      d.n_temps = c->var_nl_h[v];
      // Bool root: bit 0, and the packed lane-mask index + 1 above it (store_column)
      d.depth = T->cq_bool[i] ? 1u | ((uint32_t)(v < (int)c->bmask_of_var.size() ? c->bmask_of_var[v] + 1 : 0) << 1) : 0u;
      d.alg_ops = (uint32_t)std::min(x.alg_ops, 4.0e9);
      if (pack_block) prog.insert(prog.end(), tr.begin(), tr.end());
      consts.insert(consts.end(), x.consts.begin(), x.consts.end());
      consts.insert(consts.end(), extra.begin(), extra.end());
      descs.push_back(d);
    }
  }
  const uint32_t endw = hword(1, c->qsa_off[1][c->qsa_index[1][QK_END][0][0]]);
  if (pack_pos) prog.insert(prog.end(), 64 - pack_pos, endw);   // (whole blocks)
  prog.insert(prog.end(), 130, endw);   // the window + next-window prefetch read up to 127 words past the last END
  consts.resize(consts.size() + 16, 0);
  HIPCHK(T->cqdescs.upload(descs.data(), descs.size(), c->stream));
  HIPCHK(T->cqprog.upload(prog.data(), prog.size(), c->stream));
  HIPCHK(T->cqconsts.upload(consts.data(), consts.size(), c->stream));
  HIPCHK(T->cqargs.ensure(sizeof(QArgs) * T->clevels.size()));
  if (T->cq_stage_rows.empty()) HIPCHK(T->cq_stage_dev.ensure(sizeof(uint32_t)));
  else HIPCHK(T->cq_stage_dev.upload(T->cq_stage_rows.data(), T->cq_stage_rows.size(), c->stream));
  if (T->cq_group_tab.empty()) T->cq_group_tab.assign(5, 0);
  HIPCHK(T->cq_group_dev.upload(T->cq_group_tab.data(), T->cq_group_tab.size(), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  T->cqargs_host.assign(T->clevels.size(), QArgs{});
  T->cq_live = true;
  return MQ_OK;
}

static mq_tapes::Variant cut_front(mq_tapes::Variant v, int n) {
  v.begin += n;
  v.count -= n;
  return v;
}

// G kernel tape-group size.  Each wave evaluates its group on the 64 models of its workgroup's
// tile; small groups put many waves on the same tile at once (model rows shared through L1/L2),
// large ones amortise the per-wave preload of the 8 most pushed variables.  The 4 waves of a
// workgroup take one group each, so a launch of n <= 64 programs (a column level, a small batch)
// is cut into 4 groups: min(n, 16) left 3 of 4 waves idle below 16 programs.  MQ_G_TPG overrides.
static int64_t g_tapes_per_group(int64_t n, int64_t M) {
  (void)M;
  if (const char* e = std::getenv("MQ_G_TPG")) {
    const long v = std::atol(e);
    if (v > 0) return v;
  }
  return std::max<int64_t>(1, std::min<int64_t>(16, (n + 3) / 4));
}

// programs per wave of a hoisted-column level launch (mode 3); MQ_CQ_TPG overrides
static int64_t cq_tapes_per_group(int64_t n, int64_t M) {
  if (const char* e = std::getenv("MQ_CQ_TPG")) {
    const long v = std::atol(e);
    if (v > 0) return v;
  }
  return g_tapes_per_group(n, M);
}

// Launch every evaluation kernel for a compiled batch: the assembly interpreter for the
// QSA-eligible tapes (when the model batch fits its register file), the HIP C++ kernels for
// the rest.  verdicts == nullptr -> first-hit mode into best.
// (MQ_LATENCY_ASM_NODES overrides; the translation runs on the host pool, ~50 ns per node per
// thread)
static int64_t latency_asm_nodes() {
  static const int64_t v = [] {
    if (const char* e = std::getenv("MQ_LATENCY_ASM_NODES")) return (int64_t)std::atoll(e);
    return (int64_t)131072;
  }();
  return v;
}

// Tapes with a wide-key lookup of a function that some model of the current batch holds more
// than kWideMaxEntries entries of are unsupported (-2) under that batch (mq.h MQ_OP_UF_WIDE).
static int refresh_wide_unsupported(mq_ctx* c, mq_tapes* T, hipStream_t st) {
  if (!T->wide_any || T->wide_gen == c->batch_gen) return MQ_OK;
  T->wide_gen = c->batch_gen;
  T->unsupported = T->unsupported_base;
  int n = 0;
  for (int t = 0; t < T->n_tapes; t++) {
    for (uint32_t f : T->wide_funcs[t])
      if (f < c->func_max_entries.size() && c->func_max_entries[f] > kWideMaxEntries) T->unsupported[t] = 1;
    n += T->unsupported[t];
  }
  T->n_unsupported = n;
  HIPCHK(T->unsup_dev.upload_staged(T->unsupported.data(), T->unsupported.size(), st, c->stage));
  return MQ_OK;
}

static int launch_all(mq_ctx* c, mq_tapes* T, int32_t* best, uint8_t* verdicts, hipStream_t st) {
  T->in_flight = true;   // (cleared where the host waits for the launch: mq_tapes_free skips its sync)
  if (const int rc = refresh_wide_unsupported(c, T, st)) return rc;
  bool use_qsa = c->qsa_ready && c->use_asm && T->qsa.count > 0;
  // latency-bound launch (a few tapes over a few models): G runs one tape per wave instead of
  // batching tapes per wave for throughput -- unless the batch is large enough that translating
  // it for P / G (host, ~50 ns per node) costs more than the C++ kernel's extra latency
  // (profiles/r02dv2: 256 EVM-shaped queries x 100 models, 13 ms of translation for 0.6 ms)
  const bool latency = (int64_t)T->n_tapes * ((c->M + 63) / 64) <= c->latency_waves;
  if (use_qsa && latency) {
    int64_t nodes = 0;
    for (int64_t n : T->n_nodes) nodes += n;
    if (nodes > latency_asm_nodes()) use_qsa = false;
  }
  if (use_qsa) {
    const int rc = qsa_prepare(c, T, latency);
    if (rc) return rc;
    use_qsa = T->qsa_live;
  }
  std::vector<mq_tapes::Variant> cpp(T->gen, T->gen + kGen);
  if (!use_qsa) cpp[0] = T->l8_all;
  hipEvent_t kend = nullptr;
  if (c->time_kernels) {
    if (c->kev_used == c->kev.size()) {
      std::pair<hipEvent_t, hipEvent_t> e{};
      HIPCHK(hipEventCreate(&e.first));
      HIPCHK(hipEventCreate(&e.second));
      c->kev.push_back(e);
    }
    auto& e = c->kev[c->kev_used++];
    kend = e.second;
  }
  // the start event is recorded right before the first evaluation kernel (after any argument
  // upload), the end event right after the last one
  bool started = false;
  auto start_timer = [&]() -> hipError_t {
    if (!kend || started) return hipSuccess;
    started = true;
    return hipEventRecord(c->kev[c->kev_used - 1].first, st);
  };
  if (c->M == 0) {   // an empty model shard: every tape keeps "no hit" (the caller's init)
    if (kend) {
      HIPCHK(start_timer());
      HIPCHK(hipEventRecord(kend, st));
    }
    return MQ_OK;
  }
  // hoisted columns first (they write model variable rows the tapes read)
  for (size_t i = 0; i < T->col_var.size(); i++) {
    const int v = T->col_var[i];
    if (v < 0 || v >= c->n_vars || nl_of(c->var_width[v]) != nl_of(T->col_width[i])) {
      g_last_error = "column target variable does not match the uploaded model batch";
      return MQ_ERR_ARG;
    }
  }
  bool use_cq = c->qsa_ready && c->use_asm && !T->cq_ct.empty();
  if (use_cq) {
    const int rc = cq_prepare(c, T);
    if (rc) return rc;
    use_cq = T->cq_live;
  } else {
    T->cq_live = false;   // (re-translated when the assembly path is enabled again)
    T->cq_gen = ~0ull;
  }
  if (st != c->stream) {
    // the batch's tables were copied on the context stream (tape upload, translations): a
    // launch on a caller's stream waits for them
    HIPCHK(hipEventRecord(c->stage_ev, c->stream));
    HIPCHK(hipStreamWaitEvent(st, c->stage_ev, 0));
  }
  const uint32_t zero_row = (uint32_t)(c->var_off_h.empty() ? 0 : c->var_off_h.back() + c->var_nl_h.back());
  if (T->bmask_gen != c->layout_gen) {
    // the mask indices of each level's Bool columns under this model batch
    T->lvl_bmask_h.assign(T->clevels.size(), {});
    T->lvl_bmask_cpp_h.assign(T->clevels.size(), {});
    std::vector<char> on_g(c->n_vars, 0);
    for (int v : T->cq_var)
      if (v >= 0 && v < c->n_vars) on_g[v] = 1;
    for (size_t i = 0; i < T->col_var.size(); i++) {
      const int v = T->col_var[i];
      if (T->col_width[i] == 0 && v < (int)c->bmask_of_var.size() && c->bmask_of_var[v] >= 0 &&
          T->col_level[i] < (int)T->clevels.size()) {
        const bool direct = i < T->col_direct_mask.size() && T->col_direct_mask[i];   // the keccak kernel stores it
        if (!direct) T->lvl_bmask_h[T->col_level[i]].push_back(c->bmask_of_var[v]);
        if (!on_g[v] && !direct) T->lvl_bmask_cpp_h[T->col_level[i]].push_back(c->bmask_of_var[v]);
      }
    }
    T->lvl_bmask.resize(T->clevels.size());
    T->lvl_bmask_cpp.resize(T->clevels.size());
    for (size_t li = 0; li < T->clevels.size(); li++) {
      if (!T->lvl_bmask_h[li].empty())
        HIPCHK(T->lvl_bmask[li].upload(T->lvl_bmask_h[li].data(), T->lvl_bmask_h[li].size(), st));
      if (!T->lvl_bmask_cpp_h[li].empty())
        HIPCHK(T->lvl_bmask_cpp[li].upload(T->lvl_bmask_cpp_h[li].data(), T->lvl_bmask_cpp_h[li].size(), st));
    }
    HIPCHK(hipStreamSynchronize(st));
    T->bmask_gen = c->layout_gen;
  }
  if (!T->kc.empty() && T->kc_gen != c->layout_gen) {
    // the keccak columns' message maps under this model batch's variable rows
    std::vector<KcCol> cols;
    std::vector<KcMapEntry> map;
    std::vector<KcPred> preds;
    for (const auto& h : T->kc) {
      if (h.target < 0 || h.target >= c->n_vars || c->var_nl_h[h.target] != 8) {
        g_last_error = "keccak column target is not a 256-bit variable of the uploaded model batch";
        return MQ_ERR_ARG;
      }
      KcCol kc{};
      kc.map_off = (uint32_t)map.size();
      kc.target_row = c->var_off_h[h.target];
      kc.n_nodes = h.n_nodes;
      kc.alg_ops = h.alg_ops;
      for (const auto& p : h.pieces) {
        if (p.var >= 0 && (p.var >= c->n_vars || c->var_nl_h[p.var] != p.nl)) {
          g_last_error = "keccak column piece does not match the uploaded model batch";
          return MQ_ERR_ARG;
        }
        for (int l = (int)p.nl - 1; l >= 0; l--)
          map.push_back(p.var >= 0 ? KcMapEntry{c->var_off_h[p.var] + (uint32_t)l, 0u}
                                   : KcMapEntry{~0u, T->kc_consts[p.coff + (uint32_t)l]});
      }
      kc.nwords = (uint32_t)map.size() - kc.map_off;
      kc.pred_off = (uint32_t)preds.size();
      for (const auto& ph : h.preds) {
        if (ph.target < 0 || ph.target >= c->n_vars || c->var_width[ph.target] != 0) {
          g_last_error = "keccak predicate column target is not a Bool variable of the uploaded model batch";
          return MQ_ERR_ARG;
        }
        KcPred kp{};
        kp.kind = ph.kind;
        kp.bits = ph.bits;
        kp.row = c->var_off_h[ph.target];
        kp.mask = ph.target < (int)c->bmask_of_var.size() ? c->bmask_of_var[ph.target] : -1;
        std::memcpy(kp.c, ph.c, sizeof(kp.c));
        preds.push_back(kp);
      }
      kc.n_pred = (uint32_t)h.preds.size();
      cols.push_back(kc);
    }
    HIPCHK(T->kc_cols_dev.upload(cols.data(), cols.size(), st));
    HIPCHK(T->kc_map_dev.upload(map.data(), map.size(), st));
    if (preds.empty()) HIPCHK(T->kc_pred_dev.ensure(sizeof(KcPred)));
    else HIPCHK(T->kc_pred_dev.upload(preds.data(), preds.size(), st));
    HIPCHK(hipStreamSynchronize(st));
    T->kc_gen = c->layout_gen;
  }
  if (!T->cw.empty() && T->cw_gen != c->layout_gen) {
    // the bit-gather columns' slots under this model batch's variable rows (a variable the batch
    // lacks, or a limb past its width, reads the zero row: VAR of an absent variable is 0)
    std::vector<CwCol> cols;
    std::vector<CwChunk> chunks;
    auto row_of = [&](int32_t v, uint32_t l) -> uint32_t {
      return (v >= 0 && v < c->n_vars && l < c->var_nl_h[v]) ? c->var_off_h[v] + l : zero_row;
    };
    for (const auto& h : T->cw) {
      const uint32_t nl = (uint32_t)h.limb_slots.size();
      if (h.target < 0 || h.target >= c->n_vars || c->var_nl_h[h.target] != nl) {
        g_last_error = "bit-gather column target does not match the uploaded model batch";
        return MQ_ERR_ARG;
      }
      if (h.size_var >= 0 && (h.size_var >= c->n_vars || c->var_nl_h[h.size_var] != 8)) {
        g_last_error = "bit-gather column size variable is not a 256-bit variable of the uploaded model batch";
        return MQ_ERR_ARG;
      }
      CwCol col{};
      col.chunk_off = (uint32_t)chunks.size();
      col.target_row = c->var_off_h[h.target];
      col.size_row = h.size_var >= 0 ? c->var_off_h[h.size_var] : ~0u;
      col.n_nodes = h.n_nodes;
      col.alg_ops = h.alg_ops;
      for (uint32_t l = 0; l < nl; l++) {
        const auto& sl = h.limb_slots[l];
        const size_t nch = std::max<size_t>(1, (sl.size() + 3) / 4);
        for (size_t q = 0; q < nch; q++) {
          CwChunk ch{};
          for (int j = 0; j < 4; j++) {
            const size_t i = 4 * q + j;
            ch.s[j] = i < sl.size() ? CwSlot{row_of(sl[i].var, sl[i].vlimb), sl[i].mask, sl[i].shifts, sl[i].gate}
                                    : CwSlot{zero_row, 0u, 0u, ~0u};
          }
          ch.limb = l;
          ch.store = q + 1 == nch ? 1u : 0u;
          ch.const_or = q == 0 ? h.const_or[l] : 0u;
          chunks.push_back(ch);
        }
      }
      col.n_chunks = (uint32_t)chunks.size() - col.chunk_off;
      cols.push_back(col);
    }
    HIPCHK(T->cw_cols_dev.upload(cols.data(), cols.size(), st));
    HIPCHK(T->cw_chunks_dev.upload(chunks.data(), chunks.size(), st));
    HIPCHK(hipStreamSynchronize(st));
    T->cw_gen = c->layout_gen;
  }
  // Bool columns' 0/1 rows are read only by the HIP C++ kernels (the assembly interpreters read
  // the packed lane masks, which G's column store writes itself): G writes the rows only when a
  // C++ tape or column kernel, or P (rows of preloaded variables), runs in this launch
  bool bool_rows = !use_qsa || T->q_count[0] > 0;
  for (int g = 0; g < kGen && !bool_rows; g++) bool_rows = cpp[g].count > 0;
  for (size_t li = 0; li < T->clevels.size() && !bool_rows; li++) {
    const auto& lv = T->clevels[li];
    for (int g = 0; g < kGen && !bool_rows; g++)
      bool_rows = (g == 0 ? (use_cq ? lv.v[0].count - lv.v8q : lv.v[0].count) : lv.v[g].count) > 0;
  }
  // MQ_NO_LEVEL_STREAMS=1: every kernel of a level on the launch stream, one after another
  static const bool level_streams = std::getenv("MQ_NO_LEVEL_STREAMS") == nullptr;
  for (size_t li = 0; li < T->clevels.size(); li++) {
    const auto& lv = T->clevels[li];
    // the level's kernels that run beside the interpreters: keccak columns on aux[0], bit-gather
    // and flat columns on aux[1], each stream waiting for the level's start on the launch stream
    // and the launch stream for them before the next level
    const bool has_kc = li < T->kc_level.size() && T->kc_level[li].second > 0;
    const bool has_cw = li < T->cw_level.size() && T->cw_level[li].second > 0;
    const bool has_fc = use_cq && li < T->fc_lvl.size() && T->fc_lvl[li] && T->fc_lvl[li]->count > 0;
    const bool fork = level_streams && (has_kc || has_cw || has_fc);
    hipStream_t s_kc = st, s_cf = st;
    if (fork) {
      HIPCHK(start_timer());
      HIPCHK(hipEventRecord(c->fork_ev, st));
      if (has_kc) {
        s_kc = c->aux[0];
        HIPCHK(hipStreamWaitEvent(s_kc, c->fork_ev, 0));
      }
      if (has_cw || has_fc) {
        s_cf = c->aux[1];
        HIPCHK(hipStreamWaitEvent(s_cf, c->fork_ev, 0));
      }
    }
    if (has_kc) {
      HIPCHK(start_timer());
      HIPCHK(launch_keccak_columns(T->kc_cols_dev.as<KcCol>() + T->kc_level[li].first, T->kc_level[li].second,
                                   T->kc_map_dev.as<KcMapEntry>(), T->kc_pred_dev.as<KcPred>(),
                                   const_cast<uint32_t*>(c->vars.as<uint32_t>()), c->M,
                                   c->counters.as<unsigned long long>(), c->bmasks.as<uint64_t>(), c->n_bmask,
                                   bool_rows ? 1 : 0, s_kc));
    }
    if (has_cw) {
      HIPCHK(start_timer());
      HIPCHK(launch_cw_columns(T->cw_cols_dev.as<CwCol>() + T->cw_level[li].first, T->cw_level[li].second,
                               T->cw_chunks_dev.as<CwChunk>(), const_cast<uint32_t*>(c->vars.as<uint32_t>()), c->M,
                               c->counters.as<unsigned long long>(), s_cf));
    }
    const mq_tapes::Variant v8 = use_cq ? cut_front(lv.v[0], lv.v8q) : lv.v[0];
    if (has_fc) {
      // the level's flat Bool columns on fca_kernel, mode 3
      const mq_tapes::FcLevel& fl = *T->fc_lvl[li];
      for (const FcaPlanSeg& sg : fl.segs) {
        FcaArgs f{};
        f.n = sg.n_tapes;
        f.n_atoms = sg.n_atoms;
        f.n_groups = sg.n_groups;
        f.groups = fl.groups.as<FcaGroup>() + sg.group_off;
        f.atoms = fl.atoms.as<FcCmp>() + sg.atom_off;
        f.xfs = fl.any_xf ? fl.xfs.as<FcXf>() + sg.atom_off : nullptr;
        f.lists = fl.lists.as<uint32_t>();
        f.chunk_off = fl.chunk.as<uint32_t>() + sg.chunk_first;
        f.tape_out = fl.out.as<uint32_t>() + sg.tape_first;
        f.tape_metric = fl.metric.as<uint32_t>() + 2 * (size_t)sg.tape_first;
        f.col_mask = fl.colmask.as<int32_t>() + sg.tape_first;
        f.vars = c->vars.as<uint32_t>();
        f.bool_masks = c->bmasks.as<uint64_t>();
        f.bool_masks_out = c->bmasks.as<uint64_t>();
        f.vars_out = const_cast<uint32_t*>(c->vars.as<uint32_t>());
        f.n_bool_masks = c->n_bmask;
        f.bool_rows = bool_rows ? 1 : 0;
        f.mode = 3;
        f.M = c->M;
        f.index_base = c->index_base;
        f.counters = c->counters.as<unsigned long long>();
        f.stage_masks = fl.smask.as<uint32_t>() + sg.smask_off;
        f.n_smask = sg.n_smask;
        HIPCHK(start_timer());
        HIPCHK(launch_fca(f, s_cf));
      }
    }
    const int n_gcol = use_cq && li < T->cq_lvl_desc_n.size() ? T->cq_lvl_desc_n[li] : 0;
    if (n_gcol > 0) {
      // the level's G columns on qsg_kernel, mode 3 (no preloaded variables)
      const int n = n_gcol;
      const int64_t tpg = std::max<int64_t>(1, std::min<int64_t>(cq_tapes_per_group(n, c->M), n));
      QArgs q{};
      q.descs = T->cqdescs.as<GDesc>() + T->cq_lvl_desc_off[li];
      q.prog = T->cqprog.p;
      q.consts = T->cqconsts.p;
      q.vars = c->vars.p;
      q.best = best;
      q.counters = c->counters.as<unsigned long long>();
      q.verdicts = nullptr;
      q.M = (uint32_t)c->M;
      q.index_base = (uint32_t)c->index_base;
      q.n_desc = (uint32_t)n;
      q.tapes_per_group = (uint32_t)tpg;
      q.early_exit = 0;
      q.mode = 3;
      q.table_out = T->cq_group_dev.as<uint32_t>() + T->cq_lvl_tab_off[li];   // the level's group bounds
      q.bool_rows = bool_rows ? 1u : 0u;
      q.lds_wave_bytes = (uint32_t)T->cq_lvl_temps[li] * 2048u;
      q.n_stage = T->cq_lvl_stage_n[li];
      q.stage_base = 4u * q.lds_wave_bytes;
      q.stage_rows = T->cq_stage_dev.as<uint32_t>() + T->cq_lvl_stage_off[li];
      for (int j = 0; j < 64; j++) q.var_row[j] = zero_row;
      q.funcs = c->funcs.p;
      q.entry_ptr = c->entry_ptr.p;
      q.entry_words = c->entry_words.p;
      q.else_words = c->else_words.p;
      q.n_funcs = (uint32_t)c->n_funcs;
      q.dense_words = c->dense_words.as<uint32_t>();
      q.bool_masks = c->bmasks.as<uint64_t>();
      q.n_bool_masks = (uint32_t)c->n_bmask;
      q.prof_out = prof_buffer(c, (int)li);
      const size_t lds_other = (size_t)q.lds_wave_bytes * 4 + (size_t)q.n_stage * 256 + 4 * (size_t)kQsaProfBytes;
      const size_t lds = lds_other;
      QArgs* dq = T->cqargs.as<QArgs>() + li;
      if (std::memcmp(&T->cqargs_host[li], &q, sizeof(QArgs)) != 0) {
        PhaseTimer pq(&c->host_t[6]);
        void* h = c->stage.put(&q, sizeof(QArgs), st);   // (q is on the stack: staged)
        if (!h) return MQ_ERR_NOMEM;
        HIPCHK(hipMemcpyAsync(dq, h, sizeof(QArgs), hipMemcpyHostToDevice, st));
        T->cqargs_host[li] = q;
      }
      const int64_t groups = T->cq_lvl_groups[li];
      const int64_t rows = ((c->M + 63) / 64 + 7) / 8;
      if (rows > 65535) {
        g_last_error = "G kernel: more than 33.5M models in one launch (grid.y limit); shard the model axis";
        return MQ_ERR_ARG;
      }
      HIPCHK(start_timer());
      HIPCHK(launch_qsa(1, dq, 8u * (unsigned)((groups + 3) / 4), (unsigned)rows, lds, st));
    }
    for (int g = 0; g < kGen; g++) {
      const mq_tapes::Variant* v = g == 0 ? &v8 : &lv.v[g];
      if (v->count <= 0) continue;
      KArgs a = make_col_args(c, T, *v);
      const size_t scratch_bytes = (size_t)a.grid * (size_t)a.tmp_words_per_wave * 4;
      if (scratch_bytes) {
        HIPCHK(c->scratch.ensure(scratch_bytes));
        a.scratch = c->scratch.as<uint32_t>();
      }
      HIPCHK(start_timer());
      HIPCHK(launch_columns(a, v->L, v->keccak, st));
    }
    // the level's Bool columns as lane masks, for the levels and tapes after it (those G
    // computed are stored as masks already)
    const auto& pk_h = use_cq ? T->lvl_bmask_cpp_h[li] : T->lvl_bmask_h[li];
    if (!pk_h.empty()) {
      HIPCHK(start_timer());
      HIPCHK(launch_pack_bool(c->vars.as<uint32_t>(), c->bmasks.as<uint64_t>(), c->bmask_rows.as<uint32_t>(),
                              (use_cq ? T->lvl_bmask_cpp[li] : T->lvl_bmask[li]).as<int32_t>(), (int)pk_h.size(),
                              c->n_bmask, c->M, st));
    }
    if (fork) {   // join: the next level (or the tapes) reads this level's columns
      if (s_kc != st) {
        HIPCHK(hipEventRecord(c->join_ev[0], s_kc));
        HIPCHK(hipStreamWaitEvent(st, c->join_ev[0], 0));
      }
      if (s_cf != st) {
        HIPCHK(hipEventRecord(c->join_ev[1], s_cf));
        HIPCHK(hipStreamWaitEvent(st, c->join_ev[1], 0));
      }
    }
  }
  for (int k = 0; use_qsa && k < 2; k++) {
    const int n = T->q_count[k];
    if (n <= 0) continue;
    // P: grid = (256-model tiles) x (tape groups), groups sized for ~32k workgroups (C2: 120
    //    tapes a group; 8k / 16k / 24k / 32k / 64k: 23.75 / 23.15 / 22.88 / 22.87 / 22.87 ms,
    //    profiles/r05bf, r05bg — finer groups shorten the last wave of workgroups; the model rows
    //    are re-read once per group, ~2 GB per launch, far from the HBM bound of a VALU-bound kernel)
    // G: 64-model tiles, 4 tape groups per workgroup (one per wave), XCD-interleaved grid
    //    (qsa.hip); groups of g_tapes_per_group() tapes.
    const int64_t tiles256 = (c->M + 255) / 256;
    int64_t p_wg = 32768;   // P: target workgroup count (MQ_P_WG overrides)
    if (const char* e = std::getenv("MQ_P_WG")) p_wg = std::max(256L, std::atol(e));
    int64_t tpg = k == 0 ? (int64_t(n) * tiles256 + p_wg - 1) / p_wg : latency ? 1 : g_tapes_per_group(n, c->M);
    tpg = std::max<int64_t>(1, std::min<int64_t>(tpg, n));
    QArgs q{};
    q.descs = T->qdescs.as<GDesc>() + (k == 0 ? 0 : T->q_count[0]);
    q.prog = T->qprog.p;
    q.consts = T->consts.p;
    q.vars = c->vars.p;
    q.best = best;
    q.counters = c->counters.as<unsigned long long>();
    q.verdicts = verdicts;
    q.M = (uint32_t)c->M;
    q.index_base = (uint32_t)c->index_base;
    q.n_desc = (uint32_t)n;
    q.tapes_per_group = (uint32_t)tpg;
    q.early_exit = verdicts ? 0u : (uint32_t)c->early_exit;
    q.mode = verdicts ? 1u : 0u;
    q.lds_wave_bytes = (uint32_t)T->q_temps[k] * 2048u;
    if (k == 1) {
      q.n_stage = (uint32_t)T->stage_rows.size();
      q.stage_base = 4u * q.lds_wave_bytes;
      q.stage_rows = T->stage_dev.as<uint32_t>();
    }
    std::memcpy(q.var_row, k == 0 ? c->qsa_var_row : T->g_var_row, sizeof(q.var_row));
    q.funcs = c->funcs.p;
    q.entry_ptr = c->entry_ptr.p;
    q.entry_words = c->entry_words.p;
    q.else_words = c->else_words.p;
    q.n_funcs = (uint32_t)c->n_funcs;
    q.dense_words = c->dense_words.as<uint32_t>();
    q.bool_masks = c->bmasks.as<uint64_t>();
    q.n_bool_masks = (uint32_t)c->n_bmask;
    if (k == 1) q.prof_out = prof_buffer(c, -1);
    size_t lds = (size_t)q.lds_wave_bytes * 4 + (size_t)q.n_stage * 256 + (k == 1 ? 4 * (size_t)kQsaProfBytes : 0);
    // the argument block only changes with the output buffer / mode / models: re-upload then
    if (!T->qargs_valid[k] || std::memcmp(&T->qargs_dev_copy[k], &q, sizeof(QArgs)) != 0) {
      PhaseTimer pq(&c->host_t[6]);
      void* h = c->stage.put(&q, sizeof(QArgs), st);   // (q is on the stack: staged)
      if (!h) return MQ_ERR_NOMEM;
      HIPCHK(hipMemcpyAsync(T->qargs[k].p, h, sizeof(QArgs), hipMemcpyHostToDevice, st));
      T->qargs_dev_copy[k] = q;
      T->qargs_valid[k] = true;
    }
    // P: tiles fastest, so the workgroups running together share a tape group's program and
    // constants in the scalar caches (the XCD-interleaved order G uses measured 22.8 -> 26.4 ms
    // on C2, profiles/r05bi: P's program reads are scalar, its model rows preloaded once)
    unsigned gx = (unsigned)tiles256;
    unsigned gy = (unsigned)((n + tpg - 1) / tpg);
    if (k == 1) {
      const int64_t groups = (n + tpg - 1) / tpg;
      gx = 8u * (unsigned)((groups + 3) / 4);          // xcd + 8 * (workgroup's group quad)
      gy = (unsigned)(((c->M + 63) / 64 + 7) / 8);     // tiles of 64 models, 8 per row
      if (((c->M + 63) / 64 + 7) / 8 > 65535) {
        g_last_error = "G kernel: more than 33.5M models in one launch (grid.y limit); shard the model axis";
        return MQ_ERR_ARG;
      }
    }
    HIPCHK(start_timer());
    HIPCHK(launch_qsa(k, T->qargs[k].as<QArgs>(), gx, gy, lds, st));
  }
  for (size_t sgi = 0; use_qsa && T->fc_count > 0 && T->fca && sgi < T->fca_segs.size(); sgi++) {
    const FcaPlanSeg& sg = T->fca_segs[sgi];
    FcaArgs f{};
    f.n = sg.n_tapes;
    f.n_atoms = sg.n_atoms;
    f.n_groups = sg.n_groups;
    f.groups = T->fca_group_dev.as<FcaGroup>() + sg.group_off;
    f.atoms = T->fc_cmp_dev.as<FcCmp>() + sg.atom_off;
    f.xfs = T->fca_any_xf ? T->fca_xf_dev.as<FcXf>() + sg.atom_off : nullptr;
    f.lists = T->fc_mask_dev.as<uint32_t>();
    f.chunk_off = T->fca_chunk_dev.as<uint32_t>() + sg.chunk_first;
    f.tape_out = T->fca_out_dev.as<uint32_t>() + sg.tape_first;
    f.tape_metric = T->fca_metric_dev.as<uint32_t>() + 2 * (size_t)sg.tape_first;
    f.vars = c->vars.as<uint32_t>();
    f.bool_masks = c->bmasks.as<uint64_t>();
    f.n_bool_masks = c->n_bmask;
    f.mode = verdicts ? 1 : 0;
    f.early_exit = verdicts ? 0 : c->early_exit;
    f.M = c->M;
    f.index_base = c->index_base;
    f.best = best;
    f.verdicts = verdicts;
    f.counters = c->counters.as<unsigned long long>();
    f.stage_masks = T->fc_smask_dev.as<uint32_t>() + sg.smask_off;
    f.n_smask = sg.n_smask;
    HIPCHK(start_timer());
    HIPCHK(launch_fca(f, st));
  }
  if (use_qsa && T->fc_count > 0 && !T->fca) {
    FcArgs f{};
    f.tapes = T->fc_tapes_dev.as<FcTape>();
    f.n = T->fc_count;
    const int64_t tiles = (c->M + 63) / 64;
    // a workgroup's 4 waves split the launch's tapes on one tile (the staged rows serve all of
    // them); more tapes than ~256 a tile, or a latency-bound launch, go to several workgroups
    f.tpg = latency ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>((f.n + 3) / 4, 64));
    (void)tiles;
    f.stage_rows = T->fc_stage_dev.as<uint32_t>();
    f.n_stage = T->fc_stage_n;
    f.stage_masks = T->fc_smask_dev.as<uint32_t>();
    f.n_smask = T->fc_smask_n;
    f.prefix = T->fc_prefix_dev.as<unsigned long long>();
    f.mask_lds = T->fc_mask_dev.as<uint32_t>();
    f.cmps = T->fc_cmp_dev.as<FcCmp>();
    f.vars = c->vars.as<uint32_t>();
    f.bool_masks = c->bmasks.as<uint64_t>();
    f.n_bool_masks = c->n_bmask;
    f.mode = verdicts ? 1 : 0;
    f.early_exit = verdicts ? 0 : c->early_exit;
    f.M = c->M;
    f.index_base = c->index_base;
    f.best = best;
    f.verdicts = verdicts;
    f.counters = c->counters.as<unsigned long long>();
    HIPCHK(start_timer());
    HIPCHK(launch_fc(f, st));
  }
  for (const auto& v : cpp) {
    if (v.count <= 0) continue;
    KArgs a = make_args(c, T, v);
    const size_t scratch_bytes = (size_t)a.grid * (size_t)a.tmp_words_per_wave * 4;
    if (scratch_bytes) {
      HIPCHK(c->scratch.ensure(scratch_bytes));
      a.scratch = c->scratch.as<uint32_t>();
    }
    a.best = best;
    a.verdicts = verdicts;
    a.early_exit = verdicts ? 0 : c->early_exit;
    HIPCHK(start_timer());
    HIPCHK(launch_qs(a, v.L, v.keccak, verdicts != nullptr, st));
  }
  if (kend) {
    HIPCHK(start_timer());
    HIPCHK(hipEventRecord(kend, st));
  }
  return MQ_OK;
}

static int kernel_times_one(mq_ctx* c, std::vector<float>& ms_out, int reset) {
  HIPCHK(hipSetDevice(c->device));
  ms_out.clear();
  for (size_t i = 0; i < c->kev_used; i++) {
    HIPCHK(hipEventSynchronize(c->kev[i].second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->kev[i].first, c->kev[i].second));
    ms_out.push_back(ms);
  }
  if (reset) c->kev_used = 0;
  return MQ_OK;
}

int mq_kernel_times_device(mq_ctx* c, int32_t device_index, float* out_ms, int32_t max_out, int32_t* n_out,
                           int reset) {
  if (!c || (max_out > 0 && !out_ms)) return MQ_ERR_ARG;
  const std::vector<mq_ctx*> devs = devices_of(c);
  if (device_index < 0 || device_index >= (int32_t)devs.size()) return MQ_ERR_ARG;
  std::vector<float> one;
  const int rc = kernel_times_one(devs[device_index], one, reset);
  HIPCHK(hipSetDevice(c->device));
  if (rc) return rc;
  const int32_t n = (int32_t)one.size();
  for (int32_t i = 0; i < n && i < max_out; i++) out_ms[i] = one[i];
  if (n_out) *n_out = n;
  return MQ_OK;
}

int mq_launch_times(mq_ctx* c, float* reduce_ms, double* issue_ms, double* peer_issue_ms, int32_t max_out,
                    int32_t* n_out, int reset) {
  if (!c || !n_out || (max_out > 0 && (!reduce_ms || !issue_ms || !peer_issue_ms))) return MQ_ERR_ARG;
  HIPCHK(hipSetDevice(c->device));
  const int32_t n = (int32_t)c->issue_ms.size();
  for (int32_t i = 0; i < n && i < max_out; i++) {
    float ms = 0.f;
    if ((size_t)i < c->rev_used) {
      HIPCHK(hipEventSynchronize(c->rev[i].second));
      HIPCHK(hipEventElapsedTime(&ms, c->rev[i].first, c->rev[i].second));
    }
    reduce_ms[i] = ms;
    issue_ms[i] = c->issue_ms[i];
    peer_issue_ms[i] = c->peer_issue_ms[i];
  }
  *n_out = n;
  if (reset) {
    c->rev_used = 0;
    c->issue_ms.clear();
    c->peer_issue_ms.clear();
  }
  return MQ_OK;
}

int mq_kernel_times(mq_ctx* c, float* out_ms, int32_t max_out, int32_t* n_out, int reset) {
  if (!c || (max_out > 0 && !out_ms)) return MQ_ERR_ARG;
  // several devices: launch i took as long as its slowest device
  std::vector<float> all, one;
  for (mq_ctx* d : devices_of(c)) {
    const int rc = kernel_times_one(d, one, reset);
    if (rc) return rc;
    if (all.size() < one.size()) all.resize(one.size(), 0.f);
    for (size_t i = 0; i < one.size(); i++) all[i] = std::max(all[i], one[i]);
  }
  HIPCHK(hipSetDevice(c->device));
  const int32_t n = (int32_t)all.size();
  for (int32_t i = 0; i < n && i < max_out; i++) out_ms[i] = all[i];
  if (n_out) *n_out = n;
  return MQ_OK;
}

static int launch_one(mq_ctx* c, mq_tapes* T, int32_t* d_best, hipStream_t st) {
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_init_best(d_best, T->n_tapes, st));
  return launch_all(c, T, d_best, nullptr, st);
}

int mq_launch_first_hit(mq_ctx* c, mq_tapes* T, int32_t* d_best, void* stream) {
  if (!c || !T || !d_best) return MQ_ERR_ARG;
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  if (T->ctx != c || T->peers.size() != c->peers.size()) return MQ_ERR_STATE;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  if (st != c->stream) DevPool::get().mark_foreign(c->device);
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = clk::now();
  int rc = launch_one(c, T, d_best, st);
  if (rc || c->comms.empty()) return rc;
  // every device evaluates its contiguous shard of candidates (global indices), then ONE RCCL
  // MIN all-reduce of int32[N] (4N bytes over xGMI) leaves the global first hit in d_best
  std::vector<mq_ctx*> devs = devices_of(c);
  std::vector<int32_t*> bufs{d_best};
  std::vector<hipStream_t> streams{st};
  const clk::time_point t1 = clk::now();
  for (size_t i = 0; i < c->peers.size(); i++) {
    mq_ctx* p = c->peers[i];
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(p->best_tmp.ensure(sizeof(int32_t) * std::max(T->n_tapes, 1)));
    rc = launch_one(p, T->peers[i], p->best_tmp.as<int32_t>(), p->stream);
    if (rc) return rc;
    bufs.push_back(p->best_tmp.as<int32_t>());
    streams.push_back(p->stream);
  }
  const clk::time_point t2 = clk::now();
  std::pair<hipEvent_t, hipEvent_t>* re = nullptr;
  if (c->time_kernels) {
    HIPCHK(hipSetDevice(c->device));
    if (c->rev_used == c->rev.size()) {
      std::pair<hipEvent_t, hipEvent_t> e{};
      HIPCHK(hipEventCreate(&e.first));
      HIPCHK(hipEventCreate(&e.second));
      c->rev.push_back(e);
    }
    re = &c->rev[c->rev_used++];
    HIPCHK(hipEventRecord(re->first, st));
  }
  if (T->n_tapes > 0) {
    ncclResult_t r = ncclGroupStart();
    for (size_t g = 0; r == ncclSuccess && g < devs.size(); g++)
      r = ncclAllReduce(bufs[g], bufs[g], (size_t)T->n_tapes, ncclInt32, ncclMin, c->comms[g], streams[g]);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return rccl_fail(r, "ncclAllReduce(ncclMin)");
    if (r2 != ncclSuccess) return rccl_fail(r2, "ncclGroupEnd");
  }
  HIPCHK(hipSetDevice(c->device));
  if (re) {
    HIPCHK(hipEventRecord(re->second, st));
    const clk::time_point t3 = clk::now();
    c->issue_ms.push_back(std::chrono::duration<double, std::milli>(t3 - t0).count());
    c->peer_issue_ms.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
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

int mq_host_times(mq_ctx* c, double* out, int32_t max_out, int32_t* n_out, int reset) {
  if (!c || !n_out || (max_out > 0 && !out)) return MQ_ERR_ARG;
  *n_out = MQ_HOST_PHASES;
  for (int i = 0; i < MQ_HOST_PHASES && i < max_out; i++) out[i] = c->host_t[i];
  if (reset)
    for (double& x : c->host_t) x = 0;
  return MQ_OK;
}

int mq_counters(mq_ctx* c, double* out3, int reset) {
  if (!c || !out3) return MQ_ERR_ARG;
  for (int i = 0; i < 3; i++) out3[i] = 0;
  for (mq_ctx* d : devices_of(c)) {
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> raw(kCounterBytes / sizeof(unsigned long long));
    HIPCHK(hipMemcpy(raw.data(), d->counters.p, kCounterBytes, hipMemcpyDeviceToHost));
    unsigned long long cnt[3];
    sum_counter_slots(raw, cnt);
    for (int i = 0; i < 3; i++) out3[i] += (double)cnt[i];
    if (reset) HIPCHK(hipMemset(d->counters.p, 0, kCounterBytes));
  }
  HIPCHK(hipSetDevice(c->device));
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
  const std::vector<mq_ctx*> devs = devices_of(c);
  for (mq_ctx* d : devs) {
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipMemsetAsync(d->counters.p, 0, kCounterBytes, d->stream));
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(c->best_tmp.ensure(sizeof(int32_t) * T->n_tapes));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  int rc = mq_launch_first_hit(c, T, c->best_tmp.as<int32_t>(), c->stream);
  if (rc) return rc;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  rc = mq_finalize_first_hit(c, T, c->best_tmp.as<int32_t>(), c->stream);
  if (rc) return rc;
  // both readbacks through pinned staging: [counter slots | first hits]
  const size_t best_bytes = sizeof(int32_t) * T->n_tapes;
  const bool pinned = c->readback_host.ensure(kCounterBytes + best_bytes) == hipSuccess;
  uint8_t* stage = pinned ? (uint8_t*)c->readback_host.p : nullptr;
  HIPCHK(hipMemcpyAsync(pinned ? (void*)(stage + kCounterBytes) : (void*)out, c->best_tmp.p, best_bytes,
                        hipMemcpyDeviceToHost, c->stream));
  unsigned long long total[3] = {0, 0, 0};
  for (mq_ctx* d : devs) {
    HIPCHK(hipSetDevice(d->device));
    std::vector<unsigned long long> raw(kCounterBytes / sizeof(unsigned long long));
    if (d == c && pinned) {
      HIPCHK(hipMemcpyAsync(stage, d->counters.p, kCounterBytes, hipMemcpyDeviceToHost, d->stream));
      HIPCHK(hipStreamSynchronize(d->stream));
      std::memcpy(raw.data(), stage, kCounterBytes);
    } else {
      HIPCHK(hipMemcpyAsync(raw.data(), d->counters.p, kCounterBytes, hipMemcpyDeviceToHost, d->stream));
      HIPCHK(hipStreamSynchronize(d->stream));
    }
    unsigned long long cnt[3];
    sum_counter_slots(raw, cnt);
    for (int i = 0; i < 3; i++) total[i] += cnt[i];
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  // (every device's stream was waited for above; the RCCL reduce runs on them)
  T->in_flight = false;
  for (mq_tapes* p : T->peers) p->in_flight = false;
  if (pinned) std::memcpy(out, stage + kCounterBytes, best_bytes);
  if (stats) {
    float ms = 0;
    // lead stream: from before the first launch to after the RCCL reduce (all devices)
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    stats->kernel_ms = ms;
    stats->pairs_evaluated = (int64_t)total[0];
    stats->node_evals = (double)total[1];
    stats->alg_ops = (double)total[2];  // exact: per evaluated (tape, model) pair, the tape's cost
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
  return mq_eval_tapes_verdicts(c, T, bits, first_hit_out);
}

// verdict bytes [tape][local model] of ONE device
static int verdict_bytes_one(mq_ctx* c, mq_tapes* T, std::vector<uint8_t>& host) {
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  PhaseTimer pt(&c->host_t[7]);   // (includes phases 3-6 of this launch)
  HIPCHK(hipSetDevice(c->device));
  const size_t nbytes = (size_t)T->n_tapes * (size_t)c->M;
  HIPCHK(c->verdict_buf.ensure(std::max<size_t>(nbytes, 1)));
  HIPCHK(hipMemsetAsync(c->verdict_buf.p, 0, std::max<size_t>(nbytes, 1), c->stream));
  const int rc = launch_all(c, T, nullptr, c->verdict_buf.as<uint8_t>(), c->stream);
  if (rc) return rc;
  host.resize(nbytes);
  // small batches (the drop-in path) through pinned memory; large ones straight into the vector
  constexpr size_t kPinnedVerdictBytes = size_t(8) << 20;
  if (nbytes && nbytes <= kPinnedVerdictBytes && c->verdict_host.ensure(nbytes) == hipSuccess) {
    HIPCHK(hipMemcpyAsync(c->verdict_host.p, c->verdict_buf.p, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    T->in_flight = false;
    std::memcpy(host.data(), c->verdict_host.p, nbytes);
    return MQ_OK;
  }
  if (nbytes) HIPCHK(hipMemcpyAsync(host.data(), c->verdict_buf.p, nbytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  T->in_flight = false;
  return MQ_OK;
}

int mq_eval_tapes_verdicts(mq_ctx* c, mq_tapes* T, uint8_t* bits, int32_t* first_hit_out) {
  if (!c || !T || !bits) return MQ_ERR_ARG;
  if (!c->have_models) return MQ_ERR_NO_MODELS;
  if (T->ctx != c || T->peers.size() != c->peers.size()) return MQ_ERR_STATE;
  const std::vector<mq_ctx*> devs = devices_of(c);
  const int64_t M = c->peers.empty() ? c->M : c->M_total;
  std::memset(bits, 0, ((size_t)T->n_tapes * (size_t)M + 7) / 8);
  std::vector<int32_t> fh(T->n_tapes, -1);
  std::vector<uint8_t> host;
  // devices in global candidate order: the first set bit met per tape is its global first hit
  for (size_t g = 0; g < devs.size(); g++) {
    mq_tapes* tg = g == 0 ? T : T->peers[g - 1];
    const int rc = verdict_bytes_one(devs[g], tg, host);
    if (rc) return rc;
    const int64_t Mg = devs[g]->M, lo = g < c->shard_lo.size() ? c->shard_lo[g] : 0;
    for (int t = 0; t < T->n_tapes; t++) {
      const uint8_t* row = host.data() + (size_t)t * Mg;
      for (int64_t m = 0; m < Mg; m++) {
        if (!row[m]) continue;
        const size_t i = (size_t)t * M + lo + m;
        bits[i >> 3] |= (uint8_t)(1u << (i & 7));
        if (fh[t] < 0) fh[t] = (int32_t)(devs[g]->index_base + m);
      }
    }
  }
  HIPCHK(hipSetDevice(c->device));
  if (first_hit_out)
    for (int t = 0; t < T->n_tapes; t++) first_hit_out[t] = T->unsupported[t] ? -2 : fh[t];
  return MQ_OK;
}

int mq_ctx_set_option(mq_ctx* c, int option, int value) {
  if (!c) return MQ_ERR_ARG;
  if (option == MQ_OPT_USE_RCCL) {
    if (value) return rccl_init(c);
    if (!c->peers.empty()) return MQ_ERR_ARG;   // several devices always reduce over RCCL
    for (ncclComm_t cm : c->comms) (void)ncclCommDestroy(cm);
    c->comms.clear();
    return MQ_OK;
  }
  if (option == MQ_OPT_RCCL_ACTIVE) return c->comms.empty() ? 0 : 1;
  for (mq_ctx* p : c->peers) {
    const int rc = mq_ctx_set_option(p, option, value);
    if (rc < 0) return rc;
  }
  switch (option) {
    case MQ_OPT_USE_ASM: c->use_asm = value ? 1 : 0; return MQ_OK;
    case MQ_OPT_EARLY_EXIT: c->early_exit = value ? 1 : 0; return MQ_OK;
    case MQ_OPT_LATENCY_WAVES: c->latency_waves = value > 0 ? value : 0; return MQ_OK;
    case MQ_OPT_KECCAK_HOST_BLOCKS: c->keccak_host_blocks = value > 0 ? value : 0; return MQ_OK;
    case MQ_OPT_ASM_READY: return c->qsa_ready ? 1 : 0;
    case MQ_OPT_TIME_KERNELS:
      c->time_kernels = value ? 1 : 0;
      c->kev_used = 0;
      c->rev_used = 0;
      c->issue_ms.clear();
      c->peer_issue_ms.clear();
      return MQ_OK;
    default: return MQ_ERR_ARG;
  }
}

int mq_tapes_qsa_split(mq_tapes* T, int32_t* n_p, int32_t* n_g, int32_t* live) {
  if (!T) return MQ_ERR_ARG;
  if (n_p) *n_p = T->qsa_live ? T->q_count[0] : 0;
  if (n_g) *n_g = T->qsa_live ? T->q_count[1] : 0;
  if (live) *live = T->qsa_live ? 1 : 0;
  return MQ_OK;
}

int mq_tapes_qsa_histogram(mq_tapes* T, int32_t which, int64_t* hist_out, int32_t cap, int64_t* pairs_out,
                           int32_t* n_kinds_out) {
  if (!T || which < 0 || which > 2 || cap < 0) return MQ_ERR_ARG;
  if (n_kinds_out) *n_kinds_out = QK_COUNT;
  const int n = std::min<int>(cap, QK_COUNT);
  const auto& h = T->qhist[which];
  for (int i = 0; i < n; i++) hist_out[i] = h.empty() ? 0 : h[i];
  if (pairs_out)
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++)
        pairs_out[(size_t)i * n + j] = (which == 1 && !T->qpairs.empty()) ? T->qpairs[(size_t)i * QK_COUNT + j]
                                       : (which == 0 && !T->qpairs_p.empty()) ? T->qpairs_p[(size_t)i * QK_COUNT + j] : 0;
  return MQ_OK;
}

const char* mq_qsa_kind_name(int32_t kind) {
  if (kind >= QK_COUNT && kind < QK_COUNT + kQsaProfExtra) return kQsaProfExtraNames[kind - QK_COUNT];
  return (kind >= 0 && kind < QK_COUNT) ? kQsaKindNames[kind] : nullptr;
}

int mq_qsa_profile(mq_ctx* c, int64_t* out, int32_t cap, int32_t* n_out, int reset) {
  if (!c || cap < 0 || (cap > 0 && !out)) return MQ_ERR_ARG;
  const int n = kQsaProfBytes > 0 ? 2 * (QK_COUNT + kQsaProfExtra) : 0;
  if (n_out) *n_out = n;
  if (n == 0) return MQ_OK;
  std::vector<int64_t> sum(n, 0);
  for (mq_ctx* d : devices_of(c)) {
    if (!d->prof.p) continue;
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<int64_t> v(n);
    HIPCHK(hipMemcpy(v.data(), d->prof.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
    for (int i = 0; i < n; i++) sum[i] += v[i];
    if (reset) HIPCHK(hipMemset(d->prof.p, 0, (size_t)kQsaProfBytes));
  }
  for (int i = 0; i < std::min(n, cap); i++) out[i] = sum[i];
  return MQ_OK;
}

int mq_tapes_flat_split(mq_tapes* T, int32_t* n_flat_tapes, int32_t* n_flat_columns) {
  if (!T) return MQ_ERR_ARG;
  if (n_flat_tapes) *n_flat_tapes = T->qsa_live ? T->fc_count : 0;
  if (n_flat_columns) {
    int32_t n = 0;
    if (T->cq_live)
      for (const auto& fl : T->fc_lvl) n += fl ? fl->count : 0;
    *n_flat_columns = n;
  }
  return MQ_OK;
}

int mq_tapes_column_split(mq_tapes* T, int32_t* n_asm, int32_t* live) {
  if (!T) return MQ_ERR_ARG;
  if (n_asm) {   // (on qsg_kernel: the G-eligible columns less the flat ones fc_kernel runs)
    int32_t n = 0;
    if (T->cq_live)
      for (int x : T->cq_lvl_desc_n) n += x;
    *n_asm = n;
  }
  if (live) *live = T->cq_live ? 1 : 0;
  return MQ_OK;
}

int mq_tapes_column_gather(mq_tapes* T, int32_t* n_gather_columns) {
  if (!T || !n_gather_columns) return MQ_ERR_ARG;
  *n_gather_columns = (int32_t)T->cw.size();
  return MQ_OK;
}

int mq_tapes_column_keccak(mq_tapes* T, int32_t* n_keccak_columns) {
  if (!T || !n_keccak_columns) return MQ_ERR_ARG;
  *n_keccak_columns = (int32_t)T->kc.size();
  return MQ_OK;
}

int mq_tapes_column_keccak_predicates(mq_tapes* T, int32_t* n_predicate_columns) {
  if (!T || !n_predicate_columns) return MQ_ERR_ARG;
  size_t n = 0;
  for (const auto& h : T->kc) n += h.preds.size();
  *n_predicate_columns = (int32_t)n;
  return MQ_OK;
}

int mq_tapes_info(mq_tapes* T, int32_t* n_asm, int32_t* n_generic_l8, int32_t* n_generic_l16) {
  if (!T) return MQ_ERR_ARG;
  if (n_asm) *n_asm = T->qsa.count;
  if (n_generic_l8) *n_generic_l8 = T->gen[0].count;
  int wide = 0;
  for (int g = 1; g < kGen; g++) wide += T->gen[g].count;
  if (n_generic_l16) *n_generic_l16 = wide;
  return MQ_OK;
}

double mq_tape_alg_ops(const mq_tape_batch* tb, int32_t t) {
  if (!tb || t < 0 || t >= tb->n_tapes) return -1;
  return tape_alg_ops(tb, t);
}

int mq_keccak256_host(const uint8_t* data, const int64_t* offsets, int32_t n, uint8_t* out) {
  if ((n > 0 && (!data || !offsets || !out)) || n < 0) return MQ_ERR_ARG;
  for (int32_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return MQ_ERR_ARG;
  for (int32_t i = 0; i < n; i++) host_keccak256(data + offsets[i], offsets[i + 1] - offsets[i], out + 32 * (int64_t)i);
  return MQ_OK;
}

int mq_keccak256(mq_ctx* c, const uint8_t* data, const int64_t* offsets, int32_t n, uint8_t* out) {
  if (!c || (n > 0 && (!data || !offsets || !out)) || n < 0) return MQ_ERR_ARG;
  if (n == 0) return MQ_OK;
  // a small batch (the reference's call size: one to a few messages) is hashed on the host
  int64_t blocks = 0;
  for (int32_t i = 0; i < n && blocks <= c->keccak_host_blocks; i++) {
    if (offsets[i + 1] < offsets[i]) return MQ_ERR_ARG;
    blocks += (offsets[i + 1] - offsets[i]) / 136 + 1;
  }
  if (blocks <= c->keccak_host_blocks) return mq_keccak256_host(data, offsets, n, out);
  HIPCHK(hipSetDevice(c->device));
  const int64_t total = offsets[n];
  // (kept in the context: a hipMalloc / hipFree pair per call cost more than the hashing)
  DevBuf& d_data = c->kec_data;
  DevBuf& d_off = c->kec_off;
  DevBuf& d_out = c->kec_out;
  HIPCHK(d_data.upload(data, (size_t)std::max<int64_t>(total, 1), c->stream));
  HIPCHK(d_off.upload(offsets, (size_t)n + 1, c->stream));
  HIPCHK(d_out.ensure((size_t)32 * n));
  HIPCHK(launch_keccak(d_data.as<uint8_t>(), d_off.as<int64_t>(), n, d_out.as<uint8_t>(), c->stream));
  HIPCHK(hipMemcpyAsync(out, d_out.p, (size_t)32 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MQ_OK;
}

}  // extern "C"
