/*
 * mq.h — C-ABI of the MI355X quick-sat evaluator (libmq.so).
 *
 * The reference has no native boundary: quick-sat is the Python loop
 *   ModelCache.check_quick_sat   mythril/support/support_utils.py:60-67
 * which, for each cached z3 model in MRU-first order (`reversed(lru_cache.keys())`,
 * support_utils.py:62), evaluates `is_true(deepcopy(model).eval(expr, model_completion=True))`
 * (support_utils.py:63-64) and returns the first satisfying model.  It is reached from
 *   get_model                    mythril/support/model.py:100-103
 * This header is the native replacement of that loop, batched: N constraint tapes x M
 * candidate models -> first satisfying candidate index per tape.  Every entry point below
 * names the reference interface it replaces.  See INTEGRATION.md for the ctypes binding a
 * Mythril maintainer adds at model.py:101 / support_utils.py:60.
 *
 * Conventions:
 *   - every function returns 0 (MQ_OK) or a negative mq_status; nothing throws across the ABI;
 *   - input buffers are copied; the caller keeps ownership of host memory;
 *   - a context is confined to one host thread; calls are synchronous unless named *_async;
 *   - candidate index 0 is the MRU model (reversed(LRU.keys())[0]).
 */
#ifndef MQ_H
#define MQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status codes */
typedef enum mq_status {
  MQ_OK = 0,
  MQ_ERR_ARG = -1,         /* malformed argument (null pointer, bad size, bad node reference) */
  MQ_ERR_HIP = -2,         /* HIP runtime error */
  MQ_ERR_NOMEM = -3,       /* device allocation failed */
  MQ_ERR_NO_MODELS = -4,   /* mq_eval_* before mq_models_upload */
  MQ_ERR_NODEV = -5,       /* no usable gfx950 device */
  MQ_ERR_TAPE = -6,        /* tape is not well sorted (type error) */
  MQ_ERR_STATE = -7        /* context used after destroy / wrong thread */
} mq_status;

/* first_hit sentinels: */
#define MQ_NO_HIT (-1)       /* no candidate satisfies the tape -> caller falls through to z3 */
#define MQ_UNSUPPORTED (-2)  /* tape uses something the evaluator does not implement -> z3 eval */

/* ------------------------------------------------------------------ tape IR
 * A tape is a topologically ordered DAG of nodes (postfix order: operands precede users);
 * the LAST node of a tape is its root and must be Bool-sorted.  Operands a/b/c are indices of
 * earlier nodes of the same tape unless the opcode says they are immediates.
 * width: result width in bits; 0 means Bool sort.  Array-sorted nodes (STORE, CONST_ARRAY,
 * ARRAY_VAR) carry the range width.
 * Semantics: SMT-LIB 2.6 FixedSizeBitVectors + z3 model completion.
 * Widths up to 2048 bits (keccak256_<n> inputs of up to 256 bytes: Concat of memory bytes,
 * mythril/laser/ethereum/instructions.py:1043-1052); MUL / *DIV / *REM / SMOD and the *MUL_NO*
 * predicates up to 512 bits.  Anything wider makes the tape MQ_UNSUPPORTED (fail closed).
 * Vocabulary: mythril/laser/smt/{bitvec,bitvec_helper,bool,array,function}.py.
 */
typedef enum mq_op {
  /* leaves */
  MQ_OP_CONST = 1,        /* a = word offset of the value in const_words (ceil(width/32) LE limbs);
                             Bool consts use MQ_OP_TRUE/FALSE */
  MQ_OP_VAR = 2,          /* a = model variable index (BV or Bool); absent => 0 / false */
  MQ_OP_TRUE = 3,
  MQ_OP_FALSE = 4,
  /* Bool connectives (args Bool) */
  MQ_OP_NOT = 10,         /* a */
  MQ_OP_AND = 11,         /* a, b   (n-ary z3 and is folded into a chain) */
  MQ_OP_OR = 12,          /* a, b */
  MQ_OP_XOR = 13,         /* a, b */
  MQ_OP_IMPLIES = 14,     /* a => b */
  MQ_OP_IFF = 15,         /* a == b on Bool */
  MQ_OP_BITE = 16,        /* a ? b : c on Bool */
  /* BV predicates (-> Bool) */
  MQ_OP_EQ = 20,          /* a == b (same width) */
  MQ_OP_ULT = 21,
  MQ_OP_ULE = 22,
  MQ_OP_SLT = 23,
  MQ_OP_SLE = 24,
  MQ_OP_UMUL_NOOVFL = 25, /* a*b < 2^W (unsigned) */
  MQ_OP_SMUL_NOOVFL = 26, /* signed a*b <= 2^(W-1)-1 */
  MQ_OP_SMUL_NOUDFL = 27, /* signed a*b >= -2^(W-1) */
  /* BV arithmetic (mod 2^W) */
  MQ_OP_ADD = 30,
  MQ_OP_SUB = 31,
  MQ_OP_MUL = 32,
  MQ_OP_NEG = 33,         /* a */
  MQ_OP_UDIV = 34,        /* udiv(a,0) = 2^W-1 */
  MQ_OP_UREM = 35,        /* urem(a,0) = a */
  MQ_OP_SDIV = 36,        /* sdiv(a,0) = a<0 ? 1 : -1 */
  MQ_OP_SREM = 37,        /* srem(a,0) = a (sign of dividend) */
  MQ_OP_SMOD = 38,        /* smod(a,0) = a (sign of divisor) */
  /* bitwise / shifts */
  MQ_OP_BAND = 40,
  MQ_OP_BOR = 41,
  MQ_OP_BXOR = 42,
  MQ_OP_BNOT = 43,        /* a */
  MQ_OP_SHL = 44,         /* amount = full W-bit value of b; >= W -> 0 */
  MQ_OP_LSHR = 45,
  MQ_OP_ASHR = 46,        /* >= W -> sign fill */
  /* width changes */
  MQ_OP_EXTRACT = 50,     /* a = arg, b = hi, c = lo (immediates) */
  MQ_OP_CONCAT = 51,      /* a = high part, b = low part */
  MQ_OP_ZEXT = 52,        /* a = arg, b = k (immediate) */
  MQ_OP_SEXT = 53,        /* a = arg, b = k (immediate) */
  MQ_OP_ITE = 54,         /* a = Bool cond, b = then, c = else (BV) */
  /* arrays and uninterpreted functions (per-model interpretations) */
  MQ_OP_SELECT = 60,      /* a = array node, b = index */
  MQ_OP_STORE = 61,       /* a = array node, b = index, c = value   (array sort) */
  MQ_OP_CONST_ARRAY = 62, /* a = value node (K(sort, v))            (array sort) */
  MQ_OP_ARRAY_VAR = 63,   /* a = function id of the model table     (array sort) */
  MQ_OP_UF = 64,          /* a = function id, b = arg0, c = arg1 (MQ_NONE if arity 1) */
  /* An arity-1 lookup whose key is wider than 2048 bits (keccak256_<n> of a > 256-byte SHA3
     input, instructions.py:1018-1055), matched 256 bits at a time so that no value is wider:
     MQ_OP_UF_CHUNK: width 64, a = function id, b = key chunk k (bits [256k, 256k + width(b))),
       c = the UF_CHUNK of chunk k - 1, MQ_NONE for k = 0 (k = the length of that chain).  Its
       value is the set of the model's table entries (bit e = entry e, e < 64) whose key chunks
       0..k all equal the given ones.
     MQ_OP_UF_WIDE: a = function id, b = the last UF_CHUNK; the value of the first entry in the
       set, or the table's else value when it is empty — exactly the lookup of the whole key.
     A tape with these ops is unsupported (-2) under a model batch in which some model's table
     of that function holds more than 64 entries. */
  MQ_OP_UF_CHUNK = 65,
  MQ_OP_UF_WIDE = 66,
  /* interpreted keccak256 (Ethereum padding) of the big-endian bytes of a; width 256.
     NOT z3 semantics: only for keccak-consistent synthetic models and constant folding
     (keccak_function_manager.py:56-69). */
  MQ_OP_KECCAK = 70
} mq_op;

#define MQ_NONE 0xFFFFFFFFu

typedef struct mq_node {
  uint16_t op;     /* mq_op */
  uint16_t width;  /* result width in bits, 0 = Bool */
  uint32_t a, b, c;
} mq_node;

typedef struct mq_tape_batch {
  int32_t n_tapes;
  const int64_t* tape_offsets;   /* [n_tapes+1]: tape t = nodes[tape_offsets[t] .. tape_offsets[t+1]) */
  const mq_node* nodes;
  const uint32_t* const_words;   /* pool shared by all tapes (MQ_OP_CONST.a indexes it) */
  int64_t n_const_words;
} mq_tape_batch;

/* A stream of queries over ONE hash-consed DAG (the z3 AST table of a run: paths forked from a
 * common parent share their constraints, and the keccak axioms ride on every query,
 * constraints.py:127-128).  nodes[0..n_nodes) is postfix (operands precede users) and grows
 * append-only on the caller's side; tape t is the AND of the conjunct roots
 * roots[root_offsets[t] .. root_offsets[t+1]) (none: true), i.e. And(*constraints) of
 * model.py:101 without re-lowering shared conjuncts.  The evaluator extracts each tape's
 * reachable nodes itself. */
typedef struct mq_dag_batch {
  int64_t n_nodes;
  const mq_node* nodes;
  const uint32_t* const_words;
  int64_t n_const_words;
  int32_t n_tapes;
  const int64_t* root_offsets;   /* [n_tapes+1] */
  const uint32_t* roots;
} mq_dag_batch;

/* ------------------------------------------------------------------ candidate models
 * One batch = M candidate models in global candidate order (0 = MRU), the z3 ModelRef
 * contents serialized WITHOUT completion (support_utils.py:63 deep-copies because eval with
 * completion mutates the model; absence is encoded as 0 / empty table here).
 *   scalar variables: SoA, u32 limbs: var_words[(var_word_off[v] + limb) * n_models + m],
 *                     var_word_off[v] = sum_{u<v} limbs(var_width[u]), limbs(0) = 1.
 *   functions (UFs keccak256_<n>, keccak256_<n>-1, Power; array interpretations as-array):
 *     function f, model m has entries [entry_ptr[f*(M+1)+m], entry_ptr[f*(M+1)+m+1]) of its
 *     own list; entry e of f occupies words entry_words[entry_base[f] + e*stride_f ..] with
 *     stride_f = sum_i limbs(arg_width[i]) + limbs(result_width): args first, then value.
 *     else value of (f, m): else_words[else_base[f] + m*limbs(result_width) ..].
 *     A function absent from a model has no entries and else value 0 (z3 completion).
 *   Variable words are reduced mod 2^width on upload (bits above a width are ignored); function
 *   entry keys must already be canonical (they are matched word for word).
 */
typedef struct mq_func_desc {
  uint16_t arity;          /* 1 or 2 */
  uint16_t result_width;   /* 0 = Bool */
  uint16_t arg_width[2];
} mq_func_desc;

typedef struct mq_model_batch {
  int64_t n_models;
  int64_t index_base;              /* global candidate index of local model 0 (model-axis shard) */
  int32_t n_vars;
  const uint16_t* var_width;       /* [n_vars] */
  const uint32_t* var_words;
  int32_t n_funcs;
  const mq_func_desc* funcs;       /* [n_funcs] */
  const int64_t* entry_ptr;        /* [n_funcs * (n_models + 1)] */
  const int64_t* entry_base;       /* [n_funcs] */
  const uint32_t* entry_words;
  int64_t n_entry_words;
  const int64_t* else_base;        /* [n_funcs] */
  const uint32_t* else_words;
  int64_t n_else_words;
} mq_model_batch;

/* ------------------------------------------------------------------ statistics */
typedef struct mq_stats {
  double kernel_ms;        /* device time of the evaluation kernels (HIP events) */
  double node_evals;       /* sum over evaluated (tape, model) pairs of |tape| nodes */
  double alg_ops;          /* algorithmic 32-bit VALU ops (SURVEY §8(d) cost table) */
  int64_t pairs_evaluated; /* (tape, model) pairs actually evaluated (early exit skips the rest) */
  int32_t n_hits;
  int32_t n_unsupported;
} mq_stats;

typedef struct mq_ctx mq_ctx;
typedef struct mq_tapes mq_tapes;

/* Create a context over n_dev devices dev_ids[0..n_dev) (dev_ids may be NULL for n_dev = 1:
   device 0).  Mythril is one process (mythril/mythril/mythril_analyzer.py:136-185), so one
   context drives every GPU of the node: mq_models_upload splits the candidate
   axis into contiguous shards in global candidate order (device g holds [g*M/n, (g+1)*M/n)),
   tapes are compiled once and replicated, and the per-tape first hits are combined by an
   in-library RCCL ncclAllReduce(ncclMin) over xGMI (communicators from ncclCommInitAll), so the
   global MRU-first order of support_utils.py:62 survives the merge.  With
   n_dev = 1 the RCCL path is off unless MQ_OPT_USE_RCCL is set.  The alternative of one process
   per GPU (torch.distributed, mythril_amd/dist.py) uses n_dev = 1 contexts. */
int mq_ctx_create(int n_dev, const int* dev_ids, mq_ctx** out);
void mq_ctx_destroy(mq_ctx* ctx);
const char* mq_strerror(int code);

/* Replace the candidate set (ModelCache contents, support_utils.py:56-58 / model.py:125).
   n_models may be 0 (an empty model-axis shard: every tape reports MQ_NO_HIT). */
int mq_models_upload(mq_ctx* ctx, const mq_model_batch* models);

/* Host-only (no device needed): candidates [lo, hi) of `models` as a batch of their own, with
   index_base + lo — exactly the shard device g of a multi-device context holds (contiguous in
   global candidate order); also what a one-process-per-GPU caller uploads per rank.
   Variable rows and function entries are packed into a buffer owned by *handle (else values
   point into `models`, which must outlive *out); release it with mq_models_shard_free. */
int mq_models_shard(const mq_model_batch* models, int64_t lo, int64_t hi, mq_model_batch* out, void** handle);
void mq_models_shard_free(void* handle);

/* Compile + upload a tape batch once (the lowering of simplify(And(*constraints)).raw,
   model.py:101); reusable across evaluations.  n_unsupported_out may be NULL. */
int mq_tapes_upload(mq_ctx* ctx, const mq_tape_batch* batch, mq_tapes** out, int32_t* n_unsupported_out);
void mq_tapes_free(mq_tapes* tapes);

/* Same for a DAG batch (the drop-in query stream; see mq_dag_batch). */
int mq_tapes_upload_dag(mq_ctx* ctx, const mq_dag_batch* dag, mq_tapes** out, int32_t* n_unsupported_out);

/* Host-only: tape t of a DAG batch as a self-contained postfix block (reachable nodes in DAG
   order, references renumbered, AND chain over the roots last; CONST nodes index the DAG's
   const pool) into nodes_out[cap]; *n_out = its length (nothing copied when cap is too small).
   For parity dumps / the oracle.  Returns 0, MQ_ERR_ARG or MQ_ERR_TAPE. */
int mq_dag_expand(const mq_dag_batch* dag, int32_t t, mq_node* nodes_out, int64_t cap, int64_t* n_out);

/* Batch-level hoisting: sub-terms shared by several tapes of the batch depend only on the model,
   so the lowering can replace them by derived model variables.  Column program k (a tape whose
   LAST node is the BV/Bool value to store, not necessarily Bool) is evaluated once per model and
   written into model variable var_index[k] before every evaluation launch of `tapes`; columns
   of level j may read columns of levels < j.  The uploaded model batch must contain the target
   variables with matching widths (their uploaded values are overwritten).  MQ_ERR_TAPE if a
   program is not supported (the caller then lowers without hoisting). */
int mq_tapes_set_columns(mq_tapes* tapes, const mq_tape_batch* programs, const int32_t* var_index,
                         const int32_t* level, int32_t n_columns);

/* check_quick_sat over the batch (support_utils.py:60-67): first_hit_out[t] = smallest
   global candidate index whose model satisfies tape t, MQ_NO_HIT, or MQ_UNSUPPORTED. */
int mq_eval_first_hit(mq_ctx* ctx, const mq_tape_batch* batch, int32_t* first_hit_out, mq_stats* stats);
int mq_eval_tapes_first_hit(mq_ctx* ctx, mq_tapes* tapes, int32_t* first_hit_out, mq_stats* stats);

/* Asynchronous form for the multi-GPU path: writes int32 first_hit[n_tapes] to DEVICE memory
   d_first_hit on HIP stream `stream` (NULL = context stream); INT32_MAX encodes "no hit" so a
   min-allreduce over ranks combines shards; mq_finalize_first_hit maps it back to MQ_NO_HIT. */
int mq_launch_first_hit(mq_ctx* ctx, mq_tapes* tapes, int32_t* d_first_hit, void* stream);
int mq_finalize_first_hit(mq_ctx* ctx, mq_tapes* tapes, int32_t* d_first_hit, void* stream);

/* Device work counters accumulated by every evaluation launch on this context since the last
   reset: out[0] (tape, model) pairs evaluated, out[1] node-evals, out[2] algorithmic ops
   (SURVEY §8(d)).  Synchronizes the context stream. */
int mq_counters(mq_ctx* ctx, double* out3, int reset);

/* Full verdict matrix for parity dumps: bit (t*M + m) of bits_out = tape t true on model m
   (M = all models of the last mq_models_upload, every device's shard in place).
   bits_out has ceil(n_tapes*M/8) bytes.  Unsupported tapes yield all-zero rows and are
   reported through first_hit_out (may be NULL). */
int mq_eval_verdicts(mq_ctx* ctx, const mq_tape_batch* batch, uint8_t* bits_out, int32_t* first_hit_out);
int mq_eval_tapes_verdicts(mq_ctx* ctx, mq_tapes* tapes, uint8_t* bits_out, int32_t* first_hit_out);

/* Concrete keccak256 (Ethereum padding 0x01) of n messages on the GPU (keccak-f[1600] kernel);
   message i = data[offsets[i] .. offsets[i+1]), digests_out = 32*n bytes.  A batch of at most
   MQ_OPT_KECCAK_HOST_BLOCKS 136-byte blocks in total is hashed on the host instead (one launch
   plus two copies cost more than that); 0 sends every batch to the GPU.
   Replaces eth_hash in sha3 (support_utils.py:92-100) / find_concrete_keccak (kfm.py:56-69). */
int mq_keccak256(mq_ctx* ctx, const uint8_t* data, const int64_t* offsets, int32_t n, uint8_t* digests_out);
/* The same on the host only (no context, no GPU): what mq_keccak256 runs below its threshold. */
int mq_keccak256_host(const uint8_t* data, const int64_t* offsets, int32_t n, uint8_t* digests_out);

/* Context options.  MQ_OPT_USE_ASM (default 1): run eligible 256-bit tapes on the gfx950
   assembly interpreter, the rest on the HIP C++ interpreter (0: HIP C++ for all — the A/B and
   parity cross-check).  MQ_OPT_EARLY_EXIT (default 1): waves skip a tape once a lower first
   hit is published.  MQ_OPT_ASM_READY (query): returns 1 if the assembly interpreter loaded.
   MQ_OPT_TIME_KERNELS (default 0): bracket the evaluation kernels of every launch with a HIP
   event pair on the launch stream (read back with mq_kernel_times; setting it clears them).
   MQ_OPT_USE_RCCL (default 1 when n_dev > 1, else 0): combine first hits with the RCCL MIN
   all-reduce; 1 on a single-device context runs that path with one rank (0 is refused when
   n_dev > 1).  MQ_OPT_RCCL_ACTIVE (query): 1 if the context reduces over RCCL.
   MQ_OPT_LATENCY_WAVES (default 0 = off): a launch of at most this many waves (tapes x 64-model
   tiles) runs the general assembly kernel with one tape per wave instead of several tapes per
   wave: a few tapes over a few models are latency-bound (the drop-in path at the reference's
   shape sets it).  Such a launch with more than 131 072 tape nodes (MQ_LATENCY_ASM_NODES)
   skips the assembly translation (host time) and runs on the HIP C++ kernel.
   MQ_OPT_KECCAK_HOST_BLOCKS (default 128): mq_keccak256 batches of at most this many blocks are
   hashed on the host (0: always on the GPU). */
enum mq_option {
  MQ_OPT_USE_ASM = 1,
  MQ_OPT_EARLY_EXIT = 2,
  MQ_OPT_ASM_READY = 3,
  MQ_OPT_TIME_KERNELS = 4,
  MQ_OPT_USE_RCCL = 5,
  MQ_OPT_RCCL_ACTIVE = 6,
  MQ_OPT_LATENCY_WAVES = 7,
  MQ_OPT_KECCAK_HOST_BLOCKS = 8
};
int mq_ctx_set_option(mq_ctx* ctx, int option, int value);

/* Device durations (ms) of the evaluation kernels of each launch since the last reset, in
   launch order (MQ_OPT_TIME_KERNELS on; several devices: the slowest device per launch).  Waits for those launches.  *n_out = number recorded
   (may exceed max_out; only max_out are written).  reset != 0 forgets them. */
int mq_kernel_times(mq_ctx* ctx, float* out_ms, int32_t max_out, int32_t* n_out, int reset);

/* The same for ONE device of a multi-device context (device_index 0 = the lead, i = dev_ids[i]),
   so a one-process N-GPU launch is attributable per device.  reset != 0 forgets that device's
   records only.  No reference counterpart (SURVEY §8(e) measurement). */
int mq_kernel_times_device(mq_ctx* ctx, int32_t device_index, float* out_ms, int32_t max_out, int32_t* n_out,
                           int reset);

/* Per mq_launch_first_hit since the last reset, on a context that reduces in-library
   (MQ_OPT_USE_RCCL) with MQ_OPT_TIME_KERNELS on: reduce_ms[i] = HIP events on the lead stream
   around the ncclGroup of the MIN all-reduce; issue_ms[i] = host milliseconds the call spent
   issuing every device's kernels and the reduce; peer_issue_ms[i] = the peers' share of it (their
   launches are issued one after another from the calling thread).  Waits for the reduce events.
   *n_out = number recorded (only max_out written).  No reference counterpart. */
int mq_launch_times(mq_ctx* ctx, float* reduce_ms, double* issue_ms, double* peer_issue_ms, int32_t max_out,
                    int32_t* n_out, int reset);

/* Diagnostic: host seconds this context spent per phase since the last reset (out[i], i <
   MQ_HOST_PHASES; *n_out = MQ_HOST_PHASES): 0 DAG expansion + tape compilation, 1 structural
   P/G translation at upload, 2 tape upload, 3 P translation at launch, 4 G translation at
   launch, 5 translated-program upload, 6 kernel-argument upload, 7 launch + readback, 8 model
   upload, 9 tape release.  No reference counterpart (the drop-in leg's host-time breakdown). */
#define MQ_HOST_PHASES 10
int mq_host_times(mq_ctx* ctx, double* out, int32_t max_out, int32_t* n_out, int reset);

/* How a compiled batch is split: tapes on the assembly interpreter, on the generic 256-bit
   and on the wider (512 / 1024 / 2048-bit) HIP C++ kernels (any pointer may be NULL). */
int mq_tapes_info(mq_tapes* tapes, int32_t* n_asm, int32_t* n_generic_l8, int32_t* n_generic_l16);

/* After a launch: how the assembly-eligible tapes were split between the preloaded-variable
   kernel (*n_p) and the general kernel (*n_g); *live = 0 when the batch fell back to the HIP C++
   kernel for the current model batch.  Returns 0 or MQ_ERR_ARG. */
int mq_tapes_qsa_split(mq_tapes* tapes, int32_t* n_p, int32_t* n_g, int32_t* live);

/* After a launch: hoisted column programs evaluated by the general assembly kernel (qsg_kernel,
   mode 3) for the current model batch, and whether that path ran (the others, and all of them
   when it did not, run on the HIP C++ column kernel).  Introspection for tests and the bench. */
int mq_tapes_column_split(mq_tapes* tapes, int32_t* n_asm, int32_t* live);
/* Tapes / hoisted Bool columns of the current translation that run on the flat-conjunction
   kernel (an AND of Bool variables and variable-constant compares: no interpreter). */
int mq_tapes_flat_split(mq_tapes* tapes, int32_t* n_flat_tapes, int32_t* n_flat_columns);

/* Hoisted columns that only arrange model-variable bits and constants, runs of bits gated by
   `i <s size` — the calldata words of calldata.py:48-55 (Concat of calldata.py:234-247 bytes
   If(i < calldatasize, calldata[i], 0)), their extracts and constant masks — evaluated by the
   bit-gather column kernel (cw.hip) instead of an interpreter.  Introspection for tests and the
   bench (MQ_NO_GATHER_COLUMNS=1 disables the path). */
int mq_tapes_column_gather(mq_tapes* tapes, int32_t* n_gather_columns);

/* Hoisted columns that are exactly keccak256(concat of model variables and constants) — the
   keccak applications of kfm.py:95-114 / instructions.py:1043-1052 over candidate models —
   evaluated by the dedicated keccak-f[1600] column kernel instead of an interpreter.
   Introspection for tests and the bench (MQ_NO_KECCAK_COLUMNS=1 disables the path). */
int mq_tapes_column_keccak(mq_tapes* tapes, int32_t* n_keccak_columns);

/* The Bool columns the same kernel evaluates from the digests it computes: a keccak column
   compared with a constant (h < c, h > c, h <= c, h >= c, h == c, low k bits of h zero — the
   keccak manager's axioms, keccak_function_manager.py:150-179), their lane masks stored
   directly (MQ_NO_KECCAK_PREDICATES=1 leaves them to the interpreters). */
int mq_tapes_column_keccak_predicates(mq_tapes* tapes, int32_t* n_predicate_columns);

/* After a launch: handler-kind histogram of the current assembly translation (which = 0: P
   tapes, 1: G tapes, 2: G column programs) into hist_out[cap]; each tape's program runs once per
   (tape, model) pair, so these are the dispatches per pair summed over tapes.  pairs_out
   (cap x cap, may be NULL): (kind, next kind) counts over the G tapes (which = 1, else zeros).
   *n_kinds_out = number of kinds.  Diagnostic (superinstruction planning).  Returns 0 or
   MQ_ERR_ARG. */
int mq_tapes_qsa_histogram(mq_tapes* tapes, int32_t which, int64_t* hist_out, int32_t cap, int64_t* pairs_out,
                           int32_t* n_kinds_out);

/* Name of handler kind `kind` of the assembly interpreters; past the last kind, the profile's
   tape-frame entries ("FRAME", "F_HDR", "F_EE", "F_END"); NULL when out of range. */
const char* mq_qsa_kind_name(int32_t kind);

/* Diagnostic G profile build only (gen_qsa.py QSA_PROF=1): the cycles charged to each handler
   kind and its dispatch count, interleaved (cycles, count) per kind plus the tape frame, into
   out[cap]; *n_out = entries (0 in product builds).  reset != 0 zeroes the accumulators. */
int mq_qsa_profile(mq_ctx* ctx, int64_t* out, int32_t cap, int32_t* n_out, int reset);

/* Static algorithmic cost of a tape; -1 if malformed. */
double mq_tape_alg_ops(const mq_tape_batch* batch, int32_t t);

/* Host-only compile report for tape t (no device needed): *supported (0/1), limbs per value L
   (8, 16, 32 or 64), register-stack depth, LDS temp slots, program words; reason (if unsupported) is
   copied into why[why_len].  Returns 0 or MQ_ERR_ARG. */
int mq_tape_compile_info(const mq_tape_batch* batch, int32_t t, int32_t* supported, int32_t* limbs,
                         int32_t* depth, int32_t* n_temps, int32_t* prog_words, char* why, int32_t why_len);

/* Host-only: how tape t compiles for the G assembly interpreter, whose operand stack has fewer
   slots than the other kernels' (kQsaStackG = 4): *depth_g / *n_temps_g / *prog_words_g of the
   program G runs (subtrees deeper than its stack spilled to LDS temps; the plain program when it
   already fits).  Returns 0, MQ_ERR_ARG, or MQ_ERR_TAPE when the tape does not compile. */
int mq_tape_compile_info_g(const mq_tape_batch* batch, int32_t t, int32_t* depth_g, int32_t* n_temps_g,
                           int32_t* prog_words_g);

/* Host-only: the compiled stack program of tape t (gprog.h instruction words, G_END last) into
   words[cap]; *n_words = its length (also when cap is too small, then nothing is copied).
   Returns 0, MQ_ERR_ARG, or MQ_ERR_TAPE when the tape does not compile. */
int mq_tape_program(const mq_tape_batch* batch, int32_t t, uint32_t* words, int32_t cap, int32_t* n_words);

/* Library version string. */
const char* mq_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MQ_H */
