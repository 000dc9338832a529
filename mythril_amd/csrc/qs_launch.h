// qs_launch.h — kernel argument block and launchers shared by mq_api.cpp and qs_kernels.hip.
#ifndef MQ_QS_LAUNCH_H
#define MQ_QS_LAUNCH_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gprog.h"

namespace mq {

// Work counters (pairs evaluated, node-evals, algorithmic ops): kCounterSlots slots of
// kCounterStride u64 (128 B apart), a wave adds into slot (workgroup id mod kCounterSlots) so a
// launch of 10^6 waves does not serialise on one cache line; the host sums the slots.
constexpr int kCounterSlots = 256;
constexpr int kCounterStride = 16;

// device view of one model function (UF or as-array interpretation)
struct FuncDev {
  uint32_t arity;
  uint32_t nl_a0, nl_a1, nl_res;
  uint32_t stride;      // words per entry
  uint32_t dense_e;     // > 0: also held as dense slots (G lookups): entry slots per model
  int64_t entry_base;   // word offset of entry 0 in entry_words
  int64_t ptr_base;     // offset of row pointers [M+1] in entry_ptr
  int64_t else_base;    // word offset of the SoA else block: else_words[else_base + limb*M + m]
  // dense slots (dense_e > 0): key limb l of entry slot e of model m at
  // dense_words[dense_base + (e * nl_a0 + l) * M + m], value limb l at
  // dense_words[dense_base + (dense_e * nl_a0 + e * nl_res + l) * M + m]; a model's entries keep
  // their order, slots past its count are never read (the count is entry_ptr's)
  int64_t dense_base;
};
static_assert(sizeof(FuncDev) == 56, "FuncDev layout (gen_qsa.py sub_uf1 reads it)");

struct KArgs {
  // tapes
  const GDesc* descs;
  int n_desc;
  int tapes_per_group;
  const uint32_t* prog;
  const uint32_t* consts;
  const uint32_t* tape_consts;  // unused on host; kept for layout stability
  // models
  const uint32_t* vars;
  const uint32_t* var_off;
  const uint32_t* var_nl;
  int n_vars;
  int n_funcs;
  const FuncDev* funcs;
  const int64_t* entry_ptr;
  const uint32_t* entry_words;
  const uint32_t* else_words;
  int64_t M;
  int64_t index_base;
  // outputs
  int32_t* best;                 // first-hit accumulator (global index, INT32_MAX = none)
  uint8_t* verdicts;             // verdict mode: [tape][M] bytes
  unsigned long long* counters;  // [slot][0] pairs evaluated, [1] node-evals, [2] algorithmic ops
  int tmp_words_per_wave;        // temp words per wave (slot, limb, lane)
  int early_exit;
  uint32_t* scratch;             // per-wave temp slots in HBM: [gridDim.x][tmp_words_per_wave]
  int64_t tiles;                 // model tiles of 64 (one wave = one workgroup)
  int64_t n_items;               // tiles x tape groups; workgroups stride over them
  int grid;                      // workgroups launched (persistent, <= n_items)
  int stack_slots;               // LDS operand-stack slots per wave (max program depth)
  int mode;                      // 0 first hit, 1 verdicts, 2 columns (GDesc.tape = target var)
};

// argument block of the assembly interpreter (layout fixed by gen_qsa.py's prologue)
struct QArgs {
  const void* descs;             // 0x00 GDesc[] (prog_off indexes the QSA program words)
  const void* prog;              // 0x08
  const void* consts;            // 0x10
  const void* vars;              // 0x18
  int32_t* best;                 // 0x20
  unsigned long long* counters;  // 0x28
  uint8_t* verdicts;             // 0x30
  uint32_t* table_out;           // 0x38 (mode 2)
  uint32_t M;                    // 0x40
  uint32_t index_base;           // 0x44
  uint32_t n_desc;               // 0x48
  uint32_t tapes_per_group;      // 0x4c
  uint32_t early_exit;           // 0x50
  uint32_t mode;                 // 0x54: 0 first-hit, 1 verdicts, 2 dump handler offsets
  uint32_t lds_wave_bytes;       // 0x58
  uint32_t pad;                  // 0x5c
  uint32_t var_row[64];          // 0x60: limb row of var v limb l (v < 8), or the zero row
  const void* funcs;             // 0x160 FuncDev[] (G kernel: UF1 lookups)
  const void* entry_ptr;         // 0x168
  const void* entry_words;       // 0x170
  const void* else_words;        // 0x178
  uint32_t n_funcs;              // 0x180
  uint32_t n_stage;              // 0x184 G: model rows staged in LDS per workgroup (multiple of 8)
  uint32_t stage_base;           // 0x188 G: LDS byte offset of the staged rows
  uint32_t bool_rows;            // 0x18c G mode 3: also write Bool columns' 0/1 rows (a C++ kernel reads them)
  const uint32_t* stage_rows;    // 0x190 G: global row of each staged slot
  const uint64_t* bool_masks;    // 0x198 G: packed Bool rows, [tile][n_bool_masks] lane masks
  uint32_t n_bool_masks;         // 0x1a0
  uint32_t reserved_1a4;         // 0x1a4 (unused; keeps the layout the generated code addresses)
  unsigned long long* prof_out;  // 0x1a8 G profile build only: (cycles, count) per handler kind
  const uint32_t* dense_words;   // 0x1b0 G: dense lookup slots (FuncDev dense_base / dense_e)
};
static_assert(sizeof(void*) == 8, "64-bit");
static_assert(__builtin_offsetof(QArgs, M) == 0x40, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, var_row) == 0x60, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, funcs) == 0x160, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, n_funcs) == 0x180, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, n_stage) == 0x184, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, bool_rows) == 0x18c, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, stage_rows) == 0x190, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, bool_masks) == 0x198, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, n_bool_masks) == 0x1a0, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, reserved_1a4) == 0x1a4, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, prof_out) == 0x1a8, "QArgs layout");
static_assert(__builtin_offsetof(QArgs, dense_words) == 0x1b0, "QArgs layout");

// variant 0 = P (preloaded variables, qsa_kernel), 1 = G (general, qsg_kernel)
hipError_t launch_qsa(int variant, const QArgs* d_args, unsigned gx, unsigned gy, size_t lds, hipStream_t st);
hipError_t launch_qs(const KArgs& a, int L, bool keccak, bool verdict, hipStream_t st);
hipError_t launch_columns(const KArgs& a, int L, bool keccak, hipStream_t st);
hipError_t launch_init_best(int32_t* best, int n, hipStream_t st);
hipError_t launch_mask_rows(uint32_t* vars, const uint32_t* rowmask, int64_t rows, int64_t M, hipStream_t st);
// masks[tile * n_masks + j] = lane mask of (vars[rows[j]][64 * tile + i] != 0), for j in list[0..n)
// (list == nullptr: j = 0..n-1)
hipError_t launch_pack_bool(const uint32_t* vars, uint64_t* masks, const uint32_t* rows, const int32_t* list, int n,
                            int n_masks, int64_t M, hipStream_t st);
hipError_t launch_finalize_best(int32_t* best, const uint8_t* unsupported, int n, hipStream_t st);
hipError_t launch_keccak(const uint8_t* data, const int64_t* offsets, int n, uint8_t* out, hipStream_t st);

// Keccak columns (mq_api.cpp kc_*): a hoisted column that is exactly keccak256(concat of model
// variables and constants), evaluated by a dedicated keccak-f[1600] kernel, one model per lane.
// Message word i (little-endian u32 of the big-endian message bytes) = bswap32 of map entry i:
// a variable row (vars[row * M + m]) or, with row == ~0u, the constant word `value`.
struct KcMapEntry {
  uint32_t row;
  uint32_t value;
};
struct KcCol {
  uint32_t map_off;     // first map entry of the column
  uint32_t nwords;      // message words (<= 64: at most 2048 bits, two 136-byte blocks)
  uint32_t target_row;  // first of the 8 rows of the column's variable
  uint32_t n_nodes;     // DAG nodes of the column program (metric; + its predicates')
  uint32_t alg_ops;     // SURVEY §8(d) algorithmic ops of the program (metric; + its predicates')
  uint32_t pred_off;    // its predicate columns (KcPred) evaluated from the digest in registers
  uint32_t n_pred;
  uint32_t pad;
};
// A Bool column comparing a keccak column h with a constant (lower.py keccak_predicates,
// mq_api.cpp kp_match): evaluated by the keccak column kernel right after h
enum KcPredKind : uint32_t { KP_LT = 0, KP_GT = 1, KP_GE = 2, KP_LE = 3, KP_EQ = 4, KP_LOWZ = 5 };
struct KcPred {
  uint32_t kind;        // h < c, h > c, h >= c, h <= c, h == c, low `bits` bits of h zero
  uint32_t bits;        // KP_LOWZ: number of low bits
  uint32_t row;         // the Bool column's variable row (0/1 per model)
  int32_t mask;         // its packed lane-mask index (-1: none)
  uint32_t c[8];        // the constant, limbs little-endian
};
hipError_t launch_keccak_columns(const KcCol* cols, int n_cols, const KcMapEntry* map, const KcPred* preds,
                                 uint32_t* vars, int64_t M, unsigned long long* counters, uint64_t* bool_masks,
                                 int n_bool_masks, int bool_rows, hipStream_t st);

// Bit-gather columns (cw.hip, mq_api.cpp cw_compile): a hoisted column whose value is model
// variable bits and constants, runs of bits optionally gated by `i <s size` (one 256-bit size
// variable per column).  Output limb `limb` = const_or | OR over its slots of
// (((vars[row] >> sb) & mask) << db), a slot whose gate fails giving 0; chunks of one limb are
// consecutive, the last one with store = 1.
struct CwSlot {
  uint32_t row;     // the variable row (a zero row, mask 0: an empty slot)
  uint32_t mask;
  uint32_t shifts;  // sb | db << 8
  uint32_t gate;    // i (< 2^31): the slot counts when i <s size; ~0u: ungated
};
struct CwChunk {
  CwSlot s[4];
  uint32_t limb, store, const_or, pad;
};
struct CwCol {
  uint32_t chunk_off, n_chunks;
  uint32_t target_row;  // limb 0 row of the column's variable
  uint32_t size_row;    // limb 0 row of the size variable (~0u: no gated slots)
  uint32_t n_nodes, alg_ops;   // of the column program (metric)
  uint32_t pad[2];
};
hipError_t launch_cw_columns(const CwCol* cols, int n_cols, const CwChunk* chunks, uint32_t* vars, int64_t M,
                             unsigned long long* counters, hipStream_t st);

// Flat conjunctions (fc.hip, mq_api.cpp fc_match): a tape or Bool column that is an AND of Bool
// model variables (negated or not) and comparisons of one variable with a constant.
struct FcCmpHead {    // (one 32-byte scalar load: all a variable of one or two limbs needs)
  uint32_t slot;      // LDS slot of the variable's limb 0 (limb l at slot + l; padded with zero rows)
  uint32_t nl;        // its limbs (1..8): <= 2 reads two slots, else eight
  uint32_t accept;    // bit 0: x < c, bit 1: x == c, bit 2: x > c (unsigned over the limbs)
  uint32_t pad;
  uint64_t c01;       // the constant's limbs 0-1 (sign bit flipped for a signed compare)
  uint64_t f01;       // XOR-ed into the variable's limbs 0-1: the sign bit of a signed compare
};
struct FcCmpTail {    // limbs 2-7 of a wider variable
  uint32_t c[6];
  uint32_t f[6];
};
struct alignas(16) FcCmp {
  FcCmpHead h;
  FcCmpTail t;
};
struct FcTape {
  uint32_t out;       // modes 0/1: tape index; mode 3: the Bool column's variable row
  int32_t mask_out;   // mode 3: its packed lane-mask index (-1: none, the 0/1 row is written)
  uint32_t mask_off;  // its Bool variables: FcArgs.mask_lds[mask_off ..] = 8 x LDS mask slot | negated,
  uint32_t n_mask;    //   n_mask of them, padded to a multiple of 16 with the last (bit 31: the
                      //   result is negated, an OR of atoms)
  uint32_t cmp_off;   // its compares: FcArgs.cmps[cmp_off ..]
  uint32_t n_cmp;
  uint32_t n_nodes;   // DAG nodes (metric)
  uint32_t alg_ops;   // SURVEY §8(d) algorithmic ops per model (metric)
};
struct FcArgs {
  const FcTape* tapes;
  int n;                         // tapes / columns of the launch
  int tpg;                       // per wave (a workgroup's 4 waves take 4 groups of one tile)
  const uint32_t* mask_lds;
  const FcCmp* cmps;
  const uint32_t* vars;
  const uint64_t* bool_masks;    // [tile][n_bool_masks] packed Bool rows (read)
  uint64_t* bool_masks_out;      // mode 3: the same array, the level's columns written
  uint32_t* vars_out;            // mode 3: 0/1 rows
  int n_bool_masks;
  int mode;                      // 0 first hit, 1 verdict bytes, 3 Bool columns
  int early_exit;
  int bool_rows;                 // mode 3: also write the 0/1 row of a column with a mask index
  int64_t M;
  int64_t index_base;
  int32_t* best;
  uint8_t* verdicts;             // mode 1: [tape][M] bytes
  unsigned long long* counters;
  const uint32_t* stage_rows;    // variable rows staged in LDS per workgroup, slot order
  int n_stage;
  const uint32_t* stage_masks;   // mask indices staged in LDS per workgroup (after the rows)
  int n_smask;
  const unsigned long long* prefix;   // [2 (n + 1)]: running sums of n_nodes, alg_ops
};
// fc_kernel's by-value block (the read-only tables are separate __restrict__ arguments)
struct FcRun {
  int n, tpg, n_bool_masks, mode, early_exit, bool_rows;
  int64_t M, index_base;
  int32_t* best;
  uint8_t* verdicts;
  uint64_t* masks_out;
  uint32_t* vars_out;
  unsigned long long* counters;
  int n_stage, n_smask;
  const unsigned long long* prefix;
};
hipError_t launch_fc(const FcArgs& a, hipStream_t st);

// Two-phase flat conjunctions (fc.hip fca_kernel, mq_api.cpp fca_plan), for tapes: the launch's
// distinct compares ("atoms") are evaluated once per 64-model tile into lane masks in LDS (model
// lanes), grouped by the variable they read (one read of its limbs per group), then every tape
// ANDs its atoms' and Bool variables' masks with one lane per tape.  A workgroup's LDS table per
// tile: entry 0 all ones, 1 .. n_smask the Bool masks, then the atoms; a list entry is a table
// index | negated << 31.
// Unary atoms (round 6): an atom may compare a constant with a UNARY function of its variable —
// a chain of at most kFcMaxXops constant-operand steps (the narrow / sign-extended column reads,
// shifts, extracts and divisions by small constants of C3's path conditions, instructions.py:
// 510-573).  Step k transforms the 8-limb value of width w_in (bits above it zero).
enum FcXcode : uint32_t {
  FX_SEXT = 1,     // p0 = result width
  FX_EXTRACT = 2,  // p0 = lo, p1 = result width
  FX_LSHR = 3,     // p0 = shift (>= w_in: 0)
  FX_SHL = 4,      // p0 = shift (>= w_in: 0)
  FX_ASHR = 5,     // p0 = shift (clamped to w_in - 1)
  FX_UREM = 6,     // p0 = divisor, 0 < d < 2^21
  FX_UDIV = 7,     // p0 = divisor
  FX_SMOD = 8,     // p0 = |divisor|, p1 = divisor negative (SMT-LIB bvsmod)
  FX_SREM = 9,     // p0 = |divisor|, p1 = divisor negative (bvsrem)
  FX_SDIV = 10     // p0 = |divisor|, p1 = divisor negative (bvsdiv)
};
constexpr int kFcMaxXops = 3;
struct FcXop {
  uint32_t code;   // FcXcode | w_in << 8
  uint32_t p0, p1, p2;
};
struct FcXf {      // per atom (FcaArgs.xfs, parallel to atoms); n = 0: the variable itself
  uint32_t n, pad[3];
  FcXop op[kFcMaxXops];
};
struct FcaGroup {
  uint32_t rows[8];   // the variable's limb rows (nl <= 2: rows[0..1]; else 8, the zero row past nl)
  uint32_t first;     // its atoms: atoms[first .. first + count)
  uint32_t count;
  uint32_t nl;
  uint32_t pad;
};
struct FcaArgs {
  int n;                          // tapes
  int n_atoms;
  int n_groups;
  const FcaGroup* groups;
  const FcCmp* atoms;             // accept in {1, 2, 3} (x < c, x == c, x <= c); negations in the lists
  const FcXf* xfs;                // per atom: its unary transform (n = 0: none); groups with one have nl = 8;
                                  // nullptr: no unary atom (the kernel without the transforms)
  const uint32_t* lists;          // chunk c of 64 tapes: kmax(c) entries x 64 lanes, k-major, from chunk_off[c]
  const uint32_t* chunk_off;      // [n_chunks + 1]: kmax(c) = (chunk_off[c + 1] - chunk_off[c]) / 64
  const uint32_t* tape_out;       // per tape: its best / verdict row | negated result << 31
  const uint32_t* tape_metric;    // per tape: n_nodes, alg_ops
  const uint32_t* vars;
  const uint64_t* bool_masks;
  int n_bool_masks;
  int mode;                       // 0 first hit, 1 verdict bytes, 3 Bool columns (tape_out = the column's row)
  int early_exit;
  int64_t M;
  int64_t index_base;
  int32_t* best;
  uint8_t* verdicts;
  unsigned long long* counters;
  const int32_t* col_mask;        // mode 3: per column its packed lane-mask index (-1: none, the 0/1 row is written)
  uint64_t* bool_masks_out;       // mode 3: the same array as bool_masks, the level's columns written
  uint32_t* vars_out;             // mode 3: 0/1 rows
  int bool_rows;                  // mode 3: also write the 0/1 row of a column with a mask index
  const uint32_t* stage_masks;    // the Bool mask indices of table entries 1 .. n_smask
  int n_smask;
};
hipError_t launch_fca(const FcaArgs& a, hipStream_t st);

}  // namespace mq
#endif
