// gprog.h — the GPU stack-program format produced by the host tape compiler
// (tape_compiler.cpp) and interpreted by the gfx950 kernels (qs_kernels.hip).
//
// A boundary tape (mq.h, a hash-consed DAG) is compiled into straight-line code for a
// register-resident operand stack: every value lives in L u32 limbs (L = 8 for <= 256-bit
// tapes, 16 for <= 512-bit), the stack slot of every operand is known at compile time and is
// carried in the instruction word, so each handler touches statically named VGPRs
// (no dynamic register indexing, no memory traffic for intermediate values).  DAG nodes with
// several users are hoisted: computed once per model into a per-lane LDS temp slot and pushed
// from there at each use.
#ifndef MQ_GPROG_H
#define MQ_GPROG_H
#include <stdint.h>

namespace mq {

// instruction word: op[7:0] | d[11:8] | imm[31:12]
//   push ops:    d = slot written (new top of stack)
//   unary ops:   d = operand slot, result in place
//   binary ops:  operands d-1 (left) and d (right), result in d-1
//   ternary:     operands d-2 (cond), d-1, d; result in d-2
enum GOp : uint32_t {
  G_END = 0,
  G_PUSH_VAR = 1,    // imm = var index
  G_PUSH_CONST = 2,  // imm = word offset from the tape's const base (L limbs, zero padded)
  G_PUSH_TMP = 3,    // imm = temp slot
  G_STORE_TMP = 4,   // imm = temp slot; pops
  G_PUSH_BOOL = 5,   // imm = 0/1
  G_PUSH_VAR_B = 6,  // Bool variable (same as G_PUSH_VAR for the C++ kernel)
  G_PUSH_TMP_B = 7,  // Bool temp
  G_STORE_TMP_B = 8, // Bool temp
  // Bool (limb 0 holds 0/1)
  G_NOT = 10,
  G_AND = 11,
  G_OR = 12,
  G_XOR = 13,
  G_IFF = 14,
  G_IMPLIES = 15,
  G_BITE = 16,
  // BV predicates; imm = operand width
  G_EQ = 20,
  G_ULT = 21,
  G_ULE = 22,
  G_UGT = 23,
  G_UGE = 24,
  G_SLT = 25,
  G_SLE = 26,
  G_SGT = 27,
  G_SGE = 28,
  G_UMUL_NOOVFL = 29,
  G_SMUL_NOOVFL = 30,
  G_SMUL_NOUDFL = 31,
  // BV arithmetic; imm = result width
  G_ADD = 40,
  G_SUB = 41,
  G_MUL = 42,
  G_NEG = 43,
  G_UDIV = 44,
  G_UREM = 45,
  G_SDIV = 46,
  G_SREM = 47,
  G_SMOD = 48,
  G_BAND = 49,
  G_BOR = 50,
  G_BXOR = 51,
  G_BNOT = 52,
  G_SHL = 53,
  G_LSHR = 54,
  G_ASHR = 55,
  G_EXTRACT = 56,    // imm = lo; next word = result width
  G_CONCAT = 57,     // imm = width of the low (right) operand; next word = result width
  G_SEXT = 58,       // imm = source width; next word = result width
  G_ITE = 59,
  G_UF1 = 60,        // imm = function id; result width from the function table
  G_UF2 = 61,
  G_KECCAK = 62,     // imm = argument width (bits, multiple of 8)
  // else-first ternaries: operands d-2 (else), d-1 (cond), d (then); result in d-2.  Chosen by
  // the compiler when the else operand is the deep one (select over a store chain lowers to
  // ite(k == i, v, <rest of the chain>)), so the chain costs O(1) stack slots, not 2 per store.
  G_ITE_EF = 63,
  G_BITE_EF = 9,
  // arity-1 lookup of a key wider than any value, 256 bits at a time (mq.h MQ_OP_UF_CHUNK /
  // MQ_OP_UF_WIDE); imm = function id.  The running value is the set of the model's table
  // entries still matching (a 64-bit mask in limbs 0-1)
  G_UFK0 = 32,       // S[d] = entries whose key chunk 0 equals S[d]; next word = chunk index (0)
  G_UFK = 33,        // S[d-1] = S[d-1] & entries whose key chunk k equals S[d]; next word = k
  G_UFKV = 34,       // S[d] = value of the first entry in the set S[d], else the else value;
                     // next word = result width
  G_NUM_OPS = 64
};

#ifdef __HIPCC__
#define GPROG_HD __host__ __device__
#else
#define GPROG_HD
#endif

// ops followed by a second instruction word (imm2)
GPROG_HD static inline bool has_imm2(uint32_t op) {
  return op == 56 || op == 57 || op == 58 || op == 60 || op == 61 || op == 32 || op == 33 || op == 34;
}

static inline uint32_t gword(uint32_t op, uint32_t d, uint32_t imm) { return op | (d << 8) | (imm << 12); }

// per-tape descriptor (device), 8 x u32
struct GDesc {
  uint32_t prog_off;    // word offset of the program
  uint32_t prog_len;    // words (excluding G_END)
  uint32_t tape;        // index into first_hit
  uint32_t const_base;  // word offset of the tape's constants in the device pool
  uint32_t n_nodes;     // DAG size (metric)
  uint32_t n_temps;
  uint32_t depth;       // max stack depth
  uint32_t alg_ops;     // SURVEY §8(d) algorithmic 32-bit ops per model (metric)
};

constexpr int kMaxImm = (1 << 20) - 1;

}  // namespace mq
#endif
