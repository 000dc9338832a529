// tape_compiler.h — boundary tape (mq.h DAG) -> GPU stack program (gprog.h).
#ifndef MQ_TAPE_COMPILER_H
#define MQ_TAPE_COMPILER_H
#include <stdint.h>
#include <string>
#include <vector>
#include "../../include/mq.h"
#include "gprog.h"

namespace mq {

constexpr int kMaxWidth = 2048;   // widest value a tape may hold (64 limbs)

// keccak-f[1600] cost per absorbed 136-byte block in 32-bit ops, counted from the
// permutation's definition in two-input operations with the lane-complementing transform (the
// Keccak team's implementation overview: one NOT per row of chi instead of five), every 64-bit
// lane operation on two 32-bit halves (a 64-bit rotation is two funnel shifts):
//   theta: 20 XOR (column parities) + 5 ROT + 5 XOR (D) + 25 XOR (apply) = 55
//   rho: 24 ROT (lane 0 is not rotated); pi: a lane permutation, no op   = 24
//   chi: 25 AND/OR + 25 XOR + 5 NOT                                      = 55
//   iota: 1 XOR                                                          =  1
// 135 lane ops = 270 32-bit ops per round; 24 rounds = 6 480, + 34 XOR absorbing the block's 17
// lanes = 6 514.  (Round 4 froze the kernel's counted VALU instructions instead, 7 974 per block
// before the v_bitop3 kernel: a count the three-input instructions then beat, 1.17 of the peak.)
constexpr double kKeccakOpsPerBlock = 24.0 * 2.0 * (55 + 24 + 55 + 1) + 34.0;
static_assert(kKeccakOpsPerBlock == 6514.0, "keccak-f[1600] op count");

struct CompiledTape {
  bool supported = false;
  std::string why;               // reason when unsupported
  int L = 0;                     // limbs per value (8, 16, 32 or 64)
  bool keccak = false;           // uses interpreted keccak (G_KECCAK): runs on an L >= 16 keccak kernel
  int depth = 0;                 // max stack slots used
  int n_temps = 0;               // LDS temp slots
  std::vector<uint32_t> prog;    // instruction words, terminated by G_END
  std::vector<uint32_t> consts;  // L-limb padded constants (PUSH_CONST imm indexes this)
  // the program again for the G assembly interpreter (CompileLimits::g_depth slots) when prog
  // needs more: deeper subtrees spilled to temps; empty when prog fits (or spilling failed)
  std::vector<uint32_t> prog_g;
  int depth_g = 0;
  int n_temps_g = 0;
  uint32_t n_nodes = 0;          // DAG size of the boundary tape (metric)
  std::vector<uint32_t> wide_funcs;   // functions looked up by a chunked wide key (MQ_OP_UF_WIDE)
  double alg_ops = 0;            // SURVEY §8(d) algorithmic cost per model
};

struct CompileLimits {
  // LDS operand stack per wave: depth x L x 256 B (L = 8: 2 KB, 16: 4 KB, 32: 8 KB, 64: 16 KB
  // per slot; gfx950 has 160 KB of LDS per CU, so a 2048-bit tape of depth 8 runs one wave per CU)
  int max_depth_l8 = 8;
  int max_depth_l16 = 6;
  int max_depth_l32 = 10;
  int max_depth_l64 = 8;
  // temps live in a per-wave HBM scratch slot (L x 256 B each): 64 x 2 KB, 32 x 4 KB, 32 x 8 KB,
  // 32 x 16 KB (the wide kinds run on a 4x smaller persistent grid, mq_api.cpp make_args)
  int max_temps_l8 = 64;
  int max_temps_l16 = 32;
  int max_temps_l32 = 32;
  int max_temps_l64 = 32;
  int remat_max_nodes = 3;    // shared sub-terms up to this many cheap nodes are re-evaluated
  int g_depth = 0;            // > 0: also build prog_g for a stack of this many slots
  bool value_root = false;    // column program: any BV/Bool root, its value is the result
};

// Compile tape t of the batch. n_funcs/funcs describe the model function table (result
// widths); pass n_funcs = -1 when unknown (UF widths are then taken from the nodes).
CompiledTape compile_tape(const mq_tape_batch* batch, int32_t t, const CompileLimits& lim);

// SURVEY §8(d) algorithmic 32-bit op cost of one evaluation of tape t; -1 if malformed.
double tape_alg_ops(const mq_tape_batch* batch, int32_t t);

}  // namespace mq
#endif
