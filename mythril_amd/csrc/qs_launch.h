// qs_launch.h — kernel argument block and launchers shared by mq_api.cpp and qs_kernels.hip.
#ifndef MQ_QS_LAUNCH_H
#define MQ_QS_LAUNCH_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gprog.h"

namespace mq {

// device view of one model function (UF or as-array interpretation)
struct FuncDev {
  uint32_t arity;
  uint32_t nl_a0, nl_a1, nl_res;
  uint32_t stride;      // words per entry
  uint32_t pad;
  int64_t entry_base;   // word offset of entry 0 in entry_words
  int64_t ptr_base;     // offset of row pointers [M+1] in entry_ptr
  int64_t else_base;    // word offset of the SoA else block: else_words[else_base + limb*M + m]
};

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
  unsigned long long* counters;  // [0] pairs evaluated, [1] node-evals, [2] algorithmic ops
  int tmp_words_per_wave;        // LDS temp words per wave
  int early_exit;
};

hipError_t launch_qs(const KArgs& a, int L, bool verdict, hipStream_t st);
hipError_t launch_init_best(int32_t* best, int n, hipStream_t st);
hipError_t launch_finalize_best(int32_t* best, const uint8_t* unsupported, int n, hipStream_t st);
hipError_t launch_keccak(const uint8_t* data, const int64_t* offsets, int n, uint8_t* out, hipStream_t st);

}  // namespace mq
#endif
