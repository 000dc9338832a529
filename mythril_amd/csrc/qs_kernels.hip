// qs_kernels.hip — gfx950 quick-sat kernels: N constraint tapes x M candidate models.
//
// Replaces the per-model Python/z3 loop of ModelCache.check_quick_sat
// (mythril/support/support_utils.py:60-67): lane = one candidate model (index m), the
// wave runs the SAME compiled tape (wave-uniform instruction stream read through the scalar
// cache, handlers specialized per register-stack slot), and the per-lane Bool verdict is
// reduced with a wave ballot; the lowest satisfying lane is published with an agent-scope
// atomicMin on first_hit[tape] (global candidate index, INT32_MAX = none).  Waves whose first
// model index is already >= the published minimum skip the tape (first-hit early exit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvops.h"
#include "gprog.h"
#include "qs_launch.h"

namespace mq {

// Uniform, read-only-for-the-launch data (programs, constants, descriptors, var/func tables)
// is read through the CONSTANT address space: loads at uniform addresses then lower to
// s_load (scalar cache) instead of global_load + readfirstlane.  Plain global pointers are
// not provably unclobbered here (the kernel also stores: atomicMin, verdicts, LDS temps).
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) GDesc* cdescp;
typedef const __attribute__((address_space(4))) FuncDev* cfuncp;
#define CONSTP(T, p) ((T)(const void*)(p))

template <int L>
struct VecT;
template <>
struct VecT<8> { typedef uint32_t type __attribute__((ext_vector_type(8))); };
template <>
struct VecT<16> { typedef uint32_t type __attribute__((ext_vector_type(16))); };

MQ_DEV GDesc load_desc(const GDesc* descs, int i) {
  cu32p w = CONSTP(cu32p, descs) + (size_t)i * 8;
  GDesc d;
  d.prog_off = w[0];
  d.prog_len = w[1];
  d.tape = w[2];
  d.const_base = w[3];
  d.n_nodes = w[4];
  d.n_temps = w[5];
  d.depth = w[6];
  d.alg_ops = w[7];
  return d;
}

template <int L, int D>
struct Stack {
  typename VecT<L>::type s[D];
};

// Everything a handler may read; built once per wave from the kernel arguments and fully
// scalar-replaced after inlining (uniform fields stay in SGPRs).
struct Ctx {
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
  cu32p consts;            // constants of the current tape
  int64_t m;               // local model index of this lane (clamped to M-1)
  uint32_t* tmp;           // this wave's LDS temp region (slot, limb, lane)
  int lane;
};

MQ_DEV Ctx make_ctx(const KArgs& a, int64_t m, uint32_t* tmp, int lane) {
  Ctx c;
  c.vars = a.vars;
  c.var_off = a.var_off;
  c.var_nl = a.var_nl;
  c.n_vars = a.n_vars;
  c.n_funcs = a.n_funcs;
  c.funcs = a.funcs;
  c.entry_ptr = a.entry_ptr;
  c.entry_words = a.entry_words;
  c.else_words = a.else_words;
  c.M = a.M;
  c.consts = CONSTP(cu32p, a.consts);
  c.m = m;
  c.tmp = tmp;
  c.lane = lane;
  return c;
}

#define H_DEV template <int d> __device__ __forceinline__ static void

// ---------------------------------------------------------------- leaves
template <int L, int D>
struct HPushVar {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t imm, uint32_t, const Ctx& cx) {
    uint32_t nl = 0, off = 0;
    if (imm < (uint32_t)cx.n_vars) {
      off = CONSTP(cu32p, cx.var_off)[imm];
      nl = CONSTP(cu32p, cx.var_nl)[imm];
    }
    const uint32_t* base = cx.vars + (int64_t)off * cx.M + cx.m;
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d][i] = ((uint32_t)i < nl) ? base[(int64_t)i * cx.M] : 0u;
  }
};

template <int L, int D>
struct HPushConst {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t imm, uint32_t, const Ctx& cx) {
    cu32p c = cx.consts + imm;
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d][i] = c[i];
  }
};

template <int L, int D>
struct HPushTmp {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t imm, uint32_t, const Ctx& cx) {
    const uint32_t* p = cx.tmp + (imm * L) * 64 + cx.lane;
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d][i] = p[i * 64];
  }
};

template <int L, int D>
struct HStoreTmp {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t imm, uint32_t, const Ctx& cx) {
    uint32_t* p = cx.tmp + (imm * L) * 64 + cx.lane;
#pragma unroll
    for (int i = 0; i < L; i++) p[i * 64] = S.s[d][i];
  }
};

template <int L, int D>
struct HPushBool {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t imm, uint32_t, const Ctx&) { S.s[d][0] = imm & 1u; }
};

// ---------------------------------------------------------------- Bool connectives (limb 0)
template <int L, int D>
struct HNot {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) { S.s[d][0] ^= 1u; }
};

#define BOOL_BIN(NAME, EXPR)                                                 \
  template <int L, int D>                                                    \
  struct NAME {                                                              \
    static constexpr int kMin = 1;                                           \
    H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {              \
      const uint32_t x = S.s[d - 1][0], y = S.s[d][0];                       \
      S.s[d - 1][0] = (EXPR);                                                \
    }                                                                        \
  };
BOOL_BIN(HAnd, x & y)
BOOL_BIN(HOr, x | y)
BOOL_BIN(HXor, x ^ y)
BOOL_BIN(HIff, (x == y) ? 1u : 0u)
BOOL_BIN(HImplies, (x ^ 1u) | y)

template <int L, int D>
struct HBIte {
  static constexpr int kMin = 2;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {
    S.s[d - 2][0] = S.s[d - 2][0] ? S.s[d - 1][0] : S.s[d][0];
  }
};

// ---------------------------------------------------------------- predicates (imm = operand width)
template <int L, int D>
struct HEq {
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {
    S.s[d - 1][0] = eq_n<L>(S.s[d - 1], S.s[d]) ? 1u : 0u;
  }
};

// kind: 0 ult, 1 ule, 2 ugt, 3 uge ; signed variants flip the sign bits first
template <int L, int D, int KIND, bool SIGNED>
struct HCmpT {
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
    if (SIGNED) {
      sext_full<L>(S.s[d - 1], W);
      sext_full<L>(S.s[d], W);
      S.s[d - 1][L - 1] ^= 0x80000000u;
      S.s[d][L - 1] ^= 0x80000000u;
    }
    bool r;
    if (KIND == 0) r = ult_n<L>(S.s[d - 1], S.s[d]);
    else if (KIND == 1) r = !ult_n<L>(S.s[d], S.s[d - 1]);
    else if (KIND == 2) r = ult_n<L>(S.s[d], S.s[d - 1]);
    else r = !ult_n<L>(S.s[d - 1], S.s[d]);
    S.s[d - 1][0] = r ? 1u : 0u;
  }
};
template <int L, int D> struct HUlt : HCmpT<L, D, 0, false> {};
template <int L, int D> struct HUle : HCmpT<L, D, 1, false> {};
template <int L, int D> struct HUgt : HCmpT<L, D, 2, false> {};
template <int L, int D> struct HUge : HCmpT<L, D, 3, false> {};
template <int L, int D> struct HSlt : HCmpT<L, D, 0, true> {};
template <int L, int D> struct HSle : HCmpT<L, D, 1, true> {};
template <int L, int D> struct HSgt : HCmpT<L, D, 2, true> {};
template <int L, int D> struct HSge : HCmpT<L, D, 3, true> {};

// ---------------------------------------------------------------- arithmetic (imm = result width)
template <int L, int D>
struct HAdd {
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
    add_n<L>(S.s[d - 1], S.s[d - 1], S.s[d]);
    mask_w<L>(S.s[d - 1], W);
  }
};
template <int L, int D>
struct HSub {
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
    (void)sub_n<L>(S.s[d - 1], S.s[d - 1], S.s[d]);
    mask_w<L>(S.s[d - 1], W);
  }
};
template <int L, int D>
struct HMul {
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
    mul_lo_n<L>(S.s[d - 1], S.s[d - 1], S.s[d]);
    mask_w<L>(S.s[d - 1], W);
  }
};
template <int L, int D>
struct HNeg {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
    neg_n<L>(S.s[d]);
    mask_w<L>(S.s[d], W);
  }
};
#define BV_BITWISE(NAME, OP)                                                 \
  template <int L, int D>                                                    \
  struct NAME {                                                              \
    static constexpr int kMin = 1;                                           \
    H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {              \
      _Pragma("unroll") for (int i = 0; i < L; i++) S.s[d - 1][i] OP S.s[d][i]; \
    }                                                                        \
  };
BV_BITWISE(HBAnd, &=)
BV_BITWISE(HBOr, |=)
BV_BITWISE(HBXor, ^=)
template <int L, int D>
struct HBNot {
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t W, uint32_t, const Ctx&) {
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d][i] = ~S.s[d][i];
    mask_w<L>(S.s[d], W);
  }
};
template <int L, int D>
struct HIte {
  static constexpr int kMin = 2;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {
    const bool c = (S.s[d - 2][0] & 1u) != 0;
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d - 2][i] = c ? S.s[d - 1][i] : S.s[d][i];
  }
};
template <int L, int D>
struct HIteEF {  // else at d-2, cond at d-1, then at d
  static constexpr int kMin = 2;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {
    const bool c = (S.s[d - 1][0] & 1u) != 0;
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d - 2][i] = c ? S.s[d][i] : S.s[d - 2][i];
  }
};
template <int L, int D>
struct HBIteEF {
  static constexpr int kMin = 2;
  H_DEV run(Stack<L, D>& S, uint32_t, uint32_t, const Ctx&) {
    S.s[d - 2][0] = S.s[d - 1][0] ? S.s[d][0] : S.s[d - 2][0];
  }
};
template <int L, int D>
struct HExtract {  // imm = lo, imm2 = result width
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t lo, uint32_t W, const Ctx&) {
    shr_uni<L>(S.s[d], lo);
    mask_w<L>(S.s[d], W);
  }
};
template <int L, int D>
struct HConcat {  // imm = low operand width
  static constexpr int kMin = 1;
  H_DEV run(Stack<L, D>& S, uint32_t wl, uint32_t, const Ctx&) {
    shl_uni<L>(S.s[d - 1], wl);
#pragma unroll
    for (int i = 0; i < L; i++) S.s[d - 1][i] |= S.s[d][i];
  }
};
template <int L, int D>
struct HSext {  // imm = source width, imm2 = result width
  static constexpr int kMin = 0;
  H_DEV run(Stack<L, D>& S, uint32_t w0, uint32_t W, const Ctx&) {
    sext_full<L>(S.s[d], w0);
    mask_w<L>(S.s[d], W);
  }
};

// ---------------------------------------------------------------- cold ops: operands copied
// into X/Y, one shared implementation, result copied back (keeps code size bounded).
template <int L, int D, class TX>
MQ_DEV void load_xy(Stack<L, D>& S, int d, TX& X, TX& Y) {
  switch (d) {
#define LXY(k)                                      \
  case k:                                           \
    if constexpr (k >= 1 && k < D) {                \
      _Pragma("unroll") for (int i = 0; i < L; i++) { \
        X[i] = S.s[k - 1][i];                       \
        Y[i] = S.s[k][i];                           \
      }                                             \
    }                                               \
    break;
    LXY(0) LXY(1) LXY(2) LXY(3) LXY(4) LXY(5) LXY(6) LXY(7) LXY(8) LXY(9) LXY(10) LXY(11)
#undef LXY
  }
}
template <int L, int D, class TX>
MQ_DEV void load_x(Stack<L, D>& S, int d, TX& X) {
  switch (d) {
#define LX(k)                                                                   \
  case k:                                                                       \
    if constexpr (k < D) { _Pragma("unroll") for (int i = 0; i < L; i++) X[i] = S.s[k][i]; } \
    break;
    LX(0) LX(1) LX(2) LX(3) LX(4) LX(5) LX(6) LX(7) LX(8) LX(9) LX(10) LX(11)
#undef LX
  }
}
template <int L, int D, class TX>
MQ_DEV void store_x(Stack<L, D>& S, int d, const TX& X) {
  switch (d) {
#define SX(k)                                                                   \
  case k:                                                                       \
    if constexpr (k < D) { _Pragma("unroll") for (int i = 0; i < L; i++) S.s[k][i] = X[i]; } \
    break;
    SX(0) SX(1) SX(2) SX(3) SX(4) SX(5) SX(6) SX(7) SX(8) SX(9) SX(10) SX(11)
#undef SX
  }
}

// table lookup of a model function (UF or as-array): entries first, else value
template <int L, class T0, class T1, class TO>
MQ_DEV void func_lookup(const Ctx& cx, uint32_t f, uint32_t W, const T0& k0, const T1& k1, TO& out) {
#pragma unroll
  for (int i = 0; i < L; i++) out[i] = 0;
  if (f >= (uint32_t)cx.n_funcs) return;
  FuncDev fd;
  {
    cu32p w = CONSTP(cu32p, cx.funcs) + (size_t)f * (sizeof(FuncDev) / 4);
    fd.arity = w[0];
    fd.nl_a0 = w[1];
    fd.nl_a1 = w[2];
    fd.nl_res = w[3];
    fd.stride = w[4];
    fd.entry_base = (int64_t)((uint64_t)w[6] | ((uint64_t)w[7] << 32));
    fd.ptr_base = (int64_t)((uint64_t)w[8] | ((uint64_t)w[9] << 32));
    fd.else_base = (int64_t)((uint64_t)w[10] | ((uint64_t)w[11] << 32));
  }
  const int64_t M = cx.M;
  // else value (SoA, coalesced)
  const uint32_t* ev = cx.else_words + fd.else_base + cx.m;
#pragma unroll
  for (int i = 0; i < L; i++) out[i] = ((uint32_t)i < fd.nl_res) ? ev[(int64_t)i * M] : 0u;
  const int64_t lo = cx.entry_ptr[fd.ptr_base + cx.m], hi = cx.entry_ptr[fd.ptr_base + cx.m + 1];
  for (int64_t e = lo; e < hi; e++) {
    const uint32_t* ent = cx.entry_words + fd.entry_base + e * (int64_t)fd.stride;
    bool match = true;
#pragma unroll
    for (int i = 0; i < L; i++)
      if ((uint32_t)i < fd.nl_a0) match = match && (ent[i] == k0[i]);
    if (fd.arity > 1) {
#pragma unroll
      for (int i = 0; i < L; i++)
        if ((uint32_t)i < fd.nl_a1) match = match && (ent[fd.nl_a0 + i] == k1[i]);
    }
    if (match) {
      const uint32_t* v = ent + fd.nl_a0 + fd.nl_a1;
#pragma unroll
      for (int i = 0; i < L; i++) out[i] = ((uint32_t)i < fd.nl_res) ? v[i] : 0u;
      break;
    }
  }
  mask_w<L>(out, W);
}

// ---------------------------------------------------------------- interpreted keccak256
// keccak256 (Ethereum padding) of the big-endian bytes of S[d] (imm = width in bits, a multiple
// of 8, <= 512 -> one 136-byte block); the digest read big-endian replaces S[d] (256 bits).
// kfm.py:56-69 semantics; only bit-exact with UF table lookup on keccak-consistent models.
__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

MQ_DEV uint64_t krol(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

// state by reference and inlined: the 25 lanes stay in VGPRs (a pointer argument to a
// non-inlined function put them in scratch memory)
MQ_DEV void keccak_f1600(uint64_t (&a)[25]) {
  constexpr int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int r = 0; r < 24; r++) {
    uint64_t C[5], Dd[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; x++) C[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) Dd[x] = C[(x + 4) % 5] ^ krol(C[(x + 1) % 5], 1);
#pragma unroll
    for (int i = 0; i < 25; i++) a[i] ^= Dd[i % 5];
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
      for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = krol(a[x + 5 * y], R[x + 5 * y]);
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++) a[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
    a[0] ^= kKeccakRC[r];
  }
}

template <int L, int D>
MQ_DEV void keccak_op(Stack<L, D>& S, int d, uint32_t W) {
  uint32_t X[L];
  load_x<L, D>(S, d, X);
  const uint32_t nbytes = W >> 3;
  // full-width byte reversal, then shift the message to byte 0: message byte p = LE byte p
  uint32_t R[L];
#pragma unroll
  for (int k = 0; k < L; k++) R[k] = __builtin_bswap32(X[L - 1 - k]);
  shr_uni<L>(R, 8u * (4u * L - nbytes));
  // padding: 0x01 right after the message (bytes >= nbytes are zero after the shift)
#pragma unroll
  for (int k = 0; k < L; k++)
    if ((uint32_t)k == (nbytes >> 2)) R[k] |= 1u << (8u * (nbytes & 3u));
  uint64_t A[25];
#pragma unroll
  for (int w = 0; w < 25; w++) A[w] = (2 * w + 1 < L) ? ((uint64_t)R[2 * w] | ((uint64_t)R[2 * w + 1] << 32)) : 0ull;
  // nbytes == 4L (a 512-bit argument): the 0x01 pad byte is byte 64, outside R
  if (nbytes >= 4u * L) A[nbytes >> 3] |= 1ull << (8u * (nbytes & 7u));
  A[16] |= 0x8000000000000000ull;
  keccak_f1600(A);
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint32_t v = 0;
    if (i < 8) {
      const uint64_t q = A[(7 - i) >> 1];
      v = __builtin_bswap32((uint32_t)(((7 - i) & 1) ? (q >> 32) : q));
    }
    X[i] = v;
  }
  store_x<L, D>(S, d, X);
}

template <int L, int D>
MQ_DEV void cold_op(Stack<L, D>& S, uint32_t op, int d, uint32_t imm, uint32_t imm2, const Ctx& cx) {
  uint32_t X[L], Y[L], R[L];
  if (op == G_UF1) {
    load_x<L, D>(S, d, X);
#pragma unroll
    for (int i = 0; i < L; i++) Y[i] = 0;
    func_lookup<L>(cx, imm, imm2, X, Y, R);
    store_x<L, D>(S, d, R);
    return;
  }
  load_xy<L, D>(S, d, X, Y);
  const uint32_t W = (op == G_UF2) ? imm2 : imm;
  switch (op) {
    case G_UF2:
      func_lookup<L>(cx, imm, imm2, X, Y, R);
      break;
    case G_UDIV:
    case G_UREM: {
      uint32_t Q[L];
      udivrem_n<L>(Q, R, X, Y);
      if (op == G_UDIV) {
#pragma unroll
        for (int i = 0; i < L; i++) R[i] = Q[i];
      }
      mask_w<L>(R, W);
      break;
    }
    case G_SDIV:
    case G_SREM:
    case G_SMOD: {
      sext_full<L>(X, W);
      sext_full<L>(Y, W);
      const bool sa = (X[L - 1] >> 31) != 0, sb = (Y[L - 1] >> 31) != 0;
      uint32_t NA[L], NB[L], Q[L], U[L];
#pragma unroll
      for (int i = 0; i < L; i++) {
        NA[i] = X[i];
        NB[i] = Y[i];
      }
      if (sa) neg_n<L>(NA);  // per-lane: the compiler predicates with exec masks
      if (sb) neg_n<L>(NB);
      udivrem_n<L>(Q, U, NA, NB);
      if (op == G_SDIV) {
#pragma unroll
        for (int i = 0; i < L; i++) R[i] = Q[i];
        if (sa != sb) neg_n<L>(R);
      } else if (op == G_SREM) {
#pragma unroll
        for (int i = 0; i < L; i++) R[i] = U[i];
        if (sa) neg_n<L>(R);
      } else {
        const bool uz = is_zero_n<L>(U);
#pragma unroll
        for (int i = 0; i < L; i++) R[i] = U[i];
        if (!uz) {
          if (sa && !sb) {
            neg_n<L>(R);
            add_n<L>(R, R, Y);
          } else if (!sa && sb) {
            add_n<L>(R, R, Y);
          } else if (sa && sb) {
            neg_n<L>(R);
          }
        }
      }
      mask_w<L>(R, W);
      break;
    }
    case G_SHL: {
      uint32_t s;
      const bool ok = shift_amount<L>(Y, W, s);
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = X[i];
      shl_var<L>(R, ok ? s : 0u);
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = ok ? R[i] : 0u;
      mask_w<L>(R, W);
      break;
    }
    case G_LSHR: {
      uint32_t s;
      const bool ok = shift_amount<L>(Y, W, s);
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = X[i];
      shr_var<L>(R, ok ? s : 0u, 0u);
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = ok ? R[i] : 0u;
      break;
    }
    case G_ASHR: {
      uint32_t s;
      const bool ok = shift_amount<L>(Y, W, s);
      sext_full<L>(X, W);
      const uint32_t fill = (X[L - 1] >> 31) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = X[i];
      shr_var<L>(R, ok ? s : (32u * L - 1u), fill);
      mask_w<L>(R, W);
      break;
    }
    case G_UMUL_NOOVFL: {
      uint32_t LO[L], HI[L];
      mul_full_n<L>(LO, HI, X, Y);
      uint32_t acc = 0;
#pragma unroll
      for (int i = 0; i < L; i++) acc |= HI[i] | (LO[i] & ~limb_mask(i, W));
      R[0] = acc == 0 ? 1u : 0u;
      break;
    }
    case G_SMUL_NOOVFL:
    case G_SMUL_NOUDFL: {
      sext_full<L>(X, W);
      sext_full<L>(Y, W);
      const bool sa = (X[L - 1] >> 31) != 0, sb = (Y[L - 1] >> 31) != 0;
      if (sa) neg_n<L>(X);
      if (sb) neg_n<L>(Y);
      uint32_t LO[L], HI[L];
      mul_full_n<L>(LO, HI, X, Y);
      // compare |p| (2L limbs) with 2^(W-1)
      const uint32_t hb = W - 1, hk = hb >> 5, hbit = 1u << (hb & 31);
      bool gt = false, eq = true;
#pragma unroll
      for (int i = 2 * L - 1; i >= 0; i--) {
        const uint32_t pw = (i < L) ? LO[i] : HI[i - L];
        const uint32_t tw = ((uint32_t)i == hk) ? hbit : 0u;
        gt = eq ? (pw > tw) : gt;
        eq = eq && (pw == tw);
      }
      const bool neg = sa != sb;
      const bool pz = is_zero_n<L>(LO) && is_zero_n<L>(HI);
      bool ok;
      if (op == G_SMUL_NOOVFL) ok = (neg || pz) ? true : (!gt && !eq);
      else ok = (!neg || pz) ? true : !gt;
      R[0] = ok ? 1u : 0u;
      break;
    }
    default:
      break;
  }
  store_x<L, D>(S, d - 1, R);
}

// ---------------------------------------------------------------- dispatch
template <template <int, int> class H, int L, int D>
MQ_DEV void dispatch(Stack<L, D>& S, int d, uint32_t imm, uint32_t imm2, const Ctx& cx) {
  using T = H<L, D>;
  switch (d) {
#define DC(k)                                                           \
  case k:                                                               \
    if constexpr (k >= T::kMin && k < D) T::template run<k>(S, imm, imm2, cx); \
    break;
    DC(0) DC(1) DC(2) DC(3) DC(4) DC(5) DC(6) DC(7) DC(8) DC(9) DC(10) DC(11)
#undef DC
  }
}

template <int L, int D, bool K>
MQ_DEV bool run_tape(cu32p prog, const Ctx& cx) {
  Stack<L, D> S;
#pragma unroll
  for (int k = 0; k < D; k++)
#pragma unroll
    for (int i = 0; i < L; i++) S.s[k][i] = 0;
  uint32_t pc = 0;
  for (;;) {
    const uint32_t ins = prog[pc++];
    const uint32_t op = ins & 0xFFu;
    const int d = (int)((ins >> 8) & 0xFu);
    const uint32_t imm = ins >> 12;
    if (op == G_END) break;
    uint32_t imm2 = 0;
    if (op == G_EXTRACT || op == G_CONCAT || op == G_SEXT || op == G_UF1 || op == G_UF2) imm2 = prog[pc++];
    switch (op) {
      case G_PUSH_VAR:
      case G_PUSH_VAR_B: dispatch<HPushVar, L, D>(S, d, imm, imm2, cx); break;
      case G_PUSH_CONST: dispatch<HPushConst, L, D>(S, d, imm, imm2, cx); break;
      case G_PUSH_TMP:
      case G_PUSH_TMP_B: dispatch<HPushTmp, L, D>(S, d, imm, imm2, cx); break;
      case G_STORE_TMP:
      case G_STORE_TMP_B: dispatch<HStoreTmp, L, D>(S, d, imm, imm2, cx); break;
      case G_PUSH_BOOL: dispatch<HPushBool, L, D>(S, d, imm, imm2, cx); break;
      case G_NOT: dispatch<HNot, L, D>(S, d, imm, imm2, cx); break;
      case G_AND: dispatch<HAnd, L, D>(S, d, imm, imm2, cx); break;
      case G_OR: dispatch<HOr, L, D>(S, d, imm, imm2, cx); break;
      case G_XOR: dispatch<HXor, L, D>(S, d, imm, imm2, cx); break;
      case G_IFF: dispatch<HIff, L, D>(S, d, imm, imm2, cx); break;
      case G_IMPLIES: dispatch<HImplies, L, D>(S, d, imm, imm2, cx); break;
      case G_BITE: dispatch<HBIte, L, D>(S, d, imm, imm2, cx); break;
      case G_EQ: dispatch<HEq, L, D>(S, d, imm, imm2, cx); break;
      case G_ULT: dispatch<HUlt, L, D>(S, d, imm, imm2, cx); break;
      case G_ULE: dispatch<HUle, L, D>(S, d, imm, imm2, cx); break;
      case G_UGT: dispatch<HUgt, L, D>(S, d, imm, imm2, cx); break;
      case G_UGE: dispatch<HUge, L, D>(S, d, imm, imm2, cx); break;
      case G_SLT: dispatch<HSlt, L, D>(S, d, imm, imm2, cx); break;
      case G_SLE: dispatch<HSle, L, D>(S, d, imm, imm2, cx); break;
      case G_SGT: dispatch<HSgt, L, D>(S, d, imm, imm2, cx); break;
      case G_SGE: dispatch<HSge, L, D>(S, d, imm, imm2, cx); break;
      case G_ADD: dispatch<HAdd, L, D>(S, d, imm, imm2, cx); break;
      case G_SUB: dispatch<HSub, L, D>(S, d, imm, imm2, cx); break;
      case G_MUL: dispatch<HMul, L, D>(S, d, imm, imm2, cx); break;
      case G_NEG: dispatch<HNeg, L, D>(S, d, imm, imm2, cx); break;
      case G_BAND: dispatch<HBAnd, L, D>(S, d, imm, imm2, cx); break;
      case G_BOR: dispatch<HBOr, L, D>(S, d, imm, imm2, cx); break;
      case G_BXOR: dispatch<HBXor, L, D>(S, d, imm, imm2, cx); break;
      case G_BNOT: dispatch<HBNot, L, D>(S, d, imm, imm2, cx); break;
      case G_ITE: dispatch<HIte, L, D>(S, d, imm, imm2, cx); break;
      case G_ITE_EF: dispatch<HIteEF, L, D>(S, d, imm, imm2, cx); break;
      case G_BITE_EF: dispatch<HBIteEF, L, D>(S, d, imm, imm2, cx); break;
      case G_EXTRACT: dispatch<HExtract, L, D>(S, d, imm, imm2, cx); break;
      case G_CONCAT: dispatch<HConcat, L, D>(S, d, imm, imm2, cx); break;
      case G_SEXT: dispatch<HSext, L, D>(S, d, imm, imm2, cx); break;
      case G_KECCAK:
        if constexpr (K) keccak_op<L, D>(S, d, imm);
        break;
      default: cold_op<L, D>(S, op, d, imm, imm2, cx); break;
    }
  }
  return (S.s[0][0] & 1u) != 0;
}

// ---------------------------------------------------------------- kernels
// grid.x: model tiles of 64*WAVES models; grid.y: groups of tapes_per_group descriptors.
// Persistent grid: workgroup w handles items w, w + grid, ... with item = group * tiles + tile
// (model tiles of 256 fastest, so low candidate indices are evaluated first and their hits
// feed the early exit).  A wave's temp slots live in HBM at a fixed per-(workgroup, wave)
// offset: coalesced 256-byte rows, L1/L2-resident, no LDS occupancy limit on the temp count.
template <int L, int D, bool K>
__global__ __launch_bounds__(256) void qs_first_hit_kernel(KArgs args) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* tmp = args.scratch + ((size_t)blockIdx.x * 4 + wave) * (size_t)args.tmp_words_per_wave;
  uint64_t pairs = 0, nodes = 0, ops = 0;
  for (int64_t item = blockIdx.x; item < args.n_items; item += gridDim.x) {
    const int64_t tile = item % args.tiles;
    const int group = (int)(item / args.tiles);
    const int64_t m0 = tile * 256 + wave * 64;
    if (m0 >= args.M) continue;
    const int64_t m = m0 + lane;
    const bool valid = m < args.M;
    Ctx cx = make_ctx(args, valid ? m : args.M - 1, tmp, lane);
    const int gbeg = group * args.tapes_per_group;
    const int gend = min(gbeg + args.tapes_per_group, args.n_desc);
    const int32_t gfirst = (int32_t)(args.index_base + m0);
    const uint64_t vmask = __ballot(valid);
    for (int i = gbeg; i < gend; i++) {
      const GDesc dsc = load_desc(args.descs, i);
      int32_t cur = __hip_atomic_load(&args.best[dsc.tape], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      cur = __builtin_amdgcn_readfirstlane(cur);
      if (args.early_exit && gfirst >= cur) continue;
      cx.consts = CONSTP(cu32p, args.consts) + dsc.const_base;
      const bool r = run_tape<L, D, K>(CONSTP(cu32p, args.prog) + dsc.prog_off, cx);
      const uint64_t mask = __ballot(r && valid);
      pairs += __popcll(vmask);
      nodes += (uint64_t)__popcll(vmask) * dsc.n_nodes;
      ops += (uint64_t)__popcll(vmask) * dsc.alg_ops;
      if (mask != 0 && lane == 0) {
        const int32_t hit = (int32_t)(args.index_base + m0 + __builtin_ctzll(mask));
        atomicMin(&args.best[dsc.tape], hit);
      }
    }
  }
  if (lane == 0 && args.counters) {
    atomicAdd(&args.counters[0], (unsigned long long)pairs);
    atomicAdd(&args.counters[1], (unsigned long long)nodes);
    atomicAdd(&args.counters[2], (unsigned long long)ops);
  }
}

template <int L, int D, bool K>
__global__ __launch_bounds__(256) void qs_verdict_kernel(KArgs args) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* tmp = args.scratch + ((size_t)blockIdx.x * 4 + wave) * (size_t)args.tmp_words_per_wave;
  for (int64_t item = blockIdx.x; item < args.n_items; item += gridDim.x) {
    const int64_t tile = item % args.tiles;
    const int group = (int)(item / args.tiles);
    const int64_t m0 = tile * 256 + wave * 64;
    if (m0 >= args.M) continue;
    const int64_t m = m0 + lane;
    const bool valid = m < args.M;
    Ctx cx = make_ctx(args, valid ? m : args.M - 1, tmp, lane);
    const int gbeg = group * args.tapes_per_group;
    const int gend = min(gbeg + args.tapes_per_group, args.n_desc);
    for (int i = gbeg; i < gend; i++) {
      const GDesc dsc = load_desc(args.descs, i);
      cx.consts = CONSTP(cu32p, args.consts) + dsc.const_base;
      const bool r = run_tape<L, D, K>(CONSTP(cu32p, args.prog) + dsc.prog_off, cx);
      if (valid) args.verdicts[(int64_t)dsc.tape * args.M + m] = r ? 1 : 0;
    }
  }
}

__global__ void qs_mask_rows(uint32_t* vars, const uint32_t* rowmask, int64_t rows, int64_t M) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows * M) vars[i] &= rowmask[i / M];
}

hipError_t launch_mask_rows(uint32_t* vars, const uint32_t* rowmask, int64_t rows, int64_t M, hipStream_t st) {
  const int64_t n = rows * M;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(qs_mask_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, vars, rowmask, rows, M);
  return hipGetLastError();
}

__global__ void qs_init_best(int32_t* best, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) best[i] = 0x7FFFFFFF;
}

__global__ void qs_finalize_best(int32_t* best, const uint8_t* unsupported, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int32_t b = best[i];
    best[i] = unsupported[i] ? -2 : (b == 0x7FFFFFFF ? -1 : b);
  }
}

// ---------------------------------------------------------------- host launchers
template <int L, int D, bool K>
static hipError_t launch_variant(const KArgs& a, bool verdict, hipStream_t st) {
  if (a.n_desc <= 0 || a.grid <= 0) return hipSuccess;
  if (verdict) hipLaunchKernelGGL((qs_verdict_kernel<L, D, K>), dim3((unsigned)a.grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((qs_first_hit_kernel<L, D, K>), dim3((unsigned)a.grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_qs(const KArgs& a, int L, bool keccak, bool verdict, hipStream_t st) {
  if (keccak) return L == 16 ? launch_variant<16, 6, true>(a, verdict, st) : hipErrorInvalidValue;
  if (L == 8) return launch_variant<8, 8, false>(a, verdict, st);
  if (L == 16) return launch_variant<16, 6, false>(a, verdict, st);
  return hipErrorInvalidValue;
}

hipError_t launch_init_best(int32_t* best, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(qs_init_best, dim3((n + 255) / 256), dim3(256), 0, st, best, n);
  return hipGetLastError();
}

hipError_t launch_finalize_best(int32_t* best, const uint8_t* unsupported, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(qs_finalize_best, dim3((n + 255) / 256), dim3(256), 0, st, best, unsupported, n);
  return hipGetLastError();
}

}  // namespace mq
