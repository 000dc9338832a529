// qs_kernels.hip — gfx950 quick-sat kernels (general vocabulary): N constraint tapes x M models.
//
// Replaces the per-model Python/z3 loop of ModelCache.check_quick_sat
// (mythril/support/support_utils.py:60-67): lane = one candidate model (index m), the wave
// runs the SAME compiled tape (wave-uniform instruction stream read through the scalar cache),
// and the per-lane Bool verdict is reduced with a wave ballot; the lowest satisfying lane is
// published with an agent-scope atomicMin on first_hit[tape] (global candidate index,
// INT32_MAX = none).  Waves whose first model index is already >= the published minimum skip
// the tape (first-hit early exit).
//
// Operand stack in LDS.  The straight-line stack programs of gprog.h address stack slots by a
// runtime (wave-uniform) depth d.  A register-resident stack forced a per-slot specialisation of
// every handler, and the switch joins of that dispatch made the register allocator copy the
// whole stack around each node (~440 VALU per node measured with rocprofv3 on the C3 workload,
// profiles/r01_c3_pmc.json).  Here slot d lives in LDS at a uniform offset; a handler reads its
// operands into registers, computes, and writes the canonical result back, so nothing is live
// across the dispatch.  Layout per wave: [slot][limb group of 4][lane] of uint4, i.e.
// ds_read_b128 / ds_write_b128 with consecutive lanes on consecutive 16-byte words (no bank
// conflicts).  Every slot holds a canonical L-limb value (zeros above its width), so a reader
// may skip limb groups above its operand width, and values <= 32 bits take 1-limb fast paths.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvops.h"
#include "gprog.h"
#include "qs_launch.h"

namespace mq {

typedef const __attribute__((address_space(4))) uint32_t* cu32p;
#define CONSTP(T, p) ((T)(const void*)(p))

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

// Everything a handler may read; uniform fields stay in SGPRs.
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
  uint32_t* tmp;           // this wave's temp slots in HBM (slot, limb, lane)
  uint4* stk;              // this wave's LDS operand stack, offset by the lane
  int lane;
};

MQ_DEV Ctx make_ctx(const KArgs& a, int64_t m, uint32_t* tmp, uint4* stk, int lane) {
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
  c.stk = stk + lane;
  c.lane = lane;
  return c;
}

MQ_DEV uint32_t nl_of_w(uint32_t W) { return W == 0 ? 1u : (W + 31u) >> 5; }

// ---------------------------------------------------------------- LDS stack access
// Multiplication, division and the multiplication-overflow predicates work on at most
// kArithLimbs limbs (512 bits): the tape compiler rejects them wider, so on the 1024/2048-bit
// stacks (L = 32, 64: wide Concat / Extract / EQ / ITE / UF keys / keccak inputs) they read
// and write only the low limbs of a slot and keep the register footprint of L = 16.
constexpr int kArithLimbs = 16;
template <int L>
constexpr int arith_limbs() { return L > kArithLimbs ? kArithLimbs : L; }

// the low A limbs of slot d (A <= L, a multiple of 4); limb groups at or above nl read as zero
template <int L, int A>
MQ_DEV void sld_a(const Ctx& cx, int d, uint32_t (&x)[A], uint32_t nl = A) {
  const uint4* p = cx.stk + (d * (L / 4)) * 64;
#pragma unroll
  for (int g = 0; g < A / 4; g++) {
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (g == 0 || (uint32_t)(4 * g) < nl) v = p[g * 64];
    x[4 * g] = v.x;
    x[4 * g + 1] = v.y;
    x[4 * g + 2] = v.z;
    x[4 * g + 3] = v.w;
  }
}
// write A limbs into slot d and zero its limbs above them (slots stay canonical)
template <int L, int A>
MQ_DEV void sst_a(const Ctx& cx, int d, const uint32_t (&x)[A]) {
  uint4* p = cx.stk + (d * (L / 4)) * 64;
#pragma unroll
  for (int g = 0; g < A / 4; g++) p[g * 64] = make_uint4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
#pragma unroll
  for (int g = A / 4; g < L / 4; g++) p[g * 64] = make_uint4(0u, 0u, 0u, 0u);
}
template <int L>
MQ_DEV void sld(const Ctx& cx, int d, uint32_t (&x)[L], uint32_t nl = L) {
  sld_a<L, L>(cx, d, x, nl);
}
template <int L>
MQ_DEV void sst(const Ctx& cx, int d, const uint32_t (&x)[L]) {
  sst_a<L, L>(cx, d, x);
}
template <int L>
MQ_DEV uint32_t sld0(const Ctx& cx, int d) {
  return reinterpret_cast<const uint32_t*>(cx.stk + (d * (L / 4)) * 64)[0];
}
// a value of at most 32 bits: limb 0, zeros above (keeps the slot canonical)
template <int L>
MQ_DEV void sst0(const Ctx& cx, int d, uint32_t v) {
  uint4* p = cx.stk + (d * (L / 4)) * 64;
  p[0] = make_uint4(v, 0u, 0u, 0u);
#pragma unroll
  for (int g = 1; g < L / 4; g++) p[g * 64] = make_uint4(0u, 0u, 0u, 0u);
}
// Bool results: limb 0 only.  Bool slots are only ever read through limb 0 (Bool connectives,
// ite conditions, temps copy all limbs but their Bool readers again look at limb 0).
template <int L>
MQ_DEV void sstb(const Ctx& cx, int d, bool b) {
  reinterpret_cast<uint32_t*>(cx.stk + (d * (L / 4)) * 64)[0] = b ? 1u : 0u;
}

MQ_DEV uint32_t mask32(uint32_t W) { return W >= 32u ? 0xFFFFFFFFu : ((1u << W) - 1u); }

// ---------------------------------------------------------------- leaves
template <int L>
MQ_DEV void h_push_var(const Ctx& cx, int d, uint32_t imm) {
  uint32_t nl = 0, off = 0;
  if (imm < (uint32_t)cx.n_vars) {
    off = CONSTP(cu32p, cx.var_off)[imm];
    nl = CONSTP(cu32p, cx.var_nl)[imm];
  }
  const uint32_t* base = cx.vars + (int64_t)off * cx.M + cx.m;
  if (nl == 1) {
    sst0<L>(cx, d, base[0]);
    return;
  }
  uint32_t x[L];
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = ((uint32_t)i < nl) ? base[(int64_t)i * cx.M] : 0u;
  sst<L>(cx, d, x);
}

template <int L>
MQ_DEV void h_push_const(const Ctx& cx, int d, uint32_t imm) {
  cu32p c = cx.consts + imm;
  uint32_t x[L];
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = c[i];
  sst<L>(cx, d, x);
}

template <int L>
MQ_DEV void h_push_tmp(const Ctx& cx, int d, uint32_t imm) {
  const uint32_t* p = cx.tmp + (imm * L) * 64 + cx.lane;
  uint32_t x[L];
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = p[i * 64];
  sst<L>(cx, d, x);
}

template <int L>
MQ_DEV void h_store_tmp(const Ctx& cx, int d, uint32_t imm) {
  uint32_t x[L];
  sld<L>(cx, d, x);
  uint32_t* p = cx.tmp + (imm * L) * 64 + cx.lane;
#pragma unroll
  for (int i = 0; i < L; i++) p[i * 64] = x[i];
}

// ---------------------------------------------------------------- predicates (W = operand width)
template <int L>
MQ_DEV void h_eq(const Ctx& cx, int d, uint32_t W) {
  if (W <= 32u) {
    sstb<L>(cx, d - 1, sld0<L>(cx, d - 1) == sld0<L>(cx, d));
    return;
  }
  const uint32_t nl = nl_of_w(W);
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x, nl);
  sld<L>(cx, d, y, nl);
  sstb<L>(cx, d - 1, eq_n<L>(x, y));
}

// kind: 0 ult, 1 ule, 2 ugt, 3 uge ; signed compares flip the sign bit at W-1 first
template <int L>
MQ_DEV void h_cmp(const Ctx& cx, int d, uint32_t W, int kind, bool sgn) {
  if (W <= 32u) {
    uint32_t a = sld0<L>(cx, d - 1), b = sld0<L>(cx, d);
    if (sgn) {
      const uint32_t sb = 1u << (W - 1u);
      a ^= sb;
      b ^= sb;
    }
    const bool r = kind == 0 ? a < b : kind == 1 ? a <= b : kind == 2 ? a > b : a >= b;
    sstb<L>(cx, d - 1, r);
    return;
  }
  const uint32_t nl = nl_of_w(W);
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x, nl);
  sld<L>(cx, d, y, nl);
  if (sgn) {
    sext_full<L>(x, W);
    sext_full<L>(y, W);
    x[L - 1] ^= 0x80000000u;
    y[L - 1] ^= 0x80000000u;
  }
  bool r;
  if (kind == 0) r = ult_n<L>(x, y);
  else if (kind == 1) r = !ult_n<L>(y, x);
  else if (kind == 2) r = ult_n<L>(y, x);
  else r = !ult_n<L>(x, y);
  sstb<L>(cx, d - 1, r);
}

// ---------------------------------------------------------------- arithmetic (W = result width)
template <int L>
MQ_DEV void h_add_sub(const Ctx& cx, int d, uint32_t W, bool sub) {
  if (W <= 32u) {
    const uint32_t a = sld0<L>(cx, d - 1), b = sld0<L>(cx, d);
    sst0<L>(cx, d - 1, (sub ? a - b : a + b) & mask32(W));
    return;
  }
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x);
  sld<L>(cx, d, y);
  if (sub) (void)sub_n<L>(x, x, y);
  else add_n<L>(x, x, y);
  mask_w<L>(x, W);
  sst<L>(cx, d - 1, x);
}

template <int L>
MQ_DEV void h_mul(const Ctx& cx, int d, uint32_t W) {
  if (W <= 32u) {
    sst0<L>(cx, d - 1, (sld0<L>(cx, d - 1) * sld0<L>(cx, d)) & mask32(W));
    return;
  }
  constexpr int A = arith_limbs<L>();
  uint32_t x[A], y[A], r[A];
  sld_a<L, A>(cx, d - 1, x);
  sld_a<L, A>(cx, d, y);
  mul_lo_n<A>(r, x, y);
  mask_w<A>(r, W);
  sst_a<L, A>(cx, d - 1, r);
}

template <int L>
MQ_DEV void h_neg_not(const Ctx& cx, int d, uint32_t W, bool is_not) {
  if (W <= 32u) {
    const uint32_t a = sld0<L>(cx, d);
    sst0<L>(cx, d, (is_not ? ~a : 0u - a) & mask32(W));
    return;
  }
  uint32_t x[L];
  sld<L>(cx, d, x);
  if (is_not) {
#pragma unroll
    for (int i = 0; i < L; i++) x[i] = ~x[i];
  } else {
    neg_n<L>(x);
  }
  mask_w<L>(x, W);
  sst<L>(cx, d, x);
}

// bitwise: 0 and, 1 or, 2 xor
template <int L>
MQ_DEV void h_bitwise(const Ctx& cx, int d, uint32_t W, int kind) {
  if (W <= 32u) {
    const uint32_t a = sld0<L>(cx, d - 1), b = sld0<L>(cx, d);
    sst0<L>(cx, d - 1, kind == 0 ? (a & b) : kind == 1 ? (a | b) : (a ^ b));
    return;
  }
  const uint32_t nl = nl_of_w(W);
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x, nl);
  sld<L>(cx, d, y, nl);
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = kind == 0 ? (x[i] & y[i]) : kind == 1 ? (x[i] | y[i]) : (x[i] ^ y[i]);
  sst<L>(cx, d - 1, x);
}

// ite: cond at slot c, then at t, else at e, result to r
template <int L>
MQ_DEV void h_ite(const Ctx& cx, int c, int t, int e, int r, uint32_t W) {
  const bool cond = (sld0<L>(cx, c) & 1u) != 0;
  if (W <= 32u) {
    const uint32_t a = sld0<L>(cx, t), b = sld0<L>(cx, e);
    sst0<L>(cx, r, cond ? a : b);
    return;
  }
  const uint32_t nl = nl_of_w(W);
  uint32_t x[L], y[L];
  sld<L>(cx, t, x, nl);
  sld<L>(cx, e, y, nl);
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = cond ? x[i] : y[i];
  sst<L>(cx, r, x);
}

template <int L>
MQ_DEV void h_extract(const Ctx& cx, int d, uint32_t lo, uint32_t W) {
  if (lo + W <= 32u) {
    sst0<L>(cx, d, (sld0<L>(cx, d) >> lo) & mask32(W));
    return;
  }
  uint32_t x[L];
  sld<L>(cx, d, x, nl_of_w(lo + W));
  shr_uni<L>(x, lo);
  mask_w<L>(x, W);
  sst<L>(cx, d, x);
}

template <int L>
MQ_DEV void h_concat(const Ctx& cx, int d, uint32_t wl, uint32_t W) {
  if (W <= 32u) {
    sst0<L>(cx, d - 1, (sld0<L>(cx, d - 1) << wl) | sld0<L>(cx, d));
    return;
  }
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x, nl_of_w(W - wl));
  sld<L>(cx, d, y, nl_of_w(wl));
  shl_uni<L>(x, wl);
#pragma unroll
  for (int i = 0; i < L; i++) x[i] |= y[i];
  sst<L>(cx, d - 1, x);
}

template <int L>
MQ_DEV void h_sext(const Ctx& cx, int d, uint32_t w0, uint32_t W) {
  uint32_t x[L];
  sld<L>(cx, d, x, nl_of_w(w0));
  sext_full<L>(x, w0);
  mask_w<L>(x, W);
  sst<L>(cx, d, x);
}

// ---------------------------------------------------------------- division
// per-lane bit length of a canonical value
template <int L>
MQ_DEV uint32_t bitlen_n(const uint32_t (&a)[L]) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r = a[i] ? 32u * i + 32u - (uint32_t)__clz(a[i]) : r;
  return r;
}

// q = a / b, r = a % b (unsigned, full 32L bits); b == 0 -> q = all ones, r = a (SMT-LIB).
// Divisors < 2^32 in every lane: schoolbook 64/32 long division (L steps).  Otherwise
// restoring division over only the quotient's bit length (bitlen(a) - bitlen(b) + 1 steps,
// the wave's maximum), with the divisor pre-aligned to the dividend's top bit.
template <int L>
MQ_DEV void udivrem_fast(uint32_t (&q)[L], uint32_t (&r)[L], const uint32_t (&a)[L], const uint32_t (&b)[L]) {
  const bool bz = is_zero_n<L>(b);
  uint32_t bhi = 0;
#pragma unroll
  for (int i = 1; i < L; i++) bhi |= b[i];
  if (__ballot(bhi != 0u) == 0) {
    const uint32_t dv = bz ? 1u : b[0];
    uint32_t rem = 0;
#pragma unroll
    for (int i = L - 1; i >= 0; i--) {
      const uint64_t n = ((uint64_t)rem << 32) | a[i];
      const uint64_t qq = n / dv;
      q[i] = (uint32_t)qq;
      rem = (uint32_t)(n - qq * dv);
    }
#pragma unroll
    for (int i = 0; i < L; i++) r[i] = i == 0 ? rem : 0u;
  } else {
    const int la = (int)bitlen_n<L>(a), lb = (int)bitlen_n<L>(b);
    const int k = bz ? -1 : la - lb;  // the quotient has at most k+1 bits
    uint32_t bs[L];
#pragma unroll
    for (int i = 0; i < L; i++) {
      bs[i] = b[i];
      q[i] = 0;
      r[i] = a[i];
    }
    shl_var<L>(bs, k > 0 ? (uint32_t)k : 0u);
    for (int it = 0; __ballot(it <= k) != 0; it++) {
      if (it <= k) {
        uint32_t t[L];
        const uint32_t borrow = sub_n<L>(t, r, bs);
        const uint32_t bit = (uint32_t)(k - it);
        if (!borrow) {
#pragma unroll
          for (int i = 0; i < L; i++) {
            r[i] = t[i];
            q[i] |= ((uint32_t)i == (bit >> 5)) ? (1u << (bit & 31u)) : 0u;
          }
        }
#pragma unroll
        for (int i = 0; i < L; i++) bs[i] = __builtin_amdgcn_alignbit(i + 1 < L ? bs[i + 1] : 0u, bs[i], 1u);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < L; i++) {
    q[i] = bz ? 0xFFFFFFFFu : q[i];
    r[i] = bz ? a[i] : r[i];
  }
}

template <int Ls>
MQ_DEV void h_div(const Ctx& cx, int d, uint32_t op, uint32_t W) {
  constexpr int L = arith_limbs<Ls>();   // (the tape compiler keeps divisions <= 512 bits)
  uint32_t x[L], y[L], Q[L], R[L];
  const uint32_t nl = nl_of_w(W);
  sld_a<Ls, L>(cx, d - 1, x, nl);
  sld_a<Ls, L>(cx, d, y, nl);
  if (op == G_UDIV || op == G_UREM) {
    udivrem_fast<L>(Q, R, x, y);
    if (op == G_UDIV) {
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = Q[i];
    }
    mask_w<L>(R, W);
    sst_a<Ls, L>(cx, d - 1, R);
    return;
  }
  sext_full<L>(x, W);
  sext_full<L>(y, W);
  const bool sa = (x[L - 1] >> 31) != 0, sb = (y[L - 1] >> 31) != 0;
  uint32_t NA[L], NB[L];
#pragma unroll
  for (int i = 0; i < L; i++) {
    NA[i] = x[i];
    NB[i] = y[i];
  }
  if (sa) neg_n<L>(NA);
  if (sb) neg_n<L>(NB);
  udivrem_fast<L>(Q, R, NA, NB);
  if (op == G_SDIV) {
#pragma unroll
    for (int i = 0; i < L; i++) R[i] = Q[i];
    if (sa != sb) neg_n<L>(R);
  } else if (op == G_SREM) {
    if (sa) neg_n<L>(R);
  } else {  // smod: sign of the divisor
    if (!is_zero_n<L>(R)) {
      if (sa && !sb) {
        neg_n<L>(R);
        add_n<L>(R, R, y);
      } else if (!sa && sb) {
        add_n<L>(R, R, y);
      } else if (sa && sb) {
        neg_n<L>(R);
      }
    }
  }
  mask_w<L>(R, W);
  sst_a<Ls, L>(cx, d - 1, R);
}

// ---------------------------------------------------------------- shifts by a stack value
template <int L>
MQ_DEV void h_shift(const Ctx& cx, int d, uint32_t op, uint32_t W) {
  const uint32_t nl = nl_of_w(W);
  uint32_t x[L], y[L];
  sld<L>(cx, d - 1, x, nl);
  sld<L>(cx, d, y, nl);
  uint32_t s;
  const bool ok = shift_amount<L>(y, W, s);
  if (op == G_SHL) {
    shl_var<L>(x, ok ? s : 0u);
#pragma unroll
    for (int i = 0; i < L; i++) x[i] = ok ? x[i] : 0u;
    mask_w<L>(x, W);
  } else if (op == G_LSHR) {
    shr_var<L>(x, ok ? s : 0u, 0u);
#pragma unroll
    for (int i = 0; i < L; i++) x[i] = ok ? x[i] : 0u;
  } else {
    sext_full<L>(x, W);
    const uint32_t fill = (x[L - 1] >> 31) ? 0xFFFFFFFFu : 0u;
    shr_var<L>(x, ok ? s : (32u * L - 1u), fill);
    mask_w<L>(x, W);
  }
  sst<L>(cx, d - 1, x);
}

// ---------------------------------------------------------------- overflow predicates
template <int Ls>
MQ_DEV void h_mul_ovfl(const Ctx& cx, int d, uint32_t op, uint32_t W) {
  constexpr int L = arith_limbs<Ls>();   // (operands <= 512 bits, tape compiler)
  uint32_t X[L], Y[L];
  sld_a<Ls, L>(cx, d - 1, X);
  sld_a<Ls, L>(cx, d, Y);
  uint32_t LO[L], HI[L];
  bool res;
  if (op == G_UMUL_NOOVFL) {
    mul_full_n<L>(LO, HI, X, Y);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < L; i++) acc |= HI[i] | (LO[i] & ~limb_mask(i, W));
    res = acc == 0;
  } else {
    sext_full<L>(X, W);
    sext_full<L>(Y, W);
    const bool sa = (X[L - 1] >> 31) != 0, sb = (Y[L - 1] >> 31) != 0;
    if (sa) neg_n<L>(X);
    if (sb) neg_n<L>(Y);
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
    if (op == G_SMUL_NOOVFL) res = (neg || pz) ? true : (!gt && !eq);
    else res = (!neg || pz) ? true : !gt;
  }
  sstb<Ls>(cx, d - 1, res);
}

// ---------------------------------------------------------------- model functions
// table lookup of a model function (UF or as-array): entries first, else value
template <int L>
MQ_DEV void func_lookup(const Ctx& cx, uint32_t f, uint32_t W, const uint32_t (&k0)[L], const uint32_t (&k1)[L],
                        uint32_t (&out)[L]) {
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
  mask_w<L>(out, W == 0 ? 1u : W);  // Bool range: limb 0 holds 0/1
}

// the function descriptor of f (qs_launch.h FuncDev); false if f is out of range
MQ_DEV bool load_func(const Ctx& cx, uint32_t f, FuncDev& fd) {
  if (f >= (uint32_t)cx.n_funcs) return false;
  cu32p w = CONSTP(cu32p, cx.funcs) + (size_t)f * (sizeof(FuncDev) / 4);
  fd.arity = w[0];
  fd.nl_a0 = w[1];
  fd.nl_a1 = w[2];
  fd.nl_res = w[3];
  fd.stride = w[4];
  fd.entry_base = (int64_t)((uint64_t)w[6] | ((uint64_t)w[7] << 32));
  fd.ptr_base = (int64_t)((uint64_t)w[8] | ((uint64_t)w[9] << 32));
  fd.else_base = (int64_t)((uint64_t)w[10] | ((uint64_t)w[11] << 32));
  return true;
}

// wide-key lookup, one 256-bit key chunk k at a time (mq.h MQ_OP_UF_CHUNK): the set of this
// model's entries of f (bit e = entry e; the host guarantees at most 64 entries per model) whose
// key limbs [8k, 8k + 8) equal the chunk, within the set so far (G_UFK) or all entries (G_UFK0)
template <int L>
MQ_DEV void h_ufk(const Ctx& cx, int d, uint32_t op, uint32_t f, uint32_t k) {
  uint32_t X[L];
  sld<L>(cx, d, X);
  const int out = op == G_UFK0 ? d : d - 1;
  uint64_t mask = 0;
  FuncDev fd;
  if (load_func(cx, f, fd) && fd.arity == 1) {
    const int64_t lo = cx.entry_ptr[fd.ptr_base + cx.m], hi = cx.entry_ptr[fd.ptr_base + cx.m + 1];
    const int64_t E = min<int64_t>(hi - lo, 64);
    if (op == G_UFK0) {
      mask = E >= 64 ? ~0ull : ((1ull << E) - 1ull);
    } else {
      uint32_t P[L];
      sld<L>(cx, d - 1, P);
      mask = (uint64_t)P[0] | ((uint64_t)P[1] << 32);
    }
    const int nk = (int)fd.nl_a0 - 8 * (int)k;   // key limbs in this chunk (the last may be short)
    if (nk <= 0) mask = 0;
    for (int64_t e = 0; e < E && mask; e++) {
      if (!((mask >> e) & 1ull)) continue;
      const uint32_t* ent = cx.entry_words + fd.entry_base + (lo + e) * (int64_t)fd.stride + 8 * k;
      bool eq = true;
#pragma unroll
      for (int i = 0; i < 8 && i < L; i++)
        if (i < nk) eq = eq && ent[i] == X[i];
      if (!eq) mask &= ~(1ull << e);
    }
  }
  uint32_t R[L];
#pragma unroll
  for (int i = 0; i < L; i++) R[i] = i == 0 ? (uint32_t)mask : i == 1 ? (uint32_t)(mask >> 32) : 0u;
  sst<L>(cx, out, R);
}

// the value of the first entry of the set S[d] (mq.h MQ_OP_UF_WIDE), or f's else value
template <int L>
MQ_DEV void h_ufkv(const Ctx& cx, int d, uint32_t f, uint32_t W) {
  uint32_t P[L], R[L];
  sld<L>(cx, d, P);
  const uint64_t mask = (uint64_t)P[0] | ((uint64_t)P[1] << 32);
#pragma unroll
  for (int i = 0; i < L; i++) R[i] = 0;
  FuncDev fd;
  if (load_func(cx, f, fd)) {
    const int64_t M = cx.M;
    const uint32_t* ev = cx.else_words + fd.else_base + cx.m;
#pragma unroll
    for (int i = 0; i < L; i++) R[i] = ((uint32_t)i < fd.nl_res) ? ev[(int64_t)i * M] : 0u;
    if (mask) {
      const int64_t lo = cx.entry_ptr[fd.ptr_base + cx.m];
      const int e = __builtin_ctzll(mask);
      const uint32_t* v = cx.entry_words + fd.entry_base + (lo + e) * (int64_t)fd.stride + fd.nl_a0;
#pragma unroll
      for (int i = 0; i < L; i++) R[i] = ((uint32_t)i < fd.nl_res) ? v[i] : 0u;
    }
  }
  mask_w<L>(R, W == 0 ? 1u : W);
  sst<L>(cx, d, R);
}

template <int L>
MQ_DEV void h_uf(const Ctx& cx, int d, uint32_t op, uint32_t f, uint32_t W) {
  uint32_t X[L], Y[L], R[L];
  if (op == G_UF1) {
    sld<L>(cx, d, X);
#pragma unroll
    for (int i = 0; i < L; i++) Y[i] = 0;
    func_lookup<L>(cx, f, W, X, Y, R);
    sst<L>(cx, d, R);
  } else {
    sld<L>(cx, d - 1, X);
    sld<L>(cx, d, Y);
    func_lookup<L>(cx, f, W, X, Y, R);
    sst<L>(cx, d - 1, R);
  }
}

// ---------------------------------------------------------------- interpreted keccak256
// keccak256 (Ethereum padding) of the big-endian bytes of S[d] (imm = width in bits, a multiple
// of 8, at most 32L bits: one 136-byte block up to 1080 bits, two up to 2048); the digest read
// big-endian replaces S[d] (256 bits).  kfm.py:56-69 semantics; only bit-exact with UF table
// lookup on keccak-consistent models.
__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

MQ_DEV uint64_t krol(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

// state by reference and inlined: the 25 lanes stay in VGPRs
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

template <int L>
MQ_DEV void h_keccak(const Ctx& cx, int d, uint32_t W) {
  uint32_t X[L];
  sld<L>(cx, d, X);
  const uint32_t nbytes = W >> 3;
  // full-width byte reversal, then shift the message to byte 0: message byte p = LE byte p of R
  // (bytes >= nbytes are zero)
  uint32_t R[L];
#pragma unroll
  for (int k = 0; k < L; k++) R[k] = __builtin_bswap32(X[L - 1 - k]);
  shr_uni<L>(R, 8u * (4u * L - nbytes));
  // absorb: block b holds message bytes [136 b, 136 b + 136) = R words 34 b .. 34 b + 33; the
  // final block carries the 0x01 pad byte at message position nbytes and 0x80 in its last byte
  constexpr int kMaxBlocks = (4 * L) / 136 + 1;
  const uint32_t nblocks = nbytes / 136u + 1u;   // uniform
  uint64_t A[25];
#pragma unroll
  for (int w = 0; w < 25; w++) A[w] = 0ull;
#pragma unroll
  for (int b = 0; b < kMaxBlocks; b++) {
    if ((uint32_t)b >= nblocks) break;
#pragma unroll
    for (int w = 0; w < 17; w++) {
      const int i0 = 34 * b + 2 * w;
      uint64_t lane = 0ull;
      if (i0 < L) lane = R[i0];
      if (i0 + 1 < L) lane |= (uint64_t)R[i0 + 1] << 32;
      A[w] ^= lane;
    }
    if ((uint32_t)b == nblocks - 1u) {
      const uint32_t pp = nbytes - 136u * (uint32_t)b;   // pad position inside the final block
#pragma unroll
      for (int w = 0; w < 17; w++)
        if ((uint32_t)w == (pp >> 3)) A[w] ^= 1ull << (8u * (pp & 7u));
      A[16] ^= 0x8000000000000000ull;
    }
    keccak_f1600(A);
  }
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint32_t v = 0;
    if (i < 8) {
      const uint64_t q = A[(7 - i) >> 1];
      v = __builtin_bswap32((uint32_t)(((7 - i) & 1) ? (q >> 32) : q));
    }
    X[i] = v;
  }
  sst<L>(cx, d, X);
}

// ---------------------------------------------------------------- interpreter
template <int L, bool K>
MQ_DEV bool run_tape(cu32p prog, const Ctx& cx) {
  uint32_t pc = 0;
  for (;;) {
    const uint32_t ins = prog[pc++];
    const uint32_t op = ins & 0xFFu;
    const int d = (int)((ins >> 8) & 0xFu);
    const uint32_t imm = ins >> 12;
    if (op == G_END) break;
    uint32_t imm2 = 0;
    if (has_imm2(op)) imm2 = prog[pc++];
    switch (op) {
      case G_PUSH_VAR:
      case G_PUSH_VAR_B: h_push_var<L>(cx, d, imm); break;
      case G_PUSH_CONST: h_push_const<L>(cx, d, imm); break;
      case G_PUSH_TMP:
      case G_PUSH_TMP_B: h_push_tmp<L>(cx, d, imm); break;
      case G_STORE_TMP:
      case G_STORE_TMP_B: h_store_tmp<L>(cx, d, imm); break;
      case G_PUSH_BOOL: sstb<L>(cx, d, (imm & 1u) != 0); break;
      // Bool connectives: limb 0
      case G_NOT: sstb<L>(cx, d, (sld0<L>(cx, d) & 1u) == 0); break;
      case G_AND: sstb<L>(cx, d - 1, (sld0<L>(cx, d - 1) & sld0<L>(cx, d) & 1u) != 0); break;
      case G_OR: sstb<L>(cx, d - 1, ((sld0<L>(cx, d - 1) | sld0<L>(cx, d)) & 1u) != 0); break;
      case G_XOR: sstb<L>(cx, d - 1, ((sld0<L>(cx, d - 1) ^ sld0<L>(cx, d)) & 1u) != 0); break;
      case G_IFF: sstb<L>(cx, d - 1, (sld0<L>(cx, d - 1) & 1u) == (sld0<L>(cx, d) & 1u)); break;
      case G_IMPLIES: sstb<L>(cx, d - 1, (((sld0<L>(cx, d - 1) ^ 1u) | sld0<L>(cx, d)) & 1u) != 0); break;
      case G_BITE: {
        const bool c = (sld0<L>(cx, d - 2) & 1u) != 0;
        sstb<L>(cx, d - 2, ((c ? sld0<L>(cx, d - 1) : sld0<L>(cx, d)) & 1u) != 0);
        break;
      }
      case G_BITE_EF: {
        const bool c = (sld0<L>(cx, d - 1) & 1u) != 0;
        sstb<L>(cx, d - 2, ((c ? sld0<L>(cx, d) : sld0<L>(cx, d - 2)) & 1u) != 0);
        break;
      }
      case G_EQ: h_eq<L>(cx, d, imm); break;
      case G_ULT: h_cmp<L>(cx, d, imm, 0, false); break;
      case G_ULE: h_cmp<L>(cx, d, imm, 1, false); break;
      case G_UGT: h_cmp<L>(cx, d, imm, 2, false); break;
      case G_UGE: h_cmp<L>(cx, d, imm, 3, false); break;
      case G_SLT: h_cmp<L>(cx, d, imm, 0, true); break;
      case G_SLE: h_cmp<L>(cx, d, imm, 1, true); break;
      case G_SGT: h_cmp<L>(cx, d, imm, 2, true); break;
      case G_SGE: h_cmp<L>(cx, d, imm, 3, true); break;
      case G_ADD: h_add_sub<L>(cx, d, imm, false); break;
      case G_SUB: h_add_sub<L>(cx, d, imm, true); break;
      case G_MUL: h_mul<L>(cx, d, imm); break;
      case G_NEG: h_neg_not<L>(cx, d, imm, false); break;
      case G_BNOT: h_neg_not<L>(cx, d, imm, true); break;
      case G_BAND: h_bitwise<L>(cx, d, imm, 0); break;
      case G_BOR: h_bitwise<L>(cx, d, imm, 1); break;
      case G_BXOR: h_bitwise<L>(cx, d, imm, 2); break;
      case G_ITE: h_ite<L>(cx, d - 2, d - 1, d, d - 2, imm); break;
      case G_ITE_EF: h_ite<L>(cx, d - 1, d, d - 2, d - 2, imm); break;
      case G_EXTRACT: h_extract<L>(cx, d, imm, imm2); break;
      case G_CONCAT: h_concat<L>(cx, d, imm, imm2); break;
      case G_SEXT: h_sext<L>(cx, d, imm, imm2); break;
      case G_UDIV:
      case G_UREM:
      case G_SDIV:
      case G_SREM:
      case G_SMOD: h_div<L>(cx, d, op, imm); break;
      case G_SHL:
      case G_LSHR:
      case G_ASHR: h_shift<L>(cx, d, op, imm); break;
      case G_UMUL_NOOVFL:
      case G_SMUL_NOOVFL:
      case G_SMUL_NOUDFL: h_mul_ovfl<L>(cx, d, op, imm); break;
      case G_UF1:
      case G_UF2: h_uf<L>(cx, d, op, imm, imm2); break;
      case G_UFK0:
      case G_UFK: h_ufk<L>(cx, d, op, imm, imm2); break;
      case G_UFKV: h_ufkv<L>(cx, d, imm, imm2); break;
      case G_KECCAK:
        if constexpr (K) h_keccak<L>(cx, d, imm);
        break;
      default: break;
    }
  }
  return (sld0<L>(cx, 0) & 1u) != 0;
}

// ---------------------------------------------------------------- kernels
// One wave per workgroup; a persistent grid strides over items (model tile of 64, tape group),
// item = group * tiles + tile (low candidate indices first, feeding the early exit).  A wave's
// operand stack lives in LDS (stack_slots x L x 256 B), its temp slots in HBM scratch.
template <int L, bool K>
__global__ __launch_bounds__(64) void qs_first_hit_kernel(KArgs args) {
  extern __shared__ uint4 lds_stack[];
  const int lane = threadIdx.x & 63;
  uint32_t* tmp = args.scratch + (size_t)blockIdx.x * (size_t)args.tmp_words_per_wave;
  uint64_t pairs = 0, nodes = 0, ops = 0;
  for (int64_t item = blockIdx.x; item < args.n_items; item += gridDim.x) {
    const int64_t tile = item % args.tiles;
    const int group = (int)(item / args.tiles);
    const int64_t m0 = tile * 64;
    const int64_t m = m0 + lane;
    const bool valid = m < args.M;
    Ctx cx = make_ctx(args, valid ? m : args.M - 1, tmp, lds_stack, lane);
    const int gbeg = group * args.tapes_per_group;
    const int gend = min(gbeg + args.tapes_per_group, args.n_desc);
    const int32_t gfirst = (int32_t)(args.index_base + m0);
    const uint64_t vmask = __ballot(valid);
    for (int i = gbeg; i < gend; i++) {
      const GDesc dsc = load_desc(args.descs, i);
      // workgroup scope: an ordinary (L1-cached) load, not a coherent L2 round trip per tape; a
      // stale value only skips less (best[] only decreases within a launch)
      int32_t cur = __hip_atomic_load(&args.best[dsc.tape], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      cur = __builtin_amdgcn_readfirstlane(cur);
      if (args.early_exit && gfirst >= cur) continue;
      cx.consts = CONSTP(cu32p, args.consts) + dsc.const_base;
      const bool r = run_tape<L, K>(CONSTP(cu32p, args.prog) + dsc.prog_off, cx);
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
    unsigned long long* cnt = args.counters + (blockIdx.x % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[0], (unsigned long long)pairs);
    atomicAdd(&cnt[1], (unsigned long long)nodes);
    atomicAdd(&cnt[2], (unsigned long long)ops);
  }
}

template <int L, bool K>
__global__ __launch_bounds__(64) void qs_verdict_kernel(KArgs args) {
  extern __shared__ uint4 lds_stack[];
  const int lane = threadIdx.x & 63;
  uint32_t* tmp = args.scratch + (size_t)blockIdx.x * (size_t)args.tmp_words_per_wave;
  for (int64_t item = blockIdx.x; item < args.n_items; item += gridDim.x) {
    const int64_t tile = item % args.tiles;
    const int group = (int)(item / args.tiles);
    const int64_t m0 = tile * 64;
    const int64_t m = m0 + lane;
    const bool valid = m < args.M;
    Ctx cx = make_ctx(args, valid ? m : args.M - 1, tmp, lds_stack, lane);
    const int gbeg = group * args.tapes_per_group;
    const int gend = min(gbeg + args.tapes_per_group, args.n_desc);
    for (int i = gbeg; i < gend; i++) {
      const GDesc dsc = load_desc(args.descs, i);
      cx.consts = CONSTP(cu32p, args.consts) + dsc.const_base;
      const bool r = run_tape<L, K>(CONSTP(cu32p, args.prog) + dsc.prog_off, cx);
      if (valid) args.verdicts[(int64_t)dsc.tape * args.M + m] = r ? 1 : 0;
    }
  }
}

// Column programs of batch-level hoisting (tape.py ColumnSet): each descriptor evaluates a
// sub-term shared by many tapes ONCE per model and writes its value into model variable
// dsc.tape's rows, which the batch's tapes then read as an ordinary variable.  One launch per
// nesting level (a level only reads columns written by earlier launches on the same stream).
template <int L, bool K>
__global__ __launch_bounds__(64) void qs_column_kernel(KArgs args) {
  extern __shared__ uint4 lds_stack[];
  const int lane = threadIdx.x & 63;
  uint32_t* tmp = args.scratch + (size_t)blockIdx.x * (size_t)args.tmp_words_per_wave;
  uint64_t nodes = 0, ops = 0;
  for (int64_t item = blockIdx.x; item < args.n_items; item += gridDim.x) {
    const int64_t tile = item % args.tiles;
    const int group = (int)(item / args.tiles);
    const int64_t m = tile * 64 + lane;
    const bool valid = m < args.M;
    Ctx cx = make_ctx(args, valid ? m : args.M - 1, tmp, lds_stack, lane);
    const int gbeg = group * args.tapes_per_group;
    const int gend = min(gbeg + args.tapes_per_group, args.n_desc);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    for (int i = gbeg; i < gend; i++) {
      const GDesc dsc = load_desc(args.descs, i);
      cx.consts = CONSTP(cu32p, args.consts) + dsc.const_base;
      (void)run_tape<L, K>(CONSTP(cu32p, args.prog) + dsc.prog_off, cx);
      uint32_t x[L];
      sld<L>(cx, 0, x);
      const uint32_t off = CONSTP(cu32p, args.var_off)[dsc.tape];
      const uint32_t nl = CONSTP(cu32p, args.var_nl)[dsc.tape];
      if (valid) {
        uint32_t* dst = const_cast<uint32_t*>(args.vars) + (int64_t)off * args.M + m;
#pragma unroll
        for (int l = 0; l < L; l++)
          if ((uint32_t)l < nl) dst[(int64_t)l * args.M] = x[l];
      }
      nodes += (uint64_t)nvalid * dsc.n_nodes;
      ops += (uint64_t)nvalid * dsc.alg_ops;
    }
  }
  if (lane == 0 && args.counters) {
    unsigned long long* cnt = args.counters + (blockIdx.x % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[1], (unsigned long long)nodes);
    atomicAdd(&cnt[2], (unsigned long long)ops);
  }
}

// The 1024/2048-bit stacks may need more than 64 KB of dynamic LDS (up to 8 x 16 KB per wave).
template <class F>
static hipError_t allow_lds(F* kernel, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

template <int L, bool K>
static hipError_t launch_column_variant(const KArgs& a, hipStream_t st) {
  if (a.n_desc <= 0 || a.grid <= 0) return hipSuccess;
  const size_t lds = (size_t)a.stack_slots * L * 64 * 4;
  hipError_t e = allow_lds(qs_column_kernel<L, K>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((qs_column_kernel<L, K>), dim3((unsigned)a.grid), dim3(64), lds, st, a);
  return hipGetLastError();
}

// kernel variants: (8, plain), (16, plain), (16, keccak), (32, keccak), (64, keccak); the wide
// stacks always carry the keccak handler (their registers are dominated by the wide operands)
hipError_t launch_columns(const KArgs& a, int L, bool keccak, hipStream_t st) {
  if (L == 8 && !keccak) return launch_column_variant<8, false>(a, st);
  if (L == 16) return keccak ? launch_column_variant<16, true>(a, st) : launch_column_variant<16, false>(a, st);
  if (L == 32) return launch_column_variant<32, true>(a, st);
  if (L == 64) return launch_column_variant<64, true>(a, st);
  return hipErrorInvalidValue;
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

// Bool variable rows as 64-bit lane masks per 64-model tile (the G interpreter's PUSH_PKB reads a
// tile's mask with one scalar load).  One wave per (tile, row).
__global__ __launch_bounds__(256) void qs_pack_bool(const uint32_t* vars, uint64_t* masks, const uint32_t* rows,
                                                    const int32_t* list, int n_masks, int64_t M) {
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile * 64 >= M) return;   // wave-uniform
  const int j = list ? list[blockIdx.y] : (int)blockIdx.y;
  const int64_t m = tile * 64 + (threadIdx.x & 63);
  const bool bit = m < M && vars[(int64_t)rows[j] * M + m] != 0u;
  const unsigned long long mask = __ballot(bit);
  if ((threadIdx.x & 63) == 0) masks[tile * n_masks + j] = mask;
}

hipError_t launch_pack_bool(const uint32_t* vars, uint64_t* masks, const uint32_t* rows, const int32_t* list, int n,
                            int n_masks, int64_t M, hipStream_t st) {
  const int64_t tiles = (M + 63) / 64;
  if (n <= 0 || tiles <= 0) return hipSuccess;
  if (n > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(qs_pack_bool, dim3((unsigned)((tiles + 3) / 4), (unsigned)n), dim3(256), 0, st, vars, masks, rows,
                     list, n_masks, M);
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
template <int L, bool K>
static hipError_t launch_variant(const KArgs& a, bool verdict, hipStream_t st) {
  if (a.n_desc <= 0 || a.grid <= 0) return hipSuccess;
  const size_t lds = (size_t)a.stack_slots * L * 64 * 4;
  hipError_t e = verdict ? allow_lds(qs_verdict_kernel<L, K>, lds) : allow_lds(qs_first_hit_kernel<L, K>, lds);
  if (e != hipSuccess) return e;
  if (verdict) hipLaunchKernelGGL((qs_verdict_kernel<L, K>), dim3((unsigned)a.grid), dim3(64), lds, st, a);
  else hipLaunchKernelGGL((qs_first_hit_kernel<L, K>), dim3((unsigned)a.grid), dim3(64), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_qs(const KArgs& a, int L, bool keccak, bool verdict, hipStream_t st) {
  if (L == 8 && !keccak) return launch_variant<8, false>(a, verdict, st);
  if (L == 16) return keccak ? launch_variant<16, true>(a, verdict, st) : launch_variant<16, false>(a, verdict, st);
  if (L == 32) return launch_variant<32, true>(a, verdict, st);
  if (L == 64) return launch_variant<64, true>(a, verdict, st);
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
