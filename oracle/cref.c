/*
 * ORACLE — test infrastructure and the CPU baseline only; never linked into libmq.so.
 *
 * Plain-C restatement of the reference quick-sat hot path on the mq.h tape/model layouts:
 *   cref_first_hit  = ModelCache.check_quick_sat  (mythril/support/support_utils.py:60-67):
 *                     candidates in order (0 = MRU, support_utils.py:62), first one whose
 *                     evaluation is literally true (is_true, support_utils.py:64) wins.
 *   cref_eval_tape  = z3 model.eval(expr, model_completion=True) (support_utils.py:64 via
 *                     mythril/laser/smt/model.py:45-58) on the lowered tape: SMT-LIB 2.6
 *                     FixedSizeBitVectors + z3 model completion.
 * The executable spec it must agree with bit for bit is oracle/pyoracle.py; both are pinned
 * by the reference's vectors in tests/golden (EIP-145 shift vectors from
 * tests/instructions/{shl,shr,sar}_test.py, VMTests arithmetic/bitwise/sha3 KATs).
 * z3 itself (z3-solver <=4.12.5.0, requirements.txt:36) is absent: model completion and
 * UF/array evaluation are spec-derived ("parity unpinned" by any reference test).
 *
 * Values are little-endian u32 limbs, canonical (bits >= width are zero); Bool = 0/1.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/mq.h"

#define MAXL 64 /* 2048-bit values */

static inline int nlimbs(int w) { return w == 0 ? 1 : (w + 31) / 32; }

static void mask_top(uint32_t* x, int w) {
  int n = nlimbs(w);
  if (w && (w & 31)) x[n - 1] &= (1u << (w & 31)) - 1u;
}

static int is_zero(const uint32_t* x, int n) {
  for (int i = 0; i < n; i++) if (x[i]) return 0;
  return 1;
}

static int cmp_u(const uint32_t* a, const uint32_t* b, int n) {
  for (int i = n - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}

static int sign_bit(const uint32_t* x, int w) { return (x[(w - 1) >> 5] >> ((w - 1) & 31)) & 1; }

static void neg_w(uint32_t* r, const uint32_t* a, int w) {
  int n = nlimbs(w);
  uint64_t carry = 1;
  for (int i = 0; i < n; i++) {
    uint64_t t = (uint64_t)(uint32_t)~a[i] + carry;
    r[i] = (uint32_t)t;
    carry = t >> 32;
  }
  mask_top(r, w);
}

static void add_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  uint64_t carry = 0;
  for (int i = 0; i < n; i++) {
    uint64_t t = (uint64_t)a[i] + b[i] + carry;
    r[i] = (uint32_t)t;
    carry = t >> 32;
  }
  mask_top(r, w);
}

static void sub_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  int64_t borrow = 0;
  for (int i = 0; i < n; i++) {
    int64_t t = (int64_t)a[i] - b[i] - borrow;
    r[i] = (uint32_t)t;
    borrow = t < 0;
  }
  mask_top(r, w);
}

/* full product of n-limb a and b into 2n limbs */
static void mul_full(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  memset(r, 0, sizeof(uint32_t) * 2 * n);
  for (int i = 0; i < n; i++) {
    uint64_t carry = 0;
    if (!a[i]) continue;
    for (int j = 0; j < n; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + n] = (uint32_t)carry;
  }
}

static void mul_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  uint32_t t[MAXL];
  memset(t, 0, sizeof(uint32_t) * n);
  for (int i = 0; i < n; i++) {
    uint64_t carry = 0;
    for (int j = 0; i + j < n; j++) {
      uint64_t p = (uint64_t)a[i] * b[j] + t[i + j] + carry;
      t[i + j] = (uint32_t)p;
      carry = p >> 32;
    }
  }
  memcpy(r, t, sizeof(uint32_t) * n);
  mask_top(r, w);
}

/* Knuth algorithm D (Hacker's Delight divmnu) on n-limb canonical operands, b != 0. */
static void divmod_u(uint32_t* q, uint32_t* r, const uint32_t* a, const uint32_t* b, int nl) {
  int n = nl, m = nl;
  while (n > 0 && b[n - 1] == 0) n--;
  while (m > 0 && a[m - 1] == 0) m--;
  memset(q, 0, sizeof(uint32_t) * nl);
  memset(r, 0, sizeof(uint32_t) * nl);
  if (m < n) { memcpy(r, a, sizeof(uint32_t) * nl); return; }
  if (n == 1) {
    uint64_t rem = 0, d = b[0];
    for (int i = m - 1; i >= 0; i--) {
      uint64_t cur = (rem << 32) | a[i];
      q[i] = (uint32_t)(cur / d);
      rem = cur % d;
    }
    r[0] = (uint32_t)rem;
    return;
  }
  int s = __builtin_clz(b[n - 1]);
  uint32_t vn[MAXL], un[MAXL + 1];
  for (int i = n - 1; i > 0; i--) vn[i] = s ? (b[i] << s) | (b[i - 1] >> (32 - s)) : b[i];
  vn[0] = b[0] << s;
  un[m] = s ? a[m - 1] >> (32 - s) : 0;
  for (int i = m - 1; i > 0; i--) un[i] = s ? (a[i] << s) | (a[i - 1] >> (32 - s)) : a[i];
  un[0] = a[0] << s;
  const uint64_t B = 1ull << 32;
  for (int j = m - n; j >= 0; j--) {
    uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
    uint64_t qhat = num / vn[n - 1];
    uint64_t rhat = num % vn[n - 1];
    while (qhat >= B || qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
      qhat--;
      rhat += vn[n - 1];
      if (rhat >= B) break;
    }
    int64_t borrow = 0, t;
    for (int i = 0; i < n; i++) {
      uint64_t p = qhat * vn[i];
      t = (int64_t)un[i + j] - borrow - (int64_t)(p & 0xFFFFFFFFull);
      un[i + j] = (uint32_t)t;
      borrow = (int64_t)(p >> 32) - (t >> 32);
    }
    t = (int64_t)un[j + n] - borrow;
    un[j + n] = (uint32_t)t;
    q[j] = (uint32_t)qhat;
    if (t < 0) {
      q[j]--;
      uint64_t carry = 0;
      for (int i = 0; i < n; i++) {
        uint64_t tt = (uint64_t)un[i + j] + vn[i] + carry;
        un[i + j] = (uint32_t)tt;
        carry = tt >> 32;
      }
      un[j + n] += (uint32_t)carry;
    }
  }
  for (int i = 0; i < n; i++) r[i] = s ? (un[i] >> s) | (un[i + 1] << (32 - s)) : un[i];
}

static void udiv_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  if (is_zero(b, n)) { for (int i = 0; i < n; i++) r[i] = 0xFFFFFFFFu; mask_top(r, w); return; }
  uint32_t q[MAXL], rr[MAXL];
  divmod_u(q, rr, a, b, n);
  memcpy(r, q, sizeof(uint32_t) * n);
}

static void urem_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  if (is_zero(b, n)) { memcpy(r, a, sizeof(uint32_t) * n); return; }
  uint32_t q[MAXL], rr[MAXL];
  divmod_u(q, rr, a, b, n);
  memcpy(r, rr, sizeof(uint32_t) * n);
}

static void sdiv_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  int sa = sign_bit(a, w), sb = sign_bit(b, w);
  uint32_t na[MAXL], nb[MAXL], q[MAXL];
  if (sa) neg_w(na, a, w); else memcpy(na, a, 4 * n);
  if (sb) neg_w(nb, b, w); else memcpy(nb, b, 4 * n);
  udiv_w(q, na, nb, w);
  if (sa ^ sb) neg_w(r, q, w); else memcpy(r, q, 4 * n);
}

static void srem_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  int sa = sign_bit(a, w), sb = sign_bit(b, w);
  uint32_t na[MAXL], nb[MAXL], q[MAXL];
  if (sa) neg_w(na, a, w); else memcpy(na, a, 4 * n);
  if (sb) neg_w(nb, b, w); else memcpy(nb, b, 4 * n);
  urem_w(q, na, nb, w);
  if (sa) neg_w(r, q, w); else memcpy(r, q, 4 * n);
}

static void smod_w(uint32_t* r, const uint32_t* a, const uint32_t* b, int w) {
  int n = nlimbs(w);
  int sa = sign_bit(a, w), sb = sign_bit(b, w);
  uint32_t na[MAXL], nb[MAXL], u[MAXL], t[MAXL];
  if (sa) neg_w(na, a, w); else memcpy(na, a, 4 * n);
  if (sb) neg_w(nb, b, w); else memcpy(nb, b, 4 * n);
  urem_w(u, na, nb, w);
  if (is_zero(u, n) || (!sa && !sb)) { memcpy(r, u, 4 * n); return; }
  if (sa && !sb) { neg_w(t, u, w); add_w(r, t, b, w); return; }
  if (!sa && sb) { add_w(r, u, b, w); return; }
  neg_w(r, u, w);
}

/* shift amount: full W-bit value of b; returns UINT32_MAX when >= w */
static uint32_t shamt(const uint32_t* b, int w) {
  int n = nlimbs(w);
  for (int i = 1; i < n; i++) if (b[i]) return 0xFFFFFFFFu;
  return b[0] >= (uint32_t)w ? 0xFFFFFFFFu : b[0];
}

static void shl_bits(uint32_t* r, const uint32_t* a, uint32_t s, int n) {
  uint32_t t[MAXL];
  int ls = s >> 5, bs = s & 31;
  for (int i = n - 1; i >= 0; i--) {
    uint32_t hi = (i - ls >= 0) ? a[i - ls] : 0;
    uint32_t lo = (i - ls - 1 >= 0) ? a[i - ls - 1] : 0;
    t[i] = bs ? (hi << bs) | (lo >> (32 - bs)) : hi;
  }
  memcpy(r, t, 4 * n);
}

static void lshr_bits(uint32_t* r, const uint32_t* a, uint32_t s, int n, uint32_t fill) {
  uint32_t t[MAXL];
  int ls = s >> 5, bs = s & 31;
  for (int i = 0; i < n; i++) {
    uint32_t lo = (i + ls < n) ? a[i + ls] : fill;
    uint32_t hi = (i + ls + 1 < n) ? a[i + ls + 1] : fill;
    t[i] = bs ? (lo >> bs) | (hi << (32 - bs)) : lo;
  }
  memcpy(r, t, 4 * n);
}

/* sign-extend canonical w-bit x to n limbs in place */
static void sext_to(uint32_t* x, int w, int n) {
  int nw = nlimbs(w);
  if (!sign_bit(x, w)) { for (int i = nw; i < n; i++) x[i] = 0; return; }
  if (w & 31) x[nw - 1] |= ~((1u << (w & 31)) - 1u);
  for (int i = nw; i < n; i++) x[i] = 0xFFFFFFFFu;
}

/* ------------------------------------------------------------------ keccak */
static const uint64_t RC[24] = {
  0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
  0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
  0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
  0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
  0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
  0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int ROTC[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline uint64_t rol64(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

static void keccakf(uint64_t* A) {
  for (int r = 0; r < 24; r++) {
    uint64_t C[5], D[5], Bv[25];
    for (int x = 0; x < 5; x++) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) A[i] ^= D[i % 5];
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) Bv[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(A[x + 5 * y], ROTC[x + 5 * y]);
    for (int y = 0; y < 5; y++)
      for (int x = 0; x < 5; x++) A[x + 5 * y] = Bv[x + 5 * y] ^ ((~Bv[(x + 1) % 5 + 5 * y]) & Bv[(x + 2) % 5 + 5 * y]);
    A[0] ^= RC[r];
  }
}

void cref_keccak256(const uint8_t* data, int64_t len, uint8_t* out) {
  uint64_t A[25];
  memset(A, 0, sizeof(A));
  const int rate = 136;
  int64_t off = 0;
  uint8_t block[136];
  for (;;) {
    int64_t take = len - off;
    if (take >= rate) {
      memcpy(block, data + off, rate);
      off += rate;
    } else {
      memset(block, 0, rate);
      if (take > 0) memcpy(block, data + off, (size_t)take);
      block[take] ^= 0x01;
      block[rate - 1] ^= 0x80;
      off = len + 1;
    }
    for (int i = 0; i < rate / 8; i++) {
      uint64_t lane = 0;
      for (int k = 0; k < 8; k++) lane |= (uint64_t)block[8 * i + k] << (8 * k);
      A[i] ^= lane;
    }
    keccakf(A);
    if (off > len) break;
  }
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(A[i] >> (8 * k));
}

/* ------------------------------------------------------------------ evaluator */
typedef struct {
  const mq_tape_batch* tb;
  const mq_model_batch* mb;
  int64_t* var_off; /* word offset of each var */
} cref_env;

static int64_t func_stride(const mq_func_desc* f) {
  int64_t s = nlimbs(f->result_width);
  for (int i = 0; i < f->arity; i++) s += nlimbs(f->arg_width[i]);
  return s;
}

/* UF / as-array lookup: entries first (exact match), else value. */
static void func_lookup(const cref_env* env, uint32_t f, int64_t m, const uint32_t* const* args, uint32_t* out) {
  const mq_model_batch* mb = env->mb;
  int64_t M = mb->n_models;
  if ((int32_t)f >= mb->n_funcs) { memset(out, 0, 4); return; }
  const mq_func_desc* fd = &mb->funcs[f];
  int nv = nlimbs(fd->result_width);
  int64_t stride = func_stride(fd);
  int64_t lo = mb->entry_ptr[f * (M + 1) + m], hi = mb->entry_ptr[f * (M + 1) + m + 1];
  for (int64_t e = lo; e < hi; e++) {
    const uint32_t* ent = mb->entry_words + mb->entry_base[f] + e * stride;
    int ok = 1, pos = 0;
    for (int i = 0; i < fd->arity && ok; i++) {
      int na = nlimbs(fd->arg_width[i]);
      if (memcmp(ent + pos, args[i], 4 * na)) ok = 0;
      pos += na;
    }
    if (ok) { memcpy(out, ent + pos, 4 * nv); return; }
  }
  memcpy(out, mb->else_words + mb->else_base[f] + m * nv, 4 * nv);
}

/* Evaluate tape t under model m. vals: scratch of (n_nodes * MAXL) words. Returns 1/0, or
   -2 for an unsupported construct (width > 2048). */
static int eval_tape(const cref_env* env, int32_t t, int64_t m, uint32_t* vals) {
  const mq_tape_batch* tb = env->tb;
  const mq_model_batch* mb = env->mb;
  int64_t base = tb->tape_offsets[t], nn = tb->tape_offsets[t + 1] - base;
  const mq_node* nodes = tb->nodes + base;
  int64_t M = mb->n_models;
  for (int64_t i = 0; i < nn; i++) {
    const mq_node* nd = &nodes[i];
    int w = nd->width, n = nlimbs(w);
    if (n > MAXL) return -2;
    uint32_t* r = vals + i * MAXL;
    const uint32_t* A = nd->a < (uint32_t)nn ? vals + (int64_t)nd->a * MAXL : NULL;
    const uint32_t* Bv = nd->b < (uint32_t)nn ? vals + (int64_t)nd->b * MAXL : NULL;
    const uint32_t* Cv = nd->c < (uint32_t)nn ? vals + (int64_t)nd->c * MAXL : NULL;
    int aw = A ? nodes[nd->a].width : 0;
    memset(r, 0, 4 * n);
    switch (nd->op) {
      case MQ_OP_CONST: memcpy(r, tb->const_words + nd->a, 4 * n); mask_top(r, w); break;
      case MQ_OP_VAR:
        if ((int32_t)nd->a < mb->n_vars) {
          int vn = nlimbs(mb->var_width[nd->a]);
          for (int k = 0; k < n && k < vn; k++) r[k] = mb->var_words[(env->var_off[nd->a] + k) * M + m];
          if (w == 0) r[0] &= 1; else mask_top(r, w);
        }
        break;
      case MQ_OP_TRUE: r[0] = 1; break;
      case MQ_OP_FALSE: r[0] = 0; break;
      case MQ_OP_NOT: r[0] = A[0] ^ 1; break;
      case MQ_OP_AND: r[0] = A[0] & Bv[0]; break;
      case MQ_OP_OR: r[0] = A[0] | Bv[0]; break;
      case MQ_OP_XOR: r[0] = A[0] ^ Bv[0]; break;
      case MQ_OP_IMPLIES: r[0] = (A[0] ^ 1) | Bv[0]; break;
      case MQ_OP_IFF: r[0] = A[0] == Bv[0]; break;
      case MQ_OP_BITE: r[0] = A[0] ? Bv[0] : Cv[0]; break;
      case MQ_OP_EQ: r[0] = cmp_u(A, Bv, nlimbs(aw)) == 0; break;
      case MQ_OP_ULT: r[0] = cmp_u(A, Bv, nlimbs(aw)) < 0; break;
      case MQ_OP_ULE: r[0] = cmp_u(A, Bv, nlimbs(aw)) <= 0; break;
      case MQ_OP_SLT:
      case MQ_OP_SLE: {
        int sa = sign_bit(A, aw), sb = sign_bit(Bv, aw);
        int c = sa != sb ? (sa ? -1 : 1) : cmp_u(A, Bv, nlimbs(aw));
        r[0] = nd->op == MQ_OP_SLT ? c < 0 : c <= 0;
        break;
      }
      case MQ_OP_UMUL_NOOVFL:
      case MQ_OP_SMUL_NOOVFL:
      case MQ_OP_SMUL_NOUDFL: {
        int na = nlimbs(aw);
        uint32_t p[2 * MAXL], xa[MAXL], xb[MAXL];
        if (nd->op == MQ_OP_UMUL_NOOVFL) {
          mul_full(p, A, Bv, na);
          /* product < 2^aw  <=>  no bit >= aw set */
          int ok = 1;
          for (int k = 0; k < 2 * na; k++) {
            uint32_t word = p[k];
            int lo_bit = 32 * k;
            if (lo_bit + 32 <= aw) continue;
            if (lo_bit >= aw) { if (word) ok = 0; }
            else if (word >> (aw - lo_bit)) ok = 0;
          }
          r[0] = ok;
        } else {
          int sa = sign_bit(A, aw), sb = sign_bit(Bv, aw);
          if (sa) neg_w(xa, A, aw); else memcpy(xa, A, 4 * na);
          if (sb) neg_w(xb, Bv, aw); else memcpy(xb, Bv, 4 * na);
          /* |a| as unsigned aw-bit: for a = -2^(aw-1), neg gives 2^(aw-1) (fits) */
          mul_full(p, xa, xb, na);
          int neg = sa ^ sb;
          int pz = is_zero(p, 2 * na);
          /* limit: overflow check: product <= 2^(aw-1)-1 when positive;
                    underflow check: -product >= -2^(aw-1) i.e. product <= 2^(aw-1) when negative */
          int hb = aw - 1; /* compare p against 2^hb */
          int gt_pow = 0, eq_pow = 1; /* p > 2^hb ?  p == 2^hb ? */
          for (int k = 2 * na - 1; k >= 0; k--) {
            uint32_t pw = (k == (hb >> 5)) ? (1u << (hb & 31)) : 0u;
            if (p[k] != pw) { eq_pow = 0; gt_pow = p[k] > pw; break; }
          }
          if (nd->op == MQ_OP_SMUL_NOOVFL) r[0] = (neg || pz) ? 1 : (!gt_pow && !eq_pow);
          else r[0] = (!neg || pz) ? 1 : (!gt_pow);
        }
        break;
      }
      case MQ_OP_ADD: add_w(r, A, Bv, w); break;
      case MQ_OP_SUB: sub_w(r, A, Bv, w); break;
      case MQ_OP_MUL: mul_w(r, A, Bv, w); break;
      case MQ_OP_NEG: neg_w(r, A, w); break;
      case MQ_OP_UDIV: udiv_w(r, A, Bv, w); break;
      case MQ_OP_UREM: urem_w(r, A, Bv, w); break;
      case MQ_OP_SDIV: sdiv_w(r, A, Bv, w); break;
      case MQ_OP_SREM: srem_w(r, A, Bv, w); break;
      case MQ_OP_SMOD: smod_w(r, A, Bv, w); break;
      case MQ_OP_BAND: for (int k = 0; k < n; k++) r[k] = A[k] & Bv[k]; break;
      case MQ_OP_BOR: for (int k = 0; k < n; k++) r[k] = A[k] | Bv[k]; break;
      case MQ_OP_BXOR: for (int k = 0; k < n; k++) r[k] = A[k] ^ Bv[k]; break;
      case MQ_OP_BNOT: for (int k = 0; k < n; k++) r[k] = ~A[k]; mask_top(r, w); break;
      case MQ_OP_SHL: {
        uint32_t s = shamt(Bv, w);
        if (s != 0xFFFFFFFFu) { shl_bits(r, A, s, n); mask_top(r, w); }
        break;
      }
      case MQ_OP_LSHR: {
        uint32_t s = shamt(Bv, w);
        if (s != 0xFFFFFFFFu) lshr_bits(r, A, s, n, 0);
        break;
      }
      case MQ_OP_ASHR: {
        uint32_t s = shamt(Bv, w), x[MAXL];
        int neg = sign_bit(A, w);
        memcpy(x, A, 4 * n);
        sext_to(x, w, n);
        if (s == 0xFFFFFFFFu) { for (int k = 0; k < n; k++) r[k] = neg ? 0xFFFFFFFFu : 0; }
        else lshr_bits(r, x, s, n, neg ? 0xFFFFFFFFu : 0);
        mask_top(r, w);
        break;
      }
      case MQ_OP_EXTRACT: {
        uint32_t x[MAXL];
        int na = nlimbs(aw);
        memcpy(x, A, 4 * na);
        lshr_bits(x, x, nd->c, na, 0);
        memcpy(r, x, 4 * n);
        mask_top(r, w);
        break;
      }
      case MQ_OP_CONCAT: {
        int bw = nodes[nd->b].width;
        uint32_t x[MAXL];
        memset(x, 0, 4 * n);
        memcpy(x, A, 4 * nlimbs(aw));
        shl_bits(x, x, bw, n);
        for (int k = 0; k < nlimbs(bw); k++) x[k] |= Bv[k];
        memcpy(r, x, 4 * n);
        mask_top(r, w);
        break;
      }
      case MQ_OP_ZEXT: memcpy(r, A, 4 * nlimbs(aw)); break;
      case MQ_OP_SEXT: memcpy(r, A, 4 * nlimbs(aw)); sext_to(r, aw, n); mask_top(r, w); break;
      case MQ_OP_ITE: memcpy(r, A[0] ? Bv : Cv, 4 * n); break;
      case MQ_OP_STORE: case MQ_OP_CONST_ARRAY: case MQ_OP_ARRAY_VAR: break; /* array values are node refs */
      case MQ_OP_SELECT: {
        /* walk the store chain: select(store(A,k,v), i) = i==k ? v : select(A, i) */
        uint32_t arr = nd->a;
        int kl = nlimbs(nodes[nd->b].width);
        for (;;) {
          const mq_node* an = &nodes[arr];
          if (an->op == MQ_OP_STORE) {
            if (memcmp(vals + (int64_t)an->b * MAXL, Bv, 4 * kl) == 0) { memcpy(r, vals + (int64_t)an->c * MAXL, 4 * n); break; }
            arr = an->a;
          } else if (an->op == MQ_OP_CONST_ARRAY) {
            memcpy(r, vals + (int64_t)an->a * MAXL, 4 * n);
            break;
          } else if (an->op == MQ_OP_ARRAY_VAR) {
            const uint32_t* args[1] = {Bv};
            func_lookup(env, an->a, m, args, r);
            break;
          } else {
            return -2;
          }
        }
        break;
      }
      case MQ_OP_UF_CHUNK: {
        /* wide-key lookup, key chunk k (mq.h): the entries of the model's table of f (bit e,
           at most 64 of them, else unsupported) whose key limbs [8k, 8k + 8) equal the chunk,
           within the previous chunk's set (or all entries for k = 0) */
        const mq_func_desc* fd = (int32_t)nd->a < mb->n_funcs ? &mb->funcs[nd->a] : NULL;
        int k = 0;
        for (uint32_t q = nd->c; q != MQ_NONE && q < (uint32_t)i; q = nodes[q].c) k++;
        uint64_t mask = 0;
        if (fd && fd->arity == 1) {
          int64_t lo = mb->entry_ptr[nd->a * (M + 1) + m], hi = mb->entry_ptr[nd->a * (M + 1) + m + 1];
          int64_t E = hi - lo, stride = func_stride(fd);
          int nk = nlimbs(fd->arg_width[0]) - 8 * k;
          if (E > 64) return -2;
          mask = nd->c == MQ_NONE ? (E == 64 ? ~0ull : ((1ull << E) - 1)) : ((uint64_t)Cv[0] | ((uint64_t)Cv[1] << 32));
          for (int64_t e = 0; e < E; e++) {
            const uint32_t* ent = mb->entry_words + mb->entry_base[nd->a] + (lo + e) * stride + 8 * k;
            int eq = nk > 0;
            for (int l = 0; l < 8 && l < nk && eq; l++) eq = ent[l] == Bv[l];
            if (!eq) mask &= ~(1ull << e);
          }
        }
        r[0] = (uint32_t)mask;
        r[1] = (uint32_t)(mask >> 32);
        break;
      }
      case MQ_OP_UF_WIDE: {
        /* the first entry of the set, else the else value (the lookup of the whole key) */
        uint64_t mask = (uint64_t)Bv[0] | ((uint64_t)Bv[1] << 32);
        const mq_func_desc* fd = (int32_t)nd->a < mb->n_funcs ? &mb->funcs[nd->a] : NULL;
        if (!fd) break;
        int nv = nlimbs(fd->result_width);
        if (mask) {
          int e = __builtin_ctzll(mask);
          int64_t lo = mb->entry_ptr[nd->a * (M + 1) + m];
          const uint32_t* ent = mb->entry_words + mb->entry_base[nd->a] + (lo + e) * func_stride(fd);
          memcpy(r, ent + nlimbs(fd->arg_width[0]), 4 * nv);
        } else {
          memcpy(r, mb->else_words + mb->else_base[nd->a] + m * nv, 4 * nv);
        }
        mask_top(r, w ? w : 1);
        break;
      }
      case MQ_OP_UF: {
        const uint32_t* args[2] = {Bv, Cv};
        func_lookup(env, nd->a, m, args, r);
        break;
      }
      case MQ_OP_KECCAK: {
        int nbytes = aw / 8;
        uint8_t buf[MAXL * 4], dig[32];
        for (int k = 0; k < nbytes; k++) {
          int bit = 8 * (nbytes - 1 - k); /* big-endian byte k */
          buf[k] = (uint8_t)(A[bit >> 5] >> (bit & 31));
        }
        cref_keccak256(buf, nbytes, dig);
        for (int k = 0; k < 8; k++)
          r[k] = ((uint32_t)dig[31 - 4 * k]) | ((uint32_t)dig[30 - 4 * k] << 8) | ((uint32_t)dig[29 - 4 * k] << 16) | ((uint32_t)dig[28 - 4 * k] << 24);
        break;
      }
      default:
        return -2;
    }
  }
  return vals[(nn - 1) * MAXL] == 1;
}

static int64_t* make_var_off(const mq_model_batch* mb) {
  int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (mb->n_vars + 1));
  off[0] = 0;
  for (int v = 0; v < mb->n_vars; v++) off[v + 1] = off[v] + nlimbs(mb->var_width[v]);
  return off;
}

static int64_t max_tape_len(const mq_tape_batch* tb) {
  int64_t mx = 1;
  for (int t = 0; t < tb->n_tapes; t++) {
    int64_t l = tb->tape_offsets[t + 1] - tb->tape_offsets[t];
    if (l > mx) mx = l;
  }
  return mx;
}

int cref_eval_tape(const mq_tape_batch* tb, int32_t t, const mq_model_batch* mb, int64_t m) {
  cref_env env = {tb, mb, make_var_off(mb)};
  int64_t nn = tb->tape_offsets[t + 1] - tb->tape_offsets[t];
  uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * MAXL * (nn + 1));
  int r = eval_tape(&env, t, m, vals);
  free(vals);
  free(env.var_off);
  return r;
}

/* A wide-key lookup (MQ_OP_UF_CHUNK) of a function that some model of the batch holds more than
   64 entries of: the tape is unsupported under the whole batch (mq.h; the evaluator's rule). */
static int wide_unsupported(const mq_tape_batch* tb, const mq_model_batch* mb, int32_t t) {
  int64_t base = tb->tape_offsets[t], nn = tb->tape_offsets[t + 1] - base, M = mb->n_models;
  for (int64_t i = 0; i < nn; i++) {
    const mq_node* nd = &tb->nodes[base + i];
    if (nd->op != MQ_OP_UF_CHUNK || (int32_t)nd->a >= mb->n_funcs) continue;
    const int64_t* p = mb->entry_ptr + (int64_t)nd->a * (M + 1);
    for (int64_t m = 0; m < M; m++)
      if (p[m + 1] - p[m] > 64) return 1;
  }
  return 0;
}

/* check_quick_sat for every tape; out[t] = global index (index_base + m) | -1 | -2.
   Parallel over tapes with OpenMP (nthreads <= 0: runtime default). Returns evaluated pairs. */
int64_t cref_first_hit(const mq_tape_batch* tb, const mq_model_batch* mb, int32_t* out, int nthreads) {
  cref_env env = {tb, mb, make_var_off(mb)};
  int64_t mx = max_tape_len(tb);
  int64_t pairs = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : pairs)
  {
    uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * MAXL * (mx + 1));
#pragma omp for schedule(dynamic, 4)
    for (int t = 0; t < tb->n_tapes; t++) {
      int32_t hit = wide_unsupported(tb, mb, t) ? -2 : -1;
      for (int64_t m = 0; m < mb->n_models && hit == -1; m++) {
        int r = eval_tape(&env, t, m, vals);
        pairs++;
        if (r == -2) { hit = -2; break; }
        if (r == 1) { hit = (int32_t)(mb->index_base + m); break; }
      }
      out[t] = hit;
    }
    free(vals);
  }
  free(env.var_off);
  return pairs;
}

/* Full verdict bit matrix (row-major tape x model), -2 rows stay zero. */
int cref_verdicts(const mq_tape_batch* tb, const mq_model_batch* mb, uint8_t* bits, int nthreads) {
  cref_env env = {tb, mb, make_var_off(mb)};
  int64_t mx = max_tape_len(tb);
  int64_t M = mb->n_models;
  memset(bits, 0, (size_t)((tb->n_tapes * M + 7) / 8));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  int bad = 0;
#pragma omp parallel reduction(| : bad)
  {
    uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * MAXL * (mx + 1));
#pragma omp for schedule(dynamic, 4)
    for (int t = 0; t < tb->n_tapes; t++) {
      if (wide_unsupported(tb, mb, t)) { bad = 1; continue; }
      for (int64_t m = 0; m < M; m++) {
        int r = eval_tape(&env, t, m, vals);
        if (r == -2) { bad = 1; break; }
        if (r == 1) {
          int64_t bit = (int64_t)t * M + m;
#pragma omp atomic
          bits[bit >> 3] |= (uint8_t)(1u << (bit & 7));
        }
      }
    }
    free(vals);
  }
  free(env.var_off);
  return bad ? -2 : 0;
}

/* Value of the root-or-any node n of tape t under model m (tests: per-op golden vectors).
   out must hold MAXL words; returns the node's limb count or -2. */
int cref_eval_node(const mq_tape_batch* tb, int32_t t, const mq_model_batch* mb, int64_t m, int64_t node, uint32_t* out) {
  cref_env env = {tb, mb, make_var_off(mb)};
  int64_t nn = tb->tape_offsets[t + 1] - tb->tape_offsets[t];
  uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * MAXL * (nn + 1));
  /* evaluate fully (root must exist); ignore the root verdict */
  int r = eval_tape(&env, t, m, vals);
  int n = nlimbs(tb->nodes[tb->tape_offsets[t] + node].width);
  if (r != -2) memcpy(out, vals + node * MAXL, 4 * n);
  free(vals);
  free(env.var_off);
  return r == -2 ? -2 : n;
}
