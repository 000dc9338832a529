// bvops.h — per-lane multi-limb bit-vector arithmetic for gfx950 (one model per lane).
//
// Values are L little-endian u32 limbs held in VGPRs, canonical (bits >= width are zero).
// Every loop is fully unrolled so limbs stay in statically named registers; widths and
// uniform shift amounts arrive in SGPRs, so width masks and limb moves are scalar-selected.
// Semantics: SMT-LIB 2.6 FixedSizeBitVectors, restated in
// oracle/cref.c; every helper here is checked against it by tests/test_gpu_parity.py.
#ifndef MQ_BVOPS_H
#define MQ_BVOPS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mq {

#define MQ_DEV __device__ __forceinline__

// mask word for limb i at width W (uniform)
MQ_DEV uint32_t limb_mask(int i, uint32_t W) {
  const uint32_t lo = 32u * (uint32_t)i;
  return W <= lo ? 0u : (W >= lo + 32u ? 0xFFFFFFFFu : ((1u << (W - lo)) - 1u));
}

template <int L, class T_x>
MQ_DEV void mask_w(T_x& x, uint32_t W) {
  if (W >= 32u * L) return;
#pragma unroll
  for (int i = 0; i < L; i++) x[i] &= limb_mask(i, W);
}

// sign-extend a canonical W-bit value to the full 32L bits (W uniform)
template <int L, class T_x>
MQ_DEV void sext_full(T_x& x, uint32_t W) {
  if (W >= 32u * L || W == 0) return;
  const uint32_t k = (W - 1) >> 5, b = (W - 1) & 31;
  uint32_t top = 0;
#pragma unroll
  for (int i = 0; i < L; i++) top |= ((uint32_t)i == k) ? x[i] : 0u;
  const uint32_t neg = ((top >> b) & 1u) ? 0xFFFFFFFFu : 0u;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const uint32_t keep = limb_mask(i, W);
    x[i] = (x[i] & keep) | (neg & ~keep);
  }
}

template <int L, class T_r, class T_a, class T_b>
MQ_DEV void add_n(T_r& r, const T_a& a, const T_b& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
}

template <int L, class T_r, class T_a, class T_b>
MQ_DEV uint32_t sub_n(T_r& r, const T_a& a, const T_b& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) r[i] = __builtin_subc(a[i], b[i], c, &c);
  return c;  // borrow out: a < b
}

template <int L, class T_x>
MQ_DEV void neg_n(T_x& x) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = __builtin_subc(0u, x[i], c, &c);
}

template <int L, class T_a, class T_b>
MQ_DEV bool ult_n(const T_a& a, const T_b& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) (void)__builtin_subc(a[i], b[i], c, &c);
  return c != 0;
}

template <int L, class T_a, class T_b>
MQ_DEV bool eq_n(const T_a& a, const T_b& b) {
  bool e = true;
#pragma unroll
  for (int i = 0; i < L; i++) e = e && (a[i] == b[i]);
  return e;
}

template <int L, class T_a>
MQ_DEV bool is_zero_n(const T_a& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; i++) acc |= a[i];
  return acc == 0;
}

// r = a*b mod 2^(32L)   (row-wise schoolbook, L(L+1)/2 partial products)
template <int L, class T_r, class T_a, class T_b>
MQ_DEV void mul_lo_n(T_r& r, const T_a& a, const T_b& b) {
  uint32_t t[L];
#pragma unroll
  for (int i = 0; i < L; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; i + j < L - 1; j++) {
      const uint64_t p = (uint64_t)a[i] * b[j] + (uint64_t)t[i + j] + carry;
      t[i + j] = (uint32_t)p;
      carry = (uint32_t)(p >> 32);
    }
    t[L - 1] += a[i] * b[L - 1 - i] + carry;
  }
#pragma unroll
  for (int i = 0; i < L; i++) r[i] = t[i];
}

// full 2L-limb product
template <int L, class T_lo, class T_hi, class T_a, class T_b>
MQ_DEV void mul_full_n(T_lo& lo, T_hi& hi, const T_a& a, const T_b& b) {
  uint32_t t[2 * L];
#pragma unroll
  for (int i = 0; i < 2 * L; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const uint64_t p = (uint64_t)a[i] * b[j] + (uint64_t)t[i + j] + carry;
      t[i + j] = (uint32_t)p;
      carry = (uint32_t)(p >> 32);
    }
    t[i + L] = carry;
  }
#pragma unroll
  for (int i = 0; i < L; i++) {
    lo[i] = t[i];
    hi[i] = t[i + L];
  }
}

// ---------------------------------------------------------------- shifts
// uniform right shift by s < 32L (zero fill)
template <int L, class T_x>
MQ_DEV void shr_uni(T_x& x, uint32_t s) {
  const uint32_t ls = s >> 5, bs = s & 31;
#pragma unroll
  for (int k = 1; k < L; k <<= 1) {
    if (ls & (uint32_t)k) {
#pragma unroll
      for (int i = 0; i < L; i++) x[i] = (i + k < L) ? x[i + k] : 0u;
    }
  }
  if (bs) {
#pragma unroll
    for (int i = 0; i < L; i++) x[i] = __builtin_amdgcn_alignbit(i + 1 < L ? x[i + 1] : 0u, x[i], bs);
  }
}

// uniform left shift by s < 32L
template <int L, class T_x>
MQ_DEV void shl_uni(T_x& x, uint32_t s) {
  const uint32_t ls = s >> 5, bs = s & 31;
#pragma unroll
  for (int k = 1; k < L; k <<= 1) {
    if (ls & (uint32_t)k) {
#pragma unroll
      for (int i = L - 1; i >= 0; i--) x[i] = (i >= k) ? x[i - k] : 0u;
    }
  }
  if (bs) {
#pragma unroll
    for (int i = L - 1; i >= 0; i--) x[i] = __builtin_amdgcn_alignbit(x[i], i > 0 ? x[i - 1] : 0u, 32u - bs);
  }
}

// per-lane left shift by s < 32L
template <int L, class T_x>
MQ_DEV void shl_var(T_x& x, uint32_t s) {
  const uint32_t ls = s >> 5, bs = s & 31;
#pragma unroll
  for (int k = 1; k < L; k <<= 1) {
    const bool c = (ls & (uint32_t)k) != 0;
#pragma unroll
    for (int i = L - 1; i >= 0; i--) x[i] = c ? ((i >= k) ? x[i - k] : 0u) : x[i];
  }
#pragma unroll
  for (int i = L - 1; i >= 1; i--) x[i] = (x[i] << bs) | ((x[i - 1] >> 1) >> (31u - bs));
  x[0] <<= bs;
}

// per-lane right shift by s < 32L with fill word (0 or ~0)
template <int L, class T_x>
MQ_DEV void shr_var(T_x& x, uint32_t s, uint32_t fill) {
  const uint32_t ls = s >> 5, bs = s & 31;
#pragma unroll
  for (int k = 1; k < L; k <<= 1) {
    const bool c = (ls & (uint32_t)k) != 0;
#pragma unroll
    for (int i = 0; i < L; i++) x[i] = c ? ((i + k < L) ? x[i + k] : fill) : x[i];
  }
#pragma unroll
  for (int i = 0; i < L; i++) x[i] = __builtin_amdgcn_alignbit(i + 1 < L ? x[i + 1] : fill, x[i], bs);
}

// shift amount of a W-bit canonical value: returns true (and s) when amount < W
template <int L, class T_b>
MQ_DEV bool shift_amount(const T_b& b, uint32_t W, uint32_t& s) {
  uint32_t hi = 0;
#pragma unroll
  for (int i = 1; i < L; i++) hi |= b[i];
  s = b[0];
  return hi == 0 && b[0] < W;
}

// ---------------------------------------------------------------- division
// unsigned q = a / b, r = a % b at full 32L bits; b == 0 -> q = all ones, r = a.
// Restoring radix-2 division, skipping the dividend limbs that are zero in every lane.
template <int L, class T_q, class T_r, class T_a, class T_b>
MQ_DEV void udivrem_n(T_q& q, T_r& r, const T_a& a, const T_b& b) {
  int top = 0;
#pragma unroll
  for (int i = L - 1; i >= 0; i--) {
    if (top == 0 && __ballot(a[i] != 0u)) top = i + 1;
  }
#pragma unroll
  for (int i = 0; i < L; i++) {
    q[i] = a[i];
    r[i] = 0;
  }
  shl_uni<L>(q, 32u * (uint32_t)(L - top));
  const bool bz = is_zero_n<L>(b);
  for (int it = 0; it < 32 * top; it++) {
    const uint32_t rtop = r[L - 1] >> 31;
    const uint32_t qtop = q[L - 1] >> 31;
#pragma unroll
    for (int i = L - 1; i >= 1; i--) r[i] = __builtin_amdgcn_alignbit(r[i], r[i - 1], 31u);
    r[0] = (r[0] << 1) | qtop;
#pragma unroll
    for (int i = L - 1; i >= 1; i--) q[i] = __builtin_amdgcn_alignbit(q[i], q[i - 1], 31u);
    q[0] <<= 1;
    uint32_t t[L];
    const uint32_t borrow = sub_n<L>(t, r, b);
    const bool ge = rtop != 0u || borrow == 0u;
#pragma unroll
    for (int i = 0; i < L; i++) r[i] = ge ? t[i] : r[i];
    q[0] |= ge ? 1u : 0u;
  }
#pragma unroll
  for (int i = 0; i < L; i++) {
    q[i] = bz ? 0xFFFFFFFFu : q[i];
    r[i] = bz ? a[i] : r[i];
  }
}

}  // namespace mq
#endif
