// felt.hpp — winter-math f128 field (p = 2^128 - 45*2^40 + 1) for gfx950 and host.
//
// Replaces `fields::f128::BaseElement` (reference: src/aggregation/air.rs:10).
// Storage is the canonical 16-byte little-endian value (two u64 limbs), so a
// felt array in HBM is byte-identical to winterfell's `elements_as_bytes` and
// can be hashed directly (Blake3_256::hash_elements, IS_CANONICAL).
//
// Multiplication: 4x4 schoolbook on 32-bit limbs (v_mad_u64_u32 chains), then a
// two-step special-form reduction using 2^128 = 45*2^40 - 1 (mod p):
// H*(45*2^40 - 1) is a small multiply, a shift and a subtraction — no second
// full-width multiply.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZKP_HD __host__ __device__ __forceinline__

struct __attribute__((aligned(16))) felt {
  uint64_t lo, hi;
};

namespace fp {

constexpr uint64_t P_LO = 0xffffd30000000001ULL;
constexpr uint64_t P_HI = 0xffffffffffffffffULL;
constexpr uint64_t C = 0x2cffffffffffULL;  // 2^128 mod p = 45*2^40 - 1

ZKP_HD felt make(uint64_t lo, uint64_t hi) { felt r; r.lo = lo; r.hi = hi; return r; }
ZKP_HD felt zero() { return make(0, 0); }
ZKP_HD felt one() { return make(1, 0); }
ZKP_HD felt from_u64(uint64_t v) { return make(v, 0); }
ZKP_HD bool eq(felt a, felt b) { return a.lo == b.lo && a.hi == b.hi; }
ZKP_HD bool is_zero(felt a) { return (a.lo | a.hi) == 0; }

ZKP_HD felt add_portable(felt a, felt b) {
  unsigned long long c1, c2, c3, c4;
  uint64_t s0 = __builtin_addcll(a.lo, b.lo, 0ULL, &c1);
  uint64_t s1 = __builtin_addcll(a.hi, b.hi, c1, &c2);
  // t = s + (2^128 - p) = s - p (mod 2^128); carry out <=> s >= p
  uint64_t t0 = __builtin_addcll(s0, C, 0ULL, &c3);
  uint64_t t1 = __builtin_addcll(s1, 0ULL, c3, &c4);
  bool take = (c2 | c4) != 0;
  return make(take ? t0 : s0, take ? t1 : s1);
}

ZKP_HD felt sub_portable(felt a, felt b) {
  unsigned long long b1, b2, c1, c2;
  uint64_t d0 = __builtin_subcll(a.lo, b.lo, 0ULL, &b1);
  uint64_t d1 = __builtin_subcll(a.hi, b.hi, b1, &b2);
  // on borrow add p (mod 2^128)
  uint64_t e0 = __builtin_addcll(d0, P_LO, 0ULL, &c1);
  uint64_t e1 = __builtin_addcll(d1, P_HI, c1, &c2);
  return make(b2 ? e0 : d0, b2 ? e1 : d1);
}


// reduce the 256-bit product r[0..7] (32-bit limbs, little-endian)
ZKP_HD felt reduce8(const uint32_t r[8]) {
  // m = 45 * H, H = r[4..7]
  uint64_t t = (uint64_t)r[4] * 45u;
  uint32_t m0 = (uint32_t)t;
  t = (t >> 32) + (uint64_t)r[5] * 45u;
  uint32_t m1 = (uint32_t)t;
  t = (t >> 32) + (uint64_t)r[6] * 45u;
  uint32_t m2 = (uint32_t)t;
  t = (t >> 32) + (uint64_t)r[7] * 45u;
  uint32_t m3 = (uint32_t)t;
  uint32_t m4 = (uint32_t)(t >> 32);
  // S = m * 2^40 occupies limbs 1..5
  uint32_t s1 = m0 << 8;
  uint32_t s2 = (m1 << 8) | (m0 >> 24);
  uint32_t s3 = (m2 << 8) | (m1 >> 24);
  uint32_t s4 = (m3 << 8) | (m2 >> 24);
  uint32_t s5 = (m4 << 8) | (m3 >> 24);
  // X = L + S - H  (>= 0, < 2^175)
  int64_t acc = (int64_t)r[0] - (int64_t)r[4];
  uint32_t x0 = (uint32_t)acc; acc >>= 32;
  acc += (int64_t)r[1] + (int64_t)s1 - (int64_t)r[5];
  uint32_t x1 = (uint32_t)acc; acc >>= 32;
  acc += (int64_t)r[2] + (int64_t)s2 - (int64_t)r[6];
  uint32_t x2 = (uint32_t)acc; acc >>= 32;
  acc += (int64_t)r[3] + (int64_t)s3 - (int64_t)r[7];
  uint32_t x3 = (uint32_t)acc; acc >>= 32;
  acc += (int64_t)s4;
  uint32_t x4 = (uint32_t)acc; acc >>= 32;
  acc += (int64_t)s5;
  uint32_t x5 = (uint32_t)acc;
  // Y = X_lo - X_hi + 45 * X_hi * 2^40, X_hi = x4 + x5*2^32 < 2^47
  uint64_t q = (uint64_t)x4 * 45u;
  uint32_t q0 = (uint32_t)q;
  uint32_t q1 = (uint32_t)(q >> 32) + x5 * 45u;  // < 2^21
  int64_t a2 = (int64_t)x0 - (int64_t)x4;
  uint32_t y0 = (uint32_t)a2; a2 >>= 32;
  a2 += (int64_t)x1 - (int64_t)x5 + (int64_t)(uint32_t)(q0 << 8);
  uint32_t y1 = (uint32_t)a2; a2 >>= 32;
  a2 += (int64_t)x2 + (int64_t)((q1 << 8) | (q0 >> 24));
  uint32_t y2 = (uint32_t)a2; a2 >>= 32;
  a2 += (int64_t)x3;
  uint32_t y3 = (uint32_t)a2; a2 >>= 32;  // a2 in {0, 1}: carry past 2^128
  uint64_t lo = (uint64_t)y0 | ((uint64_t)y1 << 32);
  uint64_t hi = (uint64_t)y2 | ((uint64_t)y3 << 32);
  unsigned long long c1, c2, c3, c4;
  // carry: value = 2^128 + (hi,lo) = (hi,lo) + C (mod p), and (hi,lo) < 2^94 there
  uint64_t add0 = a2 ? C : 0ULL;
  lo = __builtin_addcll(lo, add0, 0ULL, &c1);
  hi = __builtin_addcll(hi, 0ULL, c1, &c2);
  // final conditional subtraction of p
  uint64_t t0 = __builtin_addcll(lo, C, 0ULL, &c3);
  uint64_t t1 = __builtin_addcll(hi, 0ULL, c3, &c4);
  return c4 ? make(t0, t1) : make(lo, hi);
}

ZKP_HD felt mul_portable(felt a, felt b) {
  const uint32_t x0 = (uint32_t)a.lo, x1 = (uint32_t)(a.lo >> 32), x2 = (uint32_t)a.hi, x3 = (uint32_t)(a.hi >> 32);
  const uint32_t y0 = (uint32_t)b.lo, y1 = (uint32_t)(b.lo >> 32), y2 = (uint32_t)b.hi, y3 = (uint32_t)(b.hi >> 32);
  uint32_t r[8];
  uint64_t t;
  t = (uint64_t)x0 * y0;                 r[0] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x0 * y1;     r[1] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x0 * y2;     r[2] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x0 * y3;     r[3] = (uint32_t)t; r[4] = (uint32_t)(t >> 32);
  t = (uint64_t)x1 * y0 + r[1];          r[1] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x1 * y1 + r[2]; r[2] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x1 * y2 + r[3]; r[3] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x1 * y3 + r[4]; r[4] = (uint32_t)t; r[5] = (uint32_t)(t >> 32);
  t = (uint64_t)x2 * y0 + r[2];          r[2] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x2 * y1 + r[3]; r[3] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x2 * y2 + r[4]; r[4] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x2 * y3 + r[5]; r[5] = (uint32_t)t; r[6] = (uint32_t)(t >> 32);
  t = (uint64_t)x3 * y0 + r[3];          r[3] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x3 * y1 + r[4]; r[4] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x3 * y2 + r[5]; r[5] = (uint32_t)t;
  t = (t >> 32) + (uint64_t)x3 * y3 + r[6]; r[6] = (uint32_t)t; r[7] = (uint32_t)(t >> 32);
  return reduce8(r);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// host path: 64-bit limbs with 128-bit products (x86-64 mulq); same reduction
// identity 2^128 = C (mod p), applied twice, then one conditional subtraction
inline felt mul_host(felt a, felt b) {
  typedef unsigned __int128 u128;
  const u128 p00 = (u128)a.lo * b.lo, p01 = (u128)a.lo * b.hi, p10 = (u128)a.hi * b.lo, p11 = (u128)a.hi * b.hi;
  const u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  const uint64_t w0 = (uint64_t)p00, w1 = (uint64_t)mid;
  const u128 h = (mid >> 64) + (p01 >> 64) + (p10 >> 64) + p11;  // high 128 bits of the product
  const u128 t0 = (u128)(uint64_t)h * C + w0;
  const u128 t1 = (u128)(uint64_t)(h >> 64) * C + w1 + (uint64_t)(t0 >> 64);
  const u128 x = ((u128)(uint64_t)t1 << 64) | (uint64_t)t0;  // L + H*C = x + x2 * 2^128
  const uint64_t x2 = (uint64_t)(t1 >> 64);                   // < 2^47
  u128 s = x + (u128)x2 * C;
  if (s < x) s += C;  // wrapped past 2^128 (then s < 2^94: no second wrap)
  const u128 P = ((u128)P_HI << 64) | P_LO;
  if (s >= P) s -= P;
  return make((uint64_t)s, (uint64_t)(s >> 64));
}
#endif

}  // namespace fp

#if defined(__HIP_DEVICE_COMPILE__)
#include "felt_dev.hpp"
#endif

namespace fp {

// Public field ops: carry-chain asm on gfx950 (felt_dev.hpp), portable C on the host.
ZKP_HD felt add(felt a, felt b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fpd::add(a, b);
#else
  return add_portable(a, b);
#endif
}
ZKP_HD felt sub(felt a, felt b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fpd::sub(a, b);
#else
  return sub_portable(a, b);
#endif
}
ZKP_HD felt mul(felt a, felt b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fpd::mul(a, b);
#else
  return mul_host(a, b);
#endif
}
// a * k for a 32-bit k (fpd::mul_u32 on the device)
ZKP_HD felt mul_u32(felt a, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fpd::mul_u32(a, k);
#else
  return mul_host(a, make(k, 0));
#endif
}
ZKP_HD felt neg(felt a) { return sub(zero(), a); }
ZKP_HD felt sqr(felt a) { return mul(a, a); }

ZKP_HD felt pow_u64(felt b, uint64_t e) {
  felt r = one();
  while (e) {
    if (e & 1) r = mul(r, b);
    b = sqr(b);
    e >>= 1;
  }
  return r;
}

ZKP_HD felt sqr_n(felt a, int k) {
  for (int i = 0; i < k; i++) a = sqr(a);
  return a;
}

// x^(p-2); inv(0) = 0 like winter-math.
// p - 2 = [1 x 80][1101 0010][1 x 40] (binary, high to low): addition chain on
// a_k = x^(2^k - 1) — 135 squarings + 13 products (square-and-multiply: 252)
ZKP_HD felt inv(felt x) {
  felt a2 = mul(sqr(x), x);
  felt a4 = mul(sqr_n(a2, 2), a2);
  felt a8 = mul(sqr_n(a4, 4), a4);
  felt a16 = mul(sqr_n(a8, 8), a8);
  felt a32 = mul(sqr_n(a16, 16), a16);
  felt a64 = mul(sqr_n(a32, 32), a32);
  felt a40 = mul(sqr_n(a32, 8), a8);
  felt t = mul(sqr_n(a64, 16), a16);  // a80
  const int bits[8] = {1, 1, 0, 1, 0, 0, 1, 0};
  for (int i = 0; i < 8; i++) {
    t = sqr(t);
    if (bits[i]) t = mul(t, x);
  }
  return mul(sqr_n(t, 40), a40);
}

ZKP_HD felt from_u128_bytes(const uint8_t* p) {
  uint64_t lo = 0, hi = 0;
  for (int i = 7; i >= 0; i--) lo = (lo << 8) | p[i];
  for (int i = 15; i >= 8; i--) hi = (hi << 8) | p[i];
  return make(lo, hi);
}
ZKP_HD void to_bytes(felt a, uint8_t* p) {
  for (int i = 0; i < 8; i++) { p[i] = (uint8_t)(a.lo >> (8 * i)); p[8 + i] = (uint8_t)(a.hi >> (8 * i)); }
}
// value >= p ?  (canonical check used by the random coin's `from_random_bytes`)
ZKP_HD bool ge_p(felt a) { return a.hi == P_HI && a.lo >= P_LO; }

}  // namespace fp
