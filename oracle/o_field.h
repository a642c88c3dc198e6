/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into libzkp.so.
 *
 * f128 prime field of winter-math 0.12 (`fields::f128::BaseElement`, used by
 * the reference at src/aggregation/air.rs:10, src/training/air.rs:13,
 * src/helper.rs:11). The crate is not vendored; constants are
 * pinned by SURVEY.md F1 / Appendix D and tests/golden/f128.json.
 *   p = 2^128 - 45*2^40 + 1, GENERATOR = 3, TWO_ADICITY = 40.
 * Elements are canonical u128 (< p). Plain C with unsigned __int128.
 */
#ifndef O_FIELD_H
#define O_FIELD_H
#include <stdint.h>

typedef unsigned __int128 u128;

#define O_P ((((u128)0xffffffffffffffffULL) << 64) | (u128)0xffffd30000000001ULL)
/* 2^128 mod p = 45*2^40 - 1 */
#define O_C ((u128)0x2cffffffffffULL)
#define O_TWO_ADICITY 40

static inline u128 o_new(u128 v) { return v >= O_P ? v - O_P : v; }

static inline u128 o_add(u128 a, u128 b) {
  u128 s = a + b;
  if (s < a) s += O_C; /* carried out of 2^128 */
  if (s >= O_P) s -= O_P;
  return s;
}

static inline u128 o_sub(u128 a, u128 b) {
  u128 d = a - b;
  if (a < b) d += O_P;
  return d;
}

static inline u128 o_neg(u128 a) { return a == 0 ? 0 : O_P - a; }

/* reduce hi*2^128 + lo using 2^128 = C (mod p) */
static inline u128 o_reduce(u128 hi, u128 lo) {
  uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
  u128 x0 = (u128)h0 * (uint64_t)O_C;          /* < 2^110 */
  u128 x1 = (u128)h1 * (uint64_t)O_C;          /* < 2^110, weight 2^64 */
  /* t = lo + x0 + (x1 << 64): 3-limb */
  u128 t = lo + x0;
  uint64_t top = (t < lo);
  u128 x1lo = x1 << 64;
  u128 t2 = t + x1lo;
  top += (t2 < t);
  top += (uint64_t)(x1 >> 64);
  /* value = top*2^128 + t2, top < 2^47 */
  u128 r = t2 + (u128)top * (uint64_t)O_C;
  if (r < t2) r += O_C;
  if (r >= O_P) r -= O_P;
  return r;
}

static inline u128 o_mul(u128 a, u128 b) {
  uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64);
  uint64_t b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  u128 mid = p01 + p10;
  u128 midc = (mid < p01) ? ((u128)1 << 64) : 0;
  u128 lo = p00 + (mid << 64);
  u128 c1 = lo < p00;
  u128 hi = p11 + (mid >> 64) + midc + c1;
  return o_reduce(hi, lo);
}

static inline u128 o_sq(u128 a) { return o_mul(a, a); }

static inline u128 o_exp(u128 b, u128 e) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = o_mul(r, b);
    b = o_mul(b, b);
    e >>= 1;
  }
  return r;
}

/* winter-math `inv`: inv(0) = 0 */
static inline u128 o_inv(u128 a) { return a == 0 ? 0 : o_exp(a, O_P - 2); }

static inline u128 o_two_adic_root(void) {
  /* 23953097886125630542083529559205016746 */
  return ((u128)0x120532e7b364080aULL << 64) | (u128)0x86b8723e1920f4aaULL;
}

/* StarkField::get_root_of_unity(log_n) = ROOT^(2^(40 - log_n)) */
static inline u128 o_root_of_unity(unsigned log_n) {
  u128 r = o_two_adic_root();
  for (unsigned i = log_n; i < O_TWO_ADICITY; i++) r = o_sq(r);
  return r;
}

static inline u128 o_load(const uint8_t* p) {
  u128 v = 0;
  for (int i = 15; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
static inline void o_store(uint8_t* p, u128 v) {
  for (int i = 0; i < 16; i++) { p[i] = (uint8_t)v; v >>= 8; }
}

#endif
