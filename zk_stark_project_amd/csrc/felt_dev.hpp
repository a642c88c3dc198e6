// felt_dev.hpp — gfx950 carry-chain implementations of the f128 field ops.
//
// hipcc lowers 64-bit add-with-carry to 64-bit adds + 64-bit compares +
// selects; here every carry lives in an SGPR pair (the per-lane carry mask)
// and flows through v_add_co/v_addc_co/v_sub_co/v_subb_co and the carry-out of
// v_mad_u64_u32, so a 128-bit add is 4 VALU ops + the select. Only the
// instruction choice is pinned (non-volatile asm): scheduling and register
// allocation stay with the compiler. Semantics are identical to the portable
// versions in felt.hpp (checked bit-exactly by the GPU parity tests).
#pragma once
#include <stdint.h>
// included from felt.hpp inside the device compilation pass only

// ZKP_ASM_VOLATILE (tuning experiment): volatile asm keeps the source order of
// the carry chains (the interleaving below) instead of the machine scheduler's
#ifdef ZKP_ASM_VOLATILE
#define ZKP_ASM asm volatile
#else
#define ZKP_ASM asm
#endif

namespace fpd {

// ---- 32-bit carry-chain primitives (carry masks in SGPR pairs)
__device__ __forceinline__ uint32_t add_co(uint32_t a, uint32_t b, uint64_t& co) {
  uint32_t r;
  ZKP_ASM("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(co) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t addc_co(uint32_t a, uint32_t b, uint64_t ci, uint64_t& co) {
  uint32_t r;
  ZKP_ASM("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(co) : "v"(a), "v"(b), "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint64_t ci) {
  uint32_t r;
  uint64_t dead;
  ZKP_ASM("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(dead) : "v"(a), "v"(b), "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& bo) {
  uint32_t r;
  ZKP_ASM("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(bo) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t subb_co(uint32_t a, uint32_t b, uint64_t bi, uint64_t& bo) {
  uint32_t r;
  ZKP_ASM("v_subb_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(bo) : "v"(a), "v"(b), "s"(bi));
  return r;
}
__device__ __forceinline__ uint32_t subb(uint32_t a, uint32_t b, uint64_t bi) {
  uint32_t r;
  uint64_t dead;
  ZKP_ASM("v_subb_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(dead) : "v"(a), "v"(b), "s"(bi));
  return r;
}
// d = a*b + c (64-bit), carry-out of the 64-bit add in co
__device__ __forceinline__ uint64_t mad_co(uint32_t a, uint32_t b, uint64_t c, uint64_t& co) {
  uint64_t d;
  ZKP_ASM("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t d, dead;
  ZKP_ASM("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(dead) : "v"(a), "v"(b), "v"(c));
  return d;
}
// the same with an inline-constant operand (-1 = 0xffffffff or 0), which
// needs no VGPR (VOP3 takes inline constants; 0x2cff is not one)
__device__ __forceinline__ uint32_t add_co_m1(uint32_t a, uint64_t& co) {
  uint32_t r;
  ZKP_ASM("v_add_co_u32_e64 %0, %1, %2, -1" : "=v"(r), "=s"(co) : "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t addc_co_0(uint32_t a, uint64_t ci, uint64_t& co) {
  uint32_t r;
  ZKP_ASM("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(a), "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t addc_0(uint32_t a, uint64_t ci) {
  uint32_t r;
  uint64_t dead;
  ZKP_ASM("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(dead) : "v"(a), "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t carry_0(uint64_t ci) {  // 0 + 0 + carry
  uint32_t r;
  uint64_t dead;
  ZKP_ASM("v_addc_co_u32_e64 %0, %1, 0, 0, %2" : "=v"(r), "=s"(dead) : "s"(ci));
  return r;
}
__device__ __forceinline__ uint32_t subb_co_0(uint32_t a, uint64_t bi, uint64_t& bo) {
  uint32_t r;
  ZKP_ASM("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(bo) : "v"(a), "s"(bi));
  return r;
}
__device__ __forceinline__ uint32_t subb_0(uint32_t a, uint64_t bi) {
  uint32_t r;
  uint64_t dead;
  ZKP_ASM("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(dead) : "v"(a), "s"(bi));
  return r;
}
__device__ __forceinline__ uint32_t sel_0_m1(uint64_t m) {  // m ? 0xffffffff : 0
  uint32_t r;
  ZKP_ASM("v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(r) : "s"(m));
  return r;
}
__device__ __forceinline__ uint64_t mul_wide(uint32_t a, uint32_t b) {  // a*b + 0 (inline)
  uint64_t d, dead;
  ZKP_ASM("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(d), "=s"(dead) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint64_t or_mask(uint64_t a, uint64_t b) {
  uint64_t r;
  ZKP_ASM("s_or_b64 %0, %1, %2" : "=s"(r) : "s"(a), "s"(b) : "scc");
  return r;
}
__device__ __forceinline__ uint32_t sel(uint32_t f, uint32_t t, uint64_t m) {  // m ? t : f
  uint32_t r;
  ZKP_ASM("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}

struct L4 {
  uint32_t w0, w1, w2, w3;
};
__device__ __forceinline__ L4 split(felt a) {
  return {(uint32_t)a.lo, (uint32_t)(a.lo >> 32), (uint32_t)a.hi, (uint32_t)(a.hi >> 32)};
}
__device__ __forceinline__ felt join(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  felt r;
  r.lo = (uint64_t)w0 | ((uint64_t)w1 << 32);
  r.hi = (uint64_t)w2 | ((uint64_t)w3 << 32);
  return r;
}

constexpr uint32_t C0 = 0xffffffffu;  // 2^128 - p = 0x2cff_ffffffff
constexpr uint32_t C1 = 0x2cffu;
constexpr uint32_t P1 = 0xffffd300u;  // p = 0xffffffff_ffffffff_ffffd300_00000001

// s + C (= s - p mod 2^128) with its carry-out; result = (k | carry) ? s - p : s
__device__ __forceinline__ felt canon_from(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint64_t k) {
  uint64_t c;
  uint32_t t0 = add_co_m1(s0, c);
  uint32_t t1 = addc_co(s1, C1, c, c);
  uint32_t t2 = addc_co_0(s2, c, c);
  uint32_t t3 = addc_co_0(s3, c, c);
  uint64_t m = or_mask(k, c);
  return join(sel(s0, t0, m), sel(s1, t1, m), sel(s2, t2, m), sel(s3, t3, m));
}

__device__ __forceinline__ felt add(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t c;
  uint32_t s0 = add_co(x.w0, y.w0, c);
  uint32_t s1 = addc_co(x.w1, y.w1, c, c);
  uint32_t s2 = addc_co(x.w2, y.w2, c, c);
  uint32_t s3 = addc_co(x.w3, y.w3, c, c);
  return canon_from(s0, s1, s2, s3, c);
}

__device__ __forceinline__ felt sub(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t bw;
  uint32_t d0 = sub_co(x.w0, y.w0, bw);
  uint32_t d1 = subb_co(x.w1, y.w1, bw, bw);
  uint32_t d2 = subb_co(x.w2, y.w2, bw, bw);
  uint32_t d3 = subb_co(x.w3, y.w3, bw, bw);
  // on borrow: d - C (mod 2^128) == d + p
  uint32_t m0 = sel_0_m1(bw), m1 = sel(0u, C1, bw);
  uint64_t b2;
  uint32_t e0 = sub_co(d0, m0, b2);
  uint32_t e1 = subb_co(d1, m1, b2, b2);
  uint32_t e2 = subb_co_0(d2, b2, b2);
  uint32_t e3 = subb_0(d3, b2);
  return join(e0, e1, e2, e3);
}

// 256-bit product in 32-bit limbs (product scanning, 96-bit column accumulator)
__device__ __forceinline__ void mul256(L4 x, L4 y, uint32_t r[8]) {
  uint64_t acc, c;
  uint32_t ov;
  // column 0
  acc = mul_wide(x.w0, y.w0);
  r[0] = (uint32_t)acc;
  acc >>= 32;
  // column 1
  acc = mad_co(x.w0, y.w1, acc, c); ov = carry_0(c);
  acc = mad_co(x.w1, y.w0, acc, c); ov = addc_0(ov, c);
  r[1] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)ov << 32);
  // column 2
  acc = mad_co(x.w0, y.w2, acc, c); ov = carry_0(c);
  acc = mad_co(x.w1, y.w1, acc, c); ov = addc_0(ov, c);
  acc = mad_co(x.w2, y.w0, acc, c); ov = addc_0(ov, c);
  r[2] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)ov << 32);
  // column 3
  acc = mad_co(x.w0, y.w3, acc, c); ov = carry_0(c);
  acc = mad_co(x.w1, y.w2, acc, c); ov = addc_0(ov, c);
  acc = mad_co(x.w2, y.w1, acc, c); ov = addc_0(ov, c);
  acc = mad_co(x.w3, y.w0, acc, c); ov = addc_0(ov, c);
  r[3] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)ov << 32);
  // column 4
  acc = mad_co(x.w1, y.w3, acc, c); ov = carry_0(c);
  acc = mad_co(x.w2, y.w2, acc, c); ov = addc_0(ov, c);
  acc = mad_co(x.w3, y.w1, acc, c); ov = addc_0(ov, c);
  r[4] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)ov << 32);
  // column 5
  acc = mad_co(x.w2, y.w3, acc, c); ov = carry_0(c);
  acc = mad_co(x.w3, y.w2, acc, c); ov = addc_0(ov, c);
  r[5] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)ov << 32);
  // column 6 (cannot overflow: the full product is < 2^256)
  acc = mad(x.w3, y.w3, acc);
  r[6] = (uint32_t)acc;
  r[7] = (uint32_t)(acc >> 32);
}

// reduce hi*2^128 + lo with 2^128 = 0x2D00*2^32 - 1 (mod p)
__device__ __forceinline__ felt reduce(const uint32_t r[8]) {
  const uint32_t K = 0x2d00u;  // 45 * 2^8
  // q = H * K (5 limbs)
  uint64_t t = mul_wide(r[4], K);
  uint32_t q0 = (uint32_t)t;
  t = mad(r[5], K, t >> 32);
  uint32_t q1 = (uint32_t)t;
  t = mad(r[6], K, t >> 32);
  uint32_t q2 = (uint32_t)t;
  t = mad(r[7], K, t >> 32);
  uint32_t q3 = (uint32_t)t, q4 = (uint32_t)(t >> 32);
  // X = L + q*2^32 - H  (6 limbs, X >= 0, X < 2^175)
  uint64_t c;
  uint32_t s1 = add_co(r[1], q0, c);
  uint32_t s2 = addc_co(r[2], q1, c, c);
  uint32_t s3 = addc_co(r[3], q2, c, c);
  uint32_t s4 = addc_co_0(q3, c, c);
  uint32_t s5 = addc_0(q4, c);
  uint64_t b;
  uint32_t x0 = sub_co(r[0], r[4], b);
  uint32_t x1 = subb_co(s1, r[5], b, b);
  uint32_t x2 = subb_co(s2, r[6], b, b);
  uint32_t x3 = subb_co(s3, r[7], b, b);
  uint32_t x4 = subb_co_0(s4, b, b);
  uint32_t x5 = subb_0(s5, b);
  // Y = Xl + (Xh*K)*2^32 - Xh, Xh = x4 + x5*2^32 < 2^47
  uint64_t u = mul_wide(x4, K);
  uint32_t u0 = (uint32_t)u;
  uint32_t u1 = (uint32_t)(u >> 32) + x5 * K;  // < 2^29
  uint32_t y1 = add_co(x1, u0, c);
  uint32_t y2 = addc_co(x2, u1, c, c);
  uint32_t y3 = addc_co_0(x3, c, c);
  uint64_t top = c;  // carry past 2^128
  uint32_t z0 = sub_co(x0, x4, b);
  uint32_t z1 = subb_co(y1, x5, b, b);
  uint32_t z2 = subb_co_0(y2, b, b);
  uint32_t z3 = subb_co_0(y3, b, b);
  // net bit 128 = top - borrow (>= 0 overall); set when top & !borrow
  uint64_t k;
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k) : "s"(top), "s"(b) : "scc");
  return canon_from(z0, z1, z2, z3, k);
}

__device__ __forceinline__ felt mul(felt a, felt b) {
  uint32_t r[8];
  mul256(split(a), split(b), r);
  return reduce(r);
}

// a * k for a 32-bit k (e.g. GlobalUpdate's k = devices * 10^6): a 160-bit product
// and one fold of its top limb r4 (r4 * 2^128 = r4 * K * 2^32 - r4, K = 0x2d00),
// ~21 VALU instructions instead of mul's ~63
__device__ __forceinline__ felt mul_u32(felt a, uint32_t k) {
  const L4 x = split(a);
  uint64_t t = mul_wide(x.w0, k);
  const uint32_t r0 = (uint32_t)t;
  t = mad(x.w1, k, t >> 32);
  const uint32_t r1 = (uint32_t)t;
  t = mad(x.w2, k, t >> 32);
  const uint32_t r2 = (uint32_t)t;
  t = mad(x.w3, k, t >> 32);
  const uint32_t r3 = (uint32_t)t, r4 = (uint32_t)(t >> 32);
  const uint64_t u = mul_wide(r4, 0x2d00u);  // < 2^46
  uint64_t c, b;
  const uint32_t s1 = add_co(r1, (uint32_t)u, c);
  const uint32_t s2 = addc_co(r2, (uint32_t)(u >> 32), c, c);
  const uint32_t s3 = addc_co_0(r3, c, c);  // c: bit 128
  const uint32_t z0 = sub_co(r0, r4, b);
  const uint32_t z1 = subb_co_0(s1, b, b);
  const uint32_t z2 = subb_co_0(s2, b, b);
  const uint32_t z3 = subb_co_0(s3, b, b);
  // net bit 128 = c - borrow (the value is >= 0): set when c & !borrow
  uint64_t kk;
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(kk) : "s"(c), "s"(b) : "scc");
  return canon_from(z0, z1, z2, z3, kk);
}


// Two independent products with their instruction streams interleaved, so that
// each SGPR carry is consumed >= 2 instructions after it is produced (gfx950
// needs 2 wait states between a VALU carry-out and its VALU consumer; with
// one chain the compiler pads with s_nop).
__device__ __forceinline__ void mul256x2(L4 x, L4 y, L4 u, L4 v, uint32_t r[8], uint32_t s[8]) {
  uint64_t acc, c, bcc, d;
  uint32_t ov, bov;
  acc = mul_wide(x.w0, y.w0);
  bcc = mul_wide(u.w0, v.w0);
  r[0] = (uint32_t)acc; acc >>= 32;
  s[0] = (uint32_t)bcc; bcc >>= 32;
#define ZKP_COL_BEGIN(i0, j0)                      \
  acc = mad_co(x.w##i0, y.w##j0, acc, c);          \
  bcc = mad_co(u.w##i0, v.w##j0, bcc, d);          \
  ov = carry_0(c);                                 \
  bov = carry_0(d);
#define ZKP_COL_STEP(i0, j0)                       \
  acc = mad_co(x.w##i0, y.w##j0, acc, c);          \
  bcc = mad_co(u.w##i0, v.w##j0, bcc, d);          \
  ov = addc_0(ov, c);                              \
  bov = addc_0(bov, d);
#define ZKP_COL_END(k)                             \
  r[k] = (uint32_t)acc;                            \
  s[k] = (uint32_t)bcc;                            \
  acc = (acc >> 32) | ((uint64_t)ov << 32);        \
  bcc = (bcc >> 32) | ((uint64_t)bov << 32);
  ZKP_COL_BEGIN(0, 1) ZKP_COL_STEP(1, 0) ZKP_COL_END(1)
  ZKP_COL_BEGIN(0, 2) ZKP_COL_STEP(1, 1) ZKP_COL_STEP(2, 0) ZKP_COL_END(2)
  ZKP_COL_BEGIN(0, 3) ZKP_COL_STEP(1, 2) ZKP_COL_STEP(2, 1) ZKP_COL_STEP(3, 0) ZKP_COL_END(3)
  ZKP_COL_BEGIN(1, 3) ZKP_COL_STEP(2, 2) ZKP_COL_STEP(3, 1) ZKP_COL_END(4)
  ZKP_COL_BEGIN(2, 3) ZKP_COL_STEP(3, 2) ZKP_COL_END(5)
#undef ZKP_COL_BEGIN
#undef ZKP_COL_STEP
#undef ZKP_COL_END
  acc = mad(x.w3, y.w3, acc);
  bcc = mad(u.w3, v.w3, bcc);
  r[6] = (uint32_t)acc; r[7] = (uint32_t)(acc >> 32);
  s[6] = (uint32_t)bcc; s[7] = (uint32_t)(bcc >> 32);
}

// Two independent reductions, interleaved like mul256x2.
__device__ __forceinline__ void reduce_x2(const uint32_t r[8], const uint32_t s[8], felt& out_r, felt& out_s) {
  const uint32_t K = 0x2d00u;
  uint64_t t = mul_wide(r[4], K), tt = mul_wide(s[4], K);
  uint32_t q0 = (uint32_t)t, p0 = (uint32_t)tt;
  t = mad(r[5], K, t >> 32); tt = mad(s[5], K, tt >> 32);
  uint32_t q1 = (uint32_t)t, p1 = (uint32_t)tt;
  t = mad(r[6], K, t >> 32); tt = mad(s[6], K, tt >> 32);
  uint32_t q2 = (uint32_t)t, p2 = (uint32_t)tt;
  t = mad(r[7], K, t >> 32); tt = mad(s[7], K, tt >> 32);
  uint32_t q3 = (uint32_t)t, q4 = (uint32_t)(t >> 32), p3 = (uint32_t)tt, p4 = (uint32_t)(tt >> 32);
  uint64_t c, e, b, f;
  uint32_t s1 = add_co(r[1], q0, c);
  uint32_t S1 = add_co(s[1], p0, e);
  uint32_t x0 = sub_co(r[0], r[4], b);
  uint32_t X0 = sub_co(s[0], s[4], f);
  uint32_t s2 = addc_co(r[2], q1, c, c);
  uint32_t S2 = addc_co(s[2], p1, e, e);
  uint32_t x1 = subb_co(s1, r[5], b, b);
  uint32_t X1 = subb_co(S1, s[5], f, f);
  uint32_t s3 = addc_co(r[3], q2, c, c);
  uint32_t S3 = addc_co(s[3], p2, e, e);
  uint32_t x2 = subb_co(s2, r[6], b, b);
  uint32_t X2 = subb_co(S2, s[6], f, f);
  uint32_t s4 = addc_co_0(q3, c, c);
  uint32_t S4 = addc_co_0(p3, e, e);
  uint32_t x3 = subb_co(s3, r[7], b, b);
  uint32_t X3 = subb_co(S3, s[7], f, f);
  uint32_t s5 = addc_0(q4, c);
  uint32_t S5 = addc_0(p4, e);
  uint32_t x4 = subb_co_0(s4, b, b);
  uint32_t X4 = subb_co_0(S4, f, f);
  uint32_t x5 = subb_0(s5, b);
  uint32_t X5 = subb_0(S5, f);
  uint64_t uu = mul_wide(x4, K), UU = mul_wide(X4, K);
  uint32_t u0 = (uint32_t)uu, U0 = (uint32_t)UU;
  uint32_t u1 = (uint32_t)(uu >> 32) + x5 * K, U1 = (uint32_t)(UU >> 32) + X5 * K;
  uint32_t y1 = add_co(x1, u0, c);
  uint32_t Y1 = add_co(X1, U0, e);
  uint32_t z0 = sub_co(x0, x4, b);
  uint32_t Z0 = sub_co(X0, X4, f);
  uint32_t y2 = addc_co(x2, u1, c, c);
  uint32_t Y2 = addc_co(X2, U1, e, e);
  uint32_t z1 = subb_co(y1, x5, b, b);
  uint32_t Z1 = subb_co(Y1, X5, f, f);
  uint32_t y3 = addc_co_0(x3, c, c);
  uint32_t Y3 = addc_co_0(X3, e, e);
  uint32_t z2 = subb_co_0(y2, b, b);
  uint32_t Z2 = subb_co_0(Y2, f, f);
  uint32_t z3 = subb_co_0(y3, b, b);
  uint32_t Z3 = subb_co_0(Y3, f, f);
  uint64_t k1, k2;
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k1) : "s"(c), "s"(b) : "scc");
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k2) : "s"(e), "s"(f) : "scc");
  // canonicalize both (interleaved)
  uint64_t g1, g2;
  uint32_t t0 = add_co_m1(z0, g1);
  uint32_t T0 = add_co_m1(Z0, g2);
  uint32_t t1 = addc_co(z1, C1, g1, g1);
  uint32_t T1 = addc_co(Z1, C1, g2, g2);
  uint32_t t2 = addc_co_0(z2, g1, g1);
  uint32_t T2 = addc_co_0(Z2, g2, g2);
  uint32_t t3 = addc_co_0(z3, g1, g1);
  uint32_t T3 = addc_co_0(Z3, g2, g2);
  uint64_t m1 = or_mask(k1, g1), m2 = or_mask(k2, g2);
  out_r = join(sel(z0, t0, m1), sel(z1, t1, m1), sel(z2, t2, m1), sel(z3, t3, m1));
  out_s = join(sel(Z0, T0, m2), sel(Z1, T1, m2), sel(Z2, T2, m2), sel(Z3, T3, m2));
}

__device__ __forceinline__ void mul_x2(felt a, felt b, felt c, felt d, felt& ab, felt& cd) {
  uint32_t r[8], s[8];
  mul256x2(split(a), split(b), split(c), split(d), r, s);
  reduce_x2(r, s, ab, cd);
}

// x + y and x - y with the two carry chains interleaved (the butterfly's add/sub pair)
__device__ __forceinline__ void addsub(felt a, felt b, felt& sum, felt& diff) {
  L4 x = split(a), y = split(b);
  uint64_t c, bw;
  uint32_t s0 = add_co(x.w0, y.w0, c);
  uint32_t d0 = sub_co(x.w0, y.w0, bw);
  uint32_t s1 = addc_co(x.w1, y.w1, c, c);
  uint32_t d1 = subb_co(x.w1, y.w1, bw, bw);
  uint32_t s2 = addc_co(x.w2, y.w2, c, c);
  uint32_t d2 = subb_co(x.w2, y.w2, bw, bw);
  uint32_t s3 = addc_co(x.w3, y.w3, c, c);
  uint32_t d3 = subb_co(x.w3, y.w3, bw, bw);
  uint64_t g, b2;
  uint32_t m0 = sel_0_m1(bw), m1 = sel(0u, C1, bw);
  uint32_t t0 = add_co_m1(s0, g);
  uint32_t e0 = sub_co(d0, m0, b2);
  uint32_t t1 = addc_co(s1, C1, g, g);
  uint32_t e1 = subb_co(d1, m1, b2, b2);
  uint32_t t2 = addc_co_0(s2, g, g);
  uint32_t e2 = subb_co_0(d2, b2, b2);
  uint32_t t3 = addc_co_0(s3, g, g);
  uint32_t e3 = subb_0(d3, b2);
  uint64_t m = or_mask(c, g);
  sum = join(sel(s0, t0, m), sel(s1, t1, m), sel(s2, t2, m), sel(s3, t3, m));
  diff = join(e0, e1, e2, e3);
}


// N independent products with every step issued for all N chains before the
// next step: each SGPR carry is consumed N instructions after it is produced,
// so with N >= 3 no s_nop is needed for the carry hazard (N = 2 leaves one
// wait state per step, which the compiler fills with s_nop 0: ~25% of the
// NTT's instructions were such nops). Loops have constant trip counts and are
// fully unrolled, so every array below lives in registers.
template <int N>
__device__ __forceinline__ void mul_xn(const felt* a, const felt* b, felt* out) {
  L4 x[N], y[N];
  uint32_t r[N][8];
  uint64_t acc[N], c[N];
  uint32_t ov[N];
#pragma unroll
  for (int k = 0; k < N; k++) { x[k] = split(a[k]); y[k] = split(b[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) acc[k] = mul_wide(x[k].w0, y[k].w0);
#pragma unroll
  for (int k = 0; k < N; k++) { r[k][0] = (uint32_t)acc[k]; acc[k] >>= 32; }
  auto wi = [](const L4& v, int i) { return i == 0 ? v.w0 : i == 1 ? v.w1 : i == 2 ? v.w2 : v.w3; };
  // column col = i + j over the pairs (i, j); first pair starts the overflow word
#define ZKP_XN_COL(col, ...)                                                            \
  {                                                                                     \
    constexpr int pairs[][2] = {__VA_ARGS__};                                           \
    constexpr int np = sizeof(pairs) / sizeof(pairs[0]);                                \
    _Pragma("unroll") for (int q = 0; q < np; q++) {                                    \
      _Pragma("unroll") for (int k = 0; k < N; k++)                                     \
        acc[k] = mad_co(wi(x[k], pairs[q][0]), wi(y[k], pairs[q][1]), acc[k], c[k]);    \
      _Pragma("unroll") for (int k = 0; k < N; k++)                                     \
        ov[k] = q == 0 ? carry_0(c[k]) : addc_0(ov[k], c[k]);                           \
    }                                                                                   \
    _Pragma("unroll") for (int k = 0; k < N; k++) {                                     \
      r[k][col] = (uint32_t)acc[k];                                                     \
      acc[k] = (acc[k] >> 32) | ((uint64_t)ov[k] << 32);                                \
    }                                                                                   \
  }
  ZKP_XN_COL(1, {0, 1}, {1, 0})
  ZKP_XN_COL(2, {0, 2}, {1, 1}, {2, 0})
  ZKP_XN_COL(3, {0, 3}, {1, 2}, {2, 1}, {3, 0})
  ZKP_XN_COL(4, {1, 3}, {2, 2}, {3, 1})
  ZKP_XN_COL(5, {2, 3}, {3, 2})
#undef ZKP_XN_COL
#pragma unroll
  for (int k = 0; k < N; k++) acc[k] = mad(x[k].w3, y[k].w3, acc[k]);  // column 6 cannot overflow
#pragma unroll
  for (int k = 0; k < N; k++) { r[k][6] = (uint32_t)acc[k]; r[k][7] = (uint32_t)(acc[k] >> 32); }
  // reduction (as reduce(), N chains interleaved step by step)
  const uint32_t K = 0x2d00u;
  uint32_t q0[N], q1[N], q2[N], q3[N], q4[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint64_t t = mul_wide(r[k][4], K);
    q0[k] = (uint32_t)t;
    t = mad(r[k][5], K, t >> 32);
    q1[k] = (uint32_t)t;
    t = mad(r[k][6], K, t >> 32);
    q2[k] = (uint32_t)t;
    t = mad(r[k][7], K, t >> 32);
    q3[k] = (uint32_t)t;
    q4[k] = (uint32_t)(t >> 32);
  }
  uint64_t cc[N], bb[N];
  uint32_t s1[N], s2[N], s3[N], s4[N], s5[N], x0[N], x1[N], x2[N], x3[N], x4[N], x5[N];
#pragma unroll
  for (int k = 0; k < N; k++) s1[k] = add_co(r[k][1], q0[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x0[k] = sub_co(r[k][0], r[k][4], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) s2[k] = addc_co(r[k][2], q1[k], cc[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x1[k] = subb_co(s1[k], r[k][5], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) s3[k] = addc_co(r[k][3], q2[k], cc[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x2[k] = subb_co(s2[k], r[k][6], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) s4[k] = addc_co_0(q3[k], cc[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x3[k] = subb_co(s3[k], r[k][7], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) s5[k] = addc_0(q4[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x4[k] = subb_co_0(s4[k], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) x5[k] = subb_0(s5[k], bb[k]);
  uint32_t u0[N], u1[N], y1[N], y2[N], y3[N], z0[N], z1[N], z2[N], z3[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint64_t u = mul_wide(x4[k], K);
    u0[k] = (uint32_t)u;
    u1[k] = (uint32_t)(u >> 32) + x5[k] * K;
  }
#pragma unroll
  for (int k = 0; k < N; k++) y1[k] = add_co(x1[k], u0[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) z0[k] = sub_co(x0[k], x4[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) y2[k] = addc_co(x2[k], u1[k], cc[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) z1[k] = subb_co(y1[k], x5[k], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) y3[k] = addc_co_0(x3[k], cc[k], cc[k]);
#pragma unroll
  for (int k = 0; k < N; k++) z2[k] = subb_co_0(y2[k], bb[k], bb[k]);
#pragma unroll
  for (int k = 0; k < N; k++) z3[k] = subb_co_0(y3[k], bb[k], bb[k]);
  uint64_t kk[N], g[N];
#pragma unroll
  for (int k = 0; k < N; k++) asm("s_andn2_b64 %0, %1, %2" : "=s"(kk[k]) : "s"(cc[k]), "s"(bb[k]) : "scc");
  uint32_t t0[N], t1[N], t2[N], t3[N];
#pragma unroll
  for (int k = 0; k < N; k++) t0[k] = add_co_m1(z0[k], g[k]);
#pragma unroll
  for (int k = 0; k < N; k++) t1[k] = addc_co(z1[k], C1, g[k], g[k]);
#pragma unroll
  for (int k = 0; k < N; k++) t2[k] = addc_co_0(z2[k], g[k], g[k]);
#pragma unroll
  for (int k = 0; k < N; k++) t3[k] = addc_co_0(z3[k], g[k], g[k]);
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint64_t m = or_mask(kk[k], g[k]);
    out[k] = join(sel(z0[k], t0[k], m), sel(z1[k], t1[k], m), sel(z2[k], t2[k], m), sel(z3[k], t3[k], m));
  }
}

// N independent (x + y, x - y) pairs, step-interleaved like mul_xn
template <int N>
__device__ __forceinline__ void addsub_xn(const felt* a, const felt* b, felt* sum, felt* diff) {
  L4 x[N], y[N];
  uint64_t c[N], bw[N], g[N], b2[N];
  uint32_t s0[N], s1[N], s2[N], s3[N], d0[N], d1[N], d2[N], d3[N];
#pragma unroll
  for (int k = 0; k < N; k++) { x[k] = split(a[k]); y[k] = split(b[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { s0[k] = add_co(x[k].w0, y[k].w0, c[k]); d0[k] = sub_co(x[k].w0, y[k].w0, bw[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { s1[k] = addc_co(x[k].w1, y[k].w1, c[k], c[k]); d1[k] = subb_co(x[k].w1, y[k].w1, bw[k], bw[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { s2[k] = addc_co(x[k].w2, y[k].w2, c[k], c[k]); d2[k] = subb_co(x[k].w2, y[k].w2, bw[k], bw[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { s3[k] = addc_co(x[k].w3, y[k].w3, c[k], c[k]); d3[k] = subb_co(x[k].w3, y[k].w3, bw[k], bw[k]); }
  uint32_t m0[N], m1[N], t0[N], t1[N], t2[N], t3[N], e0[N], e1[N], e2[N], e3[N];
#pragma unroll
  for (int k = 0; k < N; k++) { m0[k] = sel_0_m1(bw[k]); m1[k] = sel(0u, C1, bw[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { t0[k] = add_co_m1(s0[k], g[k]); e0[k] = sub_co(d0[k], m0[k], b2[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { t1[k] = addc_co(s1[k], C1, g[k], g[k]); e1[k] = subb_co(d1[k], m1[k], b2[k], b2[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { t2[k] = addc_co_0(s2[k], g[k], g[k]); e2[k] = subb_co_0(d2[k], b2[k], b2[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) { t3[k] = addc_co_0(s3[k], g[k], g[k]); e3[k] = subb_0(d3[k], b2[k]); }
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint64_t m = or_mask(c[k], g[k]);
    sum[k] = join(sel(s0[k], t0[k], m), sel(s1[k], t1[k], m), sel(s2[k], t2[k], m), sel(s3[k], t3[k], m));
    diff[k] = join(e0[k], e1[k], e2[k], e3[k]);
  }
}
}  // namespace fpd
