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

#define ZKP_ASM asm

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

// Fast canonical forms. A 128-bit value z (plus a carry bit k past 2^128) with
// k = 0 and z3 != 0xffffffff is below 2^128 - 2^96 < p, so already canonical; a
// random z misses that with probability 2^-32 per lane. The check is one v_cmp
// whose wave ballot, OR'd with k, is uniform (SGPR masks), so `rare` is a scalar
// branch: a wave runs the exact select (canon_from) only when one of its lanes
// needs it, and the result is the same field element either way.
__device__ __forceinline__ felt canon_rare(uint32_t z0, uint32_t z1, uint32_t z2, uint32_t z3, uint64_t k) {
  const uint64_t rare = k | __builtin_amdgcn_ballot_w64(z3 == 0xffffffffu);
  if (rare) return canon_from(z0, z1, z2, z3, k);
  return join(z0, z1, z2, z3);
}

// a + b for canonical a, b: the sum S < 2p. Carry c set: S - p = s + C, which is
// < p. Carry clear: s is S, canonical unless s >= p (then s3 = 0xffffffff: the
// rare branch takes the exact select).
__device__ __forceinline__ felt add_sum(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint64_t c) {
  if (__builtin_amdgcn_ballot_w64(s3 == 0xffffffffu)) return canon_from(s0, s1, s2, s3, c);
  const uint32_t m0 = sel_0_m1(c), m1 = m0 & C1;  // c ? C : 0
  uint64_t g;
  const uint32_t t0 = add_co(s0, m0, g);
  const uint32_t t1 = addc_co(s1, m1, g, g);
  const uint32_t t2 = addc_co_0(s2, g, g);
  const uint32_t t3 = addc_0(s3, g);
  return join(t0, t1, t2, t3);
}

__device__ __forceinline__ felt add(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t c;
  uint32_t s0 = add_co(x.w0, y.w0, c);
  uint32_t s1 = addc_co(x.w1, y.w1, c, c);
  uint32_t s2 = addc_co(x.w2, y.w2, c, c);
  uint32_t s3 = addc_co(x.w3, y.w3, c, c);
  return add_sum(s0, s1, s2, s3, c);
}

__device__ __forceinline__ felt sub(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t bw;
  uint32_t d0 = sub_co(x.w0, y.w0, bw);
  uint32_t d1 = subb_co(x.w1, y.w1, bw, bw);
  uint32_t d2 = subb_co(x.w2, y.w2, bw, bw);
  uint32_t d3 = subb_co(x.w3, y.w3, bw, bw);
  // on borrow: d - C (mod 2^128) == d + p
  uint32_t m0 = sel_0_m1(bw), m1 = m0 & C1;
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

// reduce hi*2^128 + lo with 2^128 = 0x2D00*2^32 - 1 (mod p): z (4 limbs) and k,
// the carry past 2^128, with z + k*2^128 < 2^128 + 2^93 congruent to the input
__device__ __forceinline__ void reduce_core(const uint32_t r[8], uint32_t& z0, uint32_t& z1, uint32_t& z2,
                                            uint32_t& z3, uint64_t& k) {
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
  z0 = sub_co(x0, x4, b);
  z1 = subb_co(y1, x5, b, b);
  z2 = subb_co_0(y2, b, b);
  z3 = subb_co_0(y3, b, b);
  // net bit 128 = top - borrow (>= 0 overall); set when top & !borrow
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k) : "s"(top), "s"(b) : "scc");
}

__device__ __forceinline__ felt reduce(const uint32_t r[8]) {
  uint32_t z0, z1, z2, z3;
  uint64_t k;
  reduce_core(r, z0, z1, z2, z3, k);
  return canon_rare(z0, z1, z2, z3, k);
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
  return canon_rare(z0, z1, z2, z3, kk);
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

// Two independent reductions, interleaved like mul256x2 (z, k as reduce_core).
__device__ __forceinline__ void reduce_x2_core(const uint32_t r[8], const uint32_t s[8], uint32_t z[4], uint32_t Z[4],
                                               uint64_t& k1, uint64_t& k2) {
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
  z[0] = sub_co(x0, x4, b);
  Z[0] = sub_co(X0, X4, f);
  uint32_t y2 = addc_co(x2, u1, c, c);
  uint32_t Y2 = addc_co(X2, U1, e, e);
  z[1] = subb_co(y1, x5, b, b);
  Z[1] = subb_co(Y1, X5, f, f);
  uint32_t y3 = addc_co_0(x3, c, c);
  uint32_t Y3 = addc_co_0(X3, e, e);
  z[2] = subb_co_0(y2, b, b);
  Z[2] = subb_co_0(Y2, f, f);
  z[3] = subb_co_0(y3, b, b);
  Z[3] = subb_co_0(Y3, f, f);
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k1) : "s"(c), "s"(b) : "scc");
  ZKP_ASM("s_andn2_b64 %0, %1, %2" : "=s"(k2) : "s"(e), "s"(f) : "scc");
}

__device__ __forceinline__ void reduce_x2(const uint32_t r[8], const uint32_t s[8], felt& out_r, felt& out_s) {
  uint32_t z[4], Z[4];
  uint64_t k1, k2;
  reduce_x2_core(r, s, z, Z, k1, k2);
  // canonical forms (canon_rare): one scalar branch for both products
  const uint64_t rare = k1 | k2 | __builtin_amdgcn_ballot_w64(max(z[3], Z[3]) == 0xffffffffu);
  if (rare) {
    out_r = canon_from(z[0], z[1], z[2], z[3], k1);
    out_s = canon_from(Z[0], Z[1], Z[2], Z[3], k2);
  } else {
    out_r = join(z[0], z[1], z[2], z[3]);
    out_s = join(Z[0], Z[1], Z[2], Z[3]);
  }
}

__device__ __forceinline__ void mul_x2(felt a, felt b, felt c, felt d, felt& ab, felt& cd) {
  uint32_t r[8], s[8];
  mul256x2(split(a), split(b), split(c), split(d), r, s);
  reduce_x2(r, s, ab, cd);
}

// ---- deferred-check forms (the NTT rounds): no branch per operation. Each
// result is taken as canonical and the evidence that it may not be — a carry
// past 2^128 (k) or a top limb 0xffffffff — is accumulated in a Rare; a round
// whose Rare is set is recomputed from its inputs with the exact forms. Valid
// when every input is canonical, which holds until the first rare event.
struct Rare {
  uint64_t k = 0;    // OR of the products' carries past 2^128 (SGPR lane masks)
  uint32_t top = 0;  // max of the results' top limbs
  __device__ __forceinline__ bool any() const { return (k | __builtin_amdgcn_ballot_w64(top == 0xffffffffu)) != 0; }
};

__device__ __forceinline__ felt mul_z(felt a, felt b, Rare& q) {
  uint32_t r[8], z0, z1, z2, z3;
  uint64_t k;
  mul256(split(a), split(b), r);
  reduce_core(r, z0, z1, z2, z3, k);
  q.k |= k;
  q.top = max(q.top, z3);
  return join(z0, z1, z2, z3);
}

__device__ __forceinline__ void mul_x2_z(felt a, felt b, felt c, felt d, felt& ab, felt& cd, Rare& q) {
  uint32_t r[8], s[8], z[4], Z[4];
  uint64_t k1, k2;
  mul256x2(split(a), split(b), split(c), split(d), r, s);
  reduce_x2_core(r, s, z, Z, k1, k2);
  q.k |= k1 | k2;
  q.top = max(q.top, max(z[3], Z[3]));
  ab = join(z[0], z[1], z[2], z[3]);
  cd = join(Z[0], Z[1], Z[2], Z[3]);
}

// a + b: carry set -> s + C (< p); carry clear -> s, canonical unless s3 = 0xffffffff
__device__ __forceinline__ felt add_z(felt a, felt b, Rare& q) {
  L4 x = split(a), y = split(b);
  uint64_t c, g;
  const uint32_t s0 = add_co(x.w0, y.w0, c);
  const uint32_t s1 = addc_co(x.w1, y.w1, c, c);
  const uint32_t s2 = addc_co(x.w2, y.w2, c, c);
  const uint32_t s3 = addc_co(x.w3, y.w3, c, c);
  q.top = max(q.top, s3);
  const uint32_t m0 = sel_0_m1(c), m1 = m0 & C1;
  const uint32_t t0 = add_co(s0, m0, g);
  const uint32_t t1 = addc_co(s1, m1, g, g);
  const uint32_t t2 = addc_co_0(s2, g, g);
  const uint32_t t3 = addc_0(s3, g);
  return join(t0, t1, t2, t3);
}
}  // namespace fpd
