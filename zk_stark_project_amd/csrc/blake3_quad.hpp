// blake3_quad.hpp — one BLAKE3 compression by a quad of lanes (device only):
// the latency-bound places (narrow tree levels, coin steps) where one lane's
// serial chain of 8 G functions per round would set the time.
#pragma once
#include <stdint.h>

#include "blake3.hpp"

namespace {

// Quad-cooperative 2-to-1 merge for the narrow (latency-bound) tree levels: the
// 4 lanes of a quad compute one BLAKE3(l || r) together, lane q holding state
// column q (v[q], v[4+q], v[8+q], v[12+q]). A round is the column G on every
// lane, a DPP quad rotation of rows b, c, d by 1, 2, 3 (the diagonals become
// columns), the diagonal G, and the inverse rotation: ~3x shorter dependency
// chain than one lane doing all 8 G's. Lane q returns output words q and 4+q.
template <int K>
__device__ __forceinline__ uint32_t quad_rot(uint32_t x) {  // value of lane (q + K) & 3
  constexpr int ctrl = K == 1 ? 0x39 : (K == 2 ? 0x4E : 0x93);  // quad_perm [1,2,3,0] / [2,3,0,1] / [3,0,1,2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  const uint32_t lo = (q & 1) ? x1 : x0, hi = (q & 1) ? x3 : x2;
  return (q & 2) ? hi : lo;
}
// One BLAKE3 compression (chunk counter 0, 64-byte block) by a quad: lane q
// holds chaining-value words q (a) and 4+q (b) in and out.
__device__ __forceinline__ void compress_quad(const uint32_t m[16], uint32_t q, uint32_t flags, uint32_t& a,
                                              uint32_t& b, uint32_t blen = 64, uint32_t ctr = 0) {
  constexpr uint8_t S[7][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                                {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                                {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                                {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                                {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                                {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                                {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
  uint32_t c = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));  // v[8..12) = IV[0..4)
  uint32_t d = sel4(q, ctr, 0u, blen, flags);                        // counter, block_len, flags
#define B3Q_G(x, y)                 \
  a = a + b + (x);                  \
  d = b3::rotr(d ^ a, 16);          \
  c = c + d;                        \
  b = b3::rotr(b ^ c, 12);          \
  a = a + b + (y);                  \
  d = b3::rotr(d ^ a, 8);           \
  c = c + d;                        \
  b = b3::rotr(b ^ c, 7);
#pragma unroll
  for (int r = 0; r < 7; r++) {
    B3Q_G(sel4(q, m[S[r][0]], m[S[r][2]], m[S[r][4]], m[S[r][6]]),
          sel4(q, m[S[r][1]], m[S[r][3]], m[S[r][5]], m[S[r][7]]))
    b = quad_rot<1>(b);
    c = quad_rot<2>(c);
    d = quad_rot<3>(d);
    B3Q_G(sel4(q, m[S[r][8]], m[S[r][10]], m[S[r][12]], m[S[r][14]]),
          sel4(q, m[S[r][9]], m[S[r][11]], m[S[r][13]], m[S[r][15]]))
    b = quad_rot<3>(b);
    c = quad_rot<2>(c);
    d = quad_rot<1>(d);
  }
#undef B3Q_G
  a ^= c;
  b ^= d;
}

// compress_quad with its rounds as a loop: the 16 message words are permuted in
// registers between rounds (BLAKE3 MSG_PERMUTATION), so each round selects the
// same word slots. ~6x less code, for the narrow tree levels that run on few
// waves per CU (their fully unrolled code streams through a cold I-cache).
// (blen: the block's byte length, 64 but for a coin draw's 40-byte seed || counter)
__device__ __forceinline__ void compress_quad_r(const uint32_t m_in[16], uint32_t q, uint32_t flags, uint32_t& a,
                                                uint32_t& b, uint32_t blen = 64) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = m_in[i];
  uint32_t c = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  uint32_t d = sel4(q, 0u, 0u, blen, flags);
#define B3Q_G(x, y)                 \
  a = a + b + (x);                  \
  d = b3::rotr(d ^ a, 16);          \
  c = c + d;                        \
  b = b3::rotr(b ^ c, 12);          \
  a = a + b + (y);                  \
  d = b3::rotr(d ^ a, 8);           \
  c = c + d;                        \
  b = b3::rotr(b ^ c, 7);
#pragma unroll 1
  for (int r = 0; r < 7; r++) {
    B3Q_G(sel4(q, m[0], m[2], m[4], m[6]), sel4(q, m[1], m[3], m[5], m[7]))
    b = quad_rot<1>(b);
    c = quad_rot<2>(c);
    d = quad_rot<3>(d);
    B3Q_G(sel4(q, m[8], m[10], m[12], m[14]), sel4(q, m[9], m[11], m[13], m[15]))
    b = quad_rot<3>(b);
    c = quad_rot<2>(c);
    d = quad_rot<1>(d);
    const uint32_t t0 = m[2], t1 = m[6], t2 = m[3], t3 = m[10], t4 = m[7], t5 = m[0], t6 = m[4], t7 = m[13];
    const uint32_t t8 = m[1], t9 = m[11], t10 = m[12], t11 = m[5], t12 = m[9], t13 = m[14], t14 = m[15],
                   t15 = m[8];
    m[0] = t0; m[1] = t1; m[2] = t2; m[3] = t3; m[4] = t4; m[5] = t5; m[6] = t6; m[7] = t7;
    m[8] = t8; m[9] = t9; m[10] = t10; m[11] = t11; m[12] = t12; m[13] = t13; m[14] = t14; m[15] = t15;
  }
#undef B3Q_G
  a ^= c;
  b ^= d;
}

// the quad's 8-word state (lane q holds words q and 4+q) in every lane of the quad
__device__ __forceinline__ void quad_gather8(uint32_t a, uint32_t b, uint32_t out[8]) {
  out[0] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0x00, 0xF, 0xF, false);  // quad_perm [0,0,0,0]
  out[1] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0x55, 0xF, 0xF, false);  // [1,1,1,1]
  out[2] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xAA, 0xF, 0xF, false);  // [2,2,2,2]
  out[3] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xFF, 0xF, 0xF, false);  // [3,3,3,3]
  out[4] = (uint32_t)__builtin_amdgcn_mov_dpp((int)b, 0x00, 0xF, 0xF, false);
  out[5] = (uint32_t)__builtin_amdgcn_mov_dpp((int)b, 0x55, 0xF, 0xF, false);
  out[6] = (uint32_t)__builtin_amdgcn_mov_dpp((int)b, 0xAA, 0xF, 0xF, false);
  out[7] = (uint32_t)__builtin_amdgcn_mov_dpp((int)b, 0xFF, 0xF, 0xF, false);
}

// ---- the device coin and small hashes by a quad (lanes q = 0..3 of one quad, all
// active): the serial transcript steps between the proof's stages, at ~1/4 of one
// lane's compression latency. Lane q holds words q and 4+q of every 8-word value.

// chaining value of chunk `ci` over felts [f0, f1) (<= 64) by a quad (hash_chunk's quad form):
// lane q returns words q and 4+q
template <typename Get>
__device__ __forceinline__ void quad_hash_chunk(Get get, uint32_t f0, uint32_t f1, uint32_t ci, bool root, uint32_t q,
                                                uint32_t& o0, uint32_t& o1) {
  o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
  const uint32_t nblk = f1 > f0 ? (f1 - f0 + 3) / 4 : 1;
  for (uint32_t blk = 0; blk < nblk; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t i = f0 + 4 * blk + k;
      const felt v = i < f1 ? get(i) : fp::zero();
      m[4 * k + 0] = (uint32_t)v.lo;
      m[4 * k + 1] = (uint32_t)(v.lo >> 32);
      m[4 * k + 2] = (uint32_t)v.hi;
      m[4 * k + 3] = (uint32_t)(v.hi >> 32);
    }
    const uint32_t left = f1 - f0 - 4 * blk, cnt = left < 4 ? left : 4;
    uint32_t fl = (blk == 0 ? b3::CHUNK_START : 0u) | (blk + 1 == nblk ? b3::CHUNK_END : 0u);
    if (root && blk + 1 == nblk) fl |= b3::ROOT;
    compress_quad(m, q, fl, o0, o1, f1 > f0 ? 16 * cnt : 0u, ci);
  }
}

// Blake3_256::hash_elements of nf <= 64 felts (one chunk), get(i) read by every lane
template <typename Get>
__device__ __forceinline__ void quad_hash_felts(Get get, uint32_t nf, uint32_t q, uint32_t& o0, uint32_t& o1) {
  o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
  const uint32_t nblk = nf ? (nf + 3) / 4 : 1;
  for (uint32_t blk = 0; blk < nblk; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t i = 4 * blk + k;
      const felt v = i < nf ? get(i) : fp::zero();
      m[4 * k + 0] = (uint32_t)v.lo;
      m[4 * k + 1] = (uint32_t)(v.lo >> 32);
      m[4 * k + 2] = (uint32_t)v.hi;
      m[4 * k + 3] = (uint32_t)(v.hi >> 32);
    }
    const uint32_t cnt = nf - 4 * blk < 4 ? nf - 4 * blk : 4;
    const uint32_t fl = (blk == 0 ? b3::CHUNK_START : 0u) | (blk + 1 == nblk ? (b3::CHUNK_END | b3::ROOT) : 0u);
    compress_quad(m, q, fl, o0, o1, nf ? 16 * cnt : 0u);
  }
}

// reseed: seed <- BLAKE3(seed || d), d given whole (8 words) to every lane
__device__ __forceinline__ void qcoin_reseed(uint32_t q, uint32_t& s0, uint32_t& s1, const uint32_t d[8]) {
  uint32_t m[16];
  quad_gather8(s0, s1, m);
#pragma unroll
  for (int i = 0; i < 8; i++) m[8 + i] = d[i];
  s0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  s1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
  compress_quad(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, s0, s1);
}

// draw candidate ctr: the first 16 bytes of BLAKE3(seed || ctr_le64), in every lane
__device__ __forceinline__ felt qcoin_candidate(uint32_t q, uint32_t s0, uint32_t s1, uint64_t ctr) {
  uint32_t m[16];
  quad_gather8(s0, s1, m);
  m[8] = (uint32_t)ctr;
  m[9] = (uint32_t)(ctr >> 32);
#pragma unroll
  for (int i = 10; i < 16; i++) m[i] = 0;
  uint32_t o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  uint32_t o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
  compress_quad(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, o0, o1, 40);
  uint32_t g[8];
  quad_gather8(o0, o1, g);
  return fp::make((uint64_t)g[0] | ((uint64_t)g[1] << 32), (uint64_t)g[2] | ((uint64_t)g[3] << 32));
}

// DefaultRandomCoin::draw: the first candidate < p (counter advanced), in every lane
__device__ __forceinline__ felt qcoin_draw(uint32_t q, uint32_t s0, uint32_t s1, uint64_t* ctr) {
  for (int i = 0; i < 1000; i++) {
    const felt v = qcoin_candidate(q, s0, s1, ++*ctr);
    if (!fp::ge_p(v)) return v;
  }
  return fp::zero();
}

}  // namespace
