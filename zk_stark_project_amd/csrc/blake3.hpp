// blake3.hpp — BLAKE3-256 compression for gfx950 and host (winter-crypto
// `Blake3_256`, blake3 1.5.4 in the reference's Cargo.lock:195-205).
//
// Device use is one thread per message: leaf rows of the trace / constraint /
// FRI matrices (hash_elements), Merkle 2-to-1 merges (64-byte single block),
// and grinding (seed || nonce, 40 bytes). All inputs here are at most 4
// chunks (255 felts = 4080 bytes), so the chunk tree is resolved statically.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "felt.hpp"

namespace b3 {

enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

ZKP_HD uint32_t iv(int i) {
  switch (i) {
    case 0: return 0x6A09E667u; case 1: return 0xBB67AE85u; case 2: return 0x3C6EF372u;
    case 3: return 0xA54FF53Au; case 4: return 0x510E527Fu; case 5: return 0x9B05688Cu;
    case 6: return 0x1F83D9ABu; default: return 0x5BE0CD19u;
  }
}

ZKP_HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define B3_G(a, b, c, d, x, y)          \
  s##a = s##a + s##b + (x);             \
  s##d = rotr(s##d ^ s##a, 16);         \
  s##c = s##c + s##d;                   \
  s##b = rotr(s##b ^ s##c, 12);         \
  s##a = s##a + s##b + (y);             \
  s##d = rotr(s##d ^ s##a, 8);          \
  s##c = s##c + s##d;                   \
  s##b = rotr(s##b ^ s##c, 7);

// message word schedule: m index used by round r at slot k (permutation applied r times)
#define B3_ROUND(m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11, m12, m13, m14, m15) \
  B3_G(0, 4, 8, 12, m[m0], m[m1]) B3_G(1, 5, 9, 13, m[m2], m[m3])                         \
  B3_G(2, 6, 10, 14, m[m4], m[m5]) B3_G(3, 7, 11, 15, m[m6], m[m7])                       \
  B3_G(0, 5, 10, 15, m[m8], m[m9]) B3_G(1, 6, 11, 12, m[m10], m[m11])                     \
  B3_G(2, 7, 8, 13, m[m12], m[m13]) B3_G(3, 4, 9, 14, m[m14], m[m15])

// cv[8] <- compress(cv, m[16], counter, block_len, flags)[0..8]
ZKP_HD void compress(uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                     uint32_t flags) {
  uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  uint32_t s8 = 0x6A09E667u, s9 = 0xBB67AE85u, s10 = 0x3C6EF372u, s11 = 0xA54FF53Au;
  uint32_t s12 = (uint32_t)counter, s13 = (uint32_t)(counter >> 32), s14 = block_len, s15 = flags;
  B3_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  B3_ROUND(2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
  B3_ROUND(3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1)
  B3_ROUND(10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6)
  B3_ROUND(12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4)
  B3_ROUND(9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7)
  B3_ROUND(11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13)
  cv[0] = s0 ^ s8; cv[1] = s1 ^ s9; cv[2] = s2 ^ s10; cv[3] = s3 ^ s11;
  cv[4] = s4 ^ s12; cv[5] = s5 ^ s13; cv[6] = s6 ^ s14; cv[7] = s7 ^ s15;
}

// The same compression with its 7 rounds as a loop (the message permuted in
// registers between rounds, BLAKE3's MSG_PERMUTATION): ~7x less code than
// compress(). For latency-bound code that runs on few waves per CU (tree tops,
// the device transcript, the FRI tail), whose fully unrolled straight-line
// code otherwise streams through a cold instruction cache.
ZKP_HD void compress_r(uint32_t cv[8], const uint32_t m_in[16], uint64_t counter, uint32_t block_len,
                       uint32_t flags) {
  uint32_t m[16];
  for (int i = 0; i < 16; i++) m[i] = m_in[i];
  uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
  uint32_t s8 = 0x6A09E667u, s9 = 0xBB67AE85u, s10 = 0x3C6EF372u, s11 = 0xA54FF53Au;
  uint32_t s12 = (uint32_t)counter, s13 = (uint32_t)(counter >> 32), s14 = block_len, s15 = flags;
#pragma unroll 1
  for (int r = 0; r < 7; r++) {
    B3_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
    const uint32_t t0 = m[2], t1 = m[6], t2 = m[3], t3 = m[10], t4 = m[7], t5 = m[0], t6 = m[4], t7 = m[13];
    const uint32_t t8 = m[1], t9 = m[11], t10 = m[12], t11 = m[5], t12 = m[9], t13 = m[14], t14 = m[15],
                   t15 = m[8];
    m[0] = t0; m[1] = t1; m[2] = t2; m[3] = t3; m[4] = t4; m[5] = t5; m[6] = t6; m[7] = t7;
    m[8] = t8; m[9] = t9; m[10] = t10; m[11] = t11; m[12] = t12; m[13] = t13; m[14] = t14; m[15] = t15;
  }
  cv[0] = s0 ^ s8; cv[1] = s1 ^ s9; cv[2] = s2 ^ s10; cv[3] = s3 ^ s11;
  cv[4] = s4 ^ s12; cv[5] = s5 ^ s13; cv[6] = s6 ^ s14; cv[7] = s7 ^ s15;
}

ZKP_HD void set_iv(uint32_t cv[8]) {
  for (int i = 0; i < 8; i++) cv[i] = iv(i);
}

// compress() or its rolled form (ROLLED: latency-bound call sites, see compress_r)
template <bool ROLLED>
ZKP_HD void compress_t(uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len, uint32_t flags) {
  if constexpr (ROLLED)
    compress_r(cv, m, counter, block_len, flags);
  else
    compress(cv, m, counter, block_len, flags);
}

// merge(a, b) = BLAKE3(a || b): one 64-byte block, single chunk, root
template <bool ROLLED = false>
ZKP_HD void merge(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
  uint32_t m[16];
  for (int i = 0; i < 8; i++) { m[i] = a[i]; m[8 + i] = b[i]; }
  set_iv(out);
  compress_t<ROLLED>(out, m, 0, 64, CHUNK_START | CHUNK_END | ROOT);
}

// parent node of the BLAKE3 chunk tree
template <bool ROLLED = false>
ZKP_HD void parent(const uint32_t l[8], const uint32_t r[8], bool root, uint32_t out[8]) {
  uint32_t m[16];
  for (int i = 0; i < 8; i++) { m[i] = l[i]; m[8 + i] = r[i]; }
  set_iv(out);
  compress_t<ROLLED>(out, m, 0, 64, PARENT | (root ? ROOT : 0u));
}

// chaining value of chunk `ci` covering felts [f0, f1) (at most 64 felts = 1024 bytes)
// The next block's felts are fetched before the current block is compressed
// (a register double buffer), so a row read from HBM overlaps its hashing
// instead of waiting once per 64-byte block.
template <bool ROLLED = false, typename Get>
ZKP_HD void hash_chunk(Get get, uint32_t f0, uint32_t f1, uint64_t ci, bool root, uint32_t cv[8]) {
  set_iv(cv);
  uint32_t nblocks = f1 > f0 ? (f1 - f0 + 3) / 4 : 1;
  felt cur[4];
#pragma unroll
  for (int k = 0; k < 4; k++) cur[k] = f0 + k < f1 ? get(f0 + k) : fp::zero();
  for (uint32_t b = 0; b < nblocks; b++) {
    const uint32_t base = f0 + 4 * b, nb = base + 4;
    felt nxt[4];
#pragma unroll
    for (int k = 0; k < 4; k++) nxt[k] = b + 1 < nblocks && nb + k < f1 ? get(nb + k) : fp::zero();
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      m[4 * k + 0] = (uint32_t)cur[k].lo;
      m[4 * k + 1] = (uint32_t)(cur[k].lo >> 32);
      m[4 * k + 2] = (uint32_t)cur[k].hi;
      m[4 * k + 3] = (uint32_t)(cur[k].hi >> 32);
    }
    const uint32_t cnt = f1 - base < 4 ? f1 - base : 4;  // (nblocks = 1 with f1 == f0: cnt = 0)
    uint32_t fl = (b == 0 ? CHUNK_START : 0u) | (b == nblocks - 1 ? CHUNK_END : 0u);
    if (root && b == nblocks - 1) fl |= ROOT;
    compress_t<ROLLED>(cv, m, ci, 16 * (f1 > f0 ? cnt : 0u), fl);
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = nxt[k];
  }
}

// hash_elements over `nf` felts supplied by get(k) (nf <= 256).
// 4 felts per 64-byte block, 64 felts per 1024-byte chunk; chunk tree for
// 2..4 chunks resolved statically (left subtree = largest power of two).
template <typename Get>
ZKP_HD void hash_felts(Get get, uint32_t nf, uint32_t out[8]) {
  if (nf <= 64) {
    hash_chunk(get, 0, nf, 0, true, out);
    return;
  }
  uint32_t c0[8], c1[8], c2[8], c3[8];
  hash_chunk(get, 0, 64, 0, false, c0);
  hash_chunk(get, 64, nf < 128 ? nf : 128, 1, false, c1);
  if (nf <= 128) {
    parent(c0, c1, true, out);
    return;
  }
  uint32_t l[8];
  parent(c0, c1, false, l);
  hash_chunk(get, 128, nf < 192 ? nf : 192, 2, false, c2);
  if (nf <= 192) {
    parent(l, c2, true, out);
    return;
  }
  hash_chunk(get, 192, nf, 3, false, c3);
  uint32_t r[8];
  parent(c2, c3, false, r);
  parent(l, r, true, out);
}

// hash_elements over a compile-time count NF <= 64 felts (one chunk): the block
// loop is unrolled, so get(k) sees constant k (register-resident rows, no scratch)
template <int NF, int B = 0, typename Get>
ZKP_HD void hash_felts_c(Get get, uint32_t cv[8]) {
  static_assert(NF >= 1 && NF <= 64, "one chunk");
  constexpr int NB = (NF + 3) / 4;
  if constexpr (B == 0) set_iv(cv);
  uint32_t m[16];
  constexpr int cnt = NF - 4 * B < 4 ? NF - 4 * B : 4;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    felt v = fp::zero();
    if (k < cnt) v = get(4 * B + k);
    m[4 * k + 0] = (uint32_t)v.lo;
    m[4 * k + 1] = (uint32_t)(v.lo >> 32);
    m[4 * k + 2] = (uint32_t)v.hi;
    m[4 * k + 3] = (uint32_t)(v.hi >> 32);
  }
  constexpr uint32_t fl = (B == 0 ? CHUNK_START : 0u) | (B == NB - 1 ? (CHUNK_END | ROOT) : 0u);
  compress(cv, m, 0, 16 * cnt, fl);
  if constexpr (B + 1 < NB) hash_felts_c<NF, B + 1>(get, cv);
}

// ---------------------------------------------------------------- host one-shot
// (transcript / random coin use; inputs are small)
static inline void host_hash(const uint8_t* data, size_t len, uint8_t out[32]);

static inline void host_chunk_cv(const uint8_t* data, size_t len, uint64_t idx, bool root, uint32_t cv[8]) {
  set_iv(cv);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    uint8_t blk[64] = {0};
    size_t off = b * 64, bl = len > off ? (len - off < 64 ? len - off : 64) : 0;
    if (bl) memcpy(blk, data + off, bl);
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
      m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) |
             ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t fl = (b == 0 ? CHUNK_START : 0u) | (b == nblocks - 1 ? CHUNK_END : 0u);
    if (root && b == nblocks - 1) fl |= ROOT;
    compress(cv, m, idx, (uint32_t)bl, fl);
  }
}

static inline void host_subtree(const uint8_t* data, size_t len, uint64_t first, bool root, uint32_t out[8]) {
  size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
  if (nchunks == 1) { host_chunk_cv(data, len, first, root, out); return; }
  size_t left = 1;
  while (left * 2 < nchunks) left *= 2;
  uint32_t l[8], r[8];
  host_subtree(data, left * 1024, first, false, l);
  host_subtree(data + left * 1024, len - left * 1024, first + left, false, r);
  parent(l, r, root, out);
}

static inline void host_hash(const uint8_t* data, size_t len, uint8_t out[32]) {
  uint32_t cv[8];
  host_subtree(data, len, 0, true, cv);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(cv[i] >> (8 * k));
}

}  // namespace b3
