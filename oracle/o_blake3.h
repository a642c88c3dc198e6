/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Portable one-shot BLAKE3-256 restated from the published BLAKE3
 * specification (reference dependency blake3 1.5.4, Cargo.lock:195-205, not
 * vendored). Used through winter-crypto `Blake3_256`:
 *   hash_elements(els) = BLAKE3(LE bytes of els)      (f128 IS_CANONICAL)
 *   merge([a, b])      = BLAKE3(a || b)               (64 B)
 *   merge_with_int(s,v)= BLAKE3(s || v.to_le_bytes())  (40 B)
 * Pinned by tests/golden/blake3.json (published digests of "" / "abc" /
 * the 1025-byte test vector, plus Python-spec multi-chunk vectors).
 */
#ifndef O_BLAKE3_H
#define O_BLAKE3_H
#include <stdint.h>
#include <string.h>
#include <stddef.h>

static const uint32_t OB3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                   0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t OB3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { OB3_CHUNK_START = 1, OB3_CHUNK_END = 2, OB3_PARENT = 4, OB3_ROOT = 8 };

static inline uint32_t ob3_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define OB3_G(a, b, c, d, mx, my)          \
  do {                                     \
    s[a] = s[a] + s[b] + (mx);             \
    s[d] = ob3_rotr(s[d] ^ s[a], 16);      \
    s[c] = s[c] + s[d];                    \
    s[b] = ob3_rotr(s[b] ^ s[c], 12);      \
    s[a] = s[a] + s[b] + (my);             \
    s[d] = ob3_rotr(s[d] ^ s[a], 8);       \
    s[c] = s[c] + s[d];                    \
    s[b] = ob3_rotr(s[b] ^ s[c], 7);       \
  } while (0)

static inline void ob3_compress(uint32_t cv[8], const uint8_t block[64], uint64_t counter,
                                uint32_t block_len, uint32_t flags) {
  uint32_t m[16], t[16], s[16];
  for (int i = 0; i < 16; i++)
    m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) |
           ((uint32_t)block[4 * i + 2] << 16) | ((uint32_t)block[4 * i + 3] << 24);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  for (int i = 0; i < 4; i++) s[8 + i] = OB3_IV[i];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  for (int r = 0; r < 7; r++) {
    OB3_G(0, 4, 8, 12, m[0], m[1]);
    OB3_G(1, 5, 9, 13, m[2], m[3]);
    OB3_G(2, 6, 10, 14, m[4], m[5]);
    OB3_G(3, 7, 11, 15, m[6], m[7]);
    OB3_G(0, 5, 10, 15, m[8], m[9]);
    OB3_G(1, 6, 11, 12, m[10], m[11]);
    OB3_G(2, 7, 8, 13, m[12], m[13]);
    OB3_G(3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      for (int i = 0; i < 16; i++) t[i] = m[OB3_PERM[i]];
      memcpy(m, t, sizeof m);
    }
  }
  for (int i = 0; i < 8; i++) cv[i] = s[i] ^ s[i + 8];
}

/* chaining value of one chunk (<= 1024 bytes); root flag on last block if `root` */
static inline void ob3_chunk(const uint8_t* data, size_t len, uint64_t chunk_idx, int root,
                             uint32_t cv[8]) {
  uint8_t block[64];
  memcpy(cv, OB3_IV, 32);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    size_t off = b * 64, bl = len - off < 64 ? len - off : 64;
    if (len == 0) bl = 0;
    memset(block, 0, 64);
    if (bl) memcpy(block, data + off, bl);
    uint32_t fl = (b == 0 ? OB3_CHUNK_START : 0) | (b == nblocks - 1 ? OB3_CHUNK_END : 0);
    if (root && b == nblocks - 1) fl |= OB3_ROOT;
    ob3_compress(cv, block, chunk_idx, (uint32_t)bl, fl);
  }
}

static inline void ob3_parent(const uint32_t l[8], const uint32_t r[8], int root, uint32_t out[8]) {
  uint8_t block[64];
  for (int i = 0; i < 8; i++) {
    for (int k = 0; k < 4; k++) {
      block[4 * i + k] = (uint8_t)(l[i] >> (8 * k));
      block[32 + 4 * i + k] = (uint8_t)(r[i] >> (8 * k));
    }
  }
  memcpy(out, OB3_IV, 32);
  ob3_compress(out, block, 0, 64, OB3_PARENT | (root ? OB3_ROOT : 0));
}

static void ob3_subtree(const uint8_t* data, size_t len, uint64_t first_chunk, int root,
                        uint32_t out[8]) {
  size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
  if (nchunks == 1) {
    ob3_chunk(data, len, first_chunk, root, out);
    return;
  }
  size_t left = 1;
  while (left * 2 < nchunks) left *= 2;
  uint32_t l[8], r[8];
  ob3_subtree(data, left * 1024, first_chunk, 0, l);
  ob3_subtree(data + left * 1024, len - left * 1024, first_chunk + left, 0, r);
  ob3_parent(l, r, root, out);
}

static inline void ob3_hash(const uint8_t* data, size_t len, uint8_t out[32]) {
  uint32_t cv[8];
  ob3_subtree(data, len, 0, 1, cv);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(cv[i] >> (8 * k));
}

static inline void ob3_merge(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  uint8_t buf[64];
  memcpy(buf, a, 32);
  memcpy(buf + 32, b, 32);
  ob3_hash(buf, 64, out);
}

static inline void ob3_merge_with_int(const uint8_t seed[32], uint64_t v, uint8_t out[32]) {
  uint8_t buf[40];
  memcpy(buf, seed, 32);
  for (int i = 0; i < 8; i++) buf[32 + i] = (uint8_t)(v >> (8 * i));
  ob3_hash(buf, 40, out);
}

#endif
