// merkle.hip — CDNA4 (gfx950) kernels of the prover's hashing side: BLAKE3
// leaf rows and Merkle trees (winter-crypto MerkleTree<Blake3_256>), the device
// transcript (DefaultRandomCoin), grinding, query positions and openings, and
// the FRI layers (fold-by-16, the fused small-layer tail, the remainder).
#include "kernels_dev.hpp"
#include "blake3_quad.hpp"

#include <cstdlib>

using kc::rev_bits;
using kc::static_for;

namespace {

// ------------------------------------------------------------------ hashing
__global__ __launch_bounds__(TPB) void k_leaf_hash_lde(const felt* __restrict__ lde, uint32_t cols, uint32_t logB,
                                                       uint64_t n, uint32_t* __restrict__ nodes, uint64_t L) {
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= L) return;
  uint64_t j = i & ((1ull << logB) - 1), t = i >> logB;
  const felt* base = lde + j * n + t;
  const uint64_t cstride = n << logB;
  uint32_t d[8];
  b3::hash_felts([&](uint32_t c) { return base[c * cstride]; }, cols, d);
  store_digest(nodes + (L + i) * 8, d);
}

__global__ __launch_bounds__(TPB) void k_leaf_hash_fri(const felt* __restrict__ E, uint64_t R, uint32_t F,
                                                       uint32_t* __restrict__ nodes) {
  uint64_t r = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (r >= R) return;
  uint32_t d[8];
  b3::hash_felts([&](uint32_t k) { return E[r + k * R]; }, F, d);
  store_digest(nodes + (R + r) * 8, d);
}

// nodes[s + i] = merge(nodes[2(s+i)], nodes[2(s+i)+1]) for i < s
__global__ __launch_bounds__(TPB) void k_merkle_level(uint32_t* nodes, uint64_t s) {
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= s) return;
  uint64_t node = s + i;
  uint32_t m[16];
  load_digest(nodes + 2 * node * 8, m);
  load_digest(nodes + (2 * node + 1) * 8, m + 8);
  uint32_t out[8];
  b3::set_iv(out);
  b3::compress(out, m, 0, 64, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
  store_digest(nodes + node * 8, out);
}

// remaining top levels (s_start .. 1) inside one workgroup
__global__ __launch_bounds__(1024) void k_merkle_top(uint32_t* nodes, uint64_t s_start) {
  for (uint64_t s = s_start; s >= 1; s >>= 1) {
    for (uint64_t i = threadIdx.x; i < s; i += blockDim.x) {
      uint64_t node = s + i;
      uint32_t m[16];
      load_digest(nodes + 2 * node * 8, m);
      load_digest(nodes + (2 * node + 1) * 8, m + 8);
      uint32_t out[8];
      b3::set_iv(out);
      b3::compress(out, m, 0, 64, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
      store_digest(nodes + node * 8, out);
    }
    __threadfence_block();
    __syncthreads();
  }
}

// Fused Merkle build: each block turns up to 512 consecutive leaves into all
// 9 levels of their subtree (leaf digests -> subtree root) with the levels
// held in LDS and every node written once to nodes[] (tree layout: level d of
// an L-leaf tree at nodes[(L >> d) .. (2L >> d))). MODE 0: leaves = rows of a
// coset-major LDE matrix; MODE 1: leaves = FRI rows [E[r + k*R]]; MODE 2:
// leaves already stored in nodes[L..2L); MODE 3: leaf digests in a sharded
// commitment's all-to-all receive buffer (src; k_leaf_unpack's layout), stored
// to nodes[L..2L) on the way up.
struct MerkleArgs {
  const felt* src;
  uint64_t n;       // MODE 0: rows per coset
  uint32_t cols;    // MODE 0: columns; MODE 1: F; MODE 3: log2 rows per chunk and source (logrc)
  uint32_t logB;    // MODE 0/1/3: cosets of the (coset-major) source
  uint64_t R;       // MODE 1: rows per coset (m/16)
  uint32_t* nodes;
  uint64_t L;       // leaves of this (sub)tree level
  MerkleTail tail;  // k_merkle_fused: finish the tree (+ FRI coin step) in the last block
  LastCol lc;       // k_merkle_leaf2<COLS, true>: column COLS-1 derived from H (zkp_internal.hpp)
  GuLazy gl;        // MODE 4: LDE rows whose columns >= gl.wi are derived (zkp_internal.hpp)
};

// value of a lazy GlobalUpdate column c >= gl.wi of the row at base (prev = the
// previous row of its coset, l = L_0 at the row)
__device__ __forceinline__ felt gu_lazy_value(const GuLazy& gl, const felt* base, const felt* prev, uint64_t cstride,
                                              felt l, uint32_t c) {
  const uint32_t ic = c - gl.d;
  const felt df = sub(base[ic * cstride], prev[ic * cstride]);
  const felt kd = gl.smallk ? mul_u32(df, (uint32_t)gl.k.lo) : mul(gl.k, df);
  return add(kd, mul(gl.cval[ic], l));
}

// rows gu_row_hash takes (MODE 5): the reference's GlobalUpdate width, every paired column lazy
static inline bool gu_row_shape(uint32_t cols, const GuLazy& gl) { return cols == 120 && gl.d == 60 && gl.wi == 60; }

// 4 felts -> one 64-byte BLAKE3 message block
__device__ __forceinline__ void pack4(const felt v[4], uint32_t m[16]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    m[4 * k + 0] = (uint32_t)v[k].lo;
    m[4 * k + 1] = (uint32_t)(v[k].lo >> 32);
    m[4 * k + 2] = (uint32_t)v[k].hi;
    m[4 * k + 3] = (uint32_t)(v[k].hi >> 32);
  }
}

// A lazy GlobalUpdate row of the reference shape (120 felts, columns 0..59 stored and
// 60..119 derived from them: d = wi = 60). Its two BLAKE3 chunks (columns 0..63 and
// 64..119) are independent chains until their parent node, so they are compressed
// interleaved: chunk 1's block b (columns 64+4b..67+4b, derived from stored columns
// 4b+4..4b+7) right after chunk 0's block b+1, which holds exactly those columns. Every
// stored felt is then fetched once per row (the generic getter re-read 56 of the 60 from
// HBM for the derived half, after the row's other loads had evicted them); only chunk 0's
// last block (columns 60..63, derived from 0..3) re-reads four.
__device__ __forceinline__ void gu_row_hash(const GuLazy& gl, const felt* base, const felt* prev, uint64_t cstride,
                                            felt l, uint32_t out[8]) {
  auto derive = [&](felt cur, felt pre, uint32_t ic) {
    const felt df = sub(cur, pre);
    const felt kd = gl.smallk ? mul_u32(df, (uint32_t)gl.k.lo) : mul(gl.k, df);
    return add(kd, mul(gl.cval[ic], l));
  };
  uint32_t cv0[8], cv1[8];
  b3::set_iv(cv0);
  b3::set_iv(cv1);
  felt cur[4], prv[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    cur[k] = base[k * cstride];
    prv[k] = fp::zero();
  }
#pragma unroll 1
  for (uint32_t b = 0; b < 16; b++) {
    // next block's stored felts and their previous-row values (block 15: columns 0..3)
    const uint32_t nb = b < 14 ? 4 * (b + 1) : 0;
    felt nxt[4], npr[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      nxt[k] = b < 15 ? base[(nb + k) * cstride] : fp::zero();
      npr[k] = b < 15 ? prev[(nb + k) * cstride] : fp::zero();
    }
    uint32_t m[16];
    pack4(cur, m);
    b3::compress(cv0, m, 0, 64, (b == 0 ? b3::CHUNK_START : 0u) | (b == 15 ? b3::CHUNK_END : 0u));
    if (b >= 1 && b <= 14) {  // chunk 1, block b - 1: columns 60 + 4b + k from 4b + k
      felt dv[4];
#pragma unroll
      for (int k = 0; k < 4; k++) dv[k] = derive(cur[k], prv[k], 4 * b + k);
      pack4(dv, m);
      b3::compress(cv1, m, 1, 64, (b == 1 ? b3::CHUNK_START : 0u) | (b == 14 ? b3::CHUNK_END : 0u));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      cur[k] = b == 14 ? derive(nxt[k], npr[k], k) : nxt[k];  // block 15: columns 60..63
      prv[k] = npr[k];
    }
  }
  b3::parent(cv0, cv1, true, out);
}

// v[COLS-1] = (h - sum_{c<COLS-1} kappa^c v[c]) * kappa^-(COLS-1)  (LastCol; Horner
// over the known columns: COLS-1 products)
template <int COLS>
__device__ __forceinline__ felt derive_last(const felt* v, felt h, felt kappa, felt kinv) {
  felt acc = v[COLS - 2];
#pragma unroll
  for (int c = COLS - 3; c >= 0; c--) acc = add(mul(acc, kappa), v[c]);
  return mul(sub(h, acc), kinv);
}

template <int MODE>
__device__ __forceinline__ void merkle_leaf(const MerkleArgs& a, uint64_t i, uint32_t d[8]) {
  if (MODE == 0) {
    uint64_t j = i & ((1ull << a.logB) - 1), t = i >> a.logB;
    const felt* base = a.src + j * a.n + t;
    const uint64_t cstride = a.n << a.logB;
    b3::hash_felts([&](uint32_t c) { return base[c * cstride]; }, a.cols, d);
  } else if (MODE == 1) {
    // natural row i = j + B*t' -> coset j, positions t' + k*R
    const felt* base = a.src + ((i & ((1ull << a.logB) - 1)) * 16) * a.R + (i >> a.logB);
    b3::hash_felts([&](uint32_t k) { return base[k * a.R]; }, a.cols, d);
  } else if (MODE == 4 || MODE == 5) {  // MODE 0 with lazy GlobalUpdate columns (5: gu_row_shape)
    const uint64_t j = i & ((1ull << a.logB) - 1), t = i >> a.logB;
    const felt* base = a.src + j * a.n + t;
    const felt* prev = a.src + j * a.n + (t == 0 ? a.n - 1 : t - 1);
    const uint64_t cstride = a.n << a.logB;
    const felt l = a.gl.l0[j * a.n + t];
    if constexpr (MODE == 5)
      gu_row_hash(a.gl, base, prev, cstride, l, d);
    else
      b3::hash_felts([&](uint32_t c) { return c < a.gl.wi ? base[c * cstride] : gu_lazy_value(a.gl, base, prev, cstride, l, c); },
                     a.cols, d);
  } else if (MODE == 3) {
    // leaf i = j + B*tl sits in chunk k = tl >> logrc, source block j, row tl mod rc
    const uint64_t j = i & ((1ull << a.logB) - 1), tl = i >> a.logB;
    const uint64_t k = tl >> a.cols, tc = tl & ((1ull << a.cols) - 1);
    load_digest(reinterpret_cast<const uint32_t*>(a.src) + (((k << a.logB) + j) << a.cols | tc) * 8, d);
  } else {
    load_digest(a.nodes + (a.L + i) * 8, d);
  }
}

template <bool ROLLED = false>
__device__ __forceinline__ void merge_quad(const uint32_t m[16], uint32_t q, uint32_t& o0, uint32_t& o1) {
  o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
  if constexpr (ROLLED)
    compress_quad_r(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, o0, o1);
  else
    compress_quad(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, o0, o1);
}

// Quad-cooperative digest of one FRI row of 16 felts (256 bytes: one chunk of
// four blocks, hash_felts' nf <= 64 case); lane q returns words q and 4+q.
__device__ __forceinline__ void fri_leaf_quad(const MerkleArgs& a, uint64_t i, uint32_t q, uint32_t& o0,
                                              uint32_t& o1) {
  const felt* base = a.src + ((i & ((1ull << a.logB) - 1)) * 16) * a.R + (i >> a.logB);
  o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
  o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
#pragma unroll
  for (uint32_t blk = 0; blk < 4; blk++) {
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const felt v = base[(4 * blk + k) * a.R];
      m[4 * k + 0] = (uint32_t)v.lo;
      m[4 * k + 1] = (uint32_t)(v.lo >> 32);
      m[4 * k + 2] = (uint32_t)v.hi;
      m[4 * k + 3] = (uint32_t)(v.hi >> 32);
    }
    const uint32_t fl = (blk == 0 ? b3::CHUNK_START : 0u) | (blk == 3 ? (b3::CHUNK_END | b3::ROOT) : 0u);
    compress_quad(m, q, fl, o0, o1);
  }
}

template <bool ROLLED = false>
__device__ __forceinline__ void merge8(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { m[i] = l[i]; m[8 + i] = r[i]; }
  b3::set_iv(out);
  b3::compress_t<ROLLED>(out, m, 0, 64, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
}

__device__ __forceinline__ void merkle_tail_op(const MerkleTail& tl, const uint32_t* root);

// QUAD (MODE 1 with 16-felt rows only): 64 leaves per block, each hashed by a
// quad of lanes (compress_quad), so a small FRI layer's leaf stage is four
// short-chain compressions instead of eight serial ones per lane; the layers
// below 2^16 rows are latency-bound, not throughput-bound.
template <int MODE, bool QUAD = false>
__global__ __launch_bounds__(256) void k_merkle_fused(MerkleArgs a) {
  __shared__ uint32_t sd[256 * 9];
  const uint32_t t = threadIdx.x;
  const uint64_t L = a.L;
  constexpr uint64_t LB = QUAD ? 64 : 512;        // leaves per block
  const uint64_t cnt = L < LB ? L : LB;           // leaves in this block's subtree
  const uint64_t base = (uint64_t)blockIdx.x * LB;
  uint64_t lvl, lbase;
  uint32_t s0;  // nodes of the level above the one held in sd[]
  if constexpr (QUAD) {
    const uint32_t nd = t >> 2, q = t & 3;
    if (nd < cnt) {  // the 4 lanes of a quad are active together (DPP)
      uint32_t o0, o1;
      fri_leaf_quad(a, base + nd, q, o0, o1);
      sd[nd * 9 + q] = o0;
      sd[nd * 9 + 4 + q] = o1;
      uint32_t* dst = a.nodes + (L + base + nd) * 8;
      dst[q] = o0;
      dst[4 + q] = o1;
    }
    lvl = L;
    lbase = base;
    s0 = (uint32_t)(cnt >> 1);
  } else {
    uint32_t m[8];
    if (2 * t < cnt) {
      uint32_t d0[8], d1[8];
      merkle_leaf<MODE>(a, base + 2 * t, d0);
      merkle_leaf<MODE>(a, base + 2 * t + 1, d1);
      if (MODE != 2) {
        store_digest(a.nodes + (L + base + 2 * t) * 8, d0);
        store_digest(a.nodes + (L + base + 2 * t + 1) * 8, d1);
      }
      merge8<false>(d0, d1, m);
      store_digest(a.nodes + ((L >> 1) + (base >> 1) + t) * 8, m);
#pragma unroll
      for (int i = 0; i < 8; i++) sd[t * 9 + i] = m[i];
    }
    lvl = L >> 1;
    lbase = base >> 1;
    s0 = (uint32_t)(cnt >> 2);
  }
  for (uint32_t s = s0; s >= 1; s >>= 1) {
    __syncthreads();
    if (s <= 64) {  // narrow level: one quad per node
      const uint32_t nd = t >> 2, q = t & 3;
      uint32_t o0 = 0, o1 = 0;
      if (t < 4 * s) {
        uint32_t mm[16];
#pragma unroll
        for (int i = 0; i < 8; i++) { mm[i] = sd[(2 * nd) * 9 + i]; mm[8 + i] = sd[(2 * nd + 1) * 9 + i]; }
        merge_quad<false>(mm, q, o0, o1);
      }
      lvl >>= 1;
      lbase >>= 1;
      __syncthreads();
      if (t < 4 * s) {
        sd[nd * 9 + q] = o0;
        sd[nd * 9 + 4 + q] = o1;
        uint32_t* dst = a.nodes + (lvl + lbase + nd) * 8;
        dst[q] = o0;
        dst[4 + q] = o1;
      }
      continue;
    }
    uint32_t o[8];
    if (t < s) {
      uint32_t l[8], r[8];
#pragma unroll
      for (int i = 0; i < 8; i++) { l[i] = sd[(2 * t) * 9 + i]; r[i] = sd[(2 * t + 1) * 9 + i]; }
      merge8<false>(l, r, o);
    }
    lvl >>= 1;
    lbase >>= 1;
    __syncthreads();
    if (t < s) {
#pragma unroll
      for (int i = 0; i < 8; i++) sd[t * 9 + i] = o[i];
      store_digest(a.nodes + (lvl + lbase + t) * 8, o);
    }
  }
  if (!a.tail.done) return;
  // the last block to finish builds the levels above the G = gridDim.x subtree
  // roots (nodes[G .. 2G), G <= 512) up to nodes[1], then runs the FRI coin step
  // (release: fence + counter; acquire: fence after seeing the count)
  __shared__ int s_last;
  __threadfence();
  __syncthreads();
  if (t == 0) s_last = atomicAdd(a.tail.done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const uint32_t G = gridDim.x;
  if (G > 1) {
    if (G / 2 <= 64) {  // level G/2 from the roots in global memory, one quad per node
      const uint32_t nd = t >> 2, q = t & 3;
      if (t < 4 * (G / 2)) {
        uint32_t mm[16], o0, o1;
        const uint32_t* src = a.nodes + (uint64_t)(G + 2 * nd) * 8;  // the node's two children, adjacent
#pragma unroll
        for (int k = 0; k < 16; k++) mm[k] = src[k];
        merge_quad<false>(mm, q, o0, o1);
        sd[nd * 9 + q] = o0;
        sd[nd * 9 + 4 + q] = o1;
        uint32_t* dst = a.nodes + (uint64_t)(G / 2 + nd) * 8;
        dst[q] = o0;
        dst[4 + q] = o1;
      }
    } else {
      for (uint32_t i = t; i < G / 2; i += 256) {  // level G/2 from the roots in global memory
        uint32_t l[8], r[8], o[8];
        load_digest(a.nodes + (uint64_t)(G + 2 * i) * 8, l);
        load_digest(a.nodes + (uint64_t)(G + 2 * i + 1) * 8, r);
        merge8<false>(l, r, o);
        store_digest(a.nodes + (uint64_t)(G / 2 + i) * 8, o);
#pragma unroll
        for (int k = 0; k < 8; k++) sd[i * 9 + k] = o[k];
      }
    }
    for (uint32_t sl = G / 4; sl >= 1; sl >>= 1) {
      __syncthreads();
      if (sl <= 64) {  // narrow level: one quad per node
        const uint32_t nd = t >> 2, q = t & 3;
        uint32_t o0 = 0, o1 = 0;
        if (t < 4 * sl) {
          uint32_t mm[16];
#pragma unroll
          for (int k = 0; k < 8; k++) { mm[k] = sd[(2 * nd) * 9 + k]; mm[8 + k] = sd[(2 * nd + 1) * 9 + k]; }
          merge_quad<false>(mm, q, o0, o1);
        }
        __syncthreads();
        if (t < 4 * sl) {
          sd[nd * 9 + q] = o0;
          sd[nd * 9 + 4 + q] = o1;
          uint32_t* dst = a.nodes + (uint64_t)(sl + nd) * 8;
          dst[q] = o0;
          dst[4 + q] = o1;
        }
        continue;
      }
      uint32_t o[8];
      if (t < sl) {
        uint32_t l[8], r[8];
#pragma unroll
        for (int k = 0; k < 8; k++) { l[k] = sd[(2 * t) * 9 + k]; r[k] = sd[(2 * t + 1) * 9 + k]; }
        merge8<false>(l, r, o);
      }
      __syncthreads();
      if (t < sl) {
#pragma unroll
        for (int k = 0; k < 8; k++) sd[t * 9 + k] = o[k];
        store_digest(a.nodes + (uint64_t)(sl + t) * 8, o);
      }
    }
  }
  __syncthreads();
  if (t == 0) *a.tail.done = 0;  // ready for the next launch on this stream
  if (a.tail.op != MERKLE_TAIL_NONE) merkle_tail_op(a.tail, a.nodes + 8);  // whole block
}

// Lane-subtree Merkle build: every lane turns 2^H consecutive leaves into their
// height-H subtree sequentially in registers (compile-time recursion, <= H+1
// live digests), writing every node it creates. No LDS, no barriers, no idle
// lanes; the levels above are built by further passes over the subtree roots.
template <int MODE, int H>
__device__ __forceinline__ void lane_subtree(const MerkleArgs& a, uint64_t base, uint32_t out[8]) {
  if constexpr (H == 0) {
    merkle_leaf<MODE>(a, base, out);
    if (MODE != 2) store_digest(a.nodes + (a.L + base) * 8, out);
  } else {
    uint32_t l[8], r[8];
    lane_subtree<MODE, H - 1>(a, base, l);
    lane_subtree<MODE, H - 1>(a, base + (1ull << (H - 1)), r);
    merge8(l, r, out);
    store_digest(a.nodes + ((a.L >> H) + (base >> H)) * 8, out);
  }
}

// Leaf pass of an LDE-row tree for narrow rows (COLS <= 8 felts): each lane
// loads BOTH of its rows' felts before any hashing, then hashes them and
// merges (as k_merkle_lane<0, 1>). The generic lane kernel reads each row
// inside its hash and its digest stores may alias the LDE (no restrict), so
// the second row's loads wait behind the first row's hash and stores; here the
// HBM latency of both rows is exposed once per lane.
// DERIVE: column COLS-1 is not read but derived from the constraint evaluations
// (a.lc) and written out before hashing.
template <int COLS, bool DERIVE = false>
__global__ __launch_bounds__(256) void k_merkle_leaf2(MerkleArgs a) {
  const uint64_t lane = blockIdx.x * (uint64_t)256 + threadIdx.x;
  if (lane >= (a.L >> 1)) return;
  const uint64_t cstride = a.n << a.logB, bmask = (1ull << a.logB) - 1;
  constexpr int RD = DERIVE ? COLS - 1 : COLS;  // columns read from the source
  felt v[2][COLS], h[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint64_t i = 2 * lane + r;
    const uint64_t off = (i & bmask) * a.n + (i >> a.logB);
    const felt* base = a.src + off;
#pragma unroll
    for (int c = 0; c < RD; c++) v[r][c] = base[c * cstride];
    if constexpr (DERIVE) h[r] = a.lc.H[off];
  }
  if constexpr (DERIVE) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const uint64_t i = 2 * lane + r, j = i & bmask;
      v[r][COLS - 1] = derive_last<COLS>(v[r], h[r], a.lc.kap[2 * j], a.lc.kap[2 * j + 1]);
      a.lc.out[j * a.n + (i >> a.logB)] = v[r][COLS - 1];
    }
  }
  uint32_t d0[8], d1[8], m[8];
  b3::hash_felts_c<COLS>([&](int c) { return v[0][c]; }, d0);
  b3::hash_felts_c<COLS>([&](int c) { return v[1][c]; }, d1);
  store_digest(a.nodes + (a.L + 2 * lane) * 8, d0);
  store_digest(a.nodes + (a.L + 2 * lane + 1) * 8, d1);
  merge8(d0, d1, m);
  store_digest(a.nodes + ((a.L >> 1) + lane) * 8, m);
}

// Leaf pass of an LDE-row tree for wide rows (65..255 felts: 2-4 BLAKE3 chunks) on few
// rows, e.g. the reference's TrainingUpdate trace (2^13 x 240 at blowup 16: 2^17 rows, which
// a lane per row pair spreads as one 256-thread block per CU). Here a row's chunks are
// hashed by 4 lanes at once (chunk ch by lane ch of its quad; the chunk chains are
// independent until their parents, hash_felts' chunk tree), and an octet holds two sibling
// rows, (2jp, t) and (2jp + 1, t). Consecutive octets take consecutive positions t of the
// same coset pair, so each column load of a wave reads whole 128-byte lines.
__global__ __launch_bounds__(256) void k_merkle_wide(MerkleArgs a) {
  const uint64_t g = blockIdx.x * 256ull + threadIdx.x;
  const uint32_t ch = threadIdx.x & 3, sib = (threadIdx.x >> 2) & 1;
  const uint32_t logn = 63 - __builtin_clzll(a.n);
  const uint64_t oct = g >> 3, t = oct & (a.n - 1), jp = oct >> logn;
  const bool valid = jp < (1ull << (a.logB - 1));  // block-uniform (the grid covers L / 2 octets exactly)
  const uint32_t nch = (a.cols + 63) / 64;
  const uint64_t j = 2 * jp + sib, i = j + (t << a.logB);
  uint32_t cv[8];
  if (valid && ch < nch) {
    const felt* base = a.src + j * a.n + t;
    const uint64_t cstride = a.n << a.logB;
    const uint32_t f0 = 64 * ch, f1 = f0 + 64 < a.cols ? f0 + 64 : a.cols;
    b3::hash_chunk([&](uint32_t c) { return base[c * cstride]; }, f0, f1, ch, nch == 1, cv);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) cv[k] = 0;
  }
  // the row's chunk tree (nch is uniform): lane ch of a quad holds chunk ch's chaining value
  uint32_t c1[8], root[8];
#pragma unroll
  for (int k = 0; k < 8; k++) c1[k] = (uint32_t)__shfl_down((int)cv[k], 1);
  if (nch == 1) {
#pragma unroll
    for (int k = 0; k < 8; k++) root[k] = cv[k];
  } else if (nch == 2) {
    b3::parent(cv, c1, true, root);
  } else {
    uint32_t p[8], q[8];
    b3::parent(cv, c1, false, p);  // lanes 0 and 2: parents of chunks (0, 1) and (2, 3)
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = (uint32_t)__shfl_down((int)(nch == 3 ? cv[k] : p[k]), 2);
    b3::parent(p, q, true, root);
  }
  // level 1: the octet's two sibling rows
  uint32_t sr[8];
#pragma unroll
  for (int k = 0; k < 8; k++) sr[k] = (uint32_t)__shfl_down((int)root[k], 4);
  if (valid && ch == 0) {
    store_digest(a.nodes + (a.L + i) * 8, root);
    if (sib == 0) {
      uint32_t m[8];
      merge8(root, sr, m);
      store_digest(a.nodes + ((a.L >> 1) + (i >> 1)) * 8, m);
    }
  }
}

// (MODE 4, lazy GlobalUpdate rows: held to 128 VGPRs for 4 waves per SIMD instead of
// the 134 and 3 waves it compiles to unbounded)
template <int MODE, int H>
__global__ __launch_bounds__(256, MODE == 4 || MODE == 5 ? 4 : 1) void k_merkle_lane(MerkleArgs a) {
  const uint64_t lane = blockIdx.x * (uint64_t)256 + threadIdx.x;
  if (lane >= (a.L >> H)) return;
  uint32_t root[8];
  lane_subtree<MODE, H>(a, lane << H, root);
}

// ---- sharded commitments: the rank hashes the rows it owns (cosets
// [j0, j0+Bl), rows t < rows) and scatters the digests by destination rank
// (contiguous natural leaf ranges) for the all-to-all. The exchange runs in
// K = 2^logK chunks along the destination's rows (so chunk k's all-to-all
// overlaps the hashing of chunk k+1): chunk k holds, for every destination s,
// the rows t = s*rr + k*rc + tc (tc < rc = rr / K) at
// send_k[((s*Bl + jl)*rc + tc)], rr = rows / R.
// COLS > 0 (narrow LDE rows, MODE 0): the row's felts are loaded into registers
// before hashing (compile-time row length, see k_merkle_leaf2)
// (MODE 4, lazy GlobalUpdate rows: held to 128 VGPRs for 4 waves per SIMD, as k_merkle_lane)
template <int MODE, int COLS = 0, bool DERIVE = false>
__global__ __launch_bounds__(TPB, MODE == 4 || MODE == 5 ? 4 : 1) void k_leaf_hash_shard(const felt* __restrict__ src, uint64_t n, uint32_t cols,
                                                         uint32_t logBl, uint32_t logrows, uint32_t logrr,
                                                         uint32_t logK, uint32_t k, uint32_t* __restrict__ send,
                                                         LastCol lc, GuLazy gl) {
  const uint64_t q = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  const uint32_t logrc = logrr - logK, logrk = logrows - logK;  // rows per chunk: per destination, in all
  if (q >= (1ull << (logrk + logBl))) return;
  const uint64_t jl = q >> logrk, u = q & ((1ull << logrk) - 1);
  const uint64_t sd = u >> logrc, tc = u & ((1ull << logrc) - 1);
  const uint64_t t = (sd << logrr) + ((uint64_t)k << logrc) + tc;
  const uint64_t rows = 1ull << logrows;
  uint32_t d[8];
  if constexpr (MODE == 0 && COLS > 0) {
    const felt* base = src + jl * n + t;
    const uint64_t cstride = n << logBl;
    felt v[COLS];
    constexpr int RD = DERIVE ? COLS - 1 : COLS;
#pragma unroll
    for (int c = 0; c < RD; c++) v[c] = base[c * cstride];
    if constexpr (DERIVE) {  // LastCol over the rank's cosets (lc.kap offset to coset j0)
      v[COLS - 1] = derive_last<COLS>(v, lc.H[jl * n + t], lc.kap[2 * jl], lc.kap[2 * jl + 1]);
      lc.out[jl * n + t] = v[COLS - 1];
    }
    b3::hash_felts_c<COLS>([&](int c) { return v[c]; }, d);
  } else if (MODE == 0) {  // LDE row t of coset jl: (c*Bl + jl)*n + t
    const felt* base = src + jl * n + t;
    const uint64_t cstride = n << logBl;
    b3::hash_felts([&](uint32_t c) { return base[c * cstride]; }, cols, d);
  } else if (MODE == 4 || MODE == 5) {  // MODE 0 with lazy GlobalUpdate columns (5: gu_row_shape)
    const felt* base = src + jl * n + t;
    const felt* prev = src + jl * n + (t == 0 ? n - 1 : t - 1);
    const uint64_t cstride = n << logBl;
    const felt l = gl.l0[jl * n + t];
    if constexpr (MODE == 5)
      gu_row_hash(gl, base, prev, cstride, l, d);
    else
      b3::hash_felts([&](uint32_t c) { return c < gl.wi ? base[c * cstride] : gu_lazy_value(gl, base, prev, cstride, l, c); },
                     cols, d);
  } else {  // FRI row: positions t + k*rows of coset jl (16*rows per coset)
    const felt* base = src + (jl << (logrows + 4)) + t;
    b3::hash_felts([&](uint32_t kk) { return base[kk * rows]; }, cols, d);
  }
  store_digest(send + ((((sd << logBl) + jl) << logrc) + tc) * 8, d);
}

// received leaf digests -> natural leaf order of this rank's range: chunk k
// (L/K digests, source-rank-major = global coset j major, rc rows each) holds
// the range rows tl = k*rc + tc: leaf j + B*tl
__global__ __launch_bounds__(TPB) void k_leaf_unpack(const uint32_t* __restrict__ recv, uint32_t logB, uint32_t logrr,
                                                     uint32_t logK, uint32_t* __restrict__ nodes, uint64_t L) {
  const uint64_t idx = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (idx >= L) return;
  const uint32_t logrc = logrr - logK;
  const uint64_t k = idx >> (logB + logrc), r = idx & ((1ull << (logB + logrc)) - 1);
  const uint64_t j = r >> logrc, tl = (k << logrc) + (r & ((1ull << logrc) - 1));
  uint32_t d[8];
  load_digest(recv + idx * 8, d);
  store_digest(nodes + (L + j + (tl << logB)) * 8, d);
}

// Fiat-Shamir step of the FRI commit loop on the device (winter-crypto
// DefaultRandomCoin<Blake3_256>: reseed = merge(seed, root), counter = 0; draw
// = first merge_with_int(seed, ++counter) whose low 16 bytes are < p). `root`
// is the layer's Merkle root; the host replays the same steps afterwards and
// checks every alpha. coin = [seed words 0..8), alphas[l], roots[l] (8 words).
// ---------------------------------------------------------- device transcript
// winter-crypto DefaultRandomCoin<Blake3_256> on the device: seed = 8 LE words;
// reseed(d) = BLAKE3(seed || d); draw = first 16 B of BLAKE3(seed || ctr_le64),
// ctr = 1, 2, ... since the last reseed, rejected while >= p.
__device__ __forceinline__ void dcoin_reseed(uint32_t s[8], const uint32_t d[8]) {
  uint32_t m[16];
  for (int i = 0; i < 8; i++) { m[i] = s[i]; m[8 + i] = d[i]; }
  b3::set_iv(s);
  b3::compress_r(s, m, 0, 64, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
}
__device__ __forceinline__ felt dcoin_candidate(const uint32_t s[8], uint64_t ctr) {
  uint32_t m[16], o[8];
  for (int i = 0; i < 8; i++) m[i] = s[i];
  m[8] = (uint32_t)ctr;
  m[9] = (uint32_t)(ctr >> 32);
  for (int i = 10; i < 16; i++) m[i] = 0;
  b3::set_iv(o);
  b3::compress_r(o, m, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
  return fp::make((uint64_t)o[0] | ((uint64_t)o[1] << 32), (uint64_t)o[2] | ((uint64_t)o[3] << 32));
}
// sequential draw (thread-local), advancing *ctr
__device__ __forceinline__ felt dcoin_draw(const uint32_t s[8], uint64_t* ctr) {
  for (int i = 0; i < 1000; i++) {
    felt v = dcoin_candidate(s, ++*ctr);
    if (!fp::ge_p(v)) return v;
  }
  return fp::zero();
}

// draw `ncoef` coefficients into out (whole block; the coin state s was just
// reseeded, counter 0): Linear = ncoef draws (parallel candidates, sequential redo
// on a rejection), Algebraic = powers of one draw, Horner = the powers reversed
__device__ __forceinline__ void dcoin_draw_coeffs_block(const uint32_t s[8], uint32_t method, uint32_t ncoef, felt* out,
                                        felt* s_alpha, int* s_rej) {
  if (threadIdx.x == 0) *s_rej = 0;
  if (method != ZKP_BATCHING_LINEAR && threadIdx.x < 4) {  // one draw, by the first quad
    const uint32_t q = threadIdx.x;
    uint64_t ctr = 0;
    const felt a = qcoin_draw(q, s[q], s[4 + q], &ctr);
    if (q == 0) *s_alpha = a;
  }
  __syncthreads();
  if (method == ZKP_BATCHING_LINEAR) {
    for (uint32_t i = threadIdx.x; i < ncoef; i += blockDim.x) {
      felt v = dcoin_candidate(s, (uint64_t)i + 1);
      if (fp::ge_p(v)) *s_rej = 1;
      out[i] = v;
    }
    __syncthreads();
    if (*s_rej && threadIdx.x == 0) {
      uint64_t ctr = 0;
      for (uint32_t i = 0; i < ncoef; i++) out[i] = dcoin_draw(s, &ctr);
    }
    __syncthreads();
    return;
  }
  // a^i for i = t + k * blockDim: a^t and a^blockDim by two independent short ladders, then
  // one product per further i (was a full ladder per i: 4 x ~16 dependent products for the
  // reference's w + C = 241 DEEP coefficients on a 64-thread block)
  const felt a = *s_alpha;
  const felt step = fp::pow_u64(a, blockDim.x);
  felt p = fp::pow_u64(a, threadIdx.x);
  for (uint32_t i = threadIdx.x; i < ncoef; i += blockDim.x) {
    out[method == ZKP_BATCHING_HORNER ? ncoef - 1 - i : i] = p;
    p = mul(p, step);
  }
  __syncthreads();
}

// Blake3_256::hash_elements over nf felts get(i) by a whole block: chunk c (64 felts)
// by quad c (quad_hash_chunk: a quad's compression has a ~3x shorter dependency chain
// than one lane's, and these transcript hashes run on one block), then the chunk tree
// (left subtree = largest power of two) by the first quad with the incremental stack.
// nf <= 64 * 32; blockDim >= 64.
template <typename Get>
__device__ __forceinline__ void hash_felts_block(Get get, uint32_t nf, uint32_t out[8], uint32_t (*s_cv)[8]) {
  const uint32_t nch = nf ? (nf + 63) / 64 : 1, q = threadIdx.x & 3;
  for (uint32_t c = threadIdx.x >> 2; c < nch; c += blockDim.x >> 2) {
    uint32_t o0, o1;
    const uint32_t f0 = 64 * c, f1 = f0 + 64 < nf ? f0 + 64 : nf;
    quad_hash_chunk(get, f0, f1, c, nch == 1, q, o0, o1);
    s_cv[c][q] = o0;
    s_cv[c][4 + q] = o1;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    if (nch == 1) {
      for (int i = 0; i < 8; i++) out[i] = s_cv[0][i];
    } else {
      // parent(l, cur) by the quad (cur: lane q holds words q, 4+q; quad_gather8)
      auto parent_q = [&](const uint32_t* l, uint32_t& a, uint32_t& b, bool root) {
        uint32_t m[16];
        quad_gather8(a, b, m + 8);
#pragma unroll
        for (int i = 0; i < 8; i++) m[i] = l[i];
        a = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
        b = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
        compress_quad(m, q, b3::PARENT | (root ? b3::ROOT : 0u), a, b);
      };
      // the incremental chunk-tree stack lives in s_cv itself: after chunk c the stack
      // holds popcount(c + 1) <= c + 1 entries, at indices below the next chunk to read
      uint32_t (*st)[8] = s_cv;
      int top = 0;
      for (uint32_t c = 0; c + 1 < nch; c++) {
        uint32_t a = s_cv[c][q], b = s_cv[c][4 + q];
        uint64_t total = c + 1;
        while ((total & 1) == 0) {
          --top;
          parent_q(st[top], a, b, false);
          total >>= 1;
        }
        st[top][q] = a;
        st[top][4 + q] = b;
        top++;
      }
      uint32_t a = s_cv[nch - 1][q], b = s_cv[nch - 1][4 + q];
      while (top > 0) {
        top--;
        parent_q(st[top], a, b, top == 0);
      }
      quad_gather8(a, b, out);
    }
  }
  __syncthreads();
}

// hash_elements for the transcript: one chunk (<= 64 felts) by the block's first
// quad (quad_hash_felts), longer inputs by hash_felts_block; out[] in every thread
template <typename Get>
__device__ __forceinline__ void hash_felts_fast(Get get, uint32_t nf, uint32_t out[8], uint32_t (*s_cv)[8]) {
  if (nf > 64) {
    hash_felts_block(get, nf, out, s_cv);
    if (threadIdx.x == 0)
      for (int i = 0; i < 8; i++) s_cv[0][i] = out[i];
  } else if (threadIdx.x < 4) {
    const uint32_t q = threadIdx.x;
    uint32_t o0, o1;
    quad_hash_felts(get, nf, q, o0, o1);
    s_cv[0][q] = o0;
    s_cv[0][4 + q] = o1;
  }
  __syncthreads();
  for (int i = 0; i < 8; i++) out[i] = s_cv[0][i];
  __syncthreads();
}

// the block's first quad: seed <- BLAKE3(src || d) into dst (and dst2 when given)
__device__ __forceinline__ void quad_reseed_to(const uint32_t* src, const uint32_t d[8], uint32_t* dst,
                                               uint32_t* dst2 = nullptr) {
  if (threadIdx.x >= 4) return;
  const uint32_t q = threadIdx.x;
  uint32_t s0 = src[q], s1 = src[4 + q];
  qcoin_reseed(q, s0, s1, d);
  dst[q] = s0;
  dst[4 + q] = s1;
  if (dst2) {
    dst2[q] = s0;
    dst2[4 + q] = s1;
  }
}

// OOD frame -> transcript -> DEEP coefficients, on the device: reseed with
// H(T(z) || T(zg)) and H(H_j(z)), draw the w + C DEEP coefficients, and the
// constants kz = sum gamma_i T_i(z) + sum gamma_j H_j(z), kzg = sum gamma_i T_i(zg).
// ood[2a + {0,1}] = array a at (z, zg), arrays = w trace columns then C composition columns.
// dk = [z, zg] on entry; [z, zg, kz, kzg] on exit.
__global__ __launch_bounds__(64) void k_dt_deep_coeffs(uint32_t* __restrict__ seed, const felt* __restrict__ ood,
                                                       uint32_t w, uint32_t C, uint32_t method,
                                                       felt* __restrict__ gamma, felt* __restrict__ dk) {
  __shared__ uint32_t s_cv[32][8];
  __shared__ uint32_t s[8];
  __shared__ felt s_alpha;
  __shared__ int s_rej;
  __shared__ felt red0[64], red1[64];
  uint32_t h[8];
  hash_felts_fast([&](uint32_t i) { return i < w ? ood[2 * i] : ood[2 * (i - w) + 1]; }, 2 * w, h, s_cv);
  quad_reseed_to(seed, h, s);
  __syncthreads();
  hash_felts_fast([&](uint32_t i) { return ood[2 * (w + i)]; }, C, h, s_cv);
  quad_reseed_to(s, h, s, seed);
  __syncthreads();
  uint32_t t[8];
  for (int i = 0; i < 8; i++) t[i] = s[i];
  dcoin_draw_coeffs_block(t, method, w + C, gamma, &s_alpha, &s_rej);
  felt a = zero(), b = zero();
  for (uint32_t i = threadIdx.x; i < w + C; i += blockDim.x) {
    a = add(a, mul(gamma[i], ood[2 * i]));
    if (i < w) b = add(b, mul(gamma[i], ood[2 * i + 1]));
  }
  red0[threadIdx.x] = a;
  red1[threadIdx.x] = b;
  __syncthreads();
  for (uint32_t k = 32; k >= 1; k >>= 1) {
    if (threadIdx.x < k) {
      red0[threadIdx.x] = add(red0[threadIdx.x], red0[threadIdx.x + k]);
      red1[threadIdx.x] = add(red1[threadIdx.x], red1[threadIdx.x + k]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    dk[2] = red0[0];
    dk[3] = red1[0];
  }
}

// reseed with the trace root, then the constraint composition coefficients
// (ConstraintCompositionCoefficients::draw: Linear = n draws, Algebraic = powers
// of one draw, Horner = the powers reversed). One block; Linear draws run in
// parallel with a sequential redo if any candidate was rejected.
__device__ __forceinline__ void dt_draw_coeffs_block(uint32_t* __restrict__ seed, const uint32_t* __restrict__ root, uint32_t method,
                                     uint32_t ncoef, felt* __restrict__ cc) {
  __shared__ uint32_t s[8];
  __shared__ felt s_alpha;
  __shared__ int s_rej;
  {
    uint32_t d[8];
    for (int i = 0; i < 8; i++) d[i] = root[i];
    quad_reseed_to(seed, d, s, seed);
  }
  __syncthreads();
  uint32_t t[8];
  for (int i = 0; i < 8; i++) t[i] = s[i];
  dcoin_draw_coeffs_block(t, method, ncoef, cc, &s_alpha, &s_rej);
}
__global__ __launch_bounds__(TPB) void k_dt_draw_coeffs(uint32_t* __restrict__ seed, const uint32_t* __restrict__ root,
                                                        uint32_t method, uint32_t ncoef, felt* __restrict__ cc) {
  dt_draw_coeffs_block(seed, root, method, ncoef, cc);
}


// reseed with the constraint root, draw z; zz = (z, z*w_n); pw tables
// pw[l] = z^(2^l), pw[logn + l] = (z w_n)^(2^l) for the OOD evaluation
__device__ __forceinline__ void dt_draw_z_block(uint32_t* __restrict__ seed, const uint32_t* __restrict__ root, felt wn, uint32_t logn,
                                felt* __restrict__ zz, felt* __restrict__ pw) {
  __shared__ felt s_z;
  if (threadIdx.x < 4) {  // the first quad: reseed with the root, draw z
    const uint32_t q = threadIdx.x;
    uint32_t s0 = seed[q], s1 = seed[4 + q], d[8];
    for (int i = 0; i < 8; i++) d[i] = root[i];
    qcoin_reseed(q, s0, s1, d);
    seed[q] = s0;
    seed[4 + q] = s1;
    uint64_t ctr = 0;
    const felt z = qcoin_draw(q, s0, s1, &ctr);
    if (q == 0) {
      zz[0] = z;
      zz[1] = mul(z, wn);
      s_z = z;
    }
  }
  __syncthreads();
  if (threadIdx.x >= 2) return;
  // the two squaring chains (z and z*w_n) on two lanes
  felt a = threadIdx.x == 0 ? s_z : mul(s_z, wn);
  felt* out = pw + threadIdx.x * logn;
  for (uint32_t l = 0; l < logn; l++) {
    out[l] = a;
    a = sqr(a);
  }
}
__global__ void k_dt_draw_z(uint32_t* __restrict__ seed, const uint32_t* __restrict__ root, felt wn, uint32_t logn,
                            felt* __restrict__ zz, felt* __restrict__ pw) {
  dt_draw_z_block(seed, root, wn, logn, zz, pw);
}

__device__ __forceinline__ void coin_fri_step(uint32_t* __restrict__ seed, const uint32_t* root, felt* __restrict__ alpha_out,
                              uint32_t* __restrict__ root_out);

// what the last block of a finished Merkle tree does with its root (all threads
// of the block call it; root = nodes + 8, written by this block)
__device__ __forceinline__ void merkle_tail_op(const MerkleTail& tl, const uint32_t* root) {
  if (tl.op == MERKLE_TAIL_FRI_COIN) {
    coin_fri_step(tl.coin_seed, root, tl.alpha_out, tl.root_out);  // threads 0..3
  } else if (tl.op == MERKLE_TAIL_DRAW_COEFFS) {
    dt_draw_coeffs_block(tl.coin_seed, root, tl.method, tl.ncoef, tl.out);
  } else if (tl.op == MERKLE_TAIL_DRAW_Z) {
    dt_draw_z_block(tl.coin_seed, root, tl.wn, tl.logn, tl.out, tl.pw);
  }
}

// FRI commit-loop Fiat-Shamir step by the block's first quad (threads 0..3): seed <-
// BLAKE3(seed || root), alpha = first draw < p; root copied to root_out
__device__ __forceinline__ void coin_fri_step(uint32_t* __restrict__ seed, const uint32_t* root, felt* __restrict__ alpha_out,
                              uint32_t* __restrict__ root_out) {
  if (threadIdx.x >= 4) return;
  const uint32_t q = threadIdx.x;
  uint32_t r[8];
  for (int i = 0; i < 8; i++) r[i] = root[i];
  uint32_t s0 = seed[q], s1 = seed[4 + q];
  qcoin_reseed(q, s0, s1, r);
  uint64_t ctr = 0;
  const felt a = qcoin_draw(q, s0, s1, &ctr);
  if (q == 0) *alpha_out = a;
  seed[q] = s0;
  seed[4 + q] = s1;
  root_out[q] = r[q];
  root_out[4 + q] = r[4 + q];
}

__global__ void k_coin_fri_layer(uint32_t* __restrict__ seed, const uint32_t* __restrict__ root,
                                 felt* __restrict__ alpha_out, uint32_t* __restrict__ root_out) {
  if (blockIdx.x != 0) return;
  coin_fri_step(seed, root, alpha_out, root_out);  // threads 0..3
}

struct SeedArg {
  uint32_t w[8];
};

// gathers up to PACK_MAX device segments (4-byte multiples) into one staging
// buffer, so a host round trip is one kernel + one D2H copy instead of one
// copy call per segment
__global__ __launch_bounds__(TPB) void k_pack(PackArgs a, uint32_t* __restrict__ dst) {
  const uint32_t seg = blockIdx.y;
  if (seg >= a.n) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.src[seg]);
  const uint64_t words = a.bytes[seg] / 4, o = a.off[seg] / 4;
  for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < words; i += (uint64_t)gridDim.x * TPB)
    dst[o + i] = src[i];
}

// FriProver::set_remainder's interpolation by a whole block: the D = m*B last-layer
// values (coset-major: natural index i = j + B*t at E[j*m + t]) -> the first ncoef
// coefficients c_k = D^-1 off^-k sum_i v_i w_D^-ik into s_c. The powers w_D^-j are
// a table (one pow per thread); each wave sums the D terms of one coefficient
// (lanes over i, then a shuffle reduction), so the chain is ~log D products long
// instead of 2D sequential ones. D <= 256 (host-checked); s_tw holds D felts.
__device__ __forceinline__ felt shfl_down_felt(felt v, int d) {
  const int a = __shfl_down((int)(uint32_t)v.lo, d), b = __shfl_down((int)(uint32_t)(v.lo >> 32), d);
  const int c = __shfl_down((int)(uint32_t)v.hi, d), e = __shfl_down((int)(uint32_t)(v.hi >> 32), d);
  return fp::make((uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32),
                  (uint64_t)(uint32_t)c | ((uint64_t)(uint32_t)e << 32));
}
__device__ __forceinline__ void remainder_coeffs_block(const felt* __restrict__ E, uint32_t logB, uint32_t m,
                                                       uint32_t ncoef, felt off_inv, felt wd_inv, felt d_inv,
                                                       felt* s_c, felt* s_tw) {
  const uint32_t D = m << logB, t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
  for (uint32_t j = t; j < D; j += blockDim.x) s_tw[j] = fp::pow_u64(wd_inv, j);
  __syncthreads();
  for (uint32_t k = wave; k < ncoef; k += nw) {
    felt acc = zero();
    for (uint32_t i = lane; i < D; i += 64)
      acc = add(acc, mul(E[(i & ((1u << logB) - 1)) * m + (i >> logB)], s_tw[(i * k) & (D - 1)]));
    for (int d = 32; d >= 1; d >>= 1) acc = add(acc, shfl_down_felt(acc, d));
    if (lane == 0) s_c[k] = mul(mul(acc, d_inv), fp::pow_u64(off_inv, k));
  }
  __syncthreads();
}

// FriProver::set_remainder on the device for small last layers (D <= 256): the
// D values E (coset-major: natural index i = j + B*t at E[j*m + t]) interpolated
// over off*<w_D>, the first ncoef = D/B coefficients kept:
// c_k = D^-1 off^-k sum_i v_i w_D^-ik. Then the coin absorbs H(remainder)
// (seed <- BLAKE3(seed || H)) so grinding can start from the device seed.
// rem_out = [ncoef coefficients], commit_out = H(remainder) (8 words).
__global__ __launch_bounds__(TPB) void k_fri_remainder(const felt* __restrict__ E, uint32_t logB, uint32_t m,
                                                       felt off_inv, felt wd_inv, felt d_inv, uint32_t ncoef,
                                                       uint32_t* __restrict__ seed, felt* __restrict__ rem_out,
                                                       uint32_t* __restrict__ commit_out) {
  __shared__ felt s_c[256];
  __shared__ felt s_tw[256];
  __shared__ uint32_t s_cv[32][8];
  remainder_coeffs_block(E, logB, m, ncoef, off_inv, wd_inv, d_inv, s_c, s_tw);
  for (uint32_t k = threadIdx.x; k < ncoef; k += TPB) rem_out[k] = s_c[k];
  uint32_t h[8];
  hash_felts_fast([&](uint32_t i) { return s_c[i]; }, ncoef, h, s_cv);
  quad_reseed_to(seed, h, seed);
  if (threadIdx.x < 8) commit_out[threadIdx.x] = h[threadIdx.x];
}

// Minimum nonce in [base, base + count) whose BLAKE3(seed || nonce) has >= bits
// trailing zeros (atomicMin). seedp (device coin state) overrides seed. A block
// whose nonces all exceed a result already found exits at once (blocks are
// dispatched in index order, so most blocks after the first hit do no work).
__global__ __launch_bounds__(TPB) void k_grind(SeedArg seed, const uint32_t* __restrict__ seedp, uint64_t base,
                                               uint64_t count, uint32_t bits, unsigned long long* result) {
  __shared__ int s_skip;
  const uint64_t b0 = base + blockIdx.x * (uint64_t)TPB;
  if (threadIdx.x == 0) s_skip = __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < b0;
  __syncthreads();
  if (s_skip) return;
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= count) return;
  uint64_t nonce = base + i;
  uint32_t m[16];
#pragma unroll
  for (int k = 0; k < 8; k++) m[k] = seedp ? seedp[k] : seed.w[k];
  m[8] = (uint32_t)nonce;
  m[9] = (uint32_t)(nonce >> 32);
#pragma unroll
  for (int k = 10; k < 16; k++) m[k] = 0;
  uint32_t out[8];
  b3::set_iv(out);
  b3::compress(out, m, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
  uint64_t h = (uint64_t)out[0] | ((uint64_t)out[1] << 32);
  uint32_t tz = h == 0 ? 64u : (uint32_t)__builtin_ctzll(h);
  if (tz >= bits) atomicMin(result, (unsigned long long)nonce);
}

// Grinding to completion on the device: the minimum nonce >= base whose
// BLAKE3(seed || nonce) has >= bits trailing zeros (seed = the device coin).
// Thread g tests base + it*T + g in iteration it (T = all threads); it stops
// once its iteration's first nonce exceeds a found nonce, so every smaller
// candidate is still tested (minimum = sequential semantics) and every wave
// exits (or at `limit`, leaving result untouched: the host reports no nonce).
__global__ __launch_bounds__(TPB) void k_grind_all(const uint32_t* __restrict__ seedp, uint64_t base, uint64_t limit,
                                                   uint32_t bits, unsigned long long* result) {
  const uint64_t T = (uint64_t)gridDim.x * TPB, g = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  using b3::rotr;
  uint32_t m[16];
#pragma unroll
  for (int k = 0; k < 8; k++) m[k] = seedp[k];
#pragma unroll
  for (int k = 8; k < 16; k++) m[k] = 0;
  // Round 1 touches the nonce (message words 8, 9) only in its first diagonal G:
  // the column step and the other three diagonal G's are the same for every
  // nonce, so they run once here (7 of the compression's 56 G's)
  uint32_t p0 = b3::iv(0), p1 = b3::iv(1), p2 = b3::iv(2), p3 = b3::iv(3), p4 = b3::iv(4), p5 = b3::iv(5),
           p6 = b3::iv(6), p7 = b3::iv(7), p8 = b3::iv(0), p9 = b3::iv(1), p10 = b3::iv(2), p11 = b3::iv(3),
           p12 = 0, p13 = 0, p14 = 40, p15 = b3::CHUNK_START | b3::CHUNK_END | b3::ROOT;
  {
#define sp(i) p##i
#define B3_GP(a, b, c, d, x, y)            \
  sp(a) = sp(a) + sp(b) + (x);              \
  sp(d) = rotr(sp(d) ^ sp(a), 16);          \
  sp(c) = sp(c) + sp(d);                    \
  sp(b) = rotr(sp(b) ^ sp(c), 12);          \
  sp(a) = sp(a) + sp(b) + (y);              \
  sp(d) = rotr(sp(d) ^ sp(a), 8);           \
  sp(c) = sp(c) + sp(d);                    \
  sp(b) = rotr(sp(b) ^ sp(c), 7);
    B3_GP(0, 4, 8, 12, m[0], m[1]) B3_GP(1, 5, 9, 13, m[2], m[3])
    B3_GP(2, 6, 10, 14, m[4], m[5]) B3_GP(3, 7, 11, 15, m[6], m[7])
    B3_GP(1, 6, 11, 12, 0u, 0u) B3_GP(2, 7, 8, 13, 0u, 0u) B3_GP(3, 4, 9, 14, 0u, 0u)
#undef B3_GP
#undef sp
  }
  for (uint64_t start = base;; start += T) {
    if (start > limit || __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < start) return;
    const uint64_t nonce = start + g;
    m[8] = (uint32_t)nonce;
    m[9] = (uint32_t)(nonce >> 32);
    uint32_t s0 = p0, s1 = p1, s2 = p2, s3 = p3, s4 = p4, s5 = p5, s6 = p6, s7 = p7, s8 = p8, s9 = p9, s10 = p10,
             s11 = p11, s12 = p12, s13 = p13, s14 = p14, s15 = p15;
    B3_G(0, 5, 10, 15, m[8], m[9])  // round 1's nonce G
    // rounds 2..7 (b3::compress's schedule)
    B3_ROUND(2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
    B3_ROUND(3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1)
    B3_ROUND(10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6)
    B3_ROUND(12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4)
    B3_ROUND(9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7)
    B3_ROUND(11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13)
    const uint64_t h = (uint64_t)(s0 ^ s8) | ((uint64_t)(s1 ^ s9) << 32);
    const uint32_t tz = h == 0 ? 64u : (uint32_t)__builtin_ctzll(h);
    if (tz >= bits) atomicMin(result, (unsigned long long)nonce);
  }
}

// DefaultRandomCoin::draw_integers(q, N, nonce) on the device coin: seed' =
// merge_with_int(seed, nonce); position i = u64_le(merge_with_int(seed', i + 1)) & (N - 1).
// Raw draws (unsorted, with repeats: the host sorts and dedups, as the prover does).
__global__ void k_query_positions(const uint32_t* __restrict__ seedp, const unsigned long long* __restrict__ nonce_p,
                                  uint32_t q, uint64_t N, uint64_t* __restrict__ pos) {
  const uint64_t nonce = *nonce_p;
  uint32_t m[16], s2[8];
#pragma unroll
  for (int k = 0; k < 8; k++) m[k] = seedp[k];
  m[8] = (uint32_t)nonce;
  m[9] = (uint32_t)(nonce >> 32);
#pragma unroll
  for (int k = 10; k < 16; k++) m[k] = 0;
  b3::set_iv(s2);
  b3::compress_r(s2, m, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
  for (uint32_t i = threadIdx.x; i < q; i += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 8; k++) m[k] = s2[k];
    m[8] = i + 1;
    m[9] = 0;
#pragma unroll
    for (int k = 10; k < 16; k++) m[k] = 0;
    uint32_t out[8];
    b3::set_iv(out);
    b3::compress_r(out, m, 0, 40, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT);
    pos[i] = ((uint64_t)out[0] | ((uint64_t)out[1] << 32)) & (N - 1);
  }
}

// Every opening any batch proof over the drawn positions can need, gathered
// without a host plan: for raw position i (block x) and segment y (0 = trace +
// constraint rows, 1 + l = FRI layer l) the row values and the full sibling path
// of the leaf (a batch proof's nodes are a subset of its leaves' sibling paths).
// Layout per segment: q records of rec_words words at out + seg_off[y].
__global__ __launch_bounds__(128) void k_gather_full(FullGatherArgs a, const uint64_t* __restrict__ pos,
                                                     uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x, y = blockIdx.y, t = threadIdx.x;
  const uint64_t p = pos[i];
  const uint64_t B = 1ull << a.logB;
  uint32_t* rec = out + a.seg_off[y] + (uint64_t)i * a.rec_words[y];
  if (y == 0) {
    const uint64_t j = p & (B - 1), tt = p >> a.logB;
    const uint32_t nv = a.w + a.C, depth = a.logN;
    for (uint32_t e = t; e < 4 * nv; e += blockDim.x) {  // row values: w trace then C constraint felts
      const uint32_t c = e >> 2;
      const felt* src = c < a.w ? a.tlde + ((uint64_t)c * B + j) * a.n : a.clde + ((uint64_t)(c - a.w) * B + j) * a.n;
      rec[e] = reinterpret_cast<const uint32_t*>(src + tt)[e & 3];
    }
    uint32_t* paths = rec + 4 * nv;
    for (uint32_t e = t; e < 2 * depth * 8; e += blockDim.x) {  // trace path, then constraint path
      const uint32_t tree = e / (depth * 8), d = (e / 8) % depth, wd = e & 7;
      const uint64_t node = (((1ull << a.logN) + p) >> d) ^ 1ull;
      paths[e] = (tree ? a.cnodes : a.tnodes)[node * 8 + wd];
    }
  } else {
    const uint32_t l = y - 1, logR = a.logrows[l];
    const uint64_t r = p & ((1ull << logR) - 1), m = a.m[l];
    for (uint32_t e = t; e < 64; e += blockDim.x) {  // 16 values E[r + k*Rows] (coset-major)
      const uint64_t idx = r + ((uint64_t)(e >> 2) << logR);
      const uint64_t j = idx & (B - 1), tt = idx >> a.logB;
      rec[e] = reinterpret_cast<const uint32_t*>(a.E[l] + j * m + tt)[e & 3];
    }
    for (uint32_t e = t; e < logR * 8; e += blockDim.x) {
      const uint32_t d = e / 8, wd = e & 7;
      const uint64_t node = (((1ull << logR) + r) >> d) ^ 1ull;
      rec[64 + e] = a.fnodes[l][node * 8 + wd];
    }
  }
}

// fold-by-16: u = iDFT16(row) (unscaled), result = (1/16) sum_k u_k beta^k,
// beta = alpha / x_r; eps_inv[m] = w_16^-m for m < 8, eps_inv[8] = 1/16.
// Layer evaluations are coset-major (coset jl of Bl, m = 16*m16 positions):
// local row q = jl*m16 + t' is the natural row r = (j0 + jl) + B*t' whose 16
// values sit at positions t' + k*m16 of the same coset; out is coset-major.
__device__ __forceinline__ felt fri_fold_row(const felt* __restrict__ E, uint64_t q, uint32_t logm16, uint32_t j0,
                                             uint32_t logB, const felt* alpha_p, felt off_inv,
                                             const felt* __restrict__ itw_lev, const felt* __restrict__ eps_inv) {
  const uint64_t m16 = 1ull << logm16;
  const uint64_t jl = q >> logm16, tp = q & (m16 - 1);
  const uint64_t r = (j0 + jl) + (tp << logB);
  const felt* src = E + (jl << (logm16 + 4)) + tp;
  felt v[16];
#pragma unroll
  for (int k = 0; k < 16; k++) v[k] = src[k * m16];
  // Gentleman-Sande, natural in -> bit-reversed out (fully unrolled, constant indices)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    felt x = v[i], y = v[i + 8];
    v[i] = add(x, y);
    v[i + 8] = i == 0 ? sub(x, y) : mul(sub(x, y), eps_inv[i]);
  }
#pragma unroll
  for (int blk = 0; blk < 16; blk += 8) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      felt x = v[blk + i], y = v[blk + i + 4];
      v[blk + i] = add(x, y);
      v[blk + i + 4] = i == 0 ? sub(x, y) : mul(sub(x, y), eps_inv[2 * i]);
    }
  }
#pragma unroll
  for (int blk = 0; blk < 16; blk += 4) {
    felt x0 = v[blk], y0 = v[blk + 2], x1 = v[blk + 1], y1 = v[blk + 3];
    v[blk] = add(x0, y0);
    v[blk + 2] = sub(x0, y0);
    v[blk + 1] = add(x1, y1);
    v[blk + 3] = mul(sub(x1, y1), eps_inv[4]);
  }
#pragma unroll
  for (int blk = 0; blk < 16; blk += 2) {
    felt x = v[blk], y = v[blk + 1];
    v[blk] = add(x, y);
    v[blk + 1] = sub(x, y);
  }
  felt beta = mul(*alpha_p, mul(off_inv, itw_lev[r]));
  // Horner over k = 15..0 with u_k = v[rev4(k)], rev4 = {0,8,4,12,2,10,6,14,1,9,5,13,3,11,7,15}
  // (Estrin's scheme measured slower: 18 products instead of 15, and one wave
  // per SIMD issues in order, so the shorter chain buys nothing)
  felt acc = v[15];
  acc = add(mul(acc, beta), v[7]);
  acc = add(mul(acc, beta), v[11]);
  acc = add(mul(acc, beta), v[3]);
  acc = add(mul(acc, beta), v[13]);
  acc = add(mul(acc, beta), v[5]);
  acc = add(mul(acc, beta), v[9]);
  acc = add(mul(acc, beta), v[1]);
  acc = add(mul(acc, beta), v[14]);
  acc = add(mul(acc, beta), v[6]);
  acc = add(mul(acc, beta), v[10]);
  acc = add(mul(acc, beta), v[2]);
  acc = add(mul(acc, beta), v[12]);
  acc = add(mul(acc, beta), v[4]);
  acc = add(mul(acc, beta), v[8]);
  acc = add(mul(acc, beta), v[0]);
  return mul(acc, eps_inv[8]);
}

// The same fold by a quad of lanes (the latency-bound small layers: one row's
// 35 serial products become 19). Lane qd holds v[qd + 4i], i < 4: the iDFT's
// span-8 and span-4 stages stay in the lane, the span-2 and span-1 stages pair
// lanes qd^2 and qd^1 (DPP). Lane qd then holds u_k for k = 4*rev2(qd) + rev2(i),
// evaluates its 4 coefficients by Horner, scales by beta^(4*rev2(qd)), and the
// quad sums the four partials; every lane of the quad returns the folded value.
// All 4 lanes of a quad must be active (callers clamp the row, not the lanes).
template <int K>
__device__ __forceinline__ felt quad_xor(felt v) {  // lane qd ^ K's value (K = 1 or 2)
  constexpr int ctrl = K == 1 ? 0xB1 : 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
  uint32_t w[4] = {(uint32_t)v.lo, (uint32_t)(v.lo >> 32), (uint32_t)v.hi, (uint32_t)(v.hi >> 32)};
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[i], ctrl, 0xF, 0xF, false);
  felt r;
  r.lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  r.hi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  return r;
}

__device__ __forceinline__ felt fri_fold_row_quad(const felt* __restrict__ E, uint64_t q, uint32_t qd, uint32_t logm16,
                                                  uint32_t j0, uint32_t logB, const felt* alpha_p, felt off_inv,
                                                  const felt* __restrict__ itw_lev,
                                                  const felt* __restrict__ eps_inv) {
  const uint64_t m16 = 1ull << logm16;
  const uint64_t jl = q >> logm16, tp = q & (m16 - 1);
  const uint64_t r = (j0 + jl) + (tp << logB);
  const felt* src = E + (jl << (logm16 + 4)) + tp;
  felt v[4];
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = src[(qd + 4 * i) * m16];
  const felt beta = mul(*alpha_p, mul(off_inv, itw_lev[r]));
  // span 8: pairs (qd, qd+8) = (v0, v2) and (qd+4, qd+12) = (v1, v3)
  {
    const felt a0 = add(v[0], v[2]), a1 = add(v[1], v[3]);
    v[2] = mul(sub(v[0], v[2]), eps_inv[qd]);
    v[3] = mul(sub(v[1], v[3]), eps_inv[qd + 4]);
    v[0] = a0;
    v[1] = a1;
  }
  // span 4 in each half: pairs (v0, v1) and (v2, v3), twiddle w^-(2 qd)
  {
    const felt e = eps_inv[2 * qd];
    const felt a0 = add(v[0], v[1]), a2 = add(v[2], v[3]);
    v[1] = mul(sub(v[0], v[1]), e);
    v[3] = mul(sub(v[2], v[3]), e);
    v[0] = a0;
    v[2] = a2;
  }
  // span 2 (lanes qd, qd^2; position 3 of each 4-block takes w^-4), span 1 (lanes qd, qd^1)
  const bool up2 = qd & 2, up1 = qd & 1;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const felt p = quad_xor<2>(v[i]);
    v[i] = up2 ? sub(p, v[i]) : add(v[i], p);
  }
  if (qd == 3) {
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = mul(v[i], eps_inv[4]);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const felt p = quad_xor<1>(v[i]);
    v[i] = up1 ? sub(p, v[i]) : add(v[i], p);
  }
  // v[i] = u_{4 rq + rev2(i)}, rq = rev2(qd): Horner over u_{4rq+3}, u_{4rq+2}, u_{4rq+1}, u_{4rq}
  felt acc = add(mul(v[3], beta), v[1]);
  acc = add(mul(acc, beta), v[2]);
  acc = add(mul(acc, beta), v[0]);
  const uint32_t rq = ((qd & 1) << 1) | (qd >> 1);
  const felt b2 = mul(beta, beta), b4 = mul(b2, b2), b8 = mul(b4, b4), b12 = mul(b8, b4);
  const felt sc = rq == 0 ? one() : (rq == 1 ? b4 : (rq == 2 ? b8 : b12));
  acc = mul(acc, sc);
  acc = add(acc, quad_xor<1>(acc));
  acc = add(acc, quad_xor<2>(acc));
  return mul(acc, eps_inv[8]);
}

// small layers (latency-bound): one quad per row
__global__ __launch_bounds__(TPB) void k_fri_fold16_quad(const felt* __restrict__ E, uint64_t rows, uint32_t logm16,
                                                         uint32_t j0, uint32_t logB, const felt* __restrict__ alpha_p,
                                                         felt off_inv, const felt* __restrict__ itw_lev,
                                                         const felt* __restrict__ eps_inv, felt* __restrict__ out) {
  const uint64_t tq = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  const uint64_t q = tq >> 2;
  const uint32_t qd = (uint32_t)(tq & 3);
  const felt v = fri_fold_row_quad(E, q < rows ? q : rows - 1, qd, logm16, j0, logB, alpha_p, off_inv, itw_lev,
                                   eps_inv);  // whole quads active; clamped rows are not stored
  if (q < rows && qd == 0) out[q] = v;
}

__global__ __launch_bounds__(TPB) void k_fri_fold16(const felt* __restrict__ E, uint64_t rows, uint32_t logm16,
                                                    uint32_t j0, uint32_t logB, const felt* __restrict__ alpha_p,
                                                    felt off_inv,
                                                    const felt* __restrict__ itw_lev,
                                                    const felt* __restrict__ eps_inv, felt* __restrict__ out) {
  const uint64_t q = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (q >= rows) return;
  out[q] = fri_fold_row(E, q, logm16, j0, logB, alpha_p, off_inv, itw_lev, eps_inv);
}

// The FRI tail in one 512-thread block (world 1): for each layer of <= 128
// rows, quad-hashed leaves -> tree (quad merges, levels in LDS, every node
// written) -> coin step (alpha, root) -> fold into the next layer; then the
// remainder (as k_fri_remainder). Replaces 2 launches per small layer + the
// remainder launch, each of which costs its ~15-25 us launch/latency floor.
__global__ __launch_bounds__(512) void k_fri_tail(FriTailArgs a) {
  __shared__ uint32_t sd[128 * 9];
  __shared__ felt s_c[256];
  __shared__ felt s_tw[256];
  __shared__ uint32_t s_cv[32][8];
  const uint32_t t = threadIdx.x, nd = t >> 2, q = t & 3;
  for (uint32_t l = 0; l < a.nl; l++) {
    const FriTailLayer y = a.ly[l];
    const uint32_t R = 1u << (y.logm16 + a.logB);  // rows = leaves (<= 128, host-checked)
    MerkleArgs ma{};
    ma.src = y.E;
    ma.R = 1ull << y.logm16;
    ma.logB = a.logB;
    ma.cols = 16;
    if (nd < R) {  // whole quads
      uint32_t o0, o1;
      fri_leaf_quad(ma, nd, q, o0, o1);
      sd[nd * 9 + q] = o0;
      sd[nd * 9 + 4 + q] = o1;
      uint32_t* dst = y.nodes + (uint64_t)(R + nd) * 8;
      dst[q] = o0;
      dst[4 + q] = o1;
    }
    for (uint32_t s = R >> 1; s >= 1; s >>= 1) {
      __syncthreads();
      uint32_t o0 = 0, o1 = 0;
      if (nd < s) {
        uint32_t mm[16];
#pragma unroll
        for (int i = 0; i < 8; i++) { mm[i] = sd[(2 * nd) * 9 + i]; mm[8 + i] = sd[(2 * nd + 1) * 9 + i]; }
        merge_quad<false>(mm, q, o0, o1);
      }
      __syncthreads();
      if (nd < s) {
        sd[nd * 9 + q] = o0;
        sd[nd * 9 + 4 + q] = o1;
        uint32_t* dst = y.nodes + (uint64_t)(s + nd) * 8;
        dst[q] = o0;
        dst[4 + q] = o1;
      }
    }
    __syncthreads();
    if (t < 4) {
      uint32_t r[8];
#pragma unroll
      for (int i = 0; i < 8; i++) r[i] = sd[i];  // the root (node 1)
      coin_fri_step(a.coin_seed, r, y.alpha_out, y.root_out);
    }
    __threadfence();  // alpha (and this layer's fold output below) visible block-wide
    __syncthreads();
    {  // one quad per row (R <= 128 rows, 128 quads): whole quads active, rows clamped
      const felt fv = fri_fold_row_quad(y.E, nd < R ? nd : R - 1, q, y.logm16, 0, a.logB, y.alpha_out, y.off_inv,
                                        y.lev, a.eps_inv);
      if (nd < R && q == 0) y.out[nd] = fv;
    }
    __threadfence();
    __syncthreads();
  }
  // remainder: interpolate the last layer (D = m * B points) into ncoef = m
  // coefficients, commit, reseed (k_fri_remainder)
  const uint32_t m = a.rem_m;
  remainder_coeffs_block(a.rem_E, a.logB, m, m, a.rem_off_inv, a.wd_inv, a.d_inv, s_c, s_tw);
  for (uint32_t k = t; k < m; k += blockDim.x) a.rem_out[k] = s_c[k];
  uint32_t h[8];
  hash_felts_fast([&](uint32_t i) { return s_c[i]; }, m, h, s_cv);
  quad_reseed_to(a.coin_seed, h, a.coin_seed);
  if (t < 8) a.commit_out[t] = h[t];
}

}  // namespace


// tree build by lane-subtree passes: each lane hashes or merges 2^H nodes of the
// level below into one subtree root (the leaf passes H = 1, the rest H = 2)
template <int MODE, int H>
static void merkle_pass(Prof& prof, hipStream_t s, const MerkleArgs& a, const char* name, double bytes) {
  if ((a.L >> H) == 0) launch_fail(ZKP_ERR_DEVICE, "internal: lane pass over fewer nodes than one subtree");
  const dim3 g(blocks_for(a.L >> H));
  LAUNCH(prof, name, s, bytes, hipLaunchKernelGGL((k_merkle_lane<MODE, H>), g, dim3(256), 0, s, a));
}

// upper levels: wide levels by lane passes (4 levels each), the narrow top by
// the LDS-fused kernel (9 levels per launch, parallel tail)
bool merkle_upper(Prof& prof, hipStream_t s, uint32_t* nodes, uint64_t L, const MerkleTail* tail) {
  // lane passes down to 2^18 nodes (2^10-2^16 measured slower: profiles/r03_ab_merkle_lane_min.txt,
  // r04_ab_merkle_lane_min16.txt)
  constexpr uint32_t lane_min_log = 18;
  while (L > 1) {
    MerkleArgs a{};
    a.nodes = nodes;
    a.L = L;
    // lane passes only while they have >= 2^14 lanes (4 levels, 15 serial merges
    // per lane); below that the 9-level LDS-fused blocks have the shorter
    // critical path (9 merges) and fill more CUs
    if (L >= (1ull << lane_min_log)) {
      // 2 levels per lane: measured faster than 3-4 (fewer live digests, more waves;
      // tests/native/kbench_merkle.cpp, profiles/r02_kbench_merkle.txt)
      merkle_pass<2, 2>(prof, s, a, "merkle_upper", (double)L * 32.0 * 1.5);
      L >>= 2;
    } else {
      uint64_t blocks = (L + 511) / 512;
      const bool finish = tail && tail->done && blocks <= 512;  // this launch completes the tree
      if (finish) a.tail = *tail;
      LAUNCH(prof, "merkle_top9", s, (double)L * 64.0,
             hipLaunchKernelGGL(k_merkle_fused<2>, dim3((uint32_t)blocks), dim3(256), 0, s, a));
      if (finish) return true;
      L = L >= 512 ? L / 512 : 1;
    }
  }
  return false;
}

bool launch_merkle_lde(Prof& prof, hipStream_t s, const felt* lde, uint32_t cols, uint32_t logB, uint64_t n,
                       uint32_t* nodes, uint64_t L, const MerkleTail* tail, const LastCol* lc, const GuLazy* gl) {
  MerkleArgs a{};
  a.src = lde;
  a.n = n;
  a.cols = cols;
  a.logB = logB;
  a.nodes = nodes;
  a.L = L;
  // each lane hashes 2 rows and merges them (H = 1): measured faster than deeper
  // lane subtrees, whose extra live digests cost waves (kbench_merkle.cpp)
  constexpr uint32_t H = 1;
  if (L < 2) launch_fail(ZKP_ERR_DEVICE, "internal: LDE tree of one row");
  if (gl) {  // lazy GlobalUpdate columns (wide rows: the generic lane pass)
    a.gl = *gl;
    if (gu_row_shape(cols, *gl))
      merkle_pass<5, H>(prof, s, a, "merkle_lde", (double)L * (gl->wi * 16.0 + 64.0));
    else
      merkle_pass<4, H>(prof, s, a, "merkle_lde", (double)L * (gl->wi * 16.0 + 64.0));
  } else if (lc) {  // the caller checked merkle_can_derive(cols, L)
    if (cols < 2 || cols > 8) launch_fail(ZKP_ERR_DEVICE, "internal: derived-column leaf shape");
    a.lc = *lc;
    const double bytes = (double)L * (cols * 16.0 + 48.0);
    const dim3 g(blocks_for(L >> 1));
#define ZKP_LEAF2D(CC)                                                                                      \
  case CC:                                                                                                  \
    LAUNCH(prof, "merkle_lde", s, bytes, hipLaunchKernelGGL((k_merkle_leaf2<CC, true>), g, dim3(256), 0, s, a)); \
    break;
    switch (cols) { ZKP_LEAF2D(2) ZKP_LEAF2D(3) ZKP_LEAF2D(4) ZKP_LEAF2D(5) ZKP_LEAF2D(6) ZKP_LEAF2D(7) ZKP_LEAF2D(8) }
#undef ZKP_LEAF2D
  } else if (cols > 64 && logB >= 1 && L <= (1ull << 20)) {  // wide rows, few of them: a quad of lanes per row
    LAUNCH(prof, "merkle_lde", s, (double)L * (cols * 16.0 + 48.0),
           hipLaunchKernelGGL(k_merkle_wide, dim3(blocks_for(L * 4)), dim3(256), 0, s, a));
  } else if (cols <= 8) {  // rows preloaded (profiles/r03_ab_leaf_preload.txt)
    const double bytes = (double)L * (cols * 16.0 + 48.0);
    const dim3 g(blocks_for(L >> 1));
#define ZKP_LEAF2(CC) \
  case CC: LAUNCH(prof, "merkle_lde", s, bytes, hipLaunchKernelGGL(k_merkle_leaf2<CC>, g, dim3(256), 0, s, a)); break;
    switch (cols) { ZKP_LEAF2(1) ZKP_LEAF2(2) ZKP_LEAF2(3) ZKP_LEAF2(4) ZKP_LEAF2(5) ZKP_LEAF2(6) ZKP_LEAF2(7)
                    ZKP_LEAF2(8) }
#undef ZKP_LEAF2
  } else {
    merkle_pass<0, H>(prof, s, a, "merkle_lde", (double)L * (cols * 16.0 + 64.0));
  }
  return merkle_upper(prof, s, nodes, L >> H, tail);
}

// largest FRI layer (log2 rows) whose leaves are hashed by quads (tuned with
// tests/native/kbench_top.cpp, which builds this file with -DZKP_FRI_QUAD_TUNING)
#ifdef ZKP_FRI_QUAD_TUNING
uint32_t fri_quad_max_log = 13;
#else
static constexpr uint32_t fri_quad_max_log = 13;
#endif

bool launch_merkle_fri(Prof& prof, hipStream_t s, const felt* E, uint64_t m16, uint32_t logB, uint32_t F,
                       uint32_t* nodes, const MerkleTail* tail) {
  const uint64_t R = m16 << logB;
  MerkleArgs a{};
  a.src = E;
  a.R = m16;
  a.logB = logB;
  a.cols = F;
  a.nodes = nodes;
  a.L = R;
  if (F == 16 && R <= (1ull << fri_quad_max_log)) {  // profiles/r02_ab_quad_leaves.txt
    // small layers (<= 2^13 rows): one quad of lanes per row, 64 rows and 6 levels
    // per block. At 2^15 rows the quads' extra instructions made it slower
    // (72 vs 53 us); at 2^11 / 2^7 / 2^3 rows it is faster (30/22/21 vs 40/34/29 us)
    uint64_t blocks = (R + 63) / 64;
    const bool finish = tail && tail->done && blocks <= 512;
    if (finish) a.tail = *tail;
    LAUNCH(prof, "merkle_fri", s, (double)R * (F * 16.0 + 64.0),
           hipLaunchKernelGGL((k_merkle_fused<1, true>), dim3((uint32_t)blocks), dim3(256), 0, s, a));
    if (finish) return true;
    return merkle_upper(prof, s, nodes, blocks, tail);
  }
  if (R <= (1ull << 16)) {
    // small layers: a lane subtree would serialise 19 compressions per lane on a
    // few waves; hash 2 rows per thread and build 9 levels per block instead
    uint64_t blocks = (R + 511) / 512;
    const bool finish = tail && tail->done && blocks <= 512;
    if (finish) a.tail = *tail;
    LAUNCH(prof, "merkle_fri", s, (double)R * (F * 16.0 + 64.0),
           hipLaunchKernelGGL(k_merkle_fused<1>, dim3((uint32_t)blocks), dim3(256), 0, s, a));
    if (finish) return true;
    return merkle_upper(prof, s, nodes, R >= 512 ? R / 512 : 1, tail);
  }
  merkle_pass<1, 2>(prof, s, a, "merkle_fri", (double)R * (F * 16.0 + 64.0));  // R > 2^16
  return merkle_upper(prof, s, nodes, R >> 2, tail);
}

void preload_merkle_module() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, (const void*)k_merkle_level);
}

void launch_leaf_hash_lde(Prof& prof, hipStream_t s, const felt* lde, uint32_t cols, uint32_t logB, uint64_t n,
                          uint32_t* nodes, uint64_t L) {
  LAUNCH(prof, "leaf_hash_lde", s, (double)L * (cols * 16.0 + 32.0),
         hipLaunchKernelGGL(k_leaf_hash_lde, dim3(blocks_for(L)), dim3(TPB), 0, s, lde, cols, logB, n, nodes, L));
}

void launch_leaf_hash_fri(Prof& prof, hipStream_t s, const felt* E, uint64_t R, uint32_t F, uint32_t* nodes) {
  LAUNCH(prof, "leaf_hash_fri", s, (double)R * (F * 16.0 + 32.0),
         hipLaunchKernelGGL(k_leaf_hash_fri, dim3(blocks_for(R)), dim3(TPB), 0, s, E, R, F, nodes));
}

void launch_merkle_tree(Prof& prof, hipStream_t s, uint32_t* nodes, uint64_t L) {
  uint64_t lvl = L / 2;
  for (; lvl >= 2048; lvl >>= 1)
    LAUNCH(prof, "merkle_level", s, (double)lvl * 96.0,
           hipLaunchKernelGGL(k_merkle_level, dim3(blocks_for(lvl)), dim3(TPB), 0, s, nodes, lvl));
  if (lvl >= 1)
    LAUNCH(prof, "merkle_top", s, (double)lvl * 2.0 * 96.0, hipLaunchKernelGGL(k_merkle_top, dim3(1), dim3(1024), 0, s, nodes, lvl));
}

void launch_grind(Prof& prof, hipStream_t s, const uint32_t* seed_words, const uint32_t* seed_dev, uint64_t base,
                  uint64_t count, uint32_t bits, unsigned long long* result) {
  SeedArg sa;
  for (int i = 0; i < 8; i++) sa.w[i] = seed_words ? seed_words[i] : 0u;
  LAUNCH(prof, "grind", s, 0.0,
         hipLaunchKernelGGL(k_grind, dim3(blocks_for(count)), dim3(TPB), 0, s, sa, seed_dev, base, count, bits,
                            result));
}

void launch_grind_all(Prof& prof, hipStream_t s, const uint32_t* seed_dev, uint64_t base, uint64_t limit,
                      uint32_t bits, unsigned long long* result) {
  LAUNCH(prof, "grind", s, 0.0,
         // 1024 x 256 threads: 4 waves per SIMD, and 2^18 nonces per iteration keeps the
         // overshoot past the minimum small (2^21 expected tries at the reference's 21 bits;
         // 2048 blocks measured no faster)
         hipLaunchKernelGGL(k_grind_all, dim3(1024), dim3(TPB), 0, s, seed_dev, base, limit, bits, result));
}

void launch_query_positions(Prof& prof, hipStream_t s, const uint32_t* seed_dev, const unsigned long long* nonce,
                            uint32_t q, uint64_t N, uint64_t* pos) {
  LAUNCH(prof, "positions", s, 0.0, hipLaunchKernelGGL(k_query_positions, dim3(1), dim3(256), 0, s, seed_dev, nonce, q,
                                                       N, pos));
}

void launch_gather_full(Prof& prof, hipStream_t s, const FullGatherArgs& a, uint32_t q, const uint64_t* pos,
                        uint32_t* out) {
  LAUNCH(prof, "gather", s, 0.0,
         hipLaunchKernelGGL(k_gather_full, dim3(q, 1 + a.nlayers), dim3(128), 0, s, a, pos, out));
}

void launch_pack(Prof& prof, hipStream_t s, const PackArgs& a, void* dst) {
  uint64_t mx = 0;
  for (uint32_t i = 0; i < a.n; i++) mx = a.bytes[i] > mx ? a.bytes[i] : mx;
  const uint32_t bx = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((mx / 4 + TPB - 1) / TPB, 1), 64);
  LAUNCH(prof, "gather", s, 0.0,
         hipLaunchKernelGGL(k_pack, dim3(bx, a.n), dim3(TPB), 0, s, a, reinterpret_cast<uint32_t*>(dst)));
}

void launch_fri_remainder(Prof& prof, hipStream_t s, const felt* E, uint32_t logB, uint32_t m, felt off_inv,
                          felt wd_inv, felt d_inv, uint32_t* seed, felt* rem_out, uint32_t* commit_out) {
  const uint32_t D = m << logB, ncoef = m;
  if (D > 256) launch_fail(ZKP_ERR_DEVICE, "internal: device remainder over 256 values");  // larger ones stay on the host
  LAUNCH(prof, "coin", s, 0.0,
         hipLaunchKernelGGL(k_fri_remainder, dim3(1), dim3(TPB), 0, s, E, logB, m, off_inv, wd_inv, d_inv, ncoef,
                            seed, rem_out, commit_out));
}

void launch_coin_fri_layer(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, felt* alpha_out,
                           uint32_t* root_out) {
  LAUNCH(prof, "coin", s, 0.0, hipLaunchKernelGGL(k_coin_fri_layer, dim3(1), dim3(64), 0, s, seed, root, alpha_out, root_out));
}

void launch_fri_fold(Prof& prof, hipStream_t s, const felt* E, uint64_t m16, uint32_t Bl, uint32_t j0,
                     uint32_t logB, uint32_t F, const felt* alpha, felt off_inv, const felt* itw, uint32_t logD,
                     const felt* eps_inv, felt* out) {
  (void)F;  // only 16 is compiled (the reference's fri_folding_factor)
  const felt* lev = itw + ((1ull << (logD - 1)) - 1);  // w_D^-r, r < D/2
  uint32_t logm16 = 0;
  while ((1ull << logm16) < m16) logm16++;
  const uint64_t rows = m16 * Bl;
  // up to 2^15 rows the layer is latency-bound (under one wave per SIMD): a quad
  // per row shortens the chain; above that the one-lane form issues fewer products
  if (rows <= (1ull << 15)) {
    LAUNCH(prof, "fri_fold16", s, (double)rows * (16 * 16.0 + 16.0),
           hipLaunchKernelGGL(k_fri_fold16_quad, dim3(blocks_for(rows * 4)), dim3(TPB), 0, s, E, rows, logm16, j0,
                              logB, alpha, off_inv, lev, eps_inv, out));
    return;
  }
  LAUNCH(prof, "fri_fold16", s, (double)rows * (16 * 16.0 + 16.0),
         hipLaunchKernelGGL(k_fri_fold16, dim3(blocks_for(rows)), dim3(TPB), 0, s, E, rows, logm16, j0, logB, alpha,
                            off_inv, lev, eps_inv, out));
}

void launch_fri_tail(Prof& prof, hipStream_t s, const FriTailArgs& a) {
  if (a.nl > FRI_TAIL_MAX || (a.rem_m << a.logB) > 256) launch_fail(ZKP_ERR_DEVICE, "internal: FRI tail shape");
  for (uint32_t l = 0; l < a.nl; l++)
    if (a.ly[l].logm16 + a.logB > 7)  // <= 128 rows: one quad per row in 512 threads
      launch_fail(ZKP_ERR_DEVICE, "internal: FRI tail layer over 128 rows");
  LAUNCH(prof, "fri_tail", s, 0.0, hipLaunchKernelGGL(k_fri_tail, dim3(1), dim3(512), 0, s, a));
}

void launch_leaf_hash_shard(Prof& prof, hipStream_t s, int mode, const felt* src, uint64_t n, uint32_t cols,
                            uint32_t logBl, uint32_t logrows, uint32_t logrr, uint32_t logK, uint32_t k,
                            uint32_t* send, const LastCol* lc, const GuLazy* gl) {
  const uint64_t cnt = 1ull << (logrows - logK + logBl);
  const double bytes = (double)cnt * (cols * 16.0 + 32.0);
  const dim3 g(blocks_for(cnt));
  const LastCol lcv = lc ? *lc : LastCol{};
  const GuLazy glv = gl ? *gl : GuLazy{};
#define ZKP_SHARD_LEAF(CC)                                                                                   \
  case CC:                                                                                                   \
    LAUNCH(prof, "leaf_hash_shard", s, bytes,                                                                \
           hipLaunchKernelGGL((k_leaf_hash_shard<0, CC>), g, dim3(TPB), 0, s, src, n, cols, logBl, logrows, \
                              logrr, logK, k, send, lcv, glv));                                                   \
    break;
#define ZKP_SHARD_LEAFD(CC)                                                                                  \
  case CC:                                                                                                   \
    LAUNCH(prof, "leaf_hash_shard", s, bytes,                                                                \
           hipLaunchKernelGGL((k_leaf_hash_shard<0, CC, true>), g, dim3(TPB), 0, s, src, n, cols, logBl,    \
                              logrows, logrr, logK, k, send, lcv, glv));                                          \
    break;
  if (gl) {  // lazy GlobalUpdate columns
    if (mode != 0) launch_fail(ZKP_ERR_DEVICE, "internal: lazy columns in a FRI leaf pass");
    if (gu_row_shape(cols, *gl))
      LAUNCH(prof, "leaf_hash_shard", s, (double)cnt * (gl->wi * 16.0 + 32.0),
             hipLaunchKernelGGL(k_leaf_hash_shard<5>, g, dim3(TPB), 0, s, src, n, cols, logBl, logrows, logrr, logK,
                                k, send, lcv, glv));
    else
      LAUNCH(prof, "leaf_hash_shard", s, (double)cnt * (gl->wi * 16.0 + 32.0),
             hipLaunchKernelGGL(k_leaf_hash_shard<4>, g, dim3(TPB), 0, s, src, n, cols, logBl, logrows, logrr, logK,
                                k, send, lcv, glv));
  } else if (lc) {  // the caller checked merkle_can_derive
    if (mode != 0 || cols < 2 || cols > 8) launch_fail(ZKP_ERR_DEVICE, "internal: derived-column shard leaf shape");
    switch (cols) { ZKP_SHARD_LEAFD(2) ZKP_SHARD_LEAFD(3) ZKP_SHARD_LEAFD(4) ZKP_SHARD_LEAFD(5)
                    ZKP_SHARD_LEAFD(6) ZKP_SHARD_LEAFD(7) ZKP_SHARD_LEAFD(8) }
  } else if (mode == 0 && cols <= 8) {
    switch (cols) { ZKP_SHARD_LEAF(1) ZKP_SHARD_LEAF(2) ZKP_SHARD_LEAF(3) ZKP_SHARD_LEAF(4) ZKP_SHARD_LEAF(5)
                    ZKP_SHARD_LEAF(6) ZKP_SHARD_LEAF(7) ZKP_SHARD_LEAF(8) }
  } else if (mode == 0)
    LAUNCH(prof, "leaf_hash_shard", s, bytes,
           hipLaunchKernelGGL(k_leaf_hash_shard<0>, g, dim3(TPB), 0, s, src, n, cols, logBl,
                              logrows, logrr, logK, k, send, lcv, glv));
  else
    LAUNCH(prof, "leaf_hash_shard", s, (double)cnt * (cols * 16.0 + 32.0),
           hipLaunchKernelGGL(k_leaf_hash_shard<1>, dim3(blocks_for(cnt)), dim3(TPB), 0, s, src, n, cols, logBl,
                              logrows, logrr, logK, k, send, lcv, glv));
}
#undef ZKP_SHARD_LEAFD
#undef ZKP_SHARD_LEAF

void launch_merkle_from_shards(Prof& prof, hipStream_t s, const uint32_t* recv, uint32_t logB, uint32_t logrr,
                               uint32_t logK, uint32_t* nodes, uint32_t* done) {
  // with done (a zeroed per-stream counter) the top launch's last block finishes the
  // subtree instead of a separate one-block launch
  MerkleTail fin{};
  fin.done = done;
  const MerkleTail* tail = done ? &fin : nullptr;
  const uint64_t L = 1ull << (logB + logrr);
  if (L < 4) {
    LAUNCH(prof, "leaf_unpack", s, (double)L * 64.0,
           hipLaunchKernelGGL(k_leaf_unpack, dim3(blocks_for(L)), dim3(TPB), 0, s, recv, logB, logrr, logK, nodes, L));
    merkle_upper(prof, s, nodes, L, tail);
    return;
  }
  // the unpack fused into the first 2-level lane pass: each lane loads its 4 leaf
  // digests from the receive buffer, stores them as leaves and merges 2 levels
  MerkleArgs a{};
  a.src = reinterpret_cast<const felt*>(recv);
  a.cols = logrr - logK;
  a.logB = logB;
  a.nodes = nodes;
  a.L = L;
  merkle_pass<3, 2>(prof, s, a, "merkle_upper", (double)L * 32.0 * 2.5);
  merkle_upper(prof, s, nodes, L >> 2, tail);
}

// top levels of a sharded tree from the all-gathered subtree roots (R <= 64):
// top[R + s] = root of rank s's subtree, top[k] = merge(top[2k], top[2k+1]);
// the root (top[1]) stays on the device, and the block then runs the
// commitment's coin step (MerkleTail op: coefficients, z or the FRI alpha) as a
// world-1 tree's last block does
__global__ __launch_bounds__(256) void k_shard_top(const uint32_t* __restrict__ roots, uint32_t R,
                                                   uint32_t* __restrict__ top, MerkleTail tail) {
  const uint32_t t = threadIdx.x;
  if (t < R)
    for (int i = 0; i < 8; i++) top[(R + t) * 8 + i] = roots[t * 8 + i];
  for (uint32_t h = R >> 1; h >= 1; h >>= 1) {
    __syncthreads();
    if (t < h) {
      uint32_t l[8], r[8], o[8];
      load_digest(top + (2 * (h + t)) * 8, l);
      load_digest(top + (2 * (h + t) + 1) * 8, r);
      merge8<false>(l, r, o);
      store_digest(top + (h + t) * 8, o);
    }
  }
  __syncthreads();
  if (tail.op != MERKLE_TAIL_NONE) merkle_tail_op(tail, top + 8);  // whole block
}

void launch_shard_top(Prof& prof, hipStream_t s, const uint32_t* roots, uint32_t R, uint32_t* top,
                      const MerkleTail* tail) {
  const MerkleTail tl = tail ? *tail : MerkleTail{};
  LAUNCH(prof, "merkle_top9", s, (double)R * 64.0,
         hipLaunchKernelGGL(k_shard_top, dim3(1), dim3(256), 0, s, roots, R, top, tl));
}

void launch_dt_draw_coeffs(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, uint32_t method,
                           uint32_t ncoef, felt* cc) {
  LAUNCH(prof, "coin", s, 0.0,
         hipLaunchKernelGGL(k_dt_draw_coeffs, dim3(1), dim3(TPB), 0, s, seed, root, method, ncoef, cc));
}

void launch_dt_draw_z(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, felt wn, uint32_t logn,
                      felt* zz, felt* pw) {
  LAUNCH(prof, "coin", s, 0.0, hipLaunchKernelGGL(k_dt_draw_z, dim3(1), dim3(64), 0, s, seed, root, wn, logn, zz, pw));
}

void launch_dt_deep_coeffs(Prof& prof, hipStream_t s, uint32_t* seed, const felt* ood, uint32_t w, uint32_t C,
                           uint32_t method, felt* gamma, felt* dk) {
  LAUNCH(prof, "coin", s, 0.0,
         hipLaunchKernelGGL(k_dt_deep_coeffs, dim3(1), dim3(64), 0, s, seed, ood, w, C, method, gamma, dk));
}
