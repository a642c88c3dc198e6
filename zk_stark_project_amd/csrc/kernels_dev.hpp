// kernels_dev.hpp — device helpers shared by the kernel translation units
// (kernels.hip: tables, constraint evaluation, OOD, DEEP, composition, gathers;
// merkle.hip: BLAKE3 leaves and trees, the device transcript, grinding, FRI).
#pragma once
#include "kernels_common.hpp"

namespace {

constexpr int EVAL_CH = 8;  // points per thread (batch-inversion chunk)

// w_N^e for e < N (table holds e < N/2; w_N^(N/2) = -1)
__device__ __forceinline__ felt tw_full(const felt* tw, uint64_t e, uint32_t logN) {
  uint64_t half = 1ull << (logN - 1);
  return e < half ? tw[e] : neg(tw[e - half]);
}

// domain point of local index q of a coset-major shard: cx[q / n] * w_n^(q % n)
__device__ __forceinline__ felt point_x(const PointMap& m, uint64_t q) {
  return mul(m.cx[q >> m.logn], tw_full(m.twn, q & ((1ull << m.logn) - 1), m.logn));
}

// point handled by (thread, slot k) of a block of EVAL_CH*TPB points: slots
// are TPB apart so that every load/store of a wave is contiguous
#define EVAL_POINT(k) ((uint64_t)blockIdx.x * (TPB * EVAL_CH) + (uint64_t)(k) * TPB + threadIdx.x)

__device__ __forceinline__ void store_digest(uint32_t* dst, const uint32_t d[8]) {
  uint4* p = reinterpret_cast<uint4*>(dst);
  p[0] = make_uint4(d[0], d[1], d[2], d[3]);
  p[1] = make_uint4(d[4], d[5], d[6], d[7]);
}
__device__ __forceinline__ void load_digest(const uint32_t* src, uint32_t d[8]) {
  const uint4* p = reinterpret_cast<const uint4*>(src);
  uint4 a = p[0], b = p[1];
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

inline uint32_t blocks_for(uint64_t n, uint32_t per_block = TPB) {
  uint64_t b = (n + per_block - 1) / per_block;
  return (uint32_t)(b == 0 ? 1 : b);
}
inline uint32_t grid_stride_blocks(uint64_t n) {
  uint64_t b = (n + TPB - 1) / TPB;
  if (b > 8192) b = 8192;
  return (uint32_t)(b == 0 ? 1 : b);
}
inline uint32_t ilog2_u64(uint64_t v) {
  uint32_t l = 0;
  while ((1ull << l) < v) l++;
  return l;
}

}  // namespace
