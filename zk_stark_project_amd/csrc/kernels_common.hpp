// kernels_common.hpp — helpers shared by the kernel translation units
// (kernels.hip, ntt.hip): launch accounting, compile-time loops, domain points.
#pragma once
#include "../../include/zkp.h"
#include "zkp_internal.hpp"
#include "blake3.hpp"

#include <algorithm>
#include <type_traits>

using namespace fp;

#define TPB 256

#define LAUNCH(prof, name, stream, bytes, ...)                 \
  do {                                                          \
    (prof).begin(name, stream, (double)(bytes));                \
    __VA_ARGS__;                                                \
    (prof).end(stream);                                         \
  } while (0)

// Deferred-check field ops (felt_dev.hpp fpd::Rare). dmul / dadd with FAST take
// every result as canonical and record the evidence that one may not be (a carry
// past 2^128, a top limb 0xffffffff); a kernel whose Rare is set recomputes its
// values with FAST = false, the exact forms. kc::opaque_tid gives that exact pass
// thread indices the compiler cannot match with the fast pass's, so nothing the
// fast pass loaded is kept live for it.
#if defined(__HIP_DEVICE_COMPILE__)
using Rare = fpd::Rare;
#else
struct Rare {
  bool any() const { return false; }
};
#endif

template <bool FAST>
__device__ __forceinline__ felt dmul(felt a, felt b, Rare& q) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (FAST) return fpd::mul_z(a, b, q);
#endif
  (void)q;
  return mul(a, b);
}
template <bool FAST>
__device__ __forceinline__ felt dadd(felt a, felt b, Rare& q) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (FAST) return fpd::add_z(a, b, q);
#endif
  (void)q;
  return add(a, b);
}

namespace kc {

template <bool FAST>
__device__ __forceinline__ uint32_t opaque_tid() {
  uint32_t t = threadIdx.x;
  if constexpr (!FAST) asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ uint32_t rev_bits(uint32_t x, uint32_t bits) {
  return bits == 0 ? 0u : (__brev(x) >> (32 - bits));
}

// compile-time unrolled loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

constexpr int ilog2_const(int v) { return v <= 1 ? 0 : 1 + ilog2_const(v / 2); }
constexpr int rev_const(int x, int bits) { return bits == 0 ? 0 : ((x & 1) << (bits - 1)) | rev_const(x >> 1, bits - 1); }

inline uint32_t ilog2_u64(uint64_t v) {
  uint32_t l = 0;
  while ((1ull << l) < v) l++;
  return l;
}

}  // namespace kc
