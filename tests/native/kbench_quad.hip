// kbench_quad.hip — latency of the pieces of a Merkle tree top level (TUNING ONLY):
// one wave's chain of dependent quad-cooperative BLAKE3 merges (compress_quad /
// compress_quad_r), the same with each level's hand-off through LDS and a block
// barrier (256 threads), and with the level's digest stored to global memory.
// Prints microseconds per level.  make -C tests/native kbench_quad
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../zk_stark_project_amd/csrc/felt.hpp"
#include "../../zk_stark_project_amd/csrc/blake3_quad.hpp"

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(2);                                                \
    }                                                         \
  } while (0)

constexpr int LEVELS = 64;

// MODE 0: registers only (the digest feeds the next message directly)
// MODE 1: + LDS store, barrier, LDS load of the next level's 16 message words
// MODE 2: + the digest stored to global memory per level (as the tree writes every node)
template <int MODE, bool ROLLED>
__global__ __launch_bounds__(256) void k_chain(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t sd[64 * 9];
  const uint32_t t = threadIdx.x, q = t & 3, nd = t >> 2;
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = seed * (i + 1) + t;
  uint32_t o0 = 0, o1 = 0;
  for (int lv = 0; lv < LEVELS; lv++) {
    o0 = sel4(q, b3::iv(0), b3::iv(1), b3::iv(2), b3::iv(3));
    o1 = sel4(q, b3::iv(4), b3::iv(5), b3::iv(6), b3::iv(7));
    if (ROLLED)
      compress_quad_r(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, o0, o1);
    else
      compress_quad(m, q, b3::CHUNK_START | b3::CHUNK_END | b3::ROOT, o0, o1);
    if (MODE == 0) {
      uint32_t g[8];
      quad_gather8(o0, o1, g);
#pragma unroll
      for (int i = 0; i < 8; i++) { m[i] = g[i]; m[8 + i] ^= g[i]; }
    } else {
      __syncthreads();
      if (nd < 64) { sd[nd * 9 + q] = o0; sd[nd * 9 + 4 + q] = o1; }
      if (MODE == 2) { out[(lv * 64 + nd) * 8 + q] = o0; out[(lv * 64 + nd) * 8 + 4 + q] = o1; }
      __syncthreads();
      const uint32_t a = (2 * nd) & 63, b = (2 * nd + 1) & 63;
#pragma unroll
      for (int i = 0; i < 8; i++) { m[i] = sd[a * 9 + i]; m[8 + i] = sd[b * 9 + i]; }
    }
  }
  if (t < 4) { out[LEVELS * 64 * 8 + 2 * t] = o0; out[LEVELS * 64 * 8 + 2 * t + 1] = o1; }
}

template <int MODE, bool ROLLED>
static void run(const char* name, uint32_t* out, int threads) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL((k_chain<MODE, ROLLED>), dim3(1), dim3(threads), 0, 0, out, 7u);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL((k_chain<MODE, ROLLED>), dim3(1), dim3(threads), 0, 0, out, 7u);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-34s threads=%3d  %6.3f us per level (%d levels, launch included)\n", name, threads,
         ms * 1e3 / reps / LEVELS, LEVELS);
}

int main() {
  setvbuf(stdout, NULL, _IONBF, 0);
  uint32_t* out;
  CK(hipMalloc(&out, (LEVELS * 64 * 8 + 64) * 4));
  run<0, false>("regs only, unrolled", out, 64);
  run<0, true>("regs only, rolled", out, 64);
  run<0, false>("regs only, unrolled", out, 256);
  run<1, false>("LDS + barrier, unrolled", out, 256);
  run<1, true>("LDS + barrier, rolled", out, 256);
  run<2, false>("LDS + barrier + global store, unrolled", out, 256);
  run<2, true>("LDS + barrier + global store, rolled", out, 256);
  run<1, false>("LDS + barrier, unrolled", out, 64);
  return 0;
}
