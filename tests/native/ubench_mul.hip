// Microbenchmark of f128 multiplication variants on gfx950 (TEST/TUNING ONLY).
// Each thread runs 4 independent chains x_k <- x_k * y for ITERS iterations.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "../../zk_stark_project_amd/csrc/felt.hpp"
#include "../../zk_stark_project_amd/csrc/felt_dev.hpp"

using namespace fp;

// --- variant 2: 64-bit limbs via unsigned __int128 products
__device__ __forceinline__ felt mul_v2(felt a, felt b) {
  typedef unsigned __int128 u128;
  u128 p00 = (u128)a.lo * b.lo, p01 = (u128)a.lo * b.hi, p10 = (u128)a.hi * b.lo, p11 = (u128)a.hi * b.hi;
  u128 mid = p01 + p10;
  u128 midc = (mid < p01) ? ((u128)1 << 64) : 0;
  u128 lo = p00 + (mid << 64);
  u128 c1 = lo < p00;
  u128 hi = p11 + (mid >> 64) + midc + c1;
  uint32_t r[8] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)(lo >> 64), (uint32_t)(lo >> 96),
                   (uint32_t)hi, (uint32_t)(hi >> 32), (uint32_t)(hi >> 64), (uint32_t)(hi >> 96)};
  return reduce8(r);
}

// --- variant 3: product scanning (column sums) with explicit 96-bit accumulator
__device__ __forceinline__ felt mul_v3(felt a, felt b) {
  const uint32_t x[4] = {(uint32_t)a.lo, (uint32_t)(a.lo >> 32), (uint32_t)a.hi, (uint32_t)(a.hi >> 32)};
  const uint32_t y[4] = {(uint32_t)b.lo, (uint32_t)(b.lo >> 32), (uint32_t)b.hi, (uint32_t)(b.hi >> 32)};
  uint32_t r[8];
  uint64_t acc = 0;  // low 64 of column accumulator
  uint32_t ov = 0;   // overflow word
#pragma unroll
  for (int k = 0; k < 7; k++) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int j = k - i;
      if (j < 0 || j > 3) continue;
      uint64_t p = (uint64_t)x[i] * y[j];
      uint64_t s = acc + p;
      ov += (s < p);
      acc = s;
    }
    r[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
  r[7] = (uint32_t)acc;
  return reduce8(r);
}

template <int V>
__global__ void k_bench(felt* io, int iters) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  felt x0 = io[4 * t], x1 = io[4 * t + 1], x2 = io[4 * t + 2], x3 = io[4 * t + 3];
  felt y = make(0x123456789abcdefULL + t, 0x0fedcba987654321ULL);
  for (int i = 0; i < iters; i++) {
    if (V == 1) { x0 = mul(x0, y); x1 = mul(x1, y); x2 = mul(x2, y); x3 = mul(x3, y); }
    if (V == 2) { x0 = mul_v2(x0, y); x1 = mul_v2(x1, y); x2 = mul_v2(x2, y); x3 = mul_v2(x3, y); }
    if (V == 3) { x0 = mul_v3(x0, y); x1 = mul_v3(x1, y); x2 = mul_v3(x2, y); x3 = mul_v3(x3, y); }
    if (V == 5) { x0 = add(x0, y); x1 = add(x1, y); x2 = add(x2, y); x3 = add(x3, y); }
    if (V == 6) { x0 = fpd::mul(x0, y); x1 = fpd::mul(x1, y); x2 = fpd::mul(x2, y); x3 = fpd::mul(x3, y); }
    if (V == 7) { x0 = fpd::add(x0, y); x1 = fpd::add(x1, y); x2 = fpd::add(x2, y); x3 = fpd::add(x3, y); }
    if (V == 8) { x0 = sub(x0, y); x1 = sub(x1, y); x2 = sub(x2, y); x3 = sub(x3, y); }
    if (V == 10) { fpd::mul_x2(x0, y, x1, y, x0, x1); fpd::mul_x2(x2, y, x3, y, x2, x3); }
    if (V == 11) { felt s0, d0, s1, d1; fpd::addsub(x0, x1, s0, d0); fpd::addsub(x2, x3, s1, d1); x0 = s0; x1 = d0; x2 = s1; x3 = d1; }
    if (V == 12) { felt s0, d0, s1, d1; s0 = add(x0, x1); d0 = sub(x0, x1); s1 = add(x2, x3); d1 = sub(x2, x3); x0 = s0; x1 = d0; x2 = s1; x3 = d1; }
    if (V == 9) { x0 = fpd::sub(x0, y); x1 = fpd::sub(x1, y); x2 = fpd::sub(x2, y); x3 = fpd::sub(x3, y); }
  }
  io[4 * t] = x0; io[4 * t + 1] = x1; io[4 * t + 2] = x2; io[4 * t + 3] = x3;
}

// raw v_mad_u64_u32 throughput: 8 independent chains
__global__ void k_mad(uint64_t* io, int iters) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t a[8];
  for (int k = 0; k < 8; k++) a[k] = io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = (uint64_t)(uint32_t)a[k] * m + a[k];
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

int main() {
  setvbuf(stdout, NULL, _IONBF, 0);
  const int blocks = 256 * 16, tpb = 256, iters = 2000;
  const size_t nthr = (size_t)blocks * tpb;
  felt* d;
  hipMalloc(&d, nthr * 4 * sizeof(felt));
  hipMemset(d, 1, nthr * 4 * sizeof(felt));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // correctness cross-check between variants on a few values
  {
    felt h[8];
    for (int i = 0; i < 8; i++) h[i] = make(0x9e3779b97f4a7c15ULL * (i + 1), 0x7fffffffffffffffULL - i);
    felt* dd;
    hipMalloc(&dd, 4096 * 4 * sizeof(felt));
    hipMemcpy(dd, h, sizeof h, hipMemcpyHostToDevice);
    (void)dd;
  }
  auto run = [&](const char* name, auto launch, double ops_per_thread_iter) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double ops = 3.0 * nthr * (double)iters * ops_per_thread_iter;
    printf("%-28s %8.3f ms  %8.2f Gop/s\n", name, ms, ops / (ms * 1e-3) / 1e9);
  };
  run("mul v1 (32b schoolbook)", [&] { hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("mul v2 (u128 products)", [&] { hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("mul v3 (product scan)", [&] { hipLaunchKernelGGL(k_bench<3>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("mul v6 (asm carry chains)", [&] { hipLaunchKernelGGL(k_bench<6>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("mul x2 interleaved", [&] { hipLaunchKernelGGL(k_bench<10>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("addsub interleaved", [&] { hipLaunchKernelGGL(k_bench<11>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("add+sub separate", [&] { hipLaunchKernelGGL(k_bench<12>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("add asm", [&] { hipLaunchKernelGGL(k_bench<7>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("sub", [&] { hipLaunchKernelGGL(k_bench<8>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("sub asm", [&] { hipLaunchKernelGGL(k_bench<9>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("add", [&] { hipLaunchKernelGGL(k_bench<5>, dim3(blocks), dim3(tpb), 0, 0, d, iters); }, 4);
  run("v_mad_u64_u32 raw", [&] { hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(tpb), 0, 0, (uint64_t*)d, iters); }, 8);
  // verify variants agree (random inputs incl. values near p and 2^128)
  {
    felt* a;
    hipMalloc(&a, nthr * 4 * sizeof(felt));
    const size_t cnt = 4096 * 4;
    felt* h0 = (felt*)malloc(cnt * sizeof(felt));
    felt* h1 = (felt*)malloc(cnt * sizeof(felt));
    felt* h2 = (felt*)malloc(cnt * sizeof(felt));
    uint64_t st = 88172645463325252ULL;
    for (size_t i = 0; i < cnt; i++) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      uint64_t lo = st;
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      uint64_t hi = st;
      if (i % 7 == 0) hi = 0xffffffffffffffffULL;  // near p
      if (i % 11 == 0) lo = 0xffffd30000000000ULL + (st & 3);
      felt v = make(lo, hi);
      if (ge_p(v)) v = make(lo - 0xffffd30000000001ULL, 0);  // keep canonical
      h0[i] = v;
    }
    int pairs[6][2] = {{1, 2}, {1, 6}, {5, 7}, {8, 9}, {1, 10}, {12, 11}};
    for (auto& pr : pairs) {
      felt* outs[2] = {h1, h2};
      for (int k = 0; k < 2; k++) {
        hipMemcpy(a, h0, cnt * sizeof(felt), hipMemcpyHostToDevice);
        int v = pr[k];
        if (v == 1) hipLaunchKernelGGL(k_bench<1>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 2) hipLaunchKernelGGL(k_bench<2>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 5) hipLaunchKernelGGL(k_bench<5>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 6) hipLaunchKernelGGL(k_bench<6>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 7) hipLaunchKernelGGL(k_bench<7>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 8) hipLaunchKernelGGL(k_bench<8>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 9) hipLaunchKernelGGL(k_bench<9>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 10) hipLaunchKernelGGL(k_bench<10>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 11) hipLaunchKernelGGL(k_bench<11>, dim3(16), dim3(256), 0, 0, a, 3);
        if (v == 12) hipLaunchKernelGGL(k_bench<12>, dim3(16), dim3(256), 0, 0, a, 3);
        hipMemcpy(outs[k], a, cnt * sizeof(felt), hipMemcpyDeviceToHost);
      }
      printf("variant %d agrees with %d: %s\n", pr[1], pr[0], memcmp(h1, h2, cnt * sizeof(felt)) == 0 ? "yes" : "NO");
    }
  }
  return 0;
}
