// Wide-matrix read-rate harness (TUNING ONLY): how fast can a kernel read
// W column arrays of N felts (C3 trace LDE: W = 120, N = 2^22) when every point
// reads all W columns (DEEP, row hashing, linear constraints)? Variants: column
// stride N (the product's layout) or N + pad, and points per thread.
#include "../../zk_stark_project_amd/csrc/kernels_common.hpp"

#include <cstdio>
#include <cstdlib>

using kc::static_for;

struct F {
  uint64_t lo, hi;
};

// lazy dot-product variants (as csrc/kernels.hip k_lincomb): PT points per
// thread, U columns per round, PF = prefetch the next round's columns
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void lacc(uint64_t acc[7], uint32_t top[7], fpd::L4 g, fpd::L4 t) {
  const uint32_t gw[4] = {g.w0, g.w1, g.w2, g.w3}, tw[4] = {t.w0, t.w1, t.w2, t.w3};
  static_for<0, 4>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    static_for<0, 4>([&](auto jj) {
      constexpr int j = decltype(jj)::value;
      uint64_t co;
      acc[i + j] = fpd::mad_co(gw[i], tw[j], acc[i + j], co);
      top[i + j] = fpd::addc_0(top[i + j], co);
    });
  });
}
#endif
template <int PT, int U, bool PF>
__global__ __launch_bounds__(256) void k_lin(const felt* __restrict__ base, uint64_t cstride, uint32_t W,
                                             const felt* __restrict__ coef, felt* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * PT) + threadIdx.x;
  uint64_t acc[PT][7];
  uint32_t top[PT][7];
  for (int p = 0; p < PT; p++)
    for (int k = 0; k < 7; k++) { acc[p][k] = 0; top[p][k] = 0; }
  felt v[U][PT];
  auto load = [&](uint32_t c) {
    static_for<0, U>([&](auto uu) {
      constexpr int u = decltype(uu)::value;
      static_for<0, PT>([&](auto pp) {
        constexpr int p = decltype(pp)::value;
        v[u][p] = base[(uint64_t)(c + u) * cstride + q0 + (uint64_t)p * 256];
      });
    });
  };
  if (PF) load(0);
  for (uint32_t c = 0; c + U <= W; c += U) {
    felt cur[U][PT];
    if (PF) {
      static_for<0, U>([&](auto uu) { static_for<0, PT>([&](auto pp) {
        cur[decltype(uu)::value][decltype(pp)::value] = v[decltype(uu)::value][decltype(pp)::value]; }); });
      if (c + 2 * U <= W) load(c + U);
    } else {
      load(c);
      static_for<0, U>([&](auto uu) { static_for<0, PT>([&](auto pp) {
        cur[decltype(uu)::value][decltype(pp)::value] = v[decltype(uu)::value][decltype(pp)::value]; }); });
    }
    asm volatile("" ::: "memory");
    static_for<0, U>([&](auto uu) {
      constexpr int u = decltype(uu)::value;
      const fpd::L4 g = fpd::split(coef[c + u]);
      static_for<0, PT>([&](auto pp) {
        constexpr int p = decltype(pp)::value;
        lacc(acc[p], top[p], g, fpd::split(cur[u][p]));
      });
    });
  }
  static_for<0, PT>([&](auto pp) {
    constexpr int p = decltype(pp)::value;
    felt r;
    r.lo = 0; r.hi = 0;
    for (int k = 0; k < 7; k++) { r.lo ^= acc[p][k] + k; r.hi += top[p][k] ^ (uint64_t)k; }
    out[q0 + (uint64_t)p * 256] = r;
  });
#endif
}

template <int PT>
__global__ __launch_bounds__(256) void k_cols(const F* __restrict__ base, uint64_t cstride, uint32_t W, uint64_t N,
                                              F* __restrict__ out) {
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * PT) + threadIdx.x;
  uint64_t a[PT], b[PT];
#pragma unroll
  for (int p = 0; p < PT; p++) a[p] = b[p] = 0;
  uint32_t c = 0;
  for (; c + 4 <= W; c += 4) {
    F v[4][PT];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int p = 0; p < PT; p++) v[u][p] = base[(uint64_t)(c + u) * cstride + q0 + (uint64_t)p * 256];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int p = 0; p < PT; p++) { a[p] ^= v[u][p].lo; b[p] += v[u][p].hi; }
  }
  for (; c < W; c++)
#pragma unroll
    for (int p = 0; p < PT; p++) {
      F v = base[(uint64_t)c * cstride + q0 + (uint64_t)p * 256];
      a[p] ^= v.lo; b[p] += v.hi;
    }
#pragma unroll
  for (int p = 0; p < PT; p++) out[q0 + (uint64_t)p * 256] = F{a[p], b[p]};
}

int main() {
  const uint32_t W = 120;
  const uint64_t N = 1ull << 22, PAD = 512;
  F *base, *out;
  if (hipMalloc(&base, (size_t)W * (N + PAD) * sizeof(F)) != hipSuccess) return 1;
  if (hipMalloc(&out, N * sizeof(F)) != hipSuccess) return 1;
  if (getenv("KB_RANDOM")) {  // random canonical-ish felts instead of a byte pattern
    const size_t cnt = (size_t)W * (N + PAD) * 2;
    uint64_t* h = (uint64_t*)malloc(cnt * 8);
    uint64_t x = 88172645463325252ull;
    for (size_t i = 0; i < cnt; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (i & 1) ? (x >> 1) : x; }
    (void)hipMemcpy(base, h, cnt * 8, hipMemcpyHostToDevice);
    free(h);
  } else {
    (void)hipMemset(base, 1, (size_t)W * (N + PAD) * sizeof(F));
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char* name, uint64_t stride, int pt) {
    auto launch = [&] {
      if (pt == 1) hipLaunchKernelGGL(k_cols<1>, dim3(N / 256), dim3(256), 0, 0, base, stride, W, N, out);
      if (pt == 2) hipLaunchKernelGGL(k_cols<2>, dim3(N / 512), dim3(256), 0, 0, base, stride, W, N, out);
      if (pt == 4) hipLaunchKernelGGL(k_cols<4>, dim3(N / 1024), dim3(256), 0, 0, base, stride, W, N, out);
      if (pt == 8) hipLaunchKernelGGL(k_cols<8>, dim3(N / 2048), dim3(256), 0, 0, base, stride, W, N, out);
    };
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < 10; i++) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s PT=%d  %7.3f ms  %6.2f TB/s\n", name, pt, ms, (double)W * N * 16 / (ms * 1e-3) / 1e12);
  };
  for (int pt : {1, 2, 8}) run("stride N (product layout)", N, pt);
  felt* coef;
  if (hipMalloc(&coef, W * sizeof(felt)) != hipSuccess) return 1;
  (void)hipMemset(coef, 3, W * sizeof(felt));
  auto lin = [&](const char* name, auto kern, int pt) {
    auto launch = [&] {
      hipLaunchKernelGGL(kern, dim3(N / (256 * pt)), dim3(256), 0, 0, (const felt*)base, N, W, coef, (felt*)out);
    };
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < 10; i++) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s %7.3f ms  %6.2f TB/s\n", name, ms, (double)W * N * 16 / (ms * 1e-3) / 1e12);
  };
  lin("lin PT2 U4 (product)", k_lin<2, 4, false>, 2);
  lin("lin PT1 U8", k_lin<1, 8, false>, 1);
  lin("lin PT1 U4", k_lin<1, 4, false>, 1);
  lin("lin PT2 U4 prefetch", k_lin<2, 4, true>, 2);
  lin("lin PT1 U4 prefetch", k_lin<1, 4, true>, 1);
  lin("lin PT1 U8 prefetch", k_lin<1, 8, true>, 1);
  lin("lin PT4 U2", k_lin<4, 2, false>, 4);
  return 0;
}
