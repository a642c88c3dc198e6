// NTT kernel timing harness (TUNING ONLY): builds with csrc/ntt.hip directly
// (variant flags on the hipcc line) and times launch_ntt on the C2 shapes with
// random canonical data. Prints ms per launch_ntt call and an output checksum,
// which must agree across variants (all variants compute identical values).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../zk_stark_project_amd/csrc/zkp_internal.hpp"

// profiling stubs (the product's Prof lives in kernels.hip)
hipEvent_t Prof::get_event() { return nullptr; }
void Prof::begin(const char*, hipStream_t, double) {}
void Prof::end(hipStream_t) {}
void launch_fail(int, const char*) { abort(); }

__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

static void fill(std::vector<felt>& v, uint64_t seed) {
  for (auto& x : v) {
    seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
    uint64_t lo = seed;
    seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17;
    x.lo = lo;
    x.hi = seed & 0x7fffffffffffffffull;  // < p
  }
}

int main(int argc, char** argv) {
  const uint32_t logn = argc > 1 ? atoi(argv[1]) : 20, logB = 3, logN = logn + logB;
  const uint64_t n = 1ull << logn, N = 1ull << logN;
  const uint32_t cols = 6, B = 1u << logB;
  std::vector<felt> h_src((size_t)cols * n), h_tw(N), h_S((size_t)B * n);
  fill(h_src, 1); fill(h_tw, 2); fill(h_S, 3);
  felt *src, *dst, *tw, *S;
  hipMalloc(&src, h_src.size() * 16); hipMalloc(&dst, (size_t)cols * N * 16);
  hipMalloc(&tw, N * 16); hipMalloc(&S, h_S.size() * 16);
  hipMemcpy(src, h_src.data(), h_src.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(tw, h_tw.data(), N * 16, hipMemcpyHostToDevice);
  hipMemcpy(S, h_S.data(), h_S.size() * 16, hipMemcpyHostToDevice);
  hipStream_t st;
  hipStreamCreate(&st);
  Prof pf;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, auto fn, int iters) {
    fn();
    hipStreamSynchronize(st);
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; i++) fn();
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> out((size_t)cols * N * 2);
    hipMemcpy(out.data(), dst, out.size() * 8, hipMemcpyDeviceToHost);
    uint64_t ck = 0;
    for (size_t i = 0; i < out.size(); i++) ck = ck * 0x9e3779b97f4a7c15ull + out[i];
    printf("%-34s %8.4f ms/call  checksum %016llx\n", name, ms / iters, (unsigned long long)ck);
  };
  {
    felt* big;
    hipMalloc(&big, (size_t)cols * N * 16);
    const uint64_t nv = (uint64_t)cols * N;  // 16-B elements
    hipEvent_t c0, c1;
    hipEventCreate(&c0); hipEventCreate(&c1);
    hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, st, (const uint4*)dst, (uint4*)big, nv);
    hipEventRecord(c0, st);
    for (int i = 0; i < 10; i++)
      hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, st, (const uint4*)dst, (uint4*)big, nv);
    hipEventRecord(c1, st);
    hipEventSynchronize(c1);
    float ms;
    hipEventElapsedTime(&ms, c0, c1);
    printf("%-34s %8.4f ms/call  %.2f TB/s (read+write)\n", "copy 6 x 8 x n felts", ms / 10,
           2.0 * nv * 16 / (ms / 10 * 1e-3) / 1e12);
    hipFree(big);
  }
  if (argc > 2 && std::string(argv[2]) == "tu") {
    // the reference's TrainingUpdate proof (2^13 x 240, blowup 16): one upload group of
    // 64 columns, extended to 16 cosets, and its 64-column interpolation
    const uint32_t tc = 64, tB = 16, tlogN = logn + 4;
    felt *tsrc, *tdst, *tS, *ttw;
    std::vector<felt> hs((size_t)tc * n), hS((size_t)tB * n), ht(1ull << tlogN);
    fill(hs, 4); fill(hS, 5); fill(ht, 6);
    hipMalloc(&tsrc, hs.size() * 16); hipMalloc(&tdst, (size_t)tc * tB * n * 16);
    hipMalloc(&tS, hS.size() * 16); hipMalloc(&ttw, ht.size() * 16);
    hipMemcpy(tsrc, hs.data(), hs.size() * 16, hipMemcpyHostToDevice);
    hipMemcpy(tS, hS.data(), hS.size() * 16, hipMemcpyHostToDevice);
    hipMemcpy(ttw, ht.data(), ht.size() * 16, hipMemcpyHostToDevice);
    hipEvent_t a0, a1;
    hipEventCreate(&a0); hipEventCreate(&a1);
    auto time = [&](const char* name, auto fn) {
      fn();
      hipStreamSynchronize(st);
      hipEventRecord(a0, st);
      for (int i = 0; i < 20; i++) fn();
      hipEventRecord(a1, st);
      hipEventSynchronize(a1);
      float ms;
      hipEventElapsedTime(&ms, a0, a1);
      std::vector<uint64_t> out((size_t)tc * n * 2);
      hipMemcpy(out.data(), tdst, out.size() * 8, hipMemcpyDeviceToHost);
      uint64_t ck = 0;
      for (size_t i = 0; i < out.size(); i++) ck = ck * 0x9e3779b97f4a7c15ull + out[i];
      printf("%-34s %8.4f ms/call  checksum %016llx\n", name, ms / 20, (unsigned long long)ck);
    };
    NttBatch lb{tsrc, tdst, tS, n, n, tB, tB, tc * tB};
    time("TU: DIT lde 64 cols x 16 cosets", [&] { launch_ntt(pf, st, lb, logn, true, ttw, tlogN); });
    NttBatch ib{tsrc, tdst, nullptr, n, n, 1, 1, tc};
    time("TU: DIF 64 columns", [&] { launch_ntt(pf, st, ib, logn, false, ttw, tlogN); });
    return 0;
  }
  if (argc > 2) {  // one rank of a coset-sharded proof (C4 at 2^22): 5 batch-1 coset LDEs
    hipStream_t st2;
    hipStreamCreate(&st2);
    hipEvent_t fork, join;
    hipEventCreate(&fork); hipEventCreate(&join);
    auto col = [&](uint32_t m, hipStream_t s) {
      NttBatch b{src + (size_t)m * n, dst + (size_t)m * n, S, n, n, 1, 1, 1};
      launch_ntt(pf, s, b, logn, true, tw, logN);
    };
    run("rank: 5 batch-1 LDEs, one stream", [&] { for (uint32_t m = 0; m < 5; m++) col(m, st); }, 10);
    run("rank: 5 batch-1 LDEs, alternating", [&] {
      hipEventRecord(fork, st);
      hipStreamWaitEvent(st2, fork, 0);
      for (uint32_t m = 0; m < 5; m++) col(m, (m & 1) ? st2 : st);
      hipEventRecord(join, st2);
      hipStreamWaitEvent(st, join, 0);
    }, 10);
    NttBatch b5{src, dst, S, n, n, 1, 1, 5};
    run("rank: 5 columns in one batch", [&] { launch_ntt(pf, st, b5, logn, true, tw, logN); }, 10);
    return 0;
  }
  // composition LDE: 6 columns x 8 cosets (DIT, coset scale fused)
  NttBatch lde{src, dst, S, n, n, B, B, cols * B};
  run("DIT lde 6 cols x 8 cosets", [&] { launch_ntt(pf, st, lde, logn, true, tw, logN); }, 10);
  run("DIT lde 6x8, first pass only", [&] { launch_ntt(pf, st, lde, logn, true, tw, logN, 0); }, 10);
  run("DIT lde 6x8, second pass only", [&] { launch_ntt(pf, st, lde, logn, true, tw, logN, 1); }, 10);
  {
    // the same, pipelined over two streams in column chunks: pass 1 of chunk k+1 (VALU-bound)
    // beside pass 2 of chunk k (HBM-heavier)
    hipStream_t st2;
    hipStreamCreate(&st2);
    std::vector<hipEvent_t> ev(16);
    for (auto& e : ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
    hipEvent_t fork, join;
    hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    hipEventCreateWithFlags(&join, hipEventDisableTiming);
    for (uint32_t per : {1u, 2u, 3u}) {
      char name[64];
      snprintf(name, sizeof name, "DIT lde 6x8, pipelined %u col/chunk", per);
      run(name, [&] {
        hipEventRecord(fork, st);
        hipStreamWaitEvent(st2, fork, 0);
        uint32_t k = 0;
        for (uint32_t c0 = 0; c0 < cols; c0 += per, k++) {
          const uint32_t cw = c0 + per <= cols ? per : cols - c0;
          NttBatch cb{src + (size_t)c0 * n, dst + (size_t)c0 * B * n, S, n, n, B, B, cw * B};
          launch_ntt(pf, st, cb, logn, true, tw, logN, 0);
          hipEventRecord(ev[k], st);
          hipStreamWaitEvent(st2, ev[k], 0);
          launch_ntt(pf, st2, cb, logn, true, tw, logN, 1);
        }
        hipEventRecord(join, st2);
        hipStreamWaitEvent(st, join, 0);
      }, 10);
    }
  }
  // trace LDE: 1 column x 8 cosets
  NttBatch lde1{src, dst, S, n, n, B, B, B};
  run("DIT lde 1 col x 8 cosets", [&] { launch_ntt(pf, st, lde1, logn, true, tw, logN); }, 20);
  // CE-coset interpolation: 8 inverse transforms (DIF)
  NttBatch inv8{src, dst, nullptr, n, n, 1, 1, 6};
  run("DIF 6 arrays", [&] { launch_ntt(pf, st, inv8, logn, false, tw, logN); }, 20);
  return 0;
}
