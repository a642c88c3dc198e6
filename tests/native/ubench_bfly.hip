// ubench_bfly.hip — butterfly floor of the f128 NTT on gfx950 (TEST/TUNING ONLY,
// not linked into libzkp). DESIGN.md §4 "The butterfly floor" rests on it, and
// bench.py's roofline.valu_floor_frac divides by the rate it prints.
//
// A register-resident stream of radix-2 DIT butterflies x, y <- x + w*y, x - w*y:
// each thread holds 8 values and runs radix-8 rounds of 12 butterflies (spans 1,
// 2, 4, two independent butterflies interleaved per step) — the dataflow of
// k_ntt8's 3-stage register rounds with no HBM, LDS or twiddle traffic. Variants:
//   lib    the library's forms: fpd::mul_x2 + fp::add / fp::sub (canon_rare and
//          add_sum fast paths, felt_dev.hpp);
//   exact  the round-3 forms, kept here for the A/B: the exact canonical select
//          after every product and every sum (4 adds + 4 selects each).
// Both must give identical values (checked). `--check` runs the field-op edge
// cases (values at p - 1, sums in [p, 2^128), products whose residue sits at the
// top of the range or below 2^128 - p) against the host's portable arithmetic.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tests/native/ubench_bfly.hip -o tests/native/ubench_bfly
// Run:   tests/native/ubench_bfly [--check]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../zk_stark_project_amd/csrc/felt.hpp"

using namespace fp;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

#if defined(__HIP_DEVICE_COMPILE__)
namespace exact {
using namespace fpd;
// round 3: every product and every sum ends in the exact select
__device__ __forceinline__ void mul_x2(felt a, felt b, felt c, felt d, felt& ab, felt& cd) {
  uint32_t r[8], s[8];
  mul256x2(split(a), split(b), split(c), split(d), r, s);
  const uint32_t K = 0x2d00u;
  uint64_t t = mul_wide(r[4], K), tt = mul_wide(s[4], K);
  uint32_t q0 = (uint32_t)t, p0 = (uint32_t)tt;
  t = mad(r[5], K, t >> 32); tt = mad(s[5], K, tt >> 32);
  uint32_t q1 = (uint32_t)t, p1 = (uint32_t)tt;
  t = mad(r[6], K, t >> 32); tt = mad(s[6], K, tt >> 32);
  uint32_t q2 = (uint32_t)t, p2 = (uint32_t)tt;
  t = mad(r[7], K, t >> 32); tt = mad(s[7], K, tt >> 32);
  uint32_t q3 = (uint32_t)t, q4 = (uint32_t)(t >> 32), p3 = (uint32_t)tt, p4 = (uint32_t)(tt >> 32);
  uint64_t c_, e, b_, f;
  uint32_t s1 = add_co(r[1], q0, c_), S1 = add_co(s[1], p0, e);
  uint32_t x0 = sub_co(r[0], r[4], b_), X0 = sub_co(s[0], s[4], f);
  uint32_t s2 = addc_co(r[2], q1, c_, c_), S2 = addc_co(s[2], p1, e, e);
  uint32_t x1 = subb_co(s1, r[5], b_, b_), X1 = subb_co(S1, s[5], f, f);
  uint32_t s3 = addc_co(r[3], q2, c_, c_), S3 = addc_co(s[3], p2, e, e);
  uint32_t x2 = subb_co(s2, r[6], b_, b_), X2 = subb_co(S2, s[6], f, f);
  uint32_t s4 = addc_co_0(q3, c_, c_), S4 = addc_co_0(p3, e, e);
  uint32_t x3 = subb_co(s3, r[7], b_, b_), X3 = subb_co(S3, s[7], f, f);
  uint32_t s5 = addc_0(q4, c_), S5 = addc_0(p4, e);
  uint32_t x4 = subb_co_0(s4, b_, b_), X4 = subb_co_0(S4, f, f);
  uint32_t x5 = subb_0(s5, b_), X5 = subb_0(S5, f);
  uint64_t uu = mul_wide(x4, K), UU = mul_wide(X4, K);
  uint32_t u0 = (uint32_t)uu, U0 = (uint32_t)UU;
  uint32_t u1 = (uint32_t)(uu >> 32) + x5 * K, U1 = (uint32_t)(UU >> 32) + X5 * K;
  uint32_t y1 = add_co(x1, u0, c_), Y1 = add_co(X1, U0, e);
  uint32_t z0 = sub_co(x0, x4, b_), Z0 = sub_co(X0, X4, f);
  uint32_t y2 = addc_co(x2, u1, c_, c_), Y2 = addc_co(X2, U1, e, e);
  uint32_t z1 = subb_co(y1, x5, b_, b_), Z1 = subb_co(Y1, X5, f, f);
  uint32_t y3 = addc_co_0(x3, c_, c_), Y3 = addc_co_0(X3, e, e);
  uint32_t z2 = subb_co_0(y2, b_, b_), Z2 = subb_co_0(Y2, f, f);
  uint32_t z3 = subb_co_0(y3, b_, b_), Z3 = subb_co_0(Y3, f, f);
  uint64_t k1, k2;
  asm("s_andn2_b64 %0, %1, %2" : "=s"(k1) : "s"(c_), "s"(b_) : "scc");
  asm("s_andn2_b64 %0, %1, %2" : "=s"(k2) : "s"(e), "s"(f) : "scc");
  ab = canon_from(z0, z1, z2, z3, k1);
  cd = canon_from(Z0, Z1, Z2, Z3, k2);
}
__device__ __forceinline__ felt add(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t c;
  uint32_t s0 = add_co(x.w0, y.w0, c);
  uint32_t s1 = addc_co(x.w1, y.w1, c, c);
  uint32_t s2 = addc_co(x.w2, y.w2, c, c);
  uint32_t s3 = addc_co(x.w3, y.w3, c, c);
  return canon_from(s0, s1, s2, s3, c);
}
__device__ __forceinline__ felt sub(felt a, felt b) {
  L4 x = split(a), y = split(b);
  uint64_t bw;
  uint32_t d0 = sub_co(x.w0, y.w0, bw);
  uint32_t d1 = subb_co(x.w1, y.w1, bw, bw);
  uint32_t d2 = subb_co(x.w2, y.w2, bw, bw);
  uint32_t d3 = subb_co(x.w3, y.w3, bw, bw);
  uint32_t m0 = sel_0_m1(bw), m1 = sel(0u, C1, bw);
  uint64_t b2;
  uint32_t e0 = sub_co(d0, m0, b2);
  uint32_t e1 = subb_co(d1, m1, b2, b2);
  uint32_t e2 = subb_co_0(d2, b2, b2);
  uint32_t e3 = subb_0(d3, b2);
  return join(e0, e1, e2, e3);
}
}  // namespace exact
#endif

// two interleaved DIT butterflies (k_ntt8's bfly2<true>)
template <int V>
__device__ __forceinline__ void bfly2(felt& x0, felt& y0, felt w0, felt& x1, felt& y1, felt w1) {
#if defined(__HIP_DEVICE_COMPILE__)
  felt t0, t1;
  if (V == 0) {
    fpd::mul_x2(y0, w0, y1, w1, t0, t1);
    y0 = fp::sub(x0, t0); x0 = fp::add(x0, t0);
    y1 = fp::sub(x1, t1); x1 = fp::add(x1, t1);
  } else {
    exact::mul_x2(y0, w0, y1, w1, t0, t1);
    y0 = exact::sub(x0, t0); x0 = exact::add(x0, t0);
    y1 = exact::sub(x1, t1); x1 = exact::add(x1, t1);
  }
#endif
}

template <int V>
__global__ __launch_bounds__(256) void k_bfly(felt* io, const felt* tw, int iters) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  felt x[8], w[4];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = io[8 * t + i];
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = tw[(t & 1023) * 4 + i];
  for (int it = 0; it < iters; it++) {
    bfly2<V>(x[0], x[1], w[0], x[2], x[3], w[0]);
    bfly2<V>(x[4], x[5], w[0], x[6], x[7], w[0]);
    bfly2<V>(x[0], x[2], w[1], x[1], x[3], w[2]);
    bfly2<V>(x[4], x[6], w[1], x[5], x[7], w[2]);
    bfly2<V>(x[0], x[4], w[3], x[1], x[5], w[1]);
    bfly2<V>(x[2], x[6], w[2], x[3], x[7], w[0]);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) io[8 * t + i] = x[i];
}

// ------------------------------------------------------------ edge cases
// out[4i..4i+4) = a*b, a+b, a-b, a*(low word of b) for the pairs (a[i], b[i])
__global__ void k_ops(const felt* a, const felt* b, felt* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[4 * i] = fp::mul(a[i], b[i]);
  out[4 * i + 1] = fp::add(a[i], b[i]);
  out[4 * i + 2] = fp::sub(a[i], b[i]);
  out[4 * i + 3] = fp::mul_u32(a[i], (uint32_t)b[i].lo);
}
// the interleaved pair, products and butterflies (the NTT's forms)
__global__ void k_ops2(const felt* a, const felt* b, felt* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
#if defined(__HIP_DEVICE_COMPILE__)
  felt p0, p1;
  fpd::mul_x2(a[2 * i], b[2 * i], a[2 * i + 1], b[2 * i + 1], p0, p1);
  out[2 * i] = p0;
  out[2 * i + 1] = p1;
#endif
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
  return rng_state;
}
static felt rand_felt() {
  for (;;) {
    felt v = make(rnd(), rnd());
    if (!ge_p(v)) return v;
  }
}


static int run_check() {
  const felt pm1 = make(0xffffd30000000000ull, 0xffffffffffffffffull);  // p - 1
  const int n = 1 << 16;
  felt* ha = (felt*)malloc(n * sizeof(felt));
  felt* hb = (felt*)malloc(n * sizeof(felt));
  for (int i = 0; i < n; i++) {
    felt a = rand_felt(), b = rand_felt();
    switch (i % 10) {  // cases 8, 9: random pairs
      case 0: a = sub(pm1, make(rnd() & 0xff, 0)); b = make(rnd() & 0xffff, 0); break;  // sums in [p, 2^128)
      case 1: a = sub(pm1, make(rnd() & 0xff, 0)); b = sub(pm1, make(rnd() & 0xff, 0)); break;  // carry past 2^128
      case 2: {  // a*b = r with r at the top: r3 = 0xffffffff
        felt r = sub(pm1, make(rnd(), rnd() & 0xffffffffull));
        b = rand_felt();
        a = mul(r, inv(b));
        break;
      }
      case 3: {  // a*b = r < 2^128 - p (a residue whose alias r + p is < 2^128)
        felt r = make(rnd() & 0x1fffffffffffull, 0);
        b = rand_felt();
        a = mul(r, inv(b));
        break;
      }
      case 4: b = a; break;  // a - a = 0, a + a
      case 5: a = make(rnd() & 0xf, 0); break;  // small minus large: borrow
      case 6: {  // a*k at the top of the range for a 32-bit k (mul_u32)
        b = make((rnd() & 0xffffffffull) | 1, 0);
        a = mul(sub(pm1, make(rnd() & 0xffffffffffull, 0)), inv(b));
        break;
      }
      case 7: {  // a*k below 2^128 - p
        b = make((rnd() & 0xffffffffull) | 1, 0);
        a = mul(make(rnd() & 0xfffffffffull, 0), inv(b));
        break;
      }
      default: break;
    }
    ha[i] = a;
    hb[i] = b;
  }
  felt *da, *db, *dout, *dout2;
  CHECK(hipMalloc(&da, n * sizeof(felt)));
  CHECK(hipMalloc(&db, n * sizeof(felt)));
  CHECK(hipMalloc(&dout, 4 * n * sizeof(felt)));
  CHECK(hipMalloc(&dout2, n * sizeof(felt)));
  CHECK(hipMemcpy(da, ha, n * sizeof(felt), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb, n * sizeof(felt), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_ops, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dout, n);
  hipLaunchKernelGGL(k_ops2, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, da, db, dout2, n);
  CHECK(hipDeviceSynchronize());
  felt* ho = (felt*)malloc(4 * n * sizeof(felt));
  felt* ho2 = (felt*)malloc(n * sizeof(felt));
  CHECK(hipMemcpy(ho, dout, 4 * n * sizeof(felt), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(ho2, dout2, n * sizeof(felt), hipMemcpyDeviceToHost));
  int bad = 0, top = 0, alias = 0, sumtop = 0;
  for (int i = 0; i < n; i++) {
    const felt m = mul(ha[i], hb[i]), s = add(ha[i], hb[i]), d = sub(ha[i], hb[i]);
    const felt mk = mul_u32(ha[i], (uint32_t)hb[i].lo);
    if ((m.hi >> 32) == 0xffffffffull) top++;
    if (m.hi == 0 && m.lo < 0x2d0000000000ull) alias++;
    if (ha[i].hi + hb[i].hi >= ha[i].hi && (ha[i].hi >> 32) == 0xffffffffull && (hb[i].hi >> 32) == 0) sumtop++;
    if (!eq(ho[4 * i], m) || !eq(ho[4 * i + 1], s) || !eq(ho[4 * i + 2], d) || !eq(ho[4 * i + 3], mk) ||
        !eq(ho2[i], m)) {
      if (bad < 5) fprintf(stderr, "mismatch at %d (case %d)\n", i, i % 10);
      bad++;
    }
  }
  printf("edge check: %d pairs (products at the top of the range %d, below 2^128-p %d, sums near p %d): %s\n", n,
         top, alias, sumtop, bad ? "MISMATCH" : "all equal to the host's portable arithmetic");
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  if (argc > 1 && !strcmp(argv[1], "--check")) return run_check();
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // --occ W: W waves per SIMD (W blocks of 4 waves per CU) instead of a full chip
  const int occ = (argc > 2 && !strcmp(argv[1], "--occ")) ? atoi(argv[2]) : 20;
  const int tpb = 256, blocks = cus * occ, iters = occ < 20 ? 400 * 20 / occ : 400;
  if (occ != 20) printf("occupancy: %d wave(s) per SIMD\n", occ);
  const size_t nthr = (size_t)blocks * tpb;
  felt *d0, *d1, *tw;
  CHECK(hipMalloc(&d0, nthr * 8 * sizeof(felt)));
  CHECK(hipMalloc(&d1, nthr * 8 * sizeof(felt)));
  CHECK(hipMalloc(&tw, 4096 * sizeof(felt)));
  {
    felt* h = (felt*)malloc(nthr * 8 * sizeof(felt));
    for (size_t i = 0; i < nthr * 8; i++) h[i] = rand_felt();
    CHECK(hipMemcpy(d0, h, nthr * 8 * sizeof(felt), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d1, h, nthr * 8 * sizeof(felt), hipMemcpyHostToDevice));
    for (int i = 0; i < 4096; i++) h[i] = rand_felt();
    CHECK(hipMemcpy(tw, h, 4096 * sizeof(felt), hipMemcpyHostToDevice));
    free(h);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bflies = (double)nthr * iters * 12;
  double rate[2] = {0, 0};
  for (int rep = 0; rep < 2; rep++) {
    for (int v = 0; v < 2; v++) {
      felt* d = v ? d1 : d0;
      auto launch = [&] {
        if (v == 0) hipLaunchKernelGGL(k_bfly<0>, dim3(blocks), dim3(tpb), 0, 0, d, tw, iters);
        else hipLaunchKernelGGL(k_bfly<1>, dim3(blocks), dim3(tpb), 0, 0, d, tw, iters);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 3; r++) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double g = 3 * bflies / (ms * 1e-3) / 1e9;
      rate[v] = rep ? (rate[v] > g ? rate[v] : g) : g;
      printf("%-6s %-62s %9.3f ms  %7.1f Gbfly/s  (%.0f SIMD cycles per wave64 butterfly at 2.4 GHz)\n",
             v ? "exact" : "lib", v ? "round-3 forms: exact select after every product and sum"
                                   : "library forms: fpd::mul_x2 + fp::add/sub (canon_rare, add_sum)",
             ms / 3, g, (double)cus * 4 * 2.4e9 * 64 / (g * 1e9));
    }
  }
  felt* h0 = (felt*)malloc(nthr * 8 * sizeof(felt));
  felt* h1 = (felt*)malloc(nthr * 8 * sizeof(felt));
  CHECK(hipMemcpy(h0, d0, nthr * 8 * sizeof(felt), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h1, d1, nthr * 8 * sizeof(felt), hipMemcpyDeviceToHost));
  const bool same = memcmp(h0, h1, nthr * 8 * sizeof(felt)) == 0;
  printf("{\"gbfly_per_s\": %.1f, \"gbfly_per_s_exact\": %.1f, \"cus\": %d, \"values_identical\": %s}\n", rate[0],
         rate[1], cus, same ? "true" : "false");
  return same ? 0 : 1;
}
