// eval_check.cpp — k_eval_mimc's exact recomputation (TEST ONLY; run by
// tests/test_gpu_ntt.py). The MiMC constraint evaluator takes every product and sum
// as canonical and recomputes a point with the exact forms when a lane of its wave
// saw a carry past 2^128 or a top limb 0xffffffff (kernels.hip).
// Random data reaches that branch about once per 2^32 operations, so no proof takes
// it; here the inputs put p - 1 and values of [2^128 - 2^96, p) into the sums and
// products of every wave (dense), of one lane in 97 (sparse), and into the domain
// point x, and every output is compared with the host's portable arithmetic of the
// same formula. kernels.hip is built with ZKP_COUNT_REDO, which counts the waves
// that took the exact pass: the run fails unless that count is > 0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../zk_stark_project_amd/csrc/zkp_internal.hpp"
#include "../../zk_stark_project_amd/csrc/host_stark.hpp"

using namespace fp;
using namespace zkh;

void launch_fail(int code, const char* what) { throw std::runtime_error(std::string(what) + " " + std::to_string(code)); }
unsigned long long zkp_redo_waves_take();  // kernels.hip (ZKP_COUNT_REDO)

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(2);                                                \
    }                                                         \
  } while (0)

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return rs;
}
static felt rand_felt() {
  for (;;) {
    felt v = make(rnd(), rnd());
    if (!ge_p(v)) return v;
  }
}
static const felt PM1 = make(0xffffd30000000000ull, 0xffffffffffffffffull);  // p - 1
// a canonical value whose top limb is 0xffffffff: [2^128 - 2^96, p)
static felt top_felt() { return make(rnd() % 0xffffd30000000000ull, 0xffffffff00000000ull | (rnd() & 0xffffffffull)); }
static felt small_felt() { return make(rnd() & 0xffffffull, 0); }

template <typename T>
static T* up(const std::vector<T>& h) {
  T* d;
  CK(hipMalloc(&d, h.size() * sizeof(T) + 16));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main() {
  setvbuf(stdout, NULL, _IONBF, 0);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Prof pf;
  const uint32_t logn = 12, logce = 3, logB = 3, ce = 1u << logce;
  const uint64_t n = 1ull << logn, M = (uint64_t)ce * n;
  int bad = 0, cases = 0;
  unsigned long long redo_total = 0;
  (void)zkp_redo_waves_take();
  for (int pattern = 0; pattern < 5; pattern++) {
    // inputs: lde rows (coset-major, CE coset u = LDE coset u), the periodic column on
    // the CE domain, 1/Z_T per CE coset, the boundary divisor inverses, the regrouped
    // boundary constants, the domain offsets and the w_n table
    std::vector<felt> lde(M), kper(64 * (size_t)ce), zinv(ce), dinv(M), bc(4), cx(ce), twn(n / 2);
    for (auto& v : lde) v = rand_felt();
    for (auto& v : kper) v = rand_felt();
    for (auto& v : zinv) v = rand_felt();
    for (auto& v : dinv) v = rand_felt();
    for (auto& v : bc) v = rand_felt();
    for (auto& v : cx) v = rand_felt();
    for (auto& v : twn) v = rand_felt();
    if (pattern == 1) {  // dense: cur = p - 1 with a small K, so x + K lands in [p, 2^128) in every lane
      for (auto& v : lde) v = PM1;
      for (auto& v : kper) v = small_felt();
    }
    if (pattern == 2) {  // sparse: one lane in 97
      for (auto& v : kper) v = small_felt();
      for (uint64_t q = 0; q < M; q++)
        if (q % 97 == 5) lde[q] = PM1;
    }
    if (pattern == 3) {  // x = +-(p - 1): the domain point's products and (x - w_last) at the top of the range
      for (auto& v : cx) v = PM1;
      for (auto& v : twn) v = one();
    }
    if (pattern == 4) {  // operands with a top limb 0xffffffff everywhere
      for (auto& v : lde) v = top_felt();
      for (auto& v : dinv) v = top_felt();
      for (auto& v : bc) v = top_felt();
    }
    const felt w_last = pattern == 3 ? PM1 : rand_felt();
    felt *dl = up(lde), *dk = up(kper), *dz = up(zinv), *dd = up(dinv), *db = up(bc), *dc = up(cx), *dt = up(twn);
    felt* dout;
    CK(hipMalloc(&dout, M * 16));
    EvalCommon c{};
    c.logn = logn; c.logB = logB; c.logce = logce; c.logN = logn + logB;
    c.u0 = 0; c.cel = ce; c.j0 = 0; c.logBl = logB;
    c.g = make(3, 0);
    c.w_last = w_last;
    c.pm = PointMap{dc, dt, logn};
    c.zinv = dz;
    MimcEvalArgs a{};
    a.bcoef = db; a.kper = dk; a.binv = nullptr; a.dinv = dd; a.binv_ready = true;
    launch_eval_mimc(pf, st, c, a, dl, dout);
    CK(hipStreamSynchronize(st));
    std::vector<felt> got(M);
    CK(hipMemcpy(got.data(), dout, M * 16, hipMemcpyDeviceToHost));
    const unsigned long long redo = zkp_redo_waves_take();
    redo_total += redo;
    // the same formula with the host's exact arithmetic
    uint64_t mism = 0;
    const uint64_t kmask = (64ull << logce) - 1;
    for (uint64_t q = 0; q < M; q++) {
      const uint32_t u = (uint32_t)(q >> logn);
      const uint64_t t = q & (n - 1);
      const uint64_t s = u + (t << logce);
      const felt cur = lde[(uint64_t)u * n + t], nxt = lde[(uint64_t)u * n + ((t + 1) & (n - 1))];
      const felt tw = t < n / 2 ? twn[t] : neg(twn[t - n / 2]);
      const felt x = mul(cx[u], tw);
      const felt uu = add(cur, kper[s & kmask]);
      const felt u2 = mul(uu, uu), u3 = mul(u2, uu), u6 = mul(u3, u3), u7 = mul(u6, uu);
      const felt tpart = mul(mul(sub(nxt, u7), sub(x, w_last)), zinv[u]);
      const felt bnum = add(sub(mul(cur, sub(mul(x, bc[0]), bc[1])), mul(x, bc[2])), bc[3]);
      const felt want = add(tpart, mul(bnum, dinv[q]));
      if (!eq(want, got[q])) mism++;
    }
    cases++;
    if (mism) bad++;
    printf("pattern %d: %llu of %llu points mismatching, %llu waves took the exact pass\n", pattern,
           (unsigned long long)mism, (unsigned long long)M, redo);
    for (felt* p : {dl, dk, dz, dd, db, dc, dt, dout}) CK(hipFree(p));
  }
  printf("k_eval_mimc: %d cases, %d mismatching, %llu redo waves\n", cases, bad, redo_total);
  return (bad || redo_total == 0) ? 1 : 0;
}
