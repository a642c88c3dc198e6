// host_stark.hpp — host-side STARK protocol pieces shared by the prover
// (prover.cpp) and the verifier (verifier.cpp): field helpers, the Fiat-Shamir
// transcript (winter-crypto DefaultRandomCoin<Blake3_256>), composition
// coefficient draws, proof serialization primitives, AIR metadata for the
// AIR ids of include/zkp.h, winterfell `Context` elements and the Merkle
// batch-opening plan. Pure host code: no HIP calls.
#pragma once
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/zkp.h"
#include "blake3.hpp"
#include "felt.hpp"

namespace zkh {
using namespace fp;

struct ZkpFail {
  int code;
  std::string msg;
};


// ------------------------------------------------------------------ field helpers
inline uint32_t ilog2(uint64_t v) {
  uint32_t l = 0;
  while ((1ull << l) < v) l++;
  return l;
}
inline uint64_t revb(uint64_t x, uint32_t bits) {
  uint64_t r = 0;
  for (uint32_t i = 0; i < bits; i++) r |= ((x >> i) & 1ull) << (bits - 1 - i);
  return r;
}
inline felt two_adic_root() { return make(0x86b8723e1920f4aaULL, 0x120532e7b364080aULL); }
inline felt root_of_unity(uint32_t log_n) {
  felt r = two_adic_root();
  for (uint32_t i = log_n; i < 40; i++) r = sqr(r);
  return r;
}
inline felt felt_u64(uint64_t v) { return make(v, 0); }

// natural-order radix-2 NTT on the host (only for tiny arrays: remainder, periodic column)
inline void host_ntt(std::vector<felt>& a, felt root) {
  size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    felt wl = pow_u64(root, n / len);
    for (size_t i = 0; i < n; i += len) {
      felt w = one();
      for (size_t k = 0; k < len / 2; k++) {
        felt u = a[i + k], v = mul(a[i + k + len / 2], w);
        a[i + k] = add(u, v);
        a[i + k + len / 2] = sub(u, v);
        w = mul(w, wl);
      }
    }
  }
}
// fft::interpolate_poly_with_offset
inline void host_interpolate(std::vector<felt>& v, felt offset) {
  size_t n = v.size();
  host_ntt(v, inv(root_of_unity(ilog2(n))));
  felt s = inv(felt_u64(n)), oi = inv(offset);
  for (size_t k = 0; k < n; k++) { v[k] = mul(v[k], s); s = mul(s, oi); }
}
// fft::evaluate_poly_with_offset (coefficients zero-padded to N)
inline std::vector<felt> host_evaluate(const std::vector<felt>& c, size_t N, felt offset) {
  std::vector<felt> out(N, zero());
  felt s = one();
  for (size_t k = 0; k < c.size(); k++) { out[k] = mul(c[k], s); s = mul(s, offset); }
  host_ntt(out, root_of_unity(ilog2(N)));
  return out;
}

// ------------------------------------------------------------------ transcript
inline void hash_elements(const felt* e, size_t n, uint8_t out[32]) {
  std::vector<uint8_t> buf(n * 16);
  for (size_t i = 0; i < n; i++) to_bytes(e[i], buf.data() + 16 * i);
  b3::host_hash(buf.data(), buf.size(), out);
}
inline void merge_bytes(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  uint8_t buf[64];
  memcpy(buf, a, 32);
  memcpy(buf + 32, b, 32);
  b3::host_hash(buf, 64, out);
}
inline void merge_with_int(const uint8_t s[32], uint64_t v, uint8_t out[32]) {
  uint8_t buf[40];
  memcpy(buf, s, 32);
  for (int i = 0; i < 8; i++) buf[32 + i] = (uint8_t)(v >> (8 * i));
  b3::host_hash(buf, 40, out);
}

// winter-crypto DefaultRandomCoin<Blake3_256>
struct Coin {
  uint8_t seed[32];
  uint64_t counter = 0;
  void init(const std::vector<felt>& els) { hash_elements(els.data(), els.size(), seed); counter = 0; }
  void reseed(const uint8_t d[32]) {
    uint8_t s[32];
    merge_bytes(seed, d, s);
    memcpy(seed, s, 32);
    counter = 0;
  }
  void next(uint8_t out[32]) { counter++; merge_with_int(seed, counter, out); }
  felt draw() {
    for (int i = 0; i < 1000; i++) {
      uint8_t v[32];
      next(v);
      felt x = from_u128_bytes(v);
      if (!ge_p(x)) return x;
    }
    throw ZkpFail{ZKP_ERR_ARGUMENT, "failed to draw a field element"};
  }
  // check_leading_zeros: trailing zeros of u64_le(merge_with_int(seed, nonce)[..8])
  uint32_t leading_zeros(uint64_t nonce) const {
    uint8_t v[32];
    merge_with_int(seed, nonce, v);
    uint64_t h = 0;
    for (int b = 7; b >= 0; b--) h = (h << 8) | v[b];
    return h == 0 ? 64u : (uint32_t)__builtin_ctzll(h);
  }
  std::vector<uint64_t> draw_integers(uint32_t k, uint64_t domain, uint64_t nonce) {
    uint8_t s[32];
    merge_with_int(seed, nonce, s);
    memcpy(seed, s, 32);
    counter = 0;
    std::vector<uint64_t> out(k);
    for (uint32_t i = 0; i < k; i++) {
      uint8_t v[32];
      next(v);
      uint64_t x = 0;
      for (int b = 7; b >= 0; b--) x = (x << 8) | v[b];
      out[i] = x & (domain - 1);
    }
    return out;
  }
};

// ConstraintCompositionCoefficients / DeepCompositionCoefficients
inline std::vector<felt> draw_coeffs(Coin& c, uint32_t method, uint32_t n) {
  std::vector<felt> out(n);
  if (method == ZKP_BATCHING_LINEAR) {
    for (uint32_t i = 0; i < n; i++) out[i] = c.draw();
    return out;
  }
  felt alpha = c.draw(), acc = one();
  for (uint32_t i = 0; i < n; i++) {
    out[method == ZKP_BATCHING_HORNER ? n - 1 - i : i] = acc;
    acc = mul(acc, alpha);
  }
  return out;
}

// ------------------------------------------------------------------ serialization
struct Writer {
  std::vector<uint8_t> b;
  void put(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  void u8(uint8_t v) { b.push_back(v); }
  void u16(uint16_t v) { u8((uint8_t)v); u8((uint8_t)(v >> 8)); }
  void u32(uint32_t v) { for (int i = 0; i < 4; i++) u8((uint8_t)(v >> (8 * i))); }
  void u64(uint64_t v) { for (int i = 0; i < 8; i++) u8((uint8_t)(v >> (8 * i))); }
  void fe(felt v) { uint8_t t[16]; to_bytes(v, t); put(t, 16); }
};

// ------------------------------------------------------------------ AIR metadata
constexpr uint32_t GU_D = 60;  // AC*FE + AC (src/helper.rs:18-20)
constexpr uint32_t TU_W = 240;  // 4*(AC*FE + AC), src/training/prover.rs:98-103
constexpr uint32_t TU_AC = 6, TU_FE = 9;

struct AirDesc {
  int id;
  uint32_t w;
  uint64_t n;
  uint32_t num_t, base_degree, cycle;
  std::vector<uint32_t> a_col;
  std::vector<uint64_t> a_step;
  std::vector<felt> a_val;
  felt k;
  uint32_t ce_blowup() const {
    uint32_t v = base_degree - 1, p = 1;
    while (p < v) p <<= 1;
    return p < 2 ? 2 : p;
  }
  uint32_t comp_cols() const {
    uint64_t hi = (uint64_t)base_degree * (n - 1), div = n - 1;
    uint64_t c = (hi - div + n - 1) / n;
    return c < 1 ? 1 : (uint32_t)c;
  }
};

inline int build_air(AirDesc& a, int id, uint32_t w, uint64_t n, const std::vector<felt>& pub) {
  a.id = id;
  a.w = w;
  a.n = n;
  if (id == ZKP_AIR_MIMC) {
    // builder-defined MiMC AIR, round constants src/helper.rs:404-406
    if (w != 1 || n < 64 || pub.size() != 2) return ZKP_ERR_PUB_INPUTS;
    a.num_t = 1;
    a.base_degree = 7;
    a.cycle = 64;
    a.a_col = {0, 0};
    a.a_step = {0, n - 1};
    a.a_val = {pub[0], pub[1]};
    return 0;
  }
  if (id == ZKP_AIR_GLOBAL_UPDATE) {
    // src/aggregation/air.rs:93-147
    if (w != 2 * GU_D || pub.size() != 123) return ZKP_ERR_PUB_INPUTS;
    if (pub[122].hi != 0 || pub[122].lo == 0 || pub[122].lo > n) return ZKP_ERR_PUB_INPUTS;
    uint64_t steps = pub[122].lo;
    a.num_t = GU_D;
    a.base_degree = 1;
    a.cycle = 0;
    a.k = pub[120];
    for (uint32_t i = 0; i < 2 * GU_D; i++) {
      a.a_col.push_back(i);
      a.a_step.push_back(steps - 1);
      a.a_val.push_back(i < GU_D ? pub[60 + i] : zero());
    }
    return 0;
  }
  if (id == ZKP_AIR_TRAINING_UPDATE) {
    // src/training/air.rs:101-151; public inputs (to_elements :74-98): initial (w/2) || final (w/2) ||
    // f64(steps) || f64(bs) || x_batch (bs*FE) || y_batch (bs*AC) || lr || precision
    if (w != TU_W || pub.size() < TU_W + 4) return ZKP_ERR_PUB_INPUTS;
    felt bsf = pub[TU_W + 1];
    if (bsf.hi != 0 || bsf.lo % 1000000ull) return ZKP_ERR_PUB_INPUTS;
    uint64_t bs = bsf.lo / 1000000ull;
    if (pub.size() != (uint64_t)TU_W + 4 + bs * (TU_FE + TU_AC)) return ZKP_ERR_PUB_INPUTS;
    const uint32_t half = TU_W / 2;
    a.num_t = TU_W;  // all degree 1, all identically zero (current_step() == 0)
    a.base_degree = 1;
    a.cycle = 0;
    a.a_col.resize(2 * half);
    a.a_step.resize(2 * half);
    a.a_val.resize(2 * half);
    for (uint32_t i = 0; i < half; i++) {  // air.rs:140-147
      a.a_col[i] = i; a.a_step[i] = 0; a.a_val[i] = pub[i];
      a.a_col[half + i] = i; a.a_step[half + i] = n - 1; a.a_val[half + i] = pub[half + i];
    }
    return 0;
  }
  return ZKP_ERR_UNSUPPORTED_AIR;
}

inline int check_options(const zkp_proof_options* o) {
  if (!o) return ZKP_ERR_ARGUMENT;
  if (o->field_extension != ZKP_FIELD_EXTENSION_NONE) return ZKP_ERR_UNSUPPORTED_FIELD_EXTENSION;
  if (o->num_queries == 0 || o->num_queries > 255) return ZKP_ERR_INVALID_OPTIONS;
  uint32_t b = o->blowup_factor;
  if (b < 2 || b > 128 || (b & (b - 1))) return ZKP_ERR_INVALID_OPTIONS;
  if (o->grinding_factor > 32) return ZKP_ERR_INVALID_OPTIONS;
  if (o->fri_folding_factor != 16) return ZKP_ERR_INVALID_OPTIONS;  // the reference's value; only 16 is built
  uint32_t r = o->fri_remainder_max_degree;
  if (r > 255 || ((r + 1) & r)) return ZKP_ERR_INVALID_OPTIONS;
  if (o->batching_constraints > 2 || o->batching_deep > 2) return ZKP_ERR_INVALID_OPTIONS;
  return 0;
}

// Context::to_elements
inline std::vector<felt> context_elements(const AirDesc& a, const zkp_proof_options* o) {
  std::vector<felt> e;
  e.push_back(felt_u64((uint64_t)a.w << 16));
  e.push_back(felt_u64((uint32_t)a.n));
  e.push_back(felt_u64(0xffffd30000000001ULL));
  e.push_back(felt_u64(0xffffffffffffffffULL));
  e.push_back(felt_u64(a.num_t + a.a_col.size()));
  uint32_t buf = o->field_extension;
  buf = (buf << 8) | o->fri_folding_factor;
  buf = (buf << 8) | o->fri_remainder_max_degree;
  buf = (buf << 8) | o->blowup_factor;
  e.push_back(felt_u64(buf));
  e.push_back(felt_u64(o->grinding_factor));
  e.push_back(felt_u64(o->num_queries));
  return e;
}

inline void write_context(Writer& w, const AirDesc& a, const zkp_proof_options* o) {
  w.u8((uint8_t)a.w); w.u8(0); w.u8(0); w.u8((uint8_t)ilog2(a.n)); w.u16(0);
  w.u8(16); w.fe(make(P_LO, P_HI));
  w.u8((uint8_t)o->num_queries); w.u8((uint8_t)o->blowup_factor); w.u8((uint8_t)o->grinding_factor);
  w.u8((uint8_t)o->field_extension); w.u8((uint8_t)o->fri_folding_factor); w.u8((uint8_t)o->fri_remainder_max_degree);
  w.u8((uint8_t)o->batching_constraints); w.u8((uint8_t)o->batching_deep);
  w.u32((uint32_t)(a.num_t + a.a_col.size()));
}

// MerkleTree::prove_batch plan: emission order of (path slot, node index).
// Node numbering: leaves at L + i, internal nodes 1..L-1 (same as the device tree).
struct BatchPlan {
  uint32_t depth;
  std::vector<std::vector<uint64_t>> paths;  // node indices per path
};
inline BatchPlan plan_batch(uint64_t L, const std::vector<uint64_t>& idx) {
  BatchPlan bp;
  bp.depth = ilog2(L);
  std::vector<uint64_t> sorted_idx(idx);
  std::sort(sorted_idx.begin(), sorted_idx.end());
  std::vector<uint64_t> norm;
  norm.reserve(idx.size());
  for (uint64_t i : sorted_idx) norm.push_back(i & ~1ull);
  norm.erase(std::unique(norm.begin(), norm.end()), norm.end());
  auto has = [&](uint64_t v) { return std::binary_search(sorted_idx.begin(), sorted_idx.end(), v); };
  bp.paths.resize(norm.size());
  for (auto& p : bp.paths) p.reserve(bp.depth);
  std::vector<uint64_t> next, cur;
  next.reserve(norm.size());
  cur.reserve(norm.size());
  for (size_t i = 0; i < norm.size(); i++) {
    uint64_t a = norm[i];
    bool ha = has(a), hb = has(a + 1);
    if (ha && !hb) bp.paths[i].push_back(L + a + 1);
    else if (!ha) bp.paths[i].push_back(L + a);
    next.push_back((a + L) >> 1);
  }
  for (uint32_t d = 1; d < bp.depth; d++) {
    cur.swap(next);
    next.clear();
    for (size_t i = 0; i < cur.size(); i++) {
      uint64_t node = cur[i], sib = node ^ 1;
      if (i + 1 < cur.size() && cur[i + 1] == sib) i++;
      else bp.paths[i].push_back(sib);
      next.push_back(sib >> 1);
    }
  }
  return bp;
}

inline std::vector<uint64_t> fold_positions(const std::vector<uint64_t>& pos, uint64_t target) {
  std::vector<uint64_t> out;
  for (uint64_t p : pos) {
    uint64_t q = p % target;
    if (std::find(out.begin(), out.end(), q) == out.end()) out.push_back(q);
  }
  return out;
}


}  // namespace zkh
