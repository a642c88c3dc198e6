// verifier.cpp — zkp_verify: the proof check of winter-verifier 0.12
// `verify::<AIR, Blake3_256, DefaultRandomCoin, MerkleTree>(proof, pub_inputs,
// &AcceptableOptions::OptionSet(vec![options]))`, which the reference calls
// after every proof (/root/reference/src/main.rs:251-257, 430-436, 478-484),
// restated for the proof bytes zkp_prove emits.
//
// Host-only code (no HIP calls): it runs on any host that can load libzkp.so
// and shares the transcript/serialization pieces of host_stark.hpp with the
// prover, so a proof the prover emits and this check are one protocol.
// Stages, in the verifier's order:
//   1. parse (Proof::from_bytes) and check the options against the acceptable set
//   2. replay the channel: trace root -> composition coefficients -> constraint
//      root -> z -> OOD frame -> DEEP coefficients -> FRI roots/alphas -> remainder
//   3. OOD consistency: H(z) == sum_j z^(jn) H_j(z)
//   4. proof of work on the query seed, query positions
//   5. trace / constraint openings against their Merkle roots
//   6. DEEP values at the queries, FRI layer openings + folding, remainder
#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/zkp.h"
#include "host_stark.hpp"

using namespace zkh;

namespace {

struct VFail {
  int code;
};

[[noreturn]] void fail(int code) { throw VFail{code}; }

struct Reader {
  const uint8_t* p;
  size_t len, pos = 0;
  const uint8_t* take(size_t n) {
    if (n > len - pos) fail(ZKP_VERIFY_DESERIALIZATION);
    const uint8_t* r = p + pos;
    pos += n;
    return r;
  }
  uint64_t uint(int nbytes) {
    const uint8_t* b = take((size_t)nbytes);
    uint64_t v = 0;
    for (int i = nbytes - 1; i >= 0; i--) v = (v << 8) | b[i];
    return v;
  }
  // length-prefixed byte section (u32 / u16 prefix)
  Reader section(int prefix_bytes) {
    uint64_t n = uint(prefix_bytes);
    return Reader{take(n), n};
  }
  bool done() const { return pos == len; }
};

felt read_felt(const uint8_t* b) {
  felt v = from_u128_bytes(b);
  if (ge_p(v)) fail(ZKP_VERIFY_DESERIALIZATION);  // Felt::read_from rejects non-canonical bytes
  return v;
}

std::vector<felt> read_felts(const Reader& r, size_t count) {
  if (r.len != count * 16) fail(ZKP_VERIFY_DESERIALIZATION);
  std::vector<felt> out(count);
  for (size_t i = 0; i < count; i++) out[i] = read_felt(r.p + 16 * i);
  return out;
}

using Digest = std::array<uint8_t, 32>;

Digest leaf_digest(const felt* row, uint32_t cols) {
  Digest d;
  hash_elements(row, cols, d.data());
  return d;
}

Digest merge2(const uint8_t* a, const uint8_t* b) {
  Digest d;
  merge_bytes(a, b, d.data());
  return d;
}

// MerkleTree::verify_batch over the node order plan_batch() emits (leaves at
// L + i, internal nodes 1..L-1; a path holds, level by level, the siblings its
// subtree cannot compute itself).
bool verify_batch(const uint8_t root[32], uint64_t L, const std::vector<uint64_t>& idx,
                  const std::vector<Digest>& leaves, Reader pr) {
  const uint32_t depth = (uint32_t)pr.uint(1);
  const uint64_t npaths = pr.uint(1);
  if ((1ull << depth) != L || depth == 0) return false;
  std::vector<std::pair<uint64_t, Digest>> known;  // node index -> digest
  auto find = [&](uint64_t node) -> const Digest* {
    for (size_t i = known.size(); i-- > 0;)
      if (known[i].first == node) return &known[i].second;
    return nullptr;
  };
  auto leaf_of = [&](uint64_t i) -> const Digest* {
    for (size_t k = 0; k < idx.size(); k++)
      if (idx[k] == i) return &leaves[k];
    return nullptr;
  };
  for (size_t a = 0; a < idx.size(); a++) {
    if (idx[a] >= L) return false;
    for (size_t b = 0; b < a; b++)
      if (idx[a] == idx[b]) return false;
  }
  std::vector<uint64_t> norm;
  for (uint64_t i : idx) norm.push_back(i & ~1ull);
  std::sort(norm.begin(), norm.end());
  norm.erase(std::unique(norm.begin(), norm.end()), norm.end());
  if (norm.size() != npaths) return false;
  std::vector<std::vector<const uint8_t*>> paths(npaths);
  for (uint64_t i = 0; i < npaths; i++) {
    uint64_t cnt = pr.uint(1);
    const uint8_t* b = pr.take(32 * cnt);
    for (uint64_t k = 0; k < cnt; k++) paths[i].push_back(b + 32 * k);
  }
  if (!pr.done()) return false;
  std::vector<size_t> used(npaths, 0);
  auto next_sibling = [&](size_t path) -> const uint8_t* {
    if (path >= npaths || used[path] >= paths[path].size()) return nullptr;
    return paths[path][used[path]++];
  };
  std::vector<uint64_t> cur, next;
  for (size_t i = 0; i < norm.size(); i++) {
    const uint64_t a = norm[i];
    const Digest *la = leaf_of(a), *lb = leaf_of(a + 1);
    Digest parent;
    if (la && lb) {
      parent = merge2(la->data(), lb->data());
    } else if (la) {
      const uint8_t* s = next_sibling(i);
      if (!s) return false;
      parent = merge2(la->data(), s);
    } else {
      const uint8_t* s = next_sibling(i);
      if (!s) return false;
      parent = merge2(s, lb->data());
    }
    known.push_back({(L + a) >> 1, parent});
    next.push_back((L + a) >> 1);
  }
  for (uint32_t d = 1; d < depth; d++) {
    cur.swap(next);
    next.clear();
    for (size_t i = 0; i < cur.size(); i++) {
      const uint64_t node = cur[i], sib = node ^ 1;
      const Digest* nd = find(node);
      if (!nd) return false;
      Digest sd;
      if (i + 1 < cur.size() && cur[i + 1] == sib) {
        const Digest* f = find(sib);
        if (!f) return false;
        sd = *f;
        i++;
      } else {
        const uint8_t* s = next_sibling(i);
        if (!s) return false;
        memcpy(sd.data(), s, 32);
      }
      Digest parent = (node & 1) ? merge2(sd.data(), nd->data()) : merge2(nd->data(), sd.data());
      known.push_back({node >> 1, parent});
      next.push_back(node >> 1);
    }
  }
  for (size_t i = 0; i < npaths; i++)
    if (used[i] != paths[i].size()) return false;  // every sent node must be consumed
  const Digest* r = find(1);
  return r && memcmp(r->data(), root, 32) == 0;
}

felt horner(const std::vector<felt>& c, felt x) {
  felt acc = zero();
  for (size_t i = c.size(); i-- > 0;) acc = add(mul(acc, x), c[i]);
  return acc;
}

// periodic column of the MiMC AIR (cycle 64, get_round_constants(),
// src/helper.rs:404-406) at x: p(x^(n/64)) with p interpolated over <w_64>
felt periodic_at(const AirDesc& a, felt x) {
  if (!a.cycle) return zero();
  std::vector<felt> c(a.cycle);
  for (uint32_t j = 0; j < a.cycle; j++) c[j] = felt_u64((uint64_t)(j + 1) * 1000000ull);
  host_interpolate(c, one());
  return horner(c, pow_u64(x, a.n / a.cycle));
}

// Air::evaluate_transition at the OOD frame
std::vector<felt> eval_transition(const AirDesc& a, const felt* cur, const felt* nxt, felt kper) {
  std::vector<felt> out(a.num_t, zero());
  if (a.id == ZKP_AIR_MIMC) {
    felt t = add(cur[0], kper);
    felt t2 = sqr(t), t3 = mul(t2, t), t6 = sqr(t3);
    out[0] = sub(nxt[0], mul(t6, t));
  } else if (a.id == ZKP_AIR_GLOBAL_UPDATE) {
    // src/aggregation/air.rs:111-115: k*next - k*curr - update
    for (uint32_t i = 0; i < GU_D; i++) out[i] = sub(sub(mul(a.k, nxt[i]), mul(a.k, cur[i])), nxt[i + GU_D]);
  }
  // TrainingUpdate: identically zero (current_step() == 0, src/helper.rs:136-147)
  return out;
}

struct FriOpening {
  Reader values, paths;
};

int verify_impl(int air_id, const uint8_t* proof, uint64_t len, const zkp_felt* pub_elems, uint64_t n_pub,
                const zkp_proof_options* acc) {
  if (!proof || (n_pub && !pub_elems) || !acc) return ZKP_ERR_ARGUMENT;
  Reader r{proof, (size_t)len};
  // ---- 1. Context (Proof::context): trace info, field modulus, options
  const uint32_t w = (uint32_t)r.uint(1);
  r.uint(1);
  r.uint(1);
  const uint32_t logn = (uint32_t)r.uint(1);
  r.take(r.uint(2));  // trace metadata
  if (r.uint(1) != 16) return ZKP_VERIFY_INCONSISTENT_BASE_FIELD;
  felt modulus = from_u128_bytes(r.take(16));
  if (modulus.lo != P_LO || modulus.hi != P_HI) return ZKP_VERIFY_INCONSISTENT_BASE_FIELD;
  zkp_proof_options o;
  o.num_queries = (uint32_t)r.uint(1);
  o.blowup_factor = (uint32_t)r.uint(1);
  o.grinding_factor = (uint32_t)r.uint(1);
  o.field_extension = (uint32_t)r.uint(1);
  o.fri_folding_factor = (uint32_t)r.uint(1);
  o.fri_remainder_max_degree = (uint32_t)r.uint(1);
  o.batching_constraints = (uint32_t)r.uint(1);
  o.batching_deep = (uint32_t)r.uint(1);
  const uint32_t num_constraints = (uint32_t)r.uint(4);
  if (memcmp(&o, acc, sizeof o) != 0 || check_options(&o) != 0) return ZKP_VERIFY_UNACCEPTABLE_OPTIONS;
  if (logn < 3 || logn > 32) return ZKP_VERIFY_DESERIALIZATION;
  const uint64_t n = 1ull << logn;
  const uint32_t B = o.blowup_factor, F = o.fri_folding_factor;
  const uint32_t logN = logn + ilog2(B);
  if (logN > 40) return ZKP_VERIFY_DESERIALIZATION;
  const uint64_t N = 1ull << logN;
  std::vector<felt> pub(n_pub);
  for (uint64_t i = 0; i < n_pub; i++) pub[i] = make(pub_elems[i].lo, pub_elems[i].hi);
  AirDesc air;
  if (build_air(air, air_id, w, n, pub) != 0) return ZKP_VERIFY_PUB_INPUTS;
  if (num_constraints != air.num_t + air.a_col.size()) return ZKP_VERIFY_DESERIALIZATION;
  const uint32_t C = air.comp_cols();
  uint32_t L = 0;
  {
    uint64_t D = N, maxrem = (uint64_t)(o.fri_remainder_max_degree + 1) * B;
    while (D > maxrem) { D /= F; L++; }
  }
  // ---- commitments, queries, OOD frame, FRI proof, nonce
  const uint64_t num_unique = r.uint(1);
  Reader com = r.section(2);
  if (com.len != 32ull * (2 + L + 1)) return ZKP_VERIFY_DESERIALIZATION;
  const uint8_t* trace_root = com.p;
  const uint8_t* constraint_root = com.p + 32;
  const uint8_t* fri_roots = com.p + 64;
  const uint8_t* remainder_commitment = com.p + 64 + 32 * (size_t)L;
  if (r.uint(1) != 1) return ZKP_VERIFY_DESERIALIZATION;  // one trace segment
  Reader tq_vals = r.section(4), tq_paths = r.section(4);
  Reader cq_vals = r.section(4), cq_paths = r.section(4);
  Reader ood_t = r.section(2);
  if (ood_t.len != 1 + 32ull * w || ood_t.p[0] != 2) return ZKP_VERIFY_DESERIALIZATION;
  Reader ood_c = r.section(2);
  std::vector<felt> ood_trace = read_felts(Reader{ood_t.p + 1, ood_t.len - 1}, 2 * (size_t)w);
  std::vector<felt> ood_comp = read_felts(ood_c, C);
  if (r.uint(1) != L) return ZKP_VERIFY_DESERIALIZATION;
  std::vector<FriOpening> fri(L);
  for (uint32_t l = 0; l < L; l++) {
    fri[l].values = r.section(4);
    fri[l].paths = r.section(4);
  }
  Reader rem_r = r.section(2);
  if (r.uint(1) != 1) return ZKP_VERIFY_DESERIALIZATION;
  const uint64_t nonce = r.uint(8);
  r.uint(1);
  if (!r.done()) return ZKP_VERIFY_DESERIALIZATION;

  // ---- 2. channel replay
  Coin coin;
  {
    std::vector<felt> se = context_elements(air, &o);
    se.insert(se.end(), pub.begin(), pub.end());
    coin.init(se);
  }
  coin.reseed(trace_root);
  std::vector<felt> cc = draw_coeffs(coin, o.batching_constraints, num_constraints);
  coin.reseed(constraint_root);
  const felt z = coin.draw();
  const felt wn = root_of_unity(logn);

  // ---- 3. OOD consistency (DefaultConstraintEvaluator at z vs the composition columns)
  {
    std::vector<felt> ev = eval_transition(air, ood_trace.data(), ood_trace.data() + w, periodic_at(air, z));
    felt t = zero();
    for (uint32_t i = 0; i < air.num_t; i++) t = add(t, mul(cc[i], ev[i]));
    const felt zn = pow_u64(z, n);
    felt lhs = mul(mul(t, sub(z, pow_u64(wn, n - 1))), inv(sub(zn, one())));
    for (size_t i = 0; i < air.a_col.size(); i++) {
      felt num = sub(ood_trace[air.a_col[i]], air.a_val[i]);
      lhs = add(lhs, mul(mul(cc[air.num_t + i], num), inv(sub(z, pow_u64(wn, air.a_step[i])))));
    }
    felt rhs = zero(), zp = one();
    for (uint32_t j = 0; j < C; j++) {
      rhs = add(rhs, mul(zp, ood_comp[j]));
      zp = mul(zp, zn);
    }
    if (!eq(lhs, rhs)) return ZKP_VERIFY_INCONSISTENT_OOD;
  }
  uint8_t d[32];
  hash_elements(ood_trace.data(), ood_trace.size(), d);
  coin.reseed(d);
  hash_elements(ood_comp.data(), ood_comp.size(), d);
  coin.reseed(d);
  std::vector<felt> gam = draw_coeffs(coin, o.batching_deep, w + C);
  std::vector<felt> alphas(L);
  for (uint32_t l = 0; l < L; l++) {
    coin.reseed(fri_roots + 32 * (size_t)l);
    alphas[l] = coin.draw();
  }
  uint64_t Dfin = N;
  for (uint32_t l = 0; l < L; l++) Dfin /= F;
  std::vector<felt> remainder = read_felts(rem_r, Dfin / B);
  hash_elements(remainder.data(), remainder.size(), d);
  if (memcmp(d, remainder_commitment, 32) != 0) return ZKP_VERIFY_FRI;
  coin.reseed(d);

  // ---- 4. proof of work + query positions
  {
    if (coin.leading_zeros(nonce) < o.grinding_factor) return ZKP_VERIFY_POW;
  }
  std::vector<uint64_t> pos = coin.draw_integers(o.num_queries, N, nonce);
  std::sort(pos.begin(), pos.end());
  pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
  if (pos.size() != num_unique) return ZKP_VERIFY_DESERIALIZATION;
  const size_t np = pos.size();

  // ---- 5. trace / constraint openings
  std::vector<felt> tv = read_felts(tq_vals, np * w), cv = read_felts(cq_vals, np * C);
  {
    std::vector<Digest> lt(np), lc(np);
    for (size_t i = 0; i < np; i++) {
      lt[i] = leaf_digest(tv.data() + i * w, w);
      lc[i] = leaf_digest(cv.data() + i * C, C);
    }
    if (!verify_batch(trace_root, N, pos, lt, tq_paths)) return ZKP_VERIFY_TRACE_QUERY;
    if (!verify_batch(constraint_root, N, pos, lc, cq_paths)) return ZKP_VERIFY_CONSTRAINT_QUERY;
  }

  // ---- 6. DEEP composition at the queries, then FRI
  const felt g = felt_u64(3), zg = mul(z, wn), gN = root_of_unity(logN);
  std::vector<felt> evals(np);
  for (size_t i = 0; i < np; i++) {
    const felt x = mul(g, pow_u64(gN, pos[i]));
    felt a1 = zero(), a2 = zero();
    for (uint32_t c = 0; c < w; c++) {
      const felt t = tv[i * w + c];
      a1 = add(a1, mul(gam[c], sub(t, ood_trace[c])));
      a2 = add(a2, mul(gam[c], sub(t, ood_trace[w + c])));
    }
    for (uint32_t j = 0; j < C; j++) a1 = add(a1, mul(gam[w + j], sub(cv[i * C + j], ood_comp[j])));
    evals[i] = add(mul(a1, inv(sub(x, z))), mul(a2, inv(sub(x, zg))));
  }
  std::vector<uint64_t> cur = pos;
  uint64_t D = N;
  felt off = g;
  const felt w16inv = inv(root_of_unity(ilog2(F))), finv = inv(felt_u64(F));
  for (uint32_t l = 0; l < L; l++) {
    const uint64_t Rows = D / F;
    std::vector<uint64_t> nxt = fold_positions(cur, Rows);
    std::vector<felt> vals = read_felts(fri[l].values, nxt.size() * F);
    std::vector<Digest> leaves(nxt.size());
    for (size_t i = 0; i < nxt.size(); i++) leaves[i] = leaf_digest(vals.data() + i * F, F);
    if (!verify_batch(fri_roots + 32 * (size_t)l, Rows, nxt, leaves, fri[l].paths)) return ZKP_VERIFY_FRI;
    // the opened rows must hold the previous layer's values at the previous positions
    for (size_t i = 0; i < cur.size(); i++) {
      const uint64_t row = cur[i] % Rows, k = cur[i] / Rows;
      size_t slot = std::find(nxt.begin(), nxt.end(), row) - nxt.begin();
      if (!eq(vals[slot * F + k], evals[i])) return ZKP_VERIFY_FRI;
    }
    // fold each row: the degree-<F polynomial through (x_r * w_F^k, v_k), evaluated at alpha
    const felt gD = root_of_unity(ilog2(D));
    std::vector<felt> folded(nxt.size());
    for (size_t i = 0; i < nxt.size(); i++) {
      const felt xr = mul(off, pow_u64(gD, nxt[i]));
      std::vector<felt> row(vals.begin() + i * F, vals.begin() + (i + 1) * F);
      host_ntt(row, w16inv);  // iDFT (unscaled)
      const felt beta = mul(alphas[l], inv(xr));
      folded[i] = mul(horner(row, beta), finv);
    }
    evals.swap(folded);
    cur.swap(nxt);
    D = Rows;
    off = pow_u64(off, F);
  }
  const felt gD = root_of_unity(ilog2(D));
  for (size_t i = 0; i < cur.size(); i++) {
    const felt x = mul(off, pow_u64(gD, cur[i]));
    if (!eq(horner(remainder, x), evals[i])) return ZKP_VERIFY_FRI;
  }
  return ZKP_OK;
}

}  // namespace

extern "C" int zkp_verify(zkp_air_id air, const uint8_t* proof, uint64_t proof_len, const zkp_felt* pub_elems,
                          uint64_t n_pub, const zkp_proof_options* acceptable) {
  try {
    return verify_impl((int)air, proof, proof_len, pub_elems, n_pub, acceptable);
  } catch (const VFail& f) {
    return f.code;
  } catch (const ZkpFail&) {
    return ZKP_VERIFY_RANDOM_COIN;  // the coin failed to draw a field element
  } catch (...) {
    return ZKP_VERIFY_DESERIALIZATION;
  }
}
