// prover_stages.cpp — the stage helpers of a proof (prover_internal.hpp): row
// commitments, the OOD evaluation, constraint evaluation, the composition constants,
// DEEP, and the query openings. World-1 paths; the sharded parts of the commitment
// and the OOD are in prover_shard.cpp.
#include "prover_internal.hpp"

using namespace zkpi;

namespace zkpi {

// commit the rows of a coset-major source held by this rank (cosets [j0, j0+Bl)):
// mode 0 = LDE rows (cols columns, n rows per coset), mode 1 = FRI rows (16
// values, 2^logrows rows per coset). Unsharded sources hold all B cosets.
// Unsharded trees finish in the last block of their top launch (MerkleTail);
// sharded trees in k_shard_top over the all-gathered subtree roots. With coin
// (coefficients, z or a FRI layer's alpha) that block also runs the coin step,
// and the function returns true when it did.
bool commit_rows(zkp_ctx* ctx, zkp_comm* cm, int mode, const felt* src, uint64_t n, uint32_t cols, uint32_t logB,
                 uint32_t logrows, bool sharded, const std::string& name, TreeShard& tr, uint8_t root[32],
                 bool fetch_root, const MerkleTail* coin, const LastCol* lc, const GuLazy* gl) {
  Prof& pf = ctx->prof;
  hipStream_t st = ctx->stream;
  const uint64_t L = 1ull << (logB + logrows);
  if (!sharded) {
    tr.logR = 0;
    tr.Lr = L;
    tr.nodes = ctx->buf<uint32_t>(name, (size_t)16 * L);
    uint32_t* done = ctx->buf<uint32_t>("merkle_done", 1);
    if (!ctx->have_cached("merkle_done")) HIP_CHECK(hipMemsetAsync(done, 0, 4, st));
    MerkleTail tail = coin ? *coin : MerkleTail{};
    tail.done = done;
    bool ran = mode == 0 ? launch_merkle_lde(pf, st, src, cols, logB, n, tr.nodes, L, &tail, lc, gl)
                         : launch_merkle_fri(pf, st, src, 1ull << logrows, logB, 16, tr.nodes, &tail);
    tr.top.assign(2, {});
    if (fetch_root) {  // otherwise the caller reads nodes[1] later
      ctx->download(root, tr.nodes + 8, 32);
      memcpy(tr.top[1].data(), root, 32);
    }
    return ran && coin;
  }
  return commit_rows_sharded(ctx, cm, mode, src, n, cols, logB, logrows, name, tr, root, fetch_root, coin, lc, gl);
}

// device -> host copies of one round trip (one sync)
void fetch_all(zkp_ctx* ctx, const std::vector<Fetch>& fs) {
  size_t tot = 0;
  for (const Fetch& f : fs) tot += (f.bytes + 15) & ~(size_t)15;
  uint8_t* hp = (uint8_t*)ctx->pinned(tot + 16);
  uint8_t* stage = ctx->buf<uint8_t>("fetch_stage", tot + 16);
  // pack the segments on the device (k_pack, PACK_MAX per launch), then one D2H copy
  size_t o = 0;
  PackArgs pa{};
  auto flush = [&] {
    if (pa.n) launch_pack(ctx->prof, ctx->stream, pa, stage);
    pa.n = 0;
  };
  for (const Fetch& f : fs) {
    if (f.bytes % 4) throw ZkpFail{ZKP_ERR_ARGUMENT, "fetch of a non-word-sized segment"};
    if (f.bytes) {
      pa.src[pa.n] = f.dev;
      pa.bytes[pa.n] = f.bytes;
      pa.off[pa.n] = o;
      if (++pa.n == PACK_MAX) flush();
    }
    o += (f.bytes + 15) & ~(size_t)15;
  }
  flush();
  HIP_CHECK(hipMemcpyAsync(hp, stage, tot, hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  o = 0;
  for (const Fetch& f : fs) {
    memcpy(f.host, hp + o, f.bytes);
    o += (f.bytes + 15) & ~(size_t)15;
  }
}

// OOD values of bit-reversed arrays at the two points whose power tables
// dpw[0..logn) / dpw[logn..2logn) are in device memory; returns the device
// array ood[2a + {0,1}] (array a at the two points; arrays a >= ntwo at the
// first point only, their second entry is zero)
// Sharded (cm world R > 1, at least R blocks of 2048 coefficients): each rank
// evaluates 1/R of every array's blocks (the partial Horner sums of SURVEY
// §8(e)(4)), the rank blocks are all-gathered (narrays * nb * 32 bytes in all)
// and every rank combines them: the same values as one rank evaluating it all.
felt* ood_launch(zkp_ctx* ctx, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn,
                 const felt* dpw, zkp_comm* cm) {
  uint32_t logE = logn < 11 ? logn : 11;
  if (logn - logE > 12) throw ZkpFail{ZKP_ERR_TRACE_SHAPE, "OOD evaluation supports n <= 2^23"};
  const uint32_t nb = 1u << (logn - logE);
  felt* part = ctx->buf<felt>("ood_part", (size_t)2 * narrays * nb);
  felt* dv = ctx->buf<felt>("ood_vals", (size_t)2 * narrays);
  const felt ninv = inv(felt_u64(1ull << logn));
  const uint32_t R = cm ? (uint32_t)cm->world : 1u;
  if (R == 1 || nb < R) {
    launch_eval_bitrev(ctx->prof, ctx->stream, arrays, narrays, ntwo, logn, dpw, dpw + logn, part, ninv, dv);
    return dv;
  }
  return ood_launch_sharded(ctx, arrays, narrays, ntwo, logn, dpw, cm, part, dv);
}

// Domain points of every LDE coset j (g*w_N^j, entries [0, B)) and CE coset u
// (g*w_M^u, entries [B, B+ce)); domain-only, cached per (n, B, ce).
felt* coset_points(zkp_ctx* ctx, uint32_t logn, uint32_t logB, uint32_t logce) {
  const uint32_t B = 1u << logB, ce = 1u << logce;
  const std::string cxkey = "coset_x_" + std::to_string(logn) + "_" + std::to_string(logB) + "_" +
                            std::to_string(logce);
  felt* cx = ctx->buf<felt>(cxkey, B + ce);
  if (!ctx->have_cached(cxkey)) {
    std::vector<felt> h(B + ce);
    const felt g = felt_u64(3);
    felt wN = root_of_unity(logn + logB), wM = root_of_unity(logn + logce);
    for (uint32_t j = 0; j < B; j++) h[j] = mul(g, pow_u64(wN, j));
    for (uint32_t u = 0; u < ce; u++) h[B + u] = mul(g, pow_u64(wM, u));
    ctx->upload(cx, h.data(), h.size() * 16);
  }
  return cx;
}

// DefaultConstraintEvaluator::evaluate over the CE cosets [u0, u0 + cel) held by
// this rank (its LDE cosets are [j0, j0 + 2^logBl)): composition evaluations
// comp[ul * n + t] = H(g * w_M^(u0+ul) * w_n^t), i.e. CE domain index (u0+ul) + ce*t.
// dt_cc = the composition coefficients (device; transition then boundary).
// Linear AIRs (GlobalUpdate, TrainingUpdate) evaluate in coefficient form when
// `coef` (the trace coefficient columns) is given (k_lin_lincomb): sharded, every
// rank of `cm` combines 1/R of the positions and the combined columns are
// all-gathered, so every rank calls this, with or without CE cosets (cel = 0).
// ZKP_EVAL_POINTWISE=1 (A/B switch) keeps k_eval_linear over the trace LDE.
void constraint_eval(zkp_ctx* ctx, const AirDesc& air, uint32_t logn, uint32_t logB, uint32_t logce, uint32_t u0,
                     uint32_t cel, uint32_t j0, uint32_t logBl, const felt* cx, const felt* twn, const felt* dt_cc,
                     const felt* dt_aval, const felt* tlde, felt* comp, const felt* coef, zkp_comm* cm) {
  Prof& pf = ctx->prof;
  hipStream_t st = ctx->stream;
  const uint32_t B = 1u << logB, ce = 1u << logce, logN = logn + logB, w = air.w;
  const uint64_t n = 1ull << logn;
  const felt g = felt_u64(3);
  felt wn = root_of_unity(logn);
  EvalCommon ec;
  ec.logn = logn; ec.logB = logB; ec.logce = logce; ec.logN = logN;
  ec.u0 = u0; ec.cel = cel; ec.j0 = j0; ec.logBl = logBl;
  ec.g = g;
  ec.w_last = pow_u64(wn, n - 1);
  ec.pm = PointMap{cx + B + u0, twn, logn};
  // 1/(x^n - 1) on the CE domain: x^n = g^n * w_ce^s (domain-only: cached per (n, ce))
  const std::string zkey = "zinv_" + std::to_string(logn) + "_" + std::to_string(logce);
  std::vector<felt>& zinv = ctx->host_cache[zkey];
  if (zinv.empty()) {
    zinv.resize(ce);
    felt gn = pow_u64(g, n), wce = root_of_unity(logce);
    for (uint32_t s = 0; s < ce; s++) zinv[s] = inv(sub(mul(gn, pow_u64(wce, s)), one()));
  }
  felt* dz = ctx->buf<felt>(zkey, ce);
  if (!ctx->have_cached(zkey)) ctx->upload(dz, zinv.data(), ce * 16);
  // coefficient-dependent constants, built on the device from the drawn coefficients
  // (MiMC: Z_T constants with the transition coefficient folded in, then b0, b1;
  // linear AIRs: the 4 coefficient rows + the two boundary sums)
  const uint32_t lw = air.id == ZKP_AIR_TRAINING_UPDATE ? w / 2 : w;
  felt* dconst = ctx->buf<felt>("eval_consts", air.id == ZKP_AIR_MIMC ? (size_t)ce + 4 : 4 * (size_t)lw + 2);
  launch_dt_eval_consts(pf, st, air.id, dt_cc, air.k, ec.w_last, dt_aval, dz, ce, w, air.num_t, dconst);
  ec.zinv = air.id == ZKP_AIR_MIMC ? dconst : dz;
  const std::string dom = std::to_string(logn) + "_" + std::to_string(logB) + "_" + std::to_string(u0) + "_" +
                          std::to_string(cel);
  // coefficient form for the linear AIRs (profiles/r03_ab_linear_coef_eval.txt)
  const bool coef_form = air.id != ZKP_AIR_MIMC && coef;
  if (!cel && !coef_form) return;
  // linear AIRs: the divisor tables and the final per-point formula (both forms)
  auto linear = [&](LinearEvalArgs& la, const std::string& key) {
    la.binv_ready = ctx->have_cached(key);
    la.binv = ctx->buf<felt>("binv_scratch", ((uint64_t)cel * n) / 2048 + 1);
    la.dinv = ctx->buf<felt>(key, (uint64_t)cel * n);
    if (!coef_form) {
      launch_eval_linear(pf, st, ec, la, tlde, comp);
      return;
    }
    const uint32_t R = cm ? (uint32_t)cm->world : 1u, rank = cm ? (uint32_t)cm->rank : 0u;
    const uint32_t narr = (la.transition ? 1u : 0u) + 1u + (la.two_groups ? 1u : 0u);
    const uint64_t nR = n / R;
    felt* lc = ctx->buf<felt>("lin_coef", (size_t)narr * n);
    felt* mine = R > 1 ? ctx->buf<felt>("lin_mine", (size_t)narr * nR) : lc;
    felt* part = ctx->buf<felt>("lincomb_part", (size_t)4 * lincomb_groups(nR, la.width) * nR);
    launch_lin_lincomb(pf, st, la.transition, la.two_groups, coef, la.width, logn, (uint64_t)rank * nR, nR,
                       dconst, twn, mine, part);
    for (uint32_t i = 0; R > 1 && i < narr; i++) cm->all_gather(st, mine + i * nR, lc + i * n, nR * 16);
    if (!cel) return;
    // extend to the CE cosets u0..u0+cel (LDE cosets u*B/ce): their coset-scale rows
    // gathered into one table per (n, B, ce), cached
    const uint32_t cstep = logB - logce;
    const std::string skey = "Sce_" + std::to_string(logn) + "_" + std::to_string(logB) + "_" + std::to_string(logce);
    const felt* S = ctx->S(logn, logB);
    const felt* Sce = S;
    if (cstep) {
      felt* t = ctx->buf<felt>(skey, (size_t)ce * n);
      if (!ctx->have_cached(skey))
        HIP_CHECK(hipMemcpy2DAsync(t, n * 16, S, (n << cstep) * 16, n * 16, ce, hipMemcpyDeviceToDevice, st));
      Sce = t;
    }
    felt* ev = ctx->buf<felt>("lin_ev", (size_t)narr * cel * n);
    NttBatch eb{lc, ev, Sce + (uint64_t)u0 * n, n, n, cel, cel, narr * cel};
    launch_ntt(pf, st, eb, logn, true, ctx->tws(logN), logN);
    launch_eval_linear_pts(pf, st, ec, la, ev, comp);
  };
  if (air.id == ZKP_AIR_MIMC) {
    // periodic column K over the CE domain: interpolate over <w_64>, evaluate at g^(n/64) * <w_{64 ce}>
    // (domain-only: cached per (n, ce))
    const std::string kkey = "kper_" + std::to_string(logn) + "_" + std::to_string(logce);
    felt* dk = ctx->buf<felt>(kkey, 64 * (size_t)ce);
    if (!ctx->have_cached(kkey)) {
      std::vector<felt> kc(64);
      for (int j = 0; j < 64; j++) kc[j] = felt_u64((uint64_t)(j + 1) * 1000000ull);
      host_interpolate(kc, one());
      std::vector<felt> kv = host_evaluate(kc, 64 * ce, pow_u64(g, n / 64));
      ctx->upload(dk, kv.data(), kv.size() * 16);
    }
    MimcEvalArgs ma;
    ma.bcoef = dconst + ce;  // the regrouped boundary constants A, Bc, Cc, D
    ma.kper = dk;
    // divisor inverses depend only on the domain and the assertion steps: cache per config
    std::string key = "binv_mimc_" + dom;
    ma.binv_ready = ctx->have_cached(key);
    ma.binv = ctx->buf<felt>("binv_scratch", ((uint64_t)cel * n) / 2048 + 1);
    ma.dinv = ctx->buf<felt>(key, (uint64_t)cel * n);
    launch_eval_mimc(pf, st, ec, ma, tlde, comp);
  } else if (air.id == ZKP_AIR_GLOBAL_UPDATE) {
    // GlobalUpdate: T = sum_i a^i (k*next_i - k*cur_i - next_{i+60}); B = sum_c b_c (cur_c - v_c)
    LinearEvalArgs la;
    la.width = w;
    la.transition = true;
    la.two_groups = false;
    la.coefs = dconst;  // [next | cur | beta0 | beta1 | bconst0, bconst1]
    la.w_bstep = pow_u64(wn, air.a_step[0]);
    la.w_bstep1 = zero();
    linear(la, "binv_lin_" + dom + "_" + std::to_string(air.a_step[0]));
  } else {
    // TrainingUpdate: transitions identically zero; boundary groups at rows 0 and n-1 over
    // the masked columns 0..w/2 (the mask columns are never read)
    const uint32_t half = w / 2;
    LinearEvalArgs la;
    la.width = half;
    la.transition = false;
    la.two_groups = true;
    la.coefs = dconst;
    la.w_bstep = one();
    la.w_bstep1 = ec.w_last;
    linear(la, "binv_tu_" + dom);
  }
}

// LastCol constants per LDE coset j (ce == B): kappa_j = (g w_N^j)^n = g^n w_B^j and
// kappa_j^-(C-1), at [2j, 2j+1] (shape-only: cached per (n, B, C))
const felt* last_col_kappa(zkp_ctx* ctx, uint32_t logn, uint32_t logB, uint32_t C) {
  const uint32_t B = 1u << logB;
  const std::string key = "lastcol_kap_" + std::to_string(logn) + "_" + std::to_string(logB) + "_" +
                          std::to_string(C);
  felt* d = ctx->buf<felt>(key, 2 * (size_t)B);
  if (!ctx->have_cached(key)) {
    std::vector<felt> h(2 * (size_t)B);
    const felt gn = pow_u64(felt_u64(3), 1ull << logn), wB = root_of_unity(logB);
    for (uint32_t j = 0; j < B; j++) {
      h[2 * j] = mul(gn, pow_u64(wB, j));
      h[2 * j + 1] = inv(pow_u64(h[2 * j], C - 1));
    }
    ctx->upload(d, h.data(), h.size() * 16);
  }
  return d;
}

// constants of k_comp_dft: [g^-mn / ce for m < C | w_ce^-k for k < ce/2]
std::vector<felt> comp_dft_consts(uint64_t n, uint32_t logce, uint32_t C) {
  const uint32_t ce = 1u << logce;
  std::vector<felt> dc((size_t)C + ce / 2);
  const felt g = felt_u64(3), ce_inv = inv(felt_u64(ce)), gn_inv = inv(pow_u64(g, n)),
             wce_inv = inv(root_of_unity(logce));
  for (uint32_t m = 0; m < C; m++) dc[m] = mul(pow_u64(gn_inv, m), ce_inv);
  for (uint32_t k = 0; k < ce / 2; k++) dc[C + k] = pow_u64(wce_inv, k);
  return dc;
}

// Sharded, each rank combines 1/R of the positions and the combined column is
// all-gathered (n * 16 bytes in all) instead of every rank reading all w columns.
void deep_evaluations(zkp_ctx* ctx, zkp_comm* cm, hipStream_t st, DeepArgs da, const felt* coef, uint64_t n,
                      const felt* Sj0, uint32_t logN, felt* out) {
  if (da.w < DEEP_COEF_MIN_W) {
    launch_deep(ctx->prof, st, da, out);
    return;
  }
  const uint32_t Bl = 1u << da.logBl;
  const uint32_t R = (uint32_t)cm->world;
  felt* acomb = ctx->buf<felt>("deep_acoef", n);
  const uint64_t nR = n / R;
  felt* part = ctx->buf<felt>("lincomb_part", (size_t)lincomb_groups(nR, da.w) * nR);
  if (R == 1) {
    launch_deep_lincomb(ctx->prof, st, coef, da.w, n, 0, n, da.gamma, acomb, part);
  } else {
    felt* mine = ctx->buf<felt>("deep_acoef_rank", nR);
    launch_deep_lincomb(ctx->prof, st, coef, da.w, n, (uint64_t)cm->rank * nR, nR, da.gamma, mine, part);
    cm->all_gather(st, mine, acomb, nR * 16);
  }
  felt* alde = ctx->buf<felt>("deep_alde", (size_t)Bl * n);
  NttBatch lb{acomb, alde, Sj0, n, n, Bl, Bl, Bl};
  launch_ntt(ctx->prof, st, lb, da.logn, true, ctx->tws(logN), logN);
  felt* g1 = ctx->buf<felt>("deep_g1", (size_t)da.C + 1);  // [1 | delta_0 .. delta_{C-1}]
  if (!ctx->have_cached("deep_g1")) {
    const felt unit = one();
    ctx->upload(g1, &unit, 16);
  }
  HIP_CHECK(hipMemcpyAsync(g1 + 1, da.gamma + da.w, (size_t)da.C * 16, hipMemcpyDeviceToDevice, st));
  da.w = 1;
  da.tlde = alde;
  da.gamma = g1;
  launch_deep(ctx->prof, st, da, out);
}

// Gathers every opening at the sorted unique LDE positions `pos` (this rank
// holds the LDE cosets [j0, j0 + Bl)); collective over cm when sharded.
void gather_openings(zkp_ctx* ctx, zkp_comm* cm, const std::vector<uint64_t>& pos, uint64_t n, uint32_t logB,
                     uint32_t j0, const felt* tlde, uint32_t w, const TreeShard& ttree, const felt* clde, uint32_t C,
                     const TreeShard& ctree, const std::vector<FriLayer>& layers, uint32_t L, uint32_t F,
                     Openings& op) {
  Prof& pf = ctx->prof;
  hipStream_t st = ctx->stream;
  const uint32_t R = (uint32_t)cm->world, rank = (uint32_t)cm->rank;
  const uint32_t B = 1u << logB, Bl = B / R;
  const uint64_t N = n << logB;
  // Openings: every item is (owner rank, local index) or a host-side top node.
  // Each rank gathers all items from its own memory (index 0 for items it does
  // not own), the gathered buffers are all-gathered, and every item is taken
  // from its owner's copy.
  struct SegPlan {
    const void* src;
    std::vector<uint64_t> idx;
    std::vector<int32_t> owner;  // -1: host top node (value in host_dig)
    std::vector<const uint8_t*> host_dig;
    uint32_t words;
  };
  auto row_owner = [&](uint64_t j) -> uint32_t { return R > 1 ? (uint32_t)(j / Bl) : 0; };
  auto lde_values = [&](const felt* src, uint32_t cols) {
    SegPlan sp{src, {}, {}, {}, 4};
    sp.idx.reserve(pos.size() * cols);
    sp.owner.reserve(pos.size() * cols);
    sp.host_dig.reserve(pos.size() * cols);
    for (uint64_t p : pos) {
      uint64_t j = p & (B - 1), t = p >> logB;
      uint32_t ow = row_owner(j);
      for (uint32_t c = 0; c < cols; c++) {
        sp.idx.push_back(ow == rank ? ((uint64_t)c * Bl + (j - j0)) * n + t : 0);
        sp.owner.push_back((int32_t)ow);
        sp.host_dig.push_back(nullptr);
      }
    }
    return sp;
  };
  auto path_nodes = [&](const TreeShard& tr, const BatchPlan& bp) {
    SegPlan sp{tr.nodes, {}, {}, {}, 8};
    for (auto& pth : bp.paths)
      for (uint64_t k : pth) {
        TreeShard::Loc lc = tr.locate(k);
        if (lc.host) {
          sp.idx.push_back(0);
          sp.owner.push_back(-1);
          sp.host_dig.push_back(tr.top[lc.local].data());
        } else {
          sp.idx.push_back(lc.owner == (tr.logR ? rank : 0u) ? lc.local : 0);
          sp.owner.push_back(tr.logR ? (int32_t)lc.owner : (int32_t)rank);
          sp.host_dig.push_back(nullptr);
        }
      }
    return sp;
  };
  op.bt = plan_batch(N, pos);
  const BatchPlan& bt = op.bt;
  const BatchPlan& bc = bt;  // the constraint tree has the same shape and positions
  std::vector<std::vector<uint64_t>> fpos(L);
  op.bf.assign(L, BatchPlan{});
  std::vector<BatchPlan>& bf = op.bf;
  std::vector<SegPlan> plan;
  plan.push_back(lde_values(tlde, w));
  plan.push_back(path_nodes(ttree, bt));
  plan.push_back(lde_values(clde, C));
  plan.push_back(path_nodes(ctree, bc));
  {
    std::vector<uint64_t> cur = pos;
    for (uint32_t l = 0; l < L; l++) {
      const FriLayer& ly = layers[l];
      const uint64_t m16 = ly.m / F, Rows = (uint64_t)B * m16;
      fpos[l] = fold_positions(cur, Rows);
      bf[l] = plan_batch(Rows, fpos[l]);
      SegPlan sp{ly.E, {}, {}, {}, 4};
      for (uint64_t r : fpos[l])
        for (uint32_t k = 0; k < F; k++) {
          uint64_t i = r + k * Rows;  // natural index in the layer
          uint64_t j = i & (B - 1), tt = i >> logB;
          uint32_t ow = ly.sharded ? (uint32_t)(j / Bl) : rank;
          sp.idx.push_back(ow == rank ? (j - ly.jc) * ly.m + tt : 0);
          sp.owner.push_back((int32_t)ow);
          sp.host_dig.push_back(nullptr);
        }
      plan.push_back(sp);
      plan.push_back(path_nodes(ly.tree, bf[l]));
      cur = fpos[l];
    }
  }
  std::vector<GatherSeg>& segs = op.segs;
  segs.clear();
  std::vector<uint64_t> all_idx;
  uint64_t out_words = 0, max_count = 1;
  for (auto& sp : plan) {
    GatherSeg gs;
    gs.src = sp.src;
    gs.idx_off = all_idx.size();
    gs.count = sp.idx.size();
    gs.out_off = out_words;
    gs.words = sp.words;
    gs.pad = 0;
    all_idx.insert(all_idx.end(), sp.idx.begin(), sp.idx.end());
    out_words += gs.count * sp.words;
    max_count = std::max<uint64_t>(max_count, gs.count);
    segs.push_back(gs);
  }
  size_t seg_bytes = segs.size() * sizeof(GatherSeg), idx_bytes = all_idx.size() * 8;
  size_t up_bytes = seg_bytes + idx_bytes, down_bytes = out_words * 4;
  ctx->stage_end("7a_query_plan");
  uint8_t* hp = (uint8_t*)ctx->pinned(std::max(up_bytes, down_bytes * R) + 64);
  memcpy(hp, segs.data(), seg_bytes);
  memcpy(hp + seg_bytes, all_idx.data(), idx_bytes);
  uint8_t* dup = ctx->buf<uint8_t>("gather_in", up_bytes + 16);
  uint32_t* dout = ctx->buf<uint32_t>("gather_out", out_words + 4);
  uint32_t* dall = R > 1 ? ctx->buf<uint32_t>("gather_all", out_words * R + 4) : dout;
  HIP_CHECK(hipMemcpyAsync(dup, hp, up_bytes, hipMemcpyHostToDevice, st));
  launch_gather_multi(pf, st, (const GatherSeg*)dup, (uint32_t)segs.size(), max_count,
                      (const uint64_t*)(dup + seg_bytes), dout, (double)down_bytes * 2);
  if (R > 1) cm->all_gather(st, dout, dall, down_bytes);
  HIP_CHECK(hipMemcpyAsync(hp, dall, down_bytes * R, hipMemcpyDeviceToHost, st));
  ctx->sync();
  ctx->stage_end("7b_gather");
  op.gathered.assign(out_words, 0);
  std::vector<uint32_t>& gathered = op.gathered;
  {
    const uint32_t* all = reinterpret_cast<const uint32_t*>(hp);
    for (size_t si = 0; si < plan.size(); si++) {
      const SegPlan& sp = plan[si];
      const GatherSeg& gs = segs[si];
      for (size_t it = 0; it < sp.idx.size(); it++) {
        uint32_t* dst = gathered.data() + gs.out_off + it * sp.words;
        if (sp.owner[it] < 0) {
          memcpy(dst, sp.host_dig[it], 32);
        } else {
          uint32_t ow = R > 1 ? (uint32_t)sp.owner[it] : 0;
          memcpy(dst, all + (size_t)ow * out_words + gs.out_off + it * sp.words, sp.words * 4);
        }
      }
    }
  }
}

// Openings assembled on the host from the device's full gather (k_gather_full,
// world 1): the row values of every drawn position and the full sibling path of
// every leaf; the batch plans (plan_batch) pick their nodes from those paths.
// `raw` = the drawn positions in draw order (the gather's record order), `pos`
// = sorted unique; the result has gather_openings' segment layout.
void openings_from_full(const std::vector<uint64_t>& raw, const std::vector<uint64_t>& pos, const uint32_t* full,
                        const FullGatherArgs& ga, const std::vector<FriLayer>& layers, uint32_t L, uint32_t F,
                        Openings& op) {
  const uint32_t w = ga.w, C = ga.C, nv = w + C, logN = ga.logN;
  const uint64_t N = 1ull << logN, B = 1ull << ga.logB;
  auto missing = [] { return ZkpFail{ZKP_ERR_DEVICE, "device query gather is missing an opening"}; };
  // (leaf node index L + row, record index) sorted by node: node k at height d is on
  // the path of the leaves whose node index lies in [k << d, (k + 1) << d)
  struct Leaves {
    std::vector<std::pair<uint64_t, uint32_t>> v;
    uint32_t logL;
    // record of any drawn leaf below node k (height d above the leaves); -1 if none
    int64_t below(uint64_t k, uint32_t d) const {
      auto it = std::lower_bound(v.begin(), v.end(), std::make_pair(k << d, 0u));
      return it != v.end() && (it->first >> d) == k ? (int64_t)it->second : -1;
    }
    // height of node k above the leaves
    uint32_t height(uint64_t k) const { return logL - (63 - __builtin_clzll(k)); }
  };
  auto leaves_of = [&](uint64_t Lcount, uint32_t logL) {
    Leaves lv;
    lv.logL = logL;
    lv.v.reserve(raw.size());
    for (size_t i = 0; i < raw.size(); i++) lv.v.push_back({Lcount + (raw[i] & (Lcount - 1)), (uint32_t)i});
    std::sort(lv.v.begin(), lv.v.end());
    return lv;
  };
  op.segs.clear();
  op.gathered.clear();
  op.gathered.reserve(full ? 4096 : 0);
  auto begin_seg = [&](uint32_t words) {
    GatherSeg g{};
    g.out_off = op.gathered.size();
    g.words = words;
    op.segs.push_back(g);
  };
  auto put = [&](const uint32_t* src, uint32_t words) {
    op.gathered.insert(op.gathered.end(), src, src + words);
    op.segs.back().count++;
  };
  // a batch path node k is the sibling, at height d, of a drawn leaf's path: the record
  // of a leaf below k ^ 1 holds it at path slot d
  auto paths = [&](const BatchPlan& bp, const Leaves& lv, uint32_t seg, uint32_t path_off) {
    begin_seg(8);
    for (auto& pth : bp.paths)
      for (uint64_t k : pth) {
        const uint32_t d = lv.height(k);
        const int64_t i = lv.below(k ^ 1ull, d);
        if (i < 0) throw missing();
        put(full + ga.seg_off[seg] + (uint64_t)i * ga.rec_words[seg] + path_off + 8 * d, 8);
      }
  };
  const Leaves l0 = leaves_of(N, logN);
  op.bt = plan_batch(N, pos);
  for (int seg = 0; seg < 2; seg++) {  // values, then batch paths, of the trace and constraint commitments
    begin_seg(4);
    for (uint64_t p : pos) {
      const int64_t i = l0.below(N + p, 0);
      if (i < 0) throw missing();
      const uint32_t* r = full + (uint64_t)i * ga.rec_words[0];
      for (uint32_t c = seg ? w : 0; c < (seg ? nv : w); c++) put(r + 4 * c, 4);
    }
    paths(op.bt, l0, 0, 4 * nv + (seg ? 8 * logN : 0));
  }
  op.bf.assign(L, BatchPlan{});
  std::vector<uint64_t> cur = pos;
  for (uint32_t l = 0; l < L; l++) {
    const uint64_t Rows = B * (layers[l].m / F);
    const Leaves lv = leaves_of(Rows, ga.logrows[l]);
    std::vector<uint64_t> fp = fold_positions(cur, Rows);
    op.bf[l] = plan_batch(Rows, fp);
    begin_seg(4);
    for (uint64_t r : fp) {
      const int64_t i = lv.below(Rows + r, 0);
      if (i < 0) throw missing();
      const uint32_t* rec = full + ga.seg_off[1 + l] + (uint64_t)i * ga.rec_words[1 + l];
      for (uint32_t k = 0; k < F; k++) put(rec + 4 * k, 4);
    }
    paths(op.bf[l], lv, 1 + l, 64);
    cur = fp;
  }
}

// constants of the fold-16 iDFT (w_16^-m for m < 8, then 16^-1), cached per context
const felt* fold_constants(zkp_ctx* ctx) {
  felt* deps = ctx->buf<felt>("eps_inv", 9);
  if (!ctx->have_cached("eps_inv")) {
    std::vector<felt> eps(9);
    felt einv = inv(root_of_unity(4));
    eps[0] = one();
    for (int m = 1; m < 8; m++) eps[m] = mul(eps[m - 1], einv);
    eps[8] = inv(felt_u64(16));
    ctx->upload(deps, eps.data(), 9 * 16);
  }
  return deps;
}

}  // namespace zkpi
