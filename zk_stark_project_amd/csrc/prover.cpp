// prover.cpp — host orchestration of the MI355X STARK prover + the C-ABI of
// include/zkp.h.
//
// Mirrors winterfell 0.12 `Prover::generate_proof` (the path selected by the
// reference's plug-ins, src/aggregation/prover.rs:194-248): channel seeding,
// trace LDE + commitment, constraint evaluation, composition commitment, OOD,
// DEEP, FRI, grinding, queries, serialization. Every O(n) stage runs on the
// GPU (kernels.hip); the host only drives the Fiat-Shamir transcript and
// assembles the proof bytes from the few values the verifier needs.
#include "prover_internal.hpp"

#include <mutex>

using namespace zkpi;

namespace zkpi {

// option / shape checks and the derived shapes (ZKP_ERR_* on a bad request)
int ProofRun::init(int air_id, const felt* d_trace_in, uint32_t width, uint64_t n_rows, const zkp_felt* pub_elems,
                   uint64_t n_pub, uint8_t** proof, uint64_t* proof_len) {
  d_trace = d_trace_in;
  w = width;
  n = n_rows;
  int rc = check_options(o);
  if (rc) return rc;
  if (n < 8 || (n & (n - 1)) || w == 0 || w > 255) return ZKP_ERR_TRACE_SHAPE;
  if (!proof || !proof_len || (n_pub && !pub_elems)) return ZKP_ERR_ARGUMENT;
  B = o->blowup_factor; F = o->fri_folding_factor;
  logn = ilog2(n); logB = ilog2(B); logN = logn + logB;
  N = 1ull << logN;
  if (logN > MAX_LOG_DOMAIN || logn > MAX_LOG_TRACE) return ZKP_ERR_TRACE_SHAPE;
  // coset sharding: rank r owns the LDE cosets [j0, j0 + Bl)
  R = (uint32_t)cm->world; rank = (uint32_t)cm->rank;
  if (R == 0 || (R & (R - 1)) || R > B || rank >= R) return ZKP_ERR_ARGUMENT;
  logR = ilog2(R); Bl = B >> logR; logBl = logB - logR; j0 = rank * Bl;
  if (R > 1 && logn < logR + 8) return ZKP_ERR_TRACE_SHAPE;  // each rank's Merkle range needs >= 256 rows/coset
  pub.resize(n_pub);
  for (uint64_t i = 0; i < n_pub; i++) pub[i] = make(pub_elems[i].lo, pub_elems[i].hi);
  rc = build_air(air, air_id, w, n, pub);
  if (rc) return rc;
  ce = air.ce_blowup(); C = air.comp_cols();
  if (B < ce) return ZKP_ERR_INVALID_OPTIONS;
  logce = ilog2(ce);
  if (ce > 16 || C > ce) return ZKP_ERR_UNSUPPORTED_AIR;
  // CE coset u lives in LDE coset u << (logB - logce); this rank evaluates the CE cosets it holds
  cstep = logB - logce;
  u0 = ce_first(rank);
  cel = 0;
  while (u0 + cel < ce && ce_owner(u0 + cel) == rank) cel++;
  celmax = ce >= R ? ce / R : 1;
  g = felt_u64(3);
  ood_trace.assign(2 * (size_t)w, felt{});
  ood_comp.assign(C, felt{});
  return 0;
}

// 1. channel: Context::to_elements || pub_inputs.to_elements; device transcript seed, domain tables
void ProofRun::setup() {
  ctx->sync();
  ctx->ring_reset();
  ctx->stage_begin();
  // 1. channel: Context::to_elements || pub_inputs.to_elements
  {
    std::vector<felt> se = context_elements(air, o);
    se.insert(se.end(), pub.begin(), pub.end());
    coin.init(se);
  }
  // device transcript: the coin state lives in HBM from here until
  // the OOD download; the device draws the composition coefficients and z, the
  // host replays both draws from the downloaded roots and checks them
  ncoef = air.num_t + (uint32_t)air.a_col.size();
  dt_seed = ctx->buf<uint32_t>("dt_seed", 8);
  dt_cc = ctx->buf<felt>("dt_cc", ncoef);
  dt_zz = ctx->buf<felt>("dt_zz", 2);
  dt_pw = ctx->buf<felt>("dt_pw", 2 * (size_t)logn);
  dt_aval = ctx->buf<felt>("dt_aval", air.a_val.size());
  {
    uint32_t sw[8];
    for (int i = 0; i < 8; i++)
      sw[i] = (uint32_t)coin.seed[4 * i] | ((uint32_t)coin.seed[4 * i + 1] << 8) |
              ((uint32_t)coin.seed[4 * i + 2] << 16) | ((uint32_t)coin.seed[4 * i + 3] << 24);
    ctx->upload(dt_seed, sw, 32);
    ctx->upload(dt_aval, air.a_val.data(), air.a_val.size() * 16);
  }
  ctx->stage_end("0a_seed");
  ctx->ensure_coset(logn, logB, logce);
  ctx->stage_end("0b_coset");
  Sj0 = ctx->S(logn, logB) + (uint64_t)j0 * n;
  // domain points: coset offsets g*w_N^j (LDE cosets) and g*w_M^u (CE cosets), w_n^t table
  // (domain-only: cached per (n, B, ce), so no upload sits between the proof's kernels)
  cx = coset_points(ctx, logn, logB, logce);
  twn = ctx->tws(logN) + ((1ull << (logn - 1)) - 1);
  ctx->stage_end("0_setup");
}

// 2. trace LDE + commitment (DefaultTraceLde::new)
void ProofRun::trace_stage(const zkp_felt* h_trace) {
  // 2. trace LDE + commitment (DefaultTraceLde::new): interpolation (by column
  // over the ranks for wide traces), coset LDE of this rank's cosets, sharded
  // row commitment
  coef = ctx->buf<felt>("coef", (size_t)(w + C) * n);
  tlde = ctx->buf<felt>("tlde", (size_t)w * Bl * n);
  bool coeffs_drawn = false;
  // GlobalUpdate column pairing (k_gu_check): only columns [0, wi)
  // are interpolated and extended; column d+i >= wi is checked against its
  // transition constraint and derived from column i. A trace that fails the check
  // is proven again unpaired (prove_impl), so the result never depends on the
  // shortcut. Sharded proofs pair device-resident traces (every rank holds the
  // whole trace; a host trace uploads only the rank's share).
  static const bool no_pair = getenv("ZKP_NO_GU_PAIR") != nullptr;  // A/B switch
  paired = allow_shortcuts && !no_pair && air.id == ZKP_AIR_GLOBAL_UPDATE && w == 2 * GU_D && (R == 1 || !h_trace);
  const uint32_t d = w / 2;
  // wide traces shard the interpolation by column (cpt columns per rank) when the
  // width divides over the ranks; narrow ones interpolate on every rank
  uint32_t wi = paired && R > 1 ? (d + R - 1) / R * R : w;
  uint32_t cpt = (R > 1 && wi % R == 0 && wi >= 2 * R && wi <= w) ? wi / R : 0;
  if (R > 1 && !cpt) wi = w, cpt = (w % R == 0 && w >= 2 * R) ? w / R : 0;
  if (paired) {
    gu_cval = ctx->buf<felt>("gu_cval", d);
    gu_bad = ctx->buf<uint32_t>("gu_bad", 4);
    HIP_CHECK(hipMemsetAsync(gu_bad, 0, 16, st));
    // lazy: the paired LDE columns are never materialized — the trace tree's row
    // hash derives them and the openings fill the queried rows (launch_gu_fill);
    // the coefficient-form constraint evaluation and DEEP never read the trace LDE
    // (profiles/r03_ab_gu_lazy.txt)
    gu_lazy_on = w >= DEEP_COEF_MIN_W;
    gu_lazy = GuLazy{gu_cval, l0_table(), air.k, d, R > 1 && cpt && wi < w ? wi : d,
                     (uint32_t)(air.k.hi == 0 && (air.k.lo >> 32) == 0)};
  }
  if (cpt) {
    trace_column_sharded(h_trace, cpt, wi, d);
  } else {
    if (h_trace && R > 1) h_trace = gather_host_slices(h_trace);  // resident on every rank from here
    const uint32_t wd = paired ? d : w;  // columns interpolated and extended here
    // groups (first column, columns) of [0, wd): one for device-resident traces.
    // Host traces upload group g+1 on the side stream while the main stream
    // interpolates and extends group g; the groups grow geometrically (x1.5 from
    // ~w/40 columns: C3 unpaired 3, 4, 6, ..., 38), so only the small first group's
    // upload is exposed and every later one hides behind the previous group's LDE
    // (a column uploads in ~0.55x its LDE at C3).
    std::vector<std::pair<uint32_t, uint32_t>> grp;
    constexpr uint32_t growth = 150;  // percent (x1.25 and x2.0 slower: profiles/r03_ab_upload_groups.txt)
    // Short traces start from >= 2^19 felts per group (8 MiB): a group's transforms are
    // latency-bound launches below that (TrainingUpdate at bs = 50, 2^13 x 240: 9 groups
    // of 6..54 columns became 3 of 64, 96, 80)
    if (h_trace && wd >= 4) {
      // (at least two groups: the late paired upload rides on the pipeline's side stream)
      uint32_t cw = std::min(std::max({1u, w / 40, (uint32_t)((1ull << 19) >> std::min(logn, 19u))}),
                             std::max(1u, wd / 2));
      for (uint32_t c = 0; c < wd;) {
        cw = std::min(cw, wd - c);
        grp.push_back({c, cw});
        c += cw;
        cw = std::max(cw + 1, cw * growth / 100);
      }
    } else {
      grp.push_back({0u, wd});
    }
    // paired, device-resident: one group that checks and derives every pair. A host
    // trace derives from row 0 of the paired columns alone (c_i), so the trace
    // commitment waits only for columns [0, d): the paired columns' bulk upload and
    // the check of their rows 1..n-1 follow on the copy stream once the proof's
    // kernels are queued (late_pairs_upload; pair_failed joins it)
    const bool late_pairs = paired && h_trace;
    if (paired && !h_trace) grp.push_back({d, d});
    // a device-resident paired trace is checked before its columns are transformed:
    // a failing pair falls back to the plain interpolation of [d, w) in the group
    // loop below, instead of a second proof (world 1; sharded proofs all-gather
    // their flags and prove again)
    // (the checks run on the side stream, beside the first columns' transforms)
    const bool early_pairs = paired && !h_trace && R == 1;
    if (early_pairs) {
      HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
      HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
      launch_gu_check(pf, ctx->side, d_trace, d, logn, air.k, 0, d, 0, logn, gu_cval, gu_bad);
      early_check_launch(gu_bad, ctx->side);
    }
    // MiMC: the trace against its transitions and assertions (k_mimc_check), read by
    // composition_stage to choose the derived last column (LastCol)
    // (world 1: a sharded rank would check the whole replicated trace, 56 us of extra
    // work at C4 for every valid proof; sharded proofs keep the all-gathered LastCol flags)
    // (only where LastCol can read it: blowup 16, say, has ce != B and never derives)
    const bool mimc_check = air.id == ZKP_AIR_MIMC && w == 1 && R == 1 && lastcol_shape();
    const bool piped = h_trace && grp.size() > 1;
    const size_t G = grp.size();
    if (piped) {  // the copy stream starts after everything already queued
      ctx->events(G + 2);
      HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
      HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    }
    if (late_pairs) {  // row 0 of the paired columns first (one 2-D copy of d felts)
      if (!piped) throw ZkpFail{ZKP_ERR_DEVICE, "paired host trace without column groups"};
      HIP_CHECK(hipMemcpy2DAsync(const_cast<felt*>(d_trace) + (size_t)d * n, n * 16, h_trace + (size_t)d * n, n * 16,
                                 16, d, hipMemcpyHostToDevice, ctx->side));
      HIP_CHECK(hipEventRecord(ctx->up_ev[G], ctx->side));
    }
    for (uint32_t g = 0; g < grp.size(); g++) {
      const uint32_t c0 = grp[g].first, cw = grp[g].second;
      felt* dcol = const_cast<felt*>(d_trace) + (size_t)c0 * n;
      if (piped) {
        HIP_CHECK(hipMemcpyAsync(dcol, h_trace + (size_t)c0 * n, (size_t)cw * n * 16, hipMemcpyHostToDevice,
                                 ctx->side));
        HIP_CHECK(hipEventRecord(ctx->up_ev[g], ctx->side));
        HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[g], 0));
      } else if (h_trace && g == 0) {
        ctx->upload(dcol, h_trace, (size_t)w * n * 16);
      }
      if (g == 0 && mimc_check) {
        uint32_t* dflag = ctx->buf<uint32_t>("mimc_bad", 4);
        HIP_CHECK(hipEventRecord(ctx->ev_fork, st));  // the trace is on the device
        HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
        HIP_CHECK(hipMemsetAsync(dflag, 0, 16, ctx->side));
        launch_mimc_check(pf, ctx->side, d_trace, n, air.a_val[0], air.a_val[1], dflag);
        early_check_launch(dflag, ctx->side);
      }
      if (c0 >= wd && early_pairs) HIP_CHECK(hipStreamWaitEvent(st, ctx->ev_check, 0));  // gu_cval
      if (c0 >= wd && early_pairs && early_check_failed()) {
        // a pair fails its transition: these columns are interpolated and extended
        // like the others, and nothing downstream derives them
        paired = false;
        gu_lazy_on = false;
      } else if (c0 >= wd) {  // paired columns d+i, i in [c0 - d, c0 - d + cw): check, then derive
        const uint32_t i0 = c0 - d;
        if (!early_pairs) launch_gu_check(pf, st, d_trace, d, logn, air.k, i0, cw, 0, logn, gu_cval, gu_bad);
        launch_gu_coef(pf, st, coef, d, logn, air.k, ctx->itws(logN) + ((n >> 1) - 1), i0, cw, 0, n, gu_cval);
        if (!gu_lazy_on) launch_gu_lde(pf, st, tlde, d, logn, logBl, air.k, i0, cw, gu_cval, l0_table());
        continue;
      }
      NttBatch ib{dcol, coef + (size_t)c0 * n, nullptr, n, n, 1, 1, cw};
      launch_ntt(pf, st, ib, logn, false, ctx->itws(logN), logN);
      NttBatch lb{coef + (size_t)c0 * n, tlde + (size_t)c0 * Bl * n, Sj0, n, n, Bl, Bl, cw * Bl};
      launch_ntt(pf, st, lb, logn, true, ctx->tws(logN), logN);
    }
    if (late_pairs) {
      // main stream: c_i from row 0, the derived coefficients (and LDE unless lazy)
      HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[G], 0));
      launch_gu_check(pf, st, d_trace, d, logn, air.k, 0, d, 0, 0, gu_cval, gu_bad);
      launch_gu_coef(pf, st, coef, d, logn, air.k, ctx->itws(logN) + ((n >> 1) - 1), 0, d, 0, n, gu_cval);
      if (!gu_lazy_on) launch_gu_lde(pf, st, tlde, d, logn, logBl, air.k, 0, d, gu_cval, l0_table());
      // copy stream, after the last group's upload: the paired columns and their check,
      // issued by late_pairs_upload() once the proof's kernels are all queued (a
      // pageable upload holds the host thread for its whole length)
      HIP_CHECK(hipEventRecord(ctx->up_ev[G + 1], ctx->side));
      HIP_CHECK(hipStreamWaitEvent(ctx->copy, ctx->up_ev[G + 1], 0));
      late_h_trace = h_trace;
    }
  }
  {
    // unsharded: the tree's last block also reseeds with the root and draws the
    // composition coefficients (MERKLE_TAIL_DRAW_COEFFS)
    MerkleTail draw{};
    draw.op = MERKLE_TAIL_DRAW_COEFFS;
    draw.coin_seed = dt_seed;
    draw.method = o->batching_constraints;
    draw.ncoef = ncoef;
    draw.out = dt_cc;
    // host channel with a late paired upload: the root is read after that upload is
    // issued, so its PCIe time (the host thread blocks on a pageable copy) overlaps the
    // trace tree instead of following the root read
    const bool late_first = host_channel && late_h_trace && R == 1;
    coeffs_drawn = commit_rows(ctx, cm, 0, tlde, n, w, logB, logn, R > 1, "ttree", ttree, T.trace_root,
                               /*fetch_root=*/host_channel && !late_first, host_channel ? nullptr : &draw, nullptr,
                               gu_lazy_on ? &gu_lazy : nullptr);
    if (late_first) {
      late_pairs_upload();
      ctx->download(T.trace_root, ttree.nodes + 8, 32);
      memcpy(ttree.top[1].data(), T.trace_root, 32);
    }
  }
  troot_d = R > 1 ? ttree.top_d + 8 : ttree.nodes + 8;  // sharded: the device-built top
  // the composition coefficients (drawn on the device from the trace root)
  if (!coeffs_drawn && !host_channel)
    launch_dt_draw_coeffs(pf, st, dt_seed, troot_d, o->batching_constraints, ncoef, dt_cc);
  ctx->stage_end("1_trace_commit");
}

// 3-4. constraint evaluation (DefaultConstraintEvaluator) and the composition
// polynomial + its commitment (CompositionPoly::new + DefaultConstraintCommitment)
void ProofRun::constraint_stage() {
  eval_stage();
  composition_stage();
}

// 3. constraint evaluation (DefaultConstraintEvaluator) with the coefficients in
// dt_cc (device-drawn; a session's caller uploads its own)
void ProofRun::eval_stage() {
  comp = ctx->buf<felt>("comp", (size_t)(cel ? cel : 1) * n);
  constraint_eval(ctx, air, logn, logB, logce, u0, cel, j0, logBl, cx, twn, dt_cc, dt_aval, tlde, comp, coef, cm);
}

bool ProofRun::lastcol_shape() const {
  static const bool no_derive = getenv("ZKP_NO_DERIVE_LAST") != nullptr;  // A/B switch
  return allow_shortcuts && !no_derive && logce == logB && C >= 2 && C <= 8 && cel == Bl && u0 == j0;
}

// 4. composition polynomial + commitment (CompositionPoly::new +
// DefaultConstraintCommitment) from the evaluations in `comp`: per-CE-coset
// interpolation, exchange of coefficient slices, ce-point DFT per coefficient,
// all-gather, coset LDE
void ProofRun::composition_stage() {
  comp = ctx->buf<felt>("comp", (size_t)(cel ? cel : 1) * n);
  acoef = coef + (size_t)w * n;
  clde = ctx->buf<felt>("clde", (size_t)C * Bl * n);
  bool z_drawn = false;
  wn_root = root_of_unity(logn);
  {
    // this rank's slice of bit-reversed coefficient positions: [p0, p0 + nR)
    const uint64_t nR = n >> logR, p0 = (uint64_t)rank * nR;
    // the last composition column derived in the leaf pass (LastCol): the rank's
    // LDE cosets are exactly its CE cosets, whose evaluations stay in `comp`
    // a trace that fails k_mimc_check proves without it (its dropped segments would
    // not be zero); one that passes cannot raise lc_bad, which stays as the backstop
    const bool derive = lastcol_shape() && !(pre_checked && early_check_failed());
    derive_last = derive;
    if (derive) {
      lc_bad = ctx->buf<uint32_t>("lc_bad", 4);
      HIP_CHECK(hipMemsetAsync(lc_bad, 0, 16, st));
    }
    felt* cint = derive ? ctx->buf<felt>("comp_int", (size_t)(cel ? cel : 1) * n) : comp;
    if (cel) {
      NttBatch ib{comp, cint, nullptr, n, n, 1, 1, cel};
      launch_ntt(pf, st, ib, logn, false, ctx->itws(logN), logN);
    }
    felt* recv = cint;  // world 1: the rank holds every CE coset in full
    if (R > 1) recv = composition_exchange(cint, nR);
    // coefs[u*C + m] = w_ce^-um * g^-mn / ce ; blk[u] = receive block holding CE coset u
    // (shape-only: cached per (n, ce, C, R, celmax))
    const std::string dkey = "comp_dft_" + std::to_string(logn) + "_" + std::to_string(logce) + "_" +
                             std::to_string(C) + "_" + std::to_string(R) + "_" + std::to_string(celmax);
    felt* dcoefs = ctx->buf<felt>(dkey + "_coefs", (size_t)C + ce / 2);
    uint32_t* dblk = ctx->buf<uint32_t>(dkey + "_blk", ce);
    if (!ctx->have_cached(dkey)) {
      const std::vector<felt> dc = comp_dft_consts(n, logce, C);
      std::vector<uint32_t> blk(ce);
      for (uint32_t u = 0; u < ce; u++) {
        uint32_t s = ce_owner(u);
        blk[u] = s * celmax + (u - ce_first(s));
      }
      ctx->upload(dcoefs, dc.data(), dc.size() * 16);
      ctx->upload(dblk, blk.data(), blk.size() * 4);
    }
    felt* slice = R > 1 ? ctx->buf<felt>("comp_ag_send", (size_t)C * nR) : acoef;
    launch_comp_dft(pf, st, recv, dblk, ctx->Si(logn, logB, logce), dcoefs, ce, C, logn, p0, nR, slice,
                    derive ? lc_bad : nullptr);
    if (R > 1 && derive) {  // every rank's check of its position slice
      lc_flags = ctx->buf<uint32_t>("lc_flags", 4 * (size_t)R);
      cm->all_gather(st, lc_bad, lc_flags, 16);
    }
    if (R > 1) {
      composition_gather_lde(slice, derive, nR, p0);
    } else {
      NttBatch lb{acoef, clde, Sj0, n, n, Bl, Bl, (derive ? C - 1 : C) * Bl};
      launch_ntt(pf, st, lb, logn, true, ctx->tws(logN), logN);
    }
    LastCol lc{};
    if (derive) lc = LastCol{comp, last_col_kappa(ctx, logn, logB, C) + 2 * (size_t)j0, clde + (size_t)(C - 1) * Bl * n};
    MerkleTail draw{};  // unsharded: the tree's last block draws z (MERKLE_TAIL_DRAW_Z)
    draw.op = MERKLE_TAIL_DRAW_Z;
    draw.coin_seed = dt_seed;
    draw.wn = wn_root;
    draw.logn = logn;
    draw.out = dt_zz;
    draw.pw = dt_pw;
    z_drawn = commit_rows(ctx, cm, 0, clde, n, C, logB, logn, R > 1, "ctree", ctree, T.constraint_root,
                          /*fetch_root=*/host_channel, host_channel ? nullptr : &draw, derive ? &lc : nullptr);
  }
  croot_d = R > 1 ? ctree.top_d + 8 : ctree.nodes + 8;
  if (!z_drawn && !host_channel) launch_dt_draw_z(pf, st, dt_seed, croot_d, wn_root, logn, dt_zz, dt_pw);
  ctx->stage_end("2_constraints_commit");
}

// 5. OOD frame and the DEEP coefficients (device transcript)
// 5a. OOD frame at z = dt_zz[0] (powers in dt_pw; sharded: every rank holds all
// coefficients and sums 1/R of each array's blocks) and the DEEP denominators
void ProofRun::ood_values() {
  // the DEEP denominators (x - z)(x - zg) only need z: their batch-inversion
  // phases run on the side stream beside the OOD evaluation and its transcript
  deep_binv = ctx->buf<felt>("binv", ((uint64_t)Bl * n) / 2048 + 1);
  deep_pm = PointMap{cx + j0, twn, logn};
  HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
  HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  launch_deep_denominators(pf, ctx->side, deep_pm, (uint64_t)Bl * n, dt_zz, dt_pw, deep_binv);
  HIP_CHECK(hipEventRecord(ctx->ev_join, ctx->side));
  dv = ood_launch(ctx, coef, w + C, w, logn, dt_pw, cm);  // composition columns at z only
}

// 5. OOD frame and the DEEP coefficients on the device (device transcript); the
// host replays both at the FRI round trip
void ProofRun::ood_stage() {
  ood_values();
  dgam = ctx->buf<felt>("gamma", w + C);
  dk = ctx->buf<felt>("dt_dk", 4);
  HIP_CHECK(hipMemcpyAsync(dk, dt_zz, 32, hipMemcpyDeviceToDevice, st));
  launch_dt_deep_coeffs(pf, st, dt_seed, dv, w, C, o->batching_deep, dgam, dk);
  ctx->stage_end("3_ood");
}

// 6. DEEP composition evaluations over this rank's cosets
void ProofRun::deep_stage() {
  // 6. DEEP composition evaluations over this rank's cosets (coset-major)
  deep = ctx->buf<felt>("deep", (size_t)Bl * n);
  {
    DeepArgs da;
    da.w = w; da.C = C; da.logB = logB; da.logn = logn; da.logN = logN;
    da.j0 = j0; da.logBl = logBl;
    da.tlde = tlde; da.clde = clde; da.gamma = dgam; da.dk = dk; da.g = g;
    da.pm = deep_pm;
    da.binv = deep_binv;
    HIP_CHECK(hipStreamWaitEvent(st, ctx->ev_join, 0));
    deep_evaluations(ctx, cm, st, da, coef, n, Sj0, logN, deep);
  }
  ctx->stage_end("4_deep_launch");
}

// 7. FRI layers (FriProver::build_layers), remainder, the proof's host round trip
// and the host replay of the device transcript
void ProofRun::fri_stage() {
  const FriCursor c = fri_layers();
  fri_round_trip(c);
  ctx->stage_end("5_fri");
}

// the layer loop on the device: trees, coin steps, folds; then the remainder,
// the first grinding chunk and (world 1) the query tail
FriCursor ProofRun::fri_layers() {
  // 7. FRI layers (FriProver::build_layers), folding factor 16. Layers stay
  // coset-sharded while each rank's Merkle range has >= 16 rows per coset,
  // then are all-gathered and finished identically on every rank.
  L = 0;
  {
    uint64_t D = N, maxrem = (uint64_t)(o->fri_remainder_max_degree + 1) * B;
    while (D > maxrem) { D /= F; L++; }
  }
  layers.assign(L + 1, FriLayer{});
  dres = ctx->buf<unsigned long long>("grind_res", 1);
  {
    uint64_t tot_e = 0, D = N;
    for (uint32_t l = 0; l < L; l++) { tot_e += D / F; D /= F; }
    felt* fe = ctx->buf<felt>("fri_evals", tot_e + 1);
    const felt* deps = fold_constants(ctx);
    felt* E = deep;
    uint64_t m = n, eo = 0;
    uint32_t Bc = Bl, jc = j0;
    bool sh = R > 1;
    D = N;
    felt off = g;
    auto replicate = [&](uint32_t l) {  // all-gather the layer: rank blocks = coset blocks in order
      felt* full = ctx->buf<felt>("fri_full_" + std::to_string(l), (size_t)B * m);
      cm->all_gather(st, E, full, (size_t)Bl * m * 16);
      E = full;
      Bc = B;
      jc = 0;
      sh = false;
    };
    // Fiat-Shamir of the commit loop on the device: coin[0..8) = seed, then per
    // layer alpha (4 words) and root (8 words); no host round trip per layer
    uint32_t* coin_d = ctx->buf<uint32_t>("fri_coin", 8 + 12 * (size_t)(L + 1));
    felt* alphas_d = reinterpret_cast<felt*>(coin_d + 8);
    uint32_t* roots_d = coin_d + 8 + 4 * (size_t)L;
    HIP_CHECK(hipMemcpyAsync(coin_d, dt_seed, 32, hipMemcpyDeviceToDevice, st));  // device transcript
    // world 1 with a device remainder: the layers of <= 128 rows, their coin
    // steps and the remainder run as one single-block launch (k_fri_tail)
    static const bool no_fri_tail = getenv("ZKP_NO_FRI_TAIL") != nullptr;  // A/B switch
    const bool fuse_tail = R == 1 && o->grinding_factor > 0 && F == 16 && (N >> (4 * L)) <= 256 && !no_fri_tail;
    FriTailArgs fta{};
    for (uint32_t l = 0; l < L; l++) {
      const uint64_t m16 = m / F;
      if (sh && (m16 >> logR) < 16) replicate(l);
      FriLayer& ly = layers[l];
      ly.E = E; ly.m = m; ly.Bc = Bc; ly.jc = jc; ly.sharded = sh;
      if (fuse_tail && (m16 << logB) <= 128) {
        if (fta.nl >= FRI_TAIL_MAX) throw ZkpFail{ZKP_ERR_DEVICE, "FRI tail: too many small layers"};
        ly.tree.logR = 0;
        ly.tree.Lr = m16 << logB;
        ly.tree.nodes = ctx->buf<uint32_t>("ftree_" + std::to_string(l), (size_t)16 * ly.tree.Lr);
        ly.tree.top.assign(2, {});
        FriTailLayer& y = fta.ly[fta.nl++];
        y.E = E;
        y.nodes = ly.tree.nodes;
        y.logm16 = ilog2(m16);
        y.off_inv = inv(off);
        y.lev = ctx->itws(logN) + ((1ull << (ilog2(D) - 1)) - 1);  // as launch_fri_fold
        y.out = fe + eo;
        y.alpha_out = alphas_d + l;
        y.root_out = roots_d + 8 * (size_t)l;
        E = fe + eo;
        eo += (uint64_t)Bc * m16;
        m = m16;
        D /= F;
        off = pow_u64(off, F);
        continue;
      }
      if (fta.nl) throw ZkpFail{ZKP_ERR_DEVICE, "FRI tail: a large layer after a small one"};
      // sharded layers assemble the root on the host (top levels); it is staged back for the coin
      MerkleTail coin{};
      coin.op = MERKLE_TAIL_FRI_COIN;
      coin.coin_seed = coin_d;
      coin.alpha_out = alphas_d + l;
      coin.root_out = roots_d + 8 * (size_t)l;
      const bool coin_done = commit_rows(ctx, cm, 1, E, 0, F, logB, ilog2(m16), sh, "ftree_" + std::to_string(l),
                                         ly.tree, T.fri_roots[l], /*fetch_root=*/false, &coin);
      if (!coin_done)
        launch_coin_fri_layer(pf, st, coin_d, sh ? ly.tree.top_d + 8 : ly.tree.nodes + 8, alphas_d + l,
                              roots_d + 8 * (size_t)l);
      felt* nxt = fe + eo;
      launch_fri_fold(pf, st, E, m16, Bc, jc, logB, F, alphas_d + l, inv(off), ctx->itws(logN), ilog2(D), deps,
                      nxt);
      eo += (uint64_t)Bc * m16;
      E = nxt;
      m = m16;
      D /= F;
      off = pow_u64(off, F);
    }
    if (sh) replicate(L);
    layers[L].E = E; layers[L].m = m; layers[L].Bc = B; layers[L].jc = 0; layers[L].sharded = false;
    // small remainders: remainder, its commitment, the coin reseed and the first
    // grinding chunk run on the device too, so the round trip below also
    // returns the nonce (the host replays and checks all of it)
    const uint64_t Dlast = (uint64_t)B * m;
    dev_tail = Dlast <= 256 && o->grinding_factor > 0;
    if (fuse_tail && !dev_tail) throw ZkpFail{ZKP_ERR_DEVICE, "FRI tail fused without a device remainder"};
    // world 1: the whole query tail runs on the device too (grinding to completion,
    // query positions, every opening the batch proofs can need), so the proof has
    // a single host round trip, at its end
    dev_query = dev_tail && R == 1 && L <= GATHER_MAX_LAYERS;
    if (dev_tail) {
      rem_d = ctx->buf<felt>("rem_d", m + 1);
      rcommit_d = ctx->buf<uint32_t>("rem_commit", 8);
      if (fuse_tail) {
        fta.logB = logB;
        fta.coin_seed = coin_d;
        fta.eps_inv = deps;
        fta.rem_E = E;
        fta.rem_m = (uint32_t)m;
        fta.rem_off_inv = inv(off);
        fta.wd_inv = inv(root_of_unity(ilog2(Dlast)));
        fta.d_inv = inv(felt_u64(Dlast));
        fta.rem_out = rem_d;
        fta.commit_out = rcommit_d;
        launch_fri_tail(pf, st, fta);
      } else {
        launch_fri_remainder(pf, st, E, logB, (uint32_t)m, inv(off), inv(root_of_unity(ilog2(Dlast))),
                             inv(felt_u64(Dlast)), coin_d, rem_d, rcommit_d);
      }
      HIP_CHECK(hipMemsetAsync(dres, 0xff, 8, st));
      if (dev_query)
        launch_grind_all(pf, st, coin_d, 1, 1ull << 40, o->grinding_factor, dres);
      else
        launch_grind(pf, st, nullptr, coin_d, 1, grind_chunk, o->grinding_factor, dres);
    }
    if (dev_query) {
      dpos = ctx->buf<uint64_t>("query_pos", o->num_queries);
      launch_query_positions(pf, st, coin_d, dres, o->num_queries, N, dpos);
      ga.tlde = tlde; ga.clde = clde; ga.tnodes = ttree.nodes; ga.cnodes = ctree.nodes;
      ga.n = n; ga.w = w; ga.C = C; ga.logB = logB; ga.logN = logN; ga.nlayers = L;
      uint64_t off_w = 0;
      ga.seg_off[0] = 0;
      ga.rec_words[0] = 4 * (w + C) + 16 * logN;
      off_w += (uint64_t)o->num_queries * ga.rec_words[0];
      for (uint32_t l = 0; l < L; l++) {
        ga.E[l] = layers[l].E;
        ga.fnodes[l] = layers[l].tree.nodes;
        ga.m[l] = layers[l].m;
        ga.logrows[l] = logB + ilog2(layers[l].m / F);
        ga.seg_off[1 + l] = off_w;
        ga.rec_words[1 + l] = 64 + 8 * ga.logrows[l];
        off_w += (uint64_t)o->num_queries * ga.rec_words[1 + l];
      }
      full_h.resize(off_w);
      uint32_t* dfull = ctx->buf<uint32_t>("query_full", off_w + 4);
      if (gu_lazy_on) launch_gu_fill(pf, st, tlde, w, logn, logB, j0, logBl, dpos, o->num_queries, gu_lazy);
      launch_gather_full(pf, st, ga, o->num_queries, dpos, dfull);
      raw_pos.resize(o->num_queries);
      full_d = dfull;
    }
    return FriCursor{E, m, D, off, coin_d, alphas_d, roots_d};
  }
}

// the proof's host round trip and the replay of the device transcript
void ProofRun::fri_round_trip(const FriCursor& c) {
  late_pairs_upload();  // every kernel up to the query tail is queued: the host may block now
  felt* const E = c.E;
  const uint64_t m = c.m, D = c.D;
  const felt off = c.off;
  uint32_t* const coin_d = c.coin_d;
  felt* const alphas_d = c.alphas_d;
  uint32_t* const roots_d = c.roots_d;
  {
    // the proof's first host round trip: the device transcript so far (commitment
    // roots, coefficients, z, OOD frame, DEEP coefficients, FRI roots + alphas)
    // and the last FRI layer
    std::vector<uint8_t> rb((size_t)L * 32);
    std::vector<felt> dalpha(L);
    std::vector<felt> cm_vals((size_t)B * m);
    std::vector<felt> dcc(ncoef), dzz(2), hood((size_t)2 * (w + C)), hgam(w + C), hdk(4);
    std::vector<felt> drem(dev_tail ? m : 0);
    uint8_t roots[64], drcommit[32], dseed[32];
    std::vector<Fetch> fs = {{dalpha.data(), alphas_d, (size_t)L * 16}, {rb.data(), roots_d, (size_t)L * 32},
                             {cm_vals.data(), E, cm_vals.size() * 16}, {dcc.data(), dt_cc, (size_t)ncoef * 16},
                             {dzz.data(), dt_zz, 32}, {hood.data(), dv, hood.size() * 16},
                             {hgam.data(), dgam, hgam.size() * 16}, {hdk.data(), dk, 64},
                             {roots, troot_d, 32}, {roots + 32, croot_d, 32}};
    if (dev_tail) {
      fs.push_back({drem.data(), rem_d, drem.size() * 16});
      fs.push_back({drcommit, rcommit_d, 32});
      fs.push_back({dseed, coin_d, 32});
      fs.push_back({&dnonce, dres, 8});
    }
    if (dev_query) {
      fs.push_back({raw_pos.data(), dpos, raw_pos.size() * 8});
      fs.push_back({full_h.data(), full_d, full_h.size() * 4});
    }
    // sharded trees: their device-built top levels (the openings' host part)
    for (TreeShard* t : {&ttree, &ctree})
      if (t->top_d) fs.push_back({t->top.data(), t->top_d, t->top.size() * 32});
    for (uint32_t l = 0; l < L; l++)
      if (layers[l].tree.top_d) fs.push_back({layers[l].tree.top.data(), layers[l].tree.top_d, layers[l].tree.top.size() * 32});
    fetch_all(ctx, fs);
    memcpy(T.trace_root, roots, 32);
    memcpy(T.constraint_root, roots + 32, 32);
    if (R == 1) {
      memcpy(ttree.top[1].data(), T.trace_root, 32);
      memcpy(ctree.top[1].data(), T.constraint_root, 32);
    }
    // host replay of the device transcript, checked value by value
    bool same = true;
    coin.reseed(T.trace_root);
    std::vector<felt> cc = draw_coeffs(coin, o->batching_constraints, ncoef);
    for (uint32_t i = 0; i < ncoef && same; i++) same = eq(cc[i], dcc[i]);
    coin.reseed(T.constraint_root);
    const felt z = coin.draw(), zg = mul(z, wn_root);
    same = same && eq(z, dzz[0]) && eq(zg, dzz[1]);
    T.z.lo = z.lo; T.z.hi = z.hi;
    for (uint32_t c = 0; c < w; c++) { ood_trace[c] = hood[2 * c]; ood_trace[w + c] = hood[2 * c + 1]; }
    for (uint32_t h = 0; h < C; h++) ood_comp[h] = hood[2 * (w + h)];
    uint8_t dg[32];
    hash_elements(ood_trace.data(), ood_trace.size(), dg);
    coin.reseed(dg);
    hash_elements(ood_comp.data(), ood_comp.size(), dg);
    coin.reseed(dg);
    std::vector<felt> gam = draw_coeffs(coin, o->batching_deep, w + C);
    felt kz = zero(), kzg = zero();
    for (uint32_t c = 0; c < w; c++) { kz = add(kz, mul(gam[c], ood_trace[c])); kzg = add(kzg, mul(gam[c], ood_trace[w + c])); }
    for (uint32_t h = 0; h < C; h++) kz = add(kz, mul(gam[w + h], ood_comp[h]));
    for (uint32_t i = 0; i < w + C && same; i++) same = eq(gam[i], hgam[i]);
    same = same && eq(kz, hdk[2]) && eq(kzg, hdk[3]);
    if (!same) throw ZkpFail{ZKP_ERR_DEVICE, "device transcript diverged from the host (coefficients / z / DEEP)"};
    // host transcript replay (the proof's commitments and the coin state)
    for (uint32_t l = 0; l < L; l++) {
      memcpy(T.fri_roots[l], rb.data() + 32 * (size_t)l, 32);
      memcpy(layers[l].tree.top[1].data(), T.fri_roots[l], 32);
      coin.reseed(T.fri_roots[l]);
      felt alpha = coin.draw();
      if (!eq(alpha, dalpha[l])) throw ZkpFail{ZKP_ERR_DEVICE, "device FRI transcript diverged from the host"};
    }
    // remainder polynomial (FriProver::set_remainder): interpolate the last layer, keep D/B coefficients
    remainder.resize(D);
    for (uint64_t j = 0; j < B; j++)
      for (uint64_t t = 0; t < m; t++) remainder[j + B * t] = cm_vals[j * m + t];
    host_interpolate(remainder, off);
    remainder.resize(D / B);
    hash_elements(remainder.data(), remainder.size(), T.remainder_commitment);
    coin.reseed(T.remainder_commitment);
    if (dev_tail) {
      bool ok = memcmp(drcommit, T.remainder_commitment, 32) == 0 && memcmp(dseed, coin.seed, 32) == 0;
      for (size_t i = 0; i < drem.size() && ok; i++) ok = eq(drem[i], remainder[i]);
      if (!ok) throw ZkpFail{ZKP_ERR_DEVICE, "device remainder / grinding seed diverged from the host"};
    }
    T.num_fri_layers = L;
  }
}

void ProofRun::grind_stage() {
  nonce = 0;
  if (o->grinding_factor == 0) {
    nonce = 1;
  } else {
    uint32_t sw[8];
    for (int i = 0; i < 8; i++)
      sw[i] = (uint32_t)coin.seed[4 * i] | ((uint32_t)coin.seed[4 * i + 1] << 8) |
              ((uint32_t)coin.seed[4 * i + 2] << 16) | ((uint32_t)coin.seed[4 * i + 3] << 24);
    const uint64_t chunk = grind_chunk;
    uint64_t base0 = 1;
    if (dev_tail) {  // the first chunk ran on the device seed (checked equal to coin.seed above)
      if (dnonce != ~0ull) nonce = dnonce;
      base0 = 1 + chunk;
      if (dev_query && nonce == 0) throw ZkpFail{ZKP_ERR_NONCE, "nonce not found"};
      if (dev_query && coin.leading_zeros(nonce) < o->grinding_factor)
        throw ZkpFail{ZKP_ERR_DEVICE, "device grinding nonce fails the host check"};
    }
    for (uint64_t base = base0; nonce == 0; base += chunk) {
      unsigned long long init = ~0ull;
      ctx->upload(dres, &init, 8);
      launch_grind(pf, st, sw, nullptr, base, chunk, o->grinding_factor, dres);
      unsigned long long res;
      ctx->download(&res, dres, 8);
      if (res != ~0ull) nonce = res;
      if (base > (1ull << 40)) throw ZkpFail{ZKP_ERR_NONCE, "nonce not found"};
    }
  }
  T.pow_nonce = nonce;
  ctx->stage_end("6_grind");
}

// 9-10. query positions, openings, serialization (≙ Proof::to_bytes)
int ProofRun::finish(uint8_t** proof, uint64_t* proof_len, zkp_transcript* tr_out) {
  // 9. query positions
  std::vector<uint64_t> pos = coin.draw_integers(o->num_queries, N, nonce);
  if (dev_query && pos != raw_pos) throw ZkpFail{ZKP_ERR_DEVICE, "device query positions diverged from the host"};
  std::sort(pos.begin(), pos.end());
  pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
  const uint64_t np = pos.size();
  T.num_unique_queries = (uint32_t)np;
  for (uint64_t i = 0; i < np; i++) T.query_positions[i] = pos[i];
  T.num_composition_columns = C;

  Openings op;
  if (dev_query)
    openings_from_full(raw_pos, pos, full_h.data(), ga, layers, L, F, op);
  else {
    if (gu_lazy_on) {  // the lazy paired columns of the queried rows this rank holds
      uint64_t* dq = ctx->buf<uint64_t>("gu_fill_pos", np);
      ctx->upload(dq, pos.data(), np * 8);
      launch_gu_fill(pf, st, tlde, w, logn, logB, j0, logBl, dq, (uint32_t)np, gu_lazy);
    }
    gather_openings(ctx, cm, pos, n, logB, j0, tlde, w, ttree, clde, C, ctree, layers, L, F, op);
  }
  const uint64_t out_words = op.gathered.size();
  // 10. serialize (≙ Proof::to_bytes)
  Writer wr;
  wr.b.reserve((size_t)out_words * 4 + 64 * (size_t)(L + 4) + 32 * (size_t)(w + C) + 16 * remainder.size() + 4096);
  write_context(wr, air, o);
  wr.u8((uint8_t)np);
  wr.u16((uint16_t)(32 * (2 + L + 1)));
  wr.put(T.trace_root, 32);
  wr.put(T.constraint_root, 32);
  for (uint32_t l = 0; l < L; l++) wr.put(T.fri_roots[l], 32);
  wr.put(T.remainder_commitment, 32);
  wr.u8(1);
  op.write_commitment_queries(wr);
  wr.u16((uint16_t)(1 + 16 * 2 * w));
  wr.u8(2);
  for (felt v : ood_trace) wr.fe(v);
  wr.u16((uint16_t)(16 * C));
  for (felt v : ood_comp) wr.fe(v);
  wr.u8((uint8_t)L);
  op.write_fri_queries(wr);
  wr.u16((uint16_t)(16 * remainder.size()));
  for (felt v : remainder) wr.fe(v);
  wr.u8(1);
  wr.u64(nonce);
  wr.u8(0);

  ctx->stage_end("7_queries_serialize");
  ctx->collect_prof();
  ctx->free_retired();  // buffers a new shape outgrew (none on a warm shape)
  uint8_t* out = (uint8_t*)malloc(wr.b.size());
  if (!out) return ZKP_ERR_OOM;
  memcpy(out, wr.b.data(), wr.b.size());
  *proof = out;
  *proof_len = wr.b.size();
  if (tr_out) *tr_out = T;
  return 0;
}

// L_0 over this rank's LDE cosets (domain-only: cached per (n, B, j0, Bl))
const felt* ProofRun::l0_table() {
  const std::string key = "l0_" + std::to_string(logn) + "_" + std::to_string(logB) + "_" + std::to_string(j0) + "_" +
                          std::to_string(Bl);
  felt* t = ctx->buf<felt>(key, (size_t)Bl * n);
  if (!ctx->have_cached(key)) {
    const uint64_t count = (uint64_t)Bl * n;
    felt* scratch = ctx->buf<felt>("l0_scratch", l0_scratch_felts(count, logn));
    launch_l0_table(pf, st, PointMap{cx + j0, twn, logn}, count, inv(felt_u64(n)), t, scratch);
  }
  return t;
}

// host trace, paired: the paired columns [d, w) over PCIe and the check of their rows
// 1..n-1 on the copy stream (the trace commitment only needed their row 0)
void ProofRun::late_pairs_upload() {
  if (!late_h_trace) return;
  const uint32_t d = w / 2;
  HIP_CHECK(hipMemcpyAsync(const_cast<felt*>(d_trace) + (size_t)d * n, late_h_trace + (size_t)d * n,
                           (size_t)d * n * 16, hipMemcpyHostToDevice, ctx->copy));
  launch_gu_check(pf, ctx->copy, d_trace, d, logn, air.k, 0, d, 0, logn, nullptr, gu_bad);
  late_h_trace = nullptr;
  gu_late_check = true;
}

// the early trace check: its flag word to the host behind the check kernel, and the event
void ProofRun::early_check_launch(uint32_t* dflag, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(ctx->host_flag(), dflag, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipEventRecord(ctx->ev_check, s));
  pre_checked = true;
}

// the early check's flag (waits for the check kernel only: everything queued after it
// keeps the GPU busy meanwhile)
bool ProofRun::early_check_failed() {
  if (!pre_checked) return false;
  HIP_CHECK(hipEventSynchronize(ctx->ev_check));
  return *ctx->host_flag() != 0;
}

// a paired trace whose transitions did not hold (one 4-byte read after the proof's last kernels)
bool ProofRun::pair_failed() {
  if (!paired) return false;
  late_pairs_upload();  // (a proof whose FRI round trip did not issue it)
  if (gu_late_check) HIP_CHECK(hipStreamSynchronize(ctx->copy));
  std::vector<uint32_t> f(gu_flags ? 4 * (size_t)R : 4);
  ctx->download(f.data(), gu_flags ? gu_flags : gu_bad, f.size() * 4);
  for (uint32_t v : f)
    if (v) return true;
  return false;
}

// a derived last composition column whose dropped segments were not zero (the trace
// does not satisfy its constraints): one 16-byte read after the proof's last kernels
bool ProofRun::lastcol_failed() {
  if (!derive_last) return false;
  std::vector<uint32_t> f(lc_flags ? 4 * (size_t)R : 4);
  ctx->download(f.data(), lc_flags ? lc_flags : lc_bad, f.size() * 4);
  for (uint32_t v : f)
    if (v) return true;
  return false;
}

// h_trace (nullable): the trace is still in host memory and d_trace is its
// device buffer; the upload is pipelined with the trace interpolation and LDE
// by column groups (wide traces), so PCIe overlaps the first stage's kernels.
int prove_impl(zkp_ctx* ctx, zkp_comm* cm, int air_id, const felt* d_trace, uint32_t w, uint64_t n,
               const zkp_felt* pub_elems, uint64_t n_pub, const zkp_proof_options* o, uint8_t** proof,
               uint64_t* proof_len, zkp_transcript* tr_out, const zkp_felt* h_trace) {
  for (int attempt = 0;; attempt++) {
    ProofRun run(ctx, cm, o);
    run.allow_shortcuts = attempt == 0;
    int rc = run.init(air_id, d_trace, w, n, pub_elems, n_pub, proof, proof_len);
    if (rc) return rc;
    run.setup();
    run.trace_stage(h_trace);
    run.constraint_stage();
    run.ood_stage();
    run.deep_stage();
    run.fri_stage();
    run.grind_stage();
    // the paired columns and the derived composition column rest on the trace's
    // constraints: if they do not hold, prove the (now device-resident) trace again
    // without the shortcuts
    if (run.pair_failed() || run.lastcol_failed()) {
      if (!run.h_partial) h_trace = nullptr;  // resident from here
      continue;
    }
    return run.finish(proof, proof_len, tr_out);
  }
}

// every stream of the context idle: nothing queued by a failed call (a late
// upload, a check writing its flag, a column round) may run into the next call's
// buffers or outlive the context
void drain_streams(zkp_ctx* ctx) {
  (void)hipStreamSynchronize(ctx->copy);
  (void)hipStreamSynchronize(ctx->side);
  (void)hipStreamSynchronize(ctx->stream);
}

}  // namespace zkpi

void launch_fail(int code, const char* what) { throw ZkpFail{code, what}; }

namespace {
std::mutex g_stream_pool_mu;
std::map<int, std::vector<std::array<hipStream_t, 3>>> g_stream_pool;
constexpr size_t STREAM_POOL_MAX = 4;  // idle sets kept per device
}  // namespace

bool zkp_ctx::acquire_streams(int device, hipStream_t out[3]) {
  std::lock_guard<std::mutex> lk(g_stream_pool_mu);
  auto& v = g_stream_pool[device];
  if (v.empty()) return false;
  for (int i = 0; i < 3; i++) out[i] = v.back()[i];
  v.pop_back();
  return true;
}

void zkp_ctx::release_streams(int device, const hipStream_t s[3]) {
  for (int i = 0; i < 3; i++) (void)hipStreamSynchronize(s[i]);
  {
    std::lock_guard<std::mutex> lk(g_stream_pool_mu);
    auto& v = g_stream_pool[device];
    if (v.size() < STREAM_POOL_MAX) {
      v.push_back({s[0], s[1], s[2]});
      return;
    }
  }
  for (int i = 0; i < 3; i++) (void)hipStreamDestroy(s[i]);
}

// a context on `device` with its streams and events (nullptr on failure)
zkp_ctx* new_ctx(int device) {
  zkp_ctx* c = new (std::nothrow) zkp_ctx();
  if (!c) return nullptr;
  c->device = device;
  hipStream_t pooled[3];
  const bool reuse = zkp_ctx::acquire_streams(device, pooled);
  if (reuse) {
    c->stream = pooled[0];
    c->side = pooled[1];
    c->copy = pooled[2];
  }
  if ((!reuse && (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) != hipSuccess)) ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_check, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return nullptr;
  }
  // HIP binds a stream to a hardware queue at its first dispatch: do that here,
  // not inside the context's first proof (pooled streams are bound already)
  if (!reuse)
    for (hipStream_t s : {c->stream, c->side, c->copy}) warm_stream(s);
  return c;
}

// ====================================================================== C-ABI
extern "C" {

int zkp_prove_device(zkp_ctx* ctx, zkp_air_id air, const void* d_trace, uint32_t width, uint64_t n,
                     const zkp_felt* pub, uint64_t n_pub, const zkp_proof_options* opts, uint8_t** proof,
                     uint64_t* proof_len, zkp_transcript* transcript) {
  return guarded(ctx, [&] {
    ctx->err.clear();
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!d_trace) return (int)ZKP_ERR_ARGUMENT;
    return prove_impl(ctx, ctx->self_comm(), air, (const felt*)d_trace, width, n, pub, n_pub, opts, proof,
                      proof_len, transcript);
  });
}

int zkp_prove(zkp_ctx* ctx, zkp_air_id air, const zkp_felt* trace, uint32_t width, uint64_t n, const zkp_felt* pub,
              uint64_t n_pub, const zkp_proof_options* opts, uint8_t** proof, uint64_t* proof_len,
              zkp_transcript* transcript) {
  return guarded(ctx, [&] {
    ctx->err.clear();
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!trace) return (int)ZKP_ERR_ARGUMENT;
    if (n < 8 || (n & (n - 1)) || width == 0 || width > 255) return (int)ZKP_ERR_TRACE_SHAPE;
    felt* d = ctx->buf<felt>("trace_in", (size_t)width * n);
    return prove_impl(ctx, ctx->self_comm(), air, d, width, n, pub, n_pub, opts, proof, proof_len, transcript,
                      trace);
  });
}
}  // extern "C"
