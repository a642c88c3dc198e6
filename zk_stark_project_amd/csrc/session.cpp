// session.cpp — the stage sessions and the host channel of include/zkp.h.
#include "prover_internal.hpp"

using namespace zkpi;

// ====================================================================== stage sessions
// The stage entry points of include/zkp.h: one proof's
// device-resident state, driven stage by stage by a caller that keeps its own
// Fiat-Shamir channel (a winter-prover 0.12 fork keeping `Prover::prove`). The
// stages are zkp_prove's own (ProofRun in host-channel mode: grouped upload,
// GlobalUpdate column pairing, coefficient-form linear evaluation, the derived
// last composition column, coefficient-form DEEP for wide traces), with the coin
// draws coming from the caller. The shortcuts' device checks are read before the
// stage returns its root: a failed check redoes that stage without the shortcut,
// so every returned value is the one winterfell computes. World 1 (one GPU).
struct zkp_session {
  zkp_ctx* parent = nullptr;  // the caller's context (errors, kernel statistics)
  zkp_ctx* ctx = nullptr;     // this session's context (from the parent's pool)
  zkp_proof_options o{};
  std::unique_ptr<ProofRun> run;
  int air_id = 0;
  std::vector<zkp_felt> pub;
  uint32_t w = 0, B = 0, ce = 0, C = 0, F = 16, L = 0;
  uint32_t logn = 0, logB = 0, logN = 0;
  uint64_t n = 0, N = 0;
  int stage = 0;  // 1 trace committed, 2 evaluated, 3 composition committed, 4 OOD, 5 DEEP/FRI done
  std::vector<FriLayer> layers;
  felt z{}, zg{};
  std::vector<felt> ood;  // [2a + {0,1}]: array a (trace columns, then composition columns) at z, zg

  void begin(int need) {
    if (stage != need) throw ZkpFail{ZKP_ERR_ARGUMENT, "stage entry point called out of order"};
    HIP_CHECK(hipSetDevice(ctx->device));
    ctx->sync();
    ctx->ring_reset();
  }
  // a fresh ProofRun over the session's trace buffer, set up for host-channel stages
  void start_run(bool shortcuts) {
    run.reset(new ProofRun(ctx, ctx->self_comm(), &o));
    run->host_channel = true;
    run->allow_shortcuts = shortcuts;
    uint8_t* dummy = nullptr;
    uint64_t dlen = 0;
    felt* d = ctx->buf<felt>("trace_in", (size_t)w * n);
    const int rc = run->init(air_id, d, w, n, pub.data(), pub.size(), &dummy, &dlen);
    if (rc) throw ZkpFail{rc, "session: proof shape"};
    run->setup();
  }
};

// the host channel of include/zkp.h (zkp_channel_*)
struct zkp_channel {
  Coin coin;
  uint64_t lde_size = 0;
  uint32_t num_queries = 0;
};

namespace {

template <typename Fn>
int session_guard(zkp_session* s, Fn&& f) {
  if (!s) return ZKP_ERR_ARGUMENT;
  zkp_ctx* sc = s->ctx;
  sc->prof.enabled = s->parent->prof.enabled;
  sc->prof.only = s->parent->prof.only;
  const int rc = guarded(sc, [&] {
    sc->err.clear();
    int r = f();
    sc->collect_prof();
    return r;
  });
  // the caller reads errors and kernel statistics from its own context
  s->parent->err = sc->err;
  for (auto& kv : sc->stats) {
    auto& d = s->parent->stats[kv.first];
    d.launches += kv.second.launches;
    d.ms += kv.second.ms;
    d.bytes += kv.second.bytes;
  }
  sc->stats.clear();
  return rc;
}

void upload_felts(zkp_ctx* ctx, felt* d, const std::vector<felt>& h) { ctx->upload(d, h.data(), h.size() * 16); }

// the host channel's entry points allocate (felt vectors, query positions): no C++
// exception crosses the ABI, an allocation failure is ZKP_ERR_OOM
template <typename Fn>
int channel_guard(Fn&& f) {
  try {
    return f();
  } catch (const ZkpFail& e) {
    return e.code;
  } catch (const std::bad_alloc&) {
    return ZKP_ERR_OOM;
  } catch (...) {
    return ZKP_ERR_ARGUMENT;
  }
}

}  // namespace

extern "C" {

int zkp_session_create(zkp_ctx* ctx, zkp_air_id air_id, uint32_t width, uint64_t n, const zkp_felt* pub_elems,
                       uint64_t n_pub, const zkp_proof_options* o, zkp_session** out) {
  return guarded(ctx, [&] {
    if (!out) return (int)ZKP_ERR_ARGUMENT;
    *out = nullptr;
    int rc = check_options(o);
    if (rc) return rc;
    if (n < 8 || (n & (n - 1)) || width == 0 || width > 255) return (int)ZKP_ERR_TRACE_SHAPE;
    if (n_pub && !pub_elems) return (int)ZKP_ERR_ARGUMENT;
    std::vector<felt> pub(n_pub);
    for (uint64_t i = 0; i < n_pub; i++) pub[i] = make(pub_elems[i].lo, pub_elems[i].hi);
    AirDesc air;
    rc = build_air(air, air_id, width, n, pub);
    if (rc) return rc;
    auto s = std::make_unique<zkp_session>();
    s->parent = ctx;
    s->o = *o;
    s->air_id = air_id;
    s->pub.assign(pub_elems, pub_elems + n_pub);
    s->w = width; s->n = n; s->B = o->blowup_factor; s->F = o->fri_folding_factor;
    s->ce = air.ce_blowup(); s->C = air.comp_cols();
    if (s->B < s->ce) return (int)ZKP_ERR_INVALID_OPTIONS;
    if (s->ce > 16 || s->C > s->ce) return (int)ZKP_ERR_UNSUPPORTED_AIR;
    s->logn = ilog2(n); s->logB = ilog2(s->B); s->logN = s->logn + s->logB;
    s->N = n << s->logB;
    if (s->logN > MAX_LOG_DOMAIN || s->logn > MAX_LOG_TRACE) return (int)ZKP_ERR_TRACE_SHAPE;
    uint64_t D = s->N, maxrem = (uint64_t)(o->fri_remainder_max_degree + 1) * s->B;
    while (D > maxrem) { D /= s->F; s->L++; }
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!ctx->session_pool.empty()) {
      s->ctx = ctx->session_pool.back();
      ctx->session_pool.pop_back();
    } else {
      s->ctx = new_ctx(ctx->device);
      if (!s->ctx) return (int)ZKP_ERR_DEVICE;
    }
    *out = s.release();
    return 0;
  });
}

void zkp_session_destroy(zkp_session* s) {
  if (!s) return;
  s->run.reset();
  if (s->ctx) {
    (void)hipSetDevice(s->ctx->device);
    drain_streams(s->ctx);
    s->ctx->err.clear();
    // one idle session context is kept (buffers and domain tables reused by the next
    // session); more would each hold a proof's HBM until zkp_ctx_destroy
    if (s->parent->session_pool.empty()) {
      s->parent->session_pool.push_back(s->ctx);
    } else {
      delete s->ctx;
    }
  }
  delete s;
}

int zkp_session_shape(const zkp_session* s, uint32_t* ce, uint32_t* num_columns, uint32_t* fri_layers) {
  if (!s) return ZKP_ERR_ARGUMENT;
  if (ce) *ce = s->ce;
  if (num_columns) *num_columns = s->C;
  if (fri_layers) *fri_layers = s->L;
  return ZKP_OK;
}

// ≙ Prover::new_trace_lde + the trace commitment (DefaultTraceLde::new)
int zkp_session_trace_lde(zkp_session* s, const zkp_felt* trace_cols, uint8_t root[32]) {
  return session_guard(s, [&] {
    if (!trace_cols || !root) return (int)ZKP_ERR_ARGUMENT;
    s->begin(0);
    s->start_run(true);
    s->run->trace_stage(trace_cols);
    // GlobalUpdate pairing: the check of every row (the late host columns joined)
    // before the root is returned; a failed check extends every column instead
    if (s->run->pair_failed()) {
      s->start_run(false);
      s->run->trace_stage(s->run->h_partial ? trace_cols : nullptr);
    }
    memcpy(root, s->run->T.trace_root, 32);
    s->stage = 1;
    return 0;
  });
}

// ≙ new_evaluator(..).evaluate: the caller's composition coefficients
int zkp_eval_constraints(zkp_session* s, const zkp_felt* coeffs, uint32_t n_coeffs, zkp_felt* evals_out) {
  return session_guard(s, [&] {
    if (!coeffs) return (int)ZKP_ERR_ARGUMENT;
    s->begin(1);
    ProofRun& r = *s->run;
    if (n_coeffs != r.ncoef) return (int)ZKP_ERR_ARGUMENT;
    s->ctx->upload(r.dt_cc, coeffs, (size_t)n_coeffs * 16);
    r.eval_stage();
    if (evals_out) {  // CE-coset-major on the device -> natural CE domain order
      std::vector<felt> h((size_t)s->ce * s->n);
      s->ctx->download(h.data(), r.comp, h.size() * 16);
      for (uint32_t u = 0; u < s->ce; u++)
        for (uint64_t t = 0; t < s->n; t++) {
          const felt v = h[(size_t)u * s->n + t];
          evals_out[u + (size_t)s->ce * t] = zkp_felt{v.lo, v.hi};
        }
    }
    s->ctx->sync();
    s->stage = 2;
    return 0;
  });
}

// ≙ build_constraint_commitment (CompositionPoly::new + DefaultConstraintCommitment);
// evals (nullable): the caller's own evaluations in natural CE-domain order
int zkp_composition_commit(zkp_session* s, const zkp_felt* evals, uint8_t root[32], uint32_t* num_columns) {
  return session_guard(s, [&] {
    if (!root) return (int)ZKP_ERR_ARGUMENT;
    if (evals && s->stage == 1) s->stage = 2;  // caller-evaluated constraints (natural CE order)
    s->begin(2);
    ProofRun& r = *s->run;
    const uint64_t n = s->n;
    const uint32_t ce = s->ce;
    if (evals) {
      std::vector<felt> h((size_t)ce * n);
      for (uint32_t u = 0; u < ce; u++)
        for (uint64_t t = 0; t < n; t++) {
          const zkp_felt& v = evals[u + (size_t)ce * t];
          h[(size_t)u * n + t] = make(v.lo, v.hi);
          if (ge_p(h[(size_t)u * n + t])) throw ZkpFail{ZKP_ERR_ARGUMENT, "non-canonical evaluation"};
        }
      upload_felts(s->ctx, s->ctx->buf<felt>("comp", (size_t)ce * n), h);
    }
    r.composition_stage();
    // the derived last column holds only if the dropped segments are zero: else
    // the composition is committed again with the column extended
    if (r.lastcol_failed()) {
      r.allow_shortcuts = false;
      r.composition_stage();
    }
    memcpy(root, r.T.constraint_root, 32);
    if (num_columns) *num_columns = s->C;
    s->stage = 3;
    return 0;
  });
}

int zkp_ood_frame(zkp_session* s, zkp_felt zf, zkp_felt* trace_ood, zkp_felt* comp_ood) {
  return session_guard(s, [&] {
    if (!trace_ood || !comp_ood) return (int)ZKP_ERR_ARGUMENT;
    s->begin(3);
    ProofRun& r = *s->run;
    s->z = make(zf.lo, zf.hi);
    if (ge_p(s->z)) return (int)ZKP_ERR_ARGUMENT;
    s->zg = mul(s->z, root_of_unity(s->logn));
    std::vector<felt> pw(2 * (size_t)s->logn), zz = {s->z, s->zg};
    felt a = s->z, b = s->zg;
    for (uint32_t l = 0; l < s->logn; l++) { pw[l] = a; pw[s->logn + l] = b; a = sqr(a); b = sqr(b); }
    upload_felts(s->ctx, r.dt_pw, pw);
    upload_felts(s->ctx, r.dt_zz, zz);
    r.ood_values();
    s->ood.resize(2 * (size_t)(s->w + s->C));
    s->ctx->download(s->ood.data(), r.dv, s->ood.size() * 16);
    for (uint32_t c = 0; c < s->w; c++) {
      trace_ood[c] = zkp_felt{s->ood[2 * c].lo, s->ood[2 * c].hi};
      trace_ood[s->w + c] = zkp_felt{s->ood[2 * c + 1].lo, s->ood[2 * c + 1].hi};
    }
    for (uint32_t h = 0; h < s->C; h++) comp_ood[h] = zkp_felt{s->ood[2 * (s->w + h)].lo, s->ood[2 * (s->w + h)].hi};
    s->stage = 4;
    return 0;
  });
}

int zkp_deep_fri(zkp_session* s, const zkp_felt* deep_coeffs, zkp_fri_channel channel, void* user,
                 zkp_felt* remainder, uint64_t* remainder_len, uint8_t remainder_commitment[32]) {
  return session_guard(s, [&] {
    if (!deep_coeffs || !channel || !remainder_len || !remainder_commitment) return (int)ZKP_ERR_ARGUMENT;
    s->begin(4);
    zkp_ctx* ctx = s->ctx;
    ProofRun& r = *s->run;
    Prof& pf = ctx->prof;
    hipStream_t st = ctx->stream;
    const uint32_t w = s->w, C = s->C, B = s->B, F = s->F;
    const uint64_t n = s->n;
    const felt g = felt_u64(3);
    // DEEP coefficients and the OOD combinations kz = sum gamma_i T_i(z) (+ composition), kzg
    std::vector<felt> gam(w + C), dkh(4);
    for (uint32_t i = 0; i < w + C; i++) gam[i] = make(deep_coeffs[i].lo, deep_coeffs[i].hi);
    felt kz = zero(), kzg = zero();
    for (uint32_t c = 0; c < w; c++) {
      kz = add(kz, mul(gam[c], s->ood[2 * c]));
      kzg = add(kzg, mul(gam[c], s->ood[2 * c + 1]));
    }
    for (uint32_t h = 0; h < C; h++) kz = add(kz, mul(gam[w + h], s->ood[2 * (w + h)]));
    dkh[0] = s->z; dkh[1] = s->zg; dkh[2] = kz; dkh[3] = kzg;
    r.dgam = ctx->buf<felt>("gamma", w + C);
    r.dk = ctx->buf<felt>("dt_dk", 4);
    upload_felts(ctx, r.dgam, gam);
    upload_felts(ctx, r.dk, dkh);
    r.deep_stage();
    // FriProver::build_layers: commit each layer, the caller's channel returns alpha, fold
    s->layers.assign(s->L + 1, FriLayer{});
    uint64_t tot = 0, D = s->N;
    for (uint32_t l = 0; l < s->L; l++) { tot += D / F; D /= F; }
    felt* fe = ctx->buf<felt>("fri_evals", tot + 1);
    felt* alphas = ctx->buf<felt>("alphas", s->L + 1);
    const felt* deps = fold_constants(ctx);
    felt* E = r.deep;
    uint64_t m = n, eo = 0;
    felt off = g;
    D = s->N;
    for (uint32_t l = 0; l < s->L; l++) {
      const uint64_t m16 = m / F;
      FriLayer& ly = s->layers[l];
      ly.E = E; ly.m = m; ly.Bc = B; ly.jc = 0; ly.sharded = false;
      uint8_t root[32];
      commit_rows(ctx, ctx->self_comm(), 1, E, 0, F, s->logB, ilog2(m16), false, "ftree_" + std::to_string(l),
                  ly.tree, root);
      zkp_felt af{0, 0};
      if (channel(user, l, root, &af) != 0) throw ZkpFail{ZKP_ERR_ARGUMENT, "FRI channel callback failed"};
      felt alpha = make(af.lo, af.hi);
      if (ge_p(alpha)) throw ZkpFail{ZKP_ERR_ARGUMENT, "non-canonical FRI alpha"};
      ctx->upload(alphas + l, &alpha, 16);
      felt* nxt = fe + eo;
      launch_fri_fold(pf, st, E, m16, B, 0, s->logB, F, alphas + l, inv(off), ctx->itws(s->logN), ilog2(D), deps, nxt);
      eo += (uint64_t)B * m16;
      E = nxt;
      m = m16;
      D /= F;
      off = pow_u64(off, F);
    }
    s->layers[s->L].E = E; s->layers[s->L].m = m; s->layers[s->L].Bc = B;
    // FriProver::set_remainder: interpolate the last layer (coset-major -> natural), keep D/B coefficients
    std::vector<felt> last((size_t)B * m), rem(D);
    ctx->download(last.data(), E, last.size() * 16);
    for (uint64_t j = 0; j < B; j++)
      for (uint64_t t = 0; t < m; t++) rem[j + B * t] = last[j * m + t];
    host_interpolate(rem, off);
    rem.resize(D / B);
    hash_elements(rem.data(), rem.size(), remainder_commitment);
    if (remainder) {
      if (*remainder_len < rem.size()) return (int)ZKP_ERR_ARGUMENT;
      for (size_t i = 0; i < rem.size(); i++) remainder[i] = zkp_felt{rem[i].lo, rem[i].hi};
    }
    *remainder_len = rem.size();
    s->stage = 5;
    return 0;
  });
}

int zkp_query(zkp_session* s, const uint64_t* positions, uint64_t n_positions, uint8_t** out, uint64_t* out_len) {
  return session_guard(s, [&] {
    if (!positions || !out || !out_len || n_positions == 0 || n_positions > 255) return (int)ZKP_ERR_ARGUMENT;
    s->begin(5);
    std::vector<uint64_t> pos(positions, positions + n_positions);
    for (uint64_t i = 0; i < n_positions; i++)
      if (pos[i] >= s->N || (i && pos[i] <= pos[i - 1])) return (int)ZKP_ERR_ARGUMENT;  // sorted, unique, in range
    zkp_ctx* ctx = s->ctx;
    ProofRun& r = *s->run;
    if (r.gu_lazy_on) {  // the lazy paired columns of the queried rows
      uint64_t* dq = ctx->buf<uint64_t>("gu_fill_pos", pos.size());
      ctx->upload(dq, pos.data(), pos.size() * 8);
      launch_gu_fill(ctx->prof, ctx->stream, r.tlde, s->w, s->logn, s->logB, 0, s->logB, dq, (uint32_t)pos.size(),
                     r.gu_lazy);
    }
    Openings op;
    gather_openings(ctx, ctx->self_comm(), pos, s->n, s->logB, 0, r.tlde, s->w, r.ttree, r.clde, s->C, r.ctree,
                    s->layers, s->L, s->F, op);
    Writer wr;
    wr.u8(1);  // one trace segment
    op.write_commitment_queries(wr);
    wr.u8((uint8_t)s->L);
    op.write_fri_queries(wr);
    uint8_t* p = (uint8_t*)malloc(wr.b.size());
    if (!p) return (int)ZKP_ERR_OOM;
    memcpy(p, wr.b.data(), wr.b.size());
    *out = p;
    *out_len = wr.b.size();
    s->stage = 5;  // queries may be asked again (e.g. after a re-grind)
    return 0;
  });
}

// ---- host channel (≙ ProverChannel over DefaultRandomCoin<Blake3_256>)
int zkp_channel_create(zkp_air_id air_id, uint32_t width, uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
                       const zkp_proof_options* o, zkp_channel** out) {
  if (!out) return ZKP_ERR_ARGUMENT;
  *out = nullptr;
  try {
    int rc = check_options(o);
    if (rc) return rc;
    if (n < 8 || (n & (n - 1)) || width == 0 || width > 255) return ZKP_ERR_TRACE_SHAPE;
    if (n_pub && !pub_elems) return ZKP_ERR_ARGUMENT;
    std::vector<felt> pub(n_pub);
    for (uint64_t i = 0; i < n_pub; i++) pub[i] = make(pub_elems[i].lo, pub_elems[i].hi);
    AirDesc air;
    rc = build_air(air, air_id, width, n, pub);
    if (rc) return rc;
    auto ch = std::make_unique<zkp_channel>();
    std::vector<felt> se = context_elements(air, o);
    se.insert(se.end(), pub.begin(), pub.end());
    ch->coin.init(se);
    ch->lde_size = n * o->blowup_factor;
    ch->num_queries = o->num_queries;
    *out = ch.release();
    return ZKP_OK;
  } catch (const ZkpFail& e) {
    return e.code;
  } catch (...) {
    return ZKP_ERR_OOM;
  }
}

void zkp_channel_destroy(zkp_channel* ch) { delete ch; }

int zkp_channel_commit(zkp_channel* ch, const uint8_t root[32]) {
  if (!ch || !root) return ZKP_ERR_ARGUMENT;
  return channel_guard([&] {
    ch->coin.reseed(root);
    return (int)ZKP_OK;
  });
}

int zkp_channel_commit_felts(zkp_channel* ch, const zkp_felt* els, uint64_t n) {
  if (!ch || (n && !els)) return ZKP_ERR_ARGUMENT;
  return channel_guard([&] {
    std::vector<felt> v(n);
    for (uint64_t i = 0; i < n; i++) v[i] = make(els[i].lo, els[i].hi);
    uint8_t d[32];
    hash_elements(v.data(), v.size(), d);
    ch->coin.reseed(d);
    return (int)ZKP_OK;
  });
}

int zkp_channel_draw(zkp_channel* ch, uint32_t method, uint32_t count, zkp_felt* out) {
  if (!ch || !out || method > ZKP_BATCHING_HORNER) return ZKP_ERR_ARGUMENT;
  return channel_guard([&] {
    if (count == 0) {
      const felt v = ch->coin.draw();
      out[0] = zkp_felt{v.lo, v.hi};
      return (int)ZKP_OK;
    }
    const std::vector<felt> v = draw_coeffs(ch->coin, method, count);
    for (uint32_t i = 0; i < count; i++) out[i] = zkp_felt{v[i].lo, v[i].hi};
    return (int)ZKP_OK;
  });
}

int zkp_channel_seed(const zkp_channel* ch, uint8_t seed[32]) {
  if (!ch || !seed) return ZKP_ERR_ARGUMENT;
  memcpy(seed, ch->coin.seed, 32);
  return ZKP_OK;
}

int zkp_channel_query_positions(zkp_channel* ch, uint64_t nonce, uint64_t* out, uint32_t* n_unique) {
  if (!ch || !out || !n_unique) return ZKP_ERR_ARGUMENT;
  return channel_guard([&] {
    std::vector<uint64_t> pos = ch->coin.draw_integers(ch->num_queries, ch->lde_size, nonce);
    std::sort(pos.begin(), pos.end());
    pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
    for (size_t i = 0; i < pos.size(); i++) out[i] = pos[i];
    *n_unique = (uint32_t)pos.size();
    return (int)ZKP_OK;
  });
}

}  // extern "C"
