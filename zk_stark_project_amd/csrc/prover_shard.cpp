// prover_shard.cpp — one proof over several GPUs: the sharded
// commitments and the multi-GPU entry points of include/zkp.h (zkp_prove_sharded,
// zkp_comm_*). A rank owns a slice of the LDE cosets; the exchanges run over the
// group's zkp_comm (RCCL over xGMI, the in-process group, or a caller transport).
#include "prover_internal.hpp"

using namespace zkpi;

namespace zkpi {

// the sharded tree of commit_rows: rank s hashes its own rows into per-destination
// blocks, a leaf-digest all-to-all (side stream, in chunks behind the hashing) gives
// it the contiguous leaf range [s*L/R, (s+1)*L/R), it builds that subtree, and the
// top log2(R) levels are built on every rank from the all-gathered subtree roots
bool commit_rows_sharded(zkp_ctx* ctx, zkp_comm* cm, int mode, const felt* src, uint64_t n, uint32_t cols,
                         uint32_t logB, uint32_t logrows, const std::string& name, TreeShard& tr, uint8_t root[32],
                         bool fetch_root, const MerkleTail* coin, const LastCol* lc, const GuLazy* gl) {
  Prof& pf = ctx->prof;
  hipStream_t st = ctx->stream;
  const uint32_t R = cm->world, logR = ilog2(R), logBl = logB - logR;
  const uint32_t logrr = logrows - logR;
  tr.logR = logR;
  tr.Lr = 1ull << (logB + logrr);
  uint32_t* send = ctx->buf<uint32_t>("shard_send", (size_t)8 << (logBl + logrows));
  uint32_t* recv = ctx->buf<uint32_t>("shard_recv", (size_t)8 << (logBl + logrows));
  // the leaf-digest all-to-all in K chunks on the side stream, chunk k's exchange
  // overlapping the hashing of chunk k+1 (every hash launch is queued before the
  // first collective, so host-synchronous transports overlap too)
  // 4 chunks (1, 2, 8 and 16 measured no better: profiles/r03_ab_shard_logk.txt)
  const uint32_t logK = logrr >= 12 ? 2u : 0u, K = 1u << logK;
  const size_t chunk_words = (size_t)8 << (logBl + logrows - logK), block = (size_t)32 << (logBl + logrr - logK);
  ctx->events(K + 1);
  for (uint32_t k = 0; k < K; k++) {
    launch_leaf_hash_shard(pf, st, mode, src, n, cols, logBl, logrows, logrr, logK, k, send + k * chunk_words, lc,
                           gl);
    HIP_CHECK(hipEventRecord(ctx->up_ev[k], st));
  }
  for (uint32_t k = 0; k < K; k++) {
    HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->up_ev[k], 0));
    cm->all_to_all(ctx->side, send + k * chunk_words, recv + k * chunk_words, block);
  }
  HIP_CHECK(hipEventRecord(ctx->up_ev[K], ctx->side));
  HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[K], 0));
  tr.nodes = ctx->buf<uint32_t>(name, (size_t)16 * tr.Lr);
  uint32_t* done = ctx->buf<uint32_t>("merkle_done", 1);
  if (!ctx->have_cached("merkle_done")) HIP_CHECK(hipMemsetAsync(done, 0, 4, st));
  launch_merkle_from_shards(pf, st, recv, logB, logrr, logK, tr.nodes, done);
  // the top levels on the device from the all-gathered subtree roots: the coin
  // kernels read the root there, and the host fetches tr.top with the transcript
  // (fetch_root = false) instead of a round trip per commitment
  uint32_t* roots = ctx->buf<uint32_t>("shard_roots", (size_t)8 * R);
  cm->all_gather(st, tr.nodes + 8, roots, 32);
  tr.top_d = ctx->buf<uint32_t>(name + "_top", (size_t)16 * R);
  launch_shard_top(pf, st, roots, R, tr.top_d, coin);  // + the coin step, as a world-1 tree's last block
  tr.top.assign(2 * R, {});
  if (fetch_root) {
    ctx->download(tr.top.data(), tr.top_d, (size_t)64 * R);
    memcpy(root, tr.top[1].data(), 32);
  }
  return coin && coin->op != MERKLE_TAIL_NONE;
}

// the OOD of ood_launch split by blocks: each rank evaluates 1/R of every array's
// blocks (the partial Horner sums of SURVEY §8(e)(4)), the rank blocks are
// all-gathered (narrays * nb * 32 bytes in all) and every rank combines them
felt* ood_launch_sharded(zkp_ctx* ctx, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn,
                         const felt* dpw, zkp_comm* cm, felt* part, felt* dv) {
  const uint32_t logE = logn < 11 ? logn : 11, nb = 1u << (logn - logE), R = (uint32_t)cm->world;
  const felt ninv = inv(felt_u64(1ull << logn));
  const uint32_t nbl = nb / R;
  felt* mine = ctx->buf<felt>("ood_part_rank", (size_t)2 * narrays * nbl);
  launch_eval_bitrev_blocks(ctx->prof, ctx->stream, arrays, narrays, ntwo, logn, dpw, dpw + logn,
                            (uint32_t)cm->rank * nbl, nbl, mine);
  cm->all_gather(ctx->stream, mine, part, (size_t)2 * narrays * nbl * 16);
  launch_eval_bitrev_tail(ctx->prof, ctx->stream, part, narrays, logn, nbl, dpw, dpw + logn, ninv, dv);
  return dv;
}


// ---- the sharded exchanges of ProofRun's stages

// trace_stage, wide traces over R ranks (cpt columns per rank, `wi` of the w columns
// interpolated, d = w / 2 when GlobalUpdate-paired)
void ProofRun::trace_column_sharded(const zkp_felt* h_trace, uint32_t cpt, uint32_t wi, uint32_t d) {
  // column-sharded interpolation: in round k rank r interpolates
  // columns [k*R*cpr + r*cpr, +cpr) — uploading only those columns of a host
  // trace — and round k's coefficient all-gather (side stream) lands its R*cpr
  // columns in order at coef + k*R*cpr*n while the main stream extends round
  // k - 1's columns on this rank's cosets. Nothing but coefficients crosses xGMI.
  // rounds: the most that divide cpt, up to 6 — only round 0's exchange is
  // exposed (C5 at R = 8: 4 rounds of 2 of the 64 paired-trace columns per rank,
  // 16 columns per LDE; unpaired 5 rounds of 3)
  uint32_t K = 6;
  while (cpt % K) K--;
  const uint32_t cpr = cpt / K;
  felt* own = ctx->buf<felt>("coef_own", (size_t)cpt * n);
  ctx->events(3 * (size_t)K);
  // the copy stream starts after everything already queued on the main stream
  HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
  HIP_CHECK(hipStreamWaitEvent(ctx->copy, ctx->ev_fork, 0));
  HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  // per round k: upload (host traces) + interpolation on the copy stream, the
  // coefficient all-gather on the side stream, the coset LDE on the main stream;
  // a pageable upload holds the host, and by then round k-1's LDE is queued
  for (uint32_t k = 0; k < K; k++) {
    const uint64_t cown = (uint64_t)k * R * cpr + (uint64_t)rank * cpr, c0 = (uint64_t)k * R * cpr;
    felt* dcol = const_cast<felt*>(d_trace) + cown * n;
    if (h_trace) {
      HIP_CHECK(hipMemcpyAsync(dcol, h_trace + cown * n, (size_t)cpr * n * 16, hipMemcpyHostToDevice, ctx->copy));
      h_partial = true;
    }
    NttBatch ib{dcol, own + (size_t)k * cpr * n, nullptr, n, n, 1, 1, cpr};
    launch_ntt(pf, ctx->copy, ib, logn, false, ctx->itws(logN), logN);
    HIP_CHECK(hipEventRecord(ctx->up_ev[k], ctx->copy));
    HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->up_ev[k], 0));
    cm->all_gather(ctx->side, own + (size_t)k * cpr * n, coef + c0 * n, (size_t)cpr * n * 16);
    HIP_CHECK(hipEventRecord(ctx->up_ev[K + k], ctx->side));
    HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[K + k], 0));
    NttBatch lb{coef + c0 * n, tlde + c0 * Bl * n, Sj0, n, n, Bl, Bl, R * cpr * Bl};
    launch_ntt(pf, st, lb, logn, true, ctx->tws(logN), logN);
  }
  // nothing on the copy stream may outlive the stage (the next proof reuses its buffers)
  HIP_CHECK(hipEventRecord(ctx->up_ev[2 * K], ctx->copy));
  HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[2 * K], 0));
  if (paired && wi < w) {
    // derived columns [wi, w) from [i0, i0 + np): each rank checks its 1/R of the
    // rows (the flags are all-gathered; every rank computes c_i from row 0), derives
    // the coefficients its consumers read (the OOD blocks and the lincombs take
    // the positions [rank*nR, +nR) when the OOD is split, else all) and the LDE
    // of its cosets from its own extended columns
    const uint32_t i0 = wi - d, np = w - wi;
    const uint64_t nR = n >> logR;
    launch_gu_check(pf, st, d_trace, d, logn, air.k, i0, np, (uint64_t)rank * nR, logn - logR, gu_cval, gu_bad);
    if (rank) launch_gu_check(pf, st, d_trace, d, logn, air.k, i0, np, 0, 0, gu_cval, gu_bad);
    gu_flags = ctx->buf<uint32_t>("gu_flags", 4 * (size_t)R);
    cm->all_gather(st, gu_bad, gu_flags, 16);
    const bool slice = (n >> std::min(logn, 11u)) >= R;  // ood_launch splits its blocks
    launch_gu_coef(pf, st, coef, d, logn, air.k, ctx->itws(logN) + ((n >> 1) - 1), i0, np,
                   slice ? (uint64_t)rank * nR : 0, slice ? nR : n, gu_cval);
    if (!gu_lazy_on) launch_gu_lde(pf, st, tlde, d, logn, logBl, air.k, i0, np, gu_cval, l0_table());
  } else {
    paired = false;
    gu_lazy_on = false;
  }
}

// trace_stage, a narrow host trace over R ranks: returns nullptr (the trace is
// resident on every rank afterwards)
const zkp_felt* ProofRun::gather_host_slices(const zkp_felt* h_trace) {
  // sharded host trace: each rank uploads only its 1/R row
  // slice of every column over PCIe; the slices are all-gathered over the
  // comm (xGMI) into the whole trace on every rank, which then interpolates it
  const uint64_t nR = n >> logR;
  felt* dfull = const_cast<felt*>(d_trace);
  felt* slice = ctx->buf<felt>("trace_slice", (size_t)w * nR);
  HIP_CHECK(hipMemcpy2DAsync(slice, nR * 16, h_trace + (size_t)rank * nR, n * 16, nR * 16, w,
                             hipMemcpyHostToDevice, st));
  if (w == 1) {
    cm->all_gather(st, slice, dfull, nR * 16);
  } else {  // rank blocks [s][col][nR] -> column-major [col][s*nR + t]
    felt* gat = ctx->buf<felt>("trace_gather", (size_t)w * n);
    cm->all_gather(st, slice, gat, (size_t)w * nR * 16);
    for (uint32_t sr = 0; sr < R; sr++)
      HIP_CHECK(hipMemcpy2DAsync(dfull + (size_t)sr * nR, n * 16, gat + (size_t)sr * w * nR, nR * 16, nR * 16, w,
                                 hipMemcpyDeviceToDevice, st));
  }
  return nullptr;
}

// composition_stage: the all-to-all of the CE cosets' interpolated position slices
// (`cint`: this rank's CE cosets); returns the receive buffer k_comp_dft reads
felt* ProofRun::composition_exchange(felt* cint, uint64_t nR) {
  // send block s = positions [s*nR, (s+1)*nR) of every owned CE coset
  felt* send = ctx->buf<felt>("comp_send", (size_t)celmax * n);
  felt* recv = ctx->buf<felt>("comp_recv", (size_t)celmax * n);
  for (uint32_t ul = 0; ul < cel; ul++)
    HIP_CHECK(hipMemcpy2DAsync(send + (size_t)ul * nR, (size_t)celmax * nR * 16, cint + (size_t)ul * n, nR * 16,
                               nR * 16, R, hipMemcpyDeviceToDevice, st));
  cm->all_to_all(st, send, recv, (size_t)celmax * nR * 16);
  return recv;
}

// composition_stage: the coefficient columns' all-gather (this rank's position slice
// [p0, p0 + nR) of each, in `slice`) and their coset LDE
void ProofRun::composition_gather_lde(felt* slice, bool derive, uint64_t nR, uint64_t p0) {
  // column by column: the all-gather of coefficient column m (rank s's slice of
  // positions [s*nR, (s+1)*nR) lands at acoef + m*n + s*nR, i.e. the column in
  // order) runs on the side stream while the column before it is extended
  // (the largest exchange of a sharded proof, hidden behind the
  // composition LDE). The extensions alternate between the main and the copy stream:
  // one column's batch-1 passes (2048 blocks at C4) leave the last of their ~1.6 rounds
  // of blocks part-empty, and the next column's blocks fill it
  ctx->events(C + 1);
  HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
  HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
  HIP_CHECK(hipStreamWaitEvent(ctx->copy, ctx->ev_fork, 0));
  bool on_copy = false;
  // a derived last column (LastCol) is never extended: only the OOD reads its
  // coefficients, and a split OOD reads exactly this rank's slice of them
  const bool ood_split = (n >> std::min(logn, 11u)) >= R;  // ood_launch splits its blocks
  for (uint32_t m = 0; m < C; m++) {
    if (derive && ood_split && m == C - 1) {
      HIP_CHECK(hipMemcpyAsync(acoef + (size_t)m * n + p0, slice + (size_t)m * nR, nR * 16,
                               hipMemcpyDeviceToDevice, st));
      break;
    }
    cm->all_gather(ctx->side, slice + (size_t)m * nR, acoef + (size_t)m * n, nR * 16);
    HIP_CHECK(hipEventRecord(ctx->up_ev[m], ctx->side));
    if (derive && m == C - 1) {  // derived in the leaf pass (the OOD still reads its coefficients)
      HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[m], 0));
      break;
    }
    hipStream_t ls = (m & 1) ? ctx->copy : st;
    on_copy = on_copy || ls == ctx->copy;
    HIP_CHECK(hipStreamWaitEvent(ls, ctx->up_ev[m], 0));
    NttBatch lb{acoef + (size_t)m * n, clde + (size_t)m * Bl * n, Sj0, n, n, Bl, Bl, Bl};
    launch_ntt(pf, ls, lb, logn, true, ctx->tws(logN), logN);
  }
  if (on_copy) {  // the copy stream's columns (and through them their gathers) before anything reads clde
    HIP_CHECK(hipEventRecord(ctx->up_ev[C], ctx->copy));
    HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[C], 0));
  }
}

}  // namespace zkpi

extern "C" {

int zkp_prove_sharded(zkp_ctx* ctx, zkp_comm* comm, zkp_air_id air, const zkp_felt* trace, uint32_t width,
                      uint64_t n, const zkp_felt* pub, uint64_t n_pub, const zkp_proof_options* opts, uint8_t** proof,
                      uint64_t* proof_len, zkp_transcript* transcript) {
  int rc = guarded(ctx, [&] {
    ctx->err.clear();
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!trace || !comm) return (int)ZKP_ERR_ARGUMENT;
    if (n < 8 || (n & (n - 1)) || width == 0 || width > 255) return (int)ZKP_ERR_TRACE_SHAPE;
    felt* d = ctx->buf<felt>("trace_in", (size_t)width * n);
    return prove_impl(ctx, comm, air, d, width, n, pub, n_pub, opts, proof, proof_len, transcript, trace);
  });
  // a rank that fails (argument checks included) releases peers blocked in a collective
  if (rc && comm) comm->abort();
  return rc;
}

int zkp_prove_sharded_device(zkp_ctx* ctx, zkp_comm* comm, zkp_air_id air, const void* d_trace, uint32_t width,
                             uint64_t n, const zkp_felt* pub, uint64_t n_pub, const zkp_proof_options* opts,
                             uint8_t** proof, uint64_t* proof_len, zkp_transcript* transcript) {
  int rc = guarded(ctx, [&] {
    ctx->err.clear();
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!d_trace || !comm) return (int)ZKP_ERR_ARGUMENT;
    return prove_impl(ctx, comm, air, (const felt*)d_trace, width, n, pub, n_pub, opts, proof, proof_len,
                      transcript);
  });
  if (rc && comm) comm->abort();
  return rc;
}

int zkp_comm_local_group(int world, zkp_comm** comms) {
  if (!comms || world < 1 || world > 64) return ZKP_ERR_ARGUMENT;
  try {
    make_local_group(world, comms);
  } catch (...) {
    return ZKP_ERR_OOM;
  }
  return ZKP_OK;
}

int zkp_comm_rccl_unique_id(uint8_t id[128]) {
  if (!id) return ZKP_ERR_ARGUMENT;
  try {
    rccl_unique_id(id);
  } catch (...) {
    return ZKP_ERR_DEVICE;
  }
  return ZKP_OK;
}

int zkp_comm_rccl_create(zkp_ctx* ctx, const uint8_t id[128], int world, int rank, zkp_comm** out) {
  return guarded(ctx, [&] {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return (int)ZKP_ERR_ARGUMENT;
    *out = make_rccl_comm(ctx->device, id, world, rank);
    return 0;
  });
}

int zkp_comm_host_create(int world, int rank, const zkp_host_transport* t, zkp_comm** out) {
  if (!t || !out || !t->all_to_all || !t->all_gather || world < 1 || world > 64 || rank < 0 || rank >= world)
    return ZKP_ERR_ARGUMENT;
  try {
    *out = make_host_comm(world, rank, *t);
  } catch (...) {
    return ZKP_ERR_OOM;
  }
  return ZKP_OK;
}

void zkp_comm_destroy(zkp_comm* comm) { delete comm; }

int zkp_comm_check(zkp_ctx* ctx, zkp_comm* comm, uint64_t block_bytes, double* a2a_ms, double* ag_ms) {
  int rc = guarded(ctx, [&] {
    ctx->err.clear();
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!comm || block_bytes == 0 || (block_bytes & 3)) return (int)ZKP_ERR_ARGUMENT;
    const uint32_t W = (uint32_t)comm->world, me = (uint32_t)comm->rank;
    const uint64_t words = block_bytes / 4;
    // rank-tagged words: tag(src, dst, i); dst = W marks the all-gather block
    auto tag = [](uint32_t src, uint32_t dst, uint64_t i) {
      return ((src + 1) * 0x9E3779B1u) ^ ((dst + 7) * 0x85EBCA77u) ^ ((uint32_t)i * 0xC2B2AE3Du) ^ (uint32_t)(i >> 32);
    };
    std::vector<uint32_t> h((size_t)W * words);
    for (uint32_t s = 0; s < W; s++)
      for (uint64_t i = 0; i < words; i++) h[s * words + i] = tag(me, s, i);
    uint32_t* send = ctx->buf<uint32_t>("cc_send", (size_t)W * words);
    uint32_t* recv = ctx->buf<uint32_t>("cc_recv", (size_t)W * words);
    ctx->upload(send, h.data(), h.size() * 4);
    ctx->sync();
    auto timed = [&](bool a2a) {
      double best = 1e30;
      for (int it = 0; it < 2; it++) {  // the first round also sets up the transport's connections
        HIP_CHECK(hipMemsetAsync(recv, 0, (size_t)W * block_bytes, ctx->stream));
        ctx->sync();
        auto t0 = std::chrono::steady_clock::now();
        if (a2a) comm->all_to_all(ctx->stream, send, recv, block_bytes);
        else comm->all_gather(ctx->stream, send, recv, block_bytes);
        ctx->sync();
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      }
      ctx->download(h.data(), recv, h.size() * 4);
      for (uint32_t s = 0; s < W; s++)
        for (uint64_t i = 0; i < words; i++)
          if (h[s * words + i] != (a2a ? tag(s, me, i) : tag(s, 0, i)))
            throw ZkpFail{ZKP_ERR_DEVICE, std::string(a2a ? "all_to_all" : "all_gather") + ": block from rank " +
                                              std::to_string(s) + " differs at word " + std::to_string(i)};
      return best;
    };
    // the all-gather sends block 0 of `send`, i.e. tag(me, 0, i)
    const double ta = timed(true), tg = timed(false);
    if (a2a_ms) *a2a_ms = ta;
    if (ag_ms) *ag_ms = tg;
    return 0;
  });
  if (rc && comm) comm->abort();
  return rc;
}

int zkp_comm_rank(const zkp_comm* comm) { return comm ? comm->rank : -1; }
int zkp_comm_world(const zkp_comm* comm) { return comm ? comm->world : -1; }

int zkp_comm_backend_world(const zkp_comm* comm) { return comm ? comm->backend_world() : -1; }

}  // extern "C"
