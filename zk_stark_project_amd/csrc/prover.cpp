// prover.cpp — host orchestration of the MI355X STARK prover + the C-ABI of
// include/zkp.h.
//
// Mirrors winterfell 0.12 `Prover::generate_proof` (the path selected by the
// reference's plug-ins, src/aggregation/prover.rs:194-248): channel seeding,
// trace LDE + commitment, constraint evaluation, composition commitment, OOD,
// DEEP, FRI, grinding, queries, serialization. Every O(n) stage runs on the
// GPU (kernels.hip); the host only drives the Fiat-Shamir transcript and
// assembles the proof bytes from the few values the verifier needs.
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/zkp.h"
#include "blake3.hpp"
#include "comm.hpp"
#include "zkp_internal.hpp"

using namespace fp;

#include "host_stark.hpp"

using namespace zkh;

namespace {

#define HIP_CHECK(x)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess)                                                                          \
      throw ZkpFail{e_ == hipErrorOutOfMemory ? ZKP_ERR_OOM : ZKP_ERR_DEVICE,                      \
                    std::string(#x) + ": " + hipGetErrorString(e_)};                               \
  } while (0)


}  // namespace

// ====================================================================== context
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct zkp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // side stream: work that only needs domain data runs there while the main
  // stream waits on a host round trip (ordered back in with events)
  hipStream_t side = nullptr;
  // copy stream: a sharded wide trace's column uploads and interpolations, ahead
  // of the main stream's coset LDEs (ordered in with events)
  hipStream_t copy = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  Prof prof;
  std::string err;
  std::map<std::string, DevBuf> bufs;
  struct Stat {
    uint64_t launches = 0;
    double ms = 0, bytes = 0;
  };
  std::map<std::string, Stat> stats;
  std::vector<void*> user_allocs;
  // pinned host staging (fast small H2D/D2H transfers)
  void* pinned_p = nullptr;
  size_t pinned_bytes = 0;
  void* pinned(size_t bytes) {
    if (pinned_bytes < bytes) {
      if (pinned_p) HIP_CHECK(hipHostFree(pinned_p));
      pinned_p = nullptr;
      size_t nb = bytes < (1u << 20) ? (1u << 20) : bytes;
      HIP_CHECK(hipHostMalloc(&pinned_p, nb, hipHostMallocDefault));
      pinned_bytes = nb;
    }
    return pinned_p;
  }

  template <typename T>
  T* buf(const std::string& name, size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 16;
    DevBuf& b = bufs[name];
    if (b.bytes < bytes) {
      if (b.p) HIP_CHECK(hipFree(b.p));
      b.p = nullptr;
      HIP_CHECK(hipMalloc(&b.p, bytes));
      b.bytes = bytes;
    }
    return reinterpret_cast<T*>(b.p);
  }
  void sync() { HIP_CHECK(hipStreamSynchronize(stream)); }
  // true if `key` was already produced by an earlier call (the caller fills it otherwise)
  std::map<std::string, bool> cached;
  std::map<std::string, std::vector<felt>> host_cache;  // domain-only host values
  bool have_cached(const std::string& key) {
    bool had = cached[key];
    cached[key] = true;
    return had;
  }
  // small uploads are staged in a pinned ring that is only reset between proofs
  // (the stream is in order, so a slot is never overwritten while in flight)
  uint8_t* ring_p = nullptr;
  size_t ring_cap = 0, ring_off = 0;
  void ring_reset() { ring_off = 0; }
  void upload(void* d, const void* h, size_t bytes) {
    if (bytes > (1u << 20)) {
      HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream));
      return;
    }
    if (!ring_p) {
      ring_cap = 8u << 20;
      HIP_CHECK(hipHostMalloc((void**)&ring_p, ring_cap, hipHostMallocDefault));
    }
    size_t need = (bytes + 255) & ~(size_t)255;
    if (ring_off + need > ring_cap) {  // wrap: wait until earlier copies are done
      sync();
      ring_off = 0;
    }
    memcpy(ring_p + ring_off, h, bytes);
    HIP_CHECK(hipMemcpyAsync(d, ring_p + ring_off, bytes, hipMemcpyHostToDevice, stream));
    ring_off += need;
  }
  void download(void* h, const void* d, size_t bytes) {
    if (bytes > (1u << 20)) {
      HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream));
      sync();
      return;
    }
    void* hp = pinned(bytes);
    HIP_CHECK(hipMemcpyAsync(hp, d, bytes, hipMemcpyDeviceToHost, stream));
    sync();
    memcpy(h, hp, bytes);
  }
  // host-side stage clock (profiling only): adds wall ms per stage as "host_<stage>"
  std::chrono::steady_clock::time_point stage_t0;
  void stage_begin() { if (prof.enabled) stage_t0 = std::chrono::steady_clock::now(); }
  void stage_end(const char* name) {
    if (!prof.enabled) return;
    auto t = std::chrono::steady_clock::now();
    auto& s = stats[std::string("host_") + name];
    s.launches += 1;
    s.ms += std::chrono::duration<double, std::milli>(t - stage_t0).count();
    stage_t0 = t;
  }
  void collect_prof() {
    if (prof.pending.empty()) return;
    sync();
    // ZKP_TIMELINE=1: per-launch (start, duration, gap to the previous launch) of
    // this call on stderr, relative to its first launch (diagnostics only)
    static const bool timeline = getenv("ZKP_TIMELINE") != nullptr;
    if (timeline) {
      const hipEvent_t t0 = prof.pending.front().start;
      float prev_end = 0;
      for (auto& r : prof.pending) {
        float st = 0, en = 0;
        (void)hipEventElapsedTime(&st, t0, r.start);
        (void)hipEventElapsedTime(&en, t0, r.stop);
        fprintf(stderr, "TL %-18s start %8.3f dur %7.3f gap %7.3f\n", r.name, st, en - st, st - prev_end);
        prev_end = en;
      }
      fprintf(stderr, "TL end\n");
    }
    for (auto& r : prof.pending) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, r.start, r.stop));
      auto& s = stats[r.name];
      s.launches += 1;
      s.ms += ms;
      s.bytes += r.bytes;
      prof.pool.push_back(r.start);
      prof.pool.push_back(r.stop);
    }
    prof.pending.clear();
  }

  // ---- stage-major twiddle tables for domain 2^logN: level t (t < logN) holds
  // w_{2^(t+1)}^(+-j), j < 2^t, at [2^t - 1, 2^(t+1) - 1). Level logN-1 is
  // w_N^(+-e), e < N/2 (the x-coordinate table of the LDE domain).
  std::map<uint32_t, bool> have_tw;
  void ensure_twiddles(uint32_t logN) {
    if (have_tw[logN]) return;
    uint64_t half = 1ull << (logN - 1);
    for (int dir = 0; dir < 2; dir++) {
      felt w = root_of_unity(logN);
      if (dir) w = inv(w);
      std::vector<felt> lo(2048), hi((half + 2047) / 2048 + 1);
      lo[0] = one();
      for (int i = 1; i < 2048; i++) lo[i] = mul(lo[i - 1], w);
      felt step = mul(lo[2047], w);
      hi[0] = one();
      for (size_t i = 1; i < hi.size(); i++) hi[i] = mul(hi[i - 1], step);
      felt* dlo = buf<felt>("tmp_lo", lo.size());
      felt* dhi = buf<felt>("tmp_hi", hi.size());
      upload(dlo, lo.data(), lo.size() * 16);
      upload(dhi, hi.data(), hi.size() * 16);
      felt* t = buf<felt>((dir ? "itw_" : "tw_") + std::to_string(logN), 2 * half);
      launch_expand_powers(prof, stream, t + (half - 1), half, dlo, dhi);
      if (logN > 1) launch_build_levels(prof, stream, t, logN - 1);
      sync();
    }
    have_tw[logN] = true;
  }
  // stage-major tables (NTT kernels, FRI fold)
  felt* tws(uint32_t logN) { return reinterpret_cast<felt*>(bufs["tw_" + std::to_string(logN)].p); }
  felt* itws(uint32_t logN) { return reinterpret_cast<felt*>(bufs["itw_" + std::to_string(logN)].p); }
  // top level: w_N^e, e < N/2 (x-coordinates)
  felt* tw(uint32_t logN) { return tws(logN) + ((1ull << (logN - 1)) - 1); }
  felt* itw(uint32_t logN) { return itws(logN) + ((1ull << (logN - 1)) - 1); }

  // ---- coset tables for (n, B, ce): S[j*n + p] = n^-1 (g w_N^j)^rev(p) (LDE cosets j < B);
  // Si[u*n + p] = (g w_M^u)^-rev(p) (CE cosets u < ce, M = n*ce)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, bool> have_coset;
  void ensure_coset(uint32_t logn, uint32_t logB, uint32_t logce) {
    auto key = std::make_tuple(logn, logB, logce);
    if (have_coset[key]) return;
    uint32_t logN = logn + logB;
    ensure_twiddles(logN);
    uint64_t n = 1ull << logn;
    felt g = felt_u64(3);
    for (int dir = 0; dir < 2; dir++) {
      felt base = dir ? inv(g) : g;
      std::vector<felt> lo(2048), hi(n / 2048 + 2);
      lo[0] = one();
      for (int i = 1; i < 2048; i++) lo[i] = mul(lo[i - 1], base);
      felt step = mul(lo[2047], base);
      hi[0] = one();
      for (size_t i = 1; i < hi.size(); i++) hi[i] = mul(hi[i - 1], step);
      felt* dlo = buf<felt>("tmp_lo", lo.size());
      felt* dhi = buf<felt>("tmp_hi", hi.size());
      upload(dlo, lo.data(), lo.size() * 16);
      upload(dhi, hi.data(), hi.size() * 16);
      std::string sfx = std::to_string(logn) + "_" + std::to_string(logB);
      if (dir == 0) {
        felt* S = buf<felt>("S_" + sfx, n << logB);
        launch_build_coset_scale(prof, stream, S, logn, 1u << logB, tw(logN), logN, dlo, dhi, inv(felt_u64(n)));
      } else {
        const uint32_t logM = logn + logce;
        felt* Si = buf<felt>("Si_" + sfx + "_" + std::to_string(logce), n << logce);
        launch_build_coset_scale(prof, stream, Si, logn, 1u << logce, itws(logN) + ((1ull << (logM - 1)) - 1), logM,
                                 dlo, dhi, one());
      }
      sync();
    }
    have_coset[key] = true;
  }
  felt* S(uint32_t logn, uint32_t logB) {
    return reinterpret_cast<felt*>(bufs["S_" + std::to_string(logn) + "_" + std::to_string(logB)].p);
  }
  felt* Si(uint32_t logn, uint32_t logB, uint32_t logce) {
    return reinterpret_cast<felt*>(
        bufs["Si_" + std::to_string(logn) + "_" + std::to_string(logB) + "_" + std::to_string(logce)].p);
  }

  // release the buffers whose names start with `prefix` (a stage session's state)
  void drop(const std::string& prefix) {
    sync();
    for (auto it = bufs.begin(); it != bufs.end();) {
      if (it->first.compare(0, prefix.size(), prefix) == 0) {
        if (it->second.p) HIP_CHECK(hipFree(it->second.p));
        it = bufs.erase(it);
      } else {
        ++it;
      }
    }
    for (auto it = cached.begin(); it != cached.end();)
      it = it->first.compare(0, prefix.size(), prefix) == 0 ? cached.erase(it) : std::next(it);
  }
  // stage sessions run on contexts of their own (own streams and buffers, so a
  // session's state survives zkp_prove calls on this context between its stages);
  // idle ones are kept here with their domain tables for the next session
  std::vector<zkp_ctx*> session_pool;
  std::vector<hipEvent_t> up_ev;  // pipeline events (column-group uploads, per-column all-gathers)
  void events(size_t k) {  // grows only: events already recorded may still be waited on
    while (up_ev.size() < k) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      up_ev.push_back(e);
    }
  }

  zkp_comm* self = nullptr;
  zkp_comm* self_comm() {
    if (!self) self = make_self_comm();
    return self;
  }

  ~zkp_ctx() {
    delete self;
    for (auto& kv : bufs)
      if (kv.second.p) (void)hipFree(kv.second.p);
    for (void* p : user_allocs) (void)hipFree(p);
    if (pinned_p) (void)hipHostFree(pinned_p);
    if (ring_p) (void)hipHostFree(ring_p);
    for (auto e : prof.pool) (void)hipEventDestroy(e);
    for (auto e : up_ev) (void)hipEventDestroy(e);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (copy) (void)hipStreamDestroy(copy);
    if (side) (void)hipStreamDestroy(side);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// ------------------------------------------------------------------ sharded commitments
// A Merkle tree over LDE-domain rows. When the rows are sharded over R ranks,
// rank s builds the subtree of the leaf range [s*L/R, (s+1)*L/R) in `nodes`
// and every rank holds the top log2(R) levels on the host (`top`, heap
// layout with top[1] = root and top[R + s] = subtree root of rank s).
struct TreeShard {
  uint32_t* nodes = nullptr;  // device subtree (nodes[1..2Lr)), or the whole tree when logR == 0
  uint64_t Lr = 0;
  uint32_t logR = 0;
  std::vector<std::array<uint8_t, 32>> top;
  uint32_t* top_d = nullptr;  // sharded: top[1..2R) on the device (root at top_d + 8)
  // global node k -> host digest (top levels) or (owner rank, local node index)
  struct Loc {
    bool host;
    uint32_t owner;
    uint64_t local;
  };
  Loc locate(uint64_t k) const {
    uint32_t d = 63 - __builtin_clzll(k);
    if (d <= logR && logR > 0) return {true, 0, k};
    uint32_t below = d - logR;
    uint64_t s = (k >> below) - (1ull << logR);
    return {false, (uint32_t)s, (1ull << below) + (k & ((1ull << below) - 1))};
  }
};

// commit the rows of a coset-major source held by this rank (cosets [j0, j0+Bl)):
// mode 0 = LDE rows (cols columns, n rows per coset), mode 1 = FRI rows (16
// values, 2^logrows rows per coset). Unsharded sources hold all B cosets.
// Unsharded trees finish in the last block of their top launch (MerkleTail);
// sharded trees in k_shard_top over the all-gathered subtree roots. With coin
// (coefficients, z or a FRI layer's alpha) that block also runs the coin step,
// and the function returns true when it did.
bool commit_rows(zkp_ctx* ctx, zkp_comm* cm, int mode, const felt* src, uint64_t n, uint32_t cols, uint32_t logB,
                 uint32_t logrows, bool sharded, const std::string& name, TreeShard& tr, uint8_t root[32],
                 bool fetch_root = true, const MerkleTail* coin = nullptr, const LastCol* lc = nullptr,
                 const GuLazy* gl = nullptr) {
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
  const uint32_t R = cm->world, logR = ilog2(R), logBl = logB - logR;
  const uint32_t logrr = logrows - logR;
  tr.logR = logR;
  tr.Lr = 1ull << (logB + logrr);
  uint32_t* send = ctx->buf<uint32_t>("shard_send", (size_t)8 << (logBl + logrows));
  uint32_t* recv = ctx->buf<uint32_t>("shard_recv", (size_t)8 << (logBl + logrows));
  // the leaf-digest all-to-all in K chunks on the side stream, chunk k's exchange
  // overlapping the hashing of chunk k+1 (every hash launch is queued before the
  // first collective, so host-synchronous transports overlap too)
  static const int logK_env = getenv("ZKP_SHARD_LOGK") ? atoi(getenv("ZKP_SHARD_LOGK")) : -1;  // A/B switch
  const uint32_t logK = logrr >= 12 ? (logK_env >= 0 && logK_env <= 4 ? (uint32_t)logK_env : 2u) : 0u, K = 1u << logK;
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

// evaluate bit-reversed coefficient arrays (scaled by n) at x0, x1 -> values (x n^-1)
// a device -> host copy folded into a round trip
struct Fetch {
  void* host;
  const void* dev;
  size_t bytes;
};

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
                 const felt* dpw, zkp_comm* cm = nullptr) {
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
  const uint32_t nbl = nb / R;
  felt* mine = ctx->buf<felt>("ood_part_rank", (size_t)2 * narrays * nbl);
  launch_eval_bitrev_blocks(ctx->prof, ctx->stream, arrays, narrays, ntwo, logn, dpw, dpw + logn,
                            (uint32_t)cm->rank * nbl, nbl, mine);
  cm->all_gather(ctx->stream, mine, part, (size_t)2 * narrays * nbl * 16);
  launch_eval_bitrev_tail(ctx->prof, ctx->stream, part, narrays, logn, nbl, dpw, dpw + logn, ninv, dv);
  return dv;
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
                     const felt* dt_aval, const felt* tlde, felt* comp, const felt* coef = nullptr,
                     zkp_comm* cm = nullptr) {
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
  static const bool pointwise = getenv("ZKP_EVAL_POINTWISE") != nullptr;
  const bool coef_form = air.id != ZKP_AIR_MIMC && coef && !pointwise;
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

// DEEP composition evaluations over the rank's cosets [j0, j0 + Bl) (coset-major).
// Narrow traces: pointwise k_deep over every trace and composition column's LDE.
// Wide traces (w >= DEEP_COEF_MIN_W): winterfell's own dataflow
// — the gamma-combination of the trace polynomials in coefficient form
// (k_deep_lincomb over `coef`, read once), its coset LDE, then k_deep over that one
// column and the composition columns with coefficients [1 | delta]: w column reads
// per LDE point become one (C3: 8.2 GB -> ~1 GB per proof). Same field values.
constexpr uint32_t DEEP_COEF_MIN_W = 16;
// Sharded, each rank combines 1/R of the positions and the combined column is
// all-gathered (n * 16 bytes in all) instead of every rank reading all w columns.
void deep_evaluations(zkp_ctx* ctx, zkp_comm* cm, hipStream_t st, DeepArgs da, const felt* coef, uint64_t n,
                      const felt* Sj0, uint32_t logN, felt* out) {
  static const bool pointwise_only = getenv("ZKP_DEEP_POINTWISE") != nullptr;  // A/B switch
  if (da.w < DEEP_COEF_MIN_W || pointwise_only) {
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

// one FRI layer as the prover holds it: coset-major evaluations of the cosets
// [jc, jc + Bc) (m positions each), and its (possibly sharded) Merkle tree
struct FriLayer {
  felt* E = nullptr;
  uint64_t m = 0;
  uint32_t Bc = 0, jc = 0;
  bool sharded = false;
  TreeShard tree;
};

// Query openings of one proof: trace and constraint rows + their batch Merkle
// paths, FRI layer rows + paths, gathered from device memory (from the owning
// rank when sharded) and written in the proof's wire format (Queries /
// FriProof of winterfell's Proof::to_bytes).
struct Openings {
  std::vector<uint32_t> gathered;
  std::vector<GatherSeg> segs;
  BatchPlan bt;               // trace and constraint trees (same shape and positions)
  std::vector<BatchPlan> bf;  // FRI layer trees
  size_t cursor = 0;
  // values and batch paths are written straight from the gathered words
  // (felts are stored canonical LE, i.e. already in their wire format)
  void write_values(Writer& wr) {
    const GatherSeg& gs = segs[cursor++];
    wr.u32((uint32_t)(gs.count * 16));
    wr.put(gathered.data() + gs.out_off, gs.count * 16);
  }
  void write_batch(Writer& wr, const BatchPlan& bp) {
    const GatherSeg& gs = segs[cursor++];
    const uint32_t* d = gathered.data() + gs.out_off;
    size_t nodes = 0;
    for (auto& p : bp.paths) nodes += p.size();
    wr.u32((uint32_t)(2 + bp.paths.size() + 32 * nodes));
    wr.u8((uint8_t)bp.depth);
    wr.u8((uint8_t)bp.paths.size());
    size_t k = 0;
    for (auto& p : bp.paths) {
      wr.u8((uint8_t)p.size());
      wr.put(d + 8 * k, 32 * p.size());
      k += p.size();
    }
  }
  // trace + constraint queries: values and batch paths of each commitment
  void write_commitment_queries(Writer& wr) {
    cursor = 0;
    for (int seg = 0; seg < 2; seg++) {
      write_values(wr);
      write_batch(wr, bt);
    }
  }
  // FRI proof layers (values + batch paths per layer), after the commitment queries
  void write_fri_queries(Writer& wr) {
    cursor = 4;
    for (const BatchPlan& b : bf) {
      write_values(wr);
      write_batch(wr, b);
    }
  }
};

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

// where the FRI layer loop left off: the last layer (E: m per coset, D values
// in all, domain offset off) and the device coin / alphas / roots
struct FriCursor {
  felt* E;
  uint64_t m, D;
  felt off;
  uint32_t* coin_d;
  felt* alphas_d;
  uint32_t* roots_d;
};

// One proof (prove_impl): the shapes, device buffers, commitments and transcript
// that its stages share. Each stage method is one step of the reference's
// Prover::prove (winter-prover 0.12 generate_proof); what a later
// step reads is a member, everything else stays local to its stage.
struct ProofRun {
  zkp_ctx* ctx;
  zkp_comm* cm;
  const zkp_proof_options* o;
  hipStream_t st;
  Prof& pf;
  // shapes; coset sharding: rank r owns the LDE cosets [j0, j0 + Bl)
  uint32_t w = 0, B = 0, F = 0, logn = 0, logB = 0, logN = 0, R = 1, rank = 0, logR = 0, Bl = 0, logBl = 0, j0 = 0;
  uint64_t n = 0, N = 0;
  std::vector<felt> pub;
  AirDesc air;
  // CE cosets: CE coset u lives in LDE coset u << cstep; this rank evaluates [u0, u0 + cel)
  uint32_t ce = 0, C = 0, logce = 0, cstep = 0, u0 = 0, cel = 0, celmax = 0;
  felt g{};
  zkp_transcript T;
  Coin coin;
  // device transcript and domain tables
  uint32_t ncoef = 0;
  uint32_t* dt_seed = nullptr;
  felt *dt_cc = nullptr, *dt_zz = nullptr, *dt_pw = nullptr, *dt_aval = nullptr;
  const felt* Sj0 = nullptr;
  felt* cx = nullptr;
  const felt* twn = nullptr;
  // trace, composition, OOD, DEEP
  const felt* d_trace = nullptr;
  felt *coef = nullptr, *tlde = nullptr, *comp = nullptr, *acoef = nullptr, *clde = nullptr;
  TreeShard ttree, ctree;
  const uint32_t *troot_d = nullptr, *croot_d = nullptr;
  felt wn_root{};
  felt *deep_binv = nullptr, *dv = nullptr, *dgam = nullptr, *dk = nullptr, *deep = nullptr;
  PointMap deep_pm{};
  std::vector<felt> ood_trace, ood_comp;  // filled by the host replay of the FRI round trip
  // FRI, grinding, queries
  uint32_t L = 0;
  std::vector<FriLayer> layers;
  std::vector<felt> remainder;
  bool dev_tail = false;   // remainder + first grinding chunk on the device
  bool dev_query = false;  // ... and the whole query tail (world 1)
  FullGatherArgs ga{};
  uint64_t* dpos = nullptr;
  const uint32_t* full_d = nullptr;
  std::vector<uint32_t> full_h;
  std::vector<uint64_t> raw_pos;
  felt* rem_d = nullptr;
  uint32_t* rcommit_d = nullptr;
  unsigned long long* dres = nullptr;
  unsigned long long dnonce = ~0ull;
  static constexpr uint64_t grind_chunk = 1ull << 22;
  uint64_t nonce = 0;
  // exact shortcuts whose result rests on the trace satisfying its constraints
  // (GlobalUpdate column pairing, the derived last composition column): the first
  // attempt takes them and checks on the device; a failed check proves again without
  bool allow_shortcuts = true;
  // GlobalUpdate column pairing (trace_stage)
  bool paired = false;
  felt* gu_cval = nullptr;
  uint32_t* gu_bad = nullptr;    // this rank's check flag (4 words)
  uint32_t* gu_flags = nullptr;  // column-sharded: every rank's flags (all-gathered)
  bool gu_lazy_on = false;       // the paired LDE columns are derived in the row hash and for the queried rows only
  bool gu_late_check = false;    // host trace: the paired columns' upload and check still run on the copy stream
  const zkp_felt* late_h_trace = nullptr;  // host trace whose paired columns late_pairs_upload() still has to send
  void late_pairs_upload();
  GuLazy gu_lazy{};
  const felt* l0_table();
  bool pair_failed();
  // derived last composition column (LastCol, constraint_stage): the segments that
  // CompositionPoly::new drops must be zero (k_comp_dft raises lc_bad otherwise)
  bool derive_last = false;
  uint32_t* lc_bad = nullptr;    // this rank's flag (4 words)
  uint32_t* lc_flags = nullptr;  // sharded: every rank's flags (all-gathered)
  bool lastcol_failed();
  bool h_partial = false;  // a host trace of which only this rank's columns were uploaded
  // stage sessions (zkp_session_*): the caller's channel draws every coefficient, so
  // commitments return their roots to the host and no device transcript runs
  bool host_channel = false;

  ProofRun(zkp_ctx* c, zkp_comm* m, const zkp_proof_options* opts)
      : ctx(c), cm(m), o(opts), st(c->stream), pf(c->prof) {
    memset(&T, 0, sizeof T);
  }
  uint32_t ce_owner(uint32_t u) const { return (u << cstep) / Bl; }
  uint32_t ce_first(uint32_t s) const {
    uint32_t u = 0;
    while (u < ce && ce_owner(u) < s) u++;
    return u;
  }
  int init(int air_id, const felt* d_trace_in, uint32_t width, uint64_t n_rows, const zkp_felt* pub_elems,
           uint64_t n_pub, uint8_t** proof, uint64_t* proof_len);
  void setup();
  void trace_stage(const zkp_felt* h_trace);
  void constraint_stage();
  void eval_stage();
  void composition_stage();
  void ood_values();
  void ood_stage();
  void deep_stage();
  void fri_stage();
  FriCursor fri_layers();
  void fri_round_trip(const FriCursor& c);
  void grind_stage();
  int finish(uint8_t** proof, uint64_t* proof_len, zkp_transcript* tr_out);
};

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
  ctx->ensure_coset(logn, logB, logce);
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
    // (the pointwise A/B switches do, so they keep the columns).
    static const bool no_lazy = getenv("ZKP_NO_GU_LAZY") || getenv("ZKP_EVAL_POINTWISE") ||
                                getenv("ZKP_DEEP_POINTWISE");
    gu_lazy_on = !no_lazy && w >= DEEP_COEF_MIN_W;
    gu_lazy = GuLazy{gu_cval, l0_table(), air.k, d, R > 1 && cpt && wi < w ? wi : d,
                     (uint32_t)(air.k.hi == 0 && (air.k.lo >> 32) == 0)};
  }
  if (cpt) {
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
  } else {
    if (h_trace && R > 1) {
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
      h_trace = nullptr;  // resident on every rank from here
    }
    const uint32_t wd = paired ? d : w;  // columns interpolated and extended here
    // groups (first column, columns) of [0, wd): one for device-resident traces.
    // Host traces upload group g+1 on the side stream while the main stream
    // interpolates and extends group g; the groups grow geometrically (x1.5 from
    // ~w/40 columns: C3 unpaired 3, 4, 6, ..., 38), so only the small first group's
    // upload is exposed and every later one hides behind the previous group's LDE
    // (a column uploads in ~0.55x its LDE at C3).
    std::vector<std::pair<uint32_t, uint32_t>> grp;
    static const uint32_t growth =  // percent (A/B switch ZKP_UPLOAD_GROWTH)
        getenv("ZKP_UPLOAD_GROWTH") ? std::max(110, atoi(getenv("ZKP_UPLOAD_GROWTH"))) : 150u;
    if (h_trace && wd >= 4) {
      uint32_t cw = std::max(1u, w / 40);
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
      if (c0 >= wd) {  // paired columns d+i, i in [c0 - d, c0 - d + cw): check, then derive
        const uint32_t i0 = c0 - d;
        launch_gu_check(pf, st, d_trace, d, logn, air.k, i0, cw, 0, logn, gu_cval, gu_bad);
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
    static const bool no_derive = getenv("ZKP_NO_DERIVE_LAST") != nullptr;  // A/B switch
    const bool derive = allow_shortcuts && !no_derive && logce == logB && C >= 2 && C <= 8 && cel == Bl && u0 == j0;
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
    if (R > 1) {
      // send block s = positions [s*nR, (s+1)*nR) of every owned CE coset
      felt* send = ctx->buf<felt>("comp_send", (size_t)celmax * n);
      recv = ctx->buf<felt>("comp_recv", (size_t)celmax * n);
      for (uint32_t ul = 0; ul < cel; ul++)
        HIP_CHECK(hipMemcpy2DAsync(send + (size_t)ul * nR, (size_t)celmax * nR * 16, cint + (size_t)ul * n, nR * 16,
                                   nR * 16, R, hipMemcpyDeviceToDevice, st));
      cm->all_to_all(st, send, recv, (size_t)celmax * nR * 16);
    }
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
      // column by column: the all-gather of coefficient column m (rank s's slice of
      // positions [s*nR, (s+1)*nR) lands at acoef + m*n + s*nR, i.e. the column in
      // order) runs on the side stream while the main stream extends column m - 1
      // (the largest exchange of a sharded proof, hidden behind the
      // composition LDE)
      ctx->events(C);
      HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
      HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
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
        HIP_CHECK(hipStreamWaitEvent(st, ctx->up_ev[m], 0));
        if (derive && m == C - 1) break;  // derived in the leaf pass (the OOD still reads its coefficients)
        NttBatch lb{acoef + (size_t)m * n, clde + (size_t)m * Bl * n, Sj0, n, n, Bl, Bl, Bl};
        launch_ntt(pf, st, lb, logn, true, ctx->tws(logN), logN);
      }
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
  if (!ctx->have_cached(key)) launch_l0_table(pf, st, PointMap{cx + j0, twn, logn}, (uint64_t)Bl * n, inv(felt_u64(n)), t);
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
               uint64_t* proof_len, zkp_transcript* tr_out, const zkp_felt* h_trace = nullptr) {
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

}  // namespace

void launch_fail(int code, const char* what) { throw ZkpFail{code, what}; }

namespace {

template <typename F>
int guarded(zkp_ctx* ctx, F&& f) {
  if (!ctx) return ZKP_ERR_ARGUMENT;
  try {
    int rc = f();
    if (rc && ctx->err.empty()) ctx->err = "status " + std::to_string(rc);
    return rc;
  } catch (const ZkpFail& e) {
    ctx->err = e.msg;
    ctx->prof.pending.clear();
    drain_streams(ctx);
    return e.code;
  } catch (const std::bad_alloc&) {
    ctx->err = "host out of memory";
    drain_streams(ctx);
    return ZKP_ERR_OOM;
  } catch (const CommError& e) {
    ctx->err = std::string("collective failed: ") + e.what();
    ctx->prof.pending.clear();
    drain_streams(ctx);
    return ZKP_ERR_DEVICE;
  } catch (...) {
    ctx->err = "unknown failure";
    drain_streams(ctx);
    return ZKP_ERR_DEVICE;
  }
}

}  // namespace

// a context on `device` with its streams and events (nullptr on failure)
zkp_ctx* new_ctx(int device) {
  zkp_ctx* c = new (std::nothrow) zkp_ctx();
  if (!c) return nullptr;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return nullptr;
  }
  return c;
}

// ====================================================================== C-ABI
extern "C" {

int zkp_ctx_create(int device, zkp_ctx** out) {
  if (!out) return ZKP_ERR_ARGUMENT;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0) return ZKP_ERR_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return ZKP_ERR_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ZKP_ERR_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZKP_ERR_DEVICE;  // code objects are gfx950-only
  zkp_ctx* c = new_ctx(device);
  if (!c) return ZKP_ERR_DEVICE;
  *out = c;
  return ZKP_OK;
}

void zkp_ctx_destroy(zkp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (zkp_ctx* sc : ctx->session_pool) {  // idle session contexts (stage sessions)
    drain_streams(sc);
    delete sc;
  }
  ctx->session_pool.clear();
  drain_streams(ctx);
  delete ctx;
}

const char* zkp_last_error(const zkp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void zkp_free(void* p) { free(p); }

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

int zkp_device_alloc(zkp_ctx* ctx, uint64_t bytes, void** d_ptr) {
  return guarded(ctx, [&] {
    if (!d_ptr) return (int)ZKP_ERR_ARGUMENT;
    HIP_CHECK(hipSetDevice(ctx->device));
    HIP_CHECK(hipMalloc(d_ptr, bytes ? bytes : 16));
    ctx->user_allocs.push_back(*d_ptr);
    return 0;
  });
}

int zkp_device_free(zkp_ctx* ctx, void* d_ptr) {
  return guarded(ctx, [&] {
    auto it = std::find(ctx->user_allocs.begin(), ctx->user_allocs.end(), d_ptr);
    if (it == ctx->user_allocs.end()) return (int)ZKP_ERR_ARGUMENT;
    ctx->user_allocs.erase(it);
    HIP_CHECK(hipFree(d_ptr));
    return 0;
  });
}

int zkp_copy_to_device(zkp_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes) {
  return guarded(ctx, [&] {
    HIP_CHECK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
    ctx->sync();
    return 0;
  });
}

int zkp_copy_to_host(zkp_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes) {
  return guarded(ctx, [&] {
    ctx->download(h_dst, d_src, bytes);
    return 0;
  });
}

int zkp_trace_lde_commit(zkp_ctx* ctx, const zkp_felt* trace, uint32_t w, uint64_t n, uint32_t blowup,
                         zkp_felt* lde_out, uint8_t root[32]) {
  return guarded(ctx, [&] {
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!trace || !root) return (int)ZKP_ERR_ARGUMENT;
    if (n < 8 || (n & (n - 1)) || w == 0 || w > 255) return (int)ZKP_ERR_TRACE_SHAPE;
    if (blowup < 2 || (blowup & (blowup - 1)) || blowup > 128) return (int)ZKP_ERR_INVALID_OPTIONS;
    uint32_t logn = ilog2(n), logB = ilog2(blowup);
    if (logn + logB > MAX_LOG_DOMAIN) return (int)ZKP_ERR_TRACE_SHAPE;
    uint64_t N = n * blowup;
    felt* d = ctx->buf<felt>("trace_in", (size_t)w * n);
    ctx->upload(d, trace, (size_t)w * n * 16);
    felt* coef = ctx->buf<felt>("coef", (size_t)w * n);
    felt* lde = ctx->buf<felt>("tlde", (size_t)w * N);
    ctx->ensure_coset(logn, logB, 1);
    const uint32_t logN = logn + logB;
    NttBatch ib{d, coef, nullptr, n, n, 1, 1, w};
    launch_ntt(ctx->prof, ctx->stream, ib, logn, false, ctx->itws(logN), logN);
    NttBatch lb{coef, lde, ctx->S(logn, logB), n, n, blowup, blowup, w * blowup};
    launch_ntt(ctx->prof, ctx->stream, lb, logn, true, ctx->tws(logN), logN);
    TreeShard tr;
    commit_rows(ctx, ctx->self_comm(), 0, lde, n, w, logB, logn, false, "ttree", tr, root);
    if (lde_out) {
      std::vector<felt> h((size_t)w * N);
      ctx->download(h.data(), lde, h.size() * 16);
      for (uint32_t c = 0; c < w; c++)
        for (uint64_t i = 0; i < N; i++) {
          felt v = h[((size_t)c * blowup + (i & (blowup - 1))) * n + (i >> logB)];
          lde_out[(size_t)c * N + i].lo = v.lo;
          lde_out[(size_t)c * N + i].hi = v.hi;
        }
    }
    ctx->collect_prof();
    return 0;
  });
}

int zkp_merkle_commit_rows(zkp_ctx* ctx, const zkp_felt* cols, uint32_t w, uint64_t rows, uint8_t root[32]) {
  return guarded(ctx, [&] {
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!cols || !root) return (int)ZKP_ERR_ARGUMENT;
    if (rows < 2 || (rows & (rows - 1)) || w == 0 || w > 255) return (int)ZKP_ERR_TRACE_SHAPE;
    felt* d = ctx->buf<felt>("mrows", (size_t)w * rows);
    ctx->upload(d, cols, (size_t)w * rows * 16);
    uint32_t* tree = ctx->buf<uint32_t>("mtree", (size_t)16 * rows);
    launch_merkle_lde(ctx->prof, ctx->stream, d, w, 0, rows, tree, rows);
    ctx->download(root, tree + 8, 32);
    ctx->collect_prof();
    return 0;
  });
}

int zkp_grind(zkp_ctx* ctx, const uint8_t seed[32], uint32_t bits, uint64_t* nonce) {
  return guarded(ctx, [&] {
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!seed || !nonce || bits > 64) return (int)ZKP_ERR_ARGUMENT;
    uint32_t sw[8];
    for (int i = 0; i < 8; i++)
      sw[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
              ((uint32_t)seed[4 * i + 3] << 24);
    // one launch to the minimum nonce (k_grind_all), as zkp_prove's device query tail
    unsigned long long* dres = ctx->buf<unsigned long long>("grind_res", 1);
    uint32_t* dseed = ctx->buf<uint32_t>("grind_seed", 8);
    ctx->upload(dseed, sw, 32);
    HIP_CHECK(hipMemsetAsync(dres, 0xff, 8, ctx->stream));
    launch_grind_all(ctx->prof, ctx->stream, dseed, 1, 1ull << 40, bits, dres);
    unsigned long long res;
    ctx->download(&res, dres, 8);
    if (res == ~0ull) return (int)ZKP_ERR_NONCE;
    *nonce = res;
    ctx->collect_prof();
    return 0;
  });
}

int zkp_build_global_update_trace(zkp_ctx* ctx, const zkp_felt* raw_global, const zkp_felt* blinding,
                                  const zkp_felt* local_updates, uint64_t ndev, zkp_felt k, uint64_t n,
                                  void* d_trace_out, zkp_felt* final_state) {
  return guarded(ctx, [&] {
    HIP_CHECK(hipSetDevice(ctx->device));
    if (!raw_global || !blinding || !d_trace_out || (ndev && !local_updates)) return (int)ZKP_ERR_ARGUMENT;
    if (n < 8 || (n & (n - 1)) || n < ndev + 2) return (int)ZKP_ERR_TRACE_SHAPE;
    const felt kf = make(k.lo, k.hi);
    if (ge_p(kf)) return (int)ZKP_ERR_PUB_INPUTS;  // k = 0 is accepted: winterfell inv(0) = 0
    auto canon = [](const zkp_felt* v, uint64_t cnt) {
      for (uint64_t i = 0; i < cnt; i++)
        if (ge_p(make(v[i].lo, v[i].hi))) return false;
      return true;
    };
    if (!canon(raw_global, GU_D) || !canon(blinding, GU_D) || !canon(local_updates, ndev * GU_D))
      return (int)ZKP_ERR_ARGUMENT;
    // masked global model (prover.rs:68-79): raw + blinding
    std::vector<felt> hm(2 * GU_D);
    for (uint32_t c = 0; c < GU_D; c++) {
      hm[c] = add(make(raw_global[c].lo, raw_global[c].hi), make(blinding[c].lo, blinding[c].hi));
      hm[GU_D + c] = make(raw_global[c].lo, raw_global[c].hi);
    }
    felt* dm = ctx->buf<felt>("gu_masked_raw", 2 * GU_D);
    ctx->upload(dm, hm.data(), hm.size() * 16);
    felt* dl = ctx->buf<felt>("gu_local", ndev ? ndev * GU_D : 1);
    if (ndev) HIP_CHECK(hipMemcpyAsync(dl, local_updates, ndev * GU_D * 16, hipMemcpyHostToDevice, ctx->stream));
    const uint64_t tiles = (n + 4095) / 4096;
    felt* tb = ctx->buf<felt>("gu_tiles", tiles * GU_D);
    launch_gu_trace(ctx->prof, ctx->stream, dm, dm + GU_D, dl, ndev, inv(kf), n, tb, (felt*)d_trace_out);
    if (final_state)  // row ndev + 1 of the S columns (the state get_pub_inputs reads, prover.rs:168-172)
      HIP_CHECK(hipMemcpy2DAsync(final_state, 16, (const felt*)d_trace_out + ndev + 1, n * 16, 16, GU_D,
                                 hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    ctx->collect_prof();
    return 0;
  });
}

int zkp_set_profiling(zkp_ctx* ctx, int enabled) {
  return guarded(ctx, [&] {
    ctx->prof.enabled = enabled != 0;
    return 0;
  });
}

int zkp_set_profiling_kernel(zkp_ctx* ctx, const char* kernel_name) {
  return guarded(ctx, [&] {
    ctx->prof.only = kernel_name ? kernel_name : "";
    return 0;
  });
}

int zkp_kernel_stats(zkp_ctx* ctx, const char* kernel_name, uint64_t* launches, double* total_ms) {
  return guarded(ctx, [&] {
    if (!kernel_name || !launches || !total_ms) return (int)ZKP_ERR_ARGUMENT;
    auto it = ctx->stats.find(kernel_name);
    *launches = it == ctx->stats.end() ? 0 : it->second.launches;
    *total_ms = it == ctx->stats.end() ? 0.0 : it->second.ms;
    return 0;
  });
}

int zkp_reset_stats(zkp_ctx* ctx) {
  return guarded(ctx, [&] {
    ctx->stats.clear();
    return 0;
  });
}

int zkp_kernel_stats_table(zkp_ctx* ctx, char** table) {
  return guarded(ctx, [&] {
    if (!table) return (int)ZKP_ERR_ARGUMENT;
    std::string s;
    char line[256];
    for (auto& kv : ctx->stats) {
      snprintf(line, sizeof line, "%s %llu %.6f %.0f\n", kv.first.c_str(), (unsigned long long)kv.second.launches,
               kv.second.ms, kv.second.bytes);
      s += line;
    }
    *table = (char*)malloc(s.size() + 1);
    memcpy(*table, s.c_str(), s.size() + 1);
    return 0;
  });
}

// Host-side MiMC AIR trace builder (trace construction, like TraceTable building
// in the reference; not part of the proving hot path).
int zkp_build_mimc_trace(const uint8_t seed[16], uint64_t n, zkp_felt* out) {
  if (!seed || !out || n == 0) return ZKP_ERR_ARGUMENT;
  felt v = from_u128_bytes(seed);
  if (ge_p(v)) v = sub(v, make(P_LO, P_HI));
  for (uint64_t i = 0; i < n; i++) {
    out[i].lo = v.lo;
    out[i].hi = v.hi;
    felt u = add(v, felt_u64((i % 64 + 1) * 1000000ull));
    felt u2 = sqr(u), u3 = mul(u2, u), u6 = sqr(u3);
    v = mul(u6, u);
  }
  return 0;
}

}  // extern "C"

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
    s->parent->session_pool.push_back(s->ctx);  // buffers and domain tables kept for the next session
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
  ch->coin.reseed(root);
  return ZKP_OK;
}

int zkp_channel_commit_felts(zkp_channel* ch, const zkp_felt* els, uint64_t n) {
  if (!ch || (n && !els)) return ZKP_ERR_ARGUMENT;
  std::vector<felt> v(n);
  for (uint64_t i = 0; i < n; i++) v[i] = make(els[i].lo, els[i].hi);
  uint8_t d[32];
  hash_elements(v.data(), v.size(), d);
  ch->coin.reseed(d);
  return ZKP_OK;
}

int zkp_channel_draw(zkp_channel* ch, uint32_t method, uint32_t count, zkp_felt* out) {
  if (!ch || !out || method > ZKP_BATCHING_HORNER) return ZKP_ERR_ARGUMENT;
  try {
    if (count == 0) {
      const felt v = ch->coin.draw();
      out[0] = zkp_felt{v.lo, v.hi};
      return ZKP_OK;
    }
    const std::vector<felt> v = draw_coeffs(ch->coin, method, count);
    for (uint32_t i = 0; i < count; i++) out[i] = zkp_felt{v[i].lo, v[i].hi};
    return ZKP_OK;
  } catch (const ZkpFail& e) {
    return e.code;
  }
}

int zkp_channel_seed(const zkp_channel* ch, uint8_t seed[32]) {
  if (!ch || !seed) return ZKP_ERR_ARGUMENT;
  memcpy(seed, ch->coin.seed, 32);
  return ZKP_OK;
}

int zkp_channel_query_positions(zkp_channel* ch, uint64_t nonce, uint64_t* out, uint32_t* n_unique) {
  if (!ch || !out || !n_unique) return ZKP_ERR_ARGUMENT;
  std::vector<uint64_t> pos = ch->coin.draw_integers(ch->num_queries, ch->lde_size, nonce);
  std::sort(pos.begin(), pos.end());
  pos.erase(std::unique(pos.begin(), pos.end()), pos.end());
  for (size_t i = 0; i < pos.size(); i++) out[i] = pos[i];
  *n_unique = (uint32_t)pos.size();
  return ZKP_OK;
}

}  // extern "C"
