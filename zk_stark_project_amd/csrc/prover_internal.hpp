// prover_internal.hpp — the prover's host-side internals shared by its translation
// units: the context (zkp_ctx: streams, buffers, domain tables), the proof state
// (ProofRun) and the stage helpers. prover.cpp runs a proof's stages,
// prover_stages.cpp holds the stage helpers (commitments, OOD, constraint evaluation,
// DEEP, openings), prover_shard.cpp the sharded exchanges and the multi-GPU entry
// points, session.cpp the stage sessions and the host channel, abi.cpp the rest of
// include/zkp.h.
#pragma once
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

#define HIP_CHECK(x)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess)                                                                          \
      throw ZkpFail{e_ == hipErrorOutOfMemory ? ZKP_ERR_OOM : ZKP_ERR_DEVICE,                      \
                    std::string(#x) + ": " + hipGetErrorString(e_)};                               \
  } while (0)

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
  // a proof's early trace check (MiMC transitions, GlobalUpdate pairs): its flag is
  // copied to flag_h (pinned) and ev_check recorded, so a later stage reads it
  // without stalling the queue (the GPU passed it long before)
  hipEvent_t ev_check = nullptr;
  uint32_t* flag_h = nullptr;
  uint32_t* host_flag() {
    if (!flag_h) HIP_CHECK(hipHostMalloc((void**)&flag_h, 64, hipHostMallocDefault));
    return flag_h;
  }
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
      auto t0 = std::chrono::steady_clock::now();
      // the smaller buffer is retired, not freed: hipFree waits for the whole device,
      // which mid-proof would drain the queued work of this and every other stream
      // (a new shape's first proof grows dozens of buffers); free_retired() releases
      // them once the proof's streams are idle
      if (b.p) retired.push_back(b.p);
      b.p = nullptr;
      HIP_CHECK(hipMalloc(&b.p, bytes));
      b.bytes = bytes;
      if (prof.enabled) {  // first-use allocations (the cold proof's cost, bench first_proof)
        auto& s = stats["host_alloc"];
        s.launches += 1;
        s.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        s.bytes += (double)bytes;
      }
    }
    return reinterpret_cast<T*>(b.p);
  }
  std::vector<void*> retired;  // outgrown buffers (buf()), freed by free_retired()
  void free_retired() {
    if (retired.empty()) return;
    for (hipStream_t s : {stream, side, copy}) HIP_CHECK(hipStreamSynchronize(s));
    for (void* p : retired) (void)hipFree(p);
    retired.clear();
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
    // the call's device-busy time: the union of its launches' [start, stop) intervals
    // over every stream (overlapping launches counted once; idle gaps not at all),
    // reported as the pseudo-entry "host_device_busy" (not a kernel: host_* rows are
    // left out of the kernel tables)
    if (prof.only.empty()) {
      const hipEvent_t t0 = prof.pending.front().start;
      std::vector<std::pair<float, float>> iv;
      iv.reserve(prof.pending.size());
      for (auto& r : prof.pending) {
        float st = 0, en = 0;
        HIP_CHECK(hipEventElapsedTime(&st, t0, r.start));
        HIP_CHECK(hipEventElapsedTime(&en, t0, r.stop));
        iv.emplace_back(st, en);
      }
      std::sort(iv.begin(), iv.end());
      double busy = 0;
      float cs = iv[0].first, ce = iv[0].second;
      for (size_t i = 1; i < iv.size(); i++) {
        if (iv[i].first > ce) {
          busy += ce - cs;
          cs = iv[i].first;
          ce = iv[i].second;
        } else if (iv[i].second > ce) {
          ce = iv[i].second;
        }
      }
      busy += ce - cs;
      auto& b = stats["host_device_busy"];
      b.launches += 1;
      b.ms += busy;
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
    stage_end("0_pre_tw");
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
      stage_end(dir ? "0_tw_inv" : "0_tw_fwd");
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
    for (void* p : retired) (void)hipFree(p);
    for (auto& kv : bufs)
      if (kv.second.p) (void)hipFree(kv.second.p);
    for (void* p : user_allocs) (void)hipFree(p);
    if (pinned_p) (void)hipHostFree(pinned_p);
    if (ring_p) (void)hipHostFree(ring_p);
    for (auto e : prof.pool) (void)hipEventDestroy(e);
    for (auto e : up_ev) (void)hipEventDestroy(e);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_check) (void)hipEventDestroy(ev_check);
    if (flag_h) (void)hipHostFree(flag_h);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (stream && side && copy) {
      const hipStream_t ss[3] = {stream, side, copy};
      release_streams(device, ss);
    } else {
      if (copy) (void)hipStreamDestroy(copy);
      if (side) (void)hipStreamDestroy(side);
      if (stream) (void)hipStreamDestroy(stream);
    }
  }
  // A process-wide pool of idle (stream, side, copy) sets per device: creating a
  // context's streams binds each to a new hardware queue at its first dispatch, ≈ 8 ms
  // for the three (BENCH reference_flow ctx_create_phases_ms); a context created after
  // another was destroyed takes that one's bound streams instead.
  static bool acquire_streams(int device, hipStream_t out[3]);
  static void release_streams(int device, const hipStream_t s[3]);
};

// a context on `device` with its streams and events (nullptr on failure)
zkp_ctx* new_ctx(int device);

namespace zkpi {

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

// evaluate bit-reversed coefficient arrays (scaled by n) at x0, x1 -> values (x n^-1)
// a device -> host copy folded into a round trip
struct Fetch {
  void* host;
  const void* dev;
  size_t bytes;
};

// DEEP composition evaluations over the rank's cosets [j0, j0 + Bl) (coset-major).
// Narrow traces: pointwise k_deep over every trace and composition column's LDE.
// Wide traces (w >= DEEP_COEF_MIN_W): winterfell's own dataflow
// — the gamma-combination of the trace polynomials in coefficient form
// (k_deep_lincomb over `coef`, read once), its coset LDE, then k_deep over that one
// column and the composition columns with coefficients [1 | delta]: w column reads
// per LDE point become one (C3: 8.2 GB -> ~1 GB per proof). Same field values.
constexpr uint32_t DEEP_COEF_MIN_W = 16;

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
  // the shapes on which LastCol applies at all (the CE domain is the rank's LDE cosets)
  bool lastcol_shape() const;
  uint32_t* lc_bad = nullptr;    // this rank's flag (4 words)
  uint32_t* lc_flags = nullptr;  // sharded: every rank's flags (all-gathered)
  bool lastcol_failed();
  // the early trace check (trace_stage -> composition_stage / the paired group)
  bool pre_checked = false;
  void early_check_launch(uint32_t* dflag, hipStream_t s);
  bool early_check_failed();
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
  // the sharded exchanges (prover_shard.cpp)
  void trace_column_sharded(const zkp_felt* h_trace, uint32_t cpt, uint32_t wi, uint32_t d);
  const zkp_felt* gather_host_slices(const zkp_felt* h_trace);
  felt* composition_exchange(felt* cint, uint64_t nR);
  void composition_gather_lde(felt* slice, bool derive, uint64_t nR, uint64_t p0);
};

// ---- stage helpers (prover_stages.cpp; the sharded parts in prover_shard.cpp)
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
                 const GuLazy* gl = nullptr);
bool commit_rows_sharded(zkp_ctx* ctx, zkp_comm* cm, int mode, const felt* src, uint64_t n, uint32_t cols,
                         uint32_t logB, uint32_t logrows, const std::string& name, TreeShard& tr, uint8_t root[32],
                         bool fetch_root, const MerkleTail* coin, const LastCol* lc, const GuLazy* gl);
// device -> host copies of one round trip (one sync)
void fetch_all(zkp_ctx* ctx, const std::vector<Fetch>& fs);
felt* ood_launch(zkp_ctx* ctx, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn, const felt* dpw,
                 zkp_comm* cm = nullptr);
felt* ood_launch_sharded(zkp_ctx* ctx, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn,
                         const felt* dpw, zkp_comm* cm, felt* part, felt* dv);
felt* coset_points(zkp_ctx* ctx, uint32_t logn, uint32_t logB, uint32_t logce);
void constraint_eval(zkp_ctx* ctx, const AirDesc& air, uint32_t logn, uint32_t logB, uint32_t logce, uint32_t u0,
                     uint32_t cel, uint32_t j0, uint32_t logBl, const felt* cx, const felt* twn, const felt* dt_cc,
                     const felt* dt_aval, const felt* tlde, felt* comp, const felt* coef = nullptr,
                     zkp_comm* cm = nullptr);
const felt* last_col_kappa(zkp_ctx* ctx, uint32_t logn, uint32_t logB, uint32_t C);
std::vector<felt> comp_dft_consts(uint64_t n, uint32_t logce, uint32_t C);
void deep_evaluations(zkp_ctx* ctx, zkp_comm* cm, hipStream_t st, DeepArgs da, const felt* coef, uint64_t n,
                      const felt* Sj0, uint32_t logN, felt* out);
void gather_openings(zkp_ctx* ctx, zkp_comm* cm, const std::vector<uint64_t>& pos, uint64_t n, uint32_t logB,
                     uint32_t j0, const felt* tlde, uint32_t w, const TreeShard& ttree, const felt* clde, uint32_t C,
                     const TreeShard& ctree, const std::vector<FriLayer>& layers, uint32_t L, uint32_t F,
                     Openings& op);
void openings_from_full(const std::vector<uint64_t>& raw, const std::vector<uint64_t>& pos, const uint32_t* full,
                        const FullGatherArgs& ga, const std::vector<FriLayer>& layers, uint32_t L, uint32_t F,
                        Openings& op);
const felt* fold_constants(zkp_ctx* ctx);

// ---- proofs (prover.cpp)
// h_trace (nullable): the trace is still in host memory and d_trace is its
// device buffer; the upload is pipelined with the trace interpolation and LDE
// by column groups (wide traces), so PCIe overlaps the first stage's kernels.
int prove_impl(zkp_ctx* ctx, zkp_comm* cm, int air_id, const felt* d_trace, uint32_t w, uint64_t n,
               const zkp_felt* pub_elems, uint64_t n_pub, const zkp_proof_options* o, uint8_t** proof,
               uint64_t* proof_len, zkp_transcript* tr_out, const zkp_felt* h_trace = nullptr);
// every stream of the context idle
void drain_streams(zkp_ctx* ctx);

// an entry point's body: C++ failures become its ZKP_ERR_* status (never an
// exception across the C ABI) with the message in ctx->err
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

}  // namespace zkpi
