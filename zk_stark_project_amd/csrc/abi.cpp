// abi.cpp — the context, device-memory, stateless-stage and statistics entry points
// of include/zkp.h (the proofs are in prover.cpp, the sharded ones in
// prover_shard.cpp, the stage sessions in session.cpp).
#include "prover_internal.hpp"

#include <mutex>

using namespace zkpi;

namespace {
// gfx950 check once per device and process (hipGetDeviceProperties queries every
// attribute of the device: milliseconds, paid again by every context otherwise)
bool device_is_gfx950(int device) {
  static std::mutex mu;
  static std::map<int, bool> known;
  std::lock_guard<std::mutex> lk(mu);
  auto it = known.find(device);
  if (it != known.end()) return it->second;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return false;
  const bool ok = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
  known[device] = ok;
  return ok;
}
}  // namespace

extern "C" {

int zkp_ctx_create(int device, zkp_ctx** out) {
  if (!out) return ZKP_ERR_ARGUMENT;
  *out = nullptr;
  // phase wall times, kept in the context's statistics as host_ctx_* rows
  using clk = std::chrono::steady_clock;
  auto t = clk::now();
  std::vector<std::pair<const char*, double>> phases;
  auto lap = [&](const char* name) {
    const auto now = clk::now();
    phases.emplace_back(name, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  };
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0) return ZKP_ERR_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return ZKP_ERR_DEVICE;
  if (!device_is_gfx950(device)) return ZKP_ERR_DEVICE;  // code objects are gfx950-only
  lap("host_ctx_device_check");
  zkp_ctx* c = new_ctx(device);
  if (!c) return ZKP_ERR_DEVICE;
  lap("host_ctx_streams");
  // the kernels' code objects, the streams' hardware queues and the pinned staging
  // buffers, ahead of the first proof (a process's first proof was ≈ 4x a warm one)
  preload_kernels_module();
  preload_merkle_module();
  preload_ntt_module();
  lap("host_ctx_code_objects");
  try {
    c->pinned(1u << 20);
    lap("host_ctx_pinned");
    const felt zero[1]{};
    c->upload(c->buf<felt>("ring_warm", 1), zero, 16);
    drain_streams(c);  // this context's streams only (not other contexts' proofs in flight)
    lap("host_ctx_first_copy");
  } catch (const ZkpFail& f) {
    delete c;
    return f.code;
  }
  for (auto& ph : phases) {
    auto& st = c->stats[ph.first];
    st.launches += 1;
    st.ms += ph.second;
  }
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

int zkp_ctx_trim(zkp_ctx* ctx) {
  if (!ctx) return ZKP_ERR_ARGUMENT;
  (void)hipSetDevice(ctx->device);
  for (zkp_ctx* sc : ctx->session_pool) {
    drain_streams(sc);
    delete sc;
  }
  ctx->session_pool.clear();
  return ZKP_OK;
}

const char* zkp_last_error(const zkp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void zkp_free(void* p) { free(p); }

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
    // chunks of 2^32 nonces (≈ 40 ms of full-chip BLAKE3 each), the host checking
    // between them, up to 2^40 (≈ 11 s): the first chunk with a hit holds the minimum.
    // bits <= 32 expects 2^bits tries, so the first chunk nearly always ends it
    unsigned long long res = ~0ull;
    for (uint64_t base = 1; base <= (1ull << 40) && res == ~0ull; base += 1ull << 32) {
      launch_grind_all(ctx->prof, ctx->stream, dseed, base, base + (1ull << 32) - 1, bits, dres);
      ctx->download(&res, dres, 8);
    }
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
