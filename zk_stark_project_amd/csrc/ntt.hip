// ntt.hip — the NTT kernels of the prover (gfx950): radix-8 register-blocked
// LDS passes over stage-major twiddles, and their launch planning. Split from
// kernels.hip so the hottest kernel rebuilds on its own.
#include "kernels_common.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>

using kc::static_for;
using kc::rev_bits;

namespace {

// --------------------------------------------------------------------- NTT
struct NttKArgs {
  const felt* src;
  felt* dst;
  const felt* scale;
  const felt* tw;
  uint64_t src_stride, dst_stride;
  uint32_t src_div, scale_mod;
  uint32_t logn, s0, K, lo, T, Tl, logT, logTl, tw_shift, dit;
};

// One LDS pass of K radix-2 stages over T interleaved groups of 2^K elements.
// Group g = (hi, l): elements hi*2^(lo+K) + q*2^lo + l, q < 2^K. Loads are
// ordered so each wave reads runs of Tl (>= 8 when lo allows) contiguous felts.
__global__ __launch_bounds__(TPB) void k_ntt_pass(NttKArgs a) {
  extern __shared__ felt lds[];
  const uint32_t bidx = blockIdx.y;
  const felt* src = a.src + (uint64_t)(bidx / a.src_div) * a.src_stride;
  felt* dst = a.dst + (uint64_t)bidx * a.dst_stride;
  const felt* scale = a.scale ? a.scale + ((uint64_t)(bidx % a.scale_mod) << a.logn) : nullptr;
  const uint32_t K = a.K, T = a.T, Tl = a.Tl, lo = a.lo;
  const uint32_t E = T << K;
  const uint64_t g0 = (uint64_t)blockIdx.x * T;
  const uint64_t hi0 = g0 >> lo;
  const uint64_t l0 = (Tl == T) ? (g0 & ((1ull << lo) - 1)) : 0;
  const uint32_t qmask = (1u << K) - 1;

  for (uint32_t e = threadIdx.x; e < E; e += TPB) {
    uint32_t ll = e & (Tl - 1);
    uint32_t rest = e >> a.logTl;
    uint32_t q = rest & qmask;
    uint32_t hl = rest >> K;
    uint64_t addr = ((hi0 + hl) << (lo + K)) + ((uint64_t)q << lo) + l0 + ll;
    felt v = src[addr];
    if (scale) v = mul(v, scale[addr]);
    lds[(q << a.logT) + (hl * Tl) + ll] = v;
  }
  __syncthreads();
  for (uint32_t ls = 0; ls < K; ls++) {
    const uint32_t s = a.s0 + ls;
    const uint32_t pbit = a.dit ? ls : (K - 1 - ls);
    const uint32_t lev = a.dit ? s : (a.logn - 1 - s);  // stage-major twiddle level
    const felt* twl = a.tw + ((1ull << lev) - 1);
    const uint32_t pmask = (1u << pbit) - 1;
    for (uint32_t bf = threadIdx.x; bf < (E >> 1); bf += TPB) {
      uint32_t gg = bf & (T - 1);
      uint32_t qq = bf >> a.logT;
      uint32_t q = ((qq >> pbit) << (pbit + 1)) | (qq & pmask);
      uint32_t q2 = q | (1u << pbit);
      uint64_t l = l0 + (gg & (Tl - 1));
      uint64_t j = ((uint64_t)(q & pmask) << lo) | l;
      felt w = twl[j];
      uint32_t i0 = (q << a.logT) + gg, i1 = (q2 << a.logT) + gg;
      felt x = lds[i0], y = lds[i1];
      if (a.dit) {
        felt t = mul(y, w);
        lds[i0] = add(x, t);
        lds[i1] = sub(x, t);
      } else {
        lds[i0] = add(x, y);
        lds[i1] = mul(sub(x, y), w);
      }
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < E; e += TPB) {
    uint32_t ll = e & (Tl - 1);
    uint32_t rest = e >> a.logTl;
    uint32_t q = rest & qmask;
    uint32_t hl = rest >> K;
    uint64_t addr = ((hi0 + hl) << (lo + K)) + ((uint64_t)q << lo) + l0 + ll;
    dst[addr] = lds[(q << a.logT) + (hl * Tl) + ll];
  }
}

// ------------------------------------------------------------- NTT radix-8
// Register-blocked pass: each of NT threads owns 8 elements; a pass of K <= 10
// stages runs as rounds of up to 3 stages (radix-8 / 2x radix-4 / 4x radix-2)
// in registers with one LDS exchange per round. Global traffic is staged
// through LDS in the coalesced (gg-fastest) order.
struct Ntt8Args {
  const felt* src;
  felt* dst;
  const felt* scale;
  const felt* tw;
  uint64_t src_stride, dst_stride;
  uint32_t src_div, scale_mod;
  uint32_t logn, s0, K, lo, logT, logTl, tw_shift, nrounds;
  uint32_t rbits[4];
  uint32_t tile_major;  // 1: deal whole position blocks to XCDs (k_ntt8)
  uint32_t batches, items;  // k_ntt8_pipe: batches of the pass, tiles x batches
};

// stage-major twiddles: level t holds w_{2^(t+1)}^j at tw[(2^t - 1) + j]
template <bool DIT>
__device__ __forceinline__ felt ntt_tw(const Ntt8Args& a, uint32_t j, uint32_t pbit) {
  uint32_t s = DIT ? a.s0 + pbit : a.s0 + a.K - 1 - pbit;
  uint32_t lev = DIT ? s : a.logn - 1 - s;
  return a.tw[((1u << lev) - 1) + j];
}

// Tuning builds only (tests/native/kbench_ntt.cpp, never the library): ZKP_NTT_NOBFLY
// replaces the field arithmetic of the butterflies by two cheap ops, ZKP_NTT_NOGMEM the
// HBM loads and stores of the array data by register values, so the time of each side
// alone can be read against the whole pass.
#ifdef ZKP_NTT_NOGMEM
#define NTT_LD(p) (make((uint64_t)(uintptr_t)(p), (uint64_t)threadIdx.x))
#define NTT_ST(p, v)                                               \
  do {                                                            \
    const felt v_ = (v);                                          \
    if (v_.lo == 0x123456789ull && v_.hi == 0xabcdefull) *(p) = v_; \
  } while (0)
#else
#define NTT_LD(p) (*(p))
#define NTT_ST(p, v) (*(p) = (v))
#endif

// Butterflies of a register round. FAST: the deferred-check forms (dmul, dadd;
// the round's Rare decides whether it is recomputed with the exact forms,
// FAST = false); the difference of canonical values needs no check.
#ifdef ZKP_NTT_NOBFLY
template <bool FAST>
__device__ __forceinline__ felt bmul(felt a, felt b, Rare& q) { return make(a.lo ^ b.lo, a.hi ^ b.hi); }
template <bool FAST>
__device__ __forceinline__ felt badd(felt a, felt b, Rare& q) { return make(a.lo + b.lo, a.hi + b.hi); }
__device__ __forceinline__ felt nsub(felt a, felt b) { return make(a.lo - b.lo, a.hi - b.hi); }
#else
template <bool FAST>
__device__ __forceinline__ felt bmul(felt a, felt b, Rare& q) { return dmul<FAST>(a, b, q); }
template <bool FAST>
__device__ __forceinline__ felt badd(felt a, felt b, Rare& q) { return dadd<FAST>(a, b, q); }
__device__ __forceinline__ felt nsub(felt a, felt b) { return sub(a, b); }
#endif

template <bool DIT, bool FAST>
__device__ __forceinline__ void bfly(felt& x, felt& y, felt w, Rare& q) {
  if (DIT) {
    felt t = bmul<FAST>(y, w, q);
    y = nsub(x, t);
    x = badd<FAST>(x, t, q);
  } else {
    felt d = nsub(x, y);
    x = badd<FAST>(x, y, q);
    y = bmul<FAST>(d, w, q);
  }
}

// butterfly with twiddle 1 (no product)
template <bool DIT, bool FAST>
__device__ __forceinline__ void bfly1(felt& x, felt& y, Rare& q) {
  felt d = nsub(x, y);
  x = badd<FAST>(x, y, q);
  y = d;
}

// rounds of a K-stage pass: <= 3 stages each, larger first
template <int K>
struct NttRounds {
  static constexpr int n = (K + 2) / 3;
  static constexpr int bits(int r) {
    int rem = K;
    for (int i = 0; i < r; i++) {
      int left = n - i;
      int b = (rem + left - 1) / left;
      rem -= b > 3 ? 3 : b;
    }
    int left = n - r;
    int b = (rem + left - 1) / left;
    return b > 3 ? 3 : b;
  }
};

// two independent butterflies with their products interleaved (fpd::mul_x2), so
// each carry consumer sits two instructions after its producer
template <bool DIT, bool FAST>
__device__ __forceinline__ void bfly2(felt& x0, felt& y0, felt w0, felt& x1, felt& y1, felt w1, Rare& q) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ZKP_NTT_NOBFLY)
  auto mx2 = [&](felt a, felt b, felt c, felt d, felt& ab, felt& cd) {
    if constexpr (FAST) fpd::mul_x2_z(a, b, c, d, ab, cd, q);
    else fpd::mul_x2(a, b, c, d, ab, cd);
  };
  if (DIT) {
    felt t0, t1;
    mx2(y0, w0, y1, w1, t0, t1);
    y0 = sub(x0, t0); x0 = badd<FAST>(x0, t0, q);
    y1 = sub(x1, t1); x1 = badd<FAST>(x1, t1, q);
  } else {
    felt d0 = sub(x0, y0), d1 = sub(x1, y1);
    x0 = badd<FAST>(x0, y0, q); x1 = badd<FAST>(x1, y1, q);
    mx2(d0, w0, d1, w1, y0, y1);
  }
#else
  bfly<DIT, FAST>(x0, y0, w0, q);
  bfly<DIT, FAST>(x1, y1, w1, q);
#endif
}

// SMALL: this pass holds the transform's smallest stages 0..2 (DIT first pass /
// DIF last pass, lo = 0); its round over them has jb = 0, so every twiddle of
// stage 0, half of stage 1 and a quarter of stage 2 is 1 and those products are
// skipped. A template flag, so the other passes keep their register budget.
// (5 waves/SIMD for the 6-stage passes spills 4-10 VGPRs and is slower:
// profiles/r05_ab_ntt_5waves_not_adopted.txt)
// LDS barrier of the passes: every wave's LDS operations retired, then s_barrier. No
// vmcnt wait: the pipelined pass keeps its next tile's LDS-DMA loads in flight across
// it (a __syncthreads() would drain them, cdna_hip_programming.md §5).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// One tile of a k_ntt8 pass (block-local elements (gg, q) of batch bidx, position block
// `tile`) in the block's LDS `lds`. PIPE: round 0 reads the tile from `lds`, where
// k_ntt8_pipe's LDS-DMA put it (the pass has no coset scale and loads directly).
template <bool DIT, int NT, int KC, bool SMALL, bool PIPE = false>
__device__ __forceinline__ void ntt8_tile(const Ntt8Args& a, uint32_t bidx, uint32_t tile, felt* lds) {
  constexpr int E = NT * 8;
  constexpr uint32_t K = KC;
  auto tile_barrier = [] {
    if constexpr (PIPE) lds_barrier();
    else __syncthreads();
  };
  constexpr uint32_t LOGNT = NT == 1024 ? 10 : (NT == 512 ? 9 : 8);
  constexpr uint32_t logT = LOGNT + 3 - KC;  // E = NT * 8 elements per block
  constexpr uint32_t T = 1u << logT;
  static_assert(T == 1 || T >= 4, "the LDS swizzles take rows of 1 or >= 4 felts");
  const uint32_t Tl = 1u << a.logTl, lo = a.lo;
  // LDS rows of T felts (T >= 8), XOR-swizzled by the row's low 3 bits: a wave's
  // 8-lane groups then hit 8 distinct 16-B bank slots both when lanes walk a row
  // (compute rounds) and when they walk down a column (staged loads, Tl = 1),
  // with no padding: 2048 felts = 32 KB per block, 5 blocks per CU
  // Rows of 4 felts (10-stage passes in 512-thread blocks) cover 4 of the 16-B
  // slots of a bank line. The row's low two bits are XORed with (b2^b3, b2^b5)
  // and the felt index with (b1, b2^b3): every 8-lane ds_write_b128 group and
  // every 16-lane ds_read_b128 group (MI355X_MICROARCH.md §LDS) then hits
  // distinct slots, in all compute rounds of both directions (whose two or four
  // rows per group differ in the row bits 0-5 that those rounds spread) and in
  // the staged column walks (checked exhaustively by tests/native/lds_swizzle.py).
  // (Fully conflict-free layouts for the 8-felt and >= 32-felt rows exist —
  // tests/native/lds_swizzle.py — but measured no faster: DESIGN.md §4.)
  // Rows of 1 felt (11-stage passes in 256-thread blocks: one 2048-element group per
  // block): the 16-B slot bits 0-2 are XORed with q bits 3-5 and bit 3 with q bit 6, so
  // every round of both directions and the staged walk are conflict-free (checked by
  // tests/native/lds_swizzle.py's T = 1 model).
  // Round 6: conflict-free in the model (tests/native/lds_swizzle.py, the `r06` layouts)
  // for every row length: rows of 8 also flip the row's bit 0 with q bits 2^3, rows of 16
  // (DIF) flip the felt index's bit 3 with q bits 2^4, rows of >= 32 swizzle the felt index
  // by q bits 0-3.
  auto lidx = [](uint32_t q, uint32_t x) -> uint32_t {
    if constexpr (T == 1) {
      (void)x;
      return q ^ ((q >> 3) & 7u) ^ (((q >> 6) & 1u) << 3);
    } else if constexpr (T >= 32) {
      return q * T + (x ^ (q & 15u));
    } else if constexpr (T == 16 && DIT) {
      return q * T + (x ^ (q & 7u));
    } else if constexpr (T == 16) {
      // DIF rounds: felt bits 0-2 ^= q bits 0-2, bit 3 ^= q bit 2 ^ q bit 4 (x ^ (q & 7)
      // conflicted on these rounds' reads). Conflict-free in the model for both directions,
      // but the DIT passes measured 1-3% slower with it and have no conflicts without it
      // (profiles/r06_ab_ntt_rows16_swizzle.txt).
      return q * T + (x ^ ((q & 7u) | ((((q >> 2) ^ (q >> 4)) & 1u) << 3)));
    } else if constexpr (T == 8) {
      return (q ^ (((q >> 2) ^ (q >> 3)) & 1u)) * T + (x ^ (q & 7u));
    } else {
      const uint32_t b1 = (q >> 1) & 1u, b23 = ((q >> 2) ^ (q >> 3)) & 1u, b25 = ((q >> 2) ^ (q >> 5)) & 1u;
      return (q ^ (b23 | (b25 << 1))) * T + (x ^ (b1 | (b23 << 1)));
    }
  };
  // grid: x = batch (fastest in dispatch order), y = position block. The
  // batches of one position block run back to back, dealt round-robin over the
  // 8 XCDs: with B = 8 cosets batch b = col*B + j lands on XCD j, so the
  // columns of a coset share its scale rows and every batch shares the pass's
  // twiddles in that XCD's L2 instead of refetching them per array.
  const felt* src = a.src + (uint64_t)(bidx / a.src_div) * a.src_stride;
  felt* dst = a.dst + (uint64_t)bidx * a.dst_stride;
  const felt* scale = a.scale ? a.scale + ((uint64_t)(bidx % a.scale_mod) << a.logn) : nullptr;
  const uint64_t g0 = (uint64_t)tile << logT;
  const uint32_t hi0 = (uint32_t)(g0 >> lo);
  const uint32_t l0 = (Tl == T) ? (uint32_t)(g0 & ((1ull << lo) - 1)) : 0;
  const uint32_t qmask = (1u << K) - 1;
  const uint32_t tid = threadIdx.x;

  // global address of block-local element (gg, q)
  // element offsets within one array fit 32 bits (launch_ntt checks logn), so
  // loads and stores take a scalar base + one 32-bit VGPR offset
  auto gaddr = [&](uint32_t gg, uint32_t q) -> uint32_t {
    uint32_t hl = gg >> a.logTl, ll = gg & (Tl - 1);
    return ((hi0 + hl) << (lo + K)) + (q << lo) + l0 + ll;
  };
  (void)qmask;
  // Passes whose groups have < 8 contiguous felts (lo < 3, e.g. the first DIT
  // pass) would make every lane of a direct load/store touch its own 128-B
  // line; those go through LDS in (ll, q, hl) order, contiguous along the wave.
  // (rows of 1: loading each lane's 8 contiguous felts directly instead, 128 B per lane,
  // was slower: profiles/r05_kbench_ntt_two_pass.txt)
  const bool staged = a.logTl < (T >= 8 ? 3u : 2u);  // rows of 4: 64-B runs go direct
  auto staged_elem = [&](uint32_t e, uint32_t& slot) -> uint32_t {
    uint32_t ll = e & (Tl - 1), rest = e >> a.logTl;
    uint32_t q = rest & ((1u << K) - 1), hl = rest >> K;
    slot = lidx(q, hl * Tl + ll);
    return ((hi0 + hl) << (lo + K)) + (q << lo) + l0 + ll;
  };
  if (staged) {
    // coset scale with the deferred check (the loads are redone exactly if it trips)
    auto stage_in = [&](auto fast_c, Rare& q) {
      constexpr bool FAST = decltype(fast_c)::value;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        uint32_t slot;
        uint32_t ad = staged_elem(tid + i * NT, slot);
        felt v = NTT_LD(src + ad);
        if (scale) v = bmul<FAST>(v, NTT_LD(scale + ad), q);
        lds[slot] = v;
      }
    };
    Rare q;
    stage_in(std::true_type{}, q);
    if (scale && q.any()) stage_in(std::false_type{}, q);
    tile_barrier();
  }
  uint32_t b0 = DIT ? 0 : K;
  static_for<0, NttRounds<KC>::n>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    constexpr uint32_t rb = NttRounds<KC>::bits(r);
    if (!DIT) b0 -= rb;
    constexpr bool first = r == 0, last = r + 1 == NttRounds<KC>::n;
    if (!first) tile_barrier();
    felt x[8];
    uint32_t ggs[2], qlow[2];
    // block-local coordinates (gg, q) of register m in this round (for thread tr)
    auto coord_gg = [&](int m, uint32_t tr) { return ((uint32_t)(m >> rb) << LOGNT | tr) & (T - 1); };
    auto coord_q = [&](int m, uint32_t tr) {
      uint32_t extra = m >> rb, bf = m & ((1u << rb) - 1);
      uint32_t qo = ((extra << LOGNT) | tr) >> logT;
      uint32_t ql = qo & ((1u << b0) - 1);
      return ((qo >> b0) << (b0 + rb)) | (bf << b0) | ql;
    };
    // the round: its inputs (HBM + coset scale, or LDS, which stays intact until
    // the barrier below), then its butterflies. It runs with the deferred-check
    // forms, and again with the exact ones when a lane of the wave saw a carry past
    // 2^128 or a top limb 0xffffffff: one scalar branch per round.
    // The exact pass derives every index from an opaque copy of the thread id, so
    // nothing it loads is shared with (and kept live across) the fast pass.
    auto round = [&](auto fast_c, Rare& qq) {
    constexpr bool FAST = decltype(fast_c)::value;
    uint32_t tr = tid;
    if constexpr (!FAST) asm volatile("" : "+v"(tr));
    const uint32_t zo = tr - tid;  // 0, opaque on the exact pass
#pragma unroll
    for (int m = 0; m < 8; m++) {
      uint32_t extra = m >> rb, bf = m & ((1u << rb) - 1);
      uint32_t c = (extra << LOGNT) | tr;
      if (first && !staged && !PIPE) {  // straight from HBM (coalesced along gg), coset scale fused
        uint32_t ad = gaddr(coord_gg(m, tr), coord_q(m, tr));
        felt v = NTT_LD(src + ad);
        if (scale) v = bmul<FAST>(v, NTT_LD(scale + ad), qq);
        x[m] = v;
      } else {
        x[m] = lds[lidx(coord_q(m, tr), coord_gg(m, tr))];
      }
      if (bf == 0 && extra < 2) { ggs[extra] = c & (T - 1); qlow[extra] = (c >> logT) & ((1u << b0) - 1); }
    }
    if constexpr (rb == 3) {
      const uint32_t l = l0 + (ggs[0] & (Tl - 1));
      const uint32_t jb = (qlow[0] << lo) | l;
      const uint32_t jstep = 1u << (b0 + lo);
      // stages 0..2 (b0 = 0, lo = 0, so jb = 0): 7 of the 12 products are by 1
      constexpr bool smallest = SMALL && (DIT ? first : last);
      if constexpr (DIT && smallest) {
        bfly1<true, FAST>(x[0], x[1], qq); bfly1<true, FAST>(x[2], x[3], qq); bfly1<true, FAST>(x[4], x[5], qq); bfly1<true, FAST>(x[6], x[7], qq);
        const felt w1 = ntt_tw<true>(a, 1 + zo, 1);
        bfly1<true, FAST>(x[0], x[2], qq); bfly1<true, FAST>(x[4], x[6], qq);
        bfly2<true, FAST>(x[1], x[3], w1, x[5], x[7], w1, qq);
        const felt w21 = ntt_tw<true>(a, 1 + zo, 2), w22 = ntt_tw<true>(a, 2 + zo, 2), w23 = ntt_tw<true>(a, 3 + zo, 2);
        bfly1<true, FAST>(x[0], x[4], qq);
        bfly2<true, FAST>(x[1], x[5], w21, x[2], x[6], w22, qq);
        bfly<true, FAST>(x[3], x[7], w23, qq);
      } else if constexpr (!DIT && smallest) {
        const felt w21 = ntt_tw<false>(a, 1 + zo, 2), w22 = ntt_tw<false>(a, 2 + zo, 2), w23 = ntt_tw<false>(a, 3 + zo, 2);
        bfly1<false, FAST>(x[0], x[4], qq);
        bfly2<false, FAST>(x[1], x[5], w21, x[2], x[6], w22, qq);
        bfly<false, FAST>(x[3], x[7], w23, qq);
        const felt w1 = ntt_tw<false>(a, 1 + zo, 1);
        bfly1<false, FAST>(x[0], x[2], qq); bfly1<false, FAST>(x[4], x[6], qq);
        bfly2<false, FAST>(x[1], x[3], w1, x[5], x[7], w1, qq);
        bfly1<false, FAST>(x[0], x[1], qq); bfly1<false, FAST>(x[2], x[3], qq); bfly1<false, FAST>(x[4], x[5], qq); bfly1<false, FAST>(x[6], x[7], qq);
      } else if constexpr (DIT) {
        {
          felt w0 = ntt_tw<true>(a, jb, b0);
          bfly2<true, FAST>(x[0], x[1], w0, x[2], x[3], w0, qq); bfly2<true, FAST>(x[4], x[5], w0, x[6], x[7], w0, qq);
        }
        {
          felt w1a = ntt_tw<true>(a, jb, b0 + 1);
          felt w1b = ntt_tw<true>(a, jb | jstep, b0 + 1);
          bfly2<true, FAST>(x[0], x[2], w1a, x[1], x[3], w1b, qq); bfly2<true, FAST>(x[4], x[6], w1a, x[5], x[7], w1b, qq);
        }
        static_for<0, 2>([&](auto k2) {
          felt w2a = ntt_tw<true>(a, jb | ((uint32_t)(2 * k2) << (b0 + lo)), b0 + 2);
          felt w2b = ntt_tw<true>(a, jb | ((uint32_t)(2 * k2 + 1) << (b0 + lo)), b0 + 2);
          bfly2<true, FAST>(x[2 * k2], x[2 * k2 + 4], w2a, x[2 * k2 + 1], x[2 * k2 + 5], w2b, qq);
        });
      } else {
        static_for<0, 2>([&](auto k2) {
          felt w2a = ntt_tw<false>(a, jb | ((uint32_t)(2 * k2) << (b0 + lo)), b0 + 2);
          felt w2b = ntt_tw<false>(a, jb | ((uint32_t)(2 * k2 + 1) << (b0 + lo)), b0 + 2);
          bfly2<false, FAST>(x[2 * k2], x[2 * k2 + 4], w2a, x[2 * k2 + 1], x[2 * k2 + 5], w2b, qq);
        });
        {
          felt w1a = ntt_tw<false>(a, jb, b0 + 1);
          felt w1b = ntt_tw<false>(a, jb | jstep, b0 + 1);
          bfly2<false, FAST>(x[0], x[2], w1a, x[1], x[3], w1b, qq); bfly2<false, FAST>(x[4], x[6], w1a, x[5], x[7], w1b, qq);
        }
        {
          felt w0 = ntt_tw<false>(a, jb, b0);
          bfly2<false, FAST>(x[0], x[1], w0, x[2], x[3], w0, qq); bfly2<false, FAST>(x[4], x[5], w0, x[6], x[7], w0, qq);
        }
      }
    } else if constexpr (rb == 2) {
      if constexpr (!DIT && SMALL && last) {  // DIF stages 1, 0: one product of four is not by 1
        const felt w1 = ntt_tw<false>(a, 1 + zo, 1);
#pragma unroll
        for (int u = 0; u < 2; u++) {
          felt* y = x + 4 * u;
          bfly1<false, FAST>(y[0], y[2], qq);
          bfly<false, FAST>(y[1], y[3], w1, qq);
          bfly1<false, FAST>(y[0], y[1], qq); bfly1<false, FAST>(y[2], y[3], qq);
        }
      } else {
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const uint32_t l = l0 + (ggs[u] & (Tl - 1));
        const uint32_t jb = (qlow[u] << lo) | l;
        felt w0 = ntt_tw<DIT>(a, jb, b0);
        felt w1a = ntt_tw<DIT>(a, jb, b0 + 1), w1b = ntt_tw<DIT>(a, jb | (1u << (b0 + lo)), b0 + 1);
        felt* y = x + 4 * u;
        if (DIT) {
          bfly2<true, FAST>(y[0], y[1], w0, y[2], y[3], w0, qq);
          bfly2<true, FAST>(y[0], y[2], w1a, y[1], y[3], w1b, qq);
        } else {
          bfly2<false, FAST>(y[0], y[2], w1a, y[1], y[3], w1b, qq);
          bfly2<false, FAST>(y[0], y[1], w0, y[2], y[3], w0, qq);
        }
      }
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        uint32_t c = ((uint32_t)u << LOGNT) | tr;
        uint32_t gg = c & (T - 1);
        uint32_t ql = (c >> logT) & ((1u << b0) - 1);
        const uint32_t jb = (ql << lo) | (l0 + (gg & (Tl - 1)));
        bfly<DIT, FAST>(x[2 * u], x[2 * u + 1], ntt_tw<DIT>(a, jb, b0), qq);
      }
    }
    };
    Rare qq;
    round(std::true_type{}, qq);
    if (qq.any()) round(std::false_type{}, qq);
    if (!last || staged) tile_barrier();  // everyone has read this round's slots
#pragma unroll
    for (int m = 0; m < 8; m++) {
      if (last && !staged) NTT_ST(dst + gaddr(coord_gg(m, tid), coord_q(m, tid)), x[m]);  // straight to HBM
      else lds[lidx(coord_q(m, tid), coord_gg(m, tid))] = x[m];
    }
    if (DIT) b0 += rb;
  });
  if (staged) {  // LDS -> HBM in the contiguous order
    tile_barrier();
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t slot;
      uint32_t ad = staged_elem(tid + i * NT, slot);
      NTT_ST(dst + ad, lds[slot]);
    }
  }
  (void)E;
}

// The 11-stage passes are held to 5 waves per SIMD (the DIT lo = 0 pass took 97 VGPRs, one
// over the 5-wave budget: 92 now, no spills; profiles/r06_ab_ntt_11stage_5waves.txt). The
// 6- and 7-stage passes would spill at 5 waves (100-116 VGPRs) and keep 4.
template <bool DIT, int NT, int KC, bool SMALL>
__global__ __launch_bounds__(NT, (NT == 256 && KC == 11) ? 5 : 1) void k_ntt8(Ntt8Args a) {
  extern __shared__ felt lds[];
  uint32_t bidx = blockIdx.x, tile = blockIdx.y;
  if (a.tile_major) {
    // dispatch order i = y * B + x goes round-robin over the 8 XCDs; XCD i % 8 takes
    // position blocks i % 8, i % 8 + 8, ... with all B batches of each back to back, so
    // the coefficient rows and the 8 cosets' scale rows of a block are fetched once
    const uint32_t B = gridDim.x, i = blockIdx.y * B + blockIdx.x, k = i >> 3;
    tile = (k / B) * 8 + (i & 7);
    bidx = k % B;
  }
  ntt8_tile<DIT, NT, KC, SMALL>(a, bidx, tile, lds);
}

// The 9-stage pass in rows of 8 felts (512 threads, 4096 felts per tile) with direct loads
// (2^20: DIT pass 2, DIF pass 1), software-pipelined: one persistent block per CU over the
// pass's tiles (item = tile * batches + batch, batch fastest as in k_ntt8), two 64-KB LDS
// buffers. While a tile's three rounds run, the next tile streams into the other buffer by
// LDS-DMA (global_load_lds_dwordx4: no VGPRs held, so the rounds keep their registers);
// the swizzle of k_ntt8's rows of 8 goes on the per-lane source address (the DMA writes a
// wave's 1 KB lane-linearly).
// TUNING BUILDS ONLY (ZKP_NTT_PIPE=1; not adopted): bit-exact, but
// 1.68 against 1.51 ms for the C2 composition-shape LDE (profiles/r06_ab_ntt_pipe_not_adopted.txt).
// The twiddle loads of the rounds are ordinary loads, beside which hipcc waits vmcnt(0) and
// so drains the prefetch; and even with the loads perfectly hidden, one 512-thread block per
// CU is 2 waves per SIMD, where the register-resident butterfly rate is 393 G/s against
// 430 G/s at the 4 waves the library's pass keeps (tests/native/ubench_bfly --occ,
// profiles/r06_ubench_bfly_occupancy.txt): no headroom left for the overlap to win.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;
template <bool DIT>
__global__ __launch_bounds__(512) void k_ntt8_pipe(Ntt8Args a) {
  extern __shared__ felt lds[];
  constexpr uint32_t NT = 512, K = 9, E = 4096, LOGNT = 9;
  const uint32_t B = a.batches, items = a.items, tid = threadIdx.x;
  // LDS-DMA of item `it` into buf: instruction i of wave w fills slots [(8i + w) * 64, +64);
  // slot s = P(q) * 8 + (gg ^ (q & 7)) (k_ntt8's rows-of-8 lidx, P(q) = q ^ ((q2 ^ q3) & 1),
  // an involution), so lane L loads the element whose slot is its own
  auto prefetch = [&](uint32_t it, felt* buf) {
    const uint32_t bidx = it % B, tile = it / B;
    const felt* src = a.src + (uint64_t)(bidx / a.src_div) * a.src_stride;
    const uint32_t g0 = tile << 3, hi0 = g0 >> a.lo, l0 = g0 & ((1u << a.lo) - 1);
    const uint32_t w = tid >> 6, L = tid & 63;
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
      const uint32_t s0 = (8 * i + w) * 64, sl = s0 + L, r = sl >> 3, c = sl & 7;
      const uint32_t q = r ^ (((r >> 2) ^ (r >> 3)) & 1u), gg = c ^ (q & 7u);
      const uint32_t ad = (hi0 << (a.lo + K)) + (q << a.lo) + l0 + gg;
      __builtin_amdgcn_global_load_lds((glob_void_t*)(src + ad), (lds_void_t*)(buf + s0), 16, 0, 0);
    }
  };
  uint32_t it = blockIdx.x;
  if (it < items) prefetch(it, lds);
  for (uint32_t k = 0; it < items; it += gridDim.x, k ^= 1) {
    felt* cur = lds + k * E;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's DMA (and the last tile's stores)
    lds_barrier();  // every wave's DMA landed; every wave is past the other buffer's last reads
    if (it + gridDim.x < items) prefetch(it + gridDim.x, lds + (k ^ 1) * E);
    ntt8_tile<DIT, NT, K, false, true>(a, it % B, it / B, cur);
  }
  (void)LOGNT;
}

}  // namespace

void preload_ntt_module() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, (const void*)k_ntt_pass);
}

std::vector<NttPass> ntt_plan(uint32_t logn, bool dit) {
  const uint32_t KMAX = 8, LOGE = 12;
  std::vector<NttPass> out;
  if (logn == 0) return out;
  uint32_t npass = (logn + KMAX - 1) / KMAX;
  // pass sizes: prefer multiples of 3 (whole radix-8 rounds), largest pass last
  uint32_t Ks[4] = {0, 0, 0, 0};
  {
    uint32_t rem = logn;
    for (uint32_t p = 0; p < npass; p++) {
      uint32_t left = npass - p;
      uint32_t k = (rem + left - 1) / left;
      if (left > 1) {
        uint32_t k3 = k / 3 * 3;  // round down to whole radix-8 rounds if the rest still fits
        if (k3 >= 3 && rem - k3 <= KMAX * (left - 1)) k = k3;
      }
      Ks[p] = k;
      rem -= k;
    }
  }
  uint32_t s0 = 0;
  for (uint32_t p = 0; p < npass; p++) {
    uint32_t K = Ks[p];
    NttPass ps;
    ps.logn = logn;
    ps.s0 = s0;
    ps.K = K;
    ps.lo = dit ? s0 : logn - s0 - K;
    uint32_t logG = logn - K;
    uint32_t logT = LOGE - K < logG ? LOGE - K : logG;
    uint32_t logTl = logT < ps.lo ? logT : ps.lo;
    ps.T = 1u << logT;
    ps.Tl = 1u << logTl;
    out.push_back(ps);
    s0 += K;
  }
  return out;
}

static void launch_ntt_radix2(Prof& prof, hipStream_t s, const NttBatch& b, uint32_t logn, bool dit,
                              const felt* tw, uint32_t logN) {
  auto plan = ntt_plan(logn, dit);
  bool first = true;
  for (const auto& ps : plan) {
    NttKArgs a;
    a.src = first ? b.src : b.dst;
    a.dst = b.dst;
    a.scale = first ? b.scale : nullptr;
    a.tw = tw;
    a.src_stride = first ? b.src_stride : b.dst_stride;
    a.dst_stride = b.dst_stride;
    a.src_div = first ? b.src_div : 1;
    a.scale_mod = b.scale_mod ? b.scale_mod : 1;
    a.logn = logn;
    a.s0 = ps.s0;
    a.K = ps.K;
    a.lo = ps.lo;
    a.T = ps.T;
    a.Tl = ps.Tl;
    a.logT = kc::ilog2_u64(ps.T);
    a.logTl = kc::ilog2_u64(ps.Tl);
    a.tw_shift = logN - logn;
    a.dit = dit ? 1 : 0;
    uint64_t groups = 1ull << (logn - ps.K);
    dim3 grid((uint32_t)(groups / ps.T), b.batches);
    size_t shmem = (size_t)(ps.T << ps.K) * sizeof(felt);
    LAUNCH(prof, dit ? "ntt_dit_r2" : "ntt_dif_r2", s, (double)b.batches * (1ull << logn) * 16.0 * (a.scale ? 3 : 2),
           hipLaunchKernelGGL(k_ntt_pass, grid, dim3(TPB), shmem, s, a));
    first = false;
  }
}

// radix-8 register-blocked passes: 256-thread blocks (E = 2048 elements, K <= 8)
// for the big transforms (several blocks per CU overlap load and compute);
// n must be >= 2^11.
#ifndef ZKP_NTT_PIPE
#define ZKP_NTT_PIPE 0  // tuning builds set 1 (k_ntt8_pipe for the 9-stage direct-load passes)
#endif
#ifndef ZKP_NTT_ONE_PASS_MAX
#define ZKP_NTT_ONE_PASS_MAX 11  // (tuning builds set 13: see one_pass in launch_ntt)
#endif

uint32_t ntt_passes(uint32_t logn) {
  if (logn < 11 || logn <= ZKP_NTT_ONE_PASS_MAX) return 1;
  if (logn == 19 || logn == 20) return 2;
#ifdef ZKP_NTT_PLAN22
  if (logn == 21 || logn == 22) return ZKP_NTT_PLAN22 == 1165 ? 3 : 2;
#endif
#ifdef ZKP_NTT_KFIRST
  if (logn >= 12 && logn <= 16 && logn - ZKP_NTT_KFIRST >= 5 && logn - ZKP_NTT_KFIRST <= 9) return 2;
#endif
  const uint32_t KMAX = (logn == 17 || logn == 18) ? 9 : 8;
  return (logn + KMAX - 1) / KMAX;
}

void launch_ntt(Prof& prof, hipStream_t s, const NttBatch& b, uint32_t logn, bool dit, const felt* tw,
                uint32_t logN, int only_pass) {
  const uint32_t LOGE = 11;
  // passes of up to KMAX stages. 2^17-2^18 run two passes of <= 9 stages instead
  // of three: 9-stage passes use 512-thread blocks of 4096 elements (64 KB LDS,
  // 2 blocks per CU = the same 4 waves/SIMD as 256-thread blocks; strided groups
  // still load 8-felt runs), a third less HBM traffic for the same rounds.
  // (10-stage passes for 2^19-2^20 — 512-thread blocks with rows of 4 felts, the
  // T = 4 layout of k_ntt8's lidx — measured slower than 6+6+8: DESIGN.md §4.)
  const uint32_t KMAX = (logn == 17 || logn == 18) ? 9 : 8;
  // 2^19-2^20: two passes in 256-thread blocks, 11 stages over one contiguous
  // 2048-element group per block (the pass with lo = 0: rows of 1 felt, staged through
  // LDS) and the rest (8 or 9 stages) over 8 or 4 adjacent groups per block: 7 LDS rounds
  // as before (3+3+3+2 | 3+3(+3)) and a third less HBM traffic than 6+6+8
  // (tests/native/kbench_ntt.cpp: with the butterflies compiled out the 6+6+8 passes
  // take 1.13 of the 1.65 ms of a 48-array 2^20 LDE, about three copies of the data).
  // Round 6: 2^17-2^18 as 11 + 6/7 too (instead of 9 + 8/9 in 512-thread blocks): the 11-stage
  // pass runs 5 waves per SIMD against the 9-stage pass's 4 (tests/native/kbench_ntt 18: the
  // 48-array LDE 0.368 -> 0.352 ms, the DIF 0.065 -> 0.057; profiles/r06_ab_ntt_11_7_2e18.txt)
#ifndef ZKP_NTT_TWO11_LOW
#define ZKP_NTT_TWO11_LOW 1  // tuning builds set 0: the 9 + 8/9 plan
#endif
  const bool two11 = logn == 19 || logn == 20 || (ZKP_NTT_TWO11_LOW && (logn == 17 || logn == 18));
  // 2^11: the whole transform in one 11-stage pass (one array per 256-thread block, rows
  // of 1 felt): one HBM read and write per array instead of 6 + 5 stages' two.
  // (2^13 in one 1024-thread pass — 128 KB of LDS, one block per CU — was slower than
  // 6 + 7 on the reference's TrainingUpdate proof, 2^13 x 240 at blowup 16: ntt_dit
  // 0.76 -> 0.83 ms per proof, BENCH reference_flow.training_proof_profile; the 12- and
  // 13-stage kernels stay for tuning builds, ZKP_NTT_ONE_PASS_MAX)
  const bool one_pass = logn >= 11 && logn <= ZKP_NTT_ONE_PASS_MAX;
  if (logN > 28)  // k_ntt8 indexes arrays and twiddles with 32-bit element offsets
    launch_fail(ZKP_ERR_TRACE_SHAPE, "NTT domain over 2^28 points (n * blowup)");
  if (logn < LOGE) {
    if (only_pass <= 0) launch_ntt_radix2(prof, s, b, logn, dit, tw, logN);
    return;
  }
  uint32_t npass = one_pass ? 1 : two11 ? 2 : (logn + KMAX - 1) / KMAX;
  // the dynamic-LDS attributes are per device: set them once for each device this
  // process launches on (threads of an in-process group drive different devices)
  static std::mutex attr_mu;
  static uint64_t attr_devs = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  {
  std::lock_guard<std::mutex> attr_lock(attr_mu);
  if (!(attr_devs >> (dev & 63) & 1)) {
    size_t maxb = (size_t)(1u << LOGE) * sizeof(felt);
    const void* fns[] = {
        (const void*)k_ntt8<true, 256, 5, false>,  (const void*)k_ntt8<true, 256, 6, false>,
        (const void*)k_ntt8<true, 256, 7, false>,  (const void*)k_ntt8<true, 256, 8, false>,
        (const void*)k_ntt8<false, 256, 5, false>, (const void*)k_ntt8<false, 256, 6, false>,
        (const void*)k_ntt8<false, 256, 7, false>, (const void*)k_ntt8<false, 256, 8, false>,
        (const void*)k_ntt8<true, 256, 5, true>,   (const void*)k_ntt8<true, 256, 6, true>,
        (const void*)k_ntt8<true, 256, 7, true>,   (const void*)k_ntt8<true, 256, 8, true>,
        (const void*)k_ntt8<false, 256, 5, true>,  (const void*)k_ntt8<false, 256, 6, true>,
        (const void*)k_ntt8<false, 256, 7, true>,  (const void*)k_ntt8<false, 256, 8, true>,
        (const void*)k_ntt8<true, 256, 9, false>,  (const void*)k_ntt8<false, 256, 9, false>,
        (const void*)k_ntt8<true, 256, 11, true>,  (const void*)k_ntt8<false, 256, 11, true>,
        (const void*)k_ntt8<true, 256, 9, true>,   (const void*)k_ntt8<false, 256, 9, true>,
        (const void*)k_ntt8<true, 256, 11, false>, (const void*)k_ntt8<false, 256, 11, false>};
    for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)maxb);
    const void* k9[] = {(const void*)k_ntt8<true, 512, 9, false>,  (const void*)k_ntt8<false, 512, 9, false>,
                        (const void*)k_ntt8<true, 512, 9, true>,   (const void*)k_ntt8<false, 512, 9, true>};
    for (const void* f : k9) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 16);
    const void* k7[] = {(const void*)k_ntt8<true, 512, 7, false>, (const void*)k_ntt8<false, 512, 7, false>,
                        (const void*)k_ntt8<true, 512, 7, true>, (const void*)k_ntt8<false, 512, 7, true>};
    for (const void* f : k7) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 16);
    const void* k12[] = {(const void*)k_ntt8<true, 512, 12, true>, (const void*)k_ntt8<false, 512, 12, true>};
    for (const void* f : k12) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 16);
#ifdef ZKP_NTT_PLAN22
    const void* k10[] = {(const void*)k_ntt8<true, 512, 10, false>, (const void*)k_ntt8<false, 512, 10, false>,
                         (const void*)k_ntt8<true, 512, 10, true>, (const void*)k_ntt8<false, 512, 10, true>};
    for (const void* f : k10) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 16);
#endif
#if ZKP_NTT_PIPE
    const void* kp[] = {(const void*)k_ntt8_pipe<true>, (const void*)k_ntt8_pipe<false>};
    for (const void* f : kp) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 4096 * 16);
#endif
    const void* k13[] = {(const void*)k_ntt8<true, 1024, 13, true>, (const void*)k_ntt8<false, 1024, 13, true>};
    for (const void* f : k13) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 * 16);
    attr_devs |= 1ull << (dev & 63);
  }
  }
  // pass sizes: prefer multiples of 3 (whole radix-8 rounds), largest pass last
  uint32_t Ks[4] = {0, 0, 0, 0};
#ifdef ZKP_NTT_PLAN22  // tuning builds only (tests/native kbench22): 2^21-2^22 in two passes, 12 + 9/10 or 11 + 10/11
  if ((logn == 21 || logn == 22) && ZKP_NTT_PLAN22 == 1165) {  // 11 + 6 + 5/4
    npass = 3;
    const uint32_t k1 = 6, k2 = logn - 17;
    Ks[0] = dit ? 11 : k2;
    Ks[1] = k1;
    Ks[2] = dit ? k2 : 11;
  } else if (logn == 21 || logn == 22) {
    npass = 2;
    const uint32_t k0 = ZKP_NTT_PLAN22 == 1210 ? 12 : 11;  // the lo = 0 pass
    Ks[0] = dit ? k0 : logn - k0;
    Ks[1] = dit ? logn - k0 : k0;
  } else
#endif
#ifdef ZKP_NTT_KFIRST  // tuning builds only (tests/native kbench13): the lo = 0 pass takes KFIRST stages
  if (!one_pass && !two11 && logn >= 12 && logn <= 16 && logn - ZKP_NTT_KFIRST >= 5 && logn - ZKP_NTT_KFIRST <= 9) {
    npass = 2;
    Ks[0] = dit ? ZKP_NTT_KFIRST : logn - ZKP_NTT_KFIRST;
    Ks[1] = dit ? logn - ZKP_NTT_KFIRST : ZKP_NTT_KFIRST;
  } else
#endif
  if (one_pass) {
    Ks[0] = logn;
  } else if (two11) {  // the 11-stage pass is the one with lo = 0: first for DIT, last for DIF
    Ks[0] = dit ? 11 : logn - 11;
    Ks[1] = dit ? logn - 11 : 11;
  } else {
    uint32_t rem = logn;
    for (uint32_t p = 0; p < npass; p++) {
      uint32_t left = npass - p;
      uint32_t k = (rem + left - 1) / left;
      if (left > 1) {
        uint32_t k3 = k / 3 * 3;  // round down to whole radix-8 rounds if the rest still fits
        if (k3 >= 3 && rem - k3 <= KMAX * (left - 1)) k = k3;
      }
      Ks[p] = k;
      rem -= k;
    }
  }
  if (npass != ntt_passes(logn)) launch_fail(ZKP_ERR_DEVICE, "internal: NTT pass count");
  uint32_t s0 = 0;
  for (uint32_t p = 0; p < npass; s0 += Ks[p], p++) {
    uint32_t K = Ks[p];
    if (only_pass >= 0 && (uint32_t)only_pass != p) continue;
    // 9 stages: 512 threads x 8 = 4096 elements, rows of 8 felts = whole 128-B lines
    // (64 KB: 2 blocks per CU, the same 4 waves per SIMD as the 256-thread 9-stage pass,
    // whose 64-B runs cost 1.7x their bytes in L2 fetches: profiles/r05_ab_ntt_k512_tmaj.txt);
    // 11 stages: 256-thread blocks of one group (rows of 1)
    // (2^19-2^20 with < 8 arrays, e.g. a sharded rank's 2-column interpolation rounds beside
    // its LDE: the 64-KB blocks wait for LDS next to the other stream's kernels — C5 rank
    // ntt_dif 0.75 -> 2.04 ms, profiles/r05_ab_rank_c5_ntt9.txt — so those keep 256 threads)
    // 7 stages beside an 11-stage pass (2^18): 256-thread blocks, rows of 16 felts (the DIF
    // rounds take lidx's rows-of-16 DIF swizzle)
#ifdef ZKP_NTT_K7_512
    // tuning builds: 2^18's 7-stage pass in 512-thread blocks (rows of 32, no LDS bank
    // conflicts) -- the DIF pass measured 0.0571 -> 0.0606 ms at 2^18 x 6 arrays (half as
    // many workgroups), DIT unchanged: profiles/r06_kbench_ntt_k7.txt
    const bool k7_512 = K == 7 && two11 && logn == 18;
#else
    const bool k7_512 = false;
#endif
    const uint32_t lognt = one_pass ? logn - 3
                           : (K == 12 || K == 10 || k7_512) ? 9
                           : K == 9 && (!two11 || b.batches >= 8) ? 9 : 8,
                   loge = lognt + 3;
    Ntt8Args a;
    bool first = p == 0;
    a.src = first ? b.src : b.dst;
    a.dst = b.dst;
    a.scale = first ? b.scale : nullptr;
    a.tw = tw;
    a.src_stride = first ? b.src_stride : b.dst_stride;
    a.dst_stride = b.dst_stride;
    a.src_div = first ? b.src_div : 1;
    a.scale_mod = b.scale_mod ? b.scale_mod : 1;
    a.logn = logn;
    a.s0 = s0;
    a.K = K;
    a.lo = dit ? s0 : logn - s0 - K;
    a.logT = loge - K;
    a.logTl = a.logT < a.lo ? a.logT : a.lo;
    a.tw_shift = logN - logn;
    // rounds of <= 3 bits, larger first
    uint32_t nr = (K + 2) / 3, rem = K;
    a.nrounds = nr;
    for (uint32_t r = 0; r < 4; r++) a.rbits[r] = 0;
    for (uint32_t r = 0; r < nr; r++) {
      uint32_t rb = rem / (nr - r) + (rem % (nr - r) ? 1 : 0);
      if (rb > 3) rb = 3;
      a.rbits[r] = rb;
      rem -= rb;
    }
    uint64_t groups = 1ull << (logn - K);
    dim3 grid(b.batches, (uint32_t)(groups >> a.logT));  // batch fastest (see k_ntt8)
    // the coset LDE's first pass reads each coefficient row for 8 cosets: whole position
    // blocks per XCD (k_ntt8) keep those reads, and the scale rows, to one fetch
    a.tile_major = first && b.src_div > 1 && grid.y % 8 == 0;
    size_t shmem = (size_t)(1u << K) * (1u << a.logT) * sizeof(felt);
    // compulsory bytes of this launch: every distinct input array once (the
    // coefficient arrays are shared by src_div coset batches, the scale table
    // has scale_mod rows) + every output once
    const double arr = (double)(1ull << logn) * 16.0;
    const uint32_t src_arrays = first ? (b.batches + a.src_div - 1) / a.src_div : b.batches;
    const uint32_t scale_rows = a.scale ? (a.scale_mod < b.batches ? a.scale_mod : b.batches) : 0;
    const double bytes = arr * ((double)src_arrays + scale_rows + b.batches);
    // the pass over stages 0..2 (lo = 0): the trivial-twiddle variant
    const bool small = a.lo == 0;
    a.batches = b.batches;
    a.items = grid.x * grid.y;
#if ZKP_NTT_PIPE
    // the 9-stage direct-load pass in rows of 8, software-pipelined (k_ntt8_pipe): one
    // persistent block per CU
    if (K == 9 && lognt == 9 && !a.scale && a.logT == 3 && a.logTl == 3 && !a.tile_major) {
      static int cus = 0;
      if (!cus) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const uint32_t blocks = std::min<uint32_t>(a.items, cus > 0 ? (uint32_t)cus : 256u);
      LAUNCH(prof, dit ? "ntt_dit" : "ntt_dif", s, bytes,
             if (dit) hipLaunchKernelGGL(k_ntt8_pipe<true>, dim3(blocks), dim3(512), 2 * shmem, s, a);
             else hipLaunchKernelGGL(k_ntt8_pipe<false>, dim3(blocks), dim3(512), 2 * shmem, s, a));
      continue;
    }
#endif
#define ZKP_NTT8(D, NTT, KK)                                                                                   \
  LAUNCH(prof, D ? "ntt_dit" : "ntt_dif", s, bytes,                                                           \
         if (small) hipLaunchKernelGGL((k_ntt8<D, NTT, KK, true>), grid, dim3(NTT), shmem, s, a);              \
         else hipLaunchKernelGGL((k_ntt8<D, NTT, KK, false>), grid, dim3(NTT), shmem, s, a))
    switch (K * 2 + (dit ? 1 : 0)) {
      case 11: ZKP_NTT8(true, 256, 5); break;
      case 13: ZKP_NTT8(true, 256, 6); break;
      case 15: if (lognt == 9) ZKP_NTT8(true, 512, 7); else ZKP_NTT8(true, 256, 7); break;
      case 17: ZKP_NTT8(true, 256, 8); break;
      case 10: ZKP_NTT8(false, 256, 5); break;
      case 12: ZKP_NTT8(false, 256, 6); break;
      case 14: if (lognt == 9) ZKP_NTT8(false, 512, 7); else ZKP_NTT8(false, 256, 7); break;
      case 16: ZKP_NTT8(false, 256, 8); break;
      case 19: if (lognt == 8) ZKP_NTT8(true, 256, 9); else ZKP_NTT8(true, 512, 9); break;
      case 18: if (lognt == 8) ZKP_NTT8(false, 256, 9); else ZKP_NTT8(false, 512, 9); break;
#ifdef ZKP_NTT_PLAN22
      case 21: ZKP_NTT8(true, 512, 10); break;
      case 20: ZKP_NTT8(false, 512, 10); break;
      case 23: ZKP_NTT8(true, 256, 11); break;
      case 22: ZKP_NTT8(false, 256, 11); break;
#else
      case 23: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 11-stage NTT pass off lo = 0");
               ZKP_NTT8(true, 256, 11); break;
      case 22: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 11-stage NTT pass off lo = 0");
               ZKP_NTT8(false, 256, 11); break;
#endif
      case 25: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 12-stage NTT pass off lo = 0");
               LAUNCH(prof, "ntt_dit", s, bytes,
                      hipLaunchKernelGGL((k_ntt8<true, 512, 12, true>), grid, dim3(512), shmem, s, a)); break;
      case 24: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 12-stage NTT pass off lo = 0");
               LAUNCH(prof, "ntt_dif", s, bytes,
                      hipLaunchKernelGGL((k_ntt8<false, 512, 12, true>), grid, dim3(512), shmem, s, a)); break;
      case 27: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 13-stage NTT pass off lo = 0");
               LAUNCH(prof, "ntt_dit", s, bytes,
                      hipLaunchKernelGGL((k_ntt8<true, 1024, 13, true>), grid, dim3(1024), shmem, s, a)); break;
      case 26: if (!small) launch_fail(ZKP_ERR_DEVICE, "internal: 13-stage NTT pass off lo = 0");
               LAUNCH(prof, "ntt_dif", s, bytes,
                      hipLaunchKernelGGL((k_ntt8<false, 1024, 13, true>), grid, dim3(1024), shmem, s, a)); break;
      default: launch_fail(ZKP_ERR_DEVICE, "internal: NTT pass of an unplanned size");
    }
#undef ZKP_NTT8
  }
}
