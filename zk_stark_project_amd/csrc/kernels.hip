// kernels.hip — CDNA4 (gfx950) kernels of the STARK prover hot path: domain
// tables, constraint evaluation, composition DFT, OOD, DEEP, gathers and the
// aggregation trace builder (BLAKE3 / Merkle / transcript / FRI: merkle.hip).
//
// All arithmetic is exact f128 integer arithmetic, so results are
// order-independent and bit-identical to the CPU restatement in oracle/.
// Layouts (see DESIGN.md "Data layout in HBM"):
//  * coefficient arrays: bit-reversed order, scaled by n (output of the
//    Gentleman-Sande inverse NTT, never permuted);
//  * LDE matrices: coset-major, column c, coset j, row t at (c*B + j)*n + t,
//    holding P_c(g * w_N^j * w_n^t) = LDE index i = j + B*t. A shard owns the
//    cosets [j0, j0 + Bl) and stores them the same way with B -> Bl, j -> j - j0;
//  * DEEP / FRI layer evaluations: coset-major too (coset j, position t);
//  * Merkle trees: nodes[1..2L) of 8-word digests, leaves at nodes[L..2L).
#include "kernels_dev.hpp"

using kc::rev_bits;
using kc::static_for;

namespace {

// ------------------------------------------------------------------ tables
__global__ void k_expand_powers(felt* out, uint64_t count, const felt* lo_tab, const felt* hi_tab) {
  for (uint64_t e = blockIdx.x * (uint64_t)TPB + threadIdx.x; e < count; e += (uint64_t)gridDim.x * TPB)
    out[e] = mul(lo_tab[e & 2047], hi_tab[e >> 11]);
}

// stage-major table: level t (< top) = top level gathered with stride 2^(top - t)
__global__ void k_build_levels(felt* tab, uint32_t top) {
  const felt* topl = tab + ((1ull << top) - 1);
  uint64_t total = (1ull << top) - 1;  // entries of levels 0..top-1
  for (uint64_t e = blockIdx.x * (uint64_t)TPB + threadIdx.x; e < total; e += (uint64_t)gridDim.x * TPB) {
    uint32_t t = 63 - __builtin_clzll(e + 1);
    uint64_t j = e + 1 - (1ull << t);
    tab[e] = topl[j << (top - t)];
  }
}

__global__ void k_build_coset_scale(felt* S, uint32_t logn, uint32_t B, const felt* tw, uint32_t logN,
                                    const felt* glo, const felt* ghi, felt ninv) {
  uint64_t total = (uint64_t)B << logn;
  for (uint64_t idx = blockIdx.x * (uint64_t)TPB + threadIdx.x; idx < total; idx += (uint64_t)gridDim.x * TPB) {
    uint64_t j = idx >> logn;
    uint32_t p = (uint32_t)(idx & ((1ull << logn) - 1));
    uint32_t k = rev_bits(p, logn);
    felt gk = mul(glo[k & 2047], ghi[k >> 11]);
    S[idx] = mul(ninv, mul(gk, tw_full(tw, j * k, logN)));
  }
}


// ---- composition polynomial from CE-coset evaluations.
// recv: slices [pl0, pl0 + nR) (bit-reversed positions p) of the CE cosets'
// Gentleman-Sande inverse NTTs (position p holds n * V_u[rev(p)]); blk[u] =
// receive block of CE coset u. Si[u*n + p] = (g w_M^u)^-rev(p) turns them into
// n * U_u[rev(p)], and n * c_m[rev(p)] = (sum_u n U_u w_ce^-um) * g^-mn / ce: a
// CE-point inverse DFT per position (radix-2 in registers, compile-time indices)
// and one scale per kept column. consts = [g^-mn / ce for m < C | w_ce^-k for k < CE/2].
// out[m*nR + pl]: the bit-reversed, n-scaled coefficient layout of the LDE input
// (directly the columns when nR = n).
template <int CE>
__global__ __launch_bounds__(TPB) void k_comp_dft(const felt* __restrict__ recv, const uint32_t* __restrict__ blk,
                                                  const felt* __restrict__ Si, const felt* __restrict__ consts,
                                                  uint32_t C, uint32_t logn, uint64_t p0, uint64_t nR,
                                                  felt* __restrict__ out, uint32_t* __restrict__ hi_flag) {
  const uint64_t pl = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (pl >= nR) return;
  felt x[CE];
  static_for<0, CE>([&](auto uu) {
    constexpr int u = decltype(uu)::value;
    x[u] = mul(recv[blk[u] * nR + pl], Si[((uint64_t)u << logn) + p0 + pl]);
  });
  const felt* winv = consts + C;
  // Gentleman-Sande: natural in, bit-reversed out; x[rev(m)] = sum_u U_u w_ce^-um
  static_for<0, kc::ilog2_const(CE)>([&](auto ss) {
    constexpr int len = CE >> decltype(ss)::value, h = len / 2;
    static_for<0, CE / len>([&](auto bb) {
      constexpr int b0 = decltype(bb)::value * len;
      static_for<0, h>([&](auto jj) {
        constexpr int j = decltype(jj)::value;
        const felt u = x[b0 + j], v = x[b0 + j + h];
        x[b0 + j] = add(u, v);
        x[b0 + j + h] = j == 0 ? sub(u, v) : mul(sub(u, v), winv[j * (CE / len)]);
      });
    });
  });
  static_for<0, CE>([&](auto mm) {
    constexpr int m = decltype(mm)::value;
    if ((uint32_t)m < C) out[m * nR + pl] = mul(x[kc::rev_const(m, kc::ilog2_const(CE))], consts[m]);
  });
  // segments C..CE-1 of the interpolated polynomial, which CompositionPoly::new's
  // segment() drops (`.take(num_cols)`): zero for a trace that satisfies its
  // constraints. A derived last column (LastCol) equals winterfell's only then, so
  // any nonzero one raises the flag and the proof is made again without it.
  if (hi_flag) {
    uint32_t nz = 0;
    static_for<0, CE>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      const felt v = x[kc::rev_const(m, kc::ilog2_const(CE))];
      if ((uint32_t)m >= C) nz |= (uint32_t)((v.lo | v.hi) != 0);
    });
    if (__builtin_amdgcn_ballot_w64(nz != 0) && (threadIdx.x & 63) == 0) hi_flag[0] = 1u;
  }
}

// coefficient-dependent constants of the constraint evaluation kernels, from cc:
//  MIMC  : out[u] = zinv[u] * cc[0] (u < ce), out[ce] = cc[1], out[ce+1] = cc[2]
//  GLOBAL_UPDATE (w = 120): out[0..4w) = lin coefs, out[4w] = sum_c cc[num_t+c]*aval[c], out[4w+1] = 0
//  TRAINING_UPDATE (half = w/2): out[0..4half) = lin coefs, out[4half] / [4half+1] = the two boundary sums
__global__ __launch_bounds__(TPB) void k_dt_eval_consts(int air, const felt* __restrict__ cc, felt k, felt wl,
                                                        const felt* __restrict__ aval, const felt* __restrict__ zinv,
                                                        uint32_t ce, uint32_t w, uint32_t num_t,
                                                        felt* __restrict__ out) {
  __shared__ felt red0[TPB], red1[TPB];
  const uint32_t t = threadIdx.x;
  if (air == ZKP_AIR_MIMC) {
    for (uint32_t u = t; u < ce; u += TPB) out[u] = mul(zinv[u], cc[0]);
    // the boundary numerator b0 (cur - v0)(x - wl) + b1 (cur - v1)(x - 1)
    //   = cur (x A - Bc) - x Cc + D,  A = b0 + b1, Bc = b0 wl + b1,
    //   Cc = b0 v0 + b1 v1, D = b0 v0 wl + b1 v1  (three products per point, not four)
    if (t == 0) {
      const felt b0 = cc[1], b1 = cc[2], c0 = mul(b0, aval[0]), c1 = mul(b1, aval[1]);
      out[ce] = add(b0, b1);
      out[ce + 1] = add(mul(b0, wl), b1);
      out[ce + 2] = add(c0, c1);
      out[ce + 3] = add(mul(c0, wl), c1);
    }
    return;
  }
  const bool gu = air == ZKP_AIR_GLOBAL_UPDATE;
  const uint32_t W = gu ? w : w / 2;  // columns the kernel reads
  felt s0 = zero(), s1 = zero();
  for (uint32_t c = t; c < W; c += TPB) {
    felt a = zero(), b = zero(), b0 = zero(), b1 = zero();
    if (gu) {
      const uint32_t d = W / 2;  // 60 state columns, then 60 update columns
      if (c < d) { a = mul(cc[c], k); b = neg(a); }
      else a = neg(cc[c - d]);
      b0 = cc[num_t + c];
      s0 = add(s0, mul(b0, aval[c]));
    } else {
      b0 = cc[num_t + c];
      b1 = cc[num_t + W + c];
      s0 = add(s0, mul(b0, aval[c]));
      s1 = add(s1, mul(b1, aval[W + c]));
    }
    out[c] = a;
    out[W + c] = b;
    out[2 * W + c] = b0;
    out[3 * W + c] = b1;
  }
  red0[t] = s0;
  red1[t] = s1;
  __syncthreads();
  for (uint32_t h = TPB / 2; h >= 1; h >>= 1) {
    if (t < h) { red0[t] = add(red0[t], red0[t + h]); red1[t] = add(red1[t], red1[t + h]); }
    __syncthreads();
  }
  if (t == 0) { out[4 * W] = red0[0]; out[4 * W + 1] = red1[0]; }
}

// -------------------------------------------------------------- constraints

// Inverts v[0..EVAL_CH) of every thread of the block given the inverse of the
// product of all of the block's values (Montgomery's trick over thread-local
// prefixes + two LDS scans).
// Entries with k >= cnt must hold 1. Every thread of the block must call it.
__device__ __forceinline__ void block_batch_inverse(felt* v, felt* s_pre, felt* s_suf, felt block_inv) {
  felt pre[EVAL_CH];
  felt acc = one();
  static_for<0, EVAL_CH>([&](auto i) {
    pre[i] = acc;
    acc = mul(acc, v[i]);
  });
  const uint32_t t = threadIdx.x;
  s_pre[t] = acc;
  s_suf[t] = acc;
  __syncthreads();
  // inclusive scans: prefix (from the left) and suffix (from the right)
  for (uint32_t d = 1; d < TPB; d <<= 1) {
    felt a = t >= d ? s_pre[t - d] : one();
    felt b = t + d < TPB ? s_suf[t + d] : one();
    __syncthreads();
    s_pre[t] = mul(s_pre[t], a);
    s_suf[t] = mul(s_suf[t], b);
    __syncthreads();
  }
  // inv(acc_t) = inv(total) * prefix_excl(t) * suffix_excl(t); inv(total) was
  // computed by k_den_products + k_invert_products (one inversion per launch)
  felt ia = block_inv;
  if (t > 0) ia = mul(ia, s_pre[t - 1]);
  if (t + 1 < TPB) ia = mul(ia, s_suf[t + 1]);
  static_for<0, EVAL_CH>([&](auto ii) {
    constexpr int i = EVAL_CH - 1 - decltype(ii)::value;
    felt r = mul(ia, pre[i]);
    ia = mul(ia, v[i]);
    v[i] = r;
  });
}

// Phase 1 of the split batch inversion: product of the denominators
// (x_q - c0)(x_q - c1) (or (x_q - c0) when !two) of each block's EVAL_CH*TPB
// local points q (EVAL_POINT), x_q = point_x(m, q). Same point->block mapping
// as the phase-3 kernels.
// With pw (DEEP: pw[l] = c0^(2^l), pw[logn + l] = c1^(2^l)), block 0 also writes
// the inverse of the product over ALL points to *tinv, from the closed form
// prod_t (cx_j w_n^t - c) = c^n - cx_j^n per coset (n even): prod_j (c0^n -
// cx_j^n)(c1^n - cx_j^n). Its field inversion then runs beside the other
// blocks instead of after them in k_invert_products.
__global__ __launch_bounds__(TPB) void k_den_products(PointMap m, uint64_t count, felt c0, felt c1, int two,
                                                      const felt* __restrict__ cdev, const felt* __restrict__ pw,
                                                      felt* __restrict__ tinv, felt* __restrict__ prod) {
  __shared__ felt s[TPB];
  if (cdev) {  // points drawn on the device (DEEP: z, z*w_n)
    c0 = cdev[0];
    c1 = cdev[1];
  }
  if (pw && blockIdx.x == 0) {
    const uint32_t ncos = (uint32_t)(count >> m.logn);
    const felt zn = sqr(pw[m.logn - 1]), zgn = sqr(pw[2 * m.logn - 1]);
    felt acc = one();
    for (uint32_t j = threadIdx.x; j < ncos; j += TPB) {
      felt cn = m.cx[j];
      for (uint32_t l = 0; l < m.logn; l++) cn = sqr(cn);
      acc = mul(acc, mul(sub(zn, cn), sub(zgn, cn)));
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t h = TPB / 2; h >= 1; h >>= 1) {
      if (threadIdx.x < h) s[threadIdx.x] = mul(s[threadIdx.x], s[threadIdx.x + h]);
      __syncthreads();
    }
    if (threadIdx.x == 0) *tinv = inv(s[0]);
    __syncthreads();
  }
  felt acc = one();
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    if (q < count) {
      felt x = point_x(m, q);
      felt d = sub(x, c0);
      if (two) d = mul(d, sub(x, c1));
      acc = mul(acc, d);
    }
  });
  s[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t h = TPB / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) s[threadIdx.x] = mul(s[threadIdx.x], s[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) prod[blockIdx.x] = s[0];
}

// Phase 2: invert all block products in place with one field inversion (or
// none: tinv = the inverse of their product, precomputed by k_den_products).
__global__ __launch_bounds__(1024) void k_invert_products(felt* prod, uint32_t nb, const felt* __restrict__ tinv) {
  __shared__ felt s_pre[1024], s_suf[1024];
  __shared__ felt s_inv;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nb + 1023) / 1024;
  felt acc = one();
  for (uint32_t i = 0; i < per; i++) {
    uint32_t j = t * per + i;
    if (j < nb) acc = mul(acc, prod[j]);
  }
  s_pre[t] = acc;
  s_suf[t] = acc;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    felt a = t >= d ? s_pre[t - d] : one();
    felt b = t + d < 1024 ? s_suf[t + d] : one();
    __syncthreads();
    s_pre[t] = mul(s_pre[t], a);
    s_suf[t] = mul(s_suf[t], b);
    __syncthreads();
  }
  if (t == 0) s_inv = tinv ? *tinv : inv(s_pre[1023]);
  __syncthreads();
  felt ia = s_inv;
  if (t > 0) ia = mul(ia, s_pre[t - 1]);
  if (t + 1 < 1024) ia = mul(ia, s_suf[t + 1]);
  // back-substitute this thread's run (recomputing its prefix products)
  for (uint32_t i = per; i-- > 0;) {
    uint32_t j = t * per + i;
    if (j >= nb) continue;
    felt pre = one();
    for (uint32_t m = 0; m < i; m++) pre = mul(pre, prod[t * per + m]);
    felt r = mul(ia, pre);
    ia = mul(ia, prod[j]);
    prod[j] = r;
  }
}

// Phase 3 for domain-only divisors: writes 1/den of every point into a table
// (cached per domain in the ctx, so constraint evaluation reads one felt per
// point instead of redoing the batch inversion every proof).
__global__ __launch_bounds__(TPB) void k_den_table(PointMap m, uint64_t count, felt c0, felt c1, int two,
                                                   const felt* __restrict__ binv, felt* __restrict__ out) {
  __shared__ felt s_pre[TPB], s_suf[TPB];
  felt den[EVAL_CH];
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    den[k] = one();
    if (q < count) {
      felt x = point_x(m, q);
      felt d = sub(x, c0);
      if (two) d = mul(d, sub(x, c1));
      den[k] = d;
    }
  });
  block_batch_inverse(den, s_pre, s_suf, binv[blockIdx.x]);
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    if (q < count) out[q] = den[k];
  });
}

// CE point of local index q (CE-coset-major over the shard's CE cosets):
// CE coset u = u0 + q/n, row t = q % n, CE index s = u + ce*t, LDE coset
// j = u * B/ce (local jl = j - j0); the frame rows are t and t+1 of that coset.
struct CePoint {
  uint64_t s, off, off_next;  // CE index; local LDE offsets of rows t, t+1
  uint32_t u;
};
__device__ __forceinline__ CePoint ce_point(const EvalCommon& c, uint64_t q) {
  const uint64_t n = 1ull << c.logn;
  CePoint p;
  p.u = c.u0 + (uint32_t)(q >> c.logn);
  const uint64_t t = q & (n - 1);
  p.s = p.u + (t << c.logce);
  const uint64_t jl = ((uint64_t)p.u << (c.logB - c.logce)) - c.j0;
  p.off = jl * n + t;
  p.off_next = jl * n + ((t + 1) & (n - 1));
  return p;
}

// ZKP_COUNT_REDO (tests/native/eval_check.cpp builds this file with it): count the waves
// that take the exact recomputation, so the test knows its inputs reached it
#ifdef ZKP_COUNT_REDO
__device__ unsigned long long zkp_redo_waves;
#define ZKP_REDO_TAKEN()                                                             \
  do {                                                                               \
    if ((threadIdx.x & 63) == 0) atomicAdd(&zkp_redo_waves, 1ull);                   \
  } while (0)
#else
#define ZKP_REDO_TAKEN() \
  do {                   \
  } while (0)
#endif

__global__ __launch_bounds__(TPB) void k_eval_mimc(EvalCommon c, MimcEvalArgs a, const felt* __restrict__ lde,
                                                   const felt* __restrict__ dinv, felt* __restrict__ comp) {
  const uint64_t M = (uint64_t)c.cel << c.logn;
  const uint64_t kmask = (64ull << c.logce) - 1;
  const felt bA = a.bcoef[0], bB = a.bcoef[1], bC = a.bcoef[2], bD = a.bcoef[3];
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    if (q >= M) return;
    const CePoint pt = ce_point(c, q);
    const felt cur = lde[pt.off];
    const felt nxt = lde[pt.off_next];
    const felt kv = a.kper[pt.s & kmask];
    const felt zi = c.zinv[pt.u], di = dinv[q];
    // the point with the deferred-check forms, again with the exact ones if a lane
    // of the wave needs it (kernels_common.hpp dmul / dadd)
    auto point = [&](auto fast_c, Rare& rq) {
      constexpr bool F = decltype(fast_c)::value;
      felt x = dmul<F>(c.pm.cx[q >> c.pm.logn], tw_full(c.pm.twn, q & ((1ull << c.pm.logn) - 1), c.pm.logn), rq);
      felt u = dadd<F>(cur, kv, rq);
      felt u2 = dmul<F>(u, u, rq), u3 = dmul<F>(u2, u, rq), u6 = dmul<F>(u3, u3, rq), u7 = dmul<F>(u6, u, rq);
      felt tr = sub(nxt, u7);  // coef_t is folded into c.zinv (per CE coset)
      felt tpart = dmul<F>(dmul<F>(tr, sub(x, c.w_last), rq), zi, rq);
      // b0 (cur - v0)(x - w_last) + b1 (cur - v1)(x - 1), regrouped (k_dt_eval_consts)
      felt bnum = add(sub(dmul<F>(cur, sub(dmul<F>(x, bA, rq), bB), rq), dmul<F>(x, bC, rq)), bD);
      return dadd<F>(tpart, dmul<F>(bnum, di, rq), rq);  // dinv = 1/((x - 1)(x - w^(n-1)))
    };
    Rare rq;
    felt v = point(std::true_type{}, rq);
    if (rq.any()) {
      v = point(std::false_type{}, rq);
      ZKP_REDO_TAKEN();
    }
    comp[q] = v;
  });
}

// Linear AIRs. TRANS: transition sum_c a_c*next_c + b_c*cur_c divided by Z_T
// (GlobalUpdate); without it the transition part is identically zero
// (TrainingUpdate). Boundary: group 0 = sum_c beta0_c*cur_c - bconst0
// over (x - w_b0); TWO adds group 1 = sum_c beta1_c*cur_c - bconst1 over (x - w_b1).
// LIN_CH points per thread, TPB apart (contiguous per wave); column-outer loop
// so the LIN_CH (and next-row) loads of a column are in flight together
constexpr int LIN_CH = 4;
#define LIN_POINT(k) ((uint64_t)blockIdx.x * (TPB * LIN_CH) + (uint64_t)(k) * TPB + threadIdx.x)

template <bool TRANS, bool TWO>
__global__ __launch_bounds__(TPB) void k_eval_linear(EvalCommon c, LinearEvalArgs a, const felt* __restrict__ lde,
                                                     const felt* __restrict__ dinv, felt* __restrict__ comp) {
  const uint64_t M = (uint64_t)c.cel << c.logn;
  const uint64_t cstride = 1ull << (c.logn + c.logBl);
  const uint32_t W = a.width;
  uint64_t off[LIN_CH], offn[LIN_CH];
  felt tr[LIN_CH], bs0[LIN_CH], bs1[LIN_CH];
  static_for<0, LIN_CH>([&](auto k) {
    const uint64_t q = LIN_POINT(k) < M ? LIN_POINT(k) : 0;
    const CePoint pt = ce_point(c, q);
    off[k] = pt.off;
    offn[k] = pt.off_next;
    tr[k] = zero();
    bs0[k] = zero();
    bs1[k] = zero();
  });
  for (uint32_t col = 0; col < W; col++) {
    const felt* base = lde + col * cstride;
    felt cur[LIN_CH];
    static_for<0, LIN_CH>([&](auto k) { cur[k] = base[off[k]]; });
    if (TRANS) {
      felt nxt[LIN_CH];
      static_for<0, LIN_CH>([&](auto k) { nxt[k] = base[offn[k]]; });
      const felt ca = a.coefs[col], cb = a.coefs[W + col];
      static_for<0, LIN_CH>([&](auto k) { tr[k] = add(tr[k], add(mul(ca, nxt[k]), mul(cb, cur[k]))); });
    }
    const felt b0 = a.coefs[2 * W + col];
    static_for<0, LIN_CH>([&](auto k) { bs0[k] = add(bs0[k], mul(b0, cur[k])); });
    if (TWO) {
      const felt b1 = a.coefs[3 * W + col];
      static_for<0, LIN_CH>([&](auto k) { bs1[k] = add(bs1[k], mul(b1, cur[k])); });
    }
  }
  const felt bconst = a.coefs[4 * W], bconst1 = a.coefs[4 * W + 1];
  static_for<0, LIN_CH>([&](auto k) {
    const uint64_t q = LIN_POINT(k);
    if (q >= M) return;
    const CePoint pt = ce_point(c, q);
    felt x = point_x(c.pm, q);
    felt tpart = TRANS ? mul(mul(tr[k], sub(x, c.w_last)), c.zinv[pt.u]) : zero();
    felt bnum;
    if (TWO) {
      felt e0 = sub(x, a.w_bstep), e1 = sub(x, a.w_bstep1);
      bnum = add(mul(sub(bs0[k], bconst), e1), mul(sub(bs1[k], bconst1), e0));
    } else {
      bnum = sub(bs0[k], bconst);
    }
    comp[q] = add(tpart, mul(bnum, dinv[q]));  // dinv: 1/((x - w^b0)(x - w^b1)) or 1/(x - w^b0)
  });
}

// Linear AIRs in coefficient form. Every term of their constraints is linear in
// the trace, so the sums k_eval_linear forms per CE point are polynomials:
//   A  = sum_c a_c T_c(w_n X) + b_c T_c(X)  (transition numerator; T_c(w_n X) has
//        coefficients w_n^d t_{c,d}),  B0 = sum_c beta0_c T_c,  B1 = sum_c beta1_c T_c.
// k_lin_lincomb forms their coefficients over the bit-reversed positions
// [p0, p0 + np) of the coefficient columns (one read of each column, 3 products
// per coefficient instead of 6 per CE point over ce cosets); the prover extends
// them to its CE cosets and k_eval_linear_pts applies k_eval_linear's final
// formula point by point: the same field values.
// out = [A (TRANS) | B0 | B1 (TWO)], np felts each; twn[j] = w_n^j (j < n/2).
// Column groups (blockIdx.y, cpg columns each) keep small position ranges (a
// rank's 1/R slice) from running a few waves per CU: with PART each group writes
// its partial sums [sa | sb | s0 | s1] (np each) to out + 4*np*group and
// k_lin_reduce adds the groups and applies the final formula.
__device__ __forceinline__ felt lin_finish_a(uint64_t p, uint32_t logn, const felt* twn, felt sa, felt sb) {
  const uint64_t n = 1ull << logn;
  const uint64_t d = __brevll(p) >> (64 - logn);  // the coefficient's degree
  const felt wd = d < (n >> 1) ? twn[d] : neg(twn[d - (n >> 1)]);
  return add(mul(wd, sa), sb);
}
template <bool TRANS, bool TWO, bool PART>
__global__ __launch_bounds__(TPB) void k_lin_lincomb(const felt* __restrict__ coef, uint32_t W, uint32_t logn,
                                                     uint64_t p0, uint64_t np, const felt* __restrict__ coefs,
                                                     const felt* __restrict__ twn, uint32_t cpg,
                                                     felt* __restrict__ out) {
  const uint64_t n = 1ull << logn;
  const uint32_t c0 = blockIdx.y * cpg, c1 = c0 + cpg < W ? c0 + cpg : W;
  felt sa[LIN_CH], sb[LIN_CH], s0[LIN_CH], s1[LIN_CH];
  uint64_t p[LIN_CH];
  static_for<0, LIN_CH>([&](auto k) {
    p[k] = p0 + (LIN_POINT(k) < np ? LIN_POINT(k) : 0);
    sa[k] = zero(); sb[k] = zero(); s0[k] = zero(); s1[k] = zero();
  });
  for (uint32_t c = c0; c < c1; c++) {
    const felt* col = coef + (uint64_t)c * n;
    felt v[LIN_CH];
    static_for<0, LIN_CH>([&](auto k) { v[k] = col[p[k]]; });
    if (TRANS) {
      const felt ca = coefs[c], cb = coefs[W + c];
      static_for<0, LIN_CH>([&](auto k) { sa[k] = add(sa[k], mul(ca, v[k])); sb[k] = add(sb[k], mul(cb, v[k])); });
    }
    const felt b0 = coefs[2 * W + c];
    static_for<0, LIN_CH>([&](auto k) { s0[k] = add(s0[k], mul(b0, v[k])); });
    if (TWO) {
      const felt b1 = coefs[3 * W + c];
      static_for<0, LIN_CH>([&](auto k) { s1[k] = add(s1[k], mul(b1, v[k])); });
    }
  }
  static_for<0, LIN_CH>([&](auto k) {
    const uint64_t i = LIN_POINT(k);
    if (i >= np) return;
    if (PART) {
      felt* o = out + (uint64_t)blockIdx.y * 4 * np + i;
      if (TRANS) { o[0] = sa[k]; o[np] = sb[k]; }
      o[2 * np] = s0[k];
      if (TWO) o[3 * np] = s1[k];
      return;
    }
    felt* o = out + i;
    if (TRANS) {
      *o = lin_finish_a(p[k], logn, twn, sa[k], sb[k]);
      o += np;
    }
    *o = s0[k];
    if (TWO) o[np] = s1[k];
  });
}
template <bool TRANS, bool TWO>
__global__ __launch_bounds__(TPB) void k_lin_reduce(const felt* __restrict__ part, uint32_t G, uint32_t logn,
                                                    uint64_t p0, uint64_t np, const felt* __restrict__ twn,
                                                    felt* __restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= np) return;
  felt sa = zero(), sb = zero(), s0 = zero(), s1 = zero();
  for (uint32_t g = 0; g < G; g++) {
    const felt* q = part + (uint64_t)g * 4 * np + i;
    if (TRANS) { sa = add(sa, q[0]); sb = add(sb, q[np]); }
    s0 = add(s0, q[2 * np]);
    if (TWO) s1 = add(s1, q[3 * np]);
  }
  felt* o = out + i;
  if (TRANS) {
    *o = lin_finish_a(p0 + i, logn, twn, sa, sb);
    o += np;
  }
  *o = s0;
  if (TWO) o[np] = s1;
}

// k_eval_linear's final formula over the extended arrays ev = [A | B0 | B1]
// (each cel*n, CE-coset-major like comp)
template <bool TRANS, bool TWO>
__global__ __launch_bounds__(TPB) void k_eval_linear_pts(EvalCommon c, LinearEvalArgs a, const felt* __restrict__ ev,
                                                         const felt* __restrict__ dinv, felt* __restrict__ comp) {
  const uint64_t M = (uint64_t)c.cel << c.logn;
  const felt* eb0 = TRANS ? ev + M : ev;
  const felt bconst = a.coefs[4 * a.width], bconst1 = a.coefs[4 * a.width + 1];
  static_for<0, LIN_CH>([&](auto k) {
    const uint64_t q = LIN_POINT(k);
    if (q >= M) return;
    const uint32_t u = c.u0 + (uint32_t)(q >> c.logn);
    felt x = point_x(c.pm, q);
    felt tpart = TRANS ? mul(mul(ev[q], sub(x, c.w_last)), c.zinv[u]) : zero();
    felt bnum;
    if (TWO) {
      felt e0 = sub(x, a.w_bstep), e1 = sub(x, a.w_bstep1);
      bnum = add(mul(sub(eb0[q], bconst), e1), mul(sub(eb0[M + q], bconst1), e0));
    } else {
      bnum = sub(eb0[q], bconst);
    }
    comp[q] = add(tpart, mul(bnum, dinv[q]));
  });
}

// bit-reversed polynomial evaluation: tree with level multipliers x^(2^l)
constexpr uint32_t OOD_LOGE = 11;
// Arrays a >= ntwo (the composition columns, whose OOD frame is at z only) skip
// the second point (their partials at it are left zero).
// A rank of a sharded proof evaluates the blocks [b0, b0 + gridDim.x) only;
// partial[(a * gridDim.x + b - b0) * 2 + {0,1}] (the all-gathered rank blocks
// are what k_eval_bitrev_tail reads).
// The array's block of E = 2^logE bit-reversed coefficients is a multilinear form in the
// level multipliers: sum_p c[p] prod_b m_b^(bit b of p), m_b = x^(2^(logn-1-b)) for local
// bit b (pw0 / pw1 tables), so its bits may be contracted in any order (exact field
// arithmetic: the value is the same). With E = 2048 each thread loads elements t + 256 i
// (i < 8: every load of a wave is 64 consecutive felts) and contracts local bits 8..10 in
// registers; the thread bits 7..0 then pair s[t] with s[t + h] (h = 128 .. 1), so every
// LDS access of the tree is to consecutive slots (the pairing p, p + d of the round-5 tree
// conflicted 6.5 cycles per LDS instruction at C3).
__global__ __launch_bounds__(TPB) void k_eval_bitrev(const felt* __restrict__ arrays, uint32_t logn, uint32_t logE,
                                                     const felt* __restrict__ pw0, const felt* __restrict__ pw1,
                                                     uint32_t ntwo, uint32_t b0, felt* __restrict__ partial) {
  __shared__ felt s0[TPB];
  __shared__ felt s1[TPB];
  const uint32_t E = 1u << logE;
  const bool two = blockIdx.y < ntwo;  // block-uniform
  const felt* src = arrays + ((uint64_t)blockIdx.y << logn) + ((uint64_t)(b0 + blockIdx.x) << logE);
  const uint32_t t = threadIdx.x;
  uint32_t m, tb0;  // threads holding data, local bit of thread bit 0
  if (E == 8 * TPB) {
    felt v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = src[t + TPB * i];
    felt a[4], b[4];
    {  // local bit 8 (i bit 0)
      const felt m0 = pw0[logn - 9], m1 = pw1[logn - 9];
#pragma unroll
      for (int i = 0; i < 4; i++) a[i] = add(v[2 * i], mul(m0, v[2 * i + 1]));
      if (two)
#pragma unroll
        for (int i = 0; i < 4; i++) b[i] = add(v[2 * i], mul(m1, v[2 * i + 1]));
    }
    {  // local bit 9
      const felt m0 = pw0[logn - 10], m1 = pw1[logn - 10];
      a[0] = add(a[0], mul(m0, a[1])); a[2] = add(a[2], mul(m0, a[3]));
      if (two) { b[0] = add(b[0], mul(m1, b[1])); b[2] = add(b[2], mul(m1, b[3])); }
    }
    {  // local bit 10
      const felt m0 = pw0[logn - 11], m1 = pw1[logn - 11];
      s0[t] = add(a[0], mul(m0, a[2]));
      s1[t] = two ? add(b[0], mul(m1, b[2])) : zero();
    }
    m = TPB;
    tb0 = 0;
  } else {  // smaller blocks: per = E / TPB consecutive elements per thread (or one)
    // (E < 2048: per <= 4; compile-time register indices, guarded by the runtime per)
    const uint32_t per = E >= TPB ? E / TPB : 1;
    uint32_t l = 0;
    felt v0[4], v1[4];
    static_for<0, 4>([&](auto ii) {
      constexpr uint32_t i = decltype(ii)::value;
      const felt x = (i < per && t * per + i < E) ? src[t * per + i] : zero();
      v0[i] = x;
      v1[i] = x;
    });
    static_for<0, 2>([&](auto lv) {
      constexpr uint32_t w = 4u >> decltype(lv)::value;  // 4, then 2 values reduced per level
      if (w <= per) {
        const felt m0 = pw0[logn - 1 - l], m1 = pw1[logn - 1 - l];
        static_for<0, (int)(w / 2)>([&](auto ii) {
          constexpr uint32_t i = decltype(ii)::value;
          v0[i] = add(v0[2 * i], mul(m0, v0[2 * i + 1]));
          v1[i] = add(v1[2 * i], mul(m1, v1[2 * i + 1]));
        });
        l++;
      }
    });
    s0[t] = v0[0];
    s1[t] = v1[0];
    m = E >= TPB ? TPB : E;
    tb0 = l;
  }
  __syncthreads();
  // thread bits from the top: s[t] += m_b * s[t + h] for t < h, b = tb0 + log2 h
  for (uint32_t h = m >> 1; h >= 1; h >>= 1) {
    const uint32_t lb = 31 - __builtin_clz(h);
    if (t < h) {
      const felt m0 = pw0[logn - 1 - tb0 - lb];
      s0[t] = add(s0[t], mul(m0, s0[t + h]));
      if (two) {
        const felt m1 = pw1[logn - 1 - tb0 - lb];
        s1[t] = add(s1[t], mul(m1, s1[t + h]));
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    uint64_t o = ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * 2;
    partial[o] = s0[0];
    partial[o + 1] = two ? s1[0] : zero();
  }
}

// second level of the OOD tree: the nb block partials of each (array, point)
// (bit-reversed order continues: level logE + l uses pw[logn - 1 - logE - l]);
// one block per array; nb <= 2 * 2048 (pairs are combined while loading).
// The partials come in rank blocks of nbl = 2^lognbl blocks each (world 1: one
// rank block): block b of array a at ((b / nbl * narrays + a) * nbl + b % nbl) * 2.
__global__ __launch_bounds__(TPB) void k_eval_bitrev_tail(const felt* __restrict__ partial, uint32_t nb,
                                                          uint32_t lognbl, uint32_t narrays, uint32_t logn,
                                                          uint32_t logE, const felt* __restrict__ pw0,
                                                          const felt* __restrict__ pw1, felt ninv,
                                                          felt* __restrict__ out) {
  __shared__ felt s0[1u << OOD_LOGE];
  __shared__ felt s1[1u << OOD_LOGE];
  const uint32_t a = blockIdx.x, nblm = (1u << lognbl) - 1;
  auto P = [&](uint32_t b, uint32_t k) {
    return partial[((((uint64_t)(b >> lognbl) * narrays + a) << lognbl) + (b & nblm)) * 2 + k];
  };
  uint32_t l = logE, m = nb;
  if (nb > (1u << OOD_LOGE)) {  // fold one level while loading
    const felt a0 = pw0[logn - 1 - l], a1 = pw1[logn - 1 - l];
    for (uint32_t i = threadIdx.x; i < nb / 2; i += TPB) {
      s0[i] = add(P(2 * i, 0), mul(a0, P(2 * i + 1, 0)));
      s1[i] = add(P(2 * i, 1), mul(a1, P(2 * i + 1, 1)));
    }
    l++;
    m = nb / 2;
  } else {
    for (uint32_t i = threadIdx.x; i < nb; i += TPB) {
      s0[i] = P(i, 0);
      s1[i] = P(i, 1);
    }
  }
  __syncthreads();
  for (uint32_t d = 1; d < m; d <<= 1, l++) {
    const felt a0 = pw0[logn - 1 - l], a1 = pw1[logn - 1 - l];
    for (uint32_t i = threadIdx.x; i < m / (2 * d); i += TPB) {
      uint32_t p = i * 2 * d;
      s0[p] = add(s0[p], mul(a0, s0[p + d]));
      s1[p] = add(s1[p], mul(a1, s1[p + d]));
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = mul(s0[0], ninv);
    out[2 * blockIdx.x + 1] = mul(s1[0], ninv);
  }
}

// local point q = jl*n + t of the shard's cosets: LDE index i = (j0 + jl) + B*t;
// the LDE matrices are read at offset q (contiguous), output is coset-major.
__global__ __launch_bounds__(TPB) void k_deep(DeepArgs a, const felt* __restrict__ binv, felt* __restrict__ out) {
  __shared__ felt s_pre[TPB], s_suf[TPB];
  const felt z = a.dk[0], zg = a.dk[1], kz = a.dk[2], kzg = a.dk[3];
  const uint64_t N = 1ull << (a.logn + a.logBl);
  const uint64_t cstride = N;
  felt A[EVAL_CH], Bh[EVAL_CH];
  uint64_t off[EVAL_CH];
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q0 = EVAL_POINT(k);
    off[k] = q0 < N ? q0 : 0;
    A[k] = zero();
    Bh[k] = zero();
  });
  // column-outer: the EVAL_CH loads of a column are independent and in flight
  // together (wide AIRs read w + C columns per point; C3/C5 have 121)
  for (uint32_t c = 0; c < a.w; c++) {
    const felt gc = a.gamma[c];
    const felt* col = a.tlde + c * cstride;
    felt v[EVAL_CH];
    static_for<0, EVAL_CH>([&](auto k) { v[k] = col[off[k]]; });
    static_for<0, EVAL_CH>([&](auto k) { A[k] = add(A[k], mul(gc, v[k])); });
  }
  for (uint32_t h = 0; h < a.C; h++) {
    const felt gh = a.gamma[a.w + h];
    const felt* col = a.clde + h * cstride;
    felt v[EVAL_CH];
    static_for<0, EVAL_CH>([&](auto k) { v[k] = col[off[k]]; });
    static_for<0, EVAL_CH>([&](auto k) { Bh[k] = add(Bh[k], mul(gh, v[k])); });
  }
  felt num[EVAL_CH], den[EVAL_CH];
  static_for<0, EVAL_CH>([&](auto k) {
    const bool valid = EVAL_POINT(k) < N;
    felt x = point_x(a.pm, off[k]);
    felt e1 = sub(x, z), e2 = sub(x, zg);
    num[k] = add(mul(sub(add(A[k], Bh[k]), kz), e2), mul(sub(A[k], kzg), e1));
    den[k] = valid ? mul(e1, e2) : one();
  });
  block_batch_inverse(den, s_pre, s_suf, binv[blockIdx.x]);
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    if (q < N) out[q] = mul(num[k], den[k]);
  });
}

// Coefficient-form DEEP, step 1 (wide traces): the gamma-combination of the w
// trace polynomials in coefficient form, out[p] = sum_c gamma_c * coef_c[p]
// (bit-reversed, n-scaled like its inputs). LIN_CH positions per thread, TPB
// apart; column-outer so each column's loads are in flight together. Its coset
// LDE then replaces w column reads per LDE point of the pointwise k_deep by one.
// A rank of a sharded proof combines the positions [p0, p0 + np) (out[0, np)).
template <bool PART>
__global__ __launch_bounds__(TPB) void k_deep_lincomb(const felt* __restrict__ coef, uint32_t w, uint64_t n,
                                                      uint64_t p0, uint64_t np, const felt* __restrict__ gamma,
                                                      uint32_t cpg, felt* __restrict__ out) {
  const uint32_t c0 = blockIdx.y * cpg, c1 = c0 + cpg < w ? c0 + cpg : w;
  felt acc[LIN_CH];
  uint64_t p[LIN_CH];
  static_for<0, LIN_CH>([&](auto k) {
    p[k] = p0 + (LIN_POINT(k) < np ? LIN_POINT(k) : 0);
    acc[k] = zero();
  });
  for (uint32_t c = c0; c < c1; c++) {
    const felt g = gamma[c];
    const felt* col = coef + (uint64_t)c * n;
    felt v[LIN_CH];
    static_for<0, LIN_CH>([&](auto k) { v[k] = col[p[k]]; });
    static_for<0, LIN_CH>([&](auto k) { acc[k] = add(acc[k], mul(g, v[k])); });
  }
  felt* o = out + (PART ? (uint64_t)blockIdx.y * np : 0);
  static_for<0, LIN_CH>([&](auto k) {
    if (LIN_POINT(k) < np) o[LIN_POINT(k)] = acc[k];
  });
}
// out[i] = sum_g part[g*np + i]
__global__ __launch_bounds__(TPB) void k_sum_groups(const felt* __restrict__ part, uint32_t G, uint64_t np,
                                                    felt* __restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= np) return;
  felt a = part[i];
  for (uint32_t g = 1; g < G; g++) a = add(a, part[(uint64_t)g * np + i]);
  out[i] = a;
}

// multi-segment gather: segment s copies seg[s].count items of seg[s].words
// 32-bit words from src (item index idx[seg.idx_off + i]) to out + seg.out_off
__global__ void k_gather_multi(const GatherSeg* __restrict__ segs, const uint64_t* __restrict__ idx,
                               uint32_t* __restrict__ out) {
  const GatherSeg sg = segs[blockIdx.y];
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i >= sg.count) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(sg.src) + idx[sg.idx_off + i] * sg.words;
  uint32_t* dst = out + sg.out_off + i * sg.words;
  for (uint32_t w = 0; w < sg.words; w += 4)
    *reinterpret_cast<uint4*>(dst + w) = *reinterpret_cast<const uint4*>(src + w);
}

__global__ void k_gather_felts(const felt* __restrict__ src, const uint64_t* __restrict__ idx, felt* __restrict__ out,
                               uint64_t count) {
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i < count) out[i] = src[idx[i]];
}

__global__ void k_gather_digests(const uint32_t* __restrict__ nodes, const uint64_t* __restrict__ idx,
                                 uint32_t* __restrict__ out, uint64_t count) {
  uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (i < count) {
    uint32_t d[8];
    load_digest(nodes + idx[i] * 8, d);
    store_digest(out + i * 8, d);
  }
}

// ------------------------------------------------- aggregation trace builder
// GlobalUpdateProver::build_trace on the device (src/aggregation/prover.rs:98-160):
// S column c (c < 60) at row r = masked_c + kinv * sum_{i < min(r, ndev)} (local_i,c - raw_c),
// U column c at row r = local_{r-1},c - raw_c for 1 <= r <= ndev, else 0; rows past
// ndev + 1 repeat row ndev + 1 (the prefix stops growing there, so padding is free).
// Rows are scanned in tiles of GU_TILE: per-tile sums, a per-column scan of the
// tile sums, then the tile-local scans with their carry-in.
constexpr uint32_t GU_D_DEV = 60, GU_RPT = 16, GU_TILE = TPB * GU_RPT;

__device__ __forceinline__ felt gu_step(const felt* __restrict__ masked, const felt* __restrict__ raw,
                                        const felt* __restrict__ local, uint64_t ndev, felt kinv, uint32_t c,
                                        uint64_t r) {
  if (r == 0) return masked[c];
  if (r > ndev) return zero();
  return mul(sub(local[(r - 1) * GU_D_DEV + c], raw[c]), kinv);
}

__global__ __launch_bounds__(TPB) void k_gu_tile_sums(const felt* __restrict__ masked, const felt* __restrict__ raw,
                                                      const felt* __restrict__ local, uint64_t ndev, felt kinv,
                                                      uint64_t n, felt* __restrict__ tile_sum) {
  __shared__ felt s[TPB];
  const uint32_t c = blockIdx.y;
  const uint64_t r0 = (uint64_t)blockIdx.x * GU_TILE + (uint64_t)threadIdx.x * GU_RPT;
  felt acc = zero();
  for (uint32_t i = 0; i < GU_RPT; i++)
    if (r0 + i < n && r0 + i <= ndev) acc = add(acc, gu_step(masked, raw, local, ndev, kinv, c, r0 + i));
  s[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t h = TPB / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) s[threadIdx.x] = add(s[threadIdx.x], s[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sum[(uint64_t)c * gridDim.x + blockIdx.x] = s[0];
}

// exclusive scan of the tile sums of column blockIdx.x (serial: tiles are few)
__global__ void k_gu_tile_scan(felt* tile_sum, uint32_t tiles) {
  if (threadIdx.x != 0) return;
  felt* t = tile_sum + (uint64_t)blockIdx.x * tiles;
  felt acc = zero();
  for (uint32_t i = 0; i < tiles; i++) {
    felt v = t[i];
    t[i] = acc;
    acc = add(acc, v);
  }
}

__global__ __launch_bounds__(TPB) void k_gu_tile_write(const felt* __restrict__ masked, const felt* __restrict__ raw,
                                                       const felt* __restrict__ local, uint64_t ndev, felt kinv,
                                                       uint64_t n, const felt* __restrict__ tile_carry,
                                                       felt* __restrict__ out) {
  __shared__ felt s[TPB];
  const uint32_t c = blockIdx.y;
  const uint64_t base = (uint64_t)blockIdx.x * GU_TILE;
  felt* col = out + (uint64_t)c * n;
  if (c >= GU_D_DEV) {  // U columns: the scaled-out update of row r (coalesced across the block)
    const uint32_t j = c - GU_D_DEV;
    for (uint32_t i = 0; i < GU_RPT; i++) {
      const uint64_t r = base + (uint64_t)i * TPB + threadIdx.x;
      if (r >= n) break;
      col[r] = (r >= 1 && r <= ndev) ? sub(local[(r - 1) * GU_D_DEV + j], raw[j]) : zero();
    }
    return;
  }
  // S columns: GU_RPT row blocks of TPB consecutive rows (coalesced), each a
  // block-wide inclusive scan (LDS) on top of the running carry
  felt carry = tile_carry[(uint64_t)c * gridDim.x + blockIdx.x];
  for (uint32_t i = 0; i < GU_RPT; i++) {
    const uint64_t r = base + (uint64_t)i * TPB + threadIdx.x;
    felt v = (r < n && r <= ndev) ? gu_step(masked, raw, local, ndev, kinv, c, r) : zero();
    __syncthreads();
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < TPB; d <<= 1) {
      felt a = threadIdx.x >= d ? s[threadIdx.x - d] : zero();
      __syncthreads();
      if (threadIdx.x >= d) s[threadIdx.x] = add(s[threadIdx.x], a);
      __syncthreads();
    }
    if (r < n) col[r] = add(carry, s[threadIdx.x]);
    carry = add(carry, s[TPB - 1]);
  }
}

// ---- GlobalUpdate column pairing. The transition constraints
// k*next[i] - k*cur[i] - next[i+d] = 0 (src/aggregation/air.rs:101-119) fix
// column d+i on rows 1..n-1 from column i, so as polynomials of degree < n
//   T_{d+i}(X) = k*(T_i(X) - T_i(w_n^-1 X)) + c_i * L_0(X),
//   c_i = T_{d+i}[0] - k*(T_i[0] - T_i[n-1]),  L_0(X) = (X^n - 1) / (n (X - 1)).
// A trace that satisfies them (checked here, every row) gets the columns d..2d-1
// of its coefficients and LDE from columns 0..d-1 at a few products per value
// instead of an interpolation and B coset NTTs per column; the values are the
// same field elements, so the proof bytes are too.

// check rows [t0, t0 + 2^logtn) (row 0 excepted) of the column pairs (c0+ci, d+c0+ci),
// ci < cw, of the natural trace T (column-major); set *bad on any mismatch; c_i
// when the rows include row 0 (cval non-null)
__global__ __launch_bounds__(TPB) void k_gu_check(const felt* __restrict__ T, uint32_t d, uint32_t logn, felt k,
                                                  uint32_t c0, uint32_t cw, uint64_t t0, uint32_t logtn,
                                                  felt* __restrict__ cval, uint32_t* __restrict__ bad) {
  const uint64_t n = 1ull << logn, q = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (q >= (uint64_t)cw << logtn) return;
  const uint32_t i = c0 + (uint32_t)(q >> logtn);
  const uint64_t t = t0 + (q & ((1ull << logtn) - 1));
  const felt* a = T + (uint64_t)i * n;
  const felt* b = T + (uint64_t)(d + i) * n;
  const felt prev = a[t == 0 ? n - 1 : t - 1];
  const felt kd = mul(k, sub(a[t], prev));
  if (t == 0) {
    if (cval) cval[i] = sub(b[0], kd);
  } else if (!eq(b[t], kd)) {
    *bad = 1u;
  }
}

// The MiMC trace against its AIR before the proof's shortcuts are chosen: every row's
// transition x[t+1] = (x[t] + K[t mod 64])^7 (K = get_round_constants(), helper.rs:404-406)
// and the two assertions x[0] = v0, x[n-1] = v1. A trace that satisfies them has a
// composition polynomial of degree < 6n, so the derived last composition column
// (LastCol) is exact; any failure sets *bad (one store per failing wave).
__global__ __launch_bounds__(TPB) void k_mimc_check(const felt* __restrict__ T, uint64_t n, felt v0, felt v1,
                                                    uint32_t* __restrict__ bad) {
  const uint64_t t = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  bool ok = true;
  if (t < n) {
    const felt x = T[t];
    if (t + 1 < n) {
      const felt u = add(x, make((t % 64 + 1) * 1000000ull, 0));
      const felt u3 = mul(mul(u, u), u), u7 = mul(mul(u3, u3), u);
      ok = eq(T[t + 1], u7);
    }
    if (t == 0) ok = ok && eq(x, v0);
    if (t == n - 1) ok = ok && eq(x, v1);
  }
  const uint64_t failing = __builtin_amdgcn_ballot_w64(!ok);
  if (failing && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(failing)) *bad = 1u;
}

// coefficient columns (bit-reversed, scaled by n) at the positions [p0, p0 + np):
// coef_{d+i}[p] = k*(1 - w_n^-rev(p))*coef_i[p] + c_i
__global__ __launch_bounds__(TPB) void k_gu_coef(felt* __restrict__ coef, uint32_t d, uint32_t logn, felt k,
                                                 const felt* __restrict__ itwn, uint32_t c0, uint32_t cw,
                                                 uint64_t p0, uint64_t np, const felt* __restrict__ cval) {
  const uint64_t n = 1ull << logn, p = p0 + blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (p >= p0 + np) return;
  const felt kw = mul(k, sub(one(), tw_full(itwn, rev_bits((uint32_t)p, logn), logn)));
  for (uint32_t i = c0; i < c0 + cw; i++)
    coef[(uint64_t)(d + i) * n + p] = add(mul(kw, coef[(uint64_t)i * n + p]), cval[i]);
}

// LDE columns over the cosets [0, Bl) (coset-major: column c at c*Bl*n, coset jl, row t):
// lde_{d+i}(x) = k*(lde_i(x) - lde_i(w_n^-1 x)) + c_i*L_0(x), w_n^-1 x = the previous row of the coset
// SMALLK: k < 2^32 (the reference's k = devices * 10^6), multiplied with mul_u32
template <bool SMALLK>
__global__ __launch_bounds__(TPB) void k_gu_lde(felt* __restrict__ lde, uint32_t d, uint32_t logn, uint32_t logBl,
                                                felt k, uint32_t c0, uint32_t cw, const felt* __restrict__ cval,
                                                const felt* __restrict__ l0) {
  const uint64_t n = 1ull << logn, q = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (q >= (n << logBl)) return;
  const uint64_t t = q & (n - 1), qp = t == 0 ? q + n - 1 : q - 1;
  const uint64_t cs = n << logBl;
  const felt l = l0[q];
  for (uint32_t i = c0; i < c0 + cw; i++) {
    const felt* src = lde + (uint64_t)i * cs;
    const felt df = sub(src[q], src[qp]);
    const felt kd = SMALLK ? mul_u32(df, (uint32_t)k.lo) : mul(k, df);
    lde[(uint64_t)(d + i) * cs + q] = add(kd, mul(cval[i], l));
  }
}

// the lazy paired columns [wi, w) of the queried rows held here (GuLazy): thread per
// (position, column)
__global__ __launch_bounds__(TPB) void k_gu_fill(felt* __restrict__ lde, uint32_t w, uint32_t logn, uint32_t logB,
                                                 uint32_t j0, uint32_t logBl, const uint64_t* __restrict__ pos,
                                                 uint32_t npos, GuLazy gl) {
  const uint32_t nc = w - gl.wi;
  const uint64_t q = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  if (q >= (uint64_t)npos * nc) return;
  const uint64_t i = pos[q / nc];
  const uint32_t c = gl.wi + (uint32_t)(q % nc);
  const uint64_t n = 1ull << logn, j = i & ((1ull << logB) - 1), t = i >> logB;
  if (j < j0 || j >= j0 + (1ull << logBl)) return;
  const uint64_t jl = j - j0, cstride = n << logBl;
  const felt* base = lde + jl * n + t;
  const felt* prev = lde + jl * n + (t == 0 ? n - 1 : t - 1);
  const uint32_t ic = c - gl.d;
  const felt v = add(mul(gl.k, sub(base[ic * cstride], prev[ic * cstride])), mul(gl.cval[ic], gl.l0[jl * n + t]));
  lde[c * cstride + jl * n + t] = v;
}

// L_0(x) = (x^n - 1) / (n (x - 1)) over the points of a coset-major shard (domain-only table).
// x^n is constant on a coset ((c w_n^t)^n = c^n): k_l0_consts forms K_j = (c_j^n - 1) / n once
// per coset, and k_l0_table scales the batch inverses of (x - 1) (k_den_products +
// k_invert_products, as k_den_table) by it. (It used to do a Fermat inversion and a
// pow per point: 1.24 ms for a cold C3 shape.)
__global__ __launch_bounds__(64) void k_l0_consts(PointMap pm, uint32_t ncos, felt ninv, felt* __restrict__ K) {
  for (uint32_t j = threadIdx.x; j < ncos; j += 64) {
    felt cn = pm.cx[j];
    for (uint32_t l = 0; l < pm.logn; l++) cn = sqr(cn);
    K[j] = mul(sub(cn, one()), ninv);
  }
}

__global__ __launch_bounds__(TPB) void k_l0_table(PointMap pm, uint64_t count, const felt* __restrict__ K,
                                                  const felt* __restrict__ binv, felt* __restrict__ out) {
  __shared__ felt s_pre[TPB], s_suf[TPB];
  felt den[EVAL_CH];
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    den[k] = q < count ? sub(point_x(pm, q), one()) : one();
  });
  block_batch_inverse(den, s_pre, s_suf, binv[blockIdx.x]);
  static_for<0, EVAL_CH>([&](auto k) {
    const uint64_t q = EVAL_POINT(k);
    if (q < count) out[q] = mul(den[k], K[q >> pm.logn]);
  });
}

}  // namespace

// ======================================================================= host
hipEvent_t Prof::get_event() {
  if (!pool.empty()) {
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}
void Prof::begin(const char* name, hipStream_t s, double bytes) {
  open = enabled && (only.empty() || only == name);
  if (!open) return;
  ProfRec r;
  r.name = name;
  r.bytes = bytes;
  r.start = get_event();
  r.stop = get_event();
  (void)hipEventRecord(r.start, s);
  pending.push_back(r);
}
void Prof::end(hipStream_t s) {
  if (!open) return;
  (void)hipEventRecord(pending.back().stop, s);
  open = false;
}



__global__ void k_noop() {}

void preload_kernels_module() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, (const void*)k_expand_powers);
}

void warm_stream(hipStream_t s) { hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s); }

void launch_build_levels(Prof& prof, hipStream_t s, felt* tab, uint32_t top) {
  LAUNCH(prof, "build_levels", s, (double)(1ull << top) * 32.0,
         hipLaunchKernelGGL(k_build_levels, dim3(grid_stride_blocks(1ull << top)), dim3(TPB), 0, s, tab, top));
}

void launch_expand_powers(Prof& prof, hipStream_t s, felt* out, uint64_t count, const felt* lo_tab,
                          const felt* hi_tab) {
  LAUNCH(prof, "expand_powers", s, count * 16.0,
         hipLaunchKernelGGL(k_expand_powers, dim3(grid_stride_blocks(count)), dim3(TPB), 0, s, out, count, lo_tab,
                            hi_tab));
}

void launch_build_coset_scale(Prof& prof, hipStream_t s, felt* S, uint32_t logn, uint32_t B, const felt* tw,
                              uint32_t logN, const felt* glo, const felt* ghi, felt ninv) {
  LAUNCH(prof, "build_coset_scale", s, (double)((uint64_t)B << logn) * 16.0,
         hipLaunchKernelGGL(k_build_coset_scale, dim3(grid_stride_blocks((uint64_t)B << logn)), dim3(TPB), 0, s, S,
                            logn, B, tw, logN, glo, ghi, ninv));
}


// prod: nb block products (+1 slot for the closed-form total inverse when pw is given)
static void launch_den_inverse(Prof& prof, hipStream_t s, const PointMap& m, uint64_t count, felt c0, felt c1,
                               int two, felt* prod, const felt* cdev = nullptr, const felt* pw = nullptr) {
  uint32_t nb = blocks_for((count + EVAL_CH - 1) / EVAL_CH);
  felt* tinv = pw ? prod + nb : nullptr;
  LAUNCH(prof, "den_products", s, (double)count * 16.0,
         hipLaunchKernelGGL(k_den_products, dim3(nb), dim3(TPB), 0, s, m, count, c0, c1, two, cdev, pw, tinv, prod));
  LAUNCH(prof, "invert_products", s, (double)nb * 32.0,
         hipLaunchKernelGGL(k_invert_products, dim3(1), dim3(1024), 0, s, prod, nb, tinv));
}

static void launch_den_table(Prof& prof, hipStream_t s, const PointMap& m, uint64_t count, felt c0, felt c1,
                             int two, felt* prod, felt* table) {
  launch_den_inverse(prof, s, m, count, c0, c1, two, prod);
  LAUNCH(prof, "den_table", s, (double)count * 16.0,
         hipLaunchKernelGGL(k_den_table, dim3(blocks_for((count + EVAL_CH - 1) / EVAL_CH)), dim3(TPB), 0, s, m, count,
                            c0, c1, two, prod, table));
}

#ifdef ZKP_COUNT_REDO
// host: the exact-pass waves of k_eval_mimc since the last call (and reset)
unsigned long long zkp_redo_waves_take() {
  unsigned long long v = 0, z = 0;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(zkp_redo_waves), sizeof v);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(zkp_redo_waves), &z, sizeof z);
  return v;
}
#endif

void launch_eval_mimc(Prof& prof, hipStream_t s, const EvalCommon& c, const MimcEvalArgs& a, const felt* lde,
                      felt* comp) {
  uint64_t M = (uint64_t)c.cel << c.logn;
  if (!a.binv_ready) launch_den_table(prof, s, c.pm, M, one(), c.w_last, 1, a.binv, a.dinv);
  LAUNCH(prof, "eval_mimc", s, (double)M * 48.0,
         hipLaunchKernelGGL(k_eval_mimc, dim3(blocks_for((M + EVAL_CH - 1) / EVAL_CH)), dim3(TPB), 0, s, c, a, lde,
                            a.dinv, comp));
}

void launch_eval_linear(Prof& prof, hipStream_t s, const EvalCommon& c, const LinearEvalArgs& a, const felt* lde,
                        felt* comp) {
  uint64_t M = (uint64_t)c.cel << c.logn;
  const bool two = a.two_groups;
  if (!a.binv_ready) launch_den_table(prof, s, c.pm, M, a.w_bstep, a.w_bstep1, two ? 1 : 0, a.binv, a.dinv);
  dim3 g(blocks_for((M + LIN_CH - 1) / LIN_CH));
  const double bytes = (double)M * (a.width * (a.transition ? 32.0 : 16.0) + 32.0);
  if (a.transition && !two)
    LAUNCH(prof, "eval_linear", s, bytes,
           hipLaunchKernelGGL((k_eval_linear<true, false>), g, dim3(TPB), 0, s, c, a, lde, a.dinv, comp));
  else if (!a.transition && two)
    LAUNCH(prof, "eval_linear", s, bytes,
           hipLaunchKernelGGL((k_eval_linear<false, true>), g, dim3(TPB), 0, s, c, a, lde, a.dinv, comp));
  else
    LAUNCH(prof, "eval_linear", s, bytes,
           hipLaunchKernelGGL((k_eval_linear<true, true>), g, dim3(TPB), 0, s, c, a, lde, a.dinv, comp));
}

uint32_t lincomb_groups(uint64_t np, uint32_t W) {
  const uint64_t waves = ((np + LIN_CH - 1) / LIN_CH + 63) / 64;
  uint64_t G = (4096 + waves - 1) / waves;  // aim at >= 4 waves per SIMD
  const uint64_t gmax = W >= 8 ? W / 4 : 1;  // >= 4 columns per group
  if (G > gmax) G = gmax;
  if (G > 16) G = 16;
  return G ? (uint32_t)G : 1u;
}

void launch_lin_lincomb(Prof& prof, hipStream_t s, bool trans, bool two, const felt* coef, uint32_t W, uint32_t logn,
                        uint64_t p0, uint64_t np, const felt* coefs, const felt* twn, felt* out, felt* scratch) {
  const uint32_t G = scratch ? lincomb_groups(np, W) : 1u, cpg = (W + G - 1) / G;
  const dim3 g(blocks_for((np + LIN_CH - 1) / LIN_CH), G);
  const double bytes = (double)np * 16.0 * (W + (trans ? 1 : 0) + 1 + (two ? 1 : 0));
#define ZKP_LINC(T, O)                                                                                          \
  if (G == 1)                                                                                                   \
    LAUNCH(prof, "lin_lincomb", s, bytes,                                                                       \
           hipLaunchKernelGGL((k_lin_lincomb<T, O, false>), g, dim3(TPB), 0, s, coef, W, logn, p0, np, coefs, twn, \
                              cpg, out));                                                                       \
  else {                                                                                                        \
    LAUNCH(prof, "lin_lincomb", s, bytes,                                                                       \
           hipLaunchKernelGGL((k_lin_lincomb<T, O, true>), g, dim3(TPB), 0, s, coef, W, logn, p0, np, coefs, twn,  \
                              cpg, scratch));                                                                   \
    LAUNCH(prof, "lin_lincomb", s, (double)np * 16.0 * 4 * G,                                                  \
           hipLaunchKernelGGL((k_lin_reduce<T, O>), dim3(blocks_for(np)), dim3(TPB), 0, s, scratch, G, logn, p0,  \
                              np, twn, out));                                                                   \
  }
  if (trans && two) { ZKP_LINC(true, true) }
  else if (trans) { ZKP_LINC(true, false) }
  else if (two) { ZKP_LINC(false, true) }
  else { ZKP_LINC(false, false) }
#undef ZKP_LINC
}

void launch_eval_linear_pts(Prof& prof, hipStream_t s, const EvalCommon& c, const LinearEvalArgs& a, const felt* ev,
                            felt* comp) {
  uint64_t M = (uint64_t)c.cel << c.logn;
  const bool two = a.two_groups, trans = a.transition;
  if (!a.binv_ready) launch_den_table(prof, s, c.pm, M, a.w_bstep, a.w_bstep1, two ? 1 : 0, a.binv, a.dinv);
  const dim3 g(blocks_for((M + LIN_CH - 1) / LIN_CH));
  const double bytes = (double)M * 16.0 * ((trans ? 1 : 0) + 1 + (two ? 1 : 0) + 2);
#define ZKP_LINP(T, O)                                                                                      \
  LAUNCH(prof, "eval_linear", s, bytes,                                                                     \
         hipLaunchKernelGGL((k_eval_linear_pts<T, O>), g, dim3(TPB), 0, s, c, a, ev, a.dinv, comp))
  if (trans && two) ZKP_LINP(true, true);
  else if (trans) ZKP_LINP(true, false);
  else if (two) ZKP_LINP(false, true);
  else ZKP_LINP(false, false);
#undef ZKP_LINP
}

void launch_eval_bitrev_blocks(Prof& prof, hipStream_t s, const felt* arrays, uint32_t narrays, uint32_t ntwo,
                               uint32_t logn, const felt* pw0, const felt* pw1, uint32_t b0, uint32_t nbl,
                               felt* partial) {
  const uint32_t logE = logn < OOD_LOGE ? logn : OOD_LOGE;
  LAUNCH(prof, "eval_bitrev", s, (double)narrays * nbl * (1ull << logE) * 16.0,
         hipLaunchKernelGGL(k_eval_bitrev, dim3(nbl, narrays), dim3(TPB), 0, s, arrays, logn, logE, pw0, pw1,
                            ntwo, b0, partial));
}

void launch_eval_bitrev_tail(Prof& prof, hipStream_t s, const felt* partial, uint32_t narrays, uint32_t logn,
                             uint32_t nbl, const felt* pw0, const felt* pw1, felt ninv, felt* out) {
  const uint32_t logE = logn < OOD_LOGE ? logn : OOD_LOGE;
  const uint32_t nb = 1u << (logn - logE);
  LAUNCH(prof, "eval_bitrev_tail", s, (double)narrays * nb * 32.0,
         hipLaunchKernelGGL(k_eval_bitrev_tail, dim3(narrays), dim3(TPB), 0, s, partial, nb,
                            (uint32_t)kc::ilog2_u64(nbl), narrays, logn, logE, pw0, pw1, ninv, out));
}

void launch_eval_bitrev(Prof& prof, hipStream_t s, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn,
                        const felt* pw0, const felt* pw1, felt* partial, felt ninv, felt* out) {
  const uint32_t logE = logn < OOD_LOGE ? logn : OOD_LOGE;
  const uint32_t nb = 1u << (logn - logE);
  launch_eval_bitrev_blocks(prof, s, arrays, narrays, ntwo, logn, pw0, pw1, 0, nb, partial);
  launch_eval_bitrev_tail(prof, s, partial, narrays, logn, nb, pw0, pw1, ninv, out);
}

void launch_deep_denominators(Prof& prof, hipStream_t s, const PointMap& m, uint64_t count, const felt* zz,
                              const felt* pw, felt* binv) {
  if (count & ((1ull << m.logn) - 1))  // whole cosets only (closed-form total)
    launch_fail(ZKP_ERR_DEVICE, "internal: DEEP denominators over a partial coset");
  launch_den_inverse(prof, s, m, count, zero(), zero(), 1, binv, zz, pw);
}

void launch_deep_lincomb(Prof& prof, hipStream_t s, const felt* coef, uint32_t w, uint64_t n, uint64_t p0,
                         uint64_t np, const felt* gamma, felt* out, felt* scratch) {
  const uint32_t G = scratch ? lincomb_groups(np, w) : 1u, cpg = (w + G - 1) / G;
  const dim3 g(blocks_for((np + LIN_CH - 1) / LIN_CH), G);
  if (G == 1) {
    LAUNCH(prof, "deep_lincomb", s, (double)(w + 1) * np * 16.0,
           hipLaunchKernelGGL(k_deep_lincomb<false>, g, dim3(TPB), 0, s, coef, w, n, p0, np, gamma, cpg, out));
    return;
  }
  LAUNCH(prof, "deep_lincomb", s, (double)(w + 1) * np * 16.0,
         hipLaunchKernelGGL(k_deep_lincomb<true>, g, dim3(TPB), 0, s, coef, w, n, p0, np, gamma, cpg, scratch));
  LAUNCH(prof, "deep_lincomb", s, (double)(G + 1) * np * 16.0,
         hipLaunchKernelGGL(k_sum_groups, dim3(blocks_for(np)), dim3(TPB), 0, s, scratch, G, np, out));
}

void launch_deep(Prof& prof, hipStream_t s, const DeepArgs& a, felt* out) {
  uint64_t N = 1ull << (a.logn + a.logBl);
  LAUNCH(prof, "deep", s, (double)N * ((a.w + a.C) * 16.0 + 16.0),
         hipLaunchKernelGGL(k_deep, dim3(blocks_for((N + EVAL_CH - 1) / EVAL_CH)), dim3(TPB), 0, s, a, a.binv, out));
}

void launch_comp_dft(Prof& prof, hipStream_t s, const felt* recv, const uint32_t* blk, const felt* Si,
                     const felt* consts, uint32_t ce, uint32_t C, uint32_t logn, uint64_t p0, uint64_t nR, felt* out,
                     uint32_t* hi_flag) {
  const double bytes = (double)nR * (2 * ce + C) * 16.0;
  const dim3 g(blocks_for(nR));
  switch (ce) {
    case 2: LAUNCH(prof, "comp_dft", s, bytes, hipLaunchKernelGGL(k_comp_dft<2>, g, dim3(TPB), 0, s, recv, blk, Si,
                                                                   consts, C, logn, p0, nR, out, hi_flag)); break;
    case 4: LAUNCH(prof, "comp_dft", s, bytes, hipLaunchKernelGGL(k_comp_dft<4>, g, dim3(TPB), 0, s, recv, blk, Si,
                                                                   consts, C, logn, p0, nR, out, hi_flag)); break;
    case 8: LAUNCH(prof, "comp_dft", s, bytes, hipLaunchKernelGGL(k_comp_dft<8>, g, dim3(TPB), 0, s, recv, blk, Si,
                                                                   consts, C, logn, p0, nR, out, hi_flag)); break;
    case 16: LAUNCH(prof, "comp_dft", s, bytes, hipLaunchKernelGGL(k_comp_dft<16>, g, dim3(TPB), 0, s, recv, blk,
                                                                    Si, consts, C, logn, p0, nR, out, hi_flag)); break;
    default: launch_fail(ZKP_ERR_UNSUPPORTED_AIR, "composition DFT supports ce in {2, 4, 8, 16}");
  }
}

void launch_gather_multi(Prof& prof, hipStream_t s, const GatherSeg* segs, uint32_t nseg, uint64_t max_count,
                         const uint64_t* idx, uint32_t* out, double bytes) {
  LAUNCH(prof, "gather", s, bytes,
         hipLaunchKernelGGL(k_gather_multi, dim3(blocks_for(max_count), nseg), dim3(TPB), 0, s, segs, idx, out));
}

void launch_gather_felts(Prof& prof, hipStream_t s, const felt* src, const uint64_t* idx, felt* out, uint64_t count) {
  LAUNCH(prof, "gather", s, count * 32.0,
         hipLaunchKernelGGL(k_gather_felts, dim3(blocks_for(count)), dim3(TPB), 0, s, src, idx, out, count));
}

void launch_gather_digests(Prof& prof, hipStream_t s, const uint32_t* nodes, const uint64_t* idx, uint32_t* out,
                           uint64_t count) {
  LAUNCH(prof, "gather", s, count * 40.0,
         hipLaunchKernelGGL(k_gather_digests, dim3(blocks_for(count)), dim3(TPB), 0, s, nodes, idx, out, count));
}

void launch_gu_trace(Prof& prof, hipStream_t s, const felt* masked, const felt* raw, const felt* local,
                     uint64_t ndev, felt kinv, uint64_t n, felt* tile_buf, felt* out) {
  const uint32_t tiles = (uint32_t)((n + GU_TILE - 1) / GU_TILE);
  LAUNCH(prof, "gu_trace_sums", s, (double)ndev * GU_D_DEV * 16.0,
         hipLaunchKernelGGL(k_gu_tile_sums, dim3(tiles, GU_D_DEV), dim3(TPB), 0, s, masked, raw, local, ndev, kinv,
                            n, tile_buf));
  LAUNCH(prof, "gu_trace_scan", s, (double)tiles * GU_D_DEV * 32.0,
         hipLaunchKernelGGL(k_gu_tile_scan, dim3(GU_D_DEV), dim3(64), 0, s, tile_buf, tiles));
  LAUNCH(prof, "gu_trace_write", s, (double)n * 2 * GU_D_DEV * 16.0 + (double)ndev * GU_D_DEV * 16.0,
         hipLaunchKernelGGL(k_gu_tile_write, dim3(tiles, 2 * GU_D_DEV), dim3(TPB), 0, s, masked, raw, local, ndev,
                            kinv, n, tile_buf, out));
}

void launch_dt_eval_consts(Prof& prof, hipStream_t s, int air, const felt* cc, felt k, felt w_last, const felt* aval,
                           const felt* zinv, uint32_t ce, uint32_t w, uint32_t num_t, felt* out) {
  LAUNCH(prof, "coin", s, 0.0,
         hipLaunchKernelGGL(k_dt_eval_consts, dim3(1), dim3(TPB), 0, s, air, cc, k, w_last, aval, zinv, ce, w, num_t, out));
}

void launch_gu_check(Prof& prof, hipStream_t s, const felt* T, uint32_t d, uint32_t logn, felt k, uint32_t c0,
                     uint32_t cw, uint64_t t0, uint32_t logtn, felt* cval, uint32_t* bad) {
  const uint64_t cnt = (uint64_t)cw << logtn;
  LAUNCH(prof, "gu_pair", s, (double)cnt * 32.0,
         hipLaunchKernelGGL(k_gu_check, dim3(blocks_for(cnt)), dim3(TPB), 0, s, T, d, logn, k, c0, cw, t0, logtn,
                            cval, bad));
}

void launch_mimc_check(Prof& prof, hipStream_t s, const felt* T, uint64_t n, felt v0, felt v1, uint32_t* bad) {
  LAUNCH(prof, "trace_check", s, (double)n * 16.0,
         hipLaunchKernelGGL(k_mimc_check, dim3(blocks_for(n)), dim3(TPB), 0, s, T, n, v0, v1, bad));
}

void launch_gu_coef(Prof& prof, hipStream_t s, felt* coef, uint32_t d, uint32_t logn, felt k, const felt* itwn,
                    uint32_t c0, uint32_t cw, uint64_t p0, uint64_t np, const felt* cval) {
  LAUNCH(prof, "gu_pair", s, (double)np * cw * 32.0,
         hipLaunchKernelGGL(k_gu_coef, dim3(blocks_for(np)), dim3(TPB), 0, s, coef, d, logn, k, itwn, c0, cw, p0, np,
                            cval));
}

void launch_gu_lde(Prof& prof, hipStream_t s, felt* lde, uint32_t d, uint32_t logn, uint32_t logBl, felt k,
                   uint32_t c0, uint32_t cw, const felt* cval, const felt* l0) {
  const uint64_t cnt = 1ull << (logn + logBl);
  const bool smallk = k.hi == 0 && (k.lo >> 32) == 0;
  if (smallk)
    LAUNCH(prof, "gu_pair", s, (double)cnt * (cw * 32.0 + 16.0),
           hipLaunchKernelGGL(k_gu_lde<true>, dim3(blocks_for(cnt)), dim3(TPB), 0, s, lde, d, logn, logBl, k, c0, cw,
                              cval, l0));
  else
    LAUNCH(prof, "gu_pair", s, (double)cnt * (cw * 32.0 + 16.0),
           hipLaunchKernelGGL(k_gu_lde<false>, dim3(blocks_for(cnt)), dim3(TPB), 0, s, lde, d, logn, logBl, k, c0, cw,
                              cval, l0));
}

size_t l0_scratch_felts(uint64_t count, uint32_t logn) {
  return (size_t)blocks_for((count + EVAL_CH - 1) / EVAL_CH) + (size_t)(count >> logn) + 1;
}

void launch_l0_table(Prof& prof, hipStream_t s, const PointMap& pm, uint64_t count, felt ninv, felt* out,
                     felt* scratch) {
  const uint32_t nb = blocks_for((count + EVAL_CH - 1) / EVAL_CH), ncos = (uint32_t)(count >> pm.logn);
  felt* K = scratch + nb;
  LAUNCH(prof, "l0_consts", s, (double)ncos * 16.0,
         hipLaunchKernelGGL(k_l0_consts, dim3(1), dim3(64), 0, s, pm, ncos, ninv, K));
  launch_den_inverse(prof, s, pm, count, one(), one(), 0, scratch);
  LAUNCH(prof, "l0_table", s, (double)count * 16.0,
         hipLaunchKernelGGL(k_l0_table, dim3(nb), dim3(TPB), 0, s, pm, count, K, scratch, out));
}

void launch_gu_fill(Prof& prof, hipStream_t s, felt* lde, uint32_t w, uint32_t logn, uint32_t logB, uint32_t j0,
                    uint32_t logBl, const uint64_t* pos, uint32_t npos, const GuLazy& gl) {
  const uint64_t cnt = (uint64_t)npos * (w - gl.wi);
  if (!cnt) return;
  LAUNCH(prof, "gu_pair", s, (double)cnt * 48.0,
         hipLaunchKernelGGL(k_gu_fill, dim3(blocks_for(cnt)), dim3(TPB), 0, s, lde, w, logn, logB, j0, logBl, pos, npos,
                            gl));
}
