// zkp_internal.hpp — declarations shared by the kernel TU and the host prover.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "felt.hpp"

// ---------------------------------------------------------------- profiling
// Every launch goes through Prof::begin/end; when enabled each launch is
// bracketed by HIP events recorded on the stream it runs on.
struct ProfRec {
  const char* name;
  double bytes;  // algorithmic (compulsory) HBM bytes of this launch
  hipEvent_t start, stop;
};
struct Prof {
  bool enabled = false;
  std::string only;   // non-empty: bracket only the launches of this name
  bool open = false;  // the current launch is bracketed
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool;
  hipEvent_t get_event();
  void begin(const char* name, hipStream_t s, double bytes);
  void end(hipStream_t s);
};

// A launch the kernels cannot take (a shape past their 32-bit offsets, a broken
// internal invariant): thrown as the calling entry point's ZKP_ERR_* status
// (prover.cpp), never an abort() across the C ABI.
[[noreturn]] void launch_fail(int code, const char* what);
// largest LDE domain (n * blowup) the NTT passes index with 32-bit element
// offsets, and the largest trace the OOD evaluation's block tree takes; entry
// points return ZKP_ERR_TRACE_SHAPE past them
constexpr uint32_t MAX_LOG_DOMAIN = 28, MAX_LOG_TRACE = 23;
// Load each kernel translation unit's gfx950 code object on the current device
// now (zkp_ctx_create) instead of at its first launch inside a proof: HIP loads
// a fat binary's code object lazily, on the first use of one of its kernels.
void preload_kernels_module();
void preload_merkle_module();
void preload_ntt_module();
// one empty launch on `s`: HIP binds a stream to a hardware queue at its first dispatch
void warm_stream(hipStream_t s);

// ---------------------------------------------------------------- NTT
// One LDS pass of K radix-2 stages (see kernels.hip). `dit` = bit-reversed in
// -> natural out (Cooley-Tukey); otherwise natural in -> bit-reversed out
// (Gentleman-Sande). Stages [s0, s0+K).
struct NttPass {
  uint32_t logn, s0, K, lo, T, Tl;
};
std::vector<NttPass> ntt_plan(uint32_t logn, bool dit);

struct NttBatch {
  const felt* src;     // batch b reads src + (b / src_div) * src_stride
  felt* dst;           // batch b writes dst + b * dst_stride
  const felt* scale;   // nullable; multiplies element p of batch b by scale[(b % scale_mod) * n + p] on load
  uint64_t src_stride, dst_stride;
  uint32_t src_div, scale_mod, batches;
};

// Full transform over `batches` arrays of size 2^logn using the stage-major
// twiddle table tw (level t at tw[2^t - 1 .. 2^(t+1) - 1) holds w_{2^(t+1)}^j;
// forward table for DIT, inverse table for DIF).
// only_pass >= 0: launch that pass of the plan alone (a caller pipelining the passes of
// several batches over two streams: pass 1 of batch k+1 beside pass 2 of batch k);
// ntt_passes(logn) = the number of passes of the plan (1 for the radix-2 path)
void launch_ntt(Prof& prof, hipStream_t s, const NttBatch& b, uint32_t logn, bool dit, const felt* tw,
                uint32_t logN, int only_pass = -1);
uint32_t ntt_passes(uint32_t logn);

// ---------------------------------------------------------------- tables
// fill levels 0..top-1 of a stage-major table whose level `top` is present
void launch_build_levels(Prof& prof, hipStream_t s, felt* tab, uint32_t top);
void launch_expand_powers(Prof& prof, hipStream_t s, felt* out, uint64_t count, const felt* lo_tab,
                          const felt* hi_tab);
// S[j*n + p] = ninv * (g * w_N^j)^rev(p)   (j < B; with g^-1 powers and the
// inverse table of a 2^logN domain this builds the inverse coset tables)
void launch_build_coset_scale(Prof& prof, hipStream_t s, felt* S, uint32_t logn, uint32_t B,
                              const felt* tw, uint32_t logN, const felt* glo, const felt* ghi, felt ninv);

// ---------------------------------------------------------------- hashing
// leaves L (= n*B) of a coset-major LDE matrix (cols x B x n) -> nodes[L + i] (8 words each)
void launch_leaf_hash_lde(Prof& prof, hipStream_t s, const felt* lde, uint32_t cols, uint32_t logB,
                          uint64_t n, uint32_t* nodes, uint64_t L);
// leaves of FRI layer: row r = [E[r + k*R] for k < F] -> nodes[R + r]
void launch_leaf_hash_fri(Prof& prof, hipStream_t s, const felt* E, uint64_t R, uint32_t F, uint32_t* nodes);
// fused builders: leaves + all levels (nodes[1..2L)) in ceil(log2(L)/9) launches
// Optional tree tail: with done (a zeroed per-stream counter) the launch that
// produces the top subtree roots also finishes the tree in its last block and,
// with coin_seed, runs the FRI coin step (seed <- H(seed || root), alpha_out,
// root_out). The launchers return true when the tail ran.
// op: what the last block does with the root (coin state in coin_seed):
//   MERKLE_TAIL_FRI_COIN    reseed, draw alpha -> alpha_out, root -> root_out
//   MERKLE_TAIL_DRAW_COEFFS reseed, draw ncoef composition coefficients -> out
//   MERKLE_TAIL_DRAW_Z      reseed, draw z -> out = (z, z wn), pw tables (logn each)
enum { MERKLE_TAIL_NONE = 0, MERKLE_TAIL_FRI_COIN = 1, MERKLE_TAIL_DRAW_COEFFS = 2, MERKLE_TAIL_DRAW_Z = 3 };
struct MerkleTail {
  uint32_t* done;
  uint32_t* coin_seed;
  felt* alpha_out;
  uint32_t* root_out;
  uint32_t op, method, ncoef, logn;
  felt wn;
  felt* out;
  felt* pw;
};
// The last composition column derived in the leaf pass instead of extended by an
// NTT. On an LDE coset j that is also a CE coset (ce == B), x^n = kappa_j is
// constant and H(x) = sum_c kappa_j^c H_c(x) (CompositionPoly splits H into C
// columns of n coefficients), so H_{C-1}(x) = (H(x) - sum_{c<C-1} kappa_j^c H_c(x))
// * kappa_j^-(C-1): C-1 products per row instead of one coset NTT per coset.
// H = the constraint evaluations (H[jl*n + t], coset jl of the source), kap[2*jl]
// = kappa, kap[2*jl+1] = kappa^-(C-1); the derived value is written to out[jl*n + t]
// (the source's column C-1) and hashed with the row.
struct LastCol {
  const felt* H;
  const felt* kap;
  felt* out;
};
// GlobalUpdate paired columns that are never materialized: the row hash derives
// column c >= wi as k*(lde_{c-d}[t] - lde_{c-d}[t-1]) + cval[c-d]*l0[q] (q = the
// row's index over the source's cosets, t-1 the previous row of its coset; see
// kernels.hip k_gu_lde), and launch_gu_fill writes them for the queried rows only
struct GuLazy {
  const felt* cval;
  const felt* l0;
  felt k;
  uint32_t d, wi, smallk;
};
bool launch_merkle_lde(Prof& prof, hipStream_t s, const felt* lde, uint32_t cols, uint32_t logB, uint64_t n,
                       uint32_t* nodes, uint64_t L, const MerkleTail* tail = nullptr, const LastCol* lc = nullptr,
                       const GuLazy* gl = nullptr);
// FRI layer tree over coset-major evaluations (B cosets of 16*m16): leaf r = j + B*t'
bool launch_merkle_fri(Prof& prof, hipStream_t s, const felt* E, uint64_t m16, uint32_t logB, uint32_t F,
                       uint32_t* nodes, const MerkleTail* tail = nullptr);
// nodes[1..L) from leaf digests already in nodes[L..2L)
bool merkle_upper(Prof& prof, hipStream_t s, uint32_t* nodes, uint64_t L, const MerkleTail* tail = nullptr);
// sharded commitments: hash the shard's rows (mode 0: LDE rows of cols columns;
// mode 1: FRI rows of 16) into per-destination blocks; then, after the
// all-to-all, rebuild the natural-order leaves of this rank's range and its subtree
// all-to-all in 2^logK chunks along the destination rows: launch_leaf_hash_shard hashes chunk k
void launch_leaf_hash_shard(Prof& prof, hipStream_t s, int mode, const felt* src, uint64_t n, uint32_t cols,
                            uint32_t logBl, uint32_t logrows, uint32_t logrr, uint32_t logK, uint32_t k,
                            uint32_t* send, const LastCol* lc = nullptr, const GuLazy* gl = nullptr);
// sharded tree tops (R <= 64 subtree roots, all-gathered) -> top[1..2R) on the device,
// then the tail's coin step on the root (tail nullable / MERKLE_TAIL_NONE: none)
void launch_shard_top(Prof& prof, hipStream_t s, const uint32_t* roots, uint32_t R, uint32_t* top,
                      const MerkleTail* tail);
void launch_merkle_from_shards(Prof& prof, hipStream_t s, const uint32_t* recv, uint32_t logB, uint32_t logrr,
                               uint32_t logK, uint32_t* nodes, uint32_t* done = nullptr);
// internal nodes nodes[1..L) from leaves nodes[L..2L)
void launch_merkle_tree(Prof& prof, hipStream_t s, uint32_t* nodes, uint64_t L);
constexpr uint32_t PACK_MAX = 16;
struct PackArgs {
  const void* src[PACK_MAX];
  uint64_t bytes[PACK_MAX], off[PACK_MAX];
  uint32_t n;
};
// dst[off[i] ..) = src[i][0 .. bytes[i]) for i < n (byte counts multiples of 4)
void launch_pack(Prof& prof, hipStream_t s, const PackArgs& a, void* dst);
// seed from host words, or (seed_words == nullptr) from the device coin state seed_dev
void launch_grind(Prof& prof, hipStream_t s, const uint32_t* seed_words, const uint32_t* seed_dev, uint64_t base,
                  uint64_t count, uint32_t bits, unsigned long long* result);
// remainder of a last FRI layer of D = m * 2^logB <= 256 values (coefficients
// rem_out[0..m)), commitment H(remainder) and the coin reseed with it (seed in place)
void launch_fri_remainder(Prof& prof, hipStream_t s, const felt* E, uint32_t logB, uint32_t m, felt off_inv,
                          felt wd_inv, felt d_inv, uint32_t* seed, felt* rem_out, uint32_t* commit_out);

// ---- device query tail (world 1): grinding to completion, query positions,
// and every opening of every possible batch proof (rows + full sibling paths)
void launch_grind_all(Prof& prof, hipStream_t s, const uint32_t* seed_dev, uint64_t base, uint64_t limit,
                      uint32_t bits, unsigned long long* result);
// raw DefaultRandomCoin::draw_integers(q, N, *nonce) from the device coin state
void launch_query_positions(Prof& prof, hipStream_t s, const uint32_t* seed_dev, const unsigned long long* nonce,
                            uint32_t q, uint64_t N, uint64_t* pos);
constexpr uint32_t GATHER_MAX_LAYERS = 16;
struct FullGatherArgs {
  const felt* tlde;      // w x B x n (coset-major)
  const felt* clde;      // C x B x n
  const uint32_t* tnodes;
  const uint32_t* cnodes;
  uint64_t n;
  uint32_t w, C, logB, logN, nlayers;
  const felt* E[GATHER_MAX_LAYERS];         // FRI layer l evaluations, coset-major (m[l] per coset)
  const uint32_t* fnodes[GATHER_MAX_LAYERS];
  uint64_t m[GATHER_MAX_LAYERS];
  uint32_t logrows[GATHER_MAX_LAYERS];      // log2 of the layer's tree leaves (rows)
  uint64_t seg_off[GATHER_MAX_LAYERS + 1];  // words
  uint32_t rec_words[GATHER_MAX_LAYERS + 1];
};
// record of raw position i in segment 0: [w + C row felts | trace path | constraint path]
// (logN sibling digests each, leaf level first); segment 1 + l: [16 felts | logrows[l] digests]
void launch_gather_full(Prof& prof, hipStream_t s, const FullGatherArgs& a, uint32_t q, const uint64_t* pos,
                        uint32_t* out);

// ---------------------------------------------------------------- device transcript
// (seed = 8 LE words of the DefaultRandomCoin state, in device memory)
// reseed with `root` (device), then draw `ncoef` composition coefficients into cc
void launch_dt_draw_coeffs(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, uint32_t method,
                           uint32_t ncoef, felt* cc);
// coefficient-dependent constants of the eval kernels (layout in kernels.hip)
void launch_dt_eval_consts(Prof& prof, hipStream_t s, int air, const felt* cc, felt k, felt w_last, const felt* aval,
                           const felt* zinv, uint32_t ce, uint32_t w, uint32_t num_t, felt* out);
// OOD frame -> reseeds -> DEEP coefficients gamma (w + C) and dk[2..4) = kz, kzg
// (ood[2a + {0,1}] = array a at z, zg; dk[0..2) = z, zg already)
void launch_dt_deep_coeffs(Prof& prof, hipStream_t s, uint32_t* seed, const felt* ood, uint32_t w, uint32_t C,
                           uint32_t method, felt* gamma, felt* dk);
// reseed with the constraint root, draw z: zz = (z, z w_n), pw = z^(2^l) || (z w_n)^(2^l), l < logn
void launch_dt_draw_z(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, felt wn, uint32_t logn,
                      felt* zz, felt* pw);

// ---------------------------------------------------------------- trace building
// GlobalUpdate trace (120 x n, column-major) from masked/raw global models (60 each),
// ndev x 60 local models and k^-1 (src/aggregation/prover.rs:98-160); tile_buf holds
// 60 * ceil(n / 4096) felts
void launch_gu_trace(Prof& prof, hipStream_t s, const felt* masked, const felt* raw, const felt* local,
                     uint64_t ndev, felt kinv, uint64_t n, felt* tile_buf, felt* out);

// ---------------------------------------------------------------- constraints
// Points of a coset-major shard: local index q = c*n + t is cx[c] * w_n^t,
// cx[c] = g * w_N^(j of local coset c), twn = w_n^t for t < n/2 (the
// stage-major twiddle level logn-1, read contiguously).
struct PointMap {
  const felt* cx;
  const felt* twn;
  uint32_t logn;
};

// The shard evaluates the CE cosets u in [u0, u0 + cel) (CE coset u lives in
// LDE coset u * B/ce); its LDE matrices hold the cosets [j0, j0 + 2^logBl).
struct EvalCommon {
  uint32_t logn, logB, logce, logN;
  uint32_t u0, cel, j0, logBl;
  felt g, w_last;        // domain offset (3), w_n^(n-1)
  PointMap pm;           // x of the shard's CE points (cx per owned CE coset)
  const felt* zinv;      // ce entries: 1/(x^n - 1) on the CE domain (x^n = g^n * w_ce^s);
                         // for MiMC pre-multiplied by the transition coefficient
};
// MiMC: x' - (x + K)^7 ; boundary steps 0 and n-1 on column 0
struct MimcEvalArgs {
  const felt* bcoef;     // device: A, Bc, Cc, D of the regrouped boundary numerator (k_dt_eval_consts)
  const felt* kper;      // 64*ce periodic values on the CE domain
  felt* binv;            // scratch: one felt per 2048 CE points (per-block inverse products)
  felt* dinv;            // M felts: 1/((x - 1)(x - w^(n-1))) per CE point (domain-only, cached in the ctx)
  bool binv_ready;       // dinv already holds this domain's values
};
void launch_eval_mimc(Prof& prof, hipStream_t s, const EvalCommon& c, const MimcEvalArgs& a, const felt* lde,
                      felt* comp);
// linear AIRs (GlobalUpdate, TrainingUpdate): optional transition
// T = sum_c a_c*next_c + b_c*cur_c over Z_T; boundary group 0 at step b0
// (sum_c beta0_c*cur_c - bconst over x - w^b0) and optional group 1 at step b1.
// coefs = [a (width) | b (width) | beta0 (width) | beta1 (width)], width = columns read
struct LinearEvalArgs {
  uint32_t width;
  bool transition, two_groups;
  const felt* coefs;     // device: 4 * width coefficient rows, then bconst0, bconst1
  felt w_bstep, w_bstep1;
  felt* binv;            // scratch: one felt per 2048 CE points
  felt* dinv;            // M felts: the boundary divisor inverses per CE point (cached in the ctx)
  bool binv_ready;       // dinv already holds this domain's values
};
void launch_eval_linear(Prof& prof, hipStream_t s, const EvalCommon& c, const LinearEvalArgs& a, const felt* lde,
                        felt* comp);
// the same in coefficient form (kernels.hip, k_lin_lincomb): the coefficients of
// [A (trans) | B0 | B1 (two)] over bit-reversed positions [p0, p0 + np) of the
// first W coefficient columns (out: np felts per array; twn[j] = w_n^j, j < n/2),
// then, once they are extended to the shard's CE cosets (ev: cel*n per array),
// the per-point formula of k_eval_linear
// Small position ranges split the columns into lincomb_groups(np, W) groups
// (partial sums in `scratch`: 4 * np felts per group, nullable = one group).
uint32_t lincomb_groups(uint64_t np, uint32_t W);
void launch_lin_lincomb(Prof& prof, hipStream_t s, bool trans, bool two, const felt* coef, uint32_t W, uint32_t logn,
                        uint64_t p0, uint64_t np, const felt* coefs, const felt* twn, felt* out, felt* scratch);
void launch_eval_linear_pts(Prof& prof, hipStream_t s, const EvalCommon& c, const LinearEvalArgs& a, const felt* ev,
                            felt* comp);

// GlobalUpdate column pairing (kernels.hip): columns d+i from columns i < d for a
// trace whose transitions hold. check: rows [t0, t0 + 2^logtn) of pairs c0..c0+cw of
// the natural trace (*bad = 1 on a mismatch; row 0 gives c_i); coef: the derived
// coefficient columns at positions [p0, p0 + np) (itwn = the inverse w_n table
// level); lde: the derived LDE columns over Bl cosets (l0 = L_0 over those cosets,
// launch_l0_table)
// MiMC trace vs its transition and assertions (sets *bad on any failing row)
void launch_mimc_check(Prof& prof, hipStream_t s, const felt* T, uint64_t n, felt v0, felt v1, uint32_t* bad);
void launch_gu_check(Prof& prof, hipStream_t s, const felt* T, uint32_t d, uint32_t logn, felt k, uint32_t c0,
                     uint32_t cw, uint64_t t0, uint32_t logtn, felt* cval, uint32_t* bad);
void launch_gu_coef(Prof& prof, hipStream_t s, felt* coef, uint32_t d, uint32_t logn, felt k, const felt* itwn,
                    uint32_t c0, uint32_t cw, uint64_t p0, uint64_t np, const felt* cval);
void launch_gu_lde(Prof& prof, hipStream_t s, felt* lde, uint32_t d, uint32_t logn, uint32_t logBl, felt k,
                   uint32_t c0, uint32_t cw, const felt* cval, const felt* l0);
// scratch: l0_scratch_felts(count, logn) felts (block products + per-coset constants)
size_t l0_scratch_felts(uint64_t count, uint32_t logn);
void launch_l0_table(Prof& prof, hipStream_t s, const PointMap& pm, uint64_t count, felt ninv, felt* out,
                     felt* scratch);
// the lazy paired columns [wi, w) of the queried rows: pos = natural LDE indices
// (npos of them), the rows of cosets [j0, j0 + 2^logBl) held here are written
void launch_gu_fill(Prof& prof, hipStream_t s, felt* lde, uint32_t w, uint32_t logn, uint32_t logB, uint32_t j0,
                    uint32_t logBl, const uint64_t* pos, uint32_t npos, const GuLazy& gl);

// composition polynomial from CE-coset interpolations (see kernels.hip): for the
// bit-reversed positions [p0, p0 + nR), n * c_m = (sum_u Si_u * W_u * w_ce^-um) * g^-mn / ce;
// consts = [g^-mn / ce for m < C | w_ce^-k for k < ce/2] (ce in {2, 4, 8, 16})
void launch_comp_dft(Prof& prof, hipStream_t s, const felt* recv, const uint32_t* blk, const felt* Si,
                     const felt* consts, uint32_t ce, uint32_t C, uint32_t logn, uint64_t p0, uint64_t nR, felt* out,
                     uint32_t* hi_flag = nullptr);

// OOD evaluation of bit-reversed arrays (arrays contiguous, stride n) at x0 and x1
// partial[(a * nblocks + b) * 2 + {0,1}] ; pw0/pw1 = x^(2^l) tables (logn entries, device)
// (arrays a >= ntwo at x0 only)
void launch_eval_bitrev(Prof& prof, hipStream_t s, const felt* arrays, uint32_t narrays, uint32_t ntwo, uint32_t logn,
                        const felt* pw0, const felt* pw1, felt* partial, felt ninv, felt* out);
// its two halves for a sharded proof: a rank evaluates the 2048-coefficient blocks
// [b0, b0 + nbl) of every array (partial[(a * nbl + b - b0) * 2 + k]); after the
// all-gather of those rank blocks the tail combines all n / 2048 of them
void launch_eval_bitrev_blocks(Prof& prof, hipStream_t s, const felt* arrays, uint32_t narrays, uint32_t ntwo,
                               uint32_t logn, const felt* pw0, const felt* pw1, uint32_t b0, uint32_t nbl,
                               felt* partial);
void launch_eval_bitrev_tail(Prof& prof, hipStream_t s, const felt* partial, uint32_t narrays, uint32_t logn,
                             uint32_t nbl, const felt* pw0, const felt* pw1, felt ninv, felt* out);

// DEEP composition over the LDE domain (natural order out)
struct DeepArgs {
  uint32_t w, C, logB, logn, logN;
  uint32_t j0, logBl;    // shard cosets [j0, j0 + 2^logBl); output coset-major
  const felt* tlde;      // w x Bl x n
  const felt* clde;      // C x Bl x n
  const felt* gamma;     // w + C
  const felt* dk;        // device: z, z*w_n, kz, kzg (drawn / formed on the device)
  felt g;
  PointMap pm;           // x of the shard's LDE points (cx per owned coset)
  felt* binv;            // scratch: one felt per 2048 LDE points
};
// phases 1-2 of the DEEP batch inversion (block inverse products of (x - z)(x - zg)
// into binv); launch_deep then runs phase 3 + the composition
void launch_deep_denominators(Prof& prof, hipStream_t s, const PointMap& m, uint64_t count, const felt* zz,
                              const felt* pw, felt* binv);
void launch_deep(Prof& prof, hipStream_t s, const DeepArgs& a, felt* out);
// coefficient-form DEEP for wide traces (winterfell combines the trace polynomials
// before extending): out[p] = sum_{c < w} gamma[c] * coef[c*n + p]
// over the bit-reversed, n-scaled coefficient columns -> one combined column (same layout)
void launch_deep_lincomb(Prof& prof, hipStream_t s, const felt* coef, uint32_t w, uint64_t n, uint64_t p0,
                         uint64_t np, const felt* gamma, felt* out,  // positions [p0, p0 + np) -> out[0, np)
                         felt* scratch);  // column-group partials (np per group, see lincomb_groups), nullable

// FRI fold-by-F (F = 16) over coset-major evaluations of the cosets [j0, j0+Bl)
// (16*m16 positions each): natural row r = j + B*t', x_r = off * w_D^r; alpha read from device
void launch_fri_fold(Prof& prof, hipStream_t s, const felt* E, uint64_t m16, uint32_t Bl, uint32_t j0,
                     uint32_t logB, uint32_t F, const felt* alpha, felt off_inv, const felt* itw, uint32_t logD,
                     const felt* eps_inv_dev, felt* out);
// the FRI tail in one block (world 1): layers of <= 128 rows (tree, coin step,
// fold) and the remainder, in order
constexpr uint32_t FRI_TAIL_MAX = 4;
struct FriTailLayer {
  const felt* E;        // layer evaluations, coset-major (B cosets of 16 * 2^logm16)
  uint32_t* nodes;      // the layer's tree (16 * rows words)
  uint32_t logm16;
  felt off_inv;
  const felt* lev;      // w_D^-r table of the layer's domain
  felt* out;            // folded evaluations (the next layer)
  felt* alpha_out;      // device transcript slots
  uint32_t* root_out;
};
struct FriTailArgs {
  uint32_t nl, logB;
  FriTailLayer ly[FRI_TAIL_MAX];
  uint32_t* coin_seed;
  const felt* eps_inv;
  const felt* rem_E;    // last layer: rem_m positions per coset
  uint32_t rem_m;
  felt rem_off_inv, wd_inv, d_inv;
  felt* rem_out;
  uint32_t* commit_out;
};
void launch_fri_tail(Prof& prof, hipStream_t s, const FriTailArgs& a);
// device-side coin step of the FRI loop: seed = merge(seed, root); *alpha_out = draw(); root copied to root_out
void launch_coin_fri_layer(Prof& prof, hipStream_t s, uint32_t* seed, const uint32_t* root, felt* alpha_out,
                           uint32_t* root_out);

// gathers for query openings
struct GatherSeg {
  const void* src;
  uint64_t idx_off, count, out_off;  // out_off in 32-bit words
  uint32_t words;                    // 4 (felt) or 8 (digest)
  uint32_t pad;
};
void launch_gather_multi(Prof& prof, hipStream_t s, const GatherSeg* segs, uint32_t nseg, uint64_t max_count,
                         const uint64_t* idx, uint32_t* out, double bytes);
void launch_gather_felts(Prof& prof, hipStream_t s, const felt* src, const uint64_t* idx, felt* out, uint64_t count);
void launch_gather_digests(Prof& prof, hipStream_t s, const uint32_t* nodes, const uint64_t* idx, uint32_t* out,
                           uint64_t count);
