/*
 * zkp.h — C-ABI of the MI355X-native STARK prover (libzkp.so).
 *
 * Drop-in boundary for the reference's proving path: winterfell 0.12's
 * `Prover::prove(&self, trace) -> Result<Proof, ProverError>` as driven by the
 * project's plug-ins
 *   /root/reference/src/aggregation/prover.rs:194-248  (GlobalUpdateProver)
 *   /root/reference/src/training/prover.rs:221-300     (TrainingUpdateProver)
 * and called from /root/reference/src/main.rs:228,424,468.
 * The `Default*` engine components those plug-ins select (DefaultTraceLde,
 * DefaultConstraintEvaluator, DefaultConstraintCommitment, Blake3_256,
 * MerkleTree, DefaultRandomCoin, FRI) are what this library replaces.
 *
 * Conventions
 *  - Field: winter-math f128 (p = 2^128 - 45*2^40 + 1). A felt is 16 bytes,
 *    canonical, little-endian: identical to `BaseElement` memory and to
 *    `Serializable` bytes (reference: src/aggregation/air.rs:10).
 *  - Traces are column-major (`ColMatrix`, what `TraceTable::init(transpose(rows))`
 *    produces: src/aggregation/prover.rs:157-160, src/helper.rs:197-211):
 *    element (row r, column c) lives at cols[c * n + r].
 *  - Inputs are borrowed for the call; outputs are callee-allocated and
 *    released with zkp_free(). No exceptions or aborts cross the ABI: every
 *    entry point returns a zkp_status.
 *  - Calls on one zkp_ctx are synchronous and must not overlap (the
 *    reference's `prove(&self)` is blocking). Use one ctx per thread.
 *  - There is no CPU fallback: if no gfx950 device is present every compute
 *    entry point fails with ZKP_ERR_DEVICE.
 */
#ifndef ZKP_H
#define ZKP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct zkp_felt {
  uint64_t lo;
  uint64_t hi;
} zkp_felt;

/* AIRs are identified by id because the device cannot run Rust
 * `Air::evaluate_transition`; parameters come from `pub_inputs.to_elements()`.
 *  MIMC          : builder-defined MiMC AIR (the reference has none, F2).
 *                  width 1, pub = [x0, x_last].
 *  GLOBAL_UPDATE : GlobalUpdateAir, src/aggregation/air.rs:89-151. width 120,
 *                  pub = GlobalUpdateInputs::to_elements() (123 felts, air.rs:57-81).
 *  TRAINING_UPDATE: TrainingUpdateAir, src/training/air.rs:101-292. width 240,
 *                  pub = TrainingUpdateInputs::to_elements() (air.rs:74-98: 244 + bs*(FE+AC)
 *                  felts); transitions identically zero (current_step() == 0). */
typedef enum zkp_air_id {
  ZKP_AIR_MIMC = 1,
  ZKP_AIR_GLOBAL_UPDATE = 2,
  ZKP_AIR_TRAINING_UPDATE = 3
} zkp_air_id;

/* winterfell `BatchingMethod`. */
enum { ZKP_BATCHING_LINEAR = 0, ZKP_BATCHING_ALGEBRAIC = 1, ZKP_BATCHING_HORNER = 2 };
/* winterfell `FieldExtension` (only None is supported, as in the reference). */
enum { ZKP_FIELD_EXTENSION_NONE = 1 };

/* winterfell `ProofOptions::new(num_queries, blowup_factor, grinding_factor,
 * field_extension, fri_folding_factor, fri_remainder_max_degree,
 * batching_constraints, batching_deep)`; the reference's set is
 * (40, 16, 21, None, 16, 7, Algebraic, Algebraic) at src/main.rs:98-107. */
typedef struct zkp_proof_options {
  uint32_t num_queries;
  uint32_t blowup_factor;
  uint32_t grinding_factor;
  uint32_t field_extension;
  uint32_t fri_folding_factor;
  uint32_t fri_remainder_max_degree;
  uint32_t batching_constraints;
  uint32_t batching_deep;
} zkp_proof_options;

/* Status codes; non-zero values map onto winterfell `ProverError` classes. */
typedef enum zkp_status {
  ZKP_OK = 0,
  ZKP_ERR_INVALID_OPTIONS = 1,
  ZKP_ERR_UNSUPPORTED_FIELD_EXTENSION = 2,
  ZKP_ERR_TRACE_SHAPE = 3,   /* n < 8, n not a power of two, width 0 or > 255, n > 2^23, n*blowup > 2^28 */
  ZKP_ERR_PUB_INPUTS = 4,    /* wrong number of public input elements / inconsistent values */
  ZKP_ERR_DEVICE = 5,        /* HIP failure or no device */
  ZKP_ERR_NONCE = 6,         /* grinding nonce not found */
  ZKP_ERR_OOM = 7,
  ZKP_ERR_UNSUPPORTED_AIR = 8,
  ZKP_ERR_ARGUMENT = 9
} zkp_status;

typedef struct zkp_ctx zkp_ctx;

/* Per-proof transcript summary (debug / parity aid; optional out-param). */
typedef struct zkp_transcript {
  uint8_t trace_root[32];
  uint8_t constraint_root[32];
  uint8_t fri_roots[16][32];
  uint8_t remainder_commitment[32];
  uint32_t num_fri_layers;
  uint32_t num_composition_columns;
  uint64_t pow_nonce;
  zkp_felt z;
  uint32_t num_unique_queries;
  uint64_t query_positions[255];
} zkp_transcript;

/* ---- context --------------------------------------------------------- */
/* Bind to HIP device `device` (ordinal). One ctx per caller thread. */
int zkp_ctx_create(int device, zkp_ctx** out);
void zkp_ctx_destroy(zkp_ctx* ctx);
/* Free the idle stage-session context the ctx keeps for its next zkp_session_create
 * (at most one; it holds the last session's device buffers and domain tables). */
int zkp_ctx_trim(zkp_ctx* ctx);
/* Last error message for ctx (static storage owned by ctx). */
const char* zkp_last_error(const zkp_ctx* ctx);
void zkp_free(void* p);

/* ---- whole-proof entry points (≙ Prover::prove) ------------------------ */
/* Host trace (column-major, width*n felts) -> serialized proof
 * (≙ winterfell `Proof::to_bytes()`, src/main.rs:229,425,469). */
int zkp_prove(zkp_ctx* ctx, zkp_air_id air, const zkp_felt* trace_cols, uint32_t width,
              uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
              const zkp_proof_options* opts, uint8_t** proof, uint64_t* proof_len,
              zkp_transcript* transcript /* nullable */);

/* Same, with the trace already resident in device memory (HBM). */
int zkp_prove_device(zkp_ctx* ctx, zkp_air_id air, const void* d_trace_cols, uint32_t width,
                     uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
                     const zkp_proof_options* opts, uint8_t** proof, uint64_t* proof_len,
                     zkp_transcript* transcript /* nullable */);

/* ---- multi-GPU: coset-sharded proving ----
 * One proof is split over `world` ranks by LDE coset (rank r owns the cosets
 * [r*B/world, (r+1)*B/world)); the exchange steps are leaf-digest all-to-alls
 * for the Merkle commitments, an all-to-all + all-gather that reassemble the
 * composition polynomial, and all-gathers of subtree roots, small FRI layers
 * and query openings. Every rank passes the full trace and returns the same
 * proof bytes (identical to zkp_prove's). world must be a power of two <= the
 * blowup factor; n >= 256 * world.
 * Replaces, for a multi-GPU node, the single `Prover::prove` call
 * (src/main.rs:424,468) — the reference itself has no multi-device path. */
typedef struct zkp_comm zkp_comm;
/* RCCL communicator (one process per GPU): rank 0 makes the id, the caller
 * broadcasts its 128 bytes (e.g. with torch.distributed), every rank creates. */
int zkp_comm_rccl_unique_id(uint8_t id[128]);
int zkp_comm_rccl_create(zkp_ctx* ctx, const uint8_t id[128], int world, int rank, zkp_comm** out);
/* In-process group: `world` communicators for ranks run as threads of one
 * process (each with its own zkp_ctx; GPUs may be shared). comms[world]. */
int zkp_comm_local_group(int world, zkp_comm** comms);
/* Caller transport: one process per rank, the collectives carried by the
 * caller's own channel (torch.distributed/gloo, MPI, sockets ...) through pinned
 * host staging. Each callback is a blocking collective over all ranks that
 * returns 0 on success: all_to_all sends block s of `send` (block_bytes each) to
 * rank s and receives rank s's block for this rank into block s of `recv`;
 * all_gather puts rank s's `send` (bytes) at recv + s*bytes. abort (nullable)
 * is called when this rank's proof fails, to release blocked peers. The
 * exchange points are those of the RCCL backend; RCCL stays the production
 * transport over xGMI. */
typedef struct zkp_host_transport {
  void* user;
  int (*all_to_all)(void* user, const void* send, void* recv, uint64_t block_bytes);
  int (*all_gather)(void* user, const void* send, void* recv, uint64_t bytes);
  void (*abort)(void* user);
} zkp_host_transport;
int zkp_comm_host_create(int world, int rank, const zkp_host_transport* transport, zkp_comm** out);
void zkp_comm_destroy(zkp_comm* comm);
int zkp_comm_rank(const zkp_comm* comm);
int zkp_comm_world(const zkp_comm* comm);
/* The rank count the transport itself reports: ncclCommCount for an RCCL
 * communicator (so a run can show that RCCL saw every rank), the group size for
 * the in-process and caller transports; -1 on error. */
int zkp_comm_backend_world(const zkp_comm* comm);
/* Fabric check before proving (collective; no reference counterpart): one
 * all-to-all of world blocks of block_bytes (multiple of 4) and one all-gather
 * of block_bytes per rank, each run twice on the context's stream with
 * rank-tagged words verified on the host. a2a_ms / ag_ms (nullable) receive
 * the faster round's wall time of each collective on this rank. A mismatch
 * is ZKP_ERR_DEVICE naming the peer and word. */
int zkp_comm_check(zkp_ctx* ctx, zkp_comm* comm, uint64_t block_bytes, double* a2a_ms, double* ag_ms);
/* Collective: every rank of `comm` must call it with the same arguments. */
int zkp_prove_sharded(zkp_ctx* ctx, zkp_comm* comm, zkp_air_id air, const zkp_felt* trace_cols,
                      uint32_t width, uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
                      const zkp_proof_options* opts, uint8_t** proof, uint64_t* proof_len,
                      zkp_transcript* transcript /* nullable */);

/* As zkp_prove_sharded with the full trace already in this rank's HBM. */
int zkp_prove_sharded_device(zkp_ctx* ctx, zkp_comm* comm, zkp_air_id air, const void* d_trace_cols,
                             uint32_t width, uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
                             const zkp_proof_options* opts, uint8_t** proof, uint64_t* proof_len,
                             zkp_transcript* transcript /* nullable */);

/* Device scratch helpers so callers (bench, tests) can keep traces in HBM. */
int zkp_device_alloc(zkp_ctx* ctx, uint64_t bytes, void** d_ptr);
int zkp_device_free(zkp_ctx* ctx, void* d_ptr);
int zkp_copy_to_device(zkp_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes);
int zkp_copy_to_host(zkp_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes);

/* ---- stage entry points (for a winter-prover fork / stage parity) ------ */
/* ≙ DefaultTraceLde::new (src/aggregation/prover.rs:216-224): interpolate each
 * column over <w_n>, evaluate on 3*<w_{n*blowup}>, hash rows with BLAKE3 and
 * build the Merkle tree. Outputs: LDE (column-major, natural domain order,
 * width*n*blowup felts; nullable) and root. */
int zkp_trace_lde_commit(zkp_ctx* ctx, const zkp_felt* trace_cols, uint32_t width, uint64_t n,
                         uint32_t blowup, zkp_felt* lde_out /* nullable */, uint8_t root[32]);

/* Batched BLAKE3 of rows of a column-major felt matrix (≙ RowMatrix::commit_to_rows
 * leaf hashing) followed by MerkleTree::new; returns the root. */
int zkp_merkle_commit_rows(zkp_ctx* ctx, const zkp_felt* cols, uint32_t width, uint64_t rows,
                           uint8_t root[32]);

/* Minimum-nonce grinding (sequential winterfell semantics):
 * smallest nonce >= 1 with trailing_zeros(u64_le(BLAKE3(seed || nonce_le)[0..8])) >= bits. */
int zkp_grind(zkp_ctx* ctx, const uint8_t seed[32], uint32_t bits, uint64_t* nonce);

/* ---- stage sessions: the plug-in hooks of a winter-prover fork ----------
 * A zkp_session holds one proof's device-resident state (trace polynomials and
 * LDE, composition evaluations and LDE, DEEP and FRI layers, Merkle trees), so
 * a fork of winter-prover 0.12 keeps `Prover::prove` / `generate_proof` and its
 * own channel (`DefaultRandomCoin<Blake3_256>`) and replaces only the stages:
 *   zkp_session_trace_lde  ≙ Prover::new_trace_lde -> DefaultTraceLde::new
 *                            (src/aggregation/prover.rs:216-224, src/training/prover.rs:273-281)
 *   zkp_eval_constraints   ≙ Prover::new_evaluator(..).evaluate(..)
 *                            (src/aggregation/prover.rs:226-233, src/training/prover.rs:283-290)
 *   zkp_composition_commit ≙ Prover::build_constraint_commitment
 *                            (src/aggregation/prover.rs:235-248, src/training/prover.rs:292-300)
 *   zkp_ood_frame          ≙ the OOD frame of generate_proof (trace at z, z*g; composition at z)
 *   zkp_deep_fri           ≙ DeepCompositionPoly + its LDE + FriProver::build_layers / set_remainder
 *   zkp_query              ≙ trace_lde.query, constraint_commitment.query, fri_prover.build_proof
 * (the last three are internal to winterfell 0.12's generate_proof).
 * Calls must come in that order (ZKP_ERR_ARGUMENT otherwise); zkp_query may be
 * repeated. Every value is bit-identical to the matching part of zkp_prove's proof
 * when the caller's channel draws what zkp_prove's transcript draws. One GPU. */
typedef struct zkp_session zkp_session;
int zkp_session_create(zkp_ctx* ctx, zkp_air_id air, uint32_t width, uint64_t n, const zkp_felt* pub_elems,
                       uint64_t n_pub, const zkp_proof_options* opts, zkp_session** out);
/* Releases the session's device buffers (the ctx stays usable). */
void zkp_session_destroy(zkp_session* s);
/* The session's shape as the AIR defines it (each pointer nullable): ce = the
 * constraint-evaluation blowup (zkp_eval_constraints' evals_out holds n*ce values),
 * num_columns = C composition columns, fri_layers = FRI layers before the remainder. */
int zkp_session_shape(const zkp_session* s, uint32_t* ce, uint32_t* num_columns, uint32_t* fri_layers);
/* Host trace (column-major width*n) -> interpolation, coset LDE, row commitment; root out. */
int zkp_session_trace_lde(zkp_session* s, const zkp_felt* trace_cols, uint8_t root[32]);
/* Composition coefficients as the caller's channel drew them (ConstraintCompositionCoefficients:
 * the num_transition transition coefficients, then one per assertion) -> composition
 * evaluations over the CE domain g*<w_{n*ce}> (stay in HBM for zkp_composition_commit;
 * evals_out, nullable, receives the n*ce values in natural domain order). */
int zkp_eval_constraints(zkp_session* s, const zkp_felt* coeffs, uint32_t n_coeffs, zkp_felt* evals_out);
/* CompositionPoly::new (segments into C columns of n coefficients) + LDE + row commitment.
 * evals = NULL: the session's zkp_eval_constraints output; otherwise n*ce host values in
 * natural CE-domain order (e.g. from a CPU evaluator). num_columns (nullable) = C. */
int zkp_composition_commit(zkp_session* s, const zkp_felt* evals, uint8_t root[32], uint32_t* num_columns);
/* OOD frame at z: trace_ood[0..w) = T(z), trace_ood[w..2w) = T(z*w_n); comp_ood[0..C) = H_j(z). */
int zkp_ood_frame(zkp_session* s, zkp_felt z, zkp_felt* trace_ood, zkp_felt* comp_ood);
/* Called once per FRI layer with its Merkle root; returns that layer's alpha in *alpha
 * (a fork binds it to `channel.commit_fri_layer(root); channel.draw_fri_alpha()`); non-zero aborts. */
typedef int (*zkp_fri_channel)(void* user, uint32_t layer, const uint8_t root[32], zkp_felt* alpha);
/* DEEP composition with the caller's coefficients (width + C), then the FRI layers (fold 16)
 * and the remainder polynomial: remainder (nullable; capacity *remainder_len) receives its
 * coefficients, *remainder_len their count, remainder_commitment = hash_elements(remainder). */
int zkp_deep_fri(zkp_session* s, const zkp_felt* deep_coeffs, zkp_fri_channel channel, void* user,
                 zkp_felt* remainder, uint64_t* remainder_len, uint8_t remainder_commitment[32]);
/* Openings at sorted, unique LDE positions (< n*blowup): returns, in zkp_prove's wire
 * format, u8(1) | trace values | trace batch paths | constraint values | constraint batch
 * paths | u8(L) | per FRI layer: values | batch paths. Free with zkp_free. */
int zkp_query(zkp_session* s, const uint64_t* positions, uint64_t n_positions, uint8_t** out, uint64_t* out_len);

/* ---- host channel for stage sessions -------------------------------------
 * ≙ winter-prover 0.12 ProverChannel over DefaultRandomCoin<Blake3_256>, seeded as
 * generate_proof seeds it (Context::to_elements() || pub_inputs.to_elements(), the
 * same seed as zkp_prove's transcript). A winter-prover fork keeps its own channel;
 * a C or Python caller of the session stages draws from this one. Host-only. */
typedef struct zkp_channel zkp_channel;
int zkp_channel_create(zkp_air_id air, uint32_t width, uint64_t n, const zkp_felt* pub_elems, uint64_t n_pub,
                       const zkp_proof_options* opts, zkp_channel** out);
void zkp_channel_destroy(zkp_channel* ch);
/* reseed(root): a commitment (trace, constraint, FRI layer, remainder) */
int zkp_channel_commit(zkp_channel* ch, const uint8_t root[32]);
/* reseed(hash_elements(els)): the OOD frame, trace part (T(z) || T(z*g)) then composition part */
int zkp_channel_commit_felts(zkp_channel* ch, const zkp_felt* els, uint64_t n);
/* count coefficients drawn with `method` (ZKP_BATCHING_*: ConstraintCompositionCoefficients,
 * DeepCompositionCoefficients), or with count = 0 one element (the OOD point z, a FRI alpha) */
int zkp_channel_draw(zkp_channel* ch, uint32_t method, uint32_t count, zkp_felt* out);
/* the coin's seed (the grinding seed for zkp_grind after the remainder commitment) */
int zkp_channel_seed(const zkp_channel* ch, uint8_t seed[32]);
/* query positions: draw_integers(num_queries, n*blowup, nonce), sorted and deduplicated;
 * out holds num_queries values, *n_unique receives the count kept */
int zkp_channel_query_positions(zkp_channel* ch, uint64_t nonce, uint64_t* out, uint32_t* n_unique);

/* ---- verification (≙ winterfell `verify`) ------------------------------ */
/* Status codes of zkp_verify; values map onto winter-verifier `VerifierError`. */
typedef enum zkp_verify_status {
  ZKP_VERIFY_OK = 0,
  ZKP_VERIFY_INCONSISTENT_BASE_FIELD = 32,  /* InconsistentBaseField */
  ZKP_VERIFY_UNACCEPTABLE_OPTIONS = 33,     /* UnacceptableProofOptions */
  ZKP_VERIFY_DESERIALIZATION = 34,          /* ProofDeserializationError */
  ZKP_VERIFY_PUB_INPUTS = 35,               /* public inputs rejected by Air::new */
  ZKP_VERIFY_INCONSISTENT_OOD = 36,         /* InconsistentOodConstraintEvaluations */
  ZKP_VERIFY_TRACE_QUERY = 37,              /* TraceQueryDoesNotMatchCommitment */
  ZKP_VERIFY_CONSTRAINT_QUERY = 38,         /* ConstraintQueryDoesNotMatchCommitment */
  ZKP_VERIFY_POW = 39,                      /* QuerySeedProofOfWorkVerificationFailed */
  ZKP_VERIFY_FRI = 40,                      /* FriVerificationFailed */
  ZKP_VERIFY_RANDOM_COIN = 41               /* RandomCoinError */
} zkp_verify_status;

/* Checks a proof produced by zkp_prove / zkp_prove_sharded against the public
 * inputs (`pub_inputs.to_elements()`) and the one acceptable option set.
 * Replaces `verify::<AIR, Blake3_256<Felt>, DefaultRandomCoin<..>, MerkleTree<..>>(
 * proof, pub_inputs, &AcceptableOptions::OptionSet(vec![options]))` at
 * src/main.rs:251-257, 430-436, 478-484. Host-only: needs no device and no ctx.
 * Returns ZKP_VERIFY_OK, a zkp_verify_status or ZKP_ERR_ARGUMENT. */
int zkp_verify(zkp_air_id air, const uint8_t* proof, uint64_t proof_len, const zkp_felt* pub_elems,
               uint64_t n_pub, const zkp_proof_options* acceptable);

/* ---- trace construction helper ---------------------------------------- */
/* Host-side MiMC AIR trace: out[0] = seed mod p,
 * out[i+1] = (out[i] + K[i % 64])^7 with K[j] = (j+1)*10^6
 * (get_round_constants, src/helper.rs:404-406). Trace building, like
 * `TraceTable` construction in the reference — not part of the proving path. */
int zkp_build_mimc_trace(const uint8_t seed[16], uint64_t n, zkp_felt* out);

/* GlobalUpdateProver::build_trace on the device (src/aggregation/prover.rs:98-160;
 * SURVEY.md §8(f) row 4): writes the 120 x n column-major trace into HBM at
 * d_trace_out (ready for zkp_prove_device). raw_global = flattened raw global
 * model (54 weights then 6 biases), blinding = the 60 masks (prover.rs:68-72),
 * local_updates = ndev x 60 flattened local models (row-major), k = the
 * aggregation factor (pub element 120). Rows: 0 = [masked | 0], 1..ndev =
 * [masked + k^-1 * prefix sum of (local_i - raw) | local_{r-1} - raw],
 * ndev+1.. = [final | 0]. n must be a power of two >= max(8, ndev + 2).
 * final_state (nullable, 60 felts) receives row ndev + 1's masked state, the
 * `new_global` of GlobalUpdateProver::get_pub_inputs (prover.rs:163-190). */
int zkp_build_global_update_trace(zkp_ctx* ctx, const zkp_felt* raw_global, const zkp_felt* blinding,
                                  const zkp_felt* local_updates, uint64_t ndev, zkp_felt k, uint64_t n,
                                  void* d_trace_out, zkp_felt* final_state /* nullable */);

/* ---- profiling ------------------------------------------------------- */
/* When enabled, every kernel launch is bracketed with HIP events on the
 * stream it runs on; zkp_kernel_stats reports per-kernel launch count and
 * total device milliseconds since the last reset. */
int zkp_set_profiling(zkp_ctx* ctx, int enabled);
/* Restrict the bracketing to launches named `kernel_name` (as in the stats
 * table, e.g. "ntt_dit"); NULL = every launch. Fewer events in a timed region. */
int zkp_set_profiling_kernel(zkp_ctx* ctx, const char* kernel_name /* nullable */);
int zkp_kernel_stats(zkp_ctx* ctx, const char* kernel_name, uint64_t* launches, double* total_ms);
int zkp_reset_stats(zkp_ctx* ctx);
/* Returns a newline-separated "name launches total_ms algorithmic_bytes" table (free with zkp_free). */
int zkp_kernel_stats_table(zkp_ctx* ctx, char** table);

#ifdef __cplusplus
}
#endif
#endif /* ZKP_H */
