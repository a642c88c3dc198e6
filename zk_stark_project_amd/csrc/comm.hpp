// comm.hpp — the exchange steps of the coset-sharded prover.
//
// A proof is sharded over `world` ranks by LDE coset: rank r owns the cosets
// [r*B/world, (r+1)*B/world) of every LDE-domain array. The prover needs only
// two collectives, both on equal-sized blocks of device memory, ordered on
// the prover's HIP stream:
//   all_to_all — leaf digests to the rank owning their Merkle range, and the
//                composition evaluations to the rank owning a coefficient slice;
//   all_gather — subtree roots, composition coefficient slices, small FRI
//                layers and query openings.
// Backends: self (world 1), an in-process group (ranks = threads, e.g. several
// ranks sharing one GPU in tests), and RCCL over xGMI (one process per GPU).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/zkp.h"
#include <stddef.h>

#include <stdexcept>
#include <string>

struct zkp_comm {
  int rank = 0, world = 1;
  virtual ~zkp_comm() = default;
  virtual const char* kind() const = 0;
  // block s of `send` goes to rank s; block s of `recv` comes from rank s
  virtual void all_to_all(hipStream_t st, const void* send, void* recv, size_t block_bytes) = 0;
  // recv[s * bytes ..] = `send` of rank s
  virtual void all_gather(hipStream_t st, const void* send, void* recv, size_t bytes) = 0;
  // called when this rank's proof fails, so that peers blocked in a collective return
  virtual void abort() {}
  // the rank count the transport itself reports (RCCL: ncclCommCount), or -1 on error
  virtual int backend_world() const { return world; }
};

struct CommError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

zkp_comm* make_self_comm();
// caller transport through pinned host staging (include/zkp.h zkp_host_transport)
zkp_comm* make_host_comm(int world, int rank, const zkp_host_transport& t);
// `world` communicators of one in-process group (out[0..world))
void make_local_group(int world, zkp_comm** out);
// RCCL; `id` = NCCL_UNIQUE_ID_BYTES from rccl_unique_id on one rank
void rccl_unique_id(unsigned char id[128]);
zkp_comm* make_rccl_comm(int device, const unsigned char id[128], int world, int rank);
