// kbench_top.cpp — latency of the Merkle tree tops (merkle_upper over L subtree
// roots already in nodes[L..2L)) and of the tail ops the last block runs
// (TEST/BENCH ONLY). Links csrc/merkle.hip directly.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../zk_stark_project_amd/csrc/zkp_internal.hpp"
#include "../../zk_stark_project_amd/csrc/host_stark.hpp"

hipEvent_t Prof::get_event() { return nullptr; }
void Prof::begin(const char*, hipStream_t, double) {}
void Prof::end(hipStream_t) {}
void launch_fail(int code, const char* what) { throw std::runtime_error(std::string(what) + " " + std::to_string(code)); }

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Prof pf;
  const uint64_t Lmax = 1ull << 16;
  uint32_t *nodes, *done, *seed, *root_out;
  felt *alpha, *out, *pw;
  CK(hipMalloc(&nodes, 2 * Lmax * 32));
  CK(hipMalloc(&done, 4));
  CK(hipMalloc(&seed, 32));
  CK(hipMalloc(&root_out, 32));
  CK(hipMalloc(&alpha, 16 * 64));
  CK(hipMalloc(&out, 16 * 64));
  CK(hipMalloc(&pw, 16 * 64));
  CK(hipMemset(done, 0, 4));
  CK(hipMemset(seed, 0x5a, 32));
  std::vector<uint32_t> h(2 * Lmax * 8);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(nodes, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* opn[] = {"none", "fri_coin", "draw_coeffs", "draw_z"};
  for (uint64_t L : {512ull, 1ull << 12, 1ull << 14, 1ull << 16}) {
    for (int op = 0; op < 4; op++) {
      MerkleTail t{};
      t.done = done;
      t.coin_seed = seed;
      t.alpha_out = alpha;
      t.root_out = root_out;
      t.op = op;
      t.method = 0;
      t.ncoef = 3;
      t.logn = 20;
      t.wn = zkh::root_of_unity(20);
      t.out = out;
      t.pw = pw;
      for (int i = 0; i < 5; i++) merkle_upper(pf, st, nodes, L, &t);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; i++) merkle_upper(pf, st, nodes, L, &t);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("L=2^%-2d tail=%-12s %8.2f us per tree top\n", __builtin_ctzll(L), opn[op], ms * 1e3 / reps);
    }
  }
  // FRI layer commitments (leaf hashing of 16-felt rows + the tree + the coin step) by
  // the rows' size and the quad-leaf threshold
  extern uint32_t fri_quad_max_log;
  felt* E;
  const uint64_t Rmax = 1ull << 16;
  CK(hipMalloc(&E, Rmax * 16 * 16));
  CK(hipMemset(E, 0x11, Rmax * 16 * 16));
  for (uint32_t logR : {11u, 13u, 15u}) {
    for (uint32_t qmax : {12u, 13u, 15u}) {
      fri_quad_max_log = qmax;
      MerkleTail t{};
      t.done = done;
      t.coin_seed = seed;
      t.alpha_out = alpha;
      t.root_out = root_out;
      t.op = MERKLE_TAIL_FRI_COIN;
      const uint64_t m16 = (1ull << logR) >> 3;  // B = 8 cosets
      for (int i = 0; i < 5; i++) launch_merkle_fri(pf, st, E, m16, 3, 16, nodes, &t);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; i++) launch_merkle_fri(pf, st, E, m16, 3, 16, nodes, &t);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("FRI layer 2^%-2u rows quad_max=2^%-2u %8.2f us per commitment\n", logR, qmax, ms * 1e3 / reps);
    }
  }
  return 0;
}
