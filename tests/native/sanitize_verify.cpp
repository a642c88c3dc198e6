// Host ASan/UBSan driver (TEST ONLY): runs the product verifier (zkp_verify,
// csrc/verifier.cpp) and the oracle verifier (oracle_verify) on proofs read
// from files and on a deterministic mutation set of each (bit flips across the
// whole proof, truncations, appended bytes, random garbage). Both parse
// untrusted bytes; any out-of-bounds read or UB aborts the run (built with
// -fsanitize=address,undefined -fno-sanitize-recover=all).
// Usage: sanitize_verify <case_dir>...  (case_dir holds proof.bin, pub.bin, meta.txt)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "../../include/zkp.h"

extern "C" int oracle_verify(int air_id, const uint8_t* proof, uint64_t len, const uint8_t* pub_bytes, uint64_t npub,
                             const zkp_proof_options* o);

static std::vector<uint8_t> slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char** argv) {
  uint64_t rng = 0x9e3779b97f4a7c15ull;
  auto next = [&] { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; };
  long total = 0, rejected_both = 0, disagree = 0;
  for (int a = 1; a < argc; a++) {
    std::string d = argv[a];
    std::vector<uint8_t> proof = slurp(d + "/proof.bin"), pub = slurp(d + "/pub.bin");
    zkp_proof_options o{};
    int air = 0;
    FILE* m = fopen((d + "/meta.txt").c_str(), "r");
    if (!m || fscanf(m, "%d %u %u %u %u %u %u %u %u", &air, &o.num_queries, &o.blowup_factor, &o.grinding_factor,
                     &o.field_extension, &o.fri_folding_factor, &o.fri_remainder_max_degree,
                     &o.batching_constraints, &o.batching_deep) != 9) {
      fprintf(stderr, "bad meta in %s\n", d.c_str());
      return 2;
    }
    fclose(m);
    const uint64_t npub = pub.size() / 16;
    auto check = [&](const std::vector<uint8_t>& p) {
      // copy into an exactly-sized heap block so ASan sees reads past the end
      uint8_t* buf = (uint8_t*)malloc(p.size() ? p.size() : 1);
      if (!p.empty()) memcpy(buf, p.data(), p.size());
      int r1 = zkp_verify((zkp_air_id)air, buf, p.size(), (const zkp_felt*)pub.data(), npub, &o);
      int r2 = oracle_verify(air, buf, p.size(), pub.data(), npub, &o);
      free(buf);
      total++;
      if (r1 != 0 && r2 != 0) rejected_both++;
      if ((r1 == 0) != (r2 == 0)) disagree++;
      return r1;
    };
    if (check(proof) != 0) {
      fprintf(stderr, "%s: valid proof rejected\n", d.c_str());
      return 3;
    }
    for (size_t i = 0; i < proof.size(); i += 1 + proof.size() / 1500) {  // bit flips over the whole proof
      std::vector<uint8_t> p = proof;
      p[i] ^= (uint8_t)(1u << (next() % 8));
      check(p);
    }
    for (size_t len = 0; len < proof.size(); len += 1 + proof.size() / 300) {  // truncations
      std::vector<uint8_t> p(proof.begin(), proof.begin() + len);
      check(p);
    }
    for (int k = 1; k <= 64; k *= 2) {  // trailing bytes
      std::vector<uint8_t> p = proof;
      p.resize(p.size() + k, 0xa5);
      check(p);
    }
    for (int k = 0; k < 200; k++) {  // garbage of random lengths, and garbage after a valid prefix
      std::vector<uint8_t> p(next() % (proof.size() + 64));
      size_t keep = k % 2 ? (size_t)(next() % proof.size()) : 0;
      for (size_t i = 0; i < p.size(); i++) p[i] = i < keep ? proof[i] : (uint8_t)next();
      check(p);
    }
    for (int k = 0; k < 200; k++) {  // length fields blown up: random 4-byte windows set to 0xff
      std::vector<uint8_t> p = proof;
      size_t i = next() % (proof.size() - 4);
      for (int b = 0; b < 4; b++) p[i + b] = 0xff;
      check(p);
    }
  }
  printf("checked %ld proofs: rejected by both %ld, verifiers disagree %ld\n", total, rejected_both, disagree);
  return disagree ? 4 : 0;
}
