// TEST INFRASTRUCTURE: exposes the product's felt.hpp / blake3.hpp host
// instantiations (the same source the gfx950 kernels compile) through a C ABI
// so CPU tests can check them against tests/golden vectors.
#include "../../zk_stark_project_amd/csrc/felt.hpp"
#include "../../zk_stark_project_amd/csrc/blake3.hpp"

extern "C" {
void hc_f128(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  felt x = fp::from_u128_bytes(a), y = fp::from_u128_bytes(b), r;
  switch (op) {
    case 0: r = fp::add(x, y); break;
    case 1: r = fp::sub(x, y); break;
    case 2: r = fp::mul(x, y); break;
    case 3: r = fp::inv(x); break;
    default: r = fp::pow_u64(x, y.lo); break;
  }
  fp::to_bytes(r, out);
}
void hc_blake3(const uint8_t* d, uint64_t n, uint8_t* out) { b3::host_hash(d, n, out); }
// device-style hash_felts over a felt array (4 felts / block, chunk tree)
void hc_hash_felts(const uint8_t* felts, uint32_t nf, uint8_t* out) {
  uint32_t d[8];
  b3::hash_felts([&](uint32_t k) { return fp::from_u128_bytes(felts + 16 * k); }, nf, d);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(d[i] >> (8 * k));
}
}
