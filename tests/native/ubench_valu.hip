// VALU issue-rate microbenchmark on gfx950 (TUNING ONLY, not product code).
// Each thread runs 8 independent chains of one instruction (asm-pinned) for
// ITERS iterations; the rate is reported in lane-ops/s and as SIMD cycles per
// wave64 instruction (1024 SIMDs at the clock given on the command line).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 4096

#define CHAIN8(STMT) \
  STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_mad_u64(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t a[8];
  for (int k = 0; k < 8; k++) a[k] = io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a[k]) : "v"((uint32_t)a[k]), "v"(m) : "s0", "s1");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mul_lo(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(m));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mul_hi(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(m));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_add_u32(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(m));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

// add with carry-out into an SGPR pair, consumed by the next chain's addc (carry hazard)
__global__ void k_addc_chain(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_co_u32_e64 %0, s[4:5], %0, %8\n\t"
        "v_addc_co_u32_e64 %1, s[4:5], %1, %8, s[4:5]\n\t"
        "v_addc_co_u32_e64 %2, s[4:5], %2, %8, s[4:5]\n\t"
        "v_addc_co_u32_e64 %3, s[4:5], %3, %8, s[4:5]\n\t"
        "v_add_co_u32_e64 %4, s[6:7], %4, %8\n\t"
        "v_addc_co_u32_e64 %5, s[6:7], %5, %8, s[6:7]\n\t"
        "v_addc_co_u32_e64 %6, s[6:7], %6, %8, s[6:7]\n\t"
        "v_addc_co_u32_e64 %7, s[6:7], %7, %8, s[6:7]"
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
        : "v"(m)
        : "s4", "s5", "s6", "s7");
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

// the same two chains interleaved (each carry consumed 2 instructions later)
__global__ void k_addc_inter(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_co_u32_e64 %0, s[4:5], %0, %8\n\t"
        "v_add_co_u32_e64 %4, s[6:7], %4, %8\n\t"
        "v_addc_co_u32_e64 %1, s[4:5], %1, %8, s[4:5]\n\t"
        "v_addc_co_u32_e64 %5, s[6:7], %5, %8, s[6:7]\n\t"
        "v_addc_co_u32_e64 %2, s[4:5], %2, %8, s[4:5]\n\t"
        "v_addc_co_u32_e64 %6, s[6:7], %6, %8, s[6:7]\n\t"
        "v_addc_co_u32_e64 %3, s[4:5], %3, %8, s[4:5]\n\t"
        "v_addc_co_u32_e64 %7, s[6:7], %7, %8, s[6:7]"
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
        : "v"(m)
        : "s4", "s5", "s6", "s7");
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

// add with carry-out written to VCC (the VOP2 encoding) — no SGPR-pair hazard?
__global__ void k_addc_vcc(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_add_co_u32 %0, vcc, %0, %8\n\t"
        "v_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\t"
        "v_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
        "v_add_co_u32 %4, vcc, %4, %8\n\t"
        "v_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
        "v_addc_co_u32 %6, vcc, %6, %8, vcc\n\t"
        "v_addc_co_u32 %7, vcc, %7, %8, vcc"
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
        : "v"(m)
        : "vcc");
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_fma_f64(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  double a[8];
  for (int k = 0; k < 8; k++) a[k] = (double)(io[8 * t + k] & 0xffff);
  double m = 1.0000001 + (double)(t & 7) * 1e-9, c = 1e-3;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(m), "v"(c));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = (uint64_t)a[k];
}

__global__ void k_lshl_add(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[k]) : "v"(m) : "s8", "s9");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_lshlrev_b64(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t a[8];
  for (int k = 0; k < 8; k++) a[k] = io[8 * t + k];
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(a[k]));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}


__global__ void k_xor(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_add3(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_alignbit(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_perm(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_lshl_or(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_xad(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mov(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mov_b32 %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_sub(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mul_u24(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mad_u24(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_add_co_vcc(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_alignbit_e(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_alignbit_b32 %0, %1, %0, 16" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_lshrrev(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_or3(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_or3_b32 %0, %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_and_or(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_and_or_b32 %0, %0, %1, %0" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_add_e64(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_cndmask_vcc(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mul_hi_u24(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_pk_add_u16(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_bfe(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_bfe_u32 %0, %0, 3, 17" : "+v"(a[k]) : "v"(m) : "vcc");
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_mix(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t a[4]; uint32_t b[4];
  for (int k = 0; k < 4; k++) { a[k] = io[8 * t + k]; b[k] = (uint32_t)io[8*t+4+k]; }
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a[k]) : "v"((uint32_t)a[k]), "v"(m) : "s0", "s1"); \
             asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[k]) : "v"(m));
    S(0) S(1) S(2) S(3)
#undef S
  }
  for (int k = 0; k < 4; k++) { io[8 * t + k] = a[k]; io[8*t+4+k] = b[k]; }
}

// rotr16(a ^ m) as two SDWA xors (word selects) vs xor + alignbit
__global__ void k_xor_sdwa(uint64_t* io) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a[k]) : "v"(m));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_rot16_sdwa(uint64_t* io) {  // per op = one xor + rotr16 pair
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) { uint32_t r; asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "=&v"(r) : "v"(a[k]), "v"(m)); a[k] = r; }
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

__global__ void k_rot16_align(uint64_t* io) {  // per op = one xor + rotr16 pair
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t a[8];
  for (int k = 0; k < 8; k++) a[k] = (uint32_t)io[8 * t + k];
  uint32_t m = (uint32_t)t | 1;
  for (int i = 0; i < ITERS; i++) {
#define S(k) asm volatile("v_xor_b32 %0, %0, %1\n v_alignbit_b32 %0, %0, %0, 16" : "+v"(a[k]) : "v"(m));
    CHAIN8(S)
#undef S
  }
  for (int k = 0; k < 8; k++) io[8 * t + k] = a[k];
}

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
  const int blocks = 256 * 32, tpb = 256;
  const size_t nthr = (size_t)blocks * tpb;
  uint64_t* d;
  if (hipMalloc(&d, nthr * 8 * sizeof(uint64_t)) != hipSuccess) return 1;
  hipMemset(d, 1, nthr * 8 * sizeof(uint64_t));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, void (*k)(uint64_t*)) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(tpb), 0, 0, d);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(tpb), 0, 0, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double lane_ops = 3.0 * nthr * (double)ITERS * 8;
    double rate = lane_ops / (ms * 1e-3);
    double wave_insts_per_simd_cycle = rate / 64 / (1024 * ghz * 1e9);
    printf("%-22s %8.3f ms  %8.1f G lane-op/s  %6.2f SIMD cycles / wave64 inst\n", name, ms, rate / 1e9,
           1.0 / wave_insts_per_simd_cycle);
  };
  run("v_add_u32", k_add_u32);
  run("v_cndmask_b32", k_lshl_add);
  run("v_lshrrev_b64", k_lshlrev_b64);
  run("v_mad_u64_u32", k_mad_u64);
  run("v_mul_lo_u32", k_mul_lo);
  run("v_mul_hi_u32", k_mul_hi);
  run("add_co/addc chains", k_addc_chain);
  run("add_co/addc interleave", k_addc_inter);
  run("add_co/addc vcc", k_addc_vcc);
  run("v_fma_f64", k_fma_f64);
  run("xor", k_xor);
  run("add3", k_add3);
  run("alignbit", k_alignbit);
  run("perm", k_perm);
  run("lshl_or", k_lshl_or);
  run("xad", k_xad);
  run("mov", k_mov);
  run("sub", k_sub);
  run("mul_u24", k_mul_u24);
  run("mad_u24", k_mad_u24);
  run("add_co_vcc", k_add_co_vcc);
  run("alignbit_e", k_alignbit_e);
  run("lshrrev", k_lshrrev);
  run("or3", k_or3);
  run("and_or", k_and_or);
  run("add_e64", k_add_e64);
  run("cndmask_vcc", k_cndmask_vcc);
  run("mul_hi_u24", k_mul_hi_u24);
  run("pk_add_u16", k_pk_add_u16);
  run("bfe", k_bfe);
  run("mix mad+add (per op)", k_mix);
  run("xor_sdwa", k_xor_sdwa);
  run("xor+rot16 sdwa (pair)", k_rot16_sdwa);
  run("xor+rot16 align (pair)", k_rot16_align);
  return 0;
}
