# NTT timing-harness variants (tuning only): build with the flags below and run
# on the GPU box, e.g.
#   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DZKP_EXP_NOBFLY -o tests/native/kbench_ntt_v_NOBFLY \
#         tests/native/kbench_ntt.cpp zk_stark_project_amd/csrc/ntt.hip
# flags: ZKP_EXP_NOGMEM (no HBM traffic), ZKP_EXP_NOBFLY (no butterflies), ZKP_EXP_NOSCALE (no coset-scale reads),
#        ZKP_NTT_POSFAST (position-fastest grid), ZKP_NTT_KMAX=10 (2-pass 2^20)
set -e
for b in tests/native/kbench_ntt_v*; do echo "== $b"; timeout -k 10 60 $b; done
