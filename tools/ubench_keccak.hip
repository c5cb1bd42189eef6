// Micro-benchmark: Keccak-p[1600,12] issue rate on gfx950 for round-scheduling variants at
// 1-8 waves/SIMD (no memory traffic): one state per lane; two states per lane permuted one
// after the other; two states with their rounds interleaved (one round of each per step).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../janus_amd/csrc/prio3_device.h"

DEV void keccak_p12x2(KState& a, KState& b) {
#pragma unroll 1
  for (int r = 0; r < 12; r++) {
    keccak_round(a, KRC_LO[r], KRC_HI[r]);
    keccak_round(b, KRC_LO[r], KRC_HI[r]);
  }
}

#define PERMS 16


template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_one(uint32_t* out, uint32_t s) {
  KState st;
  for (int i = 0; i < 25; i++) {
    st.lo[i] = s * (i + 1) ^ threadIdx.x;
    st.hi[i] = s + i;
  }
  for (int it = 0; it < PERMS; it++) keccak_p12(st);
  uint32_t acc = 0;
  for (int i = 0; i < 25; i++) acc ^= st.lo[i] ^ st.hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int OCC, int IL>
__global__ __launch_bounds__(256, OCC) void k_two(uint32_t* out, uint32_t s) {
  KState a, b;
  for (int i = 0; i < 25; i++) {
    a.lo[i] = s * (i + 1) ^ threadIdx.x;
    a.hi[i] = s + i;
    b.lo[i] = s * (i + 3) ^ threadIdx.x;
    b.hi[i] = s + 2 * i;
  }
  for (int it = 0; it < PERMS / 2; it++) {
    if (IL) {
      keccak_p12x2(a, b);
    } else {
      keccak_p12(a);
      keccak_p12(b);
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 25; i++) acc ^= a.lo[i] ^ a.hi[i] ^ b.lo[i] ^ b.hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
void run(const char* name, K kern, uint32_t* buf, int w) {
  int threads = 256, blocks = 256 * w;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<blocks, threads>>>(buf, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) kern<<<blocks, threads>>>(buf, r + 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double ops = 5.0 * blocks * threads * PERMS;
  printf("%-28s waves/SIMD=%d  %8.3f ms  %8.2f G perm/s  %6.2f T lane-instr/s\n", name, w, ms,
         ops / (ms * 1e-3) / 1e9, ops * 12 * 180 / (ms * 1e-3) / 1e12);
}
int main() {
  uint32_t* buf;
  (void)hipMalloc(&buf, (size_t)256 * 256 * 8 * 4);
  for (int w : {1, 2, 3, 4, 8}) {
    run("one state", k_one<1>, buf, w);
    run("two states, sequential", k_two<1, 0>, buf, w);
    run("two states, interleaved", k_two<1, 1>, buf, w);
  }
  run("one state (bounds 3)", k_one<3>, buf, 3);
  run("two interleaved (bounds 3)", k_two<3, 1>, buf, 3);
  run("two interleaved (bounds 2)", k_two<2, 1>, buf, 2);
  return 0;
}
