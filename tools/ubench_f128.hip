// Micro-benchmark: issue rate of the Field128 building blocks on gfx950 at 1-8 waves/SIMD.
// Reports VALU lane-instructions/s (static VALU count per iteration x lanes / time) and
// operations/s.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_f128 tools/ubench_f128.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../janus_amd/csrc/prio3_device.h"
#define ITER 256

__global__ void k_mac(uint32_t* out, uint32_t s) {
  f128 x = mk128(s ^ threadIdx.x, s * 3, s * 5, s * 7), y = mk128(s * 11, s ^ 13, s * 17, s + 19);
  mac128 a;
  mac_zero(a);
  for (int it = 0; it < ITER; it++) {
    mac_add(a, x, y);
    x.w[0] ^= it;
  }
  f128 z = mac_reduce_f(a);
  out[blockIdx.x * blockDim.x + threadIdx.x] = z.w[0] ^ z.w[1] ^ z.w[2] ^ z.w[3];
}
__global__ void k_mac2(uint32_t* out, uint32_t s) {  // two independent accumulators
  f128 x = mk128(s ^ threadIdx.x, s * 3, s * 5, s * 7), y = mk128(s * 11, s ^ 13, s * 17, s + 19);
  mac128 a, b;
  mac_zero(a);
  mac_zero(b);
  for (int it = 0; it < ITER / 2; it++) {
    mac_add(a, x, y);
    mac_add(b, y, x);
    x.w[0] ^= it;
  }
  f128 z = mac_reduce_f(a), w = mac_reduce_f(b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = z.w[0] ^ z.w[1] ^ w.w[2] ^ w.w[3];
}
__global__ void k_mulc(uint32_t* out, uint32_t s) {
  f128 x = mk128(s ^ threadIdx.x, s * 3, s * 5, 7), y = mk128(s * 11, s ^ 13, s * 17, 19);
  for (int it = 0; it < ITER / 4; it++) x = mul128(x, y);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x.w[0] ^ x.w[1] ^ x.w[2] ^ x.w[3];
}
__global__ void k_mula(uint32_t* out, uint32_t s) {
  f128 x = mk128(s ^ threadIdx.x, s * 3, s * 5, 7), y = mk128(s * 11, s ^ 13, s * 17, 19);
  for (int it = 0; it < ITER / 4; it++) x = mul128_asm(x, y);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x.w[0] ^ x.w[1] ^ x.w[2] ^ x.w[3];
}
__global__ void k_mula2(uint32_t* out, uint32_t s) {  // two independent chains
  f128 x = mk128(s ^ threadIdx.x, s * 3, s * 5, 7), y = mk128(s * 11, s ^ 13, s * 17, 19);
  f128 z = y;
  for (int it = 0; it < ITER / 8; it++) {
    x = mul128_asm(x, y);
    z = mul128_asm(z, x);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x.w[0] ^ x.w[1] ^ z.w[2] ^ z.w[3];
}
__global__ void k_redasm(uint32_t* out, uint32_t s) {
  mac128 a;
  for (int k = 0; k < 7; k++) {
    a.c[k] = ((uint64_t)(s * (k + 3)) << 32) | (threadIdx.x + k);
    a.h[k] = s ^ k;
  }
  uint32_t acc = 0;
  for (int it = 0; it < ITER / 4; it++) {
    f128 z = mac_reduce_f(a);
    acc ^= z.w[0];
    a.c[0] += z.w[1];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Keccak-p[1600,12]: PERMS permutations per work-item, no memory traffic
#define PERMS 16
__global__ __launch_bounds__(256) void k_keccak(uint32_t* out, uint32_t s) {
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
__global__ __launch_bounds__(256) void k_keccak2(uint32_t* out, uint32_t s) {  // 2 states / lane
  KState a, b;
  for (int i = 0; i < 25; i++) {
    a.lo[i] = s * (i + 1) ^ threadIdx.x;
    a.hi[i] = s + i;
    b.lo[i] = s * (i + 3) ^ threadIdx.x;
    b.hi[i] = s + 2 * i;
  }
  for (int it = 0; it < PERMS / 2; it++) {
    keccak_p12(a);
    keccak_p12(b);
  }
  uint32_t acc = 0;
  for (int i = 0; i < 25; i++) acc ^= a.lo[i] ^ a.hi[i] ^ b.lo[i] ^ b.hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
void run(const char* name, K kern, uint32_t* buf, int w, double ops_per_thread, double valu_per_op) {
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
  double ops = 5.0 * blocks * threads * ops_per_thread;
  printf("%-22s waves/SIMD=%d  %8.3f ms  %8.2f G ops/s  %6.2f T lane-instr/s\n", name, w, ms,
         ops / (ms * 1e-3) / 1e9, ops * valu_per_op / (ms * 1e-3) / 1e12);
}
int main() {
  uint32_t* buf;
  (void)hipMalloc(&buf, (size_t)256 * 256 * 8 * 4);
  for (int w : {1, 2, 3, 4, 8}) {
    run("mac_add (1 acc)", k_mac, buf, w, ITER, 32);
    run("mac_add (2 acc)", k_mac2, buf, w, ITER, 32);
    run("mul128 (compiler)", k_mulc, buf, w, ITER / 4, 110);
    run("mul128_asm", k_mula, buf, w, ITER / 4, 80);
    run("mul128_asm (2 chains)", k_mula2, buf, w, ITER / 4, 80);
    run("mac_reduce_f", k_redasm, buf, w, ITER / 4, 70);
    run("keccak_p12", k_keccak, buf, w, PERMS, 12 * 190);
    run("keccak_p12 (2 states)", k_keccak2, buf, w, PERMS, 12 * 190);
  }
  return 0;
}
