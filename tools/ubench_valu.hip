// Micro-benchmark: issue rate and dependent latency of the VALU instructions the engine is
// built from on gfx950.  Each kernel runs ITER iterations of CH independent chains (CH=1:
// fully dependent chain -> latency-bound); reports lane-instructions/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 2048

#define KERN(NAME, CH, ASM, CONS, ...)                                          \
  __global__ void NAME(uint32_t* out, uint32_t a0) {                             \
    uint32_t x[CH * 2];                                                          \
    for (int i = 0; i < CH * 2; i++) x[i] = a0 + i + threadIdx.x;               \
    uint32_t b = a0 * 3, c = a0 * 7;                                             \
    for (int it = 0; it < ITER; it++) {                                          \
      _Pragma("unroll") for (int i = 0; i < CH; i++) {                           \
        uint64_t& v = *reinterpret_cast<uint64_t*>(&x[2 * i]);                   \
        (void)v;                                                                 \
        asm volatile(ASM : CONS : "v"(b), "v"(c) __VA_ARGS__);                          \
      }                                                                          \
    }                                                                            \
    uint32_t s = 0;                                                              \
    for (int i = 0; i < CH * 2; i++) s ^= x[i];                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                              \
  }

KERN(k_bitop3_8, 8, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "+v"(x[2 * i]), )
KERN(k_bitop3_1, 1, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "+v"(x[2 * i]), )
KERN(k_xor_8, 8, "v_xor_b32 %0, %0, %1", "+v"(x[2 * i]), )
KERN(k_add_8, 8, "v_add_u32 %0, %0, %1", "+v"(x[2 * i]), )
KERN(k_alignbit_8, 8, "v_alignbit_b32 %0, %0, %1, 7", "+v"(x[2 * i]), )
KERN(k_alignbit_1, 1, "v_alignbit_b32 %0, %0, %1, 7", "+v"(x[2 * i]), )
KERN(k_addco_vcc_8, 8, "v_add_co_u32 %0, vcc, %0, %1", "+v"(x[2 * i]), : "vcc")
KERN(k_addco_s_8, 8, "v_add_co_u32 %0, s[20:21], %0, %1", "+v"(x[2 * i]), : "s20", "s21")
KERN(k_add64_8, 8, "v_lshl_add_u64 %0, %0, 0, %0", "+v"(v), )
KERN(k_mad_vcc_8, 8, "v_mad_u64_u32 %0, vcc, %1, %2, %0", "+v"(v), : "vcc")
KERN(k_mad_s_8, 8, "v_mad_u64_u32 %0, s[20:21], %1, %2, %0", "+v"(v), : "s20", "s21")
KERN(k_mad_1, 1, "v_mad_u64_u32 %0, s[20:21], %1, %2, %0", "+v"(v), : "s20", "s21")
KERN(k_mullo_8, 8, "v_mul_lo_u32 %0, %0, %1", "+v"(x[2 * i]), )
KERN(k_mulhi_8, 8, "v_mul_hi_u32 %0, %0, %1", "+v"(x[2 * i]), )
KERN(k_mov_8, 8, "v_mov_b32 %0, %1", "=v"(x[2 * i]), )
KERN(k_perm_8, 8, "v_perm_b32 %0, %0, %1, %2", "+v"(x[2 * i]), )
KERN(k_lshlor_8, 8, "v_lshl_or_b32 %0, %0, 7, %1", "+v"(x[2 * i]), )
KERN(k_addc_8, 8, "v_addc_co_u32 %0, vcc, %0, %1, vcc", "+v"(x[2 * i]), : "vcc")
KERN(k_subb_8, 8, "v_subb_co_u32 %0, vcc, %0, %1, vcc", "+v"(x[2 * i]), : "vcc")
KERN(k_cmp64_8, 8, "v_cmp_lt_u64 vcc, %0, %0", "+v"(v), : "vcc")
KERN(k_mov64_8, 8, "v_mov_b64 %0, %0", "+v"(v), )
KERN(k_add3_8, 8, "v_add3_u32 %0, %0, %1, %2", "+v"(x[2 * i]), )

// Mixed pairs: one instruction of each class per chain step (independent registers), to see
// whether a half-rate op and another op overlap in the issue pipeline (ops counted: 2 per step).
#define KERN2(NAME, CH, ASM, CLOB)                                               \
  __global__ void NAME(uint32_t* out, uint32_t a0) {                             \
    uint32_t x[CH * 2], y[CH];                                                   \
    for (int i = 0; i < CH * 2; i++) x[i] = a0 + i + threadIdx.x;               \
    for (int i = 0; i < CH; i++) y[i] = a0 * 5 + i;                              \
    uint32_t b = a0 * 3, c = a0 * 7;                                             \
    for (int it = 0; it < ITER; it++) {                                          \
      _Pragma("unroll") for (int i = 0; i < CH; i++) {                           \
        uint64_t& v = *reinterpret_cast<uint64_t*>(&x[2 * i]);                   \
        asm volatile(ASM : "+v"(v), "+v"(y[i]) : "v"(b), "v"(c) : CLOB);         \
      }                                                                          \
    }                                                                            \
    uint32_t s = 0;                                                              \
    for (int i = 0; i < CH * 2; i++) s ^= x[i];                                  \
    for (int i = 0; i < CH; i++) s ^= y[i];                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                              \
  }
KERN2(k_mad_addc, 8, "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc", "vcc")
KERN2(k_mad_xor, 8, "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n\tv_xor_b32 %1, %1, %2", "vcc")
KERN2(k_addc_xor, 8, "v_addc_co_u32 %1, vcc, %1, %2, vcc\n\tv_xor_b32 %1, %1, %3", "vcc")
KERN2(k_align_xor, 8, "v_alignbit_b32 %1, %1, %2, 7\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96", "vcc")
KERN2(k_mad_mad, 8, "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n\tv_mad_u64_u32 %0, s[22:23], %3, %2, %0", "vcc")

template <typename K>
void run(const char* name, K kern, uint32_t* buf, int blocks, int threads, int ch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<blocks, threads>>>(buf, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 3; r++) kern<<<blocks, threads>>>(buf, r + 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double ops = 3.0 * blocks * threads * (double)ITER * ch;
  printf("%-16s waves/SIMD=%-2d %8.3f ms %7.2f T lane-instr/s\n", name, blocks * threads / 64 / 1024,
         ms, ops / (ms * 1e-3) / 1e12);
}
int main() {
  void* buf;
  hipMalloc(&buf, (size_t)256 * 32 * 256 * 8);
  uint32_t* o = (uint32_t*)buf;
  for (int w : {1, 2, 4, 8}) {
    int threads = 256, blocks = 256 * w;  // w waves per SIMD (4 SIMDs per CU, 4 waves/block)
    printf("--- %d waves per SIMD\n", w);
    run("bitop3 x8", k_bitop3_8, o, blocks, threads, 8);
    run("bitop3 dep", k_bitop3_1, o, blocks, threads, 1);
    run("xor x8", k_xor_8, o, blocks, threads, 8);
    run("add_u32 x8", k_add_8, o, blocks, threads, 8);
    run("alignbit x8", k_alignbit_8, o, blocks, threads, 8);
    run("alignbit dep", k_alignbit_1, o, blocks, threads, 1);
    run("add_co vcc x8", k_addco_vcc_8, o, blocks, threads, 8);
    run("add_co sgpr x8", k_addco_s_8, o, blocks, threads, 8);
    run("add64 x8", k_add64_8, o, blocks, threads, 8);
    run("mad64 vcc x8", k_mad_vcc_8, o, blocks, threads, 8);
    run("mad64 sgpr x8", k_mad_s_8, o, blocks, threads, 8);
    run("mad64 dep", k_mad_1, o, blocks, threads, 1);
    run("mul_lo x8", k_mullo_8, o, blocks, threads, 8);
    run("mul_hi x8", k_mulhi_8, o, blocks, threads, 8);
    run("mov x8", k_mov_8, o, blocks, threads, 8);
    run("perm x8", k_perm_8, o, blocks, threads, 8);
    run("lshl_or x8", k_lshlor_8, o, blocks, threads, 8);
    run("addc x8", k_addc_8, o, blocks, threads, 8);
    run("subb x8", k_subb_8, o, blocks, threads, 8);
    run("cmp_lt_u64 x8", k_cmp64_8, o, blocks, threads, 8);
    run("mov_b64 x8", k_mov64_8, o, blocks, threads, 8);
    run("add3 x8", k_add3_8, o, blocks, threads, 8);
    run("mad64+addc", k_mad_addc, o, blocks, threads, 16);
    run("mad64+xor", k_mad_xor, o, blocks, threads, 16);
    run("addc+xor", k_addc_xor, o, blocks, threads, 16);
    run("alignbit+bitop3", k_align_xor, o, blocks, threads, 16);
    run("mad64+mad64", k_mad_mad, o, blocks, threads, 16);
  }
  return 0;
}
