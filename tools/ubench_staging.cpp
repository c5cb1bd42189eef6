// Host staging microbenchmark: stream_copy (rows as they are) against stream_transpose16 (the leader
// staging's [cell][report] form, 8 or 16 reports per cell) over 500-report jobs of 5.6 KB rows.
//   g++ -O2 -march=x86-64-v3 -std=c++17 -pthread -o /tmp/ubs tools/ubench_staging.cpp; /tmp/ubs MODE THREADS
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <thread>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <vector>
#include <algorithm>
static void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m128i a = _mm_loadu_si128((const __m128i*)(src + i)), b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32)), d = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a); _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c); _mm_stream_si128((__m128i*)(dst + i + 48), d);
  }
  memcpy(dst + i, src + i, n - i); _mm_sfence();
}
static void tr(uint8_t* dst, size_t cap, size_t c0, const uint8_t* src, uint32_t n, uint32_t cells) {
  const size_t row = 16 * (size_t)cells;
  for (uint32_t r0 = 0; r0 < n; r0 += 8) {
    const uint32_t k = std::min(8u, n - r0);
    const uint8_t* s0 = src + row * r0;
    for (uint32_t e = 0; e < cells; e++) {
      __m128i* d = (__m128i*)(dst + 16 * (e * cap + c0 + r0));
      for (uint32_t i = 0; i < k; i++) _mm_stream_si128(d + i, _mm_loadu_si128((const __m128i*)(s0 + row * i + 16 * (size_t)e)));
    }
  }
  _mm_sfence();
}
// variant: 16 reports per cell (4 full lines), e-blocked
static void tr16(uint8_t* dst, size_t cap, size_t c0, const uint8_t* src, uint32_t n, uint32_t cells) {
  const size_t row = 16 * (size_t)cells;
  for (uint32_t r0 = 0; r0 < n; r0 += 16) {
    const uint32_t k = std::min(16u, n - r0);
    const uint8_t* s0 = src + row * r0;
    for (uint32_t e = 0; e < cells; e++) {
      __m128i* d = (__m128i*)(dst + 16 * (e * cap + c0 + r0));
      for (uint32_t i = 0; i < k; i++) _mm_stream_si128(d + i, _mm_loadu_si128((const __m128i*)(s0 + row * i + 16 * (size_t)e)));
    }
  }
  _mm_sfence();
}
// variant: AVX-512, 4 reports x 4 cells per step -- four 64-byte row loads, a 4x4 transpose of
// 16-byte lanes, four full-line non-temporal stores (64-byte aligned columns)
__attribute__((target("avx512f"))) static void tr512(uint8_t* dst, size_t cap, size_t c0,
                                                     const uint8_t* src, uint32_t n, uint32_t cells) {
  const size_t row = 16 * (size_t)cells;
  const uint32_t n4 = n & ~3u, e4 = cells & ~3u;
  for (uint32_t r0 = 0; r0 < n4; r0 += 4) {
    const uint8_t* s0 = src + row * r0;
    for (uint32_t e = 0; e < e4; e += 4) {
      const __m512i z0 = _mm512_loadu_si512(s0 + 16 * (size_t)e);
      const __m512i z1 = _mm512_loadu_si512(s0 + row + 16 * (size_t)e);
      const __m512i z2 = _mm512_loadu_si512(s0 + 2 * row + 16 * (size_t)e);
      const __m512i z3 = _mm512_loadu_si512(s0 + 3 * row + 16 * (size_t)e);
      const __m512i t0 = _mm512_shuffle_i64x2(z0, z1, 0x44), t1 = _mm512_shuffle_i64x2(z0, z1, 0xEE);
      const __m512i t2 = _mm512_shuffle_i64x2(z2, z3, 0x44), t3 = _mm512_shuffle_i64x2(z2, z3, 0xEE);
      uint8_t* d = dst + 16 * (e * cap + c0 + r0);
      _mm512_stream_si512((__m512i*)d, _mm512_shuffle_i64x2(t0, t2, 0x88));
      _mm512_stream_si512((__m512i*)(d + 16 * cap), _mm512_shuffle_i64x2(t0, t2, 0xDD));
      _mm512_stream_si512((__m512i*)(d + 32 * cap), _mm512_shuffle_i64x2(t1, t3, 0x88));
      _mm512_stream_si512((__m512i*)(d + 48 * cap), _mm512_shuffle_i64x2(t1, t3, 0xDD));
    }
    for (uint32_t e = e4; e < cells; e++)
      for (uint32_t i = 0; i < 4; i++)
        _mm_stream_si128((__m128i*)(dst + 16 * (e * cap + c0 + r0 + i)),
                         _mm_loadu_si128((const __m128i*)(s0 + row * i + 16 * (size_t)e)));
  }
  for (uint32_t r = n4; r < n; r++)
    for (uint32_t e = 0; e < cells; e++)
      _mm_stream_si128((__m128i*)(dst + 16 * (e * cap + c0 + r)),
                       _mm_loadu_si128((const __m128i*)(src + row * r + 16 * (size_t)e)));
  _mm_sfence();
}
// variant: plain (cached) 16-byte stores
static void tr_cached(uint8_t* dst, size_t cap, size_t c0, const uint8_t* src, uint32_t n, uint32_t cells) {
  const size_t row = 16 * (size_t)cells;
  for (uint32_t r0 = 0; r0 < n; r0 += 8) {
    const uint32_t k = std::min(8u, n - r0);
    const uint8_t* s0 = src + row * r0;
    for (uint32_t e = 0; e < cells; e++) {
      __m128i* d = (__m128i*)(dst + 16 * (e * cap + c0 + r0));
      for (uint32_t i = 0; i < k; i++) _mm_storeu_si128(d + i, _mm_loadu_si128((const __m128i*)(s0 + row * i + 16 * (size_t)e)));
    }
  }
}
int main(int argc, char** argv) {
  int mode = atoi(argv[1]), T = atoi(argv[2]);
  // PIN (argv[3]): 0 none; 1 main and workers on CPUs 0.. (one socket, where the data is touched);
  // 2 workers alternate between CPUs 0.. and 64.. (half of them on the other socket)
  const int pin = argc > 3 ? atoi(argv[3]) : 0;
  const int huge = argc > 4 ? atoi(argv[4]) : 0;  // 1: destination on transparent 2 MB pages
  auto pin_to = [](int cpu) {
    cpu_set_t cs; CPU_ZERO(&cs); CPU_SET(cpu, &cs); pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
  };
  if (pin) pin_to(0);
  const uint32_t cells = 352, js = 500, pool = 4 * 32768; const size_t row = 16 * cells;
  std::vector<uint8_t> src((size_t)pool * row); for (size_t i = 0; i < src.size(); i += 4096) src[i] = i;
  const uint32_t cap = 16384; std::vector<uint8_t*> dst(T);
  for (int t = 0; t < T; t++) {
    const size_t bytes = ((size_t)cap * row + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    dst[t] = (uint8_t*)aligned_alloc(2u << 20, bytes);
    if (huge) madvise(dst[t], bytes, MADV_HUGEPAGE);
    memset(dst[t], 0, bytes);
  }
  if (mode == 9) {  // tr512 against tr on odd shapes
    for (uint32_t n : {500u, 503u, 1u, 7u}) for (uint32_t cl : {352u, 351u, 5u}) {
      const size_t rw = 16 * (size_t)cl;
      uint8_t* a = (uint8_t*)aligned_alloc(64, (size_t)cap * rw); uint8_t* b = (uint8_t*)aligned_alloc(64, (size_t)cap * rw);
      memset(a, 0, (size_t)cap * rw); memset(b, 0, (size_t)cap * rw);
      std::vector<uint8_t> sr((size_t)n * rw); for (size_t i = 0; i < sr.size(); i++) sr[i] = (uint8_t)(i * 131 + 7);
      tr(a, cap, 1000, sr.data(), n, cl); tr512(b, cap, 1000, sr.data(), n, cl);
      printf("n %u cells %u: %s\n", n, cl, memcmp(a, b, (size_t)cap * rw) ? "DIFFER" : "equal");
      free(a); free(b);
    }
    return 0;
  }
  const int jobs_per_thread = 64;
  if (FILE* f = fopen("/proc/self/smaps_rollup", "r")) {  // did the destination get 2 MB pages?
    char ln[256];
    while (fgets(ln, sizeof ln, f))
      if (!strncmp(ln, "AnonHugePages", 13)) fprintf(stderr, "%s", ln);
    fclose(f);
  }
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back([&, t] {
    for (int j = 0; j < jobs_per_thread; j++) {
      size_t r0 = ((size_t)(t * jobs_per_thread + j) * js * 7) % (pool - js);
      uint32_t c0 = (j % 32) * js;
      if (mode == 0) stream_copy(dst[t] + (size_t)c0 * row, src.data() + r0 * row, (size_t)js * row);
      else if (mode == 1) tr(dst[t], cap, c0, src.data() + r0 * row, js, cells);
      else if (mode == 2) tr16(dst[t], cap, c0, src.data() + r0 * row, js, cells);
      else if (mode == 3) tr512(dst[t], cap, c0, src.data() + r0 * row, js, cells);
      else tr_cached(dst[t], cap, c0, src.data() + r0 * row, js, cells);
    }
  });
  for (auto& x : th) x.join();
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  double gb = (double)T * jobs_per_thread * js * row / 1e9;
  printf("huge %d pin %d mode %d T %d: %.2f GB in %.3f s = %.2f GB/s total, %.2f GB/s per thread\n", huge, pin, mode, T, gb, dt, gb / dt, gb / dt / T);
  (void)pin;
}
