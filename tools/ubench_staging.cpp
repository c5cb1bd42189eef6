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
int main(int argc, char** argv) {
  int mode = atoi(argv[1]), T = atoi(argv[2]);
  const uint32_t cells = 352, js = 500, pool = 4 * 32768; const size_t row = 16 * cells;
  std::vector<uint8_t> src((size_t)pool * row); for (size_t i = 0; i < src.size(); i += 4096) src[i] = i;
  const uint32_t cap = 16384; std::vector<uint8_t*> dst(T);
  for (int t = 0; t < T; t++) { dst[t] = (uint8_t*)aligned_alloc(4096, (size_t)cap * row); memset(dst[t], 0, (size_t)cap * row); }
  const int jobs_per_thread = 64;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back([&, t] {
    for (int j = 0; j < jobs_per_thread; j++) {
      size_t r0 = ((size_t)(t * jobs_per_thread + j) * js * 7) % (pool - js);
      uint32_t c0 = (j % 32) * js;
      if (mode == 0) stream_copy(dst[t] + (size_t)c0 * row, src.data() + r0 * row, (size_t)js * row);
      else if (mode == 1) tr(dst[t], cap, c0, src.data() + r0 * row, js, cells);
      else tr16(dst[t], cap, c0, src.data() + r0 * row, js, cells);
    }
  });
  for (auto& x : th) x.join();
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  double gb = (double)T * jobs_per_thread * js * row / 1e9;
  printf("mode %d T %d: %.2f GB in %.3f s = %.2f GB/s total, %.2f GB/s per thread\n", mode, T, gb, dt, gb / dt, gb / dt / T);
}
