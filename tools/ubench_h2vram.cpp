// Host threads writing straight into fine-grained device memory (hipExtMallocWithFlags
// hipDeviceMallocFinegrained, CPU access through the PCIe BAR) against writing pinned host
// memory: can the jobs line's callers stage their shares into HBM themselves, so the launch
// reads HBM instead of pulling 17 MB per group over PCIe inside k_prep_h?  A kernel checks the
// bytes afterwards.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread -o tools/ubench_h2vram tools/ubench_h2vram.cpp
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_sum(const uint32_t* p, size_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += p[i];
  atomicAdd(out, s);
}

static void fill_nt(uint8_t* dst, const uint8_t* src, size_t n) {  // 16-byte streaming stores
  for (size_t i = 0; i < n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
    const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
    const __m128i d = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a);
    _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c);
    _mm_stream_si128((__m128i*)(dst + i + 48), d);
  }
  _mm_sfence();
}

static double run(uint8_t* dst, const uint8_t* src, size_t bytes, int T, bool nt, int reps) {
  const size_t per = (bytes / T) & ~(size_t)63;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; r++) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([=] {
        if (nt)
          fill_nt(dst + t * per, src + t * per, per);
        else
          memcpy(dst + t * per, src + t * per, per);
      });
    for (auto& x : th) x.join();
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return (double)per * T * reps / s / 1e9;
}

int main() {
  const size_t B = (size_t)64 << 20;
  uint8_t* src = (uint8_t*)aligned_alloc(64, B);
  for (size_t i = 0; i < B / 4; i++) ((uint32_t*)src)[i] = (uint32_t)(i * 2654435761u);
  uint8_t *pinned = nullptr, *vram = nullptr;
  CK(hipHostMalloc((void**)&pinned, B, hipHostMallocDefault));
  CK(hipExtMallocWithFlags((void**)&vram, B, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, vram));
  printf("fine-grained VRAM %p: type %d device %d host pointer %p\n", (void*)vram, (int)at.type,
         at.device, at.hostPointer);
  fflush(stdout);
  for (int T : {1, 4, 16, 32, 64}) {
    for (int nt = 0; nt < 2; nt++) {
      const double gp = run(pinned, src, B, T, nt, 5);
      const double gv = run(vram, src, B, T, nt, 5);
      printf("threads %2d %-8s pinned host %6.1f GB/s   fine-grained VRAM %6.1f GB/s\n", T,
             nt ? "stream" : "memcpy", gp, gv);
      fflush(stdout);
    }
  }
  // the GPU sees what the host wrote
  unsigned long long* d_sum;
  CK(hipMalloc((void**)&d_sum, 8));
  CK(hipMemset(d_sum, 0, 8));
  k_sum<<<1024, 256>>>((const uint32_t*)vram, B / 4, d_sum);
  unsigned long long got = 0, want = 0;
  CK(hipMemcpy(&got, d_sum, 8, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < B / 4; i++) want += ((uint32_t*)src)[i];
  printf("kernel sum over the VRAM the host wrote: %s\n", got == want ? "matches" : "MISMATCH");
  return got == want ? 0 : 1;
}
