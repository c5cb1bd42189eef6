// Host -> device bandwidth on MI355X for the host-buffer ABI (bench.py --role jobs): pinned
// hipMemcpyAsync (one stream, two streams, chunked), and a kernel that reads pinned host memory
// directly (hipHostMalloc mapped; 16-byte loads per lane) into device memory.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_h2d tools/ubench_h2d.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) dst[i] = src[i];
}

int main() {
  const size_t MAXB = (size_t)64 << 20;
  uint8_t *h, *hm, *d;
  CK(hipHostMalloc((void**)&h, MAXB, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hm, MAXB, hipHostMallocMapped));
  memset(h, 1, MAXB);
  memset(hm, 2, MAXB);
  uint8_t* hm_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&hm_dev, hm, 0));
  CK(hipMalloc((void**)&d, 2 * MAXB));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t sizes[] = {(size_t)1 << 20, (size_t)4 << 20, (size_t)16 << 20, (size_t)64 << 20};
  for (size_t sz : sizes) {
    float ms = 0;
    const int R = 10;
    // 1) one pinned copy
    CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s0));
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < R; r++) CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    const double g1 = sz * R / (ms / 1e3) / 1e9;
    // 2) two halves on two streams at once
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, s0));
    CK(hipStreamWaitEvent(s1, a, 0));
    for (int r = 0; r < R; r++) {
      CK(hipMemcpyAsync(d, h, sz / 2, hipMemcpyHostToDevice, s0));
      CK(hipMemcpyAsync(d + MAXB, h + sz / 2, sz / 2, hipMemcpyHostToDevice, s1));
    }
    hipEvent_t c;
    CK(hipEventCreate(&c));
    CK(hipEventRecord(c, s1));
    CK(hipStreamWaitEvent(s0, c, 0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    const double g2 = sz * R / (ms / 1e3) / 1e9;
    // 3) eight chunks on one stream
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < R; r++)
      for (int k = 0; k < 8; k++)
        CK(hipMemcpyAsync(d + k * (sz / 8), h + k * (sz / 8), sz / 8, hipMemcpyHostToDevice, s0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    const double g3 = sz * R / (ms / 1e3) / 1e9;
    // 4) kernel pull from mapped pinned memory
    const size_t n16 = sz / 16;
    for (int blocks : {256, 1024, 4096}) {
      k_pull<<<blocks, 256, 0, s0>>>((const uint4*)hm_dev, (uint4*)d, n16);
      CK(hipStreamSynchronize(s0));
      CK(hipEventRecord(a, s0));
      for (int r = 0; r < R; r++) k_pull<<<blocks, 256, 0, s0>>>((const uint4*)hm_dev, (uint4*)d, n16);
      CK(hipEventRecord(b, s0));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      printf("size %3zu MiB  kernel pull (%4d blocks) %6.1f GB/s\n", sz >> 20, blocks,
             sz * R / (ms / 1e3) / 1e9);
    }
    // 5) D2H one copy
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < R; r++) CK(hipMemcpyAsync(h, d, sz, hipMemcpyDeviceToHost, s0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    const double g5 = sz * R / (ms / 1e3) / 1e9;
    printf("size %3zu MiB  H2D one %6.1f  two-streams %6.1f  8-chunks %6.1f  D2H %6.1f GB/s\n",
           sz >> 20, g1, g2, g3, g5);
    fflush(stdout);
  }
  return 0;
}
