// rocprim onesweep configurations on the COO->CSR sort shape: 200M stable (row < 2^26, u32) pairs.
#include <hip/hip_runtime.h>
#include <string.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(uint32_t* k, uint32_t* v, uint64_t n, uint32_t n_rows) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  uint64_t h = t * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  k[t] = (uint32_t)(h % n_rows);
  v[t] = (uint32_t)(h >> 40);
}

template <class Cfg>
void run(const char* name, uint32_t* k0, uint32_t* k1, uint32_t* v0, uint32_t* v1, uint64_t n, int bits) {
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k0, k1, v0, v1, n, 0u, (unsigned)bits, 0));
  void* tmp;
  CK(hipMalloc(&tmp, tb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k0, k1, v0, v1, n, 0u, (unsigned)bits, 0));
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CK(hipEventRecord(a));
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k0, k1, v0, v1, n, 0u, (unsigned)bits, 0));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  // stability / order check on a sample
  uint32_t hk[4096];
  CK(hipMemcpy(hk, k1 + n / 2, sizeof(hk), hipMemcpyDeviceToHost));
  bool ok = true;
  for (int q = 1; q < 4096; q++) ok = ok && hk[q - 1] <= hk[q];
  printf("{\"config\": \"%s\", \"n\": %llu, \"bits\": %d, \"ms\": %.3f, \"Gpairs_per_s\": %.1f, \"sorted_sample\": %s}\n",
         name, (unsigned long long)n, bits, best, n / best / 1e6, ok ? "true" : "false");
  CK(hipFree(tmp));
}

using namespace rocprim;
template <unsigned B, unsigned T, unsigned I>
using OS = radix_sort_config<default_config, default_config,
                             radix_sort_onesweep_config<kernel_config<T, I>, kernel_config<T, I>, B,
                                                        block_radix_rank_algorithm::match>>;

int main() {
  const uint64_t n = 200000000ull;
  const uint32_t n_rows = 50000000u;
  uint32_t *k0, *k1, *v0, *v1;
  CK(hipMalloc(&k0, n * 4));
  CK(hipMalloc(&k1, n * 4));
  CK(hipMalloc(&v0, n * 4));
  CK(hipMalloc(&v1, n * 4));
  k_fill<<<(unsigned)((n + 255) / 256), 256>>>(k0, v0, n, n_rows);
  CK(hipDeviceSynchronize());
  run<default_config>("default", k0, k1, v0, v1, n, 26);
  run<OS<8, 1024, 8>>("os8_1024x8", k0, k1, v0, v1, n, 26);
  run<OS<8, 512, 16>>("os8_512x16", k0, k1, v0, v1, n, 26);
  run<OS<9, 1024, 8>>("os9_1024x8", k0, k1, v0, v1, n, 26);
  run<OS<9, 512, 16>>("os9_512x16", k0, k1, v0, v1, n, 26);
  run<OS<9, 1024, 12>>("os9_1024x12", k0, k1, v0, v1, n, 26);
  run<OS<10, 1024, 8>>("os10_1024x8", k0, k1, v0, v1, n, 26);
  run<OS<11, 1024, 8>>("os11_1024x8", k0, k1, v0, v1, n, 26);
  run<OS<11, 512, 8>>("os11_512x8", k0, k1, v0, v1, n, 26);
  return 0;
}
