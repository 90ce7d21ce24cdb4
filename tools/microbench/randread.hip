// Random-read ceiling of the MI355X for the dictionary's access shape: every lane reads one
// B-byte record at a hashed position of a T-byte table (no reuse), as k_insert_round's probe
// does.  Prints GB/s of useful bytes and records/s per (record size, table size).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ inline uint64_t mix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

template <int kWords>  // record = kWords x 16 B
__global__ void __launch_bounds__(256) k_rand(const uint4* __restrict__ table, uint64_t n_rec, uint64_t n,
                                              uint32_t* __restrict__ out, uint64_t seed) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const uint64_t r = mix(t + seed) % n_rec;
  uint32_t acc = 0;
#pragma unroll
  for (int w = 0; w < kWords; w++) {
    const uint4 v = table[r * kWords + w];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[t] = acc;
}

__global__ void k_seq(const uint4* __restrict__ table, uint64_t n16, uint32_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n16) return;
  const uint4 v = table[t];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const uint64_t table_bytes = 4ull << 30;  // the C4 dictionary is 4.3 GB
  const uint64_t n = 400000000ull;          // the C4 lookup round: 400M touches
  uint4* table;
  uint32_t* out;
  CK(hipMalloc(&table, table_bytes));
  CK(hipMalloc(&out, n * 4));
  CK(hipMemset(table, 0x5A, table_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  // streaming reference
  {
    const uint64_t n16 = table_bytes / 16;
    k_seq<<<(unsigned)((n16 + 255) / 256), 256>>>(table, n16, out);
    CK(hipEventRecord(a));
    k_seq<<<(unsigned)((n16 + 255) / 256), 256>>>(table, n16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"shape\": \"stream 16B/lane\", \"table_GB\": %.2f, \"ms\": %.3f, \"GBps\": %.1f}\n", table_bytes / 1e9, ms,
           table_bytes / ms / 1e6);
  }
  const uint64_t sizes[] = {table_bytes, 256ull << 20, 32ull << 20};
  for (uint64_t tb : sizes) {
    for (int words = 1; words <= 4; words *= 2) {
      const uint64_t n_rec = tb / (16ull * words);
      const unsigned grid = (unsigned)((n + 255) / 256);
      auto launch = [&](uint64_t seed) {
        if (words == 1) k_rand<1><<<grid, 256>>>(table, n_rec, n, out, seed);
        else if (words == 2) k_rand<2><<<grid, 256>>>(table, n_rec, n, out, seed);
        else k_rand<4><<<grid, 256>>>(table, n_rec, n, out, seed);
      };
      launch(1);
      CK(hipEventRecord(a));
      launch(2);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"shape\": \"random %dB records\", \"table_GB\": %.3f, \"records\": %llu, \"ms\": %.3f, "
             "\"Grec_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
             16 * words, tb / 1e9, (unsigned long long)n, ms, n / ms / 1e6, n * 16.0 * words / ms / 1e6);
    }
  }
  CK(hipFree(table));
  CK(hipFree(out));
  return 0;
}
