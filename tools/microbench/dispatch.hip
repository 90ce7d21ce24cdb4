// Workgroup dispatch / ticket costs on gfx950: near-empty kernels timed with hipEvents; one
// JSON line per shape.  k_empty: LDS write + barrier; k_ticket: thread 0 takes an atomic
// ticket from ONE counter (the ordered-block-id idiom), barrier; k_ticket_batch: one ticket per
// 8 blocks' worth of work (the block loops 8 times).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int kLds>
__global__ void k_empty(unsigned* out) {
  __shared__ unsigned s[kLds / 4 > 0 ? kLds / 4 : 1];
  s[threadIdx.x % (kLds / 4 > 0 ? kLds / 4 : 1)] = threadIdx.x;
  __syncthreads();
  if (s[0] == 0xFFFFFFFFu) out[blockIdx.x] = 1;
}

__global__ void k_ticket(unsigned* out, unsigned* ticket) {
  __shared__ unsigned s[5504];
  __shared__ unsigned t;
  if (threadIdx.x == 0) t = atomicAdd(ticket, 1u);
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (s[t & 255] == 0xFFFFFFFFu) out[blockIdx.x] = t;
}

__global__ void k_ticket_relaxed(unsigned* out, unsigned* ticket) {
  __shared__ unsigned s[5504];
  __shared__ unsigned t;
  if (threadIdx.x == 0) t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (s[t & 255] == 0xFFFFFFFFu) out[blockIdx.x] = t;
}

template <class F>
void time_it(const char* name, int blocks, F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < 5; i++) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("{\"kernel\": \"%s\", \"blocks\": %d, \"ms\": %.4f, \"ns_per_block\": %.2f}\n", name, blocks, ms / 5,
         ms / 5 * 1e6 / blocks);
}

int main() {
  unsigned *d, *tk;
  (void)hipMalloc(&d, 1 << 24);
  (void)hipMalloc(&tk, 4096);
  for (int blocks : {2048, 24576, 196608}) {
    time_it("empty_lds16k_256", blocks, [&] { hipLaunchKernelGGL(k_empty<16384>, dim3(blocks), dim3(256), 0, 0, d); });
    time_it("ticket_256", blocks, [&] { hipLaunchKernelGGL(k_ticket, dim3(blocks), dim3(256), 0, 0, d, tk); });
    time_it("ticket_relaxed_256", blocks,
            [&] { hipLaunchKernelGGL(k_ticket_relaxed, dim3(blocks), dim3(256), 0, 0, d, tk); });
  }
  return 0;
}
