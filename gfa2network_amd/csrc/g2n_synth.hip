// g2n_synth.hip — host and device drivers of the synthetic GFA generator (synth.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/g2n_synth.h"
#include "g2n_internal.h"
#include "g2n_scan.hip"
#include "synth.h"

namespace g2n {

__global__ void __launch_bounds__(256) k_synth_len(SynthSpec s, uint64_t n, uint64_t* __restrict__ len) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) len[i] = synth_line_len(s, i);
}

__global__ void __launch_bounds__(256) k_synth_write(SynthSpec s, uint64_t n, const uint64_t* __restrict__ off,
                                                     char* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) synth_write_line(s, i, out + off[i]);
}

static SynthSpec to_spec(const g2n_synth_spec* p) {
  SynthSpec s{};
  s.n_s = p->n_segments;
  s.n_l = p->n_links;
  s.seed = p->seed;
  s.rc = p->rc_tag;
  s.names = p->names;
  s.far = p->far_links;
  s.pmul = s.names == 2 ? synth_perm_mul(s.n_s) : 1;
  return s;
}

}  // namespace g2n

extern "C" {

int g2n_synth_host(const g2n_synth_spec* spec, int n_threads, uint8_t** out, size_t* len) {
  using namespace g2n;
  if (!spec || !out || !len || (spec->n_links && !spec->n_segments)) return G2N_E_ARG;
  if (spec->names && spec->n_segments >= (1ull << 32)) return G2N_E_ARG;  // hashed names: a u32 bijection
  const SynthSpec s = to_spec(spec);
  const uint64_t n = synth_n_lines(s);
  int T = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  T = (int)std::min<uint64_t>((uint64_t)T, n);
  std::vector<uint64_t> part(T + 1, 0);
  auto chunk = [&](int t, uint64_t* a, uint64_t* b) {
    *a = n * (uint64_t)t / (uint64_t)T;
    *b = n * (uint64_t)(t + 1) / (uint64_t)T;
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        uint64_t a, b, sum = 0;
        chunk(t, &a, &b);
        for (uint64_t i = a; i < b; i++) sum += synth_line_len(s, i);
        part[t + 1] = sum;
      });
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < T; t++) part[t + 1] += part[t];
  uint8_t* buf = (uint8_t*)std::malloc(part[T] ? part[T] : 1);
  if (!buf) return G2N_E_NOMEM;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        uint64_t a, b;
        chunk(t, &a, &b);
        char* o = (char*)buf + part[t];
        for (uint64_t i = a; i < b; i++) {
          synth_write_line(s, i, o);
          o += synth_line_len(s, i);
        }
      });
    for (auto& x : th) x.join();
  }
  *out = buf;
  *len = part[T];
  return G2N_OK;
}

void g2n_synth_free_host(uint8_t* buf) { std::free(buf); }

int g2n_synth_device(int device, const g2n_synth_spec* spec, void** d_out, size_t* len) {
  using namespace g2n;
  if (!spec || !d_out || !len || (spec->n_links && !spec->n_segments)) return G2N_E_ARG;
  if (spec->names && spec->n_segments >= (1ull << 32)) return G2N_E_ARG;
  const SynthSpec s = to_spec(spec);
  const uint64_t n = synth_n_lines(s);
  if (hipSetDevice(device) != hipSuccess) return G2N_E_DEVICE;
  uint64_t *dlen = nullptr, *doff = nullptr;
  void* tmp = nullptr;
  char* out = nullptr;
  int rc = G2N_OK;
  size_t tb = 0;
  uint64_t last_len = 0, last_off = 0, total = 0;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (hipMalloc(&dlen, n * 8) != hipSuccess || hipMalloc(&doff, n * 8) != hipSuccess) { rc = G2N_E_NOMEM; goto done; }
  hipLaunchKernelGGL(k_synth_len, dim3(grid), dim3(256), 0, 0, s, n, dlen);
  {  // line offsets: the pipeline's single-pass scan (g2n_scan.hip)
    const uint64_t tiles = scan_tiles(n);
    tb = (tiles + 1) * sizeof(unsigned long long);
    if (hipMalloc(&tmp, tb) != hipSuccess) { rc = G2N_E_NOMEM; goto done; }
    if (hipMemset(tmp, 0, tb) != hipSuccess) { rc = G2N_E_DEVICE; goto done; }
    auto* st = (unsigned long long*)tmp;
    hipLaunchKernelGGL((k_scan_excl<uint64_t, uint64_t>), dim3((unsigned)tiles), dim3(256), 0, 0, (const uint64_t*)dlen,
                       doff, n, st + 1, st, (uint64_t*)nullptr, 1u, 0ull);  // (zeroed: epoch 1, ticket 0)
  }
  if (hipMemcpy(&last_len, dlen + n - 1, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&last_off, doff + n - 1, 8, hipMemcpyDeviceToHost) != hipSuccess) { rc = G2N_E_DEVICE; goto done; }
  total = last_off + last_len;
  if (hipMalloc(&out, total + 64) != hipSuccess) { rc = G2N_E_NOMEM; goto done; }
  hipLaunchKernelGGL(k_synth_write, dim3(grid), dim3(256), 0, 0, s, n, doff, out);
  if (hipDeviceSynchronize() != hipSuccess) { rc = G2N_E_DEVICE; goto done; }
  *d_out = out;
  *len = total;
  out = nullptr;
done:
  if (dlen) (void)hipFree(dlen);
  if (doff) (void)hipFree(doff);
  if (tmp) (void)hipFree(tmp);
  if (out) (void)hipFree(out);
  if (rc != G2N_OK) (void)hipGetLastError();
  return rc;
}

void g2n_synth_free_device(void* d_buf) {
  if (d_buf) (void)hipFree(d_buf);
}

int g2n_synth_download(void* host_dst, const void* d_src, size_t len) {
  return hipMemcpy(host_dst, d_src, len, hipMemcpyDeviceToHost) == hipSuccess ? G2N_OK : G2N_E_DEVICE;
}

}  // extern "C"
