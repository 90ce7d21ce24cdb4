// Host <-> HBM transfer shapes for the end-to-end ingest (file -> HBM -> CSR -> host):
// pageable hipMemcpy, pinned staging rings driven by T host threads, hipHostRegister,
// and page-cache pread / zlib inflate rates on the box's cores.  Prints one JSON line per
// measurement (GB/s).  Build: hipcc -O3 --offload-arch=gfx950 xfer.hip -lz -lpthread
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void report(const char* what, int threads, size_t chunk, size_t bytes, double s) {
  printf("{\"what\": \"%s\", \"threads\": %d, \"chunk_mib\": %zu, \"bytes\": %zu, \"s\": %.4f, \"gbs\": %.2f}\n", what,
         threads, chunk >> 20, bytes, s, bytes / s / 1e9);
  fflush(stdout);
}

// T threads, each with 2 pinned slots + its own stream: memcpy (or pread) into a slot, H2D async.
static double staged_h2d(uint8_t* d, const uint8_t* src, int fd, size_t bytes, int T, size_t chunk) {
  std::vector<std::thread> th;
  std::atomic<size_t> next{0};
  const size_t nchunks = (bytes + chunk - 1) / chunk;
  std::vector<uint8_t*> slots(2 * T);
  for (auto& s : slots) CK(hipHostMalloc((void**)&s, chunk, hipHostMallocDefault));
  double t0 = now();
  for (int t = 0; t < T; t++) {
    th.emplace_back([&, t] {
      hipStream_t st;
      CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      hipEvent_t ev[2];
      CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
      bool used[2] = {false, false};
      int k = 0;
      for (;;) {
        size_t i = next.fetch_add(1);
        if (i >= nchunks) break;
        size_t off = i * chunk, n = std::min(chunk, bytes - off);
        uint8_t* s = slots[2 * t + k];
        if (used[k]) CK(hipEventSynchronize(ev[k]));
        if (src) memcpy(s, src + off, n);
        else {
          size_t got = 0;
          while (got < n) {
            ssize_t r = pread(fd, s + got, n - got, off + got);
            if (r <= 0) { perror("pread"); exit(1); }
            got += r;
          }
        }
        CK(hipMemcpyAsync(d + off, s, n, hipMemcpyHostToDevice, st));
        CK(hipEventRecord(ev[k], st));
        used[k] = true;
        k ^= 1;
      }
      CK(hipStreamSynchronize(st));
      hipEventDestroy(ev[0]);
      hipEventDestroy(ev[1]);
      hipStreamDestroy(st);
    });
  }
  for (auto& x : th) x.join();
  double s = now() - t0;
  for (auto& p : slots) CK(hipHostFree(p));
  return s;
}

// T threads D2H into pinned slots then memcpy out to a pageable destination.
static double staged_d2h(uint8_t* dst, const uint8_t* d, size_t bytes, int T, size_t chunk) {
  std::vector<std::thread> th;
  std::atomic<size_t> next{0};
  const size_t nchunks = (bytes + chunk - 1) / chunk;
  std::vector<uint8_t*> slots(T);
  for (auto& s : slots) CK(hipHostMalloc((void**)&s, chunk, hipHostMallocDefault));
  double t0 = now();
  for (int t = 0; t < T; t++) {
    th.emplace_back([&, t] {
      hipStream_t st;
      CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      for (;;) {
        size_t i = next.fetch_add(1);
        if (i >= nchunks) break;
        size_t off = i * chunk, n = std::min(chunk, bytes - off);
        CK(hipMemcpyAsync(slots[t], d + off, n, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        memcpy(dst + off, slots[t], n);
      }
      hipStreamDestroy(st);
    });
  }
  for (auto& x : th) x.join();
  double s = now() - t0;
  for (auto& p : slots) CK(hipHostFree(p));
  return s;
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 4096ull) << 20;
  uint8_t* d;
  CK(hipMalloc((void**)&d, bytes));
  uint8_t* h = (uint8_t*)malloc(bytes);
  for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)(i * 131 + (i >> 13));
  CK(hipMemcpy(d, h, 1 << 20, hipMemcpyHostToDevice));  // warm the runtime

  double t0 = now();
  CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  report("h2d_pageable_hipMemcpy", 1, 0, bytes, now() - t0);

  uint8_t* o = (uint8_t*)malloc(bytes);  // untouched pages
  t0 = now();
  CK(hipMemcpy(o, d, bytes, hipMemcpyDeviceToHost));
  report("d2h_pageable_untouched", 1, 0, bytes, now() - t0);
  t0 = now();
  CK(hipMemcpy(o, d, bytes, hipMemcpyDeviceToHost));
  report("d2h_pageable_touched", 1, 0, bytes, now() - t0);

  for (int T : {1, 2, 4, 8, 16})
    for (size_t ch : {(size_t)8 << 20, (size_t)32 << 20}) report("h2d_staged_memcpy", T, ch, bytes, staged_h2d(d, h, -1, bytes, T, ch));
  for (int T : {2, 4, 8, 16}) {
    uint8_t* o2 = (uint8_t*)malloc(bytes);
    report("d2h_staged_untouched", T, 32 << 20, bytes, staged_d2h(o2, d, bytes, T, 32 << 20));
    free(o2);
  }

  t0 = now();
  CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
  double treg = now() - t0;
  report("hipHostRegister", 1, 0, bytes, treg);
  t0 = now();
  CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  report("h2d_registered", 1, 0, bytes, now() - t0);
  t0 = now();
  CK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
  report("d2h_registered", 1, 0, bytes, now() - t0);
  CK(hipHostUnregister(h));

  // page-cache file reads
  const char* path = "/tmp/g2n_xfer.bin";
  {
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0600);
    size_t w = 0;
    while (w < bytes) { ssize_t r = write(fd, h + w, bytes - w); if (r <= 0) { perror("write"); return 1; } w += r; }
    close(fd);
  }
  int fd = open(path, O_RDONLY);
  for (int T : {1, 4, 8, 16}) report("pread_staged_h2d", T, 32, bytes, staged_h2d(d, nullptr, fd, bytes, T, 32 << 20));
  close(fd);
  unlink(path);

  // zlib inflate rate of GFA-like text, per core and with T cores on separate members
  {
    const size_t mb = 64 << 20;
    std::vector<uint8_t> txt(mb);
    size_t p = 0;
    unsigned long long x = 88172645463325252ull;
    unsigned id = 1;
    while (p + 64 < mb) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      p += snprintf((char*)txt.data() + p, 64, "L\t%u\t+\t%u\t%c\t0M\n", id, id + (unsigned)(x % 7) + 1, (x >> 8) % 10 ? '+' : '-');
      id += (x >> 16) % 3;
    }
    uLongf cl = compressBound(p);
    std::vector<uint8_t> comp(cl);
    compress2(comp.data(), &cl, txt.data(), p, 6);
    for (int T : {1, 4, 8, 16}) {
      std::vector<std::thread> th;
      t0 = now();
      for (int t = 0; t < T; t++)
        th.emplace_back([&] {
          std::vector<uint8_t> out(p);
          uLongf ol = p;
          uncompress(out.data(), &ol, comp.data(), cl);
        });
      for (auto& y : th) y.join();
      report("zlib_inflate_out", T, 64, p * T, now() - t0);
    }
    printf("{\"what\": \"zlib_ratio\", \"raw\": %zu, \"comp\": %lu}\n", p, (unsigned long)cl);
  }
  return 0;
}
