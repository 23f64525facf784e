// regprobe -- dev probe: can the drop-in path DMA straight out of the page cache?  A page-cached
// file is mmap'ed and each 1 GiB slab hipHostRegister'ed, copied to HBM and unregistered; the
// pread-into-pinned-staging copy the fd pipeline does now is timed beside it.
// Build: hipcc -O2 -o tools/probes/regprobe tools/probes/regprobe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); } } while (0)

int main(int argc, char **argv) {
  const char *path = argc > 1 ? argv[1] : "/tmp/regprobe.bin";
  const size_t G = 1ull << 30, N = 4 * G;
  {  // the file, then read once so it is page-cached
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    std::vector<char> buf(64 << 20, 'A');
    for (size_t o = 0; o < N; o += buf.size()) if (write(fd, buf.data(), buf.size()) != (ssize_t)buf.size()) return 1;
    close(fd);
    fd = open(path, O_RDONLY);
    for (size_t o = 0; o < N; o += buf.size()) if (pread(fd, buf.data(), buf.size(), o) <= 0) return 1;
    close(fd);
  }
  void *d = nullptr;
  CK(hipMalloc(&d, G));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int fd = open(path, O_RDONLY);
  char *m = (char *)mmap(nullptr, N, PROT_READ, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) { printf("mmap failed\n"); return 1; }
  for (unsigned flags : {0u, 0x8u}) {
    for (size_t k = 0; k < N / G; ++k) {
      char *p = m + k * G;
      const double t0 = now();
      hipError_t e = hipHostRegister(p, G, flags);
      const double t1 = now();
      if (e != hipSuccess) { printf("flags %u slab %zu: hipHostRegister: %s\n", flags, k, hipGetErrorString(e)); (void)hipGetLastError(); break; }
      CK(hipMemcpyAsync(d, p, G, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      const double t2 = now();
      CK(hipHostUnregister(p));
      const double t3 = now();
      printf("flags %u slab %zu: register %.1f ms (%.1f GB/s)  H2D %.1f ms (%.1f GB/s)  unregister %.1f ms\n", flags, k,
             (t1 - t0) * 1e3, G / (t1 - t0) / 1e9, (t2 - t1) * 1e3, G / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
    }
  }
  // the current path: pread by 16 threads into pinned staging (64 MiB pieces), then H2D
  char *h = nullptr;
  CK(hipHostMalloc((void **)&h, G, 0));
  for (size_t k = 0; k < 2; ++k) {
    const double t0 = now();
    std::vector<std::thread> th;
    for (int i = 0; i < 16; ++i)
      th.emplace_back([&, i] {
        for (size_t o = (size_t)i * (64 << 20); o < G; o += 16ull * (64 << 20)) (void)!pread(fd, h + o, 64 << 20, k * G + o);
      });
    for (auto &t : th) t.join();
    const double t1 = now();
    CK(hipMemcpyAsync(d, h, G, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    const double t2 = now();
    printf("pread x16 into pinned: %.1f ms (%.1f GB/s)  H2D %.1f ms (%.1f GB/s)\n", (t1 - t0) * 1e3, G / (t1 - t0) / 1e9,
           (t2 - t1) * 1e3, G / (t2 - t1) / 1e9);
  }
  munmap(m, N);
  close(fd);
  unlink(path);
  return 0;
}
