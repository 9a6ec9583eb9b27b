// Host microbench for the /dev/shm restore path: pread of 1 GiB pieces on N threads with and without the
// per-64 MiB CRC32C, and the CRC32C loop alone (1 stream vs 3 interleaved streams). Build on the CPU:
//   g++ -O3 -msse4.2 -pthread tools/diag/shm_read_bench.cpp -o tools/diag/shm_read_bench
#include <fcntl.h>
#include <nmmintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static uint32_t crc1(const uint8_t* p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i + 8 <= n; i += 8) { uint64_t v; memcpy(&v, p + i, 8); c = _mm_crc32_u64(c, v); }
  return ~(uint32_t)c;
}
static uint32_t crc3(const uint8_t* p, size_t n) {  // three independent streams (throughput only)
  uint64_t a = 0xFFFFFFFFu, b = 0, c = 0;
  size_t t = n / 3 / 8 * 8;
  const uint8_t *p1 = p + t, *p2 = p + 2 * t;
  for (size_t i = 0; i < t; i += 8) {
    uint64_t x, y, z;
    memcpy(&x, p + i, 8); memcpy(&y, p1 + i, 8); memcpy(&z, p2 + i, 8);
    a = _mm_crc32_u64(a, x); b = _mm_crc32_u64(b, y); c = _mm_crc32_u64(c, z);
  }
  return (uint32_t)(a ^ b ^ c);
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/dev/shm/dlgm_read_bench";
  const int nth = argc > 2 ? atoi(argv[2]) : 16;
  const size_t piece = 1ull << 30, chunk = 64ull << 20, total = 8ull << 30;
  int fd = open(path, O_RDWR | O_CREAT, 0600);
  if (fd < 0 || ftruncate(fd, total) != 0) { perror("file"); return 1; }
  {  // fill the file (pages resident in shm)
    std::vector<uint8_t> buf(chunk, 7);
    for (size_t off = 0; off < total; off += chunk) pwrite(fd, buf.data(), chunk, off);
  }
  uint8_t* dst = (uint8_t*)aligned_alloc(4096, piece);
  memset(dst, 0, piece);
  for (int pass = 0; pass < 2; ++pass) {  // first touch through a fresh shared mapping: memcpy from the map
    // drop this process's mapping state: a new mmap each pass (page-cache pages stay resident)
    uint8_t* m = (uint8_t*)mmap(nullptr, total, PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { perror("mmap"); return 1; }
    double t0 = now();
    for (size_t off = 0; off < total; off += piece) {
      std::vector<std::thread> ts;
      for (int t = 0; t < nth; ++t)
        ts.emplace_back([&, t] {
          for (size_t c = t; c < piece / chunk; c += nth) memcpy(dst + c * chunk, m + off + c * chunk, chunk);
        });
      for (auto& th : ts) th.join();
    }
    double dt = now() - t0;
    printf("{\"mode\": \"mmap+memcpy pass %d\", \"threads\": %d, \"GBps\": %.2f}\n", pass, nth, total / dt / 1e9);
    munmap(m, total);
  }
  for (int it = 0; it < 6; ++it) {  // twice: 0 pread only, 1 pread + crc1, 2 pread + crc3
    const int mode = it % 3;
    double t0 = now();
    for (size_t off = 0; off < total; off += piece) {
      std::vector<std::thread> ts;
      for (int t = 0; t < nth; ++t)
        ts.emplace_back([&, t] {
          for (size_t c = t; c < piece / chunk; c += nth) {
            pread(fd, dst + c * chunk, chunk, off + c * chunk);
            if (mode == 1) crc1(dst + c * chunk, chunk);
            if (mode == 2) crc3(dst + c * chunk, chunk);
          }
        });
      for (auto& th : ts) th.join();
    }
    double dt = now() - t0;
    printf("{\"mode\": \"%s\", \"threads\": %d, \"GBps\": %.2f}\n", mode == 0 ? "pread" : mode == 1 ? "pread+crc1" : "pread+crc3",
           nth, total / dt / 1e9);
  }
  {  // CRC alone, one thread
    double t0 = now(); volatile uint32_t s = crc1(dst, piece); double d1 = now() - t0;
    t0 = now(); s = crc3(dst, piece); double d3 = now() - t0; (void)s;
    printf("{\"crc1_GBps_1thread\": %.2f, \"crc3_GBps_1thread\": %.2f}\n", piece / d1 / 1e9, piece / d3 / 1e9);
  }
  close(fd); unlink(path);
  return 0;
}
