// Host-runtime self test, built with -fsanitize=address,undefined (tests/test_host_sanitizers.py):
// CRC32C against published check values, multi-threaded write/read round trips with per-chunk
// CRCs (odd sizes, chunk tails), streamed pwrite_at pieces, and the AVX2 AdamW against a scalar
// double-precision reference on a length that exercises the vector body and the scalar tail.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

extern "C" {
uint32_t dlgm_crc32c(const void* p, size_t n, uint32_t seed);
int dlgm_write_file(const char* path, const void* ptr, size_t n, size_t chunk, int nthreads, uint32_t* crcs,
                    int do_fsync);
int dlgm_read_file(const char* path, void* ptr, size_t n, size_t chunk, int nthreads, uint32_t* crcs);
void dlgm_cpu_adamw(float* p, float* m, float* v, const float* g, uint16_t* p16, size_t n, float lr, float b1,
                    float b2, float eps, float wd, float bc1, float bc2, float gscale);
int dlgm_open_write(const char* path, size_t total);
int dlgm_pwrite_at(int fd, const void* ptr, size_t n, size_t offset, size_t chunk, int nthreads, uint32_t* crcs);
int dlgm_close_file(int fd, int do_fsync);
uint64_t dlgm_touch_pages(const void* ptr, size_t n, int nthreads);
int dlgm_populate_pages(void* ptr, size_t n, int nthreads, int write);
}

static int failures = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // CRC32C (Castagnoli) check values
  CHECK(dlgm_crc32c("123456789", 9, 0) == 0xE3069283u);
  std::vector<uint8_t> zeros(32, 0);
  CHECK(dlgm_crc32c(zeros.data(), 32, 0) == 0x8A9136AAu);
  // unaligned start / odd lengths must agree with a byte-wise split
  std::vector<uint8_t> buf(1000003);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 2654435761u >> 13);
  const uint32_t whole = dlgm_crc32c(buf.data() + 1, buf.size() - 1, 0);
  const uint32_t part = dlgm_crc32c(buf.data() + 1 + 777, buf.size() - 1 - 777, dlgm_crc32c(buf.data() + 1, 777, 0));
  CHECK(whole == part);

  // write / read round trip, 4 threads, chunk 64 KiB, size not a multiple of the chunk
  const size_t chunk = 64 << 10, n = buf.size();
  const size_t nch = (n + chunk - 1) / chunk;
  std::vector<uint32_t> wc(nch), rc(nch);
  const std::string path = dir + "/dlgm_host_selftest.bin";
  CHECK(dlgm_write_file(path.c_str(), buf.data(), n, chunk, 4, wc.data(), 0) == 0);
  std::vector<uint8_t> back(n, 0);
  CHECK(dlgm_read_file(path.c_str(), back.data(), n, chunk, 4, rc.data()) == 0);
  CHECK(std::memcmp(back.data(), buf.data(), n) == 0);
  CHECK(wc == rc);
  for (size_t i = 0; i < nch; ++i) {
    const size_t len = std::min(chunk, n - i * chunk);
    CHECK(wc[i] == dlgm_crc32c(buf.data() + i * chunk, len, 0));
  }
  // streamed pieces at chunk-aligned offsets (the checkpoint ring path)
  int fd = dlgm_open_write(path.c_str(), n);
  CHECK(fd >= 0);
  std::vector<uint32_t> pc(nch);
  for (size_t off = 0; off < n; off += 3 * chunk) {
    const size_t len = std::min(3 * chunk, n - off);
    CHECK(dlgm_pwrite_at(fd, buf.data() + off, len, off, chunk, 2, pc.data() + off / chunk) == 0);
  }
  CHECK(dlgm_close_file(fd, 0) == 0);
  std::fill(back.begin(), back.end(), 0);
  CHECK(dlgm_read_file(path.c_str(), back.data(), n, chunk, 3, rc.data()) == 0);
  CHECK(std::memcmp(back.data(), buf.data(), n) == 0);
  CHECK(pc == rc);
  std::remove(path.c_str());
  // reading a missing file fails cleanly
  CHECK(dlgm_read_file((dir + "/does_not_exist.bin").c_str(), back.data(), 16, chunk, 1, rc.data()) != 0);

  // a shared file mapping: populate (write and read advice) on threads keeps every byte, touch sums one per page;
  // the length leaves a short last 64 MiB slice
  {
    const size_t fn = (130u << 20) + 3 * 4096;
    const std::string fpath = dir + "/dlgm_host_selftest.map";
    int mfd = open(fpath.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    CHECK(mfd >= 0 && ftruncate(mfd, (off_t)fn) == 0);
    uint8_t* mp = (uint8_t*)mmap(nullptr, fn, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
    CHECK(mp != MAP_FAILED);
    if (mp != MAP_FAILED) {
      mp[0] = 3;
      mp[(64u << 20) + 4096] = 5;
      mp[fn - 4096] = 11;
      const int w = dlgm_populate_pages(mp, fn, 8, 1), r = dlgm_populate_pages(mp, fn, 3, 0);
      CHECK((w == 0 && r == 0) || (w == EINVAL && r == EINVAL));  // EINVAL: a kernel older than 5.14
      CHECK(mp[0] == 3 && mp[(64u << 20) + 4096] == 5 && mp[fn - 4096] == 11);
      CHECK(dlgm_touch_pages(mp, fn, 4) == 3 + 5 + 11);
      munmap(mp, fn);
    }
    if (mfd >= 0) close(mfd);
    std::remove(fpath.c_str());
  }

  // AdamW vs a double-precision scalar reference
  const size_t m = 8192 * 3 + 13;
  std::vector<float> p(m), mo(m), vo(m), g(m);
  std::vector<uint16_t> p16(m);
  for (size_t i = 0; i < m; ++i) {
    p[i] = std::sin(0.1 * i);
    mo[i] = 0.01f * std::cos(0.3 * i);
    vo[i] = 0.001f * (1.0f + std::sin(0.7 * i)) + 1e-6f;
    g[i] = std::cos(0.05 * i + 1.0);
  }
  std::vector<double> rp(p.begin(), p.end()), rm(mo.begin(), mo.end()), rv(vo.begin(), vo.end());
  const float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.01f, gs = 0.5f;
  const float bc1 = 1.f - std::pow(b1, 3.f), bc2 = 1.f - std::pow(b2, 3.f);
  dlgm_cpu_adamw(p.data(), mo.data(), vo.data(), g.data(), p16.data(), m, lr, b1, b2, eps, wd, bc1, bc2, gs);
  double maxerr = 0.0;
  for (size_t i = 0; i < m; ++i) {
    const double gg = (double)g[i] * gs;
    rm[i] = b1 * rm[i] + (1 - b1) * gg;
    rv[i] = b2 * rv[i] + (1 - b2) * gg * gg;
    rp[i] = rp[i] * (1 - (double)lr * wd) - (lr / bc1) * rm[i] / (std::sqrt(rv[i]) / std::sqrt(bc2) + eps);
    maxerr = std::fmax(maxerr, std::fabs(rp[i] - p[i]));
    uint32_t bits;
    std::memcpy(&bits, &p[i], 4);
    CHECK(std::abs((int)(bits >> 16) - (int)p16[i]) <= 1);  // bf16 copy = rounded fp32 master
  }
  CHECK(maxerr < 1e-6);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("host runtime self-test OK (adamw max err %.3g)\n", maxerr);
  return 0;
}
