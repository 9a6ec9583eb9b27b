// AIO engine self-test (csrc/host/aio.cpp), run under ASan+UBSan and under ThreadSanitizer by
// tests/test_host_sanitizers.py: several submitter threads, each with its own file, overlapping
// async writes and reads split into small pieces across the I/O pool, O_DIRECT + buffered twins,
// poll/wait, and an engine destroyed while requests are still queued.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* dlgm_aio_create(int nthreads, size_t block_size);
void dlgm_aio_destroy(void* e);
int dlgm_aio_open(void* e, const char* path, int direct, size_t size);
int dlgm_aio_close(void* e, int h, int do_fsync);
int64_t dlgm_aio_submit(void* e, int h, void* buf, size_t n, size_t off, int write);
int dlgm_aio_wait(void* e, int64_t ticket);
int dlgm_aio_poll(void* e, int64_t ticket);
void* dlgm_aio_alloc(size_t n);
void dlgm_aio_free(void* p);
}

static std::atomic<int>* g_fail;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail->fetch_add(1);                                             \
    }                                                                   \
  } while (0)

int main(int argc, char** argv) {
  std::atomic<int> fails{0};
  g_fail = &fails;
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  void* e = dlgm_aio_create(4, 4096);
  constexpr int kSubmitters = 4;
  constexpr size_t kBytes = (1 << 18) + 4096 * 3 + 100;  // ragged tail -> buffered fallback piece
  std::vector<std::thread> th;
  for (int t = 0; t < kSubmitters; ++t) {
    th.emplace_back([&, t] {
      const std::string path = dir + "/aio_" + std::to_string(t);
      const int h = dlgm_aio_open(e, path.c_str(), t % 2, kBytes);
      CHECK(h > 0);
      auto* src = static_cast<uint8_t*>(dlgm_aio_alloc(kBytes));
      auto* dst = static_cast<uint8_t*>(dlgm_aio_alloc(kBytes));
      for (int round = 0; round < 3; ++round) {
        for (size_t i = 0; i < kBytes; ++i) src[i] = (uint8_t)(i * 31 + t * 7 + round);
        // two halves in flight at once, then read both back concurrently
        const size_t half = (kBytes / 2) / 4096 * 4096;
        int64_t w0 = dlgm_aio_submit(e, h, src, half, 0, 1);
        int64_t w1 = dlgm_aio_submit(e, h, src + half, kBytes - half, half, 1);
        CHECK(w0 > 0 && w1 > 0);
        CHECK(dlgm_aio_wait(e, w0) == 0);
        CHECK(dlgm_aio_wait(e, w1) == 0);
        std::memset(dst, 0, kBytes);
        int64_t r0 = dlgm_aio_submit(e, h, dst + half, kBytes - half, half, 0);
        int64_t r1 = dlgm_aio_submit(e, h, dst, half, 0, 0);
        while (dlgm_aio_poll(e, r0) == 0) std::this_thread::yield();
        CHECK(dlgm_aio_wait(e, r0) == 0);
        CHECK(dlgm_aio_wait(e, r1) == 0);
        CHECK(std::memcmp(src, dst, kBytes) == 0);
      }
      CHECK(dlgm_aio_wait(e, 1 << 30) < 0);  // unknown ticket
      CHECK(dlgm_aio_close(e, h, 1) == 0);
      dlgm_aio_free(src);
      dlgm_aio_free(dst);
      std::remove(path.c_str());
    });
  }
  for (auto& x : th) x.join();
  // destroy with work still queued: the pool drains it before joining
  const std::string path = dir + "/aio_tail";
  const int h = dlgm_aio_open(e, path.c_str(), 0, 0);
  std::vector<uint8_t> buf(1 << 16, 3);
  for (int i = 0; i < 8; ++i) dlgm_aio_submit(e, h, buf.data(), buf.size(), (size_t)i << 16, 1);
  dlgm_aio_destroy(e);
  std::remove(path.c_str());
  if (fails.load()) {
    std::fprintf(stderr, "%d failure(s)\n", fails.load());
    return 1;
  }
  std::printf("aio self-test OK\n");
  return 0;
}
