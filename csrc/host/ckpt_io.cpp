// Host runtime for the checkpoint path and CPU-side optimizer.
//
//  * dlgm_write_file / dlgm_read_file: multi-threaded pwrite/pread of one large buffer
//    (a pinned host snapshot of a rank's ZeRO shard) in fixed-size chunks, computing a
//    CRC32C per chunk on the fly (SSE4.2 crc32 instruction) so the manifest can prove
//    the checkpoint intact on restore; fsync before returning so a published tag is on
//    disk. Called from a Python background thread through ctypes (the GIL is released
//    for the whole call), i.e. completely off the training critical path.
//  * dlgm_cpu_adamw: AVX2/FMA AdamW over fp32 master/m/v with bf16 write-back, OpenMP
//    parallel -- the ZeRO-Offload optimizer (reference preset offload_optimizer=cpu).
//
// Plain C ABI, no HIP/torch dependency: built with g++ into _dlgm_host.so.
#include <errno.h>
#include <fcntl.h>
#include <immintrin.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>
#include <vector>

namespace {

uint32_t crc32c_sw_table[256];
bool crc_init = false;

void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    crc32c_sw_table[i] = c;
  }
  crc_init = true;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}

uint32_t crc32c_sw(const uint8_t* p, size_t n, uint32_t crc) {
  if (!crc_init) init_table();
  uint32_t c = ~crc;
  while (n--) c = crc32c_sw_table[(c ^ *p++) & 0xFF] ^ (c >> 8);
  return ~c;
}

bool have_sse42() { return __builtin_cpu_supports("sse4.2"); }

// pwrite/pread `n` bytes of `buf` at file offset `file_off` in `chunk`-byte pieces on `nthreads` threads.
// Per chunk (relative to `buf`): CRC32C into `crcs` (our manifests) and, when `zcrcs` is given, the zip
// CRC-32 (zlib polynomial) that a torch-zip (.pt) record header carries -- combined by the caller.
int run_chunks(int fd, uint8_t* buf, size_t n, size_t file_off, size_t chunk, int nthreads, uint32_t* crcs,
               uint32_t* zcrcs, bool write) {
  const size_t nchunks = (n + chunk - 1) / chunk;
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  const bool hw = have_sse42();
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nchunks || err.load()) return;
      const size_t off = i * chunk;
      const size_t len = std::min(chunk, n - off);
      size_t done = 0;
      if (write && crcs) crcs[i] = hw ? crc32c_hw(buf + off, len, 0) : crc32c_sw(buf + off, len, 0);
      if (write && zcrcs) zcrcs[i] = (uint32_t)crc32_z(0L, buf + off, len);
      while (done < len) {
        ssize_t r = write ? pwrite(fd, buf + off + done, len - done, (off_t)(file_off + off + done))
                          : pread(fd, buf + off + done, len - done, (off_t)(file_off + off + done));
        if (r < 0) {
          if (errno == EINTR) continue;
          err.store(-errno);
          return;
        }
        if (r == 0) {
          err.store(-EIO);
          return;
        }
        done += (size_t)r;
      }
      if (!write && crcs) crcs[i] = hw ? crc32c_hw(buf + off, len, 0) : crc32c_sw(buf + off, len, 0);
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)nchunks));
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  return err.load();
}

inline float bf16_to_f32(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // keep NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace

extern "C" {

uint32_t dlgm_crc32c(const void* p, size_t n, uint32_t seed) {
  return have_sse42() ? crc32c_hw((const uint8_t*)p, n, seed) : crc32c_sw((const uint8_t*)p, n, seed);
}

int dlgm_write_file(const char* path, const void* ptr, size_t n, size_t chunk, int nthreads, uint32_t* crcs,
                    int do_fsync) {
  int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return -errno;
  if (n && ftruncate(fd, (off_t)n) != 0) {
    int e = -errno;
    close(fd);
    return e;
  }
  int rc = run_chunks(fd, (uint8_t*)ptr, n, 0, chunk, nthreads, crcs, nullptr, true);
  if (rc == 0 && do_fsync && fsync(fd) != 0) rc = -errno;
  if (close(fd) != 0 && rc == 0) rc = -errno;
  return rc;
}

int dlgm_read_file(const char* path, void* ptr, size_t n, size_t chunk, int nthreads, uint32_t* crcs) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < n) {
    close(fd);
    return -EIO;
  }
  int rc = run_chunks(fd, (uint8_t*)ptr, n, 0, chunk, nthreads, crcs, nullptr, false);
  close(fd);
  return rc;
}

// pread of `n` bytes starting at `file_off` (a tensor record inside a .pt zip), per-chunk CRC32C.
int dlgm_read_file_at(const char* path, void* ptr, size_t n, size_t file_off, size_t chunk, int nthreads,
                      uint32_t* crcs) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < file_off + n) {
    close(fd);
    return -EIO;
  }
  int rc = run_chunks(fd, (uint8_t*)ptr, n, file_off, chunk, nthreads, crcs, nullptr, false);
  close(fd);
  return rc;
}

// pwrite at an arbitrary file offset with per-chunk CRC32C and zip CRC-32 (either list may be null).
int dlgm_pwrite_at2(int fd, const void* ptr, size_t n, size_t file_off, size_t chunk, int nthreads, uint32_t* crcs,
                    uint32_t* zcrcs) {
  return run_chunks(fd, (uint8_t*)ptr, n, file_off, chunk, nthreads, crcs, zcrcs, true);
}

// zip CRC-32 of B appended to A, from crc(A), crc(B) and len(B) (zlib crc32_combine).
uint32_t dlgm_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return (uint32_t)crc32_combine64(crc_a, crc_b, (z_off64_t)len_b);
}

// zip CRC-32 of a small buffer (headers / pickles).
uint32_t dlgm_crc32_zip(const void* p, size_t n) { return (uint32_t)crc32_z(0L, (const Bytef*)p, n); }

// Per-chunk CRC32C of an in-memory buffer on `nthreads` threads (verifying a /dev/shm snapshot tier).
void dlgm_crc32c_chunks(const void* ptr, size_t n, size_t chunk, int nthreads, uint32_t* crcs) {
  const size_t nchunks = (n + chunk - 1) / chunk;
  std::atomic<size_t> next{0};
  const bool hw = have_sse42();
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nchunks) return;
      const uint8_t* b = (const uint8_t*)ptr + i * chunk;
      const size_t len = std::min(chunk, n - i * chunk);
      crcs[i] = hw ? crc32c_hw(b, len, 0) : crc32c_sw(b, len, 0);
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<size_t>(nchunks, 1)));
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
}

// Map the n bytes at ptr (a MAP_SHARED view of a reserved /dev/shm file) into this process by reading one byte
// per 4 KiB page on `nthreads` threads, 16 MiB slices handed out in order. A reserved tmpfs page is zeroed on its
// first touch, not by posix_fallocate, so this is where a fresh snapshot file's pages are cleared; one thread
// ran that at ~5.4 GB/s on the MI355X host, eight at ~10 GB/s. Returns the byte sum (keeps the reads).
uint64_t dlgm_touch_pages(const void* ptr, size_t n, int nthreads) {
  constexpr size_t kSlice = 16u << 20, kPage = 4096;
  const size_t nslices = (n + kSlice - 1) / kSlice;
  std::atomic<size_t> next{0};
  std::atomic<uint64_t> total{0};
  auto worker = [&]() {
    uint64_t s = 0;
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nslices) break;
      const volatile uint8_t* b = (const volatile uint8_t*)ptr + i * kSlice;
      const size_t len = std::min(kSlice, n - i * kSlice);
      for (size_t o = 0; o < len; o += kPage) s += b[o];
    }
    total.fetch_add(s);
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<size_t>(nslices, 1)));
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  return total.load();
}

// Map the pages of [ptr, ptr + n) (a shared /dev/shm file mapping) WRITABLE into this process on `nthreads`
// threads: madvise(MADV_POPULATE_WRITE) over 64 MiB slices. On the MI355X host (24 GiB of a reserved snapshot
// file) this maps at 64 GB/s on 8-16 threads where touching one byte per page ran at 13-14 GB/s on any number of
// threads, and the page-lock (hipHostRegister) of pages mapped this way runs at 118-133 GB/s instead of 37-41 GB/s
// (no write upgrade of read-mapped pages): profiles/shm_map_bench_r06.json. write = 0: MADV_POPULATE_READ instead.
// Returns 0, or the errno of the first failed slice (EINVAL on kernels older than 5.14: the caller touches instead).
int dlgm_populate_pages(void* ptr, size_t n, int nthreads, int write) {
  constexpr size_t kSlice = 64u << 20;
  const int advice = write ? 23 : 22;  // MADV_POPULATE_WRITE / MADV_POPULATE_READ (Linux 5.14)
  const size_t nslices = (n + kSlice - 1) / kSlice;
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nslices || err.load()) break;
      const size_t len = std::min(kSlice, n - i * kSlice);
      if (madvise((char*)ptr + i * kSlice, len, advice) != 0) {
        int e = errno, zero = 0;
        err.compare_exchange_strong(zero, e);
      }
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<size_t>(nslices, 1)));
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  return err.load();
}

// dst <- src (n bytes) on `nthreads` threads in `chunk` pieces, with the CRC32C of every chunk of the copied
// bytes. Used to restore from a memory-mapped /dev/shm snapshot: first touch of the shared pages through the
// mapping runs at ~90 GB/s on 16 threads where pread of the same never-read pages ran at ~16 GB/s.
void dlgm_copy_crc32c_chunks(const void* src, void* dst, size_t n, size_t chunk, int nthreads, uint32_t* crcs) {
  const size_t nchunks = (n + chunk - 1) / chunk;
  std::atomic<size_t> next{0};
  const bool hw = have_sse42();
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nchunks) return;
      const size_t len = std::min(chunk, n - i * chunk);
      const uint8_t* a = (const uint8_t*)src + i * chunk;
      uint8_t* b = (uint8_t*)dst + i * chunk;
      // copy and checksum in 1 MiB steps so the checksum reads the copy while it is still in cache
      uint32_t c = 0;
      for (size_t o = 0; o < len; o += (1u << 20)) {
        const size_t l = std::min<size_t>(1u << 20, len - o);
        memcpy(b + o, a + o, l);
        if (crcs) c = hw ? crc32c_hw(b + o, l, c) : crc32c_sw(b + o, l, c);
      }
      if (crcs) crcs[i] = c;
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<size_t>(nchunks, 1)));
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
}

// AdamW on host fp32 state (ZeRO-Offload). g may be pre-scaled; gscale multiplies it.
void dlgm_cpu_adamw(float* p, float* m, float* v, const float* g, uint16_t* p16, size_t n, float lr, float b1,
                    float b2, float eps, float wd, float bc1, float bc2, float gscale) {
  const float decay = 1.f - lr * wd;
  const float step_size = lr / bc1;
  const float isb2 = 1.f / std::sqrt(bc2);
#pragma omp parallel for schedule(static)
  for (size_t blk = 0; blk < (n + 8191) / 8192; ++blk) {
    const size_t s = blk * 8192, e = std::min(n, s + 8192);
    size_t i = s;
#if defined(__AVX2__) && defined(__FMA__)
    const __m256 vb1 = _mm256_set1_ps(b1), vb2 = _mm256_set1_ps(b2), v1b1 = _mm256_set1_ps(1.f - b1),
                 v1b2 = _mm256_set1_ps(1.f - b2), vdec = _mm256_set1_ps(decay), vss = _mm256_set1_ps(step_size),
                 visb2 = _mm256_set1_ps(isb2), veps = _mm256_set1_ps(eps), vgs = _mm256_set1_ps(gscale);
    for (; i + 8 <= e; i += 8) {
      __m256 gg = _mm256_mul_ps(_mm256_loadu_ps(g + i), vgs);
      __m256 mm = _mm256_fmadd_ps(vb1, _mm256_loadu_ps(m + i), _mm256_mul_ps(v1b1, gg));
      __m256 vv = _mm256_fmadd_ps(vb2, _mm256_loadu_ps(v + i), _mm256_mul_ps(v1b2, _mm256_mul_ps(gg, gg)));
      __m256 den = _mm256_fmadd_ps(_mm256_sqrt_ps(vv), visb2, veps);
      __m256 pp = _mm256_sub_ps(_mm256_mul_ps(_mm256_loadu_ps(p + i), vdec), _mm256_div_ps(_mm256_mul_ps(vss, mm), den));
      _mm256_storeu_ps(m + i, mm);
      _mm256_storeu_ps(v + i, vv);
      _mm256_storeu_ps(p + i, pp);
    }
#endif
    for (; i < e; ++i) {
      const float gg = g[i] * gscale;
      m[i] = b1 * m[i] + (1.f - b1) * gg;
      v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
      p[i] = p[i] * decay - step_size * m[i] / (std::sqrt(v[i]) * isb2 + eps);
    }
    if (p16)
      for (size_t j = s; j < e; ++j) p16[j] = f32_to_bf16(p[j]);
  }
}

// Incremental writer for snapshots streamed through a small pinned ring: open once, write
// chunk-aligned pieces at their file offsets (CRC per 64 MiB file chunk), close (+fsync).
int dlgm_open_write(const char* path, size_t total) {
  int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return -errno;
  if (total && ftruncate(fd, (off_t)total) != 0) {
    int e = -errno;
    close(fd);
    return e;
  }
  return fd;
}

int dlgm_pwrite_at(int fd, const void* ptr, size_t n, size_t offset, size_t chunk, int nthreads, uint32_t* crcs) {
  // `offset` must be a multiple of `chunk` so the CRC list composes across calls
  const size_t nchunks = (n + chunk - 1) / chunk;
  std::atomic<size_t> next{0};
  std::atomic<int> err{0};
  const bool hw = have_sse42();
  auto worker = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= nchunks || err.load()) return;
      const size_t off = i * chunk, len = std::min(chunk, n - off);
      const uint8_t* b = (const uint8_t*)ptr + off;
      if (crcs) crcs[i] = hw ? crc32c_hw(b, len, 0) : crc32c_sw(b, len, 0);
      size_t done = 0;
      while (done < len) {
        ssize_t r = pwrite(fd, b + done, len - done, (off_t)(offset + off + done));
        if (r < 0) {
          if (errno == EINTR) continue;
          err.store(-errno);
          return;
        }
        done += (size_t)r;
      }
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)nchunks));
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  return err.load();
}

int dlgm_close_file(int fd, int do_fsync) {
  int rc = 0;
  if (do_fsync && fsync(fd) != 0) rc = -errno;
  if (close(fd) != 0 && rc == 0) rc = -errno;
  return rc;
}

int dlgm_host_abi_version() { return 2; }
}
