// Asynchronous file I/O engine for NVMe swapping.
//
// The reference emits DeepSpeed's `offload_optimizer: {device: "nvme", buffer_count, ...}`
// (ai_engine/deepspeed_launcher.py:197-212), which DeepSpeed serves with its libaio-based
// `aio` op. Here: a persistent pool of I/O threads that executes pread/pwrite requests split into
// `block_size` pieces, so one request keeps several NVMe queues busy and several requests overlap.
// Requests are submitted without blocking and return a ticket; the caller waits on the ticket
// when it needs the data (or the buffer back). The ZeRO-Offload NVMe path (parallel/offload.py)
// keeps `buffer_count` staging slots in flight: reads of chunk i+2, host AdamW of chunk i and
// write-back of chunk i-1 all proceed at once.
//
// Files may be opened for O_DIRECT (no page-cache copy; buffers, offsets and lengths must be
// 4 KiB aligned). Every file also gets a buffered twin descriptor, which a piece whose address
// or length is not aligned falls back to, so unaligned tails need no caller-side handling and
// a filesystem without O_DIRECT (tmpfs, some overlays) works unchanged.
//
// Plain C ABI (ctypes), no HIP/torch dependency; built into _dlgm_host.so with ckpt_io.cpp.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr size_t kAlign = 4096;

struct File {
  int direct_fd = -1;    // O_DIRECT descriptor (== buffered_fd when O_DIRECT is unavailable / not asked)
  int buffered_fd = -1;
};

struct Request {
  std::atomic<int> remaining{0};
  std::atomic<int> err{0};
};

struct Piece {
  std::shared_ptr<Request> req;
  File file;
  char* buf;
  size_t len;
  off_t off;
  bool write;
};

class Engine {
 public:
  Engine(int nthreads, size_t block) : block_(block < kAlign ? kAlign : block / kAlign * kAlign) {
    if (nthreads < 1) nthreads = 1;
    for (int i = 0; i < nthreads; ++i) threads_.emplace_back([this] { worker(); });
  }
  ~Engine() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
    for (auto& kv : files_) close_file(kv.second);
  }

  int open(const char* path, bool direct, size_t size) {
    File f;
    f.buffered_fd = ::open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (f.buffered_fd < 0) return -errno;
    if (size > 0) {
      struct stat st;
      if (fstat(f.buffered_fd, &st) == 0 && (size_t)st.st_size < size && ftruncate(f.buffered_fd, size) != 0) {
        int e = errno;
        ::close(f.buffered_fd);
        return -e;
      }
    }
    f.direct_fd = f.buffered_fd;
    if (direct) {
      int d = ::open(path, O_RDWR | O_DIRECT | O_CLOEXEC);
      if (d >= 0) f.direct_fd = d;  // EINVAL on filesystems without O_DIRECT: stay buffered
    }
    std::lock_guard<std::mutex> g(mu_);
    int h = next_file_++;
    files_[h] = f;
    return h;
  }

  bool is_direct(int h) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = files_.find(h);
    return it != files_.end() && it->second.direct_fd != it->second.buffered_fd;
  }

  int close(int h, bool do_fsync) {
    File f;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = files_.find(h);
      if (it == files_.end()) return -EBADF;
      f = it->second;
      files_.erase(it);
    }
    int rc = 0;
    if (do_fsync && fsync(f.buffered_fd) != 0) rc = -errno;
    close_file(f);
    return rc;
  }

  int64_t submit(int h, char* buf, size_t n, size_t off, bool write) {
    auto req = std::make_shared<Request>();
    std::unique_lock<std::mutex> g(mu_);
    auto it = files_.find(h);
    if (it == files_.end()) return -EBADF;
    const File f = it->second;
    const size_t np = n == 0 ? 0 : (n + block_ - 1) / block_;
    req->remaining.store((int)np);
    const int64_t ticket = next_ticket_++;
    reqs_[ticket] = req;
    for (size_t i = 0; i < np; ++i) {
      const size_t o = i * block_;
      q_.push_back(Piece{req, f, buf + o, n - o < block_ ? n - o : block_, (off_t)(off + o), write});
    }
    g.unlock();
    cv_.notify_all();
    return ticket;
  }

  int wait(int64_t ticket) {
    std::unique_lock<std::mutex> g(mu_);
    auto it = reqs_.find(ticket);
    if (it == reqs_.end()) return -ENOENT;
    auto req = it->second;
    done_cv_.wait(g, [&] { return req->remaining.load() == 0; });
    reqs_.erase(ticket);
    return req->err.load();
  }

  int poll(int64_t ticket) {  // 1 done, 0 in flight, <0 unknown ticket
    std::lock_guard<std::mutex> g(mu_);
    auto it = reqs_.find(ticket);
    if (it == reqs_.end()) return -ENOENT;
    return it->second->remaining.load() == 0 ? 1 : 0;
  }

 private:
  static void close_file(const File& f) {
    if (f.direct_fd != f.buffered_fd && f.direct_fd >= 0) ::close(f.direct_fd);
    if (f.buffered_fd >= 0) ::close(f.buffered_fd);
  }

  static int run(const Piece& p) {
    const bool aligned = ((uintptr_t)p.buf % kAlign) == 0 && p.len % kAlign == 0 && p.off % kAlign == 0;
    const int fd = aligned ? p.file.direct_fd : p.file.buffered_fd;
    size_t done = 0;
    while (done < p.len) {
      ssize_t r = p.write ? pwrite(fd, p.buf + done, p.len - done, p.off + done)
                          : pread(fd, p.buf + done, p.len - done, p.off + done);
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      if (r == 0) {  // read past EOF: the file is shorter than the request -> zeros
        if (!p.write) std::memset(p.buf + done, 0, p.len - done);
        break;
      }
      done += (size_t)r;
    }
    return 0;
  }

  void worker() {
    for (;;) {
      Piece p;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        p = std::move(q_.front());
        q_.pop_front();
      }
      const int rc = run(p);
      if (rc != 0) {
        int zero = 0;
        p.req->err.compare_exchange_strong(zero, rc);
      }
      if (p.req->remaining.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(mu_);  // pairs with the predicate check in wait()
        done_cv_.notify_all();
      }
    }
  }

  const size_t block_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Piece> q_;
  std::unordered_map<int64_t, std::shared_ptr<Request>> reqs_;
  std::unordered_map<int, File> files_;
  int64_t next_ticket_ = 1;
  int next_file_ = 1;
  bool stop_ = false;
};

}  // namespace

extern "C" {

void* dlgm_aio_create(int nthreads, size_t block_size) { return new Engine(nthreads, block_size); }

void dlgm_aio_destroy(void* e) { delete static_cast<Engine*>(e); }

// Open (create; grow to `size` bytes if shorter) for swapping. Returns a handle > 0 or -errno.
int dlgm_aio_open(void* e, const char* path, int direct, size_t size) {
  return static_cast<Engine*>(e)->open(path, direct != 0, size);
}

int dlgm_aio_is_direct(void* e, int h) { return static_cast<Engine*>(e)->is_direct(h) ? 1 : 0; }

int dlgm_aio_close(void* e, int h, int do_fsync) { return static_cast<Engine*>(e)->close(h, do_fsync != 0); }

// Asynchronous pread (write=0) / pwrite (write=1) of n bytes at file offset `off`. Returns a ticket.
int64_t dlgm_aio_submit(void* e, int h, void* buf, size_t n, size_t off, int write) {
  return static_cast<Engine*>(e)->submit(h, static_cast<char*>(buf), n, off, write != 0);
}

// Block until the request finished; 0 or the first -errno of its pieces. Each ticket is waited once.
int dlgm_aio_wait(void* e, int64_t ticket) { return static_cast<Engine*>(e)->wait(ticket); }

int dlgm_aio_poll(void* e, int64_t ticket) { return static_cast<Engine*>(e)->poll(ticket); }

// Page-aligned host buffer for O_DIRECT staging (free with dlgm_aio_free).
void* dlgm_aio_alloc(size_t n) {
  void* p = nullptr;
  return posix_memalign(&p, kAlign, n < kAlign ? kAlign : n) == 0 ? p : nullptr;
}

void dlgm_aio_free(void* p) { free(p); }

}  // extern "C"
