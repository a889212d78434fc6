// Pure C++ core of the host runtime (no Python, no torch, no HIP): included by the pybind11 module
// (runtime.cpp) and by the sanitizer self-test (selftest.cpp, built with -fsanitize=address /
// undefined / thread on the host). See runtime.cpp for the component overview.
#pragma once
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace cmlrt {

// ============================================================================ RecordLoader
class RecordLoader {
 public:
  RecordLoader(const std::string& path, int64_t record_bytes, int64_t batch, int64_t rank,
               int64_t world, uint64_t seed, int threads, bool drop_last)
      : rec_(record_bytes), batch_(batch), rank_(rank), world_(world), seed_(seed),
        threads_(std::max(1, threads)), drop_last_(drop_last) {
    if (record_bytes <= 0 || batch <= 0 || world <= 0 || rank < 0 || rank >= world)
      throw std::invalid_argument("RecordLoader: bad geometry");
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("RecordLoader: cannot open " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) throw std::runtime_error("RecordLoader: stat failed");
    size_ = static_cast<size_t>(st.st_size);
    if (size_ == 0 || size_ % static_cast<size_t>(rec_))
      throw std::runtime_error("RecordLoader: file size is not a positive multiple of record size");
    void* m = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (m == MAP_FAILED) throw std::runtime_error("RecordLoader: mmap failed");
    base_ = static_cast<const uint8_t*>(m);
    ::madvise(m, size_, MADV_RANDOM);
    n_ = static_cast<int64_t>(size_ / static_cast<size_t>(rec_));
    if (n_ < world_) throw std::runtime_error("RecordLoader: fewer records than ranks");
  }
  ~RecordLoader() {
    stop();
    if (base_) ::munmap(const_cast<uint8_t*>(base_), size_);
    if (fd_ >= 0) ::close(fd_);
  }

  int64_t num_records() const { return n_; }
  int64_t batches_per_epoch() const {
    const int64_t share = n_ / world_;
    return drop_last_ ? share / batch_ : (share + batch_ - 1) / batch_;
  }

  // Record indices of (epoch, batch b) for this rank — also exposed for tests.
  std::vector<int64_t> batch_indices(int64_t epoch, int64_t b) {
    std::lock_guard<std::mutex> lk(perm_mu_);
    const std::vector<int64_t>& p = perm(epoch);
    const int64_t share = n_ / world_;
    const int64_t lo = rank_ * share + b * batch_;
    const int64_t hi = std::min(lo + batch_, (rank_ + 1) * share);
    return std::vector<int64_t>(p.begin() + lo, p.begin() + std::max(lo, hi));
  }

  void start(const std::vector<uintptr_t>& slots, int64_t slot_bytes, int64_t epoch0) {
    std::lock_guard<std::mutex> lk(mu_);
    if (running_) throw std::runtime_error("RecordLoader already running");
    if (slots.empty()) throw std::invalid_argument("RecordLoader: no slots");
    if (slot_bytes < batch_ * rec_) throw std::invalid_argument("RecordLoader: slot buffer too small");
    if (batches_per_epoch() <= 0) throw std::runtime_error("RecordLoader: empty epoch");
    slots_ = slots;
    const size_t S = slots.size();
    ready_ticket_.assign(S, -1);
    rows_.assign(S, 0);
    epoch_of_.assign(S, 0);
    free_.assign(S, 1);
    epoch0_ = epoch0;
    claim_ = 0;
    take_ = 0;
    running_ = true;
    for (int t = 0; t < threads_; ++t) pool_.emplace_back([this] { work(); });
  }

  struct Batch {
    int64_t slot, rows, epoch, ticket;
  };
  // Next batch in ticket order (blocks until the workers have filled it).
  Batch next_batch() {
    std::unique_lock<std::mutex> lk(mu_);
    const int64_t t = take_;
    const size_t s = static_cast<size_t>(t % static_cast<int64_t>(slots_.size()));
    cv_.wait(lk, [&] { return !running_ || ready_ticket_[s] == t; });
    if (ready_ticket_[s] != t) throw std::runtime_error("RecordLoader stopped");
    ready_ticket_[s] = -1;
    ++take_;
    return Batch{static_cast<int64_t>(s), rows_[s], epoch_of_[s], t};
  }

  void release(int64_t slot) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.at(static_cast<size_t>(slot)) = 1;
    }
    cv_.notify_all();
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      running_ = false;
    }
    cv_.notify_all();
    for (auto& th : pool_)
      if (th.joinable()) th.join();
    pool_.clear();
  }

 private:
  const std::vector<int64_t>& perm(int64_t epoch) {   // perm_mu_ held
    auto it = perms_.find(epoch);
    if (it != perms_.end()) return it->second;
    while (perms_.size() >= 3) perms_.erase(perms_.begin());
    std::vector<int64_t> p(static_cast<size_t>(n_));
    std::iota(p.begin(), p.end(), 0);
    std::mt19937_64 rng(seed_ * 0x9E3779B97F4A7C15ull ^ (static_cast<uint64_t>(epoch) + 1) * 0xBF58476D1CE4E5B9ull);
    std::shuffle(p.begin(), p.end(), rng);
    return perms_.emplace(epoch, std::move(p)).first->second;
  }

  void work() {
    const int64_t per = batches_per_epoch();
    const size_t S = slots_.size();
    for (;;) {
      int64_t t;
      size_t s;
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (!running_) return;
        t = claim_++;
        s = static_cast<size_t>(t % static_cast<int64_t>(S));
        // slot s is reusable once its previous ticket (t - S) was taken and released
        cv_.wait(lk, [&] { return !running_ || (free_[s] && take_ >= t - static_cast<int64_t>(S) + 1 &&
                                                ready_ticket_[s] == -1); });
        if (!running_) return;
        free_[s] = 0;
      }
      const int64_t ep = epoch0_ + t / per;
      const std::vector<int64_t> idx = batch_indices(ep, t % per);
      uint8_t* dst = reinterpret_cast<uint8_t*>(slots_[s]);
      for (size_t k = 0; k < idx.size(); ++k)
        std::memcpy(dst + k * static_cast<size_t>(rec_), base_ + idx[k] * rec_,
                    static_cast<size_t>(rec_));
      {
        std::lock_guard<std::mutex> lk(mu_);
        rows_[s] = static_cast<int64_t>(idx.size());
        epoch_of_[s] = ep;
        ready_ticket_[s] = t;
      }
      cv_.notify_all();
    }
  }

  int fd_ = -1;
  size_t size_ = 0;
  const uint8_t* base_ = nullptr;
  int64_t n_ = 0, rec_, batch_, rank_, world_;
  uint64_t seed_;
  int threads_;
  bool drop_last_;

  std::mutex mu_;
  std::condition_variable cv_;
  bool running_ = false;
  std::vector<uintptr_t> slots_;
  std::vector<int64_t> ready_ticket_, rows_, epoch_of_;
  std::vector<char> free_;
  int64_t epoch0_ = 0, claim_ = 0, take_ = 0;
  std::vector<std::thread> pool_;

  std::mutex perm_mu_;
  std::map<int64_t, std::vector<int64_t>> perms_;
};

// ============================================================================ Watchdog
class Watchdog {
 public:
  Watchdog(double timeout_s, const std::string& report_path, bool hard_abort)
      : timeout_(timeout_s), report_(report_path), abort_(hard_abort) {
    last_ = now();
    th_ = std::thread([this] { run(); });
  }
  ~Watchdog() { stop(); }

  void beat(int64_t step) {
    step_.store(step);
    last_.store(now());
  }
  void set_phase(const std::string& p) {
    std::lock_guard<std::mutex> lk(mu_);
    phase_ = p;
  }
  bool fired() const { return fired_.load(); }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

 private:
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      // system_clock deadline -> pthread_cond_timedwait (wait_for's steady-clock path uses
      // pthread_cond_clockwait, which gcc-11 ThreadSanitizer does not intercept)
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100));
      if (stop_) break;
      const double idle = now() - last_.load();
      if (idle > timeout_ && !fired_.load()) {
        fired_ = true;
        if (!report_.empty()) {
          std::ofstream o(report_, std::ios::app);
          o << "{\"event\": \"watchdog\", \"idle_s\": " << idle << ", \"step\": " << step_.load()
            << ", \"phase\": \"" << phase_ << "\", \"pid\": " << ::getpid() << "}\n";
        }
        std::fprintf(stderr, "[consensusml watchdog] no progress for %.1f s at step %lld (phase %s)\n",
                     idle, static_cast<long long>(step_.load()), phase_.c_str());
        if (abort_) {
          std::fflush(stderr);
          ::kill(::getpid(), SIGABRT);
        }
      }
    }
  }
  double timeout_;
  std::string report_;
  bool abort_;
  std::atomic<double> last_{0.0};
  std::atomic<int64_t> step_{0};
  std::atomic<bool> fired_{false};
  std::string phase_ = "init";
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::thread th_;
};

// ============================================================================ helpers
struct BucketPlan {
  std::vector<int64_t> offsets, lengths, shards, param_offsets, param_bucket;
  int64_t total = 0, shard_total = 0;
};

// Parameters in the given order; a bucket closes when adding the next parameter would exceed
// bucket_elems; every parameter is padded to 8 elements; buckets to a multiple of world*align.
inline BucketPlan plan_buckets(const std::vector<int64_t>& numels, int64_t world, int64_t align,
                        int64_t bucket_elems) {
  BucketPlan p;
  p.param_offsets.assign(numels.size(), 0);
  p.param_bucket.assign(numels.size(), 0);
  const int64_t unit = world * align;
  int64_t off = 0, cur = 0, count = 0;
  auto close = [&]() {
    if (count == 0) return;
    const int64_t L = (cur + unit - 1) / unit * unit;
    p.offsets.push_back(off);
    p.lengths.push_back(L);
    p.shards.push_back(L / world);
    off += L;
    p.shard_total += L / world;
    cur = 0;
    count = 0;
  };
  for (size_t i = 0; i < numels.size(); ++i) {
    if (count && cur + numels[i] > bucket_elems) close();
    p.param_offsets[i] = off + cur;
    p.param_bucket[i] = static_cast<int64_t>(p.offsets.size());
    cur += (numels[i] + 7) / 8 * 8;
    ++count;
  }
  close();
  p.total = off;
  return p;
}

inline uint32_t crc32_update(uint32_t crc, const uint8_t* d, size_t n) {
  static uint32_t table[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
  });
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ d[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

inline uint32_t crc32_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("crc32_file: cannot open " + path);
  std::vector<char> buf(1 << 20);
  uint32_t crc = 0;
  while (f) {
    f.read(buf.data(), static_cast<std::streamsize>(buf.size()));
    const std::streamsize got = f.gcount();
    if (got > 0) crc = crc32_update(crc, reinterpret_cast<const uint8_t*>(buf.data()), static_cast<size_t>(got));
  }
  return crc;
}

inline void write_file_atomic(const std::string& path, const std::string& s) {
  const std::string tmp = path + ".tmp." + std::to_string(::getpid());
  {
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw std::runtime_error("write_file_atomic: cannot create " + tmp);
    size_t done = 0;
    while (done < s.size()) {
      const ssize_t w = ::write(fd, s.data() + done, s.size() - done);
      if (w <= 0) {
        ::close(fd);
        throw std::runtime_error("write_file_atomic: write failed");
      }
      done += static_cast<size_t>(w);
    }
    ::fsync(fd);
    ::close(fd);
  }
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("write_file_atomic: rename failed");
}

// One CSV table in R write.csv style: quoted header / row names, cells already formatted.
inline std::string format_csv(const std::vector<std::string>& row_names,
                              const std::vector<std::string>& col_names,
                              const std::vector<std::vector<std::string>>& cells) {
  const size_t n = row_names.size();
  std::string out = "\"\"";
  for (auto& c : col_names) out += ",\"" + c + "\"";
  out += "\n";
  for (size_t i = 0; i < n; ++i) {
    out += "\"" + row_names[i] + "\"";
    for (size_t c = 0; c < cells.size(); ++c) out += "," + cells[c][i];
    out += "\n";
  }
  return out;
}

inline std::string format_number(double v) {   // NaN -> NA like R
  if (v != v) return "NA";
  char b[64];
  std::snprintf(b, sizeof(b), "%.15g", v);
  return b;
}

}  // namespace cmlrt
