// Parallel positional reader for checkpoint restore (host C++).
//
// Resume streams 48 GB of Llama-3-8B state (parameters + AdamW moments) from the
// checkpoint file into HBM. The file is usually NOT in the page cache (the writer
// uses O_DIRECT), so restoring through the mmap that torch.load(mmap=True) returns
// turns into 4 KiB page faults with kernel readahead — ~2 GB/s measured on the
// MI355X box. Here each chunk is read by a few threads with large O_DIRECT preads
// straight into pinned host memory (the HIP copy engine then moves it to HBM while
// the next chunk is read), like the save path's writer in reverse.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

namespace ftrt {

namespace {
constexpr uint64_t ALIGN = 4096;

void pread_all(int fd, uint8_t* p, uint64_t len, uint64_t off) {
  uint64_t done = 0;
  while (done < len) {
    const ssize_t n = ::pread(fd, p + done, std::min<uint64_t>(len - done, 1ull << 30), (off_t)(off + done));
    if (n < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pread: ") + strerror(errno));
    }
    if (n == 0) throw std::runtime_error("pread: unexpected end of file");
    done += (uint64_t)n;
  }
}

// O_DIRECT read of an aligned body; false if the kernel refuses it (EINVAL) before any byte.
bool pread_direct(int dfd, uint8_t* p, uint64_t len, uint64_t off) {
  uint64_t done = 0;
  while (done < len) {
    const ssize_t n = ::pread(dfd, p + done, std::min<uint64_t>(len - done, 1ull << 30), (off_t)(off + done));
    if (n < 0) {
      if (errno == EINTR) continue;
      if (errno == EINVAL && done == 0) return false;
      throw std::runtime_error(std::string("pread(O_DIRECT): ") + strerror(errno));
    }
    if (n == 0) throw std::runtime_error("pread(O_DIRECT): unexpected end of file");
    done += (uint64_t)n;
  }
  return true;
}
}  // namespace

FileReader::FileReader(const std::string& path, int nthreads, bool direct)
    : path_(path), nthreads_(std::max(1, nthreads)) {
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("open(" + path + "): " + strerror(errno));
  dfd_ = direct ? ::open(path.c_str(), O_RDONLY | O_DIRECT | O_CLOEXEC) : -1;  // -1: fs without O_DIRECT
}

FileReader::~FileReader() {
  if (dfd_ >= 0) ::close(dfd_);
  if (fd_ >= 0) ::close(fd_);
}

void FileReader::read(uint64_t off, uintptr_t ptr, uint64_t len) {
  uint8_t* dst = reinterpret_cast<uint8_t*>(ptr);
  // split into per-thread ranges at ALIGN boundaries of the file offset
  const uint64_t per = std::max<uint64_t>(ALIGN, (len / nthreads_ + ALIGN - 1) / ALIGN * ALIGN);
  std::vector<std::pair<uint64_t, uint64_t>> parts;  // (offset within the request, length)
  for (uint64_t o = 0; o < len; o += per) parts.push_back({o, std::min(per, len - o)});
  std::string err;
  std::mutex mu;
  std::atomic<uint64_t> direct{0};
  auto work = [&](uint64_t o, uint64_t n) {
    try {
      const uint64_t foff = off + o;
      uint8_t* p = dst + o;
      uint64_t body = 0;
      if (dfd_ >= 0 && foff % ALIGN == 0 && reinterpret_cast<uintptr_t>(p) % ALIGN == 0) {
        body = n / ALIGN * ALIGN;
        if (body && !pread_direct(dfd_, p, body, foff)) body = 0;
      }
      if (body) direct += body;
      if (n > body) pread_all(fd_, p + body, n - body, foff + body);
    } catch (const std::exception& ex) {
      std::lock_guard<std::mutex> g(mu);
      if (err.empty()) err = ex.what();
    }
  };
  if (parts.size() == 1) {
    work(parts[0].first, parts[0].second);
  } else {
    std::vector<std::thread> th;
    th.reserve(parts.size());
    for (const auto& pr : parts) th.emplace_back(work, pr.first, pr.second);
    for (auto& t : th) t.join();
  }
  if (!err.empty()) throw std::runtime_error(path_ + ": " + err);
  direct_bytes_ += direct.load();
  bytes_ += len;
}

}  // namespace ftrt
