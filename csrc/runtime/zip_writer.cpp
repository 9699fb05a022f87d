// Native writer for PyTorch-format (zip) checkpoints.
//
// The reference writes its checkpoint with a synchronous torch.save straight to
// the final path (reference utils.py:74-80; ~33.6 s for 48 GB, non-atomic —
// SURVEY.md §A.6). This writer keeps the same on-disk format (a torch.load-able
// zip: archive/data.pkl + archive/data/<key> storages, 64-B aligned, zip64) but
// writes from host memory with a thread pool that checksums and pwrite()s
// 64 MiB chunks in parallel, then publishes atomically (fsync + rename + dir
// fsync). data.pkl is produced by torch's own pickler in Python.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <hip/hip_runtime_api.h>

#include "runtime.h"

namespace ftrt {
namespace {

constexpr uint64_t U32MAX = 0xFFFFFFFFull;
constexpr uint64_t ALIGN = 64;
// Large storages start on a 4 KiB file offset so their bytes can be written with
// O_DIRECT straight from the pinned snapshot (no page-cache copy, no writeback
// storm at fsync). 4096 is a multiple of the 64 B torch.load expects.
constexpr uint64_t DIRECT_ALIGN = 4096;
constexpr uint64_t DIRECT_MIN = 1ull << 20;
constexpr uint16_t DOS_TIME = 0;
constexpr uint16_t DOS_DATE = (0 << 9) | (1 << 5) | 1;  // 1980-01-01

struct Buf {
  std::string s;
  void u16(uint16_t v) { s.append(reinterpret_cast<const char*>(&v), 2); }
  void u32(uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
  void u64(uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
  void str(const std::string& v) { s.append(v); }
};

void pwrite_all(int fd, const void* p, uint64_t n, uint64_t off) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    ssize_t w = ::pwrite(fd, c, n > (1ull << 30) ? (1ull << 30) : n, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pwrite failed: ") + strerror(errno));
    }
    c += w;
    n -= (uint64_t)w;
    off += (uint64_t)w;
  }
}

// O_DIRECT write of an aligned body; false if the kernel/filesystem rejects it.
bool pwrite_direct(int fd, const uint8_t* p, uint64_t n, uint64_t off) {
  while (n > 0) {
    const uint64_t k = n > (1ull << 30) ? (1ull << 30) : n;
    ssize_t w = ::pwrite(fd, p, k, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EINVAL) return false;
      throw std::runtime_error(std::string("pwrite(O_DIRECT) failed: ") + strerror(errno));
    }
    if ((uint64_t)w % DIRECT_ALIGN) throw std::runtime_error("short unaligned O_DIRECT write");
    p += w;
    n -= (uint64_t)w;
    off += (uint64_t)w;
  }
  return true;
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string dirname_of(const std::string& p) {
  auto pos = p.find_last_of('/');
  if (pos == std::string::npos) return ".";
  if (pos == 0) return "/";
  return p.substr(0, pos);
}

}  // namespace

uint64_t write_pieces_fd(int fd, int dfd, std::vector<FilePiece>& pieces, int nthreads, uint64_t chunk) {
  // split into <= chunk work items so the pool stays balanced
  struct Item {
    size_t piece;
    uint64_t off, len;
    uint32_t crc;
  };
  std::vector<Item> items;
  for (size_t i = 0; i < pieces.size(); ++i) {
    if (pieces[i].len == 0) items.push_back({i, 0, 0, 0});
    for (uint64_t o = 0; o < pieces[i].len; o += chunk) items.push_back({i, o, std::min(chunk, pieces[i].len - o), 0});
  }
  std::atomic<size_t> next{0};
  std::atomic<uint64_t> direct_bytes{0};
  std::string err;
  std::mutex err_mu;
  auto worker = [&] {
    for (;;) {
      size_t k = next.fetch_add(1);
      if (k >= items.size()) return;
      Item& c = items[k];
      const FilePiece& pc = pieces[c.piece];
      try {
        const uint8_t* p = pc.ptr + c.off;
        uLong crc = crc32(0L, Z_NULL, 0);
        uint64_t done = 0;
        while (done < c.len) {
          const uInt n = (uInt)std::min<uint64_t>(c.len - done, 1u << 30);
          crc = crc32(crc, p + done, n);
          done += n;
        }
        c.crc = (uint32_t)crc;
        if (c.len) {
          const uint64_t foff = pc.file_off + c.off;
          const uint64_t body = (dfd >= 0 && foff % DIRECT_ALIGN == 0 &&
                                 reinterpret_cast<uintptr_t>(p) % DIRECT_ALIGN == 0)
                                    ? c.len / DIRECT_ALIGN * DIRECT_ALIGN
                                    : 0;
          if (body) {
            if (!pwrite_direct(dfd, p, body, foff)) {
              pwrite_all(fd, p, body, foff);  // O_DIRECT refused at write time
            } else {
              direct_bytes.fetch_add(body);
            }
          }
          if (c.len > body) pwrite_all(fd, p + body, c.len - body, foff + body);
        }
      } catch (const std::exception& ex) {
        std::lock_guard<std::mutex> g(err_mu);
        err = ex.what();
        next.store(items.size());
      }
    }
  };
  std::vector<std::thread> pool;
  const int nt = (int)std::min<size_t>(nthreads < 1 ? 1 : nthreads, std::max<size_t>(1, items.size()));
  for (int t = 0; t < nt; ++t) pool.emplace_back(worker);
  for (auto& t : pool) t.join();
  if (!err.empty()) throw std::runtime_error(err);
  // fold the item CRCs into per-piece CRCs (in order)
  std::vector<bool> first(pieces.size(), true);
  for (const auto& c : items) {
    auto& pc = pieces[c.piece];
    if (first[c.piece]) {
      pc.crc = c.crc;
      first[c.piece] = false;
    } else {
      pc.crc = (uint32_t)crc32_combine64(pc.crc, c.crc, (z_off64_t)c.len);
    }
  }
  return direct_bytes.load();
}

std::vector<uint32_t> write_pieces(const std::string& path, const std::vector<uint64_t>& file_offs,
                                   const std::vector<uint64_t>& ptrs, const std::vector<uint64_t>& lens,
                                   int nthreads, uintptr_t wait_event, bool do_fsync, bool direct) {
  if (file_offs.size() != ptrs.size() || ptrs.size() != lens.size())
    throw std::runtime_error("write_pieces: length mismatch");
  if (wait_event) {
    hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(wait_event));
    if (e != hipSuccess) throw std::runtime_error(std::string("hipEventSynchronize: ") + hipGetErrorString(e));
  }
  std::vector<FilePiece> pieces(file_offs.size());
  for (size_t i = 0; i < pieces.size(); ++i) {
    pieces[i].file_off = file_offs[i];
    pieces[i].ptr = reinterpret_cast<const uint8_t*>(ptrs[i]);
    pieces[i].len = lens[i];
  }
  int fd = ::open(path.c_str(), O_WRONLY | O_CLOEXEC);
  if (fd < 0) throw std::runtime_error("open(" + path + "): " + strerror(errno));
  int dfd = direct ? ::open(path.c_str(), O_WRONLY | O_DIRECT | O_CLOEXEC) : -1;
  std::string err;
  try {
    write_pieces_fd(fd, dfd, pieces, nthreads, 64ull << 20);
  } catch (const std::exception& ex) {
    err = ex.what();
  }
  if (dfd >= 0) {
    if (do_fsync) ::fdatasync(dfd);
    ::close(dfd);
  }
  if (do_fsync) ::fdatasync(fd);
  ::close(fd);
  if (!err.empty()) throw std::runtime_error(err);
  std::vector<uint32_t> crcs;
  for (const auto& p : pieces) crcs.push_back(p.crc);
  return crcs;
}

uint32_t crc32_combine_u32(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return (uint32_t)crc32_combine64(crc1, crc2, (z_off64_t)len2);
}

ZipWriter::ZipWriter(std::string tmp_path, std::string final_path, std::string archive,
                     int nthreads, uint64_t chunk_bytes, bool direct)
    : tmp_(std::move(tmp_path)),
      final_(std::move(final_path)),
      archive_(std::move(archive)),
      nthreads_(nthreads < 1 ? 1 : nthreads),
      chunk_(chunk_bytes ? chunk_bytes : (64ull << 20)),
      direct_(direct) {}

ZipWriter::~ZipWriter() {
  if (th_.joinable()) th_.join();
}

void ZipWriter::add_bytes(const std::string& name, const std::string& bytes) {
  ZipRecord r;
  r.name = archive_ + "/" + name;
  r.owned = bytes;
  r.size = bytes.size();
  recs_.push_back(std::move(r));
  laid_out_ = false;
}

void ZipWriter::add_buffer(const std::string& name, uintptr_t ptr, uint64_t nbytes) {
  ZipRecord r;
  r.name = archive_ + "/" + name;
  r.data = reinterpret_cast<const uint8_t*>(ptr);
  r.size = nbytes;
  recs_.push_back(std::move(r));
  laid_out_ = false;
}

void ZipWriter::add_external(const std::string& name, uint64_t nbytes, uint32_t crc) {
  ZipRecord r;
  r.name = archive_ + "/" + name;
  r.size = nbytes;
  r.crc = crc;
  r.external = true;
  recs_.push_back(std::move(r));
  laid_out_ = false;
}

void ZipWriter::set_external_crc(const std::string& name, uint32_t crc) {
  const std::string full = archive_ + "/" + name;
  for (auto& r : recs_)
    if (r.name == full && r.external) {
      r.crc = crc;
      return;
    }
  throw std::runtime_error("set_external_crc: no external record " + name);
}

std::vector<std::tuple<std::string, uint64_t, uint64_t>> ZipWriter::layout_records() {
  if (!laid_out_) layout();
  std::vector<std::tuple<std::string, uint64_t, uint64_t>> out;
  for (const auto& r : recs_) out.emplace_back(r.name.substr(archive_.size() + 1), r.data_off, r.size);
  return out;
}

void ZipWriter::create_file() {
  if (!laid_out_) layout();
  int fd = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("open(" + tmp_ + "): " + strerror(errno));
  if (::ftruncate(fd, (off_t)cd_off_) != 0) {
    ::close(fd);
    throw std::runtime_error(std::string("ftruncate: ") + strerror(errno));
  }
  ::close(fd);
  truncate_ = false;
}

void ZipWriter::layout() {
  uint64_t off = 0;
  for (auto& r : recs_) {
    if (!r.external && (!r.owned.empty() || r.data == nullptr))
      r.data = reinterpret_cast<const uint8_t*>(r.owned.data());
    r.header_off = off;
    const bool z64_local = r.size >= U32MAX;
    r.zip64 = z64_local;
    uint64_t base = off + 30 + r.name.size() + (z64_local ? 20 : 0) + 4;  // + FB header
    const uint64_t al = (r.size >= DIRECT_MIN && direct_) ? DIRECT_ALIGN : ALIGN;
    uint64_t pad = (al - base % al) % al;
    r.extra_len = (uint16_t)((z64_local ? 20 : 0) + 4 + pad);
    r.data_off = base + pad;
    off = r.data_off + r.size;
  }
  cd_off_ = off;
  laid_out_ = true;
}

uint64_t ZipWriter::total_size() {
  if (!laid_out_) layout();
  return cd_off_;
}

void ZipWriter::start(uintptr_t wait_event, bool do_fsync) {
  if (th_.joinable()) throw std::runtime_error("ZipWriter already started");
  if (!laid_out_) layout();
  th_ = std::thread([this, wait_event, do_fsync] { run(wait_event, do_fsync); });
}

void ZipWriter::run_sync(uintptr_t wait_event, bool do_fsync) {
  if (!laid_out_) layout();
  run(wait_event, do_fsync);
}

ZipStats ZipWriter::wait() {
  if (th_.joinable()) th_.join();
  return stats_;
}

void ZipWriter::run(uintptr_t wait_event, bool do_fsync) {
  const double t0 = now();
  int fd = -1;
  try {
    if (wait_event) {
      hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(wait_event));
      if (e != hipSuccess) throw std::runtime_error(std::string("hipEventSynchronize: ") + hipGetErrorString(e));
    }
    const double t1 = now();
    stats_.wait_seconds = t1 - t0;
    fd = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | (truncate_ ? O_TRUNC : 0) | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("open(" + tmp_ + "): " + strerror(errno));
    int dfd_direct = -1;
    if (direct_) {
      dfd_direct = ::open(tmp_.c_str(), O_WRONLY | O_DIRECT | O_CLOEXEC);
      if (dfd_direct < 0) direct_used_ = false;  // filesystem without O_DIRECT: buffered only
    }

    // ---- data records: parallel CRC + pwrite in chunks --------------------------
    // (records whose bytes other ranks write — sharded save — carry a given CRC)
    std::vector<FilePiece> pieces;
    std::vector<std::pair<size_t, size_t>> rec_pieces(recs_.size(), {0, 0});
    for (size_t i = 0; i < recs_.size(); ++i) {
      const auto& r = recs_[i];
      if (r.external) continue;
      rec_pieces[i].first = pieces.size();
      for (uint64_t o = 0; o < r.size; o += chunk_) {
        FilePiece p;
        p.file_off = r.data_off + o;
        p.ptr = r.data + o;
        p.len = std::min(chunk_, r.size - o);
        pieces.push_back(p);
      }
      rec_pieces[i].second = pieces.size();
    }
    std::string err;
    try {
      stats_.direct_bytes = write_pieces_fd(fd, dfd_direct, pieces, nthreads_, chunk_);
    } catch (const std::exception& ex) {
      err = ex.what();
    }
    if (dfd_direct >= 0) {
      if (do_fsync) ::fdatasync(dfd_direct);
      ::close(dfd_direct);
    }
    if (!err.empty()) throw std::runtime_error(err);
    for (size_t i = 0; i < recs_.size(); ++i) {
      auto& r = recs_[i];
      if (r.external) continue;
      uint32_t crc = (uint32_t)crc32(0L, Z_NULL, 0);
      bool first = true;
      for (size_t k = rec_pieces[i].first; k < rec_pieces[i].second; ++k) {
        crc = first ? pieces[k].crc : (uint32_t)crc32_combine64(crc, pieces[k].crc, (z_off64_t)pieces[k].len);
        first = false;
      }
      r.crc = crc;
    }

    // ---- local headers ----------------------------------------------------------
    for (const auto& r : recs_) {
      Buf b;
      b.u32(0x04034b50);
      b.u16(r.zip64 ? 45 : 20);
      b.u16(0);
      b.u16(0);
      b.u16(DOS_TIME);
      b.u16(DOS_DATE);
      b.u32(r.crc);
      b.u32(r.zip64 ? (uint32_t)U32MAX : (uint32_t)r.size);
      b.u32(r.zip64 ? (uint32_t)U32MAX : (uint32_t)r.size);
      b.u16((uint16_t)r.name.size());
      b.u16(r.extra_len);
      b.str(r.name);
      uint16_t used = 0;
      if (r.zip64) {
        b.u16(0x0001);
        b.u16(16);
        b.u64(r.size);
        b.u64(r.size);
        used = 20;
      }
      const uint16_t pad = (uint16_t)(r.extra_len - used - 4);
      b.u16(0x4246);  // "FB": PyTorch's alignment padding field
      b.u16(pad);
      b.s.append(pad, 'Z');
      pwrite_all(fd, b.s.data(), b.s.size(), r.header_off);
    }

    // ---- central directory --------------------------------------------------------
    Buf cd;
    bool need64 = recs_.size() >= 0xFFFF;
    for (const auto& r : recs_) {
      const bool big = r.size >= U32MAX;
      const bool far = r.header_off >= U32MAX;
      std::string ex;
      Buf e;
      if (big || far) {
        e.u16(0x0001);
        e.u16((uint16_t)((big ? 16 : 0) + (far ? 8 : 0)));
        if (big) {
          e.u64(r.size);
          e.u64(r.size);
        }
        if (far) e.u64(r.header_off);
        need64 = true;
      }
      cd.u32(0x02014b50);
      cd.u16(45);
      cd.u16((big || far) ? 45 : 20);
      cd.u16(0);
      cd.u16(0);
      cd.u16(DOS_TIME);
      cd.u16(DOS_DATE);
      cd.u32(r.crc);
      cd.u32(big ? (uint32_t)U32MAX : (uint32_t)r.size);
      cd.u32(big ? (uint32_t)U32MAX : (uint32_t)r.size);
      cd.u16((uint16_t)r.name.size());
      cd.u16((uint16_t)e.s.size());
      cd.u16(0);
      cd.u16(0);
      cd.u16(0);
      cd.u32(0);
      cd.u32(far ? (uint32_t)U32MAX : (uint32_t)r.header_off);
      cd.str(r.name);
      cd.str(e.s);
    }
    const uint64_t cd_size = cd.s.size();
    if (cd_off_ >= U32MAX || cd_size >= U32MAX) need64 = true;
    Buf tail;
    const uint64_t n = recs_.size();
    if (need64) {
      const uint64_t z64_off = cd_off_ + cd_size;
      tail.u32(0x06064b50);
      tail.u64(44);
      tail.u16(45);
      tail.u16(45);
      tail.u32(0);
      tail.u32(0);
      tail.u64(n);
      tail.u64(n);
      tail.u64(cd_size);
      tail.u64(cd_off_);
      tail.u32(0x07064b50);
      tail.u32(0);
      tail.u64(z64_off);
      tail.u32(1);
    }
    tail.u32(0x06054b50);
    tail.u16(0);
    tail.u16(0);
    tail.u16((uint16_t)std::min<uint64_t>(n, 0xFFFF));
    tail.u16((uint16_t)std::min<uint64_t>(n, 0xFFFF));
    tail.u32(cd_size >= U32MAX ? (uint32_t)U32MAX : (uint32_t)cd_size);
    tail.u32(cd_off_ >= U32MAX ? (uint32_t)U32MAX : (uint32_t)cd_off_);
    tail.u16(0);
    cd.str(tail.s);
    pwrite_all(fd, cd.s.data(), cd.s.size(), cd_off_);
    stats_.bytes = cd_off_ + cd.s.size();
    const double t2 = now();
    stats_.write_seconds = t2 - t1;
    if (do_fsync && ::fsync(fd) != 0) throw std::runtime_error(std::string("fsync: ") + strerror(errno));
    ::close(fd);
    fd = -1;
    if (tmp_ != final_) {
      if (::rename(tmp_.c_str(), final_.c_str()) != 0)
        throw std::runtime_error("rename(" + tmp_ + "): " + strerror(errno));
      if (do_fsync) {
        int dfd = ::open(dirname_of(final_).c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
        if (dfd >= 0) {
          ::fsync(dfd);
          ::close(dfd);
        }
      }
    }
    stats_.fsync_seconds = now() - t2;
  } catch (const std::exception& ex) {
    stats_.error = ex.what();
    if (fd >= 0) ::close(fd);
  }
  stats_.seconds = now() - t0;
  done_.store(true);
}

}  // namespace ftrt
