// Native runtime for the fault-tolerance path (host C++ + HIP runtime API).
#pragma once

#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace ftrt {

// ---- signals.cpp ---------------------------------------------------------------
void signals_install(const std::vector<int>& signums);
void signals_restore_default(const std::vector<int>& signums);
int signals_pending();
uint64_t signals_mask();
uint64_t signals_count();
void signals_clear();
void signals_block(const std::vector<int>& signums, bool block);

// ---- zip_writer.cpp --------------------------------------------------------------
// Writes a PyTorch-compatible zip checkpoint (stored entries, 64-B aligned
// records, zip64) from host memory with a pool of threads: each thread CRCs and
// pwrite()s 64 MiB chunks; headers and the central directory are written last,
// then fsync + atomic rename. A range of the file can be restricted to one rank
// for the sharded multi-writer mode (each DP rank writes its byte range of the
// shared storages into the same file).
struct ZipRecord {
  std::string name;
  std::string owned;       // small records (data.pkl, version, ...)
  const uint8_t* data = nullptr;
  uint64_t size = 0;
  // filled by layout()
  uint64_t header_off = 0, data_off = 0;
  uint16_t extra_len = 0;
  bool zip64 = false;
  uint32_t crc = 0;
  bool external = false;   // bytes written by other processes (sharded save); crc given
};

// One contiguous piece of a file: `len` bytes from host `ptr` to file offset `file_off`.
struct FilePiece {
  uint64_t file_off = 0;
  const uint8_t* ptr = nullptr;
  uint64_t len = 0;
  uint32_t crc = 0;
};

// Parallel CRC32 + pwrite of pieces (O_DIRECT for 4 KiB-aligned bodies when dfd >= 0).
// Fills each piece's crc; returns bytes written with O_DIRECT.
uint64_t write_pieces_fd(int fd, int dfd, std::vector<FilePiece>& pieces, int nthreads, uint64_t chunk);

// Sharded-save helpers (every rank writes its own pieces of one shared file).
std::vector<uint32_t> write_pieces(const std::string& path, const std::vector<uint64_t>& file_offs,
                                   const std::vector<uint64_t>& ptrs, const std::vector<uint64_t>& lens,
                                   int nthreads, uintptr_t wait_event, bool do_fsync, bool direct);
uint32_t crc32_combine_u32(uint32_t crc1, uint32_t crc2, uint64_t len2);

struct ZipStats {
  double seconds = 0, write_seconds = 0, fsync_seconds = 0, wait_seconds = 0;
  uint64_t bytes = 0;
  uint64_t direct_bytes = 0;  // written with O_DIRECT
  std::string error;
};

class ZipWriter {
 public:
  ZipWriter(std::string tmp_path, std::string final_path, std::string archive, int nthreads,
            uint64_t chunk_bytes, bool direct = true);
  ~ZipWriter();
  void add_bytes(const std::string& name, const std::string& bytes);
  void add_buffer(const std::string& name, uintptr_t ptr, uint64_t nbytes);
  // A record whose bytes other processes write into the same file (sharded save).
  void add_external(const std::string& name, uint64_t nbytes, uint32_t crc);
  void set_external_crc(const std::string& name, uint32_t crc);
  // (name, data offset, size) of every record after layout.
  std::vector<std::tuple<std::string, uint64_t, uint64_t>> layout_records();
  // Create the temp file sized to the data region so other ranks can pwrite into it;
  // the final run() then does not truncate it.
  void create_file();
  // Spawn the writer thread. If wait_event != 0 it is a hipEvent_t that must
  // complete before host memory is read (the D2H snapshot).
  void start(uintptr_t wait_event, bool do_fsync);
  void run_sync(uintptr_t wait_event, bool do_fsync);
  bool done() const { return done_.load(); }
  ZipStats wait();
  uint64_t total_size();  // file size after layout

 private:
  void layout();
  void run(uintptr_t wait_event, bool do_fsync);
  std::string tmp_, final_, archive_;
  int nthreads_;
  uint64_t chunk_;
  std::vector<ZipRecord> recs_;
  uint64_t cd_off_ = 0;
  bool laid_out_ = false;
  bool direct_ = true;       // align big records and try O_DIRECT
  bool direct_used_ = true;
  bool truncate_ = true;
  std::thread th_;
  std::atomic<bool> done_{false};
  ZipStats stats_;
};

// ---- file_reader.cpp -------------------------------------------------------------
// Parallel pread (O_DIRECT for 4 KiB-aligned bodies) of a file range into host memory:
// the checkpoint restore path (file -> pinned chunk -> HBM), see ckpt/restore.py.
class FileReader {
 public:
  FileReader(const std::string& path, int nthreads, bool direct);
  ~FileReader();
  void read(uint64_t off, uintptr_t ptr, uint64_t len);
  uint64_t bytes() const { return bytes_; }
  uint64_t direct_bytes() const { return direct_bytes_; }

 private:
  std::string path_;
  int nthreads_;
  int fd_ = -1, dfd_ = -1;
  uint64_t bytes_ = 0, direct_bytes_ = 0;
};

// ---- snapshot.cpp (HIP) ------------------------------------------------------------
// Side-stream copy engine: D2D snapshot into reserved HBM and D2H drain into
// pinned host memory, ordered after the compute stream by events.
class SnapshotEngine {
 public:
  explicit SnapshotEngine(int device);
  ~SnapshotEngine();
  void begin(uintptr_t compute_stream);  // side stream waits for all prior compute work
  void copy(uintptr_t dst, uintptr_t src, uint64_t nbytes);
  int mark();                           // record an event on the side stream
  void stream_wait(uintptr_t compute_stream, int ev);  // compute waits for event
  bool query(int ev);
  void sync(int ev);
  uintptr_t event_handle(int ev);
  uintptr_t stream_handle();
  int num_events();  // events created so far (a fixed pool: reused by every save)

 private:
  static constexpr int kPool = 8;
  int next_event();
  int device_;
  int next_ = 0;
  void* stream_ = nullptr;
  std::vector<void*> events_;
  std::mutex mu_;
};

uintptr_t pinned_alloc(uint64_t nbytes);
void pinned_free(uintptr_t p);

}  // namespace ftrt
