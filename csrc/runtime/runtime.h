// Native runtime for the fault-tolerance path (host C++ + HIP runtime API).
#pragma once

#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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
};

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
  std::thread th_;
  std::atomic<bool> done_{false};
  ZipStats stats_;
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

 private:
  int device_;
  void* stream_ = nullptr;
  std::vector<void*> events_;
  std::mutex mu_;
};

uintptr_t pinned_alloc(uint64_t nbytes);
void pinned_free(uintptr_t p);

}  // namespace ftrt
