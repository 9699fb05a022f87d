// Side-stream snapshot engine (HIP runtime API, host code).
//
// MI355X-first replacement for the reference's synchronous, pageable D2H inside
// torch.save (reference utils.py:75-80). The training state
// lives in a few flat HBM buffers, so a checkpoint is a handful of large
// copies: an optional D2D snapshot into reserved HBM (288 GB leaves room for a
// second copy of the 48 GB Llama-3-8B state), then a D2H drain into pinned
// host memory, both on a dedicated non-blocking stream ordered after the
// compute stream by an event. The compute stream only has to wait for the
// snapshot event before the next optimizer step mutates the state.
#include <hip/hip_runtime_api.h>

#include "runtime.h"

namespace ftrt {
namespace {
void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

SnapshotEngine::SnapshotEngine(int device) : device_(device) {
  check(hipSetDevice(device_), "hipSetDevice");
  hipStream_t s;
  check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
  stream_ = s;
}

SnapshotEngine::~SnapshotEngine() {
  for (void* e : events_) hipEventDestroy(reinterpret_cast<hipEvent_t>(e));
  if (stream_) hipStreamDestroy(reinterpret_cast<hipStream_t>(stream_));
}

// Events are a small pool reused by every save: a save starts only after the previous
// one is durable (CheckpointEngine.save waits for it), so its begin() may re-record slot 0
// and its mark()s the next slots; a long --save-every run creates at most kPool events.
int SnapshotEngine::next_event() {
  if (next_ >= (int)events_.size()) {
    if ((int)events_.size() >= kPool) throw std::runtime_error("SnapshotEngine: too many events in one save");
    hipEvent_t e;
    check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    events_.push_back(e);
  }
  return next_++;
}

void SnapshotEngine::begin(uintptr_t compute_stream) {
  std::lock_guard<std::mutex> g(mu_);
  check(hipSetDevice(device_), "hipSetDevice");
  next_ = 0;
  hipEvent_t e = reinterpret_cast<hipEvent_t>(events_[next_event()]);  // slot 0
  check(hipEventRecord(e, reinterpret_cast<hipStream_t>(compute_stream)), "hipEventRecord");
  check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream_), e, 0), "hipStreamWaitEvent");
}

void SnapshotEngine::copy(uintptr_t dst, uintptr_t src, uint64_t nbytes) {
  check(hipSetDevice(device_), "hipSetDevice");
  // 1 GiB pieces keep each DMA command short so D2D/D2H traffic interleaves
  // fairly with the compute stream's own memory traffic.
  const uint64_t piece = 1ull << 30;
  for (uint64_t o = 0; o < nbytes; o += piece) {
    const uint64_t n = std::min(piece, nbytes - o);
    check(hipMemcpyAsync(reinterpret_cast<void*>(dst + o), reinterpret_cast<const void*>(src + o), n,
                         hipMemcpyDefault, reinterpret_cast<hipStream_t>(stream_)),
          "hipMemcpyAsync");
  }
}

int SnapshotEngine::mark() {
  std::lock_guard<std::mutex> g(mu_);
  const int i = next_event();
  check(hipEventRecord(reinterpret_cast<hipEvent_t>(events_[i]), reinterpret_cast<hipStream_t>(stream_)),
        "hipEventRecord");
  return i;
}

int SnapshotEngine::num_events() { return (int)events_.size(); }

void SnapshotEngine::stream_wait(uintptr_t compute_stream, int ev) {
  check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(compute_stream),
                           reinterpret_cast<hipEvent_t>(events_.at(ev)), 0),
        "hipStreamWaitEvent");
}

bool SnapshotEngine::query(int ev) {
  hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(events_.at(ev)));
  if (e == hipSuccess) return true;
  if (e == hipErrorNotReady) return false;
  check(e, "hipEventQuery");
  return false;
}

void SnapshotEngine::sync(int ev) {
  check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(events_.at(ev))), "hipEventSynchronize");
}

uintptr_t SnapshotEngine::event_handle(int ev) { return reinterpret_cast<uintptr_t>(events_.at(ev)); }
uintptr_t SnapshotEngine::stream_handle() { return reinterpret_cast<uintptr_t>(stream_); }

uintptr_t pinned_alloc(uint64_t nbytes) {
  void* p = nullptr;
  check(hipHostMalloc(&p, nbytes, hipHostMallocDefault), "hipHostMalloc");
  return reinterpret_cast<uintptr_t>(p);
}

void pinned_free(uintptr_t p) {
  if (p) hipHostFree(reinterpret_cast<void*>(p));
}

}  // namespace ftrt
