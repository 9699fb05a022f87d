// Host self-test of the native fault-tolerance runtime, built under AddressSanitizer +
// UndefinedBehaviorSanitizer or ThreadSanitizer (the reference has no race
// detection; its only concurrency hazard was signal-vs-main-thread, reference utils.py:93-97).
//
// Exercises every host-side concurrent path of csrc/runtime without touching a GPU:
//   * signals.cpp    — SIGUSR1/SIGTERM delivered from other threads while the main thread
//                      polls the atomic flags (first-signal, mask, count, clear);
//   * zip_writer.cpp — ZipWriter with a pool of CRC/pwrite threads (async start()/wait(),
//                      buffered and O_DIRECT bodies, ragged sizes), write_pieces() from
//                      several "ranks" into one pre-sized file, crc32_combine_u32;
//   * file_reader.cpp — parallel pread (O_DIRECT + buffered head/tail) of unaligned ranges.
// Built and run by tests/test_runtime_sanitizers.py; exits non-zero on any mismatch.
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/runtime.h"

namespace {

int g_fail = 0;

#define CHECK(cond, ...)                                    \
  do {                                                      \
    if (!(cond)) {                                          \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                         \
      fprintf(stderr, "\n");                                \
      ++g_fail;                                             \
    }                                                       \
  } while (0)

std::vector<uint8_t> random_bytes(size_t n, uint32_t seed) {
  std::vector<uint8_t> v(n);
  std::mt19937 g(seed);
  for (size_t i = 0; i < n; ++i) v[i] = static_cast<uint8_t>(g());
  return v;
}

uint32_t crc_of(const uint8_t* p, size_t n) {
  uLong c = crc32(0L, Z_NULL, 0);
  while (n) {
    const uInt k = n > (1u << 30) ? (1u << 30) : static_cast<uInt>(n);
    c = crc32(c, p, k);
    p += k;
    n -= k;
  }
  return static_cast<uint32_t>(c);
}

void test_signals() {
  using namespace ftrt;
  signals_clear();
  const std::vector<int> sigs = {SIGUSR1, SIGTERM, SIGUSR2, SIGHUP};
  signals_install(sigs);
  // deliveries from several threads race with the main thread's polling (distinct
  // signals: standard signals of one number coalesce while pending)
  std::vector<std::thread> senders;
  for (int s : sigs) senders.emplace_back([s] { kill(getpid(), s); });
  for (auto& th : senders) th.join();
  for (int spin = 0; spin < 2000 && signals_count() < 4; ++spin) usleep(500);
  CHECK(signals_count() == 4, "signal count %llu", (unsigned long long)signals_count());
  const int first = signals_pending();
  CHECK(first == SIGUSR1 || first == SIGTERM || first == SIGUSR2 || first == SIGHUP, "first signal %d", first);
  uint64_t want = 0;
  for (int s : sigs) want |= 1ull << s;
  CHECK(signals_mask() == want, "mask %llx", (unsigned long long)signals_mask());
  signals_clear();
  CHECK(signals_pending() == 0 && signals_mask() == 0, "clear");
  // blocked signals stay pending in the kernel until unblocked
  signals_block({SIGUSR1}, true);
  raise(SIGUSR1);
  CHECK(signals_pending() == 0, "blocked signal delivered");
  signals_block({SIGUSR1}, false);
  for (int spin = 0; spin < 2000 && signals_pending() == 0; ++spin) usleep(500);
  CHECK(signals_pending() == SIGUSR1, "unblocked signal not delivered");
  signals_restore_default(sigs);
  signals_clear();
}

void read_back(const std::string& path, uint64_t off, std::vector<uint8_t>& out, bool direct) {
  ftrt::FileReader rd(path, 4, direct);
  rd.read(off, reinterpret_cast<uintptr_t>(out.data()), out.size());
}

void test_zip_writer(const std::string& dir, bool direct) {
  // sizes: multi-chunk, ragged (not 4 KiB aligned), tiny, empty
  const std::vector<size_t> sizes = {(9u << 20) + 12345, (3u << 20), 777, 0};
  std::vector<std::vector<uint8_t>> bufs;
  for (size_t i = 0; i < sizes.size(); ++i) bufs.push_back(random_bytes(sizes[i], 17 + i));
  const std::string fin = dir + (direct ? "/ck_direct.ckpt" : "/ck_buffered.ckpt");
  const std::string tmp = fin + ".tmp";
  ftrt::ZipWriter zw(tmp, fin, "archive", 4, 1u << 20, direct);
  zw.add_bytes("data.pkl", std::string("\x80\x02}q\x00.", 6));
  for (size_t i = 0; i < bufs.size(); ++i)
    zw.add_buffer("data/" + std::to_string(i), reinterpret_cast<uintptr_t>(bufs[i].data()), bufs[i].size());
  zw.start(0, true);  // writer thread + CRC/pwrite pool; main thread keeps running
  volatile uint64_t spin = 0;
  while (!zw.done()) ++spin;
  ftrt::ZipStats st = zw.wait();
  CHECK(st.error.empty(), "zip writer error: %s", st.error.c_str());
  CHECK(access(fin.c_str(), F_OK) == 0 && access(tmp.c_str(), F_OK) != 0, "atomic rename");
  for (const auto& rec : zw.layout_records()) {
    const std::string& name = std::get<0>(rec);
    const uint64_t off = std::get<1>(rec), size = std::get<2>(rec);
    if (name.rfind("archive/data/", 0) != 0) continue;
    const size_t i = std::stoul(name.substr(13));
    CHECK(size == bufs[i].size(), "%s size", name.c_str());
    std::vector<uint8_t> back(size);
    if (size) read_back(fin, off, back, direct);
    CHECK(back == bufs[i], "%s bytes differ", name.c_str());
  }
}

void test_sharded_pieces(const std::string& dir) {
  // 4 "ranks" write disjoint pieces of one pre-sized file concurrently; the CRC of the
  // whole region is rebuilt from the pieces' CRCs (the sharded-save path)
  const size_t n = (6u << 20) + 4096 * 3 + 100;
  auto all = random_bytes(n, 99);
  const std::string path = dir + "/sharded.bin";
  int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
  CHECK(fd >= 0 && ftruncate(fd, n) == 0, "create");
  close(fd);
  const int W = 4;
  const size_t per = (n + W - 1) / W;
  std::vector<uint32_t> crcs(W);
  std::vector<std::thread> ranks;
  for (int r = 0; r < W; ++r)
    ranks.emplace_back([&, r] {
      const size_t lo = r * per, hi = std::min(n, lo + per);
      auto c = ftrt::write_pieces(path, {lo}, {reinterpret_cast<uint64_t>(all.data() + lo)}, {hi - lo},
                                  2, 0, r == 0, true);
      crcs[r] = c.at(0);
    });
  for (auto& t : ranks) t.join();
  uint32_t crc = crcs[0];
  for (int r = 1; r < W; ++r) crc = ftrt::crc32_combine_u32(crc, crcs[r], std::min(n, (r + 1) * per) - r * per);
  CHECK(crc == crc_of(all.data(), n), "combined crc %08x vs %08x", crc, crc_of(all.data(), n));
  std::vector<uint8_t> back(n - 4097);
  read_back(path, 4097, back, true);  // unaligned start and length
  CHECK(memcmp(back.data(), all.data() + 4097, back.size()) == 0, "sharded bytes differ");
}

}  // namespace

int main() {
  char tmpl[] = "/tmp/ftrt_selftest_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  if (!dir) {
    perror("mkdtemp");
    return 2;
  }
  try {
    test_signals();
    test_zip_writer(dir, false);
    test_zip_writer(dir, true);
    test_sharded_pieces(dir);
  } catch (const std::exception& e) {
    fprintf(stderr, "FAIL exception: %s\n", e.what());
    ++g_fail;
  }
  std::string cmd = std::string("rm -rf ") + dir;
  if (system(cmd.c_str()) != 0) fprintf(stderr, "cleanup failed\n");
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("runtime selftest ok\n");
  return 0;
}
