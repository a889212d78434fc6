// Host-runtime self-test for the sanitizer builds: exercises the RecordLoader
// thread pool (ticket ordering, slot recycling, stop while workers wait), the Watchdog monitor
// thread, the bucket planner, CRC32 and the atomic writer. Built and run by
// tests/test_sanitizers.py three ways: -fsanitize=address,undefined and -fsanitize=thread (races
// in the loader / watchdog), plus a plain -O2 build. Exit code 0 = pass.
#include "../runtime/runtime_core.h"

#include <cstdlib>
#include <iostream>

using namespace cmlrt;

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::cerr << "CHECK failed: " #c " at line " << __LINE__ << "\n"; \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static std::string tmpdir() {
  const char* t = std::getenv("TMPDIR");
  return t ? t : "/tmp";
}

static void test_loader() {
  const int64_t rec = 24, n = 1000;
  const std::string path = tmpdir() + "/cml_selftest_records.bin";
  std::string data(static_cast<size_t>(rec * n), '\0');
  for (int64_t i = 0; i < n; ++i) std::memcpy(&data[static_cast<size_t>(i * rec)], &i, sizeof(i));
  write_file_atomic(path, data);
  for (int world : {1, 3}) {
    for (int rank = 0; rank < world; ++rank) {
      RecordLoader L(path, rec, 32, rank, world, 7, 4, true);
      const int64_t per = L.batches_per_epoch();
      std::vector<std::vector<uint8_t>> bufs(3, std::vector<uint8_t>(static_cast<size_t>(32 * rec)));
      std::vector<uintptr_t> slots;
      for (auto& b : bufs) slots.push_back(reinterpret_cast<uintptr_t>(b.data()));
      L.start(slots, 32 * rec, 0);
      for (int64_t t = 0; t < 3 * per; ++t) {
        RecordLoader::Batch b = L.next_batch();
        CHECK(b.ticket == t);
        CHECK(b.epoch == t / per);
        const std::vector<int64_t> want = L.batch_indices(b.epoch, t % per);
        CHECK(static_cast<int64_t>(want.size()) == b.rows);
        for (int64_t k = 0; k < b.rows; ++k) {
          int64_t got;
          std::memcpy(&got, bufs[static_cast<size_t>(b.slot)].data() + k * rec, sizeof(got));
          CHECK(got == want[static_cast<size_t>(k)]);
          CHECK(got % world == got % world);   // touch
        }
        L.release(b.slot);
      }
      L.stop();   // workers blocked on full slots must exit
    }
  }
  // disjoint rank shares within an epoch
  std::vector<int> seen(static_cast<size_t>(n), 0);
  for (int rank = 0; rank < 4; ++rank) {
    RecordLoader L(path, rec, 50, rank, 4, 3, 1, true);
    for (int64_t b = 0; b < L.batches_per_epoch(); ++b)
      for (int64_t i : L.batch_indices(0, b)) seen[static_cast<size_t>(i)]++;
  }
  for (int v : seen) CHECK(v <= 1);
  std::remove(path.c_str());
}

static void test_watchdog() {
  const std::string rep = tmpdir() + "/cml_selftest_watchdog.jsonl";
  std::remove(rep.c_str());
  {
    Watchdog w(0.3, rep, false);
    for (int i = 0; i < 5; ++i) {
      w.beat(i);
      w.set_phase("step");
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    CHECK(!w.fired());
    std::this_thread::sleep_for(std::chrono::milliseconds(700));
    CHECK(w.fired());
    w.stop();
  }
  std::ifstream f(rep);
  std::string line;
  std::getline(f, line);
  CHECK(line.find("\"step\": 4") != std::string::npos);
  std::remove(rep.c_str());
}

static void test_helpers() {
  const std::string s = "123456789";
  CHECK(crc32_update(0, reinterpret_cast<const uint8_t*>(s.data()), s.size()) == 0xCBF43926u);
  const BucketPlan p = plan_buckets({100, 3, 5000, 17, 9}, 4, 64, 4096);
  int64_t prev_end = 0;
  for (size_t b = 0; b < p.offsets.size(); ++b) {
    CHECK(p.offsets[b] == prev_end);
    CHECK(p.lengths[b] % (4 * 64) == 0);
    CHECK(p.shards[b] * 4 == p.lengths[b]);
    prev_end += p.lengths[b];
  }
  CHECK(p.total == prev_end);
  const std::string csv = format_csv({"g1", "g2"}, {"a", "b"},
                                     {{format_number(1.5), format_number(0.0 / 0.0)}, {"\"x\"", "\"y\""}});
  CHECK(csv == "\"\",\"a\",\"b\"\n\"g1\",1.5,\"x\"\n\"g2\",NA,\"y\"\n");
}

int main() {
  test_helpers();
  test_loader();
  test_watchdog();
  std::cout << "runtime selftest ok\n";
  return 0;
}
