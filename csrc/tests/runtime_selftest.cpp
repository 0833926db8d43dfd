// Standalone self-test of the host runtime (csrc/runtime), built with the
// sanitizers by tests/test_native_sanitizers.py:
//   -fsanitize=thread             : the multi-threaded Prefetcher (data races,
//                                   lock-order problems) under skip-ahead and
//                                   early destruction
//   -fsanitize=address,undefined  : TensorBundle write/read round trip,
//                                   SSTable parse with CRC verification,
//                                   CRC32C, synthetic batch generation
// Exit status 0 = all checks passed; sanitizer reports fail the test.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "native_common.h"

using namespace tdgn;

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

static void test_prefetcher() {
  SynthConfig c;
  c.batch = 8;
  c.src_len = 33;
  c.tgt_len = 34;
  c.min_len = 3;
  c.copy_task = 1;
  const size_t ns = (size_t)c.batch * c.src_len, nt = (size_t)c.batch * c.tgt_len;
  std::vector<int64_t> s(ns), t(nt), s2(ns), t2(nt);
  for (int threads : {1, 3, 8}) {
    Prefetcher pf(c, 4, threads);
    for (int64_t step = 0; step < 40; ++step) {
      if (step == 17) step = 25;  // skip ahead (resume path)
      pf.get(step, s.data(), t.data());
      synth_fill(c, step, s2.data(), t2.data());  // the prefetched batch == direct generation
      CHECK(std::memcmp(s.data(), s2.data(), ns * sizeof(int64_t)) == 0);
      CHECK(std::memcmp(t.data(), t2.data(), nt * sizeof(int64_t)) == 0);
    }
    bool threw = false;
    try {
      pf.get(3, s.data(), t.data());  // going backwards is an error
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
  }
  for (int i = 0; i < 20; ++i) {  // destroyed while workers are mid-batch
    Prefetcher pf(c, 8, 4);
    pf.get(0, s.data(), t.data());
  }
}

static void test_bundle(const std::string& dir) {
  const std::string prefix = dir + "/selftest_bundle";
  std::vector<float> a(1000), b(7);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0.5f * (float)i - 3.f;
  for (size_t i = 0; i < b.size(); ++i) b[i] = -(float)i;
  {
    BundleWriter w(prefix);
    w.add("layer/kernel", 1, {25, 40}, reinterpret_cast<const uint8_t*>(a.data()), a.size() * 4);
    w.add("layer/bias", 1, {7}, reinterpret_cast<const uint8_t*>(b.data()), b.size() * 4);
    w.add_string("_CHECKPOINTABLE_OBJECT_GRAPH", std::string("\x0a\x03\x01\x02\x03", 5));
    w.finish();
  }
  BundleReader r(prefix, true);
  const auto keys = r.keys();
  CHECK(keys.size() == 3);
  const BundleEntry& e = r.entry("layer/kernel");
  CHECK(e.dtype == 1 && e.shape.size() == 2 && e.shape[0] == 25 && e.shape[1] == 40);
  const std::string bytes = r.read("layer/kernel", true);
  CHECK(bytes.size() == a.size() * 4 && std::memcmp(bytes.data(), a.data(), bytes.size()) == 0);
  const std::string bb = r.read("layer/bias", true);
  CHECK(std::memcmp(bb.data(), b.data(), bb.size()) == 0);
  // entry proto round trip and CRC32C masking
  BundleEntry x = decode_entry(encode_entry(e));
  CHECK(x.offset == e.offset && x.size == e.size && x.crc32c == e.crc32c);
  const uint8_t msg[] = "123456789";
  CHECK(crc32c_extend(0, msg, 9) == 0xE3069283u);  // the CRC-32C check value
  CHECK(crc_unmask(crc_mask(0xdeadbeefu)) == 0xdeadbeefu);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const std::string what = argc > 2 ? argv[2] : "all";
  if (what == "all" || what == "prefetch") test_prefetcher();
  if (what == "all" || what == "bundle") test_bundle(dir);
  std::printf("runtime selftest ok (%s)\n", what.c_str());
  return 0;
}
