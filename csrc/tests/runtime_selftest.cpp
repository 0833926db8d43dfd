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

// Malformed index files must fail with an exception, never read out of
// bounds (this runs under ASan/UBSan): every 4-byte window overwritten with
// 0xFFFFFFFF / 0x7FFFFFFF / 0x00000000 (huge restart counts, block handles,
// varints), every truncation, and single-byte flips everywhere.
static void test_malformed_sstable() {
  std::vector<std::pair<std::string, std::string>> kv;
  for (int i = 0; i < 40; ++i) {
    char k[32];
    std::snprintf(k, sizeof(k), "key/%03d/kernel", i);
    kv.emplace_back(k, std::string((size_t)(i % 7) * 3 + 1, (char)('a' + i % 26)));
  }
  const std::string good = build_sstable(kv);
  CHECK(parse_sstable(good, true).size() == kv.size());
  int rejected = 0, parsed = 0;
  auto attempt = [&](const std::string& f, bool verify) {
    try {
      parse_sstable(f, verify);
      ++parsed;
    } catch (const std::exception&) {
      ++rejected;
    }
  };
  for (uint32_t pat : {0xFFFFFFFFu, 0x7FFFFFFFu, 0u}) {
    for (size_t off = 0; off + 4 <= good.size(); ++off) {
      std::string f = good;
      std::memcpy(&f[off], &pat, 4);
      attempt(f, false);
      attempt(f, true);
    }
  }
  for (size_t n = 0; n < good.size(); ++n) attempt(good.substr(0, n), false);
  for (size_t off = 0; off < good.size(); ++off) {
    for (uint8_t x : {(uint8_t)0x80, (uint8_t)0x01, (uint8_t)0xFF}) {
      std::string f = good;
      f[off] = (char)((uint8_t)f[off] ^ x);
      attempt(f, false);
    }
  }
  CHECK(rejected > 0);
  // the entry decoder on garbage
  for (size_t off = 0; off + 4 <= good.size(); off += 3) {
    try {
      decode_entry(good.substr(off, 16));
    } catch (const std::exception&) {
    }
  }
  (void)parsed;
}

// A bundle whose index points past its data file is rejected before any
// allocation of the claimed size.
static void test_bundle_entry_bounds(const std::string& dir) {
  const std::string prefix = dir + "/selftest_bounds";
  std::vector<float> a(16, 1.f);
  {
    BundleWriter w(prefix);
    w.add("x", 1, {16}, reinterpret_cast<const uint8_t*>(a.data()), a.size() * 4);
    w.finish();
  }
  // rewrite the index with a huge offset / size for "x"
  BundleReader ok(prefix, true);
  BundleEntry e = ok.entry("x");
  for (int which = 0; which < 3; ++which) {
    BundleEntry bad = e;
    if (which == 0) bad.offset = (int64_t)1 << 60;
    if (which == 1) bad.size = (int64_t)1 << 60;
    if (which == 2) bad.offset = 60;  // runs past the 64-byte file end
    std::vector<std::pair<std::string, std::string>> kv = {{"", encode_header(1, 1)},
                                                           {"x", encode_entry(bad)}};
    const std::string idx = build_sstable(kv);
    std::FILE* f = std::fopen((prefix + ".index").c_str(), "wb");
    CHECK(f != nullptr);
    std::fwrite(idx.data(), 1, idx.size(), f);
    std::fclose(f);
    BundleReader r(prefix, true);
    bool threw = false;
    try {
      r.read("x", false);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const std::string what = argc > 2 ? argv[2] : "all";
  if (what == "all" || what == "prefetch") test_prefetcher();
  if (what == "all" || what == "bundle") {
    test_bundle(dir);
    test_malformed_sstable();
    test_bundle_entry_bounds(dir);
  }
  std::printf("runtime selftest ok (%s)\n", what.c_str());
  return 0;
}
