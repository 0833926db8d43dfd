// Host-side native runtime (module `_native`): checkpoint I/O and the data
// loader. Pure C++17 + pybind11, no GPU dependency.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tdgn {

// --- CRC32C (Castagnoli), TF/LevelDB masking
uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
uint32_t crc_mask(uint32_t crc);
uint32_t crc_unmask(uint32_t m);

// --- TensorBundle
struct BundleEntry {
  int dtype = 0;  // TF DataType enum (DT_FLOAT = 1, DT_STRING = 7, ...)
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0;
  int64_t size = 0;
  uint32_t crc32c = 0;  // masked
};

std::string encode_entry(const BundleEntry& e);
BundleEntry decode_entry(const std::string& s);
std::string encode_header(int num_shards, int producer);
std::string build_sstable(const std::vector<std::pair<std::string, std::string>>& sorted_kv);
std::vector<std::pair<std::string, std::string>> parse_sstable(const std::string& file,
                                                               bool verify);

class BundleWriter {
 public:
  explicit BundleWriter(const std::string& prefix);
  ~BundleWriter();
  void add(const std::string& key, int dtype, const std::vector<int64_t>& shape,
           const uint8_t* bytes, size_t n);
  void add_string(const std::string& key, const std::string& value);
  void finish();

 private:
  std::string prefix_;
  std::FILE* data_ = nullptr;
  int64_t offset_ = 0;
  bool finished_ = false;
  std::map<std::string, BundleEntry> entries_;
};

class BundleReader {
 public:
  BundleReader(const std::string& prefix, bool verify);
  std::vector<std::string> keys() const;
  const BundleEntry& entry(const std::string& key) const;
  std::string read(const std::string& key, bool verify) const;
  int num_shards() const { return num_shards_; }

 private:
  std::string prefix_;
  int num_shards_ = 1;
  std::map<std::string, BundleEntry> entries_;
};

// --- Synthetic translation-pair source + prefetching loader
struct SynthConfig {
  uint64_t seed = 0;
  int rank = 0, world = 1;
  int batch = 64;       // per-rank sentence pairs
  int src_len = 128;    // padded source length
  int tgt_len = 129;    // padded target length (incl. START; decoder sees tgt_len-1)
  int src_vocab = 7765, tgt_vocab = 7010;
  int min_len = 0;      // 0 => every sequence full length; else uniform in [min_len, len]
  int start_id = 2, end_id = 3;  // reference tokenizer convention: [START]=2, [END]=3
  int copy_task = 0;    // target = f(source) so that loss can actually decrease
};

void synth_fill(const SynthConfig& c, int64_t step, int64_t* src, int64_t* tgt);

class Prefetcher {
 public:
  Prefetcher(const SynthConfig& c, int depth, int threads);
  ~Prefetcher();
  // Blocks until batch `step` is ready; copies into caller buffers.
  void get(int64_t step, int64_t* src, int64_t* tgt);

 private:
  void worker();
  SynthConfig cfg_;
  int depth_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int64_t, std::pair<std::vector<int64_t>, std::vector<int64_t>>> ready_;
  int64_t next_ = 0;       // next step to hand to a worker
  int64_t consumer_ = 0;   // lowest step not yet consumed
  bool stop_ = false;
  std::vector<std::thread> threads_;
};

}  // namespace tdgn
