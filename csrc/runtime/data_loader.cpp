// Synthetic (source, target) token-pair generator and a multi-threaded
// prefetching loader.
//
// Stands in for the reference's TFDS ted_hrlr_translate/pt_to_en pipeline
// (reference: distributed_training_transformer/english_portugese_dataset.py:
// 21-51: cache -> shuffle -> batch -> tokenize -> pad -> prefetch, auto-sharded
// per worker with AutoShardPolicy.DATA) with batches of the same shape and
// vocabulary: [START] w.. [END] then PAD=0 right-padding, per-rank disjoint
// deterministic streams (the DATA auto-shard analogue), generated ahead of the
// training loop on host threads.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "native_common.h"

namespace tdgn {

namespace {
inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline int uniform(uint64_t& s, int lo, int hi) {  // [lo, hi]
  return lo + (int)(splitmix(s) % (uint64_t)(hi - lo + 1));
}
}  // namespace

void synth_fill(const SynthConfig& c, int64_t step, int64_t* src, int64_t* tgt) {
  if (c.src_len < 2 || c.tgt_len < 2) throw std::runtime_error("synth: lengths must be >= 2");
  const int sv = std::max(c.src_vocab - 4, 1), tv = std::max(c.tgt_vocab - 4, 1);
  for (int b = 0; b < c.batch; ++b) {
    uint64_t s = c.seed * 0x100000001B3ull ^ ((uint64_t)step * 0x9E3779B1ull) ^
                 ((uint64_t)(c.rank) << 48) ^ ((uint64_t)b << 20);
    splitmix(s);
    int ls = c.src_len, lt = c.tgt_len;
    if (c.min_len > 0) {
      ls = uniform(s, std::min(c.min_len, c.src_len), c.src_len);
      lt = c.copy_task ? std::min(ls, c.tgt_len) : uniform(s, std::min(c.min_len, c.tgt_len), c.tgt_len);
    }
    int64_t* sr = src + (size_t)b * c.src_len;
    int64_t* tr = tgt + (size_t)b * c.tgt_len;
    std::fill(sr, sr + c.src_len, 0);
    std::fill(tr, tr + c.tgt_len, 0);
    sr[0] = c.start_id;
    for (int i = 1; i < ls - 1; ++i) sr[i] = 4 + uniform(s, 0, sv - 1);
    sr[ls - 1] = c.end_id;
    tr[0] = c.start_id;
    for (int i = 1; i < lt - 1; ++i) {
      if (c.copy_task && i < ls - 1)
        tr[i] = 4 + (int64_t)(((sr[i] - 4) * 7 + 3) % tv);
      else
        tr[i] = 4 + uniform(s, 0, tv - 1);
    }
    tr[lt - 1] = c.end_id;
  }
}

Prefetcher::Prefetcher(const SynthConfig& c, int depth, int threads)
    : cfg_(c), depth_(std::max(1, depth)) {
  for (int i = 0; i < std::max(1, threads); ++i) threads_.emplace_back([this] { worker(); });
}

Prefetcher::~Prefetcher() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void Prefetcher::worker() {
  for (;;) {
    int64_t step;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || next_ < consumer_ + depth_; });
      if (stop_) return;
      step = next_++;
    }
    std::vector<int64_t> s((size_t)cfg_.batch * cfg_.src_len), t((size_t)cfg_.batch * cfg_.tgt_len);
    synth_fill(cfg_, step, s.data(), t.data());
    {
      std::lock_guard<std::mutex> g(mu_);
      // a skip-ahead (resume) may have passed this step while it was being
      // filled: nobody will consume it, so do not keep it
      if (step >= consumer_) ready_[step] = {std::move(s), std::move(t)};
    }
    cv_.notify_all();
  }
}

void Prefetcher::get(int64_t step, int64_t* src, int64_t* tgt) {
  std::unique_lock<std::mutex> lk(mu_);
  if (step < consumer_) throw std::runtime_error("Prefetcher: steps must be consumed in order");
  if (step > consumer_) {  // skip ahead (resume): drop older batches
    consumer_ = step;
    for (auto it = ready_.begin(); it != ready_.end();)
      it = it->first < step ? ready_.erase(it) : std::next(it);
    if (next_ < step) next_ = step;
    cv_.notify_all();
  }
  cv_.wait(lk, [&] { return ready_.count(step) > 0; });
  auto& e = ready_[step];
  std::memcpy(src, e.first.data(), e.first.size() * sizeof(int64_t));
  std::memcpy(tgt, e.second.data(), e.second.size() * sizeof(int64_t));
  ready_.erase(step);
  consumer_ = step + 1;
  lk.unlock();
  cv_.notify_all();
}

}  // namespace tdgn
