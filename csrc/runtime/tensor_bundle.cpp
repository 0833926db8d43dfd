// TensorFlow TensorBundle (tf.train.Checkpoint / Keras save_weights) reader
// and writer, without TensorFlow.
//
// On-disk format (what the reference's `model.save_weights` writes,
// reference: distributed_training_transformer/checkpoint.py:75-88,
// saved_weights/{1,2}/model_weights.index; decoded in SURVEY.md §2.6):
//   <prefix>.index                : LevelDB-style SSTable, keys sorted bytewise.
//       ""            -> BundleHeaderProto{num_shards, version{producer}}
//       <var key>     -> BundleEntryProto{dtype, shape, shard_id, offset, size, crc32c}
//   <prefix>.data-00000-of-00001  : raw little-endian tensor bytes, no padding,
//                                   in write order.
// SSTable: uncompressed data blocks (prefix-compressed entries, restart
// interval 16) each followed by a 5-byte trailer (type 0 + masked CRC32C),
// an empty metaindex block, an index block of (separator -> BlockHandle) and a
// 48-byte footer ending in magic 0xdb4775248b80fb57.
// CRC32C uses the SSE4.2 crc32 instruction.
#include "native_common.h"

#include <nmmintrin.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace tdgn {

// ------------------------------------------------------------------ CRC32C
uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
static constexpr uint32_t kMaskDelta = 0xa282ead8u;
uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
uint32_t crc_unmask(uint32_t m) {
  const uint32_t rot = m - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}

// ------------------------------------------------------------------ varints / protobuf
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
void put_fixed32(std::string& s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
}
void put_fixed64(std::string& s, uint64_t v) {
  for (int i = 0; i < 8; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
}
bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64 && p < end; shift += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}
uint32_t get_fixed32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
uint64_t get_fixed64(const uint8_t* p) {
  return (uint64_t)get_fixed32(p) | ((uint64_t)get_fixed32(p + 4) << 32);
}

// protobuf field helpers
static void pb_varint(std::string& s, int field, uint64_t v) {
  put_varint(s, ((uint64_t)field << 3) | 0);
  put_varint(s, v);
}
static void pb_bytes(std::string& s, int field, const std::string& b) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, b.size());
  s += b;
}
static void pb_fixed32(std::string& s, int field, uint32_t v) {
  put_varint(s, ((uint64_t)field << 3) | 5);
  put_fixed32(s, v);
}

std::string encode_entry(const BundleEntry& e) {
  std::string s;
  if (e.dtype) pb_varint(s, 1, (uint64_t)e.dtype);
  std::string shape;
  for (int64_t d : e.shape) {
    std::string dim;
    if (d) pb_varint(dim, 1, (uint64_t)d);
    pb_bytes(shape, 2, dim);
  }
  pb_bytes(s, 2, shape);  // TF always emits the shape message (empty for scalars)
  if (e.shard_id) pb_varint(s, 3, (uint64_t)e.shard_id);
  if (e.offset) pb_varint(s, 4, (uint64_t)e.offset);
  if (e.size) pb_varint(s, 5, (uint64_t)e.size);
  if (e.crc32c) pb_fixed32(s, 6, e.crc32c);
  return s;
}

std::string encode_header(int num_shards, int producer) {
  std::string s, ver;
  if (num_shards) pb_varint(s, 1, (uint64_t)num_shards);
  if (producer) pb_varint(ver, 1, (uint64_t)producer);
  pb_bytes(s, 3, ver);
  return s;
}

// Minimal protobuf walker used by the decoders.
struct PbField {
  int field, wire;
  uint64_t v;
  const uint8_t* data;
  size_t len;
};
static std::vector<PbField> pb_parse(const uint8_t* p, size_t n) {
  std::vector<PbField> out;
  const uint8_t* end = p + n;
  while (p < end) {
    uint64_t tag;
    if (!get_varint(p, end, tag)) throw std::runtime_error("protobuf: bad tag");
    PbField f{(int)(tag >> 3), (int)(tag & 7), 0, nullptr, 0};
    if (f.wire == 0) {
      if (!get_varint(p, end, f.v)) throw std::runtime_error("protobuf: bad varint");
    } else if (f.wire == 2) {
      uint64_t l;
      if (!get_varint(p, end, l) || l > (uint64_t)(end - p)) throw std::runtime_error("protobuf: bad length");
      f.data = p;
      f.len = l;
      p += l;
    } else if (f.wire == 5) {
      if (end - p < 4) throw std::runtime_error("protobuf: short fixed32");
      f.v = get_fixed32(p);
      p += 4;
    } else if (f.wire == 1) {
      if (end - p < 8) throw std::runtime_error("protobuf: short fixed64");
      f.v = get_fixed64(p);
      p += 8;
    } else {
      throw std::runtime_error("protobuf: unsupported wire type");
    }
    out.push_back(f);
  }
  return out;
}

BundleEntry decode_entry(const std::string& s) {
  BundleEntry e;
  for (const auto& f : pb_parse((const uint8_t*)s.data(), s.size())) {
    switch (f.field) {
      case 1: e.dtype = (int)f.v; break;
      case 2:
        for (const auto& d : pb_parse(f.data, f.len)) {
          if (d.field != 2) continue;
          int64_t size = 0;
          for (const auto& x : pb_parse(d.data, d.len))
            if (x.field == 1) size = (int64_t)x.v;
          e.shape.push_back(size);
        }
        break;
      case 3: e.shard_id = (int)f.v; break;
      case 4: e.offset = (int64_t)f.v; break;
      case 5: e.size = (int64_t)f.v; break;
      case 6: e.crc32c = (uint32_t)f.v; break;
      case 7: throw std::runtime_error("TensorBundle: sliced tensors are not supported");
      default: break;
    }
  }
  return e;
}

// ------------------------------------------------------------------ SSTable
namespace {
constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr int kRestartInterval = 16;
constexpr size_t kBlockSize = 262144;

struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  int counter = 0;
  std::string last_key;
  bool empty() const { return buf.empty(); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < kRestartInterval) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, key.size() - shared);
    put_varint(buf, value.size());
    buf.append(key.data() + shared, key.size() - shared);
    buf += value;
    last_key = key;
    ++counter;
  }
  size_t estimate() const { return buf.size() + restarts.size() * 4 + 4; }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(out, r);
    put_fixed32(out, (uint32_t)restarts.size());
    return out;
  }
  void reset() {
    buf.clear();
    restarts.assign(1, 0);
    counter = 0;
    last_key.clear();
  }
};

// Bytewise-comparator helpers (LevelDB semantics).
void shortest_separator(std::string& start, const std::string& limit) {
  const size_t mn = std::min(start.size(), limit.size());
  size_t i = 0;
  while (i < mn && start[i] == limit[i]) ++i;
  if (i >= mn) return;
  const uint8_t b = (uint8_t)start[i];
  if (b < 0xff && b + 1 < (uint8_t)limit[i]) {
    start[i] = (char)(b + 1);
    start.resize(i + 1);
  }
}
void short_successor(std::string& key) {
  for (size_t i = 0; i < key.size(); ++i) {
    const uint8_t b = (uint8_t)key[i];
    if (b != 0xff) {
      key[i] = (char)(b + 1);
      key.resize(i + 1);
      return;
    }
  }
}

struct Handle {
  uint64_t offset, size;
};

std::string write_block(std::string& file, const std::string& contents, Handle& h) {
  h.offset = file.size();
  h.size = contents.size();
  file += contents;
  std::string trailer;
  trailer.push_back(0);  // kNoCompression
  uint32_t crc = crc32c_extend(0, (const uint8_t*)contents.data(), contents.size());
  crc = crc32c_extend(crc, (const uint8_t*)trailer.data(), 1);
  put_fixed32(trailer, crc_mask(crc));
  file += trailer;
  return file;
}

std::string read_block(const std::string& file, Handle h, bool verify) {
  // block + 5-byte trailer inside the file, written so no sum can wrap
  if (file.size() < 5 || h.size > file.size() - 5 || h.offset > file.size() - 5 - h.size)
    throw std::runtime_error("sstable: block out of range");
  const std::string contents = file.substr(h.offset, h.size);
  const uint8_t* tr = (const uint8_t*)file.data() + h.offset + h.size;
  if (tr[0] != 0) throw std::runtime_error("sstable: compressed blocks are not supported");
  if (verify) {
    uint32_t crc = crc32c_extend(0, (const uint8_t*)contents.data(), contents.size());
    crc = crc32c_extend(crc, tr, 1);
    if (crc_unmask(get_fixed32(tr + 1)) != crc)
      throw std::runtime_error("sstable: block checksum mismatch");
  }
  return contents;
}

std::vector<std::pair<std::string, std::string>> parse_block(const std::string& b) {
  std::vector<std::pair<std::string, std::string>> out;
  if (b.size() < 4) throw std::runtime_error("sstable: short block");
  const uint32_t nr = get_fixed32((const uint8_t*)b.data() + b.size() - 4);
  // the restart array (nr fixed32 entries) must fit in front of its count
  if ((size_t)nr > (b.size() - 4) / 4) throw std::runtime_error("sstable: corrupt restart count");
  const size_t limit = b.size() - 4 - 4 * (size_t)nr;
  const uint8_t* p = (const uint8_t*)b.data();
  const uint8_t* end = p + limit;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, nonshared) ||
        !get_varint(p, end, vlen) || nonshared > (uint64_t)(end - p) ||
        vlen > (uint64_t)(end - p) - nonshared || shared > key.size())
      throw std::runtime_error("sstable: corrupt entry");
    key.resize(shared);
    key.append((const char*)p, nonshared);
    p += nonshared;
    out.emplace_back(key, std::string((const char*)p, vlen));
    p += vlen;
  }
  return out;
}
}  // namespace

std::string build_sstable(const std::vector<std::pair<std::string, std::string>>& sorted_kv) {
  std::string file;
  BlockBuilder data, index;
  std::string last_key;
  bool pending = false;
  Handle pending_handle{0, 0};
  for (const auto& kv : sorted_kv) {
    if (pending) {
      std::string sep = last_key;
      shortest_separator(sep, kv.first);
      std::string hv;
      put_varint(hv, pending_handle.offset);
      put_varint(hv, pending_handle.size);
      index.add(sep, hv);
      pending = false;
    }
    data.add(kv.first, kv.second);
    last_key = kv.first;
    if (data.estimate() >= kBlockSize) {
      write_block(file, data.finish(), pending_handle);
      data.reset();
      pending = true;
    }
  }
  if (!data.empty()) {
    write_block(file, data.finish(), pending_handle);
    data.reset();
    pending = true;
  }
  BlockBuilder meta;
  Handle meta_h;
  write_block(file, meta.finish(), meta_h);
  if (pending) {
    std::string succ = last_key;
    short_successor(succ);
    std::string hv;
    put_varint(hv, pending_handle.offset);
    put_varint(hv, pending_handle.size);
    index.add(succ, hv);
  }
  Handle index_h;
  write_block(file, index.finish(), index_h);
  std::string footer;
  put_varint(footer, meta_h.offset);
  put_varint(footer, meta_h.size);
  put_varint(footer, index_h.offset);
  put_varint(footer, index_h.size);
  footer.resize(40, '\0');
  put_fixed64(footer, kTableMagic);
  file += footer;
  return file;
}

std::vector<std::pair<std::string, std::string>> parse_sstable(const std::string& file,
                                                               bool verify) {
  if (file.size() < 48) throw std::runtime_error("sstable: file too short");
  const uint8_t* f = (const uint8_t*)file.data() + file.size() - 48;
  if (get_fixed64(f + 40) != kTableMagic) throw std::runtime_error("sstable: bad magic");
  const uint8_t* p = f;
  const uint8_t* end = f + 40;
  Handle meta_h, index_h;
  if (!get_varint(p, end, meta_h.offset) || !get_varint(p, end, meta_h.size) ||
      !get_varint(p, end, index_h.offset) || !get_varint(p, end, index_h.size))
    throw std::runtime_error("sstable: bad footer");
  std::vector<std::pair<std::string, std::string>> out;
  for (const auto& ie : parse_block(read_block(file, index_h, verify))) {
    const uint8_t* hp = (const uint8_t*)ie.second.data();
    const uint8_t* he = hp + ie.second.size();
    Handle h;
    if (!get_varint(hp, he, h.offset) || !get_varint(hp, he, h.size))
      throw std::runtime_error("sstable: bad block handle");
    for (auto& kv : parse_block(read_block(file, h, verify))) out.push_back(std::move(kv));
  }
  return out;
}

// ------------------------------------------------------------------ BundleWriter
BundleWriter::BundleWriter(const std::string& prefix) : prefix_(prefix) {
  data_ = std::fopen((prefix + ".data-00000-of-00001.tmp").c_str(), "wb");
  if (!data_) throw std::runtime_error("BundleWriter: cannot open data file for " + prefix);
}
BundleWriter::~BundleWriter() {
  if (data_) std::fclose(data_);
}
void BundleWriter::add(const std::string& key, int dtype, const std::vector<int64_t>& shape,
                       const uint8_t* bytes, size_t n) {
  if (finished_) throw std::runtime_error("BundleWriter: already finished");
  if (key.empty()) throw std::runtime_error("BundleWriter: empty key is reserved");
  if (entries_.count(key)) throw std::runtime_error("BundleWriter: duplicate key " + key);
  BundleEntry e;
  e.dtype = dtype;
  e.shape = shape;
  e.offset = offset_;
  e.size = (int64_t)n;
  e.crc32c = crc_mask(crc32c_extend(0, bytes, n));
  if (n && std::fwrite(bytes, 1, n, data_) != n) throw std::runtime_error("BundleWriter: write");
  offset_ += (int64_t)n;
  entries_[key] = e;
}
void BundleWriter::add_string(const std::string& key, const std::string& value) {
  // scalar DT_STRING: [varint len][masked crc of lengths][bytes]
  std::string buf;
  put_varint(buf, value.size());
  const uint32_t len32 = (uint32_t)value.size();
  uint32_t crc = crc32c_extend(0, (const uint8_t*)&len32, 4);
  const uint32_t lc = crc_mask(crc);
  put_fixed32(buf, lc);
  crc = crc32c_extend(crc, (const uint8_t*)&lc, 4);
  buf += value;
  crc = crc32c_extend(crc, (const uint8_t*)value.data(), value.size());
  BundleEntry e;
  e.dtype = 7;  // DT_STRING
  e.offset = offset_;
  e.size = (int64_t)buf.size();
  e.crc32c = crc_mask(crc);
  if (std::fwrite(buf.data(), 1, buf.size(), data_) != buf.size())
    throw std::runtime_error("BundleWriter: write");
  offset_ += (int64_t)buf.size();
  entries_[key] = e;
}
void BundleWriter::finish() {
  if (finished_) return;
  std::fclose(data_);
  data_ = nullptr;
  std::vector<std::pair<std::string, std::string>> kv;
  kv.emplace_back("", encode_header(1, 1));
  for (const auto& it : entries_) kv.emplace_back(it.first, encode_entry(it.second));
  const std::string table = build_sstable(kv);
  const std::string tmp = prefix_ + ".index.tmp";
  {
    std::ofstream out(tmp, std::ios::binary);
    out.write(table.data(), (std::streamsize)table.size());
    if (!out) throw std::runtime_error("BundleWriter: index write failed");
  }
  // publish atomically: data first, then the index that references it
  if (std::rename((prefix_ + ".data-00000-of-00001.tmp").c_str(),
                  (prefix_ + ".data-00000-of-00001").c_str()) != 0 ||
      std::rename(tmp.c_str(), (prefix_ + ".index").c_str()) != 0)
    throw std::runtime_error("BundleWriter: rename failed");
  finished_ = true;
}

// ------------------------------------------------------------------ BundleReader
BundleReader::BundleReader(const std::string& prefix, bool verify) : prefix_(prefix) {
  std::ifstream in(prefix + ".index", std::ios::binary);
  if (!in) throw std::runtime_error("BundleReader: cannot open " + prefix + ".index");
  std::string file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  for (auto& kv : parse_sstable(file, verify)) {
    if (kv.first.empty()) {
      for (const auto& f : pb_parse((const uint8_t*)kv.second.data(), kv.second.size()))
        if (f.field == 1) num_shards_ = (int)f.v;
      continue;
    }
    entries_[kv.first] = decode_entry(kv.second);
  }
  if (num_shards_ != 1) throw std::runtime_error("BundleReader: only single-shard bundles");
}
std::vector<std::string> BundleReader::keys() const {
  std::vector<std::string> k;
  for (const auto& it : entries_) k.push_back(it.first);
  return k;
}
const BundleEntry& BundleReader::entry(const std::string& key) const {
  auto it = entries_.find(key);
  if (it == entries_.end()) throw std::runtime_error("BundleReader: no key " + key);
  return it->second;
}
std::string BundleReader::read(const std::string& key, bool verify) const {
  const BundleEntry& e = entry(key);
  std::FILE* f = std::fopen((prefix_ + ".data-00000-of-00001").c_str(), "rb");
  if (!f) throw std::runtime_error("BundleReader: cannot open data file for " + prefix_);
  // entry bounds against the data file before allocating (a corrupt or
  // crafted index may carry any offset / size)
  long fsize = -1;
  if (std::fseek(f, 0, SEEK_END) == 0) fsize = std::ftell(f);
  if (e.offset < 0 || e.size < 0 || fsize < 0 || e.size > fsize || e.offset > fsize - e.size) {
    std::fclose(f);
    throw std::runtime_error("BundleReader: entry out of range for " + key);
  }
  std::string buf((size_t)e.size, '\0');
  if (std::fseek(f, (long)e.offset, SEEK_SET) != 0 ||
      std::fread(&buf[0], 1, (size_t)e.size, f) != (size_t)e.size) {
    std::fclose(f);
    throw std::runtime_error("BundleReader: short read for " + key);
  }
  std::fclose(f);
  if (verify && e.dtype != 7 &&
      crc_mask(crc32c_extend(0, (const uint8_t*)buf.data(), buf.size())) != e.crc32c)
    throw std::runtime_error("BundleReader: crc32c mismatch for " + key);
  if (e.dtype == 7) {  // scalar string: strip length prefix + length crc
    const uint8_t* p = (const uint8_t*)buf.data();
    const uint8_t* end = p + buf.size();
    uint64_t len;
    if (!get_varint(p, end, len) || end - p < 4 || len > (uint64_t)(end - p - 4))
      throw std::runtime_error("BundleReader: bad string tensor " + key);
    return std::string((const char*)p + 4, len);
  }
  return buf;
}

}  // namespace tdgn
