#include "tfbundle.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "../common/util.h"

namespace tfk {
namespace ckpt {

static const uint64_t kTableMagic = 0xdb4775248b80fb57ull;

int dtype_size(int dt) {
  switch (dt) {
    case DT_FLOAT: case DT_INT32: return 4;
    case DT_DOUBLE: case DT_INT64: return 8;
    case DT_UINT8: case DT_INT8: case DT_BOOL: return 1;
    case DT_INT16: case DT_BFLOAT16: case DT_HALF: return 2;
    default: return 0;
  }
}
int dtype_from_name(const std::string& s) {
  if (s == "float32" || s == "float") return DT_FLOAT;
  if (s == "float64" || s == "double") return DT_DOUBLE;
  if (s == "int32") return DT_INT32;
  if (s == "int64") return DT_INT64;
  if (s == "uint8") return DT_UINT8;
  if (s == "int8") return DT_INT8;
  if (s == "int16") return DT_INT16;
  if (s == "bool") return DT_BOOL;
  if (s == "bfloat16") return DT_BFLOAT16;
  if (s == "float16" || s == "half") return DT_HALF;
  return 0;
}
std::string dtype_name(int dt) {
  switch (dt) {
    case DT_FLOAT: return "float32";
    case DT_DOUBLE: return "float64";
    case DT_INT32: return "int32";
    case DT_INT64: return "int64";
    case DT_UINT8: return "uint8";
    case DT_INT8: return "int8";
    case DT_INT16: return "int16";
    case DT_BOOL: return "bool";
    case DT_BFLOAT16: return "bfloat16";
    case DT_HALF: return "float16";
    default: return "unknown";
  }
}

// ------------------------------------------------------------------------------ wire format
void put_varint64(std::string* dst, uint64_t v) {
  while (v >= 0x80) {
    dst->push_back((char)(v | 0x80));
    v >>= 7;
  }
  dst->push_back((char)v);
}
static void put_varint32(std::string* d, uint32_t v) { put_varint64(d, v); }
static void put_fixed32(std::string* d, uint32_t v) {
  char b[4];
  memcpy(b, &v, 4);
  d->append(b, 4);
}
static void put_fixed64(std::string* d, uint64_t v) {
  char b[8];
  memcpy(b, &v, 8);
  d->append(b, 8);
}
bool get_varint64(const char** p, const char* limit, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && *p < limit; shift += 7) {
    uint64_t b = (unsigned char)**p;
    (*p)++;
    r |= (b & 0x7f) << shift;
    if (!(b & 0x80)) { *v = r; return true; }
  }
  return false;
}
static uint32_t get_fixed32(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

// protobuf helpers
static void pb_tag(std::string* d, int field, int wt) { put_varint32(d, (uint32_t)(field << 3 | wt)); }
static void pb_varint(std::string* d, int field, uint64_t v) { pb_tag(d, field, 0); put_varint64(d, v); }
static void pb_bytes(std::string* d, int field, const std::string& s) {
  pb_tag(d, field, 2);
  put_varint64(d, s.size());
  d->append(s);
}

std::string encode_header(int num_shards) {
  std::string h, ver;
  pb_varint(&ver, 1, 1);  // VersionDef.producer = 1
  if (num_shards != 0) pb_varint(&h, 1, (uint64_t)num_shards);
  // endianness LITTLE = 0 (default, omitted)
  pb_bytes(&h, 3, ver);
  return h;
}

std::string encode_entry(const Entry& e) {
  std::string s, shape;
  for (int64_t d : e.shape) {
    std::string dim;
    pb_varint(&dim, 1, (uint64_t)d);
    pb_bytes(&shape, 2, dim);
  }
  if (e.dtype) pb_varint(&s, 1, (uint64_t)e.dtype);
  pb_bytes(&s, 2, shape);
  if (e.shard_id) pb_varint(&s, 3, (uint64_t)e.shard_id);
  if (e.offset) pb_varint(&s, 4, (uint64_t)e.offset);
  if (e.size) pb_varint(&s, 5, (uint64_t)e.size);
  pb_tag(&s, 6, 5);
  put_fixed32(&s, e.crc32c);
  return s;
}

static bool skip_field(const char** p, const char* lim, int wt) {
  uint64_t v;
  if (wt == 0) return get_varint64(p, lim, &v);
  if (wt == 1) { *p += 8; return *p <= lim; }
  if (wt == 5) { *p += 4; return *p <= lim; }
  if (wt == 2) {
    if (!get_varint64(p, lim, &v)) return false;
    *p += v;
    return *p <= lim;
  }
  return false;
}

bool decode_entry(const std::string& s, Entry* e) {
  const char* p = s.data();
  const char* lim = p + s.size();
  while (p < lim) {
    uint64_t tag;
    if (!get_varint64(&p, lim, &tag)) return false;
    int field = (int)(tag >> 3), wt = (int)(tag & 7);
    uint64_t v;
    if (field == 1 && wt == 0) { if (!get_varint64(&p, lim, &v)) return false; e->dtype = (int)v; }
    else if (field == 2 && wt == 2) {
      if (!get_varint64(&p, lim, &v)) return false;
      const char* sl = p + v;
      while (p < sl) {
        uint64_t t2;
        if (!get_varint64(&p, sl, &t2)) return false;
        if ((t2 >> 3) == 2 && (t2 & 7) == 2) {
          uint64_t dl;
          if (!get_varint64(&p, sl, &dl)) return false;
          const char* dlim = p + dl;
          int64_t size = 0;
          while (p < dlim) {
            uint64_t t3;
            if (!get_varint64(&p, dlim, &t3)) return false;
            if ((t3 >> 3) == 1 && (t3 & 7) == 0) { uint64_t sz; get_varint64(&p, dlim, &sz); size = (int64_t)sz; }
            else if (!skip_field(&p, dlim, (int)(t3 & 7))) return false;
          }
          e->shape.push_back(size);
        } else if (!skip_field(&p, sl, (int)(t2 & 7))) return false;
      }
    } else if (field == 3 && wt == 0) { get_varint64(&p, lim, &v); e->shard_id = (int)v; }
    else if (field == 4 && wt == 0) { get_varint64(&p, lim, &v); e->offset = (int64_t)v; }
    else if (field == 5 && wt == 0) { get_varint64(&p, lim, &v); e->size = (int64_t)v; }
    else if (field == 6 && wt == 5) { e->crc32c = get_fixed32(p); p += 4; }
    else if (!skip_field(&p, lim, wt)) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------ SSTable
namespace {
class BlockBuilder {
 public:
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < 16) {
      size_t n = std::min(last_.size(), key.size());
      while (shared < n && last_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back((uint32_t)buf_.size());
      counter_ = 0;
    }
    put_varint32(&buf_, (uint32_t)shared);
    put_varint32(&buf_, (uint32_t)(key.size() - shared));
    put_varint32(&buf_, (uint32_t)value.size());
    buf_.append(key.data() + shared, key.size() - shared);
    buf_.append(value);
    last_ = key;
    counter_++;
    entries_++;
  }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) put_fixed32(&out, r);
    put_fixed32(&out, (uint32_t)restarts_.size());
    return out;
  }
  size_t size_estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return entries_ == 0; }
  void reset() {
    buf_.clear();
    restarts_ = {0};
    counter_ = 0;
    entries_ = 0;
    last_.clear();
  }
  BlockBuilder() { restarts_.push_back(0); }

 private:
  std::string buf_, last_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  size_t entries_ = 0;
};

void write_block(std::string* file, const std::string& contents, uint64_t* off, uint64_t* size) {
  *off = file->size();
  *size = contents.size();
  file->append(contents);
  char type = 0;
  uint32_t crc = crc32c(contents.data(), contents.size());
  crc = crc32c(&type, 1, crc);
  file->push_back(type);
  put_fixed32(file, crc32c_mask(crc));
}

std::string handle(uint64_t off, uint64_t size) {
  std::string h;
  put_varint64(&h, off);
  put_varint64(&h, size);
  return h;
}

bool read_block(const std::string& file, uint64_t off, uint64_t size, std::string* out, std::string* err) {
  if (off + size + 5 > file.size()) { *err = "block out of range"; return false; }
  uint32_t stored = crc32c_unmask(get_fixed32(file.data() + off + size + 1));
  uint32_t crc = crc32c(file.data() + off, size + 1);
  if (crc != stored) { *err = "block checksum mismatch"; return false; }
  if (file[off + size] != 0) { *err = "compressed blocks unsupported"; return false; }
  *out = file.substr(off, size);
  return true;
}

bool iterate_block(const std::string& b, std::vector<std::pair<std::string, std::string>>* kv, std::string* err) {
  if (b.size() < 4) { *err = "short block"; return false; }
  uint32_t nrestarts = get_fixed32(b.data() + b.size() - 4);
  size_t data_end = b.size() - 4 - (size_t)nrestarts * 4;
  if (data_end > b.size()) { *err = "bad restart array"; return false; }
  const char* p = b.data();
  const char* lim = b.data() + data_end;
  std::string key;
  while (p < lim) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint64(&p, lim, &shared) || !get_varint64(&p, lim, &nonshared) || !get_varint64(&p, lim, &vlen)) {
      *err = "bad entry"; return false;
    }
    if (shared > key.size() || p + nonshared + vlen > lim) { *err = "corrupt entry"; return false; }
    key = key.substr(0, shared) + std::string(p, nonshared);
    p += nonshared;
    kv->push_back({key, std::string(p, vlen)});
    p += vlen;
  }
  return true;
}
}  // namespace

std::string build_table(const std::vector<std::pair<std::string, std::string>>& kv, size_t block_size) {
  std::string file;
  BlockBuilder data, index;
  std::string last_key;
  auto flush = [&]() {
    if (data.empty()) return;
    uint64_t off, size;
    write_block(&file, data.finish(), &off, &size);
    index.add(last_key, handle(off, size));
    data.reset();
  };
  for (auto& e : kv) {
    data.add(e.first, e.second);
    last_key = e.first;
    if (data.size_estimate() >= block_size) flush();
  }
  flush();
  BlockBuilder meta;
  uint64_t moff, msize, ioff, isize;
  write_block(&file, meta.finish(), &moff, &msize);
  write_block(&file, index.finish(), &ioff, &isize);
  std::string footer = handle(moff, msize) + handle(ioff, isize);
  footer.resize(40, '\0');
  put_fixed64(&footer, kTableMagic);
  file += footer;
  return file;
}

bool parse_table(const std::string& file, std::vector<std::pair<std::string, std::string>>* kv, std::string* err) {
  if (file.size() < 48) { *err = "file too short for a table footer"; return false; }
  const char* f = file.data() + file.size() - 48;
  uint64_t magic;
  memcpy(&magic, f + 40, 8);
  if (magic != kTableMagic) { *err = "bad table magic"; return false; }
  const char* p = f;
  uint64_t moff, msize, ioff, isize;
  if (!get_varint64(&p, f + 40, &moff) || !get_varint64(&p, f + 40, &msize) || !get_varint64(&p, f + 40, &ioff) ||
      !get_varint64(&p, f + 40, &isize)) {
    *err = "bad footer"; return false;
  }
  std::string ib;
  if (!read_block(file, ioff, isize, &ib, err)) return false;
  std::vector<std::pair<std::string, std::string>> index;
  if (!iterate_block(ib, &index, err)) return false;
  for (auto& ie : index) {
    const char* hp = ie.second.data();
    uint64_t off, size;
    if (!get_varint64(&hp, hp + ie.second.size(), &off) || !get_varint64(&hp, ie.second.data() + ie.second.size(), &size)) {
      *err = "bad block handle"; return false;
    }
    std::string db;
    if (!read_block(file, off, size, &db, err)) return false;
    if (!iterate_block(db, kv, err)) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------ bundle
static bool write_file_atomic(const std::string& path, const std::string& data, std::string* err) {
  std::string tmp = path + ".tmp" + rand_string(6);
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) { *err = "open " + tmp + ": " + strerror(errno); return false; }
  // Fault injection (k8s-operator.md:5 "disk failure"): TFK_FAULT_CKPT_ENOSPC=<substring> makes
  // writes of matching files fail as a full disk would, half-way through the file.
  const char* fault = getenv("TFK_FAULT_CKPT_ENOSPC");
  const bool inject = fault && *fault && path.find(fault) != std::string::npos;
  size_t off = 0;
  while (off < data.size()) {
    ssize_t n = (inject && off >= data.size() / 2) ? (errno = ENOSPC, -1)
                                                   : write(fd, data.data() + off, inject ? data.size() / 2 - off : data.size() - off);
    if (n < 0) {
      *err = "write " + tmp + ": " + strerror(errno) + (errno == ENOSPC ? " (disk full)" : "");
      close(fd);
      unlink(tmp.c_str());
      return false;
    }
    off += (size_t)n;
  }
  if (fsync(fd) != 0) { *err = "fsync failed"; close(fd); unlink(tmp.c_str()); return false; }
  close(fd);
  if (rename(tmp.c_str(), path.c_str()) != 0) { *err = "rename failed"; unlink(tmp.c_str()); return false; }
  return true;
}

bool write_bundle(const std::string& prefix, std::vector<TensorRef> tensors, std::string* err) {
  std::sort(tensors.begin(), tensors.end(), [](const TensorRef& a, const TensorRef& b) { return a.name < b.name; });
  std::string data;
  size_t total = 0;
  for (auto& t : tensors) total += t.nbytes;
  data.reserve(total);
  std::vector<std::pair<std::string, std::string>> kv;
  kv.push_back({"", encode_header(1)});
  for (size_t i = 0; i < tensors.size(); ++i) {
    auto& t = tensors[i];
    if (t.name.empty()) { *err = "empty tensor name"; return false; }
    if (i && tensors[i - 1].name == t.name) { *err = "duplicate tensor " + t.name; return false; }
    int64_t n = 1;
    for (auto d : t.shape) n *= d;
    if ((size_t)(n * dtype_size(t.dtype)) != t.nbytes) { *err = "size mismatch for " + t.name; return false; }
    Entry e;
    e.name = t.name;
    e.dtype = t.dtype;
    e.shape = t.shape;
    e.offset = (int64_t)data.size();
    e.size = (int64_t)t.nbytes;
    e.crc32c = crc32c_mask(crc32c(t.data, t.nbytes));
    data.append((const char*)t.data, t.nbytes);
    kv.push_back({t.name, encode_entry(e)});
  }
  if (!write_file_atomic(prefix + ".data-00000-of-00001", data, err)) return false;
  return write_file_atomic(prefix + ".index", build_table(kv), err);
}

static bool slurp(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

bool BundleReader::open(const std::string& prefix, std::string* err) {
  prefix_ = prefix;
  std::string idx;
  if (!slurp(prefix + ".index", &idx)) { *err = "cannot read " + prefix + ".index"; return false; }
  std::vector<std::pair<std::string, std::string>> kv;
  if (!parse_table(idx, &kv, err)) return false;
  for (auto& e : kv) {
    if (e.first.empty()) {
      const char* p = e.second.data();
      const char* lim = p + e.second.size();
      while (p < lim) {
        uint64_t tag, v;
        if (!get_varint64(&p, lim, &tag)) break;
        if ((tag >> 3) == 1 && (tag & 7) == 0) { get_varint64(&p, lim, &v); num_shards_ = (int)v; }
        else if (!skip_field(&p, lim, (int)(tag & 7))) break;
      }
      continue;
    }
    Entry en;
    en.name = e.first;
    if (!decode_entry(e.second, &en)) { *err = "corrupt entry " + e.first; return false; }
    entries_[e.first] = en;
  }
  return true;
}

bool BundleReader::read(const std::string& name, std::string* out, std::string* err) const {
  auto it = entries_.find(name);
  if (it == entries_.end()) { *err = "no tensor " + name; return false; }
  const Entry& e = it->second;
  char shard[64];
  snprintf(shard, sizeof shard, ".data-%05d-of-%05d", e.shard_id, num_shards_);
  std::ifstream f(prefix_ + shard, std::ios::binary);
  if (!f) { *err = std::string("cannot open data shard ") + shard; return false; }
  f.seekg(e.offset);
  out->resize((size_t)e.size);
  f.read(&(*out)[0], e.size);
  if (f.gcount() != e.size) { *err = "short read for " + name; return false; }
  if (crc32c_mask(crc32c(out->data(), out->size())) != e.crc32c) { *err = "crc mismatch for " + name; return false; }
  return true;
}

bool write_checkpoint_state(const std::string& dir, const std::string& latest, const std::vector<std::string>& all,
                            std::string* err) {
  std::string s = "model_checkpoint_path: \"" + latest + "\"\n";
  for (auto& a : all) s += "all_model_checkpoint_paths: \"" + a + "\"\n";
  return write_file_atomic(dir + "/checkpoint", s, err);
}

bool read_checkpoint_state(const std::string& dir, std::string* latest, std::vector<std::string>* all) {
  std::string s;
  if (!slurp(dir + "/checkpoint", &s)) return false;
  for (auto& line : split(s, '\n')) {
    size_t a = line.find('"'), b = line.rfind('"');
    if (a == std::string::npos || b <= a) continue;
    std::string v = line.substr(a + 1, b - a - 1);
    if (starts_with(trim(line), "model_checkpoint_path")) *latest = v;
    else if (starts_with(trim(line), "all_model_checkpoint_paths") && all) all->push_back(v);
  }
  return !latest->empty();
}

}  // namespace ckpt
}  // namespace tfk
