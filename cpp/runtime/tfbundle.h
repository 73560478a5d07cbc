// TensorFlow V2 checkpoint ("tensor bundle") writer/reader, dependency-free C++.
// Layout (what TF-era TFJob workloads wrote into the job's train dir):
//   <prefix>.index                   LevelDB-format SSTable: ""->BundleHeaderProto, name->BundleEntryProto
//   <prefix>.data-00000-of-00001     concatenated little-endian tensor bytes
//   <dir>/checkpoint                 text: model_checkpoint_path / all_model_checkpoint_paths
// SSTable details: prefix-compressed block entries, restart interval 16, 5-byte block trailer
// (compression type 0 + masked crc32c), metaindex + index block handles in a 48-byte footer with
// magic 0xdb4775248b80fb57. Protos are hand-encoded (varint / fixed32 wire format).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace tfk {
namespace ckpt {

enum DType { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT16 = 5, DT_INT8 = 6, DT_STRING = 7,
             DT_INT64 = 9, DT_BOOL = 10, DT_BFLOAT16 = 14, DT_HALF = 19 };
int dtype_size(int dt);
int dtype_from_name(const std::string& s);  // "float32", "bfloat16", "int64", ...
std::string dtype_name(int dt);

struct Entry {
  std::string name;
  int dtype = DT_FLOAT;
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc32c = 0;  // masked crc of the tensor bytes
};

struct TensorRef {
  std::string name;
  int dtype;
  std::vector<int64_t> shape;
  const void* data;
  size_t nbytes;
};

// Writes <prefix>.index and <prefix>.data-00000-of-00001 (tmp files + fsync + rename).
bool write_bundle(const std::string& prefix, std::vector<TensorRef> tensors, std::string* err);

class BundleReader {
 public:
  bool open(const std::string& prefix, std::string* err);
  const std::map<std::string, Entry>& entries() const { return entries_; }
  bool has(const std::string& name) const { return entries_.count(name) > 0; }
  // Reads tensor bytes into out (resized); verifies crc. false on error.
  bool read(const std::string& name, std::string* out, std::string* err) const;
  int num_shards() const { return num_shards_; }

 private:
  std::string prefix_;
  std::map<std::string, Entry> entries_;
  int num_shards_ = 1;
};

// "checkpoint" state file
bool write_checkpoint_state(const std::string& dir, const std::string& latest, const std::vector<std::string>& all,
                            std::string* err);
bool read_checkpoint_state(const std::string& dir, std::string* latest, std::vector<std::string>* all);

// low level (exposed for golden-byte tests)
void put_varint64(std::string* dst, uint64_t v);
bool get_varint64(const char** p, const char* limit, uint64_t* v);
std::string encode_header(int num_shards);
std::string encode_entry(const Entry& e);
bool decode_entry(const std::string& s, Entry* e);
std::string build_table(const std::vector<std::pair<std::string, std::string>>& sorted_kv, size_t block_size = 262144);
bool parse_table(const std::string& file, std::vector<std::pair<std::string, std::string>>* kv, std::string* err);

}  // namespace ckpt
}  // namespace tfk
