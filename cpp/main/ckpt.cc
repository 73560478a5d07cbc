// tfk-ckpt: inspect / verify TF V2 checkpoints (tensor bundles) written by the tfk runtime.
//   tfk-ckpt ls <prefix|dir>      list tensors (name dtype shape bytes)
//   tfk-ckpt verify <prefix|dir>  read every tensor and check its crc32c
#include <cstdio>
#include <sys/stat.h>

#include "../runtime/tfbundle.h"

int main(int argc, char** argv) {
  using namespace tfk::ckpt;
  if (argc < 3) { fprintf(stderr, "usage: tfk-ckpt ls|verify <prefix|dir>\n"); return 2; }
  std::string cmd = argv[1], prefix = argv[2];
  struct stat st;
  if (stat(prefix.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) {
    std::string latest;
    if (!read_checkpoint_state(prefix, &latest, nullptr)) { fprintf(stderr, "no checkpoint state in %s\n", prefix.c_str()); return 1; }
    prefix = prefix + "/" + latest;
  }
  BundleReader r;
  std::string err;
  if (!r.open(prefix, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
  long long total = 0;
  for (auto& kv : r.entries()) {
    const Entry& e = kv.second;
    std::string shape = "[";
    for (size_t i = 0; i < e.shape.size(); ++i) shape += (i ? "," : "") + std::to_string(e.shape[i]);
    shape += "]";
    if (cmd == "verify") {
      std::string data;
      if (!r.read(e.name, &data, &err)) { fprintf(stderr, "FAIL %s: %s\n", e.name.c_str(), err.c_str()); return 1; }
    } else {
      printf("%-60s %-9s %-20s %lld\n", e.name.c_str(), dtype_name(e.dtype).c_str(), shape.c_str(), (long long)e.size);
    }
    total += e.size;
  }
  printf("%s: %zu tensors, %lld bytes%s\n", prefix.c_str(), r.entries().size(), total, cmd == "verify" ? ", all crc32c OK" : "");
  return 0;
}
