// mx-cdi-gen: write the ROCm CDI spec for amd.com/gpu.
//   mx-cdi-gen [--root DIR] [--kind amd.com/gpu] [--output /etc/cdi/amd.com-gpu.json] [--check]
// Replaces `nvidia-ctk runtime configure` (/root/reference/README.md:145-149):
// containerd resolves CDI device names returned by the device plugin against
// this file, with the default runc runtime and no shim.
//   --output  write atomically (tmp file + rename) instead of stdout
//   --check   exit 0 iff the file at --output equals what would be generated
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

int main(int argc, char** argv) {
  std::string root, kind = "amd.com/gpu", output;
  bool check = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!std::strcmp(argv[i], "--kind") && i + 1 < argc) kind = argv[++i];
    else if (!std::strcmp(argv[i], "--output") && i + 1 < argc) output = argv[++i];
    else if (!std::strcmp(argv[i], "--check")) check = true;
    else if (!std::strcmp(argv[i], "-h") || !std::strcmp(argv[i], "--help")) {
      std::printf("usage: %s [--root DIR] [--kind K] [--output FILE] [--check]\n", argv[0]);
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  char err[512] = {0};
  long need = mx_cdi_spec(root.c_str(), kind.c_str(), nullptr, 0, err, sizeof(err));
  if (need < 0) {
    std::fprintf(stderr, "mx-cdi-gen: %s\n", err);
    return 1;
  }
  std::vector<char> buf(static_cast<size_t>(need) + 1);
  mx_cdi_spec(root.c_str(), kind.c_str(), buf.data(), buf.size(), err, sizeof(err));
  std::string spec(buf.data(), static_cast<size_t>(need));
  spec += "\n";
  if (output.empty()) {
    std::fputs(spec.c_str(), stdout);
    return 0;
  }
  if (check) {
    std::string cur;
    if (!mx::read_file(output, &cur)) {
      std::fprintf(stderr, "mx-cdi-gen: %s missing\n", output.c_str());
      return 1;
    }
    if (cur != spec) {
      std::fprintf(stderr, "mx-cdi-gen: %s is stale\n", output.c_str());
      return 1;
    }
    return 0;
  }
  const std::string tmp = output + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f) {
    std::perror(tmp.c_str());
    return 1;
  }
  std::fputs(spec.c_str(), f);
  if (std::fclose(f) != 0 || std::rename(tmp.c_str(), output.c_str()) != 0) {
    std::perror(output.c_str());
    return 1;
  }
  return 0;
}
