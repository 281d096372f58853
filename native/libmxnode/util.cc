#include "util.h"

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace mx {

std::string rooted(const std::string& root, const std::string& abs_path) {
  if (root.empty() || root == "/") return abs_path;
  std::string r = root;
  while (r.size() > 1 && r.back() == '/') r.pop_back();
  if (!abs_path.empty() && abs_path[0] == '/') return r + abs_path;
  return r + "/" + abs_path;
}

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::in | std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

bool path_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 || ::lstat(path.c_str(), &st) == 0;
}

bool is_dir(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> names;
  DIR* d = ::opendir(path.c_str());
  if (!d) return names;
  while (struct dirent* e = ::readdir(d)) {
    if (std::strcmp(e->d_name, ".") == 0 || std::strcmp(e->d_name, "..") == 0) continue;
    names.emplace_back(e->d_name);
  }
  ::closedir(d);
  std::sort(names.begin(), names.end());
  return names;
}

bool read_link(const std::string& path, std::string* target) {
  char buf[4096];
  ssize_t n = ::readlink(path.c_str(), buf, sizeof(buf) - 1);
  if (n < 0) return false;
  buf[n] = 0;
  *target = buf;
  return true;
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\t' || s[b] == '\n' || s[b] == '\r')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\n' || s[e - 1] == '\r')) --e;
  return s.substr(b, e - b);
}

std::map<std::string, std::string> parse_properties(const std::string& text) {
  std::map<std::string, std::string> m;
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    line = trim(line);
    if (line.empty()) continue;
    size_t sp = line.find_first_of(" \t");
    if (sp == std::string::npos) {
      m[line] = "";
      continue;
    }
    m[line.substr(0, sp)] = trim(line.substr(sp + 1));
  }
  return m;
}

uint64_t prop_u64(const std::map<std::string, std::string>& p, const char* key, uint64_t dflt) {
  auto it = p.find(key);
  if (it == p.end() || it->second.empty()) return dflt;
  errno = 0;
  char* end = nullptr;
  unsigned long long v = std::strtoull(it->second.c_str(), &end, 0);
  if (errno || end == it->second.c_str()) return dflt;
  return static_cast<uint64_t>(v);
}

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      case '\r': o += "\\r"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

void set_err(char* err, size_t errlen, const std::string& msg) {
  if (!err || errlen == 0) return;
  std::snprintf(err, errlen, "%s", msg.c_str());
}

std::string gfx_name(uint32_t v) {
  if (v == 0) return "";
  const uint32_t major = v / 10000, minor = (v / 100) % 100, step = v % 100;
  char b[32];
  std::snprintf(b, sizeof(b), "gfx%u%x%x", major, minor, step);
  return b;
}

std::string product_name(uint32_t device_id) {
  switch (device_id) {
    case 0x75a3: return "MI355X";
    case 0x75a0: return "MI350X";
    case 0x74a1: return "MI300X";
    case 0x74a5: return "MI325X";
    case 0x74a0: return "MI300A";
    case 0x74b5: return "MI300X-VF";
    case 0x75b3: return "MI355X-VF";
    default: return "";
  }
}

}  // namespace mx
