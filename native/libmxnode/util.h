// Small internal helpers for libmxnode (file IO under a fake-able root, JSON).
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace mx {

// Join ROOT and an absolute host path ("" or "/" root = the real host).
std::string rooted(const std::string& root, const std::string& abs_path);

bool read_file(const std::string& path, std::string* out);
bool path_exists(const std::string& path);
bool is_dir(const std::string& path);
std::vector<std::string> list_dir(const std::string& path);   // sorted names, no . / ..
bool read_link(const std::string& path, std::string* target);

// KFD "key value" property files -> map.
std::map<std::string, std::string> parse_properties(const std::string& text);
uint64_t prop_u64(const std::map<std::string, std::string>& p, const char* key, uint64_t dflt = 0);

std::string trim(const std::string& s);
std::string json_escape(const std::string& s);
void set_err(char* err, size_t errlen, const std::string& msg);

// "gfx950" from gfx_target_version 90500 (major*10000 + minor*100 + step,
// minor/step printed in hex as in the LLVM target names).
std::string gfx_name(uint32_t target_version);

// Product name from the PCI device id ("" if unknown).
std::string product_name(uint32_t device_id);

}  // namespace mx
