// cl_text.h -- helpers shared by the host runtimes (cl_host.cpp, cg_host.cpp): the
// thread-local error string behind cl_last_error(), and Go-style text parsing used by
// the readTopologyFile / readEventsFile restatements (test_common.go:29-140).
#pragma once
#include <stdint.h>

#include <cstdarg>
#include <fstream>
#include <sstream>
#include <string>
#include <string_view>
#include <vector>

namespace clsnap {

int set_error_v(int code, const char* fmt, va_list ap);
const char* last_error();

// ---------------------------------------------------------------------------
// Go-style text helpers (strings.Fields, strconv.Atoi, FieldsFunc(s, '\n'))
// ---------------------------------------------------------------------------
inline bool go_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

inline std::vector<std::string> go_fields(const std::string& s) {
  std::vector<std::string> f;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && go_space(s[i])) ++i;
    if (i >= s.size()) break;
    size_t j = i;
    while (j < s.size() && !go_space(s[j])) ++j;
    f.emplace_back(s.substr(i, j - i));
    i = j;
  }
  return f;
}

inline bool go_atoi(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  int64_t v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    if (v > (INT64_MAX - (s[i] - '0')) / 10) return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = neg ? -v : v;
  return true;
}

inline std::vector<std::string> go_lines(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('\n', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) out.emplace_back(s.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

// ---- the same helpers over string_views: no per-line or per-field copies, for the
// streaming loaders of large .top / .events files ----------------------
// Non-empty lines in order (strings.FieldsFunc(s, r == '\n')).
struct LineIter {
  std::string_view s;
  size_t i = 0;
  bool next(std::string_view* line) {
    while (i < s.size() && s[i] == '\n') ++i;
    if (i >= s.size()) return false;
    const size_t j = s.find('\n', i);
    const size_t e = j == std::string_view::npos ? s.size() : j;
    *line = s.substr(i, e - i);
    i = e;
    return true;
  }
};

// strings.Fields of a line into f[0..max); returns the field count (which may exceed max).
inline int go_fields_sv(std::string_view s, std::string_view* f, int max) {
  int n = 0;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && go_space(s[i])) ++i;
    if (i >= s.size()) break;
    size_t j = i;
    while (j < s.size() && !go_space(s[j])) ++j;
    if (n < max) f[n] = s.substr(i, j - i);
    ++n;
    i = j;
  }
  return n;
}

inline bool go_atoi_sv(std::string_view s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  int64_t v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    if (v > (INT64_MAX - (s[i] - '0')) / 10) return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = neg ? -v : v;
  return true;
}

inline bool read_file(const char* path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

}  // namespace clsnap
