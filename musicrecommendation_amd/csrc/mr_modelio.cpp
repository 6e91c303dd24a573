// mr_modelio.cpp — model files of the reference (host only):
//   writeModelOnFile  MR:489-497  one "user\tsong\tscore\n" line per pair, the
//                                 score as Scala's s"${x}" = java.lang.Double.toString
//   importModelFromFile MR:505-512 parse "user\tsong\tscore" lines (MatchError on
//                                 anything else), sorted (user, song, -score)
// The engine's exchange format is the dense n_test x n_songs model (NaN = no
// pair) over interned names; these calls convert between it and the files.
//
// Double.toString digits: the shortest decimal that reads back to the same
// double, the closest one among those (JDK 19+, JDK-4511638); JDK 8-18's
// FloatingDecimal occasionally printed one more digit (e.g. 2.0E23 as
// 2.0000000000000002E23) — both read back to the same double, so files
// written by either side import identically.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "mr_engine.h"

namespace mr_host {
int fail(int code, const char* fmt, ...);
}

namespace {

using mr_host::fail;

// Shortest round-trip significant digits of finite x != 0: digits (no dot)
// and the decimal exponent e of the first digit (x = d.ddd x 10^e). The JDK 19
// rule: among the decimals of minimal length m that read back to x, the one
// closest to x; when m = 1, the closest among lengths 1 and 2 (so
// Double.MIN_VALUE is 4.9E-324, not 5.0E-324). At each length p the
// correctly rounded p-digit decimal is the closest one; when it does not read
// back (the rounding interval of a power of two is asymmetric, e.g. 2^-24), its
// p-digit neighbours one unit in the last digit away still may: they are
// tried before moving on to p + 1 digits (the closest one that reads back wins).
namespace {
bool reads_back(unsigned long long m, int exp10, double x, long double* dist) {
  char b[48];
  std::snprintf(b, sizeof b, "%llue%d", m, exp10);
  const double y = std::strtod(b, nullptr);
  if (y != std::fabs(x)) return false;
  *dist = std::fabs(std::strtold(b, nullptr) - (long double)std::fabs(x));
  return true;
}
}  // namespace

void shortest_digits(double x, std::string& digits, int& e) {
  char buf[64];
  auto take = [&](const char* str) {
    const char* s = str;
    if (*s == '-') ++s;
    digits.clear();
    for (; *s && *s != 'e'; ++s)
      if (*s >= '0' && *s <= '9') digits.push_back(*s);
    e = std::atoi(s + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  };
  for (int p = 1; p <= 17; ++p) {
    std::snprintf(buf, sizeof buf, "%.*e", p - 1, x);  // correctly rounded to p digits
    if (std::strtod(buf, nullptr) == x || p == 17) {
      if (p == 1) {
        char b2[64];
        std::snprintf(b2, sizeof b2, "%.1e", x);
        if (std::strtod(b2, nullptr) == x) std::memcpy(buf, b2, sizeof b2);
      }
      take(buf);
      return;
    }
    if (p == 1) continue;  // 1-digit neighbours are 2-digit decimals, tried at p = 2
    // neighbours of the p-digit mantissa M (x ~ M * 10^(e - p + 1))
    take(buf);
    unsigned long long m = 0;
    for (char ch : digits) m = m * 10 + (unsigned long long)(ch - '0');
    for (size_t i = digits.size(); i < (size_t)p; ++i) m *= 10;
    const int exp10 = e - p + 1;
    unsigned long long lo_p = 1;
    for (int i = 1; i < p; ++i) lo_p *= 10;  // 10^(p-1): smallest p-digit mantissa
    long double best = 0, d;
    unsigned long long pick = 0;
    for (unsigned long long cand : {m - 1, m + 1}) {
      if (cand < lo_p || cand >= lo_p * 10) continue;  // stays a p-digit decimal
      if (reads_back(cand, exp10, x, &d) && (pick == 0 || d < best)) { best = d; pick = cand; }
    }
    if (pick) {
      digits = std::to_string(pick);
      e = exp10 + p - 1;
      while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
      return;
    }
  }
}

std::string java_double(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
  std::string d;
  int e;
  shortest_digits(x, d, e);
  std::string out = x < 0 ? "-" : "";
  const double a = std::fabs(x);
  if (a >= 1e-3 && a < 1e7) {  // plain decimal, at least one fraction digit
    if (e >= 0) {
      std::string ip = d.substr(0, std::min<size_t>(d.size(), (size_t)e + 1));
      while ((int)ip.size() < e + 1) ip.push_back('0');
      std::string fp = (size_t)e + 1 < d.size() ? d.substr(e + 1) : "0";
      out += ip + "." + fp;
    } else {
      out += "0." + std::string((size_t)(-e - 1), '0') + d;
    }
  } else {  // computerized scientific notation d.dddE[-]n
    out += d.substr(0, 1) + "." + (d.size() > 1 ? d.substr(1) : "0") + "E" + std::to_string(e);
  }
  return out;
}

struct Names {
  std::unordered_map<std::string, int> id;
  int build(const char* const* names, int n, const char* what) {
    id.reserve((size_t)n * 2);
    for (int i = 0; i < n; ++i) {
      if (!names[i]) return fail(MR_E_INVALID, "null %s name %d", what, i);
      if (!id.emplace(names[i], i).second) return fail(MR_E_INVALID, "duplicate %s name %s", what, names[i]);
    }
    return MR_OK;
  }
};

}  // namespace

extern "C" {

int mr_java_double_string(double x, char* buf, int32_t cap) {
  if (!buf || cap <= 0) return fail(MR_E_INVALID, "null or empty buffer");
  const std::string s = java_double(x);
  if ((int32_t)s.size() + 1 > cap) return fail(MR_E_INVALID, "buffer of %d bytes too small", cap);
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

int mr_model_write_tsv(const char* path, int32_t n_test, int32_t n_songs, const char* const* user_names,
                       const char* const* song_names, const double* dense, int32_t order) {
  if (!path || !user_names || !song_names || !dense || n_test < 0 || n_songs < 0)
    return fail(MR_E_INVALID, "bad argument");
  if (order != 0 && order != 1) return fail(MR_E_INVALID, "order %d: 0 = emission (song-major), 1 = sorted", order);
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(MR_E_IO, "cannot open %s for writing", path);
  std::vector<char> big(1 << 20);
  std::setvbuf(f, big.data(), _IOFBF, big.size());
  std::string line;
  auto emit = [&](int u, int s) {
    const double x = dense[(size_t)u * n_songs + s];
    if (std::isnan(x)) return;  // no pair (MR:109)
    line.assign(user_names[u]);
    line.push_back('\t');
    line.append(song_names[s]);
    line.push_back('\t');
    line.append(java_double(x));
    line.push_back('\n');
    std::fwrite(line.data(), 1, line.size(), f);
  };
  if (order == 0) {  // getModel's enumeration: songs outer, users inner (MR:106-108)
    for (int s = 0; s < n_songs; ++s)
      for (int u = 0; u < n_test; ++u) emit(u, s);
  } else {  // the driver's (user, song) order; assumes names sorted like their ids
    for (int u = 0; u < n_test; ++u)
      for (int s = 0; s < n_songs; ++s) emit(u, s);
  }
  const bool bad = std::ferror(f) != 0;
  if (std::fclose(f) != 0 || bad) return fail(MR_E_IO, "write to %s failed", path);
  return MR_OK;
}

int mr_model_read_tsv(const char* path, int32_t n_test, int32_t n_songs, const char* const* user_names,
                      const char* const* song_names, double* dense) {
  if (!path || !user_names || !song_names || !dense || n_test < 0 || n_songs < 0)
    return fail(MR_E_INVALID, "bad argument");
  Names users, songs;
  int rc;
  if ((rc = users.build(user_names, n_test, "user"))) return rc;
  if ((rc = songs.build(song_names, n_songs, "song"))) return rc;
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(MR_E_IO, "cannot open %s", path);
  for (size_t i = 0; i < (size_t)n_test * n_songs; ++i) dense[i] = NAN;
  std::vector<unsigned char> seen((size_t)n_test * n_songs, 0);
  char* buf = nullptr;
  size_t cap = 0;
  ssize_t len;
  size_t lineno = 0;
  rc = MR_OK;
  std::vector<std::string> fld;
  while ((len = getline(&buf, &cap, f)) >= 0) {
    ++lineno;
    std::string l(buf, (size_t)len);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    fld.clear();  // Java split("\t"): trailing empty fields dropped; exactly 3 (MR:508)
    size_t a = 0;
    while (true) {
      const size_t b = l.find('\t', a);
      if (b == std::string::npos) { fld.emplace_back(l.substr(a)); break; }
      fld.emplace_back(l.substr(a, b - a));
      a = b + 1;
    }
    while (!fld.empty() && fld.back().empty()) fld.pop_back();
    if (fld.size() != 3) { rc = fail(MR_E_PARSE, "%s:%zu: expected 3 tab-separated fields", path, lineno); break; }
    const char* num = fld[2].c_str();
    char* end = nullptr;
    errno = 0;
    const double x = std::strtod(num, &end);  // String.toDouble (NaN / Infinity / exponents)
    while (end && (*end == ' ' || *end == 'd' || *end == 'D' || *end == 'f' || *end == 'F')) ++end;
    if (end == num || (end && *end)) {
      rc = fail(MR_E_PARSE, "%s:%zu: bad number '%s' (NumberFormatException)", path, lineno, num);
      break;
    }
    auto ui = users.id.find(fld[0]);
    auto si = songs.id.find(fld[1]);
    if (ui == users.id.end() || si == songs.id.end()) {
      rc = fail(MR_E_INVALID, "%s:%zu: unknown %s '%s'", path, lineno, ui == users.id.end() ? "user" : "song",
                ui == users.id.end() ? fld[0].c_str() : fld[1].c_str());
      break;
    }
    const size_t o = (size_t)ui->second * n_songs + si->second;
    if (seen[o]) { rc = fail(MR_E_INVALID, "%s:%zu: duplicate pair (%s, %s)", path, lineno, fld[0].c_str(), fld[1].c_str()); break; }
    seen[o] = 1;
    dense[o] = x;
  }
  std::free(buf);
  std::fclose(f);
  return rc;
}

}  // extern "C"
