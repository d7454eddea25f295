// String / number helpers used by parsers, the config system and model IO.
// Formatting functions reproduce the reference model-text format exactly
// (%.17g for ArrayToString, %g for float/double "fast" arrays; reference
// include/LightGBM/utils/common.h:411-500), and Atof reproduces the reference's
// hand-rolled decimal parser so that binned data is identical (common.h:224-322).
#pragma once

#include <algorithm>
#include <atomic>
#include <exception>
#include <mutex>
#include <cctype>
#include <dlfcn.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <limits>
#include <map>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

#include "lgbm_amd/log.h"
#include "lgbm_amd/meta.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {
namespace common {

inline char tolower_c(char c) { return static_cast<char>(std::tolower(static_cast<unsigned char>(c))); }

inline std::string ToLower(std::string s) {
  std::transform(s.begin(), s.end(), s.begin(), tolower_c);
  return s;
}

inline std::string Trim(std::string s) {
  if (s.empty()) return s;
  size_t b = s.find_first_not_of(" \f\n\r\t\v");
  if (b == std::string::npos) return std::string();
  size_t e = s.find_last_not_of(" \f\n\r\t\v");
  return s.substr(b, e - b + 1);
}

inline std::string RemoveQuotationSymbol(std::string s) {
  if (s.empty()) return s;
  size_t b = s.find_first_not_of("'\"");
  if (b == std::string::npos) return std::string();
  size_t e = s.find_last_not_of("'\"");
  return s.substr(b, e - b + 1);
}

inline bool StartsWith(const std::string& s, const std::string& prefix) {
  return s.size() >= prefix.size() && s.compare(0, prefix.size(), prefix) == 0;
}

inline std::vector<std::string> Split(const char* c_str, char delim) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = c_str; *p; ++p) {
    if (*p == delim) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

// split on any character of `delims`, dropping empty tokens
inline std::vector<std::string> Split(const char* c_str, const char* delims) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = c_str; *p; ++p) {
    if (std::strchr(delims, *p) != nullptr) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

// split keeping empty tokens (used for CSV/TSV rows with missing cells)
inline std::vector<std::string> SplitKeepEmpty(const std::string& s, char delim) {
  std::vector<std::string> out;
  size_t start = 0;
  while (true) {
    size_t pos = s.find(delim, start);
    if (pos == std::string::npos) { out.push_back(s.substr(start)); break; }
    out.push_back(s.substr(start, pos - start));
    start = pos + 1;
  }
  return out;
}

template <typename T>
inline const char* Atoi(const char* p, T* out) {
  while (*p == ' ') ++p;
  int sign = 1;
  if (*p == '-') { sign = -1; ++p; } else if (*p == '+') { ++p; }
  T value = 0;
  for (; *p >= '0' && *p <= '9'; ++p) value = static_cast<T>(value * 10 + (*p - '0'));
  *out = static_cast<T>(sign * value);
  while (*p == ' ') ++p;
  return p;
}

// same recursion order as the reference so rounding of 10^n (n > 22) matches
inline double PowRec(double base, int power) {
  if (power < 0) return 1.0 / PowRec(base, -power);
  if (power == 0) return 1.0;
  if (power % 2 == 0) return PowRec(base * base, power / 2);
  if (power % 3 == 0) return PowRec(base * base * base, power / 3);
  return base * PowRec(base, power - 1);
}

// Decimal parser with the same rounding behaviour as the reference (which is NOT
// strtod: digits are accumulated in double, fraction divided by 10^n).
inline const char* Atof(const char* p, double* out) {
  *out = NAN;
  while (*p == ' ') ++p;
  double sign = 1.0;
  if (*p == '-') { sign = -1.0; ++p; } else if (*p == '+') { ++p; }
  if ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E') {
    double value = 0.0;
    for (; *p >= '0' && *p <= '9'; ++p) value = value * 10.0 + (*p - '0');
    if (*p == '.') {
      double right = 0.0;
      int nn = 0;
      ++p;
      while (*p >= '0' && *p <= '9') { right = (*p - '0') + right * 10.0; ++nn; ++p; }
      value += right / PowRec(10.0, nn);
    }
    bool neg_exp = false;
    double scale = 1.0;
    if (*p == 'e' || *p == 'E') {
      ++p;
      if (*p == '-') { neg_exp = true; ++p; } else if (*p == '+') { ++p; }
      uint32_t e = 0;
      for (; *p >= '0' && *p <= '9'; ++p) e = e * 10 + (*p - '0');
      if (e > 308) e = 308;
      while (e >= 50) { scale *= 1E50; e -= 50; }
      while (e >= 8) { scale *= 1E8; e -= 8; }
      while (e > 0) { scale *= 10.0; e -= 1; }
    }
    *out = sign * (neg_exp ? (value / scale) : (value * scale));
  } else {
    size_t n = 0;
    while (p[n] != '\0' && p[n] != ' ' && p[n] != '\t' && p[n] != ',' && p[n] != '\n' && p[n] != '\r' &&
           p[n] != ':') {
      ++n;
    }
    if (n > 0) {
      std::string tok = ToLower(std::string(p, n));
      if (tok == "na" || tok == "nan" || tok == "null") {
        *out = NAN;
      } else if (tok == "inf" || tok == "infinity") {
        *out = sign * 1e308;
      } else {
        Log::Fatal("Unknown token %s in data file", tok.c_str());
      }
      p += n;
    }
  }
  while (*p == ' ') ++p;
  return p;
}

inline bool AtofAndCheck(const char* p, double* out) { return *Atof(p, out) == '\0'; }
inline bool AtoiAndCheck(const char* p, int* out) { return *Atoi(p, out) == '\0'; }

// Exact round-trip double parse used for model files (thresholds, leaf values).
inline double ParseDoublePrecise(const std::string& s) {
  std::string t = ToLower(Trim(s));
  if (t == "nan" || t == "-nan") return NAN;
  if (t == "inf" || t == "infinity") return std::numeric_limits<double>::infinity();
  if (t == "-inf" || t == "-infinity") return -std::numeric_limits<double>::infinity();
  return std::strtod(t.c_str(), nullptr);
}

template <typename T>
inline std::vector<T> StringToArray(const std::string& s, char delim) {
  std::vector<T> out;
  for (const auto& tok : Split(s.c_str(), delim)) {
    if constexpr (std::is_floating_point<T>::value) {
      out.push_back(static_cast<T>(ParseDoublePrecise(tok)));
    } else {
      long long v = 0;
      Atoi(Trim(tok).c_str(), &v);
      out.push_back(static_cast<T>(v));
    }
  }
  return out;
}

// "[0,1],[2,3]" -> {{0,1},{2,3}}
template <typename T>
inline std::vector<std::vector<T>> StringToArrayOfArrays(const std::string& s, char open, char close, char delim) {
  std::vector<std::vector<T>> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t b = s.find(open, i);
    if (b == std::string::npos) break;
    size_t e = s.find(close, b + 1);
    if (e == std::string::npos) break;
    out.push_back(StringToArray<T>(s.substr(b + 1, e - b - 1), delim));
    i = e + 1;
  }
  return out;
}

template <typename T>
inline std::string Join(const std::vector<T>& v, const char* delim) {
  std::stringstream ss;
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) ss << delim;
    if constexpr (std::is_same<T, int8_t>::value || std::is_same<T, uint8_t>::value) {
      ss << static_cast<int>(v[i]);
    } else {
      ss << v[i];
    }
  }
  return ss.str();
}

inline std::string DoubleToStr(double v) {
  char buf[40];
  snprintf(buf, sizeof(buf), "%.17g", v);
  return std::string(buf);
}

// %.17g per element (thresholds, leaf values/weights)
inline std::string ArrayToString(const std::vector<double>& arr, size_t n) {
  std::string out;
  n = std::min(n, arr.size());
  for (size_t i = 0; i < n; ++i) {
    if (i) out.push_back(' ');
    out += DoubleToStr(arr[i]);
  }
  return out;
}

// %g for floating types, decimal for integers (split_gain, internal_value, counts...)
template <typename T>
inline std::string ArrayToStringFast(const std::vector<T>& arr, size_t n) {
  std::string out;
  n = std::min(n, arr.size());
  char buf[40];
  for (size_t i = 0; i < n; ++i) {
    if (i) out.push_back(' ');
    if constexpr (std::is_floating_point<T>::value) {
      snprintf(buf, sizeof(buf), "%g", static_cast<double>(arr[i]));
    } else if constexpr (std::is_unsigned<T>::value) {
      snprintf(buf, sizeof(buf), "%u", static_cast<unsigned>(arr[i]));
    } else {
      snprintf(buf, sizeof(buf), "%d", static_cast<int>(arr[i]));
    }
    out += buf;
  }
  return out;
}

inline double AvoidInf(double x) {
  if (std::isnan(x)) return 0.0;
  if (x >= 1e300) return 1e300;
  if (x <= -1e300) return -1e300;
  return x;
}

inline float AvoidInf(float x) {
  if (std::isnan(x)) return 0.0f;
  if (x >= 1e38f) return 1e38f;
  if (x <= -1e38f) return -1e38f;
  return x;
}

template <typename T>
inline std::vector<uint32_t> ConstructBitset(const T* vals, int n) {
  std::vector<uint32_t> bits;
  for (int i = 0; i < n; ++i) {
    int word = static_cast<int>(vals[i]) / 32;
    int bit = static_cast<int>(vals[i]) % 32;
    if (static_cast<int>(bits.size()) < word + 1) bits.resize(word + 1, 0);
    bits[word] |= (1u << bit);
  }
  return bits;
}

template <typename T>
LGBM_HD bool FindInBitset(const uint32_t* bits, int n, T pos) {
  int word = static_cast<int>(pos) / 32;
  if (word >= n || pos < 0) return false;
  return (bits[word] >> (static_cast<int>(pos) % 32)) & 1;
}

inline bool CheckDoubleEqualOrdered(double a, double b) { return b <= std::nextafter(a, INFINITY); }
inline double GetDoubleUpperBound(double a) { return std::nextafter(a, INFINITY); }

LGBM_HD int RoundInt(double x) { return static_cast<int>(x + 0.5f); }

template <typename T>
LGBM_HD int Sign(T x) { return (x > T(0)) - (x < T(0)); }

template <typename T>
inline T SafeLog(T x) { return x > 0 ? std::log(x) : -INFINITY; }

inline size_t GetLine(const char* s) {
  const char* b = s;
  while (*s != '\0' && *s != '\n' && *s != '\r') ++s;
  return static_cast<size_t>(s - b);
}

inline const char* SkipNewLine(const char* s) {
  if (*s == '\r') ++s;
  if (*s == '\n') ++s;
  return s;
}

inline void Softmax(std::vector<double>* v) {
  double mx = (*v)[0];
  for (double x : *v) mx = std::max(mx, x);
  double s = 0;
  for (double& x : *v) { x = std::exp(x - mx); s += x; }
  for (double& x : *v) x /= s;
}

inline void Softmax(const double* in, double* out, int n) {
  double mx = in[0];
  for (int i = 1; i < n; ++i) mx = std::max(mx, in[i]);
  double s = 0;
  for (int i = 0; i < n; ++i) { out[i] = std::exp(in[i] - mx); s += out[i]; }
  for (int i = 0; i < n; ++i) out[i] /= s;
}

// stable sort of (keys, values) pairs by key (used by categorical binning)
template <typename K, typename V>
inline void SortPairsByKey(std::vector<K>* keys, std::vector<V>* vals, bool descending) {
  std::vector<size_t> idx(keys->size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  if (descending) {
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return (*keys)[a] > (*keys)[b]; });
  } else {
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return (*keys)[a] < (*keys)[b]; });
  }
  std::vector<K> k2(keys->size());
  std::vector<V> v2(vals->size());
  for (size_t i = 0; i < idx.size(); ++i) { k2[i] = (*keys)[idx[i]]; v2[i] = (*vals)[idx[i]]; }
  *keys = std::move(k2);
  *vals = std::move(v2);
}

// Phase timer: accumulates named scopes, printed at exit when enabled (reference USE_TIMETAG,
// include/LightGBM/utils/common.h:1054-1135).  Always compiled; enabled by LGBM_AMD_TIMETAG=1.
// monotonic wall clock in seconds
inline double NowSeconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class PhaseTimer {
 public:
  static PhaseTimer& Global() { static PhaseTimer t; return t; }
  bool enabled() const { return enabled_; }
  void Add(const std::string& name, double ms) { acc_[name] += ms; cnt_[name] += 1; }
  std::string Report() const {
    std::stringstream ss;
    for (auto& kv : acc_) ss << kv.first << " costs:\t " << kv.second / 1000.0 << " s (" << cnt_.at(kv.first) << ")\n";
    return ss.str();
  }
  void Reset() { acc_.clear(); cnt_.clear(); }
  ~PhaseTimer() { if (enabled_ && !acc_.empty()) fprintf(stdout, "%s", Report().c_str()); }
  PhaseTimer() { const char* e = tuning::Get(tuning::Knob::Timetag); enabled_ = e && e[0] == '1'; }
  void set_enabled(bool e) { enabled_ = e; }
  const std::map<std::string, double>& totals() const { return acc_; }

 private:
  bool enabled_ = false;
  std::map<std::string, double> acc_;
  std::map<std::string, long> cnt_;
};

// roctx ranges under LGBM_AMD_ROCTX=1 (libroctx64 loaded at run time, so the library has no
// link dependency on it): the same scope names as the reference's TIMETAG scopes, visible
// in `rocprofv3 --marker-trace` next to the kernels they launch
struct Roctx {
  using Push = int (*)(const char*);
  using Pop = int (*)();
  Push push = nullptr;
  Pop pop = nullptr;
  static const Roctx& Get() {
    static const Roctx r = [] {
      Roctx x;
      const char* e = tuning::Get(tuning::Knob::Roctx);
      if (e == nullptr || e[0] != '1') return x;
      void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
      if (h == nullptr) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
      if (h == nullptr) return x;
      x.push = reinterpret_cast<Push>(dlsym(h, "roctxRangePushA"));
      x.pop = reinterpret_cast<Pop>(dlsym(h, "roctxRangePop"));
      if (x.push == nullptr || x.pop == nullptr) x.push = nullptr;
      return x;
    }();
    return r;
  }
};

class ScopedTimer {
 public:
  explicit ScopedTimer(const char* name) : name_(name) {
    if (PhaseTimer::Global().enabled()) start_ = std::chrono::steady_clock::now();
    if (Roctx::Get().push != nullptr) Roctx::Get().push(name);
  }
  ~ScopedTimer() {
    if (Roctx::Get().push != nullptr) Roctx::Get().pop();
    if (PhaseTimer::Global().enabled()) {
      auto d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start_).count();
      PhaseTimer::Global().Add(name_, d);
    }
  }

 private:
  const char* name_;
  std::chrono::steady_clock::time_point start_;
};

// Exceptions may not leave an OpenMP structured block (the runtime would terminate the
// process): parallel loop bodies run through Run(), which keeps the first exception, and the
// thread that opened the region rethrows it with Check() after the loop (reference
// OMP_INIT_EX / OMP_LOOP_EX_BEGIN / OMP_THROW_EX, include/LightGBM/utils/openmp_wrapper.h).
class OmpErrors {
 public:
  template <typename F>
  void Run(F&& body) {
    if (failed_.load(std::memory_order_relaxed)) return;  // stop early once a body failed
    try {
      body();
    } catch (...) {
      std::lock_guard<std::mutex> l(mu_);
      if (!error_) error_ = std::current_exception();
      failed_.store(true, std::memory_order_relaxed);
    }
  }
  void Check() {
    if (error_) std::rethrow_exception(error_);
  }

 private:
  std::exception_ptr error_;
  std::atomic<bool> failed_{false};
  std::mutex mu_;
};

}  // namespace common
}  // namespace lgbm_amd
