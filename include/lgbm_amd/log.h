// Logging with the reference's user-visible format "[LightGBM] [Info] ..." so that
// log-scraping scripts keep working (reference: include/LightGBM/utils/log.h:71-175).
// Fatal throws std::runtime_error; the C API converts it into an error code.
#pragma once

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace lgbm_amd {

enum class LogLevel : int { Fatal = -1, Warning = 0, Info = 1, Debug = 2 };

class Log {
 public:
  using Callback = void (*)(const char*);
  // (atomics: every C API call sets the level from its parameters, concurrently with the
  // log calls of other threads)
  static void ResetLevel(LogLevel level) { level_().store(level, std::memory_order_relaxed); }
  static LogLevel Level() { return level_().load(std::memory_order_relaxed); }
  static void ResetCallback(Callback cb) { callback_().store(cb, std::memory_order_relaxed); }

  static void Debug(const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); Write(LogLevel::Debug, "Debug", fmt, ap); va_end(ap);
  }
  static void Info(const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); Write(LogLevel::Info, "Info", fmt, ap); va_end(ap);
  }
  static void Warning(const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); Write(LogLevel::Warning, "Warning", fmt, ap); va_end(ap);
  }
  [[noreturn]] static void Fatal(const char* fmt, ...) {
    char buf[2048];
    va_list ap; va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    throw std::runtime_error(std::string(buf));
  }

 private:
  static void Write(LogLevel lvl, const char* tag, const char* fmt, va_list ap) {
    if (static_cast<int>(lvl) > static_cast<int>(Level())) return;
    char buf[4096];
    vsnprintf(buf, sizeof(buf), fmt, ap);
    const Callback cb = callback_().load(std::memory_order_relaxed);
    if (cb != nullptr) {
      std::string s = std::string("[LightGBM] [") + tag + "] " + buf + "\n";
      cb(s.c_str());
    } else {
      fprintf(stdout, "[LightGBM] [%s] %s\n", tag, buf);
      fflush(stdout);
    }
  }
  static std::atomic<LogLevel>& level_() { static std::atomic<LogLevel> l{LogLevel::Info}; return l; }
  static std::atomic<Callback>& callback_() { static std::atomic<Callback> c{nullptr}; return c; }
};

#define LGBM_CHECK(cond) \
  do { if (!(cond)) ::lgbm_amd::Log::Fatal("Check failed: " #cond " at %s, line %d .", __FILE__, __LINE__); } while (0)
#define LGBM_CHECK_EQ(a, b) LGBM_CHECK((a) == (b))
#define LGBM_CHECK_LE(a, b) LGBM_CHECK((a) <= (b))
#define LGBM_CHECK_LT(a, b) LGBM_CHECK((a) < (b))
#define LGBM_CHECK_GE(a, b) LGBM_CHECK((a) >= (b))
#define LGBM_CHECK_GT(a, b) LGBM_CHECK((a) > (b))

}  // namespace lgbm_amd
