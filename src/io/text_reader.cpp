// Pipelined text reader (see text_reader.h).
#include "text_reader.h"

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <fstream>
#include <mutex>
#include <thread>

#include "lgbm_amd/log.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

// two blocks: the reader thread fills one while the consumer scans the other
struct BlockPipe {
  std::vector<char> block[2];
  size_t fill[2] = {0, 0};
  bool ready[2] = {false, false};
  bool eof = false;
  bool stop = false;
  std::exception_ptr error;
  std::mutex mu;
  std::condition_variable cv;
};

bool IsBlank(const char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    if (p[i] != ' ' && p[i] != '\t' && p[i] != '\r' && p[i] != '\n' && p[i] != '\f' && p[i] != '\v') return false;
  }
  return true;
}

}  // namespace

void TextReader::ForEachLine(const std::string& path, bool skip_header, const LineFn& fn, size_t block_bytes) {
  if (const char* e = tuning::Get(tuning::Knob::TextBlockBytes)) {  // (tests: lines across block edges)
    block_bytes = static_cast<size_t>(std::max(16L, std::atol(e)));
  }
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (f == nullptr) Log::Fatal("Data file %s doesn't exist.", path.c_str());
  BlockPipe pipe;
  pipe.block[0].resize(block_bytes);
  pipe.block[1].resize(block_bytes);
  std::thread reader([&] {
    try {
      for (int b = 0;; b ^= 1) {
        std::unique_lock<std::mutex> l(pipe.mu);
        pipe.cv.wait(l, [&] { return !pipe.ready[b] || pipe.stop; });
        if (pipe.stop) return;
        l.unlock();
        const size_t got = std::fread(pipe.block[b].data(), 1, block_bytes, f);
        if (got < block_bytes && std::ferror(f)) throw std::runtime_error("read error in " + path);
        l.lock();
        pipe.fill[b] = got;
        pipe.ready[b] = true;
        if (got < block_bytes) pipe.eof = true;
        pipe.cv.notify_all();
        if (pipe.eof) return;
      }
    } catch (...) {
      std::lock_guard<std::mutex> l(pipe.mu);
      pipe.error = std::current_exception();
      pipe.eof = true;
      pipe.cv.notify_all();
    }
  });
  auto finish = [&] {
    {
      std::lock_guard<std::mutex> l(pipe.mu);
      pipe.stop = true;
      pipe.cv.notify_all();
    }
    reader.join();
    std::fclose(f);
  };
  try {
    std::string carry;        // a line that continues into the next block
    int64_t carry_off = 0;
    int64_t pos = 0;          // file offset of the current block
    bool header_pending = skip_header;
    auto emit = [&](const char* p, size_t n, int64_t off) {
      if (n > 0 && p[n - 1] == '\r') --n;
      if (header_pending) {
        header_pending = false;
        return;
      }
      if (IsBlank(p, n)) return;
      fn(p, n, off);
    };
    for (int b = 0;; b ^= 1) {
      size_t n;
      {
        std::unique_lock<std::mutex> l(pipe.mu);
        pipe.cv.wait(l, [&] { return pipe.ready[b] || pipe.error || (pipe.eof && !pipe.ready[b]); });
        if (pipe.error) std::rethrow_exception(pipe.error);
        if (!pipe.ready[b]) break;  // end of file, nothing more
        n = pipe.fill[b];
      }
      const char* d = pipe.block[b].data();
      size_t start = 0;
      for (size_t i = 0; i < n; ++i) {
        if (d[i] != '\n') continue;
        if (!carry.empty()) {
          carry.append(d + start, i - start);
          emit(carry.data(), carry.size(), carry_off);
          carry.clear();
        } else {
          emit(d + start, i - start, pos + static_cast<int64_t>(start));
        }
        start = i + 1;
      }
      if (start < n) {
        if (carry.empty()) carry_off = pos + static_cast<int64_t>(start);
        carry.append(d + start, n - start);
      }
      pos += static_cast<int64_t>(n);
      bool last;
      {
        std::lock_guard<std::mutex> l(pipe.mu);
        pipe.ready[b] = false;
        last = pipe.eof && !pipe.ready[b ^ 1];
        pipe.cv.notify_all();
      }
      if (last) break;
    }
    if (!carry.empty()) emit(carry.data(), carry.size(), carry_off);
  } catch (...) {
    finish();
    throw;
  }
  finish();
}

std::vector<std::string> TextReader::ReadAt(const std::string& path, const std::vector<int64_t>& offsets) {
  std::ifstream f(path, std::ios::binary);
  if (!f) Log::Fatal("Data file %s doesn't exist.", path.c_str());
  std::vector<std::string> out;
  out.reserve(offsets.size());
  std::string line;
  for (int64_t off : offsets) {
    f.seekg(off);
    std::getline(f, line);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    out.push_back(line);
  }
  return out;
}

}  // namespace lgbm_amd
