// Pipelined text reading (reference src/utils/pipeline_reader.h + text_reader.h: a reader
// thread fills one block while the caller consumes the other).  Lines are handed out with
// their byte offset in the file, so a later pass can seek straight to selected lines
// (two_round loading).  Empty (whitespace-only) lines are skipped and a trailing '\r' is
// dropped, as the in-memory reader does.  Errors of the reader thread are rethrown on the
// caller; the thread is always joined.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace lgbm_amd {

class TextReader {
 public:
  // fn(line, length, byte offset of the line); the line is not NUL-terminated
  using LineFn = std::function<void(const char* line, size_t len, int64_t offset)>;
  static void ForEachLine(const std::string& path, bool skip_header, const LineFn& fn,
                          size_t block_bytes = size_t(16) << 20);
  // the lines starting at the given byte offsets (ascending), in that order
  static std::vector<std::string> ReadAt(const std::string& path, const std::vector<int64_t>& offsets);
};

}  // namespace lgbm_amd
