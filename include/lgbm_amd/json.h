// Minimal JSON value + recursive-descent parser (forced splits / forced bins files,
// reference uses vendored json11: src/io/json11.cpp).
#pragma once

#include <cctype>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/log.h"

namespace lgbm_amd {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };
  Json() = default;
  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_object() const { return type_ == Type::Object; }
  double number_value() const { return num_; }
  int int_value() const { return static_cast<int>(num_); }
  bool bool_value() const { return b_; }
  const std::string& string_value() const { return str_; }
  const std::vector<Json>& array_items() const { return arr_; }
  const std::map<std::string, Json>& object_items() const { return obj_; }
  bool has(const std::string& k) const { return obj_.count(k) > 0; }
  const Json& operator[](const std::string& k) const {
    static const Json null;
    auto it = obj_.find(k);
    return it == obj_.end() ? null : it->second;
  }

  static Json Parse(const std::string& s) {
    size_t i = 0;
    Json j = ParseValue(s, &i);
    return j;
  }

 private:
  static void Skip(const std::string& s, size_t* i) {
    while (*i < s.size() && std::isspace(static_cast<unsigned char>(s[*i]))) ++*i;
  }
  static std::string ParseString(const std::string& s, size_t* i) {
    std::string out;
    ++*i;  // opening quote
    while (*i < s.size() && s[*i] != '"') {
      if (s[*i] == '\\' && *i + 1 < s.size()) {
        ++*i;
        char c = s[*i];
        out.push_back(c == 'n' ? '\n' : (c == 't' ? '\t' : c));
      } else {
        out.push_back(s[*i]);
      }
      ++*i;
    }
    ++*i;
    return out;
  }
  static Json ParseValue(const std::string& s, size_t* i) {
    Skip(s, i);
    Json j;
    if (*i >= s.size()) return j;
    char c = s[*i];
    if (c == '{') {
      j.type_ = Type::Object;
      ++*i;
      Skip(s, i);
      if (s[*i] == '}') { ++*i; return j; }
      while (*i < s.size()) {
        Skip(s, i);
        std::string k = ParseString(s, i);
        Skip(s, i);
        if (s[*i] != ':') Log::Fatal("JSON parse error: expected ':'");
        ++*i;
        j.obj_[k] = ParseValue(s, i);
        Skip(s, i);
        if (s[*i] == ',') { ++*i; continue; }
        if (s[*i] == '}') { ++*i; break; }
        Log::Fatal("JSON parse error in object");
      }
    } else if (c == '[') {
      j.type_ = Type::Array;
      ++*i;
      Skip(s, i);
      if (s[*i] == ']') { ++*i; return j; }
      while (*i < s.size()) {
        j.arr_.push_back(ParseValue(s, i));
        Skip(s, i);
        if (s[*i] == ',') { ++*i; continue; }
        if (s[*i] == ']') { ++*i; break; }
        Log::Fatal("JSON parse error in array");
      }
    } else if (c == '"') {
      j.type_ = Type::String;
      j.str_ = ParseString(s, i);
    } else if (s.compare(*i, 4, "true") == 0) {
      j.type_ = Type::Bool;
      j.b_ = true;
      *i += 4;
    } else if (s.compare(*i, 5, "false") == 0) {
      j.type_ = Type::Bool;
      *i += 5;
    } else if (s.compare(*i, 4, "null") == 0) {
      *i += 4;
    } else {
      j.type_ = Type::Number;
      char* end = nullptr;
      j.num_ = std::strtod(s.c_str() + *i, &end);
      *i = static_cast<size_t>(end - s.c_str());
    }
    return j;
  }

  Type type_ = Type::Null;
  double num_ = 0;
  bool b_ = false;
  std::string str_;
  std::vector<Json> arr_;
  std::map<std::string, Json> obj_;
};

}  // namespace lgbm_amd
