// Minimal JSON reader for execution-plan files (the reference parses them with nlohmann::json,
// src/core/executor/execution_plan.cc:124-135; that library is not in this image).  Supports the
// whole JSON grammar; integers keep full uint64 range (plans carry max_message_size = 2^64 - 1).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mscclpp_amd {
namespace json {

struct Value {
  enum Kind { Null, Bool, Int, Uint, Double, String, Array, Object } kind = Null;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double d = 0;
  std::string s;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;  // insertion order kept

  bool isObject() const { return kind == Object; }
  bool isArray() const { return kind == Array; }
  bool contains(const std::string& key) const {
    for (auto& kv : obj)
      if (kv.first == key) return true;
    return false;
  }
  const Value& operator[](const std::string& key) const {
    for (auto& kv : obj)
      if (kv.first == key) return kv.second;
    throw std::runtime_error("json: missing key '" + key + "'");
  }
  const Value& operator[](size_t idx) const {
    if (kind != Array || idx >= arr.size()) throw std::runtime_error("json: index out of range");
    return arr[idx];
  }
  size_t size() const { return kind == Array ? arr.size() : obj.size(); }
  const std::string& str() const {
    if (kind != String) throw std::runtime_error("json: not a string");
    return s;
  }
  uint64_t asU64() const {
    if (kind == Uint) return u;
    if (kind == Int && i >= 0) return (uint64_t)i;
    if (kind == Double && d >= 0) return (uint64_t)d;
    throw std::runtime_error("json: not an unsigned number");
  }
  int64_t asI64() const {
    if (kind == Int) return i;
    if (kind == Uint) return (int64_t)u;
    if (kind == Double) return (int64_t)d;
    throw std::runtime_error("json: not a number");
  }
  bool asBool() const {
    if (kind != Bool) throw std::runtime_error("json: not a bool");
    return b;
  }
  // value(key, default) as nlohmann::json::value
  uint64_t u64Or(const std::string& key, uint64_t def) const { return contains(key) ? (*this)[key].asU64() : def; }
  bool boolOr(const std::string& key, bool def) const { return contains(key) ? (*this)[key].asBool() : def; }
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(text) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t p_ = 0;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(p_));
  }
  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) ++p_;
  }
  char peek() {
    ws();
    if (p_ >= t_.size()) fail("unexpected end");
    return t_[p_];
  }
  void expect(char c) {
    if (peek() != c) fail("unexpected character");
    ++p_;
  }
  bool lit(const char* w) {
    size_t n = std::char_traits<char>::length(w);
    if (t_.compare(p_, n, w) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  Value value() {
    char c = peek();
    Value v;
    if (c == '{') {
      v.kind = Value::Object;
      ++p_;
      if (peek() == '}') {
        ++p_;
        return v;
      }
      for (;;) {
        std::string k = string();
        expect(':');
        v.obj.emplace_back(std::move(k), value());
        char d = peek();
        ++p_;
        if (d == '}') break;
        if (d != ',') fail("expected , or }");
      }
    } else if (c == '[') {
      v.kind = Value::Array;
      ++p_;
      if (peek() == ']') {
        ++p_;
        return v;
      }
      for (;;) {
        v.arr.push_back(value());
        char d = peek();
        ++p_;
        if (d == ']') break;
        if (d != ',') fail("expected , or ]");
      }
    } else if (c == '"') {
      v.kind = Value::String;
      v.s = string();
    } else if (lit("true")) {
      v.kind = Value::Bool;
      v.b = true;
    } else if (lit("false")) {
      v.kind = Value::Bool;
    } else if (lit("null")) {
      v.kind = Value::Null;
    } else {
      number(v);
    }
    return v;
  }
  std::string string() {
    expect('"');
    std::string out;
    while (p_ < t_.size() && t_[p_] != '"') {
      char c = t_[p_++];
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (p_ >= t_.size()) fail("bad escape");
      char e = t_[p_++];
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'u': {
          if (p_ + 4 > t_.size()) fail("bad \\u escape");
          unsigned cp = (unsigned)std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
          p_ += 4;
          if (cp < 0x80) {
            out.push_back((char)cp);
          } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
          } else {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
          }
          break;
        }
        default: out.push_back(e);
      }
    }
    if (p_ >= t_.size()) fail("unterminated string");
    ++p_;
    return out;
  }
  void number(Value& v) {
    size_t start = p_;
    bool neg = false, frac = false;
    if (t_[p_] == '-') {
      neg = true;
      ++p_;
    }
    while (p_ < t_.size() && ((t_[p_] >= '0' && t_[p_] <= '9') || t_[p_] == '.' || t_[p_] == 'e' || t_[p_] == 'E' ||
                              t_[p_] == '+' || t_[p_] == '-')) {
      if (t_[p_] == '.' || t_[p_] == 'e' || t_[p_] == 'E') frac = true;
      ++p_;
    }
    if (p_ == start) fail("unexpected character");
    std::string tok = t_.substr(start, p_ - start);
    if (frac) {
      v.kind = Value::Double;
      v.d = std::strtod(tok.c_str(), nullptr);
    } else if (neg) {
      v.kind = Value::Int;
      v.i = std::strtoll(tok.c_str(), nullptr, 10);
    } else {
      v.kind = Value::Uint;
      v.u = std::strtoull(tok.c_str(), nullptr, 10);
    }
  }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace json
}  // namespace mscclpp_amd
