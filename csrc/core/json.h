// Minimal JSON DOM parser + writer for the HF Hub API, the Xet CAS reconstruction document,
// the local REST API (/v1/status) and bench output.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "common.h"

namespace zest::json {

class Value {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };
  Value() = default;
  static Value parse(std::string_view text);  // throws Error("InvalidJson")

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_object() const { return type_ == Type::Object; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_string() const { return type_ == Type::String; }
  bool is_number() const { return type_ == Type::Number; }
  bool as_bool() const { return b_; }
  double as_double() const { return num_; }
  int64_t as_int() const { return is_int_ ? i_ : int64_t(num_); }
  uint64_t as_u64() const { return is_int_ ? uint64_t(i_) : uint64_t(num_); }
  const std::string& as_string() const { return s_; }
  const std::vector<Value>& array() const { return arr_; }
  const std::vector<std::pair<std::string, Value>>& object() const { return obj_; }
  // Object member (static null Value when missing).
  const Value& operator[](std::string_view key) const;
  const Value& at(size_t i) const { return arr_.at(i); }
  size_t size() const { return type_ == Type::Array ? arr_.size() : obj_.size(); }
  bool has(std::string_view key) const;
  std::string str_or(std::string_view key, std::string dflt) const;
  int64_t int_or(std::string_view key, int64_t dflt) const;

 private:
  friend class Parser;
  Type type_ = Type::Null;
  bool b_ = false;
  bool is_int_ = false;
  int64_t i_ = 0;
  double num_ = 0;
  std::string s_;
  std::vector<Value> arr_;
  std::vector<std::pair<std::string, Value>> obj_;
};

std::string escape(std::string_view s);  // quoted JSON string literal

// Tiny streaming writer: w.obj().key("a").num(1).key("b").str("x").end()
class Writer {
 public:
  Writer& obj();
  Writer& arr();
  Writer& end();
  Writer& key(std::string_view k);
  Writer& str(std::string_view v);
  Writer& num(int64_t v);
  Writer& num_u(uint64_t v);
  Writer& num(double v, int precision = 3);
  Writer& boolean(bool v);
  Writer& null();
  Writer& raw(std::string_view json);
  const std::string& out() const { return out_; }

 private:
  void sep();
  std::string out_;
  std::vector<bool> first_;    // per open container: next element is first
  std::vector<char> closers_;  // per open container: '}' or ']'
  bool after_key_ = false;
};

}  // namespace zest::json
