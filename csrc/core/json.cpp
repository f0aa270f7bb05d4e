#include "json.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace zest::json {

class Parser {
 public:
  explicit Parser(std::string_view t) : t_(t) {}
  Value parse_root() {
    Value v = value(0);
    ws();
    if (p_ != t_.size()) fail("trailing data");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* why) { throw Error("InvalidJson", std::string(why) + " at " + std::to_string(p_)); }
  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) ++p_;
  }
  bool lit(std::string_view s) {
    if (t_.substr(p_, s.size()) == s) {
      p_ += s.size();
      return true;
    }
    return false;
  }
  Value value(int depth) {
    if (depth > 128) fail("too deep");
    ws();
    if (p_ >= t_.size()) fail("unexpected end");
    Value v;
    const char c = t_[p_];
    if (c == '{') {
      ++p_;
      v.type_ = Value::Type::Object;
      ws();
      if (p_ < t_.size() && t_[p_] == '}') {
        ++p_;
        return v;
      }
      while (true) {
        ws();
        if (p_ >= t_.size() || t_[p_] != '"') fail("expected key");
        std::string k = string();
        ws();
        if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
        ++p_;
        v.obj_.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (p_ < t_.size() && t_[p_] == ',') {
          ++p_;
          continue;
        }
        if (p_ < t_.size() && t_[p_] == '}') {
          ++p_;
          return v;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      v.type_ = Value::Type::Array;
      ws();
      if (p_ < t_.size() && t_[p_] == ']') {
        ++p_;
        return v;
      }
      while (true) {
        v.arr_.push_back(value(depth + 1));
        ws();
        if (p_ < t_.size() && t_[p_] == ',') {
          ++p_;
          continue;
        }
        if (p_ < t_.size() && t_[p_] == ']') {
          ++p_;
          return v;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.type_ = Value::Type::String;
      v.s_ = string();
      return v;
    }
    if (lit("true")) {
      v.type_ = Value::Type::Bool;
      v.b_ = true;
      return v;
    }
    if (lit("false")) {
      v.type_ = Value::Type::Bool;
      return v;
    }
    if (lit("null")) return v;
    // number
    size_t s = p_;
    if (p_ < t_.size() && (t_[p_] == '-' || t_[p_] == '+')) ++p_;
    bool is_int = true;
    while (p_ < t_.size()) {
      char d = t_[p_];
      if (d >= '0' && d <= '9') {
        ++p_;
      } else if (d == '.' || d == 'e' || d == 'E' || d == '-' || d == '+') {
        is_int = false;
        ++p_;
      } else {
        break;
      }
    }
    if (s == p_) fail("unexpected character");
    std::string num(t_.substr(s, p_ - s));
    v.type_ = Value::Type::Number;
    if (is_int) {
      int64_t iv = 0;
      auto r = std::from_chars(num.data(), num.data() + num.size(), iv);
      if (r.ec == std::errc()) {
        v.is_int_ = true;
        v.i_ = iv;
        v.num_ = double(iv);
        return v;
      }
    }
    v.num_ = std::strtod(num.c_str(), nullptr);
    return v;
  }
  std::string string() {
    ++p_;  // opening quote
    std::string out;
    while (true) {
      if (p_ >= t_.size()) fail("unterminated string");
      char c = t_[p_++];
      if (c == '"') return out;
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (p_ >= t_.size()) fail("bad escape");
      char e = t_[p_++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          if (p_ + 4 > t_.size()) fail("bad \\u escape");
          uint32_t cp = uint32_t(std::stoul(std::string(t_.substr(p_, 4)), nullptr, 16));
          p_ += 4;
          if (cp >= 0xD800 && cp <= 0xDBFF && p_ + 6 <= t_.size() && t_[p_] == '\\' && t_[p_ + 1] == 'u') {
            uint32_t lo = uint32_t(std::stoul(std::string(t_.substr(p_ + 2, 4)), nullptr, 16));
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (cp < 0x80) {
            out.push_back(char(cp));
          } else if (cp < 0x800) {
            out.push_back(char(0xC0 | (cp >> 6)));
            out.push_back(char(0x80 | (cp & 0x3F)));
          } else if (cp < 0x10000) {
            out.push_back(char(0xE0 | (cp >> 12)));
            out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(char(0x80 | (cp & 0x3F)));
          } else {
            out.push_back(char(0xF0 | (cp >> 18)));
            out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(char(0x80 | (cp & 0x3F)));
          }
          break;
        }
        default: fail("bad escape");
      }
    }
  }
  std::string_view t_;
  size_t p_ = 0;
};

Value Value::parse(std::string_view text) { return Parser(text).parse_root(); }

const Value& Value::operator[](std::string_view key) const {
  static const Value null_value;
  if (type_ != Type::Object) return null_value;
  for (const auto& kv : obj_)
    if (kv.first == key) return kv.second;
  return null_value;
}

bool Value::has(std::string_view key) const {
  if (type_ != Type::Object) return false;
  for (const auto& kv : obj_)
    if (kv.first == key) return true;
  return false;
}

std::string Value::str_or(std::string_view key, std::string dflt) const {
  const Value& v = (*this)[key];
  return v.is_string() ? v.as_string() : dflt;
}

int64_t Value::int_or(std::string_view key, int64_t dflt) const {
  const Value& v = (*this)[key];
  return v.is_number() ? v.as_int() : dflt;
}

std::string escape(std::string_view s) {
  std::string out;
  out.reserve(s.size() + 2);
  out.push_back('"');
  for (char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", unsigned(c));
          out += buf;
        } else {
          out.push_back(c);
        }
    }
  }
  out.push_back('"');
  return out;
}

void Writer::sep() {
  if (after_key_) {
    after_key_ = false;
    return;
  }
  if (!first_.empty()) {
    if (!first_.back()) out_.push_back(',');
    first_.back() = false;
  }
}

Writer& Writer::obj() {
  sep();
  out_.push_back('{');
  first_.push_back(true);
  closers_.push_back('}');
  return *this;
}
Writer& Writer::arr() {
  sep();
  out_.push_back('[');
  first_.push_back(true);
  closers_.push_back(']');
  return *this;
}
Writer& Writer::end() {
  out_.push_back(closers_.back());
  closers_.pop_back();
  first_.pop_back();
  return *this;
}
Writer& Writer::key(std::string_view k) {
  sep();
  out_ += escape(k);
  out_.push_back(':');
  after_key_ = true;
  return *this;
}
Writer& Writer::str(std::string_view v) {
  sep();
  out_ += escape(v);
  return *this;
}
Writer& Writer::num(int64_t v) {
  sep();
  out_ += std::to_string(v);
  return *this;
}
Writer& Writer::num_u(uint64_t v) {
  sep();
  out_ += std::to_string(v);
  return *this;
}
Writer& Writer::num(double v, int precision) {
  sep();
  if (!std::isfinite(v)) {
    out_ += "null";
    return *this;
  }
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.*f", precision, v);
  out_ += buf;
  return *this;
}
Writer& Writer::boolean(bool v) {
  sep();
  out_ += v ? "true" : "false";
  return *this;
}
Writer& Writer::null() {
  sep();
  out_ += "null";
  return *this;
}
Writer& Writer::raw(std::string_view j) {
  sep();
  out_ += j;
  return *this;
}

}  // namespace zest::json
