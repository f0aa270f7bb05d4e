#include "bencode.h"

#include <charconv>

namespace zest::bencode {

namespace {
constexpr int kMaxDepth = 64;

size_t parse_uint(std::string_view s, size_t pos, size_t end, uint64_t& out) {
  uint64_t v = 0;
  size_t i = pos;
  for (; i < end; ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') break;
    const uint64_t d = uint64_t(c - '0');
    if (v > (UINT64_MAX - d) / 10) throw Error("InvalidStringLength", "overflow");
    v = v * 10 + d;
  }
  out = v;
  return i;
}
}  // namespace

void Document::value(std::string_view in, size_t& pos, int depth, std::string_view key) {
  if (pos >= in.size()) throw Error("UnexpectedEnd");
  if (depth > kMaxDepth) throw Error("InvalidFormat", "nesting too deep");
  const char c = in[pos];
  const uint32_t self = uint32_t(nodes_.size());
  nodes_.push_back(Node{Type::Int});
  nodes_[self].key = key;
  if (c == 'i') {
    ++pos;
    const size_t start = pos;
    const size_t e = in.find('e', pos);
    if (e == std::string_view::npos) throw Error("UnexpectedEnd");
    std::string_view num = in.substr(start, e - start);
    pos = e + 1;
    if (num.empty()) throw Error("InvalidInteger");
    if (num.size() > 1 && num[0] == '0') throw Error("LeadingZero");
    if (num == "-0") throw Error("NegativeZero");
    if (num.size() > 2 && num[0] == '-' && num[1] == '0') throw Error("LeadingZero");
    int64_t v = 0;
    auto r = std::from_chars(num.data(), num.data() + num.size(), v);
    if (r.ec != std::errc() || r.ptr != num.data() + num.size()) throw Error("InvalidInteger");
    nodes_[self].type = Type::Int;
    nodes_[self].ival = v;
  } else if (c >= '0' && c <= '9') {
    const size_t colon = in.find(':', pos);
    if (colon == std::string_view::npos) throw Error("UnexpectedEnd");
    uint64_t len = 0;
    if (parse_uint(in, pos, colon, len) != colon) throw Error("InvalidStringLength");
    pos = colon + 1;
    if (len > in.size() - pos) throw Error("UnexpectedEnd");
    nodes_[self].type = Type::Str;
    nodes_[self].sval = in.substr(pos, len);
    pos += len;
  } else if (c == 'l') {
    ++pos;
    nodes_[self].type = Type::List;
    while (pos < in.size() && in[pos] != 'e') value(in, pos, depth + 1, {});
    if (pos >= in.size()) throw Error("UnexpectedEnd");
    ++pos;
  } else if (c == 'd') {
    ++pos;
    nodes_[self].type = Type::Dict;
    std::string_view last;
    bool have_last = false;
    while (pos < in.size() && in[pos] != 'e') {
      // key must be a string
      if (in[pos] < '0' || in[pos] > '9') throw Error("InvalidFormat", "dict key must be a string");
      const size_t colon = in.find(':', pos);
      if (colon == std::string_view::npos) throw Error("UnexpectedEnd");
      uint64_t len = 0;
      if (parse_uint(in, pos, colon, len) != colon) throw Error("InvalidStringLength");
      pos = colon + 1;
      if (len > in.size() - pos) throw Error("UnexpectedEnd");
      std::string_view k = in.substr(pos, len);
      pos += len;
      if (have_last && !(last < k)) throw Error("UnsortedDictKeys");
      last = k;
      have_last = true;
      value(in, pos, depth + 1, k);
    }
    if (pos >= in.size()) throw Error("UnexpectedEnd");
    ++pos;
  } else {
    throw Error("InvalidFormat");
  }
  nodes_[self].end = uint32_t(nodes_.size());
}

size_t Document::parse(std::string_view in) {
  nodes_.clear();
  size_t pos = 0;
  value(in, pos, 0, {});
  return pos;
}

Type Ref::type() const { return d_->nodes_[i_].type; }

int64_t Ref::as_int() const {
  if (!is_int()) throw Error("InvalidFormat", "not an integer");
  return d_->nodes_[i_].ival;
}

std::string_view Ref::as_str() const {
  if (!is_str()) throw Error("InvalidFormat", "not a string");
  return d_->nodes_[i_].sval;
}

std::string_view Ref::key() const { return valid() ? d_->nodes_[i_].key : std::string_view(); }

Ref Ref::get(std::string_view k) const {
  if (!is_dict()) return {};
  const auto& n = d_->nodes_;
  uint32_t c = i_ + 1;
  while (c < n[i_].end) {
    if (n[c].key == k) return Ref(d_, c);
    c = n[c].end;
  }
  return {};
}

int64_t Ref::get_int(std::string_view k, int64_t dflt) const {
  Ref r = get(k);
  return r.is_int() ? r.as_int() : dflt;
}

std::string_view Ref::get_str(std::string_view k, std::string_view dflt) const {
  Ref r = get(k);
  return r.is_str() ? r.as_str() : dflt;
}

std::vector<Ref> Ref::children() const {
  std::vector<Ref> out;
  if (!is_list() && !is_dict()) return out;
  const auto& n = d_->nodes_;
  uint32_t c = i_ + 1;
  while (c < n[i_].end) {
    out.emplace_back(d_, c);
    c = n[c].end;
  }
  return out;
}

size_t Ref::size() const {
  if (!is_list() && !is_dict()) return 0;
  const auto& n = d_->nodes_;
  size_t k = 0;
  uint32_t c = i_ + 1;
  while (c < n[i_].end) {
    ++k;
    c = n[c].end;
  }
  return k;
}

Encoder& Encoder::integer(int64_t v) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out_.push_back('i');
  out_.append(buf, size_t(r.ptr - buf));
  out_.push_back('e');
  return *this;
}

Encoder& Encoder::str(std::string_view s) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), uint64_t(s.size()));
  out_.append(buf, size_t(r.ptr - buf));
  out_.push_back(':');
  out_.append(s.data(), s.size());
  return *this;
}

Encoder& Encoder::begin_list() {
  out_.push_back('l');
  return *this;
}
Encoder& Encoder::begin_dict() {
  out_.push_back('d');
  return *this;
}
Encoder& Encoder::end() {
  out_.push_back('e');
  return *this;
}

namespace {
void enc(Encoder& e, Ref v) {
  switch (v.type()) {
    case Type::Int: e.integer(v.as_int()); break;
    case Type::Str: e.str(v.as_str()); break;
    case Type::List:
      e.begin_list();
      for (Ref c : v.children()) enc(e, c);
      e.end();
      break;
    case Type::Dict:
      e.begin_dict();
      for (Ref c : v.children()) {
        e.str(c.key());
        enc(e, c);
      }
      e.end();
      break;
  }
}
}  // namespace

std::string encode(Ref v) {
  std::string out;
  Encoder e(out);
  enc(e, v);
  return out;
}

}  // namespace zest::bencode
