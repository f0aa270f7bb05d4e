// BEP 3 bencode: strict zero-copy decoder (flat node arena, string views borrow the input) and an
// append-only encoder.
//
// Reference: src/bencode.zig:1-368.  Same strictness: rejects leading zeros (:68), "-0" (:70) and
// unsorted / duplicate dict keys (:121-124); error codes keep the reference's names.  Unlike the
// reference, nesting depth is bounded (64) so hostile input cannot exhaust the stack, and the
// encoder can sort dict keys for canonical output.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "common.h"

namespace zest::bencode {

enum class Type : uint8_t { Int, Str, List, Dict };

struct Node {
  Type type;
  int64_t ival = 0;
  std::string_view sval;  // Str payload
  std::string_view key;   // set when this node is a dict value
  uint32_t end = 0;       // index one past this node's subtree
};

class Document;

class Ref {
 public:
  Ref() = default;
  Ref(const Document* d, uint32_t i) : d_(d), i_(i) {}
  bool valid() const { return d_ != nullptr; }
  explicit operator bool() const { return valid(); }
  Type type() const;
  bool is_int() const { return valid() && type() == Type::Int; }
  bool is_str() const { return valid() && type() == Type::Str; }
  bool is_list() const { return valid() && type() == Type::List; }
  bool is_dict() const { return valid() && type() == Type::Dict; }
  int64_t as_int() const;
  std::string_view as_str() const;
  std::string_view key() const;
  // Dict lookup (invalid Ref when missing or not a dict).
  Ref get(std::string_view key) const;
  int64_t get_int(std::string_view key, int64_t dflt) const;
  std::string_view get_str(std::string_view key, std::string_view dflt = {}) const;
  // Children of a list/dict.
  std::vector<Ref> children() const;
  size_t size() const;

 private:
  const Document* d_ = nullptr;
  uint32_t i_ = 0;
};

class Document {
 public:
  // Parse `in` (the Document keeps views into it: `in` must outlive the Document).  Returns the
  // number of bytes consumed; trailing bytes are ignored like the reference decoder.
  size_t parse(std::string_view in);
  Ref root() const { return nodes_.empty() ? Ref() : Ref(this, 0); }
  const std::vector<Node>& nodes() const { return nodes_; }

 private:
  friend class Ref;
  void value(std::string_view in, size_t& pos, int depth, std::string_view key);
  std::vector<Node> nodes_;
};

// Convenience: parse + return root; throws Error on malformed input.
inline Ref decode(Document& doc, std::string_view in) {
  doc.parse(in);
  return doc.root();
}

class Encoder {
 public:
  explicit Encoder(std::string& out) : out_(out) {}
  Encoder& integer(int64_t v);
  Encoder& str(std::string_view s);
  Encoder& begin_list();
  Encoder& begin_dict();
  Encoder& end();
  // dict entry helpers (caller keeps keys sorted for canonical bencode)
  Encoder& key(std::string_view k) { return str(k); }

 private:
  std::string& out_;
};

// Re-encode a decoded value (round-trip; preserves the input's key order).
std::string encode(Ref v);

}  // namespace zest::bencode
