// Minimal JSON DOM for the extender's request path (no external library in the image).
//
// Parses one document into a flat node array: objects/arrays link their children through
// `first`/`next`, strings are unescaped into one arena, and every value remembers its byte
// span in the source so the raw Pod object can be cached for bind without re-encoding.
// Depth is bounded; any syntax error fails the whole parse (the caller then hands the
// request to the Python path, which produces the reference's error message).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

namespace nanogpu::json {

enum class Type : uint8_t { kNull, kBool, kNum, kStr, kArr, kObj };

struct Node {
  Type type = Type::kNull;
  bool b = false;
  int32_t first = -1;     // first child (arrays / objects)
  int32_t next = -1;      // next sibling
  int32_t count = 0;      // children
  uint32_t key_off = 0, key_len = 0;  // member key (arena or source, see Doc::kInSrc), objects' children only
  uint32_t str_off = 0, str_len = 0;  // string value (arena or source) or number text (source)
  uint32_t src_begin = 0, src_end = 0;
};

class Doc {
 public:
  bool parse(std::string_view src);
  // One value at the start of `src` (leading whitespace skipped); `*end` gets the offset just
  // past it. Whatever follows is the caller's business (a member of an enclosing document).
  bool parse_prefix(std::string_view src, size_t* end);
  // Objects and arrays nested deeper than `max_depth` (the root is depth 0) are checked for
  // balanced brackets and well-formed strings but get no child nodes: they read as empty,
  // and raw() still spans their text. For readers that need a few shallow fields of a large
  // document (the pod watch's filter); a caller that needs more parses again in full.
  bool parse_shallow(std::string_view src, int max_depth);
  const Node& at(int32_t i) const { return nodes_[i]; }
  int32_t root() const { return nodes_.empty() ? -1 : 0; }
  // A string with no escape is not copied: its length carries kInSrc and its offset points
  // into the source; only unescaped text lives in the arena.
  static constexpr uint32_t kInSrc = 0x80000000u;
  std::string_view str(int32_t i) const {
    const Node& n = nodes_[i];
    if (n.type == Type::kNum) return src_.substr(n.str_off, n.str_len);
    return text(n.str_off, n.str_len);
  }
  std::string_view key(int32_t i) const { return text(nodes_[i].key_off, nodes_[i].key_len); }
  std::string_view raw(int32_t i) const { return src_.substr(nodes_[i].src_begin, nodes_[i].src_end - nodes_[i].src_begin); }
  // Member lookup; `ci` = ASCII case-insensitive (Go encoding/json field matching).
  int32_t get(int32_t obj, std::string_view k, bool ci = false) const;
  bool is(int32_t i, Type t) const { return i >= 0 && nodes_[i].type == t; }
  size_t size() const { return nodes_.size(); }
  // skip_container (or its scalar fallback) from offset 0 of `src`: the end offset, -1 = fails
  static long skip_for_test(std::string_view src, bool scalar);
  static bool skip_uses_avx2();   // the AVX2 walk is the one skip_container runs

 private:
  std::string_view text(uint32_t off, uint32_t len) const {
    return (len & kInSrc) ? src_.substr(off, len & ~kInSrc) : std::string_view(arena_).substr(off, len);
  }
  int32_t value(int depth);
  bool string(uint32_t* off, uint32_t* len);
  bool skip_container();
  bool skip_scalar();   // SSE2 fallback of skip_container (and its reference in the tests)
  int max_depth_ = 1 << 30;
  void ws() {
    while (p_ < src_.size() && (src_[p_] == ' ' || src_[p_] == '\n' || src_[p_] == '\r' || src_[p_] == '\t')) ++p_;
  }
  std::string_view src_;
  size_t p_ = 0;
  std::vector<Node> nodes_;
  std::string arena_;
};

// Appends `s` as a JSON string literal (quotes included).
void append_quoted(std::string* out, std::string_view s);
// The same without the quotes.
void append_escaped(std::string* out, std::string_view s);

}  // namespace nanogpu::json
