// JSON DOM parser (see json.h).
#include "nanogpu/json.h"

#include <emmintrin.h>
#include <immintrin.h>
#include <wmmintrin.h>

namespace nanogpu::json {

namespace {
constexpr int kMaxDepth = 64;

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

void put_utf8(std::string* a, uint32_t cp) {
  if (cp < 0x80) {
    a->push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    a->push_back(static_cast<char>(0xC0 | (cp >> 6)));
    a->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    a->push_back(static_cast<char>(0xE0 | (cp >> 12)));
    a->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    a->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    a->push_back(static_cast<char>(0xF0 | (cp >> 18)));
    a->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    a->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    a->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = static_cast<char>(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = static_cast<char>(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}
}  // namespace

bool Doc::parse_shallow(std::string_view src, int max_depth) {
  max_depth_ = max_depth;
  const bool ok = parse(src);
  max_depth_ = 1 << 30;
  return ok;
}

// At an opening bracket: to just past its matching close. Strings are skipped whole (an
// escaped quote does not end one); control characters inside them are rejected as parse()
// would. Sixteen bytes at a time (SSE2, the x86-64 baseline of the extender's host): only the
// bytes that can change the state are looked at one by one. The bodies skipped this way are
// kube-scheduler's node lists (6 KB for 420 sampled nodes) and the pod's deep parts.
namespace {
// The same walk 64 bytes at a time with AVX2 (the extender's hosts: EPYC), as simdjson's stage 1
// classifies bytes: escaped characters from the backslash runs (carry across blocks), string
// interiors from a prefix XOR of the unescaped quotes (carry-less multiply), brackets outside
// strings counted by popcount. A block in which the depth can neither reach zero nor pass the
// limit is taken whole; otherwise its brackets are walked bit by bit. Same verdicts as the
// scalar walk on JSON text; on non-JSON (a backslash outside a string) it fails where the
// scalar walk skipped the byte. `p` is at the opening bracket; on success it is just past the
// matching close.
__attribute__((target("avx2,pclmul,popcnt,bmi"))) bool skip_avx2(const char* s, size_t n, size_t* p, int max_depth) {
  const __m256i quote = _mm256_set1_epi8('"'), bslash = _mm256_set1_epi8('\\'), ctl = _mm256_set1_epi8(0x1f);
  const __m256i lsq = _mm256_set1_epi8('['), rsq = _mm256_set1_epi8(']'), lcu = _mm256_set1_epi8('{'),
                rcu = _mm256_set1_epi8('}');
  const uint64_t even = 0x5555555555555555ULL;
  uint64_t prev_escaped = 0, prev_in_str = 0;
  int depth = 0;
  alignas(32) char pad[64];
  for (size_t b = *p; b < n; b += 64) {
    const char* src = s + b;
    if (n - b < 64) {   // the tail, padded with spaces (neutral outside strings)
      std::memset(pad, ' ', sizeof pad);
      std::memcpy(pad, src, n - b);
      src = pad;
    }
    const __m256i x0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src));
    const __m256i x1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 32));
#define NGPU_EQ(c)                                                                                   \
  (static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x0, (c))))) |    \
   (static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x1, (c))))) << 32))
    uint64_t bs = NGPU_EQ(bslash);
    uint64_t escaped = 0;
    if (bs | prev_escaped) {
      bs &= ~prev_escaped;
      const uint64_t follows = (bs << 1) | prev_escaped;
      const uint64_t odd_starts = bs & ~even & ~follows;
      uint64_t seq_even;
      prev_escaped = __builtin_add_overflow(odd_starts, bs, &seq_even) ? 1 : 0;
      escaped = (even ^ (seq_even << 1)) & follows;
    }
    const uint64_t q = NGPU_EQ(quote) & ~escaped;
    const uint64_t in_str =
        static_cast<uint64_t>(_mm_cvtsi128_si64(_mm_clmulepi64_si128(_mm_set_epi64x(0, static_cast<int64_t>(q)),
                                                                      _mm_set1_epi8(static_cast<char>(0xff)), 0))) ^
        prev_in_str;
    prev_in_str = static_cast<uint64_t>(static_cast<int64_t>(in_str) >> 63);
    const uint64_t ctl_m =
        static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_min_epu8(x0, ctl), x0)))) |
        (static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_min_epu8(x1, ctl), x1))))
         << 32);
    if ((ctl_m & in_str) || (bs & ~in_str)) return false;   // a control character in a string; a stray backslash
    const uint64_t open = (NGPU_EQ(lsq) | NGPU_EQ(lcu)) & ~in_str, close = (NGPU_EQ(rsq) | NGPU_EQ(rcu)) & ~in_str;
#undef NGPU_EQ
    const int no = __builtin_popcountll(open), nc = __builtin_popcountll(close);
    if (depth > nc && depth + no <= max_depth) {
      depth += no - nc;
      continue;
    }
    for (uint64_t oc = open | close; oc; oc &= oc - 1) {
      const int i = __builtin_ctzll(oc);
      if ((open >> i) & 1) {
        if (++depth > max_depth) return false;
      } else if (--depth == 0) {
        *p = b + static_cast<size_t>(i) + 1;
        return true;
      }
    }
  }
  return false;
}

// a static initializer of a shared library may run before libgcc's own CPU-model constructor
const bool kHaveAvx2 = [] {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("pclmul");
}();
}  // namespace

bool Doc::skip_container() {
  if (kHaveAvx2) return skip_avx2(src_.data(), src_.size(), &p_, kMaxDepth);
  return skip_scalar();
}

bool Doc::skip_uses_avx2() { return kHaveAvx2; }

long Doc::skip_for_test(std::string_view src, bool scalar) {
  Doc d;
  d.src_ = src;
  d.p_ = 0;
  const bool ok = scalar ? d.skip_scalar() : d.skip_container();
  return ok ? static_cast<long>(d.p_) : -1;
}

bool Doc::skip_scalar() {
  const char* s = src_.data();
  const size_t n = src_.size();
  int depth = 0;
  bool in_str = false;
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1f);
  const __m128i lsq = _mm_set1_epi8('['), rsq = _mm_set1_epi8(']'), lcu = _mm_set1_epi8('{'), rcu = _mm_set1_epi8('}');
  while (p_ < n) {
    if (p_ + 16 <= n) {
      const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + p_));
      __m128i m;
      if (in_str)   // a quote, a backslash, or a control character (x <= 0x1f unsigned)
        m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, quote), _mm_cmpeq_epi8(x, bslash)),
                         _mm_cmpeq_epi8(_mm_min_epu8(x, ctl), x));
      else
        m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, quote), _mm_cmpeq_epi8(x, lsq)),
                         _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, rsq), _mm_cmpeq_epi8(x, lcu)),
                                      _mm_cmpeq_epi8(x, rcu)));
      const unsigned mask = static_cast<unsigned>(_mm_movemask_epi8(m));
      if (!mask) {
        p_ += 16;
        continue;
      }
      p_ += static_cast<size_t>(__builtin_ctz(mask));
    }
    const unsigned char c = static_cast<unsigned char>(s[p_++]);
    if (in_str) {
      if (c == '"') {
        in_str = false;
      } else if (c == '\\') {
        if (p_ >= n) return false;
        ++p_;
      } else if (c < 0x20) {
        return false;
      }
    } else if (c == '"') {
      in_str = true;
    } else if (c == '{' || c == '[') {
      if (++depth > kMaxDepth) return false;
    } else if (c == '}' || c == ']') {
      if (--depth == 0) return true;
    }
  }
  return false;
}

bool Doc::parse(std::string_view src) {
  src_ = src;
  p_ = 0;
  nodes_.clear();
  arena_.clear();
  nodes_.reserve(src.size() / 8 + 16);
  arena_.reserve(src.size());
  ws();
  if (value(0) < 0) return false;
  ws();
  return p_ == src_.size();
}

bool Doc::parse_prefix(std::string_view src, size_t* end) {
  src_ = src;
  p_ = 0;
  nodes_.clear();
  arena_.clear();
  nodes_.reserve(src.size() / 8 + 16);
  arena_.reserve(src.size());
  max_depth_ = 1 << 30;
  ws();
  if (value(0) < 0) return false;
  *end = p_;
  return true;
}

// The first quote, backslash or control character at or after q (n if none): sixteen bytes at
// a time, the bytes of a string that need no look one by one.
static inline size_t plain_run_end(const char* s, size_t q, size_t n) {
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1f);
  while (q + 16 <= n) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + q));
    const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, quote), _mm_cmpeq_epi8(x, bslash)),
                                   _mm_cmpeq_epi8(_mm_min_epu8(x, ctl), x));
    const unsigned mask = static_cast<unsigned>(_mm_movemask_epi8(m));
    if (mask) return q + static_cast<size_t>(__builtin_ctz(mask));
    q += 16;
  }
  while (q < n) {
    const unsigned char ch = static_cast<unsigned char>(s[q]);
    if (ch == '"' || ch == '\\' || ch < 0x20) break;
    ++q;
  }
  return q;
}

bool Doc::string(uint32_t* off, uint32_t* len) {
  if (p_ >= src_.size() || src_[p_] != '"') return false;
  ++p_;
  const char* s = src_.data();
  const size_t n = src_.size();
  {
    // common case: no escape before the closing quote -> the text stays in the source
    const size_t q = plain_run_end(s, p_, n);
    if (q < n && s[q] == '"') {
      *off = static_cast<uint32_t>(p_);
      *len = static_cast<uint32_t>(q - p_) | kInSrc;
      p_ = q + 1;
      return true;
    }
  }
  *off = static_cast<uint32_t>(arena_.size());
  while (p_ < n) {
    // a run of plain characters is copied in one go; only quotes, escapes and control
    // characters need a look
    const size_t run = p_;
    p_ = plain_run_end(s, p_, n);
    if (p_ > run) arena_.append(s + run, p_ - run);
    if (p_ >= n) return false;
    const char c = s[p_++];
    if (c == '"') {
      *len = static_cast<uint32_t>(arena_.size() - *off);
      return true;
    }
    if (static_cast<unsigned char>(c) < 0x20) return false;
    if (p_ >= src_.size()) return false;
    const char e = src_[p_++];
    switch (e) {
      case '"': arena_.push_back('"'); break;
      case '\\': arena_.push_back('\\'); break;
      case '/': arena_.push_back('/'); break;
      case 'b': arena_.push_back('\b'); break;
      case 'f': arena_.push_back('\f'); break;
      case 'n': arena_.push_back('\n'); break;
      case 'r': arena_.push_back('\r'); break;
      case 't': arena_.push_back('\t'); break;
      case 'u': {
        auto hex4 = [&](uint32_t* v) {
          if (p_ + 4 > src_.size()) return false;
          *v = 0;
          for (int i = 0; i < 4; ++i) {
            const int h = hexval(src_[p_ + i]);
            if (h < 0) return false;
            *v = (*v << 4) | static_cast<uint32_t>(h);
          }
          p_ += 4;
          return true;
        };
        uint32_t cp;
        if (!hex4(&cp)) return false;
        if (cp >= 0xD800 && cp < 0xDC00 && p_ + 1 < src_.size() && src_[p_] == '\\' && src_[p_ + 1] == 'u') {
          p_ += 2;
          uint32_t lo;
          if (!hex4(&lo)) return false;
          if (lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else {
            put_utf8(&arena_, 0xFFFD);
            cp = lo;
          }
        }
        put_utf8(&arena_, cp);
        break;
      }
      default:
        return false;
    }
  }
  return false;
}

int32_t Doc::value(int depth) {
  if (depth > kMaxDepth || p_ >= src_.size()) return -1;
  const int32_t idx = static_cast<int32_t>(nodes_.size());
  nodes_.emplace_back();
  nodes_[idx].src_begin = static_cast<uint32_t>(p_);
  const char c = src_[p_];
  if ((c == '{' || c == '[') && depth >= max_depth_) {
    nodes_[idx].type = c == '{' ? Type::kObj : Type::kArr;
    if (!skip_container()) return -1;
  } else if (c == '{' || c == '[') {
    const bool obj = c == '{';
    nodes_[idx].type = obj ? Type::kObj : Type::kArr;
    ++p_;
    ws();
    int32_t prev = -1;
    if (p_ < src_.size() && src_[p_] == (obj ? '}' : ']')) {
      ++p_;
    } else {
      for (;;) {
        uint32_t koff = 0, klen = 0;
        if (obj) {
          if (!string(&koff, &klen)) return -1;
          ws();
          if (p_ >= src_.size() || src_[p_] != ':') return -1;
          ++p_;
          ws();
        }
        const int32_t child = value(depth + 1);
        if (child < 0) return -1;
        nodes_[child].key_off = koff;
        nodes_[child].key_len = klen;
        if (prev < 0)
          nodes_[idx].first = child;
        else
          nodes_[prev].next = child;
        prev = child;
        nodes_[idx].count += 1;
        ws();
        if (p_ >= src_.size()) return -1;
        if (src_[p_] == ',') {
          ++p_;
          ws();
          continue;
        }
        if (src_[p_] == (obj ? '}' : ']')) {
          ++p_;
          break;
        }
        return -1;
      }
    }
  } else if (c == '"') {
    nodes_[idx].type = Type::kStr;
    uint32_t off, len;
    if (!string(&off, &len)) return -1;
    nodes_[idx].str_off = off;
    nodes_[idx].str_len = len;
  } else if (c == 't' && src_.substr(p_, 4) == "true") {
    nodes_[idx].type = Type::kBool;
    nodes_[idx].b = true;
    p_ += 4;
  } else if (c == 'f' && src_.substr(p_, 5) == "false") {
    nodes_[idx].type = Type::kBool;
    p_ += 5;
  } else if (c == 'n' && src_.substr(p_, 4) == "null") {
    nodes_[idx].type = Type::kNull;
    p_ += 4;
  } else if (c == '-' || (c >= '0' && c <= '9')) {
    nodes_[idx].type = Type::kNum;
    const size_t b = p_;
    if (src_[p_] == '-') ++p_;
    bool digits = false;
    while (p_ < src_.size()) {
      const char d = src_[p_];
      if ((d >= '0' && d <= '9')) {
        digits = true;
      } else if (!(d == '.' || d == 'e' || d == 'E' || d == '+' || d == '-')) {
        break;
      }
      ++p_;
    }
    if (!digits) return -1;
    nodes_[idx].str_off = static_cast<uint32_t>(b);
    nodes_[idx].str_len = static_cast<uint32_t>(p_ - b);
  } else {
    return -1;
  }
  nodes_[idx].src_end = static_cast<uint32_t>(p_);
  return idx;
}

int32_t Doc::get(int32_t obj, std::string_view k, bool ci) const {
  if (obj < 0 || nodes_[obj].type != Type::kObj) return -1;
  int32_t found = -1;
  for (int32_t c = nodes_[obj].first; c >= 0; c = nodes_[c].next) {
    const std::string_view ck = key(c);
    if (ck == k) return c;  // an exact match wins (Go prefers it as well)
    if (ci && found < 0 && ieq(ck, k)) found = c;
  }
  return found;
}

void append_quoted(std::string* out, std::string_view s) {
  out->push_back('"');
  append_escaped(out, s);
  out->push_back('"');
}

void append_escaped(std::string* out, std::string_view s) {
  size_t run = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    const unsigned char u = static_cast<unsigned char>(c);
    if (c != '"' && c != '\\' && u >= 0x20) continue;
    out->append(s.data() + run, i - run);   // the plain run before it, in one copy
    run = i + 1;
    switch (c) {
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      case '\b': out->append("\\b"); break;
      case '\f': out->append("\\f"); break;
      default: {
        static const char* hex = "0123456789abcdef";
        char esc[7] = {'\\', 'u', '0', '0', hex[u >> 4], hex[u & 15], 0};
        out->append(esc, 6);
      }
    }
  }
  out->append(s.data() + run, s.size() - run);
}

}  // namespace nanogpu::json
