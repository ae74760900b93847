// libprl_data.so: the trainer's input path in native code (include/prl_data.h).
//
// JSON micro-batch codec for the training_data stream (reference: pipelinerl/streams.py:238-277
// writes one JSON document per packed micro-batch, pipelinerl/finetune_loop.py:92-115 decodes it in
// the loader thread into a PipelineBatchEncoding, pipelinerl/finetune/types.py:48-117 validators
// turn lists into tensors with numpy.asarray + torch.as_tensor) and the preprocessing arithmetic of
// populate_rl_data / collate_packed (pipelinerl/finetune/rl/__init__.py:380-501,
// pipelinerl/finetune/data.py:215-279).  Host code only: g++ -O3, no HIP, no Python.
#include "prl_data.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

struct Cursor {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && is_ws(*p)) ++p;
  }
};

// Skip one JSON string starting at '"'; p ends after the closing quote.
bool skip_string(Cursor& c) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  while (c.p < c.e) {
    const char* q = static_cast<const char*>(memchr(c.p, '"', c.e - c.p));
    if (!q) return false;
    // count the backslashes right before the quote: an odd number escapes it
    const char* b = q;
    while (b > c.p && b[-1] == '\\') --b;
    c.p = q + 1;
    if (((q - b) & 1) == 0) return true;
  }
  return false;
}

// Skip one JSON value of any kind (string, number, literal, array, object).
bool skip_value(Cursor& c) {
  c.ws();
  if (c.p >= c.e) return false;
  const char ch = *c.p;
  if (ch == '"') return skip_string(c);
  if (ch == '[' || ch == '{') {
    int depth = 0;
    while (c.p < c.e) {
      const char x = *c.p;
      if (x == '"') {
        if (!skip_string(c)) return false;
        continue;
      }
      if (x == '[' || x == '{') ++depth;
      else if (x == ']' || x == '}') {
        if (--depth == 0) {
          ++c.p;
          return true;
        }
      }
      ++c.p;
    }
    return false;
  }
  const char* s = c.p;
  while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']' && !is_ws(*c.p)) ++c.p;
  return c.p > s;
}

// ---- number tokens ------------------------------------------------------------------------

enum TokKind { TOK_INT = 0, TOK_FLOAT = 1, TOK_BAD = 2 };

// Classify a scalar token [s, t): JSON integer, JSON float / NaN / Infinity, or not a number.
inline TokKind classify(const char* s, const char* t) {
  if (s >= t) return TOK_BAD;
  const char* q = s;
  if (*q == '-') ++q;
  if (q >= t) return TOK_BAD;
  if (*q == 'N' || *q == 'I') return TOK_FLOAT;  // NaN, Infinity, -Infinity
  if (*q < '0' || *q > '9') return TOK_BAD;      // true / false / null / strings
  for (; q < t; ++q)
    if (*q == '.' || *q == 'e' || *q == 'E') return TOK_FLOAT;
  return TOK_INT;
}

inline bool parse_double(const char* s, const char* t, double& v) {
  const char* q = s;
  const bool neg = *q == '-';
  if (neg) ++q;
  if (q < t && (*q == 'N' || *q == 'I')) {
    if (t - q == 3 && !neg && memcmp(q, "NaN", 3) == 0) {
      v = std::numeric_limits<double>::quiet_NaN();
      return true;
    }
    if (t - q == 8 && memcmp(q, "Infinity", 8) == 0) {
      v = neg ? -std::numeric_limits<double>::infinity() : std::numeric_limits<double>::infinity();
      return true;
    }
    return false;
  }
  // Clinger's fast path: a mantissa of at most 2^53 scaled by 10^|e| <= 10^22 is one correctly
  // rounded IEEE multiply / divide of two exact doubles (short literals: 0.0, 1792.0, -0.5, ...)
  {
    static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const char* x = q;
    uint64_t m = 0;
    int nd = 0, scale = 0;
    while (x < t && *x >= '0' && *x <= '9' && nd < 19) {
      m = m * 10 + (*x++ - '0');
      nd += m != 0;
    }
    bool ok = x > q && !(x < t && *x >= '0' && *x <= '9');
    if (ok && x < t && *x == '.') {
      ++x;
      const char* f = x;
      while (x < t && *x >= '0' && *x <= '9' && nd < 19) {
        m = m * 10 + (*x++ - '0');
        nd += m != 0;
        --scale;
      }
      ok = x > f && !(x < t && *x >= '0' && *x <= '9');
    }
    if (ok && x < t && (*x == 'e' || *x == 'E')) {
      ++x;
      int ev = 0;
      const char* es = x + (x < t && (*x == '+' || *x == '-'));
      auto er = std::from_chars(es, t, ev);
      ok = er.ec == std::errc() && er.ptr == t && es < t;
      if (ok) scale += (*x == '-') ? -ev : ev;
      x = t;
    }
    if (ok && x == t && m <= (uint64_t(1) << 53) && scale >= -22 && scale <= 22) {
      double d = static_cast<double>(m);
      d = scale < 0 ? d / kPow10[-scale] : d * kPow10[scale];
      v = neg ? -d : d;
      return true;
    }
  }
  // from_chars takes no leading '+' and is locale-independent and correctly rounded
  auto r = std::from_chars(s, t, v);
  if (r.ec == std::errc::result_out_of_range) {  // beyond double: Python's float() gives +-inf / 0
    v = strtod(std::string(s, t).c_str(), nullptr);
    return true;
  }
  return r.ec == std::errc() && r.ptr == t;
}

inline bool parse_int(const char* s, const char* t, int64_t& v) {
  auto r = std::from_chars(s, t, v);
  return r.ec == std::errc() && r.ptr == t;
}

// ---- structure pass -------------------------------------------------------------------------

struct ShapeWalk {
  int ndim = -1;  // fixed by the first leaf's depth
  int64_t shape[PRL_JSON_MAX_DIMS] = {0};
  bool seen[PRL_JSON_MAX_DIMS] = {false};
  bool has_float = false;
  int err = PRL_DATA_OK;
};

// Byte classes of the leaf-list fast scan.
enum : uint8_t { C_OTHER = 0, C_NUM, C_FLT, C_COMMA, C_CLOSE, C_WS };
struct ByteClass {
  uint8_t k[256];
  ByteClass() {
    memset(k, C_OTHER, sizeof(k));
    for (int ch = '0'; ch <= '9'; ++ch) k[ch] = C_NUM;
    k['-'] = k['+'] = C_NUM;
    k['.'] = k['e'] = k['E'] = C_FLT;
    k[','] = C_COMMA;
    k[']'] = C_CLOSE;
    k[' '] = k['\n'] = k['\r'] = k['\t'] = C_WS;
  }
};
const ByteClass kClass;

// A list of plain numeric literals (c.p just after '['): count = commas + 1, float-ness from the
// characters, one table lookup per byte.  False (cursor restored) for anything else (nested
// lists, NaN / Infinity, strings, literals): the token-by-token walk takes it.  Malformed tokens
// ("1-2", ",,") pass here and fail the value pass.
bool leaf_scan(Cursor& c, int64_t& count, ShapeWalk& w, int d) {
  const char* p = c.p;
  int64_t commas = 0;
  bool flt = false;
  for (; p < c.e; ++p) {
    const uint8_t k = kClass.k[static_cast<uint8_t>(*p)];
    if (k == C_NUM || k == C_WS) continue;
    if (k == C_COMMA) {
      ++commas;
      continue;
    }
    if (k == C_FLT) {
      flt = true;
      continue;
    }
    if (k == C_CLOSE) break;
    return false;
  }
  if (p >= c.e) return false;
  if (w.ndim < 0) w.ndim = d + 1;
  else if (w.ndim != d + 1) return false;
  c.p = p + 1;
  count = commas + 1;
  w.has_float |= flt;
  return true;
}

// Walk the array at c.p (a '[') at nesting depth d, recording / checking the length of every
// list at each depth and classifying the leaves.
bool walk(Cursor& c, int d, ShapeWalk& w) {
  if (d >= PRL_JSON_MAX_DIMS) {
    w.err = PRL_DATA_ESHAPE;
    return false;
  }
  ++c.p;  // '['
  int64_t count = 0;
  c.ws();
  if (c.p < c.e && *c.p == ']') {
    ++c.p;
    // an empty list is a leaf list at this depth: numpy gives shape (..., 0)
    if (w.ndim < 0) w.ndim = d + 1;
    else if (w.ndim != d + 1) return (w.err = PRL_DATA_ESHAPE), false;
  } else {
    if (*c.p != '[' && leaf_scan(c, count, w, d)) goto counted;
    while (true) {
      c.ws();
      if (c.p >= c.e) return (w.err = PRL_DATA_ESYNTAX), false;
      if (*c.p == '[') {
        if (w.ndim >= 0 && w.ndim <= d + 1) return (w.err = PRL_DATA_ESHAPE), false;
        if (!walk(c, d + 1, w)) return false;
      } else {
        if (w.ndim < 0) w.ndim = d + 1;
        else if (w.ndim != d + 1) return (w.err = PRL_DATA_ESHAPE), false;
        const char* s = c.p;
        while (c.p < c.e && *c.p != ',' && *c.p != ']' && !is_ws(*c.p)) ++c.p;
        const TokKind k = classify(s, c.p);
        if (k == TOK_BAD) return (w.err = (*s == '"' || *s == '{' || *s == 't' || *s == 'f' || *s == 'n')
                                              ? PRL_DATA_ETYPE : PRL_DATA_ESYNTAX), false;
        if (k == TOK_FLOAT) w.has_float = true;
      }
      ++count;
      c.ws();
      if (c.p >= c.e) return (w.err = PRL_DATA_ESYNTAX), false;
      if (*c.p == ',') {
        ++c.p;
        continue;
      }
      if (*c.p == ']') {
        ++c.p;
        break;
      }
      return (w.err = PRL_DATA_ESYNTAX), false;
    }
  }
counted:
  if (!w.seen[d]) {
    w.seen[d] = true;
    w.shape[d] = count;
  } else if (w.shape[d] != count) {
    return (w.err = PRL_DATA_ESHAPE), false;
  }
  return true;
}

// ---- value pass -------------------------------------------------------------------------------

template <typename T>
int fill_typed(const PrlJsonArray& a, T* out, int64_t n) {
  const char* p = a.text;
  const char* e = a.text + a.len;
  int64_t i = 0;
  while (p < e) {
    const char ch = *p;
    if (ch == '[' || ch == ']' || ch == ',' || is_ws(ch)) {
      ++p;
      continue;
    }
    const char* s = p;
    while (p < e && *p != ',' && *p != ']' && !is_ws(*p)) ++p;
    if (i >= n) return PRL_DATA_ECAP;
    if constexpr (std::is_floating_point_v<T>) {
      if (!a.has_float) {  // all integers: numpy holds int64, torch converts int64 -> float directly
        int64_t v;
        if (!parse_int(s, p, v)) return PRL_DATA_ERANGE;
        out[i++] = static_cast<T>(v);
        continue;
      }
      double v;
      if (!parse_double(s, p, v)) return PRL_DATA_ESYNTAX;
      out[i++] = static_cast<T>(v);  // float64 -> float32: round to nearest even (numpy / torch)
    } else {
      if (a.has_float) {  // numpy holds float64: torch's float -> int conversion truncates
        double v;
        if (!parse_double(s, p, v)) return PRL_DATA_ESYNTAX;
        if (!std::isfinite(v) || v >= 9.2233720368547758e18 || v < -9.2233720368547758e18) return PRL_DATA_ERANGE;
        out[i++] = static_cast<T>(static_cast<int64_t>(v));
      } else {
        int64_t v;
        if (!parse_int(s, p, v)) return PRL_DATA_ERANGE;  // beyond int64: numpy would make an object array
        out[i++] = static_cast<T>(v);                     // int64 -> int32 wraps, as torch's .to(int)
      }
    }
  }
  return i == n ? PRL_DATA_OK : PRL_DATA_ESHAPE;
}

int fill_one(PrlJsonArray& a) {
  if (!a.text || a.len < 0 || a.ndim < 1 || a.ndim > PRL_JSON_MAX_DIMS) return PRL_DATA_EINVAL;
  int64_t n = 1;
  for (int d = 0; d < a.ndim; ++d) n *= a.shape[d];
  if (n > 0 && !a.out) return PRL_DATA_EINVAL;
  switch (a.dtype) {
    case PRL_DT_I64: return fill_typed(a, static_cast<int64_t*>(a.out), n);
    case PRL_DT_I32: return fill_typed(a, static_cast<int32_t*>(a.out), n);
    case PRL_DT_F32: return fill_typed(a, static_cast<float*>(a.out), n);
    case PRL_DT_F64: return fill_typed(a, static_cast<double*>(a.out), n);
    default: return PRL_DATA_EINVAL;
  }
}

// ---- formatting -------------------------------------------------------------------------------

// Python's float repr (json.dumps writes floats with it): the shortest round-trip digits, fixed
// notation when the decimal point position is in (-4, 16], else d.ddde+XX; NaN / Infinity.
inline char* fmt_double(char* o, char* end, double v) {
  if (std::isnan(v)) {
    memcpy(o, "NaN", 3);
    return o + 3;
  }
  if (std::isinf(v)) {
    if (v < 0) *o++ = '-';
    memcpy(o, "Infinity", 8);
    return o + 8;
  }
  char sci[40];
  auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
  const char* p = sci;
  if (*p == '-') {
    *o++ = '-';
    ++p;
  }
  char digits[24];
  int nd = 0;
  for (; p < r.ptr && *p != 'e'; ++p)
    if (*p != '.') digits[nd++] = *p;
  int exp10 = 0;
  std::from_chars(p + (p[1] == '+' ? 2 : 1), r.ptr, exp10);
  const int decpt = exp10 + 1;
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *o++ = '0';
      *o++ = '.';
      for (int k = 0; k < -decpt; ++k) *o++ = '0';
      memcpy(o, digits, nd);
      o += nd;
    } else if (decpt >= nd) {
      memcpy(o, digits, nd);
      o += nd;
      for (int k = nd; k < decpt; ++k) *o++ = '0';
      *o++ = '.';
      *o++ = '0';
    } else {
      memcpy(o, digits, decpt);
      o += decpt;
      *o++ = '.';
      memcpy(o, digits + decpt, nd - decpt);
      o += nd - decpt;
    }
  } else {
    *o++ = digits[0];
    if (nd > 1) {
      *o++ = '.';
      memcpy(o, digits + 1, nd - 1);
      o += nd - 1;
    }
    *o++ = 'e';
    *o++ = exp10 < 0 ? '-' : '+';
    const int a = exp10 < 0 ? -exp10 : exp10;
    if (a < 10) *o++ = '0';
    o = std::to_chars(o, end, a).ptr;
  }
  return o;
}

template <typename T>
char* fmt_elem(char* o, char* end, T v) {
  if constexpr (std::is_floating_point_v<T>) return fmt_double(o, end, static_cast<double>(v));
  else return std::to_chars(o, end, static_cast<int64_t>(v)).ptr;
}

template <typename T>
int format_typed(const T* data, int ndim, const int64_t* shape, char* out, int64_t cap, int64_t* written) {
  char* o = out;
  char* end = out + cap;
  int64_t idx[PRL_JSON_MAX_DIMS] = {0};
  int64_t total = 1;
  for (int d = 0; d < ndim; ++d) total *= shape[d];
  if (total == 0) {
    // tolist() of an empty array: lists nested down to the first zero-length dim
    int d0 = 0;
    while (d0 < ndim && shape[d0] != 0) ++d0;
    // dims before d0 are non-empty: write them as lists of empty lists
    std::vector<char> buf;
    std::function<void(int)> rec = [&](int d) {
      buf.push_back('[');
      if (d < d0) {
        for (int64_t i = 0; i < shape[d]; ++i) {
          if (i) buf.push_back(',');
          rec(d + 1);
        }
      }
      buf.push_back(']');
    };
    rec(0);
    if ((int64_t)buf.size() > cap) return PRL_DATA_ECAP;
    memcpy(out, buf.data(), buf.size());
    *written = (int64_t)buf.size();
    return PRL_DATA_OK;
  }
  for (int d = 0; d < ndim; ++d) *o++ = '[';
  for (int64_t i = 0; i < total; ++i) {
    if (end - o < 64 + ndim * 2) return PRL_DATA_ECAP;
    o = fmt_elem(o, end, data[i]);
    // advance the multi-index, closing / opening lists
    int d = ndim - 1;
    while (d >= 0 && ++idx[d] == shape[d]) {
      idx[d] = 0;
      *o++ = ']';
      --d;
    }
    if (d >= 0) {
      *o++ = ',';
      for (int k = d + 1; k < ndim; ++k) *o++ = '[';
    }
  }
  *written = o - out;
  return PRL_DATA_OK;
}

}  // namespace

extern "C" {

int prl_data_abi_version(void) { return PRL_DATA_ABI; }

const char* prl_data_error_string(int code) {
  switch (code) {
    case PRL_DATA_OK: return "ok";
    case PRL_DATA_EINVAL: return "invalid argument";
    case PRL_DATA_ESYNTAX: return "JSON syntax error";
    case PRL_DATA_ESHAPE: return "ragged or too deeply nested array";
    case PRL_DATA_ETYPE: return "array element is not a number";
    case PRL_DATA_ECAP: return "output capacity too small";
    case PRL_DATA_ERANGE: return "value not representable in the requested type";
    default: return "unknown prl_data error";
  }
}

int prl_json_members(const char* doc, int64_t len, PrlJsonMember* out, int32_t cap, int32_t* n) {
  if (!doc || len < 0 || !n || (cap > 0 && !out)) return PRL_DATA_EINVAL;
  Cursor c{doc, doc + len};
  c.ws();
  if (c.p >= c.e || *c.p != '{') return PRL_DATA_ESYNTAX;
  ++c.p;
  int32_t k = 0;
  c.ws();
  if (c.p < c.e && *c.p == '}') {
    *n = 0;
    return PRL_DATA_OK;
  }
  while (true) {
    c.ws();
    const char* ks = c.p;
    if (!skip_string(c)) return PRL_DATA_ESYNTAX;
    const char* ke = c.p;
    c.ws();
    if (c.p >= c.e || *c.p != ':') return PRL_DATA_ESYNTAX;
    ++c.p;
    c.ws();
    const char* vs = c.p;
    if (!skip_value(c)) return PRL_DATA_ESYNTAX;
    if (k < cap) out[k] = PrlJsonMember{(ks + 1) - doc, (ke - 1) - (ks + 1), vs - doc, c.p - vs};
    ++k;
    c.ws();
    if (c.p >= c.e) return PRL_DATA_ESYNTAX;
    if (*c.p == ',') {
      ++c.p;
      continue;
    }
    if (*c.p == '}') break;
    return PRL_DATA_ESYNTAX;
  }
  *n = k;
  return k > cap ? PRL_DATA_ECAP : PRL_DATA_OK;
}

int prl_json_array_shape(PrlJsonArray* a) {
  if (!a || !a->text || a->len < 0) return PRL_DATA_EINVAL;
  Cursor c{a->text, a->text + a->len};
  c.ws();
  if (c.p >= c.e || *c.p != '[') return a->status = PRL_DATA_ETYPE;
  ShapeWalk w;
  if (!walk(c, 0, w)) return a->status = w.err;
  c.ws();
  if (c.p != c.e) return a->status = PRL_DATA_ESYNTAX;
  a->ndim = w.ndim;
  for (int d = 0; d < PRL_JSON_MAX_DIMS; ++d) a->shape[d] = d < w.ndim ? w.shape[d] : 0;
  a->has_float = w.has_float;
  return a->status = PRL_DATA_OK;
}

int prl_json_array_fill(PrlJsonArray* arrays, int32_t n, int32_t threads) {
  if (n < 0 || (n > 0 && !arrays)) return PRL_DATA_EINVAL;
  if (threads < 1) threads = 1;
  if (threads > n) threads = n;
  if (threads <= 1) {
    for (int32_t i = 0; i < n; ++i) arrays[i].status = fill_one(arrays[i]);
  } else {
    // static interleaved assignment: arrays are of similar size (token fields of one batch)
    std::vector<std::thread> pool;
    pool.reserve(threads - 1);
    auto work = [arrays, n, threads](int t) {
      for (int32_t i = t; i < n; i += threads) arrays[i].status = fill_one(arrays[i]);
    };
    for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
  }
  for (int32_t i = 0; i < n; ++i)
    if (arrays[i].status) return arrays[i].status;
  return PRL_DATA_OK;
}

int64_t prl_json_format_bound(int64_t count, int32_t ndim, const int64_t* shape) {
  if (count < 0 || ndim < 1 || ndim > PRL_JSON_MAX_DIMS || !shape) return -1;
  // 26 chars for the longest double ("-2.2250738585072014e-308") + ".0" slack + separator,
  // and two brackets per list
  int64_t lists = 1, prod = 1;
  for (int d = 0; d < ndim - 1; ++d) {
    prod *= shape[d] > 0 ? shape[d] : 1;
    lists += prod;
  }
  return count * 30 + lists * 3 + 64;
}

int prl_json_array_format(const void* data, int32_t dtype, int32_t ndim, const int64_t* shape, char* out,
                          int64_t cap, int64_t* written) {
  if (ndim < 1 || ndim > PRL_JSON_MAX_DIMS || !shape || !out || !written) return PRL_DATA_EINVAL;
  int64_t total = 1;
  for (int d = 0; d < ndim; ++d) {
    if (shape[d] < 0) return PRL_DATA_EINVAL;
    total *= shape[d];
  }
  if (total > 0 && !data) return PRL_DATA_EINVAL;
  if (cap < prl_json_format_bound(total, ndim, shape)) return PRL_DATA_ECAP;
  switch (dtype) {
    case PRL_DT_I64: return format_typed(static_cast<const int64_t*>(data), ndim, shape, out, cap, written);
    case PRL_DT_I32: return format_typed(static_cast<const int32_t*>(data), ndim, shape, out, cap, written);
    case PRL_DT_F32: return format_typed(static_cast<const float*>(data), ndim, shape, out, cap, written);
    case PRL_DT_F64: return format_typed(static_cast<const double*>(data), ndim, shape, out, cap, written);
    default: return PRL_DATA_EINVAL;
  }
}

// pandas' groupby mean (Kahan-compensated sum / count) and std (Welford, ddof = 1), the
// aggregations rl/__init__.py:408-416 asks for, in the rollouts' order.
int prl_rl_group_stats(int64_t n_rollouts, const int64_t* group_of, int64_t n_groups, const double* reward0,
                       const int64_t* length, double* mean, double* std, double* tokens_mean) {
  if (n_rollouts < 0 || n_groups < 0 || (n_rollouts > 0 && (!group_of || !reward0 || !length)) ||
      (n_groups > 0 && (!mean || !std || !tokens_mean)))
    return PRL_DATA_EINVAL;
  std::vector<double> rsum(n_groups, 0.0), rcomp(n_groups, 0.0), lsum(n_groups, 0.0), lcomp(n_groups, 0.0);
  std::vector<double> wmean(n_groups, 0.0), m2(n_groups, 0.0);
  std::vector<int64_t> cnt(n_groups, 0);
  auto kahan = [](double& sum, double& comp, double x) {
    const double y = x - comp;
    const double t = sum + y;
    comp = t - sum - y;
    sum = t;
  };
  for (int64_t i = 0; i < n_rollouts; ++i) {
    const int64_t g = group_of[i];
    if (g < 0 || g >= n_groups) return PRL_DATA_EINVAL;
    const double r = reward0[i];
    ++cnt[g];
    kahan(rsum[g], rcomp[g], r);
    kahan(lsum[g], lcomp[g], static_cast<double>(length[i]));
    const double old = wmean[g];
    wmean[g] += (r - old) / static_cast<double>(cnt[g]);
    m2[g] += (r - wmean[g]) * (r - old);
  }
  for (int64_t g = 0; g < n_groups; ++g) {
    if (cnt[g] == 0) return PRL_DATA_EINVAL;
    mean[g] = rsum[g] / static_cast<double>(cnt[g]);
    tokens_mean[g] = lsum[g] / static_cast<double>(cnt[g]);
    std[g] = cnt[g] > 1 ? std::sqrt(m2[g] / static_cast<double>(cnt[g] - 1)) : std::numeric_limits<double>::quiet_NaN();
  }
  return PRL_DATA_OK;
}

int prl_collate_packed(int64_t n, const int64_t* lengths, const int64_t* ids, const int64_t* labels, int64_t label_pad,
                       int64_t* out_ids, int64_t* out_labels, int64_t* out_pos, int32_t* boundaries) {
  if (n < 0 || !boundaries || (n > 0 && !lengths)) return PRL_DATA_EINVAL;
  int64_t total = 0;
  boundaries[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (lengths[i] < 0) return PRL_DATA_EINVAL;
    total += lengths[i];
    if (total > std::numeric_limits<int32_t>::max()) return PRL_DATA_ERANGE;
    boundaries[i + 1] = static_cast<int32_t>(total);
  }
  if (total > 0 && (!ids || !labels || !out_ids || !out_labels || !out_pos)) return PRL_DATA_EINVAL;
  memcpy(out_ids, ids, total * sizeof(int64_t));
  memcpy(out_labels, labels, total * sizeof(int64_t));
  int64_t a = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t L = lengths[i];
    for (int64_t t = 0; t < L; ++t) out_pos[a + t] = t;
    if (i > 0 && L > 0) out_labels[a] = label_pad;  // no prediction across a sequence boundary
    a += L;
  }
  return PRL_DATA_OK;
}

}  // extern "C"
