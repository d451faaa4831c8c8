// Wire-format ingest: Binance kline websocket events ->
// structure-of-arrays, on the host, in one native pass over a batch of raw
// frames.
//
// The reference decodes every frame with json.loads
// (producers/klines_connector.py:77-90), keeps closed candles of "kline"
// events and copies the fields as strings into a KlineProduceModel
// (:148-164: s, t, T, o, h, l, c, v); the store later coerces them with
// pd.to_numeric (market_regime/market_state_store.py:82-83). Here the decimal
// strings are converted with strtod — correctly rounded, so each value is
// the same double Python's float() / pandas produce — straight into the
// arrays the device store ingests (bq_store_update), with no per-frame
// Python objects.
//
// Frames are separated by '\n' (one JSON object per line). A frame that is
// not a "kline" event is skipped; a kline frame missing a field or holding
// a malformed value is counted in n_bad and skipped.
#include "binquant_amd.h"

#include <cerrno>
#include <cstdlib>
#include <cstring>

namespace {

struct Cursor {
  const char* p;
  const char* end;
  bool ok = true;
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < end && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
};

// JSON string starting at '"': returns [b, e) of the raw contents (escapes
// left in place; kline fields never carry them except possibly the symbol).
bool read_string(Cursor& c, const char*& b, const char*& e) {
  c.ws();
  if (c.p >= c.end || *c.p != '"') return false;
  b = ++c.p;
  while (c.p < c.end && *c.p != '"') {
    if (*c.p == '\\') ++c.p;
    ++c.p;
  }
  if (c.p >= c.end) return false;
  e = c.p++;
  return true;
}

bool skip_value(Cursor& c, int depth = 0);

bool skip_container(Cursor& c, char open, char close, int depth) {
  if (depth > 64) return false;
  ++c.p;   // open
  c.ws();
  if (c.p < c.end && *c.p == close) {
    ++c.p;
    return true;
  }
  for (;;) {
    if (open == '{') {
      const char *b, *e;
      if (!read_string(c, b, e) || !c.eat(':')) return false;
    }
    if (!skip_value(c, depth + 1)) return false;
    c.ws();
    if (c.p < c.end && *c.p == ',') {
      ++c.p;
      continue;
    }
    if (c.p < c.end && *c.p == close) {
      ++c.p;
      return true;
    }
    return false;
  }
}

bool skip_value(Cursor& c, int depth) {
  c.ws();
  if (c.p >= c.end) return false;
  const char ch = *c.p;
  if (ch == '"') {
    const char *b, *e;
    return read_string(c, b, e);
  }
  if (ch == '{') return skip_container(c, '{', '}', depth);
  if (ch == '[') return skip_container(c, '[', ']', depth);
  // number / true / false / null: up to the next delimiter
  const char* s = c.p;
  while (c.p < c.end && *c.p != ',' && *c.p != '}' && *c.p != ']' && *c.p != ' ' && *c.p != '\t' && *c.p != '\r')
    ++c.p;
  return c.p > s;
}

// raw value token (string contents or bare token) -> [b, e)
bool value_token(Cursor& c, const char*& b, const char*& e, bool& quoted) {
  c.ws();
  if (c.p >= c.end) return false;
  if (*c.p == '"') {
    quoted = true;
    return read_string(c, b, e);
  }
  quoted = false;
  b = c.p;
  if (*c.p == '{' || *c.p == '[') return false;
  if (!skip_value(c)) return false;
  e = c.p;
  return true;
}

bool to_double(const char* b, const char* e, double& out) {
  char tmp[64];
  const size_t n = (size_t)(e - b);
  if (n == 0 || n >= sizeof(tmp)) return false;
  memcpy(tmp, b, n);
  tmp[n] = 0;
  char* endp = nullptr;
  errno = 0;
  out = strtod(tmp, &endp);
  return endp == tmp + n && errno != ERANGE;
}

bool to_int64(const char* b, const char* e, int64_t& out) {
  char tmp[32];
  const size_t n = (size_t)(e - b);
  if (n == 0 || n >= sizeof(tmp)) return false;
  memcpy(tmp, b, n);
  tmp[n] = 0;
  char* endp = nullptr;
  errno = 0;
  const long long v = strtoll(tmp, &endp, 10);
  if (endp != tmp + n || errno == ERANGE) return false;
  out = (int64_t)v;
  return true;
}

enum Field { F_T = 0, F_TT, F_S, F_O, F_H, F_L, F_C, F_V, F_X, F_N };

int field_of(const char* b, const char* e) {
  if (e - b != 1) return -1;
  switch (*b) {
    case 't': return F_T;
    case 'T': return F_TT;
    case 's': return F_S;
    case 'o': return F_O;
    case 'h': return F_H;
    case 'l': return F_L;
    case 'c': return F_C;
    case 'v': return F_V;
    case 'x': return F_X;
    default: return -1;
  }
}

struct Row {
  int64_t t, tt;
  double v[5];
  const char *sb, *se;
  bool x;
};

// parse the "k" object; returns false on a malformed / incomplete kline
bool parse_k(Cursor& c, Row& r) {
  if (!c.eat('{')) return false;
  unsigned seen = 0;
  c.ws();
  if (c.p < c.end && *c.p == '}') return false;
  for (;;) {
    const char *kb, *ke;
    if (!read_string(c, kb, ke) || !c.eat(':')) return false;
    const int f = field_of(kb, ke);
    if (f < 0) {
      if (!skip_value(c)) return false;
    } else {
      const char *b, *e;
      bool quoted;
      if (!value_token(c, b, e, quoted)) return false;
      switch (f) {
        case F_T:
          if (!to_int64(b, e, r.t)) return false;
          break;
        case F_TT:
          if (!to_int64(b, e, r.tt)) return false;
          break;
        case F_S:
          if (!quoted) return false;
          r.sb = b;
          r.se = e;
          break;
        case F_X:
          if (quoted) return false;
          if (e - b == 4 && !memcmp(b, "true", 4)) r.x = true;
          else if (e - b == 5 && !memcmp(b, "false", 5)) r.x = false;
          else return false;
          break;
        default:
          if (!to_double(b, e, r.v[f - F_O])) return false;
      }
      seen |= 1u << f;
    }
    c.ws();
    if (c.p < c.end && *c.p == ',') {
      ++c.p;
      continue;
    }
    if (c.p < c.end && *c.p == '}') {
      ++c.p;
      break;
    }
    return false;
  }
  return seen == (1u << F_N) - 1;
}

// 1 = kline row parsed, 0 = not a kline event (skipped), -1 = malformed kline
int parse_frame(const char* b, const char* e, Row& r) {
  Cursor c{b, e};
  if (!c.eat('{')) return -1;
  bool is_kline = false, have_k = false, k_ok = false;
  c.ws();
  if (c.p < c.end && *c.p == '}') return 0;
  for (;;) {
    const char *kb, *ke;
    if (!read_string(c, kb, ke) || !c.eat(':')) return is_kline ? -1 : 0;
    if (ke - kb == 1 && *kb == 'e') {
      const char *vb, *ve;
      bool quoted;
      if (!value_token(c, vb, ve, quoted)) return -1;
      is_kline = quoted && ve - vb == 5 && !memcmp(vb, "kline", 5);
    } else if (ke - kb == 1 && *kb == 'k') {
      have_k = true;
      c.ws();
      if (c.p < c.end && *c.p == '{') {
        const char* save = c.p;
        k_ok = parse_k(c, r);
        if (!k_ok) {   // resync past the object so "e" may still be read
          c.p = save;
          if (!skip_value(c)) return -1;
        }
      } else if (!skip_value(c)) {
        return -1;
      }
    } else if (!skip_value(c)) {
      return is_kline ? -1 : 0;
    }
    c.ws();
    if (c.p < c.end && *c.p == ',') {
      ++c.p;
      continue;
    }
    if (c.p < c.end && *c.p == '}') break;
    return is_kline ? -1 : 0;
  }
  if (!is_kline) return 0;
  return have_k && k_ok ? 1 : -1;
}

}  // namespace

extern "C" int bq_parse_kline_events(const char* buf, int64_t len, int64_t max_rows, char* sym, int64_t sym_stride,
                                     int64_t* open_time, int64_t* close_time, double* const* ohlcv,
                                     uint8_t* closed, int64_t* n_rows, int64_t* n_bad) {
  if (!buf || len < 0 || max_rows < 0 || !sym || sym_stride < 2 || !open_time || !close_time || !ohlcv || !closed ||
      !n_rows || !n_bad)
    return BQ_EINVAL;
  for (int i = 0; i < 5; ++i)
    if (!ohlcv[i]) return BQ_EINVAL;
  int64_t n = 0, bad = 0;
  const char* p = buf;
  const char* end = buf + len;
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    const char* fe = nl ? nl : end;
    const char* q = p;
    while (q < fe && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
    if (q < fe) {
      Row r{};
      const int st = parse_frame(q, fe, r);
      if (st < 0) {
        ++bad;
      } else if (st > 0) {
        const int64_t slen = r.se - r.sb;
        if (slen + 1 > sym_stride) {
          ++bad;
        } else {
          if (n >= max_rows) {
            *n_rows = n;
            *n_bad = bad;
            return BQ_EINVAL;   // caller's arrays are too small
          }
          memcpy(sym + n * sym_stride, r.sb, (size_t)slen);
          sym[n * sym_stride + slen] = 0;
          open_time[n] = r.t;
          close_time[n] = r.tt;
          for (int i = 0; i < 5; ++i) ohlcv[i][n] = r.v[i];
          closed[n] = r.x ? 1 : 0;
          ++n;
        }
      }
    }
    p = fe + 1;
  }
  *n_rows = n;
  *n_bad = bad;
  return BQ_OK;
}
