// codec.cpp -- the reference's wire codec (pubsub.go:122-153), host side.
//
// writeMessage is json.NewEncoder(s).Encode(m): one JSON object per line,
// fields in struct order, `omitempty` on everything but Type, []byte as
// standard base64 with padding, strings with Go's default (HTML-safe)
// escaping, then '\n'.  readMessage is json.NewDecoder(r).Decode(m): field
// names match case-insensitively, unknown fields are skipped, null leaves a
// field unset.  This is the interop edge of the engine: the
// GPU moves message ids; a Go peer on the other side of a stream still sees
// byte-identical lines.
#include <cctype>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "psengine.h"

namespace {

const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

void b64_encode(const uint8_t* p, size_t n, std::string& out) {
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += kB64[v & 63];
  }
  if (n - i == 1) {
    const uint32_t v = p[i] << 16;
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += "==";
  } else if (n - i == 2) {
    const uint32_t v = (p[i] << 16) | (p[i + 1] << 8);
    out += kB64[v >> 18];
    out += kB64[(v >> 12) & 63];
    out += kB64[(v >> 6) & 63];
    out += '=';
  }
}

int b64_val(char c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// encoding/base64 StdEncoding.DecodeString as encoding/json uses it
// (padding required; \r and \n are ignored)
bool b64_decode(const std::string& s, std::vector<uint8_t>& out) {
  std::string t;
  for (char c : s)
    if (c != '\r' && c != '\n') t += c;
  if (t.size() % 4) return false;
  for (size_t i = 0; i < t.size(); i += 4) {
    int v[4];
    int pad = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = t[i + k];
      if (c == '=') {
        if (i + 4 != t.size() || k < 2) return false;
        v[k] = 0;
        ++pad;
      } else {
        if (pad) return false;
        v[k] = b64_val(c);
        if (v[k] < 0) return false;
      }
    }
    const uint32_t x = (v[0] << 18) | (v[1] << 12) | (v[2] << 6) | v[3];
    out.push_back(static_cast<uint8_t>(x >> 16));
    if (pad < 2) out.push_back(static_cast<uint8_t>((x >> 8) & 0xFF));
    if (pad < 1) out.push_back(static_cast<uint8_t>(x & 0xFF));
  }
  return true;
}

// Length of the valid UTF-8 sequence at p (0: invalid), as utf8.DecodeRune.
size_t utf8_len(const unsigned char* p, size_t n, uint32_t* cp) {
  const unsigned c = p[0];
  if (c < 0x80) {
    *cp = c;
    return 1;
  }
  size_t len;
  uint32_t v, min;
  if ((c & 0xE0) == 0xC0) {
    len = 2, v = c & 0x1F, min = 0x80;
  } else if ((c & 0xF0) == 0xE0) {
    len = 3, v = c & 0x0F, min = 0x800;
  } else if ((c & 0xF8) == 0xF0) {
    len = 4, v = c & 0x07, min = 0x10000;
  } else {
    return 0;
  }
  if (len > n) return 0;
  for (size_t k = 1; k < len; ++k) {
    if ((p[k] & 0xC0) != 0x80) return 0;
    v = (v << 6) | (p[k] & 0x3F);
  }
  if (v < min || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
  *cp = v;
  return len;
}

// encoding/json string encoding with HTML escaping (the Encoder default)
void json_string(const char* s, size_t n, std::string& out) {
  static const char hex[] = "0123456789abcdef";
  out += '"';
  const auto* p = reinterpret_cast<const unsigned char*>(s);
  for (size_t i = 0; i < n;) {
    const unsigned char c = p[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') {
        out += '\\';
        out += static_cast<char>(c);
      } else if (c == '\n') {
        out += "\\n";
      } else if (c == '\r') {
        out += "\\r";
      } else if (c == '\t') {
        out += "\\t";
      } else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
        out += "\\u00";
        out += hex[c >> 4];
        out += hex[c & 15];
      } else {
        out += static_cast<char>(c);
      }
      ++i;
      continue;
    }
    uint32_t cp = 0;
    const size_t len = utf8_len(p + i, n - i, &cp);
    if (len == 0) {  // invalid UTF-8 becomes U+FFFD
      out += "\\ufffd";
      ++i;
      continue;
    }
    if (cp == 0x2028 || cp == 0x2029) {
      out += cp == 0x2028 ? "\\u2028" : "\\u2029";
    } else {
      out.append(s + i, len);
    }
    i += len;
  }
  out += '"';
}

// ------------------------------------------------------------- decoding ---
struct Parser {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* w) {
    const size_t n = std::strlen(w);
    if (static_cast<size_t>(e - p) < n || std::strncmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  static void put_utf8(uint32_t cp, std::string& out) {
    if (cp < 0x80) {
      out += static_cast<char>(cp);
    } else if (cp < 0x800) {
      out += static_cast<char>(0xC0 | (cp >> 6));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += static_cast<char>(0xE0 | (cp >> 12));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      out += static_cast<char>(0xF0 | (cp >> 18));
      out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    *v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = *p++;
      *v <<= 4;
      if (c >= '0' && c <= '9')
        *v |= c - '0';
      else if (c >= 'a' && c <= 'f')
        *v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F')
        *v |= c - 'A' + 10;
      else
        return false;
    }
    return true;
  }
  bool str(std::string& out) {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      if (static_cast<unsigned char>(*p) < 0x20) return false;
      if (*p != '\\') {
        out += *p++;
        continue;
      }
      ++p;
      if (p >= e) return false;
      const char c = *p++;
      switch (c) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t v;
          if (!hex4(&v)) return false;
          if (v >= 0xD800 && v < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) {
              v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              p = save;
              v = 0xFFFD;
            }
          } else if (v >= 0xD800 && v < 0xE000) {
            v = 0xFFFD;
          }
          put_utf8(v, out);
          break;
        }
        default: return false;
      }
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  bool integer(int64_t* v) {  // Go decodes a JSON number into an int field
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p >= e || !std::isdigit(static_cast<unsigned char>(*p))) return false;
    while (p < e && std::isdigit(static_cast<unsigned char>(*p))) ++p;
    if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;  // not an int
    *v = std::strtoll(std::string(s, p).c_str(), nullptr, 10);
    return true;
  }
  bool skip() {  // any JSON value
    ws();
    if (p >= e) return false;
    if (*p == '"') {
      std::string t;
      return str(t);
    }
    if (*p == '{' || *p == '[') {
      const char close = *p == '{' ? '}' : ']';
      const bool obj = *p == '{';
      ++p;
      ws();
      if (p < e && *p == close) {
        ++p;
        return true;
      }
      while (true) {
        if (obj) {
          std::string k;
          ws();
          if (!str(k)) return false;
          ws();
          if (p >= e || *p++ != ':') return false;
        }
        if (!skip()) return false;
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == close) {
          ++p;
          return true;
        }
        return false;
      }
    }
    if (lit("true") || lit("false") || lit("null")) return true;
    if (*p == '-' || std::isdigit(static_cast<unsigned char>(*p))) {
      ++p;
      while (p < e && (std::isdigit(static_cast<unsigned char>(*p)) || *p == '.' || *p == 'e' ||
                       *p == 'E' || *p == '+' || *p == '-'))
        ++p;
      return true;
    }
    return false;
  }
};

bool ieq(const std::string& a, const char* b) {
  if (a.size() != std::strlen(b)) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
      return false;
  return true;
}

}  // namespace

extern "C" {

int ps_msg_encode(const ps_message* m, char* out, size_t cap, size_t* len_out) {
  if (!m || !len_out || (m->data_len && !m->data) || (m->n_peers && !m->peers)) return PS_E_INVAL;
  std::string s = "{\"Type\":" + std::to_string(m->type);
  if (m->data_len) {
    s += ",\"data\":\"";
    b64_encode(m->data, m->data_len, s);
    s += '"';
  }
  if (m->n_peers) {
    s += ",\"parents\":[";
    for (size_t i = 0; i < m->n_peers; ++i) {
      if (i) s += ',';
      const char* pid = m->peers[i] ? m->peers[i] : "";
      json_string(pid, std::strlen(pid), s);
    }
    s += ']';
  }
  if (m->tree_width) s += ",\"treewidth\":" + std::to_string(m->tree_width);
  if (m->tree_max_width) s += ",\"treemaxwidth\":" + std::to_string(m->tree_max_width);
  if (m->num_peers) s += ",\"numpeers\":" + std::to_string(m->num_peers);
  s += "}\n";  // json.Encoder.Encode terminates each value with a newline
  *len_out = s.size();
  if (!out || cap < s.size()) return PS_E_RANGE;
  std::memcpy(out, s.data(), s.size());
  return PS_OK;
}

int ps_msg_decode(const char* in, size_t len, ps_message_buf* out, size_t* consumed) {
  if (!in || !out) return PS_E_INVAL;
  Parser P{in, in + len};
  int64_t type = 0, tw = 0, tmw = 0, np = 0;
  std::vector<uint8_t> data;
  std::vector<std::string> peers;
  P.ws();
  if (P.p >= P.e || *P.p != '{') return PS_E_INVAL;
  ++P.p;
  P.ws();
  if (P.p < P.e && *P.p == '}') {
    ++P.p;
  } else {
    while (true) {
      std::string key;
      P.ws();
      if (!P.str(key)) return PS_E_INVAL;
      P.ws();
      if (P.p >= P.e || *P.p++ != ':') return PS_E_INVAL;
      P.ws();
      if (P.lit("null")) {  // leaves the field as it is
      } else if (ieq(key, "Type")) {
        if (!P.integer(&type)) return PS_E_INVAL;
      } else if (ieq(key, "data")) {
        std::string b;
        data.clear();  // a repeated key replaces the value, as in encoding/json
        if (!P.str(b) || !b64_decode(b, data)) return PS_E_INVAL;
      } else if (ieq(key, "parents")) {
        if (P.p >= P.e || *P.p != '[') return PS_E_INVAL;
        ++P.p;
        peers.clear();
        P.ws();
        if (P.p < P.e && *P.p == ']') {
          ++P.p;
        } else {
          while (true) {
            std::string v;
            P.ws();
            if (!P.str(v)) return PS_E_INVAL;
            peers.push_back(v);
            P.ws();
            if (P.p < P.e && *P.p == ',') {
              ++P.p;
              continue;
            }
            if (P.p < P.e && *P.p == ']') {
              ++P.p;
              break;
            }
            return PS_E_INVAL;
          }
        }
      } else if (ieq(key, "treewidth")) {
        if (!P.integer(&tw)) return PS_E_INVAL;
      } else if (ieq(key, "treemaxwidth")) {
        if (!P.integer(&tmw)) return PS_E_INVAL;
      } else if (ieq(key, "numpeers")) {
        if (!P.integer(&np)) return PS_E_INVAL;
      } else if (!P.skip()) {  // unknown field: ignored
        return PS_E_INVAL;
      }
      P.ws();
      if (P.p < P.e && *P.p == ',') {
        ++P.p;
        continue;
      }
      if (P.p < P.e && *P.p == '}') {
        ++P.p;
        break;
      }
      return PS_E_INVAL;
    }
  }
  // the decoder consumes the value; the encoder's trailing newline is
  // whitespace the next Decode skips
  P.ws();
  out->type = static_cast<int32_t>(type);
  out->tree_width = tw;
  out->tree_max_width = tmw;
  out->num_peers = np;
  out->data_len = data.size();
  size_t need = 0;
  for (const auto& v : peers) need += v.size() + 1;
  out->n_peers = peers.size();
  out->peers_len = need;
  if (consumed) *consumed = static_cast<size_t>(P.p - in);
  if (data.size() > out->data_cap || need > out->peers_cap) return PS_E_RANGE;
  if (!data.empty()) std::memcpy(out->data, data.data(), data.size());
  size_t o = 0;
  for (const auto& v : peers) {  // NUL-separated
    std::memcpy(out->peers + o, v.data(), v.size());
    out->peers[o + v.size()] = '\0';
    o += v.size() + 1;
  }
  return PS_OK;
}

}  // extern "C"
