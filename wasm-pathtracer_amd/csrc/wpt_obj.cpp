// wpt_obj.cpp — OBJ mesh ingestion (wpt_obj.h): parseObj of
// src_ts/client/obj_parser.ts:3-51 with JavaScript's number semantics.
#include "wpt_obj.h"

#include <clocale>
#include <cmath>
#include <locale.h>
#include <cstdlib>
#include <cstring>
#include <limits>

namespace wpt {

namespace {

const double kNaN = std::numeric_limits<double>::quiet_NaN();

bool js_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
bool digit(char c) { return c >= '0' && c <= '9'; }

// parseFloat (ECMA-262 StrDecimalLiteral prefix): leading white space, sign,
// "Infinity" or digits [. digits] [e[sign]digits]; NaN when no digit. The
// prefix goes to strtod_l ("C" locale), correctly rounded to f64 as JS does.
double js_parse_float(const char* s, const char* e) {
  while (s < e && js_space(*s)) s++;
  const char* p = s;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) {
    neg = *p == '-';
    p++;
  }
  if (e - p >= 8 && std::strncmp(p, "Infinity", 8) == 0)
    return neg ? -std::numeric_limits<double>::infinity() : std::numeric_limits<double>::infinity();
  const char* q = p;
  bool any = false;
  while (q < e && digit(*q)) { q++; any = true; }
  if (q < e && *q == '.') {
    q++;
    while (q < e && digit(*q)) { q++; any = true; }
  }
  if (!any) return kNaN;
  if (q < e && (*q == 'e' || *q == 'E')) {
    const char* r = q + 1;
    if (r < e && (*r == '+' || *r == '-')) r++;
    if (r < e && digit(*r)) {
      while (r < e && digit(*r)) r++;
      q = r;
    }
  }
  // strtod in the "C" locale: correctly rounded, overflow to +-inf and
  // underflow to +-0 as JS, and independent of the process locale (plain
  // strtod would read "1.5" as 1 under a locale with a decimal comma)
  static const locale_t c_locale = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  const std::string tok(s, q);
  return strtod_l(tok.c_str(), nullptr, c_locale);
}

// parseInt with no radix: white space, sign, "0x" -> base 16, else base 10;
// NaN when no digit.
double js_parse_int(const char* s, const char* e) {
  while (s < e && js_space(*s)) s++;
  bool neg = false;
  if (s < e && (*s == '+' || *s == '-')) {
    neg = *s == '-';
    s++;
  }
  int base = 10;
  if (e - s >= 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) {
    base = 16;
    s += 2;
  }
  double v = 0.0;
  bool any = false;
  for (; s < e; s++) {
    int d;
    if (digit(*s)) d = *s - '0';
    else if (base == 16 && *s >= 'a' && *s <= 'f') d = *s - 'a' + 10;
    else if (base == 16 && *s >= 'A' && *s <= 'F') d = *s - 'A' + 10;
    else break;
    v = v * base + d;
    any = true;
  }
  if (!any) return kNaN;
  return neg ? -v : v;
}

struct Span {
  const char* b;
  const char* e;
};

// String.prototype.split on one character: empty fields kept
void split(const char* b, const char* e, char c, std::vector<Span>& out) {
  out.clear();
  const char* s = b;
  for (const char* p = b; p < e; p++) {
    if (*p == c) {
      out.push_back({s, p});
      s = p + 1;
    }
  }
  out.push_back({s, e});
}

bool equals(const Span& s, const char* lit) {
  const size_t n = std::strlen(lit);
  return (size_t)(s.e - s.b) == n && std::strncmp(s.b, lit, n) == 0;
}

}  // namespace

bool parse_obj(const char* text, size_t len, std::vector<float>& out, std::string& err) {
  std::vector<double> vertices;  // JS numbers
  std::vector<double> faces;     // parseInt(..) - 1 per corner (NaN kept)
  std::vector<Span> lines, segs, parts;
  split(text, text + len, '\n', lines);
  auto field = [&](size_t i) { return i < segs.size() ? js_parse_float(segs[i].b, segs[i].e) : kNaN; };
  for (const Span& l : lines) {
    split(l.b, l.e, ' ', segs);
    if (equals(segs[0], "v")) {
      vertices.push_back(field(1));  // parseFloat(undefined) is NaN
      vertices.push_back(field(2));
      vertices.push_back(field(3));
    } else if (equals(segs[0], "f")) {
      if (segs.size() != 4) {
        err = "Non-triangular face in OBJ file";
        return false;
      }
      for (int k = 1; k <= 3; k++) {
        split(segs[k].b, segs[k].e, '/', parts);
        faces.push_back(js_parse_int(parts[0].b, parts[0].e) - 1.0);
      }
    }
    // 'vn', '#' and anything else: ignored (normals are parsed but unused, :24-27)
  }
  // outVertices[i*3+c] = vertices[face*3+c]; a missing vertex reads
  // undefined, which a Float32Array stores as NaN
  const size_t nv = vertices.size() / 3;
  out.assign(faces.size() * 3, 0.0f);
  for (size_t i = 0; i < faces.size(); i++) {
    const double f = faces[i];
    const bool ok = f == f && f >= 0.0 && f < (double)nv;
    for (int c = 0; c < 3; c++) out[3 * i + c] = ok ? (float)vertices[3 * (size_t)f + c] : std::nanf("");
  }
  return true;
}

void scale_vertices(std::vector<float>& v, const float scale[3]) {
  // index.ts:216-220: `vertices[i*3+c] *= s` on a Float32Array (f64 product, stored as f32)
  for (size_t i = 0; i < v.size(); i++) v[i] = (float)((double)v[i] * (double)scale[i % 3]);
}

}  // namespace wpt
