// Host-side CSV text of the fused engines' per-step loss rows.
//
// The reference logs every step (demo_pytorch_lightning.py: log_every_n_steps=0.03125,
// demo.py:114-121).  With a ~3 us training step on the GPU, writing those rows through
// Python's csv module (~5 us per row) made the host, not the GPU, the limit of the fused
// Trainer.  This formats a block of rows in one call with the csv module's exact text:
// Python's repr() of each value as a double (the shortest digits that round-trip, in
// exponent form when the decimal point sits at <= -4 or > 16, else fixed with at least one
// fractional digit), the row sum accumulated left to right as Python's sum() does, excel's
// "\r\n" line ends; and the JSONL lines of the engine logger.  Host code only (no kernels).
#include <charconv>
#include <cmath>
#include <cstring>

namespace {

int py_repr(double v, char* o) {
  if (std::isnan(v)) {
    std::memcpy(o, "nan", 3);
    return 3;
  }
  if (std::isinf(v)) {
    if (v < 0) {
      std::memcpy(o, "-inf", 4);
      return 4;
    }
    std::memcpy(o, "inf", 3);
    return 3;
  }
  char b[48];
  const auto r = std::to_chars(b, b + sizeof(b), v, std::chars_format::scientific);  // [-]d[.ddd]e[+-]XX
  const char* p = b;
  int n = 0;
  if (*p == '-') {
    o[n++] = '-';
    ++p;
  }
  char dig[32];
  int nd = 0;
  for (; p < r.ptr && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  int e = 0;
  bool eneg = false;
  for (++p; p < r.ptr; ++p) {
    if (*p == '-') eneg = true;
    else if (*p >= '0' && *p <= '9') e = 10 * e + (*p - '0');
  }
  if (eneg) e = -e;
  while (nd > 1 && dig[nd - 1] == '0') --nd;  // (shortest digits carry none, but "0e+00")
  const int decpt = e + 1;                    // value = 0.d1d2... x 10^decpt
  if (decpt <= -4 || decpt > 16) {
    o[n++] = dig[0];
    if (nd > 1) {
      o[n++] = '.';
      for (int i = 1; i < nd; ++i) o[n++] = dig[i];
    }
    o[n++] = 'e';
    int x = decpt - 1;
    o[n++] = x < 0 ? '-' : '+';
    if (x < 0) x = -x;
    char xb[8];
    int nx = 0;
    do {
      xb[nx++] = char('0' + x % 10);
      x /= 10;
    } while (x);
    if (nx < 2) xb[nx++] = '0';
    while (nx) o[n++] = xb[--nx];
  } else if (decpt <= 0) {
    o[n++] = '0';
    o[n++] = '.';
    for (int i = 0; i < -decpt; ++i) o[n++] = '0';
    for (int i = 0; i < nd; ++i) o[n++] = dig[i];
  } else if (nd <= decpt) {
    for (int i = 0; i < nd; ++i) o[n++] = dig[i];
    for (int i = nd; i < decpt; ++i) o[n++] = '0';
    o[n++] = '.';
    o[n++] = '0';
  } else {
    for (int i = 0; i < decpt; ++i) o[n++] = dig[i];
    o[n++] = '.';
    for (int i = decpt; i < nd; ++i) o[n++] = dig[i];
  }
  return n;
}

}  // namespace

extern "C" {

// Rows r = row0 + k * row_stride (k < count) of vals [*, ncols] (fp32): one line each,
// "step,v_0,...,v_{ncols-1}[,sum]\r\n" with step = step0 + k * step_stride.  Returns the
// bytes written, or -1 when `cap` cannot hold them (the caller sizes it with
// dtp_format_loss_rows_bound).
long long dtp_format_loss_rows(const float* vals, int ncols, long long row0, long long count, long long row_stride,
                               long long step0, long long step_stride, int with_sum, char* out, long long cap) {
  if (!vals || !out || ncols <= 0 || count < 0) return -1;
  long long n = 0;
  const long long line_max = 24 + (long long)(ncols + 1) * 28;
  for (long long k = 0; k < count; ++k) {
    if (n + line_max > cap) return -1;
    const float* r = vals + (row0 + k * row_stride) * ncols;
    const auto t = std::to_chars(out + n, out + cap, step0 + k * step_stride);
    n = t.ptr - out;
    double s = 0.0;
    for (int c = 0; c < ncols; ++c) {
      out[n++] = ',';
      const double v = (double)r[c];
      s += v;
      n += py_repr(v, out + n);
    }
    if (with_sum) {
      out[n++] = ',';
      n += py_repr(s, out + n);
    }
    out[n++] = '\r';
    out[n++] = '\n';
  }
  return n;
}

long long dtp_format_loss_rows_bound(int ncols, long long count) { return count * (24 + (long long)(ncols + 1) * 28); }

// The JSONL form of the same rows (utils/logging.py MetricLogger): one line
// '{"step": S, K0: v0, K1: v1}\n' per row, `keys` the json-quoted names each followed by
// '\n'; numbers as json.dumps spells them (repr, NaN, Infinity, -Infinity).
long long dtp_format_loss_rows_jsonl(const float* vals, int ncols, long long row0, long long count,
                                     long long row_stride, long long step0, long long step_stride, const char* keys,
                                     char* out, long long cap) {
  if (!vals || !out || !keys || ncols <= 0 || count < 0) return -1;
  const char* kp[64];
  int kl[64];
  if (ncols > 64) return -1;
  const char* q = keys;
  long long klen = 0;
  for (int c = 0; c < ncols; ++c) {
    kp[c] = q;
    while (*q && *q != '\n') ++q;
    if (!*q) return -1;
    kl[c] = (int)(q - kp[c]);
    klen += kl[c];
    ++q;
  }
  long long n = 0;
  const long long line_max = 40 + klen + (long long)ncols * 32;
  for (long long k = 0; k < count; ++k) {
    if (n + line_max > cap) return -1;
    const float* r = vals + (row0 + k * row_stride) * ncols;
    std::memcpy(out + n, "{\"step\": ", 9);
    n += 9;
    const auto t = std::to_chars(out + n, out + cap, step0 + k * step_stride);
    n = t.ptr - out;
    for (int c = 0; c < ncols; ++c) {
      out[n++] = ',';
      out[n++] = ' ';
      std::memcpy(out + n, kp[c], kl[c]);
      n += kl[c];
      out[n++] = ':';
      out[n++] = ' ';
      const double v = (double)r[c];
      if (std::isnan(v)) {
        std::memcpy(out + n, "NaN", 3);
        n += 3;
      } else if (std::isinf(v)) {
        const char* s = v < 0 ? "-Infinity" : "Infinity";
        const int ls = v < 0 ? 9 : 8;
        std::memcpy(out + n, s, ls);
        n += ls;
      } else {
        n += py_repr(v, out + n);
      }
    }
    out[n++] = '}';
    out[n++] = '\n';
  }
  return n;
}

long long dtp_format_loss_rows_jsonl_bound(int ncols, long long count, long long keys_len) {
  return count * (40 + keys_len + (long long)ncols * 32);
}

}  // extern "C"
