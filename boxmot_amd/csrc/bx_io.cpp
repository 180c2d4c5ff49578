// bx_io.cpp — host-side MOT I/O (include/bxio.h): numpy-identical parsing of BoxMOT's det / emb
// text files and writing of MOT-challenge result rows.  Plain C++ on the host; no device code.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bxassoc.h"
#include "../../include/bxio.h"

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)

namespace {

struct File {
  std::vector<char> buf;
  bool ok = false;
  explicit File(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize((size_t)(n > 0 ? n : 0) + 1);
    ok = n <= 0 || std::fread(buf.data(), 1, (size_t)n, f) == (size_t)n;
    buf[(size_t)(n > 0 ? n : 0)] = '\0';
    std::fclose(f);
  }
};

// visit every data row: cb(row_index, begin, end) over the text before any '#'
template <class CB>
int64_t for_rows(const char* s, CB cb) {
  int64_t r = 0;
  while (*s) {
    const char* e = std::strchr(s, '\n');
    const char* end = e ? e : s + std::strlen(s);
    const char* h = (const char*)std::memchr(s, '#', (size_t)(end - s));
    const char* stop = h ? h : end;
    const char* p = s;
    while (p < stop && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
    if (p < stop) {
      if (!cb(r, p, stop)) return -1;
      r++;
    }
    s = e ? e + 1 : end;
  }
  return r;
}

int count_cols(const char* p, const char* stop) {
  int c = 0;
  while (p < stop) {
    while (p < stop && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
    if (p >= stop) break;
    c++;
    while (p < stop && !(*p == ' ' || *p == '\t' || *p == '\r')) p++;
  }
  return c;
}

}  // namespace

extern "C" {

int bx_txt_shape(const char* path, int64_t* rows, int32_t* cols) {
  if (!path || !rows || !cols) return bx_record_error(BX_ERR_INVALID, "null argument");
  File f(path);
  if (!f.ok) return bx_record_error(BX_ERR_INVALID, (std::string("cannot read ") + path).c_str());
  int c0 = -1;
  const int64_t n = for_rows(f.buf.data(), [&](int64_t, const char* p, const char* stop) {
    const int c = count_cols(p, stop);
    if (c0 < 0) c0 = c;
    return c == c0;
  });
  if (n < 0) return bx_record_error(BX_ERR_SHAPE, "rows with different numbers of columns");
  *rows = n;
  *cols = c0 < 0 ? 0 : c0;
  return BX_OK;
}

int bx_txt_read(const char* path, double* out, int64_t rows, int32_t cols) {
  if (!path || (!out && rows && cols)) return bx_record_error(BX_ERR_INVALID, "null argument");
  File f(path);
  if (!f.ok) return bx_record_error(BX_ERR_INVALID, (std::string("cannot read ") + path).c_str());
  bool bad = false;
  const int64_t n = for_rows(f.buf.data(), [&](int64_t r, const char* p, const char* stop) {
    if (r >= rows) return false;
    std::string line(p, stop);  // strtod needs a terminated run
    const char* q = line.c_str();
    for (int c = 0; c < cols; c++) {
      char* e = nullptr;
      errno = 0;
      const double v = std::strtod(q, &e);
      if (e == q) {
        bad = true;
        return false;
      }
      out[(size_t)r * cols + c] = v;
      q = e;
    }
    while (*q == ' ' || *q == '\t' || *q == '\r') q++;
    if (*q) {
      bad = true;
      return false;
    }
    return true;
  });
  if (bad || n != rows) return bx_record_error(BX_ERR_SHAPE, "text file does not match its shape");
  return BX_OK;
}

int bx_mot_format(const double* t, int64_t n, int32_t ncol, int32_t frame_idx, double* out) {
  if (n < 0 || ncol < 7 || (n && (!t || !out))) return bx_record_error(BX_ERR_INVALID, "bad arguments");
  for (int64_t k = 0; k < n; k++) {
    const double* r = t + (size_t)k * ncol;
    // ops.xyxy2ltwh: [x1, y1, x2 - x1, y2 - y1]; .round() half-to-even; astype(int32)
    const double l = r[0], tp = r[1], w = r[2] - r[0], h = r[3] - r[1];
    double* o = out + (size_t)k * 9;
    o[0] = (double)frame_idx;
    o[1] = (double)(int32_t)r[4];
    o[2] = (double)(int32_t)std::nearbyint(l);
    o[3] = (double)(int32_t)std::nearbyint(tp);
    o[4] = (double)(int32_t)std::nearbyint(w);
    o[5] = (double)(int32_t)std::nearbyint(h);
    o[6] = 1.0;
    o[7] = (double)(int32_t)r[6];
    o[8] = r[5];
  }
  return BX_OK;
}

int bx_mot_write(const char* path, const double* mot, int64_t n, int32_t append) {
  if (!path || (n && !mot)) return bx_record_error(BX_ERR_INVALID, "null argument");
  FILE* f = std::fopen(path, append ? "a" : "w");
  if (!f) return bx_record_error(BX_ERR_INVALID, (std::string("cannot write ") + path).c_str());
  for (int64_t k = 0; k < n; k++) {
    const double* o = mot + (size_t)k * 9;
    std::fprintf(f, "%lld,%lld,%lld,%lld,%lld,%lld,%lld,%lld,%.6f\n", (long long)o[0],
                 (long long)o[1], (long long)o[2], (long long)o[3], (long long)o[4],
                 (long long)o[5], (long long)o[6], (long long)o[7], o[8]);
  }
  std::fclose(f);
  return BX_OK;
}

}  // extern "C"
