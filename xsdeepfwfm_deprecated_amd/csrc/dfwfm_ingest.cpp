// dfwfm_ingest.cpp -- native CSV / feature-map ingest (include/dfwfm_ingest.h).
//
// Host-side step before the forward (reference utils/data_preprocess.py:18-26, :54-72): the file is
// mmap'ed, split into n_threads byte ranges at line boundaries, each range counts its rows, a prefix
// sum gives every range its first output row, and the ranges parse in parallel straight into the
// caller's arrays.  No intermediate Python objects (the reference builds a list of lists per row).
#include "../../include/dfwfm_ingest.h"

#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

constexpr int kInvalid = -1, kUnsupported = -2, kIo = -3;

inline bool blank(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }

// [b, e) with surrounding blanks removed (Python str.strip())
inline void trim(const char*& b, const char*& e) {
  while (b < e && blank(*b)) ++b;
  while (e > b && blank(e[-1])) --e;
}

// Python int() of a decimal token
bool parse_int(const char* b, const char* e, int64_t* out) {
  trim(b, e);
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = *b == '-';
    ++b;
  }
  if (b == e) return false;
  uint64_t v = 0;
  for (; b < e; ++b) {
    if (*b < '0' || *b > '9') return false;
    const uint64_t d = (uint64_t)(*b - '0');
    if (v > (UINT64_MAX - d) / 10) return false;
    v = v * 10 + d;
  }
  if (v > (uint64_t)INT64_MAX + (neg ? 1u : 0u)) return false;
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

// Python float() of a token: decimal / exponent forms, inf / nan (no hex floats, as Python)
bool parse_float(const char* b, const char* e, double* out) {
  trim(b, e);
  if (b == e || e - b > 400) return false;
  char buf[416];
  memcpy(buf, b, (size_t)(e - b));
  buf[e - b] = 0;
  for (const char* p = buf; *p; ++p)
    if (*p == 'x' || *p == 'X') return false;
  char* end = nullptr;
  errno = 0;
  const double v = strtod(buf, &end);
  if (end != buf + (e - b)) return false;
  *out = v;  // ERANGE: strtod's +-inf / denormal / 0, as Python
  return true;
}

struct Range {
  size_t begin, end;   // byte range, whole lines
  int64_t rows = 0;    // non-empty lines
  int64_t lines = 0;   // all lines (for error line numbers)
  int64_t row0 = 0, line0 = 0;
};

bool empty_line(const char* b, const char* e) {
  trim(b, e);
  return b == e;
}

}  // namespace

struct dfwfm_csv {
  int fd = -1;
  const char* data = nullptr;
  size_t size = 0;
  int64_t rows = 0;
  int32_t cols = 0;
  std::vector<Range> ranges;
};

extern "C" {

const char* dfwfm_ingest_last_error(void) { return g_err.c_str(); }

void dfwfm_csv_close(dfwfm_csv* h) {
  if (!h) return;
  if (h->data && h->size) munmap(const_cast<char*>(h->data), h->size);
  if (h->fd >= 0) close(h->fd);
  delete h;
}

int dfwfm_csv_open(const char* path, int32_t n_threads, dfwfm_csv** out, int64_t* n_rows, int32_t* n_cols) {
  if (!path || !out || !n_rows || !n_cols) return fail(kInvalid, "null argument");
  *out = nullptr;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  dfwfm_csv* h = new dfwfm_csv();
  h->fd = open(path, O_RDONLY);
  if (h->fd < 0) {
    delete h;
    return fail(kIo, "%s: %s", path, strerror(errno));
  }
  struct stat st;
  if (fstat(h->fd, &st) != 0) {
    dfwfm_csv_close(h);
    return fail(kIo, "%s: %s", path, strerror(errno));
  }
  h->size = (size_t)st.st_size;
  if (h->size) {
    void* p = mmap(nullptr, h->size, PROT_READ, MAP_PRIVATE, h->fd, 0);
    if (p == MAP_FAILED) {
      h->size = 0;
      dfwfm_csv_close(h);
      return fail(kIo, "mmap %s: %s", path, strerror(errno));
    }
    madvise(p, h->size, MADV_SEQUENTIAL);
    h->data = static_cast<const char*>(p);
  }
  // byte ranges ending on line boundaries
  const char* d = h->data;
  const size_t n = h->size;
  size_t prev = 0;
  const int T = n < (size_t)1 << 20 ? 1 : n_threads;
  for (int t = 1; t <= T && prev < n; ++t) {
    size_t cut = t == T ? n : n * (size_t)t / (size_t)T;
    if (cut <= prev) continue;
    while (cut < n && d[cut - 1] != '\n') ++cut;
    Range r;
    r.begin = prev;
    r.end = cut;
    h->ranges.push_back(r);
    prev = cut;
  }
  // count rows and lines per range
  std::vector<std::thread> th;
  for (auto& r : h->ranges)
    th.emplace_back([&r, d]() {
      size_t i = r.begin;
      while (i < r.end) {
        const char* nl = static_cast<const char*>(memchr(d + i, '\n', r.end - i));
        const size_t e = nl ? (size_t)(nl - d) : r.end;
        r.lines += 1;
        if (!empty_line(d + i, d + e)) r.rows += 1;
        i = e + 1;
      }
    });
  for (auto& x : th) x.join();
  int64_t rows = 0, lines = 0;
  for (auto& r : h->ranges) {
    r.row0 = rows;
    r.line0 = lines;
    rows += r.rows;
    lines += r.lines;
  }
  h->rows = rows;
  // columns of the first non-empty line
  size_t i = 0;
  while (i < n) {
    const char* nl = static_cast<const char*>(memchr(d + i, '\n', n - i));
    const size_t e = nl ? (size_t)(nl - d) : n;
    const char* b = d + i;
    const char* eb = d + e;
    trim(b, eb);
    if (b < eb) {
      int32_t c = 1;
      for (const char* p = b; p < eb; ++p) c += *p == ',';
      h->cols = c;
      break;
    }
    i = e + 1;
  }
  *out = h;
  *n_rows = h->rows;
  *n_cols = h->cols;
  return 0;
}

int dfwfm_csv_parse(dfwfm_csv* h, const uint8_t* is_num, int64_t* labels, double* values, int64_t* indices,
                    int32_t n_threads) {
  (void)n_threads;  // the ranges fixed at open time set the parallelism
  if (!h || !is_num) return fail(kInvalid, "null argument");
  if (h->rows == 0) return 0;
  if (!labels) return fail(kInvalid, "null labels");
  const int C = h->cols;
  int nv = 0, ni = 0;
  for (int c = 1; c < C; ++c) (is_num[c] ? nv : ni) += 1;
  if ((nv && !values) || (ni && !indices)) return fail(kInvalid, "null output array");
  std::atomic<int> status{0};
  std::vector<std::string> errs(h->ranges.size());
  std::vector<std::thread> th;
  const char* d = h->data;
  for (size_t ri = 0; ri < h->ranges.size(); ++ri)
    th.emplace_back([&, ri]() {
      const Range& r = h->ranges[ri];
      int64_t row = r.row0, line = r.line0;
      size_t i = r.begin;
      while (i < r.end && status.load(std::memory_order_relaxed) == 0) {
        const char* nl = static_cast<const char*>(memchr(d + i, '\n', r.end - i));
        const size_t e = nl ? (size_t)(nl - d) : r.end;
        line += 1;
        const char* b = d + i;
        const char* eb = d + e;
        i = e + 1;
        trim(b, eb);
        if (b == eb) continue;
        int cc = 1;
        for (const char* p = b; p < eb; ++p) cc += *p == ',';
        if (cc != C) {
          errs[ri] = "line " + std::to_string(line) + ": " + std::to_string(cc) + " columns, expected " +
                     std::to_string(C);
          status.store(kInvalid);
          return;
        }
        int c = 0, v = 0, k = 0;
        const char* tok = b;
        for (const char* p = b;; ++p) {
          if (p == eb || *p == ',') {
            bool ok;
            if (c == 0) {
              ok = parse_int(tok, p, &labels[row]);
            } else if (is_num[c]) {
              ok = parse_float(tok, p, &values[row * nv + v]);
              ++v;
            } else {
              ok = parse_int(tok, p, &indices[row * ni + k]);
              ++k;
            }
            if (!ok) {
              errs[ri] = "line " + std::to_string(line) + ", column " + std::to_string(c) + ": invalid " +
                         (c != 0 && is_num[c] ? "float" : "int") + " '" + std::string(tok, (size_t)(p - tok)) + "'";
              status.store(kInvalid);
              return;
            }
            ++c;
            tok = p + 1;
            if (p == eb) break;
          }
        }
        ++row;
      }
    });
  for (auto& x : th) x.join();
  if (status.load() != 0) {
    for (auto& e : errs)
      if (!e.empty()) return fail(kInvalid, "%s", e.c_str());
    return fail(kInvalid, "parse error");
  }
  return 0;
}

int dfwfm_feature_map_counts(const char* path, int32_t start, int32_t dim, int64_t* counts) {
  if (!path || !counts || dim <= 0) return fail(kInvalid, "null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(kIo, "%s: %s", path, strerror(errno));
  std::vector<std::unordered_set<std::string>> keys((size_t)dim);
  std::string line;
  char buf[1 << 16];
  int64_t lineno = 0;
  int rc = 0;
  std::string carry;
  size_t got;
  auto handle = [&](const char* b, const char* e) -> int {
    lineno += 1;
    trim(b, e);
    if (b == e) return 0;
    const char* c1 = static_cast<const char*>(memchr(b, ',', (size_t)(e - b)));
    if (!c1) return fail(kInvalid, "%s line %lld: expected field,value,index", path, (long long)lineno);
    const char* c2 = static_cast<const char*>(memchr(c1 + 1, ',', (size_t)(e - c1 - 1)));
    if (!c2) return fail(kInvalid, "%s line %lld: expected field,value,index", path, (long long)lineno);
    int64_t field, idx;
    if (!parse_int(b, c1, &field) || !parse_int(c2 + 1, e, &idx))
      return fail(kInvalid, "%s line %lld: invalid int", path, (long long)lineno);
    const int64_t fi = field - start;
    if (fi < 0 || fi >= dim)
      return fail(kUnsupported, "%s line %lld: field %lld outside [%d, %d)", path, (long long)lineno,
                  (long long)field, start, start + dim);
    keys[(size_t)fi].emplace(c1 + 1, (size_t)(c2 - c1 - 1));
    return 0;
  };
  while (rc == 0 && (got = fread(buf, 1, sizeof buf, f)) > 0) {
    size_t i = 0;
    while (i < got && rc == 0) {
      const char* nl = static_cast<const char*>(memchr(buf + i, '\n', got - i));
      if (!nl) {
        carry.append(buf + i, got - i);
        break;
      }
      if (!carry.empty()) {
        carry.append(buf + i, (size_t)(nl - (buf + i)));
        rc = handle(carry.data(), carry.data() + carry.size());
        carry.clear();
      } else {
        rc = handle(buf + i, nl);
      }
      i = (size_t)(nl - buf) + 1;
    }
  }
  if (rc == 0 && !carry.empty()) rc = handle(carry.data(), carry.data() + carry.size());
  fclose(f);
  if (rc != 0) return rc;
  for (int i = 0; i < dim; ++i) counts[i] = (int64_t)keys[(size_t)i].size();
  return 0;
}

}  // extern "C"
