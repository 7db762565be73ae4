// wellflow native runtime — multithreaded CSV ingest (replaces spark.read.csv, cnn.py:65).
//
// The file is memory-mapped and cut into one byte range per worker at line boundaries; every
// worker parses its lines into typed per-column vectors (rows keep file order: ranges are
// concatenated in order). A row is dropped (and counted) when its field count differs from
// the schema or a numeric cell does not parse — Spark would turn such a cell into a null
// that the regression models cannot use (wellflow/data/io.py drops them the same way).
// Quoting: RFC-4180 double quotes inside one line ("" = a literal quote); a quoted field may
// not contain a newline. String columns are dictionary-encoded: per-worker dictionaries are
// merged in range order, so codes follow the first appearance in the file.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "wf_runtime.h"

namespace {

struct Column {
  int kind = WF_FLOAT;
  std::vector<int64_t> i64;
  std::vector<float> f32;
  std::vector<int32_t> codes;
  std::vector<std::string> vocab;
};

}  // namespace

struct wf_table {
  int64_t rows = 0, dropped = 0;
  std::vector<Column> cols;
};

namespace {

inline std::string_view trim(std::string_view s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
  return s.substr(a, b - a);
}

inline bool parse_int(std::string_view s, int64_t& v) {
  s = trim(s);
  if (s.empty()) return false;
  const char* b = s.data();
  const char* e = b + s.size();
  if (*b == '+') ++b;
  auto r = std::from_chars(b, e, v);
  if (r.ec == std::errc() && r.ptr == e) return true;
  // integral value written as a float ("3.0", "1e3"): accepted, like the tolerant Arrow path
  double d;
  auto r2 = std::from_chars(s.data() + (s[0] == '+'), e, d);
  if (r2.ec != std::errc() || r2.ptr != e || !std::isfinite(d) || std::floor(d) != d) return false;
  v = (int64_t)d;
  return true;
}

inline bool parse_float(std::string_view s, float& v) {
  s = trim(s);
  if (s.empty()) return false;
  const char* b = s.data();
  const char* e = b + s.size();
  if (*b == '+') ++b;
  auto r = std::from_chars(b, e, v);
  return r.ec == std::errc() && r.ptr == e;
}

struct Worker {
  std::vector<Column> cols;
  std::vector<std::unordered_map<std::string, int32_t>> dict;
  int64_t rows = 0, dropped = 0;
};

// Split one line into fields (quote-aware). Unquoted fields are views into the line; quoted
// ones are unescaped into `store`. Returns the field count (stops counting past `maxf`).
int split_line(std::string_view line, char delim, int maxf, std::vector<std::string_view>& f,
               std::vector<std::string>& store) {
  f.clear();
  size_t i = 0, n = line.size();
  int k = 0;
  while (true) {
    if (i < n && line[i] == '"') {  // quoted field
      std::string& s = store[k < maxf ? k : maxf];
      s.clear();
      ++i;
      while (i < n) {
        if (line[i] == '"') {
          if (i + 1 < n && line[i + 1] == '"') {
            s.push_back('"');
            i += 2;
          } else {
            ++i;
            break;
          }
        } else {
          s.push_back(line[i++]);
        }
      }
      while (i < n && line[i] != delim) ++i;  // junk after the closing quote is ignored
      if (k < maxf) f.emplace_back(s);
    } else {
      size_t j = i;
      while (j < n && line[j] != delim) ++j;
      if (k < maxf) f.emplace_back(line.substr(i, j - i));
      i = j;
    }
    ++k;
    if (i >= n) break;
    ++i;  // the delimiter
    if (i == n) {  // trailing delimiter: one more empty field
      if (k < maxf) f.emplace_back(std::string_view());
      ++k;
      break;
    }
  }
  return k;
}

void parse_range(const char* b, const char* e, char delim, const std::vector<int>& kinds, Worker& w) {
  const int nc = (int)kinds.size();
  w.cols.resize(nc);
  w.dict.resize(nc);
  for (int c = 0; c < nc; ++c) w.cols[c].kind = kinds[c];
  std::vector<std::string_view> f;
  f.reserve(nc + 1);
  std::vector<std::string> store(nc + 1);
  std::vector<int64_t> iv(nc);
  std::vector<float> fv(nc);
  const char* p = b;
  while (p < e) {
    const char* q = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p)));
    if (q == nullptr) q = e;
    std::string_view line(p, (size_t)(q - p));
    p = q + 1;
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    if (trim(line).empty()) continue;  // blank line
    if (split_line(line, delim, nc, f, store) != nc) {
      ++w.dropped;
      continue;
    }
    bool ok = true;
    for (int c = 0; c < nc && ok; ++c) {
      if (kinds[c] == WF_INT) ok = parse_int(f[c], iv[c]);
      else if (kinds[c] == WF_FLOAT) ok = parse_float(f[c], fv[c]);
    }
    if (!ok) {
      ++w.dropped;
      continue;
    }
    for (int c = 0; c < nc; ++c) {
      Column& col = w.cols[c];
      if (kinds[c] == WF_INT) {
        col.i64.push_back(iv[c]);
      } else if (kinds[c] == WF_FLOAT) {
        col.f32.push_back(fv[c]);
      } else {
        auto& d = w.dict[c];
        std::string key(f[c]);
        auto it = d.find(key);
        int32_t code;
        if (it == d.end()) {
          code = (int32_t)col.vocab.size();
          d.emplace(key, code);
          col.vocab.push_back(std::move(key));
        } else {
          code = it->second;
        }
        col.codes.push_back(code);
      }
    }
    ++w.rows;
  }
}

void set_err(char* err, int len, const std::string& msg) {
  if (err != nullptr && len > 0) {
    std::strncpy(err, msg.c_str(), (size_t)len - 1);
    err[len - 1] = 0;
  }
}

}  // namespace

extern "C" wf_table* wf_csv_read(const char* path, int ncols, const int* kinds_in, char delim, int header,
                                 int nthreads, char* err, int errlen) {
  if (ncols <= 0) {
    set_err(err, errlen, "no columns");
    return nullptr;
  }
  std::vector<int> kinds(kinds_in, kinds_in + ncols);
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    set_err(err, errlen, std::string("cannot open ") + path + ": " + std::strerror(errno));
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    set_err(err, errlen, std::string("cannot stat ") + path);
    close(fd);
    return nullptr;
  }
  const size_t size = (size_t)st.st_size;
  const char* data = nullptr;
  void* map = MAP_FAILED;
  if (size > 0) {
    map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (map == MAP_FAILED) {
      set_err(err, errlen, std::string("mmap failed for ") + path);
      close(fd);
      return nullptr;
    }
    madvise(map, size, MADV_SEQUENTIAL);
    data = static_cast<const char*>(map);
  }
  close(fd);

  const char* b = data;
  const char* e = data + size;
  if (header && b < e) {
    const char* nl = static_cast<const char*>(memchr(b, '\n', size));
    b = nl ? nl + 1 : e;
  }
  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  const size_t span = (size_t)(e - b);
  if (span < ((size_t)1 << 20)) nt = 1;  // small files: no thread start-up
  nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>(1, span >> 16));
  std::vector<const char*> cut(nt + 1);
  cut[0] = b;
  cut[nt] = e;
  for (int i = 1; i < nt; ++i) {
    const char* c = b + span * (size_t)i / (size_t)nt;
    if (c < cut[i - 1]) c = cut[i - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', (size_t)(e - c)));
    cut[i] = nl ? nl + 1 : e;
  }
  std::vector<Worker> ws(nt);
  {
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(parse_range, cut[i], cut[i + 1], delim, std::cref(kinds), std::ref(ws[i]));
    parse_range(cut[0], cut[1], delim, kinds, ws[0]);
    for (auto& t : th) t.join();
  }
  if (map != MAP_FAILED) munmap(map, size);

  auto* t = new wf_table();
  t->cols.resize(ncols);
  std::vector<int64_t> base(nt + 1, 0);
  for (int i = 0; i < nt; ++i) {
    base[i + 1] = base[i] + ws[i].rows;
    t->dropped += ws[i].dropped;
  }
  t->rows = base[nt];
  for (int c = 0; c < ncols; ++c) {
    Column& out = t->cols[c];
    out.kind = kinds[c];
    if (kinds[c] == WF_INT) {
      out.i64.resize(t->rows);
      for (int i = 0; i < nt; ++i)
        if (ws[i].rows) std::memcpy(out.i64.data() + base[i], ws[i].cols[c].i64.data(), ws[i].rows * sizeof(int64_t));
    } else if (kinds[c] == WF_FLOAT) {
      out.f32.resize(t->rows);
      for (int i = 0; i < nt; ++i)
        if (ws[i].rows) std::memcpy(out.f32.data() + base[i], ws[i].cols[c].f32.data(), ws[i].rows * sizeof(float));
    } else {
      // merge dictionaries in range order -> codes in first-appearance order over the file
      std::unordered_map<std::string, int32_t> gdict;
      std::vector<std::vector<int32_t>> remap(nt);
      for (int i = 0; i < nt; ++i) {
        if (ws[i].cols.empty()) continue;
        auto& lv = ws[i].cols[c].vocab;
        remap[i].resize(lv.size());
        for (size_t k = 0; k < lv.size(); ++k) {
          auto it = gdict.find(lv[k]);
          if (it == gdict.end()) {
            const int32_t g = (int32_t)out.vocab.size();
            gdict.emplace(lv[k], g);
            out.vocab.push_back(lv[k]);
            remap[i][k] = g;
          } else {
            remap[i][k] = it->second;
          }
        }
      }
      out.codes.resize(t->rows);
      for (int i = 0; i < nt; ++i) {
        if (ws[i].rows == 0) continue;
        const auto& lc = ws[i].cols[c].codes;
        int32_t* dst = out.codes.data() + base[i];
        for (int64_t r = 0; r < ws[i].rows; ++r) dst[r] = remap[i][lc[r]];
      }
    }
  }
  return t;
}

extern "C" int64_t wf_table_rows(const wf_table* t) { return t->rows; }
extern "C" int64_t wf_table_dropped(const wf_table* t) { return t->dropped; }
extern "C" const int64_t* wf_table_int(const wf_table* t, int c) { return t->cols[c].i64.data(); }
extern "C" const float* wf_table_float(const wf_table* t, int c) { return t->cols[c].f32.data(); }
extern "C" const int32_t* wf_table_codes(const wf_table* t, int c) { return t->cols[c].codes.data(); }
extern "C" int32_t wf_table_vocab_size(const wf_table* t, int c) { return (int32_t)t->cols[c].vocab.size(); }
extern "C" int64_t wf_table_vocab_bytes(const wf_table* t, int c) {
  int64_t n = 0;
  for (const auto& s : t->cols[c].vocab) n += (int64_t)s.size();
  return n;
}
extern "C" void wf_table_vocab(const wf_table* t, int c, char* bytes, int64_t* offsets) {
  int64_t o = 0;
  const auto& v = t->cols[c].vocab;
  for (size_t k = 0; k < v.size(); ++k) {
    offsets[k] = o;
    std::memcpy(bytes + o, v[k].data(), v[k].size());
    o += (int64_t)v[k].size();
  }
  offsets[v.size()] = o;
}
extern "C" void wf_table_free(wf_table* t) { delete t; }
