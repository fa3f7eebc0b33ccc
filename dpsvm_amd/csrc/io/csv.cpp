// Dense CSV / LIBSVM readers (C5 in SURVEY §2).
//
// Reference: parse.cpp:10-43 reads the first n lines with getline + stringstream
// + stoi/stof, one rank at a time, the whole file on every rank.  Here the file
// is mmapped, line starts are found once, and rows are parsed in parallel with
// std::from_chars.  read_csv_rows() lets a rank parse only its own shard.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <fstream>
#include <thread>

#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"

namespace dpsvm {

int default_threads() {
  unsigned hc = std::thread::hardware_concurrency();
  if (const char* e = std::getenv("DPSVM_THREADS")) return std::max(1, atoi(e));
  if (const char* e = std::getenv("OMP_NUM_THREADS")) return std::max(1, atoi(e));
  return (int)std::max(1u, std::min(hc, 16u));
}

void parallel_for(int64_t n, int threads, const std::function<void(int64_t, int64_t)>& fn) {
  if (threads <= 0) threads = default_threads();
  if (n <= 0) return;
  int64_t t = std::min<int64_t>(threads, std::max<int64_t>(1, n / 256));
  if (t <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> ws;
  ws.reserve(t);
  for (int64_t i = 0; i < t; ++i) {
    int64_t b = n * i / t, e = n * (i + 1) / t;
    ws.emplace_back([&fn, b, e] { fn(b, e); });
  }
  for (auto& w : ws) w.join();
}

namespace {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit MappedFile(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) fail("Couldn't open file " + path);
    struct stat st;
    if (fstat(fd, &st) != 0) fail("stat failed: " + path);
    size = (size_t)st.st_size;
    if (size) {
      void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) fail("mmap failed: " + path);
      data = (const char*)p;
    }
  }
  ~MappedFile() {
    if (data) munmap((void*)data, size);
    if (fd >= 0) ::close(fd);
  }
};

// Offsets of the starts of non-empty lines [skip, skip+max_lines).
std::vector<size_t> line_starts(const MappedFile& f, int64_t skip, int64_t max_lines) {
  std::vector<size_t> starts;
  size_t pos = 0;
  int64_t seen = 0;
  while (pos < f.size) {
    const char* nl = (const char*)memchr(f.data + pos, '\n', f.size - pos);
    size_t end = nl ? (size_t)(nl - f.data) : f.size;
    bool blank = true;
    for (size_t i = pos; i < end; ++i)
      if (f.data[i] != '\r' && f.data[i] != ' ' && f.data[i] != '\t') { blank = false; break; }
    if (!blank) {
      if (seen >= skip) {
        starts.push_back(pos);
        if (max_lines > 0 && (int64_t)starts.size() >= max_lines) break;
      }
      ++seen;
    }
    pos = end + 1;
  }
  return starts;
}

inline const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t')) ++p;
  return p;
}

// parse one float; returns pointer after it or nullptr
inline const char* parse_float(const char* p, const char* e, float& out) {
  p = skip_ws(p, e);
  if (p < e && *p == '+') ++p;
  auto r = std::from_chars(p, e, out);
  if (r.ec != std::errc()) return nullptr;
  return r.ptr;
}

int count_fields(const char* p, const char* e) {
  int c = 1;
  for (; p < e && *p != '\n'; ++p)
    if (*p == ',') ++c;
  return c;
}

}  // namespace

Dataset read_csv_rows(const std::string& path, int64_t row0, int64_t rows, int d, int threads) {
  MappedFile f(path);
  auto starts = line_starts(f, row0, rows);
  Dataset ds;
  ds.n = (int64_t)starts.size();
  if (rows > 0 && ds.n < rows)
    fail("CSV " + path + " has only " + std::to_string(ds.n + row0) + " rows, need " +
         std::to_string(rows + row0));
  if (ds.n == 0) fail("CSV " + path + ": no rows");
  if (d <= 0) d = count_fields(f.data + starts[0], f.data + f.size) - 1;
  DPSVM_CHECK(d > 0, "CSV needs at least one feature column");
  ds.d = d;
  ds.x.assign((size_t)ds.n * d, 0.f);
  ds.y.assign((size_t)ds.n, 0.f);
  std::atomic<int64_t> bad_row{-1};
  parallel_for(ds.n, threads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      const char* p = f.data + starts[i];
      const char* end = (const char*)memchr(p, '\n', f.size - starts[i]);
      if (!end) end = f.data + f.size;
      float lab;
      const char* q = parse_float(p, end, lab);
      if (!q) { bad_row = i; continue; }
      ds.y[i] = lab > 0.f ? 1.f : -1.f;
      float* xr = &ds.x[(size_t)i * d];
      int k = 0;
      q = skip_ws(q, end);
      while (q < end && *q == ',') {
        ++q;
        q = skip_ws(q, end);
        if (q >= end || *q == '\r') break;
        if (k >= d) { bad_row = i; break; }
        float v;
        const char* r = parse_float(q, end, v);
        if (!r) { bad_row = i; break; }
        xr[k++] = v;
        q = skip_ws(r, end);
      }
    }
  });
  if (bad_row >= 0)
    fail("CSV " + path + ": malformed row " + std::to_string(bad_row + row0 + 1) +
         " (expected label + " + std::to_string(d) + " numeric features)");
  return ds;
}

Dataset read_csv(const std::string& path, int64_t n, int d, int threads) {
  return read_csv_rows(path, 0, n, d, threads);
}

void write_csv(const std::string& path, const Dataset& ds) {
  FILE* fp = fopen(path.c_str(), "w");
  if (!fp) fail("cannot write " + path);
  std::vector<char> buf(1 << 20);
  setvbuf(fp, buf.data(), _IOFBF, buf.size());
  char tmp[64];
  for (int64_t i = 0; i < ds.n; ++i) {
    fputs(ds.y[i] > 0 ? "1" : "-1", fp);
    const float* xr = &ds.x[(size_t)i * ds.d];
    for (int k = 0; k < ds.d; ++k) {
      float v = xr[k];
      if (v == 0.f) {
        fputs(",0", fp);
      } else {
        auto r = std::to_chars(tmp, tmp + sizeof(tmp), v);
        *r.ptr = 0;
        fputc(',', fp);
        fputs(tmp, fp);
      }
    }
    fputc('\n', fp);
  }
  fclose(fp);
}

Dataset read_libsvm(const std::string& path, int d, int64_t n) {
  MappedFile f(path);
  auto starts = line_starts(f, 0, n);
  Dataset ds;
  ds.n = (int64_t)starts.size();
  DPSVM_CHECK(d > 0, "read_libsvm needs d");
  ds.d = d;
  ds.x.assign((size_t)ds.n * d, 0.f);
  ds.y.assign((size_t)ds.n, 0.f);
  std::atomic<int64_t> bad{-1};
  parallel_for(ds.n, 0, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      const char* p = f.data + starts[i];
      const char* end = (const char*)memchr(p, '\n', f.size - starts[i]);
      if (!end) end = f.data + f.size;
      float lab;
      const char* q = parse_float(p, end, lab);
      if (!q) { bad = i; continue; }
      ds.y[i] = lab > 0 ? 1.f : -1.f;
      while (true) {
        q = skip_ws(q, end);
        if (q >= end || *q == '\r' || *q == '#') break;
        long idx;
        auto r = std::from_chars(q, end, idx);
        if (r.ec != std::errc() || r.ptr >= end || *r.ptr != ':') { bad = i; break; }
        float v;
        const char* r2 = parse_float(r.ptr + 1, end, v);
        if (!r2) { bad = i; break; }
        if (idx >= 1 && idx <= d) ds.x[(size_t)i * d + (idx - 1)] = v;
        q = r2;
      }
    }
  });
  if (bad >= 0) fail("libsvm file " + path + ": malformed line " + std::to_string(bad + 1));
  return ds;
}

}  // namespace dpsvm
