// Model file I/O (C4 writer, C11 reader in SURVEY §2).
//
// dpsvm format (svmTrainMain.cpp:386-416):   gamma \n b \n (alpha,y,x1,...,xd \n)*
// legacy seq format (seq.cpp:295-321):        gamma \n (alpha,y,x1,...,xd \n)*
// The reference writes with the ostream default of 6 significant digits; we
// default to 9 (round-trips every f32) and keep 6 available for byte parity.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"

namespace dpsvm {

Model make_model(const Dataset& ds, const std::vector<float>& alpha, float b, float gamma) {
  DPSVM_CHECK((int64_t)alpha.size() == ds.n, "alpha length != n");
  Model m;
  m.gamma = gamma;
  m.b = b;
  m.d = ds.d;
  for (int64_t i = 0; i < ds.n; ++i) {
    if (alpha[i] != 0.f) {
      m.alpha.push_back(alpha[i]);
      m.y.push_back(ds.y[i]);
      m.x.insert(m.x.end(), ds.x.begin() + (size_t)i * ds.d, ds.x.begin() + (size_t)(i + 1) * ds.d);
    }
  }
  return m;
}

void write_model(const std::string& path, const Model& m, int precision, bool legacy) {
  FILE* fp = fopen(path.c_str(), "w");
  if (!fp) fail("Model output file " + path + " could not be opened for writing.");
  std::vector<char> buf(1 << 20);
  setvbuf(fp, buf.data(), _IOFBF, buf.size());
  char fmt[16];
  snprintf(fmt, sizeof(fmt), "%%.%dg", precision);
  fprintf(fp, fmt, (double)m.gamma);
  fputc('\n', fp);
  if (!legacy) {
    fprintf(fp, fmt, (double)m.b);
    fputc('\n', fp);
  }
  char tmp[64];
  for (int64_t i = 0; i < m.nsv(); ++i) {
    fprintf(fp, fmt, (double)m.alpha[i]);
    fputs(m.y[i] > 0 ? ",1" : ",-1", fp);
    const float* xr = &m.x[(size_t)i * m.d];
    for (int k = 0; k < m.d; ++k) {
      if (xr[k] == 0.f) {
        fputs(",0", fp);
      } else {
        int len = snprintf(tmp, sizeof(tmp), fmt, (double)xr[k]);
        (void)len;
        fputc(',', fp);
        fputs(tmp, fp);
      }
    }
    fputc('\n', fp);
  }
  if (fclose(fp) != 0) fail("error writing model " + path);
}

namespace {
std::vector<float> split_floats(const std::string& line) {
  std::vector<float> v;
  const char* p = line.data();
  const char* e = p + line.size();
  while (p < e) {
    while (p < e && (*p == ' ' || *p == '\t')) ++p;
    if (p < e && *p == '+') ++p;
    float f;
    auto r = std::from_chars(p, e, f);
    if (r.ec != std::errc()) fail("model: bad number in line: " + line.substr(0, 80));
    v.push_back(f);
    p = r.ptr;
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
    if (p < e && *p == ',') ++p;
  }
  return v;
}
}  // namespace

Model read_model(const std::string& path, bool force_legacy) {
  std::ifstream in(path);
  if (!in.is_open()) fail("Couldn't open model file " + path);
  std::string line;
  Model m;
  if (!std::getline(in, line)) fail("model file " + path + " is empty");
  m.gamma = split_floats(line).at(0);
  std::string second;
  bool have_second = (bool)std::getline(in, second);
  bool legacy = force_legacy || (have_second && second.find(',') != std::string::npos);
  m.has_b = !legacy;
  std::vector<std::string> rows;
  if (legacy) {
    m.b = 0.f;
    if (have_second) rows.push_back(second);
  } else if (have_second) {
    m.b = split_floats(second).at(0);
  }
  while (std::getline(in, line)) {
    if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
    rows.push_back(line);
  }
  m.d = -1;
  for (auto& r : rows) {
    auto v = split_floats(r);
    if (v.size() < 2) fail("model: SV line too short");
    int d = (int)v.size() - 2;
    if (m.d < 0) m.d = d;
    if (d != m.d) fail("model: inconsistent SV dimensionality");
    m.alpha.push_back(v[0]);
    m.y.push_back(v[1] > 0 ? 1.f : -1.f);
    m.x.insert(m.x.end(), v.begin() + 2, v.end());
  }
  if (m.d < 0) m.d = 0;
  return m;
}

}  // namespace dpsvm
