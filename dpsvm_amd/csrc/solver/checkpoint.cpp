// Binary SMO checkpoint (absent from the reference).
// Layout: "DPSVMCK1" | u32 version | i64 n | i32 d | f32 C,gamma,eps | i32 clip |
//         i64 iter | f32 b_hi,b_lo | u8 has_f | f32 alpha[n] | f32 f[n] (if has_f)
// A checkpoint written at P ranks resumes at any P' (alpha and f are global).
#include <cstdio>

#include "dpsvm/solver.hpp"

namespace dpsvm {
namespace {
constexpr char kMagic[8] = {'D', 'P', 'S', 'V', 'M', 'C', 'K', '1'};
template <class T>
void put(FILE* fp, const T& v) {
  if (fwrite(&v, sizeof(T), 1, fp) != 1) fail("checkpoint write failed");
}
template <class T>
T get(FILE* fp) {
  T v;
  if (fread(&v, sizeof(T), 1, fp) != 1) fail("checkpoint truncated");
  return v;
}
}  // namespace

void write_checkpoint(const std::string& path, const Checkpoint& ck) {
  std::string tmp = path + ".tmp";
  FILE* fp = fopen(tmp.c_str(), "wb");
  if (!fp) fail("cannot write checkpoint " + tmp);
  fwrite(kMagic, 1, 8, fp);
  put<uint32_t>(fp, 1);
  put<int64_t>(fp, ck.n);
  put<int32_t>(fp, ck.d);
  put<float>(fp, ck.C);
  put<float>(fp, ck.gamma);
  put<float>(fp, ck.eps);
  put<int32_t>(fp, ck.clip);
  put<int64_t>(fp, ck.iter);
  put<float>(fp, ck.b_hi);
  put<float>(fp, ck.b_lo);
  DPSVM_CHECK((int64_t)ck.alpha.size() == ck.n, "checkpoint alpha size");
  uint8_t has_f = (int64_t)ck.f.size() == ck.n ? 1 : 0;
  put<uint8_t>(fp, has_f);
  if (fwrite(ck.alpha.data(), 4, (size_t)ck.n, fp) != (size_t)ck.n) fail("checkpoint write failed");
  if (has_f && fwrite(ck.f.data(), 4, (size_t)ck.n, fp) != (size_t)ck.n) fail("checkpoint write failed");
  if (fclose(fp) != 0) fail("checkpoint close failed");
  if (std::rename(tmp.c_str(), path.c_str()) != 0) fail("checkpoint rename failed");
}

Checkpoint read_checkpoint(const std::string& path) {
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) fail("cannot open checkpoint " + path);
  char magic[8];
  if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, kMagic, 8) != 0) {
    fclose(fp);
    fail("not a dpsvm checkpoint: " + path);
  }
  Checkpoint ck;
  try {
    uint32_t ver = get<uint32_t>(fp);
    if (ver != 1) fail("unsupported checkpoint version");
    ck.n = get<int64_t>(fp);
    ck.d = get<int32_t>(fp);
    ck.C = get<float>(fp);
    ck.gamma = get<float>(fp);
    ck.eps = get<float>(fp);
    ck.clip = get<int32_t>(fp);
    ck.iter = get<int64_t>(fp);
    ck.b_hi = get<float>(fp);
    ck.b_lo = get<float>(fp);
    uint8_t has_f = get<uint8_t>(fp);
    DPSVM_CHECK(ck.n > 0 && ck.n < (int64_t)1 << 40, "checkpoint: bad n");
    ck.alpha.resize((size_t)ck.n);
    if (fread(ck.alpha.data(), 4, (size_t)ck.n, fp) != (size_t)ck.n) fail("checkpoint truncated");
    if (has_f) {
      ck.f.resize((size_t)ck.n);
      if (fread(ck.f.data(), 4, (size_t)ck.n, fp) != (size_t)ck.n) fail("checkpoint truncated");
    }
  } catch (...) {
    fclose(fp);
    throw;
  }
  fclose(fp);
  return ck;
}

void check_resume(const Checkpoint& ck, int64_t n, int d, const SolverParams& p, float gamma) {
  auto bad = [&](const std::string& what, const std::string& ckv, const std::string& now) {
    fail("checkpoint does not match this problem: " + what + " = " + ckv + " in the checkpoint, " + now +
         " now (resume needs the same n, d, C, gamma and clip mode)");
  };
  if (ck.n != n || (int64_t)ck.alpha.size() != n) bad("n", std::to_string(ck.n), std::to_string(n));
  if (ck.d != d) bad("d", std::to_string(ck.d), std::to_string(d));
  if (ck.C != p.C) bad("C", std::to_string(ck.C), std::to_string(p.C));
  if (ck.gamma != gamma) bad("gamma", std::to_string(ck.gamma), std::to_string(gamma));
  if (ck.clip != (int)p.clip) bad("clip", std::to_string(ck.clip), std::to_string((int)p.clip));
  if (!ck.f.empty() && (int64_t)ck.f.size() != n) bad("f length", std::to_string(ck.f.size()), std::to_string(n));
}

}  // namespace dpsvm
