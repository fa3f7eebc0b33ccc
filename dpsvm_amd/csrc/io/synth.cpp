// Deterministic synthetic datasets of the reference's benchmark shapes.
//
// No datasets ship with the reference (.MISSING_LARGE_BLOBS) and there is no
// network, so every benchmark config (BASELINE.json) runs on generated data of
// the same shape.  Generation is row-seeded: row i depends only on (seed, i), so
// a rank can generate exactly its shard and every rank agrees bit-for-bit.
#include <algorithm>
#include <array>
#include <cmath>

#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"

namespace dpsvm {
namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(mix64(seed)) {}
  uint64_t next() { return s = mix64(s); }
  float uni() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }  // [0,1)
  float normal() {
    float u1 = std::max(uni(), 1e-7f), u2 = uni();
    return std::sqrt(-2.f * std::log(u1)) * std::cos(6.28318530718f * u2);
  }
};

constexpr uint64_t kTaskSeed = 0x5eed5eedull;

inline uint64_t row_seed(uint64_t seed, uint64_t kind, int64_t row) {
  return mix64(seed * 0x100000001b3ull ^ (kind << 56) ^ mix64((uint64_t)row + 0x51ed27ull));
}

// 10 digit-like 28x28 prototypes made of random gaussian strokes.
std::vector<float> digit_prototypes(uint64_t seed, int side) {
  std::vector<float> protos(10 * side * side, 0.f);
  for (int c = 0; c < 10; ++c) {
    Rng r(mix64(seed ^ (0xd161ull + c)));
    float* p = &protos[(size_t)c * side * side];
    int strokes = 3 + (int)(r.next() % 3);
    for (int s = 0; s < strokes; ++s) {
      float x0 = side * (0.25f + 0.5f * r.uni()), y0 = side * (0.25f + 0.5f * r.uni());
      float x1 = side * (0.25f + 0.5f * r.uni()), y1 = side * (0.25f + 0.5f * r.uni());
      for (int t = 0; t <= 24; ++t) {
        float cx = x0 + (x1 - x0) * t / 24.f, cy = y0 + (y1 - y0) * t / 24.f;
        for (int yy = 0; yy < side; ++yy)
          for (int xx = 0; xx < side; ++xx) {
            float dx = xx - cx, dy = yy - cy;
            float v = std::exp(-(dx * dx + dy * dy) / 2.0f);
            float& q = p[yy * side + xx];
            q = std::max(q, v);
          }
      }
    }
    for (int i = 0; i < side * side; ++i) p[i] = p[i] > 0.15f ? std::min(1.f, p[i] * 1.2f) : 0.f;
  }
  return protos;
}

}  // namespace

Synth synth_from_name(const std::string& name) {
  if (name == "mnist" || name == "mnist-shape" || name == "mnist_shape") return Synth::MnistShape;
  if (name == "mnist-parity" || name == "mnist_parity") return Synth::MnistParity;
  if (name == "adult" || name == "adult-shape" || name == "a9a") return Synth::AdultShape;
  if (name == "covtype" || name == "covtype-shape") return Synth::CovtypeShape;
  if (name == "blobs") return Synth::Blobs;
  if (name == "uniform" || name == "dense") return Synth::Uniform;
  fail("unknown synthetic dataset '" + name +
       "' (mnist, mnist-parity, adult, covtype, blobs, uniform)");
}

std::string synth_name(Synth s) {
  switch (s) {
    case Synth::MnistShape: return "mnist";
    case Synth::MnistParity: return "mnist-parity";
    case Synth::AdultShape: return "adult";
    case Synth::CovtypeShape: return "covtype";
    case Synth::Blobs: return "blobs";
    case Synth::Uniform: return "uniform";
  }
  return "?";
}

int synth_default_d(Synth s) {
  switch (s) {
    case Synth::MnistShape:
    case Synth::MnistParity: return 784;
    case Synth::AdultShape: return 123;
    case Synth::CovtypeShape: return 54;
    default: return 32;
  }
}

Dataset make_synthetic(Synth kind, int64_t n, int d, uint64_t seed, int64_t row0, int64_t rows,
                       float sep, int threads) {
  if (d <= 0) d = synth_default_d(kind);
  if (rows < 0) rows = n - row0;
  DPSVM_CHECK(row0 >= 0 && rows >= 0 && row0 + rows <= n, "synthetic row range out of bounds");
  Dataset ds;
  ds.n = rows;
  ds.d = d;
  ds.x.assign((size_t)rows * d, 0.f);
  ds.y.assign((size_t)rows, 0.f);
  const uint64_t k = (uint64_t)kind;

  std::vector<float> protos;
  int side = 0;
  if (kind == Synth::MnistParity) {
    side = (int)std::lround(std::sqrt((double)d));
    if (side * side != d) side = 0;
    // the "distribution" (prototypes, hidden rules) is fixed; the seed only
    // picks the samples, so different seeds give train/test splits of one task
    protos = digit_prototypes(kTaskSeed, side ? side : 28);
  }
  // adult: 14 categorical groups one-hot over 123 columns (a9a layout sizes)
  static const std::array<int, 14> adult_groups = {5, 8, 16, 16, 7, 14, 6, 5, 2, 3, 3, 3, 40, 2};
  // hidden linear rule for adult / covtype labels
  std::vector<float> w(d);
  {
    Rng r(mix64(kTaskSeed ^ 0xabcdefull ^ k));
    for (int j = 0; j < d; ++j) w[j] = r.normal();
  }

  parallel_for(rows, threads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      int64_t g = row0 + i;
      Rng r(row_seed(seed, k, g));
      float* x = &ds.x[(size_t)i * d];
      float y = 1.f;
      switch (kind) {
        case Synth::MnistShape: {
          // pixel-like: ~19% nonzero, values in (0,1], random +/-1 labels
          y = (r.next() & 1) ? 1.f : -1.f;
          for (int j = 0; j < d; ++j) {
            uint64_t u = r.next();
            if ((u & 0xffff) < 12452) x[j] = 1.0f - (float)(u >> 40) * (1.0f / 16777216.0f);
          }
          break;
        }
        case Synth::MnistParity: {
          int c = (int)(r.next() % 10);
          y = (c % 2 == 0) ? 1.f : -1.f;
          float inten = 0.7f + 0.3f * r.uni();
          int sd = side ? side * side : 784;
          for (int j = 0; j < d; ++j) {
            float p = protos[(size_t)c * sd + (j % sd)];
            float v = p > 0.f ? p * inten + 0.15f * r.normal() : (r.uni() < 0.02f ? r.uni() : 0.f);
            x[j] = std::min(1.f, std::max(0.f, v));
          }
          break;
        }
        case Synth::AdultShape: {
          int col = 0;
          float s = -1.1f;
          for (int gi = 0; gi < (int)adult_groups.size() && col < d; ++gi) {
            int gsz = std::min(adult_groups[gi], d - col);
            // skewed categorical: geometric-ish preference for low codes
            float u = r.uni();
            int pick = std::min(gsz - 1, (int)(gsz * u * u));
            x[col + pick] = 1.f;
            s += 0.45f * w[col + pick];
            col += gsz;
          }
          s += 0.6f * r.normal();
          y = s > 0.f ? 1.f : -1.f;
          break;
        }
        case Synth::CovtypeShape: {
          int ncont = std::min(10, d);
          float s = 0.f;
          for (int j = 0; j < ncont; ++j) {
            x[j] = r.uni();
            s += w[j] * std::sin(3.0f * x[j] + j);
          }
          int rem = d - ncont;
          if (rem > 0) {
            int wild = std::min(4, rem);
            int pw = (int)(r.next() % wild);
            x[ncont + pw] = 1.f;
            s += 0.5f * w[ncont + pw];
            if (rem > wild) {
              int soil = rem - wild;
              int ps = (int)(r.next() % soil);
              x[ncont + wild + ps] = 1.f;
              s += 0.5f * w[ncont + wild + ps];
            }
          }
          s += 0.3f * r.normal();
          y = s > 0.f ? 1.f : -1.f;
          break;
        }
        case Synth::Blobs: {
          y = (r.next() & 1) ? 1.f : -1.f;
          for (int j = 0; j < d; ++j) x[j] = r.normal();
          x[0] += y * sep * 0.5f;
          break;
        }
        case Synth::Uniform: {
          y = (r.next() & 1) ? 1.f : -1.f;
          for (int j = 0; j < d; ++j) x[j] = r.uni();
          break;
        }
      }
      ds.y[i] = y;
    }
  });
  return ds;
}

}  // namespace dpsvm
