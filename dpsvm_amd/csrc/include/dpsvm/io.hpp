// Data and model I/O.
//
// Reference behaviour:
//   CSV loader  parse.cpp:10-43        (label first, then d features; first n lines)
//   model file  svmTrainMain.cpp:386-416  ("gamma\nb\n" then "alpha,y,x1..xd" per SV)
//   seq model   seq.cpp:295-321        (legacy: same without the b line)
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace dpsvm {

struct Dataset {
  int64_t n = 0;
  int d = 0;
  std::vector<float> x;  // n*d row-major
  std::vector<float> y;  // +1 / -1
};

// Read the first `n` rows (n <= 0: all rows) of a dense CSV "label,f1,...,fd".
// d <= 0 infers the feature count from the first row.  Rows with fewer than d
// features are zero-padded; extra columns are an error (reference: no checks).
// Labels are parsed as numbers and mapped to +1 / -1 (anything > 0 -> +1).
Dataset read_csv(const std::string& path, int64_t n, int d, int threads = 0);
// Rows [row0, row0+rows) only (shard-aware loading for partitioned X).
Dataset read_csv_rows(const std::string& path, int64_t row0, int64_t rows, int d, int threads = 0);
void write_csv(const std::string& path, const Dataset& ds);

// Sparse LIBSVM text ("+1 3:1 11:1 ...") -> dense, feature k (1-based) -> column k-1.
Dataset read_libsvm(const std::string& path, int d, int64_t n = 0);

struct Model {
  float gamma = 0.f;
  float b = 0.f;
  int d = 0;
  bool has_b = true;           // false: legacy seq format (no b line)
  std::vector<float> alpha;    // nsv
  std::vector<float> y;        // nsv
  std::vector<float> x;        // nsv*d
  int64_t nsv() const { return (int64_t)alpha.size(); }
};

// Support vectors (alpha != 0) in global index order (svmTrainMain.cpp:397).
Model make_model(const Dataset& ds, const std::vector<float>& alpha, float b, float gamma);
// precision: significant digits (reference: ostream default 6; we default to 9 = exact f32)
void write_model(const std::string& path, const Model& m, int precision = 9, bool legacy = false);
// Auto-detects the dpsvm format vs the legacy seq format (2nd line has commas).
Model read_model(const std::string& path, bool force_legacy = false);

// Deterministic synthetic generators (identical on every rank; row-seeded so a
// rank can generate only its own rows).
enum class Synth : int {
  MnistShape = 0,   // 784-d pixel-like features in [0,1] (~19% nonzero), random +/-1 labels
  MnistParity = 1,  // 784-d digit-like prototypes + noise, label = parity of the prototype
  AdultShape = 2,   // 123-d binary one-hot features, labels from a hidden rule (~24% +1)
  CovtypeShape = 3, // 54-d: 10 continuous in [0,1] + 44 binary; nonlinear labels
  Blobs = 4,        // two isotropic gaussians, unit variance, centres +/- sep/2 on axis 0
  Uniform = 5,      // dense uniform [0,1) features, random labels
};
Synth synth_from_name(const std::string& name);
std::string synth_name(Synth s);
int synth_default_d(Synth s);
Dataset make_synthetic(Synth kind, int64_t n, int d, uint64_t seed, int64_t row0 = 0,
                       int64_t rows = -1, float sep = 2.0f, int threads = 0);

// small helpers
void parallel_for(int64_t n, int threads, const std::function<void(int64_t, int64_t)>& fn);
int default_threads();

}  // namespace dpsvm
