// svmTest — predictor (reference: seq_test.cpp; the Makefile's svmTest target
// had no source).  Reads the dpsvm model format (auto-detects the
// legacy seq format), applies b (the reference ignored it, Q14) and computes
// decision values on MFMA (GpuPredictor) or on the CPU (--cpu / no GPU).
#include <getopt.h>

#include <iostream>

#include "cli_common.hpp"

using namespace dpsvm;

int main(int argc, char** argv) {
  int num_att = -1, device = 0;
  int64_t num_ex = -1;
  std::string file, model, synthetic, out_path;
  uint64_t seed = 0;
  float gamma = -1.f;
  bool cpu = false, legacy = false;
  enum { OPT_CPU = 1000, OPT_DEV, OPT_LEG, OPT_SYN, OPT_SEED, OPT_OUT };
  static struct option longopts[] = {
      {"num-att", required_argument, 0, 'a'}, {"num-ex", required_argument, 0, 'x'},
      {"file-path", required_argument, 0, 'f'}, {"gamma", required_argument, 0, 'g'},
      {"model", required_argument, 0, 'm'},   {"cpu", no_argument, 0, OPT_CPU},
      {"device", required_argument, 0, OPT_DEV}, {"legacy-model", no_argument, 0, OPT_LEG},
      {"synthetic", required_argument, 0, OPT_SYN}, {"seed", required_argument, 0, OPT_SEED},
      {"decision-out", required_argument, 0, OPT_OUT}, {0, 0, 0, 0}};
  while (true) {
    int idx = 0;
    int c = getopt_long(argc, argv, "a:x:f:g:m:", longopts, &idx);
    if (c == -1) break;
    switch (c) {
      case 'a': num_att = atoi(optarg); break;
      case 'x': num_ex = atoll(optarg); break;
      case 'f': file = optarg; break;
      case 'g': gamma = (float)atof(optarg); break;  // the model file's gamma takes precedence
      case 'm': model = optarg; break;
      case OPT_CPU: cpu = true; break;
      case OPT_DEV: device = atoi(optarg); break;
      case OPT_LEG: legacy = true; break;
      case OPT_SYN: synthetic = optarg; break;
      case OPT_SEED: seed = strtoull(optarg, nullptr, 10); break;
      case OPT_OUT: out_path = optarg; break;
      default:
        std::cerr << "usage: svmTest -a NUM_ATT -x NUM_EX -f TEST.csv -m MODEL [-g GAMMA] [--cpu] [--device N]\n"
                     "               [--legacy-model] [--synthetic NAME --seed N] [--decision-out PATH]\n";
        return -1;
    }
  }
  if ((file.empty() && synthetic.empty()) || model.empty() || num_att <= 0 || num_ex <= 0) {
    std::cerr << "Missing a required parameter, or invalid parameter\n"
                 "usage: svmTest -a NUM_ATT -x NUM_EX -f TEST.csv -m MODEL\n";
    return -1;
  }
  (void)gamma;
  try {
    Dataset ds = synthetic.empty() ? read_csv(file, num_ex, num_att)
                                   : make_synthetic(synth_from_name(synthetic), num_ex, num_att, seed);
    std::cout << "Populated test data\n";
    Model m = read_model(model, legacy);
    if (m.nsv() > 0 && m.d != num_att)
      fail("model has " + std::to_string(m.d) + " features, -a says " + std::to_string(num_att));
    m.d = num_att;
    std::cout << "Total number of Support Vectors: " << m.nsv() << "\n";
    std::cout << "Populated training model\n";
    std::vector<float> dec;
    const double t0 = cli::now_s();
    if (!cpu && device_count() > 0) {
      GpuPredictor p(m, device);
      dec = p.decision(ds.x.data(), ds.n, ds.d);
    } else {
      dec = decision_cpu(m, ds.x.data(), ds.n, ds.d);
    }
    const double t1 = cli::now_s();
    std::cout << "Test accuracy: " << accuracy_from_decision(dec, ds.y.data(), ds.n) << "\n";
    std::cout << "Prediction time in seconds: " << (t1 - t0) << "\n";
    if (!out_path.empty()) {
      FILE* fp = fopen(out_path.c_str(), "w");
      if (!fp) fail("cannot write " + out_path);
      for (float v : dec) fprintf(fp, "%.9g\n", v);
      fclose(fp);
    }
    return 0;
  } catch (const std::exception& e) {
    std::cerr << "svmTest: " << e.what() << "\n";
    return 1;
  }
}
