// svmSeq — CPU trainer (reference: seq.cpp, the single-threaded CBLAS SMO).
// Same flags (no -s); writes the dpsvm model format (with b) unless
// --legacy-model, and applies b in the training accuracy.
#include <iostream>

#include "cli_common.hpp"

using namespace dpsvm;

int main(int argc, char** argv) {
  cli::Options o = cli::parse_train(argc, argv, true);
  try {
    const double tl0 = cli::now_s();
    Dataset ds = cli::load_data(o);
    const double t_load = cli::now_s() - tl0;
    std::cout << "Populated Data from input file\n";
    std::unique_ptr<Checkpoint> resume;
    if (!o.resume.empty()) resume = std::make_unique<Checkpoint>(read_checkpoint(o.resume));
    ProgressFn prog = [](const Progress& p) {
      std::cout << "Current iteration number: " << p.iter << "  b_hi " << p.b_hi << "  b_lo " << p.b_lo << "\n";
    };
    SolveResult r = solve_cpu(ds, o.p, nullptr, resume.get(), prog);
    cli::print_outcome(r, o.p.eps);
    Model mdl = make_model(ds, r.alpha, r.b, o.p.gamma);
    cli::RunExtras extras;
    extras.t_load = t_load;
    double acc = -1;
    if (!o.skip_accuracy) {
      const double ta0 = cli::now_s();
      auto dec = decision_cpu(mdl, ds.x.data(), ds.n, ds.d);
      acc = accuracy_from_decision(dec, ds.y.data(), ds.n);
      extras.t_accuracy = cli::now_s() - ta0;
      std::cout << "Training accuracy: " << acc << "\n";
    }
    const double tw0 = cli::now_s();
    write_model(o.model, mdl, o.precision, o.legacy_model);
    extras.t_model_write = cli::now_s() - tw0;
    std::cout << "Training model has been saved to the file " << o.model << "\n";
    if (!o.metrics_json.empty())
      cli::write_metrics(o.metrics_json, o, r, ds.n, ds.d, mdl.nsv(), acc, "cpu", "cpu", extras);
    return 0;
  } catch (const std::exception& e) {
    std::cerr << "svmSeq: " << e.what() << "\n";
    return 1;
  }
}
