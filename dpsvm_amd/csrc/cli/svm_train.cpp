// svmTrain — distributed RBF C-SVM trainer (reference: svmTrainMain.cpp).
//
// Same flags and stdout lines as the reference.  Instead of `mpirun -np P`
// over TCP (Makefile:74), ranks are the GPUs of this node driven by one thread
// each over RCCL/xGMI (-p N), or simulated ranks sharing one device (--ranks N).
// Each rank binds its own GPU (the reference never calls cudaSetDevice).
#include <atomic>
#include <iostream>
#include <mutex>
#include <thread>

#include "cli_common.hpp"
#include "dpsvm/comm.hpp"

using namespace dpsvm;

int main(int argc, char** argv) {
  cli::Options o = cli::parse_train(argc, argv, false);
  try {
    const double tl0 = cli::now_s();
    Dataset ds = cli::load_data(o);
    const double t_load = cli::now_s() - tl0;
    cli::RunExtras extras;
    extras.t_load = t_load;
    const int64_t n = ds.n;
    const int d = ds.d;
    int world = o.ranks > 0 ? o.ranks : (o.cpu ? 1 : o.gpus);
    if (world < 1) world = 1;
    for (int r = 0; r < world; ++r) std::cout << "Populated Data from input file at node: " << r << "\n";
    for (int r = 0; r < world; ++r) {
      Shard s = shard_of(n, r, world);
      std::cout << s.offset << '\t' << s.size << '\n';
    }
    std::unique_ptr<Checkpoint> resume;
    if (!o.resume.empty()) {
      resume = std::make_unique<Checkpoint>(read_checkpoint(o.resume));
      std::cout << "Resuming from " << o.resume << " at iteration " << resume->iter << "\n";
    }

    std::vector<SolveResult> results((size_t)world);
    std::vector<double> accs((size_t)world, -1.0);
    std::string backend = o.cpu ? "cpu" : "hip";
    std::string devname = "cpu";
    std::mutex out_mu;
    auto progress = [&](const Progress& pr) {
      std::lock_guard<std::mutex> lk(out_mu);
      std::cout << "iter " << pr.iter << "  b_hi " << pr.b_hi << "  b_lo " << pr.b_lo << "  gap "
                << (pr.b_lo - pr.b_hi) << "  " << (pr.elapsed > 0 ? pr.iter / pr.elapsed : 0.0) << " it/s"
                << "  hits " << pr.hits << "  misses " << pr.misses << "\n";
    };

    std::vector<std::unique_ptr<Communicator>> comms;
    std::unique_ptr<ThreadCommGroup> group;
    if (world > 1) {
      if (o.ranks > 0 || o.cpu) {
        group = std::make_unique<ThreadCommGroup>(world);
        for (int r = 0; r < world; ++r) comms.push_back(group->comm(r));
        backend += o.cpu ? "+threads" : "+simulated-ranks";
      } else {
        int ndev = device_count();
        if (ndev < world) fail("requested " + std::to_string(world) + " GPUs, found " + std::to_string(ndev));
        std::vector<int> devs;
        for (int r = 0; r < world; ++r) devs.push_back(r);
        comms = make_rccl_comms_all(devs);
        backend += "+rccl";
      }
    } else {
      comms.push_back(make_local_comm());
    }

    std::vector<std::exception_ptr> errs((size_t)world);
    std::atomic<int> first_fail{-1};  // the rank whose error is the root cause
    auto rank_main = [&](int r) {
      try {
        Communicator* comm = comms[r].get();
        ProgressFn prog = r == 0 ? ProgressFn(progress) : ProgressFn();
        if (o.cpu) {
          results[r] = solve_cpu(ds, o.p, world > 1 ? comm : nullptr, resume.get(), prog);
          if (r == 0) std::cout << "SETUP DONE\n";
          return;
        }
        const int dev = (o.ranks > 0 || world == 1) ? o.device : r;
        if (o.shrink == 2 || (o.shrink == 0 && shrink_auto(o.p, n, d, dev, world > 1 ? comm : nullptr))) {
          // shrinking phases, each a (multi-rank) device solver on the active
          // rows (solver/gpu_shrink.cpp); training accuracy by the GPU predictor
          if (r == 0) {
            std::cout << "SETUP DONE\n";
            extras.engine = "ws+shrinking";
          }
          results[r] = solve_shrinking(o.p, dev, ds.x.data(), n, d, ds.y.data(), resume.get(), prog,
                                       world > 1 ? comm : nullptr);
          const double ta0 = cli::now_s();
          if (!o.skip_accuracy) {
            GpuPredictor pred(make_model(ds, results[r].alpha, results[r].b, o.p.gamma), dev);
            accs[r] = accuracy_from_decision(pred.decision(ds.x.data(), n, d), ds.y.data(), n);
          }
          extras.t_accuracy = cli::now_s() - ta0;
          return;
        }
        GpuSolver solver(o.p, comm, dev);
        GpuSetupInfo info = solver.setup(ds.x.data(), n, n, d, ds.y.data());
        if (world > 1) comm->barrier();
        if (r == 0) {
          std::lock_guard<std::mutex> lk(out_mu);
          devname = info.device_name;
          std::cout << "Device " << info.device << ": " << info.device_name << "  (X "
                    << (info.x_replicated ? "replicated" : "partitioned") << ", cache lines " << info.cache_lines
                    << (info.cache_lines >= n ? " = whole Gram shard resident" : " LRU") << ")\n";
          std::cout << "SETUP DONE\n";
        }
        if (r == 0) {
          extras.engine = info.iteration;
          extras.exchange = info.exchange;
          extras.setup = info;
        }
        results[r] = solver.solve(resume.get(), prog);
        const double ta0 = cli::now_s();
        if (!o.skip_accuracy) accs[r] = solver.train_accuracy(results[r]);
        if (r == 0) extras.t_accuracy = cli::now_s() - ta0;
      } catch (...) {
        errs[r] = std::current_exception();
        int none = -1;
        first_fail.compare_exchange_strong(none, r);
        // abort EVERY rank's communicator: peers blocked in a collective (or a
        // captured round graph) on a dead rank return now instead of at their
        // watchdog, and fail with "communicator aborted".  Only a REQUEST for
        // the other ranks' communicators: each owning thread carries it out
        // (RCCL: ncclCommAbort on the thread that enqueues, never under it)
        if (world > 1)
          for (int q = 0; q < world; ++q) {
            if (q == r)
              comms[q]->abort();
            else
              comms[q]->request_abort();
          }
      }
    };
    if (world == 1) {
      rank_main(0);
    } else {
      std::vector<std::thread> ts;
      for (int r = 0; r < world; ++r) ts.emplace_back(rank_main, r);
      for (auto& t : ts) t.join();
    }
    if (first_fail.load() >= 0) {
      // the peers' errors are consequences (aborted communicators): report
      // them after the root cause, which is what the process fails with
      for (int q = 0; q < world; ++q) {
        if (q == first_fail.load() || !errs[q]) continue;
        try {
          std::rethrow_exception(errs[q]);
        } catch (const std::exception& e) {
          std::cerr << "svmTrain: rank " << q << " (after rank " << first_fail.load() << " failed): " << e.what()
                    << "\n";
        }
      }
      std::cerr << "svmTrain: rank " << first_fail.load() << " failed first (root cause)\n";
      std::rethrow_exception(errs[first_fail.load()]);
    }

    SolveResult& r0 = results[0];
    cli::print_outcome(r0, o.p.eps);
    int64_t nsv = 0;
    for (float a : r0.alpha) nsv += a > 0.f;
    std::cout << "Number of SVs: " << nsv << "\n";
    double acc = accs[0];
    if (!o.skip_accuracy) {
      if (acc < 0) {
        const double ta0 = cli::now_s();
        Model mdl = make_model(ds, r0.alpha, r0.b, o.p.gamma);
        auto dec = decision_cpu(mdl, ds.x.data(), n, d);
        acc = accuracy_from_decision(dec, ds.y.data(), n);
        extras.t_accuracy = cli::now_s() - ta0;
      }
      std::cout << "Training accuracy: " << acc << "\n";
    }
    const double tw0 = cli::now_s();
    Model mdl = make_model(ds, r0.alpha, r0.b, o.p.gamma);
    write_model(o.model, mdl, o.precision, o.legacy_model);
    extras.t_model_write = cli::now_s() - tw0;
    std::cout << "Training model has been saved to the file " << o.model << "\n";
    if (!o.metrics_json.empty())
      cli::write_metrics(o.metrics_json, o, r0, n, d, nsv, acc, backend, devname, extras);
    return 0;
  } catch (const std::exception& e) {
    std::cerr << "svmTrain: " << e.what() << "\n";
    return 1;
  }
}
