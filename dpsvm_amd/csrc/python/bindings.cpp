// pybind11 bindings of the native core (module dpsvm_amd._C).
//
// Host arrays cross as numpy float32 (zero-copy where C-contiguous); device
// tensors cross as raw pointers + a hipStream_t handle (torch tensors'
// data_ptr() / torch.cuda.current_stream().cuda_stream), so this module has
// no compile-time dependency on torch.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "dpsvm/comm.hpp"
#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "dpsvm/io.hpp"
#include "dpsvm/solver.hpp"
#include "dpsvm/params_io.hpp"
#include "../kernels/kernels.hpp"

namespace py = pybind11;
using namespace dpsvm;

namespace {

using F32 = py::array_t<float, py::array::c_style | py::array::forcecast>;

py::array_t<float> to_np(const std::vector<float>& v) {
  py::array_t<float> a((py::ssize_t)v.size());
  if (!v.empty()) memcpy(a.mutable_data(), v.data(), v.size() * 4);
  return a;
}
py::array_t<float> to_np2(const std::vector<float>& v, int64_t rows, int cols) {
  py::array_t<float> a({(py::ssize_t)rows, (py::ssize_t)cols});
  if (!v.empty()) memcpy(a.mutable_data(), v.data(), v.size() * 4);
  return a;
}
std::vector<float> from_np(const F32& a) { return std::vector<float>(a.data(), a.data() + a.size()); }

void check_xy(const F32& x, const F32& y, int64_t& n, int& d) {
  if (x.ndim() != 2) throw py::value_error("x must be 2-D (n, d)");
  n = x.shape(0);
  d = (int)x.shape(1);
  if (y.ndim() != 1 || y.shape(0) != n) throw py::value_error("y must be 1-D with len(y) == x.shape[0]");
}

// Communicator backed by Python callables (torch.distributed / gloo, tests).
class CallbackComm final : public Communicator {
 public:
  CallbackComm(int rank, int size, py::function ar_min_u64, py::function ar_sum_f64, py::function ar_sum_f32,
               py::function allgather, py::function broadcast, py::function barrier)
      : rank_(rank), size_(size), min_(ar_min_u64), sum64_(ar_sum_f64), sum32_(ar_sum_f32),
        ag_(allgather), bc_(broadcast), bar_(barrier) {}
  ~CallbackComm() override {
    py::gil_scoped_acquire g;
    min_ = py::function(); sum64_ = py::function(); sum32_ = py::function();
    ag_ = py::function(); bc_ = py::function(); bar_ = py::function();
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  bool device_memory() const override { return false; }
  std::string name() const override { return "callback"; }
  void allreduce_min_u64(uint64_t* buf, size_t count, hipStream_t) override {
    py::gil_scoped_acquire g;
    py::array_t<uint64_t> a({(py::ssize_t)count}, {8}, buf, py::none());
    min_(a);
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t) override {
    py::gil_scoped_acquire g;
    py::array_t<double> a({(py::ssize_t)count}, {8}, buf, py::none());
    sum64_(a);
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t) override {
    py::gil_scoped_acquire g;
    py::array_t<float> a({(py::ssize_t)count}, {4}, buf, py::none());
    sum32_(a);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t) override {
    py::gil_scoped_acquire g;
    py::array_t<uint8_t> s({(py::ssize_t)bytes}, {1}, (const uint8_t*)send, py::none());
    py::array_t<uint8_t> r({(py::ssize_t)(bytes * size_)}, {1}, (uint8_t*)recv, py::none());
    // the send block may alias recv: hand Python a copy
    py::array_t<uint8_t> sc((py::ssize_t)bytes);
    memcpy(sc.mutable_data(), send, bytes);
    ag_(sc, r);
    (void)s;
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t) override {
    py::gil_scoped_acquire g;
    py::array_t<uint8_t> a({(py::ssize_t)bytes}, {1}, (uint8_t*)buf, py::none());
    bc_(a, root);
  }
  void barrier() override {
    py::gil_scoped_acquire g;
    bar_();
  }

 private:
  int rank_, size_;
  py::function min_, sum64_, sum32_, ag_, bc_, bar_;
};

py::dict result_dict(const SolveResult& r) {
  py::dict d;
  d["b"] = r.b;
  d["b_hi"] = r.b_hi;
  d["b_lo"] = r.b_lo;
  d["iters"] = r.iters;
  d["status"] = r.status;
  d["converged"] = r.converged();
  d["t_setup"] = r.t_setup;
  d["t_solve"] = r.t_solve;
  d["t_gram"] = r.t_gram;
  d["gram_tiles"] = r.gram_tiles;
  d["gram_hot_tiles"] = r.gram_hot_tiles;
  d["verify_f_err"] = r.verify_f_err;
  d["cache_hits"] = r.cache_hits;
  d["cache_misses"] = r.cache_misses;
  d["rows_computed"] = r.rows_computed;
  d["x_passes"] = r.x_passes;
  d["spec_rows"] = r.spec_rows;
  d["host_hits"] = r.host_hits;
  d["outer"] = r.outer;
  d["ws_blocks"] = r.ws_blocks;
  d["ws_blocks_end"] = r.ws_blocks_end;
  d["ws_p1_round"] = r.ws_p1_round;
  d["ws_damped"] = r.ws_damped;
  d["shrink_phases"] = r.shrink_phases;
  d["phase_log"] = r.phase_log;
  d["host_cache_lines"] = r.host_cache_lines;
  d["cache_lines"] = r.cache_lines;
  d["world"] = r.world;
  return d;
}

py::dict setup_dict(const GpuSetupInfo& i) {
  py::dict d;
  d["device"] = i.device;
  d["device_name"] = i.device_name;
  d["n"] = i.n;
  d["n_local"] = i.n_local;
  d["offset"] = i.offset;
  d["d"] = i.d;
  d["dp"] = i.dp;
  d["x_replicated"] = i.x_replicated;
  d["iteration"] = i.iteration;
  d["exchange"] = i.exchange;
  d["exchange_mem"] = i.exchange_mem;
  d["ws_exchange"] = i.ws_exchange;
  d["cache_lines"] = i.cache_lines;
  d["blocks"] = i.blocks;
  d["bytes_device"] = i.bytes_device;
  d["dp_policy"] = i.dp_policy;
  d["rows_per_group"] = i.rows_per_group;
  d["groups"] = i.groups;
  d["poll_batch"] = i.poll_batch;
  d["cus"] = i.cus;
  d["blocks_per_cu"] = i.blocks_per_cu;
  d["census"] = i.census;
  d["engine_note"] = i.engine_note;
  d["cache_note"] = i.cache_note;
  d["ws_wss"] = i.ws_wss;
  d["ws_rounds"] = i.ws_rounds;
  d["ws_rows"] = i.ws_rows;
  d["gram"] = i.gram;
  d["xch_selftest"] = i.xch_selftest;
  d["comm_kind"] = i.comm_kind;
  d["ws_blocks"] = i.ws_blocks;
  d["ws_q_max"] = i.ws_q_max;
  return d;
}

ProgressFn wrap_progress(py::object cb) {
  if (cb.is_none()) return {};
  py::function fn = cb;
  return [fn](const Progress& p) {
    py::gil_scoped_acquire g;
    fn(p.iter, p.b_hi, p.b_lo, p.elapsed, p.hits, p.misses);
  };
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "dpsvm_amd native core: MI355X modified-SMO RBF C-SVM";

  py::register_exception<Error>(m, "NativeError", PyExc_RuntimeError);

  py::enum_<ClipMode>(m, "ClipMode")
      .value("independent", ClipMode::Independent)
      .value("box", ClipMode::Box);

  py::class_<SolverParams>(m, "SolverParams")
      .def(py::init<>())
      .def_readwrite("C", &SolverParams::C)
      .def_readwrite("gamma", &SolverParams::gamma)
      .def_readwrite("eps", &SolverParams::eps)
      .def_readwrite("max_iter", &SolverParams::max_iter)
      .def_readwrite("clip", &SolverParams::clip)
      .def_readwrite("tau", &SolverParams::tau)
      .def_readwrite("cache_lines", &SolverParams::cache_lines)
      .def_readwrite("cache_mb", &SolverParams::cache_mb)
      .def_readwrite("cache_frac", &SolverParams::cache_frac)
      .def_readwrite("host_cache_lines", &SolverParams::host_cache_lines)
      .def_readwrite("spec_rows", &SolverParams::spec_rows)
      .def_readwrite("graph_block", &SolverParams::graph_block)
      .def_readwrite("use_graph", &SolverParams::use_graph)
      .def_readwrite("x_mode", &SolverParams::x_mode)
      .def_readwrite("log_every", &SolverParams::log_every)
      .def_readwrite("verbose", &SolverParams::verbose)
      .def_readwrite("checkpoint_every", &SolverParams::checkpoint_every)
      .def_readwrite("checkpoint_path", &SolverParams::checkpoint_path)
      .def_readwrite("sync_debug", &SolverParams::sync_debug)
      .def_readwrite("force_collectives", &SolverParams::force_collectives)
      .def_readwrite("exchange", &SolverParams::exchange)
      .def_readwrite("persist", &SolverParams::persist)
      .def_readwrite("persist_block", &SolverParams::persist_block)
      .def_readwrite("force_cache", &SolverParams::force_cache)
      .def_readwrite("cache_engine", &SolverParams::cache_engine)
      .def_readwrite("engines", &SolverParams::engines)
      .def_readwrite("cache_groups", &SolverParams::cache_groups)
      .def_readwrite("rows_per_group", &SolverParams::rows_per_group)
      .def_readwrite("xch_poll_batch", &SolverParams::xch_poll_batch)
      .def_readwrite("xch_sleep", &SolverParams::xch_sleep)
      .def_readwrite("xch_stride", &SolverParams::xch_stride)
      .def_readwrite("xch_mem", &SolverParams::xch_mem)
      .def_readwrite("xch_timeout_s", &SolverParams::xch_timeout_s)
      .def_readwrite("watchdog_s", &SolverParams::watchdog_s)
      .def_readwrite("census_groups", &SolverParams::census_groups)
      .def_readwrite("eta", &SolverParams::eta)
      .def_readwrite("verify_ranks", &SolverParams::verify_ranks)
      .def_readwrite("dp_policy", &SolverParams::dp_policy)
      .def_readwrite("solver", &SolverParams::solver)
      .def_readwrite("ws_size", &SolverParams::ws_size)
      .def_readwrite("ws_new", &SolverParams::ws_new)
      .def_readwrite("ws_rel", &SolverParams::ws_rel)
      .def_readwrite("ws_blocks", &SolverParams::ws_blocks)
      .def_readwrite("ws_inner", &SolverParams::ws_inner)
      .def_readwrite("ws_wss", &SolverParams::ws_wss)
      .def_readwrite("ws_t_halve", &SolverParams::ws_t_halve)
      .def_readwrite("ws_clip_fallback", &SolverParams::ws_clip_fallback)
      .def_readwrite("ws_block", &SolverParams::ws_block)
      .def_readwrite("ws_recompute", &SolverParams::ws_recompute)
      .def_readwrite("gram_precision", &SolverParams::gram_precision)
      .def_readwrite("gram_adapt", &SolverParams::gram_adapt)
      .def_readwrite("gram_cold_tau", &SolverParams::gram_cold_tau)
      .def("to_json", [](const SolverParams& p) { return params_json(p); })
      .def("update_from_json", [](SolverParams& p, const std::string& t) { apply_params_json(t, p); });

  py::class_<Checkpoint>(m, "Checkpoint")
      .def(py::init<>())
      .def_readwrite("n", &Checkpoint::n)
      .def_readwrite("d", &Checkpoint::d)
      .def_readwrite("C", &Checkpoint::C)
      .def_readwrite("gamma", &Checkpoint::gamma)
      .def_readwrite("eps", &Checkpoint::eps)
      .def_readwrite("clip", &Checkpoint::clip)
      .def_readwrite("iter", &Checkpoint::iter)
      .def_readwrite("b_hi", &Checkpoint::b_hi)
      .def_readwrite("b_lo", &Checkpoint::b_lo)
      .def_property("alpha", [](const Checkpoint& c) { return to_np(c.alpha); },
                    [](Checkpoint& c, F32 a) { c.alpha = from_np(a); })
      .def_property("f", [](const Checkpoint& c) { return to_np(c.f); },
                    [](Checkpoint& c, F32 a) { c.f = from_np(a); });
  // the device solver's engine choice (device_state.hpp kEngineTable, then
  // kQuarantineTable with engines=all), for docs and tests
  m.def("quarantine_loaded", []() { return quarantine_loaded(); },
        "true once the pair-cache plugin (libdpsvm_pairq.so) registered the quarantined engines");
  m.def("engine_table", [](bool quarantine) {
    std::vector<std::pair<std::string, std::string>> out;
    for (const EngineRule& r : kEngineTable) out.emplace_back(engine_name(r.kind), r.use);
    if (quarantine)
      for (const EngineRule& r : kQuarantineTable) out.emplace_back(engine_name(r.kind), r.use);
    return out;
  }, py::arg("quarantine") = false);
  m.def("choose_engine", [](bool ws_dense, bool ws_cache, bool dense, bool cache_replicated, bool persistent,
                            bool quarantine) -> py::object {
    EngineFacts f;
    f.ws_dense = ws_dense;
    f.ws_cache = ws_cache;
    f.dense = dense;
    f.cache_replicated = cache_replicated;
    f.persistent = persistent;
    f.quarantine = quarantine;
    EngineKind k;
    if (!choose_engine(f, &k)) return py::none();
    return py::str(engine_name(k));
  }, py::arg("ws_dense") = false, py::arg("ws_cache") = false, py::arg("dense") = false,
        py::arg("cache_replicated") = false, py::arg("persistent") = false, py::arg("quarantine") = false);
  m.def("write_checkpoint", &write_checkpoint, py::arg("path"), py::arg("ck"));
  m.def("read_checkpoint", &read_checkpoint, py::arg("path"));

  // ---------------- communicators ----------------
  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("size", &Communicator::size)
      .def_property_readonly("name", &Communicator::name)
      .def_property_readonly("device_memory", &Communicator::device_memory)
      .def("barrier", [](Communicator& c) { py::gil_scoped_release r; c.barrier(); });
  m.def("local_comm", []() { return std::shared_ptr<Communicator>(make_local_comm()); });
  py::class_<ThreadCommGroup, std::shared_ptr<ThreadCommGroup>>(m, "ThreadCommGroup")
      .def(py::init<int>(), py::arg("world"))
      .def("comm", [](ThreadCommGroup& g, int r) { return std::shared_ptr<Communicator>(g.comm(r)); });
  m.def("rccl_unique_id", []() {
    auto v = rccl_unique_id();
    return py::bytes((const char*)v.data(), v.size());
  });
  m.def("rccl_comm", [](py::bytes uid, int rank, int world, int device) {
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    py::gil_scoped_release r;
    return std::shared_ptr<Communicator>(make_rccl_comm(v, rank, world, device));
  }, py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"));
  m.def("callback_comm", [](int rank, int size, py::function a, py::function b, py::function c, py::function d,
                            py::function e, py::function f) {
    return std::shared_ptr<Communicator>(new CallbackComm(rank, size, a, b, c, d, e, f));
  });

  // ---------------- data ----------------
  m.def("read_csv", [](const std::string& path, int64_t n, int d, int threads) {
    Dataset ds;
    {
      py::gil_scoped_release r;
      ds = read_csv(path, n, d, threads);
    }
    return py::make_tuple(to_np2(ds.x, ds.n, ds.d), to_np(ds.y));
  }, py::arg("path"), py::arg("n") = 0, py::arg("d") = 0, py::arg("threads") = 0);
  m.def("read_csv_rows", [](const std::string& path, int64_t row0, int64_t rows, int d) {
    Dataset ds;
    {
      py::gil_scoped_release r;
      ds = read_csv_rows(path, row0, rows, d, 0);
    }
    return py::make_tuple(to_np2(ds.x, ds.n, ds.d), to_np(ds.y));
  });
  m.def("write_csv", [](const std::string& path, F32 x, F32 y) {
    Dataset ds;
    check_xy(x, y, ds.n, ds.d);
    ds.x = from_np(x);
    ds.y = from_np(y);
    py::gil_scoped_release r;
    write_csv(path, ds);
  });
  m.def("read_libsvm", [](const std::string& path, int d, int64_t n) {
    Dataset ds = read_libsvm(path, d, n);
    return py::make_tuple(to_np2(ds.x, ds.n, ds.d), to_np(ds.y));
  }, py::arg("path"), py::arg("d"), py::arg("n") = 0);
  m.def("make_synthetic", [](const std::string& name, int64_t n, int d, uint64_t seed, int64_t row0,
                             int64_t rows, float sep) {
    Dataset ds;
    {
      py::gil_scoped_release r;
      ds = make_synthetic(synth_from_name(name), n, d, seed, row0, rows, sep, 0);
    }
    return py::make_tuple(to_np2(ds.x, ds.n, ds.d), to_np(ds.y));
  }, py::arg("name"), py::arg("n"), py::arg("d") = 0, py::arg("seed") = 0, py::arg("row0") = 0,
     py::arg("rows") = -1, py::arg("sep") = 2.0f);
  m.def("synth_default_d", [](const std::string& name) { return synth_default_d(synth_from_name(name)); });

  // ---------------- model ----------------
  py::class_<Model>(m, "Model")
      .def(py::init<>())
      .def_readwrite("gamma", &Model::gamma)
      .def_readwrite("b", &Model::b)
      .def_readwrite("d", &Model::d)
      .def_readwrite("has_b", &Model::has_b)
      .def_property_readonly("nsv", &Model::nsv)
      .def_property("alpha", [](const Model& md) { return to_np(md.alpha); },
                    [](Model& md, F32 a) { md.alpha = from_np(a); })
      .def_property("y", [](const Model& md) { return to_np(md.y); }, [](Model& md, F32 a) { md.y = from_np(a); })
      .def_property("x", [](const Model& md) { return to_np2(md.x, md.nsv(), md.d); },
                    [](Model& md, F32 a) { md.x = from_np(a); });
  m.def("make_model", [](F32 x, F32 y, F32 alpha, float b, float gamma) {
    Dataset ds;
    check_xy(x, y, ds.n, ds.d);
    ds.x = from_np(x);
    ds.y = from_np(y);
    return make_model(ds, from_np(alpha), b, gamma);
  });
  m.def("write_model", &write_model, py::arg("path"), py::arg("model"), py::arg("precision") = 9,
        py::arg("legacy") = false);
  m.def("read_model", &read_model, py::arg("path"), py::arg("force_legacy") = false);
  m.def("decision_cpu", [](const Model& md, F32 x, int threads) {
    if (x.ndim() != 2) throw py::value_error("x must be 2-D");
    std::vector<float> dec;
    {
      py::gil_scoped_release r;
      dec = decision_cpu(md, x.data(), x.shape(0), (int)x.shape(1), threads);
    }
    return to_np(dec);
  }, py::arg("model"), py::arg("x"), py::arg("threads") = 0);

  // ---------------- solvers ----------------
  m.def("solve_cpu", [](F32 x, F32 y, const SolverParams& p, std::shared_ptr<Communicator> comm,
                        const Checkpoint* resume, py::object progress) {
    Dataset ds;
    check_xy(x, y, ds.n, ds.d);
    ds.x = from_np(x);
    ds.y = from_np(y);
    for (auto& v : ds.y) v = v > 0 ? 1.f : -1.f;
    auto prog = wrap_progress(progress);
    SolveResult r;
    {
      py::gil_scoped_release rel;
      r = solve_cpu(ds, p, comm.get(), resume, prog);
    }
    return py::make_tuple(to_np(r.alpha), result_dict(r));
  }, py::arg("x"), py::arg("y"), py::arg("params"), py::arg("comm") = nullptr, py::arg("resume") = nullptr,
     py::arg("progress") = py::none());

  m.def("solve_shrinking", [](F32 x, F32 y, const SolverParams& p, int device, const Checkpoint* resume,
                              py::object progress, std::shared_ptr<Communicator> comm) {
    int64_t n = 0;
    int d = 0;
    check_xy(x, y, n, d);
    auto prog = wrap_progress(progress);
    SolveResult r;
    {
      py::gil_scoped_release rel;
      r = solve_shrinking(p, device, x.data(), n, d, y.data(), resume, prog, comm.get());
    }
    return py::make_tuple(to_np(r.alpha), result_dict(r));
  }, py::arg("x"), py::arg("y"), py::arg("params"), py::arg("device") = 0, py::arg("resume") = nullptr,
     py::arg("progress") = py::none(), py::arg("comm") = nullptr);
  m.def("shrink_auto", [](const SolverParams& p, int64_t n, int d, int device, std::shared_ptr<Communicator> comm) {
          py::gil_scoped_release rel;
          return shrink_auto(p, n, d, device, comm.get());
        }, py::arg("params"), py::arg("n"), py::arg("d"), py::arg("device") = 0, py::arg("comm") = nullptr,
        "shrink='auto': shrinking phases where they pay (working-set rounds, the whole Gram not resident on "
        "one device; agreed over comm)");

  py::class_<GpuSolver, std::shared_ptr<GpuSolver>>(m, "GpuSolver")
      .def(py::init([](const SolverParams& p, std::shared_ptr<Communicator> comm, int device) {
             // keep the communicator alive as long as the solver
             auto* s = new GpuSolver(p, comm.get(), device);
             return std::shared_ptr<GpuSolver>(s, [comm](GpuSolver* q) { delete q; });
           }),
           py::arg("params"), py::arg("comm") = nullptr, py::arg("device") = 0)
      .def("setup", [](GpuSolver& s, F32 x, int64_t n, F32 y) {
        if (x.ndim() != 2) throw py::value_error("x must be 2-D");
        if (y.ndim() != 1 || y.shape(0) != n) throw py::value_error("y must have n entries");
        GpuSetupInfo i;
        {
          py::gil_scoped_release r;
          i = s.setup(x.data(), x.shape(0), n, (int)x.shape(1), y.data());
        }
        return setup_dict(i);
      })
      .def("solve", [](GpuSolver& s, const Checkpoint* resume, py::object progress) {
        auto prog = wrap_progress(progress);
        SolveResult r;
        {
          py::gil_scoped_release rel;
          r = s.solve(resume, prog);
        }
        return py::make_tuple(to_np(r.alpha), result_dict(r));
      }, py::arg("resume") = nullptr, py::arg("progress") = py::none())
      .def("train_accuracy", [](GpuSolver& s, F32 alpha, float b) {
        SolveResult r;
        r.alpha = from_np(alpha);
        r.b = b;
        py::gil_scoped_release rel;
        return s.train_accuracy(r);
      })
      .def("decision", [](GpuSolver& s, F32 alpha, float b, F32 x) {
        SolveResult r;
        r.alpha = from_np(alpha);
        r.b = b;
        std::vector<float> out;
        {
          py::gil_scoped_release rel;
          out = s.decision(r, x.data(), x.shape(0), (int)x.shape(1));
        }
        return to_np(out);
      });

  // shrinking phases with the whole-problem solver set up once (setup() outside
  // a timed region, as GpuSolver's); keeps X / y and the communicator alive
  struct PyShrink {
    std::shared_ptr<Communicator> comm;
    std::unique_ptr<ShrinkingSolver> s;
    F32 x, y;
  };
  py::class_<PyShrink, std::shared_ptr<PyShrink>>(m, "ShrinkingSolver")
      .def(py::init([](const SolverParams& p, std::shared_ptr<Communicator> comm, int device) {
             auto h = std::make_shared<PyShrink>();
             h->comm = comm;
             h->s.reset(new ShrinkingSolver(p, comm.get(), device));
             return h;
           }),
           py::arg("params"), py::arg("comm") = nullptr, py::arg("device") = 0)
      .def("setup", [](PyShrink& h, F32 x, F32 y) {
        int64_t n = 0;
        int d = 0;
        check_xy(x, y, n, d);
        h.x = x;
        h.y = y;
        GpuSetupInfo i;
        {
          py::gil_scoped_release r;
          i = h.s->setup(h.x.data(), n, d, h.y.data());
        }
        py::dict out = setup_dict(i);
        out["phase0_engine"] = i.iteration;
        out["iteration"] = "ws+shrinking";
        return out;
      }, py::arg("x"), py::arg("y"))
      .def("solve", [](PyShrink& h, const Checkpoint* resume, py::object progress) {
        auto prog = wrap_progress(progress);
        SolveResult r;
        {
          py::gil_scoped_release rel;
          r = h.s->solve(resume, prog);
        }
        return py::make_tuple(to_np(r.alpha), result_dict(r));
      }, py::arg("resume") = nullptr, py::arg("progress") = py::none());

  py::class_<GpuPredictor, std::shared_ptr<GpuPredictor>>(m, "GpuPredictor")
      .def(py::init<const Model&, int, int>(), py::arg("model"), py::arg("device") = 0, py::arg("precision") = 0)
      .def("decision", [](GpuPredictor& p, F32 x) {
        if (x.ndim() != 2) throw py::value_error("x must be 2-D");
        std::vector<float> out;
        {
          py::gil_scoped_release rel;
          out = p.decision(x.data(), x.shape(0), (int)x.shape(1));
        }
        return to_np(out);
      })
      .def("decision_device", [](GpuPredictor& p, uintptr_t x, int64_t n, int d, int ld, uintptr_t out,
                                 uintptr_t stream) {
        py::gil_scoped_release rel;
        p.decision_device((const float*)x, n, d, ld, (float*)out, (void*)stream);
      });

  // ---------------- kernel test entry points (device pointers) ----------------
  m.def("k_row_sqnorm", [](uintptr_t x, int64_t n, int d, int ld, uintptr_t out, uintptr_t stream) {
    kernels::row_sqnorm((const float*)x, n, d, ld, (float*)out, (void*)stream);
  });
  m.def("k_rbf_rows", [](uintptr_t x, uintptr_t xsq, int64_t n, int ld, uintptr_t w, uintptr_t wsq, int nq,
                         float gamma, uintptr_t out, int64_t out_ld, uintptr_t stream) {
    kernels::rbf_rows((const float*)x, (const float*)xsq, n, ld, (const float*)w, (const float*)wsq, nq, gamma,
                      (float*)out, out_ld, (void*)stream);
  });
  m.def("k_select_partials", [](uintptr_t f, uintptr_t alpha, uintptr_t y, int64_t n, int64_t off, float C,
                                uintptr_t partials, uintptr_t stream) {
    int blocks = 0;
    kernels::select_partials((const float*)f, (const float*)alpha, (const float*)y, n, off, C,
                             (uint64_t*)partials, &blocks, (void*)stream);
    return blocks;
  });
  m.def("k_predict", [](uintptr_t x, uintptr_t xsq, int64_t n, int ld, uintptr_t sv, uintptr_t svsq,
                        uintptr_t coef, int64_t nsv, float gamma, float b, uintptr_t dec, uintptr_t stream) {
    kernels::predict((const float*)x, (const float*)xsq, n, ld, (const float*)sv, (const float*)svsq,
                     (const float*)coef, nsv, ld, gamma, b, (float*)dec, (void*)stream);
  });
  m.def("k_rbf_gram", [](uintptr_t a, uintptr_t asq, int64_t m_, uintptr_t b, uintptr_t bsq, int64_t n, int ld,
                         float gamma, uintptr_t out, int64_t out_ld, bool symmetric, uintptr_t stream) {
    kernels::rbf_gram((const float*)a, (const float*)asq, m_, (const float*)b, (const float*)bsq, n, ld, gamma,
                      (float*)out, out_ld, symmetric, (void*)stream);
  });
  m.def("k_compact", [](uintptr_t alpha, int64_t n, uintptr_t idx, uintptr_t stream) {
    return kernels::compact_nonzero((const float*)alpha, n, (int*)idx, (void*)stream);
  });
  m.def("k_xpass_rows", [](uintptr_t x, uintptr_t xsq, int64_t n, int ld, uintptr_t keys, int nq, float gamma,
                           uintptr_t out, int64_t out_ld, int rows, uintptr_t stream) {
    kernels::xpass_rows((const float*)x, (const float*)xsq, n, ld, (const int*)keys, nq, gamma, (float*)out, out_ld,
                        rows, (void*)stream);
  });
  m.def("k_rbf_rows_indexed", [](uintptr_t x, uintptr_t xsq, int64_t n, int ld, uintptr_t rows, int m_, float gamma,
                                 uintptr_t out, int64_t out_ld, uintptr_t out_rows, uintptr_t stream, bool split) {
    kernels::rbf_rows_indexed((const float*)x, (const float*)xsq, n, ld, (const int*)rows, m_, gamma, (float*)out,
                              out_ld, (const int*)out_rows, (void*)stream, split);
  }, py::arg("x"), py::arg("xsq"), py::arg("n"), py::arg("ld"), py::arg("rows"), py::arg("m"), py::arg("gamma"),
        py::arg("out"), py::arg("out_ld"), py::arg("out_rows"), py::arg("stream"), py::arg("split") = false);
  m.def("k_rows_split_bench", [](uintptr_t x, uintptr_t xsq, int64_t n, int ld, uintptr_t rows, int m_, float gamma,
                                 uintptr_t out, int64_t out_ld, uintptr_t out_rows, int reps, uintptr_t stream) {
    py::gil_scoped_release rel;
    return kernels::rbf_rows_indexed_split_bench((const float*)x, (const float*)xsq, n, ld, (const int*)rows, m_,
                                                 gamma, (float*)out, out_ld, (const int*)out_rows, reps,
                                                 (void*)stream);
  }, "diagnostics: the split row GEMM alone, ms per launch");
  m.def("k_set_rows_stamps", [](uintptr_t p) { launch::set_rows_stamps((uint64_t*)p); },
        "diagnostics: the LDS-DMA rows kernel writes 8 u64 stamps per workgroup at p (0: off)");
  m.def("k_set_gram_stamps", [](uintptr_t p) { launch::set_gram_stamps((uint64_t*)p); },
        "diagnostics: the wide-wave Gram kernel writes 8 u64 stamps per workgroup at p (0: off)");
  m.def("k_set_split_gemm_variant", [](int v) { launch::set_split_gemm_variant(v); },
        "split STORE GEMM: 0 auto (4, or 3 when dp <= 128), 1 register-staged tile per workgroup, 3 LDS-DMA, 4 persistent LDS-DMA (tests / A/B)");
  m.def("k_split_gemm_variant", []() { return launch::split_gemm_variant(); });
  m.def("k_split_rows", [](uintptr_t x, int64_t rows, int dp, int ldx, uintptr_t out, uintptr_t shift,
                           uintptr_t stream) {
    launch::split_rows_f16((const float*)x, rows, dp, ldx, (void*)out, (int32_t*)shift, (hipStream_t)stream);
  });
  m.def("k_rbf_gram_split", [](uintptr_t a, uintptr_t asq, int64_t m_, uintptr_t b, uintptr_t bsq, int64_t n, int ld,
                               float gamma, uintptr_t out, int64_t out_ld, bool sym, uintptr_t stream,
                               float cold_tau) {
    kernels::rbf_gram_split((const float*)a, (const float*)asq, m_, (const float*)b, (const float*)bsq, n, ld, gamma,
                            (float*)out, out_ld, sym, (void*)stream, cold_tau);
  }, py::arg("a"), py::arg("asq"), py::arg("m"), py::arg("b"), py::arg("bsq"), py::arg("n"), py::arg("ld"),
     py::arg("gamma"), py::arg("out"), py::arg("out_ld"), py::arg("sym"), py::arg("stream"), py::arg("cold_tau") = 0.f);
  m.def("split_cold_consts", [](float gamma, float tau) {
    float c0 = 0.f, c1 = 0.f;
    launch::split_cold_consts(gamma, tau, &c0, &c1);
    return py::make_tuple(c0, c1);
  }, "the adaptive Gram's element rule constants (c0, c1): cold iff R_i + R_j <= c1 and t1 <= c0 - (R_i + R_j)");
  m.def("k_gram_adapt_last", []() { return kernels::gram_adapt_last(); },
        "(one-product tiles, hot tiles) of the calling thread's last adaptive split Gram, or (-1, -1)");
  m.def("k_fused_select", [](uintptr_t f, uintptr_t alpha, uintptr_t y, int64_t n, float C, int rows, uintptr_t out,
                             uintptr_t stream) {
    kernels::fused_select((const float*)f, (const float*)alpha, (const float*)y, n, C, rows, (uint64_t*)out,
                          (void*)stream);
  });
  // working-set kernels on crafted state (ws_kernel_entry.hip)
  using U64 = py::array_t<uint64_t, py::array::c_style | py::array::forcecast>;
  using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
  auto vi = [](const I32& a) { return std::vector<int32_t>(a.data(), a.data() + a.size()); };
  m.def("k_ws_merge_multi", [vi](const U64& cand, int G, int blocks, int p_act, int q_max, int n_new, float eps,
                                 const I32& prev, int64_t iter, int64_t max_iter) {
    const auto r = kernels::ws_merge_multi_probe(std::vector<uint64_t>(cand.data(), cand.data() + cand.size()), G,
                                                 blocks, p_act, q_max, n_new, eps, vi(prev), iter, max_iter);
    py::dict d;
    d["uidx"] = r.uidx;
    d["idx"] = r.idx;
    d["qb"] = r.qb;
    d["b_hi"] = r.b_hi;
    d["b_lo"] = r.b_lo;
    d["done"] = r.done;
    d["p_round"] = r.p_round;
    return d;
  });
  m.def("k_ws_solve", [vi](const F32& K, const F32& f, const F32& alpha, const F32& y, const I32& qb, int q_max,
                           int blocks, int p_round, float C, int clip, float eps, float rel, float eps_floor, float tau,
                           float b_hi, float b_lo, int inner_max, int64_t iter0, int64_t max_iter, int wss) {
    const auto r = kernels::ws_solve_probe(from_np(K), from_np(f), from_np(alpha), from_np(y), vi(qb), q_max, blocks,
                                           p_round, C, clip, eps, rel, eps_floor, tau, b_hi, b_lo, inner_max, iter0,
                                           max_iter, wss);
    py::dict d;
    d["alpha"] = to_np(r.alpha);
    d["steps"] = r.steps;
    d["apply_idx"] = r.apply_idx;
    d["apply_coef"] = to_np(r.apply_coef);
    d["nab"] = r.nab;
    d["iter"] = r.iter;
    d["outer"] = r.outer;
    d["done"] = r.done;
    d["p_act"] = r.p_act;
    d["p1_round"] = r.p1_round;
    return d;
  });
  m.def("k_ws_select", [vi](const F32& gram, int64_t L, int64_t ldg, const F32& f, const F32& alpha, const F32& y,
                            const F32& dalpha, const I32& lines, const F32& coef, const I32& nab, int blocks,
                            int p_round, int p_act, int q_max, float C, int64_t outer, int ks, int reps, bool wide) {
    const auto r = kernels::ws_select_probe(from_np(gram), L, ldg, from_np(f), from_np(alpha), from_np(y),
                                            from_np(dalpha), vi(lines), from_np(coef), vi(nab), blocks, p_round, p_act,
                                            q_max, C, outer, ks, reps, wide);
    py::dict d;
    d["f"] = to_np(r.f);
    d["alpha"] = to_np(r.alpha);
    d["dalpha"] = to_np(r.dalpha);
    d["dfs"] = to_np(r.dfs);
    d["part"] = r.part;
    d["cand"] = r.cand;
    d["G"] = r.G;
    d["rpt"] = r.rpt;
    d["p1G"] = r.p1G;
    d["t"] = r.t;
    d["pass1_us"] = r.pass1_us;
    d["p_act"] = r.p_act;
    d["n_damped"] = r.n_damped;
    d["p1_round"] = r.p1_round;
    d["nonfinite"] = r.nonfinite;
    return d;
  }, py::arg("gram"), py::arg("L"), py::arg("ldg"), py::arg("f"), py::arg("alpha"), py::arg("y"), py::arg("dalpha"),
        py::arg("lines"), py::arg("coef"), py::arg("nab"), py::arg("blocks"), py::arg("p_round"), py::arg("p_act"),
        py::arg("q_max"), py::arg("C"), py::arg("outer"), py::arg("ks") = 0, py::arg("reps") = 0,
        py::arg("wide") = false);
  m.def("production_line_cap", &production_line_cap, py::arg("cache_lines"), py::arg("ws_size"),
        py::arg("engines") = 0, "-s N on the engines a setup may choose (device_state.hpp)");
  m.def("ws_cache_min_lines", &ws_cache_min_lines, py::arg("ws_size"));
  m.def("make_key", [](float f, uint32_t idx) { return make_key(f, idx); });
  m.def("key_value", [](uint64_t k) { return key_value(k); });
  m.def("key_index", [](uint64_t k) { return key_index(k); });
  m.def("pad_features", &pad_features);
  m.def("shard_of", [](int64_t n, int rank, int world) {
    Shard s = shard_of(n, rank, world);
    return py::make_tuple(s.offset, s.size);
  });
  m.def("k_stream_read", [](uintptr_t x, int64_t bytes, uintptr_t out, int blocks, uintptr_t stream) {
    kernels::stream_read((const void*)x, bytes, (float*)out, blocks, (void*)stream);
  });
  m.def("launch_floor_us", &launch::launch_floor_us, py::arg("blocks") = 256, py::arg("threads") = 256,
        py::arg("chain") = 64, py::arg("reps") = 50, py::call_guard<py::gil_scoped_release>());
  m.def("device_count", &device_count);
  m.def("device_name", &device_name);
  m.attr("NQ") = 16;
  m.attr("STEP_ROWS") = 128;
}
