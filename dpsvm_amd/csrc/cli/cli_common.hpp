// Shared CLI plumbing: option parsing, data loading, metrics JSON.
// Flag surface follows the reference (svmTrainMain.cpp:22-136, seq.cpp:47-155,
// seq_test.cpp:36-124); new flags are long-only.
#pragma once

#include <getopt.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"
#include "dpsvm/params_io.hpp"
#include "dpsvm/solver.hpp"

namespace dpsvm {
namespace cli {

struct Options {
  int num_att = -1;
  int64_t num_ex = -1;
  std::string file, model;
  SolverParams p;
  bool gamma_set = false;
  bool legacy_gamma = false;  // integer 1/d like the reference (== 0 for d > 1)
  // new
  int gpus = 1;               // one GPU per rank (threads, ncclCommInitAll)
  int ranks = 0;              // simulated ranks on one device (ThreadComm)
  int device = 0;
  bool cpu = false;
  std::string synthetic;      // generator name instead of -f
  uint64_t seed = 0;
  std::string metrics_json;
  std::string resume;
  int precision = 9;
  bool legacy_model = false;  // write/read the seq format (no b line)
  bool quiet = false;
  bool skip_accuracy = false;
  int shrink = 0;             // one GPU, shrinking phases (solve_shrinking): 0 auto (shrink_auto), 1 off, 2 on
};

inline void usage_train(const char* prog, bool seq) {
  std::cerr << "   Command Line (" << prog << "):\n\n"
               "   -a/--num-att        :  [REQUIRED] The number of attributes /features\n"
               "   -x/--num-ex         :  [REQUIRED] The number of training examples\n"
               "   -f/--file-path      :  [REQUIRED] Path to the training file (or --synthetic)\n"
               "   -c/--cost           :  Parameter c of the SVM (default 1)\n"
               "   -g/--gamma          :  Parameter gamma of the radial basis function: exp(-gamma*|u-v|^2)\n"
               "                          (default: 1.0/num-att; --legacy-gamma: integer 1/num-att)\n"
               "   -e/--epsilon        :  Tolerance of termination criterion (default 0.001)\n"
               "   -n/--max-iter       :  Maximum number of iterations (default 150,000)\n"
               "   -m/--model          :  [REQUIRED] Path of model to be saved\n";
  if (!seq) std::cerr << "   -s/--cache-size     :  Size of cache (num cache lines; default: fill HBM)\n";
  std::cerr << "\n   MI355X extensions:\n"
               "   -p/--gpus N         :  ranks = GPUs of this node (RCCL over xGMI)\n"
               "   --ranks N           :  simulate N ranks on one device (in-process comm)\n"
               "   --cpu               :  CPU solver\n"
               "   --device N          :  GPU for a single-rank run\n"
               "   --synthetic NAME    :  mnist | mnist-parity | adult | covtype | blobs | uniform\n"
               "   --seed N            :  synthetic seed (default 0)\n"
               "   --clip MODE         :  independent (reference) | box (LIBSVM joint box)\n"
               "   --cache-mb MB       :  device cache budget\n"
               "   --x-mode MODE       :  auto | replicated | partitioned\n"
               "   --spec N            :  speculative kernel rows per X pass (LRU mode, default 14)\n"
               "   --host-cache-lines N:  pinned host spill tier for evicted kernel rows (LRU mode)\n"
               "   --graph-block N     :  SMO iterations per hipGraph (default 64); --no-graph\n"
               "   --persist MODE      :  engine: auto | off (one launch/iteration) | on (persistent; dense and cache mode)\n"
               "   --persist-block N   :  SMO iterations per persistent launch (default 2048)\n"
               "   --exchange MODE     :  per-iteration keys: auto | allreduce | peer (in-kernel, xGMI)\n"
               "   --dp MODE           :  data parallelism at world > 1: auto | shard | replicate\n"
               "   --force-cache       :  kernel-row cache mode even when the Gram fits\n"
               "   --cache-engine E    :  cache mode, one launch per iteration: fused | chain (--engines all)\n"
               "   --engines E         :  production (default) | all: also the quarantined pair-at-a-time cache /\n"
               "                         partitioned-X engines (tests, A/B probes; --host-cache-lines needs it)\n"
               "   --cache-groups N    :  cache mode workgroups per rank (default 256)\n"
               "   --rows-per-group N  :  rows per workgroup of the fused/persistent engines (multiple of 256)\n"
               "   --xch-poll-batch N --xch-sleep N --xch-stride N --xch-mem auto|uncached|coarse\n"
               "   --xch-timeout S     :  give-up bound of one in-kernel exchange poll (default 120)\n"
               "   --watchdog S        :  host bound on one block of iterations (default 0 = auto: 1800 s,\n"
               "                          adaptive to the block time with several ranks)\n"
               "   --census-groups N   :  residency census grid of the persistent engines (tests)\n"
               "   --no-verify-ranks   :  skip the cross-rank alpha digest (world > 1)\n"
               "   --solver S          :  auto (ws from 50k rows, else smo) | smo (pair-at-a-time engines) | ws (working-set rounds)\n"
               "   --ws-size N         :  working-set rows of the ws engine (<= 192, default 192)\n"
               "   --ws-new N --ws-rel R --ws-inner N --ws-block N :  ws engine round parameters\n"
               "   --ws-wss 1|2        :  sub-problem pair choice: 1 first order (reference), 2 second order\n"
               "   --ws-blocks P       :  up to P sub-problems per round on P workgroups (1..32, P x ws-size <= 3072;\n"
               "                          default 0 = auto:\n"
               "                          32 blocks of 96 rows from 50k rows, halved after every damped round)\n"
               "   --shrink[=auto|on|off] :  one GPU: LIBSVM-style shrinking (phases on the rows that can still\n"
               "                         violate; auto, the default: on when the whole Gram is not resident)\n"
               "   --eta x|gram        :  pair engines' K(hi, lo): from the X rows (default) | the resident Gram\n"
               "   --gram auto|f32|split :  Gram / kernel-row GEMMs: f32-input MFMA, or fp16 MFMA over hi/lo split\n"
               "                          operands (fp32 accuracy); auto = split for the ws engines\n"
               "   --gram-adapt auto|on|off : resident ws-dense Gram: one-product tiles where every value is provably\n"
               "                          within 2^-22 of the three-product one, the rest recomputed (auto: on when a\n"
               "                          row sample passes the bound)\n"
               "   --params-json PATH  :  solver parameters from a --metrics-json run summary\n"
               "   --checkpoint PATH --checkpoint-every N --resume PATH\n"
               "   --metrics-json PATH :  run summary\n"
               "   --log-every N       :  progress line every N iterations\n"
               "   --precision N       :  model-file significant digits (reference: 6; default 9)\n"
               "   --legacy-model      :  write the seq model format (no b line)\n"
               "   --skip-accuracy     :  do not compute the training accuracy\n";
  exit(-1);
}

inline Options parse_train(int argc, char** argv, bool seq) {
  Options o;
  enum {
    OPT_RANKS = 1000, OPT_CPU, OPT_DEVICE, OPT_SYN, OPT_SEED, OPT_CLIP, OPT_CMB, OPT_XMODE, OPT_SPEC,
    OPT_GB, OPT_NOGRAPH, OPT_CK, OPT_CKE, OPT_RESUME, OPT_METRICS, OPT_LOG, OPT_PREC, OPT_LEGM,
    OPT_LEGG, OPT_QUIET, OPT_SKIPACC, OPT_VERBOSE, OPT_HOSTC, OPT_PERSIST, OPT_PBLOCK, OPT_XCH,
    OPT_DP, OPT_FCACHE, OPT_CENG, OPT_CGROUPS, OPT_ROWS, OPT_XKB, OPT_XSLEEP, OPT_XSTRIDE, OPT_XMEM,
    OPT_XTMO, OPT_WDOG, OPT_CENSUS, OPT_NOVR, OPT_PJSON, OPT_SOLVER, OPT_WSSIZE, OPT_WSNEW, OPT_WSREL, OPT_WSBLOCKS,
    OPT_WSINNER, OPT_WSBLOCK, OPT_ETA, OPT_WSWSS, OPT_GRAM, OPT_SHRINK, OPT_ENGINES, OPT_GRAM_ADAPT
  };
  static struct option longopts[] = {
      {"num-att", required_argument, 0, 'a'},     {"num-ex", required_argument, 0, 'x'},
      {"cost", required_argument, 0, 'c'},        {"gamma", required_argument, 0, 'g'},
      {"file-path", required_argument, 0, 'f'},   {"epsilon", required_argument, 0, 'e'},
      {"max-iter", required_argument, 0, 'n'},    {"model", required_argument, 0, 'm'},
      {"cache-size", required_argument, 0, 's'},  {"gpus", required_argument, 0, 'p'},
      {"ranks", required_argument, 0, OPT_RANKS}, {"cpu", no_argument, 0, OPT_CPU},
      {"device", required_argument, 0, OPT_DEVICE}, {"synthetic", required_argument, 0, OPT_SYN},
      {"seed", required_argument, 0, OPT_SEED},   {"clip", required_argument, 0, OPT_CLIP},
      {"cache-mb", required_argument, 0, OPT_CMB}, {"x-mode", required_argument, 0, OPT_XMODE},
      {"spec", required_argument, 0, OPT_SPEC},   {"graph-block", required_argument, 0, OPT_GB},
      {"host-cache-lines", required_argument, 0, OPT_HOSTC},
      {"no-graph", no_argument, 0, OPT_NOGRAPH},  {"checkpoint", required_argument, 0, OPT_CK},
      {"checkpoint-every", required_argument, 0, OPT_CKE}, {"resume", required_argument, 0, OPT_RESUME},
      {"metrics-json", required_argument, 0, OPT_METRICS}, {"log-every", required_argument, 0, OPT_LOG},
      {"precision", required_argument, 0, OPT_PREC}, {"legacy-model", no_argument, 0, OPT_LEGM},
      {"legacy-gamma", no_argument, 0, OPT_LEGG}, {"quiet", no_argument, 0, OPT_QUIET},
      {"skip-accuracy", no_argument, 0, OPT_SKIPACC}, {"verbose", no_argument, 0, OPT_VERBOSE},
      {"persist", required_argument, 0, OPT_PERSIST}, {"persist-block", required_argument, 0, OPT_PBLOCK},
      {"exchange", required_argument, 0, OPT_XCH},
      {"dp", required_argument, 0, OPT_DP},       {"force-cache", no_argument, 0, OPT_FCACHE},
      {"cache-engine", required_argument, 0, OPT_CENG}, {"cache-groups", required_argument, 0, OPT_CGROUPS},
      {"rows-per-group", required_argument, 0, OPT_ROWS}, {"xch-poll-batch", required_argument, 0, OPT_XKB},
      {"xch-sleep", required_argument, 0, OPT_XSLEEP}, {"xch-stride", required_argument, 0, OPT_XSTRIDE},
      {"xch-mem", required_argument, 0, OPT_XMEM}, {"xch-timeout", required_argument, 0, OPT_XTMO},
      {"watchdog", required_argument, 0, OPT_WDOG}, {"census-groups", required_argument, 0, OPT_CENSUS},
      {"no-verify-ranks", no_argument, 0, OPT_NOVR}, {"params-json", required_argument, 0, OPT_PJSON},
      {"solver", required_argument, 0, OPT_SOLVER}, {"ws-size", required_argument, 0, OPT_WSSIZE},
      {"ws-new", required_argument, 0, OPT_WSNEW}, {"eta", required_argument, 0, OPT_ETA}, {"ws-rel", required_argument, 0, OPT_WSREL},
      {"ws-blocks", required_argument, 0, OPT_WSBLOCKS},
      {"ws-inner", required_argument, 0, OPT_WSINNER}, {"ws-block", required_argument, 0, OPT_WSBLOCK},
      {"ws-wss", required_argument, 0, OPT_WSWSS}, {"gram", required_argument, 0, OPT_GRAM},
      {"gram-adapt", required_argument, 0, OPT_GRAM_ADAPT},
      {"shrink", optional_argument, 0, OPT_SHRINK}, {"engines", required_argument, 0, OPT_ENGINES},
      {0, 0, 0, 0}};
  while (true) {
    int idx = 0;
    int c = getopt_long(argc, argv, seq ? "a:x:c:g:f:e:n:m:p:" : "a:x:c:g:f:e:n:m:s:p:", longopts, &idx);
    if (c == -1) break;
    switch (c) {
      case 'a': o.num_att = atoi(optarg); break;
      case 'x': o.num_ex = atoll(optarg); break;
      case 'c': o.p.C = (float)atof(optarg); break;
      case 'g': o.p.gamma = (float)atof(optarg); o.gamma_set = true; break;
      case 'f': o.file = optarg; break;
      case 'e': o.p.eps = (float)atof(optarg); break;
      case 'n': o.p.max_iter = atoll(optarg); break;
      case 'm': o.model = optarg; break;
      case 's': o.p.cache_lines = atoll(optarg); break;
      case 'p': o.gpus = atoi(optarg); break;
      case OPT_RANKS: o.ranks = atoi(optarg); break;
      case OPT_CPU: o.cpu = true; break;
      case OPT_DEVICE: o.device = atoi(optarg); break;
      case OPT_SYN: o.synthetic = optarg; break;
      case OPT_SEED: o.seed = strtoull(optarg, nullptr, 10); break;
      case OPT_CLIP:
        if (std::string(optarg) == "box") o.p.clip = ClipMode::Box;
        else if (std::string(optarg) == "independent") o.p.clip = ClipMode::Independent;
        else usage_train(argv[0], seq);
        break;
      case OPT_CMB: o.p.cache_mb = atof(optarg); break;
      case OPT_XMODE: {
        std::string v = optarg;
        o.p.x_mode = v == "replicated" ? 1 : v == "partitioned" ? 2 : 0;
        break;
      }
      case OPT_SPEC: o.p.spec_rows = atoi(optarg); break;
      case OPT_HOSTC: o.p.host_cache_lines = atoll(optarg); break;
      case OPT_GB: o.p.graph_block = atoi(optarg); break;
      case OPT_NOGRAPH: o.p.use_graph = false; break;
      case OPT_CK: o.p.checkpoint_path = optarg; break;
      case OPT_CKE: o.p.checkpoint_every = atoll(optarg); break;
      case OPT_RESUME: o.resume = optarg; break;
      case OPT_METRICS: o.metrics_json = optarg; break;
      case OPT_LOG: o.p.log_every = atoi(optarg); break;
      case OPT_PREC: o.precision = atoi(optarg); break;
      case OPT_LEGM: o.legacy_model = true; break;
      case OPT_LEGG: o.legacy_gamma = true; break;
      case OPT_QUIET: o.quiet = true; break;
      case OPT_SKIPACC: o.skip_accuracy = true; break;
      case OPT_SHRINK: {
        const std::string v = optarg ? optarg : "on";
        if (v != "auto" && v != "off" && v != "on") usage_train(argv[0], seq);
        o.shrink = v == "on" ? 2 : v == "off" ? 1 : 0;
        break;
      }
      case OPT_VERBOSE: o.p.verbose = true; break;
      case OPT_PERSIST: {
        const std::string v = optarg;
        if (v != "auto" && v != "off" && v != "on") usage_train(argv[0], seq);
        o.p.persist = v == "on" ? 2 : v == "off" ? 1 : 0;
        break;
      }
      case OPT_PBLOCK: o.p.persist_block = atoi(optarg); break;
      case OPT_XCH: {
        const std::string v = optarg;
        if (v != "auto" && v != "allreduce" && v != "peer") usage_train(argv[0], seq);
        o.p.exchange = v == "peer" ? 2 : v == "allreduce" ? 1 : 0;
        break;
      }
      case OPT_DP: {
        const std::string v = optarg;
        if (v != "auto" && v != "shard" && v != "replicate") usage_train(argv[0], seq);
        o.p.dp_policy = v == "shard" ? 1 : v == "replicate" ? 2 : 0;
        break;
      }
      case OPT_FCACHE: o.p.force_cache = true; break;
      case OPT_CENG: {
        const std::string v = optarg;
        if (v != "fused" && v != "chain") usage_train(argv[0], seq);
        o.p.cache_engine = v == "chain" ? 1 : 0;
        break;
      }
      case OPT_ENGINES: {
        const std::string v = optarg;
        if (v != "production" && v != "all") usage_train(argv[0], seq);
        o.p.engines = v == "all" ? 1 : 0;
        break;
      }
      case OPT_CGROUPS: o.p.cache_groups = atoi(optarg); break;
      case OPT_ROWS: o.p.rows_per_group = atoi(optarg); break;
      case OPT_XKB: o.p.xch_poll_batch = atoi(optarg); break;
      case OPT_XSLEEP: o.p.xch_sleep = atoi(optarg); break;
      case OPT_XSTRIDE: o.p.xch_stride = atoi(optarg); break;
      case OPT_XMEM: {
        const std::string v = optarg;
        if (v != "auto" && v != "uncached" && v != "coarse") usage_train(argv[0], seq);
        o.p.xch_mem = v == "uncached" ? 1 : v == "coarse" ? 2 : 0;
        break;
      }
      case OPT_XTMO: o.p.xch_timeout_s = atof(optarg); break;
      case OPT_WDOG: o.p.watchdog_s = atof(optarg); break;
      case OPT_CENSUS: o.p.census_groups = atoi(optarg); break;
      case OPT_NOVR: o.p.verify_ranks = false; break;
      case OPT_SOLVER: {
        const std::string v = optarg;
        if (v != "auto" && v != "smo" && v != "ws") usage_train(argv[0], seq);
        o.p.solver = v == "ws" ? 2 : v == "smo" ? 1 : 0;
        break;
      }
      case OPT_WSSIZE: o.p.ws_size = atoi(optarg); break;
      case OPT_WSNEW: o.p.ws_new = atoi(optarg); break;
      case OPT_WSREL: o.p.ws_rel = (float)atof(optarg); break;
      case OPT_WSBLOCKS: o.p.ws_blocks = atoi(optarg); break;
      case OPT_WSINNER: o.p.ws_inner = atoi(optarg); break;
      case OPT_WSWSS: o.p.ws_wss = atoi(optarg); break;
      case OPT_WSBLOCK: o.p.ws_block = atoi(optarg); break;
      case OPT_ETA: {
        const std::string v = optarg;
        if (v != "x" && v != "gram") usage_train(argv[0], seq);
        o.p.eta = v == "gram" ? 1 : 0;
        break;
      }
      case OPT_GRAM_ADAPT: {
        const std::string v = optarg;
        if (v != "auto" && v != "on" && v != "off") usage_train(argv[0], seq);
        o.p.gram_adapt = v == "on" ? 1 : v == "off" ? 2 : 0;
        break;
      }
      case OPT_GRAM: {
        const std::string v = optarg;
        if (v != "auto" && v != "f32" && v != "split") usage_train(argv[0], seq);
        o.p.gram_precision = v == "split" ? 2 : v == "f32" ? 1 : 0;
        break;
      }
      case OPT_PJSON: {
        FILE* fp = fopen(optarg, "r");
        if (!fp) {
          std::cerr << "cannot read " << optarg << "\n";
          usage_train(argv[0], seq);
        }
        std::string text;
        char buf[4096];
        size_t k;
        while ((k = fread(buf, 1, sizeof(buf), fp)) > 0) text.append(buf, k);
        fclose(fp);
        apply_params_json(text, o.p);
        o.gamma_set = o.p.gamma >= 0;
        break;
      }
      default:
        std::cerr << "\nERROR: Unknown option: -" << (char)c << "\n";
        usage_train(argv[0], seq);
    }
  }
  if ((o.file.empty() && o.synthetic.empty()) || o.model.empty()) {
    std::cerr << "Enter a valid file name\n";
    usage_train(argv[0], seq);
  }
  if (o.num_att <= 0 || o.num_ex <= 0) {
    std::cerr << "Missing a required parameter, or invalid parameter\n";
    usage_train(argv[0], seq);
  }
  if (!o.gamma_set || o.p.gamma < 0) {
    // reference: `1 / num_attributes` in int arithmetic
    o.p.gamma = o.legacy_gamma ? (float)(1 / o.num_att) : 1.0f / (float)o.num_att;
  }
  if (o.p.cache_lines == 1) o.p.cache_lines = 2;  // two lines in flight
  return o;
}

inline Dataset load_data(const Options& o, int64_t row0 = 0, int64_t rows = -1) {
  if (!o.synthetic.empty())
    return make_synthetic(synth_from_name(o.synthetic), o.num_ex, o.num_att, o.seed, row0, rows);
  if (rows >= 0) return read_csv_rows(o.file, row0, rows, o.num_att);
  return read_csv(o.file, o.num_ex, o.num_att);
}

inline std::string json_escape(const std::string& s) {
  std::string r;
  for (char c : s) {
    if (c == '"' || c == '\\') r += '\\';
    r += c;
  }
  return r;
}

// per-phase wall times and the engine actually used
struct RunExtras {
  double t_load = 0.0, t_accuracy = 0.0, t_model_write = 0.0;
  std::string engine = "cpu", exchange = "none";
  GpuSetupInfo setup;  // engine, geometry, exchange, residency (GPU runs)
};

inline void write_metrics(const std::string& path, const Options& o, const SolveResult& r, int64_t n, int d,
                          int64_t nsv, double acc, const std::string& backend, const std::string& device,
                          const RunExtras& x) {
  FILE* fp = fopen(path.c_str(), "w");
  if (!fp) {
    std::cerr << "cannot write metrics " << path << "\n";
    return;
  }
  fprintf(fp,
          "{\"backend\": \"%s\", \"device\": \"%s\", \"world\": %d, \"n\": %lld, \"d\": %d, \"C\": %g, "
          "\"gamma\": %g, \"eps\": %g, \"clip\": \"%s\", \"iterations\": %lld, \"status\": %d, "
          "\"converged\": %s, \"b\": %.9g, \"b_hi\": %.9g, \"b_lo\": %.9g, \"n_sv\": %lld, "
          "\"train_accuracy\": %.9g, \"t_load_s\": %.6f, \"t_setup_s\": %.6f, \"t_solve_s\": %.6f, "
          "\"t_gram_s\": %.6f, \"t_accuracy_s\": %.6f, \"t_model_write_s\": %.6f, \"engine\": \"%s\", "
          "\"exchange\": \"%s\", "
          "\"iters_per_s\": %.3f, \"cache_lines\": %lld, \"cache_hits\": %lld, \"cache_misses\": %lld, "
          "\"rows_computed\": %lld, \"x_passes\": %lld, \"spec_rows\": %lld, \"data\": \"%s\", "
          "\"exchange_mem\": \"%s\", \"dp_policy\": \"%s\", \"rows_per_group\": %lld, \"groups\": %lld, "
          "\"poll_batch\": %d, \"cus\": %d, \"blocks_per_cu\": %d, \"census\": \"%s\", \"engine_note\": \"%s\", \"cache_note\": \"%s\", "
          "\"rounds\": %lld, \"ws_blocks\": %d, \"ws_blocks_end\": %d, \"ws_one_block_from_round\": %lld, "
          "\"ws_damped_rounds\": %lld, \"gram\": \"%s\", \"params\": %s}\n",
          backend.c_str(), json_escape(device).c_str(), r.world, (long long)n, d, o.p.C, o.p.gamma, o.p.eps,
          o.p.clip == ClipMode::Box ? "box" : "independent", (long long)r.iters, r.status,
          r.converged() ? "true" : "false", r.b, r.b_hi, r.b_lo, (long long)nsv, acc, x.t_load, r.t_setup,
          r.t_solve, r.t_gram, x.t_accuracy, x.t_model_write, x.engine.c_str(), x.exchange.c_str(),
          r.t_solve > 0 ? r.iters / r.t_solve : 0.0, (long long)r.cache_lines,
          (long long)r.cache_hits, (long long)r.cache_misses, (long long)r.rows_computed,
          (long long)r.x_passes, (long long)r.spec_rows,
          json_escape(o.synthetic.empty() ? o.file : "synthetic:" + o.synthetic).c_str(),
          x.setup.exchange_mem.c_str(), x.setup.dp_policy.c_str(), (long long)x.setup.rows_per_group,
          (long long)x.setup.groups, x.setup.poll_batch, x.setup.cus, x.setup.blocks_per_cu,
          x.setup.census.c_str(), json_escape(x.setup.engine_note).c_str(),
          json_escape(x.setup.cache_note).c_str(), (long long)r.outer, r.ws_blocks,
          r.ws_blocks_end, (long long)r.ws_p1_round, (long long)r.ws_damped, x.setup.gram.c_str(),
          params_json(o.p).c_str());
  fclose(fp);
}

inline void print_outcome(const SolveResult& r, float eps) {
  std::cout << "TOTAL TIME TAKEN in seconds: " << r.t_solve << "\n";
  if (r.status == 2 || (r.status != 1 && gap_open(r.b_hi, r.b_lo, eps))) {
    std::cout << "Could not converge in " << r.iters << " iterations. SVM training has been stopped\n";
  } else {
    std::cout << "Converged at iteration number: " << r.iters << "\n";
  }
  if (r.outer > 0)  // working-set engines: "iterations" are pair steps inside the rounds' sub-problems
    std::cout << "Working-set rounds: " << r.outer << " (pair steps counted as iterations; blocks per round "
              << r.ws_blocks << (r.ws_blocks_end != r.ws_blocks ? " -> " + std::to_string(r.ws_blocks_end) : "")
              << ")\n";
  if (r.status == 4) std::cout << "WARNING: non-finite b_hi/b_lo encountered; training stopped\n";
  if (r.outer > 0 && r.status == 2) {
    // a capped, unconverged working-set solve is not the reference's iterate at that cap
    std::cerr << "warning: stopped at the iteration cap with gap " << (r.b_lo - r.b_hi) << " > 2 eps: the "
              << "working-set rounds' unconverged model differs from the reference's pair-at-a-time iterate at the "
              << "same cap; raise --max-iter (-n) to converge, or --solver smo for the reference's trajectory "
              << "(with --engines all when the Gram is not resident)\n";
  }
  std::cout << "b: " << r.b << "\n";
}

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace cli
}  // namespace dpsvm
