// SolverParams <-> flat JSON object, so a run summary (--metrics-json,
// bench.py) records every knob that selected its engine and geometry, and
// `svmTrain --params-json RUN.json` reruns with exactly those settings.
#pragma once

#include <cctype>
#include <cstdio>
#include <functional>
#include <map>
#include <string>
#include <type_traits>

#include "dpsvm/common.hpp"

namespace dpsvm {

namespace detail {
template <class F>
void for_each_param(SolverParams& p, F&& f) {
  f("C", p.C);
  f("gamma", p.gamma);
  f("eps", p.eps);
  f("max_iter", p.max_iter);
  int clip = (int)p.clip;
  f("clip", clip);
  p.clip = (ClipMode)clip;
  f("tau", p.tau);
  f("cache_lines", p.cache_lines);
  f("cache_mb", p.cache_mb);
  f("cache_frac", p.cache_frac);
  f("host_cache_lines", p.host_cache_lines);
  f("spec_rows", p.spec_rows);
  f("graph_block", p.graph_block);
  f("use_graph", p.use_graph);
  f("x_mode", p.x_mode);
  f("exchange", p.exchange);
  f("persist", p.persist);
  f("persist_block", p.persist_block);
  f("force_cache", p.force_cache);
  f("cache_engine", p.cache_engine);
  f("engines", p.engines);
  f("cache_groups", p.cache_groups);
  f("rows_per_group", p.rows_per_group);
  f("xch_poll_batch", p.xch_poll_batch);
  f("xch_sleep", p.xch_sleep);
  f("xch_stride", p.xch_stride);
  f("xch_mem", p.xch_mem);
  f("xch_timeout_s", p.xch_timeout_s);
  f("watchdog_s", p.watchdog_s);
  f("census_groups", p.census_groups);
  f("verify_ranks", p.verify_ranks);
  f("dp_policy", p.dp_policy);
  f("force_collectives", p.force_collectives);
  f("solver", p.solver);
  f("ws_size", p.ws_size);
  f("ws_new", p.ws_new);
  f("ws_rel", p.ws_rel);
  f("ws_blocks", p.ws_blocks);
  f("ws_inner", p.ws_inner);
  f("ws_wss", p.ws_wss);
  f("ws_t_halve", p.ws_t_halve);
  f("ws_clip_fallback", p.ws_clip_fallback);
  f("ws_block", p.ws_block);
  f("ws_recompute", p.ws_recompute);
  f("eta", p.eta);
  f("gram_precision", p.gram_precision);
  f("gram_adapt", p.gram_adapt);
  f("gram_cold_tau", p.gram_cold_tau);
}

inline std::string num(double v) {
  char b[64];
  snprintf(b, sizeof(b), "%.9g", v);
  return b;
}
}  // namespace detail

inline std::string params_json(const SolverParams& in) {
  SolverParams p = in;
  std::string s = "{";
  bool first = true;
  detail::for_each_param(p, [&](const char* k, auto& v) {
    if (!first) s += ", ";
    first = false;
    s += std::string("\"") + k + "\": " + detail::num((double)v);
  });
  return s + "}";
}

// Applies every "key": number pair of the first JSON object named "params"
// (or of the top-level object when there is none) to p; unknown keys are
// ignored.  Only the flat format written by params_json is understood.
inline void apply_params_json(const std::string& text, SolverParams& p) {
  size_t at = text.find("\"params\"");
  at = text.find('{', at == std::string::npos ? 0 : at);
  DPSVM_CHECK(at != std::string::npos, "params json: no object");
  const size_t end = text.find('}', at);
  DPSVM_CHECK(end != std::string::npos, "params json: unterminated object");
  std::map<std::string, double> kv;
  size_t i = at + 1;
  while (i < end) {
    const size_t q0 = text.find('"', i);
    if (q0 == std::string::npos || q0 >= end) break;
    const size_t q1 = text.find('"', q0 + 1);
    const size_t colon = text.find(':', q1);
    DPSVM_CHECK(q1 != std::string::npos && colon != std::string::npos && colon < end, "params json: bad key");
    const std::string key = text.substr(q0 + 1, q1 - q0 - 1);
    size_t v0 = colon + 1;
    while (v0 < end && isspace((unsigned char)text[v0])) ++v0;
    size_t v1 = v0;
    while (v1 < end && text[v1] != ',' && !isspace((unsigned char)text[v1])) ++v1;
    kv[key] = atof(text.substr(v0, v1 - v0).c_str());
    i = v1;
  }
  detail::for_each_param(p, [&](const char* k, auto& v) {
    auto it = kv.find(k);
    if (it != kv.end()) v = (std::remove_reference_t<decltype(v)>)it->second;
  });
}

}  // namespace dpsvm
