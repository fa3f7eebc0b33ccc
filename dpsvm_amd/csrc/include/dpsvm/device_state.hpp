// Device-resident SMO state shared by the HIP kernels and the host driver.
//
// One SMO iteration on a rank is a short, host-free kernel chain
//     [smo_rows]  -> smo_step -> [collective] -> smo_finalize
// and blocks of iterations are captured into a hipGraph.  The host only polls
// a status record in pinned host-mapped memory (SURVEY §7.1 design 1).
// Reference per-iteration path for contrast: svmTrainMain.cpp:235-310 with >=7
// blocking host<->device round trips (SURVEY §3.1 hot-loop cost structure).
#pragma once

#include <cstdint>

namespace dpsvm {

constexpr int kNQ = 16;             // kernel rows per X pass (MFMA 16x16x4 N width)
constexpr int kStepRows = 128;      // rows per step/rows workgroup
constexpr int kStepThreads = 256;   // 4 waves
constexpr int kFinThreads = 1024;   // finalize: one workgroup, 16 waves
constexpr int kRowsKC = 1008;       // k-chunk of query vectors staged in LDS (16 x 1012 floats < 64 KiB)

enum CacheMode : int32_t {
  kCacheDense = 0,  // whole Gram shard resident: line i == global row i
  kCacheLRU = 1,    // CLOCK-replaced lines filled on demand by smo_rows (+ host tier)
};

// smo_rows per-query operation
enum RowOp : int32_t {
  kOpCompute = 0,   // MFMA X pass
  kOpFetch = 1,     // copy from the pinned host tier (zero-copy PCIe loads)
};

enum DoneCode : int32_t {
  kRunning = 0,
  kConverged = 1,
  kMaxIter = 2,
  kNoPair = 3,
  kNonFinite = 4,
  kCommFail = 5,   // peer exchange gave up waiting (a rank stopped or diverged)
};

// Iteration engines of the device solver (GpuSetupInfo::iteration names them).
enum class EngineKind : int32_t {
  PersistDense = 0,  // Gram resident, persistent kernel, in-kernel key exchange
  FusedDense = 1,    // Gram resident, one launch per iteration (hipGraph blocks)
  PersistCache = 2,  // kernel-row cache, persistent kernel, private cache metadata
  FusedCache = 3,    // kernel-row cache, one launch per iteration (+ host spill tier)
  Chain = 4,         // rows / step / finalize kernels + collective (partitioned X fallback)
  WsDense = 5,       // Gram resident, working-set rounds (sub-problem in LDS, ws_*.hip)
  WsCache = 6,       // kernel-row cache, working-set rounds (the set's missing rows by one MFMA GEMM)
};
inline const char* engine_name(EngineKind k) {
  switch (k) {
    case EngineKind::WsDense: return "ws-dense";
    case EngineKind::WsCache: return "ws-cache";
    case EngineKind::PersistDense: return "persistent-dense";
    case EngineKind::FusedDense: return "fused-dense";
    case EngineKind::PersistCache: return "persistent-cache";
    case EngineKind::FusedCache: return "fused-cache";
    default: return "chain";
  }
}

// What gpu_setup established before choosing an engine (every flag already
// agreed across ranks).
struct EngineFacts {
  bool ws_dense = false;          // working-set rounds wanted and supported, Gram resident
  bool ws_cache = false;          // ... Gram not resident, cache holds >= 2 q + 512 lines, no host tier
  bool dense = false;             // Gram resident
  bool cache_replicated = false;  // Gram not resident, X replicated (the pair cache engines' X pass)
  bool persistent = false;        // in-kernel exchange set up and its candidate's geometry fits
  bool quarantine = false;        // engines=all: the quarantined rows may match
};

// The engine choice: first matching row wins.  `use` is the path that reaches
// the row (docs/DESIGN.md §2 lists the same table).  A persistent row whose
// grid then fails the co-residency census drops to the fused row below it.
// Production: the four rows of kEngineTable.  The pair-at-a-time engines for a
// Gram that is not resident or an X that is partitioned (kQuarantineTable) are
// reached only with SolverParams::engines = 1 (tests, A/B probes): with 288 GB
// per GPU the Gram of the pair engines' problems (< 50k rows) is resident, and
// ws-cache is 5-10x faster on the problems whose Gram is not.
struct EngineRule {
  EngineKind kind;
  bool (*when)(const EngineFacts&);
  const char* use;
};
inline constexpr EngineRule kEngineTable[] = {
    {EngineKind::WsDense, [](const EngineFacts& f) { return f.ws_dense; },
     "default from 50k rows (solver auto) or solver=ws, Gram resident"},
    {EngineKind::WsCache, [](const EngineFacts& f) { return f.ws_cache; },
     "default from 50k rows (solver auto) or solver=ws, Gram not resident"},
    {EngineKind::PersistDense, [](const EngineFacts& f) { return f.dense && f.persistent; },
     "default below 50k rows (solver auto) or solver=smo: the reference's trajectory"},
    {EngineKind::FusedDense, [](const EngineFacts& f) { return f.dense; },
     "fallback of persistent-dense (census or exchange self-test failed, persist=off, forced collectives)"},
};
inline constexpr EngineRule kQuarantineTable[] = {
    {EngineKind::PersistCache, [](const EngineFacts& f) { return f.cache_replicated && f.persistent; },
     "engines=all: pair-at-a-time in cache mode (solver=smo, or a cache too small for ws-cache)"},
    {EngineKind::FusedCache, [](const EngineFacts& f) { return f.cache_replicated; },
     "engines=all: fallback of persistent-cache; host spill tier (host_cache_lines); persist=off"},
    {EngineKind::Chain, [](const EngineFacts&) { return true; },
     "engines=all: pair-at-a-time with X partitioned (x_mode=partitioned, solver=smo); cache_engine=chain"},
};
// false: no production row matches and the quarantined rows are off (the
// setup reports why: the configuration needs engines=all)
inline bool choose_engine(const EngineFacts& f, EngineKind* out) {
  for (const EngineRule& r : kEngineTable)
    if (r.when(f)) return *out = r.kind, true;
  if (f.quarantine)
    for (const EngineRule& r : kQuarantineTable)
      if (r.when(f)) return *out = r.kind, true;
  return false;
}

// Rows a one-block working-set round replaces (ws_new = 0: auto): all q with
// >= 128 padded features, 3/4 of the set (the newest quarter kept) below.
// Measured with full replacement: synthetic-2m 2M x 1024 47.9 -> 44.4 s,
// mnist-parity 0.0226 -> 0.0219 s, adult (solver=ws) 0.207 -> 0.191 s;
// covtype (54 features, strongly coupled at C = 2048) stalls without retained
// rows and keeps 3/4 (profiles/r4_ws_new_ab.txt, r4_ws_param_sweep_1gpu.txt).
// A function of the shape only, so ws-dense and ws-cache (and every rank) take
// the same sets: the cache engine stays bit-identical to the dense one.
inline int ws_new_auto(int ws_new, int q, int dp) {
  const int n = ws_new > 0 ? (ws_new < q ? ws_new : q) : (dp >= 128 ? q : 3 * q / 4);
  return n > 2 ? n : 2;
}

// Written by smo_finalize, read by the next iteration's kernels.
struct alignas(16) SmoCtrl {
  int32_t iter;        // SMO updates applied so far
  int32_t done;        // DoneCode of the last finalize (0 = running)
  int32_t final_applied;  // 1 once the step after `done` applied the last f update
  int32_t nq;          // rows smo_rows must fill this iteration (compute or fetch)
  int32_t i_hi, i_lo;
  int32_t line_hi, line_lo;  // lines holding K(hi,.) / K(lo,.) for the pending update
  float c_hi, c_lo;    // (alpha_new - alpha_old) * y, pending f-update coefficients
  float b_hi, b_lo;    // selection values of the last finalize
  int32_t n_compute;   // queries with op kOpCompute (0: no X pass this iteration)
  int32_t n_spill;     // queries whose victim line must first be copied to the host tier
  int32_t q_idx[kNQ];  // global rows to compute
  int32_t q_line[kNQ]; // destination lines
  int32_t q_op[kNQ];   // RowOp
  int32_t q_hsrc[kNQ];   // kOpFetch: host-tier line to copy from
  int32_t q_hspill[kNQ]; // >= 0: host-tier line receiving the victim's old content
  float q_sq[kNQ];     // |x_q|^2
  const float* q_ptr[kNQ];  // query vectors (device X row, or a gathered record row)
  // CLOCK hands (device lines, host-tier FIFO)
  int32_t hand, hhand, pad0, pad1;
  // statistics
  int64_t hits, misses, rows_computed, x_passes, spec_rows, host_hits, spills;
};

// Host-mapped status record (pinned, written by finalize thread 0).
struct alignas(16) SmoStatus {
  int64_t iter;
  int32_t done;
  int32_t seq;
  float b_hi, b_lo;
  int64_t hits, misses, rows_computed, x_passes, spec_rows, host_hits, spills;
  int64_t outer;  // working-set engine: rounds (selection + sub-problem solve) so far
  // multi-block working-set rounds: rounds completed when the adaptive block
  // count reached 1 (0: not yet; identical on every rank), the current count,
  // damped rounds so far
  int64_t ws_p1_round;
  int32_t ws_p, ws_damped;
};

// Partitioned-X candidate record: one per rank, all-gathered each iteration.
// Row payload follows the header: x_hi[dp], x_lo[dp].
struct alignas(16) CandRecord {
  uint64_t key_hi, key_lo;
};

// Dense-mode fused iteration (smo_fused): kernel t derives pair t from the
// partials of kernel t-1 redundantly in every workgroup, so one launch (+ one
// collective when world > 1) is one SMO iteration.  The record carries pair
// t's new alphas; they are committed to the alpha array by kernel t+1 (lazy
// commit avoids a read/write race between workgroups of kernel t).
struct alignas(16) FusedRec {
  int32_t i_hi, i_lo;   // pair updated by the producing kernel (-1: none)
  float a_hi, a_lo;     // its new alphas (a_hi wins when i_hi == i_lo)
  int32_t iter, done;   // SMO iterations completed; DoneCode
  float b_hi, b_lo;
};
// Cache-mode fused iteration (smo_fused_lru): as FusedRec plus the cache
// decisions of the producing kernel, committed lazily by workgroup 0 of the
// next launch while every reader applies them as corrections.
struct alignas(16) FusedCacheRec {
  int32_t i_hi, i_lo;
  float a_hi, a_lo;
  int32_t iter, done;
  float b_hi, b_lo;
  int32_t n_new;          // lines (re)assigned by the producing kernel
  int32_t hand0, span;    // CLOCK window scanned: ref bits cleared except new/hit lines
  int32_t hand;           // CLOCK hand after the scan
  int32_t hit_line[2];    // lines hit by the producing kernel (ref set)
  int32_t hhand, pad0;
  int32_t line[kNQ];      // assigned lines
  int32_t key[kNQ];       // their new rows
  int32_t old[kNQ];       // evicted rows (-1: none)
  int32_t hline[kNQ];     // host-tier line receiving old[q] (-1: no spill)
  int32_t hold[kNQ];      // row evicted from that host line (-1)
  int64_t hits, misses, rows_computed, x_passes, spec_rows, host_hits, spills;
};

constexpr int kFusedThreads = 256;
constexpr int kStatusEvery = 32;  // host-mapped status refresh period (iterations)

struct SmoArgs {
  const float* x;        // device X rows [x_rows][dp] (zero padded)
  const float* xsq;      // [n] global |x|^2
  const float* y;        // [n] global labels (+1/-1)
  float* alpha;          // [n] global (replicated, updated identically on every rank)
  float* f;              // [nl] local gradient
  float* lines;          // [L][ldl] cache lines (K values)
  int64_t ldl;           // line stride in floats (>= G*kStepRows)
  int32_t* slot_of;      // [n] line of a global row or -1 (LRU)
  int32_t* key_of;       // [L] global row in a line or -1
  uint8_t* ref;          // [L] CLOCK reference bits
  float* hlines;         // [H][ldl] pinned host tier (device-mapped pointer) or nullptr
  int32_t* hslot_of;     // [n] host-tier line of a global row or -1
  int32_t* hkey_of;      // [H]
  int32_t H;             // host-tier lines (0 = off)
  uint64_t* partials;    // [G][2] per-workgroup selection keys
  SmoCtrl* ctrl;
  SmoStatus* status;     // host-mapped
  const uint8_t* records;  // partitioned: [world][rec_bytes] after all-gather
  uint8_t* my_record;      // partitioned: this rank's record (all-gather source)
  int64_t rec_bytes;
  int64_t n, nl, off;
  int64_t x_row0;        // global index of device X row 0 (0 replicated, off partitioned)
  int32_t d, dp, G, L;
  int32_t world;
  int32_t cache_mode;    // CacheMode
  int32_t partitioned;   // 1: X rows only local, query rows travel in records
  int32_t spec;          // speculative rows per X pass (LRU, replicated)
  int32_t clip;
  float C, gamma, eps, tau;
  int64_t max_iter;
  int32_t fused_rows;   // rows per workgroup of smo_fused (multiple of kFusedThreads)
  int32_t fused_G;      // workgroups of smo_fused (same on every rank)
  // diagnostics (DPSVM_STAMPS): s_memrealtime stamps of workgroups 0 and G-1,
  // ring of kStampRing iterations x 2 workgroups x kStampSlots
  uint64_t* stamps;
  // persistent cache engine (smo_persist_lru): every workgroup's private copy
  // of the cache metadata, plru_stride int32 words each:
  //   [0] CLOCK hand, [1..3] unused, slot_of[n], key_of[L], ref bits (L bytes)
  int32_t* plru_meta;
  int64_t plru_stride;
  // peer exchange (fused / persistent engines, xworld > 0): every workgroup
  // pushes its two selection keys as tagged granules straight into every rank's
  // receive buffer (xGMI peer stores); the next iteration polls its own buffer
  // until all tags match.  Layout per rank: [2 parity][xworld * fused_G][4] u64,
  // granule = 16-bit tag << 48 | 48-bit payload (xch.hpp).  Replaces the
  // per-iteration all-reduce (no collective launch, no host involvement).
  uint64_t* const* xpeer;  // [xworld] receive buffers (device-accessible)
  int32_t xrank, xworld;
  int32_t xstride;  // u64 slots per entry (>= kXchGranules; a multiple pads entries apart)
  int32_t xpoll_kb;  // 0: poll batch from the entry count; else fixed (2, 4, 8)
  int32_t xpoll_sleep;  // s_sleep(1) count between poll rounds
  int64_t xtimeout_ticks;  // give-up bound of one poll loop (s_memrealtime, 100 MHz)
  // residency census of the persistent engines (steps < 0: every workgroup
  // counts itself in and waits for the whole grid, bounded by census_ticks;
  // words [arrivals, abort])
  int32_t* census;
  int64_t census_ticks;
  int32_t eta_gram;  // 1: K(i_hi, i_lo) from the resident Gram (every column local)
};
constexpr int kXchGranules = 4;  // per workgroup entry: per side {key bits 63..16}, {key bits 15..0, alpha}

// ---- working-set engine (ws_*.hip) ----
// Decomposition around the reference's pair update: each round selects a
// working set of q rows (the most violating of I_up / I_low plus the newest
// part of the previous set), one workgroup solves the q-row sub-problem with
// the reference's pair rule from a q x q sub-Gram held in LDS, and one grid
// pass applies the round's alpha changes to every f_j and selects the next
// candidates.  ~10^5 dependent pair steps then cost an LDS round trip each
// instead of a grid-wide exchange.
constexpr int kWsMax = 192;          // working-set capacity: q x q fp32 sub-Gram in LDS (147 KiB)
constexpr int kWsCand = 16;          // candidates per side per selection workgroup (list capacity)
constexpr int kWsCandStd = 8;        // ... written by rounds of unions <= kWsAutoUnion (WsArgs::ncand)
constexpr int kWsCand1 = 4;          // ... of them read by the one-block merge and the peer exchange
constexpr int kWsSelThreads = 256;   // selection / f-update workgroup
constexpr int kWsMaxGroups = 256;    // selection workgroups per rank
constexpr int kWsListsPerThread = 4; // candidate lists a merge thread folds into one (<= 1024 lists over ranks)
constexpr int kWsMaxRPT = 32;        // rows per selection thread (256 x 256 x 32 = 2.1M rows per rank)
constexpr int kWsSolveThreads = 1024;
constexpr int64_t kWsAutoRows = 50000;   // solver auto: working-set engines from this many rows on (60k headline: ws 0.048 s vs smo 0.45 s)
// multi-block rounds (ws_blocks = P > 1, ws-dense at world 1): a round selects
// up to P x q_max rows and solves P disjoint q-row sub-problems at once on P
// workgroups; the combined step is scaled by the exact line-search factor
// t = min(1, g'd / d'Qd) of the dual (ws_*.hip "multi-block rounds")
constexpr int kWsMaxBlocks = 128;                 // blocks per round (P x q_max <= kWsMaxAll)
constexpr int kWsAutoBlocks = 32;                 // ws_blocks auto, coupled kernels: 32 blocks of kWsAutoUnion / 32 rows
constexpr int kWsAutoUnion = 16 * kWsMax;         // 3072 rows (the top 1536 of each side): coupled, ws-cache, world > 1
constexpr int kWsMaxAll = 32 * kWsMax;            // union capacity (6144 rows): uncoupled ws-dense rounds at world 1
constexpr int kWsCacheWindow = 512;               // ws-cache: victim lines searched after the CLOCK hand (ws_merge.hip)

// ws-cache needs the round's rows (2 q_max: this round's and last round's
// members are pinned) plus the victim window
inline int64_t ws_cache_min_lines(int q_max) { return 2 * (int64_t)q_max + kWsCacheWindow; }

// -s N (cache_lines > 0) on the engines a setup may choose: the reference takes
// any count (svmTrainMain.cpp:71, default 10; cache.cu:49-60, 82-105).  The
// production engines (engines = 0) raise a count below the working-set cache's
// minimum to that minimum; engines = 1 (the quarantined pair-at-a-time cache
// engines, which take any >= 2) keep it.  0 = no user cap.
inline int64_t production_line_cap(int64_t cache_lines, int ws_q, int engines) {
  if (cache_lines <= 0 || engines != 0) return cache_lines;
  const int64_t lo = ws_cache_min_lines(ws_q);
  return cache_lines < lo ? lo : cache_lines;
}
constexpr int kWsMergeThreads = 1024;             // multi-block merge: one workgroup
constexpr int kWsMaxPass1Splits = 16;             // multi-block f-update pass 1: list slices over workgroups
constexpr int64_t kWsAutoBlocksRows = 50000;      // ws_blocks auto: multi-block rounds from this many rows on
constexpr int64_t kWsSwitchRounds = 32;           // multi-block -> one-block graph switch granularity (rounds)

struct alignas(16) WsCtrl {
  int64_t iter;      // pair updates applied so far
  int64_t outer;     // rounds completed (round r builds its set into parity r & 1)
  int32_t done;      // DoneCode
  int32_t n_apply;   // alpha changes the next f update applies (0: none)
  int32_t q[2];      // working-set size per round parity (q[1] = 0 before round 0)
  float b_hi, b_lo;  // global selection of the current round
  int32_t nonfinite; // set by ws_select when an f value is not finite
  int32_t n_miss;    // cache mode: rows of the current set without a line (computed this round)
  int32_t hand;      // cache mode: next line the victim window starts at
  int32_t solve_cnt; // multi-block: solve workgroups finished this round (the last one commits)
  int32_t rank_cnt;  // multi-block: rank workgroups finished this round (the last one merges)
  int32_t pad[1];
  // block p's rows at [p * q_max, p * q_max + qb[par][p]) (one block: idx[par][0..q))
  int32_t idx[2][kWsMaxAll];     // working set per round parity (global rows), newest first
  int32_t line[2][kWsMaxAll];    // the line holding each member's kernel row (dense mode: the row itself)
  int32_t apply_idx[kWsMaxAll];  // rows whose alpha changed in the last round (multi-block: per-block segments)
  int32_t apply_line[kWsMaxAll]; // their lines
  float apply_coef[kWsMaxAll];   // their (alpha_new - alpha_old) * y
  int32_t miss_row[kWsMaxAll], miss_line[kWsMaxAll];  // cache mode: rows to compute this round, their lines
  int64_t rows_computed, row_hits;              // cache mode statistics
  // multi-block rounds
  int32_t uidx[2][kWsMaxAll];    // the union, newest first (previous-set retention)
  int32_t uq[2];                 // its size
  int32_t qb[2][kWsMaxBlocks];   // rows per block
  int32_t nab[kWsMaxBlocks];     // alpha changes per block (apply segment p at p * q_max)
  int32_t inb[kWsMaxBlocks];     // pair steps per block
  int32_t badb[kWsMaxBlocks];    // non-finite per block
  int32_t pad2[3];
  float t_last;                  // line-search factor of the last applied round
  int32_t n_damped;              // rounds applied with t < 1
  // adaptive block count: the next round's merge takes p_act blocks (seeded with
  // blocks; halved after every damped round — strongly coupled blocks; 1 after an
  // independent-clip event, which breaks sum(alpha y) = 0 and would drift P times
  // as fast with P blocks).  p_round: the blocks of the current round (its merge
  // writes it; the solve and the line search read it).
  int32_t p_act;
  int32_t p_round;
  int32_t clipb[kWsMaxBlocks];   // per block: a pair step was clipped (independent clipping)
  int64_t p1_round;              // rounds completed when p_act reached 1 (0: not yet) — the host
                                 // then switches to the one-block round graph at a block boundary
};

struct WsArgs {
  const float* gram;   // kernel-row lines: K(i, off + j) at gram[line(i) * ldg + j]
  int64_t ldg;
  const float* y;      // [n] global labels
  float* alpha;        // [n] global
  float* f;            // [nl] local gradient
  int64_t n, nl, off;
  int32_t G, rpt;      // selection geometry: G workgroups x 256 threads x rpt rows (same on every rank)
  int32_t world;       // ranks (> 1: candidates all-gathered, the sub-Gram all-reduced)
  int32_t G_all;       // candidate lists the merge reads: world * G
  int32_t q_max, n_new, inner_max;
  float rel_local;     // sub-problem tolerance: max(eps_floor, rel_local * global gap / 2)
  float eps_floor;     // its floor (rel_local * eps: rounds near the end keep taking steps)
  float C, eps, tau;
  int32_t clip;
  int64_t max_iter;
  int32_t cache;       // 0: gram = the resident Gram (line i = row i); 1: kernel-row cache
  int32_t L;           // cache mode: lines
  int32_t* slot_of;    // cache mode: [n] line of a global row or -1
  int32_t* key_of;     // cache mode: [L] row held by a line or -1
  uint64_t* cand_out;  // [G][2][kWsCand] this rank's per-workgroup candidate keys (up, low), ascending
  uint64_t* cand;      // [G_all][2][kWsCand] every rank's lists (== cand_out at world 1)
  float* subg;         // [q_max][q_max] sub-Gram of the current working set (row stride q_max; at
                       // world > 1 each rank fills the columns it owns, zeros elsewhere: summed)
  float* aux;          // [3][kWsMax] f (owner-filled, summed with subg), alpha, y of the working set
  WsCtrl* ctrl;
  SmoStatus* status;   // host-mapped
  uint64_t* stamps;    // DPSVM_STAMPS diagnostics: s_memrealtime per phase, ring of kStampRing rounds
  // in-kernel peer exchange of the rounds (world > 1; nullptr: the communicator's
  // collectives).  Every rank's receive buffer (uncached, IPC-mapped by its
  // peers; ws_common.hpp "peer exchange"): [2 parity][G_all][xcw] candidate
  // granules (per side xcw / 4 keys of two granules: up at 0, low at xcw / 2),
  // from word xsub [2 parity][xsub_rows][q_max + 1] sub-Gram rows with the row's
  // f in the last column, and (multi-block rounds) from word xpart [2 parity]
  // [G_all * ks][4] line-search partials (two doubles of two granules each)
  uint64_t* const* xpeer;
  int32_t xrank;
  int32_t xcw;       // granules per candidate slot: 4 kWsCand1 (one-block engine) or 4 kWsCand (multi-block)
  int64_t xsub;
  int64_t xsub_rows; // sub-Gram rows per parity (blocks x q_max of the widest view)
  int64_t xpart;
  int64_t xtimeout_ticks;  // give-up bound of one poll (s_memrealtime, 100 MHz)
  // multi-block rounds (P = blocks > 1): subg / aux hold P blocks
  // ([P][q_max][q_max], [P][3][kWsMax]); the f update runs in two passes
  int32_t blocks;
  float* dfs;          // [nl] the round's f change before the line search
  float* dalpha;       // [n] alpha_new - alpha_old of the round's changed rows (0 elsewhere)
  double* part;        // [G_all][2] per-workgroup partial sums: d'Qd, g'd (this rank's at rank * G)
  int32_t rank;        // this rank (its partials slot)
  int32_t aux_stride;  // aux: [3][blocks][kWsMax] (f of every block first: one sum all-reduce with subg)
  int32_t wss;         // sub-problem pair selection: 1 first order (the reference's), 2 second order (WSS2)
  float t_halve;       // multi-block: a round damped to t < t_halve halves the block count
  int32_t clip_fallback;  // multi-block, independent clipping: a clip event drops to one block (1) or not (0)
  int32_t ks;          // multi-block pass 1: list slices over workgroups (dfs [ks][nl], part [world p1G][ks][2])
  int32_t p1G;         // multi-block pass 1: column groups per rank (= G; the wide pass 1: ceil(nl_max / 1024))
  int32_t p1v4;        // multi-block pass 1: 1 = wide column groups, 4 columns (16-B loads) per thread
  uint64_t* sorted;    // multi-block: [2][kWsMaxGroups * kWsCand] every candidate key per side, ascending (ws_rank)
  int32_t direct_sub;  // multi-block solve loads its sub-Gram / f / alpha / y straight from the resident Gram
                       // (world 1, dense, blocks of <= 64 rows: no ws_gather launch)
  int32_t ncand;       // multi-block selection: keys per side a list holds (kWsCandStd for unions of <=
                       // kWsAutoUnion rows, kWsCand beyond; 0 = kWsCand); the tail of a list is kKeyNone
};
// keys per side and list of the multi-block selection (ws_select pass 2, the peer exchange)
constexpr int ws_ncand(int ncand) { return ncand > 0 && ncand < kWsCand ? ncand : kWsCand; }
// u64 words of the working-set exchange region (both parities): one-block
// engine
constexpr int64_t ws_xch_words(int64_t G_all, int64_t q_max) {
  return 2 * G_all * 4 * kWsCand1 + 2 * q_max * (q_max + 1);
}
// multi-block engine (P blocks of q rows; its one-block rounds use q1 rows):
// candidates (kWsCand keys per side), line-search partials, sub-Gram rows
constexpr int64_t ws_xch_cand_words_multi(int64_t G_all) { return 2 * G_all * 4 * kWsCand; }
// (P1_all = world x p1G pass-1 groups: the selection groups, or the wide pass 1's)
constexpr int64_t ws_xch_part_words(int64_t P1_all, int64_t ks) { return 2 * P1_all * ks * 4; }
constexpr int64_t ws_xch_sub_words(int64_t P, int64_t q, int64_t q1) {
  return 2 * ((P * q * (q + 1)) > (q1 * (q1 + 1)) ? P * q * (q + 1) : q1 * (q1 + 1));
}
constexpr int64_t ws_xch_words_multi(int64_t G_all, int64_t P1_all, int64_t ks, int64_t P, int64_t q, int64_t q1) {
  return ws_xch_cand_words_multi(G_all) + ws_xch_part_words(P1_all, ks) + ws_xch_sub_words(P, q, q1);
}
constexpr int kStampRing = 4096;
constexpr int kStampSlots = 12;

}  // namespace dpsvm
