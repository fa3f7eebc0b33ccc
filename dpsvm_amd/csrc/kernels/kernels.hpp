// Host-side launchers of the HIP kernels (implemented in *.hip under kernels/).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/device_state.hpp"

namespace dpsvm {
namespace launch {

void row_sqnorm(const float* x, int64_t n, int d, int ld, float* out, hipStream_t s);
void init_f(const float* y, int64_t off, int64_t nl, float* f, hipStream_t s);
void fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s);

// One SMO iteration's kernels (see device_state.hpp)
void smo_rows(const SmoArgs& a, hipStream_t s);
void smo_step(const SmoArgs& a, hipStream_t s);
void smo_local_record(const SmoArgs& a, hipStream_t s);
void smo_finalize(const SmoArgs& a, hipStream_t s);
size_t smo_rows_lds_bytes(int dp);
// cache mode, replicated X: one fused SMO iteration with in-launch line fills
bool smo_fused_lru_supported(int dp);
size_t smo_fused_lru_lds_bytes(int dp, int fused_rows);
void smo_fused_lru(const SmoArgs& a, const uint64_t* p_in, uint64_t* p_out, const FusedCacheRec* r_in,
                   FusedCacheRec* r_out, hipStream_t s);
// dense mode: init (selection only, mode 0; r_in = the seed record when
// a.xworld > 0) or one fused SMO iteration (mode 1)
void smo_fused(const SmoArgs& a, int mode, const uint64_t* p_in, uint64_t* p_out, const FusedRec* r_in,
               FusedRec* r_out, hipStream_t s);
// dense mode, persistent: up to `steps` SMO iterations in one launch (every
// workgroup co-resident; keys exchanged as tagged granules, a.xworld >= 1);
// st: state record in/out (iteration, done, b_hi, b_lo; no pending pair)
void smo_persist(const SmoArgs& a, FusedRec* st, int steps, hipStream_t s);
// publications watched per lane per poll round for a's exchange geometry
int poll_batch(const SmoArgs& a);
// residency of the persistent engines' kernels (the instantiation `a` runs):
// occupancy API answer per CU, and the census launch (steps < 0) with `groups`
// workgroups; a.census = two zeroed words, a.census_ticks = give-up bound
int smo_persist_blocks_per_cu(const SmoArgs& a);
void smo_persist_census(const SmoArgs& a, int groups, hipStream_t s);
// test entry: the cache engines' X pass (xpass_fill) over a.nl rows, queries
// keys_dev[0..n_new) into lines 0..n_new-1 (a.lines / a.ldl / a.fused_rows)
void xpass_rows(const SmoArgs& a, const int* keys_dev, int n_new, hipStream_t s);
int smo_persist_lru_blocks_per_cu(const SmoArgs& a);
void smo_persist_lru_census(const SmoArgs& a, int groups, hipStream_t s);
// cache mode, persistent (smo_persist_lru.hip): up to `steps` SMO iterations in
// one launch, private per-workgroup cache metadata (a.plru_meta, plru_init);
// stats: int64 [hits, misses, rows computed, X passes, speculative rows] in/out
bool smo_persist_lru_supported(int dp, int fused_rows, int fused_G);
int64_t plru_stride_words(int64_t n, int64_t L);
void plru_init(int32_t* meta, int64_t stride, int64_t G, int64_t n, int64_t L, hipStream_t s);
void smo_persist_lru(const SmoArgs& a, FusedRec* st, int steps, int64_t* stats, hipStream_t s);
void preload_persist_lru_kernel(hipStream_t s);
// load the code objects of the kernels that spin on other ranks/workgroups
// BEFORE any of them runs: a first launch that loads its code object while a
// peer's spinning kernel occupies the device can stall behind it
void preload_fused_kernels(hipStream_t s);
void preload_persist_kernel(hipStream_t s);
// peer-exchange self test: every rank pushes a tagged granule to every rank and
// polls its own; *ok = 1 when all arrived within timeout_ticks
//   (ping slots at u64 offset ping_off of every receive buffer)
void xch_ping(uint64_t* const* peers, int rank, int world, int64_t ping_off, uint32_t tag, int64_t timeout_ticks,
              int32_t* ok, hipStream_t s);

// working-set engine (ws_*.hip): selection geometry for the largest shard
// (<= 256 / world workgroups x 256 threads x rpt rows); one round = ws_gather (merge,
// stop test, working set, sub-Gram rows), ws_solve (the sub-problem), then
// ws_select (f update, next candidates)
bool ws_supported(int64_t nl_max, int world, int q_max);
void ws_geometry(int64_t nl_max, int world, int32_t* G, int32_t* rpt);
int ws_pass1_splits(int G);  // multi-block pass 1: workgroups per selection group
int ws_pass1_v4_groups(int64_t nl_max);  // the wide pass 1: 1024-column groups per rank
int ws_pass1_v4_splits(int p1G);         // ... and its list slices per group
void ws_select(const WsArgs& a, hipStream_t s);
// multi-block rounds: pass 1 (d_f + line-search partials), pass 2 (apply, candidates); at
// world > 1 the partials are all-gathered between them
void ws_select_pass(const WsArgs& a, int pass, hipStream_t s);
void ws_gather(const WsArgs& a, hipStream_t s);
void ws_solve(const WsArgs& a, hipStream_t s);
// ws-cache without the cache (ws_recompute.hip): merge + sub-Gram from the split
// X rows, and the round's f update with the kernel rows recomputed (d <= 64)
bool ws_recompute_supported(const WsArgs& a, int dp);
void ws_subgram_split(const WsArgs& a, const void* xs, const int32_t* xsh, const float* xsq, int dp, float gamma,
                      hipStream_t s);
void ws_fupdate_split(const WsArgs& a, const void* xs, const int32_t* xsh, const float* xsq, int dp, float gamma,
                      hipStream_t s);
// cache mode: the merge + line assignment (one workgroup) runs before the
// row GEMM; ws_gather then reads the sub-Gram from the members' lines
void ws_merge(const WsArgs& a, hipStream_t s);
// multi-block rounds (a.blocks > 1, ws-dense at one rank): the union merge before ws_gather
// multi-block rounds over the peer exchange: every rank's candidate lists / line-search
// partials from this rank's receive buffer into cand / part (the all-gathers' layout)
void ws_xcollect_cand(const WsArgs& a, hipStream_t s);
void ws_xcollect_part(const WsArgs& a, hipStream_t s);
void ws_merge_multi(const WsArgs& a, hipStream_t s);
// the adaptive block count reached 1: the last union becomes the one-block
// kernels' previous set (run once, between two rounds)
void ws_to_single(const WsArgs& a, hipStream_t s);
bool ws_cache_supported(int64_t L, int q_max);
// multi-block rounds in cache mode: the union's lines come from a 4096-line window
bool ws_cache_multi_supported(int64_t L, int blocks, int q_max);
// partitioned X, cache mode: out[i] = X row ctrl->miss_row[i] if this rank owns
// it (rows off..off+nl-1 at x), else zeros; out_sq[i] = its global |x|^2
void ws_pack_rows(const float* x, int64_t off, int64_t nl, int dp, const float* xsq, const WsCtrl* ctrl, int q_max,
                  float* out, float* out_sq, hipStream_t s);

// RBF GEMM: out[i*ldo + j] = K(A_i, B_j) for i < M, j < N
//   A: [M_pad][lda], B: [N_pad][ldb] (rows padded to 128, zero filled; rbf_rows_indexed
//   reads B rows to a multiple of 512)
//   symmetric: B == A (one rank): tiles above the diagonal only, each also
//   stores its transpose (half the MFMA work, bit-identical values)
void rbf_gemm_store(const float* A, const float* Asq, int64_t M, int lda, const float* B,
                    const float* Bsq, int64_t N, int ldb, int dp, float gamma, float* out,
                    int64_t ldo, hipStream_t s, bool symmetric = false);
// Kernel rows by index: lines[out_rows[i]][j] = K(X[a_rows[i]], B_j) for i < *m_dev
// (<= M_max, read on the device), j < N — one MFMA GEMM for a set of cache misses
void rbf_rows_indexed(const float* X, const float* Xsq, const int32_t* a_rows, const int32_t* m_dev, int64_t M_max,
                      const float* B, const float* Bsq, int64_t N, int dp, float gamma, float* lines,
                      const int32_t* out_rows, int64_t ldl, hipStream_t s);
// The same two GEMMs on fp16 MFMA over split operands (rbf_gemm_split.hip):
// every X row scaled by 2^shift and stored as fp16 hi / lo planes ("split
// rows", split_row_u4(dp) 16-B units per row; buffers hold split_pad_rows(rows)
// rows, pad zeroed); fp32 accuracy, bit-identical under operand swap
int64_t split_row_u4(int dp);
int64_t split_pad_rows(int64_t rows);
void split_rows_f16(const float* x, int64_t rows, int dp, int ldx, void* out, int32_t* shift, hipStream_t s);
// split STORE GEMM variant: 0 auto (4 when dp > 128, else 3), 1 register-staged tile per workgroup, 3 LDS-DMA,
// 4 persistent LDS-DMA
int split_gemm_variant();
void set_split_gemm_variant(int v);
// diagnostics: per-workgroup s_memtime stamps of the wide-wave Gram kernel (nullptr: off)
void set_gram_stamps(uint64_t* p);
void set_rows_stamps(uint64_t* p);  // diagnostics: the LDS-DMA rows kernel's per-workgroup stamps (0: off)
// cold_tau > 0: the adaptive Gram (docs/DESIGN.md §13) — a one-product pass, then the tiles holding an element
// split_cold rejects recomputed with all three products; every stored value within cold_tau of the three-product
// one.  Falls back to the three-product kernel where the persistent wide-wave path does not apply.
void rbf_gemm_store_split(const void* A, const int32_t* Ash, const float* Asq, int64_t M, const void* B,
                          const int32_t* Bsh, const float* Bsq, int64_t N, int dp, float gamma, float* out,
                          int64_t ldo, hipStream_t s, bool symmetric = false, float cold_tau = 0.f);
// split_cold's constants c0, c1 for gamma, tau (host; docs/DESIGN.md §13)
void split_cold_consts(float gamma, float tau, float* c0, float* c1);
// the calling thread's last adaptive Gram: tiles of the one-product pass and the hot ones recomputed (valid once
// the stream passed the GEMM; -1 / -1 when the last Gram was not adaptive)
void gram_adapt_last(int64_t* tiles, int64_t* hot);
void rbf_rows_indexed_split(const void* X, const int32_t* Xsh, const float* Xsq, const int32_t* a_rows,
                            const int32_t* m_dev, int64_t M_max, const void* B, const int32_t* Bsh, const float* Bsq,
                            int64_t N, int dp, float gamma, float* lines, const int32_t* out_rows, int64_t ldl,
                            hipStream_t s);
// Decision values: dec[i] = sum_j coef[j] K(A_i, B_j) - b   (B = SVs, coef = alpha*y)
//   partial: scratch [splits][M_pad] (returned by predict_scratch_floats)
int64_t predict_scratch_floats(int64_t M, int64_t N);
// the split-operand decision GEMM behind rbf_predict (dp >= 128; DPSVM_PREDICT=f32 forces the f32 kernel):
// f32 A / B split into stream-ordered scratch, partial [<= max_splits][ldp] (unused splits zeroed)
void rbf_predict_split(const float* A, const float* Asq, int64_t M, int lda, const float* B, const float* Bsq,
                       const float* coef, int64_t N, int ldb, int dp, float gamma, float* partial, int64_t ldp,
                       int max_splits, hipStream_t s);
// which decision GEMM rbf_predict runs for this dp: the split-operand one (dp >= 128) or the f32 one
bool predict_uses_split(int dp);
// precision: 0 auto (predict_uses_split), 1 the f32-input MFMA GEMM, 2 the split-operand GEMM (any dp)
void rbf_predict(const float* A, const float* Asq, int64_t M, int lda, const float* B,
                 const float* Bsq, const float* coef, int64_t N, int ldb, int dp, float gamma,
                 float b, float* partial, float* dec, const float* y, int32_t* correct,
                 hipStream_t s, int precision = 0);

// SV compaction: idx_out[k] = i for the k-th alpha[i] > 0 (index order)
// scratch: >= compact_scratch_ints(n) ints; count written to *count_dev
int64_t compact_scratch_ints(int64_t n);
void compact_positive(const float* alpha, int64_t n, int32_t* idx_out, int32_t* count_dev,
                      int32_t* scratch, hipStream_t s);
// sv[r] = x[idx[r]-x_row0], svsq[r] = xsq[idx[r]], coef[r] = alpha[idx[r]] * y[idx[r]]
void gather_sv(const float* x, int64_t x_row0, const float* xsq, const float* alpha,
               const float* y, const int32_t* idx, int64_t nsv, int dp, float* sv, float* svsq,
               float* coef, hipStream_t s);

}  // namespace launch
}  // namespace dpsvm

namespace dpsvm {
namespace launch {
// microsecond cost per kernel of a graph-replayed chain of dependent empty kernels
double launch_floor_us(int blocks, int threads, int chain, int reps);
// known-bytes 16-B streaming read (FETCH_SIZE probe); out[blocks] per-workgroup sums
void stream_read(const void* x, int64_t bytes, float* out, int blocks, hipStream_t s);
}  // namespace launch
}  // namespace dpsvm
