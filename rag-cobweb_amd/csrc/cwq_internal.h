// Internal declarations shared by the libcwq kernels (cwq_kernels.hip) and the
// C-ABI host runtime (cwq_api.hip).  Not part of the public interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cwq {

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kWavesPerWG = 4;   // 256-thread workgroups
constexpr int kXQ = 16;         // queries per scalar-load group (queries per wave)
constexpr int kDChunk = 32;      // D is padded to a multiple of this (largest compute chunk)

// Per leaf-class row constants (one float4 load per lane in the epilogue).
struct RowMeta {
  float logdet;  // sum_d log v  (fp64-accumulated, rounded once)
  float iv;      // 1/v for isotropic rows (v identical across d), unused otherwise
  float cw;      // fp32(level_w[depth] / path_len)   -- CobwebWrapper.py:166-168
  float invL;    // fp32(1 / path_len)
};

enum Epi { EPI_RAW = 0, EPI_KEY = 1, EPI_TOPK = 2 };

// The exact key of an isotropic row from its raw sum acc = sum_d (x_d - mu_d)^2 (16-dim
// fma partials summed in slice order): lp = -(logdet + dconst + iv acc)/2, Fast key
// fmaf(pp, invL, cw lp) (pp = the parent's prefix), categorize min(pp, lp) (pp = BF).  One
// expression shared by the rerank kernels and group pruning's seed, so their keys agree bit
// for bit with each other and with the scan's epilogue.
// The sum of n partials p[0] + p[1] + ... in index order (the scan's slice order, so the
// rounding is the scan's): 16 LDS reads issued before their adds, not one read latency per add.
__device__ __forceinline__ float sum_in_order(const float* p, int n) {
  float acc = 0.f;
  int v = 0;
  for (; v + 16 <= n; v += 16) {
    float t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) t[u] = p[v + u];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += t[u];
  }
  for (; v < n; ++v) acc += p[v];
  return acc;
}

__device__ __forceinline__ float iso_key_tail(float acc, const RowMeta& md, float pp, float& lp, int cat,
                                              float dconst) {
  const float S = md.iv * acc;
  lp = -0.5f * (md.logdet + dconst + S);
  return cat ? fminf(pp, lp) : fmaf(pp, md.invL, md.cw * lp);
}

// Row flags
constexpr int FLAG_HAS_SENT = 1;   // the row's node holds >= 1 sentence
constexpr int FLAG_INT_COPY = 2;   // the row duplicates an internal node that holds sentences

// Arguments of the scan (score) kernel that are not hot pointers.
struct ScanArgs {
  int DP;              // padded dimension (multiple of kDChunk)
  int nq;              // valid queries in this call
  int64_t ld;          // leading dimension of the dim-major row arrays
  int nrows;           // valid rows in the segment
  int nrows_pad;       // rows rounded up to 64
  int rows_per_slab;   // rows per workgroup (multiple of 64)
  int n_qblocks;       // query blocks (a multiple of 8 when xcd_map)
  int xcd_map;         // XCD-aware block -> (slab, query block) mapping
  int seg_base;        // global leaf-row id of segment row 0
  const RowMeta* meta; // [nrows]
  const int* par;      // [nrows] internal-node id of the parent (-1: none)
  const int* flags;    // [nrows]
  const float* P;      // [nq_pad][ldP] prefix sums (fast) or bottleneck lp (categorize)
  int64_t ldP;
  float dconst;        // 0 for lp', D*log(2*pi) for the full log-likelihood
  float* out;          // RAW / KEY output [nq][ldo]
  int64_t ldo;
  int out_base;        // column offset of segment row 0 in `out`
  float* pkey;         // TOPK partial lists [nq_pad][nslab_total][K]
  float* paux;
  int* prow;
  int nslab_total;
  int slab_off;
  int K;
};

// Heap entry of the categorize simulation.
struct HeapEnt {
  float score;   // lp(node) (full, with 2*pi) -- CobwebTorchTree.py:243,285
  float pscore;  // parent's lp (0 for the root)
  int tb;        // BFS index (deterministic stand-in for random())
  int node;      // >= 0: internal id; < 0: -(leaf row + 1)
};

struct SimArgs {
  int nq, k, R;
  int64_t max_nodes;
  int NI, NL;
  const float* LPF;  // [nq_pad][NI] full lp of internal nodes
  const float* BF;   // [nq_pad][NI] bottleneck (path-min) lp of internal nodes
  int64_t ldI;
  // LIST mode: top-R leaf rows by bottleneck key; DENSE mode (R == 0): all rows
  const float* lkey; const float* laux; const int* lrow;   // [nq][R]
  const float* dense_lpf;                                   // [nq][NL] (DENSE)
  int64_t ldL;
  int complete;      // the LIST covers every leaf row
  const int* int_child_begin; const int* int_child_end;     // internal children ranges [NI]
  const int* int_nchild;     // all children (for the log_prob call count)
  const int* int_bfs; const int* int_has_sent;
  const int* int_leaf_a0; const int* int_leaf_a1;           // leaf-row child ranges (iso segment)
  const int* int_leaf_b0; const int* int_leaf_b1;           // (aniso segment)
  const int* row_par; const int* row_bfs; const int* row_flags;
  HeapEnt* heap; int64_t heap_cap;
  int64_t* out_nodes; int* n_found; int64_t* n_calls; int* status;
  const int* par_int;  // parent internal id of every internal node (cat_count_kernel)
  int pre_status;      // simulate: skip the queries whose status the count pass already set to 0
  // two-level replay (simulate_two_kernel, §4.7): the second-level table T2 [nq_pad][NI]
  // (cat_t2_kernel) and the list by the second-level key [nq][R]
  const float* T2;
  const float* lkey2; const float* laux2; const int* lrow2;
  // simulate_two_kernel: skip the queries whose gate[q] is 0 (the first replay resolved them;
  // launched before the host has read that status), writing nothing for them; null: none
  const int* gate;
  // lazy DENSE replay (simulate_lazy_kernel): a popped node's leaf rows get their full lp
  // computed on the spot from the query's padded slices X (chunk layout) and the rows'
  // operands -- isotropic mu row-major (Mf [row][DP], the rerank's copy), anisotropic A / B
  // dim-major -- with the scan's arithmetic
  const float* X; int DP;
  const float* Mf; int NL_iso;
  const float* anA; const float* anB; int64_t ld_an;
  const RowMeta* meta; float dconst;
};

// Node variances read by the index build.  Full: [n_nodes][D] rows (compute_var of every
// node, CobwebWrapper.py:186-203).  Compact (cwq_index_create_cv): one scalar per node --
// a node whose D variances are one repeated value, as every count-1 leaf's are
// (var = prior_var, CobwebTorchTree.py:336-342) -- plus full rows for the nodes listed in
// an_map (an_map[node] >= 0: that node's row of an_var).  Both give the same values.
struct VarSrc {
  const float* full;     // [n_nodes][D], or nullptr (compact)
  const float* row;      // compact: [n_nodes]
  const int* an_map;     // compact: [n_nodes], row of an_var or -1
  const float* an_var;   // compact: [n_an][D]
  __device__ __forceinline__ float at(int64_t node, int d, int D) const {
    if (full) return full[node * D + d];
    const int m = an_map[node];
    return m >= 0 ? an_var[(int64_t)m * D + d] : row[node];
  }
};

// ---- launchers (cwq_kernels.hip) ----
hipError_t launch_pad_queries(const float* q, int64_t nq, int D, float* X, int64_t nq_pad, int DP, hipStream_t s);
// out[c][r] = in[r][c] (r < rows, c < cols), leading dimensions ld_in / ld_out
hipError_t launch_transpose(const float* in, int64_t rows, int64_t cols, int64_t ld_in, float* out, int64_t ld_out,
                            hipStream_t s);
// rows of `words` 4-byte words: dst[di ? di[i] : i] = src[si ? si[i] : i] (strides in words)
hipError_t launch_copy_rows(const void* src, int64_t src_stride_w, const int64_t* src_idx, void* dst,
                            int64_t dst_stride_w, const int64_t* dst_idx, int64_t n, int64_t words, hipStream_t s);
hipError_t launch_iso_flags(const VarSrc& var, int D, const int64_t* nodes, int64_t n, int* flags, hipStream_t s);
// mode 0: dst = mean, 1: dst = 1/sqrt(var), 2: dst = mean/sqrt(var)
hipError_t launch_gather_T(const float* mean, const VarSrc& var, int D, const int64_t* nodes, int64_t n, int mode,
                           float* dst, int64_t ld, int DP, hipStream_t s);
hipError_t launch_logdet(const VarSrc& var, int D, const int64_t* nodes, int64_t n, float* out, hipStream_t s);
hipError_t launch_inv_var0(const VarSrc& var, int D, const int64_t* nodes, int64_t n, float* out, hipStream_t s);

// The fused scan: ISO/ANISO rows x {RAW, KEY, TOPK} x {fast, categorize}.
// the internal pass of a one-query call (anisotropic rows, EPI_RAW), D split over 4 waves
hipError_t launch_raw_split(const float* X, const float* A, const float* B, const ScanArgs& a, hipStream_t s);
hipError_t launch_scan(bool iso, int epi, bool cat, int kl, const float* X, const float* A, const float* B,
                       const ScanArgs& a, int nslab, hipStream_t s);
constexpr int kScanSmallQ = 256;     // calls with at most this many queries use the shared-query scan
void scan_cfg_begin(int64_t nq);     // scan configuration for the current call (thread-local)
void scan_cfg_end();
int scan_tq(int kl);                 // queries per wave for a list width
int scan_rows_per_tile(int kl);      // rows per workgroup step (64 * rows per lane [* 4 if shared queries])
int scan_queries_per_block(int kl);  // queries per workgroup
int scan_dchunk(int kl);             // dims per compute phase (D is padded to a multiple of 32)
int scan_lists_per_slab(int kl);     // partial top-k lists a workgroup writes per query
int scan_xcd_map();                  // XCD-aware block mapping (CWQ_XCD_MAP, default 1)
int scan_wgs_per_cu(int kl);         // resident workgroups per CU (occupancy query, cached)

// Small-corpus exact scan (isotropic rows, fast top-K lists of K <= 16): lane = query,
// blocks of 16 or 32 rows staged in LDS.  For segments of at most kSmallScanMaxRows rows
// with many queries, where the row-sliced scan has few waves (few slabs per query block)
// and waits on its scalar query loads.  Writes one list per slab, like the scan
// (a.slab_off, a.nslab_total).
constexpr int kSmallScanMaxRows = 16384;  // segment size limit (lists per query <= 128)
constexpr int kSmallScanMinQ = 64;        // one full wave of queries
constexpr int kSmallScanMaxK = 16;
int small_scan_slabs(int64_t nq, int nrows);   // slab count (= lists per query)
hipError_t launch_scan_small(const float* X, const float* M, const ScanArgs& a, int nslab, hipStream_t s);

hipError_t launch_int_small(const float* X, const float* A, const float* B, int64_t ld, int NI, int DP, int nq,
                            float* out, int64_t ldo, hipStream_t s);
hipError_t launch_prefix_level(const float* S, int64_t ldS, int nq, int i0, int i1, const int* par_int,
                               const float* w_int, const float* logdet_int, float dfull, float* P, float* BF,
                               float* LPF, hipStream_t s);
// Internal nodes' raw sums -> prefixes for a few queries (internal_chain_kernel,
// cwq_group.hip): one thread per (query, node) down the node's path with
// prefix_level_kernel's arithmetic, then (G > 0) the group-centred prefix tables with
// group_shift_kernel / group_pprime_kernel's.
struct IntFinishArgs {
  const float* S; int64_t ldS; int nq; int NI;
  const int* lv0; int nlev;                      // level starts, lv0[nlev] = NI
  const int* par_int; const float* w_int; const float* logdet_int; float dfull;
  float* P; float* BF; float* LPF;               // [nq][ldS]; BF / LPF optional
  const float* q; int D; const float* c0; const float* cent; int G;   // groups (G > 0)
  const int* grp; const double* F; const double* Fc; double* sh;
  float* Plo; float* Phi; float* Pclo; float* Pchi;
};
hipError_t launch_internal_finish(const IntFinishArgs& f, hipStream_t s);

// ---- group pruning for the Fast query on group-centred trees (cwq_prune.hip) ----
// Per (query, group g): an upper bound KUB of every Fast key of the rows below the depth-1
// node g, from the query's distance to the group centre.  Stage A computes
// the exact internal pass only for each query's best group g* (argmax KUB); every other
// (query, node) gets the sentinel prefix kPruneSent in the filters' tables (its rows can
// never be candidates).  Once the filter's first threshold T[q] (<= tau_K) is known, stage
// B computes the groups with KUB >= T[q]; the groups left are certified to hold no top-K row.
constexpr float kPruneSent = -1e24f;   // the pruned prefix (any real prefix is > kPruneCut)
constexpr float kPruneCut = -1e20f;
struct GroupBound {   // per group, fp64 (cwq_api.hip build_prune)
  double r;           // >= max |mu_a - c_g| over the group's members (internal nodes and rows)
  double wmin, wmax;  // min / max per-dimension weight (A^2 or iv) over the members
  double ldmin, ldabs;   // min logdet, max |logdet| over the members
  double mmax;        // >= max |mu_a|
  double iLmin, iLmax, Cmin, Cmax;   // usable rows: 1/L and C = invL * sum_{path, a != root} w_a + cw
  int valid;          // the group has a usable row (else never relevant)
  int pad_;
};
struct PruneArgs {
  int nq, G, NI, DP, D, K;
  int64_t ldS;                  // [nq][ldS] tables (S_int, P, Pg_lo, Pg_hi)
  const float* q;               // the caller's queries [nq][D]
  const float* X;               // the chunk's padded query slices (kXQ interleave)
  const float* c0;              // the root centre; cent: group centres [G][D]
  const float* cent;
  const float* Ar; const float* Br;   // row-major fp32 A, B of the internal nodes [NI][DP]
  const int* par_int; const float* w_int; const float* logdet_int;
  const int* gint;              // pruning group of each internal node (-1: a top node)
  const int* gi_ptr; const int* gi_nodes;   // group-major internal node lists (BFS order)
  const int* gi_dep; const int* gi_ppos;    // per list entry: tree depth, the parent's list position (-1: the root)
  int gmaxdep, gmindep;                     // deepest / shallowest internal node of any group
  // top nodes (no group: the root and the centres' ancestors), BFS order, computed exactly by
  // the head kernel for every query; per group the top-list position of its centre's parent
  const int* top_nodes; const int* top_ppos; const int* top_dep; int n_top, top_maxdep;
  const int* grp_tpos;
  const GroupBound* gb;
  double* kpart;                // [2][nq][G]: P0-free part of KUB, and the margin's magnitude term
  float* S; float* P;           // [nq][ldS]
  float* Plo; float* Phi;       // the filters' shifted prefix tables (group-centred rows)
  const int* grp; const double* F; double* sh;   // centring group, F, shifts + errors [2][nq][G]
  int fillP;                    // also write the sentinel into P (anisotropic leaf rows read P)
  float* kub;                   // [nq][G] key upper bounds (rounded up)
  int* gstar;                   // [nq] best group (-1: none)
  int2* pairs; int* ctr;        // stage B pair list; ctr[0] pair count, [3] claim counter, [4] call total
  // the seed threshold: up to 64 sample rows per group, their exact keys (cwq_mfma.hip's arithmetic)
  const int* gs_ptr; const int* gs_rows; const float* Mf; const RowMeta* meta; const int* row_par;
  float* Tseed;                 // [nq]
  float* T0; int64_t ldT0;      // optional: also written (the per-call filter's threshold, no probe)
  int gnodes_max;               // the most internal nodes of one group (g*'s pass: workgroups per query)
  int zero_total;               // the head kernel also zeroes ctr[4] (the call's first pruned chunk)
  // optional (the per-call filter): the 16-row blocks of the isotropic rows it must pass over
  // -- blk_grp[b] the pruning group of all the block's rows (-1: mixed, or rows outside every
  // group), kept when some query of the call keeps that group -- appended to live, count ctr[5]
  const int* blk_grp; int64_t nblk;
  int* live;
};
// launches: head (shifts, the bound terms, the root, KUB, g*; the counters zeroed), g*'s exact
// pass (many workgroups per query), seed (g*'s prefixes and tables, T, stage-B pairs, sentinel
// fill), stage B (the pairs' exact passes)
hipError_t launch_prune(const PruneArgs& a, int cus, bool first, hipStream_t s);
constexpr int kPruneMaxTop = 1024;                   // top nodes the head kernel holds in LDS
constexpr size_t kPruneLdsCap = (size_t)150 * 1024;  // the seed / stage-B kernels' dynamic LDS
size_t prune_lds_max(int DP, int gmax);
// a kernel's dynamic-LDS attribute raised to `bytes` once per (kernel, device), thread-safe
hipError_t ensure_dyn_lds(const void* fn, size_t bytes);
hipError_t launch_raise_threshold(float* T, int64_t ldT, const float* Tfloor, int nq, hipStream_t s);
hipError_t launch_prune_members(const float* mean, const VarSrc& var, int D, const int64_t* nodes, const float* iv,
                                const int* grp, const float* cent, int64_t n, double4* out, hipStream_t s);
hipError_t launch_cat_t2(const float* BF, const float* LPF, int64_t ldI, int NI, int nq, const int* par_int,
                         const float* lkey, int R, float* T2, hipStream_t s);
hipError_t launch_simulate_two(const SimArgs& a, hipStream_t s);
hipError_t launch_skip_failed(int* status, const int* okf, int nq, int init, hipStream_t s);
// dst[j * nq + q] = src[j] ? src[j][q] : 0 for j < 5: a call's per-query flag arrays into one
// host-mapped buffer, read back with a single stream sync (no pageable copies)
// nodes (optional): also nodes[q][i] = -1 for i >= n_found[q] (clear_tail_kernel's work)
hipError_t launch_gather_flags(int* dst, int nq, const int* s0, const int* s1, const int* s2, const int* s3,
                               const int* s4, hipStream_t s, int64_t* nodes = nullptr, const int* n_found = nullptr,
                               int k = 0);
hipError_t launch_clear_tail(int64_t* nodes, const int* n_found, int64_t nq, int k, hipStream_t s);
hipError_t launch_merge(const float* pkey, const float* paux, const int* prow, int nq, int nent, int K,
                        float* okey, float* oaux, int* orow, hipStream_t s, bool cat);
hipError_t launch_merge_expand(const float* pkey, const float* paux, const int* prow, int nq, int nent, int K, int k,
                               const int64_t* sent_ptr, const int64_t* sent_ids, int64_t* ids, float* scores,
                               hipStream_t s);
hipError_t launch_expand(const float* okey, const int* orow, int nq, int K, int k, const int64_t* sent_ptr,
                         const int64_t* sent_ids, int64_t* ids, float* scores, hipStream_t s);
hipError_t launch_sort_rows(float* keys, int* rows, int nq, int n, int n_pow2, hipStream_t s);
hipError_t launch_init_rows(const float* src, int64_t lds, int nq, int n, int n_pow2, float* keys, int* rows,
                            hipStream_t s);
hipError_t launch_gather_sentences(const float* rowkey, int64_t ldr, int nq, const int* row_of_sent, int64_t n_sent,
                                   float* out, hipStream_t s);
hipError_t launch_node_lp(const float* S_int, int64_t ldI, const float* S_leaf, int64_t ldL, int nq,
                          const int* node_src, const float* logdet_int, const float* logdet_row, float dconst,
                          int64_t n_nodes, float* out, hipStream_t s);
hipError_t launch_simulate(const SimArgs& a, hipStream_t s);
hipError_t launch_simulate_lazy(const SimArgs& a, hipStream_t s);
hipError_t launch_simulate_lazy_runs(const SimArgs& a, hipStream_t s);
// Categorize by counting (cat_count_kernel): resolves a query's pop sequence from the
// bottleneck order (status 0), or leaves it to the heap replay (status 2).
hipError_t launch_cat_count(const SimArgs& a, hipStream_t s);
hipError_t launch_welford_groups(const float* X, int D, const int64_t* order, const int64_t* gptr, int64_t n_groups,
                                 float* count, float* mean, float* meanSq, hipStream_t s);

// bf16-MFMA candidate filter (cwq_mfma.hip)
constexpr int kFgTile = 256;      // fgemm tile edge (queries and rows); operands are padded to it
constexpr int kFgCap = 512;       // candidate records per tile (LDS staging)
constexpr int kFgChunk = 2048;    // record slots a workgroup claims at a time
constexpr int kFgCapQ = 4096;     // candidate records per query
constexpr int kFinalWideMaxQ = 256;   // final_kernel: workgroup per query up to this many queries

// Per filter row (isotropic leaf-class row) constants, 32 B.
struct RowF {
  float R0;      // pretest row term on uniform tiles (-inf: never a candidate)
  float beta;    // |mu_lo| + gamma |mu_hi|
  float delta;   // |mu_hi| + |mu_lo|
  float rn2;     // |mu - c|^2
  float hs;      // -cw*iv/2
  float hl;      // -cw*logdet/2
  float invL;    // 1/path length
  int par;       // internal id of the parent (-1: none), -2: unusable row (no sentence / padding)
};
// Per row tile: "uniform" when every usable row shares parent, path length and g = cw*iv > 0.
// Row tile class for the filter pretest.  uniform 1: every row has parent `par`, the same
// depth (invL) and g; uniform 2: the same invL and g, parents in [par, par_hi] (BFS order
// keeps a tile's parents contiguous) -- the pretest takes the most permissive parent;
// 0: generic (per-element bounds).
struct TileF {
  int uniform;
  int par;
  float invL;
  float g;
  float beta_max, delta_max;
  int par_hi;
  float pad1;
};
constexpr int kFgMaxTileParents = 257;  // uniform 2 up to this many parents per tile (all: a tile has 256 rows)

// Rigorous bounds l <= key_fp32 <= u of an isotropic row's Fast key from an approximate
// bf16-MFMA dot product x_hi.mu_hi (error eextra on top of the bf16 split terms; see the
// cwq_mfma.hip header).  Shared by the fgemm filter and the small-batch stream filter.
// pi_u / pi_l: upper / lower bound of the parent-prefix term P[parent]/L (equal when the
// prefix is exact; internal-node bounds otherwise, cwq_mfma.hip int_bounds).
__device__ __forceinline__ void fg_bounds2(float dot, float eextra, float4 qi, const RowF& rf, float pi_u, float pi_l,
                                           float eps_n, float slack, float& u, float& l) {
  const float n2 = qi.x + rf.rn2;
  const float S = fmaf(-2.f, dot, n2);
  const float kr = fmaf(rf.hs, S, rf.hl);
  const float ES = 2.f * fmaf(qi.y, rf.beta, fmaf(qi.z, rf.delta, eextra)) + eps_n * n2;
  const float ahs = fabsf(rf.hs);
  const float err = fmaf(ahs, ES, slack * (fmaxf(fabsf(pi_u), fabsf(pi_l)) + fabsf(rf.hl) + 3.f * ahs * n2));
  u = (pi_u + kr) + err;
  l = (pi_l + kr) - err;
}
__device__ __forceinline__ void fg_bounds(float dot, float eextra, float4 qi, const RowF& rf, float pi, float eps_n,
                                          float slack, float& u, float& l) {
  fg_bounds2(dot, eextra, qi, rf, pi, pi, eps_n, slack, u, l);
}

// Element (query q, internal node p) of a prefix matrix: query-major [q][ld] (the exact
// pass) or node-major [p][ld] (pT: the path-sum bounds -- the filter's reads of one
// parent over a tile's queries and the tile ranges' reads are then coalesced).
__host__ __device__ __forceinline__ size_t pidx(int64_t ld, int pT, int64_t q, int64_t p) {
  return pT ? (size_t)(p * ld + q) : (size_t)(q * ld + p);
}

// Path-sum row (int_path_prep_kernel): bounds lo <= P_fp32(n) <= hi of the exact pass's
// path prefix from the MFMA dot a_hi.Bsum_hi and the exact root prefix proot.  RowF fields:
// rn2 = K0, beta/delta = Bsum's split norms, hs = Zq, R0 = Zc, hl = cr; qinfo {qx, |a_hi|,
// |a_lo|}.  2^-21 (|dot| + |K0| + |proot|) covers the dot's last rounding and the two fp32
// additions; (1 + 2^-20) the evaluation of E and the final subtractions.
__device__ __forceinline__ void path_bounds(float dot, float4 qi, const RowF& f, float proot, float& lo, float& hi) {
  const float s = proot + (f.rn2 + dot);
  const float ap = fabsf(proot);
  const float E = (fmaf(qi.y, f.beta, qi.z * f.delta) + fmaf(f.hs, qi.x, f.R0) + f.hl * ap +
                   0x1p-21f * (fabsf(dot) + fabsf(f.rn2) + ap)) *
                  (1.f + 0x1p-20f);
  lo = s - E;
  hi = s + E;
}

// Bounded path prefixes of the leaf parents (int_path, run_internal_bounds): the internal
// GEMM stores only its dot per (node, query), node-major [node][ld] -- node 0's line holds
// the root's exact prefix -- and every reader turns a dot into [lo, hi] with path_bounds
// (the per-query [x'^2, x'] norms qi2, the node's RowF nrf, indexed by internal id; par -2:
// a node with no operand row, i.e. no isotropic leaf row below it).  Half the bytes of
// storing lo and hi, bit-identical bounds.
struct PathB {
  const float* dot;     // [node][ld]; nullptr: not in use (the readers take P / Phi)
  int64_t ld;
  const float4* qi2;    // [nq]
  const RowF* nrf;      // [NI]
};
// f: node p's RowF (b.nrf[p]), loaded by the caller (hoisted out of per-query loops)
__device__ __forceinline__ void pathb_bounds_f(const PathB& b, int64_t q, int p, const RowF& f, float& lo,
                                               float& hi) {
  const float d = b.dot[(size_t)p * b.ld + q];
  if (p == 0) {   // the root: its exact prefix
    lo = hi = d;
    return;
  }
  if (f.par < -1) {   // no operand row: unbounded (never read for a parent of a filter row)
    lo = -__builtin_inff();
    hi = __builtin_inff();
    return;
  }
  path_bounds(d, b.qi2[q], f, b.dot[q], lo, hi);
}
__device__ __forceinline__ void pathb_bounds(const PathB& b, int64_t q, int p, float& lo, float& hi) {
  pathb_bounds_f(b, q, p, p > 0 ? b.nrf[p] : RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -1}, lo, hi);
}

struct FgArgs {
  int DPB, nq, n_qt, n_rt, nrows, mode;   // mode 0: filter (records), 1: sample (dense lower bounds),
                                          // 2: internal-node lp' bounds (dense lo/hi)
  int rt_off;                             // first row tile of this launch (filter phases)
  int all_uniform;                        // every row tile of the launch is uniform (TileF)
  int qgroups, rgroups;                   // XCD split (qgroups * rgroups == 8)
  int order;                              // tile order: 0 static q-fastest, 1 static r-fastest, 2 dynamic
  int* tctr;                              // order 2: per-XCD tile counters [8] (zeroed before the launch)
  int dbg;                                // ablation (perf experiments only): 1 no operand loads, 2 no epilogue
  int cat;                                // categorize key: bounds min'ed with P[q][par] (P = BF)
  int path_sum;                           // mode 2: rows are path sums (int_path_prep): bounds of the path
                                          // prefix P itself (path_bounds); 0: per-node lp' bounds
  const int* row_id;                      // mode 2: operand row -> internal node id (-1: padding)
  const float4* qinfo;                    // [nq_pad] {|x'|^2, |x_hi|, |x_lo|, -}
  const float* T;                         // thresholds, T[q * ldT]
  int64_t ldT;
  const RowF* rf;
  const TileF* tf;
  const float2* pmm;                      // multi-parent tiles: {min, max} parent prefix x invL, [tile][ldq]
  int64_t ldq;
  const int* rowmap;                      // sample pass: operand row -> filter row (-1 pad)
  const float* P;                         // [nq][ldP] path prefixes of internal nodes (lower bounds when Phi)
  const float* Phi;                       // [nq][ldP] upper bounds of the prefixes (NULL: P is exact)
  const float* BFt;                       // categorize with group-centred rows: the bottleneck table (P then
                                          // holds the rows' group terms); NULL: P is the bottleneck
  PathB pb;                               // path-sum bounds (pb.dot set: read instead of P / Phi)
  int64_t ldP;
  int pT;                                 // P / Phi (and mode-2 lb / lb_hi) node-major: [node][ldP] (pidx)
  float gamma, eps_n, slack;              // error-bound constants (cwq_mfma.hip header)
  float* lb;                              // sample: [nq_pad][ldlb]; internal bounds (mode 2): lp' lower bounds
  float* lb_hi;                           // internal bounds (mode 2): lp' upper bounds [nq][ldlb]
  const float* Sroot;                     // mode 2: exact raw sum of the root per query
  float root_w, root_ld;                  // mode 2: the root's level weight and logdet
  int64_t ldlb;
  int lbg;                                // sample: rows per lower-bound group (1 or 4)
  int4* rec;                              // filter: appended records {q, row, u, l}
  int64_t rec_cap;                        // record slots (a multiple of kFgChunk)
  int* gctr;                              // [0] chunks claimed, [1] direct records (zeroed before the launch)
  int4* rec_dir;                          // direct records (a tile with more than kFgCap)
  int dir_cap;
  int* chunk_fill;                        // valid records per claimed chunk
  int* qover;                             // queries whose records were lost (re-run exactly)
  unsigned long long* stamp;              // FG_STAMP diagnostic builds only: s_memtime stamps
};
// ---------------------------------------------------------------------------
// 64-lane lists (order: key desc, row asc), shared by the filter kernels
// ---------------------------------------------------------------------------
// whole-wave shift by one lane (lane i <- lane i-1; lane 0 keeps v): DPP wave_shr:1
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ float rl_f2(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ void list64_insert(float& lk, int& lr, int lane, float ck, int cr, int K) {
  const bool prec = lk > ck || (lk == ck && lr < cr);
  const int pos = __popcll(__ballot(prec));
  if (pos < K) {
    const float sk = __int_as_float(wave_shr1(__float_as_int(lk)));
    const int sr = wave_shr1(lr);
    if (lane == pos) {
      lk = ck;
      lr = cr;
    } else if (lane > pos) {
      lk = sk;
      lr = sr;
    }
  }
}

// Bitonic sort of one value per lane into a list64 list: descending by key, ascending row
// on equal keys (the list order list64_insert keeps), an aux value carried along.  21
// exchange steps instead of up to 64 serial inserts when a list is filled from empty.
// cat (AUX only): categorize lists order equal keys by the smaller aux (the row's own lp)
// first, then row -- list_before<true> (cwq_kernels.hip), so a list cut inside a tie at its
// last key keeps the rows that attain it.
template <bool AUX>
__device__ __forceinline__ void wave_sort64(float& k, int& r, float& a, int lane, bool cat = false) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int st = size >> 1; st > 0; st >>= 1) {
      const float pk = __shfl_xor(k, st, 64);
      const int pr = __shfl_xor(r, st, 64);
      const float pa = AUX ? __shfl_xor(a, st, 64) : 0.f;
      const bool hold_better = ((lane & st) == 0) == ((lane & size) == 0);
      const bool ca = AUX && cat && pa != a;
      const bool pbet = pk > k || (pk == k && (ca ? pa < a : pr < r));
      const bool obet = k > pk || (k == pk && (ca ? a < pa : r < pr));
      if (hold_better ? pbet : obet) {
        k = pk;
        r = pr;
        if (AUX) a = pa;
      }
    }
  }
}

// (key, aux, row) list order: key descending; equal keys by row, or for categorize lists
// (cat) by the smaller aux first, then row (list_before<true>, cwq_kernels.hip)
__device__ __forceinline__ bool entry_before(float k, float a, int r, float k2, float a2, int r2, bool cat) {
  return k > k2 || (k == k2 && (cat && a != a2 ? a < a2 : r < r2));
}

// float -> u32 whose unsigned order is the float order (NaN as -inf, -0 as +0: equal floats
// equal keys); 0 is below them all.  unord_f32 inverts it.
__device__ __forceinline__ unsigned ord_f32(float f) {
  const unsigned u = __float_as_uint(f == f ? (f == 0.f ? 0.f : f) : -__builtin_inff());
  return u ^ ((unsigned)((int)u >> 31) | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

// list64_insert with an aux value carried along (final_wide_kernel's (key, lp, row) lists)
__device__ __forceinline__ void list64_insert_aux(float& lk, float& la, int& lr, int lane, float ck, float ca, int cr,
                                                  int K, bool cat = false) {
  const bool prec = entry_before(lk, la, lr, ck, ca, cr, cat);
  const int pos = __popcll(__ballot(prec));
  if (pos < K) {
    const float sk = __int_as_float(wave_shr1(__float_as_int(lk)));
    const float sa = __int_as_float(wave_shr1(__float_as_int(la)));
    const int sr = wave_shr1(lr);
    if (lane == pos) {
      lk = ck;
      la = ca;
      lr = cr;
    } else if (lane > pos) {
      lk = sk;
      la = sa;
      lr = sr;
    }
  }
}

// The best 64 of this sorted list and another (lane i holds each list's i-th entry in
// entry_before order, lanes past a list's length invalid: key -inf, row INT_MAX): the other
// list reversed against this one keeps the better of each pair -- a bitonic sequence that
// holds the union's best 64 -- and six half-cleaner stages sort it.  Rows are distinct
// across the two lists, so the result's first K lanes are exactly what K serial
// list64_insert_aux calls would leave, in ~7 shuffle rounds instead of up to 64 inserts
// (categorize lists, whose ties make most entries enter; short Fast lists insert).
__device__ __forceinline__ void list64_merge_aux(float& lk, float& la, int& lr, int lane, float ok, float oa, int orow,
                                                 bool cat) {
  {
    const int rl = 63 - lane;
    const float rk = __shfl(ok, rl, 64), ra = __shfl(oa, rl, 64);
    const int rr = __shfl(orow, rl, 64);
    if (entry_before(rk, ra, rr, lk, la, lr, cat)) {
      lk = rk;
      la = ra;
      lr = rr;
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    const float pk = __shfl_xor(lk, s, 64), pa = __shfl_xor(la, s, 64);
    const int pr = __shfl_xor(lr, s, 64);
    const bool take = (lane & s) ? entry_before(lk, la, lr, pk, pa, pr, cat) : entry_before(pk, pa, pr, lk, la, lr, cat);
    if (take) {
      lk = pk;
      la = pa;
      lr = pr;
    }
  }
}

__device__ __forceinline__ void list64_offer(float& lk, int& lr, int lane, float key, int row, int K) {
  const float tk = rl_f2(lk, K - 1);
  const int tr = __builtin_amdgcn_readlane(lr, K - 1);
  const bool c = key != -__builtin_inff() && (key > tk || (key == tk && row < tr));
  uint64_t mask = __ballot(c);
  while (mask) {
    const int j = __builtin_ctzll(mask);
    mask &= mask - 1;
    list64_insert(lk, lr, lane, rl_f2(key, j), __builtin_amdgcn_readlane(row, j), K);
  }
}

// One wave: the top-Kp list (lk, lr) of the values uq[lo, hi) one by one (rows = indices);
// 8 chunks of 64 values in flight per round trip.
__device__ __forceinline__ void select_values_wave(const float* __restrict__ uq, int lo, int hi, int Kp, int lane,
                                                   float& lk, int& lr) {
  lk = -__builtin_inff();
  lr = 0x7fffffff;
  bool first = true;
  for (int r0 = lo; r0 < hi; r0 += 512) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int r = r0 + c * 64 + lane;
      v[c] = r < hi ? uq[r] : -__builtin_inff();
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int r = r0 + c * 64 + lane;
      if (r0 + c * 64 >= hi) break;
      const float x = v[c] == v[c] ? v[c] : -__builtin_inff();
      if (first) {
        lk = x;
        lr = x == -__builtin_inff() ? 0x7fffffff : r;
        float dummy = 0.f;
        wave_sort64<false>(lk, lr, dummy, lane);
        first = false;
      } else {
        list64_offer(lk, lr, lane, x, r, Kp);
      }
    }
  }
}

// One wave: the top-Kp list (lk, lr: lane i holds the i-th) of the per-lane maxima of up to
// 16 values of uq[0, nrows) -- the K-th largest of maxima over distinct rows is still a
// lower bound of the K-th largest value.  Reads whole 1024-value steps (the buffer carries
// >= 1024 floats of tail slack, masked here); g values per maximum, up to 16 while at
// least 8*Kp maxima remain.  select_kernel (cwq_mfma.hip) and the per-call stream filter's
// fused select (cwq_stream.hip) both run this, so their thresholds are identical.
__device__ __forceinline__ void select_wave(const float* __restrict__ uq, int nrows, int Kp, int lane, float& lk,
                                            int& lr) {
  lk = -__builtin_inff();
  lr = 0x7fffffff;
  constexpr int STEP = 1024;
  int g = 16;
  while (g > 1 && nrows / g < 8 * Kp) g >>= 1;
  for (int r0 = 0; r0 < nrows; r0 += STEP) {
    float4 v4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v4[t] = *reinterpret_cast<const float4*>(uq + r0 + t * 256 + lane * 4);
    float m = -__builtin_inff();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float vv[4] = {v4[t].x, v4[t].y, v4[t].z, v4[t].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = r0 + t * 256 + lane * 4 + c;
        m = fmaxf(m, r < nrows ? vv[c] : -__builtin_inff());
        if (((t * 4 + c + 1) & (g - 1)) == 0) {
          if (r0 == 0 && t * 4 + c + 1 == g) {   // the empty list: sort the first maxima
            lk = m;
            lr = m == -__builtin_inff() ? 0x7fffffff : r;
            float dummy = 0.f;
            wave_sort64<false>(lk, lr, dummy, lane);
          } else {
            list64_offer(lk, lr, lane, m, r, Kp);
          }
          m = -__builtin_inff();
        }
      }
    }
  }
}

// Small-batch stream filter (cwq_stream.hip): nq <= kStreamMaxQ queries per launch
constexpr int kStreamMaxQ = 64;
// small-batch prep (launch_sb_prep): pad + query prep + exact internal pass + counter clear
constexpr int kSbMaxNI = 64;
struct SbPrepArgs {
  const float* q;       // [nq][D] caller queries
  int nq, D, DP, DPB;
  int64_t nq_pad, nq16;
  float* X;             // scan layout, nq_pad rows
  void* Xb;             // bf16 hi parts [nq16][DPB]
  float4* qinfo;        // [nq16]
  void* Xq;             // int8 parts [nq16][DPB] of the stream filter's int8 pass (NULL: none)
  float4* qinfo8;       // [nq16] {|x'|^2, |x_hi8|, |x_lo8|, scale}
  const float* c;       // centre (root mean)
  const float *A, *B;   // internal nodes, dim-major [DP][ld]
  int64_t ld;
  int NI;
  const int* par_int;
  const float *w_int, *logdet_int;
  float* P;             // [nq][ldP] exact prefixes
  int64_t ldP;
  int* qcnt;            // [5][nq] counters to clear
  int nlev;
  int lv0[kSbMaxNI + 1];   // level ranges [lv0[l], lv0[l+1])
};
hipError_t launch_sb_prep(const SbPrepArgs& a, hipStream_t s);
constexpr int kStreamMaxLds = 160 * 1024;
constexpr int kStreamChunk = 8;   // K fragments (of 32 dims) per stream-kernel load chunk
// query fragments in LDS, K padded with zero fragments to whole chunks
constexpr int kStreamSlots = 32;   // filter: candidate slots per query in each workgroup's LDS buffer
inline size_t stream_lds_bytes(int nqb, int DPB, bool i8 = false, bool cand = false) {
  const int nk = DPB / (i8 ? 64 : 32);   // 16-B fragments per row: 32 bf16 / 64 int8 dims
  return (size_t)nqb * ((nk + kStreamChunk - 1) / kStreamChunk * kStreamChunk) * 64 * 16 +
         (cand ? (size_t)nqb * 16 * (2 + 3 * kStreamSlots) * 4 : 0);
}
// int8 operands of the stream filter pass (built on the first small-batch call, launch_rows_i8):
// per row r, s_r = max_d |mu'_d| / 127, q = rint(mu' / s_r) (int8, DPB wide, zero padded),
// RowF = iso_rf[r] with beta = |mu' - s_r q|, delta = |s_r q| + beta and R0 = s_r.  The
// products are exact (int32 sums), so the bound has no accumulation term (gamma = 0).
hipError_t launch_rows_i8(const float* Mf, int DP, int D, const float* c, int DPB, int64_t ld, const RowF* rf,
                          void* Mq, RowF* rf8, hipStream_t s);
// queries likewise: Xq [nq16][DPB], qinfo8 {|x'|^2, |x_hi|, |x_lo|, s_x}
hipError_t launch_query_prep_i8(const float* q, int64_t nq, int D, const float* c, int DPB, int64_t nq16, void* Xq,
                                float4* qinfo8, hipStream_t s);
struct StreamArgs {
  int DPB, nq, nqb;            // queries, 16-query blocks (nqb * 16 >= nq)
  int64_t nrows;               // isotropic filter rows
  int K;                       // top-K width = threshold blocks
  int64_t n_probe;             // probe: 16-row groups sampled
  int64_t probe_stride;        // probe: group stride
  float* lb;                   // probe: [nq][ldlb] per-group max lower bound
  int64_t ldlb;
  const float* T0;             // filter: initial threshold T0[q * ldT0 + K - 1] (select over lb)
  int64_t ldT0;
  int i8;                      // filter: int8 operands (Xb, Mb int8; qinfo.w, rf.R0 the scales)
  int slots;                   // filter: LDS candidate slots per query (set by launch_stream)
  const uint16_t* Xb;          // [>= nqb*16][DPB] bf16 hi of the centred queries
  const float4* qinfo;         // [>= nqb*16]
  const uint16_t* Mb;          // [ld_f][DPB] bf16 row panel
  const RowF* rf;              // [ld_f]
  const float* P;              // [nq][ldP] internal-node path prefixes (lower bounds when Phi)
  const float* Phi;            // [nq][ldP] upper bounds (NULL: P exact)
  PathB pb;                    // path-sum bounds (pb.dot set: read instead of P / Phi)
  int64_t ldP;
  int pT;                      // node-major P / Phi (pidx)
  float eps_n, slack;
  int* Tb;                     // [K][nq] ordered-int block maxima of candidate lower bounds (filter)
  int* Tlive;                  // [nq] ordered-int live threshold (= Tb + K * nq)
  int live_every;              // filter: raise T to Tlive every this many groups (0: off)
  float* T;                    // [nq] initial threshold (written by the filter launch, read by final_kernel)
  // MODE 2 (path-sum dots): operand row -> internal id, the root's exact raw sum and terms,
  // output lines [internal id][ldpout]
  const int* row_id;
  const float* Sroot;
  float root_w, root_ld;
  float* pout;
  int64_t ldpout;
  int* qcnt;                   // [nq] candidates per query
  int* qover;                  // [nq] list overflow
  int capq;                    // candidate slots per query
  int* crow;                   // [nq][capq]
  float* cu;
  float* cl;
  // probe with the select fused (sel_ctr set, zero at launch): the last workgroup to finish
  // runs select_wave over lb and writes the top-K lists [nq][64] (sel_lk, sel_lr), as
  // select_kernel does, then clears sel_ctr
  int* sel_ctr;
  float* sel_lk;
  int* sel_lr;
  const float* sel_floor;      // optional [nq]: the K-th entry written is max(it, floor) (group pruning's seed)
  // categorize (cwq_categorize's per-call lists): the key is min(BFk[q][parent], lp) -- both
  // bounds are min'ed with it (BFk: the path bottleneck BF, or the second-level T2); rf are
  // then the categorize RowF (cat_rf) and P / Phi its group-term tables
  const float* BFk;
  int64_t ldBF;
  // probe (MODE 1): every probed row's lower bound to lb[q][g * 16 + row] instead of the
  // group's maximum, and the fused select takes them one by one (all waves of the last
  // workgroup per query): categorize's lists (R = 64) cluster in a few 16-row blocks, where
  // group maxima leave the threshold far below the R-th key
  int probe_rows;
  // filter pass (MODE 0) over a list of 16-row blocks instead of all of them: live[0..*live_n)
  // (group pruning: the blocks whose rows are all in groups pruned for every query of the call
  // are left out, prune_stage_b_kernel)
  const int* live;
  const int* live_n;
  // probe with the query prep fused (flat trees, nq <= 16, bf16; fprep set): every workgroup
  // forms the bf16 query fragments, the {|x'|^2, |x_hi|, |x_lo|} terms and the root's exact
  // prefix itself (sb_prep_kernel's arithmetic), and workgroup 0 also writes them to Xb /
  // qinfo / P with the scan-layout X and the cleared counters for the launches after it
  int fprep;
  const float* fq;             // [nq][D] caller queries
  const float* fc;             // centre
  int fD, fDP;
  int64_t f_nq_pad;
  float* fX;                   // scan layout, f_nq_pad rows
  const float *fA, *fB;        // root row of the internal arrays, dim-major [DP][fld]
  int64_t fld;
  float fw0, flogdet0;         // root w and logdet
  float* fP;                   // [nq][fldP] root prefix (column 0)
  int64_t fldP;
  int* fqcnt;                  // [5][nq] counters to clear
};
hipError_t launch_stream(const StreamArgs& a, int mode, int n_wg, hipStream_t s);   // 0 filter, 1 probe, 2 path dots
hipError_t launch_stream_init(int* Tb, int n, hipStream_t s);

hipError_t launch_rows_prep(const float* mean, int D, const int64_t* nodes, int64_t n, const float* c, int DP,
                            int DPB, int64_t ld, float* Mf, void* Mb, float* n2, float* nlo, float* nhi,
                            hipStream_t s, const float* cent = nullptr, const int* grp = nullptr, float* nm = nullptr);
// Group-centred filter rows (cwq_group.hip)
hipError_t launch_gather_rows_f32(const float* mean, int D, const int64_t* nodes, int64_t n, float* out,
                                  hipStream_t s);
hipError_t launch_group_anc_dist(const float* mean, int D, const int64_t* rows, int64_t n, const float* c0,
                                 const int* rpar, const int* par_int, const int* idep, const int64_t* int_nodes,
                                 int maxd, double* out, hipStream_t s);
hipError_t launch_group_norms(const float* mean, int D, const int64_t* nodes, int64_t n, const float* c0,
                              const float* cent, const int* grp, double* root2, double* grp2, hipStream_t s);
// sh [2][nq][G]: -2 x'.d_g and its error bound; dist2 (optional) [nq][G]: |x - c_g|^2 in fp64
hipError_t launch_group_shift(const float* q, int nq, int D, const float* c0, const float* cent, int G, double* sh,
                              double* dist2, hipStream_t s);
hipError_t launch_group_prefixes(const float* q, int nq, int D, const float* c0, const float* cent, int G,
                                 const float* P, int64_t ldP, int NI, const int* grp, const double* F, const double* Fc,
                                 double* sh, float* Plo, float* Phi, float* Pclo, float* Pchi, hipStream_t s);
hipError_t launch_gather_bf16_rows(const void* Mb, int DPB, const int* srow, int64_t n, void* Sb, hipStream_t s);
hipError_t launch_query_prep(const float* q, int64_t nq, int D, const float* c, int DPB, int64_t nq_pad, void* Xb,
                             float4* qinfo, hipStream_t s, int* zero = nullptr, int nzero = 0);
hipError_t launch_fgemm(const void* Xb, const void* Mb, const FgArgs& a, int n_wg, hipStream_t s);
int fgemm_dpb(int D);   // padded bf16 operand width the fgemm build needs
hipError_t launch_select(const float* u, int64_t ldu, int nq, int nrows, int Kp, float* cu, int* crow, hipStream_t s);
// Internal-node bound operands (hierarchical trees): for internal node i (ids [0, n)),
// b' = [-w/2, mu'w] (w = A^2, A = 1/sqrtf(var), mu' = mean - c) as bf16 hi [ld][DPB2],
// its RowF {R0 = M_n, beta, delta, rn2 = c_n, hs = wmax, hl = logdet, invL = level weight
// w_int, par = parent internal id (-1 root, -2 padding)}, and row-major
// fp32 copies Ar = A, Br = mean * A (bit-identical to the exact scan's int_A / int_B).
hipError_t launch_int_prep(const float* mean, const VarSrc& var, int D, const int64_t* nodes, int64_t n,
                           const float* c, const float* logdet, const int* par_int, const float* w_int, int DP, int DPB2,
                           int64_t ld, void* Mb2, RowF* rf, float* Ar, float* Br, float gamma, hipStream_t s);
// Path-sum operands (the Fast filter's leaf parents): for internal node i = rows[r] (the
// root: an exact row, par -1), Bsum = sum over the path's non-root nodes a of w_a b'_a as
// bf16 hi [ld][DPB2] and RowF {R0 = Zc, beta, delta, rn2 = K0, hs = Zq, hl = cr, invL 0,
// par} for path_bounds (cwq_mfma.hip); padding rows par -2.  nodes: node id per internal id.
hipError_t launch_int_path_prep(const float* mean, const VarSrc& var, int D, const int64_t* nodes, const int* rows,
                                int64_t n, const float* c, const float* logdet, const int* par_int,
                                const float* w_int, int DP, int DPB2, int64_t ld, void* Mb2, RowF* rf, float gamma,
                                hipStream_t s);
// Queries for the internal bounds: a = [x'^2, x'] bf16 hi [nq_pad][DPB2], qinfo =
// {sum x^2 + sum x'^2, |a_hi|, |a_lo|, 0}.
hipError_t launch_query_prep2(const float* q, int64_t nq, int D, const float* c, int DP, int DPB2, int64_t nq_pad,
                              void* Xb2, float4* qinfo, hipStream_t s);
// P bounds level by level: lp' bounds (Plo, Phi) -> prefix bounds in place; the root
// level (i0 == 0, one node) from its exact raw sum Sroot[q].
hipError_t launch_prefix_bounds(float* Plo, float* Phi, int64_t ldP, int nq, int i0, int i1, const int* par_int,
                                const float* w_int, const float* logdet_int, const float* Sroot, hipStream_t s);
// Exact internal-node chain for final_kernel (bounded prefixes): P of a parent recomputed
// with the scan's arithmetic from the exact root prefix P[q][0].
constexpr int kMaxChain = 64;   // deepest internal-node chain final_kernel recomputes (host checks max depth)
struct IntChain {
  const float* Ar;
  const float* Br;
  const int* par_int;
  const float* w_int;
  const float* logdet_int;
};
hipError_t launch_pathb_expand(const PathB& pb, int nq, int NI, float* lo, float* hi, hipStream_t s);
hipError_t launch_tile_prange(const float* P, const float* Phi, int64_t ldP, int pT, int nq, const TileF* tf,
                              int n_rt, float2* pmm, int64_t ldq, hipStream_t s, const PathB* pb = nullptr);
hipError_t launch_bucket(const int4* rec, const int* gctr, const int* chunk_fill, int64_t rec_cap, const int4* rec_dir,
                         int dir_cap, int capq, int* qcnt, int* qover, int* crow, float* cu, float* cl, hipStream_t s);
// lkb/lrb [nq][64] and done [nq] carry each query's top-K candidate lower bounds between
// the tighten calls and into final (done must start at 0); zero16[0..15] is cleared
// (the filter's record and tile-claim counters for the next launch)
hipError_t launch_tighten(int nq, int K, int capq, const int* qcnt, const int* qover, const float* cl, float* T,
                          int64_t ldT, float* lkb, int* lrb, int* done, int* zero16, hipStream_t s);
// Fused tail of the per-call path (final_wide_kernel, one candidate list per query): the
// top-K rows expanded to sentence ids into ids/scores (merge_expand_kernel's work) and the
// per-query {candidates, ok, exact reranks} written to hflags[0..3nq) (host-mapped).
struct FwExpand {
  const int64_t* sent_ptr;
  const int64_t* sent_ids;
  int64_t* ids;
  float* scores;
  int k;
  int* hflags;
  // split > 1: `split` workgroups per query, each reranking its own slice of the candidate
  // list into a top-K list in sk/sa/sr ([nq][split][64]); the last to finish (arrival count
  // in sctr[q], or with sctr null the call's zeroed ok_flag[q]; exact reranks summed in the
  // zeroed n_exact[q]) merges, then expands (ids) or writes the list (no ids)
  int split;
  float* sk;
  float* sa;
  int* sr;
  int* sctr;
};
size_t final_wide_lds(int DP, int capq);   // dynamic LDS of final_wide_kernel (SIZE_MAX: cannot run)
int final_wide_rows(int DP, int capq);     // survivors per rerank round
hipError_t launch_final(const float* X, const float* Mf, int DP, int nq, int K, int capq, const int* qcnt,
                        const int* qover, const int* crow, const float* cu, const float* cl, const float* T,
                        int64_t ldT, const RowMeta* meta, const int* par, const float* P, int64_t ldP, int seg_base,
                        float* pkey, float* paux, int* prow, int64_t lstride, int* ok_flag, int* n_exact,
                        const float* lkb, const int* lrb, const int* done, const IntChain* chain, int cat,
                        float dconst, hipStream_t s, const FwExpand* fx = nullptr);

// PCA + ICA whitening (cwq_whiten.hip): C[m][n] = sum_k (A[m][k] - ctr[k]) B[n][k] (/ denom[n])
hipError_t launch_gemm_nt_f32(const float* A, int64_t M, int K, const float* ctr, const float* B, int N,
                              const float* denom, float* C, hipStream_t s);

}  // namespace cwq
