// libcwq C ABI: index construction and query orchestration (host side).
// Public contract: include/cobweb_query.h.  Kernels: cwq_kernels.hip.
//
// Index layout in HBM:
//   internal nodes (nodes with children), BFS order:     A = 1/sigma, B = mu/sigma  [DP][ld_int]
//   leaf-class rows (childless nodes + internal nodes that hold sentences),
//     isotropic rows first (var identical across d):    M = mu                      [DP][ld_iso]
//     then anisotropic rows:                            A = 1/sigma, B = mu/sigma   [DP][ld_an]
//   dim-major ("transposed") so a wave's 64 lanes = 64 consecutive rows read one
//   coalesced 256-B line per dimension.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cobweb_query.h"
#include "cwq_internal.h"

using namespace cwq;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess) return fail(CWQ_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Bump allocator over the handle's workspace.
struct Bump {
  char* base;
  size_t off = 0, cap;
  Bump(void* b, size_t c) : base((char*)b), cap(c) {}
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = (T*)(base + off);
    off += n * sizeof(T);
    return p;
  }
};

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace

struct cwq_index {
  int device = 0;
  int64_t n_nodes = 0, n_sent = 0;
  int D = 0, DP = 0;
  int NI = 0, NL = 0, NL_iso = 0, NL_an = 0;
  int64_t ld_int = 0, ld_iso = 0, ld_an = 0;
  int max_depth = 0;
  int cus = 256;
  std::vector<std::pair<int, int>> levels;   // internal-node ranges, one per depth
  int* d_lv = nullptr;                       // device copy: level starts + end [levels + 1]
  int* sel_ctr = nullptr;                    // per-call path: fused select counter (probe with fused prep)
  float root_w0 = 0.f, root_logdet0 = 0.f;   // the root's w and logdet (host copies)
  std::vector<void*> allocs;
  size_t bytes = 0;
  // row data
  float *int_A = nullptr, *int_B = nullptr, *iso_M = nullptr, *an_A = nullptr, *an_B = nullptr;
  RowMeta* row_meta = nullptr;
  int *row_par = nullptr, *row_flags = nullptr, *row_bfs = nullptr;
  float* logdet_row = nullptr;
  float *logdet_int = nullptr, *w_int = nullptr;
  int *par_int = nullptr, *int_child_begin = nullptr, *int_child_end = nullptr, *int_nchild = nullptr;
  int *int_bfs = nullptr, *int_has_sent = nullptr;
  bool any_int_sent = false;   // an internal node holds sentences (categorize: heap replay only)
  int *int_leaf_a0 = nullptr, *int_leaf_a1 = nullptr, *int_leaf_b0 = nullptr, *int_leaf_b1 = nullptr;
  int64_t *sent_ptr = nullptr, *sent_ids = nullptr;
  int* row_of_sent = nullptr;
  int* node_src = nullptr;
  float* dummy = nullptr;
  // bf16-MFMA filter operands for the isotropic rows (cwq_mfma.hip): row-major
  // fp32 (exact rerank, DP wide) and bf16 hi-part (GEMM, DPB wide) copies padded to
  // whole 256-row tiles, per-row / per-tile bound constants, the threshold sample
  int64_t ld_f = 0;
  int DPB = 0;
  float *iso_Mf = nullptr, *iso_c = nullptr;   // iso_c: centre [D] (root mean)
  uint16_t* iso_Mb = nullptr;
  RowF* iso_rf = nullptr;
  TileF* iso_tf = nullptr;
  // int8 operands of the stream filter pass (launch_rows_i8), built on the first small-batch
  // call: 0 not yet, 1 built, -1 off (CWQ_STREAM_I8=0, DPB % 64, or too little free memory)
  int8_t* iso_Mq = nullptr;
  RowF* iso_rf8 = nullptr;
  int i8_state = 0;
  std::vector<int> tile_uni_prefix;   // prefix counts of uniform row tiles (all_uniform per launch range)
  int n_multi_tiles = 0;              // tiles with several parents (TileF uniform 2)
  // the same tables for the categorize key min(BF[parent], lp) (cwq_categorize through the
  // filter): lp with the 2*pi constant, no prefix term (invL 0), the categorize usable rule
  RowF* cat_rf = nullptr;
  TileF* cat_tf = nullptr;
  std::vector<int> cat_uni_prefix;
  float cat_dconst = 0.f;
  int n_samp = 0, ld_s = 0;                    // sample rows, padded to 256
  // group-centred filter rows (cwq_group.hip; clustered trees): the isotropic rows below a
  // depth-1 internal node g are centred at its mean grp_c[g]; grp_par[p] = the group of
  // internal node p's rows (-1: root-centred), grp_F[p] = hs / invL of p's rows (Fast),
  // grp_Fc[p] = their categorize hs.  grp_mode: the filters read the shifted prefix tables.
  bool grp_mode = false;
  int G = 0;
  int64_t n_grp_rows = 0;
  // the cut plan_groups chose (host copies, build_prune reads them): the group of every
  // internal node (-1: a top node -- the root and the ancestors of the group centres, which
  // every query computes exactly), each group's centre (internal id) and whether its rows are
  // centred there (grp_ok; a group that fails the centring rule is still a pruning group)
  std::vector<int> cut_gint, cut_centre;
  std::vector<char> cut_ok;
  int cut_maxdep = 0, cut_top = 0;   // deepest centre, number of top nodes (filter_info)
  float* grp_c = nullptr;
  int* grp_par = nullptr;
  double *grp_F = nullptr, *grp_Fc = nullptr;
  // group pruning of the Fast query (cwq_prune.hip; group-centred trees with every level
  // weight >= 0): the pruning group of each internal node, group-major internal node lists,
  // per-group bound constants.  prune_ctr: the last call's stage-B pair count (diagnostics).
  bool prune_ok = false;
  int *prn_gint = nullptr, *gi_ptr = nullptr, *gi_nodes = nullptr;
  // top nodes in BFS order (root first) with their parents' list positions and depths; per
  // group the list position of its centre's parent (a top node)
  int *top_nodes = nullptr, *top_ppos = nullptr, *top_dep = nullptr, *grp_tpos = nullptr;
  int n_top = 0, top_maxdep = 0;
  // auto mode's record of the filter on this index: queries filtered / re-run exactly; when
  // at least 9 in 10 of >= 256 queries had to be re-run (the bounds too loose for this
  // tree's rows), auto mode takes the exact scan from then on (same results, less work)
  int64_t filt_q = 0, filt_fb = 0;
  bool filt_auto_off = false;
  int filt_off_calls = 0;   // auto-mode Fast calls on the exact scan since the filter went off
  // categorize: the last call's queries all went to the two-level replay, so the next call
  // launches the second list with the first replay (gated on its status) instead of after
  // reading that status back (categorize_impl)
  bool cat_two_spec = false;
  bool cat_tail_done = false;   // categorize_impl: the node tails are cleared, nothing runs after its last sync
  // categorize, calls of <= 64 queries: the list paths, or straight to the exact lazy replay
  // (simulate_lazy_runs_kernel; categorize_impl's path choice).  The choice is measured: per-query
  // wall time of each path (EMA), the faster one taken, the other tried every kCatExplore calls
  // -- but the lazy path is only ever tried while the list paths recently left queries to the
  // DENSE re-run (cat_dense_seen: ties nested deeper than the two-level replay certifies; a
  // tree the lists resolve, C2's or a flat one, never pays for the trial).  lazy_stats: the last
  // call's queries replayed lazily straight away / after the list paths (cwq_last_lazy_stats)
  // [0]: calls of <= 64 queries, [1]: batches (tried on any tree whose widest node fits the
  // replay's arena, max_fanout <= kLzFanout: the lazy replays of a batch run side by side)
  double cat_ema_list[2] = {-1.0, -1.0}, cat_ema_direct[2] = {-1.0, -1.0};
  int cat_dense_seen = 0, cat_pol_calls[2] = {0, 0};
  bool cat_pref_direct[2] = {false, false};
  int max_fanout = 0;   // the most children (internal + leaf rows) of one internal node
  int64_t lazy_stats[2] = {0, 0};
  // categorize: calls since the counting pass last resolved a query (after 8 such calls
  // cat_count_kernel is skipped -- every query then goes to the replay anyway -- and tried
  // again every kCatCountRetry calls)
  int cat_count_idle = 0;
  int prn_gmax = 1;   // the most internal nodes of one pruning group
  int prn_maxdep = 0, prn_mindep = 1;   // deepest / shallowest internal node of any group
  int *gi_dep = nullptr, *gi_ppos = nullptr;   // per group-list entry: depth, the parent's list position
  int* blk_grp = nullptr;   // per 16-row block of isotropic rows: the pruning group of all its rows (-1: mixed)
  int *gs_ptr = nullptr, *gs_rows = nullptr;   // per group: up to 64 usable isotropic rows (the seed threshold)
  GroupBound* gbound = nullptr;
  int* prune_ctr = nullptr;     // device [8]: per chunk pair count + claim counters, [4] the call's pair total
  int64_t prune_nq = 0;         // queries the last Fast call pruned (0: none)
  // internal-node bounds (hierarchical trees): bf16 operand rows, their RowF constants,
  // row-major fp32 A/B copies for the exact chain in final_kernel.  int_path (default):
  // the Fast filter reads the path prefix P of leaf parents only, so there is one row per
  // leaf parent (and the root), its b' vectors summed along the path (cwq_mfma.hip
  // int_path_prep) -- one GEMM, no prefix passes.  Otherwise (CWQ_INT_PATH=0 at index
  // creation) one row per internal node, levels 0-1 together and each deeper level from
  // a new 256-row tile, then prefix_bounds_kernel level by level.
  bool int_bounds = false;
  bool int_path = true;
  int DPB2 = 0;
  int64_t ld_i2 = 0;                  // operand rows (padded to 256)
  uint16_t* int_Mb2 = nullptr;
  RowF* int_rf2 = nullptr;
  int* int_rowid = nullptr;           // operand row -> internal id (-1: padding)
  RowF* int_nrf = nullptr;            // int_path: int_rf2 by internal id (par -2: no operand row), PathB
  float *int_Ar = nullptr, *int_Br = nullptr;
  float root_w = 1.f, root_ld = 0.f;   // the root's level weight and logdet (host copies)
  int* samp_rows = nullptr;
  uint16_t* iso_Sb = nullptr;
  int64_t stats[6] = {0, 0, 0, 0, 0, 0};   // cwq_last_stats
  // timing (cwq_set_timing)
  bool timing = false;
  int filter = -1;   // cwq_set_filter
  int n_fg_launch = 0;   // filter launches of the last chunk (timing report)
  hipEvent_t ev[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  float t_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // workspace.  Every query call carves its buffers from `ws`; the call's kernels may
  // still be running when it returns, so the end of each call records `ws_ev` on its
  // stream and the next call makes its own stream wait for it (ws_begin / ws_end):
  // calls on different streams reuse the workspace in order.
  std::mutex mu;
  void* ws = nullptr;
  size_t ws_size = 0;
  size_t ws_budget = 0;   // query-chunk workspace budget, from the free memory at the first call
  hipEvent_t ws_ev = nullptr;
  bool ws_ev_live = false;
  bool ws_idle = false;   // set by a call that ends with its stream synchronized: no event needed
  int* hflags = nullptr;   // pinned host copy of the per-query filter flags (one D2H per chunk)
  size_t hflags_n = 0;
  // cwq_score_topk_host: pinned staging of the host queries, their device copy, and mapped
  // (coherent) host memory the kernels write the results into
  void* hq = nullptr;
  void* dq = nullptr;
  size_t hq_n = 0;
  void* hout = nullptr;
  size_t hout_n = 0;
  // fallback re-runs (cwq_score_topk / cwq_categorize): gathered queries, their results
  // and the device index lists, kept between calls (grown on demand)
  void* fb = nullptr;
  size_t fb_size = 0;
  void* fb2 = nullptr;    // categorize's filter fallback (its exact re-run uses fb itself)
  size_t fb2_size = 0;

  template <class T>
  int alloc(T** p, size_t n) {
    void* q = nullptr;
    const size_t b = std::max<size_t>(n, 1) * sizeof(T);
    if (hipMalloc(&q, b) != hipSuccess) return fail(CWQ_ERR_OOM, "hipMalloc failed (" + std::to_string(b) + " B)");
    allocs.push_back(q);
    bytes += b;
    *p = (T*)q;
    return CWQ_OK;
  }
  template <class T>
  int upload(T** p, const std::vector<T>& v, hipStream_t s) {
    int rc = alloc(p, v.size());
    if (rc) return rc;
    if (!v.empty()) HIPCHK(hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return CWQ_OK;
  }
  int reserve(size_t b) {
    if (b <= ws_size) return CWQ_OK;
    if (ws_ev_live) (void)hipEventSynchronize(ws_ev);   // earlier calls' kernels may still read it
    if (ws) (void)hipFree(ws);
    ws = nullptr;
    ws_size = 0;
    b = round_up((int64_t)b, 1 << 20);
    if (hipMalloc(&ws, b) != hipSuccess) return fail(CWQ_ERR_OOM, "workspace hipMalloc failed (" + std::to_string(b) + " B)");
    ws_size = b;
    return CWQ_OK;
  }
  int reserve_fb(size_t b) {
    if (b <= fb_size) return CWQ_OK;
    if (ws_ev_live) (void)hipEventSynchronize(ws_ev);
    if (fb) (void)hipFree(fb);
    fb = nullptr;
    fb_size = 0;
    b = round_up((int64_t)b, 1 << 20);
    if (hipMalloc(&fb, b) != hipSuccess) return fail(CWQ_ERR_OOM, "fallback hipMalloc failed (" + std::to_string(b) + " B)");
    fb_size = b;
    return CWQ_OK;
  }
  // start of a query call on stream s: wait for the previous call's use of the workspace
  int ws_begin(hipStream_t s) {
    if (!ws_ev && hipEventCreateWithFlags(&ws_ev, hipEventDisableTiming) != hipSuccess)
      return fail(CWQ_ERR_HIP, "hipEventCreate failed");
    // always wait, also on the previous call's stream handle: a destroyed stream's handle
    // can come back as a new stream.  The per-call path ends synchronized (ws_idle), so
    // it leaves no live event and queues no barrier packet here.
    if (ws_ev_live && hipStreamWaitEvent(s, ws_ev, 0) != hipSuccess)
      return fail(CWQ_ERR_HIP, "hipStreamWaitEvent failed");
    return CWQ_OK;
  }
  // end of a query call: the workspace is busy until the work queued on s so far is done
  int ws_end(hipStream_t s) {
    if (!ws_ev) return fail(CWQ_ERR_HIP, "workspace event missing");
    if (ws_idle) {   // every kernel of the call has finished: the workspace is free now
      ws_idle = false;
      ws_ev_live = false;
      return CWQ_OK;
    }
    if (hipEventRecord(ws_ev, s) != hipSuccess) {
      // the event no longer marks this call's work: wait for it here instead
      ws_ev_live = false;
      (void)hipStreamSynchronize(s);
      return fail(CWQ_ERR_HIP, "hipEventRecord failed");
    }
    ws_ev_live = true;
    return CWQ_OK;
  }
  ~cwq_index() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    if (ws_ev_live) (void)hipEventSynchronize(ws_ev);
    if (ws_ev) (void)hipEventDestroy(ws_ev);
    for (void* p : allocs) (void)hipFree(p);
    if (ws) (void)hipFree(ws);
    if (fb) (void)hipFree(fb);
    if (fb2) (void)hipFree(fb2);
    if (hflags) (void)hipHostFree(hflags);
    if (hq) (void)hipHostFree(hq);
    if (dq) (void)hipFree(dq);
    if (hout) (void)hipHostFree(hout);
  }
  int host_io(size_t qbytes, size_t obytes) {
    if (qbytes > hq_n) {
      if (hq) (void)hipHostFree(hq);
      if (dq) (void)hipFree(dq);
      hq = dq = nullptr;
      hq_n = 0;
      const size_t b = (size_t)round_up((int64_t)qbytes, 1 << 16);
      if (hipHostMalloc(&hq, b, hipHostMallocDefault) != hipSuccess || hipMalloc(&dq, b) != hipSuccess)
        return fail(CWQ_ERR_OOM, "host query staging allocation failed");
      hq_n = b;
    }
    if (obytes > hout_n) {
      if (hout) (void)hipHostFree(hout);
      hout = nullptr;
      hout_n = 0;
      const size_t b = (size_t)round_up((int64_t)obytes, 1 << 16);
      if (hipHostMalloc(&hout, b, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return fail(CWQ_ERR_OOM, "host result buffer allocation failed");
      hout_n = b;
    }
    return CWQ_OK;
  }
  int host_flags(size_t n) {
    if (n <= hflags_n) return CWQ_OK;
    if (hflags) (void)hipHostFree(hflags);
    hflags = nullptr;
    hflags_n = 0;
    // coherent (fine-grained) host memory: final_wide_kernel writes the flags of the
    // per-call path straight into it; the batch paths copy into it
    if (hipHostMalloc((void**)&hflags, n * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(CWQ_ERR_OOM, "hipHostMalloc failed");
    hflags_n = n;
    return CWQ_OK;
  }
};

// RAII: a query entry point's use of the handle workspace on stream s (cwq_index::ws_begin)
struct WsUse {
  cwq_index* ix;
  hipStream_t s;
  int rc;
  WsUse(cwq_index* i, hipStream_t st) : ix(i), s(st) {
    rc = ix->ws_begin(s);
  }
  ~WsUse() {
    if (rc == CWQ_OK) (void)ix->ws_end(s);   // ws_begin failed: nothing was queued on s
  }
};

#ifndef CWQ_BUILD_ID
#define CWQ_BUILD_ID "unversioned"
#endif
extern "C" int cwq_version(void) { return 200; }
// "CWQ_BUILD_ID=<id>" is also searched for in the file by build.py (no dlopen needed)
static const char kBuildId[] = "CWQ_BUILD_ID=" CWQ_BUILD_ID;
extern "C" const char* cwq_build_id(void) { return kBuildId + 13; }
extern "C" const char* cwq_last_error(void) { return g_err.c_str(); }

namespace {

// Error-bound constants of the filter (cwq_mfma.hip header): fp32 accumulation of the
// MFMA products (2x the textbook (n-1)u, n = DPB + 64), norm/centring rounding, and the
// relative slack that covers the fp32 evaluation of both the bounds and the exact keys.
struct FiltConsts {
  double gamma, eps_n, slack;
};
FiltConsts filt_consts(int DPB) {
  return {(DPB + 64) * std::ldexp(1.0, -23), std::ldexp(1.0, -20), std::ldexp(1.0, -16)};
}

float round_up_f(double v) {
  float f = (float)v;
  if ((double)f < v) f = std::nextafter(f, INFINITY);
  return f;
}

// bf16 operands, fp32 rerank copy, per-row and per-tile bound constants, and the
// strided threshold sample of the isotropic rows.
// Group-centred rows and the pruning cut (cwq_group.hip, cwq_prune.hip).
// A cut is a set of internal nodes, the group centres, such that every internal node lies in
// exactly one centre's subtree (its group) or is an ancestor of centres (a top node; the root
// is always one).  A group's rows -- the isotropic rows whose parent is in the group -- are
// centred at the centre's mean when every one of them is at most twice as far from it as
// from the root mean (then the rounding terms stay within the bound's eps and beta margins)
// and all rows of each of its parents share the key coefficients (the group term is folded
// into the parent's prefix): the group is "ok".  The rows of the other groups, and the rows
// whose parent is a top node, stay root-centred; every group is still a pruning group.
//
// The cut is tree-adaptive: a DP over the internal tree (children before parents) minimises
// the rows' summed squared norms as stored -- an ok group's rows at their centre, the rest at
// the root -- plus a penalty lam per group and per top node:
//   best(c) = min( centre at c:  cost(c) + lam,
//                  split c:      (rows directly below c, at the root) + sum best(internal child) + lam )
// A broad root child spanning many clusters (a 500k x 768 ifit tree: 37 root children over
// 500 clusters) is split down to its cluster-level nodes; a tight one stays one group (in
// high dimension splitting a Gaussian cluster saves ~1/D of its norms, far below lam).
// Centres are at depth <= 8 (CWQ_GROUP_MAXDEP); lam = the mean squared root norm of a row
// (CWQ_GROUP_LAMBDA scales it), doubled while the cut has more than kCutMaxGroups groups or
// kCutMaxTop top nodes.  CWQ_GROUP_CUT=1 keeps the round-4 cut (every depth-1 node a centre).  The
// mode is on when the centred rows cut the summed squared norms at least 4x
// (CWQ_GROUP_CENTRE=0 / 1: off / on whenever they shrink).  rgrp[r] = the group a row is
// centred at, or -1.
constexpr int kCutMaxGroups = 4096, kCutMaxTop = kPruneMaxTop;
int plan_groups(cwq_index* ix, const float* mean, const int64_t* d_rows, const std::vector<RowMeta>& meta,
                const std::vector<int>& row_par, const std::vector<int64_t>& int_nodes, const std::vector<int>& par_int,
                std::vector<int>& rgrp, hipStream_t s) {
  int rc;
  const int NLi = ix->NL_iso, NI = ix->NI, D = ix->D;
  rgrp.assign(NLi, -1);
  const char* ge = getenv("CWQ_GROUP_CENTRE");
  const int force = ge && *ge ? atoi(ge) : -1;
  if (force == 0 || NI < 2 || NLi == 0) return CWQ_OK;
  std::vector<int> idep(NI, 0);
  int maxdep_all = 0;
  for (int i = 1; i < NI; ++i) {
    idep[i] = idep[par_int[i]] + 1;   // BFS internal ids: the parent first
    maxdep_all = std::max(maxdep_all, idep[i]);
  }
  const char* ec = getenv("CWQ_GROUP_CUT");
  const bool depth1 = ec && *ec && atoi(ec) == 1;
  const char* em = getenv("CWQ_GROUP_MAXDEP");
  const int maxd = depth1 ? 1 : std::max(1, std::min(maxdep_all, em && *em && atoi(em) > 0 ? atoi(em) : 8));
  const int W = maxd + 1;
  // per row: the squared norm centred at the root ([0]) and at each ancestor of depth 1..maxd
  int *d_rpar = nullptr, *d_pint = nullptr, *d_idep = nullptr;
  int64_t* d_inodes = nullptr;
  double* d_dist = nullptr;
  if ((rc = ix->upload(&d_rpar, row_par, s)) || (rc = ix->upload(&d_pint, par_int, s)) ||
      (rc = ix->upload(&d_idep, idep, s)) || (rc = ix->upload(&d_inodes, int_nodes, s)) ||
      (rc = ix->alloc(&d_dist, (size_t)NLi * W)))
    return rc;
  HIPCHK(launch_group_anc_dist(mean, D, d_rows, NLi, ix->iso_c, d_rpar, d_pint, d_idep, d_inodes, maxd, d_dist, s));
  std::vector<double> dist((size_t)NLi * W);
  HIPCHK(hipMemcpyAsync(dist.data(), d_dist, dist.size() * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  // per internal node: the rows below it -- their squared norms centred at its mean (depth <=
  // maxd) and at the root, their count, and whether they qualify for centring at it; the
  // rows directly below it at the root
  std::vector<double> cost(NI, 0.0), rsub(NI, 0.0), rdir(NI, 0.0);
  std::vector<int64_t> nrow(NI, 0);
  std::vector<char> ok(NI, 1);
  std::vector<float> pcw(NI, NAN), piv(NI, NAN), pinvL(NI, NAN);
  std::vector<char> pbad(NI, 0);
  double sum_root = 0.0;
  for (int r = 0; r < NLi; ++r) {
    const double r0 = dist[(size_t)r * W];
    sum_root += r0;
    const int p = row_par[r];
    if (p < 0) continue;
    rdir[p] += r0;
    if (std::isnan(pcw[p])) {
      pcw[p] = meta[r].cw;
      piv[p] = meta[r].iv;
      pinvL[p] = meta[r].invL;
    } else if (pcw[p] != meta[r].cw || piv[p] != meta[r].iv || pinvL[p] != meta[r].invL) {
      pbad[p] = 1;
    }
    for (int a = p; a > 0; a = par_int[a]) {
      rsub[a] += r0;
      nrow[a]++;
      if (idep[a] <= maxd) {
        const double v = dist[(size_t)r * W + idep[a]];
        cost[a] += v;
        if (!(v <= 4.0 * r0)) ok[a] = 0;   // |M_g| <= 2 |M_0|: the rounding cross term stays in eps
      }
    }
  }
  for (int p = 1; p < NI; ++p)
    if (pbad[p])
      for (int a = p; a > 0; a = par_int[a]) ok[a] = 0;
  std::vector<int> kptr(NI + 1, 0), kids(NI > 0 ? NI - 1 : 0);
  for (int i = 1; i < NI; ++i) kptr[par_int[i] + 1]++;
  for (int i = 0; i < NI; ++i) kptr[i + 1] += kptr[i];
  {
    std::vector<int> fill(kptr.begin(), kptr.end() - 1);
    for (int i = 1; i < NI; ++i) kids[fill[par_int[i]]++] = i;
  }
  const char* el = getenv("CWQ_GROUP_LAMBDA");
  double lam = (el && *el ? atof(el) : 1.0) * sum_root / NLi;
  std::vector<double> best(NI);
  std::vector<char> centre(NI, 0);
  std::vector<int> gint(NI, -1);
  std::vector<int64_t> gnode;
  std::vector<int> gcent;
  int ntop = 0;
  for (int it = 0; it < 64; ++it, lam = lam > 0.0 ? 2.0 * lam : 1.0) {
    for (int c = NI - 1; c >= 1; --c) {
      double cc = INFINITY, sp = INFINITY;
      cc = (ok[c] ? cost[c] : rsub[c]) + lam;
      if (idep[c] < maxd && kptr[c + 1] > kptr[c]) {
        sp = rdir[c] + lam;
        for (int j = kptr[c]; j < kptr[c + 1]; ++j) sp += best[kids[j]];
      }
      centre[c] = cc <= sp ? 1 : 0;
      best[c] = std::min(cc, sp);
    }
    // top-down: group ids in BFS order of the centres
    gnode.clear();
    gcent.clear();
    ntop = 1;
    for (int i = 1; i < NI; ++i) {
      const int p = par_int[i];
      if (gint[p] >= 0) {   // inside p's group
        gint[i] = gint[p];
      } else if (centre[i]) {   // p is a top node (the root, or split): i a centre ...
        gint[i] = (int)gnode.size();
        gnode.push_back(int_nodes[i]);
        gcent.push_back(i);
      } else {   // ... or a top node itself
        gint[i] = -1;
        ++ntop;
      }
    }
    if ((int)gnode.size() <= kCutMaxGroups && ntop <= kCutMaxTop) break;
  }
  const int G = (int)gnode.size();
  if (G == 0 || G > kCutMaxGroups || ntop > kCutMaxTop) return CWQ_OK;
  std::vector<char> gok(G, 0);
  for (int g = 0; g < G; ++g) gok[g] = ok[gcent[g]];
  std::vector<int> cand(NLi, -1);
  double sum_sel = 0.0;
  for (int r = 0; r < NLi; ++r) {
    cand[r] = row_par[r] >= 0 ? gint[row_par[r]] : -1;
    const int g = cand[r];
    sum_sel += (g >= 0 && gok[g]) ? dist[(size_t)r * W + idep[gcent[g]]] : dist[(size_t)r * W];
  }
  ix->cut_gint = gint;
  ix->cut_centre = gcent;
  ix->cut_ok = gok;
  ix->cut_top = ntop;
  ix->cut_maxdep = 0;
  for (int c : gcent) ix->cut_maxdep = std::max(ix->cut_maxdep, idep[c]);
  const bool on = force == 1 ? sum_sel < sum_root : sum_sel * 4.0 <= sum_root;
  if (!on) return CWQ_OK;
  int64_t* d_gnode = nullptr;
  float* cent = nullptr;
  if ((rc = ix->upload(&d_gnode, gnode, s)) || (rc = ix->alloc(&cent, (size_t)G * D))) return rc;
  HIPCHK(launch_gather_rows_f32(mean, D, d_gnode, G, cent, s));
  for (int r = 0; r < NLi; ++r) {
    rgrp[r] = (cand[r] >= 0 && gok[cand[r]]) ? cand[r] : -1;
    ix->n_grp_rows += rgrp[r] >= 0;
  }
  std::vector<int> gpar(NI, -1);
  std::vector<double> F(NI, 0.0), Fc(NI, 0.0);
  for (int p = 1; p < NI; ++p) {
    const int g = gint[p];
    if (g < 0 || !gok[g] || std::isnan(pcw[p])) continue;
    gpar[p] = g;
    const double hs = (double)(float)(-0.5 * (double)pcw[p] * (double)piv[p]);   // RowF.hs (fp32)
    const double hsc = (double)(float)(-0.5 * (double)piv[p]);                    // categorize RowF.hs
    F[p] = hs / (double)pinvL[p];
    Fc[p] = hsc;
  }
  ix->grp_mode = true;
  ix->G = G;
  ix->grp_c = cent;
  if ((rc = ix->upload(&ix->grp_par, gpar, s)) || (rc = ix->upload(&ix->grp_F, F, s)) ||
      (rc = ix->upload(&ix->grp_Fc, Fc, s)))
    return rc;
  HIPCHK(hipStreamSynchronize(s));
  return CWQ_OK;
}

int build_filter(cwq_index* ix, const float* mean, const int64_t* d_rows, const std::vector<RowMeta>& meta,
                 const std::vector<int>& row_par, const std::vector<int>& row_flags,
                 const std::vector<int64_t>& int_nodes, const std::vector<int>& par_int, hipStream_t s) {
  int rc;
  const int DP = ix->DP, D = ix->D, NLi = ix->NL_iso;
  ix->DPB = fgemm_dpb(D);   // whole fgemm stages (cwq_mfma.hip)
  const int DPB = ix->DPB;
  ix->ld_f = round_up(NLi, kFgTile);
  const int64_t ld = ix->ld_f;
  float *n2 = nullptr, *nlo = nullptr, *nhi = nullptr, *nm = nullptr;
  if ((rc = ix->alloc(&ix->iso_Mf, (size_t)DP * ld))) return rc;
  if ((rc = ix->alloc(&ix->iso_Mb, (size_t)DPB * ld))) return rc;
  if ((rc = ix->alloc(&n2, ld))) return rc;
  if ((rc = ix->alloc(&nlo, ld))) return rc;
  if ((rc = ix->alloc(&nhi, ld))) return rc;
  if ((rc = ix->alloc(&nm, ld))) return rc;
  if ((rc = ix->alloc(&ix->iso_c, D))) return rc;
  HIPCHK(hipMemcpyAsync(ix->iso_c, mean, (size_t)D * 4, hipMemcpyDeviceToDevice, s));   // root mean
  std::vector<int> rgrp;
  if ((rc = plan_groups(ix, mean, d_rows, meta, row_par, int_nodes, par_int, rgrp, s))) return rc;
  int* d_rgrp = nullptr;
  if (ix->grp_mode && (rc = ix->upload(&d_rgrp, rgrp, s))) return rc;
  HIPCHK(launch_rows_prep(mean, D, d_rows, NLi, ix->iso_c, DP, DPB, ld, ix->iso_Mf, ix->iso_Mb, n2, nlo, nhi, s,
                          ix->grp_c, d_rgrp, nm));
  std::vector<float> hn2(ld), hlo(ld), hhi(ld), hnm(ld);
  HIPCHK(hipMemcpyAsync(hn2.data(), n2, ld * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hlo.data(), nlo, ld * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hhi.data(), nhi, ld * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hnm.data(), nm, ld * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const FiltConsts fc = filt_consts(DPB);
  // per-row and per-tile constants.  Fast key (cat = false): pi + hs*S + hl with
  // hs = -cw*iv/2, hl = -cw*logdet/2, pi = P[parent]/L.  Categorize (cat = true): the
  // full lp = -(logdet + D log 2pi)/2 - iv*S/2 (cw = 1, no prefix term: invL = 0, tiles
  // parent-free), min'ed with BF[parent] in the kernels; usable = not an internal copy.
  const float dfull = (float)((double)ix->D * (double)logf(2.0f * (float)M_PI));
  ix->cat_dconst = dfull;
  // multi-parent tiles keep the pretest up to this many parents (deep trees: ~4 leaves
  // per parent puts ~64 parents in a 256-row tile); CWQ_FG_MAX_PARENTS overrides
  const int max_parents = [] {
    const char* e = getenv("CWQ_FG_MAX_PARENTS");
    return e && *e ? std::max(1, atoi(e)) : kFgMaxTileParents;
  }();
  auto tables = [&](bool cat, std::vector<RowF>& rf, std::vector<TileF>& tf) {
    rf.assign(ld, RowF{});
    std::vector<double> gr(ld, 0.0);
    for (int64_t r = 0; r < ld; ++r) {
      RowF& f = rf[r];
      const bool usable = r < NLi && (cat ? !(row_flags[r] & FLAG_INT_COPY) : (row_flags[r] & FLAG_HAS_SENT) != 0);
      if (!usable) {
        f = RowF{-INFINITY, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2};
        continue;
      }
      const RowMeta& m = meta[r];
      const double cw = cat ? 1.0 : (double)m.cw;
      const double ldet = cat ? (double)(m.logdet + dfull) : (double)m.logdet;   // fp32 add, as the scan
      const double hs = -0.5 * cw * (double)m.iv, hl = -0.5 * cw * ldet;
      const double g = cw * (double)m.iv;
      const bool grow = ix->grp_mode && rgrp[r] >= 0;
      // group-centred rows: the fp32 rounding of M = fl(mu - c_g) enters the dot through
      // |x'| |M| -- 2^-23 |M| on both split norms covers it (cwq_group.hip)
      const double ge = grow ? std::ldexp((double)hnm[r], -23) * (1.0 + std::ldexp(1.0, -20)) : 0.0;
      f.beta = round_up_f((double)hlo[r] + fc.gamma * (double)hhi[r] + ge);
      f.delta = round_up_f((double)hhi[r] + (double)hlo[r] + ge);
      f.rn2 = hn2[r];
      f.hs = (float)hs;
      f.hl = (float)hl;
      // categorize reads a prefix term only for group-centred rows: their group term
      f.invL = cat ? (grow ? 1.f : 0.f) : m.invL;
      f.par = row_par[r];
      gr[r] = g;
      if (g > 0.0 && std::isfinite(g) && std::isfinite(hl)) {
        const double rn2 = hn2[r];
        double R = hl / g - 0.5 * rn2 + 0.5 * fc.eps_n * rn2 + fc.slack * (std::fabs(hl) / g + 1.5 * rn2);
        R += 4.0 * fc.gamma * (std::fabs(R) + std::fabs(hl) / g + rn2);
        f.R0 = round_up_f(R);
      } else {
        f.R0 = 0.f;   // only ever on non-uniform tiles
      }
    }
    const int n_rt = (int)(ld / kFgTile);
    tf.assign(n_rt, TileF{});
    for (int t = 0; t < n_rt; ++t) {
      TileF& T = tf[t];
      T = TileF{1, -1, 1.f, 1.f, 0.f, 0.f, -1, 0.f};
      bool first = true, same_par = true;
      int plo = INT32_MAX, phi = -1, tgrp = -1;
      for (int64_t r = (int64_t)t * kFgTile; r < (int64_t)(t + 1) * kFgTile; ++r) {
        if (rf[r].par < -1) continue;
        const double g = gr[r];
        if (!(g > 0.0) || !std::isfinite(g) || !std::isfinite(rf[r].R0)) T.uniform = 0;
        // categorize tiles: parent-free, or (group-centred rows) all rows of one group,
        // whose term any of their parents carries
        const int cg = ix->grp_mode && r < NLi ? rgrp[r] : -1;
        if (first) {
          T.par = cat ? (cg >= 0 ? rf[r].par : -1) : rf[r].par;
          T.invL = rf[r].invL;
          T.g = (float)g;
          tgrp = cg;
          first = false;
        } else if (rf[r].invL != T.invL || (float)g != T.g || (cat && cg != tgrp)) {
          T.uniform = 0;
        }
        if (!cat && rf[r].par != T.par) same_par = false;
        plo = std::min(plo, rf[r].par);
        phi = std::max(phi, rf[r].par);
        T.beta_max = std::max(T.beta_max, rf[r].beta);
        T.delta_max = std::max(T.delta_max, rf[r].delta);
      }
      T.par_hi = T.par;
      if (T.uniform && !same_par) {
        if (plo >= 0 && phi - plo < max_parents && !getenv("CWQ_FG_NO_MULTI")) {
          T.uniform = 2;
          T.par = plo;
          T.par_hi = phi;
        } else {
          T.uniform = 0;
        }
      }
    }
  };
  std::vector<RowF> rf;
  std::vector<TileF> tf;
  tables(false, rf, tf);
  const int n_rt = (int)(ld / kFgTile);
  if ((rc = ix->upload(&ix->iso_rf, rf, s))) return rc;
  if ((rc = ix->upload(&ix->iso_tf, tf, s))) return rc;
  ix->tile_uni_prefix.assign(n_rt + 1, 0);
  // all_uniform launches (fgemm_kernel<0, true>) need single-parent tiles
  for (int t = 0; t < n_rt; ++t) ix->tile_uni_prefix[t + 1] = ix->tile_uni_prefix[t] + (tf[t].uniform == 1 ? 1 : 0);
  ix->n_multi_tiles = 0;
  for (int t = 0; t < n_rt; ++t) ix->n_multi_tiles += tf[t].uniform == 2 ? 1 : 0;
  HIPCHK(hipStreamSynchronize(s));   // the uploads read rf / tf, rebuilt below
  tables(true, rf, tf);
  if ((rc = ix->upload(&ix->cat_rf, rf, s))) return rc;
  if ((rc = ix->upload(&ix->cat_tf, tf, s))) return rc;
  ix->cat_uni_prefix.assign(n_rt + 1, 0);
  for (int t = 0; t < n_rt; ++t) ix->cat_uni_prefix[t + 1] = ix->cat_uni_prefix[t] + (tf[t].uniform == 1 ? 1 : 0);
  HIPCHK(hipStreamSynchronize(s));   // the host vectors above are freed on return
  // threshold sample: ~NL_iso/128 rows at a fixed stride, 256 <= S <= 32768 (the filter
  // phases tighten T afterwards, so a small sample only costs the first phase)
  const char* sd = getenv("CWQ_FG_SAMPLE_DIV");
  const int sdiv = sd && atoi(sd) > 0 ? atoi(sd) : 128;
  int S = (int)std::min<int64_t>(32768, std::max<int64_t>(kFgTile, NLi / sdiv / kFgTile * kFgTile));
  const int stride = std::max(1, NLi / S);
  std::vector<int> srow;
  srow.reserve(S);
  for (int j = 0; j < S; ++j) {
    const int64_t r = (int64_t)j * stride;
    if (r < NLi) srow.push_back((int)r);
  }
  if (ix->grp_mode) {
    // clustered trees: the query's own cluster decides its top-k, and a strided sample
    // holds only ~1/sdiv of it, so T stayed at other clusters' keys and most of the
    // cluster passed the filter (C2 ifit tree: ~1,100 candidates per query, overflowing
    // the record buffers).  Add kPerGroup rows of every group, spread over its rows
    // (distinct rows only: T must bound the K-th best key over distinct rows).
    // (fewer per group on a deep cut: the sample stays within 32,768 rows)
    const int kPerGroup = std::max(8, std::min(64, (32768 - (int)srow.size()) / std::max(1, ix->G)));
    std::vector<std::vector<int>> gr(ix->G);
    for (int64_t r = 0; r < NLi; ++r)
      if (rgrp[r] >= 0) gr[rgrp[r]].push_back((int)r);
    std::vector<char> in(NLi, 0);
    for (int r : srow) in[r] = 1;
    for (int g = 0; g < ix->G && (int64_t)srow.size() + kPerGroup <= 32768; ++g) {
      const int n = (int)gr[g].size();
      const int m = std::min(n, kPerGroup);
      for (int j = 0; j < m; ++j) {
        const int r = gr[g][(int64_t)j * n / m];
        if (!in[r]) {
          in[r] = 1;
          srow.push_back(r);
        }
      }
    }
  }
  const int ns = (int)srow.size();
  srow.resize(round_up(ns, kFgTile), -1);
  ix->n_samp = ns;
  ix->ld_s = (int)srow.size();
  if ((rc = ix->upload(&ix->samp_rows, srow, s))) return rc;
  if ((rc = ix->alloc(&ix->iso_Sb, (size_t)DPB * ix->ld_s))) return rc;
  HIPCHK(launch_gather_bf16_rows(ix->iso_Mb, DPB, ix->samp_rows, ix->ld_s, ix->iso_Sb, s));
  HIPCHK(hipStreamSynchronize(s));
  return CWQ_OK;
}

// Group pruning constants (cwq_prune.hip).  Groups are plan_groups' cut:
// a group's members are the internal nodes of its centre's subtree and the leaf-class rows
// below them (a row that is itself an internal node belongs to that node's group); the top
// nodes (the root and the centres' ancestors) belong to no group and every query computes
// them exactly (prune_head_kernel).  Needs the group-centred mode (group centres), the
// row-major A/B copies (exact pass of a group), and every level weight and row weight >= 0
// (the key bound adds upper bounds of lp' with non-negative coefficients).
// CWQ_GROUP_PRUNE=0 at index creation leaves it off.
int build_prune(cwq_index* ix, const float* mean, const VarSrc& var, const std::vector<int64_t>& int_nodes,
                const std::vector<int>& par_int, const std::vector<float>& w_int, const std::vector<int64_t>& rows,
                const std::vector<int>& int_id, const std::vector<RowMeta>& meta, const std::vector<int>& row_par,
                const std::vector<int>& row_flags, hipStream_t s) {
  const char* e = getenv("CWQ_GROUP_PRUNE");
  if ((e && *e && atoi(e) == 0) || !ix->grp_mode || ix->G <= 0 || !ix->int_Ar || ix->NI < 2 || ix->DP > 2048)
    return CWQ_OK;
  const int NI = ix->NI, NL = ix->NL, G = ix->G;
  for (float w : w_int)
    if (!(w >= 0.f)) return CWQ_OK;
  for (int r = 0; r < NL; ++r)
    if (!(meta[r].cw >= 0.f) || !(meta[r].invL >= 0.f)) return CWQ_OK;
  // pruning group of every internal node (plan_groups' cut; -1: a top node)
  const std::vector<int>& gint = ix->cut_gint;
  if ((int)gint.size() != NI || (int)ix->cut_centre.size() != G) return CWQ_OK;
  // top nodes, BFS order: their parents are top nodes too (a cut)
  std::vector<int> tnodes, tpos(NI, -1), tpp, tdep;
  std::vector<int> idep(NI, 0);
  for (int i = 1; i < NI; ++i) idep[i] = idep[par_int[i]] + 1;
  for (int i = 0; i < NI; ++i) {
    if (gint[i] >= 0) continue;
    const int p = i == 0 ? -1 : par_int[i];
    if (p >= 0 && tpos[p] < 0) return CWQ_OK;   // never: the parent of a top node is a top node
    tpos[i] = (int)tnodes.size();
    tnodes.push_back(i);
    tpp.push_back(p >= 0 ? tpos[p] : -1);
    tdep.push_back(idep[i]);
  }
  std::vector<int> gtpos(G);
  for (int g = 0; g < G; ++g) {
    const int c = ix->cut_centre[g];
    if (gint[c] != g || tpos[par_int[c]] < 0) return CWQ_OK;   // never: a centre's parent is a top node
    gtpos[g] = tpos[par_int[c]];
  }
  // members: internal nodes 1.. (top nodes: no group), then rows
  std::vector<int64_t> mnode;
  std::vector<float> miv;
  std::vector<int> mgrp;
  for (int i = 1; i < NI; ++i) {
    mnode.push_back(int_nodes[i]);
    miv.push_back(0.f);
    mgrp.push_back(gint[i]);
  }
  std::vector<int> rgrp(NL, -1);
  for (int r = 0; r < NL; ++r) {
    const int own = int_id[rows[r]];
    rgrp[r] = own >= 0 ? gint[own] : (row_par[r] >= 0 ? gint[row_par[r]] : -1);
    mnode.push_back(rows[r]);
    miv.push_back(r < ix->NL_iso ? meta[r].iv : 0.f);
    mgrp.push_back(rgrp[r]);
  }
  const int64_t nm = (int64_t)mnode.size();
  int64_t* d_mnode = nullptr;
  float* d_miv = nullptr;
  int* d_mgrp = nullptr;
  double4* d_out = nullptr;
  int rc;
  if ((rc = ix->upload(&d_mnode, mnode, s)) || (rc = ix->upload(&d_miv, miv, s)) || (rc = ix->upload(&d_mgrp, mgrp, s)) ||
      (rc = ix->alloc(&d_out, nm)))
    return rc;
  HIPCHK(launch_prune_members(mean, var, ix->D, d_mnode, d_miv, d_mgrp, ix->grp_c, nm, d_out, s));
  std::vector<double4> mo(nm);
  std::vector<float> ldi(NI);
  HIPCHK(hipMemcpyAsync(mo.data(), d_out, nm * sizeof(double4), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(ldi.data(), ix->logdet_int, NI * sizeof(float), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<GroupBound> gb(G);
  std::vector<double> d2max(G, 0.0), m2max(G, 0.0);
  for (auto& b : gb) {
    b = GroupBound{};
    b.wmin = INFINITY;
    b.wmax = 0.0;
    b.ldmin = INFINITY;
    b.ldabs = 0.0;
    b.iLmin = b.Cmin = INFINITY;
    b.iLmax = b.Cmax = -INFINITY;
    b.valid = 0;
  }
  for (int64_t m = 0; m < nm; ++m) {
    const int g = mgrp[m];
    if (g < 0) continue;
    GroupBound& b = gb[g];
    b.wmin = std::min(b.wmin, mo[m].x);
    b.wmax = std::max(b.wmax, mo[m].y);
    d2max[g] = std::max(d2max[g], mo[m].z);
    m2max[g] = std::max(m2max[g], mo[m].w);
    const double ld = m < NI - 1 ? (double)ldi[m + 1] : (double)meta[m - (NI - 1)].logdet;
    b.ldmin = std::min(b.ldmin, ld);
    b.ldabs = std::max(b.ldabs, std::fabs(ld));
  }
  // the key coefficients of the usable rows: 1/L and C = invL * sum_{a in path, a in g} w_a + cw
  // (the path's top nodes -- the root down to the centre's parent t_g -- are P(t_g), exact)
  std::vector<double> wsum(NI, 0.0);   // sum of w over the path of internal node i within its group
  for (int i = 1; i < NI; ++i)
    if (gint[i] >= 0) wsum[i] = (gint[par_int[i]] == gint[i] ? wsum[par_int[i]] : 0.0) + (double)w_int[i];
  for (int r = 0; r < NL; ++r) {
    const int g = rgrp[r];
    if (g < 0 || !(row_flags[r] & FLAG_HAS_SENT)) continue;
    GroupBound& b = gb[g];
    const int rp = row_par[r];
    const double iL = meta[r].invL, C = iL * (rp >= 0 && gint[rp] == g ? wsum[rp] : 0.0) + (double)meta[r].cw;
    b.iLmin = std::min(b.iLmin, iL);
    b.iLmax = std::max(b.iLmax, iL);
    b.Cmin = std::min(b.Cmin, C * (1.0 - 0x1p-40));
    b.Cmax = std::max(b.Cmax, C * (1.0 + 0x1p-40));
    b.valid = 1;
  }
  for (int g = 0; g < G; ++g) {
    GroupBound& b = gb[g];
    b.r = std::sqrt(d2max[g]) * (1.0 + 0x1p-40) + 1e-30;
    b.mmax = std::sqrt(m2max[g]) * (1.0 + 0x1p-40);
    b.wmin *= 1.0 - 0x1p-40;
    b.wmax *= 1.0 + 0x1p-40;
    if (!(b.wmin > 0.0) || !std::isfinite(b.wmax) || !std::isfinite(b.ldmin)) b.valid = b.valid ? -1 : 0;
  }
  for (auto& b : gb)
    if (b.valid < 0) return CWQ_OK;   // a member without a finite positive weight: no bound
  // group-major internal node lists (ascending internal id)
  std::vector<int> gptr(G + 1, 0), gnodes;
  for (int i = 1; i < NI; ++i)
    if (gint[i] >= 0) gptr[gint[i] + 1]++;
  for (int g = 0; g < G; ++g) gptr[g + 1] += gptr[g];
  gnodes.assign(gptr[G], 0);
  std::vector<int> fillp(gptr.begin(), gptr.end() - 1);
  for (int i = 1; i < NI; ++i)
    if (gint[i] >= 0) gnodes[fillp[gint[i]]++] = i;
  ix->prn_gmax = 1;
  for (int g = 0; g < G; ++g) ix->prn_gmax = std::max(ix->prn_gmax, gptr[g + 1] - gptr[g]);
  // LDS of the seed and stage-B kernels (their group-prefix arrays grow with the largest group)
  if (prune_lds_max(ix->DP, ix->prn_gmax) > kPruneLdsCap) return CWQ_OK;
  // per list entry: depth (root 0) and the parent's position in the same list (-1: the
  // centre, whose parent is a top node; the lists are BFS-ordered, so a level is finished
  // before the next starts)
  std::vector<int> lpos(NI, -1), gdep(gnodes.size()), gpp(gnodes.size());
  for (size_t j = 0; j < gnodes.size(); ++j) lpos[gnodes[j]] = (int)j;
  ix->prn_maxdep = 0;
  ix->prn_mindep = INT32_MAX;
  for (size_t j = 0; j < gnodes.size(); ++j) {
    const int i = gnodes[j], p = par_int[i];
    gdep[j] = idep[i];
    const bool inner = gint[p] == gint[i];
    gpp[j] = inner ? lpos[p] : -1;
    ix->prn_maxdep = std::max(ix->prn_maxdep, idep[i]);
    ix->prn_mindep = std::min(ix->prn_mindep, idep[i]);
    if (inner ? lpos[p] >= (int)j : i != ix->cut_centre[gint[i]]) return CWQ_OK;   // never: a group is a subtree in BFS order
  }
  if (ix->prn_mindep == INT32_MAX) ix->prn_mindep = 1;
  if (gdep.empty()) {
    gdep.push_back(0);
    gpp.push_back(-1);
  }
  // the seed threshold's rows: up to 64 usable isotropic rows of each group, spread over it
  std::vector<std::vector<int>> grows(G);
  for (int r = 0; r < ix->NL_iso; ++r)
    if (rgrp[r] >= 0 && (row_flags[r] & FLAG_HAS_SENT)) grows[rgrp[r]].push_back(r);
  std::vector<int> sptr2(G + 1, 0), srows2;
  for (int g = 0; g < G; ++g) {
    const int n = (int)grows[g].size(), m = std::min(n, 64);
    for (int j = 0; j < m; ++j) srows2.push_back(grows[g][(int64_t)j * n / m]);
    sptr2[g + 1] = (int)srows2.size();
  }
  if (srows2.empty()) srows2.push_back(0);
  if ((rc = ix->upload(&ix->gs_ptr, sptr2, s)) || (rc = ix->upload(&ix->gs_rows, srows2, s))) return rc;
  // the per-call filter's blocks: a block is left out when its rows' one group is pruned
  std::vector<int> bg((size_t)std::max<int64_t>(1, ((int64_t)ix->NL_iso + 15) / 16), -1);
  for (int64_t b = 0; b * 16 < ix->NL_iso; ++b) {
    const int r0 = (int)(b * 16), r1 = (int)std::min<int64_t>(ix->NL_iso, b * 16 + 16);
    int g = rgrp[r0];
    for (int r = r0 + 1; r < r1 && g >= 0; ++r)
      if (rgrp[r] != g) g = -1;
    bg[b] = g;
  }
  if ((rc = ix->upload(&ix->blk_grp, bg, s))) return rc;
  if ((rc = ix->upload(&ix->gi_dep, gdep, s)) || (rc = ix->upload(&ix->gi_ppos, gpp, s))) return rc;
  ix->n_top = (int)tnodes.size();
  ix->top_maxdep = 0;
  for (int d : tdep) ix->top_maxdep = std::max(ix->top_maxdep, d);
  if ((rc = ix->upload(&ix->top_nodes, tnodes, s)) || (rc = ix->upload(&ix->top_ppos, tpp, s)) ||
      (rc = ix->upload(&ix->top_dep, tdep, s)) || (rc = ix->upload(&ix->grp_tpos, gtpos, s)))
    return rc;
  if ((rc = ix->upload(&ix->prn_gint, gint, s)) || (rc = ix->upload(&ix->gi_ptr, gptr, s)) ||
      (rc = ix->upload(&ix->gi_nodes, gnodes, s)) || (rc = ix->upload(&ix->gbound, gb, s)) ||
      (rc = ix->alloc(&ix->prune_ctr, 8)))
    return rc;
  HIPCHK(hipMemsetAsync(ix->prune_ctr, 0, 8 * sizeof(int), s));
  HIPCHK(hipStreamSynchronize(s));
  ix->prune_ok = true;
  return CWQ_OK;
}

}  // namespace

namespace {
// cwq_index_create / cwq_index_create_cv: `var` is either the full [n_nodes][D] array or
// the compact per-node form (VarSrc); both give the same index.
bool use_int_bounds(const cwq_index* ix);
bool ensure_i8(cwq_index* ix, hipStream_t s);

int index_create_impl(int device, int64_t n_nodes, int32_t dim, const float* mean, const VarSrc& var,
                      const int64_t* parent, const int64_t* node_of_sentence, int64_t n_sent, const double* level_w,
                      int32_t n_w, hipStream_t s, cwq_index** out) {

  // ---- structure (host) ----
  if (parent[0] != -1) return fail(CWQ_ERR_ARG, "parent[0] must be -1 (root first, BFS order)");
  std::vector<int> depth(n_nodes, 0), nchild(n_nodes, 0);
  for (int64_t i = 1; i < n_nodes; ++i) {
    const int64_t p = parent[i];
    if (p < 0 || p >= i) return fail(CWQ_ERR_ARG, "parent[i] must be in [0, i) (BFS order)");
    if (p < parent[i - 1]) return fail(CWQ_ERR_ARG, "parent array must be non-decreasing (BFS order)");
    depth[i] = depth[p] + 1;
    nchild[p]++;
  }
  std::vector<std::vector<int64_t>> sents(n_nodes);
  for (int64_t sidx = 0; sidx < n_sent; ++sidx) {
    const int64_t nd = node_of_sentence[sidx];
    if (nd < -1 || nd >= n_nodes) return fail(CWQ_ERR_ARG, "node_of_sentence out of range");
    if (nd >= 0) sents[nd].push_back(sidx);
  }
  std::unique_ptr<cwq_index> ix(new cwq_index());
  ix->device = device;
  ix->n_nodes = n_nodes;
  ix->n_sent = n_sent;
  ix->D = dim;
  ix->DP = (int)round_up(dim, kDChunk);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ix->cus = prop.multiProcessorCount;

  std::vector<int64_t> int_nodes, leaf_nodes;
  std::vector<int> int_id(n_nodes, -1);
  for (int64_t i = 0; i < n_nodes; ++i) {
    if (nchild[i] > 0) {
      int_id[i] = (int)int_nodes.size();
      int_nodes.push_back(i);
    }
    if (nchild[i] == 0 || !sents[i].empty()) leaf_nodes.push_back(i);
    ix->max_depth = std::max(ix->max_depth, depth[i]);
  }
  ix->NI = (int)int_nodes.size();
  const int64_t nleaf = (int64_t)leaf_nodes.size();

  // isotropy of leaf-class rows (device)
  int64_t* d_leaf_nodes = nullptr;
  int* d_iso = nullptr;
  int rc = ix->upload(&d_leaf_nodes, leaf_nodes, s);
  if (rc) return rc;
  if ((rc = ix->alloc(&d_iso, nleaf))) return rc;
  HIPCHK(launch_iso_flags(var, dim, d_leaf_nodes, nleaf, d_iso, s));
  std::vector<int> iso(nleaf);
  HIPCHK(hipMemcpyAsync(iso.data(), d_iso, nleaf * sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));

  std::vector<int64_t> rows_iso, rows_an;
  for (int64_t r = 0; r < nleaf; ++r) (iso[r] ? rows_iso : rows_an).push_back(leaf_nodes[r]);
  ix->NL_iso = (int)rows_iso.size();
  ix->NL_an = (int)rows_an.size();
  ix->NL = ix->NL_iso + ix->NL_an;
  std::vector<int64_t> rows(rows_iso);
  rows.insert(rows.end(), rows_an.begin(), rows_an.end());
  std::vector<int> row_of_node(n_nodes, -1);
  for (int r = 0; r < ix->NL; ++r) row_of_node[rows[r]] = r;

  auto wdepth = [&](int d) -> double { return d < n_w ? level_w[d] : 1.0; };

  // leaf-row metadata
  std::vector<RowMeta> meta(ix->NL);
  std::vector<int> row_par(ix->NL), row_flags(ix->NL), row_bfs(ix->NL);
  std::vector<int64_t> sptr(ix->NL + 1, 0), sids;
  std::vector<int> row_of_sent(n_sent, -1);
  for (int r = 0; r < ix->NL; ++r) {
    const int64_t nd = rows[r];
    const int L = depth[nd] + 1;
    meta[r].cw = (float)(wdepth(depth[nd]) / L);
    meta[r].invL = (float)(1.0 / L);
    row_par[r] = parent[nd] >= 0 ? int_id[parent[nd]] : -1;
    row_flags[r] = (sents[nd].empty() ? 0 : FLAG_HAS_SENT) | (nchild[nd] > 0 ? FLAG_INT_COPY : 0);
    row_bfs[r] = (int)nd;
    for (int64_t sidx : sents[nd]) {
      sids.push_back(sidx);
      row_of_sent[sidx] = r;
    }
    sptr[r + 1] = (int64_t)sids.size();
  }
  // internal-node metadata
  std::vector<int> par_int(ix->NI), cb(ix->NI, 0), ce(ix->NI, 0), ibfs(ix->NI), ihs(ix->NI), inch(ix->NI);
  std::vector<int> la0(ix->NI, 0), la1(ix->NI, 0), lb0(ix->NI, 0), lb1(ix->NI, 0);
  std::vector<float> w_int(ix->NI);
  for (int i = 0; i < ix->NI; ++i) {
    const int64_t nd = int_nodes[i];
    par_int[i] = parent[nd] >= 0 ? int_id[parent[nd]] : -1;
    ibfs[i] = (int)nd;
    ihs[i] = sents[nd].empty() ? 0 : 1;
    inch[i] = nchild[nd];
    ix->max_fanout = std::max(ix->max_fanout, (int)nchild[nd]);
    w_int[i] = (float)wdepth(depth[nd]);
    cb[i] = ce[i] = -1;
    la0[i] = la1[i] = lb0[i] = lb1[i] = -1;
  }
  for (int64_t nd = 1; nd < n_nodes; ++nd) {   // children ranges (contiguous in each ordering)
    const int pi = int_id[parent[nd]];
    if (int_id[nd] >= 0) {
      if (cb[pi] < 0) cb[pi] = int_id[nd];
      ce[pi] = int_id[nd] + 1;
    }
    const int r = row_of_node[nd];
    if (r >= 0) {
      if (r < ix->NL_iso) {
        if (la0[pi] < 0) la0[pi] = r;
        la1[pi] = r + 1;
      } else {
        if (lb0[pi] < 0) lb0[pi] = r;
        lb1[pi] = r + 1;
      }
    }
  }
  for (int i = 0; i < ix->NI; ++i) {
    if (cb[i] < 0) cb[i] = ce[i] = 0;
    if (la0[i] < 0) la0[i] = la1[i] = 0;
    if (lb0[i] < 0) lb0[i] = lb1[i] = 0;
  }
  for (int i = 0; i < ix->NI;) {   // levels (BFS -> depth non-decreasing)
    int j = i;
    const int d0 = depth[int_nodes[i]];
    while (j < ix->NI && depth[int_nodes[j]] == d0) ++j;
    ix->levels.push_back({i, j});
    i = j;
  }
  std::vector<int> node_src(n_nodes);
  for (int64_t nd = 0; nd < n_nodes; ++nd) node_src[nd] = int_id[nd] >= 0 ? int_id[nd] : -(row_of_node[nd] + 1);
  std::vector<int> lv_starts;
  for (auto& lv : ix->levels) lv_starts.push_back(lv.first);
  lv_starts.push_back(ix->NI);

  // ---- device arrays ----
  const int DP = ix->DP;
  ix->ld_int = round_up(std::max(ix->NI, 1), kWave);
  ix->ld_iso = round_up(std::max(ix->NL_iso, 1), kWave);
  ix->ld_an = round_up(std::max(ix->NL_an, 1), kWave);
  int64_t *d_int_nodes = nullptr, *d_rows = nullptr;
  if ((rc = ix->upload(&d_int_nodes, int_nodes, s))) return rc;
  if ((rc = ix->upload(&d_rows, rows, s))) return rc;
  if ((rc = ix->alloc(&ix->int_A, (size_t)DP * ix->ld_int))) return rc;
  if ((rc = ix->alloc(&ix->int_B, (size_t)DP * ix->ld_int))) return rc;
  if ((rc = ix->alloc(&ix->iso_M, (size_t)DP * ix->ld_iso))) return rc;
  if ((rc = ix->alloc(&ix->an_A, (size_t)DP * ix->ld_an))) return rc;
  if ((rc = ix->alloc(&ix->an_B, (size_t)DP * ix->ld_an))) return rc;
  HIPCHK(launch_gather_T(mean, var, dim, d_int_nodes, ix->NI, 1, ix->int_A, ix->ld_int, DP, s));
  HIPCHK(launch_gather_T(mean, var, dim, d_int_nodes, ix->NI, 2, ix->int_B, ix->ld_int, DP, s));
  HIPCHK(launch_gather_T(mean, var, dim, d_rows, ix->NL_iso, 0, ix->iso_M, ix->ld_iso, DP, s));
  HIPCHK(launch_gather_T(mean, var, dim, d_rows + ix->NL_iso, ix->NL_an, 1, ix->an_A, ix->ld_an, DP, s));
  HIPCHK(launch_gather_T(mean, var, dim, d_rows + ix->NL_iso, ix->NL_an, 2, ix->an_B, ix->ld_an, DP, s));
  if ((rc = ix->alloc(&ix->logdet_int, ix->NI))) return rc;
  if ((rc = ix->alloc(&ix->logdet_row, ix->NL))) return rc;
  HIPCHK(launch_logdet(var, dim, d_int_nodes, ix->NI, ix->logdet_int, s));
  HIPCHK(launch_logdet(var, dim, d_rows, ix->NL, ix->logdet_row, s));
  float* d_iv = nullptr;
  if ((rc = ix->alloc(&d_iv, ix->NL))) return rc;
  HIPCHK(hipMemsetAsync(d_iv, 0, std::max(ix->NL, 1) * sizeof(float), s));
  HIPCHK(launch_inv_var0(var, dim, d_rows, ix->NL_iso, d_iv, s));
  std::vector<float> ldr(ix->NL), ivh(ix->NL);
  if (ix->NL) {
    HIPCHK(hipMemcpyAsync(ldr.data(), ix->logdet_row, ix->NL * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ivh.data(), d_iv, ix->NL * sizeof(float), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  for (int r = 0; r < ix->NL; ++r) {
    meta[r].logdet = ldr[r];
    meta[r].iv = ivh[r];
  }
  if ((rc = ix->upload(&ix->row_meta, meta, s))) return rc;
  if (ix->NL_iso > 0 && (rc = build_filter(ix.get(), mean, d_rows, meta, row_par, row_flags, int_nodes, par_int, s)))
    return rc;
  if ((rc = ix->upload(&ix->row_par, row_par, s))) return rc;
  if ((rc = ix->upload(&ix->row_flags, row_flags, s))) return rc;
  if ((rc = ix->upload(&ix->row_bfs, row_bfs, s))) return rc;
  if ((rc = ix->upload(&ix->par_int, par_int, s))) return rc;
  if ((rc = ix->upload(&ix->w_int, w_int, s))) return rc;
  if ((rc = ix->upload(&ix->int_child_begin, cb, s))) return rc;
  if ((rc = ix->upload(&ix->int_child_end, ce, s))) return rc;
  if ((rc = ix->upload(&ix->int_nchild, inch, s))) return rc;
  if ((rc = ix->upload(&ix->int_bfs, ibfs, s))) return rc;
  if ((rc = ix->upload(&ix->int_has_sent, ihs, s))) return rc;
  for (int v : ihs) ix->any_int_sent = ix->any_int_sent || v != 0;
  if ((rc = ix->upload(&ix->int_leaf_a0, la0, s))) return rc;
  if ((rc = ix->upload(&ix->int_leaf_a1, la1, s))) return rc;
  if ((rc = ix->upload(&ix->int_leaf_b0, lb0, s))) return rc;
  if ((rc = ix->upload(&ix->int_leaf_b1, lb1, s))) return rc;
  if ((rc = ix->upload(&ix->sent_ptr, sptr, s))) return rc;
  if ((rc = ix->upload(&ix->sent_ids, sids, s))) return rc;
  if ((rc = ix->upload(&ix->row_of_sent, row_of_sent, s))) return rc;
  if ((rc = ix->upload(&ix->node_src, node_src, s))) return rc;
  if ((rc = ix->upload(&ix->d_lv, lv_starts, s))) return rc;
  if (ix->NI > 0) {   // the root's terms (the per-call probe's fused prep forms its prefix)
    ix->root_w0 = w_int[0];
    HIPCHK(hipMemcpyAsync(&ix->root_logdet0, ix->logdet_int, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  if (ix->NL_iso > 0 && ix->NI >= 2 && ix->max_depth <= kMaxChain) {
    // internal-node bound operands: K = [x'^2, x'] -> DPB2 = fgemm width of 2*DP
    ix->DPB2 = fgemm_dpb(2 * ix->DP);
    const char* ep = getenv("CWQ_INT_PATH");
    ix->int_path = !(ep && *ep && atoi(ep) == 0);
    const float gamma2 = (float)((ix->DPB2 + 64) * std::ldexp(1.0, -23));
    ix->root_w = w_int[0];
    HIPCHK(hipMemcpyAsync(&ix->root_ld, ix->logdet_int, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if ((rc = ix->alloc(&ix->int_Ar, (size_t)ix->NI * DP))) return rc;
    if ((rc = ix->alloc(&ix->int_Br, (size_t)ix->NI * DP))) return rc;
    std::vector<int> rowid;
    if (ix->int_path) {
      // rows: the root (its exact prefix: final_kernel's chain starts from P[q][0]) and
      // every internal node with isotropic leaf rows below it, in id order
      for (int i = 0; i < ix->NI; ++i)
        if (i == 0 || la1[i] > la0[i]) rowid.push_back(i);
      ix->ld_i2 = round_up((int64_t)rowid.size(), kFgTile);
      const int64_t n = (int64_t)rowid.size();
      rowid.resize(ix->ld_i2, -1);
      if ((rc = ix->alloc(&ix->int_Mb2, (size_t)ix->DPB2 * ix->ld_i2))) return rc;
      if ((rc = ix->alloc(&ix->int_rf2, (size_t)ix->ld_i2))) return rc;
      if ((rc = ix->upload(&ix->int_rowid, rowid, s))) return rc;
      HIPCHK(launch_int_prep(mean, var, dim, d_int_nodes, ix->NI, ix->iso_c, ix->logdet_int, ix->par_int, ix->w_int, DP,
                             ix->DPB2, ix->NI, nullptr, nullptr, ix->int_Ar, ix->int_Br, gamma2, s));
      HIPCHK(launch_int_path_prep(mean, var, dim, d_int_nodes, ix->int_rowid, n, ix->iso_c, ix->logdet_int,
                                  ix->par_int, ix->w_int, DP, ix->DPB2, ix->ld_i2, ix->int_Mb2, ix->int_rf2, gamma2, s));
      // the same RowF by internal id, for the readers of the path-sum dots (PathB)
      std::vector<RowF> rf2h((size_t)n), nrf((size_t)ix->NI, RowF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, -2});
      HIPCHK(hipMemcpyAsync(rf2h.data(), ix->int_rf2, (size_t)n * sizeof(RowF), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      for (int64_t r = 0; r < n; ++r) nrf[rowid[r]] = rf2h[r];
      if ((rc = ix->upload(&ix->int_nrf, nrf, s))) return rc;
    } else {
      // level-aligned operand layout: segments [levels 0 and 1], [level 2], [level 3], ...,
      // each padded to whole 256-row tiles
      std::vector<std::pair<int, int>> segs;   // internal id ranges
      for (size_t lv = 0; lv < ix->levels.size(); ++lv) {
        if (lv == 1) segs.back().second = ix->levels[1].second;
        else segs.push_back(ix->levels[lv]);
      }
      std::vector<int64_t> seg_row(segs.size());
      int64_t rows = 0;
      for (size_t g = 0; g < segs.size(); ++g) {
        seg_row[g] = rows;
        rows += round_up(segs[g].second - segs[g].first, kFgTile);
      }
      ix->ld_i2 = rows;
      rowid.assign(rows, -1);
      for (size_t g = 0; g < segs.size(); ++g)
        for (int i = segs[g].first; i < segs[g].second; ++i) rowid[seg_row[g] + (i - segs[g].first)] = i;
      if ((rc = ix->alloc(&ix->int_Mb2, (size_t)ix->DPB2 * ix->ld_i2))) return rc;
      if ((rc = ix->alloc(&ix->int_rf2, (size_t)ix->ld_i2))) return rc;
      if ((rc = ix->upload(&ix->int_rowid, rowid, s))) return rc;
      for (size_t g = 0; g < segs.size(); ++g) {
        const int i0 = segs[g].first, n = segs[g].second - segs[g].first;
        HIPCHK(launch_int_prep(mean, var, dim, d_int_nodes + i0, n, ix->iso_c, ix->logdet_int + i0, ix->par_int + i0,
                               ix->w_int + i0, DP, ix->DPB2, round_up(n, kFgTile),
                               ix->int_Mb2 + (size_t)seg_row[g] * ix->DPB2, ix->int_rf2 + seg_row[g],
                               ix->int_Ar + (size_t)i0 * DP, ix->int_Br + (size_t)i0 * DP, gamma2, s));
      }
    }
    HIPCHK(hipStreamSynchronize(s));   // the rowid host vector is freed on return
    ix->int_bounds = true;
  }
  if ((rc = build_prune(ix.get(), mean, var, int_nodes, par_int, w_int, rows, int_id, meta, row_par, row_flags, s)))
    return rc;
  if ((rc = ix->alloc(&ix->dummy, 64))) return rc;
  // the per-call path's int8 row panel is built here, with the index, when its policy
  // holds (flat trees, >= kI8MinBytes of int8 rows, room on the device): no allocation or
  // first-call latency inside a query
  if (ix->NL_iso > 0 && !use_int_bounds(ix.get())) (void)ensure_i8(ix.get(), s);
  HIPCHK(hipStreamSynchronize(s));
  *out = ix.release();
  return CWQ_OK;
}

int create_args_ok(int64_t n_nodes, int32_t dim, const float* mean, const int64_t* parent,
                   const int64_t* node_of_sentence, int64_t n_sent, cwq_index** out) {
  if (!out) return fail(CWQ_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n_nodes <= 0 || dim <= 0 || !mean || !parent) return fail(CWQ_ERR_ARG, "empty tree or NULL inputs");
  if (n_nodes >= (int64_t)INT32_MAX / 2) return fail(CWQ_ERR_ARG, "too many nodes");
  if (n_sent < 0 || (n_sent > 0 && !node_of_sentence)) return fail(CWQ_ERR_ARG, "bad sentence map");
  return CWQ_OK;
}
}  // namespace

extern "C" int cwq_index_create(int device, int64_t n_nodes, int32_t dim, const float* mean, const float* var,
                                const int64_t* parent, const int64_t* node_of_sentence, int64_t n_sent,
                                const double* level_w, int32_t n_w, void* stream, cwq_index** out) {
  int rc = create_args_ok(n_nodes, dim, mean, parent, node_of_sentence, n_sent, out);
  if (rc) return rc;
  if (!var) return fail(CWQ_ERR_ARG, "var is NULL");
  DevGuard dg(device);
  const VarSrc vs{var, nullptr, nullptr, nullptr};
  return index_create_impl(device, n_nodes, dim, mean, vs, parent, node_of_sentence, n_sent, level_w, n_w,
                           (hipStream_t)stream, out);
}

extern "C" int cwq_index_create_cv(int device, int64_t n_nodes, int32_t dim, const float* mean, const float* var_row,
                                   const int64_t* an_nodes, int64_t n_an, const float* an_var, const int64_t* parent,
                                   const int64_t* node_of_sentence, int64_t n_sent, const double* level_w, int32_t n_w,
                                   void* stream, cwq_index** out) {
  int rc = create_args_ok(n_nodes, dim, mean, parent, node_of_sentence, n_sent, out);
  if (rc) return rc;
  if (!var_row || n_an < 0 || (n_an > 0 && (!an_nodes || !an_var))) return fail(CWQ_ERR_ARG, "bad compact var");
  std::vector<int> an_map(n_nodes, -1);
  for (int64_t j = 0; j < n_an; ++j) {
    const int64_t nd = an_nodes[j];
    if (nd < 0 || nd >= n_nodes) return fail(CWQ_ERR_ARG, "an_nodes out of range");
    if (an_map[nd] >= 0) return fail(CWQ_ERR_ARG, "an_nodes lists a node twice");
    an_map[nd] = (int)j;
  }
  DevGuard dg(device);
  hipStream_t s = (hipStream_t)stream;
  int* d_map = nullptr;
  if (hipMalloc(&d_map, (size_t)n_nodes * sizeof(int)) != hipSuccess)
    return fail(CWQ_ERR_OOM, "hipMalloc failed (compact var map)");
  if (hipMemcpyAsync(d_map, an_map.data(), (size_t)n_nodes * sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess) {
    (void)hipFree(d_map);
    return fail(CWQ_ERR_HIP, "compact var map upload failed");
  }
  const VarSrc vs{nullptr, var_row, d_map, an_var};
  rc = index_create_impl(device, n_nodes, dim, mean, vs, parent, node_of_sentence, n_sent, level_w, n_w, s, out);
  (void)hipStreamSynchronize(s);   // the build kernels read the map (an error path may return early)
  (void)hipFree(d_map);
  return rc;
}

extern "C" int cwq_index_destroy(cwq_index* idx) {
  if (!idx) return CWQ_OK;
  DevGuard dg(idx->device);
  delete idx;
  return CWQ_OK;
}

extern "C" int cwq_index_info(const cwq_index* idx, int64_t* o) {
  if (!idx || !o) return fail(CWQ_ERR_ARG, "NULL argument");
  o[0] = idx->n_nodes;
  o[1] = idx->D;
  o[2] = idx->n_sent;
  o[3] = idx->NI;
  o[4] = idx->NL;
  o[5] = idx->NL_iso;
  o[6] = idx->max_depth;
  o[7] = (int64_t)idx->bytes;
  return CWQ_OK;
}

extern "C" int cwq_index_filter_info(const cwq_index* idx, int64_t* o) {
  if (!idx || !o) return fail(CWQ_ERR_ARG, "NULL argument");
  o[0] = idx->grp_mode ? 1 : 0;
  o[1] = idx->G;
  o[2] = idx->n_grp_rows;
  o[3] = idx->i8_state > 0 ? 1 : 0;
  return CWQ_OK;
}

extern "C" int cwq_last_lazy_stats(const cwq_index* idx, int64_t* o) {
  if (!idx || !o) return fail(CWQ_ERR_ARG, "NULL argument");
  o[0] = idx->lazy_stats[0];
  o[1] = idx->lazy_stats[1];
  return CWQ_OK;
}

extern "C" int cwq_index_cut_info(const cwq_index* idx, int64_t* o) {
  if (!idx || !o) return fail(CWQ_ERR_ARG, "NULL argument");
  o[0] = (int64_t)idx->cut_centre.size();
  o[1] = idx->cut_centre.empty() ? 0 : idx->cut_top;
  o[2] = idx->cut_maxdep;
  int64_t n_ok = 0;
  for (char c : idx->cut_ok) n_ok += c ? 1 : 0;
  o[3] = n_ok;
  return CWQ_OK;
}

// Scan configuration of one query call (cwq_kernels.hip scan_cfg_begin): fixed from the
// call's total query count, so every chunk and workspace estimate of the call agrees.
struct ScanCfgScope {
  explicit ScanCfgScope(int64_t nq) { scan_cfg_begin(nq); }
  ~ScanCfgScope() { scan_cfg_end(); }
};

// ---------------------------------------------------------------------------
// Query orchestration
// ---------------------------------------------------------------------------
namespace {

constexpr int kQPad = 128;   // queries are padded to a multiple of the largest query block

struct Chunk {
  int nq = 0;           // valid queries
  int64_t nq_pad = 0;
  float* X = nullptr;   // [nq_pad][DP]
  float *S_int = nullptr, *P = nullptr, *BF = nullptr, *LPF = nullptr;   // [nq_pad][NI]
  // P / S_int layout (pidx): query-major [q][ldP] (the exact pass); node-major [node][nq_pad]
  // after the path-sum bounds (run_internal_bounds)
  int64_t ldP = 1;
  int pT = 0;
  const float4* qi2 = nullptr;   // path-sum bounds: the queries' [x'^2, x'] norms (PathB)
  // group-centred rows (grp_mode): the filters' prefix tables [nq_pad][NI] -- Fast
  // [Pg_lo, Pg_hi] and categorize [Pc_lo, Pc_hi] -- and the per-(query, group) shifts
  float *Pg_lo = nullptr, *Pg_hi = nullptr, *Pc_lo = nullptr, *Pc_hi = nullptr;
  double* gsh = nullptr;
  float* Tseed = nullptr;   // group pruning's seed threshold [nq] (a lower bound of tau_K), or none
  int grp_done = -1;   // the group tables run_internal's fused pass wrote: -1 none, 0 Fast, 1 + categorize
};

// The group-centred rows' prefix tables of a chunk (after the exact internal pass wrote
// c.P): q = the chunk's [nq][D] queries.  No-op without grp_mode.
int group_tables(cwq_index* ix, Chunk& c, const float* q, bool cat, hipStream_t s) {
  if (!ix->grp_mode || ix->NI == 0) return CWQ_OK;
  if (c.grp_done >= (cat ? 1 : 0)) return CWQ_OK;   // written by run_internal's fused pass
  HIPCHK(launch_group_prefixes(q, c.nq, ix->D, ix->iso_c, ix->grp_c, ix->G, c.P, c.ldP, ix->NI, ix->grp_par, ix->grp_F,
                               ix->grp_Fc, c.gsh, c.Pg_lo, c.Pg_hi, cat ? c.Pc_lo : nullptr, cat ? c.Pc_hi : nullptr,
                               s));
  return CWQ_OK;
}

// Group pruning (cwq_prune.hip) of a Fast chunk: on by default where the index built its
// constants (build_prune); CWQ_GROUP_PRUNE=0 turns it off per call (in-process A/Bs).
bool use_prune(const cwq_index* ix) {
  if (!ix->prune_ok) return false;
  const char* e = getenv("CWQ_GROUP_PRUNE");
  return !(e && *e && atoi(e) == 0);
}
size_t prune_bytes_per_query(const cwq_index* ix) { return ix->prune_ok ? (size_t)ix->G * 36 + 16 : 0; }

// The pruned Fast chunk's internal pass, in place of run_internal + group_tables (four
// launches, cwq_prune.hip): the group shifts, the bound terms, the root, KUB and g* (head);
// g*'s exact pass over many workgroups; g*'s tables, the seed threshold from its sample rows,
// the stage-B pairs and the sentinel fill; stage B.  K: the call's top-K.  T0 (optional): the seed is
// also written there (the per-call filter's threshold: no probe pass).
int prune_internal(cwq_index* ix, Chunk& c, const float* q, int K, Bump& b, hipStream_t s, float* T0 = nullptr,
                   int64_t ldT0 = 0, int* live = nullptr) {
  const int nq = c.nq, G = ix->G;
  PruneArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.nq = nq;
  pa.G = G;
  pa.NI = ix->NI;
  pa.DP = ix->DP;
  pa.D = ix->D;
  pa.K = K;
  pa.ldS = ix->NI;
  pa.q = q;
  pa.X = c.X;
  pa.c0 = ix->iso_c;
  pa.cent = ix->grp_c;
  pa.Ar = ix->int_Ar;
  pa.Br = ix->int_Br;
  pa.par_int = ix->par_int;
  pa.w_int = ix->w_int;
  pa.logdet_int = ix->logdet_int;
  pa.gint = ix->prn_gint;
  pa.gi_ptr = ix->gi_ptr;
  pa.gi_nodes = ix->gi_nodes;
  pa.gb = ix->gbound;
  pa.kpart = b.take<double>((size_t)3 * c.nq_pad * G);
  pa.S = c.S_int;
  pa.P = c.P;
  pa.Plo = c.Pg_lo;
  pa.Phi = c.Pg_hi;
  pa.grp = ix->grp_par;
  pa.F = ix->grp_F;
  pa.sh = c.gsh;
  pa.fillP = ix->NL_an > 0 ? 1 : 0;
  pa.kub = b.take<float>((size_t)c.nq_pad * G);
  pa.gstar = b.take<int>((size_t)c.nq_pad);
  pa.pairs = b.take<int2>((size_t)c.nq_pad * G);
  pa.ctr = ix->prune_ctr;   // the handle's (calls on it are serialised): [4] survives a fallback re-run
  pa.gs_ptr = ix->gs_ptr;
  pa.gs_rows = ix->gs_rows;
  pa.Mf = ix->iso_Mf;
  pa.meta = ix->row_meta;
  pa.row_par = ix->row_par;
  c.Tseed = b.take<float>((size_t)c.nq_pad);
  pa.Tseed = c.Tseed;
  pa.T0 = T0;
  pa.ldT0 = ldT0;
  pa.gnodes_max = ix->prn_gmax;
  pa.gi_dep = ix->gi_dep;
  pa.gi_ppos = ix->gi_ppos;
  pa.gmaxdep = ix->prn_maxdep;
  pa.gmindep = ix->prn_mindep;
  pa.top_nodes = ix->top_nodes;
  pa.top_ppos = ix->top_ppos;
  pa.top_dep = ix->top_dep;
  pa.n_top = ix->n_top;
  pa.top_maxdep = ix->top_maxdep;
  pa.grp_tpos = ix->grp_tpos;
  if (live) {   // the per-call filter's live block list (count in ctr[5])
    pa.blk_grp = ix->blk_grp;
    pa.nblk = ((int64_t)ix->NL_iso + 15) / 16;
    pa.live = live;
  }
  HIPCHK(launch_prune(pa, ix->cus, ix->prune_nq == 0, s));   // the call's first pruned chunk resets the total
  if (getenv("CWQ_PRUNE_DEBUG")) {   // diagnostics: the first queries' bounds and thresholds
    const int n = std::min(nq, 3);
    std::vector<float> kub((size_t)n * G), th(n);
    std::vector<int> gs(n), ctr(8);
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(kub.data(), pa.kub, kub.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(gs.data(), pa.gstar, n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ctr.data(), pa.ctr, 32, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(th.data(), pa.Tseed, n * 4, hipMemcpyDeviceToHost));
    fprintf(stderr, "[prune] nq %d G %d pairs %d total %d\n", nq, G, ctr[0], ctr[4]);
    for (int i = 0; i < n; ++i) {
      float mx = -INFINITY;
      for (int g = 0; g < G; ++g)
        if (g != gs[i]) mx = std::max(mx, kub[(size_t)i * G + g]);
      fprintf(stderr, "[prune] q %d T %g g* %d kub* %g others max %g\n", i, th[i], gs[i],
              gs[i] >= 0 ? kub[(size_t)i * G + gs[i]] : NAN, mx);
    }
  }
  c.grp_done = 0;   // the Fast tables are written (group_tables is a no-op)
  ix->prune_nq += nq;
  return CWQ_OK;
}

// The path-sum dots of a chunk after run_internal_bounds (int_path), or none.
PathB path_b(const cwq_index* ix, const Chunk& c) {
  if (c.pT && ix->int_path && c.qi2 && ix->int_nrf) return PathB{c.P, c.ldP, c.qi2, ix->int_nrf};
  return PathB{nullptr, 0, nullptr, nullptr};
}

// Query blocks of a launch; a multiple of 8 under the XCD-aware mapping (the
// extra blocks exit at once).
int n_qblocks_for(int64_t nq, int kl) {
  const int qpb = scan_queries_per_block(kl);
  const int n = (int)((nq + qpb - 1) / qpb);
  // XCD-aware mapping needs a multiple of 8 blocks; below 8 the padding blocks would be
  // 7/8 of the grid and of the slab count chosen for it, so small calls map plainly
  return scan_xcd_map() && n >= 8 ? (int)round_up(n, 8) : n;
}

// Choose the slab split of a segment: enough workgroups for >= ~5 waves of the
// resident grid, with the last wave as full as possible (tail balance).
int pick_nslab(const cwq_index* ix, int nrows, int n_qblocks, int kl = 16) {
  if (nrows <= 0) return 0;
  const int max_slab = (int)std::max<int64_t>(1, round_up(nrows, kWave) / 256);
  const int64_t slots = (int64_t)ix->cus * scan_wgs_per_cu(kl);
  int best = 1;
  double best_fill = -1.0;
  for (int r = 5; r <= 10; ++r) {
    const int n = (int)std::max<int64_t>(1, std::min<int64_t>(max_slab, r * slots / std::max(1, n_qblocks)));
    const int64_t wgs = (int64_t)n * n_qblocks;
    const int64_t rounds = (wgs + slots - 1) / slots;
    const double fill = (double)wgs / (double)(rounds * slots);
    if (fill >= best_fill - 1e-9) {
      best_fill = fill;
      best = n;
    }
  }
  return best;
}

ScanArgs base_args(const cwq_index* ix, const Chunk& c) {
  ScanArgs a;
  memset(&a, 0, sizeof(a));
  a.DP = ix->DP;
  a.nq = c.nq;
  a.meta = ix->row_meta;
  a.par = ix->row_par;
  a.flags = ix->row_flags;
  a.P = c.P ? c.P : ix->dummy;   // query-major: the scans run with the exact pass's P (never after pT bounds)
  a.ldP = std::max(ix->NI, 1);
  a.xcd_map = scan_xcd_map();
  return a;
}

// Internal nodes: raw sums -> P (path prefix), BF (bottleneck), LPF (full lp).
// bf_lpf: also the path bottleneck BF and full lp LPF (categorize / log_prob); the fast
// keys need only P.
// The raw sums -> prefixes step of run_internal: one prefix_level_kernel launch per level,
// or (several levels, a few queries, shallow trees) internal_chain_kernel -- one thread per
// (query, node) down its path, same values -- which also writes the group-centred rows'
// prefix tables when q (the caller's queries) is given: grp_cat 0 Fast, 1 + categorize.
constexpr int kChainMaxQ = 64, kChainMaxDepth = 16;
int internal_prefixes(cwq_index* ix, Chunk& c, hipStream_t s, float* BF, float* LPF, float dfull, const float* q,
                      int grp_cat) {
  const char* fe = getenv("CWQ_INT_FINISH");
  const bool fin = ix->levels.size() > 1 && c.nq <= kChainMaxQ && ix->max_depth <= kChainMaxDepth &&
                   !(fe && *fe && atoi(fe) == 0);
  if (!fin) {
    for (auto& lv : ix->levels)
      HIPCHK(launch_prefix_level(c.S_int, ix->NI, c.nq, lv.first, lv.second, ix->par_int, ix->w_int, ix->logdet_int,
                                 dfull, c.P, BF, LPF, s));
    return CWQ_OK;
  }
  IntFinishArgs f;
  memset(&f, 0, sizeof(f));
  f.S = c.S_int;
  f.ldS = ix->NI;
  f.nq = c.nq;
  f.NI = ix->NI;
  f.lv0 = ix->d_lv;
  f.nlev = (int)ix->levels.size();
  f.par_int = ix->par_int;
  f.w_int = ix->w_int;
  f.logdet_int = ix->logdet_int;
  f.dfull = dfull;
  f.P = c.P;
  f.BF = BF;
  f.LPF = LPF;
  const bool grp = q && grp_cat >= 0 && ix->grp_mode && c.Pg_lo && ix->G > 0;
  if (grp) {
    f.q = q;
    f.D = ix->D;
    f.c0 = ix->iso_c;
    f.cent = ix->grp_c;
    f.G = ix->G;
    f.grp = ix->grp_par;
    f.F = ix->grp_F;
    f.Fc = ix->grp_Fc;
    f.sh = c.gsh;
    f.Plo = c.Pg_lo;
    f.Phi = c.Pg_hi;
    f.Pclo = grp_cat ? c.Pc_lo : nullptr;
    f.Pchi = grp_cat ? c.Pc_hi : nullptr;
  }
  HIPCHK(launch_internal_finish(f, s));
  if (grp) c.grp_done = grp_cat;
  return CWQ_OK;
}

int run_internal(cwq_index* ix, Chunk& c, hipStream_t s, bool bf_lpf = true, const float* q = nullptr,
                 int grp_cat = -1) {
  float* BF = bf_lpf ? c.BF : nullptr;
  float* LPF = bf_lpf ? c.LPF : nullptr;
  if (ix->NI == 0) return CWQ_OK;
  const float dfull = (float)((double)ix->D * (double)logf(2.0f * (float)M_PI));
  if (ix->NI <= kWave && (size_t)ix->DP * 8 <= 65536) {   // a few internal nodes: lane = query, same arithmetic
    HIPCHK(launch_int_small(c.X, ix->int_A, ix->int_B, ix->ld_int, ix->NI, ix->DP, c.nq, c.S_int, ix->NI, s));
    return internal_prefixes(ix, c, s, BF, LPF, dfull, q, grp_cat);
  }
  ScanArgs a = base_args(ix, c);
  // raw sums need no top-k list: the hot (list width 16, two rows per lane) configuration
  const int kl = 16, tq = scan_tq(kl);
  a.ld = ix->ld_int;
  a.nrows = ix->NI;
  a.nrows_pad = (int)round_up(ix->NI, kWave);
  a.n_qblocks = n_qblocks_for(c.nq, kl);
  const int nslab = pick_nslab(ix, ix->NI, a.n_qblocks, kl);
  a.rows_per_slab = (int)round_up((a.nrows_pad + nslab - 1) / nslab, scan_rows_per_tile(kl));
  const int nslab2 = (a.nrows_pad + a.rows_per_slab - 1) / a.rows_per_slab;
  a.out = c.S_int;
  a.ldo = ix->NI;
  const char* rse = getenv("CWQ_RAW_SPLIT");   // 0: the scan kernel for one query too (A/B)
  if (c.nq == 1 && (size_t)(ix->DP / 16) * kWave * 4 <= 65536 && !(rse && *rse && atoi(rse) == 0))
    HIPCHK(launch_raw_split(c.X, ix->int_A, ix->int_B, a, s));
  else
    HIPCHK(launch_scan(false, EPI_RAW, false, kl, c.X, ix->int_A, ix->int_B, a, nslab2, s));
  return internal_prefixes(ix, c, s, BF, LPF, dfull, q, grp_cat);
}

int fg_order();
void fg_groups(int n_qt, int& qg, int& rg);

// Filter paths on hierarchical trees: bounded internal prefixes instead of the exact
// internal pass (CWQ_INT_BOUND=0 disables).  Anisotropic leaf rows need exact prefixes
// (the exact scan reads them), so such trees keep the exact pass.
bool use_int_bounds(const cwq_index* ix) {
  // group-centred rows need the exact prefixes (their group terms are folded into them)
  if (!ix->int_bounds || ix->NL_an > 0 || ix->grp_mode) return false;
  const char* e = getenv("CWQ_INT_BOUND");
  return !(e && *e && atoi(e) == 0);
}

size_t int_bounds_bytes(const cwq_index* ix, int64_t nqf) {
  return ix->int_bounds ? (size_t)nqf * ix->DPB2 * 2 + (size_t)nqf * 16 + (size_t)nqf * 4 + 5 * 256 : 0;
}

// Internal nodes by bounds: c.P <- lower, c.S_int <- upper bounds of the path prefix of
// the internal nodes the Fast filter reads (int_path: the leaf parents and the root;
// otherwise every internal node), the root exact in both.  q: the caller's [nq][D] queries.
int run_internal_bounds(cwq_index* ix, Chunk& c, const float* q, int64_t nqf, Bump& b, hipStream_t s) {
  uint16_t* Xb2 = b.take<uint16_t>((size_t)nqf * ix->DPB2);
  float4* qinfo2 = b.take<float4>(nqf);
  float* Sroot = b.take<float>(nqf);
  int* tctr = b.take<int>(64);
  HIPCHK(launch_query_prep2(q, c.nq, ix->D, ix->iso_c, ix->DP, ix->DPB2, nqf, Xb2, qinfo2, s));
  HIPCHK(launch_int_small(c.X, ix->int_A, ix->int_B, ix->ld_int, 1, ix->DP, c.nq, Sroot, 1, s));   // root, exact
  FgArgs g;
  memset(&g, 0, sizeof(g));
  g.DPB = ix->DPB2;
  g.nq = c.nq;
  g.n_qt = (int)(nqf / kFgTile);
  fg_groups(g.n_qt, g.qgroups, g.rgroups);
  g.qinfo = qinfo2;
  g.order = fg_order();
  g.tctr = tctr;
  g.rf = ix->int_rf2;
  g.tf = ix->iso_tf;
  g.P = ix->dummy;
  g.ldP = 1;
  g.ldq = nqf;
  g.mode = 2;
  g.path_sum = ix->int_path ? 1 : 0;
  g.n_rt = (int)(ix->ld_i2 / kFgTile);
  g.lb = c.P;
  g.lb_hi = c.S_int;
  g.ldlb = std::max(ix->NI, 1);
  if (ix->int_path) {   // node-major lines of nq_pad queries (the chunk's [nq_pad][NI] space): dots
    g.pT = 1;
    g.lb_hi = nullptr;
    g.ldlb = c.nq_pad;
    c.pT = 1;
    c.ldP = c.nq_pad;
    c.qi2 = qinfo2;
  }
  g.Sroot = Sroot;
  g.root_w = ix->root_w;
  g.root_ld = ix->root_ld;
  g.row_id = ix->int_rowid;
  g.nrows = (int)ix->ld_i2;
  const int nqb = (c.nq + 15) / 16;
  if (ix->int_path && c.nq <= kStreamMaxQ && stream_lds_bytes(nqb, ix->DPB2) <= (size_t)kStreamMaxLds &&
      !getenv("CWQ_INT_STREAM_OFF")) {
    // a few queries (the per-call path): the path-sum rows streamed once against <= 64
    // queries (stream_kernel<2>) instead of 256-query MFMA tiles that are mostly padding;
    // the same dots and root lines
    StreamArgs sa;
    memset(&sa, 0, sizeof(sa));
    sa.DPB = ix->DPB2;
    sa.nq = c.nq;
    sa.nqb = nqb;
    sa.nrows = ix->ld_i2;
    sa.K = 1;
    sa.Xb = Xb2;
    sa.qinfo = qinfo2;
    sa.Mb = ix->int_Mb2;
    sa.rf = ix->int_rf2;
    sa.row_id = ix->int_rowid;
    sa.Sroot = Sroot;
    sa.root_w = ix->root_w;
    sa.root_ld = ix->root_ld;
    sa.pout = c.P;
    sa.ldpout = g.ldlb;
    const char* iwe = getenv("CWQ_INT_STREAM_WGS");   // workgroups per CU (A/B; read per call)
    HIPCHK(launch_stream(sa, 2, ix->cus * (iwe && atoi(iwe) > 0 ? std::min(4, atoi(iwe)) : 1), s));
  } else {
    HIPCHK(hipMemsetAsync(tctr, 0, 64 * 4, s));   // the tile claim counters (the stream pass has none)
    HIPCHK(launch_fgemm(Xb2, ix->int_Mb2, g, ix->cus, s));
  }
  if (!ix->int_path)
    for (size_t lv = 2; lv < ix->levels.size(); ++lv)
      HIPCHK(launch_prefix_bounds(c.P, c.S_int, std::max(ix->NI, 1), c.nq, ix->levels[lv].first,
                                  ix->levels[lv].second, ix->par_int, ix->w_int, ix->logdet_int, Sroot, s));
  return CWQ_OK;
}

IntChain int_chain(const cwq_index* ix) { return IntChain{ix->int_Ar, ix->int_Br, ix->par_int, ix->w_int, ix->logdet_int}; }

// Fast top-K over a small isotropic segment with many queries: the lane-per-query scan
// (scan_small_kernel).
bool small_scan_fits(const cwq_index* ix, int K) {   // size limits only (workspace sizing)
  return ix->NL_iso > 0 && ix->NL_iso <= kSmallScanMaxRows && K <= kSmallScanMaxK;
}
bool use_small_scan(const cwq_index* ix, int64_t nq, int K) {
  if (!small_scan_fits(ix, K) || nq < kSmallScanMinQ) return false;
  const char* e = getenv("CWQ_SCAN_SMALL");   // 0: never, 1: whenever it applies
  if (e && *e) return atoi(e) != 0;
  // by wave counts: the row-sliced scan's slabs are >= 256 rows, so on a small corpus it
  // has few waves, each waiting on its scalar query loads; the lane-per-query scan wins
  // with ~0.9x as many waves, or with half as many once it fills the SIMDs
  // (measured crossover, profiles/r02_small_scan.log)
  const int nqb = n_qblocks_for(nq, 16);
  const int64_t nqb_real = (nq + scan_queries_per_block(16) - 1) / scan_queries_per_block(16);
  const int64_t rs_waves = (int64_t)pick_nslab(ix, ix->NL_iso, nqb) * nqb_real * kWavesPerWG;
  const int64_t small_waves = (nq + kWave - 1) / kWave * small_scan_slabs(nq, ix->NL_iso);
  return small_waves * 10 >= rs_waves * 9 || (small_waves * 2 >= rs_waves && small_waves >= 4 * (int64_t)ix->cus);
}

// One scan over both leaf-row segments.
// seg_mask: bit 0 = isotropic segment, bit 1 = anisotropic; TOPK lists start at
// slab_off0 (slots before it are filled by the caller).
int run_leaf_scan(cwq_index* ix, const Chunk& c, int epi, bool cat, int kl, float dconst, float* out, int64_t ldo,
                  float* pkey, float* paux, int* prow, int K, int* nslab_total_out, hipStream_t s,
                  int seg_mask = 3, int slab_off0 = 0, int max_lists = INT_MAX) {
  if (c.pT && ((seg_mask & 1) ? ix->NL : ix->NL_an) > 0)   // the scans read query-major exact prefixes
    return fail(CWQ_ERR_ARG, "leaf scan after node-major prefix bounds (internal error)");
  const int tq = scan_tq(kl);
  const int nqb = n_qblocks_for(c.nq, kl);
  const bool small = epi == EPI_TOPK && !cat && (seg_mask & 1) && use_small_scan(ix, c.nq, K);
  struct Seg {
    bool iso;
    int n;
    int base;
    const float *A, *B;
    int64_t ld;
  } segs[2] = {{true, ix->NL_iso, 0, ix->iso_M, ix->iso_M, ix->ld_iso},
               {false, ix->NL_an, ix->NL_iso, ix->an_A, ix->an_B, ix->ld_an}};
  int ns[2], rps[2];
  for (int i = 0; i < 2; ++i) {
    ns[i] = 0;
    rps[i] = 0;
    if (!((seg_mask >> i) & 1)) segs[i].n = 0;
    if (segs[i].n == 0) continue;
    const int tile = scan_rows_per_tile(kl);
    const int npad = (int)round_up(segs[i].n, kWave);
    if (i == 0 && small) {
      ns[0] = small_scan_slabs(c.nq, segs[0].n);
      continue;
    }
    const int n = pick_nslab(ix, segs[i].n, nqb);
    rps[i] = (int)round_up((npad + n - 1) / n, tile);   // slabs hold whole tiles: no row scanned twice
    ns[i] = (npad + rps[i] - 1) / rps[i];
  }
  const int lps = scan_lists_per_slab(kl);
  const int nslab_total = slab_off0 + (small ? ns[0] : ns[0] * lps) + ns[1] * lps;
  if (nslab_total > max_lists)
    return fail(CWQ_ERR_ARG, "internal: partial-list buffer too small (" + std::to_string(nslab_total) +
                                 " lists needed, " + std::to_string(max_lists) + " allocated)");
  if (nslab_total_out) *nslab_total_out = nslab_total;
  int slab_off = slab_off0;
  for (int i = 0; i < 2; ++i) {
    if (segs[i].n == 0) continue;
    ScanArgs a = base_args(ix, c);
    // categorize keys min(BF[parent], lp) read the path BOTTLENECK (the Fast keys read the
    // path prefix P); with P here the key was min(prefix, lp), equal to the bottleneck
    // key only while the leaf's lp stays below its ancestors' (a near-duplicate query
    // broke the top-R list's order)
    if (cat) a.P = c.BF ? c.BF : ix->dummy;
    a.ld = segs[i].ld;
    a.nrows = segs[i].n;
    a.nrows_pad = (int)round_up(segs[i].n, kWave);
    a.rows_per_slab = rps[i];
    a.n_qblocks = nqb;
    a.seg_base = segs[i].base;
    a.meta = ix->row_meta + segs[i].base;
    a.par = ix->row_par + segs[i].base;
    a.flags = ix->row_flags + segs[i].base;
    a.dconst = dconst;
    a.out = out;
    a.ldo = ldo;
    a.out_base = segs[i].base;
    a.pkey = pkey;
    a.paux = paux;
    a.prow = prow;
    a.nslab_total = nslab_total;
    a.slab_off = slab_off;
    a.K = K;
    if (i == 0 && small) {
      HIPCHK(launch_scan_small(c.X, segs[0].A, a, ns[0], s));
      slab_off += ns[0];
      continue;
    }
    HIPCHK(launch_scan(segs[i].iso, epi, cat, kl, c.X, segs[i].A, segs[i].B, a, ns[i], s));
    slab_off += ns[i] * lps;
  }
  return CWQ_OK;
}

// Workspace for one chunk: X + internal arrays.
// Workspace of one chunk: X + the [nq][NI] internal arrays -- S_int and P always; BF and
// LPF (path bottleneck, full log_prob) only for categorize / log_prob (`full`).
size_t group_bytes_per_query(const cwq_index* ix) {
  return ix->grp_mode ? (size_t)ix->G * 16 + (size_t)4 * std::max(ix->NI, 1) * 4 + 5 * 256 + prune_bytes_per_query(ix) : 0;
}
size_t chunk_bytes(const cwq_index* ix, int64_t nq_pad, bool full = true) {
  return (size_t)nq_pad * ix->DP * 4 + (full ? 4 : 2) * (size_t)nq_pad * std::max(ix->NI, 1) * 4 + 8 * 256 +
         (size_t)nq_pad * group_bytes_per_query(ix);
}

void carve_chunk(cwq_index* ix, Bump& b, Chunk& c, int nq, bool full = true) {
  c.nq = nq;
  c.nq_pad = round_up(nq, kQPad);
  c.X = b.take<float>((size_t)c.nq_pad * ix->DP);
  c.ldP = std::max(ix->NI, 1);
  c.pT = 0;
  if (ix->NI > 0) {
    const size_t n = (size_t)c.nq_pad * ix->NI;
    c.S_int = b.take<float>(n);
    c.P = b.take<float>(n);
    if (full) {
      c.BF = b.take<float>(n);
      c.LPF = b.take<float>(n);
    }
    if (ix->grp_mode) {
      c.gsh = b.take<double>((size_t)2 * c.nq_pad * ix->G);   // the shifts, then their error bounds
      c.Pg_lo = b.take<float>(n);
      c.Pg_hi = b.take<float>(n);
      c.Pc_lo = b.take<float>(n);
      c.Pc_hi = b.take<float>(n);
    }
  }
}

// Query-chunk size that keeps the per-chunk workspace within the budget (16 GiB by
// default -- 288 GB of HBM hold it beside the largest indexes; CWQ_WS_BUDGET_MB; at
// least 128 queries).
int64_t chunk_queries(const cwq_index* ix, int64_t nq, size_t per_query_extra, bool full = true) {
  const size_t per_q = (size_t)ix->DP * 4 + (full ? 4 : 2) * (size_t)std::max(ix->NI, 1) * 4 + per_query_extra +
                       group_bytes_per_query(ix);
  // budget: CWQ_WS_BUDGET_MB, else 40% of what the device has free (plus the workspace
  // already held), between 2 and 48 GiB -- one chunk for 10k queries over trees with
  // ~350k internal nodes (whose [lo, hi] prefix matrices alone are 28 GB), which beats two
  // chunks by 11% (balanced 4/9 tree, 1M x 768)
  // (hipMemGetInfo is a driver query of ~0.3 ms: once per handle, not per call)
  const char* e = getenv("CWQ_WS_BUDGET_MB");
  size_t budget = (size_t)16 << 30;
  if (e && atoll(e) > 0) {
    budget = (size_t)atoll(e) << 20;
  } else if (ix->ws_budget) {
    budget = ix->ws_budget;
  } else {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess)
      budget = std::min<size_t>((size_t)48 << 30, std::max<size_t>((size_t)2 << 30, (fr + ix->ws_size) / 5 * 2));
    const_cast<cwq_index*>(ix)->ws_budget = budget;
  }
  int64_t c = (int64_t)std::max<size_t>(kQPad, budget / std::max<size_t>(per_q, 1));
  c = std::max<int64_t>(kQPad, c / kQPad * kQPad);
  return std::min(nq, c);
}
}  // namespace

namespace {

constexpr int kFiltMinRows = 16384;   // automatic mode: below this the exact scan is as fast
constexpr int kFiltMaxK = 64;         // the filter serves the list-based top-k path (k <= 64)
constexpr int kFgRecPerQ = 512;       // candidate-record slots per query (append buffer)
constexpr int kFgDirPerQ = 256;       // direct-record slots per query (tiles past kFgCap)
// Clustered (group-centred) trees: a query's whole cluster can pass -- categorize keys tie at
// the cluster node's lp for every row of the cluster (~1,000 rows at C2) -- so the record
// buffers hold 4x as many per query (48 KB instead of 12 KB per query).
inline int rec_per_q(const cwq_index* ix) { return ix->grp_mode ? 4 * kFgRecPerQ : kFgRecPerQ; }
inline int dir_per_q(const cwq_index* ix) { return ix->grp_mode ? 4 * kFgDirPerQ : kFgDirPerQ; }

// min_rows: the automatic mode's threshold (the batch filter: kFiltMinRows; the per-call
// stream path pays no batch pipeline and wins from a few hundred rows on -- the exact
// scan's per-call cost on a 1.5k-row tree is its scalar query-slice latency chain, 0.3 ms)
constexpr int kStreamMinRows = 512;
// fast: a Fast call (score_topk), which the auto-mode record can turn off; categorize keeps
// its own rule (its per-call lists still pay on a tree whose Fast filter fails: 500k x 768
// Basic one query per call 4.0 ms with the filter, 8.3 ms without,
// profiles/r05_c500k_probe_v1.log / _v2.log)
bool use_filter(const cwq_index* ix, int k, int min_rows = kFiltMinRows, bool fast = true) {
  if (k > kFiltMaxK || ix->NL_iso == 0 || !ix->iso_Mb) return false;
  int mode = ix->filter;
  if (mode < 0) {
    const char* e = getenv("CWQ_FILTER");
    if (e && *e) mode = atoi(e) ? 1 : 0;
  }
  if (mode < 0) return ix->NL_iso >= min_rows && !(fast && ix->filt_auto_off);
  return mode == 1;
}

// After a Fast call (cwq_last_stats' record): the auto-mode filter record of the index.  The
// exact-scan choice is not for good: after kFiltRetryCalls auto-mode Fast calls on the exact
// scan the record starts afresh and the filter is tried again (an early query mix that
// defeated the bounds costs speed for a while, never for the index's life).
constexpr int kFiltRetryCalls = 64;
void note_filter(cwq_index* ix) {
  if (ix->filter >= 0) return;
  if (ix->stats[2] == 0) {
    if (ix->filt_auto_off && ++ix->filt_off_calls >= kFiltRetryCalls) {
      ix->filt_auto_off = false;
      ix->filt_q = ix->filt_fb = 0;
      ix->filt_off_calls = 0;
    }
    return;
  }
  if (ix->stats[0] <= 0) return;
  ix->filt_q += ix->stats[0];
  ix->filt_fb += ix->stats[1];
  if (ix->filt_q >= 256 && ix->filt_fb * 10 >= ix->filt_q * 9) {
    ix->filt_auto_off = true;
    ix->filt_off_calls = 0;
  }
}

// fgemm launch geometry: query groups over the 8 XCDs (each keeps its query panel in
// L2), row groups for the remaining factor.
int fg_phases() {
  const char* e = getenv("CWQ_FG_PHASES");
  return e && *e ? atoi(e) : 1;
}

// filter phases over the row tiles: cut points at n_rt * f / 1024 for the fractions f in
// CWQ_FG_CUTS (comma separated, increasing, at most 4; default 32,96,256,512: five
// launches, the first over 1/32 of the tiles; in-process A/B vs 1/16,1/4: x1.02 per call)
int fg_phase_cuts(int n_rt, int* cuts) {
  if (n_rt < 16 || !fg_phases()) return 1;
  int f[4] = {32, 96, 256, 512}, nf = 4;
  if (const char* e = getenv("CWQ_FG_CUTS")) {
    nf = 0;
    for (const char* p = e; *p && nf < 4;) {
      const int v = atoi(p);
      if (v > 0 && v < 1024) f[nf++] = v;
      while (*p && *p != ',') ++p;
      if (*p == ',') ++p;
    }
  }
  int n = 1;
  for (int i = 0; i < nf; ++i) {
    const int c = std::max(cuts[n - 1] + 1, (int)((int64_t)n_rt * f[i] / 1024));
    if (c >= n_rt) break;
    cuts[n++] = c;
  }
  cuts[n] = n_rt;
  return n;
}

int fg_order() {   // default: dynamic per-XCD tile claims (measured fastest)
  const char* e = getenv("CWQ_FG_ORDER");
  return e && *e ? atoi(e) : 2;
}

// XCD split of the tiles: qg query groups x rg row groups (qg * rg = 8).  Default: all 8
// XCDs split the queries (each keeps its query panels in its L2 and streams every row
// panel); CWQ_FG_QG = 4 / 2 / 1 caps qg (row panels fetched by fewer XCDs, more query
// panels per XCD).
void fg_groups(int n_qt, int& qg, int& rg) {
  qg = n_qt >= 8 ? 8 : n_qt >= 4 ? 4 : n_qt >= 2 ? 2 : 1;
  if (const char* e = getenv("CWQ_FG_QG")) {
    const int v = atoi(e);
    if ((v == 1 || v == 2 || v == 4) && v < qg) qg = v;
  }
  rg = 8 / qg;
}

int score_topk_impl(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                    hipStream_t s, bool allow_filter);

// Wait for a one-query call's kernels by polling the stream: a blocking
// hipStreamSynchronize issued ~0.3 ms before the work ends falls back to an interrupt
// wait, whose wake-up is a large share of the per-call path's fixed cost.  Polls for at
// most ~20 ms, then blocks.
hipError_t sync_spin(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return hipStreamSynchronize(s);
  }
}

// Queries whose certificate failed: exact scan, results scattered back in place.
int rerun_exact(cwq_index* ix, const float* q, const std::vector<int64_t>& qi, int32_t k, int64_t* ids, float* scores,
                hipStream_t s) {
  // buffers from the handle's fallback region; one gather launch in, one scatter out
  const int64_t n = (int64_t)qi.size();
  const size_t D = (size_t)ix->D;
  const size_t o_tq = round_up(n * 8, 256), o_tid = o_tq + round_up(n * D * 4, 256),
               o_ts = o_tid + round_up((int64_t)n * k * 8, 256), tot = o_ts + round_up((int64_t)n * k * 4, 256);
  int rc = ix->reserve_fb(tot);
  if (rc) return rc;
  char* fb = (char*)ix->fb;
  int64_t* d_idx = (int64_t*)fb;
  float* tq = (float*)(fb + o_tq);
  int64_t* tid = (int64_t*)(fb + o_tid);
  float* ts = scores ? (float*)(fb + o_ts) : nullptr;
  HIPCHK(hipMemcpyAsync(d_idx, qi.data(), n * 8, hipMemcpyHostToDevice, s));
  HIPCHK(launch_copy_rows(q, (int64_t)D, d_idx, tq, (int64_t)D, nullptr, n, (int64_t)D, s));
  if ((rc = score_topk_impl(ix, tq, n, k, tid, ts, s, false))) return rc;
  HIPCHK(launch_copy_rows(tid, 2 * (int64_t)k, nullptr, ids, 2 * (int64_t)k, d_idx, n, 2 * (int64_t)k, s));
  if (scores) HIPCHK(launch_copy_rows(ts, k, nullptr, scores, k, d_idx, n, k, s));
  HIPCHK(hipStreamSynchronize(s));   // qi (pageable host memory) must outlive the upload
  return CWQ_OK;
}

// Small-batch path (cwq_stream.hip): nq <= kStreamMaxQ queries, isotropic rows through
// the stream filter (probe -> filter -> exact rerank), anisotropic rows through the exact
// scan; the reference harness's one-query-per-call mode.  false: not applicable.
bool use_stream(const cwq_index* ix, int64_t nq, int k) {
  if (nq > kStreamMaxQ || k > kFiltMaxK || !ix->iso_Mb) return false;
  if (stream_lds_bytes((int)((nq + 15) / 16), ix->DPB) > (size_t)kStreamMaxLds) return false;
  const char* e = getenv("CWQ_STREAM");
  return !(e && *e && atoi(e) == 0);
}

// The stream filter's int8 row panel (half the bf16 panel's bytes per row; the per-call pass
// is HBM-bound).  Built once, from the fp32 rerank copy, when the device has room for it.
// Used when it pays: the pass saves ~half its HBM time, the wider int8 bounds cost the
// exact rerank ~9x the reranks per query (one workgroup per query).  Measured at D = 768
// (profiles/r03_i8_*): 1M rows nq = 1 341 -> 271 us, nq = 64 385 -> 347 us; 100k rows
// nq = 1 110 -> 126 us (a loss); so by default for an int8 panel of >= kI8MinBytes.
// CWQ_STREAM_I8=0 / 1: off / forced on (read per call, for in-process A/Bs).  The panel
// is built by cwq_index_create when the policy holds there; a call that forces it on an
// index created without it builds it then (A/B and test use only).
constexpr int64_t kI8MinBytes = (int64_t)384 << 20;
bool ensure_i8(cwq_index* ix, hipStream_t s) {
  const char* e = getenv("CWQ_STREAM_I8");
  if ((e && *e && atoi(e) == 0) || ix->grp_mode) return false;   // the int8 rows are root-centred
  if (!(e && *e && atoi(e) == 1) && (int64_t)ix->NL_iso * ix->DPB < kI8MinBytes) return false;
  if (ix->i8_state) return ix->i8_state > 0;
  ix->i8_state = -1;
  if (ix->DPB % 64 || !ix->iso_Mf || !ix->iso_rf) return false;
  const size_t need = (size_t)ix->ld_f * ix->DPB + (size_t)ix->ld_f * sizeof(RowF);
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < need + std::max<size_t>((size_t)4 << 30, tot / 20)) return false;
  if (ix->alloc(&ix->iso_Mq, (size_t)ix->ld_f * ix->DPB) || ix->alloc(&ix->iso_rf8, (size_t)ix->ld_f)) return false;
  if (launch_rows_i8(ix->iso_Mf, ix->DP, ix->D, ix->iso_c, ix->DPB, ix->ld_f, ix->iso_rf, ix->iso_Mq, ix->iso_rf8, s) !=
      hipSuccess)
    return false;
  ix->i8_state = 1;
  return true;
}

// CWQ_SELECT_UNFUSED=1: the per-call path keeps select_kernel (and sb_prep) -- A/B only
bool sel_unfused() {
  const char* e = getenv("CWQ_SELECT_UNFUSED");
  return e && *e && atoi(e) != 0;
}

// Workgroups of the per-call filter pass: one per CU (8 waves); CWQ_STREAM_WGS = m runs m
// per CU (more loads in flight on short passes -- an A/B knob).
int stream_wgs(const cwq_index* ix) {
  const char* e = getenv("CWQ_STREAM_WGS");   // read per call: in-process A/Bs switch it
  const int m = e && atoi(e) > 0 ? std::min(4, atoi(e)) : 1;
  return ix->cus * m;
}

// Workgroups per query of the per-call path's rerank tail (FwExpand::split): after the int8
// pass a query's ~1k-row candidate list reranked by one workgroup leaves the chip idle, so
// up to kFwSplitMax per query, about one per CU in total (C3 one query per call 267 -> 262
// us); the bf16 pass's lists are short and the split's merge costs more than it saves (C2:
// 142 -> 154 us, profiles/r05_c2_probe_envab_v1.log), so one there.  CWQ_FW_SPLIT = n caps it.
constexpr int kFwSplitMax = 32;
int fw_split(const cwq_index* ix, int nq, bool i8) {
  int S = i8 ? std::max(1, std::min(kFwSplitMax, ix->cus / std::max(nq, 1))) : 1;
  if (const char* e = getenv("CWQ_FW_SPLIT"))
    if (atoi(e) > 0) S = std::min(S, atoi(e));
  return S;
}

int stream_topk_impl(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                     hipStream_t s) {
  const int K = k, kl = k <= 16 ? 16 : 64;
  const int nqc = (int)nq;
  const int nqb = (nqc + 15) / 16, nq16 = nqb * 16;
  const int64_t nq_pad = round_up(nqc, kQPad);
  const int nqb_scan = n_qblocks_for(nqc, kl);
  const int slabs = 1 + (pick_nslab(ix, ix->NL_an, nqb_scan) + 1) * scan_lists_per_slab(kl);
  const int capq = kFgCapQ;
  size_t need = chunk_bytes(ix, nq_pad, false) + 64 * 256 + (size_t)nq_pad * ((size_t)slabs * K * 12 + (size_t)K * 12) +
                (size_t)nq16 * ix->DPB * 2 + (size_t)nq16 * 16 + (size_t)64 * nqc * 4 + (size_t)nqc * 4 +
                (size_t)5 * nqc * 4 + (size_t)nqc * capq * 12 + (size_t)nqc * 64 * 16 +
                (size_t)nqc * 4 * (round_up((ix->NL_iso + 15) / 16 + 1, 1024) + 1024) + 32 * 256 +
                int_bounds_bytes(ix, kFgTile) + (size_t)nq16 * ix->DPB + (size_t)nq16 * 16 + 512 +
                (size_t)nqc * kFwSplitMax * 64 * 12 + 3 * 256 + (size_t)((ix->NL_iso + 15) / 16) * 4 + 256;
  const bool ib = use_int_bounds(ix);
  // int8 pass: flat trees, and hierarchical ones for calls of <= 8 queries.  With bounded
  // internal prefixes the ~9x exact reranks pay the exact parent chains too: round 3, b4/L9
  // one query per call 692 -> 1166 us (profiles/r03_i8_ab_hier_*.log); with the split rerank
  // tail and its radix T2 it pays at a few queries (nq 1 / 8: 670 -> 601 / 722 -> 664 us) and
  // not at 64 (1373 -> 3161 us), profiles/r05_percall_b4d9_i8_ab.log.  CWQ_STREAM_I8=1 / 0
  // forces it on / off.
  const char* e8 = getenv("CWQ_STREAM_I8");
  const int e8v = e8 && *e8 ? atoi(e8) : -1;
  const bool i8 = e8v != 0 && (!ib || nqc <= 8 || e8v == 1) && ensure_i8(ix, s);
  int rc;
  if ((rc = ix->reserve(need))) return rc;
  Bump b(ix->ws, ix->ws_size);
  Chunk c;
  carve_chunk(ix, b, c, nqc, false);
  float* pkey = b.take<float>((size_t)nq_pad * slabs * K);
  float* paux = b.take<float>((size_t)nq_pad * slabs * K);
  int* prow = b.take<int>((size_t)nq_pad * slabs * K);
  uint16_t* Xb = b.take<uint16_t>((size_t)nq16 * ix->DPB);
  float4* qinfo = b.take<float4>(nq16);
  int8_t* Xq = i8 ? b.take<int8_t>((size_t)nq16 * ix->DPB) : nullptr;
  float4* qinfo8 = i8 ? b.take<float4>(nq16) : nullptr;
  int* Tb = b.take<int>((size_t)(K + 1) * nqc);   // [K][nq] blocks + [nq] live threshold
  float* T = b.take<float>(nqc);
  int* qcnt = b.take<int>((size_t)5 * nqc + 1);   // [qcnt | ok | n_exact | qover | done | select counter]
  int* okf = qcnt + nqc;
  int* nex = qcnt + 2 * nqc;
  int* qover = qcnt + 3 * nqc;
  int* done = qcnt + 4 * nqc;
  int* sel_ctr = qcnt + 5 * nqc;
  int* crow = b.take<int>((size_t)nqc * capq);
  float* cu = b.take<float>((size_t)nqc * capq);
  float* cl = b.take<float>((size_t)nqc * capq);
  float* lkb = b.take<float>((size_t)nqc * 64);
  int* lrb = b.take<int>((size_t)nqc * 64);
  const int64_t ldlb = round_up((ix->NL_iso + 15) / 16 + 1, 1024) + 1024;   // select reads whole 1024 steps
  float* lb = b.take<float>((size_t)nqc * ldlb);
  float* tl = b.take<float>((size_t)nqc * 64);
  int* tr = b.take<int>((size_t)nqc * 64);
  const int fws = fw_split(ix, nqc, i8);
  float* fsk = b.take<float>((size_t)nqc * fws * 64);
  float* fsa = b.take<float>((size_t)nqc * fws * 64);
  int* fsr = b.take<int>((size_t)nqc * fws * 64);
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[0], s));
  // one fused prep launch when the exact internal pass is small (flat trees: the root)
  bool fused = !ib && ix->NI <= kSbMaxNI && (int)ix->levels.size() <= kSbMaxNI &&
               ((size_t)2 * std::max(ix->DP, ix->DPB) + (size_t)ix->NI * (ix->DP / 16) + ix->NI) * 4 <= 65536 &&
               !getenv("CWQ_SB_UNFUSED");
  SbPrepArgs sp;
  const bool prn = !ib && use_prune(ix);
  int* live = nullptr;   // group pruning: the filter's 16-row blocks
  if (prn) fused = false;
  if (fused) {
    memset(&sp, 0, sizeof(sp));
    sp.q = q;
    sp.nq = nqc;
    sp.D = ix->D;
    sp.DP = ix->DP;
    sp.DPB = ix->DPB;
    sp.nq_pad = c.nq_pad;
    sp.nq16 = nq16;
    sp.X = c.X;
    sp.Xb = Xb;
    sp.qinfo = qinfo;
    sp.Xq = Xq;
    sp.qinfo8 = qinfo8;
    sp.c = ix->iso_c;
    sp.A = ix->int_A;
    sp.B = ix->int_B;
    sp.ld = ix->ld_int;
    sp.NI = ix->NI;
    sp.par_int = ix->par_int;
    sp.w_int = ix->w_int;
    sp.logdet_int = ix->logdet_int;
    sp.P = c.P;
    sp.ldP = std::max(ix->NI, 1);
    sp.qcnt = qcnt;
    sp.nlev = (int)ix->levels.size();
    for (int l = 0; l < sp.nlev && fused; ++l) {
      sp.lv0[l] = ix->levels[l].first;
      if (l > 0 && ix->levels[l].first != ix->levels[l - 1].second) fused = false;   // BFS: contiguous levels
    }
    if (sp.nlev > 0) sp.lv0[sp.nlev] = ix->levels.back().second;
    if (ix->NI > 0 && (!c.P || sp.nlev == 0 || sp.lv0[0] != 0 || sp.lv0[sp.nlev] != ix->NI)) fused = false;
  }
  // flat trees, up to 16 queries, bf16 pass: the prep inside the probe launch (stream_kernel<1>
  // with fprep) -- one launch less, but measured slower (C2 one query per call 101.5 ->
  // 104.9 us: the probe's workgroups all wait for the prep, profiles/r04_percall_ab_c2_v1.log),
  // so opt-in: CWQ_PROBE_PREP=1
  const char* fpe = getenv("CWQ_PROBE_PREP");
  const bool fprep = fused && ix->NI == 1 && nqb == 1 && !i8 && ix->DP <= 1024 && !sel_unfused() &&
                     (fpe && *fpe && atoi(fpe) == 1);
  if (fprep && !ix->sel_ctr)   // the fused select's counter (lives across calls)
    if ((rc = ix->alloc(&ix->sel_ctr, 1))) return rc;
  if (fprep) {
    // re-zeroed on every such call: its last workgroup resets it too, but an aborted launch
    // or one with another grid size would leave it nonzero and later calls would read stale
    // thresholds (this opt-in path only; the default path's counter is zeroed by the prep)
    HIPCHK(hipMemsetAsync(ix->sel_ctr, 0, 4, s));
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[1], s));
  } else if (fused) {
    HIPCHK(launch_sb_prep(sp, s));
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[1], s));
  } else {
    HIPCHK(launch_pad_queries(q, nqc, ix->D, c.X, c.nq_pad, ix->DP, s));
    if (ib) {
      if ((rc = run_internal_bounds(ix, c, q, kFgTile, b, s))) return rc;
    } else if (prn) {
      // the seed threshold goes straight to the filter's T0: no probe pass; the filter pass
      // covers the live blocks only
      live = b.take<int>((size_t)std::max<int64_t>(1, (ix->NL_iso + 15) / 16));
      if ((rc = prune_internal(ix, c, q, K, b, s, tl + (K - 1), 64, live))) return rc;
    } else if ((rc = run_internal(ix, c, s, false, q, 0))) {
      return rc;
    }
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[1], s));
    // the counters (qcnt, qover, done, ..., the fused select's) zeroed by the prep's block 0
    HIPCHK(launch_query_prep(q, nqc, ix->D, ix->iso_c, ix->DPB, nq16, Xb, qinfo, s, qcnt, (int)(5 * nqc + 1)));
    if (i8) HIPCHK(launch_query_prep_i8(q, nqc, ix->D, ix->iso_c, ix->DPB, nq16, Xq, qinfo8, s));
  }
  if ((rc = group_tables(ix, c, q, false, s))) return rc;
  const FiltConsts fc = filt_consts(ix->DPB);
  StreamArgs a;
  memset(&a, 0, sizeof(a));
  a.DPB = ix->DPB;
  a.nq = nqc;
  a.nqb = nqb;
  a.nrows = ix->NL_iso;
  a.K = K;
  a.Xb = Xb;
  a.qinfo = qinfo;
  a.Mb = ix->iso_Mb;
  a.rf = ix->iso_rf;
  a.P = c.P ? c.P : ix->dummy;
  a.pb = ib ? path_b(ix, c) : PathB{nullptr, 0, nullptr, nullptr};
  a.Phi = ib && !a.pb.dot ? c.S_int : nullptr;
  if (ix->grp_mode && c.Pg_lo) {   // group-centred rows: the shifted prefix tables
    a.P = c.Pg_lo;
    a.Phi = c.Pg_hi;
  }
  a.ldP = c.ldP;
  a.pT = c.pT;
  a.eps_n = (float)fc.eps_n;
  a.slack = (float)fc.slack;
  a.Tb = Tb;
  a.Tlive = Tb + (size_t)K * nqc;
  // live threshold (CWQ_STREAM_LIVE=n: refresh every n groups): measured slower at C3 --
  // the publishing atomics cost more than the ~3x fewer candidates save -- so off
  a.live_every = 0;
  if (const char* e = getenv("CWQ_STREAM_LIVE")) a.live_every = std::max(0, atoi(e));
  if (a.live_every > 0) HIPCHK(launch_stream_init(Tb, (K + 1) * nqc, s));   // only the live threshold reads Tb
  a.T = T;
  a.qcnt = qcnt;
  a.qover = qover;
  a.capq = capq;
  a.crow = crow;
  a.cu = cu;
  a.cl = cl;
  // probe: ~3*K*rows/1024 rows (a 16-row group per probe_stride groups), so that the
  // K-th largest probe bound leaves ~1k candidates per query before the live threshold
  // takes over; CWQ_STREAM_PROBE_DIV overrides (groups / div)
  const int64_t ngroups = (ix->NL_iso + 15) / 16;
  int64_t n_probe = std::max<int64_t>((int64_t)3 * K * ngroups / 1024, (int64_t)8 * K);
  if (const char* e = getenv("CWQ_STREAM_PROBE_DIV"))
    if (atoi(e) > 0) n_probe = std::max<int64_t>(ngroups / atoi(e), (int64_t)K);
  n_probe = std::min(n_probe, ngroups);
  a.probe_stride = std::max<int64_t>(1, ngroups / std::max<int64_t>(n_probe, 1));
  a.n_probe = std::min<int64_t>(n_probe, (ngroups + a.probe_stride - 1) / a.probe_stride);
  a.lb = lb;
  a.ldlb = ldlb;
  a.T0 = tl;
  a.ldT0 = 64;
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[4], s));
  const char* lve = getenv("CWQ_PRUNE_LIVE");   // 0: the pass over every block (A/B)
  const bool use_live = live && !(lve && *lve && atoi(lve) == 0);
  // the select runs in the probe launch's last workgroup (one launch less per call);
  // CWQ_SELECT_UNFUSED=1 keeps select_kernel (same thresholds: both run select_wave)
  const bool fsel = !sel_unfused();
  if (fsel) {
    a.sel_ctr = fprep ? ix->sel_ctr : sel_ctr;
    a.sel_lk = tl;
    a.sel_lr = tr;
    a.sel_floor = c.Tseed;   // group pruning: the probe saw only the groups kept
  }
  if (fprep) {
    a.fprep = 1;
    a.fq = q;
    a.fc = ix->iso_c;
    a.fD = ix->D;
    a.fDP = ix->DP;
    a.f_nq_pad = c.nq_pad;
    a.fX = c.X;
    a.fA = ix->int_A;
    a.fB = ix->int_B;
    a.fld = ix->ld_int;
    a.fw0 = ix->root_w0;
    a.flogdet0 = ix->root_logdet0;
    a.fP = c.P;
    a.fldP = std::max(ix->NI, 1);
    a.fqcnt = qcnt;
  }
  // group pruning: the seed threshold (exact keys of the best group's sample rows) is T0 --
  // the probe would only see the groups kept, so it is skipped
  if (!prn) HIPCHK(launch_stream(a, 1, (int)std::max<int64_t>(1, std::min<int64_t>(ix->cus, (a.n_probe + 7) / 8)), s));
  a.sel_ctr = nullptr;
  a.sel_floor = nullptr;
  a.fprep = 0;
  if (!fsel && !prn) {
    HIPCHK(launch_select(lb, ldlb, nqc, (int)a.n_probe, K, tl, tr, s));
    if (c.Tseed) HIPCHK(launch_raise_threshold(tl + (K - 1), 64, c.Tseed, nqc, s));
  }
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[5], s));
  if (i8) {   // the filter pass over the int8 panel (the probe above: bf16, a tighter T0)
    StreamArgs a8 = a;
    a8.i8 = 1;
    a8.Xb = reinterpret_cast<const uint16_t*>(Xq);
    a8.qinfo = qinfo8;
    a8.Mb = reinterpret_cast<const uint16_t*>(ix->iso_Mq);
    a8.rf = ix->iso_rf8;
    HIPCHK(launch_stream(a8, 0, stream_wgs(ix), s));
  } else {
    StreamArgs a0 = a;
    if (use_live) {
      a0.live = live;
      a0.live_n = ix->prune_ctr + 5;
    }
    HIPCHK(launch_stream(a0, 0, stream_wgs(ix), s));
  }
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[6], s));
  int nst = 0;
  if ((rc = run_leaf_scan(ix, c, EPI_TOPK, false, kl, 0.f, nullptr, 0, pkey, paux, prow, K, &nst, s, 2, 1, slabs)))
    return rc;
  const IntChain chain = int_chain(ix);
  if ((rc = ix->host_flags((size_t)3 * nqc))) return rc;
  // one candidate list per query (no anisotropic rows): final_wide expands the top-K to
  // sentence ids and writes the host flags itself (no merge launch, no flag copy)
  const bool ftail = nst == 1 && final_wide_rows(ix->DP, capq) > 0 && !getenv("CWQ_FW_UNFUSED");
  // okf / nex: the split tail's arrival count and exact-rerank sum (zeroed with the counters;
  // the fused tail reports through hflags, not these)
  const FwExpand fx{ix->sent_ptr, ix->sent_ids, ids, scores, k, ix->hflags, fws, fsk, fsa, fsr};
  HIPCHK(launch_final(c.X, ix->iso_Mf, ix->DP, nqc, K, capq, qcnt, qover, crow, cu, cl, T, 1, ix->row_meta,
                      ix->row_par, c.P ? c.P : ix->dummy, c.pT ? 1 : c.ldP, 0, pkey, paux, prow, (int64_t)nst * K, okf,
                      nex, lkb, lrb, done, ib ? &chain : nullptr, 0, 0.f, s, ftail ? &fx : nullptr));
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[7], s));
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[2], s));
  if (!ftail) {
    HIPCHK(launch_merge_expand(pkey, paux, prow, nqc, nst * K, K, k, ix->sent_ptr, ix->sent_ids, ids, scores, s));
    HIPCHK(hipMemcpyAsync(ix->hflags, qcnt, (size_t)3 * nqc * 4, hipMemcpyDeviceToHost, s));
  }
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[3], s));
  HIPCHK(sync_spin(s));
  std::vector<int64_t> redo;
  int64_t cand_sum = 0, exact_sum = 0;
  for (int i = 0; i < nqc; ++i) {
    if (!ix->hflags[nqc + i]) redo.push_back(i);
    cand_sum += ix->hflags[i];
    exact_sum += ix->hflags[2 * nqc + i];
  }
  if (ix->timing) {
    float e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(hipEventElapsedTime(&e[0], ix->ev[1], ix->ev[2]));
    HIPCHK(hipEventElapsedTime(&e[1], ix->ev[0], ix->ev[1]));
    HIPCHK(hipEventElapsedTime(&e[2], ix->ev[2], ix->ev[3]));
    HIPCHK(hipEventElapsedTime(&e[3], ix->ev[0], ix->ev[3]));
    HIPCHK(hipEventElapsedTime(&e[5], ix->ev[4], ix->ev[5]));
    HIPCHK(hipEventElapsedTime(&e[6], ix->ev[5], ix->ev[6]));
    HIPCHK(hipEventElapsedTime(&e[7], ix->ev[6], ix->ev[7]));
    for (int i = 0; i < 8; ++i) ix->t_ms[i] += e[i];
    ix->t_ms[4] += 1;   // one filter launch
  }
  if (!redo.empty() && (rc = rerun_exact(ix, q, redo, k, ids, scores, s))) return rc;
  ix->ws_idle = true;   // synchronized above (rerun_exact synchronizes too): no end event
  ix->stats[0] = nq;
  ix->stats[1] = (int64_t)redo.size();
  ix->stats[2] = 2 + (i8 ? 256 : 0);   // the stream filter (+256: its int8 pass)
  ix->stats[3] = (cand_sum + nq / 2) / nq;
  ix->stats[4] = (exact_sum + nq / 2) / nq;
  ix->stats[5] = a.n_probe * 16;
  return CWQ_OK;
}

// Isotropic leaf rows through the batch bf16-MFMA filter (cwq_mfma.hip): sample pass ->
// select -> filter launches over row-tile phases (bucket / tighten between them).  The
// caller then runs final_kernel on the returned candidate lists (exact keys -> list
// slot 0).  cat: the categorize key min(BF[parent], lp) (cwq_categorize) instead of the
// Fast key; ib: bounded internal prefixes (c.P lower, c.S_int upper).
struct IsoFilter {
  int *qcnt, *okf, *nex, *qover, *tdone, *crow, *tr;
  float *cu, *cl, *tl, *tlk;
};

size_t iso_filter_bytes_per_query(const cwq_index* ix, int n_rt) {
  return (size_t)ix->DPB * 2 + 16 + (size_t)ix->ld_s * 4 + 64 * 8 + (size_t)kFgCapQ * 12 + 32 +
         (size_t)(rec_per_q(ix) + dir_per_q(ix)) * 16 + 64 + ((size_t)2 * ix->cus * kFgChunk * 16) / 256 +
         (ix->n_multi_tiles ? (size_t)n_rt * 8 : 0) + 4 + 64 * 4;
}

int run_iso_filter(cwq_index* ix, Chunk& c, const float* qsrc, int64_t nqf, int K, bool cat, bool ib, Bump& b,
                   IsoFilter& o, hipStream_t s) {
  const int nqc = c.nq;
  const int n_rt = (int)(ix->ld_f / kFgTile);
  const int n_rts = ix->ld_s / kFgTile;
  const FiltConsts fc = filt_consts(ix->DPB);
  const int n_qt = (int)(nqf / kFgTile);
  uint16_t* Xb = b.take<uint16_t>((size_t)nqf * ix->DPB);
  float4* qinfo = b.take<float4>(nqf);
  float* lb = b.take<float>((size_t)nqf * ix->ld_s + 4096);
  float* tl = b.take<float>((size_t)nqf * 64);
  int* tr = b.take<int>((size_t)nqf * 64);
  // [qcnt | ok | n_exact | qover | tdone | gctr]: the host reads the first three with one
  // copy; one memset clears the block before the filter launches (tighten_kernel
  // clears gctr between them)
  int* qcnt = b.take<int>((size_t)5 * nqf + 64);
  int* okf = qcnt + nqf;
  int* nex = qcnt + 2 * nqf;
  int* qover = qcnt + 3 * nqf;
  int* tdone = qcnt + 4 * nqf;                       // tighten/final incremental state
  int* gctr = qcnt + 5 * nqf;
  float* tlk = b.take<float>((size_t)nqf * 64);
  int* crow = b.take<int>((size_t)nqf * kFgCapQ);
  float* cu = b.take<float>((size_t)nqf * kFgCapQ);
  float* cl = b.take<float>((size_t)nqf * kFgCapQ);
  // every workgroup holds one partly filled chunk at a time: keep room for two per workgroup
  const int64_t rec_cap = round_up(std::max<int64_t>((int64_t)nqf * rec_per_q(ix), (int64_t)2 * ix->cus * kFgChunk),
                                   kFgChunk);
  int4* rec = b.take<int4>((size_t)rec_cap);
  int* chunk_fill = b.take<int>((size_t)(rec_cap / kFgChunk));
  const int dir_cap = (int)std::min<int64_t>((int64_t)nqf * dir_per_q(ix), INT32_MAX / 2);
  int4* rec_dir = b.take<int4>((size_t)dir_cap);
  float2* pmm = (!cat && ix->n_multi_tiles) ? b.take<float2>((size_t)n_rt * nqf) : nullptr;
  HIPCHK(launch_query_prep(qsrc, nqc, ix->D, ix->iso_c, ix->DPB, nqf, Xb, qinfo, s));
  const PathB pb = (!cat && ib) ? path_b(ix, c) : PathB{nullptr, 0, nullptr, nullptr};
  const bool grp = ix->grp_mode && c.Pg_lo;   // group-centred rows: the shifted prefix tables
  if (pmm)   // multi-parent tiles: parent-prefix range per (tile, query) for the pretest
    HIPCHK(launch_tile_prange(grp ? c.Pg_lo : c.P, grp ? c.Pg_hi : ib ? c.S_int : nullptr, c.ldP, c.pT, nqc, ix->iso_tf,
                              n_rt, pmm, nqf, s, &pb));
  FgArgs g;
  memset(&g, 0, sizeof(g));
  g.DPB = ix->DPB;
  g.nq = nqc;
  g.n_qt = n_qt;
  fg_groups(n_qt, g.qgroups, g.rgroups);
  g.qinfo = qinfo;
  g.order = fg_order();
  g.dbg = getenv("CWQ_FG_DBG") ? atoi(getenv("CWQ_FG_DBG")) : 0;
  g.tctr = gctr + 8;
  g.rf = cat ? ix->cat_rf : ix->iso_rf;
  g.tf = cat ? ix->cat_tf : ix->iso_tf;
  g.cat = cat ? 1 : 0;
  g.pmm = pmm;
  g.ldq = nqf;
  g.P = cat ? (c.BF ? c.BF : ix->dummy) : (c.P ? c.P : ix->dummy);
  g.pb = pb;
  g.Phi = (!cat && ib && !pb.dot) ? c.S_int : nullptr;
  if (grp) {
    g.P = cat ? c.Pc_lo : c.Pg_lo;
    g.Phi = cat ? c.Pc_hi : c.Pg_hi;
    g.BFt = cat ? (c.BF ? c.BF : ix->dummy) : nullptr;
  }
  g.ldP = cat ? std::max(ix->NI, 1) : c.ldP;
  g.pT = cat ? 0 : c.pT;
  g.gamma = (float)fc.gamma;
  g.eps_n = (float)fc.eps_n;
  g.slack = (float)fc.slack;
  // 1. sample pass -> T[q] = K-th largest lower bound over the sample rows
  if (ix->timing) HIPCHK(hipEventRecord(ix->ev[4], s));
  g.mode = 1;
  if (g.order == 2) HIPCHK(hipMemsetAsync(g.tctr, 0, 32, s));
  g.n_rt = n_rts;
  g.nrows = ix->ld_s;
  g.rowmap = ix->samp_rows;
  // large samples: lower bounds reduced to maxima over groups of 4 rows in the
  // kernel (fgemm_kernel<1>); small ones keep one value per row so that K groups exist
  g.lb = lb;
  g.lbg = ix->n_samp >= 64 * K && !pb.dot ? 4 : 1;   // path-sum bounds: per-row values (fgemm_kernel<1>)
  g.ldlb = ix->ld_s / g.lbg;
  HIPCHK(launch_fgemm(Xb, ix->iso_Sb, g, ix->cus, s));
  HIPCHK(launch_select(lb, g.ldlb, nqc, (int)g.ldlb, K, tl, tr, s));
  // group pruning: the sample saw only the groups kept; its seed threshold is a floor
  if (!cat && c.Tseed) HIPCHK(launch_raise_threshold(tl + (K - 1), 64, c.Tseed, nqc, s));

  // 2. filter launches over row-tile phases (fg_phase_cuts: 1/32, 2/32, 5/32, 8/32,
  // 16/32 of the tiles); after each the candidates go to per-query lists and T[q] is
  // raised to the K-th largest candidate lower bound, so later phases emit fewer
  g.mode = 0;
  g.nrows = ix->NL_iso;
  g.rowmap = nullptr;
  g.T = tl + (K - 1);
  g.ldT = 64;
  g.rec = rec;
  g.rec_cap = rec_cap;
  g.gctr = gctr;
  g.chunk_fill = chunk_fill;
  g.qover = qover;
  g.rec_dir = rec_dir;
  g.dir_cap = dir_cap;
  HIPCHK(hipMemsetAsync(qcnt, 0, ((size_t)5 * nqf + 64) * 4, s));
  int cuts[6] = {0, n_rt, n_rt, n_rt, n_rt, n_rt};
  const int nph = fg_phase_cuts(n_rt, cuts);
  ix->n_fg_launch = nph;
  for (int ph = 0; ph < nph; ++ph) {
    g.rt_off = cuts[ph];
    g.n_rt = cuts[ph + 1] - cuts[ph];
    const std::vector<int>& up = cat ? ix->cat_uni_prefix : ix->tile_uni_prefix;
    g.all_uniform = up[cuts[ph + 1]] - up[cuts[ph]] == g.n_rt && !getenv("CWQ_FG_NO_ALLUNI");
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[5], s));
    unsigned long long* stamp_d = nullptr;
    const char* stamp_f = ph == nph - 1 ? getenv("CWQ_FG_STAMP") : nullptr;   // diagnostic builds
    if (stamp_f) {
      HIPCHK(hipMalloc(&stamp_d, 1 << 20));
      HIPCHK(hipMemsetAsync(stamp_d, 0, 1 << 20, s));
    }
    g.stamp = stamp_d;
    HIPCHK(launch_fgemm(Xb, ix->iso_Mb, g, ix->cus, s));
    if (stamp_f) {
      std::vector<unsigned long long> hs(1 << 17);
      HIPCHK(hipMemcpyAsync(hs.data(), stamp_d, 1 << 20, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipFree(stamp_d));
      g.stamp = nullptr;
      if (FILE* fo = fopen(stamp_f, "wb")) {
        fwrite(hs.data(), 8, hs.size(), fo);
        fclose(fo);
      }
    }
    if (ix->timing) {   // per-launch fgemm time (timing mode synchronises)
      float e = 0, e0 = 0;
      HIPCHK(hipEventRecord(ix->ev[6], s));
      HIPCHK(hipEventSynchronize(ix->ev[6]));
      HIPCHK(hipEventElapsedTime(&e, ix->ev[5], ix->ev[6]));
      ix->t_ms[6] += e;
      if (ph == 0) {
        HIPCHK(hipEventElapsedTime(&e0, ix->ev[4], ix->ev[5]));
        ix->t_ms[5] += e0;
      }
    }
    HIPCHK(launch_bucket(rec, gctr, chunk_fill, rec_cap, rec_dir, dir_cap, kFgCapQ, qcnt, qover, crow, cu, cl,
                         s));
    if (ph + 1 < nph)
      HIPCHK(launch_tighten(nqc, K, kFgCapQ, qcnt, qover, cl, tl + (K - 1), 64, tlk, tr, tdone, gctr, s));
  }
  o = IsoFilter{qcnt, okf, nex, qover, tdone, crow, tr, cu, cl, tl, tlk};
  return CWQ_OK;
}

int score_topk_impl(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                    hipStream_t s, bool allow_filter) {
  const bool general = k > 64;
  const bool filt = !general && allow_filter && use_filter(ix, k);
  if (!general && allow_filter && use_filter(ix, k, kStreamMinRows) && use_stream(ix, nq, k))
    return stream_topk_impl(ix, q, nq, k, ids, scores, s);
  const int kl = k <= 16 ? 16 : 64;
  const int K = std::min<int>(k, 64);
  const int n_pow2 = (int)std::max<int64_t>(2, 1LL << (int)ceil(log2((double)std::max(ix->NL, 2))));
  // partial-list entries per query (upper bound over both segments; one list for the filter)
  const int nqb_est = n_qblocks_for(nq, kl);
  auto n_slabs = [&](int nqb) {
    // a chunk may take either scan (use_small_scan on its own query count): room for both
    // (small_scan_slabs(1, n) is its largest slab count)
    const int n_iso = std::max(pick_nslab(ix, ix->NL_iso, nqb), small_scan_fits(ix, K) ? small_scan_slabs(1, ix->NL_iso) : 0);
    return filt ? 1 + (pick_nslab(ix, ix->NL_an, nqb) + 1) * scan_lists_per_slab(kl)
                : (n_iso + pick_nslab(ix, ix->NL_an, nqb) + 2) * scan_lists_per_slab(kl);
  };
  const int n_rt = filt ? (int)(ix->ld_f / kFgTile) : 0;
  const int n_rts = filt ? ix->ld_s / kFgTile : 0;
  // per query: bf16 query, info, sample bounds, threshold list, candidate lists, flags, records
  const size_t filt_q = filt ? iso_filter_bytes_per_query(ix, n_rt) : 0;
  const size_t extra = general ? (size_t)ix->NL * 4 + (size_t)n_pow2 * 8
                               : (size_t)n_slabs(nqb_est) * K * 12 + K * 12 + filt_q;
  int64_t cq = chunk_queries(ix, nq, extra, false);
  if (filt && cq < nq) cq = std::max<int64_t>(kFgTile, cq / kFgTile * kFgTile);   // whole query tiles
  int64_t n_fallback = 0, cand_sum = 0, exact_sum = 0;
  std::vector<int64_t> redo;
  int rc;
  for (int64_t q0 = 0; q0 < nq; q0 += cq) {
    const int nqc = (int)std::min(cq, nq - q0);
    const int64_t nq_pad = round_up(nqc, kQPad);
    const int nqb = n_qblocks_for(nqc, kl);
    const int slabs = n_slabs(nqb);
    const int64_t nqf = round_up(nqc, kFgTile);
    size_t need = chunk_bytes(ix, nq_pad, false) + 64 * 256;
    need += general ? (size_t)nq_pad * ((size_t)ix->NL * 4 + (size_t)n_pow2 * 8)
                    : (size_t)nq_pad * ((size_t)slabs * K * 12 + (size_t)K * 12) + (size_t)nqf * filt_q + 4096 * 8;
    const bool ib = filt && use_int_bounds(ix);
    if (ib) need += int_bounds_bytes(ix, nqf);
    const bool prn = filt && !ib && !general && use_prune(ix);
    if ((rc = ix->reserve(need))) return rc;
    Bump b(ix->ws, ix->ws_size);
    Chunk c;
    carve_chunk(ix, b, c, nqc, false);
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[0], s));
    HIPCHK(launch_pad_queries(q + q0 * ix->D, nqc, ix->D, c.X, c.nq_pad, ix->DP, s));
    if (ib) {
      if ((rc = run_internal_bounds(ix, c, q + q0 * ix->D, nqf, b, s))) return rc;
    } else if (prn) {
      if ((rc = prune_internal(ix, c, q + q0 * ix->D, K, b, s))) return rc;
    } else if ((rc = run_internal(ix, c, s, false, q + q0 * ix->D, filt ? 0 : -1))) {
      return rc;
    }
    if (filt && (rc = group_tables(ix, c, q + q0 * ix->D, false, s))) return rc;
    if (ix->timing) HIPCHK(hipEventRecord(ix->ev[1], s));
    if (!general) {
      float* pkey = b.take<float>((size_t)nq_pad * slabs * K);
      float* paux = b.take<float>((size_t)nq_pad * slabs * K);
      int* prow = b.take<int>((size_t)nq_pad * slabs * K);
      int nst = 0;
      int* okf = nullptr;
      int *qcnt_d = nullptr, *nex_d = nullptr;
      if (filt) {
        // isotropic rows: sample bounds -> thresholds -> MFMA filter -> candidates ->
        // exact rerank into list slot 0; anisotropic rows: exact scan into slots 1..
        IsoFilter fo;
        if ((rc = run_iso_filter(ix, c, q + q0 * ix->D, nqf, K, false, ib, b, fo, s))) return rc;
        int* qcnt = fo.qcnt;
        int* nex = fo.nex;
        okf = fo.okf;
        float* tl = fo.tl;
        float* tlk = fo.tlk;
        int* tr = fo.tr;
        int* tdone = fo.tdone;
        int* qover = fo.qover;
        int* crow = fo.crow;
        float* cu = fo.cu;
        float* cl = fo.cl;
        if ((rc = run_leaf_scan(ix, c, EPI_TOPK, false, kl, 0.f, nullptr, 0, pkey, paux, prow, K, &nst, s, 2, 1, slabs)))
          return rc;
        const IntChain chain = int_chain(ix);
        HIPCHK(launch_final(c.X, ix->iso_Mf, ix->DP, nqc, K, kFgCapQ, qcnt, qover, crow, cu, cl, tl + (K - 1), 64,
                            ix->row_meta, ix->row_par, c.P ? c.P : ix->dummy, c.pT ? 1 : c.ldP, 0, pkey, paux,
                            prow, (int64_t)nst * K, okf, nex, tlk, tr, tdone, ib ? &chain : nullptr, 0, 0.f, s));
        qcnt_d = qcnt;
        nex_d = nex;
        if (ix->timing) HIPCHK(hipEventRecord(ix->ev[7], s));
      } else {
        if ((rc = run_leaf_scan(ix, c, EPI_TOPK, false, kl, 0.f, nullptr, 0, pkey, paux, prow, K, &nst, s, 3, 0, slabs)))
          return rc;
      }
      if (ix->timing) HIPCHK(hipEventRecord(ix->ev[2], s));
      HIPCHK(launch_merge_expand(pkey, paux, prow, nqc, nst * K, K, k, ix->sent_ptr, ix->sent_ids, ids + q0 * k,
                                 scores ? scores + q0 * k : nullptr, s));
      if (filt) {
        if ((rc = ix->host_flags((size_t)3 * nqf))) return rc;
        HIPCHK(hipMemcpyAsync(ix->hflags, qcnt_d, (size_t)3 * nqf * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const int* cnth = ix->hflags;
        const int* okh = cnth + nqf;
        const int* nexh = cnth + 2 * nqf;
        for (int i = 0; i < nqc; ++i) {
          if (!okh[i]) redo.push_back(q0 + i);
          cand_sum += cnth[i];
          exact_sum += nexh[i];
        }
      }
    } else {
      float* rowkey = b.take<float>((size_t)nq_pad * std::max(ix->NL, 1));
      float* skey = b.take<float>((size_t)nq_pad * n_pow2);
      int* srow = b.take<int>((size_t)nq_pad * n_pow2);
      if ((rc = run_leaf_scan(ix, c, EPI_KEY, false, 16, 0.f, rowkey, ix->NL, nullptr, nullptr, nullptr, 1, nullptr, s)))
        return rc;
      if (ix->timing) HIPCHK(hipEventRecord(ix->ev[2], s));
      HIPCHK(launch_init_rows(rowkey, ix->NL, nqc, ix->NL, n_pow2, skey, srow, s));
      HIPCHK(launch_sort_rows(skey, srow, nqc, ix->NL, n_pow2, s));
      HIPCHK(launch_expand(skey, srow, nqc, n_pow2, k, ix->sent_ptr, ix->sent_ids, ids + q0 * k,
                           scores ? scores + q0 * k : nullptr, s));
    }
    if (ix->timing) {
      HIPCHK(hipEventRecord(ix->ev[3], s));
      HIPCHK(hipEventSynchronize(ix->ev[3]));
      float a = 0, b2 = 0, c2 = 0, d = 0;
      HIPCHK(hipEventElapsedTime(&a, ix->ev[1], ix->ev[2]));
      HIPCHK(hipEventElapsedTime(&b2, ix->ev[0], ix->ev[1]));
      HIPCHK(hipEventElapsedTime(&c2, ix->ev[2], ix->ev[3]));
      HIPCHK(hipEventElapsedTime(&d, ix->ev[0], ix->ev[3]));
      ix->t_ms[0] += a;
      ix->t_ms[1] += b2;
      ix->t_ms[2] += c2;
      ix->t_ms[3] += d;
      ix->t_ms[4] += filt ? ix->n_fg_launch : (ix->NL_iso > 0) + (ix->NL_an > 0);   // filter: fgemm launches
      if (filt) {
        float e3 = 0;
        HIPCHK(hipEventElapsedTime(&e3, ix->ev[6], ix->ev[7]));
        ix->t_ms[7] += e3;
      }
    }
  }
  if (!redo.empty()) {
    n_fallback = (int64_t)redo.size();
    if ((rc = rerun_exact(ix, q, redo, k, ids, scores, s))) return rc;
  }
  if (allow_filter) {
    ix->stats[0] = filt ? nq : 0;
    ix->stats[1] = n_fallback;
    ix->stats[2] = filt ? 1 : 0;
    ix->stats[3] = filt && nq > 0 ? (cand_sum + nq / 2) / nq : 0;
    ix->stats[4] = filt && nq > 0 ? (exact_sum + nq / 2) / nq : 0;
    ix->stats[5] = filt ? ix->n_samp : 0;
  }
  return CWQ_OK;
}

}  // namespace

extern "C" int cwq_score_topk(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                              void* stream) {
  if (!ix || (!q && nq > 0) || (!ids && nq > 0)) return fail(CWQ_ERR_ARG, "NULL argument");
  if (k <= 0) return fail(CWQ_ERR_ARG, "k must be >= 1");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  for (float& t : ix->t_ms) t = 0.f;
  for (int64_t& t : ix->stats) t = 0;
  ix->prune_nq = 0;
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const int rc = score_topk_impl(ix, q, nq, k, ids, scores, s, true);
  if (!rc) note_filter(ix);
  return rc;
}

// The reference harness's call with host memory on both sides (benchmark_utils.py:801-805:
// a numpy query in, sentence ids out): the query is copied into pinned staging and sent with
// one async copy, the kernels write the ids / scores straight into mapped host memory, and
// the call returns synchronized -- no torch tensors, no device allocations, no separate
// device-to-host copy per call.
extern "C" int cwq_score_topk_host(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                                   void* stream) {
  if (!ix || (!q && nq > 0) || (!ids && nq > 0)) return fail(CWQ_ERR_ARG, "NULL argument");
  if (k <= 0) return fail(CWQ_ERR_ARG, "k must be >= 1");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  for (float& t : ix->t_ms) t = 0.f;
  for (int64_t& t : ix->stats) t = 0;
  ix->prune_nq = 0;
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const size_t qb = (size_t)nq * ix->D * 4, ib = (size_t)round_up(nq * k * 8, 256), sb = (size_t)nq * k * 4;
  int rc;
  if ((rc = ix->host_io(qb, ib + sb))) return rc;
  memcpy(ix->hq, q, qb);
  HIPCHK(hipMemcpyAsync(ix->dq, ix->hq, qb, hipMemcpyHostToDevice, s));
  int64_t* hid = (int64_t*)ix->hout;
  float* hsc = (float*)((char*)ix->hout + ib);
  if ((rc = score_topk_impl(ix, (const float*)ix->dq, nq, k, hid, hsc, s, true))) return rc;
  note_filter(ix);
  HIPCHK(sync_spin(s));
  ix->ws_idle = true;   // synchronized
  memcpy(ids, hid, (size_t)nq * k * 8);
  if (scores) memcpy(scores, hsc, sb);
  return CWQ_OK;
}

extern "C" int cwq_set_filter(cwq_index* ix, int mode) {
  if (!ix) return fail(CWQ_ERR_ARG, "NULL index");
  if (mode < -1 || mode > 1) return fail(CWQ_ERR_ARG, "mode must be -1, 0 or 1");
  ix->filter = mode;
  ix->filt_q = ix->filt_fb = 0;   // a fresh auto-mode record
  ix->filt_auto_off = false;
  ix->filt_off_calls = 0;
  return CWQ_OK;
}

extern "C" int cwq_last_stats(cwq_index* ix, int64_t* out) {
  if (!ix || !out) return fail(CWQ_ERR_ARG, "NULL argument");
  for (int i = 0; i < 6; ++i) out[i] = ix->stats[i];
  return CWQ_OK;
}

extern "C" int cwq_last_prune_stats(cwq_index* ix, int64_t* out) {
  if (!ix || !out) return fail(CWQ_ERR_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  out[0] = ix->prune_ok ? 1 : 0;
  out[1] = ix->prune_nq;
  out[2] = 0;
  out[3] = ix->G;
  if (ix->prune_ctr && ix->prune_nq > 0) {
    int v = 0;
    if (ix->ws_ev_live) HIPCHK(hipEventSynchronize(ix->ws_ev));
    HIPCHK(hipMemcpy(&v, ix->prune_ctr + 4, sizeof(int), hipMemcpyDeviceToHost));
    out[2] = v;
  }
  return CWQ_OK;
}

extern "C" int cwq_set_timing(cwq_index* ix, int enable) {
  if (!ix) return fail(CWQ_ERR_ARG, "NULL index");
  DevGuard dg(ix->device);
  for (int i = 0; i < 8; ++i)
    if (!ix->ev[i]) HIPCHK(hipEventCreate(&ix->ev[i]));
  ix->timing = enable != 0;
  return CWQ_OK;
}

extern "C" int cwq_last_timing(cwq_index* ix, float* out) {
  if (!ix || !out) return fail(CWQ_ERR_ARG, "NULL argument");
  for (int i = 0; i < 8; ++i) out[i] = ix->t_ms[i];
  return CWQ_OK;
}

extern "C" int cwq_rank_scores(cwq_index* ix, const float* q, int64_t nq, float* out, void* stream) {
  if (!ix || (!q && nq > 0) || (!out && nq > 0)) return fail(CWQ_ERR_ARG, "NULL argument");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const int64_t cq = chunk_queries(ix, nq, (size_t)ix->NL * 4, false);
  int rc;
  for (int64_t q0 = 0; q0 < nq; q0 += cq) {
    const int nqc = (int)std::min(cq, nq - q0);
    const int64_t nq_pad = round_up(nqc, kQPad);
    if ((rc = ix->reserve(chunk_bytes(ix, nq_pad, false) + (size_t)nq_pad * std::max(ix->NL, 1) * 4 + 8 * 256))) return rc;
    Bump b(ix->ws, ix->ws_size);
    Chunk c;
    carve_chunk(ix, b, c, nqc, false);
    float* rowkey = b.take<float>((size_t)nq_pad * std::max(ix->NL, 1));
    HIPCHK(launch_pad_queries(q + q0 * ix->D, nqc, ix->D, c.X, c.nq_pad, ix->DP, s));
    if ((rc = run_internal(ix, c, s, false))) return rc;
    if ((rc = run_leaf_scan(ix, c, EPI_KEY, false, 16, 0.f, rowkey, ix->NL, nullptr, nullptr, nullptr, 1, nullptr, s)))
      return rc;
    HIPCHK(launch_gather_sentences(rowkey, ix->NL, nqc, ix->row_of_sent, ix->n_sent, out + q0 * ix->n_sent, s));
  }
  return CWQ_OK;
}

extern "C" int cwq_node_logprob(cwq_index* ix, const float* q, int64_t nq, int32_t full, float* out, void* stream) {
  if (!ix || (!q && nq > 0) || (!out && nq > 0)) return fail(CWQ_ERR_ARG, "NULL argument");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const float dconst = full ? (float)((double)ix->D * (double)logf(2.0f * (float)M_PI)) : 0.f;
  const int64_t cq = chunk_queries(ix, nq, (size_t)ix->NL * 4);
  int rc;
  for (int64_t q0 = 0; q0 < nq; q0 += cq) {
    const int nqc = (int)std::min(cq, nq - q0);
    const int64_t nq_pad = round_up(nqc, kQPad);
    if ((rc = ix->reserve(chunk_bytes(ix, nq_pad) + (size_t)nq_pad * std::max(ix->NL, 1) * 4 + 8 * 256))) return rc;
    Bump b(ix->ws, ix->ws_size);
    Chunk c;
    carve_chunk(ix, b, c, nqc);
    float* sleaf = b.take<float>((size_t)nq_pad * std::max(ix->NL, 1));
    HIPCHK(launch_pad_queries(q + q0 * ix->D, nqc, ix->D, c.X, c.nq_pad, ix->DP, s));
    if ((rc = run_internal(ix, c, s))) return rc;
    if ((rc = run_leaf_scan(ix, c, EPI_RAW, false, 16, 0.f, sleaf, ix->NL, nullptr, nullptr, nullptr, 1, nullptr, s)))
      return rc;
    HIPCHK(launch_node_lp(c.S_int ? c.S_int : ix->dummy, std::max(ix->NI, 1), sleaf, std::max(ix->NL, 1), nqc,
                          ix->node_src, ix->logdet_int, ix->logdet_row, dconst, ix->n_nodes, out + q0 * ix->n_nodes, s));
  }
  return CWQ_OK;
}

extern "C" int cwq_prefix_bounds(cwq_index* ix, const float* q, int64_t nq, float* lo, float* hi, float* exact,
                                 void* stream) {
  if (!ix || !q || !lo || !hi || !exact) return fail(CWQ_ERR_ARG, "NULL argument");
  if (nq <= 0 || nq > 4096) return fail(CWQ_ERR_ARG, "nq must be in [1, 4096]");
  if (!ix->int_bounds)
    return fail(CWQ_ERR_ARG, "no internal-node bounds on this index (flat tree, no isotropic leaf rows or too deep)");
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const int64_t nq_pad = round_up(nq, kQPad), nqf = round_up(nq, kFgTile);
  int rc;
  if ((rc = ix->reserve(chunk_bytes(ix, nq_pad, false) + int_bounds_bytes(ix, nqf) + 64 * 256))) return rc;
  Bump b(ix->ws, ix->ws_size);
  Chunk c;
  carve_chunk(ix, b, c, (int)nq, false);
  const size_t n = (size_t)nq * ix->NI * 4;
  HIPCHK(launch_pad_queries(q, nq, ix->D, c.X, c.nq_pad, ix->DP, s));
  if ((rc = run_internal(ix, c, s, false))) return rc;
  HIPCHK(hipMemcpyAsync(exact, c.P, n, hipMemcpyDeviceToDevice, s));
  const size_t nall = (size_t)c.nq_pad * ix->NI * 4;
  HIPCHK(hipMemsetAsync(c.P, 0xff, nall, s));   // NaN where the bound pass writes nothing
  HIPCHK(hipMemsetAsync(c.S_int, 0xff, nall, s));
  if ((rc = run_internal_bounds(ix, c, q, nqf, b, s))) return rc;
  const PathB pb = path_b(ix, c);
  if (pb.dot) {   // path-sum dots, node-major [NI][nq_pad] -> bounds [nq][NI]
    HIPCHK(launch_pathb_expand(pb, (int)nq, ix->NI, lo, hi, s));
  } else if (c.pT) {   // node-major [NI][nq_pad] -> [nq][NI]
    HIPCHK(launch_transpose(c.P, ix->NI, nq, c.ldP, lo, ix->NI, s));
    HIPCHK(launch_transpose(c.S_int, ix->NI, nq, c.ldP, hi, ix->NI, s));
  } else {
    HIPCHK(hipMemcpyAsync(lo, c.P, n, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(hi, c.S_int, n, hipMemcpyDeviceToDevice, s));
  }
  return CWQ_OK;
}

namespace {
// cwq_categorize body.  allow_filter: the isotropic leaf rows go through the bf16-MFMA
// filter with the categorize key (run_iso_filter, cat); queries whose candidate lists
// overflow are re-run with allow_filter = false (the exact scan of every leaf row).
// Categorize's top-R row list for a few queries (nq <= kStreamMaxQ) through the per-call
// stream filter instead of the batch pipeline (sample pass, select, five fgemm launches with
// bucket / tighten): query prep, probe + fused select, one pass, final_wide_kernel with the
// categorize key -- the key min(BFk[parent], lp_full) bounded by the categorize RowF and
// min'ed with BFk in the kernels (cwq_stream.hip), exact keys and the list order of
// list_before<true> in final_wide.  BFk: the chunk's BF (list 1) or the second-level T2
// (the two-level replay's list 2).  The list goes to slot 0 of pkey/paux/prow (stride lstride),
// the per-query certified flags to okf (a query whose candidates overflow: 0).
// the probe's 16-row groups for a list of R and the per-row bound lines they fill
int64_t cat_n_probe(const cwq_index* ix, int R) {
  const int64_t ngroups = (ix->NL_iso + 15) / 16;
  return std::min<int64_t>(std::max<int64_t>((int64_t)3 * R * ngroups / 1024, (int64_t)8 * R), ngroups);
}
int64_t cat_ldlb(const cwq_index* ix, int R) { return round_up(cat_n_probe(ix, R) * 16 + 1, 1024) + 1024; }
size_t stream_cat_bytes(const cwq_index* ix, int nqc) {
  const int nq16 = (nqc + 15) / 16 * 16;
  const int64_t ldlb = cat_ldlb(ix, 64);
  return (size_t)nq16 * ix->DPB * 2 + (size_t)nq16 * 16 + (size_t)nqc * 4 + (size_t)(5 * nqc + 1) * 4 +
         (size_t)nqc * kFgCapQ * 12 + (size_t)nqc * 64 * 16 + (size_t)nqc * ldlb * 4 + 16 * 256 +
         (size_t)nqc * kFwSplitMax * 64 * 12 + 3 * 256;
}
bool stream_cat_ok(const cwq_index* ix, int nqc, int R) {
  return ix->iso_Mb && ix->NL_iso >= kStreamMinRows && nqc <= kStreamMaxQ && R <= kFiltMaxK &&
         stream_lds_bytes((nqc + 15) / 16, ix->DPB) <= (size_t)kStreamMaxLds && final_wide_rows(ix->DP, kFgCapQ) > 0 &&
         !getenv("CWQ_CAT_STREAM_OFF");
}
int stream_cat_list(cwq_index* ix, Chunk& c, const float* q, int nqc, int R, const float* BFk, float dfull, float* pkey,
                    float* paux, int* prow, int64_t lstride, int* okf, Bump& b, hipStream_t s) {
  const int nqb = (nqc + 15) / 16, nq16 = nqb * 16;
  const int capq = kFgCapQ;
  uint16_t* Xb = b.take<uint16_t>((size_t)nq16 * ix->DPB);
  float4* qinfo = b.take<float4>(nq16);
  float* T = b.take<float>(nqc);
  int* qcnt = b.take<int>((size_t)5 * nqc + 1);   // [qcnt | ok | n_exact | qover | done | select counter]
  int* nex = qcnt + 2 * nqc;
  int* qover = qcnt + 3 * nqc;
  int* done = qcnt + 4 * nqc;
  int* sel_ctr = qcnt + 5 * nqc;
  int* crow = b.take<int>((size_t)nqc * capq);
  float* cu = b.take<float>((size_t)nqc * capq);
  float* cl = b.take<float>((size_t)nqc * capq);
  float* lkb = b.take<float>((size_t)nqc * 64);
  int* lrb = b.take<int>((size_t)nqc * 64);
  const int64_t ldlb = cat_ldlb(ix, R);   // every probed row's bound (probe_rows)
  float* lb = b.take<float>((size_t)nqc * ldlb);
  float* tl = b.take<float>((size_t)nqc * 64);
  int* tr = b.take<int>((size_t)nqc * 64);
  // the rerank split over workgroups (categorize lists: ~1k candidates, most reranked --
  // their keys tie at the parents' bottlenecks); arrivals counted in the zeroed ok slot
  // (at most 8: the last workgroup's merge inserts the others' tie-heavy lists serially --
  // C2 list 2: 8 workgroups end at 33 us, 32 at 61 us, profiles/r05_basic_percall_stamps_radix_s{8,32}.log)
  const int fws = std::min(8, fw_split(ix, nqc, true));
  FwExpand fx{nullptr, nullptr, nullptr, nullptr, 0, nullptr, fws, b.take<float>((size_t)nqc * fws * 64),
              b.take<float>((size_t)nqc * fws * 64), b.take<int>((size_t)nqc * fws * 64), qcnt + nqc};
  // the counters (qcnt, qover, done, the fused select's) zeroed by the prep's block 0
  HIPCHK(launch_query_prep(q, nqc, ix->D, ix->iso_c, ix->DPB, nq16, Xb, qinfo, s, qcnt, (int)(5 * nqc + 1)));
  const FiltConsts fc = filt_consts(ix->DPB);
  StreamArgs a;
  memset(&a, 0, sizeof(a));
  a.DPB = ix->DPB;
  a.nq = nqc;
  a.nqb = nqb;
  a.nrows = ix->NL_iso;
  a.K = R;
  a.Xb = Xb;
  a.qinfo = qinfo;
  a.Mb = ix->iso_Mb;
  a.rf = ix->cat_rf;
  const bool grp = ix->grp_mode && c.Pc_lo;
  a.P = grp ? c.Pc_lo : (c.BF ? c.BF : ix->dummy);   // non-group rows: invL 0 (no prefix term)
  a.Phi = grp ? c.Pc_hi : nullptr;
  a.ldP = std::max(ix->NI, 1);
  a.pT = 0;
  a.BFk = BFk;
  a.ldBF = std::max(ix->NI, 1);
  a.eps_n = (float)fc.eps_n;
  a.slack = (float)fc.slack;
  a.T = T;
  a.qcnt = qcnt;
  a.qover = qover;
  a.capq = capq;
  a.crow = crow;
  a.cu = cu;
  a.cl = cl;
  const int64_t ngroups = (ix->NL_iso + 15) / 16;
  const int64_t n_probe = cat_n_probe(ix, R);
  a.probe_stride = std::max<int64_t>(1, ngroups / std::max<int64_t>(n_probe, 1));
  a.n_probe = std::min<int64_t>(n_probe, (ngroups + a.probe_stride - 1) / a.probe_stride);
  a.probe_rows = getenv("CWQ_CAT_PROBE_MAX") ? 0 : 1;   // 1: group maxima (A/B)
  a.lb = lb;
  a.ldlb = ldlb;
  a.T0 = tl;
  a.ldT0 = 64;
  a.sel_ctr = sel_ctr;
  a.sel_lk = tl;
  a.sel_lr = tr;
  HIPCHK(launch_stream(a, 1, (int)std::max<int64_t>(1, std::min<int64_t>(ix->cus, (a.n_probe + 7) / 8)), s));
  a.sel_ctr = nullptr;
  a.probe_rows = 0;
  HIPCHK(launch_stream(a, 0, stream_wgs(ix), s));
  HIPCHK(launch_final(c.X, ix->iso_Mf, ix->DP, nqc, R, capq, qcnt, qover, crow, cu, cl, T, 1, ix->row_meta, ix->row_par,
                      BFk ? BFk : ix->dummy, std::max(ix->NI, 1), 0, pkey, paux, prow, lstride, okf, nex, lkb, lrb,
                      done, nullptr, 1, dfull, s, fws > 1 ? &fx : nullptr));
  if (getenv("CWQ_CAT_DEBUG")) {   // diagnostics: per query candidates, overflow, threshold, certified
    std::vector<int> hc(nqc), ho(nqc), hk(nqc), hx(nqc);
    std::vector<float> ht(nqc), hl(64);
    HIPCHK(hipMemcpyAsync(hc.data(), qcnt, nqc * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ho.data(), qover, nqc * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hk.data(), okf, nqc * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hx.data(), nex, nqc * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ht.data(), T, nqc * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hl.data(), tl, 64 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < std::min(nqc, 4); ++i)
      fprintf(stderr, "[cat stream] q %d R %d cand %d over %d T %.6g ok %d exact %d probe T0 %.6g | tl[R-2..R] %.6g %.6g\n",
              i, R, hc[i], ho[i], ht[i], hk[i], hx[i], i == 0 ? hl[R - 1] : 0.f, i == 0 ? hl[R - 2] : 0.f,
              i == 0 && R < 64 ? hl[R] : 0.f);
  }
  return CWQ_OK;
}

constexpr int kCatCountRetry = 16;   // (cwq_index::cat_count_idle)
constexpr int kCatExplore = 32, kCatDenseMemory = 64;   // (cwq_index::cat_ema_*)
constexpr int kLzFanout = 1024;   // batches try the lazy path when no node has more children
int categorize_impl(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t max_nodes, int64_t* nodes,
                    int32_t* n_found, int64_t* n_calls, hipStream_t s, bool allow_filter) {
  const float dfull = (float)((double)ix->D * (double)logf(2.0f * (float)M_PI));
  const int R = std::max(1, std::min(64, ix->NL));
  const bool complete = ix->NL <= R;
  const int64_t cap_list = 1 + (int64_t)ix->NI + R;
  const int kl = 64;
  int rc;
  const char* ce = getenv("CWQ_CAT_FILTER");
  // a call of a few queries takes the per-call stream lists from kStreamMinRows rows on (as
  // Fast does): the exact 64-wide list scan of a small tree is its latency chain -- qqp1k
  // (1,000 rows x 1,024): 285 us a list, profiles/r05_published_shapes_v4.log
  const bool filt = allow_filter && use_filter(ix, R, nq <= 64 ? kStreamMinRows : kFiltMinRows, false) &&
                    !(ce && *ce && atoi(ce) == 0);
  const int n_rt = filt ? (int)(ix->ld_f / kFgTile) : 0;
  const size_t filt_q = filt ? iso_filter_bytes_per_query(ix, n_rt) : 0;
  const int nqb_est = n_qblocks_for(nq, kl);
  auto n_slabs = [&](int nqb) {
    return filt ? 1 + (pick_nslab(ix, ix->NL_an, nqb) + 1) * scan_lists_per_slab(kl)
                : (pick_nslab(ix, ix->NL_iso, nqb) + pick_nslab(ix, ix->NL_an, nqb) + 2) * scan_lists_per_slab(kl);
  };
  const int max_slabs = n_slabs(nqb_est);
  int64_t cq = chunk_queries(ix, nq, (size_t)cap_list * 16 + (size_t)max_slabs * R * 12 + R * 12 + filt_q);
  if (filt && cq < nq) cq = std::max<int64_t>(kFgTile, cq / kFgTile * kFgTile);   // whole query tiles
  std::vector<int64_t> fredo;   // queries the filter could not certify
  // a few queries (the reference's one cobweb_predict per query): the lists through the
  // per-call stream filter (stream_cat_list), and a two-level replay of every query of the
  // call reuses the chunk's internal pass instead of gathering and recomputing it
  const bool scat = filt && nq <= cq && stream_cat_ok(ix, (int)nq, R);
  // a few queries without the filter (small trees): the two-level replay on the chunk too,
  // list 2 by the exact scan (instead of gathering the queries and re-running the internal
  // pass: qqp1k's Basic call 1.02 ms, profiles/r05_published_shapes_v3.log)
  const bool small2 = !filt && nq <= std::min<int64_t>(cq, 64);
  // every query resolved in the first chunk by the list paths: the flag gathers cleared the
  // node tails after the last results, so the caller needs no clear_tail launch / sync
  ix->cat_tail_done = nq <= cq;
  const int64_t cap2 = 1 + (int64_t)ix->NI + 2 * R;
  // straight to the exact lazy replay (a call of <= 64 queries; CWQ_CAT_DIRECT=0 / 1: never /
  // always where it applies)
  const char* cde = getenv("CWQ_CAT_DIRECT");
  const int cdv = cde && *cde ? atoi(cde) : -1;
  const int64_t cap_dense = 1 + (int64_t)ix->NI + ix->NL;
  const int pk = nq <= 64 ? 0 : 1;   // the policy slot: small call / batch
  const bool direct_ok = (pk == 1 || nq <= cq) && ix->NI > 0 && ix->DP <= 2048;
  const bool top = allow_filter;   // (not the filter-overflow re-run of a call)
  const bool measure = direct_ok && cdv < 0 && top;
  bool direct = false;
  if (direct_ok) {
    if (cdv >= 0) {
      direct = cdv == 1;
    } else if (!top) {
      direct = ix->cat_pref_direct[pk];
    } else {
      ++ix->cat_pol_calls[pk];
      const bool may = ix->cat_dense_seen > 0 || (pk == 1 && ix->max_fanout <= kLzFanout);
      if (!may) direct = false;                                     // the lists resolve this tree
      else if (ix->cat_ema_list[pk] < 0.0) direct = false;          // the lists first
      else if (ix->cat_ema_direct[pk] < 0.0) direct = true;         // then one trial
      else direct = (ix->cat_ema_direct[pk] < ix->cat_ema_list[pk]) != (ix->cat_pol_calls[pk] % kCatExplore == 0);
    }
  }
  const auto t_call = std::chrono::steady_clock::now();
  int64_t n_dense_call = 0;
  for (int64_t q0 = 0; q0 < nq; q0 += cq) {
    const int nqc = (int)std::min(cq, nq - q0);
    const int64_t nq_pad = round_up(nqc, kQPad);
    const int nqb = n_qblocks_for(nqc, kl);
    const int slabs = n_slabs(nqb);
    const int64_t nqf = round_up(nqc, kFgTile);
    size_t need = chunk_bytes(ix, nq_pad) + (size_t)nq_pad * ((size_t)slabs * R * 12 + (size_t)R * 12 +
                                                              (size_t)cap_list * 16 + 12) + 17 * 256 +
                  (filt ? (size_t)nqf * filt_q + 4096 * 8 : 0);
    if (direct && pk == 0) need += (size_t)nq_pad * ((size_t)cap_dense * 16 + 16) + 2 * 256;
    if (scat || small2)   // + the second list's stream pass, T2, lists and heap (the two-level replay in place)
      need += (scat ? 2 * stream_cat_bytes(ix, nqc) : 0) + (size_t)nq_pad * ((size_t)std::max(ix->NI, 1) * 4 + (size_t)slabs * R * 12 +
                                                                 (size_t)R * 12 + (size_t)cap2 * 16 + 16) + 32 * 256;
    if ((rc = ix->reserve(need))) return rc;
    Bump b(ix->ws, ix->ws_size);
    Chunk c;
    carve_chunk(ix, b, c, nqc);
    float* pkey = b.take<float>((size_t)nq_pad * slabs * R);
    float* paux = b.take<float>((size_t)nq_pad * slabs * R);
    int* prow = b.take<int>((size_t)nq_pad * slabs * R);
    float* okey = b.take<float>((size_t)nq_pad * R);
    float* oaux = b.take<float>((size_t)nq_pad * R);
    int* orow = b.take<int>((size_t)nq_pad * R);
    HeapEnt* heap = b.take<HeapEnt>((size_t)nq_pad * cap_list);
    int* status = b.take<int>((size_t)nq_pad);
    // the replay arguments every path shares (the tree; the per-chunk fields set by the caller)
    auto base_args = [&]() {
      SimArgs sd;
      memset(&sd, 0, sizeof(sd));
      sd.k = k;
      sd.max_nodes = max_nodes;
      sd.NI = ix->NI;
      sd.NL = ix->NL;
      sd.ldI = std::max(ix->NI, 1);
      sd.complete = complete ? 1 : 0;
      sd.int_child_begin = ix->int_child_begin;
      sd.int_child_end = ix->int_child_end;
      sd.int_nchild = ix->int_nchild;
      sd.int_bfs = ix->int_bfs;
      sd.int_has_sent = ix->int_has_sent;
      sd.int_leaf_a0 = ix->int_leaf_a0;
      sd.int_leaf_a1 = ix->int_leaf_a1;
      sd.int_leaf_b0 = ix->int_leaf_b0;
      sd.int_leaf_b1 = ix->int_leaf_b1;
      sd.row_par = ix->row_par;
      sd.row_bfs = ix->row_bfs;
      sd.row_flags = ix->row_flags;
      sd.par_int = ix->par_int;
      sd.X = nullptr;
      sd.DP = ix->DP;
      sd.Mf = ix->iso_Mf;
      sd.NL_iso = ix->NL_iso;
      sd.anA = ix->an_A;
      sd.anB = ix->an_B;
      sd.ld_an = ix->ld_an;
      sd.meta = ix->row_meta;
      sd.dconst = dfull;
      return sd;
    };
    // the DENSE re-run of the chunk's queries `redo` (chunk-local indices): the exact heap replay
    // (exact by construction), results scattered into the outputs
    auto dense_rerun = [&](const std::vector<int>& redo) -> int {
      ix->cat_tail_done = false;   // the DENSE re-run below writes after the last flag gather

      // DENSE re-run: the exact heap replay of the hard queries (exact by construction).  By
      // default lazily (simulate_lazy_kernel: a popped node's leaf rows scored when their
      // parent is popped); CWQ_CAT_LAZY=0: every leaf row materialised first by the exact scan.
      const char* lze = getenv("CWQ_CAT_LAZY");
      const bool lazy = !(lze && *lze && atoi(lze) == 0) && ix->DP <= 2048;
      const int64_t ldL = lazy ? 1 : std::max(ix->NL, 1);
      const int64_t cap_dense = 1 + (int64_t)ix->NI + ix->NL;
      const size_t per_q = (size_t)ix->DP * 4 + 4 * (size_t)std::max(ix->NI, 1) * 4 + (size_t)ldL * 4 +
                           (size_t)cap_dense * 16 + 64 + (size_t)k * 8 + (size_t)ix->D * 4;
      const int64_t sub = std::max<int64_t>(1, std::min<int64_t>((int64_t)redo.size(), ((size_t)2 << 30) / per_q));
      std::vector<float> hx;
      for (size_t r0 = 0; r0 < redo.size(); r0 += sub) {
        const int ns = (int)std::min<int64_t>(sub, (int64_t)redo.size() - (int64_t)r0);
        const int64_t ns_pad = round_up(ns, kQPad);
        // per hard query: dense keys, heap, then status / nodes[k] / found / calls
        if ((rc = ix->reserve(chunk_bytes(ix, ns_pad) +
                              (size_t)ns_pad * ((size_t)ldL * 4 + cap_dense * 16 + 64 + (size_t)k * 8) + 16 * 256 +
                              (size_t)ns_pad * ix->D * 4)))
          return rc;
        Bump b2(ix->ws, ix->ws_size);
        Chunk c2;
        carve_chunk(ix, b2, c2, ns);
        float* qsub = b2.take<float>((size_t)ns * ix->D);
        float* dense = b2.take<float>((size_t)ns_pad * ldL);
        HeapEnt* heap2 = b2.take<HeapEnt>((size_t)ns_pad * cap_dense);
        int* status2 = b2.take<int>(ns_pad);
        int64_t* nodes2 = b2.take<int64_t>((size_t)ns_pad * k);
        int* found2 = b2.take<int>(ns_pad);
        int64_t* calls2 = b2.take<int64_t>(ns_pad);
        std::vector<int64_t> gq(ns);   // global query index of each hard query
        for (int i = 0; i < ns; ++i) gq[i] = q0 + redo[r0 + i];
        if ((rc = ix->reserve_fb((size_t)ns * 8))) return rc;
        int64_t* d_gq = (int64_t*)ix->fb;
        HIPCHK(hipMemcpyAsync(d_gq, gq.data(), (size_t)ns * 8, hipMemcpyHostToDevice, s));
        HIPCHK(launch_copy_rows(q, ix->D, d_gq, qsub, ix->D, nullptr, ns, ix->D, s));
        HIPCHK(launch_pad_queries(qsub, ns, ix->D, c2.X, c2.nq_pad, ix->DP, s));
        if ((rc = run_internal(ix, c2, s))) return rc;
        if (!lazy && (rc = run_leaf_scan(ix, c2, EPI_KEY, true, 16, dfull, dense, ix->NL, nullptr, nullptr, nullptr, 1,
                                         nullptr, s)))
          return rc;
        SimArgs sd = base_args();
        sd.pre_status = 0;   // every hard query replays (status2 is fresh scratch)
        sd.nq = ns;
        sd.R = 0;
        sd.LPF = c2.LPF ? c2.LPF : ix->dummy;
        sd.BF = c2.BF ? c2.BF : ix->dummy;
        sd.dense_lpf = dense;
        sd.ldL = ldL;
        sd.heap = heap2;
        sd.heap_cap = cap_dense;
        sd.out_nodes = nodes2;
        sd.n_found = found2;
        sd.n_calls = calls2;
        sd.status = status2;
        if (lazy) {
          sd.X = c2.X;
          sd.DP = ix->DP;
          sd.Mf = ix->iso_Mf;
          sd.NL_iso = ix->NL_iso;
          sd.anA = ix->an_A;
          sd.anB = ix->an_B;
          sd.ld_an = ix->ld_an;
          sd.meta = ix->row_meta;
          sd.dconst = dfull;
          // the run-merge replay in LDS; a query that overflows its arena is re-run on the
          // global heap (status 1 gates it; the second kernel writes status 0)
          const char* lre = getenv("CWQ_CAT_LAZY_RUNS");
          if (!(lre && *lre && atoi(lre) == 0)) {
            HIPCHK(launch_simulate_lazy_runs(sd, s));
            sd.pre_status = 1;
          }
          HIPCHK(launch_simulate_lazy(sd, s));
          ix->lazy_stats[1] += ns;
        } else {
          HIPCHK(launch_simulate(sd, s));
        }
        HIPCHK(launch_copy_rows(nodes2, 2 * (int64_t)k, nullptr, nodes, 2 * (int64_t)k, d_gq, ns, 2 * (int64_t)k, s));
        HIPCHK(launch_copy_rows(found2, 1, nullptr, n_found, 1, d_gq, ns, 1, s));
        if (n_calls) HIPCHK(launch_copy_rows(calls2, 2, nullptr, n_calls, 2, d_gq, ns, 2, s));
        HIPCHK(hipStreamSynchronize(s));   // gq (pageable host memory) must outlive the upload
      }
      return CWQ_OK;
    };
    HIPCHK(launch_pad_queries(q + q0 * ix->D, nqc, ix->D, c.X, c.nq_pad, ix->DP, s));
    if ((rc = run_internal(ix, c, s, true, q + q0 * ix->D, direct ? -1 : (filt ? 1 : -1)))) return rc;
    if (direct) {
      // the exact replay straight away: every pushed entry scored when its parent is popped
      SimArgs sd = base_args();
      sd.nq = nqc;
      sd.R = 0;
      sd.LPF = c.LPF ? c.LPF : ix->dummy;
      sd.BF = c.BF ? c.BF : ix->dummy;
      sd.out_nodes = nodes + q0 * k;
      sd.n_found = n_found + q0;
      sd.n_calls = n_calls ? n_calls + q0 : nullptr;
      sd.status = status;
      sd.X = c.X;
      ix->cat_tail_done = false;
      if (pk == 0) {   // a few queries: the global-heap form queued behind for arena overflows
        sd.heap = b.take<HeapEnt>((size_t)nq_pad * cap_dense);
        sd.heap_cap = cap_dense;
        HIPCHK(launch_simulate_lazy_runs(sd, s));
        sd.pre_status = 1;
        HIPCHK(launch_simulate_lazy(sd, s));
        ix->stats[4] += nqc;
        ix->lazy_stats[0] += nqc;
        continue;
      }
      // a batch: the run-merge replays side by side; a query that overflows its arena goes
      // to the DENSE re-run (its heap memory only for those)
      HIPCHK(launch_simulate_lazy_runs(sd, s));
      std::vector<int> hst(nqc);
      HIPCHK(hipMemcpyAsync(hst.data(), status, (size_t)nqc * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      std::vector<int> redo;
      for (int i = 0; i < nqc; ++i)
        if (hst[i]) redo.push_back(i);
      ix->stats[4] += nqc - (int64_t)redo.size();
      ix->lazy_stats[0] += nqc - (int64_t)redo.size();
      ix->stats[1] += (int64_t)redo.size();
      if (!redo.empty() && (rc = dense_rerun(redo))) return rc;
      continue;
    }
    if (filt && (rc = group_tables(ix, c, q + q0 * ix->D, true, s))) return rc;
    int nst = 0;
    std::vector<char> fbad(nqc, 0);
    int* okf_d = nullptr;   // filter: per-query list-certified flags
    std::vector<int> okh(filt ? nqc : 0);
    if (filt && scat) {
      // anisotropic rows: the exact scan into slots 1..; isotropic rows: the stream filter
      // with the categorize key -> exact keys in list slot 0
      if ((rc = run_leaf_scan(ix, c, EPI_TOPK, true, kl, dfull, nullptr, 0, pkey, paux, prow, R, &nst, s, 2, 1, slabs)))
        return rc;
      okf_d = b.take<int>((size_t)nq_pad);
      // no anisotropic rows (nst == 1): the rerank writes list 1 itself, no merge launch
      if ((rc = nst == 1 ? stream_cat_list(ix, c, q + q0 * ix->D, nqc, R, c.BF, dfull, okey, oaux, orow, R, okf_d, b, s)
                         : stream_cat_list(ix, c, q + q0 * ix->D, nqc, R, c.BF, dfull, pkey, paux, prow,
                                           (int64_t)nst * R, okf_d, b, s)))
        return rc;
    } else if (filt) {
      // isotropic rows: the filter with the categorize key -> exact keys in list slot 0;
      // anisotropic rows: the exact scan into slots 1..
      IsoFilter fo;
      if ((rc = run_iso_filter(ix, c, q + q0 * ix->D, nqf, R, true, false, b, fo, s))) return rc;
      if ((rc = run_leaf_scan(ix, c, EPI_TOPK, true, kl, dfull, nullptr, 0, pkey, paux, prow, R, &nst, s, 2, 1, slabs)))
        return rc;
      HIPCHK(launch_final(c.X, ix->iso_Mf, ix->DP, nqc, R, kFgCapQ, fo.qcnt, fo.qover, fo.crow, fo.cu, fo.cl,
                          fo.tl + (R - 1), 64, ix->row_meta, ix->row_par, c.BF ? c.BF : ix->dummy, std::max(ix->NI, 1), 0,
                          pkey, paux, prow, (int64_t)nst * R, fo.okf, fo.nex, fo.tlk, fo.tr, fo.tdone, nullptr, 1, dfull,
                          s));
      okf_d = fo.okf;
    } else if ((rc = run_leaf_scan(ix, c, EPI_TOPK, true, kl, dfull, nullptr, 0, pkey, paux, prow, R, &nst, s, 3, 0, slabs))) {
      return rc;
    }
    if (!(filt && scat && nst == 1)) HIPCHK(launch_merge(pkey, paux, prow, nqc, nst * R, R, okey, oaux, orow, s, true));
    SimArgs sa;
    memset(&sa, 0, sizeof(sa));
    sa.nq = nqc;
    sa.k = k;
    sa.R = R;
    sa.max_nodes = max_nodes;
    sa.NI = ix->NI;
    sa.NL = ix->NL;
    sa.LPF = c.LPF ? c.LPF : ix->dummy;
    sa.BF = c.BF ? c.BF : ix->dummy;
    sa.ldI = std::max(ix->NI, 1);
    sa.lkey = okey;
    sa.laux = oaux;
    sa.lrow = orow;
    sa.complete = complete ? 1 : 0;
    sa.int_child_begin = ix->int_child_begin;
    sa.int_child_end = ix->int_child_end;
    sa.int_nchild = ix->int_nchild;
    sa.int_bfs = ix->int_bfs;
    sa.int_has_sent = ix->int_has_sent;
    sa.int_leaf_a0 = ix->int_leaf_a0;
    sa.int_leaf_a1 = ix->int_leaf_a1;
    sa.int_leaf_b0 = ix->int_leaf_b0;
    sa.int_leaf_b1 = ix->int_leaf_b1;
    sa.row_par = ix->row_par;
    sa.row_bfs = ix->row_bfs;
    sa.row_flags = ix->row_flags;
    sa.heap = heap;
    sa.heap_cap = cap_list;
    sa.out_nodes = nodes + q0 * k;
    sa.n_found = n_found + q0;
    sa.n_calls = n_calls ? n_calls + q0 : nullptr;
    sa.status = status;
    sa.par_int = ix->par_int;
    // the pop sequence by counting over the bottleneck order (cat_count_kernel); the
    // queries it cannot certify go through the heap replay (CWQ_CAT_COUNT=0: replay all)
    const char* cce = getenv("CWQ_CAT_COUNT");
    const int ccv = cce && *cce ? atoi(cce) : 1;   // 0: never, 2: always (tests)
    const bool by_count = ix->NI > 0 && !ix->any_int_sent && ccv != 0 &&
                          (ccv == 2 || ix->cat_count_idle < 8 || ix->cat_count_idle % kCatCountRetry == 0);
    if (by_count) {
      HIPCHK(launch_cat_count(sa, s));
      sa.pre_status = 1;
    }
    // the count pass's status, kept on the device for the one read-back below
    int* cst_d = by_count ? b.take<int>((size_t)nq_pad) : nullptr;
    if (by_count) HIPCHK(hipMemcpyAsync(cst_d, status, nqc * sizeof(int), hipMemcpyDeviceToDevice, s));
    if (okf_d) {
      // queries whose filter lists overflowed have no list (every entry -inf, which the
      // replay would read as "every leaf listed" and search the whole tree for: 117 ms of a
      // 142 ms C2 batch for 4 such queries); they are re-run whole below, so skip them
      HIPCHK(launch_skip_failed(status, okf_d, nqc, by_count ? 0 : 1, s));
      sa.pre_status = 1;
    }
    HIPCHK(launch_simulate(sa, s));
    // Two-level replay (simulate_two_kernel, §4.7) of the queries whose top-R list ended
    // inside a tie: a second exact leaf scan keyed by the second-level bottleneck, then
    // the replay on both lists; what it cannot certify goes to the DENSE re-run below.
    const char* tle = getenv("CWQ_CAT_TWO");
    const bool two = ix->NI > 0 && !ix->any_int_sent && !complete && R == 64 && !(tle && *tle && atoi(tle) == 0);
    // the replay on the chunk itself -- its BF / LPF, the group term tables and list 1 (okey)
    // stay on the device; list 2 by the stream filter keyed by T2 (plus the anisotropic
    // rows' exact scan); results straight into the outputs.  gate: the first replay's
    // status (queries it resolved are skipped)
    int* status2 = nullptr;
    int* okf2 = nullptr;
    auto two_chunk = [&](const int* gate) -> int {
      const size_t ldI = (size_t)std::max(ix->NI, 1);
      float* T2 = b.take<float>((size_t)nq_pad * ldI);
      float* pk2 = b.take<float>((size_t)nq_pad * slabs * R);
      float* pa2 = b.take<float>((size_t)nq_pad * slabs * R);
      int* pr2 = b.take<int>((size_t)nq_pad * slabs * R);
      float* l2k = b.take<float>((size_t)nq_pad * R);
      float* l2a = b.take<float>((size_t)nq_pad * R);
      int* l2r = b.take<int>((size_t)nq_pad * R);
      HeapEnt* heap2 = b.take<HeapEnt>((size_t)nq_pad * cap2);
      status2 = b.take<int>((size_t)nq_pad);
      okf2 = scat ? b.take<int>((size_t)nq_pad) : nullptr;   // (the exact scan's lists are certified)
      HIPCHK(launch_cat_t2(c.BF, c.LPF, (int64_t)ldI, ix->NI, nqc, ix->par_int, okey, R, T2, s));
      Chunk c2t = c;
      c2t.BF = T2;   // the categorize key reads min(T2[parent], lp)
      int nst2 = 0;
      int rc2;
      if (!scat) {   // both segments by the exact scan
        if ((rc2 = run_leaf_scan(ix, c2t, EPI_TOPK, true, kl, dfull, nullptr, 0, pk2, pa2, pr2, R, &nst2, s, 3, 0, slabs)))
          return rc2;
      } else {
        if ((rc2 = run_leaf_scan(ix, c2t, EPI_TOPK, true, kl, dfull, nullptr, 0, pk2, pa2, pr2, R, &nst2, s, 2, 1, slabs)))
          return rc2;
        if ((rc2 = nst2 == 1 ? stream_cat_list(ix, c2t, q + q0 * ix->D, nqc, R, T2, dfull, l2k, l2a, l2r, R, okf2, b, s)
                             : stream_cat_list(ix, c2t, q + q0 * ix->D, nqc, R, T2, dfull, pk2, pa2, pr2,
                                               (int64_t)nst2 * R, okf2, b, s)))
          return rc2;
      }
      if (!(scat && nst2 == 1)) HIPCHK(launch_merge(pk2, pa2, pr2, nqc, nst2 * R, R, l2k, l2a, l2r, s, true));
      SimArgs st2 = sa;
      st2.pre_status = 0;
      st2.lkey2 = l2k;
      st2.laux2 = l2a;
      st2.lrow2 = l2r;
      st2.T2 = T2;
      st2.heap = heap2;
      st2.heap_cap = cap2;
      st2.status = status2;
      st2.gate = gate;
      HIPCHK(launch_simulate_two(st2, s));
      return 0;
    };
    // speculative: the second list goes out with the first replay, one status read-back for
    // both (the last call needed it for every query; CWQ_CAT_SPEC=0 turns it off, =2 forces
    // it -- tests)
    const char* spe = getenv("CWQ_CAT_SPEC");
    const int spv = spe && *spe ? atoi(spe) : 1;
    const bool spec = two && (scat || small2) && spv != 0 && (ix->cat_two_spec || spv == 2);
    if (spec && (rc = two_chunk(status))) return rc;
    // the count status, the replay status, the filter's certified flags (and the second
    // list's) written by one kernel into host-mapped memory: one sync, no pageable copies
    if ((rc = ix->host_flags((size_t)5 * nqc))) return rc;
    HIPCHK(launch_gather_flags(ix->hflags, nqc, cst_d, status, okf_d, spec ? status2 : nullptr, spec ? okf2 : nullptr, s,
                               nodes + q0 * k, n_found + q0, k));
    HIPCHK(hipStreamSynchronize(s));
    const int* hf = ix->hflags;
    std::vector<int> cst(hf, hf + (by_count ? nqc : 0)), st(hf + nqc, hf + 2 * (size_t)nqc);
    std::vector<int> hs(spec ? hf + 3 * (size_t)nqc : hf, spec ? hf + 4 * (size_t)nqc : hf);
    std::vector<int> ho(spec ? hf + 4 * (size_t)nqc : hf, spec ? hf + 5 * (size_t)nqc : hf);
    if (okf_d) okh.assign(hf + 2 * (size_t)nqc, hf + 3 * (size_t)nqc);
    for (int i = 0; i < (int)okh.size(); ++i)
      if (!okh[i]) {
        fbad[i] = 1;
        fredo.push_back(q0 + i);
      }
    std::vector<int> redo;
    for (int i = 0; i < nqc; ++i)
      if (st[i] && !fbad[i]) redo.push_back(i);   // filter failures are re-run whole below
    int n_counted = 0;
    for (int i = 0; i < nqc; ++i) {
      if (by_count && cst[i] == 0 && !fbad[i]) ++ix->stats[3], ++n_counted;
      else if (!fbad[i]) ++ix->stats[4];
    }
    if (ccv != 0) ix->cat_count_idle = by_count && n_counted > 0 ? 0 : std::min(ix->cat_count_idle + 1, 1 << 30);
    if ((scat || small2) && two) ix->cat_two_spec = (int)redo.size() == nqc;
    if (redo.empty()) continue;

    if (spec || (two && ((scat && (int)redo.size() == nqc) || small2))) {
      if (!spec) {   // after the status read-back (gated: the first replay's resolved queries keep their results)
        if ((rc = two_chunk(status))) return rc;
        HIPCHK(launch_gather_flags(ix->hflags, nqc, status2, okf2, nullptr, nullptr, nullptr, s, nodes + q0 * k,
                                   n_found + q0, k));
        HIPCHK(hipStreamSynchronize(s));
        hs.assign(ix->hflags, ix->hflags + nqc);
        ho.assign(ix->hflags + nqc, ix->hflags + 2 * (size_t)nqc);
      }
      std::vector<int> left;
      for (const int i : redo) {
        if (hs[i] || (okf2 && !ho[i])) left.push_back(i);   // uncertified, or list 2 overflowed: DENSE
        else ++ix->stats[5];
      }
      redo.swap(left);
    } else if (two) {
      ix->cat_tail_done = false;   // the gathered replay writes after the flag gather
      std::vector<float> h1k((size_t)nqc * R), h1a((size_t)nqc * R);
      std::vector<int> h1r((size_t)nqc * R);
      HIPCHK(hipMemcpyAsync(h1k.data(), okey, h1k.size() * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(h1a.data(), oaux, h1a.size() * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(h1r.data(), orow, h1r.size() * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      std::vector<int> left;
      const size_t per_q2 = chunk_bytes(ix, kQPad) / kQPad + (size_t)std::max(ix->NI, 1) * 4 + (size_t)cap2 * 16 +
                            (size_t)R * 12 * 2 + 64 + (size_t)k * 8 + (size_t)ix->D * 4 +
                            (size_t)R * 12 * (pick_nslab(ix, ix->NL_iso, 1) + pick_nslab(ix, ix->NL_an, 1) + 2) *
                                scan_lists_per_slab(kl);
      const int64_t sub2 = std::max<int64_t>(1, std::min<int64_t>((int64_t)redo.size(), ((size_t)2 << 30) / per_q2));
      for (size_t r0 = 0; r0 < redo.size(); r0 += sub2) {
        const int ns = (int)std::min<int64_t>(sub2, (int64_t)redo.size() - (int64_t)r0);
        const int64_t ns_pad = round_up(ns, kQPad);
        const int nqb2 = n_qblocks_for(ns, kl);
        const int slabs2 = (pick_nslab(ix, ix->NL_iso, nqb2) + pick_nslab(ix, ix->NL_an, nqb2) + 2) *
                           scan_lists_per_slab(kl);
        const size_t ldI = (size_t)std::max(ix->NI, 1);
        if ((rc = ix->reserve(chunk_bytes(ix, ns_pad) +
                              (size_t)ns_pad * (ldI * 4 + (size_t)slabs2 * R * 12 + (size_t)R * 24 + cap2 * 16 + 64 +
                                                (size_t)k * 8) +
                              (size_t)ns * ix->D * 4 + 24 * 256)))
          return rc;
        Bump b2(ix->ws, ix->ws_size);
        Chunk c2;
        carve_chunk(ix, b2, c2, ns);
        float* qsub = b2.take<float>((size_t)ns * ix->D);
        float* T2 = b2.take<float>((size_t)ns_pad * ldI);
        float* pk2 = b2.take<float>((size_t)ns_pad * slabs2 * R);
        float* pa2 = b2.take<float>((size_t)ns_pad * slabs2 * R);
        int* pr2 = b2.take<int>((size_t)ns_pad * slabs2 * R);
        float* l1k = b2.take<float>((size_t)ns_pad * R);
        float* l1a = b2.take<float>((size_t)ns_pad * R);
        int* l1r = b2.take<int>((size_t)ns_pad * R);
        float* l2k = b2.take<float>((size_t)ns_pad * R);
        float* l2a = b2.take<float>((size_t)ns_pad * R);
        int* l2r = b2.take<int>((size_t)ns_pad * R);
        HeapEnt* heap2 = b2.take<HeapEnt>((size_t)ns_pad * cap2);
        int* status2 = b2.take<int>(ns_pad);
        int64_t* nodes2 = b2.take<int64_t>((size_t)ns_pad * k);
        int* found2 = b2.take<int>(ns_pad);
        int64_t* calls2 = b2.take<int64_t>(ns_pad);
        std::vector<int64_t> gq(ns);
        std::vector<float> s1k((size_t)ns * R), s1a((size_t)ns * R);
        std::vector<int> s1r((size_t)ns * R);
        for (int i = 0; i < ns; ++i) {
          const int li = redo[r0 + i];
          gq[i] = q0 + li;
          std::copy(h1k.begin() + (size_t)li * R, h1k.begin() + (size_t)(li + 1) * R, s1k.begin() + (size_t)i * R);
          std::copy(h1a.begin() + (size_t)li * R, h1a.begin() + (size_t)(li + 1) * R, s1a.begin() + (size_t)i * R);
          std::copy(h1r.begin() + (size_t)li * R, h1r.begin() + (size_t)(li + 1) * R, s1r.begin() + (size_t)i * R);
        }
        if ((rc = ix->reserve_fb((size_t)ns * 8))) return rc;
        int64_t* d_gq = (int64_t*)ix->fb;
        HIPCHK(hipMemcpyAsync(d_gq, gq.data(), (size_t)ns * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(l1k, s1k.data(), s1k.size() * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(l1a, s1a.data(), s1a.size() * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(l1r, s1r.data(), s1r.size() * 4, hipMemcpyHostToDevice, s));
        HIPCHK(launch_copy_rows(q, ix->D, d_gq, qsub, ix->D, nullptr, ns, ix->D, s));
        HIPCHK(launch_pad_queries(qsub, ns, ix->D, c2.X, c2.nq_pad, ix->DP, s));
        if ((rc = run_internal(ix, c2, s))) return rc;
        HIPCHK(launch_cat_t2(c2.BF, c2.LPF, (int64_t)ldI, ix->NI, ns, ix->par_int, l1k, R, T2, s));
        Chunk c2t = c2;
        c2t.BF = T2;   // the leaf scan's categorize key reads min(T2[parent], lp)
        int nst2 = 0;
        if ((rc = run_leaf_scan(ix, c2t, EPI_TOPK, true, kl, dfull, nullptr, 0, pk2, pa2, pr2, R, &nst2, s, 3, 0,
                                slabs2)))
          return rc;
        HIPCHK(launch_merge(pk2, pa2, pr2, ns, nst2 * R, R, l2k, l2a, l2r, s, true));
        SimArgs st = sa;
        st.nq = ns;
        st.pre_status = 0;
        st.LPF = c2.LPF;
        st.BF = c2.BF;
        st.lkey = l1k;
        st.laux = l1a;
        st.lrow = l1r;
        st.lkey2 = l2k;
        st.laux2 = l2a;
        st.lrow2 = l2r;
        st.T2 = T2;
        st.heap = heap2;
        st.heap_cap = cap2;
        st.out_nodes = nodes2;
        st.n_found = found2;
        st.n_calls = calls2;
        st.status = status2;
        HIPCHK(launch_simulate_two(st, s));
        // every result goes back; the uncertified ones are overwritten by the DENSE re-run
        HIPCHK(launch_copy_rows(nodes2, 2 * (int64_t)k, nullptr, nodes, 2 * (int64_t)k, d_gq, ns, 2 * (int64_t)k, s));
        HIPCHK(launch_copy_rows(found2, 1, nullptr, n_found, 1, d_gq, ns, 1, s));
        if (n_calls) HIPCHK(launch_copy_rows(calls2, 2, nullptr, n_calls, 2, d_gq, ns, 2, s));
        std::vector<int> hs(ns);
        HIPCHK(hipMemcpyAsync(hs.data(), status2, (size_t)ns * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));   // the pageable host sources must outlive their uploads
        for (int i = 0; i < ns; ++i) {
          if (hs[i]) left.push_back(redo[r0 + i]);
          else ++ix->stats[5];
        }
      }
      redo.swap(left);
    }
    ix->stats[1] += (int64_t)redo.size();
    n_dense_call += (int64_t)redo.size();
    if (redo.empty()) continue;
    if ((rc = dense_rerun(redo))) return rc;
  }
  if (measure && !direct) ix->cat_dense_seen = n_dense_call > 0 ? kCatDenseMemory : std::max(0, ix->cat_dense_seen - 1);
  ix->stats[2] += (int64_t)fredo.size();
  if (!fredo.empty()) {
    // filter overflow: those queries through the exact path, results scattered back
    const int64_t n = (int64_t)fredo.size();
    const size_t D = (size_t)ix->D;
    const size_t o_q = round_up(n * 8, 256), o_nd = o_q + round_up(n * D * 4, 256),
                 o_f = o_nd + round_up((int64_t)n * k * 8, 256), o_c = o_f + round_up(n * 4, 256),
                 tot = o_c + round_up(n * 8, 256);
    if (tot > ix->fb2_size) {
      if (ix->ws_ev_live) (void)hipEventSynchronize(ix->ws_ev);
      if (ix->fb2) (void)hipFree(ix->fb2);
      ix->fb2 = nullptr;
      ix->fb2_size = 0;
      if (hipMalloc(&ix->fb2, tot) != hipSuccess) return fail(CWQ_ERR_OOM, "categorize fallback buffers");
      ix->fb2_size = tot;
    }
    char* f = (char*)ix->fb2;
    int64_t* d_idx = (int64_t*)f;
    float* qs = (float*)(f + o_q);
    int64_t* nd = (int64_t*)(f + o_nd);
    int* fd = (int*)(f + o_f);
    int64_t* cl = (int64_t*)(f + o_c);
    HIPCHK(hipMemcpyAsync(d_idx, fredo.data(), n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(launch_copy_rows(q, (int64_t)D, d_idx, qs, (int64_t)D, nullptr, n, (int64_t)D, s));
    if ((rc = categorize_impl(ix, qs, n, k, max_nodes, nd, fd, cl, s, false))) return rc;
    HIPCHK(launch_copy_rows(nd, 2 * (int64_t)k, nullptr, nodes, 2 * (int64_t)k, d_idx, n, 2 * (int64_t)k, s));
    HIPCHK(launch_copy_rows(fd, 1, nullptr, n_found, 1, d_idx, n, 1, s));
    if (n_calls) HIPCHK(launch_copy_rows(cl, 2, nullptr, n_calls, 2, d_idx, n, 2, s));
    HIPCHK(hipStreamSynchronize(s));
    ix->cat_tail_done = false;
  }
  if (measure) {   // the path's per-query wall time, completed (the caller syncs after a small call anyway)
    HIPCHK(hipStreamSynchronize(s));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call).count() /
                      (double)nq;
    double& ema = direct ? ix->cat_ema_direct[pk] : ix->cat_ema_list[pk];
    ema = ema < 0.0 ? us : 0.75 * ema + 0.25 * us;
    ix->cat_pref_direct[pk] = ix->cat_ema_direct[pk] >= 0.0 && ix->cat_ema_list[pk] >= 0.0 &&
                              ix->cat_ema_direct[pk] < ix->cat_ema_list[pk];
  }
  return CWQ_OK;
}
}  // namespace

extern "C" int cwq_categorize(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t max_nodes, int64_t* nodes,
                              int32_t* n_found, int64_t* n_calls, void* stream) {
  if (!ix || (!q && nq > 0) || (nq > 0 && (!nodes || !n_found))) return fail(CWQ_ERR_ARG, "NULL argument");
  if (k <= 0) return fail(CWQ_ERR_ARG, "k must be >= 1");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  for (int64_t& t : ix->stats) t = 0;
  ix->lazy_stats[0] = ix->lazy_stats[1] = 0;
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const int rc = categorize_impl(ix, q, nq, k, max_nodes, nodes, n_found, n_calls, s, true);
  ix->stats[0] = nq;
  if (rc) return rc;
  if (!ix->cat_tail_done) HIPCHK(launch_clear_tail(nodes, n_found, nq, k, s));
  return CWQ_OK;
}

// Basic in the harness's shape (benchmark_utils.py:580-581: cobweb_predict(numpy_query, k)):
// the query through pinned staging, the pop-order node ids / found counts / call counts
// written by the kernels straight into mapped host memory, the call returning synchronized.
extern "C" int cwq_categorize_host(cwq_index* ix, const float* q, int64_t nq, int32_t k, int64_t max_nodes,
                                   int64_t* nodes, int32_t* n_found, int64_t* n_calls, void* stream) {
  if (!ix || (!q && nq > 0) || (nq > 0 && (!nodes || !n_found))) return fail(CWQ_ERR_ARG, "NULL argument");
  if (k <= 0) return fail(CWQ_ERR_ARG, "k must be >= 1");
  if (nq == 0) return CWQ_OK;
  std::lock_guard<std::mutex> lk(ix->mu);
  DevGuard dg(ix->device);
  for (int64_t& t : ix->stats) t = 0;
  ix->lazy_stats[0] = ix->lazy_stats[1] = 0;
  hipStream_t s = (hipStream_t)stream;
  WsUse wu(ix, s);
  ScanCfgScope scs(nq);
  if (wu.rc) return wu.rc;
  const size_t qb = (size_t)nq * ix->D * 4, nb = (size_t)round_up(nq * k * 8, 256), cb = (size_t)round_up(nq * 8, 256),
               fb = (size_t)nq * 4;
  int rc;
  if ((rc = ix->host_io(qb, nb + cb + fb))) return rc;
  memcpy(ix->hq, q, qb);
  HIPCHK(hipMemcpyAsync(ix->dq, ix->hq, qb, hipMemcpyHostToDevice, s));
  int64_t* hn = (int64_t*)ix->hout;
  int64_t* hc = (int64_t*)((char*)ix->hout + nb);
  int32_t* hf = (int32_t*)((char*)ix->hout + nb + cb);
  rc = categorize_impl(ix, (const float*)ix->dq, nq, k, max_nodes, hn, hf, hc, s, true);
  ix->stats[0] = nq;
  if (rc) return rc;
  if (!ix->cat_tail_done) {   // (otherwise categorize_impl's last sync already covers every write)
    HIPCHK(launch_clear_tail(hn, hf, nq, k, s));
    HIPCHK(sync_spin(s));
  }
  ix->ws_idle = true;   // synchronized
  memcpy(nodes, hn, (size_t)nq * k * 8);
  memcpy(n_found, hf, fb);
  if (n_calls) memcpy(n_calls, hc, (size_t)nq * 8);
  return CWQ_OK;
}

extern "C" int cwq_welford_groups(const float* X, int64_t n_rows, int32_t dim, const int64_t* order,
                                  const int64_t* group_ptr, int64_t n_groups, float* count, float* mean,
                                  float* meanSq, void* stream) {
  if (!X || !order || !group_ptr || !count || !mean || !meanSq || dim <= 0 || n_rows < 0)
    return fail(CWQ_ERR_ARG, "bad arguments");
  if (n_groups > 65535) return fail(CWQ_ERR_ARG, "at most 65535 groups per call");
  HIPCHK(launch_welford_groups(X, dim, order, group_ptr, n_groups, count, mean, meanSq, (hipStream_t)stream));
  return CWQ_OK;
}

// PCA + ICA whitening transform (F4) -- PCAICAWhiteningModel.transform, src/whitening/pca_ica.py:30-51.
extern "C" int cwq_whiten(const float* X, int64_t n, int32_t d_in, const float* mean, const float* comps,
                          int32_t d_pca, const float* denom, const float* unmix, int32_t d_out, float* out,
                          float* work, void* stream) {
  if (n < 0 || d_in <= 0 || d_pca <= 0 || (unmix && d_out <= 0)) return fail(CWQ_ERR_ARG, "bad whitening shape");
  if (n == 0) return CWQ_OK;
  if (!X || !mean || !comps || !denom || !out || (unmix && !work)) return fail(CWQ_ERR_ARG, "NULL argument");
  hipStream_t s = (hipStream_t)stream;
  float* pca = unmix ? work : out;
  HIPCHK(launch_gemm_nt_f32(X, n, d_in, mean, comps, d_pca, denom, pca, s));
  if (unmix) HIPCHK(launch_gemm_nt_f32(pca, n, d_pca, nullptr, unmix, d_out, nullptr, out, s));
  return CWQ_OK;
}
