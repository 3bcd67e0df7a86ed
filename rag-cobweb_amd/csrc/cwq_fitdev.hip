// libcwq: device-resident incremental fit (ifit) -- the whole insert loop
// of CobwebTorchTree.cobweb (CobwebTorchTree.py:143-233) on the GPU, with no host
// round trip per insert or per level.
//
// The tree lives in device memory: a pool of node statistics (count, mean, meanSq =
// Welford M2, CobwebTorchNode.py:31-68), parent links and per-node child lists in list
// order (slabs of an arena; append at the end, remove with the tail shifted left, as
// Python's list.append / list.remove).  The launch is one master workgroup plus (CUs - 1)
// helper workgroups, each of 512 threads (kFdThreads; one per CU).  The master runs the
// inserts in order; per tree level every child's KL terms are computed (one wave per child;
// a level with >= fork_min children -- CWQ_FIT_FORK_MIN, default 64 -- is forked: the master
// publishes a job and every workgroup claims 4-child slices, fd_fork / fd_helper), then the
// reference's scalar decisions are made in its float32 op order:
//   two_best_children (CobwebTorchNode.py:374-420): gain = p1*KL(c+x || P+x) -
//     p2*KL(c || P+x), sorted by (gain, count, random()) descending;
//   pu_for_insert / pu_for_new_child / pu_for_merge / pu_for_split (:422-650), each a
//     sequential float32 sum over the children (Python's `score += ...`);
//   get_best_operation (CobwebTorchTree.py:287-372 via fit.py): max of (pu, random(), name);
// and applies best / new / merge / split / fringe split / exact-match increment to the
// device tree.  random() is Python's own MT19937 stream (genrand_res53), run on the
// device from the state the host hands over (random.getstate()) and handed back after,
// so the draws -- b per level for the child sort, then best, new, [merge], [split] --
// are the reference's.  KL (compute_score, CobwebTorchTree.py:344-364) per element in
// the reference's fp32 op order (contraction off, correctly rounded logs: ref_logf), the
// two D-sums in torch's own float32 cascade-sum order (cwq_refmath.h torch_sum2) -- the
// reference's CPU arithmetic, and exactly cwq_fit_kl's, so this and the host-driven
// fitter (fit.py TreeFitter.ifit) build identical trees.  Every cross-workgroup wait is
// bounded; a join that times out ends the insert with FD_HANG (CWQ_ERR_HIP to the caller).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cobweb_query.h"
#include "cwq_refmath.h"

namespace cwq {

// ---------------------------------------------------------------------------
// MT19937 with Python's random.random() (genrand_res53): state = 624 words + index
// ---------------------------------------------------------------------------
constexpr int kMtN = 624, kMtM = 397;
__host__ __device__ inline uint32_t mt_u32(uint32_t* mt, int& idx) {
  if (idx >= kMtN) {
    int kk = 0;
    uint32_t y;
    for (; kk < kMtN - kMtM; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + kMtM] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    for (; kk < kMtN - 1; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (kMtM - kMtN)] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    y = (mt[kMtN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[kMtN - 1] = mt[kMtM - 1] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    idx = 0;
  }
  uint32_t y = mt[idx++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
__host__ __device__ inline double mt_random(uint32_t* mt, int& idx) {
  const uint32_t a = mt_u32(mt, idx) >> 5, b = mt_u32(mt, idx) >> 6;
  return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}
__host__ __device__ inline double mt_res53(uint32_t a, uint32_t b) {   // random() from two outputs
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
__host__ __device__ inline uint32_t mt_step(uint32_t a, uint32_t b, uint32_t m) {   // the twist of one word
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
// The twist as 227 independent chains: word kk < 227 reads old words only (kk, kk+1,
// kk+397); word kk in [227, 623) reads old kk, kk+1 and the NEW word kk-227 -- the same
// chain's previous step -- so chain t owns t, t+227, t+454; word 623 reads new 0 and 396.
// o: the 7 old words chain t reads (t, t+1, t+397, t+227, t+228, t+454, t+455); nw: its
// up to 3 new words.
constexpr int kMtChains = kMtN - kMtM;   // 227
__host__ __device__ inline int mt_chain_len(int t) { return t + 454 < kMtN - 1 ? 3 : 2; }
__host__ __device__ inline void mt_chain_load(const uint32_t* mt, int t, uint32_t o[7]) {
  o[0] = mt[t];
  o[1] = mt[t + 1];
  o[2] = mt[t + kMtM];
  o[3] = mt[t + 227];
  o[4] = mt[t + 228];
  o[5] = t + 454 < kMtN - 1 ? mt[t + 454] : 0u;
  o[6] = t + 454 < kMtN - 1 ? mt[t + 455] : 0u;
}
__host__ __device__ inline void mt_chain_run(const uint32_t o[7], int t, uint32_t nw[3]) {
  nw[0] = mt_step(o[0], o[1], o[2]);
  nw[1] = mt_step(o[3], o[4], nw[0]);
  nw[2] = t + 454 < kMtN - 1 ? mt_step(o[5], o[6], nw[1]) : 0u;
}
// Host form of the chain twist (the device runs the chains across a wave's lanes); the
// CPU test cwq_mt19937_words checks it against Python's own getrandbits(32) stream.
inline void mt_twist_chains_host(uint32_t* mt) {
  uint32_t o[kMtChains][7], n[kMtChains][3];
  const uint32_t old623 = mt[kMtN - 1];
  for (int t = 0; t < kMtChains; ++t) mt_chain_load(mt, t, o[t]);
  for (int t = 0; t < kMtChains; ++t) {
    mt_chain_run(o[t], t, n[t]);
    for (int s = 0; s < mt_chain_len(t); ++s) mt[t + 227 * s] = n[t][s];
  }
  mt[kMtN - 1] = mt_step(old623, mt[0], mt[kMtM - 1]);
}

// ---------------------------------------------------------------------------
// Device tree
// ---------------------------------------------------------------------------
struct FitDev {
  int D;
  float pv;
  int cap;                      // node slots
  float *count, *mean, *meanSq; // [cap], [cap][D]
  float* lvar;                  // [cap][D] ref_logf(meanSq / count + pv): a node's log-variances, kept
                                // current by fd_increment / fd_combine and set for every loaded node
  int *parent, *ccnt, *ccap;    // [cap]
  int64_t* coff;                // [cap] child slab offset in the arena
  int* arena;
  int64_t arena_cap;
  int* ctrl;                    // [0] used [2] root [3] status [4] mt index
  int64_t* ctrl64;              // [0] arena_top [1] rows done [2] randoms drawn
  uint32_t* mt;                 // [624]
  float *kres, *gain, *tall, *tins, *ncv;   // per-level scratch [cap]
  int* jobs;                    // [cap] split job nodes
  // the chip-wide KL pass (fork / join between the master workgroup and its helpers)
  struct FdJob* job;
  float* pvec;                  // [3][D] the job's reference vectors (mean, var, log var)
  uint32_t* rnd;                // [2*cap + 8] a level's tempered MT outputs (the sort's draws)
  int fork_min;                 // fork a level's KL pass when it has >= fork_min children
  uint64_t spin_ticks;          // bound of every spin (100 MHz steady counter ticks)
  int* dbg;                     // [16] progress words (read back by the host on FD_HANG)
  int prof;                     // CWQ_FIT_PROFILE: forked levels' phase ticks into dbg[8..13], count dbg[14] ("all": every level)
};

// 512 threads (8 waves): up to 256 VGPRs per lane -- the torch-order KL sums
// (cwq_refmath.h) spilled at 1024 threads' 128 (the kernel takes ~170, so one workgroup per CU)
constexpr int kFdThreads = 512;
constexpr int kFdWaves = kFdThreads / 64;
constexpr int kFdMaxD = 1024;   // 7 D-vectors + the MT state stay within 64 KiB of LDS
constexpr int kFdChunk = 1024;
constexpr int kFdRing = 64;     // per-job claim / completion counters, by epoch
constexpr int kFdWaveClaim = 4; // children per claim of a master wave
constexpr int kFdHelperPer = 2; // children per helper wave per workgroup claim
constexpr int kFdParTop = 8;    // unforked levels of >= this many children: parallel draws + top-2
constexpr int kFdForkMin = 64;  // default fork threshold (children of a level; 64 measured best of 32-256 on clustered 768-d data)
enum { FD_OK = 0, FD_ROOM = 1, FD_FULL = 2, FD_HANG = 3 };
// bounded spins (the steady counter runs at 100 MHz): a helper with no new job for
// spin_ticks leaves (the master never depends on helpers: it claims work itself); the master
// gives up a join after spin_ticks (status FD_HANG).  Default 20 s; CWQ_FIT_SPIN_MS.
constexpr uint64_t kFdSpinTicks = 2000000000ull;
// dbg words: 0 row, 1 forks, 2 last fork size, 3 phase, 4 done at the last join, 5 helper
// job starts, 6 helper exits, 7 helper claims

// The job a forked level hands to the helper workgroups.  Every word here is shared
// between workgroups and is only ever accessed by agent-scope atomics (loads, stores,
// adds) -- never plain (cdna_hip_programming.md §6 Guideline 16): the block is zeroed by
// a memset before every launch; epoch = job number (1, 2, ...), polled by the helpers; the
// job's descriptor and its claim / completion counters live in rings by epoch (each
// counter on a 128-B line of its own), so a helper late for job e only ever touches job
// e's own words.
struct FdDesc {
  int type;        // 0: U, T of the children arena[base .. base+n) vs (P + x); 1: KL(c || P) of jobs[0..n)
  int n;
  int kofs;        // type 1: output offset in kres
  int pad;
  int64_t base;
  int64_t row;     // the row being inserted (x = X[row])
};
struct FdJob {
  int epoch;
  int quit;
  int pad0[30];
  FdDesc desc[kFdRing];
  int next[kFdRing][32];
  int done[kFdRing][32];
};

struct FdShared {
  float x[kFdMaxD], mu2[kFdMaxD], v2[kFdMaxD], lv2[kFdMaxD];
  float muP[kFdMaxD], vP[kFdMaxD], lvP[kFdMaxD];
  float rv2[kFdMaxD], rvP[kFdMaxD];   // div_recip of v2 / vP (the KL terms' divisor per dimension)
  uint32_t mt[kMtN];
  uint32_t mtn[kMtN];   // the parallel twist's new words
  alignas(16) float cg[kFdChunk];
  alignas(16) float cn[kFdChunk];
  int ci[10];
  float cf[8];
  double cr[2];   // random() of "best" and "new"
  int flag;
  int epoch;      // master: the last job published
  // parallel top-2: every wave's two best (gain, count, random, index)
  float tg[kFdWaves][2], tn[kFdWaves][2];
  double tr[kFdWaves][2];
  int ti[kFdWaves][2];
  double logl[128];   // ref_logf's tables (kRefLogL, kRefLogC), copied in at launch
  float logc[128];
};
static_assert(sizeof(FdShared) <= 160 * 1024, "the fit workgroup's LDS");
__device__ __forceinline__ float fd_logf(const FdShared& sh, float v) { return ref_logf_tab(v, sh.logc, sh.logl); }
// the KL terms' divisions: the compiler's IEEE division.  A/B builds: FIT_DIV_RN=1 takes
// div_rn (a reciprocal per divisor and two Markstein corrections, equal to IEEE division:
// scripts/check_div_rn.hip) -- measured slower on gfx950 (clustered 20k x 768: 9.51 vs 8.19
// s, profiles/r05_fit_divrn_ab.log): the hardware sequence (v_div_scale, v_rcp, four fma,
// v_div_fmas, v_div_fixup) is cheaper than the guarded corrections plus the per-dimension
// reciprocal reads; FIT_PROBE_DIV (timing only) the bare reciprocal.
#ifdef FIT_PROBE_DIV
#define KDIV(a, b, y) ((a) * __builtin_amdgcn_rcpf(b))
#elif defined(FIT_DIV_RN)
#define KDIV(a, b, y) div_rn((a), (b), (y))
#define FIT_RECIP(b) div_recip(b)
#else
#define KDIV(a, b, y) ((a) / (b))
#endif
#ifndef FIT_RECIP
#define FIT_RECIP(b) 0.f   // the reciprocals are read by div_rn only
#endif


__device__ __forceinline__ int ld_agent(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t ld_agent64(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent_f(const float* p) {   // L1-bypassing (sc1) load
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent_f(float* p, float v) {   // write-through (sc1) store
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ONE wave: advance the MT19937 state (mt in LDS, idx) by n outputs exactly as n mt_u32
// calls would, writing the tempered outputs to out[0..n).  Every lane passes the same idx.
// A twist is 227 chains over the 64 lanes (mt_chain_*), the new words into tmp (LDS) while
// mt still holds the old ones, then copied back with word 623.
__device__ __attribute__((noinline)) void mt_gen_wave(uint32_t* mt, uint32_t* tmp, int& idx, int64_t n, uint32_t* out, int lane) {
  int64_t done = 0;
  while (done < n) {
    if (idx >= kMtN) {
      for (int t = lane; t < kMtChains; t += 64) {
        uint32_t o[7], nw[3];
        mt_chain_load(mt, t, o);
        mt_chain_run(o, t, nw);
        tmp[t] = nw[0];
        tmp[t + 227] = nw[1];
        if (t + 454 < kMtN - 1) tmp[t + 454] = nw[2];
      }
      wave_sync();
      const uint32_t last = mt_step(mt[kMtN - 1], tmp[0], tmp[kMtM - 1]);   // every lane: the same word
      wave_sync();
      tmp[kMtN - 1] = last;
      wave_sync();
      for (int i = lane; i < kMtN; i += 64) mt[i] = tmp[i];
      wave_sync();
      idx = 0;
    }
    const int take = (int)((int64_t)(kMtN - idx) < n - done ? (int64_t)(kMtN - idx) : n - done);
    for (int i = lane; i < take; i += 64) out[done + i] = mt_temper(mt[idx + i]);
    wave_sync();
    idx += take;
    done += take;
  }
}

#pragma clang fp contract(off)

// WG-wide node operations (every thread calls; barriers inside)
__device__ __forceinline__ void fd_zero(const FitDev& f, int s) {
#pragma clang fp contract(off)
  for (int d = threadIdx.x; d < f.D; d += kFdThreads) {
    f.mean[(size_t)s * f.D + d] = 0.f;
    f.meanSq[(size_t)s * f.D + d] = 0.f;
  }
  if (threadIdx.x == 0) f.count[s] = 0.f;
  __syncthreads();
}

// increment_counts (CobwebTorchNode.py:57-68)
__device__ __forceinline__ void fd_increment(const FitDev& f, int s, const float* x) {
#pragma clang fp contract(off)
  const float cd = f.count[s];
  for (int d = threadIdx.x; d < f.D; d += kFdThreads) {
    const size_t o = (size_t)s * f.D + d;
    const float cnt = cd + 1.0f;
    const float delta = x[d] - f.mean[o];
    const float m = f.mean[o] + delta / cnt;
    const float m2 = f.meanSq[o] + delta * (x[d] - m);
    f.meanSq[o] = m2;
    f.mean[o] = m;
    f.lvar[o] = ref_logf(m2 / cnt + f.pv);   // the T / split terms' log (count = cnt below)
  }
  __syncthreads();
  if (threadIdx.x == 0) f.count[s] = cd + 1.0f;
  __syncthreads();
}

// update_counts_from_node (CobwebTorchNode.py:70-85)
__device__ __forceinline__ void fd_combine(const FitDev& f, int dst, int src) {
#pragma clang fp contract(off)
  const float cd = f.count[dst], cs = f.count[src];
  for (int d = threadIdx.x; d < f.D; d += kFdThreads) {
    const size_t o = (size_t)dst * f.D + d, os = (size_t)src * f.D + d;
    const float delta = f.mean[os] - f.mean[o];
    const float tot = cd + cs;
    const float m2 = (f.meanSq[o] + f.meanSq[os]) + (delta * delta) * ((cd * cs) / tot);
    f.meanSq[o] = m2;
    f.mean[o] = (cd * f.mean[o] + cs * f.mean[os]) / tot;
    f.lvar[o] = ref_logf(m2 / tot + f.pv);
  }
  __syncthreads();
  if (threadIdx.x == 0) f.count[dst] = cd + cs;
  __syncthreads();
}

// is_exact_match (CobwebTorchNode.py:652-666, torch.isclose defaults)
__device__ __forceinline__ bool fd_exact(const FitDev& f, FdShared& sh, int s) {
#pragma clang fp contract(off)
  if (threadIdx.x == 0) sh.flag = 1;
  __syncthreads();
  const float cd = f.count[s];
  bool ok = true;
  for (int d = threadIdx.x; d < f.D; d += kFdThreads) {
    const size_t o = (size_t)s * f.D + d;
    const float sd = sqrtf(f.meanSq[o] / cd);
    if (!(fabsf(sd) <= 1e-8f)) ok = false;
    if (!(fabsf(sh.x[d] - f.mean[o]) <= 1e-8f + 1e-5f * fabsf(f.mean[o]))) ok = false;
  }
  if (!ok) sh.flag = 0;
  __syncthreads();
  const bool r = sh.flag != 0;
  __syncthreads();
  return r;
}

// thread 0; -1: pool full.  Slots are never reused within a load (a node freed by a split
// keeps its slot, marked parent = -2), so the host maps every slot it loaded to the same
// node object afterwards; slot numbers never enter a decision.
__device__ __forceinline__ int fd_alloc(const FitDev& f) {
  if (f.ctrl[0] >= f.cap) return -1;
  const int s = f.ctrl[0]++;
  f.parent[s] = -1;
  f.ccnt[s] = 0;
  f.ccap[s] = 0;
  f.coff[s] = 0;
  return s;
}

// a new zeroed node (WG-wide); s_out via LDS
__device__ __forceinline__ int fd_new_node(const FitDev& f, FdShared& sh) {
  if (threadIdx.x == 0) {
    sh.ci[0] = fd_alloc(f);
    if (sh.ci[0] < 0) f.ctrl[3] = FD_FULL;
  }
  __syncthreads();
  const int s = sh.ci[0];
  __syncthreads();
  if (s >= 0) fd_zero(f, s);
  return s;
}

// children[p].append(c)
__device__ __forceinline__ void fd_append(const FitDev& f, FdShared& sh, int p, int c) {
  if (threadIdx.x == 0) {
    sh.ci[1] = 0;
    if (f.ccnt[p] == f.ccap[p]) {   // grow: a new slab of twice the capacity at the arena top
      const int nc = f.ccap[p] < 4 ? 4 : 2 * f.ccap[p];
      const int64_t off = f.ctrl64[0];
      if (off + nc > f.arena_cap) {
        f.ctrl[3] = FD_FULL;
      } else {
        f.ctrl64[0] = off + nc;
        sh.ci[1] = 1;
        sh.ci[2] = (int)(f.coff[p] >> 32);
        sh.ci[3] = (int)(f.coff[p] & 0xffffffff);
        f.coff[p] = off;
        f.ccap[p] = nc;
      }
    }
  }
  __syncthreads();
  if (sh.ci[1]) {   // move the list into the new slab
    const int64_t old = ((int64_t)sh.ci[2] << 32) | (uint32_t)sh.ci[3];
    const int64_t nw = f.coff[p];
    const int n = f.ccnt[p];
    for (int i = threadIdx.x; i < n; i += kFdThreads) f.arena[nw + i] = f.arena[old + i];
  }
  __syncthreads();
  if (threadIdx.x == 0 && f.ctrl[3] != FD_FULL) {
    f.arena[f.coff[p] + f.ccnt[p]] = c;
    f.ccnt[p] = f.ccnt[p] + 1;
  }
  __syncthreads();
}

// children[p].remove(c): first occurrence, the tail shifted left by one
__device__ __forceinline__ void fd_remove(const FitDev& f, FdShared& sh, int p, int c) {
  const int n = f.ccnt[p];
  const int64_t base = f.coff[p];
  if (threadIdx.x == 0) sh.ci[4] = n;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kFdThreads)
    if (f.arena[base + i] == c) atomicMin(&sh.ci[4], i);
  __syncthreads();
  const int j = sh.ci[4];
  __syncthreads();
  if (j >= n) return;
  for (int c0 = j; c0 < n - 1; c0 += kFdThreads) {
    const int i = c0 + threadIdx.x;
    const int v = i < n - 1 ? f.arena[base + i + 1] : 0;
    __syncthreads();
    if (i < n - 1) f.arena[base + i] = v;
    __syncthreads();
  }
  if (threadIdx.x == 0) f.ccnt[p] = n - 1;
  __syncthreads();
}

// KL(cand || ref) of one wave: per-lane fp64 sums over d = lane, lane + 64, ..., then the
// butterfly, then (sa + sb - D) / 2 in fp32 -- cwq_fit_kl's arithmetic
// mean_var_insert (CobwebTorchNode.py:214-222) of one element, float32 op order
__device__ __forceinline__ void fd_insert_mv(float c, float m, float m2, float x, float pv, float& mo, float& vo) {
#pragma clang fp contract(off)
  const float cnt = c + 1.0f;
  const float delta = x - m;
  const float mm = m + CWQ_KDIV(delta, cnt);
  const float mm2 = m2 + delta * (x - mm);
  mo = mm;
  vo = CWQ_KDIV(mm2, cnt) + pv;
}

// KL(cand || ref) of one wave from its two sums: (Sa + Sb - D) / 2 in float32 --
// compute_score's op order (CobwebTorchTree.py:344-356)
__device__ __forceinline__ float fd_kl_score(float sa, float sb, int D) {
#pragma clang fp contract(off)
  float score = sa;
  score = score + sb;
  score = score - (float)D;
  score = score / 2.0f;
  return score;
}
// The per-child KL terms, summed in torch's order (torch_sum2), two children per wave (c0 on
// lanes 0-31, c1 on 32-63).  U = KL(c + x || P + x): mean_var_insert's ops, a log per term
// (x enters the variance)
__device__ __forceinline__ void fd_kl_U2(const FitDev& f, const FdShared& sh, int c0, int c1, int lane, float& U0,
                                        float& U1) {
#pragma clang fp contract(off)
  const int D = f.D;
  const float pv = f.pv;
  const int c = (lane >> 5) ? c1 : c0;
  const float cnt = f.count[c] + 1.0f;
  const float ycnt = FIT_RECIP(cnt);
  float sa, sb;
  torch_sum2_halves(D, lane, [&](int d, int h, float& a, float& b) {
    const size_t o = (size_t)(h ? c1 : c0) * D + d;
    const float m = f.mean[o], m2 = f.meanSq[o];
    const float xd = sh.x[d];
    const float delta = xd - m;
    const float mm = m + KDIV(delta, cnt, ycnt);
    const float num = m2 + delta * (xd - mm);
    const float v1 = KDIV(num, cnt, ycnt) + pv;
    a = sh.lv2[d] - fd_logf(sh, v1);
    const float df = mm - sh.mu2[d];
    b = KDIV((v1 + df * df), sh.v2[d], sh.rv2[d]);
  }, sa, sb);
  const float k = fd_kl_score(sa, sb, D);
  U0 = __shfl(k, 0, 64);
  U1 = __shfl(k, 32, 64);
}
// T = KL(c || P + x) of two children in one wave: the child's log-variance from its cache
// (lvar: the same ref_logf of the same m2 / cc + pv), so no log per term
__device__ __forceinline__ void fd_kl_T2(const FitDev& f, const FdShared& sh, int c0, int c1, int lane, float& T0,
                                        float& T1) {
#pragma clang fp contract(off)
  const int D = f.D;
  const float pv = f.pv;
  const float cc = f.count[(lane >> 5) ? c1 : c0];
  const float ycc = FIT_RECIP(cc);
  float sa, sb;
  torch_sum2_halves(D, lane, [&](int d, int h, float& a, float& b) {
    const size_t o = (size_t)(h ? c1 : c0) * D + d;
    const float m = f.mean[o], m2 = f.meanSq[o];
    const float v1 = KDIV(m2, cc, ycc) + pv;
    a = sh.lv2[d] - f.lvar[o];
    const float df = m - sh.mu2[d];
    b = KDIV((v1 + df * df), sh.v2[d], sh.rv2[d]);
  }, sa, sb);
  const float k = fd_kl_score(sa, sb, D);
  T0 = __shfl(k, 0, 64);
  T1 = __shfl(k, 32, 64);
}
// KL(c || ref) with the reference vectors (mu, v, log v) given
__device__ __forceinline__ float fd_kl_ref(const FitDev& f, const FdShared& sh, const float* mu, const float* v,
                                           const float* rv, const float* lv, int c, int lane) {
#pragma clang fp contract(off)
  const int D = f.D;
  const float cc = f.count[c];
  const float ycc = FIT_RECIP(cc);
  float sa, sb;
  torch_sum2(D, lane, [&](int d, float& a, float& b) {
    const float mu1 = f.mean[(size_t)c * D + d], v1 = KDIV(f.meanSq[(size_t)c * D + d], cc, ycc) + f.pv;
    a = lv[d] - f.lvar[(size_t)c * D + d];   // = fd_logf(sh, v1), cached
    const float df = mu1 - mu[d];
    b = KDIV((v1 + df * df), v[d], rv[d]);
  }, sa, sb);
  return fd_kl_score(sa, sb, D);
}
// KL(c0 || ref) and KL(c1 || ref) in one wave (c0 on lanes 0-31, c1 on lanes 32-63)
__device__ __forceinline__ void fd_kl_ref2(const FitDev& f, const FdShared& sh, const float* mu, const float* v,
                                           const float* rv, const float* lv, int c0, int c1, int lane, float& K0,
                                           float& K1) {
#pragma clang fp contract(off)
  const int D = f.D;
  const float cc0 = f.count[c0], cc1 = f.count[c1];
  const float ycc = FIT_RECIP((lane >> 5) ? cc1 : cc0);
  float sa, sb;
  torch_sum2_halves(D, lane, [&](int d, int h, float& a, float& b) {
    const size_t o = (size_t)(h ? c1 : c0) * D + d;
    const float mu1 = f.mean[o], v1 = KDIV(f.meanSq[o], (h ? cc1 : cc0), ycc) + f.pv;
    a = lv[d] - f.lvar[o];   // = fd_logf(sh, v1), cached
    const float df = mu1 - mu[d];
    b = KDIV((v1 + df * df), v[d], rv[d]);
  }, sa, sb);
  const float k = fd_kl_score(sa, sb, D);
  K0 = __shfl(k, 0, 64);
  K1 = __shfl(k, 32, 64);
}
// KL(new leaf || P + x)
__device__ __forceinline__ float fd_kl_new(const FitDev& f, const FdShared& sh, int lane) {
#pragma clang fp contract(off)
  float sa, sb;
  const float v1 = 0.f + f.pv;
  const float lv1 = fd_logf(sh, v1);
  torch_sum2(f.D, lane, [&](int d, float& a, float& b) {
    a = sh.lv2[d] - lv1;
    const float df = sh.x[d] - sh.mu2[d];
    b = KDIV((v1 + df * df), sh.v2[d], sh.rv2[d]);
  }, sa, sb);
  return fd_kl_score(sa, sb, f.D);
}

// one child of a job (ONE wave): its KL terms to kres by write-through stores
__device__ __forceinline__ void fd_job_child(const FitDev& f, const FdShared& sh, int type, int64_t base, int kofs, int j,
                                             int lane) {
  // the butterfly leaves the sums in every lane: every lane stores the same words (no
  // lane-divergent region inside the claim loops -- cf. fd_fork)
  if (type == 0) {   // kofs = the level's children b: items 0..nP-1 U pairs, nP..2nP-1 T pairs
    const int b = kofs, nP = (b + 1) / 2, i = j < nP ? j : j - nP;
    const int j0 = 2 * i, j1 = 2 * i + 1 < b ? 2 * i + 1 : 2 * i;
    const int c0 = f.arena[base + j0], c1 = f.arena[base + j1];
    float K0, K1;
    if (j < nP) fd_kl_U2(f, sh, c0, c1, lane, K0, K1);
    else fd_kl_T2(f, sh, c0, c1, lane, K0, K1);
    const int w = j < nP ? 0 : 1;
    st_agent_f(&f.kres[2 * j0 + w], K0);
    st_agent_f(&f.kres[2 * j1 + w], K1);
  } else {
    const float K = fd_kl_ref(f, sh, sh.muP, sh.vP, sh.rvP, sh.lvP, f.jobs[j], lane);
    st_agent_f(&f.kres[kofs + j], K);
  }
}

// (gain, count, random) descending; ties keep list order (Python's stable sort)
__device__ __forceinline__ bool fd_rel_before(float g1, float n1, double r1, int i1, float g2, float n2, double r2,
                                              int i2) {
  if (g1 != g2) return g1 > g2;
  if (n1 != n2) return n1 > n2;
  if (r1 != r2) return r1 > r2;
  return i1 < i2;
}

// ---------------------------------------------------------------------------
// The chip-wide KL pass.  The master workgroup (block 0) runs the insert loop; the other
// workgroups are helpers.  A level with >= fork_min children is forked: the master writes
// the job (the reference vectors, the child list) and publishes its epoch behind an agent
// release; helpers poll the epoch, acquire, and claim children per workgroup; every result
// goes out by a write-through store, and each claim's count is added to the job's done
// counter after its stores have drained; the master claims too (per wave), waits until done
// covers every child, acquires, and reads the results.  Protocol: cdna_hip_programming.md
// §6 Guideline 16 (R1 producer/consumer forms; every spin bounded).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fd_help_job(const FitDev& f, FdShared& sh, const float* X, int e) {
  FdJob* job = f.job;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, D = f.D;
  const int slot = e % kFdRing;
  FdDesc* dd = &job->desc[slot];
  const int type = ld_agent(&dd->type), n = ld_agent(&dd->n), kofs = ld_agent(&dd->kofs);
  const int64_t base = ld_agent64(&dd->base), row = ld_agent64(&dd->row);
  if (n <= 0 || n > 3 * f.cap || base < 0 || row < 0) return;   // never: a descriptor not (yet) seen
  float* mu = type ? sh.muP : sh.mu2;
  float* v = type ? sh.vP : sh.v2;
  float* rv = type ? sh.rvP : sh.rv2;
  float* lv = type ? sh.lvP : sh.lv2;
  for (int d = tid; d < D; d += kFdThreads) {
    mu[d] = f.pvec[d];
    v[d] = f.pvec[D + d];
    rv[d] = FIT_RECIP(v[d]);
    lv[d] = f.pvec[2 * D + d];
    if (type == 0) sh.x[d] = X[row * D + d];
  }
  __syncthreads();
  constexpr int per = kFdWaves * kFdHelperPer;
  for (;;) {
    // wave 0 claims for the workgroup: every lane takes part in the atomic (lane 0 adds
    // `per`, the others 0) -- no lane-divergent region in these loops: the compiler's
    // restructuring of one (an atomic under `if (lane == 0)` plus a readlane in the loop
    // head) re-ran an iteration without its claim
    if (wave == 0) {
      const bool live = ld_agent(&job->epoch) == e;
      const int v = atomicAdd(&job->next[slot][0], (lane == 0 && live) ? per : 0);
      sh.ci[0] = live ? __builtin_amdgcn_readlane(v, 0) : n;
    }
    __syncthreads();
    const int j0 = __builtin_amdgcn_readfirstlane(sh.ci[0]);   // uniform loop control
    __syncthreads();
    if (j0 >= n) break;
    const int j1 = j0 + per < n ? j0 + per : n;
    for (int j = j0 + wave; j < j1; j += kFdWaves) fd_job_child(f, sh, type, base, kofs, j, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave's stores drained
    __syncthreads();
    if (wave == 0) {
      atomicAdd(&job->done[slot][0], lane == 0 ? j1 - j0 : 0);
      atomicAdd(&f.dbg[7], lane == 0 ? 1 : 0);
    }
  }
}

__device__ __forceinline__ void fd_helper(const FitDev& f, FdShared& sh, const float* X) {
  const int tid = threadIdx.x;
  int seen = 0;
  for (;;) {
    if (tid == 0) {
      int e = -1;
      const uint64_t t0 = (uint64_t)wall_clock64();
      for (;;) {
        if (ld_agent(&f.job->quit)) break;
        const int ep = ld_agent(&f.job->epoch);
        if (ep != seen) {
          e = ep;
          break;
        }
        if ((uint64_t)wall_clock64() - t0 > f.spin_ticks) break;   // bounded: the master needs no helper
        __builtin_amdgcn_s_sleep(2);
      }
      if (e > 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      sh.ci[1] = e;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int e = __builtin_amdgcn_readfirstlane(sh.ci[1]);
    __syncthreads();
    if (e <= 0) {
      if (tid == 0) atomicAdd(&f.dbg[6], 1);
      return;
    }
    seen = e;
    if (tid == 0) atomicAdd(&f.dbg[5], 1);
    fd_help_job(f, sh, X, e);
  }
}

// master (all threads): fork a job over n items and join it.  Wave 0 first generates
// `nrnd` MT outputs of the level's sort draws into f.rnd (advancing thread 0's mt_idx),
// wave 1 first computes the new leaf's term (type 0, into kres[2n]); then every master
// wave claims items too.  false: the join timed out.
__device__ __forceinline__ bool fd_fork(const FitDev& f, FdShared& sh, int64_t row, int type, int n, int64_t base, int kofs,
                        int64_t nrnd, int& mt_idx) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, D = f.D;
  FdJob* job = f.job;
  const float* mu = type ? sh.muP : sh.mu2;
  const float* v = type ? sh.vP : sh.v2;
  const float* lv = type ? sh.lvP : sh.lv2;
  for (int d = tid; d < D; d += kFdThreads) {
    f.pvec[d] = mu[d];
    f.pvec[D + d] = v[d];
    f.pvec[2 * D + d] = lv[d];
  }
  const int e = sh.epoch + 1;
  const int slot = e % kFdRing;
  if (tid == 0) {
    FdDesc* dd = &job->desc[slot];
    st_agent(&dd->type, type);
    st_agent(&dd->n, n);
    st_agent(&dd->kofs, kofs);
    st_agent64(&dd->base, base);
    st_agent64(&dd->row, row);
    st_agent(&job->next[slot][0], 0);
    st_agent(&job->done[slot][0], 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {   // publish: agent release of everything the master wrote, then the epoch
    st_agent(&f.dbg[1], e);
    st_agent(&f.dbg[2], n);
    st_agent(&f.dbg[3], 1);
    sh.epoch = e;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_agent(&job->epoch, e);
  }
  if (wave == 0 && nrnd > 0) {
    int idx = __builtin_amdgcn_readlane(mt_idx, 0);
    mt_gen_wave(sh.mt, sh.mtn, idx, nrnd, f.rnd, lane);
    if (lane == 0) mt_idx = idx;
  }
  if (wave == 1 && type == 0) {   // kofs = the level's children
    const float K = fd_kl_new(f, sh, lane);
    if (lane == 0) f.kres[2 * kofs] = K;
  }
  for (;;) {   // per wave; every lane in every atomic (fd_help_job)
    const int v = atomicAdd(&job->next[slot][0], lane == 0 ? kFdWaveClaim : 0);
    const int j0 = __builtin_amdgcn_readlane(v, 0);   // wave-uniform (scalar) loop control
    if (j0 >= n) break;
    const int j1 = j0 + kFdWaveClaim < n ? j0 + kFdWaveClaim : n;
    for (int j = j0; j < j1; ++j) fd_job_child(f, sh, type, base, kofs, j, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicAdd(&job->done[slot][0], lane == 0 ? j1 - j0 : 0);
  }
  __syncthreads();
  if (tid == 0) {
    st_agent(&f.dbg[3], 2);
    const uint64_t t0 = (uint64_t)wall_clock64();
    int ok = 1;
    while (ld_agent(&job->done[slot][0]) < n) {
      if ((uint64_t)wall_clock64() - t0 > f.spin_ticks) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    st_agent(&f.dbg[4], ld_agent(&job->done[slot][0]));
    st_agent(&f.dbg[3], ok ? 3 : 4);
    sh.ci[1] = ok;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bool ok = sh.ci[1] != 0;
  __syncthreads();
  return ok;
}

// acc += v[a], v[a+1], ..., v[e-1] in order (sequential float32, Python's `score += ...`);
// the first term is taken as is while `fst` (the reference's first `+=` onto 0 keeps its
// sign of zero only this way).  One lane: 16 values read ahead of their adds (four
// ds_read_b128 in flight while the previous adds run), so the chain runs at the VALU's
// dependent-add rate instead of one LDS round trip per value.
__device__ __forceinline__ void fd_add_run(float& acc, bool& fst, const float* v, int a, int e) {
  if (a < e && fst) {
    acc = v[a++];
    fst = false;
  }
  while (a < e && (a & 3)) acc = acc + v[a++];
  for (; a + 16 <= e; a += 16) {
    float4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = *reinterpret_cast<const float4*>(v + a + 4 * u);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = acc + w[u].x;
      acc = acc + w[u].y;
      acc = acc + w[u].z;
      acc = acc + w[u].w;
    }
  }
  for (; a + 4 <= e; a += 4) {
    const float4 w = *reinterpret_cast<const float4*>(v + a);
    acc = acc + w.x;
    acc = acc + w.y;
    acc = acc + w.z;
    acc = acc + w.w;
  }
  while (a < e) acc = acc + v[a++];
}

// top-2 lists of (gain, count, random, index), best first; index -1 = empty
struct FdTop2 {
  float g1, n1, g2, n2;
  double r1, r2;
  int i1, i2;
};
__device__ __forceinline__ bool fd_before(float g, float n, double r, int i, float g2, float n2, double r2, int i2) {
  if (i2 < 0) return i >= 0;
  if (i < 0) return false;
  return fd_rel_before(g, n, r, i, g2, n2, r2, i2);
}
__device__ __forceinline__ void fd_top2_offer(FdTop2& t, float g, float n, double r, int i) {
  if (fd_before(g, n, r, i, t.g1, t.n1, t.r1, t.i1)) {
    t.g2 = t.g1; t.n2 = t.n1; t.r2 = t.r1; t.i2 = t.i1;
    t.g1 = g; t.n1 = n; t.r1 = r; t.i1 = i;
  } else if (fd_before(g, n, r, i, t.g2, t.n2, t.r2, t.i2)) {
    t.g2 = g; t.n2 = n; t.r2 = r; t.i2 = i;
  }
}

// two_best_children over b children in parallel (master, all threads): the same order as
// the sequential sort (gain, count, random() descending, list order), the random() of child
// j being the level's draws 2j, 2j+1 in f.rnd.  Returns the indices in sh.ci[2], sh.ci[3].
__device__ __forceinline__ void fd_top2_parallel(const FitDev& f, FdShared& sh, int b) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  FdTop2 t{0.f, 0.f, 0.f, 0.f, 0.0, 0.0, -1, -1};
  for (int j = tid; j < b; j += kFdThreads)
    fd_top2_offer(t, f.gain[j], f.ncv[j], mt_res53(f.rnd[2 * j], f.rnd[2 * j + 1]), j);
  for (int off = 32; off > 0; off >>= 1) {
    const float og1 = __shfl_xor(t.g1, off, 64), on1 = __shfl_xor(t.n1, off, 64);
    const float og2 = __shfl_xor(t.g2, off, 64), on2 = __shfl_xor(t.n2, off, 64);
    const double or1 = __shfl_xor(t.r1, off, 64), or2 = __shfl_xor(t.r2, off, 64);
    const int oi1 = __shfl_xor(t.i1, off, 64), oi2 = __shfl_xor(t.i2, off, 64);
    fd_top2_offer(t, og1, on1, or1, oi1);
    fd_top2_offer(t, og2, on2, or2, oi2);
  }
  if (lane == 0) {
    sh.tg[wave][0] = t.g1; sh.tn[wave][0] = t.n1; sh.tr[wave][0] = t.r1; sh.ti[wave][0] = t.i1;
    sh.tg[wave][1] = t.g2; sh.tn[wave][1] = t.n2; sh.tr[wave][1] = t.r2; sh.ti[wave][1] = t.i2;
  }
  __syncthreads();
  if (tid == 0) {
    FdTop2 r{0.f, 0.f, 0.f, 0.f, 0.0, 0.0, -1, -1};
    for (int w = 0; w < kFdWaves; ++w)
      for (int k = 0; k < 2; ++k) fd_top2_offer(r, sh.tg[w][k], sh.tn[w][k], sh.tr[w][k], sh.ti[w][k]);
    sh.ci[2] = r.i1;
    sh.ci[3] = r.i2;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kFdThreads) void fit_insert_kernel(const FitDev f, const float* __restrict__ X, int64_t n,
                                                                int* leaf_out) {
#pragma clang fp contract(off)
  extern __shared__ char fd_smem[];
  FdShared& sh = *reinterpret_cast<FdShared*>(fd_smem);
  for (int i = threadIdx.x; i < 128; i += kFdThreads) {
    sh.logc[i] = kRefLogC[i];
    sh.logl[i] = kRefLogL[i];
  }
  __syncthreads();
  if (blockIdx.x > 0) {   // a helper of the chip-wide KL passes
    fd_helper(f, sh, X);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = f.D;
  const float pv = f.pv;
  if (tid == 0) sh.epoch = 0;
  for (int i = tid; i < kMtN; i += kFdThreads) sh.mt[i] = f.mt[i];
  int mt_idx = f.ctrl[4];   // thread 0's copy is the live one
  double drawn = 0;
  __syncthreads();
  int64_t row = f.ctrl64[1];
  for (; row < n; ++row) {
    // room for one more insert: arena below half, a few free slots (host compacts/grows)
    if (f.ctrl64[0] > f.arena_cap / 2 || f.ctrl[0] + 64 > f.cap) {
      if (tid == 0) f.ctrl[3] = FD_ROOM;
      break;
    }
    for (int d = tid; d < D; d += kFdThreads) sh.x[d] = X[row * D + d];
    if (tid == 0 && f.dbg) st_agent(&f.dbg[0], (int)row);
    __syncthreads();
    int cur = f.ctrl[2];
    int leaf = -1;
    while (cur >= 0) {
      const int b = f.ccnt[cur];
      if (b == 0) {
        // leaf: exact match or the empty root -> increment (CobwebTorchTree.py:184-188)
        if (f.count[cur] == 0.f || fd_exact(f, sh, cur)) {
          fd_increment(f, cur, sh.x);
          leaf = cur;
          break;
        }
        // fringe split (:190-204): new = copy of cur in cur's place, cur and a new leaf under it
        const int nw = fd_new_node(f, sh);
        if (nw < 0) break;
        const int gp = f.parent[cur];
        if (tid == 0) f.parent[nw] = gp;
        __syncthreads();
        fd_combine(f, nw, cur);
        if (tid == 0) f.parent[cur] = nw;
        __syncthreads();
        fd_append(f, sh, nw, cur);
        if (gp >= 0) {
          fd_remove(f, sh, gp, cur);
          fd_append(f, sh, gp, nw);
        } else if (tid == 0) {
          f.ctrl[2] = nw;
        }
        __syncthreads();
        fd_increment(f, nw, sh.x);
        const int ch = fd_new_node(f, sh);
        if (ch < 0) break;
        if (tid == 0) f.parent[ch] = nw;
        __syncthreads();
        fd_increment(f, ch, sh.x);
        fd_append(f, sh, nw, ch);
        leaf = ch;
        break;
      }
      // ---- internal node: the CU terms of every operation ----
      const bool prof = f.prof && f.dbg && f.job != nullptr && (b >= f.fork_min || f.prof == 2);
      uint64_t tprev = prof ? (uint64_t)wall_clock64() : 0;
      auto stamp = [&](int k) {   // thread 0: ticks since the previous stamp into dbg[8 + k]
        if (prof && tid == 0) {
          const uint64_t t = (uint64_t)wall_clock64();
          atomicAdd(&f.dbg[8 + k], (int)(t - tprev));
          tprev = t;
        }
      };
      const float cP = f.count[cur];
      for (int d = tid; d < D; d += kFdThreads) {   // P + x (mean_var_insert of the parent)
        float m, v;
        fd_insert_mv(cP, f.mean[(size_t)cur * D + d], f.meanSq[(size_t)cur * D + d], sh.x[d], pv, m, v);
        sh.mu2[d] = m;
        sh.v2[d] = v;
        sh.rv2[d] = FIT_RECIP(v);
        sh.lv2[d] = fd_logf(sh, v);
      }
      __syncthreads();
      stamp(5);   // P + x (into dbg[13])
      const int64_t cbase = f.coff[cur];
      // per child: U = KL(c + x || P + x), T = KL(c || P + x); the new leaf's KL(new || P + x).
      // A level of >= fork_min children goes over the whole chip (fd_fork), the level's b
      // sort draws generated meanwhile; a smaller one stays in this workgroup (one wave per
      // child, the draws sequential below)
      const bool forked = f.job != nullptr && b >= f.fork_min;
      if (forked) {
        if (!fd_fork(f, sh, row, 0, 2 * ((b + 1) / 2), cbase, b, 2 * (int64_t)b, mt_idx)) {
          if (tid == 0) f.ctrl[3] = FD_HANG;
          break;
        }
        if (tid == 0) drawn += b;
      } else {
        if (b >= kFdParTop && wave == 0) {   // the level's sort draws, as a fork makes them
          int idx = __builtin_amdgcn_readlane(mt_idx, 0);
          mt_gen_wave(sh.mt, sh.mtn, idx, 2 * (int64_t)b, f.rnd, lane);
          if (lane == 0) mt_idx = idx;
        }
        if (b >= kFdParTop && tid == 0) drawn += b;
        // tasks: the U pairs (a log per term) first, then the new leaf, then the T pairs
        // (cached logs), so the heavy waves go in the first round
        const int nP = (b + 1) / 2;
        for (int t = wave; t < 2 * nP + 1; t += kFdWaves) {
          if (t == nP) {
            const float K = fd_kl_new(f, sh, lane);
            if (lane == 0) f.kres[2 * b] = K;
            continue;
          }
          const int i = t < nP ? t : t - nP - 1;
          const int j0 = 2 * i, j1 = 2 * i + 1 < b ? 2 * i + 1 : 2 * i;
          const int c0 = f.arena[cbase + j0], c1 = f.arena[cbase + j1];
          float K0, K1;
          if (t < nP) fd_kl_U2(f, sh, c0, c1, lane, K0, K1);
          else fd_kl_T2(f, sh, c0, c1, lane, K0, K1);
          const int w = t < nP ? 0 : 1;
          if (lane == 0) {
            f.kres[2 * j0 + w] = K0;
            f.kres[2 * j1 + w] = K1;
          }
        }
      }
      __syncthreads();
      stamp(0);   // the KL pass (fork / join)
      // fp32 terms per child (parallel; numpy's elementwise float32 ops of fit.py)
      const float nP1 = cP + 1.0f;
      for (int j = tid; j < b; j += kFdThreads) {
        const int c = f.arena[cbase + j];
        const float nc = f.count[c];
        const float U = forked ? ld_agent_f(&f.kres[2 * j]) : f.kres[2 * j];
        const float T = forked ? ld_agent_f(&f.kres[2 * j + 1]) : f.kres[2 * j + 1];
        const float p1 = (nc + 1.0f) / nP1, p2 = nc / nP1;
        f.gain[j] = p1 * U - p2 * T;
        f.tall[j] = p2 * T;
        f.tins[j] = p1 * U;
        f.ncv[j] = nc;
      }
      __syncthreads();
      stamp(1);   // the per-child terms
      // two_best_children: one random() per child, in list order
      int i1 = -1, i2 = -1;
      if (forked || b >= kFdParTop) {
        fd_top2_parallel(f, sh, b);   // the draws are in f.rnd already
        i1 = sh.ci[2];
        i2 = sh.ci[3];
        __syncthreads();
      } else {
        float g1 = 0.f, n1 = 0.f, g2 = 0.f, n2 = 0.f;
        double r1 = 0.0, r2 = 0.0;
        for (int c0 = 0; c0 < b; c0 += kFdChunk) {   // chunks staged in LDS
          const int m = b - c0 < kFdChunk ? b - c0 : kFdChunk;
          for (int j = tid; j < m; j += kFdThreads) {
            sh.cg[j] = f.gain[c0 + j];
            sh.cn[j] = f.ncv[c0 + j];
          }
          __syncthreads();
          if (tid == 0) {
            for (int j = 0; j < m; ++j) {
              const double r = mt_random(sh.mt, mt_idx);
              drawn += 1;
              const float g = sh.cg[j], nn = sh.cn[j];
              const int id = c0 + j;
              if (i1 < 0 || fd_rel_before(g, nn, r, id, g1, n1, r1, i1)) {
                i2 = i1; g2 = g1; n2 = n1; r2 = r1;
                i1 = id; g1 = g; n1 = nn; r1 = r;
              } else if (i2 < 0 || fd_rel_before(g, nn, r, id, g2, n2, r2, i2)) {
                i2 = id; g2 = g; n2 = nn; r2 = r;
              }
            }
          }
          __syncthreads();
        }
      }
      // every thread needs the two best (the pu sums' chains run in three waves); the
      // sequential form above leaves them in thread 0
      if (tid == 0) {
        sh.ci[8] = i1;
        sh.ci[9] = i2;
      }
      __syncthreads();
      i1 = sh.ci[8];
      i2 = sh.ci[9];
      stamp(2);   // two_best_children
      // pu sums (sequential float32 in list order -- Python's `score += ...`): the three sums
      // are three dependent chains, so each runs in its own wave (lane 0; waves 0-2 sit on
      // different SIMDs) as runs of plain adds over LDS chunks (fd_add_run).  One thread
      // running all three with a read and a first-term select per value was 1.3 ms per level
      // at fan-out 19k -- 90% of a chip-wide insert (profiles/r04_fit_flat20k_profile_v1.log).
      float q_all = 0.f, q_ins = 0.f, q_keep = 0.f;
      {
        // chain 0: all terms; chain 1: term i1 replaced by tins[i1]; chain 2: i1, i2 skipped.
        // Each chain is runs of plain adds between its special indices (s0 <= s1).  The
        // chunks are double-buffered: waves 3.. stage chunk c+1 while waves 0-2 add chunk c.
        float acc = 0.f;
        bool fst = true;
        const float tins1 = (wave == 1 && lane == 0 && i1 >= 0) ? f.tins[i1] : 0.f;
        int s0 = 0x7fffffff, s1 = 0x7fffffff;
        if (wave == 1 && i1 >= 0) s0 = i1;
        if (wave == 2) {
          const int a0 = i1 >= 0 ? i1 : 0x7fffffff, a1 = i2 >= 0 ? i2 : 0x7fffffff;
          s0 = a0 < a1 ? a0 : a1;
          s1 = a0 < a1 ? a1 : a0;
        }
        {
          const int m = b < kFdChunk ? b : kFdChunk;
          for (int j = tid; j < m; j += kFdThreads) sh.cg[j] = f.tall[j];
        }
        __syncthreads();
        int cur = 0;
        for (int c0 = 0; c0 < b; c0 += kFdChunk) {
          const int m = b - c0 < kFdChunk ? b - c0 : kFdChunk;
          float* cb = cur ? sh.cn : sh.cg;
          float* nb = cur ? sh.cg : sh.cn;
          if (wave >= 3) {
            const int n0 = c0 + kFdChunk;
            const int nm = b - n0 < kFdChunk ? b - n0 : kFdChunk;
            for (int j = tid - 192; j < nm; j += kFdThreads - 192) nb[j] = f.tall[n0 + j];
          } else if (lane == 0) {
            __builtin_amdgcn_s_setprio(3);   // the chains are the critical path; staging waits
            int lo = c0;
            const int hi = c0 + m;
            while (lo < hi) {
              const int sp = s0 >= lo ? s0 : (s1 >= lo ? s1 : 0x7fffffff);
              const int end = sp < hi ? sp : hi;
              fd_add_run(acc, fst, cb, lo - c0, end - c0);
              lo = end;
              if (lo < hi) {   // lo == sp: chain 1 takes tins[i1] there, chain 2 skips it
                if (wave == 1) {
                  acc = fst ? tins1 : acc + tins1;
                  fst = false;
                }
                ++lo;
              }
            }
            __builtin_amdgcn_s_setprio(0);
          }
          __syncthreads();
          cur ^= 1;
        }
        if (lane == 0 && (wave == 1 || wave == 2)) sh.cf[4 + wave] = acc;   // cf[5] ins, cf[6] keep
        if (wave == 0) q_all = acc;
        __syncthreads();
        q_ins = sh.cf[5];
        q_keep = sh.cf[6];
      }
      stamp(3);   // the pu sums
      // the operation choice: thread 0
      if (tid == 0) {
        const float knew = f.kres[2 * b];
        const float pu_best = q_ins / (float)b;
        const float pu_new = (q_all + (1.0f / nP1) * knew) / (float)(b + 1);
        const double r_best = mt_random(sh.mt, mt_idx), r_new = mt_random(sh.mt, mt_idx);
        drawn += 2;
        sh.ci[0] = f.arena[cbase + i1];
        sh.ci[1] = i2 >= 0 ? f.arena[cbase + i2] : -1;
        sh.ci[2] = i1;
        sh.ci[3] = i2;
        sh.ci[5] = (b > 2 && i2 >= 0) ? 1 : 0;          // merge applies
        sh.ci[6] = f.ccnt[sh.ci[0]] > 0 ? 1 : 0;        // split applies
        sh.cf[0] = pu_best;
        sh.cf[1] = pu_new;
        sh.cf[2] = q_keep;
        sh.cr[0] = r_best;
        sh.cr[1] = r_new;
      }
      __syncthreads();
      const int b1 = sh.ci[0], b2 = sh.ci[1];
      const bool do_merge = sh.ci[5] != 0, do_split = sh.ci[6] != 0;
      const float pu_best = sh.cf[0], pu_new = sh.cf[1], s_keep = sh.cf[2];
      const double r_best = sh.cr[0], r_new = sh.cr[1];
      // merge / split terms
      float k_merge = 0.f;
      int n_split = 0;
      if (do_split) {
        for (int d = tid; d < D; d += kFdThreads) {   // P without x
          const float m = f.mean[(size_t)cur * D + d], v = f.meanSq[(size_t)cur * D + d] / cP + pv;
          sh.muP[d] = m;
          sh.vP[d] = v;
          sh.rvP[d] = FIT_RECIP(v);
          sh.lvP[d] = fd_logf(sh, v);
        }
        // the split's nodes: cur's children except b1, then b1's children (list order)
        const int nb1 = f.ccnt[b1];
        const int64_t b1base = f.coff[b1];
        n_split = b - 1 + nb1;
        for (int j = tid; j < b; j += kFdThreads) {
          if (j == sh.ci[2]) continue;
          f.jobs[j < sh.ci[2] ? j : j - 1] = f.arena[cbase + j];
        }
        for (int j = tid; j < nb1; j += kFdThreads) f.jobs[b - 1 + j] = f.arena[b1base + j];
      }
      __syncthreads();
      if (do_merge && wave == kFdWaves - 1) {   // mean_var_merge(b1, b2) with x vs P + x
        const float c1 = f.count[b1], c2 = f.count[b2];
        const float ytot = FIT_RECIP(c1 + c2), ycn = FIT_RECIP((c1 + c2) + 1.0f);
        float sa, sb;
        torch_sum2(D, lane, [&](int d, float& a, float& bb) {
#pragma clang fp contract(off)
          const float ma = f.mean[(size_t)b1 * D + d], mb = f.mean[(size_t)b2 * D + d];
          const float sa2 = f.meanSq[(size_t)b1 * D + d], sb2 = f.meanSq[(size_t)b2 * D + d];
          const float delta = mb - ma;
          const float tot = c1 + c2;
          float m2 = (sa2 + sb2) + (delta * delta) * ((c1 * c2) / tot);
          float m = KDIV((c1 * ma + c2 * mb), tot, ytot);
          const float cnt = tot + 1.0f;
          const float xd = sh.x[d];
          const float dl = xd - m;
          m = m + KDIV(dl, cnt, ycn);
          m2 = m2 + dl * (xd - m);
          const float v1 = KDIV(m2, cnt, ycn) + pv;
          a = sh.lv2[d] - fd_logf(sh, v1);
          const float df = m - sh.mu2[d];
          bb = KDIV((v1 + df * df), sh.v2[d], sh.rv2[d]);
        }, sa, sb);
        const float K = fd_kl_score(sa, sb, D);
        if (lane == 0) sh.cf[3] = K;
      }
      const bool split_forked = do_split && f.job != nullptr && n_split >= f.fork_min;
      if (do_split) {   // KL(c || P) of the split's nodes
        if (split_forked) {
          if (!fd_fork(f, sh, row, 1, n_split, 0, 2 * b + 1, 0, mt_idx)) {
            if (tid == 0) f.ctrl[3] = FD_HANG;
            break;
          }
        } else {
          // two nodes per wave; the merge's wave (the last) sits this out when there is one
          const int nsw = do_merge ? kFdWaves - 1 : kFdWaves;
          for (int j = 2 * wave; wave < nsw && j < n_split; j += 2 * nsw) {
            const int j1 = j + 1 < n_split ? j + 1 : j;
            float K0, K1;
            fd_kl_ref2(f, sh, sh.muP, sh.vP, sh.rvP, sh.lvP, f.jobs[j], f.jobs[j1], lane, K0, K1);
            if (lane == 0) {
              f.kres[2 * b + 1 + j] = K0;
              f.kres[2 * b + 1 + j1] = K1;
            }
          }
        }
      }
      __syncthreads();
      stamp(7);   // the merge and split KL terms (into dbg[15])
      if (do_split) {
        // the split's partition-utility sum, sequential float32 in list order (Python's
        // `score += ...`): the terms formed by all threads into LDS chunks (their KL results
        // and counts are global loads -- one at a time in thread 0 they were a serial chain
        // of uncached loads, milliseconds at fan-out 16k), thread 0 adds them in order
        float ssum = 0.f;
        bool sfirst = true;
        for (int c0 = 0; c0 < n_split; c0 += kFdChunk) {
          const int m = n_split - c0 < kFdChunk ? n_split - c0 : kFdChunk;
          for (int j = tid; j < m; j += kFdThreads) {
            const int jj = c0 + j;
            const float ks = split_forked ? ld_agent_f(&f.kres[2 * b + 1 + jj]) : f.kres[2 * b + 1 + jj];
            sh.cg[j] = (f.count[f.jobs[jj]] / cP) * ks;
          }
          __syncthreads();
          if (tid == 0) fd_add_run(ssum, sfirst, sh.cg, 0, m);
          __syncthreads();
        }
        if (tid == 0) sh.cf[4] = ssum;
        __syncthreads();
      }
      if (tid == 0) {
        // get_best_operation: max of (pu, random(), name); names "best" < "merge" < "new" < "split"
        float bp = pu_best;
        double br = r_best;
        int bn = 0;   // 0 best, 1 merge, 2 new, 3 split (the names' order)
        auto offer = [&](float pu, double r, int nm) {
          if (pu > bp || (pu == bp && (r > br || (r == br && nm > bn)))) {
            bp = pu;
            br = r;
            bn = nm;
          }
        };
        offer(pu_new, r_new, 2);
        if (do_merge) {
          k_merge = sh.cf[3];
          const float pm = ((f.count[b1] + f.count[b2]) + 1.0f) / nP1;
          const float pu_merge = (s_keep + pm * k_merge) / (float)(b - 1);
          const double r = mt_random(sh.mt, mt_idx);
          drawn += 1;
          offer(pu_merge, r, 1);
        }
        if (do_split) {
          const float pu_split = sh.cf[4] / (float)(b - 1 + f.ccnt[b1]);
          const double r = mt_random(sh.mt, mt_idx);
          drawn += 1;
          offer(pu_split, r, 3);
        }
        sh.ci[7] = bn;
      }
      __syncthreads();
      stamp(4);   // merge / split terms and the choice
      if (prof && tid == 0) atomicAdd(&f.dbg[14], 1);
      const int op = sh.ci[7];
      __syncthreads();
      if (op == 0) {          // best: into b1
        fd_increment(f, cur, sh.x);
        cur = b1;
      } else if (op == 2) {   // new child
        fd_increment(f, cur, sh.x);
        const int ch = fd_new_node(f, sh);
        if (ch < 0) break;
        if (tid == 0) f.parent[ch] = cur;
        __syncthreads();
        fd_increment(f, ch, sh.x);
        fd_append(f, sh, cur, ch);
        leaf = ch;
        break;
      } else if (op == 1) {   // merge (CobwebTorchNode.py:517-548)
        fd_increment(f, cur, sh.x);
        const int nc = fd_new_node(f, sh);
        if (nc < 0) break;
        if (tid == 0) f.parent[nc] = cur;
        __syncthreads();
        fd_combine(f, nc, b1);
        fd_combine(f, nc, b2);
        if (tid == 0) {
          f.parent[b1] = nc;
          f.parent[b2] = nc;
        }
        __syncthreads();
        fd_append(f, sh, nc, b1);
        fd_append(f, sh, nc, b2);
        fd_remove(f, sh, cur, b1);
        fd_remove(f, sh, cur, b2);
        fd_append(f, sh, cur, nc);
        cur = nc;
      } else {                // split (CobwebTorchNode.py:593-609): b1's children move up to cur
        fd_remove(f, sh, cur, b1);
        const int nb1 = f.ccnt[b1];
        for (int j = 0; j < nb1; ++j) {
          const int c = f.arena[f.coff[b1] + j];
          if (tid == 0) f.parent[c] = cur;
          __syncthreads();
          fd_append(f, sh, cur, c);
        }
        if (tid == 0) {
          f.ccnt[b1] = 0;
          f.parent[b1] = -2;   // freed
        }
        __syncthreads();
      }
      if (f.ctrl[3] >= FD_FULL) break;
      __syncthreads();
    }
    __syncthreads();
    if (f.ctrl[3] >= FD_FULL) break;
    if (tid == 0) {
      leaf_out[row] = leaf;
      f.ctrl64[1] = row + 1;
    }
    __syncthreads();
  }
  __syncthreads();
  for (int i = tid; i < kMtN; i += kFdThreads) f.mt[i] = sh.mt[i];
  if (tid == 0) {
    f.ctrl[4] = mt_idx;
    f.ctrl64[2] += (int64_t)drawn;
    if (f.job != nullptr) st_agent(&f.job->quit, 1);   // the helpers leave
  }
}

// lvar[n][d] = ref_logf(meanSq / count + pv) for nodes 0..n-1 (count 0: unused slot, 0)
__global__ void fd_lvar_kernel(const FitDev f, int n) {
#pragma clang fp contract(off)
  const int64_t nt = (int64_t)n * f.D;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nt; t += (int64_t)gridDim.x * blockDim.x) {
    const float c = f.count[t / f.D];
    f.lvar[t] = c > 0.f ? ref_logf(f.meanSq[t] / c + f.pv) : 0.f;
  }
}

}  // namespace cwq

using namespace cwq;

struct cwq_fit {
  int device = 0;
  FitDev f{};
  std::vector<void*> allocs;
  void* zero = nullptr;
};

static thread_local std::string g_fit_err;
static int fit_fail(int code, const std::string& m) {
  g_fit_err = m;
  return code;
}

extern "C" const char* cwq_fit_last_error(void) { return g_fit_err.c_str(); }

extern "C" int cwq_fit_create(int device, int32_t dim, float prior_var, int32_t cap_nodes, cwq_fit** out) {
  if (!out || dim <= 0 || dim > kFdMaxD || cap_nodes <= 0) return fit_fail(CWQ_ERR_ARG, "bad cwq_fit_create arguments");
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "hipSetDevice failed");
  std::unique_ptr<cwq_fit> h(new cwq_fit());
  h->device = device;
  FitDev& f = h->f;
  f.D = dim;
  f.pv = prior_var;
  f.cap = cap_nodes;
  // child-list arena: a load uses <= 6 entries per node (lists at twice their length, >= 4),
  // inserts stop for room at half of it, which keeps room for the largest list to double
  f.arena_cap = (int64_t)16 * cap_nodes + 4096;
  auto al = [&](void** p, size_t b) -> bool {
    if (hipMalloc(p, b < 256 ? 256 : b) != hipSuccess) return false;
    h->allocs.push_back(*p);
    return true;
  };
  const size_t C = (size_t)cap_nodes;
  bool ok = al((void**)&f.count, C * 4) && al((void**)&f.mean, C * dim * 4) && al((void**)&f.meanSq, C * dim * 4) &&
            al((void**)&f.lvar, C * dim * 4) &&
            al((void**)&f.parent, C * 4) && al((void**)&f.ccnt, C * 4) && al((void**)&f.ccap, C * 4) &&
            al((void**)&f.coff, C * 8) && al((void**)&f.arena, (size_t)f.arena_cap * 4) &&
            al((void**)&f.ctrl, 64) && al((void**)&f.ctrl64, 64) &&
            al((void**)&f.mt, kMtN * 4) && al((void**)&f.kres, (3 * C + 8) * 4) && al((void**)&f.gain, C * 4) &&
            al((void**)&f.tall, C * 4) && al((void**)&f.tins, C * 4) && al((void**)&f.ncv, C * 4) &&
            al((void**)&f.jobs, (2 * C + 8) * 4) && al((void**)&f.job, sizeof(FdJob)) &&
            al((void**)&f.pvec, (size_t)3 * dim * 4) && al((void**)&f.rnd, (2 * C + 8) * 4) &&
            al((void**)&f.dbg, 64);
  if (!ok) {
    for (void* p : h->allocs) (void)hipFree(p);
    return fit_fail(CWQ_ERR_OOM, "cwq_fit_create: device allocation failed");
  }
  *out = h.release();
  return CWQ_OK;
}

extern "C" int cwq_fit_destroy(cwq_fit* h) {
  if (!h) return CWQ_OK;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (void* p : h->allocs) (void)hipFree(p);
  delete h;
  return CWQ_OK;
}

// Load a tree into slots 0..n_nodes-1 (parent -1 for the root; child lists as CSR in list
// order; statistics from the host) and the random() state (mt: 624 words + index,
// Python's random.getstate()[1]).
extern "C" int cwq_fit_load(cwq_fit* h, int32_t n_nodes, int32_t root, const int32_t* parent,
                            const int32_t* child_ptr, const int32_t* child_idx, const float* count,
                            const float* mean, const float* meanSq, const uint32_t* mt_state, void* stream) {
  if (!h || n_nodes <= 0 || n_nodes > h->f.cap || root < 0 || root >= n_nodes || !parent || !child_ptr || !count ||
      !mean || !meanSq || !mt_state)
    return fit_fail(CWQ_ERR_ARG, "bad cwq_fit_load arguments");
  FitDev& f = h->f;
  if ((int64_t)child_ptr[n_nodes] > f.arena_cap / 4) return fit_fail(CWQ_ERR_ARG, "child lists exceed the arena");
  hipStream_t s = (hipStream_t)stream;
  if (hipSetDevice(h->device) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "hipSetDevice failed");
  std::vector<int> ccnt(n_nodes), ccap(n_nodes);
  std::vector<int64_t> coff(n_nodes);
  std::vector<int> arena;
  arena.reserve((size_t)child_ptr[n_nodes] * 2 + 16);
  for (int i = 0; i < n_nodes; ++i) {
    const int c0 = child_ptr[i], c1 = child_ptr[i + 1];
    ccnt[i] = c1 - c0;
    ccap[i] = ccnt[i] < 4 ? 4 : ccnt[i] * 2;
    coff[i] = (int64_t)arena.size();
    for (int j = c0; j < c1; ++j) arena.push_back(child_idx[j]);
    arena.resize(arena.size() + (ccap[i] - ccnt[i]), 0);
  }
  if ((int64_t)arena.size() > f.arena_cap / 2) return fit_fail(CWQ_ERR_ARG, "child lists exceed the arena");
  std::vector<int> ctrl(16, 0);
  ctrl[0] = n_nodes;
  ctrl[2] = root;
  ctrl[3] = FD_OK;
  ctrl[4] = (int)mt_state[kMtN];
  std::vector<int64_t> ctrl64(8, 0);
  ctrl64[0] = (int64_t)arena.size();
  const size_t D = (size_t)f.D;
#define FCPY(dst, src, bytes)                                                                        \
  if ((bytes) && hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) != hipSuccess)            \
    return fit_fail(CWQ_ERR_HIP, "cwq_fit_load upload failed");
  FCPY(f.parent, parent, (size_t)n_nodes * 4);
  FCPY(f.ccnt, ccnt.data(), (size_t)n_nodes * 4);
  FCPY(f.ccap, ccap.data(), (size_t)n_nodes * 4);
  FCPY(f.coff, coff.data(), (size_t)n_nodes * 8);
  FCPY(f.arena, arena.data(), arena.size() * 4);
  FCPY(f.count, count, (size_t)n_nodes * 4);
  FCPY(f.mean, mean, (size_t)n_nodes * D * 4);
  FCPY(f.meanSq, meanSq, (size_t)n_nodes * D * 4);
  FCPY(f.ctrl, ctrl.data(), ctrl.size() * 4);
  FCPY(f.ctrl64, ctrl64.data(), ctrl64.size() * 8);
  FCPY(f.mt, mt_state, (size_t)kMtN * 4);
#undef FCPY
  {   // the loaded nodes' log-variances (the cache fd_increment / fd_combine keep current)
    const int64_t nt = (int64_t)n_nodes * D;
    hipLaunchKernelGGL(fd_lvar_kernel, dim3((unsigned)std::min<int64_t>((nt + 255) / 256, 65536)), dim3(256), 0, s, f,
                       n_nodes);
    if (hipGetLastError() != hipSuccess) return fit_fail(CWQ_ERR_HIP, "cwq_fit_load log-variance launch failed");
  }
  if (hipStreamSynchronize(s) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "cwq_fit_load sync failed");
  return CWQ_OK;
}

// Insert rows X[rows_done..n) (device [n][dim]) in order; leaf_out[i] (device) = the slot
// of the node row i ended in (ifit's return value).  Runs until every row is in or the
// pool/arena needs room (info[2] = 1: export, reload with a larger capacity, call again).
// info (host): {rows done, randoms drawn (total), status, slots in use}.
extern "C" int cwq_fit_insert(cwq_fit* h, const float* X, int64_t n, int32_t* leaf_out, int64_t* info,
                              void* stream) {
  if (!h || (!X && n > 0) || (!leaf_out && n > 0) || !info) return fit_fail(CWQ_ERR_ARG, "bad cwq_fit_insert arguments");
  if (hipSetDevice(h->device) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = sizeof(FdShared);
  // helper workgroups for the chip-wide KL passes: one per other CU (CWQ_FIT_HELPERS
  // overrides; 0 = the single-workgroup loop); levels of >= CWQ_FIT_FORK_MIN children fork
  int cus = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) cus = 1;
  int helpers = cus > 1 ? cus - 1 : 0;
  if (const char* e = getenv("CWQ_FIT_HELPERS")) helpers = atoi(e) < 0 ? 0 : atoi(e);
  FitDev f = h->f;
  f.fork_min = kFdForkMin;
  if (const char* e = getenv("CWQ_FIT_FORK_MIN")) f.fork_min = atoi(e) < 2 ? 2 : atoi(e);
  f.spin_ticks = kFdSpinTicks;
  if (const char* e = getenv("CWQ_FIT_SPIN_MS")) f.spin_ticks = (uint64_t)(atoll(e) > 0 ? atoll(e) : 1) * 100000ull;
  f.prof = getenv("CWQ_FIT_PROFILE") ? (strcmp(getenv("CWQ_FIT_PROFILE"), "all") == 0 ? 2 : 1) : 0;
  if (helpers == 0) f.job = nullptr;
  else if (hipMemsetAsync(f.job, 0, sizeof(FdJob), s) != hipSuccess || hipMemsetAsync(f.dbg, 0, 64, s) != hipSuccess)
    return fit_fail(CWQ_ERR_HIP, "job reset failed");
  hipLaunchKernelGGL(fit_insert_kernel, dim3(1 + helpers), dim3(kFdThreads), lds, s, f, X, n, leaf_out);
  if (hipGetLastError() != hipSuccess) return fit_fail(CWQ_ERR_HIP, "fit_insert_kernel launch failed");
  if (getenv("CWQ_FIT_WATCH") && f.dbg) {
    // diagnostics: the kernel's progress words, read on a second stream while it runs
    hipStream_t ws = nullptr;
    int* hd = nullptr;
    if (hipStreamCreateWithFlags(&ws, hipStreamNonBlocking) == hipSuccess &&
        hipHostMalloc((void**)&hd, 64, hipHostMallocDefault) == hipSuccess) {
      for (int it = 0; hipStreamQuery(s) == hipErrorNotReady; ++it) {
        if (hipMemcpyAsync(hd, f.dbg, 64, hipMemcpyDeviceToHost, ws) == hipSuccess && hipStreamSynchronize(ws) == hipSuccess)
          fprintf(stderr, "[fit watch %d] row %d forks %d n %d phase %d done %d hjobs %d hexits %d hclaims %d\n", it, hd[0],
                  hd[1], hd[2], hd[3], hd[4], hd[5], hd[6], hd[7]);
        usleep(500000);
      }
    }
    if (hd) (void)hipHostFree(hd);
    if (ws) (void)hipStreamDestroy(ws);
  }
  int ctrl[16];
  int64_t c64[8];
  if (hipMemcpyAsync(ctrl, h->f.ctrl, 64, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(c64, h->f.ctrl64, 64, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fit_fail(CWQ_ERR_HIP, "cwq_fit_insert sync failed");
  info[0] = c64[1];
  info[1] = c64[2];
  info[2] = ctrl[3];
  info[3] = ctrl[0];
  if (f.prof && f.dbg && f.job) {   // diagnostics: where a forked level's time goes (100 MHz ticks)
    int dbg[16];
    if (hipMemcpy(dbg, f.dbg, 64, hipMemcpyDeviceToHost) == hipSuccess && dbg[14] > 0)
      fprintf(stderr, "[fit profile] %d %s levels, us per level: P+x %.1f, KL pass %.1f, child terms %.1f, top-2 %.1f, "
                      "pu sums %.1f, merge/split KL %.1f, split sum + choice %.1f\n", dbg[14], f.prof == 2 ? "internal" : "forked",
              dbg[13] * 0.01 / dbg[14], dbg[8] * 0.01 / dbg[14], dbg[9] * 0.01 / dbg[14], dbg[10] * 0.01 / dbg[14],
              dbg[11] * 0.01 / dbg[14], dbg[15] * 0.01 / dbg[14], dbg[12] * 0.01 / dbg[14]);
  }
  if (ctrl[3] == FD_FULL) return fit_fail(CWQ_ERR_OOM, "cwq_fit_insert: node pool or child arena exhausted mid-insert");
  if (ctrl[3] == FD_HANG) {
    int dbg[16];
    std::string m = "cwq_fit_insert: a chip-wide KL pass did not complete; state";
    if (hipMemcpy(dbg, h->f.dbg, 64, hipMemcpyDeviceToHost) == hipSuccess)
      for (int i = 0; i < 8; ++i) m += " " + std::to_string(dbg[i]);
    return fit_fail(CWQ_ERR_HIP, m);
  }
  // the next call resumes: clear the room flag
  if (ctrl[3] == FD_ROOM) {
    const int z = 0;
    if (hipMemcpyAsync(h->f.ctrl + 3, &z, 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return fit_fail(CWQ_ERR_HIP, "cwq_fit_insert reset failed");
  }
  return CWQ_OK;
}

// Export the device tree: slots in use (out2[0]), root (out2[1]); parent [cap] (-2: a
// node removed by a split), child CSR (child_ptr [cap+1], child_idx [cap]), count [cap],
// mean / meanSq [cap][dim] (host), mt_state [625] (the random() state to hand back).
extern "C" int cwq_fit_export(cwq_fit* h, int32_t* out2, int32_t* parent, int32_t* child_ptr, int32_t* child_idx,
                              float* count, float* mean, float* meanSq, uint32_t* mt_state, void* stream) {
  if (!h || !out2 || !parent || !child_ptr || !child_idx || !count || !mean || !meanSq || !mt_state)
    return fit_fail(CWQ_ERR_ARG, "bad cwq_fit_export arguments");
  if (hipSetDevice(h->device) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  FitDev& f = h->f;
  int ctrl[16];
  int64_t c64[8];
  if (hipMemcpyAsync(ctrl, f.ctrl, 64, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(c64, f.ctrl64, 64, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fit_fail(CWQ_ERR_HIP, "cwq_fit_export failed");
  const int used = ctrl[0];
  const size_t D = (size_t)f.D;
  std::vector<int> ccnt(used);
  std::vector<int64_t> coff(used);
  std::vector<int> arena((size_t)c64[0]);
#define FGET(dst, src, bytes)                                                                        \
  if ((bytes) && hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s) != hipSuccess)            \
    return fit_fail(CWQ_ERR_HIP, "cwq_fit_export download failed");
  FGET(parent, f.parent, (size_t)used * 4);
  FGET(ccnt.data(), f.ccnt, (size_t)used * 4);
  FGET(coff.data(), f.coff, (size_t)used * 8);
  FGET(arena.data(), f.arena, arena.size() * 4);
  FGET(count, f.count, (size_t)used * 4);
  FGET(mean, f.mean, (size_t)used * D * 4);
  FGET(meanSq, f.meanSq, (size_t)used * D * 4);
  FGET(mt_state, f.mt, (size_t)kMtN * 4);
#undef FGET
  if (hipStreamSynchronize(s) != hipSuccess) return fit_fail(CWQ_ERR_HIP, "cwq_fit_export sync failed");
  mt_state[kMtN] = (uint32_t)ctrl[4];
  child_ptr[0] = 0;
  for (int i = 0; i < used; ++i) {
    const int nc = parent[i] == -2 ? 0 : ccnt[i];
    for (int j = 0; j < nc; ++j) child_idx[child_ptr[i] + j] = arena[coff[i] + j];
    child_ptr[i + 1] = child_ptr[i] + nc;
  }
  out2[0] = used;
  out2[1] = ctrl[2];
  return CWQ_OK;
}

// Host run of the chain-form twist (mt_twist_chains_host, the device's mt_gen_wave
// arithmetic): n 32-bit outputs -- Python's getrandbits(32) stream -- from state625 (updated).
extern "C" int cwq_mt19937_words(uint32_t* state625, int64_t n, uint32_t* out) {
  if (!state625 || n < 0 || (n > 0 && !out)) return CWQ_ERR_ARG;
  int idx = (int)state625[kMtN];
  for (int64_t i = 0; i < n; ++i) {
    if (idx >= kMtN) {
      mt_twist_chains_host(state625);
      idx = 0;
    }
    out[i] = mt_temper(state625[idx++]);
  }
  state625[kMtN] = (uint32_t)idx;
  return CWQ_OK;
}

// Advance state625 past nwords 32-bit outputs (Python's genrand_uint32 stream) without
// tempering them: the rest of the current block by its index, then whole twists.  A
// Basic query advances the global random() stream by the draws the reference makes
// (CobwebTorchTree.py:243,268,285 -- 2 words per random()): ~2M words on a flat 1M tree,
// where getrandbits(64 n) built an 8 MB integer (4.5 ms).  The twist is the standard
// three-segment loop (no loop-carried dependence closer than 227 words, so the compiler
// vectorises each segment).
namespace {
void mt_twist_plain(uint32_t* __restrict__ mt) {
  for (int kk = 0; kk < kMtN - kMtM; ++kk) {
    const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
    mt[kk] = mt[kk + kMtM] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  for (int base = kMtN - kMtM; base < kMtN - 1; base += kMtN - kMtM) {   // reads words >= 227 back
    const int end = std::min(base + (kMtN - kMtM), kMtN - 1);
    for (int kk = base; kk < end; ++kk) {
      const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (kMtM - kMtN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
  }
  const uint32_t y = (mt[kMtN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
  mt[kMtN - 1] = mt[kMtM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}
}  // namespace

extern "C" int cwq_mt19937_skip(uint32_t* state625, int64_t nwords) {
  if (!state625 || nwords < 0) return CWQ_ERR_ARG;
  int64_t idx = state625[kMtN];
  if (idx > kMtN) return CWQ_ERR_ARG;
  const int64_t avail = kMtN - idx;
  if (nwords <= avail) {
    state625[kMtN] = (uint32_t)(idx + nwords);
    return CWQ_OK;
  }
  nwords -= avail;
  while (nwords > 0) {   // Python twists when the index reaches 624, then takes words 0..
    mt_twist_plain(state625);
    const int64_t take = std::min<int64_t>(nwords, kMtN);
    idx = take;
    nwords -= take;
  }
  state625[kMtN] = (uint32_t)idx;
  return CWQ_OK;
}

// Host run of the device MT19937 code (CPU test of the random() stream; no GPU).
extern "C" int cwq_mt19937_draw(uint32_t* state625, int64_t n, double* out) {
  if (!state625 || n < 0 || (n > 0 && !out)) return CWQ_ERR_ARG;
  int idx = (int)state625[kMtN];
  for (int64_t i = 0; i < n; ++i) out[i] = mt_random(state625, idx);
  state625[kMtN] = (uint32_t)idx;
  return CWQ_OK;
}
