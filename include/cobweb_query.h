/*
 * cobweb_query.h -- C ABI of libcwq, the MI355X (gfx950) query engine for the
 * Cobweb retrieval path of Teachable-AI-Lab/RAG-Cobweb (reference @ 2025-09-26).
 *
 * The reference exposes no native boundary: its interface is the Python class
 * CobwebWrapper (src/cobweb/CobwebWrapper.py).  Each entry point below replaces
 * one op sequence of that class (file:line cited per function).  The Python
 * drop-in (rag-cobweb_amd/wrapper.py) binds these symbols with ctypes.
 *
 * Conventions
 *   - Every function returns int status: CWQ_OK (0) or a negative CWQ_ERR_*;
 *     cwq_last_error() returns a thread-local message for the last failure.
 *   - Pointers documented "device" are HIP device pointers (e.g. a torch tensor's
 *     data_ptr()); "host" pointers are ordinary CPU memory.  Outputs are written
 *     into caller-allocated buffers; the library never frees caller memory.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).  All
 *     query calls are stream-ordered and asynchronous unless stated otherwise.
 *   - Node numbering is the reference's BFS order (CobwebWrapper.py:107-132):
 *     node 0 is the root and the children of a node are consecutive, in the
 *     order of its children list.  Sentence ids are the reference's sentence ids.
 *   - A handle serialises its query calls (host mutex) and owns one device
 *     workspace.  Calls may be issued on different streams: each call makes its
 *     stream wait for the previous call's work (an event recorded at the end of every
 *     call), so the workspace is never shared by two in-flight calls.  For concurrent
 *     execution use one handle per stream.
 */
#ifndef COBWEB_QUERY_H
#define COBWEB_QUERY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CWQ_OK 0
#define CWQ_ERR_ARG (-1)        /* invalid argument / malformed tree            */
#define CWQ_ERR_HIP (-2)        /* HIP runtime error                            */
#define CWQ_ERR_OOM (-3)        /* device allocation failed                     */
#define CWQ_ERR_NOT_FOUND (-4)  /* categorize retrieved < k nodes (the reference
                                   raises IndexError, CobwebTorchTree.py:289)    */

typedef struct cwq_index cwq_index;

/* Library version (major*10000 + minor*100 + patch). */
int cwq_version(void);

/* Build id: a hash of the sources, this header and the compile flags the library was
 * built from (rag-cobweb_amd/build.py); the Python binding refuses a library whose id
 * differs from the sources next to it. */
const char* cwq_build_id(void);

/* Thread-local message describing the last error on this thread. */
const char* cwq_last_error(void);

/*
 * Build the immutable query index from a flattened tree.
 * Replaces CobwebWrapper.build_prediction_index (CobwebWrapper.py:91-208): the
 * caller passes the BFS-ordered node statistics the reference caches in
 * _node_means / _node_vars (:186-203) and the structure the reference keeps in
 * _index_to_node / _leaf_to_path_indices / _path_matrix (:107-184).
 *
 *   device            HIP device ordinal the index lives on
 *   n_nodes, dim      Nn nodes of dimension D
 *   mean, var         device, [n_nodes*dim] fp32 row-major; var = compute_var
 *                     (meanSq/count + prior_var, or prior_var for empty nodes)
 *   parent            host, [n_nodes] int64; parent[0] = -1 and parent is
 *                     non-decreasing (BFS order)
 *   node_of_sentence  host, [n_sent] int64; the BFS node holding sentence id s
 *                     (-1: the sentence is not in the tree)
 *   level_w, n_w      host level weights (CobwebWrapper.py:153-166); depth >= n_w
 *                     uses 1.0; each path term is weighted level_w[depth]/len(path)
 *   stream            stream for the build kernels (the call synchronises it)
 */
int cwq_index_create(int device, int64_t n_nodes, int32_t dim, const float* mean, const float* var,
                     const int64_t* parent, const int64_t* node_of_sentence, int64_t n_sent,
                     const double* level_w, int32_t n_w, void* stream, cwq_index** out);

/*
 * cwq_index_create with the variances in compact form (same index, same results).
 * In the reference every count-1 leaf has var = meanSq/1 + prior_var = prior_var in all
 * D dimensions (CobwebTorchTree.py:336-342, CobwebWrapper.py:186-203), so a flat 10M x
 * 1024 tree's _node_vars is 41 GB of one repeated value.  Here:
 *   var_row   device [n_nodes] fp32: the variance of node i in every dimension, for the
 *             nodes NOT listed in an_nodes
 *   an_nodes  host [n_an] int64: the nodes whose variances differ across dimensions
 *             (internal nodes, leaves holding several points), each listed once
 *   an_var    device [n_an*dim] fp32: their compute_var rows, in an_nodes order
 * Other arguments as cwq_index_create.  The caller may free every input on return.
 */
int cwq_index_create_cv(int device, int64_t n_nodes, int32_t dim, const float* mean, const float* var_row,
                        const int64_t* an_nodes, int64_t n_an, const float* an_var, const int64_t* parent,
                        const int64_t* node_of_sentence, int64_t n_sent, const double* level_w, int32_t n_w,
                        void* stream, cwq_index** out);

int cwq_index_destroy(cwq_index* idx);

/* Index facts: out[0]=n_nodes out[1]=dim out[2]=n_sent out[3]=internal nodes
 * out[4]=leaf-class rows out[5]=isotropic rows out[6]=max depth out[7]=device bytes
 * (the handle's own copies; the workspace grows on demand up to 40% of the free device
 * memory, 2-48 GiB, per call; CWQ_WS_BUDGET_MB overrides).
 * Device footprint per node row: internal nodes 8*DP B (1/sigma, mu/sigma), isotropic
 * leaf rows 4*DP (dim-major mean) + 4*DP (row-major mean) + 2*DPB (bf16) + 32 B,
 * anisotropic leaf rows 8*DP B; C3 (1M x 768) 7.8 GB, C4 (10M x 1024) 104 GB -- the
 * largest flat tree one 288 GB MI355X holds is ~25M x 1024 (the caller may free its
 * mean/var tensors after cwq_index_create). */
int cwq_index_info(const cwq_index* idx, int64_t* out8);

/* How the filters centre their rows (no reference counterpart: a property of this
 * index's bf16 filter operands): out[0] = 1 when isotropic rows are stored centred at
 * their group centre's mean (clustered trees, cwq_group.hip; CWQ_GROUP_CENTRE=0 / 1 at
 * index creation: off / on wherever it applies), out[1] = groups, out[2] = group-centred
 * rows, out[3] = 1 when the per-call int8 panel was built. */
int cwq_index_filter_info(const cwq_index* idx, int64_t* out4);

/* The tree-adaptive cut the index chose (no reference counterpart): out[0] =
 * groups (centre nodes; 0: none planned), out[1] = top nodes (the root and the centres'
 * ancestors, computed exactly by every pruned query), out[2] = the deepest centre's depth,
 * out[3] = groups whose rows qualify for centring at their centre.  CWQ_GROUP_CUT=1 at index
 * creation keeps the depth-1 cut. */
int cwq_index_cut_info(const cwq_index* idx, int64_t* out4);

/* After cwq_categorize / cwq_categorize_host (no reference counterpart): out[0] =
 * queries replayed straight away by the exact lazy replay (a call of <= 64 queries on an
 * index whose list paths left every query of the last calls to the DENSE re-run; env
 * CWQ_CAT_DIRECT=0 / 1: never / always), out[1] = queries whose DENSE re-run was that lazy
 * replay (leaf rows scored when their parent is popped; CWQ_CAT_LAZY=0: the materialised
 * form).  Either way the pop order, n_found and call counts are the heap search's. */
int cwq_last_lazy_stats(const cwq_index* idx, int64_t* out2);

/*
 * "Cobweb Fast" batched top-k (A6).  Replaces CobwebWrapper.cobweb_predict_indexed
 * (CobwebWrapper.py:210-265, alias cobweb_predict_fast :428-433) for nq queries:
 * score(s) = sum over the root->leaf path of (w[depth]/len) * lp'(node), with
 * lp'(n) = -0.5*(sum_d log v + sum_d (x-mu)^2/v) (:230-241); top-k descending.
 *   q        device [nq*dim] fp32 queries
 *   ids      device [nq*k] int64 sentence ids (-1 past the number of sentences)
 *   scores   device [nq*k] fp32 scores (may be NULL)
 * Ties are broken by lower node index, then lower sentence id (the reference
 * adds randn*1e-6 noise instead, :246-256).  Any k >= 1 is accepted; k >= n_sent
 * returns the full ranking like the reference's argsort branch (:246-251).
 */
int cwq_score_topk(cwq_index* idx, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                   void* stream);

/*
 * All sentence scores (A8).  Replaces CobwebWrapper.cobweb_rank_scores
 * (CobwebWrapper.py:267-294).  out: device [nq*n_sent] fp32 (sentences that are
 * not in the tree get -inf).
 */
int cwq_rank_scores(cwq_index* idx, const float* q, int64_t nq, float* out, void* stream);

/*
 * Per-node Gaussian log-likelihood for every node in BFS order.
 *   full = 0: lp'(n) as CobwebWrapper.py:232-236 (no 2*pi term)
 *   full = 1: CobwebTorchNode.log_prob (CobwebTorchNode.py:100-104, with 2*pi)
 * out: device [nq*n_nodes] fp32.
 */
int cwq_node_logprob(cwq_index* idx, const float* q, int64_t nq, int32_t full, float* out, void* stream);

/*
 * Diagnostic (parity tests): the Fast path's internal path prefixes P (the level-
 * weighted sum of lp' along the path: the reference's sparse path matrix,
 * CobwebWrapper.py:145-180, restricted to ancestors) of every internal node by the
 * exact fp32 pass -> exact, and the rigorous bf16-MFMA bounds lo <= exact <= hi the
 * filter uses on hierarchical trees (NaN for nodes the filter does not read: with the
 * default path-sum bounds, internal nodes without isotropic leaf children).  All
 * device [nq][n_internal] fp32, internal nodes in BFS order; 1 <= nq <= 4096.
 * CWQ_ERR_ARG when the index keeps no bounds (flat tree, no isotropic leaf rows).
 */
int cwq_prefix_bounds(cwq_index* idx, const float* q, int64_t nq, float* lo, float* hi, float* exact, void* stream);

/*
 * "Cobweb Basic" best-first categorize (A4).  Replaces CobwebTorchTree.categorize
 * / _cobweb_categorize with retrieve_k=k (CobwebTorchTree.py:235-310) as called by
 * CobwebWrapper.cobweb_predict (CobwebWrapper.py:435-461).
 *   nodes     device [nq*k] int64: BFS indices of the retrieved nodes in pop order
 *             (-1 past n_found)
 *   n_found   device [nq] int32: number retrieved (< k where the reference raises
 *             IndexError: too few leaves, or max_nodes reached, :264-289)
 *   n_calls   device [nq] int64: log_prob evaluations the reference would make
 *             (may be NULL)
 * Heap ties: (-lp, parent lp, BFS index) -- the reference uses random() as the
 * third key.  The call synchronises `stream` (it may re-run hard queries).
 * Returns CWQ_OK also when some queries found < k nodes: callers check n_found
 * (the Python drop-in raises IndexError there, as the reference does).
 */
int cwq_categorize(cwq_index* idx, const float* q, int64_t nq, int32_t k, int64_t max_nodes, int64_t* nodes,
                   int32_t* n_found, int64_t* n_calls, void* stream);

/*
 * Device timing of the phases of the last cwq_score_topk call, measured with HIP
 * events recorded on the stream the kernels run on (enable first; timing mode
 * synchronises the stream once per query chunk).  Milliseconds:
 *   out[0] leaf rows (scan, or the whole filter pipeline)   out[1] internal-node pass
 *   out[2] merge + sentence expansion                        out[3] whole call
 *   out[4] number of leaf-row launches
 *   filter pipeline only: out[5] threshold sample pass (fgemm + select)
 *   out[6] the filter fgemm launches (sum)                  out[7] last bucket + exact rerank
 */
int cwq_set_timing(cwq_index* idx, int enable);
int cwq_last_timing(cwq_index* idx, float* out8);

/*
 * Isotropic-row strategy of cwq_score_topk (no reference counterpart: an execution
 * choice; results are identical either way).
 *   mode -1: automatic (default; env CWQ_FILTER=0/1 overrides): the bf16-MFMA
 *            candidate filter + exact rerank when k <= 64 and the index holds
 *            >= 16384 isotropic rows, the exact fp32 scan otherwise; an index on which
 *            >= 9 in 10 of its first >= 256 filtered queries had to be re-run exactly (the
 *            bounds too loose for its rows) stays on the exact scan from then on
 *   mode  0: always the exact fp32 scan      mode 1: the filter whenever k <= 64
 * Calls with nq <= 64 take the small-batch stream filter instead of the batch MFMA
 * filter (one HBM pass over the bf16 row panel; env CWQ_STREAM=0 disables it).
 * cwq_last_stats(out6): [queries served by the filter, of which re-run by the exact
 * scan (candidate list overflow / no threshold), filter used (0 exact scan, 1 batch
 * MFMA filter, 2 small-batch stream filter; + 256 when the stream filter's pass ran on
 * the int8 row panel), mean candidate records per query, mean
 * exact reranks per query, threshold-sample rows].
 * After cwq_categorize, cwq_last_stats reports instead: [queries, queries re-run with
 * every leaf row materialised (DENSE), queries re-run after a filter list overflow,
 * queries resolved by counting over the bottleneck order, queries resolved by the heap
 * replay, queries the two-level replay resolved after their list ended inside a
 * bottleneck tie].
 */
int cwq_set_filter(cwq_index* idx, int mode);
/*
 * cwq_score_topk with host memory on both sides: q (host [nq*dim]) in, ids (host [nq*k])
 * and scores (host [nq*k] or NULL) out; returns synchronized.  The reference harness's
 * timed call shape (benchmark_utils.py:801-805: cobweb_predict_fast on a numpy embedding,
 * CobwebWrapper.py:428-433 -> :210-265).  Same results as cwq_score_topk.
 */
int cwq_score_topk_host(cwq_index* idx, const float* q, int64_t nq, int32_t k, int64_t* ids, float* scores,
                        void* stream);
/*
 * cwq_categorize with host memory on both sides: q (host [nq*dim]) in; nodes (host
 * [nq*k]), n_found (host [nq]) and n_calls (host [nq] or NULL) out; returns synchronized.
 * The reference harness's Basic call shape (benchmark_utils.py:580-581: cobweb_predict on a
 * numpy embedding, CobwebWrapper.py:435-461 -> CobwebTorchTree.py:235-289).  Same results
 * as cwq_categorize.
 */
int cwq_categorize_host(cwq_index* idx, const float* q, int64_t nq, int32_t k, int64_t max_nodes, int64_t* nodes,
                        int32_t* n_found, int64_t* n_calls, void* stream);

int cwq_last_stats(cwq_index* idx, int64_t* out6);

/*
 * Group pruning of the Fast query (clustered trees whose rows are
 * group-centred, every level weight >= 0): per (query, depth-1 group) a certified upper
 * bound of every key in the group; the exact internal pass runs for each query's best group
 * and then only for the groups whose bound reaches the filter's first threshold.  Results
 * are unchanged (bit-identical to the exact scan); CWQ_GROUP_PRUNE=0 turns it off (at index
 * creation: never built; per call: not used).  Replaces no reference call: the reference
 * evaluates every node (CobwebWrapper.py:222-241).
 * cwq_last_prune_stats(out4): [pruning available on this index, queries of the last Fast
 * call's pruned chunk (0: not pruned), its stage-B (query, group) pairs, groups].
 */
int cwq_last_prune_stats(cwq_index* idx, int64_t* out4);

/*
 * Sequential Welford statistics of row groups (synthetic-tree builder).
 * For group g, folds rows X[order[group_ptr[g]] .. order[group_ptr[g+1]-1]] in
 * that order with exactly the fp32 op sequence of CobwebTorchNode.increment_counts
 * (CobwebTorchNode.py:57-68: count += 1; delta = x - mean; mean += delta / count;
 * meanSq += delta * (x - mean)), so a synthesised internal node carries the stats
 * the reference's ifit would accumulate for those inserts.
 *   X [n_rows*dim], order [n_order], group_ptr [n_groups+1]: device
 *   count [n_groups], mean/meanSq [n_groups*dim]: device outputs
 */
int cwq_welford_groups(const float* X, int64_t n_rows, int32_t dim, const int64_t* order, const int64_t* group_ptr,
                       int64_t n_groups, float* count, float* mean, float* meanSq, void* stream);

/*
 * Incremental fit (ifit) support: category-utility scoring on the GPU (add path,
 * CobwebTorchTree.cobweb, CobwebTorchTree.py:143-233).  Node statistics live in a
 * caller-owned device pool: count[cap], mean[cap*dim], meanSq[cap*dim] (slot = row).
 *
 * cwq_fit_kl: out[j] = compute_score(cand_j, ref_j) = KL(cand || ref)
 *   (CobwebTorchTree.py:344-364, use_info=True, use_kl=True) for jobs[4*j..4*j+3] =
 *   {cand_type, n1, n2, ref_type}:
 *     cand_type 0: node n1                    (CobwebTorchNode.mean_var, :211-212)
 *               1: node n1 with x inserted    (mean_var_insert, :214-222)
 *               2: new leaf from x            (mean_var_new, :204-209)
 *               3: merge(n1, n2) with x       (mean_var_merge, :224-239)
 *     ref_type  0: parent p_slot; 1: parent with x inserted.
 *   x, jobs, out: device.  Asynchronous on `stream`.
 */
int cwq_fit_kl(const float* count, const float* mean, const float* meanSq, int32_t dim, const float* x,
               float prior_var, int32_t p_slot, const int32_t* jobs, int32_t n_jobs, float* out, void* stream);

/*
 * cwq_fit_node_op: one node update in the pool, same fp32 op order as the reference:
 *   op 0 increment_counts(dst, x)           (CobwebTorchNode.py:57-68)
 *   op 1 update_counts_from_node(dst, src)  (:70-85; merge and the copy constructor)
 *   op 2 zero(dst)                          (a fresh node)
 *   op 3 *flag = is_exact_match(dst, x)     (:652-666, torch.isclose defaults)
 */
int cwq_fit_node_op(int32_t op, float* count, float* mean, float* meanSq, int32_t dim, int32_t dst, int32_t src,
                    const float* x, int32_t* flag, void* stream);

/*
 * Device-resident incremental fit (F1): CobwebTorchTree.cobweb's insert loop
 * (CobwebTorchTree.py:143-233; CobwebTorchNode.py:57-85, 374-666) run entirely on the
 * GPU -- the tree (statistics, parent links, ordered child lists) in device memory, one
 * master workgroup inserting the rows in order, every decision on the device, the
 * reference's random() draws from Python's MT19937 stream run on the device; a level with
 * many children (>= CWQ_FIT_FORK_MIN, default 64) has its KL terms computed by helper
 * workgroups on every CU (CWQ_FIT_HELPERS, default CUs - 1; 0 = one workgroup).  Builds the
 * same trees as the host-driven cwq_fit_kl / cwq_fit_node_op path (fit.py).  dim <= 1024.
 * Errors: CWQ_ERR_OOM only for a node pool / child arena that cannot be allocated or
 * runs out inside an insert (fit.py then continues on the host fitter); a chip-wide KL
 * pass that did not complete is CWQ_ERR_HIP (fit.py raises).
 *   cwq_fit_create   a handle with room for cap_nodes nodes
 *   cwq_fit_load     the tree in slots 0..n_nodes-1: parent (host, -1 at the root),
 *                    children in list order as CSR (host child_ptr [n+1], child_idx),
 *                    count / mean / meanSq (host, [n], [n*dim]); mt_state (host [625]) =
 *                    Python's random.getstate()[1] (624 words + index)
 *   cwq_fit_insert   X (device [n*dim]): the rows inserted in order; leaf_out (device
 *                    [n] int32) = the slot of the node each row ended in (ifit's return
 *                    value).  info (host int64[4]) = {rows done, random() draws, status,
 *                    slots in use}; status 1: the node pool / child arena needs room --
 *                    export, load into a larger handle and insert the remaining rows
 *   cwq_fit_export   out2 = {slots in use, root}; parent (-2: a node a split removed),
 *                    child CSR, count, mean, meanSq (host, [cap] / [cap*dim]) and the
 *                    random() state after the draws (host [625])
 *   cwq_mt19937_draw n draws of Python's random.random() from state625 (host; updates it)
 *   cwq_mt19937_words n 32-bit outputs (Python's getrandbits(32)) from state625 through the
 *                    chain-form twist the device's parallel generator runs (host; updates it)
 *   cwq_mt19937_skip  advance state625 past nwords 32-bit outputs without producing them
 *                    (host; updates it): the Basic query's random() advance -- one random()
 *                    = 2 words per heap push and retrieval (CobwebTorchTree.py:243,268,285),
 *                    replacing getrandbits(64 n) (CobwebWrapper.cobweb_predict, wrapper.py)
 */
typedef struct cwq_fit cwq_fit;
int cwq_fit_create(int device, int32_t dim, float prior_var, int32_t cap_nodes, cwq_fit** out);
int cwq_fit_destroy(cwq_fit* h);
int cwq_fit_load(cwq_fit* h, int32_t n_nodes, int32_t root, const int32_t* parent, const int32_t* child_ptr,
                 const int32_t* child_idx, const float* count, const float* mean, const float* meanSq,
                 const uint32_t* mt_state, void* stream);
int cwq_fit_insert(cwq_fit* h, const float* X, int64_t n, int32_t* leaf_out, int64_t* info, void* stream);
int cwq_fit_export(cwq_fit* h, int32_t* out2, int32_t* parent, int32_t* child_ptr, int32_t* child_idx, float* count,
                   float* mean, float* meanSq, uint32_t* mt_state, void* stream);
const char* cwq_fit_last_error(void);
int cwq_mt19937_draw(uint32_t* state625, int64_t n, double* out);
int cwq_mt19937_words(uint32_t* state625, int64_t n, uint32_t* out);
int cwq_mt19937_skip(uint32_t* state625, int64_t nwords);

/*
 * PCA + ICA whitening transform (F4).  Replaces PCAICAWhiteningModel.transform
 * (src/whitening/pca_ica.py:30-51), the embedding normalisation of the "PCA + ICA"
 * benchmark rows and of config C5:
 *   x_pca = ((X - mean) @ comps^T) / denom,   out = x_pca @ unmix^T   (unmix != NULL)
 *                                             out = x_pca            (unmix == NULL, is_ica=False)
 *   X      device [n*d_in] fp32          mean   device [d_in]
 *   comps  device [d_pca*d_in]           denom  device [d_pca] = sqrt(explained_var + eps),
 *                                               computed by the caller in fp32 like numpy
 *   unmix  device [d_out*d_pca] or NULL  work   device [n*d_pca] scratch (when unmix)
 *   out    device [n*d_out] (or [n*d_pca])
 * fp32 MFMA GEMMs; results equal numpy's fp32 up to the dot-product summation order.
 */
int cwq_whiten(const float* X, int64_t n, int32_t d_in, const float* mean, const float* comps, int32_t d_pca,
               const float* denom, const float* unmix, int32_t d_out, float* out, float* work, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* COBWEB_QUERY_H */
