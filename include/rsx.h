/*
 * rsx.h — flat C ABI of librsx.so, the MI355X (gfx950) graph-CF training path.
 *
 * The reference (EXLYSHA/Recommendar-Systems, an MMRec fork) is pure Python on
 * PyTorch; its hot path is a handful of torch call sites inside the models'
 * forward / calculate_loss / full_sort_predict and Trainer.evaluate.  Each entry
 * point below replaces one of those call sites (cited per function, paths relative
 * to the reference's root).  The Python host side in recommendar-systems_amd/rsx
 * binds these with ctypes; INTEGRATION.md shows the binding a maintainer adds to
 * the reference.
 *
 * Conventions (all entry points):
 *   - every array argument is a DEVICE pointer unless its name ends in `_host`;
 *   - the caller owns and allocates every buffer, including workspaces (sizes
 *     from the matching *_ws_bytes query); no entry point allocates or syncs, so
 *     every call is stream-ordered and can be captured into a hipGraph;
 *   - matrices are row-major and contiguous: an [n, d] f32 matrix has row stride d;
 *   - the return value is a hipError_t as int, or one of the RSX_ERR_* codes
 *     below for argument errors (0 = success).  The Python wrappers raise
 *     RuntimeError on a nonzero return (the reference raises Python exceptions).
 */
#ifndef RSX_H
#define RSX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rsx_stream_t; /* a hipStream_t (0 = the null stream) */

#define RSX_OK 0
#define RSX_ERR_ARG 1001         /* bad size / null pointer */
#define RSX_ERR_UNSUPPORTED 1002 /* embedding width not compiled (d in {32,64,128,256}) */
#define RSX_ERR_WORKSPACE 1003   /* workspace too small */
#define RSX_ERR_COMM 1004        /* RCCL missing or a collective failed */

/* Version string of the library ("rsx <ver> gfx950"). */
const char* rsx_version(void);

/* ------------------------------------------------------------------------ */
/* CSR adjacency with an nnz-balanced work schedule                           */
/* ------------------------------------------------------------------------ */
/*
 * Replaces the torch COO sparse adjacency the models build
 * (src/models/lightgcn.py:65-103, src/models/layergcn.py:91-117,
 *  src/models/smore.py:176-207).  Rows are split into work items of at most
 * `chunk` nonzeros so that power-law hub rows (10^3..10^6 neighbours) spread
 * over many wavefronts; a row split over several items is summed in chunk order
 * by a fixup pass, so results are deterministic.
 */
typedef struct rsx_csr {
    int64_t n_rows;
    int64_t n_cols;
    int64_t nnz;
    const int64_t* rowptr;    /* [n_rows + 1] */
    const int32_t* col;       /* [nnz] */
    const float* val;         /* [nnz] */
    int32_t chunk;            /* max nonzeros per work item */
    int32_t pad0;
    int64_t n_work;           /* work items */
    const int32_t* work;      /* [n_work][4] = {row, slot, begin, end}; slot -1: whole row, else
                                 {long-row index, slot, begin, end}; long-row chunks come first */
    int64_t n_long;           /* rows split over more than one work item */
    const int32_t* long_rows; /* [n_long][4] = {row, slot_begin, n_slots, 0} */
    int64_t n_slots;          /* partial-sum slab rows (slab = n_slots * d floats + n_long int32) */
} rsx_csr;

/*
 * Host-side schedule builder.  Pass work_host/long_host = NULL to query the
 * counts (n_work, n_long, n_slots); then call again with arrays of
 * [n_work*4] and [n_long*4] int32.  rowptr_host is the host copy of rowptr.
 * Returns RSX_ERR_ARG if nnz >= 2^31 (work items keep 32-bit offsets).
 */
int rsx_csr_schedule_host(const int64_t* rowptr_host, int64_t n_rows, int32_t chunk,
                          int32_t* work_host, int32_t* long_host,
                          int64_t* n_work, int64_t* n_long, int64_t* n_slots);

/*
 * The work schedule of a CSR built on the device, without a host round trip, for a
 * graph whose every row holds at most as many nonzeros as the same row of a template
 * CSR with a schedule (a per-epoch edge-dropout graph, reference
 * src/models/layergcn.py:51-81, against the full training graph): the template's
 * layout is kept (same n_work / n_long / n_slots / long_rows / slab), `work`
 * [tmpl->n_work][4] receives the new begin/end of every item; a long row's chunks past
 * its new end are empty (they contribute zero partials).  rowptr: device, the new
 * graph's [n_rows + 1].
 */
int rsx_csr_schedule_rebind(const rsx_csr* tmpl, const int64_t* rowptr, int32_t* work, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* SpMM with fused row epilogues                                              */
/* ------------------------------------------------------------------------ */
/*
 * Y = A * X for one propagation layer (src/models/lightgcn.py:122,
 * src/models/layergcn.py:133, src/models/smore.py:282,293,297,303,307,313,317)
 * and its autograd twin (SparseAddmmBackward; A is symmetric for the
 * user-item Laplacian so the backward is the same product), with the
 * per-row work that follows the product in the reference fused into the
 * write-out:
 *
 *   RSX_EPI_STORE     y = alpha*acc
 *   RSX_EPI_LAYERSUM  y = alpha*acc;  s_out = s_in + alpha*acc
 *                     (running layer sum of lightgcn.py:124-125 / Horner backward)
 *   RSX_EPI_FINAL     f = ((((s_in + r_add) + aux) + e0) + alpha*acc) * beta (NULL
 *                     terms skipped);  zero0/zero1 rows := 0  (last layer: mean over
 *                     K+1 layers, lightgcn.py:124-125, from a running sum in s_in or
 *                     from the stored layers E0 = s_in, E1 = r_add, E2 = aux, E3 = e0)
 *   RSX_EPI_ADAM      g = (s_in + alpha*acc) * beta + r_add;  Adam(p, m, v, g)
 *                     (last backward layer fused with torch.optim.Adam,
 *                      src/common/trainer.py:133,238)
 *   RSX_EPI_LAYERGCN  c = cos(acc, e0) (eps 1e-8, F.cosine_similarity);
 *                     y = c*acc;  s_out = s_in + c*acc (s_in may be NULL = 0);
 *                     saves acc (pre-scale) into `aux` and c into `aux_w`
 *                     (src/models/layergcn.py:133-138)
 *   RSX_EPI_AXPBY     y = alpha*acc + beta*s_in   (general accumulate)
 *   RSX_EPI_LAYERGCN_BWD  backward of the LayerGCN row scaling: with
 *                     dE = alpha*acc + r_add (grad reaching E^k), z = aux (saved
 *                     pre-scale rows), c = aux_w, e = e0, nz/ne eps-clamped norms:
 *                       y     = c*dE + <dE,z> (e/(nz ne) - c z/nz^2)      (dZ^k)
 *                       s_out = s_in + <dE,z> (z/(nz ne) - c e/ne^2)     (d ego)
 *   RSX_EPI_ADD     y = (alpha*acc + s_in + r_add) * beta  (s_in / r_add may be NULL;
 *                     y may alias s_in) — row-block sums of the sharded path
 *   Every kind also zeroes the zero0 / zero1 rows when those are non-NULL.
 *
 * Each output row is written by exactly one wavefront group; s_out may alias
 * s_in, never X.  `slab` is the workspace of the split (long) rows: n_slots * d
 * floats of partial sums followed by n_long int32 arrival counters, which must
 * be zero before the first call (allocate zero-filled; every call leaves them
 * zero again).  NULL is allowed when n_long == 0.  One launch does the whole
 * product: the long rows' chunk partials first, then one block per long row sums
 * them in chunk order, so results are deterministic.  A slab (with its
 * counters) must not be shared by two calls in flight at once.
 * d must be one of 32, 64, 128, 256.
 */
enum {
    RSX_EPI_STORE = 0,
    RSX_EPI_LAYERSUM = 1,
    RSX_EPI_FINAL = 2,
    RSX_EPI_ADAM = 3,
    RSX_EPI_LAYERGCN = 4,
    RSX_EPI_AXPBY = 5,
    RSX_EPI_LAYERGCN_BWD = 6,
    RSX_EPI_ADD = 7
};

typedef struct rsx_adam {
    float lr, beta1, beta2, eps, weight_decay;
    int32_t pad0;
    const int64_t* step_dev; /* if non-NULL the (already incremented) step count is read here */
    int64_t step;            /* otherwise this host value is used (1-based) */
} rsx_adam;

typedef struct rsx_epilogue {
    int32_t kind;
    int32_t pad0;
    float alpha;
    float beta;
    float* y;
    const float* s_in;
    float* s_out;
    float* f;
    float* zero0;
    float* zero1;
    const float* r_add;
    float* p;
    float* m;
    float* v;
    float* g_out;      /* ADAM: optional copy of the gradient row (autograd path) */
    const float* e0;   /* LAYERGCN(_BWD): ego rows */
    float* aux;        /* LAYERGCN: pre-scale rows written; LAYERGCN_BWD: read */
    float* aux_w;      /* LAYERGCN: cosine weight per row written; LAYERGCN_BWD: read */
    rsx_adam adam;
    /* Batch-row tags (optional): row r is "tagged" when row_tag[r] == tag.  The
     * tag_flags bits say which operands are known to be zero / unused off the
     * tagged rows, so their memory traffic is skipped (results are unchanged):
     *   RSX_TAG_ROWS      output rows not tagged are skipped entirely (no loads,
     *                     no stores: their outputs keep their old contents);
     *   RSX_TAG_SPARSE_X  X rows not tagged are zero: their gathers are skipped;
     *   RSX_TAG_SPARSE_S  s_in rows not tagged are zero (not loaded);
     *   RSX_TAG_SPARSE_R  r_add rows not tagged are zero (not loaded);
     *   RSX_TAG_ZERO      zero0 / zero1 are cleared on tagged rows only. */
    const int32_t* row_tag;
    int32_t tag;
    int32_t tag_flags;
    /* ADAM and ADD (optional): the regulariser gradient as occurrence counts,
     * r = (cnt[3r] k[0] + cnt[3r+1] k[1] + cnt[3r+2] k[2]) * p_old (what the fused
     * LightGCN BPR leaves instead of a dense R; p_old = the row of `p`).  Used
     * instead of r_add when non-NULL.  ADAM: with RSX_TAG_ZERO the counts of the
     * tagged rows are cleared too.  ADD: s = ((acc + s_in) + r) * beta, and every
     * row's counts are cleared (rows here are relative to reg_cnt and p). */
    int32_t* reg_cnt;
    const float* reg_k;
    /* optional: the tag is read from device memory (graph-captured steps) */
    const int32_t* tag_dev;
    /* ADAM (optional): when *halt != 0 the parameters and moments are left unchanged
     * (a NaN loss stopped training, rsx_lgcn_step.halt) */
    const int32_t* halt;
    /* RSX_TAG_SPARSE_X (optional): the tags of X's rows where they are numbered apart
     * from the output rows (a rectangular operator, e.g. R^T: items x users); NULL:
     * row_tag for both */
    const int32_t* x_tag;
} rsx_epilogue;

#define RSX_TAG_ROWS 1
#define RSX_TAG_SPARSE_X 2
#define RSX_TAG_SPARSE_S 4
#define RSX_TAG_SPARSE_R 8
#define RSX_TAG_ZERO 16

int rsx_spmm(const rsx_csr* a, const float* x, int32_t d, const rsx_epilogue* epi,
             float* slab, rsx_stream_t stream);

/* Up to 4 independent products Y_p = A_p X_p of one epilogue kind (STORE, ADD or
 * AXPBY) and one width d in a single launch (SMORE's three item views through their
 * kNN graphs, or through R: src/models/smore.py:299-317): every product's work
 * blocks, then every product's hub-row fixups.  Each product is exactly what
 * rsx_spmm(a[p], x[p], d, &epis[p], slabs[p]) computes (no product may write
 * another's inputs). */
int rsx_spmm_batch(int32_t count, const rsx_csr* const* a, const float* const* x, int32_t d,
                   const rsx_epilogue* epis, float* const* slabs, rsx_stream_t stream);

/* Row-wise epilogue with acc = 0 over rows [0, n_rows): e.g. a stand-alone Adam
 * step (kind RSX_EPI_ADAM, s_in = grad, beta = 1) — torch.optim.Adam in
 * src/common/trainer.py:133,238 — or the K = 0 forward. */
int rsx_rowwise(int64_t n_rows, int32_t d, const rsx_epilogue* epi, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* BPR triplet loss, forward + backward fused                                 */
/* ------------------------------------------------------------------------ */
/*
 * Variants:
 *   RSX_BPR_LIGHTGCN  mean -log(1e-10 + sigmoid(s+ - s-)) + reg * (|U0|_F+|P0|_F+|N0|_F)/B
 *                     on ego rows (src/models/lightgcn.py:132-156, src/common/loss.py:33-51)
 *   RSX_BPR_LAYERGCN  sum -logsigmoid(s+ - s-) + reg * 0.5*sum(ego^2)
 *                     (src/models/layergcn.py:142-177, src/common/loss.py:58-61)
 *   RSX_BPR_SMORE     mean -logsigmoid(s+ - s-) + reg * 0.5*(|u|^2+|p|^2+|n|^2)/batch_cfg
 *                     on propagated rows (src/models/smore.py:366-378)
 * Row layout: final/ego are [n_users + n_items, d] (users first, as torch.cat in
 * the reference); triplets are int64 [3][B] = (user, pos item, neg item) with item
 * ids local to the item block (reference TrainDataLoader, dataloader.py:226-250).
 * Outputs: g_final (+= dL/dfinal, rows touched only), g_ego (+= dL/dego; may be
 * NULL for SMORE), loss_out[0] = loss (f32); if loss_acc != NULL, loss is also
 * added into loss_acc[0] (f64, per-epoch accumulator without a host sync).
 * Workspace: rsx_bpr_ws_bytes(B).
 * RSX_BPR_SMORE_ROWS: RSX_BPR_SMORE on compact batch rows — n_users = B, n_items = 2 B and
 * triplets (b, b, B + b), so every row of the [3 B, d] g_final is one triplet's: written
 * (=), not added, and g_final needs no zero fill. Triplets of any other layout make the
 * loss NaN (checked on the device, so the NaN halt stops the step; rsx/ops.py only lets
 * rsx.smore_fuse's compact-rows loss, which builds the triplets itself, request it).
 */
enum { RSX_BPR_LIGHTGCN = 0, RSX_BPR_LAYERGCN = 1, RSX_BPR_SMORE = 2, RSX_BPR_SMORE_ROWS = 3 };

size_t rsx_bpr_ws_bytes(int64_t batch);
int rsx_bpr(int32_t variant, const float* final_emb, const float* ego_emb, int64_t n_users,
            int64_t n_items, int32_t d, const int64_t* triplets, int64_t batch, float reg,
            float batch_cfg, float* g_final, float* g_ego, float* loss_out, double* loss_acc,
            void* ws, size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Full-sort scoring fused with train-item masking and top-K                  */
/* ------------------------------------------------------------------------ */
/*
 * Replaces  scores = u_emb[users] @ item_emb^T            (lightgcn.py:164 etc.)
 *           scores[mask] = -1e10; topk(scores, k)          (src/common/trainer.py:521-526)
 * without materialising the score matrix.  k <= 64 (default): bf16 MFMA tiles
 * bound every score within eps |u| |v_i| (eps < 2^-7 + 2^-16 + 2 d 2^-23); a first
 * pass bounds the user's k-th score from below, a second computes exact f32 scores
 * (an fmaf chain over d in order: rsx_score_dense's bits) only for items whose upper
 * bound reaches it; k 65..96 (or env RSX_FS_SCREEN=0): exact f32 MFMA tiles with a
 * running threshold.  Per-user candidate rows in the workspace; a merge pass orders
 * the result by (score desc, item index asc).  Masked (user, item) pairs — the user's
 * training items, CSR mask_rowptr/mask_col over user ids with sorted columns —
 * score exactly -1e10 as in the reference.
 *   user_emb: [*, d] rows selected by users[b] (int64); item_emb: [n_items, d]
 *   out_val: [n_batch, k] f32, out_idx: [n_batch, k] int64
 * Requires k <= n_items and k <= 96. Workspace: rsx_fullsort_ws_bytes.
 */
size_t rsx_fullsort_ws_bytes(int64_t n_batch, int64_t n_items, int32_t k);
/* The item-chunk plan rsx_fullsort_topk uses for (n_batch, n_items, d): chunks per
 * 32-user wave and items per chunk (tests assert which selection path they cover). */
int rsx_fullsort_plan(int64_t n_batch, int64_t n_items, int32_t d, int32_t* n_chunks, int64_t* chunk_items);
int rsx_fullsort_topk(const float* user_emb, const int64_t* users, int64_t n_batch,
                      const float* item_emb, int64_t n_items, int32_t d,
                      const int64_t* mask_rowptr, const int32_t* mask_col, int32_t k,
                      float* out_val, int64_t* out_idx, void* ws, size_t ws_bytes,
                      rsx_stream_t stream);

/* Dense scores (full_sort_predict) for the API path: out[b, i] = <u[users[b]], item[i]>. */
int rsx_score_dense(const float* user_emb, const int64_t* users, int64_t n_batch,
                    const float* item_emb, int64_t n_items, int32_t d, float* out,
                    rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Training-triplet sampler (throughput mode)                                 */
/* ------------------------------------------------------------------------ */
/*
 * Device replacement of TrainDataLoader's per-epoch shuffle + rejection
 * negative sampling (src/utils/dataloader.py:226-275,307-309,
 * src/utils/dataset.py:98-101): batch slot t of batch `start/B` takes training
 * interaction perm(start + t) (a keyed Feistel bijection of [0, n_inter) per
 * (seed, epoch)) and a negative item drawn uniformly from all_items, redrawn
 * while it is in the user's training history (CSR hist_rowptr/hist_col, columns
 * sorted).  Writes int64 [3][count] triplets (count = min(B, n_inter - start)).
 */
int rsx_sample_triplets(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter,
                        const int64_t* hist_rowptr, const int32_t* hist_col,
                        const int32_t* all_items, int64_t n_all_items, uint64_t seed,
                        int64_t epoch, int64_t start, int64_t batch, int64_t* out,
                        rsx_stream_t stream);

/* The whole epoch at once (one launch per epoch): all n_inter triplets of
 * `epoch`, batch-major — batch j (size Bj = min(batch, n_inter - j*batch)) is
 * [3][Bj] contiguous at out + 3*batch*j, identical to what rsx_sample_triplets
 * returns for start = j*batch.  out holds 3*n_inter int64. */
int rsx_sample_epoch(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter,
                     const int64_t* hist_rowptr, const int32_t* hist_col, const int32_t* all_items,
                     int64_t n_all_items, uint64_t seed, int64_t epoch, int64_t batch, int64_t* out,
                     rsx_stream_t stream);

/* The same epoch stream cut into n_slices balanced slices instead of fixed batches:
 * slice j = epoch positions [floor(j n_inter / S), floor((j+1) n_inter / S)) (sizes
 * differ by at most one; 1 <= S <= n_inter), stored [3][Bj] contiguous at
 * out + 3*floor(j n_inter / S).  The sharded trainers' epochs: every rank runs the
 * same step count S and visits each of its interactions once (replaces the reference
 * DataLoader's per-epoch batch walk, src/utils/dataloader.py:226-258). */
int rsx_sample_epoch_slices(const int32_t* inter_u, const int32_t* inter_i, int64_t n_inter,
                            const int64_t* hist_rowptr, const int32_t* hist_col, const int32_t* all_items,
                            int64_t n_all_items, uint64_t seed, int64_t epoch, int64_t n_slices, int64_t* out,
                            rsx_stream_t stream);

/* Gather rows: out[b] = src[idx[b] + offset]  (u_embeddings = user_all[user] etc.). */
int rsx_gather_rows(const float* src, const int64_t* idx, int64_t n, int64_t offset, int32_t d,
                    float* out, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Fused LightGCN training step                                               */
/* ------------------------------------------------------------------------ */
/*
 * One LightGCN batch end to end (src/models/lightgcn.py:117-156 forward + loss,
 * autograd backward, src/common/trainer.py:238 Adam step), as 2K+2 launches:
 *   K propagation layers (last fused with the layer mean and zeroing of the
 *   gradient buffers), BPR fwd+bwd, K backward layers (last fused with Adam).
 * If `sample` != NULL the triplets are drawn on device first (same contract as
 * rsx_sample_triplets; `triplets` then receives them), otherwise `triplets`
 * holds the batch.  Buffers are [n_rows, d] f32 unless noted:
 *   p (parameters = ego embeddings, users then items), m, v (Adam moments),
 *   s, h0, h1 (scratch), final_emb (mean of layers), g, r (gradient scratch;
 *   the forward's last layer zeroes them before the loss scatters into them).
 *   s may be NULL for n_layers == 1, s/h0/h1 may be NULL for n_layers == 0.
 */
typedef struct rsx_sampler_args {
    const int32_t* inter_u;
    const int32_t* inter_i;
    int64_t n_inter;
    const int64_t* hist_rowptr;
    const int32_t* hist_col;
    const int32_t* all_items;
    int64_t n_all_items;
    uint64_t seed;
    int64_t epoch;
    int64_t start;
} rsx_sampler_args;

typedef struct rsx_lgcn_step {
    const rsx_csr* adj;
    int64_t n_users, n_items;
    int32_t d, n_layers;
    float reg;
    int32_t pad0;
    float* p; float* m; float* v;
    float* s; float* h0; float* h1;
    float* final_emb; float* g; float* r;
    float* slab;
    int64_t* triplets;  /* [3][batch] */
    int64_t batch;
    const rsx_sampler_args* sample;
    rsx_adam adam;
    float* loss_out;    /* [1] */
    double* loss_acc;   /* [1] or NULL */
    void* ws; size_t ws_bytes; /* >= rsx_bpr_ws_bytes(batch) */
    /* Optional [n_users + n_items] int32 scratch, zero-filled before the first step
     * (K >= 2 only; NULL = dense path).  Each step tags its batch rows with a fresh
     * value (`tag`, > 0 and different from every earlier step's, e.g. the step
     * count) and uses the tags to skip the work a batch does not need: the last
     * forward layer computes the batch rows only (only they reach the loss), the
     * first backward layer skips gathers of the all-zero rows of G = dL/dfinal, and
     * the gradient scratch G, R is cleared on the batch rows after Adam instead of
     * densely before the loss.  With tags, G and R must be zero between steps
     * (true from zero-filled buffers and after every tagged step). */
    int32_t* row_tag;
    int64_t tag;
    /* Optional with row_tag: [3 (n_users + n_items) + 4] int32, zero-filled before the
     * first step.  BPR then runs as ONE launch and leaves the regulariser gradient as
     * per-row occurrence counts (+ a done counter and three scales in the tail) that
     * the Adam layer applies and clears; R is not used. */
    int32_t* reg_cnt;
    /* Optional (any path: tagged or dense, any K): [2] int32, zero-filled.  The first step whose loss is NaN
     * sets halt[0] = 1 and halt[1] = its tag; from then on the Adam layer leaves the
     * parameters and moments unchanged, so they stay those of the last finite step (the
     * reference checks the loss before backward and stops, src/common/trainer.py:201-203). */
    int32_t* halt;
} rsx_lgcn_step;

int rsx_lightgcn_step(const rsx_lgcn_step* st, rsx_stream_t stream);

/*
 * One LayerGCN training batch (reference src/models/layergcn.py:127-177 with the
 * autograd backward and src/common/trainer.py:238 Adam) as ONE call: K layers
 * E^k = c_k * (A E^{k-1}) with c_k = cos(A E^{k-1}, E^0) (RSX_EPI_LAYERGCN, out =
 * sum_k E^k; the pre-scale rows and c_k saved in zs[k-1] / cs[k-1]), BPR-sum + L2
 * (RSX_BPR_LAYERGCN: g = d/d out, r = d reg / d E^0), the cosine-gate backward
 * (RSX_EPI_LAYERGCN_BWD, rowwise for layer K, fused into the SpMMs of layers K-1..1),
 * the last product fused with Adam.  `adj` is the epoch's (edge-dropout) training
 * graph; g, r are zeroed by the last forward layer.  Same kernels and order as the
 * Python-issued sequence, one host call instead of 2K + 3.
 */
typedef struct rsx_layergcn_step_args {
    const rsx_csr* adj;
    int64_t n_users, n_items;
    int32_t d, n_layers;
    float reg;
    int32_t pad0;
    float* p; float* m; float* v;
    float* out; float* g; float* r; float* acc;
    float* h0; float* h1;
    float* const* zs;   /* [n_layers] -> [N, d] */
    float* const* cs;   /* [n_layers] -> [N] */
    float* slab;
    const int64_t* triplets;  /* [3][batch] */
    int64_t batch;
    rsx_adam adam;
    float* loss_out;    /* [1] or NULL */
    double* loss_acc;   /* [1] or NULL */
    void* ws; size_t ws_bytes;  /* >= rsx_bpr_ws_bytes(batch) */
} rsx_layergcn_step_args;

int rsx_layergcn_step(const rsx_layergcn_step_args* st, rsx_stream_t stream);

/* Forward only (evaluation): final_emb = mean_k A^k p, using s, h0, h1 as scratch. */
int rsx_lightgcn_forward(const rsx_csr* adj, int32_t d, int32_t n_layers, const float* p,
                         float* s, float* h0, float* h1, float* final_emb, float* slab,
                         rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* SMORE: fused modality projection + spectral denoise / fusion               */
/* ------------------------------------------------------------------------ */
/*
 * Replaces image_trs / text_trs and spectrum_convolution
 * (src/models/smore.py:256-259 and :209-237), two launches on fp32 MFMA:
 *   img = V Wv^T + bv   (V [n_items, dv], Wv [d, dv], nn.Linear layout)
 *   txt = T Wt^T + bt   (T [n_items, dt], Wt [d, dt])
 *   Fi = rfft(img, norm='ortho'), Ft = rfft(txt)       (d/2+1 bins)
 *   conv_v = irfft(Fi * wv), conv_t = irfft(Ft * wt), conv_f = irfft(Ft * Fi * wf)
 * wv / wt / wf are the [(d/2+1)][2] complex weights AFTER the reference's unit
 * normalisation w / (|w| + 1e-8) (:221-229; the caller applies it, so autograd
 * of that step stays with the caller).  img and txt are written out; `spec`
 * [rsx_smore_spectral_spec_floats(n, d)] receives Fi and Ft in an internal
 * layout for the backward; `ws` [rsx_smore_spectral_fwd_ws_bytes(...)] holds
 * the split-K partial projections.  d in {64, 128}; dv, dt multiples of 4.
 */
size_t rsx_smore_spectral_spec_floats(int64_t n_items, int32_t d);
size_t rsx_smore_spectral_fwd_ws_bytes(int64_t n_items, int32_t d, int32_t dv, int32_t dt);
int rsx_smore_spectral_fwd(const float* V, int32_t dv, const float* Wv, const float* bv,
                           const float* T, int32_t dt, const float* Wt, const float* bt,
                           const float* wv, const float* wt, const float* wf,
                           int64_t n_items, int32_t d, float* img, float* txt,
                           float* conv_v, float* conv_t, float* conv_f, float* spec,
                           void* ws, size_t ws_bytes, rsx_stream_t stream);

/*
 * The whole SMORE item side of smore.py:256-272 (image_trs / text_trs,
 * spectrum_convolution and, with `item` set, the modality gates
 *   img_i = item + scale * sigmoid(gate_v(conv_v))   (mul: item * sigmoid(..)),
 * likewise txt_i / fus_i with gate_t / gate_f) as ONE launch: every block projects
 * its share and the last block to finish an item tile runs the spectral part and
 * the gates of that tile.  Same arguments and outputs as rsx_smore_spectral_fwd
 * (bit-identical values), plus `tile_cnt` [rsx_smore_item_tiles(n)] uint32
 * arrival counters (zero before the first call; the kernel re-arms them, so one
 * buffer serves every later call on the same stream) and the gate arguments:
 * gate_W[3] [d, d] nn.Linear weights, gate_b[3] [d], gate_out[3] [n_items, d]
 * (all ignored when item == NULL).  Gate outputs equal rsx_smore_gates(0, ...)'s.
 */
size_t rsx_smore_item_tiles(int64_t n_items);
int rsx_smore_item_fwd(const float* V, int32_t dv, const float* Wv, const float* bv,
                       const float* T, int32_t dt, const float* Wt, const float* bt,
                       const float* wv, const float* wt, const float* wf,
                       int64_t n_items, int32_t d, float* img, float* txt,
                       float* conv_v, float* conv_t, float* conv_f, float* spec,
                       void* ws, size_t ws_bytes, uint32_t* tile_cnt,
                       const float* item, const float* const* gate_W, const float* const* gate_b,
                       float scale, int32_t mul, float* const* gate_out, rsx_stream_t stream);

/*
 * Backward of the spectral part: given the forward's `spec` and d conv_v /
 * d conv_t / d conv_f (each may be NULL = zero), writes d img, d txt
 * [n_items, d] and per-block partial sums of d wv / d wt / d wf into
 * g_w_partial [rsx_smore_spectral_bwd_partials(n, d)] floats laid out
 * [ceil(n/64)][3][d/2+1][2] (sum over the first axis for the weight gradients).
 * The projection gradients d Wv = d img^T V, d V = d img Wv, d bv = colsum(d img)
 * (and the text twins) are left to the caller: rsx_linear_bwd, one pass each.
 * `ws` [rsx_smore_spectral_bwd_ws_bytes(n, d)] carries d Fi / d Ft between the two
 * passes (frequency side, then feature side).
 */
size_t rsx_smore_spectral_bwd_partials(int64_t n_items, int32_t d);
size_t rsx_smore_spectral_bwd_ws_bytes(int64_t n_items, int32_t d);
int rsx_smore_spectral_bwd(const float* spec, const float* wv, const float* wt, const float* wf,
                           const float* g_v, const float* g_t, const float* g_f,
                           int64_t n_items, int32_t d, float* g_img, float* g_txt,
                           float* g_w_partial, void* ws, size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Evaluation tail: top-K ranking metrics                                     */
/* ------------------------------------------------------------------------ */
/*
 * Replaces TopKEvaluator.evaluate's hit matrix (the per-(user, rank) Python
 * `i in m` loop, src/utils/topk_evaluator.py:90-101) and utils/metrics.py
 * (:12-118) for recall / recall2 / precision / ndcg / map.
 *   topk_idx    [n_users][k_max] int64: ranked items per evaluation user
 *   eval_rowptr [n_users+1] int64, eval_col int32: each user's held-out items,
 *               SORTED within the user (binary-searched)
 *   cutoffs     [n_cut] int32, ascending, each in [1, k_max]
 *   gain        [k_max] float64: 1/log2(r+1), r = 1..k_max (the caller computes it
 *               as the reference does, so results match bit for bit)
 *   out_sums    [5][n_cut] float64: over users, summed sequentially in user order
 *               (numpy's mean(axis=0) order) of recall, precision, ndcg, map, and
 *               the hit count (recall2's numerator).  Divide the first four by
 *               n_users for the reference's means; recall2 = hits / sum(|pos|).
 *   ws          >= rsx_topk_metrics_ws_bytes(n_users, n_cut) bytes.
 */
size_t rsx_topk_metrics_ws_bytes(int64_t n_users, int32_t n_cut);
int rsx_topk_metrics(const int64_t* topk_idx, int64_t n_users, int32_t k_max,
                     const int64_t* eval_rowptr, const int32_t* eval_col,
                     const int32_t* cutoffs, int32_t n_cut, const double* gain,
                     double* out_sums, void* ws, size_t ws_bytes, rsx_stream_t stream);
/*
 * Same arguments and outputs, but each column summed in a fixed parallel order
 * (nblk = min(1024, max(1, ceil(n_users/256))) blocks of 256 threads with
 * grid-strided users, a 64-lane butterfly and 4 wave sums per block; then per
 * column one wave over the nblk block sums and a butterfly): deterministic, and
 * within (gamma_h + gamma_{n_users-1}) * sum of the sequential sums, h =
 * ceil(n_users/(256*nblk)) + 16 + ceil(nblk/64), gamma_j = j*2^-53/(1-j*2^-53)
 * (every value is >= 0).  The evaluator rounds the means to 4 decimals from these
 * and falls back to rsx_topk_metrics only when a mean lies within that bound of a
 * rounding boundary, so the metric dict is the same as from the sequential sums.
 */
int rsx_topk_metrics_fast(const int64_t* topk_idx, int64_t n_users, int32_t k_max,
                          const int64_t* eval_rowptr, const int32_t* eval_col,
                          const int32_t* cutoffs, int32_t n_cut, const double* gain,
                          double* out_sums, void* ws, size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Weight gradient of a small Linear over many rows                           */
/* ------------------------------------------------------------------------ */
/*
 * dW = g^T x for nn.Linear(in_dim, out_dim) applied to n rows (g [n, out_dim],
 * x [n, in_dim], dW [out_dim, in_dim], row-major): the AddmmBackward weight
 * gradient of SMORE's gate / query / preference layers
 * (src/models/smore.py:106-120, applied to all users+items).  The rows are split
 * over blocks, partials are summed in block order (deterministic).
 * out_dim a multiple of 32, in_dim a multiple of 4 (a ragged last 32-column tile is
 * masked).
 */
/*
 * The whole backward of a Linear applied to many rows in one pass over them
 * (the SMORE modality projections image_trs / text_trs, src/models/smore.py:256-259):
 * dw = g^T x [out, in], dx = g W [n, in] (W [out, in], nn.Linear layout) and, when db
 * is non-NULL, db = colsum(g) [out].  out_dim in {32, 64, 128}, in_dim a multiple
 * of 4 (e.g. the golden fixture's 48 / 24-wide features; a ragged last 32-column tile
 * is masked).  Deterministic (split-K partials added in a fixed order).
 */
size_t rsx_linear_bwd_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim);
int rsx_linear_bwd(const float* g, const float* x, const float* W, int64_t n, int32_t out_dim, int32_t in_dim,
                   float* dw, float* dx, float* db, void* ws, size_t ws_bytes, rsx_stream_t stream);
/*
 * rsx_linear_bwd of two Linears over the same n rows and out_dim in one launch pair (the
 * image_trs / text_trs backward of src/models/smore.py:256-259): problem 0 (g0, x0 [n, in0],
 * W0) and problem 1 (g1, x1 [n, in1], W1), each result as rsx_linear_bwd defines it
 * (deterministic).  RSX_ERR_UNSUPPORTED when the two shapes need different kernel tilings
 * (the caller then issues two rsx_linear_bwd).
 */
size_t rsx_linear_bwd_pair_ws_bytes(int64_t n, int32_t out_dim, int32_t in0, int32_t in1);
int rsx_linear_bwd_pair(const float* g0, const float* x0, const float* W0, int32_t in0, float* dw0, float* dx0,
                        float* db0, const float* g1, const float* x1, const float* W1, int32_t in1, float* dw1,
                        float* dx1, float* db1, int64_t n, int32_t out_dim, void* ws, size_t ws_bytes,
                        rsx_stream_t stream);
size_t rsx_linear_wgrad_ws_bytes(int64_t n, int32_t out_dim, int32_t in_dim);
int rsx_linear_wgrad(const float* g, const float* x, int64_t n, int32_t out_dim, int32_t in_dim, float* dw,
                     void* ws, size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* SMORE per-row blocks, InfoNCE and the multi-tensor Adam (smore_fuse.hip)   */
/* ------------------------------------------------------------------------ */
/*
 * Modality gates (reference src/models/smore.py:262-272):
 *   forward  (backward = 0): out[m] = item + scale * sigmoid(conv[m] W[m]^T + b[m])
 *            (mul = 1: item * sigmoid(..)), m = v, t, f; rows [n, d], W [d, d].
 *   backward (backward = 1): given gout[m] (NULL = zero) writes g_item, g_conv[m]
 *            and dz[m] = d pre-activation (rows of the gate Linear's weight gradient,
 *            dW = dz^T conv: rsx_smore_wgrad).
 * d in {64, 128}.  Replaces gate_v/gate_t/gate_f + the inject step, forward and
 * autograd backward.
 */
int rsx_smore_gates(int32_t backward, const float* const* conv, const float* item, const float* const* W,
                    const float* const* b, int64_t n, int32_t d, float scale, int32_t mul, float* const* out,
                    const float* const* gout, float* g_item, float* const* g_conv, float* const* dz,
                    rsx_stream_t stream);
/*
 * rsx_smore_gates keeping the sigmoid rows (same reference site): with `saved`
 * ([3][n][d]) the forward also writes each gate's sigmoid(Linear(conv)) rows, and the
 * residual-mode backward reads them instead of recomputing the product (one matrix
 * product a row instead of two).  The mul-mode backward ignores it.  saved = NULL is
 * rsx_smore_gates.
 */
int rsx_smore_gates_saved(int32_t backward, const float* const* conv, const float* item, const float* const* W,
                          const float* const* b, int64_t n, int32_t d, float scale, int32_t mul, float* const* out,
                          const float* const* gout, float* g_item, float* const* g_conv, float* const* dz,
                          float* saved, rsx_stream_t stream);
/*
 * Preference block (reference src/models/smore.py:320-341), over every user+item row:
 *   W[7] / b[7]: query_v.0, query_v.2 (no bias), query_t.0, query_t.2 (no bias),
 *   gate_image_prefer.0, gate_text_prefer.0, gate_fusion_prefer.0.
 *   forward: side = mean(ip * softmax(qv(F)) * I, tp * softmax(qt(F)) * T, fp * F),
 *            all = content + side; ip/tp/fp = dropout(sigmoid(Linear(content)), p_drop)
 *            with the mask a hash of (*seed_dev, gate, row, feature) (p_drop = 0: off).
 *   backward: from g_all (and g_side, may be NULL) writes g_content, g_image,
 *            g_text, g_fusion, the recomputed tanh rows hv / ht and dz[7] (each
 *            Linear's pre-activation gradient; wgrad inputs: F, hv, F, ht, content x3).
 */
int rsx_smore_pref(int32_t backward, const float* const* W, const float* const* b, const float* content,
                   const float* image_emb, const float* text_emb, const float* fusion_emb, int64_t n, int32_t d,
                   float p_drop, const int64_t* seed_dev, float* all_out, float* side_out, const float* g_all,
                   const float* g_side, float* g_content, float* g_image, float* g_text, float* g_fusion,
                   float* hv, float* ht, float* const* dz, rsx_stream_t stream);
/*
 * The same block on the batch rows only (the training forward: only the rows of the
 * batch's users, positives and negatives reach the BPR and InfoNCE terms, and the
 * block is row-local).  Logical row r < n is table row rows[r] (rows may repeat):
 *   forward: all_out / side_out [n, d] compact; content_out / fusion_out (optional)
 *            receive the gathered content / fusion rows (the InfoNCE content rows and
 *            a weight-gradient input); the dropout key is the table row.  With the
 *            scratch hv ([n, d], optional) the three views' chains run as three block
 *            rows and a combine pass adds them (the same arithmetic, shorter chains).
 *   backward: g_all / g_side / g_content_in (gradient of content_out, optional) are
 *            compact; g_content / g_image / g_text / g_fusion are full [N, d] tables
 *            the row gradients are ADDED into (zero them first); hv / ht / dz compact.
 *            With `occ` ([rsx_smore_pref_rows_occ_floats(n, d)] scratch, backward only)
 *            no float atomics: the row gradients are written per occurrence and each
 *            table row of `rows` is SET to their sum in a fixed order (deterministic run
 *            to run); the other rows are untouched (zero them first).
 */
/*
 * Batch-row tags (the SMORE loss rows, src/models/smore.py:366-411): row_tag[rows[j]] =
 * *tag_dev for j < n (stream-ordered, graph-capturable; the caller bumps *tag_dev first).
 * A product with row_tag / tag_dev then treats exactly these rows as tagged.
 */
int rsx_tag_rows(int32_t* row_tag, const int64_t* rows, int64_t n, const int32_t* tag_dev, rsx_stream_t stream);
/*
 * rsx_tag_rows with the bump in the same launch: tag2 = {tag, ticket} (int32 [2], zero
 * before the first call); row_tag[rows[j]] = tag2[0] + 1, then tag2[0] holds the new tag
 * (the caller does not bump).  Products then take tag_dev = tag2.
 */
int rsx_tag_rows_next(int32_t* row_tag, const int64_t* rows, int64_t n, int32_t* tag2, rsx_stream_t stream);

int rsx_smore_pref_rows(int32_t backward, const float* const* W, const float* const* b, const float* content,
                        const float* image_emb, const float* text_emb, const float* fusion_emb, const int64_t* rows,
                        int64_t n, int32_t d, float p_drop, const int64_t* seed_dev, float* all_out,
                        float* side_out, float* content_out, float* fusion_out, const float* g_all,
                        const float* g_side, const float* g_content_in, float* g_content, float* g_image,
                        float* g_text, float* g_fusion, float* hv, float* ht, float* const* dz, float* occ,
                        rsx_stream_t stream);
size_t rsx_smore_pref_rows_occ_floats(int64_t n, int32_t d);
/*
 * rsx_smore_pref_rows with the forward's activations kept (same reference site,
 * src/models/smore.py:320-341, and its autograd backward): `saved`
 * ([rsx_smore_pref_rows_saved_floats(n, d)], compact rows) is written by the split batch-row
 * forward (scratch hv required) -- the fusion gate's sigmoid, then per view the query
 * MLP's tanh row, its softmax row and the preference gate's sigmoid, slots
 * [fusion, h_img, s_img, p_img, h_txt, s_txt, p_txt] -- and read by the backward, which then
 * recomputes no forward product (7 matrix products instead of 20); hv / ht may be NULL
 * there (the weight gradients read the saved tanh rows, slots 1 and 4).  saved = plan =
 * lead = NULL is rsx_smore_pref_rows.
 */
int rsx_smore_pref_rows_saved(int32_t backward, const float* const* W, const float* const* b, const float* content,
                              const float* image_emb, const float* text_emb, const float* fusion_emb,
                              const int64_t* rows, int64_t n, int32_t d, float p_drop, const int64_t* seed_dev,
                              float* all_out, float* side_out, float* content_out, float* fusion_out,
                              const float* g_all, const float* g_side, const float* g_content_in, float* g_content,
                              float* g_image, float* g_text, float* g_fusion, float* hv, float* ht, float* const* dz,
                              float* occ, float* saved, int32_t* plan, uint64_t* lead, rsx_stream_t stream);
size_t rsx_smore_pref_rows_saved_floats(int64_t n, int32_t d);
/*
 * The occurrence plan of rsx_smore_pref_rows_saved (optional, `plan` int32
 * [rsx_smore_pref_plan_words(n)]): the split forward lists, for each table row of `rows`,
 * its occurrences under its first one (no scan of the row ids); the backward's per-row
 * sums read the lists instead of scanning (same order, same result).  The forward needs
 * `lead`, u64 [1 + table rows] scratch, zero before its first use and then owned by the
 * caller's stream (word 0 counts the calls; keys are tagged with it, so no clearing).
 */
size_t rsx_smore_pref_plan_words(int64_t n);
/*
 * Data-parallel SMORE's batch-row gradient exchange (csrc/rowx.hip; the objective is the
 * sum over ranks of src/models/smore.py:366-411's loss of each rank's batch, and every
 * path from that loss to the parameters runs through the preference block's backward,
 * smore.py:320-341, whose table gradients are defined on the batch rows only).
 *   rsx_rowx_pack: bumps *tag_dev, then packs this rank's n occurrences (rows may
 *     repeat) into packed[n_max][rsx_rowx_entry_floats(T, d)]: per entry the row (int64 in
 *     two f32 words), a flag 1.0 on the first occurrence of its row, a pad word, then
 *     the row of each of the T [N, d] tables; entries n..n_max-1 pad (row = rows[0],
 *     flag 0).  lead: uint64 [N] scratch, zeroed once and kept across calls.
 *   rsx_rowx_combine: packed = the world ranks' packs in rank order (after an
 *     all-gather); zeroes every packed row of the T tables, writes the rows to
 *     union_rows[world * n_max], then adds each rank's flagged rows in rank order: every
 *     rank that runs it on the same packs gets bit-identical tables.
 * T <= 8, d a multiple of 4.
 */
size_t rsx_rowx_entry_floats(int32_t n_tables, int32_t d);
int rsx_rowx_pack(const int64_t* rows, int64_t n, int64_t n_max, const float* const* tables, int32_t n_tables,
                  int32_t d, uint64_t* lead, int32_t* tag_dev, float* packed, rsx_stream_t stream);
int rsx_rowx_combine(const float* packed, int32_t world, int64_t n_max, float* const* tables, int32_t n_tables,
                     int32_t d, int64_t* union_rows, rsx_stream_t stream);
/*
 * dW[p] = dz[p]^T x[p] ([d, d]) and db[p] = colsum(dz[p]) (db[p] may be NULL) for up to
 * 8 pairs of [n, d] row sets: row-split partials + one ordered reduction.
 */
size_t rsx_smore_wgrad_ws_bytes(int64_t n, int32_t d, int32_t n_pairs);
int rsx_smore_wgrad(int32_t n_pairs, const float* const* dz, const float* const* x, float* const* dw,
                    float* const* db, int64_t n, int32_t d, void* ws, size_t ws_bytes, rsx_stream_t stream);
/*
 * SMORE's two InfoNCE terms (reference src/models/smore.py:380-387, called at :398-404):
 *   loss_out[0] = InfoNCE(side[n_users + pos], content[n_users + pos], tau)   (cl_items)
 *   loss_out[1] = InfoNCE(side[users], content[users], tau)                   (cl_users)
 * InfoNCE(a, b) = mean_i -log(exp(<a_i, b_i>/tau) / sum_j exp(<a_i, b_j>/tau)) on
 * F.normalize'd rows.  The workspace [rsx_smore_infonce_ws_bytes] written by the
 * forward (normalised rows, norms, row sums and, for batch <= 4096, the two terms'
 * [batch x batch] exp(S / tau) tiles: the backward reads them instead of recomputing
 * the similarity products) is read by the backward, which ADDS
 * g_loss[0] * d cl_items + g_loss[1] * d cl_users into g_side / g_content [N, d].
 */
size_t rsx_smore_infonce_ws_bytes(int64_t batch, int32_t d);
int rsx_smore_infonce_fwd(const float* side, const float* content, const int64_t* users, const int64_t* pos_items,
                          int64_t n_users, int64_t batch, int32_t d, float tau, float* loss_out, void* ws,
                          size_t ws_bytes, rsx_stream_t stream);
int rsx_smore_infonce_bwd(const float* side, const float* content, const int64_t* users, const int64_t* pos_items,
                          int64_t n_users, int64_t batch, int32_t d, float tau, const float* g_loss, float* g_side,
                          float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream);
/* The same forward, also writing the model's loss total_out[0] = add_loss[0] + cl *
 * (cl_items + cl_users) in f32 (the reference's bpr + cl_loss * (cl_items + cl_users),
 * src/models/smore.py:411; add_loss = the BPR part); and the backward with the two
 * upstream gradients read as g_loss[term * g_stride] * g_scale (g_stride 0: one
 * gradient, the total's, for both terms, g_scale = cl). */
int rsx_smore_infonce_fwd_total(const float* side, const float* content, const int64_t* users,
                                const int64_t* pos_items, int64_t n_users, int64_t batch, int32_t d, float tau,
                                float* loss_out, const float* add_loss, float cl, float* total_out, void* ws,
                                size_t ws_bytes, rsx_stream_t stream);
int rsx_smore_infonce_bwd_scaled(const float* side, const float* content, const int64_t* users,
                                 const int64_t* pos_items, int64_t n_users, int64_t batch, int32_t d, float tau,
                                 const float* g_loss, int32_t g_stride, float g_scale, float* g_side,
                                 float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream);
/* The backward of the training loss on the compact batch rows ([users; positives;
 * negatives], 3 batch rows of d; reference src/models/smore.py:366-411): users = positives
 * = ar = arange(batch), n_users = batch, as rsx_smore_infonce_fwd_total ran them (same ws).
 * Writes (does not add) g_side / g_content [3 batch, d]: the InfoNCE rows of the users and
 * positives (each written once), zeros on the negatives' rows; g_all [3 batch, d] =
 * g_bpr * g_total[0] (the BPR rows' gradient, from rsx_bpr, times the total's upstream
 * gradient); the InfoNCE part is scaled by g_total[0] * cl.  One launch. */
int rsx_smore_loss_rows_bwd(const float* side_c, const float* content_c, const int64_t* ar, int64_t batch, int32_t d,
                            float tau, const float* g_total, float cl, const float* g_bpr, float* g_all,
                            float* g_side, float* g_content, void* ws, size_t ws_bytes, rsx_stream_t stream);
/*
 * Model-level mirror gradient (reference src/common/trainer.py:285-336) over `count`
 * (param, grad) pairs of n[i] floats:
 *   rsx_mg_alpha: alpha_out (device f64) = min(max(base, rel_step * rms(p) /
 *     (lr * rms(g) + 1e-12)), base * max_scale), rms over all pairs together (sums of
 *     squares in f64, per-block partials reduced in order: deterministic);
 *   rsx_axpy_multi: y[i] += float(*alpha_dev * mult) * x[i] (the mirror step with
 *     mult = -lr, its restore with mult = +lr), one launch per 32 tensors.
 * lr_dev (optional, device f64): the learning rate is read there instead (lr is
 * ignored; axpy uses mult * *lr_dev), so a captured step stays valid when the
 * LambdaLR schedule changes lr between epochs.  halt (optional, device int32, set by
 * rsx_nan_gate): when *halt != 0 nothing is updated.
 */
size_t rsx_mg_alpha_ws_bytes(int32_t count, const int64_t* n);
int rsx_mg_alpha(int32_t count, const float* const* params, const float* const* grads, const int64_t* n,
                 double base, double lr, double rel_step, double max_scale, double* alpha_out, void* ws,
                 size_t ws_bytes, const double* lr_dev, rsx_stream_t stream);
int rsx_axpy_multi(int32_t count, float* const* y, const float* const* x, const int64_t* n,
                   const double* alpha_dev, double mult, const double* lr_dev, const int32_t* halt,
                   rsx_stream_t stream);
/*
 * The batch loss's NaN check (reference src/common/trainer.py:192-203: a NaN loss ends
 * training before backward) without a host sync: counter[0] += 1 (the batch's 1-based
 * index in the epoch), and on the first NaN *loss halt = {1, that index}.  The
 * optimizer launches that take `halt` (rsx_adam_multi_scaled, rsx_axpy_multi) then
 * leave every parameter and moment as it was, so the parameters stay those before the
 * NaN batch; the trainer reads halt once at the end of the epoch.  Capturable.
 */
int rsx_nan_gate(const float* loss, int32_t* halt, int32_t* counter, rsx_stream_t stream);
/*
 * SMORE's spectral filter weights (reference src/models/smore.py:221-229): three
 * [d/2+1][2] (re, im) parameters -> out [3][d/2+1][2], each w / (|w| + 1e-8) when
 * normalize (else copied): the unit weights rsx_smore_spectral_fwd/bwd take.  The
 * backward sums rsx_smore_spectral_bwd's per-block partials [n_blocks][3][d/2+1][2]
 * in block order and applies the normalisation's Jacobian: gradients of the raw
 * parameters.
 */
int rsx_smore_unit_weights(const float* wv, const float* wt, const float* wf, int32_t d, int32_t normalize,
                           float* out, rsx_stream_t stream);
int rsx_smore_unit_weights_bwd(const float* partials, int64_t n_blocks, const float* wv, const float* wt,
                               const float* wf, int32_t d, int32_t normalize, float* gv, float* gt, float* gf,
                               rsx_stream_t stream);
/*
 * torch.optim.Adam (single-tensor arithmetic, as rsx_rowwise's ADAM epilogue) over
 * `count` flat tensors in one launch per 32 tensors; step_dev[i]: tensor i's
 * (already incremented) int64 step count on the device.  Replaces the per-parameter
 * optimizer loop of reference src/common/trainer.py:238 (optimizer.step()).
 */
int rsx_adam_multi(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2, float eps,
                   float weight_decay, rsx_stream_t stream);
/* The same with the gradient taken as g * grad_scale (an f32 product, as the
 * reference's p.grad.mul_(-mg_beta) before the mirror-gradient step,
 * src/common/trainer.py:327-330, folded into the update); lr_dev (optional, device
 * f64): the learning rate read on the device (rounded to f32) instead of lr; halt
 * (optional, rsx_nan_gate's flag): when *halt != 0 nothing is updated. */
int rsx_adam_multi_scaled(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                          const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2,
                          float eps, float weight_decay, float grad_scale, const double* lr_dev,
                          const int32_t* halt, rsx_stream_t stream);
/* The same with the mirror gradient's restore folded in (reference
 * src/common/trainer.py:332-335, `p.add_(+alpha_eff * lr * g)` then optimizer.step()):
 * each p first becomes p + rx * float(*ralpha * rmult) (with lr_dev:
 * float(*ralpha * (rmult * *lr_dev))), two roundings as rsx_axpy_multi, then the Adam
 * update of rsx_adam_multi_scaled — bit-equal to rsx_axpy_multi followed by it, with
 * one pass over p instead of two.  rx[i]: tensor i's saved gradient g(theta); rx and
 * ralpha are both NULL (no restore) or both given. */
int rsx_adam_multi_mg(int32_t count, float* const* p, const float* const* g, float* const* m, float* const* v,
                      const int64_t* const* step_dev, const int64_t* n, float lr, float beta1, float beta2, float eps,
                      float weight_decay, float grad_scale, const double* lr_dev, const int32_t* halt,
                      const float* const* rx, const double* ralpha, double rmult, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* SMORE kNN item graph (knn.hip)                                             */
/* ------------------------------------------------------------------------ */
/*
 * build_sim + build_knn_normalized_graph(sparse, 'sym') (reference
 * src/utils/utils.py:134-181, called at src/models/smore.py:58-61,69-71) from the
 * raw feature table feat [n, f] f32 (device): rows L2-normalised (x / ||x||), the
 * cosine similarities on f32 MFMA with the per-row top-k kept in registers (the
 * n x n matrix is never formed), k <= 32:
 *   vals [n, k]    kept similarities, (value desc, index asc) per row (self included)
 *   idx  [n, k]    int64 neighbour ids
 *   weights [n, k] d_r^-1/2 * v * d_c^-1/2, d = the row's kept-value sum (inf -> 0)
 * Workspace rsx_knn_ws_bytes(n, f) (the normalised table).
 */
size_t rsx_knn_ws_bytes(int64_t n, int32_t f);
int rsx_knn_graph(const float* feat, int64_t n, int32_t f, int32_t k, float* vals, int64_t* idx, float* weights,
                  void* ws, size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Graph builders on the device (graph.hip)                                   */
/* ------------------------------------------------------------------------ */
/*
 * rsx_adj_build: the normalised symmetric user-item adjacency from the interaction
 * list (u, i) [n_edges] int64 (duplicates collapse), CSR over n = n_users + n_items
 * rows (users first, item column ids offset by n_users), columns sorted per row:
 *   mode 0  LightGCN / LayerGCN eval graph (src/models/lightgcn.py:65-103):
 *           (d_r + 1e-7)^-1/2 (d_c + 1e-7)^-1/2 in float64, cast to float32;
 *   mode 1  SMORE (src/models/smore.py:176-207): float32 d^-1/2, inf -> 0, d_r*1*d_c.
 * dinv_table (device, optional): [table_len] float64, the per-node factor of every
 * degree 0 .. table_len-1 (mode 0: (deg + 1e-7)^-1/2; mode 1: the float32 value
 * widened).  The caller computes it with the same host pow the reference uses
 * (numpy's; np.power is not guaranteed to be correctly rounded, and neither is the
 * device's pow), so every edge value equals the reference's bit for bit whatever the
 * degree range (rsx.ops.adj_build builds it from a degree bound).  A node whose
 * degree is >= table_len, or dinv_table NULL, falls back to the device's float64
 * pow (correctly rounded to within an ulp: bit-equal on the graphs tested, not
 * guaranteed).
 * rowptr [n+1]; col, val have capacity 2 n_edges (nnz = rowptr[n], twice the number
 * of distinct pairs).  Workspace rsx_adj_build_ws_bytes.
 *
 * rsx_edge_dropout_build: LayerGCN's per-epoch graph (src/models/layergcn.py:51-81)
 * from the kept-edge mask keep [n_edges] (uint8) over the training edges (e_u, e_i)
 * and the symmetric template of all edges sorted by (row, col) (t_rowptr [n+1],
 * t_col [2 n_edges], t_eid [2 n_edges]: the edge each entry comes from): values
 * float32 1/sqrt(1e-7 + kept degree) products, the kept entries compacted in order.
 * rowptr [n+1]; col, val capacity 2 n_edges.
 */
size_t rsx_adj_build_ws_bytes(int64_t n_edges, int64_t n_users, int64_t n_items);
int rsx_adj_build(const int64_t* u, const int64_t* i, int64_t n_edges, int64_t n_users, int64_t n_items,
                  int32_t mode, const double* dinv_table, int64_t table_len, int64_t* rowptr, int32_t* col,
                  float* val, void* ws, size_t ws_bytes, rsx_stream_t stream);
size_t rsx_edge_dropout_ws_bytes(int64_t n_edges, int64_t n_users, int64_t n_items);
int rsx_edge_dropout_build(const int64_t* e_u, const int64_t* e_i, const uint8_t* keep, int64_t n_edges,
                           int64_t n_users, int64_t n_items, const int64_t* t_rowptr, const int32_t* t_col,
                           const int64_t* t_eid, int64_t* rowptr, int32_t* col, float* val, void* ws,
                           size_t ws_bytes, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Row-sharded LightGCN over RCCL (one process per GPU)                       */
/* ------------------------------------------------------------------------ */
/*
 * The reference is single-device (src/utils/configurator.py:114-118 pins one
 * GPU); SURVEY.md 8(e) scales the propagation by sharding users in contiguous
 * per-rank row blocks with the item rows replicated.  Per layer the item rows are
 * a per-rank partial (R_g^T users_g) summed across ranks by an in-place RCCL
 * all-reduce on the communicator's own stream, fenced by events against the
 * caller's stream (fork after the partial, join before the first reader).
 *
 * rsx_comm_t wraps an RCCL communicator plus that stream and its events.  RCCL is
 * resolved at run time (the copy torch loaded, else librccl.so.1); without it the
 * rsx_comm_* calls return RSX_ERR_COMM.  Create with the usual unique-id
 * handshake: rank 0 calls rsx_comm_get_unique_id, broadcasts the
 * rsx_comm_unique_id_bytes() bytes, and every rank calls rsx_comm_init (a
 * collective: all ranks must call it).  The device is the current HIP device.
 * rsx_comm_init / rsx_comm_destroy allocate, create streams and synchronise;
 * everything else is stream-ordered.
 */
typedef struct rsx_comm_s* rsx_comm_t;
size_t rsx_comm_unique_id_bytes(void);
int rsx_comm_get_unique_id(void* id_host);
int rsx_comm_init(rsx_comm_t* out, const void* id_host, int32_t rank, int32_t world);
int rsx_comm_destroy(rsx_comm_t comm);
/* Test hook: a communicator whose exchanges call `fn(op, buf, count, dtype, ctx)`
 * on the host (after synchronising the caller's stream) instead of RCCL — lets a
 * host-side collective (e.g. torch gloo) drive the sharded step with several ranks
 * on one GPU.  In place on device memory `buf`:
 *   op RSX_COLL_ALLREDUCE      buf[0, count) := sum over ranks
 *   op RSX_COLL_ALLGATHER      buf[r count, (r+1) count) := rank r's slice, every r
 *   op RSX_COLL_REDUCESCATTER  buf[rank count, (rank+1) count) := sum over ranks of
 *                              that slice (buf holds world * count elements)
 * dtype RSX_COLL_F32 / RSX_COLL_I64.  `fn` returns 0 on success. */
enum { RSX_COLL_ALLREDUCE = 0, RSX_COLL_ALLGATHER = 1, RSX_COLL_REDUCESCATTER = 2 };
enum { RSX_COLL_F32 = 0, RSX_COLL_I64 = 1 };
typedef int (*rsx_host_collective_fn)(int32_t op, void* buf, int64_t count, int32_t dtype, void* ctx);
int rsx_comm_init_host(rsx_comm_t* out, int32_t rank, int32_t world, rsx_host_collective_fn fn, void* ctx);
/* Latency injection (a one-GPU stand-in for a sim_world-rank job): a communicator of
 * world 1 whose collectives leave the data as it is (the one-rank result) and instead
 * run, on the communicator's stream, a kernel of `blocks` 256-thread workgroups that
 * streams the collective's HBM bytes through a `scratch_mb` scratch buffer and holds
 * its slots for the modelled time of the collective at sim_world ranks: a ring moves
 * 2 (W-1)/W X bytes per rank for an all-reduce of X, (W-1)/W X for an all-gather or
 * reduce-scatter whose whole buffer is X, at `busbw_gbs` GB/s per rank, plus
 * `latency_us`.  A one-rank step over it has the compute of one rank of the modelled
 * job and the exchanges' time and CU / HBM footprint on the comm stream, so its
 * measured step time is the modelled job's critical path.
 * rsx_comm_sim_seconds: the modelled time of one collective (the buffer's bytes). */
int rsx_comm_init_sim(rsx_comm_t* out, int32_t sim_world, double busbw_gbs, double latency_us, int32_t blocks,
                      int64_t scratch_mb);
double rsx_comm_sim_seconds(rsx_comm_t comm, int32_t op, double bytes);
/* buf[0, n) := sum over ranks, in place, ordered after the work queued on `stream`
 * and before the work queued on it afterwards. */
int rsx_comm_allreduce_f32(rsx_comm_t comm, float* buf, int64_t n, rsx_stream_t stream);
/* The same all-reduce without the wait: the caller's stream goes on (work that does not
 * read buf overlaps the exchange) until rsx_comm_wait(comm, stream), which orders the
 * stream after the started all-reduce.  One in flight per communicator: a second start
 * before the wait returns RSX_ERR_ARG (its join would otherwise replace the first's). */
int rsx_comm_allreduce_f32_start(rsx_comm_t comm, float* buf, int64_t n, rsx_stream_t stream);
int rsx_comm_wait(rsx_comm_t comm, rsx_stream_t stream);
/* buf[r n, (r+1) n) := rank r's slice for every rank r (buf holds world * n floats), in
 * place, stream-ordered as above. */
int rsx_comm_allgather_f32(rsx_comm_t comm, float* buf, int64_t n, rsx_stream_t stream);

/*
 * One LightGCN batch on this rank's shard (the sharded twin of rsx_lightgcn_step;
 * reference src/models/lightgcn.py:117-156 + src/common/trainer.py:238):
 *   adj_u  rows = the rank's n_users users, cols = [local users | items]
 *          (only the item columns are populated), values d_u^-1/2 d_i^-1/2 with
 *          GLOBAL item degrees (so every value equals the unsharded matrix's);
 *   adj_i  rows = the n_items items, cols populated with the local users only.
 * Every [n_users + n_items, d] table is local users first, then the replicated
 * items; `t` is [n_items, d] scratch.  A step issues 2K+1 all-reduces of
 * n_items*d floats: the forward's item partials of layers 1..K, G's item rows,
 * the backward's layers 1..K-1, and the item gradient t.  Item Adam then runs
 * identically on every rank (its inputs are bit-identical after the sums), user
 * Adam locally.  With `row_tag` ([n_users + n_items] int32, zero-filled before
 * the first step, `tag` fresh per step as in rsx_lgcn_step) and K = 2 or 3 the
 * step keeps the layers instead of running sums, computes the last user layer on
 * the batch rows only and runs the backward as Horner on G/(K+1) (2K SpMM
 * launches and one item-Adam launch per step, no layer-sum passes); G and R must
 * then be zero between steps.  The loss is this rank's mean BPR + its regulariser; the
 * objective is the sum over ranks (data-parallel batches of `batch` per rank).
 * rsx_sharded_lightgcn_forward fills final_emb only (evaluation).
 *
 * Sparse exchange (union_items != NULL, K = 2 or 3 with row_tag): the step first
 * all-gathers every rank's (pos, neg) item ids into union_items [world][2 union_cap];
 * the last forward layer's item rows are computed only on that union (item_tag
 * [n_items] int32, zero-filled once) and summed as a compact [world 2 batch, d]
 * block (cbuf0), G's item rows likewise (cbuf1) — the loss reads nothing else; the
 * item gradient t is REDUCE-SCATTERED over n_items_pad = world * ceil(n_items /
 * world) rows (t and the item block of p, m, v padded to that; pad rows zero), each
 * rank runs Adam on its own n_items_pad / world item rows, and the updated item
 * rows are ALL-GATHERED back into every replica.  Per step: 2(K-1) dense
 * all-reduces + one reduce-scatter + one all-gather of n_items*d floats (the
 * volume of 2K-1 dense all-reduces for K = 3, against 2K+1) plus two
 * compact all-reduces of world*2*batch rows.
 */
typedef struct rsx_sharded_lgcn_step {
    const rsx_csr* adj_u;
    const rsx_csr* adj_i;
    int64_t n_users, n_items;   /* local users, all items */
    int32_t d, n_layers;
    float reg;
    int32_t pad0;
    float* p; float* m; float* v;
    float* s; float* h0; float* h1;
    float* final_emb; float* g; float* r;
    float* t;                   /* [n_items, d] */
    float* slab_u; float* slab_i;
    int64_t* triplets;          /* [3][batch], item ids in [0, n_items) */
    int64_t batch;
    rsx_adam adam;
    float* loss_out;            /* [1] */
    double* loss_acc;           /* [1] or NULL */
    void* ws; size_t ws_bytes;  /* >= rsx_bpr_ws_bytes(batch) */
    rsx_comm_t comm;
    int32_t* row_tag;           /* optional, see above */
    int64_t tag;
    /* optional: read the tag from here instead (device int32, e.g. the low word of
     * the adam.step_dev counter), so that the step can be captured once in a hipGraph
     * and replayed: with adam.step_dev and tag_dev every per-step value lives on
     * the device and the step's launches and collectives are fixed. */
    const int32_t* tag_dev;
    /* optional with row_tag: [3 (n_users + n_items) + 4] int32, zero-filled before
     * the first step (as rsx_lgcn_step.reg_cnt): BPR runs as ONE launch and leaves
     * the regulariser gradient as per-row occurrence counts; the user rows' Adam and
     * the last item partial apply and clear them; r is not used. */
    int32_t* reg_cnt;
    /* optional sparse exchange (see above) */
    int64_t* union_items;       /* [world][2 union_cap] */
    int32_t* item_tag;          /* [n_items] */
    float* cbuf0; float* cbuf1; /* [world 2 union_cap, d] each */
    int64_t n_items_pad;        /* rows of t and of p/m/v's item block (>= n_items) */
    int64_t union_cap;          /* per-rank slice of union_items: 2 union_cap ids (>= batch; the
                                 * unused tail is zero-filled, so every rank sends the same count) */
    /* optional, dense schedule with row_tag and n_layers 2 or 3: [2 n_items, d] floats.
     * The step then sums two layers' item partials per collective (an item partial
     * needs only the rank's own user rows): 4 collectives per step at K = 3 (3 at
     * K = 2) instead of 2K + 1, the same bytes, the compute between rounds serialised
     * (csrc/dist.hip:sharded_fused_rounds; rsx.dist enables it with RSX_SHARDED_FUSED=1). */
    float* xch;
    /* optional (the stored-layer step, n_layers 2 or 3): the first forward item partial
     * issued as n_head > 1 row pieces of adj_i, each piece's rows all-reduced as soon as
     * that piece is computed, so the step's first exchange starts after 1/n_head of the
     * product instead of after all of it (nothing else of the step can hide it).
     * head_i[p] (host array) is the CSR of item rows [head_row0[p], head_row0[p+1]) of
     * adj_i with its own work schedule (row ids local to the piece, nonzero offsets
     * into adj_i's col/val) and its own slab head_slab[p]; results are bit-identical to
     * the one-launch product (same chunks, same fixup order). */
    int32_t n_head;
    int32_t pad1;
    const rsx_csr* head_i;
    const int64_t* head_row0;   /* host, [n_head + 1] */
    float* const* head_slab;    /* host, [n_head] (NULL entries for pieces without long rows) */
    /* optional with the sparse exchange (training): the last stored forward layer's item
     * rows E^{K-1}_I are read only by the final rows of the batch users (their neighbour
     * items) and of the union items, so they are summed over exactly those rows: every
     * rank lists its batch users' neighbour items and its own (pos, neg) items in its
     * nbr_cap slice of nbr_items (unused slots item 0), the lists are all-gathered, and
     * one compact [world nbr_cap, d] all-reduce (cbufN) replaces the dense one of
     * n_items*d floats.  nbr_cap >= 2 union_cap + the largest neighbour count of any
     * union_cap of this rank's users (the host bounds it); nbr_count is a device int. */
    int64_t* nbr_items;         /* [world][nbr_cap] */
    int32_t* nbr_count;         /* [1] */
    float* cbufN;               /* [world nbr_cap, d] */
    int64_t nbr_cap;
    /* optional with the sparse exchange: 1 = the all-gather of the owners' updated item rows
     * is issued at the START of the next step (on the comm stream, waited on only before the
     * first product that reads item rows of p, so it overlaps the first item partial) instead
     * of at the end of this one.  Between steps the item rows owned by other ranks are then
     * one step old on this rank: call rsx_sharded_lightgcn_flush before reading p (forward,
     * evaluation, checkpoints).  Issuing it when nothing is pending is harmless (idempotent). */
    int32_t defer_ag;
    int32_t pad2;
    /* optional [1] device int32, zero-filled: the sparse exchange's row lists never
     * dereference an id outside [0, n_items); such an id sets bit 0 instead (the lists are
     * built from the triplets, so it means a corrupt batch), and a neighbour list longer than
     * nbr_cap sets bit 1 (impossible under the host bound: each distinct batch user is listed
     * once).  The host reads it at its sync points (rsx.dist: flush / forward / close). */
    int32_t* err;
} rsx_sharded_lgcn_step;

int rsx_sharded_lightgcn_step(const rsx_sharded_lgcn_step* st, rsx_stream_t stream);
/* the deferred parameter all-gather of a defer_ag step (see above), stream-ordered */
int rsx_sharded_lightgcn_flush(const rsx_sharded_lgcn_step* st, rsx_stream_t stream);
int rsx_sharded_lightgcn_forward(const rsx_sharded_lgcn_step* st, rsx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Data-parallel LightGCN over RCCL (one process per GPU, graph replicated)   */
/* ------------------------------------------------------------------------ */
/*
 * Every rank holds the whole graph and a bit-identical replica of p, m, v; a step
 * trains the global batch of all ranks' triplets (rank r its own [3][batch]): the
 * reference objective at batch sum_r batch_r (src/models/lightgcn.py:132-156 with the
 * mean and the Frobenius norms over the global batch; src/common/trainer.py:186-238
 * at batch W B).  The step is lgcn_step_stored_layers' (K = 2..4) with ONE exchange:
 * an all-gather of every rank's triplets (`slots`, [world][3 cap + 1] int64: count,
 * users, positives, negatives), issued on the communicator's stream while the forward
 * runs.  Every rank then evaluates the whole global batch itself — the last forward
 * layer on the union of the ranks' batch rows, the BPR loss and G' = dL/dfinal/(K+1)
 * of every triplet (G' accumulated per row in 64-bit fixed point, so the sum does not
 * depend on the order of its atomics), the backward and Adam — with the same kernels
 * on the same inputs, so the replicas stay bit-identical with no other exchange.
 * row_tag [N] int32 (zero-filled once): the union's tags; reg_cnt [3 N + 4] (zero-
 * filled once): the global regulariser's occurrence counts; tag_dev: the step's tag on
 * the device (> 0, fresh per step, e.g. the low word of adam.step_dev), so the step
 * captures once in a hipGraph.  g, reg_cnt and `work` must be zero-filled before the
 * first step (every step leaves them so).  `work`: rsx_dp_work_bytes(n_users + n_items,
 * d, cap, world) bytes (the fixed-point accumulators, the occurrence sort, the loss
 * partials).  Over a latency-injected communicator (rsx_comm_init_sim, modelled world
 * W) the one rank times rank 0 of a W-rank job: slots hold W ranks, the caller fills
 * slots 1..W-1 (the other ranks' triplets), `work` is sized for W, and the stand-in
 * all-gather moves (W-1)/W of the W-slot buffer.
 */
typedef struct rsx_dp_lgcn_step {
    const rsx_csr* adj;         /* the whole graph */
    int64_t n_users, n_items;
    int32_t d, n_layers;        /* n_layers 2..4 */
    float reg;
    /* nonzero: the step's first launch increments *adam.step_dev itself (whose low word
     * is then tag_dev), so a captured step needs no separate counter launch; zero: the
     * caller has already incremented it */
    int32_t inc_step;
    float* p; float* m; float* v;
    float* s; float* h0; float* h1;   /* E^1, E^2 (h0, h1), E^3 (s, K = 4 only) */
    float* final_emb; float* g;
    float* slab;
    int64_t* triplets;          /* this rank's [3][batch] */
    int64_t batch;              /* 1 <= batch <= cap */
    rsx_adam adam;
    float* loss_out;            /* [1]: the global batch's loss */
    double* loss_acc;           /* [1] or NULL */
    rsx_comm_t comm;
    int32_t* row_tag;           /* [N] */
    const int32_t* tag_dev;     /* [1] */
    int32_t* reg_cnt;           /* [3 N + 4] */
    int32_t* halt;              /* [2] or NULL: set by a NaN global loss (as rsx_lgcn_step.halt) */
    int64_t cap;                /* per-rank batch capacity (every rank the same) */
    int64_t* slots;             /* [world][3 cap + 1] */
    void* work; size_t work_bytes;  /* >= rsx_dp_work_bytes(...), zero-filled once */
} rsx_dp_lgcn_step;

int rsx_dp_lightgcn_step(const rsx_dp_lgcn_step* st, rsx_stream_t stream);
size_t rsx_dp_work_bytes(int64_t n_rows, int32_t d, int64_t cap, int32_t world);

/* ------------------------------------------------------------------------ */
/* CPU kernels (host memory): the CPU dispatch key of torch.ops.rsx.*        */
/* ------------------------------------------------------------------------ */
/*
 * the custom operators carry CPU and HIP kernels, so the reference's
 * CPU configuration (C1: "CPU PyTorch reference path, no GPU") runs through the same
 * operator boundary.  Host pointers, synchronous, rows split over RSX_CPU_THREADS workers
 * (default: the hardware threads); each output row is written by one worker in a fixed
 * order (results independent of the thread count).  Same formulas as the HIP kernels:
 *   rsx_cpu_spmm              y = A x (CSR, f32)                     torch.sparse.mm
 *   rsx_cpu_propagate_mean    out = (x + A x + ... + A^K x) / (K+1)  lightgcn.py:117-130
 *   rsx_cpu_layergcn_forward  out = sum_k c_k A E^{k-1}, c_k the cosine gate;
 *                             zs [K][n][d], cs [K][n] optional saves  layergcn.py:127-140
 *   rsx_cpu_layergcn_backward dx from G = d/d out and the saves (RSX_EPI_LAYERGCN_BWD)
 *   rsx_cpu_bpr               rsx_bpr's variants; gradients ADDED     loss.py:33-61
 *   rsx_cpu_fullsort_topk     rsx_fullsort_topk's contract (scores, mask -1e10, top-k in
 *                             (score desc, item asc) order)          trainer.py:509-528
 *   rsx_cpu_adam              torch.optim.Adam, `step` already incremented  trainer.py:238
 */
int rsx_cpu_spmm(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows, const float* x,
                 int32_t d, float* y);
int rsx_cpu_propagate_mean(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n, const float* x,
                           int32_t d, int32_t n_layers, float* out);
int rsx_cpu_layergcn_forward(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n, const float* x,
                             int32_t d, int32_t n_layers, float* out, float* zs, float* cs);
int rsx_cpu_layergcn_backward(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n,
                              const float* x, int32_t d, int32_t n_layers, const float* G, const float* zs,
                              const float* cs, float* dx);
int rsx_cpu_bpr(int32_t variant, const float* final_emb, const float* ego_emb, int64_t n_users, int64_t n_items,
                int32_t d, const int64_t* triplets, int64_t batch, float reg, float batch_cfg, float* g_final,
                float* g_ego, float* loss_out);
int rsx_cpu_fullsort_topk(const float* user_emb, const int64_t* users, int64_t n_batch, const float* item_emb,
                          int64_t n_items, int32_t d, const int64_t* mask_rowptr, const int32_t* mask_col, int32_t k,
                          float* scores_out, int64_t* idx_out);
int rsx_cpu_adam(float* p, const float* g, float* m, float* v, int64_t n, int64_t step, float lr, float beta1,
                 float beta2, float eps, float weight_decay);
/*
 * One training batch of the CPU configuration in one call (the C1 path; replaces the
 * reference's calculate_loss + loss.backward() + optimizer.step(), trainer.py:186-238, for
 * lightgcn.py:117-156 (kind 0) and layergcn.py:127-177 (kind 1)): propagation with the last
 * layer on the batch rows only, BPR + regulariser on those rows, the backward propagation
 * (LightGCN: Horner on G, A symmetric; LayerGCN: the cosine-gate backward layer by layer),
 * Adam (`step` already incremented) over the whole [n_users + n_items, d] table p.
 * triplets int64 [3][batch] (item ids local); loss_out[0] = the batch loss.
 * Workspace: rsx_cpu_gcn_step_ws_floats(kind, n, d, n_layers, batch) floats.
 */
size_t rsx_cpu_gcn_step_ws_floats(int32_t kind, int64_t n, int32_t d, int32_t n_layers, int64_t batch);
int rsx_cpu_gcn_step(int32_t kind, const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_users,
                     int64_t n_items, int32_t d, int32_t n_layers, const int64_t* triplets, int64_t batch, float reg,
                     float* p, float* m, float* v, int64_t step, float lr, float beta1, float beta2, float eps,
                     float weight_decay, float* ws, size_t ws_floats, float* loss_out);

#ifdef __cplusplus
}
#endif
#endif /* RSX_H */
