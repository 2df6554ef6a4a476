/*
 * retrieval_core.h — C ABI of the MI355X-native retrieval core.
 *
 * One hipcc-built shared library (libretrieval_core.so, gfx950) behind the
 * reference's own API for the hot path "embed a batch of images → exact cosine
 * top-k over an in-HBM index".  The reference has no FFI of its own: its hot
 * path is remote Python (transformers in the embedding pod, Pinecone SaaS for
 * the index).  Each entry point below names the reference call it replaces;
 * INTEGRATION.md shows the ctypes binding a maintainer would add.
 *
 * Conventions
 *   - every function returns int status (RC_OK = 0); on error the message is
 *     in the thread-local rc_last_error(); no C++ exception crosses the ABI;
 *   - device buffers are caller-owned (e.g. torch tensors' data_ptr) unless a
 *     function says otherwise; `stream` is a hipStream_t (NULL = default);
 *   - hot calls (rc_index_search, rc_index_upsert, rc_embed) allocate nothing
 *     once the workspace is reserved (rc_index_reserve / rc_model_create);
 *   - each handle is bound to the device it was created on and guarded by a
 *     mutex, so a multi-threaded caller may share it.
 */
#ifndef RETRIEVAL_CORE_H
#define RETRIEVAL_CORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RC_ABI_VERSION 1

/* status codes */
#define RC_OK 0
#define RC_ERR_INVALID 1     /* bad argument (maps to ValueError)            */
#define RC_ERR_HIP 2         /* HIP runtime failure                          */
#define RC_ERR_OOM 3         /* device allocation failed                     */
#define RC_ERR_UNSUPPORTED 4 /* valid request outside what the build handles */
#define RC_ERR_STATE 5       /* handle not ready (e.g. weights missing)      */

/* storage dtypes of index rows */
#define RC_F32 0
#define RC_F16 1
#define RC_BF16 2

/* Pillow resampling filters (PIL.Image.Resampling values) */
#define RC_RESAMPLE_BILINEAR 2
#define RC_RESAMPLE_BICUBIC 3

#define RC_TOPK_MAX 256 /* largest k a single search call accepts */

typedef struct rc_index rc_index;
typedef struct rc_sharded rc_sharded;
typedef struct rc_model rc_model;

const char *rc_last_error(void);
int rc_abi_version(void);
/* Device and pinned-host allocations the library has made so far (all handles).
 * Diagnostic: the tests check that steady-state hot calls (search, fetch,
 * upsert, embed once their workspaces exist) leave it unchanged. */
int64_t rc_alloc_count(void);

/* ------------------------------------------------------------------------
 * In-HBM exact cosine index.  Replaces the Pinecone index:
 *   get_index(name)            ingesting/utils.py:23-38, retriever/utils.py:23-38
 *   index.upsert([(id,v,md)])  ingesting/main.py:156-158
 *   index.query(v, top_k)      retriever/utils.py:62-64
 *   index.fetch(ids)           retriever/main.py:142
 * Rows are stored L2-normalised in `dtype`, row-major with leading dimension
 * ld = round_up(dim, 128) (zero padded).  String ids and metadata stay on the
 * host; the device only knows row numbers.  A search returns
 * row_base + local_row * row_stride (row_stride = 1 unless rc_index_set_row_map
 * says otherwise): the global row of a shard in a multi-GPU index.
 * ---------------------------------------------------------------------- */

/* replaces pc.create_index(metric="cosine", dimension=dim) — ingesting/utils.py:29-36 */
int rc_index_create(int device, int dim, int dtype, int64_t capacity, int64_t row_base, rc_index **out);
int rc_index_destroy(rc_index *h);
int rc_index_info(const rc_index *h, int *dim, int *dtype, int64_t *capacity, int64_t *ld);
/* device pointer to row 0 of the stored (normalised, cast) rows */
int rc_index_data(const rc_index *h, void **rows_dev, float **norms_dev);

/* Shard row map: local row l is reported as row_base + l * row_stride (a
 * round-robin shard s of n uses row_base = s, row_stride = n). */
int rc_index_set_row_map(rc_index *h, int64_t row_base, int64_t row_stride);

/* Grow the row capacity in place (rows and norms are copied to a larger
 * allocation; new slots are zero).  Pinecone indexes have no fixed capacity
 * (ingesting/utils.py:29-36 creates one without a size); the host layer grows
 * on demand.  The caller orders earlier work on other streams; the call
 * synchronises the device before releasing the old buffers. */
int rc_index_grow(rc_index *h, int64_t new_capacity, void *stream);

/* Size the search workspace for up to max_nq queries and k <= max_k.  Called
 * once before the hot loop; search grows it on demand otherwise. */
int rc_index_reserve(rc_index *h, int max_nq, int max_k);

/* replaces index.upsert — ingesting/main.py:156-158.
 * vecs: device f32 [n, dim]; rows: device i64 [n] local row slots (host-assigned:
 * an existing id keeps its row, so upsert overwrites).  Each row is L2-normalised
 * in f32, cast to the storage dtype and scattered; its norm is kept so fetch can
 * return the original values.  An all-zero vector is rejected by the host layer.
 * Rows must be distinct within one call (one wave per vector writes its row: a
 * repeated row would interleave two vectors); Index.upsert keeps the last
 * occurrence of a repeated id before calling. */
int rc_index_upsert(rc_index *h, const float *vecs, int64_t n, const int64_t *rows, void *stream);

/* replaces index.fetch(ids)["vectors"][id]["values"] — retriever/main.py:142.
 * rows: device i64 [n]; out: device f32 [n, dim] = stored row × stored norm. */
int rc_index_fetch(rc_index *h, const int64_t *rows, int64_t n, float *out, void *stream);
/* The stored (normalised, dtype-rounded) rows as f32, without the norm —
 * what the search actually scores against (parity tests run the oracle on these). */
int rc_index_fetch_stored(rc_index *h, const int64_t *rows, int64_t n, float *out, void *stream);

/* Snapshot / restore (Pinecone keeps an index durable server-side; the in-HBM
 * index is saved by the host layer — Index.save / Index.load — through these).
 * Raw copy of the stored rows [row0, row0+n) exactly as searched (storage dtype,
 * ld-padded, normalised) and their norms.  Buffers may be device or host memory
 * (hipMemcpyDefault); the copy is ordered on `stream`. */
int rc_index_export(rc_index *h, int64_t row0, int64_t n, void *rows_out, float *norms_out, void *stream);
int rc_index_import(rc_index *h, int64_t row0, int64_t n, const void *rows_in, const float *norms_in, void *stream);

/* replaces index.query(vector, top_k) — retriever/utils.py:62-64.
 * queries: device f32 [nq, dim] (normalised inside); rows [0, n_rows) are searched.
 * scores: device f32 [nq, k] cosine, descending; out_rows: device i64 [nq, k]
 * (global rows, see the row map).  Ties: score desc, then row asc.  Slots beyond
 * n_rows get score -inf and row -1 (n_rows = 0, an empty shard, is valid in
 * every mode).  1 <= k <= RC_TOPK_MAX; a larger top_k is RC_ERR_INVALID. */
int rc_index_search(rc_index *h, const float *queries, int nq, int64_t n_rows, int k,
                    float *scores, int64_t *out_rows, void *stream);

/* Search algorithm selection for rc_index_search_ex (same results either way):
 *   RC_SEARCH_SCAN — HBM-bound streaming scan, 1-4 queries per pass over the rows;
 *   RC_SEARCH_MFMA — batched: query-block x row-tile MFMA GEMM (f16/bf16 index only)
 *                    whose epilogue keeps candidates within a proven error bound
 *                    of the running kth score, exact f32 rescoring of candidates;
 *                    a query whose candidates overflow is re-run through the
 *                    exact scan ON THE DEVICE (no host synchronisation);
 *   RC_SEARCH_AUTO — MFMA for >= 8 queries on an f16/bf16 index of >= 64k rows.
 * This is the batched form of index.query (retriever/utils.py:62-64) that
 * BASELINE config 4 (1024 queries, top-100) exercises. */
#define RC_SEARCH_AUTO 0
#define RC_SEARCH_SCAN 1
#define RC_SEARCH_MFMA 2
int rc_index_search_ex(rc_index *h, const float *queries, int nq, int64_t n_rows, int k,
                       float *scores, int64_t *out_rows, int mode, void *stream);

/* Filter copy for the batched search (no reference counterpart: Pinecone's query
 * internals; results are unchanged, only the speed of RC_SEARCH_MFMA):
 *   RC_FILTER_NATIVE — the filter GEMM reads the stored rows (f16/bf16 MFMA);
 *   RC_FILTER_I8     — the index also keeps an int8 copy of every row (per-row
 *                      scale and residual norm, ld + 8 bytes per row, maintained
 *                      by upsert / fill / import / grow); the filter GEMM runs on
 *                      int8 MFMA at twice the f16 rate with a per-(query, row) error
 *                      bound, and candidates are rescored exactly on the stored rows.
 *                      Row widths (dim rounded up to 128) 256, 512 or 768; makes
 *                      RC_SEARCH_MFMA available on f32 indexes too.
 * Enabling quantises every row (synchronous on `stream`). */
#define RC_FILTER_NATIVE 0
#define RC_FILTER_I8 1
int rc_index_set_filter(rc_index *h, int kind, void *stream);
int rc_index_get_filter(const rc_index *h, int *kind);

/* Synthetic rows for benchmarks (no reference counterpart): rows
 * [row0, row0+n) get uniform[-1,1) values from a counter-based hash of
 * (seed, row, col), normalised and cast like an upsert. */
int rc_index_fill_random(rc_index *h, uint64_t seed, int64_t row0, int64_t n, void *stream);

/* Merge nlists top-k lists per query into one (cross-shard merge after the
 * all-gather; no reference counterpart — Pinecone merges server-side).
 * scores/rows: device [nlists, nq, k_in] of (score, global row); rows < 0 are
 * empty slots; global rows must be < 2^32 - 1 (every rc_index row map is
 * checked against that bound at create / set_row_map / grow).  Result ordered score desc, then
 * row asc — whatever the routing of rows to lists.  out: device [nq, k]. */
int rc_topk_merge(const float *scores, const int64_t *rows, int nlists, int nq, int k_in, int k,
                  float *out_scores, int64_t *out_rows, void *stream);

/* ------------------------------------------------------------------------
 * One index over several shards in one process (SURVEY §8(b):
 * rc_index_create(dim, dtype, capacity_per_gpu, n_gpus)).  Shard s is an
 * rc_index on devices[s] (devices may repeat: several shards on one GPU);
 * global row g lives on shard g % n_shards as local row g / n_shards
 * (round-robin, so every shard fills from the first upsert).  Queries and
 * results live on devices[0] (the leader); shards search concurrently on their
 * own streams and their lists are merged on the leader (rc_topk_merge).
 * Total capacity < 2^32 rows.
 * ---------------------------------------------------------------------- */
int rc_sharded_create(int n_shards, const int *devices, int dim, int dtype, int64_t capacity_per_shard,
                      rc_sharded **out);
int rc_sharded_destroy(rc_sharded *h);
/* Test hook: drive every shard but the leader through the cross-device path (subset
 * gather on the leader, peer copies of queries / subsets / result lists, leader merge)
 * even where shards share the leader's GPU — the code an 8-GPU node runs, on one GPU. */
int rc_sharded_force_remote(rc_sharded *h);
int rc_sharded_info(const rc_sharded *h, int *n_shards, int64_t *capacity_per_shard, int64_t *ld);
/* Borrowed handle of shard s (persistence, parity tests); owned by h. */
int rc_sharded_shard(rc_sharded *h, int s, rc_index **out);
int rc_sharded_grow(rc_sharded *h, int64_t new_capacity_per_shard);
/* replaces index.upsert — ingesting/main.py:156-158.  vecs: leader-device f32
 * [n, dim]; rows: HOST i64 [n] global rows.  Synchronous (ordered after work
 * already queued on `stream`). */
int rc_sharded_upsert(rc_sharded *h, const float *vecs, int64_t n, const int64_t *rows, void *stream);
/* replaces index.fetch — retriever/main.py:142.  rows: HOST i64 [n] global rows;
 * out: HOST f32 [n, dim] (stored = 0: the upserted values; 1: the normalised
 * stored rows the search scores).  Synchronous. */
int rc_sharded_fetch(rc_sharded *h, const int64_t *rows, int64_t n, float *out, int stored);
/* replaces index.query — retriever/utils.py:62-64.  queries: leader-device f32
 * [nq, dim]; n_rows: global rows [0, n_rows) are searched; scores / out_rows:
 * leader-device [nq, k], identical to one rc_index holding the same rows. */
int rc_sharded_search(rc_sharded *h, const float *queries, int nq, int64_t n_rows, int k, float *scores,
                      int64_t *out_rows, int mode, void *stream);
/* replaces index.query(vector, top_k, include_values=True) on the request path —
 * retriever/utils.py:62-64 (the call retriever/main.py:127-130 times).  Host in,
 * host out: queries HOST f32 [nq, dim]; scores HOST f32 [nq, k], out_rows HOST i64
 * [nq, k] (global rows, -1 past the index), values HOST f32 [nq, k, dim] (the
 * upserted values of each match, NaN for -1 slots; only when with_values).  One
 * H2D copy, the search, the matched rows' gather and ONE D2H copy on the index's
 * own leader stream, then one synchronisation; no allocation once the staging
 * has grown to the call's size.  Results equal rc_sharded_search +
 * rc_sharded_fetch. */
int rc_sharded_query_host(rc_sharded *h, const float *queries, int nq, int64_t n_rows, int k, int with_values,
                          float *scores, int64_t *out_rows, float *values);
/* rc_index_set_filter on every shard; all or nothing (a failure restores
 * RC_FILTER_NATIVE on every shard). */
int rc_sharded_set_filter(rc_sharded *h, int kind);

/* ------------------------------------------------------------------------
 * ViT-MSN image embedding.  Replaces the /embed compute path —
 * embedding/main.py:97-114: PIL decode (stays on host) → ViTImageProcessor
 * (resize, rescale, normalize) → ViTMSNModel → last_hidden_state[:, 0, :].
 * ---------------------------------------------------------------------- */
typedef struct rc_vit_config {
    int image_size;   /* 224 */
    int patch;        /* 16 */
    int hidden;       /* 768 */
    int layers;       /* 12 */
    int heads;        /* 12 */
    int mlp;          /* 3072 */
    float ln_eps;     /* 1e-6 */
    int max_batch;    /* workspace is sized for this many images per rc_embed call */
} rc_vit_config;

/* replaces ViTMSNModel.from_pretrained(...).to(DEVICE) — embedding/main.py:37-39 */
int rc_model_create(int device, const rc_vit_config *cfg, rc_model **out);
int rc_model_destroy(rc_model *m);
/* One state-dict tensor by checkpoint key (legacy layout, e.g.
 * "encoder.layer.3.attention.attention.query.weight"; an optional "vit."
 * prefix and the transformers-5 names "layers.N.attention.q_proj.weight" are
 * also accepted).  host_data: host f32, numel must match. */
int rc_model_set_weight(rc_model *m, const char *name, const float *host_data, int64_t numel);
/* Preprocessor parameters (ViTImageProcessor: resample, rescale_factor, image_mean, image_std). */
int rc_model_set_preprocess(rc_model *m, int resample, double rescale_factor, const float mean[3], const float std_[3]);
/* Verify every weight was set and build the fused device layouts. */
int rc_model_finalize(rc_model *m);

/* replaces embedding/main.py:107-114 for a batch.
 * images: device u8 [n, h, w, 3] (HWC RGB, as decoded by PIL); n <= max_batch.
 * (h, w) != (image_size, image_size) → Pillow-exact resize on the device first.
 * raw_out: device f32 [n, hidden] = last_hidden_state[:, 0, :] (the /embed body);
 * normed_out: device f32 [n, hidden] L2-normalised copy for the index (may be NULL). */
int rc_embed(rc_model *m, const uint8_t *images, int n, int h, int w,
             float *raw_out, float *normed_out, void *stream);

/* Preprocess only: device u8 [n,h,w,3] → device f32 pixel_values [n,3,S,S]
 * exactly as ViTImageProcessor produces them (for parity tests). */
int rc_preprocess(rc_model *m, const uint8_t *images, int n, int h, int w, float *pixel_values, void *stream);

/* Encode a batch as `parts` (1..4) concurrent slices on their own HIP streams
 * (default 2; slices below 32 images are merged).  Results are bit-identical
 * for every setting: each image's arithmetic is the same.  One slice's memory-
 * bound kernels (LayerNorm, attention) and GEMM store bursts then overlap the
 * other slices' MFMA main loops.  rc_embed still returns ordered on `stream`. */
int rc_model_set_parts(rc_model *m, int parts);

/* Last encoder layer on the CLS rows only (default 1).  /embed returns
 * last_hidden_state[:, 0, :] (embedding/main.py:113-114), and row 0 of the last
 * layer (modeling_vit_msn.py:254-283) reads only its own query row plus every
 * token's K/V: with cls_only = 1 the last layer runs LN1 + QKV on all rows, then
 * CLS-query attention, O-proj, LN2 and the MLP on the CLS rows alone.
 * cls_only = 0 runs the whole layer (A/B and parity tests). */
int rc_model_set_last_layer(rc_model *m, int cls_only);

/* LayerNorm fold (default 1): the two LayerNorms of each layer
 * (modeling_vit_msn.py:258-259) are folded into the GEMMs around them — the residual producers (patch embed, O-proj, fc2) also
 * write bf16(x) and per-256-column (mean, M2) partials, and QKV / fc1 apply
 * rstd·(x·(W∘γ)ᵀ − μ·Σ_k W∘γ) + (b + W·β) in their epilogues — instead of a
 * standalone LayerNorm pass over the f32 stream.  0 runs the LN kernel (A/B and
 * parity tests). */
int rc_model_set_ln_fold(rc_model *m, int on);

/* Batch-1 HIP graphs (default 1): an rc_embed of one image at the model's input size
 * (the reference's /embed request, embedding/main.py:88-124) replays a HIP graph of its
 * launch chain, captured on first use per (images, raw_out, normed_out) buffer triple
 * (at most 8 kept, least recently used evicted; after 8 misses in a row only a triple that
 * misses twice in a row is captured, the others run the stream form): one host launch per
 * request instead of ~70.  Same kernels, same bits.  Every setter drops the captured graphs.
 * 0 = stream form. */
int rc_model_set_graphs(rc_model *m, int on);

/* Per-kernel timing with HIP events on the launch stream (bench/roofline).
 * kernel ids: 0 = all GEMMs, 1 = fc1 GEMM, 2 = attention, 3 = layernorm,
 * 4 = preprocess, 5 = QKV GEMM, 6 = O-proj GEMM, 7 = fc2 GEMM (5-7 and 1: the
 * full-batch launches of that projection); `mask` bit i enables id i (-1 = all, 0 = off). */
int rc_model_timing(rc_model *m, int mask);
int rc_model_timing_read(rc_model *m, int kernel_id, double *total_ms, int64_t *launches, double *flops);
int rc_model_timing_reset(rc_model *m);

/* Kernel-level entry to the projection GEMM (parity tests / microbenchmarks;
 * inside rc_embed this is every nn.Linear of modeling_vit_msn.py:199-202,243-244).
 * out = epilogue(A[M][K] · W[N][K]ᵀ + bias): epi 0 → bf16 out, 1 → bf16 GELU(out),
 * 2 → f32 out += (residual, in place), 3 → f32 patch scatter (+pos, tokens/image).
 * A must have round_up(M, 256) readable rows; N % 256 == 0 (M > 256), K % 64 == 0.
 * variant: 0 auto, 4 256x256 ping-pong, 8 128x256 two-workgroup, 9 skinny (M <= 256),
 * 10 image-aligned 224-row tiles (the model's O-proj / fc2 kernel; epi 2 only, `tokens` =
 * rows per image, tile t = rows [t·tokens, t·tokens + tokens); A must then hold
 * ceil(M / tokens)·tokens + 224 − tokens readable rows). */
int rc_gemm_bf16(int epi, int variant, const uint16_t *A, const uint16_t *W, const float *bias, int M, int N, int K,
                 void *out, const float *pos, int tokens, void *stream);

/* Index-side timing of the dominant search kernel (scan), same conventions. */
int rc_index_timing(rc_index *h, int enable);
int rc_index_timing_read(rc_index *h, double *total_ms, int64_t *launches, double *bytes);
/* Same for the batched search's filter GEMM (flops = 2 * query slots * rows * ld per launch);
 * fallbacks = queries re-run through the on-device exact scan since the last
 * read (candidate overflow; synchronises the device to read the counter). */
int rc_index_gemm_timing_read(rc_index *h, double *total_ms, int64_t *launches, double *flops, int64_t *fallbacks);


/* ------------------------------------------------------------------------
 * JPEG decode.  Replaces Image.open(BytesIO(bytes)).convert("RGB") —
 * embedding/main.py:97 — for baseline JPEGs: Huffman decode on the host
 * (one thread per image), dequantisation + islow IDCT + fancy upsampling +
 * YCbCr->RGB on the GPU, bit-exact with Pillow/libjpeg-turbo defaults.
 * Other streams (progressive, arithmetic, 12-bit, CMYK/RGB colour spaces,
 * multi-scan) report supported = 0 and stay on the host decode path.
 * ---------------------------------------------------------------------- */
typedef struct rc_jpeg_info {
    int32_t width, height, ncomp, supported;
    int32_t hmax, vmax, restart_interval, mcux, mcuy;
    int32_t h[3], v[3];   /* sampling factors per component */
    int32_t bw[3], bh[3]; /* 8x8 blocks per component plane (MCU padded) */
    int64_t blocks;       /* coefficient blocks of the image, all planes */
} rc_jpeg_info;
typedef struct rc_jpeg_decoder rc_jpeg_decoder;

/* Header walk: size, components, sampling, whether rc_jpeg_decode handles it.
 * RC_ERR_INVALID if the bytes are not a JPEG stream (the caller's
 * UnidentifiedImageError path, embedding/main.py:115-119). */
int rc_jpeg_probe(const uint8_t *jpg, int64_t len, rc_jpeg_info *info);
/* Host-only entropy decode (test hook): quantised coefficients of every block,
 * natural order, planes in component order ([blocks][64] int16), and each
 * component's quantisation table in natural order ([ncomp][64] u16). */
int rc_jpeg_decode_coefficients(const uint8_t *jpg, int64_t len, int16_t *coef, uint16_t *qtab);
/* Pinned host staging + device workspace for up to max_images images and
 * max_blocks coefficient blocks per call (no allocation in rc_jpeg_decode). */
int rc_jpeg_decoder_create(int device, int max_images, int64_t max_blocks, rc_jpeg_decoder **out);
int rc_jpeg_decoder_destroy(rc_jpeg_decoder *h);
/* Decode n JPEGs (host buffers) into device HWC RGB u8: image i is written at
 * rgb + rgb_offsets[i] (host array, bytes), height x width x 3.  The host
 * buffers may be reused once the call returns; the reconstruction is ordered
 * on `stream`.  RC_ERR_UNSUPPORTED if any image is outside what the decoder
 * handles (probe first), RC_ERR_INVALID for damaged or truncated data. */
int rc_jpeg_decode(rc_jpeg_decoder *h, int n, const uint8_t *const *jpgs, const int64_t *lens, uint8_t *rgb,
                   const int64_t *rgb_offsets, void *stream);
/* Decode n JPEGs (any sizes, mixed) straight to out_size x out_size: the decode above
 * followed by Pillow's resample (`resample` = RC_RESAMPLE_BICUBIC / _BILINEAR, the
 * ViTImageProcessor resize of embedding/main.py:107), with the colour pass fused into
 * the horizontal resample (the full-size RGB image is never written).  out: device u8
 * [n][out_size][out_size][3], bit-exact with PIL decode + Image.resize.  A horizontal
 * pass buffer grows with the largest batch seen (no allocation once warm). */
int rc_jpeg_decode_resized(rc_jpeg_decoder *h, int n, const uint8_t *const *jpgs, const int64_t *lens, int out_size,
                           int resample, uint8_t *out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* RETRIEVAL_CORE_H */
