// index.hip — the in-HBM exact cosine index that replaces Pinecone
// (reference: get_index ingesting/utils.py:23-38, upsert ingesting/main.py:156-158,
//  query retriever/utils.py:59-66, fetch retriever/main.py:142).
//
// HBM layout: rows [capacity][ld] in the storage dtype (f32 / f16 / bf16),
// L2-normalised at upsert, ld = 128 * nch (zero-padded), plus norms [capacity] f32.
//
// Search (single / few queries) is one streaming pass over the rows:
//   scan_topk_kernel: 16 lanes per row, 16-B loads, f32 FMA against the
//     query held in registers, DPP reduction across the 16 lanes, then a
//     wavefront top-k (ballot-filtered append against a running threshold +
//     register bitonic sort) per wave, merged per block → partial keys;
//   merge_partials_kernel: per query, top-k over all blocks' partial lists.
// Algorithmic HBM bytes per query pass: n_rows * ld * sizeof(T).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "index_common.h"

namespace rc {

static thread_local std::string g_last_error;
void set_last_error(const std::string &m) { g_last_error = m; }

// ------------------------------------------------------- upsert / fetch --
// One wave per vector: norm in f32, normalise, cast, scatter to its row slot.
// src (optional): vector v is read from vecs[src[v]] (a shard's subset of a batch).
template <typename T>
__global__ __launch_bounds__(256) void upsert_kernel(T *__restrict__ rows, float *__restrict__ norms, int64_t ld, int dim,
                                                    const float *__restrict__ vecs, const int64_t *__restrict__ src_idx,
                                                    const int64_t *__restrict__ slot, int64_t n, int64_t cap) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= n) return;
    const int64_t r = slot[v];
    if (r < 0 || r >= cap) return;  // device-side guard: never write outside the row slots (hosts validate first)
    const float *src = vecs + (src_idx ? src_idx[v] : v) * dim;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss = fmaf(src[c], src[c], ss);
    ss = wave_sum(ss);
    const float nrm = sqrtf(ss);
    const float inv = nrm > 0.f ? 1.0f / nrm : 0.f;
    T *dst = rows + r * ld;
    for (int c = lane; c < ld; c += 64) dst[c] = Elem<T>::cast(c < dim ? src[c] * inv : 0.f);
    if (lane == 0) norms[r] = nrm;
}

template <typename T>
__global__ __launch_bounds__(256) void fetch_kernel(const T *__restrict__ rows, const float *__restrict__ norms, int64_t ld,
                                                   int dim, const int64_t *__restrict__ slot, int64_t n,
                                                   float *__restrict__ out, int64_t cap) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= n) return;
    const int64_t r = slot[v];
    if (r < 0 || r >= cap) {  // out of range: NaN values, never a read outside the rows
        for (int c = lane; c < dim; c += 64) out[v * dim + c] = __builtin_nanf("");
        return;
    }
    const float nrm = norms ? norms[r] : 1.0f;
    for (int c = lane; c < dim; c += 64) out[v * dim + c] = Elem<T>::load(rows, r * ld + c) * nrm;
}

// splitmix64 finaliser: the synthetic-row generator (reproducible in numpy).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ float synth_value(uint64_t seed, int64_t row, int dim, int c) {
    const uint64_t h = splitmix64(seed * 0xD1342543DE82EF95ull + (uint64_t)row * (uint64_t)dim + (uint64_t)c);
    return (float)(int32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;  // 24-bit uniform in [-1, 1)
}

template <typename T>
__global__ __launch_bounds__(256) void fill_random_kernel(T *__restrict__ rows, float *__restrict__ norms, int64_t ld,
                                                         int dim, uint64_t seed, int64_t row0, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); v < n; v += nw) {
        const int64_t r = row0 + v;
        float ss = 0.f;
        for (int c = lane; c < dim; c += 64) {
            const float x = synth_value(seed, r, dim, c);
            ss = fmaf(x, x, ss);
        }
        ss = wave_sum(ss);
        const float nrm = sqrtf(ss);
        const float inv = 1.0f / nrm;
        T *dst = rows + r * ld;
        for (int c = lane; c < ld; c += 64) dst[c] = Elem<T>::cast(c < dim ? synth_value(seed, r, dim, c) * inv : 0.f);
        if (lane == 0) norms[r] = nrm;
    }
}

// The int8 filter copy (search_mfma.hip, filter_i8_kernel): one wave per stored row x̂,
// sx = max|x̂| / 127, x8 = rne(x̂ / sx) clamped to [-127, 127], ex = ||x̂ - sx·x8||₂ rounded
// up (x1.001 covers the f32 sum of squares, +1e-7 the f32 residuals), sx and ex at
// i8_slot(row).  Rows come from slots[v] (upsert) or row0 + v (fill / import / enable).
template <typename T>
__global__ __launch_bounds__(256) void quantize_rows_kernel(const T *__restrict__ rows, int64_t ld,
                                                           const int64_t *__restrict__ slots, int64_t row0, int64_t n,
                                                           int64_t cap, int8_t *__restrict__ rows8, float *__restrict__ rsx,
                                                           float *__restrict__ rex) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); v < n; v += nw) {
        const int64_t r = slots ? slots[v] : row0 + v;
        if (r < 0 || r >= cap) continue;  // wave-uniform
        const T *src = rows + r * ld;
        float mx = 0.f;
        for (int c = lane; c < ld; c += 64) mx = fmaxf(mx, fabsf(Elem<T>::load(src, c)));
        mx = wave_max(mx);
        const float s = mx * (1.0f / 127.0f), is = mx > 0.f ? 127.0f / mx : 0.f;
        float e = 0.f;
        int8_t *dst = rows8 + r * ld;
        for (int c = lane; c < ld; c += 64) {
            const float x = Elem<T>::load(src, c);
            const float q = fminf(127.f, fmaxf(-127.f, rintf(x * is)));
            dst[c] = (int8_t)q;
            const float d = x - s * q;
            e = fmaf(d, d, e);
        }
        e = wave_sum(e);
        if (lane == 0) {
            rsx[i8_slot(r)] = s;
            rex[i8_slot(r)] = sqrtf(e) * 1.001f + 1e-7f;
        }
    }
}

// queries [nq, dim] f32 → normalised, zero-padded [nq, ld]
// rows >= nq (padding up to a multiple of the scan's queries-per-pass) are zero.
__global__ __launch_bounds__(64) void normalize_queries_kernel(const float *__restrict__ q, int nq, int dim, int64_t ld,
                                                              float *__restrict__ qn) {
    const int lane = threadIdx.x;
    const bool valid = (int)blockIdx.x < nq;
    const float *src = q + (int64_t)(valid ? blockIdx.x : 0) * dim;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss = valid ? fmaf(src[c], src[c], ss) : 0.f;
    ss = wave_sum(ss);
    const float inv = ss > 0.f ? 1.0f / sqrtf(ss) : 0.f;
    for (int c = lane; c < ld; c += 64) qn[(int64_t)blockIdx.x * ld + c] = (valid && c < dim) ? src[c] * inv : 0.f;
}

// One block per query: top-k over nlist sorted partial lists of k keys each.
// flags (optional): only queries with flags[q] != 0 are merged (the batched
// search's exact fallback).  Returned row = row_base + local row * row_stride.
template <int CAP>
__global__ __launch_bounds__(256) void merge_partials_kernel(const uint64_t *__restrict__ partial, int nlist,
                                                            int nq_total, int k, int64_t row_base, int64_t row_stride,
                                                            const int *__restrict__ flags,
                                                            float *__restrict__ out_scores,
                                                            int64_t *__restrict__ out_rows) {
    __shared__ uint64_t lds[4][CAP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = blockIdx.x;
    if (flags != nullptr && flags[qi] == 0) return;  // block-uniform
    WaveTopK<CAP> tk;
    merge_partial_lists<CAP>(partial, nlist, nq_total, qi, k, lds, tk);
    if (wave == 0) {
        for (int j = lane; j < k; j += 64) {
            const uint64_t key = tk.buf[j];
            const bool ok = key != KEY_EMPTY;
            out_scores[(int64_t)qi * k + j] = ok ? key_score(key) : -INFINITY;
            out_rows[(int64_t)qi * k + j] = ok ? row_base + (int64_t)key_idx(key) * row_stride : -1;
        }
    }
}

// Top-k of many sorted partial lists, one query per block (config 3: 1M rows = 1024 scan blocks,
// lists of k keys).  The answer's k-th key is at most hk, the k-th smallest of the lists' heads
// (k heads are <= hk), and a sorted list can only contribute its prefix <= hk: so the block takes
// the heads' top-k (one load per list, all in flight), then appends the prefixes <= hk of the
// lists whose head qualifies (usually about k keys in all), then sorts those.  The same keys as
// merging every list (merge_partial_lists, which loads all nlist·k keys: round 4's one block over
// ~2000 lists was 30.5 us, the two-level form after it 11 + 12 us); more than CAP candidates
// (adversarial inputs) fall back to that full merge inside the block.
constexpr int MERGE_HEADS_MIN = 64;  // fewer lists: merge_partials_kernel (all keys) is as fast
template <int CAP>
__global__ __launch_bounds__(256) void merge_heads_kernel(const uint64_t *__restrict__ partial, int nlist, int nq_total,
                                                         int k, int64_t row_base, int64_t row_stride,
                                                         const int *__restrict__ flags, float *__restrict__ out_scores,
                                                         int64_t *__restrict__ out_rows) {
    __shared__ uint64_t lds[4][CAP];
    __shared__ uint64_t cand[CAP];
    __shared__ uint64_t hk_s;
    __shared__ int ccount;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
    const int qi = blockIdx.x;
    if (flags != nullptr && flags[qi] == 0) return;  // block-uniform
    auto at = [&](int l, int t) { return partial[((int64_t)l * nq_total + qi) * k + t]; };
    WaveTopK<CAP> tk;
    tk.init(as_lds(&lds[wave][0]), k);
    // 1. the heads' top-k: HU heads per lane in flight, then per-wave top-k, then wave 0 over 4·k
    constexpr int HU = 8;
    for (int l0 = 0; l0 < nlist; l0 += 256 * HU) {
        uint64_t h[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            const int l = l0 + u * 256 + tid;
            h[u] = l < nlist ? at(l, 0) : KEY_EMPTY;
        }
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            tk.reserve(64);
            tk.push(h[u] != KEY_EMPTY, h[u]);
        }
    }
    tk.compact();
    if (tid == 0) ccount = 0;
    __syncthreads();
    if (wave == 0) {
        for (int w = 1; w < 4; ++w)
            for (int j = 0; j < k; j += 64) {
                const uint64_t key = (j + lane < k) ? as_lds(&lds[w][0])[j + lane] : KEY_EMPTY;
                tk.reserve(64);
                tk.push(key != KEY_EMPTY, key);
            }
        tk.compact();
        if (lane == 0) hk_s = tk.count >= k ? tk.buf[k - 1] : KEY_EMPTY;
    }
    __syncthreads();
    const uint64_t hk = hk_s;
    // 2. the prefixes <= hk of the lists whose head is <= hk (a list is sorted, EMPTY-padded)
    for (int l = tid; l < nlist; l += 256) {
        if (at(l, 0) > hk) continue;  // (an L2 hit: loaded in step 1)
        for (int t0 = 0; t0 < k; t0 += 8) {
            uint64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = t0 + u < k ? at(l, t0 + u) : KEY_EMPTY;
            bool more = true;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (v[u] <= hk && v[u] != KEY_EMPTY) {
                    const int pos = atomicAdd(&ccount, 1);
                    if (pos < CAP) cand[pos] = v[u];
                } else {
                    more = false;
                }
            }
            if (!more) break;
        }
    }
    __syncthreads();
    const int nc = ccount;
    if (nc > CAP) {  // block-uniform: the full merge
        merge_partial_lists<CAP>(partial, nlist, nq_total, qi, k, lds, tk);
    } else if (wave == 0) {
        tk.init(as_lds(&lds[0][0]), k);
        for (int j = 0; j < nc; j += 64) {
            tk.reserve(64);
            tk.push(j + lane < nc, j + lane < nc ? cand[j + lane] : KEY_EMPTY);
        }
        tk.compact();
    }
    if (wave == 0) {
        for (int j = lane; j < k; j += 64) {
            const uint64_t key = tk.buf[j];
            const bool ok = key != KEY_EMPTY;
            out_scores[(int64_t)qi * k + j] = ok ? key_score(key) : -INFINITY;
            out_rows[(int64_t)qi * k + j] = ok ? row_base + (int64_t)key_idx(key) * row_stride : -1;
        }
    }
}

// Cross-shard merge: nlists lists of (score, global row) per query.  The key's
// low word is the global row itself (< 2^32), so equal scores order by row
// whatever the row → shard routing (contiguous ranges or round-robin).  Rows
// < 0 are empty slots.
template <int CAP>
__global__ __launch_bounds__(256) void merge_lists_kernel(const float *__restrict__ scores,
                                                         const int64_t *__restrict__ rows, int nlists, int nq,
                                                         int k_in, int k, float *__restrict__ out_scores,
                                                         int64_t *__restrict__ out_rows) {
    __shared__ uint64_t lds[4][CAP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = blockIdx.x;
    WaveTopK<CAP> tk;
    tk.init(as_lds(&lds[wave][0]), k);
    const int64_t total = (int64_t)nlists * k_in;
    for (int64_t j0 = (int64_t)wave * 64; j0 < total; j0 += 256) {
        const int64_t j = j0 + lane;
        uint64_t key = KEY_EMPTY;
        bool ok = false;
        if (j < total) {
            const int64_t l = j / k_in, t = j - l * k_in;
            const int64_t src = (l * nq + qi) * k_in + t;
            const int64_t row = rows[src];
            ok = row >= 0;
            key = make_key(scores[src], (uint32_t)row);
        }
        tk.reserve(64);
        tk.push(ok, key);
    }
    tk.compact();
    __syncthreads();
    if (wave == 0) {
        for (int w = 1; w < 4; ++w)
            for (int j = 0; j < k; j += 64) {
                const uint64_t key = (j + lane < k) ? as_lds(&lds[w][0])[j + lane] : KEY_EMPTY;
                tk.reserve(64);
                tk.push(key != KEY_EMPTY, key);
            }
        tk.compact();
        for (int j = lane; j < k; j += 64) {
            const uint64_t key = tk.buf[j];
            const bool ok = key != KEY_EMPTY;
            out_scores[(int64_t)qi * k + j] = ok ? key_score(key) : -INFINITY;
            out_rows[(int64_t)qi * k + j] = ok ? (int64_t)key_idx(key) : -1;
        }
    }
}

// Search over zero rows (an empty shard): every slot is (-inf, -1).
__global__ __launch_bounds__(256) void empty_result_kernel(int64_t n, float *__restrict__ scores, int64_t *__restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    scores[i] = -INFINITY;
    rows[i] = -1;
}

}  // namespace rc

// ================================================================= host ====
using namespace rc;

struct rc_index {
    std::mutex mu;
    int device = 0;
    int dim = 0;
    int dtype = RC_F32;
    int nch = 1;  // ld = 128 * nch
    int64_t ld = 0;
    int64_t capacity = 0;
    int64_t row_base = 0;    // a search returns row_base + local row * row_stride (shard → global rows)
    int64_t row_stride = 1;
    int ncu = 256;           // compute units of the device (scan grid rounds)
    void *rows = nullptr;
    float *norms = nullptr;
    // int8 filter copy (RC_FILTER_I8): [cap_pad][ld] x8, sx / ex [cap_pad] at i8_slot(row)
    int filter = RC_FILTER_NATIVE;
    int8_t *rows8 = nullptr;
    float *rsx = nullptr, *rex = nullptr;
    // search workspace
    int ws_nq = 0, ws_k = 0, ws_nblk = 0;
    float *qn = nullptr;
    uint64_t *partial = nullptr;
    unsigned *q1_done = nullptr;    // host-coherent completion word of the polled query1 path
    unsigned q1_seq = 0;
    BatchWs bws;         // batched MFMA search workspace (search_mfma.hip)
    KernelTimer timer;   // scan_topk_kernel launches (bytes)
    KernelTimer gtimer;  // filter_gemm_kernel launches (flops)
};

namespace {

constexpr int kNchSet[] = {1, 2, 3, 4, 6, 8, 12, 16};
constexpr int kMaxBlocks = 2048;
constexpr int kBatchMinQueries = 8;      // below this the HBM-bound scan wins (1-4 queries per pass)
constexpr int64_t kBatchMinRows = 65536;  // tiny shards: the staged path's fixed cost dominates

// Every global row a shard can report must fit the 32-bit row word of the top-k
// keys (merge_lists_kernel) below the all-ones value: row_base + (cap - 1) * stride < 2^32 - 1.
bool row_map_fits(int64_t row_base, int64_t row_stride, int64_t cap) {
    return (double)row_base + (double)(cap - 1) * (double)row_stride < 4294967295.0;
}

int pick_nch(int dim) {
    const int need = (dim + 127) / 128;
    for (int n : kNchSet)
        if (n >= need) return n;
    return -1;
}

void ensure_workspace(rc_index *h, int nq, int k) {
    if (nq <= h->ws_nq && k <= h->ws_k) return;
    const int nq2 = std::max(nq, h->ws_nq), k2 = std::max(k, h->ws_k);
    dfree(h->qn);
    dfree(h->partial);
    h->qn = nullptr;
    h->partial = nullptr;
    h->qn = (float *)dmalloc((size_t)nq2 * h->ld * sizeof(float));
    h->partial = (uint64_t *)dmalloc((size_t)kMaxBlocks * nq2 * k2 * sizeof(uint64_t));
    h->ws_nq = nq2;
    h->ws_k = k2;
}

int64_t cap_pad(int64_t capacity) { return (capacity + INDEX_ROW_PAD - 1) / INDEX_ROW_PAD * INDEX_ROW_PAD; }

// refresh the int8 filter copy of rows slots[0..n) (or row0 .. row0 + n) after a write
template <typename T>
void launch_quantize(rc_index *h, const int64_t *slots, int64_t row0, int64_t n, hipStream_t s) {
    if (h->rows8 == nullptr || n == 0) return;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 3) / 4, 256 * 32);
    hipLaunchKernelGGL(quantize_rows_kernel<T>, dim3(grid), dim3(256), 0, s, (const T *)h->rows, h->ld, slots, row0, n,
                       h->capacity, h->rows8, h->rsx, h->rex);
    RC_LAUNCH_CHECK();
}

void free_filter(rc_index *h) {
    dfree(h->rows8);
    dfree(h->rsx);
    dfree(h->rex);
    h->rows8 = nullptr;
    h->rsx = h->rex = nullptr;
    h->filter = RC_FILTER_NATIVE;
}

template <typename T>
void launch_upsert(rc_index *h, const float *vecs, const int64_t *src_idx, int64_t n, const int64_t *slots, hipStream_t s) {
    const unsigned grid = (unsigned)((n + 3) / 4);
    hipLaunchKernelGGL(upsert_kernel<T>, dim3(grid), dim3(256), 0, s, (T *)h->rows, h->norms, h->ld, h->dim, vecs, src_idx,
                       slots, n, h->capacity);
    RC_LAUNCH_CHECK();
    launch_quantize<T>(h, slots, 0, n, s);
}

template <typename T>
void launch_fetch(rc_index *h, const int64_t *slots, int64_t n, float *out, bool stored, hipStream_t s) {
    const unsigned grid = (unsigned)((n + 3) / 4);
    hipLaunchKernelGGL(fetch_kernel<T>, dim3(grid), dim3(256), 0, s, (const T *)h->rows, stored ? nullptr : h->norms, h->ld,
                       h->dim, slots, n, out, h->capacity);
    RC_LAUNCH_CHECK();
}

template <typename T>
void launch_fill(rc_index *h, uint64_t seed, int64_t row0, int64_t n, hipStream_t s) {
    const int64_t waves = (n + 0) ;
    unsigned grid = (unsigned)std::min<int64_t>((waves + 3) / 4, 256 * 32);
    if (grid == 0) return;
    hipLaunchKernelGGL(fill_random_kernel<T>, dim3(grid), dim3(256), 0, s, (T *)h->rows, h->norms, h->ld, h->dim, seed, row0, n);
    RC_LAUNCH_CHECK();
    launch_quantize<T>(h, nullptr, row0, n, s);
}

void launch_scan(rc_index *h, const ScanArgs &a) {
    switch (h->dtype) {
        case RC_F32: return launch_scan_f32(a);
        case RC_F16: return launch_scan_f16(a);
        case RC_BF16: return launch_scan_bf16(a);
        default: throw Error(RC_ERR_INVALID, "unknown dtype");
    }
}

// Top-k over nlist sorted partial lists per query, one block per query: past MERGE_HEADS_MIN lists
// through the lists' heads (merge_heads_kernel), else over every key (merge_partials_kernel).  The
// same keys either way.
template <int CAP>
void launch_merge_partials_t(rc_index *h, const uint64_t *partial, const int *flags, int nlist, int nq, int nq_stride, int k,
                             float *scores, int64_t *rows, hipStream_t s) {
    if (nlist >= MERGE_HEADS_MIN)
        hipLaunchKernelGGL(merge_heads_kernel<CAP>, dim3(nq), dim3(256), 0, s, partial, nlist, nq_stride, k, h->row_base,
                           h->row_stride, flags, scores, rows);
    else
        hipLaunchKernelGGL(merge_partials_kernel<CAP>, dim3(nq), dim3(256), 0, s, partial, nlist, nq_stride, k, h->row_base,
                           h->row_stride, flags, scores, rows);
    RC_LAUNCH_CHECK();
}

void launch_merge_partials(rc_index *h, const uint64_t *partial, const int *flags, int nlist, int nq, int nq_stride, int k,
                           float *scores, int64_t *rows, hipStream_t s) {
    const int cap = topk_cap(k);
    if (cap <= 128) return launch_merge_partials_t<128>(h, partial, flags, nlist, nq, nq_stride, k, scores, rows, s);
    if (cap <= 256) return launch_merge_partials_t<256>(h, partial, flags, nlist, nq, nq_stride, k, scores, rows, s);
    return launch_merge_partials_t<512>(h, partial, flags, nlist, nq, nq_stride, k, scores, rows, s);
}

template <typename F>
void dispatch_dtype(int dtype, F &&f) {
    switch (dtype) {
        case RC_F32: f(float{}); break;
        case RC_F16: f(f16_t{}); break;
        case RC_BF16: f(bf16_t{}); break;
        default: throw Error(RC_ERR_INVALID, "unknown dtype");
    }
}


void scan_search(rc_index *h, const float *queries, int nq, int64_t n_rows, int k, float *scores, int64_t *out_rows,
                 hipStream_t s) {
    // queries per scan pass: a power of two the kernel is instantiated for (1, 2, 4)
    int qb = 1;
    while (qb * 2 <= std::min(nq, scan_max_qb(h->nch, k))) qb *= 2;
    const int nq_pad = (nq + qb - 1) / qb * qb;  // every scan pass runs qb real-or-zero query slots
    ensure_workspace(h, nq_pad, k);  // (the scan normalises the queries itself: no separate launch)
    int nblk = (int)std::min<int64_t>(kMaxBlocks, std::max<int64_t>(1, (n_rows + 511) / 512));
    // past one round of resident blocks (4 per CU), whole rounds: 1M rows were 1954 blocks = 1.9
    // rounds, a tail of CUs with one block fewer; 1024 blocks of ~1000 rows are one round (and a
    // merge over half the lists)
    const int round_blocks = 4 * h->ncu;
    if (nblk > round_blocks) nblk = nblk / round_blocks * round_blocks;
    int64_t rpb = (n_rows + nblk - 1) / nblk;
    rpb = ((rpb + 31) / 32) * 32;
    if (rpb == 0) rpb = 32;
    nblk = (int)std::max<int64_t>(1, (n_rows + rpb - 1) / rpb);
    const double bytes = (double)n_rows * h->ld * dtype_size(h->dtype);
    if (h->timer.enabled) h->timer.create();
    for (int q0 = 0; q0 < nq_pad; q0 += qb) {
        const int slot = h->timer.begin(s);
        ScanArgs a{h->rows, h->ld, h->nch, n_rows, rpb, nblk, h->qn, q0, qb, nq_pad, k, h->partial, s};
        a.qraw = queries;
        a.dim = h->dim;
        a.nq_real = nq;
        launch_scan(h, a);
        h->timer.end(slot, s, bytes);
    }
    launch_merge_partials(h, h->partial, nullptr, nblk, nq, nq_pad, k, scores, out_rows, s);
}

// Batched MFMA search, then — still on the device, no host synchronisation —
// the exact scan for every query whose candidates overflowed: scan_topk_kernel
// in fallback mode (blocks early-exit for unflagged queries) over the batched
// path's normalised queries (the same f32 arithmetic as normalize_queries_kernel),
// and merge_partials_kernel over the flagged queries' partial lists.
void batched_search_exact(rc_index *h, const float *queries, int nq, int64_t n_rows, int k, float *scores,
                          int64_t *out_rows, hipStream_t s) {
    h->bws.ensure(nq, k, h->ld, (int)dtype_size(h->dtype));
    BatchPlan p{h->rows, h->dtype, h->dim, h->nch, h->ld, n_rows, h->row_base, h->row_stride, queries, nq, k, scores, out_rows};
    p.rows8 = h->rows8;
    p.rsx = h->rsx;
    p.rex = h->rex;
    if (h->gtimer.enabled) h->gtimer.create();
    batched_search(p, h->bws, s, h->gtimer.enabled ? &h->gtimer : nullptr);
    int nblk = (int)std::min<int64_t>(h->bws.fb_blocks, std::max<int64_t>(1, (n_rows + 511) / 512));
    int64_t rpb = (n_rows + nblk - 1) / nblk;
    rpb = std::max<int64_t>(32, (rpb + 31) / 32 * 32);
    nblk = (int)std::max<int64_t>(1, (n_rows + rpb - 1) / rpb);
    ScanArgs a{h->rows, h->ld, h->nch, n_rows, rpb, nblk, h->bws.qn, 0, 1, nq, k, h->bws.fb_partial, s};
    a.flags = h->bws.flags;
    a.grid_y = std::min(nq, FB_QSTRIDE);
    launch_scan(h, a);
    launch_merge_partials(h, h->bws.fb_partial, h->bws.flags, nblk, nq, nq, k, scores, out_rows, s);
}

void empty_search(int nq, int k, float *scores, int64_t *out_rows, hipStream_t s) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(empty_result_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, scores, out_rows);
    RC_LAUNCH_CHECK();
}

}  // namespace

namespace rc {
// Internal (sharded.hip): upsert vectors vecs[src_idx[i]] into local rows rows[i].
void index_upsert_gather(rc_index *h, const float *vecs, const int64_t *src_idx, int64_t n, const int64_t *rows,
                         hipStream_t s) {
    if (n == 0) return;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceScope ds(h->device);
    dispatch_dtype(h->dtype, [&](auto t) { launch_upsert<decltype(t)>(h, vecs, src_idx, n, rows, s); });
}

// Internal (sharded.hip, rc_sharded_query_host): one query as ONE launch (query1_kernel) —
// normalise, scan, merge, gather values — writing scores [k], rows [k] and (with_values)
// values [k][dim] to out_* (host-mapped memory is fine: nothing is copied back).  Returns
// false, enqueuing nothing, when the shape is outside the kernel's range (the caller takes
// the multi-kernel path).  n_rows >= 1.
bool index_query1(rc_index *h, const float *query, int64_t n_rows, int k, int with_values, float *out_scores,
                  int64_t *out_rows, float *out_values, hipStream_t s, volatile unsigned **done, unsigned *seq) {
    if (h->dim > QUERY1_MAX_DIM || h->nch > 6 || topk_cap(k) > 256 || n_rows < 1 || n_rows > QUERY1_MAX_ROWS) return false;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceScope ds(h->device);
    ensure_workspace(h, 1, k);
    Query1Args a{};
    a.rows = h->rows;
    a.norms = h->norms;
    a.ld = h->ld;
    a.dim = h->dim;
    a.nch = h->nch;
    a.n_rows = n_rows;
    // >= 64 rows a block (two passes of the block's 32-row step), at most QUERY1_MAX_BLOCKS lists
    int64_t rpb = std::max<int64_t>(64, (n_rows + QUERY1_MAX_BLOCKS - 1) / QUERY1_MAX_BLOCKS);
    rpb = (rpb + 31) / 32 * 32;
    a.rows_per_block = rpb;
    a.nblk = (int)((n_rows + rpb - 1) / rpb);
    a.k = k;
    a.with_values = with_values;
    a.row_base = h->row_base;
    a.row_stride = h->row_stride;
    a.partial = h->partial;
    a.out_scores = out_scores;
    a.out_rows = out_rows;
    a.out_values = out_values;
    if (done != nullptr) {  // the caller polls a host-coherent completion word (see spin_until)
        if (h->q1_done == nullptr) {
            RC_HIP(hipHostMalloc((void **)&h->q1_done, 64, hipHostMallocCoherent));
            *h->q1_done = 0u;
        }
        a.done = h->q1_done;
        a.seq = ++h->q1_seq;
        if (a.seq == 0u) a.seq = ++h->q1_seq;  // 0 is the initial word
        *done = h->q1_done;
        *seq = a.seq;
    }
    std::memcpy(a.q, query, (size_t)h->dim * sizeof(float));
    switch (h->dtype) {
        case RC_F32: launch_query1_f32(a, s); break;
        case RC_F16: launch_query1_f16(a, s); break;
        case RC_BF16: launch_query1_bf16(a, s); break;
        default: throw Error(RC_ERR_INVALID, "unknown dtype");
    }
    return true;
}
}  // namespace rc

namespace {

}  // namespace

extern "C" {

const char *rc_last_error(void) { return g_last_error.c_str(); }
int rc_abi_version(void) { return RC_ABI_VERSION; }
int64_t rc_alloc_count(void) { return g_alloc_count.load(std::memory_order_relaxed); }

int rc_index_create(int device, int dim, int dtype, int64_t capacity, int64_t row_base, rc_index **out) {
    return guard([&] {
        RC_REQUIRE(out != nullptr, RC_ERR_INVALID, "out is NULL");
        RC_REQUIRE(dim > 0, RC_ERR_INVALID, "dimension must be positive");
        RC_REQUIRE(dtype == RC_F32 || dtype == RC_F16 || dtype == RC_BF16, RC_ERR_INVALID, "dtype must be RC_F32/RC_F16/RC_BF16");
        RC_REQUIRE(capacity > 0 && capacity < (int64_t(1) << 32), RC_ERR_INVALID, "capacity must be in [1, 2^32)");
        RC_REQUIRE(row_base >= 0 && row_map_fits(row_base, 1, capacity), RC_ERR_INVALID,
                   "row_base + capacity must stay below 2^32 - 1 (global rows key the top-k merge)");
        const int nch = pick_nch(dim);
        RC_REQUIRE(nch > 0, RC_ERR_UNSUPPORTED, "dimension > 2048 is not supported");
        DeviceScope ds(device);
        auto *h = new rc_index();
        h->device = device;
        h->dim = dim;
        h->dtype = dtype;
        h->nch = nch;
        h->ld = 128LL * nch;
        h->capacity = capacity;
        h->row_base = row_base;
        try {
            RC_HIP(hipDeviceGetAttribute(&h->ncu, hipDeviceAttributeMultiprocessorCount, device));
            // whole 256-row tiles: the batched search reads row tiles without a bounds check
            const int64_t cap_pad = (capacity + INDEX_ROW_PAD - 1) / INDEX_ROW_PAD * INDEX_ROW_PAD;
            h->rows = dmalloc((size_t)cap_pad * h->ld * dtype_size(dtype));
            h->norms = (float *)dmalloc((size_t)capacity * sizeof(float));
            RC_HIP(hipMemset(h->rows, 0, (size_t)cap_pad * h->ld * dtype_size(dtype)));
            RC_HIP(hipMemset(h->norms, 0, (size_t)capacity * sizeof(float)));
            ensure_workspace(h, 4, 16);
        } catch (...) {
            dfree(h->rows);
            dfree(h->norms);
            dfree(h->qn);
            dfree(h->partial);
            delete h;
            throw;
        }
        *out = h;
    });
}

int rc_index_destroy(rc_index *h) {
    return guard([&] {
        if (!h) return;
        DeviceScope ds(h->device);
        h->timer.destroy();
        h->gtimer.destroy();
        h->bws.release();
        free_filter(h);
        dfree(h->rows);
        dfree(h->norms);
        dfree(h->qn);
        dfree(h->partial);
        if (h->q1_done != nullptr) (void)hipHostFree(h->q1_done);
        delete h;
    });
}

int rc_index_info(const rc_index *h, int *dim, int *dtype, int64_t *capacity, int64_t *ld) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        if (dim) *dim = h->dim;
        if (dtype) *dtype = h->dtype;
        if (capacity) *capacity = h->capacity;
        if (ld) *ld = h->ld;
    });
}

int rc_index_data(const rc_index *h, void **rows_dev, float **norms_dev) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        if (rows_dev) *rows_dev = h->rows;
        if (norms_dev) *norms_dev = h->norms;
    });
}

int rc_index_set_row_map(rc_index *h, int64_t row_base, int64_t row_stride) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(row_base >= 0 && row_stride >= 1, RC_ERR_INVALID, "row_base must be >= 0 and row_stride >= 1");
        std::lock_guard<std::mutex> lk(h->mu);
        RC_REQUIRE(row_map_fits(row_base, row_stride, h->capacity), RC_ERR_INVALID,
                   "row map exceeds 2^32 - 1 global rows (row_base + (capacity - 1) * row_stride)");
        h->row_base = row_base;
        h->row_stride = row_stride;
    });
}

int rc_index_grow(rc_index *h, int64_t new_capacity, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(new_capacity < (int64_t(1) << 32), RC_ERR_INVALID, "capacity must be < 2^32");
        std::lock_guard<std::mutex> lk(h->mu);
        if (new_capacity <= h->capacity) return;
        RC_REQUIRE(row_map_fits(h->row_base, h->row_stride, new_capacity), RC_ERR_INVALID,
                   "grown capacity exceeds 2^32 - 1 global rows under this shard's row map");
        DeviceScope ds(h->device);
        hipStream_t s = (hipStream_t)stream;
        const size_t rb = (size_t)h->ld * dtype_size(h->dtype);
        const int64_t old_pad = (h->capacity + INDEX_ROW_PAD - 1) / INDEX_ROW_PAD * INDEX_ROW_PAD;
        const int64_t new_pad = (new_capacity + INDEX_ROW_PAD - 1) / INDEX_ROW_PAD * INDEX_ROW_PAD;
        void *rows = dmalloc((size_t)new_pad * rb);
        float *norms = nullptr;
        int8_t *rows8 = nullptr;
        float *rsx = nullptr, *rex = nullptr;
        try {
            norms = (float *)dmalloc((size_t)new_capacity * sizeof(float));
            RC_HIP(hipMemcpyAsync(rows, h->rows, (size_t)old_pad * rb, hipMemcpyDeviceToDevice, s));
            RC_HIP(hipMemsetAsync((uint8_t *)rows + (size_t)old_pad * rb, 0, (size_t)(new_pad - old_pad) * rb, s));
            RC_HIP(hipMemcpyAsync(norms, h->norms, (size_t)h->capacity * sizeof(float), hipMemcpyDeviceToDevice, s));
            RC_HIP(hipMemsetAsync(norms + h->capacity, 0, (size_t)(new_capacity - h->capacity) * sizeof(float), s));
            if (h->rows8) {  // the filter copy keeps its slots (i8_slot is position-stable)
                const size_t rb8 = (size_t)h->ld;
                rows8 = (int8_t *)dmalloc((size_t)new_pad * rb8);
                rsx = (float *)dmalloc((size_t)new_pad * sizeof(float));
                rex = (float *)dmalloc((size_t)new_pad * sizeof(float));
                RC_HIP(hipMemcpyAsync(rows8, h->rows8, (size_t)old_pad * rb8, hipMemcpyDeviceToDevice, s));
                RC_HIP(hipMemsetAsync(rows8 + (size_t)old_pad * rb8, 0, (size_t)(new_pad - old_pad) * rb8, s));
                RC_HIP(hipMemcpyAsync(rsx, h->rsx, (size_t)old_pad * sizeof(float), hipMemcpyDeviceToDevice, s));
                RC_HIP(hipMemsetAsync(rsx + old_pad, 0, (size_t)(new_pad - old_pad) * sizeof(float), s));
                RC_HIP(hipMemcpyAsync(rex, h->rex, (size_t)old_pad * sizeof(float), hipMemcpyDeviceToDevice, s));
                RC_HIP(hipMemsetAsync(rex + old_pad, 0, (size_t)(new_pad - old_pad) * sizeof(float), s));
            }
            RC_HIP(hipStreamSynchronize(s));  // work queued earlier on other streams is the caller's to order
        } catch (...) {
            dfree(rows);
            dfree(norms);
            dfree(rows8);
            dfree(rsx);
            dfree(rex);
            throw;
        }
        RC_HIP(hipDeviceSynchronize());  // no kernel may still read the old buffers
        dfree(h->rows);
        dfree(h->norms);
        h->rows = rows;
        h->norms = norms;
        if (h->rows8) {
            dfree(h->rows8);
            dfree(h->rsx);
            dfree(h->rex);
            h->rows8 = rows8;
            h->rsx = rsx;
            h->rex = rex;
        }
        h->capacity = new_capacity;
    });
}

int rc_index_reserve(rc_index *h, int max_nq, int max_k) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(max_nq > 0 && max_k > 0 && max_k <= RC_TOPK_MAX, RC_ERR_INVALID, "bad reserve sizes");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        ensure_workspace(h, max_nq, max_k);
    });
}

int rc_index_set_filter(rc_index *h, int kind, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(kind == RC_FILTER_NATIVE || kind == RC_FILTER_I8, RC_ERR_INVALID, "filter must be RC_FILTER_NATIVE or RC_FILTER_I8");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        hipStream_t s = (hipStream_t)stream;
        if (kind == h->filter) return;
        if (kind == RC_FILTER_NATIVE) {
            RC_HIP(hipDeviceSynchronize());  // no search may still read the copy
            free_filter(h);
            return;
        }
        RC_REQUIRE(i8_filter_supported(h->ld), RC_ERR_UNSUPPORTED,
                   "the int8 filter needs a row width (dim rounded up to 128) of 256, 512 or 768");
        const int64_t pad = cap_pad(h->capacity);
        try {
            h->rows8 = (int8_t *)dmalloc((size_t)pad * h->ld);
            h->rsx = (float *)dmalloc((size_t)pad * sizeof(float));
            h->rex = (float *)dmalloc((size_t)pad * sizeof(float));
            RC_HIP(hipMemsetAsync(h->rows8, 0, (size_t)pad * h->ld, s));
            RC_HIP(hipMemsetAsync(h->rsx, 0, (size_t)pad * sizeof(float), s));
            RC_HIP(hipMemsetAsync(h->rex, 0, (size_t)pad * sizeof(float), s));
            dispatch_dtype(h->dtype, [&](auto t) { launch_quantize<decltype(t)>(h, nullptr, 0, h->capacity, s); });
            RC_HIP(hipStreamSynchronize(s));
        } catch (...) {
            free_filter(h);
            throw;
        }
        h->filter = RC_FILTER_I8;
    });
}

int rc_index_get_filter(const rc_index *h, int *kind) {
    return guard([&] {
        RC_REQUIRE(h && kind, RC_ERR_INVALID, "null argument");
        *kind = h->filter;
    });
}

int rc_index_upsert(rc_index *h, const float *vecs, int64_t n, const int64_t *rows, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(n >= 0, RC_ERR_INVALID, "negative count");
        if (n == 0) return;
        RC_REQUIRE(vecs && rows, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        dispatch_dtype(h->dtype, [&](auto t) { launch_upsert<decltype(t)>(h, vecs, nullptr, n, rows, (hipStream_t)stream); });
    });
}

int rc_index_fetch(rc_index *h, const int64_t *rows, int64_t n, float *out, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(n >= 0, RC_ERR_INVALID, "negative count");
        if (n == 0) return;
        RC_REQUIRE(rows && out, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        dispatch_dtype(h->dtype, [&](auto t) { launch_fetch<decltype(t)>(h, rows, n, out, false, (hipStream_t)stream); });
    });
}

int rc_index_fetch_stored(rc_index *h, const int64_t *rows, int64_t n, float *out, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(n >= 0, RC_ERR_INVALID, "negative count");
        if (n == 0) return;
        RC_REQUIRE(rows && out, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        dispatch_dtype(h->dtype, [&](auto t) { launch_fetch<decltype(t)>(h, rows, n, out, true, (hipStream_t)stream); });
    });
}

int rc_index_fill_random(rc_index *h, uint64_t seed, int64_t row0, int64_t n, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(row0 >= 0 && n >= 0 && row0 + n <= h->capacity, RC_ERR_INVALID, "rows out of capacity");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        dispatch_dtype(h->dtype, [&](auto t) { launch_fill<decltype(t)>(h, seed, row0, n, (hipStream_t)stream); });
    });
}

int rc_index_export(rc_index *h, int64_t row0, int64_t n, void *rows_out, float *norms_out, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(row0 >= 0 && n >= 0 && row0 + n <= h->capacity, RC_ERR_INVALID, "rows out of capacity");
        if (n == 0) return;
        RC_REQUIRE(rows_out && norms_out, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        const size_t rb = (size_t)h->ld * dtype_size(h->dtype);
        hipStream_t s = (hipStream_t)stream;
        RC_HIP(hipMemcpyAsync(rows_out, (const uint8_t *)h->rows + (size_t)row0 * rb, (size_t)n * rb, hipMemcpyDefault, s));
        RC_HIP(hipMemcpyAsync(norms_out, h->norms + row0, (size_t)n * sizeof(float), hipMemcpyDefault, s));
    });
}

int rc_index_import(rc_index *h, int64_t row0, int64_t n, const void *rows_in, const float *norms_in, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(row0 >= 0 && n >= 0 && row0 + n <= h->capacity, RC_ERR_INVALID, "rows out of capacity");
        if (n == 0) return;
        RC_REQUIRE(rows_in && norms_in, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        const size_t rb = (size_t)h->ld * dtype_size(h->dtype);
        hipStream_t s = (hipStream_t)stream;
        RC_HIP(hipMemcpyAsync((uint8_t *)h->rows + (size_t)row0 * rb, rows_in, (size_t)n * rb, hipMemcpyDefault, s));
        RC_HIP(hipMemcpyAsync(h->norms + row0, norms_in, (size_t)n * sizeof(float), hipMemcpyDefault, s));
        dispatch_dtype(h->dtype, [&](auto t) { launch_quantize<decltype(t)>(h, nullptr, row0, n, s); });
    });
}

int rc_index_search(rc_index *h, const float *queries, int nq, int64_t n_rows, int k, float *scores, int64_t *out_rows,
                    void *stream) {
    return rc_index_search_ex(h, queries, nq, n_rows, k, scores, out_rows, RC_SEARCH_AUTO, stream);
}

int rc_index_search_ex(rc_index *h, const float *queries, int nq, int64_t n_rows, int k, float *scores,
                       int64_t *out_rows, int mode, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(nq >= 0, RC_ERR_INVALID, "negative query count");
        RC_REQUIRE(k >= 1 && k <= RC_TOPK_MAX, RC_ERR_INVALID, "top_k must be in [1, 256]");
        RC_REQUIRE(n_rows >= 0 && n_rows <= h->capacity, RC_ERR_INVALID, "n_rows out of range");
        RC_REQUIRE(mode == RC_SEARCH_AUTO || mode == RC_SEARCH_SCAN || mode == RC_SEARCH_MFMA, RC_ERR_INVALID,
                   "unknown search mode");
        if (nq == 0) return;
        RC_REQUIRE(queries && scores && out_rows, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        hipStream_t s = (hipStream_t)stream;
        if (n_rows == 0) {  // an empty shard answers (-inf, -1) in every mode
            empty_search(nq, k, scores, out_rows, s);
            return;
        }
        const bool mfma_ok = h->dtype != RC_F32 || h->rows8 != nullptr;
        RC_REQUIRE(mode != RC_SEARCH_MFMA || mfma_ok, RC_ERR_UNSUPPORTED,
                   "batched MFMA search needs an f16/bf16 index or the int8 filter copy");
        const bool use_mfma = mode == RC_SEARCH_MFMA ||
                              (mode == RC_SEARCH_AUTO && mfma_ok && nq >= kBatchMinQueries && n_rows >= kBatchMinRows);
        if (!use_mfma) {
            scan_search(h, queries, nq, n_rows, k, scores, out_rows, s);
            return;
        }
        batched_search_exact(h, queries, nq, n_rows, k, scores, out_rows, s);
    });
}

int rc_topk_merge(const float *scores, const int64_t *rows, int nlists, int nq, int k_in, int k, float *out_scores,
                  int64_t *out_rows, void *stream) {
    return guard([&] {
        RC_REQUIRE(nlists >= 1 && nq >= 0 && k_in >= 1 && k >= 1 && k <= RC_TOPK_MAX, RC_ERR_INVALID, "bad merge sizes");
        if (nq == 0) return;
        hipStream_t s = (hipStream_t)stream;
        const int cap = topk_cap(k);
        if (cap <= 128)
            hipLaunchKernelGGL(merge_lists_kernel<128>, dim3(nq), dim3(256), 0, s, scores, rows, nlists, nq, k_in, k, out_scores, out_rows);
        else if (cap <= 256)
            hipLaunchKernelGGL(merge_lists_kernel<256>, dim3(nq), dim3(256), 0, s, scores, rows, nlists, nq, k_in, k, out_scores, out_rows);
        else
            hipLaunchKernelGGL(merge_lists_kernel<512>, dim3(nq), dim3(256), 0, s, scores, rows, nlists, nq, k_in, k, out_scores, out_rows);
        RC_LAUNCH_CHECK();
    });
}

int rc_index_timing(rc_index *h, int enable) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        if (enable) {
            h->timer.create();
            h->gtimer.create();
        }
        h->timer.enabled = enable != 0;
        h->gtimer.enabled = enable != 0;
    });
}

int rc_index_timing_read(rc_index *h, double *total_ms, int64_t *launches, double *bytes) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        h->timer.flush();
        if (total_ms) *total_ms = h->timer.total_ms;
        if (launches) *launches = h->timer.launches;
        if (bytes) *bytes = h->timer.work;
        h->timer.total_ms = 0;
        h->timer.launches = 0;
        h->timer.work = 0;
    });
}

int rc_index_gemm_timing_read(rc_index *h, double *total_ms, int64_t *launches, double *flops, int64_t *fallbacks) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        h->gtimer.flush();
        if (total_ms) *total_ms = h->gtimer.total_ms;
        if (launches) *launches = h->gtimer.launches;
        if (flops) *flops = h->gtimer.work;
        if (fallbacks) {
            int ovf = 0;
            if (h->bws.ovf) {
                RC_HIP(hipDeviceSynchronize());
                RC_HIP(hipMemcpy(&ovf, h->bws.ovf, sizeof(int), hipMemcpyDeviceToHost));
                RC_HIP(hipMemset(h->bws.ovf, 0, sizeof(int)));
            }
            *fallbacks = ovf;
        }
        h->gtimer.total_ms = 0;
        h->gtimer.launches = 0;
        h->gtimer.work = 0;
    });
}

}  // extern "C"
