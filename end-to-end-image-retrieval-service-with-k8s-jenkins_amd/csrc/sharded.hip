// sharded.hip — one exact cosine index spread over several shards in ONE process
// (rc_index_create(dim, dtype, capacity_per_gpu, n_gpus); §8(e)).
//
// The Pinecone index the reference opens in get_index (ingesting/utils.py:23-38)
// is one logical index whatever its size; here it is n shards, each an rc_index
// on its own GPU (or several on one GPU).  Routing is round-robin on the
// host-assigned global row g: shard g % n holds it as local row g / n, so rows
// fill every shard evenly from the first upsert on.  A shard returns global rows
// directly (rc_index row map: row_base = s, row_stride = n).
//
// query (retriever/utils.py:62-64): the leader stream's query batch is handed to
// every shard's stream (event wait; a peer copy over xGMI when the shard lives
// on another GPU), each shard runs its own scan / MFMA search over its n_local
// rows, its top-k lists land in a leader-side gather buffer (peer copies of
// nq*k*12 B), and merge_lists_kernel (rc_topk_merge) keys candidates by
// (score desc, global row asc) — the same order a single rc_index gives.
// A multi-PROCESS deployment (one process per GPU) uses the same shard row map
// with an RCCL all-gather instead (sharded.py).
#include <atomic>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "index_common.h"

namespace rc {
void index_upsert_gather(rc_index *h, const float *vecs, const int64_t *src_idx, int64_t n, const int64_t *rows,
                         hipStream_t s);
bool index_query1(rc_index *h, const float *query, int64_t n_rows, int k, int with_values, float *out_scores,
                  int64_t *out_rows, float *out_values, hipStream_t s, volatile unsigned **done = nullptr,
                  unsigned *seq = nullptr);

// Wait for query1's completion word instead of the stream: the word is stored after the results
// (system-scope release), so the host can read them the moment it changes, without the
// end-of-kernel signal round trip.  Every 256 polls the stream is queried, so a faulted or
// finished launch ends the wait too (a fault surfaces as the stream's error).
static void spin_until(volatile unsigned *word, unsigned want, hipStream_t s) {
    for (uint32_t it = 1;; ++it) {
        if (*word == want) return;
        if ((it & 255u) == 0u) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) {
                if (*word == want) return;
                RC_HIP(hipStreamSynchronize(s));
                return;
            }
            if (e != hipErrorNotReady) RC_HIP(e);
        }
        __builtin_ia32_pause();
    }
}

// dst[i][:] = src[idx[i]][:] (one wave per row): a remote shard's subset of an upsert
// batch, made contiguous on the leader so only those rows cross xGMI.
__global__ __launch_bounds__(256) void gather_rows_kernel(const float *__restrict__ src, const int64_t *__restrict__ idx,
                                                         int64_t m, int dim, float *__restrict__ dst) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= m) return;
    const float *s = src + idx[i] * dim;
    float *d = dst + i * dim;
    for (int c = lane; c < dim; c += 64) d[c] = s[c];
}
}

using namespace rc;

struct rc_sharded {
    std::mutex mu;
    int n = 0, dim = 0, dtype = 0;
    int64_t cap = 0;  // rows per shard
    std::vector<int> dev;
    // shard s is driven through the cross-device path (peer copies to / from the leader):
    // dev[s] != dev[0], or every shard s > 0 after rc_sharded_force_remote (a test hook: the
    // 8-GPU code path — gather, peer copies, leader merge — exercised on one GPU)
    std::vector<char> remote;
    std::vector<rc_index *> shard;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev_done;   // per shard, recorded on st[s]
    std::vector<hipEvent_t> ev_start;  // per shard, recorded on the caller's (leader) stream
    // search buffers
    int nq_cap = 0, k_cap = 0;
    std::vector<float *> q;       // [nq_cap][dim] query copy on a non-leader shard's device
    std::vector<float *> s_loc;   // [nq_cap][k_cap] a non-leader shard's own result
    std::vector<int64_t *> r_loc;
    float *g_s = nullptr;         // leader [n][nq_cap][k_cap] gathered lists
    int64_t *g_r = nullptr;
    // upsert / fetch staging (grown on demand, reused: no allocation in steady state)
    int64_t st_cap = 0;
    std::vector<int64_t *> idx_d;  // [st_cap] source index per shard (on the leader for a remote shard)
    std::vector<int64_t *> row_d;  // [st_cap] local row per shard (on the shard's device)
    std::vector<float *> vec_d;    // [st_cap][dim] a remote shard's subset of the batch, on its device
    std::vector<float *> gat_d;    // [st_cap][dim] that subset gathered on the leader (peer-copy source)
    std::vector<float *> fo_d;     // [st_cap][dim] fetched rows on the shard's device
    std::vector<int64_t *> idx_h;  // [st_cap] pinned host copies of the per-shard lists
    std::vector<int64_t *> row_h;
    std::vector<float *> fo_h;     // [st_cap][dim] pinned host landing of fetched rows
    hipEvent_t ev_gather = nullptr;  // leader stream: the remote subsets are gathered
    // host-in / host-out query (rc_sharded_query_host): its own leader stream, one pinned
    // staging block and one device block, each laid out [queries | scores | rows | values]
    hipStream_t qs = nullptr;
    int64_t qh_bytes = 0;
    uint8_t *qh = nullptr;  // pinned
    uint8_t *qd = nullptr;  // leader device
};

namespace {

void free_search(rc_sharded *h) {
    for (int s = 0; s < h->n; ++s) {
        DeviceScope ds(h->dev[s]);
        dfree(h->q[s]);
        dfree(h->s_loc[s]);
        dfree(h->r_loc[s]);
        h->q[s] = nullptr;
        h->s_loc[s] = nullptr;
        h->r_loc[s] = nullptr;
    }
    DeviceScope ds(h->dev[0]);
    dfree(h->g_s);
    dfree(h->g_r);
    h->g_s = nullptr;
    h->g_r = nullptr;
    h->nq_cap = h->k_cap = 0;
}

void ensure_search(rc_sharded *h, int nq, int k) {
    if (nq <= h->nq_cap && k <= h->k_cap) return;
    const int nq2 = std::max(nq, h->nq_cap), k2 = std::max(k, h->k_cap);
    free_search(h);
    for (int s = 0; s < h->n; ++s) {
        if (!h->remote[s]) continue;
        DeviceScope ds(h->dev[s]);
        h->q[s] = (float *)dmalloc((size_t)nq2 * h->dim * sizeof(float));
        h->s_loc[s] = (float *)dmalloc((size_t)nq2 * k2 * sizeof(float));
        h->r_loc[s] = (int64_t *)dmalloc((size_t)nq2 * k2 * sizeof(int64_t));
    }
    DeviceScope ds(h->dev[0]);
    h->g_s = (float *)dmalloc((size_t)h->n * nq2 * k2 * sizeof(float));
    h->g_r = (int64_t *)dmalloc((size_t)h->n * nq2 * k2 * sizeof(int64_t));
    h->nq_cap = nq2;
    h->k_cap = k2;
}

void free_staging(rc_sharded *h) {
    for (int s = 0; s < h->n; ++s) {
        DeviceScope ds(h->dev[s]);
        dfree(h->row_d[s]);
        dfree(h->vec_d[s]);
        dfree(h->fo_d[s]);
        hfree(h->idx_h[s]);
        hfree(h->row_h[s]);
        hfree(h->fo_h[s]);
        h->row_d[s] = nullptr;
        h->vec_d[s] = h->fo_d[s] = h->fo_h[s] = nullptr;
        h->idx_h[s] = h->row_h[s] = nullptr;
    }
    DeviceScope dl(h->dev[0]);
    for (int s = 0; s < h->n; ++s) {
        dfree(h->idx_d[s]);
        dfree(h->gat_d[s]);
        h->idx_d[s] = nullptr;
        h->gat_d[s] = nullptr;
    }
    h->st_cap = 0;
}

// Per shard, room for m rows of one call: index lists (pinned host + device), the
// remote shards' gathered subset (leader) and its landing (shard device), fetch
// buffers.  Grows geometrically, so a steady stream of calls allocates nothing.
void ensure_staging(rc_sharded *h, int64_t m) {
    if (m <= h->st_cap) return;
    const int64_t m2 = std::max<int64_t>(m, 2 * h->st_cap);
    free_staging(h);
    const size_t vb = (size_t)m2 * h->dim * sizeof(float);
    for (int s = 0; s < h->n; ++s) {
        const bool remote = h->remote[s];
        {
            DeviceScope ds(h->dev[s]);
            h->row_d[s] = (int64_t *)dmalloc((size_t)m2 * sizeof(int64_t));
            h->fo_d[s] = (float *)dmalloc(vb);
            if (remote) h->vec_d[s] = (float *)dmalloc(vb);
        }
        DeviceScope dl(h->dev[0]);  // the source index lists are read on the leader (gather / local upsert)
        h->idx_d[s] = (int64_t *)dmalloc((size_t)m2 * sizeof(int64_t));
        if (remote) h->gat_d[s] = (float *)dmalloc(vb);
        h->idx_h[s] = (int64_t *)hmalloc((size_t)m2 * sizeof(int64_t));
        h->row_h[s] = (int64_t *)hmalloc((size_t)m2 * sizeof(int64_t));
        h->fo_h[s] = (float *)hmalloc(vb);
    }
    h->st_cap = m2;
}

// rows of the global range [0, n_rows) that shard s holds
int64_t shard_rows(const rc_sharded *h, int s, int64_t n_rows) { return n_rows > s ? (n_rows - s + h->n - 1) / h->n : 0; }

void free_query(rc_sharded *h) {
    DeviceScope dl(h->dev[0]);
    hfree(h->qh);
    dfree(h->qd);
    h->qh = nullptr;
    h->qd = nullptr;
    h->qh_bytes = 0;
}

// offsets of the query block for nq queries, top-k, with or without values (16-B aligned parts)
struct QueryLayout {
    int64_t q, sc, rw, val, total;
};
QueryLayout query_layout(const rc_sharded *h, int nq, int k, bool values) {
    auto al = [](int64_t b) { return (b + 15) & ~(int64_t)15; };
    QueryLayout L;
    L.q = 0;
    L.sc = al((int64_t)nq * h->dim * 4);
    L.rw = L.sc + al((int64_t)nq * k * 4);
    L.val = L.rw + al((int64_t)nq * k * 8);
    L.total = L.val + (values ? al((int64_t)nq * k * h->dim * 4) : 0);
    return L;
}

void ensure_query(rc_sharded *h, int64_t bytes) {
    if (bytes <= h->qh_bytes) return;
    const int64_t b2 = std::max<int64_t>(bytes, 2 * h->qh_bytes);
    RC_HIP(hipStreamSynchronize(h->qs));
    free_query(h);
    DeviceScope dl(h->dev[0]);
    h->qh = (uint8_t *)hmalloc((size_t)b2);
    h->qd = (uint8_t *)dmalloc((size_t)b2);
    h->qh_bytes = b2;
}

void destroy(rc_sharded *h) {
    free_search(h);
    free_staging(h);
    if (h->qs) {
        free_query(h);
        DeviceScope dl(h->dev[0]);
        (void)hipStreamDestroy(h->qs);
    }
    for (int s = 0; s < h->n; ++s) {
        DeviceScope ds(h->dev[s]);
        if (h->st[s]) (void)hipStreamDestroy(h->st[s]);
        if (h->ev_done[s]) (void)hipEventDestroy(h->ev_done[s]);
        if (h->ev_start[s]) (void)hipEventDestroy(h->ev_start[s]);
        if (h->shard[s]) (void)rc_index_destroy(h->shard[s]);
    }
    if (h->ev_gather) {
        DeviceScope dl(h->dev[0]);
        (void)hipEventDestroy(h->ev_gather);
    }
    delete h;
}

void check_status(int st) {
    if (st != RC_OK) throw Error(st, rc_last_error());
}

}  // namespace

extern "C" {

int rc_sharded_create(int n_shards, const int *devices, int dim, int dtype, int64_t capacity_per_shard, rc_sharded **out) {
    return guard([&] {
        RC_REQUIRE(out && devices, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(n_shards >= 1 && n_shards <= 64, RC_ERR_INVALID, "n_shards must be in [1, 64]");
        RC_REQUIRE(capacity_per_shard > 0 && (double)capacity_per_shard * n_shards < 4294967296.0, RC_ERR_INVALID,
                   "total capacity must be in [1, 2^32) rows (global rows key the cross-shard merge)");
        auto *h = new rc_sharded();
        h->n = n_shards;
        h->dim = dim;
        h->dtype = dtype;
        h->cap = capacity_per_shard;
        h->dev.assign(devices, devices + n_shards);
        h->remote.assign(n_shards, 0);
        for (int s = 1; s < n_shards; ++s) h->remote[s] = devices[s] != devices[0] ? 1 : 0;
        h->shard.assign(n_shards, nullptr);
        h->st.assign(n_shards, nullptr);
        h->ev_done.assign(n_shards, nullptr);
        h->ev_start.assign(n_shards, nullptr);
        h->q.assign(n_shards, nullptr);
        h->s_loc.assign(n_shards, nullptr);
        h->r_loc.assign(n_shards, nullptr);
        h->idx_d.assign(n_shards, nullptr);
        h->row_d.assign(n_shards, nullptr);
        h->vec_d.assign(n_shards, nullptr);
        h->gat_d.assign(n_shards, nullptr);
        h->fo_d.assign(n_shards, nullptr);
        h->idx_h.assign(n_shards, nullptr);
        h->row_h.assign(n_shards, nullptr);
        h->fo_h.assign(n_shards, nullptr);
        try {
            for (int s = 0; s < n_shards; ++s) {
                check_status(rc_index_create(h->dev[s], dim, dtype, capacity_per_shard, s, &h->shard[s]));
                check_status(rc_index_set_row_map(h->shard[s], s, n_shards));
                DeviceScope ds(h->dev[s]);
                RC_HIP(hipStreamCreateWithFlags(&h->st[s], hipStreamNonBlocking));
                RC_HIP(hipEventCreateWithFlags(&h->ev_done[s], hipEventDisableTiming));
                if (h->dev[s] != h->dev[0]) {  // direct xGMI peer copies where the platform allows them
                    if (hipDeviceEnablePeerAccess(h->dev[0], 0) != hipSuccess) (void)hipGetLastError();
                    DeviceScope dl(h->dev[0]);
                    if (hipDeviceEnablePeerAccess(h->dev[s], 0) != hipSuccess) (void)hipGetLastError();
                }
            }
            DeviceScope dl(h->dev[0]);
            for (int s = 0; s < n_shards; ++s) RC_HIP(hipEventCreateWithFlags(&h->ev_start[s], hipEventDisableTiming));
            RC_HIP(hipEventCreateWithFlags(&h->ev_gather, hipEventDisableTiming));
            RC_HIP(hipStreamCreateWithFlags(&h->qs, hipStreamNonBlocking));
        } catch (...) {
            destroy(h);
            throw;
        }
        *out = h;
    });
}

int rc_sharded_destroy(rc_sharded *h) {
    return guard([&] {
        if (h) destroy(h);
    });
}

int rc_sharded_force_remote(rc_sharded *h) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        std::lock_guard<std::mutex> lk(h->mu);
        {
            DeviceScope dl(h->dev[0]);
            RC_HIP(hipDeviceSynchronize());  // nothing of the old routing is in flight
        }
        free_search(h);  // both are sized by the remote flags; regrown on the next call
        free_staging(h);
        for (int s = 1; s < h->n; ++s) h->remote[s] = 1;
    });
}

int rc_sharded_info(const rc_sharded *h, int *n_shards, int64_t *capacity_per_shard, int64_t *ld) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        if (n_shards) *n_shards = h->n;
        if (capacity_per_shard) *capacity_per_shard = h->cap;
        if (ld) check_status(rc_index_info(h->shard[0], nullptr, nullptr, nullptr, ld));
    });
}

int rc_sharded_shard(rc_sharded *h, int s, rc_index **out) {
    return guard([&] {
        RC_REQUIRE(h && out, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(s >= 0 && s < h->n, RC_ERR_INVALID, "shard out of range");
        *out = h->shard[s];
    });
}

int rc_sharded_grow(rc_sharded *h, int64_t new_capacity_per_shard) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE((double)new_capacity_per_shard * h->n < 4294967296.0, RC_ERR_INVALID, "total capacity must be < 2^32 rows");
        std::lock_guard<std::mutex> lk(h->mu);
        if (new_capacity_per_shard <= h->cap) return;
        for (int s = 0; s < h->n; ++s) check_status(rc_index_grow(h->shard[s], new_capacity_per_shard, h->st[s]));
        h->cap = new_capacity_per_shard;
    });
}

int rc_sharded_set_filter(rc_sharded *h, int kind) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        std::lock_guard<std::mutex> lk(h->mu);
        try {
            for (int s = 0; s < h->n; ++s) check_status(rc_index_set_filter(h->shard[s], kind, h->st[s]));
        } catch (...) {  // all or nothing: a failed shard (e.g. no room for the int8 copy) rolls every shard back
            for (int s = 0; s < h->n; ++s) (void)rc_index_set_filter(h->shard[s], RC_FILTER_NATIVE, h->st[s]);
            throw;
        }
    });
}

int rc_sharded_upsert(rc_sharded *h, const float *vecs, int64_t n, const int64_t *rows, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(n >= 0, RC_ERR_INVALID, "negative count");
        if (n == 0) return;
        RC_REQUIRE(vecs && rows, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        std::vector<int64_t> cnt(h->n, 0);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t g = rows[i];
            RC_REQUIRE(g >= 0 && g / h->n < h->cap, RC_ERR_INVALID, "row out of capacity");
            ++cnt[g % h->n];
        }
        int64_t m = 0;
        for (int s = 0; s < h->n; ++s) m = std::max<int64_t>(m, cnt[s]);
        ensure_staging(h, m);
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t i = 0; i < n; ++i) {  // per-shard (source index, local row) lists, pinned
            const int64_t g = rows[i];
            const int s = (int)(g % h->n);
            h->idx_h[s][cnt[s]] = i;
            h->row_h[s][cnt[s]] = g / h->n;
            ++cnt[s];
        }
        hipStream_t ls = (hipStream_t)stream;
        {
            // leader stream: source lists of every shard, then each remote shard's subset gathered
            // contiguous (cnt[s] rows, not the whole batch, cross xGMI)
            DeviceScope dl(h->dev[0]);
            for (int s = 0; s < h->n; ++s) {
                if (cnt[s] == 0) continue;
                RC_HIP(hipMemcpyAsync(h->idx_d[s], h->idx_h[s], cnt[s] * sizeof(int64_t), hipMemcpyHostToDevice, ls));
                if (h->remote[s]) {
                    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((cnt[s] + 3) / 4)), dim3(256), 0, ls, vecs,
                                       h->idx_d[s], cnt[s], h->dim, h->gat_d[s]);
                    RC_LAUNCH_CHECK();
                }
            }
            RC_HIP(hipEventRecord(h->ev_gather, ls));
        }
        for (int s = 0; s < h->n; ++s) {
            if (cnt[s] == 0) continue;
            DeviceScope ds(h->dev[s]);
            const int64_t ms = cnt[s];
            RC_HIP(hipStreamWaitEvent(h->st[s], h->ev_gather, 0));
            RC_HIP(hipMemcpyAsync(h->row_d[s], h->row_h[s], ms * sizeof(int64_t), hipMemcpyHostToDevice, h->st[s]));
            if (h->remote[s]) {
                RC_HIP(hipMemcpyPeerAsync(h->vec_d[s], h->dev[s], h->gat_d[s], h->dev[0], (size_t)ms * h->dim * sizeof(float),
                                          h->st[s]));
                index_upsert_gather(h->shard[s], h->vec_d[s], nullptr, ms, h->row_d[s], h->st[s]);
            } else {
                index_upsert_gather(h->shard[s], vecs, h->idx_d[s], ms, h->row_d[s], h->st[s]);
            }
        }
        // the pinned lists are reused by the next call: finish here (upsert is synchronous,
        // like the Pinecone call it replaces)
        for (int s = 0; s < h->n; ++s) {
            if (cnt[s] == 0) continue;
            DeviceScope ds(h->dev[s]);
            RC_HIP(hipStreamSynchronize(h->st[s]));
        }
    });
}

}  // extern "C"

namespace {

// rc_sharded_fetch's body (caller holds h->mu)
void fetch_locked(rc_sharded *h, const int64_t *rows, int64_t n, float *out, int stored) {
        std::vector<int64_t> cnt(h->n, 0);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t g = rows[i];
            RC_REQUIRE(g >= 0 && g / h->n < h->cap, RC_ERR_INVALID, "row out of capacity");
            ++cnt[g % h->n];
        }
        int64_t m = 0;
        for (int s = 0; s < h->n; ++s) m = std::max<int64_t>(m, cnt[s]);
        ensure_staging(h, m);
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t g = rows[i];
            const int s = (int)(g % h->n);
            h->idx_h[s][cnt[s]] = i;  // destination row of out
            h->row_h[s][cnt[s]] = g / h->n;
            ++cnt[s];
        }
        // every shard's fetch and D2H copy in flight at once, one wait at the end
        for (int s = 0; s < h->n; ++s) {
            if (cnt[s] == 0) continue;
            DeviceScope ds(h->dev[s]);
            const int64_t ms = cnt[s];
            RC_HIP(hipMemcpyAsync(h->row_d[s], h->row_h[s], ms * sizeof(int64_t), hipMemcpyHostToDevice, h->st[s]));
            check_status(stored ? rc_index_fetch_stored(h->shard[s], h->row_d[s], ms, h->fo_d[s], h->st[s])
                                : rc_index_fetch(h->shard[s], h->row_d[s], ms, h->fo_d[s], h->st[s]));
            RC_HIP(hipMemcpyAsync(h->fo_h[s], h->fo_d[s], (size_t)ms * h->dim * sizeof(float), hipMemcpyDeviceToHost,
                                  h->st[s]));
        }
        for (int s = 0; s < h->n; ++s) {
            if (cnt[s] == 0) continue;
            DeviceScope ds(h->dev[s]);
            RC_HIP(hipStreamSynchronize(h->st[s]));
            for (int64_t j = 0; j < cnt[s]; ++j)
                std::memcpy(out + h->idx_h[s][j] * h->dim, h->fo_h[s] + j * h->dim, (size_t)h->dim * sizeof(float));
        }
}

// rc_sharded_search's body (caller holds h->mu; device buffers on the leader, stream = leader stream)
void search_locked(rc_sharded *h, const float *queries, int nq, int64_t n_rows, int k, float *scores, int64_t *out_rows,
                   int mode, void *stream) {
        hipStream_t ls = (hipStream_t)stream;
        if (h->n == 1) {
            check_status(rc_index_search_ex(h->shard[0], queries, nq, n_rows, k, scores, out_rows, mode, stream));
            return;
        }
        ensure_search(h, nq, k);
        const int64_t slice = (int64_t)nq * k;
        {
            DeviceScope dl(h->dev[0]);
            for (int s = 0; s < h->n; ++s) RC_HIP(hipEventRecord(h->ev_start[s], ls));
        }
        for (int s = 0; s < h->n; ++s) {
            DeviceScope ds(h->dev[s]);
            RC_HIP(hipStreamWaitEvent(h->st[s], h->ev_start[s], 0));
            const bool local = !h->remote[s];
            const float *q = queries;
            if (!local) {
                RC_HIP(hipMemcpyPeerAsync(h->q[s], h->dev[s], queries, h->dev[0], (size_t)nq * h->dim * sizeof(float), h->st[s]));
                q = h->q[s];
            }
            float *so = local ? h->g_s + s * slice : h->s_loc[s];
            int64_t *ro = local ? h->g_r + s * slice : h->r_loc[s];
            check_status(rc_index_search_ex(h->shard[s], q, nq, shard_rows(h, s, n_rows), k, so, ro, mode, h->st[s]));
            if (!local) {
                RC_HIP(hipMemcpyPeerAsync(h->g_s + s * slice, h->dev[0], so, h->dev[s], slice * sizeof(float), h->st[s]));
                RC_HIP(hipMemcpyPeerAsync(h->g_r + s * slice, h->dev[0], ro, h->dev[s], slice * sizeof(int64_t), h->st[s]));
            }
            RC_HIP(hipEventRecord(h->ev_done[s], h->st[s]));
        }
        DeviceScope dl(h->dev[0]);
        for (int s = 0; s < h->n; ++s) RC_HIP(hipStreamWaitEvent(ls, h->ev_done[s], 0));
        check_status(rc_topk_merge(h->g_s, h->g_r, h->n, nq, k, k, scores, out_rows, stream));
}

}  // namespace

extern "C" {

int rc_sharded_fetch(rc_sharded *h, const int64_t *rows, int64_t n, float *out, int stored) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(n >= 0, RC_ERR_INVALID, "negative count");
        if (n == 0) return;
        RC_REQUIRE(rows && out, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        fetch_locked(h, rows, n, out, stored);
    });
}

int rc_sharded_search(rc_sharded *h, const float *queries, int nq, int64_t n_rows, int k, float *scores,
                      int64_t *out_rows, int mode, void *stream) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(nq >= 0, RC_ERR_INVALID, "negative query count");
        RC_REQUIRE(k >= 1 && k <= RC_TOPK_MAX, RC_ERR_INVALID, "top_k must be in [1, 256]");
        RC_REQUIRE(n_rows >= 0 && n_rows <= h->cap * h->n, RC_ERR_INVALID, "n_rows out of range");
        if (nq == 0) return;
        RC_REQUIRE(queries && scores && out_rows, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(h->mu);
        search_locked(h, queries, nq, n_rows, k, scores, out_rows, mode, stream);
    });
}

int rc_sharded_query_host(rc_sharded *h, const float *queries, int nq, int64_t n_rows, int k, int with_values,
                          float *scores, int64_t *out_rows, float *values) {
    return guard([&] {
        RC_REQUIRE(h, RC_ERR_INVALID, "null index");
        RC_REQUIRE(nq >= 0, RC_ERR_INVALID, "negative query count");
        RC_REQUIRE(k >= 1 && k <= RC_TOPK_MAX, RC_ERR_INVALID, "top_k must be in [1, 256]");
        RC_REQUIRE(n_rows >= 0 && n_rows <= h->cap * h->n, RC_ERR_INVALID, "n_rows out of range");
        if (nq == 0) return;
        RC_REQUIRE(queries && scores && out_rows && (!with_values || values), RC_ERR_INVALID, "null buffer");
        const int64_t nk = (int64_t)nq * k;
        if (n_rows == 0) {  // an empty index: empty lists, no device work
            std::fill(scores, scores + nk, -INFINITY);
            std::fill(out_rows, out_rows + nk, (int64_t)-1);
            return;
        }
        std::lock_guard<std::mutex> lk(h->mu);
        // one shard: the matched rows' values are gathered on the device and come back in the
        // same copy as the lists; several shards: values through the staged fetch afterwards
        const bool dev_values = with_values && h->n == 1;
        const QueryLayout L = query_layout(h, nq, k, dev_values);
        ensure_query(h, L.total);
        DeviceScope dl(h->dev[0]);
        if (h->n == 1 && nq == 1) {
            // the request path: one launch pair (query in the kernel arguments, results written
            // straight into the pinned block), no copies; the host polls the completion word
            float *hs = (float *)(h->qh + L.sc);
            int64_t *hr = (int64_t *)(h->qh + L.rw);
            float *hv = (float *)(h->qh + L.val);
            volatile unsigned *word = nullptr;
            unsigned want = 0;
            if (index_query1(h->shard[0], queries, n_rows, k, with_values, hs, hr, hv, h->qs, &word, &want)) {
                spin_until(word, want, h->qs);
                std::atomic_thread_fence(std::memory_order_acquire);  // the result reads stay below
                std::memcpy(scores, hs, (size_t)k * sizeof(float));
                std::memcpy(out_rows, hr, (size_t)k * sizeof(int64_t));
                if (with_values) std::memcpy(values, hv, (size_t)k * h->dim * sizeof(float));
                return;
            }
        }
        std::memcpy(h->qh + L.q, queries, (size_t)nq * h->dim * sizeof(float));
        RC_HIP(hipMemcpyAsync(h->qd + L.q, h->qh + L.q, (size_t)nq * h->dim * sizeof(float), hipMemcpyHostToDevice, h->qs));
        float *dsc = (float *)(h->qd + L.sc);
        int64_t *drw = (int64_t *)(h->qd + L.rw);
        search_locked(h, (const float *)(h->qd + L.q), nq, n_rows, k, dsc, drw, RC_SEARCH_AUTO, h->qs);
        if (dev_values) check_status(rc_index_fetch(h->shard[0], drw, nk, (float *)(h->qd + L.val), h->qs));
        RC_HIP(hipMemcpyAsync(h->qh + L.sc, h->qd + L.sc, (size_t)(L.total - L.sc), hipMemcpyDeviceToHost, h->qs));
        RC_HIP(hipStreamSynchronize(h->qs));
        std::memcpy(scores, h->qh + L.sc, (size_t)nk * sizeof(float));
        std::memcpy(out_rows, h->qh + L.rw, (size_t)nk * sizeof(int64_t));
        if (dev_values) {
            std::memcpy(values, h->qh + L.val, (size_t)nk * h->dim * sizeof(float));
        } else if (with_values) {
            std::vector<int64_t> live;
            std::vector<int64_t> at;
            for (int64_t i = 0; i < nk; ++i)
                if (out_rows[i] >= 0) {
                    live.push_back(out_rows[i]);
                    at.push_back(i);
                } else {
                    std::fill(values + i * h->dim, values + (i + 1) * h->dim, NAN);
                }
            if (!live.empty()) {
                std::vector<float> tmp(live.size() * (size_t)h->dim);
                fetch_locked(h, live.data(), (int64_t)live.size(), tmp.data(), 0);
                for (size_t j = 0; j < live.size(); ++j)
                    std::memcpy(values + at[j] * h->dim, tmp.data() + j * h->dim, (size_t)h->dim * sizeof(float));
            }
        }
    });
}

}  // extern "C"
