// index_common.h — storage dtypes and the single-query streaming scan
// (HBM-bound GEMV + fused wavefront top-k) of the exact cosine index.
// The scan is instantiated per storage dtype in scan_{f32,f16,bf16}.hip so
// the three translation units compile in parallel.
#pragma once

#include "rc_common.h"
#include "topk.h"

namespace rc {

struct f16_t { uint16_t b; };
struct bf16_t { uint16_t b; };

template <typename T> struct Elem;
template <> struct Elem<float> {
    __device__ static float load(const float *p, int64_t i) { return p[i]; }
    __device__ static float cast(float x) { return x; }
};
template <> struct Elem<f16_t> {
    __device__ static float load(const f16_t *p, int64_t i) { return f16_to_f32(p[i].b); }
    __device__ static f16_t cast(float x) { return f16_t{f32_to_f16(x)}; }
};
template <> struct Elem<bf16_t> {
    __device__ static float load(const bf16_t *p, int64_t i) { return bf16_to_f32(p[i].b); }
    __device__ static bf16_t cast(float x) { return bf16_t{f32_to_bf16(x)}; }
};

inline size_t dtype_size(int dtype) { return dtype == RC_F32 ? 4 : 2; }

// unpack one 16-B chunk into its 4 (f32) or 8 (f16/bf16) values
template <typename T>
__device__ __forceinline__ void unpack16(const uint4 &x, float *out);
template <>
__device__ __forceinline__ void unpack16<float>(const uint4 &x, float *o) {
    o[0] = __uint_as_float(x.x);
    o[1] = __uint_as_float(x.y);
    o[2] = __uint_as_float(x.z);
    o[3] = __uint_as_float(x.w);
}
template <>
__device__ __forceinline__ void unpack16<f16_t>(const uint4 &x, float *o) {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = f16_to_f32((uint16_t)(w[i] & 0xffffu));
        o[2 * i + 1] = f16_to_f32((uint16_t)(w[i] >> 16));
    }
}
template <>
__device__ __forceinline__ void unpack16<bf16_t>(const uint4 &x, float *o) {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w[i] << 16);
        o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

inline int topk_cap(int k) {
    int kp = 16;
    while (kp < k) kp <<= 1;
    return kp * 2 < 128 ? 128 : kp * 2;
}

struct ScanArgs {
    const void *rows;
    int64_t ld;
    int nch;
    int64_t n_rows;
    int64_t rows_per_block;
    int nblk;
    const float *qn;
    int q0;
    int qb;
    int nq_total;
    int k;
    uint64_t *partial;
    hipStream_t stream;
    // Exact fallback of the batched search: when set, grid.y strides over the
    // queries [0, nq_total) and only queries with flags[q] != 0 are scanned
    // (qb = 1; q0 unused); partial is then [nblk][nq_total][k].
    const int *flags = nullptr;
    int grid_y = 1;
    // Single-query scans (scan_search): the raw queries [nq_real][dim]; every wave normalises its
    // query itself, with normalize_queries_kernel's exact arithmetic (no separate launch), and
    // qn is not read.  nullptr: qn holds the normalised queries.
    const float *qraw = nullptr;
    int dim = 0, nq_real = 0;
};

// largest queries-per-pass for a row width: query registers per lane = QB*nch*8 floats <= 64
inline int scan_max_qb(int nch, int k) {
    if (k > 128) return 1;
    return nch <= 2 ? 4 : (nch <= 4 ? 2 : 1);
}

void launch_scan_f32(const ScanArgs &a);
void launch_scan_f16(const ScanArgs &a);
void launch_scan_bf16(const ScanArgs &a);

// One query, one launch (rc_sharded_query_host's request path): query1_kernel normalises the
// query (carried in the kernel arguments: no copy), scans its block's rows, and the last block
// to finish merges every block's partial list and gathers the matched rows' values, writing
// scores / rows / values straight into (host-mapped) output memory.
constexpr int QUERY1_MAX_DIM = 768;       // the query rides in the kernarg segment (< 4 KB); a multiple of 256
constexpr int QUERY1_MAX_BLOCKS = 256;    // partial lists the last block merges, at most
constexpr int64_t QUERY1_MAX_ROWS = 1 << 20;  // beyond this the multi-kernel scan has more blocks in flight
struct Query1Args {
    const void *rows;
    const float *norms;
    int64_t ld;
    int dim;
    int nch;
    int64_t n_rows;
    int64_t rows_per_block;
    int nblk;
    int k;
    int with_values;
    int64_t row_base, row_stride;
    uint64_t *partial;      // [nblk][k]
    float *out_scores;      // [k]
    int64_t *out_rows;      // [k]
    float *out_values;      // [k][dim] (with_values)
    unsigned *done;         // optional host-coherent word: the finishing block stores seq there last
    unsigned seq;
    float q[QUERY1_MAX_DIM];
};
void launch_query1_f32(const Query1Args &a, hipStream_t s);
void launch_query1_f16(const Query1Args &a, hipStream_t s);
void launch_query1_bf16(const Query1Args &a, hipStream_t s);

// Merge nlist sorted partial lists of k keys (query qi of nq_total) into wave 0's tk: the body
// of merge_partials_kernel, shared with query1_kernel's last block.  Block-collective.
template <int CAP>
__device__ __forceinline__ void merge_partial_lists(const uint64_t *__restrict__ partial, int nlist, int nq_total, int qi, int k,
                                                    uint64_t (&lds)[4][CAP], WaveTopK<CAP> &tk) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    tk.init(as_lds(&lds[wave][0]), k);
    const int64_t total = (int64_t)nlist * k;
    // MERGE_U independent loads in flight per lane before any is consumed: the
    // loop is latency-bound otherwise (one dependent HBM/L2 round trip per 64 keys)
    constexpr int MERGE_U = 8;
    for (int64_t j0 = (int64_t)wave * 64 * MERGE_U; j0 < total; j0 += 256 * MERGE_U) {
        uint64_t key[MERGE_U];
#pragma unroll
        for (int u = 0; u < MERGE_U; ++u) {
            const int64_t j = j0 + u * 64 + lane;
            key[u] = KEY_EMPTY;
            if (j < total) {
                const int64_t l = j / k, t = j - l * k;
                key[u] = partial[(l * nq_total + qi) * k + t];
            }
        }
#pragma unroll
        for (int u = 0; u < MERGE_U; ++u) {
            tk.reserve(64);
            tk.push(key[u] != KEY_EMPTY, key[u]);
        }
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
    }
}

// ------------------------------------------- batched MFMA search (search_mfma.hip)
constexpr int BATCH_CAND_CAP = 4096;  // candidate slots per query per stage
constexpr int INDEX_ROW_PAD = 256;    // row storage is allocated in whole 256-row tiles
constexpr int FB_BLOCKS = 256;        // blocks of the on-device exact fallback scan (overflowed queries), at most
constexpr int FB_MIN_BLOCKS = 32;     // ... and at least, whatever the memory budget below says
constexpr int64_t FB_BUDGET_BYTES = int64_t(256) << 20;  // cap on its partial-key buffer per index
constexpr int FB_QSTRIDE = 64;        // its grid.y: block (b, y) scans queries y, y + 64, ... that overflowed

struct BatchWs {
    int nq_cap = 0, k_cap = 0;
    int64_t ld_cap = 0;
    int cap = BATCH_CAND_CAP;
    float *qn = nullptr;        // [nq_cap][ld] normalised queries (f32)
    void *qh = nullptr;         // [nq_cap][ld] queries in the storage dtype (MFMA operand)
    float *eps = nullptr;       // [nq_cap] bound on |s' - s|
    float *thr = nullptr;       // [nq_cap] current filter threshold
    uint32_t *cnt = nullptr;    // [nq_cap] candidates appended this stage
    uint32_t *cand = nullptr;   // [nq_cap][cap] candidate rows
    uint64_t *keys = nullptr;   // [nq_cap][k_cap] running top-k keys (sorted)
    int *flags = nullptr;       // [nq_cap] 1 = candidate overflow, exact fallback needed
    float *sq = nullptr;        // [nq_cap] int8 filter: query scale (q̃ = sq · q8)
    float *aq = nullptr;        // [nq_cap] int8 filter: coefficient of a row's residual norm in the bound
    int *ovf = nullptr;         // overflowed queries since the last timing read (device counter)
    int fb_blocks = 0;               // blocks of the fallback scan: FB_BUDGET_BYTES / (nq_cap * k_cap * 8), clamped
    uint64_t *fb_partial = nullptr;  // [fb_blocks][nq_cap][k_cap] partial keys of the exact fallback scan
    void ensure(int nq, int k, int64_t ld, int dtype_bytes);
    void release();
};

struct BatchPlan {
    const void *rows;
    int dtype;
    int dim;
    int nch;
    int64_t ld;
    int64_t n_rows;
    int64_t row_base;      // returned row = row_base + local row * row_stride
    int64_t row_stride;
    const float *queries;  // device f32 [nq][dim]
    int nq;
    int k;
    float *out_scores;
    int64_t *out_rows;
    // int8 filter copy of the rows (rc_index_set_filter(RC_FILTER_I8)), or null
    const int8_t *rows8 = nullptr;  // [cap_pad][ld] x8, x̃ = sx · x8
    const float *rsx = nullptr;     // [cap_pad] sx, at i8_slot(row)
    const float *rex = nullptr;     // [cap_pad] ||x̂ - x̃||₂ (rounded up), at i8_slot(row)
};

// The int8 filter keeps a row's scale and residual norm at a tile-transposed slot:
// within each 128-row tile, row 16·rf + li sits at 8·li + rf, so the filter lane that
// holds rows {16·rf + li : rf} reads its 8 values as two 16-B loads.
__host__ __device__ __forceinline__ int64_t i8_slot(int64_t row) {
    return (row & ~int64_t(127)) + (row & 15) * 8 + ((row & 127) >> 4);
}
bool i8_filter_supported(int64_t ld);  // row widths filter_i8_kernel is instantiated for

// Enqueue the staged filter-GEMM / rescore search on `s` (no host sync).
void batched_search(const BatchPlan &p, BatchWs &ws, hipStream_t s, KernelTimer *timer);
int batch_stage_ratio(int k, int cap, int inflation = 1);

#if defined(SCAN_INSTANTIATE)
// qn holds nq_total (a multiple of QB) query rows, zero beyond the caller's
// queries, so every slot is computed and stored unconditionally.
// Block = 4 waves over a contiguous row range.  Lane = (row-in-group rg = lane>>4,
// position sub = lane&15); 16-B chunk j = sub + 16 i of a row holds elements
// [j*EPC, (j+1)*EPC).  SCAN_U row-groups are loaded before any is consumed.
constexpr int SCAN_U = 2;

typedef uint32_t u32x4_nt __attribute__((ext_vector_type(4)));  // the nontemporal load's operand type

// One block's pass over its row range for queries [q0, q0 + QB): partial top-k keys.
template <typename T, int NCH>
struct ScanShape {
    static constexpr int EPC = 16 / sizeof(T);           // values per 16-B chunk
    static constexpr int CPL = NCH * 128 / (16 * EPC);   // chunks per lane
};

// One block's pass over its row range for the QB queries held in registers q (lane sub's
// chunks sub + 16 i): partial top-k keys of queries q0 .. q0 + QB.
template <typename T, int NCH, int QB, int CAP>
__device__ __forceinline__ void scan_rows_q(const T *__restrict__ rows, int64_t ld, int64_t n_rows, int64_t rows_per_block,
                                            const float (&q)[QB][ScanShape<T, NCH>::CPL][ScanShape<T, NCH>::EPC], int q0,
                                            int nq_total, int k, uint64_t *__restrict__ partial) {
    constexpr int EPC = ScanShape<T, NCH>::EPC;
    constexpr int CPL = ScanShape<T, NCH>::CPL;
    __shared__ uint64_t lds[4][QB][CAP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane & 15, rg = lane >> 4;

    WaveTopK<CAP> tk[QB];
    static_for<QB>([&](auto bc) { tk[bc.value].init(as_lds(&lds[wave][bc.value][0]), k); });

    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(n_rows, r0 + rows_per_block);
    const uint4 *base4 = reinterpret_cast<const uint4 *>(rows);
    const int64_t ld4 = ld / EPC;  // row stride in 16-B chunks

    for (int64_t g = r0 + wave * 4 * SCAN_U; g < r1; g += 16 * SCAN_U) {
        uint4 x[SCAN_U][CPL];
#pragma unroll
        for (int u = 0; u < SCAN_U; ++u) {
            const int64_t r = g + u * 4 + rg;
            const int64_t rr = r < r1 ? r : r0;  // clamp to a valid row; result discarded below
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                // nontemporal: the rows stream through once (scan lab, 1M x 512 f32: 6.2 -> 7.0 TB/s)
                const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt *>(base4 + rr * ld4 + sub + 16 * i));
                x[u][i] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
#pragma unroll
        for (int u = 0; u < SCAN_U; ++u) {
            const int64_t r = g + u * 4 + rg;
            float acc[QB];
#pragma unroll
            for (int b = 0; b < QB; ++b) acc[b] = 0.f;
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                float f[EPC];
                unpack16<T>(x[u][i], f);
#pragma unroll
                for (int e = 0; e < EPC; ++e)
#pragma unroll
                    for (int b = 0; b < QB; ++b) acc[b] = fmaf(f[e], q[b][i][e], acc[b]);
            }
            static_for<QB>([&](auto bc) {
                constexpr int b = bc.value;
                const float s = sum16(acc[b]);
                tk[b].reserve(4);
                tk[b].push(sub == 0 && r < r1, make_key(s, (uint32_t)r));
            });
        }
    }

    // per-wave final selection, then wave 0 merges the other three waves' lists
    static_for<QB>([&](auto bc) { tk[bc.value].compact(); });
    __syncthreads();
    if (wave == 0) {
        static_for<QB>([&](auto bc) {
            constexpr int b = bc.value;
            const int qi = q0 + b;
            for (int w = 1; w < 4; ++w) {
                const lds_u64 *src = as_lds(&lds[w][b][0]);
                for (int j = 0; j < k; j += 64) {
                    const uint64_t key = (j + lane < k) ? src[j + lane] : KEY_EMPTY;
                    tk[b].reserve(64);
                    tk[b].push(key != KEY_EMPTY, key);
                }
            }
            tk[b].compact();
            uint64_t *dst = partial + ((int64_t)blockIdx.x * nq_total + qi) * k;
            for (int j = lane; j < k; j += 64) dst[j] = tk[b].buf[j];
        });
    }
}

template <typename T, int NCH, int QB, int CAP>
__device__ __forceinline__ void scan_rows(const T *__restrict__ rows, int64_t ld, int64_t n_rows, int64_t rows_per_block,
                                          const float *__restrict__ qn, int q0, int nq_total, int k,
                                          uint64_t *__restrict__ partial, const float *__restrict__ qraw = nullptr,
                                          int dim = 0, int nq_real = 0) {
    constexpr int EPC = ScanShape<T, NCH>::EPC;
    constexpr int CPL = ScanShape<T, NCH>::CPL;
    const int lane = threadIdx.x & 63, sub = lane & 15;
    float q[QB][CPL][EPC];
    if (qraw != nullptr) {  // block-uniform: normalise in the wave, as normalize_queries_kernel does
#pragma unroll
        for (int b = 0; b < QB; ++b) {
            const bool valid = q0 + b < nq_real;
            const float *src = qraw + (int64_t)(valid ? q0 + b : 0) * dim;
            float ss = 0.f;
            for (int c = lane; c < dim; c += 64) ss = valid ? fmaf(src[c], src[c], ss) : 0.f;
            ss = wave_sum(ss);
            const float inv = ss > 0.f ? 1.0f / sqrtf(ss) : 0.f;
#pragma unroll
            for (int i = 0; i < CPL; ++i)
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const int c = (sub + 16 * i) * EPC + e;
                    q[b][i][e] = (valid && c < dim) ? src[c] * inv : 0.f;
                }
        }
    } else {
#pragma unroll
        for (int b = 0; b < QB; ++b)
#pragma unroll
            for (int i = 0; i < CPL; ++i)
#pragma unroll
                for (int e = 0; e < EPC; ++e) q[b][i][e] = qn[(int64_t)(q0 + b) * ld + (sub + 16 * i) * EPC + e];
    }
    scan_rows_q<T, NCH, QB, CAP>(rows, ld, n_rows, rows_per_block, q, q0, nq_total, k, partial);
}

// f32 rows of 512 (config 3): 131 VGPRs by default = 3 waves per SIMD; capped at 128 (no spill)
// the CU holds 4 blocks and a 1M-row scan runs as one round of 4 blocks per CU
template <typename T, int NCH, int QB, int CAP>
constexpr int scan_min_waves() { return (sizeof(T) == 4 && NCH == 4 && QB == 1 && CAP <= 256) ? 4 : 1; }

template <typename T, int NCH, int QB, int CAP>
__global__ __launch_bounds__(256, (scan_min_waves<T, NCH, QB, CAP>())) void scan_topk_kernel(const T *__restrict__ rows, int64_t ld, int64_t n_rows,
                                                       int64_t rows_per_block, const float *__restrict__ qn, int q0,
                                                       int nq_total, int k, uint64_t *__restrict__ partial,
                                                       const int *__restrict__ flags, const float *__restrict__ qraw,
                                                       int dim, int nq_real) {
    if (flags != nullptr) {  // exact fallback: the overflowed queries only (block-uniform branches)
        for (int qf = blockIdx.y; qf < nq_total; qf += gridDim.y)
            if (flags[qf]) {
                scan_rows<T, NCH, QB, CAP>(rows, ld, n_rows, rows_per_block, qn, qf, nq_total, k, partial);
                __syncthreads();  // the next query reuses the LDS lists
            }
        return;
    }
    scan_rows<T, NCH, QB, CAP>(rows, ld, n_rows, rows_per_block, qn, q0, nq_total, k, partial, qraw, dim, nq_real);
}

template <typename T, int NCH, int QB, int CAP>
void launch_scan_t(const ScanArgs &a) {
    hipLaunchKernelGGL((scan_topk_kernel<T, NCH, QB, CAP>), dim3(a.nblk, a.grid_y), dim3(256), 0, a.stream, (const T *)a.rows,
                       a.ld, a.n_rows, a.rows_per_block, a.qn, a.q0, a.nq_total, a.k, a.partial, a.flags, a.qraw, a.dim,
                       a.nq_real);
    RC_LAUNCH_CHECK();
}

template <typename T, int NCH, int QB>
void launch_scan_cap(const ScanArgs &a) {
    const int cap = topk_cap(a.k);
    if (cap <= 128) return launch_scan_t<T, NCH, QB, 128>(a);
    if (cap <= 256) return launch_scan_t<T, NCH, QB, 256>(a);
    if constexpr (QB == 1) return launch_scan_t<T, NCH, QB, 512>(a);
    throw Error(RC_ERR_UNSUPPORTED, "multi-query pass needs k <= 128");
}

template <typename T, int NCH>
void launch_scan_qb(const ScanArgs &a) {
    if constexpr (NCH <= 2) {
        if (a.qb == 4) return launch_scan_cap<T, NCH, 4>(a);
    }
    if constexpr (NCH <= 4) {
        if (a.qb == 2) return launch_scan_cap<T, NCH, 2>(a);
    }
    if (a.qb == 1) return launch_scan_cap<T, NCH, 1>(a);
    throw Error(RC_ERR_INVALID, "internal: no scan instantiation for this queries-per-pass");
}

template <typename T>
void launch_scan_dtype(const ScanArgs &a) {
    switch (a.nch) {
        case 1: return launch_scan_qb<T, 1>(a);
        case 2: return launch_scan_qb<T, 2>(a);
        case 3: return launch_scan_qb<T, 3>(a);
        case 4: return launch_scan_qb<T, 4>(a);
        case 6: return launch_scan_qb<T, 6>(a);
        case 8: return launch_scan_qb<T, 8>(a);
        case 12: return launch_scan_qb<T, 12>(a);
        case 16: return launch_scan_qb<T, 16>(a);
        default: throw Error(RC_ERR_UNSUPPORTED, "unsupported row width");
    }
}

// rc_sharded_query_host's single-query launch pair (see Query1Args).  Every wave normalises the
// query exactly as normalize_queries_kernel does (same lane partition of the sum of squares,
// same wave_sum, same products), so scores are bit-identical to the multi-kernel path; the
// top-k of a total order does not depend on how rows are split over blocks.  PHASE 1: the scan
// blocks, each writing its partial list; PHASE 2: one block merges them (the kernel boundary
// orders the lists: a one-launch form with a last-block ticket behind device-scope fences
// measured 5.6 us slower per 10k-row call, round 4) and gathers the values.
template <typename T, int NCH, int CAP>
__device__ __forceinline__ void query1_scan(const Query1Args &a) {
    constexpr int EPC = ScanShape<T, NCH>::EPC;
    constexpr int CPL = ScanShape<T, NCH>::CPL;
    const int lane = threadIdx.x & 63, sub = lane & 15;
    // the kernarg segment may sit in host memory: one round of independent loads into LDS
    // (no branches), then every read is local
    __shared__ float qs[QUERY1_MAX_DIM];
    {
        constexpr int PER = QUERY1_MAX_DIM / 256;
        float v[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = a.q[threadIdx.x + 256 * i];
#pragma unroll
        for (int i = 0; i < PER; ++i) qs[threadIdx.x + 256 * i] = v[i];
    }
    __syncthreads();
    float ss = 0.f;
    for (int c = lane; c < a.dim; c += 64) ss = fmaf(qs[c], qs[c], ss);
    ss = wave_sum(ss);
    const float inv = ss > 0.f ? 1.0f / sqrtf(ss) : 0.f;
    float q[1][CPL][EPC];
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            const int c = (sub + 16 * i) * EPC + e;
            q[0][i][e] = c < a.dim ? qs[c] * inv : 0.f;
        }
    scan_rows_q<T, NCH, 1, CAP>((const T *)a.rows, a.ld, a.n_rows, a.rows_per_block, q, 0, 1, a.k, a.partial);
}

template <typename T, int CAP>
__device__ __forceinline__ void query1_finish(const Query1Args &a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint64_t lds[4][CAP];
    WaveTopK<CAP> tk;
    merge_partial_lists<CAP>(a.partial, a.nblk, 1, 0, a.k, lds, tk);
    __shared__ uint64_t best[CAP];
    if (wave == 0) {
        for (int j = lane; j < a.k; j += 64) {
            const uint64_t key = tk.buf[j];
            const bool ok = key != KEY_EMPTY;
            best[j] = key;
            a.out_scores[j] = ok ? key_score(key) : -INFINITY;
            a.out_rows[j] = ok ? a.row_base + (int64_t)key_idx(key) * a.row_stride : -1;
        }
    }
    __syncthreads();
    if (a.with_values) {  // fetch_kernel's arithmetic: stored row x norm, NaN for an empty slot
        const T *rows = (const T *)a.rows;
        for (int j = wave; j < a.k; j += 4) {
            const uint64_t key = best[j];
            float *dst = a.out_values + (int64_t)j * a.dim;
            if (key == KEY_EMPTY) {
                for (int c = lane; c < a.dim; c += 64) dst[c] = __builtin_nanf("");
            } else {
                const int64_t r = key_idx(key);
                const float nrm = a.norms[r];
                if ((a.dim & 3) == 0) {  // 16-B stores: a quarter of the write transactions to host memory
                    for (int c = 4 * lane; c < a.dim; c += 256) {
                        const int64_t o = r * a.ld + c;
                        *reinterpret_cast<float4 *>(dst + c) =
                            make_float4(Elem<T>::load(rows, o) * nrm, Elem<T>::load(rows, o + 1) * nrm,
                                        Elem<T>::load(rows, o + 2) * nrm, Elem<T>::load(rows, o + 3) * nrm);
                    }
                } else {
                    for (int c = lane; c < a.dim; c += 64) dst[c] = Elem<T>::load(rows, r * a.ld + c) * nrm;
                }
            }
        }
    }
    if (a.done != nullptr) {  // completion word for a host that polls instead of synchronising
        // Every wave releases its OWN result stores to system scope (a workgroup barrier does not
        // wait for another wave's outstanding stores), then the barrier, then one lane publishes.
        // The explicit vmcnt waits stay in inline asm: hipcc may drop a fence's own wait when it
        // believes the store counter is already empty (MI355X_MICROARCH.md, compiler hazard).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __threadfence_system();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.done, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename T, int NCH, int CAP, int PHASE>
__global__ __launch_bounds__(256) void query1_kernel(const Query1Args a) {
    if constexpr (PHASE == 2) query1_finish<T, CAP>(a);
    else query1_scan<T, NCH, CAP>(a);
}

template <typename T, int NCH, int CAP>
void launch_query1_phases(const Query1Args &a, hipStream_t s) {
    hipLaunchKernelGGL((query1_kernel<T, NCH, CAP, 1>), dim3(a.nblk), dim3(256), 0, s, a);
    RC_LAUNCH_CHECK();
    hipLaunchKernelGGL((query1_kernel<T, NCH, CAP, 2>), dim3(1), dim3(256), 0, s, a);
    RC_LAUNCH_CHECK();
}

template <typename T, int NCH>
void launch_query1_cap(const Query1Args &a, hipStream_t s) {
    const int cap = topk_cap(a.k);
    if (cap <= 128) launch_query1_phases<T, NCH, 128>(a, s);
    else if (cap <= 256) launch_query1_phases<T, NCH, 256>(a, s);
    else throw Error(RC_ERR_UNSUPPORTED, "single-query launch needs k <= 128");
}

template <typename T>
void launch_query1_dtype(const Query1Args &a, hipStream_t s) {
    switch (a.nch) {
        case 1: return launch_query1_cap<T, 1>(a, s);
        case 2: return launch_query1_cap<T, 2>(a, s);
        case 3: return launch_query1_cap<T, 3>(a, s);
        case 4: return launch_query1_cap<T, 4>(a, s);
        case 6: return launch_query1_cap<T, 6>(a, s);
        default: throw Error(RC_ERR_UNSUPPORTED, "single-query launch: row width beyond 768");
    }
}
#endif  // SCAN_INSTANTIATE

}  // namespace rc
