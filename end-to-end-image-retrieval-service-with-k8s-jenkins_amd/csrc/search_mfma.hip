// search_mfma.hip — batched exact cosine top-k on CDNA4 matrix cores
// (BASELINE config 4: 1024 queries x top-100 over a 125M x 512 fp16 shard).
//
// Replaces index.query(vector, top_k) (retriever/utils.py:62-64) for a batch of
// query vectors; the single-query path is the HBM-bound scan (index_common.h).
//
// A query batch is a GEMM: S = Q · Xᵀ (queries x rows, K = ld).  S is never
// materialised.  The search runs in STAGES over growing row ranges
// [0, b1), [b1, b2), ... with b(i+1) = g · b(i):
//   filter_gemm_kernel  MFMA (f16/bf16 in, f32 acc) 256 queries x 256 rows x 64
//                       tiles; the epilogue keeps (query, row) iff
//                       s'(q,r) >= thr[q] and appends the row to the query's
//                       candidate list (atomic counter, capacity CAND_CAP);
//   rescore_kernel      per query: exact f32 score of every candidate (the same
//                       arithmetic as the single-query scan, so both paths give
//                       bit-identical scores), wavefront top-k merge with the
//                       running top-k keys, thr[q] = kth_best - eps[q].
// Why it is exact: s' uses the query rounded to the storage dtype q̂.  For a
// stored row x̂ (||x̂|| <= 1.01) |s' - s| <= ||q - q̂||·||x̂|| + two f32
// accumulation bounds (512·2^-24 each) =: eps[q] (computed per query).  The
// running kth best T of the rows seen so far is a lower bound of the final kth
// best, so any row of the final top-k has s >= T, hence s' >= T - eps: the
// filter never drops a true member.  The stage ratio g keeps the expected
// candidates per stage at ≈ k·(g-1) ≪ CAND_CAP.  A query whose candidates
// overflow CAND_CAP in some stage (adversarial / duplicate-heavy data) is
// flagged and re-run on the device through the exact scan (index.hip,
// scan_topk_kernel's fallback mode): no host synchronisation.
//
// HBM layout: rows [cap256][ld] T (capacity rounded up to 256 rows so whole
// row tiles are readable), queries q̂ [nqb*256][ld] T (zero rows past nq).
#include <algorithm>
#include <vector>

#include "index_common.h"

namespace rc {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

template <typename T> struct MfmaOp;
template <> struct MfmaOp<f16_t> {
    typedef _Float16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x4_t mma(v8 a, v8 b, f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};
template <> struct MfmaOp<bf16_t> {
    typedef __bf16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x4_t mma(v8 a, v8 b, f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

constexpr int SB_TILE = 256;  // queries per query block = rows per row tile

// ------------------------------------------------------ query preparation --
// One wave per query slot q < nq_pad: qn = q/||q|| (f32, the exact rescoring
// operand, same arithmetic as normalize_queries_kernel), qh = cast(qn) (the
// MFMA operand), eps = error bound of s' (see header), thr = -inf (real
// query) or +inf (padding slot: never appends).
template <typename T>
__global__ __launch_bounds__(64) void prepare_queries_kernel(const float *__restrict__ q, int nq, int dim, int64_t ld,
                                                            float *__restrict__ qn, T *__restrict__ qh,
                                                            float *__restrict__ eps, float *__restrict__ thr) {
    const int lane = threadIdx.x;
    const int qi = blockIdx.x;
    const bool valid = qi < nq;
    const float *src = q + (int64_t)(valid ? qi : 0) * dim;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss = valid ? fmaf(src[c], src[c], ss) : 0.f;
    ss = wave_sum(ss);
    const float inv = ss > 0.f ? 1.0f / sqrtf(ss) : 0.f;
    float err = 0.f;
    for (int c = lane; c < ld; c += 64) {
        const float v = (valid && c < dim) ? src[c] * inv : 0.f;
        const T h = Elem<T>::cast(v);
        const float d = v - Elem<T>::load(&h, 0);
        err = fmaf(d, d, err);
        if (valid) qn[(int64_t)qi * ld + c] = v;
        qh[(int64_t)qi * ld + c] = h;
    }
    err = wave_sum(err);
    if (lane == 0) {
        eps[qi] = 1.01f * sqrtf(err) + 6.5e-5f;
        thr[qi] = valid ? -INFINITY : INFINITY;
    }
}

// ------------------------------------------------------- filter GEMM -------
struct FilterArgs {
    const void *rows;  // [>= roundup(r_end, 256)][ld]
    const void *qh;    // [nqb*256][ld]
    int64_t ld;
    int nkt;           // ld / 64
    int64_t r_begin;   // multiple of 256
    int64_t r_end;
    int64_t tiles_per_chunk;
    int nqb;
    const float *thr;  // [nqb*256]
    uint32_t *cnt;     // [nqb*256]
    uint32_t *cand;    // [nqb*256][cap]
    int cap;
    // int8 filter only (filter_i8_kernel): per-row sx / ex at i8_slot(row), per-query sq / aq
    const float *rsx = nullptr, *rex = nullptr, *sq = nullptr, *aq = nullptr;
};

// 256x256x64 tile, 512 threads = 8 waves in two groups (G0 = waves 0-3 own
// query rows 0-127, G1 = waves 4-7 rows 128-255; wave w and w+4 share a SIMD).
// Each wave owns 128 queries x 64 index rows as 4 quadrants of 64x32.  The
// (row tile, K-tile) steps of the block's chunk are one flattened sequence, so
// the next row tile's first K-tile streams in under the current tile's last
// MFMAs.  A K-tile is 4 phases; each phase is an M segment (ds_read the
// quadrant's fragments, issue this wave's LDS-DMA share of the next step,
// lgkmcnt(0)) and a C segment (16 MFMAs), each closed by a block barrier; G1
// runs one segment behind G0 so one wave per SIMD is in MFMAs while its partner
// reads LDS.  MFMA roles: A operand = index rows, B operand = queries, so a
// lane's accumulator holds 4 consecutive ROWS of one query: the epilogue tests
// one per-lane threshold against 16 values at a time.
// Block → (query block, chunk): blocks b and b+8 share an XCD; the nqb blocks
// of one chunk are consecutive on one XCD, so each row tile is read from HBM
// once and served to the other query blocks from that XCD's L2.
template <typename T>
__global__ __launch_bounds__(512, 1) void filter_gemm_kernel(FilterArgs a) {
    using Op = MfmaOp<T>;
    using v8 = typename Op::v8;
    constexpr int BK = 64;
    constexpr int A_BYTES = SB_TILE * BK * 2, STAGE = 2 * A_BYTES;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;

    const int b = blockIdx.x, xcd = b & 7, jx = b >> 3;
    const int qb = jx % a.nqb;
    const int64_t chunk = (int64_t)(jx / a.nqb) * 8 + xcd;
    const int64_t rt_total = (a.r_end - a.r_begin + SB_TILE - 1) / SB_TILE;
    const int64_t rt0 = chunk * a.tiles_per_chunk;
    const int64_t rt1 = min(rt_total, rt0 + a.tiles_per_chunk);
    if (rt0 >= rt1) return;  // block-uniform
    const int nkt = a.nkt;
    const int64_t ld = a.ld;
    const int64_t nsteps = (rt1 - rt0) * nkt;
    const uint16_t *Ag = (const uint16_t *)a.qh + (int64_t)qb * SB_TILE * ld;
    const uint16_t *Rg = (const uint16_t *)a.rows + (a.r_begin + rt0 * SB_TILE) * ld;

    // 64 pieces of 1 KB per step (queries: 0-31, rows: 32-63); wave w owns pieces w + 8 i.
    auto stage4 = [&](int buf, int64_t step, int i0) {
        uint8_t *base = smem + buf * STAGE;
        const int64_t rt = step / nkt;
        const int k0 = (int)(step - rt * nkt) * BK;
        const uint16_t *Wg = Rg + rt * SB_TILE * ld;
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i) {
            const int piece = wave + 8 * i;
            const bool is_q = i < 4;
            const int r = (is_q ? piece : piece - 32) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const uint16_t *src = (is_q ? Ag : Wg) + (int64_t)r * ld + k0 + c * 8;
            __builtin_amdgcn_global_load_lds((const void *)src, (lds_void *)(base + piece * 1024), 16, 0, 0);
        }
    };
    auto bar = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // thresholds of this lane's 8 query rows: q = qb*256 + grp*128 + mq*64 + mi*16 + li
    float thr[2][4];
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) thr[mq][mi] = a.thr[qb * SB_TILE + grp * 128 + mq * 64 + mi * 16 + li];

    f32x4_t acc[2][2][4][2];
    auto zero_acc = [&] {
#pragma unroll
        for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
            for (int a1 = 0; a1 < 2; ++a1)
#pragma unroll
                for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
                    for (int a3 = 0; a3 < 2; ++a3) acc[a0][a1][a2][a3] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    };
    zero_acc();

    stage4(0, 0, 0);
    stage4(0, 0, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (grp == 1) bar();  // stagger: G1 one segment behind

    v8 af[4][2], wf[2][2];  // queries [mi][s], rows [ni][s]
    for (int64_t step = 0; step < nsteps; ++step) {
        const int cur = (int)(step & 1);
        const uint8_t *As = smem + cur * STAGE;
        const uint8_t *Ws = As + A_BYTES;
        const bool more = step + 1 < nsteps;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mq = p >> 1;
            const int nq = (p == 1 || p == 2);
            if (p == 0 || p == 2) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int r = grp * 128 + mq * 64 + mi * 16 + li;
                        const int c = s * 4 + g;
                        af[mi][s] = *reinterpret_cast<const v8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int r = wc * 64 + nq * 32 + ni * 16 + li;
                    const int c = s * 4 + g;
                    wf[ni][s] = *reinterpret_cast<const v8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                }
            if (more && p < 2) stage4(cur ^ 1, step + 1, p * 4);
            if (p == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        acc[mq][nq][mi][ni] = Op::mma(wf[ni][s], af[mi][s], acc[mq][nq][mi][ni]);
            __builtin_amdgcn_s_setprio(0);
            bar();
        }

        if ((step + 1) % nkt == 0) {
            // ---- epilogue of row tile rt: lane holds S[q][r .. r+3] for 8 q x 4 r-groups
            const int64_t rt = rt0 + step / nkt;
            const int64_t rbase = a.r_begin + rt * SB_TILE + wc * 64 + 4 * g;
#pragma unroll
            for (int mq = 0; mq < 2; ++mq)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const float t = thr[mq][mi];
                    float m = -INFINITY;
#pragma unroll
                    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
                        for (int ni = 0; ni < 2; ++ni) {
                            const f32x4_t v = acc[mq][nq][mi][ni];
                            m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
                        }
                    if (__ballot(m >= t) == 0) continue;  // wave-uniform: the common case
                    if (m >= t) {
                        const int q = qb * SB_TILE + grp * 128 + mq * 64 + mi * 16 + li;
#pragma unroll
                        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
                            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    const int64_t row = rbase + nq * 32 + ni * 16 + j;
                                    if (acc[mq][nq][mi][ni][j] >= t && row < a.r_end) {
                                        const uint32_t pos = atomicAdd(&a.cnt[q], 1u);
                                        if ((int)pos < a.cap) a.cand[(int64_t)q * a.cap + pos] = (uint32_t)row;
                                    }
                                }
                    }
                }
            zero_acc();
        }
    }
    if (grp == 0) bar();  // balance the stagger barrier
}

// Query-stationary filter GEMM (ld = 64·NKT <= 512).  The filter GEMM above
// streams BOTH operands through LDS (256 queries x 256 rows per 64 KB K-step:
// 128 flop/B), which the L2->LDS fill rate caps near 45 % of MFMA peak.  Here a
// block's 256 queries live in REGISTERS for the whole launch and only index rows
// stream: one wave per SIMD (4 waves, up to 512 VGPRs each), wave w holds
// queries [64w, 64w+64) of the block's query group as 4 x 2·NKT B-fragments
// (256 VGPRs at ld 512) plus a 64 x 128 f32 accumulator (128 VGPRs).  Rows come
// in 128-row tiles, one 16 KB K-step (128 rows x 64) per stage of an 8-deep LDS
// ring (7 steps ≈ 112 KB in flight: enough to hide the HBM latency of a row
// tile's first touch): 2·256·128·64 flop per 16 KB = 256 flop/B, half the fill
// bytes of filter_gemm_kernel.  DMA through a per-step buffer descriptor (uniform
// base, 32-bit lane offsets) keeps addresses out of the VGPR budget.
// MFMA roles as above (A = index rows, B = queries): lane (li, g) of acc[rf][qt]
// holds rows 16·rf + 4g + j of query 16·qt + li.  Same thresholds, candidate
// appends and exactness argument as filter_gemm_kernel.
// Each wave holds 32 queries (2 x 16, QS_QT) for 128-row tiles: 8 waves, 2 per SIMD,
// every row-fragment read feeds two MFMAs and the SIMD partner wave's MFMAs cover
// its latency.  (A 4-wave form with 64 queries per wave pinned in AGPRs and
// inline-asm MFMAs was measured against it in round 2 — within 1 %, behind after
// the 2-GB sub-launches — and removed.)
constexpr int QS_QT = 2, QS_RT = 128, QS_NS = 8;  // queries/16 per wave, rows per tile, LDS ring steps

// ABL (A/B diagnostics, diagnostic builds only; 0 in production): bit0 no DMA in the
// loop, bit1 no MFMA, bit2 no fragment reads (MFMAs on the query registers), bit3 no
// epilogue.
template <typename T, int NKT, int ABL = 0>  // 256 queries per block
__global__ __launch_bounds__(512, 1) void filter_qs_kernel(FilterArgs a) {
    constexpr int QS_WAVES = 16 / QS_QT;
    constexpr int RF = QS_RT / 16;
    using Op = MfmaOp<T>;
    using v8 = typename Op::v8;
    constexpr int STEP_BYTES = QS_RT * 128;  // 16 KB at QT = 2
    __shared__ __attribute__((aligned(16))) uint8_t smem[QS_NS * STEP_BYTES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;

    const int b = blockIdx.x, xcd = b & 7, jx = b >> 3;
    const int qb = jx % a.nqb;
    const int64_t chunk = (int64_t)(jx / a.nqb) * 8 + xcd;
    const int64_t rt_total = (a.r_end - a.r_begin + QS_RT - 1) / QS_RT;
    const int64_t rt0 = chunk * a.tiles_per_chunk;
    const int64_t rt1 = min(rt_total, rt0 + a.tiles_per_chunk);
    if (rt0 >= rt1) return;  // block-uniform
    const int64_t ld = a.ld;
    const int ntiles = (int)(rt1 - rt0);  // per-block counters in 32 bits: uniform SALU compares
    const int nsteps = ntiles * NKT;
    const uint16_t *Rg = (const uint16_t *)a.rows + (a.r_begin + rt0 * QS_RT) * ld;

    // this lane's query fragments for the whole K: qf[qt][kk], kk = 32-wide k chunk
    v8 qf[QS_QT][2 * NKT];
    const int q0 = qb * SB_TILE + wave * 16 * QS_QT;
#pragma unroll
    for (int qt = 0; qt < QS_QT; ++qt)
#pragma unroll
        for (int kk = 0; kk < 2 * NKT; ++kk)
            qf[qt][kk] = *reinterpret_cast<const v8 *>((const uint16_t *)a.qh + (int64_t)(q0 + qt * 16 + li) * ld +
                                                       kk * 32 + g * 8);
    float thr[QS_QT];
#pragma unroll
    for (int qt = 0; qt < QS_QT; ++qt) thr[qt] = a.thr[q0 + qt * 16 + li];
    // consume the query loads here, so the compiler's vmcnt waits for them sit
    // before the K loop instead of inside it (where they would drain the DMA ring)
#pragma unroll
    for (int qt = 0; qt < QS_QT; ++qt) {
        asm volatile("" ::"v"(thr[qt]));
#pragma unroll
        for (int kk = 0; kk < 2 * NKT; ++kk) asm volatile("" ::"v"(qf[qt][kk]));
    }

    // step t = (tile, k-step): 2·RF pieces of 1 KB (8 rows x 128 B); wave w issues pieces w + QS_WAVES·i.
    constexpr int PPW = 2 * RF / QS_WAVES;
    uint32_t loff[PPW];  // byte offset of this lane's 16 B within the step's rows
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int r = (wave + QS_WAVES * i) * 8 + (lane >> 3);
        loff[i] = (uint32_t)(r * (int)ld + (((lane & 7) ^ ((r >> 1) & 7)) << 3)) * 2u;
    }
    auto issue = [&](int t) {
        const int tile = t / NKT;
        const int ks = (int)(t - tile * NKT);
        uint8_t *base = smem + (int)(t % QS_NS) * STEP_BYTES;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(Rg + (int64_t)tile * QS_RT * ld + ks * 64), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            // (the builtin's operands kept non-dependent: a template-dependent operand defers
            // its target check to instantiation, where the host pass drops the kernel's stub)
            lds_void *dst = (lds_void *)(base + (wave + QS_WAVES * i) * 1024);
            const uint32_t off = loff[i];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, off, 0, 0, 0);
        }
    };
    // one barrier per SPS = 2 k-steps (nsteps is a multiple): steps t..t+SPS-1 land
    // together, steps t+NS-SPS..t+NS-1 go into the slots freed by t-SPS..t-1; NS - SPS
    // steps in flight
    constexpr int SPS = 2;
    for (int t = 0; t < min(QS_NS - SPS, nsteps); ++t) issue(t);

    f32x4_t acc[RF][QS_QT];
    for (int tile = 0; tile < ntiles; ++tile) {
#pragma unroll
        for (int rf = 0; rf < RF; ++rf)
#pragma unroll
            for (int qt = 0; qt < QS_QT; ++qt)
                acc[rf][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kp = 0; kp < NKT / SPS; ++kp) {
            const int t = tile * NKT + SPS * kp;
            // steps t..t+SPS-1 landed: the NS - 2·SPS younger steps (PPW DMAs each) may be in flight
            static_assert(NKT % SPS == 0 && (QS_NS - 2 * SPS) * PPW < 64, "whole sync groups; vmcnt is 6 bits");
            if (t + QS_NS - SPS - 1 < nsteps) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((QS_NS - 2 * SPS) * PPW) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave's DMA of t..t+SPS-1 landed; slots of t-SPS..t-1 are free
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = QS_NS - SPS; j < QS_NS; ++j)
                if (!(ABL & 1) && t + j < nsteps) issue(t + j);
            // groups of 4 row fragments, (k half kl, k sub-chunk sh, row quarter rh): 4 reads,
            // then their 4·QT MFMAs with counted lgkmcnt waits.  Row r = 16 rf + li: its
            // swizzle (r >> 1) & 7 = (li >> 1) & 7 does not depend on rf.  The SIMD
            // partner wave's MFMAs cover the read latency.
            constexpr int RH = RF / 4, NG = SPS * 2 * RH;
            auto frag_ptr = [&](int gi) {
                const int kl = gi / (2 * RH), sh = (gi / RH) % 2, rh = gi % RH;
                return smem + ((t + kl) % QS_NS) * STEP_BYTES + li * 128 + (((sh * 4 + g) ^ ((li >> 1) & 7)) << 4) +
                       rh * 4 * 2048;
            };
            auto load_group = [&](int gi, v8 *dst) {
                const uint8_t *Sr = frag_ptr(gi);
                const int ks = SPS * kp + gi / (2 * RH), sh = (gi / RH) % 2;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    dst[i] = (ABL & 4) ? qf[i & 1][(ks * 2 + sh + i) % (2 * NKT)]
                                       : *reinterpret_cast<const v8 *>(Sr + i * 2048);
            };
#pragma unroll
            for (int gi = 0; gi < NG; ++gi) {
                const int ks = SPS * kp + gi / (2 * RH), sh = (gi / RH) % 2, rh = gi % RH;
                v8 cur[4];
                load_group(gi, cur);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int qt = 0; qt < QS_QT; ++qt)
                        if constexpr (ABL & 2)
                            asm volatile("" ::"v"(cur[i]));
                        else
                            acc[rh * 4 + i][qt] = Op::mma(cur[i], qf[qt][ks * 2 + sh], acc[rh * 4 + i][qt]);
                __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            }
        }
        // ---- epilogue of row tile rt0 + tile: candidates s' >= thr[q]
        const int64_t rbase = a.r_begin + (rt0 + tile) * QS_RT + 4 * g;
        if constexpr (ABL & 8) {  // diagnostics: no epilogue (accumulators kept live)
#pragma unroll
            for (int rf = 0; rf < RF; ++rf)
#pragma unroll
                for (int qt = 0; qt < QS_QT; ++qt) asm volatile("" ::"v"(acc[rf][qt]));
            continue;
        }
#pragma unroll
        for (int qt = 0; qt < QS_QT; ++qt) {
            const float th = thr[qt];
            float m = -INFINITY;
#pragma unroll
            for (int rf = 0; rf < RF; ++rf) {
                const f32x4_t v = acc[rf][qt];
                m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
            }
            if (__ballot(m >= th) == 0) continue;  // wave-uniform: the common case
            if (m >= th) {
                const int q = q0 + qt * 16 + li;
#pragma unroll
                for (int rf = 0; rf < RF; ++rf)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int64_t row = rbase + rf * 16 + j;
                        if (acc[rf][qt][j] >= th && row < a.r_end) {
                            const uint32_t pos = atomicAdd(&a.cnt[q], 1u);
                            if ((int)pos < a.cap) a.cand[(int64_t)q * a.cap + pos] = (uint32_t)row;
                        }
                    }
            }
        }
    }
}

// ------------------------------------------------ int8 filter (optional) --
// With the index's int8 filter copy (rc_index_set_filter(RC_FILTER_I8)) the filter GEMM
// runs on v_mfma_i32_16x16x64_i8 — twice the f16/bf16 MFMA rate, half the row bytes —
// and the candidates are still rescored exactly on the stored rows (rescore_kernel).
// A stored row x̂ is kept as x̃ = sx·x8 (x8 = rne(x̂/sx) in [-127, 127], sx = max|x̂|/127)
// with ex >= ||x̂ - x̃||₂; a normalised query qn as q̃ = sq·q8 with eq >= ||qn - q̃||₂.
// The integer dot D = q8·x8 is exact (|D| <= ld·127² < 2^24: exact in f32 too), and
//   |sq·sx·D - qn·x̂| <= ||qn||·ex + eq·||x̃|| <= ex·(1.0001 + eq) + 1.01·eq
// (||qn|| <= 1.0001, ||x̃|| <= ||x̂|| + ex, ||x̂|| <= 1.01).  A row is kept iff
//   sq·(sx·D) + ex·aq >= thr[q],   aq = 1.0001 + eq,   thr = kth - eps,
//   eps = 1.01·eq + 6.5e-5 (the f32 bound of the exact scores, as above) + 1e-6 (the
// f32 rounding of the left side), so the filter never drops a row of the final top-k.
// For unit rows in 512-d, ex and eq are ≈ 0.004-0.008: the candidate lists are a few
// times longer than with the f16 filter, so the stages grow more slowly
// (batch_stage_ratio's inflation).
//
// Queries: as prepare_queries_kernel (same qn arithmetic), plus q8 / sq / aq.
__global__ __launch_bounds__(64) void prepare_queries_i8_kernel(const float *__restrict__ q, int nq, int dim, int64_t ld,
                                                               float *__restrict__ qn, int8_t *__restrict__ q8,
                                                               float *__restrict__ sq, float *__restrict__ aq,
                                                               float *__restrict__ eps, float *__restrict__ thr) {
    const int lane = threadIdx.x;
    const int qi = blockIdx.x;
    const bool valid = qi < nq;
    const float *src = q + (int64_t)(valid ? qi : 0) * dim;
    float ss = 0.f;
    for (int c = lane; c < dim; c += 64) ss = valid ? fmaf(src[c], src[c], ss) : 0.f;
    ss = wave_sum(ss);
    const float inv = ss > 0.f ? 1.0f / sqrtf(ss) : 0.f;
    float mx = 0.f;
    for (int c = lane; c < ld; c += 64) {
        const float v = (valid && c < dim) ? src[c] * inv : 0.f;
        mx = fmaxf(mx, fabsf(v));
        if (valid) qn[(int64_t)qi * ld + c] = v;
    }
    mx = wave_max(mx);
    const float s = mx * (1.0f / 127.0f), is = mx > 0.f ? 127.0f / mx : 0.f;
    float err = 0.f;
    for (int c = lane; c < ld; c += 64) {
        const float v = (valid && c < dim) ? src[c] * inv : 0.f;  // the value stored in qn above
        const float r = fminf(127.f, fmaxf(-127.f, rintf(v * is)));
        q8[(int64_t)qi * ld + c] = (int8_t)r;
        const float d = v - s * r;
        err = fmaf(d, d, err);
    }
    err = wave_sum(err);
    if (lane == 0) {
        const float eq = sqrtf(err) * 1.001f + 1e-7f;
        sq[qi] = s;
        aq[qi] = 1.0001f + eq;
        eps[qi] = 1.01f * eq + 6.6e-5f;
        thr[qi] = valid ? -INFINITY : INFINITY;
    }
}

// Query-stationary like filter_qs_kernel (same LDS ring, buffer-descriptor DMA, 128-row
// tiles, 8 waves x 32 queries), with the MFMA roles swapped: A = queries (registers),
// B = index rows (LDS), so lane (li, g) of acc[rf][qt] holds queries 16·qt + 4g + j of
// row 16·rf + li — one row per (lane, rf): its sx / ex are 8 values per lane per tile
// (i8_slot layout), loaded with the previous tile's epilogue.  A K-step is 128 bytes
// = 128 int8 elements, NKT = row bytes / 128 steps per tile.  Every ring step is
// issued (a step past the block's range reads nothing: zero-size buffer descriptor), so
// each wait counts a fixed number of younger loads: the DMA of the younger steps, plus
// this tile's 4 scale loads while they are younger than the awaited step.
// RT = rows per tile: 128, or 64 at ld 768 (NKT 6), where the 96 query-fragment registers
// leave room for only half the accumulators.
constexpr int I8_SL = 24;  // candidate rows staged in LDS per query per block (filter_i8_kernel)

// LDS atomic add / store as inline asm: written in C++, hipcc cannot tell these words from the
// LDS-DMA ring in the same __shared__ array and waits vmcnt(0) (the whole ring) before each one.
// The add's own lgkmcnt(0) is inside the statement, so its result is ready when it ends; the
// stores are retired by an explicit lgkmcnt(0) ahead of the block barrier before the flush.
__device__ __forceinline__ uint32_t lds_add_rtn_u32(uint32_t *p, uint32_t v) {
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void lds_write_u32(uint32_t *p, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
}

// AUX: cache-policy bits of the row DMA (0; 2 = nontemporal: diagnostic builds' A/B)
template <int NKT, int RT, int AUX = 0>
__global__ __launch_bounds__(512, 1) void filter_i8_kernel(FilterArgs a) {
    typedef int i32x4_t __attribute__((ext_vector_type(4)));
    constexpr int QT = QS_QT, WAVES = 16 / QS_QT, RF = RT / 16, RH = RF / 4;
    constexpr int STEP_BYTES = RT * 128;
    constexpr int SPS = 2, SXL = 2 * RH;
    constexpr int PPW = 2 * RF / WAVES;
    static_assert((RT == 128 || RT == 64) && NKT % SPS == 0 && (QS_NS - 2 * SPS) * PPW + SXL < 64, "layout");
    // behind the ring (one __shared__ array): per query of the block a counter and I8_SL staged
    // candidate rows, appended with LDS atomics (lgkmcnt only) and flushed to the global lists
    // once at the block's end — a returning global atomic per append would wait for every
    // older vector-memory op, i.e. drain the DMA ring (vmcnt(0)) in the middle of the K loop
    __shared__ __attribute__((aligned(16))) uint8_t smem[QS_NS * STEP_BYTES + SB_TILE * 4 * (1 + I8_SL) + SB_TILE * 12];
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(smem + QS_NS * STEP_BYTES);
    uint32_t *lbuf = lcnt + SB_TILE;
    // the block's per-query thr, sq, aq: read by each epilogue instead of held in 24 VGPRs, which
    // the K loop needs (in registers the kernel spilled; from LDS it is 0.7 % faster)
    float *lq = reinterpret_cast<float *>(lbuf + SB_TILE * I8_SL);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;

    const int b = blockIdx.x, xcd = b & 7, jx = b >> 3;
    const int qb = jx % a.nqb;
    const int64_t chunk = (int64_t)(jx / a.nqb) * 8 + xcd;
    const int64_t rt_total = (a.r_end - a.r_begin + RT - 1) / RT;
    const int64_t rt0 = chunk * a.tiles_per_chunk;
    const int64_t rt1 = min(rt_total, rt0 + a.tiles_per_chunk);
    if (rt0 >= rt1) return;  // block-uniform
    const int64_t ldb = a.ld;  // bytes per row
    const int ntiles = (int)(rt1 - rt0);
    const int nsteps = ntiles * NKT;
    const int64_t row0 = a.r_begin + rt0 * RT;  // a multiple of RT (host check)
    const uint8_t *Rg = (const uint8_t *)a.rows + row0 * ldb;
    if (tid < SB_TILE) {  // visible to every wave after the K loop's first barrier
        const int q = qb * SB_TILE + tid;
        lcnt[tid] = 0u;
        lq[tid] = a.thr[q];
        lq[SB_TILE + tid] = a.sq[q];
        lq[2 * SB_TILE + tid] = a.aq[q];
    }

    i32x4_t qf[QT][2 * NKT];  // bytes [64 kk + 16 g, +16) of query q0 + 16 qt + li
    const int q0 = qb * SB_TILE + wave * 16 * QT;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int kk = 0; kk < 2 * NKT; ++kk)
            qf[qt][kk] = *reinterpret_cast<const i32x4_t *>((const uint8_t *)a.qh + (int64_t)(q0 + qt * 16 + li) * ldb +
                                                            kk * 64 + g * 16);
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int kk = 0; kk < 2 * NKT; ++kk) asm volatile("" ::"v"(qf[qt][kk]));
    // an epilogue's per-query operands: 3·QT LDS reads (inline asm: as C++, hipcc would wait for
    // the whole DMA ring first), retired together
    auto epi_params = [&](float (&thr)[QT][4], float (&sq)[QT][4], float (&aq)[QT][4]) __attribute__((always_inline)) {
        f32x4_t v[3][QT];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                asm volatile("ds_read_b128 %0, %1"
                             : "=v"(v[c][qt])
                             : "v"((uint32_t)(uintptr_t)(lq + c * SB_TILE + wave * 16 * QT + qt * 16 + 4 * g)));
        static_assert(QT == 2, "the wait below ties 3 x 2 values");
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(v[0][0]), "+v"(v[0][1]), "+v"(v[1][0]), "+v"(v[1][1]), "+v"(v[2][0]), "+v"(v[2][1]));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                thr[qt][j] = v[0][qt][j];
                sq[qt][j] = v[1][qt][j];
                aq[qt][j] = v[2][qt][j];
            }
    };

    uint32_t loff[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int r = (wave + WAVES * i) * 8 + (lane >> 3);
        loff[i] = (uint32_t)(r * (int)ldb + (((lane & 7) ^ ((r >> 1) & 7)) << 4));
    }
    auto issue = [&](int t) {
        const bool ok = t < nsteps;
        const int tile = t / NKT;
        const int ks = t - tile * NKT;
        uint8_t *base = smem + (t % QS_NS) * STEP_BYTES;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(ok ? Rg + (int64_t)tile * RT * ldb + ks * 128 : Rg), (short)0, ok ? 0x7fffffff : 0, 0x00020000);
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            lds_void *dst = (lds_void *)(base + (wave + WAVES * i) * 1024);
            const uint32_t off = loff[i];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, off, 0, 0, AUX);
        }
    };
    f32x4_t sxv[RH], exv[RH];  // rows 16 rf + li of the tile, rf = 4 h + e → sxv[h][e]
    auto load_scales = [&](int tile) {
        const int64_t tb = row0 + (int64_t)tile * RT;  // i8_slot(tb + 16 rf + li) = p + rf
        const int64_t p = (tb & ~int64_t(127)) + li * 8 + ((tb & 127) >> 4);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int h = 0; h < RH; ++h) sxv[h] = *reinterpret_cast<const f32x4_t *>(a.rsx + p + 4 * h);
#pragma unroll
        for (int h = 0; h < RH; ++h) exv[h] = *reinterpret_cast<const f32x4_t *>(a.rex + p + 4 * h);
        asm volatile("" ::: "memory");
    };
    for (int t = 0; t < QS_NS - SPS; ++t) issue(t);
    load_scales(0);

    i32x4_t acc[RF][QT];
    for (int tile = 0; tile < ntiles; ++tile) {
#pragma unroll
        for (int rf = 0; rf < RF; ++rf)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) acc[rf][qt] = i32x4_t{0, 0, 0, 0};
#pragma unroll
        for (int kp = 0; kp < NKT / SPS; ++kp) {
            const int t = tile * NKT + SPS * kp;
            // steps t..t+SPS-1 must have landed; younger: NS - 2·SPS steps, and this tile's
            // scale loads while they were issued after step t + SPS - 1
            if (t + QS_NS - SPS - 1 < nsteps) {
                if (SPS * (kp + 2) <= QS_NS)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((QS_NS - 2 * SPS) * PPW + SXL) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((QS_NS - 2 * SPS) * PPW) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = QS_NS - SPS; j < QS_NS; ++j) issue(t + j);
            constexpr int NG = SPS * 2 * RH;
            // row-fragment group gi: 4 rows-of-16 x (k-step kl, half sh) — read into cur, then 4 x QT
            // MFMAs.  Rolling schedule: each fragment of group gi + 1 is read as soon as the MFMAs
            // of the same slot of group gi have issued, so a group's LDS latency runs under the
            // previous group's MFMAs instead of in front of its own (no extra registers: the new
            // fragment takes the slot just freed).
            auto frag_addr = [&](int gi) {
                const int kl = gi / (2 * RH), sh = (gi / RH) % 2, rh = gi % RH;
                return smem + ((t + kl) % QS_NS) * STEP_BYTES + li * 128 + (((sh * 4 + g) ^ ((li >> 1) & 7)) << 4) +
                       rh * 4 * 2048;
            };
            i32x4_t cur[4];
            {
                const uint8_t *Sr = frag_addr(0);
#pragma unroll
                for (int i = 0; i < 4; ++i) cur[i] = *reinterpret_cast<const i32x4_t *>(Sr + i * 2048);
            }
            __builtin_amdgcn_sched_barrier(0);  // group 0's reads go out together, ahead of the pattern
#pragma unroll
            for (int gi = 0; gi < NG; ++gi) {
                const int kl = gi / (2 * RH), sh = (gi / RH) % 2, rh = gi % RH;
                const int ks = SPS * kp + kl;
                const uint8_t *Sn = frag_addr(gi + 1 < NG ? gi + 1 : gi);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
                        acc[rh * 4 + i][qt] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(qf[qt][ks * 2 + sh], cur[i], acc[rh * 4 + i][qt], 0, 0, 0);
                    if (gi + 1 < NG) cur[i] = *reinterpret_cast<const i32x4_t *>(Sn + i * 2048);
                    __builtin_amdgcn_sched_group_barrier(0x008, QT, 0);
                    if (gi + 1 < NG) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
            }
        }
        // ---- epilogue: keep (q, row) iff sq·(sx·D) + ex·aq >= thr[q]
        float sx[RF], ex[RF];
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
            sx[rf] = sxv[rf >> 2][rf & 3];
            ex[rf] = exv[rf >> 2][rf & 3];
        }
        float exm = ex[0], sxmax = sx[0], sxmin = sx[0];
#pragma unroll
        for (int rf = 1; rf < RF; ++rf) {
            exm = fmaxf(exm, ex[rf]);
            sxmax = fmaxf(sxmax, sx[rf]);
            sxmin = fminf(sxmin, sx[rf]);
        }
        float thr[QT][4], sq[QT][4], aq[QT][4];
        epi_params(thr, sq, aq);
        // the gate: for every rf, sx[rf]·D[rf] <= sxb·Dmax with Dmax = max_rf D[rf] and sxb = sxmax
        // (Dmax >= 0) or sxmin (Dmax < 0); f32 products and the fma are monotonic, so the gate
        // passes whenever one of the lane's 8 per-element conditions below holds (the appends are
        // decided by those alone): an integer max per accumulator instead of cvt + mul + max
        bool hit = false, hq[QT][4];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int dm = acc[0][qt][j];
#pragma unroll
                for (int rf = 1; rf < RF; ++rf) dm = max(dm, acc[rf][qt][j]);
                const float m = (dm >= 0 ? sxmax : sxmin) * (float)dm;
                hq[qt][j] = fmaf(exm, aq[qt][j], sq[qt][j] * m) >= thr[qt][j];
                hit |= hq[qt][j];
            }
        if (__ballot(hit) != 0 && hit) {
            const int64_t rbase = row0 + (int64_t)tile * RT + li;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    // only the (qt, j) whose gate passed walk their 8 rows (the looser int8 bound
                    // sends about a quarter of the wave-tiles here)
                    if (!hq[qt][j]) continue;
                    const int q = q0 + qt * 16 + 4 * g + j;
#pragma unroll
                    for (int rf = 0; rf < RF; ++rf) {
                        const int64_t row = rbase + rf * 16;
                        const float v = fmaf(ex[rf], aq[qt][j], sq[qt][j] * (sx[rf] * (float)acc[rf][qt][j]));
                        if (v >= thr[qt][j] && row < a.r_end) {
                            const int ql = q - qb * SB_TILE;
                            const uint32_t p = lds_add_rtn_u32(&lcnt[ql], 1u);
                            if (p < (uint32_t)I8_SL) {
                                lds_write_u32(&lbuf[ql * I8_SL + p], (uint32_t)row);
                            } else {  // this block's slots of q are full: straight to the global list
                                const uint32_t pos = atomicAdd(&a.cnt[q], 1u);
                                if ((int)pos < a.cap) a.cand[(int64_t)q * a.cap + pos] = (uint32_t)row;
                            }
                        }
                    }
                }
        }
        load_scales(min(tile + 1, ntiles - 1));  // unconditional: the same wait counts on every path
    }
    // flush the staged candidates: one global atomic per query that has any.  The asm stores are
    // invisible to the compiler's wait-count tracking, so retire them explicitly before the barrier.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < SB_TILE) {
        const uint32_t n = min(lcnt[tid], (uint32_t)I8_SL);
        if (n) {
            const int q = qb * SB_TILE + tid;
            const uint32_t base = atomicAdd(&a.cnt[q], n);
            for (uint32_t i = 0; i < n; ++i)
                if (base + i < (uint32_t)a.cap) a.cand[(int64_t)q * a.cap + base + i] = lbuf[tid * I8_SL + i];
        }
    }
}

// ------------------------------------------------------- exact rescoring --
// One block per query.  Candidates are scored exactly as scan_topk_kernel
// scores a row (16 lanes per row, 16-B chunks, f32 FMA in chunk order, DPP
// reduction), merged with the running top-k keys, and the threshold for the
// next stage is set.  Overflow (more candidates than cap) is flagged for the
// host's exact fallback; the counter is reset for the next stage.
template <typename T, int NCH, int CAP>
__global__ __launch_bounds__(256) void rescore_kernel(const T *__restrict__ rows, int64_t ld, const float *__restrict__ qn,
                                                     int k, uint32_t *__restrict__ cnt, const uint32_t *__restrict__ cand,
                                                     int cap, uint64_t *__restrict__ keys, const float *__restrict__ eps,
                                                     float *__restrict__ thr, int *__restrict__ flags,
                                                     int *__restrict__ ovf_total, int final_pass, int64_t row_base,
                                                     int64_t row_stride, float *__restrict__ out_scores,
                                                     int64_t *__restrict__ out_rows) {
    constexpr int EPC = 16 / sizeof(T);
    constexpr int CPL = NCH * 128 / (16 * EPC);
    constexpr int U = 2;
    __shared__ uint64_t lds[4][CAP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane & 15, rg = lane >> 4;
    const int qi = blockIdx.x;

    float q[CPL][EPC];
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int e = 0; e < EPC; ++e) q[i][e] = qn[(int64_t)qi * ld + (sub + 16 * i) * EPC + e];

    const uint32_t n = cnt[qi];
    const int nn = (int)min<uint32_t>(n, (uint32_t)cap);
    const uint32_t *cl = cand + (int64_t)qi * cap;
    const uint4 *base4 = reinterpret_cast<const uint4 *>(rows);
    const int64_t ld4 = ld / EPC;

    WaveTopK<CAP> tk;
    tk.init(as_lds(&lds[wave][0]), k);
    if (wave == 0) {  // the running top-k of the earlier stages
        for (int j = 0; j < k; j += 64) {
            const uint64_t key = (j + lane < k) ? keys[(int64_t)qi * k + j + lane] : KEY_EMPTY;
            tk.reserve(64);
            tk.push(key != KEY_EMPTY, key);
        }
    }
    for (int j0 = wave * 4 * U; j0 < nn; j0 += 16 * U) {
        uint4 x[U][CPL];
        uint32_t rr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * 4 + rg;
            rr[u] = cl[j < nn ? j : 0];
#pragma unroll
            for (int i = 0; i < CPL; ++i) x[u][i] = base4[(int64_t)rr[u] * ld4 + sub + 16 * i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * 4 + rg;
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                float f[EPC];
                unpack16<T>(x[u][i], f);
#pragma unroll
                for (int e = 0; e < EPC; ++e) acc = fmaf(f[e], q[i][e], acc);
            }
            const float s = sum16(acc);
            tk.reserve(4);
            tk.push(sub == 0 && j < nn, make_key(s, rr[u]));
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
        for (int j = lane; j < k; j += 64) {
            const uint64_t key = tk.buf[j];
            keys[(int64_t)qi * k + j] = key;
            if (final_pass) {
                const bool ok = key != KEY_EMPTY;
                out_scores[(int64_t)qi * k + j] = ok ? key_score(key) : -INFINITY;
                out_rows[(int64_t)qi * k + j] = ok ? row_base + (int64_t)key_idx(key) * row_stride : -1;
            }
        }
        if (lane == 0) {
            thr[qi] = tk.count >= k ? key_score(tk.buf[k - 1]) - eps[qi] : -INFINITY;
            if (n > (uint32_t)cap && flags[qi] == 0) {
                flags[qi] = 1;
                atomicAdd(ovf_total, 1);
            }
            cnt[qi] = 0;
        }
    }
}

// ------------------------------------------------------------------ host ---
template <typename T, int NCH>
void launch_rescore_cap(const BatchPlan &p, const BatchWs &ws, int final_pass, hipStream_t s) {
    const int cap = topk_cap(p.k);
#define RC_RESCORE(CAPV)                                                                                         \
    hipLaunchKernelGGL((rescore_kernel<T, NCH, CAPV>), dim3(p.nq), dim3(256), 0, s, (const T *)p.rows, p.ld, ws.qn, \
                       p.k, ws.cnt, ws.cand, ws.cap, ws.keys, ws.eps, ws.thr, ws.flags, ws.ovf, final_pass, p.row_base,  \
                       p.row_stride, p.out_scores, p.out_rows)
    if (cap <= 128) RC_RESCORE(128);
    else if (cap <= 256) RC_RESCORE(256);
    else RC_RESCORE(512);
#undef RC_RESCORE
    RC_LAUNCH_CHECK();
}

template <typename T>
void launch_rescore(const BatchPlan &p, const BatchWs &ws, int final_pass, hipStream_t s) {
    switch (p.nch) {
        case 1: return launch_rescore_cap<T, 1>(p, ws, final_pass, s);
        case 2: return launch_rescore_cap<T, 2>(p, ws, final_pass, s);
        case 3: return launch_rescore_cap<T, 3>(p, ws, final_pass, s);
        case 4: return launch_rescore_cap<T, 4>(p, ws, final_pass, s);
        case 6: return launch_rescore_cap<T, 6>(p, ws, final_pass, s);
        case 8: return launch_rescore_cap<T, 8>(p, ws, final_pass, s);
        case 12: return launch_rescore_cap<T, 12>(p, ws, final_pass, s);
        case 16: return launch_rescore_cap<T, 16>(p, ws, final_pass, s);
        default: throw Error(RC_ERR_UNSUPPORTED, "unsupported row width");
    }
}

int batch_stage_ratio(int k, int cap, int inflation) {
    const int g = cap / (5 * k / 2 * inflation + 1);
    return std::max(2, std::min(64, g));
}

// The stages: stage 1 takes the first cap rows as candidates (thr = -inf), each later
// stage filters the next g-times-larger row range against the running thresholds, then
// rescore_kernel merges its candidates.  filter(c0, c1, nchunk) enqueues one filter
// dispatch over rows [c0, c1) split into nchunk row chunks.
#if defined(RC_GEMM_ABLATION)
int g_diag_filter_split_log2 = 31;
int g_diag_filter_aux = 0;  // the int8 filter's row DMA cache policy (rc_diag_set_filter_aux)
#endif
template <typename T, typename F>
void run_stages(const BatchPlan &p, BatchWs &ws, hipStream_t s, KernelTimer *timer, int g, int64_t row_bytes, F &&filter) {
    const int nqb = (p.nq + SB_TILE - 1) / SB_TILE;
    const int nq_pad = nqb * SB_TILE;
    RC_HIP(hipMemsetAsync(ws.keys, 0xFF, (size_t)p.nq * p.k * sizeof(uint64_t), s));
    RC_HIP(hipMemsetAsync(ws.cnt, 0, (size_t)nq_pad * sizeof(uint32_t), s));
    RC_HIP(hipMemsetAsync(ws.flags, 0, (size_t)p.nq * sizeof(int), s));
    int64_t b0 = 0, b1 = std::min<int64_t>(p.n_rows, ws.cap);
    // With nq > 256 the nqb query blocks that read one row chunk run side by side on one
    // XCD so that its L2 serves the second to last reader; over a long chunk their
    // progress drifts apart by more than the L2 holds (memory-side reads 2.8x the rows
    // at 125M rows).  Sub-launches of <= 2 GB of rows realign them: reads fall to 1.05x
    // and the filter runs 3-5 % faster (profiles/r02/r02_ab_results.txt).
#if defined(RC_GEMM_ABLATION)
    const int split_log2 = g_diag_filter_split_log2;  // diagnostic builds: the sub-launch size A/B
#else
    constexpr int split_log2 = 31;
#endif
    const int64_t split = nqb > 1 ? std::max<int64_t>(SB_TILE, ((int64_t)1 << split_log2) / row_bytes / SB_TILE * SB_TILE)
                                  : (int64_t)0;
    while (b0 < p.n_rows) {
        for (int64_t c0 = b0; c0 < b1;) {
            const int64_t c1 = split > 0 ? std::min(b1, c0 + split) : b1;
            const int slot = timer ? timer->begin(s) : -1;  // per dispatch, as rocprofv3 counts them
            const int64_t rt_total = (c1 - c0 + SB_TILE - 1) / SB_TILE;
            int64_t nchunk = std::min<int64_t>(rt_total, std::max<int64_t>(1, (256 + nqb - 1) / nqb));
            nchunk = (nchunk + 7) / 8 * 8;
            filter(c0, c1, nchunk, nqb);
            RC_LAUNCH_CHECK();
            if (timer) timer->end(slot, s, 2.0 * (double)nq_pad * (double)(c1 - c0) * (double)p.ld);
            c0 = c1;
        }
        launch_rescore<T>(p, ws, b1 == p.n_rows ? 1 : 0, s);
        b0 = b1;
        b1 = std::min<int64_t>(p.n_rows, b1 * g);
    }
}

template <typename T>
void run_batched(const BatchPlan &p, BatchWs &ws, hipStream_t s, KernelTimer *timer) {
    const int nq_pad = (p.nq + SB_TILE - 1) / SB_TILE * SB_TILE;
    hipLaunchKernelGGL(prepare_queries_kernel<T>, dim3(nq_pad), dim3(64), 0, s, p.queries, p.nq, p.dim, p.ld, ws.qn,
                       (T *)ws.qh, ws.eps, ws.thr);
    RC_LAUNCH_CHECK();
    auto filter = [&](int64_t c0, int64_t c1, int64_t nchunk, int nqb) {
        const int64_t rt_total = (c1 - c0 + SB_TILE - 1) / SB_TILE;
        const int64_t tpc = (rt_total + nchunk - 1) / nchunk;
        FilterArgs fa{p.rows, ws.qh, p.ld, (int)(p.ld / 64), c0, c1, tpc, nqb, ws.thr, ws.cnt, ws.cand, ws.cap};
        const int nkt = (int)(p.ld / 64);
        if (nkt == 2 || nkt == 4 || nkt == 8) {
            fa.tiles_per_chunk = ((c1 - c0 + QS_RT - 1) / QS_RT + nchunk - 1) / nchunk;
            const dim3 gr((unsigned)(nchunk * nqb)), bl(64 * 16 / QS_QT);
            if (nkt == 8) hipLaunchKernelGGL((filter_qs_kernel<T, 8>), gr, bl, 0, s, fa);
            else if (nkt == 4) hipLaunchKernelGGL((filter_qs_kernel<T, 4>), gr, bl, 0, s, fa);
            else hipLaunchKernelGGL((filter_qs_kernel<T, 2>), gr, bl, 0, s, fa);
        } else {
            hipLaunchKernelGGL(filter_gemm_kernel<T>, dim3((unsigned)(nchunk * nqb)), dim3(512), 0, s, fa);
        }
    };
    run_stages<T>(p, ws, s, timer, batch_stage_ratio(p.k, ws.cap), p.ld * (int64_t)sizeof(T), filter);
}

// Candidates per stage grow by exp(z·eps/σ) over the f16 filter's (≈ 3x for random unit
// rows in 512-d at top-100 of 125M); the stage ratio assumes 3x.
constexpr int I8_STAGE_INFLATION = 3;

template <typename T>
void run_batched_i8(const BatchPlan &p, BatchWs &ws, hipStream_t s, KernelTimer *timer) {
    const int nq_pad = (p.nq + SB_TILE - 1) / SB_TILE * SB_TILE;
    hipLaunchKernelGGL(prepare_queries_i8_kernel, dim3(nq_pad), dim3(64), 0, s, p.queries, p.nq, p.dim, p.ld, ws.qn,
                       (int8_t *)ws.qh, ws.sq, ws.aq, ws.eps, ws.thr);
    RC_LAUNCH_CHECK();
    const int nkt = (int)(p.ld / 128);
    auto filter = [&](int64_t c0, int64_t c1, int64_t nchunk, int nqb) {
        const int rt = nkt == 6 ? 64 : 128;
        RC_REQUIRE(c0 % rt == 0, RC_ERR_INVALID, "internal: int8 filter range not tile-aligned");
        const int64_t tpc = ((c1 - c0 + rt - 1) / rt + nchunk - 1) / nchunk;
        FilterArgs fa{p.rows8, ws.qh, p.ld, nkt, c0, c1, tpc, nqb, ws.thr, ws.cnt, ws.cand, ws.cap};
        fa.rsx = p.rsx;
        fa.rex = p.rex;
        fa.sq = ws.sq;
        fa.aq = ws.aq;
        const dim3 gr((unsigned)(nchunk * nqb)), bl(64 * 16 / QS_QT);
#if defined(RC_GEMM_ABLATION)
        if (nkt == 4 && g_diag_filter_aux == 2) {
            hipLaunchKernelGGL((filter_i8_kernel<4, 128, 2>), gr, bl, 0, s, fa);
            return;
        }
#endif
        if (nkt == 4) hipLaunchKernelGGL((filter_i8_kernel<4, 128>), gr, bl, 0, s, fa);
        else if (nkt == 6) hipLaunchKernelGGL((filter_i8_kernel<6, 64>), gr, bl, 0, s, fa);
        else hipLaunchKernelGGL((filter_i8_kernel<2, 128>), gr, bl, 0, s, fa);
    };
    run_stages<T>(p, ws, s, timer, batch_stage_ratio(p.k, ws.cap, I8_STAGE_INFLATION), p.ld, filter);
}

bool i8_filter_supported(int64_t ld) { return ld == 256 || ld == 512 || ld == 768; }

void batched_search(const BatchPlan &p, BatchWs &ws, hipStream_t s, KernelTimer *timer) {
    RC_REQUIRE(p.ld % 64 == 0, RC_ERR_UNSUPPORTED, "batched search needs ld % 64 == 0");
    RC_REQUIRE(p.n_rows > 0, RC_ERR_INVALID, "batched search over an empty range");
    if (p.rows8 != nullptr) {
        RC_REQUIRE(i8_filter_supported(p.ld), RC_ERR_UNSUPPORTED, "int8 filter needs ld 256, 512 or 768");
        if (p.dtype == RC_F16) return run_batched_i8<f16_t>(p, ws, s, timer);
        if (p.dtype == RC_BF16) return run_batched_i8<bf16_t>(p, ws, s, timer);
        if (p.dtype == RC_F32) return run_batched_i8<float>(p, ws, s, timer);
    }
    if (p.dtype == RC_F16) return run_batched<f16_t>(p, ws, s, timer);
    if (p.dtype == RC_BF16) return run_batched<bf16_t>(p, ws, s, timer);
    throw Error(RC_ERR_UNSUPPORTED, "batched MFMA search needs an f16 or bf16 index (or the int8 filter copy)");
}

void BatchWs::ensure(int nq, int k, int64_t ld, int dtype_bytes) {
    const int nq_pad = (nq + SB_TILE - 1) / SB_TILE * SB_TILE;
    if (nq_pad <= nq_cap && k <= k_cap && ld <= ld_cap) return;
    release();
    nq_cap = std::max(nq_pad, 256);
    k_cap = std::max(k, 16);
    ld_cap = ld;
    qn = (float *)dmalloc((size_t)nq_cap * ld * sizeof(float));
    qh = dmalloc((size_t)nq_cap * ld * dtype_bytes);
    eps = (float *)dmalloc((size_t)nq_cap * sizeof(float));
    thr = (float *)dmalloc((size_t)nq_cap * sizeof(float));
    cnt = (uint32_t *)dmalloc((size_t)nq_cap * sizeof(uint32_t));
    cand = (uint32_t *)dmalloc((size_t)nq_cap * cap * sizeof(uint32_t));
    keys = (uint64_t *)dmalloc((size_t)nq_cap * k_cap * sizeof(uint64_t));
    flags = (int *)dmalloc((size_t)nq_cap * sizeof(int));
    sq = (float *)dmalloc((size_t)nq_cap * sizeof(float));
    aq = (float *)dmalloc((size_t)nq_cap * sizeof(float));
    ovf = (int *)dmalloc(sizeof(int));
    RC_HIP(hipMemset(ovf, 0, sizeof(int)));
    // the fallback scan's partial lists are sized by a memory budget, not by the row count:
    // 1024 queries x top-100 keep all 256 blocks (210 MB); 4096 x 256 get 32 (268 MB) instead of 2.1 GB
    const int64_t per_block = (int64_t)nq_cap * k_cap * (int64_t)sizeof(uint64_t);
    fb_blocks = (int)std::max<int64_t>(FB_MIN_BLOCKS, std::min<int64_t>(FB_BLOCKS, FB_BUDGET_BYTES / per_block));
    fb_partial = (uint64_t *)dmalloc((size_t)fb_blocks * per_block);
}

void BatchWs::release() {
    dfree(qn);
    dfree(qh);
    dfree(eps);
    dfree(thr);
    dfree(cnt);
    dfree(cand);
    dfree(keys);
    dfree(flags);
    dfree(sq);
    dfree(aq);
    dfree(ovf);
    dfree(fb_partial);
    qn = nullptr;
    qh = nullptr;
    eps = thr = nullptr;
    cnt = cand = nullptr;
    keys = nullptr;
    flags = ovf = nullptr;
    sq = aq = nullptr;
    fb_partial = nullptr;
    fb_blocks = 0;
    nq_cap = k_cap = 0;
    ld_cap = 0;
}

}  // namespace rc

#if defined(RC_GEMM_ABLATION)
// diagnostic builds: log2 of the bytes of rows per filter sub-launch (31 = the product's 2 GB)
extern "C" int rc_diag_set_filter_aux(int aux) {
    return rc::guard([&] {
        RC_REQUIRE(aux == 0 || aux == 2, RC_ERR_INVALID, "aux 0 or 2");
        rc::g_diag_filter_aux = aux;
    });
}
extern "C" int rc_diag_set_filter_split(int log2_bytes) {
    return rc::guard([&] {
        RC_REQUIRE(log2_bytes >= 24 && log2_bytes <= 40, RC_ERR_INVALID, "log2 bytes in [24, 40]");
        rc::g_diag_filter_split_log2 = log2_bytes;
    });
}
#endif
