// vit_kernels.h — device kernels of the ViT-MSN embedding path (gfx950).
//
// Reference arithmetic (transformers models/vit_msn/modeling_vit_msn.py, called
// from embedding/main.py:111-113):
//   patch embed Conv2d(3,768,16,16) (:57)  → patch_gemm_kernel (gemm.h): implicit GEMM
//                                            reading the u8 images through a bf16 LUT
//   q/k/v/o, fc1, fc2 nn.Linear (:199-202,243-244) → gemm_pp_kernel & co (gemm.h: bias /
//                                            GELU / residual / LayerNorm-fold epilogues fused)
//   LayerNorm eps 1e-6 (:258-259,327)      → layernorm_kernel (f32 in, bf16 out)
//   eager attention, scale 1/8, fp32 softmax (:161-186) → attention_v2_kernel
//   last_hidden_state[:,0,:] (main.py:113) → cls_final_kernel (final LN on the
//                                            CLS rows, raw + L2-normalised outputs)
// Preprocessing (ViTImageProcessor, main.py:107): resize_{h,v}_kernel (Pillow
// fixed-point resample); rescale+normalize is an exact f32 LUT, applied inside the
// patch GEMM's A loads (and by pixel_values_kernel for the parity hook).
#pragma once

#include "rc_common.h"

namespace rc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

// EPI_BF16_LN / EPI_GELU_BF16_LN: the bf16 epilogues as consumers of the LayerNorm fold
// EPI_RESID_BF16 / EPI_PATCH_BF16: the residual-stream producers with the stream kept in bf16
// (see "Residual stream in bf16"; GemmArgs::ln_x)
enum GemmEpi { EPI_BF16 = 0, EPI_GELU_BF16 = 1, EPI_RESID_F32 = 2, EPI_PATCH_F32 = 3, EPI_BF16_LN = 4, EPI_GELU_BF16_LN = 5,
               EPI_RESID_BF16 = 6, EPI_PATCH_BF16 = 7 };
constexpr bool epi_bf16_out(int e) { return e == EPI_BF16 || e == EPI_GELU_BF16 || e == EPI_BF16_LN || e == EPI_GELU_BF16_LN; }
constexpr bool epi_resid(int e) { return e == EPI_RESID_F32 || e == EPI_RESID_BF16; }
constexpr bool epi_patch(int e) { return e == EPI_PATCH_F32 || e == EPI_PATCH_BF16; }
constexpr bool epi_bf16_stream(int e) { return e == EPI_RESID_BF16 || e == EPI_PATCH_BF16; }
constexpr bool epi_gelu(int e) { return e == EPI_GELU_BF16 || e == EPI_GELU_BF16_LN; }
constexpr bool epi_ln(int e) { return e == EPI_BF16_LN || e == EPI_GELU_BF16_LN; }

struct GemmArgs {
    const uint16_t *A;  // [rows >= roundup(M, BM)][K] bf16, row-major
    const uint16_t *W;  // [N][K] bf16 (nn.Linear weight layout)
    const float *bias;  // [N]
    int M, N, K;        // M = valid rows; N % 128 == 0; K % 64 == 0
    uint16_t *out_bf16; // EPI_BF16 / EPI_GELU_BF16: [M][N]
    float *out_f32;     // EPI_RESID_F32 (in place: out += A W^T + b) / EPI_PATCH_F32
    const float *pos;   // EPI_PATCH_F32: position embeddings [tokens][N]
    int tokens;         // EPI_PATCH_F32: tokens per image (patches + 1)
    int group_m = 0;                 // ping-pong tile order: 0 = row-major, G = groups of G row tiles
    // image-aligned row tiles (the residual producers O-proj / fc2, N = 768): row tile tm covers
    // the rows [tm·row_step, tm·row_step + row_step) of one image (row_step = tokens = 197), computed
    // as a 224-row tile, so a batch of n images is exactly n × (N / 256) tiles (0: BM-row tiles)
    int row_step = 0;
    int ldc = 0;                     // bf16 outputs: row stride in elements (0 = N)
    // LayerNorm folded across a GEMM pair (see "LayerNorm fold" below):
    //   producer (f32 epilogues): ln_x != null → also write bf16(x) rows and per-(row, 64-column
    //     block) partial statistics (mean, M2) into ln_stats[row][LN_PARTS][2]
    //   consumer (bf16 epilogues): ln_c != null → A is bf16(x), W = W∘γ, bias = b + W·β, and the
    //     epilogue applies rstd·(acc − μ·c) + bias with μ, rstd from ln_stats[row][LN_PARTS][2]
    uint16_t *ln_x = nullptr;
    float *ln_stats = nullptr;
    //   EPI_RESID_BF16 / EPI_PATCH_BF16 (resid_bf16): the residual stream is ln_x itself, bf16,
    //     instead of out_f32 (see "Residual stream in bf16"): the residual is read from and the
    //     result written to ln_x; the statistics only when ln_stats != null
    bool resid_bf16 = false;
    const float *ln_c = nullptr;
    float ln_eps = 1e-6f;
    // implicit-GEMM patch embedding (patch_gemm_kernel): A[m][k] is read from the u8
    // HWC images, rescale→normalize as bf16(fma(u, pre_a[c], pre_b[c])) per channel c — an
    // affine form rc_model verifies, for all 256 byte values, to give exactly the bf16 of
    // ViTImageProcessor's f32 value (transformers rescale in f64 → f32, normalize in f32)
    const uint8_t *img = nullptr;  // [images][S][S][3]
    float pre_a[3] = {}, pre_b[3] = {};
    int img_size = 0;              // S
};

// ------------------------------------------------------------ LayerNorm fold
// modeling_vit_msn.py:258-259 LayerNorm(768, eps) then nn.Linear:
//   LN(x)·Wᵀ + b = rstd·(x·W′ᵀ − μ·c) + b′,  W′ = W·diag(γ),  c_n = Σ_k W′[n][k],  b′ = b + W·β.
// The residual stream's producer epilogue (patch GEMM, O-proj, fc2, cls_init)
// writes bf16(x) next to the f32 x plus, per 64-column block of each row, the
// block mean and M2 = Σ (x − block mean)²; the consumer GEMM (QKV, fc1) combines
// the twelve blocks by Chan's formula (exact in exact arithmetic, no E[x²] − μ²
// cancellation) and applies the correction in its epilogue.  What this removes:
// the standalone LayerNorm pass (f32 read + bf16 write of the whole stream, 24
// launches per batch).  Accuracy: bf16(x) carries the same relative error as
// bf16(LN(x)) while |μ| ≲ σ per token; c is summed from the bf16 W′ the MFMAs
// use, so the μ·c term cancels exactly what the MFMAs add for the mean.
//
// Partials (round 3): per row, LN_PARTS = 12 blocks of 64 columns, each (mean, M2) —
// the 64 columns one wave of a tiled GEMM holds per row, so the producer epilogues reduce
// inside the wave (two permlane swaps) and never across waves.  Canonical order, which
// every producer (tiled epilogues, gemm_skinny_ln_kernel, cls_init_kernel) reproduces bit for
// bit: "slice" g = 0..3 of a block holds the 16 columns 32c + 16(g & 1) + 8(g >> 1) + k
// (c = 0, 1; k = 0..7 — after one v_permlane16_swap, the 8 consecutive columns a lane of
// the accumulator layout holds per 32-column chunk); ln_slice_stats gives its (mean, M2),
// then ln_combine(g0, g1), ln_combine(g2, g3) and ln_combine(g01, g23) (Chan, equal
// counts).  The consumer combines the 12 block partials in ln_row_scale.
constexpr int LN_PARTS = 12;            // 768 columns / 64
constexpr int LN_STRIDE = 2 * LN_PARTS;  // floats of partials per row
__device__ __forceinline__ int ln_slice_col(int g, int c) { return 32 * c + 16 * (g & 1) + 8 * (g >> 1); }

// ------------------------------------------- Residual stream in bf16
// Under the LayerNorm fold the residual stream x is kept as bf16 RNE(x) alone — exactly the
// bf16(x) the QKV / fc1 GEMMs read as A.  Producers (patch GEMM, O-proj, fc2, cls_init) round
// once and write 2 B per element; the residual epilogues read 2 B.  Every producer computes the
// LN statistics from the rounded value it stored, so the skinny (gemm_skinny_ln_kernel) and
// tiled paths stay bit-identical.  (Rounds 2-5 kept a low part beside it — a second bf16, then
// one byte, ~2^-16 relative — at 6 B per element per epilogue and ~20 more VALU ops per element;
// the bf16 stream costs 1.8e-4 cosine against the fp32 oracle where the pair gave 1.0e-4,
// tools/resid_precision_sim.py, inside the 1e-3 fp32 tier.)
__device__ __forceinline__ float4 bf16x4_f32(uint2 u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ uint2 pack_bf16x4(float4 v) { return make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w)); }
// four consecutive stream elements -> f32
__device__ __forceinline__ float4 rs_load4(const uint16_t *p) { return bf16x4_f32(*reinterpret_cast<const uint2 *>(p)); }
// round four values to the stream, store them when `valid`; returns the value stored
__device__ __forceinline__ float4 rs_store4(float4 x, uint16_t *p, bool valid) {
    const uint2 h = pack_bf16x4(x);
    if (valid) *reinterpret_cast<uint2 *>(p) = h;
    return bf16x4_f32(h);
}

// 8 bf16 (one 16-B load) <-> 8 f32
__device__ __forceinline__ void bf16x8_unpack(uint4 u, float (&f)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ uint4 bf16x8_pack(const float (&f)[8]) {
    return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}
// (mean, M2) of one canonical 16-column slice (x[8c + k] = column 32c + slice offset + k).
// Written with explicit fmaf and no multiply-add left to the compiler's contraction, so
// every kernel that inlines it rounds identically.
__device__ __forceinline__ float ln_sum8(const float *x) {
    return ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]));
}
__device__ __forceinline__ float ln_sq8(const float *x, float m) {
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = x[k] - m;
    const float t0 = fmaf(d[0], d[0], d[1] * d[1]), t1 = fmaf(d[2], d[2], d[3] * d[3]);
    const float t2 = fmaf(d[4], d[4], d[5] * d[5]), t3 = fmaf(d[6], d[6], d[7] * d[7]);
    return (t0 + t1) + (t2 + t3);
}
__device__ __forceinline__ float2 ln_slice_stats(const float (&x)[16]) {
    const float m = (ln_sum8(x) + ln_sum8(x + 8)) * 0.0625f;
    return make_float2(m, ln_sq8(x, m) + ln_sq8(x + 8, m));
}
// Chan's combination of two equal-count partials (n columns each): a is the lower slice
// (or pair of slices), b the upper; w = n / 2 (= n·n / 2n)
__device__ __forceinline__ float2 ln_combine(float2 a, float2 b, float w) {
    const float d = a.x - b.x;
    return make_float2((a.x + b.x) * 0.5f, fmaf(d * d, w, a.y + b.y));
}
// The block partial from the four slices held by lanes l, l ^ 16, l ^ 32, l ^ 48 (slice
// g = lane >> 4: the accumulator layout of the tiled GEMMs).  Every lane gets the result.
__device__ __forceinline__ float2 ln_block_reduce_rows(float2 s) {
    // rows (16-lane groups) 0 <-> 1 and 2 <-> 3: [0] = the even row's value, [1] = the odd row's
    const auto px = __builtin_amdgcn_permlane16_swap(__float_as_uint(s.x), __float_as_uint(s.x), false, false);
    const auto py = __builtin_amdgcn_permlane16_swap(__float_as_uint(s.y), __float_as_uint(s.y), false, false);
    s = ln_combine(make_float2(__uint_as_float(px[0]), __uint_as_float(py[0])),
                   make_float2(__uint_as_float(px[1]), __uint_as_float(py[1])), 8.0f);
    // rows {0, 1} <-> {2, 3}: [0] = the lower half's value, [1] = the upper half's
    const auto qx = __builtin_amdgcn_permlane32_swap(__float_as_uint(s.x), __float_as_uint(s.x), false, false);
    const auto qy = __builtin_amdgcn_permlane32_swap(__float_as_uint(s.y), __float_as_uint(s.y), false, false);
    return ln_combine(make_float2(__uint_as_float(qx[0]), __uint_as_float(qy[0])),
                      make_float2(__uint_as_float(qx[1]), __uint_as_float(qy[1])), 16.0f);
}
// The same reduction with slice g = lane & 3 (the emitter kernels: 4 lanes per block)
__device__ __forceinline__ float2 ln_block_reduce_quad(float2 s, int g) {
    float2 o = make_float2(__shfl_xor(s.x, 1), __shfl_xor(s.y, 1));
    s = (g & 1) ? ln_combine(o, s, 8.0f) : ln_combine(s, o, 8.0f);
    o = make_float2(__shfl_xor(s.x, 2), __shfl_xor(s.y, 2));
    return (g & 2) ? ln_combine(o, s, 16.0f) : ln_combine(s, o, 16.0f);
}

// Chan combination of the LN_PARTS block partials of one row → (rstd, −rstd·μ)
__device__ __forceinline__ float2 ln_row_scale(const float *__restrict__ st, float eps) {
    float m[LN_PARTS], q[LN_PARTS];
#pragma unroll
    for (int t = 0; t < LN_PARTS / 2; ++t) {
        const float4 v = reinterpret_cast<const float4 *>(st)[t];
        m[2 * t] = v.x;
        q[2 * t] = v.y;
        m[2 * t + 1] = v.z;
        q[2 * t + 1] = v.w;
    }
    static_assert(LN_PARTS == 12, "the combination tree below is written for 12 partials");
    const float sm = (((m[0] + m[1]) + (m[2] + m[3])) + ((m[4] + m[5]) + (m[6] + m[7]))) + ((m[8] + m[9]) + (m[10] + m[11]));
    float M2 = (((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]))) + ((q[8] + q[9]) + (q[10] + q[11]));
    const float mu = sm * (1.0f / LN_PARTS);
#pragma unroll
    for (int t = 0; t < LN_PARTS; ++t) M2 = fmaf(64.0f * (m[t] - mu), m[t] - mu, M2);
    const float rstd = 1.0f / sqrtf(fmaf(M2, 1.0f / (64 * LN_PARTS), eps));
    return make_float2(rstd, -rstd * mu);
}

// One wave per row of H = 256*NV f32 values → bf16 LayerNorm output.
template <int NV>
__global__ __launch_bounds__(256) void layernorm_kernel(const float *__restrict__ x, const float *__restrict__ g,
                                                       const float *__restrict__ b, uint16_t *__restrict__ y, int M,
                                                       float eps) {
    constexpr int H = 256 * NV;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float4 *xr = reinterpret_cast<const float4 *>(x + (int64_t)row * H);
    float4 v[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        v[i] = xr[lane + 64 * i];
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) * (1.0f / H);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
        ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(ss) * (1.0f / H) + eps);
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    const float4 *b4 = reinterpret_cast<const float4 *>(b);
    uint2 *yr = reinterpret_cast<uint2 *>(y + (int64_t)row * H);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float4 gg = g4[lane + 64 * i], bb = b4[lane + 64 * i];
        const float o0 = (v[i].x - mean) * rstd * gg.x + bb.x;
        const float o1 = (v[i].y - mean) * rstd * gg.y + bb.y;
        const float o2 = (v[i].z - mean) * rstd * gg.z + bb.z;
        const float o3 = (v[i].w - mean) * rstd * gg.w + bb.w;
        yr[lane + 64 * i] = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
    }
}

// Final LayerNorm of the CLS row of each image + the two /embed outputs.
template <int NV>
// hi != null: the rows are the bf16 residual stream `hi` instead of `hidden`.
__global__ __launch_bounds__(64) void cls_final_kernel(const float *__restrict__ hidden, const uint16_t *__restrict__ hi,
                                                      int tokens,
                                                      const float *__restrict__ g, const float *__restrict__ b,
                                                      float eps, float *__restrict__ raw, float *__restrict__ normed) {
    constexpr int H = 256 * NV;
    const int lane = threadIdx.x;
    const int img = blockIdx.x;
    const int64_t r0 = (int64_t)img * tokens * H;
    const float4 *xr = reinterpret_cast<const float4 *>(hidden + r0);
    float4 v[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        v[i] = hi ? rs_load4(hi + r0 + 4 * (lane + 64 * i)) : xr[lane + 64 * i];
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) * (1.0f / H);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
        ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(ss) * (1.0f / H) + eps);
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    const float4 *b4 = reinterpret_cast<const float4 *>(b);
    float4 o[NV];
    float n2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float4 gg = g4[lane + 64 * i], bb = b4[lane + 64 * i];
        o[i].x = (v[i].x - mean) * rstd * gg.x + bb.x;
        o[i].y = (v[i].y - mean) * rstd * gg.y + bb.y;
        o[i].z = (v[i].z - mean) * rstd * gg.z + bb.z;
        o[i].w = (v[i].w - mean) * rstd * gg.w + bb.w;
        n2 += (o[i].x * o[i].x + o[i].y * o[i].y) + (o[i].z * o[i].z + o[i].w * o[i].w);
        reinterpret_cast<float4 *>(raw + (int64_t)img * H)[lane + 64 * i] = o[i];
    }
    if (normed) {
        const float nrm = sqrtf(wave_sum(n2));
        const float inv = nrm > 0.f ? 1.0f / nrm : 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i)
            reinterpret_cast<float4 *>(normed + (int64_t)img * H)[lane + 64 * i] =
                make_float4(o[i].x * inv, o[i].y * inv, o[i].z * inv, o[i].w * inv);
    }
}

// hidden[img*tokens + 0] = cls + pos[0]; with ln_x: the row into the bf16 residual stream
// instead, plus its LN partials (the LayerNorm fold's producer for the CLS rows; H = 768: 48
// lanes, one canonical slice each, see LN_PARTS)
__global__ __launch_bounds__(256) void cls_init_kernel(float *__restrict__ hidden, int tokens, int H,
                                                      const float *__restrict__ cls, const float *__restrict__ pos,
                                                      uint16_t *__restrict__ ln_x, float *__restrict__ ln_stats) {
    const int img = blockIdx.x;
    const int64_t row = (int64_t)img * tokens;
    if (ln_x == nullptr) {
        for (int c = threadIdx.x; c < H; c += 256) hidden[row * H + c] = cls[c] + pos[c];
        return;
    }
    if (threadIdx.x >= 64) return;  // one wave: lanes 0-47 = (block, slice), 48-63 only join the shuffles
    const int t = threadIdx.x, g = t & 3, ok = t < 4 * LN_PARTS;
    const int blk = ok ? t >> 2 : 0;
    float xs[16];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int col = blk * 64 + ln_slice_col(g, c);
        float x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = cls[col + k] + pos[col + k];
        const uint4 h = bf16x8_pack(x);
        if (ok) *reinterpret_cast<uint4 *>(ln_x + row * H + col) = h;
        float xv[8];
        bf16x8_unpack(h, xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) xs[8 * c + k] = xv[k];
    }
    const float2 st = ln_block_reduce_quad(ln_slice_stats(xs), g);
    if (ok && g == 0) *reinterpret_cast<float2 *>(ln_stats + row * LN_STRIDE + 2 * blk) = st;
}

// Self-attention v2 for one (image, head), tokens <= 208, head dim 64.
// K and V of the head are staged by LDS-DMA (global_load_lds_dwordx4, 8 rows of
// 128 B per wave-instruction) into XOR-swizzled rows: K chunk ^ ((row>>1)&7)
// (conflict-free ds_read_b128 A-fragments), V chunk ^ (((row>>1)&3)<<1)
// (conflict-free ds_read_b64_tr_b16); the swizzle is applied to the per-lane
// source address.  Keys pad to 13 tiles of 16 (rows >= tokens re-read the last
// token: finite, and masked to p = 0).  Sᵀ = K·Qᵀ (13 tiles), softmax in f32 with
// scores pre-scaled by log2(e)/8 so p = exp2(s - max); Oᵀ = Vᵀ·Pᵀ in 6 steps of 32
// keys (16x16x32) + one 16-key step (16x16x16).  3 blocks per CU (52 KB LDS).
constexpr int ATT2_TILES = 13, ATT2_ROWS = ATT2_TILES * 16;  // 208 keys

typedef short s16x8 __attribute__((ext_vector_type(8)));

// Scores + softmax of one 16-query tile (K of the head in LDS, the tile's Q fragments qf): st = p,
// sum = Σp over the lane's query row.  Padded keys (only in tiles that reach past `tokens`: a
// uniform branch) are masked to -inf; the max runs on the raw scores and the scale is folded into
// one fma per score: p = exp2(s·c − max·c), c = log2(e)/8 > 0.
template <int TOK>
__device__ __forceinline__ void att_scores(const uint8_t *Ks, const bf16x8 (&qf)[2], int tokens, float scale_log2e,
                                           f32x4 (&st)[ATT2_TILES], float &sum) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int t = 0; t < ATT2_TILES; ++t) {
        st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int r = t * 16 + li;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = s * 4 + g;
            const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(Ks + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
            st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], st[t], 0, 0, 0);
        }
        if (t & 1) asm volatile("" ::: "memory");  // cap the K-fragment loads in flight (VGPRs)
    }
#pragma unroll
    for (int t = 0; t < ATT2_TILES; ++t)
        if ((t + 1) * 16 > tokens) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (t * 16 + g * 4 + j >= tokens) st[t][j] = -INFINITY;
        }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < ATT2_TILES; ++t) mx = fmaxf(mx, fmaxf(fmaxf(st[t][0], st[t][1]), fmaxf(st[t][2], st[t][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float nmc = -mx * scale_log2e;
    sum = 0.f;
#pragma unroll
    for (int t = 0; t < ATT2_TILES; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float p = __builtin_amdgcn_exp2f(fmaf(st[t][j], scale_log2e, nmc));
            st[t][j] = p;
            sum += p;
        }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
}

// O = P·V of query tile qt (V of the head in LDS), normalised and stored to obase (the image's
// output rows at this head's columns, row stride H)
__device__ __forceinline__ void att_pv_store(const uint8_t *Vs, const f32x4 (&st)[ATT2_TILES], float sum, int qt,
                                             int tokens, uint16_t *obase, int H) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int qq = li >> 2, pp = li & 3;
    f32x4 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto vrow_addr = [&](int row, int d) {
        // bytes 32d + 8pp of the row, through the V swizzle (16-B chunk ^ ((row>>1)&3)*2)
        const int chunk = (2 * d + (pp >> 1)) ^ (((row >> 1) & 3) << 1);
        return (lds_s16x4_t *)(Vs + row * 128 + chunk * 16 + (pp & 1) * 8);
    };
#pragma unroll
    for (int tp = 0; tp < ATT2_TILES / 2; ++tp) {
        const int t = tp * 2;
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            pf[j] = (__bf16)st[t][j];
            pf[j + 4] = (__bf16)st[t + 1][j];
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(vrow_addr(t * 16 + g * 4 + qq, d));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(vrow_addr(t * 16 + 16 + g * 4 + qq, d));
            const s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, o[d], 0, 0, 0);
        }
        asm volatile("" ::: "memory");  // cap the V transposed reads in flight (VGPRs)
    }
    {   // last 16-key tile: K = 16 MFMA, lane group g holds keys 192 + 4g + j
        constexpr int t = ATT2_TILES - 1;
        s16x4 pf4;
#pragma unroll
        for (int j = 0; j < 4; ++j) pf4[j] = __builtin_bit_cast(short, (__bf16)st[t][j]);
        s16x4 v4[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) v4[d] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(vrow_addr(t * 16 + g * 4 + qq, d));
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(v4[d], pf4, o[d], 0, 0, 0);
    }
    const int q = qt * 16 + li;
    if (q < tokens) {
        const float inv = 1.0f / sum;
        uint16_t *orow = obase + (int64_t)q * H;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            *reinterpret_cast<uint2 *>(orow + d * 16 + g * 4) =
                make_uint2(pack_bf16x2(o[d][0] * inv, o[d][1] * inv), pack_bf16x2(o[d][2] * inv, o[d][3] * inv));
    }
}

// TOK > 0: the token count as a compile-time constant (197 for ViT-B/16 at 224),
// so only the last key tile carries the padding mask; TOK = 0 reads `tokens`.
// qsplit > 1 (small batches: a lone image is 12 (image, head) items for 256 CUs): block b is
// part b % qsplit of item b / qsplit and takes query tiles qs·4 + wave, stepping 4·qsplit — each
// part stages the head's K and V (L2 hits after the first) and runs the same per-tile arithmetic.
// STAG > 0 (diagnostic builds): the first round's second and third blocks of each CU (blockIdx
// 256..767 under the dispatcher's round-robin placement) start STAG and 2·STAG s_memrealtime
// ticks (10 ns) late, so that co-resident blocks are out of phase (one's K/V DMA under the others'
// math) for the rest of the launch.
// AUX: the cache-policy bits of the K/V LDS-DMA — 2 = nontemporal: every K/V row is read by exactly
// one block (round 6 in-model A/B, bit-identical: 72.8 -> 71.5 us per launch, step 9.19 -> 9.14 ms
// at parts = 2, profiles/r06/r06u_attention_nt_dma_ab_p{1,2}.log); 0 = the default policy (rounds
// 1-5, diagnostic builds)
template <int TOK, int STAG = 0, int AUX = 2>
__global__ __launch_bounds__(256, 3) void attention_v2_kernel(const uint16_t *__restrict__ qkv, uint16_t *__restrict__ out,
                                                          int tokens_rt, int heads, float scale_log2e, int qsplit) {
    if constexpr (STAG > 0) {
        if (blockIdx.x >= 256 && blockIdx.x < 768) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), d = (uint64_t)STAG * (blockIdx.x >> 8);
            while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
        }
    }
    constexpr int W = 4, HALF = W / 2, HD = 64, PPW = ATT2_TILES * 2 / HALF;  // 13 DMA pieces per wave
    const int tokens = TOK > 0 ? TOK : tokens_rt;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * ATT2_ROWS * 128];
    uint8_t *Ks = lds, *Vs = lds + ATT2_ROWS * 128;
    const int H = heads * HD, H3 = 3 * H;
    const int item = blockIdx.x / qsplit, qs = blockIdx.x % qsplit;
    const int img = item / heads, h = item % heads;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint16_t *base = qkv + (int64_t)img * tokens * H3 + h * HD;

    const int g = lane >> 4, li = lane & 15;
    const int nqt = (tokens + 15) / 16;
    // Q of a query tile: 2 x 16 B per lane, as inline asm — beside LDS-DMA, hipcc waits vmcnt(0)
    // (every DMA, and in the loop the loads just issued) before the first use of a plain load;
    // the counted waits below are exact (every load here is waited for by an explicit vmcnt)
    auto load_q = [&](int qt, bf16x8 (&qv)[2]) {
        const int q = qt * 16 + li;
        const uint16_t *qp = base + (int64_t)(q < tokens ? q : tokens - 1) * H3 + g * 8;
        asm volatile("global_load_dwordx4 %0, %2, off nt\n\tglobal_load_dwordx4 %1, %2, off offset:64 nt"
                     : "=&v"(qv[0]), "=&v"(qv[1])
                     : "v"(qp)
                     : "memory");
    };
    // the first query tile's Q (older than every DMA below), then 13 pieces of 1 KB per wave:
    // waves 0-1 stage K (pieces 0-25), waves 2-3 stage V (26-51).  K is waited for before the
    // scores, V only before the first P·V: V's transfer runs under the first tile's QKᵀ and
    // softmax (one block's load is no longer one serial phase ahead of its math).
    const int t0 = qs * W + wave, tstep = W * qsplit;  // this wave's query tiles
    bf16x8 qf[2];
    load_q(t0 < nqt ? t0 : 0, qf);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        // waves 0-1 stage K pieces w PPW + i, waves 2-3 the V pieces
        const bool isv = wave >= HALF;
        const int kp = min((wave - (isv ? HALF : 0)) * PPW + i, ATT2_TILES * 2 - 1);
        const int piece = isv ? ATT2_TILES * 2 + kp : kp;
        const int r = kp * 8 + (lane >> 3);
        const int pc = lane & 7;
        const int c = isv ? (pc ^ (((r >> 1) & 3) << 1)) : (pc ^ ((r >> 1) & 7));
        const int rr = r < tokens ? r : tokens - 1;
        const uint16_t *src = base + (int64_t)rr * H3 + (isv ? 2 * H : H) + c * 8;
        __builtin_amdgcn_global_load_lds((const void *)src, (lds_void_t *)(lds + piece * 1024), 16, 0, AUX);
    }
    auto bar = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    if (wave < HALF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K staged (and Q)
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");     // Q only: V may fly
    bar();
    __builtin_amdgcn_sched_barrier(0);  // nothing that reads qf moves above the wait

    f32x4 st[ATT2_TILES];
    float sum = 0.f;
    auto scores = [&](const bf16x8 (&qf)[2]) { att_scores<TOK>(Ks, qf, tokens, scale_log2e, st, sum); };
    auto pv_store = [&](int qt) { att_pv_store(Vs, st, sum, qt, tokens, out + (int64_t)img * tokens * H + h * HD, H); };

    // first tile: scores while V lands, then every wave waits for V once
    const bool first = t0 < nqt;
    bf16x8 qn[2];
    if (first && t0 + tstep < nqt) load_q(t0 + tstep, qn);  // the next tile's queries, under the scores
    if (first) scores(qf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // V staged (waves HALF..), qn landed
    bar();
    __builtin_amdgcn_sched_barrier(0);
    if (first) pv_store(t0);
    for (int qt = t0 + tstep; qt < nqt; qt += tstep) {
        // qn (issued a tile ago) has landed; the previous tile's 4 output stores may still fly
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        qf[0] = qn[0];
        qf[1] = qn[1];
        if (qt + tstep < nqt) load_q(qt + tstep, qn);  // prefetch the next tile's queries
        scores(qf);
        pv_store(qt);
    }
}

// Self-attention v3: the per-(image, head) arithmetic of attention_v2_kernel (att_scores /
// att_pv_store: the same bits), re-scheduled so that HBM never idles.  In v2 every block loads
// its K and V, then computes, then stores — and with all blocks of a round doing the same
// thing at the same time, the chip alternates between an HBM-bound load phase and a latency-
// bound math phase (0.5 of HBM, mfma_busy 0.18).  Here the grid is persistent: two blocks per
// CU, each walking items (image, head) = blockIdx.x, + gridDim.x, ...; while it computes item i
// from LDS, the block's lanes already hold item i+1's Q, K and V in registers (20 16-B loads per
// lane, issued before the math: register staging, issue early / write late), which are written
// into LDS between two barriers once every wave is done with item i.  Q joins K and V in LDS
// (3 x 208 rows x 128 B = 78 KB per block, XOR-swizzled as in v2: conflict-free ds_read_b128
// fragments and ds_write_b128 rows).
constexpr int ATT3_CHUNKS = 3 * ATT2_ROWS * 8;             // 16-B chunks of Q, K, V (208 rows each)
constexpr int ATT3_PER_LANE = (ATT3_CHUNKS + 255) / 256;   // 20 (the last one on lanes 0-127 only)
typedef unsigned int att_u32x4 __attribute__((ext_vector_type(4)));  // (a HIP uint4 array stayed in scratch)

// (Diagnostic builds only, rc_diag_set_attention: measured 92.4 vs 75.3 us per launch for v2 —
// two blocks of 4 waves per CU leave the latency-bound math too few waves, and each item's
// barrier waits for the wave with the 13th query tile; profiles/r05/.)
template <int TOK>
__global__ __launch_bounds__(256, 2) void attention_v3_kernel(const uint16_t *__restrict__ qkv, uint16_t *__restrict__ out,
                                                          int tokens_rt, int heads, int items, float scale_log2e) {
    constexpr int W = 4, HD = 64, TB = ATT2_ROWS * 128;  // waves, head dim, bytes per staged tensor
    const int tokens = TOK > 0 ? TOK : tokens_rt;
    __shared__ __attribute__((aligned(16))) uint8_t lds[3 * TB];  // Q | K | V
    const uint8_t *Qs = lds, *Ks = lds + TB, *Vs = lds + 2 * TB;
    const int H = heads * HD, H3 = 3 * H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int nqt = (tokens + 15) / 16;

    // chunk c = tid + 256 i: tensor c / (208·8) (0 Q, 1 K, 2 V; the tensors sit at column
    // offsets 0, H, 2H of a qkv row), row (c / 8) % 208, 16-B column chunk c % 8 — eight lanes
    // read one 128-B row segment; rows >= tokens re-read the last token (finite, masked later)
    // (tensor ts, row r) of chunk i: 208·8 = 6.5·256, so ts and r follow from compares; the
    // column chunk is tid & 7 for every i
    const int ch = tid & 7;
    // (lanes past the last chunk, i = 19, tid >= 128, re-load the last chunk: every pf[i] is loaded
    // on every lane — no conditional load, which made hipcc keep pf in scratch — and only stored
    // where it is real)
    auto chunk_rows = [&](int i, int &ts, int &r) __attribute__((always_inline)) {
        const int c = min(tid + 256 * i, ATT3_CHUNKS - 8 + ch);
        ts = (c >= ATT2_ROWS * 8) + (c >= 2 * ATT2_ROWS * 8);
        r = (c - ts * (ATT2_ROWS * 8)) >> 3;
    };
    att_u32x4 pf[ATT3_PER_LANE];
    auto load_item = [&](int item) __attribute__((always_inline)) {
        const int img = item / heads, h = item - img * heads;
        const uint16_t *base = qkv + (int64_t)img * tokens * H3 + h * HD + ch * 8;
#pragma unroll
        for (int i = 0; i < ATT3_PER_LANE; ++i) {
            int ts, r;
            chunk_rows(i, ts, r);
            const int rr = r < tokens ? r : tokens - 1;
            pf[i] = *reinterpret_cast<const att_u32x4 *>(base + (int64_t)rr * H3 + ts * H);
        }
    };
    // source chunk ch of row r goes to 16-B slot ch ^ s(r): s = (r >> 1) & 7 for Q and K (the
    // att_scores fragment reads), ((r >> 1) & 3) << 1 for V (the transposed P·V reads)
    auto store_item = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < ATT3_PER_LANE; ++i) {
            int ts, r;
            chunk_rows(i, ts, r);
            const int slot = ts == 2 ? (ch ^ (((r >> 1) & 3) << 1)) : (ch ^ ((r >> 1) & 7));
            if (i < ATT3_PER_LANE - 1 || tid < ATT3_CHUNKS - 256 * (ATT3_PER_LANE - 1))
                *reinterpret_cast<att_u32x4 *>(lds + ts * TB + r * 128 + slot * 16) = pf[i];
        }
    };

    int item = blockIdx.x;
    if (item >= items) return;  // (the host launches at most `items` blocks)
    load_item(item);
    store_item();
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int nxt = item + gridDim.x;  // block-uniform
        if (nxt < items) load_item(nxt);   // lands under this item's math
        const int img = item / heads, h = item - img * heads;
        uint16_t *obase = out + (int64_t)img * tokens * H + h * HD;
        for (int qt = wave; qt < nqt; qt += W) {
            bf16x8 qf[2];
            const int q = qt * 16 + li;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int c = s * 4 + g;
                qf[s] = *reinterpret_cast<const bf16x8 *>(Qs + q * 128 + ((c ^ ((q >> 1) & 7)) << 4));
            }
            f32x4 st[ATT2_TILES];
            float sum = 0.f;
            att_scores<TOK>(Ks, qf, tokens, scale_log2e, st, sum);
            att_pv_store(Vs, st, sum, qt, tokens, obase, H);
        }
        __syncthreads();  // every wave is done reading this item from LDS
        if (nxt < items) {
            store_item();
            __syncthreads();
        }
    }
}

// ------------------------------------------------- last layer, CLS rows only
// /embed returns last_hidden_state[:, 0, :] (embedding/main.py:113-114), and in
// the last encoder layer (modeling_vit_msn.py:254-283) row 0 of an image depends
// only on its own query row plus every token's K and V.  So the last layer runs
// LN1 + QKV over all rows, then attention for the CLS query alone and O-proj /
// LN2 / MLP on the n CLS rows gathered into a compact [n][768] stream.

// hc[i][:] = hidden[i * tokens][:]   (one block of 192 lanes per image, float4)
// With hc_ln: also the CLS rows' bf16 hi and LN statistics, compact (the A operand and
// row scales of the last layer's CLS-only Q GEMM).
__global__ __launch_bounds__(192) void gather_cls_kernel(const float *__restrict__ hidden, const uint16_t *__restrict__ hi,
                                                        int tokens, float *__restrict__ hc,
                                                        uint16_t *__restrict__ hc_ln, const float *__restrict__ st,
                                                        float *__restrict__ hc_st) {
    constexpr int H = 768;
    const int img = blockIdx.x;
    const int64_t r0 = (int64_t)img * tokens * H;
    if (hc_ln != nullptr) {
        reinterpret_cast<uint2 *>(hc_ln + (int64_t)img * H)[threadIdx.x] = reinterpret_cast<const uint2 *>(hi + r0)[threadIdx.x];
        if (threadIdx.x < LN_STRIDE)
            hc_st[img * LN_STRIDE + threadIdx.x] = st[(int64_t)img * tokens * LN_STRIDE + threadIdx.x];
    }
    reinterpret_cast<float4 *>(hc + (int64_t)img * H)[threadIdx.x] =
        hi ? rs_load4(hi + r0 + 4 * threadIdx.x)
           : reinterpret_cast<const float4 *>(hidden + r0)[threadIdx.x];
}

// CLS-query attention, one wave per (image, head), tokens <= 256, head dim 64.
// Numerics follow attention_v2_kernel: f32 dot products of the bf16 q/k rows,
// p = exp2(s·c − max·c) with c = log2(e)/8, P rounded to bf16 for P·V, f32 sum
// of the unrounded p, out = (P·V)·(1/sum) rounded to bf16.
// Scores: lane j owns keys j, j+64, j+128, j+192 (16-B loads of its key row);
// P·V: 8 lanes per V row, 8 rows per load instruction (see below).
// q != null: the CLS query rows come compact ([images][H], the last layer's Q computed
// for the CLS rows only) instead of from qkv.
__global__ __launch_bounds__(256) void attention_cls_kernel(const uint16_t *__restrict__ qkv, uint16_t *__restrict__ out,
                                                           int tokens, int heads, int items, float scale_log2e,
                                                           const uint16_t *__restrict__ qc) {
    constexpr int HD = 64, MAXT = 256;
    __shared__ float ps[4][MAXT];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + w;
    const bool live = item < items;
    const int img = live ? item / heads : 0, h = live ? item % heads : 0;
    const int H = heads * HD, H3 = 3 * H;
    const uint16_t *base = qkv + (int64_t)img * tokens * H3 + h * HD;
    float sum = 0.f;
    if (live) {
        float q[HD];
        const uint4 *q4 = reinterpret_cast<const uint4 *>(qc ? qc + (int64_t)img * H + h * HD : base);
#pragma unroll
        for (int i = 0; i < HD / 8; ++i) {
            const uint4 u = q4[i];
            const uint32_t wv[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                q[8 * i + 2 * j] = __uint_as_float(wv[j] << 16);
                q[8 * i + 2 * j + 1] = __uint_as_float(wv[j] & 0xffff0000u);
            }
        }
        float s[MAXT / 64];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < MAXT / 64; ++j) {
            const int t = lane + 64 * j;
            s[j] = -INFINITY;
            if (t < tokens) {
                const uint4 *k4 = reinterpret_cast<const uint4 *>(base + (int64_t)t * H3 + H);
                float acc = 0.f;
#pragma unroll
                for (int i = 0; i < HD / 8; ++i) {
                    const uint4 u = k4[i];
                    const uint32_t wv[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        acc = fmaf(q[8 * i + 2 * e], __uint_as_float(wv[e] << 16), acc);
                        acc = fmaf(q[8 * i + 2 * e + 1], __uint_as_float(wv[e] & 0xffff0000u), acc);
                    }
                }
                s[j] = acc;
                mx = fmaxf(mx, acc);
            }
        }
        mx = wave_max(mx);
        const float nmc = -mx * scale_log2e;
#pragma unroll
        for (int j = 0; j < MAXT / 64; ++j) {
            const int t = lane + 64 * j;
            if (t < tokens) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[j], scale_log2e, nmc));
                sum += p;
                ps[w][t] = (float)(__bf16)p;
            }
        }
        sum = wave_sum(sum);
    }
    __syncthreads();
    if (!live) return;
    // P·V: lane (grp, c8) accumulates dims 8·c8 .. 8·c8+7 over keys t ≡ grp (mod 8), one
    // 16-B load per key (a wave reads 8 whole V rows per instruction, 8 in flight per
    // lane); the 8 key groups are then summed across lanes.
    const int grp = lane >> 3, c8 = lane & 7;
    const uint16_t *vb = base + 2 * H + c8 * 8;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll 8
    for (int t = grp; t < tokens; t += 8) {
        const uint4 u = *reinterpret_cast<const uint4 *>(vb + (int64_t)t * H3);
        const float p = ps[w][t];
        const uint32_t wv[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            o[2 * e] = fmaf(p, __uint_as_float(wv[e] << 16), o[2 * e]);
            o[2 * e + 1] = fmaf(p, __uint_as_float(wv[e] & 0xffff0000u), o[2 * e + 1]);
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 8);
        o[e] += __shfl_xor(o[e], 16);
        o[e] += __shfl_xor(o[e], 32);
    }
    if (grp == 0) {
        const float inv = 1.0f / sum;
        *reinterpret_cast<uint4 *>(out + (int64_t)img * H + h * HD + c8 * 8) =
            make_uint4(pack_bf16x2(o[0] * inv, o[1] * inv), pack_bf16x2(o[2] * inv, o[3] * inv),
                       pack_bf16x2(o[4] * inv, o[5] * inv), pack_bf16x2(o[6] * inv, o[7] * inv));
    }
}

// ---------------------------------------------------------------- preprocess
// Pillow 8bpc separable resample (horizontal then vertical), fixed point 22 bits.
__device__ __forceinline__ uint8_t clip8_fixed(int acc) {
    int v = acc >> 22;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// src [n, H, W, 3] rows [y0, y0+Hs) → tmp [n, Hs, OW, 3]
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t *__restrict__ src, int H, int W, int y0, int Hs,
                                                      uint8_t *__restrict__ dst, int OW, const int *__restrict__ bounds,
                                                      const int *__restrict__ coef, int ks, int n) {
    const int64_t total = (int64_t)n * Hs * OW;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int x = (int)(i % OW);
        const int64_t t = i / OW;
        const int y = (int)(t % Hs), img = (int)(t / Hs);
        const int xmin = bounds[2 * x], xn = bounds[2 * x + 1];
        const uint8_t *row = src + (((int64_t)img * H + y0 + y) * W + xmin) * 3;
        int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
        for (int k = 0; k < xn; ++k) {
            const int c = coef[x * ks + k];
            a0 = resample_tap(a0, row[3 * k], c);
            a1 = resample_tap(a1, row[3 * k + 1], c);
            a2 = resample_tap(a2, row[3 * k + 2], c);
        }
        uint8_t *o = dst + i * 3;
        o[0] = clip8_fixed(a0);
        o[1] = clip8_fixed(a1);
        o[2] = clip8_fixed(a2);
    }
}

// src [n, Hs, W, 3] → dst [n, OH, W, 3]
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t *__restrict__ src, int Hs, int W,
                                                      uint8_t *__restrict__ dst, int OH, const int *__restrict__ bounds,
                                                      const int *__restrict__ coef, int ks, int n) {
    const int64_t total = (int64_t)n * OH * W;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int x = (int)(i % W);
        const int64_t t = i / W;
        const int y = (int)(t % OH), img = (int)(t / OH);
        const int ymin = bounds[2 * y], yn = bounds[2 * y + 1];
        const uint8_t *col = src + (((int64_t)img * Hs + ymin) * W + x) * 3;
        int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
        for (int k = 0; k < yn; ++k) {
            const int c = coef[y * ks + k];
            const uint8_t *p = col + (int64_t)k * W * 3;
            a0 = resample_tap(a0, p[0], c);
            a1 = resample_tap(a1, p[1], c);
            a2 = resample_tap(a2, p[2], c);
        }
        uint8_t *o = dst + i * 3;
        o[0] = clip8_fixed(a0);
        o[1] = clip8_fixed(a1);
        o[2] = clip8_fixed(a2);
    }
}

// u8 [n, S, S, 3] → f32 pixel_values [n, 3, S, S] (what ViTImageProcessor returns)
__global__ __launch_bounds__(256) void pixel_values_kernel(const uint8_t *__restrict__ img, const float *__restrict__ lut,
                                                          float *__restrict__ out, int n, int S) {
    const int64_t total = (int64_t)n * 3 * S * S;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int x = (int)(i % S);
        const int64_t t = i / S;
        const int y = (int)(t % S);
        const int64_t t2 = t / S;
        const int c = (int)(t2 % 3), b = (int)(t2 / 3);
        out[i] = lut[c * 256 + img[(((int64_t)b * S + y) * S + x) * 3 + c]];
    }
}

}  // namespace rc
