// gemm.h — the projection GEMMs of ViT-MSN (QKV, O, fc1, fc2, patch embed) on
// CDNA4 matrix cores: C[M][N] = A[M][K] · W[N][K]ᵀ + bias, bf16 in, f32 accumulate,
// fused epilogues (bf16 store, exact-erf GELU, f32 residual add, patch→token scatter
// + position embedding).
//
// Tile BM x 256 x 64 (BM = 256 or 128), 512 threads = 8 waves as 2 (M) x 4 (N);
// each wave owns (BM/2) x 64 outputs = (BM/32) x 4 tiles of mfma_f32_16x16x32_bf16.
// The MFMA operand roles are swapped — A-operand = weight rows, B-operand =
// activation rows — so a lane's accumulator holds 4 CONSECUTIVE output columns
// of one row: the epilogue reads bias/residual/pos as float4 and stores 8 B
// (bf16) or 16 B (f32) per lane.
// Staging: global_load_lds_dwordx4 into a 2-deep LDS ring, rows of 128 B with the
// 16-B chunk XOR-swizzled by (row>>1)&7 (conflict-free ds_read_b128 fragments;
// swizzle applied to the per-lane SOURCE address, LDS destination lane-linear).
// One raw s_barrier per K-step behind an explicit vmcnt(0): the next K-tile's
// DMA is issued before this K-tile's MFMAs and lands under them.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "vit_kernels.h"

namespace rc {

constexpr int G2_BN = 256, G2_BK = 64;

// Exact-erf GELU, x·Φ(x), evaluated as x·σ(x·P(x²)): Φ(x) = σ(logit Φ(x)) and
// logit Φ is odd, so x·P(x²) with P a degree-4 minimax fit on |x| <= 6.5
// (max |Δ Φ| 1.4e-6; max |Δ GELU| 6.3e-6 over all f32 x, checked in
// tests/test_gemm_gpu.py against torch's erf GELU).  x² is clamped at 42.25,
// where Φ = 1 - 8e-11 and P > 0 keeps σ saturated; for x -> -inf the exp2
// overflows to +inf and x·rcp(inf) = -0.  One exp2 + one rcp per element
// (the A&S 7.1.26 erf this replaces needed an exp, an rcp and twice the FMAs:
// fc1 GELU epilogue 60 us of a 288 us launch, tools/gemm_calib.py ablation 116).
// Coefficients are pre-scaled by -log2(e): exp2(x·P'(u)) = exp(-x·P(u)).
constexpr float GELU_P0 = -2.302165355e+00f, GELU_P1 = -1.050059413e-01f, GELU_P2 = 2.534135658e-04f,
                GELU_P3 = 1.058749684e-04f, GELU_P4 = -4.111701558e-06f, GELU_UMAX = 42.25f;

__device__ __forceinline__ float gelu_fast(float x) {
    const float u = fminf(x * x, GELU_UMAX);
    float p = fmaf(GELU_P4, u, GELU_P3);
    p = fmaf(p, u, GELU_P2);
    p = fmaf(p, u, GELU_P1);
    p = fmaf(p, u, GELU_P0);
    const float e = __builtin_amdgcn_exp2f(x * p);
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// The same on two values with packed f32 math (v_pk_mul_f32 / v_pk_fma_f32 /
// v_pk_add_f32); exp2 / rcp stay per element.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
    f32x2 u = x * x;
    u = f32x2{fminf(u.x, GELU_UMAX), fminf(u.y, GELU_UMAX)};
    f32x2 p = u * GELU_P4 + GELU_P3;
    p = p * u + GELU_P2;
    p = p * u + GELU_P1;
    p = p * u + GELU_P0;
    const f32x2 y = x * p;
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + 1.0f;
    return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// 16-B store with the non-temporal (streaming) hint
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ void nt_store16(T *dst, const T &v) {
    static_assert(sizeof(T) == 16, "16-byte values");
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4 *>(dst));
}

// f32 epilogues (residual add / patch scatter + position embedding, optionally the bf16
// copy and LayerNorm partials), straight from the accumulators — no LDS, no barrier.
// One wave, NR output rows per lane (rows[r]: lane li's row of row slot r, the same for
// its four 16-lane groups g), each as two 32-column chunks c of the wave's 64 columns
// [colw, colw + 64): A[r][c][h] = columns colw + 32c + 16h + 4g + 0..3 (the tiled kernels'
// swapped-operand accumulator layout).  One v_permlane16_swap per accumulator register
// pair gives lane g the 8 consecutive columns colw + 32c + ln_slice_col(g) — 16-B loads and
// stores, and exactly the canonical LayerNorm slice of the lane (LN_PARTS), so the block
// partial is two more swaps (ln_block_reduce_rows).  bq: the bias of those 8 columns.
// Values: x = (acc + bias) + residual (or + position), the skinny kernel's order.  BS: the
// residual stream is bf16 in a.ln_x (the statistics from the rounded values); otherwise f32
// a.out_f32, plus the bf16 copy in a.ln_x and the partials when a.ln_x is set.  All lanes run the swaps; rows
// >= mlim (M, or the end of an image-aligned tile's image) load a clamped row and store nothing.
// ABL (diagnostic builds): 1024 = the residual read nontemporal, 2048 = the stores nontemporal
template <int EPI, int NR, int ABL = 0>
__device__ __forceinline__ void f32_rows_epilogue(const GemmArgs &a, const f32x4 (&A)[NR][2][2], const int (&rows)[NR],
                                                  int colw, int g, const float4 (&bq)[2][2], int mlim) {
    constexpr bool BS = epi_bf16_stream(EPI);
    const bool stats = BS ? a.ln_stats != nullptr : a.ln_x != nullptr;
    const int cl = ln_slice_col(g, 0);
    // every source load of the NR rows first (16 B each), then the arithmetic and stores
    uint4 sh[NR][2];
    float4 sf[NR][2][2];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int rr = rows[r] < mlim ? rows[r] : mlim - 1;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int col = colw + 32 * c + cl;
            if constexpr (epi_resid(EPI)) {
                const int64_t off = (int64_t)rr * a.N + col;
                if constexpr (BS) {
                    if constexpr ((ABL & 1024) != 0)
                        sh[r][c] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.ln_x + off)));
                    else
                        sh[r][c] = *reinterpret_cast<const uint4 *>(a.ln_x + off);
                } else {
                    sf[r][c][0] = *reinterpret_cast<const float4 *>(a.out_f32 + off);
                    sf[r][c][1] = *reinterpret_cast<const float4 *>(a.out_f32 + off + 4);
                }
            } else {
                const int p = rr % (a.tokens - 1);
                const float *pr = a.pos + (int64_t)(1 + p) * a.N + col;
                sf[r][c][0] = *reinterpret_cast<const float4 *>(pr);
                sf[r][c][1] = *reinterpret_cast<const float4 *>(pr + 4);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int row = rows[r];
        int64_t orow = row;
        if constexpr (epi_patch(EPI)) {
            const int np = a.tokens - 1;
            const int img = row / np, p = row - img * np;
            orow = (int64_t)img * a.tokens + 1 + p;
        }
        const bool ok = row < mlim;
        float xs[16];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(A[r][c][0][j]),
                                                                 __float_as_uint(A[r][c][1][j]), false, false);
                v[j] = __uint_as_float(sw[0]);
                v[4 + j] = __uint_as_float(sw[1]);
            }
            const float b[8] = {bq[c][0].x, bq[c][0].y, bq[c][0].z, bq[c][0].w,
                                bq[c][1].x, bq[c][1].y, bq[c][1].z, bq[c][1].w};
            float add[8];
            if constexpr (EPI == EPI_RESID_BF16) {
                bf16x8_unpack(sh[r][c], add);
            } else {
                const float4 s0 = sf[r][c][0], s1 = sf[r][c][1];
                add[0] = s0.x, add[1] = s0.y, add[2] = s0.z, add[3] = s0.w;
                add[4] = s1.x, add[5] = s1.y, add[6] = s1.z, add[7] = s1.w;
            }
            float x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = (v[k] + b[k]) + add[k];
            const int64_t off = orow * a.N + colw + 32 * c + cl;
            if constexpr (BS) {
                const uint4 h = bf16x8_pack(x);
                if constexpr ((ABL & 2048) != 0) {
                    if (ok) nt_store16(reinterpret_cast<uint4 *>(a.ln_x + off), h);
                } else {
                    if (ok) *reinterpret_cast<uint4 *>(a.ln_x + off) = h;
                }
                float xv[8];
                bf16x8_unpack(h, xv);
#pragma unroll
                for (int k = 0; k < 8; ++k) xs[8 * c + k] = xv[k];
            } else {
                if (ok) {
                    *reinterpret_cast<float4 *>(a.out_f32 + off) = make_float4(x[0], x[1], x[2], x[3]);
                    *reinterpret_cast<float4 *>(a.out_f32 + off + 4) = make_float4(x[4], x[5], x[6], x[7]);
                    if (stats) *reinterpret_cast<uint4 *>(a.ln_x + off) = bf16x8_pack(x);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) xs[8 * c + k] = x[k];
            }
        }
        if (stats) {  // LayerNorm fold producer: this row's partial of the wave's 64-column block
            const float2 st = ln_block_reduce_rows(ln_slice_stats(xs));
            if (ok && g == 0) *reinterpret_cast<float2 *>(a.ln_stats + orow * LN_STRIDE + 2 * (colw >> 6)) = st;
        }
    }
}

// Epilogue of the BM x 256 tile the 8 waves of gemm_pp_kernel hold as acc[mq][nq][mi][ni]
// (wave = grp * 4 + wc: rows grp*BM/2 + mq*64 + mi*16 + li, columns wc*64 + nq*32 + ni*16 +
// 4g + j; BM = 224 leaves acc[1][*][3][*] unused).  smem: the ring (>= 128 KB, every read and
// DMA of the K loop retired by its final barrier); ln_off: the LayerNorm-fold row scales
// (EPI_*_LN); biasr: the bf16 epilogues' bias, loaded before the K loop; mlim: rows >= mlim
// are not stored (M, or the end of an image-aligned tile's image).
template <int EPI, int ABL, int BM = 256, int NR = 4>
__device__ __forceinline__ void pp_epilogue(const GemmArgs &a, f32x4 (&acc)[2][2][4][2], uint8_t *smem, int ln_off,
                                            int m0, int n0, const float4 (&biasr)[2][2], int tid, int mlim) {
    static_assert(BM == 256 || (BM == 224 && epi_resid(EPI)), "224-row tiles: residual epilogues only");
    constexpr int HALF = BM / 2, MI1 = (HALF - 64) / 16;  // row blocks of quadrant mq = 1
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    // epilogue: acc[mq][nq][mi][ni][j] = C[m0 + grp*128 + mq*64 + mi*16 + li][n0 + wc*64 + nq*32 + ni*16 + 4g + j]
    // fc1 (GELU + LayerNorm-fold consumer): no LDS staging — bf16 pairs of 16-lane rows
    // swapped with v_permlane16_swap so each lane stores 16 B (8 consecutive columns);
    // lane (g, li) of rows 16-block holds columns 4g..4g+3 of both 16-column halves ni, the
    // swap of rows 1<->0 and 3<->2 between the ni halves makes them 8 contiguous columns.
    // (Also ABL 64 for the other bf16 epilogues, QKV's LN consumer included, in diagnostic builds.)
    // Round 6 measured fc1 through the LDS-staged path with its nontemporal 512-B row stores
    // (ABL 512): fc1 itself +1.5…6 us per launch, the fc2 after it −8 us, step +0.3 % (r06s, r06t)
    // — within the run-to-run spread, so fc1 keeps this form.
    constexpr bool DIRECT = (EPI == EPI_GELU_BF16_LN && (ABL & 512) == 0) || (epi_bf16_out(EPI) && (ABL & 64) != 0);
    if constexpr (DIRECT) {
        float4 bq[2][2], cq[2][2];
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int cl = wc * 64 + nq * 32 + ni * 16 + 4 * g;
                if constexpr (epi_ln(EPI)) {
                    bq[nq][ni] = *reinterpret_cast<const float4 *>(a.bias + n0 + cl);
                    cq[nq][ni] = *reinterpret_cast<const float4 *>(a.ln_c + n0 + cl);
                } else {
                    bq[nq][ni] = biasr[nq][ni];
                }
            }
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int rl = grp * 128 + mq * 64 + mi * 16 + li;
                const int row = m0 + rl;
                float2 r = make_float2(1.f, 0.f);
                if constexpr (epi_ln(EPI)) r = *reinterpret_cast<const float2 *>(smem + ln_off + rl * 8);
#pragma unroll
                for (int nq = 0; nq < 2; ++nq) {
                    uint32_t u[2][2];
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni) {
                        const f32x4 v4 = acc[mq][nq][mi][ni];
                        const float4 b4 = bq[nq][ni];
                        f32x2 lo, hi;
                        if constexpr (epi_ln(EPI)) {  // rstd·(acc − μ·c) + b′, as the staged epilogue
                            const float4 c4 = cq[nq][ni];
                            lo = f32x2{fmaf(r.x, v4[0], fmaf(r.y, c4.x, b4.x)), fmaf(r.x, v4[1], fmaf(r.y, c4.y, b4.y))};
                            hi = f32x2{fmaf(r.x, v4[2], fmaf(r.y, c4.z, b4.z)), fmaf(r.x, v4[3], fmaf(r.y, c4.w, b4.w))};
                        } else {
                            lo = f32x2{v4[0] + b4.x, v4[1] + b4.y};
                            hi = f32x2{v4[2] + b4.z, v4[3] + b4.w};
                        }
                        if constexpr (epi_gelu(EPI) && !(ABL & 16)) {
                            lo = gelu_fast2(lo);
                            hi = gelu_fast2(hi);
                        }
                        u[ni][0] = pack_bf16x2(lo.x, lo.y);
                        u[ni][1] = pack_bf16x2(hi.x, hi.y);
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const auto r2 = __builtin_amdgcn_permlane16_swap(u[0][h], u[1][h], false, false);
                        u[0][h] = r2[0];
                        u[1][h] = r2[1];
                    }
                    const int col = n0 + wc * 64 + nq * 32 + (g & 1) * 16 + (g >> 1) * 8;
                    if constexpr ((ABL & 8) != 0) {  // diagnostic: no C stores
                        asm volatile("" ::"v"(u[0][0]), "v"(u[0][1]), "v"(u[1][0]), "v"(u[1][1]));
                    } else if (row < mlim) {
                        uint4 *dst = reinterpret_cast<uint4 *>(a.out_bf16 + (int64_t)row * (a.ldc ? a.ldc : a.N) + col);
                        const uint4 val = make_uint4(u[0][0], u[0][1], u[1][0], u[1][1]);
                        if constexpr ((ABL & 32) != 0) nt_store16(dst, val);
                        else *dst = val;
                    }
                }
            }
        return;
    }
    if constexpr (epi_bf16_out(EPI)) {
        // Stage the 256x256 bf16 tile in LDS (512-B rows, 16-B chunk XOR (row & 31)),
        // then every wave stores whole 512-B row segments with 16-B stores.
        // (The K loop's final barrier retired every ds_read and DMA: LDS is free.)
        float2 lrs[2][4];  // LayerNorm fold: (rstd, -rstd*mu) of this lane's 8 rows
        if constexpr (epi_ln(EPI)) {
#pragma unroll
            for (int mq = 0; mq < 2; ++mq)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    lrs[mq][mi] = *reinterpret_cast<const float2 *>(smem + ln_off + (grp * 128 + mq * 64 + mi * 16 + li) * 8);
        }
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int cl = wc * 64 + nq * 32 + ni * 16 + 4 * g;  // tile-local column
                float4 bias, lc;
                if constexpr (epi_ln(EPI)) {
                    bias = *reinterpret_cast<const float4 *>(a.bias + n0 + cl);
                    lc = *reinterpret_cast<const float4 *>(a.ln_c + n0 + cl);
                } else {
                    bias = biasr[nq][ni];
                }
#pragma unroll
                for (int mq = 0; mq < 2; ++mq)
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi) {
                        const int rl = grp * 128 + mq * 64 + mi * 16 + li;
                        const f32x4 v4 = acc[mq][nq][mi][ni];
                        float v0, v1, v2, v3;
                        if constexpr (epi_ln(EPI)) {  // rstd·(acc − μ·c) + b′
                            const float2 r = lrs[mq][mi];
                            v0 = fmaf(r.x, v4[0], fmaf(r.y, lc.x, bias.x));
                            v1 = fmaf(r.x, v4[1], fmaf(r.y, lc.y, bias.y));
                            v2 = fmaf(r.x, v4[2], fmaf(r.y, lc.z, bias.z));
                            v3 = fmaf(r.x, v4[3], fmaf(r.y, lc.w, bias.w));
                        } else {
                            v0 = v4[0] + bias.x, v1 = v4[1] + bias.y, v2 = v4[2] + bias.z, v3 = v4[3] + bias.w;
                        }
                        if constexpr (epi_gelu(EPI) && !(ABL & 16)) {
                            const f32x2 lo = gelu_fast2(f32x2{v0, v1}), hi = gelu_fast2(f32x2{v2, v3});
                            v0 = lo.x;
                            v1 = lo.y;
                            v2 = hi.x;
                            v3 = hi.y;
                        }
                        const int off = rl * 512 + ((((cl >> 3) ^ (rl & 31))) << 4) + (cl & 7) * 2;
                        *reinterpret_cast<uint2 *>(smem + off) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
                    }
            }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int id = it * 512 + tid;
            const int rl = id >> 5, ch = id & 31;
            const uint4 v = *reinterpret_cast<const uint4 *>(smem + rl * 512 + ((ch ^ (rl & 31)) << 4));
            if constexpr ((ABL & 8) != 0) {
                asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
            } else if (m0 + rl < mlim) {
                uint4 *dst = reinterpret_cast<uint4 *>(a.out_bf16 + (int64_t)(m0 + rl) * (a.ldc ? a.ldc : a.N) + n0 + ch * 8);
                // nontemporal: whole 512-B row segments stream out without allocating in L2, where
                // they would evict the A / W panels the next tiles read (QKV at batch 256: reads
                // 376 -> 348 MB, 181.5 -> 175.6 us per launch; round 6, r06q).  (fc1's direct
                // 64-B row pieces are not: nontemporal there raised its writes 311 -> 430 MB.)
                nt_store16(dst, v);
            }
        }
        return;
    }
    // f32 epilogues (residual add): straight from the accumulators, 4 rows per lane at a time
    float4 bq[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float *bp = a.bias + n0 + wc * 64 + 32 * c + ln_slice_col(g, 0);
        bq[c][0] = *reinterpret_cast<const float4 *>(bp);
        bq[c][1] = *reinterpret_cast<const float4 *>(bp + 4);
    }
    static_assert(NR == 1 || NR == 2 || NR == 4, "rows per lane per epilogue pass");
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int m4 = 0; m4 < 4; m4 += NR) {
            f32x4 A[NR][2][2];
            int rows[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int mi = m4 + r;
                // a row block past the tile (BM = 224: mq = 1, mi = 3) is masked like a row past M
                rows[r] = (mq == 1 && mi >= MI1) ? mlim : m0 + grp * HALF + mq * 64 + mi * 16 + li;
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int h = 0; h < 2; ++h) A[r][c][h] = acc[mq][c][mi][h];
            }
            f32_rows_epilogue<EPI, NR, ABL>(a, A, rows, n0 + wc * 64, g, bq, mlim);
        }
}

// ----------------------------------------------------------- ping-pong GEMM --
// BM x 256 x 64 tile (BM = 256, or 224 for image-aligned tiles), 8 waves in two groups:
// G0 = waves 0-3 (output rows 0 .. BM/2), G1 = waves 4-7 (rows BM/2 .. BM); wave w and w+4
// share a SIMD.  Each wave owns (BM/2) x 64 outputs as 4 quadrants of 64x32 (16 MFMAs per
// quadrant per K-tile; 12 in the mq = 1 quadrants of a 224-row tile).
// A K-tile is 4 phases; a phase is an M segment (ds_read this quadrant's
// fragments, issue this wave's LDS-DMA share of K-tile t+1, lgkmcnt(0)) and a
// C segment (16 MFMAs), each closed by a block barrier.  G1 runs one segment
// behind G0 (one extra barrier up front), so on every SIMD one wave's MFMAs
// overlap its partner's LDS reads / DMA issue / waits.  A wave's W fragments of a K-tile
// are read once (phases 0-1) and kept for both row quadrants (24 LDS reads per wave per
// K-tile instead of 32; round 4 in-model A/B: QKV 178.0 -> 175.3, fc1 274.5 -> 269.9, fc2
// 297.7 -> 294.4 us per launch).
// Hazards: DMA for t+1 goes to buffer (t+1)&1 only in phases 0-1 of K-tile t,
// after the barrier that closes both groups' last reads of K-tile t-1 (every M
// segment retires its ds_reads before its barrier); every wave waits vmcnt(0)
// in its phase-3 M segment, and the barrier after G1's phase-3 M segment
// precedes G0's first read of t+1.
// ABL (diagnostic builds only): bit0 = no DMA in the K loop, bit1 = no MFMA,
// bit2 = no epilogue (accumulators kept live), bit3 = no global stores in the
// bf16 epilogue (LDS staging kept), bit4 = no GELU.  ABL = 0 is the product kernel.
// NKT: K / 64 fixed at compile time for the model's shapes (12: QKV / O-proj / fc1,
// 48: fc2), 0 = from a.K.  It also names the launch: O-proj (EPI 6, NKT 12) and fc2
// (EPI 6, NKT 48) share an epilogue but are separate rows in a kernel trace.
constexpr int PP_BM = 256, PP_BK = 64, PP_STAGE = 2 * PP_BM * PP_BK * 2;  // A tile then W tile, 32 KB each
constexpr int PP_IMG_BM = 224;  // image-aligned tiles: 197 rows of one image in 14 row blocks of 16

// Diagnostic builds (tools/build_diag.sh) only: s_memrealtime stamps of a workgroup's phases
// into g_rc_stamps (set by rc_diag_set_stamps; tools/gemm_timeline.py reads them).  The
// product build compiles RC_STAMP to nothing.
#if defined(RC_GEMM_ABLATION)
static __device__ uint64_t *g_rc_stamps = nullptr;
#define RC_STAMP(idx, val)                                                 \
    do {                                                                    \
        if (g_rc_stamps != nullptr && threadIdx.x == 0) g_rc_stamps[idx] = (val); \
    } while (0)
#else
#define RC_STAMP(idx, val) \
    do {                   \
    } while (0)
#endif
#define RC_NOW() __builtin_amdgcn_s_memrealtime()

// XCD-aware bijective remap of blockIdx.x: blocks b, b + 8, ... share an XCD and get a
// contiguous run of ids
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
}
// tile id -> (row tile, column tile): row-major, or groups of group_m row tiles walked
// column-major inside a group
__device__ __forceinline__ void pp_tile_coords(const GemmArgs &a, int ntm, int tile, int &tm, int &tn) {
    const int ntn = a.N / PP_BM;
    tm = tile / ntn;
    tn = tile % ntn;
    if (a.group_m > 0) {
        const int gt = a.group_m * ntn, gi = tile / gt, in = tile - gi * gt;
        const int gm = min(a.group_m, ntm - gi * a.group_m);
        tm = gi * a.group_m + in % gm;
        tn = in / gm;
    }
}

// Prologue + K loop of one BM x 256 tile over the K-steps [kb, ke) (64 deep each), adding
// into acc (which the caller zeroes).  The ping-pong schedule described above.  smem: the
// 2-stage ring (2 * PP_STAGE) then, for the LayerNorm-fold consumers, the tile rows'
// (rstd, -rstd*mu) at 2 * PP_STAGE.  On return every wave has passed the loop's last barrier
// (the ring is free for the epilogue).
template <int EPI, int ABL, int BM>
__device__ __forceinline__ void pp_kloop(const GemmArgs &a, uint8_t *smem, int m0, int n0, int kb, int ke,
                                         f32x4 (&acc)[2][2][4][2], int tid, int64_t sb = -1) {
    constexpr int BK = PP_BK, A_BYTES = PP_BM * BK * 2, STAGE = PP_STAGE;
    constexpr int HALF = BM / 2, MI1 = (HALF - 64) / 16;  // row blocks of quadrant mq = 1
    constexpr int A_PIECES = BM / 8;                      // 1-KB pieces (8 rows x 128 B) of the A tile
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;

    // 64 pieces of 1 KB per K-tile (A: 0-31, W: 32-63); wave w owns pieces w + 8 i.  Piece rows
    // r = 8 w + 64 (i % 4) + lane / 8: the chunk swizzle (r >> 1) & 7 does not depend on i.  A
    // 224-row tile skips the A pieces past its rows (28-31: waves 4-7 at i = 3; wave-uniform).
    auto stage4 = [&](int buf, int k0, int i0) {
        uint8_t *base = smem + buf * STAGE;
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i) {
            const int piece = wave + 8 * i;
            const bool is_a = i < 4;
            if (is_a && piece >= A_PIECES) continue;
            const int r = (is_a ? piece : piece - 32) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            const uint16_t *src = (is_a ? Ag : Wg) + (int64_t)r * K + k0 + c * 8;
            // The residual producers' A operand (fc2: fc1's 310 MB output, each row panel read by its
            // three column tiles at about the same time) is staged nontemporal (aux 2), so it does not
            // displace W and the residual rows in L2 (round 6 in-model A/B: fc2 277.6 -> 264.9 us,
            // r06x); QKV / fc1 re-read their A panels over several rounds and keep the default
            // (ABL 4096, diagnostic: nontemporal for every GEMM: QKV 186 -> 200, fc1 294 -> 310 us)
            if (is_a && (epi_resid(EPI) || (ABL & 4096) != 0))
                __builtin_amdgcn_global_load_lds((const void *)src, (lds_void_t *)(base + piece * 1024), 16, 0, 2);
            else
                __builtin_amdgcn_global_load_lds((const void *)src, (lds_void_t *)(base + piece * 1024), 16, 0, 0);
        }
    };
    auto bar = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto kofs = [](int kt) { return kt * BK; };
    stage4(0, kofs(kb), 0);
    stage4(0, kofs(kb), 4);
    if constexpr (epi_ln(EPI)) {  // LayerNorm fold: this tile's row scales, under the first DMA
        if (tid < BM)
            *reinterpret_cast<float2 *>(smem + 2 * STAGE + tid * 8) =
                ln_row_scale(a.ln_stats + (int64_t)(m0 + tid) * LN_STRIDE, a.ln_eps);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (sb >= 0) RC_STAMP(sb, RC_NOW());
    if (grp == 1) bar();  // stagger: G1 one segment behind

    bf16x8 af[4][2], wf[2][2][2];  // [mi][s], [nq][ni][s]
#pragma nounroll
    for (int kt = kb; kt < ke; ++kt) {
        const int cur = (kt - kb) & 1;
        const uint8_t *As = smem + cur * STAGE;
        const uint8_t *Ws = As + A_BYTES;
        const bool more = kt + 1 < ke;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mq = p >> 1;                 // quadrant rows
            const int nq = (p == 1 || p == 2);     // snake: (0,0) (0,1) (1,1) (1,0)
            const int nmi = mq == 0 ? 4 : MI1;     // row blocks of this quadrant (compile-time)
            // ---- M segment
            if (p == 0 || p == 2) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        if (mi >= nmi) continue;
                        const int r = grp * HALF + mq * 64 + mi * 16 + li;
                        const int c = s * 4 + g;
                        af[mi][s] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
            if (p < 2) {
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int r = wc * 64 + nq * 32 + ni * 16 + li;
                        const int c = s * 4 + g;
                        wf[nq][ni][s] = *reinterpret_cast<const bf16x8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
            if (!(ABL & 1) && more && p < 2) stage4(cur ^ 1, kofs(kt + 1), p * 4);
            if (p == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            // ---- C segment
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni) {
                        if (mi >= nmi) continue;
                        if constexpr (!(ABL & 2))
                            acc[mq][nq][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nq][ni][s], af[mi][s],
                                                                                         acc[mq][nq][mi][ni], 0, 0, 0);
                        else
                            asm volatile("" ::"v"(wf[nq][ni][s]), "v"(af[mi][s]));
                    }
            __builtin_amdgcn_s_setprio(0);
            bar();
        }
    }
    if (grp == 0) bar();  // balance the stagger barrier
    if (sb >= 0) RC_STAMP(sb + 1, RC_NOW());
}

// bf16 epilogues: bias of this lane's 16 output columns, loaded before the K loop so its
// latency hides under the prologue wait (the other epilogues load their own)
template <int EPI>
__device__ __forceinline__ void pp_bias_regs(const GemmArgs &a, int n0, float4 (&biasr)[2][2], int tid) {
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16) {
        const int lane = tid & 63, g = lane >> 4;
        const int wc = __builtin_amdgcn_readfirstlane(tid >> 6) & 3;
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
                biasr[nq][ni] = *reinterpret_cast<const float4 *>(a.bias + n0 + wc * 64 + nq * 32 + ni * 16 + 4 * g);
    }
}

// BM = 256: row tile tm covers rows [256 tm, 256 tm + 256).  BM = 224 (image-aligned, a.row_step
// = tokens): row tile tm covers the rows of image tm, [tm·row_step, tm·row_step + row_step), so
// a batch of n images is n × N/256 tiles — for the N = 768 residual producers (O-proj, fc2)
// exactly 3 rounds of 256 CUs at n = 256, where 256-row tiles (197 × 3 = 591 tiles) left the
// third round 31 % full.  The extra rows a tile computes (224 − 197) are never stored.
template <int EPI, int ABL = 0, int NKT = 0, int BM = PP_BM>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs a) {
    // LayerNorm-fold consumers keep the tile rows' (rstd, -rstd*mu) behind the ring (one
    // __shared__ array: a second one would make hipcc drain the LDS-DMA queue every K-step)
    constexpr int LN_LDS = epi_ln(EPI) ? PP_BM * 8 : 0;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * PP_STAGE + LN_LDS];
    const int step = BM == PP_BM ? PP_BM : a.row_step;
    const int ntm = (a.M + step - 1) / step;
    int tm, tn;
    pp_tile_coords(a, ntm, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * step, n0 = tn * PP_BM;
    const int mlim = min(m0 + step, a.M);

    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
        for (int a1 = 0; a1 < 2; ++a1)
#pragma unroll
            for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
                for (int a3 = 0; a3 < 2; ++a3) acc[a0][a1][a2][a3] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t sb = (int64_t)blockIdx.x * 64;
    RC_STAMP(sb, RC_NOW());
    RC_STAMP(sb + 4, (uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) | ((uint64_t)__builtin_amdgcn_s_getreg(20 | (3 << 11)) << 32));
    RC_STAMP(sb + 5, (uint64_t)tm | ((uint64_t)tn << 32));
    if constexpr ((ABL & (128 | 256)) != 0) {
        // diagnostic: staggered start — the first round's workgroups on every other CU of an XCD
        // (block b runs on XCD b % 8, consecutive b / 8 on neighbouring CUs) wait ~half a tile, so
        // later rounds' epilogue store bursts fall beside other CUs' K loops
        constexpr uint64_t D = (ABL & 128) ? 1000 : 500;  // s_memrealtime ticks (100 MHz)
        if (blockIdx.x < 256 && ((blockIdx.x >> 3) & 1)) {
            const uint64_t t0 = RC_NOW();
            while (RC_NOW() - t0 < D) __builtin_amdgcn_s_sleep(8);
        }
    }
    float4 biasr[2][2];
    pp_bias_regs<EPI>(a, n0, biasr, threadIdx.x);
    pp_kloop<EPI, ABL, BM>(a, smem, m0, n0, 0, NKT > 0 ? NKT : a.K / PP_BK, acc, threadIdx.x, sb + 1);
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
        for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
            for (int a1 = 0; a1 < 2; ++a1)
#pragma unroll
                for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
                    for (int a3 = 0; a3 < 2; ++a3) asm volatile("" ::"v"(acc[a0][a1][a2][a3]));
        return;
    }
    pp_epilogue<EPI, ABL, BM>(a, acc, smem, 2 * PP_STAGE, m0, n0, biasr, threadIdx.x, mlim);
    RC_STAMP(sb + 3, RC_NOW());
}

// Epilogue of a 128 x 256 tile held as acc[mi][ni] by 4 waves (wave w: columns
// [64w, 64w + 64)): acc[mi][ni][j] = C[m0 + mi*16 + li][n0 + w*64 + ni*16 + 4g + j].
// The bf16 epilogues stage through `smem` (>= 64 KB; the caller's main loop must be done
// with it); the f32 ones store from the accumulators.  LayerNorm-fold consumers (EPI_*_LN): the
// tile rows' (rstd, -rstd*mu) at smem + ln_off, as gemm_pp_kernel keeps them, and the same
// rstd·(acc − μ·c) + b′ arithmetic (the same bits).
template <int EPI, int MI = 8, int ABL = 0>
__device__ __forceinline__ void w2_epilogue(const GemmArgs &a, f32x4 (&acc)[MI][4], uint8_t *smem, int m0, int n0,
                                            int ln_off = 0) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    if constexpr (epi_bf16_out(EPI)) {
        static_assert(MI == 8, "bf16 epilogues stage a 128-row tile");
        float4 bias[4], lc[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            bias[ni] = *reinterpret_cast<const float4 *>(a.bias + n0 + wave * 64 + ni * 16 + 4 * g);
            if constexpr (epi_ln(EPI)) lc[ni] = *reinterpret_cast<const float4 *>(a.ln_c + n0 + wave * 64 + ni * 16 + 4 * g);
        }
        __syncthreads();  // every wave's last fragment reads are done: the ring is free
        // 128 x 256 bf16 tile staged in LDS (512-B rows, 16-B chunk XOR (row & 31)),
        // stored as whole 512-B row segments, 16 B per lane.
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int cl = wave * 64 + ni * 16 + 4 * g;
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const int rl = mi * 16 + li;
                const f32x4 v4 = acc[mi][ni];
                float v0, v1, v2, v3;
                if constexpr (epi_ln(EPI)) {  // rstd·(acc − μ·c) + b′
                    const float2 r = *reinterpret_cast<const float2 *>(smem + ln_off + rl * 8);
                    v0 = fmaf(r.x, v4[0], fmaf(r.y, lc[ni].x, bias[ni].x));
                    v1 = fmaf(r.x, v4[1], fmaf(r.y, lc[ni].y, bias[ni].y));
                    v2 = fmaf(r.x, v4[2], fmaf(r.y, lc[ni].z, bias[ni].z));
                    v3 = fmaf(r.x, v4[3], fmaf(r.y, lc[ni].w, bias[ni].w));
                } else {
                    v0 = v4[0] + bias[ni].x, v1 = v4[1] + bias[ni].y, v2 = v4[2] + bias[ni].z, v3 = v4[3] + bias[ni].w;
                }
                if constexpr (epi_gelu(EPI)) {
                    const f32x2 lo = gelu_fast2(f32x2{v0, v1}), hi = gelu_fast2(f32x2{v2, v3});
                    v0 = lo.x;
                    v1 = lo.y;
                    v2 = hi.x;
                    v3 = hi.y;
                }
                const int off = rl * 512 + (((cl >> 3) ^ (rl & 31)) << 4) + (cl & 7) * 2;
                *reinterpret_cast<uint2 *>(smem + off) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
            }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int id = it * 256 + tid;
            const int rl = id >> 5, ch = id & 31;
            const uint4 v = *reinterpret_cast<const uint4 *>(smem + rl * 512 + ((ch ^ (rl & 31)) << 4));
            if (m0 + rl < a.M)
                *reinterpret_cast<uint4 *>(a.out_bf16 + (int64_t)(m0 + rl) * (a.ldc ? a.ldc : a.N) + n0 + ch * 8) = v;
        }
        return;
    }
    // f32 epilogues: straight from the accumulators (f32_rows_epilogue), 4 rows per lane at a time
    float4 bq[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float *bp = a.bias + n0 + wave * 64 + 32 * c + ln_slice_col(g, 0);
        bq[c][0] = *reinterpret_cast<const float4 *>(bp);
        bq[c][1] = *reinterpret_cast<const float4 *>(bp + 4);
    }
    // 4 rows per lane per pass; a 10-row-block tile (BM = 160) in passes of 2, fewer live registers
    // beside its 160 accumulator VGPRs
    static_assert(MI % 4 == 0 || MI % 4 == 2, "row blocks in passes of 4, or of 2");
    constexpr int N4 = MI % 4 == 0 ? MI / 4 : 0;
#pragma unroll
    for (int h4 = 0; h4 < N4; ++h4) {
        f32x4 A[4][2][2];
        int rows[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            rows[r] = m0 + (h4 * 4 + r) * 16 + li;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) A[r][c][h] = acc[h4 * 4 + r][2 * c + h];
        }
        f32_rows_epilogue<EPI, 4, ABL>(a, A, rows, n0 + wave * 64, g, bq, a.M);
    }
#pragma unroll
    for (int m2 = 4 * N4; m2 < MI; m2 += 2) {
        f32x4 A[2][2][2];
        int rows[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            rows[r] = m0 + (m2 + r) * 16 + li;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) A[r][c][h] = acc[m2 + r][2 * c + h];
        }
        f32_rows_epilogue<EPI, 2, ABL>(a, A, rows, n0 + wave * 64, g, bq, a.M);
    }
}

// ------------------------------------------------- two-workgroup GEMM ----
// 128 (rows) x 256 (cols) tile per 256-thread workgroup, TWO workgroups per CU.
// A 256x256 f32 accumulator tile fills half the CU's register file, so with one
// workgroup per CU the epilogue (bias / GELU / bf16 pack / stores, 35-40 % of an
// fc1 launch when measured alone) cannot overlap any matrix work.  Two
// independent 128x256 workgroups per CU desynchronise: one's epilogue (VALU,
// LDS staging, stores) runs beside the other's MFMA main loop on every SIMD.
// The price is 1.5x the L2->LDS bytes per flop, so the ring is 3 deep (two
// K-steps in flight per workgroup, ~96 KB per CU).
// Wave w owns all 128 rows x columns [64w, 64w+64): acc[mi][ni], 8 x 4 tiles of
// mfma_f32_16x16x32_bf16 with swapped operands (A-operand = weight rows), so a
// lane's accumulator holds 4 consecutive output columns of one row.
// LDS ring: 3 slots x (A 128 rows + W 256 rows) x 64 B (BK = 32).  A 64-B row
// holds 4 16-B chunks; chunk c of row r is stored at c ^ (((r >> 3) & 1) << 1),
// which makes the fragment ds_read_b128 conflict-free for gfx950's lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same in the upper half).
// Per K-step: wait for this slot's DMA (vmcnt(6): the next slot's 6 pieces may
// still be in flight), barrier, issue the DMA two slots ahead (into the slot
// every wave finished reading before the barrier), 12 fragment reads, 32 MFMAs.
// ABL (diagnostic builds only, as gemm_pp_kernel): bit0 no DMA in the K loop,
// bit1 no MFMA, bit2 no epilogue.
// BM = 160 (the residual epilogues of large M: 10 row blocks, acc[10][4], 78 KB of ring): a batch
// of 256 images is 316 x 3 = 948 tiles = 1.85 rounds of 512 workgroup slots, where 128-row tiles are
// 1 182 = 2.31 rounds (the third 31 % full); launch_gemm picks the BM with the fewer row-rounds.
template <int EPI, int ABL = 0, int BM = 128>
__global__ __launch_bounds__(256, 2) void gemm_w2_kernel(GemmArgs a) {
    constexpr int BN = 256, BK = 32, NSLOT = 3, MI = BM / 16;
    constexpr int A_BYTES = BM * BK * 2, SLOT = A_BYTES + BN * BK * 2;  // 8 (10) KB + 16 KB
    constexpr int PIECES = SLOT / 1024;                                  // 24 (26) pieces: A then W
    constexpr int PPW = (PIECES + 3) / 4, PPW_LO = PIECES / 4;           // pieces of waves < PIECES % 4 / the rest
    constexpr int LN_OFF = NSLOT * SLOT, LN_LDS = epi_ln(EPI) ? BM * 8 : 0;  // LN-fold row scales behind the ring
    static_assert(!epi_ln(EPI) || LN_OFF >= 64 * 1024, "the staged bf16 tile must not reach the row scales");
    __shared__ __attribute__((aligned(16))) uint8_t smem[NSLOT * SLOT + LN_LDS];  // 72 (78) KB (+ 1 KB)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;

    // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; each XCD gets a
    // contiguous run of tile ids, walked in groups of GM row blocks (column-major
    // inside a group) so co-resident tiles share A rows and W columns in its L2.
    const int ntn = a.N / BN, ntm = (a.M + BM - 1) / BM;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    constexpr int GM = 8;
    const int grp_tiles = GM * ntn, grp = t / grp_tiles, in = t - grp * grp_tiles;
    const int gm = min(GM, ntm - grp * GM);
    const int tm = grp * GM + in % gm, tn = in / gm;
    const int m0 = tm * BM, n0 = tn * BN;
    const int K = a.K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;

    // piece p (1 KB = 16 rows x 64 B): 0..MI-1 A rows 16p.., then W rows 16(p-MI)..
    // lane l writes LDS bytes [16 l, 16 l + 16) of the piece: row l >> 2, stored
    // chunk l & 3, which holds source chunk (l & 3) ^ (((l >> 5) & 1) << 1).
    // A rows past M are clamped to row M - 1 (their results are never stored): a 160-row tile
    // may reach past the round_up(M, 256) rows the ABI asks callers to provide.
    const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const uint16_t *srcp[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int piece = wave + 4 * i;  // wave-uniform
        srcp[i] = piece < MI ? a.A + (int64_t)min(m0 + piece * 16 + prow, a.M - 1) * K
                             : Wg + (int64_t)((piece - MI) * 16 + prow) * K;
        srcp[i] += pchunk * 8;
    }
    auto stage = [&](int slot, int k0) {
        uint8_t *base = smem + slot * SLOT;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = wave + 4 * i;  // wave-uniform
            if (piece >= PIECES) continue;
            if ((ABL & 4096) != 0 && piece < MI)  // diagnostic: the A operand's DMA nontemporal
                __builtin_amdgcn_global_load_lds((const void *)(srcp[i] + k0), (lds_void_t *)(base + piece * 1024), 16, 0, 2);
            else
                __builtin_amdgcn_global_load_lds((const void *)(srcp[i] + k0), (lds_void_t *)(base + piece * 1024), 16, 0, 0);
        }
    };
    // fragment of rows r0 + li (r0 % 16 == 0), k chunk g: 16 B at row*64 + (g ^ h(li))*16
    const int fchunk = (g ^ (((li >> 3) & 1) << 1)) << 4;

    f32x4 acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    stage(0, 0);
    if (nk > 1) stage(1, BK);
    if constexpr (epi_ln(EPI)) {  // this tile's row scales, as gemm_pp_kernel's prologue (visible after the loop's barriers)
        if (tid < BM)
            *reinterpret_cast<float2 *>(smem + LN_OFF + tid * 8) =
                ln_row_scale(a.ln_stats + (int64_t)min(m0 + tid, a.M - 1) * LN_STRIDE, a.ln_eps);
    }
    for (int kt = 0; kt < nk; ++kt) {
        // a raw s_barrier: __syncthreads() would add a full vmcnt(0) drain (its
        // release fence), emptying the DMA pipeline every K-step.  The next slot's pieces of this
        // wave may still fly: PPW, or PPW_LO for the waves with one piece fewer (wave-uniform).
        if (kt + 1 < nk) {
            if (PPW == PPW_LO || wave < PIECES % 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW_LO) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!(ABL & 1) && kt + 2 < nk) stage((kt + 2) % NSLOT, (kt + 2) * BK);
        const uint8_t *As = smem + (kt % NSLOT) * SLOT;
        const uint8_t *Ws = As + A_BYTES;
        bf16x8 wf[4], af[MI];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
            wf[ni] = *reinterpret_cast<const bf16x8 *>(Ws + (wave * 64 + ni * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
            af[mi] = *reinterpret_cast<const bf16x8 *>(As + (mi * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                if constexpr (!(ABL & 2))
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[mi][ni], 0, 0, 0);
                else
                    asm volatile("" ::"v"(wf[ni]), "v"(af[mi]));
        // all 4 + MI fragment reads first (in source order), then the 4·MI MFMAs: the
        // compiler's counted lgkmcnt waits let MFMA (mi, *) start once af[mi] lands
        __builtin_amdgcn_sched_group_barrier(0x100, 4 + MI, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * MI, 0);
    }

    if constexpr ((ABL & 4) != 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
    }
    w2_epilogue<EPI, MI, ABL>(a, acc, smem, m0, n0, LN_OFF);
}

// ------------------------------------------- implicit-GEMM patch embedding ----
// Conv2d(3, 768, 16, stride 16) (modeling_vit_msn.py:57) as C[m][n] = A[m][k]·W[n][k]ᵀ
// with m = (image, patch) and A never materialised: the K axis is ordered
// (ky, kx, c), so the 16 K-values a lane needs per step are 16 CONTIGUOUS bytes of
// one image row (48 bytes per patch row in HWC), and the weight matrix is permuted
// to the same order once at finalize (W′[n][(ky·P + kx)·3 + c] = W[n][c][ky][kx]).
// Each byte u of channel c becomes bf16(fma(u, pre_a[c], pre_b[c])): rc_model picks the
// f32 pair (pre_a, pre_b) so that this equals, for every u, the bf16 of ViTImageProcessor's
// f32 rescale→normalize value — exactly the values the im2col kernel once wrote and the
// [3][256] LDS table after it read (round 2: 52 % of that kernel's LDS cycles were bank
// conflicts of the table's random-address reads; now the conversion is VALU only).
// 128 x 256 tile, 4 waves (as gemm_w2_kernel, whose fragment layout and epilogue it
// shares), two workgroups per CU; both operands register-staged (one 16-B A load
// and four 16-B W loads per lane per 32-deep K-step, issued two steps ahead and
// written to the other LDS slot after the MFMAs of the step before their own).
// EPI: EPI_PATCH_F32 or EPI_PATCH_BF16 (the residual stream in bf16).
template <int P, int EPI>
__global__ __launch_bounds__(256, 2) void patch_gemm_kernel(GemmArgs a) {
    constexpr int BM = 128, BN = 256, BK = 32, KC = 3 * P * P;
    constexpr int A_BYTES = BM * BK * 2, SLOT = A_BYTES + BN * BK * 2;  // 8 KB + 16 KB
    static_assert(2 * SLOT <= 64 * 1024, "ring within the epilogue's 64 KB");
    __shared__ __attribute__((aligned(16))) uint8_t smem[64 * 1024];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;

    const int ntn = a.N / BN, ntm = (a.M + BM - 1) / BM;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    constexpr int GM = 8;
    const int grp_tiles = GM * ntn, grp = t / grp_tiles, in = t - grp * grp_tiles;
    const int gm = min(GM, ntm - grp * GM);
    const int tm = grp * GM + in % gm, tn = in / gm;
    const int m0 = tm * BM, n0 = tn * BN;

    // A: lane pair (row ar, half ah) loads K [32 kt + 16 ah, +16) of patch row m0 + ar
    const int S = a.img_size, gp = S / P, np = gp * gp;
    const int ar = tid >> 1, ah = tid & 1;
    const int m = min(m0 + ar, a.M - 1);  // rows past M re-read the last patch (results unused)
    const int b = m / np, pi = m - b * np, py = pi / gp, px = pi - py * gp;
    const uint8_t *abase = a.img + (((int64_t)b * S + py * P) * S + px * P) * 3;
    const int arow_stride = S * 3;
    // W: thread t stages 16-B chunk (t & 3) of rows (t >> 2) + 64 i, i = 0..3: four lanes
    // cover a 64-B row, so each ds_write_b128 of a wave writes 16 rows x 64 B whole —
    // conflict-free (one row per lane wrote 4 rows at a 64-B stride into the same banks:
    // 2-way conflicts on every W store, 46 % of the kernel's LDS cycles, r03b PMC)
    const int wch = tid & 3, wr0 = tid >> 2;
    const uint16_t *wrow = a.W + (int64_t)(n0 + wr0) * KC + wch * 8;
    // chunk XOR of row r: bit 3 of r -> chunk bit 1, bit 1 of r -> chunk bit 0.  The fragment reads
    // (ds_read_b128, rows li of 16-row blocks) stay conflict-free, and so do the A stores: a
    // ds_write_b128 lane group of 8 covers rows ar..ar+3, whose 64-B rows alias mod 128 B in
    // pairs (0/2, 1/3) without the bit-1 term (2-way on every A store, r03e PMC)
    auto swz = [](int r) { return (((r >> 3) & 1) << 1) | ((r >> 1) & 1); };
    const int asw = swz(ar), wsw = swz(wr0);  // rows wr0 + 64 i share bits 1 and 3

    // register staging two K-steps ahead: set R holds step kt + 2 while step kt + 1's
    // set is written to LDS, so each global load has two steps of MFMAs to land
    struct Regs {
        uint4 av, wv[4];
    };
    auto load = [&](int kt, Regs &r) {
        const int k0 = kt * BK + 16 * ah;
        const int ky = k0 / (3 * P), off = k0 - ky * (3 * P);
        r.av = *reinterpret_cast<const uint4 *>(abase + ky * arow_stride + off);
#pragma unroll
        for (int i = 0; i < 4; ++i) r.wv[i] = *reinterpret_cast<const uint4 *>(wrow + (int64_t)64 * i * KC + kt * BK);
    };
    auto store = [&](int slot, int kt, const Regs &r) {
        uint8_t *As = smem + slot * SLOT;
        uint8_t *Ws = As + A_BYTES;
        // channel of byte j is (c0 + j) % 3 with c0 = (32 kt + 16 ah) % 3 (k = ky·3P + kx·3 + c):
        // rotate the three (a, b) pairs once, then byte j takes pair j % 3 (a constant index)
        const int c0 = (2 * kt + ah) % 3;
        const float a0 = c0 == 0 ? a.pre_a[0] : (c0 == 1 ? a.pre_a[1] : a.pre_a[2]);
        const float a1 = c0 == 0 ? a.pre_a[1] : (c0 == 1 ? a.pre_a[2] : a.pre_a[0]);
        const float a2 = c0 == 0 ? a.pre_a[2] : (c0 == 1 ? a.pre_a[0] : a.pre_a[1]);
        const float b0 = c0 == 0 ? a.pre_b[0] : (c0 == 1 ? a.pre_b[1] : a.pre_b[2]);
        const float b1 = c0 == 0 ? a.pre_b[1] : (c0 == 1 ? a.pre_b[2] : a.pre_b[0]);
        const float b2 = c0 == 0 ? a.pre_b[2] : (c0 == 1 ? a.pre_b[0] : a.pre_b[1]);
        const float ra[3] = {a0, a1, a2}, rb[3] = {b0, b1, b2};
        const uint32_t w4[4] = {r.av.x, r.av.y, r.av.z, r.av.w};
        uint32_t o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int e = 2 * j;
            const float uA = (float)((w4[e >> 2] >> (8 * (e & 3))) & 0xffu);
            const float uB = (float)((w4[(e + 1) >> 2] >> (8 * ((e + 1) & 3))) & 0xffu);
            o[j] = pack_bf16x2(fmaf(uA, ra[e % 3], rb[e % 3]), fmaf(uB, ra[(e + 1) % 3], rb[(e + 1) % 3]));
        }
        *reinterpret_cast<uint4 *>(As + ar * 64 + (((2 * ah) ^ asw) << 4)) = make_uint4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<uint4 *>(As + ar * 64 + (((2 * ah + 1) ^ asw) << 4)) = make_uint4(o[4], o[5], o[6], o[7]);
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4 *>(Ws + (wr0 + 64 * i) * 64 + ((wch ^ wsw) << 4)) = r.wv[i];
    };
    const int fchunk = (g ^ swz(li)) << 4;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int nk = KC / BK;
    static_assert(nk % 2 == 0 && nk >= 2, "K steps are taken in pairs");
    Regs r0, r1;
    load(0, r0);
    load(1, r1);
    store(0, 0, r0);
    __syncthreads();
    // one K-step: the MFMAs on slot kt & 1, with `nxt` (step kt + 1) written to the
    // other slot afterwards and `fre` (step kt's set, already in LDS) reloaded with kt + 2
    auto step = [&](int kt, Regs &fre, const Regs &nxt) {
        if (kt + 2 < nk) load(kt + 2, fre);
        const uint8_t *As = smem + (kt & 1) * SLOT;
        const uint8_t *Ws = As + A_BYTES;
        bf16x8 wf[4], af[8];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
            wf[ni] = *reinterpret_cast<const bf16x8 *>(Ws + (wave * 64 + ni * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) af[mi] = *reinterpret_cast<const bf16x8 *>(As + (mi * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[mi][ni], 0, 0, 0);
        if (kt + 1 < nk) store((kt + 1) & 1, kt + 1, nxt);  // the slot step kt - 1 read (closed by the last barrier)
        __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, r0, r1);
        step(kt + 1, r1, r0);
    }
    w2_epilogue<EPI>(a, acc, smem, m0, n0);
}

// The skinny kernels' K chain: nk steps of 32, acc[ni] += W[ni]·A in k order (one dependent
// 16x16x32 MFMA per step, the order of every tiled kernel: the same bits), with the operands of
// the next D steps in flight in a register ring, so the chain waits for one step's loads while
// D − 1 more are on their way (a lone image's GEMMs are latency-bound: 197 rows give 300-1250
// waves for 1024 SIMDs).  NK > 0: the step count is a constant and the chain is straight-line
// code — in a loop the wait-count pass falls back to vmcnt(0) at the loop head, one full memory
// latency per trip.  NK = 0: any even nk, a 2-deep ring in a loop.
template <int NI, int NK, int D>
__device__ __forceinline__ void skinny_chain_t(const uint16_t *Ar, const uint16_t *Wr, int K, int nk, f32x4 (&acc)[NI]) {
    bf16x8 ra[D], rw[D][NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < D; ++d) {
        ra[d] = *reinterpret_cast<const bf16x8 *>(Ar + 32 * d);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) rw[d][ni] = *reinterpret_cast<const bf16x8 *>(Wr + (int64_t)ni * 16 * K + 32 * d);
    }
    auto step = [&](int st, bf16x8 &a_, bf16x8 (&w_)[NI], bool more) __attribute__((always_inline)) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w_[ni], a_, acc[ni], 0, 0, 0);
        if (more) {
            const int kn = 32 * (st + D);
            a_ = *reinterpret_cast<const bf16x8 *>(Ar + kn);
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) w_[ni] = *reinterpret_cast<const bf16x8 *>(Wr + (int64_t)ni * 16 * K + kn);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the ring: no load hoisted or sunk across steps
    };
    if constexpr (NK > 0) {
        static_assert(NK % D == 0, "ring depth divides the step count");
#pragma unroll
        for (int st = 0; st < NK; ++st) step(st, ra[st % D], rw[st % D], st + D < NK);
    } else {
        for (int kb = 0; kb < nk; kb += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) step(kb + d, ra[d], rw[d], kb + d + D < nk);
        }
    }
}
// The skinny K chain through an LDS-DMA ring (K = 768 / 3072): per 64-deep K block the wave copies
// its 16 A rows and 16·NI W rows, 128 B each, with global_load_lds_dwordx4 — 8 whole rows per
// instruction (8 full 128-B lines) where the register form's fragment loads touch 16 rows × 64 B
// (16 half lines) per instruction: the loads are address-bound (PMC), the bytes are not.  Rows
// are 128 B in LDS with the 16-B chunk XOR-swizzled by (row >> 1) & 7 on the source address
// (conflict-free ds_read_b128 fragments, as the tiled kernels).  The ring is SK stages deep (the
// copy of block kb + SK − 1 issued while block kb is consumed); one wave per ring, no barrier: a
// counted vmcnt says a block has landed, and its fragments are read with inline-asm ds_reads (as
// C++ loads hipcc would wait for the whole DMA ring first).  The MFMAs run in the same k order as
// every other kernel: the same bits.
constexpr int SKINNY_DMA_STAGES = 6;
// fc1 on the one-wave kernel keeps 5 stages: 30 KB of LDS per wave puts five waves on a CU (measured
// on a lone image's 1 248 fc1 tiles, before gemm_skinny_shared_kernel took them: six stages left a
// second round of 224 blocks; device time 436 -> 419 us, profiles/r06/r06ae_skinny_ring_depth_b1_ab.log).
// Deeper rings for the two-wave LayerNorm producers (10 stages) and five for QKV measured no better.
constexpr int SKINNY_FC1_STAGES = 5;
template <int NI>
constexpr int skinny_dma_stage_bytes() { return (16 + 16 * NI) * 128; }

template <int NI, int NKB, int SK = SKINNY_DMA_STAGES>
__device__ __forceinline__ void skinny_chain_dma(const uint16_t *__restrict__ A, int row_a0, int M, const uint16_t *__restrict__ W,
                                                 int n0, int K, uint8_t *ring, f32x4 (&acc)[NI]) {
    constexpr int SB = skinny_dma_stage_bytes<NI>(), NA = 2, NW = 2 * NI, NP = NA + NW;
    static_assert(NKB >= SK, "the ring is primed with SK - 1 blocks");
    static_assert((SK - 1) * NP <= 63 && SK <= 11, "the copies in flight fit the 6-bit vmcnt");
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    // copy sources: instruction i (A: i < 2, W: i >= 2) moves rows 8(i mod ..) + lane / 8, chunk lane % 8
    const uint16_t *src[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int r = (i < NA ? i : i - NA) * 8 + (lane >> 3);  // row within the A or W block
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const uint16_t *rowp = i < NA ? A + (int64_t)min(row_a0 + r, M - 1) * K : W + (int64_t)(n0 + r) * K;
        src[i] = rowp + c * 8;
    }
    auto issue = [&](int kb) __attribute__((always_inline)) {
        uint8_t *st = ring + (kb % SK) * SB;
#pragma unroll
        for (int i = 0; i < NP; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + kb * 64), (lds_void_t *)(st + i * 1024), 16, 0, 0);
    };
    // fragment addresses within a stage: A row li, W row 16 ni + li; logical chunk 4 s + g
    uint32_t fa[2], fw[2][NI];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const int c = (4 * s2 + g) ^ ((li >> 1) & 7);
        fa[s2] = (uint32_t)(li * 128 + c * 16);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) fw[s2][ni] = (uint32_t)((16 + 16 * ni + li) * 128 + c * 16);
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < SK - 1; ++kb) issue(kb);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        // block kb landed: younger copies in flight are those of blocks kb + 1 .. min(kb + SK - 2, NKB - 1)
        constexpr int X = NP;
        const int younger = min(SK - 2, NKB - 1 - kb);
        if (younger >= 9) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(9 * X) : "memory");
        else if (younger == 8) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * X) : "memory");
        else if (younger == 7) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * X) : "memory");
        else if (younger == 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * X) : "memory");
        else if (younger == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * X) : "memory");
        else if (younger == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * X) : "memory");
        else if (younger == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * X) : "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * X) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t st = (uint32_t)(uintptr_t)(ring + (kb % SK) * SB);
        bf16x8 a[2], w[2][NI];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            asm volatile("ds_read_b128 %0, %1" : "=v"(a[s2]) : "v"(st + fa[s2]));
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) asm volatile("ds_read_b128 %0, %1" : "=v"(w[s2][ni]) : "v"(st + fw[s2][ni]));
        }
        static_assert(NI == 2, "the wait below ties 2 + 4 fragments");
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1]));
        // the stage block kb - 1 used is free (its reads retired a block ago): refill it
        if (kb + SK - 1 < NKB) issue(kb + SK - 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
                acc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[s2][ni], a[s2], acc[ni], 0, 0, 0);
    }
}

// K (per chain) 768 / 3072: straight-line chains; otherwise the looped form (K % 64 == 0)
template <int NI, int KT>
__device__ __forceinline__ void skinny_chain(const uint16_t *Ar, const uint16_t *Wr, int K, int nk, f32x4 (&acc)[NI]) {
    if constexpr (KT > 0) skinny_chain_t<NI, KT / 32, 12>(Ar, Wr, K, nk, acc);
    else skinny_chain_t<NI, 0, 2>(Ar, Wr, K, nk, acc);
}

// Skinny GEMM for M <= 256 (the last layer's CLS rows: O-proj, fc1, fc2 with
// M = images in the slice).  A 256-row tile kernel would put the whole launch on
// N/256 CUs with the full K loop on each (fc2: 3 CUs x 3072-deep); here every
// wave owns 16 rows x 16·NI columns over the whole K, operands straight from
// global memory (W is 1.2-4.7 MB, L2-resident after the first row tile), so the
// launch spreads over ceil(M/16)·N/(16·NI) waves.  Swapped operands as in the
// tiled kernels: the A-operand is 16 weight rows, so lane (g, li) ends with
// activation row li, output columns 4g..4g+3 of each 16-column group.
// Block b runs on XCD b % 8; skinny_block(b) numbers the blocks so that each XCD gets one
// contiguous range (bijective), and tiles are numbered column-major — so the waves of a block
// (consecutive row tiles of one column tile) read the same weight rows at about the same time
// (L1 hits), and a column tile's weights are fetched into one XCD's L2 only (W is re-read by
// every row tile: 13x for a lone image's 197 rows).
__device__ __forceinline__ int skinny_block(int b, int nwg) {
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = b % 8;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
}

// The skinny kernels' epilogue (not the LayerNorm producers): lane (g, li) holds row `row`, columns
// n0 + 16 ni + 4g .. + 3 of acc[ni]
template <int EPI, int NI>
__device__ __forceinline__ void skinny_epilogue(const GemmArgs &a, const f32x4 (&acc)[NI], int row, int n0, int g) {
    float2 lrs;  // LayerNorm fold: this row's (rstd, -rstd*mu), as gemm_pp_kernel computes it
    if constexpr (epi_ln(EPI)) lrs = ln_row_scale(a.ln_stats + (int64_t)row * LN_STRIDE, a.ln_eps);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
        const int c = n0 + ni * 16 + 4 * g;
        const float4 b = *reinterpret_cast<const float4 *>(a.bias + c);
        float v0, v1, v2, v3;
        if constexpr (epi_ln(EPI)) {  // rstd·(acc − μ·c) + b′
            const float4 lc = *reinterpret_cast<const float4 *>(a.ln_c + c);
            v0 = fmaf(lrs.x, acc[ni][0], fmaf(lrs.y, lc.x, b.x));
            v1 = fmaf(lrs.x, acc[ni][1], fmaf(lrs.y, lc.y, b.y));
            v2 = fmaf(lrs.x, acc[ni][2], fmaf(lrs.y, lc.z, b.z));
            v3 = fmaf(lrs.x, acc[ni][3], fmaf(lrs.y, lc.w, b.w));
        } else {
            v0 = acc[ni][0] + b.x, v1 = acc[ni][1] + b.y, v2 = acc[ni][2] + b.z, v3 = acc[ni][3] + b.w;
        }
        if constexpr (EPI == EPI_RESID_BF16) {  // residual stream in bf16 (LN producers: gemm_skinny_ln_kernel)
            const int64_t off = (int64_t)row * a.N + c;
            const float4 r = rs_load4(a.ln_x + off);
            rs_store4(make_float4(v0 + r.x, v1 + r.y, v2 + r.z, v3 + r.w), a.ln_x + off, true);
        } else if constexpr (EPI == EPI_RESID_F32) {
            float4 *o = reinterpret_cast<float4 *>(a.out_f32 + (int64_t)row * a.N + c);
            const float4 r = *o;
            *o = make_float4(r.x + v0, r.y + v1, r.z + v2, r.w + v3);
        } else {
            if constexpr (epi_gelu(EPI)) {
                const f32x2 lo = gelu_fast2(f32x2{v0, v1}), hi = gelu_fast2(f32x2{v2, v3});
                v0 = lo.x;
                v1 = lo.y;
                v2 = hi.x;
                v3 = hi.y;
            }
            *reinterpret_cast<uint2 *>(a.out_bf16 + (int64_t)row * (a.ldc ? a.ldc : a.N) + c) =
                make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
    }
}

// One wave per block: the loads are address-bound (PMC: the texture addresser busy for the
// whole launch on the CUs holding blocks), so a tile per CU where 4-wave blocks put four.
// WPB > 1 (diagnostic builds): WPB consecutive tiles per block, one wave and one DMA ring each —
// a one-image fc1 is 1 248 one-wave workgroups (the same bits either way).
template <int EPI, int NI, int KT, int WPB = 1, int SK = SKINNY_DMA_STAGES>
__global__ __launch_bounds__(64 * WPB) void gemm_skinny_kernel(GemmArgs a) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int wave = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    const int nct = a.N / (16 * NI), nrt = (a.M + 15) / 16;
    const int w = skinny_block(blockIdx.x, gridDim.x) * WPB + wave;
    if (w >= nct * nrt) return;
    const int ct = w / nrt, rt = w % nrt;
    const int K = a.K, n0 = ct * 16 * NI, row = rt * 16 + li;
    f32x4 acc[NI];
    if constexpr (KT > 0) {
        __shared__ __attribute__((aligned(16))) uint8_t ring[WPB][SK * skinny_dma_stage_bytes<NI>()];
        skinny_chain_dma<NI, KT / 64, SK>(a.A, rt * 16, a.M, a.W, n0, K, ring[wave], acc);
    } else {
        const uint16_t *Ar = a.A + (int64_t)min(row, a.M - 1) * K + 8 * g;  // rows past M: clamped loads, no stores
        const uint16_t *Wr = a.W + (int64_t)(n0 + li) * K + 8 * g;
        skinny_chain<NI, KT>(Ar, Wr, K, K / 32, acc);
    }
    if (row >= a.M) return;
    skinny_epilogue<EPI, NI>(a, acc, row, n0, g);
}

// Weights shared by SKR row tiles (QKV / fc1 of a lone image, K = 768 / 3072): a block of SKR waves
// owns SKR consecutive 16-row tiles of one 32-column tile; per 64-deep K block each wave copies its
// own 16 A rows and a quarter of the 32 W rows into one LDS stage, and every wave reads all 32 W rows
// from it — W crosses L2 -> CU once per row group instead of once per row tile (a one-image fc1
// moved 61 MB of W for 4.7 MB of unique weights).  Per stage: A at wave·2048 (16 rows), W at
// SKR·2048 (32 rows), 128-B rows with skinny_chain_dma's swizzle.  One barrier per K block: a wave
// has its own copies of block kb (counted vmcnt), the barrier says every wave's have landed and that
// every wave has read block kb − 1, whose stage is then refilled.  Waves of a row group past M copy
// clamped rows and skip the stores.  Each wave's MFMA chain is skinny_chain_dma's: the same bits.
constexpr int SKR = 4;
template <int NKB, int SK>
__device__ __forceinline__ void skinny_chain_dma_shared(const uint16_t *__restrict__ A, int row_a0, int M, const uint16_t *__restrict__ W,
                                                        int n0, int K, uint8_t *ring, int wave, f32x4 (&acc)[2]) {
    constexpr int NI = 2, SB = (SKR * 16 + 32) * 128, NP = 3, WOFF = SKR * 2048;
    static_assert(NKB >= SK && (SK - 1) * NP <= 63 && SK <= 11, "ring depth: primed with SK - 1 blocks, 6-bit vmcnt");
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    // copies: i = 0, 1: A rows 8i + lane / 8 of the wave's tile; i = 2: W row 8·wave + lane / 8
    const uint16_t *src[NP];
    uint32_t dst[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int r = i < 2 ? i * 8 + (lane >> 3) : wave * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        src[i] = (i < 2 ? A + (int64_t)min(row_a0 + r, M - 1) * K : W + (int64_t)(n0 + r) * K) + c * 8;
        dst[i] = i < 2 ? (uint32_t)(wave * 2048 + i * 1024) : (uint32_t)(WOFF + wave * 1024);
    }
    auto issue = [&](int kb) __attribute__((always_inline)) {
        uint8_t *st = ring + (kb % SK) * SB;
#pragma unroll
        for (int i = 0; i < NP; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + kb * 64), (lds_void_t *)(st + dst[i]), 16, 0, 0);
    };
    uint32_t fa[2], fw[2][NI];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const int c = (4 * s2 + g) ^ ((li >> 1) & 7);
        fa[s2] = (uint32_t)(wave * 2048 + li * 128 + c * 16);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) fw[s2][ni] = (uint32_t)(WOFF + (16 * ni + li) * 128 + c * 16);
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < SK - 1; ++kb) issue(kb);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        constexpr int X = NP;
        const int younger = min(SK - 2, NKB - 1 - kb);
        if (younger >= 9) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(9 * X) : "memory");
        else if (younger == 8) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * X) : "memory");
        else if (younger == 7) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * X) : "memory");
        else if (younger == 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * X) : "memory");
        else if (younger == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * X) : "memory");
        else if (younger == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * X) : "memory");
        else if (younger == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * X) : "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * X) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const uint32_t st = (uint32_t)(uintptr_t)(ring + (kb % SK) * SB);
        bf16x8 a[2], w[2][NI];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            asm volatile("ds_read_b128 %0, %1" : "=v"(a[s2]) : "v"(st + fa[s2]));
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) asm volatile("ds_read_b128 %0, %1" : "=v"(w[s2][ni]) : "v"(st + fw[s2][ni]));
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1]));
        // every wave passed this barrier after reading block kb - 1: its stage takes block kb + SK - 1
        if (kb + SK - 1 < NKB) issue(kb + SK - 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
                acc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[s2][ni], a[s2], acc[ni], 0, 0, 0);
    }
}

// grid: (N / 32) · ceil(ceil(M / 16) / SKR) blocks of SKR waves, column-tile-major through skinny_block
template <int EPI, int KT, int SK = SKINNY_DMA_STAGES>
__global__ __launch_bounds__(64 * SKR) void gemm_skinny_shared_kernel(GemmArgs a) {
    constexpr int NI = 2;
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nct = a.N / 32, nrt = (a.M + 15) / 16, nrg = (nrt + SKR - 1) / SKR;
    const int b = skinny_block(blockIdx.x, gridDim.x);
    if (b >= nct * nrg) return;  // block-uniform
    const int ct = b / nrg, rt = (b % nrg) * SKR + wave;
    const int n0 = ct * 32, row = rt * 16 + li;
    __shared__ __attribute__((aligned(16))) uint8_t ring[SK * (SKR * 16 + 32) * 128];
    f32x4 acc[NI];
    skinny_chain_dma_shared<KT / 64, SK>(a.A, rt * 16, a.M, a.W, n0, a.K, ring, wave, acc);
    if (row >= a.M) return;
    skinny_epilogue<EPI, NI>(a, acc, row, n0, g);
}

// The skinny GEMM as a LayerNorm-fold producer (residual epilogues with ln_x + ln_stats, N = 768:
// O-proj / fc2 of a batch of one image, the CLS O-proj): the block-partial statistics are
// computed in the epilogue (the canonical slices and reduction tree of every producer, bit for bit;
// round 4 ran them as a second launch, 5 us each at batch 1).
// A block of 2 waves owns one row tile × one 64-column LayerNorm block (blocks numbered column-
// block-major through skinny_block: a column block's weights stay in one XCD): wave w computes
// rows 16·rt + li, columns 64·blk + 32·w + 16·ni + 4g + e (the skinny kernel's tile and K chain),
// stores as gemm_skinny_kernel does and puts the value each element now stands for (the stored
// f32 or bf16) into LDS; then wave 0 reads the 16 rows' canonical slices
// (4 lanes per row) and reduces them with ln_block_reduce_quad.  (4-wave blocks of two row
// tiles: 84 blocks for a lone image's fc2, address-bound on 84 CUs at 34 us.)
template <int EPI, int KT>
__global__ __launch_bounds__(128) void gemm_skinny_ln_kernel(GemmArgs a) {
    static_assert(epi_resid(EPI), "LayerNorm producers are residual epilogues");
    constexpr int NI = 2, LP = 68;  // LDS row pitch (floats)
    __shared__ float xs_l[16 * LP];
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15, wave = threadIdx.x >> 6;
    const int nrt = (a.M + 15) / 16, lb = skinny_block(blockIdx.x, gridDim.x);
    const int blk = lb / nrt, rt = lb % nrt;  // column-block-major (skinny_block)
    const int K = a.K, n0 = blk * 64 + wave * 32, row = rt * 16 + li;
    f32x4 acc[NI];
    if constexpr (KT > 0) {
        __shared__ __attribute__((aligned(16))) uint8_t ring[2][SKINNY_DMA_STAGES * skinny_dma_stage_bytes<NI>()];
        skinny_chain_dma<NI, KT / 64>(a.A, rt * 16, a.M, a.W, n0, K, ring[wave], acc);
    } else {
        const uint16_t *Ar = a.A + (int64_t)min(row, a.M - 1) * K + 8 * g;
        const uint16_t *Wr = a.W + (int64_t)(n0 + li) * K + 8 * g;
        skinny_chain<NI, KT>(Ar, Wr, K, K / 32, acc);
    }
    const bool valid = row < a.M;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
        const int c = n0 + ni * 16 + 4 * g;
        const float4 b = *reinterpret_cast<const float4 *>(a.bias + c);
        const float v0 = acc[ni][0] + b.x, v1 = acc[ni][1] + b.y, v2 = acc[ni][2] + b.z, v3 = acc[ni][3] + b.w;
        const int64_t off = (int64_t)min(row, a.M - 1) * a.N + c;
        float4 x;
        if constexpr (EPI == EPI_RESID_BF16) {
            const float4 r = rs_load4(a.ln_x + off);
            x = rs_store4(make_float4(v0 + r.x, v1 + r.y, v2 + r.z, v3 + r.w), a.ln_x + off, valid);
        } else {
            float4 *o = reinterpret_cast<float4 *>(a.out_f32 + off);
            const float4 r = *o;
            x = make_float4(r.x + v0, r.y + v1, r.z + v2, r.w + v3);
            if (valid) {
                *o = x;
                *reinterpret_cast<uint2 *>(a.ln_x + off) = pack_bf16x4(x);
            }
        }
        *reinterpret_cast<float4 *>(xs_l + li * LP + wave * 32 + ni * 16 + 4 * g) = x;
    }
    __syncthreads();
    if (wave != 0) return;
    const int r = lane >> 2, sg = lane & 3;
    float xs[16];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float *q = xs_l + r * LP + ln_slice_col(sg, c);
        const float4 u = *reinterpret_cast<const float4 *>(q), v = *reinterpret_cast<const float4 *>(q + 4);
        xs[8 * c] = u.x, xs[8 * c + 1] = u.y, xs[8 * c + 2] = u.z, xs[8 * c + 3] = u.w;
        xs[8 * c + 4] = v.x, xs[8 * c + 5] = v.y, xs[8 * c + 6] = v.z, xs[8 * c + 7] = v.w;
    }
    const float2 st = ln_block_reduce_quad(ln_slice_stats(xs), sg);
    const int srow = rt * 16 + r;
    if (sg == 0 && srow < a.M) *reinterpret_cast<float2 *>(a.ln_stats + (int64_t)srow * LN_STRIDE + 2 * blk) = st;
}

// Split-K skinny GEMM with an f32 residual epilogue, for the last layer's fc2 on the
// CLS rows (M = images, N = 768, K = 3072; every batch size, so the CLS rows of an image
// get the same bits in any batch): the skinny kernel's one wave per 16
// rows x 32 columns walks all of K as a chain of dependent 16x16x32 MFMAs and global
// loads (54 us at M = 128); here KS waves split K, write f32 partials [KS][M][N], and
// skinny_reduce_kernel adds them in ks order + bias + the residual (deterministic).
// Used only on the CLS rows, so batch invariance is unaffected (the full-layer GEMMs of
// a small batch keep the skinny kernel, bit-identical to the tiled ones).
template <int NI, int KS, int KT>
__global__ __launch_bounds__(64) void gemm_skinny_splitk_kernel(GemmArgs a, float *__restrict__ part) {
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int nct = a.N / (16 * NI), nrt = (a.M + 15) / 16;
    const int w = blockIdx.x;  // one wave per block (address-bound loads: spread over CUs)
    if (w >= nct * nrt * KS) return;
    const int ks = w % KS, tile = w / KS;
    const int ct = tile % nct, rt = tile / nct;
    const int KL = a.K / KS, k0 = ks * KL;
    const int n0 = ct * 16 * NI, row = rt * 16 + li;
    const uint16_t *Ar = a.A + (int64_t)min(row, a.M - 1) * a.K + k0 + 8 * g;
    const uint16_t *Wr = a.W + (int64_t)(n0 + li) * a.K + k0 + 8 * g;
    f32x4 acc[NI];
    skinny_chain<NI, KT>(Ar, Wr, a.K, KL / 32, acc);
    if (row >= a.M) return;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
        *reinterpret_cast<f32x4 *>(part + ((int64_t)ks * a.M + row) * a.N + n0 + ni * 16 + 4 * g) = acc[ni];
}

template <int KS>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(GemmArgs a, const float *__restrict__ part) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one float4 of outputs
    if (i >= (int64_t)a.M * a.N / 4) return;
    const int64_t e = i * 4;
    const int c = (int)(e % a.N);
    float4 s = *reinterpret_cast<const float4 *>(part + e);
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) {
        const float4 p = *reinterpret_cast<const float4 *>(part + (int64_t)ks * a.M * a.N + e);
        s = make_float4(s.x + p.x, s.y + p.y, s.z + p.z, s.w + p.w);
    }
    const float4 b = *reinterpret_cast<const float4 *>(a.bias + c);
    float4 *o = reinterpret_cast<float4 *>(a.out_f32 + e);
    const float4 r = *o;
    *o = make_float4(r.x + (s.x + b.x), r.y + (s.y + b.y), r.z + (s.z + b.z), r.w + (s.w + b.w));
}

constexpr int SKINNY_KS = 4;

// out_f32 [M][N] += A·Wᵀ + bias on the split-K skinny path (part: >= SKINNY_KS·M·N floats)
inline void launch_skinny_splitk_resid(const GemmArgs &a, float *part, hipStream_t s) {
    RC_REQUIRE(a.M >= 1 && a.N % 32 == 0 && a.K % (32 * SKINNY_KS) == 0 && a.out_f32 && !a.ln_x, RC_ERR_UNSUPPORTED,
               "split-K skinny GEMM: N % 32 == 0, K % 128 == 0, f32 residual");
    const int waves = ((a.M + 15) / 16) * (a.N / 32) * SKINNY_KS;
    if (a.K == 768 * SKINNY_KS)
        hipLaunchKernelGGL((gemm_skinny_splitk_kernel<2, SKINNY_KS, 768>), dim3(waves), dim3(64), 0, s, a, part);
    else
        hipLaunchKernelGGL((gemm_skinny_splitk_kernel<2, SKINNY_KS, 0>), dim3(waves), dim3(64), 0, s, a, part);
    RC_LAUNCH_CHECK();
    const int64_t n4 = (int64_t)a.M * a.N / 4;
    hipLaunchKernelGGL(skinny_reduce_kernel<SKINNY_KS>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, a, part);
    RC_LAUNCH_CHECK();
}

// Kernel choice: 4 = ping-pong 256x256, 10 = ping-pong on image-aligned 224-row tiles,
// 8 = two-workgroup 128x256, 9 = skinny (M <= 256), 0 = auto.  Auto follows interleaved
// A/B timings on the batch-256 shapes.  (Rounds 1-4 also measured a 128x128 4-wave kernel, a
// 256x256 / 128x256 single-barrier kernel, persistent and Stream-K kernels, a deferred-store
// persistent kernel, an LDS ring of 3-5 slots and buffer-load DMA: each lost or tied and was
// removed; the forms live on in tools/gemm_lab.)
enum GemmVariant { GEMM_AUTO = 0, GEMM_PINGPONG = 4, GEMM_W2 = 8, GEMM_SKINNY = 9, GEMM_PP_IMG = 10 };

inline int gemm_pick(const GemmArgs &a, int variant, bool patch_epilogue, bool ln_epilogue = false) {
    if (variant != GEMM_AUTO) return variant;  // (100 + ABL / 200 + ABL: ablation builds, RC_GEMM_ABLATION)
    if (a.M <= 256 && !patch_epilogue && a.N % 32 == 0) return GEMM_SKINNY;
    // (Round 5 built image-aligned 224-row tiles for the residual producers — O-proj / fc2 as whole
    // rounds, n x 3 tiles: per launch at parts = 1 fc2 276 vs 297 us, but at the product's parts = 2
    // the two slices already fill each other's last round and the 12 % padded rows cost more:
    // step 10.08 vs 9.99 ms, twice (profiles/r05/r05p_gemm_ab_p2.log).  Diagnostic builds only.)
    // Short square projections without image alignment (N = K = 768) finish in ~2.3 rounds of
    // 256x256 tiles and carry a heavy epilogue: the two-workgroup kernel overlaps it with the
    // co-resident workgroup's MFMAs.  Everything else streams K at 128 flop/B: ping-pong.
    // (LayerNorm-fold consumers, e.g. the CLS rows' Q of a batch above 256 images, stay on the
    // ping-pong kernel, whose prologue computes the row scales.)
    if (a.N <= 768 && a.K <= 768 && !ln_epilogue) return GEMM_W2;
    return GEMM_PINGPONG;
}

// Ping-pong tile order: groups of 8 row tiles (column-major inside a group) when
// a row has >= 6 column tiles (QKV: 176 -> 170 us, fc1: 285 -> 274 us at batch
// 256, interleaved A/B in tools/gemm_calib.py), row-major otherwise (fc2 prefers
// it by 2 %).
#if defined(RC_GEMM_ABLATION)
inline int g_skinny_wpb = 1;    // diagnostic builds: tiles (waves) per skinny-GEMM block (rc_diag_set_skinny_wpb)
inline int g_group_m_wide = 8;  // diagnostic builds: group_m of the wide ping-pong GEMMs (rc_diag_set_group_m)
inline int gemm_group_m(const GemmArgs &a) { return a.N / 256 >= 6 ? g_group_m_wide : 0; }
#else
inline int gemm_group_m(const GemmArgs &a) { return a.N / 256 >= 6 ? 8 : 0; }
#endif

// The patch embedding of a small batch (M <= 256 patch rows, the bf16 stream: one image is
// 196 rows, and patch_gemm_kernel's 128 x 256 tiles put it on 6 workgroups, 33 us): the skinny
// form.  Block = 2 waves = one 16-row tile x one 64-column LayerNorm block (as
// gemm_skinny_ln_kernel); wave w takes columns 32w..32w+31.  A fragments are built in registers
// from the u8 images — lane (g, li), K-step s: patch row 16 rt + li, K = 32 s + 8 g .. + 7 in
// (ky, kx, c) order, 8 bytes of one image row, each bf16(fma(u, pre_a[k mod 3], pre_b[k mod 3]))
// exactly as patch_gemm_kernel converts them — and the W rows stream through the LDS-DMA ring;
// the MFMAs run in the same K order (the same bits).  Epilogue: x = (acc + bias) + position
// embedding at the patch's token row, stored to the bf16 stream, LN partials of the 64-column
// block through LDS (f32_rows_epilogue's values and canonical slices).
template <int EPI>
__global__ __launch_bounds__(128) void patch_skinny_kernel(GemmArgs a) {
    static_assert(EPI == EPI_PATCH_BF16, "the bf16 stream");
    constexpr int NI = 2, P = 16, KC = 3 * P * P, NKB = KC / 64, LP = 68;
    constexpr int SK = SKINNY_DMA_STAGES, SB = 16 * NI * 128;
    __shared__ __attribute__((aligned(16))) uint8_t ring[2][SK * SB];
    __shared__ float xs_l[16 * LP];
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15, wave = threadIdx.x >> 6;
    const int nrt = (a.M + 15) / 16, lb = skinny_block(blockIdx.x, gridDim.x);
    const int blk = lb / nrt, rt = lb % nrt;
    const int n0 = blk * 64 + wave * 32, row = rt * 16 + li;
    // this lane's patch row: 8 image bytes per K-step, all 24 steps loaded up front
    const int S = a.img_size, gp = S / P, np = gp * gp;
    const int m = min(row, a.M - 1);
    const int b = m / np, pi = m - b * np, py = pi / gp, px = pi - py * gp;
    const uint8_t *abase = a.img + (((int64_t)b * S + py * P) * S + px * P) * 3;
    uint2 ab[2 * NKB];
#pragma unroll
    for (int st = 0; st < 2 * NKB; ++st) {
        const int k0 = 32 * st + 8 * g, ky = k0 / (3 * P), off = k0 - ky * (3 * P);
        ab[st] = *reinterpret_cast<const uint2 *>(abase + ky * S * 3 + off);
    }
    // every A fragment converted up front (24 x 16 B per lane; constant indices below)
    const float pa[3] = {a.pre_a[0], a.pre_a[1], a.pre_a[2]}, pb[3] = {a.pre_b[0], a.pre_b[1], a.pre_b[2]};
    bf16x8 af[2 * NKB];
#pragma unroll
    for (int st = 0; st < 2 * NKB; ++st) {
        const int c0 = (32 * st + 8 * g) % 3;  // channel of byte 0 (k mod 3; 3P = 48 keeps rows aligned)
        // the (a, b) pair of byte e is ((c0 + e) mod 3): rotate once, then constant indices
        const float ra[3] = {c0 == 0 ? pa[0] : (c0 == 1 ? pa[1] : pa[2]), c0 == 0 ? pa[1] : (c0 == 1 ? pa[2] : pa[0]),
                             c0 == 0 ? pa[2] : (c0 == 1 ? pa[0] : pa[1])};
        const float rb[3] = {c0 == 0 ? pb[0] : (c0 == 1 ? pb[1] : pb[2]), c0 == 0 ? pb[1] : (c0 == 1 ? pb[2] : pb[0]),
                             c0 == 0 ? pb[2] : (c0 == 1 ? pb[0] : pb[1])};
        const uint32_t w[2] = {ab[st].x, ab[st].y};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 2 * j;
            const float uA = (float)((w[e >> 2] >> (8 * (e & 3))) & 0xffu);
            const float uB = (float)((w[(e + 1) >> 2] >> (8 * ((e + 1) & 3))) & 0xffu);
            o[j] = pack_bf16x2(fmaf(uA, ra[e % 3], rb[e % 3]), fmaf(uB, ra[(e + 1) % 3], rb[(e + 1) % 3]));
        }
        af[st] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
    }
    // W rows n0 .. n0 + 31 by LDS-DMA (skinny_chain_dma's ring, without the A half)
    uint8_t *rg = ring[wave];
    const uint16_t *src[2 * NI];
#pragma unroll
    for (int i = 0; i < 2 * NI; ++i) {
        const int r = i * 8 + (lane >> 3);
        src[i] = a.W + (int64_t)(n0 + r) * KC + (((lane & 7) ^ ((r >> 1) & 7)) * 8);
    }
    auto issue = [&](int kb) __attribute__((always_inline)) {
        uint8_t *stg = rg + (kb % SK) * SB;
#pragma unroll
        for (int i = 0; i < 2 * NI; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + kb * 64), (lds_void_t *)(stg + i * 1024), 16, 0, 0);
    };
    uint32_t fw[2][NI];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) fw[s2][ni] = (uint32_t)((16 * ni + li) * 128 + (((4 * s2 + g) ^ ((li >> 1) & 7)) * 16));
    f32x4 acc[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the image bytes (older than every DMA below)
#pragma unroll
    for (int kb = 0; kb < SK - 1; ++kb) issue(kb);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        constexpr int X = 2 * NI;
        const int younger = min(SK - 2, NKB - 1 - kb);
        if (younger >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * X) : "memory");
        else if (younger == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * X) : "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * X) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t st = (uint32_t)(uintptr_t)(rg + (kb % SK) * SB);
        bf16x8 w[2][NI];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) asm volatile("ds_read_b128 %0, %1" : "=v"(w[s2][ni]) : "v"(st + fw[s2][ni]));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0][0]), "+v"(w[0][1]), "+v"(w[1][0]), "+v"(w[1][1]));
        if (kb + SK - 1 < NKB) issue(kb + SK - 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
                acc[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[s2][ni], af[2 * kb + s2], acc[ni], 0, 0, 0);
    }
    // epilogue: f32_rows_epilogue's values, per element
    const bool valid = row < a.M;
    const int img = m / np, p = m - img * np;
    const int64_t orow = (int64_t)img * a.tokens + 1 + p;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
        const int c = n0 + ni * 16 + 4 * g;
        const float4 bb = *reinterpret_cast<const float4 *>(a.bias + c);
        const float4 ps = *reinterpret_cast<const float4 *>(a.pos + (int64_t)(1 + p) * a.N + c);
        const float4 xf = make_float4((acc[ni][0] + bb.x) + ps.x, (acc[ni][1] + bb.y) + ps.y, (acc[ni][2] + bb.z) + ps.z,
                                      (acc[ni][3] + bb.w) + ps.w);
        *reinterpret_cast<float4 *>(xs_l + li * LP + wave * 32 + ni * 16 + 4 * g) = rs_store4(xf, a.ln_x + orow * a.N + c, valid);
    }
    if (a.ln_stats == nullptr) return;  // block-uniform
    __syncthreads();
    if (wave != 0) return;
    const int r = lane >> 2, sg = lane & 3;
    float xs[16];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
        const float *q = xs_l + r * LP + ln_slice_col(sg, cc);
        const float4 u = *reinterpret_cast<const float4 *>(q), v = *reinterpret_cast<const float4 *>(q + 4);
        xs[8 * cc] = u.x, xs[8 * cc + 1] = u.y, xs[8 * cc + 2] = u.z, xs[8 * cc + 3] = u.w;
        xs[8 * cc + 4] = v.x, xs[8 * cc + 5] = v.y, xs[8 * cc + 6] = v.z, xs[8 * cc + 7] = v.w;
    }
    const float2 stt = ln_block_reduce_quad(ln_slice_stats(xs), sg);
    const int srow = rt * 16 + r;
    if (sg == 0 && srow < a.M) {
        const int sm = srow, simg = sm / np, sp = sm - simg * np;
        *reinterpret_cast<float2 *>(a.ln_stats + ((int64_t)simg * a.tokens + 1 + sp) * LN_STRIDE + 2 * blk) = stt;
    }
}

// Implicit-GEMM patch embedding: M = images × patches rows, N = hidden, K = 3·P² (P = 16)
inline void launch_patch_gemm(const GemmArgs &a, hipStream_t s) {
    RC_REQUIRE(a.img && a.img_size % 16 == 0 && a.N % 256 == 0 && a.K == 3 * 16 * 16 && a.M >= 1,
               RC_ERR_UNSUPPORTED, "patch GEMM: 16x16 patches, N % 256 == 0");
    const int ntm = (a.M + 127) / 128, ntn = a.N / 256;
    if (a.resid_bf16) {
        RC_REQUIRE(a.ln_x != nullptr, RC_ERR_INVALID, "bf16 residual stream needs ln_x");
        if (a.M <= 256 && a.N == 64 * LN_PARTS)  // a small batch: the skinny form (same bits)
            hipLaunchKernelGGL((patch_skinny_kernel<EPI_PATCH_BF16>), dim3(((a.M + 15) / 16) * LN_PARTS), dim3(128), 0, s, a);
        else
            hipLaunchKernelGGL((patch_gemm_kernel<16, EPI_PATCH_BF16>), dim3(ntm * ntn), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL((patch_gemm_kernel<16, EPI_PATCH_F32>), dim3(ntm * ntn), dim3(256), 0, s, a);
    }
    RC_LAUNCH_CHECK();
}

// rows the A buffer must provide beyond M (the kernels read whole tiles)
inline int gemm_row_pad() { return 256; }

template <int EPI, int ABL, int BM>
void launch_pp(const GemmArgs &a, int ntm, hipStream_t s) {
    const dim3 gr(ntm * (a.N / 256)), bl(512);
    if (a.K == 768) hipLaunchKernelGGL((gemm_pp_kernel<EPI, ABL, 12, BM>), gr, bl, 0, s, a);
    else if (a.K == 3072) hipLaunchKernelGGL((gemm_pp_kernel<EPI, ABL, 48, BM>), gr, bl, 0, s, a);
    else hipLaunchKernelGGL((gemm_pp_kernel<EPI, ABL, 0, BM>), gr, bl, 0, s, a);
}

template <int EPI>
void launch_gemm(const GemmArgs &a_in, int variant, hipStream_t s) {
    GemmArgs a = a_in;
    RC_REQUIRE(a.K % 64 == 0 && a.K >= 64, RC_ERR_UNSUPPORTED, "GEMM K must be a multiple of 64");
    const int pick = gemm_pick(a, variant, epi_patch(EPI), epi_ln(EPI));
    RC_REQUIRE(a.ldc == 0 || (a.ldc >= a.N && epi_bf16_out(EPI)), RC_ERR_UNSUPPORTED,
               "an output row stride (ldc) needs a bf16 epilogue");
    if constexpr (epi_bf16_stream(EPI)) {
        RC_REQUIRE(a.ln_x, RC_ERR_UNSUPPORTED, "bf16-stream residual epilogues need ln_x");
    }
    if constexpr (epi_ln(EPI)) {
        bool ln_ok = pick == GEMM_PINGPONG || pick == GEMM_SKINNY;
#if defined(RC_GEMM_ABLATION)
        ln_ok = ln_ok || (pick >= 100 && pick < 200) || pick == GEMM_W2;  // gemm_pp_kernel<EPI, ABL>, round-6 W2 A/B
#endif
        RC_REQUIRE(ln_ok && a.ln_c && a.ln_stats, RC_ERR_UNSUPPORTED,
                   "LayerNorm-fold consumers run on the ping-pong or skinny kernel");
    }
    switch (pick) {
        case GEMM_W2: {
#if !defined(RC_GEMM_ABLATION)
            // LayerNorm-fold consumers on this kernel: diagnostic builds only (round 6 in-model A/B,
            // bit-identical: fc1 302 vs 273 us, QKV 206 vs 183 on the ping-pong kernel)
            if constexpr (epi_ln(EPI)) throw Error(RC_ERR_UNSUPPORTED, "LayerNorm-fold consumers: ping-pong or skinny kernel");
            else
#endif
            {
                RC_REQUIRE(a.N % 256 == 0, RC_ERR_UNSUPPORTED, "GEMM N must be a multiple of 256");
                RC_REQUIRE(a.K % 32 == 0, RC_ERR_UNSUPPORTED, "GEMM K must be a multiple of 32");
                const int ntn = a.N / 256;
                if constexpr (epi_resid(EPI)) {
                    // 160-row tiles when they take fewer row-rounds of the chip's workgroup slots
                    // (2 per CU): rounds x BM, the time of one slot's chain
                    const int slots = 2 * device_cu_count();
                    const int t128 = (a.M + 127) / 128 * ntn, t160 = (a.M + 159) / 160 * ntn;
                    if ((int64_t)((t160 + slots - 1) / slots) * 160 < (int64_t)((t128 + slots - 1) / slots) * 128) {
                        hipLaunchKernelGGL((gemm_w2_kernel<EPI, 0, 160>), dim3(t160), dim3(256), 0, s, a);
                        break;
                    }
                }
                hipLaunchKernelGGL((gemm_w2_kernel<EPI>), dim3((a.M + 127) / 128 * ntn), dim3(256), 0, s, a);
            }
            break;
        }
        case GEMM_SKINNY: {
            RC_REQUIRE(!epi_patch(EPI) && a.N % 32 == 0 && a.M >= 1, RC_ERR_UNSUPPORTED,
                       "skinny GEMM: bf16 / GELU / residual epilogues, N a multiple of 32");
            if constexpr (epi_resid(EPI)) {
                if (a.ln_x != nullptr && a.ln_stats != nullptr) {  // LayerNorm-fold producer: partials in the epilogue
                    RC_REQUIRE(a.N == 64 * LN_PARTS, RC_ERR_UNSUPPORTED, "LayerNorm fold needs N = 768");
                    const dim3 gr(((a.M + 15) / 16) * LN_PARTS);
                    if (a.K == 768) hipLaunchKernelGGL((gemm_skinny_ln_kernel<EPI, 768>), gr, dim3(128), 0, s, a);
                    else if (a.K == 3072) hipLaunchKernelGGL((gemm_skinny_ln_kernel<EPI, 3072>), gr, dim3(128), 0, s, a);
                    else hipLaunchKernelGGL((gemm_skinny_ln_kernel<EPI, 0>), gr, dim3(128), 0, s, a);
                    break;
                }
            }
            const int nrt = (a.M + 15) / 16;
            const dim3 gr(nrt * (a.N / 32));  // one wave (tile) per block
#if defined(RC_GEMM_ABLATION)
            if (g_skinny_wpb > 1 && (a.K == 768 || a.K == 3072)) {  // diagnostic: WPB tiles per block
                const unsigned nb = (unsigned)(((a.M + 15) / 16) * (a.N / 32) + g_skinny_wpb - 1) / g_skinny_wpb;
                if (g_skinny_wpb == 2 && a.K == 768)
                    hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 768, 2>), dim3(nb), dim3(128), 0, s, a);
                else if (g_skinny_wpb == 2)
                    hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 3072, 2>), dim3(nb), dim3(128), 0, s, a);
                else if (a.K == 768)
                    hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 768, 4>), dim3(nb), dim3(256), 0, s, a);
                else
                    hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 3072, 4>), dim3(nb), dim3(256), 0, s, a);
                break;
            }
#endif
            // more one-wave tiles than the one-wave kernel holds resident (4-5 per CU: a lone image's
            // fc1, 1 248): row tiles share the weights, SKR per block (fc1 7.68 -> 7.16 us per launch in
            // rocprofv3; QKV's 936 tiles stay one per block: 5.84 vs 6.16 us shared,
            // profiles/r06/r06ai_skinny_shared_w_b1_ab.log)
            if (nrt > 1 && nrt * (a.N / 32) > 1024 && (a.K == 768 || a.K == 3072)) {
                const dim3 gs((unsigned)((a.N / 32) * ((nrt + SKR - 1) / SKR)));
                if (a.K == 768) hipLaunchKernelGGL((gemm_skinny_shared_kernel<EPI, 768>), gs, dim3(64 * SKR), 0, s, a);
                else hipLaunchKernelGGL((gemm_skinny_shared_kernel<EPI, 3072>), gs, dim3(64 * SKR), 0, s, a);
                break;
            }
            if (a.K == 768) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 768, 1, epi_gelu(EPI) ? SKINNY_FC1_STAGES : SKINNY_DMA_STAGES>), gr, dim3(64), 0, s, a);
            else if (a.K == 3072) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 3072>), gr, dim3(64), 0, s, a);
            else hipLaunchKernelGGL((gemm_skinny_kernel<EPI, 2, 0>), gr, dim3(64), 0, s, a);
            break;
        }
        case GEMM_PINGPONG: {
            RC_REQUIRE(a.N % 256 == 0, RC_ERR_UNSUPPORTED, "GEMM N must be a multiple of 256");
            a.group_m = gemm_group_m(a);
            launch_pp<EPI, 0, PP_BM>(a, (a.M + PP_BM - 1) / PP_BM, s);
            break;
        }
#if defined(RC_GEMM_ABLATION)
        case GEMM_PP_IMG: {
            if constexpr (epi_resid(EPI)) {
                // a tile computes 224 rows from its image's first row: the A buffer must hold
                // row_step·ntm + (224 − row_step) rows (the model's workspace pads 256)
                RC_REQUIRE(a.N % 256 == 0 && a.row_step > 0 && a.row_step <= PP_IMG_BM && a.row_step > PP_IMG_BM - 64,
                           RC_ERR_UNSUPPORTED, "image-aligned GEMM: N % 256 == 0, 160 < row_step <= 224");
                a.group_m = 0;
                launch_pp<EPI, 0, PP_IMG_BM>(a, (a.M + a.row_step - 1) / a.row_step, s);
            } else {
                throw Error(RC_ERR_UNSUPPORTED, "image-aligned GEMM tiles: residual epilogues only");
            }
            break;
        }
        case 301: case 302: case 303: {  // residual epilogue nontemporal reads / stores / both, 160-row W2 tiles
            if constexpr (epi_resid(EPI)) {
                const dim3 gr((a.M + 159) / 160 * (a.N / 256)), bl(256);
                if (variant == 301) hipLaunchKernelGGL((gemm_w2_kernel<EPI, 1024, 160>), gr, bl, 0, s, a);
                else if (variant == 302) hipLaunchKernelGGL((gemm_w2_kernel<EPI, 2048, 160>), gr, bl, 0, s, a);
                else hipLaunchKernelGGL((gemm_w2_kernel<EPI, 3072, 160>), gr, bl, 0, s, a);
            }
            break;
        }
        case 304: {  // residual producer on 160-row W2 tiles, A operand's DMA nontemporal
            if constexpr (epi_resid(EPI))
                hipLaunchKernelGGL((gemm_w2_kernel<EPI, 4096, 160>), dim3((a.M + 159) / 160 * (a.N / 256)), dim3(256), 0, s, a);
            break;
        }
        case 300: {  // the two-workgroup kernel on 128-row tiles whatever M (A/B of the 160-row pick)
            if constexpr (!epi_ln(EPI))
                hipLaunchKernelGGL((gemm_w2_kernel<EPI>), dim3((a.M + 127) / 128 * (a.N / 256)), dim3(256), 0, s, a);
            break;
        }
        case 200 + 1: case 200 + 2: case 200 + 4: case 200 + 6: {
            const int ntm = (a.M + 127) / 128, ntn = a.N / 256;
            const dim3 gr(ntm * ntn), bl(256);
            switch (variant - 200) {
                case 1: hipLaunchKernelGGL((gemm_w2_kernel<EPI, 1>), gr, bl, 0, s, a); break;
                case 2: hipLaunchKernelGGL((gemm_w2_kernel<EPI, 2>), gr, bl, 0, s, a); break;
                case 4: hipLaunchKernelGGL((gemm_w2_kernel<EPI, 4>), gr, bl, 0, s, a); break;
                case 6: hipLaunchKernelGGL((gemm_w2_kernel<EPI, 6>), gr, bl, 0, s, a); break;
            }
            break;
        }
        case 100 + 0: case 100 + 1: case 100 + 2: case 100 + 3: case 100 + 4: case 100 + 5: case 100 + 6:
        case 100 + 8: case 100 + 16: case 100 + 24: case 100 + 32: case 100 + 64: case 100 + 96: case 150: case 151: case 152: case 153: case 154: case 155: case 156: {
            a.group_m = gemm_group_m(a);  // the product tile order
            const int ntm = (a.M + 255) / 256;
            switch (variant - 100) {
                case 0: launch_pp<EPI, 0, PP_BM>(a, ntm, s); break;
                case 1: launch_pp<EPI, 1, PP_BM>(a, ntm, s); break;
                case 2: launch_pp<EPI, 2, PP_BM>(a, ntm, s); break;
                case 3: launch_pp<EPI, 3, PP_BM>(a, ntm, s); break;
                case 4: launch_pp<EPI, 4, PP_BM>(a, ntm, s); break;
                case 5: launch_pp<EPI, 5, PP_BM>(a, ntm, s); break;
                case 6: launch_pp<EPI, 6, PP_BM>(a, ntm, s); break;
                case 8: launch_pp<EPI, 8, PP_BM>(a, ntm, s); break;
                case 16: launch_pp<EPI, 16, PP_BM>(a, ntm, s); break;
                case 24: launch_pp<EPI, 24, PP_BM>(a, ntm, s); break;
                case 32: launch_pp<EPI, 32, PP_BM>(a, ntm, s); break;
                case 64: launch_pp<EPI, 64, PP_BM>(a, ntm, s); break;
                case 96: launch_pp<EPI, 96, PP_BM>(a, ntm, s); break;
                case 50: launch_pp<EPI, 128, PP_BM>(a, ntm, s); break;  // staggered start, ~10 us
                case 51: launch_pp<EPI, 256, PP_BM>(a, ntm, s); break;  // staggered start, ~5 us
                case 52: launch_pp<EPI, 512, PP_BM>(a, ntm, s); break;  // fc1 LDS-staged, nontemporal stores
                case 53: launch_pp<EPI, 1024, PP_BM>(a, ntm, s); break;  // residual read nontemporal
                case 54: launch_pp<EPI, 2048, PP_BM>(a, ntm, s); break;  // residual stores nontemporal
                case 55: launch_pp<EPI, 3072, PP_BM>(a, ntm, s); break;  // both
                case 56: launch_pp<EPI, 4096, PP_BM>(a, ntm, s); break;  // A operand's DMA nontemporal
            }
            break;
        }
#endif
        default: throw Error(RC_ERR_INVALID, "unknown GEMM variant");
    }
    RC_LAUNCH_CHECK();
}

}  // namespace rc
