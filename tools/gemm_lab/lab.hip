// GEMM lab (diagnostic, never loaded by the product): main-loop structures for the
// ViT-MSN batch-256 projection shapes, C[M][N] = A[M][K] . W[N][K]^T, bf16 in, f32
// accumulate, bf16 out (no bias / epilogue work: this isolates the K loop).
//
//  variant 0: the product's ping-pong schedule (gemm.h gemm_pp_kernel), 256x256x64, 8 waves
//  variant 1: 0 with in-LDS s_memtime stamps at every barrier (waves 0 and 4, blocks 0-7)
//  variant 2: ping-pong, W fragments kept in registers for the whole K-step (24 LDS reads
//             per wave per K-step instead of 32)
//  variant 3: 4 waves, one per SIMD, 128x128 outputs per wave, one barrier per K-step,
//             the next K-tile's LDS-DMA interleaved with this one's MFMAs
//  variant 4: 0 with the LDS-DMA as buffer loads (one lane offset, scalar row offsets)
//  variant 5: 3 at BK = 32 in a 4-slot ring, three steps in flight, one barrier per step
//  variant 6: ping-pong with 2 phases per K-step (32-MFMA segments, 4 barriers per step), W kept
//  variants 7 / 8: ping-pong over a BK = 32 ring of 4 / 5 slots (64 / 96 KB of DMA in flight)
//  variant 9: ping-pong with A through LDS-DMA and W loaded straight into registers one K-step ahead
//  variant 10: 5 software-pipelined: the next step's fragments read under this step's MFMAs
//  variant 11: 10 with MFMA / ds_read as inline asm (program order, accumulators pinned in AGPRs)
//  variants 12 / 13 / 14 / 15: persistent ping-pong, LDS-staged epilogue, 0 / 4 / 6 / 8 of each thread's
//             16 C chunks stored during the next tile's first K-steps instead of at once
//  variants 128 / 176: 0 / 48 without the C stores (the epilogue's HBM write burst)
//  variants 16 / 32 / 48 / 64: 0 without the loop's DMA / LDS reads / both / MFMAs (ablations:
//             wrong results, timing only)
// Every variant accumulates each output over K in the same order (chunks of 32, k
// ascending), so their results are bit-identical.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

struct LabArgs {
    const uint16_t *A, *W;
    uint16_t *C;
    int M, N, K;
    uint64_t *stamps;  // variant 1: [16 (block, group)][512]
    int group_m;       // tile order: groups of group_m row tiles (column-major inside); -1 = auto
};

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    bf16x2 v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
}
// tile id -> (row tile, column tile); groups of 8 row tiles (column-major inside) when N/256 >= 6
__device__ __forceinline__ void tile_coords(const LabArgs &a, int BM, int BN, int tile, int &tm, int &tn) {
    const int ntn = a.N / BN, ntm = (a.M + BM - 1) / BM;
    tm = tile / ntn;
    tn = tile % ntn;
    const int G = a.group_m >= 0 ? a.group_m : (ntn >= 6 ? 8 : 0);
    if (G > 0) {
        const int gt = G * ntn, gi = tile / gt, in = tile - gi * gt;
        const int gm = min(G, ntm - gi * G);
        tm = gi * G + in % gm;
        tn = in / gm;
    }
}

__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------ ping-pong
constexpr int PP_STAGE = 2 * 256 * 64 * 2;  // A tile then W tile, 32 KB each

template <int VAR>
__global__ __launch_bounds__(512, 1) void lab_pp(LabArgs a) {
    constexpr bool STAMP = VAR == 1, WKEEP = VAR == 2, BUF = VAR == 4;
    constexpr bool NO_DMA = (VAR & 16) != 0, NO_READ = (VAR & 32) != 0, NO_MFMA = (VAR & 64) != 0;
    constexpr bool NO_STORE = (VAR & 128) != 0;
    constexpr int A_BYTES = 256 * 64 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * PP_STAGE + (STAMP ? 8192 : 0)];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 64;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    const bool stamper = STAMP && lane == 0 && (wave & 3) == 0 && blockIdx.x < 8;
    int ns = 0;
    auto stamp = [&]() {
        if constexpr (STAMP) {
            if (stamper && ns < 512)
                *reinterpret_cast<uint64_t *>(smem + 2 * PP_STAGE + grp * 4096 + ns * 8) = __builtin_amdgcn_s_memtime();
            ++ns;
        }
    };

    const int lr = wave * 8 + (lane >> 3);
    const uint32_t voff = (uint32_t)(lr * K + (((lane & 7) ^ ((lr >> 1) & 7)) << 3)) * 2u;
    auto stage4 = [&](int buf, int k0, int i0) {
        uint8_t *base = smem + buf * PP_STAGE;
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i) {
            const int piece = wave + 8 * i;
            const bool is_a = i < 4;
            if constexpr (BUF) {  // one lane offset, the piece's rows in soffset, the K-step in the descriptor
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc((void *)((is_a ? Ag : Wg) + k0), (short)0, 0x7fffffff, 0x00020000);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)(base + piece * 1024), 16, voff, (i & 3) * 64 * K * 2, 0, 0);
            } else {
                const int r = (is_a ? piece : piece - 32) * 8 + (lane >> 3);
                const int c = (lane & 7) ^ ((r >> 1) & 7);
                const uint16_t *src = (is_a ? Ag : Wg) + (int64_t)r * K + k0 + c * 8;
                __builtin_amdgcn_global_load_lds((const void *)src, (lds_void_t *)(base + piece * 1024), 16, 0, 0);
            }
        }
    };
    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < 2; ++l) acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};

    stamp();
    stage4(0, 0, 0);
    stage4(0, 0, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    stamp();
    if (grp == 1) bar();

    bf16x8 af[4][2], wf[2][2][2];  // [mi][s], [nq][ni][s]
#pragma nounroll
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const uint8_t *As = smem + cur * PP_STAGE;
        const uint8_t *Ws = As + A_BYTES;
        const bool more = kt + 1 < nk;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mq = p >> 1;
            const int nq = (p == 1 || p == 2);
            if ((p == 0 || p == 2) && !(NO_READ && kt > 0)) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int r = grp * 128 + mq * 64 + mi * 16 + li;
                        const int c = s * 4 + g;
                        af[mi][s] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
            const bool wread = (WKEEP ? (p == 0 || p == 1) : true) && !(NO_READ && kt > 0);
            if (wread) {
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int r = wc * 64 + nq * 32 + ni * 16 + li;
                        const int c = s * 4 + g;
                        wf[WKEEP ? nq : 0][ni][s] = *reinterpret_cast<const bf16x8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
            if (more && p < 2 && !NO_DMA) stage4(cur ^ 1, (kt + 1) * 64, p * 4);
            if (p == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            stamp();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        if constexpr (NO_MFMA)
                            asm volatile("" ::"v"(wf[WKEEP ? nq : 0][ni][s]), "v"(af[mi][s]));
                        else
                            acc[mq][nq][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                wf[WKEEP ? nq : 0][ni][s], af[mi][s], acc[mq][nq][mi][ni], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            bar();
            stamp();
        }
    }
    if (grp == 0) bar();
    stamp();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    const int row = m0 + grp * 128 + mq * 64 + mi * 16 + li;
                    const int col = n0 + wc * 64 + nq * 32 + ni * 16 + 4 * g;
                    const f32x4 v = acc[mq][nq][mi][ni];
                    if constexpr (NO_STORE)
                        asm volatile("" ::"v"(v));
                    else if (row < a.M)
                        *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
                }
    if constexpr (STAMP) {
        stamp();
        __syncthreads();
        if (blockIdx.x < 8 && tid < 64 * 8 && (wave & 3) == 0) {
            const uint64_t *src = reinterpret_cast<const uint64_t *>(smem + 2 * PP_STAGE + grp * 4096);
            for (int i = lane; i < 512; i += 64) a.stamps[(blockIdx.x * 2 + grp) * 512 + i] = i < ns ? src[i] : 0;
        }
    }
}

// --------------------------------------------------- 4 waves, 128x128 per wave
// 256x256x64 tile, wave w: rows (w >> 1) * 128, columns (w & 1) * 128; acc[mi][ni] =
// 8 x 8 tiles of mfma_f32_16x16x32_bf16 (swapped operands: A-operand = weight rows).
// K-step t: vmcnt(0) (this wave's DMA of stage t) + barrier; then for each 32-deep half s:
// 16 fragment reads (8 A, 8 W) and 64 MFMAs, with this wave's 16 DMA pieces of stage t + 1
// spread over the first half's MFMAs.
__global__ __launch_bounds__(256, 1) void lab_w4(LabArgs a) {
    constexpr int A_BYTES = 256 * 64 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * PP_STAGE];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 64;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;

    // piece p = 0..63 (1 KB = 8 rows x 128 B): A rows 8p.. for p < 32, W rows 8(p-32).. after;
    // wave w issues pieces w + 4 i, i = 0..15 (i < 8: A).  Row r = 8w + 32 (i % 8) + lane / 8, so
    // the source chunk swizzle (r >> 1) & 7 does not depend on i: one lane offset for every
    // piece, the piece's rows in the scalar offset, the K-step in the descriptor base.
    const int lr = wave * 8 + (lane >> 3);
    const uint32_t voff = (uint32_t)(lr * K + (((lane & 7) ^ ((lr >> 1) & 7)) << 3)) * 2u;
    auto piece = [&](int buf, int k0, int i) {
        const uint16_t *base = (i < 8 ? Ag : Wg) + k0;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7fffffff, 0x00020000);
        lds_void_t *dst = (lds_void_t *)(smem + buf * PP_STAGE + (wave + 4 * i) * 1024);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, voff, (i & 7) * 32 * K * 2, 0, 0);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) piece(0, 0, i);

#pragma nounroll
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const uint8_t *As = smem + cur * PP_STAGE;
        const uint8_t *Ws = As + A_BYTES;
        const bool more = kt + 1 < nk;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[8], wf[8];
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const int r = wc * 128 + ni * 16 + li;
                const int c = s * 4 + g;
                wf[ni] = *reinterpret_cast<const bf16x8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const int r = wr * 128 + mi * 16 + li;
                const int c = s * 4 + g;
                af[mi] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                if (s == 0 && more) {
                    piece(cur ^ 1, (kt + 1) * 64, 2 * mi);
                    piece(cur ^ 1, (kt + 1) * 64, 2 * mi + 1);
                }
#pragma unroll
                for (int ni = 0; ni < 8; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[mi][ni], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int row = m0 + wr * 128 + mi * 16 + li;
            const int col = n0 + wc * 128 + ni * 16 + 4 * g;
            const f32x4 v = acc[mi][ni];
            if (row < a.M)
                *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
}


// --------------------------------- 4 waves, 128x128 per wave, BK = 32, 4-slot ring
// Slot = A[256][32] + W[256][32] bf16 (32 KB, 64-B rows, chunk c of row r at c ^ ((r >> 3) & 1) << 1:
// conflict-free ds_read_b128 fragments, gemm_ring_kernel's image).  Steps t+1..t+2 stay in flight
// while step t computes; step t+3 is issued into the slot step t-1 used, after the barrier that
// closes every wave's reads of it.  One barrier per 32-deep step, counted vmcnt (never 0 in the
// loop); the DMA is issued for every step (past the end: a clamped, unused re-read), so the
// counts hold on every path.
__global__ __launch_bounds__(256, 1) void lab_w4r(LabArgs a) {
    constexpr int NS = 4, SLOT = 2 * 256 * 32 * 2, A_BYTES = 256 * 32 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 32;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    // piece p (1 KB = 16 rows x 64 B): A rows 16p.. for p < 16, W rows 16(p-16).. after; wave w
    // issues p = w + 4 i, i = 0..7 (i < 4: A).  Lane l writes row l >> 2, stored chunk l & 3 =
    // source chunk (l & 3) ^ (((l >> 5) & 1) << 1): one lane offset for every piece.
    const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const uint32_t voff = (uint32_t)((16 * wave + prow) * K + pchunk * 8) * 2u;
    auto issue = [&](int t) {
        const int tc = t < nk ? t : nk - 1;
        uint8_t *base = smem + (t % NS) * SLOT;
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)(Ag + tc * 32), (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)(Wg + tc * 32), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? ra : rw, (lds_void_t *)(base + (wave + 4 * i) * 1024), 16, voff,
                                                     (i & 3) * 64 * K * 2, 0, 0);
    };
    const int fchunk = (g ^ (((li >> 3) & 1) << 1)) << 4;
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue(0);
    issue(1);
    issue(2);
#pragma nounroll
    for (int t = 0; t < nk; ++t) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // this wave's step t landed (t+1, t+2 fly)
        bar();
        issue(t + 3);
        const uint8_t *As = smem + (t % NS) * SLOT;
        const uint8_t *Ws = As + A_BYTES;
        bf16x8 af[8], wf[8];
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) wf[ni] = *reinterpret_cast<const bf16x8 *>(Ws + (wc * 128 + ni * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) af[mi] = *reinterpret_cast<const bf16x8 *>(As + (wr * 128 + mi * 16 + li) * 64 + fchunk);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[mi][ni], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail re-reads
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int row = m0 + wr * 128 + mi * 16 + li;
            const int col = n0 + wc * 128 + ni * 16 + 4 * g;
            const f32x4 v = acc[mi][ni];
            if (row < a.M)
                *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
}


// ------------------------------------- ping-pong, 2 phases per K-step, W kept
// lab_pp with the K-step in 2 phases (one per 64-row half mq of the wave's 128 rows) instead of
// 4: a C segment is 32 MFMAs (the half's 4 x 4 tiles x 2 k-halves), so a K-step has 4 barriers,
// not 8.  M0 reads the half's A fragments (8) and the step's W fragments (8, kept for both
// halves) and issues this wave's 8 DMA pieces of step t+1; M1 reads the other half's A (8) and
// waits for this wave's pieces.  G1 runs one segment behind G0 (the stagger barrier), so the
// buffer step t+1 goes to was last read in the segment before G0's M0(t) (G1's M1(t-1)).
__global__ __launch_bounds__(512, 1) void lab_pp2(LabArgs a) {
    constexpr int A_BYTES = 256 * 64 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * PP_STAGE];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 64;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    const int lr = wave * 8 + (lane >> 3);
    const uint32_t voff = (uint32_t)(lr * K + (((lane & 7) ^ ((lr >> 1) & 7)) << 3)) * 2u;
    auto stage8 = [&](int buf, int k0) {
        uint8_t *base = smem + buf * PP_STAGE;
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)(Ag + k0), (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)(Wg + k0), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? ra : rw, (lds_void_t *)(base + (wave + 8 * i) * 1024), 16, voff,
                                                     (i & 3) * 64 * K * 2, 0, 0);
    };
    f32x4 acc[2][4][4];  // [mq][mi][ni]: rows grp*128 + mq*64 + mi*16, columns wc*64 + ni*16
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[i][j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    stage8(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (grp == 1) bar();
    bf16x8 af[4][2], wf[4][2];
#pragma nounroll
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const uint8_t *As = smem + cur * PP_STAGE;
        const uint8_t *Ws = As + A_BYTES;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int r = grp * 128 + p * 64 + mi * 16 + li;
                    const int c = s * 4 + g;
                    af[mi][s] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                }
            if (p == 0) {
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int r = wc * 64 + ni * 16 + li;
                        const int c = s * 4 + g;
                        wf[ni][s] = *reinterpret_cast<const bf16x8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
                if (kt + 1 < nk) stage8(cur ^ 1, (kt + 1) * 64);
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni)
                        acc[p][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni][s], af[mi][s], acc[p][mi][ni], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            bar();
        }
    }
    if (grp == 0) bar();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int row = m0 + grp * 128 + mq * 64 + mi * 16 + li;
                const int col = n0 + wc * 64 + ni * 16 + 4 * g;
                const f32x4 v = acc[mq][mi][ni];
                if (row < a.M)
                    *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
            }
}


// ---------------------------------------------- ping-pong over a deep ring (BK = 32)
// gemm_ring_kernel's schedule (2 phases per 32-deep step, W kept for both, 4 DMA pieces per wave
// per step) with NS slots of 32 KB and NS - 2 steps in flight across every barrier: NS = 4 keeps
// the 64 KB the 2 x 64 KB ping-pong keeps in flight, NS = 5 (all 160 KB of LDS) keeps 96 KB.
// Every step is issued (past the end: the last step again, into the slot of a finished one), so
// the counted wait is the same constant on every path.
template <int NS>
__global__ __launch_bounds__(512, 1) void lab_ring(LabArgs a) {
    constexpr int BK = 32, A_BYTES = 256 * BK * 2, SLOT = 2 * A_BYTES;
    __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / BK;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    // 32 pieces of 1 KB (16 rows x 64 B) per slot: A rows = pieces 0-15, W = 16-31; wave w issues
    // pieces w + 8 i, i = 0..3.  Lane l writes row l >> 2, stored chunk l & 3 = source chunk
    // (l & 3) ^ (((l >> 5) & 1) << 1)
    const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    auto issue = [&](int t) {
        const int tc = t < nk ? t : nk - 1;
        uint8_t *base = smem + (t % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = wave + 8 * i;
            const bool is_a = piece < 16;
            const uint16_t *src = is_a ? Ag + (int64_t)(piece * 16 + prow) * K : Wg + (int64_t)((piece - 16) * 16 + prow) * K;
            __builtin_amdgcn_global_load_lds((const void *)(src + tc * BK + pchunk * 8), (lds_void_t *)(base + piece * 1024),
                                             16, 0, 0);
        }
    };
    const int fchunk = (g ^ (((li >> 3) & 1) << 1)) << 4;
    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < 2; ++l) acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NS - 1; ++t) issue(t);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NS - 2)) : "memory");
    bar();
    if (grp == 1) bar();
    bf16x8 af[4], wf[2][2];
#pragma nounroll
    for (int t = 0; t < nk; ++t) {
        const uint8_t *As = smem + (t % NS) * SLOT;
        const uint8_t *Ws = As + A_BYTES;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
                af[mi] = *reinterpret_cast<const bf16x8 *>(As + (grp * 128 + p * 64 + mi * 16 + li) * 64 + fchunk);
            if (p == 0) {
#pragma unroll
                for (int nq = 0; nq < 2; ++nq)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        wf[nq][ni] = *reinterpret_cast<const bf16x8 *>(Ws + (wc * 64 + nq * 32 + ni * 16 + li) * 64 + fchunk);
                issue(t + NS - 1);  // into the slot step t - 1 used (every wave's reads of it closed)
            } else {
                // this wave's pieces of step t + 1 landed; steps t + 2 .. t + NS - 1 may fly
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NS - 2)) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int nq = 0; nq < 2; ++nq)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        acc[p][nq][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nq][ni], af[mi], acc[p][nq][mi][ni], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            bar();
        }
    }
    if (grp == 0) bar();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's re-issued steps
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    const int row = m0 + grp * 128 + mq * 64 + mi * 16 + li;
                    const int col = n0 + wc * 64 + nq * 32 + ni * 16 + 4 * g;
                    const f32x4 v = acc[mq][nq][mi][ni];
                    if (row < a.M)
                        *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
                }
}


// ------------------------------- ping-pong, A through LDS, W straight into registers
// lab_pp's schedule with the weight tile never staged in LDS: each wave loads its own 64 W rows
// (4 fragments x 2 k-halves, 16 B per lane each) from global memory (L2: the weights are <= 4.7 MB)
// one K-step ahead into a second register set, while the LDS-DMA carries only the A tile (32 KB
// per K-step instead of 64).  The W loads are inline asm (hipcc would drain every LDS-DMA before
// their first use); the phase-3 vmcnt(0) that retires the A DMA of step t+1 also retires them.
// Two K-steps per loop iteration so the two W register sets keep fixed names.
__global__ __launch_bounds__(512, 1) void lab_ppw(LabArgs a) {
    constexpr int A_BYTES = 256 * 64 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * A_BYTES];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 64;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    // A pieces: 32 per K-step (8 rows x 128 B), wave w issues pieces w + 8 i, i = 0..3
    auto stageA = [&](int buf, int k0, int i0) {
        uint8_t *base = smem + buf * A_BYTES;
#pragma unroll
        for (int i = i0; i < i0 + 2; ++i) {
            const int piece = wave + 8 * i;
            const int r = piece * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((r >> 1) & 7);
            __builtin_amdgcn_global_load_lds((const void *)(Ag + (int64_t)r * K + k0 + c * 8), (lds_void_t *)(base + piece * 1024),
                                             16, 0, 0);
        }
    };
    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int l = 0; l < 2; ++l) acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};
    // three register slots of W fragments: nq = 1 always lives in Y (its next-step copy is loaded at
    // phase 3, after phase 2 retired it, and waited for at phase 1 of the next step); nq = 0
    // alternates between X and Z (next step's copy loaded at phase 0 into the idle slot)
    bf16x8 wX[2][2], wY[2][2], wZ[2][2], af[4][2];
    // saddr form: the wave-uniform row block + K-step in SGPRs, one 32-bit VGPR offset per (nq, ni)
    uint32_t woff[2][2];
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) woff[nq][ni] = (uint32_t)(((nq * 32 + ni * 16 + li) * K + 8 * g) * 2);
    const uint8_t *wblk = reinterpret_cast<const uint8_t *>(a.W) + (int64_t)(n0 + wc * 64) * K * 2;
    auto loadW1 = [&](bf16x8 (&w)[2][2], int t, int nq) {
        const uint8_t *base = wblk + t * 128;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
            asm volatile("global_load_dwordx4 %0, %2, %3\n\tglobal_load_dwordx4 %1, %2, %3 offset:64"
                         : "=&v"(w[ni][0]), "=&v"(w[ni][1])
                         : "v"(woff[nq][ni]), "s"(base)
                         : "memory");
    };
    stageA(0, 0, 0);
    stageA(0, 0, 2);
    loadW1(wX, 0, 0);
    loadW1(wY, 0, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_sched_barrier(0);
    if (grp == 1) bar();
    auto step = [&](int kt, bf16x8 (&w0)[2][2], bf16x8 (&w0n)[2][2]) {
        const int cur = kt & 1;
        const uint8_t *As = smem + cur * A_BYTES;
        const bool more = kt + 1 < nk;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int mq = p >> 1;
            const int nq = (p == 1 || p == 2);
            if (p == 0 || p == 2) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int r = grp * 128 + mq * 64 + mi * 16 + li;
                        const int c = s2 * 4 + g;
                        af[mi][s2] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
            }
            if (more && p < 2) stageA(cur ^ 1, (kt + 1) * 64, p * 2);
            if (more && p == 0) loadW1(w0n, kt + 1, 0);
            if (p == 1) {
                // this step's Y loads (issued at the previous step's phase 3) must have landed;
                // younger: phase 0's 2 DMA + 4 loads and phase 1's 2 DMA
                if (more) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (p == 3) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // phase 2 was Y's last use this step: refill it for the next step
                if (more) loadW1(wY, kt + 1, 1);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni)
                        acc[mq][nq][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nq ? wY[ni][s2] : w0[ni][s2], af[mi][s2],
                                                                                    acc[mq][nq][mi][ni], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            bar();
        }
    };
#pragma nounroll
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, wX, wZ);
        step(kt + 1, wZ, wX);
    }
    if (grp == 0) bar();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    const int row = m0 + grp * 128 + mq * 64 + mi * 16 + li;
                    const int col = n0 + wc * 64 + nq * 32 + ni * 16 + 4 * g;
                    const f32x4 v = acc[mq][nq][mi][ni];
                    if (row < a.M)
                        *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
                }
}


// ---------------------- 4 waves, 128x128 per wave, BK = 32 ring, fragments prefetched
// lab_w4r's tile and ring (4 slots of A[256][32] + W[256][32], one barrier per 32-deep step),
// but software-pipelined the way a one-wave-per-SIMD kernel has to be: step t's 64 MFMAs run on
// fragments read during step t-1, while the wave reads step t+1's 16 fragments (4 after each of
// the first four 8-MFMA rows) and issues its 8 DMA pieces of step t+3 (one per row).  Accumulators
// live in AGPRs (256), two fragment sets in VGPRs (128).  Per step and CU: 64 KB of ds_read_b128
// (256 LDS cycles) and 32 KB of DMA against 1024 MFMA cycles per SIMD — the 8-wave ping-pong
// spends 192 KB of reads per 64-deep step.
__global__ __launch_bounds__(256, 1) void lab_w4p(LabArgs a) {
    constexpr int NS = 4, SLOT = 2 * 256 * 32 * 2, A_BYTES = 256 * 32 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 32;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const uint32_t voff = (uint32_t)((16 * wave + prow) * K + pchunk * 8) * 2u;
    auto piece = [&](int t, int i) {
        const int tc = t < nk ? t : nk - 1;
        uint8_t *base = smem + (t % NS) * SLOT;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)((i < 4 ? Ag : Wg) + tc * 32), (short)0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)(base + (wave + 4 * i) * 1024), 16, voff, (i & 3) * 64 * K * 2, 0, 0);
    };
    const int fchunk = (g ^ (((li >> 3) & 1) << 1)) << 4;
    auto frag = [&](int t, int j) -> bf16x8 {  // j < 8: W rows wc*128 + 16j; else A rows wr*128 + 16(j-8)
        const uint8_t *base = smem + (t % NS) * SLOT + (j < 8 ? A_BYTES : 0);
        const int r = (j < 8 ? wc : wr) * 128 + (j & 7) * 16 + li;
        return *reinterpret_cast<const bf16x8 *>(base + r * 64 + fchunk);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i) piece(t, i);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    bf16x8 f0[16], f1[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f0[j] = frag(0, j);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    auto step = [&](int t, bf16x8 (&cur)[16], bf16x8 (&nxt)[16]) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's pieces of step t+1 landed
        bar();                                              // ... and everyone's; slot (t+3)%4 free
        __builtin_amdgcn_sched_barrier(0);
        const bool rd = t + 1 < nk;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[ni], cur[8 + mi], acc[mi][ni], 0, 0, 0);
            if (mi < 4 && rd) {
#pragma unroll
                for (int j = 0; j < 4; ++j) nxt[4 * mi + j] = frag(t + 1, 4 * mi + j);
            }
            piece(t + 3, mi);
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            if (mi < 4) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
#pragma nounroll
    for (int t = 0; t < nk; t += 2) {
        step(t, f0, f1);
        step(t + 1, f1, f0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail re-reads
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int row = m0 + wr * 128 + mi * 16 + li;
            const int col = n0 + wc * 128 + ni * 16 + 4 * g;
            const f32x4 v = acc[mi][ni];
            if (row < a.M)
                *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
}


// ------------------------- 10 with the loop in program order: MFMA and ds_read as inline asm
// (accumulators pinned to AGPRs with "+a"; hipcc rotated accumulator tiles through a spare
// AGPR quad every step in lab_w4p).  The compiler does not see these MFMAs: the epilogue's
// first AGPR read waits out the last MFMA's passes with explicit s_nops.
__device__ __forceinline__ void mfma_a(f32x4 &c, const bf16x8 &w, const bf16x8 &x) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(x));
}
__device__ __forceinline__ void ds_read16(bf16x8 &d, uint32_t addr) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr) : "memory");
}
__global__ __launch_bounds__(256, 1) void lab_w4a(LabArgs a) {
    constexpr int NS = 4, SLOT = 2 * 256 * 32 * 2, A_BYTES = 256 * 32 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT];
    int tm, tn;
    tile_coords(a, 256, 256, xcd_remap(blockIdx.x, gridDim.x), tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 32;
    const uint16_t *Ag = a.A + (int64_t)m0 * K;
    const uint16_t *Wg = a.W + (int64_t)n0 * K;
    const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 5) & 1) << 1);
    const uint32_t voff = (uint32_t)((16 * wave + prow) * K + pchunk * 8) * 2u;
    auto piece = [&](int t, int i) {
        const int tc = t < nk ? t : nk - 1;
        uint8_t *base = smem + (t % NS) * SLOT;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)((i < 4 ? Ag : Wg) + tc * 32), (short)0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)(base + (wave + 4 * i) * 1024), 16, voff, (i & 3) * 64 * K * 2, 0, 0);
    };
    const int fchunk = (g ^ (((li >> 3) & 1) << 1)) << 4;
    const uint32_t sbase = (uint32_t)(uintptr_t)smem;
    const uint32_t waddr = sbase + A_BYTES + (wc * 128 + li) * 64 + fchunk;  // + slot, + 1024 j
    const uint32_t aaddr = sbase + (wr * 128 + li) * 64 + fchunk;
    auto frag = [&](bf16x8 &d, int t, int j) {
        ds_read16(d, (j < 8 ? waddr : aaddr) + (t % NS) * SLOT + (j & 7) * 1024);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i) piece(t, i);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    bf16x8 f0[16], f1[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) frag(f0[j], 0, j);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    auto step = [&](int t, bf16x8 (&cur)[16], bf16x8 (&nxt)[16]) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's pieces of step t+1 landed
        bar();                                              // ... and everyone's; slot (t+3)%4 free
        const int tn1 = t + 1 < nk ? t + 1 : t;             // last step: a harmless re-read
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                mfma_a(acc[mi][ni], cur[ni], cur[8 + mi]);
                if (mi < 4 && (ni & 1)) frag(nxt[4 * mi + (ni >> 1)], tn1, 4 * mi + (ni >> 1));
                if (ni == 3) piece(t + 3, mi);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
#pragma nounroll
    for (int t = 0; t < nk; t += 2) {
        step(t, f0, f1);
        step(t + 1, f1, f0);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
            const int row = m0 + wr * 128 + mi * 16 + li;
            const int col = n0 + wc * 128 + ni * 16 + 4 * g;
            const f32x4 v = acc[mi][ni];
            if (row < a.M)
                *reinterpret_cast<uint2 *>(a.C + (int64_t)row * a.N + col) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
}


// ------------------------------ persistent ping-pong with the C stores spread over the next tile
// lab_pp's K loop (variant 0 form) in a persistent grid (one workgroup per CU walks the tiles
// t = i * grid + remap(block)).  Epilogue as the product's bf16 path: the 256 x 256 bf16 tile
// staged in LDS (512-B rows, 16-B chunk XOR (row & 31)), then 16 row-chunk stores of 16 B per
// thread.  DEF of them (0, 8 or 16) are held in registers and issued during the NEXT tile's
// first K-steps (one per M segment of phases 0 and 2), so the CUs' write bursts overlap MFMA
// work instead of stalling every CU at once; the last tile stores everything at once.
template <int DEF>
__global__ __launch_bounds__(512, 1) void lab_ppd(LabArgs a) {
    constexpr int A_BYTES = 256 * 64 * 2;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * PP_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int g = lane >> 4, li = lane & 15;
    const int K = a.K, nk = K / 64;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int lr = wave * 8 + (lane >> 3);
    const uint32_t voff = (uint32_t)(lr * K + (((lane & 7) ^ ((lr >> 1) & 7)) << 3)) * 2u;
    uint4 pend[DEF > 0 ? DEF : 1];
    int pm0 = -1, pn0 = 0;  // the previous tile (whose last DEF chunks per thread are pending)
    const int rb = xcd_remap(blockIdx.x, gridDim.x);
    // pending chunk i of this thread: epilogue iteration it = 16 - DEF + i, row (it*512+tid)>>5
    auto store_pending = [&](int i) {
        int ptid;
        asm volatile("v_mov_b32 %0, %1" : "=v"(ptid) : "v"(tid));  // recompute, do not hoist
        const int id = (16 - DEF + i) * 512 + ptid;
        const int rl = id >> 5, ch = id & 31;
        if (pm0 + rl < a.M) *reinterpret_cast<uint4 *>(a.C + (int64_t)(pm0 + rl) * a.N + pn0 + ch * 8) = pend[i];
    };
#pragma nounroll
    for (int tile = rb; tile < ntiles; tile += gridDim.x) {
        int tm, tn;
        tile_coords(a, 256, 256, tile, tm, tn);
        const int m0 = tm * 256, n0 = tn * 256;
        const uint16_t *Ag = a.A + (int64_t)m0 * K;
        const uint16_t *Wg = a.W + (int64_t)n0 * K;
        auto stage4 = [&](int buf, int k0, int i0) {  // buffer-load DMA (lab variant 4's form)
            uint8_t *base = smem + buf * PP_STAGE;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void *)((i0 < 4 ? Ag : Wg) + k0), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int i = i0; i < i0 + 4; ++i)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)(base + (wave + 8 * i) * 1024), 16, voff,
                                                         (i & 3) * 64 * K * 2, 0, 0);
        };
        f32x4 acc[2][2][4][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int l = 0; l < 2; ++l) acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};
        stage4(0, 0, 0);
        stage4(0, 0, 4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
        if (grp == 1) bar();
        bf16x8 af[4][2], wf[2][2];
        int np = 0;
        // one K-step; PS: this step issues pending chunks 2 PS and 2 PS + 1 (static indices)
        auto kstep = [&](int kt, auto psc) {
            constexpr int PS = decltype(psc)::value;
            const int cur = kt & 1;
            const uint8_t *As = smem + cur * PP_STAGE;
            const uint8_t *Ws = As + A_BYTES;
            const bool more = kt + 1 < nk;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int mq = p >> 1;
                const int nq = (p == 1 || p == 2);
                if (p == 0 || p == 2) {
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2) {
                            const int r = grp * 128 + mq * 64 + mi * 16 + li;
                            const int c = s2 * 4 + g;
                            af[mi][s2] = *reinterpret_cast<const bf16x8 *>(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                        }
                }
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int r = wc * 64 + nq * 32 + ni * 16 + li;
                        const int c = s2 * 4 + g;
                        wf[ni][s2] = *reinterpret_cast<const bf16x8 *>(Ws + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                    }
                if constexpr (PS >= 0) {  // one deferred C chunk of the previous tile per phase 0 / 2
                    if (p == 0 && pm0 >= 0) store_pending(2 * PS);
                    if (p == 2 && pm0 >= 0) store_pending(2 * PS + 1);
                }
                if (more && p < 2) stage4(cur ^ 1, (kt + 1) * 64, p * 4);
                if (p == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bar();
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                        for (int ni = 0; ni < 2; ++ni)
                            acc[mq][nq][mi][ni] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni][s2], af[mi][s2], acc[mq][nq][mi][ni], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
                bar();
            }
        };
        // the first DEF / 2 K-steps unrolled (each issues two pending chunks), then the rest
        [&]<int... I>(std::integer_sequence<int, I...>) {
            ((I < nk ? kstep(I, std::integral_constant<int, I>{}) : void()), ...);
        }(std::make_integer_sequence<int, DEF / 2>{});
#pragma nounroll
        for (int kt = DEF / 2; kt < nk; ++kt) kstep(kt, std::integral_constant<int, -1>{});
        (void)np;
        if (grp == 0) bar();
        if constexpr (DEF > 0) {  // pending chunks the loop did not reach (K shorter than the spread)
            if (pm0 >= 0)
#pragma unroll
                for (int i = 0; i < DEF; ++i)
                    if (i >= 2 * nk) store_pending(i);
        }
        // epilogue: stage the bf16 tile (every read and DMA of the loop retired by its last barrier).
        // Its addresses derive from a laundered copy of the lane id, so hipcc recomputes them per
        // tile instead of hoisting ~48 loop-invariant offsets into registers across the K loop.
        int ltid;
        asm volatile("v_mov_b32 %0, %1" : "=v"(ltid) : "v"(tid));
        const int eli = ltid & 15, eg = (ltid >> 4) & 3;
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
            for (int nq = 0; nq < 2; ++nq)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 2; ++ni) {
                        const int rl = grp * 128 + mq * 64 + mi * 16 + eli;
                        const int cl = wc * 64 + nq * 32 + ni * 16 + 4 * eg;
                        const f32x4 v = acc[mq][nq][mi][ni];
                        const int off = rl * 512 + ((((cl >> 3) ^ (rl & 31))) << 4) + (cl & 7) * 2;
                        *reinterpret_cast<uint2 *>(smem + off) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
                    }
        __syncthreads();
        const bool last = tile + (int)gridDim.x >= ntiles;
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int id = it * 512 + ltid;
            const int rl = id >> 5, ch = id & 31;
            const uint4 v = *reinterpret_cast<const uint4 *>(smem + rl * 512 + ((ch ^ (rl & 31)) << 4));
            if (it >= 16 - DEF && !last)
                pend[it - (16 - DEF)] = v;
            else if (m0 + rl < a.M)
                *reinterpret_cast<uint4 *>(a.C + (int64_t)(m0 + rl) * a.N + n0 + ch * 8) = v;
        }
        pm0 = m0;
        pn0 = n0;
        __syncthreads();  // LDS free for the next tile's prologue
    }
}

extern "C" int lab_gemm(int variant, const uint16_t *A, const uint16_t *W, uint16_t *C, int M, int N, int K,
                        uint64_t *stamps, hipStream_t s, int group_m) {
    if (N % 256 || K % 64) return 1;
    LabArgs a{A, W, C, M, N, K, stamps, group_m};
    const int tiles = ((M + 255) / 256) * (N / 256);
    switch (variant) {
        case 0: hipLaunchKernelGGL(lab_pp<0>, dim3(tiles), dim3(512), 0, s, a); break;
        case 1: hipLaunchKernelGGL(lab_pp<1>, dim3(tiles), dim3(512), 0, s, a); break;
        case 2: hipLaunchKernelGGL(lab_pp<2>, dim3(tiles), dim3(512), 0, s, a); break;
        case 3: hipLaunchKernelGGL(lab_w4, dim3(tiles), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(lab_pp<4>, dim3(tiles), dim3(512), 0, s, a); break;
        case 5: hipLaunchKernelGGL(lab_w4r, dim3(tiles), dim3(256), 0, s, a); break;
        case 6: hipLaunchKernelGGL(lab_pp2, dim3(tiles), dim3(512), 0, s, a); break;
        case 7: hipLaunchKernelGGL(lab_ring<4>, dim3(tiles), dim3(512), 0, s, a); break;
        case 8: hipLaunchKernelGGL(lab_ring<5>, dim3(tiles), dim3(512), 0, s, a); break;
        case 9: hipLaunchKernelGGL(lab_ppw, dim3(tiles), dim3(512), 0, s, a); break;
        case 10: hipLaunchKernelGGL(lab_w4p, dim3(tiles), dim3(256), 0, s, a); break;
        case 11: hipLaunchKernelGGL(lab_w4a, dim3(tiles), dim3(256), 0, s, a); break;
        case 12: hipLaunchKernelGGL(lab_ppd<0>, dim3(tiles < 256 ? tiles : 256), dim3(512), 0, s, a); break;
        case 13: hipLaunchKernelGGL(lab_ppd<4>, dim3(tiles < 256 ? tiles : 256), dim3(512), 0, s, a); break;
        case 14: hipLaunchKernelGGL(lab_ppd<6>, dim3(tiles < 256 ? tiles : 256), dim3(512), 0, s, a); break;
        case 15: hipLaunchKernelGGL(lab_ppd<8>, dim3(tiles < 256 ? tiles : 256), dim3(512), 0, s, a); break;
        case 16: hipLaunchKernelGGL(lab_pp<16>, dim3(tiles), dim3(512), 0, s, a); break;   // ablation: no DMA in the loop
        case 32: hipLaunchKernelGGL(lab_pp<32>, dim3(tiles), dim3(512), 0, s, a); break;   // no LDS reads after step 0
        case 48: hipLaunchKernelGGL(lab_pp<48>, dim3(tiles), dim3(512), 0, s, a); break;   // neither: MFMA + barriers
        case 64: hipLaunchKernelGGL(lab_pp<64>, dim3(tiles), dim3(512), 0, s, a); break;   // no MFMA
        case 128: hipLaunchKernelGGL(lab_pp<128>, dim3(tiles), dim3(512), 0, s, a); break;  // no C stores
        case 176: hipLaunchKernelGGL(lab_pp<176>, dim3(tiles), dim3(512), 0, s, a); break;  // MFMA + barriers only
        default: return 2;
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
