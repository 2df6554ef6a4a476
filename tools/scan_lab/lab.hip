// Scan lab (diagnostic, not product): how fast can a 1M x 512 f32 row stream be read on one
// MI355X with the product scan's load shape (16 lanes per row, 16-B chunks, SCAN_U row groups
// per wave in flight), and what do nontemporal loads / deeper unrolling / block counts change?
// Each kernel computes the 16-lane dot product with a query held in registers and keeps a
// per-lane running max (no top-k), so the difference to scan_topk_kernel is the top-k work.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/scan_lab/lab.hip -o tools/scan_lab/liblab.so
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
template <int U, bool NT>
__global__ __launch_bounds__(256, 4) void stream_kernel(const float *__restrict__ rows, int64_t n_rows, int64_t rows_per_block,
                                                        const float *__restrict__ q, float *__restrict__ out) {
    constexpr int CPL = 8;  // 512 floats = 128 chunks of 16 B, 16 lanes per row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15, rg = lane >> 4;
    float qr[CPL][4];
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) qr[i][e] = q[(sub + 16 * i) * 4 + e];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(n_rows, r0 + rows_per_block);
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v *b4 = reinterpret_cast<const f4v *>(rows);
    float best = -1e30f;
    for (int64_t g = r0 + wave * 4 * U; g < r1; g += 16 * U) {
        f4v x[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = g + u * 4 + rg;
            const int64_t rr = r < r1 ? r : r0;
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                const f4v *p = b4 + rr * 128 + sub + 16 * i;
                if constexpr (NT) x[u][i] = __builtin_nontemporal_load(p);
                else x[u][i] = *p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                acc = fmaf(x[u][i].x, qr[i][0], acc);
                acc = fmaf(x[u][i].y, qr[i][1], acc);
                acc = fmaf(x[u][i].z, qr[i][2], acc);
                acc = fmaf(x[u][i].w, qr[i][3], acc);
            }
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
            best = fmaxf(best, acc);
        }
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = best;
}
}  // namespace

extern "C" int lab_stream(int variant, const float *rows, int64_t n_rows, int nblk, const float *q, float *out, void *stream) {
    const int64_t rpb = (n_rows + nblk - 1) / nblk;
    hipStream_t s = (hipStream_t)stream;
    switch (variant) {
        case 0: hipLaunchKernelGGL((stream_kernel<2, false>), dim3(nblk), dim3(256), 0, s, rows, n_rows, rpb, q, out); break;
        case 1: hipLaunchKernelGGL((stream_kernel<2, true>), dim3(nblk), dim3(256), 0, s, rows, n_rows, rpb, q, out); break;
        case 2: hipLaunchKernelGGL((stream_kernel<1, false>), dim3(nblk), dim3(256), 0, s, rows, n_rows, rpb, q, out); break;
        case 3: hipLaunchKernelGGL((stream_kernel<3, false>), dim3(nblk), dim3(256), 0, s, rows, n_rows, rpb, q, out); break;
        case 4: hipLaunchKernelGGL((stream_kernel<3, true>), dim3(nblk), dim3(256), 0, s, rows, n_rows, rpb, q, out); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
