// topk.h — wavefront-level partial top-k (ballot-filtered append + register
// bitonic sort), the selection stage of the exact cosine search.
//
// A candidate is a 64-bit key: high word = ~order(score), low word = row (or
// list position).  Ascending key order is "score descending, then row
// ascending" — the oracle's tie rule (oracle/cosine_topk.py) — so selection is
// exact: a candidate enters the running top-k iff key < key_of_kth.
#pragma once

#include <type_traits>

#include "rc_common.h"

namespace rc {

constexpr uint64_t KEY_EMPTY = ~0ull;

// LDS-qualified pointer: keeps candidate-buffer traffic on ds_* (never flat_*).
typedef __attribute__((address_space(3))) uint64_t lds_u64;
template <class P>
__device__ __forceinline__ lds_u64 *as_lds(P *p) {
    return (lds_u64 *)(p);
}

// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N).
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

// monotone u32 image of an f32 (−0 folded into +0)
__device__ __forceinline__ uint32_t f32_order(float f) {
    uint32_t u = __float_as_uint(f + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float order_f32(uint32_t o) {
    uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t make_key(float score, uint32_t idx) {
    return ((uint64_t)(~f32_order(score)) << 32) | (uint64_t)idx;
}
__device__ __forceinline__ float key_score(uint64_t k) { return order_f32(~(uint32_t)(k >> 32)); }
__device__ __forceinline__ uint32_t key_idx(uint64_t k) { return (uint32_t)k; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, m);
    hi = __shfl_xor(hi, m);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a < b ? b : a; }

// Ascending bitonic sort of 64*E keys held as v[e] at index i = lane*E + e.
template <int E>
__device__ __forceinline__ void wave_bitonic_sort(uint64_t (&v)[E]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int size = 2; size <= 64 * E; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= E) {
                const int lm = stride / E;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int i = lane * E + e;
                    const uint64_t o = shfl_xor_u64(v[e], lm);
                    const bool up = (i & size) == 0;
                    const bool lower = (i & stride) == 0;
                    v[e] = (lower == up) ? umin64(v[e], o) : umax64(v[e], o);
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int p = e ^ stride;
                    if (p > e) {
                        const int i = lane * E + e;
                        const bool up = (i & size) == 0;
                        const uint64_t a = v[e], b = v[p];
                        const uint64_t lo = umin64(a, b), hi = umax64(a, b);
                        v[e] = up ? lo : hi;
                        v[p] = up ? hi : lo;
                    }
                }
            }
        }
    }
}

// Orders this wave's LDS traffic (the LDS unit executes one wave's DS ops in
// order; this stops the compiler from reordering them across lanes' hand-offs).
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Running top-k of one wave: an LDS buffer of CAP keys (CAP = 64*E), a
// wave-uniform fill count and threshold.  k <= CAP/2.
template <int CAP>
struct WaveTopK {
    static constexpr int E = CAP / 64;
    lds_u64 *buf;
    int count;
    int k;
    uint64_t thr;

    __device__ __forceinline__ void init(lds_u64 *b, int k_) {
        buf = b;
        count = 0;
        k = k_;
        thr = KEY_EMPTY;
    }

    // Wave-collective: every lane offers one candidate.
    __device__ __forceinline__ void push(bool valid, uint64_t key) {
        const bool take = valid && key < thr;
        const uint64_t m = __ballot(take);
        if (take) {
            const int pos = count + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            buf[pos] = key;
        }
        count += __popcll(m);
    }

    // Wave-collective: sort the buffer, keep the best k, refresh the threshold.
    // After compact(), buf[0..k) holds the sorted best keys (KEY_EMPTY-padded).
    __device__ __forceinline__ void compact() {
        const int lane = threadIdx.x & 63;
        wave_lds_fence();
        uint64_t v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = lane * E + e;
            v[e] = (i < count) ? buf[i] : KEY_EMPTY;
        }
        wave_bitonic_sort<E>(v);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = lane * E + e;
            if (i < k) buf[i] = v[e];
        }
        wave_lds_fence();
        count = count < k ? count : k;
        thr = (count >= k) ? buf[k - 1] : KEY_EMPTY;
    }

    __device__ __forceinline__ void reserve(int incoming) {
        if (count + incoming > CAP) compact();
    }
};

}  // namespace rc
