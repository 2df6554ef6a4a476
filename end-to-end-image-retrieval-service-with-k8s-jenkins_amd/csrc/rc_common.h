// rc_common.h — shared host/device helpers for the retrieval core (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "retrieval_core.h"

namespace rc {

// ----------------------------------------------------------------- errors --
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

#define RC_HIP(expr)                                                                             \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            throw ::rc::Error(RC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

#define RC_REQUIRE(cond, code, msg)                                                              \
    do {                                                                                         \
        if (!(cond)) throw ::rc::Error((code), (msg));                                           \
    } while (0)

#define RC_LAUNCH_CHECK() RC_HIP(hipGetLastError())

// compute units of the current device (cached per device id; launch-shape decisions)
inline int device_cu_count() {
    static std::atomic<int> cache[16] = {};
    int dev = 0;
    RC_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 16) {
        int n = 0;
        RC_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
        return n;
    }
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n == 0) {
        RC_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

template <class F>
int guard(F &&f) {
    try {
        f();
        return RC_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("host allocation failed");
        return RC_ERR_OOM;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return RC_ERR_INVALID;
    }
}

// Make `dev` current for the scope of a call, restoring the caller's device.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        RC_HIP(hipGetDevice(&prev));
        if (prev != dev) RC_HIP(hipSetDevice(dev));
    }
    ~DeviceScope() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
    }
};

// Device + pinned-host allocations made by the library (rc_alloc_count: tests check
// that steady-state hot calls allocate nothing).
inline std::atomic<int64_t> g_alloc_count{0};

inline void *dmalloc(size_t bytes) {
    void *p = nullptr;
    if (bytes == 0) return nullptr;
    g_alloc_count.fetch_add(1, std::memory_order_relaxed);
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        throw Error(RC_ERR_OOM, "hipMalloc(" + std::to_string(bytes) + " B) failed: " + hipGetErrorString(e));
    }
    return p;
}

inline void dfree(void *p) {
    if (p) (void)hipFree(p);
}

// Pinned host memory (async H2D / D2H staging).
inline void *hmalloc(size_t bytes) {
    void *p = nullptr;
    if (bytes == 0) return nullptr;
    g_alloc_count.fetch_add(1, std::memory_order_relaxed);
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        throw Error(RC_ERR_OOM, "hipHostMalloc(" + std::to_string(bytes) + " B) failed: " + hipGetErrorString(e));
    }
    return p;
}

inline void hfree(void *p) {
    if (p) (void)hipHostFree(p);
}

// Host f32 → bf16 bits, round to nearest even (NaN kept NaN).
inline uint16_t host_f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// ----------------------------------------------------------------- timing --
// Event-pair timing of selected launches on the launch stream.
struct KernelTimer {
    static constexpr int kMaxPairs = 4096;
    hipEvent_t ev[2 * kMaxPairs] = {};
    int used = 0;
    bool enabled = false;
    bool created = false;
    double total_ms = 0.0;
    int64_t launches = 0;
    double work = 0.0;  // algorithmic bytes or flops of the timed launches
    double pending_work[kMaxPairs] = {};

    void create() {
        if (created) return;
        for (auto &e : ev) RC_HIP(hipEventCreate(&e));
        created = true;
    }
    void destroy() {
        if (!created) return;
        for (auto &e : ev) (void)hipEventDestroy(e);
        created = false;
    }
    // returns pair slot or -1
    int begin(hipStream_t s) {
        if (!enabled) return -1;
        if (used >= kMaxPairs) flush();
        int slot = used++;
        RC_HIP(hipEventRecord(ev[2 * slot], s));
        return slot;
    }
    void end(int slot, hipStream_t s, double w) {
        if (slot < 0) return;
        RC_HIP(hipEventRecord(ev[2 * slot + 1], s));
        pending_work[slot] = w;
    }
    void flush() {
        for (int i = 0; i < used; ++i) {
            RC_HIP(hipEventSynchronize(ev[2 * i + 1]));
            float ms = 0.f;
            RC_HIP(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
            total_ms += ms;
            launches += 1;
            work += pending_work[i];
        }
        used = 0;
    }
    void reset() {
        flush();
        total_ms = 0.0;
        launches = 0;
        work = 0.0;
    }
};

}  // namespace rc

// ================================================================= device ==
#if defined(__HIPCC__)
namespace rc {

// Pillow's fixed-point resample tap acc + pixel·coef: the pixel is a byte and |coef| < 2^23
// (precompute_coeffs checks it), so the product is v_mad_i32_i24's — a full-rate op, where the
// 32-bit multiply hipcc emits otherwise (v_mul_lo_u32 / v_mad_u64_u32) issues at a quarter rate.
// The same bits: the exact product fits 32 bits either way.
__device__ __forceinline__ int resample_tap(int acc, int pixel, int coef) { return __mul24(pixel, coef) + acc; }
__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// f32 → bf16 bits, round to nearest even (finite inputs; hipcc lowers a plain
// conversion of this form to v_cvt_pk_bf16_f32 on gfx950 where it can).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// Two f32 → packed bf16x2, round to nearest even: one v_cvt_pk_bf16_f32 (same
// bits as f32_to_bf16 for finite inputs; keeps a NaN a NaN).
typedef __bf16 rc_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    const rc_bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
    _Float16 x = __builtin_bit_cast(_Float16, h);
    return (float)x;
}

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    _Float16 x = (_Float16)f;
    return __builtin_bit_cast(uint16_t, x);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over each aligned group of 16 lanes; every lane of the group gets the sum.
// quad_perm[1,0,3,2] → quad_perm[2,3,0,1] → row_half_mirror → row_mirror.
__device__ __forceinline__ float sum16(float v) {
    v += dpp_f32<0xB1>(v);
    v += dpp_f32<0x4E>(v);
    v += dpp_f32<0x141>(v);
    v += dpp_f32<0x140>(v);
    return v;
}

// Full wave (64-lane) sum, every lane gets the result.
__device__ __forceinline__ float wave_sum(float v) {
    v = sum16(v);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

}  // namespace rc
#endif
