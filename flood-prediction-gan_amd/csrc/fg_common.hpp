// Shared helpers for the floodgan HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>

#include "floodgan.h"

#define FG_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace fg {

// Records a message for fg_last_error() and returns `code`.
int fail(int code, const char* fmt, ...);

// Checks the most recent launch; returns 0 or the hipError_t (message recorded).
int launched(const char* what);

// Compute units of the current device (persistent-kernel grid sizing).
int num_cus();

// Blocks per XCD-aware remap: consecutive remapped ids land on the same XCD (blocks are
// dealt round-robin over the 8 XCDs), bijective for any grid size (guide §5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float act_fwd(float v, int act) {
    if (act == FG_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == FG_ACT_LRELU) return v > 0.f ? v : 0.2f * v;
    return v;
}

// derivative of the activation given its INPUT (pre-activation) value
__device__ __forceinline__ float act_grad(float pre, int act) {
    if (act == FG_ACT_RELU) return pre > 0.f ? 1.f : 0.f;
    if (act == FG_ACT_LRELU) return pre > 0.f ? 1.f : 0.2f;
    return 1.f;
}

// reflect an index into [0, n) the way F.pad(mode="reflect") does (|overhang| < n)
__device__ __forceinline__ int reflect_idx(int i, int n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * (n - 1) - i;
    return i;
}

__device__ __forceinline__ size_t vidx(const fg_view& v, int n, int y, int x) {
    const int hp = v.h + 2 * v.pad, wp = v.w + 2 * v.pad;
    return ((size_t)(n * hp + y + v.pad) * wp + (x + v.pad)) * (size_t)v.c_alloc;
}

inline size_t view_elems(const fg_view& v) {
    return (size_t)v.n * (v.h + 2 * v.pad) * (v.w + 2 * v.pad) * v.c_alloc;
}

// Cross-lane sums on the VALU (DPP / gfx950 permlane swaps) instead of ds_bpermute (__shfl_xor goes through the LDS
// crossbar): the same pairings as the xor butterflies they replace, so the results are bit-identical.
// row_sum16: every lane gets the sum over its row of 16 lanes (xor 1, 2, then the quad / half-row mirrors = xor 4, 8)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp<0xB1>(v);      // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);      // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);     // row_half_mirror: quad q <-> the other quad of the half-row
    v += dpp<0x140>(v);     // row_mirror: half-row <-> half-row
    return v;
}
// rows_sum4: every lane gets the sum of the value over lanes l, l^16, l^32, l^48 ((x0 + x1) + (x2 + x3) by row)
__device__ __forceinline__ float rows_sum4(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// head1x1.hip: the 1x1 head's weight-gradient slab reduction ([block][n_out][65] -> dw [n_out][64], db [n_out])
int conv1x1_wgrad_reduce_launch(const float* slab, int blocks, int n_out, float* dw, float* db, int accumulate,
                                hipStream_t stream);

// Timing arm (fg_timing_arm): the calling thread's next FG_LAUNCH dispatches with these start / stop events attached
// to the kernel's own dispatch packet (hipExtLaunchKernel), so the measurement adds no packet to the stream.
extern thread_local hipEvent_t g_arm_start, g_arm_stop;

template <typename F, typename... Args>
inline void launch_armed(F kernel, const dim3& grid, const dim3& block, uint32_t shmem, hipStream_t stream,
                         Args... args) {
    hipEvent_t s = g_arm_start, e = g_arm_stop;
    g_arm_start = g_arm_stop = nullptr;
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, s, e, 0, args...);
}

inline int blocks_for(long long work, int per_block, int cap = 1 << 20) {
    long long b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

}  // namespace fg

// The launch form of the convolution kernels (the kernels an fg_conv_fwd / fg_conv_wgrad call dispatches, which
// bench.py times live): a plain hipLaunchKernelGGL unless the thread holds a timing arm
#define FG_LAUNCH(K, G, B, S, ST, ...)                                              \
    do {                                                                            \
        if (fg::g_arm_start) fg::launch_armed(K, G, B, S, ST, __VA_ARGS__);         \
        else hipLaunchKernelGGL(K, G, B, S, ST, __VA_ARGS__);                       \
    } while (0)
