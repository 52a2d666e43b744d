// Shared helpers for the floodgan HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
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

inline int blocks_for(long long work, int per_block, int cap = 1 << 20) {
    long long b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

}  // namespace fg
