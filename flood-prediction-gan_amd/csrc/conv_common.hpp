// Shared pieces of the convolution engine (conv_gemm.hip: generic register-staged kernels;
// conv_f3.hip: the LDS-DMA pipelined f16x3 forward kernel).
#pragma once
#include "fg_common.hpp"

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace fgc {

// Up to four fg_conv_problems sharing one launch (the four output phases of a stride-2
// transposed conv); blocks [blk_start[i], blk_start[i+1]) belong to problem i -- or, with
// interleave set (problems of equal tile counts, set by the pipelined kernel's launcher), tile t
// belongs to problem t % count as its local tile t / count, so that the phases reading the same
// input rows run side by side and share them in L2 instead of streaming the input once per phase.
struct ConvBatch {
    fg_conv_problem p[4];
    int count;
    int ntiles_n[4];
    int blk_start[5];
    int interleave;
};

// n / d for 0 <= n < 2^22, 1 <= d < 2^22 by a float reciprocal: |n*rcp(d) - n/d| < 2^22 * 2^-22.4 < 1, so
// one correction step is exact (an integer division is a ~30-instruction VALU sequence; this is ~8)
__device__ __forceinline__ int div_small(int n, int d) {
    int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
    const int r = n - q * d;
    q += r >= d ? 1 : (r < 0 ? -1 : 0);
    return q;
}

__device__ __forceinline__ void decomp(int m, int mb, int mab, int& img, int& a, int& b) {
    if (m < (1 << 22) && mab < (1 << 22)) {
        img = div_small(m, mab);
        const int rem = m - img * mab;
        a = div_small(rem, mb);
        b = rem - a * mb;
    } else {
        img = m / mab;
        const int rem = m - img * mab;
        a = rem / mb;
        b = rem - a * mb;
    }
}

// the power-of-two scale s = 2^(14-e) of a bound m < 2^e (1 for 0 / non-finite): |v * s| < 2^14
__device__ __forceinline__ float pow2_of(float m) {
    if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
    int e;
    frexpf(m, &e);                                        // m < 2^e
    return ldexpf(1.f, 14 - e);
}

// max over an absmax slot's FG_AMAX_SHARDS shards (every lane of the wave gets it)
__device__ __forceinline__ float pow2_scale_max(const float* amax) {
    unsigned b = __float_as_uint(amax[threadIdx.x & (FG_AMAX_SHARDS - 1)]) & 0x7fffffffu;
#pragma unroll
    for (int off = 1; off < FG_AMAX_SHARDS; off <<= 1) b = max(b, (unsigned)__shfl_xor((int)b, off));
    return __uint_as_float(b);
}

// power-of-two operand scale from an absmax slot (max over its FG_AMAX_SHARDS shards, one per
// lane, reduced across the wave): |v * s| < 2^14
__device__ __forceinline__ float pow2_scale(const float* amax) {
    unsigned b = amax ? __float_as_uint(amax[threadIdx.x & (FG_AMAX_SHARDS - 1)]) & 0x7fffffffu : 0u;
#pragma unroll
    for (int off = 1; off < FG_AMAX_SHARDS; off <<= 1) b = max(b, (unsigned)__shfl_xor((int)b, off));
    return pow2_of(__uint_as_float(b));
}

// f16x3 split of 8 fp32 values: v*s = h + l, h = fp16(v*s), l = fp16(v*s - h)
__device__ __forceinline__ void split_f16(const float (&v)[8], float s, f16x8& h, f16x8& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const f32x2 x = f32x2{v[2 * e], v[2 * e + 1]} * s;
        const f16x2 hh = __builtin_convertvector(x, f16x2);
        const f16x2 ll = __builtin_convertvector(x - __builtin_convertvector(hh, f32x2), f16x2);
        h[2 * e] = hh[0];
        h[2 * e + 1] = hh[1];
        l[2 * e] = ll[0];
        l[2 * e + 1] = ll[1];
    }
}

// f16x3 split of a pair with the scale folded into mixed-precision FMAs: v_fma_mixlo/mixhi_f16 compute an fp32
// fma and round it to fp16 into one half of the destination, so h = fp16(x*s) and l = fp16(x*s - h) take four
// instructions per pair instead of two v_mul, two v_fma_mix_f32 and two v_cvt_pk (bit-identical: x*s with a
// power-of-two s and x*s - h are exact in fp32 and both are rounded once, to nearest even).
__device__ __forceinline__ void split_pair_mix(float x0, float x1, float s, unsigned& h, unsigned& l) {
    unsigned hv, lv;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %2, 0"
        : "=&v"(hv) : "v"(x0), "v"(s), "v"(x1));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%4 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, %2, -%4 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(lv) : "v"(x0), "v"(s), "v"(x1), "v"(hv));
    h = hv;
    l = lv;
}

// 16-B chunk swizzle of a pre-split pixel (fg_split_pixels): chunk k of [h | l] of the pixel in
// padded column x is stored at k ^ swz_pixel(x) -- conflict-free shifted fragment reads
// (exhaustive search over the ds_read_b128 lane groups and every row offset)
template <int C>
__device__ __forceinline__ int swz_pixel(int x) {
    if constexpr (C == 64) return (x & 7) << 1;          // 16 chunks per 256-B pixel
    else return ((x >> 1) & 3) << 1;                     // 8 chunks per 128-B pixel (C == 32)
}

// Pipelined f16x3 forward kernel (conv_f3.hip).  Returns 1 if it took the batch (launched or
// failed: *rc holds the launch status), 0 if the batch does not fit its constraints.
int launch_fwd_f3(const ConvBatch& b, int nprob, int max_n, hipStream_t stream, int* rc);
bool f3_stats_ok(const fg_conv_problem* probs, int nprob, int max_n);

// Pipelined f16x3 weight-gradient kernel (conv_wgrad_f3.hip), same contract.
int launch_wgrad_f3(const fg_wgrad_problem& p, hipStream_t stream, int* rc);

// The generator stem's weight gradient (conv_stem.hip: 7x7, 9 -> 64 channels, 64-px strips of m_chunk / 64
// rows per split), same contract; stem_wgrad_rows = its rows per split, or 0 when it does not apply.
int stem_wgrad_rows(const fg_wgrad_problem& p);
int launch_wgrad_stem(const fg_wgrad_problem& p, hipStream_t stream, int* rc);
// The stem's forward (conv_stem.hip), same contract; stem_fwd_rows = its rows per workgroup, or 0 when it does not
// apply.  It also honours fg_conv_problem.in_stats.
int stem_fwd_rows(const fg_conv_problem& p);
int launch_fwd_stem(const fg_conv_problem& p, hipStream_t stream, int* rc);

}  // namespace fgc
