// The attention head deconv3_attention (Conv2d(64, 10, 1), models/model_architectures.py:334, :369) and its
// two gradients in plain fp32 FMA.  A 1x1 conv with 10 outputs over 64-channel pixels is a per-pixel
// matrix-vector product (640 FMA per 256 B), far below the MFMA ridge: the implicit-GEMM engine's
// 32-column tiles moved it at ~2.2 TB/s (260 / 193 / 282 us forward / input gradient / weight gradient at
// bs 8, 512^2).  Each kernel here stages a 64-pixel tile of its pixel-major operands into LDS with
// coalesced 16-B loads (a thread owning a whole pixel would make every wave-wide load touch 64 lines), then
// works from LDS:
//   input gradient: thread = (pixel, group of 16 input channels), writes 4 float4 of the 64-channel row;
//   weight + bias:  thread = (output o, channel quad), sums over the block's pixels; per-block partials are
//                   reduced over blocks in fp64 in a fixed order (deterministic).
#include <algorithm>

#include "fg_common.hpp"

namespace {

constexpr int CI = 64;        // input channels
constexpr int NO = 16;        // output channels handled (n_out <= NO): the logits buffer's allocation
constexpr int TP = 64;        // pixels per tile
constexpr int XS = CI + 4;    // padded LDS row (floats): rows start 4 banks apart, b128 reads conflict-free
constexpr int GS = NO + 4;

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }

// interior pixel p of a view -> element offset of its channel 0
__device__ __forceinline__ size_t pix_off(const fg_view& v, int p) {
    const int hw = v.h * v.w;
    const int n = p / hw, r = p - n * hw, yy = r / v.w, xx = r - yy * v.w;
    return fg::vidx(v, n, yy, xx);
}

// stage `q4` float4 quads per pixel of pixels [p0, p0 + TP) of v into LDS rows of `stride` floats
__device__ __forceinline__ void stage(const fg_view& v, int q4, int p0, int P, float* lds, int stride) {
    for (int i = threadIdx.x; i < TP * q4; i += 256) {
        const int px = i / q4, q = i - px * q4, p = p0 + px;
        const f32x4 val = p < P ? ld4(v.ptr + pix_off(v, p) + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        st4(lds + px * stride + 4 * q, val);
    }
}

__global__ void __launch_bounds__(256) conv1x1_dgrad_kernel(fg_view gy, const float* __restrict__ w, int n_out,
                                                            fg_view gx) {
    __shared__ __attribute__((aligned(16))) float gs[2][TP * GS];
    __shared__ __attribute__((aligned(16))) float ws[NO * XS];
    const int P = gx.n * gx.h * gx.w, ntiles = (P + TP - 1) / TP;
    const int q4 = (n_out + 3) / 4;                    // gradient quads per pixel (<= 4)
    // persistent like the forward: weights once per block, the next tile's gradient rows in registers
    for (int i = threadIdx.x; i < NO * CI; i += 256) {
        const int o = i / CI, c = i - o * CI;
        ws[o * XS + c] = o < n_out ? w[i] : 0.f;
    }
    const int px = threadIdx.x >> 2, cg = threadIdx.x & 3;   // channels 16 cg .. 16 cg + 15
    f32x4 rv;                                          // thread t: pixel t / 4, quad t % 4 of the tile
    auto load = [&](int t) {
        const int pp = threadIdx.x >> 2, q = threadIdx.x & 3, p = t * TP + pp;
        rv = (t < ntiles && p < P && q < q4) ? ld4(gy.ptr + pix_off(gy, p) + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto store = [&](float* dst) { st4(dst + (threadIdx.x >> 2) * GS + 4 * (threadIdx.x & 3), rv); };
    int t = blockIdx.x, buf = 0;
    load(t);
    store(gs[0]);
    load(t + gridDim.x);
    __syncthreads();
    for (; t < ntiles; t += gridDim.x, buf ^= 1) {
        if (t + gridDim.x < ntiles) store(gs[buf ^ 1]);
        load(t + 2 * gridDim.x);
        const int p = t * TP + px;
        f32x4 a[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* gr = gs[buf] + px * GS;
        for (int o = 0; o < n_out; ++o) {
            const float g = gr[o];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4 wv = ld4(ws + o * XS + 16 * cg + 4 * k);
                a[k][0] = fmaf(g, wv[0], a[k][0]);
                a[k][1] = fmaf(g, wv[1], a[k][1]);
                a[k][2] = fmaf(g, wv[2], a[k][2]);
                a[k][3] = fmaf(g, wv[3], a[k][3]);
            }
        }
        if (p < P) {
            float* dst = gx.ptr + pix_off(gx, p) + 16 * cg;
#pragma unroll
            for (int k = 0; k < 4; ++k) st4(dst + 4 * k, a[k]);
        }
        __syncthreads();
    }
}

// ---- the forward's lane form (round 4): no LDS staging.  A wave takes 4 pixels per step, lane = (pixel group pg,
// channel quad cq): the 16 lanes of a pixel read its 64 channels as one contiguous 256-B segment; the weights sit in
// registers for the whole launch; LU steps' loads are in flight together.  Each lane forms the 16 outputs' partial
// dot products over its 4 channels and a DPP reduce-scatter over the 16 lanes (4 exchange steps, halving the vector
// each time) leaves output cq's sum in lane cq -- 64 B of logits written contiguously per pixel: 176 -> 131 us at
// bs 8, 512^2 (profiles/round4/r4p_kernel_stats_timed.csv).  The same form for the input gradient (the 16 lanes of a
// pixel sharing its 64-B gradient row) ran 229 us against the LDS-tile kernel's 206 and was not kept.
constexpr int LU = 4;

template <int CTRL>
__device__ __forceinline__ float dppx(float v) { return fg::dpp<CTRL>(v); }

__device__ __forceinline__ size_t pix_off_fast(const fg_view& v, long long p) {
    return v.pad == 0 ? (size_t)p * v.c_alloc : pix_off(v, (int)p);
}

__global__ void __launch_bounds__(256) conv1x1_fwd_lanes(fg_view x, const float* __restrict__ w,
                                                         const float* __restrict__ b, int n_out, fg_view y) {
    const long long P = (long long)x.n * x.h * x.w;
    const int lane = threadIdx.x & 63, pg = lane >> 4, cq = lane & 15;
    const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (long long)gridDim.x * 4;
    f32x4 wr[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) wr[o] = o < n_out ? ld4(w + o * CI + 4 * cq) : f32x4{0.f, 0.f, 0.f, 0.f};
    const float bo = (b && cq < n_out) ? b[cq] : 0.f;
    const bool h3 = cq & 8, h2 = cq & 4, h1 = cq & 2, h0 = cq & 1;
    for (long long base = gw * 4 * LU; base < P; base += nw * 4 * LU) {
        f32x4 v[LU];
#pragma unroll
        for (int u = 0; u < LU; ++u) {
            const long long p = base + u * 4 + pg;
            v[u] = p < P ? ld4(x.ptr + pix_off_fast(x, p) + 4 * cq) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < LU; ++u) {
            float acc[NO];
#pragma unroll
            for (int o = 0; o < NO; ++o)
                acc[o] = fmaf(v[u][3], wr[o][3], fmaf(v[u][2], wr[o][2], fmaf(v[u][1], wr[o][1], v[u][0] * wr[o][0])));
            float a8[8], a4[4], a2[2];
#pragma unroll
            for (int k = 0; k < 8; ++k) a8[k] = (h3 ? acc[8 + k] : acc[k]) + dppx<0x140>(h3 ? acc[k] : acc[8 + k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) a4[k] = (h2 ? a8[4 + k] : a8[k]) + dppx<0x141>(h2 ? a8[k] : a8[4 + k]);
#pragma unroll
            for (int k = 0; k < 2; ++k) a2[k] = (h1 ? a4[2 + k] : a4[k]) + dppx<0x1B>(h1 ? a4[k] : a4[2 + k]);
            const float r = (h0 ? a2[1] : a2[0]) + dppx<0xB1>(h0 ? a2[0] : a2[1]);
            const long long p = base + u * 4 + pg;
            if (p < P && cq < y.c_alloc) y.ptr[pix_off_fast(y, p) + cq] = r + bo;
        }
    }
}

// block: pixels [blockIdx.x * per, +per) in tiles of TP; thread (o = t / 16, channel quad cq = t % 16)
// accumulates 4 channels of dw[o] (+ the bias sum for cq == 0); partial slab[blk][o][CI + 1]
__global__ void __launch_bounds__(256) conv1x1_wgrad_kernel(fg_view gy, fg_view x, int n_out, int per,
                                                            float* __restrict__ slab) {
    __shared__ __attribute__((aligned(16))) float xs[TP * XS];
    __shared__ __attribute__((aligned(16))) float gs[TP * GS];
    const int P = x.n * x.h * x.w;
    const int o = threadIdx.x >> 4, cq = threadIdx.x & 15;
    const int pb = blockIdx.x * per, pe = min(P, pb + per);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float accb = 0.f;
    for (int p0 = pb; p0 < pe; p0 += TP) {
        __syncthreads();                                   // the previous tile's reads are done
        stage(x, CI / 4, p0, pe, xs, XS);
        stage(gy, (n_out + 3) / 4, p0, pe, gs, GS);
        __syncthreads();
        if (o < n_out) {
            const int np = min(TP, pe - p0);
            for (int px = 0; px < np; ++px) {
                const float g = gs[px * GS + o];
                const f32x4 v = ld4(xs + px * XS + 4 * cq);
                acc[0] = fmaf(g, v[0], acc[0]);
                acc[1] = fmaf(g, v[1], acc[1]);
                acc[2] = fmaf(g, v[2], acc[2]);
                acc[3] = fmaf(g, v[3], acc[3]);
                accb += g;
            }
        }
    }
    if (o < n_out) {
        float* s = slab + ((size_t)blockIdx.x * n_out + o) * (CI + 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * cq + e] = acc[e];
        if (cq == 0) s[CI] = accb;
    }
}

// out[t] (t < n_out * (CI + 1)) = sum over blocks; workgroup = 64 entries x 16 block lanes, fp64, fixed order
__global__ void __launch_bounds__(1024) conv1x1_wgrad_reduce(const float* __restrict__ slab, int blocks, int n_out,
                                                             float* __restrict__ dw, float* __restrict__ db,
                                                             int accumulate) {
    const int total = n_out * (CI + 1);
    const int e = threadIdx.x & 63, l = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + e;
    double s = 0.0;
    if (t < total)
        for (int bl = l; bl < blocks; bl += 16) s += slab[(size_t)bl * total + t];
    __shared__ double red[16][64];
    red[l][e] = s;
    __syncthreads();
    if (l != 0 || t >= total) return;
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum += red[i][e];
    const int o = t / (CI + 1), k = t - o * (CI + 1);
    float* dst = k < CI ? dw + o * CI + k : db ? db + o : nullptr;
    if (!dst) return;
    const float v = (float)sum;
    *dst = accumulate ? *dst + v : v;
}

bool ok(const fg_view& v, int c_min, int c_max) {
    return v.ptr && v.n > 0 && v.h > 0 && v.w > 0 && v.pad >= 0 && v.c_alloc >= c_min && v.c_alloc <= c_max &&
           v.c_alloc % 4 == 0 && ((uintptr_t)v.ptr & 15) == 0 && (long long)v.n * v.h * v.w < (1LL << 31);
}

bool same_grid(const fg_view& a, const fg_view& b) { return a.n == b.n && a.h == b.h && a.w == b.w; }

constexpr int WG_BLOCKS = 1024;

}  // namespace

FG_API int fg_conv1x1_fwd(fg_view x, const float* w, const float* bias, int n_out, fg_view y, hipStream_t stream) {
    if (!ok(x, CI, CI) || !ok(y, n_out, NO) || !w || n_out < 1 || n_out > NO || !same_grid(x, y))
        return fg::fail(FG_ERR_INVALID, "fg_conv1x1_fwd: bad args (c_in %d, n_out %d, y.c_alloc %d)", x.c_alloc, n_out,
                        y.c_alloc);
    const int P = x.n * x.h * x.w;
    const long long steps = ((long long)P + 4 * LU - 1) / (4 * LU);              // wave steps
    hipLaunchKernelGGL(conv1x1_fwd_lanes, dim3((unsigned)std::min<long long>((steps + 3) / 4, 8 * fg::num_cus())),
                       dim3(256), 0, stream, x, w, bias, n_out, y);
    return fg::launched("conv1x1_fwd");
}

FG_API int fg_conv1x1_dgrad(fg_view gy, const float* w, int n_out, fg_view gx, hipStream_t stream) {
    if (!ok(gy, (n_out + 3) / 4 * 4, 1 << 20) || !ok(gx, CI, CI) || !w || n_out < 1 || n_out > NO || !same_grid(gy, gx))
        return fg::fail(FG_ERR_INVALID, "fg_conv1x1_dgrad: bad args (n_out %d, gy.c_alloc %d, gx.c_alloc %d)", n_out,
                        gy.c_alloc, gx.c_alloc);
    const int P = gx.n * gx.h * gx.w;
    const int ntiles = (P + TP - 1) / TP;
    hipLaunchKernelGGL(conv1x1_dgrad_kernel, dim3(std::min(ntiles, 4 * fg::num_cus())), dim3(256), 0, stream, gy, w,
                       n_out, gx);
    return fg::launched("conv1x1_dgrad");
}

FG_API long long fg_conv1x1_wgrad_workspace_floats(int n_out) { return (long long)WG_BLOCKS * n_out * (CI + 1); }

namespace fg {
// the slab reduction of fg_conv1x1_wgrad, for the fused attention-head backward (fg_in_bwd_head) too
int conv1x1_wgrad_reduce_launch(const float* slab, int blocks, int n_out, float* dw, float* db, int accumulate,
                                hipStream_t stream) {
    const int total = n_out * (CI + 1);
    hipLaunchKernelGGL(conv1x1_wgrad_reduce, dim3((total + 63) / 64), dim3(1024), 0, stream, slab, blocks, n_out, dw, db,
                       accumulate);
    return fg::launched("conv1x1_wgrad_reduce");
}
}  // namespace fg

FG_API int fg_conv1x1_wgrad(fg_view gy, fg_view x, int n_out, float* dw, float* db, int accumulate, float* work,
                            hipStream_t stream) {
    if (!ok(gy, (n_out + 3) / 4 * 4, 1 << 20) || !ok(x, CI, CI) || !dw || !work || n_out < 1 || n_out > NO ||
        !same_grid(gy, x))
        return fg::fail(FG_ERR_INVALID, "fg_conv1x1_wgrad: bad args (n_out %d)", n_out);
    const int P = x.n * x.h * x.w;
    const int per = ((P + WG_BLOCKS - 1) / WG_BLOCKS + TP - 1) / TP * TP;
    const int blocks = (P + per - 1) / per;
    hipLaunchKernelGGL(conv1x1_wgrad_kernel, dim3(blocks), dim3(256), 0, stream, gy, x, n_out, per, work);
    int e = fg::launched("conv1x1_wgrad");
    if (e) return e;
    const int total = n_out * (CI + 1);
    hipLaunchKernelGGL(conv1x1_wgrad_reduce, dim3((total + 63) / 64), dim3(1024), 0, stream, work, blocks, n_out, dw, db,
                       accumulate);
    return fg::launched("conv1x1_wgrad_reduce");
}
