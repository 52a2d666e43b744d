// The PatchGAN's last conv, model.11 (Conv2d(512, 1, 4, 1, 1), models/model_architectures.py:437):
// one output channel, so it is a 8192-long dot product per output pixel -- GEMV-shaped, no
// matrix-core work.  The implicit-GEMM engine ran it as a 32-column tile with 31 idle columns,
// re-gathering each input pixel 16 times (~0.25 ms per call at batch 16).  Here, in plain fp32
// FMA (the reference's arithmetic):
//   forward: one wave per 4 consecutive output pixels, lanes over channels (8 each), the 16 taps'
//            weights held in registers, a wave reduction per pixel;
//   weight gradient: input-pixel-centric -- each thread owns 2 channels x 16 taps of dW and adds
//            g[y-r][x-s] * a[y][x][c] for the 16 output pixels that read input pixel (y, x), so
//            every input pixel is read once; per-block partial sums go to fg_wgrad_reduce slabs.
#include "fg_common.hpp"

namespace {

constexpr int C = 512, KT = 16;   // channels, 4x4 taps

// x: padded input (pad 1) of image n at (row, col) -> x + ((n*hp + row)*wp + col)*C
__global__ void __launch_bounds__(256) n1_fwd_kernel(const float* __restrict__ x, int hp, int wp,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     float* __restrict__ y, int nimg, int ho, int wo) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);            // global wave: 4 pixels of one row
    const int qpr = (wo + 3) / 4;                                   // quads per output row
    const int row = gw / qpr;                                       // n*ho + oy
    if (row >= nimg * ho) return;
    const int n = row / ho, oy = row - n * ho, ox0 = (gw - row * qpr) * 4;
    // weights of this lane's 8 channels, 16 taps: w[0][c][r][s] = w[c*16 + r*4 + s]
    float wr[8][KT];
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int t4 = 0; t4 < KT / 4; ++t4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(w + (size_t)(lane * 8 + e) * KT + t4 * 4);
            wr[e][t4 * 4 + 0] = v[0];
            wr[e][t4 * 4 + 1] = v[1];
            wr[e][t4 * 4 + 2] = v[2];
            wr[e][t4 * 4 + 3] = v[3];
        }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float* xrow = x + ((size_t)(n * hp + oy + r) * wp + ox0) * C + lane * 8;
#pragma unroll
        for (int j = 0; j < 7; ++j) {                               // input columns ox0 .. ox0+6
            if (ox0 + j >= wp) break;
            const f32x4 a = *reinterpret_cast<const f32x4*>(xrow + j * C);
            const f32x4 b = *reinterpret_cast<const f32x4*>(xrow + j * C + 4);
            const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
            for (int p = 0; p < 4; ++p) {                           // output ox0+p uses tap s = j - p
                const int s = j - p;
                if (s < 0 || s > 3) continue;
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[p] = fmaf(v[e], wr[e][r * 4 + s], acc[p]);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        float v = acc[p];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0 && ox0 + p < wo) y[(size_t)row * wo + ox0 + p] = v + (bias ? bias[0] : 0.f);
    }
}

// gp: output gradient with a zero border of 3 (so g[y-r][x-s] never leaves the buffer) of image
// n at (row, col) -> gp + (n*ghp + row)*gwp + col; block = (image, band of input rows)
__global__ void __launch_bounds__(256) n1_wgrad_kernel(const float* __restrict__ x, int hp, int wp,
                                                       const float* __restrict__ gp, int ghp, int gwp, int nimg,
                                                       int rows_per_block, float* __restrict__ slabs) {
    const int bands = (hp + rows_per_block - 1) / rows_per_block;
    const int n = blockIdx.x / bands, band = blockIdx.x - n * bands;
    const int y0 = band * rows_per_block, y1 = min(hp, y0 + rows_per_block);
    const int c0 = threadIdx.x * 2;
    float acc[2][KT];
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < KT; ++t) acc[e][t] = 0.f;
    for (int yy = y0; yy < y1; ++yy) {
        const float* xrow = x + ((size_t)(n * hp + yy) * wp) * C + c0;
        // gradient rows y = yy - r sit at padded row yy - r + 3
        const float* grow = gp + (size_t)(n * ghp + yy + 3) * gwp + 3;
        for (int xx = 0; xx < wp; ++xx) {
            const float2 a = *reinterpret_cast<const float2*>(xrow + (size_t)xx * C);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const float g = grow[-r * gwp + xx - s];
                    acc[0][r * 4 + s] = fmaf(g, a.x, acc[0][r * 4 + s]);
                    acc[1][r * 4 + s] = fmaf(g, a.y, acc[1][r * 4 + s]);
                }
        }
    }
    // slab layout of fg_conv_wgrad for n_a = 1: k = r*(4*C) + s*C + c
    float* out = slabs + (size_t)blockIdx.x * KT * C;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < KT; ++t) out[(t >> 2) * 4 * C + (t & 3) * C + c0 + e] = acc[e][t];
}

}  // namespace

FG_API int fg_conv_n1_fwd(const float* x, int nimg, int hp, int wp, int c, const float* w, const float* bias,
                          float* y, int ho, int wo, hipStream_t stream) {
    if (!x || !w || !y || c != C || nimg < 1 || ho != hp - 3 || wo != wp - 3 || ho < 1 || wo < 1 ||
        ((uintptr_t)x & 15) || ((uintptr_t)w & 15))
        return fg::fail(FG_ERR_INVALID, "fg_conv_n1_fwd: needs a 512-channel input padded by 1, a 4x4 kernel, "
                                        "stride 1 (ho = hp - 3)");
    const long long waves = (long long)nimg * ho * ((wo + 3) / 4);
    hipLaunchKernelGGL(n1_fwd_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, stream, x, hp, wp, w, bias, y,
                       nimg, ho, wo);
    return fg::launched("conv_n1_fwd");
}

FG_API int fg_conv_n1_wgrad_blocks(int nimg, int hp, int rows_per_block) {
    return nimg * ((hp + rows_per_block - 1) / rows_per_block);
}

FG_API int fg_conv_n1_wgrad(const float* x, int nimg, int hp, int wp, int c, const float* gp, int ghp, int gwp,
                            int rows_per_block, float* slabs, hipStream_t stream) {
    if (!x || !gp || !slabs || c != C || nimg < 1 || rows_per_block < 1 || ghp != hp - 3 + 6 || gwp != wp - 3 + 6 ||
        ((uintptr_t)x & 7))
        return fg::fail(FG_ERR_INVALID, "fg_conv_n1_wgrad: needs a 512-channel input padded by 1 and the output "
                                        "gradient with a zero border of 3");
    hipLaunchKernelGGL(n1_wgrad_kernel, dim3(fg_conv_n1_wgrad_blocks(nimg, hp, rows_per_block)), dim3(256), 0, stream,
                       x, hp, wp, gp, ghp, gwp, nimg, rows_per_block, slabs);
    return fg::launched("conv_n1_wgrad");
}
