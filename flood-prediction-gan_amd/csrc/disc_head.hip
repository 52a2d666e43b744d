// The PatchGAN's last conv, model.11 (Conv2d(512, 1, 4, 1, 1), models/model_architectures.py:437):
// one output channel, so it is a 8192-long dot product per output pixel -- GEMV-shaped, no
// matrix-core work.  The implicit-GEMM engine ran it as a 32-column tile with 31 idle columns,
// re-gathering each input pixel 16 times (~0.25 ms per call at batch 16).  Here, in plain fp32
// FMA (the reference's arithmetic):
//   forward: one wave per 4 x 4 output block, lanes over channels (8 each), the 16 taps'
//            weights held in registers, the block's 7 x 7 input window read once, a wave reduction per pixel;
//   weight gradient: input-pixel-centric -- each thread owns 2 channels x 16 taps of dW and adds
//            g[y-r][x-s] * a[y][x][c] for the 16 output pixels that read input pixel (y, x), so
//            every input pixel is read once; per-block partial sums go to fg_wgrad_reduce slabs.
#include <algorithm>

#include "fg_common.hpp"

namespace {

constexpr int C = 512, KT = 16;   // channels, 4x4 taps

// x: padded input (pad 1) of image n at (row, col) -> x + ((n*hp + row)*wp + col)*C.  One wave per 4 x 4 block of
// output pixels (round 5; was 1 x 4): it reads the block's 7 x 7 input window once -- 49 pixels for 16 outputs, 3.1
// reads per output pixel instead of 7 -- and adds each input pixel's 8 channels of this lane into every output of
// the block that reads it (up to 16 taps); a wave reduction per output pixel at the end.
__global__ void __launch_bounds__(256) n1_fwd_kernel(const float* __restrict__ x, int hp, int wp,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     float* __restrict__ y, int nimg, int ho, int wo) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);            // global wave: a 4 x 4 output block
    const int bpr = (wo + 3) / 4, bpi = ((ho + 3) / 4) * bpr;      // blocks per block-row, per image
    const int n = gw / bpi;
    if (n >= nimg) return;
    const int rem = gw - n * bpi, by = rem / bpr;
    const int oy0 = by * 4, ox0 = (rem - by * bpr) * 4;
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
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
#pragma unroll
    for (int iy = 0; iy < 7; ++iy) {                               // input rows oy0 .. oy0+6
        if (oy0 + iy >= hp) break;
        const float* xrow = x + ((size_t)(n * hp + oy0 + iy) * wp + ox0) * C + lane * 8;
#pragma unroll
        for (int ix = 0; ix < 7; ++ix) {                           // input columns ox0 .. ox0+6
            if (ox0 + ix >= wp) break;
            const f32x4 a = *reinterpret_cast<const f32x4*>(xrow + ix * C);
            const f32x4 b = *reinterpret_cast<const f32x4*>(xrow + ix * C + 4);
            const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
            for (int i = 0; i < 4; ++i) {                          // output row oy0+i uses tap r = iy - i
                const int r = iy - i;
                if (r < 0 || r > 3) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j) {                      // output column ox0+j uses tap s = ix - j
                    const int s = ix - j;
                    if (s < 0 || s > 3) continue;
#pragma unroll
                    for (int e = 0; e < 8; ++e) acc[i][j] = fmaf(v[e], wr[e][r * 4 + s], acc[i][j]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v = acc[i][j];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0 && oy0 + i < ho && ox0 + j < wo)
                y[((size_t)n * ho + oy0 + i) * wo + ox0 + j] = v + (bias ? bias[0] : 0.f);
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


// ---- the PatchGAN's input gradient restricted to a few input channels (model.0, Conv2d(C+3, 64, 4, 2, 1),
// models/model_architectures.py:424): the G step needs dL/d(fake) = the gradient w.r.t. D's last 3 input
// channels only (models/model.py:640-646).  As a transposed conv it is 3 outputs x 4 taps x 64 channels per pixel:
// 0.6 GMAC at bs 8, 512^2, against 136 MB of gradient to read -- memory-bound, far below the MFMA ridge (the engine
// ran it as 4 phases of a 32-column tile with 29 idle columns, ~0.29 ms).  Exact fp32 FMA here:
//   block = (image, 64-column block u0 .. u0 + 63 of the gradient, a run of gradient rows t0): per row t0 it
//   produces output rows 2 t0, 2 t0 + 1 x columns 2 u0 .. 2 u0 + 127 from gradient rows t0 - 1 .. t0 + 1, kept in a
//   3-row LDS ring (66 columns x 64 channels; each row staged once with coalesced 16-B loads, the next one in
//   flight in registers while the current pair of output rows is computed).  Wave (py, px) computes the 64 pixels of
//   one (row, column) parity, which all use the same 2 x 2 taps: their weights are loaded into the lanes' registers
//   ONCE per block; lane = (pixel group pg, channel quad cq), a 16-lane DPP reduction per pixel; the outputs go out
//   through LDS as whole rows.
//   y[n][j][Y][X] (+)= sum_{a,b} sum_ch g[n][a][b][ch] * w[ch][c0 + j][Y + 1 - 2a][X + 1 - 2b]
constexpr int D0C = 64, D0U = 64, D0COLS = D0U + 2, D0Q = D0C / 4;
constexpr int D0LD = (D0COLS * D0Q + 255) / 256;          // 16-B loads per thread per staged row

template <int CN>
__global__ void __launch_bounds__(256) d0_input_grad_kernel(fg_view g, const float* __restrict__ w, int ctot, int c0,
                                                            float* __restrict__ y, int yc, int H, int W, int accumulate,
                                                            int ublocks, int rows_per_block) {
    __shared__ f32x4 gs[3][D0COLS][D0Q];
    __shared__ float os[CN][2][2 * D0U];
    const int Ho = H / 2, Wo = W / 2;
    const int nsplit = (Ho + rows_per_block - 1) / rows_per_block;
    const int ub = blockIdx.x % ublocks, sp = (blockIdx.x / ublocks) % nsplit, n = blockIdx.x / (ublocks * nsplit);
    const int u0 = ub * D0U, tb = sp * rows_per_block, te = min(Ho, tb + rows_per_block);
    const int tid = threadIdx.x;
    f32x4 rg[D0LD];
    auto load_row = [&](int a) {        // gradient row a (-1 .. Ho: the zero border included) into registers
#pragma unroll
        for (int k = 0; k < D0LD; ++k) {
            const int i = tid + 256 * k, col = i / D0Q, q = i - col * D0Q, b = u0 - 1 + col;
            rg[k] = (i < D0COLS * D0Q && b <= Wo && a <= Ho)
                        ? *reinterpret_cast<const f32x4*>(g.ptr + fg::vidx(g, n, a, b) + 4 * q)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store_row = [&](int a) {
        f32x4* dst = &gs[(a + 3) % 3][0][0];
#pragma unroll
        for (int k = 0; k < D0LD; ++k) {
            const int i = tid + 256 * k;
            if (i < D0COLS * D0Q) dst[i] = rg[k];
        }
    };
    const int wave = tid >> 6, lane = tid & 63, py = wave >> 1, px = wave & 1, pg = lane >> 4, cq = lane & 15;
    // output row 2 t0 (py 1): taps r = 1 (gradient row t0), 3 (t0 - 1); row 2 t0 + 1 (py 0): r = 0 (t0 + 1), 2 (t0).
    // Columns likewise with px, s and the LDS column offsets.
    const int r0 = py ? 1 : 0, r1 = r0 + 2, dr0 = py ? 0 : 1, dr1 = dr0 - 1;
    const int s0 = px ? 1 : 0, s1 = s0 + 2, lc0 = px ? 1 : 2, lc1 = lc0 - 1;
    f32x4 wt[4][CN];          // taps (r0,s0) (r0,s1) (r1,s0) (r1,s1) x outputs: this lane's 4 channels
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int r = t < 2 ? r0 : r1, sc = (t & 1) ? s1 : s0;
#pragma unroll
        for (int j = 0; j < CN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) wt[t][j][e] = w[((size_t)(4 * cq + e) * ctot + c0 + j) * 16 + r * 4 + sc];
    }
    if (tb >= te) return;
    load_row(tb - 1);
    store_row(tb - 1);
    load_row(tb);
    store_row(tb);
    load_row(tb + 1);
    for (int t0 = tb; t0 < te; ++t0) {
        store_row(t0 + 1);                       // slot (t0 + 1) % 3 = (t0 - 2) % 3, last read at t0 - 1
        __syncthreads();
        if (t0 + 1 < te) load_row(t0 + 2);       // in flight during this row pair
        const f32x4(*rw0)[D0Q] = gs[(t0 + dr0 + 3) % 3];
        const f32x4(*rw1)[D0Q] = gs[(t0 + dr1 + 3) % 3];
        for (int jj = pg; jj < D0U; jj += 4) {
            float acc[CN];
#pragma unroll
            for (int j = 0; j < CN; ++j) acc[j] = 0.f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const f32x4 v = (t < 2 ? rw0 : rw1)[jj + ((t & 1) ? lc1 : lc0)][cq];
#pragma unroll
                for (int j = 0; j < CN; ++j) {
                    acc[j] = fmaf(v[0], wt[t][j][0], acc[j]);
                    acc[j] = fmaf(v[1], wt[t][j][1], acc[j]);
                    acc[j] = fmaf(v[2], wt[t][j][2], acc[j]);
                    acc[j] = fmaf(v[3], wt[t][j][3], acc[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < CN; ++j) acc[j] = fg::row_sum16(acc[j]);
            if (cq == 0)
#pragma unroll
                for (int j = 0; j < CN; ++j) os[j][1 - py][2 * jj + 1 - px] = acc[j];
        }
        __syncthreads();
        for (int i = tid; i < CN * 2 * 2 * D0U; i += 256) {
            const int j = i / (4 * D0U), rr = (i / (2 * D0U)) & 1, xl = i & (2 * D0U - 1);
            const int Y = 2 * t0 + rr, X = 2 * u0 + xl;
            if (X >= W) continue;
            float* dst = y + (((size_t)n * yc + j) * H + Y) * W + X;
            *dst = accumulate ? *dst + os[j][rr][xl] : os[j][rr][xl];
        }
    }
}

}  // namespace

FG_API int fg_conv_n1_fwd(const float* x, int nimg, int hp, int wp, int c, const float* w, const float* bias,
                          float* y, int ho, int wo, hipStream_t stream) {
    if (!x || !w || !y || c != C || nimg < 1 || ho != hp - 3 || wo != wp - 3 || ho < 1 || wo < 1 ||
        ((uintptr_t)x & 15) || ((uintptr_t)w & 15))
        return fg::fail(FG_ERR_INVALID, "fg_conv_n1_fwd: needs a 512-channel input padded by 1, a 4x4 kernel, "
                                        "stride 1 (ho = hp - 3)");
    const long long waves = (long long)nimg * ((ho + 3) / 4) * ((wo + 3) / 4);
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

FG_API int fg_d0_input_grad(fg_view g, const float* w, int ctot, int c0, int cn, float* y, int yc, int H, int W,
                            int accumulate, hipStream_t stream) {
    if (!g.ptr || !w || !y || g.c_alloc != D0C || g.pad < 1 || (H & 1) || (W & 1) || g.h != H / 2 || g.w != W / 2 ||
        cn < 1 || cn > 4 || c0 < 0 || c0 + cn > ctot || yc < cn || ((uintptr_t)g.ptr & 15))
        return fg::fail(FG_ERR_INVALID, "fg_d0_input_grad: needs the 64-channel gradient of a 4x4 stride-2 pad-1 conv "
                                        "(zero border >= 1, H and W even) and 1..4 input channels (cn=%d)", cn);
    const int ublocks = (W / 2 + D0U - 1) / D0U, Ho = H / 2;
    // ~2 blocks per CU, each walking a run of gradient rows (its weights loaded once, each gradient row staged once)
    const int want = std::max(1, 2 * fg::num_cus() / (g.n * ublocks));
    const int rows = std::max(1, (Ho + want - 1) / want);
    const dim3 grid((unsigned)(g.n * ublocks * ((Ho + rows - 1) / rows)));
    switch (cn) {
        case 1: hipLaunchKernelGGL(d0_input_grad_kernel<1>, grid, dim3(256), 0, stream, g, w, ctot, c0, y, yc, H, W, accumulate, ublocks, rows); break;
        case 2: hipLaunchKernelGGL(d0_input_grad_kernel<2>, grid, dim3(256), 0, stream, g, w, ctot, c0, y, yc, H, W, accumulate, ublocks, rows); break;
        case 3: hipLaunchKernelGGL(d0_input_grad_kernel<3>, grid, dim3(256), 0, stream, g, w, ctot, c0, y, yc, H, W, accumulate, ublocks, rows); break;
        default: hipLaunchKernelGGL(d0_input_grad_kernel<4>, grid, dim3(256), 0, stream, g, w, ctot, c0, y, yc, H, W, accumulate, ublocks, rows); break;
    }
    return fg::launched("d0_input_grad");
}
