// Evaluation metrics on the device: the reference's Model.calculate_metrics /
// ModelsGroup.compare_metrics (models/model.py:363-422, models/group.py:114-221) score generator
// outputs with torchmetrics 1.2.0 (requirements.txt:7) -- PSNR, SSIM, MS-SSIM over images in [0, 1]
// and binary confusion metrics over the flood masks of the segmentation U-Net.  Here:
//   * fg_unit_image: torch.clamp((g + 1) * 0.5, 0, 1) of a generator output, written as NCHW (the
//     metrics' operand) and as the segmentation U-Net's NHWC input in one pass;
//   * fg_ssim: per image, the mean over channels and valid 11x11 windows of the SSIM map and of the
//     contrast-sensitivity map (torchmetrics _ssim_update: gaussian sigma 1.5, k1 0.01, k2 0.03; its
//     reflect padding is cropped away again, so only windows inside the image count);
//   * fg_avg_pool2: F.avg_pool2d(x, 2) between MS-SSIM scales; fg_msssim_combine: prod relu(.)^beta;
//   * fg_sq_err_sum: the PSNR numerator;
//   * fg_mask_confusion: (sigmoid(logits) > 0.5) masks of two segmentation outputs -> tp, fp, tn, fn.
// Reductions are deterministic (per-block partials combined in a fixed order); the confusion counts are
// integer atomics.
#include "fg_common.hpp"

namespace {

constexpr int NT = 256;
constexpr int TS = 16;                 // output tile edge of the SSIM kernel
constexpr int KS = 11, KR = 5;         // gaussian window
constexpr int LT = TS + KS - 1;        // staged input tile edge (26)

__global__ void unit_image_kernel(fg_sview src, int n, int c, int h, int w, float* __restrict__ dst, fg_view buf) {
    const long long total = (long long)n * c * h * w;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(i % w);
        long long r = i / w;
        const int y = (int)(r % h);
        r /= h;
        const int ch = (int)(r % c);
        const int ni = (int)(r / c);
        const float v = src.ptr[ni * src.sn + ch * src.sc + y * src.sy + x * src.sx];
        const float u = fminf(fmaxf((v + 1.f) * 0.5f, 0.f), 1.f);
        if (dst) dst[i] = u;
        if (buf.ptr) buf.ptr[fg::vidx(buf, ni, y, x) + ch] = u;
    }
}

__device__ __forceinline__ void block_sum2(double& a, double& b) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
    }
    __shared__ double red[NT / 64][2];
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = a;
        red[threadIdx.x >> 6][1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < NT / 64; ++i) {
            a += red[i][0];
            b += red[i][1];
        }
    }
}

// grid (tiles_x, tiles_y, planes): one 16x16 tile of valid window positions of one (image, channel)
// plane; part[(plane * tiles + tile) * 2 + {0, 1}] = sums of the SSIM and contrast-sensitivity maps
__global__ void ssim_kernel(const float* __restrict__ a, const float* __restrict__ b, int h, int w,
                            const float* __restrict__ g, float c1, float c2, double* __restrict__ part) {
    __shared__ float A[LT][LT + 1], B[LT][LT + 1], G[KS];
    const int plane = blockIdx.z;
    const int Ho = h - 2 * KR, Wo = w - 2 * KR;
    const int oy0 = blockIdx.y * TS, ox0 = blockIdx.x * TS;
    const float* pa = a + (size_t)plane * h * w;
    const float* pb = b + (size_t)plane * h * w;
    if (threadIdx.x < KS) G[threadIdx.x] = g[threadIdx.x];
    for (int i = threadIdx.x; i < LT * LT; i += NT) {
        const int ly = i / LT, lx = i - ly * LT;
        const int y = min(oy0 + ly, h - 1), x = min(ox0 + lx, w - 1);
        A[ly][lx] = pa[(size_t)y * w + x];
        B[ly][lx] = pb[(size_t)y * w + x];
    }
    __syncthreads();
    const int ty = threadIdx.x / TS, tx = threadIdx.x % TS;
    double s_ssim = 0, s_cs = 0;
    if (oy0 + ty < Ho && ox0 + tx < Wo) {
        float ma = 0.f, mb = 0.f, saa = 0.f, sbb = 0.f, sab = 0.f;
        for (int i = 0; i < KS; ++i)
#pragma unroll
            for (int j = 0; j < KS; ++j) {
                const float wgt = G[i] * G[j];              // torch.matmul(gx.t(), gy): one fp32 product
                const float va = A[ty + i][tx + j], vb = B[ty + i][tx + j];
                ma += wgt * va;
                mb += wgt * vb;
                saa += wgt * (va * va);
                sbb += wgt * (vb * vb);
                sab += wgt * (va * vb);
            }
        const float ma2 = ma * ma, mb2 = mb * mb, mab = ma * mb;
        const float upper = 2.f * (sab - mab) + c2;
        const float lower = ((saa - ma2) + (sbb - mb2)) + c2;
        s_ssim = (double)(((2.f * mab + c1) * upper) / ((ma2 + mb2 + c1) * lower));
        s_cs = (double)(upper / lower);
    }
    block_sum2(s_ssim, s_cs);
    if (threadIdx.x == 0) {
        const size_t t = (size_t)plane * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
        part[t * 2] = s_ssim;
        part[t * 2 + 1] = s_cs;
    }
}

// one thread per image: mean over its c planes' tiles
__global__ void ssim_finalize_kernel(int n, int c, int tiles, double count, const double* __restrict__ part,
                                     double* out_ssim, double* out_cs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0, q = 0;
    for (size_t t = (size_t)i * c * tiles; t < (size_t)(i + 1) * c * tiles; ++t) {
        s += part[t * 2];
        q += part[t * 2 + 1];
    }
    if (out_ssim) out_ssim[i] = s / count;
    if (out_cs) out_cs[i] = q / count;
}

__global__ void avg_pool2_kernel(const float* __restrict__ src, int planes, int h, int w, float* __restrict__ dst) {
    const int ho = h / 2, wo = w / 2;
    const long long total = (long long)planes * ho * wo;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(i % wo);
        const long long r = i / wo;
        const int y = (int)(r % ho);
        const long long p = r / ho;
        const float* s = src + (size_t)p * h * w + (size_t)(2 * y) * w + 2 * x;
        dst[i] = (s[0] + s[1] + s[w] + s[w + 1]) * 0.25f;
    }
}

// per image: prod_s relu(m_s)^beta_s with m = cs at scales 0..S-2 and ssim at the last scale
__global__ void msssim_combine_kernel(int n, int scales, const double* __restrict__ cs, const double* __restrict__ ssim_last,
                                      const double* __restrict__ betas, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double p = 1.0;
    for (int s = 0; s < scales; ++s) {
        const double m = s < scales - 1 ? cs[(size_t)s * n + i] : ssim_last[i];
        p *= pow(m > 0 ? m : 0.0, betas[s]);
    }
    out[i] = p;
}

__global__ void sq_err_kernel(const float* __restrict__ a, const float* __restrict__ b, long long total,
                              double* __restrict__ part) {
    double s = 0, dummy = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const float d = a[i] - b[i];
        s += (double)(d * d);
    }
    block_sum2(s, dummy);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void sum_partials_kernel(const double* __restrict__ part, int nparts, double* out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double s = 0;
        for (int i = 0; i < nparts; ++i) s += part[i];
        out[0] = s;
    }
}

__device__ __forceinline__ bool flood(float logit) { return 1.f / (1.f + expf(-logit)) > 0.5f; }

// counts[0..3] += tp, fp, tn, fn of pred vs true masks (channel 0 of each view)
__global__ void mask_confusion_kernel(fg_view pred, fg_view truth, unsigned long long* counts) {
    const long long total = (long long)pred.n * pred.h * pred.w;
    unsigned c[4] = {0, 0, 0, 0};
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(i % pred.w);
        const long long r = i / pred.w;
        const int y = (int)(r % pred.h);
        const int ni = (int)(r / pred.h);
        const bool p = flood(pred.ptr[fg::vidx(pred, ni, y, x)]);
        const bool t = flood(truth.ptr[fg::vidx(truth, ni, y, x)]);
        c[p ? (t ? 0 : 1) : (t ? 3 : 2)] += 1;
    }
    __shared__ unsigned red[4][NT / 64];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        unsigned v = c[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += (unsigned)__shfl_xor((int)v, off);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long s = 0;
        for (int i = 0; i < NT / 64; ++i) s += red[threadIdx.x][i];
        atomicAdd(counts + threadIdx.x, s);
    }
}

}  // namespace

FG_API int fg_unit_image(fg_sview src, int n, int c, int h, int w, float* dst, fg_view buf, hipStream_t stream) {
    if (!src.ptr || n <= 0 || c <= 0 || h <= 0 || w <= 0 || (!dst && !buf.ptr) ||
        (buf.ptr && (buf.n != n || buf.h != h || buf.w != w || buf.c_alloc < c)))
        return fg::fail(FG_ERR_INVALID, "fg_unit_image: bad args");
    const long long total = (long long)n * c * h * w;
    hipLaunchKernelGGL(unit_image_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src, n, c, h, w,
                       dst, buf);
    return fg::launched("unit_image");
}

FG_API long long fg_ssim_workspace_doubles(int n, int c, int h, int w) {
    if (h <= 2 * KR || w <= 2 * KR) return 0;
    const long long tiles = (long long)((w - 2 * KR + TS - 1) / TS) * ((h - 2 * KR + TS - 1) / TS);
    return (long long)n * c * tiles * 2;
}

FG_API int fg_ssim(const float* a, const float* b, int n, int c, int h, int w, const float* gauss11, float c1, float c2,
                   double* ssim, double* cs, double* work, hipStream_t stream) {
    if (!a || !b || !gauss11 || !work || n <= 0 || c <= 0 || h <= 2 * KR || w <= 2 * KR || (!ssim && !cs))
        return fg::fail(FG_ERR_INVALID, "fg_ssim: bad args (%dx%d: an 11x11 window needs > 10 pixels)", h, w);
    const int tx = (w - 2 * KR + TS - 1) / TS, ty = (h - 2 * KR + TS - 1) / TS;
    hipLaunchKernelGGL(ssim_kernel, dim3(tx, ty, n * c), dim3(NT), 0, stream, a, b, h, w, gauss11, c1, c2, work);
    int e = fg::launched("ssim");
    if (e) return e;
    const double count = (double)c * (h - 2 * KR) * (w - 2 * KR);
    hipLaunchKernelGGL(ssim_finalize_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, n, c, tx * ty, count, work, ssim,
                       cs);
    return fg::launched("ssim_finalize");
}

FG_API int fg_avg_pool2(const float* src, int planes, int h, int w, float* dst, hipStream_t stream) {
    if (!src || !dst || planes <= 0 || h < 2 || w < 2) return fg::fail(FG_ERR_INVALID, "fg_avg_pool2: bad args");
    const long long total = (long long)planes * (h / 2) * (w / 2);
    hipLaunchKernelGGL(avg_pool2_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src, planes, h, w,
                       dst);
    return fg::launched("avg_pool2");
}

FG_API int fg_msssim_combine(int n, int scales, const double* cs, const double* ssim_last, const double* betas,
                             double* out, hipStream_t stream) {
    if (n <= 0 || scales <= 0 || !cs || !ssim_last || !betas || !out)
        return fg::fail(FG_ERR_INVALID, "fg_msssim_combine: bad args");
    hipLaunchKernelGGL(msssim_combine_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, n, scales, cs, ssim_last, betas,
                       out);
    return fg::launched("msssim_combine");
}

FG_API long long fg_sq_err_workspace_doubles(void) { return 1024; }

FG_API int fg_sq_err_sum(const float* a, const float* b, long long total, double* out, double* work,
                         hipStream_t stream) {
    if (!a || !b || !out || !work || total <= 0) return fg::fail(FG_ERR_INVALID, "fg_sq_err_sum: bad args");
    const int blocks = fg::blocks_for(total, NT, 1024);
    hipLaunchKernelGGL(sq_err_kernel, dim3(blocks), dim3(NT), 0, stream, a, b, total, work);
    int e = fg::launched("sq_err");
    if (e) return e;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, stream, work, blocks, out);
    return fg::launched("sum_partials");
}

FG_API int fg_mask_confusion(fg_view pred_logits, fg_view true_logits, unsigned long long* counts, hipStream_t stream) {
    if (!pred_logits.ptr || !true_logits.ptr || !counts || pred_logits.n != true_logits.n ||
        pred_logits.h != true_logits.h || pred_logits.w != true_logits.w)
        return fg::fail(FG_ERR_INVALID, "fg_mask_confusion: bad args");
    const long long total = (long long)pred_logits.n * pred_logits.h * pred_logits.w;
    hipLaunchKernelGGL(mask_confusion_kernel, dim3(fg::blocks_for(total, NT, 2048)), dim3(NT), 0, stream, pred_logits,
                       true_logits, counts);
    return fg::launched("mask_confusion");
}
