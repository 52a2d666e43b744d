// nn.BatchNorm2d in training mode (batch statistics, running-stat update; momentum 0.1, eps 1e-5) fused
// with what surrounds it in the Pix2Pix U-Net / PatchGAN (models/model_architectures.py:9-85) and the
// segmentation U-Net (:508-587): LeakyReLU(0.2) / ReLU on the normalised output, Dropout(0.5) with a
// caller-drawn mask, and up to two differently activated copies written into (channel slices of)
// NHWC buffers -- the U-Net's torch.cat([x, model(x)], 1) skips are channel slices of one buffer.
//
// `groups`: the images of one buffer may belong to several separate BatchNorm calls (the reference's
// D(fake) and D(real) of one training step, models/model.py:624-628, run here as one 2N pass):
// statistics are per group of N/groups consecutive images, and the running statistics are updated once
// per group, in group order, exactly as the sequential calls would.
//
// Statistics: per-(image, chunk) shifted sums (shift = the group's first pixel of the channel) in fp32
// per thread, fp64 across threads / chunks / images.  Backward: the standard batch-norm adjoint over the
// group, dL/dx = gamma * invstd * (g - mean(g) - xhat * mean(g xhat)), with g assembled from up to two
// incoming gradients through their activations and the dropout mask.
#include "fg_common.hpp"

namespace {

constexpr int NT = 256;
constexpr int MAX_CHUNKS = 128;

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

__device__ __forceinline__ void absmax_flush(unsigned m, unsigned* out) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    __shared__ unsigned red[NT / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned r = red[0];
        for (int i = 1; i < NT / 64; ++i) r = max(r, red[i]);
        atomicMax(out + (blockIdx.x & (FG_AMAX_SHARDS - 1)), r);
    }
}
__device__ __forceinline__ unsigned absbits4(const f32x4& v) {
    return max(max(__float_as_uint(v[0]) & 0x7fffffffu, __float_as_uint(v[1]) & 0x7fffffffu),
               max(__float_as_uint(v[2]) & 0x7fffffffu, __float_as_uint(v[3]) & 0x7fffffffu));
}

int choose_chunks(int n, long long hw) {
    long long c = (2048 + n - 1) / n;
    if (c > hw / 16) c = hw / 16;
    if (c > MAX_CHUNKS) c = MAX_CHUNKS;
    if (c < 1) c = 1;
    return (int)c;
}

// block (chunk, image): shifted sums of x (and x^2) per channel over the chunk's pixels
__global__ void bn_stats_kernel(fg_view src, int per_group, int chunks, double* __restrict__ work) {
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int HW = src.h * src.w, per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int g = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    __shared__ double red[NT][8];
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = s;
    if (g < PG) {
        const int n0 = (n / per_group) * per_group;                 // the group's first image
        const f32x4 K = ld4(src.ptr + fg::vidx(src, n0, 0, 0) + 4 * c4);
        for (int p = p0 + g; p < p1; p += PG) {
            const int y = p / src.w, x = p - y * src.w;
            const f32x4 v = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - K;
            s += v;
            ss += v * v;
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[threadIdx.x][e] = s[e];
        red[threadIdx.x][4 + e] = ss[e];
    }
    __syncthreads();
    if (threadIdx.x < L) {
        double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += red[gg * L + threadIdx.x][e];
        double* w = work + ((size_t)(n * chunks + chunk) * C + 4 * threadIdx.x) * 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w[2 * e] = a[e];
            w[2 * e + 1] = a[4 + e];
        }
    }
}

// one thread per channel: per group, combine its images' chunk sums; running stats in group order
__global__ void bn_finalize_kernel(fg_view src, int groups, int chunks, const double* __restrict__ work, float eps,
                                   float momentum, float* mean, float* invstd, float* running_mean,
                                   float* running_var, long long* num_batches) {
    const int C = src.c_alloc;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (c == 0 && num_batches) *num_batches += groups;      // one BatchNorm call per group
    const int per_group = src.n / groups;
    const double M = (double)per_group * src.h * src.w;
    for (int gi = 0; gi < groups; ++gi) {
        double s1 = 0, s2 = 0;
        for (int n = gi * per_group; n < (gi + 1) * per_group; ++n)
            for (int k = 0; k < chunks; ++k) {
                s1 += work[((size_t)(n * chunks + k) * C + c) * 2];
                s2 += work[((size_t)(n * chunks + k) * C + c) * 2 + 1];
            }
        const double ms = s1 / M;
        double var = s2 / M - ms * ms;
        if (var < 0) var = 0;
        const double K = src.ptr[fg::vidx(src, gi * per_group, 0, 0) + c];
        mean[gi * C + c] = (float)(K + ms);
        invstd[gi * C + c] = (float)(1.0 / sqrt(var + (double)eps));
        if (running_mean) {
            // torch: running = (1 - momentum) * running + momentum * batch (unbiased variance)
            const double unb = M > 1 ? var * M / (M - 1) : var;
            running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * (K + ms));
            running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
        }
    }
}

__device__ __forceinline__ float act_apply(float v, int act) { return fg::act_fwd(v, act); }

// y = (x - mean) * invstd * gamma + beta  (or y = x without statistics), y *= dropout mask * scale,
// dst0 = act0(y), dst1 = act1(y) (interiors; the caller zeroes the borders)
__global__ void bn_apply_kernel(fg_view src, int per_group, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ mask, float mscale, int act0,
                                fg_view d0, unsigned* am0, int act1, fg_view d1, unsigned* am1) {
    const int C = src.c_alloc, C4 = C / 4;
    const long long total = (long long)src.n * src.h * src.w * C4;
    unsigned m0 = 0, m1 = 0;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4);
        long long pix = idx / C4;
        const int x = (int)(pix % src.w);
        pix /= src.w;
        const int y = (int)(pix % src.h);
        const int n = (int)(pix / src.h);
        f32x4 v = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4);
        if (mean) {
            const int gc = (n / per_group) * C + 4 * c4;
            v = (v - ld4(mean + gc)) * ld4(invstd + gc);
            if (gamma) v = v * ld4(gamma + 4 * c4) + ld4(beta + 4 * c4);
        }
        if (mask) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                v[e] = v[e] * (mask[(((size_t)n * C + 4 * c4 + e) * src.h + y) * src.w + x] * mscale);
        }
        f32x4 o0;
#pragma unroll
        for (int e = 0; e < 4; ++e) o0[e] = act_apply(v[e], act0);
        *reinterpret_cast<f32x4*>(d0.ptr + fg::vidx(d0, n, y, x) + 4 * c4) = o0;
        m0 = max(m0, absbits4(o0));
        if (d1.ptr) {
            f32x4 o1;
#pragma unroll
            for (int e = 0; e < 4; ++e) o1[e] = act_apply(v[e], act1);
            *reinterpret_cast<f32x4*>(d1.ptr + fg::vidx(d1, n, y, x) + 4 * c4) = o1;
            m1 = max(m1, absbits4(o1));
        }
    }
    if (am0) absmax_flush(m0, am0);
    if (am1) absmax_flush(m1, am1);
}

// the incoming gradient of the normalised (and dropped-out) value: gA * actA'(u) + gB * actB'(u), then
// through the dropout (u = y * mask * scale); u's sign decides both activation derivatives
struct BwdIn {
    fg_view gA, gB, src;
    int actA, actB, per_group;
    const float *mean, *invstd, *gamma, *beta, *mask;
    float mscale;
};

__device__ __forceinline__ void grad_and_xhat(const BwdIn& I, int n, int y, int x, int c4, f32x4& gy, f32x4& xh) {
    const int C = I.src.c_alloc;
    f32x4 v = ld4(I.src.ptr + fg::vidx(I.src, n, y, x) + 4 * c4);
    xh = v;
    f32x4 u = v;
    if (I.mean) {
        const int gc = (n / I.per_group) * C + 4 * c4;
        xh = (v - ld4(I.mean + gc)) * ld4(I.invstd + gc);
        u = I.gamma ? xh * ld4(I.gamma + 4 * c4) + ld4(I.beta + 4 * c4) : xh;
    }
    f32x4 dm = {1.f, 1.f, 1.f, 1.f};
    if (I.mask) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            dm[e] = I.mask[(((size_t)n * C + 4 * c4 + e) * I.src.h + y) * I.src.w + x] * I.mscale;
            u[e] *= dm[e];
        }
    }
    const f32x4 a = ld4(I.gA.ptr + fg::vidx(I.gA, n, y, x) + 4 * c4);
#pragma unroll
    for (int e = 0; e < 4; ++e) gy[e] = a[e] * fg::act_grad(u[e], I.actA);
    if (I.gB.ptr) {
        const f32x4 b = ld4(I.gB.ptr + fg::vidx(I.gB, n, y, x) + 4 * c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) gy[e] += b[e] * fg::act_grad(u[e], I.actB);
    }
    gy = gy * dm;
}

__global__ void bn_bwd_stats_kernel(const BwdIn I, int chunks, double* __restrict__ work) {
    const int C = I.src.c_alloc, L = C / 4, PG = NT / L;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int HW = I.src.h * I.src.w, per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int g = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    __shared__ double red[NT][8];
    f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sgx = sg;
    if (g < PG)
        for (int p = p0 + g; p < p1; p += PG) {
            const int y = p / I.src.w, x = p - y * I.src.w;
            f32x4 gy, xh;
            grad_and_xhat(I, n, y, x, c4, gy, xh);
            sg += gy;
            sgx += gy * xh;
        }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[threadIdx.x][e] = sg[e];
        red[threadIdx.x][4 + e] = sgx[e];
    }
    __syncthreads();
    if (threadIdx.x < L) {
        double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += red[gg * L + threadIdx.x][e];
        double* w = work + ((size_t)(n * chunks + chunk) * C + 4 * threadIdx.x) * 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w[2 * e] = a[e];
            w[2 * e + 1] = a[4 + e];
        }
    }
}

// one thread per channel: per group sums -> apply coefficients; gamma / beta gradients summed over groups
__global__ void bn_bwd_finalize_kernel(int N, int C, int groups, int HW, int chunks, const double* __restrict__ work,
                                       float* coef, float* gamma_grad, float* beta_grad, int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int per_group = N / groups;
    const double M = (double)per_group * HW;
    double tg = 0, tgx = 0;
    for (int gi = 0; gi < groups; ++gi) {
        double sg = 0, sgx = 0;
        for (int n = gi * per_group; n < (gi + 1) * per_group; ++n)
            for (int k = 0; k < chunks; ++k) {
                sg += work[((size_t)(n * chunks + k) * C + c) * 2];
                sgx += work[((size_t)(n * chunks + k) * C + c) * 2 + 1];
            }
        coef[(size_t)(gi * C + c) * 2] = (float)(sg / M);
        coef[(size_t)(gi * C + c) * 2 + 1] = (float)(sgx / M);
        tg += sg;
        tgx += sgx;
    }
    if (beta_grad) beta_grad[c] = accumulate ? beta_grad[c] + (float)tg : (float)tg;
    if (gamma_grad) gamma_grad[c] = accumulate ? gamma_grad[c] + (float)tgx : (float)tgx;
}

__global__ void bn_bwd_apply_kernel(const BwdIn I, const float* __restrict__ coef, fg_view dst, unsigned* am) {
    const int C = I.src.c_alloc, C4 = C / 4;
    const long long total = (long long)I.src.n * I.src.h * I.src.w * C4;
    unsigned m = 0;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4);
        long long pix = idx / C4;
        const int x = (int)(pix % I.src.w);
        pix /= I.src.w;
        const int y = (int)(pix % I.src.h);
        const int n = (int)(pix / I.src.h);
        f32x4 gy, xh;
        grad_and_xhat(I, n, y, x, c4, gy, xh);
        f32x4 o = gy;
        if (I.mean) {
            const int gc = (n / I.per_group) * C + 4 * c4;
            const f32x4 is = ld4(I.invstd + gc);
            const f32x4 gam = I.gamma ? ld4(I.gamma + 4 * c4) : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = gam[e] * is[e] * (gy[e] - coef[(size_t)(gc + e) * 2] - xh[e] * coef[(size_t)(gc + e) * 2 + 1]);
        }
        *reinterpret_cast<f32x4*>(dst.ptr + fg::vidx(dst, n, y, x) + 4 * c4) = o;
        m = max(m, absbits4(o));
    }
    if (am) absmax_flush(m, am);
}

// 2x2 / stride-2 max pool (nn.MaxPool2d(2), models/model_architectures.py:558-560): floor sizes
__global__ void maxpool2_kernel(fg_view src, fg_view dst) {
    const int C = src.c_alloc, C4 = C / 4;
    const long long total = (long long)dst.n * dst.h * dst.w * C4;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4);
        long long pix = idx / C4;
        const int x = (int)(pix % dst.w);
        pix /= dst.w;
        const int y = (int)(pix % dst.h);
        const int n = (int)(pix / dst.h);
        const f32x4 a = ld4(src.ptr + fg::vidx(src, n, 2 * y, 2 * x) + 4 * c4);
        const f32x4 b = ld4(src.ptr + fg::vidx(src, n, 2 * y, 2 * x + 1) + 4 * c4);
        const f32x4 c = ld4(src.ptr + fg::vidx(src, n, 2 * y + 1, 2 * x) + 4 * c4);
        const f32x4 d = ld4(src.ptr + fg::vidx(src, n, 2 * y + 1, 2 * x + 1) + 4 * c4);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = fmaxf(fmaxf(a[e], b[e]), fmaxf(c[e], d[e]));
        *reinterpret_cast<f32x4*>(dst.ptr + fg::vidx(dst, n, y, x) + 4 * c4) = o;
    }
}

bool ok_view(const fg_view& v) { return v.ptr && v.n > 0 && v.h > 0 && v.w > 0 && v.c_alloc > 0 && v.pad >= 0; }
bool aligned(const fg_view& v) { return ((uintptr_t)v.ptr & 15) == 0 && v.c_alloc % 4 == 0; }

}  // namespace

FG_API long long fg_bn_workspace_doubles(int n, int c) { return (long long)n * c * MAX_CHUNKS * 2 + (long long)n * c + 64; }

// eval mode: mean = running_mean, invstd = 1 / sqrt(running_var + eps)
__global__ void bn_eval_stats_kernel(int C, const float* rm, const float* rv, float eps, float* mean, float* invstd) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    mean[c] = rm[c];
    invstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}

FG_API int fg_bn_stats(fg_view src, int groups, float eps, float momentum, float* mean, float* invstd,
                       float* running_mean, float* running_var, long long* num_batches_tracked, double* work,
                       hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !mean || !invstd || !work || groups < 1 || src.n % groups ||
        NT % (src.c_alloc / 4) != 0 || (!running_mean) != (!running_var))
        return fg::fail(FG_ERR_INVALID, "fg_bn_stats: bad args (C=%d, groups=%d, n=%d)", src.c_alloc, groups, src.n);
    const int chunks = choose_chunks(src.n, (long long)src.h * src.w);
    hipLaunchKernelGGL(bn_stats_kernel, dim3(chunks, src.n), dim3(NT), 0, stream, src, src.n / groups, chunks, work);
    int e = fg::launched("bn_stats");
    if (e) return e;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((src.c_alloc + 63) / 64), dim3(64), 0, stream, src, groups, chunks,
                       work, eps, momentum, mean, invstd, running_mean, running_var, num_batches_tracked);
    return fg::launched("bn_finalize");
}

FG_API int fg_bn_eval_stats(int c, const float* running_mean, const float* running_var, float eps, float* mean,
                            float* invstd, hipStream_t stream) {
    if (c <= 0 || !running_mean || !running_var || !mean || !invstd)
        return fg::fail(FG_ERR_INVALID, "fg_bn_eval_stats: bad args");
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((c + 255) / 256), dim3(256), 0, stream, c, running_mean, running_var,
                       eps, mean, invstd);
    return fg::launched("bn_eval_stats");
}

FG_API int fg_bn_apply(fg_view src, int groups, const float* mean, const float* invstd, const float* gamma,
                       const float* beta, const float* drop_mask, float drop_scale, int act0, fg_view dst0,
                       float* absmax0, int act1, fg_view dst1, float* absmax1, hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !ok_view(dst0) || !aligned(dst0) || groups < 1 || src.n % groups ||
        (mean && !invstd) || ((!gamma) != (!beta)))
        return fg::fail(FG_ERR_INVALID, "fg_bn_apply: bad args");
    for (const fg_view* d : {&dst0, &dst1}) {
        if (!d->ptr) continue;
        if (!aligned(*d) || d->n != src.n || d->h != src.h || d->w != src.w || d->c_alloc < src.c_alloc)
            return fg::fail(FG_ERR_INVALID, "fg_bn_apply: destination %dx%dx%d (c %d) vs source %dx%dx%d (c %d)", d->n,
                            d->h, d->w, d->c_alloc, src.n, src.h, src.w, src.c_alloc);
    }
    const long long total = (long long)src.n * src.h * src.w * (src.c_alloc / 4);
    hipLaunchKernelGGL(bn_apply_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src,
                       src.n / groups, mean, invstd, gamma, beta, drop_mask, drop_scale, act0, dst0,
                       reinterpret_cast<unsigned*>(absmax0), act1, dst1, reinterpret_cast<unsigned*>(absmax1));
    return fg::launched("bn_apply");
}

FG_API int fg_bn_bwd(fg_view gA, int actA, fg_view gB, int actB, fg_view src, int groups, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, const float* drop_mask,
                     float drop_scale, fg_view dst, float* gamma_grad, float* beta_grad, int accumulate,
                     double* work, float* absmax, hipStream_t stream) {
    if (!ok_view(gA) || !aligned(gA) || !ok_view(src) || !aligned(src) || !ok_view(dst) || !aligned(dst) ||
        groups < 1 || src.n % groups || NT % (src.c_alloc / 4) != 0 || (mean && (!invstd || !work)) ||
        ((!gamma) != (!beta)))
        return fg::fail(FG_ERR_INVALID, "fg_bn_bwd: bad args");
    for (const fg_view* v : {&gA, &gB, &dst}) {
        if (!v->ptr) continue;
        if (!aligned(*v) || v->n != src.n || v->h != src.h || v->w != src.w || v->c_alloc < src.c_alloc)
            return fg::fail(FG_ERR_INVALID, "fg_bn_bwd: view %dx%dx%d (c %d) vs source %dx%dx%d (c %d)", v->n, v->h,
                            v->w, v->c_alloc, src.n, src.h, src.w, src.c_alloc);
    }
    BwdIn I{gA, gB, src, actA, actB, src.n / groups, mean, invstd, gamma, beta, drop_mask, drop_scale};
    const int C = src.c_alloc;
    float* coef = nullptr;
    if (mean) {
        const int chunks = choose_chunks(src.n, (long long)src.h * src.w);
        coef = reinterpret_cast<float*>(work + (size_t)src.n * C * MAX_CHUNKS * 2);
        hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(chunks, src.n), dim3(NT), 0, stream, I, chunks, work);
        int e = fg::launched("bn_bwd_stats");
        if (e) return e;
        hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, stream, src.n, C, groups,
                           src.h * src.w, chunks, work, coef, gamma_grad, beta_grad, accumulate);
        e = fg::launched("bn_bwd_finalize");
        if (e) return e;
    }
    const long long total = (long long)src.n * src.h * src.w * (C / 4);
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, I, coef, dst,
                       reinterpret_cast<unsigned*>(absmax));
    return fg::launched("bn_bwd_apply");
}

FG_API int fg_maxpool2(fg_view src, fg_view dst, hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !ok_view(dst) || !aligned(dst) || dst.c_alloc != src.c_alloc ||
        dst.n != src.n || dst.h != src.h / 2 || dst.w != src.w / 2)
        return fg::fail(FG_ERR_INVALID, "fg_maxpool2: bad args");
    const long long total = (long long)dst.n * dst.h * dst.w * (dst.c_alloc / 4);
    hipLaunchKernelGGL(maxpool2_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src, dst);
    return fg::launched("maxpool2");
}
