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

// Reductions are two-level and deterministic: the statistics kernels write one partial per (group,
// chunk of pixels) -- each block walks its chunk over every image of its group -- and the finalize
// kernels combine a group's partials with 16 threads per channel.  At most MAX_PARTIALS partials per
// buffer keep the finalize short while the statistics pass still spreads over ~4 blocks per CU.
constexpr int MAX_PARTIALS = 1024;

int choose_chunks(int groups, long long hw) {
    long long c = MAX_PARTIALS / groups;
    if (c > hw / 16) c = hw / 16;
    if (c < 1) c = 1;
    return (int)c;
}

// block (chunk, group): shifted sums of x and x^2 per channel over the chunk's pixels of every image of
// the group (fp32 within one image's chunk, fp64 across images and threads)
__global__ void bn_stats_kernel(fg_view src, int per_group, int chunks, double* __restrict__ work) {
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    const int grp = blockIdx.y, chunk = blockIdx.x;
    const int HW = src.h * src.w, per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int g = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    const int n0 = grp * per_group;
    __shared__ double red[NT][8];
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (g < PG) {
        const f32x4 K = ld4(src.ptr + fg::vidx(src, n0, 0, 0) + 4 * c4);       // the group's first pixel
        for (int n = n0; n < n0 + per_group; ++n) {
            f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = s;
            for (int p = p0 + g; p < p1; p += PG) {
                const int y = p / src.w, x = p - y * src.w;
                const f32x4 v = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - K;
                s += v;
                ss += v * v;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                a[e] += s[e];
                a[4 + e] += ss[e];
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = a[e];
    __syncthreads();
    if (threadIdx.x < L) {
        double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += red[gg * L + threadIdx.x][e];
        double* w = work + ((size_t)(grp * chunks + chunk) * C + 4 * threadIdx.x) * 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w[2 * e] = t[e];
            w[2 * e + 1] = t[4 + e];
        }
    }
}

constexpr int FIN_CH = 16, FIN_PARTS = 256 / FIN_CH;

// sum of group grp's partial pairs for channel c (FIN_PARTS threads per channel, LDS tree); valid in
// the part-0 thread
__device__ __forceinline__ void sum_partials(const double* __restrict__ work, int C, int chunks, int grp, int c,
                                             double& s1, double& s2) {
    const int cl = threadIdx.x % FIN_CH, part = threadIdx.x / FIN_CH;
    __shared__ double red[256][2];
    double a = 0, b = 0;
    if (c < C) {
#pragma unroll 8
        for (int k = part; k < chunks; k += FIN_PARTS) {
            const double* w = work + ((size_t)(grp * chunks + k) * C + c) * 2;
            a += w[0];
            b += w[1];
        }
    }
    red[threadIdx.x][0] = a;
    red[threadIdx.x][1] = b;
    __syncthreads();
    if (part == 0) {
        for (int q = 1; q < FIN_PARTS; ++q) {
            a += red[q * FIN_CH + cl][0];
            b += red[q * FIN_CH + cl][1];
        }
    }
    __syncthreads();
    s1 = a;
    s2 = b;
}

// per group: mean / invstd; running statistics in group order (block = FIN_CH channels)
__global__ void bn_finalize_kernel(fg_view src, int groups, int chunks, const double* __restrict__ work, float eps,
                                   float momentum, float* mean, float* invstd, float* running_mean,
                                   float* running_var, long long* num_batches) {
    const int C = src.c_alloc;
    const int c = blockIdx.x * FIN_CH + threadIdx.x % FIN_CH;
    const bool lead = threadIdx.x / FIN_CH == 0 && c < C;
    if (blockIdx.x == 0 && threadIdx.x == 0 && num_batches) *num_batches += groups;   // one call per group
    const int per_group = src.n / groups;
    const double M = (double)per_group * src.h * src.w;
    for (int gi = 0; gi < groups; ++gi) {
        double s1, s2;
        sum_partials(work, C, chunks, gi, c, s1, s2);
        if (!lead) continue;
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

// Dropout keep decision of NCHW element idx under `seed` (counter-based: the backward recomputes it,
// no mask is stored): splitmix64 of (seed, idx), kept when its top 32 bits fall below keep * 2^32
__device__ __forceinline__ bool dropout_keep(unsigned long long seed, unsigned long long idx, unsigned thresh) {
    unsigned long long z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (unsigned)(z >> 32) < thresh;
}

// dropout multiplier of element (n, c, y, x): mask tensor, hashed keep bit, or 1
struct Drop {
    const float* mask;
    unsigned long long seed;
    unsigned thresh;
    float scale;
    __device__ __forceinline__ float operator()(int n, int c, int C, int y, int x, int h, int w) const {
        const size_t idx = (((size_t)n * C + c) * h + y) * w + x;
        if (mask) return mask[idx] * scale;
        if (seed) return dropout_keep(seed, idx, thresh) ? scale : 0.f;
        return 1.f;
    }
    __device__ __forceinline__ bool on() const { return mask || seed; }
};

__global__ void dropout_mask_kernel(unsigned long long seed, unsigned thresh, long long total, float* dst) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = dropout_keep(seed, (unsigned long long)i, thresh) ? 1.f : 0.f;
}

__device__ __forceinline__ float act_apply(float v, int act) { return fg::act_fwd(v, act); }

// y = (x - mean) * invstd * gamma + beta  (or y = x without statistics), y *= dropout mask * scale,
// dst0 = act0(y), dst1 = act1(y) (interiors; the caller zeroes the borders)
__global__ void bn_apply_kernel(fg_view src, int per_group, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const Drop drop, int act0, fg_view d0, unsigned* am0,
                                int act1, fg_view d1, unsigned* am1) {
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
        if (drop.on()) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] * drop(n, 4 * c4 + e, C, y, x, src.h, src.w);
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
    const float *mean, *invstd, *gamma, *beta;
    Drop drop;
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
    if (I.drop.on()) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            dm[e] = I.drop(n, 4 * c4 + e, C, y, x, I.src.h, I.src.w);
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
    const int grp = blockIdx.y, chunk = blockIdx.x;
    const int HW = I.src.h * I.src.w, per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int g = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    const int n0 = grp * I.per_group;
    __shared__ double red[NT][8];
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (g < PG)
        for (int n = n0; n < n0 + I.per_group; ++n) {
            f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sgx = sg;
            for (int p = p0 + g; p < p1; p += PG) {
                const int y = p / I.src.w, x = p - y * I.src.w;
                f32x4 gy, xh;
                grad_and_xhat(I, n, y, x, c4, gy, xh);
                sg += gy;
                sgx += gy * xh;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                a[e] += sg[e];
                a[4 + e] += sgx[e];
            }
        }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = a[e];
    __syncthreads();
    if (threadIdx.x < L) {
        double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += red[gg * L + threadIdx.x][e];
        double* w = work + ((size_t)(grp * chunks + chunk) * C + 4 * threadIdx.x) * 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w[2 * e] = t[e];
            w[2 * e + 1] = t[4 + e];
        }
    }
}

// per group: the apply coefficients (mean g, mean g*xhat); gamma / beta gradients summed over the groups
__global__ void bn_bwd_finalize_kernel(int N, int C, int groups, int HW, int chunks, const double* __restrict__ work,
                                       float* coef, float* gamma_grad, float* beta_grad, int accumulate) {
    const int c = blockIdx.x * FIN_CH + threadIdx.x % FIN_CH;
    const bool lead = threadIdx.x / FIN_CH == 0 && c < C;
    const double M = (double)(N / groups) * HW;
    double tg = 0, tgx = 0;
    for (int gi = 0; gi < groups; ++gi) {
        double sg, sgx;
        sum_partials(work, C, chunks, gi, c, sg, sgx);
        if (!lead) continue;
        coef[(size_t)(gi * C + c) * 2] = (float)(sg / M);
        coef[(size_t)(gi * C + c) * 2 + 1] = (float)(sgx / M);
        tg += sg;
        tgx += sgx;
    }
    if (!lead) return;
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

Drop make_drop(const float* mask, float scale, unsigned long long seed) {
    Drop d;
    d.mask = mask;
    d.seed = mask ? 0ull : seed;
    d.scale = scale;
    const double keep = scale > 0 ? 1.0 / scale : 0.0;
    d.thresh = keep >= 1.0 ? 0xffffffffu : (unsigned)(keep * 4294967296.0);
    return d;
}

// eval mode: mean = running_mean, invstd = 1 / sqrt(running_var + eps)
__global__ void bn_eval_stats_kernel(int C, const float* rm, const float* rv, float eps, float* mean, float* invstd) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    mean[c] = rm[c];
    invstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}

}  // namespace

FG_API long long fg_bn_workspace_doubles(int n, int c) {
    return (long long)MAX_PARTIALS * c * 2 + (long long)n * c + 64;
}

FG_API int fg_bn_stats(fg_view src, int groups, float eps, float momentum, float* mean, float* invstd,
                       float* running_mean, float* running_var, long long* num_batches_tracked, double* work,
                       hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !mean || !invstd || !work || groups < 1 || src.n % groups ||
        NT % (src.c_alloc / 4) != 0 || (!running_mean) != (!running_var))
        return fg::fail(FG_ERR_INVALID, "fg_bn_stats: bad args (C=%d, groups=%d, n=%d)", src.c_alloc, groups, src.n);
    const int chunks = choose_chunks(groups, (long long)src.h * src.w);
    hipLaunchKernelGGL(bn_stats_kernel, dim3(chunks, groups), dim3(NT), 0, stream, src, src.n / groups, chunks, work);
    int e = fg::launched("bn_stats");
    if (e) return e;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((src.c_alloc + FIN_CH - 1) / FIN_CH), dim3(256), 0, stream, src, groups,
                       chunks, work, eps, momentum, mean, invstd, running_mean, running_var, num_batches_tracked);
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
                       const float* beta, const float* drop_mask, float drop_scale, unsigned long long drop_seed,
                       int act0, fg_view dst0, float* absmax0, int act1, fg_view dst1, float* absmax1,
                       hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !ok_view(dst0) || !aligned(dst0) || groups < 1 || src.n % groups ||
        (mean && !invstd) || ((!gamma) != (!beta)) || ((drop_mask || drop_seed) && !(drop_scale >= 1.f)))
        return fg::fail(FG_ERR_INVALID, "fg_bn_apply: bad args");
    for (const fg_view* d : {&dst0, &dst1}) {
        if (!d->ptr) continue;
        if (!aligned(*d) || d->n != src.n || d->h != src.h || d->w != src.w || d->c_alloc < src.c_alloc)
            return fg::fail(FG_ERR_INVALID, "fg_bn_apply: destination %dx%dx%d (c %d) vs source %dx%dx%d (c %d)", d->n,
                            d->h, d->w, d->c_alloc, src.n, src.h, src.w, src.c_alloc);
    }
    const long long total = (long long)src.n * src.h * src.w * (src.c_alloc / 4);
    hipLaunchKernelGGL(bn_apply_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src,
                       src.n / groups, mean, invstd, gamma, beta, make_drop(drop_mask, drop_scale, drop_seed), act0,
                       dst0, reinterpret_cast<unsigned*>(absmax0), act1, dst1, reinterpret_cast<unsigned*>(absmax1));
    return fg::launched("bn_apply");
}

FG_API int fg_bn_bwd(fg_view gA, int actA, fg_view gB, int actB, fg_view src, int groups, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, const float* drop_mask,
                     float drop_scale, unsigned long long drop_seed, fg_view dst, float* gamma_grad, float* beta_grad,
                     int accumulate, double* work, float* absmax, hipStream_t stream) {
    if (!ok_view(gA) || !aligned(gA) || !ok_view(src) || !aligned(src) || !ok_view(dst) || !aligned(dst) ||
        groups < 1 || src.n % groups || NT % (src.c_alloc / 4) != 0 || (mean && (!invstd || !work)) ||
        ((!gamma) != (!beta)) || ((drop_mask || drop_seed) && !(drop_scale >= 1.f)))
        return fg::fail(FG_ERR_INVALID, "fg_bn_bwd: bad args");
    for (const fg_view* v : {&gA, &gB, &dst}) {
        if (!v->ptr) continue;
        if (!aligned(*v) || v->n != src.n || v->h != src.h || v->w != src.w || v->c_alloc < src.c_alloc)
            return fg::fail(FG_ERR_INVALID, "fg_bn_bwd: view %dx%dx%d (c %d) vs source %dx%dx%d (c %d)", v->n, v->h,
                            v->w, v->c_alloc, src.n, src.h, src.w, src.c_alloc);
    }
    BwdIn I{gA, gB, src, actA, actB, src.n / groups, mean, invstd, gamma, beta,
            make_drop(drop_mask, drop_scale, drop_seed)};
    const int C = src.c_alloc;
    float* coef = nullptr;
    if (mean) {
        const int chunks = choose_chunks(groups, (long long)src.h * src.w);
        coef = reinterpret_cast<float*>(work + (size_t)MAX_PARTIALS * C * 2);
        hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(chunks, groups), dim3(NT), 0, stream, I, chunks, work);
        int e = fg::launched("bn_bwd_stats");
        if (e) return e;
        hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FIN_CH - 1) / FIN_CH), dim3(256), 0, stream, src.n, C,
                           groups, src.h * src.w, chunks, work, coef, gamma_grad, beta_grad, accumulate);
        e = fg::launched("bn_bwd_finalize");
        if (e) return e;
    }
    const long long total = (long long)src.n * src.h * src.w * (C / 4);
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, I, coef, dst,
                       reinterpret_cast<unsigned*>(absmax));
    return fg::launched("bn_bwd_apply");
}

FG_API int fg_dropout_mask(unsigned long long seed, float keep, long long total, float* dst, hipStream_t stream) {
    if (!dst || total <= 0 || !(keep > 0.f && keep <= 1.f) || !seed)
        return fg::fail(FG_ERR_INVALID, "fg_dropout_mask: bad args");
    const Drop d = make_drop(nullptr, 1.f / keep, seed);
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, seed, d.thresh,
                       total, dst);
    return fg::launched("dropout_mask");
}

FG_API int fg_maxpool2(fg_view src, fg_view dst, hipStream_t stream) {
    if (!ok_view(src) || !aligned(src) || !ok_view(dst) || !aligned(dst) || dst.c_alloc != src.c_alloc ||
        dst.n != src.n || dst.h != src.h / 2 || dst.w != src.w / 2)
        return fg::fail(FG_ERR_INVALID, "fg_maxpool2: bad args");
    const long long total = (long long)dst.n * dst.h * dst.w * (dst.c_alloc / 4);
    hipLaunchKernelGGL(maxpool2_kernel, dim3(fg::blocks_for(total, NT, 4096)), dim3(NT), 0, stream, src, dst);
    return fg::launched("maxpool2");
}
