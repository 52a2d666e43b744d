// Losses of the paired step (models/model.py:626-644: nn.MSELoss vs constant 0/1 targets,
// nn.L1Loss x100) with their gradients, and torch.optim.Adam (models/model.py:121-122)
// as one multi-tensor kernel.  Reductions are two-stage and deterministic (fp64 partials).
#include "fg_common.hpp"

namespace {

constexpr int NT = 256;
constexpr int MAX_PARTS = 1024;

__device__ __forceinline__ double block_sum(double v, double* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    return red[0];
}

__global__ void mse_kernel(const float* __restrict__ p, long long n, float target, float gscale,
                           float* __restrict__ g, double* __restrict__ work) {
    __shared__ double red[NT];
    double acc = 0;
    const float gs = gscale * (2.f / (float)n);
    for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
        const float d = p[i] - target;
        acc += (double)d * d;
        if (g) g[i] = gs * d;
    }
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) work[blockIdx.x] = s;
}

__global__ void l1_kernel(fg_sview a, fg_sview b, int C, int H, int W, long long n, float gscale,
                          float* __restrict__ g, int accumulate, double* __restrict__ work) {
    __shared__ double red[NT];
    double acc = 0;
    const float gs = gscale / (float)n;
    for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
        const int x = (int)(i % W);
        long long t = i / W;
        const int y = (int)(t % H);
        t /= H;
        const int c = (int)(t % C);
        const int nn = (int)(t / C);
        const float d = a.ptr[nn * a.sn + c * a.sc + y * a.sy + x * a.sx] -
                        b.ptr[nn * b.sn + c * b.sc + y * b.sy + x * b.sx];
        acc += fabs((double)d);
        if (g) {
            const float sg = d > 0.f ? gs : (d < 0.f ? -gs : 0.f);
            g[i] = accumulate ? g[i] + sg : sg;
        }
    }
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) work[blockIdx.x] = s;
}

__global__ void mean_finalize(const double* __restrict__ work, int parts, long long n, float* loss, float scale) {
    __shared__ double red[NT];
    double acc = 0;
    for (int i = threadIdx.x; i < parts; i += NT) acc += work[i];
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) loss[0] = (float)(s / (double)n) * scale;
}

// ---- Adam ----
constexpr int MAXT = 24;
constexpr int ADAM_EPB = 2048;  // elements per block

struct AdamGroup {
    fg_adam_tensor t[MAXT];
    int blk_start[MAXT + 1];
    int count;
    float lr_step;      // -(lr / (1 - beta1^step))
    float bc2_sqrt;     // sqrt(1 - beta2^step)
    float one_m_b1, beta2, one_m_b2, eps;
};

__global__ void adam_kernel(const AdamGroup G) {
    int ti = 0;
    while (ti + 1 < G.count && (int)blockIdx.x >= G.blk_start[ti + 1]) ++ti;
    const fg_adam_tensor T = G.t[ti];
    const long long base = (long long)(blockIdx.x - G.blk_start[ti]) * ADAM_EPB;
    const float w = G.one_m_b1;
    const bool small_w = fabsf(w) < 0.5f;
    unsigned amax = 0;
    for (int k = threadIdx.x; k < ADAM_EPB; k += NT) {
        const long long i = base + k;
        if (i >= T.numel) break;
        const float g = T.grad[i];
        float m = T.exp_avg[i];
        // exp_avg.lerp_(grad, 1 - beta1)  (ATen lerp: small weight -> self + w*(end-self))
        m = small_w ? m + w * (g - m) : g - (g - m) * (1.f - w);
        // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
        float v = T.exp_avg_sq[i] * G.beta2;
        v = v + G.one_m_b2 * g * g;
        // denom = exp_avg_sq.sqrt() / sqrt(bias_correction2) + eps ; param.addcdiv_(m, denom, -step_size)
        const float denom = sqrtf(v) / G.bc2_sqrt + G.eps;
        const float np = T.param[i] + G.lr_step * m / denom;
        T.param[i] = np;
        T.exp_avg[i] = m;
        T.exp_avg_sq[i] = v;
        amax = max(amax, __float_as_uint(np) & 0x7fffffffu);
    }
    if (T.absmax) {     // bitwise max of |param| (uint order = float order), one shard per block
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) amax = max(amax, (unsigned)__shfl_xor((int)amax, off));
        __shared__ unsigned red[NT / 64];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < NT / 64; ++i) amax = max(amax, red[i]);
            atomicMax(reinterpret_cast<unsigned*>(T.absmax) + (blockIdx.x & (FG_AMAX_SHARDS - 1)), amax);
        }
    }
}

}  // namespace

FG_API int fg_mse_const(const float* p, long long n, float target, float gscale, float* loss, float* g,
                        double* work, hipStream_t stream) {
    if (!p || !loss || !work || n < 1) return fg::fail(FG_ERR_INVALID, "fg_mse_const: bad args");
    const int parts = fg::blocks_for(n, NT * 4, MAX_PARTS);
    hipLaunchKernelGGL(mse_kernel, dim3(parts), dim3(NT), 0, stream, p, n, target, gscale, g, work);
    int e = fg::launched("mse");
    if (e) return e;
    hipLaunchKernelGGL(mean_finalize, dim3(1), dim3(NT), 0, stream, work, parts, n, loss, 1.f);
    return fg::launched("mse_finalize");
}

FG_API int fg_l1(fg_sview a, fg_sview b, int N, int C, int H, int W, float gscale, float loss_scale, float* loss,
                 float* g, int accumulate, double* work, hipStream_t stream) {
    if (!a.ptr || !b.ptr || !loss || !work || N < 1 || C < 1 || H < 1 || W < 1)
        return fg::fail(FG_ERR_INVALID, "fg_l1: bad args");
    const long long n = (long long)N * C * H * W;
    const int parts = fg::blocks_for(n, NT * 4, MAX_PARTS);
    hipLaunchKernelGGL(l1_kernel, dim3(parts), dim3(NT), 0, stream, a, b, C, H, W, n, gscale, g, accumulate, work);
    int e = fg::launched("l1");
    if (e) return e;
    hipLaunchKernelGGL(mean_finalize, dim3(1), dim3(NT), 0, stream, work, parts, n, loss, loss_scale);
    return fg::launched("l1_finalize");
}

FG_API int fg_adam_step(const fg_adam_tensor* tensors, int count, double lr, double beta1, double beta2,
                        double eps, long long step, hipStream_t stream) {
    if (!tensors || count < 0 || step < 1) return fg::fail(FG_ERR_INVALID, "fg_adam_step: bad args");
    // scalar math in double exactly as torch.optim.Adam (_single_tensor_adam) does on the host
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    AdamGroup G;
    G.lr_step = (float)(-(lr / bc1));
    G.bc2_sqrt = (float)sqrt(bc2);
    G.one_m_b1 = (float)(1.0 - beta1);
    G.beta2 = (float)beta2;
    G.one_m_b2 = (float)(1.0 - beta2);
    G.eps = (float)eps;
    for (int s = 0; s < count; s += MAXT) {
        const int c = count - s < MAXT ? count - s : MAXT;
        int blocks = 0;
        G.count = c;
        for (int i = 0; i < c; ++i) {
            const fg_adam_tensor& t = tensors[s + i];
            if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || t.numel < 0)
                return fg::fail(FG_ERR_INVALID, "fg_adam_step: bad tensor %d", s + i);
            G.t[i] = t;
            G.blk_start[i] = blocks;
            blocks += (int)((t.numel + ADAM_EPB - 1) / ADAM_EPB);
        }
        for (int i = c; i <= MAXT; ++i) G.blk_start[i] = blocks;
        if (blocks == 0) continue;
        hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(NT), 0, stream, G);
        int e = fg::launched("adam");
        if (e) return e;
    }
    return 0;
}
