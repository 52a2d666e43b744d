// Generator tail (models/model_architectures.py:352-399): tanh over the 27 content logits,
// softmax over the 10 attention logits, composite
//     out[c] = sum_{i<9} tanh(cl[3i+c]) * att[i]  +  input[c] * att[9]
// (summed left to right as the reference does) and last_attention_mask = att[9].
// One thread per pixel; the backward recomputes tanh / softmax from the saved logits.
#include "fg_common.hpp"

namespace {

constexpr int NCONT = 27, NATT = 10;

struct PixelVals {
    float t[NCONT];
    float a[NATT];
};

__device__ __forceinline__ void load_pixel(const fg_view& cl, const fg_view& al, int n, int y, int x, PixelVals& v) {
    // c_alloc >= 28 / >= 12 and 16-byte aligned rows (checked by the launchers): vector loads
    const f32x4* cp = reinterpret_cast<const f32x4*>(cl.ptr + fg::vidx(cl, n, y, x));
    const f32x4* ap4 = reinterpret_cast<const f32x4*>(al.ptr + fg::vidx(al, n, y, x));
    float cv[28], ap[12];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const f32x4 t = cp[q];
        cv[4 * q] = t[0]; cv[4 * q + 1] = t[1]; cv[4 * q + 2] = t[2]; cv[4 * q + 3] = t[3];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const f32x4 t = ap4[q];
        ap[4 * q] = t[0]; ap[4 * q + 1] = t[1]; ap[4 * q + 2] = t[2]; ap[4 * q + 3] = t[3];
    }
#pragma unroll
    for (int i = 0; i < NCONT; ++i) v.t[i] = tanhf(cv[i]);
    float mx = ap[0];
#pragma unroll
    for (int i = 1; i < NATT; ++i) mx = fmaxf(mx, ap[i]);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NATT; ++i) {
        v.a[i] = expf(ap[i] - mx);
        s += v.a[i];
    }
#pragma unroll
    for (int i = 0; i < NATT; ++i) v.a[i] = v.a[i] / s;
}

__global__ void tail_fwd_kernel(fg_view cl, fg_view al, fg_sview x, float* __restrict__ out,
                                float* __restrict__ mask) {
    const int H = cl.h, W = cl.w;
    const long long total = (long long)cl.n * H * W;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int xx = (int)(idx % W);
        const long long t = idx / W;
        const int yy = (int)(t % H);
        const int n = (int)(t / H);
        PixelVals v;
        load_pixel(cl, al, n, yy, xx, v);
        const long long HW = (long long)H * W;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float o = v.t[c] * v.a[0];
#pragma unroll
            for (int i = 1; i < 9; ++i) o = o + v.t[3 * i + c] * v.a[i];
            o = o + x.ptr[n * x.sn + c * x.sc + yy * x.sy + xx * x.sx] * v.a[9];
            out[(n * 3 + c) * HW + yy * W + xx] = o;
        }
        mask[n * HW + yy * W + xx] = v.a[9];
    }
}

// fold a thread's max |v| bits into shard blockIdx % FG_AMAX_SHARDS of an absmax slot (256-thread blocks)
__device__ __forceinline__ void flush_amax(unsigned m, unsigned* out, unsigned* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out + (blockIdx.x & (FG_AMAX_SHARDS - 1)), max(max(red[0], red[1]), max(red[2], red[3])));
    __syncthreads();
}

__device__ __forceinline__ unsigned abits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__global__ void __launch_bounds__(256) tail_bwd_kernel(fg_view cl, fg_view al, fg_sview x, fg_sview gout, fg_sview gmask,
                                                       fg_view gc, fg_view ga, fg_wview gx, unsigned* amax_c,
                                                       unsigned* amax_a) {
    unsigned mc = 0, ma = 0;                      // max |g_content|, |g_att| written by this thread
    // iterate over gc's padded extent so its zero border is written too
    const int H = cl.h, W = cl.w;
    const int hp = H + 2 * gc.pad, wp = W + 2 * gc.pad;
    const long long total = (long long)cl.n * hp * wp;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int xp = (int)(idx % wp);
        const long long t = idx / wp;
        const int yp = (int)(t % hp);
        const int n = (int)(t / hp);
        const int yy = yp - gc.pad, xx = xp - gc.pad;
        float* gcp = gc.ptr + ((size_t)(n * hp + yp) * wp + xp) * gc.c_alloc;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) {
            for (int i = 0; i < gc.c_alloc; i += 4) *reinterpret_cast<f32x4*>(gcp + i) = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
        }
        PixelVals v;
        load_pixel(cl, al, n, yy, xx, v);
        float g[3], xin[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            g[c] = gout.ptr[n * gout.sn + c * gout.sc + yy * gout.sy + xx * gout.sx];
            xin[c] = x.ptr[n * x.sn + c * x.sc + yy * x.sy + xx * x.sx];
        }
        float gatt[NATT];
        float go[32];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            gatt[i] = g[0] * v.t[3 * i] + g[1] * v.t[3 * i + 1] + g[2] * v.t[3 * i + 2];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float tt = v.t[3 * i + c];
                go[3 * i + c] = g[c] * v.a[i] * (1.f - tt * tt);
            }
        }
#pragma unroll
        for (int i = NCONT; i < 32; ++i) go[i] = 0.f;
#pragma unroll
        for (int i = 0; i < NCONT; ++i) mc = max(mc, abits(go[i]));
#pragma unroll
        for (int q = 0; q < 8; ++q)
            *reinterpret_cast<f32x4*>(gcp + 4 * q) = f32x4{go[4 * q], go[4 * q + 1], go[4 * q + 2], go[4 * q + 3]};
        for (int i = 32; i < gc.c_alloc; i += 4) *reinterpret_cast<f32x4*>(gcp + i) = f32x4{0.f, 0.f, 0.f, 0.f};
        gatt[9] = g[0] * xin[0] + g[1] * xin[1] + g[2] * xin[2];
        // a loss on last_attention_mask = attention10 (models/model_architectures.py:396) adds its gradient here
        if (gmask.ptr) gatt[9] += gmask.ptr[n * gmask.sn + yy * gmask.sy + xx * gmask.sx];
        if (gx.ptr) {  // d(output10)/d(input[:, :3]) = attention10 (models/model_architectures.py:393, :251)
#pragma unroll
            for (int c = 0; c < 3; ++c) gx.ptr[n * gx.sn + c * gx.sc + yy * gx.sy + xx * gx.sx] = g[c] * v.a[9];
        }
        float dot = 0.f;
#pragma unroll
        for (int i = 0; i < NATT; ++i) dot += v.a[i] * gatt[i];
        float* gap = ga.ptr + fg::vidx(ga, n, yy, xx);
        float ao[16];
#pragma unroll
        for (int i = 0; i < NATT; ++i) ao[i] = v.a[i] * (gatt[i] - dot);
#pragma unroll
        for (int i = NATT; i < 16; ++i) ao[i] = 0.f;
#pragma unroll
        for (int i = 0; i < NATT; ++i) ma = max(ma, abits(ao[i]));
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4*>(gap + 4 * q) = f32x4{ao[4 * q], ao[4 * q + 1], ao[4 * q + 2], ao[4 * q + 3]};
        for (int i = 16; i < ga.c_alloc; i += 4) *reinterpret_cast<f32x4*>(gap + i) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __shared__ unsigned red[4];
    if (amax_c) flush_amax(mc, amax_c, red);
    if (amax_a) flush_amax(ma, amax_a, red);
}

// CycleGAN head (models/model_architectures.py:115-117: conv 7x7 64->3 then nn.Tanh): one thread
// per output element, x fastest (coalesced NCHW stores).
__global__ void tanh_head_fwd_kernel(fg_view logits, int c, fg_wview out) {
    const int H = logits.h, W = logits.w;
    const long long total = (long long)logits.n * c * H * W;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int xx = (int)(idx % W);
        long long q = idx / W;
        const int yy = (int)(q % H);
        q /= H;
        const int ch = (int)(q % c);
        const int n = (int)(q / c);
        out.ptr[n * out.sn + ch * out.sc + yy * out.sy + xx * out.sx] = tanhf(logits.ptr[fg::vidx(logits, n, yy, xx) + ch]);
    }
}

// g_logits = g_out * (1 - tanh^2), written over g_logits' full padded extent (zero border and
// zero channels >= c: the 7x7 input-gradient conv reads them).  One thread per padded pixel.
__global__ void tanh_head_bwd_kernel(fg_view logits, int c, fg_sview gout, fg_view gl) {
    const int H = logits.h, W = logits.w;
    const int hp = H + 2 * gl.pad, wp = W + 2 * gl.pad;
    const long long total = (long long)logits.n * hp * wp;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int xp = (int)(idx % wp);
        const long long t = idx / wp;
        const int yp = (int)(t % hp);
        const int n = (int)(t / hp);
        const int yy = yp - gl.pad, xx = xp - gl.pad;
        float* gp = gl.ptr + ((size_t)(n * hp + yp) * wp + xp) * gl.c_alloc;
        const bool inside = yy >= 0 && yy < H && xx >= 0 && xx < W;
        for (int i = 0; i < gl.c_alloc; i += 4) {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = 0.f;
                if (inside && i + j < c) {
                    const float th = tanhf(logits.ptr[fg::vidx(logits, n, yy, xx) + i + j]);
                    v[j] = gout.ptr[n * gout.sn + (i + j) * gout.sc + yy * gout.sy + xx * gout.sx] * (1.f - th * th);
                }
            }
            *reinterpret_cast<f32x4*>(gp + i) = f32x4{v[0], v[1], v[2], v[3]};
        }
    }
}

}  // namespace

FG_API int fg_tail_fwd(fg_view content_logits, fg_view att_logits, fg_sview x, float* out, float* mask,
                       hipStream_t stream) {
    if (!content_logits.ptr || !att_logits.ptr || !x.ptr || !out || !mask || content_logits.c_alloc < 28 ||
        content_logits.c_alloc % 4 || att_logits.c_alloc < 12 || att_logits.c_alloc % 4 || att_logits.h != content_logits.h || att_logits.w != content_logits.w ||
        att_logits.n != content_logits.n)
        return fg::fail(FG_ERR_INVALID, "fg_tail_fwd: bad args");
    const long long total = (long long)content_logits.n * content_logits.h * content_logits.w;
    hipLaunchKernelGGL(tail_fwd_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream,
                       content_logits, att_logits, x, out, mask);
    return fg::launched("tail_fwd");
}

FG_API int fg_tail_bwd(fg_view content_logits, fg_view att_logits, fg_sview x, fg_sview g_out, fg_sview g_mask,
                       fg_view g_content, fg_view g_att, fg_wview g_x, float* absmax_content, float* absmax_att,
                       hipStream_t stream) {
    if (!content_logits.ptr || !att_logits.ptr || !x.ptr || !g_out.ptr || !g_content.ptr || !g_att.ptr ||
        content_logits.c_alloc < 28 || content_logits.c_alloc % 4 || att_logits.c_alloc < 12 ||
        att_logits.c_alloc % 4 || g_content.c_alloc < 32 || g_content.c_alloc % 4 || g_att.c_alloc < 16 ||
        g_att.c_alloc % 4 || g_content.h != content_logits.h ||
        g_content.w != content_logits.w || g_att.h != content_logits.h || g_att.w != content_logits.w ||
        g_att.pad != 0)
        return fg::fail(FG_ERR_INVALID, "fg_tail_bwd: bad args");
    const long long total = (long long)content_logits.n * (content_logits.h + 2 * g_content.pad) *
                            (content_logits.w + 2 * g_content.pad);
    hipLaunchKernelGGL(tail_bwd_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream,
                       content_logits, att_logits, x, g_out, g_mask, g_content, g_att, g_x,
                       reinterpret_cast<unsigned*>(absmax_content), reinterpret_cast<unsigned*>(absmax_att));
    return fg::launched("tail_bwd");
}

FG_API int fg_tanh_head_fwd(fg_view logits, int c, fg_wview out, hipStream_t stream) {
    if (!logits.ptr || !out.ptr || c <= 0 || c > logits.c_alloc) return fg::fail(FG_ERR_INVALID, "fg_tanh_head_fwd: bad args");
    const long long total = (long long)logits.n * c * logits.h * logits.w;
    if (total == 0) return 0;
    hipLaunchKernelGGL(tanh_head_fwd_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, logits, c,
                       out);
    return fg::launched("tanh_head_fwd");
}

FG_API int fg_tanh_head_bwd(fg_view logits, int c, fg_sview g_out, fg_view g_logits, hipStream_t stream) {
    if (!logits.ptr || !g_out.ptr || !g_logits.ptr || c <= 0 || c > logits.c_alloc || g_logits.c_alloc % 4 ||
        g_logits.c_alloc < c || g_logits.h != logits.h || g_logits.w != logits.w || g_logits.n != logits.n)
        return fg::fail(FG_ERR_INVALID, "fg_tanh_head_bwd: bad args");
    const long long total = (long long)logits.n * (logits.h + 2 * g_logits.pad) * (logits.w + 2 * g_logits.pad);
    if (total == 0) return 0;
    hipLaunchKernelGGL(tanh_head_bwd_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, logits, c,
                       g_out, g_logits);
    return fg::launched("tanh_head_bwd");
}
