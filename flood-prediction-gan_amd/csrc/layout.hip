// Layout kernels: NCHW(any strides) -> padded NHWC packing (F.pad + torch.cat), border
// zeroing, and the adjoint of reflect padding (reflection_pad2d_backward) fused with the
// residual-gradient add of PairedAttentionBlock (models/model_architectures.py:412-418).
#include "fg_common.hpp"

namespace {

// fold this thread's max |v| bits into shard blockIdx % FG_AMAX_SHARDS of an absmax slot (256-thread
// blocks; every thread of the block must call it)
__device__ __forceinline__ void flush_amax(unsigned m, unsigned* out, int bid) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    __shared__ unsigned red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out + (bid & (FG_AMAX_SHARDS - 1)), max(max(red[0], red[1]), max(red[2], red[3])));
}

__global__ void pack_input_kernel(fg_sview a, int ca, fg_sview b, int cb, fg_view dst, int img0, int nimg,
                                  int pad_mode, unsigned* amax) {
    unsigned am = 0;
    const int hp = dst.h + 2 * dst.pad, wp = dst.w + 2 * dst.pad, C = dst.c_alloc;
    const long long total = (long long)nimg * hp * wp * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(idx % C);
        long long pix = idx / C;
        const int xp = (int)(pix % wp);
        pix /= wp;
        const int yp = (int)(pix % hp);
        const int n = (int)(pix / hp);
        int y = yp - dst.pad, x = xp - dst.pad;
        float v = 0.f;
        const bool inside = y >= 0 && y < dst.h && x >= 0 && x < dst.w;
        if (inside || pad_mode == FG_PAD_REFLECT) {
            y = fg::reflect_idx(y, dst.h);
            x = fg::reflect_idx(x, dst.w);
            if (c < ca)
                v = a.ptr[n * a.sn + c * a.sc + y * a.sy + x * a.sx];
            else if (c < ca + cb)
                v = b.ptr[n * b.sn + (c - ca) * b.sc + y * b.sy + x * b.sx];
        }
        am = max(am, __float_as_uint(v) & 0x7fffffffu);
        dst.ptr[(((size_t)(img0 + n) * hp + yp) * wp + xp) * C + c] = v;
    }
    if (amax) flush_amax(am, amax, blockIdx.x);
}

// the same packing, one thread per destination pixel for narrow buffers (C <= 16: the generator and
// discriminator inputs): per-pixel reflect indices once, NCHW reads coalesced over x, float4 stores when C % 4 == 0
// (the element-per-thread form above spent 71-112 us per 75-100 MB pack on index arithmetic)
__global__ void __launch_bounds__(256) pack_input_pix_kernel(fg_sview a, int ca, fg_sview b, int cb, fg_view dst,
                                                             int img0, int pad_mode, unsigned* amax) {
    const int hp = dst.h + 2 * dst.pad, wp = dst.w + 2 * dst.pad, C = dst.c_alloc;
    const int xp = blockIdx.x * 256 + threadIdx.x, yp = blockIdx.y, n = blockIdx.z;
    unsigned am = 0;
    if (xp < wp) {
    int y = yp - dst.pad, x = xp - dst.pad;
    const bool inside = y >= 0 && y < dst.h && x >= 0 && x < dst.w;
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = 0.f;
    if (inside || pad_mode == FG_PAD_REFLECT) {
        y = fg::reflect_idx(y, dst.h);
        x = fg::reflect_idx(x, dst.w);
        const float* ap = a.ptr + n * a.sn + y * a.sy + x * a.sx;
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (c < ca) v[c] = ap[c * a.sc];
        if (cb > 0) {
            const float* bp = b.ptr + n * b.sn + y * b.sy + x * b.sx;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                if (c >= ca && c < ca + cb) v[c] = bp[(c - ca) * b.sc];
        }
    }
    float* o = dst.ptr + (((size_t)(img0 + n) * hp + yp) * wp + xp) * C;
#pragma unroll
    for (int c = 0; c < 16; ++c) am = max(am, __float_as_uint(v[c]) & 0x7fffffffu);
    if ((C & 3) == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * q < C) *reinterpret_cast<f32x4*>(o + 4 * q) = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    } else {
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (c < C) o[c] = v[c];
    }
    }
    if (amax) flush_amax(am, amax, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
}

__global__ void zero_border_kernel(fg_view dst) {
    const int p = dst.pad, hp = dst.h + 2 * p, wp = dst.w + 2 * p, C = dst.c_alloc;
    const long long per_img = 2LL * p * wp + 2LL * p * dst.h;
    const long long total = (long long)dst.n * per_img * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(idx % C);
        long long q = idx / C;
        const int n = (int)(q / per_img);
        long long r = q - (long long)n * per_img;
        int yp, xp;
        if (r < 2LL * p * wp) {  // full rows at top and bottom
            const int row = (int)(r / wp);
            xp = (int)(r - (long long)row * wp);
            yp = row < p ? row : dst.h + row;  // rows p.. -> h+p..
        } else {
            r -= 2LL * p * wp;
            const int row = (int)(r / (2 * p));
            const int col = (int)(r - (long long)row * 2 * p);
            yp = p + row;
            xp = col < p ? col : dst.w + col;
        }
        dst.ptr[(((size_t)n * hp + yp) * wp + xp) * C + c] = 0.f;
    }
}

// sum of the reflect-padding pre-images of interior index y (padded extent h + 2p)
__device__ __forceinline__ int fold_src(int y, int h, int p, int* out) {
    int k = 0;
    out[k++] = y + p;
    if (y >= 1 && y <= p) out[k++] = p - y;
    if (y >= h - 1 - p && y <= h - 2) out[k++] = p + 2 * (h - 1) - y;
    return k;
}

__global__ void fold_add_kernel(fg_view g, int fp, fg_view add, fg_view dst) {
    // g: interior (h + 2fp) x (w + 2fp); dst/add: interior h x w; all c_alloc equal, multiple of 4
    const int h = dst.h, w = dst.w, C4 = dst.c_alloc / 4;
    const int hp = h + 2 * dst.pad, wp = w + 2 * dst.pad;
    const long long total = (long long)dst.n * hp * wp * C4;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4);
        long long pix = idx / C4;
        const int xp = (int)(pix % wp);
        pix /= wp;
        const int yp = (int)(pix % hp);
        const int n = (int)(pix / hp);
        const int y = yp - dst.pad, x = xp - dst.pad;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (y >= 0 && y < h && x >= 0 && x < w) {
            int ys[3], xs[3];
            const int ny = fp > 0 ? fold_src(y, h, fp, ys) : (ys[0] = y, 1);
            const int nx = fp > 0 ? fold_src(x, w, fp, xs) : (xs[0] = x, 1);
            for (int iy = 0; iy < ny; ++iy)
                for (int ix = 0; ix < nx; ++ix)
                    v += *reinterpret_cast<const f32x4*>(g.ptr + fg::vidx(g, n, ys[iy], xs[ix]) + 4 * c4);
            if (add.ptr) v += *reinterpret_cast<const f32x4*>(add.ptr + fg::vidx(add, n, y, x) + 4 * c4);
        }
        *reinterpret_cast<f32x4*>(dst.ptr + ((size_t)(n * hp + yp) * wp + xp) * dst.c_alloc + 4 * c4) = v;
    }
}

// One thread per (n, ch, y, x) of the NCHW destination, x fastest (coalesced stores; the
// 9-channel NHWC source rows are read at a 36-byte pixel stride, all within a few lines).
__global__ void unfold_nchw_kernel(fg_view g, int fp, int c, fg_wview dst, int h, int w, int acc) {
    const long long total = (long long)g.n * c * h * w;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(idx % w);
        long long q = idx / w;
        const int y = (int)(q % h);
        q /= h;
        const int ch = (int)(q % c);
        const int n = (int)(q / c);
        int ys[3], xs[3];
        const int ny = fp > 0 ? fold_src(y, h, fp, ys) : (ys[0] = y, 1);
        const int nx = fp > 0 ? fold_src(x, w, fp, xs) : (xs[0] = x, 1);
        float v = 0.f;
        for (int iy = 0; iy < ny; ++iy)
            for (int ix = 0; ix < nx; ++ix) v += g.ptr[fg::vidx(g, n, ys[iy], xs[ix]) + ch];
        float* d = dst.ptr + n * dst.sn + ch * dst.sc + y * dst.sy + x * dst.sx;
        *d = ch < acc ? *d + v : v;
    }
}

}  // namespace

FG_API int fg_pack_input(fg_sview a, int ca, fg_sview b, int cb, fg_view dst, int img0, int nimg, int pad_mode,
                         float* absmax, hipStream_t stream) {
    unsigned* am = reinterpret_cast<unsigned*>(absmax);
    if (!a.ptr || !dst.ptr || ca < 0 || cb < 0 || (cb > 0 && !b.ptr) || ca + cb > dst.c_alloc || img0 < 0 ||
        nimg < 0 || img0 + nimg > dst.n)
        return fg::fail(FG_ERR_INVALID, "fg_pack_input: bad args");
    if (pad_mode == FG_PAD_REFLECT && (dst.pad >= dst.h || dst.pad >= dst.w))
        return fg::fail(FG_ERR_INVALID, "fg_pack_input: reflect pad %d too large for %dx%d", dst.pad, dst.h, dst.w);
    const long long total = (long long)nimg * (dst.h + 2 * dst.pad) * (dst.w + 2 * dst.pad) * dst.c_alloc;
    if (total == 0) return 0;
    if (dst.c_alloc <= 16 && ((uintptr_t)dst.ptr & 15) == 0 && nimg <= 65535 && dst.h + 2 * dst.pad <= 65535) {
        const int wp = dst.w + 2 * dst.pad;
        hipLaunchKernelGGL(pack_input_pix_kernel, dim3((wp + 255) / 256, dst.h + 2 * dst.pad, nimg), dim3(256), 0,
                           stream, a, ca, b, cb, dst, img0, pad_mode, am);
        return fg::launched("pack_input_pix");
    }
    hipLaunchKernelGGL(pack_input_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, a, ca, b,
                       cb, dst, img0, nimg, pad_mode, am);
    return fg::launched("pack_input");
}

FG_API int fg_zero_border(fg_view dst, hipStream_t stream) {
    if (!dst.ptr) return fg::fail(FG_ERR_INVALID, "fg_zero_border: null");
    if (dst.pad == 0) return 0;
    const long long total =
        (long long)dst.n * (2LL * dst.pad * (dst.w + 2 * dst.pad) + 2LL * dst.pad * dst.h) * dst.c_alloc;
    hipLaunchKernelGGL(zero_border_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, dst);
    return fg::launched("zero_border");
}

FG_API int fg_fold_add(fg_view gpad, int fold_pad, fg_view add, fg_view dst, hipStream_t stream) {
    if (!gpad.ptr || !dst.ptr || dst.c_alloc % 4 || gpad.c_alloc != dst.c_alloc ||
        (add.ptr && add.c_alloc != dst.c_alloc))
        return fg::fail(FG_ERR_INVALID, "fg_fold_add: bad args");
    if (gpad.h != dst.h + 2 * fold_pad || gpad.w != dst.w + 2 * fold_pad || gpad.n != dst.n)
        return fg::fail(FG_ERR_INVALID, "fg_fold_add: gpad %dx%d vs dst %dx%d fold %d", gpad.h, gpad.w, dst.h,
                        dst.w, fold_pad);
    if (fold_pad >= dst.h || fold_pad >= dst.w) return fg::fail(FG_ERR_INVALID, "fg_fold_add: fold too wide");
    const long long total =
        (long long)dst.n * (dst.h + 2 * dst.pad) * (dst.w + 2 * dst.pad) * (dst.c_alloc / 4);
    hipLaunchKernelGGL(fold_add_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, gpad,
                       fold_pad, add, dst);
    return fg::launched("fold_add");
}

FG_API int fg_unfold_nchw(fg_view gpad, int fold_pad, int c, fg_wview dst, int h, int w, int acc_channels,
                          hipStream_t stream) {
    if (!gpad.ptr || !dst.ptr || c <= 0 || c > gpad.c_alloc || fold_pad < 0 || h <= 0 || w <= 0)
        return fg::fail(FG_ERR_INVALID, "fg_unfold_nchw: bad args");
    if (gpad.h != h + 2 * fold_pad || gpad.w != w + 2 * fold_pad)
        return fg::fail(FG_ERR_INVALID, "fg_unfold_nchw: gpad %dx%d vs dst %dx%d fold %d", gpad.h, gpad.w, h, w,
                        fold_pad);
    if (fold_pad >= h || fold_pad >= w) return fg::fail(FG_ERR_INVALID, "fg_unfold_nchw: fold too wide");
    const long long total = (long long)gpad.n * c * h * w;
    if (total == 0) return 0;
    hipLaunchKernelGGL(unfold_nchw_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, gpad,
                       fold_pad, c, dst, h, w, acc_channels);
    return fg::launched("unfold_nchw");
}
