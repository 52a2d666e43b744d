// InstanceNorm2d (affine=False, track_running_stats=False; models/model_architectures.py
// :313-317, :407-410, :325-332, :428-437) fused with ReLU / LeakyReLU(0.2), the residual
// add of PairedAttentionBlock and the reflect / zero padding the next conv reads.
//
// Statistics: per-(n,c) plane sums over chunked pixel ranges, shifted by the plane's first
// value (robust E[x^2]-E[x]^2), accumulated per thread in fp32, combined in fp64.
// Backward: dL/dx = rstd * (g' - mean(g') - xhat * mean(g' xhat)), g' = g * act'(xhat).
#include <algorithm>

#include "conv_common.hpp"

namespace {

// fold this thread's max |v| (as uint bits) into the absmax slot: block max, then one atomic
// per block into shard blockIdx % FG_AMAX_SHARDS (256-thread blocks)
__device__ __forceinline__ void absmax_flush(unsigned m, unsigned* out) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    __shared__ unsigned red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(out + (blockIdx.x & (FG_AMAX_SHARDS - 1)), max(max(red[0], red[1]), max(red[2], red[3])));
}
__device__ __forceinline__ unsigned absbits4(const f32x4& v) {
    return max(max(__float_as_uint(v[0]) & 0x7fffffffu, __float_as_uint(v[1]) & 0x7fffffffu),
               max(__float_as_uint(v[2]) & 0x7fffffffu, __float_as_uint(v[3]) & 0x7fffffffu));
}

constexpr int NT = 256;
constexpr int MAX_CHUNKS = 256;
constexpr int CS_CHUNKS = 1024;     // channel-sum blocks (workspace: fg_channel_sum_workspace_doubles)

int choose_chunks(int n, long long hw, int target = 2048) {
    long long c = (target + n - 1) / n;    // ~target workgroups: enough loads in flight per CU
    if (c > hw / 64) c = hw / 64;
    if (c > MAX_CHUNKS) c = MAX_CHUNKS;
    if (c < 1) c = 1;
    return (int)c;
}
// the fused attention head's statistics pass (2 waves per SIMD at its register count): 512 workgroups are one
// resident round, and its weight-gradient slab (one row per workgroup) stays 4x smaller for the reduction
int head_chunks(int n, long long hw) { return choose_chunks(n, hw, 512); }


__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
// non-temporal (streaming) load: for bytes read for the last time, so they do not displace reused ones from the
// Infinity Cache
__device__ __forceinline__ f32x4 ld4_nt(const float* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
}
template <bool NTL>
__device__ __forceinline__ f32x4 ldx(const float* p) { return NTL ? ld4_nt(p) : ld4(p); }
// the apply passes' last reads of their inputs (the conv output, the residual / gradient) are non-temporal: the
// Infinity Cache then keeps the output the next conv reads instead of bytes never read again -- step 46.08 -> 45.60
// ms (profiles/round4/r4q_ab_in_nt2.log); FLOODGAN_IN_NT2=0 turns it off (read once per process)
bool in_nt2_on() {
    static const bool env = [] { const char* e = getenv("FLOODGAN_IN_NT2"); return !e || atoi(e) != 0; }();
    return env;
}

__global__ void in_stats_kernel(fg_view src, int chunks, double* __restrict__ work) {
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int HW = src.h * src.w;
    const int per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int g = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    __shared__ float red[NT][8];     // fp32 per-thread sums (exact as floats), combined in fp64
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = {0.f, 0.f, 0.f, 0.f};
    if (g < PG) {
        const f32x4 K = ld4(src.ptr + fg::vidx(src, n, 0, 0) + 4 * c4);
        // pixel walk without divisions: (y, x) advance by PG per step; 2 loads in flight
        int p = p0 + g, y = p / src.w, x = p - (p / src.w) * src.w;
        auto next = [&]() {
            p += PG;
            x += PG;
            while (x >= src.w) {
                x -= src.w;
                ++y;
            }
        };
        for (; p + PG < p1;) {
            const f32x4 v0 = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - K;
            next();
            const f32x4 v1 = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - K;
            next();
            s += v0 + v1;
            ss += v0 * v0 + v1 * v1;
        }
        if (p < p1) {
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

// finalize: block (n, 64-channel group), 64 x FG threads: thread (c, g) sums chunks g, g+FG, ...
// (coalesced over c), then the FG partials are combined in LDS (fixed order: deterministic)
constexpr int FG = 16;

__global__ void __launch_bounds__(64 * FG) in_finalize_kernel(fg_view src, int chunks, const double* __restrict__ work,
                                                               float eps, float* __restrict__ mean,
                                                               float* __restrict__ rstd) {
    const int C = src.c_alloc;
    const int n = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
    __shared__ double red[FG][64][2];
    double s1 = 0, s2 = 0;
    if (c < C)
        for (int k = g; k < chunks; k += FG) {
            s1 += work[((size_t)(n * chunks + k) * C + c) * 2];
            s2 += work[((size_t)(n * chunks + k) * C + c) * 2 + 1];
        }
    red[g][threadIdx.x & 63][0] = s1;
    red[g][threadIdx.x & 63][1] = s2;
    __syncthreads();
    if (g != 0 || c >= C) return;
    s1 = 0;
    s2 = 0;
    for (int gg = 0; gg < FG; ++gg) {
        s1 += red[gg][threadIdx.x][0];
        s2 += red[gg][threadIdx.x][1];
    }
    const double HW = (double)src.h * src.w;
    const double ms = s1 / HW;
    double var = s2 / HW - ms * ms;
    if (var < 0) var = 0;
    const double K = src.ptr[fg::vidx(src, n, 0, 0) + c];
    const int idx = n * C + c;
    mean[idx] = (float)(K + ms);
    rstd[idx] = (float)(1.0 / sqrt(var + (double)eps));
}

__global__ void in_apply_kernel(fg_view src, const float* __restrict__ mean, const float* __restrict__ rstd,
                                int act, fg_view res, fg_view dst, int pad_mode, unsigned* __restrict__ amax) {
    unsigned am = 0;
    const int C = dst.c_alloc, C4 = C / 4;
    const int hp = dst.h + 2 * dst.pad, wp = dst.w + 2 * dst.pad;
    const long long total = (long long)dst.n * hp * wp * C4;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4);
        long long pix = idx / C4;
        const int xp = (int)(pix % wp);
        pix /= wp;
        const int yp = (int)(pix % hp);
        const int n = (int)(pix / hp);
        int y = yp - dst.pad, x = xp - dst.pad;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const bool inside = y >= 0 && y < dst.h && x >= 0 && x < dst.w;
        if (inside || pad_mode == FG_PAD_REFLECT) {
            y = fg::reflect_idx(y, dst.h);
            x = fg::reflect_idx(x, dst.w);
            const f32x4 m = ld4(mean + (size_t)n * C + 4 * c4);
            const f32x4 r = ld4(rstd + (size_t)n * C + 4 * c4);
            v = (ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - m) * r;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fg::act_fwd(v[e], act);
            if (res.ptr) v += ld4(res.ptr + fg::vidx(res, n, y, x) + 4 * c4);
        }
        am = max(am, absbits4(v));
        *reinterpret_cast<f32x4*>(dst.ptr + ((size_t)(n * hp + yp) * wp + xp) * C + 4 * c4) = v;
    }
    if (amax) absmax_flush(am, amax);
}

// FG_PRESPLIT store (include/floodgan.h) of this lane's 4 channels o (scaled by s) at p = its fp32 position:
// lanes 2q, 2q+1 hold channels 8q..8q+3, 8q+4..8q+7 of one pixel; the even lane stores h[8] there, the odd
// lane l[8] (one swap of 8 bytes between the pair: quad_perm [1,0,3,2])
__device__ __forceinline__ void store_presplit(float* p, const f32x4& o, float s, int odd) {
    f16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float x = o[e] * s;
        h[e] = (_Float16)x;
        l[e] = (_Float16)(x - (float)h[e]);
    }
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    const i32x2 hv = __builtin_bit_cast(i32x2, h), lv = __builtin_bit_cast(i32x2, l);
    const i32x2 send = odd ? hv : lv;
    i32x2 recv;
    recv[0] = __builtin_amdgcn_update_dpp(0, send[0], 0xB1, 0xF, 0xF, false);
    recv[1] = __builtin_amdgcn_update_dpp(0, send[1], 0xB1, 0xF, 0xF, false);
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 out = odd ? i32x4{recv[0], recv[1], lv[0], lv[1]} : i32x4{hv[0], hv[1], recv[0], recv[1]};
    *reinterpret_cast<i32x4*>(p) = out;
}

// fg_split_pixels-layout store (the window convs' operand, conv_win.hip) of this lane's 4 channels o (scaled by s):
// per pixel [h(C) | l(C)] in 16-B chunks, chunk k stored at k ^ swz_pixel(x) for the pixel's padded column x;
// lanes 2q, 2q+1 hold channels 8q..8q+7 of the pixel at byte base px: after the same 8-byte swap as
// store_presplit the even lane stores h of group q (chunk q), the odd lane l (chunk C/8 + q)
template <int C>
__device__ __forceinline__ void store_splitpix(char* px, const f32x4& o, float s, int c4, int x) {
    f16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float v = o[e] * s;
        h[e] = (_Float16)v;
        l[e] = (_Float16)(v - (float)h[e]);
    }
    const int odd = c4 & 1, q = c4 >> 1;
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    const i32x2 hv = __builtin_bit_cast(i32x2, h), lv = __builtin_bit_cast(i32x2, l);
    const i32x2 send = odd ? hv : lv;
    i32x2 recv;
    recv[0] = __builtin_amdgcn_update_dpp(0, send[0], 0xB1, 0xF, 0xF, false);
    recv[1] = __builtin_amdgcn_update_dpp(0, send[1], 0xB1, 0xF, 0xF, false);
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 out = odd ? i32x4{recv[0], recv[1], lv[0], lv[1]} : i32x4{hv[0], hv[1], recv[0], recv[1]};
    const int k = odd ? C / 8 + q : q;
    *reinterpret_cast<i32x4*>(px + ((k ^ fgc::swz_pixel<C>(x)) << 4)) = out;
}

// Row form of the apply pass (channel quads dividing the block: C/4 | 256): block = one padded output
// row (n, yp), thread = (pixel lane gi, channel quad c4); mean / rstd read once per thread, U pixels'
// loads issued before any of them is used (the grid-stride form above re-derived (n, y, x, c) with
// 64-bit divisions per element and held one load in flight: 5.0 TB/s).
constexpr int kRowU = 4;

// The attention head (Conv2d(64, 10, 1), models/model_architectures.py:334, :369) fused into the norm passes of its
// 64-channel input (round 5): the 16 lanes of a pixel hold its 64 channels, four each.
//   forward: the apply pass also forms the head's logits y[p][o] = b[o] + sum_c w[o][c] a[p][c] from the activation
//            it just wrote -- the same per-lane fma chain and 16-lane DPP reduce-scatter as conv1x1_fwd_lanes
//            (head1x1.hip), so the logits are bit-identical to that kernel's, without re-reading the 537-MB activation;
//   backward: the statistics and apply passes read the 16-channel logits gradient instead of the 64-channel input
//            gradient and form g[p][c] = sum_o w[o][c] gy[p][o] in registers, in conv1x1_dgrad_kernel's fma order
//            (bit-identical): the dgrad launch and its 537-MB gradient (written once, read twice) are gone.
constexpr int HEAD_CI = 64, HEAD_NO = 16;
struct HeadArgs {
    const float* w;     // [n_out][64]
    const float* b;     // forward: [n_out] or null
    int n_out;
    fg_view y;          // forward: the logits (16-ch allocation, pad 0); backward: the logits gradient (16 ch)
    float* wslab = nullptr;   // backward (round 5): per-block partials of the 1x1 weight / bias gradient,
                              // [block][n_out][65] (conv1x1_wgrad's slab layout), or null
};

template <int CTRL>
__device__ __forceinline__ float head_dpp(float v) { return fg::dpp<CTRL>(v); }

// forward: lane cq (of a pixel's 16) holds channels 4cq..4cq+3 in v and w[o][4cq..4cq+3] in wr[o]; returns output cq's
// sum (conv1x1_fwd_lanes' order)
__device__ __forceinline__ float head_logit(const f32x4& v, const f32x4 (&wr)[HEAD_NO], int cq) {
    float acc[HEAD_NO];
#pragma unroll
    for (int o = 0; o < HEAD_NO; ++o)
        acc[o] = fmaf(v[3], wr[o][3], fmaf(v[2], wr[o][2], fmaf(v[1], wr[o][1], v[0] * wr[o][0])));
    const bool h3 = cq & 8, h2 = cq & 4, h1 = cq & 2, h0 = cq & 1;
    float a8[8], a4[4], a2[2];
#pragma unroll
    for (int k = 0; k < 8; ++k) a8[k] = (h3 ? acc[8 + k] : acc[k]) + head_dpp<0x140>(h3 ? acc[k] : acc[8 + k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) a4[k] = (h2 ? a8[4 + k] : a8[k]) + head_dpp<0x141>(h2 ? a8[k] : a8[4 + k]);
#pragma unroll
    for (int k = 0; k < 2; ++k) a2[k] = (h1 ? a4[2 + k] : a4[k]) + head_dpp<0x1B>(h1 ? a4[k] : a4[2 + k]);
    return (h0 ? a2[1] : a2[0]) + head_dpp<0xB1>(h0 ? a2[0] : a2[1]);
}

// backward: the logits gradient of pixel (n, y, x) (its first HEAD_NB channels: 3 quads, loaded in the load phase with
// the other operands), then the 4 channels' input gradient from it in conv1x1_dgrad_kernel's fma order
constexpr int HEAD_NB = 12;      // logits the fused backward takes (n_out <= 12)
struct HeadG {
    f32x4 q[HEAD_NB / 4];
};
__device__ __forceinline__ HeadG head_load(const fg_view& gy, int n, int y, int x) {
    const float* gp = gy.ptr + fg::vidx(gy, n, y, x);
    HeadG g;
#pragma unroll
    for (int q = 0; q < HEAD_NB / 4; ++q) g.q[q] = *reinterpret_cast<const f32x4*>(gp + 4 * q);
    return g;
}
__device__ __forceinline__ f32x4 head_grad(const HeadG& g, const f32x4 (&wr)[HEAD_NB], int n_out) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < HEAD_NB; ++o) {
        if (o < n_out) {
            const float go = g.q[o / 4][o % 4];
            a[0] = fmaf(go, wr[o][0], a[0]);
            a[1] = fmaf(go, wr[o][1], a[1]);
            a[2] = fmaf(go, wr[o][2], a[2]);
            a[3] = fmaf(go, wr[o][3], a[3]);
        }
    }
    return a;
}

template <int NO>
__device__ __forceinline__ void head_weights(const HeadArgs& hd, int c4, f32x4 (&wr)[NO]) {
#pragma unroll
    for (int o = 0; o < NO; ++o)
        wr[o] = o < hd.n_out ? *reinterpret_cast<const f32x4*>(hd.w + o * HEAD_CI + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
}

template <bool NTL, bool HEAD = false>
__global__ void __launch_bounds__(NT) in_apply_rows_kernel(fg_view src, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, int act, fg_view res,
                                                           fg_view dst, int pad_mode, int lshift,
                                                           unsigned* __restrict__ amax, float* __restrict__ split_slot,
                                                           float* __restrict__ ps_ptr, float* __restrict__ ps_slot,
                                                           const float* __restrict__ res_amax, int splitpix,
                                                           HeadArgs hd = HeadArgs{}) {
    const int L = 1 << lshift, PG = NT >> lshift;
    const int C = dst.c_alloc, h = dst.h, w = dst.w, pad = dst.pad;
    const int hp = h + 2 * pad, wp = w + 2 * pad;
    const int n = blockIdx.x / hp, yp = blockIdx.x - n * hp;
    const int gi = threadIdx.x >> lshift, c4 = threadIdx.x & (L - 1);
    float* drow = dst.ptr + (size_t)(n * hp + yp) * wp * C + 4 * c4;
    unsigned am = 0;
    int y = yp - pad;
    const bool reflect = pad_mode == FG_PAD_REFLECT;
    // pre-split output: |act(xhat)| <= |xhat| <= sqrt(HW - 1) (Samuelson), the static bound of the scale,
    // published in the output's scale slot by block 0 (the slot comes zeroed)
    float ss = 0.f;
    if (split_slot) {
        const float bound = sqrtf((float)(h * w - 1)) * 1.001f;
        ss = fgc::pow2_of(bound);
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned*>(split_slot), __float_as_uint(bound));
    }
    // dual output (ps_ptr): dst in fp32 AND a pre-split copy at the scale of |act(xhat) + res| <= sqrt(HW - 1) +
    // max|res| (the residual's absmax slot, reduced over its shards by every block alike)
    float* psrow = nullptr;
    if (ps_ptr) {
        const float rmax = res_amax ? fgc::pow2_scale_max(res_amax) : 0.f;
        const float bound = (sqrtf((float)(h * w - 1)) + rmax) * 1.001f;
        ss = fgc::pow2_of(bound);
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned*>(ps_slot), __float_as_uint(bound));
        psrow = ps_ptr + (size_t)(n * hp + yp) * wp * C + 4 * c4;
    }
    if ((y < 0 || y >= h) && !reflect) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        for (int xp = gi; xp < wp; xp += PG) {
            *reinterpret_cast<f32x4*>(drow + (size_t)xp * C) = z;
            if (psrow) *reinterpret_cast<f32x4*>(psrow + (size_t)xp * C) = z;
        }
    } else {
        y = fg::reflect_idx(y, h);
        const f32x4 m = ld4(mean + (size_t)n * C + 4 * c4), r = ld4(rstd + (size_t)n * C + 4 * c4);
        f32x4 wr[HEAD ? HEAD_NO : 1];
        float hb = 0.f;
        if constexpr (HEAD) {
            head_weights<HEAD_NO>(hd, c4, wr);
            hb = (hd.b && c4 < hd.n_out) ? hd.b[c4] : 0.f;
        }
        const float* srow = src.ptr + fg::vidx(src, n, y, 0) + 4 * c4;
        const float* rrow = res.ptr ? res.ptr + fg::vidx(res, n, y, 0) + 4 * c4 : nullptr;
        for (int xp0 = gi; xp0 < wp; xp0 += kRowU * PG) {
            f32x4 v[kRowU], rv[kRowU];
            bool ok[kRowU];
#pragma unroll
            for (int k = 0; k < kRowU; ++k) {
                const int xp = xp0 + k * PG;
                int x = xp - pad;
                const bool inside = x >= 0 && x < w;
                ok[k] = xp < wp && (inside || reflect);
                x = ok[k] ? fg::reflect_idx(x, w) : 0;
                v[k] = ok[k] ? ldx<NTL>(srow + (size_t)x * C) : f32x4{0.f, 0.f, 0.f, 0.f};
                rv[k] = (ok[k] && rrow) ? ldx<NTL>(rrow + (size_t)x * C) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int k = 0; k < kRowU; ++k) {
                const int xp = xp0 + k * PG;
                if (xp >= wp) break;
                f32x4 o = {0.f, 0.f, 0.f, 0.f};
                if (ok[k]) {
                    o = (v[k] - m) * r;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = fg::act_fwd(o[e], act);
                    o += rv[k];
                }
                if (split_slot && splitpix) {
                    char* pxb = reinterpret_cast<char*>(drow - 4 * c4 + (size_t)xp * C);
                    if (C == 64) store_splitpix<64>(pxb, o, ss, c4, xp);
                    else store_splitpix<32>(pxb, o, ss, c4, xp);
                } else if (split_slot) {
                    store_presplit(drow + (size_t)xp * C, o, ss, c4 & 1);
                } else if (!HEAD || dst.ptr) {      // the fused head may skip its activation (dst null)
                    am = max(am, absbits4(o));
                    *reinterpret_cast<f32x4*>(drow + (size_t)xp * C) = o;
                    if (psrow) store_presplit(psrow + (size_t)xp * C, o, ss, c4 & 1);
                }
                if constexpr (HEAD) {       // the interior (the head reads an unpadded activation: pad 0)
                    const float lg = head_logit(o, wr, c4);
                    if (c4 < hd.y.c_alloc) hd.y.ptr[fg::vidx(hd.y, n, y, xp - pad) + c4] = lg + hb;
                }
            }
        }
    }
    if (amax) absmax_flush(am, amax);
}

// ---- backward ----

__device__ __forceinline__ int fold_src(int y, int h, int p, int* out) {
    int k = 0;
    out[k++] = y + p;
    if (y >= 1 && y <= p) out[k++] = p - y;
    if (y >= h - 1 - p && y <= h - 2) out[k++] = p + 2 * (h - 1) - y;
    return k;
}

__device__ __forceinline__ f32x4 load_grad(const fg_view& g, int fp, const fg_view& gadd, int n, int y, int x,
                                           int h, int w, int c4) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (fp > 0) {
        int ys[3], xs[3];
        const int ny = fold_src(y, h, fp, ys), nx = fold_src(x, w, fp, xs);
        for (int iy = 0; iy < ny; ++iy)
            for (int ix = 0; ix < nx; ++ix) v += ld4(g.ptr + fg::vidx(g, n, ys[iy], xs[ix]) + 4 * c4);
    } else {
        v = ld4(g.ptr + fg::vidx(g, n, y, x) + 4 * c4);
    }
    if (gadd.ptr) v += ld4(gadd.ptr + fg::vidx(gadd, n, y, x) + 4 * c4);
    return v;
}

// every fold term of interior pixel (y, x) except the main one (y + fp, x + fp): the reflect-pad adjoint's
// extra terms, nonzero only within fp + 1 of the border
__device__ __forceinline__ bool fold_border(int y, int x, int h, int w, int fp) {
    return fp > 0 && (y <= fp || y >= h - 1 - fp || x <= fp || x >= w - 1 - fp);
}
// (added to v = the main term in load_grad's order: bit-identical sums)
__device__ __forceinline__ f32x4 fold_extra(f32x4 v, const fg_view& g, int fp, int n, int y, int x, int h, int w,
                                            int c4) {
    int ys[3], xs[3];
    const int ny = fold_src(y, h, fp, ys), nx = fold_src(x, w, fp, xs);
    for (int iy = 0; iy < ny; ++iy)
        for (int ix = 0; ix < nx; ++ix)
            if (iy | ix) v += ld4(g.ptr + fg::vidx(g, n, ys[iy], xs[ix]) + 4 * c4);
    return v;
}

// statistics pass with kRowU pixels' loads in flight per thread (same chunking / work layout and the same
// fp32 accumulation order per thread as in_bwd_stats_kernel: results are bit-identical).  NTG: the gradient and gadd
// are read non-temporally -- with gsum the apply pass reads the gathered sum instead of them, so they are dead after
// this pass, and src + gsum (268 MB at the resblock shape) can stay in the 256-MB Infinity Cache for the apply pass
template <bool NTG, bool HEAD = false>
__global__ void __launch_bounds__(NT) in_bwd_stats_u_kernel(fg_view g, int fp, fg_view gadd, fg_view src,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int act, int chunks,
                                                            double* __restrict__ work, fg_view gsum,
                                                            float* __restrict__ gmax_part, HeadArgs hd = HeadArgs{}) {
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    unsigned gm = 0;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int h = src.h, w = src.w, HW = h * w;
    const int per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int gi = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    __shared__ float red[NT][12];    // fp32 per-thread sums (exact as floats), combined in fp64: 12 KB, not 24
    f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sgx = sg, sx = sg;
    // HEAD with wslab: the 1x1 head's weight / bias gradient, sum_p g_logits[p][o] * act(xhat[p][c]) and
    // sum_p g_logits[p][o], from the operands this pass holds anyway (the activation is recomputed from src, so the
    // forward need not write it)
    const bool wg = HEAD && hd.wslab;
    f32x4 wacc[HEAD ? HEAD_NB : 1];
    float bacc[HEAD ? HEAD_NB : 1];
#pragma unroll
    for (int o = 0; o < (HEAD ? HEAD_NB : 1); ++o) {
        wacc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
        bacc[o] = 0.f;
    }
    // (the head variant keeps 3 pixels in flight per thread, not kRowU: its logits-gradient quads, weights and
    // weight-gradient accumulators would otherwise push it past 256 VGPRs, one wave per SIMD)
    constexpr int RU = HEAD ? 3 : kRowU;
    if (gi < PG) {
        const f32x4 m = ld4(mean + (size_t)n * C + 4 * c4);
        const f32x4 r = ld4(rstd + (size_t)n * C + 4 * c4);
        f32x4 wr[HEAD ? HEAD_NB : 1];
        if constexpr (HEAD) head_weights(hd, c4, wr);
        int y = (p0 + gi) / w, x = (p0 + gi) - ((p0 + gi) / w) * w;
        for (int p = p0 + gi; p < p1; p += RU * PG) {
            int ys[RU], xs[RU];
            f32x4 sv[RU], gv[RU], av[RU];
            HeadG hg[HEAD ? RU : 1];
#pragma unroll
            for (int k = 0; k < RU; ++k) {
                ys[k] = y;
                xs[k] = x;
                const bool ok = p + k * PG < p1;
                sv[k] = ok ? ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
                const float* gp = g.ptr + fg::vidx(g, n, y + fp, x + fp) + 4 * c4;
                if constexpr (HEAD)
                    hg[k] = head_load(hd.y, n, ok ? y : 0, ok ? x : 0);
                else
                    gv[k] = ok ? (NTG ? ld4_nt(gp) : ld4(gp)) : f32x4{0.f, 0.f, 0.f, 0.f};
                const float* ap = gadd.ptr + fg::vidx(gadd, n, y, x) + 4 * c4;
                av[k] = (ok && gadd.ptr) ? (NTG ? ld4_nt(ap) : ld4(ap)) : f32x4{0.f, 0.f, 0.f, 0.f};
                x += PG;
                while (x >= w) {
                    x -= w;
                    ++y;
                }
            }
#pragma unroll
            for (int k = 0; k < RU; ++k) {
                if (p + k * PG >= p1) break;
                if constexpr (HEAD) gv[k] = head_grad(hg[k], wr, hd.n_out);
                f32x4 gk = gv[k];
                if (fold_border(ys[k], xs[k], h, w, fp)) gk = fold_extra(gk, g, fp, n, ys[k], xs[k], h, w, c4);
                gk += av[k];
                if (gsum.ptr) *reinterpret_cast<f32x4*>(gsum.ptr + fg::vidx(gsum, n, ys[k], xs[k]) + 4 * c4) = gk;
                const f32x4 xh = (sv[k] - m) * r;
                if constexpr (HEAD) {
                    if (wg) {
                        f32x4 a;
#pragma unroll
                        for (int e = 0; e < 4; ++e) a[e] = fg::act_fwd(xh[e], act);
#pragma unroll
                        for (int o = 0; o < HEAD_NB; ++o)
                            if (o < hd.n_out) {
                                const float go = hg[k].q[o / 4][o % 4];
#pragma unroll
                                for (int e = 0; e < 4; ++e) wacc[o][e] = fmaf(go, a[e], wacc[o][e]);
                                bacc[o] += go;
                            }
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) gk[e] *= fg::act_grad(xh[e], act);
                gm = max(gm, absbits4(gk));
                sg += gk;
                sgx += gk * xh;
                sx += xh;
            }
        }
    }
    if (gmax_part) {     // this block's max |g'| (the pre-split output's scale bound, fg_in_bwd_presplit)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) gm = max(gm, (unsigned)__shfl_xor((int)gm, off));
        __shared__ unsigned gred[NT / 64];
        if ((threadIdx.x & 63) == 0) gred[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < NT / 64; ++i) gm = max(gm, gred[i]);
            gmax_part[n * chunks + chunk] = __uint_as_float(gm);
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[threadIdx.x][e] = sg[e];
        red[threadIdx.x][4 + e] = sgx[e];
        red[threadIdx.x][8 + e] = sx[e];
    }
    __syncthreads();
    if (threadIdx.x < L) {
        double a[12] = {0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 12; ++e) a[e] += red[gg * L + threadIdx.x][e];
        double* wk = work + ((size_t)(n * chunks + chunk) * C + 4 * threadIdx.x) * 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            wk[3 * e] = a[e];
            wk[3 * e + 1] = a[4 + e];
            wk[3 * e + 2] = a[8 + e];
        }
    }
    if constexpr (HEAD) {
        if (wg) {
            // the block's partial: over the 4 pixel groups of a wave (lanes l, l^16, l^32, l^48: same c4), then over
            // the 4 waves in LDS; slab row o of block (n, chunk): 64 weight columns, then the bias
            constexpr int NV = HEAD_NB * 5;          // 48 weight + 12 bias values per c4
            __shared__ float wred[NT / 64][16][NV];
            const int wave = threadIdx.x >> 6;
#pragma unroll
            for (int o = 0; o < HEAD_NB; ++o) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = wacc[o][e];
                    v += __shfl_xor(v, 16);
                    v += __shfl_xor(v, 32);
                    wacc[o][e] = v;
                }
                float bv = bacc[o];
                bv += __shfl_xor(bv, 16);
                bv += __shfl_xor(bv, 32);
                bacc[o] = bv;
            }
            if ((threadIdx.x & 63) < 16) {
#pragma unroll
                for (int o = 0; o < HEAD_NB; ++o) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) wred[wave][c4][o * 4 + e] = wacc[o][e];
                    wred[wave][c4][HEAD_NB * 4 + o] = bacc[o];
                }
            }
            __syncthreads();
            float* slab = hd.wslab + (size_t)(n * chunks + chunk) * hd.n_out * (HEAD_CI + 1);
            for (int i = threadIdx.x; i < 16 * NV; i += NT) {
                const int q = i / NV, j = i - q * NV;
                float v = 0.f;
#pragma unroll
                for (int wv = 0; wv < NT / 64; ++wv) v += wred[wv][q][j];
                if (j < HEAD_NB * 4) {
                    const int o = j >> 2;
                    if (o < hd.n_out) slab[o * (HEAD_CI + 1) + 4 * q + (j & 3)] = v;
                } else if (q == 0 && j - HEAD_NB * 4 < hd.n_out) {
                    slab[(j - HEAD_NB * 4) * (HEAD_CI + 1) + HEAD_CI] = v;
                }
            }
        }
    }
}

__global__ void in_bwd_stats_kernel(fg_view g, int fp, fg_view gadd, fg_view src, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, int act, int chunks, double* __restrict__ work,
                                    fg_view gsum) {
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int h = src.h, w = src.w, HW = h * w;
    const int per = (HW + chunks - 1) / chunks;
    const int p0 = chunk * per, p1 = min(HW, p0 + per);
    const int gi = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    __shared__ float red[NT][12];    // fp32 per-thread sums (exact as floats), combined in fp64: 12 KB, not 24
    f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sgx = sg, sx = sg;
    if (gi < PG) {
        const f32x4 m = ld4(mean + (size_t)n * C + 4 * c4);
        const f32x4 r = ld4(rstd + (size_t)n * C + 4 * c4);
        int y = (p0 + gi) / w, x = (p0 + gi) - ((p0 + gi) / w) * w;   // walked without divisions
        for (int p = p0 + gi; p < p1; p += PG) {
            const f32x4 xh = (ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - m) * r;
            f32x4 gv = load_grad(g, fp, gadd, n, y, x, h, w, c4);
            if (gsum.ptr) *reinterpret_cast<f32x4*>(gsum.ptr + fg::vidx(gsum, n, y, x) + 4 * c4) = gv;
#pragma unroll
            for (int e = 0; e < 4; ++e) gv[e] *= fg::act_grad(xh[e], act);
            sg += gv;
            sgx += gv * xh;
            sx += xh;
            x += PG;
            while (x >= w) {
                x -= w;
                ++y;
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[threadIdx.x][e] = sg[e];
        red[threadIdx.x][4 + e] = sgx[e];
        red[threadIdx.x][8 + e] = sx[e];
    }
    __syncthreads();
    if (threadIdx.x < L) {
        double a[12] = {0};
        for (int gg = 0; gg < PG; ++gg)
#pragma unroll
            for (int e = 0; e < 12; ++e) a[e] += red[gg * L + threadIdx.x][e];
        double* wk = work + ((size_t)(n * chunks + chunk) * C + 4 * threadIdx.x) * 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            wk[3 * e] = a[e];
            wk[3 * e + 1] = a[4 + e];
            wk[3 * e + 2] = a[8 + e];
        }
    }
}

// block (n, 16-channel group), 1024 threads = 16 channels x 64 chunk slices (the partials of one image are ~1.5 MB:
// 64-channel blocks, 32 of them at bs 8, were bandwidth-bound on their CU -- 12.6 us per call): coefficients of the
// apply pass and the per-plane part of the (mathematically cancelled) conv-bias gradient; a fixed-order tree over the
// slices (deterministic)
constexpr int kFinC = 16, kFinS = 64;

__global__ void __launch_bounds__(kFinC * kFinS) in_bwd_finalize_kernel(int N, int C, int HWi, int chunks,
                                                                        const double* __restrict__ work,
                                                                        const float* __restrict__ rstd,
                                                                        float* __restrict__ coef,
                                                                        double* __restrict__ bpart,
                                                                        const float* __restrict__ gmax_part,
                                                                        float* __restrict__ split_slot) {
    const int n = blockIdx.x, cl = threadIdx.x % kFinC, sl = threadIdx.x / kFinC, c = blockIdx.y * kFinC + cl;
    __shared__ double red[kFinS][kFinC][3];
    __shared__ unsigned gmx, bmx;
    if (split_slot) {
        if (threadIdx.x == 0) gmx = bmx = 0;
        __syncthreads();
        unsigned m = 0;
        for (int k = threadIdx.x; k < chunks; k += blockDim.x) m = max(m, __float_as_uint(gmax_part[n * chunks + k]));
        atomicMax(&gmx, m);
    }
    double sg = 0, sgx = 0, sx = 0;
    if (c < C) {
        int k = sl;
        for (; k + 3 * kFinS < chunks; k += 4 * kFinS) {       // four chunks' loads in flight
            double v[4][3];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double* wk = work + ((size_t)(n * chunks + k + u * kFinS) * C + c) * 3;
                v[u][0] = wk[0];
                v[u][1] = wk[1];
                v[u][2] = wk[2];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sg += v[u][0];
                sgx += v[u][1];
                sx += v[u][2];
            }
        }
        for (; k < chunks; k += kFinS) {
            const double* wk = work + ((size_t)(n * chunks + k) * C + c) * 3;
            sg += wk[0];
            sgx += wk[1];
            sx += wk[2];
        }
    }
    red[sl][cl][0] = sg;
    red[sl][cl][1] = sgx;
    red[sl][cl][2] = sx;
#pragma unroll
    for (int st = kFinS / 2; st > 0; st >>= 1) {
        __syncthreads();
        if (sl < st) {
            red[sl][cl][0] += red[sl + st][cl][0];
            red[sl][cl][1] += red[sl + st][cl][1];
            red[sl][cl][2] += red[sl + st][cl][2];
        }
    }
    __syncthreads();
    if (sl == 0 && c < C) {
        sg = red[0][cl][0];
        sgx = red[0][cl][1];
        sx = red[0][cl][2];
        const double HW = (double)HWi;
        const int idx = n * C + c;
        const float c1 = (float)(sg / HW), c2 = (float)(sgx / HW);
        coef[(size_t)idx * 2] = c1;
        coef[(size_t)idx * 2 + 1] = c2;
        // sum_hw rstd*(g' - mean g' - xhat*mean(g'xhat)) = -rstd * sx * sgx / HW
        bpart[idx] = -(double)rstd[idx] * sx * sgx / HW;
        if (split_slot) {
            // |rstd (g' - c1 - xhat c2)| <= rstd (max|g'| + |c1| + sqrt(HW - 1) |c2|), with rounding slack
            const float b = rstd[idx] * (__uint_as_float(gmx) + fabsf(c1) + sqrtf((float)(HWi - 1)) * fabsf(c2)) * 1.001f;
            atomicMax(&bmx, __float_as_uint(b));
        }
    }
    if (split_slot) {
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<unsigned*>(split_slot) + ((n * gridDim.y + blockIdx.y) & (FG_AMAX_SHARDS - 1)), bmx);
    }
}

__global__ void in_bwd_apply_kernel(fg_view g, int fp, fg_view gadd, fg_view src, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ coef, int act,
                                    fg_view dst, unsigned* __restrict__ amax, const double* __restrict__ bpart,
                                    float* __restrict__ bias_grad, int bias_accumulate) {
    // block 0 also sums the per-plane bias-gradient parts of the finalize over the images (the finalize
    // has completed: kernel boundary) -- no launch of its own for a few hundred values
    if (bias_grad && blockIdx.x == 0) {
        const int C = dst.c_alloc;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            double s = 0;
            for (int n = 0; n < dst.n; ++n) s += bpart[(size_t)n * C + c];
            bias_grad[c] = bias_accumulate ? bias_grad[c] + (float)s : (float)s;
        }
    }
    unsigned am = 0;
    const int C = dst.c_alloc, C4 = C / 4;
    const int h = dst.h, w = dst.w;
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
        f32x4 out = {0.f, 0.f, 0.f, 0.f};
        if (y >= 0 && y < h && x >= 0 && x < w) {
            const size_t nc = (size_t)n * C + 4 * c4;
            const f32x4 m = ld4(mean + nc), r = ld4(rstd + nc);
            const f32x4 xh = (ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4) - m) * r;
            f32x4 gv = load_grad(g, fp, gadd, n, y, x, h, w, c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float gp = gv[e] * fg::act_grad(xh[e], act);
                out[e] = r[e] * (gp - coef[(nc + e) * 2] - xh[e] * coef[(nc + e) * 2 + 1]);
            }
        }
        am = max(am, absbits4(out));
        *reinterpret_cast<f32x4*>(dst.ptr + ((size_t)(n * hp + yp) * wp + xp) * C + 4 * c4) = out;
    }
    if (amax) absmax_flush(am, amax);
}

// row form of the backward apply (C/4 | 256): block = one padded output row, kRowU pixels' loads in flight
template <bool NTL, bool HEAD = false>
__global__ void __launch_bounds__(NT) in_bwd_apply_rows_kernel(fg_view g, int fp, fg_view gadd, fg_view src,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ coef, int act, fg_view dst,
                                                               unsigned* __restrict__ amax,
                                                               const double* __restrict__ bpart,
                                                               float* __restrict__ bias_grad, int bias_accumulate,
                                                               int lshift, const float* __restrict__ split_slot,
                                                               HeadArgs hd = HeadArgs{}) {
    // pre-split output: the scale of the bound the finalize published (the consumer derives the same one)
    const float ss = split_slot ? fgc::pow2_scale(split_slot) : 0.f;
    if (bias_grad && blockIdx.x == 0) {
        const int C = dst.c_alloc;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            double s = 0;
            for (int n = 0; n < dst.n; ++n) s += bpart[(size_t)n * C + c];
            bias_grad[c] = bias_accumulate ? bias_grad[c] + (float)s : (float)s;
        }
    }
    const int L = 1 << lshift, PG = NT >> lshift;
    const int C = dst.c_alloc, h = dst.h, w = dst.w, pad = dst.pad;
    const int hp = h + 2 * pad, wp = w + 2 * pad;
    const int n = blockIdx.x / hp, yp = blockIdx.x - n * hp;
    const int gi = threadIdx.x >> lshift, c4 = threadIdx.x & (L - 1);
    float* drow = dst.ptr + (size_t)(n * hp + yp) * wp * C + 4 * c4;
    unsigned am = 0;
    const int y = yp - pad;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if (y < 0 || y >= h) {
        for (int xp = gi; xp < wp; xp += PG) *reinterpret_cast<f32x4*>(drow + (size_t)xp * C) = z;
    } else {
        const size_t nc = (size_t)n * C + 4 * c4;
        const f32x4 m = ld4(mean + nc), r = ld4(rstd + nc);
        const f32x4 k01 = ld4(coef + nc * 2), k23 = ld4(coef + nc * 2 + 4);
        const f32x4 c1 = {k01[0], k01[2], k23[0], k23[2]}, c2 = {k01[1], k01[3], k23[1], k23[3]};
        f32x4 wr[HEAD ? HEAD_NB : 1];
        if constexpr (HEAD) head_weights(hd, c4, wr);
        const float* srow = src.ptr + fg::vidx(src, n, y, 0) + 4 * c4;
        const float* grow = HEAD ? nullptr : g.ptr + fg::vidx(g, n, y + fp, fp) + 4 * c4;
        const float* arow = gadd.ptr ? gadd.ptr + fg::vidx(gadd, n, y, 0) + 4 * c4 : nullptr;
        for (int xp0 = gi; xp0 < wp; xp0 += kRowU * PG) {
            f32x4 sv[kRowU], gv[kRowU], av[kRowU];
            HeadG hg[HEAD ? kRowU : 1];
            bool ok[kRowU];
#pragma unroll
            for (int k = 0; k < kRowU; ++k) {
                const int x = xp0 + k * PG - pad;
                ok[k] = x >= 0 && x < w;
                sv[k] = ok[k] ? ldx<NTL>(srow + (size_t)x * C) : z;
                if constexpr (HEAD)
                    hg[k] = head_load(hd.y, n, y, ok[k] ? x : 0);
                else
                    gv[k] = ok[k] ? ldx<NTL>(grow + (size_t)x * C) : z;
                av[k] = (ok[k] && arow) ? ldx<NTL>(arow + (size_t)x * C) : z;
            }
#pragma unroll
            for (int k = 0; k < kRowU; ++k) {
                const int xp = xp0 + k * PG;
                if (xp >= wp) break;
                f32x4 out = z;
                if (ok[k]) {
                    const int x = xp - pad;
                    if constexpr (HEAD) gv[k] = head_grad(hg[k], wr, hd.n_out);
                    f32x4 gk = gv[k];
                    if (fold_border(y, x, h, w, fp)) gk = fold_extra(gk, g, fp, n, y, x, h, w, c4);
                    gk += av[k];
                    const f32x4 xh = (sv[k] - m) * r;
#pragma unroll
                    for (int e = 0; e < 4; ++e) out[e] = r[e] * (gk[e] * fg::act_grad(xh[e], act) - c1[e] - xh[e] * c2[e]);
                }
                if (split_slot) {
                    store_presplit(drow + (size_t)xp * C, out, ss, c4 & 1);
                } else {
                    am = max(am, absbits4(out));
                    *reinterpret_cast<f32x4*>(drow + (size_t)xp * C) = out;
                }
            }
        }
    }
    if (amax) absmax_flush(am, amax);
}

// float4 form: block = interior row (n, yy), threads over (x, channel quad) of the row
__global__ void __launch_bounds__(256) act_bwd4_kernel(fg_view g, fg_view y, int act, unsigned* __restrict__ amax) {
    unsigned am = 0;
    const int C = g.c_alloc, C4 = C / 4, W4 = g.w * C4;
    const int n = blockIdx.x / g.h, yy = blockIdx.x - (blockIdx.x / g.h) * g.h;
    float* grow = g.ptr + fg::vidx(g, n, yy, 0);
    const float* yrow = y.ptr + fg::vidx(y, n, yy, 0);
    for (int i = threadIdx.x; i < W4; i += 256) {
        const int x = i / C4, c = (i - x * C4) * 4;
        f32x4 gv = ld4(grow + (size_t)x * C + c);
        const f32x4 yv = ld4(yrow + (size_t)x * C + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) gv[e] *= fg::act_grad(yv[e], act);
        am = max(am, absbits4(gv));
        *reinterpret_cast<f32x4*>(grow + (size_t)x * C + c) = gv;
    }
    if (amax) absmax_flush(am, amax);
}

__global__ void act_bwd_kernel(fg_view g, fg_view y, int act, unsigned* __restrict__ amax) {
    unsigned am = 0;
    const int C = g.c_alloc;
    const long long total = (long long)g.n * g.h * g.w * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(idx % C);
        long long pix = idx / C;
        const int x = (int)(pix % g.w);
        pix /= g.w;
        const int yy = (int)(pix % g.h);
        const int n = (int)(pix / g.h);
        const float yv = y.ptr[fg::vidx(y, n, yy, x) + c];
        const float v = g.ptr[fg::vidx(g, n, yy, x) + c] * fg::act_grad(yv, act);
        am = max(am, __float_as_uint(v) & 0x7fffffffu);
        g.ptr[fg::vidx(g, n, yy, x) + c] = v;
    }
    if (amax) absmax_flush(am, amax);
}

__global__ void channel_sum_kernel(fg_view src, int c_valid, int chunks, double* __restrict__ work) {
    // block (chunk, channel-group); threads = (pixel lane g, channel cl)
    const int cg = blockIdx.y;
    const int cbase = cg * NT;
    const int L = min(NT, c_valid - cbase);
    const int PG = NT / L;
    const int gi = threadIdx.x / L, cl = threadIdx.x - (threadIdx.x / L) * L;
    const long long P = (long long)src.n * src.h * src.w;
    const long long per = (P + chunks - 1) / chunks;
    const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
    __shared__ double red[NT];
    double acc = 0;
    if (gi < PG) {
        float s = 0.f;
        int cnt = 0;
        for (long long p = p0 + gi; p < p1; p += PG) {
            const int x = (int)(p % src.w);
            const long long t = p / src.w;
            const int y = (int)(t % src.h);
            const int n = (int)(t / src.h);
            s += src.ptr[fg::vidx(src, n, y, x) + cbase + cl];
            if (++cnt == 256) {
                acc += s;
                s = 0.f;
                cnt = 0;
            }
        }
        acc += s;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < L) {
        double a = 0;
        for (int gg = 0; gg < PG; ++gg) a += red[gg * L + threadIdx.x];
        work[(size_t)blockIdx.x * c_valid + cbase + threadIdx.x] = a;
    }
}

__global__ void __launch_bounds__(256) channel_sum4_kernel(fg_view src, int chunks, double* __restrict__ work) {
    // c_alloc % 4 == 0: threads = (pixel lane gi, float4 channel group c4); the block's pixel range is
    // walked as (n, y, x) without divisions, two pixels per trip
    const int C = src.c_alloc, L = C / 4, PG = NT / L;
    const int gi = threadIdx.x / L, c4 = threadIdx.x - (threadIdx.x / L) * L;
    const long long P = (long long)src.n * src.h * src.w;
    const long long per = (P + chunks - 1) / chunks;
    const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
    __shared__ float red[NT][4];     // fp32 per-thread sums, combined in fp64
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (gi < PG && p0 + gi < p1) {
        const long long q = p0 + gi;
        int x = (int)(q % src.w), y = (int)((q / src.w) % src.h), n = (int)(q / ((long long)src.w * src.h));
        auto step = [&]() {
            x += PG;
            while (x >= src.w) {
                x -= src.w;
                if (++y == src.h) { y = 0; ++n; }
            }
        };
        const int cnt = (int)((p1 - q + PG - 1) / PG);       // pixels of this lane (per <= 4096: fp32-safe)
        int k = 0;
        for (; k + 1 < cnt; k += 2) {
            const f32x4 a = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4);
            step();
            const f32x4 b = ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4);
            step();
            s += a + b;
        }
        if (k < cnt) s += ld4(src.ptr + fg::vidx(src, n, y, x) + 4 * c4);
    }
    for (int e = 0; e < 4; ++e) red[threadIdx.x][e] = s[e];
    __syncthreads();
    if (threadIdx.x < L) {
        double a[4] = {0, 0, 0, 0};
        for (int gg = 0; gg < PG; ++gg)
            for (int e = 0; e < 4; ++e) a[e] += red[gg * L + threadIdx.x][e];
        for (int e = 0; e < 4; ++e) work[(size_t)blockIdx.x * C + 4 * threadIdx.x + e] = a[e];
    }
}

// block = one channel: 256 lanes sum the chunk partials (strided), then a fixed-order tree
__global__ void __launch_bounds__(256) channel_sum4_finalize(int C, int c_valid, int chunks,
                                                             const double* __restrict__ work, float* out,
                                                             int accumulate) {
    const int c = blockIdx.x;
    __shared__ double red[256];
    double s = 0;
    for (int k = threadIdx.x; k < chunks; k += 256) s += work[(size_t)k * C + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float v = (float)red[0];
        if (accumulate) v += out[c];
        out[c] = v;
    }
}

__global__ void channel_sum_finalize(int c_valid, int chunks, const double* __restrict__ work, float* out,
                                     int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_valid) return;
    double s = 0;
    for (int k = 0; k < chunks; ++k) s += work[(size_t)k * c_valid + c];
    float v = (float)s;
    if (accumulate) v += out[c];
    out[c] = v;
}

bool ok_view(const fg_view& v) { return v.ptr && v.n > 0 && v.h > 0 && v.w > 0 && v.c_alloc > 0 && v.pad >= 0; }

// per-(image, channel) statistics from the pipelined conv kernel's epilogue partials: (mean, M2) of
// every 32-row block, merged in fp64 (S1 = sum 32 mean_i, S2 = sum M2_i + 32 mean_i^2) in two levels:
// in_partials_reduce -- block = 64 channels x 4 row slices over one of `splits` ranges of an image's blocks
// (coalesced 512-B rows of f32x2), fp64 partial sums into work; in_partials_finalize -- sums the splits.
constexpr int kPartialSplitsMax = 64;
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void in_partials_reduce(const float* __restrict__ part, int nprob, int n_img, int rb_per_img, int c,
                                   int splits, double* __restrict__ work) {
    const int img = blockIdx.x, sp = blockIdx.z, cl = threadIdx.x % 64, sl = threadIdx.x / 64;
    const int ch = blockIdx.y * 64 + cl;
    const size_t prob_stride = (size_t)n_img * rb_per_img * c * 2;
    const int K = nprob * rb_per_img;
    const int lo = (int)((long long)K * sp / splits), hi = (int)((long long)K * (sp + 1) / splits);
    double s1 = 0, s2 = 0;
    if (ch < c)
        for (int k = lo + sl; k < hi; k += 4) {
            const int pr = k / rb_per_img, rb = img * rb_per_img + (k - pr * rb_per_img);
            const f32x2 q = *reinterpret_cast<const f32x2*>(part + pr * prob_stride + ((size_t)rb * c + ch) * 2);
            const double m = q[0];
            s1 += 32.0 * m;
            s2 += (double)q[1] + 32.0 * m * m;
        }
    __shared__ double red[256][2];
    red[threadIdx.x][0] = s1;
    red[threadIdx.x][1] = s2;
    __syncthreads();
    if (sl == 0 && ch < c) {
        for (int q = 1; q < 4; ++q) {
            s1 += red[q * 64 + cl][0];
            s2 += red[q * 64 + cl][1];
        }
        double* w = work + (((size_t)img * splits + sp) * c + ch) * 2;
        w[0] = s1;
        w[1] = s2;
    }
}

__global__ void in_partials_finalize(const double* __restrict__ work, int nprob, int rb_per_img, int c, int splits,
                                     float eps, float* __restrict__ mean, float* __restrict__ rstd) {
    const int img = blockIdx.x, cl = threadIdx.x % 64, sl = threadIdx.x / 64;
    const int ch = blockIdx.y * 64 + cl;
    double s1 = 0, s2 = 0;
    if (ch < c)
        for (int sp = sl; sp < splits; sp += 4) {
            const double* w = work + (((size_t)img * splits + sp) * c + ch) * 2;
            s1 += w[0];
            s2 += w[1];
        }
    __shared__ double red[256][2];
    red[threadIdx.x][0] = s1;
    red[threadIdx.x][1] = s2;
    __syncthreads();
    if (sl == 0 && ch < c) {
        for (int q = 1; q < 4; ++q) {
            s1 += red[q * 64 + cl][0];
            s2 += red[q * 64 + cl][1];
        }
        const double n = 32.0 * nprob * rb_per_img;
        const double mu = s1 / n;
        double var = s2 / n - mu * mu;
        if (var < 0) var = 0;
        mean[img * c + ch] = (float)mu;
        rstd[img * c + ch] = (float)(1.0 / sqrt(var + (double)eps));
    }
}

// one launch for short partial lists (K = nprob * rb_per_img <= kPartialsDirectK: the resblock convs' 512 blocks
// per image): block = (image, 16 channels), thread = (channel, one of 16 slices of the 32-row blocks), the slices
// summed in LDS and finalized in the same block -- the two launches above cost ~13 us where this one streams its
// 64 KB per block
constexpr int kPartialsDirectK = 2048;
__global__ void in_partials_direct(const float* __restrict__ part, int nprob, int n_img, int rb_per_img, int c,
                                   float eps, float* __restrict__ mean, float* __restrict__ rstd) {
    const int img = blockIdx.x, cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int ch = blockIdx.y * 16 + cl;
    const size_t prob_stride = (size_t)n_img * rb_per_img * c * 2;
    double s1 = 0, s2 = 0;
    if (ch < c) {
        for (int pr = 0; pr < nprob; ++pr) {
            const float* base = part + pr * prob_stride + ((size_t)img * rb_per_img * c + ch) * 2;
#pragma unroll 8
            for (int rb = sl; rb < rb_per_img; rb += 16) {
                const f32x2 q = *reinterpret_cast<const f32x2*>(base + (size_t)rb * c * 2);
                const double m = q[0];
                s1 += 32.0 * m;
                s2 += (double)q[1] + 32.0 * m * m;
            }
        }
    }
    __shared__ double red[256][2];
    red[threadIdx.x][0] = s1;
    red[threadIdx.x][1] = s2;
    __syncthreads();
    if (sl == 0 && ch < c) {
        for (int q = 1; q < 16; ++q) {
            s1 += red[q * 16 + cl][0];
            s2 += red[q * 16 + cl][1];
        }
        const double n = 32.0 * nprob * rb_per_img;
        const double mu = s1 / n;
        double var = s2 / n - mu * mu;
        if (var < 0) var = 0;
        mean[img * c + ch] = (float)mu;
        rstd[img * c + ch] = (float)(1.0 / sqrt(var + (double)eps));
    }
}

}  // namespace

FG_API long long fg_in_partials_workspace_doubles(int n_img, int c) {
    return (long long)n_img * kPartialSplitsMax * c * 2;
}

FG_API int fg_in_stats_partials(const float* partials, int nprob, int n_img, int rb_per_img, int c, float eps,
                                float* mean, float* rstd, double* work, hipStream_t stream) {
    if (!partials || !mean || !rstd || !work || nprob < 1 || nprob > 4 || n_img < 1 || rb_per_img < 1 || c < 1)
        return fg::fail(FG_ERR_INVALID, "fg_in_stats_partials: bad args");
    const int cg = (c + 63) / 64, K = nprob * rb_per_img;
    if (K <= kPartialsDirectK) {
        hipLaunchKernelGGL(in_partials_direct, dim3(n_img, (c + 15) / 16), dim3(256), 0, stream, partials, nprob, n_img,
                           rb_per_img, c, eps, mean, rstd);
        return fg::launched("in_stats_partials");
    }
    // ~1024 blocks over the chip, each thread at least ~4 of the image's 32-row blocks
    const int splits = std::max(1, std::min({kPartialSplitsMax, (1024 + n_img * cg - 1) / (n_img * cg), K / 16}));
    hipLaunchKernelGGL(in_partials_reduce, dim3(n_img, cg, splits), dim3(256), 0, stream, partials, nprob, n_img,
                       rb_per_img, c, splits, work);
    hipLaunchKernelGGL(in_partials_finalize, dim3(n_img, cg), dim3(256), 0, stream, work, nprob, rb_per_img, c, splits,
                       eps, mean, rstd);
    return fg::launched("in_stats_partials");
}

namespace {
int g_in_rows = 1;   // fg_set_in_rows (A/B hook): 1 = row / load-batched forms of the norm passes
int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}
}  // namespace

FG_API int fg_set_in_rows(int on) {
    if (on < 0 || on > 1) return fg::fail(FG_ERR_INVALID, "fg_set_in_rows: %d", on);
    g_in_rows = on;
    return 0;
}

FG_API long long fg_in_workspace_doubles(int n, int c) {
    return (long long)n * c * (MAX_CHUNKS * 3 + 2) + (long long)n * MAX_CHUNKS / 2 + 64;
}
// layout: [stats n*c*MAX_CHUNKS*3][coef n*c*2 floats = n*c doubles][bias partials n*c][max |g'| per (n, chunk):
// n*MAX_CHUNKS floats]

FG_API int fg_in_stats(fg_view src, float eps, float* mean, float* rstd, double* work, hipStream_t stream) {
    if (!ok_view(src) || !mean || !rstd || !work || src.c_alloc % 4 || (NT % (src.c_alloc / 4)) != 0)
        return fg::fail(FG_ERR_INVALID, "fg_in_stats: bad args (C=%d)", src.c_alloc);
    const int chunks = choose_chunks(src.n, (long long)src.h * src.w);
    hipLaunchKernelGGL(in_stats_kernel, dim3(chunks, src.n), dim3(NT), 0, stream, src, chunks, work);
    int e = fg::launched("in_stats");
    if (e) return e;
    hipLaunchKernelGGL(in_finalize_kernel, dim3(src.n, (src.c_alloc + 63) / 64), dim3(64 * FG), 0, stream, src,
                       chunks, work, eps, mean, rstd);
    return fg::launched("in_finalize");
}

namespace {
int in_apply_impl(fg_view src, const float* mean, const float* rstd, int act, fg_view residual, fg_view dst,
                  int pad_mode, float* absmax, float* split_slot, hipStream_t stream, float* ps_ptr = nullptr,
                  float* ps_slot = nullptr, const float* res_amax = nullptr, int splitpix = 0,
                  const HeadArgs* head = nullptr);
int in_bwd_impl(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean, const float* rstd, int act,
                fg_view dst, float* bias_grad, int bias_accumulate, fg_view gsum, double* work, float* absmax,
                float* split_slot, hipStream_t stream, const HeadArgs* head = nullptr);
bool head_ok(const HeadArgs& h, const fg_view& v) {
    return h.w && h.n_out >= 1 && h.n_out <= HEAD_NB && v.c_alloc == HEAD_CI && h.y.ptr && h.y.c_alloc >= h.n_out &&
           h.y.c_alloc <= HEAD_NO && h.y.c_alloc % 4 == 0 && h.y.n == v.n && h.y.h == v.h && h.y.w == v.w &&
           ((uintptr_t)h.y.ptr & 15) == 0 && ((uintptr_t)h.w & 15) == 0;
}
}  // namespace

FG_API int fg_in_apply(fg_view src, const float* mean, const float* rstd, int act, fg_view residual, fg_view dst,
                       int pad_mode, float* absmax, hipStream_t stream) {
    return in_apply_impl(src, mean, rstd, act, residual, dst, pad_mode, absmax, nullptr, stream);
}

FG_API int fg_in_apply_dual(fg_view src, const float* mean, const float* rstd, int act, fg_view residual,
                            const float* residual_absmax, fg_view dst, int pad_mode, float* absmax, float* ps_dst,
                            float* ps_slot, hipStream_t stream) {
    if (!ps_dst || !ps_slot || dst.c_alloc % 8 || NT % (dst.c_alloc / 4) || ((uintptr_t)ps_dst & 31) ||
        (residual.ptr && !residual_absmax))
        return fg::fail(FG_ERR_INVALID, "fg_in_apply_dual: needs ps_dst (32-B aligned), a zeroed ps_slot, C %% 8 == 0, "
                                        "C <= 1024 and the residual's absmax slot (C=%d)", dst.c_alloc);
    return in_apply_impl(src, mean, rstd, act, residual, dst, pad_mode, absmax, nullptr, stream, ps_dst, ps_slot,
                         residual.ptr ? residual_absmax : nullptr);
}

FG_API int fg_in_apply_presplit(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                                float* scale_slot, hipStream_t stream) {
    if (!scale_slot || dst.c_alloc % 8 || NT % (dst.c_alloc / 4) || ((uintptr_t)dst.ptr & 31))
        return fg::fail(FG_ERR_INVALID, "fg_in_apply_presplit: needs a zeroed scale slot, C %% 8 == 0, C <= 1024, "
                                        "a 32-B aligned dst (C=%d)", dst.c_alloc);
    return in_apply_impl(src, mean, rstd, act, fg_view{nullptr, 0, 0, 0, 0, 0}, dst, pad_mode, nullptr, scale_slot,
                         stream);
}

FG_API int fg_in_apply_head(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                             float* absmax, const float* w, const float* b, int n_out, fg_view y, hipStream_t stream) {
    const HeadArgs h{w, b, n_out, y};
    if (!head_ok(h, dst) || dst.pad != 0 || y.pad != 0)
        return fg::fail(FG_ERR_INVALID, "fg_in_apply_head: needs C 64, an unpadded dst, n_out <= 16 logits in a 16-B "
                                        "aligned unpadded view of the same grid (C=%d, pad %d, n_out %d, y.c_alloc %d)",
                        dst.c_alloc, dst.pad, n_out, y.c_alloc);
    return in_apply_impl(src, mean, rstd, act, fg_view{nullptr, 0, 0, 0, 0, 0}, dst, pad_mode, dst.ptr ? absmax : nullptr,
                         nullptr, stream, nullptr, nullptr, nullptr, 0, &h);
}

FG_API int fg_in_head_wgrad_workspace_floats(int n, int h, int w, int n_out) {
    return head_chunks(n, (long long)h * w) * n * n_out * (HEAD_CI + 1);
}

FG_API int fg_in_bwd_head(fg_view gy, const float* w, int n_out, fg_view src, const float* mean, const float* rstd,
                          int act, fg_view dst, float* bias_grad, int bias_accumulate, double* work, float* absmax,
                          float* scale_slot, float* dw, float* db, int wg_accumulate, float* wg_work,
                          hipStream_t stream) {
    HeadArgs h{w, nullptr, n_out, gy};
    if (!head_ok(h, src) || gy.pad != 0 || gy.c_alloc < HEAD_NB ||
        (scale_slot && (dst.c_alloc % 8 || ((uintptr_t)dst.ptr & 31))) || (dw && !wg_work))
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd_head: needs C 64, n_out <= 16 logit gradients in a 16-B aligned "
                                        "unpadded view of the same grid, and a workspace with dw (C=%d, n_out %d, "
                                        "gy.c_alloc %d)", src.c_alloc, n_out, gy.c_alloc);
    if (dw) h.wslab = wg_work;
    // gsrc stands in for the 64-channel gradient the head replaces (its geometry is what the checks read)
    fg_view gs = src;
    gs.pad = 0;
    const int rc = in_bwd_impl(gs, 0, fg_view{nullptr, 0, 0, 0, 0, 0}, src, mean, rstd, act, dst, bias_grad,
                               bias_accumulate, fg_view{nullptr, 0, 0, 0, 0, 0}, work, scale_slot ? nullptr : absmax,
                               scale_slot, stream, &h);
    if (rc || !dw) return rc;
    return fg::conv1x1_wgrad_reduce_launch(wg_work, head_chunks(src.n, (long long)src.h * src.w) * src.n, n_out, dw,
                                           db, wg_accumulate, stream);
}

FG_API int fg_in_apply_splitpix(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                                 float* scale_slot, hipStream_t stream) {
    if (!scale_slot || (dst.c_alloc != 32 && dst.c_alloc != 64) || ((uintptr_t)dst.ptr & 31))
        return fg::fail(FG_ERR_INVALID, "fg_in_apply_splitpix: needs a zeroed scale slot, C 32 or 64, a 32-B aligned dst "
                                        "(C=%d)", dst.c_alloc);
    return in_apply_impl(src, mean, rstd, act, fg_view{nullptr, 0, 0, 0, 0, 0}, dst, pad_mode, nullptr, scale_slot,
                         stream, nullptr, nullptr, nullptr, 1);
}

namespace {
int in_apply_impl(fg_view src, const float* mean, const float* rstd, int act, fg_view residual, fg_view dst,
                  int pad_mode, float* absmax, float* split_slot, hipStream_t stream, float* ps_ptr, float* ps_slot,
                  const float* res_amax, int splitpix, const HeadArgs* head) {
    const bool dst_ok = ok_view(dst) || (head && !dst.ptr && dst.n > 0 && dst.h > 0 && dst.w > 0 && dst.pad == 0);
    if (!ok_view(src) || !dst_ok || !mean || !rstd || src.c_alloc % 4 || dst.c_alloc != src.c_alloc ||
        dst.h != src.h || dst.w != src.w || dst.n != src.n)
        return fg::fail(FG_ERR_INVALID, "fg_in_apply: bad args");
    if (residual.ptr && (residual.c_alloc != src.c_alloc || residual.h != src.h || residual.w != src.w))
        return fg::fail(FG_ERR_INVALID, "fg_in_apply: residual shape");
    if (pad_mode == FG_PAD_REFLECT && (dst.pad >= dst.h || dst.pad >= dst.w))
        return fg::fail(FG_ERR_INVALID, "fg_in_apply: reflect pad too large");
    const int C4 = dst.c_alloc / 4;
    if (head) {
        auto kern = in_nt2_on() ? in_apply_rows_kernel<true, true> : in_apply_rows_kernel<false, true>;
        hipLaunchKernelGGL(kern, dim3(dst.n * (dst.h + 2 * dst.pad)), dim3(NT), 0, stream, src, mean, rstd, act,
                           residual, dst, pad_mode, ilog2(C4), reinterpret_cast<unsigned*>(absmax), split_slot, ps_ptr,
                           ps_slot, res_amax, splitpix, *head);
        return fg::launched("in_apply_rows_head");
    }
    if ((g_in_rows || split_slot || ps_ptr) && NT % C4 == 0) {
        auto kern = in_nt2_on() ? in_apply_rows_kernel<true> : in_apply_rows_kernel<false>;
        hipLaunchKernelGGL(kern, dim3(dst.n * (dst.h + 2 * dst.pad)), dim3(NT), 0, stream, src, mean,
                           rstd, act, residual, dst, pad_mode, ilog2(C4), reinterpret_cast<unsigned*>(absmax),
                           split_slot, ps_ptr, ps_slot, res_amax, splitpix, HeadArgs{});
        return fg::launched("in_apply_rows");
    }
    const long long total = (long long)dst.n * (dst.h + 2 * dst.pad) * (dst.w + 2 * dst.pad) * (dst.c_alloc / 4);
    hipLaunchKernelGGL(in_apply_kernel, dim3(fg::blocks_for(total, 256, 4096)), dim3(256), 0, stream, src, mean,
                       rstd, act, residual, dst, pad_mode, reinterpret_cast<unsigned*>(absmax));
    return fg::launched("in_apply");
}
}  // namespace

FG_API int fg_in_bwd(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean, const float* rstd,
                     int act, fg_view dst, float* bias_grad, int bias_accumulate, fg_view gsum, double* work,
                     float* absmax, hipStream_t stream) {
    return in_bwd_impl(gsrc, fold_pad, gadd, src, mean, rstd, act, dst, bias_grad, bias_accumulate, gsum, work, absmax,
                       nullptr, stream);
}

FG_API int fg_in_bwd_presplit(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean,
                              const float* rstd, int act, fg_view dst, float* bias_grad, int bias_accumulate,
                              fg_view gsum, double* work, float* scale_slot, hipStream_t stream) {
    if (!scale_slot || dst.c_alloc % 8 || ((uintptr_t)dst.ptr & 31))
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd_presplit: needs a zeroed scale slot, C %% 8 == 0, a 32-B aligned "
                                        "dst (C=%d)", dst.c_alloc);
    return in_bwd_impl(gsrc, fold_pad, gadd, src, mean, rstd, act, dst, bias_grad, bias_accumulate, gsum, work, nullptr,
                       scale_slot, stream);
}

namespace {
int in_bwd_impl(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean, const float* rstd, int act,
                fg_view dst, float* bias_grad, int bias_accumulate, fg_view gsum, double* work, float* absmax,
                float* split_slot, hipStream_t stream, const HeadArgs* head) {
    if (!ok_view(gsrc) || !ok_view(src) || !ok_view(dst) || !mean || !rstd || !work || src.c_alloc % 4 ||
        (NT % (src.c_alloc / 4)) != 0 || gsrc.c_alloc != src.c_alloc || dst.c_alloc != src.c_alloc ||
        dst.h != src.h || dst.w != src.w || dst.n != src.n)
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd: bad args");
    if (gsrc.h != src.h + 2 * fold_pad || gsrc.w != src.w + 2 * fold_pad || fold_pad < 0 || fold_pad >= src.h ||
        fold_pad >= src.w)
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd: gsrc %dx%d vs src %dx%d fold %d", gsrc.h, gsrc.w, src.h, src.w,
                        fold_pad);
    if (gadd.ptr && (gadd.c_alloc != src.c_alloc || gadd.h != src.h || gadd.w != src.w))
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd: gadd shape");
    if (gsum.ptr && (gsum.c_alloc != src.c_alloc || gsum.h != src.h || gsum.w != src.w || gsum.n != src.n))
        return fg::fail(FG_ERR_INVALID, "fg_in_bwd: gsum shape");
    // ~2048 workgroups (measured against 1024 / 512 / 256 / 128 at bs 8: 512 within noise, fewer slower,
    // profiles/round3/r3ai_bwd_wg.log; round 5, interleaved in one process: 512 for a 4x smaller finalize read is
    // 0.12 ms slower per step, profiles/round5/r5n_ab_in_bwd_wg_not_kept.log)
    const int chunks = head ? head_chunks(src.n, (long long)src.h * src.w) : choose_chunks(src.n, (long long)src.h * src.w);
    const int C = src.c_alloc;
    float* coef = reinterpret_cast<float*>(work + (size_t)src.n * C * MAX_CHUNKS * 3);
    double* bpart = work + (size_t)src.n * C * MAX_CHUNKS * 3 + (size_t)src.n * C;
    float* gmax_part = split_slot ? reinterpret_cast<float*>(bpart + (size_t)src.n * C) : nullptr;
    static const bool nt_env = [] { const char* e = getenv("FLOODGAN_IN_NT"); return !e || atoi(e) != 0; }();
    const bool ntg = gsum.ptr && nt_env;
    if (head)
        hipLaunchKernelGGL((in_bwd_stats_u_kernel<false, true>), dim3(chunks, src.n), dim3(NT), 0, stream, gsrc, 0, gadd,
                           src, mean, rstd, act, chunks, work, gsum, gmax_part, *head);
    else if ((g_in_rows || split_slot) && ntg)
        hipLaunchKernelGGL(in_bwd_stats_u_kernel<true>, dim3(chunks, src.n), dim3(NT), 0, stream, gsrc, fold_pad, gadd,
                           src, mean, rstd, act, chunks, work, gsum, gmax_part, HeadArgs{});
    else if (g_in_rows || split_slot)
        hipLaunchKernelGGL(in_bwd_stats_u_kernel<false>, dim3(chunks, src.n), dim3(NT), 0, stream, gsrc, fold_pad, gadd,
                           src, mean, rstd, act, chunks, work, gsum, gmax_part, HeadArgs{});
    else
        hipLaunchKernelGGL(in_bwd_stats_kernel, dim3(chunks, src.n), dim3(NT), 0, stream, gsrc, fold_pad, gadd, src,
                           mean, rstd, act, chunks, work, gsum);
    int e = fg::launched("in_bwd_stats");
    if (e) return e;
    hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3(src.n, (C + kFinC - 1) / kFinC), dim3(kFinC * kFinS), 0, stream, src.n, C,
                       src.h * src.w, chunks, work, rstd, coef, bpart, gmax_part, split_slot);
    e = fg::launched("in_bwd_finalize");
    if (e) return e;
    const long long total = (long long)dst.n * (dst.h + 2 * dst.pad) * (dst.w + 2 * dst.pad) * (C / 4);
    // with gsum the apply pass reads the gathered gradient the statistics pass wrote (one read, no fold)
    const fg_view none = {nullptr, 0, 0, 0, 0, 0};
    if (head) {
        auto kern = in_nt2_on() ? in_bwd_apply_rows_kernel<true, true> : in_bwd_apply_rows_kernel<false, true>;
        hipLaunchKernelGGL(kern, dim3(dst.n * (dst.h + 2 * dst.pad)), dim3(NT), 0, stream, gsrc, 0, none, src, mean,
                           rstd, coef, act, dst, reinterpret_cast<unsigned*>(absmax), bpart, bias_grad,
                           bias_accumulate, ilog2(C / 4), split_slot, *head);
        return fg::launched("in_bwd_apply_rows_head");
    }
    if (g_in_rows || split_slot) {
        auto kern = in_nt2_on() ? in_bwd_apply_rows_kernel<true> : in_bwd_apply_rows_kernel<false>;
        hipLaunchKernelGGL(kern, dim3(dst.n * (dst.h + 2 * dst.pad)), dim3(NT), 0, stream,
                           gsum.ptr ? gsum : gsrc, gsum.ptr ? 0 : fold_pad, gsum.ptr ? none : gadd, src, mean, rstd,
                           coef, act, dst, reinterpret_cast<unsigned*>(absmax), bpart, bias_grad, bias_accumulate,
                           ilog2(C / 4), split_slot, HeadArgs{});
        return fg::launched("in_bwd_apply_rows");
    }
    hipLaunchKernelGGL(in_bwd_apply_kernel, dim3(fg::blocks_for(total, 256, 4096)), dim3(256), 0, stream,
                       gsum.ptr ? gsum : gsrc, gsum.ptr ? 0 : fold_pad, gsum.ptr ? none : gadd, src, mean, rstd, coef,
                       act, dst, reinterpret_cast<unsigned*>(absmax), bpart, bias_grad, bias_accumulate);
    return fg::launched("in_bwd_apply");
}
}  // namespace

FG_API int fg_act_bwd(fg_view g, fg_view y, int act, float* absmax, hipStream_t stream) {
    unsigned* am = reinterpret_cast<unsigned*>(absmax);
    if (!ok_view(g) || !ok_view(y) || g.c_alloc != y.c_alloc || g.h != y.h || g.w != y.w || g.n != y.n)
        return fg::fail(FG_ERR_INVALID, "fg_act_bwd: bad args");
    if (g.c_alloc % 4 == 0) {
        hipLaunchKernelGGL(act_bwd4_kernel, dim3(g.n * g.h), dim3(256), 0, stream, g, y, act, am);
        return fg::launched("act_bwd4");
    }
    const long long total = (long long)g.n * g.h * g.w * g.c_alloc;
    hipLaunchKernelGGL(act_bwd_kernel, dim3(fg::blocks_for(total, 256, 16384)), dim3(256), 0, stream, g, y, act, am);
    return fg::launched("act_bwd");
}

FG_API long long fg_channel_sum_workspace_doubles(int c_alloc) {
    return (long long)std::max(CS_CHUNKS, MAX_CHUNKS) * c_alloc + 64;
}

FG_API int fg_channel_sum(fg_view src, int c_valid, float* out, int accumulate, double* work, hipStream_t stream) {
    if (!ok_view(src) || !out || !work || c_valid < 1 || c_valid > src.c_alloc)
        return fg::fail(FG_ERR_INVALID, "fg_channel_sum: bad args");
    const long long P = (long long)src.n * src.h * src.w;
    if (src.c_alloc % 4 == 0 && NT % (src.c_alloc / 4) == 0) {
        // ~2048 pixels per block, at most CS_CHUNKS blocks (the workspace bound)
        int chunks = (int)std::min<long long>(CS_CHUNKS, std::max<long long>(1, (P + 2047) / 2048));
        hipLaunchKernelGGL(channel_sum4_kernel, dim3(chunks), dim3(NT), 0, stream, src, chunks, work);
        int e = fg::launched("channel_sum4");
        if (e) return e;
        hipLaunchKernelGGL(channel_sum4_finalize, dim3(c_valid), dim3(256), 0, stream, src.c_alloc, c_valid, chunks,
                           work, out, accumulate);
        return fg::launched("channel_sum4_finalize");
    }
    int chunks = (int)((P + 4095) / 4096);
    if (chunks > MAX_CHUNKS) chunks = MAX_CHUNKS;
    if (chunks < 1) chunks = 1;
    const int groups = (c_valid + NT - 1) / NT;
    hipLaunchKernelGGL(channel_sum_kernel, dim3(chunks, groups), dim3(NT), 0, stream, src, c_valid, chunks, work);
    int e = fg::launched("channel_sum");
    if (e) return e;
    hipLaunchKernelGGL(channel_sum_finalize, dim3((c_valid + 255) / 256), dim3(256), 0, stream, c_valid, chunks,
                       work, out, accumulate);
    return fg::launched("channel_sum_finalize");
}
