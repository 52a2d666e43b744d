// Row-strip ("window") f16x3 convolution for the narrow stride-1 convs with wide kernels:
// deconv3_content (7x7, 64 -> 27, models/model_architectures.py:328, :352) and its input
// gradient (7x7, 27(32) -> 64).  At N <= 64 the im2col formulation of conv_gemm.hip / conv_f3.hip
// re-gathers every input pixel kw times per output row and splits it each time: the content
// head ran at ~130 TFLOP/s (profiles/round1/r1f_kernel_stats.csv).  Here one workgroup owns 256
// consecutive output pixels (at most two output-row segments) and, per kernel row r, stages the
// input strip those pixels read -- (256 + 2(kw-1)) pixels x C channels, once -- then runs the kw
// taps as shifted reads of the same strip.
//
// The strip comes from a pre-split copy of the input (fg_split_pixels: per pixel the fp16 pieces
// h[C] and l[C] of the scaled fp32 values, 16-B chunks XOR-swizzled by the pixel's column so the
// shifted fragment reads are bank-conflict free) and the kernel row's KW taps of weights from the
// fg_pack_weight_f16 layout; both sit in LDS together.  Each kind runs on two 4-wave workgroups per
// CU that walk a kernel row per phase (conv_win2_kernel / conv_win2_dgrad_kernel below); round 4's
// one-workgroup-per-CU 8-wave form (1.21 / 1.13 ms forward / input gradient, profiles/round4/r4c_ab_win.log)
// was replaced by them (1.08 / 0.95 ms) and removed in round 5.
#include "conv_common.hpp"

namespace {

// chunk swizzles (exhaustive search over the ds_read_b128 lane groups and every row offset):
// strip pixels use fgc::swz_pixel (the layout fg_split_pixels writes), weight rows this one
template <int C>
__device__ __forceinline__ int swz_strip(int x) { return fgc::swz_pixel<C>(x); }
template <int C>
__device__ __forceinline__ int swz_wrow(int n) {         // weight image row n
    if constexpr (C == 64) return (n >> 1) & 7;          // 8 chunks per 128-B row
    else return ((n >> 3) & 1) << 1;                     // 4 chunks per 64-B row
}

// f16x3 pieces of the scaled input: dst pixel p (column x = p % wp) = 2C fp16, chunk k of the
// [h | l] pixel row stored at chunk k ^ swz_strip(x).  One thread per 8 channels of a pixel.
template <int C>
__global__ void split_pixels_kernel(const float* __restrict__ src, long long npix, int wp, const float* amax,
                                    f16x8* __restrict__ dst) {
    constexpr int Q = C / 8;
    const float s = fgc::pow2_scale(amax);
    const long long total = npix * Q;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long p = idx / Q;
        const int q = (int)(idx - p * Q);
        const f32x4 v0 = reinterpret_cast<const f32x4*>(src)[idx * 2];
        const f32x4 v1 = reinterpret_cast<const f32x4*>(src)[idx * 2 + 1];
        const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        f16x8 h, l;
        fgc::split_f16(v, s, h, l);
        const int sw = swz_strip<C>((int)(p % wp));
        dst[p * 2 * Q + (q ^ sw)] = h;
        dst[p * 2 * Q + ((Q + q) ^ sw)] = l;
    }
}

struct WinArgs {
    fg_conv_problem P;
    const char* xs;     // split input at the problem's x origin (pixel (0,0) of image 0's padded grid)
    int wp;             // pixels per padded input row (= sxr / C)
    int tiles_per_img;
};

typedef __attribute__((address_space(3))) void lds_void;

// nothing is scheduled across it
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
// one 16-B LDS-DMA per lane: lane i's bytes land at lds + 16 i (lds wave-uniform).  A device function: the builtin
// named in a lambda of the forward kernel's body left that kernel's host-side launch stub undefined.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// C = 64 forward, two workgroups per CU: a workgroup of 4 waves x 64 rows walks 14 "phases" -- one kernel row's
// 32-channel half each: the strip's half pixels (268 px x 128 B, in the 32-channel chunk swizzle) and that half of
// the row's 7 taps of weights (28 KB), 63 KB of LDS -- so two workgroups share a CU and one's copy / barriers run
// under the other's MFMAs (round 4's 8-wave kernel held 123 KB: one workgroup per CU, every wave idle during each
// row's copy; removed in round 5).  A phase's operands arrive by LDS-DMA (16-B buffer loads straight into LDS; the other workgroup's
// MFMAs cover the latency), and the registers that frees hold the next tap's fragments, read ahead of the current
// tap's MFMAs (sched_barrier keeps that order).  Per tap and wave: 8 A + 4 B fragment reads for 24 MFMAs (512 LDS
// bytes per MFMA, was 683).  Register-staged copies instead of DMA, without the read-ahead: 1.5-2.5 % slower
// (profiles/round4/r4ze_bench_win.log).
template <int KW>
__global__ void __launch_bounds__(256, 2) conv_win2_kernel(const WinArgs args) {
    constexpr int C = 64, CH = 32, NT = 256, BM = 256, TN = 2, TM = 4, WM = 64;
    constexpr int PB = 2 * CH * 2;                              // LDS strip bytes per pixel: h | l of the half
    constexpr int NR = TN * 16;
    constexpr int STRIP_PIX = BM + 2 * (KW - 1);
    constexpr int STRIP_CH = STRIP_PIX * PB / 16;               // 16-B chunks
    constexpr int SCH = (STRIP_CH + NT - 1) / NT;
    constexpr int W_TAP = 2 * NR * CH * 2;                      // [pc][NR][CH] fp16 per tap
    constexpr int TAP_CH = W_TAP / 16;
    constexpr int W_CH = KW * TAP_CH;
    constexpr int WCH = (W_CH + NT - 1) / NT;
    constexpr int W_OFF = (STRIP_PIX * PB + 1023) / 1024 * 1024;
    __shared__ __attribute__((aligned(1024))) char smem[W_OFF + KW * W_TAP];

    const fg_conv_problem& P = args.P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int img = wid / args.tiles_per_img;
    const int p0 = (wid - img * args.tiles_per_img) * BM;
    const int mab = P.m_a * P.m_b;
    const int a0 = p0 / P.m_b, b0 = p0 - (p0 / P.m_b) * P.m_b;
    const int len0 = min(BM, min(P.m_b - b0, mab - p0));
    const int len1 = (a0 + 1 < P.m_a) ? min(BM - len0, P.m_b) : 0;
    const int s0pix = len0 + KW - 1;
    const int npix = len0 + len1 + 2 * (KW - 1);
    const int wp = args.wp;
    constexpr int kOOB = 0x7fffffff;

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)args.xs, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);

    // LDS strip chunk o (pixel q = o / 8, slot j): slot j holds the half's logical chunk L = j ^ swz_pixel<32>(x)
    // (0..3: h of channels 8L.., 4..7: l), which sits in the 64-channel split pixel at chunk g ^ swz_pixel<64>(x),
    // g = 4 hc + L (h) or 8 + 4 hc + L - 4 (l)
    const int seg0_pix = img * (int)(P.sxn / C) + a0 * wp + b0;
    const int seg1_pix = img * (int)(P.sxn / C) + (a0 + 1) * wp;
    int s_src0[SCH], s_src1[SCH];
#pragma unroll
    for (int i = 0; i < SCH; ++i) {
        const int o = tid + i * NT, q = o >> 3, j = o & 7;
        const bool live = o < STRIP_CH && q < npix;
        const int x = q < s0pix ? b0 + q : q - s0pix;          // padded column of the strip pixel
        const int pix = q < s0pix ? seg0_pix + q : seg1_pix + (q - s0pix);
        const int L = j ^ fgc::swz_pixel<CH>(x);
        const int sw = fgc::swz_pixel<C>(x);
        const int g0 = L < 4 ? L : 4 + L, g1 = g0 + 4;          // logical chunk in half 0 / half 1
        s_src0[i] = live ? pix * (4 * C) + ((g0 ^ sw) << 4) : -1;
        s_src1[i] = live ? pix * (4 * C) + ((g1 ^ sw) << 4) : -1;
    }
    // weight chunk F of the half-row image [s][pc][NR][CH] (chunk slots swizzled as swz_wrow<32>)
    int w_src[WCH];
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
        const int F = tid + i * NT, s = F / TAP_CH, f = F - s * TAP_CH;
        const int pc = f / (NR * CH / 8);
        const int rem = f - pc * (NR * CH / 8);
        const int n = rem / (CH / 8);
        const int ch = (rem - n * (CH / 8)) ^ swz_wrow<CH>(n);
        w_src[i] = F >= W_CH ? -1 : (min(n, P.n_out - 1) * (P.ldw / 8) + ch) * 32 + pc * 16 + ((s * C) / 8) * 32;
    }
    const float sa = fgc::pow2_scale(P.x_absmax);
    const float sb = fgc::pow2_scale(P.w_absmax);
    const float out_scale = 1.f / (sa * sb);

    const int fr = lane & 15, g = lane >> 4;
    int q0[TM], x0[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int i = wave * WM + tm * 16 + fr;
        q0[tm] = i < len0 ? i : i + KW - 1;
        x0[tm] = i < len0 ? b0 + i : i - len0;
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct Frags {
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
    };
    auto read = [&](int s, Frags& f) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const char* px = smem + (q0[tm] + s) * PB;
            const int sw = fgc::swz_pixel<CH>(x0[tm] + s);
            f.ah[tm] = *reinterpret_cast<const f16x8*>(px + (g ^ sw) * 16);
            f.al[tm] = *reinterpret_cast<const f16x8*>(px + ((4 + g) ^ sw) * 16);
        }
        const char* wb = smem + W_OFF + s * W_TAP;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = tn * 16 + fr;
            const char* row = wb + n * (2 * CH) + (g ^ swz_wrow<CH>(n)) * 16;
            f.bh[tn] = *reinterpret_cast<const f16x8*>(row);
            f.bl[tn] = *reinterpret_cast<const f16x8*>(row + NR * 2 * CH);
        }
    };
    auto mma = [&](const Frags& f) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.al[tm], f.bh[tn], acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.ah[tm], f.bl[tn], acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.ah[tm], f.bh[tn], acc[tm][tn], 0, 0, 0);
            }
    };

    const int NPH = 2 * P.kh;
    auto dma = [&](int ph) {
        const int r = ph >> 1, hc = ph & 1;
        const int soff = r * wp * (4 * C), woff = ((r * P.jp) / 8) * 32 + hc * (CH / 8) * 32;
#pragma unroll
        for (int i = 0; i < SCH; ++i) {
            const int ob = i * NT + wave * 64;
            if (ob >= STRIP_CH) continue;
            const int src = hc ? s_src1[i] : s_src0[i];
            dma16(xr, smem + ob * 16, src >= 0 ? src + soff : kOOB);
        }
#pragma unroll
        for (int i = 0; i < WCH; ++i) {
            const int ob = i * NT + wave * 64;
            if (ob >= W_CH) continue;
            dma16(wr, smem + W_OFF + ob * 16, w_src[i] >= 0 ? w_src[i] + woff : kOOB);
        }
    };
    for (int ph = 0; ph < NPH; ++ph) {
        if (ph) __syncthreads();
        dma(ph);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        Frags fa, fb;
        read(0, fa);
#pragma unroll
        for (int s = 0; s < KW; s += 2) {
            if (s + 1 < KW) read(s + 1, fb);
            sched_fence();
            mma(fa);
            sched_fence();
            if (s + 1 < KW) {
                if (s + 2 < KW) read(s + 2, fa);
                sched_fence();
                mma(fb);
                sched_fence();
            }
        }
    }

    // ---- epilogue: scale, bias, activation, optional accumulate
    const int act = P.act;
    const bool accum = P.accumulate != 0;
    float bias_v[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias_v[tn] = P.bias ? P.bias[min(tn * 16 + fr, P.n_out - 1)] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int i = wave * WM + tm * 16 + 4 * g + reg;
            if (i >= len0 + len1) continue;
            const int a = i < len0 ? a0 : a0 + 1, b = i < len0 ? b0 + i : i - len0;
            float* yrow = P.y + img * P.syn + a * P.sya + b * P.syb;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = tn * 16 + fr;
                if (n >= P.n_out) continue;
                float v = fg::act_fwd(acc[tm][tn][reg] * out_scale + bias_v[tn], act);
                float* dst = yrow + n * P.syc;
                if (accum) v += *dst;
                *dst = v;
            }
        }
    }
}

// C = 32 (the content head's input gradient, N <= 64), two workgroups per CU: 4 waves x 64 rows x 64 outputs per
// workgroup of 256 output pixels.  Each kernel row runs as two phases that share one staged strip (268 px x 128 B):
// the weights of taps 0..3, then of taps 4..6 (32 / 24 KB), so a workgroup holds 66 KB of LDS and two share a CU.
// Operands arrive by LDS-DMA (16-B buffer loads into LDS, no staging registers: the accumulators and fragments
// need them); one workgroup's copy latency and barriers run under the other's MFMAs.  Per tap and wave: 8 A + 8 B
// fragment reads for 48 MFMAs (341 LDS bytes per MFMA, as the 8-wave 512-row kernel).
template <int KW>
__global__ void __launch_bounds__(256, 2) conv_win2_dgrad_kernel(const WinArgs args) {
    constexpr int C = 32, NT = 256, BM = 256, TN = 4, TM = 4, WM = 64;
    constexpr int PB = 4 * C;                                   // strip bytes per pixel (h | l)
    constexpr int NR = TN * 16;
    constexpr int STRIP_PIX = BM + 2 * (KW - 1);
    constexpr int STRIP_CH = STRIP_PIX * PB / 16;
    constexpr int W_TAP = 2 * NR * C * 2;                       // [pc][NR][C] fp16 per tap
    constexpr int TAP_CH = W_TAP / 16;
    constexpr int G0 = (KW + 1) / 2;                            // taps of the first phase
    constexpr int W_OFF = (STRIP_PIX * PB + 1023) / 1024 * 1024;
    __shared__ __attribute__((aligned(1024))) char smem[W_OFF + G0 * W_TAP];
    static_assert((G0 * TAP_CH) % NT == 0 && ((KW - G0) * TAP_CH) % NT == 0, "weight phases are whole wave copies");

    const fg_conv_problem& P = args.P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int img = wid / args.tiles_per_img;
    const int p0 = (wid - img * args.tiles_per_img) * BM;
    const int mab = P.m_a * P.m_b;
    const int a0 = p0 / P.m_b, b0 = p0 - (p0 / P.m_b) * P.m_b;
    const int len0 = min(BM, min(P.m_b - b0, mab - p0));
    const int len1 = (a0 + 1 < P.m_a) ? min(BM - len0, P.m_b) : 0;
    const int s0pix = len0 + KW - 1;
    const int strip_bytes = (len0 + len1 + 2 * (KW - 1)) * PB;
    const int wp = args.wp;
    constexpr int kOOB = 0x7fffffff;

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)args.xs, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);
    const int seg0_pix = img * (int)(P.sxn / C) + a0 * wp + b0;
    const int seg1_pix = img * (int)(P.sxn / C) + (a0 + 1) * wp;

    // strip: wave-instruction i of this wave copies chunks o = (i*4 + wave)*64 + lane (waves whose chunks start past
    // the strip skip it; a partial one ends inside the pad before W_OFF)
    auto dma_strip = [&](int r) {
        const int soff = r * wp * PB;
#pragma unroll
        for (int i = 0; i < (STRIP_CH + NT - 1) / NT; ++i) {
            const int ob = (i * 4 + wave) * 64;
            if (ob >= STRIP_CH) continue;
            const int o = (ob + lane) * 16;
            const int src = o >= strip_bytes ? kOOB : (o < s0pix * PB ? seg0_pix * PB + o : seg1_pix * PB + (o - s0pix * PB)) + soff;
            dma16(xr, smem + ob * 16, src);
        }
    };
    // weights of taps t0 .. t0 + nt - 1 of kernel row r: chunk F of the image [s][pc][NR][C]
    auto dma_w = [&](int r, int t0, int nt) {
        const int woff = ((r * P.jp) / 8) * 32;
        for (int i = 0; i < nt * TAP_CH / NT; ++i) {
            const int Fb = (i * 4 + wave) * 64, F = Fb + lane;
            const int sl = F / TAP_CH, f = F - sl * TAP_CH;
            const int pc = f / (NR * C / 8);
            const int rem = f - pc * (NR * C / 8);
            const int n = rem / (C / 8);
            const int ch = (rem - n * (C / 8)) ^ swz_wrow<C>(n);
            const int src = (min(n, P.n_out - 1) * (P.ldw / 8) + ch) * 32 + pc * 16 + (((t0 + sl) * C) / 8) * 32 + woff;
            dma16(wr, smem + W_OFF + Fb * 16, src);
        }
    };

    const float sa = fgc::pow2_scale(P.x_absmax);
    const float sb = fgc::pow2_scale(P.w_absmax);
    const float out_scale = 1.f / (sa * sb);

    const int fr = lane & 15, g = lane >> 4;
    int q0[TM], x0[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int i = wave * WM + tm * 16 + fr;
        q0[tm] = i < len0 ? i : i + KW - 1;
        x0[tm] = i < len0 ? b0 + i : i - len0;
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};

    // tap s of the strip with the staged weight slot sl
    auto tap = [&](int s, int sl) {
        f16x8 ah[TM], al[TM];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const char* px = smem + (q0[tm] + s) * PB;
            const int sw = swz_strip<C>(x0[tm] + s);
            ah[tm] = *reinterpret_cast<const f16x8*>(px + (g ^ sw) * 16);
            al[tm] = *reinterpret_cast<const f16x8*>(px + ((C / 8 + g) ^ sw) * 16);
        }
        const char* wb = smem + W_OFF + sl * W_TAP;
        f16x8 bh[TN], bl[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = tn * 16 + fr;
            const char* row = wb + n * (2 * C) + (g ^ swz_wrow<C>(n)) * 16;
            bh[tn] = *reinterpret_cast<const f16x8*>(row);
            bl[tn] = *reinterpret_cast<const f16x8*>(row + NR * 2 * C);
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[tm], bh[tn], acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[tm], bl[tn], acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[tm], bh[tn], acc[tm][tn], 0, 0, 0);
            }
    };

    for (int r = 0; r < P.kh; ++r) {
        __syncthreads();                              // the previous phase's reads are done
        dma_strip(r);
        dma_w(r, 0, G0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int s = 0; s < G0; ++s) tap(s, s);
        __syncthreads();
        dma_w(r, G0, KW - G0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int s = G0; s < KW; ++s) tap(s, s - G0);
    }

    // ---- epilogue: scale, bias, activation, optional accumulate
    const int act = P.act;
    const bool accum = P.accumulate != 0;
    float bias_v[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias_v[tn] = P.bias ? P.bias[min(tn * 16 + fr, P.n_out - 1)] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int i = wave * WM + tm * 16 + 4 * g + reg;
            if (i >= len0 + len1) continue;
            const int a = i < len0 ? a0 : a0 + 1, b = i < len0 ? b0 + i : i - len0;
            float* yrow = P.y + img * P.syn + a * P.sya + b * P.syb;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = tn * 16 + fr;
                if (n >= P.n_out) continue;
                float v = fg::act_fwd(acc[tm][tn][reg] * out_scale + bias_v[tn], act);
                float* dst = yrow + n * P.syc;
                if (accum) v += *dst;
                *dst = v;
            }
        }
    }
}

// the forward (C 64) and the input gradient (C 32) each on two 4-wave workgroups per CU: forward 1201 -> 1078 us
// (profiles/round4/r4z_bench_win.log), input gradient 1071 -> 952 us (r4zb_bench_win.log) against round 4's 8-wave
// kernels, which were removed in round 5 with their FLOODGAN_WIN_2WG / FLOODGAN_WIN_BM switches
template <int C, int KW>
int launch_win(const WinArgs& a, int tiles, hipStream_t stream) {
    if constexpr (C == 32) {
        hipLaunchKernelGGL((conv_win2_dgrad_kernel<KW>), dim3(tiles), dim3(256), 0, stream, a);
        return fg::launched("conv_win2_dgrad");
    } else {
        hipLaunchKernelGGL((conv_win2_kernel<KW>), dim3(tiles), dim3(256), 0, stream, a);
        return fg::launched("conv_win2");
    }
}

}  // namespace

FG_API int fg_split_pixels(const float* src, long long npix, int c, int wp, const float* amax, void* dst,
                           hipStream_t stream) {
    if (!src || !dst || !amax || npix < 0 || wp < 1 || (c != 32 && c != 64) || ((uintptr_t)src & 15) ||
        ((uintptr_t)dst & 15))
        return fg::fail(FG_ERR_INVALID, "fg_split_pixels: bad args (c=%d wp=%d)", c, wp);
    if (npix == 0) return 0;
    const long long work = npix * (c / 8);
    const int blocks = fg::blocks_for(work, 256, 16384);
    if (c == 64)
        hipLaunchKernelGGL(split_pixels_kernel<64>, dim3(blocks), dim3(256), 0, stream, src, npix, wp, amax,
                           reinterpret_cast<f16x8*>(dst));
    else
        hipLaunchKernelGGL(split_pixels_kernel<32>, dim3(blocks), dim3(256), 0, stream, src, npix, wp, amax,
                           reinterpret_cast<f16x8*>(dst));
    return fg::launched("split_pixels");
}

FG_API int fg_conv_win(const fg_conv_problem* prob, const void* x_split, long long x_pix0, hipStream_t stream) {
    if (!prob || !x_split || !prob->w || !prob->y || !prob->x_absmax || !prob->w_absmax)
        return fg::fail(FG_ERR_INVALID, "fg_conv_win: null argument");
    const fg_conv_problem& p = *prob;
    const int C = (int)p.sxb;
    const int kw = C > 0 ? p.j_valid / C : 0;
    if ((C != 32 && C != 64) || p.sxa != p.sxr || p.sxr % C || p.sxn % C || kw != 7 || p.kh != 7 ||
        p.j_valid != kw * C || p.jp != p.j_valid || p.ldw != p.kh * p.jp || p.w_split != 2 || p.n_out < 1 ||
        p.n_out > (C == 64 ? 32 : 64) || p.m_b < 256 || p.m_a < 1 || p.m_img < 1 || x_pix0 < 0 ||
        x_pix0 % (p.sxr / C))
        return fg::fail(FG_ERR_INVALID,
                        "fg_conv_win: unsupported geometry (C=%d kw=%d kh=%d n=%d m_b=%d): stride-1 7x7, C 32/64, "
                        "n_out <= 32 (C 64) / 64 (C 32), output rows >= 256 px, origin at a padded-row start",
                        C, kw, p.kh, p.n_out, p.m_b);
    const long long wp = p.sxr / C;
    const long long span = x_pix0 + (long long)(p.m_img - 1) * (p.sxn / C) + (p.m_a + 6) * wp + 4 * C;
    if (span * 4 * C >= (1LL << 31) - 4096)
        return fg::fail(FG_ERR_INVALID, "fg_conv_win: split operand beyond 2 GiB");
    WinArgs a;
    a.P = p;
    a.xs = reinterpret_cast<const char*>(x_split) + x_pix0 * 4 * C;
    a.wp = (int)wp;
    a.tiles_per_img = (p.m_a * p.m_b + 255) / 256;
    const int tiles = a.tiles_per_img * p.m_img;
    if (C == 64) return launch_win<64, 7>(a, tiles, stream);
    return launch_win<32, 7>(a, tiles, stream);
}
