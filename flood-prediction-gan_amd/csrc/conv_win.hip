// Row-strip ("window") f16x3 convolution for the narrow stride-1 convs with wide kernels:
// deconv3_content (7x7, 64 -> 27, models/model_architectures.py:328, :352) and its input
// gradient (7x7, 27(32) -> 64).  At N <= 64 the im2col formulation of conv_gemm.hip / conv_f3.hip
// re-gathers every input pixel kw times per output row and splits it each time: the content
// head ran at ~130 TFLOP/s (profiles/round1/r1f_kernel_stats.csv).  Here one workgroup owns 256
// consecutive output pixels (at most two output-row segments) and, per kernel row r, stages the
// input strip those pixels read -- (256 + 2(kw-1)) pixels x C channels, once -- then runs the kw
// taps as shifted reads of the same strip.
//
// The strip arrives by LDS-DMA from a pre-split copy of the input (fg_split_pixels: per pixel the
// fp16 pieces h[C] and l[C] of the scaled fp32 values, 16-B chunks XOR-swizzled by the pixel's
// column so the shifted fragment reads are bank-conflict free); the weights of each (r, s) tap
// arrive by LDS-DMA from the fg_pack_weight_f16 layout into a double buffer.  One barrier per
// tap; DMAs are counted by hand (vmcnt) so the next strip streams in behind five taps of MFMAs.
#include "conv_common.hpp"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

// one 1-KiB LDS-DMA piece (kept out of lambdas: hipcc drops the host stub of a kernel whose
// lambdas call this builtin directly)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, soff, 0, 0);
}

// chunk swizzles (exhaustive search over the ds_read_b128 lane groups and every row offset):
// strip pixels use fgc::swz_pixel (the layout fg_split_pixels writes), weight rows this one
template <int C>
__device__ __forceinline__ int swz_strip(int x) { return fgc::swz_pixel<C>(x); }
template <int C>
__device__ __forceinline__ int swz_wrow(int n) {         // weight image row n
    if constexpr (C == 64) return (n >> 1) & 7;          // 8 chunks per 128-B row
    else return ((n >> 3) & 1) << 1;                     // 4 chunks per 64-B row
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else static_assert(N < 0, "add the vmcnt immediate");
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

int g_win_waves = 8;   // FLOODGAN_WIN_WAVES overrides (A/B)
// strip fragments of tap t+1 read before tap t+1's barrier: -1 = for C 32 only (input gradient 1372 -> 1326 us;
// the C 64 forward, which holds twice the fragments across the barrier, 1318 -> 1360 us:
// profiles/round3/r3ap_win_apf.log); FLOODGAN_WIN_APF 0/1 overrides (A/B)
int g_win_apf = -1;

struct WinArgs {
    fg_conv_problem P;
    const char* xs;     // split input at the problem's x origin (pixel (0,0) of image 0's padded grid)
    int wp;             // pixels per padded input row (= sxr / C)
    int tiles_per_img;
};

// APF: the strip fragments of the next tap of the same kernel row are read from LDS right after this
// tap's MFMAs, so their latency runs under the next barrier instead of after it (only the weight
// fragments, whose DMA the barrier publishes, are read behind it)
template <int C, int KW, int TN, int NW = 4, bool APF = false>
__global__ void __launch_bounds__(NW * 64, 1) conv_win_kernel(const WinArgs args) {
    constexpr int BM = 256, WM = BM / NW, TM = WM / 16;
    constexpr int PB = 4 * C;                                   // strip bytes per pixel (h | l)
    constexpr int NR = TN * 16;                                 // weight rows staged
    constexpr int STRIP_PIX = BM + 2 * (KW - 1);
    constexpr int STRIP_BYTES = STRIP_PIX * PB;
    constexpr int STRIP_PIECES = (STRIP_BYTES + 1023) / 1024;
    constexpr int W_BYTES = 2 * NR * C * 2;                     // [pc][NR][C] fp16
    constexpr int W_PW = W_BYTES / 1024 / NW;                   // weight DMAs per wave per tap
    static_assert(W_BYTES % (1024 * NW) == 0, "weight tap is not a whole number of DMAs per wave");
    constexpr int NSP = 5;                                      // taps that carry strip DMAs
    constexpr int SPW = (STRIP_PIECES + NW * NSP - 1) / (NW * NSP);   // strip DMAs per wave per such tap
    static_assert(NSP < KW, "strip of r+1 must be issued before the last tap of r");
    constexpr int S_OFF = 0, W_OFF = 2 * STRIP_PIECES * 1024;
    __shared__ __attribute__((aligned(1024))) char smem[W_OFF + 2 * W_BYTES];

    const fg_conv_problem& P = args.P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int img = wid / args.tiles_per_img;
    const int p0 = (wid - img * args.tiles_per_img) * BM;
    const int mab = P.m_a * P.m_b;
    const int a0 = p0 / P.m_b, b0 = p0 - (p0 / P.m_b) * P.m_b;
    const int len0 = min(BM, min(P.m_b - b0, mab - p0));
    const int len1 = (a0 + 1 < P.m_a) ? min(BM - len0, P.m_b) : 0;
    const int s0pix = len0 + KW - 1;                            // LDS strip pixel where segment 1 starts
    const int strip_bytes = (len0 + len1 + 2 * (KW - 1)) * PB;
    const int wp = args.wp;

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)args.xs, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);

    // ---- strip DMA sources: piece j (this wave's k-th of the tap) covers LDS strip bytes
    // [j*1024, +1024); lane byte o -> segment 0 (input row a0+r, from column b0) or segment 1
    // (row a0+1+r, from column 0); bytes past the strip re-read segment 0's start
    const int seg0_pix = img * (int)(P.sxn / C) + a0 * wp + b0;      // + r*wp per kernel row
    const int seg1_pix = img * (int)(P.sxn / C) + (a0 + 1) * wp;
    int s_off[NSP * SPW];
#pragma unroll
    for (int k = 0; k < NSP * SPW; ++k) {
        const int j = min(k * NW + wave, STRIP_PIECES - 1);       // clamped: duplicates rewrite the same bytes
        const int o = j * 1024 + lane * 16;
        int src;
        if (o >= strip_bytes) src = seg0_pix * PB;
        else if (o < s0pix * PB) src = seg0_pix * PB + o;
        else src = seg1_pix * PB + (o - s0pix * PB);
        s_off[k] = src;
    }
    // ---- weight DMA sources: piece j of a tap = LDS bytes [j*1024, +1024) of [pc][NR][C]
    int w_off[W_PW];
#pragma unroll
    for (int i = 0; i < W_PW; ++i) {
        const int f = (wave * W_PW + i) * 64 + lane;             // 16-B chunk index in the image
        const int pc = f / (NR * C / 8);
        const int rem = f - pc * (NR * C / 8);
        const int n = rem / (C / 8);
        const int ch = (rem - n * (C / 8)) ^ swz_wrow<C>(n);      // logical chunk stored at this slot
        w_off[i] = (min(n, P.n_out - 1) * (P.ldw / 8) + ch) * 32 + pc * 16;
    }
    auto issue_w = [&](int t) {                                   // tap t = r*KW + s -> buffer t&1
        const int r = t / KW, s = t - (t / KW) * KW;
        const int soff = ((r * P.jp + s * C) / 8) * 32;
        char* dstb = smem + W_OFF + (t & 1) * W_BYTES;
#pragma unroll
        for (int i = 0; i < W_PW; ++i)
            dma16(wr, dstb + (wave * W_PW + i) * 1024, w_off[i], soff);
    };
    auto issue_s = [&](int r, int part) {                         // strip of kernel row r, DMA group `part`
        char* dstb = smem + S_OFF + (r & 1) * STRIP_PIECES * 1024;
        const int soff = r * wp * PB;
#pragma unroll
        for (int k = 0; k < SPW; ++k) {
            const int kk = part * SPW + k;
            const int j = min(kk * NW + wave, STRIP_PIECES - 1);
            dma16(xr, dstb + j * 1024, s_off[kk], soff);
        }
    };

    const float sa = fgc::pow2_scale(P.x_absmax);
    const float sb = fgc::pow2_scale(P.w_absmax);
    const float out_scale = 1.f / (sa * sb);

    // per-lane fragment geometry: tile row i -> strip pixel q0 and absolute column x0 (tap s adds s)
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

    constexpr int CC = C / 32;
    f16x8 ah[CC][TM], al[CC][TM];
    auto load_a = [&](int t) {
        const int r = t / KW, s = t - (t / KW) * KW;
        const char* sb_ = smem + S_OFF + (r & 1) * STRIP_PIECES * 1024;
#pragma unroll
        for (int cc = 0; cc < CC; ++cc)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const char* px = sb_ + (q0[tm] + s) * PB;
                const int sw = swz_strip<C>(x0[tm] + s);
                ah[cc][tm] = *reinterpret_cast<const f16x8*>(px + ((cc * 4 + g) ^ sw) * 16);
                al[cc][tm] = *reinterpret_cast<const f16x8*>(px + ((C / 8 + cc * 4 + g) ^ sw) * 16);
            }
    };
    auto compute = [&](int t) {
        const char* wb = smem + W_OFF + (t & 1) * W_BYTES;
#pragma unroll
        for (int cc = 0; cc < CC; ++cc) {
            f16x8 bh[TN], bl[TN];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = tn * 16 + fr;
                const char* row = wb + n * (2 * C) + ((cc * 4 + g) ^ swz_wrow<C>(n)) * 16;
                bh[tn] = *reinterpret_cast<const f16x8*>(row);
                bl[tn] = *reinterpret_cast<const f16x8*>(row + NR * 2 * C);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[cc][tm], bh[tn], acc[tm][tn], 0, 0, 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cc][tm], bl[tn], acc[tm][tn], 0, 0, 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cc][tm], bh[tn], acc[tm][tn], 0, 0, 0);
        }
    };

    // ---- tap loop.  Issue order per tap: weights of the next tap, then (taps s < NSP) one group
    // of the next kernel row's strip.  At tap t this wave waits for its weight DMAs of t, which
    // only the strip group issued with them at t-1 may follow.  The strip of row r is complete
    // from the barrier of tap (r, 0) until the barrier of tap (r + 1, 0) (only then is its buffer
    // refilled), so with APF the fragments of tap (r, s + 1) are read before that tap's barrier.
    const int KH = P.kh;
    const int ntap = KH * KW;
    issue_s(0, 0);
#pragma unroll
    for (int part = 1; part < NSP; ++part) issue_s(0, part);
    issue_w(0);
    for (int t = 0; t < ntap; ++t) {
        const int r = t / KW, s = t - (t / KW) * KW;
        if (s >= 1 && s - 1 < NSP && r + 1 < KH) vm_wait<SPW>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < ntap) issue_w(t + 1);
        if (s < NSP && r + 1 < KH) issue_s(r + 1, s);
        if (!APF || s == 0) load_a(t);
        compute(t);
        if (APF && s + 1 < KW) load_a(t + 1);
    }

    // ---- epilogue
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

// Register-staged form: one kernel row per barrier pair instead of one tap per barrier.  The whole row's
// weights (KW taps, [s][pc][NR][C]) and its input strip sit in LDS together (single-buffered: 68.6 + 57.3 KB at
// C 64); the next row's strip and weights are loaded into registers (16-B buffer loads, the same bytes the DMA
// form copies) while the KW taps of the current row run -- 168 MFMAs per wave between barriers instead of 24 --
// and written over the current ones after a barrier.
template <int C, int KW, int TN, int NW>
__global__ void __launch_bounds__(NW * 64, 1) conv_win_rs_kernel(const WinArgs args) {
    constexpr int NT = NW * 64;
    constexpr int BM = 256, WM = BM / NW, TM = WM / 16;
    constexpr int PB = 4 * C;                                   // strip bytes per pixel (h | l)
    constexpr int NR = TN * 16;                                 // weight rows staged
    constexpr int STRIP_BYTES = (BM + 2 * (KW - 1)) * PB;
    constexpr int SCH = (STRIP_BYTES / 16 + NT - 1) / NT;       // strip 16-B chunks per thread
    constexpr int W_TAP = 2 * NR * C * 2;                       // [pc][NR][C] fp16 per tap
    constexpr int TAP_CH = W_TAP / 16;
    constexpr int WCH = KW * TAP_CH / NT;                       // weight 16-B chunks per thread per kernel row
    static_assert((KW * TAP_CH) % NT == 0, "weight row is not a whole number of chunks per thread");
    constexpr int W_OFF = (STRIP_BYTES + 1023) / 1024 * 1024;
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
    const int strip_bytes = (len0 + len1 + 2 * (KW - 1)) * PB;
    const int wp = args.wp;
    constexpr int kOOB = 0x7fffffff;

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)args.xs, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);

    // strip chunk o = (tid + i NT) * 16 of the LDS strip <- its source byte (row offset r * wp * PB added per row)
    const int seg0_pix = img * (int)(P.sxn / C) + a0 * wp + b0;
    const int seg1_pix = img * (int)(P.sxn / C) + (a0 + 1) * wp;
    int s_src[SCH];
#pragma unroll
    for (int i = 0; i < SCH; ++i) {
        const int o = (tid + i * NT) * 16;
        s_src[i] = o >= strip_bytes ? -1 : o < s0pix * PB ? seg0_pix * PB + o : seg1_pix * PB + (o - s0pix * PB);
    }
    // weight chunk F = tid + i NT of the row image [s][pc][NR][C]: tap s = F / TAP_CH, in-tap chunk f
    int w_src[WCH];
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
        const int F = tid + i * NT, s = F / TAP_CH, f = F - s * TAP_CH;
        const int pc = f / (NR * C / 8);
        const int rem = f - pc * (NR * C / 8);
        const int n = rem / (C / 8);
        const int ch = (rem - n * (C / 8)) ^ swz_wrow<C>(n);
        w_src[i] = (min(n, P.n_out - 1) * (P.ldw / 8) + ch) * 32 + pc * 16 + ((s * C) / 8) * 32;
    }
    f32x4 rs[SCH], rw[WCH];
    auto load = [&](int r) {
        const int soff = r * wp * PB, woff = ((r * P.jp) / 8) * 32;
#pragma unroll
        for (int i = 0; i < SCH; ++i)
            rs[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, s_src[i] >= 0 ? s_src[i] + soff : kOOB, 0, 0));
#pragma unroll
        for (int i = 0; i < WCH; ++i)
            rw[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, w_src[i] + woff, 0, 0));
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < SCH; ++i)
            if (s_src[i] >= 0) *reinterpret_cast<f32x4*>(smem + (tid + i * NT) * 16) = rs[i];
#pragma unroll
        for (int i = 0; i < WCH; ++i) *reinterpret_cast<f32x4*>(smem + W_OFF + (tid + i * NT) * 16) = rw[i];
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

    constexpr int CC = C / 32;
    auto tap = [&](int s) {
        f16x8 ah[CC][TM], al[CC][TM];
#pragma unroll
        for (int cc = 0; cc < CC; ++cc)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const char* px = smem + (q0[tm] + s) * PB;
                const int sw = swz_strip<C>(x0[tm] + s);
                ah[cc][tm] = *reinterpret_cast<const f16x8*>(px + ((cc * 4 + g) ^ sw) * 16);
                al[cc][tm] = *reinterpret_cast<const f16x8*>(px + ((C / 8 + cc * 4 + g) ^ sw) * 16);
            }
        const char* wb = smem + W_OFF + s * W_TAP;
#pragma unroll
        for (int cc = 0; cc < CC; ++cc) {
            f16x8 bh[TN], bl[TN];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = tn * 16 + fr;
                const char* row = wb + n * (2 * C) + ((cc * 4 + g) ^ swz_wrow<C>(n)) * 16;
                bh[tn] = *reinterpret_cast<const f16x8*>(row);
                bl[tn] = *reinterpret_cast<const f16x8*>(row + NR * 2 * C);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[cc][tm], bh[tn], acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cc][tm], bl[tn], acc[tm][tn], 0, 0, 0);
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cc][tm], bh[tn], acc[tm][tn], 0, 0, 0);
                }
        }
    };

    const int KH = P.kh;
    load(0);
    store();
    __syncthreads();
    for (int r = 0; r < KH; ++r) {
        if (r + 1 < KH) load(r + 1);
#pragma unroll
        for (int s = 0; s < KW; ++s) tap(s);
        if (r + 1 < KH) {
            __syncthreads();
            store();
            __syncthreads();
        }
    }

    // ---- epilogue
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

// waves per workgroup: 4 (one per SIMD, 64 rows each) or 8 (two per SIMD, 32 rows each: a partner wave's
// MFMAs cover each wave's fragment-read latency); FLOODGAN_WIN_WAVES selects (A/B)
template <int C, int KW, int TN>
int launch_win(const WinArgs& a, int tiles, hipStream_t stream) {
    const char* rs = getenv("FLOODGAN_WIN_RS");
    if (rs && atoi(rs) == 4) {
        hipLaunchKernelGGL((conv_win_rs_kernel<C, KW, TN, 4>), dim3(tiles), dim3(256), 0, stream, a);
        return fg::launched("conv_win_rs");
    }
    if (rs && atoi(rs)) {
        hipLaunchKernelGGL((conv_win_rs_kernel<C, KW, TN, 8>), dim3(tiles), dim3(512), 0, stream, a);
        return fg::launched("conv_win_rs");
    }
    const char* e = getenv("FLOODGAN_WIN_WAVES");
    const int nw = e ? atoi(e) : g_win_waves;
    const char* ea = getenv("FLOODGAN_WIN_APF");
    const bool apf = ea ? atoi(ea) != 0 : g_win_apf < 0 ? C == 32 : g_win_apf != 0;
    if (nw == 8 && apf)
        hipLaunchKernelGGL((conv_win_kernel<C, KW, TN, 8, true>), dim3(tiles), dim3(512), 0, stream, a);
    else if (nw == 8)
        hipLaunchKernelGGL((conv_win_kernel<C, KW, TN, 8, false>), dim3(tiles), dim3(512), 0, stream, a);
    else if (apf)
        hipLaunchKernelGGL((conv_win_kernel<C, KW, TN, 4, true>), dim3(tiles), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL((conv_win_kernel<C, KW, TN, 4, false>), dim3(tiles), dim3(256), 0, stream, a);
    return fg::launched("conv_win");
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
    if (C == 64) return launch_win<64, 7, 2>(a, tiles, stream);
    return launch_win<32, 7, 4>(a, tiles, stream);
}
