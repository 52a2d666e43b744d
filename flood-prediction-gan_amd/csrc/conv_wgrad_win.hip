// Row-strip weight gradient of the content head (deconv3_content, 7x7, 64 -> 27,
// models/model_architectures.py:328): convolution_backward's weight gradient
//
//   dW[n][r][s][c] = sum over output pixels (img, a, b) of gy[img,a,b][n] * x[img, a+r, b+s][c]
//
// The reduction over output pixels runs in chunks of 32 consecutive pixels of one output row.
// A workgroup owns one kernel row r and a range of chunks; per chunk it stages the 32 gradient
// pixels (the fg_split_pixels copy of the 32-channel gradient, made for the input gradient) and
// the 38-pixel input strip of row r (the 64-channel copy the forward made) by LDS-DMA, and every
// tap s reads the strip shifted by s -- the im2col gather of the generic weight-gradient kernel
// re-read each input pixel 49 times.  Operands reach v_mfma_f32_16x16x32_f16 through transposed
// LDS reads (8 consecutive pixels of one channel per lane); partial sums go to per-split fp32
// slabs that fg_wgrad_reduce adds.
//
// L2 reuse: the seven workgroups of one split (kernel rows 0..6) read the same gradient chunks and, one
// chunk apart, the same input rows.  They are placed on one XCD (blocks b, b + 8, ... share an XCD's L2
// under the round-robin dispatch; speed only, never correctness) and a split walks its chunks DOWN the
// image (column block outer, output row inner), so the input strip that kernel row r reads at output row a
// is the one kernel row r - 1 reads at row a + 1, one chunk later: every gradient chunk and input strip
// comes from HBM once instead of seven times (5.7 GB -> ~0.9 GB per launch at bs 8, 512^2: the row-major
// walk over seven XCDs read both at a 5 % L2 hit rate, profiles/round3/r3a_pmc_step.json).
#include "conv_common.hpp"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// byte offset of 4 consecutive fp16 (piece pc, channel ch, ch % 4 == 0) inside one split pixel of
// column x (the chunk swizzle of fg_split_pixels)
template <int C>
__device__ __forceinline__ int pix_byte(int x, int pc, int ch) {
    const int k = pc * (C / 8) + (ch >> 3);
    return ((k ^ fgc::swz_pixel<C>(x)) << 4) + ((ch & 7) << 1);
}

__device__ __forceinline__ f16x8 tr2(const char* a0, const char* a1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(f16x8, v);
}

struct WgWinArgs {
    fg_wgrad_problem P;
    const char* ps;             // gradient split copy (pixel 0 of its buffer)
    const char* xs;             // input split copy (pixel 0 of its buffer)
    int p_pix0, p_col0, wpp;    // gradient origin pixel, its column, pixels per padded row
    int x_pix0, wpx;            // input origin pixel (a padded-row start), pixels per padded row
    int chunks_per_split, nchunks;
    int xcd_group;              // 1: the block -> (split, kernel row) map groups a split's 7 blocks on one XCD
};

__global__ void __launch_bounds__(256) wgrad_win_kernel(const WgWinArgs args) {
    constexpr int CP = 32, CX = 64, KW = 7, TM = 2, TN = 7;
    constexpr int PBP = 4 * CP, PBX = 4 * CX;                 // bytes per split pixel
    constexpr int P_BYTES = 32 * PBP;                         // 4 KiB: one DMA per wave
    constexpr int X_PIX = 32 + KW - 1, X_BYTES = X_PIX * PBX; // 38 px = 9.5 KiB
    constexpr int X_PIECES = (X_BYTES + 1023) / 1024;         // 10
    constexpr int XPW = (X_PIECES + 3) / 4;                   // 3 per wave (clamped duplicates)
    constexpr int STAGE = P_BYTES + X_PIECES * 1024;
    __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

    const fg_wgrad_problem& P = args.P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-grouped (blocks of one split share blockIdx % 8) when the split count is a multiple of 8
    int r, split;
    if (args.xcd_group) {
        const int q = blockIdx.x >> 3;
        r = q % KW;
        split = (blockIdx.x & 7) + 8 * (q / KW);
    } else {
        r = blockIdx.x % KW;
        split = blockIdx.x / KW;
    }
    const int c0 = split * args.chunks_per_split;
    const int c1 = min(args.nchunks, c0 + args.chunks_per_split);
    const int cpr = P.m_b / 32;                               // chunks per output row

    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)args.ps, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)args.xs, 0, 0x7fffffff, 0x00020000);
    const float sp = fgc::pow2_scale(P.p_absmax);
    const float sx = fgc::pow2_scale(P.x_absmax);

    // chunk -> first gradient pixel / first input-strip pixel (indices in the split copies), b0; chunks are
    // numbered column block outer, output row inner within an image (a split walks down the image)
    const int per_img = P.m_a * cpr;
    auto bases = [&](int ch, int& pbase, int& xbase, int& b0) {
        const int img = ch / per_img, rem = ch - img * per_img;
        const int cb = rem / P.m_a, a = rem - cb * P.m_a;
        b0 = cb * 32;
        pbase = args.p_pix0 + img * (int)(P.spn / CP) + a * args.wpp + b0;
        xbase = args.x_pix0 + img * (int)(P.sxn / CX) + (a + r) * args.wpx + b0;
    };
    auto issue = [&](int buf, int ch) {
        int pbase, xbase, b0;
        bases(ch, pbase, xbase, b0);
        char* sb = smem + buf * STAGE;
        dma16(pr, sb + wave * 1024, pbase * PBP + wave * 1024 + lane * 16);
#pragma unroll
        for (int k = 0; k < XPW; ++k) {
            const int j = min(k * 4 + wave, X_PIECES - 1);
            const int o = min(j * 1024 + lane * 16, X_BYTES - 16);
            dma16(xr, sb + P_BYTES + j * 1024, xbase * PBX + o);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read roles: group g reads pixel rows 8g+q (and 8g+4+q), lane 4q+p channels 4p..4p+3
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
    auto compute = [&](int buf, int ch) {
        int pbase, xbase, b0;
        bases(ch, pbase, xbase, b0);
        const char* sb = smem + buf * STAGE;
        const char* xb = sb + P_BYTES;
        const int xp0 = args.p_col0 + b0;             // column of the chunk's first gradient pixel
        const int r0 = 8 * g + q, r1 = r0 + 4;
        f16x8 ah[TM], al[TM];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int c_ = tm * 16 + p4;
            ah[tm] = tr2(sb + r0 * PBP + pix_byte<CP>(xp0 + r0, 0, c_), sb + r1 * PBP + pix_byte<CP>(xp0 + r1, 0, c_));
            al[tm] = tr2(sb + r0 * PBP + pix_byte<CP>(xp0 + r0, 1, c_), sb + r1 * PBP + pix_byte<CP>(xp0 + r1, 1, c_));
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int kc = wave * 112 + tn * 16;        // k column within kernel row r: s*64 + c
            const int s = kc >> 6, cc = (kc & 63) + p4;
            const int x0 = r0 + s, x1 = r1 + s;         // strip pixels (columns b0 + x0, b0 + x1)
            const f16x8 bh = tr2(xb + x0 * PBX + pix_byte<CX>(b0 + x0, 0, cc), xb + x1 * PBX + pix_byte<CX>(b0 + x1, 0, cc));
            const f16x8 bl = tr2(xb + x0 * PBX + pix_byte<CX>(b0 + x0, 1, cc), xb + x1 * PBX + pix_byte<CX>(b0 + x1, 1, cc));
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[tm], bh, acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[tm], bl, acc[tm][tn], 0, 0, 0);
                acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[tm], bh, acc[tm][tn], 0, 0, 0);
            }
        }
    };

    // double buffer: chunk ch+1 streams in while chunk ch is reduced
    if (c0 < c1) issue(0, c0);
    for (int ch = c0, buf = 0; ch < c1; ++ch, buf ^= 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (ch + 1 < c1) issue(buf ^ 1, ch + 1);
        compute(buf, ch);
    }

    // slab rows n (< n_a), columns r*448 + wave*112 + 16tn + (lane & 15)
    const int K = P.kh * P.j_valid;
    float* out = P.out + (size_t)split * P.n_a * K;
    const float osc = 1.f / (sp * sx);
    const int fr = lane & 15;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int n = tm * 16 + 4 * g + reg;
            if (n >= P.n_a) continue;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                out[(size_t)n * K + r * P.j_valid + wave * 112 + tn * 16 + fr] = acc[tm][tn][reg] * osc;
        }
}

}  // namespace

FG_API int fg_conv_wgrad_win(const fg_wgrad_problem* prob, const void* p_split, long long p_pix0, int p_col0,
                             int wp_p, const void* x_split, long long x_pix0, int wp_x, hipStream_t stream) {
    if (!prob || !p_split || !x_split || !prob->out || !prob->p_absmax || !prob->x_absmax || wp_p < 1 || wp_x < 1)
        return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad_win: null argument");
    const fg_wgrad_problem& p = *prob;
    if (p.kh != 7 || p.j_valid != 7 * 64 || p.sxb != 64 || p.sxa != p.sxr || p.sxr != (long long)wp_x * 64 ||
        p.spb != 32 || p.spa != (long long)wp_p * 32 || p.n_a < 1 || p.n_a > 32 || p.m_b % 32 || p.m_b < 32 ||
        p.m_a < 1 || p.m_img < 1 || p.spn % 32 || p.sxn % 64 || p_pix0 < 0 || x_pix0 < 0 || x_pix0 % wp_x ||
        p_col0 < 0 || (p_pix0 - p_col0) % wp_p || p.splits < 1)
        return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad_win: unsupported geometry (7x7, 64 input / 32 gradient "
                                        "channels, n_a <= 32, output rows a multiple of 32 px)");
    const long long xspan = x_pix0 + (long long)p.m_img * (p.sxn / 64) + 8LL * wp_x;
    const long long pspan = p_pix0 + (long long)p.m_img * (p.spn / 32);
    if (xspan * 256 >= (1LL << 31) || pspan * 128 >= (1LL << 31))
        return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad_win: split operand beyond 2 GiB");
    WgWinArgs a;
    a.P = p;
    a.ps = reinterpret_cast<const char*>(p_split);
    a.xs = reinterpret_cast<const char*>(x_split);
    a.p_pix0 = (int)p_pix0;
    a.p_col0 = p_col0;
    a.wpp = wp_p;
    a.x_pix0 = (int)x_pix0;
    a.wpx = wp_x;
    a.nchunks = p.m_img * p.m_a * (p.m_b / 32);
    a.chunks_per_split = (a.nchunks + p.splits - 1) / p.splits;
    a.xcd_group = p.splits % 8 == 0 ? 1 : 0;
    hipLaunchKernelGGL(wgrad_win_kernel, dim3(7 * p.splits), dim3(256), 0, stream, a);
    return fg::launched("wgrad_win");
}
