// Pipelined f16x3 weight-gradient kernel for the wide convolutions (the resblock 3x3 convs,
// conv2/conv3, deconv1 and discriminator model.2/5/8 -- n_a >= 128 result rows, K >= 256):
// convolution_backward's weight gradient of models/model_architectures.py:314-333, :407-410,
// :426-435.
//
//   out[split][a][k] = sum over the split's pixels m of  P[m][a] * X[m][koff(k)]
//
// 256 x 256 (a x k) tiles, 8 waves as 4 (a) x 2 (k), each 64 x 128 in 16x16 blocks of
// v_mfma_f32_16x16x32_f16 whose reduction index is 32 consecutive pixels.  Both operands stay in
// their natural pixel-major layout: each stage loads 32 pixel rows of P (256 channels) and of the
// X gather (256 k-columns) as float4 per slot, splits them into the scaled fp16 pieces (h, l) and
// writes [piece][32 px][256] images; the MFMA fragments (8 consecutive pixels of one column per
// lane) come out of ds_read_b64_tr_b16.  Write-after-barrier staging: at the top of stage t the
// registers holding tile t+1 go to the free LDS buffer and are refilled with tile t+2, so every
// global load has a whole stage of MFMAs to land.
#include "conv_common.hpp"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BR = 32;              // pixels per stage (the MFMA reduction depth)
constexpr int TK = 256;             // k extent of a tile (the a extent TA is 256 or 128)

// 32-B column-pair swizzle: the 8 rows a 32-lane half of a transposed read touches land on
// 8 distinct 32-B bank groups
__device__ __forceinline__ int swz_tr(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }   // in 16-B chunks

template <int COLS>
__device__ __forceinline__ int img_off(int row, int col) {   // byte offset of fp16 column col of row
    // (the swizzle stays inside the row's COLS / 8 chunks: a 64-column image has 8)
    return row * (COLS * 2) + (((col >> 3) ^ (swz_tr(row) & (COLS / 8 - 1))) << 4) + ((col & 7) << 1);
}

__device__ __forceinline__ f16x8 tr_frag(const char* base, int a0, int a1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + a0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + a1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(f16x8, v);
}

__device__ __forceinline__ void split4(const f32x4& v, float s, f16x4& h, f16x4& l) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    u32x2 hu, lu;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        unsigned a, b;
        fgc::split_pair_mix(v[2 * e], v[2 * e + 1], s, a, b);     // the mixed-FMA split (conv_common.hpp)
        hu[e] = a;
        lu[e] = b;
    }
    h = __builtin_bit_cast(f16x4, hu);
    l = __builtin_bit_cast(f16x4, lu);
}

// SCH 0: each stage = store (split + LDS writes of the staged registers) and the next global
// loads as one burst, then the MFMAs; SCH 1: the stage's MFMAs in four column groups with one
// staging slot's store + reload in front of each (the VALU split and the LDS writes run beside
// the partner wave's MFMAs instead of stalling the SIMD at the top of every stage).
// PS bit 0 / bit 1: P / X arrive in the FG_PRESPLIT format (include/floodgan.h): a float4 slot then holds
// the h (col % 8 == 0) or the l (col % 8 == 4) piece of its 8-channel group, written to its image as it stands
template <int TA, int SCH, int PS = 0>
__global__ void __launch_bounds__(512, 1)
conv_wgrad_f3_kernel(const fg_wgrad_problem P, int tiles_a, int tiles_k) {
    // 8 waves as NWA (a) x NWK (k); wave tile 64 (a) x WK (k): TA 256 -> 4 x 2, 64 x 128; TA 128 -> 2 x 4, 64 x 64;
    // TA 64 -> 1 x 8, 64 x 32 (the 64-output-channel stem / D model.0 weight gradients)
    constexpr int NT = 512, NWA = TA / 64, NWK = 8 / NWA, WK = TK / NWK, TM = 4, TN = WK / 16;
    constexpr int SPT = BR * TK / 4 / NT;           // float4 slots per thread per operand per stage (4)
    constexpr int IMGP = BR * TA * 2, IMGX = BR * TK * 2;   // bytes per piece image
    // piece images at PH = 0, PL, XH, XL: each l image 64 B past its h image's bank phase, so that the pre-split
    // staging's lane pairs (an 8-channel group's h and l halves, one 16-B store each) hit different banks
    constexpr int PL = IMGP + 64, XH = 2 * IMGP + 128, XL = XH + IMGX + 64;
    constexpr int BUF = XL + IMGX + 64;
    constexpr int kOOB = 0x7fffffff;
    __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];   // [buf][P h, P l, X h, X l]

    // wave-uniform by construction (readfirstlane): the pixel walks below live in SGPRs
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wa = wave / NWK, wk = wave - (wave / NWK) * NWK;
    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = tiles_a * tiles_k;
    const int split = wid / ntile;
    const int tile = wid - split * ntile;
    const int ta = tile / tiles_k, tk = tile - (tile / tiles_k) * tiles_k;
    const int a0 = ta * TA, k0 = tk * TK;
    const int mab = P.m_a * P.m_b;
    const int M = P.m_img * mab;
    const int mbeg = split * P.m_chunk;
    const int mend = min(M, mbeg + P.m_chunk);
    const int K = P.kh * P.j_valid;
    const int nst = mend > mbeg ? (mend - mbeg + BR - 1) / BR : 0;

    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)P.p, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
    const float sp = fgc::pow2_scale(P.p_absmax);
    const float sx = fgc::pow2_scale(P.x_absmax);

    // ---- staging slots: slot s = tid + i*NT -> pixel row s / 64 of the stage, column group (s % 64)*4.
    // Each thread's slots share one column group and walk pixel rows i*8 + tid/64, advanced by BR.
    const int col = (tid & 63) * 4;
    const int prow0 = wave;                         // + 8i
    const bool p_slot = col < TA;                   // P has TA columns: lanes past them stage nothing
    const bool p_col_ok = p_slot && a0 + col < P.n_a;   // n_a % 4 == 0 (host check)
    int x_koff = -1;                                // X column offset of this slot's k (k % 4 == 0 group)
    {
        const int k = k0 + col;
        if (k < K) {
            const int r = k / P.j_valid;
            x_koff = r * (int)P.sxr + (k - r * P.j_valid);
        }
    }
    // pixel walks (img, a, b) of the SPT slot rows
    const int i32 = BR / mab, a32 = (BR - i32 * mab) / P.m_b, b32 = BR - i32 * mab - a32 * P.m_b;
    int wm[SPT], wi[SPT], wa_[SPT], wb[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
        wm[i] = mbeg + prow0 + 8 * i;
        fgc::decomp(min(wm[i], M - 1), P.m_b, mab, wi[i], wa_[i], wb[i]);
    }
    f32x4 rp[SPT], rx[SPT];
    auto load_slot = [&](int i) {
        {
            const bool ok = wm[i] < mend;
            const int pb = wi[i] * (int)P.spn + wa_[i] * (int)P.spa + wb[i] * (int)P.spb + a0 + col;
            const int xb = wi[i] * (int)P.sxn + wa_[i] * (int)P.sxa + wb[i] * (int)P.sxb + x_koff;
            rp[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, ok && p_col_ok ? pb * 4 : kOOB, 0, 0));
            rx[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok && x_koff >= 0 ? xb * 4 : kOOB, 0, 0));
            // advance by BR pixels
            wm[i] += BR;
            wb[i] += b32;
            const int cb = wb[i] >= P.m_b;
            wb[i] -= cb ? P.m_b : 0;
            wa_[i] += a32 + cb;
            const int ca = wa_[i] >= P.m_a;
            wa_[i] -= ca ? P.m_a : 0;
            wi[i] += i32 + ca;
        }
    };
    auto load = [&]() {
#pragma unroll
        for (int i = 0; i < SPT; ++i) load_slot(i);
    };
    auto store_slot = [&](int buf, int i) {
        char* b = smem + buf * BUF;
        {
            f16x4 h, l;
            if (p_slot) {
                if constexpr (PS & 1) {
                    const int op = img_off<TA>(prow0 + 8 * i, col & ~7) + ((col & 4) ? PL : 0);
                    *reinterpret_cast<f16x8*>(b + op) = __builtin_bit_cast(f16x8, rp[i]);
                } else {
                    const int op = img_off<TA>(prow0 + 8 * i, col);
                    split4(rp[i], sp, h, l);
                    *reinterpret_cast<f16x4*>(b + op) = h;
                    *reinterpret_cast<f16x4*>(b + PL + op) = l;
                }
            }
            if constexpr (PS & 2) {
                const int ox = img_off<TK>(prow0 + 8 * i, col & ~7) + ((col & 4) ? XL : XH);
                *reinterpret_cast<f16x8*>(b + ox) = __builtin_bit_cast(f16x8, rx[i]);
            } else {
                const int ox = img_off<TK>(prow0 + 8 * i, col);
                split4(rx[i], sx, h, l);
                *reinterpret_cast<f16x4*>(b + XH + ox) = h;
                *reinterpret_cast<f16x4*>(b + XL + ox) = l;
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) store_slot(buf, i);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read lane roles: group g reads pixel rows 8g + q (and 8g + 4 + q), lane 4q+p of
    // the group addresses columns 4p..4p+3 of the 16-column block
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
    constexpr int TG = SCH == 0 ? (TN < 4 ? TN : 4) : TN / SPT;   // column blocks per group (SCH 1: a slot per group)
    static_assert(TN % TG == 0 && (SCH == 0 || TN / TG == SPT), "groups");
    auto compute = [&](int buf, bool stage_next) {
        const char* b = smem + buf * BUF;
        f16x8 ah[TM], al[TM];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int c = wa * 64 + tm * 16 + p4;
            const int o0 = img_off<TA>(8 * g + q, c), o1 = img_off<TA>(8 * g + 4 + q, c);
            ah[tm] = tr_frag(b, o0, o1);
            al[tm] = tr_frag(b + PL, o0, o1);
        }
#pragma unroll
        for (int t0 = 0; t0 < TN; t0 += TG) {
            f16x8 bh[TG], bl[TG];
#pragma unroll
            for (int t = 0; t < TG; ++t) {
                const int c = wk * WK + (t0 + t) * 16 + p4;
                const int o0 = img_off<TK>(8 * g + q, c), o1 = img_off<TK>(8 * g + 4 + q, c);
                bh[t] = tr_frag(b + XH, o0, o1);
                bl[t] = tr_frag(b + XL, o0, o1);
            }
            if constexpr (SCH == 1) {
                // this group's staging slot: split + write the registers of the next stage into the
                // free buffer, then refill them with the stage after
                if (stage_next) store_slot(buf ^ 1, t0 / TG);
                load_slot(t0 / TG);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int t = 0; t < TG; ++t)
                    acc[tm][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[t], al[tm], acc[tm][t0 + t], 0, 0, 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int t = 0; t < TG; ++t)
                    acc[tm][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[t], ah[tm], acc[tm][t0 + t], 0, 0, 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int t = 0; t < TG; ++t)
                    acc[tm][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[t], ah[tm], acc[tm][t0 + t], 0, 0, 0);
        }
    };

    // ---- write-after-barrier pipeline (one register set; loads past the range read zeros)
    load();
    store(0);
    load();
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int cur = st & 1;
        if constexpr (SCH == 0) {
            if (st + 1 < nst) store(cur ^ 1);
            load();
            __builtin_amdgcn_sched_barrier(0);
            compute(cur, false);
        } else {
            compute(cur, st + 1 < nst);
        }
        __syncthreads();
    }

    // ---- epilogue: scaled fp32 slab rows a, columns k.  The MFMAs take their operands exchanged (D^T = B^T A^T), so a
    // lane's 4 accumulator registers are 4 consecutive columns k of one row a: one 16-B store per 16 x 16 block
    // instead of four scattered dwords (K % 4 == 0, launch_wgrad_f3)
    float* out = P.out + (size_t)split * P.n_a * K;
    const float osc = 1.f / (sp * sx);
    const int fr = lane & 15;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int a = a0 + wa * 64 + tm * 16 + fr;
        if (a >= P.n_a) continue;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int k = k0 + wk * WK + tn * 16 + 4 * g;
            if (k < K) *reinterpret_cast<f32x4*>(out + (size_t)a * K + k) = acc[tm][tn] * osc;
        }
    }
}

}  // namespace

int g_wgrad_f3 = 2;   // fg_set_wgrad_f3 (A/B hook): 0 off, 1 stage schedule 0, 2 auto, 3 stage schedule 1

namespace fgc {

// Returns 1 when the pipelined kernel took the problem (status in *rc), 0 when it does not apply.
int launch_wgrad_f3(const fg_wgrad_problem& p, hipStream_t stream, int* rc) {
    // (K >= 256: D model.0's K = 192 ran 199 us here against 185 on the register-staged kernel, r3ae)
    if (!g_wgrad_f3 || p.n_a < 64 || p.kh * p.j_valid < 256 || p.n_a % 4 || p.j_valid % 4 || !p.p_absmax ||
        !p.x_absmax || ((uintptr_t)p.p & 15) || ((uintptr_t)p.x & 15) || (p.spn | p.spa | p.spb) % 4 ||
        (p.sxn | p.sxa | p.sxb | p.sxr) % 4)
        return 0;
    const int TA = p.n_a >= 256 ? 256 : p.n_a > 64 ? 128 : 64;
    const int ta = (p.n_a + TA - 1) / TA, tk = (p.kh * p.j_valid + TK - 1) / TK;
    const dim3 grid(ta * tk * p.splits);
    const int ps = (p.p_presplit ? 1 : 0) | (p.x_presplit ? 2 : 0);
    if (ps) {
        // whole 8-channel groups at 32-B aligned bases (FG_PRESPLIT); the measured staging schedule per tile
        if (p.n_a % 8 || p.j_valid % 8 || (p.p_presplit && (((uintptr_t)p.p & 31) || (p.spn | p.spa | p.spb) % 8)) ||
            (p.x_presplit && (((uintptr_t)p.x & 31) || (p.sxn | p.sxa | p.sxb | p.sxr) % 8)))
            return 0;
        if (TA == 64) {
            if (ps == 1)
                FG_LAUNCH((conv_wgrad_f3_kernel<64, 0, 1>), grid, dim3(512), 0, stream, p, ta, tk);
            else if (ps == 2)
                FG_LAUNCH((conv_wgrad_f3_kernel<64, 0, 2>), grid, dim3(512), 0, stream, p, ta, tk);
            else
                FG_LAUNCH((conv_wgrad_f3_kernel<64, 0, 3>), grid, dim3(512), 0, stream, p, ta, tk);
        } else if (TA == 256) {
            if (ps == 1)
                FG_LAUNCH((conv_wgrad_f3_kernel<256, 0, 1>), grid, dim3(512), 0, stream, p, ta, tk);
            else if (ps == 2)
                FG_LAUNCH((conv_wgrad_f3_kernel<256, 0, 2>), grid, dim3(512), 0, stream, p, ta, tk);
            else
                FG_LAUNCH((conv_wgrad_f3_kernel<256, 0, 3>), grid, dim3(512), 0, stream, p, ta, tk);
        } else {
            if (ps == 1)
                FG_LAUNCH((conv_wgrad_f3_kernel<128, 1, 1>), grid, dim3(512), 0, stream, p, ta, tk);
            else if (ps == 2)
                FG_LAUNCH((conv_wgrad_f3_kernel<128, 1, 2>), grid, dim3(512), 0, stream, p, ta, tk);
            else
                FG_LAUNCH((conv_wgrad_f3_kernel<128, 1, 3>), grid, dim3(512), 0, stream, p, ta, tk);
        }
        *rc = fg::launched("conv_wgrad_f3_presplit");
        return 1;
    }
    // measured: the interleaved staging pays off on the 128-row tiles only
    const int sch = g_wgrad_f3 == 3 || (g_wgrad_f3 == 2 && TA == 128) ? 1 : 0;
    if (TA == 64)
        FG_LAUNCH((conv_wgrad_f3_kernel<64, 0>), grid, dim3(512), 0, stream, p, ta, tk);
    else if (TA == 256 && sch == 1)
        FG_LAUNCH((conv_wgrad_f3_kernel<256, 1>), grid, dim3(512), 0, stream, p, ta, tk);
    else if (TA == 256)
        FG_LAUNCH((conv_wgrad_f3_kernel<256, 0>), grid, dim3(512), 0, stream, p, ta, tk);
    else if (sch == 1)
        FG_LAUNCH((conv_wgrad_f3_kernel<128, 1>), grid, dim3(512), 0, stream, p, ta, tk);
    else
        FG_LAUNCH((conv_wgrad_f3_kernel<128, 0>), grid, dim3(512), 0, stream, p, ta, tk);
    *rc = fg::launched("conv_wgrad_f3");
    return 1;
}

}  // namespace fgc

FG_API int fg_set_wgrad_f3(int on) {
    if (on < 0 || on > 3) return fg::fail(FG_ERR_INVALID, "fg_set_wgrad_f3: %d", on);
    g_wgrad_f3 = on;
    return 0;
}
