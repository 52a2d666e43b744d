// The generator stem's weight gradient: the 7x7 conv over the reflect-padded 9-channel input with 64
// output channels (models/model_architectures.py:312, :342-343; convolution_backward's weight gradient):
//
//   out[split][a][r*63 + j] = sum over the split's output pixels (y, x) of  gy[y][x][a] * xpad[y + r][9 x + j]
//
// with j = s*9 + c, so that for one kernel row r the 63 k-columns of an output pixel are the 63 CONTIGUOUS
// values of the padded input row starting at its own 9 channels.  A workgroup owns a 64-px column strip of
// `rows` output rows of one image and walks down it: each step stages ONE new input row of the strip (70 px x 9
// channels, split once into the scaled fp16 pieces h, l) into a ring of 8 LDS rows -- the 7 kernel rows read
// the ring, so the input is fetched once per strip instead of once per tap -- and the gradient row (64 px x 64
// channels, split once).  v_mfma_f32_16x16x32_f16 with the reduction over 32 consecutive pixels: the gradient
// operand is a transposed read (ds_read_b64_tr_b16) of its [px][channel] image; the input operand a
// transposed read of the flat input row, 8 B aligned through four copies of each row shifted by 0..3
// elements (a lane reading pixel q of its group uses copy (4 - q) & 3).  The 64 x 448 (63 per r, one padding
// column) product of a step is split over 8 waves: waves 0-3 own 4 column blocks of 16, waves 4-7 three, each
// all 64 output channels, so every SIMD carries 7 blocks.  One fp32 partial slab per workgroup
// (fg_wgrad_reduce sums them).  Replaces conv_wgrad_x6 for this shape (2x its algorithmic bytes).
#include <algorithm>

#include "conv_common.hpp"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int ST_C = 9, ST_J = 63, ST_K = 7 * ST_J, ST_N = 64;
constexpr int ST_PX = 64;                        // output pixels per strip (two reductions of 32)
constexpr int ST_FLAT = (ST_PX + 6) * ST_C;      // 630 flat input values per strip row
constexpr int ST_COPY = 640;                     // fp16 per shifted copy (>= 630 + 3 + the 4 of the last read)
constexpr int ST_COPYB = ST_COPY * 2;
constexpr int ST_PIECE = 4 * ST_COPYB;           // the four shifted copies of one piece
constexpr int ST_XROW = 2 * ST_PIECE;            // h, l
constexpr int ST_RING = 8;                       // 7 rows in use + the one being staged
constexpr int ST_GIMG = ST_PX * ST_N * 2;        // gradient row image per piece: [64 px][64 ch] fp16
constexpr int ST_GBUF = 2 * ST_GIMG;
constexpr int ST_LDS = ST_RING * ST_XROW + 2 * ST_GBUF;   // 114688 B
constexpr int kOOB = 0x7fffffff;

// 32-B column-pair swizzle of the gradient image (conv_wgrad_f3.hip): the 8 pixel rows a 32-lane half of a
// transposed read touches land on distinct bank groups
__device__ __forceinline__ int swz_tr(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int gimg_off(int row, int col) {
    return row * (ST_N * 2) + (((col >> 3) ^ (swz_tr(row) & 7)) << 4) + ((col & 7) << 1);
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
        fgc::split_pair_mix(v[2 * e], v[2 * e + 1], s, a, b);
        hu[e] = a;
        lu[e] = b;
    }
    h = __builtin_bit_cast(f16x4, hu);
    l = __builtin_bit_cast(f16x4, lu);
}

__global__ void __launch_bounds__(512, 1) stem_wgrad_kernel(const fg_wgrad_problem P, int rows) {
    __shared__ __attribute__((aligned(1024))) char smem[ST_LDS];
    char* const xring = smem;
    char* const gbuf = smem + ST_RING * ST_XROW;

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int strips = P.m_b / ST_PX, groups = P.m_a / rows;
    const int split = blockIdx.x;
    const int img = split / (strips * groups);
    const int rem = split - img * strips * groups;
    const int grp = rem / strips, strip = rem - grp * strips;      // neighbouring blocks: neighbouring strips
    const int a0 = grp * rows, b0 = strip * ST_PX;
    const int nsteps = rows + 6;

    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)P.p, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
    const float sp = fgc::pow2_scale(P.p_absmax);
    const float sx = fgc::pow2_scale(P.x_absmax);

    // the shifted copies' unwritten heads / tails read as zeros
    for (int i = tid; i < ST_RING * ST_XROW / 16; i += 512) reinterpret_cast<f32x4*>(xring)[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- staging: flat input values e = tid, tid + 512 (< 630) of row a0 + li; gradient float4 slots
    // (px = tid / 16 + 32 i, channels 4 (tid % 16) ..) of output row a0 + li - 6
    const int gpx = tid >> 4, gch = (tid & 15) * 4;
    const bool x2 = tid + 512 < ST_FLAT;
    const int xbase = img * (int)P.sxn + b0 * ST_C;
    const int gbase = img * (int)P.spn + b0 * (int)P.spb + gch;
    float rx0 = 0.f, rx1 = 0.f;
    f32x4 rg0 = {0.f, 0.f, 0.f, 0.f}, rg1 = rg0;
    auto load = [&](int li) {
        const bool ok = li < nsteps;
        const int xo = xbase + (a0 + li) * (int)P.sxr + tid;
        rx0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, ok ? xo * 4 : kOOB, 0, 0));
        rx1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, ok && x2 ? (xo + 512) * 4 : kOOB, 0, 0));
        const bool gok = ok && li >= 6;
        const int go = gbase + (a0 + li - 6) * (int)P.spa + gpx * (int)P.spb;
        rg0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, gok ? go * 4 : kOOB, 0, 0));
        rg1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            pr, gok ? (go + 32 * (int)P.spb) * 4 : kOOB, 0, 0));
    };
    auto put_x = [&](char* xs, int e, float v) {
        const float vs = v * sx;
        const _Float16 h = (_Float16)vs;
        const _Float16 l = (_Float16)(vs - (float)h);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            *reinterpret_cast<_Float16*>(xs + t * ST_COPYB + 2 * (e + t)) = h;
            *reinterpret_cast<_Float16*>(xs + ST_PIECE + t * ST_COPYB + 2 * (e + t)) = l;
        }
    };
    auto store = [&](int li) {
        char* xs = xring + (li & (ST_RING - 1)) * ST_XROW;
        put_x(xs, tid, rx0);
        if (x2) put_x(xs, tid + 512, rx1);
        if (li >= 6) {
            char* gb = gbuf + (li & 1) * ST_GBUF;
            f16x4 h, l;
            split4(rg0, sp, h, l);
            *reinterpret_cast<f16x4*>(gb + gimg_off(gpx, gch)) = h;
            *reinterpret_cast<f16x4*>(gb + ST_GIMG + gimg_off(gpx, gch)) = l;
            split4(rg1, sp, h, l);
            *reinterpret_cast<f16x4*>(gb + gimg_off(gpx + 32, gch)) = h;
            *reinterpret_cast<f16x4*>(gb + ST_GIMG + gimg_off(gpx + 32, gch)) = l;
        }
    };

    // ---- column blocks: t = 4 r + ct (ct: columns 16 ct .. of kernel row r); waves 0-3 own t = 4w .. 4w+3,
    // waves 4-7 own t = 16 + 3 (w - 4) .. +2
    const int t0 = wave < 4 ? 4 * wave : 16 + 3 * (wave - 4);
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
    const int cp = (4 - q) & 3;                     // the shifted copy that makes this lane's read 8-B aligned
    f32x4 acc[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[mt][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int k, auto NTW) {
        constexpr int NT = decltype(NTW)::value;
        const char* gb = gbuf + (k & 1) * ST_GBUF;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            f16x8 ah[4], al[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int c = mt * 16 + p4;
                const int o0 = gimg_off(32 * kk + 8 * g + q, c), o1 = gimg_off(32 * kk + 8 * g + 4 + q, c);
                ah[mt] = tr_frag(gb, o0, o1);
                al[mt] = tr_frag(gb + ST_GIMG, o0, o1);
            }
            const int f0 = 9 * (32 * kk + 8 * g + q) + p4 + cp;
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const int t = t0 + i, r = t >> 2, ct = t & 3;
                const char* xs = xring + ((k - 6 + r) & (ST_RING - 1)) * ST_XROW + cp * ST_COPYB;
                const int ad = 2 * (f0 + 16 * ct);
                const f16x8 bh = tr_frag(xs, ad, ad + 72);
                const f16x8 bl = tr_frag(xs + ST_PIECE, ad, ad + 72);
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    acc[mt][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[mt], bh, acc[mt][i], 0, 0, 0);
                    acc[mt][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mt], bl, acc[mt][i], 0, 0, 0);
                    acc[mt][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[mt], bh, acc[mt][i], 0, 0, 0);
                }
            }
        }
    };

    // ---- write-after-barrier pipeline: step k stores step k+1's registers (ring slot (k+1) & 7 and gradient
    // buffer (k+1) & 1 are not read by step k), refills them with step k+2 and reduces output row k - 6
    __syncthreads();
    load(0);
    store(0);
    load(1);
    __syncthreads();
    for (int k = 0; k < nsteps; ++k) {
        if (k + 1 < nsteps) store(k + 1);
        load(k + 2);
        if (k >= 6) {
            if (wave < 4)
                compute(k, std::integral_constant<int, 4>{});
            else
                compute(k, std::integral_constant<int, 3>{});
        }
        __syncthreads();
    }

    // ---- epilogue: scaled fp32 slab rows a (output channels), columns r*63 + j
    float* out = P.out + (size_t)split * ST_N * ST_K;
    const float osc = 1.f / (sp * sx);
    const int fr = lane & 15;
    const int ntw = wave < 4 ? 4 : 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i >= ntw) break;
        const int t = t0 + i, r = t >> 2, j = 16 * (t & 3) + fr;
        if (j >= ST_J) continue;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg)
                out[(size_t)(mt * 16 + 4 * g + reg) * ST_K + r * ST_J + j] = acc[mt][i][reg] * osc;
    }
}

// The forward's ring: copies 1-3 of each piece start 8 B past their 1280-B slot, so that the 32 lanes of a fragment
// read (16 pixels x 2 k groups, each lane on the copy of its pixel's alignment) hit 64 distinct banks -- with the
// copies 320 dwords (0 mod 64) apart the reads were 3-way conflicted (half of the kernel's LDS cycles were
// SQ_LDS_BANK_CONFLICT in round 4; after the offsets: profiles/round4/r4l_pmc_stem_fwd.json, round 5 in-step:
// profiles/round5/r5_pmc_stem_fwd.json)
constexpr int SF_PIECE = 4 * ST_COPYB + 16;
constexpr int SF_XROW = 2 * SF_PIECE;
__device__ __forceinline__ int sf_copy(int t) { return t * ST_COPYB + (t ? 8 : 0); }

// ---- the stem's forward: y[px][n] = bias[n] + sum_r sum_{j<63} xpad[a + r][9 px + j] * w[n][r*64 + j]
// 8 waves (two per SIMD) over a 64-px strip walking down `rows` output rows with the same 8-row input ring.  The
// weights (64 x 448, pre-split fp16) stay in REGISTERS for the whole launch: wave (nh, ph, kh) holds output channels
// 32 nh .. +31 for reductions 7 kh .. 7 kh + 6 of 14 (two 16-row MFMA blocks x 7 reductions of 32 x 2 pieces = 112
// VGPRs) and computes pixels 32 ph .. +31 of every row, as C^T[channel][pixel] = W[channel][k] X^T[k][pixel] on
// v_mfma_f32_16x16x32_f16; the K halves meet in LDS (double-buffered 16 KB) and the kh = 0 waves finish the row.
// The input operand (8 consecutive flat values per lane) comes from the shifted copies with two 8-B aligned reads
// (copy (4 - px % 4) % 4).  A lane's accumulator holds 4 consecutive channels of one pixel: one 16-B store, and
// each wave's 32 pixels are one InstanceNorm statistics block (mean, M2 per channel) of the epilogue.
__global__ void __launch_bounds__(512, 1) stem_fwd_kernel(const fg_conv_problem P, int rows) {
    constexpr int RED = 4 * 64 * 16 * 4;            // the kh = 1 partials of one row: 4 waves x 64 lanes x 16 floats
    __shared__ __attribute__((aligned(1024))) char smem[ST_RING * SF_XROW + 2 * RED];
    char* const xring = smem;
    float* const red = reinterpret_cast<float*>(smem + ST_RING * SF_XROW);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nh = wave & 1, ph = (wave >> 1) & 1, kh = wave >> 2;
    const int strips = P.m_b / ST_PX, groups = P.m_a / rows;
    const int split = blockIdx.x;
    const int img = split / (strips * groups);
    const int rem = split - img * strips * groups;
    const int grp = rem / strips, strip = rem - grp * strips;
    const int a0 = grp * rows, b0 = strip * ST_PX;
    const int nsteps = rows + 6;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
    const float sx = fgc::pow2_scale(P.x_absmax);
    const float sw = fgc::pow2_scale(P.w_absmax);
    const float osc = 1.f / (sx * sw);
    const int g = lane >> 4, fr = lane & 15;

    for (int i = tid; i < ST_RING * SF_XROW / 16; i += 512) reinterpret_cast<f32x4*>(xring)[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // weights: fragment (reduction 7 kh + i, block nt, piece) = the lane's 8 k of output channel 32 nh + 16 nt + fr
    f16x8 wf[7][2][2];
    {
        const f16x8* wp = reinterpret_cast<const f16x8*>(P.w);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int n = 32 * nh + 16 * nt + fr;
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                const int q = n * (P.ldw / 8) + (7 * kh + i) * 4 + g;
                wf[i][nt][0] = wp[q * 2];
                wf[i][nt][1] = wp[q * 2 + 1];
            }
        }
    }
    float bias[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) bias[nt][i] = P.bias ? P.bias[32 * nh + 16 * nt + 4 * g + i] : 0.f;

    // staging: flat values e = tid, tid + 512 (< 630) of input row a0 + li
    float rx[2];
    const int xbase = img * (int)P.sxn + b0 * ST_C + tid;
    auto load = [&](int li) {
        const bool ok = li < nsteps;
        const int xo = xbase + (a0 + li) * (int)P.sxr;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            rx[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  xr, ok && tid + 512 * i < ST_FLAT ? (xo + 512 * i) * 4 : kOOB, 0, 0));
    };
    auto store = [&](int li) {
        char* xs = xring + (li & (ST_RING - 1)) * SF_XROW;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + 512 * i;
            if (e >= ST_FLAT) continue;
            const float vs = rx[i] * sx;
            const _Float16 h = (_Float16)vs;
            const _Float16 l = (_Float16)(vs - (float)h);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                *reinterpret_cast<_Float16*>(xs + sf_copy(t) + 2 * (e + t)) = h;
                *reinterpret_cast<_Float16*>(xs + SF_PIECE + sf_copy(t) + 2 * (e + t)) = l;
            }
        }
    };

    const int cp = (4 - (lane & 3)) & 3;             // px % 4 == lane % 4 (strip and block origins are x 16)
    const int mab = P.m_a * P.m_b;
    f32x4 acc[2][2];
    auto compute_row = [&](int k) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) acc[nt][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int ks = 7 * kh + i, r = ks >> 1, kk = ks & 1;
            const char* xs = xring + ((k - 6 + r) & (ST_RING - 1)) * SF_XROW + sf_copy(cp);
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
                const int px = 32 * ph + 16 * pt + fr;
                const int ad = 2 * (9 * px + 32 * kk + 8 * g + cp);
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const u32x2 h0 = *reinterpret_cast<const u32x2*>(xs + ad);
                const u32x2 h1 = *reinterpret_cast<const u32x2*>(xs + ad + 8);
                const u32x2 l0 = *reinterpret_cast<const u32x2*>(xs + SF_PIECE + ad);
                const u32x2 l1 = *reinterpret_cast<const u32x2*>(xs + SF_PIECE + ad + 8);
                const f16x8 bh = __builtin_bit_cast(f16x8, u32x4{h0[0], h0[1], h1[0], h1[1]});
                const f16x8 bl = __builtin_bit_cast(f16x8, u32x4{l0[0], l0[1], l1[0], l1[1]});
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    acc[nt][pt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[i][nt][1], bh, acc[nt][pt], 0, 0, 0);
                    acc[nt][pt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[i][nt][0], bl, acc[nt][pt], 0, 0, 0);
                    acc[nt][pt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[i][nt][0], bh, acc[nt][pt], 0, 0, 0);
                }
            }
        }
    };
    // the kh = 0 wave of (nh, ph): add the kh = 1 partials, store the row and its statistics
    auto finish_row = [&](int k, f32x4 (&acc)[2][2]) {
        const float* rb_ = red + ((k & 1) * 4 + (wave & 3)) * 64 * 16 + lane * 4;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) acc[nt][pt] += *reinterpret_cast<const f32x4*>(rb_ + (nt * 2 + pt) * 256);
        const int a = a0 + k - 6;
        float* yrow = P.y + img * P.syn + a * P.sya + (b0 + 32 * ph) * P.syb;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
                f32x4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = acc[nt][pt][i] * osc + bias[nt][i];
                *reinterpret_cast<f32x4*>(yrow + (16 * pt + fr) * P.syb + 32 * nh + 16 * nt + 4 * g) = v;
            }
        if (P.in_stats) {
            // (mean, M2) of each channel over the 32 pixels (16 lanes x 2 blocks), from the raw accumulators
            const int rb = (img * mab + a * P.m_b + b0 + 32 * ph) / 32;
            float* dst = P.in_stats + (size_t)rb * P.n_out * 2;
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float s = acc[nt][0][i] + acc[nt][1][i];
                    s = fg::row_sum16(s);
                    const float mu = s * (1.f / 32);
                    const float d0 = acc[nt][0][i] - mu, d1 = acc[nt][1][i] - mu;
                    float q = d0 * d0 + d1 * d1;
                    q = fg::row_sum16(q);
                    if (fr == 0) {
                        const int ch = 32 * nh + 16 * nt + 4 * g + i;
                        *reinterpret_cast<float2*>(dst + ch * 2) = make_float2(mu * osc + bias[nt][i], q * (osc * osc));
                    }
                }
        }
    };

    // step k: the MFMAs of output row k - 6 (ring rows k-6 .. k) are issued first; behind them, while they run, input row
    // k + 1 is stored (ring slot (k+1) & 7, not read by row k - 6), row k + 2 loaded and -- in the kh = 0 waves -- the
    // PREVIOUS row finished (its kh = 1 partials in red[(k-1) & 1], its own accumulators saved in accp), so the
    // epilogue no longer sits between two barriers with the kh = 1 waves idle.  The kh = 1 waves leave this row's
    // partials in red[k & 1] (red[(k+1) & 1] was read before this step's barrier).
    __syncthreads();
    load(0);
    store(0);
    load(1);
    __syncthreads();
    f32x4 accp[2][2];
    for (int k = 0; k < nsteps; ++k) {
        if (k >= 6) compute_row(k);
        if (k + 1 < nsteps) store(k + 1);
        load(k + 2);
        if (k >= 7 && !kh) finish_row(k - 1, accp);
        if (k >= 6) {
            if (kh) {
                float* rb_ = red + ((k & 1) * 4 + (wave & 3)) * 64 * 16 + lane * 4;
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int pt = 0; pt < 2; ++pt) *reinterpret_cast<f32x4*>(rb_ + (nt * 2 + pt) * 256) = acc[nt][pt];
            } else {
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int pt = 0; pt < 2; ++pt) accp[nt][pt] = acc[nt][pt];
            }
        }
        __syncthreads();
    }
    if (!kh && nsteps > 6) finish_row(nsteps - 1, accp);
}

}  // namespace

namespace fgc {

// rows per workgroup of the stem forward (conv_stem.hip), or 0 when it does not take the problem: the 7x7 conv over a
// 9-channel reflect-padded input with 64 f16x3 outputs written NHWC (bias, no activation / accumulation), 64-px
// strips; about one workgroup per CU
int stem_fwd_rows(const fg_conv_problem& p) {
    if (p.kh != 7 || p.j_valid != ST_J || p.jp != 64 || p.ldw != 448 || p.sxb != ST_C || p.sxa != p.sxr ||
        p.n_out != ST_N || p.w_split != 2 || p.x_presplit || p.act || p.accumulate || p.syc != 1 || p.syb % 4 ||
        (p.sya | p.syn) % 4 || ((uintptr_t)p.y & 15) || ((uintptr_t)p.w & 15) || !p.x_absmax || !p.w_absmax ||
        p.m_b % ST_PX || p.m_a < 1 || p.m_img < 1)
        return 0;
    const long long xext = 4 * ((long long)(p.m_img - 1) * p.sxn + (long long)(p.m_a + 6) * p.sxr + p.m_b * ST_C + 64);
    const long long yext = 4 * ((long long)(p.m_img - 1) * p.syn + (long long)p.m_a * p.sya + (long long)p.m_b * p.syb);
    if (xext >= (1LL << 31) || yext >= (1LL << 31) || p.sxn < 0 || p.syn < 0) return 0;
    const long long strips = (long long)p.m_img * (p.m_b / ST_PX);
    const int want = (int)std::max(1LL, (strips * p.m_a + 255) / 256);
    for (int r = want; r <= p.m_a; ++r)
        if (p.m_a % r == 0) return r;
    return p.m_a;
}

int launch_fwd_stem(const fg_conv_problem& p, hipStream_t stream, int* rc) {
    const int rows = stem_fwd_rows(p);
    if (!rows) return 0;
    const int grid = p.m_img * (p.m_b / ST_PX) * (p.m_a / rows);
    FG_LAUNCH(stem_fwd_kernel, dim3(grid), dim3(512), 0, stream, p, rows);
    *rc = fg::launched("stem_fwd");
    return 1;
}

int stem_wgrad_rows(const fg_wgrad_problem& p) {
    // rows per split encoded as m_chunk = 64 * rows (a 64-px strip of `rows` output rows per workgroup)
    if (p.n_a != ST_N || p.kh != 7 || p.j_valid != ST_J || p.sxb != ST_C || p.sxr != p.sxa || p.m_b % ST_PX ||
        p.m_chunk % ST_PX || p.p_presplit || p.x_presplit || !p.p_absmax || !p.x_absmax || ((uintptr_t)p.p & 15) ||
        (p.spn | p.spa | p.spb) % 4 || p.spb < ST_N)
        return 0;
    const int rows = p.m_chunk / ST_PX;
    if (rows < 1 || p.m_a % rows || (long long)p.splits != (long long)p.m_img * (p.m_b / ST_PX) * (p.m_a / rows))
        return 0;
    return rows;
}

// Returns 1 when the stem kernel took the problem (status in *rc), 0 when it does not apply.
int launch_wgrad_stem(const fg_wgrad_problem& p, hipStream_t stream, int* rc) {
    const int rows = stem_wgrad_rows(p);
    if (!rows) return 0;
    FG_LAUNCH(stem_wgrad_kernel, dim3(p.splits), dim3(512), 0, stream, p, rows);
    *rc = fg::launched("stem_wgrad");
    return 1;
}

}  // namespace fgc
