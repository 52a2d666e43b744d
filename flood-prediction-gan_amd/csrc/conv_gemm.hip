// Implicit-GEMM convolution engine on fp32 MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
// One forward kernel serves every conv geometry of the PairedAttention hot path
// (models/model_architectures.py:312-334, :424-438): stride-1/2 convs over pre-padded NHWC
// inputs, stride-1 input gradients (full correlation with flipped weights), and each output
// phase of the stride-2 transposed convs / stride-2 input gradients (sub-pixel
// decomposition: phases are independent dense convs with 1, 2 or 4 taps).  Padding is never
// handled here: producers write reflect / zero borders into the operand buffers, so the
// A-operand gather is a pure affine address  x[row_x(m) + r*sxr + j]  where, for a fixed
// kernel row r, the (kernel column, channel) pairs are one contiguous run j < kw*C.
//
// Tiling: BM x BN output tile per 256-thread workgroup, BK = 16, 4 waves each owning a
// WM x WN sub-tile of 32x32 MFMA blocks.  Both operands are staged k-contiguous in LDS
// (row pitch BK+4 floats, conflict-free ds_read_b128), register-staged double buffering
// with one barrier per k-tile.  Lane l of half h = l>>5 feeds k = 8q + 4h + t at MFMA
// step t of quad q, identically for A and B, so each MFMA sums matching k.
//
// The weight-gradient kernel reduces over the M (pixel) dimension instead: both operands
// stay row(pixel)-major in LDS, split-M partial slabs are summed by wgrad_reduce.
#include <algorithm>

#include "conv_common.hpp"

namespace {

constexpr int BK = 16;
constexpr int LDK = BK + 4;
int g_conv_math = FG_MATH_F16X3;    // default: scaled split-fp16 (accuracy: scripts/bench_conv.py, tests/)

using fgc::ConvBatch;
using fgc::decomp;
using fgc::pow2_scale;

template <int BM, int BN, int WM, int WN, bool VEC>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64)
conv_fwd_kernel(const ConvBatch batch) {
    constexpr int NWN = BN / WN;
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr int A_SLOTS = BM * (BK / 4), B_SLOTS = BN * (BK / 4);
    constexpr int A_IT = (A_SLOTS + NT - 1) / NT, B_IT = (B_SLOTS + NT - 1) / NT;

    __shared__ __attribute__((aligned(16))) float As[2][BM][LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / NWN, wn = wave - (wave / NWN) * NWN;

    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    int pi = 0;
    while (pi + 1 < batch.count && wid >= batch.blk_start[pi + 1]) ++pi;
    const fg_conv_problem& P = batch.p[pi];
    const int local = wid - batch.blk_start[pi];
    const int ntn = batch.ntiles_n[pi];
    const int mt = local / ntn, nt = local - (local / ntn) * ntn;
    const int m0 = mt * BM, n0 = nt * BN;
    const int mab = P.m_a * P.m_b;
    const int M = P.m_img * mab;
    const int jtr = P.jp / BK;
    const int nkt = P.kh * jtr;
    const int jv = P.j_valid;
    const long long sxr = P.sxr;

    // ---- per-thread staging slots ----
    const float* arow[A_IT];
    int arow_i[A_IT], aq[A_IT];
    bool aok[A_IT];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
        const int s = tid + i * NT;
        arow_i[i] = s >> 2;
        aq[i] = s & 3;
        const int m = m0 + (s >> 2);
        aok[i] = (s < A_SLOTS) && (m < M);
        arow[i] = P.x;
        if (aok[i]) {
            int img, a, b;
            decomp(m, P.m_b, mab, img, a, b);
            arow[i] = P.x + img * P.sxn + a * P.sxa + b * P.sxb;
        }
    }
    const float* brow[B_IT];
    int brow_i[B_IT], bq[B_IT];
    bool bok[B_IT], bslot[B_IT];
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
        const int s = tid + i * NT;
        brow_i[i] = s >> 2;
        bq[i] = s & 3;
        bslot[i] = s < B_SLOTS;
        bok[i] = bslot[i] && (n0 + (s >> 2) < P.n_out);
        brow[i] = P.w + (size_t)(bok[i] ? n0 + (s >> 2) : 0) * P.ldw;
    }

    f32x4 ra[A_IT], rb[B_IT];
    auto load = [&](int kt) {
        const int r = kt / jtr;
        const int jb = (kt - r * jtr) * BK;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int j = jb + aq[i] * 4;
            if (aok[i]) {
                const float* src = arow[i] + r * sxr + j;
                if constexpr (VEC) {
                    if (j < jv) v = *reinterpret_cast<const f32x4*>(src);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (j + e < jv) v[e] = src[e];
                }
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (bok[i]) v = *reinterpret_cast<const f32x4*>(brow[i] + kt * BK + bq[i] * 4);
            rb[i] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i)
            if (tid + i * NT < A_SLOTS)
                *reinterpret_cast<f32x4*>(&As[buf][arow_i[i]][aq[i] * 4]) = ra[i];
#pragma unroll
        for (int i = 0; i < B_IT; ++i)
            if (bslot[i]) *reinterpret_cast<f32x4*>(&Bs[buf][brow_i[i]][bq[i] * 4]) = rb[i];
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

    const int lrow = lane & 31, lk = (lane >> 5) * 4;
    if (nkt > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) load(kt + 1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            f32x4 af[TM], bf[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
                af[tm] = *reinterpret_cast<const f32x4*>(&As[cur][wm * WM + tm * 32 + lrow][q * 8 + lk]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                bf[tn] = *reinterpret_cast<const f32x4*>(&Bs[cur][wn * WN + tn * 32 + lrow][q * 8 + lk]);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm][t], bf[tn][t],
                                                                           acc[tm][tn], 0, 0, 0);
        }
        if (kt + 1 < nkt) store(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: bias + activation, strided store (or accumulate) ----
    const int act = P.act;
    const bool accum = P.accumulate != 0;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wm * WM + tm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
            const int m = m0 + row;
            if (m >= M) continue;
            int img, a, b;
            decomp(m, P.m_b, mab, img, a, b);
            float* yrow = P.y + img * P.syn + a * P.sya + b * P.syb;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WN + tn * 32 + lrow;
                if (n >= P.n_out) continue;
                float v = acc[tm][tn][reg];
                if (P.bias) v += P.bias[n];
                v = fg::act_fwd(v, act);
                float* dst = yrow + n * P.syc;
                if (accum) v += *dst;
                *dst = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Split-bf16 forward kernel ("bf16x6"): fp32-equivalent products on bf16 MFMA.
//
// Every fp32 operand v is split at staging time into three bf16 pieces v = h + m + l
// (h = bf16(v), m = bf16(v - h), l = bf16(v - h - m): 3 x 8 significant bits = the 24 of fp32).
// A*B is accumulated in fp32 from the six bf16 products whose order is <= 2^-16:
//     hh + hm + mh + hl + lh + mm            (dropped: ml, lm ~2^-24, ll ~2^-32)
// bf16 x bf16 products are exact in fp32, so the result carries fp32-level error
// (|dropped| <= 3*2^-24 relative, the same order as fp32 rounding) while the MFMA rate is
// 6 x v_mfma_f32_32x32x16_bf16 (192 cycles) per 32x32x16 block instead of 8 x
// v_mfma_f32_32x32x2_f32 (512 cycles): 2.67x the fp32 matrix peak.
// Operand layout in LDS: [buf][piece][row][k] bf16, 16 k per stage, row pitch 24 bf16 (48 B:
// conflict-free ds_read_b128 fragment reads).  Lane l feeds rows l&31, k = 8(l>>5)..+7.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Split of two fp32 values at once: v_cvt_pk_bf16_f32 (RNE) + v_pk_add_f32 (exact residuals).
__device__ __forceinline__ void split3x2(float a, float b, bf16x2& h, bf16x2& m, bf16x2& l) {
    const f32x2 x = {a, b};
    h = __builtin_convertvector(x, bf16x2);
    const f32x2 r = x - __builtin_convertvector(h, f32x2);
    m = __builtin_convertvector(r, bf16x2);
    const f32x2 r2 = r - __builtin_convertvector(m, f32x2);
    l = __builtin_convertvector(r2, bf16x2);
}

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        bf16x2 hh, mm, ll;
        split3x2(v[2 * e], v[2 * e + 1], hh, mm, ll);
        h[2 * e] = hh[0];
        h[2 * e + 1] = hh[1];
        m[2 * e] = mm[0];
        m[2 * e + 1] = mm[1];
        l[2 * e] = ll[0];
        l[2 * e + 1] = ll[1];
    }
}

// ------------------------------------------------------------------------------------------
// Split-fp16 variant ("f16x3"): every operand is scaled by an exact power of two s (so that
// |v*s| < 2^14, from the operand's absolute maximum) and split into two fp16 pieces
// v*s = h + l (h = fp16(v*s), l = fp16(v*s - h): 11 + 11 significant bits, representation
// error <= 2^-22 |v|).  Three exact fp16 products hh + hl + lh (dropped: ll ~2^-22) are
// accumulated in fp32 by v_mfma_f32_32x32x16_f16 and the result is multiplied back by
// 1/(s_a s_b).  Half the MFMAs and 2/3 of the staging of bf16x6, at ~4x its per-product error
// (still far below the fp32 accumulation error of the convolution sums).
// ------------------------------------------------------------------------------------------

// split math traits: piece type, piece count, the products kept (PA[c] x PB[c], small first)
struct MathBF16x6 {
    using T = __bf16;
    using V8 = bf16x8;
    static constexpr int NP = 3, NPROD = 6;
    static constexpr int PA[6] = {1, 0, 2, 0, 1, 0};
    static constexpr int PB[6] = {1, 2, 0, 1, 0, 0};
    using V4 = __bf16 __attribute__((ext_vector_type(4)));
    static constexpr bool SCALED = false;
    __device__ static void split(const float (&v)[8], float, V8 (&o)[3]) { split3(v, o[0], o[1], o[2]); }
    __device__ static void split4(const f32x4& v, float, V4 (&o)[3]) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            bf16x2 h, m, l;
            split3x2(v[2 * e], v[2 * e + 1], h, m, l);
            o[0][2 * e] = h[0];
            o[0][2 * e + 1] = h[1];
            o[1][2 * e] = m[0];
            o[1][2 * e + 1] = m[1];
            o[2][2 * e] = l[0];
            o[2][2 * e + 1] = l[1];
        }
    }
    __device__ static f32x16 mfma(const V8& a, const V8& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
struct MathF16x3 {
    using T = _Float16;
    using V8 = f16x8;
    static constexpr int NP = 2, NPROD = 3;
    static constexpr int PA[3] = {1, 0, 0};
    static constexpr int PB[3] = {0, 1, 0};
    using V4 = f16x4;
    static constexpr bool SCALED = true;
    __device__ static void split4(const f32x4& v, float s, V4 (&o)[2]) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const f32x2 x = f32x2{v[2 * e], v[2 * e + 1]} * s;
            const f16x2 h = __builtin_convertvector(x, f16x2);
            const f16x2 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2);
            o[0][2 * e] = h[0];
            o[0][2 * e + 1] = h[1];
            o[1][2 * e] = l[0];
            o[1][2 * e + 1] = l[1];
        }
    }
    __device__ static void split(const float (&v)[8], float s, V8 (&o)[2]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const f32x2 x = f32x2{v[2 * e], v[2 * e + 1]} * s;
            const f16x2 h = __builtin_convertvector(x, f16x2);
            const f16x2 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2);
            o[0][2 * e] = h[0];
            o[0][2 * e + 1] = h[1];
            o[1][2 * e] = l[0];
            o[1][2 * e + 1] = l[1];
        }
    }
    __device__ static f32x16 mfma(const V8& a, const V8& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

template <class SM, int BM, int BN, int WM, int WN, bool VEC, bool WS, int MINW, int PF, bool SWZ>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, MINW)
conv_fwd_x6_kernel(const ConvBatch batch) {
    using T = typename SM::T;
    using V8 = typename SM::V8;
    constexpr int NP = SM::NP;
    constexpr int NWN = BN / WN;
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    constexpr int TM = WM / 32, TN = WN / 32;
    // bf16 per LDS row: 16 + 8 pad, or (SWZ) 16 with the two 8-k halves of a row swapped when
    // bit 3 of the row is set -- both conflict-free for the ds_read_b128 fragment reads
    constexpr int LDP = SWZ ? 16 : 24;
    constexpr int A_SLOTS = BM * 2, B_SLOTS = BN * 2;   // slot = 8 consecutive k of one row
    constexpr int A_IT = (A_SLOTS + NT - 1) / NT, B_IT = (B_SLOTS + NT - 1) / NT;

    __shared__ __attribute__((aligned(16))) T As[2][NP][BM][LDP];
    __shared__ __attribute__((aligned(16))) T Bs[2][NP][BN][LDP];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / NWN, wn = wave - (wave / NWN) * NWN;

    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    int pi = 0;
    while (pi + 1 < batch.count && wid >= batch.blk_start[pi + 1]) ++pi;
    const fg_conv_problem& P = batch.p[pi];
    const int local = wid - batch.blk_start[pi];
    const int ntn = batch.ntiles_n[pi];
    const int mt = local / ntn, nt = local - (local / ntn) * ntn;
    const int m0 = mt * BM, n0 = nt * BN;
    const int mab = P.m_a * P.m_b;
    const int M = P.m_img * mab;
    const int jtr = P.jp / 16;
    const int nkt = P.kh * jtr;
    const int jv = P.j_valid;
    const long long sxr = P.sxr;

    // Branch-free staging loads: buffer loads whose out-of-range offset (kOOB) returns zeros,
    // so the compiler can count vmcnt exactly across the pipelined loop.  fg_conv_fwd keeps
    // every byte offset below 2^31 (it splits the image range otherwise).
    constexpr bool A_FULL = A_SLOTS % NT == 0, B_FULL = B_SLOTS % NT == 0;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);
    int a_off[A_IT], a_r[A_IT], a_g[A_IT];
    bool aslot[A_IT];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
        const int s = tid + i * NT;
        a_r[i] = s >> 1;
        a_g[i] = s & 1;
        aslot[i] = A_FULL || s < A_SLOTS;
        const int m = m0 + (s >> 1);
        a_off[i] = -1;                                   // row outside the problem: loads read zeros
        if (aslot[i] && m < M) {
            int img, a, b;
            decomp(m, P.m_b, mab, img, a, b);
            a_off[i] = (int)(img * P.sxn + a * P.sxa + b * P.sxb) + a_g[i] * 8;
        }
    }
    // B: fp32 rows split at staging time, or (WS) pre-split rows of [slot][piece][8] bf16
    int b_off[B_IT], b_r[B_IT], b_g[B_IT];
    bool bslot[B_IT];
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
        const int s = tid + i * NT;
        b_r[i] = s >> 1;
        b_g[i] = s & 1;
        bslot[i] = B_FULL || s < B_SLOTS;
        const int n = n0 + (s >> 1);
        // byte offset of this slot's first k-slot (WS: NP x 16 B per 8-k slot, else 32 B of fp32)
        b_off[i] = (bslot[i] && n < P.n_out)
                       ? (WS ? (n * (P.ldw / 8) + b_g[i]) * NP * 16 : (n * P.ldw + b_g[i] * 8) * 4)
                       : -1;
    }
    constexpr int kOOB = 0x7fffffff;   // >= num_records: the load returns zeros
    // f16x3: operand scales (exact powers of two) and the epilogue's inverse
    const float sa = SM::SCALED ? pow2_scale(P.x_absmax) : 1.f;
    const float sb = SM::SCALED ? pow2_scale(P.w_absmax) : 1.f;
    const float out_scale = 1.f / (sa * sb);

    struct Stage {
        float ra[A_IT][8], rb[WS ? 1 : B_IT][8];
        V8 rbs[WS ? B_IT : 1][NP];
    };
    auto load = [&](int kt, Stage& S) {
        const int r = kt / jtr;
        const int jb = (kt - r * jtr) * 16;
        const int koff = r * (int)sxr + jb;              // element offset of this stage's k-run
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int j = jb + a_g[i] * 8;
            const int base = (a_off[i] + koff) * 4;
            if constexpr (VEC) {
                const int o0 = (a_off[i] >= 0 && j < jv) ? base : kOOB;
                const int o1 = (a_off[i] >= 0 && j + 4 < jv) ? base + 16 : kOOB;
                const f32x4 v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
                const f32x4 v1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    S.ra[i][e] = v0[e];
                    S.ra[i][4 + e] = v1[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int o = (a_off[i] >= 0 && j + e < jv) ? base + 4 * e : kOOB;
                    S.ra[i][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o, 0, 0));
                }
            }
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            if constexpr (WS) {
                const int o = b_off[i] >= 0 ? b_off[i] + kt * 32 * NP : kOOB;
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    S.rbs[i][p] = __builtin_bit_cast(V8, __builtin_amdgcn_raw_buffer_load_b128(
                                                             wr, o == kOOB ? kOOB : o + 16 * p, 0, 0));
            } else {
                const int o = b_off[i] >= 0 ? b_off[i] + kt * 64 : kOOB;
                const f32x4 v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, o, 0, 0));
                const f32x4 v1 = __builtin_bit_cast(f32x4,
                                                    __builtin_amdgcn_raw_buffer_load_b128(wr, o == kOOB ? kOOB : o + 16, 0, 0));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    S.rb[i][e] = v0[e];
                    S.rb[i][4 + e] = v1[e];
                }
            }
        }
    };
    auto store = [&](int buf, const Stage& S) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i)
            if (aslot[i]) {
                V8 pc[NP];
                SM::split(S.ra[i], sa, pc);
                const int c = (SWZ ? a_g[i] ^ ((a_r[i] >> 3) & 1) : a_g[i]) * 8;
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<V8*>(&As[buf][p][a_r[i]][c]) = pc[p];
            }
#pragma unroll
        for (int i = 0; i < B_IT; ++i)
            if (bslot[i]) {
                V8 pc[NP];
                if constexpr (WS) {
#pragma unroll
                    for (int p = 0; p < NP; ++p) pc[p] = S.rbs[i][p];
                } else {
                    SM::split(S.rb[i], sb, pc);
                }
                const int c = (SWZ ? b_g[i] ^ ((b_r[i] >> 3) & 1) : b_g[i]) * 8;
#pragma unroll
                for (int p = 0; p < NP; ++p) *reinterpret_cast<V8*>(&Bs[buf][p][b_r[i]][c]) = pc[p];
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

    const int lrow = lane & 31, lk = (SWZ ? (lane >> 5) ^ ((lane >> 3) & 1) : (lane >> 5)) * 8;
    auto compute = [&](int cur) {
        V8 af[TM][NP], bfr[TN][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
                af[tm][p] = *reinterpret_cast<const V8*>(&As[cur][p][wm * WM + tm * 32 + lrow][lk]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                bfr[tn][p] = *reinterpret_cast<const V8*>(&Bs[cur][p][wn * WN + tn * 32 + lrow][lk]);
        }
        // the kept piece products, smallest first; each product's (tm, tn) blocks interleaved
#pragma unroll
        for (int c = 0; c < SM::NPROD; ++c)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = SM::mfma(af[tm][SM::PA[c]], bfr[tn][SM::PB[c]], acc[tm][tn]);
    };
    Stage R0, R1;
    if constexpr (PF == 3) {
        // write-after-barrier: ONE register set; at the top of stage kt the registers holding
        // tile kt+1 (loaded during stage kt-1) go to the free LDS buffer and are refilled with
        // tile kt+2 at once, so every global load has a whole stage to land
        load(0, R0);
        store(0, R0);
        load(min(1, nkt - 1), R0);
        __syncthreads();
        for (int kt = 0; kt < nkt; ++kt) {
            const int cur = kt & 1;
            if (kt + 1 < nkt) store(cur ^ 1, R0);
            load(min(kt + 2, nkt - 1), R0);
            __builtin_amdgcn_sched_barrier(0);   // keep the loads issued ahead of this stage's MFMAs
            compute(cur);
            __syncthreads();
        }
    } else if constexpr (PF == 1) {
        load(0, R0);
        store(0, R0);
        __syncthreads();
        for (int kt = 0; kt < nkt; ++kt) {
            const int cur = kt & 1;
            load(min(kt + 1, nkt - 1), R0);
            compute(cur);
            if (kt + 1 < nkt) store(cur ^ 1, R0);
            __syncthreads();
        }
    } else {
        // prefetch distance 2: the global loads of stage kt+2 are issued before stage kt's
        // MFMAs and land in LDS only at the end of stage kt+1 (two register sets, loop x2)
        load(0, R0);
        load(min(1, nkt - 1), R1);
        store(0, R0);
        __syncthreads();
        // loads past the last stage are clamped (re-read the last stage, never stored): keeping
        // them unconditional lets the compiler count vmcnt exactly across iterations
        for (int kt = 0; kt < nkt; kt += 2) {
            load(min(kt + 2, nkt - 1), R0);
            compute(0);
            if (kt + 1 < nkt) store(1, R1);
            __syncthreads();
            if (kt + 1 >= nkt) break;
            load(min(kt + 3, nkt - 1), R1);
            compute(1);
            if (kt + 2 < nkt) store(0, R0);
            __syncthreads();
        }
    }

    const int act = P.act;
    const bool accum = P.accumulate != 0;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wm * WM + tm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
            const int m = m0 + row;
            if (m >= M) continue;
            int img, a, b;
            decomp(m, P.m_b, mab, img, a, b);
            float* yrow = P.y + img * P.syn + a * P.sya + b * P.syb;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WN + tn * 32 + lrow;
                if (n >= P.n_out) continue;
                float v = SM::SCALED ? acc[tm][tn][reg] * out_scale : acc[tm][tn][reg];
                if (P.bias) v += P.bias[n];
                v = fg::act_fwd(v, act);
                float* dst = yrow + n * P.syc;
                if (accum) v += *dst;
                *dst = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// weight gradient: out[split][a][k] = sum_m p[row_p(m)+a] * x[row_x(m)+koff(k)]
// ------------------------------------------------------------------------------------------
template <int BA, int BKC, int WA, int WK, bool VX, bool VP>
__global__ void __launch_bounds__((BA / WA) * (BKC / WK) * 64)
conv_wgrad_kernel(const fg_wgrad_problem P, int tiles_a, int tiles_k) {
    constexpr int NWK = BKC / WK;
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    constexpr int TM = WA / 32, TN = WK / 32;
    constexpr int BR = 16;
    constexpr int PADL = 4;
    constexpr int P_SLOTS = BR * BA / 4, X_SLOTS = BR * BKC / 4;
    constexpr int P_IT = (P_SLOTS + NT - 1) / NT, X_IT = (X_SLOTS + NT - 1) / NT;

    __shared__ __attribute__((aligned(16))) float Ps[2][BR][BA + PADL];
    __shared__ __attribute__((aligned(16))) float Xs[2][BR][BKC + PADL];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wa = wave / NWK, wk = wave - (wave / NWK) * NWK;

    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = tiles_a * tiles_k;
    const int split = wid / ntile;
    const int tile = wid - split * ntile;
    const int ta = tile / tiles_k, tk = tile - (tile / tiles_k) * tiles_k;
    const int a0 = ta * BA, k0 = tk * BKC;
    const int mab = P.m_a * P.m_b;
    const int M = P.m_img * mab;
    const int mbeg = split * P.m_chunk;
    const int mend = min(M, mbeg + P.m_chunk);
    const int K = P.kh * P.j_valid;
    const int nit = mend > mbeg ? (mend - mbeg + BR - 1) / BR : 0;

    // P slots (fixed columns)
    int p_row[P_IT], p_col[P_IT];
    bool p_slot[P_IT];
#pragma unroll
    for (int i = 0; i < P_IT; ++i) {
        const int s = tid + i * NT;
        p_slot[i] = s < P_SLOTS;
        p_row[i] = s / (BA / 4);
        p_col[i] = (s - (s / (BA / 4)) * (BA / 4)) * 4;
    }
    // X slots: fixed columns -> precomputed k offsets
    int x_row[X_IT], x_col[X_IT];
    bool x_slot[X_IT];
    long long x_off[X_IT][VX ? 1 : 4];
    bool x_kok[X_IT][VX ? 1 : 4];
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
        const int s = tid + i * NT;
        x_slot[i] = s < X_SLOTS;
        x_row[i] = s / (BKC / 4);
        x_col[i] = (s - (s / (BKC / 4)) * (BKC / 4)) * 4;
#pragma unroll
        for (int e = 0; e < (VX ? 1 : 4); ++e) {
            const int k = k0 + x_col[i] + e;
            x_kok[i][e] = k < K;
            const int kk = k < K ? k : 0;
            const int r = kk / P.j_valid;
            x_off[i][e] = r * P.sxr + (kk - r * P.j_valid);
        }
    }

    f32x4 rp[P_IT], rx[X_IT];
    auto load = [&](int it) {
        const int mb = mbeg + it * BR;
#pragma unroll
        for (int i = 0; i < P_IT; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int m = mb + p_row[i];
            if (p_slot[i] && m < mend) {
                int img, a, b;
                decomp(m, P.m_b, mab, img, a, b);
                const float* src = P.p + img * P.spn + a * P.spa + b * P.spb + a0 + p_col[i];
                const int na = P.n_a - (a0 + p_col[i]);
                if constexpr (VP) {
                    if (na > 0) {
                        v = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (e >= na) v[e] = 0.f;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (e < na) v[e] = src[e];
                }
            }
            rp[i] = v;
        }
#pragma unroll
        for (int i = 0; i < X_IT; ++i) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int m = mb + x_row[i];
            if (x_slot[i] && m < mend) {
                int img, a, b;
                decomp(m, P.m_b, mab, img, a, b);
                const float* base = P.x + img * P.sxn + a * P.sxa + b * P.sxb;
                if constexpr (VX) {
                    if (x_kok[i][0]) v = *reinterpret_cast<const f32x4*>(base + x_off[i][0]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (x_kok[i][e]) v[e] = base[x_off[i][e]];
                }
            }
            rx[i] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < P_IT; ++i)
            if (p_slot[i]) *reinterpret_cast<f32x4*>(&Ps[buf][p_row[i]][p_col[i]]) = rp[i];
#pragma unroll
        for (int i = 0; i < X_IT; ++i)
            if (x_slot[i]) *reinterpret_cast<f32x4*>(&Xs[buf][x_row[i]][x_col[i]]) = rx[i];
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

    const int lcol = lane & 31, lh = lane >> 5;
    if (nit > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
        const int cur = it & 1;
        if (it + 1 < nit) load(it + 1);
#pragma unroll
        for (int t = 0; t < BR / 2; ++t) {
            float af[TM], bf[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) af[tm] = Ps[cur][2 * t + lh][wa * WA + tm * 32 + lcol];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) bf[tn] = Xs[cur][2 * t + lh][wk * WK + tn * 32 + lcol];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
        }
        if (it + 1 < nit) store(cur ^ 1);
        __syncthreads();
    }

    float* out = P.out + (size_t)split * P.n_a * K;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int a = a0 + wa * WA + tm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * lh;
            if (a >= P.n_a) continue;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int k = k0 + wk * WK + tn * 32 + lcol;
                if (k < K) out[(size_t)a * K + k] = acc[tm][tn][reg];
            }
        }
}

// ------------------------------------------------------------------------------------------
// Split-bf16 weight gradient.  Both operands are staged in their natural pixel-major layout
// ([piece][m][column] bf16, 16 pixels per stage) from coalesced float4 loads, split into
// h/m/l pieces on the way (ds_write_b64 per piece), and the MFMA fragments -- which need 8
// consecutive pixels per lane -- are read with the gfx950 transposing LDS read
// ds_read_b64_tr_b16 (2 per fragment: pixels 0-3 and 4-7 of the lane's k-half).  Row pitch
// = columns + 32 bf16, so the four rows a 32-lane half reads land on disjoint banks.
// ------------------------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <class V8, class T>
__device__ __forceinline__ V8 tr_frag(const T* r0, const T* r4) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(r0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(r4));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(V8, v);
}

__device__ __forceinline__ void split3x4(const f32x4& v, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        bf16x2 hh, mm, ll;
        split3x2(v[2 * e], v[2 * e + 1], hh, mm, ll);
        h[2 * e] = hh[0];
        h[2 * e + 1] = hh[1];
        m[2 * e] = mm[0];
        m[2 * e + 1] = mm[1];
        l[2 * e] = ll[0];
        l[2 * e + 1] = ll[1];
    }
}

// LDS column swizzle of the weight-gradient staging tiles (pitch PITCH bf16, no padding): the
// transposed fragment reads touch 4 consecutive rows x 32 columns per 32-lane group; XOR-ing
// 32-column chunks by the row puts those 4 rows in 4 distinct 16-bank quarters.
template <int PITCH>
__device__ __forceinline__ int wg_swz(int row) {
    if constexpr (PITCH >= 128) return (row & 3) << 5;
    else if constexpr (PITCH == 64) return ((row >> 1) & 1) << 5;
    else return 0;
}

template <class SM, int BA, int BKC, int WA, int WK, bool VX, bool VP, int MINW, bool WAB>
__global__ void __launch_bounds__((BA / WA) * (BKC / WK) * 64, MINW)
conv_wgrad_x6_kernel(const fg_wgrad_problem P, int tiles_a, int tiles_k) {
    using T = typename SM::T;
    using V8 = typename SM::V8;
    using V4 = typename SM::V4;
    constexpr int NP = SM::NP;
    constexpr int NWK = BKC / WK;
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    constexpr int TM = WA / 32, TN = WK / 32;
    constexpr int BR = 16;                              // pixel rows per stage
    constexpr int P_SLOTS = BR * BA / 4, X_SLOTS = BR * BKC / 4;
    constexpr int P_IT = (P_SLOTS + NT - 1) / NT, X_IT = (X_SLOTS + NT - 1) / NT;
    constexpr bool P_FULL = P_SLOTS % NT == 0, X_FULL = X_SLOTS % NT == 0;
    constexpr int kOOB = 0x7fffffff;

    __shared__ __attribute__((aligned(16))) T Ps[2][NP][BR][BA];
    __shared__ __attribute__((aligned(16))) T Xs[2][NP][BR][BKC];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wa = wave / NWK, wk = wave - (wave / NWK) * NWK;
    const int wid = fg::xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = tiles_a * tiles_k;
    const int split = wid / ntile;
    const int tile = wid - split * ntile;
    const int ta = tile / tiles_k, tk = tile - (tile / tiles_k) * tiles_k;
    const int a0 = ta * BA, k0 = tk * BKC;
    const int mab = P.m_a * P.m_b;
    const int M = P.m_img * mab;
    const int mbeg = split * P.m_chunk;
    const int mend = min(M, mbeg + P.m_chunk);
    const int K = P.kh * P.j_valid;
    const int nit = mend > mbeg ? (mend - mbeg + BR - 1) / BR : 0;
    // advancing a pixel row index by BR = (i16 images, a16 rows, b16 columns)
    const int i16 = BR / mab, a16 = (BR - i16 * mab) / P.m_b, b16 = BR - i16 * mab - a16 * P.m_b;
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc((void*)P.p, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
    const float sp = SM::SCALED ? pow2_scale(P.p_absmax) : 1.f;
    const float sx = SM::SCALED ? pow2_scale(P.x_absmax) : 1.f;

    // per-slot pixel walk: slot rows are fixed within the stage, the pixel advances by BR
    struct Walk {
        int m, img, a, b;
    };
    auto walk_init = [&](int row) {
        Walk w;
        w.m = mbeg + row;
        decomp(min(w.m, M - 1), P.m_b, mab, w.img, w.a, w.b);
        return w;
    };
    auto walk_next = [&](Walk& w) {
        w.m += BR;
        w.b += b16;
        const int cb = w.b >= P.m_b;
        w.b -= cb ? P.m_b : 0;
        w.a += a16 + cb;
        const int ca = w.a >= P.m_a;
        w.a -= ca ? P.m_a : 0;
        w.img += i16 + ca;
    };

    int p_row[P_IT], p_col[P_IT], p_na[P_IT];
    bool p_slot[P_IT];
    Walk p_w[P_IT];
#pragma unroll
    for (int i = 0; i < P_IT; ++i) {
        const int s = tid + i * NT;
        p_slot[i] = P_FULL || s < P_SLOTS;
        p_row[i] = s / (BA / 4);
        p_col[i] = (s - (s / (BA / 4)) * (BA / 4)) * 4;
        p_na[i] = P.n_a - (a0 + p_col[i]);            // valid columns in this slot (<= 0: none)
        p_w[i] = walk_init(p_row[i]);
    }
    int x_row[X_IT], x_col[X_IT];
    bool x_slot[X_IT];
    int x_off[X_IT][VX ? 1 : 4];
    Walk x_w[X_IT];
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
        const int s = tid + i * NT;
        x_slot[i] = X_FULL || s < X_SLOTS;
        x_row[i] = s / (BKC / 4);
        x_col[i] = (s - (s / (BKC / 4)) * (BKC / 4)) * 4;
#pragma unroll
        for (int e = 0; e < (VX ? 1 : 4); ++e) {
            const int k = k0 + x_col[i] + e;
            const int r = k / P.j_valid;
            x_off[i][e] = k < K ? (int)(r * P.sxr) + (k - r * P.j_valid) : -1;
        }
        x_w[i] = walk_init(x_row[i]);
    }

    f32x4 rp[P_IT], rx[X_IT];
    // branch-free staging loads (out-of-range offsets read zeros), then advance the walks
    auto load = [&]() {
#pragma unroll
        for (int i = 0; i < P_IT; ++i) {
            const Walk& w = p_w[i];
            const int base = (w.img * (int)P.spn + w.a * (int)P.spa + w.b * (int)P.spb + a0 + p_col[i]) * 4;
            const bool ok = p_slot[i] && w.m < mend && p_na[i] > 0;
            f32x4 v;
            if constexpr (VP) {
                v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, ok ? base : kOOB, 0, 0));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         pr, ok && e < p_na[i] ? base + 4 * e : kOOB, 0, 0));
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e >= p_na[i]) v[e] = 0.f;
            rp[i] = v;
            walk_next(p_w[i]);
        }
#pragma unroll
        for (int i = 0; i < X_IT; ++i) {
            const Walk& w = x_w[i];
            const int base = w.img * (int)P.sxn + w.a * (int)P.sxa + w.b * (int)P.sxb;
            const bool ok = x_slot[i] && w.m < mend;
            f32x4 v;
            if constexpr (VX) {
                v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xr, ok && x_off[i][0] >= 0 ? (base + x_off[i][0]) * 4 : kOOB, 0, 0));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                         xr, ok && x_off[i][e] >= 0 ? (base + x_off[i][e]) * 4 : kOOB,
                                                         0, 0));
            }
            rx[i] = v;
            walk_next(x_w[i]);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < P_IT; ++i)
            if (p_slot[i]) {
                V4 pc[NP];
                SM::split4(rp[i], sp, pc);
                const int c = p_col[i] ^ wg_swz<BA>(p_row[i]);
#pragma unroll
                for (int q = 0; q < NP; ++q) *reinterpret_cast<V4*>(&Ps[buf][q][p_row[i]][c]) = pc[q];
            }
#pragma unroll
        for (int i = 0; i < X_IT; ++i)
            if (x_slot[i]) {
                V4 pc[NP];
                SM::split4(rx[i], sx, pc);
                const int c = x_col[i] ^ wg_swz<BKC>(x_row[i]);
#pragma unroll
                for (int q = 0; q < NP; ++q) *reinterpret_cast<V4*>(&Xs[buf][q][x_row[i]][c]) = pc[q];
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

    // transposed-read lane roles: group g = lane>>4 reads columns 16(g&1).. of pixel rows
    // 8(g>>1) + {0..3} and + {4..7}; lane 4q+p of the group addresses row q, columns 4p..4p+3
    const int g = lane >> 4, gi = lane & 15;
    const int tr_row = 8 * (g >> 1) + (gi >> 2);
    const int tr_col = 16 * (g & 1) + 4 * (gi & 3);
    const int swp = wg_swz<BA>(tr_row), swx = wg_swz<BKC>(tr_row);   // rows tr_row and tr_row+4 alike
    load();
    store(0);
    if constexpr (WAB) load();
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
        const int cur = it & 1;
        if constexpr (WAB) {
            // write-after-barrier: the registers (tile it+1, loaded a stage ago) go to the free
            // buffer first, then are refilled with tile it+2 ahead of this stage's MFMAs
            if (it + 1 < nit) store(cur ^ 1);
            load();
            __builtin_amdgcn_sched_barrier(0);
        } else {
            load();                     // past the last stage: reads zeros (m >= mend), never stored
        }
        V8 af[TM][NP], bfr[TN][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int c = (wa * WA + tm * 32 + tr_col) ^ swp;
                af[tm][p] = tr_frag<V8>(&Ps[cur][p][tr_row][c], &Ps[cur][p][tr_row + 4][c]);
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int c = (wk * WK + tn * 32 + tr_col) ^ swx;
                bfr[tn][p] = tr_frag<V8>(&Xs[cur][p][tr_row][c], &Xs[cur][p][tr_row + 4][c]);
            }
        }
#pragma unroll
        for (int c = 0; c < SM::NPROD; ++c)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = SM::mfma(af[tm][SM::PA[c]], bfr[tn][SM::PB[c]], acc[tm][tn]);
        if constexpr (!WAB)
            if (it + 1 < nit) store(cur ^ 1);
        __syncthreads();
    }

    float* out = P.out + (size_t)split * P.n_a * K;
    const float out_scale = 1.f / (sp * sx);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int a = a0 + wa * WA + tm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
            if (a >= P.n_a) continue;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int k = k0 + wk * WK + tn * 32 + (lane & 31);
                if (k < K) out[(size_t)a * K + k] = SM::SCALED ? acc[tm][tn][reg] * out_scale : acc[tm][tn][reg];
            }
        }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ slabs, int splits, fg_weight_map map,
                                    float* __restrict__ dw, int accumulate) {
    const int J = map.kw * map.c;
    const long long K = (long long)map.kh * J;
    const long long total = (long long)map.n_out * K;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int a = (int)(idx / K);
        const int k = (int)(idx - (long long)a * K);
        const int kr = k / J, j = k - (k / J) * J;
        const int ks = j / map.c, ch = j - (j / map.c) * map.c;
        if (ch >= map.c_valid) continue;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int sp = 0;
        for (; sp + 4 <= splits; sp += 4) {
            s0 += slabs[(size_t)sp * total + idx];
            s1 += slabs[(size_t)(sp + 1) * total + idx];
            s2 += slabs[(size_t)(sp + 2) * total + idx];
            s3 += slabs[(size_t)(sp + 3) * total + idx];
        }
        for (; sp < splits; ++sp) s0 += slabs[(size_t)sp * total + idx];
        const double s = (s0 + s1) + (s2 + s3);
        const int r = map.rtab[kr], c2 = map.stab[ks];
        const int n = a + map.n_base;
        const size_t dst = map.dim0_is_n ? (((size_t)n * map.d1 + ch) * map.KH + r) * map.KW + c2
                                         : (((size_t)ch * map.d1 + n) * map.KH + r) * map.KW + c2;
        float v = (float)s;
        if (accumulate) v += dw[dst];
        dw[dst] = v;
    }
}

// the same reduction for small weights split many ways (the 1x1 attention head: 640 elements x 512 slabs ran
// as 3 blocks of sequential 512-term sums, 41 us): block = 64 elements x 16 split lanes, each lane a strided
// fp64 sum, the 16 lanes combined in LDS in a fixed order (deterministic)
__global__ void __launch_bounds__(1024) wgrad_reduce_wide_kernel(const float* __restrict__ slabs, int splits,
                                                                  fg_weight_map map, float* __restrict__ dw,
                                                                  int accumulate) {
    const int J = map.kw * map.c;
    const long long K = (long long)map.kh * J;
    const long long total = (long long)map.n_out * K;
    const int e = threadIdx.x & 63, q = threadIdx.x >> 6;
    const long long idx = (long long)blockIdx.x * 64 + e;
    double acc = 0.0;
    if (idx < total)
        for (int sp = q; sp < splits; sp += 16) acc += slabs[(size_t)sp * total + idx];
    __shared__ double red[16][64];
    red[q][e] = acc;
    __syncthreads();
    if (q != 0 || idx >= total) return;
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum += red[i][e];
    const int a = (int)(idx / K);
    const int k = (int)(idx - (long long)a * K);
    const int kr = k / J, j = k - (k / J) * J;
    const int ks = j / map.c, ch = j - (j / map.c) * map.c;
    if (ch >= map.c_valid) return;
    const int r = map.rtab[kr], c2 = map.stab[ks];
    const int n = a + map.n_base;
    const size_t dst = map.dim0_is_n ? (((size_t)n * map.d1 + ch) * map.KH + r) * map.KW + c2
                                     : (((size_t)ch * map.d1 + n) * map.KH + r) * map.KW + c2;
    float v = (float)sum;
    if (accumulate) v += dw[dst];
    dw[dst] = v;
}

__device__ __forceinline__ float packed_w(const float* __restrict__ w, const fg_weight_map& map, int n, int kr, int j) {
    if (j >= map.kw * map.c) return 0.f;
    const int ks = j / map.c, ch = j - (j / map.c) * map.c;
    if (ch >= map.c_valid) return 0.f;
    int r, s;
    if (map.q_n > 0) {            // quad form: group q's taps (a negative index: a zero segment)
        const int q = n / map.q_n;
        n -= q * map.q_n;
        r = map.rtab[q * map.kh + kr];
        s = map.stab[q * map.kw + ks];
        if (r < 0 || s < 0) return 0.f;
    } else {
        r = map.rtab[kr];
        s = map.stab[ks];
    }
    const int nn = n + map.n_base;
    const size_t src = map.dim0_is_n ? (((size_t)nn * map.d1 + ch) * map.KH + r) * map.KW + s
                                     : (((size_t)ch * map.d1 + nn) * map.KH + r) * map.KW + s;
    return w[src];
}

__global__ void pack_weight_kernel(const float* __restrict__ w, fg_weight_map map, float* __restrict__ wp) {
    const int K = map.kh * map.jp;
    const long long total = (long long)map.n_out * K;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(idx / K);
        const int rem = (int)(idx - (long long)n * K);
        const int kr = rem / map.jp, j = rem - (rem / map.jp) * map.jp;
        wp[idx] = packed_w(w, map, n, kr, j);
    }
}

// one thread per (row, 8-k slot): 8 weights -> h, m, l pieces, 48 contiguous bytes
__global__ void pack_weight_split_kernel(const float* __restrict__ w, fg_weight_map map, bf16x8* __restrict__ wps) {
    const int QS = map.kh * map.jp / 8;
    const long long total = (long long)map.n_out * QS;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(idx / QS);
        const int k0 = (int)(idx - (long long)n * QS) * 8;
        const int kr = k0 / map.jp, j0 = k0 - (k0 / map.jp) * map.jp;   // jp % 16 == 0: one kernel row
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = packed_w(w, map, n, kr, j0 + e);
        bf16x8 h, m, l;
        split3(v, h, m, l);
        wps[idx * 3] = h;
        wps[idx * 3 + 1] = m;
        wps[idx * 3 + 2] = l;
    }
}

// f16x3 weights: one thread per (row, 8-k slot): 8 scaled weights -> h, l fp16 pieces (32 B)
__global__ void pack_weight_f16_kernel(const float* __restrict__ w, fg_weight_map map, const float* __restrict__ amax,
                                       f16x8* __restrict__ wps) {
    const int QS = map.kh * map.jp / 8;
    const long long total = (long long)map.n_out * QS;
    const float sc = pow2_scale(amax);
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(idx / QS);
        const int k0 = (int)(idx - (long long)n * QS) * 8;
        const int kr = k0 / map.jp, j0 = k0 - (k0 / map.jp) * map.jp;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = packed_w(w, map, n, kr, j0 + e);
        f16x8 pc[2];
        MathF16x3::split(v, sc, pc);
        wps[idx * 2] = pc[0];
        wps[idx * 2 + 1] = pc[1];
    }
}

// a batch of f16x3 repacks: the jobs' units (row, 8-k slot) are dealt to blocks job by job (blk[j] ..
// blk[j+1]); a block's job index is uniform, its units are grid-strided over the job's blocks
struct PackBatch {
    fg_pack_job job[FG_PACK_BATCH_MAX];
    int blk[FG_PACK_BATCH_MAX + 1];
    int n;
};
static_assert(sizeof(PackBatch) <= 4096, "kernel argument size");

__global__ void pack_weight_f16_batch_kernel(const PackBatch b) {
    int j = 0;
    while (j + 1 < b.n && (int)blockIdx.x >= b.blk[j + 1]) ++j;
    const fg_pack_job& J = b.job[j];
    const fg_weight_map& map = J.map;
    const int QS = map.kh * map.jp / 8;
    const long long total = (long long)map.n_out * QS;
    const float sc = pow2_scale(J.w_absmax);
    f16x8* wps = reinterpret_cast<f16x8*>(J.dst);
    const int nb = b.blk[j + 1] - b.blk[j];
    for (long long idx = (blockIdx.x - b.blk[j]) * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)nb * blockDim.x) {
        const int n = (int)(idx / QS);
        const int k0 = (int)(idx - (long long)n * QS) * 8;
        const int kr = k0 / map.jp, j0 = k0 - (k0 / map.jp) * map.jp;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = packed_w(J.w, map, n, kr, j0 + e);
        f16x8 pc[2];
        MathF16x3::split(v, sc, pc);
        wps[idx * 2] = pc[0];
        wps[idx * 2 + 1] = pc[1];
    }
}

// max |x| as the bit pattern of a non-negative float (uint order = float order; NaN sorts high)
__global__ void absmax_kernel(const float* __restrict__ x, long long n, unsigned* __restrict__ out) {
    unsigned m = 0;
    const long long n4 = (((uintptr_t)x & 15) == 0) ? n / 4 : 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) m = max(m, __float_as_uint(v[e]) & 0x7fffffffu);
    }
    for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        m = max(m, __float_as_uint(x[i]) & 0x7fffffffu);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    __shared__ unsigned red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = max(m, red[i]);
        atomicMax(out + (blockIdx.x & (FG_AMAX_SHARDS - 1)), m);
    }
}

template <class SM, int BM, int BN, int WM, int WN, int MINW, int PF, bool SWZ = false>
int launch_fwd_x6(const ConvBatch& b, int total, bool vec, bool ws, hipStream_t stream) {
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    if (vec && ws)
        FG_LAUNCH((conv_fwd_x6_kernel<SM, BM, BN, WM, WN, true, true, MINW, PF, SWZ>), dim3(total), dim3(NT), 0, stream, b);
    else if (vec)
        FG_LAUNCH((conv_fwd_x6_kernel<SM, BM, BN, WM, WN, true, false, MINW, PF, SWZ>), dim3(total), dim3(NT), 0, stream, b);
    else if (ws)
        FG_LAUNCH((conv_fwd_x6_kernel<SM, BM, BN, WM, WN, false, true, MINW, PF, SWZ>), dim3(total), dim3(NT), 0, stream, b);
    else
        FG_LAUNCH((conv_fwd_x6_kernel<SM, BM, BN, WM, WN, false, false, MINW, PF, SWZ>), dim3(total), dim3(NT), 0, stream, b);
    return fg::launched("conv_fwd_x6");
}

template <int BM, int BN, int WM, int WN>
int launch_fwd(const ConvBatch& b, int total, bool vec, hipStream_t stream) {
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    if (vec)
        FG_LAUNCH((conv_fwd_kernel<BM, BN, WM, WN, true>), dim3(total), dim3(NT), 0, stream, b);
    else
        FG_LAUNCH((conv_fwd_kernel<BM, BN, WM, WN, false>), dim3(total), dim3(NT), 0, stream, b);
    return fg::launched("conv_fwd");
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <class SM, int BA, int BKC, int WA, int WK, int MINW, bool WAB = false>
int launch_wgrad_x6(const fg_wgrad_problem& p, bool vx, bool vp, hipStream_t stream) {
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    const int K = p.kh * p.j_valid;
    const int ta = (p.n_a + BA - 1) / BA, tk = (K + BKC - 1) / BKC;
    dim3 g(ta * tk * p.splits), blk(NT);
    if (vx && vp)
        FG_LAUNCH((conv_wgrad_x6_kernel<SM, BA, BKC, WA, WK, true, true, MINW, WAB>), g, blk, 0, stream, p, ta, tk);
    else if (vx)
        FG_LAUNCH((conv_wgrad_x6_kernel<SM, BA, BKC, WA, WK, true, false, MINW, WAB>), g, blk, 0, stream, p, ta, tk);
    else if (vp)
        FG_LAUNCH((conv_wgrad_x6_kernel<SM, BA, BKC, WA, WK, false, true, MINW, WAB>), g, blk, 0, stream, p, ta, tk);
    else
        FG_LAUNCH((conv_wgrad_x6_kernel<SM, BA, BKC, WA, WK, false, false, MINW, WAB>), g, blk, 0, stream, p, ta, tk);
    return fg::launched("conv_wgrad_x6");
}

int g_wgrad_tile = -1;   // tuning hook (fg_set_wgrad_tile)

template <class SM>
int launch_wgrad_split_cfg(int cfg, const fg_wgrad_problem& p, bool vx, bool vp, hipStream_t stream) {
    switch (cfg) {
        case 0: return launch_wgrad_x6<SM, 128, 128, 64, 64, 3>(p, vx, vp, stream);
        case 1: return launch_wgrad_x6<SM, 256, 128, 64, 64, 4>(p, vx, vp, stream);
        case 2: return launch_wgrad_x6<SM, 64, 256, 64, 64, 3>(p, vx, vp, stream);
        case 3: return launch_wgrad_x6<SM, 32, 256, 32, 64, 3>(p, vx, vp, stream);
        case 4: return launch_wgrad_x6<SM, 256, 128, 64, 64, 4, true>(p, vx, vp, stream);
        default: return launch_wgrad_x6<SM, 128, 128, 64, 64, 3, true>(p, vx, vp, stream);
    }
}
constexpr int kWgradTiles = 6;

template <int BA, int BKC, int WA, int WK>
int launch_wgrad(const fg_wgrad_problem& p, bool vx, bool vp, hipStream_t stream) {
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    const int K = p.kh * p.j_valid;
    const int ta = (p.n_a + BA - 1) / BA, tk = (K + BKC - 1) / BKC;
    const int total = ta * tk * p.splits;
    dim3 g(total), blk(NT);
    if (vx && vp)
        FG_LAUNCH((conv_wgrad_kernel<BA, BKC, WA, WK, true, true>), g, blk, 0, stream, p, ta, tk);
    else if (vx)
        FG_LAUNCH((conv_wgrad_kernel<BA, BKC, WA, WK, true, false>), g, blk, 0, stream, p, ta, tk);
    else if (vp)
        FG_LAUNCH((conv_wgrad_kernel<BA, BKC, WA, WK, false, true>), g, blk, 0, stream, p, ta, tk);
    else
        FG_LAUNCH((conv_wgrad_kernel<BA, BKC, WA, WK, false, false>), g, blk, 0, stream, p, ta, tk);
    return fg::launched("conv_wgrad");
}

int g_fwd_tile = -1;   // tuning hook (fg_set_fwd_tile): force one bf16x6 forward tile config
// the stem forward on its strip kernel (step 46.31 -> 46.16 ms, profiles/round4/r4e_ab_stem_fwd.log); read per call
// so that scripts/bench_stem_wgrad.py can interleave it with the register-staged x6 kernel (FLOODGAN_STEM_FWD=0)
static bool stem_fwd_on() { const char* e = getenv("FLOODGAN_STEM_FWD"); return !e || atoi(e) != 0; }

// split-math forward tile configs {BM, BN, wave tile, waves/SIMD, prefetch distance, LDS swizzle}
template <class SM>
int launch_fwd_split_cfg(int cfg, const ConvBatch& b, int total, bool vec, bool ws, hipStream_t stream) {
    switch (cfg) {
        case 0: return launch_fwd_x6<SM, 128, 256, 64, 64, 2, 1, true>(b, total, vec, ws, stream);
        case 1: return launch_fwd_x6<SM, 256, 128, 64, 64, 2, 1, true>(b, total, vec, ws, stream);
        case 2: return launch_fwd_x6<SM, 128, 64, 32, 64, 3, 1, true>(b, total, vec, ws, stream);
        case 3: return launch_fwd_x6<SM, 128, 32, 32, 32, 2, 2, false>(b, total, vec, ws, stream);
        case 4: return launch_fwd_x6<SM, 128, 128, 64, 64, 3, 1, true>(b, total, vec, ws, stream);
        case 5: return launch_fwd_x6<SM, 128, 32, 32, 32, 4, 1, true>(b, total, vec, ws, stream);
        case 6: return launch_fwd_x6<SM, 256, 256, 64, 128, 2, 1, true>(b, total, vec, ws, stream);
        case 7: return launch_fwd_x6<SM, 256, 256, 128, 64, 2, 1, true>(b, total, vec, ws, stream);
        case 8: return launch_fwd_x6<SM, 128, 256, 64, 128, 1, 1, true>(b, total, vec, ws, stream);
        case 9: return launch_fwd_x6<SM, 128, 256, 64, 64, 2, 3, true>(b, total, vec, ws, stream);
        case 10: return launch_fwd_x6<SM, 256, 128, 64, 64, 2, 3, true>(b, total, vec, ws, stream);
        default: return launch_fwd_x6<SM, 128, 64, 32, 64, 3, 3, true>(b, total, vec, ws, stream);
    }
}
constexpr int kFwdTiles = 12;
constexpr int kFwdTileBM[kFwdTiles] = {128, 256, 128, 128, 128, 128, 256, 256, 128, 128, 256, 128};
constexpr int kFwdTileBN[kFwdTiles] = {256, 128, 64, 32, 128, 32, 256, 256, 256, 256, 128, 64};

}  // namespace

FG_API int fg_conv_fwd(const fg_conv_problem* probs, int nprob, hipStream_t stream) {
    if (!probs || nprob < 1 || nprob > 4) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: nprob=%d", nprob);
    ConvBatch b;
    b.count = nprob;
    b.interleave = 0;
    int max_n = 0;
    bool vec = true;
    const int ws = probs[0].w_split;
    for (int i = 0; i < nprob; ++i) {
        const fg_conv_problem& p = probs[i];
        if (!p.x || !p.w || !p.y) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: null pointer (problem %d)", i);
        if (p.m_img < 0 || p.m_a < 0 || p.m_b < 0 || p.kh < 1 || p.jp < BK || p.jp % BK || p.j_valid < 1 ||
            p.j_valid > p.jp || p.n_out < 1 || p.ldw < p.kh * p.jp || p.ldw % 8 || !aligned16(p.w))
            return fg::fail(FG_ERR_INVALID,
                            "fg_conv_fwd: bad geometry (problem %d: m=%dx%dx%d kh=%d j=%d/%d n=%d ldw=%d)", i,
                            p.m_img, p.m_a, p.m_b, p.kh, p.j_valid, p.jp, p.n_out, p.ldw);
        if ((long long)p.m_img * p.m_a * p.m_b >= (1LL << 31))
            return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: too many rows");
        if (p.w_split != ws || ws < 0 || ws > 2)
            return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: w_split must be 0, 1 or 2 and equal across problems");
        if ((g_conv_math & FG_MATH_FWD_F16X3) && (!p.x_absmax || !p.w_absmax))
            return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: the f16x3 math needs x_absmax and w_absmax (problem %d)", i);
        if (!aligned16(p.x) || (p.sxn | p.sxa | p.sxb | p.sxr) % 4 || p.j_valid % 4) vec = false;
        if (p.n_out > max_n) max_n = p.n_out;
        if (p.q_n && (nprob != 1 || !p.x_presplit || !(g_conv_math & FG_MATH_FWD_F16X3)))
            return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: the quad form (q_n) is one pre-split f16x3 problem");
        b.p[i] = p;
    }
    const bool f16 = (g_conv_math & FG_MATH_FWD_F16X3) != 0;
    const bool x6 = f16 || (g_conv_math & FG_MATH_FWD_X6) != 0;   // a split-math kernel
    bool stats = false;
    for (int i = 0; i < nprob; ++i) stats |= probs[i].in_stats != nullptr;
    // the generator stem (7x7 over 9 channels -> 64): its strip kernel, epilogue statistics included (conv_stem.hip)
    if (f16 && nprob == 1 && ws == 2 && g_fwd_tile < 0 && stem_fwd_on()) {
        int rc = 0;
        if (fgc::launch_fwd_stem(probs[0], stream, &rc)) return rc;
    }
    if (stats && !(f16 && vec && ws == 2 && g_fwd_tile < 0 && fgc::f3_stats_ok(probs, nprob, max_n)))
        return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: in_stats needs the pipelined f16x3 kernel (see fg_conv_stats_ok)");
    if ((ws == 1 && (!x6 || f16)) || (ws == 2 && !f16))
        return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: pre-split weights (w_split=%d) do not match the conv math %d",
                        ws, g_conv_math);
    int nps = 0;
    for (int i = 0; i < nprob; ++i) nps += probs[i].x_presplit != 0;
    if (nps && (nps != nprob || !f16 || !vec || ws != 2 || g_fwd_tile >= 0))
        return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: pre-split x (FG_PRESPLIT) needs every problem pre-split, the f16x3 "
                                        "math and the pipelined kernel");
    if (x6) {
        // the split-math kernels address operands with 31-bit buffer offsets: split oversized
        // problems over images (each chunk launched on its own)
        constexpr long long kLim = (1LL << 31) - 256;
        bool fits = true;
        for (int i = 0; i < nprob; ++i) {
            const fg_conv_problem& p = probs[i];
            const long long tail = (long long)(p.m_a - 1) * p.sxa + (long long)(p.m_b - 1) * p.sxb +
                                   (long long)(p.kh - 1) * p.sxr + p.jp;
            const long long ext = 4 * ((long long)(p.m_img - 1) * p.sxn + tail);
            const long long wext = (long long)p.n_out * p.ldw * (ws == 1 ? 6 : 4);
            if (wext > kLim || 4 * tail > kLim || p.sxn < 0 || p.sxa < 0 || p.sxb < 0 || p.sxr < 0)
                return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: operand extent beyond 2 GiB per image (problem %d)", i);
            if (ext > kLim) fits = false;
        }
        if (!fits) {
            if (stats) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: in_stats with an operand beyond 2 GiB");
            for (int i = 0; i < nprob; ++i) {
                fg_conv_problem q = probs[i];
                const long long tail = (long long)(q.m_a - 1) * q.sxa + (long long)(q.m_b - 1) * q.sxb +
                                       (long long)(q.kh - 1) * q.sxr + q.jp;
                const int per = (int)std::max(1LL, (kLim / 4 - tail) / std::max(1LL, q.sxn) + 1);
                for (int i0 = 0; i0 < probs[i].m_img; i0 += per) {
                    q.x = probs[i].x + (long long)i0 * probs[i].sxn;
                    q.y = probs[i].y + (long long)i0 * probs[i].syn;
                    q.m_img = std::min(per, probs[i].m_img - i0);
                    const int rc = fg_conv_fwd(&q, 1, stream);
                    if (rc) return rc;
                }
            }
            return 0;
        }
    }
    if (f16 && vec && ws == 2 && g_fwd_tile < 0) {
        // the LDS-DMA pipelined f16x3 kernel takes the wide convs (conv_f3.hip)
        int rc = 0;
        if (fgc::launch_fwd_f3(b, nprob, max_n, stream, &rc)) return rc;
    }
    if (nps) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: the pipelined kernel declined pre-split problems (geometry)");
    int cfg = -1, BM, BN;
    if (x6) {
        cfg = g_fwd_tile >= 0 ? g_fwd_tile : (max_n > 128 ? 0 : max_n > 64 ? 1 : max_n > 32 ? 2 : 3);
        BM = kFwdTileBM[cfg];
        BN = kFwdTileBN[cfg];
    } else if (max_n > 64) { BM = 128; BN = 128; }
    else if (max_n > 32) { BM = 256; BN = 64; }
    else { BM = 256; BN = 32; }
    int total = 0;
    for (int i = 0; i < nprob; ++i) {
        const long long M = (long long)probs[i].m_img * probs[i].m_a * probs[i].m_b;
        b.ntiles_n[i] = (probs[i].n_out + BN - 1) / BN;
        b.blk_start[i] = total;
        total += (int)((M + BM - 1) / BM) * b.ntiles_n[i];
    }
    for (int i = nprob; i < 4; ++i) { b.ntiles_n[i] = 1; b.blk_start[i] = total; }
    b.blk_start[nprob] = total;
    b.blk_start[4] = total;
    if (total == 0) return 0;
    if (f16) return launch_fwd_split_cfg<MathF16x3>(cfg, b, total, vec, ws != 0, stream);
    if (x6) return launch_fwd_split_cfg<MathBF16x6>(cfg, b, total, vec, ws != 0, stream);
    if (BN == 128) return launch_fwd<128, 128, 64, 64>(b, total, vec, stream);
    if (BN == 64) return launch_fwd<256, 64, 64, 64>(b, total, vec, stream);
    return launch_fwd<256, 32, 64, 32>(b, total, vec, stream);
}

FG_API int fg_conv_stats_ok(const fg_conv_problem* probs, int nprob) {
    if (!probs || nprob < 1 || nprob > 4) return 0;
    if (!(g_conv_math & FG_MATH_FWD_F16X3) || g_fwd_tile >= 0) return 0;
    if (nprob == 1 && stem_fwd_on() && fgc::stem_fwd_rows(probs[0]) && probs[0].m_b % 32 == 0) return 1;
    int max_n = 0;
    for (int i = 0; i < nprob; ++i) {
        const fg_conv_problem& p = probs[i];
        if (p.w_split != 2 || !aligned16(p.x) || (p.sxn | p.sxa | p.sxb | p.sxr) % 4 || p.j_valid % 4) return 0;
        max_n = std::max(max_n, p.n_out);
    }
    return fgc::f3_stats_ok(probs, nprob, max_n) ? 1 : 0;
}

FG_API int fg_set_wgrad_tile(int cfg) {
    if (cfg < -1 || cfg >= kWgradTiles) return fg::fail(FG_ERR_INVALID, "fg_set_wgrad_tile: %d", cfg);
    g_wgrad_tile = cfg;
    return 0;
}

FG_API int fg_set_fwd_tile(int cfg) {
    if (cfg < -1 || cfg >= kFwdTiles) return fg::fail(FG_ERR_INVALID, "fg_set_fwd_tile: %d", cfg);
    g_fwd_tile = cfg;
    return 0;
}

FG_API int fg_conv_wgrad(const fg_wgrad_problem* prob, hipStream_t stream) {
    if (!prob || !prob->p || !prob->x || !prob->out) return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: null");
    const fg_wgrad_problem& p = *prob;
    if (p.n_a < 1 || p.kh < 1 || p.j_valid < 1 || p.splits < 1 || p.m_chunk < 1 || p.m_img < 0 ||
        p.m_a < 0 || p.m_b < 0)
        return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: bad geometry n_a=%d kh=%d j=%d splits=%d chunk=%d", p.n_a,
                        p.kh, p.j_valid, p.splits, p.m_chunk);
    const long long M = (long long)p.m_img * p.m_a * p.m_b;
    if ((long long)p.splits * p.m_chunk < M)
        return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: splits*m_chunk < M");
    const bool vx = aligned16(p.x) && (p.sxn | p.sxa | p.sxb | p.sxr) % 4 == 0 && p.j_valid % 4 == 0;
    const bool vp = aligned16(p.p) && (p.spn | p.spa | p.spb) % 4 == 0;
    if (g_conv_math & (FG_MATH_WGRAD_X6 | FG_MATH_WGRAD_F16X3)) {
        // 31-bit buffer offsets: the extent of either operand must stay below 2 GiB
        const long long pext = 4 * ((long long)(p.m_img - 1) * p.spn + (long long)(p.m_a - 1) * p.spa +
                                    (long long)(p.m_b - 1) * p.spb + p.n_a + 4);
        const long long xext = 4 * ((long long)(p.m_img - 1) * p.sxn + (long long)(p.m_a - 1) * p.sxa +
                                    (long long)(p.m_b - 1) * p.sxb + (long long)(p.kh - 1) * p.sxr + p.j_valid + 4);
        if (pext >= (1LL << 31) - 256 || xext >= (1LL << 31) - 256 || p.spn < 0 || p.sxn < 0)
            return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: operand extent beyond 2 GiB; split the batch");
        const int cfg = g_wgrad_tile >= 0 ? g_wgrad_tile : (p.n_a > 128 ? 1 : p.n_a > 64 ? 0 : p.n_a > 32 ? 2 : 3);
        if (g_conv_math & FG_MATH_WGRAD_F16X3) {
            if (!p.p_absmax || !p.x_absmax)
                return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: the f16x3 math needs p_absmax and x_absmax");
            int rc = 0;
            if (g_wgrad_tile < 0 && fgc::launch_wgrad_stem(p, stream, &rc)) return rc; // conv_stem.hip
            if (g_wgrad_tile < 0 && fgc::launch_wgrad_f3(p, stream, &rc)) return rc;   // conv_wgrad_f3.hip
            if (p.p_presplit || p.x_presplit)
                return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: pre-split operands need the pipelined kernel");
            return launch_wgrad_split_cfg<MathF16x3>(cfg, p, vx, vp, stream);
        }
        if (p.p_presplit || p.x_presplit)
            return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: pre-split operands need the f16x3 math");
        return launch_wgrad_split_cfg<MathBF16x6>(cfg, p, vx, vp, stream);
    }
    if (p.p_presplit || p.x_presplit) return fg::fail(FG_ERR_INVALID, "fg_conv_wgrad: pre-split operands need f16x3");
    if (p.n_a > 64) return launch_wgrad<128, 128, 64, 64>(p, vx, vp, stream);
    if (p.n_a > 32) return launch_wgrad<64, 256, 64, 64>(p, vx, vp, stream);
    return launch_wgrad<32, 256, 32, 64>(p, vx, vp, stream);
}

FG_API int fg_wgrad_reduce(const float* slabs, int splits, const fg_weight_map* map, float* dw, int accumulate,
                           hipStream_t stream) {
    if (!slabs || !map || !dw || splits < 1) return fg::fail(FG_ERR_INVALID, "fg_wgrad_reduce: bad args");
    if (map->kh > 8 || map->kw > 8 || map->c < 1 || map->n_out < 1 || map->q_n != 0)
        return fg::fail(FG_ERR_INVALID, "fg_wgrad_reduce: bad map (the quad form packs weights only)");
    const long long total = (long long)map->n_out * map->kh * map->kw * map->c;
    if (total <= 256 * 1024 && splits >= 32 && total * 4 < (long long)splits * 1024) {
        // few elements, many slabs: parallel over the splits too
        hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)((total + 63) / 64)), dim3(1024), 0, stream, slabs,
                           splits, *map, dw, accumulate);
        return fg::launched("wgrad_reduce_wide");
    }
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, slabs,
                       splits, *map, dw, accumulate);
    return fg::launched("wgrad_reduce");
}

// the quad form (fg_weight_map.q_n): 1-2 taps per axis and group, at most 4 groups of whole rows
static bool bad_quad(const fg_weight_map& m) {
    return m.q_n < 0 || (m.q_n > 0 && (m.kh > 2 || m.kw > 2 || m.n_out % m.q_n || m.n_out / m.q_n > 4));
}

FG_API int fg_pack_weight(const float* w, const fg_weight_map* map, float* wp, hipStream_t stream) {
    if (!w || !map || !wp) return fg::fail(FG_ERR_INVALID, "fg_pack_weight: null");
    if (map->kh > 8 || map->kw > 8 || map->jp % BK || map->jp < map->kw * map->c || map->c < 1 || bad_quad(*map))
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight: bad map kh=%d kw=%d c=%d jp=%d", map->kh, map->kw, map->c,
                        map->jp);
    const long long total = (long long)map->n_out * map->kh * map->jp;
    hipLaunchKernelGGL(pack_weight_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, w, *map,
                       wp);
    return fg::launched("pack_weight");
}

FG_API int fg_pack_weight_split(const float* w, const fg_weight_map* map, void* wps, hipStream_t stream) {
    if (!w || !map || !wps || !aligned16(wps)) return fg::fail(FG_ERR_INVALID, "fg_pack_weight_split: null/unaligned");
    if (map->kh > 8 || map->kw > 8 || map->jp % BK || map->jp < map->kw * map->c || map->c < 1 || bad_quad(*map))
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight_split: bad map kh=%d kw=%d c=%d jp=%d", map->kh, map->kw,
                        map->c, map->jp);
    const long long total = (long long)map->n_out * map->kh * map->jp / 8;
    hipLaunchKernelGGL(pack_weight_split_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, w,
                       *map, reinterpret_cast<bf16x8*>(wps));
    return fg::launched("pack_weight_split");
}

FG_API int fg_pack_weight_f16(const float* w, const fg_weight_map* map, const float* w_absmax, void* wps,
                              hipStream_t stream) {
    if (!w || !map || !wps || !w_absmax || !aligned16(wps))
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight_f16: null/unaligned");
    if (map->kh > 8 || map->kw > 8 || map->jp % BK || map->jp < map->kw * map->c || map->c < 1 || bad_quad(*map))
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight_f16: bad map kh=%d kw=%d c=%d jp=%d", map->kh, map->kw,
                        map->c, map->jp);
    const long long total = (long long)map->n_out * map->kh * map->jp / 8;
    hipLaunchKernelGGL(pack_weight_f16_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, w, *map,
                       w_absmax, reinterpret_cast<f16x8*>(wps));
    return fg::launched("pack_weight_f16");
}

FG_API int fg_pack_weight_f16_batch(const fg_pack_job* jobs, int njobs, hipStream_t stream) {
    if (!jobs || njobs < 0 || njobs > FG_PACK_BATCH_MAX)
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight_f16_batch: %d jobs (at most %d)", njobs, FG_PACK_BATCH_MAX);
    if (njobs == 0) return 0;
    PackBatch b;
    b.n = njobs;
    int blocks = 0;
    for (int j = 0; j < njobs; ++j) {
        const fg_pack_job& J = jobs[j];
        const fg_weight_map& m = J.map;
        if (!J.w || !J.dst || !J.w_absmax || !aligned16(J.dst))
            return fg::fail(FG_ERR_INVALID, "fg_pack_weight_f16_batch: job %d null/unaligned", j);
        if (m.kh > 8 || m.kw > 8 || m.jp % BK || m.jp < m.kw * m.c || m.c < 1 || m.n_out < 1 || bad_quad(m))
            return fg::fail(FG_ERR_INVALID, "fg_pack_weight_f16_batch: job %d bad map kh=%d kw=%d c=%d jp=%d", j,
                            m.kh, m.kw, m.c, m.jp);
        b.job[j] = J;
        b.blk[j] = blocks;
        blocks += (int)fg::blocks_for((long long)m.n_out * m.kh * m.jp / 8, 256, 512);
    }
    b.blk[njobs] = blocks;
    hipLaunchKernelGGL(pack_weight_f16_batch_kernel, dim3(blocks), dim3(256), 0, stream, b);
    return fg::launched("pack_weight_f16_batch");
}

FG_API int fg_absmax(const float* x, long long n, float* out, hipStream_t stream) {
    if (!x || !out || n < 0) return fg::fail(FG_ERR_INVALID, "fg_absmax: bad args");
    if (n == 0) return 0;
    hipLaunchKernelGGL(absmax_kernel, dim3(fg::blocks_for((n + 3) / 4, 256, 2048)), dim3(256), 0, stream, x, n,
                       reinterpret_cast<unsigned*>(out));
    return fg::launched("absmax");
}

FG_API int fg_set_conv_math(int mode) {
    const int fwd = mode & (FG_MATH_FWD_X6 | FG_MATH_FWD_F16X3), wg = mode & (FG_MATH_WGRAD_X6 | FG_MATH_WGRAD_F16X3);
    if (mode < 0 || mode > FG_MATH_F16X3 || fwd == (FG_MATH_FWD_X6 | FG_MATH_FWD_F16X3) ||
        wg == (FG_MATH_WGRAD_X6 | FG_MATH_WGRAD_F16X3))
        return fg::fail(FG_ERR_INVALID, "fg_set_conv_math: %d", mode);
    g_conv_math = mode;
    return 0;
}

FG_API int fg_get_conv_math(void) { return g_conv_math; }
