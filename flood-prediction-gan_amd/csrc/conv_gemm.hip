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
#include "fg_common.hpp"

namespace {

constexpr int BK = 16;
constexpr int LDK = BK + 4;
int g_conv_math = FG_MATH_BF16X6;   // default: fp32-equivalent split-bf16 (tests: tests/test_gpu_parity.py)

struct ConvBatch {
    fg_conv_problem p[4];
    int count;
    int ntiles_n[4];
    int blk_start[5];
};

__device__ __forceinline__ void decomp(int m, int mb, int mab, int& img, int& a, int& b) {
    img = m / mab;
    const int rem = m - img * mab;
    a = rem / mb;
    b = rem - a * mb;
}

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

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 hh = (__bf16)v[e];
        const float r = v[e] - (float)hh;
        const __bf16 mm = (__bf16)r;
        const float r2 = r - (float)mm;
        h[e] = hh;
        m[e] = mm;
        l[e] = (__bf16)r2;
    }
}

template <int BM, int BN, int WM, int WN, bool VEC>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, 2)
conv_fwd_x6_kernel(const ConvBatch batch) {
    constexpr int NWN = BN / WN;
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr int LDP = 24;                       // bf16 per LDS row (16 + 8 pad)
    constexpr int A_SLOTS = BM * 2, B_SLOTS = BN * 2;   // slot = 8 consecutive k of one row
    constexpr int A_IT = (A_SLOTS + NT - 1) / NT, B_IT = (B_SLOTS + NT - 1) / NT;

    __shared__ __attribute__((aligned(16))) __bf16 As[2][3][BM][LDP];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][3][BN][LDP];

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

    const float* arow[A_IT];
    int a_r[A_IT], a_g[A_IT];
    bool aok[A_IT], aslot[A_IT];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
        const int s = tid + i * NT;
        a_r[i] = s >> 1;
        a_g[i] = s & 1;
        aslot[i] = s < A_SLOTS;
        const int m = m0 + (s >> 1);
        aok[i] = aslot[i] && (m < M);
        arow[i] = P.x;
        if (aok[i]) {
            int img, a, b;
            decomp(m, P.m_b, mab, img, a, b);
            arow[i] = P.x + img * P.sxn + a * P.sxa + b * P.sxb;
        }
    }
    const float* brow[B_IT];
    int b_r[B_IT], b_g[B_IT];
    bool bok[B_IT], bslot[B_IT];
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
        const int s = tid + i * NT;
        b_r[i] = s >> 1;
        b_g[i] = s & 1;
        bslot[i] = s < B_SLOTS;
        bok[i] = bslot[i] && (n0 + (s >> 1) < P.n_out);
        brow[i] = P.w + (size_t)(bok[i] ? n0 + (s >> 1) : 0) * P.ldw;
    }

    float ra[A_IT][8], rb[B_IT][8];
    auto load = [&](int kt) {
        const int r = kt / jtr;
        const int jb = (kt - r * jtr) * 16;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int j = jb + a_g[i] * 8;
            const float* src = arow[i] + r * sxr + j;
            if constexpr (VEC) {
                f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
                if (aok[i] && j < jv) v0 = *reinterpret_cast<const f32x4*>(src);
                if (aok[i] && j + 4 < jv) v1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    ra[i][e] = v0[e];
                    ra[i][4 + e] = v1[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) ra[i][e] = (aok[i] && j + e < jv) ? src[e] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
            if (bok[i]) {
                const float* src = brow[i] + kt * 16 + b_g[i] * 8;
                v0 = *reinterpret_cast<const f32x4*>(src);
                v1 = *reinterpret_cast<const f32x4*>(src + 4);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                rb[i][e] = v0[e];
                rb[i][4 + e] = v1[e];
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i)
            if (aslot[i]) {
                bf16x8 h, m, l;
                split3(ra[i], h, m, l);
                *reinterpret_cast<bf16x8*>(&As[buf][0][a_r[i]][a_g[i] * 8]) = h;
                *reinterpret_cast<bf16x8*>(&As[buf][1][a_r[i]][a_g[i] * 8]) = m;
                *reinterpret_cast<bf16x8*>(&As[buf][2][a_r[i]][a_g[i] * 8]) = l;
            }
#pragma unroll
        for (int i = 0; i < B_IT; ++i)
            if (bslot[i]) {
                bf16x8 h, m, l;
                split3(rb[i], h, m, l);
                *reinterpret_cast<bf16x8*>(&Bs[buf][0][b_r[i]][b_g[i] * 8]) = h;
                *reinterpret_cast<bf16x8*>(&Bs[buf][1][b_r[i]][b_g[i] * 8]) = m;
                *reinterpret_cast<bf16x8*>(&Bs[buf][2][b_r[i]][b_g[i] * 8]) = l;
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

    const int lrow = lane & 31, lk = (lane >> 5) * 8;
    if (nkt > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) load(kt + 1);
        bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
                af[tm][p] = *reinterpret_cast<const bf16x8*>(&As[cur][p][wm * WM + tm * 32 + lrow][lk]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                bfr[tn][p] = *reinterpret_cast<const bf16x8*>(&Bs[cur][p][wn * WN + tn * 32 + lrow][lk]);
        }
        // six fp32-relevant piece products; each pair's (tm, tn) blocks interleaved
        constexpr int PA[6] = {1, 0, 2, 0, 1, 0};
        constexpr int PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int c = 0; c < 6; ++c)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][PA[c]], bfr[tn][PB[c]], acc[tm][tn],
                                                                          0, 0, 0);
        if (kt + 1 < nkt) store(cur ^ 1);
        __syncthreads();
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

__device__ __forceinline__ bf16x8 tr_frag(const __bf16* r0, const __bf16* r4) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(r0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(r4));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void split3x4(const f32x4& v, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const __bf16 hh = (__bf16)v[e];
        const float r = v[e] - (float)hh;
        const __bf16 mm = (__bf16)r;
        const float r2 = r - (float)mm;
        h[e] = hh;
        m[e] = mm;
        l[e] = (__bf16)r2;
    }
}

template <int BA, int BKC, int WA, int WK, bool VX, bool VP>
__global__ void __launch_bounds__((BA / WA) * (BKC / WK) * 64, 2)
conv_wgrad_x6_kernel(const fg_wgrad_problem P, int tiles_a, int tiles_k) {
    constexpr int NWK = BKC / WK;
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    constexpr int TM = WA / 32, TN = WK / 32;
    constexpr int BR = 16;
    constexpr int PA_ = BA + 32, PX_ = BKC + 32;     // bf16 row pitches
    constexpr int P_SLOTS = BR * BA / 4, X_SLOTS = BR * BKC / 4;
    constexpr int P_IT = (P_SLOTS + NT - 1) / NT, X_IT = (X_SLOTS + NT - 1) / NT;

    __shared__ __attribute__((aligned(16))) __bf16 Ps[2][3][BR][PA_];
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][3][BR][PX_];

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

    int p_row[P_IT], p_col[P_IT];
    bool p_slot[P_IT];
#pragma unroll
    for (int i = 0; i < P_IT; ++i) {
        const int s = tid + i * NT;
        p_slot[i] = s < P_SLOTS;
        p_row[i] = s / (BA / 4);
        p_col[i] = (s - (s / (BA / 4)) * (BA / 4)) * 4;
    }
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
            if (p_slot[i]) {
                bf16x4 h, m, l;
                split3x4(rp[i], h, m, l);
                *reinterpret_cast<bf16x4*>(&Ps[buf][0][p_row[i]][p_col[i]]) = h;
                *reinterpret_cast<bf16x4*>(&Ps[buf][1][p_row[i]][p_col[i]]) = m;
                *reinterpret_cast<bf16x4*>(&Ps[buf][2][p_row[i]][p_col[i]]) = l;
            }
#pragma unroll
        for (int i = 0; i < X_IT; ++i)
            if (x_slot[i]) {
                bf16x4 h, m, l;
                split3x4(rx[i], h, m, l);
                *reinterpret_cast<bf16x4*>(&Xs[buf][0][x_row[i]][x_col[i]]) = h;
                *reinterpret_cast<bf16x4*>(&Xs[buf][1][x_row[i]][x_col[i]]) = m;
                *reinterpret_cast<bf16x4*>(&Xs[buf][2][x_row[i]][x_col[i]]) = l;
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
    if (nit > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
        const int cur = it & 1;
        if (it + 1 < nit) load(it + 1);
        bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int c = wa * WA + tm * 32 + tr_col;
                af[tm][p] = tr_frag(&Ps[cur][p][tr_row][c], &Ps[cur][p][tr_row + 4][c]);
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int c = wk * WK + tn * 32 + tr_col;
                bfr[tn][p] = tr_frag(&Xs[cur][p][tr_row][c], &Xs[cur][p][tr_row + 4][c]);
            }
        }
        constexpr int PA[6] = {1, 0, 2, 0, 1, 0};
        constexpr int PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int c = 0; c < 6; ++c)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][PA[c]], bfr[tn][PB[c]], acc[tm][tn],
                                                                          0, 0, 0);
        if (it + 1 < nit) store(cur ^ 1);
        __syncthreads();
    }

    float* out = P.out + (size_t)split * P.n_a * K;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int a = a0 + wa * WA + tm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
            if (a >= P.n_a) continue;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int k = k0 + wk * WK + tn * 32 + (lane & 31);
                if (k < K) out[(size_t)a * K + k] = acc[tm][tn][reg];
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

__global__ void pack_weight_kernel(const float* __restrict__ w, fg_weight_map map, float* __restrict__ wp) {
    const int K = map.kh * map.jp;
    const long long total = (long long)map.n_out * K;
    const int J = map.kw * map.c;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(idx / K);
        const int rem = (int)(idx - (long long)n * K);
        const int kr = rem / map.jp, j = rem - (rem / map.jp) * map.jp;
        float v = 0.f;
        if (j < J) {
            const int ks = j / map.c, ch = j - (j / map.c) * map.c;
            if (ch < map.c_valid) {
                const int r = map.rtab[kr], s = map.stab[ks], nn = n + map.n_base;
                const size_t src = map.dim0_is_n ? (((size_t)nn * map.d1 + ch) * map.KH + r) * map.KW + s
                                                 : (((size_t)ch * map.d1 + nn) * map.KH + r) * map.KW + s;
                v = w[src];
            }
        }
        wp[idx] = v;
    }
}

template <int BM, int BN, int WM, int WN>
int launch_fwd_x6(const ConvBatch& b, int total, bool vec, hipStream_t stream) {
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    if (vec)
        hipLaunchKernelGGL((conv_fwd_x6_kernel<BM, BN, WM, WN, true>), dim3(total), dim3(NT), 0, stream, b);
    else
        hipLaunchKernelGGL((conv_fwd_x6_kernel<BM, BN, WM, WN, false>), dim3(total), dim3(NT), 0, stream, b);
    return fg::launched("conv_fwd_x6");
}

template <int BM, int BN, int WM, int WN>
int launch_fwd(const ConvBatch& b, int total, bool vec, hipStream_t stream) {
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    if (vec)
        hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WM, WN, true>), dim3(total), dim3(NT), 0, stream, b);
    else
        hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WM, WN, false>), dim3(total), dim3(NT), 0, stream, b);
    return fg::launched("conv_fwd");
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int BA, int BKC, int WA, int WK>
int launch_wgrad_x6(const fg_wgrad_problem& p, bool vx, bool vp, hipStream_t stream) {
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    const int K = p.kh * p.j_valid;
    const int ta = (p.n_a + BA - 1) / BA, tk = (K + BKC - 1) / BKC;
    dim3 g(ta * tk * p.splits), blk(NT);
    if (vx && vp)
        hipLaunchKernelGGL((conv_wgrad_x6_kernel<BA, BKC, WA, WK, true, true>), g, blk, 0, stream, p, ta, tk);
    else if (vx)
        hipLaunchKernelGGL((conv_wgrad_x6_kernel<BA, BKC, WA, WK, true, false>), g, blk, 0, stream, p, ta, tk);
    else if (vp)
        hipLaunchKernelGGL((conv_wgrad_x6_kernel<BA, BKC, WA, WK, false, true>), g, blk, 0, stream, p, ta, tk);
    else
        hipLaunchKernelGGL((conv_wgrad_x6_kernel<BA, BKC, WA, WK, false, false>), g, blk, 0, stream, p, ta, tk);
    return fg::launched("conv_wgrad_x6");
}

template <int BA, int BKC, int WA, int WK>
int launch_wgrad(const fg_wgrad_problem& p, bool vx, bool vp, hipStream_t stream) {
    constexpr int NT = (BA / WA) * (BKC / WK) * 64;
    const int K = p.kh * p.j_valid;
    const int ta = (p.n_a + BA - 1) / BA, tk = (K + BKC - 1) / BKC;
    const int total = ta * tk * p.splits;
    dim3 g(total), blk(NT);
    if (vx && vp)
        hipLaunchKernelGGL((conv_wgrad_kernel<BA, BKC, WA, WK, true, true>), g, blk, 0, stream, p, ta, tk);
    else if (vx)
        hipLaunchKernelGGL((conv_wgrad_kernel<BA, BKC, WA, WK, true, false>), g, blk, 0, stream, p, ta, tk);
    else if (vp)
        hipLaunchKernelGGL((conv_wgrad_kernel<BA, BKC, WA, WK, false, true>), g, blk, 0, stream, p, ta, tk);
    else
        hipLaunchKernelGGL((conv_wgrad_kernel<BA, BKC, WA, WK, false, false>), g, blk, 0, stream, p, ta, tk);
    return fg::launched("conv_wgrad");
}

}  // namespace

FG_API int fg_conv_fwd(const fg_conv_problem* probs, int nprob, hipStream_t stream) {
    if (!probs || nprob < 1 || nprob > 4) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: nprob=%d", nprob);
    ConvBatch b;
    b.count = nprob;
    int max_n = 0;
    bool vec = true;
    for (int i = 0; i < nprob; ++i) {
        const fg_conv_problem& p = probs[i];
        if (!p.x || !p.w || !p.y) return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: null pointer (problem %d)", i);
        if (p.m_img < 0 || p.m_a < 0 || p.m_b < 0 || p.kh < 1 || p.jp < BK || p.jp % BK || p.j_valid < 1 ||
            p.j_valid > p.jp || p.n_out < 1 || p.ldw < p.kh * p.jp || p.ldw % 4 || !aligned16(p.w))
            return fg::fail(FG_ERR_INVALID,
                            "fg_conv_fwd: bad geometry (problem %d: m=%dx%dx%d kh=%d j=%d/%d n=%d ldw=%d)", i,
                            p.m_img, p.m_a, p.m_b, p.kh, p.j_valid, p.jp, p.n_out, p.ldw);
        if ((long long)p.m_img * p.m_a * p.m_b >= (1LL << 31))
            return fg::fail(FG_ERR_INVALID, "fg_conv_fwd: too many rows");
        if (!aligned16(p.x) || (p.sxn | p.sxa | p.sxb | p.sxr) % 4 || p.j_valid % 4) vec = false;
        if (p.n_out > max_n) max_n = p.n_out;
        b.p[i] = p;
    }
    int BM, BN;
    if (max_n > 64) { BM = 128; BN = 128; }
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
    if (BN == 128 && (g_conv_math & FG_MATH_FWD_X6)) return launch_fwd_x6<128, 128, 64, 64>(b, total, vec, stream);
    if (BN == 128) return launch_fwd<128, 128, 64, 64>(b, total, vec, stream);
    if (BN == 64) return launch_fwd<256, 64, 64, 64>(b, total, vec, stream);
    return launch_fwd<256, 32, 64, 32>(b, total, vec, stream);
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
    if (g_conv_math & FG_MATH_WGRAD_X6) {
        if (p.n_a > 64) return launch_wgrad_x6<128, 128, 64, 64>(p, vx, vp, stream);
        if (p.n_a > 32) return launch_wgrad_x6<64, 256, 64, 64>(p, vx, vp, stream);
        return launch_wgrad_x6<32, 256, 32, 64>(p, vx, vp, stream);
    }
    if (p.n_a > 64) return launch_wgrad<128, 128, 64, 64>(p, vx, vp, stream);
    if (p.n_a > 32) return launch_wgrad<64, 256, 64, 64>(p, vx, vp, stream);
    return launch_wgrad<32, 256, 32, 64>(p, vx, vp, stream);
}

FG_API int fg_wgrad_reduce(const float* slabs, int splits, const fg_weight_map* map, float* dw, int accumulate,
                           hipStream_t stream) {
    if (!slabs || !map || !dw || splits < 1) return fg::fail(FG_ERR_INVALID, "fg_wgrad_reduce: bad args");
    if (map->kh > 8 || map->kw > 8 || map->c < 1 || map->n_out < 1)
        return fg::fail(FG_ERR_INVALID, "fg_wgrad_reduce: bad map");
    const long long total = (long long)map->n_out * map->kh * map->kw * map->c;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, slabs,
                       splits, *map, dw, accumulate);
    return fg::launched("wgrad_reduce");
}

FG_API int fg_pack_weight(const float* w, const fg_weight_map* map, float* wp, hipStream_t stream) {
    if (!w || !map || !wp) return fg::fail(FG_ERR_INVALID, "fg_pack_weight: null");
    if (map->kh > 8 || map->kw > 8 || map->jp % BK || map->jp < map->kw * map->c || map->c < 1)
        return fg::fail(FG_ERR_INVALID, "fg_pack_weight: bad map kh=%d kw=%d c=%d jp=%d", map->kh, map->kw, map->c,
                        map->jp);
    const long long total = (long long)map->n_out * map->kh * map->jp;
    hipLaunchKernelGGL(pack_weight_kernel, dim3(fg::blocks_for(total, 256, 8192)), dim3(256), 0, stream, w, *map,
                       wp);
    return fg::launched("pack_weight");
}

FG_API int fg_set_conv_math(int mode) {
    if (mode < 0 || mode > (FG_MATH_FWD_X6 | FG_MATH_WGRAD_X6))
        return fg::fail(FG_ERR_INVALID, "fg_set_conv_math: %d", mode);
    g_conv_math = mode;
    return 0;
}

FG_API int fg_get_conv_math(void) { return g_conv_math; }
