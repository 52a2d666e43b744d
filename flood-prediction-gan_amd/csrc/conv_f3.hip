// Pipelined f16x3 implicit-GEMM forward kernel for the wide convolutions of the hot path
// (N >= 128: the resblock 3x3 convs and their input gradients, conv2/conv3, the deconv1 /
// deconv2 phases, discriminator model.2/5/8): models/model_architectures.py:314-333, :407-410,
// :426-435.
//
// Why a second kernel: the register-staged kernels of conv_gemm.hip stage a 16-deep k-tile
// per barrier with a one-stage prefetch; rocprofv3 counters on the resblock conv (profiles/
// round1/r1f_pmc_fwd.json) show the MFMA pipe busy 45 % of the cycles and waves parked on
// s_waitcnt/barriers 51 % -- the im2col gather misses L2 (FETCH 9x the input) and one stage
// of MFMA work does not cover that latency.  Here both operands travel global -> LDS by
// LDS-DMA (buffer_load_dwordx4 ... lds) into a 3-deep ring of 32-deep k-stages, so every load
// has two stages of MFMA work to land, no VGPRs hold staging data and the only barrier per
// stage is a raw s_barrier after a counted vmcnt.
//
// Operands per stage (LDS, one __shared__ array):
//   A: fp32 im2col rows [BM][32] (128 B rows), gathered with per-lane row addresses; the
//      fp32 -> (h, l) fp16 split happens on the MFMA fragments after the LDS read.
//   B: the pre-split fp16 weights (fg_pack_weight_f16) as [piece][BN][32] (64 B rows).
// Both images are XOR-swizzled in 16-B chunks (the DMA writes lane-linear, so the swizzle is
// applied to the per-lane SOURCE address) so that the 16x16x32 fragment reads
// (ds_read_b128: lane l reads row l&15, k-chunk l>>4) are bank-conflict free.
// MFMA: v_mfma_f32_16x16x32_f16, three products per fragment pair (lh, hl, hh).
#include <algorithm>

#include "conv_common.hpp"

namespace {

using fgc::ConvBatch;

// 16-B chunk swizzles (found by exhaustive search over the ds_read_b128 lane groups)
__device__ __forceinline__ int swz_a(int row) { return ((row >> 1) & 1) ^ (((row >> 3) & 1) << 2); }   // 8 chunks
__device__ __forceinline__ int swz_b(int row) { return ((row >> 3) & 1) << 1; }                        // 4 chunks

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// f16x3 split with scalar f32 arithmetic (packed-f32 VALU beside MFMAs costs extra issue
// cycles): v*s = h + l, h = fp16(v*s), l = fp16(v*s - h), the residual exact in fp32
__device__ __forceinline__ void split_scalar(const float (&v)[8], float s, f16x8& h, f16x8& l) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float x0 = v[2 * e] * s, x1 = v[2 * e + 1] * s;
        const f16x2 hh = __builtin_convertvector(f32x2{x0, x1}, f16x2);
        const float r0 = x0 - (float)hh[0], r1 = x1 - (float)hh[1];
        const f16x2 ll = __builtin_convertvector(f32x2{r0, r1}, f16x2);
        h[2 * e] = hh[0];
        h[2 * e + 1] = hh[1];
        l[2 * e] = ll[0];
        l[2 * e + 1] = ll[1];
    }
}

// one stage of LDS-DMA: this wave's A_GL + B_GL 1-KiB pieces (per-lane byte offsets, per-stage
// scalar offsets)
template <int A_GL, int B_GL, int A_BYTES>
__device__ __forceinline__ void dma_stage(char* sb, int wave, __amdgpu_buffer_rsrc_t xr, __amdgpu_buffer_rsrc_t wr,
                                          const int* a_off, const int* b_off, int soff_a, int soff_b) {
#pragma unroll
    for (int i = 0; i < A_GL; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(sb + (wave * A_GL + i) * 1024), 16, a_off[i], soff_a,
                                                 0, 0);
#pragma unroll
    for (int i = 0; i < B_GL; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void*)(sb + A_BYTES + (wave * B_GL + i) * 1024), 16, b_off[i],
                                                 soff_b, 0, 0);
}

// the conv's MFMA with the operands exchanged: D^T = B^T A^T, so that a lane's 4 accumulator registers are 4
// CONSECUTIVE output columns (channels) of one output row (pixel): lane l holds row (l & 15) and columns
// 4 (l >> 4) .. +3 of its 16 x 16 block.  The NHWC epilogue then stores 16 B per lane (one dwordx4 per block)
// instead of four scattered dwords: a quarter of the store instructions, which bounded the epilogue
// (round 5: the no-epilogue diagnostic ran deconv2 in 0.67 of its time, the resblock conv in 0.92)
__device__ __forceinline__ f32x4 mma_t(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c, 0, 0, 0);
}

// QUAD: the output offset of column group q (wave-uniform per column block; a select chain, not an indexed
// kernel-argument load)
__device__ __forceinline__ int quad_yoff(const fg_conv_problem& P, int q) {
    const int y0 = (int)P.q_yoff[0], y1 = (int)P.q_yoff[1], y2 = (int)P.q_yoff[2], y3 = (int)P.q_yoff[3];
    return q == 0 ? y0 : q == 1 ? y1 : q == 2 ? y2 : y3;
}

// output buffer resource: byte offsets below kYRecords are stored, kYOOB is dropped (the host keeps every output
// extent below kYRecords, f3_takes)
constexpr int kYRecords = 0x7fffff00, kYOOB = 0x7ffffff0;

// one 1-KiB LDS-DMA piece (per-lane byte offset, per-stage scalar offset)
__device__ __forceinline__ void dma_piece(char* dst, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, voff, soff, 0, 0);
}

constexpr int cap63(int n) { return n < 63 ? n : 63; }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt immediate (6 bits)");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt(min(n, 63)) for a run-time n (the deep rings of NS > 3: a jump table, a few scalar instructions per stage)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
    switch (n < 63 ? n : 63) {
        case 0: wait_vmcnt<0>(); break;
        case 1: wait_vmcnt<1>(); break;
        case 2: wait_vmcnt<2>(); break;
        case 3: wait_vmcnt<3>(); break;
        case 4: wait_vmcnt<4>(); break;
        case 5: wait_vmcnt<5>(); break;
        case 6: wait_vmcnt<6>(); break;
        case 7: wait_vmcnt<7>(); break;
        case 8: wait_vmcnt<8>(); break;
        case 9: wait_vmcnt<9>(); break;
        case 10: wait_vmcnt<10>(); break;
        case 11: wait_vmcnt<11>(); break;
        case 12: wait_vmcnt<12>(); break;
        case 13: wait_vmcnt<13>(); break;
        case 14: wait_vmcnt<14>(); break;
        case 15: wait_vmcnt<15>(); break;
        case 16: wait_vmcnt<16>(); break;
        case 17: wait_vmcnt<17>(); break;
        case 18: wait_vmcnt<18>(); break;
        case 19: wait_vmcnt<19>(); break;
        case 20: wait_vmcnt<20>(); break;
        case 21: wait_vmcnt<21>(); break;
        case 22: wait_vmcnt<22>(); break;
        case 23: wait_vmcnt<23>(); break;
        case 24: wait_vmcnt<24>(); break;
        case 25: wait_vmcnt<25>(); break;
        case 26: wait_vmcnt<26>(); break;
        case 27: wait_vmcnt<27>(); break;
        case 28: wait_vmcnt<28>(); break;
        case 29: wait_vmcnt<29>(); break;
        case 30: wait_vmcnt<30>(); break;
        case 31: wait_vmcnt<31>(); break;
        case 32: wait_vmcnt<32>(); break;
        case 33: wait_vmcnt<33>(); break;
        case 34: wait_vmcnt<34>(); break;
        case 35: wait_vmcnt<35>(); break;
        case 36: wait_vmcnt<36>(); break;
        case 37: wait_vmcnt<37>(); break;
        case 38: wait_vmcnt<38>(); break;
        case 39: wait_vmcnt<39>(); break;
        case 40: wait_vmcnt<40>(); break;
        case 41: wait_vmcnt<41>(); break;
        case 42: wait_vmcnt<42>(); break;
        case 43: wait_vmcnt<43>(); break;
        case 44: wait_vmcnt<44>(); break;
        case 45: wait_vmcnt<45>(); break;
        case 46: wait_vmcnt<46>(); break;
        case 47: wait_vmcnt<47>(); break;
        case 48: wait_vmcnt<48>(); break;
        case 49: wait_vmcnt<49>(); break;
        case 50: wait_vmcnt<50>(); break;
        case 51: wait_vmcnt<51>(); break;
        case 52: wait_vmcnt<52>(); break;
        case 53: wait_vmcnt<53>(); break;
        case 54: wait_vmcnt<54>(); break;
        case 55: wait_vmcnt<55>(); break;
        case 56: wait_vmcnt<56>(); break;
        case 57: wait_vmcnt<57>(); break;
        case 58: wait_vmcnt<58>(); break;
        case 59: wait_vmcnt<59>(); break;
        case 60: wait_vmcnt<60>(); break;
        case 61: wait_vmcnt<61>(); break;
        case 62: wait_vmcnt<62>(); break;
        case 63: wait_vmcnt<63>(); break;
        default: wait_vmcnt<63>(); break;
    }
}

// SCH selects the per-stage instruction order: 0 = read+split all of A, then the three products
// per column group smallest first; 1 = the A reads are issued before the next stage's DMA (their
// LDS latency hides behind the DMA issue) and each column group's products run hh, hl, lh, so the
// first MFMAs need only the cheap h half of the split and the l half overlaps them; 2 = as 1, with
// the B fragments double-buffered in 2-block groups, pinned (group g+1 is read while group g's
// products run; group 0 is read together with A, ahead of the DMA issue); 3 = as 1, with the
// next stage's LDS-DMA pieces spread between the column groups instead of one burst.
// PS: the A operand is in the FG_PRESPLIT format (include/floodgan.h: per 8 channels h[8] | l[8], written
// by the norm pass that produced it) -- the two 16-B chunks a lane reads ARE its h and l fragments.
// QUAD: the merged sub-pixel phases of a stride-2 transposed conv (fg_conv_problem.q_n): every stage's k
// segment (r, pixel) is recorded beside its ring slot, and a wave runs the products of a column group (one
// phase, TG*16 = q_n columns) only where q_mask says the group reads that segment; the epilogue scatters the
// groups to their output pixels.
template <int BM, int BN, int WM, int WN, int NS, int SCH, bool STATS = false, bool PS = false, bool QUAD = false>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, 1)
conv_fwd_f3_kernel(const ConvBatch batch, int total_tiles, int alt_order) {
    constexpr int NWN = BN / WN;
    constexpr int NW = (BM / WM) * NWN;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int A_BYTES = BM * 128;          // fp32 [BM][32]
    constexpr int B_BYTES = 2 * BN * 64;       // fp16 [2][BN][32]
    constexpr int STAGE = A_BYTES + B_BYTES;
    constexpr int A_GL = A_BYTES / 1024 / NW;  // 1-KiB LDS-DMA instructions per wave per stage
    constexpr int B_GL = B_BYTES / 1024 / NW;
    static_assert(A_BYTES % (1024 * NW) == 0 && B_BYTES % (1024 * NW) == 0, "stage not a whole number of DMAs");

    __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / NWN, wn = wave - (wave / NWN) * NWN;
    // order bit 2: static priority for the second half of the waves (the arbitration losers of
    // the two waves sharing each SIMD)
    if ((alt_order & 4) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);

    // ---- persistent tile loop: workgroup w runs tiles w, w + G, w + 2G, ... (G = gridDim.x) as ONE
    // stream of k-stages -- the DMAs of the next tile's first stages are in flight while the
    // current tile finishes and writes its epilogue (short-K convs were prologue-bound).
    const int G = gridDim.x;
    const int first = fg::xcd_remap(blockIdx.x, G);
    struct Geo {
        int pi, mt, m0, n0, nkt;
    };
    auto geo = [&](int t) {
        Geo q;
        int local;
        // (tile counts stay far below 2^22: fgc::div_small is exact)
        if (batch.interleave) {
            // the count consecutive tiles of one local index are the count problems, rotated by the round
            // t / G so that every workgroup takes each problem in turn (the phases differ in K)
            local = fgc::div_small(t, batch.count);
            const int r = t - local * batch.count + fgc::div_small(t, G);
            q.pi = r - fgc::div_small(r, batch.count) * batch.count;
        } else {
            q.pi = 0;
            while (q.pi + 1 < batch.count && t >= batch.blk_start[q.pi + 1]) ++q.pi;
            local = t - batch.blk_start[q.pi];
        }
        const int ntn = batch.ntiles_n[q.pi];
        q.mt = fgc::div_small(local, ntn);
        q.m0 = q.mt * BM;
        q.n0 = (local - q.mt * ntn) * BN;
        q.nkt = batch.p[q.pi].kh * (batch.p[q.pi].jp / 32);
        return q;
    };

    // ---- issue side: the tile whose stages are being staged, its per-lane DMA sources (byte
    // offsets; the per-stage k offset is a scalar soffset) and its (r, jb) walk.
    // A: instruction i of this wave fills rows (wave*A_GL+i)*8 + lane/8, physical chunk lane%8 <-
    // logical chunk (lane%8) ^ swz_a(row); rows past M are clamped to a valid row (never stored);
    // jp == j_valid, so every k of a stage is a real tap.  B: instruction q = wave*B_GL+i fills
    // piece q / (BN/16), rows (q % (BN/16))*16 + lane/4, chunk lane%4 <- slot (lane%4) ^ swz_b(row).
    // k walk of a tile: channel chunk ic (outer), kernel row ir, tap is (inner), so the kw taps of
    // one 32-channel chunk -- the same input pixels shifted by one -- and then the kh rows are
    // gathered back to back while still in L2 (the input itself is far larger than L2).  Without a
    // usable jc (channels per pixel) the run is walked as kw = jp/32 pseudo-taps of 32 (r outer).
    int it = first, ikt = 0, ic = 0, ir = 0, is = 0;
    int i_kh = 1, i_jp = 32, i_sxr = 0, i_c = 32, i_kw = 1, i_nc = 1;   // per issue tile (no kernarg reloads)
    int i_qkw = 1, i_qsh = 5;        // QUAD: pixels per kernel row, log2(jc)
    unsigned seg_ring = 0;           // QUAD: k segment of the stage in ring slot b at bits 4b..4b+3
    bool irev = false;
    Geo ig;
    __amdgpu_buffer_rsrc_t xr, wr;
    int a_off[A_GL], b_off[B_GL];
    // QUAD: column group of each B piece, the groups live per k segment (bit seg*4 + q), a buffer resource with no
    // records: a dead group's B pieces go through it (dropped by the range check: no traffic, its LDS bytes unused)
    int b_grp[QUAD ? B_GL : 1];
    unsigned i_segmask = 0;
    __amdgpu_buffer_rsrc_t wr0;
    auto setup_issue = [&]() {
        ig = geo(it);
        const fg_conv_problem& P = batch.p[ig.pi];
        xr = __builtin_amdgcn_make_buffer_rsrc((void*)P.x, 0, 0x7fffffff, 0x00020000);
        wr = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0x7fffffff, 0x00020000);
        const int mab = P.m_a * P.m_b, M = P.m_img * mab;
#pragma unroll
        for (int i = 0; i < A_GL; ++i) {
            const int row = (wave * A_GL + i) * 8 + (lane >> 3);
            const int cl = (lane & 7) ^ swz_a(row);
            int img, a, b;
            fgc::decomp(min(ig.m0 + row, M - 1), P.m_b, mab, img, a, b);
            a_off[i] = ((int)(img * P.sxn + a * P.sxa + b * P.sxb) + cl * 4) * 4;
        }
#pragma unroll
        for (int i = 0; i < B_GL; ++i) {
            const int q = wave * B_GL + i;
            const int pc = q / (BN / 16);
            const int row = (q - pc * (BN / 16)) * 16 + (lane >> 2);
            const int cl = (lane & 3) ^ swz_b(row);
            b_off[i] = min(ig.n0 + row, P.n_out - 1) * (P.ldw / 8) * 32 + cl * 32 + pc * 16;
            if constexpr (QUAD) b_grp[i] = (ig.n0 + (q - pc * (BN / 16)) * 16) / P.q_n;
        }
        // alt_order: odd M tiles walk the kernel rows backwards, so neighbouring tiles (output rows
        // 2t, 2t+1 and 2t+2, 2t+3 at 128-px rows) gather the same input rows at the same time
        // bit 4: the same by 512-row blocks of output rows instead of by tile: every tile height up to 512 then gives
        // a row the same k order, so a sample's values do not depend on the tile config its batch size selects.  The
        // blocks are counted from the tile's image when an image holds a whole number of them (mab % 512 == 0: no
        // tile of <= 512 rows straddles two images), so a sample's k order does not depend on its position in the
        // batch either; otherwise (tiles straddle images) from the batch's first row -- tile-height invariant, but a
        // sample's values can then depend on the batch it sits in
        int lrow = ig.m0;
        if ((mab & 511) == 0) {
            int i0, a0, b0;
            fgc::decomp(ig.m0, P.m_b, mab, i0, a0, b0);
            lrow = ig.m0 - i0 * mab;
        }
        irev = (alt_order & 1) && (((alt_order & 16) ? (lrow >> 9) : ig.mt) & 1);
        i_kh = P.kh;
        i_jp = P.jp;
        i_sxr = (int)P.sxr;
        i_c = ((alt_order & 2) && P.jc > 0 && P.jc % 32 == 0 && P.jp % P.jc == 0) ? P.jc : 32;
        i_kw = P.jp / i_c;
        i_nc = i_c / 32;
        if constexpr (QUAD) {
            i_qkw = P.jp / P.jc;
            i_qsh = __builtin_ctz(P.jc);
            i_segmask = 0;
            for (int sg = 0; sg < 4; ++sg)
                for (int q = 0; q < 4; ++q)
                    if ((P.q_mask >> (q * 4 + sg)) & 1) i_segmask |= 1u << (sg * 4 + q);
            wr0 = __builtin_amdgcn_make_buffer_rsrc((void*)P.w, 0, 0, 0x00020000);
        }
        ikt = ic = ir = is = 0;
    };
    auto record_seg = [&](int buf, int r, int jb) {
        if constexpr (QUAD) {
            const unsigned seg = (unsigned)(r * i_qkw + (jb >> i_qsh));
            seg_ring = (seg_ring & ~(0xFu << (4 * buf))) | (seg << (4 * buf));
        }
    };
    // stage the next k-stage of the stream into ring buffer `buf`; false once the stream is done
    auto issue_next = [&](int buf) {
        if (it >= total_tiles) return false;
        const int r = irev ? i_kh - 1 - ir : ir;
        const int jb = is * i_c + ic * 32;
        const int koff = (r * i_sxr + jb) * 4;
        const int ks = r * (i_jp / 32) + jb / 32;        // packed-weight stage of this (r, jb)
        record_seg(buf, r, jb);
        dma_stage<A_GL, B_GL, A_BYTES>(smem + buf * STAGE, wave, xr, wr, a_off, b_off, koff, ks * 128);
        if (++is == i_kw) {
            is = 0;
            if (++ir == i_kh) { ir = 0; ++ic; }
        }
        if (++ikt == ig.nkt) {
            it += G;
            if (it < total_tiles) setup_issue();
        }
        return true;
    };

    // SCH 3: the same stage split into prep / pieces / advance, so that the pieces can be issued
    // one or two at a time between the MFMA groups of the current stage (an LDS-DMA piece costs
    // ~60 issue cycles among MFMAs but 100-185 in a burst beside the fragment reads)
    int p_koff = 0, p_soffb = 0, p_buf = 0;   // p_buf: byte offset of the target stage in smem
    bool p_on = false;
    unsigned p_live = 0xF;                     // QUAD: the column groups the staged segment feeds
    auto issue_prep = [&](int buf) {
        p_on = it < total_tiles;
        if (!p_on) return;
        const int r = irev ? i_kh - 1 - ir : ir;
        const int jb = is * i_c + ic * 32;
        p_koff = __builtin_amdgcn_readfirstlane((r * i_sxr + jb) * 4);        // scalar offsets: wave-uniform
        p_soffb = __builtin_amdgcn_readfirstlane((r * (i_jp / 32) + jb / 32) * 128);
        p_buf = buf * STAGE;
        record_seg(buf, r, jb);
        if constexpr (QUAD)
            p_live = __builtin_amdgcn_readfirstlane((i_segmask >> (4 * (r * i_qkw + (jb >> i_qsh)))) & 0xFu);
    };
    auto issue_piece = [&](int i) {
        if (!p_on) return;
        // the LDS destination is wave-uniform (M0): say so, or the compiler emits a waterfall loop
        if (i < A_GL) {
            dma_piece(smem + __builtin_amdgcn_readfirstlane(p_buf + (wave * A_GL + i) * 1024), xr, a_off[i], p_koff);
        }
        else if constexpr (QUAD) {
            const bool live = __builtin_amdgcn_readfirstlane((p_live >> b_grp[i - A_GL]) & 1u) != 0;
            dma_piece(smem + __builtin_amdgcn_readfirstlane(p_buf + A_BYTES + (wave * B_GL + (i - A_GL)) * 1024),
                      live ? wr : wr0, b_off[i - A_GL], p_soffb);
        } else
            dma_piece(smem + __builtin_amdgcn_readfirstlane(p_buf + A_BYTES + (wave * B_GL + (i - A_GL)) * 1024), wr,
                      b_off[i - A_GL], p_soffb);
    };
    auto issue_advance = [&]() {
        if (it >= total_tiles) return false;
        if (++is == i_kw) {
            is = 0;
            if (++ir == i_kh) { ir = 0; ++ic; }
        }
        if (++ikt == ig.nkt) {
            it += G;
            if (it < total_tiles) setup_issue();
        }
        return true;
    };

    // ---- compute side
    int ct = first, ckt = 0;
    Geo cg = geo(ct);
    float sa = 1.f, out_scale = 1.f;
    // QUAD: bit seg * NLG + lg: the wave's local column group lg (TG blocks) reads k segment seg
    constexpr int NLG = TN / (TN < 4 ? TN : 4);
    unsigned c_live = ~0u;
    auto setup_compute = [&]() {
        cg = geo(ct);
        sa = fgc::pow2_scale(batch.p[cg.pi].x_absmax);
        out_scale = 1.f / (sa * fgc::pow2_scale(batch.p[cg.pi].w_absmax));
        ckt = 0;
        if constexpr (QUAD) {
            const fg_conv_problem& P = batch.p[cg.pi];
            const int q0 = (cg.n0 + wn * WN) / P.q_n;
            unsigned lv = 0;
#pragma unroll
            for (int sg = 0; sg < 4; ++sg)
#pragma unroll
                for (int lg = 0; lg < NLG; ++lg)
                    if (q0 + lg < 4 && ((P.q_mask >> ((q0 + lg) * 4 + sg)) & 1)) lv |= 1u << (sg * NLG + lg);
            c_live = __builtin_amdgcn_readfirstlane(lv);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fragment addressing: lane reads row (lane & 15) of each 16-row block, k-chunk g = lane >> 4
    const int fr = lane & 15, g = lane >> 4;
    // A rows wm*WM + tm*16 + fr: bits 1..3 of the row are those of fr
    const int a_c0 = ((2 * g) ^ swz_a(fr)) * 16, a_c1 = ((2 * g + 1) ^ swz_a(fr)) * 16;
    const int b_c = (g ^ swz_b(fr)) * 16;

    // B fragments are read in column groups of TG blocks (bounded live registers); each group's
    // three products are issued smallest first
    constexpr int TG = TN < 4 ? TN : 4;
    static_assert(TN % TG == 0, "column blocks per wave must be a multiple of the group");
    auto load_a = [&](int buf, f32x4 (&va)[TM][2]) {
        const char* sbuf = smem + buf * STAGE;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const char* rowp = sbuf + (wm * WM + tm * 16 + fr) * 128;
            va[tm][0] = *reinterpret_cast<const f32x4*>(rowp + a_c0);
            va[tm][1] = *reinterpret_cast<const f32x4*>(rowp + a_c1);
        }
    };
    auto compute = [&](int buf, const f32x4 (&va)[TM][2]) {
        const char* sbuf = smem + buf * STAGE;
        // QUAD: the live column groups of this stage (all of them otherwise)
        const unsigned lv = QUAD ? (c_live >> (((seg_ring >> (4 * buf)) & 0xFu) * NLG)) : ~0u;
        f16x8 ah[TM], al[TM];
        if constexpr (PS) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                ah[tm] = __builtin_bit_cast(f16x8, va[tm][0]);
                al[tm] = __builtin_bit_cast(f16x8, va[tm][1]);
            }
        } else
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const float v[8] = {va[tm][0][0], va[tm][0][1], va[tm][0][2], va[tm][0][3],
                                va[tm][1][0], va[tm][1][1], va[tm][1][2], va[tm][1][3]};
            split_scalar(v, sa, ah[tm], al[tm]);
        }
#pragma unroll
        for (int t0 = 0; t0 < TN; t0 += TG) {
            const bool live = !QUAD || ((lv >> (t0 / TG)) & 1u);
            f16x8 bh[TG], bl[TG];
            if (live) {
#pragma unroll
                for (int t = 0; t < TG; ++t) {
                    const char* rowp = sbuf + A_BYTES + (wn * WN + (t0 + t) * 16 + fr) * 64 + b_c;
                    bh[t] = *reinterpret_cast<const f16x8*>(rowp);
                    bl[t] = *reinterpret_cast<const f16x8*>(rowp + BN * 64);
                }
            }
            if constexpr (SCH >= 3) {
                // SCH 3: pieces spread over all column groups; 4: over the first half; 5: all in the
                // first group (each piece needs time to land before the stage-end vmcnt)
                constexpr int NGA = TN / TG, NGR = SCH == 3 ? NGA : SCH == 4 ? (NGA + 1) / 2 : 1;
                constexpr int NP = A_GL + B_GL, PPG = (NP + NGR - 1) / NGR;
#pragma unroll
                for (int i = (t0 / TG) * PPG; i < (t0 / TG + 1) * PPG && i < NP; ++i) issue_piece(i);
            }
            if (!live) continue;
            if constexpr (SCH == 0) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int t = 0; t < TG; ++t)
                        acc[tm][t0 + t] = mma_t(al[tm], bh[t], acc[tm][t0 + t]);
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int t = 0; t < TG; ++t)
                        acc[tm][t0 + t] = mma_t(ah[tm], bl[t], acc[tm][t0 + t]);
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int t = 0; t < TG; ++t)
                        acc[tm][t0 + t] = mma_t(ah[tm], bh[t], acc[tm][t0 + t]);
            } else {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int t = 0; t < TG; ++t) {
                        acc[tm][t0 + t] = mma_t(ah[tm], bh[t], acc[tm][t0 + t]);
                        acc[tm][t0 + t] = mma_t(ah[tm], bl[t], acc[tm][t0 + t]);
                    }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int t = 0; t < TG; ++t)
                        acc[tm][t0 + t] = mma_t(al[tm], bh[t], acc[tm][t0 + t]);
            }
        }
    };

    constexpr int TG2 = TN < 2 ? TN : 2;
    constexpr int NG2 = TN / TG2;
    auto load_b = [&](int buf, int t0, f16x8 (&bh)[TG2], f16x8 (&bl)[TG2]) {
        const char* sbuf = smem + buf * STAGE;
#pragma unroll
        for (int t = 0; t < TG2; ++t) {
            const char* rowp = sbuf + A_BYTES + (wn * WN + (t0 + t) * 16 + fr) * 64 + b_c;
            bh[t] = *reinterpret_cast<const f16x8*>(rowp);
            bl[t] = *reinterpret_cast<const f16x8*>(rowp + BN * 64);
        }
    };
    // SCH 2: the instruction order is pinned with sched_barriers (the compiler otherwise sinks
    // every fragment read to just before its first use): region g holds group g+1's B reads, then
    // group g's MFMAs; the l half of the A split sits in region 0 among group 0's MFMAs.
    auto compute2 = [&](int buf, const f32x4 (&va)[TM][2], f16x8 (&bh)[2][TG2], f16x8 (&bl)[2][TG2]) {
        f16x8 ah[TM], al[TM];
        float xs[TM][8];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x0 = va[tm][e >> 1][(e & 1) * 2] * sa, x1 = va[tm][e >> 1][(e & 1) * 2 + 1] * sa;
                xs[tm][2 * e] = x0;
                xs[tm][2 * e + 1] = x1;
                const f16x2 hh = __builtin_convertvector(f32x2{x0, x1}, f16x2);
                ah[tm][2 * e] = hh[0];
                ah[tm][2 * e + 1] = hh[1];
            }
#pragma unroll
        for (int gi = 0; gi < NG2; ++gi) {
            const int sl = gi & 1;
            if (gi + 1 < NG2) load_b(buf, (gi + 1) * TG2, bh[sl ^ 1], bl[sl ^ 1]);
            __builtin_amdgcn_sched_barrier(0);
            if (gi == 0) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float r0 = xs[tm][2 * e] - (float)ah[tm][2 * e];
                        const float r1 = xs[tm][2 * e + 1] - (float)ah[tm][2 * e + 1];
                        const f16x2 ll = __builtin_convertvector(f32x2{r0, r1}, f16x2);
                        al[tm][2 * e] = ll[0];
                        al[tm][2 * e + 1] = ll[1];
                    }
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int t = 0; t < TG2; ++t) {
                    f32x4& c = acc[tm][gi * TG2 + t];
                    c = mma_t(ah[tm], bh[sl][t], c);
                    c = mma_t(ah[tm], bl[sl][t], c);
                }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int t = 0; t < TG2; ++t) {
                    f32x4& c = acc[tm][gi * TG2 + t];
                    c = mma_t(al[tm], bh[sl][t], c);
                }
        }
    };

    // ---- epilogue of the compute tile: scale, bias, activation, strided store (or accumulate).  Accumulator
    // layout (mma_t): acc[tm][tn][r] is row m0 + tm*16 + fr, column n0 + tn*16 + 4g + r.
    constexpr int NSTV = TM * TN, NSTS = TM * TN * 4;   // stores per epilogue: dwordx4 (NHWC) / dword (strided)
    int issued = 0, done = 0, epi_issued = 0, epi_nst = NSTS;
    auto epilogue = [&]() {
        const fg_conv_problem& P = batch.p[cg.pi];
        const int mab = P.m_a * P.m_b, M = P.m_img * mab;
        const int act = P.act;
        const bool accum = P.accumulate != 0;
        // a lane's 4 columns are contiguous and 16-B aligned in y: one dwordx4 store per block
        bool vec = P.syc == 1 && P.n_out % 4 == 0 && ((uintptr_t)P.y & 15) == 0 &&
                   ((P.syn | P.sya | P.syb) & 3) == 0;
        if constexpr (QUAD) vec = vec && ((P.q_yoff[0] | P.q_yoff[1] | P.q_yoff[2] | P.q_yoff[3]) & 3) == 0;
        // QUAD: column n = q * q_n + o is channel o of the pixel at q_yoff[q] (q uniform per 16-column block); its
        // statistics partials sit in group q's region ([rb][q_n][2] at q * q_soff)
        int nc0[TN], ych[TN], yq[TN];
        f32x4 bias4[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            nc0[tn] = cg.n0 + wn * WN + tn * 16 + 4 * g;
            if constexpr (QUAD) {
                yq[tn] = nc0[tn] / P.q_n;
                ych[tn] = nc0[tn] - yq[tn] * P.q_n;
            } else {
                yq[tn] = 0;
                ych[tn] = nc0[tn];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) bias4[tn][r] = P.bias ? P.bias[min(ych[tn] + r, P.n_out - 1)] : 0.f;
        }
        const bool full_n = cg.n0 + BN <= P.n_out;
        if (STATS && P.in_stats) {
            // InstanceNorm partials of each 32-row block of this wave's rows (WM / 32 of them: tm blocks hb*TB ..
            // hb*TB+1, 16 rows each across the lanes of a DPP row), per column: two passes (mean, then M2) over the raw
            // accumulators -- the two rows of a lane summed in registers, then over the 16 lanes of the row
            // (fg::row_sum16); out_scale (a power of 2) and the bias are applied to the results
            constexpr int NB = WM / 32, TB = TM / NB;
            static_assert(WM % 32 == 0 && TB * 16 == 32, "32-row statistics blocks");
#pragma unroll
            for (int hb = 0; hb < NB; ++hb) {
            const int rb0 = cg.m0 + wm * WM + hb * 32;
            if (rb0 < M) {
                const float sc = out_scale;
                float* const dst0 = P.in_stats + (size_t)(rb0 / 32) * (QUAD ? P.q_n : P.n_out) * 2;
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    f32x4 sm, sq;
#pragma unroll
                    for (int r = 0; r < 4; ++r) sm[r] = fg::row_sum16(acc[hb * TB][tn][r] + acc[hb * TB + 1][tn][r]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float mu = sm[r] * (1.f / 32);
                        sm[r] = mu;
                        const float d0 = acc[hb * TB][tn][r] - mu, d1 = acc[hb * TB + 1][tn][r] - mu;
                        sq[r] = fg::row_sum16(d0 * d0 + d1 * d1);
                    }
                    if (fr == 0) {
                        float* const dst = dst0 + (QUAD ? yq[tn] * P.q_soff : 0) + ych[tn] * 2;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (nc0[tn] + r < P.n_out)
                                *reinterpret_cast<f32x2*>(dst + 2 * r) =
                                    f32x2{sm[r] * sc + bias4[tn][r], sq[r] * (sc * sc)};
                    }
                }
            }
            }
        }
        // the stores: TM x TN dwordx4 (vec) or TM x TN x 4 dword buffer stores per lane, ALWAYS issued (rows past M /
        // columns past n_out get an out-of-range offset, which the hardware drops), so the stage waits after this
        // epilogue can leave exactly that many younger VMEM operations in flight (see wait_stage)
        const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)P.y, 0, kYRecords, 0x00020000);
        int coff[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) coff[tn] = ych[tn] * (int)P.syc + (QUAD ? quad_yoff(P, yq[tn]) : 0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = cg.m0 + wm * WM + tm * 16 + fr;
            int img, a, b;
            fgc::decomp(min(m, M - 1), P.m_b, mab, img, a, b);
            const bool row_ok = m < M;
            const int roff = img * (int)P.syn + a * (int)P.sya + b * (int)P.syb;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fg::act_fwd(acc[tm][tn][r] * out_scale + bias4[tn][r], act);
                if (vec) {
                    const bool ok = row_ok && (full_n || nc0[tn] < P.n_out);
                    if (accum && ok) v += *reinterpret_cast<const f32x4*>(P.y + roff + coff[tn]);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yr,
                                                           ok ? (roff + coff[tn]) * 4 : kYOOB, 0, 0);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const bool ok = row_ok && (full_n || nc0[tn] + r < P.n_out);
                        const int off = roff + coff[tn] + r * (int)P.syc;
                        float w = v[r];
                        if (accum && ok) w += P.y[off];
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w), yr, ok ? off * 4 : kYOOB, 0, 0);
                    }
                }
            }
        }
        epi_issued = issued;
        epi_nst = vec ? NSTV : NSTS;
    };

    // ---- NS-deep ring over the stage stream: stage s+NS-1 is issued right after the barrier that
    // retires stage s-1's reads; before it, this wave waits for its own DMAs of stage s (counted
    // vmcnt: the younger NS-2 stages stay in flight) and the barrier makes everyone's visible
    static_assert(NS >= 2 && NS <= 6, "ring depth");
    if (first >= total_tiles) return;
    setup_issue();
    setup_compute();
#pragma unroll
    for (int s0 = 0; s0 < NS - 1; ++s0)
        if (issue_next(s0)) ++issued;
    int cur = 0, nxt = NS - 1;
    // wait for stage `done`'s own DMAs: the VMEM operations younger than them are the stages issued after it
    // and, when stage `done` was issued before the last epilogue, that epilogue's epi_nst stores (vmcnt counts
    // loads, LDS-DMA and stores together, in issue order).  Any smaller count is safe (it waits for more): each
    // branch waits for min(c, 63) with c <= younger.  The store counts are the trip counts of the epilogue's two
    // store loops (never predicated off); tests/test_isa_cpu.py checks every instantiation's code object issues
    // exactly NSTV dwordx4 and NSTS dword buffer stores and no other widths.
    constexpr int D = A_GL + B_GL;
    auto wait_stage = [&]() {
        const int younger = (issued - done - 1) * D + (done < epi_issued ? epi_nst : 0);
        if constexpr (NS > 3) {            // the latency-bound small launches' deep ring: the exact count
            wait_vmcnt_rt(younger);
            return;
        }
        if (NS == 3 && younger >= NSTS + 2 * D) wait_vmcnt<cap63(NSTS + 2 * D)>();
        else if (younger >= NSTS + D) wait_vmcnt<cap63(NSTS + D)>();
        else if (younger >= NSTS) wait_vmcnt<cap63(NSTS)>();
        else if (NS == 3 && younger >= NSTV + 2 * D) wait_vmcnt<cap63(NSTV + 2 * D)>();
        else if (younger >= NSTV + D) wait_vmcnt<cap63(NSTV + D)>();
        else if (younger >= NSTV) wait_vmcnt<cap63(NSTV)>();
        else if (NS == 3 && younger >= 2 * D) wait_vmcnt<cap63(2 * D)>();
        else if (younger >= D) wait_vmcnt<cap63(D)>();
        else wait_vmcnt<0>();
    };
    // order bit 3 (SCH >= 3): at a tile boundary the ring slot just computed is refilled BEFORE the epilogue's
    // stores (after a barrier: every wave is done reading it), and the next stage issues nothing.  vmcnt retires
    // in issue order, so the stage waits then reach the stores one stage later: they drain under two stages of
    // MFMAs instead of one (every CU finishes its tile at the same time and the write burst queues).
    const bool pre_epi = SCH >= 3 && (alt_order & 8);
    bool pre_issued = false;
    while (true) {
        wait_stage();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        f32x4 va[TM][2];
        if constexpr (SCH == 0) {
            if (issue_next(nxt)) ++issued;
            load_a(cur, va);
            compute(cur, va);
        } else if constexpr (SCH == 1) {
            load_a(cur, va);
            if (issue_next(nxt)) ++issued;
            compute(cur, va);
        } else if constexpr (SCH >= 3) {
            load_a(cur, va);
            if (pre_issued) p_on = false;
            else issue_prep(nxt);
            compute(cur, va);
            if (!pre_issued && issue_advance()) ++issued;
            pre_issued = false;
        } else {
            f16x8 bh[2][TG2], bl[2][TG2];
            load_a(cur, va);
            load_b(cur, 0, bh[0], bl[0]);
            if (issue_next(nxt)) ++issued;
            compute2(cur, va, bh, bl);
        }
        ++done;
        cur = cur == NS - 1 ? 0 : cur + 1;
        nxt = nxt == NS - 1 ? 0 : nxt + 1;
        if (++ckt == cg.nkt) {
            if constexpr (SCH >= 3) {
                bool pre = pre_epi && it < total_tiles;
                if (pre) {
                    __builtin_amdgcn_s_barrier();
                    issue_prep(nxt);
#pragma unroll
                    for (int i = 0; i < A_GL + B_GL; ++i) issue_piece(i);
                    if (issue_advance()) ++issued;
                    pre_issued = true;
                }
            }
            epilogue();
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
            ct += G;
            if (ct >= total_tiles) break;
            setup_compute();
        }
    }
}

int g_f3_alt = 31;    // fg_set_f3_order: bit 0 alternates the kernel-row order of odd M tiles,
                      // bit 1 walks k chunk-outer (taps of one channel chunk back to back),
                      // bit 2 raises the priority of the second half of the waves,
                      // bit 3 refills the freed ring slot before a tile's epilogue stores,
                      // bit 4 takes bit 0's parity from 512-row blocks instead of tiles
int g_f3_persist = 1; // fg_set_f3_persistent: 1 resident workgroups loop over tiles, 0 one workgroup per
                      // tile, n >= 2 at most n workgroups (test hook: forces the tile-crossing stream
                      // -- setup_issue() mid-stream, next tile's stages in flight over an epilogue --
                      // at small sizes)
int g_f3_interleave = 1;  // fg_set_f3_interleave: 0 = problem-major tile order (A/B hook)
int g_f3_sched = -1;  // fg_set_f3_sched: per-stage instruction order (kernel template SCH), -1 auto

template <int BM, int BN, int WM, int WN, int NS = 3>
int launch_cfg(const ConvBatch& in, int nprob, hipStream_t stream) {
    constexpr int NT = (BM / WM) * (BN / WN) * 64;
    ConvBatch b = in;
    int total = 0;
    for (int i = 0; i < nprob; ++i) {
        const long long M = (long long)b.p[i].m_img * b.p[i].m_a * b.p[i].m_b;
        b.ntiles_n[i] = (b.p[i].n_out + BN - 1) / BN;
        b.blk_start[i] = total;
        total += (int)((M + BM - 1) / BM) * b.ntiles_n[i];
    }
    for (int i = nprob; i < 4; ++i) { b.ntiles_n[i] = 1; b.blk_start[i] = total; }
    b.blk_start[nprob] = total;
    b.blk_start[4] = total;
    if (total == 0) return 0;
    if (total >= (1 << 22)) return fg::fail(FG_ERR_INVALID, "conv_fwd_f3: %d tiles (the tile walk assumes < 2^22)", total);
    // phase-interleaved tile order when every problem has the same tile count (the 4 phases of an even-sized
    // transposed conv / stride-2 input gradient): the phases gather the same input rows at the same time
    // persistent: as many workgroups as fit at once (LDS-limited), each looping over tiles
    constexpr int LDS = NS * (BM * 128 + 2 * BN * 64);
    const int per_cu = (160 * 1024) / LDS;
    const int grid = g_f3_persist ? std::min(total, g_f3_persist > 1 ? g_f3_persist : fg::num_cus() * per_cu) : total;
    b.interleave = 0;
    if (nprob > 1 && g_f3_interleave && grid % nprob == 0) {
        bool eq = true;
        for (int i = 1; i < nprob; ++i) eq &= b.blk_start[i + 1] - b.blk_start[i] == b.blk_start[1];
        b.interleave = eq ? 1 : 0;
    }
    const int sched = g_f3_sched >= 0 ? g_f3_sched : 3;
    bool stats = false;
    for (int i = 0; i < nprob; ++i) stats |= b.p[i].in_stats != nullptr;
    // pre-split A operands (every problem of the batch, checked by the caller): their own instantiations
    // (WM = 32 configs, default order)
    if (b.p[0].q_n) {
        // the quad form (fg_conv_problem.q_n): pre-split operands on the 256 x 256 tile of 64 x 128 waves only
        if constexpr (BM == 256 && BN == 256 && WM == 64 && WN == 128) {
            if (stats)
                FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3, true, true, true>), dim3(grid), dim3(NT),
                                   0, stream, b, total, g_f3_alt);
            else
                FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3, false, true, true>), dim3(grid),
                                   dim3(NT), 0, stream, b, total, g_f3_alt);
            return fg::launched("conv_fwd_f3_quad");
        }
        return fg::fail(FG_ERR_INVALID, "conv_fwd_f3: the quad form runs on the 256 x 256 pre-split tile only");
    }
    if (b.p[0].x_presplit) {
        if (stats) {
            FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3, true, true>), dim3(grid), dim3(NT), 0,
                               stream, b, total, g_f3_alt);
            return fg::launched("conv_fwd_f3_presplit");
        }
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3, false, true>), dim3(grid), dim3(NT), 0, stream, b,
                           total, g_f3_alt);
        return fg::launched("conv_fwd_f3_presplit");
    }
    // the epilogue-statistics variant is its own instantiation (WM = 32 configs, default order), so that
    // the launches without statistics keep the plain epilogue's code
    if constexpr (WM == 32) {
        if (stats) {
            FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3, true>), dim3(grid), dim3(NT), 0, stream, b,
                               total, g_f3_alt);
            return fg::launched("conv_fwd_f3");
        }
    }
    if (stats) return fg::fail(FG_ERR_INVALID, "conv_fwd_f3: epilogue statistics need a WM = 32 tile");
    if (sched == 5)
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 5>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    else if (sched == 4)
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 4>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    else if (sched == 3)
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 3>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    else if (sched == 2)
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 2>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    else if (sched == 1)
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 1>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    else
        FG_LAUNCH((conv_fwd_f3_kernel<BM, BN, WM, WN, NS, 0>), dim3(grid), dim3(NT), 0, stream, b, total,
                           g_f3_alt);
    return fg::launched("conv_fwd_f3");
}

}  // namespace

int g_f3_tile = -1;   // tuning hook (fg_set_f3_tile): -2 disables the kernel, >= 0 forces a config

namespace fgc {

int f3_config(int max_n) {
    return g_f3_tile >= 0 ? g_f3_tile : (max_n > 128 ? 4 : max_n > 64 ? 6 : max_n > 32 ? 7 : -1);
}

// tiles a batch makes on a BM x BN tile
long long batch_tiles(const fg_conv_problem* p, int nprob, int bm, int bn) {
    long long t = 0;
    for (int i = 0; i < nprob; ++i)
        t += ((long long)p[i].m_img * p[i].m_a * p[i].m_b + bm - 1) / bm * ((p[i].n_out + bn - 1) / bn);
    return t;
}

// the automatic choice for a batch that leaves at least half the CUs without a tile: narrower 256-row tiles
// (cfg 4 -> 6 -> 7) while that is so, then 128 x 64 (cfg 9).  A workgroup's time is its tile's K walk, so a
// launch with idle CUs finishes sooner on more, smaller tiles: D model.8's input gradient in the G step (bs 8,
// 128 tiles) 496 -> 354 us and model.5's forward 145 -> 103 us on cfg 6, the resblock input gradient's edge
// strips (18 tiles) 75 -> 33 us on cfg 9 (profiles/round2/r2ac_underfill.log, r2aa_strips.log).  A nearly full
// wave stays (D model.8's forward, 250 tiles: 322 us on cfg 4, 367 on cfg 6).  All have 32-row wave blocks.
int g_f3_fill = 1;    // fg_set_f3_fill: 0 = keep the tile f3_config picks by N (A/B hook)

int g_f3_ps_wide = 5;  // fg_set_f3_ps_wide: the N > 128 tile of pre-split operands (4: 8 waves of 32 x 256; 5: of
                       // 64 x 128 -- a third fewer fragment bytes per MFMA, the operand needing no split: resblock
                       // 0.371 -> 0.348 ms, profiles/round3/r3v_f3_presplit_cfg.log.  4 waves of 128 x 128 with the
                       // accumulators in AGPRs ran 3.26 ms: not kept)

// Narrow-N wave tiles: the 32 x 64 / 32 x 128 wave tiles of cfg 7 / 6 read 512 / 427 B of LDS fragments per MFMA --
// at the LDS port's 128 B per clock that is at or beyond what the four SIMDs' MFMAs consume -- where 64 x 64 wave
// tiles read 341 (the resblock's 64 x 128: 256): cfg 10 = 512 x 64 as 8 waves of 64 x 64, cfg 11 = 256 x 128 as
// 4 x 2 waves of 64 x 64.  Taken whenever the launch still fills half the CUs on them: the step 46.16 -> 46.02 ms
// (interleaved A/B, profiles/round4/r4e_ab_f3_narrow.log); FLOODGAN_F3_NARROW=0 keeps cfg 7 / 6
static bool narrow_on() {
    static const bool on = [] { const char* e = getenv("FLOODGAN_F3_NARROW"); return !e || atoi(e) != 0; }();
    return on;
}

// N = 65..128 on pre-split operands: cfg 12 = 512 x 128 as 8 waves of 64 x 128 -- the resblock tile's wave shape
// (96 MFMAs per wave between two barriers, 24 fragment reads), where the 64 x 64 waves of cfg 11 run 48 per barrier;
// its two 80 KB stages are the whole 160 KB of LDS.  Taken whenever the launch still fills half the CUs.
int g_f3_ps_tall = 1;  // fg_set_f3_ps_tall (A/B hook): 0 keeps cfg 11 / 6

int auto_cfg(const fg_conv_problem* p, int nprob, int max_n) {
    int cfg = f3_config(max_n);
    if (cfg < 0) return cfg;
    if (p[0].q_n) return 5;      // the quad form's one tile (launch_cfg), whatever tile fg_set_f3_tile forces
    if (g_f3_tile >= 0) return cfg;
    if (cfg == 6 && g_f3_ps_tall && p[0].x_presplit && 2 * batch_tiles(p, nprob, 512, 128) > fg::num_cus()) return 12;
    if (narrow_on() && (cfg == 6 || cfg == 7)) {
        const int alt = cfg == 7 ? 10 : 11;
        const int bm = alt == 10 ? 512 : 256, bn = alt == 10 ? 64 : 128;
        if (2 * batch_tiles(p, nprob, bm, bn) > fg::num_cus()) return alt;
    }
    if (cfg == 4 && p[0].x_presplit && 2 * batch_tiles(p, nprob, 256, 256) > fg::num_cus()) return g_f3_ps_wide;
    if (!g_f3_fill) return cfg;
    const int cus = fg::num_cus();
    while (cfg == 4 || cfg == 6 || cfg == 7) {
        const int bn = cfg == 4 ? 256 : cfg == 6 ? 128 : 64;
        if (2 * batch_tiles(p, nprob, 256, bn) > cus) return cfg;
        cfg = cfg == 4 ? 6 : cfg == 6 ? 7 : 9;
    }
    return cfg;
}

// a pre-split A operand: every k group of 8 is one pixel's 8-channel group (32-B aligned, whole groups)
bool presplit_ok(const fg_conv_problem& p) {
    return p.jp % 32 == 0 && p.jc % 8 == 0 && p.jc > 0 && ((uintptr_t)p.x & 31) == 0 &&
           (p.sxn | p.sxa | p.sxb | p.sxr) % 8 == 0;
}

bool f3_takes(const fg_conv_problem* probs, int nprob, int max_n) {
    if (g_f3_tile == -2 || f3_config(max_n) < 0) return false;
    for (int i = 0; i < nprob; ++i) {
        const fg_conv_problem& p = probs[i];
        if ((p.x_presplit != 0) != (probs[0].x_presplit != 0) || (p.x_presplit && !presplit_ok(p))) return false;
        // the epilogue's buffer stores address the output with 31-bit byte offsets
        long long qext = 0;
        if (p.q_n) {
            // the quad form: one pre-split problem, 256 columns in 4 groups of 64 (the 64 x 128 waves hold two
            // groups each), k segments = kh * (jp / jc) <= 4 pixels of a power-of-two jc
            if (nprob != 1 || !p.x_presplit || p.q_n != 64 || p.n_out != 256 || p.jc < 32 || (p.jc & (p.jc - 1)) ||
                p.jp % p.jc || p.kh * (p.jp / p.jc) > 4 || p.q_soff < 0 || p.q_soff > (1LL << 28))
                return false;
            for (int q = 0; q < 4; ++q) {
                if (p.q_yoff[q] < 0) return false;
                qext = std::max(qext, p.q_yoff[q]);
            }
        }
        // the epilogue's buffer stores address the output with 31-bit byte offsets
        const long long yext = 4 * ((long long)(p.m_img - 1) * p.syn + (long long)(p.m_a - 1) * p.sya +
                                    (long long)(p.m_b - 1) * p.syb +
                                    (long long)((p.q_n ? p.q_n : p.n_out) - 1) * p.syc + qext + 1);
        if (p.syn < 0 || p.sya < 0 || p.syb < 0 || p.syc < 0 || yext >= kYRecords) return false;
        // no K padding (every staged k is a real tap: padded j would gather past the row run); ldw may exceed
        // kh * jp (a kernel-row range of a larger pack: the resblock input gradient's row strips)
        if (p.w_split != 2 || p.jp % 32 || p.j_valid != p.jp || p.ldw < p.kh * p.jp || !p.x_absmax || !p.w_absmax ||
            p.m_img * p.m_a * p.m_b < 1)
            return false;
    }
    return true;
}

// the epilogue statistics need whole 32-row wave blocks inside one image (WM = 32 configs; every config on pre-split
// operands, whose instantiations take 32-row blocks of taller wave tiles)
bool f3_stats_ok(const fg_conv_problem* probs, int nprob, int max_n) {
    if (!f3_takes(probs, nprob, max_n)) return false;
    const int cfg = auto_cfg(probs, nprob, max_n);
    if (!probs[0].x_presplit && !(cfg == 0 || cfg == 3 || cfg == 4 || cfg == 6 || cfg == 7 || cfg == 9))
        return false;   // WM = 32 configs
    for (int i = 0; i < nprob; ++i) {
        const fg_conv_problem& p = probs[i];
        if ((p.m_a * p.m_b) % 32 || p.act != 0 || p.accumulate) return false;
    }
    return true;
}


int launch_fwd_f3(const ConvBatch& b, int nprob, int max_n, hipStream_t stream, int* rc) {
    if (!f3_takes(b.p, nprob, max_n)) return 0;
    // N <= 64: the 256-row tile (cfg 7) beats the 128-row one by 4-13 % on the step's N=64 convs (content
    // input gradient 1.67 vs 1.92 ms, deconv2 / conv2-dgrad phases 0.626 vs 0.653 ms at bs 8 512^2:
    // profiles/round2/r2r_diag_n64.log)
    const int cfg = auto_cfg(b.p, nprob, max_n);
    switch (cfg) {
        case 0: *rc = launch_cfg<128, 256, 32, 128>(b, nprob, stream); return 1;
        case 1: *rc = launch_cfg<256, 128, 64, 64>(b, nprob, stream); return 1;
        case 2: *rc = launch_cfg<128, 256, 64, 64>(b, nprob, stream); return 1;
        case 3: *rc = launch_cfg<128, 128, 32, 64>(b, nprob, stream); return 1;
        case 4: *rc = launch_cfg<256, 256, 32, 256, 2>(b, nprob, stream); return 1;
        case 5: *rc = launch_cfg<256, 256, 64, 128, 2>(b, nprob, stream); return 1;
        case 6: *rc = launch_cfg<256, 128, 32, 128, 2>(b, nprob, stream); return 1;
        case 7: *rc = launch_cfg<256, 64, 32, 64, 3>(b, nprob, stream); return 1;
        case 8: *rc = launch_cfg<256, 64, 64, 64, 3>(b, nprob, stream); return 1;
        case 9: *rc = launch_cfg<128, 64, 32, 64, 6>(b, nprob, stream); return 1;
        case 10: *rc = launch_cfg<512, 64, 64, 64, 2>(b, nprob, stream); return 1;
        case 11: *rc = launch_cfg<256, 128, 64, 64, 3>(b, nprob, stream); return 1;
        case 12: *rc = launch_cfg<512, 128, 64, 128, 2>(b, nprob, stream); return 1;
        default: return 0;
    }
}

}  // namespace fgc

FG_API int fg_set_f3_tile(int cfg) {
    if (cfg < -2 || cfg > 12) return fg::fail(FG_ERR_INVALID, "fg_set_f3_tile: %d", cfg);
    g_f3_tile = cfg;
    return 0;
}

FG_API int fg_set_f3_persistent(int on) {
    if (on < 0) return fg::fail(FG_ERR_INVALID, "fg_set_f3_persistent: %d", on);
    g_f3_persist = on;
    return 0;
}

FG_API int fg_set_f3_sched(int sched) {
    if (sched < -1 || sched > 5) return fg::fail(FG_ERR_INVALID, "fg_set_f3_sched: %d", sched);
    g_f3_sched = sched;
    return 0;
}

FG_API int fg_set_f3_order(int alt) {
    if (alt < 0 || alt > 31) return fg::fail(FG_ERR_INVALID, "fg_set_f3_order: %d", alt);
    g_f3_alt = alt;
    return 0;
}

FG_API int fg_set_f3_interleave(int on) {
    if (on < 0 || on > 1) return fg::fail(FG_ERR_INVALID, "fg_set_f3_interleave: %d", on);
    g_f3_interleave = on;
    return 0;
}

FG_API int fg_set_f3_ps_wide(int cfg) {
    if (cfg != 4 && cfg != 5) return fg::fail(FG_ERR_INVALID, "fg_set_f3_ps_wide: %d", cfg);
    fgc::g_f3_ps_wide = cfg;
    return 0;
}

FG_API int fg_set_f3_ps_tall(int on) {
    if (on < 0 || on > 1) return fg::fail(FG_ERR_INVALID, "fg_set_f3_ps_tall: %d", on);
    fgc::g_f3_ps_tall = on;
    return 0;
}

FG_API int fg_set_f3_fill(int on) {
    if (on < 0 || on > 1) return fg::fail(FG_ERR_INVALID, "fg_set_f3_fill: %d", on);
    fgc::g_f3_fill = on;
    return 0;
}
