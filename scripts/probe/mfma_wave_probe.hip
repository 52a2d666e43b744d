// Diagnostic probe (not part of the library): the compute-only ceiling of the resblock tile's wave structures.
//
// A 256 x 256 output tile per workgroup, f16x3 products (h*l, l*h, h*h per 16x16x32 block, as conv_f3.hip), every
// k-step's fragments re-read from LDS by ds_read_b128, no global traffic, no barriers, random operands:
//   WAVES 8: 8 waves of 64 x 128 (two per SIMD, 128 accumulator registers each) -- the product kernel's layout;
//   WAVES 4: 4 waves of 128 x 128 (one per SIMD, 256 accumulators in AGPRs) -- the verdict's proposed layout,
//            in two read schedules: all fragments of a k-step up front (SCHED 0), or A and B in halves with the
//            next quarter's reads interleaved one per MFMA (SCHED 1, sched_group_barrier).
// and the product layout with the pipeline's costs added one at a time: a barrier per k-step (SCHED 2), and the
// two-stage LDS-DMA ring (SCHED 3: 64 KB per stage by buffer_load ... lds from an L2-resident source, the issuing
// wave's vmcnt wait and the barrier before each stage's fragment reads, the next stage's DMA issued after it; SCHED 4:
// the same with each wave's 8 DMA pieces spread two per row block, pinned by sched_barrier; SCHED 5: the SCHED 3
// ring moving half the bytes, 4 pieces per wave per stage -- the DMA volume's share of the ring's cost).
// Prints f16 MFMA TFLOP/s (three products = one fp32-equivalent MAC: divide by 3 for the f16x3 rate) and the
// in-kernel clock (s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe/mfma_wave_probe scripts/probe/mfma_wave_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int TILE = 256, KS = 32;
constexpr int IMG = TILE * KS * 2;          // bytes per [256 rows][32 halfs] piece image

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ f16x8 frag(const char* img, int row, int lane) {
    // lane -> row (lane % 16) of the 16-row block, k group (lane / 16) * 8; 64-B rows, 16-B chunks swizzled by row
    const int r = row + (lane & 15), kg = lane >> 4;
    return *reinterpret_cast<const f16x8*>(img + r * 64 + ((kg ^ ((r >> 1) & 3)) << 4));
}

template <int WAVES, int SCHED>
__global__ void __launch_bounds__(WAVES * 64, 1) probe(const f16x8* __restrict__ src, float* __restrict__ out,
                                                        long long* __restrict__ clk, int iters) {
    constexpr int WM = WAVES == 8 ? 64 : 128, WN = 128, TM = WM / 16, TN = WN / 16;
    constexpr int NBUF = SCHED >= 3 ? 2 : 1;
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * 4 * IMG];   // [buffer][A h, A l, B h, B l]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 4 * IMG / 16; i += WAVES * 64)
        reinterpret_cast<f16x8*>(smem)[i] = src[(blockIdx.x * 977 + i) % (8 * 4 * IMG / 16)];
    __syncthreads();
    const int r0 = (wave / (TILE / WN)) * WM, c0 = (wave % (TILE / WN)) * WN;
    const char *ah = smem, *al = smem + IMG, *bh = smem + 2 * IMG, *bl = smem + 3 * IMG;
    // SCHED 3: each wave DMAs 8 of a stage's 64 1-KiB pieces; the source cycles over 8 stages (512 KB, L2-resident)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
    auto dma = [&](int stage, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < (SCHED == 5 ? 4 : 8); ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(smem + buf * 4 * IMG + (wave * 8 + i) * 1024), 16,
                                                     lane * 16, ((stage & 7) * 64 + wave * 8 + i) * 1024, 0, 0);
    };
    if constexpr (SCHED >= 3) {
        dma(0, 0);
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const long long t0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        asm volatile("" ::: "memory");       // the fragments are re-read every k-step, as in the real loop
        if constexpr (SCHED == 2) __builtin_amdgcn_s_barrier();
        if constexpr (SCHED >= 3) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if ((SCHED == 3 || SCHED == 5) && it + 1 < iters) dma(it + 1, (it + 1) & 1);
            const int o = (it & 1) * 4 * IMG;
            ah = smem + o;
            al = smem + o + IMG;
            bh = smem + o + 2 * IMG;
            bl = smem + o + 3 * IMG;
        }
        if constexpr (SCHED != 1) {
            f16x8 xa[TM], ya[TM], xb[TN], yb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) { xa[i] = frag(ah, r0 + 16 * i, lane); ya[i] = frag(al, r0 + 16 * i, lane); }
#pragma unroll
            for (int j = 0; j < TN; ++j) { xb[j] = frag(bh, c0 + 16 * j, lane); yb[j] = frag(bl, c0 + 16 * j, lane); }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(yb[j], xa[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb[j], ya[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb[j], xa[i], acc[i][j], 0, 0, 0);
                }
                if constexpr (SCHED == 4) {
                    // two of the wave's 8 pieces after each row block's 24 MFMAs (pinned by sched_barrier); the
                    // last stage's pieces land in the buffer nobody reads again
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const int piece = 2 * i + q;
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rs, (lds_void*)(smem + ((it + 1) & 1) * 4 * IMG + (wave * 8 + piece) * 1024), 16, lane * 16,
                            ((((it + 1) & 7) * 64) + wave * 8 + piece) * 1024, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else {
            // quarters (A half, B half): (0,0) (0,1) (1,1) (1,0); each quarter's 48 MFMAs carry the reads of the
            // next half the schedule needs (sched_group_barrier: one ds_read between consecutive MFMAs)
            constexpr int HM = TM / 2, HN = TN / 2;
            f16x8 xa[2][HM], ya[2][HM], xb[2][HN], yb[2][HN];
#pragma unroll
            for (int i = 0; i < HM; ++i) { xa[0][i] = frag(ah, r0 + 16 * i, lane); ya[0][i] = frag(al, r0 + 16 * i, lane); }
#pragma unroll
            for (int j = 0; j < HN; ++j) { xb[0][j] = frag(bh, c0 + 16 * j, lane); yb[0][j] = frag(bl, c0 + 16 * j, lane); }
            auto quarter = [&](int qa, int qb) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < HM; ++i)
#pragma unroll
                    for (int j = 0; j < HN; ++j) {
                        acc[qa * HM + i][qb * HN + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            yb[qb][j], xa[qa][i], acc[qa * HM + i][qb * HN + j], 0, 0, 0);
                        acc[qa * HM + i][qb * HN + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            xb[qb][j], ya[qa][i], acc[qa * HM + i][qb * HN + j], 0, 0, 0);
                        acc[qa * HM + i][qb * HN + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            xb[qb][j], xa[qa][i], acc[qa * HM + i][qb * HN + j], 0, 0, 0);
                    }
            };
            // B half 1 arrives under quarter (0,0)
#pragma unroll
            for (int j = 0; j < HN; ++j) { xb[1][j] = frag(bh, c0 + 16 * (HN + j), lane); yb[1][j] = frag(bl, c0 + 16 * (HN + j), lane); }
            quarter(0, 0);
#pragma unroll
            for (int g = 0; g < 2 * HN; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            // A half 1 arrives under quarter (0,1)
#pragma unroll
            for (int i = 0; i < HM; ++i) { xa[1][i] = frag(ah, r0 + 16 * (HM + i), lane); ya[1][i] = frag(al, r0 + 16 * (HM + i), lane); }
            quarter(0, 1);
#pragma unroll
            for (int g = 0; g < 2 * HM; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            quarter(1, 1);
            quarter(1, 0);
        }
    }
    if constexpr (SCHED >= 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * WAVES * 64 + tid] = s;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
}

template <int WAVES, int SCHED>
void run(const f16x8* src, float* out, long long* clk, int blocks, int iters, const char* name) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<WAVES, SCHED>), dim3(blocks), dim3(WAVES * 64), 0, 0, src, out, clk, iters);
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((probe<WAVES, SCHED>), dim3(blocks), dim3(WAVES * 64), 0, 0, src, out, clk, iters);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::vector<long long> c(2 * blocks);
    CHECK(hipMemcpy(c.data(), clk, c.size() * sizeof(long long), hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int i = 0; i < blocks; ++i) ghz += (double)c[2 * i] / (double)c[2 * i + 1] * 0.1;
    ghz /= blocks;
    const double mfmas = (double)blocks * (TILE / 16) * (TILE / 16) * 3 * iters * reps;
    const double tf = mfmas * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
    const double cyc_per_mfma = (double)c[0] / ((double)(TILE / 16) * (TILE / 16) * 3 * iters / 4);  // per SIMD
    printf("%-44s %7.1f TFLOP/s f16 (%6.1f f16x3, %.3f of 833.3)  clock %.2f GHz  %.1f cyc per MFMA per SIMD\n", name,
           tf, tf / 3, tf / 3 / 833.33, ghz, cyc_per_mfma);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t n = 8 * 4 * IMG / 16;      // 512 KB: the ring's 8 source stages
    std::vector<_Float16> h(n * 8);
    srand(7);
    for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    f16x8* src;
    float* out;
    long long* clk;
    CHECK(hipMalloc(&src, n * sizeof(f16x8)));
    CHECK(hipMalloc(&out, (size_t)cus * 512 * sizeof(float)));
    CHECK(hipMalloc(&clk, (size_t)cus * 2 * sizeof(long long)));
    CHECK(hipMemcpy(src, h.data(), n * sizeof(f16x8), hipMemcpyHostToDevice));
    printf("%d CUs, %d k-steps of 32 per launch, one 256x256 tile per workgroup\n", cus, iters);
    run<8, 0>(src, out, clk, cus, iters, "8 waves 64x128 (product layout)");
    run<4, 0>(src, out, clk, cus, iters, "4 waves 128x128, reads up front");
    run<4, 1>(src, out, clk, cus, iters, "4 waves 128x128, quarter-interleaved reads");
    run<8, 2>(src, out, clk, cus, iters, "8 waves 64x128 + barrier per k-step");
    run<8, 3>(src, out, clk, cus, iters, "8 waves 64x128 + 2-stage LDS-DMA ring");
    run<8, 4>(src, out, clk, cus, iters, "8 waves 64x128 + ring, DMA among the MFMAs");
    run<8, 5>(src, out, clk, cus, iters, "8 waves 64x128 + ring moving half the bytes");
    run<8, 0>(src, out, clk, cus, iters, "8 waves 64x128 (product layout, again)");
    CHECK(hipFree(src));
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
    return 0;
}
