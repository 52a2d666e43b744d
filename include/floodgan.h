/*
 * floodgan.h -- C-ABI of the MI355X-native PairedAttention GAN training-step kernels.
 *
 * The reference (Natasha-R/Flood-Prediction-GAN) has no native code and no FFI: its hot path
 * is PyTorch modules (models/model_architectures.py:305-441) driven by Model.train_paired
 * (models/model.py:598-658), whose arithmetic runs in ATen's conv / instance_norm / pad /
 * softmax / tanh / mse / l1 / Adam kernels.  This library replaces exactly those ATen calls.
 * Each entry point below names the reference operation it replaces.  All pointers are HIP
 * device pointers to fp32 data (doubles where stated), sizes are in elements, every call is
 * asynchronous on `stream` and returns 0 on success or a non-zero error code; the message of
 * the last failure on the calling thread is returned by fg_last_error().  No torch types
 * appear here: the Python host layer (floodgan/_lib.py) binds these with ctypes.
 *
 * Activation tensors are NHWC fp32 with an optional spatial border ("pad"): image n, interior
 * pixel (y, x), channel c lives at ptr[((n*(h+2*pad) + y+pad)*(w+2*pad) + x+pad)*c_alloc + c].
 */
#ifndef FLOODGAN_H
#define FLOODGAN_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------- */
/* common types                                                                              */
/* ---------------------------------------------------------------------------------------- */

enum { FG_PAD_ZERO = 0, FG_PAD_REFLECT = 1 };
enum { FG_ACT_NONE = 0, FG_ACT_RELU = 1, FG_ACT_LRELU = 2 };   /* LeakyReLU slope 0.2 */
enum { FG_ERR_INVALID = -1 };
/* An "absmax slot" (f16x3 operand scales) is FG_AMAX_SHARDS floats whose maximum bounds the
 * operand's |values|; writers raise one shard each (blockIdx % FG_AMAX_SHARDS) to avoid a
 * single-address atomic hot spot.  Slots are initialised to 0 by the caller. */
enum { FG_AMAX_SHARDS = 64 };
/* Convolution arithmetic, per kernel family (bit mask; at most one bit per family): fp32 MFMA
 * (v_mfma_f32_32x32x2_f32); split-bf16 "bf16x6" (each fp32 operand = 3 bf16 pieces, the 6
 * exact bf16 products of order >= 2^-16 accumulated in fp32); or split-fp16 "f16x3" (each
 * operand scaled by a power of two from its absolute maximum and split into 2 fp16 pieces, the
 * 3 exact products of order >= 2^-11 accumulated in fp32) -- for the forward/input-gradient
 * kernel and the weight-gradient kernel independently. */
enum {
    FG_MATH_FP32 = 0,
    FG_MATH_FWD_X6 = 1,
    FG_MATH_WGRAD_X6 = 2,
    FG_MATH_BF16X6 = 3,
    FG_MATH_FWD_F16X3 = 4,
    FG_MATH_WGRAD_F16X3 = 8,
    FG_MATH_F16X3 = 12
};

/* An NHWC view: interior h x w, border `pad` on every side, c_alloc channels per pixel. */
typedef struct fg_view {
    float* ptr;
    int n, h, w, c_alloc, pad;
} fg_view;

/* A strided 4-D view (any memory format), element (n,c,y,x) at ptr[n*sn + c*sc + y*sy + x*sx]. */
typedef struct fg_sview {
    const float* ptr;
    long long sn, sc, sy, sx;
} fg_sview;

/* The same strided 4-D view, writable (gradient outputs in the caller's memory format). */
typedef struct fg_wview {
    float* ptr;
    long long sn, sc, sy, sx;
} fg_wview;

/*
 * Implicit-GEMM convolution problem (forward conv, stride-1 dgrad, and one phase of a
 * stride-2 transposed conv / stride-2 dgrad).  Rows m = (img, a, b) of an m_img x m_a x m_b
 * grid; columns n < n_out; reduction k = (r, j), r < kh, j < jp (j >= j_valid reads zero):
 *     y[row_y(m) + n*syc] (+)= act( sum_k x[row_x(m) + r*sxr + j] * w[n*ldw + r*jp + j] + bias[n] )
 * with row_x(m) = img*sxn + a*sxa + b*sxb and row_y(m) = img*syn + a*sya + b*syb.
 * Replaces ATen convolution / conv_transpose forward and convolution_backward's input
 * gradient for models/model_architectures.py:312-334 (generator) and :424-438 (discriminator).
 */
typedef struct fg_conv_problem {
    const float* x;
    const float* w;
    const float* bias;
    float* y;
    long long sxn, sxa, sxb, sxr;
    long long syn, sya, syb, syc;
    int m_img, m_a, m_b;
    int kh, j_valid, jp;
    int n_out, ldw;
    int act, accumulate;
    int w_split;          /* 0: w is fp32 [n][ldw] (fg_pack_weight); 1: w is the pre-split bf16 layout
                             of fg_pack_weight_split (bf16x6 math); 2: the pre-split fp16 layout of
                             fg_pack_weight_f16 (f16x3 math)                                         */
    const float* x_absmax;   /* f16x3: absmax slot bounding |x| over every element the gather reads */
    const float* w_absmax;   /* f16x3: absmax slot bounding |w| (the one fg_pack_weight_f16 used)  */
    int jc;               /* channels per pixel of the j run (j = s*jc + ch), or 0 if unknown: lets the
                             pipelined kernel walk the taps of one channel chunk back to back (the
                             gathered input rows are re-read while still in L2)                  */
    float* in_stats;      /* optional: InstanceNorm statistics partials of the output, computed in the
                             pipelined kernel's epilogue (see fg_conv_stats_ok): for every block of 32
                             consecutive rows rb = m / 32 and column n < n_out, (mean, M2) of the 32
                             stored values at in_stats[(rb * n_out + n) * 2] -- combined per image by
                             fg_in_stats_partials                                                   */
    int x_presplit;       /* 1: x holds the PRE-SPLIT f16x3 format (FG_PRESPLIT below) written by
                             fg_in_apply_presplit / fg_in_bwd_presplit, whose scale is the pow2 scale
                             of x_absmax; the pipelined kernel reads its fragments as they stand (no
                             split).  Only the pipelined f16x3 kernel takes such problems.          */
    /* Merged sub-pixel phases ("quad" form, round 5) of a stride-2 transposed conv / stride-2 input gradient with
     * a 3-tap kernel (models/model_architectures.py:184, :190 ConvTranspose2d(128, 64, 3, 2, 1, 1) and the
     * input gradient of :172 Conv2d(64, 128, 3, 2, 1)): ONE problem whose rows m = (img, a, b) are the input
     * pixels and whose k runs over their 2 x 2 neighbourhood (kh = 2, j = 2 pixels x jc), so each input pixel
     * is gathered once for all four output phases.  q_n > 0: the columns come in n_out / q_n <= 4 groups of
     * q_n; column n = q*q_n + o is channel o of output pixel row_y(m) + q_yoff[q] (bias[o]); bit q*4 + seg of
     * q_mask says whether group q reads k segment seg = r * (jp / jc) + j / jc (the packed weights of a
     * segment a group does not read are zero, and the kernel skips their MFMAs).  in_stats: group q's partials
     * at in_stats + q * q_soff, laid out [rb][q_n][2] (fg_in_stats_partials with nprob = n_out / q_n).
     * Only the pipelined f16x3 kernel on pre-split operands takes such problems (q_n = 64, n_out = 256). */
    int q_n;
    int q_mask;
    long long q_yoff[4];
    long long q_soff;
} fg_conv_problem;

/*
 * FG_PRESPLIT: an NHWC fp32-sized buffer whose every 8-channel group of a pixel holds, in its 32 bytes,
 * the fp16 pieces h[0..7] then l[0..7] of v*s = h + l (h = fp16(v*s), l = fp16(v*s - h)) for the group's
 * 8 channels, s = 2^(14-e) the power-of-two scale of the tensor's scale slot (max < 2^e): the operand the
 * f16x3 kernels would otherwise split on the fly, produced once by the norm pass that writes it.
 * Channel counts are multiples of 8.
 */

/*
 * Weight-gradient problem: out[split][a][k] = sum_{m in split} p[row_p(m) + a] * x[row_x(m) + koff(k)]
 * with k = r*j_valid + j, koff = r*sxr + j, a < n_a.  Partial slabs are summed by
 * fg_wgrad_reduce.  Replaces convolution_backward's weight gradient.
 */
typedef struct fg_wgrad_problem {
    const float* p;
    const float* x;
    float* out;
    long long spn, spa, spb;
    long long sxn, sxa, sxb, sxr;
    int m_img, m_a, m_b;
    int n_a, kh, j_valid;
    int splits, m_chunk;
    const float* p_absmax;   /* f16x3: absmax slots bounding |p|, |x| over the elements read */
    const float* x_absmax;
    int p_presplit, x_presplit;   /* 1: p / x in the FG_PRESPLIT format (scale = pow2 of its absmax slot;
                                     pipelined f16x3 weight-gradient kernel only)                     */
} fg_wgrad_problem;

/* Maps packed-K coordinates to PyTorch weight coordinates (see fg_pack_weight). */
typedef struct fg_weight_map {
    int n_out;            /* packed rows                                                    */
    int kh, kw, c;        /* packed K = kh * jp, j = s*c + ch, j_valid = kw*c                */
    int c_valid;          /* channels ch >= c_valid are zero                                */
    int jp;               /* padded j extent (multiple of 16) -- pack only                  */
    int dim0_is_n;        /* 1: w[n][ch][r][s] ; 0: w[ch][n][r][s]                          */
    int d0, d1, KH, KW;   /* PyTorch weight shape                                           */
    int n_base;           /* packed row n reads PyTorch index n + n_base                    */
    int rtab[8];          /* kernel-row index per packed r                                  */
    int stab[8];          /* kernel-col index per packed s                                  */
    int q_n;              /* 0, or: packed row n is channel n % q_n (+ n_base) of group q = n / q_n, whose
                             taps are rtab[q*kh + r] / stab[q*kw + s] (kh, kw <= 2); a negative tap index
                             packs zeros (the quad form of fg_conv_problem)                           */
} fg_weight_map;

/* ---------------------------------------------------------------------------------------- */
/* library                                                                                   */
/* ---------------------------------------------------------------------------------------- */
const char* fg_last_error(void);
/* Name of the kernel family this thread's most recent fg_* call launched (e.g. "stem_wgrad", "conv_wgrad_f3"):
 * lets tests assert which kernel a dispatch chose. */
const char* fg_last_launch(void);
int fg_version(void);
int fg_device_ok(void);   /* 0 if a gfx950 device is current, else an error code */
/* Timing events (bench.py's live per-kernel timing).  mode 0 = hipEventDefault (system-scope release, as
 * torch.cuda.Event), 1 = hipEventReleaseToDevice, 2 = hipEventDisableSystemFence (no L2 writeback / invalidate
 * at the record).  fg_timing_event_elapsed waits for `end`. */
int fg_timing_event_create(int mode, void** ev);
int fg_timing_event_record(void* ev, hipStream_t stream);
int fg_timing_event_elapsed(void* start, void* end, float* ms);
int fg_timing_event_destroy(void* ev);
/* Arm the calling thread's next convolution kernel launch (the one conv kernel an fg_conv_fwd / fg_conv_wgrad
 * call dispatches; not the pack / absmax / reduce helpers) with start / stop events attached to the dispatch
 * itself (hipExtLaunchKernel: no marker packet in the stream).  fg_timing_disarm clears the arm and returns 1
 * if no launch consumed it. */
int fg_timing_arm(void* start, void* stop);
int fg_timing_disarm(void);

/* ---------------------------------------------------------------------------------------- */
/* convolution engine (fp32 MFMA v_mfma_f32_32x32x2_f32)                                     */
/* ---------------------------------------------------------------------------------------- */
/* Up to 4 problems in one launch (the four output phases of a stride-2 transposed conv). */
int fg_conv_fwd(const fg_conv_problem* probs, int nprob, hipStream_t stream);

/* 1 if fg_conv_fwd would run these problems on the pipelined f16x3 kernel with in_stats partials
 * (f16x3 math, pre-split weights, N > 32, rows per image a multiple of 32, no activation, no
 * accumulate); fg_conv_fwd fails on problems with in_stats that it cannot honour. */
int fg_conv_stats_ok(const fg_conv_problem* probs, int nprob);

/* Select the convolution arithmetic (FG_MATH_*) for subsequent launches (process-wide). */
int fg_set_conv_math(int mode);
int fg_get_conv_math(void);

/* Tuning hook: force one split-math forward tile configuration (0..11, see conv_gemm.hip), or -1 for
 * the automatic choice by output-channel count (the default). */
int fg_set_fwd_tile(int cfg);
/* Same for the split-math weight-gradient kernels (0..5). */
int fg_set_wgrad_tile(int cfg);
/* Tuning hook of the LDS-DMA pipelined f16x3 forward kernel (conv_f3.hip, used for N > 64 when
 * the operands allow): -1 automatic (default), -2 never use it, 0..12 force a tile config. */
int fg_set_f3_tile(int cfg);
/* Tuning hook, k-walk order of the pipelined forward kernel: bit 0 = odd M tiles walk the kernel
 * rows backwards (L2 sharing between neighbouring tiles); bit 1 = channel-chunk-outer walk (the
 * taps of one 32-channel chunk back to back, needs fg_conv_problem.jc); bit 2 = static priority
 * for the second half of the waves; bit 3 = at a tile boundary the freed LDS ring slot is refilled
 * before the epilogue's stores (stage schedules 3-5), so the stores drain under two stages; bit 4 = bit 0's
 * parity taken from 512-row blocks of output rows instead of from tiles (a row's k order then does not depend
 * on the tile height, so a sample's values do not depend on its batch size).  Default 31. */
int fg_set_f3_order(int alt);
/* Tuning hook: per-stage instruction order of the pipelined forward kernel: 0 = split all of A,
 * then the products; 1 = A reads ahead of the DMA issue, h-half products first; 2 = as 1 with
 * double-buffered B fragment groups; 3 = as 1 with the next stage's DMA pieces spread between
 * the MFMA groups; -1 (default) = the tuned choice per tile config. */
int fg_set_f3_sched(int sched);
/* Tuning hook: 1 (default) = the pipelined forward kernel runs one resident wave of workgroups that
 * loop over the tiles (the next tile's first k-stages stream in behind the current tile's last);
 * 0 = one workgroup per tile; n >= 2 = at most n resident workgroups (test hook: every workgroup then
 * streams many tiles back to back even at small problem sizes). */
int fg_set_f3_persistent(int on);
/* A/B hook: 1 (default) = a pipelined-kernel launch that would leave at least half the CUs without a tile
 * runs on narrower / shorter tiles (conv_f3.hip auto_cfg); 0 = the tile chosen by output channels only. */
int fg_set_f3_fill(int on);
/* A/B hook: the tile of the pipelined kernel for pre-split (FG_PRESPLIT) operands with N > 128 that fill the
 * chip: 4 = 256x256 as 8 waves of 32x256, 5 (default) = 8 waves of 64x128. */
int fg_set_f3_ps_wide(int cfg);
/* A/B hook: 1 (default) = pre-split operands with 64 < N <= 128 that fill the chip run on the 512x128 tile of
 * 8 waves of 64x128 (config 12); 0 = the 256x128 tiles (configs 11 / 6). */
int fg_set_f3_ps_tall(int on);
/* A/B hook: 1 (default) = a pipelined-kernel launch of problems with equal tile counts (the four phases of a
 * transposed conv or of a stride-2 input gradient) interleaves their tiles (tile t -> problem t % count), so
 * the phases read each input row at the same time; 0 = problem after problem. */
int fg_set_f3_interleave(int on);
/* A/B hook of the InstanceNorm passes (instnorm.hip): 1 (default) = the apply / backward-apply passes one
 * padded row per workgroup and the backward statistics with four pixels' loads in flight per thread
 * (bit-identical results); 0 = the grid-stride forms. */
int fg_set_in_rows(int on);
/* A/B hook of the pipelined f16x3 weight-gradient kernel (conv_wgrad_f3.hip, n_a >= 128): 0 off,
 * 1 = staging as one burst per stage, 3 = staging slots interleaved with the MFMA groups,
 * 2 (default) = the measured choice per tile (interleaved for 128-row tiles). */
int fg_set_wgrad_f3(int on);

/* Weight gradient into partial slabs (see fg_wgrad_problem). */
int fg_conv_wgrad(const fg_wgrad_problem* prob, hipStream_t stream);

/* Sum `splits` slabs [split][n_a][kh*kw*c] and scatter into the PyTorch-layout gradient
 * dw (shape map->d0,d1,KH,KW) through `map` (dim0 = a); accumulate != 0 adds into dw. */
int fg_wgrad_reduce(const float* slabs, int splits, const fg_weight_map* map, float* dw,
                    int accumulate, hipStream_t stream);

/* Repack a PyTorch conv / conv-transpose weight into the engine's [n][kh*jp] layout. */
int fg_pack_weight(const float* w, const fg_weight_map* map, float* wp, hipStream_t stream);

/* Same repack, pre-split for the bf16x6 forward kernels: for packed row n and k-slot q (8
 * consecutive k of [0, kh*jp)), wps[(n*(kh*jp/8) + q)*24 + piece*8 + e] (piece 0,1,2 = h,m,l,
 * bf16 bit patterns) with w = h + m + l exactly.  Size n_out*kh*jp*3 bf16.  Conv problems that
 * read it set w_split = 1. */
int fg_pack_weight_split(const float* w, const fg_weight_map* map, void* wps, hipStream_t stream);

/* Pre-split for the f16x3 forward kernels: w * s (s = 2^(14 - e), max(w_absmax slot) < 2^e) split into
 * fp16 pieces h, l at wps[(n*(kh*jp/8) + q)*16 + piece*8 + e] (fp16 bit patterns).  Size
 * n_out*kh*jp*2 fp16.  Conv problems that read it set w_split = 2 and w_absmax. */
int fg_pack_weight_f16(const float* w, const fg_weight_map* map, const float* w_absmax, void* wps,
                       hipStream_t stream);

/* One weight repack of a batch (fg_pack_weight_f16_batch): w through map into the f16x3 layout at dst,
 * scaled by the w_absmax slot -- the arguments of one fg_pack_weight_f16 call. */
typedef struct fg_pack_job {
    const float* w;
    const float* w_absmax;
    void* dst;
    fg_weight_map map;
} fg_pack_job;

/* Up to FG_PACK_BATCH_MAX fg_pack_weight_f16 repacks in one launch (the pack cache refreshing every
 * packed layout of the parameters an optimizer step just updated). */
#define FG_PACK_BATCH_MAX 24
int fg_pack_weight_f16_batch(const fg_pack_job* jobs, int njobs, hipStream_t stream);

/* Pre-split operand for fg_conv_win: the npix NHWC pixels of c (32 or 64) fp32 channels at src,
 * scaled by the power of two of the absmax slot (as fg_pack_weight_f16) and split into fp16
 * pieces h, l; pixel p (padded-row column x = p % wp) becomes 2c fp16 whose 16-byte chunk k
 * ([h | l] order) is stored at chunk k ^ swizzle(x).  Size npix*2c fp16. */
int fg_split_pixels(const float* src, long long npix, int c, int wp, const float* amax, void* dst,
                    hipStream_t stream);

/* Row-strip f16x3 convolution (stride 1, 7x7, C = sxb in {32, 64}, n_out <= 32 / 64, output rows
 * of >= 256 pixels): the same problem as fg_conv_fwd, with the input read from x_split (the
 * fg_split_pixels copy of the buffer x points into; x_pix0 = pixel index of x's origin in it, at
 * the start of a padded row).  Replaces the 7x7 content-head conv (models/model_architectures.py:328)
 * and its input gradient. */
int fg_conv_win(const fg_conv_problem* prob, const void* x_split, long long x_pix0, hipStream_t stream);

/* Row-strip f16x3 weight gradient of the 7x7 64 -> 32(27) content-head conv (the fg_wgrad_problem of
 * its generic form: p = 32-channel gradient, x = 64-channel input gather, output rows of a multiple of
 * 32 px), reading both operands from their fg_split_pixels copies: p_split (gradient; p_pix0 = pixel
 * index of p's origin, p_col0 = its padded column, wp_p pixels per padded row) and x_split (input;
 * x_pix0 at a padded-row start, wp_x).  Writes prob->splits slabs for fg_wgrad_reduce.  Replaces the
 * content-head weight gradient of convolution_backward (models/model_architectures.py:328). */
int fg_conv_wgrad_win(const fg_wgrad_problem* prob, const void* p_split, long long p_pix0, int p_col0,
                      int wp_p, const void* x_split, long long x_pix0, int wp_x, hipStream_t stream);

/* The attention head's 1x1 conv (Conv2d(64, n_out <= 16, 1), models/model_architectures.py:334) in fp32
 * FMA over LDS-staged 64-pixel tiles: y (4 <= c_alloc <= 16; channels >= n_out written as 0) = w x + b over
 * x's interior (c_alloc 64); replaces fg_conv_fwd on that layer (a matrix-vector product per pixel). */
int fg_conv1x1_fwd(fg_view x, const float* w, const float* bias, int n_out, fg_view y, hipStream_t stream);
/* Its input gradient: gx (c_alloc 64) = w^T gy over the interior. */
int fg_conv1x1_dgrad(fg_view gy, const float* w, int n_out, fg_view gx, hipStream_t stream);
/* Its weight and bias gradients (PyTorch layouts, written or, with accumulate, raised; db optional):
 * per-block partial sums in `work` (fg_conv1x1_wgrad_workspace_floats(n_out) floats), reduced in fp64
 * in a fixed order. */
long long fg_conv1x1_wgrad_workspace_floats(int n_out);
int fg_conv1x1_wgrad(fg_view gy, fg_view x, int n_out, float* dw, float* db, int accumulate, float* work,
                     hipStream_t stream);

/* The discriminator's last conv (Conv2d(512, 1, 4, 1, 1), models/model_architectures.py:437) in fp32:
 * y[n][oy][ox] = bias[0] + sum_{c,r,s} x(n, oy+r, ox+s, c) * w[c*16 + r*4 + s] over the 1-padded NHWC
 * input x (nimg images of hp x wp padded pixels, c = 512), y NCHW [nimg, 1, ho, wo], ho = hp-3. */
int fg_conv_n1_fwd(const float* x, int nimg, int hp, int wp, int c, const float* w, const float* bias,
                   float* y, int ho, int wo, hipStream_t stream);
/* Its weight gradient into fg_conv_n1_wgrad_blocks(nimg, hp, rows_per_block) slabs of 16*c floats
 * (the fg_conv_wgrad slab layout for n_a = 1; sum them with fg_wgrad_reduce).  gp: the output
 * gradient [nimg][ghp][gwp] with a zero border of 3 (ghp = ho + 6). */
int fg_conv_n1_wgrad_blocks(int nimg, int hp, int rows_per_block);
int fg_conv_n1_wgrad(const float* x, int nimg, int hp, int wp, int c, const float* gp, int ghp, int gwp,
                     int rows_per_block, float* slabs, hipStream_t stream);

/* The PatchGAN model.0 input gradient (Conv2d(ctot, 64, 4, 2, 1), models/model_architectures.py:424) for input
 * channels c0 .. c0 + cn - 1 only (cn <= 4: the G step's dL/d(fake), models/model.py:640-646), in exact fp32:
 * g = dL/d(model.0 output) as an NHWC view of 64 channels at H/2 x W/2 with a zero border >= 1, w = model.0.weight
 * [64][ctot][4][4]; y = NCHW [N][yc][H][W] whose channels 0 .. cn - 1 receive it (accumulate: added).  Replaces the
 * restricted 4-phase transposed conv the engine ran (ops._dgrad_s2 with n_base / n_out). */
int fg_d0_input_grad(fg_view g, const float* w, int ctot, int c0, int cn, float* y, int yc, int H, int W,
                     int accumulate, hipStream_t stream);

/* Raise the absmax slot `out` (FG_AMAX_SHARDS floats, initialised by the caller) to bound
 * max |x[i]| over n contiguous floats (bitwise max of |x|; NaN-propagating).  The operand-
 * scale source of the f16x3 math. */
int fg_absmax(const float* x, long long n, float* out, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* layout / padding                                                                          */
/* ---------------------------------------------------------------------------------------- */
/* dst(img0+n, y, x, ch) = ch < ca ? a(n,ch,y,x) : ch < ca+cb ? b(n,ch-ca,y,x) : 0, for the full
 * padded extent of dst (border filled by `pad_mode`).  Replaces F.pad(reflect) at
 * models/model_architectures.py:341 and torch.cat at models/model.py:616-617.  absmax (optional absmax slot,
 * initialised by the caller; several packs into one dst may share it) is raised to max |written values|. */
int fg_pack_input(fg_sview a, int ca, fg_sview b, int cb, fg_view dst, int img0, int nimg,
                  int pad_mode, float* absmax, hipStream_t stream);

/* Fill the border of dst with zeros (interior untouched). */
int fg_zero_border(fg_view dst, hipStream_t stream);

/* dst = fold_reflect(gpad) (+ add): the adjoint of reflect padding (reflection_pad2d_backward)
 * plus an optional residual-gradient add (models/model_architectures.py:418 `input + x`). */
int fg_fold_add(fg_view gpad, int fold_pad, fg_view add, fg_view dst, hipStream_t stream);

/* dst(n, ch, y, x) (+)= fold_reflect(gpad)(n, y, x, ch) for ch < c: the adjoint of the
 * generator's `F.pad(input, 3, reflect)` (models/model_architectures.py:342) written into
 * the caller's strided NCHW input-gradient tensor.  gpad's interior is (h + 2 fold_pad) x
 * (w + 2 fold_pad) where h x w is dst's spatial size; channels ch < acc_channels are
 * accumulated onto dst (the tail's direct x[:, :3] term), the rest overwritten. */
int fg_unfold_nchw(fg_view gpad, int fold_pad, int c, fg_wview dst, int h, int w, int acc_channels,
                   hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* instance norm (nn.InstanceNorm2d, affine=False, eps 1e-5) fused with activation           */
/* ---------------------------------------------------------------------------------------- */
/* Per-(n,c) mean and 1/sqrt(var+eps) from a conv's epilogue partials (fg_conv_problem.in_stats):
 * `partials` holds nprob consecutive problems' [rows / 32][c][2] blocks, every problem with n_img images
 * of rb_per_img 32-row blocks each (the 4 phases of a transposed conv: one image's statistics span all
 * four).  Replaces fg_in_stats for outputs of the pipelined kernel. */
int fg_in_stats_partials(const float* partials, int nprob, int n_img, int rb_per_img, int c, float eps, float* mean,
                         float* rstd, double* work, hipStream_t stream);
/* work doubles fg_in_stats_partials needs */
long long fg_in_partials_workspace_doubles(int n_img, int c);

/* Per-(n,c) mean and 1/sqrt(var+eps) of src's interior; work >= fg_in_workspace_doubles(). */
long long fg_in_workspace_doubles(int n, int c);
int fg_in_stats(fg_view src, float eps, float* mean, float* rstd, double* work,
                hipStream_t stream);

/* dst = act((src - mean) * rstd) (+ residual), written over dst's full padded extent with
 * pad_mode (reflect or zero border).  Replaces instance_norm + relu/leaky_relu + F.pad
 * (+ the residual add of PairedAttentionBlock).  absmax (optional absmax slot, initialised by
 * the caller) is raised to bound |dst| -- the f16x3 scale source of the convs reading dst. */
int fg_in_apply(fg_view src, const float* mean, const float* rstd, int act, fg_view residual,
                fg_view dst, int pad_mode, float* absmax, hipStream_t stream);

/* Backward of fg_in_apply.  g is read from gsrc's interior, or folded through reflect
 * padding of width fold_pad when fold_pad > 0 (gsrc then holds the gradient of the padded
 * tensor); optional gadd (compact) is added.  dst receives dL/dsrc (border zeroed);
 * bias_grad (optional, [c]) receives (or, with bias_accumulate, is raised by) sum over n,y,x
 * of dst = grad of the conv bias that feeds this norm.  gsum (optional, NULL ptr = none): receives
 * g = fold(gsrc) + gadd itself in its interior (the gradient of a PairedAttentionBlock's input, which the
 * residual path needs again: models/model_architectures.py:418), written by the statistics pass that reads
 * it anyway -- the separate reflect-fold + residual-add pass (fg_fold_add) is not needed. */
int fg_in_bwd(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean,
              const float* rstd, int act, fg_view dst, float* bias_grad, int bias_accumulate, fg_view gsum,
              double* work, float* absmax, hipStream_t stream);

/* fg_in_apply without residual whose dst is written in the FG_PRESPLIT format (C % 8 == 0, 32-B aligned):
 * the f16x3 pieces of act(xhat) at the static scale of |xhat| <= sqrt(HW - 1) (Samuelson), which the call
 * publishes in scale_slot (a zeroed absmax slot) -- the slot the consuming conv / weight gradient reads as
 * x_absmax.  Saves the consumer's on-the-fly split (a resblock's conv1 -> conv2 hop). */
int fg_in_apply_presplit(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                         float* scale_slot, hipStream_t stream);
/* The same pass writing dst (C = 32 or 64) in the fg_split_pixels layout -- per pixel the fp16 pieces [h(C) | l(C)]
 * of the scaled values, 16-B chunk k at k ^ swizzle(padded column) -- the operand of fg_conv_win / fg_conv_wgrad_win
 * (no fp32 copy and no separate fg_split_pixels pass): the content head's input relu(IN(deconv2_content)),
 * models/model_architectures.py:351-353.  Scale bound and slot as fg_in_apply_presplit. */
int fg_in_apply_splitpix(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                         float* scale_slot, hipStream_t stream);

/* fg_in_apply writing dst in fp32 (absmax raised as there) AND a FG_PRESPLIT copy into ps_dst (same geometry, 32-B
 * aligned) at the scale of the bound sqrt(HW - 1) + max|residual| (residual_absmax: the residual's absmax slot,
 * required with a residual), published in ps_slot (a zeroed absmax slot): the block outputs of the resblock chain,
 * whose fp32 values the next residual add needs and whose copy the next conv and its weight gradient read. */
int fg_in_apply_dual(fg_view src, const float* mean, const float* rstd, int act, fg_view residual,
                     const float* residual_absmax, fg_view dst, int pad_mode, float* absmax, float* ps_dst,
                     float* ps_slot, hipStream_t stream);

/* fg_in_bwd whose dst is written in the FG_PRESPLIT format: the statistics pass also takes max |g'| per
 * image, the coefficient pass bounds |dst| per plane by rstd (max|g'| + |mean g'| + sqrt(HW-1) |mean g'xhat|)
 * and publishes the bound in scale_slot (a zeroed absmax slot), the apply pass writes the pieces at its
 * scale (the input of the next input-gradient conv and the weight gradient's gradient operand). */
int fg_in_bwd_presplit(fg_view gsrc, int fold_pad, fg_view gadd, fg_view src, const float* mean,
                       const float* rstd, int act, fg_view dst, float* bias_grad, int bias_accumulate, fg_view gsum,
                       double* work, float* scale_slot, hipStream_t stream);

/* The attention head Conv2d(64, n_out <= 16, 1) (models/model_architectures.py:334, :369) fused into the norm
 * passes of its input (the replaced interfaces: fg_in_apply + fg_conv1x1_fwd, fg_conv1x1_dgrad + fg_in_bwd).
 * fg_in_apply_head: fg_in_apply (no residual; C = 64, dst unpadded) that also writes the logits
 * y[p][o] = b[o] + sum_c w[o][c] dst[p][c] (w [n_out][64], y: a 16-B aligned unpadded view of the same grid,
 * n_out <= c_alloc <= 16; channels n_out.. get 0) -- bit-identical to fg_conv1x1_fwd's.
 * fg_in_bwd_head: fg_in_bwd of the head's input whose incoming gradient is w^T gy, formed from the logits
 * gradient gy (unpadded, n_out <= 12, 12 <= c_alloc <= 16: three 16-B quads are read per pixel) in
 * fg_conv1x1_dgrad's fma order (bit-identical to running it first); scale_slot non-NULL: dst in the FG_PRESPLIT
 * format as fg_in_bwd_presplit (absmax ignored).
 * Round 5: fg_in_apply_head takes a dst with a NULL ptr (its geometry only): the activation is then not written,
 * only the logits.  fg_in_bwd_head with dw non-NULL also forms the head's weight gradient dw[o][c] (+)= sum_p
 * gy[p][o] act(xhat[p][c]) and db[o] (+)= sum_p gy[p][o] (the replaced fg_conv1x1_wgrad; wg_accumulate adds),
 * recomputing the activation from src; wg_work holds fg_in_head_wgrad_workspace_floats(n, h, w, n_out) floats. */
int fg_in_apply_head(fg_view src, const float* mean, const float* rstd, int act, fg_view dst, int pad_mode,
                     float* absmax, const float* w, const float* b, int n_out, fg_view y, hipStream_t stream);
int fg_in_head_wgrad_workspace_floats(int n, int h, int w, int n_out);
int fg_in_bwd_head(fg_view gy, const float* w, int n_out, fg_view src, const float* mean, const float* rstd,
                   int act, fg_view dst, float* bias_grad, int bias_accumulate, double* work, float* absmax,
                   float* scale_slot, float* dw, float* db, int wg_accumulate, float* wg_work, hipStream_t stream);


/* g *= act'(y) in place over the interior (y = saved activation output).  absmax (optional absmax slot,
 * initialised by the caller) is raised to max |g| over the interior -- a bound for the whole buffer when its
 * border is zero. */
int fg_act_bwd(fg_view g, fg_view y, int act, float* absmax, hipStream_t stream);

/* out[c] (+)= sum over n,y,x of src(n,y,x,c) for c < c_valid.  Bias gradients.  `work` holds
 * fg_channel_sum_workspace_doubles(src.c_alloc) doubles. */
int fg_channel_sum(fg_view src, int c_valid, float* out, int accumulate, double* work,
                   hipStream_t stream);
long long fg_channel_sum_workspace_doubles(int c_alloc);

/* ---------------------------------------------------------------------------------------- */
/* generator tail: tanh(27) + softmax(10) + attention composite                              */
/* (models/model_architectures.py:352-399)                                                   */
/* ---------------------------------------------------------------------------------------- */
int fg_tail_fwd(fg_view content_logits, fg_view att_logits, fg_sview x, float* out,
                float* mask, hipStream_t stream);
/* g_out: strided [N,3,H,W].  g_content: dst view (27 used of c_alloc, zero border/channels),
 * g_att: dst view (10 used).  g_x (optional, NULL ptr = skip): channels 0..2 of a strided
 * [N,C,H,W] tensor receive the direct gradient w.r.t. input[:, :3] of the background term
 * `input[:, :3] * attention10` (models/model_architectures.py:393, :251) -- the input
 * gradient that the cycle path (models/model.py:677-706) back-propagates into G.  absmax_content /
 * absmax_att (optional absmax slots, initialised by the caller) are raised to bound |g_content| / |g_att|:
 * the f16x3 scale sources of the convs reading them, with no separate pass.  g_mask (optional, NULL ptr =
 * none): a strided [N,1,H,W] view of dL/d(last_attention_mask), the mask being attention10
 * (models/model_architectures.py:396); it joins attention channel 9's gradient before the softmax backward. */
int fg_tail_bwd(fg_view content_logits, fg_view att_logits, fg_sview x, fg_sview g_out,
                fg_sview g_mask, fg_view g_content, fg_view g_att, fg_wview g_x, float* absmax_content,
                float* absmax_att, hipStream_t stream);

/* CycleGAN generator head (models/model_architectures.py:115-117, conv 7x7 64->3 + nn.Tanh):
 * out (strided [N,c,H,W]) = tanh(logits[..., :c]). */
int fg_tanh_head_fwd(fg_view logits, int c, fg_wview out, hipStream_t stream);
/* g_logits = g_out * (1 - tanh(logits)^2) for channels < c; zero border and zero channels >= c
 * (g_logits feeds the 7x7 input-gradient conv with its full-correlation border). */
int fg_tanh_head_bwd(fg_view logits, int c, fg_sview g_out, fg_view g_logits, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* losses (nn.MSELoss vs a constant target, nn.L1Loss; models/model.py:626-644)             */
/* ---------------------------------------------------------------------------------------- */
/* loss[0] = mean((p - target)^2);  g (optional) = gscale * 2 (p - target) / n */
int fg_mse_const(const float* p, long long n, float target, float gscale, float* loss,
                 float* g, double* work, hipStream_t stream);
/* loss[0] = loss_scale * mean(|a - b|) over [N,C,H,W] strided views (the mean rounded to fp32 first, then
 * scaled in fp32: the reference logs 100 * L1, models/model.py:643-651); g (optional, NCHW contiguous)
 * = gscale * sign(a - b) / n  (or += when accumulate). */
int fg_l1(fg_sview a, fg_sview b, int N, int C, int H, int W, float gscale, float loss_scale, float* loss,
          float* g, int accumulate, double* work, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* Adam (torch.optim.Adam, amsgrad=False, weight_decay=0; models/model.py:121-122)           */
/* ---------------------------------------------------------------------------------------- */
typedef struct fg_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long numel;
    float* absmax;        /* optional absmax slot (FG_AMAX_SHARDS floats, zeroed by the caller):
                             raised to bound |param| after the update -- the f16x3 scale source of
                             the next weight packing, at no extra pass                            */
} fg_adam_tensor;
/* One step for `count` tensors sharing (lr, betas, eps, step). */
int fg_adam_step(const fg_adam_tensor* tensors, int count, double lr, double beta1,
                 double beta2, double eps, long long step, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* batch norm (nn.BatchNorm2d, training mode) -- Pix2Pix U-Net / PatchGAN and the segmentation */
/* U-Net (models/model_architectures.py:9-85, :508-587)             */
/* ---------------------------------------------------------------------------------------- */
/* Images of src split into `groups` equal consecutive batches, each one separate BatchNorm call
 * (statistics over its images x H x W per channel; the running statistics, when given, are
 * updated once per group in group order with torch's momentum rule and unbiased variance).
 * mean / invstd: [groups * C].  num_batches_tracked (optional, the module's int64 buffer) is raised
 * by `groups`.  work >= fg_bn_workspace_doubles(n, c). */
long long fg_bn_workspace_doubles(int n, int c);
int fg_bn_stats(fg_view src, int groups, float eps, float momentum, float* mean, float* invstd,
                float* running_mean, float* running_var, long long* num_batches_tracked, double* work,
                hipStream_t stream);
/* Eval-mode statistics (module.eval()): mean = running_mean, invstd = 1 / sqrt(running_var + eps). */
int fg_bn_eval_stats(int c, const float* running_mean, const float* running_var, float eps, float* mean,
                     float* invstd, hipStream_t stream);
/* y = (x - mean) * invstd * gamma + beta (no normalisation when mean is NULL, no affine when gamma
 * is NULL), then nn.Dropout: y *= keep(n, c, y, x) * drop_scale (drop_scale = 1 / (1 - p)), with keep
 * read from a caller-drawn NCHW 0/1 drop_mask or -- drop_mask NULL, drop_seed != 0 -- decided on the
 * device by a counter-based hash of (drop_seed, NCHW element index) with probability 1 / drop_scale
 * (fg_dropout_mask materialises the same decisions); dst0 = act0(y) and optionally dst1 = act1(y):
 * interiors only; a destination may be a channel slice of a wider buffer (ptr offset, c_alloc = the
 * wider buffer's channels). */
int fg_bn_apply(fg_view src, int groups, const float* mean, const float* invstd, const float* gamma,
                const float* beta, const float* drop_mask, float drop_scale, unsigned long long drop_seed, int act0,
                fg_view dst0, float* absmax0, int act1, fg_view dst1, float* absmax1, hipStream_t stream);
/* Backward of fg_bn_apply: the incoming gradient of the normalised, dropped-out value u is
 * gA * actA'(u) (+ gB * actB'(u) when gB.ptr), times the dropout keep * scale (the same mask or seed as
 * the forward); dst = dL/dx through the batch statistics of each group (identity when mean is NULL);
 * gamma_grad / beta_grad (written, or added to when accumulate) summed over the groups. */
int fg_bn_bwd(fg_view gA, int actA, fg_view gB, int actB, fg_view src, int groups, const float* mean,
              const float* invstd, const float* gamma, const float* beta, const float* drop_mask,
              float drop_scale, unsigned long long drop_seed, fg_view dst, float* gamma_grad, float* beta_grad,
              int accumulate, double* work, float* absmax, hipStream_t stream);
/* The 0/1 keep decisions of fg_bn_apply's hashed dropout for elements 0 .. total-1 (NCHW order of the
 * tensor the dropout applies to) into dst as floats (tests / host inspection). */
int fg_dropout_mask(unsigned long long seed, float keep, long long total, float* dst, hipStream_t stream);
/* torch's CPU Bernoulli stream on the device, bit for bit (replaces the host draws of the reference's
 * nn.Dropout, models/model_architectures.py:52: F.dropout -> empty_like(x).bernoulli_(1 - p) per call):
 * `elements` = sum(sizes) decisions drawn in order into the float 0/1 outputs outs[0..nout) (host array of
 * device pointers, nout <= 4), element e keeping when the low 53 bits of (y(W[first + 2e]) << 32 |
 * y(W[first + 2e + 1])) times 2^-53 are below p -- W the MT19937 word stream whose words 0..623 are `state`
 * (device, the generator's 624 state words), first = 625 - the generator's `left`, y the tempering.
 * jumps: device [njumps][624] words, x^(c * chunk) mod phi for c = 1..njumps (floodgan/data/mt19937_jumps.npz);
 * final_state: the 624 words of the block holding the last word used (the state the draw leaves behind);
 * work: fg_bernoulli_mt_workspace_words(chunks) device words, chunks = (last word - 1) / chunk + 1. */
long long fg_bernoulli_mt_workspace_words(int nchunks);
int fg_bernoulli_mt(const unsigned* state, long long first, long long elements, const unsigned* jumps, int njumps,
                    long long chunk, int nout, float* const* outs, const long long* sizes, double p,
                    unsigned* final_state, unsigned* work, hipStream_t stream);
/* nn.MaxPool2d(2) over NHWC interiors (floor output size). */
int fg_maxpool2(fg_view src, fg_view dst, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* evaluation metrics (models/model.py:363-422, models/group.py:114-221) */
/* ---------------------------------------------------------------------------------------- */
/* torch.clamp((src + 1) * 0.5, 0, 1) of an [n, c, h, w] (strided) generator output into dst (contiguous
 * NCHW, optional) and into buf's interior channels 0..c-1 (NHWC, optional: the segmentation U-Net's input). */
int fg_unit_image(fg_sview src, int n, int c, int h, int w, float* dst, fg_view buf, hipStream_t stream);
/* SSIM of two contiguous NCHW [n, c, h, w] images in [0, 1] (torchmetrics 1.2.0 _ssim_update: gaussian
 * 11x11 window gauss11 (normalised 1-D taps), constants c1 = (0.01 dr)^2, c2 = (0.03 dr)^2; the mean runs
 * over channels and the (h-10) x (w-10) windows inside the image): ssim[i], cs[i] (each optional) = per
 * image means of the SSIM and contrast-sensitivity maps.  work >= fg_ssim_workspace_doubles(). */
long long fg_ssim_workspace_doubles(int n, int c, int h, int w);
int fg_ssim(const float* a, const float* b, int n, int c, int h, int w, const float* gauss11, float c1, float c2,
            double* ssim, double* cs, double* work, hipStream_t stream);
/* F.avg_pool2d(x, 2) over `planes` contiguous h x w planes (floor). */
int fg_avg_pool2(const float* src, int planes, int h, int w, float* dst, hipStream_t stream);
/* MS-SSIM per image: prod_s relu(m_s)^betas[s], m = cs[s * n + i] for s < scales-1, ssim_last[i] last. */
int fg_msssim_combine(int n, int scales, const double* cs, const double* ssim_last, const double* betas,
                      double* out, hipStream_t stream);
/* out[0] = sum (a - b)^2 over `total` floats (PSNR); work >= fg_sq_err_workspace_doubles(). */
long long fg_sq_err_workspace_doubles(void);
int fg_sq_err_sum(const float* a, const float* b, long long total, double* out, double* work, hipStream_t stream);
/* counts[0..3] += true positives, false positives, true negatives, false negatives of the flood masks
 * (sigmoid(logit) > 0.5, channel 0 of each view) of pred vs true segmentation logits. */
int fg_mask_confusion(fg_view pred_logits, fg_view true_logits, unsigned long long* counts, hipStream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* tile data path                                                    */
/* ---------------------------------------------------------------------------------------- */
/* Host-side baseline TIFF decode, replacing tifffile.imread (models/data.py:64-68) for the files
 * tifffile.imsave(..., planarconfig="contig") writes (pre_processing/data_pre_processing.py:377-418):
 * uncompressed chunky strips, either byte order, uint8 / uint16 / float32 / float64 samples.
 * fg_tiff_probe: image size, samples per pixel, sample code (100*SampleFormat + bits).
 * fg_tiff_read: the samples as float32 HWC into HOST memory `dst` (capacity in floats) -- the
 * loader decodes straight into a pinned staging slot.  Both are synchronous host calls. */
int fg_tiff_probe(const char* path, int* height, int* width, int* channels, int* sample_code);
int fg_tiff_read(const char* path, float* dst, long long capacity);

enum { FG_TILE_MAX_CH = 16 };
/* A batch of staged raw tiles -> model tensors: np.fliplr (models/data.py:63-65), topography
 * channel selection, Resize(resize, BICUBIC, antialias=True), quadrant crop and Normalize(0.5, 0.5)
 * (models/utils.py:30-61), over only the crop window of the resized image.  The resize is given as
 * separable tap tables over the RESIZED image's columns / rows (x_idx0[i] = first source index of
 * output index i, x_w[i*x_taps + k] its weights; identity tables when no resize). */
typedef struct fg_tile_batch {
    const float* src;          /* device: n raw tiles, HWC fp32, h_in x w_in x c_src each            */
    long long tile_stride;     /* floats from one raw tile to the next                              */
    int n, h_in, w_in, c_src;
    const int* flip;           /* device, per tile: 1 = mirror columns (np.fliplr); NULL = none      */
    int c_out;
    int chan[FG_TILE_MAX_CH];  /* output channel o <- source channel chan[o]                         */
    const int* crop;           /* device, per tile: (row0, col0) of the window in the resized image;
                                  NULL = (0, 0)                                                      */
    const int* row_lo;         /* device, per tile: first source row the window's row taps read
                                  (required with crop)                                              */
    int rows;                  /* source rows per tile the horizontal pass produces, from row_lo     */
    int out_h, out_w;          /* window size                                                        */
    const int* x_idx0;
    const float* x_w;
    int x_taps;
    const int* y_idx0;
    const float* y_w;
    int y_taps;
    float* tmp;                /* device workspace: n * rows * out_w * c_out floats                  */
    fg_wview dst;              /* output [n, c_out, out_h, out_w], any strides                       */
} fg_tile_batch;
int fg_tile_transform(const fg_tile_batch* batch, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FLOODGAN_H */
