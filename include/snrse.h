/* snrse.h — C-ABI of libsnrse_hip.so, the MI355X (gfx950) kernels of the
 * reverse-diffusion speech-enhancement path of yh-jun/SNR-Aligned_diffSE
 * (ScoreModel.enhance() / PC sampler, sgmse-bbed/sgmse/model.py:702-839).
 *
 * Conventions
 *   - Plain pointers to DEVICE memory, sizes as int, a hipStream_t (NULL = legacy stream);
 *     every launch is stream-ordered and asynchronous, nothing is allocated inside except
 *     where a caller-provided workspace is named.
 *   - Reentrancy: entries without a snrse_ctx argument keep no state.  The four with one
 *     (snrse_conv2d, snrse_gn_stats, snrse_input_conv, snrse_gn_resample) read their switches and
 *     split-K workspace from it and write their read-backs into it, so calls through DISTINCT
 *     contexts may run concurrently from any host threads / streams; give each concurrently issuing
 *     thread or stream its own context.  A NULL context is the process default one (edited by
 *     snrse_set_option / snrse_set_workspace; for single-stream callers).
 *   - Return 0 on success or a hipError_t code (hipErrorInvalidValue = 1 for a bad
 *     argument); snrse_error_string() maps it to text.  The Python host maps non-zero to
 *     RuntimeError, as the reference's TORCH_CHECK does (op/upfirdn2d.cpp:8-19).
 *   - dtype: SNRSE_F32 = 0 (exact fp32 "parity" mode), SNRSE_F16 = 2 (IEEE fp16 storage and MFMA
 *     operands, fp32 accumulation: the 16-bit fast path's default since round 6, whose error against the
 *     reference is ~9x below bf16's), SNRSE_BF16 = 1 (the same kernels on bf16; every entry
 *     that takes SNRSE_BF16 takes SNRSE_F16 too), SNRSE_F32X3 = 4 (snrse_conv2d only: fp32 activations and output, weights
 *     pre-split into bf16 hi / lo halves, three bf16 MFMA products per K-tile -- the fast fp32
 *     parity mode).  Activations are NHWC: [B, F(=H), T(=W), C].
 *   - Complex spectrograms are interleaved complex64 [B, F, T] (= the reference's
 *     [B, 1, F, T] tensors).
 */
#ifndef SNRSE_H_
#define SNRSE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

enum { SNRSE_F32 = 0, SNRSE_BF16 = 1, SNRSE_F16 = 2, SNRSE_F64 = 3, SNRSE_F32X3 = 4 };

int snrse_abi_version(void); /* 2: snrse_ctx arguments */
/* sha256 (hex) of the sources the library was compiled from: csrc/*.hip, *.cpp, *.h and the build
 * script (snrse/build.py source_hash()), compiled in; "unknown" for a build made without it. */
const char* snrse_build_id(void);
const char* snrse_error_string(int code);
int snrse_device_name(char* buf, int len);

/* Caller-owned launch context: tuning switches (the names of snrse_set_option), the split-K
 * workspace and the read-backs of the latest launch through it (the names of snrse_get_option).
 * Host memory only; create copies the process default's switches, with no workspace. */
typedef struct snrse_ctx snrse_ctx;
snrse_ctx* snrse_ctx_create(void);
void snrse_ctx_destroy(snrse_ctx* ctx);
int snrse_ctx_set_workspace(snrse_ctx* ctx, void* ptr, size_t bytes);
int snrse_ctx_set_option(snrse_ctx* ctx, const char* name, int value);
int snrse_ctx_get_option(const snrse_ctx* ctx, const char* name, int* value);
/* Diagnostic timing (bench.py's roofline probe): from now on every snrse_conv2d call through ctx is
 * bracketed by a pair of HIP events (created here, without the system-scope fence), up to `capacity`
 * calls; capacity 0 stops and frees them.  snrse_ctx_probe_read waits for the recorded calls and writes,
 * in call order, each call's device time in ms and the kernel generation that ran ("last_kernel"). */
int snrse_ctx_probe_begin(snrse_ctx* ctx, int capacity);
int snrse_ctx_probe_read(snrse_ctx* ctx, float* ms, int* kernel, int max, int* n);

/* Generic FIR resampling on [major, in_h, in_w, minor] — replaces the reference's only
 * native op binding, upfirdn2d(input, kernel, up_x, up_y, down_x, down_y, pad_x0, pad_x1,
 * pad_y0, pad_y1) (op/upfirdn2d.cpp:12-23, op/upfirdn2d_kernel.cu:209-369, semantics of
 * upfirdn2d_native op/upfirdn2d.py:159-200).  `kernel` is [kh, kw] f32 on the device;
 * `out` is caller-allocated [major, out_h, out_w, minor] with
 * out_h = (in_h*up_y + pad_y0 + pad_y1 - kh)/down_y + 1 (out_w likewise).
 * dtype: SNRSE_F32 / SNRSE_F16 / SNRSE_F64, the reference's float / half / double dispatch
 * (upfirdn2d_kernel.cu:311), plus SNRSE_BF16; f64 accumulates in f64, the others in f32. */
int snrse_upfirdn2d(const void* in, void* out, const float* kernel, int major, int in_h, int in_w,
                    int minor, int kh, int kw, int up_x, int up_y, int down_x, int down_y,
                    int pad_x0, int pad_x1, int pad_y0, int pad_y1, int dtype, hipStream_t stream);

/* Implicit-GEMM convolution (3x3 pad 1 or 1x1), stride 1, NHWC, on MFMA.
 * Replaces ddpm_conv3x3 / ddpm_conv1x1 / NIN (ncsnpp_utils/layers.py:100-124, 546-555).
 *   input channels = concat(src0 [.., C0], src1 [.., C1]) (torch.cat, ncsnpp.py:337)
 *   wgt    [Npad][ksize*ksize*(C0+C1)] packed (Cout, ky, kx, Cin), dtype; Npad = Cout
 *          rounded up to 128 (Cout >= 64) or 16 (Cout <= 16, zero rows)
 *   sc_src/sc_src1 (optional): 1x1 shortcut input(s) appended as extra K; sc_wgt [Npad][Csc+Csc1]
 *   out[m][n] = ((acc + bias[n] + temb[b][n] + res[m][n]) * out_scale)
 *               + (comb_src ? comb_src[m][0:4] . comb_w[n][0:4] + comb_b[n] : 0)
 *   out_f32: write float output (bf16 mode pyramid heads); res then is float too.
 *   stats (optional): per-channel (sum, sumsq) of out, [B][SNRSE_STAT_SLOTS][Cout][2] double
 *          (atomics spread over the slots; consumers fold them), for the next GroupNorm
 *          (zeroed by the call unless the context's "stats_zeroed" switch is set).
 *   gn_scale/gn_shift (optional, [B][C0+C1] f32, from snrse_gn_scale_shift): the main input
 *          is consumed as SiLU(x*scale+shift) (gn_act=1) or x*scale+shift (gn_act=0), i.e. the
 *          ResBlock's GroupNorm+SiLU fused into the GEMM's halo load (bf16, 3x3, H%4==0,
 *          W%64==0, and the pyramid heads Cout<=16 with f32 output; otherwise
 *          hipErrorInvalidValue).
 *   dtype SNRSE_F32X3: src/res/out fp32; wgt [Npad][2*ksize*ksize*(C0+C1)] and sc_wgt [Npad][2*(Csc+Csc1)]
 *          bf16, each 32-element K-tile of the fp32 packing stored as 32 hi = bf16(w) then 32
 *          lo = bf16(w - hi); Cout % 128 == 0 or Cout <= 16 (Npad 16); gn_scale only on the halo form
 *          (3x3, H % 4 == 0, >= 256 tiles or option x3_tile 4) and the pyramid head (3x3, Cout <= 16,
 *          H % 8 == 0, W % 32 == 0, C0 / C1 % 32 == 0, no stats / temb / shortcut / combine), else
 *          hipErrorInvalidValue; out_f32 ignored. */
int snrse_conv2d(snrse_ctx* ctx, const void* src0, int C0, const void* src1, int C1, int B, int H, int W, int ksize,
                 const void* wgt, const void* sc_src, int Csc, const void* sc_src1, int Csc1,
                 const void* sc_wgt, const float* bias, const float* temb, int temb_stride,
                 const void* res, int res_ld, float out_scale, const float* comb_src,
                 const float* comb_w, const float* comb_b, void* out, int Cout, int out_ld,
                 double* stats, const float* gn_scale, const float* gn_shift, int gn_act, int dtype,
                 int out_f32, hipStream_t stream);

/* Statistics buffers of the GroupNorm entries: [B][SNRSE_STAT_SLOTS][C][2] double. */
#define SNRSE_STAT_SLOTS 16

/* GroupNorm statistics (nn.GroupNorm, layerspp.py:221,233): per-channel (sum, sumsq) over
 * H*W of src0 into sums and of src1 into sums1 (slotted layout above; zeroed by the call). */
int snrse_gn_stats(snrse_ctx* ctx, const void* src0, int C0, const void* src1, int C1, int B, int HW, double* sums,
                   double* sums1, int dtype, hipStream_t stream);

/* Per-(b, c) GroupNorm scale/shift from per-channel sums (of src0 | src1, H*W pixels each). */
int snrse_gn_scale_shift(const double* sums0, int C0, const double* sums1, int C1, int B, int HW,
                         const float* gamma, const float* beta, int groups, float eps, float* scale,
                         float* shift, hipStream_t stream);

/* Fused GroupNorm-apply (+SiLU) (+FIR [1,3,3,1] down/up x2) (layerspp.py:245-257,
 * up_or_down_sampling.py:195-257).  sums == NULL: identity normalisation (plain FIR of x).
 * mode: 0 none, 1 down (out H/2 x W/2), 2 up (out 2H x 2W).  out [B][Ho][Wo][C0+C1]. */
int snrse_gn_apply(const void* src0, int C0, const void* src1, int C1, int B, int H, int W,
                   const double* sums, const double* sums1, const float* gamma, const float* beta,
                   int groups, float eps, int act, int mode, void* out, int dtype, hipStream_t stream);

/* LDS-tiled GroupNorm-apply + SiLU + FIR x2 of a ResBlock with up/down (layerspp.py:245-257):
 * out_act = FIR(act(x*scale+shift)) and, when out_raw != NULL, out_raw = FIR(x) (the shortcut input,
 * layerspp.py:249/255), both [B][Ho][Wo][C] from one pass over x.  scale/shift [B][C] f32 from
 * snrse_gn_scale_shift, or both NULL (identity).  mode 1 down (H, W even), 2 up.  dtype SNRSE_BF16: C % 8 == 0
 * with C / 8 dividing 64 (the row-strip kernel), otherwise C % 16 == 0 (the LDS-tiled kernel); SNRSE_F32
 * (the fp32 parity modes): C % 4 == 0 with C / 4 dividing 64 (row strips).  act = 1 computes SiLU in both
 * dtypes as z * rcp(-(1 + 2^z) / ln 2) on the affine prescaled by -log2(e) (v_exp_f32 + v_rcp_f32, each 1 ulp:
 * a few fp32 ulp, ~4e-7 relative), not the IEEE-division silu_exact of snrse_gn_act / snrse_gn_apply; in the
 * exact fp32 mode that is 2-3 orders below its 1e-4 tolerance (tests/test_gpu_kernels.py resample cases). */
int snrse_gn_resample(snrse_ctx* ctx, const void* src, int C, int B, int H, int W, const float* scale, const float* shift,
                      int act, int mode, void* out_act, void* out_raw, int dtype, hipStream_t stream);

/* Elementwise GroupNorm-apply (+SiLU) of the channel concatenation (src0 | src1), dtype SNRSE_BF16 or
 * SNRSE_F32 (exact SiLU), from precomputed scale/shift [B][C0+C1] (snrse_gn_scale_shift; both NULL:
 * identity).  out [B][HW][C0+C1]. */
int snrse_gn_act(const void* src0, int C0, const void* src1, int C1, int B, int HW, const float* scale,
                 const float* shift, int act, void* out, int dtype, hipStream_t stream);

/* Split-K workspace of the small-image conv GEMMs (levels whose tile grid underfills the CUs) of the
 * process default context (per context: snrse_ctx_set_workspace): a device buffer of `bytes` the
 * caller keeps alive and leaves untouched while convs run; the library keeps [splits][M][Cout] f32
 * partial sums there and splits only when they fit.  NULL disables splitting (the default).  Launches
 * that may run concurrently must be issued through contexts with different workspaces. */
int snrse_set_workspace(void* ptr, size_t bytes);

/* Tuning switches of the process default context (per context: snrse_ctx_set_option; A/B experiments;
 * the Python host also reads SNRSE_OPTS="name=value,..." at load):
 * "conv_variant" 0 auto, 1 register-staged v1, 2 LDS-DMA v2, 5 halo GEMM v5 (the default halo kernel);
 * "splitk" 0 disables the split-K small-image GEMMs, "splitk_target" workgroups a split launch aims for;
 * "epi_nt" 0 / 1 / 2 (auto above "epi_nt_mb" = 256 MB of output) non-temporal halo-GEMM output stores;
 * "h5_specialise" 1 compile-time epilogue flags for the NCSN++ ResBlock configurations (16-bit halo GEMM, and the
 *   fp32x3 halo GEMM's pair schedule);
 * "h5_tw" halo-GEMM tile: 0 auto (8 rows x 32 px where H % 8 == 0, else 4 x 64), 64 forces 4 x 64;
 * "resample_variant" 0 row-strip / 1 LDS-tiled gn_resample, "resample_nt" non-temporal stores there,
 * "resample_down_rows" 1 / 2 / 4 (default) output rows per down-sampling row strip (bit-identical results);
 * "x3_tile" split-bf16 fp32 GEMM: 0 auto (the halo kernel on 3x3 convs with H % 4 == 0 and >= 256 tiles of
 *   4 x 64 px x 128 couts, any W, else register-staged 128 x 128), register-staged tiles 1 128 px x 128 couts,
 *   2 256 x 128, 3 128 x 256 (Cout % 256 == 0), 4 the halo kernel wherever its shape conditions hold;
 * "stats_zeroed" 1 = the statistics buffers handed to snrse_conv2d / snrse_gn_stats are already zero (the
 * caller clears one arena per network evaluation), so they skip their per-call memset;
 * "ic_lds" the bf16 input conv (W <= 1024): 3 (default) its workgroup's input rows staged in LDS and its output
 *   staged through LDS for whole-KB stores, 1 input rows only, 2 with the channels split over wave pairs, 0 the
 *   streaming form (all bit-identical but 2's statistics fold order);
 * "x3_tw" fp32x3 halo GEMM tile: 0 (default) 8 x 32 px where H % 8 == 0 and W % 32 == 0, else 4 x 64; 64 forces
 *   4 x 64; "x3_nt" 1 (default) its fp32 output stores non-temporal under the "epi_nt" rule;
 * "x3_spread" fp32x3 halo GEMM schedule: 2 (default) two taps per barrier phase where its tiles are 8 x 32 px and the
 *   main input has an even number of 32-channel chunks (else 1), 1 one tap per phase with the next chunk's halo stored
 *   one piece per tap, 0 the same stored in one go;
 * "head_small" bf16 pyramid heads (Cout 4, C % 256 == 0): 1 (default) the wave-per-8-pixels head (GroupNorm fused)
 *   where the tiled head cannot take the image (H % 8 or W % 32 != 0), 2 also for up to 16384 output pixels, 0 never;
 * "head_part" tiled bf16 pyramid head with Cout 4: 1 (default) the halo's 36 tap partials as one 1x1 GEMM then their
 *   shifted sum (last_kernel 15), 0 nine tap GEMMs over the halo (last_kernel 10);
 * "gn_slice" snrse_gn_apply with statistics (no resampling): 1 (default) each block owns a 64-channel slice of its
 *   pixels and folds only that slice's statistics, 0 each block folds all channels (equal results; read from the
 *   process default context, as snrse_gn_apply takes none). */
int snrse_set_option(const char* name, int value);

/* Read back a switch (any name above) or: "halo_kernel" = generation of the halo conv kernel the current
 * setting dispatches a 3x3 conv to (5), "last_kernel" = generation of the most recent snrse_conv2d launch (1 v1, 2 v2,
 * 3 / 4 split-bf16 register-staged / halo, 5 halo, 10 pyramid head, 11 split-bf16 pyramid head, 14 small-image
 * pyramid head, 15 tap-partials pyramid head),
 * "last_ksplit" = K splits of the most recent v2 launch, "last_epi_nt" /
 * "last_chunks" = store flavour / image-range launches of the most recent halo conv, "last_tw" = its tile
 * width (32 / 64). */
int snrse_get_option(const char* name, int* value);

/* AttnBlockpp attention core (layerspp.py:84-88): qkv [B][L][3C] -> out [B][L][C],
 * softmax(q k^T / sqrt(C)) v, flash-style on MFMA.  C must be 256.  dtype SNRSE_BF16, SNRSE_F32 (exact fp32
 * MFMAs) or SNRSE_F32X3 (fp32 in / out, q, k, v and the probabilities split into bf16 hi + lo, hi.hi + hi.lo + lo.hi
 * products: the fp32x3 parity mode). */
int snrse_attention(const void* qkv, void* out, int B, int L, int C, int dtype, hipStream_t stream);

/* Time embedding (ncsnpp.py:256-275): temb[b] = W2 silu(W1 [sin, cos](2 pi log t W_gfp) + b1) + b2. */
int snrse_temb_mlp(const float* t, const float* Wg, const float* W1, const float* b1, const float* W2,
                   const float* b2, float* temb, int B, int nf, hipStream_t stream);
/* The same MLP as two row-parallel launches (the form the network executor runs; every weight row is read once
 * per launch, spread over the chip): snrse_temb_gfp_dense gives the pre-activation a[b] = W1 [sin, cos](2 pi log t
 * W_gfp) + b1 (out [B][4 nf]), then snrse_temb_dense(a, W2, b2) = W2 silu(a) + b2 = temb.  nf even, 4 nf <= 512
 * (nf <= 128: snrse_temb_dense takes D = 4 nf <= 512; NCSN++ uses nf = 128). */
int snrse_temb_gfp_dense(const float* t, const float* Wg, const float* W1, const float* b1, float* out, int B, int nf,
                         hipStream_t stream);
/* All ResBlock Dense_0 projections (layerspp.py:264-265): out[b][r] = W[r] . silu(temb[b]) + bias[r]. */
int snrse_temb_dense(const float* temb, const float* W, const float* bias, float* out, int B, int R, int D,
                     hipStream_t stream);

/* Fused input conv, 16-bit (ncsnpp.py:253-254, 282-285): complex x, y [B][H][W] -> out [B*H*W][128]
 * (dtype SNRSE_F16 or SNRSE_BF16) = conv3x3(cat(x.re, x.im, y.re, y.im), wgt) + bias, plus the f32 input pyramid
 * pyr [B*H*W][4] and out's GroupNorm statistics [B][SLOTS][128][2] (zeroed here unless option
 * stats_zeroed).  wgt: dtype [128][64], k = (ky * 3 + kx) * 4 + channel, k >= 36 zero.
 * Requires W % 64 == 0 and (H * W / 64) % 16 == 0 (else SNRSE_EINVAL: use snrse_input_pack). */
int snrse_input_conv(snrse_ctx* ctx, const void* x, const void* y, int B, int H, int W, const void* wgt, const float* bias,
                     void* out, float* pyr, double* stats, int dtype, hipStream_t stream);

/* The same input conv for the fp32x3 parity mode: wgt = ops.split_weight of the packed [128][64] weights ([128][128]
 * bf16: per 32-element K tile 32 hi then 32 lo), split-bf16 products (w_hi.x_hi + w_lo.x_hi + w_hi.x_lo), f32 out
 * [B*H*W][128]; the input rows staged in LDS (W % 64 == 0, W <= 1024, (H*W/64) % 16 == 0).  Replaces
 * snrse_input_pack + the split GEMM on its im2col. */
int snrse_input_conv_x3(snrse_ctx* ctx, const void* x, const void* y, int B, int H, int W, const void* wgt,
                        const float* bias, float* out, float* pyr, double* stats, hipStream_t stream);

/* Network input (ncsnpp.py:253-254, 282-285): complex x, y [B,F,T] -> im2col [B,F,T,64]
 * (tap-major 3x3 x {x.re, x.im, y.re, y.im}, zero padded) in dtype, and the f32 input
 * pyramid [B,F,T,4]. */
int snrse_input_pack(const void* x, const void* y, int B, int H, int W, void* col, float* pyr, int dtype,
                     hipStream_t stream);

/* Output head + preconditioning + SDE step (ncsnpp.py:398-404, model.py:481-541,
 * predictors.py:75-80, correctors.py:69-81).  pyr [B,F,T,4] (f32 if pyr_f32 else bf16),
 * t [B], score_mode 0 = -dnn ('bbed'), 1 = c_skip x + c_out dnn ('sebridge*').
 * coef [B][4] = {a, by, c, s}: x_mean = a x + by y + c score; x_out = x_mean + s z.
 * z = noise (complex64 tensor) or, if noise == NULL, Philox4x32-10(seed, offset + index)
 * complex normal with each part N(0, 1/2).  x_out == NULL: only score_out is written. */
int snrse_score_update(const void* pyr, int pyr_f32, const float* out_w, const float* out_b,
                       const float* t, int score_mode, int B, int HW, const void* x, const void* y,
                       const void* noise, uint64_t seed, uint64_t offset, const float* coef,
                       void* x_out, void* xmean_out, void* score_out, hipStream_t stream);

/* Same step for an arbitrary score tensor (generic score_fn). */
int snrse_sde_update(const void* x, const void* y, const void* score, const void* noise, uint64_t seed,
                     uint64_t offset, const float* coef, int B, int HW, void* x_out, void* xmean_out,
                     hipStream_t stream);

/* out = coef[b][0] x + coef[b][1] y + coef[b][3] z (prior sampling, sdes.py:225-232, 298-304). */
int snrse_axpby_noise(const void* x, const void* y, const void* noise, uint64_t seed, uint64_t offset,
                      const float* coef, int B, int HW, void* out, hipStream_t stream);

/* Evaluation metrics (eval.py:144-157 -> utils.py:10-35 energy_ratios, sgmse/util/other.py:71-75
 * si_sdr), batched: s_hat, s, n [B][L] f32 (n may be NULL) -> out [B][3] f64 = (SI-SDR, SI-SIR,
 * SI-SAR) in dB from six fp64 dot products per utterance; SI-SIR / SI-SAR are NaN without n. */
int snrse_energy_ratios(const float* s_hat, const float* s, const float* n, int B, int L, double* out,
                        hipStream_t stream);

/* norm_factor = max |y| per utterance (model.py:726): out[b] = max_i |sig[b][i]|. */
int snrse_absmax(const float* sig, int B, int L, float* out, hipStream_t stream);

/* STFT (data_module.py:291-293 with spec_fwd 241-254 and pad_spec other.py:83-90):
 * sig [B][L] f32 -> out complex64 [B][256][Tpad], frames 1 + L/128 (the rest zero).
 * mode 0 raw, 1 exponent transform (|X|^0.5 e^{i angle X} * 0.15).  The signal is scaled by
 * in_scale / in_div[b] (in_div: per-utterance norm factors on the device, or NULL). */
int snrse_stft(const float* sig, int B, int L, const float* in_div, float in_scale, int Tpad, int mode,
               void* out, hipStream_t stream);

/* iSTFT (data_module.py:295-297 with spec_back 256-267): spec complex64 [B][256][T] -> out [B][L]
 * f32, times out_scale[b] (NULL = 1).  frames: workspace of B*T*510 floats. */
int snrse_istft(const void* spec, int B, int T, int L, int mode, const float* out_scale, float* frames,
                float* out, hipStream_t stream);

/* Exponent spectrogram transform on interleaved complex64 (data_module.py:241-267):
 * dir 0 = spec_fwd (|c|^0.5 e^{i angle c} * 0.15), dir 1 = spec_back (inverse).  In place allowed. */
int snrse_spec_transform(const void* in, void* out, long long n, int dir, hipStream_t stream);

/* SNR estimator SNRNet.forward (snrnet.py:47-97) on the raw complex STFT spec [B][256][T]
 * (T % 16 == 0): out[b] = sigmoid(...) in (0, 1).  Weights f32 in torch layouts (see
 * csrc/snrnet.hip); ws: workspace of snrse_snrnet_workspace(B, T) bytes. */
int snrse_snrnet(const void* spec, int B, int T, const float* w5, const float* b5, const float* w3,
                 const float* b3, const float* wt1, const float* wt2, const float* wt3, const float* wt4,
                 const float* bt1, const float* bt2, const float* bt3, const float* bt4, const float* wih,
                 const float* bsum, const float* whh, const float* fcw, const float* fcb, float* ws,
                 float* out, hipStream_t stream);
size_t snrse_snrnet_workspace(int B, int T);

/* ---- Consistency-training step (ScoreModel._step, model.py:361-390, with the
 * backward pass PyTorch Lightning runs through loss.backward() and the Adam / torch_ema updates of
 * model.py:99-106).  All f32, NHWC activations; csrc/train.hip. */

/* dW[co][ky][kx][ci] += sum_p dY[p][co] X[p + (ky-1, kx-1)][ci] (ksize 3, pad 1) or the 1x1 form;
 * X is the channel concatenation of x0 [.., C0] and x1 [.., C1]; dw must be zeroed by the caller. */
int snrse_conv_wgrad(const float* dy, int Cout, const float* x0, int C0, const float* x1, int C1, int B, int H,
                     int W, int ksize, float* dw, hipStream_t stream);
/* The same with split-bf16 products (fp32 in and out; dY and X split into bf16 hi / lo, three bf16 MFMA
 * products per block): the fp32x3 training mode.  Cout, C0, C1 multiples of 4. */
int snrse_conv_wgrad_x3(const float* dy, int Cout, const float* x0, int C0, const float* x1, int C1, int B, int H,
                        int W, int ksize, float* dw, hipStream_t stream);
/* scale * per-(b, c) sums over the HW pixels of x [B][HW][C] added into out_bc [B][C] and / or the
 * per-c total into out_c [C] (bias, Dense_0 and temb gradients). */
int snrse_chan_sum(const float* x, int B, int HW, int C, float* out_bc, float* out_c, float scale,
                   hipStream_t stream);
/* per-(b, group) mean and rstd = 1/sqrt(var + eps) from the slotted (sum, sumsq) statistics of the
 * forward GroupNorm (snrse_gn_stats) of one or two channel-concatenated sources. */
int snrse_gn_moments(const double* st0, int C0, const double* st1, int C1, int B, int HW, int groups, float eps,
                     float* mean, float* rstd, hipStream_t stream);
/* GroupNorm (+SiLU when act) backward (nn.GroupNorm layerspp.py:221,233; SiLU layers.py:38-39):
 * dy [B][HW][C0+C1] -> dx0 [B][HW][C0], dx1 [B][HW][C1]; dgamma / dbeta [C] accumulated (+=);
 * R: workspace of 2*B*(C0+C1) floats. */
int snrse_gn_backward(const float* x0, int C0, const float* x1, int C1, const float* dy, int B, int HW,
                      int groups, const float* gamma, const float* beta, const float* mean, const float* rstd,
                      int act, float* R, float* dx0, float* dx1, float* dgamma, float* dbeta, hipStream_t stream);
/* batched strided GEMM on MFMA: C[b](m,n) = alpha sum_k A[b](m,k) B[b](k,n) + beta C[b](m,n) (+ bias[n]),
 * element (i, j) of operand X at X + b*sXb + i*sX(row) + j*sX(col); beta is 0 or 1. */
int snrse_bgemm(const float* A, long long sAb, long long sAm, long long sAk, const float* Bm, long long sBb,
                long long sBk, long long sBn, float* C, long long sCb, long long sCm, long long sCn, const float* bias,
                int batch, int M, int N, int K, float alpha, float beta, hipStream_t stream);
/* row softmax P = softmax(scale S) and its backward dS = scale P (dP - <dP, P>_row), rows of L. */
int snrse_softmax_rows(const float* S, float* P, long long rows, int L, float scale, hipStream_t stream);
int snrse_softmax_bwd_rows(const float* P, const float* dP, float* dS, long long rows, int L, float scale,
                           hipStream_t stream);
/* elementwise: y = silu(x); dx (+)= dy silu'(x); y = a x + b y; y = x * s[b] (recip: x / s[b]). */
int snrse_silu(const float* x, float* y, long long n, hipStream_t stream);
int snrse_silu_bwd(const float* x, const float* dy, float* dx, long long n, int accumulate, hipStream_t stream);
int snrse_axpby(const float* x, float* y, long long n, float a, float b, hipStream_t stream);
int snrse_scale_rows(const float* x, const float* s, float* y, int B, long long per, int recip, hipStream_t stream);
/* GaussianFourierProjection of log t (layerspp.py:32-43): out [B][2 nf] = [sin, cos](2 pi log t W). */
int snrse_gfp(const float* t, const float* Wg, int B, int nf, float* out, hipStream_t stream);
/* perturbation of the consistency step on complex64 [B][HW]: mu = H(H^-1(x)(1 - w_b) + H^-1(y) w_b),
 * x_t = mu + s_b z (H = exponent transform when transform != 0, model.py:304-312, 372-376). */
int snrse_ct_perturb(const void* x, const void* y, const void* z, const float* wmix, const float* nscale, int B,
                     int HW, int transform, void* mu, void* xt, hipStream_t stream);
/* sebridge_v3 outputs f_k = cs_k x_k + co_k dnn_k (coef [B][4] = cs1, co1, cs0, co0), the mse
 * (sqrt_loss = 0) or sqrt_mse (1) consistency loss per utterance into loss_b [B] (f64, the batch loss
 * is their mean), and its gradient w.r.t. dnn1 / dnn0 (complex64 [B][HW], HW % 64 == 0). */
int snrse_ct_loss(const void* dnn1, const void* dnn0, const void* x1, const void* x0, const float* coef, int B,
                  int HW, int sqrt_loss, double* loss_b, void* g1, void* g0, hipStream_t stream);
/* one torch.optim.Adam step (+ torch_ema update when a tensor's ema pointer is set) over a table of
 * device tensors {float* p, const float* g, float* m, float* v, float* ema, int64 n} (device memory),
 * split into chunks of 2048 elements (chunk_tensor / chunk_start, device arrays of nchunks). */
int snrse_adam_ema(const void* tensors, const int* chunk_tensor, const long long* chunk_start, int nchunks,
                   float lr, float beta1, float beta2, float eps, float bias_corr1, float bias_corr2_sqrt,
                   float ema_decay, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SNRSE_H_ */
