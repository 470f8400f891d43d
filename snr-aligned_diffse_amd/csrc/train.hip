// Backward-pass and optimizer kernels of the consistency-training step (reference
// ScoreModel._step, sgmse/model.py:361-390, driven by PyTorch Lightning's loss.backward() and
// torch.optim.Adam + torch_ema, model.py:99-106).  fp32 throughout, NHWC activations.
//
//   snrse_conv_wgrad      dW[co][tap][ci] += sum_p dY[p][co] X[p + tap][ci]  (3x3 pad 1 / 1x1), MFMA f32
//   snrse_conv_wgrad_x3   the same as split-bf16 products (the fp32x3 training mode)
//   snrse_chan_sum        per-(b, c) and per-c sums of an NHWC tensor (bias / temb / GroupNorm-affine grads)
//   snrse_gn_moments      per-(b, group) mean and rstd from the forward's slotted (sum, sumsq) statistics
//   snrse_gn_backward     GroupNorm (+SiLU) backward: dx of one or two (channel-concatenated) sources,
//                         dgamma / dbeta (nn.GroupNorm, layerspp.py:221,233; SiLU layers.py:38-39)
//   snrse_bgemm           batched strided f32 GEMM on MFMA: C = alpha op(A) op(B) + beta C (+ bias[n]):
//                         NIN / Linear layers and the attention products (layerspp.py:64-93, layers.py:546-555)
//   snrse_softmax_rows    P = softmax(scale S) over rows; snrse_softmax_bwd_rows dS = P (dP - <dP, P>)
//   snrse_silu_bwd        dx = dy silu'(x)
//   snrse_axpby           y = a x + b y
//   snrse_ct_perturb      mu_t = H(H^-1(x)(1-w) + H^-1(y) w), x_t = mu_t + s z (model.py:304-312, 372-376)
//   snrse_ct_loss         sebridge_v3 preconditioning of both evaluations + mse / sqrt_mse loss and its
//                         gradient w.r.t. both network outputs (model.py:378-390, 536-541)
//   snrse_adam_ema        torch.optim.Adam step (+ torch_ema 0.3 shadow update) over many tensors, one launch
#include "common.h"

#include <algorithm>

namespace {

// --------------------------------------------------------------------------------------- conv wgrad
// Block: 4 waves = 64 co x 64 ci of one conv (all KS*KS taps), a range of 32-pixel row segments.
// Wave w owns ci [ci0 + 16w, +16) and 4 co fragments: acc[4][KS*KS] of 16x16 f32 (D = [co][ci]).
// Per 32-px segment: dY tile [32 px][64 co] and the X halo [KS rows][32 + KS - 1 px][64 ci] staged in
// LDS (row stride 80 floats: the two 16-lane halves of a ds_read_b32 group hit disjoint banks).
constexpr int WG_P = 32, WG_LD = 80;

template <int KS>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const float* dy, int Cout, const float* x0, int C0,
                                                         const float* x1, int C1, int B, int H, int W, float* dw,
                                                         int segs_per_blk) {
  constexpr int T = KS * KS, HP = WG_P + KS - 1;
  __shared__ float dyl[WG_P * WG_LD];
  __shared__ float xl[KS * HP * WG_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64;
  const int Cin = C0 + C1;
  const int nws = (W + WG_P - 1) / WG_P;
  const long long nseg = (long long)B * H * nws;
  const long long s0 = (long long)blockIdx.z * segs_per_blk;
  const long long s1 = std::min(nseg, s0 + segs_per_blk);
  f32x4 acc[4][T];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < T; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ln = lane & 15, lk = lane >> 4;
  for (long long sg = s0; sg < s1; ++sg) {
    const int wsg = (int)(sg % nws);
    const int h = (int)((sg / nws) % H);
    const int b = (int)(sg / ((long long)nws * H));
    const int w0 = wsg * WG_P;
    __syncthreads();
    for (int e = tid; e < WG_P * 64; e += 256) {
      const int px = e >> 6, c = e & 63;
      const int w = w0 + px, co = co0 + c;
      dyl[px * WG_LD + c] = (w < W && co < Cout) ? dy[(((size_t)b * H + h) * W + w) * Cout + co] : 0.f;
    }
    for (int e = tid; e < KS * HP * 64; e += 256) {
      const int c = e & 63, r = e >> 6;
      const int px = r % HP, ky = r / HP;
      const int hh = h + ky - KS / 2, ww = w0 + px - KS / 2, ci = ci0 + c;
      float v = 0.f;
      if (hh >= 0 && hh < H && ww >= 0 && ww < W && ci < Cin) {
        const size_t pix = ((size_t)b * H + hh) * W + ww;
        v = ci < C0 ? x0[pix * C0 + ci] : x1[pix * C1 + ci - C0];
      }
      xl[(ky * HP + px) * WG_LD + c] = v;
    }
    __syncthreads();
#pragma unroll 2
    for (int g = 0; g < WG_P / 4; ++g) {
      const int px = 4 * g + lk;  // MFMA k index = pixel
      float a[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) a[f] = dyl[px * WG_LD + f * 16 + ln];
#pragma unroll
      for (int ky = 0; ky < KS; ++ky)
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const float bv = xl[(ky * HP + px + kx) * WG_LD + wid * 16 + ln];
#pragma unroll
          for (int f = 0; f < 4; ++f)
            acc[f][ky * KS + kx] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[f], bv, acc[f][ky * KS + kx], 0, 0, 0);
        }
    }
  }
  const int ci = ci0 + wid * 16 + ln;
  if (ci >= Cin) return;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + f * 16 + 4 * lk + e;
      if (co >= Cout) continue;
#pragma unroll
      for (int t = 0; t < T; ++t) unsafeAtomicAdd(&dw[((size_t)co * T + t) * Cin + ci], acc[f][t][e]);
    }
}

// --------------------------------------------------------------------------------------- conv wgrad, split bf16
// The fp32x3 training mode's weight gradient: the same block / segment walk as conv_wgrad_kernel, with the
// staged dY and X tiles split into bf16 hi / lo images in their natural [pixel][channel] layout, and each
// 16x16x32 block as A_hi B_hi + A_hi B_lo + A_lo B_hi on v_mfma_f32_16x16x32_bf16.  The reduction axis is
// the pixel, i.e. the ROW of both images: the operand fragments are read column-major with
// ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3; lane i receives
// column i of the 4 rows), so a tap's pixel shift is just a row offset -- no shifted copies.
constexpr int XW_RS = 144;  // LDS row stride (bytes): 64 bf16 + 16 B pad, a multiple of 8 for the tr reads

typedef short s16x4 __attribute__((ext_vector_type(4)));

SNRSE_DEV u32x4 tr_frag(const char* img, int row0, int col) {  // k = rows row0 .. row0 + 7 of column `col`
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + row0 * XW_RS + col * 2));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (row0 + 4) * XW_RS + col * 2));
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  const u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
  return u32x4{ua[0], ua[1], ub[0], ub[1]};
}

SNRSE_DEV void split_store4(char* hi, char* lo, int off, const f32x4 v) {  // 4 f32 -> 4 bf16 hi + 4 bf16 lo
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  const uint32_t h01 = pack_bf16x2(v[0], v[1]), h23 = pack_bf16x2(v[2], v[3]);
  const uint32_t l01 = pack_bf16x2(v[0] - __uint_as_float(h01 << 16), v[1] - __uint_as_float(h01 & 0xffff0000u));
  const uint32_t l23 = pack_bf16x2(v[2] - __uint_as_float(h23 << 16), v[3] - __uint_as_float(h23 & 0xffff0000u));
  *(u32x2*)(hi + off) = u32x2{h01, h23};
  *(u32x2*)(lo + off) = u32x2{l01, l23};
}

template <int KS>
__global__ __launch_bounds__(256, 2) void conv_wgrad_x3_kernel(const float* dy, int Cout, const float* x0, int C0,
                                                               const float* x1, int C1, int B, int H, int W,
                                                               float* dw, int segs_per_blk) {
  constexpr int T = KS * KS, HP = WG_P + KS - 1;
  __shared__ __attribute__((aligned(16))) char lds[(2 * WG_P + 2 * KS * HP) * XW_RS];
  char* const dyh = lds;
  char* const dyl = lds + WG_P * XW_RS;
  char* const xh = lds + 2 * WG_P * XW_RS;
  char* const xl = xh + KS * HP * XW_RS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64;
  const int Cin = C0 + C1;
  const int nws = (W + WG_P - 1) / WG_P;
  const long long nseg = (long long)B * H * nws;
  const long long s0 = (long long)blockIdx.z * segs_per_blk;
  const long long s1 = std::min(nseg, s0 + segs_per_blk);
  f32x4 acc[4][T];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < T; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane >> 2) & 3, cp = (lane & 3) * 4;  // tr-read group, row, column quad
  for (long long sg = s0; sg < s1; ++sg) {
    const int wsg = (int)(sg % nws);
    const int h = (int)((sg / nws) % H);
    const int b = (int)(sg / ((long long)nws * H));
    const int w0 = wsg * WG_P;
    __syncthreads();
    for (int e = tid; e < WG_P * 16; e += 256) {  // dY tile [32 px][64 co], 4 channels per vector
      const int px = e >> 4, c4 = (e & 15) * 4;
      const int w = w0 + px, co = co0 + c4;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (w < W && co < Cout) v = *(const f32x4*)(dy + (((size_t)b * H + h) * W + w) * Cout + co);
      split_store4(dyh, dyl, px * XW_RS + c4 * 2, v);
    }
    for (int e = tid; e < KS * HP * 16; e += 256) {  // X halo [KS rows][HP px][64 ci]
      const int c4 = (e & 15) * 4, r = e >> 4;
      const int px = r % HP, ky = r / HP;
      const int hh = h + ky - KS / 2, ww = w0 + px - KS / 2, ci = ci0 + c4;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (hh >= 0 && hh < H && ww >= 0 && ww < W && ci < Cin) {
        const size_t pix = ((size_t)b * H + hh) * W + ww;
        v = ci < C0 ? *(const f32x4*)(x0 + pix * C0 + ci) : *(const f32x4*)(x1 + pix * C1 + ci - C0);
      }
      split_store4(xh, xl, r * XW_RS + c4 * 2, v);
    }
    __syncthreads();
    u32x4 ah[4], al[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {  // A = dY^T: rows co, k = px
      ah[f] = tr_frag(dyh, 8 * g + q, f * 16 + cp);
      al[f] = tr_frag(dyl, 8 * g + q, f * 16 + cp);
    }
#pragma unroll
    for (int ky = 0; ky < KS; ++ky)
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {  // B = X shifted by the tap: rows px + kx of image row ky
        const int row0 = ky * HP + 8 * g + q + kx;
        const u32x4 bh = tr_frag(xh, row0, wid * 16 + cp), bl = tr_frag(xl, row0, wid * 16 + cp);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          f32x4& a = acc[f][ky * KS + kx];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, ah[f]),
                                                      __builtin_bit_cast(bf16x8_mfma, bh), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, ah[f]),
                                                      __builtin_bit_cast(bf16x8_mfma, bl), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, al[f]),
                                                      __builtin_bit_cast(bf16x8_mfma, bh), a, 0, 0, 0);
        }
      }
  }
  const int ln = lane & 15, lk = lane >> 4;
  const int ci = ci0 + wid * 16 + ln;
  if (ci >= Cin) return;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + f * 16 + 4 * lk + e;
      if (co >= Cout) continue;
#pragma unroll
      for (int t = 0; t < T; ++t) unsafeAtomicAdd(&dw[((size_t)co * T + t) * Cin + ci], acc[f][t][e]);
    }
}

// --------------------------------------------------------------------------------------- channel sums
// grid (nblk, B); per (b, c): sum over the block's pixel range -> atomics into out_bc[b][c] and/or out_c[c]
__global__ __launch_bounds__(256) void chan_sum_kernel(const float* x, int HW, int C, int ppb, float* out_bc,
                                                       float* out_c, float scale) {
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += x[((size_t)b * HW + p) * C + c];
    s *= scale;
    if (out_bc) unsafeAtomicAdd(&out_bc[(size_t)b * C + c], s);
    if (out_c) unsafeAtomicAdd(&out_c[c], s);
  }
}

// --------------------------------------------------------------------------------------- GroupNorm backward
__global__ void gn_moments_kernel(const double* st0, int C0, const double* st1, int C1, int B, int HW, int G,
                                  float eps, float* mean, float* rstd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * G) return;
  const int b = i / G, g = i % G;
  const int C = C0 + C1, cg = C / G;
  double s = 0.0, ss = 0.0;
  for (int c = g * cg; c < (g + 1) * cg; ++c) {
    if (c < C0) stat_fold(st0, b, c, C0, s, ss);
    else stat_fold(st1, b, c - C0, C1, s, ss);
  }
  const double n = (double)cg * HW;
  const double m = s / n;
  const double var = fmax(ss / n - m * m, 0.0);
  mean[i] = (float)m;
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

SNRSE_DEV float gn_src(const float* x0, int C0, const float* x1, int C1, size_t pix, int c) {
  return c < C0 ? x0[pix * C0 + c] : x1[pix * C1 + c - C0];
}

// pass 1: R[b][c] = (sum_p dyh, sum_p dyh xhat), dyh = dy * silu'(a) (act) or dy, a = gamma xhat + beta
__global__ __launch_bounds__(256) void gn_bwd_reduce_kernel(const float* x0, int C0, const float* x1, int C1,
                                                            const float* dy, int HW, int G, const float* gamma,
                                                            const float* beta, const float* mean, const float* rstd,
                                                            int act, int ppb, float* R) {
  const int b = blockIdx.y, C = C0 + C1, cg = C / G;
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cg;
    const float m = mean[b * G + g], r = rstd[b * G + g], ga = gamma[c], be = beta[c];
    float s1 = 0.f, s2 = 0.f;
    for (int p = p0; p < p1; ++p) {
      const size_t pix = (size_t)b * HW + p;
      const float xh = (gn_src(x0, C0, x1, C1, pix, c) - m) * r;
      float d = dy[pix * C + c];
      if (act) {
        const float a = ga * xh + be;
        const float sg = 1.f / (1.f + expf(-a));
        d *= sg * (1.f + a * (1.f - sg));
      }
      s1 += d;
      s2 = fmaf(d, xh, s2);
    }
    unsafeAtomicAdd(&R[((size_t)b * C + c) * 2], s1);
    unsafeAtomicAdd(&R[((size_t)b * C + c) * 2 + 1], s2);
  }
}

// pass 2: dx = rstd (gamma dyh - S1/n - xhat S2/n), S1 = sum_{c in g} gamma_c R1, S2 = sum gamma_c R2
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const float* x0, int C0, const float* x1, int C1,
                                                           const float* dy, int HW, int G, const float* gamma,
                                                           const float* beta, const float* mean, const float* rstd,
                                                           int act, const float* R, float* dx0, float* dx1,
                                                           long long total) {
  const int C = C0 + C1, cg = C / G;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const size_t pix = (size_t)(i / C);
    const int b = (int)(pix / HW);
    const int g = c / cg;
    float S1 = 0.f, S2 = 0.f;
    for (int k = g * cg; k < (g + 1) * cg; ++k) {
      S1 = fmaf(gamma[k], R[((size_t)b * C + k) * 2], S1);
      S2 = fmaf(gamma[k], R[((size_t)b * C + k) * 2 + 1], S2);
    }
    const float n = (float)cg * (float)HW;
    const float m = mean[b * G + g], r = rstd[b * G + g];
    const float xh = (gn_src(x0, C0, x1, C1, pix, c) - m) * r;
    float d = dy[i];
    if (act) {
      const float a = gamma[c] * xh + beta[c];
      const float sg = 1.f / (1.f + expf(-a));
      d *= sg * (1.f + a * (1.f - sg));
    }
    const float v = r * (gamma[c] * d - S1 / n - xh * S2 / n);
    if (c < C0) dx0[pix * C0 + c] = v;
    else dx1[pix * C1 + c - C0] = v;
  }
}

__global__ void gn_bwd_affine_kernel(const float* R, int B, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
  for (int b = 0; b < B; ++b) {
    s1 += R[((size_t)b * C + c) * 2];
    s2 += R[((size_t)b * C + c) * 2 + 1];
  }
  if (dbeta) dbeta[c] += s1;
  if (dgamma) dgamma[c] += s2;
}

// --------------------------------------------------------------------------------------- batched GEMM
// C[b](m, n) = alpha sum_k A[b](m, k) B[b](k, n) + beta C[b](m, n) (+ bias[n]); 64 x 64 tile per block,
// 4 waves of 32 x 32 (2 x 2 MFMA f32 16x16x4 fragments), K staged 16 at a time through LDS.
struct GemmArgs {
  const float* A; long long sAb, sAm, sAk;
  const float* Bm; long long sBb, sBk, sBn;
  float* C; long long sCb, sCm, sCn;
  const float* bias;
  int M, N, K;
  float alpha, beta;
};

__global__ __launch_bounds__(256) void bgemm_kernel(GemmArgs g) {
  __shared__ float As[16][68], Bs[16][68];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bz = blockIdx.z, m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const float* A = g.A + bz * g.sAb;
  const float* Bp = g.Bm + bz * g.sBb;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ln = lane & 15, lk = lane >> 4;
  for (int k0 = 0; k0 < g.K; k0 += 16) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      // A tile: e -> (k = e / 64, m = e % 64) when m is the fast index in memory order, else (m, k)
      const int kk = e >> 6, mm = e & 63;
      const int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < g.M && k < g.K) ? A[m * g.sAm + k * g.sAk] : 0.f;
      const int n = n0 + mm;
      Bs[kk][mm] = (n < g.N && k < g.K) ? Bp[k * g.sBk + n * g.sBn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[ks * 4 + lk][wm * 32 + i * 16 + ln];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[ks * 4 + lk][wn * 32 + j * 16 + ln];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  float* C = g.C + bz * g.sCb;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + 4 * lk + e, n = n0 + wn * 32 + j * 16 + ln;
        if (m < g.M && n < g.N) {
          float v = g.alpha * acc[i][j][e];
          if (g.bias) v += g.bias[n];
          float* cp = C + m * g.sCm + n * g.sCn;
          *cp = g.beta != 0.f ? v + g.beta * *cp : v;
        }
      }
}

// --------------------------------------------------------------------------------------- softmax rows
__global__ __launch_bounds__(64) void softmax_rows_kernel(const float* S, float* P, int L, float scale) {
  const size_t row = blockIdx.x;
  const float* s = S + row * L;
  float* p = P + row * L;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < L; j += 64) mx = fmaxf(mx, s[j] * scale);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = threadIdx.x; j < L; j += 64) sum += expf(s[j] * scale - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  for (int j = threadIdx.x; j < L; j += 64) p[j] = expf(s[j] * scale - mx) * inv;
}

__global__ __launch_bounds__(64) void softmax_bwd_rows_kernel(const float* P, const float* dP, float* dS, int L,
                                                              float scale) {
  const size_t row = blockIdx.x;
  const float* p = P + row * L;
  const float* dp = dP + row * L;
  float dot = 0.f;
  for (int j = threadIdx.x; j < L; j += 64) dot = fmaf(p[j], dp[j], dot);
  dot = wave_sum(dot);
  for (int j = threadIdx.x; j < L; j += 64) dS[row * L + j] = scale * p[j] * (dp[j] - dot);
}

// --------------------------------------------------------------------------------------- elementwise
__global__ void silu_bwd_kernel(const float* x, const float* dy, float* dx, long long n, int accumulate) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float a = x[i];
    const float sg = 1.f / (1.f + expf(-a));
    const float v = dy[i] * sg * (1.f + a * (1.f - sg));
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

__global__ void silu_kernel(const float* x, float* y, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = silu_exact(x[i]);
}

// y[b][i] = x[b][i] * s[b]  (NCSNpp.forward h / used_sigmas, ncsnpp.py:398-400; also its own adjoint)
__global__ void scale_rows_kernel(const float* x, const float* s, float* y, long long per, long long n, int recip) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float f = s[i / per];
    y[i] = recip ? x[i] / f : x[i] * f;
  }
}

// GaussianFourierProjection of log t (layerspp.py:32-43, ncsnpp.py:256-262): [sin(2 pi log t W), cos(...)]
__global__ void gfp_kernel(const float* t, const float* Wg, int nf, float* out) {
  const int b = blockIdx.x;
  const float lt = logf(t[b]);
  for (int i = threadIdx.x; i < nf; i += blockDim.x) {
    const float pr = lt * Wg[i] * 6.28318530717958647692f;
    out[(size_t)b * 2 * nf + i] = sinf(pr);
    out[(size_t)b * 2 * nf + nf + i] = cosf(pr);
  }
}

__global__ void axpby_kernel(const float* x, float* y, long long n, float a, float b) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = b == 0.f ? a * x[i] : fmaf(a, x[i], b * y[i]);
}

// exponent transform (data_module.py:241-267): H(c) = 0.15 c |c|^-1/2, H^-1(c) = |c / 0.15| c / 0.15
SNRSE_DEV float2 spec_fwd1(float2 v) {
  const float mag = sqrtf(v.x * v.x + v.y * v.y);
  const float g = mag > 0.f ? 0.15f / sqrtf(mag) : 0.f;
  return make_float2(v.x * g, v.y * g);
}
SNRSE_DEV float2 spec_back1(float2 v) {
  v.x *= (1.0f / 0.15f);
  v.y *= (1.0f / 0.15f);
  const float mag = sqrtf(v.x * v.x + v.y * v.y);
  return make_float2(v.x * mag, v.y * mag);
}

// mu = H(H^-1(x) (1 - w) + H^-1(y) w), x_t = mu + s z with per-utterance mixing weight w and noise scale s:
// snr_conditioned 'true' w = t (model.py:372-376), 'fixed' w = fixed_snr t (x_ori + y0_ori fixed_snr t,
// model.py:304-312); s = t sigma_max in both (z = randn * sigma_max)
__global__ void ct_perturb_kernel(const float2* x, const float2* y, const float2* z, const float* wmix,
                                  const float* nscale, int HW, long long n, int transform, float2* mu, float2* xt) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float w = wmix[i / HW], sc = nscale[i / HW];
    float2 a = x[i], b = y[i];
    if (transform) { a = spec_back1(a); b = spec_back1(b); }
    float2 m = make_float2(a.x * (1.f - w) + b.x * w, a.y * (1.f - w) + b.y * w);
    if (transform) m = spec_fwd1(m);
    mu[i] = m;
    const float2 zz = z[i];
    xt[i] = make_float2(m.x + sc * zz.x, m.y + sc * zz.y);
  }
}

// sqrt transform s(f) = f |f|^-1/2 (= |f|^0.5 e^{i angle f}) and its vector-Jacobian product
SNRSE_DEV float2 sqrt_c(float2 f) {
  const float u = f.x * f.x + f.y * f.y;
  const float q = u > 0.f ? rsqrtf(sqrtf(u)) : 0.f;
  return make_float2(f.x * q, f.y * q);
}
SNRSE_DEV float2 sqrt_c_vjp(float2 f, float2 g) {
  const float u = f.x * f.x + f.y * f.y;
  if (!(u > 0.f)) return make_float2(0.f, 0.f);
  const float q = rsqrtf(sqrtf(u));  // u^-1/4
  const float c = 0.5f * q / u;      // (1/2) u^-5/4
  const float dot = g.x * f.x + g.y * f.y;
  return make_float2(q * g.x - c * f.x * dot, q * g.y - c * f.y * dot);
}

// f1 = cs1 x1 + co1 dnn1, f0 = cs0 x0 + co0 dnn0 (sebridge_v3, model.py:536-541); err = f1 - f0 or
// s(f1) - s(f0); loss = mean_b 0.5 sum |err|^2 -> loss_b[b] (one per utterance, atomics), d dnn1, d dnn0.
__global__ void ct_loss_kernel(const float2* dnn1, const float2* dnn0, const float2* x1, const float2* x0,
                               const float* coef /*[B][4] cs1 co1 cs0 co0*/, int HW, long long n, int B,
                               int sqrt_loss, double* loss_b, float2* g1, float2* g0) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int b = (int)(i / HW);
    const float cs1 = coef[b * 4], co1 = coef[b * 4 + 1], cs0 = coef[b * 4 + 2], co0 = coef[b * 4 + 3];
    const float2 d1 = dnn1[i], d0 = dnn0[i], a1 = x1[i], a0 = x0[i];
    const float2 f1 = make_float2(cs1 * a1.x + co1 * d1.x, cs1 * a1.y + co1 * d1.y);
    const float2 f0 = make_float2(cs0 * a0.x + co0 * d0.x, cs0 * a0.y + co0 * d0.y);
    float2 e, gf1, gf0;
    const float w = 1.f / (float)B;
    if (sqrt_loss) {
      const float2 s1 = sqrt_c(f1), s0 = sqrt_c(f0);
      e = make_float2(s1.x - s0.x, s1.y - s0.y);
      const float2 ge = make_float2(w * e.x, w * e.y);
      gf1 = sqrt_c_vjp(f1, ge);
      const float2 t0 = sqrt_c_vjp(f0, ge);
      gf0 = make_float2(-t0.x, -t0.y);
    } else {
      e = make_float2(f1.x - f0.x, f1.y - f0.y);
      gf1 = make_float2(w * e.x, w * e.y);
      gf0 = make_float2(-gf1.x, -gf1.y);
    }
    g1[i] = make_float2(co1 * gf1.x, co1 * gf1.y);
    g0[i] = make_float2(co0 * gf0.x, co0 * gf0.y);
    const double l = 0.5 * ((double)e.x * e.x + (double)e.y * e.y);
    const double lw = wave_sum_d(l);
    if ((threadIdx.x & 63) == 0) unsafeAtomicAdd(&loss_b[b], lw);
  }
}

// torch.optim.Adam (single-tensor algorithm, fp32, no weight decay / amsgrad):
//   m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2; p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)
// then torch_ema 0.3 ExponentialMovingAverage.update: s -= (1 - decay) (s - p).
// Work is split in chunks of 2048 elements; chunk i covers tensor tix[i] from element start[i].
struct AdamTensor {
  float* p; const float* g; float* m; float* v; float* ema; long long n;
};
__global__ __launch_bounds__(256) void adam_ema_kernel(const AdamTensor* ts, const int* tix, const long long* start,
                                                       float lr, float b1, float b2, float eps, float bc1, float bc2s,
                                                       float ema_decay) {
  const AdamTensor T = ts[tix[blockIdx.x]];
  const long long s0 = start[blockIdx.x];
  const long long s1 = s0 + 2048 < T.n ? s0 + 2048 : T.n;
  const float step = lr / bc1;
  for (long long i = s0 + threadIdx.x; i < s1; i += 256) {
    const float g = T.g ? T.g[i] : 0.f;
    float m = T.m[i];
    m = m + (1.f - b1) * (g - m);
    const float v = b2 * T.v[i] + (1.f - b2) * g * g;
    T.m[i] = m;
    T.v[i] = v;
    const float denom = sqrtf(v) / bc2s + eps;
    const float p = T.p[i] - step * (m / denom);
    T.p[i] = p;
    if (T.ema) T.ema[i] = T.ema[i] - (1.f - ema_decay) * (T.ema[i] - p);
  }
}

int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 65536); }

}  // namespace

extern "C" int snrse_conv_wgrad_x3(const float* dy, int Cout, const float* x0, int C0, const float* x1, int C1,
                                   int B, int H, int W, int ksize, float* dw, hipStream_t s) {
  if (!dy || !x0 || !dw || Cout <= 0 || C0 <= 0 || C1 < 0 || (C1 && !x1) || B <= 0 || H <= 0 || W <= 0 ||
      (ksize != 1 && ksize != 3) || Cout % 4 || C0 % 4 || C1 % 4)
    return SNRSE_EINVAL;
  const int Cin = C0 + C1;
  const int nci = (Cin + 63) / 64, nco = (Cout + 63) / 64;
  const long long nseg = (long long)B * H * ((W + WG_P - 1) / WG_P);
  long long splits = std::max<long long>(1, std::min<long long>(nseg, 2048 / (nci * nco) + 1));
  const int per = (int)((nseg + splits - 1) / splits);
  splits = (nseg + per - 1) / per;
  if (ksize == 3)
    hipLaunchKernelGGL(conv_wgrad_x3_kernel<3>, dim3(nci, nco, (unsigned)splits), dim3(256), 0, s, dy, Cout, x0, C0,
                       x1, C1, B, H, W, dw, per);
  else
    hipLaunchKernelGGL(conv_wgrad_x3_kernel<1>, dim3(nci, nco, (unsigned)splits), dim3(256), 0, s, dy, Cout, x0, C0,
                       x1, C1, B, H, W, dw, per);
  return (int)hipGetLastError();
}

extern "C" int snrse_conv_wgrad(const float* dy, int Cout, const float* x0, int C0, const float* x1, int C1, int B,
                                int H, int W, int ksize, float* dw, hipStream_t s) {
  if (!dy || !x0 || !dw || Cout <= 0 || C0 <= 0 || C1 < 0 || (C1 && !x1) || B <= 0 || H <= 0 || W <= 0 ||
      (ksize != 1 && ksize != 3))
    return SNRSE_EINVAL;
  const int Cin = C0 + C1;
  const int nci = (Cin + 63) / 64, nco = (Cout + 63) / 64;
  const long long nseg = (long long)B * H * ((W + WG_P - 1) / WG_P);
  long long splits = std::max<long long>(1, std::min<long long>(nseg, 2048 / (nci * nco) + 1));
  const int per = (int)((nseg + splits - 1) / splits);
  splits = (nseg + per - 1) / per;
  if (ksize == 3)
    hipLaunchKernelGGL(conv_wgrad_kernel<3>, dim3(nci, nco, (unsigned)splits), dim3(256), 0, s, dy, Cout, x0, C0, x1,
                       C1, B, H, W, dw, per);
  else
    hipLaunchKernelGGL(conv_wgrad_kernel<1>, dim3(nci, nco, (unsigned)splits), dim3(256), 0, s, dy, Cout, x0, C0, x1,
                       C1, B, H, W, dw, per);
  return (int)hipGetLastError();
}

extern "C" int snrse_chan_sum(const float* x, int B, int HW, int C, float* out_bc, float* out_c, float scale,
                              hipStream_t s) {
  if (!x || B <= 0 || HW <= 0 || C <= 0 || (!out_bc && !out_c)) return SNRSE_EINVAL;
  const int ppb = 256;
  hipLaunchKernelGGL(chan_sum_kernel, dim3((HW + ppb - 1) / ppb, B), dim3(256), 0, s, x, HW, C, ppb, out_bc, out_c,
                     scale);
  return (int)hipGetLastError();
}

extern "C" int snrse_gn_moments(const double* st0, int C0, const double* st1, int C1, int B, int HW, int groups,
                                float eps, float* mean, float* rstd, hipStream_t s) {
  if (!st0 || (C1 && !st1) || B <= 0 || groups <= 0 || (C0 + C1) % groups) return SNRSE_EINVAL;
  hipLaunchKernelGGL(gn_moments_kernel, dim3((B * groups + 255) / 256), dim3(256), 0, s, st0, C0, st1, C1, B, HW,
                     groups, eps, mean, rstd);
  return (int)hipGetLastError();
}

extern "C" int snrse_gn_backward(const float* x0, int C0, const float* x1, int C1, const float* dy, int B, int HW,
                                 int groups, const float* gamma, const float* beta, const float* mean,
                                 const float* rstd, int act, float* R, float* dx0, float* dx1, float* dgamma,
                                 float* dbeta, hipStream_t s) {
  const int C = C0 + C1;
  if (!x0 || (C1 && (!x1 || !dx1)) || !dy || !dx0 || !R || B <= 0 || HW <= 0 || C % groups) return SNRSE_EINVAL;
  SNRSE_RET(hipMemsetAsync(R, 0, sizeof(float) * 2 * (size_t)B * C, s));
  const int ppb = 128;
  hipLaunchKernelGGL(gn_bwd_reduce_kernel, dim3((HW + ppb - 1) / ppb, B), dim3(256), 0, s, x0, C0, x1, C1, dy, HW,
                     groups, gamma, beta, mean, rstd, act, ppb, R);
  SNRSE_LAUNCH_CHECK();
  const long long total = (long long)B * HW * C;
  hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, s, x0, C0, x1, C1, dy, HW, groups,
                     gamma, beta, mean, rstd, act, R, dx0, dx1, total);
  SNRSE_LAUNCH_CHECK();
  if (dgamma || dbeta)
    hipLaunchKernelGGL(gn_bwd_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, s, R, B, C, dgamma, dbeta);
  return (int)hipGetLastError();
}

extern "C" int snrse_bgemm(const float* A, long long sAb, long long sAm, long long sAk, const float* Bm,
                           long long sBb, long long sBk, long long sBn, float* C, long long sCb, long long sCm,
                           long long sCn, const float* bias, int batch, int M, int N, int K, float alpha, float beta,
                           hipStream_t s) {
  if (!A || !Bm || !C || batch <= 0 || M <= 0 || N <= 0 || K <= 0) return SNRSE_EINVAL;
  GemmArgs g{A, sAb, sAm, sAk, Bm, sBb, sBk, sBn, C, sCb, sCm, sCn, bias, M, N, K, alpha, beta};
  hipLaunchKernelGGL(bgemm_kernel, dim3((N + 63) / 64, (M + 63) / 64, batch), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

extern "C" int snrse_softmax_rows(const float* S, float* P, long long rows, int L, float scale, hipStream_t s) {
  if (!S || !P || rows <= 0 || L <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(64), 0, s, S, P, L, scale);
  return (int)hipGetLastError();
}

extern "C" int snrse_softmax_bwd_rows(const float* P, const float* dP, float* dS, long long rows, int L, float scale,
                                      hipStream_t s) {
  if (!P || !dP || !dS || rows <= 0 || L <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(softmax_bwd_rows_kernel, dim3((unsigned)rows), dim3(64), 0, s, P, dP, dS, L, scale);
  return (int)hipGetLastError();
}

extern "C" int snrse_silu_bwd(const float* x, const float* dy, float* dx, long long n, int accumulate, hipStream_t s) {
  if (!x || !dy || !dx || n <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(silu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, dy, dx, n, accumulate);
  return (int)hipGetLastError();
}

extern "C" int snrse_axpby(const float* x, float* y, long long n, float a, float b, hipStream_t s) {
  if (!x || !y || n <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n, a, b);
  return (int)hipGetLastError();
}

extern "C" int snrse_ct_perturb(const void* x, const void* y, const void* z, const float* wmix, const float* nscale,
                                int B, int HW, int transform, void* mu, void* xt, hipStream_t s) {
  if (!x || !y || !z || !wmix || !nscale || !mu || !xt || B <= 0 || HW <= 0) return SNRSE_EINVAL;
  const long long n = (long long)B * HW;
  hipLaunchKernelGGL(ct_perturb_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const float2*)x, (const float2*)y,
                     (const float2*)z, wmix, nscale, HW, n, transform, (float2*)mu, (float2*)xt);
  return (int)hipGetLastError();
}

extern "C" int snrse_ct_loss(const void* dnn1, const void* dnn0, const void* x1, const void* x0, const float* coef,
                             int B, int HW, int sqrt_loss, double* loss_b, void* g1, void* g0, hipStream_t s) {
  if (!dnn1 || !dnn0 || !x1 || !x0 || !coef || !loss_b || !g1 || !g0 || B <= 0 || HW <= 0 || HW % 64)
    return SNRSE_EINVAL;
  SNRSE_RET(hipMemsetAsync(loss_b, 0, sizeof(double) * B, s));
  const long long n = (long long)B * HW;
  hipLaunchKernelGGL(ct_loss_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const float2*)dnn1, (const float2*)dnn0,
                     (const float2*)x1, (const float2*)x0, coef, HW, n, B, sqrt_loss, loss_b, (float2*)g1,
                     (float2*)g0);
  return (int)hipGetLastError();
}

extern "C" int snrse_adam_ema(const void* tensors, const int* chunk_tensor, const long long* chunk_start, int nchunks,
                              float lr, float beta1, float beta2, float eps, float bias_corr1, float bias_corr2_sqrt,
                              float ema_decay, hipStream_t s) {
  if (!tensors || !chunk_tensor || !chunk_start || nchunks <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(adam_ema_kernel, dim3(nchunks), dim3(256), 0, s, (const AdamTensor*)tensors, chunk_tensor,
                     chunk_start, lr, beta1, beta2, eps, bias_corr1, bias_corr2_sqrt, ema_decay);
  return (int)hipGetLastError();
}

extern "C" int snrse_silu(const float* x, float* y, long long n, hipStream_t s) {
  if (!x || !y || n <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(silu_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return (int)hipGetLastError();
}

extern "C" int snrse_scale_rows(const float* x, const float* sc, float* y, int B, long long per, int recip,
                                hipStream_t s) {
  if (!x || !sc || !y || B <= 0 || per <= 0) return SNRSE_EINVAL;
  const long long n = (long long)B * per;
  hipLaunchKernelGGL(scale_rows_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, sc, y, per, n, recip);
  return (int)hipGetLastError();
}

extern "C" int snrse_gfp(const float* t, const float* Wg, int B, int nf, float* out, hipStream_t s) {
  if (!t || !Wg || !out || B <= 0 || nf <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(gfp_kernel, dim3(B), dim3(128), 0, s, t, Wg, nf, out);
  return (int)hipGetLastError();
}
