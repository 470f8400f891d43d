// Network front/back kernels of the score model and the SDE predictor/corrector update.
//
//   snrse_temb_mlp     GaussianFourierProjection(log t) -> Linear -> SiLU -> Linear
//                      (layerspp.py:32-43, ncsnpp.py:256-275); one block per utterance.
//   snrse_temb_dense   all 49 ResBlock Dense_0(SiLU(temb)) projections in one launch
//                      (layerspp.py:264-265), weights concatenated on the host.
//   snrse_input_pack   complex (x, y) -> 4 real channels (ncsnpp.py:253-254), unrolled over
//                      the 3x3 taps of the input conv (im2col, 36 of 64 channels used) so the
//                      first conv (ncsnpp.py:285) is a K=64 GEMM on MFMA; also writes the
//                      4-channel input pyramid (ncsnpp.py:282) in f32.
//   snrse_score_update output head + preconditioning + one SDE step, fused:
//                      dnn = output_layer(pyr / t) as complex (ncsnpp.py:398-404),
//                      score = -dnn (model_type 'bbed', model.py:488-489) or
//                      c_skip x + c_out dnn (sebridge*, model.py:536-541),
//                      x_mean = a x + by y + c score,  x = x_mean + s z  with z complex
//                      normal (each part N(0,1/2), torch.randn_like on complex64), which covers
//                      ReverseDiffusionPredictor (predictors.py:75-80), AnnealedLangevinDynamics
//                      (correctors.py:69-81) and EulerMaruyamaPredictor (predictors.py:46-52).
//                      z is read from a tensor (parity mode) or drawn in-kernel (Philox4x32-10).
#include "common.h"

#include <algorithm>

namespace {

constexpr float kTwoPi = 6.28318530717958647692f;

// snrse_temb_mlp: one block (8 waves) per utterance.  Each wave owns 64 output rows in chunks of 16: a row's
// weights are read as one coalesced 1-2 KB line set (lane = 4 or 8 consecutive inputs), the 16 per-lane partial
// dot products are reduced by bfly_sum.  Every block streams all of W1 and W2 through its CU (~44 us at B = 32);
// the network executor takes the row-parallel pair snrse_temb_gfp_dense + snrse_temb_dense instead.
__global__ __launch_bounds__(512) void temb_mlp_kernel(const float* t, const float* Wg, const float* W1,
                                                       const float* b1, const float* W2, const float* b2,
                                                       float* temb, int nf) {
  // nf = 128: e[256], h[512], out[512]
  __shared__ __attribute__((aligned(16))) float e[256];
  __shared__ __attribute__((aligned(16))) float h[512];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float lt = logf(t[b]);
  if (tid < nf) {
    const float pr = lt * Wg[tid] * kTwoPi;
    e[tid] = sinf(pr);
    e[nf + tid] = cosf(pr);
  }
  __syncthreads();
  {
    const f32x4 ev = *(const f32x4*)(e + 4 * lane);  // 2 nf = 256 = 64 lanes x 4
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j0 = wid * 64 + c * 16;
      float pp[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) pp[r] = dot4(*(const f32x4*)(W1 + (size_t)(j0 + r) * 2 * nf + 4 * lane), ev);
      const float v = bfly_sum<16>(pp, lane);
      if (lane < 16) h[j0 + lane] = silu_exact(v + b1[j0 + lane]);
    }
  }
  __syncthreads();
  {
    const f32x4 h0 = *(const f32x4*)(h + 8 * lane), h1 = *(const f32x4*)(h + 8 * lane + 4);  // 4 nf = 512
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j0 = wid * 64 + c * 16;
      float pp[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* w = W2 + (size_t)(j0 + r) * 4 * nf + 8 * lane;
        pp[r] = dot4(*(const f32x4*)w, h0) + dot4(*(const f32x4*)(w + 4), h1);
      }
      const float v = bfly_sum<16>(pp, lane);
      if (lane < 16) temb[(size_t)b * 4 * nf + j0 + lane] = v + b2[j0 + lane];
    }
  }
}

// Row-parallel dense layer over a batch of <= 32 utterances, the time-embedding path (ncsnpp.py:256-275,
// layerspp.py:264-265):  out[b][r] = act_out(bias[r] + sum_d W[r][d] * in_b[d]),  D <= 512, D % 4 == 0, where in_b is
//   IN 0: x[b] as given, IN 1: silu(x[b]) (the Dense_0 input), IN 2: the Gaussian-Fourier projection of t[b]
//   ([sin, cos](2 pi log(t) W_gfp), nf = D / 2 frequencies); act_out = silu for OUT 1.
// Block = 4 waves; the [32][SR] input table is staged in LDS.  A wave owns 16 weight rows and computes all 32
// utterances as two 16 x 16 tiles on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32): per 16 inputs a lane loads 4
// consecutive weights of its row and 4 table entries of its utterance, and the 4 MFMAs take component q, so the
// tile's K index g = lane / 16 stands for input 4 g + q on both operands.  (Wave-wide shuffle reductions ran
// 20-27 us per launch on a chain of ~500 waits, a block per utterance ~44 us, a lane-per-row table ~68 us;
// profiles/r05a..r05l dispatch shapes.)
constexpr int kDenseSR = 516;  // LDS row stride (floats): 16 utterance rows x 16 B reads hit distinct banks
template <int IN, int OUT>
__global__ __launch_bounds__(256) void temb_dense_kernel(const float* x, const float* t, const float* Wg,
                                                         const float* W, const float* bias, float* out, int B, int R,
                                                         int D) {
  extern __shared__ __attribute__((aligned(16))) float st[];  // [32][kDenseSR] input rows, zero beyond (B, D)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // staging: all of a thread's loads issued before any is used
  if constexpr (IN == 2) {
    const int nf = D >> 1;
    for (int i = tid; i < 32 * 128; i += 256) {
      const int bb = i >> 7, d = (i & 127) * 4;
      if (bb >= B || d >= D) *(f32x4*)(st + bb * kDenseSR + d) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll 4
    for (int i = tid; i < B * nf; i += 256) {
      const int bb = i / nf, k = i - bb * nf;
      float sn, cs;
      sincosf(logf(t[bb]) * Wg[k] * kTwoPi, &sn, &cs);
      st[bb * kDenseSR + k] = sn;
      st[bb * kDenseSR + nf + k] = cs;
    }
  } else {
    constexpr int NQ = 32 * 512 / 4 / 256;  // f32x4 pieces per thread
    f32x4 v[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = tid + 256 * j, bb = q >> 7, d = (q & 127) * 4;
      v[j] = (bb < B && d < D) ? *(const f32x4*)(x + (size_t)bb * D + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = tid + 256 * j, bb = q >> 7, d = (q & 127) * 4;
      f32x4 a = v[j];
      if constexpr (IN == 1) {
        if (bb < B && d < D) {
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] = silu_exact(a[e]);
        }
      }
      *(f32x4*)(st + bb * kDenseSR + d) = a;
    }
  }
  __syncthreads();
  const int r0 = (blockIdx.x * 4 + wid) * 16;
  if (r0 >= R) return;  // wave-uniform, no barrier follows
  const int n = lane & 15, g = lane >> 4;
  const float* wrow = W + (size_t)min(r0 + n, R - 1) * D;
  const float* s0 = st + n * kDenseSR + 4 * g;
  const float* s1 = st + (16 + n) * kDenseSR + 4 * g;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  constexpr int KB = 8;  // 16-input steps whose weight loads are in flight together
  for (int k0 = 0; k0 < D; k0 += 16 * KB) {
    f32x4 bw[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int k = k0 + 16 * u + 4 * g;
      bw[u] = k < D ? *(const f32x4*)(wrow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int k = k0 + 16 * u;  // (table columns past D are zero, rows stay inside the 512-column table)
      const f32x4 a0 = k < D ? *(const f32x4*)(s0 + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 a1 = k < D ? *(const f32x4*)(s1 + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[q], bw[u][q], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[q], bw[u][q], acc1, 0, 0, 0);
      }
    }
  }
  // acc: D[utterance 4 g + j (+16)][row r0 + n]
  const int r = r0 + n;
  if (r < R) {
    const float bi = bias[r];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b0 = 4 * g + j, b1 = 16 + 4 * g + j;
      const float y0 = acc0[j] + bi, y1 = acc1[j] + bi;
      if (b0 < B) out[(size_t)b0 * R + r] = OUT == 1 ? silu_exact(y0) : y0;
      if (b1 < B) out[(size_t)b1 * R + r] = OUT == 1 ? silu_exact(y1) : y1;
    }
  }
}

template <int IN, int OUT>
int launch_dense(const float* x, const float* t, const float* Wg, const float* W, const float* bias, float* out, int B,
                 int R, int D, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)temb_dense_kernel<IN, OUT>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 32 * kDenseSR * 4);
  SNRSE_RET(attr);
  const int rows_per_block = 4 * 16;
  for (int b0 = 0; b0 < B; b0 += 32) {  // the LDS table holds 32 utterances
    const int nb = std::min(32, B - b0);
    hipLaunchKernelGGL((temb_dense_kernel<IN, OUT>), dim3((R + rows_per_block - 1) / rows_per_block), dim3(256),
                       sizeof(float) * 32 * kDenseSR, s, x ? x + (size_t)b0 * D : nullptr, t ? t + b0 : nullptr, Wg, W,
                       bias, out + (size_t)b0 * R, nb, R, D);
    SNRSE_LAUNCH_CHECK();
  }
  return 0;
}

// One lane per 16-byte chunk of a pixel's 64-channel im2col row (NCH = 64 / VEC chunks per pixel),
// so a wave's stores are contiguous 16-B vectors; chunk k holds channels k*VEC .. k*VEC+VEC-1,
// i.e. taps (k*VEC)/4 .. of the 4 real input channels (x.re, x.im, y.re, y.im), zero past tap 8.
template <typename T>
__global__ __launch_bounds__(256) void input_pack_kernel(const float2* x, const float2* y, int H, int W,
                                                         T* col, float* pyr, int total) {
  constexpr int VEC = 16 / sizeof(T), NCH = 64 / VEC;
  const long long gi = (long long)blockIdx.x * 256 + threadIdx.x;
  const int p = (int)(gi / NCH), k = (int)(gi % NCH);
  if (p >= total) return;
  const int HW = H * W;
  const int b = p / HW, rem = p - b * HW, h = rem / W, w = rem - (rem / W) * W;
  if (k == 0) {
    const float2 xv = x[p], yv = y[p];
    *(float4*)(pyr + (size_t)p * 4) = make_float4(xv.x, xv.y, yv.x, yv.y);
  }
  float v[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) v[i] = 0.f;
#pragma unroll
  for (int jt = 0; jt < VEC / 4; ++jt) {
    const int tap = (k * VEC) / 4 + jt;
    if (tap >= 9) break;
    const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
    if (hh < 0 || hh >= H || ww < 0 || ww >= W) continue;
    const size_t q = (size_t)b * HW + (size_t)hh * W + ww;
    const float2 a = x[q], c = y[q];
    v[jt * 4 + 0] = a.x; v[jt * 4 + 1] = a.y; v[jt * 4 + 2] = c.x; v[jt * 4 + 3] = c.y;
  }
  u32x4 o;
  if constexpr (sizeof(T) == 2) {
    o = pack8<T>(v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __float_as_uint(v[i]);
  }
  *(u32x4*)(col + (size_t)p * 64 + k * VEC) = o;
}

// ---- fused input conv (16-bit T): complex (x, y) -> h = conv3x3(4 -> 128) + bias, NHWC T -------
// (ncsnpp.py:253-254, 282-285).  Replaces input_pack's 64-channel im2col round trip through HBM +
// a K=64 GEMM: the 36 products per output come from x / y directly (cache-resident neighbours),
// so the launch is bound by the 256 B/pixel output store.  MFMA 16x16x32 with A = the packed
// weights [128 co][64 k] (k = tap * 4 + {x.re, x.im, y.re, y.im}, 36..63 zero) and B = the
// pixels' tap values, so D = [co][px]: each lane holds 4 consecutive channels of one pixel; a
// row swap pairs them into 8 (16-byte stores, a pixel's 256 B completed by the same wave).  GroupNorm statistics of h:
// f32 per lane over the workgroup's 16 tiles, DPP row sums, a fixed-order fold of the 4 waves in
// LDS, one f64 atomic pair per channel per workgroup (slot = blockIdx & 15).  Also writes the f32 input pyramid.
// Contract: W % 64 == 0, (H * W / 64) % 16 == 0 (a workgroup's 16 tiles lie in one image).
constexpr int IC_TPW = 4;  // 64-px tiles per wave
#ifndef SNRSE_IC_NT
#define SNRSE_IC_NT 0  // non-temporal stores of the 256-B-per-pixel activation: faster in an isolated
                         // micro-bench (420 -> 330 us), slower inside the network (383-388 -> 450 us per launch,
                         // profiles/r02bd_input_conv_nt_insitu.log): off
#endif
SNRSE_DEV f32x4 mfma_bf16_16x16x32(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a), __builtin_bit_cast(bf16x8_mfma, b),
                                                 c, 0, 0, 0);
}
template <int CTRL>
SNRSE_DEV float ic_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
SNRSE_DEV float ic_row_sum16(float v) {
  v += ic_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += ic_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += ic_dpp<0x141>(v);  // row_half_mirror
  v += ic_dpp<0x140>(v);  // row_mirror
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void input_conv_kernel(const float2* __restrict__ x, const float2* __restrict__ y,
                                                         int H, int W, const T* __restrict__ wgt,
                                                         const float* __restrict__ bias, T* __restrict__ out,
                                                         float* __restrict__ pyr, double* __restrict__ stats) {
  __shared__ float s_st[4][128 * 2];  // per-wave channel sums: fixed-order fold, no LDS atomics
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, lr = lane & 15;
  u32x4 wf[8][2];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) wf[j][s] = *(const u32x4*)(wgt + (16 * j + lr) * 64 + 32 * s + 8 * g);
  float bv[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 b4 = *(const f32x4*)(bias + 16 * j + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = b4[e];
  }
  float s1[8][4], s2[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[j][e] = 0.f; s2[j][e] = 0.f; }
  const int HW = H * W, tpr = W / 64;
  const long long tile0 = ((long long)blockIdx.x * 4 + wid) * IC_TPW;
  const int b = (int)(((long long)blockIdx.x * 16 * 64) / HW);
  const size_t img = (size_t)b * HW;
  // this lane's taps: 2g, 2g + 1 (K-step 0) and 8 (K-step 1, g == 0 only)
  int tdy[3], tdx[3];
  bool tuse[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int tap = u < 2 ? 2 * g + u : 8;
    tuse[u] = u < 2 || g == 0;
    tdy[u] = tap / 3 - 1;
    tdx[u] = tap % 3 - 1;
  }
  // 16 pixel blocks of 16 px per wave, software-pipelined: block q + 1's neighbour loads are
  // issued before block q's stores, so waiting for them never waits for those stores
  // (vmcnt counts stores too on gfx950)
  auto load_blk = [&](int q, float2 (&lx)[3], float2 (&ly)[3], bool (&ok)[3]) {
    const long long tile = tile0 + (q >> 2);
    const int rem = (int)(tile - (long long)b * (HW / 64));
    const int h = rem / tpr, w = (rem - h * tpr) * 64 + 16 * (q & 3) + lr;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int hh = h + tdy[u], ww = w + tdx[u];
      ok[u] = tuse[u] && hh >= 0 && hh < H && ww >= 0 && ww < W;
      const size_t qq = img + (ok[u] ? (size_t)hh * W + ww : (size_t)h * W + w);
      lx[u] = x[qq];
      ly[u] = y[qq];
    }
  };
  float2 cx[3], cy[3];
  bool cok[3];
  load_blk(0, cx, cy, cok);
  for (int q = 0; q < 4 * IC_TPW; ++q) {
    float2 nx[3], ny[3];
    bool nok[3];
    if (q + 1 < 4 * IC_TPW) load_blk(q + 1, nx, ny, nok);
    const long long tile = tile0 + (q >> 2);
    const int rem = (int)(tile - (long long)b * (HW / 64));
    const int h = rem / tpr, w = (rem - h * tpr) * 64 + 16 * (q & 3) + lr;
    u32x4 pf[2];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const float2 a = cok[u] ? cx[u] : make_float2(0.f, 0.f);
      const float2 c = cok[u] ? cy[u] : make_float2(0.f, 0.f);
      const int sl = u < 2 ? 0 : 1, hw_ = u < 2 ? 2 * u : 0;
      pf[sl][hw_] = H16<T>::pack(a.x, a.y);
      pf[sl][hw_ + 1] = H16<T>::pack(c.x, c.y);
    }
    pf[1][2] = 0u;
    pf[1][3] = 0u;
    if (g == 2)  // tap 4 = the pixel itself: the input pyramid
      *(float4*)(pyr + (img + (size_t)h * W + w) * 4) = make_float4(cx[0].x, cx[0].y, cy[0].x, cy[0].y);
    // channel blocks (2jp, 2jp + 1) are exchanged between DPP rows (v_permlane16_swap) so each lane
    // stores 8 consecutive channels: 16-B stores, 64 contiguous bytes of a pixel per instruction
    T* orow = out + (img + (size_t)h * W + w) * 128 + 8 * (g >> 1);
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      uint32_t pk[2][2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int j = 2 * jp + hh;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        acc = H16<T>::mfma(wf[j][0], pf[0], acc);
        acc = H16<T>::mfma(wf[j][1], pf[1], acc);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[e] + bv[j][e];
          s1[j][e] += v[e];
          s2[j][e] = fmaf(v[e], v[e], s2[j][e]);
        }
        pk[hh][0] = H16<T>::pack(v[0], v[1]);
        pk[hh][1] = H16<T>::pack(v[2], v[3]);
      }
      const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      const u32x4 o = {r0[0], r1[0], r0[1], r1[1]};
      if (SNRSE_IC_NT) __builtin_nontemporal_store(o, (u32x4*)(orow + 16 * (2 * jp + (g & 1))));
      else *(u32x4*)(orow + 16 * (2 * jp + (g & 1))) = o;
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      cx[u] = nx[u];
      cy[u] = ny[u];
      cok[u] = nok[u];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = ic_row_sum16(s1[j][e]), q = ic_row_sum16(s2[j][e]);
      if (lr == 0) {  // one lane per (wave, channel)
        s_st[wid][(16 * j + 4 * g + e) * 2] = a;
        s_st[wid][(16 * j + 4 * g + e) * 2 + 1] = q;
      }
    }
  __syncthreads();
  const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  const float tot = (s_st[0][tid] + s_st[1][tid]) + (s_st[2][tid] + s_st[3][tid]);
  unsafeAtomicAdd(&stats[stat_idx(b, slot, tid >> 1, 128) + (tid & 1)], (double)tot);
}

// ---- the same input conv with the workgroup's input rows staged in LDS (W <= 1024) ----------------------------
// A workgroup's 16 tiles (1024 consecutive pixels of one image) read their 3x3 neighbours from the image rows they
// span plus one above and below, loaded into LDS in one burst at the start (16 B per pixel: x.re, x.im, y.re, y.im),
// so the per-block neighbour loads of input_conv_kernel -- one block of prefetch, an HBM latency exposed per 16-px
// block -- become LDS reads, and the launch is bound by its 256 B/pixel of output stores.  Same MFMA / epilogue /
// statistics as input_conv_kernel.
// ICH: output channels per wave (128: a wave owns 4 of the workgroup's 16 tiles; 64: waves (2 s, 2 s + 1) share pixel
// stream s = 8 tiles and split the channels -- half the weight / bias / statistics registers, so more waves per SIMD
// hide the store and LDS latency)
// SST (ICH 128): the block's 16 px x 128 ch output (4 KB, contiguous in NHWC) goes through a per-wave LDS stage
// (16-B chunk c of pixel p at p * 256 + (c ^ (p & 15)) * 16: conflict-free 8-B writes and 16-B reads) and out as 4
// fully contiguous 1-KB wave stores, instead of 4 stores of 64-B pieces of 16 pixels each
template <typename T, int ICH, bool SST = false>
__global__ __launch_bounds__(256) void input_conv_lds_kernel(const float2* __restrict__ x, const float2* __restrict__ y,
                                                             int H, int W, const T* __restrict__ wgt,
                                                             const float* __restrict__ bias, T* __restrict__ out,
                                                             float* __restrict__ pyr, double* __restrict__ stats) {
  constexpr int NJ = ICH / 16, NS = 128 / ICH;  // channel blocks per wave; waves per pixel stream
  constexpr int TPS = 16 / (4 / NS);            // tiles per pixel stream (4 with ICH 128, 8 with 64)
  extern __shared__ __attribute__((aligned(16))) char ic_smem[];
  __shared__ float s_st[4][128 * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, lr = lane & 15;
  const int ps = wid / NS, jb = (wid % NS) * NJ;  // pixel stream, first channel block of this wave
  const int HW = H * W, tpr = W / 64;
  const long long p0 = (long long)blockIdx.x * 1024;  // first pixel of the workgroup (16 tiles x 64 px)
  const int b = (int)(p0 / HW);
  const size_t img = (size_t)b * HW;
  const int q0 = (int)(p0 - (long long)b * HW);
  const int r0 = q0 / W - 1, nrows = (q0 + 1023) / W + 2 - r0;  // staged image rows r0 .. r0 + nrows - 1
  // ---- stage: pixel pairs (2 x float4 loads -> 2 x 16-B LDS rows), rows outside the image zero
  float4* st = (float4*)ic_smem;
  const int npair = nrows * W / 2;
  for (int i = tid; i < npair; i += 256) {
    const int rr = (2 * i) / W, cc = 2 * i - rr * W, ih = r0 + rr;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
    if ((unsigned)ih < (unsigned)H) {
      a = *(const float4*)(x + img + (size_t)ih * W + cc);
      c = *(const float4*)(y + img + (size_t)ih * W + cc);
    }
    st[2 * i] = make_float4(a.x, a.y, c.x, c.y);
    st[2 * i + 1] = make_float4(a.z, a.w, c.z, c.w);
  }
  // output stage of this wave (SST): after the input rows of the largest launch ((1023 / W + 4) W 16 B)
  char* const ostg = ic_smem + (size_t)(1023 / W + 4) * W * 16 + wid * 4096;
  u32x4 wf[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) wf[j][s] = *(const u32x4*)(wgt + (16 * (jb + j) + lr) * 64 + 32 * s + 8 * g);
  float bv[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const f32x4 b4 = *(const f32x4*)(bias + 16 * (jb + j) + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = b4[e];
  }
  float s1[NJ][4], s2[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[j][e] = 0.f; s2[j][e] = 0.f; }
  int tdy[3], tdx[3];
  bool tuse[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int tap = u < 2 ? 2 * g + u : 8;
    tuse[u] = u < 2 || g == 0;
    tdy[u] = tap / 3 - 1;
    tdx[u] = tap % 3 - 1;
  }
  __syncthreads();
  const int tile0 = q0 / 64 + ps * TPS;  // this pixel stream's first 64-px tile within the image
  for (int q = 0; q < 4 * TPS; ++q) {
    const int tile = tile0 + (q >> 2);
    const int h = tile / tpr, w = (tile - h * tpr) * 64 + 16 * (q & 3) + lr;
    float4 v[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int hh = h + tdy[u], ww = w + tdx[u];
      const bool ok = tuse[u] && (unsigned)ww < (unsigned)W;  // (rows: staged, zero outside the image)
      const float4 t = st[(hh - r0) * W + (ok ? ww : w)];
      v[u] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    u32x4 pf[2];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int sl = u < 2 ? 0 : 1, hw_ = u < 2 ? 2 * u : 0;
      pf[sl][hw_] = H16<T>::pack(v[u].x, v[u].y);
      pf[sl][hw_ + 1] = H16<T>::pack(v[u].z, v[u].w);
    }
    pf[1][2] = 0u;
    pf[1][3] = 0u;
    if (g == 2 && jb == 0)  // tap 4 = the pixel itself: the input pyramid (written by one wave of the stream)
      *(float4*)(pyr + (img + (size_t)h * W + w) * 4) = v[0];
    T* orow = out + (img + (size_t)h * W + w) * 128 + 8 * (g >> 1);
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
#pragma unroll
    for (int jp = 0; jp < NJ / 2; ++jp) {
      uint32_t pk[2][2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int j = 2 * jp + hh;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        acc = H16<T>::mfma(wf[j][0], pf[0], acc);
        acc = H16<T>::mfma(wf[j][1], pf[1], acc);
        float vv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vv[e] = acc[e] + bv[j][e];
          s1[j][e] += vv[e];
          s2[j][e] = fmaf(vv[e], vv[e], s2[j][e]);
        }
        pk[hh][0] = H16<T>::pack(vv[0], vv[1]);
        pk[hh][1] = H16<T>::pack(vv[2], vv[3]);
        if constexpr (SST)  // channels 16 j + 4 g .. + 3 of pixel lr: half (g & 1) of 16-B chunk 2 j + (g >> 1)
          *(u32x2*)(ostg + lr * 256 + (((2 * j + (g >> 1)) ^ lr) << 4) + (g & 1) * 8) = u32x2{pk[hh][0], pk[hh][1]};
      }
      if constexpr (SST) continue;
      const auto a0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto a1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      const u32x4 o = {a0[0], a1[0], a0[1], a1[1]};
      *(u32x4*)(orow + 16 * (jb + 2 * jp + (g & 1))) = o;
    }
    if constexpr (SST) {  // the block's 4 KB: pixel 4 k + (lane >> 4), 16-B chunk lane & 15, contiguous per wave store
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      T* ob = out + (img + (size_t)h * W + (w - lr)) * 128;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int pp = 4 * k + (lane >> 4), c = lane & 15;
        const u32x4 o = *(const u32x4*)(ostg + pp * 256 + ((c ^ pp) << 4));
        *(u32x4*)(ob + pp * 128 + c * 8) = o;
      }
      asm volatile("" ::: "memory");  // (the next block's stage writes follow these reads in the wave's LDS order)
    }
  }
  // statistics: s_st[pixel stream][channel][2] (each channel written by one wave per stream), then a fixed-order
  // fold over the 4 / NS streams
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = ic_row_sum16(s1[j][e]), qq = ic_row_sum16(s2[j][e]);
      if (lr == 0) {
        s_st[ps][(16 * (jb + j) + 4 * g + e) * 2] = a;
        s_st[ps][(16 * (jb + j) + 4 * g + e) * 2 + 1] = qq;
      }
    }
  __syncthreads();
  const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  float tot = s_st[0][tid];
#pragma unroll
  for (int k = 1; k < 4 / NS; ++k) tot += s_st[k][tid];
  if (NS == 1) tot = (s_st[0][tid] + s_st[1][tid]) + (s_st[2][tid] + s_st[3][tid]);  // (the streaming kernel's order)
  unsafeAtomicAdd(&stats[stat_idx(b, slot, tid >> 1, 128) + (tid & 1)], (double)tot);
}

// ---- the fp32x3 parity mode's input conv: the same LDS staging, split-bf16 products, fp32 output --------------
// (replaces input_pack's fp32 im2col round trip through HBM + the split GEMM on it.)  Each tap value is split as the
// split GEMMs split activations (hi = bf16(x), lo = bf16(x - hi)), the packed weights come pre-split per 32-element
// K tile (ops.split_weight: 32 hi then 32 lo), and every 16x16x32 block accumulates w_hi.x_hi + w_lo.x_hi + w_hi.x_lo.
// Channels split over wave pairs as input_conv_lds_kernel<64> (4 channel blocks per wave); a lane stores its 4
// consecutive f32 channels of one pixel as one 16-B vector.  W <= 1024, as the bf16 form.
__global__ __launch_bounds__(256) void input_conv_lds_x3_kernel(const float2* __restrict__ x,
                                                                const float2* __restrict__ y, int H, int W,
                                                                const bf16_t* __restrict__ wgt,
                                                                const float* __restrict__ bias, float* __restrict__ out,
                                                                float* __restrict__ pyr, double* __restrict__ stats) {
  constexpr int NJ = 4, TPS = 8;
  extern __shared__ __attribute__((aligned(16))) char ic_smem[];
  __shared__ float s_st[2][128 * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, lr = lane & 15;
  const int ps = wid >> 1, jb = (wid & 1) * NJ;
  const int HW = H * W, tpr = W / 64;
  const long long p0 = (long long)blockIdx.x * 1024;
  const int b = (int)(p0 / HW);
  const size_t img = (size_t)b * HW;
  const int q0 = (int)(p0 - (long long)b * HW);
  const int r0 = q0 / W - 1, nrows = (q0 + 1023) / W + 2 - r0;
  float4* st = (float4*)ic_smem;
  const int npair = nrows * W / 2;
  for (int i = tid; i < npair; i += 256) {
    const int rr = (2 * i) / W, cc = 2 * i - rr * W, ih = r0 + rr;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
    if ((unsigned)ih < (unsigned)H) {
      a = *(const float4*)(x + img + (size_t)ih * W + cc);
      c = *(const float4*)(y + img + (size_t)ih * W + cc);
    }
    st[2 * i] = make_float4(a.x, a.y, c.x, c.y);
    st[2 * i + 1] = make_float4(a.z, a.w, c.z, c.w);
  }
  u32x4 wh[NJ][2], wl[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16_t* wr = wgt + (16 * (jb + j) + lr) * 128 + 64 * s + 8 * g;
      wh[j][s] = *(const u32x4*)wr;
      wl[j][s] = *(const u32x4*)(wr + 32);
    }
  f32x4 bv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bv[j] = *(const f32x4*)(bias + 16 * (jb + j) + 4 * g);
  float s1[NJ][4], s2[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[j][e] = 0.f; s2[j][e] = 0.f; }
  int tdy[3], tdx[3];
  bool tuse[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int tap = u < 2 ? 2 * g + u : 8;
    tuse[u] = u < 2 || g == 0;
    tdy[u] = tap / 3 - 1;
    tdx[u] = tap % 3 - 1;
  }
  __syncthreads();
  const int tile0 = q0 / 64 + ps * TPS;
  for (int q = 0; q < 4 * TPS; ++q) {
    const int tile = tile0 + (q >> 2);
    const int h = tile / tpr, w = (tile - h * tpr) * 64 + 16 * (q & 3) + lr;
    float4 v[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int hh = h + tdy[u], ww = w + tdx[u];
      const bool ok = tuse[u] && (unsigned)ww < (unsigned)W;
      const float4 t = st[(hh - r0) * W + (ok ? ww : w)];
      v[u] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    u32x4 ph[2], pl[2];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int sl = u < 2 ? 0 : 1, hw_ = u < 2 ? 2 * u : 0;
      const float e4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t hi = pack_bf16x2(e4[2 * k], e4[2 * k + 1]);
        ph[sl][hw_ + k] = hi;
        pl[sl][hw_ + k] = pack_bf16x2(e4[2 * k] - __uint_as_float(hi << 16),
                                      e4[2 * k + 1] - __uint_as_float(hi & 0xffff0000u));
      }
    }
    ph[1][2] = ph[1][3] = pl[1][2] = pl[1][3] = 0u;
    if (g == 2 && jb == 0) *(float4*)(pyr + (img + (size_t)h * W + w) * 4) = v[0];
    float* orow = out + (img + (size_t)h * W + w) * 128 + 4 * g;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        acc = mfma_bf16_16x16x32(wh[j][s], ph[s], acc);
        acc = mfma_bf16_16x16x32(wl[j][s], ph[s], acc);
        acc = mfma_bf16_16x16x32(wh[j][s], pl[s], acc);
      }
      const f32x4 o = acc + bv[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[j][e] += o[e];
        s2[j][e] = fmaf(o[e], o[e], s2[j][e]);
      }
      *(f32x4*)(orow + 16 * (jb + j)) = o;
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = ic_row_sum16(s1[j][e]), qq = ic_row_sum16(s2[j][e]);
      if (lr == 0) {
        s_st[ps][(16 * (jb + j) + 4 * g + e) * 2] = a;
        s_st[ps][(16 * (jb + j) + 4 * g + e) * 2 + 1] = qq;
      }
    }
  __syncthreads();
  const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  unsafeAtomicAdd(&stats[stat_idx(b, slot, tid >> 1, 128) + (tid & 1)], (double)(s_st[0][tid] + s_st[1][tid]));
}

// ---- Philox4x32-10 -> Box-Muller complex normals -------------------------------------
SNRSE_DEV uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
SNRSE_DEV u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    const uint32_t lo0 = mulhilo(0xD2511F53u, c[0], hi0);
    const uint32_t lo1 = mulhilo(0xCD9E8D57u, c[2], hi1);
    c = u32x4{hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
SNRSE_DEV float u01(uint32_t v) { return ((v >> 8) + 0.5f) * (1.0f / 16777216.0f); }  // (0,1)

SNRSE_DEV float2 cnormal(uint64_t seed, uint64_t ctr) {
  const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x5eedu, 0u}, (uint32_t)seed,
                         (uint32_t)(seed >> 32));
  const float rad = sqrtf(-2.0f * logf(u01(r[0])));
  float sn, cs;
  sincosf(kTwoPi * u01(r[1]), &sn, &cs);
  // complex normal with E|z|^2 = 1: each part N(0, 1/2)
  return make_float2(rad * cs * 0.70710678118654752f, rad * sn * 0.70710678118654752f);
}

struct StepCoef {
  float a, by, c, s;  // x_mean = a x + by y + c score ; x = x_mean + s z
};

template <typename TP>
__global__ __launch_bounds__(256) void score_update_kernel(
    const TP* pyr, const float* out_w, const float* out_b, const float* t, int score_mode, int HW, int total,
    const float2* x, const float2* y, const float2* noise, uint64_t seed, uint64_t offset, const float* coef,
    float2* x_out, float2* xmean_out, float2* score_out) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const int b = p / HW;
  const float tb = t[b];
  const float inv_t = 1.0f / tb;
  float h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) h[i] = Elem<TP>::to_f(pyr[(size_t)p * 4 + i]) * inv_t;
  float dre = out_b[0], dim = out_b[1];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dre = fmaf(out_w[i], h[i], dre);
    dim = fmaf(out_w[4 + i], h[i], dim);
  }
  const float2 xv = x[p];
  float2 sc;
  if (score_mode == 0) {  // bbed: score = -dnn
    sc = make_float2(-dre, -dim);
  } else {  // sebridge preconditioning, eps = 0.001, sigma_data = 0.5
    const float te = tb - 0.001f;
    const float c_skip = 0.25f / (te * te + 0.25f);
    const float c_out = (0.5f * te) / sqrtf(0.25f + tb * tb);
    sc = make_float2(c_skip * xv.x + c_out * dre, c_skip * xv.y + c_out * dim);
  }
  if (score_out) score_out[p] = sc;
  if (!x_out) return;
  const float* cf = coef + 4 * b;
  const float2 yv = y ? y[p] : make_float2(0.f, 0.f);
  float2 xm;
  xm.x = cf[0] * xv.x + cf[1] * yv.x + cf[2] * sc.x;
  xm.y = cf[0] * xv.y + cf[1] * yv.y + cf[2] * sc.y;
  if (xmean_out) xmean_out[p] = xm;
  float2 z = noise ? noise[p] : cnormal(seed, offset + (uint64_t)p);
  x_out[p] = make_float2(xm.x + cf[3] * z.x, xm.y + cf[3] * z.y);
}

// x = a x + by y + s z (prior sampling, sdes.py:225-232 / 298-304)
__global__ __launch_bounds__(256) void axpby_noise_kernel(const float2* x, const float2* y, const float2* noise,
                                                          uint64_t seed, uint64_t offset, const float* coef,
                                                          int HW, int total, float2* out) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const float* cf = coef + 4 * (p / HW);
  const float2 xv = x ? x[p] : make_float2(0.f, 0.f);
  const float2 yv = y ? y[p] : make_float2(0.f, 0.f);
  const float2 z = noise ? noise[p] : cnormal(seed, offset + (uint64_t)p);
  out[p] = make_float2(cf[0] * xv.x + cf[1] * yv.x + cf[3] * z.x, cf[0] * xv.y + cf[1] * yv.y + cf[3] * z.y);
}

// generic step for an arbitrary score tensor: x_mean = a x + by y + c score; x = x_mean + s z
__global__ __launch_bounds__(256) void sde_update_kernel(const float2* x, const float2* y, const float2* score,
                                                         const float2* noise, uint64_t seed, uint64_t offset,
                                                         const float* coef, int HW, int total, float2* x_out,
                                                         float2* xmean_out) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const float* cf = coef + 4 * (p / HW);
  const float2 xv = x[p];
  const float2 yv = y ? y[p] : make_float2(0.f, 0.f);
  const float2 sc = score ? score[p] : make_float2(0.f, 0.f);
  float2 xm;
  xm.x = cf[0] * xv.x + cf[1] * yv.x + cf[2] * sc.x;
  xm.y = cf[0] * xv.y + cf[1] * yv.y + cf[2] * sc.y;
  if (xmean_out) xmean_out[p] = xm;
  const float2 z = noise ? noise[p] : cnormal(seed, offset + (uint64_t)p);
  x_out[p] = make_float2(xm.x + cf[3] * z.x, xm.y + cf[3] * z.y);
}

}  // namespace

extern "C" int snrse_sde_update(const void* x, const void* y, const void* score, const void* noise, uint64_t seed,
                                uint64_t offset, const float* coef, int B, int HW, void* x_out, void* xmean_out,
                                hipStream_t s) {
  const int total = B * HW;
  if (total <= 0 || !x || !coef || !x_out) return SNRSE_EINVAL;
  hipLaunchKernelGGL(sde_update_kernel, dim3((total + 255) / 256), dim3(256), 0, s, (const float2*)x,
                     (const float2*)y, (const float2*)score, (const float2*)noise, seed, offset, coef, HW, total,
                     (float2*)x_out, (float2*)xmean_out);
  return (int)hipGetLastError();
}

extern "C" int snrse_temb_mlp(const float* t, const float* Wg, const float* W1, const float* b1,
                              const float* W2, const float* b2, float* temb, int B, int nf, hipStream_t s) {
  if (nf != 128 || B <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(temb_mlp_kernel, dim3(B), dim3(512), 0, s, t, Wg, W1, b1, W2, b2, temb, nf);
  return (int)hipGetLastError();
}

extern "C" int snrse_temb_gfp_dense(const float* t, const float* Wg, const float* W1, const float* b1, float* out,
                                    int B, int nf, hipStream_t s) {
  // 4 nf <= 512: the pair's second launch (snrse_temb_dense, D = 4 nf) holds its input rows in a 512-float table
  if (nf <= 0 || 4 * nf > 512 || nf % 2 || B <= 0 || !t || !Wg || !W1 || !b1 || !out) return SNRSE_EINVAL;
  return launch_dense<2, 0>(nullptr, t, Wg, W1, b1, out, B, 4 * nf, 2 * nf, s);
}

extern "C" int snrse_temb_dense(const float* temb, const float* W, const float* bias, float* out, int B, int R,
                                int D, hipStream_t s) {
  if (D > 512 || D % 4 || B <= 0 || R <= 0) return SNRSE_EINVAL;
  return launch_dense<1, 0>(temb, nullptr, nullptr, W, bias, out, B, R, D, s);
}

template <typename T>
static int launch_input_conv(snrse_ctx* ctx, const void* x, const void* y, int B, int H, int W, const void* wgt,
                             const float* bias, void* out, float* pyr, double* stats, hipStream_t s) {
  if (!snrse_ctx_resolve(ctx)->stats_zeroed)
    SNRSE_RET(hipMemsetAsync(stats, 0, sizeof(double) * 2 * SNRSE_STAT_SLOTS * (size_t)B * 128, s));
  const long long blocks = (long long)B * H * W / (64 * 16);
  // LDS-staged form: the rows 1024 pixels span + 2 halo rows, <= (1023 / W + 4) * W * 16 B (64 KB at W = 1024)
  const int lds_rows = 1023 / W + 4;  // (a 1024-px range can touch 1023 / W + 2 rows when W does not divide 1024)
  if (W <= 1024 && snrse_ctx_resolve(ctx)->ic_lds) {
    const size_t lds = (size_t)lds_rows * W * 16;
    static const hipError_t attr1 = hipFuncSetAttribute((const void*)input_conv_lds_kernel<T, 128>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    static const hipError_t attr2 = hipFuncSetAttribute((const void*)input_conv_lds_kernel<T, 64>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    SNRSE_RET(attr1);
    SNRSE_RET(attr2);
    static const hipError_t attr3 = hipFuncSetAttribute((const void*)input_conv_lds_kernel<T, 128, true>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    SNRSE_RET(attr3);
    if (snrse_ctx_resolve(ctx)->ic_lds == 3)
      hipLaunchKernelGGL((input_conv_lds_kernel<T, 128, true>), dim3((unsigned)blocks), dim3(256), lds + 4 * 4096, s,
                         (const float2*)x, (const float2*)y, H, W, (const T*)wgt, bias, (T*)out, pyr, stats);
    else if (snrse_ctx_resolve(ctx)->ic_lds == 2)
      hipLaunchKernelGGL((input_conv_lds_kernel<T, 64>), dim3((unsigned)blocks), dim3(256), lds, s, (const float2*)x,
                         (const float2*)y, H, W, (const T*)wgt, bias, (T*)out, pyr, stats);
    else
      hipLaunchKernelGGL((input_conv_lds_kernel<T, 128>), dim3((unsigned)blocks), dim3(256), lds, s, (const float2*)x,
                         (const float2*)y, H, W, (const T*)wgt, bias, (T*)out, pyr, stats);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(input_conv_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, (const float2*)x, (const float2*)y,
                     H, W, (const T*)wgt, bias, (T*)out, pyr, stats);
  return (int)hipGetLastError();
}

// dtype: SNRSE_BF16 or SNRSE_F16 (the format of wgt and out)
extern "C" int snrse_input_conv(snrse_ctx* ctx, const void* x, const void* y, int B, int H, int W, const void* wgt, const float* bias,
                                void* out, float* pyr, double* stats, int dtype, hipStream_t s) {
  if (B <= 0 || H <= 0 || W <= 0 || W % 64 || ((long long)H * W / 64) % 16 || !x || !y || !wgt || !bias || !out ||
      !pyr || !stats || !snrse_is16(dtype))
    return SNRSE_EINVAL;
  return dtype == SNRSE_F16 ? launch_input_conv<f16_t>(ctx, x, y, B, H, W, wgt, bias, out, pyr, stats, s)
                            : launch_input_conv<bf16_t>(ctx, x, y, B, H, W, wgt, bias, out, pyr, stats, s);
}

extern "C" int snrse_input_conv_x3(snrse_ctx* ctx, const void* x, const void* y, int B, int H, int W, const void* wgt,
                                   const float* bias, float* out, float* pyr, double* stats, hipStream_t s) {
  if (B <= 0 || H <= 0 || W <= 0 || W % 64 || W > 1024 || ((long long)H * W / 64) % 16 || !x || !y || !wgt || !bias ||
      !out || !pyr || !stats)
    return SNRSE_EINVAL;
  if (!snrse_ctx_resolve(ctx)->stats_zeroed)
    SNRSE_RET(hipMemsetAsync(stats, 0, sizeof(double) * 2 * SNRSE_STAT_SLOTS * (size_t)B * 128, s));
  const long long blocks = (long long)B * H * W / (64 * 16);
  const size_t lds = (size_t)(1023 / W + 4) * W * 16;
  static const hipError_t attr = hipFuncSetAttribute((const void*)input_conv_lds_x3_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
  SNRSE_RET(attr);
  hipLaunchKernelGGL(input_conv_lds_x3_kernel, dim3((unsigned)blocks), dim3(256), lds, s, (const float2*)x,
                     (const float2*)y, H, W, (const bf16_t*)wgt, bias, out, pyr, stats);
  return (int)hipGetLastError();
}

extern "C" int snrse_input_pack(const void* x, const void* y, int B, int H, int W, void* col, float* pyr,
                                int dtype, hipStream_t s) {
  const int total = B * H * W;
  if (total <= 0) return SNRSE_EINVAL;
  const long long lanes = (long long)total * (snrse_is16(dtype) ? 8 : 16);
  dim3 grid((unsigned)((lanes + 255) / 256));
  if (dtype == SNRSE_F16)
    hipLaunchKernelGGL(input_pack_kernel<f16_t>, grid, dim3(256), 0, s, (const float2*)x, (const float2*)y, H, W,
                       (f16_t*)col, pyr, total);
  else if (dtype == SNRSE_BF16)
    hipLaunchKernelGGL(input_pack_kernel<bf16_t>, grid, dim3(256), 0, s, (const float2*)x, (const float2*)y, H, W,
                       (bf16_t*)col, pyr, total);
  else if (dtype == SNRSE_F32)
    hipLaunchKernelGGL(input_pack_kernel<float>, grid, dim3(256), 0, s, (const float2*)x, (const float2*)y, H, W,
                       (float*)col, pyr, total);
  else
    return SNRSE_EINVAL;
  return (int)hipGetLastError();
}

extern "C" int snrse_score_update(const void* pyr, int pyr_f32, const float* out_w, const float* out_b,
                                  const float* t, int score_mode, int B, int HW, const void* x, const void* y,
                                  const void* noise, uint64_t seed, uint64_t offset, const float* coef,
                                  void* x_out, void* xmean_out, void* score_out, hipStream_t s) {
  const int total = B * HW;
  if (total <= 0 || !pyr || !x) return SNRSE_EINVAL;
  if (x_out && !coef) return SNRSE_EINVAL;
  dim3 grid((total + 255) / 256);
  if (pyr_f32)
    hipLaunchKernelGGL(score_update_kernel<float>, grid, dim3(256), 0, s, (const float*)pyr, out_w, out_b, t,
                       score_mode, HW, total, (const float2*)x, (const float2*)y, (const float2*)noise, seed,
                       offset, coef, (float2*)x_out, (float2*)xmean_out, (float2*)score_out);
  else
    hipLaunchKernelGGL(score_update_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)pyr, out_w, out_b, t,
                       score_mode, HW, total, (const float2*)x, (const float2*)y, (const float2*)noise, seed,
                       offset, coef, (float2*)x_out, (float2*)xmean_out, (float2*)score_out);
  return (int)hipGetLastError();
}

extern "C" int snrse_axpby_noise(const void* x, const void* y, const void* noise, uint64_t seed, uint64_t offset,
                                 const float* coef, int B, int HW, void* out, hipStream_t s) {
  const int total = B * HW;
  if (total <= 0 || !coef || !out) return SNRSE_EINVAL;
  hipLaunchKernelGGL(axpby_noise_kernel, dim3((total + 255) / 256), dim3(256), 0, s, (const float2*)x,
                     (const float2*)y, (const float2*)noise, seed, offset, coef, HW, total, (float2*)out);
  return (int)hipGetLastError();
}
