// SNR estimator (SNRNet, reference sgmse/backbones/snrnet.py:47-97) on gfx950, fp32.
//
// Input: the raw complex STFT of y / max|y| (model.py:715-720) as interleaved complex64
// [B, 256, T] (T a multiple of 16, pad_spec_16) — channel 0 = real, 1 = imag, read in place
// (no view_as_real / permute copies).  Per 16-frame chunk n = b*(T/16) + k:
//   K1 conv5x5(2->32, pad 2) + maxpool 2x2            -> [N, 32, 128, 8]
//   K2 conv3x3(32->32, pad 1) + maxpool (2,1)          -> [N, 32, 64, 8]
//   K3 convt_{1..4} (64 x {1,2,4,8}) + full max-pool   -> feat [N, 128]
//   K4a LSTM input projections, both directions         -> xg [B, 2, S, 512]
//   K4b bidirectional LSTM recurrence (hidden 128)      -> h [B, S, 256]
//   K4c mean / std (unbiased) / min / max over S, FC, sigmoid -> [B]
// Tiny next to one score-network NFE (~1.2 GFLOP per 4 s clip); run once per utterance.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void conv5_pool_kernel(const float2* spec, int T, const float* w,
                                                         const float* bias, float* out, int N) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= N * 32 * 128 * 8) return;
  const int to = idx & 7, fo = (idx >> 3) & 127, co = (idx >> 10) & 31, n = idx >> 15;
  const int S = T / 16;
  const int b = n / S, k = n - b * S;
  const float2* base = spec + (size_t)b * 256 * T + k * 16;
  float best = -INFINITY;
  for (int py = 0; py < 2; ++py)
    for (int px = 0; px < 2; ++px) {
      const int f = 2 * fo + py, tau = 2 * to + px;
      float acc = bias[co];
      for (int dy = 0; dy < 5; ++dy) {
        const int ff = f + dy - 2;
        if (ff < 0 || ff >= 256) continue;
        for (int dx = 0; dx < 5; ++dx) {
          const int tt = tau + dx - 2;
          if (tt < 0 || tt >= 16) continue;
          const float2 v = base[(size_t)ff * T + tt];
          acc = fmaf(w[((co * 2 + 0) * 5 + dy) * 5 + dx], v.x, acc);
          acc = fmaf(w[((co * 2 + 1) * 5 + dy) * 5 + dx], v.y, acc);
        }
      }
      best = fmaxf(best, acc);
    }
  out[idx] = best;
}

__global__ __launch_bounds__(256) void conv3_pool_kernel(const float* in, const float* w, const float* bias,
                                                         float* out, int N) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= N * 32 * 64 * 8) return;
  const int to = idx & 7, fo = (idx >> 3) & 63, co = (idx >> 9) & 31, n = idx >> 14;
  const float* src = in + (size_t)n * 32 * 128 * 8;
  float best = -INFINITY;
  for (int py = 0; py < 2; ++py) {
    const int f = 2 * fo + py;
    float acc = bias[co];
    for (int ci = 0; ci < 32; ++ci)
      for (int dy = 0; dy < 3; ++dy) {
        const int ff = f + dy - 1;
        if (ff < 0 || ff >= 128) continue;
        for (int dx = 0; dx < 3; ++dx) {
          const int tt = to + dx - 1;
          if (tt < 0 || tt >= 8) continue;
          acc = fmaf(w[((co * 32 + ci) * 3 + dy) * 3 + dx], src[(ci * 128 + ff) * 8 + tt], acc);
        }
      }
    best = fmaxf(best, acc);
  }
  out[idx] = best;
}

// block per chunk n; thread (conv kk, co) -> max over positions of the (64 x kw) conv
__global__ __launch_bounds__(128) void timeconv_kernel(const float* in, const float* w1, const float* w2,
                                                       const float* w3, const float* w4, const float* b1,
                                                       const float* b2, const float* b3, const float* b4,
                                                       float* feat) {
  __shared__ float x[32 * 64 * 8];
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < 32 * 64 * 8; i += 128) x[i] = in[(size_t)n * 32 * 64 * 8 + i];
  __syncthreads();
  const int kk = threadIdx.x >> 5, co = threadIdx.x & 31;
  const int kw = 1 << kk;
  const float* w = kk == 0 ? w1 : (kk == 1 ? w2 : (kk == 2 ? w3 : w4));
  const float bv = kk == 0 ? b1[co] : (kk == 1 ? b2[co] : (kk == 2 ? b3[co] : b4[co]));
  float best = -INFINITY;
  for (int pos = 0; pos + kw <= 8; ++pos) {
    float acc = bv;
    for (int ci = 0; ci < 32; ++ci)
      for (int fh = 0; fh < 64; ++fh) {
        const float* wr = w + ((co * 32 + ci) * 64 + fh) * kw;
        const float* xr = x + (ci * 64 + fh) * 8 + pos;
        for (int j = 0; j < kw; ++j) acc = fmaf(wr[j], xr[j], acc);
      }
    best = fmaxf(best, acc);
  }
  feat[(size_t)n * 128 + kk * 32 + co] = best;
}

// xg[b][dir][s][g] = W_ih[dir][g] . feat[b][s] + b_ih[dir][g] + b_hh[dir][g]
__global__ __launch_bounds__(256) void lstm_input_kernel(const float* feat, const float* wih, const float* bsum,
                                                         float* xg, int B, int S) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * 2 * S * 512) return;
  const int g = idx & 511;
  int r = idx >> 9;
  const int s = r % S;
  r /= S;
  const int dir = r & 1, b = r >> 1;
  const float* wr = wih + ((size_t)dir * 512 + g) * 128;
  const float* f = feat + ((size_t)b * S + s) * 128;
  float acc = bsum[dir * 512 + g];
  for (int k = 0; k < 128; ++k) acc = fmaf(wr[k], f[k], acc);
  xg[idx] = acc;
}

// block (b, dir), 512 threads: gate order i, f, g, o (torch.nn.LSTM)
__global__ __launch_bounds__(512) void lstm_rec_kernel(const float* xg, const float* whh, float* hout, int S) {
  __shared__ float h[128];
  __shared__ float gates[512];
  const int b = blockIdx.x >> 1, dir = blockIdx.x & 1, g = threadIdx.x;
  if (g < 128) h[g] = 0.f;
  float c = 0.f;
  const float* wr = whh + ((size_t)dir * 512 + g) * 128;
  __syncthreads();
  for (int step = 0; step < S; ++step) {
    const int s = dir ? S - 1 - step : step;
    float acc = xg[(((size_t)b * 2 + dir) * S + s) * 512 + g];
    for (int k = 0; k < 128; ++k) acc = fmaf(wr[k], h[k], acc);
    gates[g] = acc;
    __syncthreads();
    if (g < 128) {
      const float ig = 1.f / (1.f + expf(-gates[g]));
      const float fg = 1.f / (1.f + expf(-gates[128 + g]));
      const float gg = tanhf(gates[256 + g]);
      const float og = 1.f / (1.f + expf(-gates[384 + g]));
      c = fg * c + ig * gg;
      const float hv = og * tanhf(c);
      h[g] = hv;
      hout[((size_t)b * S + s) * 256 + dir * 128 + g] = hv;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void snr_head_kernel(const float* hout, const float* fcw, const float* fcb,
                                                       float* out, int S) {
  __shared__ float red[4];
  const int b = blockIdx.x, j = threadIdx.x;
  const float* hb = hout + (size_t)b * S * 256;
  double s1 = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int s = 0; s < S; ++s) {
    const float v = hb[s * 256 + j];
    s1 += v;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  const double mean = s1 / S;
  double s2 = 0.0;
  for (int s = 0; s < S; ++s) {
    const double d = hb[s * 256 + j] - mean;
    s2 += d * d;
  }
  const float sd = S > 1 ? (float)sqrt(s2 / (S - 1)) : NAN;
  float part = fcw[j] * (float)mean + fcw[256 + j] * sd + fcw[512 + j] * mn + fcw[768 + j] * mx;
  part = wave_sum(part);
  if ((j & 63) == 0) red[j >> 6] = part;
  __syncthreads();
  if (j == 0) {
    const float z = red[0] + red[1] + red[2] + red[3] + fcb[0];
    out[b] = 1.f / (1.f + expf(-z));
  }
}

}  // namespace

// Weights (fp32, torch layouts): w5 [32,2,5,5] b5; w3 [32,32,3,3] b3; wt1..4 [32,32,64,kw] bt1..4;
// wih [2][512][128] (forward, reverse), bsum [2][512] = b_ih + b_hh; whh [2][512][128];
// fcw [1024], fcb [1].  Workspace: ws >= N*32*128*8 + N*32*64*8 + N*128 + B*2*S*512 + B*S*256
// floats, N = B*T/16, S = T/16.
extern "C" int snrse_snrnet(const void* spec, int B, int T, const float* w5, const float* b5, const float* w3,
                            const float* b3, const float* wt1, const float* wt2, const float* wt3,
                            const float* wt4, const float* bt1, const float* bt2, const float* bt3,
                            const float* bt4, const float* wih, const float* bsum, const float* whh,
                            const float* fcw, const float* fcb, float* ws, float* out, hipStream_t s) {
  if (B <= 0 || T < 16 || T % 16 || !spec || !ws || !out) return SNRSE_EINVAL;
  const int S = T / 16, N = B * S;
  float* a1 = ws;
  float* a2 = a1 + (size_t)N * 32 * 128 * 8;
  float* feat = a2 + (size_t)N * 32 * 64 * 8;
  float* xg = feat + (size_t)N * 128;
  float* hout = xg + (size_t)B * 2 * S * 512;
  const int n1 = N * 32 * 128 * 8, n2 = N * 32 * 64 * 8;
  hipLaunchKernelGGL(conv5_pool_kernel, dim3((n1 + 255) / 256), dim3(256), 0, s, (const float2*)spec, T, w5, b5,
                     a1, N);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv3_pool_kernel, dim3((n2 + 255) / 256), dim3(256), 0, s, a1, w3, b3, a2, N);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(timeconv_kernel, dim3(N), dim3(128), 0, s, a2, wt1, wt2, wt3, wt4, bt1, bt2, bt3, bt4, feat);
  SNRSE_LAUNCH_CHECK();
  const int n4 = B * 2 * S * 512;
  hipLaunchKernelGGL(lstm_input_kernel, dim3((n4 + 255) / 256), dim3(256), 0, s, feat, wih, bsum, xg, B, S);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(lstm_rec_kernel, dim3(2 * B), dim3(512), 0, s, xg, whh, hout, S);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(snr_head_kernel, dim3(B), dim3(256), 0, s, hout, fcw, fcb, out, S);
  return (int)hipGetLastError();
}

extern "C" size_t snrse_snrnet_workspace(int B, int T) {
  const size_t S = T / 16, N = (size_t)B * S;
  return sizeof(float) * (N * 32 * 128 * 8 + N * 32 * 64 * 8 + N * 128 + (size_t)B * 2 * S * 512 + B * S * 256);
}
