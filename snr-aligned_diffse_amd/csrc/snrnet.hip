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

// The three convolution stages are LDS-tiled, register-blocked fp32 FMA kernels: the weights of a
// stage are staged in LDS once per block and read as wave-uniform broadcasts (every lane of a wave
// works for the same output channels), the input tile is staged with its zero padding, and every lane
// keeps its input patch in registers across the output channels.  (The first version, one output
// element per thread with weights read from global per FMA, ran at ~5 TFLOP/s and took 23 % of the
// C4 step; profiles/r02r_c4_kernel_stats.md.)

// K1: conv5x5(2 -> 32, pad 2) + maxpool 2x2.  Block = (chunk n, 32 input rows f) -> 16 pooled rows x
// 8 pooled frames x 32 channels.  Lane = one pooled position, wave w: positions 64 (w >> 1) + lane,
// channels 16 (w & 1) + [0, 16).
constexpr int C5_FT = 32;                   // input rows per block
constexpr int C5_IR = C5_FT + 4, C5_IC = 20;  // staged rows (pad 2) x columns (16 frames + pad 2)
__global__ __launch_bounds__(256) void conv5_pool_kernel(const float2* spec, int T, const float* w,
                                                         const float* bias, float* out, int N) {
  __shared__ float xs[2][C5_IR][C5_IC];
  __shared__ __attribute__((aligned(16))) float ws[32][2][28];  // 25 taps padded to 28 (16-B rows)
  const int tid = threadIdx.x;
  const int n = blockIdx.x >> 3, ft = blockIdx.x & 7;  // 256 rows = 8 tiles of 32
  const int S = T / 16;
  const int b = n / S, k = n - b * S;
  const float2* base = spec + (size_t)b * 256 * T + k * 16;
  const int f0 = ft * C5_FT;
  for (int i = tid; i < C5_IR * C5_IC; i += 256) {
    const int r = i / C5_IC, c = i - r * C5_IC;
    const int f = f0 + r - 2, t = c - 2;
    float2 v = make_float2(0.f, 0.f);
    if (f >= 0 && f < 256 && t >= 0 && t < 16) v = base[(size_t)f * T + t];
    xs[0][r][c] = v.x;
    xs[1][r][c] = v.y;
  }
  for (int i = tid; i < 32 * 2 * 28; i += 256) {
    const int co = i / 56, rem = i - co * 56, ci = rem / 28, tap = rem - ci * 28;
    ws[co][ci][tap] = tap < 25 ? w[(co * 2 + ci) * 25 + tap] : 0.f;
  }
  __syncthreads();
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int pos = 64 * (wid >> 1) + lane;  // pooled position in the block: fo_l * 8 + to
  const int fol = pos >> 3, to = pos & 7;
  const int cb = 16 * (wid & 1);
  // 6 x 6 input patch of the 2 x 2 pool window, both channels
  float px[2][6][6];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; ++c) px[ci][r][c] = xs[ci][2 * fol + r][2 * to + c];
  float* o = out + (size_t)n * 32 * 128 * 8 + (size_t)(f0 / 2 + fol) * 8 + to;
  for (int cc = 0; cc < 16; ++cc) {
    const int co = cb + cc;
    float acc[2][2];
    const float bv = bias[co];
#pragma unroll
    for (int py = 0; py < 2; ++py)
#pragma unroll
      for (int qx = 0; qx < 2; ++qx) acc[py][qx] = bv;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
      float wt[28];
#pragma unroll
      for (int q = 0; q < 7; ++q) *(f32x4*)&wt[4 * q] = *(const f32x4*)&ws[co][ci][4 * q];
#pragma unroll
      for (int dy = 0; dy < 5; ++dy)
#pragma unroll
        for (int dx = 0; dx < 5; ++dx)
#pragma unroll
          for (int py = 0; py < 2; ++py)
#pragma unroll
            for (int qx = 0; qx < 2; ++qx) acc[py][qx] = fmaf(wt[dy * 5 + dx], px[ci][py + dy][qx + dx], acc[py][qx]);
    }
    o[(size_t)co * 128 * 8] = fmaxf(fmaxf(acc[0][0], acc[0][1]), fmaxf(acc[1][0], acc[1][1]));
  }
}

// K2: conv3x3(32 -> 32, pad 1) + maxpool (2, 1) over f.  Block = (chunk n, 32 input rows) -> 16 pooled
// rows x 8 frames x 32 channels.  Lane = (pooled row pair, frame): 8 x 8; wave w: channels 8w + [0, 8).
// Input channels are staged 8 at a time (input tile + weights 25 KB: several blocks per CU).
constexpr int C3_IR = 34, C3_IC = 12, C3_CK = 8;  // staged rows (32 + pad) x columns (8 + pad), ci per step
__global__ __launch_bounds__(256) void conv3_pool_kernel(const float* in, const float* w, const float* bias,
                                                         float* out, int N) {
  __shared__ float xs[C3_CK][C3_IR][C3_IC];
  __shared__ __attribute__((aligned(16))) float ws[32][C3_CK][12];  // [co][ci][9 taps padded to 12]
  const int tid = threadIdx.x;
  const int n = blockIdx.x >> 2, ft = blockIdx.x & 3;  // 128 rows = 4 tiles of 32
  const int f0 = ft * 32;
  const float* src = in + (size_t)n * 32 * 128 * 8;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int fp = lane >> 3, t = lane & 7;  // pooled rows 2 fp, 2 fp + 1 = conv rows 4 fp .. 4 fp + 3
  const int cb = 8 * wid;
  float acc[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float bv = bias[cb + c];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[c][r] = bv;
  }
  for (int c0 = 0; c0 < 32; c0 += C3_CK) {
    __syncthreads();
    for (int i = tid; i < C3_CK * C3_IR * C3_IC; i += 256) {
      const int ci = i / (C3_IR * C3_IC), rem = i - ci * (C3_IR * C3_IC);
      const int r = rem / C3_IC, c = rem - r * C3_IC;
      const int f = f0 + r - 1, tt = c - 1;
      xs[ci][r][c] = (f >= 0 && f < 128 && tt >= 0 && tt < 8) ? src[((c0 + ci) * 128 + f) * 8 + tt] : 0.f;
    }
    for (int i = tid; i < 32 * C3_CK * 12; i += 256) {
      const int co = i / (C3_CK * 12), rem = i - co * (C3_CK * 12), ci = rem / 12, tap = rem - ci * 12;
      ws[co][ci][tap] = tap < 9 ? w[(co * 32 + c0 + ci) * 9 + tap] : 0.f;
    }
    __syncthreads();
    for (int ci = 0; ci < C3_CK; ++ci) {
      float px[6][3];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) px[r][c] = xs[ci][4 * fp + r][t + c];
#pragma unroll 2
      for (int c = 0; c < 8; ++c) {
        float wt[12];
#pragma unroll
        for (int q = 0; q < 3; ++q) *(f32x4*)&wt[4 * q] = *(const f32x4*)&ws[cb + c][ci][4 * q];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[c][r] = fmaf(wt[dy * 3 + dx], px[r + dy][dx], acc[c][r]);
      }
    }
  }
  float* o = out + (size_t)n * 32 * 64 * 8 + (size_t)(f0 / 2 + 2 * fp) * 8 + t;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    o[(size_t)(cb + c) * 64 * 8] = fmaxf(acc[c][0], acc[c][1]);
    o[(size_t)(cb + c) * 64 * 8 + 8] = fmaxf(acc[c][2], acc[c][3]);
  }
}

// K3: the four (64 x kw) time convolutions (kw = 1, 2, 4, 8; all 64 rows, valid in time) + max over
// the 9 - kw positions, one launch: block = (16 chunks, 16 output channels, conv kk).  The reduction
// runs over ci in 32 steps, each staging x[16 chunks][64][8] and the weights [16 co][64][kw] of that ci
// in LDS.  Lane: chunk lane & 15; channel 4 w + (lane >> 4) of the block's 16.
constexpr int TC_NB = 16;          // chunks per block
constexpr int TC_XS = 64 * 8 + 4;  // chunk stride in LDS (floats): + 4 spreads the 16 chunks over the banks
template <int KW>
SNRSE_DEV void timeconv_block(const float* in, const float* w, const float* bias, float* feat, int N, int kk,
                              float* xs, float* ws) {
  constexpr int P = 9 - KW, WR = KW < 4 ? 4 : KW;  // positions; weight row padded to a 16-B multiple
  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * TC_NB, cg = blockIdx.y * 16;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int c = lane & 15, col = 4 * wid + (lane >> 4);
  float acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) acc[p] = 0.f;
  for (int ci = 0; ci < 32; ++ci) {
    __syncthreads();  // the previous step's reads are done
    for (int i = tid; i < TC_NB * 128; i += 256) {  // 16 chunks x 64 rows x 8 frames, f32x4 pieces
      const int ch = i >> 7, q = i & 127;
      const int n = n0 + ch;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (n < N) v = *(const f32x4*)(in + ((size_t)n * 32 + ci) * 512 + 4 * q);
      *(f32x4*)&xs[ch * TC_XS + 4 * q] = v;
    }
    for (int i = tid; i < 16 * 64 * WR; i += 256) {
      const int co = i / (64 * WR), rem = i - co * (64 * WR), fh = rem / WR, j = rem - fh * WR;
      ws[i] = j < KW ? w[(((size_t)(cg + co) * 32 + ci) * 64 + fh) * KW + j] : 0.f;
    }
    __syncthreads();
    const float* xr = xs + c * TC_XS;
    const float* wr = ws + col * 64 * WR;
#pragma unroll 4
    for (int fh = 0; fh < 64; ++fh) {
      float x[8], wt[WR];
      *(f32x4*)&x[0] = *(const f32x4*)&xr[fh * 8];
      *(f32x4*)&x[4] = *(const f32x4*)&xr[fh * 8 + 4];
#pragma unroll
      for (int q = 0; q < WR / 4; ++q) *(f32x4*)&wt[4 * q] = *(const f32x4*)&wr[fh * WR + 4 * q];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int j = 0; j < KW; ++j) acc[p] = fmaf(wt[j], x[p + j], acc[p]);
    }
  }
  const int n = n0 + c;
  if (n < N) {
    float best = -INFINITY;
#pragma unroll
    for (int p = 0; p < P; ++p) best = fmaxf(best, acc[p]);
    feat[(size_t)n * 128 + kk * 32 + cg + col] = best + bias[cg + col];
  }
}

__global__ __launch_bounds__(256) void timeconv_kernel(const float* in, const float* w1, const float* w2,
                                                       const float* w3, const float* w4, const float* b1,
                                                       const float* b2, const float* b3, const float* b4,
                                                       float* feat, int N) {
  __shared__ __attribute__((aligned(16))) float xs[TC_NB * TC_XS];
  __shared__ __attribute__((aligned(16))) float ws[16 * 64 * 8];
  switch (blockIdx.z) {  // block-uniform
    case 0: timeconv_block<1>(in, w1, b1, feat, N, 0, xs, ws); break;
    case 1: timeconv_block<2>(in, w2, b2, feat, N, 1, xs, ws); break;
    case 2: timeconv_block<4>(in, w3, b3, feat, N, 2, xs, ws); break;
    default: timeconv_block<8>(in, w4, b4, feat, N, 3, xs, ws); break;
  }
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
  __shared__ __attribute__((aligned(16))) float h[128];
  __shared__ float gates[512];
  const int b = blockIdx.x >> 1, dir = blockIdx.x & 1, g = threadIdx.x;
  if (g < 128) h[g] = 0.f;
  float c = 0.f;
  // this gate's recurrent weight row stays in registers for all S steps (read once instead of per step)
  float wr[128];
  const f32x4* wsrc = (const f32x4*)(whh + ((size_t)dir * 512 + g) * 128);
#pragma unroll
  for (int k = 0; k < 32; ++k) *(f32x4*)&wr[4 * k] = wsrc[k];
  __syncthreads();
  for (int step = 0; step < S; ++step) {
    const int s = dir ? S - 1 - step : step;
    float acc = xg[(((size_t)b * 2 + dir) * S + s) * 512 + g];
#pragma unroll
    for (int k = 0; k < 128; k += 4) {
      const f32x4 hv = *(const f32x4*)&h[k];
      acc = fmaf(wr[k], hv[0], acc);
      acc = fmaf(wr[k + 1], hv[1], acc);
      acc = fmaf(wr[k + 2], hv[2], acc);
      acc = fmaf(wr[k + 3], hv[3], acc);
    }
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
  (void)n1;
  (void)n2;
  hipLaunchKernelGGL(conv5_pool_kernel, dim3(N * 8), dim3(256), 0, s, (const float2*)spec, T, w5, b5, a1, N);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv3_pool_kernel, dim3(N * 4), dim3(256), 0, s, a1, w3, b3, a2, N);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(timeconv_kernel, dim3((N + TC_NB - 1) / TC_NB, 2, 4), dim3(256), 0, s, a2, wt1, wt2, wt3, wt4,
                     bt1, bt2, bt3, bt4, feat, N);
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
