// STFT front end and iSTFT back end of the enhancement path (gfx950).
//
// Reference: SpecsDataModule.stft / istft (data_module.py:269-297: n_fft 510, hop 128,
// periodic Hann, center=True with reflect padding, onesided) and the 'exponent' spectrogram
// transform spec_fwd / spec_back (data_module.py:241-267: |c|^0.5 e^{i angle c} * 0.15 and
// its inverse), plus pad_spec (util/other.py:83-90, zero frames up to a multiple of 64).
// n_fft = 510 = 2*3*5*17 is not a power of two, so the transform is a direct DFT against an
// LDS twiddle table (0.26 GFLOP per 4 s clip, negligible next to the network).
//
// Forward transform fused: y (already on device) * in_scale -> frames -> DFT -> exponent
// compression -> zero-padded [B, 256, Tpad] complex64 (the network's Y layout).
// Inverse fused: spec_back (c |c| with c = S / 0.15) -> C2R inverse DFT (DC / Nyquist
// imaginary parts dropped) -> window -> overlap-add / sum(window^2) -> trim -> * out_scale.
#include "common.h"

namespace {

constexpr int NFFT = 510;
constexpr int HOP = 128;
constexpr int NBIN = 256;
constexpr int FPB = 8;  // frames per STFT block

SNRSE_DEV void fill_twiddles(float* cs, float* sn) {
  for (int m = threadIdx.x; m < NFFT; m += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)m / NFFT, &s, &c);
    cs[m] = (float)c;
    sn[m] = (float)s;
  }
}

// mode: 0 = raw STFT, 1 = exponent transform (e = 0.5, factor 0.15)
__global__ __launch_bounds__(256) void stft_kernel(const float* sig, int L, const float* in_div, float in_scale,
                                                   int T, int Tpad, int mode, float2* out) {
  __shared__ float cs[NFFT], sn[NFFT];
  __shared__ float xs[(FPB - 1) * HOP + NFFT];
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FPB;
  fill_twiddles(cs, sn);
  const int span = (FPB - 1) * HOP + NFFT;
  const float scale = in_div ? in_scale / in_div[b] : in_scale;
  for (int j = threadIdx.x; j < span; j += 256) {
    int s = f0 * HOP + j - NFFT / 2;
    if (s < 0) s = -s;
    if (s >= L) s = 2 * (L - 1) - s;
    // frames >= T (zero padding up to Tpad) read past the reflect range; their output is
    // discarded, clamp the address so the load stays in bounds.
    s = s < 0 ? 0 : (s >= L ? L - 1 : s);
    xs[j] = sig[(size_t)b * L + s] * scale;
  }
  __syncthreads();
  const int k = threadIdx.x;  // bin
  float re[FPB], im[FPB];
#pragma unroll
  for (int f = 0; f < FPB; ++f) { re[f] = 0.f; im[f] = 0.f; }
  int idx = 0;  // (k * n) mod 510
  for (int n = 0; n < NFFT; ++n) {
    const float w = 0.5f - 0.5f * cs[n];  // periodic Hann = 0.5 - 0.5 cos(2 pi n / N)
    const float c = cs[idx], s = sn[idx];
#pragma unroll
    for (int f = 0; f < FPB; ++f) {
      const float v = xs[f * HOP + n] * w;
      re[f] = fmaf(v, c, re[f]);
      im[f] = fmaf(-v, s, im[f]);
    }
    idx += k;
    if (idx >= NFFT) idx -= NFFT;
  }
#pragma unroll
  for (int f = 0; f < FPB; ++f) {
    const int fr = f0 + f;
    if (fr >= Tpad) break;
    float2 o = make_float2(0.f, 0.f);
    if (fr < T) {
      o = make_float2(re[f], im[f]);
      if (mode == 1) {
        const float mag = sqrtf(o.x * o.x + o.y * o.y);
        const float g = mag > 0.f ? 0.15f / sqrtf(mag) : 0.f;
        o.x *= g;
        o.y *= g;
      }
    }
    out[((size_t)b * NBIN + k) * Tpad + fr] = o;
  }
}

// frames[b][f][n] = window[n] * irfft(spec_back(S[b, :, f]))[n]
__global__ __launch_bounds__(512) void istft_frames_kernel(const float2* spec, int T, int mode, float* frames) {
  __shared__ float cs[NFFT], sn[NFFT];
  __shared__ float2 X[4][NBIN];
  const int b = blockIdx.y, f0 = blockIdx.x * 4;
  fill_twiddles(cs, sn);
  for (int i = threadIdx.x; i < 4 * NBIN; i += 512) {
    const int f = i / NBIN, k = i % NBIN;
    float2 v = make_float2(0.f, 0.f);
    if (f0 + f < T) {
      v = spec[((size_t)b * NBIN + k) * T + f0 + f];
      if (mode == 1) {  // c = S / 0.15 ; X = |c| * c
        v.x *= (1.0f / 0.15f);
        v.y *= (1.0f / 0.15f);
        const float mag = sqrtf(v.x * v.x + v.y * v.y);
        v.x *= mag;
        v.y *= mag;
      }
    }
    X[f][k] = v;
  }
  __syncthreads();
  const int n = threadIdx.x;
  if (n >= NFFT) return;
  float acc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) acc[f] = X[f][0].x + ((n & 1) ? -X[f][NBIN - 1].x : X[f][NBIN - 1].x);
  int idx = n;  // (k * n) mod 510 for k = 1
  for (int k = 1; k < NBIN - 1; ++k) {
    const float c = 2.f * cs[idx], s = 2.f * sn[idx];
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] = fmaf(X[f][k].x, c, fmaf(-X[f][k].y, s, acc[f]));
    idx += n;
    if (idx >= NFFT) idx -= NFFT;
  }
  const float w = (0.5f - 0.5f * cs[n]) * (1.0f / NFFT);
#pragma unroll
  for (int f = 0; f < 4; ++f)
    if (f0 + f < T) frames[((size_t)b * T + f0 + f) * NFFT + n] = acc[f] * w;
}

__global__ __launch_bounds__(256) void istft_ola_kernel(const float* frames, int T, int L, const float* out_scale,
                                                        float* out) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int P = i + NFFT / 2;
  int fa = (P - NFFT + HOP) / HOP;  // ceil((P - 509) / 128)
  if (P - NFFT + 1 <= 0) fa = 0;
  int fb = P / HOP;
  if (fb > T - 1) fb = T - 1;
  float y = 0.f, env = 0.f;
  for (int f = fa; f <= fb; ++f) {
    const int n = P - f * HOP;
    if (n < 0 || n >= NFFT) continue;
    const float w = 0.5f - 0.5f * (float)cospi(2.0 * (double)n / NFFT);
    y += frames[((size_t)b * T + f) * NFFT + n];
    env += w * w;
  }
  const float sc = out_scale ? out_scale[b] : 1.f;
  out[(size_t)b * L + i] = env > 1e-11f ? y / env * sc : 0.f;
}

// out[b] = max |sig[b, :]|  (norm_factor = y.abs().max(), model.py:726)
__global__ __launch_bounds__(256) void absmax_kernel(const float* sig, int L, float* out) {
  const int b = blockIdx.x;
  float m = 0.f;
  for (int i = threadIdx.x; i < L; i += 256) m = fmaxf(m, fabsf(sig[(size_t)b * L + i]));
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[b] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// spec_fwd / spec_back of the 'exponent' transform on interleaved complex64 (e = 0.5, factor 0.15)
__global__ __launch_bounds__(256) void spec_transform_kernel(const float2* in, float2* out, long long n, int dir) {
  const long long i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  float2 v = in[i];
  if (dir == 0) {
    const float mag = sqrtf(v.x * v.x + v.y * v.y);
    const float g = mag > 0.f ? 0.15f / sqrtf(mag) : 0.f;
    v.x *= g;
    v.y *= g;
  } else {
    v.x *= (1.0f / 0.15f);
    v.y *= (1.0f / 0.15f);
    const float mag = sqrtf(v.x * v.x + v.y * v.y);
    v.x *= mag;
    v.y *= mag;
  }
  out[i] = v;
}

}  // namespace

extern "C" int snrse_spec_transform(const void* in, void* out, long long n, int dir, hipStream_t s) {
  if (n <= 0 || !in || !out || (dir != 0 && dir != 1)) return SNRSE_EINVAL;
  hipLaunchKernelGGL(spec_transform_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float2*)in,
                     (float2*)out, n, dir);
  return (int)hipGetLastError();
}

extern "C" int snrse_absmax(const float* sig, int B, int L, float* out, hipStream_t s) {
  if (B <= 0 || L <= 0 || !sig || !out) return SNRSE_EINVAL;
  hipLaunchKernelGGL(absmax_kernel, dim3(B), dim3(256), 0, s, sig, L, out);
  return (int)hipGetLastError();
}

extern "C" int snrse_stft(const float* sig, int B, int L, const float* in_div, float in_scale, int Tpad, int mode,
                          void* out, hipStream_t s) {
  const int T = 1 + L / HOP;
  if (B <= 0 || L <= NFFT / 2 || Tpad < T || (mode != 0 && mode != 1)) return SNRSE_EINVAL;
  dim3 grid((Tpad + FPB - 1) / FPB, B);
  hipLaunchKernelGGL(stft_kernel, grid, dim3(256), 0, s, sig, L, in_div, in_scale, T, Tpad, mode, (float2*)out);
  return (int)hipGetLastError();
}

extern "C" int snrse_istft(const void* spec, int B, int T, int L, int mode, const float* out_scale, float* frames,
                           float* out, hipStream_t s) {
  if (B <= 0 || T <= 0 || L <= 0 || !frames) return SNRSE_EINVAL;
  hipLaunchKernelGGL(istft_frames_kernel, dim3((T + 3) / 4, B), dim3(512), 0, s, (const float2*)spec, T, mode,
                     frames);
  SNRSE_LAUNCH_CHECK();
  hipLaunchKernelGGL(istft_ola_kernel, dim3((L + 255) / 256, B), dim3(256), 0, s, frames, T, L, out_scale, out);
  return (int)hipGetLastError();
}
