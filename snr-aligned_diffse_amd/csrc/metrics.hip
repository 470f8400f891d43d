// Evaluation metrics of the enhanced waveforms (the step after the path in eval.py:144-157):
// SI-SDR / SI-SIR / SI-SAR (utils.py:10-35, energy_ratios) and the plain SI-SDR of
// sgmse/util/other.py:71-75, batched over utterances on the device.
//
// All three ratios follow from six dot products per utterance (fp64 accumulation, one pass over
// s_hat, s, n -- HBM-bound: 12 B per sample):
//   a_s = <s_hat, s> / |s|^2, a_n = <s_hat, n> / |n|^2, s_target = a_s s, e_noise = a_n n,
//   e_art = s_hat - s_target - e_noise
//   |s_target|^2 = a_s^2 |s|^2, |e_noise|^2 = a_n^2 |n|^2,
//   |e_noise + e_art|^2 = |s_hat|^2 - 2 a_s <s_hat, s> + a_s^2 |s|^2,
//   |e_art|^2 = |s_hat - a_s s - a_n n|^2 expanded with <s, n>.
#include "common.h"

namespace {

constexpr int MT = 512;

__global__ __launch_bounds__(MT) void energy_ratios_kernel(const float* s_hat, const float* s, const float* n, int L,
                                                           double* out) {
  const int b = blockIdx.x;
  const float* ph = s_hat + (size_t)b * L;
  const float* ps = s + (size_t)b * L;
  const float* pn = n ? n + (size_t)b * L : nullptr;
  double acc[6] = {0, 0, 0, 0, 0, 0};  // ss, nn, hh, hs, hn, sn
  for (int i = threadIdx.x; i < L; i += MT) {
    const double h = ph[i], x = ps[i], z = pn ? (double)pn[i] : 0.0;
    acc[0] += x * x;
    acc[1] += z * z;
    acc[2] += h * h;
    acc[3] += h * x;
    acc[4] += h * z;
    acc[5] += x * z;
  }
  __shared__ double red[MT / 64][6];
#pragma unroll
  for (int k = 0; k < 6; ++k) acc[k] = wave_sum_d(acc[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) red[threadIdx.x >> 6][k] = acc[k];
  __syncthreads();
  if (threadIdx.x != 0) return;
  double d[6] = {0, 0, 0, 0, 0, 0};
  for (int w = 0; w < MT / 64; ++w)
#pragma unroll
    for (int k = 0; k < 6; ++k) d[k] += red[w][k];
  const double ss = d[0], nn = d[1], hh = d[2], hs = d[3], hn = d[4], sn = d[5];
  const double as = hs / ss;
  const double tgt = as * as * ss;
  const double dist = fmax(hh - 2.0 * as * hs + as * as * ss, 0.0);  // |s_hat - s_target|^2
  double* o = out + (size_t)b * 3;
  o[0] = 10.0 * log10(tgt / dist);
  if (pn) {
    const double an = hn / nn;
    const double noi = an * an * nn;
    const double art = fmax(hh + tgt + noi - 2.0 * as * hs - 2.0 * an * hn + 2.0 * as * an * sn, 0.0);
    o[1] = 10.0 * log10(tgt / noi);
    o[2] = 10.0 * log10(tgt / art);
  } else {
    o[1] = o[2] = __builtin_nan("");
  }
}

}  // namespace

extern "C" int snrse_energy_ratios(const float* s_hat, const float* s, const float* n, int B, int L, double* out,
                                   hipStream_t stream) {
  if (B <= 0 || L <= 0 || !s_hat || !s || !out) return SNRSE_EINVAL;
  hipLaunchKernelGGL(energy_ratios_kernel, dim3(B), dim3(MT), 0, stream, s_hat, s, n, L, out);
  return (int)hipGetLastError();
}
