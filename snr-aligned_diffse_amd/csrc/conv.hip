// Implicit-GEMM convolution on MFMA for the NCSN++ score network (gfx950).
//
// Replaces the torch conv2d calls of ddpm_conv3x3 / ddpm_conv1x1 / NIN
// (reference: sgmse/backbones/ncsnpp_utils/layers.py:100-124, 546-555) as used by
// ResnetBlockBigGANpp (layerspp.py:244-276), AttnBlockpp (77-93), Combine (54-61) and
// the NCSNpp input/pyramid/output layers (ncsnpp.py:285, 348-366).
//
// Activations are NHWC ([B, F, T, C], channels contiguous).  GEMM view:
//   M = B*H*W output pixels, N = Cout, K = ksize^2 * Cin (+ Csc for a fused 1x1 shortcut).
// A K-tile is 128 bytes of one tap's channels (64 bf16 / 32 f32), so a tile row is one
// contiguous 16-byte-chunked load.  Concatenated inputs (torch.cat([h, skip]) of the up
// path, ncsnpp.py:337) are read from two source tensors without materialising the cat.
// The 1x1 shortcut Conv_2 of a ResBlock is appended as extra K-tiles (center tap of the
// shortcut source) so "Conv_1(h) + Conv_2(x)" is a single GEMM.
// Epilogue: y = (acc + bias[n] + temb[b][n] + res[m][n]) * out_scale  (+ combine term).
//
// MFMA: v_mfma_f32_16x16x32_bf16 (bf16) / v_mfma_f32_16x16x4_f32 (exact f32 parity mode).
// Both read one 16-byte LDS chunk per operand fragment with the same swizzled layout:
// rows of 128 B, chunk' = chunk ^ ((row >> 1) & 7) (conflict-free for the ds_read_b128
// lane groups of a 16-row fragment).
#include "common.h"

namespace {

template <typename T> struct ConvTraits;
template <> struct ConvTraits<bf16_t> {
  static constexpr int KT = 64;  // elements per K-tile (128 B)
  static constexpr int EPC = 8;  // elements per 16-B chunk
};
template <> struct ConvTraits<float> {
  static constexpr int KT = 32;
  static constexpr int EPC = 4;
};

struct ConvParams {
  const void* src0; int C0;
  const void* src1; int C1;
  int B, H, W;
  int ksize;
  const void* wgt;  // [Npad][ksize*ksize*Cin]
  const void* sc_src; int Csc;    // shortcut source(s): [M][Csc] (+ [M][Csc1])
  const void* sc_src1; int Csc1;
  const void* sc_wgt;  // [Npad][Csc + Csc1]
  const float* bias;   // [Cout]
  const float* temb; int temb_stride;  // [B][temb_stride] (pre-offset to this layer's column 0)
  const void* res; int res_ld;         // residual [M][res_ld] (same dtype as output)
  float out_scale;
  const float* comb_src;  // [M][4] f32 input-skip pyramid (Combine.Conv_0 input)
  const float* comb_w;    // [Cout][4]
  const float* comb_b;    // [Cout]
  void* out; int Cout; int out_ld;
  int M;
};

template <typename T>
SNRSE_DEV f32x4 mfma_chunk(const u32x4& a, const u32x4& b, f32x4 acc);

template <>
SNRSE_DEV f32x4 mfma_chunk<bf16_t>(const u32x4& a, const u32x4& b, f32x4 acc) {
  bf16x8_mfma av = __builtin_bit_cast(bf16x8_mfma, a);
  bf16x8_mfma bv = __builtin_bit_cast(bf16x8_mfma, b);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}
template <>
SNRSE_DEV f32x4 mfma_chunk<float>(const u32x4& a, const u32x4& b, f32x4 acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[j]), __uint_as_float(b[j]), acc, 0, 0, 0);
  return acc;
}

SNRSE_DEV int swz(int row, int chunk) { return (row << 7) + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T, typename TO, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_mfma_kernel(ConvParams p) {
  using Tr = ConvTraits<T>;
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int ROWS_PER_PASS = NT / 8;
  constexpr int A_LD = (BM + ROWS_PER_PASS - 1) / ROWS_PER_PASS;  // A rows per thread
  constexpr int B_LD = (BN + ROWS_PER_PASS - 1) / ROWS_PER_PASS;
  static_assert(BM % 16 == 0 && BN % 16 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // stage buffers: A[buf] at buf * BM * 128, B[buf] at 2 * BM * 128 + buf * BN * 128
#define AS(buf) (smem + (buf) * (BM * 128))
#define BS(buf) (smem + 2 * BM * 128 + (buf) * (BN * 128))

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int HW = p.H * p.W;
  const int Cin = p.C0 + p.C1;
  const int cblocks = Cin / Tr::KT;
  const int nk0 = p.ksize * p.ksize * cblocks;
  const int Csc_all = p.Csc + p.Csc1;
  const int nk = nk0 + (p.sc_src ? Csc_all / Tr::KT : 0);
  const int K1 = p.ksize * p.ksize * Cin;
  const int half = p.ksize >> 1;

  const int ch = tid & 7;
  // per-thread A rows: pixel coordinates
  int a_b[A_LD], a_h[A_LD], a_w[A_LD];
  bool a_ok[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int r = (tid >> 3) + i * ROWS_PER_PASS;
    const int m = m0 + r;
    a_ok[i] = (r < BM) && (m < p.M);
    const int mm = a_ok[i] ? m : 0;
    a_b[i] = mm / HW;
    const int rem = mm - a_b[i] * HW;
    a_h[i] = rem / p.W;
    a_w[i] = rem - a_h[i] * p.W;
  }

  u32x4 ra[A_LD], rb[B_LD];

  auto gload = [&](int kt) {
    const T* src;
    int cs, cc, dy, dx;
    const T* wbase;
    int wld;
    if (kt < nk0) {
      const int tap = kt / cblocks;
      const int c = (kt - tap * cblocks) * Tr::KT;
      dy = tap / p.ksize - half;
      dx = tap % p.ksize - half;
      if (c < p.C0) { src = (const T*)p.src0; cs = p.C0; cc = c; }
      else { src = (const T*)p.src1; cs = p.C1; cc = c - p.C0; }
      wbase = (const T*)p.wgt + tap * Cin + c;
      wld = K1;
    } else {
      const int c = (kt - nk0) * Tr::KT;
      if (c < p.Csc) { src = (const T*)p.sc_src; cs = p.Csc; cc = c; }
      else { src = (const T*)p.sc_src1; cs = p.Csc1; cc = c - p.Csc; }
      dy = 0; dx = 0;
      wbase = (const T*)p.sc_wgt + c;
      wld = Csc_all;
    }
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int hh = a_h[i] + dy, ww = a_w[i] + dx;
      const bool ok = a_ok[i] && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
      if (ok) {
        const T* ptr = src + ((size_t)(a_b[i] * p.H + hh) * p.W + ww) * cs + cc + ch * Tr::EPC;
        ra[i] = *(const u32x4*)ptr;
      } else {
        ra[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int r = (tid >> 3) + i * ROWS_PER_PASS;
      if (r < BN) {
        const T* ptr = wbase + (size_t)(n0 + r) * wld + ch * Tr::EPC;
        rb[i] = *(const u32x4*)ptr;
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int r = (tid >> 3) + i * ROWS_PER_PASS;
      if (r < BM) *(u32x4*)(AS(buf) + swz(r, ch)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int r = (tid >> 3) + i * ROWS_PER_PASS;
      if (r < BN) *(u32x4*)(BS(buf) + swz(r, ch)) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();

  const int lrow = lane & 15;
  const int lg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *(const u32x4*)(AS(cur) + swz(wm * TM + i * 16 + lrow, 4 * s + lg));
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *(const u32x4*)(BS(cur) + swz(wn * TN + j * 16 + lrow, 4 * s + lg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_chunk<T>(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

#undef AS
#undef BS
  // epilogue
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + lrow;
    if (n >= p.Cout) continue;
    const float bn = p.bias ? p.bias[n] : 0.f;
    float cw0 = 0.f, cw1 = 0.f, cw2 = 0.f, cw3 = 0.f, cb = 0.f;
    if (p.comb_src) {
      cw0 = p.comb_w[n * 4 + 0]; cw1 = p.comb_w[n * 4 + 1];
      cw2 = p.comb_w[n * 4 + 2]; cw3 = p.comb_w[n * 4 + 3];
      cb = p.comb_b[n];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * TM + i * 16 + lg * 4 + e;
        if (m >= p.M) continue;
        float v = acc[i][j][e] + bn;
        if (p.temb) v += p.temb[(size_t)(m / HW) * p.temb_stride + n];
        if (p.res) v += Elem<TO>::to_f(((const TO*)p.res)[(size_t)m * p.res_ld + n]);
        v *= p.out_scale;
        if (p.comb_src) {
          const float* q = p.comb_src + (size_t)m * 4;
          v += q[0] * cw0 + q[1] * cw1 + q[2] * cw2 + q[3] * cw3 + cb;
        }
        ((TO*)p.out)[(size_t)m * p.out_ld + n] = Elem<TO>::from_f(v);
      }
    }
  }
}

template <typename T, typename TO, int BM, int BN, int WM, int WN>
int launch_conv(const ConvParams& p, int npad, hipStream_t s) {
  dim3 grid((p.M + BM - 1) / BM, npad / BN);
  const size_t lds = (size_t)2 * (BM + BN) * 128;
  hipLaunchKernelGGL((conv_mfma_kernel<T, TO, BM, BN, WM, WN>), grid, dim3(64 * WM * WN), lds, s, p);
  return (int)hipGetLastError();
}

template <typename T, typename TO>
int dispatch_conv(const ConvParams& p, hipStream_t s) {
  if (p.Cout >= 64) {
    if (p.Cout % 128 != 0) return SNRSE_EINVAL;
    return launch_conv<T, TO, 128, 128, 2, 2>(p, p.Cout, s);
  }
  if (p.Cout > 16) return SNRSE_EINVAL;
  return launch_conv<T, TO, 128, 16, 4, 1>(p, 16, s);
}

}  // namespace

extern "C" int snrse_conv2d(const void* src0, int C0, const void* src1, int C1, int B, int H, int W,
                            int ksize, const void* wgt, const void* sc_src, int Csc, const void* sc_src1,
                            int Csc1, const void* sc_wgt,
                            const float* bias, const float* temb, int temb_stride, const void* res,
                            int res_ld, float out_scale, const float* comb_src, const float* comb_w,
                            const float* comb_b, void* out, int Cout, int out_ld, int dtype,
                            int out_f32, hipStream_t stream) {
  using TrB = ConvTraits<bf16_t>;
  using TrF = ConvTraits<float>;
  const int KT = dtype == SNRSE_BF16 ? TrB::KT : TrF::KT;
  if (!src0 || !wgt || !out || (ksize != 1 && ksize != 3)) return SNRSE_EINVAL;
  if (C0 % KT || C1 % KT || (sc_src && (Csc % KT || Csc1 % KT))) return SNRSE_EINVAL;
  if (sc_src && Csc1 > 0 && !sc_src1) return SNRSE_EINVAL;
  if (C1 > 0 && !src1) return SNRSE_EINVAL;
  ConvParams p;
  p.src0 = src0; p.C0 = C0; p.src1 = src1; p.C1 = C1;
  p.B = B; p.H = H; p.W = W; p.ksize = ksize; p.wgt = wgt;
  p.sc_src = sc_src; p.Csc = sc_src ? Csc : 0; p.sc_wgt = sc_wgt;
  p.sc_src1 = sc_src1; p.Csc1 = sc_src ? Csc1 : 0;
  p.bias = bias; p.temb = temb; p.temb_stride = temb_stride;
  p.res = res; p.res_ld = res_ld; p.out_scale = out_scale;
  p.comb_src = comb_src; p.comb_w = comb_w; p.comb_b = comb_b;
  p.out = out; p.Cout = Cout; p.out_ld = out_ld; p.M = B * H * W;
  if (p.M <= 0) return 0;
  if (dtype == SNRSE_BF16) {
    return out_f32 ? dispatch_conv<bf16_t, float>(p, stream) : dispatch_conv<bf16_t, bf16_t>(p, stream);
  }
  if (dtype == SNRSE_F32) return dispatch_conv<float, float>(p, stream);
  return SNRSE_EINVAL;
}
