// v10x3: the v10 halo GEMM structure (conv_h10.hip: persistent, one wave per SIMD, MFMAs as tied-AGPR asm with the
// next chunk's halo work in per-MFMA VALU slices, register-only epilogue, fused shortcut chunks) for the fp32x3
// parity mode: fp32 activations and output, split-bf16 products hi.hi + hi.lo + lo.hi (three
// v_mfma_f32_16x16x32_bf16 per 16x16x32 block; weights pre-split by ops.split_weight: per 32-channel K tile 32 hi
// then 32 lo bf16), the GroupNorm(+SiLU) of the fp32 halo applied once per element while it is split.
// Reference: ResnetBlockBigGANpp.Conv_0 / Conv_1 (+ Conv_2 shortcut), sgmse/backbones/ncsnpp_utils/layerspp.py:244-276,
// in fp32 as the reference runs it (sgmse/model.py:824).
//
// Workgroup tile 8 rows x 32 px = 256 px x 128 couts (the fp32 halo is split into hi / lo 128-B rows: 340 x 128 B =
// 43.5 KB per buffer, two buffers + two shortcut tiles of 256 x 128 B = 152.6 KB of LDS); wave w: px half (w & 1) =
// 4 rows x 32 px, cout half (w >> 1) = 64 couts: 8 x 4 blocks = 128 accumulators, 96 MFMAs per tap.
// Shapes: H % 8 == 0, W % 32 == 0, Cout % 128 == 0, shortcut channels <= 2 x main channels.
#include "conv_common.h"

#include <utility>

using namespace snrse_conv;

namespace {
namespace h10x3 {
constexpr int TH = 8, TW = 32, HC = TW + 2;
constexpr int HROWS = (TH + 2) * HC;            // 340
constexpr int HBYTES = HROWS * 128;             // 43520: 128-B rows, hi chunks 0-3, lo chunks 4-7 (swz)
constexpr int VPT = (HROWS * 8 + 255) / 256;    // 11 fp32 16-B halo vectors per thread: vector tid + 256 k
constexpr int SCBYTES = TH * TW * 128;          // shortcut tile: 256 rows x 128 B
constexpr int SCOFF = 2 * HBYTES;
constexpr int SCV = TH * TW * 8 / 256;          // 8 shortcut vectors per thread per chunk
constexpr int LDS = 2 * HBYTES + 2 * SCBYTES;   // 152,576 B
constexpr int KT = 32;
constexpr int NSTEP = 72;                       // 9 taps x 8 pixel blocks
// halo vector k: loaded at step LOAD0 + STRIDE k, transformed over 4 steps from XF0 + STRIDE k (two slots per step),
// stored at the end of the last one
constexpr int STRIDE = 5, XF0 = 16, LOAD0 = XF0 - 16;
static_assert(XF0 + STRIDE * (VPT - 1) + 4 <= NSTEP, "transform schedule fits one chunk");
// shortcut vectors (2 chunks x 8): loaded every SCSTRIDE steps from SCL0, split and stored in the step SCLAG later
constexpr int SCSTRIDE = 3, SCL0 = 1, SCLAG = 16;
static_assert(SCL0 + SCSTRIDE * 15 + SCLAG < NSTEP, "shortcut schedule fits one chunk");

SNRSE_DEV void a_fma(float& d, float b, float c) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(d) : "v"(b), "v"(c)); }
SNRSE_DEV float a_exp(float s) { float d; asm volatile("v_exp_f32 %0, %1" : "=v"(d) : "v"(s)); return d; }
SNRSE_DEV void a_fmamk(float& d, float k) { asm volatile("v_fmamk_f32 %0, %0, 0xbfb8aa3b, %1" : "+v"(d) : "v"(k)); }
SNRSE_DEV void a_rcp(float& d) { asm volatile("v_rcp_f32 %0, %0" : "+v"(d)); }
SNRSE_DEV void a_mul(float& d, float s) { asm volatile("v_mul_f32 %0, %0, %1" : "+v"(d) : "v"(s)); }
SNRSE_DEV uint32_t a_cvtpk(float a, float b) {
  uint32_t d;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
SNRSE_DEV float a_lshl16(uint32_t s) { float d; asm volatile("v_lshlrev_b32 %0, 16, %1" : "=v"(d) : "v"(s)); return d; }
SNRSE_DEV float a_andhi(uint32_t s) { float d; asm volatile("v_and_b32 %0, 0xffff0000, %1" : "=v"(d) : "v"(s)); return d; }
SNRSE_DEV void a_sub(float& d, float s) { asm volatile("v_sub_f32 %0, %0, %1" : "+v"(d) : "v"(s)); }
SNRSE_DEV void a_and(uint32_t& d, uint32_t m) { asm volatile("v_and_b32 %0, %0, %1" : "+v"(d) : "v"(m)); }
SNRSE_DEV void a_mfma(f32x4& acc, const u32x4& w, const u32x4& h) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(h));
}
template <int N, typename F, int... S>
SNRSE_DEV void static_for_impl(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, typename F>
SNRSE_DEV void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}
}  // namespace h10x3

template <int GNM, int EF>
__global__ __launch_bounds__(256, 1) void conv_halo10x3_kernel(ConvParams p, int ntiles) {
  using namespace h10x3;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ph = wid & 1, chh = wid >> 1;
  const int lrow = lane & 15, lg = lane >> 4;

  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int t_begin = (int)((long long)g * ntiles / nb), t_end = (int)((long long)(g + 1) * ntiles / nb);
  if (t_begin >= t_end) return;

  const int H = p.H, W = p.W;
  const int ntw = W / TW, nth = H / TH;
  const int Cin = p.C0 + p.C1, ncb = Cin / KT, K1 = 9 * Cin;
  const int Csc_all = p.sc_src ? p.Csc + p.Csc1 : 0, nsc = Csc_all / KT;
  auto sb = [&](int m) { return m * nsc / ncb; };
  const bool f_temb = EF < 0 ? p.temb != nullptr : (EF & EF_TEMB) != 0;
  const bool f_res = EF < 0 ? p.res != nullptr : (EF & EF_RES) != 0;
  const bool f_comb = EF < 0 ? p.comb_src != nullptr : (EF & EF_COMB) != 0;
  const bool f_stats = EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0;

  // buffer extents: the split weights are [Npad][2 K] bf16 (p.wbytes counts K fp32 = 2 K bf16 per row: the same bytes)
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);
  const __amdgpu_buffer_rsrc_t rws = make_rsrc(nsc ? p.sc_wgt : p.wgt, nsc ? p.sc_wbytes : p.wbytes);
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.src0, p.bytes0);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.C1 ? p.src1 : p.src0, p.C1 ? p.bytes1 : p.bytes0);
  const __amdgpu_buffer_rsrc_t rc0 = make_rsrc(nsc ? p.sc_src : p.src0, nsc ? p.sc_bytes0 : p.bytes0);
  const __amdgpu_buffer_rsrc_t rc1 = make_rsrc(p.Csc1 && nsc ? p.sc_src1 : p.src0, p.Csc1 && nsc ? p.sc_bytes1 : p.bytes0);

  // ---- halo fragment addresses (128-B rows, swz: chunk ^ (row & 7)); fragment i of tap (dy, dx) reads row R0 + k,
  // R0 = ph * 4 * HC + lrow, k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1; 4 * HC = 136 = 0 mod 8, so the
  // swizzle depends on (lrow + k) mod 8: 8 per-lane bases (hi; lo = hi ^ 64) plus the immediate (k / 8) * 1024
  int hbh[8], hbl[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int r = ph * 4 * HC + lrow + m;
    hbh[m] = r * 128 + ((lg ^ (r & 7)) << 4);
    hbl[m] = r * 128 + (((4 + lg) ^ (r & 7)) << 4);
  }
  // shortcut tile rows ph * 128 + 16 i + lrow: swizzle (lrow & 7)
  const int scbh = SCOFF + (ph * 128 + lrow) * 128 + ((lg ^ (lrow & 7)) << 4);
  const int scbl = SCOFF + (ph * 128 + lrow) * 128 + (((4 + lg) ^ (lrow & 7)) << 4);

  // ---- per-thread halo vectors: halo row (tid >> 3) + 32 k, fp32 16-B chunk tid & 7 (4 channels)
  const int hch = tid & 7;
  int hyx[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int hr = (tid >> 3) + 32 * k;
    const int hy = hr / HC;
    hyx[k] = hr < HROWS ? hy * 64 + (hr - hy * HC) : 63 * 64;
  }
  int hpix[VPT];
  int spix = 0;  // shortcut tile: this thread's vector r = 0 at tile row tid >> 3 (row r: + 32 r = + r W px rows)
  auto halo_geom = [&](int b, int h0, int w0) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int ih = h0 + (hyx[k] >> 6) - 1, iw = w0 + (hyx[k] & 63) - 1;
      const bool ok = ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      hpix[k] = ok ? (b * H + ih) * W + iw : -1;
    }
    spix = (b * H + h0) * W + w0 + (tid >> 3);  // tile row tid >> 3 (< 32): image row h0, column w0 + (tid >> 3)
  };
  auto tile_coords = [&](int t, int& n0, int& b, int& h0, int& w0) {
    n0 = (t % p.ntn) * 128;
    t /= p.ntn;
    w0 = (t % ntw) * TW;
    t /= ntw;
    h0 = (t % nth) * TH;
    b = t / nth;
  };

  u32x4 hv[VPT];
  u32x4 sv[2 * SCV];
  float gsc[4], gsh[4];
  int pc_ch = 0;
  bool pc_src1 = false;
  int pc_buf = 0;
  int pu0 = 0, pn = 0;
  auto prep_begin = [&](int c, int b) {
    pc_ch = c * KT;
    pc_src1 = pc_ch >= p.C0;
    pu0 = sb(c);
    pn = sb(c + 1) - pu0;
    if constexpr (GNM > 0) {
      const f32x4 s0 = *(const f32x4*)(p.gn_scale + (size_t)b * Cin + pc_ch + hch * 4);
      const f32x4 t0 = *(const f32x4*)(p.gn_shift + (size_t)b * Cin + pc_ch + hch * 4);
      const float pre = GNM == 2 ? kNegLog2e : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) { gsc[i] = s0[i] * pre; gsh[i] = t0[i] * pre; }
    }
  };
  auto prep_load = [&](int k) {
    const int cs = pc_src1 ? p.C1 : p.C0;
    const int cc = (pc_src1 ? pc_ch - p.C0 : pc_ch) + hch * 4;
    const int voff = hpix[k] >= 0 ? (hpix[k] * cs + cc) * 4 : (int)0x80000000;
    hv[k] = __builtin_amdgcn_raw_buffer_load_b128(pc_src1 ? rs1 : rs0, voff, 0, 0);
  };
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  // split x[4] into hi / lo bf16 and store both halves of halo row hr (chunk hch: 8 B of hi chunk hch >> 1, 8 B of lo)
  auto put_split = [&](char* base, int hr, const uint32_t (&hi)[2], const uint32_t (&lo)[2]) {
    *(u32x2*)(base + swz(hr, hch >> 1) + (hch & 1) * 8) = u32x2{hi[0], hi[1]};
    *(u32x2*)(base + swz(hr, 4 + (hch >> 1)) + (hch & 1) * 8) = u32x2{lo[0], lo[1]};
  };
  auto prep_store = [&](int k) {  // prologue: the whole transform at once
    const int hr = (tid >> 3) + 32 * k;
    if (k == VPT - 1 && hr >= HROWS) return;
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = __uint_as_float(hv[k][e]);
    if constexpr (GNM > 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = fmaf(x[e], gsc[e], gsh[e]);
        x[e] = hpix[k] < 0 ? 0.f : (GNM == 2 ? silu_z(z) : z);
      }
    }
    uint32_t hi[2], lo[2];
    hi[0] = pack_bf16x2(x[0], x[1]);
    hi[1] = pack_bf16x2(x[2], x[3]);
    lo[0] = pack_bf16x2(x[0] - __uint_as_float(hi[0] << 16), x[1] - __uint_as_float(hi[0] & 0xffff0000u));
    lo[1] = pack_bf16x2(x[2] - __uint_as_float(hi[1] << 16), x[3] - __uint_as_float(hi[1] & 0xffff0000u));
    put_split(smem + pc_buf * HBYTES, hr, hi, lo);
  };
  auto sc_load = [&](int q) {  // always issued (see conv_h10.hip)
    const int ch = (q / SCV < pn ? pu0 + q / SCV : pu0) * KT;
    const bool one = ch >= p.Csc;
    const int cs = one ? p.Csc1 : p.Csc;
    const int pix = spix + (q % SCV) * W;  // tile row (tid >> 3) + 32 r = image row h0 + r, column tid >> 3
    sv[q] = __builtin_amdgcn_raw_buffer_load_b128(one ? rc1 : rc0, (pix * cs + (one ? ch - p.Csc : ch) + hch * 4) * 4, 0, 0);
  };
  // shortcut vector split in three slices (dependencies only across slices): hi = bf16(x), its fp32 value, x - hi;
  // then lo = bf16(x - hi) + the store
  float sx[4];
  uint32_t shi[2];
  auto sc_slice = [&](int q, int part) {
    if (part == 0) {
      shi[0] = a_cvtpk(__uint_as_float(sv[q][0]), __uint_as_float(sv[q][1]));
      shi[1] = a_cvtpk(__uint_as_float(sv[q][2]), __uint_as_float(sv[q][3]));
    } else if (part == 1) {
      sx[0] = a_lshl16(shi[0]); sx[1] = a_andhi(shi[0]); sx[2] = a_lshl16(shi[1]); sx[3] = a_andhi(shi[1]);
    } else if (part == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float d = __uint_as_float(sv[q][e]);
        a_sub(d, sx[e]);
        sx[e] = d;
      }
    } else {
      uint32_t lo[2] = {a_cvtpk(sx[0], sx[1]), a_cvtpk(sx[2], sx[3])};
      if (q / SCV < pn) put_split(smem + SCOFF + (q / SCV) * SCBYTES, (tid >> 3) + 32 * (q % SCV), shi, lo);
    }
  };
  // halo transform in 14 half-slots, one after each of 14 MFMAs, so at most 4 VALU follow an MFMA and no VALU reads a
  // result of the same half-slot (asm VALU pairs in a dependency would get a wait state each): 0a / 0b affine of
  // elements 0-1 / 2-3, 1a / 1b exp, 2a / 2b fma, 3a / 3b rcp, 4a mul, 4b zero-padding mask, 5a hi = bf16(y),
  // 5b its fp32 value, 6a y - hi, 6b lo = bf16(y - hi) + the store of both halves.  GNM 1: no exp / fma / rcp / mul;
  // GNM 0: no mask either (raw out-of-range loads read 0)
  float xy[4], xe[4];
  uint32_t xh[2], xl[2];
  const float knl2 = kNegInvLn2;
  auto xf_half = [&](auto K, auto HS) {
    constexpr int k = decltype(K)::value, hs = decltype(HS)::value, sl = hs / 2, h = hs % 2;
    constexpr int e0 = 2 * h, e1 = 2 * h + 1;
    if constexpr (sl == 0) {
      xy[e0] = __uint_as_float(hv[k][e0]);
      xy[e1] = __uint_as_float(hv[k][e1]);
      if constexpr (GNM > 0) { a_fma(xy[e0], gsc[e0], gsh[e0]); a_fma(xy[e1], gsc[e1], gsh[e1]); }
    }
    if constexpr (sl == 1 && GNM == 2) { xe[e0] = a_exp(xy[e0]); xe[e1] = a_exp(xy[e1]); }
    if constexpr (sl == 2 && GNM == 2) { a_fmamk(xe[e0], knl2); a_fmamk(xe[e1], knl2); }
    if constexpr (sl == 3 && GNM == 2) { a_rcp(xe[e0]); a_rcp(xe[e1]); }
    if constexpr (hs == 8 && GNM == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) a_mul(xy[e], xe[e]);
    }
    if constexpr (hs == 9 && GNM > 0) {
      const uint32_t okm = hpix[k] >= 0 ? 0xffffffffu : 0u;  // the conv's zero padding
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t u = __float_as_uint(xy[e]);
        a_and(u, okm);
        xy[e] = __uint_as_float(u);
      }
    }
    if constexpr (hs == 10) { xh[0] = a_cvtpk(xy[0], xy[1]); xh[1] = a_cvtpk(xy[2], xy[3]); }
    if constexpr (hs == 11) { xe[0] = a_lshl16(xh[0]); xe[1] = a_andhi(xh[0]); xe[2] = a_lshl16(xh[1]); xe[3] = a_andhi(xh[1]); }
    if constexpr (hs == 12) {
#pragma unroll
      for (int e = 0; e < 4; ++e) a_sub(xy[e], xe[e]);
    }
    if constexpr (hs == 13) {
      xl[0] = a_cvtpk(xy[0], xy[1]);
      xl[1] = a_cvtpk(xy[2], xy[3]);
      const int hr = (tid >> 3) + 32 * k;
      if (k < VPT - 1 || hr < HROWS) {
        uint32_t hi[2] = {xh[0], xh[1]}, lo[2] = {xl[0], xl[1]};
        put_split(smem + pc_buf * HBYTES, hr, hi, lo);
      }
    }
  };

  // split weights: row co at (co * 2 ld + 2 koff) bf16, hi 64 B then lo 64 B per 32-channel tile
  auto wload = [&](u32x4 (&wh)[4], u32x4 (&wl)[4], int n0, bool sc, int tap, int c) {
    const int ld = sc ? Csc_all : K1;
    const int vb = ((n0 + chh * 64 + lrow) * 2 * ld + lg * 8) * 2;
    const int koff = 2 * ((sc ? 0 : tap * Cin) + c * KT) * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wh[j] = __builtin_amdgcn_raw_buffer_load_b128(sc ? rws : rw, vb, j * 16 * 2 * ld * 2 + koff, 0);
      wl[j] = __builtin_amdgcn_raw_buffer_load_b128(sc ? rws : rw, vb, j * 16 * 2 * ld * 2 + koff + 64, 0);
    }
  };

  f32x4 acc[8][4];
  u32x4 whc[4], wlc[4], whn[4], wln[4];

  int n0, bb, h0, w0;
  tile_coords(t_begin, n0, bb, h0, w0);
  halo_geom(bb, h0, w0);
  prep_begin(0, bb);
  pc_buf = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_load(k);
#pragma unroll
  for (int q = 0; q < 2 * SCV; ++q) sc_load(q);
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_store(k);
#pragma unroll
  for (int q = 0; q < 2 * SCV; ++q) {
    sc_slice(q, 0);
    sc_slice(q, 1);
    sc_slice(q, 2);
    sc_slice(q, 3);
  }
  wload(whn, wln, n0, pn > 0, 0, pn > 0 ? pu0 : 0);
  int gc = 0;

  for (int t = t_begin; t < t_end; ++t) {
    tile_coords(t, n0, bb, h0, w0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int nn0 = n0;
    for (int c = 0; c < ncb; ++c) {
      // ---- shortcut chunks of group c
      const int u_end = sb(c + 1);
      for (int u = sb(c); u < u_end; ++u) {
        const int sbuf = u - sb(c);
        const bool nxt_sc = u + 1 < u_end;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        u32x4 sfh[8], sfl[8];
        auto sread = [&](int i) {
          sfh[i] = *(const u32x4*)(smem + scbh + sbuf * SCBYTES + i * 2048);
          sfl[i] = *(const u32x4*)(smem + scbl + sbuf * SCBYTES + i * 2048);
        };
#pragma unroll
        for (int i = 0; i < 3; ++i) sread(i);
#pragma unroll
        for (int j = 0; j < 4; ++j) { whc[j] = whn[j]; wlc[j] = wln[j]; }
        wload(whn, wln, n0, nxt_sc, 0, nxt_sc ? u + 1 : c);
        static_for<8>([&](auto I) {
          constexpr int i = decltype(I)::value;
          if constexpr (i + 3 < 8) sread(i + 3);
          static_for<12>([&](auto M) {
            constexpr int m = decltype(M)::value, pp = m / 4, j = m % 4;
            if constexpr (i == 0 && m == 0) asm volatile("s_nop 1" ::: "memory");
            if constexpr (pp == 0) a_mfma(acc[i][j], whc[j], sfh[i]);
            if constexpr (pp == 1) a_mfma(acc[i][j], wlc[j], sfh[i]);
            if constexpr (pp == 2) a_mfma(acc[i][j], whc[j], sfl[i]);
          });
          __builtin_amdgcn_sched_barrier(0);
        });
      }
      // ---- main chunk c (prepared meanwhile: the next group, or a dummy one after the workgroup's last chunk)
      const bool last_c = c + 1 == ncb;
      int pb = bb;
      if (last_c) {
        if (t + 1 < t_end) {
          int h0n, w0n;
          tile_coords(t + 1, nn0, pb, h0n, w0n);
          halo_geom(pb, h0n, w0n);
        } else {
#pragma unroll
          for (int k = 0; k < VPT; ++k) hpix[k] = -1;
        }
      }
      prep_begin(last_c ? 0 : c + 1, pb);
      pc_buf = (gc + 1) & 1;
      const bool nsc_next = pn > 0;
      const int nc = nsc_next ? pu0 : (last_c ? 0 : c + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int boff = (gc & 1) * HBYTES;
      int hh[8], hl[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) { hh[m] = hbh[m] + boff; hl[m] = hbl[m] + boff; }
      u32x4 fh[9][8], fl[9][8];
      auto hread = [&](int tap, int i) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1;
        fh[tap][i] = *(const u32x4*)(smem + hh[k & 7] + (k >> 3) * 1024);
        fl[tap][i] = *(const u32x4*)(smem + hl[k & 7] + (k >> 3) * 1024);
      };
#pragma unroll
      for (int i = 0; i < 3; ++i) hread(0, i);
      // 9 taps x 8 steps; step (tap, i): the halo fragments 3 steps ahead, then 12 MFMAs (pixel block i x 4 cout
      // blocks x 3 split products), two of them followed by a slice of the next group's halo / shortcut work
      static_for<NSTEP>([&](auto ST) {
        constexpr int st = decltype(ST)::value, tap = st / 8, i = st % 8;
        if constexpr (i == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) { whc[j] = whn[j]; wlc[j] = wln[j]; }
          if constexpr (tap < 8) wload(whn, wln, n0, false, tap + 1, c);
          else wload(whn, wln, nn0, nsc_next, 0, nc);
        }
        if constexpr (i + 3 < 8) hread(tap, i + 3);
        else if constexpr (tap < 8) hread(tap + 1, i - 5);
        if constexpr (st >= LOAD0 && (st - LOAD0) % STRIDE == 0 && (st - LOAD0) / STRIDE < VPT) prep_load((st - LOAD0) / STRIDE);
        if constexpr (st >= SCL0 && (st - SCL0) % SCSTRIDE == 0 && (st - SCL0) / SCSTRIDE < 2 * SCV) sc_load((st - SCL0) / SCSTRIDE);
        // 12 MFMAs, product-major (hi.hi, hi.lo, lo.hi over the 4 cout blocks: consecutive MFMAs on different
        // accumulators); after MFMA (pp, j): shortcut vector parts (pp = 0, 1), the halo half-slot 4 s4 + j (pp = 2)
        static_for<12>([&](auto M) {
          constexpr int m = decltype(M)::value, pp = m / 4, j = m % 4;
          if constexpr (i == 0 && m == 0) asm volatile("s_nop 1" ::: "memory");
          if constexpr (pp == 0) a_mfma(acc[i][j], whc[j], fh[tap][i]);
          if constexpr (pp == 1) a_mfma(acc[i][j], wlc[j], fh[tap][i]);
          if constexpr (pp == 2) a_mfma(acc[i][j], whc[j], fl[tap][i]);
          // shortcut vector q = (step - SCL0 - SCLAG) / SCSTRIDE: parts 0-3 after MFMAs 1, 3, 5, 7 of its step
          constexpr int srel = st - SCL0 - SCLAG;
          if constexpr (m < 8 && m % 2 == 1 && srel >= 0 && srel % SCSTRIDE == 0 && srel / SCSTRIDE < 2 * SCV)
            sc_slice(srel / SCSTRIDE, m / 2);
          constexpr int rel = st - XF0;
          if constexpr (pp == 2 && rel >= 0 && rel % STRIDE < 4 && rel / STRIDE < VPT && 4 * (rel % STRIDE) + j < 14)
            xf_half(std::integral_constant<int, rel / STRIDE>{}, std::integral_constant<int, 4 * (rel % STRIDE) + j>{});
        });
        __builtin_amdgcn_sched_barrier(0);
      });
      ++gc;
    }
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");

    // ---- epilogue from registers: acc[i][j][e] = out[pixel(i, lrow)][co0 + 16 j + e], fp32: 16-B stores
    const int co0 = n0 + chh * 64 + 4 * lg;
    f32x4 add[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      add[j] = *(const f32x4*)(p.bias + co0 + 16 * j);
      if (f_temb) add[j] += *(const f32x4*)(p.temb + (size_t)bb * p.temb_stride + co0 + 16 * j);
    }
    f32x4 s1[4], s2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { s1[j] = f32x4{0.f, 0.f, 0.f, 0.f}; s2[j] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int pix0 = (bb * H + h0 + ph * 4) * W + w0 + lrow;
    const float osc = p.out_scale;
    auto epi = [&](auto SC) {
      constexpr bool scale = decltype(SC)::value;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pix = pix0 + (i >> 1) * W + (i & 1) * 16;
        f32x4 q = f32x4{0.f, 0.f, 0.f, 0.f};
        if (f_comb) q = *(const f32x4*)(p.comb_src + (size_t)pix * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = co0 + 16 * j;
          f32x4 v = acc[i][j] + add[j];
          if (f_res) v += *(const f32x4*)((const float*)p.res + (size_t)pix * p.res_ld + co);
          if constexpr (scale) v *= osc;
          if (f_comb) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f32x4 cw = *(const f32x4*)(p.comb_w + (size_t)(co + e) * 4);
              v[e] += q[0] * cw[0] + q[1] * cw[1] + q[2] * cw[2] + q[3] * cw[3] + p.comb_b[co + e];
            }
          }
          *(f32x4*)((float*)p.out + (size_t)pix * p.out_ld + co) = v;
          if (f_stats) {
            s1[j] += v;
            s2[j] = v * v + s2[j];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (osc != 1.f) epi(std::integral_constant<bool, true>{});
    else epi(std::integral_constant<bool, false>{});
    if (f_stats) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = s1[j][e], q2 = s2[j][e];
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x128, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x128, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x124, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x124, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x122, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x122, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x121, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x121, 0xf, 0xf, false));
          s1[j][e] = a;
          s2[j][e] = q2;
        }
      if (lrow == 0) {
        const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const size_t o = stat_idx(bb, slot, co0 + 16 * j + e, p.Cout);
            unsafeAtomicAdd(&p.stats[o], (double)s1[j][e]);
            unsafeAtomicAdd(&p.stats[o + 1], (double)s2[j][e]);
          }
      }
    }
  }
}

template <int GNM, int EF>
int launch_h10x3_ef(const ConvParams& p, int ntiles, int grid, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_halo10x3_kernel<GNM, EF>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, h10x3::LDS);
  SNRSE_RET(attr);
  hipLaunchKernelGGL((conv_halo10x3_kernel<GNM, EF>), dim3(grid), dim3(256), h10x3::LDS, s, p, ntiles);
  return (int)hipGetLastError();
}

template <int GNM>
int launch_h10x3_gn(const ConvParams& p, int ntiles, int grid, hipStream_t s) {
  return launch_h10x3_ef<GNM, EF_RT>(p, ntiles, grid, s);
}

}  // namespace

namespace snrse_conv {

bool h10x3_ok(const ConvParams& p) {
  const int ncb = (p.C0 + p.C1) / h10x3::KT, nsc = p.sc_src ? (p.Csc + p.Csc1) / h10x3::KT : 0;
  return p.ksize == 3 && p.H % h10x3::TH == 0 && p.W % h10x3::TW == 0 && p.Cout % 128 == 0 && nsc <= 2 * ncb &&
         p.bias && (p.C0 + p.C1) % h10x3::KT == 0 && p.C0 % h10x3::KT == 0;
}

int launch_h10x3(ConvParams p, hipStream_t s, int num_cu) {
  p.ntn = p.Cout / 128;
  const int ntiles = p.B * (p.H / h10x3::TH) * (p.W / h10x3::TW) * p.ntn;
  const int grid = ntiles < num_cu ? ntiles : num_cu;
  if (!p.gn_scale) return launch_h10x3_gn<0>(p, ntiles, grid, s);
  if (!p.gn_act) return launch_h10x3_gn<1>(p, ntiles, grid, s);
  return launch_h10x3_gn<2>(p, ntiles, grid, s);
}

}  // namespace snrse_conv
