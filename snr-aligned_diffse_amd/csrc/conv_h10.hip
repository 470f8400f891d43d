// v10 halo GEMM for the bf16 3x3 ResBlock convolutions (reference: ResnetBlockBigGANpp.Conv_0 / Conv_1,
// sgmse/backbones/ncsnpp_utils/layerspp.py:244-276, ddpm_conv3x3 layers.py:100-124; GroupNorm+SiLU prologue
// layerspp.py:258-266).
//
// Structure (one workgroup of 4 waves per CU, one wave per SIMD, up to 512 registers per wave, persistent):
//   * workgroup tile 16 image rows x 32 px = 512 px x 128 couts; wave w computes px half (w & 1) = 8 rows x 32 px
//     and cout half (w >> 1) = 64 couts: 16 x 4 blocks of v_mfma_f32_16x16x32_bf16 = 256 accumulators, computed
//     as D'[cout][px] (weights are the A operand) so that a lane ends with 4 consecutive couts of one pixel and the
//     epilogue stores 8-byte vectors straight from registers (no LDS staging);
//   * K runs in 32-channel chunks x 9 taps; the chunk's halo (18 x 34 rows x 64 B = 39 KB, swizzled 16-B chunks)
//     sits in one of two LDS buffers while the NEXT chunk's halo (of this tile, or of the workgroup's next tile) is
//     loaded, GroupNorm+SiLU-transformed and stored into the other one, a few vectors per tap between the MFMAs of
//     the current chunk -- the transform uses the issue slots the matrix pipe leaves free instead of a VALU-only
//     stretch at the chunk boundary (v5);
//   * weight fragments come straight from global memory (L2-resident, 295 KB per 128->128 layer) into registers,
//     one tap ahead; halo fragments are read from LDS four 16-px blocks ahead, across tap boundaries;
//   * one barrier per chunk (the halo buffers swap); the 512-px tile has 612 halo rows (1.20 x the tile, against
//     1.33 x for v5's 256-px tiles), so there is 10 % less GroupNorm+SiLU work per output.
// Shapes: H % 16 == 0, W % 32 == 0, Cout % 128 == 0, no fused 1x1 shortcut (those stay on v5).
#include "conv_common.h"

using namespace snrse_conv;

namespace {
namespace h10 {
constexpr int TH = 16, TW = 32, HC = TW + 2;
constexpr int HROWS = (TH + 2) * HC;     // 612
constexpr int HBYTES = HROWS * 64;       // 39168
constexpr int VPT = (HROWS * 4 + 255) / 256;  // 10 halo vectors (16 B) per thread: vector tid + 256 k
constexpr int LDS = 2 * HBYTES;
constexpr int KT = 32;
}  // namespace h10

template <int GNM, int EF>
__global__ __launch_bounds__(256, 1) void conv_halo10_kernel(ConvParams p, int ntiles) {
  using namespace h10;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ph = wid & 1, chh = wid >> 1;
  const int lrow = lane & 15, lg = lane >> 4;

  // contiguous tile range per workgroup; workgroups that share an XCD (blockIdx % 8) take neighbouring ranges
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int t_begin = (int)((long long)g * ntiles / nb), t_end = (int)((long long)(g + 1) * ntiles / nb);
  if (t_begin >= t_end) return;

  const int H = p.H, W = p.W;
  const int ntw = W / TW, nth = H / TH;
  const int Cin = p.C0 + p.C1, ncb = Cin / KT, K1 = 9 * Cin;
  const bool f_temb = EF < 0 ? p.temb != nullptr : (EF & EF_TEMB) != 0;
  const bool f_res = EF < 0 ? p.res != nullptr : (EF & EF_RES) != 0;
  const bool f_comb = EF < 0 ? p.comb_src != nullptr : (EF & EF_COMB) != 0;
  const bool f_stats = EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0;

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.src0, p.bytes0);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.C1 ? p.src1 : p.src0, p.C1 ? p.bytes1 : p.bytes0);

  // ---- halo fragment addresses: row hr of a buffer at hr * 64 + ((lg ^ ((hr >> 1) & 3)) << 4).  Fragment i of tap
  // (dy, dx) reads row R0 + k with R0 = ph * 8 * HC + lrow and k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1;
  // the swizzle term depends on (R0 + k) mod 8 = (lrow + k) mod 8 only (8 * HC = 272 = 0 mod 8), so 8 per-lane bases
  // (k mod 8) plus the immediate (k / 8) * 512 address every fragment
  int hb[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int r = ph * 8 * HC + lrow + m;
    hb[m] = r * 64 + ((lg ^ ((r >> 1) & 3)) << 4);
  }

  // ---- per-thread halo vectors of a tile: row (tid >> 2) + 64 k, 16-B chunk tid & 3 (8 channels)
  const int hcol = tid & 3;
  // pixel index of each vector; outside the image (the conv's zero padding) or past the halo: -1.  Branch-free
  // (unsigned range tests, no short-circuit): per-vector exec masks would pin 20 SGPRs across the main loop
  int hyx[VPT];  // halo row / column of vector k: hy * 64 + hx (hy = 63: past the halo)
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int hr = (tid >> 2) + 64 * k;
    const int hy = hr / HC;
    hyx[k] = hr < HROWS ? hy * 64 + (hr - hy * HC) : 63 * 64;
  }
  int hpix[VPT];
  auto halo_geom = [&](int b, int h0, int w0) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int ih = h0 + (hyx[k] >> 6) - 1, iw = w0 + (hyx[k] & 63) - 1;
      const bool ok = ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      hpix[k] = ok ? (b * H + ih) * W + iw : -1;
    }
  };
  auto tile_coords = [&](int t, int& n0, int& b, int& h0, int& w0) {
    n0 = (t % p.ntn) * 128;
    t /= p.ntn;
    w0 = (t % ntw) * TW;
    t /= ntw;
    h0 = (t % nth) * TH;
    b = t / nth;
  };

  // ---- state of the chunk being prepared (the "next" chunk)
  u32x4 hv[VPT];
  float gsc[8], gsh[8];
  int pc_ch = 0;      // its first channel
  bool pc_src1 = false;
  int pc_buf = 0;     // LDS buffer it goes to
  auto prep_begin = [&](int c, int b) {  // chunk c of the tile whose geometry is in hpix / hok
    pc_ch = c * KT;
    pc_src1 = pc_ch >= p.C0;
    if constexpr (GNM > 0) {
      const float* s = p.gn_scale + (size_t)b * Cin + pc_ch + hcol * 8;
      const float* t = p.gn_shift + (size_t)b * Cin + pc_ch + hcol * 8;
      const f32x4 s0 = *(const f32x4*)s, s1 = *(const f32x4*)(s + 4);
      const f32x4 t0 = *(const f32x4*)t, t1 = *(const f32x4*)(t + 4);
      const float pre = GNM == 2 ? kNegLog2e : 1.f;  // gn_xform8<2> takes the -log2(e)-prescaled affine
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gsc[i] = s0[i] * pre; gsc[4 + i] = s1[i] * pre;
        gsh[i] = t0[i] * pre; gsh[4 + i] = t1[i] * pre;
      }
    }
  };
  auto prep_load = [&](int k) {
    const int cs = pc_src1 ? p.C1 : p.C0;
    const int cc = (pc_src1 ? pc_ch - p.C0 : pc_ch) + hcol * 8;
    const int voff = hpix[k] >= 0 ? (hpix[k] * cs + cc) * 2 : (int)0x80000000;
    hv[k] = __builtin_amdgcn_raw_buffer_load_b128(pc_src1 ? rs1 : rs0, voff, 0, 0);
  };
  auto prep_store = [&](int k) {
    const int hr = (tid >> 2) + 64 * k;
    if (k == VPT - 1 && hr >= HROWS) return;
    u32x4 v = hv[k];
    if constexpr (GNM > 0) v = gn_xform8<GNM>(v, gsc, gsh, hpix[k] >= 0);
    *(u32x4*)(smem + pc_buf * HBYTES + swz64(hr, hcol)) = v;
  };

  // ---- weight fragments (A operand): cout row n0 + chh * 64 + 16 j + lrow, 8 channels at lg * 8 of K offset koff
  auto wload = [&](u32x4 (&wf)[4], int n0, int tap, int c) {
    const int vb = ((n0 + chh * 64 + lrow) * K1 + lg * 8) * 2;
    const int koff = (tap * Cin + c * KT) * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = __builtin_amdgcn_raw_buffer_load_b128(rw, vb, j * 16 * K1 * 2 + koff, 0);
  };

  f32x4 acc[16][4];
  u32x4 wcur[4], wnext[4];

  // ---- prologue: the first tile's chunk 0 halo, synchronously
  int n0, bb, h0, w0;
  tile_coords(t_begin, n0, bb, h0, w0);
  halo_geom(bb, h0, w0);
  prep_begin(0, bb);
  pc_buf = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_load(k);
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_store(k);
  wload(wnext, n0, 0, 0);
  int gc = 0;  // chunks done by this workgroup (buffer parity)

  for (int t = t_begin; t < t_end; ++t) {
    tile_coords(t, n0, bb, h0, w0);
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int nn0 = n0;  // cout tile of the weights loaded for the next tap
    for (int c = 0; c < ncb; ++c) {
      // the chunk prepared during this one: c + 1 of this tile, or chunk 0 of the next tile
      const bool last_c = c + 1 == ncb;
      const bool has_next = !last_c || t + 1 < t_end;
      int pb = bb;
      if (last_c && has_next) {
        int h0n, w0n;
        tile_coords(t + 1, nn0, pb, h0n, w0n);
        halo_geom(pb, h0n, w0n);  // (this chunk's halo is already in LDS)
      }
      if (has_next) {
        prep_begin(last_c ? 0 : c + 1, pb);
        pc_buf = (gc + 1) & 1;
      }
      const int nc = last_c ? 0 : c + 1;  // chunk of the weights prefetched at tap 8
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // halo(c) complete in buffer gc & 1; the other buffer is free
      const int boff = (gc & 1) * HBYTES;
      int hbc[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) hbc[m] = hb[m] + boff;
      u32x4 hf[9][16];
      auto hread = [&](int tap, int i) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1;
        hf[tap][i] = *(const u32x4*)(smem + hbc[k & 7] + (k >> 3) * 512);
      };
#pragma unroll
      for (int i = 0; i < 4; ++i) hread(0, i);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int j = 0; j < 4; ++j) wcur[j] = wnext[j];
        if (tap < 8) wload(wnext, n0, tap + 1, c);
        else if (has_next) wload(wnext, nn0, 0, nc);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (i + 4 < 16) hread(tap, i + 4);
          else if (tap < 8) hread(tap + 1, i - 12);
          // the next chunk's halo: vector k loaded at tap k / 2, transformed + stored two taps later
          if (has_next) {
            if (i == 0 && tap < 5) prep_load(2 * tap);
            if (i == 8 && tap < 5) prep_load(2 * tap + 1);
            if (i == 4 && tap >= 2 && tap < 7) prep_store(2 * (tap - 2));
            if (i == 12 && tap >= 2 && tap < 7) prep_store(2 * (tap - 2) + 1);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            // inline asm with the accumulator tied in AGPRs: the builtin's register allocation rotates a third of
            // the 256 accumulators through copies and spills (no spare AGPR quad); operands come from loads only
            if (i == 0 && j == 0)  // (2 wait states after any compiler VALU write of an operand, e.g. a copy)
              asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(wcur[j]), "v"(hf[tap][i]));
            else
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(wcur[j]), "v"(hf[tap][i]));
          // program order at 16-px-block granularity: the prefetch distances above are the schedule (the
          // scheduler would otherwise hoist the fragment reads of the whole chunk and spill)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      ++gc;
    }
    // the asm MFMAs' results are read by the epilogue's v_accvgpr_read: wait states hipcc does not insert
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");

#ifdef H10_EXP_NOEPI
    {
      float* o = (float*)p.out + (size_t)t * 256 * 64 + lane * 4;
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 4; ++j) *(f32x4*)(o + (i * 4 + j) * 256) = acc[i][j];
      continue;
    }
#endif
    // ---- epilogue from registers: acc[i][j][e] = out[pixel(i, lrow)][co0 + 16 j + e]
    const int co0 = n0 + chh * 64 + 4 * lg;
    float add[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 bv = *(const f32x4*)(p.bias + co0 + 16 * j);
      f32x4 tv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (f_temb) tv = *(const f32x4*)(p.temb + (size_t)bb * p.temb_stride + co0 + 16 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) add[j][e] = bv[e] + tv[e];
    }
    float s1[4][4], s2[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) { s1[j][e] = 0.f; s2[j][e] = 0.f; }
    const int pix0 = (bb * H + h0 + ph * 8) * W + w0 + lrow;
    const float osc = p.out_scale;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pix = pix0 + (i >> 1) * W + (i & 1) * 16;
      f32x4 q = f32x4{0.f, 0.f, 0.f, 0.f};
      if (f_comb) q = *(const f32x4*)(p.comb_src + (size_t)pix * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + 16 * j;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + add[j][e];
        if (f_res) {
          const uint2 rv = *(const uint2*)((const bf16_t*)p.res + (size_t)pix * p.res_ld + co);
          v[0] += __uint_as_float(rv.x << 16);
          v[1] += __uint_as_float(rv.x & 0xffff0000u);
          v[2] += __uint_as_float(rv.y << 16);
          v[3] += __uint_as_float(rv.y & 0xffff0000u);
        }
        if (osc != 1.f) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= osc;
        }
        if (f_comb) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4 cw = *(const f32x4*)(p.comb_w + (size_t)(co + e) * 4);
            v[e] += q[0] * cw[0] + q[1] * cw[1] + q[2] * cw[2] + q[3] * cw[3] + p.comb_b[co + e];
          }
        }
        uint2 o;
        o.x = pack_bf16x2(v[0], v[1]);
        o.y = pack_bf16x2(v[2], v[3]);
        *(uint2*)((bf16_t*)p.out + (size_t)pix * p.out_ld + co) = o;
        if (f_stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) { s1[j][e] += v[e]; s2[j][e] = fmaf(v[e], v[e], s2[j][e]); }
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one 16-px block at a time (the 256 accumulator reads are not hoisted)
    }
    if (f_stats) {
      // sum over the 16 pixels of a lane row (lanes with equal lg): DPP row rotations
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
int launch_h10_ef(const ConvParams& p, int ntiles, int grid, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_halo10_kernel<GNM, EF>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, h10::LDS);
  SNRSE_RET(attr);
  hipLaunchKernelGGL((conv_halo10_kernel<GNM, EF>), dim3(grid), dim3(256), h10::LDS, s, p, ntiles);
  return (int)hipGetLastError();
}

template <int GNM>
int launch_h10_gn(const ConvParams& p, int ntiles, int grid, hipStream_t s, bool specialise) {
  if (specialise && p.bias) {
    switch (epi_flags(p) & ~EF_NT) {  // (8-byte stores: no non-temporal form)
      case EF_TEMB | EF_STATS: return launch_h10_ef<GNM, EF_TEMB | EF_STATS>(p, ntiles, grid, s);
      case EF_RES | EF_STATS: return launch_h10_ef<GNM, EF_RES | EF_STATS>(p, ntiles, grid, s);
      case EF_STATS: return launch_h10_ef<GNM, EF_STATS>(p, ntiles, grid, s);
      default: break;
    }
  }
  return launch_h10_ef<GNM, EF_RT>(p, ntiles, grid, s);
}

}  // namespace

namespace snrse_conv {

bool h10_ok(const ConvParams& p) {
  return p.ksize == 3 && p.H % h10::TH == 0 && p.W % h10::TW == 0 && p.Cout % 128 == 0 && !p.sc_src && p.bias &&
         (p.C0 + p.C1) % h10::KT == 0 && p.C0 % h10::KT == 0;
}

int launch_h10(ConvParams p, hipStream_t s, int num_cu, bool specialise) {
  p.ntn = p.Cout / 128;
  const int ntiles = p.B * (p.H / h10::TH) * (p.W / h10::TW) * p.ntn;
  const int grid = ntiles < num_cu ? ntiles : num_cu;
  if (!p.gn_scale) return launch_h10_gn<0>(p, ntiles, grid, s, specialise);
  if (!p.gn_act) return launch_h10_gn<1>(p, ntiles, grid, s, specialise);
  return launch_h10_gn<2>(p, ntiles, grid, s, specialise);
}

}  // namespace snrse_conv
