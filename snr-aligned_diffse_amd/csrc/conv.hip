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
// rows of 128 B, chunk' = chunk ^ (row & 7): conflict-free for the ds_read_b128 lane groups
// of ANY 16 consecutive rows (each group's rows cover all residues mod 8), which the halo
// kernel needs because its fragments start at arbitrary (tap-shifted) rows.
#include "conv_common.h"

#include <algorithm>
#include <type_traits>

using namespace snrse_conv;

namespace {


// Shared epilogue: y = (acc + bias + temb + res) * out_scale + combine; optional GroupNorm
// statistics of y (per (b, channel) sum / sumsq) for the consumer's GroupNorm.
// acc[i][j][e]: row = mb + i*16 + (lane>>4)*4 + e, col = nb + j*16 + (lane&15).
// LDS-staged epilogue for one wave's 64 x 64 tile (rows = 64 consecutive output pixels
// mb.., cols = output channels nb..): the fp32 accumulators go to a per-wave LDS image,
// then every lane finishes 8 rows x one 16-byte chunk of channels, so residual loads and
// output stores are 16-B vectors and the GN statistics need one atomic pair per channel
// per wave.  `stage` = this wave's 64 x 68 float region (caller barriers before reuse).
// When the whole block tile lies in one image (blk_b >= 0) the GN statistics are reduced over
// the block's NWM wave rows in LDS (`red`, NWM x BN x 2 floats) and leave as one atomic pair per
// channel per block; every wave of the block must call this (it holds a barrier then).
// Block-level GN statistics flush: sum the NWM wave rows of `red` and add one (sum, sumsq)
// pair per channel to the slotted stats buffer.  Holds a barrier (all waves call it).
template <int NWM, int BN>
SNRSE_DEV void block_stats_flush(const ConvParams& p, const float* red, int blk_b, int blk_n0) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  for (int t = threadIdx.x; t < 2 * BN; t += blockDim.x) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NWM; ++w) a += red[w * 2 * BN + t];
    if (blk_n0 + (t >> 1) < p.Cout)
      unsafeAtomicAdd(&p.stats[stat_idx(blk_b, slot, blk_n0 + (t >> 1), p.Cout) + (t & 1)], (double)a);
  }
}

// nvalid < 64: only the wave's first nvalid rows are output pixels (a tile cut by the image's right
// edge, conv_x3h_kernel); the rest are skipped.
template <typename TO, int NWM, int BN, bool DEFER = false, int LA = 8>
SNRSE_DEV void epilogue_lds(const ConvParams& p, const f32x4 (&acc)[4][4], int mb, int nb, int lane, float* stage,
                            float* red, int wm, int blk_b, int blk_n0, int nvalid = 64) {
  constexpr int LDR = 68;  // padded row (floats): conflict-free C-layout writes
  constexpr int EPC = 16 / (int)sizeof(TO);  // outputs per 16-B chunk (8 bf16 / 4 f32)
  constexpr int NCH = 64 / EPC;              // chunks per row
  constexpr int RPP = 64 / NCH;              // rows per pass of 64 lanes
  const int lrow = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) stage[(i * 16 + lg * 4 + e) * LDR + j * 16 + lrow] = acc[i][j][e];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int HW = p.H * p.W;
  const int cc = lane % NCH, r0 = lane / NCH;
  const int n = nb + cc * EPC;
  const bool nok = n < p.Cout;  // Cout % 128 == 0 on these paths; kept for safety
  float bias[EPC], cw[EPC][4], cb[EPC];
#pragma unroll
  for (int k = 0; k < EPC; ++k) {
    bias[k] = (p.bias && nok) ? p.bias[n + k] : 0.f;
    cb[k] = 0.f;
    cw[k][0] = cw[k][1] = cw[k][2] = cw[k][3] = 0.f;
    if (p.comb_src && nok) {
      cw[k][0] = p.comb_w[(n + k) * 4 + 0]; cw[k][1] = p.comb_w[(n + k) * 4 + 1];
      cw[k][2] = p.comb_w[(n + k) * 4 + 2]; cw[k][3] = p.comb_w[(n + k) * 4 + 3];
      cb[k] = p.comb_b[n + k];
    }
  }
  const int m_last = min(mb + nvalid - 1, p.M - 1);
  const bool one_b = mb < p.M && (mb / HW) == (m_last / HW);
  const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  // A wave tile spanning several images (HW < 64: the 4 x 8 level of the C2 pyramid) with HW % RPP == 0:
  // every pass's RPP rows lie in one image, so the image is wave-uniform per pass and the statistics are
  // reduced per image run (one atomic pair per channel and image) instead of per element (per-element f64
  // atomics made a 1024-px 1x1 conv take 156 us, profiles/r05a_c2_dispatch_shapes.jsonl).
  const bool seg = p.stats && !one_b && HW % RPP == 0;
  int seg_b = -1;
  // the image's temb row joins the bias when the tile lies in one image; the residual / Combine inputs are
  // requested LA passes ahead of their use (LA of the 8 bf16 / 16 f32 passes; the caller sizes it to its
  // register budget), not one round trip per pass (with vmcnt in order, each such wait also drained the
  // earlier passes' stores)
  if (p.temb && one_b && nok) {
    const float* tb = p.temb + (size_t)(mb / HW) * p.temb_stride + n;
#pragma unroll
    for (int k = 0; k < EPC; ++k) bias[k] += tb[k];
  }
  constexpr int NPASS = 64 / RPP;
  static_assert(LA >= 1 && LA <= NPASS, "lookahead");
  u32x4 rpre[NPASS];
  f32x4 qpre[NPASS];
  auto epi_issue = [&](int pass) {
    const int row = r0 + pass * RPP;
    const int m = mb + row;
    if (m < p.M && nok && row < nvalid) {
      if (p.res) rpre[pass] = *(const u32x4*)((const TO*)p.res + (size_t)m * p.res_ld + n);
      if (p.comb_src) qpre[pass] = *(const f32x4*)(p.comb_src + (size_t)m * 4);
    }
  };
#pragma unroll
  for (int pass = 0; pass < LA; ++pass) epi_issue(pass);
  float s1[EPC], s2[EPC];
#pragma unroll
  for (int k = 0; k < EPC; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  auto seg_flush = [&]() {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
#pragma unroll
      for (int o = NCH; o < 64; o <<= 1) {
        s1[k] += __shfl_xor(s1[k], o, 64);
        s2[k] += __shfl_xor(s2[k], o, 64);
      }
    }
    if (r0 == 0 && nok && seg_b >= 0 && (long long)seg_b * HW < p.M) {
      const size_t base = stat_idx(seg_b, slot, n, p.Cout);
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        unsafeAtomicAdd(&p.stats[base + 2 * k], (double)s1[k]);
        unsafeAtomicAdd(&p.stats[base + 2 * k + 1], (double)s2[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < EPC; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  };
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass + LA < NPASS) epi_issue(pass + LA);
    const int row = r0 + pass * RPP;
    const int m = mb + row;
    if (seg) {
      const int bp = (mb + pass * RPP) / HW;  // wave-uniform
      if (bp != seg_b) {
        if (seg_b >= 0) seg_flush();
        seg_b = bp;
      }
    }
    if (m >= p.M || !nok || row >= nvalid) continue;
    float v[EPC];
    const float* sr = stage + row * LDR + cc * EPC;
#pragma unroll
    for (int k = 0; k < EPC; ++k) v[k] = sr[k] + bias[k];
    if (p.temb && !one_b) {
      const float* tb = p.temb + (size_t)(m / HW) * p.temb_stride + n;
#pragma unroll
      for (int k = 0; k < EPC; ++k) v[k] += tb[k];
    }
    if (p.res) {
      const u32x4 rv = rpre[pass];
      if constexpr (sizeof(TO) == 2) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += H16<TO>::lo(rv[k]);
          v[2 * k + 1] += H16<TO>::hi(rv[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += __uint_as_float(rv[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < EPC; ++k) v[k] *= p.out_scale;
    if (p.comb_src) {
      const f32x4 q = qpre[pass];
#pragma unroll
      for (int k = 0; k < EPC; ++k) v[k] += q[0] * cw[k][0] + q[1] * cw[k][1] + q[2] * cw[k][2] + q[3] * cw[k][3] + cb[k];
    }
    u32x4 o;
    if constexpr (sizeof(TO) == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = H16<TO>::pack(v[2 * k], v[2 * k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(v[k]);
    }
    if (p.epi_nt)  // (the fp32x3 halo GEMM under option x3_nt; 0 on every other launch through here)
      __builtin_nontemporal_store(o, (u32x4*)((TO*)p.out + (size_t)m * p.out_ld + n));
    else
      *(u32x4*)((TO*)p.out + (size_t)m * p.out_ld + n) = o;
    if (p.stats) {
      if (one_b || seg) {
#pragma unroll
        for (int k = 0; k < EPC; ++k) { s1[k] += v[k]; s2[k] = fmaf(v[k], v[k], s2[k]); }
      } else {
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const size_t o = stat_idx(m / HW, slot, n + k, p.Cout);
          unsafeAtomicAdd(&p.stats[o], (double)v[k]);
          unsafeAtomicAdd(&p.stats[o + 1], (double)v[k] * v[k]);
        }
      }
    }
  }
  if (seg && seg_b >= 0) seg_flush();
  if (p.stats && one_b) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
#pragma unroll
      for (int o = NCH; o < 64; o <<= 1) {
        s1[k] += __shfl_xor(s1[k], o, 64);
        s2[k] += __shfl_xor(s2[k], o, 64);
      }
    }
  }
  if (p.stats && blk_b >= 0) {  // uniform over the block
    if (r0 == 0) {
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        red[(wm * BN + nb - blk_n0 + cc * EPC + k) * 2] = s1[k];
        red[(wm * BN + nb - blk_n0 + cc * EPC + k) * 2 + 1] = s2[k];
      }
    }
    if constexpr (!DEFER) block_stats_flush<NWM, BN>(p, red, blk_b, blk_n0);
  } else if (p.stats && one_b && r0 == 0 && nok) {
    const size_t base = stat_idx(mb / HW, slot, n, p.Cout);
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      unsafeAtomicAdd(&p.stats[base + 2 * k], (double)s1[k]);
      unsafeAtomicAdd(&p.stats[base + 2 * k + 1], (double)s2[k]);
    }
  }
}

// Sum over the lanes of a wave that share lane % S (S = 8 or 16), every lane receives its sum:
// DPP row rotate by 8 inside the 16-lane rows (S = 8), then row-pair and half-wave swaps
// (v_permlane16_swap / v_permlane32_swap) -- VALU only, no ds_bpermute round trips.
template <int S>
SNRSE_DEV float sum_lanes_strided(float v) {
  static_assert(S == 8 || S == 16, "lane stride");
  if constexpr (S == 8)
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

// Lean LDS-staged epilogue of the halo kernels: the wave's 64 rows are 64 / TW segments of TW
// consecutive pixels in consecutive image rows of image `b` (pixel of wave row r: mb + r + (r / TW) *
// seg_skip, seg_skip = W - TW), and its 64 channels are in range (H % 4 == 0, W % TW == 0, Cout % 128 == 0
// there), so bias / temb / Combine weights are per-lane constants and no row or column masking is needed.
// Epilogue flags as a compile-time mask (EF >= 0: the v5 halo GEMM's common configurations, no
// per-pass branches) or read from the parameters at run time (EF = -1).

template <int TW>
SNRSE_DEV int epi_pix(int mb, int row, int seg_skip) {
  return TW == 64 ? mb + row : mb + row + (row / TW) * seg_skip;
}

// bias + temb of the lane's EPC channels of an epilogue_img call over channels nb .. nb + 63 of image b
template <typename TO, int EF>
SNRSE_DEV void epi_add(const ConvParams& p, int nb, int lane, int b, float (&add)[16 / sizeof(TO)]) {
  constexpr int EPC = 16 / (int)sizeof(TO);
  const int n = nb + (lane % (64 / EPC)) * EPC;
  const bool f_temb = EF < 0 ? p.temb != nullptr : (EF & EF_TEMB) != 0;
#pragma unroll
  for (int k = 0; k < EPC; ++k) add[k] = 0.f;
  if (p.bias) {  // (assigned, not added to 0: an add in the branch made the compiler wait for the load there)
#pragma unroll
    for (int k = 0; k < EPC; k += 4) {
      const f32x4 v = *(const f32x4*)(p.bias + n + k);
      add[k] = v[0]; add[k + 1] = v[1]; add[k + 2] = v[2]; add[k + 3] = v[3];
    }
  }
  if (f_temb) {
    const float* tb = p.temb + (size_t)b * p.temb_stride + n;
#pragma unroll
    for (int k = 0; k < EPC; ++k) add[k] += tb[k];
  }
}

// pre_add: the lane's bias + temb already loaded by the caller (epi_add), so its round trip overlaps the caller's
// drain before the epilogue instead of following it (the halo GEMMs load both halves' up front)
template <typename TO, int NWM, int BN, bool DEFER, int EF = EF_RT, int TW = 64, int LA = 8>
SNRSE_DEV void epilogue_img(const ConvParams& p, const f32x4 (&acc)[4][4], int mb, int nb, int lane, float* stage,
                            float* red, int wm, int b, int blk_n0, int seg_skip = 0,
                            const float* pre_add = nullptr) {
  const bool f_res = EF < 0 ? p.res != nullptr : (EF & EF_RES) != 0;
  const bool f_comb = EF < 0 ? p.comb_src != nullptr : (EF & EF_COMB) != 0;
  const bool f_stats = EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0;
  const bool f_nt = EF < 0 ? p.epi_nt != 0 : (EF & EF_NT) != 0;
  constexpr int LDR = 68;
  constexpr int EPC = 16 / (int)sizeof(TO);
  constexpr int NCH = 64 / EPC;
  constexpr int RPP = 64 / NCH;
  const int lrow = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) stage[(i * 16 + lg * 4 + e) * LDR + j * 16 + lrow] = acc[i][j][e];
  const int cc = lane % NCH, r0 = lane / NCH;
  const int n = nb + cc * EPC;
  float add[EPC];
  if (pre_add) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) add[k] = pre_add[k];
  } else {
    epi_add<TO, EF>(p, nb, lane, b, add);
  }
  float cw[EPC][4], cb[EPC];
  if (f_comb) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      const f32x4 w = *(const f32x4*)(p.comb_w + (size_t)(n + k) * 4);
      cw[k][0] = w[0]; cw[k][1] = w[1]; cw[k][2] = w[2]; cw[k][3] = w[3];
      cb[k] = p.comb_b[n + k];
    }
  }
  float s1[EPC], s2[EPC];
#pragma unroll
  for (int k = 0; k < EPC; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  // The residual / Combine inputs are requested LA passes ahead of their use (bf16: all 8 passes up front;
  // f32: LA of the 16, sized by the caller), so the passes do not wait on one HBM round trip each -- a wait
  // that, vmcnt being in order, also drained the earlier passes' stores (the fp32x3 halo GEMM's residual
  // convs did that 16 times per tile at one workgroup per CU).
  constexpr int NPASS = 64 / RPP;
  static_assert(LA >= 1 && LA <= NPASS, "lookahead");
  u32x4 rpre[NPASS];
  f32x4 qpre[NPASS];
  auto epi_issue = [&](int pass) {
    const size_t m = (size_t)epi_pix<TW>(mb, r0 + pass * RPP, seg_skip);
    if (f_res) rpre[pass] = *(const u32x4*)((const TO*)p.res + m * p.res_ld + n);
    if (f_comb) qpre[pass] = *(const f32x4*)(p.comb_src + m * 4);
  };
#pragma unroll
  for (int pass = 0; pass < LA; ++pass) epi_issue(pass);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (pass + LA < NPASS) epi_issue(pass + LA);
    const int row = r0 + pass * RPP;
    const size_t m = (size_t)epi_pix<TW>(mb, row, seg_skip);
    float v[EPC];
    const float* sr = stage + row * LDR + cc * EPC;
#pragma unroll
    for (int k = 0; k < EPC; ++k) v[k] = sr[k] + add[k];
    if (f_res) {
      const u32x4 rv = rpre[pass];
      if constexpr (sizeof(TO) == 2) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += H16<TO>::lo(rv[k]);
          v[2 * k + 1] += H16<TO>::hi(rv[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += __uint_as_float(rv[k]);
      }
    }
    if (p.out_scale != 1.f) {  // (uniform: Conv_0 and the other unscaled convs skip the multiply)
#pragma unroll
      for (int k = 0; k < EPC; ++k) v[k] *= p.out_scale;
    }
    if (f_comb) {
      const f32x4 q = qpre[pass];
#pragma unroll
      for (int k = 0; k < EPC; ++k) v[k] += q[0] * cw[k][0] + q[1] * cw[k][1] + q[2] * cw[k][2] + q[3] * cw[k][3] + cb[k];
    }
    u32x4 o;
    if constexpr (sizeof(TO) == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = H16<TO>::pack(v[2 * k], v[2 * k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(v[k]);
    }
    if (f_nt)  // option "epi_nt": streaming (non-temporal) output stores
      __builtin_nontemporal_store(o, (u32x4*)((TO*)p.out + m * p.out_ld + n));
    else
      *(u32x4*)((TO*)p.out + m * p.out_ld + n) = o;
    if (f_stats) {
#pragma unroll
      for (int k = 0; k < EPC; ++k) { s1[k] += v[k]; s2[k] = fmaf(v[k], v[k], s2[k]); }
    }
  }
  if (f_stats) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      s1[k] = sum_lanes_strided<NCH>(s1[k]);
      s2[k] = sum_lanes_strided<NCH>(s2[k]);
    }
    if (r0 == 0) {
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        red[(wm * BN + nb - blk_n0 + cc * EPC + k) * 2] = s1[k];
        red[(wm * BN + nb - blk_n0 + cc * EPC + k) * 2 + 1] = s2[k];
      }
    }
    if constexpr (!DEFER) block_stats_flush<NWM, BN>(p, red, b, blk_n0);
  }
}

template <typename TO, int FM, int FN>
SNRSE_DEV void epilogue(const ConvParams& p, const f32x4 (&acc)[FM][FN], int mb, int nb, int lane) {
  const int lrow = lane & 15, lg = lane >> 4;
  const int HW = p.H * p.W;
  const int m_last = min(mb + FM * 16, p.M) - 1;
  const bool one_b = mb < p.M && (mb / HW) == (m_last / HW);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nb + j * 16 + lrow;
    const bool nok = n < p.Cout;
    const float bn = (p.bias && nok) ? p.bias[n] : 0.f;
    float cw0 = 0.f, cw1 = 0.f, cw2 = 0.f, cw3 = 0.f, cb = 0.f;
    if (p.comb_src && nok) {
      cw0 = p.comb_w[n * 4 + 0]; cw1 = p.comb_w[n * 4 + 1];
      cw2 = p.comb_w[n * 4 + 2]; cw3 = p.comb_w[n * 4 + 3];
      cb = p.comb_b[n];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = mb + i * 16 + lg * 4 + e;
        if (m >= p.M || !nok) continue;
        float v = acc[i][j][e] + bn;
        if (p.temb) v += p.temb[(size_t)(m / HW) * p.temb_stride + n];
        if (p.res) v += Elem<TO>::to_f(((const TO*)p.res)[(size_t)m * p.res_ld + n]);
        v *= p.out_scale;
        if (p.comb_src) {
          const float* q = p.comb_src + (size_t)m * 4;
          v += q[0] * cw0 + q[1] * cw1 + q[2] * cw2 + q[3] * cw3 + cb;
        }
        ((TO*)p.out)[(size_t)m * p.out_ld + n] = Elem<TO>::from_f(v);
        if (p.stats) {
          if (one_b) {
            s1 += v;
            s2 = fmaf(v, v, s2);
          } else {
            const size_t o = stat_idx(m / HW, blockIdx.x & (SNRSE_STAT_SLOTS - 1), n, p.Cout);
            unsafeAtomicAdd(&p.stats[o], (double)v);
            unsafeAtomicAdd(&p.stats[o + 1], (double)v * v);
          }
        }
      }
    }
    if (p.stats && one_b) {
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lg == 0 && nok) {
        const size_t o = stat_idx(mb / HW, blockIdx.x & (SNRSE_STAT_SLOTS - 1), n, p.Cout);
        unsafeAtomicAdd(&p.stats[o], (double)s1);
        unsafeAtomicAdd(&p.stats[o + 1], (double)s2);
      }
    }
  }
}

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
  const int nbk = gridDim.x, bid = blockIdx.x;
  const int q8 = nbk >> 3, r8 = nbk & 7, xcd = bid & 7, pos = bid >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  // split-K (the small low-resolution levels of the fp32 path): the p.ksplit K ranges of one output
  // tile are adjacent logical ids, i.e. on one XCD
  const int ks = wg % p.ksplit, tl = wg / p.ksplit;
  const int m0 = (tl / p.ntn) * BM;
  const int n0 = (tl % p.ntn) * BN;
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

  const int kb = (int)((long long)ks * nk / p.ksplit), ke = (int)((long long)(ks + 1) * nk / p.ksplit);
  gload(kb);
  lstore(0);
  __syncthreads();

  const int lrow = lane & 15;
  const int lg = lane >> 4;
  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) & 1;
    if (kt + 1 < ke) gload(kt + 1);
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
    if (kt + 1 < ke) lstore(cur ^ 1);
    __syncthreads();
  }

#undef AS
#undef BS
  if (p.ksplit > 1) {  // raw fp32 partial sums of this K range; conv_splitk_finalize applies the epilogue
    float* const wsp = p.ws + (size_t)ks * p.M * p.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * TM + i * 16 + lg * 4 + e;
        if (m < p.M) {
#pragma unroll
          for (int j = 0; j < FN; ++j) wsp[(size_t)m * p.Cout + n0 + wn * TN + j * 16 + lrow] = acc[i][j][e];
        }
      }
    return;
  }
  epilogue<TO, FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, lane);
}

// ---------------------------------------------------------------------------------------
// Split-bf16 ("bf16x3") fp32 GEMM, the fast fp32 parity mode (dtype SNRSE_F32 with bf16 weights):
// fp32 activations, weights pre-split on the host into hi = bf16(w), lo = bf16(w - hi), stored per
// 32-element K-tile as one 128-B row [hi x 32 | lo x 32] ([Npad][2K] bf16).  The activation tile is
// split the same way in registers on its way to LDS, and each K-tile accumulates
//   A_hi B_hi + A_hi B_lo + A_lo B_hi
// with three v_mfma_f32_16x16x32_bf16 (exact bf16 products, fp32 accumulation): the dropped lo*lo
// term and the operands' residuals beyond 16 significant bits are ~2^-16 relative per product, and
// one K-tile costs 48 MFMA cycles per 16x16 output block instead of the 256 of the eight
// v_mfma_f32_16x16x4_f32 of the exact-fp32 kernel (measured: profiles/r03z_*).
// Same tile walk, split-K and epilogues as the v1 kernel above; LDS rows use the same swizzle, with
// the hi half in chunks 0-3 and the lo half in chunks 4-7.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_x3_kernel(ConvParams p) {
  constexpr int KT = 32;  // fp32 elements per K-tile
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int ROWS_PER_PASS = NT / 8;
  constexpr int A_LD = (BM + ROWS_PER_PASS - 1) / ROWS_PER_PASS;
  constexpr int B_LD = (BN + ROWS_PER_PASS - 1) / ROWS_PER_PASS;
  static_assert(BM % 16 == 0 && BN % 16 == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
#define AS(buf) (smem + (buf) * (BM * 128))
#define BS(buf) (smem + 2 * BM * 128 + (buf) * (BN * 128))

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nbk = gridDim.x, bid = blockIdx.x;
  const int q8 = nbk >> 3, r8 = nbk & 7, xcd = bid & 7, pos = bid >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int ks = wg % p.ksplit, tl = wg / p.ksplit;
  const int m0 = (tl / p.ntn) * BM;
  const int n0 = (tl % p.ntn) * BN;
  const int HW = p.H * p.W;
  const int Cin = p.C0 + p.C1;
  const int cblocks = Cin / KT;
  const int nk0 = p.ksize * p.ksize * cblocks;
  const int Csc_all = p.Csc + p.Csc1;
  const int nk = nk0 + (p.sc_src ? Csc_all / KT : 0);
  const int K1 = p.ksize * p.ksize * Cin;
  const int half = p.ksize >> 1;

  const int ch = tid & 7;  // A: fp32 elements 4ch..4ch+3 of the K-tile; B: 16-B chunk ch of the split row
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
    const float* src;
    int cs, cc, dy, dx;
    const bf16_t* wbase;
    int wld;
    if (kt < nk0) {
      const int tap = kt / cblocks;
      const int c = (kt - tap * cblocks) * KT;
      dy = tap / p.ksize - half;
      dx = tap % p.ksize - half;
      if (c < p.C0) { src = (const float*)p.src0; cs = p.C0; cc = c; }
      else { src = (const float*)p.src1; cs = p.C1; cc = c - p.C0; }
      wbase = (const bf16_t*)p.wgt + 2 * (tap * Cin + c);
      wld = 2 * K1;
    } else {
      const int c = (kt - nk0) * KT;
      if (c < p.Csc) { src = (const float*)p.sc_src; cs = p.Csc; cc = c; }
      else { src = (const float*)p.sc_src1; cs = p.Csc1; cc = c - p.Csc; }
      dy = 0; dx = 0;
      wbase = (const bf16_t*)p.sc_wgt + 2 * c;
      wld = 2 * Csc_all;
    }
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int hh = a_h[i] + dy, ww = a_w[i] + dx;
      const bool ok = a_ok[i] && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
      if (ok) ra[i] = *(const u32x4*)(src + ((size_t)(a_b[i] * p.H + hh) * p.W + ww) * cs + cc + ch * 4);
      else ra[i] = u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int r = (tid >> 3) + i * ROWS_PER_PASS;
      if (r < BN) rb[i] = *(const u32x4*)(wbase + (size_t)(n0 + r) * wld + ch * 8);
    }
  };
  // A: 4 fp32 -> 4 hi bf16 (8 B, hi half) + 4 lo bf16 (8 B, lo half); B: the pre-split chunk as is
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int r = (tid >> 3) + i * ROWS_PER_PASS;
      if (r < BM) {
        const u32x4 v = ra[i];
        const uint32_t h01 = pack_bf16x2(__uint_as_float(v[0]), __uint_as_float(v[1]));
        const uint32_t h23 = pack_bf16x2(__uint_as_float(v[2]), __uint_as_float(v[3]));
        const uint32_t l01 = pack_bf16x2(__uint_as_float(v[0]) - __uint_as_float(h01 << 16),
                                         __uint_as_float(v[1]) - __uint_as_float(h01 & 0xffff0000u));
        const uint32_t l23 = pack_bf16x2(__uint_as_float(v[2]) - __uint_as_float(h23 << 16),
                                         __uint_as_float(v[3]) - __uint_as_float(h23 & 0xffff0000u));
        typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
        *(u32x2*)(AS(buf) + swz(r, ch >> 1) + (ch & 1) * 8) = u32x2{h01, h23};
        *(u32x2*)(AS(buf) + swz(r, 4 + (ch >> 1)) + (ch & 1) * 8) = u32x2{l01, l23};
      }
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

  const int kb = (int)((long long)ks * nk / p.ksplit), ke = (int)((long long)(ks + 1) * nk / p.ksplit);
  gload(kb);
  lstore(0);
  __syncthreads();

  const int lrow = lane & 15;
  const int lg = lane >> 4;
  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) & 1;
    if (kt + 1 < ke) gload(kt + 1);
    u32x4 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      ah[i] = *(const u32x4*)(AS(cur) + swz(wm * TM + i * 16 + lrow, lg));
      al[i] = *(const u32x4*)(AS(cur) + swz(wm * TM + i * 16 + lrow, 4 + lg));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = *(const u32x4*)(BS(cur) + swz(wn * TN + j * 16 + lrow, lg));
      bl[j] = *(const u32x4*)(BS(cur) + swz(wn * TN + j * 16 + lrow, 4 + lg));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bh[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(al[i], bh[j], acc[i][j]);
      }
    if (kt + 1 < ke) lstore(cur ^ 1);
    __syncthreads();
  }
#undef AS
#undef BS
  if (p.ksplit > 1) {
    float* const wsp = p.ws + (size_t)ks * p.M * p.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * TM + i * 16 + lg * 4 + e;
        if (m < p.M) {
#pragma unroll
          for (int j = 0; j < FN; ++j) wsp[(size_t)m * p.Cout + n0 + wn * TN + j * 16 + lrow] = acc[i][j][e];
        }
      }
    return;
  }
  if constexpr (TM == 64 && TN == 64) {
    // LDS-staged epilogue: 16-B output stores, one statistics atomic pair per channel per block
    const int b_lo = m0 / HW, b_hi = (min(m0 + BM, p.M) - 1) / HW;
    epilogue_lds<float, WM, BN, false, 4>(p, acc, m0 + wm * TM, n0 + wn * TN, lane, (float*)(smem + wid * (64 * 68 * 4)),
                                (float*)(smem + WM * WN * (64 * 68 * 4)), wm, b_lo == b_hi ? b_lo : -1, n0);
  } else {
    epilogue<float, FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, lane);
  }
}

// ---------------------------------------------------------------------------------------
// Halo form of the split-bf16 fp32 GEMM (3x3, H % 4 == 0, W % 64 == 0): the register-staged kernel
// above re-reads every input pixel from L2 once per tap (9x); here a workgroup owns a 4-row x 64-px
// output tile x 128 couts and stages, per 32-channel chunk, the tile's (4+2) x (64+2) halo ONCE in
// LDS as split hi / lo bf16 rows (128 B: hi chunks 0-3, lo chunks 4-7, swz() layout), double
// buffered so chunk c+1's halo is fetched into registers during chunk c's first tap and stored after
// its second -- no barrier of its own.  Weights run through a 3-slot ring of one tap each (128 couts x
// 128 B of pre-split rows = 16 KB, LDS-DMA with the swizzle applied on the source chunk), issued two
// taps ahead.  8 waves: wave w computes image row w & 3 (64 px) x couts (w >> 2) * 64 .. + 63, i.e.
// 4 x 4 fragments x 3 MFMAs per tap.  Shortcut K (the fused 1x1 Conv_2) runs as chunks of one (center)
// tap over the shortcut source's halo.  LDS: 2 x 50.7 KB halo + 48 KB ring = 147 KB, one workgroup per
// CU (2 waves per SIMD); the epilogue reuses it as the per-wave staging of epilogue_lds.
namespace x3h {
constexpr int TH = 4, TW = 64, HC = TW + 2, HROWS = (TH + 2) * HC;  // 396 halo rows
constexpr int HBYTES = HROWS * 128;                                 // 50,688
constexpr int HJ = (HROWS * 8 + 511) / 512;                         // 16-B halo loads per thread: 7
constexpr int TAPB = 128 * 128;                                     // one tap's weights: 16 KB
constexpr size_t LDS_MAIN = 2 * (size_t)HBYTES + 3 * (size_t)TAPB;
constexpr size_t LDS_EPI = 8 * (64 * 68 * 4) + 4 * 128 * 2 * 4;
constexpr size_t LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
}  // namespace x3h
// the same geometry for tile width TW (64: 4 x 64 px, the namespace above; 32: 8 x 32 px, 340 halo rows per 256
// pixels instead of 396 -- 14 % less halo to load, split and GroupNorm per output, as v5's 8 x 32 form)
template <int TW_, int SPR_ = 1>
struct X3G {
  static constexpr int TW = TW_, TH = 256 / TW_, HC = TW_ + 2, HROWS = (TH + 2) * HC;
  static constexpr int HBYTES = HROWS * 128, HJ = (HROWS * 8 + 511) / 512, TAPB = x3h::TAPB;
  static constexpr int RW = 64 / TW_;  // image rows of a wave's 64 pixels
  // weight ring: 3 one-tap slots, or (SPR 2, the pair schedule) 2 two-tap slots
  static constexpr size_t LDS_MAIN = 2 * (size_t)HBYTES + (SPR_ == 2 ? 4 : 3) * (size_t)TAPB;
  static constexpr size_t LDS = LDS_MAIN > x3h::LDS_EPI ? LDS_MAIN : x3h::LDS_EPI;
};

// s_waitcnt vmcnt(n) for the counts the x3h schedule produces (anything else waits for all)
SNRSE_DEV void x3h_vm_wait(int n) {
  switch (n) {
#define SNRSE_X3H_VM(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    SNRSE_X3H_VM(2) SNRSE_X3H_VM(6) SNRSE_X3H_VM(7) SNRSE_X3H_VM(8) SNRSE_X3H_VM(9) SNRSE_X3H_VM(10)
    SNRSE_X3H_VM(11) SNRSE_X3H_VM(12) SNRSE_X3H_VM(14) SNRSE_X3H_VM(16) SNRSE_X3H_VM(18) SNRSE_X3H_VM(20)
#undef SNRSE_X3H_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// GNM: GroupNorm prologue of the main input as in the bf16 halo kernel (0 none, 1 affine, 2 affine +
// SiLU), applied once per halo element while it is split: the fp32 mode's gn_act pass disappears.
// SPR: 0 one phase per tap, the next chunk's halo stored in one go; 1 the same, stored one piece per tap; 2 (round 5,
// the pair schedule: TW 32, an even number of main chunks) TWO taps per phase -- half the barriers -- over a 2-slot
// ring of 2-tap weight slots, the main chunks in pairs (18 taps = 9 phases with compile-time taps), the next chunk's
// halo pieces stored after its taps 2..7
template <int GNM, int SPR, int TWV, int EF = EF_RT>
__global__ __launch_bounds__(512) void conv_x3h_kernel(ConvParams p) {
  using G = X3G<TWV, SPR>;
  constexpr int TH = G::TH, TW = G::TW, HC = G::HC, HROWS = G::HROWS, HBYTES = G::HBYTES, HJ = G::HJ;
  constexpr int TAPB = G::TAPB, RW = G::RW;
  constexpr int HOPS = HJ + (GNM > 0 ? 2 : 0);  // vector-memory ops of one halo prefetch per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ring = smem + 2 * HBYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 3, wc = wid >> 2;
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int n0 = (g % p.ntn) * 128;
  int tile = g / p.ntn;
  const int ntw = (p.W + TW - 1) / TW, nth = p.H / TH;  // the last tile column may be cut by the image edge
  const int w0 = (tile % ntw) * TW;
  tile /= ntw;
  const int h0 = (tile % nth) * TH;
  const int bb = tile / nth;

  const int Cin = p.C0 + p.C1;
  const int cbm = Cin / 32;
  const int Csc_all = p.Csc + p.Csc1;
  const int cbs = p.sc_src ? Csc_all / 32 : 0;
  const int ncb = cbm + cbs;
  const int nq = 9 * cbm + cbs;
  const int K1 = 9 * Cin;

  // this thread's halo pieces: halo row (tid + 512 j) >> 3, 16-B fp32 chunk tid & 7 (4 channels); pixels
  // outside the image (the padding ring, and the columns past a cut tile's edge) load as zero
  const int hch = tid & 7;
  int hpix[HJ];
  bool hok[HJ];
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int hr = (tid + 512 * j) >> 3;
    const int hy = hr / HC, hx = hr - hy * HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    hok[j] = hr < HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
    hpix[j] = (bb * p.H + ih) * p.W + iw;
  }
  u32x4 hv[HJ];
  f32x4 gsc, gsh;  // GroupNorm scale / shift of this thread's 4 channels of the prefetched chunk
  auto halo_load = [&](int c) {
    const void* base;
    long long bytes;
    int cs, cc;
    if (c < cbm) {
      const int ch = c * 32;
      if (ch < p.C0) { base = p.src0; bytes = p.bytes0; cs = p.C0; cc = ch; }
      else { base = p.src1; bytes = p.bytes1; cs = p.C1; cc = ch - p.C0; }
    } else {
      const int ch = (c - cbm) * 32;
      if (ch < p.Csc) { base = p.sc_src; bytes = p.sc_bytes0; cs = p.Csc; cc = ch; }
      else { base = p.sc_src1; bytes = p.sc_bytes1; cs = p.Csc1; cc = ch - p.Csc; }
    }
    const __amdgpu_buffer_rsrc_t r = make_rsrc(base, bytes);
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int voff = hok[j] ? (hpix[j] * cs + cc + hch * 4) * 4 : (int)0x80000000;  // outside: zero padding
      hv[j] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    }
    if constexpr (GNM > 0) {  // issued for shortcut chunks too (unused there): a fixed count per prefetch
      const long long gb = (long long)p.B * Cin * 4;
      const int go = ((bb * Cin + (c < cbm ? c : 0) * 32 + hch * 4) * 4);
      gsc = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(p.gn_scale, gb), go, 0, 0));
      gsh = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(p.gn_shift, gb), go, 0, 0));
    }
  };
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  auto halo_store = [&](int c) {  // chunk c's prefetched halo -> halo buffer c & 1
    char* const hb = smem + (c & 1) * HBYTES;
    const bool tr = GNM > 0 && c < cbm;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int hr = (tid + 512 * j) >> 3;
      if (j == HJ - 1 && hr >= HROWS) break;
      float x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = __uint_as_float(hv[j][k]);
      if constexpr (GNM > 0) {
        if (tr) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float y = fmaf(x[k], gsc[k], gsh[k]);
            x[k] = hok[j] ? (GNM == 2 ? silu(y) : y) : 0.f;  // outside the image: the conv's zero padding
          }
        }
      }
      const uint32_t h01 = pack_bf16x2(x[0], x[1]);
      const uint32_t h23 = pack_bf16x2(x[2], x[3]);
      const uint32_t l01 = pack_bf16x2(x[0] - __uint_as_float(h01 << 16), x[1] - __uint_as_float(h01 & 0xffff0000u));
      const uint32_t l23 = pack_bf16x2(x[2] - __uint_as_float(h23 << 16), x[3] - __uint_as_float(h23 & 0xffff0000u));
      *(u32x2*)(hb + swz(hr, hch >> 1) + (hch & 1) * 8) = u32x2{h01, h23};
      *(u32x2*)(hb + swz(hr, 4 + (hch >> 1)) + (hch & 1) * 8) = u32x2{l01, l23};
    }
  };
  // SPR: one halo piece j (this thread's 16-B fp32 vector of halo row (tid + 512 j) >> 3) of the prefetched
  // chunk, split (+ GroupNorm) and stored branch-free -- placed after a tap's MFMAs so the scheduler can
  // interleave its VALU with them; tr = the chunk is a main-input chunk (GroupNorm applies)
  auto halo_piece = [&](char* hb, int j, bool tr) {
    const int hr = (tid + 512 * j) >> 3;
    float x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = __uint_as_float(hv[j][k]);
    if constexpr (GNM > 0) {
      const uint32_t keep = tr ? 0u : ~0u, zero = (hok[j] || !tr) ? ~0u : 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float y = fmaf(x[k], gsc[k], gsh[k]);
        const float z = GNM == 2 ? silu(y) : y;
        x[k] = __uint_as_float(((__float_as_uint(z) & ~keep) | (__float_as_uint(x[k]) & keep)) & zero);
      }
    }
    const uint32_t h01 = pack_bf16x2(x[0], x[1]);
    const uint32_t h23 = pack_bf16x2(x[2], x[3]);
    const uint32_t l01 = pack_bf16x2(x[0] - __uint_as_float(h01 << 16), x[1] - __uint_as_float(h01 & 0xffff0000u));
    const uint32_t l23 = pack_bf16x2(x[2] - __uint_as_float(h23 << 16), x[3] - __uint_as_float(h23 & 0xffff0000u));
    if (j < HJ - 1 || hr < HROWS) {
      *(u32x2*)(hb + swz(hr, hch >> 1) + (hch & 1) * 8) = u32x2{h01, h23};
      *(u32x2*)(hb + swz(hr, 4 + (hch >> 1)) + (hch & 1) * 8) = u32x2{l01, l23};
    }
  };
  // phase q -> (chunk, tap): main chunks 9 taps each, then the shortcut chunks' center tap
  auto phase_chunk = [&](int q) { return q < 9 * cbm ? q / 9 : cbm + (q - 9 * cbm); };
  auto phase_tap = [&](int q) { return q < 9 * cbm ? q - (q / 9) * 9 : 4; };
  auto first_with_next = [&](int q) {  // phase q starts a chunk that has a successor (its halo prefetch)
    if (q < 0 || q >= nq) return false;
    const int c = phase_chunk(q);
    return (c < cbm ? phase_tap(q) == 0 : true) && c + 1 < ncb;
  };
  // weights of phase q -> ring slot q % 3: 16 pieces of 1 KB (8 rows x 128 B), 2 per wave
  auto wload = [&](int q) {  // q >= nq (SPR's branch-free schedule): zero-filling out-of-range loads
    const bool oob = q >= nq;
    char* dst = ring + (q % 3) * TAPB;  // slot q % 3 even when out of range: never read again
    if (oob) q = nq - 1;
    const int c = phase_chunk(q), tp = phase_tap(q);
    const bool mainw = c < cbm;
    const int wld = mainw ? 2 * K1 : 2 * Csc_all;                      // bf16 elements per row
    const int koff = mainw ? 2 * (tp * Cin + c * 32) : 2 * ((c - cbm) * 32);
    const __amdgpu_buffer_rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    const int rl = lane >> 3, sl = lane & 7;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pc = wid * 2 + k;
      const int row = pc * 8 + rl;
      const unsigned voff = oob ? 0x80000000u : (unsigned)(((n0 + row) * wld + koff + (sl ^ (row & 7)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16,
                                               voff, 0, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one tap's weights (chunk c, tap tp) -> dst: 16 pieces of 1 KB, 2 per wave (the pair schedule's DMA)
  auto wtap = [&](int c, int tp, char* dst) {
    const bool mainw = c < cbm;
    const int wld = mainw ? 2 * K1 : 2 * Csc_all;
    const int koff = mainw ? 2 * (tp * Cin + c * 32) : 2 * ((c - cbm) * 32);
    const __amdgpu_buffer_rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    const int rl = lane >> 3, sl = lane & 7;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pc = wid * 2 + k;
      const int row = pc * 8 + rl;
      const unsigned voff = (unsigned)(((n0 + row) * wld + koff + (sl ^ (row & 7)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16,
                                               voff, 0, 0, 0);
    }
  };
  if constexpr (SPR == 2) {
    wtap(0, 0, ring);
    wtap(0, 1, ring + TAPB);
  } else {
    wload(0);
    if (nq > 1) wload(1);
  }
  halo_load(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  halo_store(0);
  const int lrow = lane & 15, lg = lane >> 4;
  // one tap's fragment reads + 48 MFMAs from halo buffer hb and ring slot sb
  auto tap_mfma = [&](const char* hb, const char* sb, int tp) {
    const int dy = tp / 3 - 1, dx = tp - (tp / 3) * 3 - 1;
    // fragment i: the wave's pixels 16 i .. 16 i + 15 = image row wr RW + 16 i / TW, columns (16 i) % TW ..
    const int hbase = (wr * RW + dy + 1) * HC + dx + 1 + lrow;
    u32x4 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hr = hbase + (16 * i / TW) * HC + (16 * i) % TW;
      ah[i] = *(const u32x4*)(hb + swz(hr, lg));
      al[i] = *(const u32x4*)(hb + swz(hr, 4 + lg));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = *(const u32x4*)(sb + swz(wc * 64 + j * 16 + lrow, lg));
      bl[j] = *(const u32x4*)(sb + swz(wc * 64 + j * 16 + lrow, 4 + lg));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bh[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(al[i], bh[j], acc[i][j]);
      }
  };
  if constexpr (SPR == 2) {
    // The pair schedule.  Phase k of a chunk pair (c0, c1 = c0 + 1) runs taps s = 2k, 2k + 1 of the pair's 18
    // (chunk c0 + s / 9, tap s % 9) from ring slot `so`; at its top it waits for its own DMA (issued at the top of
    // phase k - 1; the halo prefetch issued behind that DMA at phase 0 / 4 may stay in flight), then issues the next
    // phase's DMA.  The halo of chunk c + 1 is prefetched at the phase holding tap (c, 0) and stored, split (+
    // GroupNorm), after the taps (c, 4 .. 7) into the other halo buffer (HJ = 6 pieces at TW 32); the last piece lands
    // a barrier before tap (c + 1, 0) is read.  Then the shortcut chunks, one tap per phase.
    static_assert(TW == 32 && HJ == 6, "pair schedule: 8 x 32 tiles, 6 halo pieces per thread");
    constexpr int SLOT2 = 2 * TAPB;
    int so = 0;
    auto wait_vm = [](int n) {  // vmcnt(n) for n in {0, HOPS} (compile-time encodings)
      if (n == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HOPS) : "memory");
    };
    for (int c0 = 0; c0 < cbm; c0 += 2) {
      const int c1 = c0 + 1;
      const bool more = c0 + 2 < cbm;        // another pair follows
      const bool pf1 = more || cbs > 0;       // a chunk follows c1 (main or shortcut): prefetched at phase 4
      bool infl = false;                       // halo loads issued behind the current phase's DMA
      static_for<9>([&](auto K) {
        constexpr int k = decltype(K)::value;
        constexpr int sa = 2 * k, sb = 2 * k + 1;
        constexpr int da = sa / 9, ta = sa % 9, db = sb / 9, tb = sb % 9;
        wait_vm(infl ? HOPS : 0);
        __builtin_amdgcn_s_barrier();
        // the next phase's DMA into the other slot
        char* const nxt = ring + (SLOT2 - so);
        if constexpr (k < 8) {
          wtap(c0 + (2 * k + 2) / 9, (2 * k + 2) % 9, nxt);
          wtap(c0 + (2 * k + 3) / 9, (2 * k + 3) % 9, nxt + TAPB);
        } else {
          if (more) {
            wtap(c0 + 2, 0, nxt);
            wtap(c0 + 2, 1, nxt + TAPB);
          } else if (cbs > 0) {
            wtap(cbm, 4, nxt);
          }
        }
        infl = false;
        if constexpr (k == 0) {
          halo_load(c1);
          infl = true;
        }
        if constexpr (k == 4) {
          if (pf1) {
            halo_load(c1 + 1);
            infl = true;
          }
        }
        const char* const sl_ = ring + so;
        // tap A, then its halo pieces; tap B, then its pieces.  The 6 pieces of chunk c's successor go after taps
        // (c, 4) [0, 1], (c, 5) [2, 3], (c, 6) [4], (c, 7) [5]: taps 4.. lie in the phases whose top wait already
        // drained the prefetch (phases 2 and 6), so the loads have 4 taps of cover and no piece waits on them (pieces
        // after taps 2 and 3 waited for HBM inside phases 1 / 5: ~12 % of the launch, profiles/r05g_x3h_ablations)
        auto piece_after = [&](int d, int t) {
          const int c = c0 + d;
          if (t < 4 || t > 7) return;
          if (d == 1 && !pf1) return;
          char* const nb_ = smem + ((c + 1) & 1) * HBYTES;
          const bool tr = c + 1 < cbm;
          if (t == 4) { halo_piece(nb_, 0, tr); halo_piece(nb_, 1, tr); }
          if (t == 5) { halo_piece(nb_, 2, tr); halo_piece(nb_, 3, tr); }
          if (t == 6) halo_piece(nb_, 4, tr);
          if (t == 7) halo_piece(nb_, 5, tr);
        };
        tap_mfma(smem + ((c0 + da) & 1) * HBYTES, sl_, ta);
        piece_after(da, ta);
        __builtin_amdgcn_sched_barrier(0);  // one tap at a time (hoisted fragment reads of the next tap spill)
        tap_mfma(smem + ((c0 + db) & 1) * HBYTES, sl_ + TAPB, tb);
        piece_after(db, tb);
        __builtin_amdgcn_sched_barrier(0);
        so = SLOT2 - so;
      });
    }
    // the shortcut chunks: one tap (the center) per phase; chunk cbm's halo was stored during the last pair
    for (int c = cbm; c < ncb; ++c) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (c + 1 < ncb) wtap(c + 1, 4, ring + (SLOT2 - so));
      if (c + 1 < ncb) halo_load(c + 1);
      tap_mfma(smem + (c & 1) * HBYTES, ring + so, 4);
      if (c + 1 < ncb) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        char* const nb_ = smem + ((c + 1) & 1) * HBYTES;
#pragma unroll
        for (int j = 0; j < HJ; ++j) halo_piece(nb_, j, false);
      }
      so = SLOT2 - so;
    }
  } else if constexpr (SPR == 1) {
    // Branch-free schedule: every phase issues its DMA two phases ahead (zero-filling past the end), every
    // chunk prefetches the next one's halo at its first phase (the last chunk re-reads itself into the
    // unused buffer), so the ops issued after DMA(q) are DMA(q+1) plus the halo prefetches of phases q-1 /
    // q-2 when those start a chunk.  Main chunks: the prefetched halo is stored one piece per tap, after
    // the MFMAs of taps 2..8 (the wait at the top of tap 2 covers the halo loads).
    int q = 0;
    for (int c = 0; c < cbm; ++c) {
      const bool tr = c + 1 < cbm;
      char* const nb_ = smem + ((c + 1) & 1) * HBYTES;
      const char* const hb = smem + (c & 1) * HBYTES;
#pragma unroll
      for (int tp = 0; tp < 9; ++tp, ++q) {
        // DMA(q): ops issued after it are DMA(q+1) and, at tap 1, this chunk's halo prefetch; at tap 2 the
        // prefetch is waited for too (its pieces are stored from this tap on)
        if (tp == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + HOPS) : "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        wload(q + 2);
        if (tp == 0) halo_load(c + 1 < ncb ? c + 1 : c);
        tap_mfma(hb, ring + (q % 3) * TAPB, tp);
        if (tp >= 2 && tp - 2 < HJ) halo_piece(nb_, tp - 2, tr);
      }
    }
    for (int c = cbm; c < ncb; ++c, ++q) {
      const int qa = q - 2, qb = q - 1;  // phase-first flags of the two previous phases
      const bool fa = qa >= 0 && (qa >= 9 * cbm || qa % 9 == 0), fb = qb >= 0 && (qb >= 9 * cbm || qb % 9 == 0);
      x3h_vm_wait(2 + HOPS * (int)fa + HOPS * (int)fb);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      wload(q + 2);
      halo_load(c + 1 < ncb ? c + 1 : c);
      tap_mfma(smem + (c & 1) * HBYTES, ring + (q % 3) * TAPB, 4);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      char* const nb_ = smem + ((c + 1) & 1) * HBYTES;
#pragma unroll
      for (int j = 0; j < HJ; ++j) halo_piece(nb_, j, false);
    }
  } else
  for (int q = 0; q < nq; ++q) {
    const int c = phase_chunk(q), tp = phase_tap(q);
    // DMA(q) done: wait for all but the ops issued after it (see the schedule in the header comment)
    x3h_vm_wait(HOPS * (int)first_with_next(q - 2) + 2 * (int)(q + 1 < nq) + HOPS * (int)first_with_next(q - 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (q + 2 < nq) wload(q + 2);
    const bool pre = first_with_next(q);
    if (pre) halo_load(c + 1);
    const char* hb = smem + (c & 1) * HBYTES;
    const char* sb = ring + (q % 3) * TAPB;
    const int dy = tp / 3 - 1, dx = tp - (tp / 3) * 3 - 1;
    // fragment i: the wave's pixels 16 i .. 16 i + 15 = image row wr RW + 16 i / TW, columns (16 i) % TW ..
    const int hbase = (wr * RW + dy + 1) * HC + dx + 1 + lrow;
    u32x4 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hr = hbase + (16 * i / TW) * HC + (16 * i) % TW;
      ah[i] = *(const u32x4*)(hb + swz(hr, lg));
      al[i] = *(const u32x4*)(hb + swz(hr, 4 + lg));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = *(const u32x4*)(sb + swz(wc * 64 + j * 16 + lrow, lg));
      bl[j] = *(const u32x4*)(sb + swz(wc * 64 + j * 16 + lrow, 4 + lg));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bh[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16_t>(al[i], bh[j], acc[i][j]);
      }
    // the next chunk's halo goes to the other buffer after this chunk's second tap (its first and only
    // one for a shortcut chunk); only the DMAs issued since the halo loads may still be in flight
    const int q0 = q < 9 * cbm ? q - tp : q;  // first phase of this chunk
    const bool last_of_chunk = c < cbm ? tp == 8 : true;
    const bool store_now = c + 1 < ncb && (c < cbm ? tp == 1 : true);
    if (store_now) {
      x3h_vm_wait(q == q0 ? 0 : 2 * (int)(q0 + 3 < nq));
      halo_store(c + 1);
    }
    (void)last_of_chunk;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // LDS is reused as the epilogue staging area
  const int mb = (bb * p.H + h0 + wr * RW) * p.W + w0;
  if constexpr (TW == 64)
    epilogue_lds<float, 4, 128>(p, acc, mb, n0 + wc * 64, lane, (float*)(smem + wid * (64 * 68 * 4)),
                                (float*)(smem + 8 * (64 * 68 * 4)), wr, bb, n0, min(TW, p.W - w0));
  else  // two 32-px row segments per wave (W % 32 == 0: no cut tiles)
    epilogue_img<float, 4, 128, false, EF, TW>(p, acc, mb, n0 + wc * 64, lane, (float*)(smem + wid * (64 * 68 * 4)),
                                                 (float*)(smem + 8 * (64 * 68 * 4)), wr, bb, n0, p.W - TW);
}

// ---------------------------------------------------------------------------------------
// v2 (bf16): 8 waves, 64x64 wave tiles, operands streamed global->LDS by buffer_load...lds
// (LDS-DMA, no VGPR staging), 3-stage ring with counted vmcnt + raw s_barrier so two
// K-tiles stay in flight across the barrier.  Zero padding of the 3x3 halo comes from the
// buffer's range check (an out-of-range voffset loads 0).  The LDS image is lane-linear per
// DMA instruction; the chunk swizzle is applied to the per-lane SOURCE address and the
// same XOR on the ds_read (conflict-free 16-row fragment reads).
template <int BM, int BN, typename T, typename TO>
__global__ __launch_bounds__(512) void conv_glds_kernel(ConvParams p) {
  constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == 8, "8 waves");
  constexpr int FM = 4, FN = 4, TM = 64, TN = 64;
  constexpr int STAGES = 3;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int AJ = BM / 64, BJ = BN / 64;  // DMA instructions per wave per stage
  constexpr int KT = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  // XCD-aware bijective remap: consecutive logical tiles share an XCD (its L2 holds the halo
  // rows and the weight tile they all re-read); N-tiles of one M-tile are adjacent.
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  // split-K: the p.ksplit K ranges of one output tile are adjacent logical ids (same XCD)
  const int ks = wg % p.ksplit, tl = wg / p.ksplit;
  const int m0 = (tl / p.ntn) * BM;
  const int n0 = (tl % p.ntn) * BN;

  const int HW = p.H * p.W;
  const int Cin = p.C0 + p.C1;
  const int cblocks = Cin / KT;
  const int nk0 = p.ksize * p.ksize * cblocks;
  const int Csc_all = p.Csc + p.Csc1;
  const int nk = nk0 + (p.sc_src ? Csc_all / KT : 0);
  const int K1 = p.ksize * p.ksize * Cin;
  const int half = p.ksize >> 1;
  const int slot = lane & 7;

  int a_pix[AJ], a_h[AJ], a_w[AJ], a_ch[AJ];
  bool a_ok[AJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int row = (wid * AJ + j) * 8 + (lane >> 3);
    const int m = m0 + row;
    a_ok[j] = m < p.M;
    const int mm = a_ok[j] ? m : 0;
    const int b = mm / HW, rem = mm - b * HW;
    a_h[j] = rem / p.W;
    a_w[j] = rem - a_h[j] * p.W;
    a_pix[j] = mm;
    a_ch[j] = slot ^ (row & 7);
  }

  // one K-tile -> one LDS stage.  Every selector below depends only on kt (wave-uniform),
  // and the buffer base / extent go through readfirstlane so the descriptor lives in SGPRs
  // (no waterfall loop around the DMA, guide T20).
#define SNRSE_ISSUE(KT_, STAGE_)                                                                      \
  do {                                                                                              \
    const int kt_ = (KT_);                                                                          \
    char* sa_ = smem + (STAGE_) * STAGE;                                                            \
    char* sb_ = sa_ + A_BYTES;                                                                      \
    int cs_, cc_, dy_, dx_, wld_, koff_;                                                            \
    const void* abase_;                                                                             \
    long long abytes_;                                                                              \
    const void* wbase_;                                                                             \
    long long wbytes_;                                                                              \
    if (kt_ < nk0) {                                                                                \
      const int tap_ = kt_ / cblocks;                                                               \
      const int c_ = (kt_ - tap_ * cblocks) * KT;                                                   \
      dy_ = tap_ / p.ksize - half;                                                                  \
      dx_ = tap_ - (tap_ / p.ksize) * p.ksize - half;                                               \
      const bool u1_ = c_ >= p.C0;                                                                  \
      abase_ = u1_ ? p.src1 : p.src0;                                                               \
      abytes_ = u1_ ? p.bytes1 : p.bytes0;                                                          \
      cs_ = u1_ ? p.C1 : p.C0;                                                                      \
      cc_ = u1_ ? c_ - p.C0 : c_;                                                                   \
      wbase_ = p.wgt;                                                                               \
      wbytes_ = p.wbytes;                                                                           \
      wld_ = K1;                                                                                    \
      koff_ = tap_ * Cin + c_;                                                                      \
    } else {                                                                                        \
      const int c_ = (kt_ - nk0) * KT;                                                              \
      const bool u1_ = c_ >= p.Csc;                                                                 \
      abase_ = u1_ ? p.sc_src1 : p.sc_src;                                                          \
      abytes_ = u1_ ? p.sc_bytes1 : p.sc_bytes0;                                                    \
      cs_ = u1_ ? p.Csc1 : p.Csc;                                                                   \
      cc_ = u1_ ? c_ - p.Csc : c_;                                                                  \
      dy_ = 0;                                                                                      \
      dx_ = 0;                                                                                      \
      wbase_ = p.sc_wgt;                                                                            \
      wbytes_ = p.sc_wbytes;                                                                        \
      wld_ = Csc_all;                                                                               \
      koff_ = c_;                                                                                   \
    }                                                                                               \
    const __amdgpu_buffer_rsrc_t ra_ = make_rsrc(abase_, abytes_);                                  \
    const __amdgpu_buffer_rsrc_t rb_ = make_rsrc(wbase_, wbytes_);                                  \
    const int shift_ = dy_ * p.W + dx_;                                                             \
    _Pragma("unroll") for (int j = 0; j < AJ; ++j) {                                                \
      const int hh_ = a_h[j] + dy_, ww_ = a_w[j] + dx_;                                             \
      const bool ok_ = a_ok[j] && hh_ >= 0 && hh_ < p.H && ww_ >= 0 && ww_ < p.W;                   \
      const unsigned voff_ =                                                                        \
          ok_ ? (unsigned)(((a_pix[j] + shift_) * cs_ + cc_ + a_ch[j] * 8) * 2) : 0x80000000u;      \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                     \
          ra_, (__attribute__((address_space(3))) void*)(sa_ + (wid * AJ + j) * 1024), 16, voff_, 0, 0, 0); \
    }                                                                                               \
    _Pragma("unroll") for (int j = 0; j < BJ; ++j) {                                                \
      const int row_ = (wid * BJ + j) * 8 + (lane >> 3);                                            \
      const int chk_ = slot ^ (row_ & 7);                                                           \
      const unsigned voff_ = (unsigned)(((n0 + row_) * wld_ + koff_ + chk_ * 8) * 2);               \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                     \
          rb_, (__attribute__((address_space(3))) void*)(sb_ + (wid * BJ + j) * 1024), 16, voff_, 0, 0, 0); \
    }                                                                                               \
  } while (0)

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this workgroup's K range (all of it unless split)
  const int kb = (int)((long long)ks * nk / p.ksplit), ke = (int)((long long)(ks + 1) * nk / p.ksplit);
  SNRSE_ISSUE(kb, 0);
  if (ke - kb > 1) SNRSE_ISSUE(kb + 1, 1);
  const int lrow = lane & 15, lg = lane >> 4;
  int stage = 0;
  for (int kt = kb; kt < ke; ++kt) {
    if (kt + 1 < ke)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AJ + BJ) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < ke) SNRSE_ISSUE(kt + 2, stage == 0 ? 2 : stage - 1);
    const char* sa = smem + stage * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *(const u32x4*)(sa + swz(wm * TM + i * 16 + lrow, 4 * s + lg));
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *(const u32x4*)(sb + swz(wn * TN + j * 16 + lrow, 4 * s + lg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_chunk<T>(af[i], bfr[j], acc[i][j]);
    }
    stage = stage == STAGES - 1 ? 0 : stage + 1;
  }
#undef SNRSE_ISSUE
  if (p.ksplit > 1) {  // raw fp32 partial sums of this K range; conv_splitk_finalize applies the epilogue
    float* const wsp = p.ws + (size_t)ks * p.M * p.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * TM + i * 16 + lg * 4 + e;
        if (m < p.M) {
#pragma unroll
          for (int j = 0; j < FN; ++j) wsp[(size_t)m * p.Cout + n0 + wn * TN + j * 16 + lrow] = acc[i][j][e];
        }
      }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int b_lo = m0 / HW, b_hi = (min(m0 + BM, p.M) - 1) / HW;
  // (f32 output: one pass ahead, so the kernel keeps the 128 registers of two workgroups per CU)
  epilogue_lds<TO, WM, BN, false, sizeof(TO) == 2 ? 8 : 1>(p, acc, m0 + wm * TM, n0 + wn * TN, lane, (float*)(smem + wid * (64 * 68 * 4)),
                           (float*)(smem + 8 * (64 * 68 * 4)), wm, b_lo == b_hi ? b_lo : -1, n0);
}

// Split-K finalize of the v2 GEMM: out = epilogue(sum of the p.ksplit partial-sum planes in p.ws).
// Block = 16 pixel rows x 16 lanes of 8 channels (128 channels) walking `ppb` pixels of one image,
// so the GroupNorm statistics leave as one atomic pair per channel per block.
template <typename TO>
__global__ __launch_bounds__(256) void conv_splitk_finalize(ConvParams p, int ppb) {
  __shared__ float red[16 * 256];
  const int HW = p.H * p.W;
  const int nbi = (HW + ppb - 1) / ppb;
  const int b = blockIdx.x / nbi;
  const int px0 = (blockIdx.x - b * nbi) * ppb, px1 = min(HW, px0 + ppb);
  const int cl = (threadIdx.x & 15) * 8, r0 = threadIdx.x >> 4;
  const int n = blockIdx.y * 128 + cl;
  float add[8], cw[8][4], cb[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    add[k] = (p.bias ? p.bias[n + k] : 0.f) + (p.temb ? p.temb[(size_t)b * p.temb_stride + n + k] : 0.f);
    s1[k] = 0.f;
    s2[k] = 0.f;
    cb[k] = 0.f;
    cw[k][0] = cw[k][1] = cw[k][2] = cw[k][3] = 0.f;
    if (p.comb_src) {
      cw[k][0] = p.comb_w[(n + k) * 4 + 0];
      cw[k][1] = p.comb_w[(n + k) * 4 + 1];
      cw[k][2] = p.comb_w[(n + k) * 4 + 2];
      cw[k][3] = p.comb_w[(n + k) * 4 + 3];
      cb[k] = p.comb_b[n + k];
    }
  }
  const size_t plane = (size_t)p.M * p.Cout;
  for (int px = px0 + r0; px < px1; px += 16) {
    const size_t m = (size_t)b * HW + px;
    const float* w = p.ws + m * p.Cout + n;
    f32x4 a0 = *(const f32x4*)w, a1 = *(const f32x4*)(w + 4);
    // four planes' loads in flight together (one dependent L2 round trip per plane held the small-level
    // finalizes at 9-14 us per launch); the planes are still added in order
    int s = 1;
    for (; s + 4 <= p.ksplit; s += 4) {
      f32x4 q[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        q[u][0] = *(const f32x4*)(w + (s + u) * plane);
        q[u][1] = *(const f32x4*)(w + (s + u) * plane + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a0 += q[u][0];
        a1 += q[u][1];
      }
    }
    for (; s < p.ksplit; ++s) {
      a0 += *(const f32x4*)(w + s * plane);
      a1 += *(const f32x4*)(w + s * plane + 4);
    }
    float v[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = a0[k] + add[k];
      v[4 + k] = a1[k] + add[4 + k];
    }
    if (p.res) {
      if constexpr (sizeof(TO) == 2) {
        const u32x4 rv = *(const u32x4*)((const TO*)p.res + m * p.res_ld + n);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += H16<TO>::lo(rv[k]);
          v[2 * k + 1] += H16<TO>::hi(rv[k]);
        }
      } else {
        const float* rp = (const float*)p.res + m * p.res_ld + n;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += rp[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= p.out_scale;
    if (p.comb_src) {
      const f32x4 q = *(const f32x4*)(p.comb_src + m * 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += q[0] * cw[k][0] + q[1] * cw[k][1] + q[2] * cw[k][2] + q[3] * cw[k][3] + cb[k];
    }
    if constexpr (sizeof(TO) == 2) {
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = H16<TO>::pack(v[2 * k], v[2 * k + 1]);
      *(u32x4*)((TO*)p.out + m * p.out_ld + n) = o;
    } else {
      float* op = (float*)p.out + m * p.out_ld + n;
#pragma unroll
      for (int k = 0; k < 8; ++k) op[k] = v[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s1[k] += v[k];
      s2[k] = fmaf(v[k], v[k], s2[k]);
    }
  }
  if (p.stats) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[r0 * 256 + (cl + k) * 2] = s1[k];
      red[r0 * 256 + (cl + k) * 2 + 1] = s2[k];
    }
    __syncthreads();
    const int t = threadIdx.x;
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) a += red[r * 256 + t];
    unsafeAtomicAdd(&p.stats[stat_idx(b, blockIdx.x & (SNRSE_STAT_SLOTS - 1), blockIdx.y * 128 + (t >> 1), p.Cout) +
                             (t & 1)],
                    (double)a);
  }
}

// ---------------------------------------------------------------------------------------------
// v5 halo GEMM, two workgroups per CU.  4 waves; tile = TH image rows x TW px x 128 couts (TH x TW =
// 256: 4 x 64 or 8 x 32); wave w computes 64 px (output rows h0 + w TH/4 ..) x all 128 couts (acc 128
// VGPRs).  K runs in 32-channel chunks: halo (TH+2)(TW+2) rows x 64 B (4 x 64: 396 rows, 25 KB; 8 x 32:
// 340 rows, 21 KB), register-staged with the fused GroupNorm+SiLU, + a 2-slot ring of 3-tap weight
// phases (2 x 24 KB, LDS-DMA), so two workgroups share a CU and one's prologue / epilogue runs under
// the other's MFMAs (v4 is 1 workgroup/CU, 152 KB).  The 8 x 32 tile has 14 % fewer halo rows per
// output pixel (340 vs 396): 14 % less GroupNorm+SiLU transform VALU and halo traffic.

// SCD: the fused 1x1 shortcut's chunks run as LDS-DMA phases interleaved with the main chunks (round 5): a shortcut
// phase stages its 128 x 32 weights AND its unpadded 256-px x 32-channel input tile (8 + 16 KB = one ring slot) by
// LDS-DMA, issued at the start of the phase before it like any weight phase, so the tile's HBM latency is covered by
// that phase's MFMAs (3 taps where a main phase precedes it).  Main chunk c carries k = sb(c + 1) - sb(c) shortcut
// phases (sb(c) = c Csc / Cin chunks): k = 0: M0 M1 M2 | 1: M0 M1 M2 S | 2: M0 M1 S M2 S | >= 3: M0 S M1 S M2 S S..;
// the next chunk's halo is stored in the shortcut phase after M2 (which reads no halo), so that chunk boundary needs
// no extra barrier.  (Round 4 ran the shortcut chunks after the main ones as one-tap chunks staged through registers
// like a halo, whose HBM latency then had one tap of cover each: 3-6 % slower on every shortcut shape, +0.9 % on the
// C2 line, profiles/r05b_h5_sc_*.)  SCD = the launch has a shortcut; without one the loop is the 3-phase chunk loop.
// T: the 16-bit input / weight format (bf16_t or f16_t), TO: the output type
template <typename T, typename TO, int GNM, int EF, int TW, bool SCD>
__global__ __launch_bounds__(256, 2) void conv_halo5_kernel(ConvParams p) {
  constexpr int TH = 256 / TW, HC = TW + 2;
  constexpr int RW = TH / 4;                // image rows per wave
  constexpr int HROWS = (TH + 2) * HC;      // 396 (4 x 64) / 340 (8 x 32)
  constexpr int HJ = (HROWS + 63) / 64;     // halo rows per thread: (tid >> 2) + 64 j
  constexpr int HALO_BYTES = HROWS * 64;
  constexpr int TAPB = 128 * 64;  // one tap's 128 couts x 32 ch bf16
  constexpr int SLOT = 3 * TAPB;
  constexpr int KT = 32;
  static_assert(64 * HJ >= HROWS, "halo rows");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const halo = smem;
  char* const ring = smem + HALO_BYTES;
  // GroupNorm scale / shift of the next chunk's 32 channels (2 x 32 f32), written by the first 16
  // lanes of wave 0 before the chunk-end barrier and read by every thread's halo transform, so no
  // thread keeps them in registers across the MFMA phases
  float* const gnl = (float*)(smem + HALO_BYTES + 2 * SLOT + 1024);  // past the stamps build's area

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef SNRSE_STAMPS
  // past both the main-loop layout and the epilogue's staging + statistics area (which reuses the ring)
  constexpr int kStampOff = (HALO_BYTES + 2 * SLOT + 1280) > (4 * (64 * 68 * 4) + 4 * 128 * 2 * 4)
                                ? (HALO_BYTES + 2 * SLOT + 1280) : (4 * (64 * 68 * 4) + 4 * 128 * 2 * 4);
  unsigned long long* const lst = (unsigned long long*)(smem + kStampOff) + wid * 32;
#endif
  SNRSE_STAMP(0);
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int wg = g;
  const int n0 = (wg % p.ntn) * 128;
  int tile = wg / p.ntn;
  const int ntw = p.W / TW, nth = p.H / TH;
  const int w0 = (tile % ntw) * TW;
  tile /= ntw;
  const int h0 = (tile % nth) * TH;
  const int bb = tile / nth;

  const int Cin = p.C0 + p.C1;
  const int cbm = Cin / KT;
  const int Csc_all = p.Csc + p.Csc1;
  const int cbs = p.sc_src ? Csc_all / KT : 0;
  const int nq = 3 * cbm + cbs;  // phases: 3 per main chunk (3 taps each) + 1 per shortcut chunk
  const int K1 = 9 * Cin;
  const int hcol = tid & 3;  // this thread's 16-B chunk (8 channels) of its halo rows

  int hpix[HJ];
  bool hok[HJ];
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int hr = (tid >> 2) + 64 * j;
    const int hy = hr / HC, hx = hr - (hr / HC) * HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    hok[j] = hr < HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
    hpix[j] = (bb * p.H + ih) * p.W + iw;
  }

  u32x4 hv[HJ];
  f32x4 gnv;  // lanes 0..15 of wave 0: 4 of the next chunk's 64 GroupNorm scale / shift values

#define SNRSE_HALO5_LOADS(BASE_, BYTES_, CS_, CC_)                                                     \
  do {                                                                                              \
    const __amdgpu_buffer_rsrc_t r_ = make_rsrc((BASE_), (BYTES_));                                 \
    const int cs_ = (CS_), cc_ = (CC_) + hcol * 8;                                                  \
    _Pragma("unroll") for (int j = 0; j < HJ; ++j) {                                                \
      const int voff_ = hok[j] ? (hpix[j] * cs_ + cc_) * 2 : (int)0x80000000;                       \
      hv[j] = __builtin_amdgcn_raw_buffer_load_b128(r_, voff_, 0, 0);                               \
    }                                                                                               \
  } while (0)
  auto halo_load = [&](int c) {  // main chunk c (the shortcut's tiles go by LDS-DMA, SCD)
    const int ch = c * KT;
    // one load sequence with the source selected by scalars (two branches, each with its own loads, made the
    // compiler's waitcnt model assume the other branch's loads pending: a vmcnt(0) on every src1 chunk)
    const bool s1 = ch >= p.C0;
    SNRSE_HALO5_LOADS(s1 ? p.src1 : p.src0, s1 ? p.bytes1 : p.bytes0, s1 ? p.C1 : p.C0, s1 ? ch - p.C0 : ch);
    if constexpr (GNM > 0) {
      if (tid < 16) gnv = *(const f32x4*)((tid < 8 ? p.gn_scale : p.gn_shift) + (size_t)bb * Cin + ch + (tid & 7) * 4);
    }
  };
#undef SNRSE_HALO5_LOADS
  auto gn_publish = [&]() {  // before the barrier that precedes halo_store
    if constexpr (GNM > 0) {
      if (tid < 16) {
        f32x4 g = gnv;
        if constexpr (GNM == 2) g *= kNegLog2e;  // gn_xform8's prescaled SiLU affine
        *(f32x4*)(gnl + tid * 4) = g;
      }
    }
  };
  auto halo_store = [&](int c) {
    const bool tr = GNM > 0;
    float gsc[8], gsh[8];
    if constexpr (GNM > 0) {
      if (tr) {
        const f32x4 s0 = *(const f32x4*)(gnl + hcol * 8), s1 = *(const f32x4*)(gnl + hcol * 8 + 4);
        const f32x4 t0 = *(const f32x4*)(gnl + 32 + hcol * 8), t1 = *(const f32x4*)(gnl + 32 + hcol * 8 + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) { gsc[i] = s0[i]; gsc[4 + i] = s1[i]; gsh[i] = t0[i]; gsh[4 + i] = t1[i]; }
      }
    }
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int hr = (tid >> 2) + 64 * j;
      if (j == HJ - 1 && hr >= HROWS) break;
      u32x4 v = hv[j];
      if constexpr (GNM > 0) {
        if (tr) v = gn_xform8<T, GNM>(v, gsc, gsh, hok[j]);  // outside the image: the conv's zero padding
      }
      *(u32x4*)(halo + swz64(hr, hcol)) = v;
    }
  };
  // LDS-DMA of a phase into ring slot dst: main (c, tap group g) = 3 weight taps; shortcut u = its weight tap
  // (8 KB) + its input tile (16 KB, tile row r = pixel (r / TW, r % TW), 64-B rows, chunk swizzle on the source)
  // oob: the phase after the last one -- the same 6 pieces per wave, out of range (no memory access; zeros land in the
  // free ring slot), so every phase issues a fixed count (vm_after_dma)
  auto dma = [&](int c, int g, int u, char* dst, bool oob = false) {
    const int rl = lane >> 2, sl = lane & 3;
    const unsigned oobm = oob ? 0x80000000u : 0u;
    if (g < 3) {
      const __amdgpu_buffer_rsrc_t r = make_rsrc(p.wgt, p.wbytes);
      const int kb = c * KT;
      // (a compile-time count per wave: 6 pieces, so the compiler's waitcnt model can count them -- vm_after_dma)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int ii = wid + 4 * k;
        const int jt = ii >> 3, pc = ii & 7;
        const int row = pc * 16 + rl;
        const unsigned voff = oobm | (unsigned)(((n0 + row) * K1 + (3 * g + jt) * Cin + kb + (sl ^ ((row >> 1) & 3)) * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(dst + jt * TAPB + pc * 1024), 16, voff, 0, 0, 0);
      }
    } else {
      const __amdgpu_buffer_rsrc_t r = make_rsrc(p.sc_wgt, p.sc_wbytes);
      const int kb = u * KT;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pc = wid + 4 * k;
        const int row = pc * 16 + rl;
        const unsigned voff = oobm | (unsigned)(((n0 + row) * Csc_all + kb + (sl ^ ((row >> 1) & 3)) * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, voff, 0, 0, 0);
      }
      const bool one = kb >= p.Csc;
      const __amdgpu_buffer_rsrc_t rx = one ? make_rsrc(p.sc_src1, p.sc_bytes1) : make_rsrc(p.sc_src, p.sc_bytes0);
      const int cs = one ? p.Csc1 : p.Csc, cb = one ? kb - p.Csc : kb;
      const int pix0 = (bb * p.H + h0) * p.W + w0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int pc = wid + 4 * k;
        const int row = pc * 16 + rl;
        const int pix = pix0 + (row / TW) * p.W + row % TW;
        const unsigned voff = oobm | (unsigned)((pix * cs + cb + (sl ^ ((row >> 1) & 3)) * 8) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(dst + TAPB + pc * 1024), 16, voff, 0, 0, 0);
      }
    }
  };
  f32x4 acc[2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lrow = lane & 15, lg = lane >> 4;
  // Where this is called, the phase's top already waited for every older vector-memory op and only the 6 LDS-DMA
  // pieces this wave issued since may be in flight, so the wait returns at once.  It is for the compiler: its
  // waitcnt model merges the loop's in-flight-halo path into every phase and would otherwise wait for those fresh
  // DMA pieces (an L2 round trip) before re-filling or storing the halo registers (round 5: a vmcnt(0) after the
  // DMA issue in every chunk's first phase, vmcnt(5..2) in the halo store).  A builtin, not asm: the model sees it.
  auto vm_after_dma = [&]() { __builtin_amdgcn_s_waitcnt(0x0f76); };  // vmcnt(6) expcnt(7) lgkmcnt(15): no lgkm wait


  if constexpr (SCD) {
    // ---- main chunks with their shortcut phases interleaved (see the kernel comment) ----
    auto nsc = [&](int c) { return (c + 1) * cbs / cbm - c * cbs / cbm; };
    // kind of position s of a chunk with k shortcut phases: 0..2 = main tap group t0 = 3 kind, 3 = shortcut (su: its
    // ordinal in the chunk)
    auto kind_of = [](int s, int k, int& su) -> int {
      su = 0;
      if (k >= 3) {
        if (s == 0 || s == 2 || s == 4) return s >> 1;
        su = s <= 3 ? s >> 1 : s - 3;
        return 3;
      }
      if (s < 2) return s;
      if (k == 0) return 2;
      if (k == 1) {
        if (s == 2) return 2;
        return 3;
      }
      if (s == 3) return 2;
      su = s == 2 ? 0 : 1;
      return 3;
    };
    auto m2_pos = [](int k) { return k >= 3 ? 4 : k == 2 ? 3 : 2; };  // position of M2
    halo_load(0);
    dma(0, 0, 0, ring);
    if constexpr (GNM > 0) {
      gn_publish();
      __syncthreads();
    }
    halo_store(0);
    // halo loads issued after a phase's DMA: each thread's HJ vectors (+ wave 0's GroupNorm affine load)
    const bool w0g = GNM > 0 && wid == 0;
    bool halo_inflight = false;
    int c = 0, pos = 0, k = nsc(0), ub = 0;  // current phase: chunk c, position pos; ub = sb(c)
    for (int q = 0; q < nq; ++q) {
      int su;
      const int kind = kind_of(pos, k, su);
      // the next phase
      int c2 = c, pos2 = pos + 1, k2 = k, ub2 = ub;
      if (pos2 == 3 + k) { c2 = c + 1; pos2 = 0; ub2 = ub + k; k2 = c2 < cbm ? nsc(c2) : 0; }
      int su2;
      const int kind2 = kind_of(pos2, k2, su2);
      if (halo_inflight) {
        if (w0g) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HJ + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HJ) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      dma(c2 < cbm ? c2 : 0, kind2, ub2 + su2, ring + ((q + 1) & 1) * SLOT, q + 1 >= nq);
      halo_inflight = false;
      if (kind == 0 && c + 1 < cbm) {
        vm_after_dma();
        halo_load(c + 1);
        halo_inflight = true;
      }
      // one MFMA code path for both kinds (two would double-allocate the accumulators): a main phase reads its 3 taps'
      // A fragments from the halo (row stride HC), a shortcut phase its one tap from the slot's input tile (stride TW)
      const char* sl = ring + (q & 1) * SLOT;
      const bool mainph = kind < 3;
      const char* abuf = mainph ? halo : sl + TAPB;
      const int ntap = mainph ? 3 : 1, rs = mainph ? HC : TW;
      for (int jt = 0; jt < ntap; ++jt) {
        const int tp = 3 * kind + jt;
        const int dy = tp / 3 - 1, dx = tp - (tp / 3) * 3 - 1;
        const int arow = mainph ? (wid * RW + dy + 1) * HC + dx + 1 + lrow : wid * RW * TW + lrow;
        const char* sb = sl + jt * TAPB;
        u32x4 af[4], bfr[8];
        // fragment i: pixels 16 i .. 16 i + 15 of the wave's 64 = image row (16 i) / TW, column (16 i) % TW
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(abuf + swz64(arow + (16 * i / TW) * rs + (16 * i) % TW, lg));
#pragma unroll
        for (int j = 0; j < 8; ++j) bfr[j] = *(const u32x4*)(sb + swz64(j * 16 + lrow, lg));
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[h][i][j] = mfma_chunk<T>(af[i], bfr[h * 4 + j], acc[h][i][j]);
      }
      if (c + 1 < cbm) {
        if (kind == 2) {
          gn_publish();  // the next chunk's GroupNorm affine, read by halo_store after the next barrier
          if (k == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave is done reading halo(c)
            vm_after_dma();
            halo_store(c + 1);
          }
        } else if (kind == 3 && pos == m2_pos(k) + 1) {
          vm_after_dma();
          halo_store(c + 1);  // the first shortcut phase after M2: no wave reads the halo here
        }
      }
      c = c2; pos = pos2; k = k2; ub = ub2;
    }
  } else {
  // no shortcut: 3 phases of 3 taps per chunk, the next chunk's halo stored behind one more barrier
  halo_load(0);
  dma(0, 0, 0, ring);
  if constexpr (GNM > 0) {
    gn_publish();
    __syncthreads();
  }
  halo_store(0);
  SNRSE_STAMP(1);
  bool halo_inflight = false;
  const bool w0g = GNM > 0 && wid == 0;
  for (int q = 0; q < nq; ++q) {
    const int c = q / 3, t0 = (q - c * 3) * 3;
    const bool first = t0 == 0, last = t0 == 6;
    // the halo prefetch issued after the previous phase's weights may stay in flight (HJ vectors + wave 0's
    // GroupNorm affine load)
    if (halo_inflight) {
      if (w0g) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HJ + 1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(HJ) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    SNRSE_STAMP(2 + 2 * (q & 15));
    dma(q + 1 < nq ? (q + 1) / 3 : 0, (q + 1) % 3, 0, ring + ((q + 1) & 1) * SLOT, q + 1 >= nq);
    halo_inflight = false;
    if (first && c + 1 < cbm) {
      vm_after_dma();
      halo_load(c + 1);
      halo_inflight = !last && q + 1 < nq;
    }
    const char* sl = ring + (q & 1) * SLOT;
    for (int jt = 0; jt < 3; ++jt) {
      const int tp = t0 + jt;
      const int dy = tp / 3 - 1, dx = tp - (tp / 3) * 3 - 1;
      const int hbase = (wid * RW + dy + 1) * HC + dx + 1 + lrow;
      const char* sb = sl + jt * TAPB;
      u32x4 af[4], bfr[8];
      // fragment i: pixels 16 i .. 16 i + 15 of the wave's 64 = image row (16 i) / TW, column (16 i) % TW
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(halo + swz64(hbase + (16 * i / TW) * HC + (16 * i) % TW, lg));
#pragma unroll
      for (int j = 0; j < 8; ++j) bfr[j] = *(const u32x4*)(sb + swz64(j * 16 + lrow, lg));
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[h][i][j] = mfma_chunk<T>(af[i], bfr[h * 4 + j], acc[h][i][j]);  // D[px][co]
    }
    SNRSE_STAMP(3 + 2 * (q & 15));
    if (last && c + 1 < cbm) {
      gn_publish();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done reading halo(c); chunk c+1's GN affine is in LDS
      vm_after_dma();
      halo_store(c + 1);
    }
  }
  }
  SNRSE_STAMP(28);
  // both epilogue halves' bias + temb, requested before the drain below so that their round trip overlaps it
  float add0[16 / sizeof(TO)], add1[16 / sizeof(TO)];
  epi_add<TO, EF>(p, n0, lane, bb, add0);
  epi_add<TO, EF>(p, n0 + 64, lane, bb, add1);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (the out-of-range DMA after the last phase too)
  __builtin_amdgcn_s_barrier();  // LDS is reused as the epilogue staging area
  float* const stage = (float*)(smem + wid * (64 * 68 * 4));
  float* const red = (float*)(smem + 4 * (64 * 68 * 4));
  const int mrow = (bb * p.H + h0 + wid * RW) * p.W + w0;
  // (f32 output, the exact mode: residuals two passes ahead -- acc[1] is still live here, 256 registers)
  constexpr int ELA = sizeof(TO) == 2 ? 8 : 2;
  epilogue_img<TO, 4, 128, true, EF, TW, ELA>(p, acc[0], mrow, n0, lane, stage, red, wid, bb, n0, p.W - TW, add0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  SNRSE_STAMP(26);
  epilogue_img<TO, 4, 128, true, EF, TW, ELA>(p, acc[1], mrow, n0 + 64, lane, stage, red, wid, bb, n0, p.W - TW, add1);
  SNRSE_STAMP(27);
  if (EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0) block_stats_flush<4, 128>(p, red, bb, n0);
#ifdef SNRSE_STAMPS
  {
    unsigned long long st_[29];
    if (lane == 0)
      for (int i = 0; i < 29; ++i) st_[i] = lst[i];
    unsigned long long t_end;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0 && p.stamps) {
      unsigned long long* g = p.stamps + ((size_t)blockIdx.x * 8 + wid) * 32;
      for (int i = 0; i < 29; ++i) g[i] = st_[i];
      g[29] = t_end;
      g[30] = hw;
      g[31] = xcc;
    }
  }
#endif
}

template <typename T, typename TO, int GNM, int EF, int TW, bool SCD>
int launch_halo5_ef(ConvParams p, int grid, hipStream_t s) {
  // halo + weight ring + (stamps build: 4 x 32 stamps) + the next chunk's GroupNorm affine (2 x 32 f32),
  // and at least the epilogue's reuse of it: 4 waves' 64 x 68 f32 staging + the 4 x 128 x 2 f32 statistics
  constexpr size_t main_lds = (256 / TW + 2) * (TW + 2) * 64 + 2 * 3 * 128 * 64 + 1024 + 256;
  constexpr size_t epi_lds = 4 * (64 * 68 * 4) + 4 * 128 * 2 * 4;
#ifdef SNRSE_STAMPS
  constexpr size_t lds = (main_lds > epi_lds ? main_lds : epi_lds) + 1024;  // + the 4 waves' stamps (kStampOff)
#else
  constexpr size_t lds = main_lds > epi_lds ? main_lds : epi_lds;
#endif
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_halo5_kernel<T, TO, GNM, EF, TW, SCD>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  SNRSE_RET(attr);  // (thread-safe one-time set: a function-local static)
  hipLaunchKernelGGL((conv_halo5_kernel<T, TO, GNM, EF, TW, SCD>), dim3(grid), dim3(256), lds, s, p);
  return (int)hipGetLastError();
}

template <typename T, typename TO, int GNM, int TW>
int launch_halo5_gn(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  p.ntn = p.Cout / 128;
  // non-temporal output stores when the output exceeds the 256 MB Infinity Cache (+1 % on the
  // full-resolution convs)
  p.epi_nt = cx.epi_nt == 2 ? ((long long)p.M * p.out_ld * (long long)sizeof(TO) > ((long long)cx.epi_nt_mb << 20))
                            : cx.epi_nt;
  cx.last_epi_nt = p.epi_nt;
  const int tiles = p.B * (p.H / (256 / TW)) * (p.W / TW) * p.ntn;
  const int grid = tiles;
  const bool scd = p.sc_src != nullptr;  // the fused shortcut's chunks as LDS-DMA phases
  // the 16-bit ResBlock configurations of the NCSN++ path get a branch-free epilogue (bias always on):
  // Conv_0 (+temb), Conv_1 (+residual | +1x1 shortcut as extra K | +Combine), each +-stats, +-NT
  if constexpr (sizeof(TO) == 2 && GNM != 1) {
    if (cx.h5_specialise && p.bias) {
#define SNRSE_H5_EF(F) \
  case (F): return launch_halo5_ef<T, TO, GNM, (F), TW, false>(p, grid, s);
#define SNRSE_H5_EFS(F) \
  case (F): return launch_halo5_ef<T, TO, GNM, (F), TW, true>(p, grid, s);
      if (!scd) {
        switch (epi_flags(p)) {
          SNRSE_H5_EF(EF_TEMB | EF_STATS)
          SNRSE_H5_EF(EF_TEMB | EF_STATS | EF_NT)
          SNRSE_H5_EF(EF_RES | EF_STATS)
          SNRSE_H5_EF(EF_RES | EF_STATS | EF_NT)
          SNRSE_H5_EF(EF_STATS)
          SNRSE_H5_EF(EF_STATS | EF_NT)
          SNRSE_H5_EF(EF_TEMB)
          default: break;
        }
      } else {  // Conv_1 with the fused Conv_2 shortcut (no residual), and the down-sampling block's + Combine
        switch (epi_flags(p)) {
          SNRSE_H5_EFS(EF_STATS)
          SNRSE_H5_EFS(EF_STATS | EF_NT)
          SNRSE_H5_EFS(EF_COMB | EF_STATS)
          default: break;
        }
      }
#undef SNRSE_H5_EF
#undef SNRSE_H5_EFS
    }
  }
  return scd ? launch_halo5_ef<T, TO, GNM, EF_RT, TW, true>(p, grid, s)
             : launch_halo5_ef<T, TO, GNM, EF_RT, TW, false>(p, grid, s);
}

// GroupNorm prologue mode and tile width as template arguments: the halo transform is straight-line
// code.  Tile 8 x 32 where H % 8 == 0 (option h5_tw: 0 auto, 64 / 32 force where legal), else 4 x 64.
template <typename T, typename TO, int TW>
int launch_halo5_tw(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  cx.last_tw = TW;
  if (!p.gn_scale) return launch_halo5_gn<T, TO, 0, TW>(p, s, cx);
  if (!p.gn_act) return launch_halo5_gn<T, TO, 1, TW>(p, s, cx);
  return launch_halo5_gn<T, TO, 2, TW>(p, s, cx);
}

inline bool halo_tile32(const ConvParams& p) { return p.H % 8 == 0 && p.W % 32 == 0; }
inline bool halo_tile64(const ConvParams& p) { return p.H % 4 == 0 && p.W % 64 == 0; }

template <typename T, typename TO>
int launch_halo5(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  if (halo_tile32(p) && cx.h5_tw != 64) return launch_halo5_tw<T, TO, 32>(p, s, cx);
  return launch_halo5_tw<T, TO, 64>(p, s, cx);
}

// K splits for a v2 launch of `tiles` output tiles over nk K-tiles: about one workgroup per CU when
// the tile grid alone underfills the chip (the small NCSN++ levels), >= 4 K-tiles per split, and
// the partial sums within the registered workspace
// (splitk_target 128/192/256/512/1024 swept on C2: 256 best, split-K off is 9 % slower)
int choose_ksplit(const ConvParams& p, int tiles, int nk, const snrse_ctx& cx, int min_kt = 4) {
  if (!cx.splitk || !cx.ws || tiles >= cx.splitk_target * 3 / 4) return 1;
  int s = (cx.splitk_target + tiles - 1) / tiles;
  if (s > nk / min_kt) s = nk / min_kt;
  const size_t plane = (size_t)p.M * p.Cout * sizeof(float);
  if ((size_t)s * plane > cx.ws_bytes) s = (int)(cx.ws_bytes / plane);
  return s >= 2 ? s : 1;
}

// v1 register-staged GEMM (the fp32 parity path and the Cout <= 16 heads).  fp32 launches whose tile
// grid underfills the chip (the low-resolution NCSN++ levels: 4-60 workgroups at 30 s, C5) split K
// across workgroups (>= 2 K-tiles each) and finish in conv_splitk_finalize.
template <typename T, typename TO, int BM, int BN, int WM, int WN>
int launch_conv(ConvParams p, int npad, hipStream_t s, snrse_ctx& cx) {
  using Tr = ConvTraits<T>;
  p.ntn = npad / BN;
  const int tiles = ((p.M + BM - 1) / BM) * p.ntn;
  const int nk = p.ksize * p.ksize * ((p.C0 + p.C1) / Tr::KT) + (p.sc_src ? (p.Csc + p.Csc1) / Tr::KT : 0);
  p.ksplit = (sizeof(T) == 4 && BN == 128 && p.Cout % 128 == 0) ? choose_ksplit(p, tiles, nk, cx, 2) : 1;
  p.ws = cx.ws;
  cx.last_ksplit = p.ksplit;
  const size_t lds = (size_t)2 * (BM + BN) * 128;
  hipLaunchKernelGGL((conv_mfma_kernel<T, TO, BM, BN, WM, WN>), dim3(tiles * p.ksplit), dim3(64 * WM * WN), lds, s, p);
  if (p.ksplit > 1) {
    SNRSE_LAUNCH_CHECK();
    const int HW = p.H * p.W, ppb = 64;
    hipLaunchKernelGGL((conv_splitk_finalize<TO>), dim3(p.B * ((HW + ppb - 1) / ppb), p.Cout / 128), dim3(256), 0, s,
                       p, ppb);
  }
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
int launch_x3(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  constexpr size_t main_lds = (size_t)2 * (BM + BN) * 128;
  constexpr size_t epi_lds = (BM / WM == 64 && BN / WN == 64) ? (size_t)WM * WN * 64 * 68 * 4 + WM * BN * 2 * 4 : 0;
  constexpr size_t lds = main_lds > epi_lds ? main_lds : epi_lds;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_x3_kernel<BM, BN, WM, WN>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  SNRSE_RET(attr);
  p.ntn = (p.Cout + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * p.ntn;
  const int nk = p.ksize * p.ksize * ((p.C0 + p.C1) / 32) + (p.sc_src ? (p.Csc + p.Csc1) / 32 : 0);
  p.ksplit = BN == 128 ? choose_ksplit(p, tiles, nk, cx, 2) : 1;  // (the finalize works on 128-cout rows)
  p.ws = cx.ws;
  cx.last_ksplit = p.ksplit;
  hipLaunchKernelGGL((conv_x3_kernel<BM, BN, WM, WN>), dim3(tiles * p.ksplit), dim3(64 * WM * WN), lds, s, p);
  if (p.ksplit > 1) {
    SNRSE_LAUNCH_CHECK();
    const int HW = p.H * p.W, ppb = 64;
    hipLaunchKernelGGL((conv_splitk_finalize<float>), dim3(p.B * ((HW + ppb - 1) / ppb), p.Cout / 128), dim3(256), 0, s,
                       p, ppb);
  }
  return (int)hipGetLastError();
}

template <int GNM, int SPR, int TWV, int EF = EF_RT>
int launch_x3h_ef(ConvParams p, hipStream_t s, int tiles) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_x3h_kernel<GNM, SPR, TWV, EF>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)X3G<TWV, SPR>::LDS);
  SNRSE_RET(attr);
  p.ntn = p.Cout / 128;
  p.ksplit = 1;
  constexpr size_t lds = X3G<TWV, SPR>::LDS;
  hipLaunchKernelGGL((conv_x3h_kernel<GNM, SPR, TWV, EF>), dim3(tiles), dim3(512), lds, s, p);
  return (int)hipGetLastError();
}

template <int GNM, int SPR, int TWV>
int launch_x3h_gn(const ConvParams& p, hipStream_t s, int tiles, bool spec) {
  // the ResBlock convs of the fp32x3 path on the pair schedule (GroupNorm+SiLU prologue, or none after a resampler;
  // 8 x 32 tiles) get a
  // compile-time epilogue like the bf16 halo GEMM's: Conv_0 (+temb), Conv_1 (+residual, or the shortcut as extra K,
  // + the down-sampling blocks' pyramid Combine), each with statistics, +-NT (fp32x3 C2 line +1.5 %,
  // profiles/r05z / r05za_x3h_specialise_ab.jsonl)
  if constexpr (GNM != 1 && SPR == 2 && TWV == 32) {
    if (spec && p.bias) {
      switch (epi_flags(p)) {
        case EF_TEMB | EF_STATS: return launch_x3h_ef<GNM, SPR, TWV, EF_TEMB | EF_STATS>(p, s, tiles);
        case EF_TEMB | EF_STATS | EF_NT: return launch_x3h_ef<GNM, SPR, TWV, EF_TEMB | EF_STATS | EF_NT>(p, s, tiles);
        case EF_RES | EF_STATS: return launch_x3h_ef<GNM, SPR, TWV, EF_RES | EF_STATS>(p, s, tiles);
        case EF_RES | EF_STATS | EF_NT: return launch_x3h_ef<GNM, SPR, TWV, EF_RES | EF_STATS | EF_NT>(p, s, tiles);
        case EF_STATS: return launch_x3h_ef<GNM, SPR, TWV, EF_STATS>(p, s, tiles);
        case EF_STATS | EF_NT: return launch_x3h_ef<GNM, SPR, TWV, EF_STATS | EF_NT>(p, s, tiles);
        case EF_COMB | EF_STATS: return launch_x3h_ef<GNM, SPR, TWV, EF_COMB | EF_STATS>(p, s, tiles);
        case EF_COMB | EF_STATS | EF_NT: return launch_x3h_ef<GNM, SPR, TWV, EF_COMB | EF_STATS | EF_NT>(p, s, tiles);
        default: break;
      }
    }
  }
  return launch_x3h_ef<GNM, SPR, TWV>(p, s, tiles);
}

template <int SPR, int TWV>
int launch_x3h_spr(const ConvParams& p, hipStream_t s, int tiles, bool spec) {
  if (!p.gn_scale) return launch_x3h_gn<0, SPR, TWV>(p, s, tiles, spec);
  if (!p.gn_act) return launch_x3h_gn<1, SPR, TWV>(p, s, tiles, spec);
  return launch_x3h_gn<2, SPR, TWV>(p, s, tiles, spec);
}

// tw 32: the 8 x 32 px tiles (H % 8 == 0, W % 32 == 0; tiles counted for them), else 4 x 64
int launch_x3h(const ConvParams& p, hipStream_t s, int tiles, int spread, int tw, bool spec) {
  // the pair schedule (spread 2) needs 8 x 32 tiles and an even number of 32-channel main chunks
  if (spread == 2 && !(tw == 32 && ((p.C0 + p.C1) / 32) % 2 == 0)) spread = 1;
  if (tw == 32) {
    if (spread == 2) return launch_x3h_spr<2, 32>(p, s, tiles, spec);
    return spread ? launch_x3h_spr<1, 32>(p, s, tiles, spec) : launch_x3h_spr<0, 32>(p, s, tiles, spec);
  }
  return spread ? launch_x3h_spr<1, 64>(p, s, tiles, spec) : launch_x3h_spr<0, 64>(p, s, tiles, spec);
}

template <int BM, int BN, typename T, typename TO>
int launch_glds(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  constexpr size_t lds = (size_t)3 * (BM + BN) * 128;
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_glds_kernel<BM, BN, T, TO>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  SNRSE_RET(attr);
  p.ntn = p.Cout / BN;
  const int ntm = (p.M + BM - 1) / BM;
  const int nk = p.ksize * p.ksize * ((p.C0 + p.C1) / 64) + (p.sc_src ? (p.Csc + p.Csc1) / 64 : 0);
  p.ksplit = choose_ksplit(p, ntm * p.ntn, nk, cx);
  p.ws = cx.ws;
  cx.last_ksplit = p.ksplit;
  hipLaunchKernelGGL((conv_glds_kernel<BM, BN, T, TO>), dim3(ntm * p.ntn * p.ksplit), dim3(512), lds, s, p);
  if (p.ksplit > 1) {
    SNRSE_LAUNCH_CHECK();
    const int HW = p.H * p.W, ppb = 64;
    hipLaunchKernelGGL((conv_splitk_finalize<TO>), dim3(p.B * ((HW + ppb - 1) / ppb), p.Cout / 128), dim3(256), 0, s,
                       p, ppb);
  }
  return (int)hipGetLastError();
}

// 0 auto, 1 force v1 (register-staged), 2 force v2 (no halo), 5 halo v5; the experimental
// v3/v4/v6/v7/v8/v9 generations (none faster than v5 on the NCSN++ shapes: profiles/r02d_h7_ablations.json,
// profiles/r02g_conv_bench_v5_v7_v9.jsonl) live in git history and tools/experimental/, outside the product library
constexpr int kHaloAuto = 5;  // halo kernel generation taken by variant 0 (fastest measured: profiles/)

template <typename T, typename TO>
int dispatch_conv(const ConvParams& p, hipStream_t s, snrse_ctx& cx) {
  if (p.Cout >= 64) {
    if (p.Cout % 128 != 0) return SNRSE_EINVAL;
    if constexpr (sizeof(T) == 2) {
      const bool fits = p.bytes0 < 0x7ff00000ll && p.bytes1 < 0x7ff00000ll && p.sc_bytes0 < 0x7ff00000ll &&
                        p.sc_bytes1 < 0x7ff00000ll;
      if (cx.conv_variant != 1 && fits) {
        // halo path on the 4 x 64-tileable images (levels 0-3 of the C2 pyramid), with 8 x 32 tiles where
        // H % 8 == 0.  Not on W = 32 (level 4): 128 tiles for 512 workgroup slots ran 11-45 % slower there
        // than the split-K LDS-DMA GEMM + gn_act (profiles/r03v_level4_halo_vs_glds.jsonl).  (Round 4's v10 halo GEMM,
        // one wave per SIMD with 512 registers, ran the concatenated-input Conv_0s until round 5's v5 changes made v5
        // 4 % faster there and +0.4 % on the C2 line, profiles/r05h_*; it was removed -- git history, conv_h10.hip.)
        if (cx.conv_variant != 2 && p.ksize == 3 && halo_tile64(p)) {
          cx.last_kernel = kHaloAuto;
          return launch_halo5<T, TO>(p, s, cx);
        }
        if (p.gn_scale) return SNRSE_EINVAL;  // fused GroupNorm exists only on the halo paths
        cx.last_kernel = 2;
        if (p.Cout % 256 == 0) return launch_glds<128, 256, T, TO>(p, s, cx);
        return launch_glds<256, 128, T, TO>(p, s, cx);
      }
    }
    if (p.gn_scale) return SNRSE_EINVAL;
    cx.last_kernel = 1;
    return launch_conv<T, TO, 128, 128, 2, 2>(p, p.Cout, s, cx);
  }
  if constexpr (sizeof(T) == 2 && sizeof(TO) == 4) {
    // small images (option head_small 2: also where the tiled head fits, up to 16384 output pixels) take the
    // wave-per-8-pixels head
    const bool small = cx.head_small == 2 && (long long)p.B * p.H * p.W <= 16384;
    if (cx.conv_variant != 1 && head_ok(p) && !small) {
      const bool part = cx.head_part != 0 && p.Cout == 4;
      cx.last_kernel = part ? 15 : 10;
      return launch_head(p, s, part, std::is_same_v<T, f16_t>);
    }
    if (cx.conv_variant != 1 && cx.head_small && head_small_ok(p)) {
      cx.last_kernel = 14;
      cx.last_ksplit = 1;
      return launch_head_small(p, s, false, std::is_same_v<T, f16_t>);
    }
  }
  if (p.gn_scale) return SNRSE_EINVAL;
  if (p.Cout > 16) return SNRSE_EINVAL;
  cx.last_kernel = 1;
  return launch_conv<T, TO, 128, 16, 4, 1>(p, 16, s, cx);
}

}  // namespace

extern "C" int snrse_conv2d(snrse_ctx* ctx, const void* src0, int C0, const void* src1, int C1, int B, int H, int W,
                            int ksize, const void* wgt, const void* sc_src, int Csc, const void* sc_src1,
                            int Csc1, const void* sc_wgt,
                            const float* bias, const float* temb, int temb_stride, const void* res,
                            int res_ld, float out_scale, const float* comb_src, const float* comb_w,
                            const float* comb_b, void* out, int Cout, int out_ld, double* stats,
                            const float* gn_scale, const float* gn_shift, int gn_act, int dtype,
                            int out_f32, hipStream_t stream) {
  using TrB = ConvTraits<bf16_t>;  // (f16: the same 64-element K-tiles)
  using TrF = ConvTraits<float>;
  snrse_ctx& cx = *snrse_ctx_resolve(ctx);
  // SNRSE_F32X3: fp32 activations / output, weights pre-split into bf16 hi / lo rows (conv_x3_kernel)
  const bool x3 = dtype == SNRSE_F32X3;
  if (x3) {
    if (Cout > 16 && Cout % 128) return SNRSE_EINVAL;  // 128-cout tiles, or one 16-row tile (pyramid heads)
    dtype = SNRSE_F32;
    out_f32 = 0;  // (the output is fp32 anyway)
  }
  const int KT = snrse_is16(dtype) ? TrB::KT : TrF::KT;
  if (!src0 || !wgt || !out || (ksize != 1 && ksize != 3)) return SNRSE_EINVAL;
  if (C0 % KT || C1 % KT || (sc_src && (Csc % KT || Csc1 % KT))) return SNRSE_EINVAL;
  if (sc_src && Csc1 > 0 && !sc_src1) return SNRSE_EINVAL;
  if (C1 > 0 && !src1) return SNRSE_EINVAL;
  ConvParams p{};
  p.src0 = src0; p.C0 = C0; p.src1 = src1; p.C1 = C1;
  p.B = B; p.H = H; p.W = W; p.ksize = ksize; p.wgt = wgt;
  p.sc_src = sc_src; p.Csc = sc_src ? Csc : 0; p.sc_wgt = sc_wgt;
  p.sc_src1 = sc_src1; p.Csc1 = sc_src ? Csc1 : 0;
  p.bias = bias; p.temb = temb; p.temb_stride = temb_stride;
  p.res = res; p.res_ld = res_ld; p.out_scale = out_scale;
#ifdef SNRSE_STAMPS
  p.stamps = g_stamp_buf;
#else
  p.stamps = nullptr;
#endif
  p.comb_src = comb_src; p.comb_w = comb_w; p.comb_b = comb_b;
  p.out = out; p.Cout = Cout; p.out_ld = out_ld; p.M = B * H * W;
  p.stats = stats;
  p.epi_nt = 0;
  p.ws = nullptr; p.ksplit = 1;
  p.gn_scale = gn_scale; p.gn_shift = gn_shift; p.gn_act = gn_act;
  if ((gn_scale == nullptr) != (gn_shift == nullptr)) return SNRSE_EINVAL;
  if (p.M <= 0) return 0;
  const long long esz = snrse_is16(dtype) ? 2 : 4;
  const long long pix = (long long)B * H * W;
  p.bytes0 = pix * C0 * esz; p.bytes1 = pix * C1 * esz;
  p.sc_bytes0 = pix * p.Csc * esz; p.sc_bytes1 = pix * p.Csc1 * esz;
  const int npad = Cout >= 64 ? Cout : 16;
  p.wbytes = (long long)npad * ksize * ksize * (C0 + C1) * esz;
  p.sc_wbytes = (long long)npad * (p.Csc + p.Csc1) * esz;
  p.ntn = 1;
  if (stats && !cx.stats_zeroed) SNRSE_RET(hipMemsetAsync(stats, 0, sizeof(double) * 2 * SNRSE_STAT_SLOTS * (size_t)B * Cout, stream));
  if (!snrse_is16(dtype) && dtype != SNRSE_F32) return SNRSE_EINVAL;
  // the split-bf16 halo-kernel decision is taken once for the whole batch (as ops.x3h_ok takes it, which
  // decides whether the caller passes a GroupNorm prologue), so every image-range chunk of a > 2 GiB call
  // runs the same kernel, however few tiles its last chunk has
  const bool x3h_all = x3 && ksize == 3 && H % x3h::TH == 0 && Cout % 128 == 0 &&
                       ((cx.x3_tile == 0 && (long long)B * (H / x3h::TH) * ((W + x3h::TW - 1) / x3h::TW) * (Cout / 128) >= 256) ||
                        cx.x3_tile == 4);
  auto run = [&](const ConvParams& q) {
    if (x3) {
      const int x3h_tiles = q.B * (q.H / x3h::TH) * ((q.W + x3h::TW - 1) / x3h::TW) * (q.Cout / 128);
      if (x3h_all) {
        cx.last_kernel = 4;
        cx.last_ksplit = 1;
        // non-temporal output stores as the bf16 halo GEMMs decide them (option x3_nt: the f32 outputs of the
        // level-0 / level-1 convs are 0.5-2 GB, far beyond the Infinity Cache)
        ConvParams r = q;
        r.epi_nt = cx.x3_nt && (cx.epi_nt == 2 ? ((long long)q.M * q.out_ld * 4ll > ((long long)cx.epi_nt_mb << 20))
                                               : cx.epi_nt != 0);
        cx.last_epi_nt = r.epi_nt;
        // 8 x 32 tiles where they fit (option x3_tw: 0 auto, 64 forces 4 x 64)
        const bool tw32 = cx.x3_tw != 64 && q.H % 8 == 0 && q.W % 32 == 0;
        cx.last_tw = tw32 ? 32 : 64;
        return launch_x3h(r, stream, tw32 ? q.B * (q.H / 8) * (q.W / 32) * (q.Cout / 128) : x3h_tiles, cx.x3_spread,
                          tw32 ? 32 : 64, cx.h5_specialise != 0);
      }
      if (q.Cout <= 16 && cx.conv_variant != 1 && head_ok(q, true)) {  // the pyramid heads, GroupNorm fused
        cx.last_kernel = 11;
        cx.last_ksplit = 1;
        return launch_head_x3(q, stream);
      }
      if (q.Cout <= 16 && cx.conv_variant != 1 && cx.head_small && head_small_ok(q)) {  // small-image heads
        cx.last_kernel = 14;
        cx.last_ksplit = 1;
        return launch_head_small(q, stream, true);
      }
      if (q.gn_scale) return SNRSE_EINVAL;  // the fused GroupNorm exists on the halo forms only
      cx.last_kernel = 3;
      if (q.Cout <= 16) return launch_x3<128, 16, 4, 1>(q, stream, cx);  // the pyramid heads (16 padded rows)
      if (cx.x3_tile == 2) return launch_x3<256, 128, 4, 2>(q, stream, cx);
      if (cx.x3_tile == 3 && q.Cout % 256 == 0) return launch_x3<128, 256, 2, 4>(q, stream, cx);
      return launch_x3<128, 128, 2, 2>(q, stream, cx);
    }
    if (dtype == SNRSE_F16)
      return out_f32 ? dispatch_conv<f16_t, float>(q, stream, cx) : dispatch_conv<f16_t, f16_t>(q, stream, cx);
    if (dtype == SNRSE_BF16)
      return out_f32 ? dispatch_conv<bf16_t, float>(q, stream, cx) : dispatch_conv<bf16_t, bf16_t>(q, stream, cx);
    return dispatch_conv<float, float>(q, stream, cx);
  };
  // The buffer-resource kernels address each source with a 32-bit byte extent and offset.  Images are
  // independent (NHWC, batch outermost), so a batch whose sources exceed 2 GiB (e.g. B >= 64 at the
  // 256 x 512 x 128 level) runs as consecutive launches over image ranges that fit -- the same kernels,
  // never a silent fallback to the register-staged GEMM.
  const long long per_img = (long long)H * W * std::max(std::max(C0, C1), std::max(p.Csc, p.Csc1)) * esz;
  constexpr long long kLim = 0x7ff00000ll;
  cx.last_chunks = 1;
  SNRSE_RET((hipError_t)snrse_ctx_probe_mark(cx, stream, false));
  struct ProbeEnd {  // closes the probe bracket on every return path below
    snrse_ctx& c;
    hipStream_t s;
    ~ProbeEnd() { (void)snrse_ctx_probe_mark(c, s, true); }
  } probe_end{cx, stream};
  if (per_img * B < kLim || per_img >= kLim) return run(p);
  const int chunk = (int)((kLim - 1) / per_img);
  cx.last_chunks = (B + chunk - 1) / chunk;
  const long long HWl = (long long)H * W;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = std::min(chunk, B - b0);
    ConvParams q = p;
    const long long px0 = (long long)b0 * HWl;
    auto off = [&](const void* ptr, long long elems, long long bytes_per) -> const void* {
      return ptr ? (const void*)((const char*)ptr + elems * bytes_per) : nullptr;
    };
    const long long osz = (snrse_is16(dtype) && !out_f32) ? 2 : 4;
    q.src0 = off(p.src0, px0 * C0, esz);
    q.src1 = off(p.src1, px0 * C1, esz);
    q.sc_src = off(p.sc_src, px0 * p.Csc, esz);
    q.sc_src1 = off(p.sc_src1, px0 * p.Csc1, esz);
    q.res = off(p.res, px0 * res_ld, osz);
    q.comb_src = (const float*)off(p.comb_src, px0 * 4, 4);
    q.out = (void*)off(p.out, px0 * out_ld, osz);
    q.temb = (const float*)off(p.temb, (long long)b0 * temb_stride, 4);
    q.stats = p.stats ? p.stats + (size_t)b0 * SNRSE_STAT_SLOTS * Cout * 2 : nullptr;
    q.gn_scale = (const float*)off(p.gn_scale, (long long)b0 * (C0 + C1), 4);
    q.gn_shift = (const float*)off(p.gn_shift, (long long)b0 * (C0 + C1), 4);
    q.B = nb;
    q.M = nb * H * W;
    const long long qpix = (long long)nb * HWl;
    q.bytes0 = qpix * C0 * esz; q.bytes1 = qpix * C1 * esz;
    q.sc_bytes0 = qpix * p.Csc * esz; q.sc_bytes1 = qpix * p.Csc1 * esz;
    const int rc = run(q);
    if (rc) return rc;
  }
  return 0;
}

#ifdef SNRSE_STAMPS
extern "C" int snrse_debug_set_stamps(void* buf) {
  g_stamp_buf = (unsigned long long*)buf;
  return 0;
}
#endif
