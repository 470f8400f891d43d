// Ping-pong halo GEMM for the NCSN++ 3x3 convs (bf16, fused GroupNorm(+SiLU) prologue), gfx950.
//
// PARKED EXPERIMENT (round 3): not compiled into libsnrse_hip.so.  Bit-identical to v5 on 19 parity cases
// but 2x slower (profiles/r03k_pp_vs_v5_conv_bench.jsonl); the stamp shares (profiles/r03l_pp_stamps.json)
// show a lone MFMA wave per SIMD exposing its LDS-read latency (an M sub-phase of 1536 MFMA cycles takes
// 3.4-6k) and a ~15k-cycle per-tile epilogue that every lock-step barrier waits for.  To rebuild it, copy
// it back to csrc/ with its launch_pp/pp_ok declarations and a conv_variant 6 dispatch in conv.hip.
//
// Same tile and K loop as the v5 halo GEMM (conv.hip: 4 image rows x 64 px x 128 couts per tile, 32-channel
// K chunks, a register-staged halo with the GroupNorm+SiLU transform, 3-tap LDS-DMA weight phases), but ONE
// 512-thread workgroup per CU made of two independent 4-wave halves that alternate roles in lock step:
// while one half runs the MFMAs of a K chunk (an "M interval": 3 phases of 3 taps), the other transforms
// its next chunk's halo or finishes a tile's epilogue (a "V interval").  Waves w and w + 4 share a SIMD,
// so every SIMD pairs one MFMA-issuing wave with one VALU-issuing wave (MI355X_MICROARCH.md, "Two waves
// per SIMD"), instead of two uncoordinated workgroups whose transforms and epilogues collide with each
// other's MFMAs.  Each half walks a short run of tiles (`tpw`), the epilogue of one tile sharing a V
// interval with the first transform of the next, so the MFMA pipe stays fed across tile boundaries.
//
// Synchronisation: every interval has 3 sub-phases opened by a workgroup barrier that all 8 waves pass
// (the two halves never wait for each other inside a sub-phase).  A sub-phase's M waves first wait for
// their own LDS-DMA weight pieces (counted vmcnt), V waves for their LDS stores; nothing else needs
// ordering: each half has its own halo, weight ring, statistics rows and GroupNorm-affine area.
//
// Reference: ddpm_conv3x3 (layers.py:100-124) inside ResnetBlockBigGANpp (layerspp.py:244-276) with its
// GroupNorm_0/1 + SiLU (layerspp.py:245-262); fused 1x1 shortcuts stay on the v5 kernel.
#include "conv_common.h"

namespace snrse_conv {
namespace {

constexpr int PP_TH = 4, PP_TW = 64, PP_HC = PP_TW + 2;
constexpr int PP_HROWS = (PP_TH + 2) * PP_HC;     // 396 halo rows of 64 B
constexpr int PP_HJ = 7;                           // halo rows per thread: (htid >> 2) + 64 j
constexpr int PP_HALO = PP_HROWS * 64;             // 25344
constexpr int PP_TAPB = 128 * 64;                  // one tap: 128 couts x 32 ch bf16
constexpr int PP_SLOT = 3 * PP_TAPB;               // one weight phase (3 taps)
constexpr int PP_RED = 4 * 128 * 2 * 4;            // statistics rows: 4 waves x 128 co x (sum, sumsq)
constexpr int PP_GNL = 2 * 32 * 4;                 // next chunk's GroupNorm scale / shift
constexpr int PP_HALF = PP_HALO + 2 * PP_SLOT + PP_RED + PP_GNL;  // 78848
constexpr int PP_LDS = 2 * PP_HALF;                // 157696: one workgroup per CU
constexpr int PP_KT = 32;
constexpr int PP_LDR = 36;                         // epilogue staging row: 32 co + 4 pad floats
constexpr int PP_STAGE = 64 * PP_LDR * 4;          // 9216 per wave
static_assert(64 * PP_HJ >= PP_HROWS, "halo rows");
static_assert(2 * PP_STAGE <= PP_SLOT, "staging fits the free ring slot");

struct PPTile {
  int n0, w0, h0, bb;
};

SNRSE_DEV PPTile pp_tile(const ConvParams& p, int t) {
  const int ntw = p.W / PP_TW, nth = p.H / PP_TH;
  PPTile r;
  r.n0 = (t % p.ntn) * 128;
  t /= p.ntn;
  r.w0 = (t % ntw) * PP_TW;
  t /= ntw;
  r.h0 = (t % nth) * PP_TH;
  r.bb = t / nth;
  return r;
}

// a value the compiler cannot see through: lane-derived address math built from it is redone where it
// is used instead of being hoisted out of the interval loops into VGPRs live across the whole kernel
SNRSE_DEV int pp_opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// sum over the 16 lanes of a wave that share lane % 4 (every lane receives its sum)
SNRSE_DEV float pp_sum16(float v) {
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

template <int GNM, int EF>
__global__ __launch_bounds__(512, 2) void conv_pp_kernel(ConvParams p, int tpw) {
  const bool f_temb = EF < 0 ? p.temb != nullptr : (EF & EF_TEMB) != 0;
  const bool f_res = EF < 0 ? p.res != nullptr : (EF & EF_RES) != 0;
  const bool f_comb = EF < 0 ? p.comb_src != nullptr : (EF & EF_COMB) != 0;
  const bool f_stats = EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0;
  const bool f_nt = EF < 0 ? p.epi_nt != 0 : (EF & EF_NT) != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wid >> 2, hw = wid & 3;  // half 0: waves 0-3, half 1: waves 4-7 (wave w + 4 shares w's SIMD)
  const int htid = tid & 255;
  char* const halo = smem + half * PP_HALF;
  char* const ring = halo + PP_HALO;
  float* const red = (float*)(ring + 2 * PP_SLOT);
  float* const gnl = red + PP_RED / 4;
  const int lrow = lane & 15, lg = lane >> 4;
  const int hcol = htid & 3;

  // XCD-aware remap: consecutive logical workgroups (neighbouring tile runs) share an XCD's L2
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int tiles = p.B * (p.H / PP_TH) * (p.W / PP_TW) * p.ntn;
  const int t_begin = g * 2 * tpw;
  const int navail = max(0, min(2 * tpw, tiles - t_begin));
  const int n_h0 = (navail + 1) / 2, n_h1 = navail / 2;
  const int nh = half ? n_h1 : n_h0;  // tiles of this half: t_begin + 2 i + half
  const int Cin = p.C0 + p.C1;
  const int C = Cin / PP_KT;
  const int K1 = 9 * Cin;
  const int nsteps = 2 * C * nh + 1;  // V, M, V, M, ..., final epilogue V
  const int K = max(2 * C * n_h0 + 1, 2 * C * n_h1 + 2);
  const int slot_stats = (bid * 2 + half) & (SNRSE_STAT_SLOTS - 1);

  u32x4 hv[PP_HJ];
  f32x4 gnv = f32x4{0.f, 0.f, 0.f, 0.f};  // lanes < 16 of wave hw == 0: 4 of the next chunk's affine values

  auto halo_load = [&](int tl, int c) {
    const int htid = pp_opaque((int)threadIdx.x) & 255, hcol = htid & 3;
    const PPTile T = pp_tile(p, t_begin + 2 * tl + half);
    const int ch = c * PP_KT;
    const bool s1 = ch >= p.C0;
    const __amdgpu_buffer_rsrc_t r = s1 ? make_rsrc(p.src1, p.bytes1) : make_rsrc(p.src0, p.bytes0);
    const int cs = s1 ? p.C1 : p.C0, cc = (s1 ? ch - p.C0 : ch) + hcol * 8;
#pragma unroll
    for (int j = 0; j < PP_HJ; ++j) {
      const int hr = (htid >> 2) + 64 * j;
      const int hy = hr / PP_HC, hx = hr - (hr / PP_HC) * PP_HC;
      const int ih = T.h0 + hy - 1, iw = T.w0 + hx - 1;
      const bool ok = hr < PP_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
      const int voff = ok ? (((T.bb * p.H + ih) * p.W + iw) * cs + cc) * 2 : (int)0x80000000;
      hv[j] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    }
    if constexpr (GNM > 0) {
      if (hw == 0 && lane < 16)
        gnv = *(const f32x4*)((lane < 8 ? p.gn_scale : p.gn_shift) + (size_t)T.bb * Cin + ch + (lane & 7) * 4);
    }
  };
  auto gn_publish = [&]() {
    if constexpr (GNM > 0) {
      if (hw == 0 && lane < 16) *(f32x4*)(gnl + lane * 4) = gnv;
    }
  };
  // weights of phase ph (taps 3 ph .. 3 ph + 2) of chunk c for output channels n0.. -> ring slot s
  auto wload = [&](int n0, int c, int ph, int s) {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(p.wgt, p.wbytes);
    char* dst = ring + s * PP_SLOT;
    const int ln = pp_opaque((int)threadIdx.x) & 63;
    const int rl = ln >> 2, sl = ln & 3;
    for (int ii = hw; ii < 24; ii += 4) {
      const int jt = ii >> 3, pc = ii & 7;
      const int koff = (3 * ph + jt) * Cin + c * PP_KT;
      const int row = pc * 16 + rl;
      const unsigned voff = (unsigned)(((n0 + row) * K1 + koff + (sl ^ ((row >> 1) & 3)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(dst + jt * PP_TAPB + pc * 1024),
                                               16, voff, 0, 0, 0);
    }
  };
  // transform + LDS store of halo vectors [j0, j1) of local tile tl
  auto halo_store = [&](int tl, int j0, int j1) {
    const int htid = pp_opaque((int)threadIdx.x) & 255, hcol = htid & 3;
    const PPTile T = pp_tile(p, t_begin + 2 * tl + half);
    float gsc[8], gsh[8];
    if constexpr (GNM > 0) {
      const f32x4 s0 = *(const f32x4*)(gnl + hcol * 8), s1 = *(const f32x4*)(gnl + hcol * 8 + 4);
      const f32x4 t0 = *(const f32x4*)(gnl + 32 + hcol * 8), t1 = *(const f32x4*)(gnl + 32 + hcol * 8 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) { gsc[i] = s0[i]; gsc[4 + i] = s1[i]; gsh[i] = t0[i]; gsh[4 + i] = t1[i]; }
    }
#pragma unroll
    for (int j = 0; j < PP_HJ; ++j) {
      if (j < j0 || j >= j1) continue;
      const int hr = (htid >> 2) + 64 * j;
      if (j == PP_HJ - 1 && hr >= PP_HROWS) break;
      u32x4 v = hv[j];
      if constexpr (GNM > 0) {
        const int hy = hr / PP_HC, hx = hr - (hr / PP_HC) * PP_HC;
        const int ih = T.h0 + hy - 1, iw = T.w0 + hx - 1;
        const bool ok = ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        v = gn_xform8<GNM>(v, gsc, gsh, ok);  // outside the image: the conv's zero padding
      }
      *(u32x4*)(halo + swz64(hr, hcol)) = v;
    }
  };

  f32x4 acc[2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one 64-px x 32-co pass of the epilogue of local tile tl (channels n0 + q * 32 ..): stage the fp32
  // accumulators in this wave's area, then every lane finishes 8 channels of 4 rows -> 16-B stores
  auto epilogue_pass = [&](int tl, int q, float* stage, float (&s1)[8], float (&s2)[8]) {
    const PPTile T = pp_tile(p, t_begin + 2 * tl + half);
    const int h = q >> 1, jb = (q & 1) * 2;
    const int cc = lane & 3, r0 = lane >> 2;
    const int n = T.n0 + q * 32 + cc * 8;
    const size_t mrow = ((size_t)(T.bb * p.H + T.h0 + hw)) * p.W + T.w0;
    u32x4 rv[4];
    f32x4 qv[4];
    if (f_res) {
#pragma unroll
      for (int rp = 0; rp < 4; ++rp) rv[rp] = *(const u32x4*)((const bf16_t*)p.res + (mrow + rp * 16 + r0) * p.res_ld + n);
    }
    if (f_comb) {
#pragma unroll
      for (int rp = 0; rp < 4; ++rp) qv[rp] = *(const f32x4*)(p.comb_src + (mrow + rp * 16 + r0) * 4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) stage[(i * 16 + lg * 4 + e) * PP_LDR + jj * 16 + lrow] = acc[h][i][jb + jj][e];
    float add[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) add[k] = 0.f;
    if (p.bias) {
      const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) { add[k] += b0[k]; add[4 + k] += b1[k]; }
    }
    if (f_temb) {
      const float* tb = p.temb + (size_t)T.bb * p.temb_stride + n;
#pragma unroll
      for (int k = 0; k < 8; ++k) add[k] += tb[k];
    }
    float cw[8][4], cb[8];
    if (f_comb) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const f32x4 w = *(const f32x4*)(p.comb_w + (size_t)(n + k) * 4);
        cw[k][0] = w[0]; cw[k][1] = w[1]; cw[k][2] = w[2]; cw[k][3] = w[3];
        cb[k] = p.comb_b[n + k];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the staging writes are in LDS
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int rp = 0; rp < 4; ++rp) {
      const int row = rp * 16 + r0;
      const f32x4 a0 = *(const f32x4*)(stage + row * PP_LDR + cc * 8), a1 = *(const f32x4*)(stage + row * PP_LDR + cc * 8 + 4);
      float v[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[k] = a0[k] + add[k]; v[4 + k] = a1[k] + add[4 + k]; }
      if (f_res) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += __uint_as_float(rv[rp][k] << 16);
          v[2 * k + 1] += __uint_as_float(rv[rp][k] & 0xffff0000u);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= p.out_scale;
      if (f_comb) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          v[k] += qv[rp][0] * cw[k][0] + qv[rp][1] * cw[k][1] + qv[rp][2] * cw[k][2] + qv[rp][3] * cw[k][3] + cb[k];
      }
      const u32x4 o = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7])};
      bf16_t* dst = (bf16_t*)p.out + (mrow + row) * p.out_ld + n;
      if (f_nt) __builtin_nontemporal_store(o, (u32x4*)dst);
      else *(u32x4*)dst = o;
      if (f_stats) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += v[k]; s2[k] = fmaf(v[k], v[k], s2[k]); }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // the reads are done before the next pass re-stages
    __builtin_amdgcn_wave_barrier();
  };
  // the whole epilogue of local tile tl for this wave (4 passes) + its statistics row
  auto epilogue = [&](int tl, float* stage) {
#ifdef PP_NO_EPI
    float sum = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) { sum += acc[h][i][jq][0] + acc[h][i][jq][3]; acc[h][i][jq] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    stage[lane] = sum + tl;
    return;
#endif
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float s1[8], s2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
      epilogue_pass(tl, q, stage, s1, s2);
      if (f_stats) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = pp_sum16(s1[k]), b = pp_sum16(s2[k]);
          if (lane < 4) {
            red[(hw * 128 + q * 32 + lane * 8 + k) * 2] = a;
            red[(hw * 128 + q * 32 + lane * 8 + k) * 2 + 1] = b;
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // statistics of local tile tl: the half's 4 wave rows folded, one atomic pair per channel
  auto stats_flush = [&](int tl) {
    const PPTile T = pp_tile(p, t_begin + 2 * tl + half);
    const int t = htid;  // 256 threads: channel t >> 1, sum / sumsq t & 1
    const float a = red[t] + red[256 + t] + red[512 + t] + red[768 + t];
    unsafeAtomicAdd(&p.stats[stat_idx(T.bb, slot_stats, T.n0 + (t >> 1), p.Cout) + (t & 1)], (double)a);
  };

  // prologue: the first tile's chunk-0 halo and affine, and its first weight phase
  int gq = 0;  // this half's weight phases so far (ring slot = gq & 1)
  if (nh > 0) {
    halo_load(0, 0);
    wload(pp_tile(p, t_begin + half).n0, 0, 0, 0);
    gn_publish();  // (waits for the affine load)
  }
  // Every wave walks its own straight sequence of intervals (3 barriers each): half 1 starts one
  // interval late, then per tile and K chunk a V interval (the chunk's halo transform; at chunk 0 of
  // every tile after the first also the previous tile's epilogue) and an M interval (the chunk's 9 taps),
  // then the last tile's epilogue; idle intervals pad both halves to the same K.
#ifdef SNRSE_STAMPS
  // diagnostic build: s_memtime before each sub-phase wait and after its barrier, lane 0 of every wave,
  // [block][wave][256] (tools/pp_stamps.py); read shares, not lengths
  int sidx = 0;
  auto stamp = [&]() {
    if (p.stamps && sidx < 256) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) p.stamps[((size_t)blockIdx.x * 8 + wid) * 256 + sidx] = t;
    }
    ++sidx;
  };
#else
  auto stamp = [&]() {};
#endif
  auto wait_m = [&](bool partial) {
    stamp();
    if (partial) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stamp();
  };
  auto wait_v = [&]() {
    stamp();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stamp();
  };
  int done = 0;  // intervals this wave has passed
  if (half) {
#pragma unroll 1
    for (int sp = 0; sp < 3; ++sp) wait_v();
    ++done;
  }
#pragma unroll 1
  for (int tl = 0; tl < nh; ++tl) {
    const int n0 = pp_tile(p, t_begin + 2 * tl + half).n0;
#pragma unroll 1
    for (int c = 0; c < C; ++c) {
      // ---- V interval: halo transform of chunk c (+ the previous tile's epilogue at c == 0)
      {
        float* const stage = (float*)(ring + ((gq + 1) & 1) * PP_SLOT + (hw & 1) * PP_STAGE);
        const bool do_epi = c == 0 && tl > 0;
#pragma unroll 1
        for (int sp = 0; sp < 3; ++sp) {
          wait_v();
          if (do_epi) {
            // waves 0, 1 finish the previous tile in sub-phase 0 and waves 2, 3 in sub-phase 1 (two
            // staging areas fit the free ring slot); the halo transform fills the other sub-phases
            const bool mine = (sp == 0) == (hw < 2);
            if (sp < 2 && mine) epilogue(tl - 1, stage);
            else if (sp < 2) halo_store(tl, 0, 4);
            else {
              halo_store(tl, 4, PP_HJ);
              if (f_stats) stats_flush(tl - 1);
            }
          } else {
            if (sp == 0) halo_store(tl, 0, 3);
            else if (sp == 1) halo_store(tl, 3, 5);
            else halo_store(tl, 5, PP_HJ);
          }
        }
      }
      // ---- M interval: the 9 taps of chunk c, 3 per sub-phase, weights from the 2-slot ring
      {
        const bool has_next = c + 1 < C || tl + 1 < nh;
        const int ntl = c + 1 < C ? tl : tl + 1, nc = c + 1 < C ? c + 1 : 0;
#pragma unroll 1
        for (int sp = 0; sp < 3; ++sp) {
          // this wave's pieces of the phase's weights have landed: in sub-phase 1 only the 7 halo loads
          // (+ the affine load) issued after them in sub-phase 0 may stay in flight
          wait_m(sp == 1 && has_next);
          if (sp < 2) wload(n0, c, sp + 1, (gq + 1) & 1);
          else if (has_next) wload(pp_tile(p, t_begin + 2 * ntl + half).n0, nc, 0, (gq + 1) & 1);
          if (sp == 0 && has_next) halo_load(ntl, nc);
          const char* sl = ring + (gq & 1) * PP_SLOT;
#pragma unroll 1
          for (int jt = 0; jt < 3; ++jt) {  // (unrolled, the next tap's fragment reads are hoisted: 2x the VGPRs)
            const int hbase = (hw + sp) * PP_HC + jt + lrow;  // tap (dy, dx) = (sp - 1, jt - 1)
            const char* sb = sl + jt * PP_TAPB;
            u32x4 af[4], bfr[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(halo + swz64(hbase + i * 16, lg));
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) bfr[jj] = *(const u32x4*)(sb + swz64(jj * 16 + lrow, lg));
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                  acc[h][i][jj] = mfma_chunk<bf16_t>(af[i], bfr[h * 4 + jj], acc[h][i][jj]);
          }
          if (sp == 2 && has_next) gn_publish();
          ++gq;
        }
      }
      done += 2;
    }
  }
  if (nh > 0) {  // the last tile's epilogue
    float* const stage = (float*)(ring + ((gq + 1) & 1) * PP_SLOT + (hw & 1) * PP_STAGE);
#pragma unroll 1
    for (int sp = 0; sp < 3; ++sp) {
      wait_v();
      if (sp < 2 && (sp == 0) == (hw < 2)) epilogue(nh - 1, stage);
      if (sp == 2 && f_stats) stats_flush(nh - 1);
    }
    ++done;
  }
#pragma unroll 1
  for (; done < K; ++done)
#pragma unroll 1
    for (int sp = 0; sp < 3; ++sp) wait_v();
}

template <int GNM, int EF>
int launch_pp_ef(const ConvParams& p, int grid, int tpw, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_pp_kernel<GNM, EF>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS);
  SNRSE_RET(attr);
  hipLaunchKernelGGL((conv_pp_kernel<GNM, EF>), dim3(grid), dim3(512), PP_LDS, s, p, tpw);
  return (int)hipGetLastError();
}

template <int GNM>
int launch_pp_gn(ConvParams p, int grid, int tpw, hipStream_t s, const snrse_ctx& cx) {
  if constexpr (GNM != 1) {
    if (cx.h5_specialise && p.bias) {
      switch (epi_flags(p)) {
#define SNRSE_PP_EF(F) \
  case (F): return launch_pp_ef<GNM, (F)>(p, grid, tpw, s);
        SNRSE_PP_EF(EF_TEMB | EF_STATS)
        SNRSE_PP_EF(EF_TEMB | EF_STATS | EF_NT)
        SNRSE_PP_EF(EF_RES | EF_STATS)
        SNRSE_PP_EF(EF_RES | EF_STATS | EF_NT)
        SNRSE_PP_EF(EF_STATS)
        SNRSE_PP_EF(EF_STATS | EF_NT)
        SNRSE_PP_EF(EF_COMB | EF_STATS)
        SNRSE_PP_EF(EF_TEMB)
#undef SNRSE_PP_EF
        default: break;
      }
    }
  }
  return launch_pp_ef<GNM, EF_RT>(p, grid, tpw, s);
}

}  // namespace

bool pp_ok(const ConvParams& p) {
  return p.ksize == 3 && p.H % PP_TH == 0 && p.W % PP_TW == 0 && p.Cout % 128 == 0 && !p.sc_src &&
         (p.C0 + p.C1) % PP_KT == 0 && p.C0 % PP_KT == 0;
}

int launch_pp(ConvParams p, hipStream_t s, snrse_ctx& cx) {
  p.ntn = p.Cout / 128;
  p.epi_nt = cx.epi_nt == 2 ? ((long long)p.M * p.out_ld * 2LL > ((long long)cx.epi_nt_mb << 20)) : cx.epi_nt;
  cx.last_epi_nt = p.epi_nt;
  const int tpw = cx.pp_tiles > 0 ? cx.pp_tiles : 4;  // tiles per half per workgroup
  const long long tiles = (long long)p.B * (p.H / PP_TH) * (p.W / PP_TW) * p.ntn;
  const long long grid = (tiles + 2 * tpw - 1) / (2 * tpw);
  if (grid <= 0 || grid > 0x7fffffffLL) return SNRSE_EINVAL;
  if (!p.gn_scale) return launch_pp_gn<0>(p, (int)grid, tpw, s, cx);
  if (!p.gn_act) return launch_pp_gn<1>(p, (int)grid, tpw, s, cx);
  return launch_pp_gn<2>(p, (int)grid, tpw, s, cx);
}

}  // namespace snrse_conv
