// Flash-style self-attention of AttnBlockpp on MFMA (gfx950).
//
// Reference: layerspp.py:77-93 —  w = softmax(q^T k * C^-1/2) over all H*W positions,
// h = v w^T.  q, k, v come from one fused QKV GEMM (conv.hip, NIN_0/1/2 concatenated,
// layers.py:546-555) laid out [B, L, 3C]; the output [B, L, C] feeds the NIN_3 GEMM whose
// epilogue adds the residual and scales by 1/sqrt(2).
//
// One wave owns 16 query rows; K/V tiles of KB keys are staged once per block in LDS and
// shared by its waves.  S = Q K^T and O += P V both run on MFMA (16x16x32 bf16 or exact
// 16x16x4 f32; fp16 as bf16); the softmax is online (running max / sum per row), so the L x L score
// matrix is never materialised (L = 3776 for a 30 s clip).
#include "common.h"

namespace {

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16_t> { static constexpr int KT = 64, EPC = 8, NW = 4, KB = 64; };
template <> struct AttnCfg<f16_t> { static constexpr int KT = 64, EPC = 8, NW = 4, KB = 64; };
template <> struct AttnCfg<float> { static constexpr int KT = 32, EPC = 4, NW = 2, KB = 32; };

SNRSE_DEV int swz(int row, int chunk) { return (row << 7) + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T>
SNRSE_DEV f32x4 mfma_chunk(const u32x4& a, const u32x4& b, f32x4 acc) {
  if constexpr (sizeof(T) == 2) {
    return H16<T>::mfma(a, b, acc);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[j]), __uint_as_float(b[j]), acc, 0, 0, 0);
    return acc;
  }
}

template <typename T, int C>
__global__ __launch_bounds__(64 * AttnCfg<T>::NW) void attn_kernel(const T* qkv, T* out, int L, float scale) {
  using Cf = AttnCfg<T>;
  constexpr int NW = Cf::NW, KB = Cf::KB, KT = Cf::KT, EPC = Cf::EPC;
  constexpr int QB = 16 * NW;
  constexpr int NTH = 64 * NW;
  constexpr int CB = C / KT;             // channel K-blocks
  constexpr int CPR = C / EPC;           // 16-B chunks per channel row
  constexpr int Q_BYTES = QB * C * (int)sizeof(T);
  constexpr int K_BYTES = KB * C * (int)sizeof(T);
  constexpr int V_BYTES = C * KB * (int)sizeof(T);  // transposed [C][KB]
  constexpr int P_BYTES = 16 * KB * (int)sizeof(T);
  constexpr int SJ = KB / 16;            // S n-subtiles per wave
  constexpr int ON = C / 16;             // O n-subtiles
  static_assert(KB * (int)sizeof(T) == 128, "one 128-B K-block of keys for P.V");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qs = smem;
  char* Ks = Qs + Q_BYTES;
  char* Vs = Ks + K_BYTES;
  char* Ps = Vs + V_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lrow = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int q0 = blockIdx.x * QB;
  const size_t ld = 3 * C;
  const T* base = qkv + (size_t)b * L * ld;

  // stage Q (rows = queries, K-dim = channels)
  for (int i = tid; i < QB * CPR; i += NTH) {
    const int r = i / CPR, cc = i % CPR;
    const int kb = cc / 8, ch = cc % 8;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (q0 + r < L) v = *(const u32x4*)(base + (size_t)(q0 + r) * ld + cc * EPC);
    *(u32x4*)(Qs + kb * QB * 128 + swz(r, ch)) = v;
  }

  f32x4 o[ON];
#pragma unroll
  for (int j = 0; j < ON; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { m_run[e] = -INFINITY; l_run[e] = 0.f; }

  char* Pw = Ps + wid * P_BYTES;
  // 16-bit: the next K / V block is loaded into registers while the current one is consumed, and V is
  // transposed in registers (8 keys x 8 channels per thread, v_perm) so it lands in LDS as 16-B stores
  // (the per-element 2-B stores of the generic path held the level-4 attention at ~67 us;
  // profiles/r05a_c2_dispatch_shapes.jsonl)
  constexpr bool kPipe = sizeof(T) == 2 && KB * CPR == 8 * NTH && (KB / 8) * CPR == NTH;
  u32x4 kreg[kPipe ? 8 : 1], vreg[kPipe ? 8 : 1];
  auto load_kv = [&](int kb0) {
    if constexpr (kPipe) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // K: 16-B chunk i = tid + NTH j
        const int i = tid + NTH * j, r = i / CPR, cc = i % CPR;
        kreg[j] = (kb0 + r < L) ? *(const u32x4*)(base + (size_t)(kb0 + r) * ld + C + cc * EPC) : u32x4{0u, 0u, 0u, 0u};
      }
      const int kg = tid / CPR, cc = tid % CPR;  // V: keys 8 kg .. 8 kg + 7 of channel chunk cc
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 8 * kg + q;
        vreg[q] = (kb0 + r < L) ? *(const u32x4*)(base + (size_t)(kb0 + r) * ld + 2 * C + cc * EPC) : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  if constexpr (kPipe) load_kv(0);
  for (int k0 = 0; k0 < L; k0 += KB) {
    __syncthreads();  // previous tile fully consumed
    if constexpr (kPipe) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = tid + NTH * j, r = i / CPR, cc = i % CPR;
        *(u32x4*)(Ks + (cc / 8) * KB * 128 + swz(r, cc % 8)) = kreg[j];
      }
      const int kg = tid / CPR, cc = tid % CPR;
      // out row c' (channel 8 cc + c'), word i = keys (2i, 2i+1): halves of word c' / 2 of key rows 2i, 2i+1
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const unsigned sel = (c & 1) ? 0x07060302u : 0x05040100u;
        u32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_perm(vreg[2 * i + 1][c >> 1], vreg[2 * i][c >> 1], sel);
        *(u32x4*)(Vs + swz(cc * 8 + c, kg)) = o;
      }
      __syncthreads();
      if (k0 + KB < L) load_kv(k0 + KB);
    }
    for (int i = tid; !kPipe && i < KB * CPR; i += NTH) {
      const int r = i / CPR, cc = i % CPR;
      const int kb = cc / 8, ch = cc % 8;
      u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = u32x4{0u, 0u, 0u, 0u};
      if (k0 + r < L) {
        kv = *(const u32x4*)(base + (size_t)(k0 + r) * ld + C + cc * EPC);
        vv = *(const u32x4*)(base + (size_t)(k0 + r) * ld + 2 * C + cc * EPC);
      }
      *(u32x4*)(Ks + kb * KB * 128 + swz(r, ch)) = kv;
      // V transposed: element (key r, channel c) -> row c, key position r
      const T* ve = (const T*)&vv;
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const int c = cc * EPC + e;
        const int kch = r / EPC, kin = r % EPC;
        *(T*)(Vs + swz(c, kch) + kin * (int)sizeof(T)) = ve[e];
      }
    }
    if constexpr (!kPipe) __syncthreads();

    // S = Q K^T  (16 x KB per wave)
    f32x4 s[SJ];
#pragma unroll
    for (int j = 0; j < SJ; ++j) s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < CB; ++kb) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const u32x4 a = *(const u32x4*)(Qs + kb * QB * 128 + swz(wid * 16 + lrow, 4 * st + lg));
#pragma unroll
        for (int j = 0; j < SJ; ++j) {
          const u32x4 bb = *(const u32x4*)(Ks + kb * KB * 128 + swz(j * 16 + lrow, 4 * st + lg));
          s[j] = mfma_chunk<T>(a, bb, s[j]);
        }
      }
    }
    // online softmax; lane holds rows 4*lg+e, key 16*j + lrow
    float alpha[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < SJ; ++j) {
        const bool valid = (k0 + j * 16 + lrow) < L;
        const float v = valid ? s[j][e] * scale : -INFINITY;
        s[j][e] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mnew = fmaxf(m_run[e], mx);
      alpha[e] = expf(m_run[e] - mnew);
      m_run[e] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < SJ; ++j) {
        const float pv = expf(s[j][e] - mnew);
        s[j][e] = pv;
        rs += pv;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l_run[e] = l_run[e] * alpha[e] + rs;
    }
#pragma unroll
    for (int j = 0; j < ON; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) o[j][e] *= alpha[e];
    // P -> LDS (rows = queries, 128 B of keys), then read as A fragments
#pragma unroll
    for (int j = 0; j < SJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * lg + e, key = j * 16 + lrow;
        *(T*)(Pw + swz(r, key / EPC) + (key % EPC) * (int)sizeof(T)) = Elem<T>::from_f(s[j][e]);
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own P stores landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const u32x4 a = *(const u32x4*)(Pw + swz(lrow, 4 * st + lg));
#pragma unroll
      for (int j = 0; j < ON; ++j) {
        const u32x4 bb = *(const u32x4*)(Vs + swz(j * 16 + lrow, 4 * st + lg));
        o[j] = mfma_chunk<T>(a, bb, o[j]);
      }
    }
  }

#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int q = q0 + wid * 16 + 4 * lg + e;
    if (q >= L) continue;
    const float inv = 1.f / l_run[e];
#pragma unroll
    for (int j = 0; j < ON; ++j)
      out[((size_t)b * L + q) * C + j * 16 + lrow] = Elem<T>::from_f(o[j][e] * inv);
  }
}

template <typename T, int C>
int launch_attn(const void* qkv, void* out, int B, int L, hipStream_t s) {
  using Cf = AttnCfg<T>;
  constexpr int QB = 16 * Cf::NW;
  const size_t lds = (size_t)QB * C * sizeof(T) + (size_t)Cf::KB * C * sizeof(T) * 2 +
                     (size_t)Cf::NW * 16 * Cf::KB * sizeof(T);
  static bool attr_set = false;
  if (!attr_set) {
    SNRSE_RET(hipFuncSetAttribute((const void*)attn_kernel<T, C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
    attr_set = true;
  }
  dim3 grid((L + QB - 1) / QB, B);
  hipLaunchKernelGGL((attn_kernel<T, C>), grid, dim3(64 * Cf::NW), lds, s, (const T*)qkv, (T*)out, L,
                     1.0f / sqrtf((float)C));
  return (int)hipGetLastError();
}

// Split-bf16 ("x3") form for the fp32x3 parity mode: fp32 q, k, v (and the softmax probabilities) are split into
// bf16 hi = bf16(x) and lo = bf16(x - hi) and every product runs as hi.hi + hi.lo + lo.hi on the bf16 MFMA (the
// dropped lo.lo and the bits beyond 16 are ~2^-16 relative, as in conv_x3h_kernel), instead of the exact
// v_mfma_f32_16x16x4_f32 at 1/16 the bf16 rate (the exact kernel ran the level-4 attention in ~358 us).
// 4 waves x 16 queries; a wave's q hi / lo fragments stay in registers; 32-key blocks of k (hi, lo: 128-B rows per
// 64 channels) and v^T (hi, lo: 64-B rows of 32 keys per channel) are staged in LDS from registers loaded one block
// ahead (v transposed 8 keys x 4 channels per thread while splitting); 72 KB of LDS.  The C2 level-4 grid is one
// workgroup per CU (8 query blocks x 32 utterances), so the register bound is one workgroup (no spills).
SNRSE_DEV int swz64a(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 1) & 3)) << 4); }

SNRSE_DEV void split8(const f32x4& a, const f32x4& b, u32x4& hi, u32x4& lo) {
  const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t h = pack_bf16x2(x[2 * i], x[2 * i + 1]);
    hi[i] = h;
    lo[i] = pack_bf16x2(x[2 * i] - __uint_as_float(h << 16), x[2 * i + 1] - __uint_as_float(h & 0xffff0000u));
  }
}

SNRSE_DEV f32x4 mfma3(const u32x4& ah, const u32x4& al, const u32x4& bh, const u32x4& bl, f32x4 acc) {
  acc = mfma_chunk<bf16_t>(ah, bh, acc);
  acc = mfma_chunk<bf16_t>(ah, bl, acc);
  return mfma_chunk<bf16_t>(al, bh, acc);
}

__global__ __launch_bounds__(256) void attn_x3_kernel(const float* qkv, float* out, int L, float scale) {
  constexpr int C = 256, NW = 4, QB = 16 * NW, KB = 32, ON = C / 16;
  constexpr int K_BYTES = 4 * KB * 128;       // one of hi / lo: 4 blocks of 64 channels x KB keys x 128 B
  constexpr int V_BYTES = C * 64;             // one of hi / lo: C rows of KB = 32 keys x 2 B
  constexpr int P_BYTES = 16 * 64;            // one of hi / lo per wave: 16 query rows x 32 keys x 2 B
  __shared__ __attribute__((aligned(16))) char smem[2 * K_BYTES + 2 * V_BYTES + NW * 2 * P_BYTES];
  char* const Kh = smem;
  char* const Kl = Kh + K_BYTES;
  char* const Vh = Kl + K_BYTES;
  char* const Vl = Vh + V_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  char* const Ph = Vl + V_BYTES + wid * 2 * P_BYTES;
  char* const Pl = Ph + P_BYTES;
  const int lrow = lane & 15, lg = lane >> 4;
  const int b = blockIdx.y;
  const int q0 = blockIdx.x * QB;
  const size_t ld = 3 * C;
  const float* base = qkv + (size_t)b * L * ld;

  // q fragments: k-step s covers channels 32 s .. 32 s + 31; lane (lrow, lg) holds 8 channels of query row lrow
  u32x4 qh[8], ql[8];
  {
    const int q = q0 + wid * 16 + lrow;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, c = a;
      if (q < L) {
        a = *(const f32x4*)(base + (size_t)q * ld + 32 * s + 8 * lg);
        c = *(const f32x4*)(base + (size_t)q * ld + 32 * s + 8 * lg + 4);
      }
      split8(a, c, qh[s], ql[s]);
    }
  }
  f32x4 o[ON];
#pragma unroll
  for (int j = 0; j < ON; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { m_run[e] = -INFINITY; l_run[e] = 0.f; }

  // next block's k (4 units of 8 channels per thread) and v (8 keys x 4 channels per thread) in registers
  f32x4 kr[8], vr[8];
  auto load_kv = [&](int kb0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = tid + 256 * i, r = u >> 5, cu = u & 31;
      const bool ok = kb0 + r < L;
      const float* kp = base + (size_t)(kb0 + r) * ld + C + 8 * cu;
      kr[2 * i] = ok ? *(const f32x4*)kp : f32x4{0.f, 0.f, 0.f, 0.f};
      kr[2 * i + 1] = ok ? *(const f32x4*)(kp + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int kg = tid >> 6, cq = tid & 63;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int r = 8 * kg + t;
      vr[t] = kb0 + r < L ? *(const f32x4*)(base + (size_t)(kb0 + r) * ld + 2 * C + 4 * cq) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load_kv(0);
  for (int k0 = 0; k0 < L; k0 += KB) {
    __syncthreads();  // previous block fully consumed
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = tid + 256 * i, r = u >> 5, cu = u & 31;
      u32x4 h, l;
      split8(kr[2 * i], kr[2 * i + 1], h, l);
      const int off = (cu >> 3) * KB * 128 + swz(r, cu & 7);
      *(u32x4*)(Kh + off) = h;
      *(u32x4*)(Kl + off) = l;
    }
    {
      const int kg = tid >> 6, cq = tid & 63;
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // channel 4 cq + c: keys 8 kg .. 8 kg + 7 as one 16-B piece (hi, lo)
        u32x4 h, l;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x0 = vr[2 * i][c], x1 = vr[2 * i + 1][c];
          const uint32_t hh = pack_bf16x2(x0, x1);
          h[i] = hh;
          l[i] = pack_bf16x2(x0 - __uint_as_float(hh << 16), x1 - __uint_as_float(hh & 0xffff0000u));
        }
        const int off = swz64a(4 * cq + c, kg);
        *(u32x4*)(Vh + off) = h;
        *(u32x4*)(Vl + off) = l;
      }
    }
    __syncthreads();
    if (k0 + KB < L) load_kv(k0 + KB);

    // S = Q K^T (16 x 32 per wave)
    f32x4 sv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      sv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int off = (s >> 1) * KB * 128 + swz(16 * j + lrow, 4 * (s & 1) + lg);
        sv[j] = mfma3(qh[s], ql[s], *(const u32x4*)(Kh + off), *(const u32x4*)(Kl + off), sv[j]);
      }
    }
    // online softmax; lane holds rows 4 lg + e, key 16 j + lrow
    float alpha[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool valid = (k0 + j * 16 + lrow) < L;
        const float v = valid ? sv[j][e] * scale : -INFINITY;
        sv[j][e] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mnew = fmaxf(m_run[e], mx);
      alpha[e] = expf(m_run[e] - mnew);
      m_run[e] = mnew;
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float pv = expf(sv[j][e] - mnew);
        sv[j][e] = pv;
        rs += pv;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l_run[e] = l_run[e] * alpha[e] + rs;
    }
#pragma unroll
    for (int j = 0; j < ON; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) o[j][e] *= alpha[e];
    // P (hi, lo) -> this wave's LDS rows (16 queries x 32 keys), read back as A fragments
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * lg + e, key = j * 16 + lrow;
        const float pv = sv[j][e];
        const bf16_t h = f2bf(pv);
        const int off = swz64a(r, key >> 3) + (key & 7) * 2;
        *(bf16_t*)(Ph + off) = h;
        *(bf16_t*)(Pl + off) = f2bf(pv - bf2f(h));
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own P stores landed
    __builtin_amdgcn_wave_barrier();
    const u32x4 ah = *(const u32x4*)(Ph + swz64a(lrow, lg)), al = *(const u32x4*)(Pl + swz64a(lrow, lg));
#pragma unroll
    for (int j = 0; j < ON; ++j) {
      const int off = swz64a(16 * j + lrow, lg);
      o[j] = mfma3(ah, al, *(const u32x4*)(Vh + off), *(const u32x4*)(Vl + off), o[j]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int q = q0 + wid * 16 + 4 * lg + e;
    if (q >= L) continue;
    const float inv = 1.f / l_run[e];
#pragma unroll
    for (int j = 0; j < ON; ++j) out[((size_t)b * L + q) * C + j * 16 + lrow] = o[j][e] * inv;
  }
}

}  // namespace

extern "C" int snrse_attention(const void* qkv, void* out, int B, int L, int C, int dtype, hipStream_t stream) {
  if (!qkv || !out || L <= 0 || B <= 0) return SNRSE_EINVAL;
  if (C != 256) return SNRSE_EINVAL;  // NCSN++ attention runs at 256 channels (ncsnpp.py:170-171)
  if (dtype == SNRSE_F16) return launch_attn<f16_t, 256>(qkv, out, B, L, stream);
  if (dtype == SNRSE_BF16) return launch_attn<bf16_t, 256>(qkv, out, B, L, stream);
  if (dtype == SNRSE_F32) return launch_attn<float, 256>(qkv, out, B, L, stream);
  if (dtype == SNRSE_F32X3) {  // fp32 in / out, split-bf16 products (the fp32x3 parity mode)
    hipLaunchKernelGGL(attn_x3_kernel, dim3((L + 63) / 64, B), dim3(256), 0, stream, (const float*)qkv, (float*)out, L,
                       1.0f / sqrtf(256.f));
    return (int)hipGetLastError();
  }
  return SNRSE_EINVAL;
}
