// Flash-style self-attention of AttnBlockpp on MFMA (gfx950).
//
// Reference: layerspp.py:77-93 —  w = softmax(q^T k * C^-1/2) over all H*W positions,
// h = v w^T.  q, k, v come from one fused QKV GEMM (conv.hip, NIN_0/1/2 concatenated,
// layers.py:546-555) laid out [B, L, 3C]; the output [B, L, C] feeds the NIN_3 GEMM whose
// epilogue adds the residual and scales by 1/sqrt(2).
//
// One wave owns 16 query rows; K/V tiles of KB keys are staged once per block in LDS and
// shared by its waves.  S = Q K^T and O += P V both run on MFMA (16x16x32 bf16 or exact
// 16x16x4 f32); the softmax is online (running max / sum per row), so the L x L score
// matrix is never materialised (L = 3776 for a 30 s clip).
#include "common.h"

namespace {

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16_t> { static constexpr int KT = 64, EPC = 8, NW = 4, KB = 64; };
template <> struct AttnCfg<float> { static constexpr int KT = 32, EPC = 4, NW = 2, KB = 32; };

SNRSE_DEV int swz(int row, int chunk) { return (row << 7) + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T>
SNRSE_DEV f32x4 mfma_chunk(const u32x4& a, const u32x4& b, f32x4 acc) {
  if constexpr (sizeof(T) == 2) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a),
                                                   __builtin_bit_cast(bf16x8_mfma, b), acc, 0, 0, 0);
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
  // bf16: the next K / V block is loaded into registers while the current one is consumed, and V is
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

}  // namespace

extern "C" int snrse_attention(const void* qkv, void* out, int B, int L, int C, int dtype, hipStream_t stream) {
  if (!qkv || !out || L <= 0 || B <= 0) return SNRSE_EINVAL;
  if (C != 256) return SNRSE_EINVAL;  // NCSN++ attention runs at 256 channels (ncsnpp.py:170-171)
  if (dtype == SNRSE_BF16) return launch_attn<bf16_t, 256>(qkv, out, B, L, stream);
  if (dtype == SNRSE_F32) return launch_attn<float, 256>(qkv, out, B, L, stream);
  return SNRSE_EINVAL;
}
