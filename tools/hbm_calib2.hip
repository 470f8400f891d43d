// HBM ceiling reconciliation: the round-3 calibration (tools/hbm_calib.hip: one 16-B vector
// per lane per iteration, grid-stride, 2048 / 8192 workgroups) measured copy 5.07-5.21 TB/s, while
// MI355X_MICROARCH.md:36 records 6.29 TB/s for a float4 copy.  This sweep varies what that calibration held fixed:
// vectors in flight per lane (U = 1, 2, 4, 8 loads issued before the first store), the grid (1-32 workgroups per
// CU of 256 threads) and the traversal (grid-stride vs one contiguous slab per workgroup), for read, write, copy and
// the 2:1 read:write mix; plain and non-temporal stores.  bytes = bytes read + bytes written; buffers 1-2 GiB
// (beyond the 256 MB Infinity Cache); median of `reps` launches after a warm-up, HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_calib2 tools/hbm_calib2.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <bool NT>
__device__ inline void st(u32x4* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// MODE 0 read, 1 write, 2 copy, 3 read2write1; SLAB: each workgroup walks one contiguous range
template <int MODE, int U, bool NT, bool SLAB>
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                u32x4* __restrict__ o, size_t n, unsigned* __restrict__ sink) {
  size_t i0, step, end;
  if (SLAB) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    i0 = blockIdx.x * per + threadIdx.x;
    end = std::min(n, (size_t)(blockIdx.x + 1) * per);
    step = 256;
  } else {
    i0 = blockIdx.x * 256ull + threadIdx.x;
    end = n;
    step = (size_t)gridDim.x * 256;
  }
  unsigned acc = 0;
  for (size_t i = i0; i < end; i += step * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = i + u * step;
      if (MODE == 1) v[u] = u32x4{(unsigned)k, 7u, (unsigned)k, 9u};
      else v[u] = k < end ? a[k] : u32x4{0u, 0u, 0u, 0u};
      if (MODE == 3 && k < end) v[u] += b[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t k = i + u * step;
      if (MODE == 0) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
      else if (k < end) st<NT>(o + k, v[u]);
    }
  }
  if (MODE == 0 && acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keeps the loads
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const size_t GB = 1ull << 30, n = GB / 16;
  u32x4 *a, *b, *o;
  unsigned* sink;
  CHECK(hipMalloc(&a, 2 * GB));
  CHECK(hipMalloc(&b, GB));
  CHECK(hipMalloc(&o, GB));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(a, 1, 2 * GB));
  CHECK(hipMemset(b, 2, GB));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int per_cu[] = {1, 2, 4, 8, 16, 32};
  const char* names[] = {"read", "write", "copy", "read2write1"};
  auto time_it = [&](auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      CHECK(hipEventRecord(e0, 0));
      launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return (double)ts[ts.size() / 2];
  };
  auto sweep = [&](auto kern, int mode, int U, bool nt, bool slab) {
    const size_t nn = mode == 0 ? 2 * n : n;
    const double bytes = mode == 0 ? 2.0 * GB : mode == 1 ? 1.0 * GB : mode == 2 ? 2.0 * GB : 3.0 * GB;
    for (int k : per_cu) {
      const int g = cus * k;
      const double ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, a, b, o, nn, sink); });
      printf("{\"mode\": \"%s\", \"U\": %d, \"nt\": %d, \"slab\": %d, \"wg_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f, "
             "\"frac_of_8TBps\": %.3f}\n",
             names[mode], U, (int)nt, (int)slab, k, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 8.0);
      fflush(stdout);
    }
  };
#define SWEEP_U(MODE, NT, SLAB)                                   \
  sweep(k_stream<MODE, 1, NT, SLAB>, MODE, 1, NT, SLAB);           \
  sweep(k_stream<MODE, 2, NT, SLAB>, MODE, 2, NT, SLAB);           \
  sweep(k_stream<MODE, 4, NT, SLAB>, MODE, 4, NT, SLAB);           \
  sweep(k_stream<MODE, 8, NT, SLAB>, MODE, 8, NT, SLAB);
  SWEEP_U(0, false, false)
  SWEEP_U(0, false, true)
  SWEEP_U(1, false, false)
  SWEEP_U(1, true, false)
  SWEEP_U(1, false, true)
  SWEEP_U(2, false, false)
  SWEEP_U(2, true, false)
  SWEEP_U(2, false, true)
  SWEEP_U(2, true, true)
  SWEEP_U(3, false, false)
  SWEEP_U(3, true, false)
  SWEEP_U(3, false, true)
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  return 0;
}
