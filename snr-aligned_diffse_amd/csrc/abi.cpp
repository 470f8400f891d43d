// C-ABI housekeeping entries of libsnrse_hip.so (see include/snrse.h): version / error text / device
// name, and the caller-owned launch contexts (snrse_ctx, common.h) with their switches.
#include <hip/hip_runtime.h>

#include <new>

#include "common.h"

extern "C" int snrse_abi_version(void) { return 2; }

// Source hash of the tree this library was compiled from (snrse/build.py: sha256 over csrc/* and the
// build script, passed as -DSNRSE_BUILD_ID), so a run can show that the binary it loaded matches HEAD.
#ifndef SNRSE_BUILD_ID
#define SNRSE_BUILD_ID "unknown"
#endif
extern "C" const char* snrse_build_id(void) { return SNRSE_BUILD_ID; }

extern "C" const char* snrse_error_string(int code) { return hipGetErrorString((hipError_t)code); }

// Name and gfx target of the current device into `buf` (nul-terminated); returns 0 or a hipError_t.
extern "C" int snrse_device_name(char* buf, int len) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  int i = 0;
  for (const char* s = prop.gcnArchName; *s && i < len - 1; ++s) buf[i++] = *s;
  if (len > 0) buf[i] = 0;
  return 0;
}

namespace {
// The process default context: what a NULL context means, and what snrse_set_option /
// snrse_set_workspace edit (single-stream callers; not reentrant).
snrse_ctx g_default_ctx;

bool name_is(const char* a, const char* b) {
  int i = 0;
  while (a[i] && a[i] == b[i]) ++i;
  return a[i] == 0 && b[i] == 0;
}

// switch name -> field (nullptr: unknown)
int* option_field(snrse_ctx& c, const char* name) {
  if (name_is(name, "conv_variant")) return &c.conv_variant;
  if (name_is(name, "splitk")) return &c.splitk;
  if (name_is(name, "splitk_target")) return &c.splitk_target;
  if (name_is(name, "epi_nt")) return &c.epi_nt;
  if (name_is(name, "epi_nt_mb")) return &c.epi_nt_mb;
  if (name_is(name, "h5_specialise")) return &c.h5_specialise;
  if (name_is(name, "h5_tw")) return &c.h5_tw;
  if (name_is(name, "stats_zeroed")) return &c.stats_zeroed;
  if (name_is(name, "resample_variant")) return &c.resample_variant;
  if (name_is(name, "resample_nt")) return &c.resample_nt;
  if (name_is(name, "resample_down_rows")) return &c.resample_down_rows;
  if (name_is(name, "x3_tile")) return &c.x3_tile;
  if (name_is(name, "x3_spread")) return &c.x3_spread;
  if (name_is(name, "ic_lds")) return &c.ic_lds;
  if (name_is(name, "x3_nt")) return &c.x3_nt;
  if (name_is(name, "x3_tw")) return &c.x3_tw;
  if (name_is(name, "head_small")) return &c.head_small;
  if (name_is(name, "head_part")) return &c.head_part;
  if (name_is(name, "gn_slice")) return &c.gn_slice;
  return nullptr;
}

int set_option(snrse_ctx& c, const char* name, int value) {
  if (!name) return SNRSE_EINVAL;
  int* f = option_field(c, name);
  if (!f) return SNRSE_EINVAL;
  if (name_is(name, "splitk_target") || name_is(name, "epi_nt_mb")) value = value > 0 ? value : 256;
  if (name_is(name, "stats_zeroed")) value = value ? 1 : 0;
  *f = value;
  return 0;
}

int get_option(const snrse_ctx& c, const char* name, int* value) {
  if (!name || !value) return SNRSE_EINVAL;
  if (const int* f = option_field(const_cast<snrse_ctx&>(c), name)) { *value = *f; return 0; }
  if (name_is(name, "halo_kernel")) { *value = 5; return 0; }  // the halo generation variant 0 takes
  if (name_is(name, "last_kernel")) { *value = c.last_kernel; return 0; }
  if (name_is(name, "last_ksplit")) { *value = c.last_ksplit; return 0; }
  if (name_is(name, "last_epi_nt")) { *value = c.last_epi_nt; return 0; }
  if (name_is(name, "last_chunks")) { *value = c.last_chunks; return 0; }
  if (name_is(name, "last_tw")) { *value = c.last_tw; return 0; }
  return SNRSE_EINVAL;
}

int set_workspace(snrse_ctx& c, void* ptr, size_t bytes) {
  if (!ptr && bytes) return SNRSE_EINVAL;
  c.ws = (float*)ptr;
  c.ws_bytes = ptr ? bytes : 0;
  return 0;
}
}  // namespace

__attribute__((visibility("hidden"))) snrse_ctx* snrse_ctx_resolve(snrse_ctx* c) { return c ? c : &g_default_ctx; }

namespace {
void probe_free(snrse_ctx& c) {
  for (int i = 0; i < 2 * c.probe_cap; ++i) (void)hipEventDestroy(c.probe_ev[i]);
  delete[] c.probe_ev;
  delete[] c.probe_kernel;
  c.probe_ev = nullptr;
  c.probe_kernel = nullptr;
  c.probe_cap = c.probe_n = 0;
}
}  // namespace

__attribute__((visibility("hidden"))) int snrse_ctx_probe_mark(snrse_ctx& c, hipStream_t s, bool end) {
  if (c.probe_n >= c.probe_cap) return 0;
  if (end) {
    c.probe_kernel[c.probe_n] = c.last_kernel;
    return (int)hipEventRecord(c.probe_ev[2 * c.probe_n++ + 1], s);
  }
  return (int)hipEventRecord(c.probe_ev[2 * c.probe_n], s);
}

// Diagnostic timing of snrse_conv2d calls: `capacity` event pairs, created without the system-scope
// fence (an event whose record flushes the caches to system scope puts that write-back inside the
// bracket: ~50 us per fp32 conv call at C5, profiles/r03g_c5_probe_vs_rocprof.json).  capacity 0 frees them.
extern "C" int snrse_ctx_probe_begin(snrse_ctx* ctx, int capacity) {
  snrse_ctx& c = *snrse_ctx_resolve(ctx);
  probe_free(c);
  if (capacity <= 0) return 0;
  c.probe_ev = new (std::nothrow) hipEvent_t[2 * (size_t)capacity];
  c.probe_kernel = new (std::nothrow) int[capacity];
  if (!c.probe_ev || !c.probe_kernel) {
    delete[] c.probe_ev;
    delete[] c.probe_kernel;
    c.probe_ev = nullptr;
    c.probe_kernel = nullptr;
    return (int)hipErrorOutOfMemory;
  }
  for (int i = 0; i < 2 * capacity; ++i) {
    const hipError_t e = hipEventCreateWithFlags(&c.probe_ev[i], hipEventDisableSystemFence);
    if (e != hipSuccess) {
      c.probe_cap = i / 2;
      for (int j = 2 * c.probe_cap; j < i; ++j) (void)hipEventDestroy(c.probe_ev[j]);
      probe_free(c);
      return (int)e;
    }
  }
  c.probe_cap = capacity;
  c.probe_n = 0;
  return 0;
}

// Waits for the probed calls and writes, in call order, each call's device time (ms, first kernel start
// to last kernel end of the call) and the kernel generation that ran; *n = number of calls recorded.
extern "C" int snrse_ctx_probe_read(snrse_ctx* ctx, float* ms, int* kernel, int max, int* n) {
  snrse_ctx& c = *snrse_ctx_resolve(ctx);
  if (!n) return SNRSE_EINVAL;
  const int m = c.probe_n < max ? c.probe_n : max;
  for (int i = 0; i < m; ++i) {
    hipError_t e = hipEventSynchronize(c.probe_ev[2 * i + 1]);
    if (e != hipSuccess) return (int)e;
    if (ms) {
      e = hipEventElapsedTime(&ms[i], c.probe_ev[2 * i], c.probe_ev[2 * i + 1]);
      if (e != hipSuccess) return (int)e;
    }
    if (kernel) kernel[i] = c.probe_kernel[i];
  }
  *n = m;
  return 0;
}

// A new context starts with the process default context's switches (so SNRSE_OPTS / snrse_set_option
// settings made before carry over), no workspace and cleared read-backs.
extern "C" snrse_ctx* snrse_ctx_create(void) {
  snrse_ctx* c = new (std::nothrow) snrse_ctx(g_default_ctx);
  if (!c) return nullptr;
  c->ws = nullptr;
  c->ws_bytes = 0;
  c->last_kernel = 0;
  c->last_ksplit = 1;
  c->last_epi_nt = 0;
  c->last_chunks = 1;
  c->last_tw = 0;
  c->probe_ev = nullptr;
  c->probe_kernel = nullptr;
  c->probe_cap = c->probe_n = 0;
  return c;
}

extern "C" void snrse_ctx_destroy(snrse_ctx* ctx) {
  if (ctx) probe_free(*ctx);
  delete ctx;
}

extern "C" int snrse_ctx_set_workspace(snrse_ctx* ctx, void* ptr, size_t bytes) {
  return set_workspace(*snrse_ctx_resolve(ctx), ptr, bytes);
}
extern "C" int snrse_ctx_set_option(snrse_ctx* ctx, const char* name, int value) {
  return set_option(*snrse_ctx_resolve(ctx), name, value);
}
extern "C" int snrse_ctx_get_option(const snrse_ctx* ctx, const char* name, int* value) {
  return get_option(*snrse_ctx_resolve(const_cast<snrse_ctx*>(ctx)), name, value);
}

// Process-default forms (a NULL context): kept for single-stream callers and SNRSE_OPTS.
extern "C" int snrse_set_workspace(void* ptr, size_t bytes) { return set_workspace(g_default_ctx, ptr, bytes); }
extern "C" int snrse_set_option(const char* name, int value) { return set_option(g_default_ctx, name, value); }
extern "C" int snrse_get_option(const char* name, int* value) { return get_option(g_default_ctx, name, value); }
