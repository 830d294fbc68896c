// HBM bandwidth sweep on one MI355X: copy variants (grid size x loads in flight x temporal hint)
// plus read-only and write-only roofs, 1 GiB buffers (4x the 256 MiB Infinity Cache).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/hbm_sweep.hip -o scripts/hbm_sweep
// Prints one JSON line per variant: {"variant", "blocks", "gbps"} (copy counts read + write bytes).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define HIP_OK(e)                                                                              \
  do {                                                                                         \
    hipError_t _e = (e);                                                                       \
    if (_e != hipSuccess) {                                                                    \
      std::fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(_e), __LINE__);         \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

template <int DEPTH, bool NT>
__global__ __launch_bounds__(256) void copy_strided(const u32x4* __restrict__ s, u32x4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (DEPTH - 1) * stride < n; i += DEPTH * stride) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) v[k] = NT ? __builtin_nontemporal_load(s + i + k * stride) : s[i + k * stride];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      if (NT)
        __builtin_nontemporal_store(v[k], d + i + k * stride);
      else
        d[i + k * stride] = v[k];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

// each block owns a contiguous span; per iteration a block moves DEPTH * 4 KiB
template <int DEPTH, bool NT>
__global__ __launch_bounds__(256) void copy_chunked(const u32x4* __restrict__ s, u32x4* __restrict__ d, size_t n) {
  const size_t per = n / gridDim.x;  // n divisible by grid * 256 * DEPTH in this sweep
  const u32x4* sb = s + blockIdx.x * per;
  u32x4* db = d + blockIdx.x * per;
  for (size_t i = threadIdx.x; i < per; i += DEPTH * 256) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) v[k] = NT ? __builtin_nontemporal_load(sb + i + k * 256) : sb[i + k * 256];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      if (NT)
        __builtin_nontemporal_store(v[k], db + i + k * 256);
      else
        db[i + k * 256] = v[k];
    }
  }
}

__global__ __launch_bounds__(256) void read_only(const u32x4* __restrict__ s, size_t n, unsigned* out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ e.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void write_only(u32x4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(u32x4{1u, 2u, 3u, (unsigned)i}, d + i);
}

template <typename F>
double time_ms(F&& f, int reps = 10) {
  hipEvent_t a, b;
  HIP_OK(hipEventCreate(&a));
  HIP_OK(hipEventCreate(&b));
  f();
  f();
  HIP_OK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  HIP_OK(hipEventRecord(b));
  HIP_OK(hipEventSynchronize(b));
  float ms;
  HIP_OK(hipEventElapsedTime(&ms, a, b));
  HIP_OK(hipGetLastError());
  return ms / reps;
}

int main() {
  const size_t bytes = size_t(1) << 30, n = bytes / 16;
  u32x4 *s, *d;
  unsigned* o;
  HIP_OK(hipMalloc(&s, bytes));
  HIP_OK(hipMalloc(&d, bytes));
  HIP_OK(hipMalloc(&o, 4));
  HIP_OK(hipMemset(s, 1, bytes));
  auto report = [&](const char* v, int blocks, double ms, double moved) {
    std::printf("{\"variant\": \"%s\", \"blocks\": %d, \"gbps\": %.1f}\n", v, blocks, moved / (ms / 1e3) / 1e9);
    std::fflush(stdout);
  };
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) {
    report("strided4", g, time_ms([&] { copy_strided<4, false><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("strided4_nt", g, time_ms([&] { copy_strided<4, true><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("strided8_nt", g, time_ms([&] { copy_strided<8, true><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("chunked4", g, time_ms([&] { copy_chunked<4, false><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("chunked4_nt", g, time_ms([&] { copy_chunked<4, true><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("chunked8_nt", g, time_ms([&] { copy_chunked<8, true><<<g, 256>>>(s, d, n); }), 2.0 * bytes);
    report("read_only", g, time_ms([&] { read_only<<<g, 256>>>(s, n, o); }), 1.0 * bytes);
    report("write_only_nt", g, time_ms([&] { write_only<<<g, 256>>>(d, n); }), 1.0 * bytes);
  }
  HIP_OK(hipFree(s));
  HIP_OK(hipFree(d));
  HIP_OK(hipFree(o));
  return 0;
}
