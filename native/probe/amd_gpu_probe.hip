// amd-gpu-probe: standalone MI355X readiness / health probe (no Python, ~100 ms warm start).
//
// Used as the readiness-check command of GPU pods (frameworks/helloworld/specs/gpu.yml): a pod
// that was given GPUs is only "ready" once the devices pass
//   --readiness : MFMA bf16 GEMM numerics (vs a host fp64 reference) + HBM address-hash pattern
//   --full      : additionally MFMA issue rate (TFLOP/s), 8192^3 GEMM rate and HBM copy bandwidth
// Exit status 0 = healthy, 1 = unhealthy, 2 = usage / HIP error. --json prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "probe_kernels.hip"

using namespace amdprobe;

#define HIP_OK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

namespace {

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);  // round to nearest even
  return static_cast<uint16_t>(u >> 16);
}

float bf16_to_f32(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

struct Lcg {
  uint64_t s;
  explicit Lcg(uint64_t seed) : s(seed * 6364136223846793005ULL + 1442695040888963407ULL) {}
  float next() {  // ~U(-1, 1)
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return static_cast<float>(static_cast<int32_t>(s >> 32)) / 2147483648.0f;
  }
};

struct Report {
  int device = 0;
  std::string arch;
  double gemm_rel_err = -1;
  unsigned long long mem_bad_words = 0;
  double mfma_tflops = -1, gemm_tflops = -1, hbm_gbps = -1;
  double seconds = 0;
  bool healthy = false;
};

// Launches the probe GEMM the way the in-process op does: the 256x256 LDS-DMA pipeline when the
// shape allows (big256 == true), else the 128x128 register-staged kernel.
void launch_gemm(hipStream_t st, bool big256, const void* a, const void* b, float* c, int M, int N, int K) {
  if (big256)
    hipLaunchKernelGGL(gemm_bf16_nt_256_kernel, dim3((M / big::BM) * (N / big::BN)), dim3(big::THREADS), 0, st,
                       static_cast<const __bf16*>(a), static_cast<const __bf16*>(b), c, M, N, K);
  else
    hipLaunchKernelGGL(gemm_bf16_nt_kernel, dim3((M / BM) * (N / BN)), dim3(GEMM_THREADS), 0, st,
                       static_cast<const __bf16*>(a), static_cast<const __bf16*>(b), c, M, N, K);
}

double gemm_check(hipStream_t st, bool big256, int M, int N, int K, uint64_t seed) {
  std::vector<uint16_t> a(static_cast<size_t>(M) * K), b(static_cast<size_t>(N) * K);
  Lcg g(seed);
  for (auto& x : a) x = f32_to_bf16(g.next());
  for (auto& x : b) x = f32_to_bf16(g.next());
  void *da, *db;
  float* dc;
  HIP_OK(hipMalloc(&da, a.size() * 2));
  HIP_OK(hipMalloc(&db, b.size() * 2));
  HIP_OK(hipMalloc(&dc, static_cast<size_t>(M) * N * 4));
  HIP_OK(hipMemcpyAsync(da, a.data(), a.size() * 2, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(db, b.data(), b.size() * 2, hipMemcpyHostToDevice, st));
  launch_gemm(st, big256, da, db, dc, M, N, K);
  HIP_OK(hipGetLastError());
  std::vector<float> c(static_cast<size_t>(M) * N);
  HIP_OK(hipMemcpyAsync(c.data(), dc, c.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  std::vector<float> af(a.size()), bfv(b.size());
  for (size_t i = 0; i < a.size(); ++i) af[i] = bf16_to_f32(a[i]);
  for (size_t i = 0; i < b.size(); ++i) bfv[i] = bf16_to_f32(b[i]);
  double num = 0, den = 0;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      double r = 0;
      const float* ar = &af[static_cast<size_t>(i) * K];
      const float* br = &bfv[static_cast<size_t>(j) * K];
      for (int k = 0; k < K; ++k) r += static_cast<double>(ar[k]) * br[k];
      double d = c[static_cast<size_t>(i) * N + j] - r;
      num += d * d;
      den += r * r;
    }
  HIP_OK(hipFree(da));
  HIP_OK(hipFree(db));
  HIP_OK(hipFree(dc));
  return std::sqrt(num / (den > 0 ? den : 1));
}

unsigned long long mem_check(hipStream_t st, size_t bytes, unsigned seed) {
  void* p;
  unsigned long long* errs;
  HIP_OK(hipMalloc(&p, bytes));
  HIP_OK(hipMalloc(&errs, sizeof(unsigned long long)));
  HIP_OK(hipMemsetAsync(errs, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(pattern_write_kernel, dim3(2048), dim3(256), 0, st, static_cast<uint4*>(p), bytes / 16, seed);
  hipLaunchKernelGGL(pattern_check_kernel, dim3(2048), dim3(256), 0, st, static_cast<const uint4*>(p), bytes / 16,
                     seed, errs);
  HIP_OK(hipGetLastError());
  unsigned long long h = 0;
  HIP_OK(hipMemcpyAsync(&h, errs, sizeof h, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipFree(p));
  HIP_OK(hipFree(errs));
  return h;
}

template <typename F>
double time_ms(hipStream_t st, int reps, F&& launch) {
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  launch();  // warm-up
  HIP_OK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) launch();
  HIP_OK(hipEventRecord(e1, st));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  return ms / reps;
}

void perf(hipStream_t st, Report& r) {
  // MFMA issue rate
  float* out;
  const int blocks = 2048, iters = 1024;
  HIP_OK(hipMalloc(&out, static_cast<size_t>(blocks) * 256 * 4));
  double ms = time_ms(st, 3, [&] {
    hipLaunchKernelGGL(mfma_peak_kernel, dim3(blocks), dim3(256), 0, st, out, iters, 1.0f);
  });
  double flops = static_cast<double>(blocks) * 4 * iters * 4 * (32.0 * 32 * 16 * 2);
  r.mfma_tflops = flops / (ms / 1e3) / 1e12;
  HIP_OK(hipFree(out));
  // GEMM rate: 8192^3 on the 256x256 pipeline (1024 tiles = 4 per CU), operands filled with an
  // address-hashed bit pattern (constant operands would understate switching power)
  const int S = 8192;
  void *a, *b;
  float* c;
  HIP_OK(hipMalloc(&a, static_cast<size_t>(S) * S * 2));
  HIP_OK(hipMalloc(&b, static_cast<size_t>(S) * S * 2));
  HIP_OK(hipMalloc(&c, static_cast<size_t>(S) * S * 4));
  hipLaunchKernelGGL(bf16_fill_kernel, dim3(2048), dim3(256), 0, st, static_cast<uint4*>(a),
                     static_cast<size_t>(S) * S / 8, 11u);
  hipLaunchKernelGGL(bf16_fill_kernel, dim3(2048), dim3(256), 0, st, static_cast<uint4*>(b),
                     static_cast<size_t>(S) * S / 8, 12u);
  ms = time_ms(st, 5, [&] { launch_gemm(st, true, a, b, c, S, S, S); });
  r.gemm_tflops = 2.0 * S * S * static_cast<double>(S) / (ms / 1e3) / 1e12;
  HIP_OK(hipFree(a));
  HIP_OK(hipFree(b));
  HIP_OK(hipFree(c));
  // HBM copy (larger than the 256 MiB Infinity Cache)
  const size_t bytes = static_cast<size_t>(1) << 30;
  void *s0, *s1;
  HIP_OK(hipMalloc(&s0, bytes));
  HIP_OK(hipMalloc(&s1, bytes));
  ms = time_ms(st, 5, [&] {
    hipLaunchKernelGGL(hbm_copy_kernel, dim3(HBM_COPY_BLOCKS), dim3(256), 0, st, static_cast<const uint4*>(s0),
                       static_cast<uint4*>(s1), bytes / 16);
  });
  r.hbm_gbps = 2.0 * bytes / (ms / 1e3) / 1e9;
  HIP_OK(hipFree(s0));
  HIP_OK(hipFree(s1));
}

void usage() {
  std::fprintf(stderr,
               "usage: amd-gpu-probe [--device N] [--readiness|--full] [--json]\n"
               "  exit 0 healthy, 1 unhealthy, 2 error\n");
}

}  // namespace

int main(int argc, char** argv) {
  int device = 0;
  bool full = false, json = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (a.rfind("--device=", 0) == 0) device = std::atoi(a.c_str() + 9);
    else if (a == "--readiness") full = false;
    else if (a == "--full") full = true;
    else if (a == "--json") json = true;
    else {
      usage();
      return 2;
    }
  }
  auto t0 = std::chrono::steady_clock::now();
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    std::fprintf(stderr, "no HIP devices visible\n");
    return 1;
  }
  if (device < 0 || device >= count) {
    std::fprintf(stderr, "device %d out of range (%d visible)\n", device, count);
    return 2;
  }
  HIP_OK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));
  Report r;
  r.device = device;
  r.arch = prop.gcnArchName;
  r.gemm_rel_err = std::max(gemm_check(st, false, 256, 256, 512, 1234 + device),
                            gemm_check(st, true, 512, 256, 512, 4321 + device));
  r.mem_bad_words = mem_check(st, 64u << 20, 77u + device);
  bool ok = r.gemm_rel_err < 1e-3 && r.mem_bad_words == 0;
  if (full) {
    perf(st, r);
    ok = ok && r.mfma_tflops > 200.0 && r.hbm_gbps > 1000.0;
  }
  HIP_OK(hipStreamDestroy(st));
  r.healthy = ok;
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (json) {
    std::printf("{\"device\": %d, \"arch\": \"%s\", \"gemm_rel_err\": %.3e, \"mem_bad_words\": %llu", r.device,
                r.arch.c_str(), r.gemm_rel_err, r.mem_bad_words);
    if (full)
      std::printf(", \"mfma_tflops\": %.1f, \"gemm_tflops\": %.1f, \"hbm_copy_gbps\": %.1f", r.mfma_tflops,
                  r.gemm_tflops, r.hbm_gbps);
    std::printf(", \"healthy\": %s, \"probe_seconds\": %.4f}\n", r.healthy ? "true" : "false", r.seconds);
  } else {
    std::printf("device %d (%s): gemm_rel_err=%.2e mem_bad_words=%llu%s -> %s\n", r.device, r.arch.c_str(),
                r.gemm_rel_err, r.mem_bad_words, full ? " (+perf)" : "", r.healthy ? "HEALTHY" : "UNHEALTHY");
  }
  return r.healthy ? 0 : 1;
}
