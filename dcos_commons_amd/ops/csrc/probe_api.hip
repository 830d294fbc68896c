// C ABI over the probe kernels; loaded in-process by dcos_commons_amd.ops (ctypes) with torch
// tensors' device pointers and the current HIP stream. Every entry point validates the shapes
// the kernel's grid assumes before launching and returns a hipError_t (0 = success) or a
// negative code for a rejected shape.
#include "probe_kernels.hip"

#define AMDPROBE_EXPORT extern "C" __attribute__((visibility("default")))

using namespace amdprobe;

enum { ERR_SHAPE = -1, ERR_ALIGN = -2 };

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

AMDPROBE_EXPORT int amdprobe_version() { return 1; }

// variant: 0 = pick (256x256 glds pipeline when the shape allows, else 128x128),
//          1 = 128x128 register-staged, 2 = 256x256 glds pipeline (M, N % 256 == 0, K % 128 == 0)
AMDPROBE_EXPORT int amdprobe_gemm_bf16_nt_variant(const void* A, const void* Bt, float* C, int M, int N, int K,
                                                  int variant, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return ERR_SHAPE;
  if (!aligned16(A) || !aligned16(Bt) || !aligned16(C)) return ERR_ALIGN;
  const bool big_ok = M % big::BM == 0 && N % big::BN == 0 && K % (2 * big::BK) == 0;
  if (variant == 0) variant = big_ok ? 2 : 1;
  if (variant == 2) {
    if (!big_ok) return ERR_SHAPE;
    const int nwg = (M / big::BM) * (N / big::BN);
    hipLaunchKernelGGL(gemm_bf16_nt_256_kernel, dim3(nwg), dim3(big::THREADS), 0, (hipStream_t)stream,
                       (const __bf16*)A, (const __bf16*)Bt, C, M, N, K);
    return (int)hipGetLastError();
  }
  if (variant != 1 || M % BM || N % BN || K % BK) return ERR_SHAPE;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(gemm_bf16_nt_kernel, dim3(nwg), dim3(GEMM_THREADS), 0, (hipStream_t)stream,
                     (const __bf16*)A, (const __bf16*)Bt, C, M, N, K);
  return (int)hipGetLastError();
}

AMDPROBE_EXPORT int amdprobe_gemm_bf16_nt(const void* A, const void* Bt, float* C, int M, int N, int K,
                                          void* stream) {
  return amdprobe_gemm_bf16_nt_variant(A, Bt, C, M, N, K, 0, stream);
}

AMDPROBE_EXPORT int amdprobe_mfma_peak(float* out, int blocks, int iters, float seed, void* stream) {
  if (blocks <= 0 || iters <= 0) return ERR_SHAPE;
  hipLaunchKernelGGL(mfma_peak_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, seed);
  return (int)hipGetLastError();
}

// FLOPs issued by one amdprobe_mfma_peak launch (for the caller's TFLOP/s).
AMDPROBE_EXPORT double amdprobe_mfma_peak_flops(int blocks, int iters) {
  const double waves = (double)blocks * 4.0;
  return waves * (double)iters * 4.0 * (32.0 * 32.0 * 16.0 * 2.0);
}

AMDPROBE_EXPORT int amdprobe_hbm_copy(const void* src, void* dst, size_t bytes, int blocks, void* stream) {
  if (bytes == 0 || bytes % 16 || blocks <= 0) return ERR_SHAPE;
  if (!aligned16(src) || !aligned16(dst)) return ERR_ALIGN;
  hipLaunchKernelGGL(hbm_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)src,
                     (uint4*)dst, bytes / 16);
  return (int)hipGetLastError();
}

AMDPROBE_EXPORT int amdprobe_pattern_write(void* p, size_t bytes, unsigned seed, int blocks, void* stream) {
  if (bytes == 0 || bytes % 16 || blocks <= 0) return ERR_SHAPE;
  if (!aligned16(p)) return ERR_ALIGN;
  hipLaunchKernelGGL(pattern_write_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (uint4*)p, bytes / 16,
                     (uint32_t)seed);
  return (int)hipGetLastError();
}

AMDPROBE_EXPORT int amdprobe_pattern_check(const void* p, size_t bytes, unsigned seed, unsigned long long* errors,
                                           int blocks, void* stream) {
  if (bytes == 0 || bytes % 16 || blocks <= 0) return ERR_SHAPE;
  if (!aligned16(p)) return ERR_ALIGN;
  hipLaunchKernelGGL(pattern_check_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p,
                     bytes / 16, (uint32_t)seed, errors);
  return (int)hipGetLastError();
}
