// C ABI over the probe kernels; loaded in-process by dcos_commons_amd.ops (ctypes) with torch
// tensors' device pointers and the current HIP stream. Every entry point validates the shapes
// the kernel's grid assumes before launching and returns a hipError_t (0 = success) or a
// negative code for a rejected shape.
#include "probe_kernels.hip"

#include <cmath>
#include <mutex>

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

// Dense fp32 check of C = A Bt^T: adds sum((C - A Bt^T)^2) to out2[0] and sum((A Bt^T)^2) to
// out2[1] (device pointer, 2 floats that the caller zeroes).
AMDPROBE_EXPORT int amdprobe_gemm_check(const void* A, const void* Bt, const float* C, int M, int N, int K,
                                        int inject, float* out2, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % CHECK_TILE || N % CHECK_TILE || K % 8 || K > CHECK_MAX_K) return ERR_SHAPE;
  if (!aligned16(A) || !aligned16(Bt)) return ERR_ALIGN;
  hipLaunchKernelGGL(gemm_check_kernel, dim3((M / CHECK_TILE) * (N / CHECK_TILE)), dim3(CHECK_THREADS), 0,
                     (hipStream_t)stream, (const __bf16*)A, (const __bf16*)Bt, C, M, N, K, inject, out2);
  return (int)hipGetLastError();
}

// The readiness operand fill on its own (tests compare it with a host model of the hash):
// `ab` gets `ab_bytes` of hashed bf16 and `res` (32 bytes) is zeroed.
AMDPROBE_EXPORT int amdprobe_readiness_fill(void* ab, size_t ab_bytes, unsigned seed, void* res, void* stream) {
  if (ab_bytes == 0 || ab_bytes % 16) return ERR_SHAPE;
  if (!aligned16(ab) || !aligned16(res)) return ERR_ALIGN;
  hipLaunchKernelGGL(readiness_prep_kernel, dim3(64), dim3(256), 0, (hipStream_t)stream, (uint4*)ab, ab_bytes / 16,
                     (uint32_t)seed, (ReadinessResult*)res);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// amdprobe_readiness: the whole readiness check of one device in one call (see the kernel file).
// Buffers, a non-blocking stream and a pinned result slot are created on first use per device
// and reused; calls for one device serialize on its context. The calling thread's current device
// is restored. inject: 0 = none, 1 = lose one 16x16 tile of the product (the check must fail), 2 = corrupt one
// pattern word (the memory check must count it), 3 = skip the GEMM launch, 4 = skip the pattern write (both
// model a kernel that silently drops its writes; the check must still fail). Returns 0 or a HIP error /
// negative shape code.
//
// The buffers outlive the call, so a kernel that dropped its writes would leave the previous call's correct
// data behind. Two things stop that from passing: C is poisoned with NaN bytes before the GEMM, and every
// call mixes a per-device call counter into the seed, so the operands and the pattern differ from the last
// call's and stale data cannot match.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int RM = 256, RN = 256, RK = 512;
constexpr size_t PATTERN_BYTES = size_t(64) << 20;
constexpr int MAX_DEVICES = 64;

struct ReadinessCtx {
  std::mutex mu;
  bool ready = false;
  hipStream_t stream = nullptr;
  __bf16* ab = nullptr;          // A (RM x RK) then Bt (RN x RK)
  float* c = nullptr;            // RM x RN
  uint4* pattern = nullptr;
  ReadinessResult* res = nullptr;
  ReadinessResult* host = nullptr;  // pinned
  uint32_t calls = 0;               // mixed into the seed: no two calls share operands or pattern
};
ReadinessCtx g_readiness[MAX_DEVICES];

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define PROBE_TRY(expr)                                  \
  do {                                                   \
    const hipError_t e_ = (expr);                        \
    if (e_ != hipSuccess) return (int)e_;                \
  } while (0)

void readiness_release(ReadinessCtx& ctx) {
  if (ctx.stream != nullptr) (void)hipStreamDestroy(ctx.stream);
  if (ctx.ab != nullptr) (void)hipFree(ctx.ab);
  if (ctx.c != nullptr) (void)hipFree(ctx.c);
  if (ctx.pattern != nullptr) (void)hipFree(ctx.pattern);
  if (ctx.res != nullptr) (void)hipFree(ctx.res);
  if (ctx.host != nullptr) (void)hipHostFree(ctx.host);
  ctx.stream = nullptr;
  ctx.ab = nullptr;
  ctx.c = nullptr;
  ctx.pattern = nullptr;
  ctx.res = nullptr;
  ctx.host = nullptr;
}

int readiness_alloc(ReadinessCtx& ctx) {
  PROBE_TRY(hipStreamCreateWithFlags(&ctx.stream, hipStreamNonBlocking));
  PROBE_TRY(hipMalloc((void**)&ctx.ab, size_t(RM + RN) * RK * sizeof(__bf16)));
  PROBE_TRY(hipMalloc((void**)&ctx.c, size_t(RM) * RN * sizeof(float)));
  PROBE_TRY(hipMalloc((void**)&ctx.pattern, PATTERN_BYTES));
  PROBE_TRY(hipMalloc((void**)&ctx.res, sizeof(ReadinessResult)));
  PROBE_TRY(hipHostMalloc((void**)&ctx.host, sizeof(ReadinessResult), hipHostMallocDefault));
  return 0;
}

// The context lives for the process (one probe per pod launch reuses it); a failed allocation
// releases whatever it got, so the next call starts clean instead of leaking.
int readiness_init(ReadinessCtx& ctx) {
  const int rc = readiness_alloc(ctx);
  if (rc) {
    readiness_release(ctx);
    return rc;
  }
  ctx.ready = true;
  return 0;
}
}  // namespace

AMDPROBE_EXPORT int amdprobe_readiness(int device, unsigned seed, int inject, double* rel_err,
                                       unsigned long long* bad_words) {
  if (rel_err == nullptr || bad_words == nullptr || device < 0 || device >= MAX_DEVICES) return ERR_SHAPE;
  int ndev = 0;
  PROBE_TRY(hipGetDeviceCount(&ndev));
  if (device >= ndev) return ERR_SHAPE;
  ReadinessCtx& ctx = g_readiness[device];
  std::lock_guard<std::mutex> lock(ctx.mu);
  DeviceGuard guard(device);
  if (!ctx.ready) {
    const int rc = readiness_init(ctx);
    if (rc) return rc;
  }
  hipStream_t s = ctx.stream;
  const __bf16* A = ctx.ab;
  const __bf16* Bt = ctx.ab + size_t(RM) * RK;
  const uint32_t call_seed = (uint32_t)seed ^ (0x9E3779B9u * ++ctx.calls);
  hipLaunchKernelGGL(readiness_prep_kernel, dim3(64), dim3(256), 0, s, (uint4*)ctx.ab,
                     size_t(RM + RN) * RK * sizeof(__bf16) / 16, call_seed, ctx.res);
  PROBE_TRY(hipGetLastError());
  PROBE_TRY(hipMemsetAsync(ctx.c, 0xFF, size_t(RM) * RN * sizeof(float), s));  // NaN until the GEMM writes
  if (inject != 3) {
    // 128x128 tiles: four workgroups for the 256x256 product (one 256x256-tile workgroup takes ~15 us)
    const int rc = amdprobe_gemm_bf16_nt_variant(A, Bt, ctx.c, RM, RN, RK, 1, s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(gemm_check_kernel, dim3((RM / CHECK_TILE) * (RN / CHECK_TILE)), dim3(CHECK_THREADS), 0, s, A,
                     Bt, (const float*)ctx.c, RM, RN, RK, inject == 1 ? 1 : 0, &ctx.res->diff2);
  PROBE_TRY(hipGetLastError());
  if (inject != 4) {
    hipLaunchKernelGGL(pattern_write_kernel, dim3(2048), dim3(256), 0, s, ctx.pattern, PATTERN_BYTES / 16,
                       call_seed);
    PROBE_TRY(hipGetLastError());
  }
  if (inject == 2) PROBE_TRY(hipMemsetAsync(ctx.pattern, 0, 4, s));
  hipLaunchKernelGGL(pattern_check_kernel, dim3(2048), dim3(256), 0, s, (const uint4*)ctx.pattern,
                     PATTERN_BYTES / 16, call_seed, &ctx.res->bad_words);
  PROBE_TRY(hipGetLastError());
  PROBE_TRY(hipMemcpyAsync(ctx.host, ctx.res, sizeof(ReadinessResult), hipMemcpyDeviceToHost, s));
  PROBE_TRY(hipStreamSynchronize(s));
  const double d2 = ctx.host->diff2, w2 = ctx.host->ref2;
  *rel_err = (w2 > 0.0 && std::isfinite(d2)) ? std::sqrt(d2 / w2) : HUGE_VAL;  // NaN C (never written) fails
  *bad_words = ctx.host->bad_words;
  return 0;
}
