// MI355X (gfx950) device-validation kernels used by the GPU readiness/health probe.
//
// A pod that asks for `gpus: N` is only "ready" once the GPUs it was given pass these checks
// (the reference has no GPU code at all: its only GPU surface is the Mesos `gpus` scalar,
// sdk/scheduler/.../offer/Constants.java:62). The probe exercises every unit a training or
// serving payload depends on:
//   * MFMA matrix cores  -- a 128x128x64-tiled bf16 GEMM on v_mfma_f32_16x16x32_bf16
//                           (checked against an fp32 reference) and a register-resident
//                           v_mfma_f32_32x32x16_bf16 issue-rate loop (peak TFLOP/s);
//   * HBM3E              -- a 16-B/lane vectorized streaming copy (bandwidth) and an
//                           address-hashed write/verify pattern test (integrity);
// All kernels are wave64-native, XCD-aware where it matters, and launch with fixed shapes
// that the host wrappers validate before launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amdprobe {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------
// bf16 GEMM:  C[M][N] (fp32) = A[M][K] * Bt[N][K]^T   (A and Bt are K-contiguous)
// Block tile 128x128, BK = 64, 256 threads = 4 waves in a 2x2 grid, each wave 64x64 =
// 4x4 MFMA 16x16x32 tiles. LDS double buffer with register staging (issue the next tile's
// global loads before the MFMA block, write them to the other LDS buffer after it), rows
// padded by 16 B so each ds_read_b128 lane group spans all 64 banks.
// ---------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int GEMM_THREADS = 256;
constexpr int LDS_ROW = BK + 8;                 // bf16 elements per padded LDS row (144 B)
constexpr int TILE_ELEMS = BM * LDS_ROW;        // one operand tile
constexpr int CHUNKS_PER_ROW = BK / 8;          // 16-B chunks per tile row
constexpr int CHUNKS_PER_THREAD = BM * CHUNKS_PER_ROW / GEMM_THREADS;  // 4

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // bijective blockIdx -> tile remap that gives each XCD (blockIdx % 8) a contiguous tile run
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

__global__ __launch_bounds__(GEMM_THREADS, 2)
void gemm_bf16_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                         float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 2 * TILE_ELEMS];  // [buf][A|B][row][k]
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const __bf16* Ablk = A + (size_t)tm * BM * K;
  const __bf16* Bblk = Bt + (size_t)tn * BN * K;

  uint4 ra[CHUNKS_PER_THREAD], rb[CHUNKS_PER_THREAD];
  // per-thread staging coordinates (row, 16-B chunk) are loop invariant
  int srow[CHUNKS_PER_THREAD], scol[CHUNKS_PER_THREAD];
#pragma unroll
  for (int i = 0; i < CHUNKS_PER_THREAD; ++i) {
    const int c = tid + i * GEMM_THREADS;
    srow[i] = c / CHUNKS_PER_ROW;
    scol[i] = (c % CHUNKS_PER_ROW) * 8;
  }
  floatx4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int ktiles = K / BK;
  {
    const int K0 = 0, BUF = 0;
#pragma unroll
    for (int i = 0; i < CHUNKS_PER_THREAD; ++i) {
      ra[i] = *reinterpret_cast<const uint4*>(Ablk + (size_t)srow[i] * K + K0 + scol[i]);
      rb[i] = *reinterpret_cast<const uint4*>(Bblk + (size_t)srow[i] * K + K0 + scol[i]);
    }
#pragma unroll
    for (int i = 0; i < CHUNKS_PER_THREAD; ++i) {
      __bf16* la_ = lds + BUF * 2 * TILE_ELEMS;
      *reinterpret_cast<uint4*>(la_ + srow[i] * LDS_ROW + scol[i]) = ra[i];
      *reinterpret_cast<uint4*>(la_ + TILE_ELEMS + srow[i] * LDS_ROW + scol[i]) = rb[i];
    }
  }
  __syncthreads();
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    {  // next tile in flight under the MFMA block (the last iteration re-loads its own tile)
      const int K0 = (kt + 1 < ktiles ? kt + 1 : kt) * BK;
  #pragma unroll
      for (int i = 0; i < CHUNKS_PER_THREAD; ++i) {
        ra[i] = *reinterpret_cast<const uint4*>(Ablk + (size_t)srow[i] * K + K0 + scol[i]);
        rb[i] = *reinterpret_cast<const uint4*>(Bblk + (size_t)srow[i] * K + K0 + scol[i]);
      }
    }
    const __bf16* la = lds + cur * 2 * TILE_ELEMS;
    const __bf16* lb = la + TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        af[m] = *reinterpret_cast<const bf16x8*>(la + (wr * 64 + m * 16 + frow) * LDS_ROW + ks * 32 + fk);
#pragma unroll
      for (int n = 0; n < 4; ++n)
        bfr[n] = *reinterpret_cast<const bf16x8*>(lb + (wc * 64 + n * 16 + frow) * LDS_ROW + ks * 32 + fk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    {  // other buffer: its last reader finished before the previous barrier
      const int BUF = cur ^ 1;
  #pragma unroll
      for (int i = 0; i < CHUNKS_PER_THREAD; ++i) {
        __bf16* la_ = lds + BUF * 2 * TILE_ELEMS;
        *reinterpret_cast<uint4*>(la_ + srow[i] * LDS_ROW + scol[i]) = ra[i];
        *reinterpret_cast<uint4*>(la_ + TILE_ELEMS + srow[i] * LDS_ROW + scol[i]) = rb[i];
      }
    }
    __syncthreads();
  }
  // epilogue: col = lane & 15, row = (lane >> 4) * 4 + j
  float* Cblk = C + (size_t)tm * BM * N + (size_t)tn * BN;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wr * 64 + m * 16 + (lane >> 4) * 4 + j;
        const int col = wc * 64 + n * 16 + (lane & 15);
        Cblk[(size_t)row * N + col] = acc[m][n][j];
      }
}

// ---------------------------------------------------------------------------------------
// MFMA issue-rate probe: each wave keeps 4 independent 32x32x16 bf16 accumulators busy
// (dependent latency is covered by the 4-deep chain), `iters` rounds. Output keeps the
// result live so nothing is dead-code eliminated.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256)
void mfma_peak_kernel(float* __restrict__ out, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (float)((lane + j) & 7) * 0.125f);
    b[j] = (__bf16)(seed * (float)((lane * 3 + j) & 7) * 0.0625f);
  }
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---------------------------------------------------------------------------------------
// HBM streaming copy: 16 B per lane per access, grid-stride, 4 independent loads in flight.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256)
void hbm_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 v0 = src[i], v1 = src[i + stride], v2 = src[i + 2 * stride], v3 = src[i + 3 * stride];
    dst[i] = v0;
    dst[i + stride] = v1;
    dst[i + 2 * stride] = v2;
    dst[i + 3 * stride] = v3;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------
// HBM integrity: write an address-hashed pattern, then verify it and count bad words.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

__global__ __launch_bounds__(256)
void pattern_write_kernel(uint4* __restrict__ p, size_t n16, uint32_t seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint64_t base = (i << 2) ^ ((uint64_t)seed << 40);
    p[i] = make_uint4(mix32(base), mix32(base + 1), mix32(base + 2), mix32(base + 3));
  }
}

__global__ __launch_bounds__(256)
void pattern_check_kernel(const uint4* __restrict__ p, size_t n16, uint32_t seed,
                          unsigned long long* __restrict__ errors) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t bad = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint64_t base = (i << 2) ^ ((uint64_t)seed << 40);
    const uint4 v = p[i];
    bad += (v.x != mix32(base)) + (v.y != mix32(base + 1)) + (v.z != mix32(base + 2)) + (v.w != mix32(base + 3));
  }
  // wave64 reduction, one atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_xor(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(errors, (unsigned long long)bad);
}

}  // namespace amdprobe
