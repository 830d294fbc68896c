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

// Grouped tile order: consecutive tile ids walk GM-row bands column by column, so the ~32 tiles
// one XCD has in flight form a GM x (32/GM) block that shares GM A-panels and 32/GM B-panels in
// that XCD's L2 instead of 1 A-panel and 32 B-panels (row-major order). Bijective; the last band
// may be shorter than GM.
__device__ __forceinline__ void grouped_tile(int tile, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int band = tile / (gm * tiles_n);
  const int first = band * gm;
  const int rows = min(gm, tiles_m - first);
  const int in = tile - band * gm * tiles_n;
  tm = first + in % rows;
  tn = in / rows;
}

__global__ __launch_bounds__(GEMM_THREADS, 2)
void gemm_bf16_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                         float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 2 * TILE_ELEMS];  // [buf][A|B][row][k]
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  int tm, tn;
  grouped_tile(xcd_remap(blockIdx.x, nwg), M / BM, tiles_n, 8, tm, tn);
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
// bf16 GEMM, 256x256 block tile, LDS-DMA staged 8-phase pipeline (the fast path).
//
// 512 threads = 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns a 128x64 output: rows
// {wr*64 + [0,64)} u {128 + wr*64 + [0,64)}, cols {wc*32 + [0,32)} u {128 + wc*32 + [0,32)},
// i.e. 8 x 4 MFMA 16x16 tiles (128 accumulator VGPRs). Interleaving the two halves means every
// wave's first A/B fragments sit in the "lo" half-tiles: a K-tile (256x64 of A and of B) is
// staged as four 16 KiB half-tiles in consumption order
//     h0 = A rows 0-127, h1 = B rows 0-127, h2 = B rows 128-255, h3 = A rows 128-255
// and read in four phases per K-tile, one C quadrant (4m x 2n tiles x K=64 = 16 MFMA) each:
//     ph0: A[m0-3] + B[n0-1] -> MFMA   ph1: B[n2-3] -> MFMA   ph2: A[m4-7] -> MFMA   ph3: MFMA
// (B[n0-1] stays in registers for ph3). Two K-tiles per loop iteration (8 phases, two LDS
// buffers of 64 KiB). Every phase issues ONE half-tile of global_load_lds_dwordx4 (2 per
// thread) six half-tiles ahead; the LDS-DMA stays in flight across the raw s_barriers and is
// retired by counted `s_waitcnt vmcnt(8)` (never 0 in steady state) one phase before it is read.
// The two wave groups (wr = 0/1, one wave of each per SIMD) run one barrier apart, so LDS reads
// of one group overlap MFMA of the other; restaging therefore waits >= 2 phases after a buffer's
// last read (see the schedule comment in the kernel).
//
// LDS image: 128 B rows, 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7). LDS-DMA writes
// lane-linearly, so the permutation is applied to the per-lane global SOURCE address and undone
// on the ds_read address; for the 16x16x32 fragment reads this is conflict-free in all four
// ds_read_b128 lane groups.
// ---------------------------------------------------------------------------------------
namespace big {
constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512;
constexpr int HALF_BYTES = 128 * BK * 2;       // 16 KiB
constexpr int TILE_BYTES = 4 * HALF_BYTES;     // one K-tile (A and B)
constexpr int LDS_BYTES = 2 * TILE_BYTES;      // 128 KiB, double buffered
}  // namespace big

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* gsrc, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)gsrc, (lds_void*)lds_wave_base, 16, 0, 0);
}

__global__ __launch_bounds__(big::THREADS, 1)
void gemm_bf16_nt_256_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                             float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = big::BM, BN = big::BN, BK = big::BK;
  constexpr int HALF_BYTES = big::HALF_BYTES, TILE_BYTES = big::TILE_BYTES, LDS_BYTES = big::LDS_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  int tm, tn;
  grouped_tile(xcd_remap(blockIdx.x, nwg), M / BM, tiles_n, 8, tm, tn);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  const __bf16* Ablk = A + (size_t)tm * BM * K;
  const __bf16* Bblk = Bt + (size_t)tn * BN * K;
  // staging: this lane's two 16-B pieces of a half-tile (loop invariant element offsets)
  size_t soff[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = q * 512 + wave * 64 + lane;      // 16-B slot in the half-tile image
    const int row = p >> 3, chunk = (p & 7) ^ ((row >> 1) & 7);
    soff[q] = (size_t)row * K + chunk * 8;
  }
  const __bf16* hsrc[4] = {Ablk, Bblk, Bblk + (size_t)128 * K, Ablk + (size_t)128 * K};
  char* const wave_dst = smem + wave * 1024;
  auto stage = [&](int t, int h) {
    const __bf16* src = hsrc[h] + (size_t)t * BK;
    char* dst = wave_dst + (t & 1) * TILE_BYTES + h * HALF_BYTES;
    glds16(src + soff[0], dst);
    glds16(src + soff[1], dst + 8192);
  };
  // fragment reads: row (lane & 15) of a 16-row group, logical chunk ks*4 + (lane >> 4)
  const int sw = (lane >> 1) & 7;
  const int cb0 = (((lane >> 4)) ^ sw) << 4, cb1 = ((4 + (lane >> 4)) ^ sw) << 4;
  const int rA = (wr * 64 + (lane & 15)) * 128;   // within an A half-tile
  const int rB = (wc * 32 + (lane & 15)) * 128;   // within a B half-tile

  floatx4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0[2][2], b1[2][2];

  // Staging stream: half-tile s = 4*t + h (h: 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi) is issued in phase
  // g = s - 6 (global phase g = 4*t + q reads K-tile t's quadrant q). A half-tile is first/last
  // read in one phase (A-lo, B-lo at q=0, B-hi at q=1, A-hi at q=2), so every restage lands >= 2
  // phases after the previous occupant's read (the staggered-groups WAR rule) and every read
  // comes >= 5 phases after its issue. Counted waits (before the phase's first barrier) retire
  // what the NEXT phase reads: q=0 -> B-hi(t), q=1 -> A-hi(t), q=3 -> A-lo/B-lo(t+1); steady
  // state keeps 4 half-tiles (8 DMA per thread) in flight.
  const int nt = K / BK, niter = nt / 2;
  // prologue: half-tiles 0..5, then retire 0 and 1 (K-tile 0's q=0 operands)
#pragma unroll
  for (int s = 0; s < 6; ++s) stage(s >> 2, s & 3);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  // wave-group stagger: group wr == 1 runs one barrier behind group 0 for the whole loop, so on
  // every SIMD (waves w and w + 4) one wave reads LDS while the other issues MFMA.
  const bool late = __builtin_amdgcn_readfirstlane(wr) == 1;
  if (late) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_s_barrier();

#define READ_A(T, H)                                                                         \
  _Pragma("unroll") for (int mm = 0; mm < 4; ++mm) {                                         \
    const char* base = smem + (T) * TILE_BYTES + (H) * HALF_BYTES + rA + mm * 16 * 128;      \
    af[mm][0] = *reinterpret_cast<const bf16x8*>(base + cb0);                                \
    af[mm][1] = *reinterpret_cast<const bf16x8*>(base + cb1);                                \
  }
#define READ_B(DST, T, H)                                                                    \
  _Pragma("unroll") for (int nn = 0; nn < 2; ++nn) {                                         \
    const char* base = smem + (T) * TILE_BYTES + (H) * HALF_BYTES + rB + nn * 16 * 128;      \
    DST[nn][0] = *reinterpret_cast<const bf16x8*>(base + cb0);                               \
    DST[nn][1] = *reinterpret_cast<const bf16x8*>(base + cb1);                               \
  }
#define MFMA_Q(MB, NB, BREG)                                                                 \
  __builtin_amdgcn_s_setprio(1);                                                             \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                           \
  _Pragma("unroll") for (int mm = 0; mm < 4; ++mm)                                           \
  _Pragma("unroll") for (int nn = 0; nn < 2; ++nn)                                           \
    acc[(MB) + mm][(NB) + nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                     \
        af[mm][ks], BREG[nn][ks], acc[(MB) + mm][(NB) + nn], 0, 0, 0);                       \
  __builtin_amdgcn_s_setprio(0);
#define SYNC_MFMA(MB, NB, BREG)                                                              \
  __builtin_amdgcn_s_barrier();                                                              \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                         \
  MFMA_Q(MB, NB, BREG)                                                                       \
  __builtin_amdgcn_s_barrier();
#define WAITV(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory");

  for (int it = 0; it < niter; ++it) {
    const bool last = it == niter - 1;   // K-tiles nt-2 (even) and nt-1 (odd)
    const int t0 = 2 * it;
    // ---- K-tile t0, buffer 0 ----  (q=0..3 issue s = 4*t0 + 6 .. 4*t0 + 9)
    READ_A(0, 0) READ_B(b0, 0, 1)
    stage(t0 + 1, 2);
    WAITV(8)                                                      // B-hi(t0)
    SYNC_MFMA(0, 0, b0)
    READ_B(b1, 0, 2)
    stage(t0 + 1, 3);
    WAITV(8)                                                      // A-hi(t0)
    SYNC_MFMA(0, 2, b1)
    READ_A(0, 3)
    if (!last) stage(t0 + 2, 0);
    SYNC_MFMA(4, 2, b1)
    if (!last) {
      stage(t0 + 2, 1);
      WAITV(8)                                                    // A-lo, B-lo(t0 + 1)
    } else {
      WAITV(4)
    }
    SYNC_MFMA(4, 0, b0)
    // ---- K-tile t0 + 1, buffer 1 ----
    READ_A(1, 0) READ_B(b0, 1, 1)
    if (!last) {
      stage(t0 + 2, 2);
      WAITV(8)
    } else {
      WAITV(2)
    }
    SYNC_MFMA(0, 0, b0)
    READ_B(b1, 1, 2)
    if (!last) {
      stage(t0 + 2, 3);
      WAITV(8)
    } else {
      WAITV(0)
    }
    SYNC_MFMA(0, 2, b1)
    READ_A(1, 3)
    if (!last) stage(t0 + 3, 0);
    SYNC_MFMA(4, 2, b1)
    if (!last) {
      stage(t0 + 3, 1);
      WAITV(8)                                                    // A-lo, B-lo(t0 + 2)
    }
    SYNC_MFMA(4, 0, b0)
  }
  if (!late) __builtin_amdgcn_s_barrier();   // balance the stagger barrier
#undef READ_A
#undef READ_B
#undef MFMA_Q
#undef SYNC_MFMA
#undef WAITV

  // epilogue: acc[m][n] element j -> row (lane >> 4) * 4 + j, col lane & 15 of its 16x16 tile
  float* Cblk = C + (size_t)tm * BM * N + (size_t)tn * BN;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int row0 = (m < 4 ? 0 : 128) + wr * 64 + (m & 3) * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = (n < 2 ? 0 : 128) + wc * 32 + (n & 1) * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) Cblk[(size_t)(row0 + j) * N + col] = acc[m][n][j];
    }
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
// HBM streaming copy: each block owns one contiguous span (DRAM-page friendly), 4 x 16 B
// nontemporal loads in flight per lane, then 4 nontemporal stores. Measured on MI355X with
// scripts/hbm_sweep.hip: 5.6-5.8 TB/s (read + write) vs 4.5 TB/s for a grid-strided loop;
// read-only and write-only roofs are ~5.4 TB/s each (profiles/hbm_sweep_r01.jsonl).
// ---------------------------------------------------------------------------------------
constexpr int HBM_COPY_BLOCKS = 4096;
__global__ __launch_bounds__(256)
void hbm_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  const size_t per = ((n16 + gridDim.x - 1) / gridDim.x + 1023) & ~size_t(1023);
  const size_t begin = (size_t)blockIdx.x * per;
  const size_t end = begin + per < n16 ? begin + per : n16;
  size_t i = begin + threadIdx.x;
  for (; i + 768 < end; i += 1024) {
    u32x4 v0 = __builtin_nontemporal_load(s + i), v1 = __builtin_nontemporal_load(s + i + 256);
    u32x4 v2 = __builtin_nontemporal_load(s + i + 512), v3 = __builtin_nontemporal_load(s + i + 768);
    __builtin_nontemporal_store(v0, d + i);
    __builtin_nontemporal_store(v1, d + i + 256);
    __builtin_nontemporal_store(v2, d + i + 512);
    __builtin_nontemporal_store(v3, d + i + 768);
  }
  for (; i < end; i += 256) d[i] = s[i];
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

// Finite bf16 operands with random sign/mantissa bits and |x| in [0.5, 1) (benchmark fill).
__global__ __launch_bounds__(256)
void bf16_fill_kernel(uint4* __restrict__ p, size_t n16, uint32_t seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint64_t base = (i << 2) ^ ((uint64_t)seed << 40);
    uint4 v = make_uint4(mix32(base), mix32(base + 1), mix32(base + 2), mix32(base + 3));
    v.x = (v.x & 0x807F807Fu) | 0x3F003F00u;
    v.y = (v.y & 0x807F807Fu) | 0x3F003F00u;
    v.z = (v.z & 0x807F807Fu) | 0x3F003F00u;
    v.w = (v.w & 0x807F807Fu) | 0x3F003F00u;
    p[i] = v;
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

// ---------------------------------------------------------------------------------------
// Fused readiness check. A pod's readiness probe is on the deploy / recovery critical path, so
// it runs as ONE host call: five launches back to back on a private stream and a single 32-byte
// read-back, instead of a chain of framework ops with a host sync in the middle.
//   readiness_prep_kernel  A, Bt <- hashed bf16 operands, result <- 0
//   gemm (MFMA)            C = A Bt^T
//   gemm_check_kernel      every element of C against an fp32 VALU reference (v_dot2_f32_bf16)
//   pattern_write/check    address-hashed write + verify over a 64 MiB buffer
// ---------------------------------------------------------------------------------------
struct ReadinessResult {
  float diff2;                  // sum over (m, n) of (C - A Bt^T)^2, reference in fp32
  float ref2;                   // sum over (m, n) of (A Bt^T)^2
  unsigned long long bad_words;
  unsigned long long reserved;
};

__global__ __launch_bounds__(256)
void readiness_prep_kernel(uint4* __restrict__ ab, size_t ab16, uint32_t seed, ReadinessResult* __restrict__ res) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < ab16; i += stride) {
    const uint64_t base = (i << 2) ^ ((uint64_t)seed << 40);
    uint4 v = make_uint4(mix32(base), mix32(base + 1), mix32(base + 2), mix32(base + 3));
    // finite bf16 pairs: random sign and mantissa, |x| in [0.5, 1)
    v.x = (v.x & 0x807F807Fu) | 0x3F003F00u;
    v.y = (v.y & 0x807F807Fu) | 0x3F003F00u;
    v.z = (v.z & 0x807F807Fu) | 0x3F003F00u;
    v.w = (v.w & 0x807F807Fu) | 0x3F003F00u;
    ab[i] = v;
  }
  if (tid == 0) {
    res->diff2 = 0.f;
    res->ref2 = 0.f;
    res->bad_words = 0ull;
    res->reserved = 0ull;
  }
}

// Dense check of C = A Bt^T: one workgroup per 16 x 16 output tile (M / 16 * N / 16 of them, so
// a 256 x 256 product spreads over 256 CUs). The tile's 16 A rows and 16 Bt rows are staged in
// LDS (rows padded by 16 B: the 16 Bt rows a wave reads at one k land on disjoint bank groups),
// each thread forms its element's fp32 reference with v_dot2_f32_bf16 (two accumulators), and
// the workgroup adds its sum of squared differences and of squared references to out2 with two
// float atomics (out2 must arrive zeroed; the prep kernel zeroes it). Needs M, N % 16 == 0,
// K % 8 == 0, K <= CHECK_MAX_K (host-checked). `inject` = 1 reads C[0:16][0:16] as zeros, a
// lost MFMA tile (tests that the check catches it).
constexpr int CHECK_TILE = 16;
constexpr int CHECK_THREADS = CHECK_TILE * CHECK_TILE;
constexpr int CHECK_MAX_K = 1024;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(CHECK_THREADS)
void gemm_check_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, const float* __restrict__ C,
                       int M, int N, int K, int inject, float* __restrict__ out2) {
  __shared__ __attribute__((aligned(16))) __bf16 la[CHECK_TILE * (CHECK_MAX_K + 8)];
  __shared__ __attribute__((aligned(16))) __bf16 lb[CHECK_TILE * (CHECK_MAX_K + 8)];
  __shared__ float red[2][CHECK_THREADS / 64];
  const int tiles_n = N / CHECK_TILE;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = K + 8;                       // LDS row stride (bf16)
  const int kchunks = K / 8;
  for (int i = tid; i < CHECK_TILE * kchunks; i += CHECK_THREADS) {
    const int r = i / kchunks, kc = i - r * kchunks;
    *reinterpret_cast<uint4*>(la + r * row + kc * 8) =
        *reinterpret_cast<const uint4*>(A + (size_t)(tm * CHECK_TILE + r) * K + kc * 8);
    *reinterpret_cast<uint4*>(lb + r * row + kc * 8) =
        *reinterpret_cast<const uint4*>(Bt + (size_t)(tn * CHECK_TILE + r) * K + kc * 8);
  }
  __syncthreads();
  const int r = tid >> 4, c = tid & 15;
  const __bf16* pa = la + r * row;
  const __bf16* pb = lb + c * row;
  float acc0 = 0.f, acc1 = 0.f;
  for (int kc = 0; kc < kchunks; ++kc) {
    const bf16x8 a8 = *reinterpret_cast<const bf16x8*>(pa + kc * 8);
    const bf16x8 b8 = *reinterpret_cast<const bf16x8*>(pb + kc * 8);
    acc0 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a8[0], a8[1]}, bf16x2{b8[0], b8[1]}, acc0, false);
    acc1 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a8[2], a8[3]}, bf16x2{b8[2], b8[3]}, acc1, false);
    acc0 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a8[4], a8[5]}, bf16x2{b8[4], b8[5]}, acc0, false);
    acc1 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a8[6], a8[7]}, bf16x2{b8[6], b8[7]}, acc1, false);
  }
  const float ref = acc0 + acc1;
  const int m = tm * CHECK_TILE + r, n = tn * CHECK_TILE + c;
  float cv = C[(size_t)m * N + n];
  if (inject == 1 && m < 16 && n < 16) cv = 0.f;   // a lost 16x16 tile
  const float d = cv - ref;
  float d2 = d * d, w2 = ref * ref;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    d2 += __shfl_xor(d2, off, 64);
    w2 += __shfl_xor(w2, off, 64);
  }
  if (lane == 0) {
    red[0][wave] = d2;
    red[1][wave] = w2;
  }
  __syncthreads();
  if (tid == 0) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < CHECK_THREADS / 64; ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    atomicAdd(&out2[0], a);
    atomicAdd(&out2[1], b);
  }
}

}  // namespace amdprobe
