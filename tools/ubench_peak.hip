// On-box peak microbenchmarks for the rooflines in bench.py.
//
//   valu   int32 lane-op rate of the Hamming-match inner loop's instructions:
//          v_xor_b32 (VGPR ^ SGPR, the train word is wave-uniform) followed by an
//          accumulating v_bcnt_u32_b32, in NCH independent chains per lane, at
//          1, 2, 4 and 8 waves per SIMD. Exact instruction counts via inline asm.
//   mfma   v_mfma_i32_16x16x64_i8 back to back (independent accumulators),
//          1 and 2 waves per SIMD: the int8 matrix peak.
//   mfma_f4  v_mfma_scale_f32_16x16x128_f8f6f4 on e2m1 operands, likewise.
//   knn_f4_mix  k_knn2_f4's per-tile MFMA + top-2 instruction mix with the
//          operands in registers: the issue-bound ceiling of that kernel.
//   fp64   v_fma_f64 chains (the RANSAC ErrorFunction2 arithmetic).
//   hbm    streaming copy (dwordx4 loads and stores, 2 x 2 GiB) and a
//          read-only reduction over 4 GiB: achievable HBM bandwidth.
//
// Prints one JSON object per measurement on stdout.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// ---- int32 VALU: xor + accumulating popcount --------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed, int iters) {
  uint32_t q[NCH], acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    q[c] = seed * (threadIdx.x + 7u * c + 1u);
    acc[c] = 0;
  }
  const uint32_t t = seed ^ blockIdx.x;  // wave-uniform operand (SGPR)
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        uint32_t x;
        asm volatile("v_xor_b32 %0, %1, %2" : "=v"(x) : "s"(t + k), "v"(q[c]));
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(acc[c]) : "v"(x));
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- int8 MFMA ---------------------------------------------------------------
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_i8(int* out, int seed, int iters) {
  v4i a = {seed, seed + 1, seed + 2, (int)threadIdx.x};
  v4i b = {seed ^ 5, seed ^ 9, (int)threadIdx.x, seed};
  v4i acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = v4i{0, 0, 0, c};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[c], 0, 0, 0);
  }
  int s = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- FP4 (e2m1) scaled MFMA, and the kNN-2 inner-loop mix on it ----------------
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v4f_t __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_f4(float* out, int seed, int iters) {
  v8i_t a = {seed, seed + 1, seed + 2, (int)threadIdx.x, 0, 0, 0, 0};
  v8i_t b = {seed ^ 5, seed ^ 9, (int)threadIdx.x, seed, 0, 0, 0, 0};
  v4f_t acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = v4f_t{0.f, 0.f, 0.f, (float)c};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < NACC; ++c)
      acc[c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[c], 4, 4, 0, 127, 0, 127);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// k_knn2_f4's irreducible per-tile work with operands in registers (no LDS, no
// staging): 4 query tiles x 2 k-steps of FP4 MFMA from an accumulator start
// advanced by integer adds, then v_min_u32 + v_med3_u32 per key. 1024 (query,
// train) comparisons per wave per iteration.
__global__ __launch_bounds__(256) void k_knn_mix(uint32_t* out, int seed, int iters) {
  v8i_t a0 = {seed, seed + 1, seed + 2, (int)threadIdx.x, 0, 0, 0, 0};
  v8i_t a1 = {seed ^ 3, seed + 7, (int)threadIdx.x, seed, 0, 0, 0, 0};
  v8i_t b[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    b[q][0] = v8i_t{seed ^ q, seed ^ 9, (int)threadIdx.x + q, seed, 0, 0, 0, 0};
    b[q][1] = v8i_t{seed + q, seed ^ 11, (int)threadIdx.x, seed - q, 0, 0, 0, 0};
  }
  typedef int v4i_t __attribute__((ext_vector_type(4)));
  v4i_t cb = {0x43800000 + 4 * (int)(threadIdx.x & 15), 0x43800004, 0x43800008, 0x4380000c};
  uint32_t k0[4], k1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) k0[q] = k1[q] = 0x46000000u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) cb[j] += 64;
    const v4f_t C = __builtin_bit_cast(v4f_t, cb);
    v4f_t acc[4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[q] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(c ? a1 : a0, b[q][c], c ? acc[q] : C, 4, 4, 0,
                                                                   127, 0, 127);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xf = acc[q][e];
        const uint32_t x = __float_as_uint(xf);
        k1[q] = max(min(k0[q], k1[q]), min(max(k0[q], k1[q]), x));
        k0[q] = min(k0[q], x);
      }
  }
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s += k0[q] ^ k1[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- FP64 FMA ----------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void k_fp64(double* out, double seed, int iters) {
  double x[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) x[c] = seed + threadIdx.x + c;
  const double m = 0.999999, a = 1e-7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(m), "v"(a));
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- HBM ---------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = __builtin_nontemporal_load(&src[i]);
}

__global__ __launch_bounds__(256) void k_read(const v4u* __restrict__ src, uint32_t* out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t s = 0;
  for (; i < n; i += stride) {
    v4u v = __builtin_nontemporal_load(&src[i]);
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;  // keeps the loads live
}

__global__ void k_fill(v4u* p, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) p[i] = v4u{(uint32_t)i, (uint32_t)(i * 3), (uint32_t)(i ^ 0x55), 7u};
}

template <typename F>
static float time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

template <int NCH>
static void run_valu(int ncu, uint32_t* out) {
  const int iters = 4096;
  for (int wps : {1, 2, 4, 8}) {
    const int grid = ncu * wps;  // 256 threads = one wave per SIMD per workgroup
    float ms = time_ms([&] { k_valu<NCH><<<grid, 256>>>(out, 0x9E3779B9u, iters); }, 5);
    CHECK(hipGetLastError());
    const double ops = (double)grid * 256 * iters * 8 * NCH * 2;  // xor + bcnt
    printf("{\"bench\": \"valu_xor_bcnt\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, "
           "\"tops\": %.3f}\n", NCH, wps, ms, ops / (ms * 1e-3) / 1e12);
  }
}

template <int NACC>
static void run_mfma(int ncu, int* out) {
  const int iters = 2048;
  for (int wps : {1, 2}) {
    const int grid = ncu * wps;
    float ms = time_ms([&] { k_mfma_i8<NACC><<<grid, 256>>>(out, 3, iters); }, 5);
    CHECK(hipGetLastError());
    const double ops = (double)grid * 4 * iters * NACC * (16.0 * 16 * 64 * 2);
    printf("{\"bench\": \"mfma_i32_16x16x64_i8\", \"accumulators\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, "
           "\"tops\": %.2f}\n", NACC, wps, ms, ops / (ms * 1e-3) / 1e12);
  }
}

template <int NACC>
static void run_mfma_f4(int ncu, float* out) {
  const int iters = 2048;
  for (int wps : {1, 2}) {
    const int grid = ncu * wps;
    float ms = time_ms([&] { k_mfma_f4<NACC><<<grid, 256>>>(out, 3, iters); }, 5);
    CHECK(hipGetLastError());
    const double ops = (double)grid * 4 * iters * NACC * (16.0 * 16 * 128 * 2);
    printf("{\"bench\": \"mfma_scale_f32_16x16x128_f4\", \"accumulators\": %d, \"waves_per_simd\": %d, "
           "\"ms\": %.4f, \"tops\": %.2f}\n", NACC, wps, ms, ops / (ms * 1e-3) / 1e12);
  }
}

static void run_knn_mix(int ncu, uint32_t* out) {
  const int iters = 2048;
  for (int wps : {1, 2, 3}) {
    const int grid = ncu * wps;
    float ms = time_ms([&] { k_knn_mix<<<grid, 256>>>(out, 3, iters); }, 5);
    CHECK(hipGetLastError());
    const double cmp = (double)grid * 4 * iters * 1024;
    printf("{\"bench\": \"knn_f4_mix\", \"waves_per_simd\": %d, \"ms\": %.4f, \"gcmp_s\": %.1f, "
           "\"tops\": %.2f}\n", wps, ms, cmp / (ms * 1e-3) / 1e9, cmp * 512 / (ms * 1e-3) / 1e12);
  }
}

template <int NCH>
static void run_fp64(int ncu, double* out) {
  const int iters = 1024;
  for (int wps : {1, 2, 4}) {
    const int grid = ncu * wps;
    float ms = time_ms([&] { k_fp64<NCH><<<grid, 256>>>(out, 1.0, iters); }, 5);
    CHECK(hipGetLastError());
    const double flops = (double)grid * 256 * iters * 8 * NCH * 2;
    printf("{\"bench\": \"fp64_fma\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"tflops\": %.2f}\n",
           NCH, wps, ms, flops / (ms * 1e-3) / 1e12);
  }
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  int clk_khz = 0;
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  printf("{\"device\": \"%s\", \"gcn_arch\": \"%s\", \"cus\": %d, \"clock_mhz\": %d}\n", prop.name,
         prop.gcnArchName, ncu, clk_khz / 1000);
  fflush(stdout);

  uint32_t* out32;
  CHECK(hipMalloc(&out32, (size_t)ncu * 8 * 256 * 8));
  run_valu<1>(ncu, out32);
  run_valu<2>(ncu, out32);
  run_valu<4>(ncu, out32);
  run_valu<8>(ncu, out32);
  fflush(stdout);
  run_mfma<1>(ncu, (int*)out32);
  run_mfma<4>(ncu, (int*)out32);
  fflush(stdout);
  run_mfma_f4<1>(ncu, (float*)out32);
  run_mfma_f4<4>(ncu, (float*)out32);
  run_knn_mix(ncu, out32);
  fflush(stdout);
  run_fp64<1>(ncu, (double*)out32);
  run_fp64<4>(ncu, (double*)out32);
  fflush(stdout);

  const size_t bytes = (size_t)2 << 30;  // 2 GiB per buffer
  const size_t n = bytes / 16;
  v4u *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  k_fill<<<ncu * 8, 256>>>(a, n);
  k_fill<<<ncu * 8, 256>>>(b, n);
  CHECK(hipDeviceSynchronize());
  for (int wpc : {8, 16, 32}) {
    const int grid = ncu * wpc;
    float ms = time_ms([&] { k_copy<<<grid, 256>>>(a, b, n); }, 10);
    printf("{\"bench\": \"hbm_copy\", \"bytes_moved\": %zu, \"workgroups_per_cu\": %d, \"ms\": %.4f, "
           "\"gbs\": %.1f}\n", 2 * bytes, wpc, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    ms = time_ms([&] { k_read<<<grid, 256>>>(a, out32, n); }, 10);
    printf("{\"bench\": \"hbm_read\", \"bytes_moved\": %zu, \"workgroups_per_cu\": %d, \"ms\": %.4f, "
           "\"gbs\": %.1f}\n", bytes, wpc, ms, 1.0 * bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(out32));
  return 0;
}
