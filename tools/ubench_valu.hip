// ubench_valu.hip -- issue cost of the VALU instructions of the KJMA inner loop on gfx950.
//
// Each kernel runs REPS x 16 independent instances of one instruction (8 register sets,
// no dependence between consecutive instructions) per wave, with `waves` waves per SIMD.
// Printed: SIMD cycles per wave-instruction = elapsed_ns * clk_GHz * 4 SIMDs * CUs / (waves*instr),
// with the clock measured in-kernel (s_memtime / s_memrealtime) -- MI355X_MICROARCH.md item (6).
//
//   hipcc -O3 --offload-arch=gfx950 -o ubench_valu tools/ubench_valu.hip && ./ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REPS 2048

#define OP8(INSTR)                                                                       \
  asm volatile(INSTR : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INSTR : "+v"(a1) : "v"(b), "v"(c)); \
  asm volatile(INSTR : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INSTR : "+v"(a3) : "v"(b), "v"(c)); \
  asm volatile(INSTR : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INSTR : "+v"(a5) : "v"(b), "v"(c)); \
  asm volatile(INSTR : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INSTR : "+v"(a7) : "v"(b), "v"(c));

template <typename T>
__device__ __forceinline__ void sink(T a, T* out) {
  if ((double)a == 12345.678) out[threadIdx.x] = a;
}

#define KERNEL(NAME, TYPE, INSTR)                                                          \
  __global__ __launch_bounds__(256) void NAME(TYPE* out, long long* clk) {                 \
    TYPE a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
         a6 = a0 + 6, a7 = a0 + 7, b = (TYPE)1, c = (TYPE)2;                               \
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();   \
    for (int i = 0; i < REPS; ++i) { OP8(INSTR) OP8(INSTR) }                              \
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();   \
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }      \
    sink(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7, out);                                     \
  }

KERNEL(k_fma_f64, double, "v_fma_f64 %0, %1, %2, %0")
KERNEL(k_add_f64, double, "v_add_f64 %0, %0, %1")
KERNEL(k_mul_f64, double, "v_mul_f64 %0, %0, %1")
KERNEL(k_fract_f64, double, "v_fract_f64 %0, %0")
KERNEL(k_rndne_f64, double, "v_rndne_f64 %0, %0")
KERNEL(k_mov_b64, double, "v_mov_b64 %0, %1")
KERNEL(k_fma_f32, float, "v_fma_f32 %0, %1, %2, %0")
KERNEL(k_and_b32, int, "v_and_b32 %0, %0, %1")
KERNEL(k_ashr_i32, int, "v_ashrrev_i32 %0, 8, %0")
KERNEL(k_lshl_add_u32, int, "v_lshl_add_u32 %0, %0, 12, %1")
KERNEL(k_bfi_b32, int, "v_bfi_b32 %0, %1, %0, %2")
KERNEL(k_lshl_sdwa, int, "v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0")
KERNEL(k_add_u32, int, "v_add_u32 %0, %0, %1")

// v_ldexp_f64 (double, int) and v_cvt_i32_f64 (int <- double) need mixed operand types
__global__ __launch_bounds__(256) void k_ldexp_f64(double* out, long long* clk) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  int b = 1, c = 0;
  (void)c;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < REPS; ++i) {
#define L1(A) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(A) : "v"(b));
    L1(a0) L1(a1) L1(a2) L1(a3) L1(a4) L1(a5) L1(a6) L1(a7) L1(a0) L1(a1) L1(a2) L1(a3) L1(a4) L1(a5) L1(a6) L1(a7)
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
  sink(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7, out);
}

__global__ __launch_bounds__(256) void k_cvt_i32_f64(double* out, long long* clk) {
  double x = threadIdx.x * 0.5;
  int a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < REPS; ++i) {
#define C1(A) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(A) : "v"(x));
    C1(a0) C1(a1) C1(a2) C1(a3) C1(a4) C1(a5) C1(a6) C1(a7) C1(a0) C1(a1) C1(a2) C1(a3) C1(a4) C1(a5) C1(a6) C1(a7)
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
  sink((double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7), out);
}


// Mixed streams: NF independent v_fma_f64 + NI independent VOP2 integer ops per group of 8 slots.
template <int NF, int NI>
__global__ __launch_bounds__(256) void k_mix(double* out, long long* clk) {
  double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
  int i0 = threadIdx.x, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
  const double b = 1.0, c = 2.0;
  const int m = 0x3fff;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < REPS; ++i) {
#define F1(A) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(A) : "v"(b), "v"(c));
#define I1(A) asm volatile("v_and_b32 %0, %0, %1" : "+v"(A) : "v"(m));
    if (NF > 0) F1(d0) if (NI > 0) I1(i0) if (NF > 1) F1(d1) if (NF > 2) F1(d2) if (NI > 1) I1(i1)
    if (NF > 3) F1(d3) if (NF > 4) F1(d4) if (NI > 2) I1(i2) if (NF > 5) F1(d5) if (NF > 6) F1(d6)
    if (NI > 3) I1(i3) if (NF > 7) F1(d7)
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
  sink(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 + (double)(i0 + i1 + i2 + i3), out);
}

typedef void (*kfn)(void*, long long*);

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  void* out;
  long long* clk;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&clk, 16);
  struct { const char* name; const void* fn; } ks[] = {
      {"v_fma_f64", (const void*)k_fma_f64},       {"v_add_f64", (const void*)k_add_f64},
      {"v_mul_f64", (const void*)k_mul_f64},       {"v_fract_f64", (const void*)k_fract_f64},
      {"v_rndne_f64", (const void*)k_rndne_f64},   {"v_mov_b64", (const void*)k_mov_b64},
      {"v_ldexp_f64", (const void*)k_ldexp_f64},   {"v_cvt_i32_f64", (const void*)k_cvt_i32_f64},
      {"v_fma_f32", (const void*)k_fma_f32},       {"v_and_b32", (const void*)k_and_b32},
      {"v_ashrrev_i32", (const void*)k_ashr_i32},  {"v_lshl_add_u32", (const void*)k_lshl_add_u32},
      {"v_bfi_b32", (const void*)k_bfi_b32},       {"v_lshlrev_b32_sdwa", (const void*)k_lshl_sdwa},
      {"v_add_u32", (const void*)k_add_u32},
      {"mix_8f64_0i", (const void*)k_mix<8, 0>}, {"mix_8f64_3i", (const void*)k_mix<8, 3>},
      {"mix_8f64_4i", (const void*)k_mix<8, 4>}, {"mix_4f64_4i", (const void*)k_mix<4, 4>},
      {"mix_0f64_4i", (const void*)k_mix<0, 4>},
  };
  // instructions per REPS iteration for each kernel (16 for the single-instruction kernels)
  auto per_iter = [](const char* n) -> double {
    if (n[0] != 'm') return 16.0;
    int f = 0, i = 0;
    sscanf(n, "mix_%df64_%di", &f, &i);
    return (double)(f + i);
  };
  printf("{\"cus\": %d, \"results\": [\n", cus);
  const int wps_list[] = {1, 2, 4, 5};
  bool first = true;
  for (auto& k : ks) {
    for (int wps : wps_list) {
      const int blocks = cus * wps;  // 256 threads = 4 waves = one per SIMD; wps blocks per CU
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipLaunchKernelGGL((kfn)k.fn, dim3(blocks), dim3(256), 0, 0, out, clk);  // warm-up
      hipEventRecord(e0, 0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((kfn)k.fn, dim3(blocks), dim3(256), 0, 0, out, clk);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      long long c[2];
      hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
      const double ghz = (double)c[0] / ((double)c[1] * 10.0);  // memrealtime = 100 MHz
      const double instr = per_iter(k.name) * REPS;               // per wave
      // per-wave in-kernel cycles / (instructions * waves sharing the SIMD)
      const double cyc_inkernel = (double)c[0] / (instr * wps);
      const double cyc_wall = (ms / 5.0) * 1e6 * ghz / (instr * wps);
      printf("%s {\"instr\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_inkernel\": %.3f, "
             "\"cyc_per_instr_wall\": %.3f, \"ghz\": %.3f}",
             first ? "" : ",\n", k.name, wps, cyc_inkernel, cyc_wall, ghz);
      first = false;
      hipEventDestroy(e0);
      hipEventDestroy(e1);
    }
  }
  printf("\n]}\n");
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { fprintf(stderr, "hip error %s\n", hipGetErrorString(e)); return 1; }
  return 0;
}
