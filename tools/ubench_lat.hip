// ubench_lat.hip -- dependent-chain latency of the instructions in the ODE step (gfx950), one
// wavefront alone on its SIMD: what a single-point integration (the CLI's case) waits on.
//
// Each kernel runs one wave of 64 lanes over REPS x 16 instructions; CHAINS independent chains
// are interleaved (1: every instruction waits for the previous one; 4: four in flight).  Printed:
// s_memtime cycles per instruction (the shader clock counter).
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ubench_lat tools/ubench_lat.hip && /tmp/ubench_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REPS 512

template <typename T>
__device__ __forceinline__ void sink(T a, T* out) {
  if ((double)a == 12345.678) out[threadIdx.x] = a;
}

#define BODY16(STMT) STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT STMT

#define CHAIN_KERNEL(NAME, TYPE, INSTR, CH)                                                   \
  __global__ __launch_bounds__(64) void NAME(TYPE* out, long long* clk) {                     \
    TYPE a[4] = {(TYPE)threadIdx.x, (TYPE)1, (TYPE)2, (TYPE)3};                               \
    TYPE b = (TYPE)1, c = (TYPE)0;                                                            \
    long long t0 = __builtin_amdgcn_s_memtime();                                              \
    for (int i = 0; i < REPS; ++i) {                                                          \
      BODY16(_Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(INSTR : "+v"(a[k]) : "v"(b), "v"(c));) \
    }                                                                                         \
    long long t1 = __builtin_amdgcn_s_memtime();                                              \
    if (threadIdx.x == 0) clk[0] = t1 - t0;                                                   \
    sink(a[0] + a[1] + a[2] + a[3], out);                                                     \
  }

CHAIN_KERNEL(fma64_1, double, "v_fma_f64 %0, %0, %1, %2", 1)
CHAIN_KERNEL(fma64_2, double, "v_fma_f64 %0, %0, %1, %2", 2)
CHAIN_KERNEL(fma64_4, double, "v_fma_f64 %0, %0, %1, %2", 4)
CHAIN_KERNEL(add64_1, double, "v_add_f64 %0, %0, %1", 1)
CHAIN_KERNEL(max64_1, double, "v_max_f64 %0, %0, %1", 1)
CHAIN_KERNEL(rcp64_1, double, "v_rcp_f64 %0, %0", 1)
CHAIN_KERNEL(fma32_1, float, "v_fma_f32 %0, %0, %1, %2", 1)
CHAIN_KERNEL(add32_1, int, "v_add_u32 %0, %0, %1", 1)
CHAIN_KERNEL(cnd32_1, int, "v_cndmask_b32 %0, %0, %1, vcc", 1)
CHAIN_KERNEL(dpp32_1, int, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", 1)
CHAIN_KERNEL(dpp32_4, int, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", 4)

// dependent LDS reads (pointer chase through a 64-entry table)
__global__ __launch_bounds__(64) void lds_chase(int* out, long long* clk) {
  __shared__ int tab[64];
  tab[threadIdx.x] = (threadIdx.x + 1) & 63;
  __syncthreads();
  int p = threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < REPS * 16; ++i) {
    asm volatile("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(p) : : "memory");
    p <<= 2;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[0] = t1 - t0;
  sink(p, out);
}

int main() {
  void* out;
  long long* clk;
  hipMalloc(&out, 64 * 8);
  hipMallocManaged(&clk, 8);
#define RUN(NAME, TYPE, CH)                                                                       \
  for (int w = 0; w < 3; ++w) {                                                                   \
    hipLaunchKernelGGL(NAME, dim3(1), dim3(64), 0, 0, (TYPE*)out, clk);                           \
    hipDeviceSynchronize();                                                                       \
  }                                                                                               \
  printf("{\"instr\": \"%s\", \"chains\": %d, \"cycles_per_instr\": %.2f}\n", #NAME, CH,          \
         (double)clk[0] / (REPS * 16.0 * CH));
  RUN(fma64_1, double, 1)
  RUN(fma64_2, double, 2)
  RUN(fma64_4, double, 4)
  RUN(add64_1, double, 1)
  RUN(max64_1, double, 1)
  RUN(rcp64_1, double, 1)
  RUN(fma32_1, float, 1)
  RUN(add32_1, int, 1)
  RUN(cnd32_1, int, 1)
  RUN(dpp32_1, int, 1)
  RUN(dpp32_4, int, 4)
  RUN(lds_chase, int, 1)
  return 0;
}
