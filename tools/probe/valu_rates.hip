// Development probe: issue throughput of single VALU instructions on gfx950,
// full occupancy (8 waves per SIMD), 8 independent chains per lane.
// Prints ns per wave-instruction per SIMD and the ratio to v_add_u32.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 2048
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define OP2(NAME, ASM)                                                                   \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t seed) {        \
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed + 17;                   \
    for (int i = 0; i < ITERS; ++i) {                                                    \
      asm volatile(ASM " %0, %0, %1" : "+v"(a0) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a1) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a2) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a3) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a4) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a5) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a6) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a7) : "v"(b));                               \
    }                                                                                    \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
  }
#define OP3(NAME, ASM)                                                                   \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t seed) {        \
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, \
             a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed + 17, c = seed + 5;      \
    for (int i = 0; i < ITERS; ++i) {                                                    \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a4) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a5) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a6) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a7) : "v"(b), "v"(c));                   \
    }                                                                                    \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
  }

OP2(add_u32, "v_add_u32")
OP2(and_b32, "v_and_b32")
OP2(lshlrev_b32, "v_lshlrev_b32")
OP2(pk_add_f16, "v_pk_add_f16")
OP2(pk_min_f16, "v_pk_min_f16")
OP2(pk_max_f16, "v_pk_max_f16")
OP2(pk_sub_i16, "v_pk_sub_i16")
OP2(pk_add_u16, "v_pk_add_u16")
OP2(pk_min_u16, "v_pk_min_u16")
OP2(add_f32, "v_add_f32")
OP2(mul_f32, "v_mul_f32")
OP2(max_f16, "v_max_f16")
OP2(mul_u32_u24, "v_mul_u32_u24")
OP2(mul_lo_u32, "v_mul_lo_u32")
OP2(bcnt, "v_bcnt_u32_b32")
OP3(alignbyte, "v_alignbyte_b32")
OP3(perm, "v_perm_b32")
OP3(bfe_u32, "v_bfe_u32")
OP3(and_or, "v_and_or_b32")
OP3(add3_u32, "v_add3_u32")
OP3(fma_f32, "v_fma_f32")
OP3(pk_fma_f16, "v_pk_fma_f16")
OP3(pk_minimum3_f16, "v_pk_minimum3_f16")
OP3(pk_maximum3_f16, "v_pk_maximum3_f16")
OP3(dot4_u32_u8, "v_dot4_u32_u8")
OP3(dot2_u32_u16, "v_dot2_u32_u16")
OP3(max3_u32, "v_max3_u32")
OP3(med3_i32, "v_med3_i32")
OP3(mad_u32_u24, "v_mad_u32_u24")

OP2(sub_u32, "v_sub_u32")
OP2(or_b32, "v_or_b32")
OP2(xor_b32, "v_xor_b32")
OP2(max_u32, "v_max_u32")
OP2(min_i32, "v_min_i32")
OP2(lshrrev_b32, "v_lshrrev_b32")
OP2(max_f32, "v_max_f32")
OP2(sub_f32, "v_sub_f32")
OP2(add_f16, "v_add_f16")
OP2(min_f16, "v_min_f16")
OP2(mul_f16, "v_mul_f16")
OP2(max_u16, "v_max_u16")
OP2(add_u16, "v_add_u16")
OP2(pk_mul_f16, "v_pk_mul_f16")
OP2(fmac_f32, "v_fmac_f32")
OP2(dot2c_f32_f16, "v_dot2c_f32_f16")
OP2(dot4c_i32_i8, "v_dot4c_i32_i8")
OP2(pk_fmac_f16, "v_pk_fmac_f16")
OP2(mul_hi_u32, "v_mul_hi_u32")
OP2(ldexp_f32, "v_ldexp_f32")
OP2(subrev_u32, "v_subrev_u32")
OP3(sad_u8, "v_sad_u8")
OP3(msad_u8, "v_msad_u8")
OP3(min3_f16, "v_min3_f16")
OP3(max3_f32, "v_max3_f32")
OP3(fma_f16, "v_fma_f16")
OP3(lshl_add_u32, "v_lshl_add_u32")
OP3(lshl_or_b32, "v_lshl_or_b32")
OP3(or3_b32, "v_or3_b32")
OP3(xad_u32, "v_xad_u32")
OP3(mad_u16, "v_mad_u16")
OP3(med3_f16, "v_med3_f16")
OP3(min3_i32, "v_min3_i32")

#define OP2D(NAME, ASM)                                                                  \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t seed) {        \
    double a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, b = seed + 17; \
    for (int i = 0; i < ITERS; ++i) {                                                    \
      asm volatile(ASM " %0, %0, %1" : "+v"(a0) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a1) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a2) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a3) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a0) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a1) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a2) : "v"(b));                               \
      asm volatile(ASM " %0, %0, %1" : "+v"(a3) : "v"(b));                               \
    }                                                                                    \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3);                 \
  }
OP2D(add_f64, "v_add_f64")
OP2D(mul_f64, "v_mul_f64")
#define OP3D(NAME, ASM)                                                                  \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t seed) {        \
    double a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, b = seed + 17, c = 3; \
    for (int i = 0; i < ITERS; ++i) {                                                    \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));                   \
      asm volatile(ASM " %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));                   \
    }                                                                                    \
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3);                 \
  }
OP3D(fma_f64, "v_fma_f64")

typedef void (*KFn)(uint32_t*, uint32_t);
struct Entry { const char* name; KFn fn; };

int main() {
  Entry es[] = {
      {"v_add_u32", k_add_u32}, {"v_add_f64", k_add_f64}, {"v_mul_f64", k_mul_f64}, {"v_fma_f64", k_fma_f64}, {"v_and_b32", k_and_b32}, {"v_lshlrev_b32", k_lshlrev_b32},
      {"v_pk_add_f16", k_pk_add_f16}, {"v_pk_min_f16", k_pk_min_f16},
      {"v_pk_max_f16", k_pk_max_f16}, {"v_pk_sub_i16", k_pk_sub_i16},
      {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_min_u16", k_pk_min_u16}, {"v_add_f32", k_add_f32},
      {"v_mul_f32", k_mul_f32}, {"v_max_f16", k_max_f16}, {"v_mul_u32_u24", k_mul_u32_u24},
      {"v_mul_lo_u32", k_mul_lo_u32}, {"v_bcnt_u32_b32", k_bcnt}, {"v_alignbyte_b32", k_alignbyte}, {"v_perm_b32", k_perm},
      {"v_bfe_u32", k_bfe_u32}, {"v_and_or_b32", k_and_or}, {"v_add3_u32", k_add3_u32},
      {"v_fma_f32", k_fma_f32}, {"v_pk_fma_f16", k_pk_fma_f16},
      {"v_pk_minimum3_f16", k_pk_minimum3_f16}, {"v_pk_maximum3_f16", k_pk_maximum3_f16},
      {"v_dot4_u32_u8", k_dot4_u32_u8}, {"v_dot2_u32_u16", k_dot2_u32_u16},
      {"v_max3_u32", k_max3_u32}, {"v_med3_i32", k_med3_i32}, {"v_mad_u32_u24", k_mad_u32_u24},
      {"v_sub_u32", k_sub_u32},
      {"v_or_b32", k_or_b32},
      {"v_xor_b32", k_xor_b32},
      {"v_max_u32", k_max_u32},
      {"v_min_i32", k_min_i32},
      {"v_lshrrev_b32", k_lshrrev_b32},
      {"v_max_f32", k_max_f32},
      {"v_sub_f32", k_sub_f32},
      {"v_add_f16", k_add_f16},
      {"v_min_f16", k_min_f16},
      {"v_mul_f16", k_mul_f16},
      {"v_max_u16", k_max_u16},
      {"v_add_u16", k_add_u16},
      {"v_pk_mul_f16", k_pk_mul_f16},
      {"v_fmac_f32", k_fmac_f32},
      {"v_dot2c_f32_f16", k_dot2c_f32_f16},
      {"v_dot4c_i32_i8", k_dot4c_i32_i8},
      {"v_pk_fmac_f16", k_pk_fmac_f16},
      {"v_mul_hi_u32", k_mul_hi_u32},
      {"v_ldexp_f32", k_ldexp_f32},
      {"v_subrev_u32", k_subrev_u32},
      {"v_sad_u8", k_sad_u8},
      {"v_msad_u8", k_msad_u8},
      {"v_min3_f16", k_min3_f16},
      {"v_max3_f32", k_max3_f32},
      {"v_fma_f16", k_fma_f16},
      {"v_lshl_add_u32", k_lshl_add_u32},
      {"v_lshl_or_b32", k_lshl_or_b32},
      {"v_or3_b32", k_or3_b32},
      {"v_xad_u32", k_xad_u32},
      {"v_mad_u16", k_mad_u16},
      {"v_med3_f16", k_med3_f16},
      {"v_min3_i32", k_min3_i32},
  };
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  double base = 0;
  printf("CUs %d, clock %d kHz\n", cus, prop.clockRate);
  for (const Entry& e : es) {
    hipLaunchKernelGGL(e.fn, dim3(blocks), dim3(256), 0, 0, out, 1u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(e.fn, dim3(blocks), dim3(256), 0, 0, out, 1u);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double waveInstr = 5.0 * blocks * 4 * ITERS * 8;
    const double simds = cus * 4.0;
    const double ns = ms * 1e6 / (waveInstr / simds);  // ns per wave-instruction per SIMD
    if (base == 0) base = ns;
    printf("%-20s %7.3f ns/wave-instr/SIMD  x%.2f of v_add_u32\n", e.name, ns, ns / base);
  }
  return 0;
}
