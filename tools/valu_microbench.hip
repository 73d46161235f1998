// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction per SIMD for the instruction
// kinds the traversal loop uses, with 8 waves per SIMD and 8 independent dependency chains per wave.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o build/valu_microbench && build/valu_microbench
// Output: ns per instruction per SIMD and cycles at the measured clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(X) X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, int iters, unsigned long long* clk) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float b = 1.0001f + out[0], c = 0.5f + out[1];
    const float2 bb = make_float2(b, c), cc = make_float2(c, b);
    float2 p0 = make_float2(a0, a1), p1 = make_float2(a2, a3), p2 = make_float2(a4, a5), p3 = make_float2(a6, a7);
    (void)p0; (void)p1; (void)p2; (void)p3;
    if constexpr (OP == 18) asm volatile("s_mov_b64 s[40:41], -1" ::: "s40", "s41");
    if constexpr (OP == 34) asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#define STEP(x)                                                                                                  \
    if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                   \
    if constexpr (OP == 1) asm volatile("v_max_f32 %0, %1, %0" : "+v"(x) : "v"(b));                              \
    if constexpr (OP == 2) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                  \
    if constexpr (OP == 3) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(x) : "v"(b));                     \
    if constexpr (OP == 4) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x) : "v"(b));                           \
    if constexpr (OP == 6) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x) : "v"(b));                          \
    if constexpr (OP == 7) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(x), "v"(b) : "vcc");                   \
    if constexpr (OP == 8) asm volatile("v_lshl_add_u32 %0, %1, 2, %0" : "+v"(x) : "v"(b));                       \
    if constexpr (OP == 9) asm volatile("v_bfe_i32 %0, %1, 0, 16" : "+v"(x) : "v"(b));                           \
    if constexpr (OP == 10) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 11) asm volatile("v_cmp_lt_f32 s[40:41], %0, %1" : : "v"(x), "v"(b) : "s40", "s41");      \
    if constexpr (OP == 12) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x));                                         \
    if constexpr (OP == 13) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));                                          \
    if constexpr (OP == 14) asm volatile("v_div_fmas_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));             \
    if constexpr (OP == 15) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 16) asm volatile("v_min_f32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 17) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 18) asm volatile("v_cndmask_b32_e64 %0, %1, %0, s[40:41]" : "+v"(x) : "v"(b) : "s40", "s41"); \
    if constexpr (OP == 19) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*(double*)&x) : "v"(*(const double*)&bb), "v"(*(const double*)&cc)); \
    if constexpr (OP == 20) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 21) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));                                   \
    if constexpr (OP == 22) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(x));                                   \
    if constexpr (OP == 23) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b));                                 \
    if constexpr (OP == 24) asm volatile("v_min3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                 \
    if constexpr (OP == 25) asm volatile("v_med3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                 \
    if constexpr (OP == 26) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 27) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(x));                                      \
    if constexpr (OP == 28) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(b), "v"(c)); \
    if constexpr (OP == 29) asm volatile("v_or_b32 %0, %1, %0" : "+v"(x) : "v"(b));                              \
    if constexpr (OP == 30) asm volatile("v_max_i32 %0, %1, %0" : "+v"(x) : "v"(b));                             \
    if constexpr (OP == 31) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(*(double*)&x) : "v"(b), "v"(c) : "s40", "s41"); \
    if constexpr (OP == 32) asm volatile("v_lshlrev_b16 %0, 3, %0" : "+v"(x));                                   \
    if constexpr (OP == 33) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));                                      \
    if constexpr (OP == 34) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(x) : "v"(b) : "vcc");            \
    if constexpr (OP == 35) asm volatile("v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc" : "+v"(x) : "v"(b) : "vcc"); \
    if constexpr (OP == 36) asm volatile("v_cmp_lt_f32 s[40:41], %0, %1\n v_cndmask_b32_e64 %0, %1, %0, s[40:41]" : "+v"(x) : "v"(b) : "s40", "s41"); \
    if constexpr (OP == 37) asm volatile("v_min_f32 %0, %1, %0\n v_fma_f32 %0, %1, %0, %0" : "+v"(x) : "v"(b));      \
    if constexpr (OP == 38) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(*(double*)&x) : "v"(*(const double*)&bb)); \
    if constexpr (OP == 39) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(*(double*)&x) : "v"(*(const double*)&bb)); \
    if constexpr (OP == 40) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));                                   \
    if constexpr (OP == 41) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                 \
    if constexpr (OP == 42) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                 \
    \
    if constexpr (OP == 44) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));                 \
    if constexpr (OP == 45) asm volatile("v_cmp_class_f32 vcc, %0, %1" : : "v"(x), "v"(b) : "vcc");              \
    if constexpr (OP == 46) asm volatile("v_div_scale_f32 %0, vcc, %1, %1, %0" : "+v"(x) : "v"(b) : "vcc");       \
    if constexpr (OP == 47) asm volatile("v_div_fixup_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));            \
    if constexpr (OP == 48) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(x) : "v"(b));                       \
    if constexpr (OP == 49) asm volatile("v_lshl_or_b32 %0, %1, 3, %0" : "+v"(x) : "v"(b));
        R8(STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7))
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    out[2 + (blockIdx.x * 256 + threadIdx.x) % 1024] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int OP>
void run(const char* name, float* out, unsigned long long* clk, int cus) {
    const int iters = 2000, blocks = cus * 8;  // 8 blocks × 4 waves per CU = 8 waves per SIMD
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // s_memrealtime runs at 100 MHz
    const double per_simd = (double)iters * 64.0 * 8.0 * 4.0;          // instrs per SIMD: iters·64·(8 waves/SIMD)·...
    // instructions per SIMD = blocks·4 waves·iters·64 / (cus·4 SIMDs)
    const double inst_per_simd = (double)blocks * 4.0 * iters * 64.0 / (cus * 4.0);
    (void)per_simd;
    std::printf("%-16s %8.3f ms  %6.2f cyc/instr/SIMD  (clock %.2f GHz)\n", name, ms,
                ms * 1e-3 * ghz * 1e9 / inst_per_simd, ghz);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, 4096 * sizeof(float));
    hipMemset(out, 0, 4096 * sizeof(float));
    hipMalloc(&clk, 2 * sizeof(unsigned long long));
    run<38>("v_pk_add_f32", out, clk, cus);
    run<39>("v_pk_mul_f32", out, clk, cus);
    run<40>("v_lshrrev_b32", out, clk, cus);
    run<41>("v_bfi_b32", out, clk, cus);
    run<42>("v_add3_u32", out, clk, cus);
    run<44>("v_perm_b32", out, clk, cus);
    run<45>("v_cmp_class_f32", out, clk, cus);
    run<46>("v_div_scale_f32", out, clk, cus);
    run<47>("v_div_fixup_f32", out, clk, cus);
    run<48>("v_alignbit_b32", out, clk, cus);
    run<49>("v_lshl_or_b32", out, clk, cus);
    return 0;
}
