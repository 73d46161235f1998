// Exhaustive check, on the GPU, that one FMA Newton step from v_rcp_f32 gives the correctly rounded
// reciprocal:  y = rcp(a), r = fma(-a, y, 1), y' = fma(r, y, y)  ==  RN(1/a)  for every binary32 a with
// |a| in [2^-40, 2^40] (both signs).  The kernels use y' where they need RN(1/a) (rcp_rn in render.hip);
// the reference value is the compiler's IEEE division.  Prints the mismatch count and the first few.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/check_rcp.hip -o ablib/check_rcp && ablib/check_rcp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        for (int sgn = 0; sgn < 2; sgn++) {
            const float a = __uint_as_float((lo + k) | (sgn ? 0x80000000u : 0u));
            const float y = __builtin_amdgcn_rcpf(a);
            const float r = __builtin_fmaf(-a, y, 1.0f);
            const float y1 = __builtin_fmaf(r, y, y);
            const float want = 1.0f / a;
            if (__float_as_uint(y1) != __float_as_uint(want)) {
                const unsigned long long i = atomicAdd(bad, 1ull);
                if (i < 16) first[i] = __float_as_uint(a);
            }
        }
    }
}

int main() {
    const uint32_t lo = 0x2B800000u, hi = 0x53800000u;  // 2^-40 .. 2^40 (inclusive of hi)
    const uint32_t n = hi - lo + 1u;
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMalloc(&first, 16 * sizeof(uint32_t)) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, sizeof(*bad));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, lo, n, bad, first);
    unsigned long long h_bad = 0;
    uint32_t h_first[16] = {0};
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(&h_bad, bad, sizeof(h_bad), hipMemcpyDeviceToHost);
    (void)hipMemcpy(h_first, first, sizeof(h_first), hipMemcpyDeviceToHost);
    printf("rcp + one fma Newton step vs IEEE 1/a: %u magnitudes x 2 signs, %llu mismatches\n", n, h_bad);
    for (unsigned long long i = 0; i < h_bad && i < 16; i++) printf("  a = %a (0x%08x)\n", (double)__builtin_bit_cast(float, h_first[i]), h_first[i]);
    return h_bad == 0 ? 0 : 1;
}
