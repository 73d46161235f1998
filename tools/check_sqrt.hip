// Exhaustive check, on the GPU, of cheaper correctly rounded square roots against the compiler's IEEE sqrtf
// for every binary32 x in [2^-96, +inf) (sqrt_rn's range in render.hip):
//   raw   v_sqrt_f32 alone
//   down  v_sqrt_f32 + the lower-neighbour residual check only
//   up    v_sqrt_f32 + the upper-neighbour residual check only
//   both  the two checks (sqrt_rn, the kernels' current sequence)
// and raw v_rcp_f32 against IEEE 1/a over |a| in [2^-40, 2^40].  Prints the mismatch count per variant.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/check_sqrt.hip -o ablib/check_sqrt && ablib/check_sqrt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const float x = __uint_as_float(lo + k);
        const float want = sqrtf(x);
        const float s = __builtin_amdgcn_sqrtf(x);
        const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
        const float down = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
        const float up = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : s;
        const float both = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : down;
        const float got[4] = {s, down, up, both};
        for (int v = 0; v < 4; v++) {
            if (__float_as_uint(got[v]) != __float_as_uint(want)) {
                const unsigned long long i = atomicAdd(&bad[v], 1ull);
                if (i < 4) first[v * 4 + i] = __float_as_uint(x);
            }
        }
    }
}

__global__ void check_rcp_raw(uint32_t lo, uint32_t n, unsigned long long* bad) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const float a = __uint_as_float(lo + k);
        if (__float_as_uint(__builtin_amdgcn_rcpf(a)) != __float_as_uint(1.0f / a)) atomicAdd(bad, 1ull);
    }
}

int main() {
    const uint32_t lo = 0x0F800000u, hi = 0x7F800000u;  // 2^-96 .. +inf
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 5 * sizeof(*bad)) != hipSuccess || hipMalloc(&first, 16 * sizeof(uint32_t)) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 5 * sizeof(*bad));
    (void)hipMemset(first, 0, 16 * sizeof(uint32_t));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, lo, hi - lo + 1u, bad, first);
    hipLaunchKernelGGL(check_rcp_raw, dim3(8192), dim3(256), 0, 0, 0x2B800000u, 0x53800000u - 0x2B800000u + 1u, bad + 4);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long h[5] = {0};
    uint32_t f[16] = {0};
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    const char* names[4] = {"raw v_sqrt_f32", "down check only", "up check only", "both checks"};
    for (int v = 0; v < 4; v++) {
        printf("sqrt %-16s: %llu mismatches in [2^-96, inf]", names[v], h[v]);
        for (unsigned long long i = 0; i < h[v] && i < 4; i++) printf("  %a", (double)__builtin_bit_cast(float, f[v * 4 + i]));
        printf("\n");
    }
    printf("raw v_rcp_f32 vs IEEE 1/a, a in [2^-40, 2^40]: %llu mismatches\n", h[4]);
    return 0;
}
