// Exhaustive check of the two-FMA reciprocal (hardware v_rcp_f32 estimate + one Newton step) against
// the correctly rounded 1.0f / x the compiler emits (div_scale / div_fmas / div_fixup), over every
// positive float whose reciprocal is a normal float; a mismatch count per binade is printed.
// Build: hipcc -O3 --offload-arch=gfx950 tools/rcp_check.hip -o tools/rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_nr(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

__global__ void k_check(uint32_t first, uint32_t n, unsigned long long* bad, uint32_t* example) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t bits = first + i;
    const float x = __uint_as_float(bits);
    const float a = 1.0f / x, b = rcp_nr(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
      atomicAdd(bad, 1ull);
      atomicMin(example, bits);
    }
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* ex;
  hipMalloc(&bad, 8);
  hipMalloc(&ex, 4);
  unsigned long long total = 0;
  // exponents 1 .. 252 (x in [2^-126, 2^126)): 1/x stays a normal float
  for (uint32_t e = 1; e <= 252; e++) {
    hipMemset(bad, 0, 8);
    hipMemset(ex, 0xFF, 4);
    hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, e << 23, 1u << 23, bad, ex);
    unsigned long long h = 0;
    uint32_t hx = 0;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hx, ex, 4, hipMemcpyDeviceToHost);
    if (h) printf("exponent %u: %llu mismatches (first x bits 0x%08x)\n", e, h, hx);
    total += h;
  }
  printf("total mismatches over [2^-126, 2^126): %llu\n", total);
  return total ? 1 : 0;
}
