// Standalone check of the DPP wave prefix scan used by the flat kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int V>
__global__ void k(const unsigned* in, unsigned* out) {
  unsigned x = in[threadIdx.x];
  if (V == 0) {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, true);
  } else {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  }
  out[threadIdx.x] = x;
}
int main() {
  unsigned h[64], r[64]; for (int i = 0; i < 64; ++i) h[i] = 1u << (i % 8) | (i << 12);
  unsigned *di, *dout; hipMalloc(&di, 256); hipMalloc(&dout, 256);
  hipMemcpy(di, h, 256, hipMemcpyHostToDevice);
  for (int v = 0; v < 2; ++v) {
    if (v == 0) k<0><<<1, 64>>>(di, dout); else k<1><<<1, 64>>>(di, dout);
    hipMemcpy(r, dout, 256, hipMemcpyDeviceToHost);
    unsigned acc = 0; int bad = 0;
    for (int i = 0; i < 64; ++i) {
      acc += h[i];
      unsigned want = v == 0 ? acc : h[i] + ((i % 16) ? h[i - 1] : 0);
      if (r[i] != want) { if (bad < 6) printf("v%d lane %d got %u want %u\n", v, i, r[i], want); ++bad; }
    }
    printf("variant %d: %d bad lanes\n", v, bad);
  }
  return 0;
}
