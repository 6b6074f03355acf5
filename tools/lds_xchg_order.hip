// Diagnostic: the order in which one wave's ds_wrxchg_rtn_b32 lanes that hit the same LDS
// address are applied.  Lane-ascending order would make an exchange on a head table give
// every position its predecessor in the same 64-position step (exact hash chains without a
// sort).  Prints the number of lanes whose returned value differs from the lane-order
// prediction, over many random hash patterns.   hipcc --offload-arch=gfx950 -O3 -o x this.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__global__ void __launch_bounds__(64) xchg(const uint32_t* __restrict__ keys, uint32_t* __restrict__ out, int nbits) {
  __shared__ uint32_t tab[4096];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4096; i += 64) tab[i] = 0xffffffffu;
  __syncthreads();
  const uint32_t k = keys[blockIdx.x * 64 + lane] & ((1u << nbits) - 1u);
  out[blockIdx.x * 64 + lane] = atomicExch(&tab[k], (uint32_t)lane);
}

int main() {
  const int nb = 20000;
  uint32_t *hk = (uint32_t*)malloc(nb * 64 * 4), *ho = (uint32_t*)malloc(nb * 64 * 4);
  uint32_t *dk, *dout;
  hipMalloc(&dk, nb * 64 * 4);
  hipMalloc(&dout, nb * 64 * 4);
  srand(7);
  for (int nbits = 0; nbits <= 11; nbits++) {
    for (int i = 0; i < nb * 64; i++) hk[i] = (uint32_t)rand();
    hipMemcpy(dk, hk, nb * 64 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(xchg, dim3(nb), dim3(64), 0, 0, dk, dout, nbits);
    hipMemcpy(ho, dout, nb * 64 * 4, hipMemcpyDeviceToHost);
    long bad = 0, desc = 0;
    for (int b = 0; b < nb; b++)
      for (int l = 0; l < 64; l++) {
        const uint32_t m = (1u << nbits) - 1u, k = hk[b * 64 + l] & m;
        uint32_t want = 0xffffffffu, wdesc = 0xffffffffu;
        for (int j = l - 1; j >= 0; j--) if ((hk[b * 64 + j] & m) == k) { want = j; break; }
        for (int j = l + 1; j < 64; j++) if ((hk[b * 64 + j] & m) == k) { wdesc = j; break; }
        bad += ho[b * 64 + l] != want;
        desc += ho[b * 64 + l] != wdesc;
      }
    printf("hash bits %2d: %ld of %d lanes differ from lane-ascending order (%ld from descending)\n", nbits, bad,
           nb * 64, desc);
  }
  return 0;
}
