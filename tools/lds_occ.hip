// occupancy (workgroups of 64 threads per CU) vs static LDS bytes, to find the
// LDS allocation granularity on this device
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N> __global__ void __launch_bounds__(64) k(int* o) {
  __shared__ unsigned char s[N];
  s[threadIdx.x] = (unsigned char)threadIdx.x;
  __syncthreads();
  o[blockIdx.x] = s[(threadIdx.x * 7) % N];
}
template <int N> void q() {
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k<N>, 64, 0);
  printf("lds=%6d occ=%d\n", N, occ);
}
int main() {
  q<16384>(); q<20480>(); q<20481>(); q<20992>(); q<22000>(); q<23000>(); q<23168>(); q<23405>(); q<23406>();
  q<23552>(); q<24000>(); q<26856>(); q<27306>(); q<27307>(); q<27648>(); q<30952>(); q<32768>(); q<32769>();
  return 0;
}
