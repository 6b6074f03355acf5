// WRITE_SIZE / FETCH_SIZE calibration for the access widths inflate2_kernel uses
// (MI355X_MICROARCH.md: only 16-B-per-lane streaming accesses are calibrated; "calibrate
// on a known byte count in your own access pattern").  Each kernel moves exactly
// BYTES bytes with one pattern, 4096 one-wave workgroups (the inflate's residency):
//   st_dword_wave   each wave stores its own contiguous region, 64 lanes x 4 B per
//                   instruction (phase M's span stores)
//   st_byte_wave    the same with 1-byte stores (M's span edges, E's partial groups)
//   st_lane16       each LANE stores its own region 16 B at a time (E's literal stream)
//   st_lane32       each lane its own region in 32-B groups of two 16-B stores (E's
//                   match records, RGRP = 2)
//   st_dwordx4_wave each wave its own region, 16 B per lane (the guide's calibrated case)
//   ld_dwordx4_wave / ld_dword_wave / ld_byte_wave: the loads of the same shapes
//   ld_byte_gather  M's far-source gathers: per lane one byte from a random offset in
//                   the wave's previous 32 KiB, 16 per lane per round
// Usage: rocprofv3 --pmc WRITE_SIZE -- ./tools/wcal (then FETCH_SIZE); tools/wcal_run.sh.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t BYTES = 1ull << 30;
constexpr int WAVES = 4096;
constexpr uint64_t PER_WAVE = BYTES / WAVES;        // 256 KiB: one F1 stream's output
constexpr uint64_t PER_LANE = PER_WAVE / 64;        // 4 KiB

__global__ void __launch_bounds__(64) st_dword_wave(uint32_t* p) {
  uint32_t* q = p + blockIdx.x * (PER_WAVE / 4);
  for (uint32_t i = threadIdx.x; i < PER_WAVE / 4; i += 64) q[i] = i;
}
__global__ void __launch_bounds__(64) st_byte_wave(uint8_t* p) {
  uint8_t* q = p + blockIdx.x * PER_WAVE;
  for (uint32_t i = threadIdx.x; i < PER_WAVE; i += 64) q[i] = (uint8_t)i;
}
__global__ void __launch_bounds__(64) st_dwordx4_wave(uint4* p) {
  uint4* q = p + blockIdx.x * (PER_WAVE / 16);
  for (uint32_t i = threadIdx.x; i < PER_WAVE / 16; i += 64) q[i] = make_uint4(i, i, i, i);
}
__global__ void __launch_bounds__(64) st_lane16(uint4* p) {
  uint4* q = p + (blockIdx.x * 64 + threadIdx.x) * (PER_LANE / 16);
  for (uint32_t i = 0; i < PER_LANE / 16; i++) q[i] = make_uint4(i, i, i, i);
}
__global__ void __launch_bounds__(64) st_lane32(uint4* p) {
  uint4* q = p + (blockIdx.x * 64 + threadIdx.x) * (PER_LANE / 16);
  for (uint32_t i = 0; i < PER_LANE / 16; i += 2) {
    q[i] = make_uint4(i, i, i, i);
    q[i + 1] = make_uint4(i, i, i, i);
  }
}
__global__ void __launch_bounds__(64) ld_dwordx4_wave(const uint4* p, uint32_t* sink) {
  const uint4* q = p + blockIdx.x * (PER_WAVE / 16);
  uint32_t a = 0;
  for (uint32_t i = threadIdx.x; i < PER_WAVE / 16; i += 64) { const uint4 v = q[i]; a ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (a == 0x9e3779b9u) sink[0] = a;
}
__global__ void __launch_bounds__(64) ld_dword_wave(const uint32_t* p, uint32_t* sink) {
  const uint32_t* q = p + blockIdx.x * (PER_WAVE / 4);
  uint32_t a = 0;
  for (uint32_t i = threadIdx.x; i < PER_WAVE / 4; i += 64) a ^= q[i];
  if (a == 0x9e3779b9u) sink[0] = a;
}
__global__ void __launch_bounds__(64) ld_byte_wave(const uint8_t* p, uint32_t* sink) {
  const uint8_t* q = p + blockIdx.x * PER_WAVE;
  uint32_t a = 0;
  for (uint32_t i = threadIdx.x; i < PER_WAVE; i += 64) a += q[i];
  if (a == 0x9e3779b9u) sink[0] = a;
}
// PER_WAVE byte loads per wave in all: rounds of 16 per lane from random offsets in the
// 32 KiB before a frontier that advances 1 KiB per round
__global__ void __launch_bounds__(64) ld_byte_gather(const uint8_t* p, uint32_t* sink) {
  const uint8_t* q = p + blockIdx.x * PER_WAVE;
  uint32_t a = 0, x = blockIdx.x * 64 + threadIdx.x + 1;
  for (uint32_t f = 32768; f < PER_WAVE; f += 1024) {     // 224 rounds x 16 x 64 lanes
#pragma unroll
    for (int k = 0; k < 16; k++) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      a += q[f - 1 - (x & 32767)];
    }
  }
  if (a == 0x9e3779b9u) sink[0] = a;
}

int main() {
  void* p;
  uint32_t* sink;
  if (hipMalloc(&p, BYTES) != hipSuccess || hipMalloc(&sink, 256) != hipSuccess) return 1;
  hipMemset(p, 1, BYTES);
  // a 1 GiB buffer is 4x the Infinity Cache: each kernel starts from a cold working set
  for (int rep = 0; rep < 2; rep++) {
    st_dword_wave<<<WAVES, 64>>>((uint32_t*)p);
    st_byte_wave<<<WAVES, 64>>>((uint8_t*)p);
    st_dwordx4_wave<<<WAVES, 64>>>((uint4*)p);
    st_lane16<<<WAVES, 64>>>((uint4*)p);
    st_lane32<<<WAVES, 64>>>((uint4*)p);
    ld_dwordx4_wave<<<WAVES, 64>>>((const uint4*)p, sink);
    ld_dword_wave<<<WAVES, 64>>>((const uint32_t*)p, sink);
    ld_byte_wave<<<WAVES, 64>>>((const uint8_t*)p, sink);
    ld_byte_gather<<<WAVES, 64>>>((const uint8_t*)p, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("wcal done: %llu bytes per kernel\n", (unsigned long long)BYTES);
  return 0;
}
