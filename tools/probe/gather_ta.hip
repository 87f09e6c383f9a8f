// Gather cost probe: per-lane random record gathers (the list walks' pattern)
// against quad-cooperative gathers (4 lanes load the 16-B pieces of one 64-B
// record). Indices are neighbour-like: j drawn from a 4096-record window that
// slides with the wave, as a Morton-sorted neighbour list. Prints ms and
// ns per record for each variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kEnt = 32;  // entries per lane

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ int jof(int wave, int e, int key, int n) {
  const int base = (int)(((long long)wave * 11) % (n - 4096));
  return base + (int)(hash((unsigned)(wave * 977 + e * 131 + key)) & 4095u);
}

// A: every lane gathers its own 48-B record (3 x 16 B) per entry
__global__ void per_lane(const float4* __restrict__ t, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  float acc = 0.f;
  for (int e = 0; e < kEnt; e++) {
    const int j = jof(wave, e, lane, n);
    const float4 a = t[4 * j], b = t[4 * j + 1], c = t[4 * j + 2];
    acc += a.x + b.y + c.z;
  }
  if (acc == 1234.5f) out[0] = acc;
}
// B: the 4 lanes of a quad share j, lane s loads piece s of the 64-B record
// (4 x kEnt entries per quad: the same records-per-lane as A)
__global__ void quad_coop(const float4* __restrict__ t, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int q = lane >> 2, s = lane & 3;
  float acc = 0.f;
  for (int e = 0; e < kEnt; e++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int j = jof(wave, e, 4 * q + k, n);
      const float4 a = t[4 * j + s];
      acc += a.x;
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}
// C: every lane gathers one 16-B piece of its own record per entry
__global__ void per_lane16(const float4* __restrict__ t, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  float acc = 0.f;
  for (int e = 0; e < kEnt; e++) {
    const int j = jof(wave, e, lane, n);
    acc += t[4 * j].x;
  }
  if (acc == 1234.5f) out[0] = acc;
}
// D: index arithmetic only (no loads), the floor of the others
__global__ void no_load(const float4* __restrict__ t, int n, float* out) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  float acc = 0.f;
  for (int e = 0; e < kEnt; e++) acc += (float)jof(wave, e, lane, n);
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const int n = 2 * 1024 * 1024;  // records (64 B each: 128 MB)
  float4* t;
  float* out;
  hipMalloc(&t, (size_t)n * 64);
  hipMalloc(&out, 64);
  hipMemset(t, 0, (size_t)n * 64);
  const int lanes = n;  // one lane per "particle"
  const dim3 grid(lanes / 256), block(256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[4] = {"per_lane 3x16B", "quad_coop 1x16B/lane", "per_lane 1x16B", "no_load"};
  for (int v = 0; v < 4; v++) {
    float best = 1e30f;
    for (int rep = 0; rep < 6; rep++) {
      hipEventRecord(e0);
      if (v == 0) per_lane<<<grid, block>>>(t, n, out);
      if (v == 1) quad_coop<<<grid, block>>>(t, n, out);
      if (v == 2) per_lane16<<<grid, block>>>(t, n, out);
      if (v == 3) no_load<<<grid, block>>>(t, n, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    const double recs = (double)lanes * kEnt;  // records fetched per launch (every variant)
    const double instr = v == 0 ? recs / 64 * 3 : v == 3 ? 0 : recs / 64 * (v == 1 ? 4 : 1);
    printf("%-24s %8.3f ms  %6.3f ns/record  %.1f cycles/wave-instr/CU\n", names[v], best,
           best * 1e6 / recs, instr > 0 ? best * 1e-3 * 2.4e9 * 256 / instr : 0.0);
  }
  return 0;
}
