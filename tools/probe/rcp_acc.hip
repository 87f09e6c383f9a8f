// Accuracy of v_rcp_f64 / v_rsq_f64 with 0, 1, 2 Newton steps vs IEEE 1/x and
// 1/sqrt(x) (fp64), over x in [1e-6, 1e6]. Prints the max relative errors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__global__ void probe(int n, double* out) {
  double e[6] = {0, 0, 0, 0, 0, 0};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double x = exp(-13.8 + 27.6 * ((double)i + 0.5) / n);
    const double r = 1.0 / x, s = 1.0 / sqrt(x);
    double y = __builtin_amdgcn_rcp(x);
    e[0] = fmax(e[0], fabs(y - r) / r);
    double t = fma(-x, y, 1.0); y = fma(y, t, y);
    e[1] = fmax(e[1], fabs(y - r) / r);
    t = fma(-x, y, 1.0); y = fma(y, t, y);
    e[2] = fmax(e[2], fabs(y - r) / r);
    double z = __builtin_amdgcn_rsq(x);
    e[3] = fmax(e[3], fabs(z - s) / s);
    const double h = 0.5 * x;
    double u = fma(-h * z, z, 0.5); z = fma(z, u, z);
    e[4] = fmax(e[4], fabs(z - s) / s);
    u = fma(-h * z, z, 0.5); z = fma(z, u, z);
    e[5] = fmax(e[5], fabs(z - s) / s);
  }
  for (int k = 0; k < 6; k++) {
    double v = e[k];
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long*)&out[k], (unsigned long long)__double_as_longlong(v));
  }
}

int main() {
  double* d;
  hipMalloc(&d, 6 * sizeof(double));
  hipMemset(d, 0, 6 * sizeof(double));
  hipLaunchKernelGGL(probe, dim3(1024), dim3(256), 0, 0, 1 << 26, d);
  double h[6];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("rcp_f64 raw %.3e  1 Newton %.3e  2 Newton %.3e\n", h[0], h[1], h[2]);
  printf("rsq_f64 raw %.3e  1 Newton %.3e  2 Newton %.3e\n", h[3], h[4], h[5]);
  hipFree(d);
  return 0;
}
