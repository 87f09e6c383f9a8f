// swh_mesh.hip — the particle-mesh long-range gravity (PM):
// src/mesh_gravity.c compute_potential_global (844-1041) for a
// non-distributed periodic mesh, on the uploaded gpart set of a swh_gspace.
//
//   cic_assign_kernel : one thread per gpart, the gpart_to_mesh_CIC (137-182)
//                       weights added to the N^3 fp64 density mesh with
//                       global fp64 atomics (CIC_set's atomic_add_d);
//   hipFFT D2Z        : the r2c transform (FFTW's fftw_plan_dft_r2c_3d; both
//                       unnormalised, row-major, z fastest);
//   green_kernel      : one thread per complex mode, the Green function with
//                       the long-range truncation and the CIC deconvolution of
//                       mesh_apply_Green_function_mapper (519-593), (0,0,0)
//                       zeroed (633-637);
//   hipFFT Z2D        : the c2r transform back to the potential mesh;
//   mesh_accel_kernel : one thread per gpart, mesh_to_gpart_CIC (308-394):
//                       the CIC potential and the 5-point-stencil
//                       accelerations, times const_G (428-470), written to the
//                       record's a_grav_mesh / potential_mesh (overwritten, as
//                       the reference zeroes them first).
//
// The mesh is HBM-streaming work (assignment and interpolation are scattered
// atomics / gathers over an N^3 mesh that L2 and the Infinity Cache hold for
// the usual N <= 512); the FFTs are hipFFT's.
#include <hipfft/hipfft.h>

#include <cfloat>

#include <cstdio>
#include <cstdlib>
#include "swh_internal.h"
#include "swh_physics.h"

namespace swh {

// row_major_id_periodic (src/row_major_id.h:39-43)
__device__ __forceinline__ int pm_id(int i, int j, int k, int N) {
  return ((i + N) % N) * N * N + ((j + N) % N) * N + ((k + N) % N);
}

struct CicW {
  int i, j, k;
  double tx, ty, tz, dx, dy, dz;
};

// box_wrap + the CIC coefficients (mesh_gravity.c:143-161, 312-329)
__device__ __forceinline__ CicW cic_weights(const double* x, double box, int N, double fac) {
  double p[3];
  for (int a = 0; a < 3; a++) p[a] = x[a] < 0. ? x[a] + box : (x[a] >= box ? x[a] - box : x[a]);
  CicW w;
  w.i = (int)(fac * p[0]);
  if (w.i >= N) w.i = N - 1;
  w.dx = fac * p[0] - w.i;
  w.tx = 1. - w.dx;
  w.j = (int)(fac * p[1]);
  if (w.j >= N) w.j = N - 1;
  w.dy = fac * p[1] - w.j;
  w.ty = 1. - w.dy;
  w.k = (int)(fac * p[2]);
  if (w.k >= N) w.k = N - 1;
  w.dz = fac * p[2] - w.k;
  w.tz = 1. - w.dz;
  return w;
}

__global__ void cic_assign_kernel(GLayout L, const char* __restrict__ aos, int64_t n, int N,
                                  double box, double fac, double* __restrict__ rho) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const char* r = aos + p * L.stride;
  if (*reinterpret_cast<const int8_t*>(r + L.time_bin) == kTimeBinInhibited) return;
  const CicW w = cic_weights(reinterpret_cast<const double*>(r + L.x), box, N, fac);
  const double value = (double)*reinterpret_cast<const float*>(r + L.mass);
  const int i = w.i, j = w.j, k = w.k;
  atomicAdd(&rho[pm_id(i + 0, j + 0, k + 0, N)], value * w.tx * w.ty * w.tz);
  atomicAdd(&rho[pm_id(i + 0, j + 0, k + 1, N)], value * w.tx * w.ty * w.dz);
  atomicAdd(&rho[pm_id(i + 0, j + 1, k + 0, N)], value * w.tx * w.dy * w.tz);
  atomicAdd(&rho[pm_id(i + 0, j + 1, k + 1, N)], value * w.tx * w.dy * w.dz);
  atomicAdd(&rho[pm_id(i + 1, j + 0, k + 0, N)], value * w.dx * w.ty * w.tz);
  atomicAdd(&rho[pm_id(i + 1, j + 0, k + 1, N)], value * w.dx * w.ty * w.dz);
  atomicAdd(&rho[pm_id(i + 1, j + 1, k + 0, N)], value * w.dx * w.dy * w.tz);
  atomicAdd(&rho[pm_id(i + 1, j + 1, k + 1, N)], value * w.dx * w.dy * w.dz);
}

// mesh_apply_Green_function_mapper (519-593) on the N x N x (N/2+1) modes
__global__ void green_kernel(hipfftDoubleComplex* __restrict__ frho, int N, double green_fac,
                             double a_smooth2, double k_fac) {
  const int Nh = N / 2, nz = Nh + 1;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)N * N * nz) return;
  const int k = (int)(q % nz), j = (int)((q / nz) % N), i = (int)(q / ((int64_t)nz * N));
  if (q == 0) {  // the singularity at (0, 0, 0) (633-637)
    frho[0].x = 0.;
    frho[0].y = 0.;
    return;
  }
  const int kx = i > Nh ? i - N : i;
  const double kx_d = (double)kx, fx = k_fac * kx_d;
  const double sinc_kx_inv = (kx != 0) ? fx / sin(fx) : 1.;
  const int ky = j > Nh ? j - N : j;
  const double ky_d = (double)ky, fy = k_fac * ky_d;
  const double sinc_ky_inv = (ky != 0) ? fy / sin(fy) : 1.;
  const int kz = k > Nh ? k - N : k;
  const double kz_d = (double)kz, fz = k_fac * kz_d;
  const double sinc_kz_inv = (kz != 0) ? fz / (sin(fz) + FLT_MIN) : 1.;
  const double k2 = kx_d * kx_d + ky_d * ky_d + kz_d * kz_d;
  if (k2 == 0.) return;
  // fourier_kernel_long_grav_eval (kernel_long_gravity.h:310-319)
  const double u = sqrt(k2 * a_smooth2);
  const double arg = M_PI_2 * u;
  const double W = arg / (sinh(arg) + FLT_MIN);
  const double green_cor = green_fac * W / (k2 + FLT_MIN);
  const double CIC_cor = sinc_kx_inv * sinc_ky_inv * sinc_kz_inv;
  const double CIC_cor2 = CIC_cor * CIC_cor;
  const double CIC_cor4 = CIC_cor2 * CIC_cor2;
  const double total_cor = green_cor * CIC_cor4;
  frho[q].x *= total_cor;
  frho[q].y *= total_cor;
}

__device__ __forceinline__ double cic_get(const double* __restrict__ pot, int N, int i, int j,
                                          int k, const CicW& w) {  // CIC_get (69-85)
  double temp;
  temp = pot[pm_id(i + 0, j + 0, k + 0, N)] * w.tx * w.ty * w.tz;
  temp += pot[pm_id(i + 0, j + 0, k + 1, N)] * w.tx * w.ty * w.dz;
  temp += pot[pm_id(i + 0, j + 1, k + 0, N)] * w.tx * w.dy * w.tz;
  temp += pot[pm_id(i + 0, j + 1, k + 1, N)] * w.tx * w.dy * w.dz;
  temp += pot[pm_id(i + 1, j + 0, k + 0, N)] * w.dx * w.ty * w.tz;
  temp += pot[pm_id(i + 1, j + 0, k + 1, N)] * w.dx * w.ty * w.dz;
  temp += pot[pm_id(i + 1, j + 1, k + 0, N)] * w.dx * w.dy * w.tz;
  temp += pot[pm_id(i + 1, j + 1, k + 1, N)] * w.dx * w.dy * w.dz;
  return temp;
}

__global__ void mesh_accel_kernel(GLayout L, char* __restrict__ aos, int64_t n, int N,
                                  double box, double fac, float const_G, int off_a_mesh,
                                  int off_pot_mesh, const double* __restrict__ pot) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  char* r = aos + p * L.stride;
  if (*reinterpret_cast<const int8_t*>(r + L.time_bin) == kTimeBinInhibited) return;
  const CicW w = cic_weights(reinterpret_cast<const double*>(r + L.x), box, N, fac);
  const int i = w.i, j = w.j, k = w.k;
  double pp = 0.;
  double a[3] = {0., 0., 0.};
  pp += cic_get(pot, N, i, j, k, w);
  a[0] += (1. / 12.) * cic_get(pot, N, i + 2, j, k, w);
  a[0] -= (2. / 3.) * cic_get(pot, N, i + 1, j, k, w);
  a[0] += (2. / 3.) * cic_get(pot, N, i - 1, j, k, w);
  a[0] -= (1. / 12.) * cic_get(pot, N, i - 2, j, k, w);
  a[1] += (1. / 12.) * cic_get(pot, N, i, j + 2, k, w);
  a[1] -= (2. / 3.) * cic_get(pot, N, i, j + 1, k, w);
  a[1] += (2. / 3.) * cic_get(pot, N, i, j - 1, k, w);
  a[1] -= (1. / 12.) * cic_get(pot, N, i, j - 2, k, w);
  a[2] += (1. / 12.) * cic_get(pot, N, i, j, k + 2, w);
  a[2] -= (2. / 3.) * cic_get(pot, N, i, j, k + 1, w);
  a[2] += (2. / 3.) * cic_get(pot, N, i, j, k - 1, w);
  a[2] -= (1. / 12.) * cic_get(pot, N, i, j, k - 2, w);
  float* am = reinterpret_cast<float*>(r + off_a_mesh);
  for (int q = 0; q < 3; q++) {
    float v = (float)(fac * a[q]);
    v *= const_G;
    am[q] = v;
  }
  float pm = 0.f;
  pm += (float)pp;  // gravity_add_comoving_mesh_potential takes a float
  pm *= const_G;
  *reinterpret_cast<float*>(r + off_pot_mesh) = pm;
}

void mesh_release(swh_gspace* g) {
  g->mesh_rho.release();
  g->mesh_frho.release();
  if (g->mesh_plans_valid) {
    hipfftDestroy((hipfftHandle)g->mesh_fwd);
    hipfftDestroy((hipfftHandle)g->mesh_inv);
  }
  g->mesh_plans_valid = false;
  g->mesh_N = 0;
}

}  // namespace swh

using namespace swh;

extern "C" {

// N in [2, 1290] (mesh_gravity.c:1172), even or odd. The plans are made with
// hipfftCreate + hipfftMakePlan3d, which report each plan's work area, so a
// failing plan is an error return, never a crash (SWH_PM_DEBUG=1 prints the
// work sizes).
swh_status swh_gspace_pm_mesh(swh_gspace* g, const swh_pm_params* M, double* potential_out) {
  if (!g || !M) return SWH_ERR_ARG;
  const GLayout& L = g->layout;
  if (M->N < 2 || M->N > 1290 || !(M->box_size > 0.) || !(M->r_s > 0.) ||
      M->off_a_grav_mesh < 0 || M->off_potential_mesh < 0 ||
      (g->n > 0 && (M->off_a_grav_mesh + 12 > L.stride || M->off_potential_mesh + 4 > L.stride))) {
    set_error("pm_mesh: N must be in [2, 1290] (mesh_gravity.c:1172), box and r_s > 0, "
              "mesh fields inside the record");
    return SWH_ERR_ARG;
  }
  SWH_HIP(hipSetDevice(g->ctx->device));
  const int N = M->N;
  const size_t N3 = (size_t)N * N * N, NC = (size_t)N * N * (N / 2 + 1);
  SWH_TRY(g->mesh_rho.reserve(N3 * sizeof(double)));
  SWH_TRY(g->mesh_frho.reserve(NC * sizeof(hipfftDoubleComplex)));
  if (g->mesh_N != N) {
    if (g->mesh_plans_valid) {
      hipfftDestroy((hipfftHandle)g->mesh_fwd);
      hipfftDestroy((hipfftHandle)g->mesh_inv);
      g->mesh_plans_valid = false;
    }
    hipfftHandle f = nullptr, b = nullptr;
    size_t wf = 0, wb = 0;
    hipfftResult rf = hipfftCreate(&f);
    if (rf == HIPFFT_SUCCESS) rf = hipfftMakePlan3d(f, N, N, N, HIPFFT_D2Z, &wf);
    hipfftResult rb = rf == HIPFFT_SUCCESS ? hipfftCreate(&b) : rf;
    if (rb == HIPFFT_SUCCESS) rb = hipfftMakePlan3d(b, N, N, N, HIPFFT_Z2D, &wb);
    if (std::getenv("SWH_PM_DEBUG"))
      std::fprintf(stderr, "swh_gspace_pm_mesh: N = %d D2Z plan %d work %zu B, Z2D plan %d work %zu B\n",
                   N, (int)rf, wf, (int)rb, wb);
    if (rf != HIPFFT_SUCCESS || rb != HIPFFT_SUCCESS) {
      if (f) hipfftDestroy(f);
      if (b) hipfftDestroy(b);
      set_error("hipfftMakePlan3d failed for N = %d (D2Z %d, Z2D %d)", N, (int)rf, (int)rb);
      return SWH_ERR_HIP;
    }
    g->mesh_fwd = (void*)f;
    g->mesh_inv = (void*)b;
    g->mesh_plans_valid = true;
    g->mesh_N = N;
  }
  hipfftHandle f = (hipfftHandle)g->mesh_fwd, b = (hipfftHandle)g->mesh_inv;
  if (hipfftSetStream(f, g->stream) != HIPFFT_SUCCESS ||
      hipfftSetStream(b, g->stream) != HIPFFT_SUCCESS)
    return SWH_ERR_HIP;
  const double box = M->box_size, fac = N / box;
  double* rho = g->mesh_rho.as<double>();
  hipfftDoubleComplex* frho = g->mesh_frho.as<hipfftDoubleComplex>();
  SWH_HIP(hipMemsetAsync(rho, 0, N3 * sizeof(double), g->stream));
  const int block = 256;
  if (g->n > 0)
    hipLaunchKernelGGL(cic_assign_kernel, dim3((int)((g->n + block - 1) / block)), dim3(block), 0,
                       g->stream, L, g->aos.as<const char>(), g->n, N, box, fac, rho);
  SWH_HIP(hipGetLastError());
  if (hipfftExecD2Z(f, rho, frho) != HIPFFT_SUCCESS) {
    set_error("hipfftExecD2Z failed");
    return SWH_ERR_HIP;
  }
  const double green_fac = -1. / (M_PI * box);
  const double a_smooth2 = 4. * M_PI * M_PI * M->r_s * M->r_s / (box * box);
  const double k_fac = M_PI / (double)N;
  hipLaunchKernelGGL(green_kernel, dim3((int)((NC + block - 1) / block)), dim3(block), 0,
                     g->stream, frho, N, green_fac, a_smooth2, k_fac);
  SWH_HIP(hipGetLastError());
  if (hipfftExecZ2D(b, frho, rho) != HIPFFT_SUCCESS) {
    set_error("hipfftExecZ2D failed");
    return SWH_ERR_HIP;
  }
  if (g->n > 0)
    hipLaunchKernelGGL(mesh_accel_kernel, dim3((int)((g->n + block - 1) / block)), dim3(block), 0,
                       g->stream, L, g->aos.as<char>(), g->n, N, box, fac, (float)M->const_G,
                       M->off_a_grav_mesh, M->off_potential_mesh, rho);
  SWH_HIP(hipGetLastError());
  if (potential_out) {
    SWH_HIP(hipMemcpyAsync(potential_out, rho, N3 * sizeof(double), hipMemcpyDeviceToHost,
                           g->stream));
    SWH_HIP(hipStreamSynchronize(g->stream));
  }
  return SWH_OK;
}

}  // extern "C"
