// swh_api.hip — context lifetime, error plumbing and layout descriptors of
// libswifthip (include/swifthip.h).
#include <cstdarg>
#include <cstddef>

#include "swh_internal.h"
#include "swh_physics.h"
#include "swift_compat.h"

namespace swh {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static bool aligned_field(int off, int size, int stride) {
  return off < 0 || (off % size == 0 && off + size <= stride);
}

swh_status make_layout(const swh_part_layout* L, Layout* o) {
  if (!L || L->stride <= 0 || (L->stride % 8) != 0) {
    set_error("invalid part layout stride");
    return SWH_ERR_ARG;
  }
  o->stride = L->stride;
  o->id = L->off_id;
  o->x = L->off_x;
  o->v = L->off_v;
  o->a_hydro = L->off_a_hydro;
  o->mass = L->off_mass;
  o->h = L->off_h;
  o->u = L->off_u;
  o->u_dt = L->off_u_dt;
  o->rho = L->off_rho;
  o->div_v = L->off_div_v;
  o->div_v_dt = L->off_div_v_dt;
  o->div_v_prev = L->off_div_v_previous_step;
  o->visc_alpha = L->off_visc_alpha;
  o->v_sig = L->off_v_sig;
  o->laplace_u = L->off_laplace_u;
  o->diff_alpha = L->off_diff_alpha;
  o->wcount = L->off_wcount;
  o->wcount_dh = L->off_wcount_dh;
  o->rho_dh = L->off_rho_dh;
  o->rot_v = L->off_rot_v;
  o->f = L->off_f;
  o->pressure = L->off_pressure;
  o->soundspeed = L->off_soundspeed;
  o->h_dt = L->off_h_dt;
  o->balsara = L->off_balsara;
  o->avmn = L->off_alpha_visc_max_ngb;
  o->time_bin = L->off_time_bin;
  o->min_tb = L->off_min_ngb_time_bin;
  o->gpart = L->off_gpart;
  if (o->gpart >= 0 && (!aligned_field(o->gpart, 8, o->stride) || o->gpart + 8 > o->stride)) {
    set_error("misaligned gpart pointer offset %d", o->gpart);
    return SWH_ERR_ARG;
  }
  const int fl[] = {o->mass, o->h, o->u, o->u_dt, o->rho, o->div_v, o->div_v_dt,
                    o->div_v_prev, o->visc_alpha, o->v_sig, o->laplace_u,
                    o->diff_alpha, o->wcount, o->wcount_dh, o->rho_dh, o->f,
                    o->pressure, o->soundspeed, o->h_dt, o->balsara, o->avmn};
  for (int f : fl)
    if (!aligned_field(f, 4, o->stride)) {
      set_error("misaligned float field offset %d", f);
      return SWH_ERR_ARG;
    }
  if (o->x < 0 || !aligned_field(o->x, 8, o->stride) || o->x + 24 > o->stride ||
      o->v < 0 || !aligned_field(o->v, 4, o->stride) || o->mass < 0 || o->h < 0 ||
      o->time_bin < 0 || o->time_bin >= o->stride) {
    set_error("part layout lacks x/v/mass/h/time_bin");
    return SWH_ERR_ARG;
  }
  return SWH_OK;
}

swh_status make_glayout(const swh_gpart_layout* L, GLayout* o) {
  if (!L || L->stride <= 0 || (L->stride % 8) != 0 || L->off_x < 0 ||
      L->off_x % 8 || L->off_mass < 0 || L->off_epsilon < 0 || L->off_a_grav < 0 ||
      L->off_potential < 0 || L->off_time_bin < 0) {
    set_error("invalid gpart layout");
    return SWH_ERR_ARG;
  }
  o->stride = L->stride;
  o->x = L->off_x;
  o->a_grav = L->off_a_grav;
  o->potential = L->off_potential;
  o->mass = L->off_mass;
  o->epsilon = L->off_epsilon;
  o->time_bin = L->off_time_bin;
  o->old_a_grav_norm = L->off_old_a_grav_norm;
  return SWH_OK;
}

}  // namespace swh

swh::TaskWorker* swh_context::lease() {
  std::lock_guard<std::mutex> g(lease_mutex);
  for (auto* w : workers)
    if (w->busy.try_lock()) return w;
  auto* w = new swh::TaskWorker();
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) {
    delete w;
    return nullptr;
  }
  w->busy.lock();
  workers.push_back(w);
  return w;
}

void swh_context::unlease(swh::TaskWorker* w) { w->busy.unlock(); }

extern "C" {

int swh_abi_version(void) { return SWH_ABI_VERSION; }

const char* swh_kernel_name(void) { return SWH_KERNEL_NAME; }

const char* swh_last_error(void) { return swh::g_err; }

const char* swh_status_string(swh_status s) {
  switch (s) {
    case SWH_OK: return "ok";
    case SWH_ERR_ARG: return "invalid argument";
    case SWH_ERR_HIP: return "HIP runtime error";
    case SWH_ERR_UNSORTED: return "Interacting unsorted cells.";
    case SWH_ERR_CELL_SMALL: return "Cell smaller than smoothing length";
    case SWH_ERR_NOT_CONVERGED: return "Smoothing length failed to converge";
    case SWH_ERR_NO_DEVICE: return "no usable gfx950 device";
    case SWH_ERR_OOM: return "device out of memory";
    case SWH_ERR_STATE: return "call out of order";
    case SWH_BUSY: return "busy (queued work still running)";
  }
  return "unknown";
}

void swh_part_layout_sphenix(swh_part_layout* o) {
  o->stride = (int32_t)sizeof(struct part);
  o->off_id = offsetof(struct part, id);
  o->off_x = offsetof(struct part, x);
  o->off_v = offsetof(struct part, v);
  o->off_a_hydro = offsetof(struct part, a_hydro);
  o->off_mass = offsetof(struct part, mass);
  o->off_h = offsetof(struct part, h);
  o->off_u = offsetof(struct part, u);
  o->off_u_dt = offsetof(struct part, u_dt);
  o->off_rho = offsetof(struct part, rho);
  o->off_div_v = offsetof(struct part, viscosity.div_v);
  o->off_div_v_dt = offsetof(struct part, viscosity.div_v_dt);
  o->off_div_v_previous_step = offsetof(struct part, viscosity.div_v_previous_step);
  o->off_visc_alpha = offsetof(struct part, viscosity.alpha);
  o->off_v_sig = offsetof(struct part, viscosity.v_sig);
  o->off_laplace_u = offsetof(struct part, diffusion.laplace_u);
  o->off_diff_alpha = offsetof(struct part, diffusion.alpha);
  o->off_wcount = offsetof(struct part, density.wcount);
  o->off_wcount_dh = offsetof(struct part, density.wcount_dh);
  o->off_rho_dh = offsetof(struct part, density.rho_dh);
  o->off_rot_v = offsetof(struct part, density.rot_v);
  o->off_f = offsetof(struct part, force.f);
  o->off_pressure = offsetof(struct part, force.pressure);
  o->off_soundspeed = offsetof(struct part, force.soundspeed);
  o->off_h_dt = offsetof(struct part, force.h_dt);
  o->off_balsara = offsetof(struct part, force.balsara);
  o->off_alpha_visc_max_ngb = offsetof(struct part, force.alpha_visc_max_ngb);
  o->off_time_bin = offsetof(struct part, time_bin);
  o->off_min_ngb_time_bin = offsetof(struct part, limiter_data.min_ngb_time_bin);
  o->off_gpart = offsetof(struct part, gpart);
}

void swh_gpart_layout_multisoftening(swh_gpart_layout* o) {
  o->stride = (int32_t)sizeof(struct gpart);
  o->off_x = offsetof(struct gpart, x);
  o->off_a_grav = offsetof(struct gpart, a_grav);
  o->off_potential = offsetof(struct gpart, potential);
  o->off_mass = offsetof(struct gpart, mass);
  o->off_epsilon = offsetof(struct gpart, epsilon);
  o->off_time_bin = offsetof(struct gpart, time_bin);
  o->off_old_a_grav_norm = offsetof(struct gpart, old_a_grav_norm);
}

swh_status swh_init(swh_context** out, int device) {
  if (!out) return SWH_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    swh::set_error("no HIP device visible");
    return SWH_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= n) {
    swh::set_error("device %d out of range (%d devices)", device, n);
    return SWH_ERR_NO_DEVICE;
  }
  hipDeviceProp_t prop;
  SWH_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    swh::set_error("device %d is %s, libswifthip is built for gfx950", device,
                   prop.gcnArchName);
    return SWH_ERR_NO_DEVICE;
  }
  SWH_HIP(hipSetDevice(device));
  auto* c = new swh_context();
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  *out = c;
  return SWH_OK;
}

swh_status swh_finalize(swh_context* c) {
  if (!c) return SWH_OK;
  (void)hipSetDevice(c->device);
  for (auto* w : c->workers) {
    if (w->stream) (void)hipStreamSynchronize(w->stream);
    w->dparts.release();
    w->dparts2.release();
    w->dind.release();
    w->dself.release();
    w->dcount.release();
    w->hstage.release();
    w->hstage2.release();
    if (w->stream) (void)hipStreamDestroy(w->stream);
    delete w;
  }
  delete c;
  return SWH_OK;
}

swh_status swh_set_precision(swh_context* c, swh_precision p) {
  if (!c || (p != SWH_PRECISION_F64 && p != SWH_PRECISION_F32)) return SWH_ERR_ARG;
  c->precision = p;
  return SWH_OK;
}

}  // extern "C"
