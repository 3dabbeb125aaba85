// pbg_capi.hip -- the C-ABI (include/pbg.h) over the step/reset kernels of pbg_step.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <new>

#include "../../include/pbg.h"
#include "pbg_step.hip"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* a = "", long b = 0) {
  snprintf(g_err, sizeof(g_err), fmt, a, b);
  return code;
}

int env_robot_id(const char* env_id) {
  if (!env_id) return -1;
  static const char* ids[5][2] = {{"InvertedPendulumPyBulletEnv-v0", "pendulum"},
                                  {"HopperPyBulletEnv-v0", "hopper"},
                                  {"HalfCheetahPyBulletEnv-v0", "halfcheetah"},
                                  {"AntPyBulletEnv-v0", "ant"},
                                  {"HumanoidPyBulletEnv-v0", "humanoid"}};
  for (int i = 0; i < 5; i++)
    if (!strcmp(env_id, ids[i][0]) || !strcmp(env_id, ids[i][1])) return i;
  return -1;
}

// compile-time robot dispatch
template <class F>
int dispatch(int rid, F&& f) {
  switch (rid) {
    case 0: return f(pbg_models::Pendulum{});
    case 1: return f(pbg_models::Hopper{});
    case 2: return f(pbg_models::HalfCheetah{});
    case 3: return f(pbg_models::Ant{});
    case 4: return f(pbg_models::Humanoid{});
  }
  return fail(PBG_E_ENV, "unknown robot id%s %ld", "", rid);
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return PBG_OK;
  return fail(PBG_E_HIP, "%s: HIP error %ld", what, (long)e);
}

inline unsigned grid_of(int n) { return (unsigned)((n + 63) / 64); }

}  // namespace

struct pbg_handle {
  int rid, device, n;
  pbg::Buffers B;
  float* scratch;
  int lds_rows;       // constraint rows kept in LDS per env
  size_t lds_bytes;   // dynamic LDS per 64-lane workgroup
  pbg_info_t info;
};

extern "C" {

const char* pbg_last_error(void) { return g_err; }

#ifdef PBG_STAMPS
// diagnostic build only: read and clear the per-phase wave-cycle sums
int pbg_debug_stamps(unsigned long long* host_out) {
  hipMemcpyFromSymbol(host_out, HIP_SYMBOL(pbg::g_stamps), sizeof(unsigned long long) * 16);
  unsigned long long z[16] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(pbg::g_stamps), z, sizeof(z));
  return 0;
}
#endif

int pbg_create(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset, pbg_handle** out) {
  if (!out) return fail(PBG_E_ARG, "pbg_create: out is NULL%s%ld");
  *out = nullptr;
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_create: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (n_envs <= 0) return fail(PBG_E_ARG, "pbg_create: n_envs must be > 0%s (got %ld)", "", n_envs);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(PBG_E_HIP, "pbg_create: no HIP device %s%ld", "", device);
  DeviceGuard dg(device);
  pbg_handle* h = new (std::nothrow) pbg_handle();
  if (!h) return fail(PBG_E_NOMEM, "pbg_create: out of host memory%s%ld");
  h->rid = rid;
  h->device = device;
  h->n = n_envs;
  int rc = dispatch(rid, [&](auto r) -> int {
    using R = decltype(r);
    const size_t n = (size_t)n_envs;
    pbg_info_t& I = h->info;
    I.robot_id = rid; I.n_envs = n_envs; I.action_dim = R::NA; I.obs_dim = R::OBS; I.n_dof = R::NDOF;
    I.n_joints = R::NJ; I.n_links = R::NL; I.n_feet = R::NF; I.state_words = pbg::Dims<R>::SD;
    I.aux_words = PBG_AUX_WORDS + R::NF; I.substeps = R::substeps; I.max_episode_steps = R::max_episode_steps;
    I.reset_dofs = R::NR; I.floating = R::floating;
    pbg::Buffers& B = h->B;
    B.n = n_envs;
    B.seed = seed;
    B.env_offset = env_offset;
    int e = 0;
    e |= hip_check(hipMalloc(&B.st, sizeof(float) * n * pbg::Dims<R>::SD), "hipMalloc state");
    e |= hip_check(hipMalloc(&B.pot, sizeof(double) * n), "hipMalloc potential");
    e |= hip_check(hipMalloc(&B.z0, sizeof(float) * n), "hipMalloc z0");
    e |= hip_check(hipMalloc(&B.elapsed, sizeof(int) * n), "hipMalloc elapsed");
    e |= hip_check(hipMalloc(&B.flags, sizeof(uint32_t) * n), "hipMalloc flags");
    e |= hip_check(hipMalloc(&B.episode, sizeof(uint32_t) * n), "hipMalloc episode");
    e |= hip_check(hipMalloc(&h->scratch, sizeof(float) * n * pbg::Rows<R>::WORDS), "hipMalloc scratch");
    if (e) return PBG_E_NOMEM;
    e |= hip_check(hipMemset(B.st, 0, sizeof(float) * n * pbg::Dims<R>::SD), "hipMemset");
    e |= hip_check(hipMemset(B.pot, 0, sizeof(double) * n), "hipMemset");
    e |= hip_check(hipMemset(B.z0, 0, sizeof(float) * n), "hipMemset");
    e |= hip_check(hipMemset(B.elapsed, 0, sizeof(int) * n), "hipMemset");
    e |= hip_check(hipMemset(B.flags, 0, sizeof(uint32_t) * n), "hipMemset");
    e |= hip_check(hipMemset(B.episode, 0, sizeof(uint32_t) * n), "hipMemset");
    // LDS budget: all resident waves of a CU share 160 KiB; one wave per workgroup.
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const int waves = (n_envs + 63) / 64;
    const int wpc = (waves + cus - 1) / cus;
    int maxlds = 163840;
    const size_t budget = (size_t)maxlds / (size_t)(wpc > 0 ? wpc : 1);
    using RW = pbg::Rows<R>;
    long words = (long)(budget / (64 * sizeof(float))) - RW::NC;
    int cap = (int)(words / RW::W);
    if (cap > RW::MR) cap = RW::MR;
    if (cap < 0) cap = 0;
    h->lds_rows = cap;
    h->lds_bytes = (size_t)64 * sizeof(float) * ((size_t)cap * RW::W + RW::NC);
    e |= hip_check(hipFuncSetAttribute((const void*)pbg::step_kernel<R>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)h->lds_bytes), "hipFuncSetAttribute");
    e |= hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return e ? PBG_E_HIP : PBG_OK;
  });
  if (rc != PBG_OK) {
    pbg_destroy(h);
    return rc;
  }
  *out = h;
  return PBG_OK;
}

void pbg_destroy(pbg_handle* h) {
  if (!h) return;
  DeviceGuard dg(h->device);
  hipFree(h->B.st);
  hipFree(h->B.pot);
  hipFree(h->B.z0);
  hipFree(h->B.elapsed);
  hipFree(h->B.flags);
  hipFree(h->B.episode);
  hipFree(h->scratch);
  delete h;
}

int pbg_info(const pbg_handle* h, pbg_info_t* out) {
  if (!h || !out) return fail(PBG_E_ARG, "pbg_info: NULL argument%s%ld");
  *out = h->info;
  return PBG_OK;
}

int pbg_reset(pbg_handle* h, const uint8_t* mask, const float* init_q, float* obs, void* stream) {
  if (!h || !obs) return fail(PBG_E_ARG, "pbg_reset: NULL handle or obs%s%ld");
  DeviceGuard dg(h->device);
  pbg::ResetIO io{mask, init_q, obs};
  return dispatch(h->rid, [&](auto r) -> int {
    using R = decltype(r);
    hipLaunchKernelGGL(pbg::reset_kernel<R>, dim3(grid_of(h->n)), dim3(64), 0, (hipStream_t)stream, h->B, io);
    return hip_check(hipGetLastError(), "reset_kernel launch");
  });
}

int pbg_step_ex(pbg_handle* h, const pbg_step_io_t* io, void* stream) {
  if (!h || !io || !io->act || !io->obs || !io->rew || !io->done)
    return fail(PBG_E_ARG, "pbg_step: NULL handle or required buffer%s%ld");
  DeviceGuard dg(h->device);
  pbg::StepIO s{io->act, io->obs, io->rew, io->rew64, io->done, io->trunc, io->term_obs, io->ncontact, io->autoreset};
  return dispatch(h->rid, [&](auto r) -> int {
    using R = decltype(r);
    hipLaunchKernelGGL(pbg::step_kernel<R>, dim3(grid_of(h->n)), dim3(64), h->lds_bytes, (hipStream_t)stream, h->B,
                       s, h->scratch, h->lds_rows);
    return hip_check(hipGetLastError(), "step_kernel launch");
  });
}

int pbg_step(pbg_handle* h, const float* act, float* obs, float* rew, uint8_t* done, void* stream) {
  pbg_step_io_t io;
  memset(&io, 0, sizeof(io));
  io.act = act; io.obs = obs; io.rew = rew; io.done = done;
  return pbg_step_ex(h, &io, stream);
}

int pbg_get_state(pbg_handle* h, double* phys, double* aux, void* stream) {
  if (!h || !phys || !aux) return fail(PBG_E_ARG, "pbg_get_state: NULL argument%s%ld");
  DeviceGuard dg(h->device);
  return dispatch(h->rid, [&](auto r) -> int {
    using R = decltype(r);
    hipLaunchKernelGGL(pbg::get_state_kernel<R>, dim3(grid_of(h->n)), dim3(64), 0, (hipStream_t)stream, h->B, phys, aux);
    return hip_check(hipGetLastError(), "get_state launch");
  });
}

int pbg_set_state(pbg_handle* h, const double* phys, const double* aux, void* stream) {
  if (!h || !phys) return fail(PBG_E_ARG, "pbg_set_state: NULL argument%s%ld");
  DeviceGuard dg(h->device);
  return dispatch(h->rid, [&](auto r) -> int {
    using R = decltype(r);
    hipLaunchKernelGGL(pbg::set_state_kernel<R>, dim3(grid_of(h->n)), dim3(64), 0, (hipStream_t)stream, h->B, phys, aux);
    return hip_check(hipGetLastError(), "set_state launch");
  });
}

int pbg_pack_record_sizes(const char* env_id, int* in_words, int* out_words) {
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_pack_record_sizes: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  return dispatch(rid, [&](auto r) -> int {
    using R = decltype(r);
    if (in_words) *in_words = pbg::PackRec<R>::IN;
    if (out_words) *out_words = pbg::PackRec<R>::OUT;
    return PBG_OK;
  });
}

int pbg_pack(const char* env_id, int n, const double* in_rec, double* out_rec, void* stream) {
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_pack: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (n <= 0 || !in_rec || !out_rec) return fail(PBG_E_ARG, "pbg_pack: bad arguments%s%ld");
  return dispatch(rid, [&](auto r) -> int {
    using R = decltype(r);
    hipLaunchKernelGGL(pbg::pack_kernel<R>, dim3(grid_of(n)), dim3(64), 0, (hipStream_t)stream, n, in_rec, out_rec);
    return hip_check(hipGetLastError(), "pack_kernel launch");
  });
}

}  // extern "C"
