// pbg_capi.hip -- the C-ABI (include/pbg.h).  Owns handles and device buffers and
// dispatches to the per-robot launchers of pbg_robot.hip (one translation unit each).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "../../include/pbg.h"
#include "models_gen.h"
#include "pbg_launch.h"
#include "pbg_records.h"
#include "pbg_math.h"
#include "pbg_types.h"
#include "sim_params.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* a = "", long b = 0) {
  snprintf(g_err, sizeof(g_err), fmt, a, b);
  return code;
}

int env_robot_id(const char* env_id) {
  if (!env_id) return -1;
  static const char* ids[17][2] = {{"InvertedPendulumPyBulletEnv-v0", "pendulum"},
                                  {"HopperPyBulletEnv-v0", "hopper"},
                                  {"HalfCheetahPyBulletEnv-v0", "halfcheetah"},
                                  {"AntPyBulletEnv-v0", "ant"},
                                  {"HumanoidPyBulletEnv-v0", "humanoid"},
                                  {"Walker2DPyBulletEnv-v0", "walker2d"},
                                  {"InvertedPendulumSwingupPyBulletEnv-v0", "pendulum_swingup"},
                                  {"InvertedDoublePendulumPyBulletEnv-v0", "double_pendulum"},
                                  {"HumanoidFlagrunPyBulletEnv-v0", "humanoid_flagrun"},
                                  {"HopperMuJoCoEnv-v0", "hopper_mujoco"},
                                  {"Walker2DMuJoCoEnv-v0", "walker2d_mujoco"},
                                  {"HalfCheetahMuJoCoEnv-v0", "halfcheetah_mujoco"},
                                  {"AntMuJoCoEnv-v0", "ant_mujoco"},
                                  {"HumanoidMuJoCoEnv-v0", "humanoid_mujoco"},
                                  {"InvertedDoublePendulumMuJoCoEnv-v0", "double_pendulum_mujoco"},
                                  {"HumanoidFlagrunHarderPyBulletEnv-v0", "humanoid_flagrun_harder"},
                                  {"AtlasPyBulletEnv-v0", "atlas"}};
  for (int i = 0; i < 17; i++)
    if (!strcmp(env_id, ids[i][0]) || !strcmp(env_id, ids[i][1])) return i;
  return -1;
}

// The per-robot kernels of one precision (pbg_robot.hip)
struct Kern {
  int (*plan)(int, int, int, pbg::Geometry*);
  int (*step)(const pbg::Buffers&, const pbg::StepIO&, float*, const pbg::Geometry&, hipStream_t);
  int (*reset)(const pbg::Buffers&, const pbg::ResetIO&, hipStream_t);
  int (*get_state)(const pbg::Buffers&, double*, double*, hipStream_t);
  int (*set_state)(const pbg::Buffers&, const double*, const double*, hipStream_t);
};
struct Ops {
  Kern k32, k64;  // float32 kernels; the float64 (reference-precision) kernels
  int (*pack)(int, const double*, double*, hipStream_t);
  pbg_info_t info;
  int pack_in, pack_out;
  pbg_sim_params_t defaults;
};

template <class R>
pbg_info_t info_of(int rid) {
  pbg_info_t I;
  I.robot_id = rid; I.n_envs = 0; I.action_dim = R::NA; I.obs_dim = R::OBS; I.n_dof = R::NDOF;
  I.n_joints = R::NJ; I.n_links = R::NL; I.n_feet = R::NF; I.state_words = pbg::Records<R>::SD;
  I.aux_words = pbg::Records<R>::AD; I.substeps = R::substeps; I.max_episode_steps = R::max_episode_steps;
  I.reset_dofs = R::NR; I.floating = R::floating;
  I.record_version = PBG_RECORD_VERSION;
  return I;
}

// the scene the reference's env builds (include/pbg.h pbg_sim_params_t)
template <class R>
pbg_sim_params_t defaults_of() {
  pbg_sim_params_t p;
  p.gravity = PBG_GRAVITY;
  p.timestep = R::dt_sub;
  p.frame_skip = R::substeps;
  p.solver_iterations = PBG_SOLVER_ITERATIONS;
  p.contact_erp = R::contact_erp;
  p.joint_limit_erp = PBG_LIMIT_ERP;
  return p;
}

int check_sim_params(const pbg_sim_params_t& p) {
  if (!isfinite(p.gravity) || fabs(p.gravity) > 1000.0)
    return fail(PBG_E_ARG, "pbg_create: gravity must be finite with |gravity| <= 1000%s%ld");
  if (!(p.timestep > 0.0 && p.timestep <= 0.1))
    return fail(PBG_E_ARG, "pbg_create: timestep must be in (0, 0.1]%s%ld");
  if (p.frame_skip < 1 || p.frame_skip > 64)
    return fail(PBG_E_ARG, "pbg_create: frame_skip must be in 1..64%s (got %ld)", "", p.frame_skip);
  if (p.solver_iterations < 1 || p.solver_iterations > 1000)
    return fail(PBG_E_ARG, "pbg_create: solver_iterations must be in 1..1000%s (got %ld)", "", p.solver_iterations);
  if (!(p.contact_erp >= 0.0 && p.contact_erp <= 1.0) || !(p.joint_limit_erp >= 0.0 && p.joint_limit_erp <= 1.0))
    return fail(PBG_E_ARG, "pbg_create: contact_erp and joint_limit_erp must be in [0, 1]%s%ld");
  return PBG_OK;
}

#define PBG_OPS(NAME, RID)                                                                                   \
  Ops{Kern{pbg::plan_##NAME, pbg::launch_step_##NAME, pbg::launch_reset_##NAME, pbg::launch_get_state_##NAME,  \
           pbg::launch_set_state_##NAME},                                                                    \
      Kern{pbg::plan64_##NAME, pbg::launch_step64_##NAME, pbg::launch_reset64_##NAME,                        \
           pbg::launch_get_state64_##NAME, pbg::launch_set_state64_##NAME},                                  \
      pbg::launch_pack_##NAME, info_of<pbg_models::NAME>(RID), pbg::PackRec<pbg_models::NAME>::IN,          \
      pbg::PackRec<pbg_models::NAME>::OUT, defaults_of<pbg_models::NAME>()}

const Ops* ops(int rid) {
  static const Ops table[17] = {PBG_OPS(Pendulum, 0), PBG_OPS(Hopper, 1), PBG_OPS(HalfCheetah, 2), PBG_OPS(Ant, 3),
                                PBG_OPS(Humanoid, 4), PBG_OPS(Walker2D, 5), PBG_OPS(PendulumSwingup, 6),
                                PBG_OPS(DoublePendulum, 7), PBG_OPS(HumanoidFlagrun, 8), PBG_OPS(HopperMuJoCo, 9),
                                PBG_OPS(Walker2DMuJoCo, 10), PBG_OPS(HalfCheetahMuJoCo, 11), PBG_OPS(AntMuJoCo, 12),
                                PBG_OPS(HumanoidMuJoCo, 13), PBG_OPS(DoublePendulumMuJoCo, 14),
                                PBG_OPS(HumanoidFlagrunHarder, 15), PBG_OPS(Atlas, 16)};
  return (rid >= 0 && rid < 17) ? &table[rid] : nullptr;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

int hip_check(int e, const char* what) {
  if (e == (int)hipSuccess) return PBG_OK;
  return fail(PBG_E_HIP, "%s: HIP error %ld", what, (long)e);
}

// The device that owns a device buffer (entry points without a handle launch there, whatever
// the caller's current device is); -1 when the pointer is not device memory.
int device_of(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ? a.device : -1;
}

}  // namespace

struct pbg_handle {
  int rid, device, n;
  int precision;  // 32 or 64 (pbg_create_v2)
  const Ops* ops;
  const Kern* k;  // the kernels of that precision
  pbg::Buffers B;
  float* scratch;
  pbg::Geometry geo;
  pbg_info_t info;
  pbg_sim_params_t params;
};

extern "C" {

const char* pbg_last_error(void) { return g_err; }

int pbg_default_sim_params(const char* env_id, pbg_sim_params_t* out) {
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_default_sim_params: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (!out) return fail(PBG_E_ARG, "pbg_default_sim_params: out is NULL%s%ld");
  *out = ops(rid)->defaults;
  return PBG_OK;
}

int pbg_create(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset, pbg_handle** out) {
  return pbg_create_ex(env_id, n_envs, device, seed, env_offset, nullptr, nullptr, out);
}

int pbg_create_debug(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                     const pbg_debug_opts_t* opts, pbg_handle** out) {
  return pbg_create_ex(env_id, n_envs, device, seed, env_offset, nullptr, opts, out);
}

int pbg_create_ex(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                  const pbg_sim_params_t* params, const pbg_debug_opts_t* opts, pbg_handle** out) {
  pbg_create_opts_t o;
  memset(&o, 0, sizeof(o));
  o.struct_size = (uint32_t)sizeof(o);
  o.precision = 64;
  o.kernel = opts ? opts->kernel : -1;
  o.lds_rows = opts ? opts->lds_rows : -1;
  o.gang_dist = opts ? opts->gang_dist : -1;
  o.gang_lanes = opts ? opts->gang_lanes : -1;
  return pbg_create_v2(env_id, n_envs, device, seed, env_offset, params, &o, out);
}

int pbg_create_v2(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                  const pbg_sim_params_t* params, const pbg_create_opts_t* copts, pbg_handle** out) {
  if (!out) return fail(PBG_E_ARG, "pbg_create: out is NULL%s%ld");
  *out = nullptr;  // every failure below leaves the caller's handle NULL
  // versioned options: read only the fields the caller's struct holds (struct_size, a whole number of
  // the struct's 4-byte fields); absent fields = defaults
  pbg_create_opts_t co;
  memset(&co, 0, sizeof(co));
  co.precision = 64; co.kernel = -1; co.lds_rows = -1; co.gang_dist = -1; co.gang_lanes = -1;
  if (copts) {
    if (copts->struct_size < (uint32_t)(2 * sizeof(uint32_t)) || copts->struct_size > (uint32_t)sizeof(co) ||
        copts->struct_size % 4u != 0u)
      return fail(PBG_E_ARG, "pbg_create_v2: opts->struct_size %s%ld is not a pbg_create_opts_t size", "",
                  (long)copts->struct_size);
    memcpy(&co, copts, copts->struct_size);
  }
  if (co.precision != 32 && co.precision != 64)
    return fail(PBG_E_ARG, "pbg_create_v2: precision must be 32 or 64%s (got %ld)", "", co.precision);
  const pbg_debug_opts_t dbg = {co.kernel, co.lds_rows, co.gang_dist, co.gang_lanes};
  const pbg_debug_opts_t* opts = &dbg;
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_create: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (n_envs <= 0) return fail(PBG_E_ARG, "pbg_create: n_envs must be > 0%s (got %ld)", "", n_envs);
  const pbg_sim_params_t sp = params ? *params : ops(rid)->defaults;
  if (check_sim_params(sp)) return PBG_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(PBG_E_HIP, "pbg_create: no HIP device %s%ld", "", device);
  DeviceGuard dg(device);
  pbg_handle* h = new (std::nothrow) pbg_handle();
  if (!h) return fail(PBG_E_NOMEM, "pbg_create: out of host memory%s%ld");
  const Ops* o = ops(rid);
  h->rid = rid;
  h->device = device;
  h->n = n_envs;
  h->precision = co.precision;
  h->ops = o;
  h->k = co.precision == 64 ? &o->k64 : &o->k32;
  h->info = o->info;
  h->info.n_envs = n_envs;
  h->info.substeps = sp.frame_skip;
  h->params = sp;
  pbg::Buffers& B = h->B;
  B.n = n_envs;
  B.seed = seed;
  B.env_offset = env_offset;
  B.sp = pbg::resolve_sim_params<float>(sp.timestep, sp.frame_skip, sp.solver_iterations, sp.gravity, sp.contact_erp,
                                        sp.joint_limit_erp, PBG_ANGULAR_MOTION_THRESHOLD);
  B.sp64 = pbg::resolve_sim_params<double>(sp.timestep, sp.frame_skip, sp.solver_iterations, sp.gravity,
                                           sp.contact_erp, sp.joint_limit_erp, PBG_ANGULAR_MOTION_THRESHOLD);
  const size_t n = (size_t)n_envs;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  // kernel variant: 1 = default (quad for Ant, gang for the other walkers), 0 = the
  // one-lane-per-env kernel for every robot, 2 = the gang kernel for every walker
  const int mode = (opts && (opts->kernel == 0 || opts->kernel == 2)) ? opts->kernel : 1;
  h->geo.force_dist = opts ? opts->gang_dist : -1;
  h->geo.gang_lanes = (opts && (opts->gang_lanes == 16 || opts->gang_lanes == 32)) ? opts->gang_lanes : -1;
  int e = hip_check(h->k->plan(n_envs, cus, mode, &h->geo), "kernel attributes");
  // diagnostic options that the chosen kernel cannot honour are refused, not ignored: an A/B
  // run must never measure another kernel than the one it asked for.  Checked before any plan failure is
  // reported, so an option's refusal is PBG_E_ARG in both precisions.
  const char* bad = nullptr;
  if (opts->kernel == 0 && (e || h->geo.team != 1))
    bad = "kernel = 0: this robot has no lane-per-env kernel (Atlas' 886 contact slots)";
  else if (!e && opts->gang_lanes == 32 && h->geo.team != 32)
    bad = "gang_lanes = 32 needs the 32-lane gang kernel (the Humanoid family on the default / gang plan)";
  else if (e && opts->gang_lanes == 32)
    bad = "gang_lanes = 32: this robot has no 32-lane gang kernel";
  else if (!e && opts->gang_lanes == 16 && h->geo.team != 16)
    bad = "gang_lanes = 16 needs a gang plan (kernel = 0 and Ant's quad plan are not gang kernels)";
  else if (!e && (opts->gang_dist == 0 || opts->gang_dist == 1) && h->geo.team < 16)
    bad = "gang_dist applies to the gang kernel only";
  else if (!e && (opts->gang_dist == 0 || opts->gang_dist == 1) && h->geo.gang_dist != opts->gang_dist)
    bad = "gang_dist: this robot / gang width has no replicated-dynamics variant";
  if (bad) {
    snprintf(g_err, sizeof(g_err), "pbg_create: %s", bad);
    delete h;
    return PBG_E_ARG;
  }
  if (e) {
    snprintf(g_err, sizeof(g_err), "pbg_create: no float%d kernel plan for %s at %d envs (HIP error %d)",
             co.precision, env_id, n_envs, e);
    delete h;
    return PBG_E_HIP;
  }
  // cap on the LDS-resident contact rows (tests of the device-workspace path)
  if (opts && opts->lds_rows >= 0 && opts->lds_rows < h->geo.lds_rows) h->geo.lds_rows = opts->lds_rows;
  const size_t wb = co.precision == 64 ? sizeof(double) : sizeof(float);  // state / z0 / workspace word
  e |= hip_check(hipMalloc(&B.st, wb * n * h->info.state_words), "hipMalloc state");
  e |= hip_check(hipMalloc(&B.pot, sizeof(double) * n), "hipMalloc potential");
  e |= hip_check(hipMalloc(&B.z0, wb * n), "hipMalloc z0");
  e |= hip_check(hipMalloc(&B.elapsed, sizeof(int) * n), "hipMalloc elapsed");
  e |= hip_check(hipMalloc(&B.flags, sizeof(uint32_t) * n), "hipMalloc flags");
  e |= hip_check(hipMalloc(&B.episode, sizeof(uint32_t) * n), "hipMalloc episode");
  e |= hip_check(hipMalloc(&B.tgt, sizeof(double) * 2 * n), "hipMalloc walk target");
  e |= hip_check(hipMalloc(&B.ftm, sizeof(int32_t) * 2 * n), "hipMalloc flag counters");
  e |= hip_check(hipMalloc(&B.hkd, sizeof(double) * 2 * n), "hipMalloc crawl potentials");
  e |= hip_check(hipMalloc(&B.hki, sizeof(int32_t) * 3 * n), "hipMalloc cube counters");
  e |= hip_check(hipMalloc(&h->scratch, (size_t)h->geo.word_bytes * n * h->geo.scratch_words_per_env), "hipMalloc scratch");
  if (!e) {
    e |= hip_check(hipMemset(B.st, 0, wb * n * h->info.state_words), "hipMemset");
    e |= hip_check(hipMemset(B.pot, 0, sizeof(double) * n), "hipMemset");
    e |= hip_check(hipMemset(B.z0, 0, wb * n), "hipMemset");
    e |= hip_check(hipMemset(B.elapsed, 0, sizeof(int) * n), "hipMemset");
    e |= hip_check(hipMemset(B.flags, 0, sizeof(uint32_t) * n), "hipMemset");
    e |= hip_check(hipMemset(B.episode, 0, sizeof(uint32_t) * n), "hipMemset");
    e |= hip_check(hipMemset(B.tgt, 0, sizeof(double) * 2 * n), "hipMemset");
    e |= hip_check(hipMemset(B.ftm, 0, sizeof(int32_t) * 2 * n), "hipMemset");
    e |= hip_check(hipMemset(B.hkd, 0, sizeof(double) * 2 * n), "hipMemset");
    e |= hip_check(hipMemset(B.hki, 0, sizeof(int32_t) * 3 * n), "hipMemset");
    e |= hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  if (e) {
    pbg_destroy(h);
    return PBG_E_HIP;
  }
  *out = h;
  return PBG_OK;
}

void pbg_destroy(pbg_handle* h) {
  if (!h) return;
  DeviceGuard dg(h->device);
  void* bufs[] = {h->B.st, h->B.pot, h->B.z0, h->B.elapsed, h->B.flags, h->B.episode, h->B.tgt, h->B.ftm,
                  h->B.hkd, h->B.hki, h->scratch};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  delete h;
}

int pbg_get_sim_params(const pbg_handle* h, pbg_sim_params_t* out) {
  if (!h || !out) return fail(PBG_E_ARG, "pbg_get_sim_params: NULL argument%s%ld");
  *out = h->params;
  return PBG_OK;
}

int pbg_precision(const pbg_handle* h) { return h ? h->precision : PBG_E_ARG; }

int pbg_info(const pbg_handle* h, pbg_info_t* out) {
  if (!h || !out) return fail(PBG_E_ARG, "pbg_info: NULL argument%s%ld");
  *out = h->info;
  out->lanes_per_env = h->geo.team;
  out->block = h->geo.block;
  out->lds_bytes = (int)h->geo.lds_bytes;
  out->vgprs = h->geo.vgprs;
  out->scratch_bytes = h->geo.scratch_bytes;
  out->lds_rows = h->geo.lds_rows;
  return PBG_OK;
}

int pbg_reset(pbg_handle* h, const uint8_t* mask, const float* init_q, float* obs, void* stream) {
  if (!h || !obs) return fail(PBG_E_ARG, "pbg_reset: NULL handle or obs%s%ld");
  DeviceGuard dg(h->device);
  pbg::ResetIO io{mask, init_q, obs};
  return hip_check(h->k->reset(h->B, io, (hipStream_t)stream), "reset_kernel launch");
}

int pbg_step_ex(pbg_handle* h, const pbg_step_io_t* io, void* stream) {
  if (!h || !io || !io->act || !io->obs || !io->rew || !io->done)
    return fail(PBG_E_ARG, "pbg_step: NULL handle or required buffer%s%ld");
  DeviceGuard dg(h->device);
  pbg::StepIO s{io->act, io->obs, io->rew, io->rew64, io->done, io->trunc, io->term_obs, io->ncontact, io->autoreset,
                io->rew_terms, io->csig};
  return hip_check(h->k->step(h->B, s, h->scratch, h->geo, (hipStream_t)stream), "step_kernel launch");
}

int pbg_step(pbg_handle* h, const float* act, float* obs, float* rew, uint8_t* done, void* stream) {
  pbg_step_io_t io;
  memset(&io, 0, sizeof(io));
  io.act = act;
  io.obs = obs;
  io.rew = rew;
  io.done = done;
  return pbg_step_ex(h, &io, stream);
}

int pbg_get_state(pbg_handle* h, double* phys, double* aux, void* stream) {
  if (!h || !phys || !aux) return fail(PBG_E_ARG, "pbg_get_state: NULL argument%s%ld");
  DeviceGuard dg(h->device);
  return hip_check(h->k->get_state(h->B, phys, aux, (hipStream_t)stream), "get_state launch");
}

int pbg_set_state(pbg_handle* h, const double* phys, const double* aux, void* stream) {
  if (!h || !phys) return fail(PBG_E_ARG, "pbg_set_state: NULL argument%s%ld");
  DeviceGuard dg(h->device);
  return hip_check(h->k->set_state(h->B, phys, aux, (hipStream_t)stream), "set_state launch");
}

int pbg_pack_record_sizes(const char* env_id, int* in_words, int* out_words) {
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_pack_record_sizes: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (in_words) *in_words = ops(rid)->pack_in;
  if (out_words) *out_words = ops(rid)->pack_out;
  return PBG_OK;
}

#ifdef PBG_STAMPS
// diagnostic build only: read and clear the per-phase wave-cycle sums of one robot's kernel
int pbg_debug_stamps(int rid, unsigned long long* host_out) {
  using F = int (*)(unsigned long long*);
  static const F table[17] = {pbg::debug_stamps_Pendulum, pbg::debug_stamps_Hopper, pbg::debug_stamps_HalfCheetah,
                              pbg::debug_stamps_Ant, pbg::debug_stamps_Humanoid, pbg::debug_stamps_Walker2D,
                              pbg::debug_stamps_PendulumSwingup, pbg::debug_stamps_DoublePendulum,
                              pbg::debug_stamps_HumanoidFlagrun, pbg::debug_stamps_HopperMuJoCo,
                              pbg::debug_stamps_Walker2DMuJoCo, pbg::debug_stamps_HalfCheetahMuJoCo,
                              pbg::debug_stamps_AntMuJoCo, pbg::debug_stamps_HumanoidMuJoCo,
                              pbg::debug_stamps_DoublePendulumMuJoCo, pbg::debug_stamps_HumanoidFlagrunHarder,
                              pbg::debug_stamps_Atlas};
  return (rid >= 0 && rid < 17) ? table[rid](host_out) : PBG_E_ENV;
}
#endif

// Batched action_space.sample(): out[s][e][i] = U(-1, 1) float32, Philox4x32-10 keyed by the
// seed, counter (step0 + s, env_offset + e, 4-wide block of i, 0xAC7), u = (r >> 8) / 2^24.
__global__ __launch_bounds__(256) void sample_actions_kernel(int na, int n, int steps, uint32_t k0, uint32_t k1,
                                                             uint32_t step0, int env_offset, float* __restrict__ out) {
  const int nb = (na + 3) / 4;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one (step, env, block) per lane
  if (idx >= (long)steps * n * nb) return;
  const int blk = (int)(idx % nb);
  const long se = idx / nb;
  const int e = (int)(se % n), st = (int)(se / n);
  u4 ctr = {step0 + (uint32_t)st, (uint32_t)(env_offset + e), (uint32_t)blk, 0xAC7u};
  const u4 r = philox4x32_10(ctr, k0, k1);
  const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
  float* o = out + ((size_t)st * n + e) * na;
#pragma unroll
  for (int t = 0; t < 4; t++)
    if (4 * blk + t < na) o[4 * blk + t] = fmaf(2.f, u01(rr[t]), -1.f);
}

int pbg_sample_actions(int action_dim, int n_envs, int n_steps, uint64_t seed, uint32_t step0, int env_offset,
                       float* out, void* stream) {
  if (action_dim <= 0 || n_envs <= 0 || n_steps <= 0 || !out)
    return fail(PBG_E_ARG, "pbg_sample_actions: bad arguments%s%ld");
  const int dev = device_of(out);
  if (dev < 0) return fail(PBG_E_ARG, "pbg_sample_actions: out is not device memory%s%ld");
  DeviceGuard dg(dev);
  const long lanes = (long)n_steps * n_envs * ((action_dim + 3) / 4);
  hipLaunchKernelGGL(sample_actions_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     action_dim, n_envs, n_steps, (uint32_t)seed, (uint32_t)(seed >> 32), step0, env_offset, out);
  return hip_check((int)hipGetLastError(), "sample_actions launch");
}

// Test support (pbg_debug_poison): fill a whole CU's LDS with a 32-bit pattern, so the next kernel's
// workgroups on that CU start on it instead of on whatever an earlier kernel left there
__global__ __launch_bounds__(256) void poison_lds_kernel(uint32_t pattern) {
  extern __shared__ uint32_t lds_poison[];
  for (int i = threadIdx.x; i < 163840 / 4; i += 256) lds_poison[i] = pattern;
  __syncthreads();
}

int pbg_debug_poison(pbg_handle* h, uint32_t pattern, void* stream) {
  int dev = 0;
  if (h) dev = h->device;
  else if (hipGetDevice(&dev) != hipSuccess) return fail(PBG_E_HIP, "pbg_debug_poison: no device%s%ld");
  DeviceGuard dg(dev);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return fail(PBG_E_HIP, "pbg_debug_poison: no CU count%s%ld");
  int e = hip_check((int)hipFuncSetAttribute((const void*)poison_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             163840), "poison attribute");
  if (e) return e;
  // one 160 KB workgroup fills a CU; 8 per CU reach every CU of every XCD whatever the dispatch order
  hipLaunchKernelGGL(poison_lds_kernel, dim3((unsigned)(8 * cus)), dim3(256), 163840, (hipStream_t)stream, pattern);
  e = hip_check((int)hipGetLastError(), "poison launch");
  if (e || !h) return e;
  const size_t words = (size_t)h->geo.word_bytes * (size_t)h->B.n * (size_t)h->geo.scratch_words_per_env / 4;
  if (words) e = hip_check((int)hipMemsetD32Async((hipDeviceptr_t)h->scratch, (int)pattern, words, (hipStream_t)stream),
                           "poison workspace");
  return e;
}

int pbg_pack(const char* env_id, int n, const double* in_rec, double* out_rec, void* stream) {
  const int rid = env_robot_id(env_id);
  if (rid < 0) return fail(PBG_E_ENV, "pbg_pack: unknown env id '%s'%ld", env_id ? env_id : "(null)");
  if (n <= 0 || !in_rec || !out_rec) return fail(PBG_E_ARG, "pbg_pack: bad arguments%s%ld");
  const int dev = device_of(out_rec);
  if (dev < 0 || device_of(in_rec) != dev)
    return fail(PBG_E_ARG, "pbg_pack: in_rec / out_rec are not device memory of one GPU%s%ld");
  DeviceGuard dg(dev);
  return hip_check(ops(rid)->pack(n, in_rec, out_rec, (hipStream_t)stream), "pack_kernel launch");
}

}  // extern "C"
