// pbg_robot.hip -- per-robot kernel instantiations + launchers.  Compiled once per robot
// with -DPBG_ROBOT=<Pendulum|Hopper|HalfCheetah|Ant|Humanoid>.
#include <hip/hip_runtime.h>

#include "pbg_launch.h"
#include "pbg_step.hip"
#include "pbg_team.hip"
#include "pbg_gang.hip"

#ifndef PBG_ROBOT
#error "compile with -DPBG_ROBOT=<robot struct name>"
#endif
#define PBG_CAT2(a, b) a##b
#define PBG_CAT(a, b) PBG_CAT2(a, b)
#define PBG_FN(prefix) PBG_CAT(prefix, PBG_ROBOT)

namespace pbg {
using R = pbg_models::PBG_ROBOT;
using R64 = F64<R>;
using R64L = F64L<R>;  // the float64 lane kernel's robot (library sin / cos: pbg_types.h)

static inline unsigned blocks(int n, int b) { return (unsigned)((n + b - 1) / b); }

// registers / private segment of the step kernel a plan selected (pbg_info occupancy)
static int kernel_attrs(const void* fn, Geometry* g) {
  hipFuncAttributes a{};
  const hipError_t e = hipFuncGetAttributes(&a, fn);
  g->vgprs = e == hipSuccess ? a.numRegs : -1;
  g->scratch_bytes = e == hipSuccess ? (int)a.localSizeBytes : -1;
  return (int)e;
}

// Geometry: one env per lane, one wave per workgroup.  With fewer than 64 envs per CU
// the workgroup shrinks to 32 or 16 active lanes so every CU gets a wave (the step is
// issue/latency bound: a wave's time barely depends on its active lanes).  All resident
// workgroups of a CU share the 160 KiB LDS for their constraint rows.
// Team geometry (pbg_team.hip): 4 lanes per env, 16 envs per one-wave workgroup; the
// per-env LDS holds [mu | owner | contact rows], rows past the capacity spill to the
// device workspace.
template <class RR>
static int plan_team(int n_envs, int cus, Geometry* g) {
  if constexpr (Team<RR>::ok) {
    using RW = TRows<RR, 16>;
    constexpr int ES = 16;
    constexpr size_t WB = sizeof(real_t<RR>);  // row word: float, or double on the float64 path
    const int wgs = (n_envs + ES - 1) / ES;
    const int wpc = (wgs + cus - 1) / cus;
    const size_t budget = (size_t)163840 / (size_t)(wpc > 0 ? wpc : 1);
    long words = (long)(budget / ((size_t)ES * WB)) - RW::HEAD;
    int cap = (int)(words / RW::W);
    if (cap > RW::MR) cap = RW::MR;
    if (cap < 0) cap = 0;
    size_t per_env = (size_t)RW::HEAD + (size_t)cap * RW::W;
    if (per_env < (size_t)(2 * RR::NL + 2 * RR::NJ)) per_env = 2 * RR::NL + 2 * RR::NJ;  // pack staging
    g->team = 4;
    g->env_words = 0;
    g->block = 64;
    g->lds_rows = cap;
    g->lds_bytes = (size_t)ES * WB * per_env;
    g->scratch_words_per_env = RW::WORDS;
    g->word_bytes = (int)WB;
    const void* fn = (const void*)team_step_kernel<RR, 16>;
    const int e = (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes);
    return e ? e : kernel_attrs(fn, g);
  } else {
    (void)n_envs; (void)cus; (void)g;
    return (int)hipErrorInvalidValue;
  }
}
template <class RR>
static bool launch_team(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if constexpr (Team<RR>::ok) {
    if (g.team != 4) return false;
    hipLaunchKernelGGL((team_step_kernel<RR, 16>), dim3(blocks(4 * B.n, 64)), dim3(64), g.lds_bytes, s, B, io, scratch,
                       g.lds_rows);
    return true;
  } else {
    (void)B; (void)io; (void)scratch; (void)g; (void)s;
    return false;
  }
}

// robots and widths with a gang kernel: walkers (the cube robot on the front path); 32-lane gangs for
// the Humanoid family (float64: its default width, a wave on every SIMD of a CU whose LDS holds 8
// float64 envs); float64 (F64<R>): Atlas-sized models excluded
template <class RR, int T>
constexpr bool gang_ok() {
  constexpr bool f64 = sizeof(real_t<RR>) == 8;
  return (RR::kind == 0 || RR::kind >= 2) && (!RR::harder || FP<RR>::NF > 0) && (T == 16 || gang32_ok<RR>()) &&
         !(f64 && gang_big<RR>() && T != 16);
}
// Gang geometry (pbg_gang.hip): T = 16 or 32 lanes per env, 256 / T envs per 4-wave workgroup;
// the per-env LDS region holds the staged dynamics, limit rows and `cap` contacts (descriptor
// + 3 rows), contacts past the capacity spill to the device workspace.
// the replicated-dynamics variant (the whole dynamics per lane, no distributed mass matrix): float32
// walkers, and the float64 robots under 8 dofs (Hopper: 512 registers, no spill, -4.5 % at 4,096 envs;
// the float64 HalfCheetah / Walker2D variants spill 1.2-1.3 KB and run 2.1-2.5x slower,
// profiles/r06_ab_f64_repl.txt)
template <class RR, int T>
constexpr bool gang_repl() {
  return T == 16 && !RR::harder && (sizeof(real_t<RR>) == 4 || RR::NDOF < 8);
}
template <class RR, int T>
static int plan_gang_t(int n_envs, int cus, Geometry* g) {
  if constexpr (gang_ok<RR, T>()) {
    using G = Gang<RR, T>;
    constexpr long WB = (long)sizeof(real_t<RR>);  // env-region word: 4 bytes, or 8 on the float64 path
    constexpr int EPB = gang_block<RR, T>() / T;  // envs per workgroup
    // the layout's floor (fixed words + the kinematic area, no LDS contact) must fit one CU's LDS
    static_assert(4L * GangTabs<RR>::WORDS + WB * EPB * ((G::FIXED + G::MIN_CONTACT_WORDS + 3L) & ~3L) <= 163840L,
                  "gang env regions exceed the CU's LDS");
    // every env region 16-byte (front path: b128 LDS loads) or 8-byte (b64 row loads) aligned:
    // round the region up, and give back a contact when the rounding crosses the budget
    auto region = [&](int c) {
      const int w = G::FIXED + (c * G::PERC > G::MIN_CONTACT_WORDS ? c * G::PERC : G::MIN_CONTACT_WORDS);
      return (w + G::REGION_ALIGN - 1) & ~(G::REGION_ALIGN - 1);
    };
    const int wgs = (n_envs + EPB - 1) / EPB;
    int wpc = (wgs + cus - 1) / cus;
    // the workgroups a CU can hold at all (no LDS contact): planning the contact capacity for more
    // resident workgroups than fit would shrink it for nothing (round 5: float64 HalfCheetah and
    // Humanoid, Atlas -- one workgroup per CU, planned for two, had no LDS contact)
    const long fit0 = 163840L / (4L * (long)GangTabs<RR>::WORDS + WB * EPB * (long)region(0));
    if (wpc > fit0) wpc = fit0 > 0 ? (int)fit0 : 1;
    // signed: with many workgroups per CU the share can be smaller than the model tables
    long budget = 163840L / (long)(wpc > 0 ? wpc : 1) - 4L * (long)GangTabs<RR>::WORDS;
    if (budget < 0) budget = 0;
    long words = budget / (long)(EPB * WB) - G::FIXED;
    int cap = (int)(words / G::PERC);
    if (cap > G::MAXC) cap = G::MAXC;
    if (cap < 0) cap = 0;
    while (cap > 0 && (long)region(cap) * EPB * WB > budget) cap--;
    // distributed dynamics from 8 dofs (Walker2D, HalfCheetah, Humanoid: round-2 A/B) or more than one wave per SIMD (its
    // smaller register footprint lets two waves share a SIMD); replicated otherwise
    constexpr bool REPL = gang_repl<RR, T>();  // has a replicated variant
    g->gang_dist = !REPL || RR::NDOF >= 8 || (size_t)n_envs * T > (size_t)64 * 4 * cus;
    // pbg_create_debug (32-lane gangs, the cube robot and float64 from 8 dofs have no replicated-dynamics variant)
    if ((g->force_dist == 0 || g->force_dist == 1) && REPL) g->gang_dist = g->force_dist;
    g->team = T;
    g->block = gang_block<RR, T>();
    g->lds_rows = cap;
    g->env_words = region(cap);
    g->lds_bytes = 4 * (size_t)GangTabs<RR>::WORDS + (size_t)WB * (size_t)EPB * (size_t)g->env_words;
    // the workgroup's regions must fit the CU's LDS (the contact floor MIN_CONTACT_WORDS is the only
    // term the budget does not bound: a model whose tables + floor exceed it is not launchable)
    if (g->lds_bytes > (size_t)163840) return (int)hipErrorInvalidConfiguration;
    g->scratch_words_per_env = G::GWORDS;
    g->word_bytes = (int)WB;
    const void* fn;
    if constexpr (REPL)
      fn = g->gang_dist ? (const void*)gang_step_kernel<RR, T, true> : (const void*)gang_step_kernel<RR, T, false>;
    else
      fn = (const void*)gang_step_kernel<RR, T, true>;
    const int e = (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes);
    return e ? e : kernel_attrs(fn, g);
  } else {
    (void)n_envs; (void)cus; (void)g;
    return (int)hipErrorInvalidValue;
  }
}
// lanes: 16 or 32 (pbg_create_debug gang_lanes), -1: the plan's choice
template <class RR>
static int plan_gang(int n_envs, int cus, Geometry* g, int lanes) {
  if (lanes < 0) lanes = 16;
  if (lanes == 32) return plan_gang_t<RR, 32>(n_envs, cus, g);
  return plan_gang_t<RR, 16>(n_envs, cus, g);
}
template <class RR, int T>
static bool launch_gang_t(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if constexpr (gang_ok<RR, T>()) {
    const dim3 grid(blocks(B.n, gang_block<RR, T>() / T)), blk(gang_block<RR, T>());
    if constexpr (gang_repl<RR, T>()) {
      if (!g.gang_dist) {
        hipLaunchKernelGGL((gang_step_kernel<RR, T, false>), grid, blk, g.lds_bytes, s, B, io, scratch, g.lds_rows,
                           g.env_words);
        return true;
      }
    }
    hipLaunchKernelGGL((gang_step_kernel<RR, T, true>), grid, blk, g.lds_bytes, s, B, io, scratch, g.lds_rows, g.env_words);
    return true;
  } else {
    (void)B; (void)io; (void)scratch; (void)g; (void)s;
    return false;
  }
}
template <class RR>
static bool launch_gang(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if (g.team == 16) return launch_gang_t<RR, 16>(B, io, scratch, g, s);
  if (g.team == 32) return launch_gang_t<RR, 32>(B, io, scratch, g, s);
  return false;
}

// Atlas (886 floor-contact candidates) has no lane kernel: its unrolled per-slot rows would not
// fit an instruction cache; the debug `kernel = 0` option gives it the gang kernel too.  (The
// lane kernel is only instantiated inside these templates, behind `if constexpr`.)
template <class RR>
constexpr bool lane_ok() {
#ifdef PBG_DEV_GANG_ONLY  // ISA experiments on the gang kernel only (never the product library)
  return false;
#else
  return RR::NS <= 128;
#endif
}
template <class RR>
static int plan_lane(int n_envs, int cus, Geometry* g) {
  if constexpr (lane_ok<RR>()) {
    g->team = 1;
    g->env_words = 0;
    const int per_cu = (n_envs + cus - 1) / cus;
    int b = 16;
    while (b < per_cu && b < 64) b *= 2;
    const int wgs = (n_envs + b - 1) / b;
    const int wpc = (wgs + cus - 1) / cus;
    const size_t budget = (size_t)163840 / (size_t)(wpc > 0 ? wpc : 1);
    using RW = Rows<RR, 64>;
    constexpr size_t WB = sizeof(real_t<RR>);  // LDS word: float, or double on the float64 path
    long words = (long)(budget / ((size_t)b * WB)) - RW::NC - RW::LIMW;
    int cap = (int)(words / RW::W);
    if (cap > RW::MR) cap = RW::MR;
    if (cap < 0) cap = 0;
    g->block = b;
    g->lds_rows = cap;
    g->lds_bytes = (size_t)b * WB * ((size_t)RW::LIMW + (size_t)cap * RW::W + RW::NC);
    g->scratch_words_per_env = RW::WORDS;
    g->word_bytes = (int)WB;
    const void* fn = b == 64 ? (const void*)step_kernel<RR, 64> : (b == 32 ? (const void*)step_kernel<RR, 32> : (const void*)step_kernel<RR, 16>);
    const int e = (int)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g->lds_bytes);
    return e ? e : kernel_attrs(fn, g);
  } else {
    (void)n_envs; (void)cus; (void)g;
    return (int)hipErrorInvalidValue;
  }
}
template <class RR>
static int launch_lane(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if constexpr (lane_ok<RR>()) {
    const dim3 grid(blocks(B.n, g.block)), blk(g.block);
    if (g.block == 64) hipLaunchKernelGGL((step_kernel<RR, 64>), grid, blk, g.lds_bytes, s, B, io, scratch, g.lds_rows);
    else if (g.block == 32) hipLaunchKernelGGL((step_kernel<RR, 32>), grid, blk, g.lds_bytes, s, B, io, scratch, g.lds_rows);
    else hipLaunchKernelGGL((step_kernel<RR, 16>), grid, blk, g.lds_bytes, s, B, io, scratch, g.lds_rows);
    return (int)hipGetLastError();
  } else {
    (void)B; (void)io; (void)scratch; (void)g; (void)s;
    return (int)hipErrorInvalidValue;
  }
}

// ---- the float64 quad kernel (Team<R64>::ok: Ant, AntMuJoCo) is its own translation unit
// (-DPBG_TEAM64_TU, Makefile T64FLAGS).  Round 5 compiled it with the AMDGPU register-pressure trackers
// in the machine scheduler: under the default schedule the round-5 source computed NaN velocities in
// every env.  Round 6 found the cause, a backend bug: the register allocator placed the VGPR->AGPR split
// copies of two live-through doubles in a divergent region's join block before its EXEC restore, so
// lanes outside the region read stale AGPRs (register-file poisoning on the GPU; DESIGN.md section 4,
// tools/isa_uninit.py --exec-copies, tests/test_isa_exec_copies.py).  The current source has no such
// copy under either schedule and ships on the default one.
template <class RR>
constexpr bool team64_ok() { return Team<RR>::ok; }
int PBG_FN(plan_team64_)(int n_envs, int cus, Geometry* g);
bool PBG_FN(launch_team64_)(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s);
int PBG_FN(debug_stamps_t64_)(unsigned long long* host_out);  // the diagnostic stamps of this TU's kernel
#ifdef PBG_TEAM64_TU
int PBG_FN(debug_stamps_t64_)(unsigned long long* host_out) {
#ifdef PBG_STAMPS
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -3;
  unsigned long long z[16] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -3;
  return 0;
#else
  (void)host_out;
  return -1;
#endif
}
#ifdef PBG_TRACE64  // diagnostic build (tools/f64_quad_trace.py): the trace of this TU's quad kernel
extern "C" int pbg_debug_trace64(double* host_out) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_trace64), sizeof(g_trace64)) != hipSuccess) return -3;
  return (int)(sizeof(g_trace64) / sizeof(double));
}
#endif
int PBG_FN(plan_team64_)(int n_envs, int cus, Geometry* g) {
  if constexpr (team64_ok<R64>()) return plan_team<R64>(n_envs, cus, g);
  else { (void)n_envs; (void)cus; (void)g; return (int)hipErrorInvalidValue; }
}
bool PBG_FN(launch_team64_)(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if constexpr (team64_ok<R64>()) return launch_team<R64>(B, io, scratch, g, s);
  else { (void)B; (void)io; (void)scratch; (void)g; (void)s; return false; }
}
#else

// mode: 0 = lane kernel; 1 = default (quad for Ant, gang for the other walkers -- HumanoidFlagrunHarder
// and Atlas included: the cube robot runs the gang kernel's front path, distributed dynamics only);
// 2 = gang for every walker (parity tests of the gang kernel on Ant).
int PBG_FN(plan_)(int n_envs, int cus, int mode, Geometry* g) {
  if (Team<R>::ok && mode == 1) return plan_team<R>(n_envs, cus, g);
  if (R::kind != 1 && (mode >= 1 || !lane_ok<R>())) return plan_gang<R>(n_envs, cus, g, g->gang_lanes);
  return plan_lane<R>(n_envs, cus, g);
}

int PBG_FN(launch_step_)(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if (launch_team<R>(B, io, scratch, g, s)) return (int)hipGetLastError();
  if (launch_gang<R>(B, io, scratch, g, s)) return (int)hipGetLastError();
  return launch_lane<R>(B, io, scratch, g, s);
}

int PBG_FN(launch_reset_)(const Buffers& B, const ResetIO& io, hipStream_t s) {
  hipLaunchKernelGGL(reset_kernel<R>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, io);
  return (int)hipGetLastError();
}

int PBG_FN(launch_get_state_)(const Buffers& B, double* phys, double* aux, hipStream_t s) {
  hipLaunchKernelGGL(get_state_kernel<R>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, phys, aux);
  return (int)hipGetLastError();
}

int PBG_FN(launch_set_state_)(const Buffers& B, const double* phys, const double* aux, hipStream_t s) {
  hipLaunchKernelGGL(set_state_kernel<R>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, phys, aux);
  return (int)hipGetLastError();
}

int PBG_FN(launch_pack_)(int n, const double* in, double* out, hipStream_t s) {
  hipLaunchKernelGGL(pack_kernel<R>, dim3(blocks(n, 64)), dim3(64), 0, s, n, in, out);
  return (int)hipGetLastError();
}

// ---- the reference-precision path (pbg_create_v2 precision 64): float64 physics state and
// arithmetic (pybullet's btScalar, scene_bases.py:75-76) for every robot with at most 128
// floor-contact slots (Atlas: PBG_E_HIP at create).  mode 0: the lane-per-env
// kernel (the float64 gang and quad kernels' parity cross-check); 1 (default): the quad kernel for Ant
// (team64_ok), the 16-lane gang kernel for the other walkers and the lane kernel for the pendulums;
// 2: the gang kernel for every walker (Ant included).
int PBG_FN(plan64_)(int n_envs, int cus, int mode, Geometry* g) {
  if (team64_ok<R64>() && mode == 1) return PBG_FN(plan_team64_)(n_envs, cus, g);
  if constexpr (gang_ok<R64, 16>()) {
    if (mode != 0) {
      // the Humanoid family's default is 32 lanes: its float64 regions let a CU hold 8 envs, which
      // 32-lane gangs spread over all four SIMDs (0.493 -> 0.471 ms at 4,096 Humanoid envs)
      if (g->gang_lanes == 32 || (g->gang_lanes < 0 && gang_ok<R64, 32>())) {
        if constexpr (gang_ok<R64, 32>()) return plan_gang_t<R64, 32>(n_envs, cus, g);
        else return (int)hipErrorInvalidValue;
      }
      return plan_gang_t<R64, 16>(n_envs, cus, g);
    }
  }
  return plan_lane<R64L>(n_envs, cus, g);
}
int PBG_FN(launch_step64_)(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s) {
  if (PBG_FN(launch_team64_)(B, io, scratch, g, s)) return (int)hipGetLastError();
  if (launch_gang<R64>(B, io, scratch, g, s)) return (int)hipGetLastError();
  return launch_lane<R64L>(B, io, scratch, g, s);
}
int PBG_FN(launch_reset64_)(const Buffers& B, const ResetIO& io, hipStream_t s) {
  hipLaunchKernelGGL(reset_kernel<R64>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, io);
  return (int)hipGetLastError();
}
int PBG_FN(launch_get_state64_)(const Buffers& B, double* phys, double* aux, hipStream_t s) {
  hipLaunchKernelGGL(get_state_kernel<R64>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, phys, aux);
  return (int)hipGetLastError();
}
int PBG_FN(launch_set_state64_)(const Buffers& B, const double* phys, const double* aux, hipStream_t s) {
  hipLaunchKernelGGL(set_state_kernel<R64>, dim3(blocks(B.n, 64)), dim3(64), 0, s, B, phys, aux);
  return (int)hipGetLastError();
}

int PBG_FN(debug_stamps_)(unsigned long long* host_out) {
#ifdef PBG_STAMPS
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -3;
  unsigned long long z[16] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -3;
  // plus the float64 quad kernel's (its own translation unit and code object)
  unsigned long long t64[16];
  if (PBG_FN(debug_stamps_t64_)(t64) == 0)
    for (int i = 0; i < 16; i++) host_out[i] += t64[i];
  return 0;
#else
  (void)host_out;
  return -1;
#endif
}
#endif  // PBG_TEAM64_TU
}  // namespace pbg
