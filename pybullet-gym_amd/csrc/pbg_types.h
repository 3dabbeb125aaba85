// Kernel argument blocks shared by the kernels (pbg_step.hip) and the C-ABI layer.
#pragma once
#include <stdint.h>

#include <type_traits>

namespace pbg {
// Scene / World parameters of a handle (include/pbg.h pbg_sim_params_t; scene_bases.py:8-18,
// 58-73), resolved once on the host at create into the constants the kernels use.  Every
// derived float is formed in float arithmetic exactly as the kernels formed it when these
// were compile-time constants, so default parameters reproduce the old bits.
template <class S>
struct SimPT {
  S dt;              // Scene.timestep: one stepSimulation sub-step
  S gravity;         // World.gravity: setGravity(0, 0, -gravity)
  S k_sep;           // position-target slope of a separated row: -1 / dt (pos_target)
  S k_contact;       // ... of a penetrating contact normal: -contact_erp / dt
  S k_limit;         // ... of a violated joint limit: -limit_erp / dt
  S ang_max;         // [EXT] angular motion threshold / dt (exponential-map integration)
  S dt3c;            // dt^3 / 48 (small-angle quaternion series)
  int substeps;      // Scene.frame_skip = numSubSteps
  int iterations;    // World.numSolverIterations
  int flag_timeout;  // HumanoidFlagrun: 600 / frame_skip steps, rounded up (robot_locomotors.py:218-223)
  double env_dt;     // Scene.dt = timestep * frame_skip (the potential's divisor, scene_bases.py:17)
};
using SimP = SimPT<float>;

// The same parameters formed in S arithmetic: S = float reproduces the bits of the compile-time
// constants the float32 kernels once folded; S = double is the scene at btScalar precision
// (scene_bases.py:75-76), as the float64 oracle forms it.
template <class S = float>
inline SimPT<S> resolve_sim_params(double timestep, int frame_skip, int iterations, double gravity, double contact_erp,
                                   double limit_erp, double angular_motion_threshold) {
  SimPT<S> p;
  p.dt = (S)timestep;
  const S inv_dt = (S)(1.0 / timestep);
  p.gravity = (S)gravity;
  p.k_sep = -inv_dt;
  p.k_contact = -(S)contact_erp * inv_dt;
  p.k_limit = -(S)limit_erp * inv_dt;
  p.ang_max = (S)angular_motion_threshold / p.dt;
  p.dt3c = p.dt * p.dt * p.dt * (sizeof(S) == 4 ? (S)0.020833333333f : (S)0.020833333333);
  p.substeps = frame_skip;
  p.iterations = iterations;
  p.flag_timeout = (600 + frame_skip - 1) / frame_skip;
  p.env_dt = timestep * frame_skip;
  return p;
}

// Scalar of a robot's physics state and arithmetic: float (the float32 kernels) or double
// (F64<R>: the reference-precision path, pbg_create_ex precision 64).  F64<R> is the robot R
// with `real = double`; every model table is R's.
template <class R, class = void>
struct RealOf {
  using type = float;
};
template <class R>
struct RealOf<R, std::void_t<typename R::real>> {
  using type = typename R::real;
};
template <class R>
using real_t = typename RealOf<R>::type;
template <class R0>
struct F64 : R0 {
  using real = double;
};
// F64L<R>: the float64 robot as the LANE kernel instantiates it -- the same tables and scalar, with the
// device library's sin / cos in the physics (lib_trig).  The float64 lane kernels of the Humanoid family
// (7 KB of scratch per lane) computed wrong states with the float64 kernels' own sincos
// (pbg_sincos64.h) under both machine schedules, while the gang kernels running the same function on
// the same inputs stay within 1e-9 of the oracle: the lane kernel, the parity
// cross-check of the others, keeps the trigonometry it was validated with.
template <class R0>
struct F64L : F64<R0> {
#ifdef PBG_DEV_LANE_OWN_TRIG  // diagnostic ISA only (tests/test_isa_exec_copies.py): the round-6 variant
  static constexpr bool lib_trig = false;
#else
  static constexpr bool lib_trig = true;
#endif
};
template <class R, class = void>
struct LibTrig {
  static constexpr bool value = false;
};
template <class R>
struct LibTrig<R, std::void_t<decltype(R::lib_trig)>> {
  static constexpr bool value = R::lib_trig;
};
template <class R>
inline constexpr bool lib_trig_v = LibTrig<R>::value;

struct Buffers {
  int n;                   // envs on this device
  void* st;                // [SD][n] physical state, SoA, in the handle's precision (st_of<R>)
  double* pot;             // [n] potential
  void* z0;                // [n] initial_z, in the handle's precision (z0_of<R>)
  int* elapsed;            // [n] steps in episode
  uint32_t* flags;         // [n] bit0 floor-in-parts, bits 8.. feet_contact
  uint32_t* episode;       // [n] resets so far (RNG counter)
  double* tgt;             // [2][n] walk target x, y (HumanoidFlagrun)
  int32_t* ftm;            // [2][n] flag_timeout, flag draws so far (HumanoidFlagrun RNG counter)
  double* hkd;             // [2][n] crawl_start_potential (NaN = None), crawl_ignored_potential (Harder)
  int32_t* hki;            // [3][n] frame, on_ground_frame_counter, cube launches so far (Harder)
  uint64_t seed;
  int env_offset;          // global id of env 0 (multi-GPU sharding)
  SimP sp;                 // the handle's scene parameters (kernel arguments), float32 kernels
  SimPT<double> sp64;      // the same scene in float64 (the reference-precision kernels)
};

struct StepIO {
  const float* act;        // [n][NA]
  float* obs;              // [n][OBS]
  float* rew;              // [n] float32 reward
  double* rew64;           // [n] nullable float64 reward
  uint8_t* done;           // [n] terminated | truncated
  uint8_t* trunc;          // [n] nullable, TimeLimit truncation
  float* term_obs;         // [n][OBS] nullable: obs before an auto-reset
  int32_t* ncontact;       // [n] nullable: contacts in the last sub-step
  int autoreset;
  double* rew_terms;       // [n][5] nullable: the terms the reward sums (reference self.rewards)
  uint32_t* csig;          // [n] nullable: contact-set signature (sim_params.h pbg_contact_hash)
};

struct ResetIO {
  const uint8_t* mask;     // [n] nullable = all
  const float* init_q;     // [n][NR] nullable = Philox noise U(-0.1, 0.1)
  float* obs;              // [n][OBS]
};

}  // namespace pbg
