// Physics parameters shared by the HIP step kernel and the CPU oracle.
//
// Scene/World constants restate the reference (file:line under /root/reference).
// Solver internals restate Bullet's btMultiBody / btMultiBodyConstraintSolver defaults,
// which live in the third-party pybullet wheel (absent here): they are [EXT] and
// unpinned by anything in this container.
#pragma once
#include <stdint.h>

#define PBG_GRAVITY 9.8                 // gym_locomotion_envs.py:19, gym_pendulum_envs.py:14
#define PBG_CONTACT_ERP 0.2             // default of models_gen.h contact_erp (per robot; codegen overrides) [EXT] btContactSolverInfo::m_erp: the multibody contact rows use m_erp;
                                        // setDefaultContactERP(0.9) (scene_bases.py:69) sets m_erp2, used only
                                        // for split-impulse penetrations deeper than 4 cm
#define PBG_SOLVER_ITERATIONS 5         // scene_bases.py:65 numSolverIterations=5
#define PBG_LIMIT_ERP 0.2               // [EXT] btContactSolverInfo::m_erp default
#define PBG_LIMIT_MAX_IMPULSE 100.0     // [EXT] btMultiBodyJointLimitConstraint max impulse
#define PBG_CONTACT_THRESHOLD 0.02      // [EXT] gContactBreakingThreshold
#define PBG_LINEAR_DAMPING 0.04         // [EXT] btMultiBody m_linearDamping (k1 = k2)
#define PBG_ANGULAR_DAMPING 0.04        // [EXT] btMultiBody m_angularDamping (k1 = k2)
#define PBG_MAX_COORD_VELOCITY 100.0    // [EXT] btMultiBody m_maxCoordinateVelocity
#define PBG_ANGULAR_MOTION_THRESHOLD 0.7853981633974483  // [EXT] 0.5*SIMD_HALF_PI
// Restitution (models_gen.h restitution, the combined robot x floor coefficient e): a contact
// normal's target gains e * (-v_n) when the approach speed |v_n| >= the threshold
// [EXT] btSequentialImpulseConstraintSolver::restitutionCurve, btContactSolverInfo::m_restitutionVelocityThreshold
#define PBG_RESTITUTION_VELOCITY_THRESHOLD 0.2
#define PBG_WALK_TARGET_X 1000.0       // robot_locomotors.py:12 walk_target_x = 1e3
#define PBG_WALK_TARGET_Y 0.0           // robot_locomotors.py:13
// HumanoidFlagrun (robot_locomotors.py:203-213): flag at U(+-halflen) x U(+-halfwidth) times
// 0.5, re-drawn when the walk target is within 1 m or after 600 / frame_skip calc_states
#define PBG_STADIUM_HALFLEN 26.25       // scene_stadium.py:14 105*0.25
#define PBG_STADIUM_HALFWIDTH 12.5      // scene_stadium.py:15 50*0.25
#define PBG_FLAG_COMPACT 0.5            // robot_locomotors.py:206 more_compact
#define PBG_FLAG_TIMEOUT 150            // robot_locomotors.py:216 600/frame_skip
#define PBG_OBS_CLIP 5.0                // robot_locomotors.py:64 np.clip(..., -5, +5)
#define PBG_JOINT_AT_LIMIT 0.99f        // robot_locomotors.py:36 (float32 compare)

// HumanoidFlagrunHarder's attacking cube (robot_locomotors.py:230-302; gym_utils.py:9-15
// get_cube: pybullet_data cube_small.urdf -- envs/assets/things/cube_small.urdf holds the same
// file: box .05, lateral_friction 1.0 (codegen.py CUBE_FRICTION -> cgeom_mu, cube_floor_mu) -- loaded at (-1.5, 0, 0.05), changeDynamics(mass=1.2)).
// [EXT] changeDynamics(mass) recomputes the base inertia from the collision shape
// (btBoxShape::calculateLocalInertia: m/12 (ly^2 + lz^2), isotropic for a cube).
#define PBG_CUBE_HALF 0.025
#define PBG_CUBE_MASS 1.2
#define PBG_CUBE_INERTIA (PBG_CUBE_MASS * (2.0 * PBG_CUBE_HALF) * (2.0 * PBG_CUBE_HALF) / 6.0)
#define PBG_CUBE_X0 (-1.5)              // robot_locomotors.py:242,244
#define PBG_CUBE_Y0 0.0
#define PBG_CUBE_Z0 0.05
#define PBG_CUBE_WORDS 13               // pos 3 | quat 4 | lin vel 3 | ang vel 3
// alive_bonus (robot_locomotors.py:250-273): a launch every 30 frames after frame 100 while the
// robot is up, from 4 m away at U(20, 30) m/s towards its predicted position; U(+-1) jitter
#define PBG_HARDER_LAUNCH_EVERY 30
#define PBG_HARDER_LAUNCH_AFTER 100
#define PBG_HARDER_GROUND_Z 0.8         // z < 0.8: on the ground (:267, :291), potential_leak clip (:277)
#define PBG_HARDER_GROUND_FRAMES 170    // :273 (alive -1 once the counter reaches it)
#define PBG_HARDER_FROM_DIST 4.0        // :255

// Per-env physical state record (float64 at the C-ABI, float32 inside the kernel):
//   [0..2] base COM position  [3..6] base quaternion (x,y,z,w)
//   [7..9] base COM linear velocity (world)  [10..12] base angular velocity (world)
//   [13 .. 13+NJ)  joint positions q   [13+NJ .. 13+2NJ)  joint velocities qd
//   HumanoidFlagrunHarder only: [13+2NJ .. 13+2NJ+13) the cube (PBG_CUBE_WORDS, same layout
//   as the base words)
// Fixed-base robots keep the 13 base words at their load values.
#define PBG_BASE_WORDS 13
#define PBG_STATE_WORDS(NJ, harder) (PBG_BASE_WORDS + 2 * (NJ) + ((harder) ? PBG_CUBE_WORDS : 0))

// Per-env bookkeeping record (float64):
//   [0] potential  [1] initial_z  [2] elapsed steps  [3] floor-in-parts flag
//   [4 .. 4+NF) feet_contact (as written into the observation)
//   HumanoidFlagrun(Harder): [4+NF .. 4+NF+4) walk target x, y, flag_timeout, flag draws so far
//   HumanoidFlagrunHarder: [8+NF .. 8+NF+5) frame, on_ground_frame_counter,
//     crawl_start_potential (NaN = None), crawl_ignored_potential, cube launches so far
//   last word: episodes started so far (the Philox counter of the next reset's noise), so a
//   checkpoint restored into a fresh handle continues the same reset stream
#define PBG_AUX_WORDS 4
#define PBG_AUX_RECORD_WORDS(NF, flagrun, harder) \
  (PBG_AUX_WORDS + (NF) + ((flagrun) ? 4 : 0) + ((harder) ? 5 : 0) + 1)

// Contact-set signature (parity tests): the term of active collision candidate `id` (floor
// slots 0..NS-1, self-collision pairs NS + p) in sub-step `sub` is murmur3's fmix32 of
// (sub << 16) + id + golden ratio; an env step's signature is the sum mod 2^32 of the terms
// of every active candidate of every sub-step (order-free, so distributed kernels reduce it
// with a plain integer sum).  Equal signatures <=> the same active contact sets (up to 2^-32).
#ifdef __HIP__
#define PBG_HD __host__ __device__ inline
#else
#define PBG_HD inline
#endif
PBG_HD uint32_t pbg_contact_hash(uint32_t sub, uint32_t id) {
  uint32_t h = (sub << 16) + id + 0x9E3779B9u;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// Solver active-set signature (parity tests): a PGS row update that ends clamped at its lower
// bound (code 1) or its upper bound (code 2), and a friction pair skipped under a non-positive
// normal impulse (code 3, on the pair's first row), add the term of (sub-step, sweep, row,
// code); rows: joint limit li (limited dofs in dof order) side s -> 2 li + s, contact c ->
// 2 NLIM + 3 c + {0 normal, 1 and 2 friction}.  With the same contact set and the same
// signature, GPU and oracle took the same branch at every update of the 5-sweep PGS, which is
// then a smooth function of the state.
PBG_HD uint32_t pbg_solver_event(uint32_t sub, uint32_t sweep, uint32_t row, uint32_t code) {
  return pbg_contact_hash(0x8000u | (sub << 4) | sweep, (row << 2) | code);
}
template <class F>
PBG_HD uint32_t pbg_clamp_code(F v, F lo, F hi) { return v < lo ? 1u : (v > hi ? 2u : 0u); }
