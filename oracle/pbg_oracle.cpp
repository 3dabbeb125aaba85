// pbg_oracle.cpp -- CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library, and only as the checker / the timed CPU baseline.  The product path
// (pybullet-gym_amd/csrc, libpbg_amd.so) never links or calls it.
//
// What it restates (file:line relative to /root/reference):
//   * WalkerBaseBulletEnv._step        pybulletgym/envs/roboschool/gym_locomotion_envs.py:54-114
//   * WalkerBase.apply_action          pybulletgym/envs/roboschool/robot_locomotors.py:26-29
//   * WalkerBase.calc_state/potential  robot_locomotors.py:31-79, robot_bases.py:209-325
//   * alive bonuses                    robot_locomotors.py:89-90,116-118,137-138,191-192
//   * WalkerBaseBulletEnv._reset       gym_locomotion_envs.py:22-39 + robot_locomotors.py:16-24
//   * InvertedPendulumBulletEnv        gym_pendulum_envs.py:16-39, robot_pendula.py:11-51
//   * World.step -> stepSimulation     scene_bases.py:47-52,58-76  [EXT: Bullet btMultiBody]
//
// The physics inside stepSimulation() is Bullet's (third-party, not in /root/reference,
// not installed here): it is restated from Bullet's published algorithm -- joint-space
// Featherstone dynamics (composite-rigid-body mass matrix + recursive Newton-Euler bias,
// Cholesky solve; equal to the articulated-body algorithm's result), Bullet-style body
// damping, sequential-impulse PGS over joint-limit / contact-normal / friction rows with
// Baumgarte ERP, semi-implicit Euler with exponential-map base rotation.  PHYSICS PARITY
// WITH PYBULLET IS UNPINNED (nothing in this container can run pybullet).  The
// observation/reward/done pack (pbg_oracle_pack) IS pinned: tests/golden/ holds vectors
// produced by the reference's own Python (tests/golden/make_golden.py).
//
// Plain double-precision scalar code; loops at run time over the model tables of
// csrc/models_gen.h.  Build: oracle/Makefile.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include "../pybullet-gym_amd/csrc/models_gen.h"
#include "../pybullet-gym_amd/csrc/sim_params.h"
#include "counted.h"
#include "mca.h"

#include <cmath>

#define MAXL 32
#define MAXD 40
#define MAXS 1024
#define MAXPAIR 72
#define MAXCG 24
#define MAXCAND (MAXS + MAXPAIR + 8 + MAXCG)  // collision candidates (HumanoidFlagrunHarder's cube: 8 + NCG)
#define MAXROWS (2 * MAXD + 6 * MAXCAND)      // 3 rows per contact + the rule study's 3 torsional

thread_local FlopCount g_flops;
thread_local uint64_t g_mca_state;
static uint64_t g_mca_seed = 0;

namespace {

// Test switches (pbg_oracle_set_flags): bit0 no joint limits, bit1 no contacts, bit2 no body
// damping, bit3 no joint damping, bit4 no gravity.  0 in every product-parity comparison.
int g_flags = 0;

// Physics-rule variants for the importer/solver-rule study (pbg_oracle_set_physics; DESIGN.md
// section 2 scores each with the reference's pretrained policies).  The defaults restate the
// rules the HIP kernels implement; every product-parity comparison runs with the defaults.
enum { OPT_CONTACT_ERP, OPT_DEEP_ERP, OPT_DEEP_THR, OPT_DEEP_MODE, OPT_LIMIT_MODE, OPT_DAMP_MODE, OPT_FRIC_MODE,
       OPT_WARM, OPT_WARM_FRIC, OPT_LIMIT_ERP, OPT_ITERS, OPT_SEP_MODE, OPT_SLOP, OPT_SEP_ABS, OPT_LIM_SEP_ABS,
       OPT_SPRINGS, OPT_ROLL_MU, OPT_SPIN_MU, OPT_LIM_DEEP_MODE, OPT_LIMIT_CFM, OPT_CONTACT_CFM, OPT_CONTACT_THR,
       OPT_MARGIN, OPT_SELF_COLLISION, OPT_GRAVITY, OPT_DT, OPT_SUBSTEPS, OPT_TORQUE_SUBSTEPS, OPT_MAX_COORD_VEL, OPT_COUNT };
double g_opt[OPT_COUNT];
const double g_opt_default[OPT_COUNT] = {
    -1.0,             // contact ERP of penetrating contact normal rows (-1: the model's, models_gen.h)
    -1.0,             // ERP for penetrations deeper than OPT_DEEP_THR (-1: same as contact ERP)
    -0.04,            // split-impulse penetration threshold (btContactSolverInfo m_splitImpulsePenetrationThreshold)
    0.0,              // deep mode: 0 = OPT_DEEP_ERP, 1 = no positional term (split impulse absent for multibodies)
    0.0,              // joint limits: 0 = rows always (separated: J dnu >= -d/dt), 1 = only when violated
    0.0,              // joint damping: 0 = per sub-step from that sub-step's velocity, 1 = once per env step
    0.0,              // friction: 0 = two directions, box, 1 = two directions, cone projection, 2 = one direction
    0.0,              // warm start factor of persistent contacts (0 = off)
    0.0,              // warm start the friction rows too
    PBG_LIMIT_ERP,    // joint-limit ERP
    PBG_SOLVER_ITERATIONS,  // PGS sweeps
    0.0,              // separated contacts: 0 = speculative row (J dnu >= -d/dt), 1 = no row
    0.0,              // linear slop added to the contact distance
    1.0,              // separated contact rows: 1 = J nu_new >= -d/dt (Bullet's absolute rhs), 0 = J dnu >= -d/dt
    1.0,              // separated joint-limit rows: the same choice
    1.0,              // joint springs: scale on the model's stiffness (mjcf.py B7): tau -= s k q
    0.0,              // rolling friction: combined coefficient of two angular rows about the contact tangents
    0.0,              // spinning friction: combined coefficient of an angular row about the contact normal
    0.0,              // joint-limit violations deeper than OPT_DEEP_THR: 0 = OPT_LIMIT_ERP, 1 = velocity only
                      //   (btMultiBodyJointLimitConstraint's split-impulse branch; split impulse is not
                      //   solved for multibodies), 2 = ERP 0.9 (m_erp2 from setDefaultContactERP)
    0.0,              // joint-limit CFM: m_eff = 1 / (J M^-1 J^T + cfm)
    0.0,              // contact CFM (normal and friction rows)
    PBG_CONTACT_THRESHOLD,  // contact processing / breaking threshold
    0.0,              // collision margin added around every robot geom (MJCF geom margin)
    1.0,              // self-collision pairs: 1 = on (URDF_USE_SELF_COLLISION, robot_bases.py:116), 0 = off
    PBG_GRAVITY,      // scene gravity (pbg_oracle_set_sim_params, the product's pbg_sim_params_t)
    -1.0,             // sub-step timestep (-1: the model's dt_sub)
    -1.0,             // sub-steps per env step (-1: the model's frame_skip)
    -1.0,             // sub-steps that carry apply_action's joint torques (-1: all of them; 1: the first
                      //   only -- Bullet clears a multibody's joint torques after each internal step
                      //   [EXT, rule study, SURVEY.md Appendix B1])
    PBG_MAX_COORD_VELOCITY,  // btMultiBody m_maxCoordinateVelocity (rule study, round 5: the pendulums)
};
struct OptInit { OptInit() { for (int i = 0; i < OPT_COUNT; i++) g_opt[i] = g_opt_default[i]; } } g_opt_init;
// persistent contact impulses per env and collision candidate (warm starting):
// [env][candidate][normal, t1, t2, active]
double* g_cache = nullptr;
size_t g_cache_n = 0;
// contact diagnostics (pbg_oracle_contact_diag; single env, single thread): per contact of every
// sub-step [sub, candidate, dist, lambda_n, lambda_t1, lambda_t2, mu, v_n, v_t1, v_t2] after the solve
double* g_diag = nullptr;
int g_diag_n = 0, g_diag_cap = 0;

// ------------------------------------------------------------------ model view
struct MV {
  int robot_id, kind, floating, NL, NJ, NDOF, NA, NO, NR, NF, NP, NS, NPAIR, OBS, alive, substeps,
      floor, max_steps, robot_body, tip_link, flagrun, harder, NCG, head_link;
  double power, elec, stall, jal, z0fixed, dt_sub, base_mass, power_cost, qvel_clip, contact_erp, cube_floor_mu;
  double restitution, spin_mu, roll_mu;  // robot x floor material (codegen.py: Bullet's combiners)
  const double *base_inertia, *base_pos, *base_quat;
  const int *link_parent, *link_jtype, *link_dof;
  const double (*off_pos)[3], (*axis)[3], (*anchor)[3], (*com)[3], (*off_quat)[4], (*inertia)[6];
  const double* mass;
  const double *lower, *upper, *damping, *stiffness, *armature;
  const int *limited, *dof_jtype;
  const int* act_dof; const double* act_gain;
  const int* obs_dof; const double* obs_vel_scale; const int* reset_dof; const double* reset_offset;
  const int* part_link; const int* foot_link; const int* knee_obs;
  const int* slot_link; const double (*slot_point)[3]; const double *slot_radius, *slot_mu;
  const int *pair_a, *pair_b; const double (*pa0)[3], (*pa1)[3], (*pb0)[3], (*pb1)[3];
  const double *pra, *prb, *pmu;
  const int* cg_link; const double (*cg_p0)[3], (*cg_p1)[3]; const double *cg_r, *cg_mu;  // cube vs robot geoms
};

template <class R>
MV view() {
  MV m;
  m.robot_id = R::robot_id; m.kind = R::kind; m.floating = R::floating; m.NL = R::NL; m.NJ = R::NJ;
  m.NDOF = R::NDOF; m.NA = R::NA; m.NO = R::NO; m.NR = R::NR; m.NF = R::NF; m.NP = R::NP;
  m.NS = R::NS; m.NPAIR = R::NPAIR; m.OBS = R::OBS; m.alive = R::alive; m.substeps = R::substeps;
  m.floor = R::floor; m.max_steps = R::max_episode_steps; m.robot_body = R::robot_body; m.tip_link = R::tip_link;
  m.head_link = R::head_link; m.knee_obs = R::knee_obs;
  m.flagrun = R::flagrun; m.harder = R::harder; m.NCG = R::NCG; m.cube_floor_mu = R::cube_floor_mu;
  m.cg_link = R::cgeom_link; m.cg_p0 = R::cgeom_p0; m.cg_p1 = R::cgeom_p1; m.cg_r = R::cgeom_r; m.cg_mu = R::cgeom_mu;
  m.power = R::power; m.elec = R::electricity_cost; m.stall = R::stall_torque_cost;
  m.jal = R::joints_at_limit_cost; m.z0fixed = R::initial_z_fixed; m.dt_sub = R::dt_sub;
  m.base_mass = R::base_mass; m.power_cost = R::power_cost; m.qvel_clip = R::qvel_clip; m.contact_erp = R::contact_erp;
  m.restitution = R::restitution; m.spin_mu = R::spin_mu; m.roll_mu = R::roll_mu; m.base_inertia = R::base_inertia; m.base_pos = R::base_pos;
  m.base_quat = R::base_quat; m.link_parent = R::link_parent; m.link_jtype = R::link_jtype;
  m.link_dof = R::link_dof; m.off_pos = R::link_offset_pos; m.axis = R::link_axis;
  m.anchor = R::link_anchor; m.com = R::link_com; m.off_quat = R::link_offset_quat;
  m.inertia = R::link_inertia; m.mass = R::link_mass; m.lower = R::dof_lower; m.upper = R::dof_upper;
  m.damping = R::dof_damping; m.stiffness = R::dof_stiffness; m.armature = R::dof_armature; m.limited = R::dof_limited;
  m.dof_jtype = R::dof_jtype; m.act_dof = R::act_dof; m.act_gain = R::act_gain;
  m.obs_dof = R::obs_dof; m.obs_vel_scale = R::obs_vel_scale; m.reset_dof = R::reset_dof;
  m.reset_offset = R::reset_offset;
  m.part_link = R::part_link; m.foot_link = R::foot_link; m.slot_link = R::slot_link;
  m.slot_point = R::slot_point; m.slot_radius = R::slot_radius; m.slot_mu = R::slot_mu;
  m.pair_a = R::pair_link_a; m.pair_b = R::pair_link_b; m.pa0 = R::pair_a0; m.pa1 = R::pair_a1;
  m.pb0 = R::pair_b0; m.pb1 = R::pair_b1; m.pra = R::pair_ra; m.prb = R::pair_rb; m.pmu = R::pair_mu;
  return m;
}

// the scene parameters in force (pbg_oracle_set_sim_params): sub-step, frame_skip, Scene.dt,
// HumanoidFlagrun's flag timeout 600 / frame_skip rounded up (robot_locomotors.py:218-223)
double sim_dt(const MV& m) { return g_opt[OPT_DT] > 0.0 ? g_opt[OPT_DT] : m.dt_sub; }
int sim_substeps(const MV& m) { return g_opt[OPT_SUBSTEPS] > 0.0 ? (int)g_opt[OPT_SUBSTEPS] : m.substeps; }
double sim_env_dt(const MV& m) { return sim_dt(m) * sim_substeps(m); }
int sim_flag_timeout(const MV& m) { return (600 + sim_substeps(m) - 1) / sim_substeps(m); }

MV* model_views() {
  static MV views[17] = {view<pbg_models::Pendulum>(), view<pbg_models::Hopper>(),
                         view<pbg_models::HalfCheetah>(), view<pbg_models::Ant>(),
                         view<pbg_models::Humanoid>(), view<pbg_models::Walker2D>(),
                         view<pbg_models::PendulumSwingup>(), view<pbg_models::DoublePendulum>(),
                         view<pbg_models::HumanoidFlagrun>(), view<pbg_models::HopperMuJoCo>(),
                         view<pbg_models::Walker2DMuJoCo>(), view<pbg_models::HalfCheetahMuJoCo>(),
                         view<pbg_models::AntMuJoCo>(), view<pbg_models::HumanoidMuJoCo>(),
                         view<pbg_models::DoublePendulumMuJoCo>(), view<pbg_models::HumanoidFlagrunHarder>(),
                         view<pbg_models::Atlas>()};
  return views;
}
const MV* model(int robot) {
  if (robot < 0 || robot > 16) return nullptr;
  return &model_views()[robot];
}
// Importer-rule study (tools/physics_rules.py): a robot's link masses, COMs and inertias replaced
// at run time (pbg_oracle_set_link_dynamics); the compiled tables stay the product's.
struct LinkDynOverride {
  bool on = false;
  double mass[MAXL], com[MAXL][3], inertia[MAXL][6], base_inertia[6], base_mass;
  MV orig;
};
LinkDynOverride g_dyn_ov[17];
// joint damping replaced at run time (importer-rule study: MJCF <default> damping inheritance)
struct DampOverride {
  bool on = false;
  double damping[MAXD];
  const double* orig = nullptr;
};
DampOverride g_damp_ov[17];

// ------------------------------------------------------------------ physics (pbg_physics.h)
#include "pbg_physics.h"
using V3 = V3T<double>;
using M3 = M3T<double>;
using Kin = KinT<double>;

// M3 -> quaternion (x,y,z,w)
inline void m3_to_quat(const M3& m, double* q) {
  double t = m.m[0][0] + m.m[1][1] + m.m[2][2];
  if (t > 0) {
    double s = sqrt(t + 1.0) * 2;
    q[3] = 0.25 * s; q[0] = (m.m[2][1] - m.m[1][2]) / s; q[1] = (m.m[0][2] - m.m[2][0]) / s; q[2] = (m.m[1][0] - m.m[0][1]) / s;
  } else if (m.m[0][0] > m.m[1][1] && m.m[0][0] > m.m[2][2]) {
    double s = sqrt(1.0 + m.m[0][0] - m.m[1][1] - m.m[2][2]) * 2;
    q[3] = (m.m[2][1] - m.m[1][2]) / s; q[0] = 0.25 * s; q[1] = (m.m[0][1] + m.m[1][0]) / s; q[2] = (m.m[0][2] + m.m[2][0]) / s;
  } else if (m.m[1][1] > m.m[2][2]) {
    double s = sqrt(1.0 + m.m[1][1] - m.m[0][0] - m.m[2][2]) * 2;
    q[3] = (m.m[0][2] - m.m[2][0]) / s; q[0] = (m.m[0][1] + m.m[1][0]) / s; q[1] = 0.25 * s; q[2] = (m.m[1][2] + m.m[2][1]) / s;
  } else {
    double s = sqrt(1.0 + m.m[2][2] - m.m[0][0] - m.m[1][1]) * 2;
    q[3] = (m.m[1][0] - m.m[0][1]) / s; q[0] = (m.m[0][2] + m.m[2][0]) / s; q[1] = (m.m[1][2] + m.m[2][1]) / s; q[2] = 0.25 * s;
  }
}


// ------------------------------------------------------------------ pack (numpy-exact)
// numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src) with the add
// identity 0 as the reduction's initial value; verified bit-exact against numpy 2.2.
double np_sum_f64(const double* a, int n, int stride) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; i++) res += a[i * stride];
    return 0.0 + res;
  }
  double r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i * stride];
  return 0.0 + res;
}
float np_sum_f32(const float* a, int n) {
  if (n < 8) {
    float res = 0.0f;
    for (int i = 0; i < n; i++) res += a[i];
    return 0.0f + res;
  }
  float r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return 0.0f + res;
}

// pybullet.getEulerFromQuaternion (pybullet.c), q = (x, y, z, w)  [EXT, restated]
void euler_from_quat(const double* q, double* rpy) {
  double sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
  rpy[0] = atan2(2 * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
  double sarg = -2 * (q[0] * q[2] - q[3] * q[1]);
  rpy[1] = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
  rpy[2] = atan2(2 * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
}

inline float clip5(float v) { return v < -5.0f ? -5.0f : (v > 5.0f ? 5.0f : v); }  // NaN passes

// Philox4x32-10 (Salmon et al. 2011), as the kernels use it for their random draws.
void philox(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0], p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ ctr[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ ctr[3] ^ k1;
    ctr[1] = (uint32_t)p1; ctr[3] = (uint32_t)p0; ctr[0] = n0; ctr[2] = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
uint64_t g_seed = 0;
int g_env_offset = 0;

// HumanoidFlagrun walk target (robot_locomotors.py:195-226): flag_reposition draws
// U(+-halflen) x U(+-halfwidth) times 0.5 (here Philox, counter (global env, draw index)).
struct Flag { double tx, ty; int timeout, count; };
void flag_draw(int e, Flag& f) {
  uint32_t c[4] = {(uint32_t)(g_env_offset + e), (uint32_t)f.count, 0xF1A6u, 0x5EEDu};
  philox(c, (uint32_t)g_seed, (uint32_t)(g_seed >> 32));
  const double u0 = (double)(c[0] >> 8) * (1.0 / 16777216.0), u1 = (double)(c[1] >> 8) * (1.0 / 16777216.0);
  f.tx = (-PBG_STADIUM_HALFLEN + 2.0 * PBG_STADIUM_HALFLEN * u0) * PBG_FLAG_COMPACT;
  f.ty = (-PBG_STADIUM_HALFWIDTH + 2.0 * PBG_STADIUM_HALFWIDTH * u1) * PBG_FLAG_COMPACT;
  f.timeout = sim_flag_timeout(*model(8));  // HumanoidFlagrun
  f.count++;
}

// HumanoidFlagrunHarder bookkeeping (robot_locomotors.py:230-302).  crawl_start NaN = None.
struct Harder { int frame, onground, launches; double crawl_start, crawl_ignored; };
// potential_leak (:275-278): clip(body z, 0, 0.8) / 0.8 + 1  (NaN passes np.clip)
double potential_leak(double z) { const double c = z < 0.0 ? 0.0 : (z > PBG_HARDER_GROUND_Z ? PBG_HARDER_GROUND_Z : z); return c / 0.8 + 1.0; }
// calc_potential (:280-302) given Humanoid.calc_potential's value fp and body_xyz[2]; mutates
// the crawl bookkeeping (every call does: env reset, _step, and the flag re-draw's
// `self.potential = self.calc_potential()` in HumanoidFlagrun.calc_state, :225)
double harder_potential(Harder& h, double fp, double bz) {
  if (bz < PBG_HARDER_GROUND_Z) {
    if (std::isnan(h.crawl_start)) h.crawl_start = fp - h.crawl_ignored;
    h.crawl_ignored = fp - h.crawl_start;
    fp = h.crawl_start;
  } else {
    fp -= h.crawl_ignored;
    h.crawl_start = NAN;
  }
  return fp + potential_leak(bz) * 100;
}
// The cube launch of alive_bonus (:251-265): angle U(-3.14, 3.14), speed U(20, 30), jitter
// U(-1, 1)^3 from np_random -- here Philox4x32-10 keyed by the seed, counter (global env, launch
// index, 0xC0BE / 0xC0BF, 0x5EED); `draws` (nullable, golden tests) = [angle, speed, jitter 3].
// cube: the env's cube state words (position and velocity set, orientation kept, w = 0).
void harder_launch(int e, Harder& h, const double* body_xyz, const double* speed, double* cube, const double* draws) {
  double d[5];
  if (draws) {
    for (int i = 0; i < 5; i++) d[i] = draws[i];
  } else {
    uint32_t c[4] = {(uint32_t)(g_env_offset + e), (uint32_t)h.launches, 0xC0BEu, 0x5EEDu};
    uint32_t c2[4] = {(uint32_t)(g_env_offset + e), (uint32_t)h.launches, 0xC0BFu, 0x5EEDu};
    philox(c, (uint32_t)g_seed, (uint32_t)(g_seed >> 32));
    philox(c2, (uint32_t)g_seed, (uint32_t)(g_seed >> 32));
    const double u[5] = {(double)(c[0] >> 8) * (1.0 / 16777216.0), (double)(c[1] >> 8) * (1.0 / 16777216.0),
                         (double)(c[2] >> 8) * (1.0 / 16777216.0), (double)(c[3] >> 8) * (1.0 / 16777216.0),
                         (double)(c2[0] >> 8) * (1.0 / 16777216.0)};
    d[0] = -3.14 + (3.14 - -3.14) * u[0];
    d[1] = 20.0 + (30.0 - 20.0) * u[1];
    for (int i = 0; i < 3; i++) d[2 + i] = -1.0 + (1.0 - -1.0) * u[2 + i];
  }
  h.launches++;
  const double ttt = PBG_HARDER_FROM_DIST / d[1];
  double t[3], pos[3], v[3];
  for (int i = 0; i < 3; i++) t[i] = body_xyz[i] + speed[i] * ttt;
  pos[0] = t[0] + PBG_HARDER_FROM_DIST * cos(d[0]);
  pos[1] = t[1] + PBG_HARDER_FROM_DIST * sin(d[0]);
  pos[2] = t[2] + 1.0;
  for (int i = 0; i < 3; i++) v[i] = t[i] - pos[i];
  const double sc = d[1] / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  for (int i = 0; i < 3; i++) {
    v[i] *= sc;
    v[i] += d[2 + i];
    cube[i] = pos[i];
    cube[7 + i] = v[i];
    cube[10 + i] = 0.0;
  }
}

}  // namespace

extern "C" {

// Pack inputs, i.e. what the reference reads back from pybullet after stepSimulation.
// part_xyz: [n_parts][3] COM positions in `parts` dict order (floor last when present).
typedef struct {
  const double* part_xyz; int n_parts;
  const double* body_quat;   // robot_body orientation (x,y,z,w)
  const double* body_pos;    // robot_body COM position
  const double* body_vel;    // robot_body COM linear velocity
  const double* jq;          // [NO] joint positions of obs joints (ordered_joints order)
  const double* jqd;         // [NO] joint velocities
  const float* feet_prev;    // [NF] feet_contact as of the previous step (goes into obs)
  const uint8_t* feet_new;   // [NF] contact with the floor after this step (nullable: reset)
  const float* act;          // [NA] raw action (nullable: reset)
  double potential_old;
  double initial_z;          // NaN: take it from this calc_state (robot_locomotors.py:44-45)
  double target_x, target_y; // robot.walk_target_x / _y (1e3, 0 except HumanoidFlagrun)
  const double* body_avel;   // base angular velocity (MuJoCo-observation Ant / Humanoid; nullable)
  double head_z;             // Atlas: the head part's height (alive_bonus, robot_locomotors.py:319)
} pbg_pack_in;

typedef struct {
  float* obs; double reward; uint8_t done; double potential; double initial_z;
  float* feet_out;           // [NF]
  double rewards[5];         // alive, progress, electricity, joints_at_limit, feet_collision
  double dist;               // walk_target_dist
  double pitch;              // body_rpy[1]
  int at_limit;              // joints_at_limit
  double body_xyz[3];        // robot.body_xyz (mean part x, y; robot_body z)
} pbg_pack_out;

void pbg_oracle_set_flags(int flags) { g_flags = flags; }


// The scene of the product's pbg_create_ex (include/pbg.h pbg_sim_params_t, fields in order):
// v = [gravity, timestep, frame_skip, solver_iterations, contact_erp, joint_limit_erp]; NULL
// restores the reference's scene.  The other rule options are left as they are.
int pbg_oracle_set_sim_params(const double* v) {
  const int ids[6] = {OPT_GRAVITY, OPT_DT, OPT_SUBSTEPS, OPT_ITERS, OPT_CONTACT_ERP, OPT_LIMIT_ERP};
  for (int i = 0; i < 6; i++) g_opt[ids[i]] = v ? v[i] : g_opt_default[ids[i]];
  return 0;
}

// Importer-rule study: joint dof damping [NJ] of robot (NULL restores the compiled table).  Never
// used by a product-parity comparison.
int pbg_oracle_set_dof_damping(int robot, const double* damping) {
  if (robot < 0 || robot > 16) return -1;
  MV& v = model_views()[robot];
  DampOverride& o = g_damp_ov[robot];
  if (!o.on) o.orig = v.damping;
  if (!damping) {
    v.damping = o.orig;
    o.on = false;
    return v.NJ;
  }
  for (int d = 0; d < v.NJ; d++) o.damping[d] = damping[d];
  o.on = true;
  v.damping = o.damping;
  return v.NJ;
}

// Physics-rule variants (see OPT_*): v[i] for i < n replaces option i; n = 0 restores the defaults.
int pbg_oracle_set_physics(const double* v, int n) {
  for (int i = 0; i < OPT_COUNT; i++) g_opt[i] = (v && i < n) ? v[i] : g_opt_default[i];
  if (g_cache && g_cache_n) memset(g_cache, 0, g_cache_n * 4 * MAXCAND * sizeof(double));
  return OPT_COUNT;
}

// Importer-rule study: replace robot's link dynamics (mass [NL], com [NL][3] link frame, inertia
// [NL][6] (xx,yy,zz,xy,xz,yz), base mass and inertia [6]); mass == NULL restores the compiled
// tables.  Returns NL (or -1).  Never used by a product-parity comparison.
int pbg_oracle_set_link_dynamics(int robot, const double* mass, const double* com, const double* inertia,
                                 double base_mass, const double* base_inertia) {
  if (robot < 0 || robot > 16) return -1;
  MV& v = model_views()[robot];
  LinkDynOverride& o = g_dyn_ov[robot];
  if (!o.on) o.orig = v;
  if (!mass) {
    v = o.orig;
    o.on = false;
    return v.NL;
  }
  for (int l = 0; l < v.NL; l++) {
    o.mass[l] = mass[l];
    for (int i = 0; i < 3; i++) o.com[l][i] = com[3 * l + i];
    for (int i = 0; i < 6; i++) o.inertia[l][i] = inertia[6 * l + i];
  }
  for (int i = 0; i < 6; i++) o.base_inertia[i] = base_inertia[i];
  o.base_mass = base_mass;
  o.on = true;
  v.mass = o.mass; v.com = o.com; v.inertia = o.inertia; v.base_inertia = o.base_inertia; v.base_mass = o.base_mass;
  return v.NL;
}

// Link frames at a state, for tests: R [NL+1][9] row-major, COM [NL+1][3] (base first).
int pbg_oracle_link_frames(int robot, const double* state, double* R_out, double* c_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) {
    for (int i = 0; i < 9; i++) R_out[9 * b + i] = k.R[b].m[i / 3][i % 3];
    c_out[3 * b] = k.c[b].x; c_out[3 * b + 1] = k.c[b].y; c_out[3 * b + 2] = k.c[b].z;
  }
  return 0;
}

// Link COM velocities / bias accelerations [NL+1][3] each (base first), for tests.
int pbg_oracle_link_vel(int robot, const double* state, double* v, double* w, double* ac, double* al) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) {
    V3* src[4] = {&k.v[b], &k.w[b], &k.ac[b], &k.al[b]};
    double* dst[4] = {v, w, ac, al};
    for (int t = 0; t < 4; t++) { dst[t][3 * b] = src[t]->x; dst[t][3 * b + 1] = src[t]->y; dst[t][3 * b + 2] = src[t]->z; }
  }
  return 0;
}

int pbg_oracle_info(int robot, int* out) {
  const MV* m = model(robot);
  if (!m) return -1;
  int v[] = {m->NL, m->NJ, m->NDOF, m->NA, m->NO, m->NR, m->NF, m->NP, m->NS, m->NPAIR, m->OBS,
             PBG_STATE_WORDS(m->NJ, m->harder), PBG_AUX_RECORD_WORDS(m->NF, m->flagrun, m->harder), m->floating, m->kind,
             sim_substeps(*m)};
  memcpy(out, v, sizeof(v));
  return 0;
}

static void pendulum_obs(const MV& m, const double* jq, const double* jqd, const double* tip, float* obs,
                         double* rew, uint8_t* done, double* terms = nullptr);
static void mujoco_planar_obs(const MV& m, const double* jq, const double* jqd, double x_after, double x_before,
                              const float* act, pbg_pack_out* out);
static void mujoco3d_obs(const MV& m, const pbg_pack_in* in, pbg_pack_out* out);

// Walker pack: calc_state (robot_locomotors.py:31-64) + the reward/done part of
// WalkerBaseBulletEnv._step (gym_locomotion_envs.py:59-114).  With act == NULL only the
// calc_state half runs (reset path).
static int walker_pack_body(const MV& m, const pbg_pack_in* in, pbg_pack_out* out);

int pbg_oracle_pack(int robot, const pbg_pack_in* in, pbg_pack_out* out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  if (m.kind == 3) {  // MuJoCo Ant / Humanoid: WalkerBase.calc_state side effects, then qpos/qvel obs
    pbg_pack_in w = *in;
    w.act = nullptr;
    walker_pack_body(m, &w, out);
    mujoco3d_obs(m, in, out);
    return 0;
  }
  if (m.kind == 2) {  // MuJoCo planar: jq/jqd all ordered joints, body_pos = robot_body, potential_old = x_before
    mujoco_planar_obs(m, in->jq, in->jqd, in->body_pos[0], in->potential_old, in->act, out);
    return 0;
  }
  if (m.kind == 1) {  // pendulums: jq/jqd = (hinge, [hinge2,] slider), pos = pole2 position
    pendulum_obs(m, in->jq, in->jqd, in->body_pos, out->obs, &out->reward, &out->done);
    if (!in->act) { out->reward = 0; out->done = 0; }
    return 0;
  }
  return walker_pack_body(m, in, out);
}

static int walker_pack_body(const MV& m, const pbg_pack_in* in, pbg_pack_out* out) {
  // joints: np.array([...], dtype=float32) of (pos_rel, vel_scaled) pairs  (robot_bases.py:306-321)
  float j[2 * MAXD];
  for (int i = 0; i < m.NO; i++) {
    int d = m.obs_dof[i];
    double pos = in->jq[i], vel = in->jqd[i];
    if (m.lower[d] < m.upper[d]) {
      double mid = 0.5 * (m.lower[d] + m.upper[d]);
      pos = 2 * (pos - mid) / (m.upper[d] - m.lower[d]);
    }
    vel *= m.obs_vel_scale[i];
    j[2 * i] = (float)pos;
    j[2 * i + 1] = (float)vel;
  }
  int at_limit = 0;
  for (int i = 0; i < m.NO; i++) at_limit += fabsf(j[2 * i]) > PBG_JOINT_AT_LIMIT;
  double bx = np_sum_f64(in->part_xyz + 0, in->n_parts, 3) / (double)in->n_parts;
  double by = np_sum_f64(in->part_xyz + 1, in->n_parts, 3) / (double)in->n_parts;
  double bz = in->body_pos[2];
  double rpy[3];
  euler_from_quat(in->body_quat, rpy);
  double z0 = isnan(in->initial_z) ? bz : in->initial_z;
  double theta = atan2(in->target_y - by, in->target_x - bx);
  double dy = in->target_y - by, dx = in->target_x - bx;
  double dist = sqrt(dy * dy + dx * dx);
  out->dist = dist;
  double ang = theta - rpy[2];
  double cy = cos(-rpy[2]), sy = sin(-rpy[2]);
  double vx = cy * in->body_vel[0] + -sy * in->body_vel[1] + 0.0 * in->body_vel[2];
  double vy = sy * in->body_vel[0] + cy * in->body_vel[1] + 0.0 * in->body_vel[2];
  double vz = 0.0 * in->body_vel[0] + 0.0 * in->body_vel[1] + 1.0 * in->body_vel[2];
  float more[8] = {(float)(bz - z0), (float)sin(ang), (float)cos(ang), (float)(0.3 * vx),
                   (float)(0.3 * vy), (float)(0.3 * vz), (float)rpy[0], (float)rpy[1]};
  int o = 0;
  for (int i = 0; i < 8; i++) out->obs[o++] = clip5(more[i]);
  for (int i = 0; i < 2 * m.NO; i++) out->obs[o++] = clip5(j[i]);
  for (int i = 0; i < m.NF; i++) out->obs[o++] = clip5(in->feet_prev[i]);
  out->initial_z = z0;
  out->pitch = rpy[1];
  out->at_limit = at_limit;
  out->body_xyz[0] = bx; out->body_xyz[1] = by; out->body_xyz[2] = bz;
  double dt = sim_env_dt(m);  // scene.dt = timestep*frame_skip (scene_bases.py:17)
  out->potential = -dist / dt;         // robot_locomotors.py:79
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_prev[i];
  if (!in->act) {
    out->reward = 0; out->done = 0;
    return 0;
  }
  // --- _step: alive / done (gym_locomotion_envs.py:61-65)
  float s0 = out->obs[0];
  double alive;
  double pitch = rpy[1];
  switch (m.alive) {
    case 0: {  // Hopper: z (f64) > 0.8 and |pitch| < 1
      double z = (double)s0 + z0;
      alive = (z > 0.8 && fabs(pitch) < 1.0) ? 1.0 : -1.0;
      break;
    }
    case 1:  // HalfCheetah: previous-step feet_contact[1,2,4,5]
      alive = (fabs(pitch) < 1.0 && !(in->feet_prev[1] != 0) && !(in->feet_prev[2] != 0) &&
               !(in->feet_prev[4] != 0) && !(in->feet_prev[5] != 0)) ? 1.0 : -1.0;
      break;
    case 2: {  // Ant: z > 0.26
      double z = (double)s0 + z0;
      alive = z > 0.26 ? 1.0 : -1.0;
      break;
    }
    case 13: {  // Atlas (robot_locomotors.py:313-324): +4 - knees at limit if head z > 1.3 else -1
      int knees = 0;
      for (int k = 0; k < 2; k++) knees += fabsf(j[2 * m.knee_obs[k]]) > PBG_JOINT_AT_LIMIT;
      alive = in->head_z > 1.3 ? (double)(4 - knees) : -1.0;
      break;
    }
    default: {  // Humanoid: np.float32 + python 0.8 stays float32 (NEP 50); z > 0.78 in f32
      float z = s0 + (float)z0;
      alive = z > 0.78f ? 2.0 : -1.0;
      break;
    }
  }
  uint8_t done = alive < 0;
  for (int i = 0; i < m.OBS; i++) if (isnan(out->obs[i])) done = 1;
  double progress = out->potential - in->potential_old;
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_new[i] ? 1.0f : 0.0f;
  // electricity: float32 arithmetic on the float32 action (gym_locomotion_envs.py:82-83)
  float tmp[MAXD];
  for (int i = 0; i < m.NA; i++) tmp[i] = fabsf(in->act[i] * j[2 * i + 1]);
  float mean_e = np_sum_f32(tmp, m.NA) / (float)m.NA;
  for (int i = 0; i < m.NA; i++) tmp[i] = in->act[i] * in->act[i];
  float mean_s = np_sum_f32(tmp, m.NA) / (float)m.NA;
  double elec = m.elec * (double)mean_e;
  elec += m.stall * (double)mean_s;
  double jal = m.jal * (double)at_limit;
  out->rewards[0] = alive; out->rewards[1] = progress; out->rewards[2] = elec;
  out->rewards[3] = jal; out->rewards[4] = 0.0;
  out->reward = ((((0.0 + alive) + progress) + elec) + jal) + 0.0;
  out->done = done;
  return 0;
}

// calc_state with HumanoidFlagrun's bookkeeping (robot_locomotors.py:219-226): timeout
// countdown, pack against the current flag, re-draw and pack again when the target is
// within 1 m or the timeout ran out.  `next` (nullable) replaces the draw (golden tests).
static void flag_pack(int robot, const MV& m, pbg_pack_in* in, pbg_pack_out* out, Flag& f, int e,
                      const double* next, Harder* h = nullptr) {
  if (!m.flagrun) { pbg_oracle_pack(robot, in, out); return; }
  f.timeout -= 1;
  in->target_x = f.tx; in->target_y = f.ty;
  pbg_oracle_pack(robot, in, out);
  if (out->dist < 1.0 || f.timeout <= 0) {
    if (next) { f.tx = next[0]; f.ty = next[1]; f.timeout = sim_flag_timeout(m); f.count++; }
    else flag_draw(e, f);
    in->target_x = f.tx; in->target_y = f.ty;
    pbg_oracle_pack(robot, in, out);
    if (h) (void)harder_potential(*h, out->potential, out->body_xyz[2]);  // robot.potential (:225)
  }
}
static Harder load_harder(const MV& m, const double* a) {
  Harder h = {0, 0, 0, NAN, 0.0};
  if (m.harder) { h.frame = (int)a[8 + m.NF]; h.onground = (int)a[9 + m.NF]; h.crawl_start = a[10 + m.NF];
                  h.crawl_ignored = a[11 + m.NF]; h.launches = (int)a[12 + m.NF]; }
  return h;
}
static void store_harder(const MV& m, double* a, const Harder& h) {
  if (m.harder) { a[8 + m.NF] = h.frame; a[9 + m.NF] = h.onground; a[10 + m.NF] = h.crawl_start;
                  a[11 + m.NF] = h.crawl_ignored; a[12 + m.NF] = h.launches; }
}
// The Harder half of _step after calc_state (gym_locomotion_envs.py:59-70 with
// HumanoidFlagrunHarder.alive_bonus / calc_potential): out holds the calc_state pack with the
// Humanoid's reward; alive, done, potential, progress and the reward are redone.  Returns 1 when
// the cube was launched (its state words in `cube` rewritten).
static int harder_step(const MV& m, const pbg_pack_in* in, pbg_pack_out* out, Harder& h, int e, double* cube,
                       const double* draws) {
  const float z = out->obs[0] + (float)m.z0fixed;  // state[0] + initial_z (float32, NEP 50)
  int launched = 0;
  if (h.frame % PBG_HARDER_LAUNCH_EVERY == 0 && h.frame > PBG_HARDER_LAUNCH_AFTER && h.onground == 0) {
    harder_launch(e, h, out->body_xyz, in->body_vel, cube, draws);
    launched = 1;
  }
  if (z < (float)PBG_HARDER_GROUND_Z) h.onground += 1;
  else if (h.onground > 0) h.onground -= 1;
  h.frame += 1;
  const double alive = h.onground < PBG_HARDER_GROUND_FRAMES ? potential_leak(out->body_xyz[2]) : -1.0;
  bool done = alive < 0;
  for (int i = 0; i < m.OBS; i++) if (std::isnan(out->obs[i])) done = true;
  out->potential = harder_potential(h, out->potential, out->body_xyz[2]);
  const double progress = out->potential - in->potential_old;
  out->rewards[0] = alive; out->rewards[1] = progress;
  out->reward = ((((0.0 + alive) + progress) + out->rewards[2]) + out->rewards[3]) + 0.0;
  out->done = done;
  return launched;
}
static Flag load_flag(const MV& m, const double* a) {
  Flag f = {0.0, 0.0, 0, 0};
  if (m.flagrun) { f.tx = a[4 + m.NF]; f.ty = a[5 + m.NF]; f.timeout = (int)a[6 + m.NF]; f.count = (int)a[7 + m.NF]; }
  return f;
}
static void store_flag(const MV& m, double* a, const Flag& f) {
  if (m.flagrun) { a[4 + m.NF] = f.tx; a[5 + m.NF] = f.ty; a[6 + m.NF] = f.timeout; a[7 + m.NF] = f.count; }
}

// Flag RNG of the kernels: Philox key = seed, env ids offset by env_offset.
void pbg_oracle_set_rng(uint64_t seed, int env_offset) { g_seed = seed; g_env_offset = env_offset; }

// Golden-vector form: flag_in = [target x, y, flag_timeout, next draw x, y],
// flag_out = [target x, y, flag_timeout] after the calc_state.
int pbg_oracle_pack_flag(int robot, const pbg_pack_in* in, pbg_pack_out* out, const double* flag_in,
                         double* flag_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  pbg_pack_in in2 = *in;
  Flag f = {flag_in[0], flag_in[1], (int)flag_in[2], 0};
  flag_pack(robot, *mp, &in2, out, f, 0, flag_in + 3);
  flag_out[0] = f.tx; flag_out[1] = f.ty; flag_out[2] = f.timeout;
  return 0;
}

// HumanoidFlagrunHarder golden form: flag_in / flag_out as above; harder_in = [frame,
// on_ground_frame_counter, crawl_start (NaN = None), crawl_ignored, launch draws: angle, speed,
// jitter 3 (NaN: no launch recorded)]; harder_out = [frame, on_ground, crawl_start,
// crawl_ignored, launched, cube position 3, cube velocity 3].  in->act NULL: the reset's
// calc_state + env.potential = calc_potential() (env_bases.py:69-70).
int pbg_oracle_pack_harder(int robot, const pbg_pack_in* in, pbg_pack_out* out, const double* flag_in,
                           double* flag_out, const double* harder_in, double* harder_out) {
  const MV* mp = model(robot);
  if (!mp || !mp->harder) return -1;
  pbg_pack_in in2 = *in;
  Flag f = {flag_in[0], flag_in[1], (int)flag_in[2], 0};
  Harder h = {(int)harder_in[0], (int)harder_in[1], 0, harder_in[2], harder_in[3]};
  flag_pack(robot, *mp, &in2, out, f, 0, flag_in + 3, &h);
  double cube[PBG_CUBE_WORDS];
  for (int i = 0; i < PBG_CUBE_WORDS; i++) cube[i] = NAN;
  int launched = 0;
  if (in->act) launched = harder_step(*mp, &in2, out, h, 0, cube, harder_in + 4);
  else out->potential = harder_potential(h, out->potential, out->body_xyz[2]);
  flag_out[0] = f.tx; flag_out[1] = f.ty; flag_out[2] = f.timeout;
  const double ho[5] = {(double)h.frame, (double)h.onground, h.crawl_start, h.crawl_ignored, (double)launched};
  for (int i = 0; i < 5; i++) harder_out[i] = ho[i];
  for (int i = 0; i < 3; i++) { harder_out[5 + i] = cube[i]; harder_out[8 + i] = cube[7 + i]; }
  return 0;
}

// MuJoCo-observation planar walkers (mujoco robot_locomotors.py:93-196, mujoco
// gym_locomotion_envs.py:121-252): obs float32 [qpos[1:], clip(qvel, +-10)] (HalfCheetah
// unclipped) over every ordered joint incl. the ignored root joints; potential =
// (x_after - x_before) / dt; reward = sum([potential, 1.0, c * sum(a^2) (float32)]).
static void mujoco_planar_obs(const MV& m, const double* jq, const double* jqd, double x_after, double x_before,
                              const float* act, pbg_pack_out* out) {
  const float c = (float)m.qvel_clip;
  int o = 0;
  for (int i = 1; i < m.NO; i++) out->obs[o++] = (float)jq[i];
  for (int i = 0; i < m.NO; i++) {
    const float v = (float)jqd[i];
    out->obs[o++] = c > 0.f ? (v < -c ? -c : (v > c ? c : v)) : v;
  }
  out->potential = x_after; out->initial_z = 0.0; out->dist = 0.0;
  for (int i = 0; i < 5; i++) out->rewards[i] = 0.0;
  if (!act) { out->reward = 0.0; out->done = 0; return; }
  const double potential = (x_after - x_before) / sim_env_dt(m);
  float sq[MAXD];
  for (int i = 0; i < m.NA; i++) sq[i] = act[i] * act[i];
  const float power_cost = (float)m.power_cost * np_sum_f32(sq, m.NA);
  bool finite = true, small = true;
  for (int i = 0; i < m.OBS; i++) {
    finite = finite && isfinite(out->obs[i]);
    if (i >= 2) small = small && fabsf(out->obs[i]) < 100.f;
  }
  const float h = out->obs[0], ang = out->obs[1];
  if (m.alive == 12) {  // rewards [potential, power_cost]
    out->reward = (0.0 + potential) + (double)power_cost;
    out->done = 0;
    out->rewards[0] = potential; out->rewards[1] = (double)power_cost;
  } else {  // rewards [potential, alive_bonus, power_cost] (mujoco gym_locomotion_envs.py:150-154)
    out->reward = ((0.0 + potential) + 1.0) + (double)power_cost;
    out->rewards[0] = potential; out->rewards[1] = 1.0; out->rewards[2] = (double)power_cost;
    out->done = m.alive == 10 ? !(finite && small && h > -0.3f && fabsf(ang) < 0.2f)
                              : !(finite && small && (1.0f > h && h > -0.2f) && (-1.0f < ang && ang < 1.0f));
  }
}

// MuJoCo-observation Ant / Humanoid (mujoco robot_locomotors.py:210-319, mujoco
// gym_locomotion_envs.py:53-114): obs [z, quat, joint q, v, w, joint qd, zeros] (float64 in
// the reference), reward sum([alive(state[0] + initial_z), progress, -0.1 at_limit, 0]).
static void mujoco3d_obs(const MV& m, const pbg_pack_in* in, pbg_pack_out* out) {
  double st[5 + 2 * MAXD + 6];
  int o = 0;
  st[o++] = in->body_pos[2];
  for (int i = 0; i < 4; i++) st[o++] = in->body_quat[i];
  for (int i = 0; i < m.NO; i++) st[o++] = in->jq[i];
  for (int i = 0; i < 3; i++) st[o++] = in->body_vel[i];
  for (int i = 0; i < 3; i++) st[o++] = in->body_avel ? in->body_avel[i] : 0.0;
  for (int i = 0; i < m.NO; i++) st[o++] = in->jqd[i];
  bool finite = true;
  for (int i = 0; i < o; i++) { out->obs[i] = (float)st[i]; finite = finite && isfinite(st[i]); }
  for (int i = o; i < m.OBS; i++) out->obs[i] = 0.f;
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_new ? (in->feet_new[i] ? 1.f : 0.f) : in->feet_prev[i];
  for (int i = 0; i < 5; i++) out->rewards[i] = 0.0;
  if (!in->act) { out->reward = 0.0; out->done = 0; return; }
  const double z = st[0] + out->initial_z;
  const double alive = m.alive == 2 ? (z > 0.26 ? 1.0 : -1.0) : (z > 0.78 ? 2.0 : -1.0);
  out->done = alive < 0 || !finite;
  const double progress = out->potential - in->potential_old;
  const double jal = -0.1 * (double)out->at_limit;
  out->rewards[0] = alive; out->rewards[1] = progress; out->rewards[2] = jal;  // [alive, progress, jal, 0]
  out->reward = (((0.0 + alive) + progress) + jal) + 0.0;
}

// Pendulum packs: calc_state + reward/done.  obs is float64 in the reference; written here
// as float32 (the C-ABI's obs dtype).
//  * InvertedPendulum / Swingup (robot_pendula.py:27-51, gym_pendulum_envs.py:26-39): non-finite
//    vx / theta / theta_dot are replaced by 0 (:32-46); balance: reward 1, done |theta| > .2;
//    swingup: reward cos(theta), never done.
//  * InvertedDoublePendulum (robot_pendula.py:76-88, gym_pendulum_envs.py:69-80): obs
//    [x, vx, pole2 x, cos th, sin th, th', cos g, sin g, g']; reward = sum([10, -dist_penalty, -0]),
//    dist_penalty = 0.01 x2^2 + (y2 + 0.3 - 2)^2 with (x2, _, y2) = pole2.pose().xyz();
//    done = y2 + 0.3 <= 1.
static void pendulum_obs(const MV& m, const double* jq, const double* jqd, const double* tip, float* obs,
                         double* rew, uint8_t* done, double* terms) {
  double tl[5] = {0, 0, 0, 0, 0};  // the reference's self.rewards (gym_pendulum_envs.py:37,81)
  if (m.alive == 7) {  // MuJoCo obs (mujoco robot_pendula.py:75-89, mujoco gym_pendulum_envs.py:60-72)
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];
    auto clip10 = [](double v) { return v < -10.0 ? -10.0 : (v > 10.0 ? 10.0 : v); };
    const double o[11] = {x, sin(th), sin(g), cos(th), cos(g), clip10(vx), clip10(thd), clip10(gd), 0.0, 0.0, 0.0};
    for (int i = 0; i < 11; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    const double vel_penalty = 1e-3 * (thd * thd) + 5e-3 * (gd * gd);
    if (rew) *rew = ((0.0 + 10.0) + -dist_penalty) + -vel_penalty;
    if (done) *done = py + 0.3 <= 1;
    tl[0] = 10.0; tl[1] = -dist_penalty; tl[2] = -vel_penalty;
    if (terms) memcpy(terms, tl, sizeof(tl));
    return;
  }
  if (m.alive == 6) {
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];
    const double o[9] = {x, vx, px, cos(th), sin(th), thd, cos(g), sin(g), gd};
    for (int i = 0; i < 9; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    if (rew) *rew = ((0.0 + 10.0) + -dist_penalty) + 0.0;
    if (done) *done = py + 0.3 <= 1;
    tl[0] = 10.0; tl[1] = -dist_penalty; tl[2] = -0.0;
    if (terms) memcpy(terms, tl, sizeof(tl));
    return;
  }
  double theta = jq[0], theta_dot = jqd[0], x = jq[1], vx = jqd[1];
  if (!isfinite(vx)) vx = 0.0;
  if (!isfinite(theta)) theta = 0.0;
  if (!isfinite(theta_dot)) theta_dot = 0.0;
  obs[0] = (float)x; obs[1] = (float)vx; obs[2] = (float)cos(theta); obs[3] = (float)sin(theta);
  obs[4] = (float)theta_dot;
  if (rew) *rew = m.alive == 5 ? cos(theta) : 1.0;
  if (done) *done = m.alive == 5 ? 0 : fabs(theta) > 0.2;
  tl[0] = m.alive == 5 ? cos(theta) : 1.0;
  if (terms) memcpy(terms, tl, sizeof(tl));
}
static void pendulum_pack(const MV& m, const double* s, float* obs, double* rew, uint8_t* done, double* terms = nullptr) {
  const double* q = s + PBG_BASE_WORDS;
  const double* qd = q + m.NJ;
  double jq[MAXD], jqd[MAXD], tip[3] = {0, 0, 0};
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = qd[m.obs_dof[i]]; }
  if (m.tip_link >= 0) {
    static thread_local Kin k;
    forward_kinematics(m, s, k);
    const V3 c = k.c[m.tip_link + 1];
    tip[0] = c.x; tip[1] = c.y; tip[2] = c.z;
  }
  pendulum_obs(m, jq, jqd, tip, obs, rew, done, terms);
}

// MuJoCo planar pack from a physical state; returns x_after (robot_body COM x).
static double mujoco_planar_pack(const MV& m, const double* s, double x_before, const float* act, float* obs,
                                 double* rew, uint8_t* done, double* terms = nullptr) {
  const double* q = s + PBG_BASE_WORDS;
  const double* qd = q + m.NJ;
  double jq[MAXD], jqd[MAXD];
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = qd[m.obs_dof[i]]; }
  static thread_local Kin k;
  forward_kinematics(m, s, k);
  const double x_after = k.c[m.robot_body + 1].x;
  float feet[8];
  pbg_pack_out out;
  out.obs = obs; out.feet_out = feet;
  mujoco_planar_obs(m, jq, jqd, x_after, x_before, act, &out);
  if (rew) *rew = out.reward;
  if (done) *done = out.done;
  if (terms) memcpy(terms, out.rewards, sizeof(out.rewards));
  return x_after;
}

// Gather the pack inputs from a physical state.
static void gather(const MV& m, const double* s, const double* aux, Kin& k, double* part_xyz,
                   int& n_parts, double* quat, double* pos, double* vel, double* jq, double* jqd,
                   double* head_z = nullptr) {
  forward_kinematics(m, s, k);
  if (head_z) *head_z = m.head_link >= 0 ? k.c[m.head_link + 1].z : 0.0;
  n_parts = 0;
  for (int p = 0; p < m.NP; p++) {
    V3 c = k.c[m.part_link[p] + 1];
    part_xyz[3 * n_parts] = c.x; part_xyz[3 * n_parts + 1] = c.y; part_xyz[3 * n_parts + 2] = c.z;
    n_parts++;
  }
  if (m.floor && aux[3] != 0.0) {  // gym_locomotion_envs.py:30-31: floor joins robot.parts
    part_xyz[3 * n_parts] = part_xyz[3 * n_parts + 1] = part_xyz[3 * n_parts + 2] = 0.0;
    n_parts++;
  }
  int b = m.robot_body + 1;
  // getBasePositionAndOrientation returns the base's own quaternion (its sign as integrated);
  // a link's orientation comes from its frame
  if (b == 0) memcpy(quat, s + 3, 4 * sizeof(double));
  else m3_to_quat(k.R[b], quat);
  pos[0] = k.c[b].x; pos[1] = k.c[b].y; pos[2] = k.c[b].z;
  vel[0] = k.v[b].x; vel[1] = k.v[b].y; vel[2] = k.v[b].z;
  const double* q = s + PBG_BASE_WORDS;
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = q[m.NJ + m.obs_dof[i]]; }
}

// Reset envs to the load snapshot with the given ordered-joint positions qinit[n][NR]
// (gym_locomotion_envs.py:22-39, robot_locomotors.py:16-24).  Writes the reset obs.
// mask (nullable): reset only the envs with mask[e] != 0 (auto-reset of the CPU baseline).
int pbg_oracle_reset_mask(int robot, int n, double* state, double* aux, const double* qinit, float* obs,
                          const uint8_t* mask) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  int SD = PBG_STATE_WORDS(m.NJ, m.harder), AD = PBG_AUX_RECORD_WORDS(m.NF, m.flagrun, m.harder);
  for (int e = 0; e < n; e++) {
    if (mask && !mask[e]) continue;
    if (g_cache && (size_t)e < g_cache_n) memset(g_cache + (size_t)e * 4 * MAXCAND, 0, sizeof(double) * 4 * MAXCAND);
    double* s = state + (size_t)e * SD;
    double* a = aux + (size_t)e * AD;
    for (int i = 0; i < 3; i++) s[i] = m.base_pos[i];
    for (int i = 0; i < 4; i++) s[3 + i] = m.base_quat[i];
    for (int i = 7; i < SD; i++) s[i] = 0.0;
    if (m.harder) {  // restoreState + resetBasePositionAndOrientation(cube, [-1.5, 0, 0.05], [0, 0, 0, 1]) (:241)
      double* cs = s + PBG_BASE_WORDS + 2 * m.NJ;
      cs[0] = PBG_CUBE_X0; cs[1] = PBG_CUBE_Y0; cs[2] = PBG_CUBE_Z0; cs[6] = 1.0;
    }
    // robot_pendula.py:16 (swingup: 3.1415 + u)
    for (int r = 0; r < m.NR; r++) s[PBG_BASE_WORDS + m.reset_dof[r]] = m.reset_offset[r] + qinit[(size_t)e * m.NR + r];
    float* ob = obs + (size_t)e * m.OBS;
    a[2] = 0.0;
    a[AD - 1] += 1.0;  // episodes started (the kernels' reset-noise Philox counter)
    for (int i = 0; i < m.NF; i++) a[4 + i] = 0.0;
    if (m.kind == 1) { pendulum_pack(m, s, ob, nullptr, nullptr); a[3] = 1.0; continue; }
    if (m.kind == 2) { a[0] = mujoco_planar_pack(m, s, 0.0, nullptr, ob, nullptr, nullptr); a[3] = 1.0; continue; }
    static thread_local Kin k;
    double part_xyz[3 * (MAXL + 2)], quat[4], pos[3], vel[3], jq[MAXD], jqd[MAXD];
    int n_parts;
    double head_z;
    gather(m, s, a, k, part_xyz, n_parts, quat, pos, vel, jq, jqd, &head_z);
    float feet_prev[8] = {0}, feet_out[8];
    pbg_pack_in in = {part_xyz, n_parts, quat, pos, vel, jq, jqd, feet_prev, nullptr, nullptr, 0.0,
                      m.z0fixed, PBG_WALK_TARGET_X, PBG_WALK_TARGET_Y, s + 10, head_z};
    pbg_pack_out out;
    out.obs = ob; out.feet_out = feet_out;
    Flag fl = load_flag(m, a);
    if (m.flagrun) flag_draw(e, fl);  // robot_specific_reset -> flag_reposition (:199-201)
    // HumanoidFlagrunHarder.robot_specific_reset (:237-248): frame, counters, crawl state
    Harder hd = load_harder(m, a);
    hd.frame = 0; hd.onground = 0; hd.crawl_start = NAN; hd.crawl_ignored = 0.0;
    flag_pack(robot, m, &in, &out, fl, e, nullptr, m.harder ? &hd : nullptr);
    store_flag(m, a, fl);
    if (m.harder) {
      out.potential = harder_potential(hd, out.potential, out.body_xyz[2]);  // env_bases.py:70
      store_harder(m, a, hd);
    }
    a[0] = out.potential;
    a[1] = out.initial_z;
    a[3] = 1.0;  // the floor is in robot.parts from now on
  }
  return 0;
}

int pbg_oracle_reset(int robot, int n, double* state, double* aux, const double* qinit, float* obs) {
  return pbg_oracle_reset_mask(robot, n, state, aux, qinit, obs, nullptr);
}

// One env step for each of n envs: apply_action, stepSimulation (substeps), pack.
// ncontact (nullable): contacts detected in the last sub-step, per env.
// csig (nullable): per env the contact-set signature of the step (sim_params.h pbg_contact_hash);
// rew_terms (nullable): [n][5] the terms the reward sums (the reference's self.rewards).
// precision: 64 = the float64 oracle; 32 = the same physics in IEEE float32 (the pack stays
// float64, as in the kernels) -- the parity tests' conditioning probe; 33 = float32 Monte Carlo
// arithmetic (mca.h: every operation randomly rounded to a float32 neighbour, stream seeded by
// pbg_oracle_set_mca_seed and the env index) -- the parity tests' outlier explanation.
// asig (nullable): per env the solver active-set signature (sim_params.h pbg_solver_event).
int pbg_oracle_step_ex(int robot, int n, double* state, double* aux, const float* act, float* obs, double* rew,
                       uint8_t* done, int32_t* ncontact, int nthreads, uint32_t* csig, double* rew_terms,
                       int precision, uint32_t* asig) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  int SD = PBG_STATE_WORDS(m.NJ, m.harder), AD = PBG_AUX_RECORD_WORDS(m.NF, m.flagrun, m.harder);
  if (g_opt[OPT_WARM] != 0.0 && g_cache_n < (size_t)n) {  // warm-start cache (rule study only)
    free(g_cache);
    g_cache = (double*)calloc((size_t)n * 4 * MAXCAND, sizeof(double));
    g_cache_n = g_cache ? (size_t)n : 0;
  }
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int e = 0; e < n; e++) {
    double* s = state + (size_t)e * SD;
    double* a = aux + (size_t)e * AD;
    const float* ac = act + (size_t)e * m.NA;
    uint8_t slot_active[MAXS];
    uint32_t sig = 0;
    double* cache = g_cache && (size_t)e < g_cache_n ? g_cache + (size_t)e * 4 * MAXCAND : nullptr;
    uint32_t as = 0;
    int nc;
    if (precision == 32) {
      nc = physics_step<float>(m, s, ac, slot_active, &sig, nullptr, &as);
    } else if (precision == 33) {
      g_mca_state = g_mca_seed * 0x9E3779B97F4A7C15ull + (uint64_t)e * 0xD1B54A32D192ED03ull + 1;
      nc = physics_step<Mca>(m, s, ac, slot_active, &sig, nullptr, &as);
    } else {
      nc = physics_step<double>(m, s, ac, slot_active, &sig, cache, &as);
    }
    if (asig) asig[e] = as;
    if (ncontact) ncontact[e] = nc;
    if (csig) csig[e] = sig;
    double* terms = rew_terms ? rew_terms + (size_t)e * 5 : nullptr;
    a[2] += 1.0;
    float* ob = obs + (size_t)e * m.OBS;
    if (m.kind == 1) { pendulum_pack(m, s, ob, rew + e, done + e, terms); continue; }
    if (m.kind == 2) { a[0] = mujoco_planar_pack(m, s, a[0], ac, ob, rew + e, done + e, terms); continue; }
    uint8_t feet_new[8];
    for (int f = 0; f < m.NF; f++) {
      feet_new[f] = 0;
      for (int sl = 0; sl < m.NS; sl++)
        if (m.slot_link[sl] == m.foot_link[f] && slot_active[sl]) feet_new[f] = 1;
    }
    static thread_local Kin k;
    double part_xyz[3 * (MAXL + 2)], quat[4], pos[3], vel[3], jq[MAXD], jqd[MAXD];
    int n_parts;
    double head_z;
    gather(m, s, a, k, part_xyz, n_parts, quat, pos, vel, jq, jqd, &head_z);
    float feet_prev[8], feet_out[8];
    for (int f = 0; f < m.NF; f++) feet_prev[f] = (float)a[4 + f];
    pbg_pack_in in = {part_xyz, n_parts, quat, pos, vel, jq, jqd, feet_prev, feet_new, ac,
                      a[0], a[1], PBG_WALK_TARGET_X, PBG_WALK_TARGET_Y, s + 10, head_z};
    pbg_pack_out out;
    out.obs = ob; out.feet_out = feet_out;
    Flag fl = load_flag(m, a);
    Harder hd = load_harder(m, a);
    flag_pack(robot, m, &in, &out, fl, e, nullptr, m.harder ? &hd : nullptr);
    store_flag(m, a, fl);
    if (m.harder) {
      (void)harder_step(m, &in, &out, hd, e, s + PBG_BASE_WORDS + 2 * m.NJ, nullptr);
      store_harder(m, a, hd);
    }
    rew[e] = out.reward;
    done[e] = out.done;
    if (terms) memcpy(terms, out.rewards, sizeof(out.rewards));
    a[0] = out.potential;
    for (int f = 0; f < m.NF; f++) a[4 + f] = feet_out[f];
  }
  return 0;
}

// Contact diagnostics of the next step calls (rule study, tools/walker_diag.py): out holds cap
// records of 10 doubles (see g_diag); returns the records written since the last call and
// re-arms the buffer (out NULL: off).
int pbg_oracle_contact_diag(double* out, int cap) {
  const int n = g_diag_n;
  g_diag = out; g_diag_cap = cap; g_diag_n = 0;
  return n;
}

// Seed of the Monte Carlo arithmetic stream (precision 33); env e of a step call draws from
// the stream keyed by (seed, e).
void pbg_oracle_set_mca_seed(uint64_t seed) { g_mca_seed = seed; }

int pbg_oracle_step(int robot, int n, double* state, double* aux, const float* act, float* obs, double* rew,
                    uint8_t* done, int32_t* ncontact, int nthreads, uint32_t* csig, double* rew_terms) {
  return pbg_oracle_step_ex(robot, n, state, aux, act, obs, rew, done, ncontact, nthreads, csig, rew_terms, 64,
                            nullptr);
}

// Algorithmic FP32 work of the physics (apply_action + the sub-steps) of one env step from
// each of n states: the physics instantiated on the op-counting scalar (counted.h), single
// thread; the states are advanced.  out[7]: adds+subs, muls, divs, sqrts, sin/cos summed
// over the n envs, then the nonzero-operand adds and muls (counted.h).  (The float64
// observation/reward pack is not FP32 work and not counted.)
int pbg_oracle_count_flops(int robot, int n, double* state, const float* act, uint64_t* out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  const int SD = PBG_STATE_WORDS(m.NJ, m.harder);
  g_flops = FlopCount{0, 0, 0, 0, 0, 0, 0};
  for (int e = 0; e < n; e++) {
    uint8_t slot_active[MAXS];
    physics_step<Counted>(m, state + (size_t)e * SD, act + (size_t)e * m.NA, slot_active, nullptr, nullptr);
  }
  out[0] = g_flops.add; out[1] = g_flops.mul; out[2] = g_flops.div; out[3] = g_flops.sqrt; out[4] = g_flops.trans;
  out[5] = g_flops.add_nz; out[6] = g_flops.mul_nz;
  return 0;
}

// Joint-space dynamics at a state, for tests: M (NDOF x NDOF, row-major) and bias C.
int pbg_oracle_dynamics(int robot, const double* state, double* M_out, double* C_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  static thread_local double M[MAXD][MAXD];
  forward_kinematics(*mp, state, k);
  mass_and_bias(*mp, k, M, C_out);
  for (int i = 0; i < mp->NDOF; i++)
    for (int j = 0; j < mp->NDOF; j++) M_out[i * mp->NDOF + j] = M[i][j];
  return 0;
}

// Link COM world positions [NL+1][3] (base first) at a state, for tests.
int pbg_oracle_link_com(int robot, const double* state, double* out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) { out[3 * b] = k.c[b].x; out[3 * b + 1] = k.c[b].y; out[3 * b + 2] = k.c[b].z; }
  return 0;
}

}  // extern "C"
