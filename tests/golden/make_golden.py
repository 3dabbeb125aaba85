"""Generate the pack golden vectors from the reference's own Python.  Runs HERE only.

The reference's WalkerBaseBulletEnv / InvertedPendulumBulletEnv (and everything they
call: robot_bases.py, robot_locomotors.py, robot_pendula.py, env_bases.py,
scene_bases.py, scene_stadium.py) is imported from /root/reference unchanged.  Its
third-party dependencies are absent here, so they are replaced by stub modules:

* ``gym`` (0.9.5-style: Env.reset -> _reset, spaces.Box, utils.seeding.np_random),
* ``pybullet`` (constants plus getEulerFromQuaternion, restated from pybullet.c),
* ``pybullet_envs.bullet.bullet_client`` and ``pybullet_data``,

and the physics client is a scripted fake (``FakeClient``) that serves link / joint /
base states and contact lists drawn from a seeded RNG in the robot topology of
``pybullet-gym_amd/models/<robot>.json``.  Whatever the reference's Python computes from
those physics queries -- observation, reward terms, done, feet_contact, potential --
is recorded together with the exact inputs it read, into ``tests/golden/pack_<robot>.npz``.

These vectors pin the observation/reward/done pack (SURVEY.md section 8a rows a3,
a5-a15, Appendix C).  They do not pin the physics (pybullet is not available).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import math
import os
import sys
import types

sys.dont_write_bytecode = True  # never write into /root/reference

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
MODELS = os.path.join(REPO, "pybullet-gym_amd", "models")

ROBOTS = {
    "pendulum": ("pybulletgym.envs.roboschool.gym_pendulum_envs", "InvertedPendulumBulletEnv"),
    "hopper": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "HopperBulletEnv"),
    "halfcheetah": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "HalfCheetahBulletEnv"),
    "ant": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "AntBulletEnv"),
    "humanoid": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "HumanoidBulletEnv"),
    "walker2d": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "Walker2DBulletEnv"),
    "pendulum_swingup": ("pybulletgym.envs.roboschool.gym_pendulum_envs", "InvertedPendulumSwingupBulletEnv"),
    "double_pendulum": ("pybulletgym.envs.roboschool.gym_pendulum_envs", "InvertedDoublePendulumBulletEnv"),
    "humanoid_flagrun": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "HumanoidFlagrunBulletEnv"),
    "hopper_mujoco": ("pybulletgym.envs.mujoco.gym_locomotion_envs", "HopperMuJoCoEnv"),
    "walker2d_mujoco": ("pybulletgym.envs.mujoco.gym_locomotion_envs", "Walker2DMuJoCoEnv"),
    "halfcheetah_mujoco": ("pybulletgym.envs.mujoco.gym_locomotion_envs", "HalfCheetahMuJoCoEnv"),
    "ant_mujoco": ("pybulletgym.envs.mujoco.gym_locomotion_envs", "AntMuJoCoEnv"),
    "humanoid_mujoco": ("pybulletgym.envs.mujoco.gym_locomotion_envs", "HumanoidMuJoCoEnv"),
    "double_pendulum_mujoco": ("pybulletgym.envs.mujoco.gym_pendulum_envs", "InvertedDoublePendulumMuJoCoEnv"),
    "humanoid_flagrun_harder": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "HumanoidFlagrunHarderBulletEnv"),
    "atlas": ("pybulletgym.envs.roboschool.gym_locomotion_envs", "AtlasBulletEnv"),
}
CUBE_UID = 6


# ----------------------------------------------------------------------------- stubs
def euler_from_quaternion(q):
    """pybullet.getEulerFromQuaternion as written in pybullet.c (double precision)."""
    x, y, z, w = [float(v) for v in q]
    sqx, sqy, sqz, squ = x * x, y * y, z * z, w * w
    roll = math.atan2(2 * (y * z + w * x), squ - sqx - sqy + sqz)
    sarg = -2 * (x * z - w * y)
    pitch = -0.5 * 3.141592538 if sarg <= -1.0 else (0.5 * 3.141592538 if sarg >= 1.0 else math.asin(sarg))
    yaw = math.atan2(2 * (x * y + w * z), squ + sqx - sqy - sqz)
    return (roll, pitch, yaw)


def quaternion_from_euler(e):
    r, p, y = e
    cr, sr, cp, sp, cy, sy = (math.cos(r / 2), math.sin(r / 2), math.cos(p / 2), math.sin(p / 2),
                              math.cos(y / 2), math.sin(y / 2))
    return (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
            cr * cp * cy + sr * sp * sy)


def install_stubs():
    gym = types.ModuleType("gym")
    gym.__version__ = "0.9.5"

    class Env:
        def reset(self):
            return self._reset()

        def seed(self, seed=None):
            return self._seed(seed)

    gym.Env = Env
    spaces = types.ModuleType("gym.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high = np.asarray(low), np.asarray(high)
            self.shape = self.low.shape

    spaces.Box = Box
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")

    def np_random(seed=None):
        seed = 0 if seed is None else seed
        return np.random.RandomState(seed), seed

    seeding.np_random = np_random
    utils.seeding = seeding
    envs = types.ModuleType("gym.envs")
    registration = types.ModuleType("gym.envs.registration")
    registration.register = lambda **kw: None
    envs.registration = registration
    gym.spaces, gym.utils, gym.envs = spaces, utils, envs
    for name, mod in [("gym", gym), ("gym.spaces", spaces), ("gym.utils", utils),
                      ("gym.utils.seeding", seeding), ("gym.envs", envs),
                      ("gym.envs.registration", registration)]:
        sys.modules[name] = mod

    pb = types.ModuleType("pybullet")
    for i, c in enumerate(["POSITION_CONTROL", "VELOCITY_CONTROL", "TORQUE_CONTROL", "COV_ENABLE_RENDERING",
                           "COV_ENABLE_GUI", "COV_ENABLE_PLANAR_REFLECTION", "GUI", "DIRECT",
                           "ER_BULLET_HARDWARE_OPENGL"]):
        setattr(pb, c, i)
    pb.URDF_USE_SELF_COLLISION = 8
    pb.URDF_USE_SELF_COLLISION_EXCLUDE_ALL_PARENTS = 16
    pb.getEulerFromQuaternion = euler_from_quaternion
    pb.getQuaternionFromEuler = quaternion_from_euler
    sys.modules["pybullet"] = pb
    pe = types.ModuleType("pybullet_envs")
    pbb = types.ModuleType("pybullet_envs.bullet")
    bc = types.ModuleType("pybullet_envs.bullet.bullet_client")

    class BulletClient:  # replaced per env by FakeClient
        def __init__(self, connection_mode=None):
            raise RuntimeError("stub")

    bc.BulletClient = BulletClient
    pe.bullet, pbb.bullet_client = pbb, bc
    sys.modules.update({"pybullet_envs": pe, "pybullet_envs.bullet": pbb,
                        "pybullet_envs.bullet.bullet_client": bc})
    pdata = types.ModuleType("pybullet_data")
    pdata.getDataPath = lambda: "/nonexistent"
    sys.modules["pybullet_data"] = pdata


# ----------------------------------------------------------------------------- fake physics
def rand_quat(rng, tilt):
    yaw = rng.uniform(-math.pi, math.pi)
    roll, pitch = rng.normal(0, tilt), rng.normal(0, tilt)
    q = np.array(quaternion_from_euler((roll, pitch, yaw)))
    if rng.random() < 0.3:
        q = -q  # a quaternion and its negation are the same rotation
    return tuple(float(v) for v in q)


class FakeClient:
    """Scripted stand-in for pybullet's BulletClient: serves seeded synthetic states."""

    def __init__(self, t, rng):
        self.t = t
        self.rng = rng
        self._client = 7
        self.floor_uid, self.robot_uid = (0, 1) if t["floor"] else (-99, 0)
        self.L = t["NL"]
        self.q = np.zeros(self.L)
        self.qd = np.zeros(self.L)
        self.saved = None
        self.target_hook = None
        self.z_hook = None       # HumanoidFlagrunHarder: scripted torso height (up / crawling)
        self.cube_pose = ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
        self.cube_events = []    # (kind, value) of every cube reset call
        self.new_state(initial=True)

    # --- state script
    def new_state(self, initial=False):
        rng, L = self.rng, self.L
        big = rng.random() < 0.1
        self.base_pos = (float(rng.uniform(-3, 3) if not big else rng.choice([-2000.0, 1500.0, 999.5])),
                         float(rng.uniform(-3, 3)), float(rng.uniform(0.05, 1.6)))
        if self.z_hook is not None:
            self.base_pos = (self.base_pos[0], self.base_pos[1], float(self.z_hook(rng)))
        self.base_orn = rand_quat(rng, 0.9 if rng.random() < 0.3 else 0.2)
        vs = 30.0 if rng.random() < 0.1 else 2.0
        self.base_lin = tuple(float(v) for v in rng.normal(0, vs, 3))
        self.base_ang = tuple(float(v) for v in rng.normal(0, 2.0, 3))
        if self.target_hook is not None and not initial and rng.random() < 0.08:
            # HumanoidFlagrun: put the body next to the flag (walk_target_dist < 1 re-draws it)
            tx, ty = self.target_hook()
            self.base_pos = (float(tx + rng.uniform(-0.3, 0.3)), float(ty + rng.uniform(-0.3, 0.3)),
                             self.base_pos[2])
        self.link_pos = [tuple(float(v) for v in np.array(self.base_pos) + rng.normal(0, 0.5, 3)) for _ in range(L)]
        self.link_orn = [rand_quat(rng, 0.7) for _ in range(L)]
        self.link_lin = [tuple(float(v) for v in rng.normal(0, vs, 3)) for _ in range(L)]
        self.link_ang = [tuple(float(v) for v in rng.normal(0, 2, 3)) for _ in range(L)]
        if not initial:
            for j in range(L):
                lo, hi = self.t["_lo"][j], self.t["_hi"][j]
                if lo < hi:
                    span = hi - lo
                    self.q[j] = rng.uniform(lo - 0.3 * span, hi + 0.3 * span)
                else:
                    self.q[j] = rng.uniform(-4, 4)
                self.qd[j] = rng.normal(0, 5.0) if rng.random() > 0.05 else rng.choice([-120.0, 80.0])
            if rng.random() < 0.03:
                self.qd[rng.integers(L)] = float("nan")
        self.contacts = [int(rng.random() < 0.4) for _ in range(L)]
        self.self_contacts = [int(rng.random() < 0.2) for _ in range(L)]

    # --- world setup
    def configureDebugVisualizer(self, *a, **k): pass
    def setGravity(self, *a, **k): pass
    def setDefaultContactERP(self, *a, **k): pass
    def setPhysicsEngineParameter(self, *a, **k): pass
    def changeDynamics(self, *a, **k): pass
    def changeVisualShape(self, *a, **k): pass
    def setJointMotorControl2(self, *a, **k): pass
    def loadSDF(self, path): return (self.floor_uid,)
    def loadMJCF(self, path, flags=0): return (self.robot_uid,)
    def loadURDF(self, path, pos=None, *a, **k):
        if "atlas" in str(path):  # URDFBasedRobot.reset (robot_bases.py:145-164)
            return self.robot_uid
        if "cube" in str(path):  # HumanoidFlagrunHarder's attacking cube (gym_utils.get_cube)
            self.cube_pose = (tuple(float(v) for v in pos), (0.0, 0.0, 0.0, 1.0))
            return CUBE_UID
        return 5  # HumanoidFlagrun's flag sphere (no collision)

    def resetBasePositionAndOrientation(self, uid, pos, orn):
        if uid == CUBE_UID:
            self.cube_pose = (tuple(float(v) for v in pos), tuple(float(v) for v in orn))
            self.cube_events.append(("pose", self.cube_pose[0]))

    def resetBaseVelocity(self, uid, linearVelocity=(0, 0, 0), angularVelocity=(0, 0, 0)):
        if uid == CUBE_UID:
            self.cube_events.append(("vel", tuple(float(v) for v in linearVelocity),
                                     tuple(float(v) for v in angularVelocity)))
    def saveState(self): return 3
    def restoreState(self, sid): self.q[:] = 0.0; self.qd[:] = 0.0
    def stepSimulation(self): self.new_state()

    def getNumJoints(self, uid):
        return self.L if uid == self.robot_uid else 0

    def getBodyInfo(self, uid):
        if uid == CUBE_UID:
            return (b"baseLink", b"cube.urdf")
        return (b"floor", b"floor_obj") if uid == self.floor_uid else (b"base", self.t["key"].encode())

    def getJointInfo(self, uid, j):
        t = self.t
        lo, hi = t["_lo"][j], t["_hi"][j]
        vmax = float(t.get("link_max_velocity", [0.0] * t["NL"])[j])  # URDF <limit velocity> (Atlas)
        return (j, t["_jname"][j].encode(), t["link_jtype"][j], 7 + j, 6 + j, 1, 0.0, 0.0, lo, hi, 0.0, vmax,
                t["link_name"][j].encode(), (0.0, 0.0, 1.0), (0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0), t["link_parent"][j])

    # --- state queries
    def resetJointState(self, uid, j, targetValue=0.0, targetVelocity=0.0):
        self.q[j], self.qd[j] = targetValue, targetVelocity

    def getJointState(self, uid, j):
        return (float(self.q[j]), float(self.qd[j]), (0.0,) * 6, 0.0)

    def getBasePositionAndOrientation(self, uid):
        if uid == self.floor_uid:
            return ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
        if uid == CUBE_UID:
            return self.cube_pose
        return (self.base_pos, self.base_orn)

    def getBaseVelocity(self, uid):
        return (self.base_lin, self.base_ang)

    def getLinkState(self, uid, j, computeLinkVelocity=0):
        out = (self.link_pos[j], self.link_orn[j], (0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0), self.link_pos[j], self.link_orn[j])
        if computeLinkVelocity:
            out = out + (self.link_lin[j], self.link_ang[j])
        return out

    def getContactPoints(self, bodyA, bodyB=-1, linkIndexA=-2, linkIndexB=-2):
        pts = []
        if linkIndexA >= 0 and self.contacts[linkIndexA]:
            pts.append((0, bodyA, self.floor_uid, linkIndexA, -1, (0, 0, 0), (0, 0, 0), (0, 0, 1), 0.001, 1.0))
        if linkIndexA >= 0 and self.self_contacts[linkIndexA]:  # robot-robot contact: must not count
            pts.append((0, bodyA, self.robot_uid, linkIndexA, (linkIndexA + 1) % self.L, (0, 0, 0), (0, 0, 0),
                        (0, 0, 1), 0.001, 1.0))
        return pts


# ----------------------------------------------------------------------------- driver
def load_tables(key):
    with open(os.path.join(MODELS, f"{key}.json")) as f:
        t = json.load(f)
    L = t["NL"]
    t["_lo"], t["_hi"], t["_jname"] = [0.0] * L, [-1.0] * L, []
    for j in range(L):
        d = t["link_dof"][j]
        if d >= 0 and t["dof_limited"][d]:
            t["_lo"][j], t["_hi"][j] = t["dof_lower"][d], t["dof_upper"][d]
    # joint names as pybullet reports them (getJointInfo[1])
    import importlib
    sys.path.insert(0, REPO)
    pkg = importlib.import_module("pybulletgym_amd")
    from pybulletgym_amd import robots
    spec = robots.spec_for(key)
    model = robots.compile_model(spec)
    t["_jname"] = [l.joint_name for l in model.links]
    return t


def generate(key, episodes=3, steps=40, seed=1234):
    modname, clsname = ROBOTS[key]
    import importlib
    envmod = importlib.import_module(modname)
    env_bases = importlib.import_module("pybulletgym.envs.roboschool.env_bases")
    t = load_tables(key)
    rng = np.random.default_rng(seed)
    fake = FakeClient(t, rng)
    env_bases.bullet_client.BulletClient = lambda connection_mode=None: fake
    env = getattr(envmod, clsname)()
    robot = env.robot
    if t.get("flagrun"):
        fake.target_hook = lambda: (robot.walk_target_x, robot.walk_target_y)
    rec = {k: [] for k in ("kind", "part_xyz", "n_parts", "body_quat", "body_pos", "body_vel", "jq", "jqd",
                           "feet_prev", "feet_new", "act", "potential_old", "initial_z_in", "obs", "reward",
                           "done", "potential", "feet_out", "initial_z_out", "rewards", "flag_in", "flag_out",
                           "body_avel", "harder_in", "harder_out", "head_z")}
    part_names = []
    captured = {}
    calc_cls = type(robot)
    orig_calc = calc_cls.calc_state

    orig_pot = calc_cls.calc_potential

    def spy_calc_potential(self):  # MuJoCo planar: x-progress of robot_body
        captured["x_before"] = float(self.pos_after)
        r = orig_pot(self)
        captured["x_after"] = float(self.pos_after)
        return r

    def spy_calc_state(self):
        if t["kind"] == 2:  # MuJoCo planar: every ordered joint incl. the ignored root joints
            captured["jq"] = np.array([j.get_position() for j in self.ordered_joints], dtype=np.float64)
            captured["jqd"] = np.array([j.get_velocity() for j in self.ordered_joints], dtype=np.float64)
        elif t["kind"] in (0, 3):
            if t["kind"] == 3:  # MuJoCo Ant / Humanoid also read the torso's angular velocity
                captured["body_avel"] = np.array(self.parts["torso"].get_velocity()[1], dtype=np.float64)
            captured["part_xyz"] = np.array([p.pose().xyz() for p in self.parts.values()], dtype=np.float64)
            captured["part_names"] = list(self.parts.keys())
            captured["body_quat"] = np.array(self.robot_body.pose().orientation(), dtype=np.float64)
            captured["body_pos"] = np.array(self.robot_body.pose().xyz(), dtype=np.float64)
            captured["body_vel"] = np.array(self.robot_body.speed(), dtype=np.float64)
            js = [j.get_state() for j in self.ordered_joints]
            captured["jq"] = np.array([s[0] for s in js]); captured["jqd"] = np.array([s[1] for s in js])
            captured["feet_prev"] = np.array(self.feet_contact, dtype=np.float32)
            captured["initial_z_in"] = np.nan if self.initial_z is None else float(self.initial_z)
            if t.get("flagrun"):  # walk target and flag_timeout before HumanoidFlagrun.calc_state
                captured["flag_before"] = (float(self.walk_target_x), float(self.walk_target_y),
                                           float(self.flag_timeout))
            if t.get("harder"):  # HumanoidFlagrunHarder bookkeeping before this calc_state
                cs = self.crawl_start_potential
                captured["harder_before"] = [float(self.frame), float(self.on_ground_frame_counter),
                                             np.nan if cs is None else float(cs), float(self.crawl_ignored_potential)]
        else:
            js = [self.j1, self.j2, self.slider] if hasattr(self, "j2") else [self.j1, self.slider]
            captured["jq"] = np.array([j.get_state()[0] for j in js])
            captured["jqd"] = np.array([j.get_state()[1] for j in js])
            if hasattr(self, "pole2"):  # InvertedDoublePendulum reads pole2.pose().xyz()
                captured["body_pos"] = np.array(self.pole2.pose().xyz(), dtype=np.float64)
        return orig_calc(self)

    calc_cls.calc_state = spy_calc_state
    orig_alive = calc_cls.alive_bonus
    if t.get("harder"):
        def spy_alive_bonus(self, z, pitch):
            # the launch draws of np_random.uniform inside alive_bonus, and the cube resets it makes
            rs = self.np_random
            draws = []

            class Recorder:  # delegates to the env's RandomState, recording uniform() values
                def uniform(self, *a, **k):
                    v = rs.uniform(*a, **k)
                    draws.extend(np.atleast_1d(v).astype(np.float64).tolist())
                    return v

                def __getattr__(self, name):
                    return getattr(rs, name)
            self.np_random = Recorder()
            fake.cube_events.clear()
            try:
                return orig_alive(self, z, pitch)
            finally:
                self.np_random = rs
                captured["launch_draws"] = draws
                captured["launch_events"] = list(fake.cube_events)
        calc_cls.alive_bonus = spy_alive_bonus
    if t["kind"] == 2:
        calc_cls.calc_potential = spy_calc_potential
    NPMAX = t["NP"] + 1
    nf = max(1, t["NF"])

    def push(kind, act, pot_old, obs, reward, done):
        rec["kind"].append(kind)
        if t["kind"] == 3:
            rec["body_avel"].append(captured["body_avel"])
        if t["kind"] in (0, 3):
            px = np.zeros((NPMAX, 3))
            n = len(captured["part_xyz"])
            px[:n] = captured["part_xyz"]
            rec["part_xyz"].append(px); rec["n_parts"].append(n)
            for k in ("body_quat", "body_pos", "body_vel"):
                rec[k].append(captured[k])
            fp = np.zeros(nf, np.float32); fp[:t["NF"]] = captured["feet_prev"]
            rec["feet_prev"].append(fp)
            fo = np.zeros(nf, np.float32); fo[:t["NF"]] = robot.feet_contact
            rec["feet_out"].append(fo)
            fn = np.zeros(nf, np.uint8)
            for i, f in enumerate(robot.foot_list):
                fn[i] = fake.contacts[t["link_name"].index(f)]
            rec["feet_new"].append(fn)
            rec["initial_z_in"].append(captured["initial_z_in"])
            if t.get("flagrun"):
                bx, by, bt = captured["flag_before"]
                after = (float(robot.walk_target_x), float(robot.walk_target_y), float(robot.flag_timeout))
                moved = after[:2] != (bx, by)
                # the draw a reposition took (NaN: none happened during this calc_state)
                rec["flag_in"].append([bx, by, bt, after[0] if moved else np.nan, after[1] if moved else np.nan])
                rec["flag_out"].append(list(after))
            if t.get("harder"):
                dr = captured.pop("launch_draws", []) if kind == 1 else []
                ev = captured.pop("launch_events", []) if kind == 1 else []
                assert len(dr) in (0, 5), dr
                rec["harder_in"].append(captured["harder_before"] + (dr if dr else [np.nan] * 5))
                cs = robot.crawl_start_potential
                pos = [e[1] for e in ev if e[0] == "pose"]
                vel = [e[1] for e in ev if e[0] == "vel"]
                assert len(pos) == len(vel) == (1 if dr else 0), ev
                rec["harder_out"].append([float(robot.frame), float(robot.on_ground_frame_counter),
                                          np.nan if cs is None else float(cs), float(robot.crawl_ignored_potential),
                                          1.0 if dr else 0.0] + (list(pos[0]) + list(vel[0]) if dr else [np.nan] * 6))
            if t.get("head_link", -1) >= 0:  # Atlas alive_bonus: the head part's height (getLinkState[0])
                rec["head_z"].append(float(fake.link_pos[t["head_link"]][2]))
            rec["initial_z_out"].append(float(robot.initial_z))
            part_names.append(captured["part_names"])
        elif t["kind"] == 2:
            rec["body_pos"].append(np.array([captured["x_after"], 0.0, 0.0]))
        elif "body_pos" in captured:
            rec["body_pos"].append(captured["body_pos"])
        rec["jq"].append(captured["jq"]); rec["jqd"].append(captured["jqd"])
        rec["act"].append(np.zeros(t["NA"], np.float32) if act is None else act)
        rec["potential_old"].append(captured["x_before"] if t["kind"] == 2 else pot_old)
        rec["obs"].append(np.asarray(obs))
        rec["reward"].append(reward)
        rec["done"].append(bool(done))
        rec["potential"].append(captured["x_after"] if t["kind"] == 2 else float(getattr(env, "potential", 0.0)))
        rw = getattr(env, "rewards", [0.0] * 5)
        rr = np.zeros(5); rr[:len(rw)] = rw
        rec["rewards"].append(rr)

    arng = np.random.default_rng(seed + 1)
    if t.get("harder"):
        # up (no crawl, cube launches every 30 frames after frame 100) most of the time, on the
        # ground in bursts; the last episode stays down until the 170-frame counter ends it
        state = {"ep": 0}
        fake.z_hook = lambda r: (r.uniform(0.05, 0.79) if state["ep"] == episodes - 1 or r.random() < 0.25
                                 else r.uniform(0.81, 1.5))
    if key == "atlas":  # head above 1.3 m (alive +4 - knees at limit) in most calls
        fake.z_hook = lambda r: r.uniform(0.3, 1.2) if r.random() < 0.25 else r.uniform(1.6, 2.4)
    for ep in range(episodes):
        if t.get("harder"):
            state["ep"] = ep
        obs = env.reset()
        push(0, None, np.nan, obs, 0.0, False)
        for s in range(steps):
            if arng.random() < 0.05:
                a = np.zeros(t["NA"], np.float32)
            else:
                a = arng.uniform(-1.5, 1.5, t["NA"]).astype(np.float32)
            pot_old = float(getattr(env, "potential", 0.0))
            obs, r, done, info = env.step(a)
            push(1, a, pot_old, obs, float(r), done)
    calc_cls.calc_state = orig_calc
    calc_cls.calc_potential = orig_pot
    calc_cls.alive_bonus = orig_alive
    out = {k: np.array(v) for k, v in rec.items() if len(v)}
    out["part_names"] = np.array(["|".join(p) for p in part_names]) if part_names else np.array([])
    out["numpy_version"] = np.array(np.__version__)
    return out


def main():
    install_stubs()
    sys.path.insert(0, REF)
    for key in (sys.argv[1:] or ROBOTS):
        # flagrun: long enough for flag_timeout (150 calc_states) to run out
        if key == "humanoid_flagrun":
            data = generate(key, episodes=2, steps=170)
        elif key == "humanoid_flagrun_harder":  # launches from frame 120; the 170-frame ground limit
            data = generate(key, episodes=3, steps=200)
        else:
            data = generate(key)
        path = os.path.join(HERE, f"pack_{key}.npz")
        np.savez_compressed(path, **data)
        print(key, "calls", len(data["kind"]), "->", os.path.relpath(path, REPO))


if __name__ == "__main__":
    main()
