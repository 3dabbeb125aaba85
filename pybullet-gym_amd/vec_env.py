"""Batched, device-resident locomotion envs over libpbg_amd.so.

``VecEnv(env_id, num_envs)`` holds the state of num_envs independent copies of one
``*PyBulletEnv-v0`` env on one GPU and steps all of them with one kernel launch per
``step()``.  Actions, observations, rewards and done flags are PyTorch-ROCm tensors
that never leave HBM.  Semantics per env are those of the reference's
``WalkerBaseBulletEnv`` (gym_locomotion_envs.py:22-114) behind gym's TimeLimit
(envs/__init__.py ``max_episode_steps``), with gym-VectorEnv style auto-reset.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native
from .spaces import Box


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


@dataclass
class StepResult:
    obs: torch.Tensor
    reward: torch.Tensor
    done: torch.Tensor
    truncated: torch.Tensor
    terminal_obs: torch.Tensor


class VecEnv:
    """``num_envs`` copies of ``env_id`` on one GPU.

    ``step`` returns views of the env's own output buffers (``obs``, ``reward``, ``done``,
    ``truncated``, ``terminal_obs``): the next ``step`` or ``reset`` overwrites them in place,
    so a learner that keeps a batch across steps must ``clone()`` it (the buffers are never
    reallocated, which is what lets a step be captured into a HIP graph).

    ``sim_params``: a dict overriding fields of the reference's scene (``gravity``, ``timestep``,
    ``frame_skip``, ``solver_iterations``, ``contact_erp``, ``joint_limit_erp``; include/pbg.h
    pbg_sim_params_t, scene_bases.py:8-18,58-73), or a ``_native.SimParams``; None = the
    reference's values (``self.sim_params`` holds the ones in force).

    ``precision``: 64 (the default: float64 physics state and arithmetic, the reference's btScalar
    precision, scene_bases.py:75-76 -> stepSimulation) or 32 (float32 physics, the opt-in fast mode);
    pbg_create_v2.  Observations stay float32 and the reward pack float64 in both, as the reference's
    (robot_locomotors.py:64, gym_locomotion_envs.py:99-105).

    ``kernel`` / ``lds_rows`` / ``gang_dist`` / ``gang_lanes`` are test and diagnostic launch
    options (``pbg_create_debug``): the lane-per-env (0) or gang (2) kernel instead of the default,
    a cap on LDS-resident contact rows, forced replicated (0) / distributed (1) gang dynamics, the
    gang width (16 or 32 lanes per env; 32 for the Humanoid family only).
    """

    def __init__(self, env_id: str, num_envs: int, device="cuda:0", seed: int = 0, env_offset: int = 0,
                 autoreset: bool = True, kernel: int = -1, lds_rows: int = -1, gang_dist: int = -1,
                 sim_params=None, gang_lanes: int = -1, precision: int = 64):
        if not torch.cuda.is_available():
            raise _native.PbgError("VecEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.env_id = env_id
        self.device = torch.device(device)
        self.num_envs = int(num_envs)
        self.autoreset = autoreset
        L = _native.lib()
        h = ctypes.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        opts = _native.CreateOpts(int(precision), int(kernel), int(lds_rows), int(gang_dist), int(gang_lanes))
        sp = sim_params if isinstance(sim_params, _native.SimParams) else _native.sim_params(env_id, sim_params)
        _native.check(L.pbg_create_v2(_native.env_id_bytes(env_id), self.num_envs, idx, seed, env_offset,
                                      ctypes.byref(sp), ctypes.byref(opts), ctypes.byref(h)), "pbg_create")
        self._h = h
        self.precision = L.pbg_precision(h)
        self.sim_params = _native.SimParams()
        _native.check(L.pbg_get_sim_params(h, ctypes.byref(self.sim_params)), "pbg_get_sim_params")
        info = _native.Info()
        _native.check(L.pbg_info(h, ctypes.byref(info)), "pbg_info")
        self.info = info
        # robot_bases.py:24-27
        self.action_space = Box(-np.ones(info.action_dim, np.float32), np.ones(info.action_dim, np.float32))
        self.observation_space = Box(np.full(info.obs_dim, -np.inf, np.float32), np.full(info.obs_dim, np.inf, np.float32))
        kw = dict(device=self.device)
        n = self.num_envs
        self.obs = torch.zeros((n, info.obs_dim), dtype=torch.float32, **kw)
        self.reward = torch.zeros(n, dtype=torch.float32, **kw)
        self.done = torch.zeros(n, dtype=torch.uint8, **kw)
        self.truncated = torch.zeros(n, dtype=torch.uint8, **kw)
        self.terminal_obs = torch.zeros((n, info.obs_dim), dtype=torch.float32, **kw)
        self.reward64 = None
        self.ncontact = None
        self.reward_terms = None
        self.contact_sig = None
        self._io = _native.StepIO()

    @staticmethod
    def default_sim_params(env_id: str) -> dict:
        """The reference's scene for env_id as a dict (pbg_default_sim_params; no GPU needed)."""
        return _native.default_sim_params(env_id).as_dict()

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            _native.lib().pbg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- gym-like API
    def reset(self, mask: torch.Tensor = None, init_q: torch.Tensor = None) -> torch.Tensor:
        """Reset all envs (or those with mask != 0).  init_q: [n, reset_dofs] float32 joint
        positions replacing the U(-0.1, 0.1) draw (trace replay)."""
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        if init_q is not None:
            init_q = init_q.to(device=self.device, dtype=torch.float32).contiguous()
            assert init_q.shape == (self.num_envs, self.info.reset_dofs)
        _native.check(_native.lib().pbg_reset(self._h, _ptr(mask), _ptr(init_q), _ptr(self.obs),
                                              _stream(self.device)), "pbg_reset")
        return self.obs

    def step(self, actions: torch.Tensor, want_reward64: bool = False, want_contacts: bool = False,
             want_terms: bool = False) -> StepResult:
        """One env step of every env.  Optional outputs (kept on the object): ``reward64``
        (float64 reward), ``ncontact`` / ``contact_sig`` (contacts of the last sub-step and the
        step's contact-set signature, want_contacts), ``reward_terms`` ([n, 5] float64: the
        reference's per-term ``self.rewards``, gym_locomotion_envs.py:99-105; want_terms)."""
        a = actions
        if a.dtype != torch.float32 or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        assert a.shape == (self.num_envs, self.info.action_dim), a.shape
        io = self._io
        io.act = a.data_ptr()
        io.obs = self.obs.data_ptr()
        io.rew = self.reward.data_ptr()
        io.done = self.done.data_ptr()
        io.trunc = self.truncated.data_ptr()
        io.term_obs = self.terminal_obs.data_ptr() if self.autoreset else None
        if want_reward64 and self.reward64 is None:
            self.reward64 = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        if want_contacts and self.ncontact is None:
            self.ncontact = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
            self.contact_sig = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)  # uint32 bits
        if want_terms and self.reward_terms is None:
            self.reward_terms = torch.zeros((self.num_envs, 5), dtype=torch.float64, device=self.device)
        io.rew64 = self.reward64.data_ptr() if want_reward64 else None
        io.ncontact = self.ncontact.data_ptr() if want_contacts else None
        io.csig = self.contact_sig.data_ptr() if want_contacts else None
        io.rew_terms = self.reward_terms.data_ptr() if want_terms else None
        io.autoreset = 1 if self.autoreset else 0
        _native.check(_native.lib().pbg_step_ex(self._h, ctypes.byref(io), _stream(self.device)), "pbg_step")
        return StepResult(self.obs, self.reward, self.done, self.truncated, self.terminal_obs)

    def capture(self, actions) -> "torch.cuda.CUDAGraph":
        """Record ``len(actions)`` consecutive steps (one action batch each, device tensors
        that stay alive) into a HIP graph; ``graph.replay()`` then runs them with a single
        launch from the host.  The step has no host synchronisation or allocation, so it
        captures as is; outputs land in the usual ``obs``/``reward``/``done`` buffers."""
        self.step(actions[0])  # first-step lazy buffers outside the capture
        dev = self.device
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for a in actions:
                self.step(a)
        torch.cuda.current_stream(dev).wait_stream(s)
        return g

    # ---------------------------------------------------------------- state records
    def get_state(self):
        phys = torch.zeros((self.num_envs, self.info.state_words), dtype=torch.float64, device=self.device)
        aux = torch.zeros((self.num_envs, self.info.aux_words), dtype=torch.float64, device=self.device)
        _native.check(_native.lib().pbg_get_state(self._h, _ptr(phys), _ptr(aux), _stream(self.device)),
                      "pbg_get_state")
        return phys, aux

    def state_dict(self) -> dict:
        """Checkpoint of every env (pybullet saveState generalised): the state records plus the
        env id, the record-layout version (include/pbg.h PBG_RECORD_VERSION) and the scene
        parameters and physics precision the states were simulated under."""
        phys, aux = self.get_state()
        return {"env_id": self.env_id, "record_version": int(self.info.record_version), "phys": phys, "aux": aux,
                "sim_params": self.sim_params.as_dict(), "precision": self.precision}

    def load_state_dict(self, sd: dict):
        """Restore a state_dict(); refuses a checkpoint of another env id, record layout, scene or
        physics precision (a float64 state rounded into a float32 handle is not the state that was
        saved; a checkpoint without "sim_params" / "precision" is taken to be of the reference's
        scene / of float32, the keys' round-4 defaults)."""
        if sd.get("env_id") != self.env_id:
            raise _native.PbgError(f"checkpoint of {sd.get('env_id')!r} loaded into {self.env_id!r}")
        if sd.get("record_version") != self.info.record_version:
            raise _native.PbgError(f"checkpoint record version {sd.get('record_version')} != library's "
                                   f"{self.info.record_version} (the aux record layout changed)")
        sp = sd.get("sim_params", self.default_sim_params(self.env_id))
        if sp != self.sim_params.as_dict():
            raise _native.PbgError(f"checkpoint scene {sp} != this handle's {self.sim_params.as_dict()}")
        if sd.get("precision", 32) != self.precision:
            raise _native.PbgError(f"checkpoint of a precision-{sd.get('precision', 32)} handle loaded into a "
                                   f"precision-{self.precision} one")
        self.set_state(sd["phys"], sd["aux"])

    def set_state(self, phys: torch.Tensor, aux: torch.Tensor = None):
        """phys / aux: [n, state_words] / [n, aux_words] float64 records (pbg_get_state layout).
        aux None: only the physical state is replaced; the handle keeps its bookkeeping,
        including the episode counter that keys the next reset's noise (include/pbg.h)."""
        phys = phys.to(device=self.device, dtype=torch.float64).contiguous()
        assert phys.shape == (self.num_envs, self.info.state_words)
        if aux is not None:
            aux = aux.to(device=self.device, dtype=torch.float64).contiguous()
            assert aux.shape == (self.num_envs, self.info.aux_words)
        _native.check(_native.lib().pbg_set_state(self._h, _ptr(phys), _ptr(aux), _stream(self.device)),
                      "pbg_set_state")


def sample_actions(action_dim: int, num_envs: int, steps: int, seed: int = 0x5EED, step0: int = 0,
                   env_offset: int = 0, device="cuda:0") -> torch.Tensor:
    """[steps, num_envs, action_dim] float32 U(-1, 1) on the device (pbg_sample_actions: Philox,
    counter (step0 + s, env_offset + e, ...), so a shard draws the same actions as a full batch)."""
    out = torch.empty((steps, num_envs, action_dim), dtype=torch.float32, device=device)
    _native.check(_native.lib().pbg_sample_actions(action_dim, num_envs, steps, seed, step0, env_offset,
                                                    _ptr(out), _stream(out.device)), "pbg_sample_actions")
    return out


def pack(env_id: str, in_rec: torch.Tensor) -> torch.Tensor:
    """Device observation/reward pack on explicit input records (golden-vector parity)."""
    L = _native.lib()
    iw, ow = ctypes.c_int(), ctypes.c_int()
    _native.check(L.pbg_pack_record_sizes(_native.env_id_bytes(env_id), ctypes.byref(iw), ctypes.byref(ow)),
                  "pbg_pack_record_sizes")
    assert in_rec.dtype == torch.float64 and in_rec.shape[1] == iw.value, (in_rec.shape, iw.value)
    in_rec = in_rec.contiguous()
    out = torch.zeros((in_rec.shape[0], ow.value), dtype=torch.float64, device=in_rec.device)
    _native.check(L.pbg_pack(_native.env_id_bytes(env_id), in_rec.shape[0], _ptr(in_rec), _ptr(out),
                             _stream(in_rec.device)), "pbg_pack")
    return out


def pack_record_sizes(env_id: str):
    L = _native.lib()
    iw, ow = ctypes.c_int(), ctypes.c_int()
    _native.check(L.pbg_pack_record_sizes(_native.env_id_bytes(env_id), ctypes.byref(iw), ctypes.byref(ow)),
                  "pbg_pack_record_sizes")
    return iw.value, ow.value
